"""Histogram images stored in the statistics (describe.py:227-228).

The reference renders `hist_data` with matplotlib into base64 PNG data URIs
(/root/reference/spark_df_profiling/plot.py:20-55) inside the stats engine.
This is host-side presentation, out of the GPU path's scope; it is restated
for current matplotlib: its Agg renderer, fonts, tick locators and formatters,
without pyplot's global state (safe in worker threads) and without the
Figure/Axis artist machinery (see _render).
"""

import base64
import struct
import threading
import zlib

import numpy as np
import pandas as pd
from matplotlib.backends.backend_agg import RendererAgg
from matplotlib.figure import Figure
from matplotlib.font_manager import FontProperties
from matplotlib.path import Path
from matplotlib.transforms import IdentityTransform

BASE = 'data:image/png;base64,'
BAR_COLOR = (0x33 / 255, 0x7a / 255, 0xb7 / 255, 1.0)      # '#337ab7'


def hist_frame(counts, edges, width):
    """The frame generate_hist_data returns (describe.py:53-61): bin_id, count
    (float when a bin was empty: reindex + fillna), left_edge, width."""
    counts = np.asarray(counts, dtype=np.int64)
    cnt = counts.astype(np.float64) if (counts == 0).any() else counts
    return pd.DataFrame({'bin_id': np.arange(len(counts)), 'count': cnt,
                         'left_edge': [float(e) for e in edges], 'width': float(width)})


def _safe_width(w):
    w = float(w)
    return w if np.isfinite(w) and w > 0 else 1.0


# ----------------------------------------------------------------------------
# The two figures of plot.py:20-55 -- bars in '#337ab7' from each left edge,
# the axes box, outward major ticks with matplotlib's own tick locations and
# labels (AutoLocator / ScalarFormatter, offset text included), 'Frequency' on
# the large one's y axis, only the first and last x ticks at 8 pt on the mini
# one -- drawn straight onto an Agg canvas.  Going through Figure.draw costs
# ~28 ms per large image, ~70 % of it in the Axis artists' generic tick and
# bounding-box bookkeeping; the same primitives issued directly (one compound
# path for the bars, one for the ticks, text laid out with matplotlib's own
# alignment rules) cost ~4 ms, and a C5 table has 1024 images.  The layout
# constants are matplotlib's defaults at 100 dpi (tests/test_plot_cpu.py
# compares the images with Figure.savefig's).
# ----------------------------------------------------------------------------
_DPI = 100.0
_PT = _DPI / 72.0
_TICK = 3.5 * _PT                # xtick/ytick.major.size, direction out
_PAD = 3.5 * _PT                 # xtick/ytick.major.pad
_OFFPAD = 3 * _PT                # Axis.OFFSETTEXTPAD
_LABELPAD = 4 * _PT              # axes.labelpad
_LW = 0.8                        # axes.linewidth = major tick width (points)
_KINDS = {'complete': dict(size=(6, 4), box=(0.15, 0.1, 0.95, 0.9), yaxis=True),
          'mini': dict(size=(2, 0.75), box=(0.15, 0.35, 0.85, 1.0), yaxis=False)}
_TLS = threading.local()


class _Canvas:
    """Per thread and kind: an undrawn Axes of the figure's geometry (its
    locators and formatters give the tick values and labels), fonts and a
    text-metrics cache."""

    def __init__(self, kind):
        g = _KINDS[kind]
        fig = Figure(figsize=g['size'], dpi=_DPI)
        self.ax = fig.add_subplot(111)
        l, b, r, t = g['box']
        fig.subplots_adjust(left=l, right=r, top=t, bottom=b, wspace=0, hspace=0)
        self.W, self.H = int(round(g['size'][0] * _DPI)), int(round(g['size'][1] * _DPI))
        bb = self.ax.bbox
        self.box = (bb.x0, bb.y0, bb.x1, bb.y1)
        self.clip = bb.frozen()
        self.yaxis = g['yaxis']
        self.fonts = {8: FontProperties(size=8), 10: FontProperties(size=10)}
        self.metrics = {}

    def ticks(self, axis, lo, hi):
        axis.set_view_interval(lo, hi, ignore=True)
        locs = np.asarray(axis.get_majorticklocs(), dtype=np.float64)
        fmt = axis.get_major_formatter()
        labels = fmt.format_ticks(locs)
        # drawn: the ticks inside the view interval, with the relative
        # tolerance of Axis._update_ticks (transforms._interval_contains_close)
        tol = 1e-10 * (hi - lo)
        inside = (locs >= lo - tol) & (locs <= hi + tol)
        return locs, labels, inside, fmt.get_offset()

    def extent(self, r, s, size):
        """(w, h, d) of a text line as Text._get_layout sizes it (at least
        the height and descent of 'lp')."""
        key = (s, size)
        m = self.metrics.get(key)
        if m is None:
            prop = self.fonts[size]
            w, h, d = r.get_text_width_height_descent(s, prop, ismath=False)
            lp = self.metrics.get(('lp', size))
            if lp is None:
                lp = self.metrics[('lp', size)] = r.get_text_width_height_descent('lp', prop, ismath=False)
            m = self.metrics[key] = (w, max(h, lp[1]), max(d, lp[2]))
        return m


def _canvas(kind):
    cache = getattr(_TLS, 'canvases', None)
    if cache is None:
        cache = _TLS.canvases = {}
    c = cache.get(kind)
    if c is None:
        c = cache[kind] = _Canvas(kind)
    return c


def _text(c, r, gc, s, x, y, ha, va, size, draw=True):
    """A horizontal single-line text anchored at display (x, y) (y up) with
    Text's alignment rules; returns its box (x0, y0, x1, y1)."""
    w, h, d = c.extent(r, s, size)
    x0 = x - {'center': w / 2, 'right': w, 'left': 0.0}[ha]
    base = {'top': y - (h - d), 'center_baseline': y - (h - d) / 2, 'baseline': y, 'bottom': y + d}[va]
    if draw:
        r.draw_text(gc, x0, c.H - base, s, c.fonts[size], 0)
    return (x0, base - d, x0 + w, base - d + h)


def _render(kind, left, height, w):
    c = _canvas(kind)
    r = RendererAgg(c.W, c.H, _DPI)
    L, B, R, T = c.box
    n = len(left)
    x0, x1 = float(left.min()), float(left.max()) + w
    y1 = float(height.max()) if n else 0.0
    if np.isfinite(x0) and np.isfinite(x1) and x1 > x0 and np.isfinite(y1) and y1 > 0:
        # the limits autoscale_view sets for these bars (axes margins 0.05,
        # bars sticky at y = 0)
        mx = 0.05 * (x1 - x0)
        xl, yl = (x0 - mx, x1 + mx), (0.0, y1 + 0.05 * y1)
    else:
        xl = (x0 - 0.5, x1 + 0.5) if np.isfinite(x0) and np.isfinite(x1) else (-0.5, 0.5)
        yl = (0.0, 1.0)
    sx, sy = (R - L) / (xl[1] - xl[0]), (T - B) / (yl[1] - yl[0])
    ident = IdentityTransform()
    gc = r.new_gc()
    gc.set_linewidth(0)
    r.draw_path(gc, Path([(0, 0), (c.W, 0), (c.W, c.H), (0, c.H), (0, 0)], closed=True), ident,
                (1.0, 1.0, 1.0, 1.0))                                    # figure and axes faces
    if n:
        xa = L + (left - xl[0]) * sx
        xb = L + (left + w - xl[0]) * sx
        yt = B + (height - yl[0]) * sy
        y0 = np.full(n, B - yl[0] * sy)
        verts = np.stack([xa, y0, xb, y0, xb, yt, xa, yt, xa, y0], 1).reshape(-1, 2)
        codes = np.tile(np.array([Path.MOVETO, Path.LINETO, Path.LINETO, Path.LINETO, Path.CLOSEPOLY],
                                 dtype=Path.code_type), n)
        gc.set_clip_rectangle(c.clip)
        r.draw_path(gc, Path(verts, codes), ident, BAR_COLOR)
    gc.restore()
    gl = r.new_gc()                                  # spines and ticks: 0.8 pt black, snapped
    gl.set_linewidth(_LW)
    gl.set_foreground('k')
    gl.set_snap(True)
    gl.set_capstyle('projecting')
    gl.set_joinstyle('miter')
    segs = [(L, B), (R, B), (L, T), (R, T), (L, B), (L, T), (R, B), (R, T)]
    seg_codes = [Path.MOVETO, Path.LINETO] * 4
    r.draw_path(gl, Path(segs, seg_codes), ident)
    gl.set_capstyle('butt')
    tick_v, label_boxes = [], []
    size = 8 if kind == 'mini' else 10
    locs, labels, inside, off = c.ticks(c.ax.xaxis, *xl)
    for i in range(len(locs)):
        if not inside[i]:
            continue
        px = L + (locs[i] - xl[0]) * sx
        shown = kind != 'mini' or i == 0 or i == len(locs) - 1
        # (the mini figure's hidden ticks keep their 10 pt labels' boxes,
        # which place the offset text, as matplotlib's do)
        box = _text(c, r, gl, labels[i], px, B - _TICK - _PAD, 'center', 'top', size if shown else 10,
                    draw=shown and bool(labels[i]))
        if labels[i]:
            label_boxes.append(box)
        if shown:
            tick_v += [(px, B), (px, B - _TICK)]
    if off:
        bottom = min(b[1] for b in label_boxes) if label_boxes else B
        _text(c, r, gl, off, R, bottom - _OFFPAD, 'right', 'top', 10)
    if c.yaxis:
        locs, labels, inside, off = c.ticks(c.ax.yaxis, *yl)
        xmin = L - 0.5 * _LW * _PT                          # the left spine's outer edge
        for i in range(len(locs)):
            if not inside[i]:
                continue
            py = B + (locs[i] - yl[0]) * sy
            tick_v += [(L, py), (L - _TICK, py)]
            if labels[i]:
                xmin = min(xmin, _text(c, r, gl, labels[i], L - _TICK - _PAD, py, 'right', 'center_baseline', 10)[0])
        if off:
            _text(c, r, gl, off, L, T + _OFFPAD, 'left', 'baseline', 10)
        # 'Frequency': rotated 90 degrees, anchored (rotation_mode 'anchor',
        # ha center, va bottom) labelpad left of the tick labels
        w_, h_, d_ = c.extent(r, 'Frequency', 10)
        ax_, ay_ = xmin - _LABELPAD, (B + T) / 2
        r.draw_text(gl, ax_ - d_, c.H - (ay_ - w_ / 2), 'Frequency', c.fonts[10], 90)
    if tick_v:
        r.draw_path(gl, Path(tick_v, [Path.MOVETO, Path.LINETO] * (len(tick_v) // 2)), ident)
    gl.restore()
    return _png(np.asarray(r.buffer_rgba()))


def _chunk(tag, data):
    return struct.pack('>I', len(data)) + tag + data + struct.pack('>I', zlib.crc32(tag + data) & 0xFFFFFFFF)


def _png(rgba):
    """The canvas as an 8-bit RGBA PNG (filter 0; zlib level 1 with the
    filtered strategy: the rows copy contiguously, and on these mostly flat
    images this beats dropping alpha first -- 2.6 vs 3.7 ms per large image)."""
    h, w = rgba.shape[:2]
    raw = np.empty((h, 1 + 4 * w), dtype=np.uint8)
    raw[:, 0] = 0
    raw[:, 1:] = rgba.reshape(h, 4 * w)
    z = zlib.compressobj(1, zlib.DEFLATED, 15, 8, zlib.Z_FILTERED)
    return (b'\x89PNG\r\n\x1a\n' + _chunk(b'IHDR', struct.pack('>IIBBBBB', w, h, 8, 6, 0, 0, 0)) +
            _chunk(b'IDAT', z.compress(raw.tobytes()) + z.flush()) + _chunk(b'IEND', b''))


def _encode(png):
    """base64 -> percent-quoted, as plot.py:35-37 stores it (quote() of base64
    text only ever escapes '+' and '=': the alphabet is alphanumerics, '+', '/'
    and '=', and '/' is quote's default safe character)."""
    b64 = base64.b64encode(png).decode('ascii')
    return BASE + b64.replace('+', '%2B').replace('=', '%3D')


def _draw(kind, hist_data):
    left = np.asarray(hist_data['left_edge'], dtype=np.float64)
    height = np.asarray(hist_data['count'], dtype=np.float64)
    w = _safe_width(hist_data['width'].iloc[0]) if len(hist_data) else 1.0
    return _encode(_render(kind, left, height, w))


def mini_histogram(hist_data):
    """Small histogram (plot.py:20-39)."""
    return _draw('mini', hist_data)


def complete_histogram(hist_data):
    """Large histogram (plot.py:42-55)."""
    return _draw('complete', hist_data)


def render_pair(counts, edges, width):
    """(histogram, mini_histogram) data URIs of one column's bins."""
    frame = hist_frame(counts, edges, width)
    return complete_histogram(frame), mini_histogram(frame)


# ----------------------------------------------------------------------------
# Rendering pool.  An image pair still costs a few ms of CPU (1024 images for
# a 512-column table), so describe() hands every column's bins to worker
# processes as soon as pass 2 has produced them and collects the strings at
# the end: the rendering overlaps the distinct counts' kernels.  Workers are
# spawned (a fresh interpreter: never a fork of a process holding the GPU)
# and import only this module's dependencies.
# ----------------------------------------------------------------------------

_POOL = None
_POOL_N = 1                        # its worker count
_POOL_LOCK = threading.Lock()      # column worker threads may submit concurrently


def _worker_init():
    # the workers fill every CPU of the job's share while describe() still
    # launches kernels and reads results back: they yield to it
    import os
    try:
        os.nice(10)
    except OSError:
        pass


def _warm():
    # imports matplotlib and sets up this worker's canvases and fonts
    return render_pair(np.arange(10), [float(i) for i in range(10)], 1.0)[1][:len(BASE)]


def start_pool(workers=None):
    """Start (once) the spawn-context worker pool and wait until every worker
    has imported matplotlib.  Call early (before heavy GPU allocation) to keep
    the one-time start-up out of the first describe()."""
    with _POOL_LOCK:
        return _start_pool_locked(workers)


def _start_pool_locked(workers):
    global _POOL, _POOL_N
    if _POOL is not None:
        return _POOL
    import multiprocessing as mp
    import os
    from concurrent.futures import ProcessPoolExecutor
    # one render process per CPU this job may use (affinity mask bounded by the
    # cgroup quota; os.cpu_count() would count the whole machine)
    from .utils import available_cpus
    n = workers or int(os.environ.get('SDP_PLOT_WORKERS', '0')) or available_cpus()[0]
    _POOL = ProcessPoolExecutor(max_workers=n, mp_context=mp.get_context('spawn'), initializer=_worker_init)
    _POOL_N = n
    # spawn re-runs the parent's __main__ in every child unless it cannot find
    # it; hide it while the workers start (they need only this module)
    import sys
    main = sys.modules.get('__main__')
    saved = {a: getattr(main, a) for a in ('__file__', '__spec__') if main is not None and hasattr(main, a)}
    try:
        if '__file__' in saved:
            del main.__file__
        if '__spec__' in saved:
            main.__spec__ = None
        futs = [_POOL.submit(_warm) for _ in range(2 * n)]
    finally:
        for a, v in saved.items():
            setattr(main, a, v)
    for f in futs:
        f.result()
    import atexit
    atexit.register(shutdown_pool)
    return _POOL


def shutdown_pool():
    global _POOL
    with _POOL_LOCK:
        if _POOL is not None:
            _POOL.shutdown(wait=True, cancel_futures=True)
            _POOL = None


class _Slot:
    """Column i's (histogram, mini histogram) of a batch task's result."""

    def __init__(self, fut, i):
        self.fut, self.i = fut, i

    def result(self):
        return self.fut.result()[self.i]


def render_pairs(items):
    return [render_pair(*it) for it in items]


def submit_batch(items):
    """Futures of render_pair(counts, edges, width) for every item, rendered
    on the pool in about two tasks per worker: a wide table's 1024 images as
    1024 tasks spent more in the executor's per-task queueing and pickling
    than in drawing (C5: ~120 ms of a step)."""
    if not items:
        return []
    pool = start_pool()
    per = max(1, -(-len(items) // (2 * _POOL_N)))
    out = []
    for i in range(0, len(items), per):
        chunk = [(np.asarray(c, dtype=np.int64), [float(e) for e in ed], float(w)) for c, ed, w in items[i:i + per]]
        fut = pool.submit(render_pairs, chunk)
        out += [_Slot(fut, j) for j in range(len(chunk))]
    return out


def submit(counts, edges, width):
    """Future of render_pair(counts, edges, width) on the pool."""
    return submit_batch([(counts, edges, width)])[0]
