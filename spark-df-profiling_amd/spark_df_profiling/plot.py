"""Histogram images stored in the statistics (describe.py:227-228).

The reference renders `hist_data` with matplotlib into base64 PNG data URIs
(/root/reference/spark_df_profiling/plot.py:20-55) inside the stats engine.
This is host-side presentation, out of the GPU path's scope; it is restated
for current matplotlib (object API, Agg canvas, no pyplot global state, so it
is safe to call from worker threads).
"""

import base64
import threading
from io import BytesIO

import numpy as np
import pandas as pd
from matplotlib.backends.backend_agg import FigureCanvasAgg
from matplotlib.figure import Figure

BASE = 'data:image/png;base64,'
BAR_COLOR = '#337ab7'


def hist_frame(counts, edges, width):
    """The frame generate_hist_data returns (describe.py:53-61): bin_id, count
    (float when a bin was empty: reindex + fillna), left_edge, width."""
    counts = np.asarray(counts, dtype=np.int64)
    cnt = counts.astype(np.float64) if (counts == 0).any() else counts
    return pd.DataFrame({'bin_id': np.arange(len(counts)), 'count': cnt,
                         'left_edge': [float(e) for e in edges], 'width': float(width)})


def _encode(canvas):
    """PNG -> base64 -> percent-quoted, as plot.py:35-37 stores it.  zlib level 1
    (the images are mostly flat colour: same pixels, ~1/6 of the encode time);
    quote() of base64 text only ever escapes '+' and '=' (the alphabet is
    alphanumerics, '+', '/' and '='; '/' is quote's default safe character)."""
    buf = BytesIO()
    canvas.print_png(buf, pil_kwargs={'compress_level': 1})
    b64 = base64.b64encode(buf.getvalue()).decode('ascii')
    return BASE + b64.replace('+', '%2B').replace('=', '%3D')


def _safe_width(w):
    w = float(w)
    return w if np.isfinite(w) and w > 0 else 1.0


# One figure per (kind, bin count) and thread, built once and re-used: only the
# bar rectangles and the view limits change between columns.  Building a
# Figure + Axes + tick artists costs about as much as drawing them, so a
# re-used figure halves the cost of an image (64 -> 33 ms on this image's
# CPU).  Thread-local, so SDP_PLOT_WORKERS=0 with column workers stays safe.
_TLS = threading.local()


def _figure(kind, nbins):
    cache = getattr(_TLS, 'figs', None)
    if cache is None:
        cache = _TLS.figs = {}
    key = (kind, nbins)
    if key not in cache:
        fig = Figure(figsize=(2, 0.75) if kind == 'mini' else (6, 4))
        ax = fig.add_subplot(111)
        bars = ax.bar(np.arange(nbins, dtype=np.float64), np.ones(nbins), width=1.0,
                      facecolor=BAR_COLOR, align='edge')
        if kind == 'mini':
            ax.get_yaxis().set_visible(False)
            ax.set_facecolor('w')
            fig.subplots_adjust(left=0.15, right=0.85, top=1, bottom=0.35, wspace=0, hspace=0)
        else:
            ax.set_ylabel('Frequency')
            fig.subplots_adjust(left=0.15, right=0.95, top=0.9, bottom=0.1, wspace=0, hspace=0)
        cache[key] = (FigureCanvasAgg(fig), ax, list(bars.patches))
    return cache[key]


def _draw(kind, hist_data):
    left = np.asarray(hist_data['left_edge'], dtype=np.float64)
    height = np.asarray(hist_data['count'], dtype=np.float64)
    w = _safe_width(hist_data['width'].iloc[0])
    canvas, ax, bars = _figure(kind, len(left))
    for r, x, h in zip(bars, left, height):
        r.set_x(x)
        r.set_width(w)
        r.set_height(h)
    x0, x1 = float(left.min()), float(left.max()) + w
    y1 = float(height.max()) if height.size else 0.0
    if np.isfinite(x0) and np.isfinite(x1) and x1 > x0 and np.isfinite(y1) and y1 > 0:
        # the limits autoscale_view would set for these bars (axes.[xy]margin
        # 0.05, bars sticky at y = 0), without relim's walk over every patch
        mx = 0.05 * (x1 - x0)
        ax.set_xlim(x0 - mx, x1 + mx)
        ax.set_ylim(0.0, y1 + 0.05 * y1)
    else:
        ax.relim()
        ax.autoscale_view()
    if kind == 'mini':
        # only the first and last x tick labels, in 8 pt (plot.py:27-36)
        ticks = ax.xaxis.get_major_ticks()
        for i, t in enumerate(ticks):
            edge = i == 0 or i == len(ticks) - 1
            t.set_visible(edge)
            if edge:
                t.label1.set_fontsize(8)
    return _encode(canvas)


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


def render_one(kind, counts, edges, width):
    frame = hist_frame(counts, edges, width)
    return complete_histogram(frame) if kind == 'complete' else mini_histogram(frame)


# ----------------------------------------------------------------------------
# Rendering pool.  matplotlib costs ~20 ms of pure-Python CPU per image (24
# images for a 12-numeric-column table), longer than the GPU statistics
# themselves, so describe() hands each column's bins to worker processes as
# soon as pass 2 has produced them and collects the strings at the end: the
# rendering overlaps the remaining columns' kernels.  Workers are spawned (a
# fresh interpreter: never a fork of a process holding the GPU) and import
# only this module's dependencies.
# ----------------------------------------------------------------------------

_POOL = None
_POOL_LOCK = threading.Lock()      # column worker threads may submit concurrently


def _warm():
    # builds the default 10-bin figures of this worker
    return render_pair(np.arange(10), [float(i) for i in range(10)], 1.0)[1][:len(BASE)]


def start_pool(workers=None):
    """Start (once) the spawn-context worker pool and wait until every worker
    has imported matplotlib.  Call early (before heavy GPU allocation) to keep
    the one-time start-up out of the first describe()."""
    with _POOL_LOCK:
        return _start_pool_locked(workers)


def _start_pool_locked(workers):
    global _POOL
    if _POOL is not None:
        return _POOL
    import multiprocessing as mp
    import os
    from concurrent.futures import ProcessPoolExecutor
    # one render process per CPU this job may use (affinity mask bounded by the
    # cgroup quota; os.cpu_count() would count the whole machine)
    from .utils import available_cpus
    n = workers or int(os.environ.get('SDP_PLOT_WORKERS', '0')) or available_cpus()[0]
    _POOL = ProcessPoolExecutor(max_workers=n, mp_context=mp.get_context('spawn'))
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


class _PairFuture:
    """The two images of one column, rendered as two pool tasks (24 tasks for
    12 columns balance over the workers better than 12 pairs)."""

    def __init__(self, a, b):
        self.a, self.b = a, b

    def result(self):
        return self.a.result(), self.b.result()


def submit(counts, edges, width):
    """Future of render_pair(counts, edges, width) on the pool."""
    pool = start_pool()
    args = (np.asarray(counts, dtype=np.int64), [float(e) for e in edges], float(width))
    return _PairFuture(pool.submit(render_one, 'complete', *args), pool.submit(render_one, 'mini', *args))
