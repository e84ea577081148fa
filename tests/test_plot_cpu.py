"""The histogram images (plot.py) against matplotlib's own rendering of the
reference's figures (/root/reference/spark_df_profiling/plot.py:20-55:
plt.bar of the bins from their left edges in '#337ab7', ylabel 'Frequency',
the mini figure's y axis hidden and only its first and last x ticks shown at
8 pt, subplots_adjust as there), drawn here through Figure.savefig.  The
product draws the same primitives straight onto an Agg canvas; the images
must agree to within anti-aliasing: mean absolute difference per channel and
the share of pixels that differ visibly."""

import base64
import io
import time
import urllib.parse

import numpy as np
import pandas as pd
import pytest
from matplotlib.backends.backend_agg import FigureCanvasAgg
from matplotlib.figure import Figure
from PIL import Image

from spark_df_profiling import plot


def _reference_png(kind, frame):
    fig = Figure(figsize=(2, 0.75) if kind == 'mini' else (6, 4))
    FigureCanvasAgg(fig)
    ax = fig.add_subplot(111)
    ax.bar(frame['left_edge'], frame['count'], width=float(frame['width'].iloc[0]), facecolor='#337ab7',
           align='edge')
    if kind == 'mini':
        ax.get_yaxis().set_visible(False)
        ax.set_facecolor('w')
        ticks = ax.xaxis.get_major_ticks()
        for t in ticks[1:-1]:
            t.set_visible(False)
        for t in (ticks[0], ticks[-1]):
            t.label1.set_fontsize(8)
        fig.subplots_adjust(left=0.15, right=0.85, top=1, bottom=0.35, wspace=0, hspace=0)
    else:
        ax.set_ylabel('Frequency')
        fig.subplots_adjust(left=0.15, right=0.95, top=0.9, bottom=0.1, wspace=0, hspace=0)
    buf = io.BytesIO()
    fig.savefig(buf, format='png')
    return buf.getvalue()


def _pixels(png):
    return np.asarray(Image.open(io.BytesIO(png)).convert('RGB')).astype(np.int32)


def _frames():
    rng = np.random.default_rng(5)
    out = []
    for i in range(14):
        n = (10, 7, 3, 25)[i % 4]
        lo = float(rng.normal()) * 10.0 ** (i % 6 - 2) + (1e9 if i == 5 else 0.0) - (3e7 if i == 9 else 0.0)
        w = abs(float(rng.normal())) * 10.0 ** (i % 5 - 2) + 1e-3
        counts = rng.integers(0, 10 ** (1 + i % 8), n)
        if i % 3 == 0:
            counts[rng.integers(0, n)] = 0
        out.append(plot.hist_frame(counts, lo + w * np.arange(n), w))
    return out


@pytest.mark.parametrize('kind', ['complete', 'mini'])
def test_images_match_matplotlib(kind):
    worst = []
    for frame in _frames():
        uri = plot._draw(kind, frame)
        assert uri.startswith(plot.BASE)
        got = base64.b64decode(urllib.parse.unquote(uri[len(plot.BASE):]))
        a, b = _pixels(got), _pixels(_reference_png(kind, frame))
        assert a.shape == b.shape
        diff = np.abs(a - b)
        worst.append((diff.mean(), (diff.max(axis=2) > 96).mean()))
    mean_abs = max(m for m, _ in worst)
    visible = max(v for _, v in worst)
    assert mean_abs < 1.5 and visible < 0.004, worst


def test_render_cost():
    frames = _frames()
    plot._draw('complete', frames[0])
    t = time.perf_counter()
    for f in frames:
        plot._draw('complete', f)
        plot._draw('mini', f)
    per_pair = (time.perf_counter() - t) / len(frames)
    assert per_pair < 0.025, per_pair          # Figure.savefig: ~35 ms per pair on this host
