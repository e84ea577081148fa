"""Histogram images stored in the statistics (describe.py:227-228).

The reference renders `hist_data` with matplotlib into base64 PNG data URIs
(/root/reference/spark_df_profiling/plot.py:20-55) inside the stats engine.
This is host-side presentation, out of the GPU path's scope; it is restated
for current matplotlib (object API, Agg canvas, no pyplot global state, so it
is safe to call from worker threads).
"""

import base64
from io import BytesIO
from urllib.parse import quote

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


def _encode(fig):
    buf = BytesIO()
    FigureCanvasAgg(fig).print_png(buf)
    return BASE + quote(base64.b64encode(buf.getvalue()))


def _safe_width(w):
    w = float(w)
    return w if np.isfinite(w) and w > 0 else 1.0


def mini_histogram(hist_data):
    """Small histogram (plot.py:20-39)."""
    fig = Figure(figsize=(2, 0.75))
    ax = fig.add_subplot(111)
    ax.bar(hist_data['left_edge'], hist_data['count'], width=_safe_width(hist_data['width'].iloc[0]),
           facecolor=BAR_COLOR, align='edge')
    ax.get_yaxis().set_visible(False)
    ax.set_facecolor('w')
    ticks = ax.xaxis.get_major_ticks()
    for t in ticks[1:-1]:
        t.set_visible(False)
    for t in (ticks[0], ticks[-1]) if ticks else ():
        t.label1.set_fontsize(8)
    fig.subplots_adjust(left=0.15, right=0.85, top=1, bottom=0.35, wspace=0, hspace=0)
    return _encode(fig)


def complete_histogram(hist_data):
    """Large histogram (plot.py:42-55)."""
    fig = Figure(figsize=(6, 4))
    ax = fig.add_subplot(111)
    ax.bar(hist_data['left_edge'], hist_data['count'], width=_safe_width(hist_data['width'].iloc[0]),
           facecolor=BAR_COLOR, align='edge')
    ax.set_ylabel('Frequency')
    fig.subplots_adjust(left=0.15, right=0.95, top=0.9, bottom=0.1, wspace=0, hspace=0)
    return _encode(fig)
