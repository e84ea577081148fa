"""Number / label formatting of the HTML report (same names and behaviour as
/root/reference/spark_df_profiling/formatters.py).

value_formatters map a statistic name to its display string; row_formatters
map it to a CSS class ('alert' / 'ignore' / '') that the report uses for the
warning list."""

from __future__ import annotations

import math

SKEWNESS_CUTOFF = 20
DEFAULT_FLOAT_FORMATTER = 'spark_df_profiling.__default_float_formatter'


def fmt_color(text, color):
    return u'<span style="color:%s">%s</span>' % (color, text)


def fmt_class(text, cls):
    return u'<span class="%s">%s</span>' % (cls, text)


def gradient_format(value, limit1, limit2, c1, c2):
    """`value` coloured on the straight line from rgb c1 (at limit1) to c2 (at limit2)."""
    t = (value - limit1) / (limit2 - limit1)
    rgb = tuple(int(a + (b - a) * t) for a, b in zip(c1, c2))
    return fmt_color(value, 'rgb%s' % (rgb,))


def fmt_bytesize(num, suffix='B'):
    for unit in ('', 'Ki', 'Mi', 'Gi', 'Ti', 'Pi', 'Ei', 'Zi'):
        if abs(num) < 1024.0:
            return '%3.1f %s%s' % (num, unit, suffix)
        num /= 1024.0
    return '%.1f %s%s' % (num, 'Yi', suffix)


def fmt_percent(v):
    return '%2.1f%%' % (v * 100)


def fmt_varname(v):
    return u'<code>%s</code>' % (v,)


def fmt_float(v):
    """Five significant digits without trailing zeros (1.0 -> '1', 0.25 -> '0.25').
    The strip is applied to the repr as is, exponent included, as the
    reference's default float formatter does (1e20 -> '1e+2')."""
    return str(float('%.5g' % v)).rstrip('0').rstrip('.')


value_formatters = {
    'freq': lambda v: gradient_format(v, 0, 62000, (30, 198, 244), (99, 200, 72)),
    'p_missing': fmt_percent,
    'p_infinite': fmt_percent,
    'p_unique': fmt_percent,
    'p_zeros': fmt_percent,
    'memorysize': fmt_bytesize,
    'total_missing': fmt_percent,
    DEFAULT_FLOAT_FORMATTER: fmt_float,
    'correlation_var': fmt_varname,
    'accuracy_idx': fmt_percent,
}


def _isnan(v):
    try:
        return math.isnan(v)
    except TypeError:
        return False


def fmt_row_severity(v):
    return 'ignore' if _isnan(v) or v <= 0.01 else 'alert'


def fmt_skewness(v):
    return 'alert' if not _isnan(v) and abs(v) > SKEWNESS_CUTOFF else ''


row_formatters = {
    'p_zeros': fmt_row_severity,
    'p_missing': fmt_row_severity,
    'p_infinite': fmt_row_severity,
    'n_duplicates': fmt_row_severity,
    'skewness': fmt_skewness,
}
