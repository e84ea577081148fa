"""HTML report over describe()'s output.

Follows /root/reference/spark_df_profiling/report.py:14-146 (value_format,
format_freq_table, to_html) and __init__.py:19-124 (ProfileReport) on modern
pandas -- no `.ix`, no jinja2 (not installed here): the markup is produced by
the small render functions below and styled by one inline stylesheet, so a
report file is self-contained.  Content per variable type follows the
reference's row templates: NUM (quantile and descriptive statistics,
histogram), DATE (min / max / range), CAT (mini and full frequency tables),
UNIQUE (first and last values), CONST and CORR (rejection notes), plus the
overview (dataset info, type counts, warnings) and the sample table.
"""

from __future__ import annotations

import os

import html as _html

import pandas as pd
import pyarrow as pa

from . import formatters
from .columns import DeviceTable
from .describe import describe

NO_OUTPUTFILE = 'spark_df_profiling.no_outputfile'
DEFAULT_OUTPUTFILE = 'spark_df_profiling.default_outputfile'
OTHER_VALUES = '***Other Values***'
OTHER_DISTINCT = '***Other Values Distinct Count***'

VAR_TYPE = {'NUM': 'Numeric', 'DATE': 'Date', 'CAT': 'Categorical', 'UNIQUE': 'Categorical, Unique',
            'CONST': 'Constant', 'CORR': 'Highly correlated'}

# warning list entries (templates.py:70-80): str.format over the formatted row
MESSAGES = {
    'CONST': u'{0[varname]} has constant value {0[mode]} <span class="label rejected">Rejected</span>',
    'CORR': u'{0[varname]} is highly correlated with {0[correlation_var]} (&rho; = {0[correlation]}) '
            u'<span class="label rejected">Rejected</span>',
    'HIGH_CARDINALITY': u'{varname} has a high cardinality: {0[distinct_count]} distinct values '
                        u'<span class="label warning">Warning</span>',
    'n_duplicates': u'Dataset has {0[n_duplicates]} duplicate rows <span class="label warning">Warning</span>',
    'skewness': u'{varname} is highly skewed (&gamma;1 = {0[skewness]})',
    'p_missing': u'{varname} has {0[n_missing]} / {0[p_missing]} missing values <span class="label">Missing</span>',
    'p_infinite': u'{varname} has {0[n_infinite]} / {0[p_infinite]} infinite values '
                  u'<span class="label">Infinite</span>',
    'p_zeros': u'{varname} has {0[n_zeros]} / {0[p_zeros]} zeros',
}

STYLE = u"""
body{font-family:Helvetica,Arial,sans-serif;font-size:13px;margin:1.5em;color:#222}
h1{font-size:22px}h2{font-size:18px;border-bottom:1px solid #ddd;padding-bottom:.2em}
.variablerow{border-bottom:1px solid #e1e1e8;padding:.6em 0;display:flex;flex-wrap:wrap;gap:1.5em}
.namecol{min-width:14em}.varname{font-size:15px;font-weight:bold}.vartype{color:#777;font-style:italic}
table.stats{border-collapse:collapse}table.stats th{text-align:left;font-weight:normal;color:#555;padding-right:1em}
table.stats td{text-align:right}td.alert,span.alert{color:#c7254e;font-weight:bold}td.ignore{color:#aaa}
table.freq td{padding:1px 4px}div.bar{background:#337ab7;color:#fff;height:1.2em;white-space:nowrap;font-size:11px}
tr.other div.bar{background:#999}tr.missing div.bar{background:#d9534f}
details summary{cursor:pointer;color:#337ab7}.label{font-size:11px;padding:1px 4px;border-radius:3px;background:#777;color:#fff}
.label.rejected{background:#337ab7}.label.warning{background:#f0ad4e}
table.sample{border-collapse:collapse;font-size:12px}table.sample td,table.sample th{border:1px solid #ddd;padding:2px 5px}
code{color:#c7254e}
"""


def value_format(value, name):
    """report.py:14-26: '' for missing, a named formatter, the float
    formatter, else str()."""
    try:
        if pd.isnull(value):
            return ''
    except (TypeError, ValueError):
        pass
    vf = formatters.value_formatters
    if name in vf:
        return vf[name](value)
    if isinstance(value, float):
        return vf[formatters.DEFAULT_FLOAT_FORMATTER](value)
    return str(value)


def _bar_row(count, label, n, max_freq, extra_class=''):
    width = int(count / float(max_freq) * 99) + 1 if max_freq else 1
    inside, after = (count, '') if width > 20 else ('&nbsp;', count)
    return (u'<tr class="%s"><td class="fillremaining">%s</td><td style="width:60%%"><div class="bar" '
            u'style="width:%d%%">%s</div>%s</td><td>%s%%</td></tr>'
            % (extra_class, _html.escape(str(label)), width, inside, after, '{:2.1f}'.format(count / float(n) * 100)))


def format_freq_table(varname, freqtable, n, var_table, max_number_of_items_in_table, mini=False):
    """report.py:29-76: the top values, then 'Other values (k)' and '(Missing)'
    when they exceed the smallest value shown."""
    other_pre = freqtable[OTHER_VALUES]
    other_pre_num = freqtable[OTHER_DISTINCT]
    table = freqtable.drop([OTHER_VALUES, OTHER_DISTINCT])
    freq_other = sum(table[max_number_of_items_in_table:]) + other_pre
    freq_missing = var_table['n_missing']
    max_freq = max(table.values[0] if len(table) else 0, freq_other, freq_missing)
    min_freq = table.values[max_number_of_items_in_table] if len(table) > max_number_of_items_in_table else 0
    rows = [_bar_row(f, label, n, max_freq) for label, f in table[:max_number_of_items_in_table].items()]
    if freq_other > min_freq:
        rows.append(_bar_row(freq_other, 'Other values (%s)' % (table.count() + other_pre_num
                                                                 - max_number_of_items_in_table),
                             n, max_freq, 'other'))
    if freq_missing > min_freq:
        rows.append(_bar_row(freq_missing, '(Missing)', n, max_freq, 'missing'))
    return u'<table class="freq%s" id="freq-%s">%s</table>' % (' mini' if mini else '', abs(hash(varname)),
                                                              ''.join(rows))


def _stats_table(rows, v, cls):
    out = [u'<table class="stats">']
    for label, key in rows:
        if key in v:
            out.append(u'<tr><th>%s</th><td class="%s">%s</td></tr>' % (label, cls.get(key, ''), v[key]))
    out.append(u'</table>')
    return ''.join(out)


def _head(v, t):
    return (u'<div class="namecol"><div class="varname">%s</div><div class="vartype">%s</div></div>'
            % (_html.escape(str(v['varname'])), VAR_TYPE.get(t, t)))


def _img(src, cls):
    return u'<img class="%s" src="%s"/>' % (cls, src) if isinstance(src, str) and src else ''


def _row_num(v, cls, raw):
    top = _stats_table([('Distinct count', 'distinct_count'), ('Unique (%)', 'p_unique'),
                        ('Missing (%)', 'p_missing'), ('Missing (n)', 'n_missing'), ('Infinite (%)', 'p_infinite'),
                        ('Infinite (n)', 'n_infinite')], v, cls)
    mid = _stats_table([('Mean', 'mean'), ('Minimum', 'min'), ('Maximum', 'max'), ('Zeros (%)', 'p_zeros'),
                        ('High Index', 'high_idx'), ('Low Index', 'low_idx')], v, cls)
    quant = _stats_table([('Minimum', 'min'), ('5-th percentile', '5%'), ('Q1', '25%'), ('Median', '50%'),
                          ('Q3', '75%'), ('95-th percentile', '95%'), ('Maximum', 'max'), ('Range', 'range'),
                          ('Interquartile range', 'iqr')], v, cls)
    desc = _stats_table([('Standard deviation', 'std'), ('Coef of variation', 'cv'), ('Kurtosis', 'kurtosis'),
                         ('Mean', 'mean'), ('MAD', 'mad'), ('Skewness', 'skewness'), ('Sum', 'sum'),
                         ('Variance', 'variance'), ('Memory size', 'memorysize')], v, cls)
    return (_head(v, 'NUM') + top + mid + _img(raw.get('mini_histogram'), 'minihistogram')
            + u'<details><summary>Toggle details</summary><div class="variablerow"><div><b>Quantile statistics'
              u'</b>%s</div><div><b>Descriptive statistics</b>%s</div><div>%s</div></div></details>'
            % (quant, desc, _img(raw.get('histogram'), 'histogram')))


def _row_date(v, cls, raw):
    return _head(v, 'DATE') + _stats_table([('Distinct count', 'distinct_count'), ('Unique (%)', 'p_unique'),
                                            ('Missing (%)', 'p_missing'), ('Missing (n)', 'n_missing'),
                                            ('Infinite (%)', 'p_infinite'), ('Infinite (n)', 'n_infinite'),
                                            ('Minimum', 'min'), ('Maximum', 'max'), ('Range', 'range'),
                                            ('Completeness', 'completeness_idx')], v, cls)


def _row_cat(v, cls, raw):
    return (_head(v, 'CAT') + _stats_table([('Distinct count', 'distinct_count'), ('Unique (%)', 'p_unique'),
                                            ('Missing (%)', 'p_missing'), ('Missing (n)', 'n_missing')], v, cls)
            + v.get('minifreqtable', '') + u'<details><summary>Toggle details</summary>%s</details>'
            % v.get('freqtable', ''))


def _row_unique(v, cls, raw):
    return (_head(v, 'UNIQUE') + v.get('firstn', '') + v.get('lastn', '')
            + u'<details><summary>Toggle details</summary><div class="variablerow"><div><b>First 20 values</b>%s'
              u'</div><div><b>Last 20 values</b>%s</div></div></details>'
            % (v.get('firstn_expanded', ''), v.get('lastn_expanded', '')))


def _row_const(v, cls, raw):
    return _head(v, 'CONST') + u'<div>This variable is constant and should be ignored for analysis: <code>%s</code>' \
                               u'</div>' % _html.escape(str(v.get('mode', '')))


def _row_corr(v, cls, raw):
    return _head(v, 'CORR') + u'<div>This variable is highly correlated with %s and should be ignored for analysis ' \
                              u'(&rho; = %s)</div>' % (v.get('correlation_var', ''), v.get('correlation', ''))


ROWS = {'NUM': _row_num, 'DISCRETE': _row_num, 'DATE': _row_date, 'CAT': _row_cat, 'UNIQUE': _row_unique,
        'CONST': _row_const, 'CORR': _row_corr}


def to_html(sample, stats_object):
    """report.py:79-187: the report body for a pandas sample and describe()'s dict."""
    if not isinstance(sample, pd.DataFrame):
        raise TypeError('sample must be of type pandas.DataFrame')
    if not isinstance(stats_object, dict):
        raise TypeError('stats_object must be of type dict. Did you generate this using the '
                        'spark_df_profiling.describe() function?')
    if set(stats_object.keys()) != {'table', 'variables', 'freq'}:
        raise TypeError('stats_object badly formatted. Did you generate this using the '
                        'spark_df_profiling-eda.describe() function?')
    n_obs = stats_object['table']['n']
    row_formatters = formatters.row_formatters
    rows_html, messages = [], []
    for idx, row in stats_object['variables'].iterrows():
        fv = {'varname': idx, 'varid': hash(idx)}
        for col, value in row.items():
            fv[col] = value_format(value, col)
        classes = {}
        for col in set(row.index) & set(row_formatters):
            classes[col] = row_formatters[col](row[col])
            if classes[col] == 'alert' and col in MESSAGES:
                messages.append(MESSAGES[col].format(fv, varname=formatters.fmt_varname(idx)))
        t = row['type']
        if t == 'CAT':
            ft = stats_object['freq'][idx]
            fv['minifreqtable'] = format_freq_table(idx, ft, n_obs, row, 3, mini=True)
            fv['freqtable'] = format_freq_table(idx, ft, n_obs, row, 20)
            if row['distinct_count'] > 50:
                messages.append(MESSAGES['HIGH_CARDINALITY'].format(fv, varname=formatters.fmt_varname(idx)))
                classes['distinct_count'] = 'alert'
            else:
                classes['distinct_count'] = ''
        if t == 'UNIQUE':
            obs = list(stats_object['freq'][idx].index)
            fv['firstn'] = pd.DataFrame(obs[0:3], columns=['First 3 values']).to_html(classes='example_values',
                                                                                      index=False)
            fv['lastn'] = pd.DataFrame(obs[-3:], columns=['Last 3 values']).to_html(classes='example_values',
                                                                                    index=False)
            if n_obs > 40:
                fv['firstn_expanded'] = pd.DataFrame(obs[0:20], index=range(1, len(obs[0:20]) + 1)).to_html(
                    classes='sample', header=False)
                last = obs[-20:]
                fv['lastn_expanded'] = pd.DataFrame(last, index=range(n_obs - len(last) + 1, n_obs + 1)).to_html(
                    classes='sample', header=False)
            else:
                fv['firstn_expanded'] = pd.DataFrame(obs, index=range(1, len(obs) + 1)).to_html(classes='sample',
                                                                                                  header=False)
                fv['lastn_expanded'] = ''
        render = ROWS.get(t)
        body = render(fv, classes, row) if render else _head(fv, t)
        rows_html.append(u'<div class="variablerow" id="var-%s">%s</div>' % (abs(fv['varid']), body))
        if t in ('CORR', 'CONST'):
            fv['varname'] = formatters.fmt_varname(idx)
            messages.append(MESSAGES[t].format(fv))
    table = stats_object['table']
    tv = {k: value_format(v, k) for k, v in table.items()}
    for col in set(table) & set(row_formatters):
        if row_formatters[col](table[col]) == 'alert' and col in MESSAGES:
            messages.append(MESSAGES[col].format(tv, varname=''))
    overview = (u'<div class="variablerow"><div><b>Dataset info</b>%s</div><div><b>Variables types</b>%s</div>'
                u'<div><b>Warnings</b><ul>%s</ul></div></div>'
                % (_stats_table([('Number of variables', 'nvar'), ('Number of observations', 'n'),
                                 ('Total Missing (%)', 'total_missing'), ('Total size in memory', 'memsize'),
                                 ('Average record size in memory', 'recordsize'),
                                 ('Accuracy Index (%)', 'accuracy_idx')], tv, {}),
                   _stats_table([('Numeric', 'NUM'), ('Categorical', 'CAT'), ('Date', 'DATE'),
                                 ('Text (Unique)', 'UNIQUE'), ('Rejected', 'REJECTED')], tv, {}),
                   ''.join(u'<li>%s</li>' % m for m in messages)))
    sample_html = sample.to_html(classes='sample', index=False)
    return (u'<div class="sdp-report"><h2>Overview</h2>%s<h2>Variables</h2>%s<h2>Sample</h2>%s</div>'
            % (overview, ''.join(rows_html), sample_html))


def _sample_frame(df, n):
    if isinstance(df, pa.Table):
        return df.slice(0, n).to_pandas()
    if isinstance(df, pa.RecordBatch):
        return pa.Table.from_batches([df]).slice(0, n).to_pandas()
    if isinstance(df, DeviceTable):
        return pd.DataFrame({c.name: [] for c in df.columns})
    if isinstance(df, (str, os.PathLike)) and str(df).endswith('.parquet'):
        import pyarrow.parquet as pq
        pf = pq.ParquetFile(str(df))
        return pa.Table.from_batches([next(pf.iter_batches(batch_size=max(n, 1)))]).slice(0, n).to_pandas() \
            if pf.metadata.num_rows else pd.DataFrame()
    if isinstance(df, (list, tuple)) and df and all(isinstance(b, pa.RecordBatch) for b in df):
        return pa.Table.from_batches(list(df)).slice(0, n).to_pandas()
    if isinstance(df, pa.RecordBatchReader):
        raise TypeError('a RecordBatchReader is read once: pass describe() the reader, or ProfileReport '
                        'an iterator of RecordBatches')
    limit = getattr(df, 'limit', None)
    if limit is not None:
        return df.limit(n).toPandas()
    raise TypeError('df must be of type pyspark.sql.DataFrame, pyarrow.Table, a .parquet path or DeviceTable')


def _sample_batches(it, n):
    """The first n rows of a RecordBatch iterator as pandas, and an iterator
    that yields every batch again (the sampled ones first)."""
    import itertools
    head, rows = [], 0
    for b in it:
        head.append(b)
        rows += b.num_rows
        if rows >= n:
            break
    if head and not all(isinstance(b, pa.RecordBatch) for b in head):
        raise TypeError('df must be of type pyspark.sql.DataFrame, pyarrow.Table, a .parquet path or DeviceTable')
    frame = pa.Table.from_batches(head).slice(0, n).to_pandas() if head else pd.DataFrame()
    return frame, itertools.chain(head, it)


class ProfileReport(object):
    """__init__.py:19-124: describe() once at construction, then HTML on demand."""
    html = ''
    file = None

    def __init__(self, df, bins=10, sample=100, corr_reject=0.9, **kwargs):
        if hasattr(df, '__next__') and hasattr(df, '__iter__'):       # a stream of RecordBatches
            sample, df = _sample_batches(df, sample)
        else:
            sample = _sample_frame(df, sample)
        description_set = describe(df, bins=bins, corr_reject=corr_reject, **kwargs)
        self.html = to_html(sample, description_set)
        self.description_set = description_set

    def render_standalone(self, mode='databricks', utils=None):
        """The reference copies bootstrap assets to DBFS for Databricks; the
        report here is self-contained, so this returns the full document."""
        return self.to_html()

    def get_description(self):
        return self.description_set

    def get_rejected_variables(self, threshold=0.9):
        variable_profile = self.description_set['variables']
        if 'correlation' not in variable_profile:
            return []
        return variable_profile.index[variable_profile.correlation > threshold].tolist()

    def to_file(self, output=DEFAULT_OUTPUTFILE):
        if output != NO_OUTPUTFILE:
            if output == DEFAULT_OUTPUTFILE:
                output = 'profile_' + str(hash(self)) + '.html'
            with open(output, 'w', encoding='utf8') as self.file:
                self.file.write(self.to_html())

    def to_html(self):
        return (u'<!doctype html><html><head><meta charset="utf-8"><title>Profile report</title><style>%s</style>'
                u'</head><body><h1>Profile report</h1>%s</body></html>' % (STYLE, self.html))

    def _repr_html_(self):
        return self.html

    def __str__(self):
        return 'Output written to file ' + str(self.file.name)
