"""ProfileReport: the reference's user entry point over the GPU describe().

Mirrors /root/reference/spark_df_profiling/__init__.py:19-142 for the parts on
the statistics path: the constructor samples `sample` rows and calls
describe(df, bins, corr_reject, **kwargs) (__init__.py:61-68);
get_description / get_rejected_variables keep their semantics.  The HTML layer
(report.py / templates) is out of this round's scope: a
compact self-contained renderer stands in so to_file / _repr_html_ work.
"""

from __future__ import annotations

import html as _html

import pandas as pd
import pyarrow as pa

from .columns import DeviceTable
from .describe import describe

NO_OUTPUTFILE = 'spark_df_profiling.no_outputfile'
DEFAULT_OUTPUTFILE = 'spark_df_profiling.default_outputfile'


def _sample_frame(df, n):
    if isinstance(df, pa.Table):
        return df.slice(0, n).to_pandas()
    if isinstance(df, pa.RecordBatch):
        return pa.Table.from_batches([df]).slice(0, n).to_pandas()
    if isinstance(df, DeviceTable):
        return pd.DataFrame({c.name: [] for c in df.columns})
    limit = getattr(df, 'limit', None)
    if limit is not None:
        return df.limit(n).toPandas()
    raise TypeError('df must be of type pyspark.sql.DataFrame, pyarrow.Table or DeviceTable')


def render_html(sample, stats):
    """Overview table, one row per variable, frequency tables, sample."""
    t = stats['table']
    esc = _html.escape
    parts = ['<div class="sdp-report"><h2>Overview</h2><table>']
    for k, v in t.items():
        parts.append('<tr><th>%s</th><td>%s</td></tr>' % (esc(str(k)), esc(str(v))))
    parts.append('</table><h2>Variables</h2>')
    for name, row in stats['variables'].iterrows():
        parts.append('<h3>%s <small>%s</small></h3><table>' % (esc(str(name)), esc(str(row.get('type')))))
        for k, v in row.items():
            if k in ('histogram', 'mini_histogram') or (not isinstance(v, str) and pd.isnull(v)):
                continue
            parts.append('<tr><th>%s</th><td>%s</td></tr>' % (esc(str(k)), esc(str(v))))
        parts.append('</table>')
        if isinstance(row.get('histogram'), str):
            parts.append('<img src="%s"/>' % row['histogram'])
        if name in stats['freq']:
            parts.append('<table class="freq">')
            for k, v in stats['freq'][name].items():
                parts.append('<tr><td>%s</td><td>%s</td></tr>' % (esc(str(k)), esc(str(v))))
            parts.append('</table>')
    parts.append('<h2>Sample</h2>')
    parts.append(sample.to_html(classes='sample', index=False))
    parts.append('</div>')
    return ''.join(parts)


class ProfileReport(object):
    html = ''
    file = None

    def __init__(self, df, bins=10, sample=100, corr_reject=0.9, **kwargs):
        sample = _sample_frame(df, sample)
        description_set = describe(df, bins=bins, corr_reject=corr_reject, **kwargs)
        self.html = render_html(sample, description_set)
        self.description_set = description_set

    def get_description(self):
        return self.description_set

    def get_rejected_variables(self, threshold=0.9):
        variable_profile = self.description_set['variables']
        return variable_profile.index[variable_profile.correlation > threshold].tolist()

    def to_file(self, output=DEFAULT_OUTPUTFILE):
        if output != NO_OUTPUTFILE:
            if output == DEFAULT_OUTPUTFILE:
                output = 'profile_' + str(hash(self)) + '.html'
            with open(output, 'w', encoding='utf8') as self.file:
                self.file.write(self.to_html())

    def to_html(self):
        return '<!doctype html><html><head><meta charset="utf-8"></head><body>%s</body></html>' % self.html

    def _repr_html_(self):
        return self.html

    def __str__(self):
        return 'Output written to file ' + str(self.file.name)
