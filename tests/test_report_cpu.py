"""Report layer (report.py / formatters.py) rendered from
the oracle's describe() dict -- the same dict the GPU path returns -- so it
runs without a GPU."""

import numpy as np
import pandas as pd
import pytest

import datagen


def _stats(n=3000):
    import oracle
    t = datagen.demo_like_table(n)
    return t, oracle.describe(t)


def test_formatters_match_reference_semantics():
    from spark_df_profiling import formatters as f
    assert f.fmt_percent(0.1234) == '12.3%'
    assert f.fmt_bytesize(1536) == '1.5 KiB'
    assert f.fmt_varname('x') == '<code>x</code>'
    assert f.value_formatters[f.DEFAULT_FLOAT_FORMATTER](100000.0) == '100000'
    assert f.value_formatters[f.DEFAULT_FLOAT_FORMATTER](3.14159265) == '3.1416'
    assert f.fmt_row_severity(0.5) == 'alert' and f.fmt_row_severity(0.0) == 'ignore'
    assert f.fmt_row_severity(float('nan')) == 'ignore'
    assert f.fmt_skewness(25.0) == 'alert' and f.fmt_skewness(1.0) == ''
    assert 'rgb(30, 198, 244)' in f.value_formatters['freq'](0)


def test_to_html_sections():
    from spark_df_profiling.report import to_html
    t, stats = _stats()
    html = to_html(t.slice(0, 10).to_pandas(), stats)
    for name in t.column_names:
        assert 'id="var-' in html and str(name) in html
    assert 'Dataset info' in html and 'Variables types' in html
    v = stats['variables']
    for typ in set(v['type']):
        assert typ in ('NUM', 'CAT', 'DATE', 'UNIQUE', 'CONST', 'CORR')
    if (v['type'] == 'CONST').any():
        assert 'has constant value' in html
    if (v['type'] == 'CORR').any():
        assert 'is highly correlated with' in html
    if (v['type'] == 'CAT').any():
        assert 'class="freq mini"' in html and 'class="bar"' in html
    if (v['type'] == 'UNIQUE').any():
        assert 'First 3 values' in html


def test_freq_table_other_and_missing_rows():
    from spark_df_profiling.report import format_freq_table
    ft = pd.Series([50, 30, 10, 40, 7], index=['a', 'b', 'c', '***Other Values***',
                                                '***Other Values Distinct Count***'])
    out = format_freq_table('v', ft, 200, pd.Series({'n_missing': 70}), 2)
    assert 'Other values (8)' in out and '(Missing)' in out
    assert out.count('<tr') == 4


def test_to_html_rejects_bad_inputs():
    from spark_df_profiling.report import to_html
    with pytest.raises(TypeError):
        to_html([1, 2], {'table': {}, 'variables': pd.DataFrame(), 'freq': {}})
    with pytest.raises(TypeError):
        to_html(pd.DataFrame(), {'table': {}})
