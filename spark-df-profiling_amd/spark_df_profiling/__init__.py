"""spark_df_profiling on MI355X: ProfileReport / describe backed by HIP kernels.

Drop-in for the reference package's public surface on the statistics path
(/root/reference/spark_df_profiling/__init__.py:19-68, describe.py:66).

The public names resolve lazily (PEP 562) so that light submodules -- e.g.
`plot`, imported by the histogram-rendering worker processes -- load without
pulling in torch and the HIP library.
"""

__version__ = '0.1.0'

_LAZY = {
    'describe': ('.describe', 'describe'),
    'DeviceTable': ('.columns', 'DeviceTable'),
    'DeviceColumn': ('.columns', 'DeviceColumn'),
    'ProfileReport': ('.report', 'ProfileReport'),
}

__all__ = list(_LAZY)


def __getattr__(name):
    if name in _LAZY:
        import importlib
        mod, attr = _LAZY[name]
        value = getattr(importlib.import_module(mod, __name__), attr)
        globals()[name] = value
        return value
    raise AttributeError('module %r has no attribute %r' % (__name__, name))
