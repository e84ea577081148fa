"""spark_df_profiling on MI355X: ProfileReport / describe backed by HIP kernels.

Drop-in for the reference package's public surface on the statistics path
(/root/reference/spark_df_profiling/__init__.py:19-68, describe.py:66).
"""

from .describe import describe  # noqa: F401
from .columns import DeviceTable, DeviceColumn  # noqa: F401
from .report import ProfileReport  # noqa: F401

__version__ = '0.1.0'
