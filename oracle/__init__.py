"""CPU oracle for the describe() statistics path -- TEST INFRASTRUCTURE ONLY.

This package restates, in numpy/pyarrow on the host, what the reference's
statistics engine (`/root/reference/spark_df_profiling/describe.py` and
`utils.py:corr_matrix`) returns when run on Apache Spark 2.x.  It is the checker
for the HIP path, never the product:

* only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
  ``cpu_baseline`` leg may import it;
* the product package (``spark-df-profiling_amd/spark_df_profiling``) never
  imports it and fails loudly when its HIP library is missing.

Pinning: the reference cannot run here (no pyspark, no JVM; see SURVEY.md
§8c -- an ordinary ModuleNotFoundError, not a permission denial).  The oracle
is pinned by the Spark-valid known answers recomputed from the reference's own
legacy test data (`tests.py.old.py:23-37`), committed as
``tests/golden/known_answers.json`` by ``tests/golden/make_golden.py``.
Behaviour the reference's fixtures do not cover (percentile_approx's exact
in-window element, top-N tie order, -0.0 grouping) is *defined* here and marked
"parity unpinned" in DESIGN.md.
"""

from .spark_describe import describe, profile_raw, spark_type_of  # noqa: F401
