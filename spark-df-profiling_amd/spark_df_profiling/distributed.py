"""Multi-GPU exchanges for distinct counts and value counts.

Placeholder until the hash-partitioned all-to-all lands: the row-sharded path
currently supports world == 1 for grouping statistics.
"""


def exchange_fixed_groups(engine, tab, with_counts):
    raise NotImplementedError('multi-rank distinct counts: not built yet')


def exchange_bytes_groups(engine, tab):
    raise NotImplementedError('multi-rank value counts: not built yet')
