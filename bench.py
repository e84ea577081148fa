#!/usr/bin/env python3
"""bench.py -- profile rows/s of describe() on MI355X (BASELINE.json metric).

Workload: a synthetic table of `--rows` rows (default
1e9) x 16 columns with 5 % nulls per cell (Arrow validity, no NaN), generated
directly in HBM by torch from fixed seeds, row-sharded in contiguous ranges
across ranks (strong scaling: the whole table is fixed, each of N ranks holds
rows/N):
  6 x fp64   N(0,1), N(1e9,1), lognormal(0,1), U(-1e6,1e6), exp(1), Student-t(3)
  4 x int64  U[0,1e6), U[-2^31,2^31), zipf(1.2), sequential id
  2 x fp32   N(0,1), U[0,1)
  3 x utf8   zipf(1.1) over 100 / 1e5 / 1e8 labels, 4-16 bytes (large_string)
  1 x date32 U[1688-01-01, 2101-12-31]

One step = one full describe() (every column's statistics, the Pearson matrix
with CORR rejection, the histogram PNGs) over the resident table.  Inputs are in
HBM when the timed region starts; H2D is not timed.

    python bench.py [--gpus N --steps K --warmup W --rows R]
    torchrun --nproc-per-node N bench.py --gpus N ...     (one rank per GPU, RCCL)

With --gpus N > 1 and no launcher (no WORLD_SIZE in the environment) bench.py
starts the N rank processes itself as children (torch.distributed.run on
127.0.0.1) and re-prints rank 0's line; a rank whose process group is not N
ranks wide exits non-zero.

Rank 0 prints one JSON line.  `roofline` is for the dominant kernel, timed with
HIP events on the launch stream; `cpu_baseline` is the oracle (CPU restatement)
on a bounded sample of the same workload, rank 0 at N=1 only.
"""

import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, 'spark-df-profiling_amd'))

METRIC = 'profile rows/sec (whole node) + % HBM roofline, 1B-row x16 col at 1/2/4/8 GPUs'
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md:36 (spec)
FP64_MFMA_PEAK_TFS = 78.6      # AMD spec for MI355X fp64 matrix (not in the local guide)
NULL_P = 0.05
SEED = 20261015


# ----------------------------------------------------------------------------
# synthetic C3 shard in HBM
# ----------------------------------------------------------------------------

def _gen(seed, device):
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    return g


def _validity(n, g, device):
    """Arrow LSB-first bitmap with P(null) = NULL_P, padded by 8 bytes."""
    nb = (n + 7) // 8
    bits = torch.rand(nb * 8, generator=g, device=device) >= NULL_P
    w = torch.tensor([1, 2, 4, 8, 16, 32, 64, 128], dtype=torch.int32, device=device)
    packed = (bits.view(nb, 8).to(torch.int32) * w).sum(1).to(torch.uint8)
    out = torch.zeros(nb + 8, dtype=torch.uint8, device=device)
    out[:nb] = packed
    return out


def _bounded_zipf(n, s, card, g, device):
    """Continuous power-law inverse CDF on [1, card+1) -> labels 0..card-1."""
    u = torch.rand(n, generator=g, device=device, dtype=torch.float64)
    a = 1.0 - s
    x = torch.pow(1.0 - u * (1.0 - (card + 1.0) ** a), 1.0 / a)
    return torch.clamp(x.floor().to(torch.int64) - 1, 0, card - 1)


def _mix(x):
    x = x ^ (x >> 31)
    x = x * 0x7FB5D329728EA185
    x = x ^ (x >> 27)
    x = x * 0x3C79AC492BA7B653
    return x ^ (x >> 33)


_HEX = torch.tensor(list(b'0123456789abcdef'), dtype=torch.uint8)
_FILL = torch.tensor(list(b'ghijklmnopqrstuvwxyzGHIJ'), dtype=torch.uint8)


def _string_column(labels, card, device, chunk=1 << 25):
    """utf8 (int64 offsets): label l -> hex digits of l then filler, 4-16 bytes."""
    ndig = max(1, math.ceil(math.log(card, 16))) if card > 1 else 1
    h = _mix(labels.clone())
    lens = torch.clamp(4 + (h & 0x7FFFFFFF) % 13, min=ndig).to(torch.int64)
    offsets = torch.zeros(labels.numel() + 1, dtype=torch.int64, device=device)
    torch.cumsum(lens, 0, out=offsets[1:])
    total = int(offsets[-1].item())
    data = torch.zeros(total + 16, dtype=torch.uint8, device=device)
    hexd, fill = _HEX.to(device), _FILL.to(device)
    n = labels.numel()
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        L = lens[s:e]
        rows = torch.repeat_interleave(torch.arange(s, e, device=device), L)
        pos = torch.arange(rows.numel(), device=device) - (offsets[rows] - offsets[s])
        lab = labels[rows]
        shift = (ndig - 1 - pos).clamp(min=0) * 4
        digit = hexd[((lab >> shift) & 15)]
        filler = fill[(_mix(lab + pos) & 0xFFFF) % fill.numel()]
        data[int(offsets[s].item()):int(offsets[e].item())] = torch.where(pos < ndig, digit, filler)
    return offsets, data


def make_c3_shard(rows_total, rank, world, device):
    from spark_df_profiling import _native as nat
    from spark_df_profiling.columns import DeviceColumn, DeviceTable
    per = rows_total // world
    start = rank * per
    n = per if rank < world - 1 else rows_total - start
    cols = []

    def fixed(name, spark_t, dtype, values, seed):
        g = _gen(seed * 131 + rank, device)
        c = DeviceColumn(name, spark_t, n, 'fixed', dtype)
        c.values = values
        c.validity = _validity(n, g, device)
        cols.append(c)

    k = 0
    f64 = [('f64_norm', lambda g: torch.randn(n, generator=g, device=device, dtype=torch.float64)),
           ('f64_shifted', lambda g: 1e9 + torch.randn(n, generator=g, device=device, dtype=torch.float64)),
           ('f64_lognormal', lambda g: torch.exp(torch.randn(n, generator=g, device=device, dtype=torch.float64))),
           ('f64_uniform', lambda g: (torch.rand(n, generator=g, device=device, dtype=torch.float64) * 2 - 1) * 1e6),
           ('f64_exp', lambda g: -torch.log1p(-torch.rand(n, generator=g, device=device, dtype=torch.float64))),
           ('f64_student_t3', lambda g: torch.randn(n, generator=g, device=device, dtype=torch.float64) / torch.sqrt(
               (torch.randn(n, generator=g, device=device, dtype=torch.float64) ** 2
                + torch.randn(n, generator=g, device=device, dtype=torch.float64) ** 2
                + torch.randn(n, generator=g, device=device, dtype=torch.float64) ** 2) / 3.0))]
    for name, fn in f64:
        k += 1
        fixed(name, 'double', nat.F64, fn(_gen(SEED + k * 1000 + rank, device)), SEED + k)
    i64 = [('i64_uniform_1e6', lambda g: torch.randint(0, 10 ** 6, (n,), generator=g, device=device)),
           ('i64_uniform_2p31', lambda g: torch.randint(-2 ** 31, 2 ** 31, (n,), generator=g, device=device)),
           ('i64_zipf', lambda g: _bounded_zipf(n, 1.2, 2 ** 40, g, device) + 1),
           ('i64_id', lambda g: torch.arange(start, start + n, dtype=torch.int64, device=device))]
    for name, fn in i64:
        k += 1
        fixed(name, 'bigint', nat.I64, fn(_gen(SEED + k * 1000 + rank, device)), SEED + k)
    f32 = [('f32_norm', lambda g: torch.randn(n, generator=g, device=device, dtype=torch.float32)),
           ('f32_uniform', lambda g: torch.rand(n, generator=g, device=device, dtype=torch.float32))]
    for name, fn in f32:
        k += 1
        fixed(name, 'float', nat.F32, fn(_gen(SEED + k * 1000 + rank, device)), SEED + k)
    for name, card in (('str_card100', 100), ('str_card1e5', 10 ** 5), ('str_card1e8', 10 ** 8)):
        k += 1
        g = _gen(SEED + k * 1000 + rank, device)
        labels = _bounded_zipf(n, 1.1, card, g, device)
        offsets, data = _string_column(labels, card, device)
        del labels
        c = DeviceColumn(name, 'string', n, 'bytes')
        c.offsets, c.data, c.offset_width = offsets, data, 8
        c.validity = _validity(n, _gen(SEED + k * 131 + rank, device), device)
        cols.append(c)
    k += 1
    lo = (np.datetime64('1688-01-01') - np.datetime64('1970-01-01')).astype(int)
    hi = (np.datetime64('2101-12-31') - np.datetime64('1970-01-01')).astype(int)
    days = torch.randint(int(lo), int(hi) + 1, (n,), generator=_gen(SEED + k * 1000 + rank, device),
                         device=device, dtype=torch.int32)
    fixed('date', 'date', nat.I32, days, SEED + k)
    torch.cuda.synchronize()
    return DeviceTable(cols, n)


C4_LABELS = 5 * 10 ** 8
_U64 = (1 << 64) - 1


def _s64(c):
    """A u64 constant as the int64 with the same bits."""
    return c - (1 << 64) if c >= (1 << 63) else c


def _srl(x, s):
    """Logical right shift of int64 tensors holding u64 bits."""
    return (x >> s) & ((1 << (64 - s)) - 1)


def mix64_t(x):
    """splitmix64's finalizer on int64 tensors with u64 semantics (wrapping
    multiplies, logical shifts) -- the same map as tests/datagen.mix64_np."""
    x = x ^ _srl(x, 30)
    x = x * _s64(0xBF58476D1CE4E5B9)
    x = x ^ _srl(x, 27)
    x = x * _s64(0x94D049BB133111EB)
    return x ^ _srl(x, 31)


def _hex16_column(keys, device, chunk=1 << 26):
    """utf8 (int64 offsets): each u64 key (int64 bits) -> its 16 lower-case hex digits."""
    n = keys.numel()
    offsets = torch.arange(n + 1, dtype=torch.int64, device=device) * 16
    data = torch.zeros(16 * n + 16, dtype=torch.uint8, device=device)
    hexd = _HEX.to(device)
    shifts = torch.arange(60, -4, -4, dtype=torch.int64, device=device)
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        nib = (keys[s:e, None] >> shifts[None, :]) & 15     # (sign-extending shift: the mask keeps the nibble)
        data[16 * s:16 * e] = hexd[nib].reshape(-1)
    return offsets, data


def make_c4_shard(rows_total, rank, world, device, labels=C4_LABELS):
    """`rows_total` rows, no nulls --
      u32_range_i64  int64 U[0, 2^32)  (near-unique: D ~ 0.9e9 at 1e9 rows; NUM)
      hex_id         utf8, the 16 hex digits of mix64(label), label ~ zipf(1.05)
                     over `labels` labels (exact distinct + top-50; CAT)
    generated in HBM from fixed seeds (the law of tests/datagen.c4_table)."""
    from spark_df_profiling.columns import DeviceColumn, DeviceTable
    from spark_df_profiling import _native as nat
    per = rows_total // world
    start = rank * per
    n = per if rank < world - 1 else rows_total - start
    g = _gen(SEED + 4001 * 1000 + rank, device)
    c = DeviceColumn('u32_range_i64', 'bigint', n, 'fixed', nat.I64)
    c.values = torch.randint(0, 2 ** 32, (n,), generator=g, device=device, dtype=torch.int64)
    lab = _bounded_zipf(n, 1.05, labels, _gen(SEED + 4002 * 1000 + rank, device), device)
    keys = mix64_t(lab)
    del lab
    h = DeviceColumn('hex_id', 'string', n, 'bytes')
    h.offsets, h.data = _hex16_column(keys, device)
    h.offset_width = 8
    del keys
    torch.cuda.synchronize()
    return DeviceTable([c, h], n)


C5_COLS = 512
C5_FACTORS = 4


def make_c5_shard(rows_total, rank, world, device, ncols=C5_COLS):
    """`rows_total` x `ncols` fp32, no nulls.  Each column is
    a low-rank shared factor plus unit noise, x_j = F a_j + e_j with F ~ N(0,1)
    (rows x 4) and loadings a_j ~ U(-1.5, 1.5)^4, so the Pearson matrix spans
    (-1, 1); generated column by column in HBM from fixed seeds."""
    from spark_df_profiling import _native as nat
    from spark_df_profiling.columns import DeviceColumn, DeviceTable
    per = rows_total // world
    start = rank * per
    n = per if rank < world - 1 else rows_total - start
    g = _gen(SEED + 777 * 1000 + rank, device)
    F = torch.randn(n, C5_FACTORS, generator=g, device=device, dtype=torch.float32)
    gl = torch.Generator()
    gl.manual_seed(SEED + 778)
    L = ((torch.rand(C5_FACTORS, ncols, generator=gl, dtype=torch.float64) * 3.0 - 1.5)
         .to(torch.float32).to(device))
    cols = []
    for j in range(ncols):
        gj = _gen(SEED + (1000 + j) * 1000 + rank, device)
        v = torch.randn(n, generator=gj, device=device, dtype=torch.float32)
        v.add_(F @ L[:, j])
        c = DeviceColumn('c%03d' % j, 'float', n, 'fixed', nat.F32)
        c.values = v
        c.validity = None
        cols.append(c)
    del F
    torch.cuda.synchronize()
    return DeviceTable(cols, n)


def table_bytes(table):
    """Resident bytes of the shard (values, offsets, string bytes, validity)."""
    b = 0
    for c in table.columns:
        for t in (c.values, c.validity, c.offsets, c.data):
            if t is not None:
                b += t.numel() * t.element_size()
    return b


# ----------------------------------------------------------------------------
# roofline: per-kernel (HIP events + algorithmic bytes annotated by the engine)
# and whole-profile (SURVEY.md §8d B_alg)
# ----------------------------------------------------------------------------

def profile_alg_bytes(table, raw):
    """B_alg = sum_numeric 3 n (w + 1/8) + sum_string n (o + L + 1/8)
    + sum_date n (w + 1/8) + sum_all 32 D, per shard (n = this rank's rows)."""
    from spark_df_profiling.engine import col_read_bytes
    b = 0.0
    for c in table.columns:
        info = raw['columns'][c.name]
        rb = col_read_bytes(c)
        if c.kind == 'fixed' and c.spark_type in ('double', 'float', 'bigint', 'int', 'smallint', 'tinyint'):
            b += 3 * rb
        else:
            b += rb
        b += 32.0 * info['distinct_count'] / max(1, int(os.environ.get('WORLD_SIZE', '1')))
    return b


_DT = {'f64': 'double', 'f32': 'float', 'i64': 'long', 'i32': 'int', 'i16': 'short', 'i8': 'signed char',
       'u64': 'unsigned long', 'u32': 'unsigned int'}


def label_kernels(label):
    """rocprof kernel-name prefixes behind one entry-point label
    (`sdp_<entry>[<dtype>/<stage>]`, engine.annotate)."""
    name, _, arg = label.partition('[')
    arg = arg.rstrip(']')
    dt, _, stage = arg.partition('/')
    if name == 'sdp_part_recs':
        b = 'true' if dt == 'bytes' else 'false'
        return ['sdp::part_%s_recs_kernel<%s>' % ('count' if stage == 'count' else 'scatter', b)]
    if name == 'sdp_part_rows':
        st = 'count' if stage == 'count' else 'scatter'
        if dt == 'bytes':
            return ['sdp::part_%s_rows_bytes_kernel' % st]
        return ['sdp::part_%s_rows_u64_kernel<%s>' % (st, _DT.get(dt, dt))]
    if name == 'sdp_part_rows_records':
        return ['sdp::part_records_rows_bytes_kernel']
    if name == 'sdp_part_dedup':
        return ['sdp::part_dedup_bytes_kernel<false>'] if dt == 'bytes' else ['sdp::part_dedup_u64']
    if name == 'sdp_part_dedup_blocks':         # the block-layout variants: <..., true>
        # (fixed keys: C3's block-layout columns are the near-unique ones, on
        # the half-space kernel; skewed columns keep the counted layout)
        return (['sdp::part_dedup_bytes_kernel<true>'] if dt == 'bytes'
                else ['sdp::part_dedup_u64_half_kernel<1, true>'])
    if name == 'sdp_part_l2_blocks':
        return ['sdp::part_l2_blocks_kernel<%s>' % ('true' if dt == 'bytes' else 'false')]
    if name in ('sdp_pass1', 'sdp_pass2', 'sdp_pass2_count', 'sdp_pass1_batch', 'sdp_pass2_count_batch'):
        return ['sdp::%s_kernel<%s' % (name[4:], _DT.get(dt, dt))]
    if name == 'sdp_distinct32':
        return ['sdp::d32_']
    if name == 'sdp_gram':
        return ['sdp::gram_kernel<', 'sdp::gram_wide_kernel', 'sdp::gram_reduce_kernel']
    return []


# PMC traffic summary the bench reads `roofline.traffic` from, chosen by name
# (never by file mtime, which a git checkout scrambles): the newest committed
# summary of the default workload (tools/gpu_traffic.sh -> tools/traffic_summary.py).
TRAFFIC_SUMMARY = {'c3': 'profiles/r06s_c3_traffic.json', 'c5': 'profiles/r06o_c5_traffic.json'}


def pmc_traffic(label, path, rows=None, workload=None):
    """HBM bytes per launch of the kernel(s) behind `label` from the PMC
    summary at `path` (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE passes over this
    bench), or (None, None).  Only a summary of the same run shape counts: its
    `rows` must equal this run's rows and its `workload` (when recorded) this
    workload, and it must hold every kernel the label stands for -- a summary of
    another size would give a meaningless bytes ratio."""
    if not path:
        return None, None
    full = path if os.path.isabs(path) else os.path.join(ROOT, path)
    if not os.path.exists(full):
        return None, None
    with open(full) as fh:
        summ = json.load(fh)
    if rows is not None and int(summ.get('rows', -1)) != int(rows):
        return None, None
    if workload is not None and summ.get('workload', workload) != workload:
        return None, None
    pre = label_kernels(label)
    if not pre or not all(any(k.startswith(p) for k in summ['kernels']) for p in pre
                          if not p.startswith('sdp::gram_kernel<')):
        return None, None
    hits = [v for k, v in summ['kernels'].items() if any(k.startswith(p) for p in pre)]
    if not hits:
        return None, None
    # one entry-point launch runs each matching kernel once (e.g. gram + reduce)
    n = max(v['dispatches'] for v in hits)
    return sum(v['traffic_bytes'] * v['dispatches'] for v in hits) / n, path


def roofline(rec, steps, step_s, prof_bytes, traffic_path=None, rows=None, workload=None):
    """Dominant kernel (entry point + label) by total HIP-event time -> achieved
    GB/s = its algorithmic bytes per launch / its mean launch duration."""
    torch.cuda.synchronize()
    tot, nbytes, nl = {}, {}, {}
    for k, v in rec.items():
        tot[k] = sum(a.elapsed_time(b) for a, b, _ in v)
        nl[k] = len(v)
        nbytes[k] = sum(x for _, _, x in v if x is not None) if any(x is not None for _, _, x in v) else None
    dom = max((k for k in tot if nbytes[k]), key=lambda k: tot[k])
    avg_ms = tot[dom] / nl[dom]
    per_launch = nbytes[dom] / nl[dom]
    achieved = per_launch / (avg_ms * 1e-3) / 1e9
    prof_gbs = prof_bytes / step_s / 1e9
    traffic, tsrc = pmc_traffic(dom, traffic_path, rows, workload)
    out = {'bound': 'hbm', 'kernel': dom, 'achieved': round(achieved, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
           'frac': round(achieved / HBM_PEAK_GBS, 4),
           'traffic': int(traffic) if traffic is not None else None,
           'traffic_unit': 'bytes per launch (PMC FETCH_SIZE x2 + WRITE_SIZE)',
           'traffic_over_alg': round(traffic / per_launch, 3) if traffic is not None else None,
           'traffic_source': tsrc,
           'launches_per_step': nl[dom] // steps, 'avg_launch_ms': round(avg_ms, 4),
           'alg_bytes_per_launch': int(per_launch),
           'share_of_step': round(tot[dom] / steps / (step_s * 1e3), 3),
           'whole_profile': {'alg_bytes_per_step': int(prof_bytes), 'achieved': round(prof_gbs, 1),
                             'frac': round(prof_gbs / HBM_PEAK_GBS, 4)}}
    per_kernel = {k: {'ms_per_step': round(tot[k] / steps, 3), 'launches_per_step': nl[k] // steps,
                      'gbs': (round(nbytes[k] / (tot[k] * 1e-3) / 1e9, 1) if nbytes[k] and tot[k] > 0 else None)}
                  for k in sorted(tot, key=lambda k: -tot[k])}
    return out, per_kernel


# ----------------------------------------------------------------------------
# CPU baseline: the oracle (CPU restatement, not reference Spark) on a sample
# ----------------------------------------------------------------------------

def shard_to_arrow(shard):
    """A device table of the C3 generator as a host Arrow table (same values)."""
    import pyarrow as pa
    arrays = {}
    for c in shard.columns:
        n = c.length
        valid = np.unpackbits(c.validity[:(n + 7) // 8].cpu().numpy(), bitorder='little')[:n].astype(bool)
        if c.kind == 'bytes':
            offs = c.offsets.cpu().numpy()
            data = c.data.cpu().numpy().tobytes()
            arr = pa.LargeStringArray.from_buffers(n, pa.py_buffer(offs.tobytes()), pa.py_buffer(data),
                                                   pa.py_buffer(np.packbits(valid, bitorder='little').tobytes()))
        elif c.spark_type == 'date':
            arr = pa.array(c.values.cpu().numpy(), type=pa.date32(), mask=~valid)
        else:
            arr = pa.array(c.values.cpu().numpy(), mask=~valid)
        arrays[c.name] = arr
    return pa.table(arrays)


def cpu_share(columns=16):
    """(processes the baseline uses, how that was decided).  The CPUs this job
    may run on are the affinity mask, bounded by the cgroup CPU quota when one
    is set (os.cpu_count() reports the whole machine); the restatement runs one
    column per process, so at most `columns` processes do work."""
    from spark_df_profiling.utils import available_cpus
    visible = os.cpu_count() or 1
    try:
        allowed = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        allowed = visible
    avail, src = available_cpus()
    return max(1, min(avail, columns)), {'os_cpu_count': visible, 'affinity_cpus': allowed,
                                         'available_cpus': avail, 'source': src, 'columns': columns}


def cpu_baseline(sample_rows, device):
    """The vectorised oracle (oracle/fast.py: chunked exact-sum moments,
    introselect quantiles, sort/hash distinct counts, Arrow value counts) over
    a bounded sample of the same C3 generator, its columns spread over a
    spawned process pool (oracle.fast.start_pool, started before this process
    touched the GPU).  A CPU restatement, not reference Spark: there is no
    pyspark or JVM in the image."""
    from oracle import fast
    shard = make_c3_shard(sample_rows, 0, 1, device)
    table = shard_to_arrow(shard)
    del shard
    torch.cuda.empty_cache()
    workers = fast.pool_workers()
    t0 = time.perf_counter()
    fast.describe(table)
    dt = time.perf_counter() - t0
    _, host = cpu_share()
    return {'value': round(sample_rows / dt, 1), 'unit': 'rows/s', 'cores': workers, 'kind': 'port',
            'host_cpus': host,
            'sample': '%d rows x 16 cols of the same C3 generator; oracle/fast.py vectorised numpy/Arrow '
                      'restatement, one column per process on %d processes (%d CPUs available by the %s; '
                      'one column per process caps it at 16) (CPU restatement, not reference Spark: '
                      'no pyspark/JVM in the image), %.1f s' % (sample_rows, workers, host['available_cpus'],
                                                               host['source'], dt)}


def gram_roofline(rec, steps, ncols, n_rows, traffic_path=None, rows=None):
    """C5: the Pearson Gram on the fp64 matrix cores.  F_alg = n C (C + 1)
    flop per launch (symmetric X^T X, one multiply-add per
    unique entry) over the launch's average HIP-event duration."""
    torch.cuda.synchronize()
    ev = rec.get('sdp_gram', [])
    if not ev:
        return None
    ms = sum(a.elapsed_time(b) for a, b, _ in ev) / len(ev)
    flop = float(n_rows) * ncols * (ncols + 1)
    tfs = flop / (ms * 1e-3) / 1e12
    alg_bytes = sum(x for _, _, x in ev if x is not None) / len(ev)
    traffic, tsrc = pmc_traffic('sdp_gram', traffic_path, rows, 'c5')
    return {'bound': 'mfma', 'kernel': 'sdp_gram (gram_wide_kernel + gram_reduce_kernel<128>, v_mfma_f64_16x16x4f64)',
            'achieved': round(tfs, 2), 'peak': FP64_MFMA_PEAK_TFS, 'unit': 'TFLOP/s',
            'frac': round(tfs / FP64_MFMA_PEAK_TFS, 4),
            'traffic': int(traffic) if traffic is not None else None,
            'traffic_unit': 'HBM bytes per launch (PMC FETCH_SIZE x2 + WRITE_SIZE)', 'traffic_source': tsrc,
            'flop_per_launch': flop, 'avg_launch_ms': round(ms, 4), 'launches_per_step': len(ev) // steps,
            'hbm_alg_bytes_per_launch': int(alg_bytes),
            'hbm_achieved_gbs': round(alg_bytes / (ms * 1e-3) / 1e9, 1)}


class ReadbackCensus:
    """Counts the blocking host syncs describe() makes while active: device->host
    readbacks (device tensors read by .cpu() / .item() / .tolist() / .to('cpu'))
    and pageable host->device copies (torch.tensor(..., device=cuda), .to(cuda) /
    .cuda() of a host tensor without non_blocking from pinned memory): PyTorch
    synchronises the stream after either, so each sits on the step's critical
    path.  (The engine's own uploads go through pinned memory with
    non_blocking=True and are not counted.)  Run on the last warmup step,
    outside the timed region."""

    def __init__(self):
        self.count = 0
        self.h2d = 0
        self._saved = []
        # SDP_READBACK_SITES=1: also tally the package line each sync comes from
        self.sites = {} if os.environ.get('SDP_READBACK_SITES') == '1' else None

    def _site(self):
        import traceback
        for fr in reversed(traceback.extract_stack()[:-2]):
            if 'spark_df_profiling' in fr.filename:
                return '%s:%d %s' % (os.path.basename(fr.filename), fr.lineno, fr.name)
        return '?'

    def _note(self, kind):
        if kind == 'h2d':
            self.h2d += 1
        else:
            self.count += 1
        if self.sites is not None:
            key = '%s %s' % (kind, self._site())
            self.sites[key] = self.sites.get(key, 0) + 1

    def _wrap(self, owner, name, pred):
        orig = getattr(owner, name)
        census = self

        def f(*a, **k):
            kind = pred(*a, **k)
            if kind:
                census._note(kind)
            return orig(*a, **k)
        self._saved.append((owner, name, orig))
        setattr(owner, name, f)

    def __enter__(self):
        def is_cuda(dev):
            return dev is not None and not isinstance(dev, torch.dtype) and str(dev).startswith('cuda')

        def to_pred(t, *a, **k):
            dev = k.get('device', a[0] if a else None)
            if isinstance(dev, torch.Tensor):
                dev = dev.device
            if isinstance(dev, torch.dtype) or dev is None:
                return None
            if t.is_cuda and str(dev).startswith('cpu'):
                return 'readback'
            if not t.is_cuda and is_cuda(dev) and not (k.get('non_blocking') and t.is_pinned()):
                return 'h2d'
            return None

        def cuda_pred(t, *a, **k):
            return 'h2d' if not t.is_cuda and not (k.get('non_blocking') and t.is_pinned()) else None

        def tensor_pred(*a, **k):
            return 'h2d' if is_cuda(k.get('device')) else None
        self._wrap(torch.Tensor, 'cpu', lambda t, *a, **k: 'readback' if t.is_cuda else None)
        self._wrap(torch.Tensor, 'item', lambda t, *a, **k: 'readback' if t.is_cuda else None)
        self._wrap(torch.Tensor, 'tolist', lambda t, *a, **k: 'readback' if t.is_cuda else None)
        self._wrap(torch.Tensor, 'to', to_pred)
        self._wrap(torch.Tensor, 'cuda', cuda_pred)
        self._wrap(torch, 'tensor', tensor_pred)
        return self

    def __exit__(self, *exc):
        for owner, name, orig in reversed(self._saved):
            setattr(owner, name, orig)
        return False


def launch_cmd(argv, gpus, env):
    """The child command that runs `gpus` rank processes of this bench, or None
    when this process should run the step itself: --gpus 1, or a launcher
    (torchrun / the driver) already set WORLD_SIZE.  One rank per GPU,
    rendezvous on 127.0.0.1 at a free port."""
    if gpus <= 1 or 'WORLD_SIZE' in env:
        return None
    import socket
    with socket.socket() as sk:
        sk.bind(('127.0.0.1', 0))
        port = sk.getsockname()[1]
    return [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', str(gpus),
            '--master-addr', '127.0.0.1', '--master-port', str(port), os.path.abspath(__file__)] + list(argv)


def check_world(gpus, world, ranks_seen):
    """A rank's world must be what --gpus asked for (a silent one-GPU run of an
    N-GPU metric point is the failure this guards)."""
    if world != gpus or ranks_seen != gpus:
        raise SystemExit('bench.py: --gpus %d but the process group has world_size %d (%d ranks answered)'
                         % (gpus, world, ranks_seen))


def run_ranks(cmd):
    """Start the rank processes as children (this process never touches the
    GPU), stream their stderr, re-print rank 0's JSON line, return their rc."""
    import subprocess
    p = subprocess.run(cmd, stdout=subprocess.PIPE, text=True)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith('{')]
    other = [ln for ln in p.stdout.splitlines() if not ln.startswith('{')]
    if other:
        print('\n'.join(other), file=sys.stderr)
    if p.returncode == 0 and not lines:
        print('bench.py: the rank processes printed no JSON line', file=sys.stderr)
        return 1
    if lines:
        print(lines[-1])
    return p.returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=3)
    ap.add_argument('--warmup', type=int, default=1)
    ap.add_argument('--workload', choices=('c3', 'c4', 'c5'), default='c3',
                    help='c3: 1e9 x 16 mixed (the metric); c4: 1e9-row high-cardinality int64 + hex ids '
                         '(exact distinct + top-50); c5: 1e7 x 512 fp32 (Pearson on MFMA)')
    ap.add_argument('--rows', type=int, default=None)
    ap.add_argument('--cpu-sample-rows', type=int, default=1 << 24)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-plots', action='store_true')
    ap.add_argument('--traffic', default=None, help='PMC traffic summary (default: TRAFFIC_SUMMARY[workload])')
    ap.add_argument('--workers', type=int, default=None,
                    help='columns profiled concurrently per GPU (default: SDP_COLUMN_WORKERS or 1)')
    args = ap.parse_args()
    # --gpus N without a launcher: N rank processes as children, started
    # before anything here touches the GPU or starts a worker pool
    cmd = launch_cmd(sys.argv[1:], args.gpus, os.environ)
    if cmd is not None:
        sys.exit(run_ranks(cmd))
    if args.rows is None:
        args.rows = 10 ** 7 if args.workload == 'c5' else 10 ** 9
    traffic_path = args.traffic if args.traffic is not None else TRAFFIC_SUMMARY.get(args.workload)

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    if not args.no_plots:
        # histogram rendering workers (spawned before this process touches the GPU)
        from spark_df_profiling import plot
        plot.start_pool()
    want_cpu = world == 1 and not args.no_cpu_baseline and args.workload == 'c3'
    if want_cpu:
        # the CPU baseline's worker processes, likewise spawned before any GPU call
        sys.path.insert(0, ROOT)
        from oracle import fast
        fast.start_pool(cpu_share()[0])
    local = int(os.environ.get('LOCAL_RANK', '0'))
    # (local % devices: a gloo rehearsal may put several ranks on one GPU)
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    device = torch.device('cuda', local)
    comm = None
    # SDP_FORCE_SHARDED=1 at one rank: the sharded code paths over a one-rank
    # RCCL group (per-round collectives, owner exchanges), for measuring their
    # cost on one GPU; the JSON line says so in config.parallelism
    force_sharded = os.environ.get('SDP_FORCE_SHARDED', '0') == '1'
    if world > 1 or force_sharded:
        import torch.distributed as dist
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        if 'MASTER_PORT' not in os.environ:
            import socket
            with socket.socket() as sk:
                sk.bind(('127.0.0.1', 0))
                os.environ['MASTER_PORT'] = str(sk.getsockname()[1])
        os.environ.setdefault('RANK', str(rank))
        os.environ.setdefault('WORLD_SIZE', str(world))
        backend = os.environ.get('SDP_DIST_BACKEND', 'nccl')      # nccl = RCCL over xGMI
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=device)
        else:
            dist.init_process_group(backend)
        from spark_df_profiling.comm import TorchComm
        comm = TorchComm()
    ranks_seen = 1
    if world > 1:
        # count the ranks through the backend itself (a one-element all-reduce)
        one = torch.ones(1, dtype=torch.float32, device=device)
        ranks_seen = int(comm.allreduce_sum(one).item())
    if world > 1 or args.gpus > 1:
        check_world(args.gpus, world, ranks_seen)

    from spark_df_profiling import describe
    from spark_df_profiling import _native as nat
    from spark_df_profiling.describe import column_workers
    from spark_df_profiling.engine import Engine

    t_gen = time.perf_counter()
    if args.workload == 'c3':
        table = make_c3_shard(args.rows, rank, world, device)
    elif args.workload == 'c4':
        table = make_c4_shard(args.rows, rank, world, device)
    else:
        table = make_c5_shard(args.rows, rank, world, device)
    t_gen = time.perf_counter() - t_gen

    column_workers_used = column_workers(Engine(device=device, comm=comm), args.workers)

    def step(raw=None):
        return describe(table, comm=comm, plots=not args.no_plots, raw=raw, workers=args.workers)

    readbacks = h2d_syncs = None
    for i in range(args.warmup):
        if i == args.warmup - 1:
            with ReadbackCensus() as census:
                step()
            readbacks, h2d_syncs = census.count, census.h2d
            if census.sites is not None and rank == 0:
                for k, v in sorted(census.sites.items(), key=lambda kv: -kv[1]):
                    print('sync site %3d  %s' % (v, k), file=sys.stderr)
        else:
            step()

    def barrier():
        # every rank's queued work done and every rank here: a one-element
        # all-reduce on the stream, then a device sync.  (dist.barrier() over
        # RCCL polls its completion in 10 ms sleeps: a kernel trace of the
        # forced-sharded 1.25e8-row step showed 16.3 ms of idle GPU inside it,
        # profiles/r03o_shd_gaps.txt.)
        if comm is not None:
            comm.allreduce_sum_(torch.ones(1, dtype=torch.float32, device=device))
        torch.cuda.synchronize()

    raw = {}
    barrier()
    ms0 = torch.cuda.memory_stats(device)
    rec = nat.start_recording()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(raw if i == 0 else None)
    barrier()
    t1 = time.perf_counter()
    nat.stop_recording()
    ms1 = torch.cuda.memory_stats(device)
    # caching-allocator activity inside the timed steps (device mallocs/frees
    # synchronise; the steady state should have none)
    alloc = {k: ms1.get(k, 0) - ms0.get(k, 0) for k in ('num_device_alloc', 'num_device_free', 'num_alloc_retries')}
    alloc['peak_reserved_gb'] = round(ms1.get('reserved_bytes.all.peak', 0) / 1e9, 1)
    elapsed = t1 - t0
    if comm is not None:
        el = torch.tensor([elapsed], dtype=torch.float64, device=device)
        elapsed = float(torch.stack(comm.allgather(el)).max().item())
    step_s = elapsed / args.steps
    rl, per_kernel = roofline(rec, args.steps, step_s, profile_alg_bytes(table, raw), traffic_path,
                              args.rows, args.workload)
    ncols = len(table.columns)
    # quantile-window candidates written by pass 1, as a fraction of each NUM
    # column's counted rows (sum over its windows of the keys strictly inside)
    cand = {}
    for name, b in raw.get('columns', {}).items():
        p1 = b.get('p1')
        if p1 and p1['count']:
            cand[name] = round(sum(p1['w_in']) / p1['count'], 4)
    if args.workload == 'c5':
        hbm_rl = rl
        rl = gram_roofline(rec, args.steps, ncols, table.num_rows, traffic_path, args.rows)
        rl['hbm_dominant'] = {k: hbm_rl[k] for k in ('kernel', 'achieved', 'frac', 'avg_launch_ms')}
        rl['whole_profile'] = hbm_rl['whole_profile']

    if rank != 0:
        return
    if args.workload == 'c3':
        workload = ('C3: %d rows x 16 mixed columns (6 f64, 4 i64, 2 f32, 3 utf8, 1 date32), 5%% nulls, '
                    'row-sharded' % args.rows)
    elif args.workload == 'c4':
        workload = ('C4: %d rows: int64 U[0,2^32) + utf8 16-byte hex ids zipf(1.05) over 5e8 labels, '
                    'exact distinct + top-50, row-sharded' % args.rows)
    else:
        workload = ('C5: %d rows x %d fp32 columns (low-rank factor + noise, no nulls), full describe() '
                    'with the Pearson matrix on fp64 MFMA' % (args.rows, ncols))
    out = {
        'metric': METRIC, 'value': round(args.rows * args.steps / elapsed, 1), 'unit': 'rows/s',
        'n_gpus': world, 'ranks_seen': ranks_seen, 'steps': args.steps, 'warmup': args.warmup,
        'ms_per_step': round(1e3 * elapsed / args.steps, 2), 'higher_is_better': True, 'scaling': 'strong',
        'vs_baseline': None, 'dtype': 'f64', 'data': 'synthetic (torch, seeded, generated in HBM)',
        'config': {'workload': workload, 'rows': args.rows, 'columns': ncols,
                   'parallelism': 'row-shard x%d%s' % (world, ' (sharded paths forced)' if force_sharded else ''),
                   'plots': not args.no_plots,
                   'column_workers': column_workers_used},
        'roofline': rl,
        'whole_profile': rl.get('whole_profile'),
        'host_readbacks_per_step': readbacks,
        'host_blocking_h2d_per_step': h2d_syncs,
        'per_kernel': per_kernel,
        'quantile_candidates_frac': {'max': max(cand.values()) if cand else None,
                                     'mean': round(sum(cand.values()) / len(cand), 4) if cand else None},
        'resident_gb_per_gpu': round(table_bytes(table) / 1e9, 2),
        'allocator': alloc,
        'gen_s': round(t_gen, 1),
    }
    if want_cpu:
        del table
        torch.cuda.empty_cache()
        out['cpu_baseline'] = cpu_baseline(args.cpu_sample_rows, device)
    print(json.dumps(out))


if __name__ == '__main__':
    main()
