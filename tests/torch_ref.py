"""Independent torch checks of describe() results at BASELINE sizes -- TEST
INFRASTRUCTURE ONLY (no libsdp call anywhere in this file).

At 1e8-1e9 rows the CPU oracle is too slow, so the GPU results are re-derived
on the same device with plain torch: comparisons, sorts (torch.unique) and
sums.  Sums are formed as 64 K-element chunk partials added exactly on the
host (math.fsum), so their error is <= ~16 eps * sum|x|, far inside the 1e-9
relative bound (the same construction as oracle/fast.py).  The formulas are
the reference's Spark aggregates:

  mean      Average: sum / count                       describe.py:194
  variance  var_samp = M2 / (n - 1); std = sqrt        describe.py:197-198
  skewness  sqrt(n) M3 / M2^1.5 (population)           describe.py:199
  kurtosis  n M4 / M2^2 - 3 (population, excess)       describe.py:196
  sum       double sum; integral columns wrap in int64 describe.py:200
  mad       sum |x - mean| / count                     describe.py:215-218
  percentile (int)  Spark Percentile interpolation     describe.py:207-208
  percentile_approx (float)  element of rank ceil(pN)  (A.5, exact element)
  histogram CASE-WHEN bins on the host-accumulated edges  describe.py:20-63
"""

import math

import numpy as np

from compare import close

CHUNK = 1 << 16
PROBS = (0.05, 0.25, 0.5, 0.75, 0.95)


def valid_mask(col, n):
    """Arrow validity bitmap -> bool tensor (all True without a bitmap)."""
    import torch
    if col.validity is None:
        return torch.ones(n, dtype=torch.bool, device=col.values.device)
    bits = col.validity[:(col.bit_offset + n + 7) // 8]
    shifts = torch.arange(8, dtype=torch.uint8, device=bits.device)
    v = ((bits[:, None] >> shifts[None, :]) & 1).bool().reshape(-1)
    return v[col.bit_offset:col.bit_offset + n]


def fsum_dev(t):
    """Sum of a 1-D fp64 tensor: chunk partials on the device, added exactly."""
    n = t.numel()
    m = n // CHUNK * CHUNK
    parts = t[:m].view(-1, CHUNK).sum(1).cpu().tolist() if m else []
    if m < n:
        parts.append(float(t[m:].sum().item()))
    return math.fsum(parts)


def fsum_cols(x):
    """Column sums of a 2-D fp64 tensor [n, C] (chunk partials added exactly)."""
    n, C = x.shape
    m = n // CHUNK * CHUNK
    parts = []
    if m:
        parts.append(x[:m].view(-1, CHUNK, C).sum(1).cpu().numpy())
    if m < n:
        parts.append(x[m:].sum(0, keepdim=True).cpu().numpy())
    p = np.concatenate(parts, axis=0)
    return [math.fsum(p[:, j].tolist()) for j in range(C)]


def moments(xs):
    """Spark's moment outputs of the fp64 values `xs` (two passes)."""
    n = xs.numel()
    s = fsum_dev(xs)
    mean = s / n
    # deviations from the ROUNDED mean K are exact (x and K are close), and the
    # central sums about the exact mean K + m follow from the power sums of d:
    # a rounded mean alone would leave 3 M2 |K - mean| in M3 (~1e-5 relative
    # skewness error for N(1e9, 1))
    d = xs - mean
    d2 = d * d
    s1 = fsum_dev(d)
    s2 = fsum_dev(d2)
    s3 = fsum_dev(d2 * d)
    s4 = fsum_dev(d2 * d2)
    del d, d2
    m = s1 / n
    m2 = s2 - s1 * s1 / n
    m3 = s3 - 3.0 * m * s2 + 2.0 * n * m ** 3
    m4 = s4 - 4.0 * m * s3 + 6.0 * m * m * s2 - 3.0 * n * m ** 4
    out = {'mean': mean, 'sum': s}
    out['variance'] = m2 / (n - 1) if n > 1 else float('nan')
    out['std'] = math.sqrt(out['variance']) if n > 1 else float('nan')
    out['skewness'] = math.sqrt(n) * m3 / math.sqrt(m2 * m2 * m2) if m2 else float('nan')
    out['kurtosis'] = n * m4 / (m2 * m2) - 3.0 if m2 else float('nan')
    return out


def spark_int_percentile(sorted_at, n, p):
    """Spark Percentile (A.4): linear interpolation at (n - 1) p; `sorted_at(r)`
    is the r-th smallest value (0-based)."""
    pos = (n - 1) * p
    lo, hi = math.floor(pos), math.ceil(pos)
    xl, xh = sorted_at(lo), sorted_at(hi)
    if lo == hi or xl == xh:
        return float(xl)
    return (hi - pos) * float(xl) + (pos - lo) * float(xh)


def accumulated_edges(vmin, vmax, bins):
    """describe.py:38-45: bin_width = (max - min) / float(bins); left edges by
    repeated addition from min, the last one popped."""
    width = (vmax - vmin) / float(bins)
    edges = [vmin]
    for _ in range(bins):
        edges.append(edges[-1] + width)
    edges.pop()
    return edges


def float_rank(n, p):
    if p <= 1e-4:
        return 1
    if p >= 1 - 1e-4:
        return n
    return min(max(int(math.ceil(p * n)), 1), n)


def check_numeric(name, col, st, row, nrows, uniq=None, counts=None, problems=None):
    """Compare one NUM column's describe() outputs (`row` of the variables
    frame, `st` = raw NumericStats) with torch re-derivations.  `uniq`,
    `counts`: torch.unique(valid values, sorted, return_counts) when the
    caller already has them (integral columns: exact quantiles + distinct).
    Returns the list of mismatches (empty = parity)."""
    import torch
    problems = [] if problems is None else problems

    def bad(key, got, want):
        problems.append('%s.%s: %r vs %r' % (name, key, got, want))

    x = col.values[:nrows]
    valid = valid_mask(col, nrows)
    xd = x.double()
    ok = valid & ~torch.isnan(xd) if col.is_float else valid
    cnt = int(ok.sum().item())
    if int(row['count']) != cnt:
        bad('count', int(row['count']), cnt)
    if int(row['n_missing']) != nrows - cnt:
        bad('n_missing', int(row['n_missing']), nrows - cnt)
    xs = xd[ok]
    del xd
    if float(xs.min().item()) != float(row['min']):
        bad('min', row['min'], float(xs.min().item()))
    if float(xs.max().item()) != float(row['max']):
        bad('max', row['max'], float(xs.max().item()))
    # moments
    mom = moments(xs)
    if not col.is_float:
        # Spark Sum of an integral column: LongType with two's-complement wrap
        mom['sum'] = float(int(x[valid].sum().item()))
    for key in ('mean', 'variance', 'std', 'sum'):
        if key == 'sum' and not col.is_float:
            # float(wrapped int64): exact (describe.py:200, upcast at :209)
            if float(row[key]) != mom[key]:
                bad(key, float(row[key]), mom[key])
            continue
        if not close(row[key], mom[key]):
            bad(key, float(row[key]), mom[key])
    for key in ('skewness', 'kurtosis'):
        if not close(row[key], mom[key], floor=1e-12):
            bad(key, float(row[key]), mom[key])
    # mad about the engine's own mean (the mean itself is checked above)
    mad = fsum_dev((xs - float(row['mean'])).abs()) / cnt
    if not close(row['mad'], mad):
        bad('mad', float(row['mad']), mad)
    # zeros over the full column (null/NaN never equal 0.0; -0.0 does)
    nz = int(((x.double() == 0.0) & valid).sum().item())
    if int(row['n_zeros']) != nz:
        bad('n_zeros', int(row['n_zeros']), nz)
    # histogram: CASE-WHEN bins from edges accumulated here from the checked
    # min / max (describe.py:40-45), not from the engine's own edges.  The
    # min / max reach generate_hist_data as float64 for every column type:
    # stats_df.ix[0] (describe.py:209) upcasts the mixed int64 / float agg row
    # before :211 and :226 (SURVEY.md A.6's int64 / float32 subtraction does
    # not happen)
    if col.is_float:
        vmin, vmax = float(xs.min().item()), float(xs.max().item())
    else:
        vmin, vmax = float(int(x[valid].min().item())), float(int(x[valid].max().item()))
    edges = accumulated_edges(vmin, vmax, len(st.hist_counts))
    if [float(e) for e in st.edges] != [float(e) for e in edges]:
        bad('histogram edges', [float(e) for e in st.edges], [float(e) for e in edges])
    ge = [int((xs >= float(e)).sum().item()) for e in edges]
    want = [ge[j] - ge[j + 1] for j in range(len(ge) - 1)] + [ge[-1]]
    if list(map(int, st.hist_counts)) != want:
        bad('histogram', list(map(int, st.hist_counts)), want)
    # outliers against the thresholds from q1/q3 (NaN counts as high, A.8)
    hi_t, lo_t = st.thresholds
    nan_valid = int((valid & torch.isnan(x.double())).sum().item()) if col.is_float else 0
    if int(row['high_idx']) != int((xs > hi_t).sum().item()) + nan_valid:
        bad('high_idx', int(row['high_idx']), int((xs > hi_t).sum().item()) + nan_valid)
    if int(row['low_idx']) != int((xs < lo_t).sum().item()):
        bad('low_idx', int(row['low_idx']), int((xs < lo_t).sum().item()))
    # quantiles
    if col.is_float:
        for p in PROBS:
            q = float(row['%d%%' % int(round(p * 100))])
            r = float_rank(cnt, p)
            below = int((xs < q).sum().item())
            le = int((xs <= q).sum().item())
            if not (below < r <= le):
                bad('%g quantile rank' % p, (below, le), r)
    else:
        if uniq is None:
            uniq, counts = torch.unique(x[valid], sorted=True, return_counts=True)
        cum = torch.cumsum(counts, 0)

        def at(r):
            i = int(torch.searchsorted(cum, torch.tensor([r], dtype=cum.dtype, device=cum.device),
                                       right=True).item())
            return int(uniq[i].item())
        for p in PROBS:
            q = float(row['%d%%' % int(round(p * 100))])
            want = spark_int_percentile(at, cnt, p)
            if q != want:
                bad('%g quantile' % p, q, want)
        if int(row['distinct_count']) != int(uniq.numel()):
            bad('distinct_count', int(row['distinct_count']), int(uniq.numel()))
    # derived driver-side arithmetic (describe.py:211-214)
    if float(row['range']) != float(row['max']) - float(row['min']):
        bad('range', row['range'], float(row['max']) - float(row['min']))
    return problems


def hex16_keys(col, nrows, chunk=1 << 26):
    """Strings of exactly 16 lower-case hex digits -> their u64 value, as int64
    with the sign bit flipped so that signed order is bytewise (= numeric)
    order.  Asserts every string is 16 hex digits."""
    import torch
    dev = col.data.device
    out = torch.empty(nrows, dtype=torch.int64, device=dev)
    offs = col.offsets
    assert col.fixed_width == 0
    lens = (offs[1:nrows + 1] - offs[:nrows]).to(torch.int64)
    assert int(lens.min().item()) == 16 and int(lens.max().item()) == 16
    base = int(offs[0].item())
    w = torch.tensor([1 << (60 - 4 * k) for k in range(15)] + [1], dtype=torch.int64, device=dev)
    for s in range(0, nrows, chunk):
        e = min(nrows, s + chunk)
        b = col.data[base + 16 * s: base + 16 * e].view(e - s, 16).to(torch.int64)
        nib = torch.where(b <= ord('9'), b - ord('0'), b - ord('a') + 10)
        assert int(nib.min().item()) >= 0 and int(nib.max().item()) <= 15
        # sum of nibble << shift; the top nibble's shift of 60 wraps into the sign bit
        v = (nib[:, :15] * w[:15]).sum(1) + nib[:, 15]
        out[s:e] = v ^ (-(1 << 63))
    return out


def key_to_hex(k_signed):
    return '%016x' % ((int(k_signed) & ((1 << 64) - 1)) ^ (1 << 63))


def top_groups(keys, k=50):
    """(distinct, [(key, count)] top-k by count desc, key asc, rows) of int64 keys."""
    import torch
    uk, uc = torch.unique(keys, sorted=True, return_counts=True)
    D = int(uk.numel())
    kk = min(k, D)
    vals, _ = torch.topk(uc, kk)
    T = int(vals[-1].item())                 # k-th largest count
    gt = uc > T
    sel_gt = torch.nonzero(gt).flatten()
    eq = torch.nonzero(uc == T).flatten()[:kk - int(sel_gt.numel())]   # smallest keys among the ties (uk sorted)
    sel = torch.cat([sel_gt, eq])
    pairs = list(zip(uk[sel].cpu().tolist(), uc[sel].cpu().tolist()))
    pairs.sort(key=lambda kc: (-kc[1], kc[0]))
    return D, pairs, int(uc.sum().item())


def short_string_keys(col, nrows, valid, chunk=1 << 24):
    """utf8/binary strings of <= 16 bytes with no NUL byte -> (k0, k1) int64
    tensors of the valid rows: bytes 0-7 and 8-15, big-endian, zero padded,
    sign bit flipped, so (k0, k1) in signed lexicographic order is the strings'
    bytewise order and equal pairs are equal strings (the padding is
    unambiguous without NULs).  Asserts both conditions."""
    import torch
    dev = col.data.device
    offs = col.offsets
    assert col.fixed_width == 0
    shifts = torch.arange(56, -8, -8, dtype=torch.int64, device=dev)          # big-endian byte weights
    j = torch.arange(16, dtype=torch.int64, device=dev)
    k0s, k1s = [], []
    flip = -(1 << 63)
    for s in range(0, nrows, chunk):
        e = min(nrows, s + chunk)
        vm = valid[s:e]
        o0 = offs[s:e][vm].to(torch.int64)
        ln = offs[s + 1:e + 1][vm].to(torch.int64) - o0
        assert int(ln.max().item()) <= 16 if ln.numel() else True
        inb = j[None, :] < ln[:, None]
        b = col.data[(o0[:, None] + j[None, :]).clamp(max=col.data.numel() - 1)].to(torch.int64) * inb
        assert not bool(((b == 0) & inb).any().item()), 'NUL byte in a string key'
        k0s.append(((b[:, :8] << shifts[None, :]).sum(1)) ^ flip)
        k1s.append(((b[:, 8:] << shifts[None, :]).sum(1)) ^ flip)
        del b, inb, o0, ln
    return torch.cat(k0s), torch.cat(k1s)


def key_pair_to_str(k0, k1):
    """Inverse of short_string_keys for one (k0, k1) pair."""
    raw = (((int(k0) ^ -(1 << 63)) & ((1 << 64) - 1)).to_bytes(8, 'big')
           + ((int(k1) ^ -(1 << 63)) & ((1 << 64) - 1)).to_bytes(8, 'big'))
    return raw.rstrip(b'\x00').decode('utf8')


def top_groups_pairs(k0, k1, k=50):
    """top_groups for 16-byte keys given as (k0, k1) pairs: groups by a
    lexicographic sort (two stable sorts), then (distinct, [((k0, k1), count)]
    top-k by count desc / key asc, rows).  Frees its inputs' copies as it goes."""
    import torch
    m = k0.numel()
    perm1 = torch.sort(k1, stable=True).indices
    k0p = k0[perm1]
    s0, perm2 = torch.sort(k0p, stable=True)
    del k0p
    perm = perm1[perm2]
    del perm1, perm2
    s1 = k1[perm]
    del perm
    new = torch.ones(m, dtype=torch.bool, device=k0.device)
    new[1:] = (s0[1:] != s0[:-1]) | (s1[1:] != s1[:-1])
    starts = torch.nonzero(new).flatten()
    del new
    D = int(starts.numel())
    counts = torch.diff(torch.cat([starts, torch.tensor([m], device=starts.device)]))
    kk = min(k, D)
    vals, _ = torch.topk(counts, kk)
    T = int(vals[-1].item())
    sel_gt = torch.nonzero(counts > T).flatten()
    eq = torch.nonzero(counts == T).flatten()[:kk - int(sel_gt.numel())]    # groups are in key order
    sel = torch.cat([sel_gt, eq])
    pos = starts[sel]
    pairs = list(zip(zip(s0[pos].cpu().tolist(), s1[pos].cpu().tolist()), counts[sel].cpu().tolist()))
    pairs.sort(key=lambda kc: (-kc[1], kc[0]))
    del s0, s1, starts, counts
    return D, pairs, m
