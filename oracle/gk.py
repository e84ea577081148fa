"""CPU restatement of Spark 2.x `percentile_approx` (TEST INFRASTRUCTURE ONLY).

Only tests/ and bench.py's cpu_baseline may import this module; the product
path runs the HIP kernels of sdp_numeric.hip (sdp_gk_quantiles).

The reference computes float-column quantiles with
``percentile_approx(c, p)`` (/root/reference/spark_df_profiling/describe.py:205-206),
i.e. Spark SQL's ApproximatePercentile with its default accuracy 10000.  Spark
is a third-party dependency that is absent here (no pyspark, no
JVM; version not pinned, effectively Spark 2.x).  This file restates the
published algorithm of Spark 2.1-2.4:

* org.apache.spark.sql.catalyst.util.QuantileSummaries -- insert into a head
  buffer of defaultHeadSize = 50000 values; a full head is sorted
  (java.util.Arrays.sort order: -0.0 before 0.0) and merged into the sorted
  samples with g = 1 and delta = floor(2 * relativeError * count) (0 for the
  first sample and for a new maximum); a summary of >= defaultCompressThreshold
  = 10000 samples is compressed (compressImmut: from the end, merge a sample into
  the head while g + head.g + head.delta < 2 * relativeError * count; the first
  sample is kept); merge = stable sort of the two sample lists by value, then
  compressImmut with the threshold of the receiving summary's count; query =
  the first sample whose [minRank, minRank + delta] lies within
  ceil(relativeError * count) of ceil(q * count) (q <= eps -> min,
  q >= 1 - eps -> max).
* ApproximatePercentile.PercentileDigest -- every add() clears isCompressed,
  so each non-empty partition's digest is compressed once more when the partial
  aggregate is serialized; the final aggregate starts from an empty digest and
  merges the partition digests (here: in partition order).

Parity is UNPINNED: no Spark run or fixture pins the element Spark returns,
which also depends on the DataFrame's partitioning.  The GPU emulation is
checked bit for bit against this restatement, and both against Spark's
documented rank window.
"""
import math
import struct

HEAD_SIZE = 50000
INT_MAX = 2 ** 31 - 1
COMPRESS_THRESHOLD = 10000


def total_key(v):
    """java.lang.Double.compare order (-0.0 < 0.0) as an unsigned key."""
    b = struct.unpack('<Q', struct.pack('<d', float(v)))[0]
    return (~b & 0xFFFFFFFFFFFFFFFF) if b >> 63 else (b | (1 << 63))


def _compress_immut(samples, threshold):
    if not samples:
        return []
    res = []
    head = samples[-1]
    i = len(samples) - 2
    while i >= 1:
        s1 = samples[i]
        if float(s1[1] + head[1] + head[2]) < threshold:
            head = (head[0], head[1] + s1[1], head[2])
        else:
            res.append(head)
            head = s1
        i -= 1
    res.append(head)
    if samples[0][0] <= head[0] and len(samples) > 1:
        res.append(samples[0])
    res.reverse()
    return res


class Summary:
    """QuantileSummaries with its head buffer (values as Python floats)."""

    def __init__(self, eps, sampled=None, count=0):
        self.eps = eps
        self.sampled = sampled if sampled is not None else []
        self.count = count
        self.head = []

    def insert(self, x):
        self.head.append(x)
        if len(self.head) >= HEAD_SIZE:
            r = self._with_head()
            if len(r.sampled) >= COMPRESS_THRESHOLD:
                return r.compress()
            return r
        return self

    def _with_head(self):
        if not self.head:
            return self
        cur = self.count
        srt = sorted(self.head, key=total_key)
        s = self.sampled
        new, si, n = [], 0, len(srt)
        for oi, x in enumerate(srt):
            while si < len(s) and s[si][0] <= x:
                new.append(s[si])
                si += 1
            cur += 1
            if not new or (si == len(s) and oi == n - 1):
                delta = 0
            else:
                delta = int(math.floor(2 * self.eps * cur))
            new.append((x, 1, delta))
        new.extend(s[si:])
        return Summary(self.eps, new, cur)

    def compress(self):
        ins = self._with_head()
        return Summary(self.eps, _compress_immut(ins.sampled, 2 * self.eps * ins.count), ins.count)

    def merge(self, other):
        if other.count == 0:
            return Summary(self.eps, list(self.sampled), self.count)
        if self.count == 0:
            return Summary(other.eps, list(other.sampled), other.count)
        res = sorted(self.sampled + other.sampled, key=lambda t: total_key(t[0]))    # stable
        return Summary(other.eps, _compress_immut(res, 2 * self.eps * self.count), other.count + self.count)

    def query(self, q):
        s = self.sampled
        if not s:
            return None
        if q <= self.eps:
            return s[0][0]
        if q >= 1 - self.eps:
            return s[-1][0]
        rank = min(int(math.ceil(q * self.count)), INT_MAX)     # Scala .toInt saturates
        target = math.ceil(self.eps * self.count)
        min_rank = 0
        for i in range(1, len(s) - 1):
            min_rank += s[i][1]
            max_rank = min_rank + s[i][2]
            if max_rank - target <= rank <= min_rank + target:
                return s[i][0]
        return s[-1][0]


def partition_digest(values, eps):
    """One partition's partial aggregate as serialized (compressed if any value was added)."""
    d = Summary(eps)
    added = False
    for v in values:
        d = d.insert(float(v))
        added = True
    return d.compress() if added else d


def percentile_approx(partitions, probs, accuracy=10000):
    """percentile_approx(c, p) for each p over `partitions` (sequences of the
    non-null, non-NaN values of each Spark partition in row order), partial
    digests merged in partition order."""
    eps = 1.0 / accuracy
    final = Summary(eps)
    for part in partitions:
        final = final.merge(partition_digest(part, eps))
    return [final.query(p) for p in probs]


def split_rows(values, valid, n_partitions):
    """Rows split into n_partitions contiguous ranges [p*n/P, (p+1)*n/P) (the
    engine's default partitioning), na.drop applied: non-null, non-NaN values."""
    n = len(values)
    out = []
    for p in range(n_partitions):
        r0, r1 = p * n // n_partitions, (p + 1) * n // n_partitions
        part = []
        for i in range(r0, r1):
            if valid is not None and not valid[i]:
                continue
            v = float(values[i])
            if v != v:
                continue
            part.append(v)
        out.append(part)
    return out
