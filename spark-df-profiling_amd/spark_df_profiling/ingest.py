"""Arrow / Parquet -> HBM staging pipeline.

The reference profiles a Spark DataFrame whose rows Spark reads from parquet
itself (`examples/Demo.ipynb:63`, `spark.read.parquet`); here the same column
chunks are decoded on the host (pyarrow, multithreaded) and streamed into the
Arrow-layout device buffers `describe()` reads:

* a decode thread produces RecordBatches (parquet row groups / Arrow chunks)
  while the main thread stages the previous batch, so host decode overlaps
  the uploads;
* every buffer of a batch is memcpy'd (several host threads) into one of two
  pinned staging buffers and copied to its final place in HBM with an
  asynchronous H2D copy on a dedicated stream; a staging buffer is reused
  once the event recorded after its copy has completed (double buffering);
* the device buffers are allocated once for the whole column (values and
  validity by row count; string bytes grow geometrically on the device), so
  nothing is concatenated on the host and nothing is re-copied.

Chunks whose bit offset is not byte aligned (validity / boolean bitmaps) are
re-aligned on the host before staging; string offsets are rebased on the
device (int32 until the column's bytes pass 2^31, then widened to int64).
Types the streaming path does not cover (decimal, nested, null, float16,
date64, dictionary) take `columns.column_from_arrow` on the whole column.
"""

from __future__ import annotations

import queue
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from typing import Iterable, List, Optional

import numpy as np
import pyarrow as pa
import torch

from . import _native as nat
from .columns import (_NUMERIC_DTYPE, _TORCH_OF, DeviceColumn, DeviceTable, column_from_arrow,
                      spark_type_string)

STAGE_BYTES = 64 << 20          # per pinned staging buffer
COPY_THREADS = 4


class PinnedStager:
    """Two pinned host buffers + a copy stream: host bytes -> device slice."""

    def __init__(self, device, stage_bytes=STAGE_BYTES, nbuf=2):
        self.device = device
        self.stream = torch.cuda.Stream(device=device)
        self.bufs = [torch.empty(stage_bytes, dtype=torch.uint8, pin_memory=True) for _ in range(nbuf)]
        self.views = [b.numpy() for b in self.bufs]
        self.events: List[Optional[torch.cuda.Event]] = [None] * nbuf
        self.i = 0
        self.pool = ThreadPoolExecutor(COPY_THREADS)
        self.bytes = 0

    def _fill(self, dst: np.ndarray, src: np.ndarray):
        n = src.nbytes
        if n < (4 << 20):
            dst[:n] = src
            return
        step = -(-n // COPY_THREADS)
        futs = [self.pool.submit(np.copyto, dst[o:min(n, o + step)], src[o:min(n, o + step)])
                for o in range(0, n, step)]
        for f in futs:
            f.result()

    def upload(self, src: np.ndarray, dst: torch.Tensor):
        """Copy the bytes of `src` (any dtype, contiguous) into the uint8 device
        tensor `dst` (same byte length), asynchronously."""
        src = np.ascontiguousarray(src).reshape(-1).view(np.uint8)
        n = src.nbytes
        assert dst.numel() == n, (dst.numel(), n)
        cap = self.bufs[0].numel()
        for o in range(0, n, cap):
            m = min(cap, n - o)
            ev = self.events[self.i]
            if ev is not None:
                ev.synchronize()                      # the copy out of this buffer is done
            self._fill(self.views[self.i], src[o:o + m])
            with torch.cuda.stream(self.stream):
                dst[o:o + m].copy_(self.bufs[self.i][:m], non_blocking=True)
                e = torch.cuda.Event()
                e.record(self.stream)
            self.events[self.i] = e
            self.i = (self.i + 1) % len(self.bufs)
        self.bytes += n

    def finish(self):
        self.stream.synchronize()
        self.pool.shutdown(wait=True)


def _bitmap_bytes(buf, offset, length, start_bit):
    """Bytes of an Arrow bitmap slice [offset, offset+length) re-aligned to begin
    at bit `start_bit % 8` of its first byte (0 when both are byte aligned).
    Returns (bytes, first_byte_is_partial)."""
    s = start_bit % 8
    tail = (s + length) % 8
    if buf is None:
        bits = np.ones(length, dtype=np.uint8)
    elif offset % 8 == 0 and s == 0:
        nb = (length + 7) // 8
        b = np.frombuffer(buf, dtype=np.uint8, count=nb, offset=offset // 8)
        if tail:                                    # Arrow leaves the padding bits unspecified
            b = b.copy()
            b[-1] &= np.uint8((1 << tail) - 1)
        return b, False
    else:
        nb = (offset % 8 + length + 7) // 8
        raw = np.frombuffer(buf, dtype=np.uint8, count=nb, offset=offset // 8)
        bits = np.unpackbits(raw, bitorder='little')[offset % 8:offset % 8 + length]
    bits = np.concatenate([np.zeros(s, np.uint8), bits])
    return np.packbits(bits, bitorder='little'), s != 0


class _ColumnSink:
    """Device buffers of one column, filled batch by batch.  `n` = the rows
    the stream will produce when known up front (buffers sized once), else a
    first capacity: the buffers then grow by 1.5x on the device (a stream of
    unknown length, e.g. Spark batches without a count)."""

    def __init__(self, name, t: pa.DataType, n, device, stager):
        self.name, self.t, self.n, self.device, self.st = name, t, n, device, stager
        self.spark_t = spark_type_string(t)
        self.row = 0
        self.nulls = 0
        self.fallback = []                          # chunks of a type the stream does not cover
        self.kind = None
        self.cap = n
        if pa.types.is_boolean(t):
            self.kind = 'bool'
        elif pa.types.is_date32(t) or pa.types.is_timestamp(t) or t in _NUMERIC_DTYPE:
            self.kind = 'fixed'
            if pa.types.is_date32(t):
                self.dtype, self.width = nat.I32, 4
            elif pa.types.is_timestamp(t):
                self.dtype, self.width = nat.I64, 8
            else:
                self.dtype = _NUMERIC_DTYPE[t][0]
                self.width = nat.ELEM_SIZE[self.dtype]
        elif pa.types.is_string(t) or pa.types.is_binary(t) or pa.types.is_large_string(t) \
                or pa.types.is_large_binary(t):
            self.kind = 'bytes'
            self.owidth = 4
            self.data = torch.empty(max(1 << 20, 16), dtype=torch.uint8, device=device)
            self.nbytes = 0
        if self.kind is not None:
            self._alloc_rows(n, 0)
            self._partials = {}                     # last byte written mid-byte, per bitmap

    def _alloc_rows(self, cap, used):
        """(Re)allocate the row-indexed buffers for `cap` rows, keeping the
        first `used` rows (copied on the staging stream, after their uploads)."""
        nbits = (cap + 7) // 8 + 8
        ub = (used + 7) // 8                       # bitmap bytes holding rows < used

        def grow(name, numel, dtype, keep, zero_from):
            old = getattr(self, name, None)
            new = torch.empty(numel, dtype=dtype, device=self.device)
            with torch.cuda.stream(self.st.stream):
                if old is not None and keep:
                    new[:keep].copy_(old[:keep], non_blocking=True)
                    old.record_stream(self.st.stream)
                new[zero_from:].zero_()
            setattr(self, name, new)
        grow('validity', nbits, torch.uint8, ub, ub)
        if self.kind == 'bool':
            grow('values', nbits, torch.uint8, ub, ub)
        elif self.kind == 'fixed':
            grow('values', cap * self.width + 16, torch.uint8, used * self.width, cap * self.width)   # padding
        elif self.kind == 'bytes':
            dt = torch.int32 if self.owidth == 4 else torch.int64
            grow('offsets', cap + 1, dt, used + 1 if used else 1, cap + 1)
            if not used:
                with torch.cuda.stream(self.st.stream):
                    self.offsets[:1].zero_()
        self.cap = cap

    def _ensure_rows(self, m):
        if self.row + m > self.cap:
            self._alloc_rows(max(self.row + m, int(self.cap * 1.5) + 8, 1 << 16), self.row)

    def _put_bits(self, which, buf, offset, length):
        """Append `length` bits (Arrow bitmap buffer at bit `offset`) at row
        self.row to the bitmap `which` ('validity' or 'values')."""
        dst = getattr(self, which)
        b, partial = _bitmap_bytes(buf, offset, length, self.row)
        first = self.row // 8
        if partial:
            # OR the first (shared) byte with what the previous chunk left in it
            b = b.copy()
            b[0] |= np.uint8(self._partials.get(which, 0))
        self.st.upload(b, dst[first:first + b.nbytes])
        self._partials[which] = int(b[-1]) if (self.row + length) % 8 else 0

    def add(self, arr: pa.Array):
        if self.kind is None:
            self.fallback.append(arr)
            return
        m = len(arr)
        self._ensure_rows(m)
        bufs = arr.buffers()
        self.nulls += arr.null_count
        self._put_bits('validity', bufs[0] if arr.null_count else None, arr.offset, m)
        if self.kind == 'bool':
            self._put_bits('values', bufs[1], arr.offset, m)
        elif self.kind == 'fixed':
            w = self.width
            src = np.frombuffer(bufs[1], dtype=np.uint8, count=m * w, offset=arr.offset * w)
            self.st.upload(src, self.values[self.row * w:(self.row + m) * w])
        else:
            large = pa.types.is_large_string(arr.type) or pa.types.is_large_binary(arr.type)
            odt = np.int64 if large else np.int32
            offs = np.frombuffer(bufs[1], dtype=odt, count=m + 1, offset=arr.offset * np.dtype(odt).itemsize)
            o0, o1 = int(offs[0]), int(offs[-1])
            nb = o1 - o0
            self._reserve(nb)
            if nb:
                data = np.frombuffer(bufs[2], dtype=np.uint8, count=nb, offset=o0)
                self.st.upload(data, self.data[self.nbytes:self.nbytes + nb])
            # offsets of rows row+1 .. row+m, rebased on the device
            if self.owidth == 4 and self.nbytes + nb >= (1 << 31):
                self._widen()
            tmp = torch.empty(m * np.dtype(odt).itemsize, dtype=torch.uint8, device=self.device)
            self.st.upload(offs[1:], tmp)
            with torch.cuda.stream(self.st.stream):
                src = tmp.view(torch.int64 if large else torch.int32).to(self.offsets.dtype)
                self.offsets[self.row + 1:self.row + m + 1] = src + (self.nbytes - o0)
                tmp.record_stream(self.st.stream)
            self.nbytes += nb
        self.row += m

    def _reserve(self, nb):
        need = self.nbytes + nb + 16
        if need <= self.data.numel():
            return
        cap = max(need, int(self.data.numel() * 1.5))
        new = torch.empty(cap, dtype=torch.uint8, device=self.device)
        with torch.cuda.stream(self.st.stream):
            new[:self.nbytes].copy_(self.data[:self.nbytes], non_blocking=True)
            self.data.record_stream(self.st.stream)
        self.data = new

    def _widen(self):
        with torch.cuda.stream(self.st.stream):
            wide = self.offsets.to(torch.int64)
            self.offsets.record_stream(self.st.stream)
        self.offsets = wide
        self.owidth = 8

    def finish(self) -> DeviceColumn:
        self.n = self.row
        if self.kind is None:
            arr = pa.chunked_array(self.fallback, type=self.t) if self.fallback else pa.array([], type=self.t)
            return column_from_arrow(self.name, arr, self.device)
        col = DeviceColumn(self.name, self.spark_t, self.n, 'fixed', arrow_type=self.t)
        col.validity = self.validity if self.nulls else None
        if self.kind == 'bool':
            col.dtype, col.values = nat.BOOL, self.values
        elif self.kind == 'fixed':
            col.dtype = self.dtype
            col.values = self.values[:self.n * self.width].view(_TORCH_OF[self.dtype])
            if pa.types.is_timestamp(self.t):
                col.ts_unit = self.t.unit
        else:
            col.kind = 'bytes'
            col.offsets, col.offset_width = self.offsets, self.owidth
            self.data[self.nbytes:self.nbytes + 16].zero_()
            col.data = self.data
        return col


def _streamable(t: pa.DataType) -> bool:
    return (pa.types.is_boolean(t) or pa.types.is_date32(t) or pa.types.is_timestamp(t) or t in _NUMERIC_DTYPE
            or pa.types.is_string(t) or pa.types.is_binary(t) or pa.types.is_large_string(t)
            or pa.types.is_large_binary(t))


def stream_batches(schema: pa.Schema, num_rows: Optional[int], batches: Iterable[pa.RecordBatch], device=None,
                   stats: Optional[dict] = None, rows_hint: Optional[int] = None) -> DeviceTable:
    """Upload a stream of RecordBatches (produced on a background thread while
    the previous one is staged) into one DeviceTable.  num_rows = the exact
    row count when known (checked), None for a stream of unknown length (the
    device buffers grow; `rows_hint` sizes them first)."""
    device = torch.device(device or 'cuda')
    t0 = time.perf_counter()
    st = PinnedStager(device)
    first_cap = num_rows if num_rows is not None else max(int(rows_hint or 0), 1 << 16)
    sinks = [_ColumnSink(f.name, f.type, first_cap, device, st) for f in schema]
    q: queue.Queue = queue.Queue(maxsize=2)
    err = []

    def produce():
        try:
            for b in batches:
                q.put(b)
        except BaseException as e:          # surfaced in the consumer
            err.append(e)
        q.put(None)

    th = threading.Thread(target=produce, daemon=True)
    th.start()
    rows = 0
    while True:
        b = q.get()
        if b is None:
            break
        if b.schema.names != schema.names:
            raise ValueError('record batch columns %s differ from the stream schema %s' % (b.schema.names,
                                                                                        schema.names))
        for s, a in zip(sinks, b.columns):
            s.add(a)
        rows += b.num_rows
    th.join()
    if err:
        raise err[0]
    if num_rows is not None and rows != num_rows:
        raise ValueError('stream produced %d rows, expected %d' % (rows, num_rows))
    num_rows = rows
    st.finish()
    table = DeviceTable([s.finish() for s in sinks], num_rows)
    torch.cuda.synchronize(device)
    if stats is not None:
        dt = time.perf_counter() - t0
        stats.update({'rows': num_rows, 'seconds': dt, 'rows_per_s': num_rows / dt if dt > 0 else 0.0,
                      'h2d_bytes': st.bytes, 'h2d_gbs': st.bytes / dt / 1e9 if dt > 0 else 0.0})
    return table


def from_arrow_streamed(table, device=None, stats=None) -> DeviceTable:
    """Arrow Table (any chunking) -> DeviceTable through the staging pipeline."""
    if isinstance(table, pa.RecordBatch):
        table = pa.Table.from_batches([table])
    return stream_batches(table.schema, table.num_rows, table.to_batches(), device, stats)


def from_parquet(path, columns=None, device=None, batch_rows=1 << 20, stats=None, readers=4) -> DeviceTable:
    """Parquet file -> DeviceTable: `readers` row groups decoded at once by
    pyarrow (each multithreaded) on background threads and handed over in file
    order, staged through pinned memory into HBM."""
    import pyarrow.parquet as pq
    pf = pq.ParquetFile(path)
    schema = pf.schema_arrow
    if columns is not None:
        schema = pa.schema([schema.field(c) for c in columns])
    batch_rows = max(8, batch_rows // 8 * 8)               # byte-aligned bitmap chunks
    ngroups = pf.metadata.num_row_groups

    local = threading.local()

    def read(i):
        # a ParquetFile reader is not safe for concurrent reads: one per thread
        if not hasattr(local, 'pf'):
            local.pf = pq.ParquetFile(path)
        return local.pf.read_row_group(i, columns=columns, use_threads=True)

    def batches():
        with ThreadPoolExecutor(max(1, readers)) as ex:
            window = []
            nxt = 0
            while nxt < ngroups and len(window) < readers:
                window.append(ex.submit(read, nxt))
                nxt += 1
            while window:
                tab = window.pop(0).result()
                if nxt < ngroups:
                    window.append(ex.submit(read, nxt))
                    nxt += 1
                for b in tab.to_batches(max_chunksize=batch_rows):
                    yield b

    return stream_batches(schema, pf.metadata.num_rows, batches(), device, stats)
