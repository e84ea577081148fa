"""Columns resident in HBM, in Arrow layout.

A `DeviceTable` is what the statistics engine reads: one `DeviceColumn` per
source column, each holding its Arrow buffers (values / validity bitmap /
offsets + bytes) as torch tensors on the GPU.  Arrow tables are uploaded once
(`DeviceTable.from_arrow`); synthetic tables can be built directly on the
device (bench.py) so no PCIe traffic is timed.

Spark type strings follow the reference's dispatch on
`df.select(column).dtypes[0][1]` (describe.py:137, :156-167).
"""

from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np
import pyarrow as pa
import torch

from . import _native as nat

INT_TYPES = ('tinyint', 'smallint', 'int', 'bigint')          # describe.py:158
FLOAT_TYPES = ('float', 'double', 'decimal')                  # describe.py:160
DATE_TYPES = ('date', 'timestamp')                            # describe.py:162


def spark_type_string(t: pa.DataType) -> str:
    """Arrow type -> Spark SQL type simpleString (what describe_1d dispatches on)."""
    if pa.types.is_dictionary(t):
        return spark_type_string(t.value_type)
    table = [
        (pa.types.is_int8, 'tinyint'), (pa.types.is_int16, 'smallint'), (pa.types.is_uint8, 'smallint'),
        (pa.types.is_int32, 'int'), (pa.types.is_uint16, 'int'), (pa.types.is_int64, 'bigint'),
        (pa.types.is_uint32, 'bigint'), (pa.types.is_uint64, 'decimal(20,0)'),
        (pa.types.is_float16, 'float'), (pa.types.is_float32, 'float'), (pa.types.is_float64, 'double'),
        (pa.types.is_boolean, 'boolean'), (pa.types.is_string, 'string'), (pa.types.is_large_string, 'string'),
        (pa.types.is_binary, 'binary'), (pa.types.is_large_binary, 'binary'),
        (pa.types.is_fixed_size_binary, 'binary'), (pa.types.is_date, 'date'),
        (pa.types.is_timestamp, 'timestamp'), (pa.types.is_null, 'null'),
    ]
    for pred, name in table:
        if pred(t):
            return name
    if pa.types.is_decimal(t):
        return 'decimal(%d,%d)' % (t.precision, t.scale)
    if pa.types.is_list(t) or pa.types.is_large_list(t) or pa.types.is_fixed_size_list(t):
        return 'array<%s>' % spark_type_string(t.value_type)
    if pa.types.is_struct(t):
        return 'struct<%s>' % ','.join('%s:%s' % (f.name, spark_type_string(f.type)) for f in t)
    if pa.types.is_map(t):
        return 'map<%s,%s>' % (spark_type_string(t.key_type), spark_type_string(t.item_type))
    raise NotImplementedError('Arrow type %s has no Spark SQL counterpart' % t)


_NUMERIC_DTYPE = {
    pa.int8(): (nat.I8, torch.int8), pa.int16(): (nat.I16, torch.int16), pa.int32(): (nat.I32, torch.int32),
    pa.int64(): (nat.I64, torch.int64), pa.uint8(): (nat.U8, torch.uint8), pa.uint16(): (nat.U16, torch.int16),
    pa.uint32(): (nat.U32, torch.int32), pa.uint64(): (nat.U64, torch.int64),
    pa.float32(): (nat.F32, torch.float32), pa.float64(): (nat.F64, torch.float64),
}


_TORCH_OF = {nat.I8: torch.int8, nat.I16: torch.int16, nat.I32: torch.int32, nat.I64: torch.int64,
             nat.U8: torch.uint8, nat.U16: torch.int16, nat.U32: torch.int32, nat.U64: torch.int64,
             nat.F32: torch.float32, nat.F64: torch.float64}


@dataclass
class DeviceColumn:
    """One Arrow column in HBM.

    kind: 'fixed' (numeric / date / timestamp / bool: `values` + `dtype`),
          'bytes' (utf8 / binary / decimal: `offsets` + `data`, or fixed width),
          'null'  (Arrow null type), 'nested' (rejected like the reference).
    """
    name: str
    spark_type: str
    length: int
    kind: str
    dtype: int = 0
    values: Optional[torch.Tensor] = None
    validity: Optional[torch.Tensor] = None
    bit_offset: int = 0
    offsets: Optional[torch.Tensor] = None
    data: Optional[torch.Tensor] = None
    offset_width: int = 4
    fixed_width: int = 0
    ts_unit: Optional[str] = None
    decimal_scale: int = 0
    arrow_type: Optional[pa.DataType] = None
    _keep: list = field(default_factory=list)

    # -- C ABI views ----------------------------------------------------------
    def sdp(self) -> nat.SdpColumn:
        c = nat.SdpColumn()
        c.d_values = self.values.data_ptr() if self.values is not None else None
        c.d_validity = self.validity.data_ptr() if self.validity is not None else None
        c.validity_bit_offset = self.bit_offset
        c.length = self.length
        c.dtype = self.dtype
        return c

    def sdp_bytes(self) -> nat.SdpBytesColumn:
        c = nat.SdpBytesColumn()
        c.d_data = self.data.data_ptr()
        c.d_offsets = self.offsets.data_ptr() if self.offsets is not None else None
        c.d_validity = self.validity.data_ptr() if self.validity is not None else None
        c.validity_bit_offset = self.bit_offset
        c.length = self.length
        c.offset_width = self.offset_width
        c.fixed_width = self.fixed_width
        return c

    @property
    def is_float(self) -> bool:
        return self.kind == 'fixed' and self.dtype in nat.FLOAT_DTYPES

    def slice_rows(self, start: int, stop: int) -> 'DeviceColumn':
        """Row range [start, stop) as a new view (used to shard across ranks)."""
        n = stop - start
        c = DeviceColumn(self.name, self.spark_type, n, self.kind, self.dtype, ts_unit=self.ts_unit,
                         decimal_scale=self.decimal_scale, arrow_type=self.arrow_type,
                         offset_width=self.offset_width, fixed_width=self.fixed_width)
        if self.validity is not None:
            b = self.bit_offset + start
            c.validity = self.validity[b // 8:]
            c.bit_offset = b % 8
        else:
            c.bit_offset = (self.bit_offset + start) % 8 if self.dtype == nat.BOOL else 0
        if self.kind == 'fixed':
            if self.dtype == nat.BOOL:
                b = self.bit_offset + start
                c.values = self.values[b // 8:]
                c.bit_offset = b % 8
                if self.validity is not None:
                    # bool values and validity must share one bit offset (Arrow)
                    assert (self.bit_offset + start) % 8 == c.bit_offset
            else:
                es = nat.ELEM_SIZE[self.dtype]
                if (start * es) % 16:
                    raise ValueError('row shard start must keep 16-byte alignment')
                c.values = self.values[start:stop]
        elif self.kind == 'bytes':
            c.data = self.data
            if self.fixed_width:
                c.data = self.data[start * self.fixed_width:]
            else:
                c.offsets = self.offsets[start:stop + 1]
        return c


@dataclass
class DeviceTable:
    columns: List[DeviceColumn]
    num_rows: int

    @property
    def column_names(self):
        return [c.name for c in self.columns]

    def column(self, name):
        for c in self.columns:
            if c.name == name:
                return c
        raise KeyError(name)

    def slice_rows(self, start, stop):
        return DeviceTable([c.slice_rows(start, stop) for c in self.columns], stop - start)

    STREAM_MIN_ROWS = 1 << 16

    @classmethod
    def from_arrow(cls, table, device=None, streamed=None):
        """Upload an Arrow table.  Tables of >= STREAM_MIN_ROWS rows (or with
        streamed=True) go through the pinned double-buffered staging pipeline
        (ingest.py); small ones column by column."""
        if isinstance(table, pa.RecordBatch):
            table = pa.Table.from_batches([table])
        device = torch.device(device or 'cuda')
        if streamed or (streamed is None and table.num_rows >= cls.STREAM_MIN_ROWS):
            from .ingest import from_arrow_streamed
            return from_arrow_streamed(table, device)
        cols = [column_from_arrow(name, table.column(name), device) for name in table.column_names]
        return cls(cols, table.num_rows)

    @classmethod
    def from_parquet(cls, path, columns=None, device=None, **kw):
        from .ingest import from_parquet
        return from_parquet(path, columns=columns, device=device, **kw)


# ----------------------------------------------------------------------------
# Arrow -> HBM upload
# ----------------------------------------------------------------------------

def _to_device(np_bytes: np.ndarray, device, pad: int = 0) -> torch.Tensor:
    n = np_bytes.nbytes
    t = torch.empty(n + pad, dtype=torch.uint8, device=device)
    if n:
        t[:n].copy_(torch.from_numpy(np.ascontiguousarray(np_bytes).view(np.uint8)), non_blocking=False)
    if pad:
        t[n:].zero_()
    return t


def _bitmap(buf, offset, length, device):
    """Arrow bitmap slice -> (device bytes padded by 8, bit offset)."""
    if buf is None:
        return None, 0
    first = offset // 8
    nbytes = (offset % 8 + length + 7) // 8
    raw = np.frombuffer(buf, dtype=np.uint8, count=nbytes, offset=first) if nbytes else np.zeros(0, np.uint8)
    return _to_device(raw, device, pad=8), offset % 8


def column_from_arrow(name, arr, device) -> DeviceColumn:
    if isinstance(arr, pa.ChunkedArray):
        arr = arr.combine_chunks() if arr.num_chunks != 1 else arr.chunk(0)
    if pa.types.is_dictionary(arr.type):
        arr = arr.dictionary_decode()
    t = arr.type
    spark_t = spark_type_string(t)
    n = len(arr)
    if any(k in spark_t for k in ('array', 'struct', 'map')):
        return DeviceColumn(name, spark_t, n, 'nested', arrow_type=t)
    if pa.types.is_null(t):
        return DeviceColumn(name, spark_t, n, 'null', arrow_type=t)
    if pa.types.is_float16(t):
        arr = arr.cast(pa.float32())
        t = arr.type
    if pa.types.is_date64(t):
        arr = arr.cast(pa.date32())
        t = arr.type
    bufs = arr.buffers()
    validity, bit_off = _bitmap(bufs[0], arr.offset, n, device) if arr.null_count else (None, 0)
    col = DeviceColumn(name, spark_t, n, 'fixed', arrow_type=t, validity=validity, bit_offset=bit_off)
    if pa.types.is_boolean(t):
        vals, voff = _bitmap(bufs[1], arr.offset, n, device)
        if validity is None:
            bit_off = voff
        col.dtype = nat.BOOL
        col.values = vals
        col.bit_offset = voff
        return col
    if pa.types.is_date32(t):
        col.dtype, tdt = nat.I32, np.int32
    elif pa.types.is_timestamp(t):
        col.dtype, tdt = nat.I64, np.int64
        col.ts_unit = t.unit
    elif t in _NUMERIC_DTYPE:
        col.dtype = _NUMERIC_DTYPE[t][0]
        tdt = {nat.I8: np.int8, nat.I16: np.int16, nat.I32: np.int32, nat.I64: np.int64, nat.U8: np.uint8,
               nat.U16: np.uint16, nat.U32: np.uint32, nat.U64: np.uint64, nat.F32: np.float32,
               nat.F64: np.float64}[col.dtype]
    elif pa.types.is_decimal(t):
        return _decimal_column(col, arr, device)
    elif (pa.types.is_string(t) or pa.types.is_binary(t) or pa.types.is_large_string(t)
          or pa.types.is_large_binary(t)):
        large = pa.types.is_large_string(t) or pa.types.is_large_binary(t)
        odt = np.int64 if large else np.int32
        offs = np.frombuffer(bufs[1], dtype=odt, count=n + 1, offset=arr.offset * np.dtype(odt).itemsize)
        data = np.frombuffer(bufs[2], dtype=np.uint8) if bufs[2] is not None else np.zeros(0, np.uint8)
        col.kind = 'bytes'
        col.offsets = _to_device(offs, device).view(torch.int64 if large else torch.int32)
        col.offset_width = 8 if large else 4
        col.data = _to_device(data, device, pad=16)
        return col
    elif pa.types.is_fixed_size_binary(t):
        w = t.byte_width
        data = np.frombuffer(bufs[1], dtype=np.uint8, count=n * w, offset=arr.offset * w)
        col.kind = 'bytes'
        col.fixed_width = w
        col.data = _to_device(data, device, pad=16)
        return col
    else:
        raise NotImplementedError('Column {c} is of type {t} and cannot be analyzed'.format(c=name, t=spark_t))
    vals = np.frombuffer(bufs[1], dtype=tdt, count=n, offset=arr.offset * np.dtype(tdt).itemsize)
    raw = _to_device(vals, device, pad=16)
    col.values = raw[:n * vals.itemsize].view(_TORCH_OF[col.dtype])
    return col


def _decimal_column(col, arr, device):
    """decimal128 -> 16-byte big-endian keys whose bytewise order is numeric order
    (sign bit flipped), grouped and tie-broken like any byte key."""
    n = len(arr)
    raw = np.frombuffer(arr.buffers()[1], dtype=np.uint8, count=n * 16, offset=arr.offset * 16).reshape(n, 16)
    dev = _to_device(raw.reshape(-1), device).view(n, 16)
    key = torch.flip(dev, dims=[1]).contiguous()        # little -> big endian
    key[:, 0] ^= 0x80                                   # two's complement -> unsigned order
    col.kind = 'bytes'
    col.fixed_width = 16
    col.decimal_scale = arr.type.scale
    flat = torch.zeros(n * 16 + 16, dtype=torch.uint8, device=device)
    flat[:n * 16] = key.reshape(-1)
    col.data = flat
    return col


def decimal_from_key(b: bytes, scale: int):
    import decimal
    v = bytearray(b)
    v[0] ^= 0x80
    i = int.from_bytes(bytes(v), 'big', signed=True)
    return decimal.Decimal(i).scaleb(-scale)
