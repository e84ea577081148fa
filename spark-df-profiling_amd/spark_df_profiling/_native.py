"""ctypes binding of libsdp.so (include/sdp.h).

The library is the product: there is no Python or CPU fallback.  Loading fails
loudly when the shared object is missing, and every call raises
``NativeError`` with the library's message when it returns a non-zero status.

torch is imported first on purpose: torch-ROCm loads its own libamdhip64.so.7,
and libsdp.so (NEEDED libamdhip64.so.7) then binds to that same runtime, so
device pointers from the torch caching allocator are valid in our kernels.
"""

from __future__ import annotations

import ctypes
import threading
import os

import torch  # noqa: F401  (must precede the dlopen, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('SDP_LIBRARY', os.path.join(_HERE, 'lib', 'libsdp.so'))

MAX_WINDOWS = 5
PASS1_WAVES = 4          # SDP_PASS1_WAVES
PART_MAX_GRID = 1024     # SDP_PART_MAX_GRID
BITMAP_MAX_BITS = 1 << 20        # SDP_BITMAP_MAX_BITS

# the grouping policy (include/sdp.h SDP_*), shared with the library's coarse
# entries; _load() refuses a library built with other values
ABI_VERSION = 7              # SDP_ABI_VERSION (7: level-2 block layout, sdp_blocks)
HEAVY_MAX = 256              # SDP_HEAVY_MAX: the row kernels' heavy-key tables
HEAVY_MAX_REC = 1024         # SDP_HEAVY_MAX_REC: byte keys on the records kernel
HEAVY_MIN = 3                # SDP_HEAVY_MIN
PART_SAMPLE = 16384          # SDP_PART_SAMPLE
PART_SAMPLE_BYTES = 65536    # SDP_PART_SAMPLE_BYTES
PART_CHUNK = 131072          # SDP_PART_CHUNK
L2_BLOCK = 64                # SDP_L2_BLOCK: records per block of sdp_part_l2_blocks
L2_DESC_W = 4                # SDP_L2_DESC_W: u32 words per final-bucket descriptor
GSORT_MAX = 8192             # SDP_GSORT_MAX
BYTE_RECORD_ARRAYS = 3       # byte-key records: k0[], k1[], meta[] (sdp_records)
RECORD_WORD = 8              # bytes between one record's words in each array

# enum sdp_dtype
I8, I16, I32, I64, F32, F64, U8, U16, U32, U64, BOOL = 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11
FLOAT_DTYPES = (F32, F64)
ELEM_SIZE = {I8: 1, I16: 2, I32: 4, I64: 8, F32: 4, F64: 8, U8: 1, U16: 2, U32: 4, U64: 8}


class NativeError(RuntimeError):
    pass


class SdpColumn(ctypes.Structure):
    _fields_ = [('d_values', ctypes.c_void_p), ('d_validity', ctypes.c_void_p),
                ('validity_bit_offset', ctypes.c_int64), ('length', ctypes.c_int64),
                ('dtype', ctypes.c_int32), ('_pad', ctypes.c_int32)]


class SdpBytesColumn(ctypes.Structure):
    _fields_ = [('d_data', ctypes.c_void_p), ('d_offsets', ctypes.c_void_p), ('d_validity', ctypes.c_void_p),
                ('validity_bit_offset', ctypes.c_int64), ('length', ctypes.c_int64),
                ('offset_width', ctypes.c_int32), ('fixed_width', ctypes.c_int32)]


class SdpRecords(ctypes.Structure):
    _fields_ = [('d_k0', ctypes.c_void_p), ('d_k1', ctypes.c_void_p), ('d_meta', ctypes.c_void_p)]


class SdpHeavy(ctypes.Structure):
    _fields_ = [('d_h', ctypes.c_void_p), ('d_k0', ctypes.c_void_p), ('d_k1', ctypes.c_void_p),
                ('d_meta', ctypes.c_void_p), ('n', ctypes.c_int32), ('_pad', ctypes.c_int32)]


class SdpChunk(ctypes.Structure):
    _fields_ = [('start', ctypes.c_int64), ('end', ctypes.c_int64), ('hbase', ctypes.c_int64),
                ('hstride', ctypes.c_int64)]


class SdpQPlan(ctypes.Structure):
    _fields_ = [('lo', ctypes.c_uint64 * MAX_WINDOWS), ('hi', ctypes.c_uint64 * MAX_WINDOWS),
                ('in_sample', ctypes.c_int32 * MAX_WINDOWS), ('shift', ctypes.c_double),
                ('n_windows', ctypes.c_int32), ('n_sample', ctypes.c_int32),
                ('excl_mask', ctypes.c_int32), ('_pad', ctypes.c_int32)]


class SdpPass1Result(ctypes.Structure):
    _fields_ = [('count', ctypes.c_uint64), ('n_valid', ctypes.c_uint64), ('n_nan', ctypes.c_uint64),
                ('n_zero', ctypes.c_uint64), ('isum', ctypes.c_int64), ('imin', ctypes.c_int64),
                ('imax', ctypes.c_int64), ('dmin', ctypes.c_double), ('dmax', ctypes.c_double),
                ('shift', ctypes.c_double), ('s1_hi', ctypes.c_double), ('s1_lo', ctypes.c_double),
                ('s2', ctypes.c_double), ('s3_hi', ctypes.c_double), ('s3_lo', ctypes.c_double),
                ('s4', ctypes.c_double),
                ('w_gt', ctypes.c_uint64 * MAX_WINDOWS), ('w_eq_lo', ctypes.c_uint64 * MAX_WINDOWS),
                ('w_eq_hi', ctypes.c_uint64 * MAX_WINDOWS), ('w_in', ctypes.c_uint64 * MAX_WINDOWS),
                ('w_overflow', ctypes.c_uint32), ('_pad', ctypes.c_uint32)]


class SdpSelectTask(ctypes.Structure):
    _fields_ = [('d_keys', ctypes.c_void_p), ('d_n', ctypes.c_void_p), ('n_cap', ctypes.c_int64),
                ('k', ctypes.c_int64), ('lo_key', ctypes.c_uint64), ('hi_key', ctypes.c_uint64),
                ('d_work', ctypes.c_void_p), ('d_result', ctypes.c_void_p)]


class SdpCompactTask(ctypes.Structure):
    _fields_ = [('d_cand', ctypes.c_void_p), ('d_counts', ctypes.c_void_p), ('nseg', ctypes.c_int64),
                ('cap', ctypes.c_int64), ('d_offsets_work', ctypes.c_void_p), ('d_out', ctypes.c_void_p),
                ('d_out_count', ctypes.c_void_p)]


class SdpPass1Task(ctypes.Structure):
    _fields_ = [('col', SdpColumn), ('d_plan', ctypes.c_void_p), ('d_work', ctypes.c_void_p),
                ('d_cand', ctypes.c_void_p), ('d_cand_counts', ctypes.c_void_p), ('slot_capacity', ctypes.c_int64),
                ('d_result', ctypes.c_void_p), ('grid', ctypes.c_int32), ('_pad', ctypes.c_int32)]


class SdpPass2Task(ctypes.Structure):
    _fields_ = [('col', SdpColumn), ('d_edges', ctypes.c_void_p), ('mean', ctypes.c_double), ('hi_t', ctypes.c_double),
                ('lo_t', ctypes.c_double), ('d_work', ctypes.c_void_p), ('d_result', ctypes.c_void_p),
                ('d_hist', ctypes.c_void_p), ('heavy', SdpHeavy), ('d_part_hist', ctypes.c_void_p),
                ('d_heavy_counts', ctypes.c_void_p), ('d_stats', ctypes.c_void_p), ('rows_per_block', ctypes.c_int64),
                ('bins', ctypes.c_int32), ('edges_monotone', ctypes.c_int32), ('b1', ctypes.c_int32),
                ('grid', ctypes.c_int32), ('key32_lo', ctypes.c_int64)]


class SdpRowsTask(ctypes.Structure):
    _fields_ = [('col', SdpColumn), ('heavy', SdpHeavy), ('d_offsets', ctypes.c_void_p), ('d_out', ctypes.c_void_p),
                ('rows_per_block', ctypes.c_int64), ('b1', ctypes.c_int32), ('grid', ctypes.c_int32)]


class SdpPass2Result(ctypes.Structure):
    _fields_ = [('abs_dev_sum', ctypes.c_double), ('n_high', ctypes.c_uint64), ('n_low', ctypes.c_uint64),
                ('n_unbinned', ctypes.c_uint64)]


class SdpMinmaxResult(ctypes.Structure):           # sdp_minmax_result (sdp_minmax_int)
    _fields_ = [('count', ctypes.c_uint64), ('imin', ctypes.c_int64), ('imax', ctypes.c_int64),
                ('dmin', ctypes.c_double), ('dmax', ctypes.c_double)]


class SdpDistinctResult(ctypes.Structure):         # sdp_distinct_result (sdp_hash_distinct_count)
    _fields_ = [('distinct', ctypes.c_uint64), ('rows', ctypes.c_uint64), ('path', ctypes.c_int32),
                ('_pad', ctypes.c_int32)]


class SdpTopkEntry(ctypes.Structure):              # sdp_topk_entry
    _fields_ = [('key', ctypes.c_uint64), ('count', ctypes.c_uint64)]


class SdpTopkResult(ctypes.Structure):             # sdp_topk_result (sdp_value_counts_topk)
    _fields_ = [('groups', ctypes.c_uint64), ('rows', ctypes.c_uint64), ('n_top', ctypes.c_int32),
                ('path', ctypes.c_int32)]


class SdpBlocks(ctypes.Structure):                 # sdp_blocks (sdp_part_l2_blocks)
    _fields_ = [('d_desc', ctypes.c_void_p), ('d_list', ctypes.c_void_p)]


QUANTILES_MAX = 16       # SDP_QUANTILES_MAX

LAYOUT_NSIZES = 18           # SDP_LAYOUT_NSIZES


class SdpLayout(ctypes.Structure):                 # sdp_layout (sdp_layout_info)
    _fields_ = [('abi_version', ctypes.c_int32), ('n_sizes', ctypes.c_int32),
                ('byte_record_arrays', ctypes.c_int32), ('byte_record_stride', ctypes.c_int32),
                ('fixed_record_bytes', ctypes.c_int32), ('heavy_max', ctypes.c_int32),
                ('heavy_max_rec', ctypes.c_int32), ('heavy_min', ctypes.c_int32),
                ('part_sample', ctypes.c_int32), ('part_sample_bytes', ctypes.c_int32),
                ('gsort_max', ctypes.c_int32), ('l2_block', ctypes.c_int32), ('part_chunk', ctypes.c_int64),
                ('sizes', ctypes.c_int64 * LAYOUT_NSIZES)]


# the structs in sdp_layout.sizes order
_LAYOUT_STRUCTS = [SdpColumn, SdpBytesColumn, SdpRecords, SdpHeavy, SdpChunk, SdpQPlan, SdpPass1Result,
                   SdpSelectTask, SdpCompactTask, SdpPass1Task, SdpPass2Task, SdpRowsTask, SdpPass2Result,
                   SdpMinmaxResult, SdpDistinctResult, SdpTopkEntry, SdpTopkResult, SdpBlocks]


def expected_layout():
    """This binding's view of the library layout, as sdp_layout_info reports it."""
    return {'abi_version': ABI_VERSION, 'n_sizes': LAYOUT_NSIZES, 'byte_record_arrays': BYTE_RECORD_ARRAYS,
            'byte_record_stride': RECORD_WORD, 'fixed_record_bytes': RECORD_WORD, 'heavy_max': HEAVY_MAX,
            'heavy_max_rec': HEAVY_MAX_REC, 'heavy_min': HEAVY_MIN, 'part_sample': PART_SAMPLE,
            'part_sample_bytes': PART_SAMPLE_BYTES, 'gsort_max': GSORT_MAX, 'part_chunk': PART_CHUNK,
            'l2_block': L2_BLOCK,
            'sizes': [ctypes.sizeof(t) for t in _LAYOUT_STRUCTS]}


def layout_mismatches(lib_layout):
    """[(field, binding, library)] where a library's sdp_layout differs from this binding."""
    want = expected_layout()
    got = {k: getattr(lib_layout, k) for k in want if k != 'sizes'}
    got['sizes'] = list(lib_layout.sizes)[:LAYOUT_NSIZES]
    bad = [(k, want[k], got[k]) for k in want if k != 'sizes' and want[k] != got[k]]
    for t, a, b in zip(_LAYOUT_STRUCTS, want['sizes'], got['sizes']):
        if a != b:
            bad.append(('sizeof(%s)' % t.__name__, a, b))
    return bad

_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_I64 = ctypes.c_int64
_U64 = ctypes.c_uint64
_D = ctypes.c_double
_COL = ctypes.POINTER(SdpColumn)
_BCOL = ctypes.POINTER(SdpBytesColumn)
_REC = ctypes.POINTER(SdpRecords)
_HVY = ctypes.POINTER(SdpHeavy)

# name -> (restype, argtypes); every status-returning entry is checked
_SIGNATURES = {
    'sdp_last_error': (ctypes.c_char_p, []),
    'sdp_version': (ctypes.c_char_p, []),
    'sdp_layout_info': (ctypes.c_int, [ctypes.POINTER(SdpLayout)]),
    'sdp_pass1_workspace_bytes': (_I64, [_I64, _I32]),
    'sdp_pass2_workspace_bytes': (_I64, [_I64, _I32, _I32]),
    'sdp_pass1_grid': (_I32, [_I64, _I32]),
    'sdp_sample_keys': (ctypes.c_int, [_COL, _I32, _P, _P]),
    'sdp_sample_keys_batch': (ctypes.c_int, [_P, _I32, _I32, _P, _P]),
    'sdp_quantile_plan': (ctypes.c_int, [_P, _I32, _P, _I32, _I32, _P, _P]),
    'sdp_quantile_plan_batch': (ctypes.c_int, [_P, _I32, _I32, _P, _I32, _P, _P, _P]),
    'sdp_quantile_refine_batch': (ctypes.c_int, [_P, _I32, _I32, _P, _I32, _P, _P]),
    'sdp_pass1': (ctypes.c_int, [_COL, _P, _P, _I64, _P, _P, _I64, _I32, _P, _P]),
    'sdp_pass1_batch': (ctypes.c_int, [_P, _I32, _I32, _I32, _I32, _I32, _P]),
    'sdp_part_sample_batch': (ctypes.c_int, [_P, _I32, _I32, _P, _P]),
    'sdp_pass2_count_batch': (ctypes.c_int, [_P, _I32, _I32, _I32, _I32, _I32, _P]),
    'sdp_part_rows_batch': (ctypes.c_int, [_P, _I32, _I32, _I32, _P]),
    'sdp_compact_candidates': (ctypes.c_int, [_P, _P, _I32, _I64, _P, _P, _P, _P]),
    'sdp_radix_hist': (ctypes.c_int, [_P, _P, _U64, _I32, _P, _P]),
    'sdp_radix_filter': (ctypes.c_int, [_P, _P, _U64, _I32, _P, _P, _P]),
    'sdp_sort_small': (ctypes.c_int, [_P, _P, _P]),
    'sdp_sort_small_batch': (ctypes.c_int, [_P, _I32, _I32, _P]),
    'sdp_select_kth_workspace_bytes': (_I64, [_I64]),
    'sdp_select_kth': (ctypes.c_int, [_P, _P, _I64, _I64, _U64, _U64, _P, _I64, _P, _P]),
    'sdp_select_rounds': (ctypes.c_int, [_U64, _U64]),
    'sdp_select_init': (ctypes.c_int, [_I64, _U64, _U64, _P, _I64, _I64, _P, _P]),
    'sdp_select_hist': (ctypes.c_int, [_P, _P, _I64, _I32, _P, _I64, _P, _P]),
    'sdp_select_step': (ctypes.c_int, [_P, _P, _I64, _I32, _I32, _P, _I64, _P, _P, _P]),
    'sdp_column_keys': (ctypes.c_int, [_COL, _P, _P, _P]),
    'sdp_column_keys_range': (ctypes.c_int, [_COL, _U64, _U64, _P, _P, _P]),
    'sdp_sorted_distinct': (ctypes.c_int, [_COL, _P, _P]),
    'sdp_select_batch': (ctypes.c_int, [_P, _I32, _I32, _P, _P]),
    'sdp_select_batch_init': (ctypes.c_int, [_P, _I32, _P, _P]),
    'sdp_select_batch_step': (ctypes.c_int, [_P, _I32, _I32, _I32, _P, _P]),
    'sdp_compact_batch': (ctypes.c_int, [_P, _I32, _I64, _P]),
    'sdp_pass2': (ctypes.c_int, [_COL, _D, _P, _I32, _I32, _D, _D, _P, _I64, _P, _P, _P]),
    'sdp_pass2_count_workspace_bytes': (_I64, [_I64, _I32]),
    'sdp_pass2_count': (ctypes.c_int, [_COL, _D, _P, _I32, _I32, _D, _D, _P, _I64, _P, _P, _HVY, _I32, _P, _P, _P,
                                       _P]),
    'sdp_gather_bytes': (ctypes.c_int, [_P, _P, _P, _P, _I64, _P, _P]),
    'sdp_owner_order_workspace_bytes': (_I64, [_I64, _I32]),
    'sdp_owner_order': (ctypes.c_int, [_P, _P, _P, _I64, _I32, _BCOL, _P, _P, _P, _P, _P, _P, _P, _P, _I64, _P]),
    'sdp_table_clear': (ctypes.c_int, [_P, _P, _I64, _I32, _P]),
    'sdp_hash_u64': (ctypes.c_int, [_COL, _P, _P, _P, _I64, _I32, _P, _P]),
    'sdp_hash_bytes': (ctypes.c_int, [_BCOL, _P, _P, _P, _I64, _P, _P]),
    'sdp_table_count_log2_hist': (ctypes.c_int, [_P, _P, _I64, _I32, _P, _P]),
    'sdp_table_count_hist': (ctypes.c_int, [_P, _P, _I64, _I32, _U64, _U64, _P, _P]),
    'sdp_table_select': (ctypes.c_int, [_P, _P, _I64, _I32, _U64, _U64, _P, _P, _U64, _P]),
    'sdp_sort_groups': (ctypes.c_int, [_P, _P, _P, _P, _BCOL, _P]),
    'sdp_group_prefix': (ctypes.c_int, [_P, _P, _P, _BCOL, _I32, _P, _P]),
    'sdp_select_by_value': (ctypes.c_int, [_P, _P, _P, _U64, _U64, _P, _P, _P, _P]),
    'sdp_count_valid': (ctypes.c_int, [_P, _I64, _I64, _P, _P]),
    'sdp_first_valid': (ctypes.c_int, [_COL, _I32, _P, _P, _P]),
    'sdp_part_rows_per_block': (_I64, [_I64, _I32]),
    'sdp_part_bucket_target': (_I64, [_I32, _I32]),
    'sdp_part_sample': (ctypes.c_int, [_COL, _BCOL, _I32, _P, _REC, _P]),
    'sdp_part_rows': (ctypes.c_int, [_COL, _BCOL, _HVY, _I32, _I32, _P, _P, _REC, _P, _P, _P]),
    'sdp_part_recs': (ctypes.c_int, [_REC, _I32, _P, _I64, _I32, _I32, _I32, _P, _P, _REC, _P]),
    'sdp_part_records_chunks': (_I64, [_I64]),
    'sdp_gk_workspace_bytes': (_I64, [_I32]),
    'sdp_gk_quantiles': (ctypes.c_int, [_COL, _I32, _I32, _P, _I32, _P, _I64, _P, _P, _P]),
    'sdp_gk_layout': (ctypes.c_int, [_I32, _P]),
    'sdp_gk_partitions': (ctypes.c_int, [_COL, _I32, _I32, _P, _I64, _P]),
    'sdp_gk_merge': (ctypes.c_int, [_I32, _I32, _P, _I32, _P, _I64, _P, _P, _P]),
    'sdp_part_rows_records': (ctypes.c_int, [_BCOL, _HVY, _I32, _P, _P, _REC, _P, _P, _P]),
    'sdp_part_dedup': (ctypes.c_int, [_REC, _I32, _BCOL, _P, _I64, _I32, _P, _P, _P, _P, _P]),
    'sdp_part_compact': (ctypes.c_int, [_P, _P, _P, _P, _P, _I64, _P, _P, _P]),
    'sdp_part_l2_blocks': (ctypes.c_int, [_REC, _I32, _P, _P, _I32, _I32, _I32, _REC, _P, ctypes.POINTER(SdpBlocks),
                                          _P]),
    'sdp_part_dedup_blocks': (ctypes.c_int, [_REC, _I32, _BCOL, ctypes.POINTER(SdpBlocks), _I64, _I32, _P, _P, _P,
                                             _P, _P]),
    'sdp_part_compact_blocks': (ctypes.c_int, [_P, _P, ctypes.POINTER(SdpBlocks), _P, _P, _I64, _P, _P, _P]),
    'sdp_debug_bounds': (ctypes.c_int, [_U64, _U64, _P, _I32]),
    'sdp_distinct32_workspace_bytes': (_I64, [_I64]),
    'sdp_distinct32': (ctypes.c_int, [_COL, _I64, _P, _P, _I64, _P, _P]),
    'sdp_scan_workspace_bytes': (_I64, [_I64]),
    'sdp_bitmap_workspace_bytes': (_I64, [_I64, _I64]),
    'sdp_distinct_bitmap': (ctypes.c_int, [_COL, _I64, _I64, _P, _I64, _P, _P, _P]),
    'sdp_bitmap_reduce': (ctypes.c_int, [_P, _I32, _I64, _P, _P, _P]),
    'sdp_scan_u32': (ctypes.c_int, [_P, _I64, _P, _P, _I64, _P]),
    'sdp_rowmask': (ctypes.c_int, [_COL, ctypes.POINTER(_I32), _I32, _P, _I64, _P, _P]),
    'sdp_gram_workspace_bytes': (_I64, [_I64, _I32]),
    'sdp_gram': (ctypes.c_int, [_COL, _I32, _P, _P, _P, _I64, _P, _P, _P, _P]),
    # coarse entries (sdp_api.cpp): one call per reference operation group
    'sdp_minmax_workspace_bytes': (_I64, [_I64, _I32]),
    'sdp_minmax_int': (ctypes.c_int, [_COL, _P, _I64, _P, _P]),
    'sdp_quantiles_workspace_bytes': (_I64, [_I64, _I32]),
    'sdp_quantiles': (ctypes.c_int, [_COL, ctypes.POINTER(_D), _I32, _P, _I64, _P, _P]),
    'sdp_distinct_workspace_bytes': (_I64, [_I64, _I32]),
    'sdp_hash_distinct_count': (ctypes.c_int, [_COL, _BCOL, _P, _I64, ctypes.POINTER(SdpDistinctResult), _P]),
    'sdp_value_counts_workspace_bytes': (_I64, [_I64, _I32]),
    'sdp_value_counts_topk': (ctypes.c_int, [_COL, _BCOL, _I32, _P, _I64, ctypes.POINTER(SdpTopkResult),
                                             ctypes.POINTER(SdpTopkEntry), _P]),
    'sdp_pearson_workspace_bytes': (_I64, [_I64, _I32]),
    'sdp_gram_f64': (ctypes.c_int, [_COL, _I32, _P, _I64, _P, _P, _P]),
}

_VALUE_FUNCS = {'sdp_last_error', 'sdp_version', 'sdp_pass1_workspace_bytes', 'sdp_pass2_workspace_bytes',
                'sdp_pass1_grid', 'sdp_gram_workspace_bytes', 'sdp_part_rows_per_block', 'sdp_part_bucket_target',
                'sdp_part_records_chunks', 'sdp_gk_workspace_bytes',
                'sdp_scan_workspace_bytes', 'sdp_bitmap_workspace_bytes', 'sdp_select_kth_workspace_bytes',
                'sdp_select_rounds', 'sdp_pass2_count_workspace_bytes', 'sdp_minmax_workspace_bytes',
                'sdp_quantiles_workspace_bytes', 'sdp_distinct_workspace_bytes', 'sdp_value_counts_workspace_bytes',
                'sdp_pearson_workspace_bytes', 'sdp_distinct32_workspace_bytes',
                'sdp_owner_order_workspace_bytes'}
_STATUS_FUNCS = set(_SIGNATURES) - _VALUE_FUNCS

_lib = None


def _load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeError('libsdp.so not found at %s -- build it with `make -C spark-df-profiling_amd/csrc` '
                          '(or __graft_entry__.build()); there is no CPU fallback' % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH)
    if not hasattr(lib, 'sdp_layout_info'):
        raise NativeError('%s exports no sdp_layout_info: a library older than ABI %d -- rebuild it'
                          % (LIB_PATH, ABI_VERSION))
    for name, (res, args) in _SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    # layout handshake: the structs, record layout and grouping policy the
    # library was built with must be this binding's (a mismatched record layout
    # once sent garbage row indices into a kernel)
    lay = SdpLayout()
    lib.sdp_layout_info(ctypes.byref(lay))
    bad = layout_mismatches(lay)
    if bad:
        raise NativeError('%s was built for another layout (%s) -- rebuild it with '
                          '`make -C spark-df-profiling_amd/csrc`' % (
                              LIB_PATH, '; '.join('%s: binding %s, library %s' % b for b in bad)))
    _lib = lib
    return lib


def exported_symbols():
    """Names declared in include/sdp.h that this binding resolves."""
    lib = _load()
    return [n for n in _SIGNATURES if hasattr(lib, n)]


class _Caller:
    def __getattr__(self, name):
        lib = _load()
        fn = getattr(lib, name)
        if name not in _STATUS_FUNCS:
            return fn

        def call(*args):
            rec = _recorder
            if rec is not None:
                note, _tls.pending = getattr(_tls, 'pending', None), None
                ev0 = torch.cuda.Event(enable_timing=True)
                ev0.record()
            rc = fn(*args)
            if rec is not None:
                ev1 = torch.cuda.Event(enable_timing=True)
                ev1.record()
                key = name if note is None or not note[0] else '%s[%s]' % (name, note[0])
                rec.setdefault(key, []).append((ev0, ev1, None if note is None else note[1]))
            if rc != 0:
                msg = lib.sdp_last_error().decode(errors='replace')
                raise NativeError('%s failed (status %d): %s' % (name, rc, msg))
            return rc
        call.__name__ = name
        return call


sdp = _Caller()

# Optional per-entry-point HIP event timing (bench.py):
# {name or name[label]: [(start, end, alg_bytes or None)]}.
# Events are recorded on the current torch stream, the stream every entry point
# is launched on; nothing synchronises until the caller reads them.
_recorder = None


_tls = threading.local()            # the pending annotation is per thread (column workers)


def annotate(label, alg_bytes):
    """Tag the next entry-point call while recording: it is keyed as
    `name[label]` and carries its algorithmic bytes (compulsory HBM traffic:
    inputs read once, outputs written once) for the roofline."""
    if _recorder is not None:
        _tls.pending = (label, float(alg_bytes))


def recorded_index(key):
    """Index of the last recorded launch keyed `key` (None when not recording)."""
    rec = _recorder
    return len(rec[key]) - 1 if rec is not None and rec.get(key) else None


def annotate_output(key, index, out_bytes):
    """Add the bytes a recorded launch (entry `index` under `key`, e.g.
    'sdp_part_rows_records[bytes/records]') wrote, once they are known from a
    later readback: a kernel whose output size is data dependent (the records
    of a byte column) is annotated with its input at launch time."""
    rec = _recorder
    if rec is not None and index is not None and rec.get(key) and index < len(rec[key]):
        ev0, ev1, b = rec[key][index]
        rec[key][index] = (ev0, ev1, (b or 0.0) + float(out_bytes))


def start_recording():
    global _recorder
    _recorder = {}
    return _recorder


def stop_recording():
    global _recorder
    rec, _recorder = _recorder, None
    return rec


def ptr(t):
    """Device pointer of a torch tensor (or None -> NULL)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


def stream_handle(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def version():
    return _load().sdp_version().decode()
