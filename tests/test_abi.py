"""libsdp.so loads, exports every entry point include/sdp.h declares, and the
ctypes mirrors have the C layout (CPU only: no kernel is launched)."""

import ctypes
import os
import re
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, 'include', 'sdp.h')


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r'/\*.*?\*/', '', text, flags=re.S)
    return sorted(set(re.findall(r'\b(sdp_[a-z0-9_]+)\s*\(', text)))


def test_header_declares_entry_points():
    names = declared_functions()
    for must in ('sdp_pass1', 'sdp_pass2', 'sdp_quantile_plan', 'sdp_hash_u64', 'sdp_hash_bytes',
                 'sdp_part_rows', 'sdp_part_recs', 'sdp_part_dedup', 'sdp_scan_u32', 'sdp_gram', 'sdp_rowmask', 'sdp_first_valid',
                 'sdp_last_error'):
        assert must in names


def test_library_exports_every_declared_symbol():
    from spark_df_profiling import _native
    lib = ctypes.CDLL(_native.LIB_PATH)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    # and the binding knows every one of them
    assert set(declared_functions()) <= set(_native._SIGNATURES), \
        set(declared_functions()) - set(_native._SIGNATURES)
    assert _native.version().startswith('sdp-mi355x')


def test_error_reporting_without_gpu():
    """Argument validation fails before any device work, with a message."""
    from spark_df_profiling import _native
    with pytest.raises(_native.NativeError, match='n_sample'):
        _native.sdp.sdp_quantile_plan(None, 0, None, 5, 1, None, None)
    with pytest.raises(_native.NativeError, match='capacity'):
        _native.sdp.sdp_table_clear(None, None, 1000, 0, None)


STRUCTS = {'sdp_column': 'SdpColumn', 'sdp_bytes_column': 'SdpBytesColumn', 'sdp_qplan': 'SdpQPlan',
           'sdp_pass1_result': 'SdpPass1Result', 'sdp_pass2_result': 'SdpPass2Result',
           'sdp_records': 'SdpRecords', 'sdp_heavy': 'SdpHeavy', 'sdp_chunk': 'SdpChunk',
           'sdp_select_task': 'SdpSelectTask', 'sdp_compact_task': 'SdpCompactTask',
           'sdp_pass1_task': 'SdpPass1Task', 'sdp_pass2_task': 'SdpPass2Task',
           'sdp_rows_task': 'SdpRowsTask', 'sdp_minmax_result': 'SdpMinmaxResult',
           'sdp_distinct_result': 'SdpDistinctResult', 'sdp_topk_entry': 'SdpTopkEntry',
           'sdp_topk_result': 'SdpTopkResult', 'sdp_blocks': 'SdpBlocks'}


def test_struct_layouts_match_c():
    from spark_df_profiling import _native
    src = ['#include <stdio.h>', '#include <stddef.h>', '#include "%s"' % HEADER, 'int main(void){']
    for c, py in STRUCTS.items():
        src.append('printf("%s %%zu\\n", sizeof(%s));' % (c, c))
        for f, _ in getattr(_native, py)._fields_:
            src.append('printf("%s.%s %%zu\\n", offsetof(%s, %s));' % (c, f, c, f))
    src.append('return 0;}')
    with tempfile.TemporaryDirectory() as d:
        cfile, exe = os.path.join(d, 'l.c'), os.path.join(d, 'l')
        open(cfile, 'w').write('\n'.join(src))
        subprocess.run(['gcc', '-o', exe, cfile], check=True)
        out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout.split('\n')
    got = dict(line.split() for line in out if line)
    for c, py in STRUCTS.items():
        cls = getattr(_native, py)
        assert int(got[c]) == ctypes.sizeof(cls), c
        for f, _ in cls._fields_:
            assert int(got['%s.%s' % (c, f)]) == getattr(cls, f).offset, (c, f)


def test_part_argument_checks_without_gpu():
    """The partition entry points reject bad arguments before any launch."""
    from spark_df_profiling import _native
    with pytest.raises(_native.NativeError, match='part_rows'):
        _native.sdp.sdp_part_rows(None, None, None, 4, 0, None, None, None, None, None, None)
    with pytest.raises(_native.NativeError, match='scan_u32'):
        _native.sdp.sdp_scan_u32(None, 0, None, None, 0, None)
    # the sharded exchange's owner order: world 1 .. 2048, outputs of its mode
    with pytest.raises(_native.NativeError, match='owner_order: n 10 world 0'):
        _native.sdp.sdp_owner_order(None, None, None, 10, 0, None, None, None, None, None, None, None, None, None, 0,
                                    None)
    with pytest.raises(_native.NativeError, match='owner_order: n 10 world 4096'):
        _native.sdp.sdp_owner_order(None, None, None, 10, 4096, None, None, None, None, None, None, None, None, None,
                                    0, None)
    with pytest.raises(_native.NativeError, match='owner_order: outputs'):
        _native.sdp.sdp_owner_order(None, None, None, 10, 8, None, None, None, None, None, None, None,
                                    ctypes.c_void_p(16), None, 0, None)     # (d_per set: not dereferenced)
    assert _native.sdp.sdp_owner_order_workspace_bytes(0, 8) > 0
    assert _native.sdp.sdp_part_rows_per_block(10 ** 9, 0) % 4096 == 0
    # an empty shard (a rank with no rows) still gets a positive block size: the
    # launchers divide by it
    assert _native.sdp.sdp_part_rows_per_block(0, 0) > 0 and _native.sdp.sdp_part_rows_per_block(0, 1) > 0
    assert _native.sdp.sdp_pass2_count_workspace_bytes(0, 10) > 0
    assert _native.sdp.sdp_part_bucket_target(1, 1) == 2048
    with pytest.raises(_native.NativeError, match='part_rows_records'):
        _native.sdp.sdp_part_rows_records(None, None, 4, None, None, None, None, None, None)
    # one chunk per wave strip: 16 per workgroup of the records grid (whole
    # 4 K-row tiles, one workgroup per CU: at most 256 workgroups)
    n = 10 ** 9
    rpb = _native.sdp.sdp_part_rows_per_block(n, 1)
    ch = _native.sdp.sdp_part_records_chunks(n)
    assert ch % 16 == 0 and 16 <= ch <= 16 * 256 and (ch // 16) * 4096 * (-(-n // 4096 // (ch // 16))) >= n
    assert _native.sdp.sdp_part_records_chunks(0) == 16 and _native.sdp.sdp_part_records_chunks(5000) == 32
    assert rpb % 1024 == 0


def test_gk_layout_host_arithmetic():
    """sdp_gk_layout (host-only): the workspace offsets the sharded GK merge
    writes gathered digests into."""
    import ctypes
    from spark_df_profiling._native import sdp
    lay = (ctypes.c_int64 * 4)()
    sdp.sdp_gk_layout(3, ctypes.addressof(lay))
    head, pb, boff, cap = list(lay)
    assert head >= 3 * 32 and head % 256 == 0
    assert pb == boff + 2 * cap * 24 and cap >= 60000
    assert sdp.sdp_gk_workspace_bytes(3) >= head + 3 * pb


def test_select_rounds_host_arithmetic():
    """sdp_select_rounds (host-only): 11-bit radix rounds a select over
    [lo, hi] needs -- every rank of a sharded select runs exactly this many
    hist / all-reduce / step rounds."""
    from spark_df_profiling._native import sdp
    assert sdp.sdp_select_rounds(5, 5) == 1
    assert sdp.sdp_select_rounds(0, 2047) == 1
    assert sdp.sdp_select_rounds(0, 2048) == 2
    assert sdp.sdp_select_rounds(1 << 40, (1 << 40) + 5) == 1
    assert sdp.sdp_select_rounds(0, (1 << 64) - 1) == 6


def test_c_caller_compiles_against_header():
    """examples/c_caller/sdp_profile.c -- a C host of the coarse entry points
    (sdp_quantiles, sdp_hash_distinct_count, sdp_value_counts_topk,
    sdp_minmax_int, sdp_gram_f64, sdp_pass1/2) -- is plain C11 against
    include/sdp.h and the HIP runtime header (gcc, no GPU needed)."""
    src = os.path.join(ROOT, 'examples', 'c_caller', 'sdp_profile.c')
    subprocess.run(['gcc', '-std=c11', '-Wall', '-Werror', '-fsyntax-only', '-D__HIP_PLATFORM_AMD__',
                    '-I/opt/rocm/include', '-I' + os.path.join(ROOT, 'include'), src], check=True)


def test_layout_handshake():
    """The loaded library reports the binding's layout and grouping policy
    (SDP_ABI_VERSION, record layout, struct sizes); a library that differs
    would be refused at load."""
    from spark_df_profiling import _native
    _native._load()                       # (raises on a mismatch)
    lay = _native.SdpLayout()
    assert _native.sdp.sdp_layout_info(ctypes.byref(lay)) == 0
    assert _native.layout_mismatches(lay) == []
    assert lay.abi_version == _native.ABI_VERSION and lay.heavy_max_rec == 1024
    # a library built with another record layout / policy / struct size is named
    lay.byte_record_stride = 24
    lay.heavy_max = 128
    lay.sizes[1] += 8
    bad = {b[0] for b in _native.layout_mismatches(lay)}
    assert bad == {'byte_record_stride', 'heavy_max', 'sizeof(SdpBytesColumn)'}


def test_policy_constants_come_from_the_header():
    """One grouping policy: engine.py's constants are _native's, which are
    sdp.h's SDP_* values (checked against the library at load)."""
    from spark_df_profiling import _native, engine
    text = open(HEADER).read()
    for c, v in (('SDP_HEAVY_MAX', _native.HEAVY_MAX), ('SDP_HEAVY_MAX_REC', _native.HEAVY_MAX_REC),
                 ('SDP_HEAVY_MIN', _native.HEAVY_MIN), ('SDP_PART_SAMPLE', _native.PART_SAMPLE),
                 ('SDP_PART_SAMPLE_BYTES', _native.PART_SAMPLE_BYTES), ('SDP_PART_CHUNK', _native.PART_CHUNK),
                 ('SDP_GSORT_MAX', _native.GSORT_MAX), ('SDP_ABI_VERSION', _native.ABI_VERSION),
                 ('SDP_L2_BLOCK', _native.L2_BLOCK)):
        m = re.search(r'#define %s\s+(\d+)' % c, text)
        assert m and int(m.group(1)) == v, c
    assert (engine.PART_SAMPLE, engine.PART_SAMPLE_BYTES, engine.HEAVY_MIN, engine.PART_CHUNK, engine.GSORT_MAX) == \
        (_native.PART_SAMPLE, _native.PART_SAMPLE_BYTES, _native.HEAVY_MIN, _native.PART_CHUNK, _native.GSORT_MAX)
    # sdp_api.cpp keeps no copies of its own
    api = open(os.path.join(ROOT, 'spark-df-profiling_amd', 'csrc', 'sdp_api.cpp')).read()
    assert not re.search(r'constexpr\s+\w+\s+(HEAVY_N|HEAVY_MIN|PART_SAMPLE\w*|PART_CHUNK|GSORT_MAX)\s*=\s*\d', api)
