"""sdp_owner_order (the sharded exchange's owner order, distributed.py) against
a torch restatement of the round-5 exchange it replaces: a stable sort of the
groups by owner rank, per-owner group and key-byte counts from the sorted
order, the byte groups' (start, length) from the column's offsets and the
payload offsets as a prefix sum of the lengths.  Bit-exact for every output,
with and without a selection array, for fixed keys and for byte groups of
int32 / int64 offsets and fixed-width keys, at world sizes 1 .. 300 and group
counts around the 2048-group chunk.  Needs an MI355X."""

import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

MIX = -7046029254386353131          # 0x9E3779B97F4A7C15 as int64


def _nat():
    from spark_df_profiling import _native as nat
    return nat


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _run(keys, sel, counts, n, world, bcol=None, with_counts=True):
    nat = _nat()
    dev = keys.device
    m = max(n, 1)
    per = torch.full((2 * world,), -7, dtype=torch.int64, device=dev)
    out = {}
    if bcol is None:
        out['keys'] = torch.full((m,), -3, dtype=torch.int64, device=dev)
        out['counts'] = torch.full((m,), -3, dtype=torch.int64, device=dev) if with_counts else None
    else:
        for k in ('starts', 'lens'):
            out[k] = torch.full((m,), -3, dtype=torch.int64, device=dev)
        out['meta'] = torch.full((2 * m,), -3, dtype=torch.int64, device=dev)
        out['offs'] = torch.full((n + 1,), -3, dtype=torch.int64, device=dev)
    wb = nat.sdp.sdp_owner_order_workspace_bytes(n, world)
    work = torch.empty(max(wb, 16), dtype=torch.uint8, device=dev)
    nat.sdp.sdp_owner_order(_ptr(keys), _ptr(sel), _ptr(counts if (with_counts or bcol is not None) else None), n,
                            world, ctypes.byref(bcol) if bcol is not None else None,
                            _ptr(out.get('keys')), _ptr(out.get('counts')),
                            _ptr(out.get('starts')), _ptr(out.get('lens')), _ptr(out.get('meta')),
                            _ptr(out.get('offs')), _ptr(per), _ptr(work), wb, None)
    torch.cuda.synchronize()
    return {k: (v.cpu() if v is not None else None) for k, v in out.items()}, per.cpu()


def _owner_fixed(k, world):
    return (((k * MIX) >> 40) & 0xFFFFFF) % world


def _check(got, per, want, want_per, n):
    for k, v in want.items():
        g = got[k]
        g = g[:2 * n] if k == 'meta' else (g[:n + 1] if k == 'offs' else g[:n])
        assert torch.equal(g, v), (k, g[:8], v[:8])
    assert torch.equal(per, want_per)


@pytest.mark.parametrize('world', [1, 2, 3, 8, 300])
@pytest.mark.parametrize('n', [0, 1, 2047, 2048, 2049, 70001])
@pytest.mark.parametrize('use_sel', [False, True])
def test_owner_order_fixed_keys(world, n, use_sel):
    g = torch.Generator().manual_seed(n * 31 + world)
    ne = n + 17 if use_sel else n
    ent = torch.randint(-2 ** 62, 2 ** 62, (max(ne, 1),), generator=g, dtype=torch.int64)
    cnt = torch.randint(1, 1000, (max(ne, 1),), generator=g, dtype=torch.int64)
    sel = torch.randperm(max(ne, 1), generator=g)[:n].to(torch.int64) if use_sel else None
    idx = sel if use_sel else torch.arange(n)
    keys, c = ent[idx], cnt[idx]
    own = _owner_fixed(keys, world)
    order = torch.sort(own, stable=True)[1]
    per = torch.zeros(2 * world, dtype=torch.int64)
    per[:world] = torch.bincount(own, minlength=world)
    for with_counts in (True, False):
        got, gp = _run(ent.cuda(), sel.cuda() if use_sel else None, cnt.cuda(), n, world,
                       with_counts=with_counts)
        want = {'keys': keys[order]}
        if with_counts:
            want['counts'] = c[order]
        _check(got, gp, want, per, n)


class _BytesCol:
    def __init__(self, lens, offset_width, fixed_width):
        from spark_df_profiling import _native as nat
        self.fixed_width = fixed_width
        total = int(lens.sum())
        self.data = torch.randint(0, 256, (total + 16,), dtype=torch.uint8).cuda()
        if fixed_width:
            self.offsets = None
            self.off_host = torch.arange(lens.numel() + 1, dtype=torch.int64) * fixed_width
        else:
            o = torch.zeros(lens.numel() + 1, dtype=torch.int64)
            o[1:] = torch.cumsum(lens, 0)
            self.off_host = o
            self.offsets = o.to(torch.int32 if offset_width == 4 else torch.int64).cuda()
        c = nat.SdpBytesColumn()
        c.d_data = self.data.data_ptr()
        c.d_offsets = self.offsets.data_ptr() if self.offsets is not None else None
        c.d_validity = None
        c.validity_bit_offset = 0
        c.length = lens.numel()
        c.offset_width = offset_width
        c.fixed_width = fixed_width
        self.sdp = c


@pytest.mark.parametrize('world', [1, 2, 5, 8, 300])
@pytest.mark.parametrize('n', [0, 1, 2048, 2049, 50000])
@pytest.mark.parametrize('layout', [(4, 0), (8, 0), (0, 12)])
def test_owner_order_byte_groups(world, n, layout):
    ow, fw = layout
    g = torch.Generator().manual_seed(n * 7 + world + ow)
    rows_total = n + 100
    lens = torch.full((rows_total,), fw, dtype=torch.int64) if fw else \
        torch.randint(0, 40, (rows_total,), generator=g, dtype=torch.int64)
    col = _BytesCol(lens, ow, fw)
    use_sel = n % 2 == 0
    ne = n + 9 if use_sel else n
    rows = torch.randint(0, rows_total, (max(ne, 1),), generator=g, dtype=torch.int64)
    tags = torch.randint(0, 1 << 24, (max(ne, 1),), generator=g, dtype=torch.int64)
    slots = (tags << 40) | (rows + 1)
    cnt = torch.randint(1, 10 ** 6, (max(ne, 1),), generator=g, dtype=torch.int64)
    sel = torch.randperm(max(ne, 1), generator=g)[:n].to(torch.int64) if use_sel else None
    idx = sel if use_sel else torch.arange(n)
    s, c = slots[idx], cnt[idx]
    own = ((s >> 40) & 0xFFFFFF) % world
    order = torch.sort(own, stable=True)[1]
    r = (s & ((1 << 40) - 1)) - 1
    st = col.off_host[r]
    ln = col.off_host[r + 1] - st
    st, ln, c, own_s = st[order], ln[order], c[order], own[order]
    offs = torch.zeros(n + 1, dtype=torch.int64)
    offs[1:] = torch.cumsum(ln, 0)
    per = torch.zeros(2 * world, dtype=torch.int64)
    per[:world] = torch.bincount(own_s, minlength=world)
    per[world:] = torch.bincount(own_s, weights=ln.double(), minlength=world).to(torch.int64)
    got, gp = _run(slots.cuda(), sel.cuda() if use_sel else None, cnt.cuda(), n, world, bcol=col.sdp)
    want = {'starts': st, 'lens': ln, 'meta': torch.stack([ln, c], 1).reshape(-1), 'offs': offs}
    _check(got, gp, want, per, n)
    # the payload sdp_gather_bytes packs from them: owner-major key bytes
    if n and int(offs[-1]):
        nat = _nat()
        pay = torch.empty(int(offs[-1]), dtype=torch.uint8, device='cuda')
        st_d, ln_d, of_d = got['starts'][:n].cuda(), got['lens'][:n].cuda(), got['offs'][:n].cuda()
        nat.sdp.sdp_gather_bytes(_ptr(col.data), _ptr(st_d), _ptr(ln_d), _ptr(of_d), n, _ptr(pay), None)
        torch.cuda.synchronize()
        host = col.data.cpu()
        want_pay = torch.cat([host[int(a):int(a) + int(b)] for a, b in zip(st[:200], ln[:200])])
        assert torch.equal(pay.cpu()[:want_pay.numel()], want_pay)

