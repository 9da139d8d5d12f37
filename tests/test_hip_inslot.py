"""GPU parity tests of the in-slot recover (qfec_recover_inslot_batch; VERDICT
r4 item 2): the receiver writes the FEC packet's redundancy into the lost
packet's row m of [G][k][L], so the lost packet is the XOR of the k rows --
encode's single contiguous stream.  Out of place (out != NULL) it runs the
encode kernels; in place (out == NULL) the kernels write each group's result
into its own row m (phase_xor_kernel / fixed_xor_kernel INPL,
fixed_small_kernel for L < 16).

Checked bit-exactly against the oracle's recover of the ordinary layout
(oracle/qfec_oracle.c, test infrastructure; parity unpinned by the reference,
DESIGN.md §2) for every drop index, against the golden shapes, and at full
size (2^20 x 10 x 1350 B) against the committed digest of the revived rows
(tests/golden/full_digests.json), through both the one-pass and the phased
kernel.
"""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from libquic_amd import qfec
from oracle import oracle_c as OC
from oracle import qfec_np as Q

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def inslot_rows(rows_np, parity_np, miss_np, k, L, n):
    """The in-slot layout: row m of each group replaced by its redundancy."""
    r = rows_np.reshape(n, k, L).copy()
    r[np.arange(n), miss_np.astype(np.int64)] = parity_np.reshape(n, L)
    return r


@pytest.mark.parametrize("k", [1, 2, 3, 5, 7, 10, 16, 17, 33])
@pytest.mark.parametrize("L", [1, 15, 16, 17, 100, 1350, 1452])
def test_every_drop_index_vs_oracle(ctx, k, L):
    n = k  # group g loses packet g: every drop index
    rows = OC.synth_fixed(0x1A5107 + k, 3, n, k, L)
    miss = np.arange(n, dtype=np.uint8) % k
    _, par = OC.encode_fixed(rows, k, L, n)
    _, want = OC.recover_fixed(rows, par, miss, k, L, n)
    ins = inslot_rows(rows, par, miss, k, L, n)
    d = torch.from_numpy(ins.ravel()).to(DEV)
    dm = torch.from_numpy(miss).to(DEV)
    out = torch.full((n * L,), 0xA5, dtype=torch.uint8, device=DEV)
    ctx.recover_inslot(d, dm, k, L, n, out)  # out of place
    ctx.recover_inslot(d, dm, k, L, n)  # in place
    ctx.sync()
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), want)
    got = d.cpu().numpy().reshape(n, k, L)
    assert np.array_equal(got[np.arange(n), miss.astype(np.int64)].ravel(), want)
    assert np.array_equal(got.ravel(), rows)  # in place: the original rows back


def test_golden_shapes(ctx, golden_shapes):
    tags = sorted({t.rsplit("_", 1)[0] for t in golden_shapes})
    for tag in tags:
        rows = golden_shapes[f"{tag}_rows"]
        n, k, L = rows.shape
        miss = golden_shapes[f"{tag}_missing"].astype(np.uint8)
        ins = inslot_rows(rows, golden_shapes[f"{tag}_parity"], miss, k, L, n)
        d = torch.from_numpy(ins.ravel()).to(DEV)
        out = torch.zeros(n * L, dtype=torch.uint8, device=DEV)
        ctx.recover_inslot(d, None, k, L, n, out)  # missing not needed out of place
        ctx.recover_inslot(d, torch.from_numpy(miss).to(DEV), k, L, n)
        ctx.sync()
        torch.cuda.synchronize()
        want = golden_shapes[f"{tag}_recovered"]
        assert np.array_equal(out.cpu().numpy().reshape(n, L), want), tag
        got = d.cpu().numpy().reshape(n, k, L)[np.arange(n), miss.astype(np.int64)]
        assert np.array_equal(got, want), tag


def test_host_and_mapped_out_of_place(ctx):
    k, L, n = 10, 1350, 33
    rows = OC.synth_fixed(0x51, 0, n, k, L)
    miss = Q.drop_index(Q.SEED_DROP, np.arange(n), k).astype(np.uint8)
    _, par = OC.encode_fixed(rows, k, L, n)
    _, want = OC.recover_fixed(rows, par, miss, k, L, n)
    ins = np.ascontiguousarray(inslot_rows(rows, par, miss, k, L, n).ravel())
    out = np.zeros(n * L, dtype=np.uint8)
    ctx.recover_inslot(ins, miss, k, L, n, out, host=True)
    assert np.array_equal(out, want)
    hb = qfec.HostBuffer(ins.size)
    ob = qfec.HostBuffer(n * L)
    try:
        hb.array[:] = ins
        ctx.recover_inslot(hb.array, None, k, L, n, ob.array, mapped=True)
        assert np.array_equal(ob.array, want)
    finally:
        hb.close()
        ob.close()
    with pytest.raises(qfec.QfecError):  # in place: device pointers only
        ctx.recover_inslot(ins, miss, k, L, n, None, host=True)


def test_in_place_invalid_index(ctx):
    k, L, n = 4, 64, 9
    d = torch.zeros(n * k * L, dtype=torch.uint8, device=DEV)
    miss = torch.zeros(n, dtype=torch.uint8, device=DEV)
    miss[3] = k  # out of range: that group is not written, the call fails
    ctx.recover_inslot(d, miss, k, L, n)
    with pytest.raises(qfec.InvalidFecData):
        ctx.sync()
    ctx.sync()  # cleared


def _phase_groups(L):
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    return ncu * 40 * (256 // ((L + 15) // 16))


@pytest.mark.parametrize("k,L", [(10, 1350), (6, 1350), (20, 700), (5, 17)])
def test_in_place_phased_and_one_pass(ctx, k, L):
    """Past the phase threshold: in place through the phased kernel (its
    stores after the grid meeting) and, forced, the one-pass kernel (a
    barrier between the loads and the stores); both equal the erased rows,
    and a second in-place call restores the redundancy."""
    n = 8 * _phase_groups(L) + 333
    rows = torch.empty(n * k * L, dtype=torch.uint8, device=DEV)
    ctx.synth_fixed(rows, k, L, 0, n, Q.SEED_FIXED)
    par = torch.empty(n * L, dtype=torch.uint8, device=DEV)
    ctx.encode(rows, k, L, n, par)
    miss_np = Q.drop_index(Q.SEED_DROP, np.arange(n), k).astype(np.uint8)
    miss = torch.from_numpy(miss_np).to(DEV)
    r3 = rows.view(n, k, L)
    idx = torch.arange(n, device=DEV)
    lost = r3[idx, miss.long()].clone()
    for one_pass in (False, True):
        r3[idx, miss.long()] = par.view(n, L)  # the redundancy into the lost slot
        ctx.recover_inslot(rows, miss, k, L, n, one_pass=one_pass)
        assert ctx.last_fixed_phased() == (0 if one_pass else 1)
        ctx.sync()
        assert torch.equal(r3[idx, miss.long()], lost), one_pass
        ctx.recover_inslot(rows, miss, k, L, n, one_pass=one_pass)  # involution
        ctx.sync()
        assert torch.equal(r3[idx, miss.long()], par.view(n, L)), one_pass
        r3[idx, miss.long()] = lost


def test_full_size_digest(ctx):
    """configs[2] at full size in the in-slot layout: 2^20 groups x 10 x
    1350 B, revived rows against the committed oracle digest, out of place and
    in place."""
    with open(os.path.join(GOLDEN, "full_digests.json")) as f:
        dg = json.load(f)["digests"]["g0=0,n=1048576"]
    k, L, n = 10, 1350, 1 << 20
    rows = torch.empty(n * k * L, dtype=torch.uint8, device=DEV)
    ctx.synth_fixed(rows, k, L, 0, n, Q.SEED_FIXED)
    par = torch.empty(n * L, dtype=torch.uint8, device=DEV)
    ctx.encode(rows, k, L, n, par)
    miss_np = Q.drop_index(Q.SEED_DROP, np.arange(n), k).astype(np.uint8)
    miss = torch.from_numpy(miss_np).to(DEV)
    r3 = rows.view(n, k, L)
    idx = torch.arange(n, device=DEV)
    r3[idx, miss.long()] = par.view(n, L)
    del par
    out = torch.empty(n * L, dtype=torch.uint8, device=DEV)
    ctx.recover_inslot(rows, miss, k, L, n, out)
    ctx.sync()
    torch.cuda.synchronize()
    assert f"{OC.group_digest(out.cpu().numpy(), n, L, L):#018x}" == dg["recovered"]
    ctx.recover_inslot(rows, miss, k, L, n)
    ctx.sync()
    assert torch.equal(r3[idx, miss.long()], out.view(n, L))
