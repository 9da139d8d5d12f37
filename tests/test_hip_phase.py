"""GPU parity tests of the phased fixed-shape kernel (phase_xor_kernel,
libquic_amd/csrc/qfec_kernels.hip), through the C-ABI.

Large nt batches (>= kPhMinPhases = 6 phases of CUs x 40 steps x
floor(256 / ceil(L/16)) groups, qfec_kernels.hip phase_plan) of a templated
k >= 5 (encode) / k >= 7 (recover) run the phased kernel by default (round 4:
below those group sizes the one-pass kernel is faster, tools/phase_k_table.py;
round 5: every k up to 16 templated, the runtime-k body for k > 16 with
batched loads, so the rule is by k alone);
QFEC_ONE_PASS forces the one-pass fixed kernel, qfec_debug_phase_min (here 6,
the default count) keeps the phase-count rule alone so every k reaches the
phased kernel, and qfec_last_fixed_phased reports which one a call ran (every
case here asserts it).  Every case is sized past that threshold (8 phases of 40 LDS steps) with
a ragged last phase, and checks the phased outputs byte-exact against the
one-pass kernel's on the same buffers, against the oracle on sampled groups,
and through the round-trip properties (revived row == erased row, parity XOR
every row == 0) on every group.
"""
import numpy as np
import pytest
import torch

from oracle import oracle_c as OC
from oracle import qfec_np as Q
from libquic_amd import qfec

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
STEPS = 40  # kPhSteps


def phase_groups(L):
    """Groups per phase on this GPU (the library's phase_plan)."""
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    return ncu * STEPS * (256 // ((L + 15) // 16))


def sample_vs_oracle(rows3, par_h, out_h, miss_np, k, L, n, ps=None, os_=None, count=48):
    """rows3: the device rows as [n][k][>= L]; sampled groups' rows go through
    the oracle's encode, the revived row must equal the lost row."""
    ps = ps or L
    os_ = os_ or L
    rng = np.random.default_rng(n + k + L)
    for g in list(rng.choice(n, count, replace=False)) + [0, n - 1]:
        g = int(g)
        rr = np.ascontiguousarray(rows3[g, :, :L].cpu().numpy()).ravel()
        _, pp = OC.encode_fixed(rr, k, L, 1)
        assert np.array_equal(par_h[g * ps:g * ps + L], pp), g
        m = int(miss_np[g])
        assert np.array_equal(out_h[g * os_:g * os_ + L], rr.reshape(k, L)[m]), g


def run_both(ctx, rows, miss, k, L, n, ps=None, os_=None, **strides):
    ps = ps or L
    os_ = os_ or L
    res = {}
    ctx.debug_phase_min(6)  # the phase-count rule alone: phased for every k
    try:
        return _run_both(ctx, rows, miss, k, L, n, ps, os_, res, strides)
    finally:
        ctx.debug_phase_min(0)


def _run_both(ctx, rows, miss, k, L, n, ps, os_, res, strides):
    for one_pass in (False, True):
        par = torch.full((n * ps,), 0xA5, dtype=torch.uint8, device=DEV)
        out = torch.full((n * os_,), 0x5A, dtype=torch.uint8, device=DEV)
        kw = dict(strides)
        if ps != L or os_ != L or strides:
            kw.update(parity_stride=ps)
        ctx.encode(rows, k, L, n, par, one_pass=one_pass, **kw)
        if ps != L or os_ != L or strides:
            kw.update(out_stride=os_)
        ctx.recover(rows, par, miss, k, L, n, out, one_pass=one_pass, **kw)
        # the library's own answer: phased unless QFEC_ONE_PASS (L >= 16 here)
        assert ctx.last_fixed_phased() == (0 if one_pass or L < 16 else 1)
        ctx.sync()
        torch.cuda.synchronize()
        res[one_pass] = (par, out)
    return res


@pytest.mark.parametrize("k", [2, 4, 5, 6, 7, 8, 10, 12, 20])
def test_default_kernel_choice_by_group_size(ctx, k):
    """The default rule (no test hook): a batch past the phase-count threshold
    runs phased for encode from k = 5 and for recover from k = 7 (round 5's
    table; round 4 had 8), one-pass below.  Round 4 phased only the
    templated sizes (2, 4, 5, 8, 10, 16); round 5 templates every k up to 16
    and fixed the runtime-k body (k > 16), so the rule is by k alone."""
    templated = True
    L = 1350
    n = 8 * phase_groups(L) + 777
    rows = torch.empty(n * k * L, dtype=torch.uint8, device=DEV)
    par = torch.empty(n * L, dtype=torch.uint8, device=DEV)
    out = torch.empty(n * L, dtype=torch.uint8, device=DEV)
    miss = torch.zeros(n, dtype=torch.uint8, device=DEV)
    ctx.encode(rows, k, L, n, par)
    assert ctx.last_fixed_phased() == (1 if templated and k >= 5 else 0)
    ctx.recover(rows, par, miss, k, L, n, out)
    assert ctx.last_fixed_phased() == (1 if templated and k >= 7 else 0)
    ctx.sync()


@pytest.mark.parametrize("k,L", [(10, 1350), (7, 1350), (33, 1350), (16, 1452), (2, 100),
                                 (5, 17), (2, 16), (4, 1350), (8, 1001), (6, 1350), (12, 1350),
                                 (20, 1350), (17, 100), (40, 64), (64, 1350), (255, 1350),
                                 (48, 300), (1, 300), (32, 1350), (24, 700), (17, 1350),
                                 (26, 512)])
def test_phased_vs_one_pass_and_oracle(ctx, k, L):
    n = 8 * phase_groups(L) + 777  # 9 phases, the last one ragged
    rows = torch.empty(n * k * L, dtype=torch.uint8, device=DEV)
    if n <= 1 << 24:
        ctx.synth_fixed(rows, k, L, 0, n, Q.SEED_FIXED)
    else:  # beyond the synthetic generator's group index range
        rows.copy_(torch.randint(0, 256, (n * k * L,), dtype=torch.uint8, device=DEV,
                                 generator=torch.Generator(device=DEV).manual_seed(k * L)))
    miss_np = Q.drop_index(Q.SEED_DROP, np.arange(n), k).astype(np.uint8)
    miss = torch.from_numpy(miss_np).to(DEV)
    before = ctx.phase_abandons()
    res = run_both(ctx, rows, miss, k, L, n)
    assert ctx.phase_abandons() == before
    (pp, po), (op, oo) = res[False], res[True]
    assert torch.equal(pp, op), "phased parity != one-pass parity"
    assert torch.equal(po, oo), "phased revived != one-pass revived"
    r3 = rows.view(n, k, L)
    assert torch.equal(r3[torch.arange(n, device=DEV), miss.long()], po.view(n, L))
    acc = pp.view(n, L).clone()
    for i in range(k):
        acc ^= r3[:, i]
    assert not bool(acc.any())
    sample_vs_oracle(r3, pp.cpu().numpy(), po.cpu().numpy(), miss_np, k, L, n)


def test_phased_strided(ctx):
    k, L = 10, 1350
    rs, ps, os_ = 1408, 1452, 1360
    n = 8 * phase_groups(L) + 5
    dense = torch.empty(n * k * L, dtype=torch.uint8, device=DEV)
    ctx.synth_fixed(dense, k, L, 0, n, Q.SEED_FIXED)
    rows = torch.zeros((n, k, rs), dtype=torch.uint8, device=DEV)
    rows[:, :, :L] = dense.view(n, k, L)
    del dense
    miss_np = Q.drop_index(Q.SEED_DROP, np.arange(n), k).astype(np.uint8)
    miss = torch.from_numpy(miss_np).to(DEV)
    res = run_both(ctx, rows.view(-1), miss, k, L, n, ps=ps, os_=os_, row_stride=rs,
                   group_stride=k * rs)
    (pp, po), (op, oo) = res[False], res[True]
    assert torch.equal(pp, op) and torch.equal(po, oo)
    # the padding between rows is never written
    assert bool((pp.view(n, ps)[:, L:] == 0xA5).all())
    assert bool((po.view(n, os_)[:, L:] == 0x5A).all())
    sample_vs_oracle(rows, pp.cpu().numpy(), po.cpu().numpy(), miss_np, k, L, n,
                     ps=ps, os_=os_)


@pytest.mark.parametrize("k", [10, 20])
def test_phased_invalid_missing(ctx, k):
    """A lost-slot index >= k latches QUIC_INVALID_FEC_DATA; that group's output
    is untouched, every other group is revived (as in the one-pass kernel).
    k = 20: the runtime-k body."""
    L = 1350
    n = 8 * phase_groups(L) + 1
    rows = torch.empty(n * k * L, dtype=torch.uint8, device=DEV)
    ctx.synth_fixed(rows, k, L, 0, n, Q.SEED_FIXED)
    par = torch.empty(n * L, dtype=torch.uint8, device=DEV)
    ctx.encode(rows, k, L, n, par)
    miss_np = Q.drop_index(Q.SEED_DROP, np.arange(n), k).astype(np.uint8)
    bad = np.array([0, 1, 2, 40 * 3, n // 2, n - 1])
    miss_np[bad] = [k, k + 1, 255, 200, k, 99]
    miss = torch.from_numpy(miss_np).to(DEV)
    out = torch.full((n * L,), 0xEE, dtype=torch.uint8, device=DEV)
    ctx.recover(rows, par, miss, k, L, n, out)
    with pytest.raises(qfec.InvalidFecData):
        ctx.sync()
    ctx.sync()
    torch.cuda.synchronize()
    o = out.view(n, L)
    badt = torch.from_numpy(bad).to(DEV)
    assert bool((o[badt] == 0xEE).all())
    good = torch.ones(n, dtype=torch.bool, device=DEV)
    good[badt] = False
    r3 = rows.view(n, k, L)
    m = miss.long().clamp(max=k - 1)
    assert torch.equal(r3[torch.arange(n, device=DEV), m][good], o[good])


def test_phased_repeated_and_rate(ctx):
    """Back-to-back launches (the last workgroup out re-zeroes the sync words
    for the next one) give identical parity, no launch gave up its meetings
    (qfec_phase_abandons), and the phased launch is within 1.2x of the
    one-pass kernel (measured 0.93-1.08x)."""
    k, L, n = 10, 1350, 1 << 20
    rows = torch.empty(n * k * L, dtype=torch.uint8, device=DEV)
    ctx.synth_fixed(rows, k, L, 0, n, Q.SEED_FIXED)
    pars = [torch.empty(n * L, dtype=torch.uint8, device=DEV) for _ in range(3)]
    s = torch.cuda.current_stream()
    times = {}
    before = ctx.phase_abandons()
    for one_pass in (True, False):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        for i in range(3):
            ev[i].record(s)
            ctx.encode(rows, k, L, n, pars[i], one_pass=one_pass)
        ev[3].record(s)
        ctx.sync()
        torch.cuda.synchronize()
        times[one_pass] = ev[1].elapsed_time(ev[3]) / 2  # launches 2 and 3
        assert torch.equal(pars[0], pars[1]) and torch.equal(pars[1], pars[2])
    assert ctx.phase_abandons() == before
    assert times[False] < 1.2 * times[True], times


def test_phased_concurrent_launches(ctx):
    """Two phased launches on two streams of two contexts (each wants every
    CU's whole LDS, so they cannot both be resident) produce the one-pass
    kernel's bytes; a later launch on the same context meets normally."""
    k, L, n = 10, 1350, 1 << 19
    rows = torch.empty(n * k * L, dtype=torch.uint8, device=DEV)
    ctx.synth_fixed(rows, k, L, 0, n, Q.SEED_FIXED)
    want = torch.empty(n * L, dtype=torch.uint8, device=DEV)
    ctx.encode(rows, k, L, n, want, one_pass=True)
    ctx.sync()
    torch.cuda.synchronize()
    ctx2 = qfec.Context(0)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    outs = [torch.zeros(n * L, dtype=torch.uint8, device=DEV) for _ in range(4)]
    torch.cuda.synchronize()  # the fills (current stream) before launches on s1 / s2
    try:
        ctx.set_stream(s1)
        ctx2.set_stream(s2)
        a0, b0 = ctx.phase_abandons(), ctx2.phase_abandons()
        for r in range(2):
            ctx.encode(rows, k, L, n, outs[2 * r])
            ctx2.encode(rows, k, L, n, outs[2 * r + 1])
        ctx.sync()
        ctx2.sync()
        torch.cuda.synchronize()
        for o in outs:
            assert torch.equal(o, want)
        print(f"abandoned launches: {ctx.phase_abandons() - a0} + {ctx2.phase_abandons() - b0}")
        # alone again: meets normally (the backoff a contended launch may
        # have engaged is cleared first)
        ctx.debug_phase(0, reset_backoff=True)
        a1 = ctx.phase_abandons()
        ctx.encode(rows, k, L, n, outs[0])
        ctx.sync()
        torch.cuda.synchronize()
        assert ctx.phase_abandons() == a1
        assert torch.equal(outs[0], want)
    finally:
        ctx.set_stream(torch.cuda.current_stream())
        ctx2.close()
        ctx.debug_phase(0, reset_backoff=True)  # contention over: phased again


def test_phased_abandon_path_and_backoff(ctx):
    """More workgroups than CUs (test hook qfec_debug_phase): the extra one is
    not resident until another exits, so the first meeting times out, the
    launch raises its abandon flag and runs to the end without meetings — same
    bytes as the one-pass kernel, counted by qfec_phase_abandons.  The next
    large batch without the hook sees the grown count (copied to host-mapped
    memory by the last workgroup out, read without a synchronisation) and runs
    one-pass: the contention backoff (16 batches).  Cleared, the phased kernel
    meets normally again.  Also times an abandoned launch against the one-pass
    kernel."""
    k, L, n = 10, 1350, 1 << 19
    rows = torch.empty(n * k * L, dtype=torch.uint8, device=DEV)
    ctx.synth_fixed(rows, k, L, 0, n, Q.SEED_FIXED)
    want = torch.empty(n * L, dtype=torch.uint8, device=DEV)
    ctx.encode(rows, k, L, n, want, one_pass=True)
    out = torch.zeros(n * L, dtype=torch.uint8, device=DEV)
    ctx.debug_phase(0, reset_backoff=True)
    a0 = ctx.phase_abandons()
    s = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    try:
        ctx.debug_phase(1, reset_backoff=False)
        ctx.encode(rows, k, L, n, out)  # warm
        ev[0].record(s)
        ctx.encode(rows, k, L, n, out)
        ev[1].record(s)
        ctx.sync()
        torch.cuda.synchronize()
        assert ctx.phase_abandons() == a0 + 2
        assert torch.equal(out, want)
    finally:
        ctx.debug_phase(0, reset_backoff=False)
    ev[2].record(s)
    ctx.encode(rows, k, L, n, out, one_pass=True)
    ev[3].record(s)
    torch.cuda.synchronize()
    t_ab, t_one = ev[0].elapsed_time(ev[1]), ev[2].elapsed_time(ev[3])
    print(f"abandoned phased launch {t_ab:.3f} ms vs one-pass {t_one:.3f} ms "
          f"(one-pass / abandoned = {t_one / t_ab:.2f})")
    # the backoff engages at the next large batch: one-pass, no new abandon
    out.zero_()
    ctx.encode(rows, k, L, n, out)
    ctx.sync()
    torch.cuda.synchronize()
    assert ctx.phase_backoff() == 15
    assert ctx.phase_abandons() == a0 + 2
    assert torch.equal(out, want)
    # cleared: phased again, meeting normally
    ctx.debug_phase(0, reset_backoff=True)
    out.zero_()
    ctx.encode(rows, k, L, n, out)
    ctx.sync()
    torch.cuda.synchronize()
    assert ctx.phase_backoff() == 0
    assert ctx.phase_abandons() == a0 + 2
    assert torch.equal(out, want)


def test_phased_one_context_two_streams(ctx):
    """phased launches of ONE context on two streams share its sync
    words; the context orders them (a phased launch on another stream waits
    for the previous one's event), so no launch is abandoned by the other's
    counters and every output equals the one-pass kernel's."""
    k, L, n = 10, 1350, 1 << 19
    rows = torch.empty(n * k * L, dtype=torch.uint8, device=DEV)
    ctx.synth_fixed(rows, k, L, 0, n, Q.SEED_FIXED)
    want = torch.empty(n * L, dtype=torch.uint8, device=DEV)
    ctx.encode(rows, k, L, n, want, one_pass=True)
    ctx.debug_phase(0, reset_backoff=True)
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    outs = [torch.zeros(n * L, dtype=torch.uint8, device=DEV) for _ in range(6)]
    torch.cuda.synchronize()
    a0 = ctx.phase_abandons()
    try:
        for i, o in enumerate(outs):
            ctx.set_stream(s1 if i % 2 == 0 else s2)
            ctx.encode(rows, k, L, n, o)
        torch.cuda.synchronize()
    finally:
        ctx.set_stream(torch.cuda.current_stream())
    for o in outs:
        assert torch.equal(o, want)
    assert ctx.phase_abandons() == a0
    assert ctx.phase_backoff() == 0


@pytest.mark.parametrize("k,L", [(4, 1350), (16, 700)])
def test_phased_register_steps_identical(ctx, k, L):
    """Every templated k runs 32 register-held steps per phase after the 40
    LDS steps (round 4; round 3: k = 10 only).  With the steps switched off
    (qfec_debug_phase_regsteps) the same batch takes more, shorter phases:
    the outputs must be byte-identical, and the round trip exact."""
    n = 8 * phase_groups(L) + 333
    rows = torch.empty(n * k * L, dtype=torch.uint8, device=DEV)
    ctx.synth_fixed(rows, k, L, 0, n, Q.SEED_FIXED)
    miss = torch.from_numpy(Q.drop_index(Q.SEED_DROP, np.arange(n), k).astype(np.uint8)).to(DEV)
    res = {}
    ctx.debug_phase_min(6)  # phased at k = 4 too (the default picks one-pass there)
    try:
        for on in (True, False):
            ctx.debug_phase_regsteps(on)
            par = torch.full((n * L,), 0xA5, dtype=torch.uint8, device=DEV)
            out = torch.full((n * L,), 0x5A, dtype=torch.uint8, device=DEV)
            ctx.encode(rows, k, L, n, par)
            assert ctx.last_fixed_phased() == 1
            ctx.recover(rows, par, miss, k, L, n, out)
            ctx.sync()
            torch.cuda.synchronize()
            res[on] = (par, out)
    finally:
        ctx.debug_phase_regsteps(True)
        ctx.debug_phase_min(0)
    assert torch.equal(res[True][0], res[False][0])
    assert torch.equal(res[True][1], res[False][1])
    r3 = rows.view(n, k, L)
    assert torch.equal(r3[torch.arange(n, device=DEV), miss.long()], res[True][1].view(n, L))


@pytest.mark.parametrize("k,L", [(20, 1350), (64, 1350), (255, 200)])
def test_runtime_k_load_batch_identical(ctx, k, L):
    """Group sizes above 16 run the runtime-k phased body, in load batches of
    16 or 32 rows (round 6: the library picks by operation and k,
    phase_rt_batch; qfec_debug_phase_rtbatch forces either).  Both batches
    give the same bytes, the revived row is the lost row, and sampled groups
    match the oracle."""
    n = 8 * phase_groups(L) + 91
    rows = torch.empty(n * k * L, dtype=torch.uint8, device=DEV)
    ctx.synth_fixed(rows, k, L, 0, n, Q.SEED_FIXED)
    miss_np = Q.drop_index(Q.SEED_DROP, np.arange(n), k).astype(np.uint8)
    miss = torch.from_numpy(miss_np).to(DEV)
    res = {}
    ctx.debug_phase_min(6)
    try:
        for b in (16, 32):
            ctx.debug_phase_rtbatch(b)
            par = torch.full((n * L,), 0xA5, dtype=torch.uint8, device=DEV)
            out = torch.full((n * L,), 0x5A, dtype=torch.uint8, device=DEV)
            ctx.encode(rows, k, L, n, par)
            assert ctx.last_fixed_phased() == 1
            ctx.recover(rows, par, miss, k, L, n, out)
            assert ctx.last_fixed_phased() == 1
            ctx.sync()
            torch.cuda.synchronize()
            res[b] = (par, out)
    finally:
        ctx.debug_phase_rtbatch(0)
        ctx.debug_phase_min(0)
    assert torch.equal(res[16][0], res[32][0])
    assert torch.equal(res[16][1], res[32][1])
    r3 = rows.view(n, k, L)
    assert torch.equal(r3[torch.arange(n, device=DEV), miss.long()], res[32][1].view(n, L))
    sample_vs_oracle(r3, res[32][0].cpu().numpy(), res[32][1].cpu().numpy(), miss_np, k, L, n,
                     count=16)
