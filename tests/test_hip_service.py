"""GPU tests of the small-batch service (round 4; qfec_capi.cpp svc_submit,
qfec_kernels.hip ragged_service_kernel): QFEC_PTR_MAPPED ragged batches of at
most 64 groups (round 5; 16 in round 4) are taken by a resident worker (8
workgroups since round 5: a leader that polls the host and followers that
take a share of any job of more than 8 groups) from a job ring in
host-mapped memory instead of a kernel launch each.  The worker leaves after
100 us without work and the next batch relaunches it (the host publishes, then
reads the worker's alive word; the worker clears it, then reads the published
count once more).  Every result is bit-exact against the oracle; the cases
below cross the idle exit on purpose, mix service jobs with launched batches
on one context, and close a context while its worker is resident.
"""
import time

import numpy as np
import pytest

from libquic_amd import qfec
from test_hip_mapped import _mapped_case
from test_hip_ragged import run_ragged

pytestmark = pytest.mark.gpu


def _check(ctx, z, want_l):
    par, plen, out = run_ragged(ctx, z, host="mapped")
    assert np.array_equal(plen, want_l)
    assert np.array_equal(par, z["parity"])
    assert np.array_equal(out, z["recovered"])


def test_service_parity_across_idle_exits():
    """Small batches of every shape (k 1-80: groups beyond the fast form run
    the exact per-group body; packets 1-1452 B), with pauses before some of
    them longer than the worker's 100-us idle time: every result exact, and the
    worker was relaunched after leaving."""
    ctx = qfec.Context(0)
    try:
        rng = np.random.default_rng(11)
        calls = 0
        for it in range(40):
            n = int(rng.integers(1, 17))
            z, want_l = _mapped_case(n, g0=20000 + 50 * it, kmin=1, kmax=80, lmin=1, lmax=1452,
                                     seed=it)
            _check(ctx, z, want_l)
            calls += 2  # an encode and a recover
            time.sleep([0.0, 0.0, 0.001, 0.004][it % 4])
        st = ctx.debug_service()
        assert st["jobs"] >= calls, st
        assert st["launches"] >= 5, st  # idle exits (1-4 ms pauses) and relaunches
    finally:
        ctx.close()


def test_service_warm():
    """qfec_service_warm (an event loop's turn start): the worker runs after
    it, a second call while it runs launches nothing, batches stay exact, and
    with the service off it is a no-op."""
    z, want_l = _mapped_case(2, g0=46000, kmin=10, kmax=10, lmin=1350, lmax=1350, seed=3)
    ctx = qfec.Context(0)
    try:
        ctx.service_warm()
        st = ctx.debug_service()
        assert st["alive"] == 1 and st["launches"] >= 1, st
        ctx.service_warm()
        assert ctx.debug_service()["launches"] == st["launches"]
        _check(ctx, z, want_l)
        ctx.debug_service(on=False)
        ctx.service_warm()
        assert ctx.debug_service()["alive"] == 0
        _check(ctx, z, want_l)
    finally:
        ctx.close()


@pytest.mark.parametrize("k", [1, 2, 10, 12, 13, 24, 33, 40, 64, 65])
@pytest.mark.parametrize("shape", ["full", "wide", "short"])
def test_service_one_group_on_all_waves(k, shape):
    """Round 5: a one-group job runs on all 8 waves of the leader (its slots
    dealt round the waves, partial windows XORed out of LDS; a group out of
    the fast form -- more than 64 received packets, a packet under 16 B --
    by wave 0 alone).  k = 13 and up needs a second chunk of slots, k = 33
    and up (full packets) the second slot table (slots 64-127); exact,
    encode and recover (one drop index per group), over repeated jobs."""
    kw = {"full": dict(lmin=1452, lmax=1452), "wide": dict(lmin=16, lmax=1452),
          "short": dict(lmin=1, lmax=40)}[shape]
    ctx = qfec.Context(0)
    try:
        for rep in range(3):
            z, want_l = _mapped_case(1, g0=45000 + 7 * k + rep, kmin=k, kmax=k, seed=100 * k + rep,
                                     **kw)
            _check(ctx, z, want_l)
        assert ctx.debug_service()["jobs"] >= 6
    finally:
        ctx.close()


@pytest.mark.parametrize("k", [1, 2, 10, 13, 33, 65])
@pytest.mark.parametrize("shape", ["full", "wide", "short"])
def test_service_two_groups_on_four_waves_each(k, shape):
    """Round 6: a two-group job runs each group on 4 of the leader's waves
    (its slots dealt round them, partial windows XORed out of LDS by two of
    them; a group out of the fast form by its first wave alone), as the
    one-group job runs on all 8.  Exact, encode and recover, the two groups
    of different sizes, over repeated jobs."""
    kw = {"full": dict(lmin=1452, lmax=1452), "wide": dict(lmin=16, lmax=1452),
          "short": dict(lmin=1, lmax=40)}[shape]
    ctx = qfec.Context(0)
    try:
        for rep in range(3):
            z, want_l = _mapped_case(2, g0=48000 + 11 * k + rep, kmin=max(1, k - 3), kmax=k,
                                     seed=300 * k + rep, **kw)
            _check(ctx, z, want_l)
        assert ctx.debug_service()["jobs"] >= 6
    finally:
        ctx.close()


@pytest.mark.parametrize("n", [8, 9, 17, 33, 63, 64])
def test_service_split_jobs(n):
    """Round 5: a job of more than 8 groups is spread over the worker's 8
    workgroups (each adds itself to the entry's done counter after its
    outputs are visible; the last stores the token).  Exact for every split
    size, many times over (the counters wrap by ring entry), mixed with
    1-group jobs the leader takes alone, across idle exits."""
    ctx = qfec.Context(0)
    try:
        z, want_l = _mapped_case(n, g0=40000 + n, kmin=2, kmax=16, lmin=1, lmax=1452, seed=n)
        z1, want_1 = _mapped_case(1, g0=41000 + n, kmin=2, kmax=16, lmin=1, lmax=1452, seed=n + 1)
        before = ctx.debug_service()
        for it in range(24):
            _check(ctx, z, want_l)
            if it % 3 == 0:
                _check(ctx, z1, want_1)
            if it % 8 == 7:
                time.sleep(0.002)  # past the idle exit: a fresh worker (new epoch)
        st = ctx.debug_service()
        assert st["jobs"] >= before["jobs"] + 2 * 24 + 2 * 8, st
        assert st["launches"] >= before["launches"] + 3, st
    finally:
        ctx.close()


def test_service_off_matches_on():
    """The same batches with the service off (the launched small-batch kernel)
    give the same bytes; no worker is launched while it is off."""
    ctx = qfec.Context(0)
    try:
        z, want_l = _mapped_case(9, g0=31000, kmin=2, kmax=20, lmin=1, lmax=1452, seed=5)
        _check(ctx, z, want_l)
        on = ctx.debug_service()
        assert on["jobs"] >= 2
        ctx.debug_service(False)
        before = ctx.debug_service()
        for _ in range(5):
            _check(ctx, z, want_l)
        after = ctx.debug_service()
        assert after["launches"] == before["launches"] and after["jobs"] == before["jobs"]
        ctx.debug_service(True)
        _check(ctx, z, want_l)
        assert ctx.debug_service()["jobs"] >= before["jobs"] + 2
    finally:
        ctx.close()


def test_service_async_mixed_with_launched_batches():
    """QFEC_ASYNC on one context: small batches (service) and a 2,000-group
    batch (the block kernel) queued back to back, completed by ticket in
    reverse order; every output exact."""
    ctx = qfec.Context(0)
    bufs = []
    try:
        cases = []
        for i, n in enumerate((3, 2000, 7)):
            z, want_l = _mapped_case(n, g0=40000 + 3000 * i, kmin=2, kmax=30, lmin=1, lmax=1452,
                                     seed=20 + i)
            data = qfec.HostBuffer(len(z["data"]))
            data.array[:] = z["data"]
            par = qfec.HostBuffer(n * 1452)
            bufs += [data, par]
            plen = np.zeros(n, dtype=np.uint16)
            ctx.encode_ragged(data.array, z["pkt_off"], z["pkt_len"], z["grp_ptr"], n, par.array,
                              z["parity_off"], plen, mapped=True, async_=True)
            cases.append((ctx.async_ticket(), z, want_l, par, plen, n))
        for t, z, want_l, par, plen, n in reversed(cases):
            assert ctx.complete_ticket(t) == 0
            assert np.array_equal(plen, want_l)
            for g in range(n):
                o, m = int(z["parity_off"][g]), int(want_l[g])
                assert np.array_equal(par.array[o:o + m], z["parity"][o:o + m]), (n, g)
    finally:
        for b in bufs:
            b.close()
        ctx.close()


def test_service_close_while_resident():
    """A context closed right after a service job (its worker still resident,
    waiting for more) closes at once: the worker leaves on the quit word."""
    z, want_l = _mapped_case(4, g0=50000, kmin=2, kmax=12, lmin=16, lmax=1350, seed=9)
    for _ in range(5):
        ctx = qfec.Context(0)
        _check(ctx, z, want_l)
        ctx.debug_service()
        t0 = time.perf_counter()
        ctx.close()
        assert time.perf_counter() - t0 < 1.0


@pytest.mark.parametrize("same_ctx", [True, False])
def test_phased_launch_right_after_service_job(same_ctx):
    """The phased fixed-shape kernel wants one workgroup on every CU.  Right
    after a service job -- its worker still resident -- a phased encode on the
    same context (the worker is stopped first) or on another context (the
    worker leaves within its 100-us idle time, below the meetings' 200-us
    timeout) keeps its meetings: no abandoned launch."""
    import torch
    from oracle import qfec_np as Q
    a = qfec.Context(0)
    b = a if same_ctx else qfec.Context(0)
    try:
        k, L = 10, 1350
        ncu = torch.cuda.get_device_properties(0).multi_processor_count
        n = 8 * ncu * 40 * (256 // ((L + 15) // 16)) + 17
        rows = torch.empty(n * k * L, dtype=torch.uint8, device="cuda:0")
        b.synth_fixed(rows, k, L, 0, n, Q.SEED_FIXED)
        par = torch.empty(n * L, dtype=torch.uint8, device="cuda:0")
        want = torch.empty(n * L, dtype=torch.uint8, device="cuda:0")
        b.encode(rows, k, L, n, want, one_pass=True)
        b.sync()
        z, want_l = _mapped_case(5, g0=60000, kmin=2, kmax=12, lmin=16, lmax=1350, seed=4)
        for _ in range(3):
            before = b.phase_abandons()
            _check(a, z, want_l)  # a service job: the worker is resident now
            b.encode(rows, k, L, n, par)
            assert b.last_fixed_phased() == 1
            b.sync()
            assert b.phase_abandons() == before
            assert torch.equal(par, want)
    finally:
        if not same_ctx:
            b.close()
        a.close()


def test_service_idle_boundary_stress():
    """Small async batches spaced around the worker's 100-us idle time (the
    window where it may be leaving just as a batch is published): every one
    completes, exact, and the worker was relaunched many times."""
    ctx = qfec.Context(0)
    z, want_l = _mapped_case(2, g0=70000, kmin=3, kmax=10, lmin=16, lmax=1350, seed=6)
    data = qfec.HostBuffer(len(z["data"]))
    data.array[:] = z["data"]
    par = qfec.HostBuffer(2 * 1452)
    try:
        rng = np.random.default_rng(3)
        for it in range(300):
            par.array[:] = 0
            plen = np.zeros(2, dtype=np.uint16)
            ctx.encode_ragged(data.array, z["pkt_off"], z["pkt_len"], z["grp_ptr"], 2, par.array,
                              z["parity_off"], plen, mapped=True, async_=True)
            assert ctx.complete_ticket(ctx.async_ticket()) == 0
            assert np.array_equal(plen, want_l), it
            for g in range(2):
                o, m = int(z["parity_off"][g]), int(want_l[g])
                assert np.array_equal(par.array[o:o + m], z["parity"][o:o + m]), (it, g)
            t_end = time.perf_counter() + float(rng.uniform(40e-6, 200e-6))
            while time.perf_counter() < t_end:  # busy-wait: sleep() is too coarse
                pass
        st = ctx.debug_service()
        assert st["jobs"] >= 300 and st["launches"] >= 10, st
    finally:
        data.close()
        par.close()
        ctx.close()


def test_service_two_threads_two_contexts():
    """One context per host thread (the C-ABI's threading rule), each with its
    own resident worker: two threads flushing small batches at once, every
    result exact on both."""
    import threading
    errors = []

    def worker(seed):
        try:
            ctx = qfec.Context(0)
            try:
                z, want_l = _mapped_case(3, g0=80000 + 100 * seed, kmin=2, kmax=14, lmin=1,
                                         lmax=1452, seed=seed)
                for _ in range(60):
                    _check(ctx, z, want_l)
                assert ctx.debug_service()["jobs"] >= 120
            finally:
                ctx.close()
        except Exception as e:  # reported on the main thread
            errors.append(repr(e))

    ts = [threading.Thread(target=worker, args=(s,)) for s in (1, 2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in ts)
    assert not errors, errors


def test_service_ring_miss_fails_the_job_and_turns_off():
    """a published group that lies in no ring entry (the
    test hook writes the next job with a wrong job number) makes the worker
    latch a fault and leave WITHOUT storing any token: the call fails with
    QUIC_INTERNAL_ERROR instead of reporting stale output as finished, the
    output buffer is untouched, the context turns its service off (the next
    batches launch and are exact), and re-enabling the service works again."""
    ctx = qfec.Context(0)
    z, want_l = _mapped_case(3, g0=90000, kmin=2, kmax=12, lmin=16, lmax=1350, seed=12)
    data = qfec.HostBuffer(len(z["data"]))
    data.array[:] = z["data"]
    par = qfec.HostBuffer(3 * 1452)
    try:
        _check(ctx, z, want_l)  # the service works
        ctx.debug_service(poison_next=True)
        par.array[:] = 0xEE
        plen = np.zeros(3, dtype=np.uint16)
        with pytest.raises(qfec.QfecError) as ei:
            ctx.encode_ragged(data.array, z["pkt_off"], z["pkt_len"], z["grp_ptr"], 3, par.array,
                              z["parity_off"], plen, mapped=True)
        assert ei.value.code == qfec.QFEC_ERR_INTERNAL
        assert "ring" in str(ei.value), str(ei.value)
        assert (par.array == 0xEE).all()  # nothing reported, nothing written
        st = ctx.debug_service()
        for _ in range(3):  # service off now: launched small batches, exact
            _check(ctx, z, want_l)
        assert ctx.debug_service()["launches"] == st["launches"]
        ctx.debug_service(True)
        _check(ctx, z, want_l)
        assert ctx.debug_service()["jobs"] > st["jobs"]
    finally:
        data.close()
        par.close()
        ctx.close()


def test_service_nowait_completion_of_a_failed_job():
    """qfec_complete(ctx, 0) on a service job whose worker
    left without its token returns an error once the worker stream has
    drained, not QFEC_PENDING forever."""
    ctx = qfec.Context(0)
    z, want_l = _mapped_case(2, g0=91000, kmin=2, kmax=12, lmin=16, lmax=1350, seed=13)
    data = qfec.HostBuffer(len(z["data"]))
    data.array[:] = z["data"]
    par = qfec.HostBuffer(2 * 1452)
    try:
        ctx.debug_service(poison_next=True)
        plen = np.zeros(2, dtype=np.uint16)
        ctx.encode_ragged(data.array, z["pkt_off"], z["pkt_len"], z["grp_ptr"], 2, par.array,
                          z["parity_off"], plen, mapped=True, async_=True)
        t = ctx.async_ticket()
        assert t != 0
        deadline = time.perf_counter() + 10.0
        rc = 1
        while time.perf_counter() < deadline:
            rc = ctx.lib.qfec_complete_ticket(ctx.ctx, t, 0)
            if rc != 1:
                break
            time.sleep(0.001)
        assert rc == qfec.QFEC_ERR_INTERNAL, rc
        _check(ctx, z, want_l)  # the context goes on (service off)
    finally:
        data.close()
        par.close()
        ctx.close()


def test_ticket_claimable_after_qfec_complete():
    """qfec_complete finishes every op, ticketed ones included; a
    ticket's owner can still claim its own code afterwards (QFEC_OK), once."""
    ctx = qfec.Context(0)
    z, want_l = _mapped_case(2, g0=92000, kmin=2, kmax=12, lmin=16, lmax=1350, seed=14)
    data = qfec.HostBuffer(len(z["data"]))
    data.array[:] = z["data"]
    par = qfec.HostBuffer(2 * 1452)
    try:
        plen = np.zeros(2, dtype=np.uint16)
        ctx.encode_ragged(data.array, z["pkt_off"], z["pkt_len"], z["grp_ptr"], 2, par.array,
                          z["parity_off"], plen, mapped=True, async_=True)
        t = ctx.async_ticket()
        assert ctx.complete() == 0
        assert np.array_equal(plen, want_l)
        assert ctx.complete_ticket(t) == 0
        with pytest.raises(qfec.QfecError):
            ctx.complete_ticket(t)  # claimed once
    finally:
        data.close()
        par.close()
        ctx.close()


def test_phased_launch_beside_a_continuously_fed_service():
    """context B's small-batch worker kept
    resident by a connection thread feeding it continuously (the reference's
    model: one thread per QuicConnection, quic_connection.h:14; here a native
    thread owning B, qfec_debug_service_feed, warming the worker at each
    turn's start and flushing one-group batches back to back), while context
    A runs phased encodes of a large batch.  The worker holds 8 CUs' LDS, so a
    one-workgroup-per-CU grid could not be resident at once (round 5: its
    meetings timed out and it abandoned them, 0.6-0.7x).  Round 6: A's phased
    launch counts the other contexts' active workers (a process-wide
    registry) and leaves their CUs out of its grid: no launch abandons its
    meetings, the grid is ncu - 8, the parity equals the one-pass parity, the
    encode rate is recorded; B's results stay exact throughout."""
    import torch
    from oracle import qfec_np as Q
    a, b = qfec.Context(0), qfec.Context(0)
    rates, grids = [], []
    try:
        k, L = 10, 1350
        ncu = torch.cuda.get_device_properties(0).multi_processor_count
        n = 8 * ncu * 40 * (256 // ((L + 15) // 16)) + 5
        rows = torch.empty(n * k * L, dtype=torch.uint8, device="cuda:0")
        a.synth_fixed(rows, k, L, 0, n, Q.SEED_FIXED)
        want = torch.empty(n * L, dtype=torch.uint8, device="cuda:0")
        a.encode(rows, k, L, n, want, one_pass=True)
        a.sync()
        b.debug_service_feed(True)  # (back once its first batch is done)
        try:
            before = a.phase_abandons()
            par = torch.empty(n * L, dtype=torch.uint8, device="cuda:0")
            s = torch.cuda.current_stream()
            a.set_stream(s)
            for _ in range(4):
                a.debug_phase(0, reset_backoff=True)  # try the phased kernel every time
                par.fill_(0)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                a.encode(rows, k, L, n, par)
                e1.record(s)
                assert a.last_fixed_phased() == 1
                grids.append(a.last_phase_grid())
                a.sync()
                e1.synchronize()
                rates.append(n * (k + 1) * L / (e0.elapsed_time(e1) * 1e-3) / 8e12)
                assert torch.equal(par, want)
        finally:
            fed = b.debug_service_feed(False)
        abandoned = a.phase_abandons() - before
        print(f"phased launches beside a fed service worker: abandoned {abandoned} of 4; "
              f"grids {grids} (ncu {ncu}); encode frac of 8 TB/s "
              f"{', '.join(f'{r:.3f}' for r in rates)}; service batches meanwhile {fed}")
        assert fed["wrong"] == 0 and fed["jobs"] > 100, fed
        assert abandoned == 0
        assert all(g == ncu - 8 for g in grids), grids
        assert min(rates) > 0.70, rates
    finally:
        a.close()
        b.close()


def test_fed_worker_rotates_and_other_work_proceeds():
    """Round 6: a worker fed back to back stays resident at most 2 ms at a
    stretch (kSvcMaxResidentNs): the runtime multiplexes a process's streams
    onto 4 hardware queues, and work on a stream sharing the worker's queue
    waited behind it -- for seconds, once for good, before the bound.  With a
    native thread feeding context B for ~0.3 s, context A's kernels on its own
    streams (one-pass encodes, then device syncs) each finish within 100 ms,
    B's worker was stopped and relaunched many times, and every B batch was
    exact."""
    import torch
    from oracle import qfec_np as Q
    a, b = qfec.Context(0), qfec.Context(0)
    try:
        k, L, n = 10, 1350, 4096
        rows = torch.empty(n * k * L, dtype=torch.uint8, device="cuda:0")
        a.synth_fixed(rows, k, L, 0, n, Q.SEED_FIXED)
        want = torch.empty(n * L, dtype=torch.uint8, device="cuda:0")
        a.encode(rows, k, L, n, want, one_pass=True)
        a.sync()
        par = torch.empty(n * L, dtype=torch.uint8, device="cuda:0")
        b.debug_service_feed(True)
        worst = 0.0
        try:
            t_end = time.perf_counter() + 0.3
            while time.perf_counter() < t_end:
                t0 = time.perf_counter()
                a.encode(rows, k, L, n, par, one_pass=True)
                a.sync()
                worst = max(worst, time.perf_counter() - t0)
        finally:
            fed = b.debug_service_feed(False)
        st = b.debug_service()
        print(f"worst one-pass encode beside a fed worker {worst * 1e3:.2f} ms; feeder {fed}; "
              f"service {st}")
        assert torch.equal(par, want)
        assert fed["wrong"] == 0 and fed["jobs"] > 100, fed
        assert st["rotations"] >= 10, st
        assert worst < 0.1, worst
    finally:
        a.close()
        b.close()


def test_warm_restarts_the_idle_time():
    """Round 6: qfec_service_warm on a running worker bumps a count the
    worker polls, and its 100-us idle time restarts from it -- a loop turn
    that takes most of the idle time to assemble its batch still finds the
    worker resident.  Warm calls 50 us apart for 2 ms, no job: without the
    restart the worker would leave every ~100 us and be relaunched ~15 times;
    with it, it stays (each hiccup of the Python loop longer than the idle
    time may cost one relaunch).  Past the residency bound a warm call no
    longer restarts it (warm calls alone have no job to rotate the worker
    at): with the bound at 0.5 ms the same loop over 4 ms relaunches it
    several times."""
    z, want_l = _mapped_case(2, g0=47000, kmin=10, kmax=10, lmin=1350, lmax=1350, seed=4)
    ctx = qfec.Context(0)

    def warm_loop(seconds):
        t_end = time.perf_counter() + seconds
        nxt = time.perf_counter()
        calls = 0
        while time.perf_counter() < t_end:
            if time.perf_counter() >= nxt:
                ctx.service_warm()
                calls += 1
                nxt += 50e-6
        return calls

    try:
        _check(ctx, z, want_l)
        ctx.debug_service_resident(50_000_000)  # 50 ms: the restart alone
        ctx.service_warm()
        before = ctx.debug_service()["launches"]
        calls = warm_loop(0.002)
        st = ctx.debug_service()
        print(f"{calls} warm calls over 2 ms: {st['launches'] - before} relaunches; {st}")
        assert calls >= 20
        assert st["launches"] - before <= 6, st  # (~20 without the restart)
        ctx.debug_service_resident(500_000)  # 0.5 ms
        before = ctx.debug_service()["launches"]
        calls = warm_loop(0.004)
        st = ctx.debug_service()
        print(f"bound 0.5 ms: {calls} warm calls over 4 ms: {st['launches'] - before} relaunches")
        assert st["launches"] - before >= 2, st
        _check(ctx, z, want_l)
    finally:
        ctx.debug_service_resident(2_000_000)
        ctx.close()


def test_rotation_at_every_job_with_jobs_in_flight():
    """Round 6: a rotation does not wait for the worker -- it is told to leave
    between turns (published jobs or not) and its successor is queued behind
    it, starting at what it consumed.  With the bound at 0 every job published
    while a worker runs rotates it (unless a split job is outstanding: the
    test below): up to three asynchronous jobs in flight (1 group: the
    leader's; 9-64 groups: split over the workgroups, whose followers leave by
    their own launch epoch), completed in order and out of order, encode and
    recover -- every byte exact, and the worker was rotated many times."""
    from test_hip_mapped import _mapped_case as mc
    ctx = qfec.Context(0)
    bufs = []
    try:
        assert ctx.debug_service_resident(0) == 2_000_000
        shapes = [mc(n, g0=52000 + 100 * i, kmin=2, kmax=16, lmin=1, lmax=1452, seed=70 + i)
                  for i, n in enumerate((1, 9, 64, 3, 40))]
        slots = []
        for z, want_l in shapes:
            n = len(z["grp_ptr"]) - 1
            data = qfec.HostBuffer(len(z["data"]))
            data.array[:] = z["data"]
            par = qfec.HostBuffer(n * 1452)
            bufs += [data, par]
            slots.append((z, want_l, data, par, n))
        before = ctx.debug_service()
        jobs = 0
        for it in range(40):
            batch = [slots[(it + j) % len(slots)] for j in range(1 + it % 3)]
            pend = []
            for z, want_l, data, par, n in batch:
                par.array[:] = 0
                plen = np.zeros(n, dtype=np.uint16)
                ctx.encode_ragged(data.array, z["pkt_off"], z["pkt_len"], z["grp_ptr"], n,
                                  par.array, z["parity_off"], plen, mapped=True, async_=True)
                pend.append((ctx.async_ticket(), z, want_l, par, plen, n))
                jobs += 1
            for t, z, want_l, par, plen, n in (reversed(pend) if it % 2 else pend):
                assert ctx.complete_ticket(t) == 0
                assert np.array_equal(plen, want_l), it
                for g in range(n):
                    o, m = int(z["parity_off"][g]), int(want_l[g])
                    assert np.array_equal(par.array[o:o + m], z["parity"][o:o + m]), (it, n, g)
            if it % 4 == 3:  # recover too (synchronous, the same rotation path)
                z, want_l = shapes[it % len(shapes)]
                _check(ctx, z, want_l)
                jobs += 2
        st = ctx.debug_service()
        print(f"rotation at every job: {jobs} jobs, service {st}")
        assert st["jobs"] >= before["jobs"] + jobs, st
        assert st["rotations"] >= jobs // 4, st  # (a slow host's gaps let the worker idle out)
    finally:
        ctx.debug_service_resident(2_000_000)
        for b in bufs:
            b.close()
        ctx.close()


def test_quiet_service_context_leaves_the_phased_grid_whole():
    """Round 6: another context counts against a phased grid only while its
    worker runs or for 2 ms after its last job or warm (kSvcRecentNs); a
    context whose service has been quiet longer costs the grid nothing
    (8 CUs left out cost the phased encode 1.4%)."""
    import torch
    from oracle import qfec_np as Q
    a, b = qfec.Context(0), qfec.Context(0)
    try:
        z, want_l = _mapped_case(2, g0=96000, kmin=2, kmax=12, lmin=16, lmax=1350, seed=23)
        _check(b, z, want_l)  # b registered, its worker resident
        k, L = 10, 1350
        ncu = torch.cuda.get_device_properties(0).multi_processor_count
        n = 8 * ncu * 40 * (256 // ((L + 15) // 16)) + 5
        rows = torch.empty(n * k * L, dtype=torch.uint8, device="cuda:0")
        a.synth_fixed(rows, k, L, 0, n, Q.SEED_FIXED)
        par = torch.empty(n * L, dtype=torch.uint8, device="cuda:0")
        b.service_warm()
        a.encode(rows, k, L, n, par)
        assert a.last_fixed_phased() == 1
        assert a.last_phase_grid() == ncu - 8  # b's worker counted
        a.sync()
        time.sleep(0.01)  # past b's idle exit and the 2-ms window
        st = b.debug_service()
        assert st["alive"] == 0, st
        assert a.debug_other_service_cus() == (0, 0), (str(st), a.debug_other_service_cus())
        a.encode(rows, k, L, n, par)
        assert a.last_phase_grid() == ncu, str(b.debug_service())
        a.sync()
    finally:
        a.close()
        b.close()


def test_no_rotation_while_a_split_job_waits_for_late_followers():
    """Round 6: a rotation is skipped while a split job is outstanding.  Its
    followers may still be waiting for CUs (test hook: held at their start);
    the old kernel cannot end before they have done their shares, so a
    successor queued behind it would hold up every later job too.  With the
    residency bound at 0 (rotate at every job) and the followers held, the
    one-group jobs behind the split job still complete (the leader serves
    them) and nothing is rotated; once the split job is claimed, rotation
    resumes."""
    ctx = qfec.Context(0)
    z, want_l = _mapped_case(40, g0=96000, kmin=2, kmax=12, lmin=16, lmax=1350, seed=23)
    z1, want_1 = _mapped_case(2, g0=97000, kmin=2, kmax=12, lmin=16, lmax=1350, seed=24)
    data, data1 = qfec.HostBuffer(len(z["data"])), qfec.HostBuffer(len(z1["data"]))
    data.array[:] = z["data"]
    data1.array[:] = z1["data"]
    par, par1 = qfec.HostBuffer(z["parity"].size), qfec.HostBuffer(z1["parity"].size)
    try:
        ctx.debug_service_resident(0)
        ctx.debug_service_idle(200_000)  # the leader stays while the followers are held
        ctx.debug_service(on=False)  # no worker resident: the next job launches one
        ctx.debug_service(on=True)
        ctx.debug_service_hold(True)
        par.array[:] = 0
        plen = np.zeros(40, np.uint16)
        ctx.encode_ragged(data.array, z["pkt_off"], z["pkt_len"], z["grp_ptr"], 40, par.array,
                          z["parity_off"], plen, mapped=True, async_=True)
        t = ctx.async_ticket()
        before = ctx.debug_service()["rotations"]
        for _ in range(2):  # (the split job holds one of the 3 slots)
            par1.array[:] = 0
            plen1 = np.zeros(2, np.uint16)
            ctx.encode_ragged(data1.array, z1["pkt_off"], z1["pkt_len"], z1["grp_ptr"], 2,
                              par1.array, z1["parity_off"], plen1, mapped=True, async_=True)
            assert ctx.complete_ticket(ctx.async_ticket()) == 0
            assert np.array_equal(par1.array, z1["parity"])
        assert ctx.debug_service()["rotations"] == before
        ctx.debug_service_hold(False)
        assert ctx.complete_ticket(t) == 0
        assert np.array_equal(plen, want_l)
        assert np.array_equal(par.array, z["parity"])
        ctx.service_warm()
        for _ in range(3):
            _check(ctx, z1, want_1)
        assert ctx.debug_service()["rotations"] > before
    finally:
        ctx.debug_service_hold(False)
        ctx.debug_service_resident(2_000_000)
        ctx.debug_service_idle(100)
        data.close()
        data1.close()
        par.close()
        par1.close()
        ctx.close()


def test_split_job_waits_for_late_followers():
    """a follower workgroup dispatched late (test hook: the
    followers held at their start) must still do its share of every split
    job the leader took meanwhile.  Round 5's followers started from the
    host's `consumed`, already past that job, so its token never came and the
    host failed a valid batch.  Now the leader announces each split job in
    device memory and a follower takes the announcements from its own count:
    leader-only jobs complete while the followers are held, the split job
    stays pending (even after the leader's idle exit), and completes exactly
    once they are released."""
    ctx = qfec.Context(0)
    z, want_l = _mapped_case(40, g0=94000, kmin=2, kmax=12, lmin=16, lmax=1350, seed=21)
    z1, want_1 = _mapped_case(2, g0=95000, kmin=2, kmax=12, lmin=16, lmax=1350, seed=22)
    data, data1 = qfec.HostBuffer(len(z["data"])), qfec.HostBuffer(len(z1["data"]))
    data.array[:] = z["data"]
    data1.array[:] = z1["data"]
    par, par1 = qfec.HostBuffer(z["parity"].size), qfec.HostBuffer(z1["parity"].size)
    try:
        # the leader's idle time 5 ms: the one-group jobs below arrive within
        # it on any host (a leader that idled out before them would have its
        # successor queued behind the held kernel); the 20-ms pause passes it
        ctx.debug_service_idle(5_000)
        ctx.debug_service(on=False)  # no worker resident: the next job launches one
        ctx.debug_service(on=True)
        ctx.debug_service_hold(True)
        par.array[:] = 0
        plen = np.zeros(40, np.uint16)
        ctx.encode_ragged(data.array, z["pkt_off"], z["pkt_len"], z["grp_ptr"], 40, par.array,
                          z["parity_off"], plen, mapped=True, async_=True)
        t = ctx.async_ticket()
        assert t != 0
        for _ in range(2):  # (the split job holds one of the 3 slots)
            par1.array[:] = 0
            plen1 = np.zeros(2, np.uint16)
            ctx.encode_ragged(data1.array, z1["pkt_off"], z1["pkt_len"], z1["grp_ptr"], 2,
                              par1.array, z1["parity_off"], plen1, mapped=True, async_=True)
            t1 = ctx.async_ticket()
            assert ctx.complete_ticket(t1) == 0
            assert np.array_equal(plen1, want_1)
            assert np.array_equal(par1.array, z1["parity"])
        time.sleep(0.02)  # past the leader's idle exit
        assert ctx.lib.qfec_complete_ticket(ctx.ctx, t, 0) == 1  # QFEC_PENDING
        ctx.debug_service_hold(False)
        assert ctx.complete_ticket(t) == 0
        assert np.array_equal(plen, want_l)
        assert np.array_equal(par.array, z["parity"])
        # and the worker goes on: a fresh launch, split and one-group jobs exact
        for _ in range(3):
            _check(ctx, z, want_l)
            _check(ctx, z1, want_1)
    finally:
        ctx.debug_service_hold(False)
        ctx.debug_service_idle(100)
        data.close()
        data1.close()
        par.close()
        par1.close()
        ctx.close()
