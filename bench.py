"""bench.py — QUIC FEC XOR encode+recover throughput on MI355X (device-resident).

Metric (BASELINE.json): "FEC XOR encode+recover GiB/s (device-resident) on
batched 1350B packet groups".  One step = one encode pass + one single-loss
recover pass over G = 2^20 groups x 10 x 1350 B per GPU (BASELINE configs[1] +
configs[2]), inputs already resident in HBM.  Algorithmic bytes (SURVEY.md
§8(d)): encode 10*1350 read + 1350 written = 14,850 B/group; recover
9*1350 + 1350 read + 1350 written = 14,850 B/group.

Multi-GPU: one process per GPU (torchrun), each rank owns the contiguous group
range [rank*G, (rank+1)*G) — independent FEC groups, no collective on the data
path (weak scaling).  Timing: barrier + synchronize on both sides of exactly K
steps, max over ranks.

Also reported (same JSON line): the encode kernel's roofline (HIP events on
the stream the kernels run on), the CPU baseline (oracle on host cores, rank 0,
N=1), the end-to-end pinned-host rate, and the ragged (k 5-15, len 64-1350)
batch.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, MI355X_MICROARCH.md (spec 8.0 TB/s)
SEED_FIXED, SEED_RAGGED, SEED_DROP = 0x51554943, 0x51554944, 0x51554945


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1,
                   help="ranks (one process per GPU); without WORLD_SIZE in the environment "
                        "bench.py starts them itself")
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--groups", type=int, default=1 << 20, help="FEC groups per GPU")
    p.add_argument("--k", type=int, default=10)
    p.add_argument("--L", type=int, default=1350)
    p.add_argument("--cached", action="store_true",
                   help="default cache policy instead of nt loads/stores")
    p.add_argument("--one-pass", action="store_true",
                   help="QFEC_ONE_PASS: the one-pass fixed kernel instead of the phased one")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-e2e", action="store_true")
    p.add_argument("--no-ragged", action="store_true")
    p.add_argument("--no-protect", action="store_true")
    p.add_argument("--no-entropy", action="store_true")
    p.add_argument("--no-connection", action="store_true")
    p.add_argument("--no-beside-service", action="store_true",
                   help="skip the phased encode beside another context's resident worker")
    p.add_argument("--beside-only", action="store_true",
                   help="only the phased-encode-beside-a-fed-service leg, as one JSON line "
                        "(the default run starts it as a child process under a time limit)")
    p.add_argument("--no-fused", action="store_true")
    p.add_argument("--no-ceilings", action="store_true")
    p.add_argument("--no-verify", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--cpu-threads", type=int, default=0,
                   help="CPU-baseline threads (default: every host CPU)")
    p.add_argument("--cpu-workload", action="store_true",
                   help="test switch: numpy stand-in for the GPU step over gloo (no GPU); "
                        "exercises the rank launch / shard / timing / JSON path on a CPU box")
    p.add_argument("--digests", action="store_true",
                   help="test switch: every rank's parity / revived digests on the line (shards)")
    p.add_argument("--profile-only", action="store_true",
                   help="only the device-resident steps (for rocprofv3 runs)")
    p.add_argument("--protect-only", action="store_true",
                   help="only the packet-protection leg, no CPU baseline (for rocprofv3 --pmc "
                        "instruction counts: tools/pmc_protect.sh)")
    return p.parse_args(argv)


def drop_indices(g0, n, k):
    from libquic_amd import synth
    return synth.drop_indices(SEED_DROP, np.arange(g0, g0 + n, dtype=np.uint64), k).astype(np.uint8)


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return ""


def _cpu_share():
    """CPUs this process may actually use: affinity mask, capped by a cgroup v2
    CPU quota when one is set."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    return n or 1


def cpu_baseline(rows, G, k, L, seconds, threads=0):
    """The CPU FEC path (the oracle's C restatement: word-wise uint64 XOR +
    byte tail, contiguous group split over pthreads) on the host cores, over
    the SAME workload the GPU step runs — G groups x k x L, encode + recover —
    timed on every host CPU and on one core, plus configs[0] (one group).
    `rows` is the step's input copied to host memory."""
    from oracle import oracle_c as OC
    lib = OC.lib()
    threads = threads or min(256, os.cpu_count() or 1)
    par = np.zeros(G * L, np.uint8)
    out = np.zeros(G * L, np.uint8)
    miss = drop_indices(0, G, k)
    bytes_per_pass = G * (k * L + L) + G * ((k - 1) * L + 2 * L)

    def one(th):
        assert lib.qo_encode_fixed_mt(OC._p(rows), k, L, G, OC._p(par), th) == 0
        assert lib.qo_recover_fixed_mt(OC._p(rows), OC._p(par), OC._p(miss), k, L, G,
                                       OC._p(out), th) == 0

    def run(th, budget):
        one(th)  # untimed: faults the output pages in
        t0 = time.perf_counter()
        reps = 0
        while True:
            one(th)
            reps += 1
            el = time.perf_counter() - t0
            if el >= budget:
                return reps * bytes_per_pass / el / 2**30, reps, el

    # thread sweep: the box's CPU share (affinity / cgroup quota) can be far
    # below nproc, where nproc threads only oversubscribe it
    share = _cpu_share()
    cands = sorted({t for t in (share, 16, 32, 64, threads) if 1 <= t <= threads})
    sweep = {}
    for th in cands:
        v, reps, el = run(th, max(1.0, seconds / 2 / len(cands)))
        sweep[th] = round(v, 3)
    best = max(sweep, key=sweep.get)
    mt, reps_mt, el_mt = sweep[best], None, None
    st, reps_st, el_st = run(1, seconds / 2)
    # configs[0]: 1 group of 10 x 1350 B, encode + recover 1 drop, ns/group (1 core)
    ns_group = lib.qo_time_single_group_ns(k, L, 200000)
    return {
        # cores = what the threads ran on (the box's CPU share caps it); the
        # thread count is reported separately
        "value": round(mt, 3), "unit": "GiB/s", "cores": min(best, share), "threads": best,
        "kind": "port",
        "sample": f"oracle encode+recover of the bench workload itself ({G} groups x {k} x {L} B,"
                  f" {bytes_per_pass / 1e9:.1f} GB per pass): best of a thread sweep "
                  f"{sweep} (GiB/s by threads; box CPU share {share} of nproc "
                  f"{os.cpu_count()}); {reps_st} passes in {el_st:.1f} s on 1 core",
        "threads_sweep": sweep, "cpu_share": share,
        "single_core_value": round(st, 3),
        "configs0_ns_per_group_1core": round(ns_group, 1),
        "cpu_model": _cpu_model(), "nproc": os.cpu_count(),
    }


class HipFixedWorkload:
    """The product path on one GPU: G groups x k x L resident in HBM; one step =
    encode (qfec_encode_batch) + single-loss recover (qfec_recover_batch), both
    on `stream`, bracketed by HIP events on that same stream."""

    def __init__(self, torch, dev, g0, G, k, L, cached=False, one_pass=False):
        from libquic_amd import qfec
        self.torch, self.dev, self.g0, self.G, self.k, self.L = torch, dev, g0, G, k, L
        self.cached = cached
        self.one_pass = one_pass
        self.ctx = qfec.Context(dev.index)
        self.stream = torch.cuda.current_stream()
        self.ctx.set_stream(self.stream)
        self.rows = torch.empty(G * k * L, dtype=torch.uint8, device=dev)
        self.par = torch.empty(G * L, dtype=torch.uint8, device=dev)
        self.out = torch.empty(G * L, dtype=torch.uint8, device=dev)
        self.miss = torch.from_numpy(drop_indices(g0, G, k)).to(dev)
        self.ctx.synth_fixed(self.rows, k, L, g0, G, SEED_FIXED)
        self.ctx.sync()
        self.bytes_encode = G * (k * L + L)
        self.bytes_recover = G * ((k - 1) * L + 2 * L)

    def new_events(self):
        return [self.torch.cuda.Event(enable_timing=True) for _ in range(3)]

    def step(self, ev=None):
        k, L, G = self.k, self.L, self.G
        if ev:
            ev[0].record(self.stream)
        self.ctx.encode(self.rows, k, L, G, self.par, cached=self.cached, one_pass=self.one_pass)
        if ev:
            ev[1].record(self.stream)
        self.ctx.recover(self.rows, self.par, self.miss, k, L, G, self.out, cached=self.cached,
                         one_pass=self.one_pass)
        if ev:
            ev[2].record(self.stream)

    def poison(self):
        """Overwrite the outputs (untimed) so verify() can only pass on what the
        timed steps wrote."""
        self.par.fill_(0xA5)
        self.out.fill_(0x5A)
        self.synchronize()

    def synchronize(self):
        self.ctx.sync()
        self.torch.cuda.synchronize()

    def kernel_seconds(self, events):
        enc = np.array([e[0].elapsed_time(e[1]) for e in events]).mean() / 1e3
        rec = np.array([e[1].elapsed_time(e[2]) for e in events]).mean() / 1e3
        return float(enc), float(rec)

    def verify(self):
        """On the LAST timed step's outputs (device, untimed): the revived row of
        every group equals the lost row, and parity XOR all k rows == 0.
        Bit-exactness against the oracle is tests/test_hip_fixed.py's job."""
        torch, G, k, L = self.torch, self.G, self.k, self.L
        r3 = self.rows.view(G, k, L)
        ok = torch.equal(r3[torch.arange(G, device=self.dev), self.miss.long()],
                         self.out.view(G, L))
        acc = self.par.view(G, L).clone()
        for i in range(k):
            acc ^= r3[:, i]
        return bool(ok) and not bool(acc.any())

    def digests(self):
        import hashlib
        return [hashlib.sha256(self.par.cpu().numpy().tobytes()).hexdigest()[:32],
                hashlib.sha256(self.out.cpu().numpy().tobytes()).hexdigest()[:32]]

    def host_rows(self):
        return self.rows.cpu().numpy()

    def release(self):
        del self.rows
        self.torch.cuda.empty_cache()


class CpuStandInWorkload:
    """`--cpu-workload` (tests only): the same shard, step and verification
    structure as HipFixedWorkload with a numpy XOR in place of the kernels, so
    the rank launch, shard assignment, timing contract and JSON line run on a
    CPU box under gloo.  Never the measured path (the line says so)."""

    def __init__(self, g0, G, k, L):
        from libquic_amd import synth
        self.g0, self.G, self.k, self.L = g0, G, k, L
        self.rows = synth.synth_fixed_host(SEED_FIXED, g0, G, k, L)
        self.miss = drop_indices(g0, G, k)
        self.par = np.zeros(G * L, np.uint8)
        self.out = np.zeros(G * L, np.uint8)
        self.bytes_encode = G * (k * L + L)
        self.bytes_recover = G * ((k - 1) * L + 2 * L)
        self.steps = 0

    def new_events(self):
        return None

    def step(self, ev=None):
        r3 = self.rows.reshape(self.G, self.k, self.L)
        par = np.bitwise_xor.reduce(r3, axis=1)
        self.par[:] = par.reshape(-1)
        keep = r3.copy()
        keep[np.arange(self.G), self.miss] = 0
        self.out[:] = (np.bitwise_xor.reduce(keep, axis=1) ^ par).reshape(-1)
        self.steps += 1

    def poison(self):
        self.par[:] = 0xA5
        self.out[:] = 0x5A

    def synchronize(self):
        pass

    def kernel_seconds(self, events):
        return None, None

    def verify(self):
        r3 = self.rows.reshape(self.G, self.k, self.L)
        return bool(np.array_equal(self.out.reshape(self.G, self.L),
                                   r3[np.arange(self.G), self.miss]))

    def digests(self):
        import hashlib
        return [hashlib.sha256(self.par.tobytes()).hexdigest()[:32],
                hashlib.sha256(self.out.tobytes()).hexdigest()[:32]]

    def host_rows(self):
        return self.rows

    def release(self):
        pass


def timed_steps(work, steps, warmup, barrier, reduce_max):
    """The measurement contract: W untimed steps, then exactly K steps bracketed
    by barrier + synchronize on both sides; elapsed = max over ranks.  The
    outputs are poisoned before the timed steps, so the verification that
    follows checks what the timed steps wrote."""
    for _ in range(warmup):
        work.step()
    work.synchronize()
    work.poison()
    events = [work.new_events() for _ in range(steps)]
    barrier()
    work.synchronize()
    t0 = time.perf_counter()
    for s in range(steps):
        work.step(events[s])
    work.synchronize()
    elapsed = reduce_max(time.perf_counter() - t0)
    barrier()
    return elapsed, events


def phased_used(work, cpu):
    """Whether the timed fixed-shape launches ran the phased kernel, as the
    library reports it (qfec_last_fixed_phased: its size rule, kPhMinPhases in
    qfec_kernels.hip, and its contention backoff), not a copy of that rule."""
    return (not cpu) and work.ctx.last_fixed_phased() == 1


def fixed_kernel_name(k, phased):
    """The encode kernel the line's roofline is about (libquic_amd/csrc/qfec_kernels.hip)."""
    if phased:
        steps = "40 LDS + 32 register steps" if k == 10 else "40 LDS steps"
        return (f"phase_xor_kernel<{k}, false> (encode, k={k}, nt; one workgroup per CU, "
                f"reads and parity writes in separate grid-wide phases of {steps})")
    return f"fixed_xor_kernel<{k}, false, true, false, false> (encode, k={k}, nt, one pass)"


def result_line(world, steps, warmup, elapsed, G, k, L, bytes_encode, bytes_recover,
                enc_s=None, rec_s=None, traffic=None, verified=None, kernel=None):
    """The JSON line (rank 0).  value = algorithmic bytes of ALL ranks / max time.
    enc_s / rec_s: the slowest rank's mean encode / recover launch (seconds)."""
    total = world * steps * (bytes_encode + bytes_recover)
    line = {
        "metric": "FEC XOR encode+recover GiB/s (device-resident) on batched 1350B packet groups",
        "value": round(total / 2**30 / elapsed, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": round(elapsed / steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (counter-based splitmix64 bytes generated in HBM)",
        "config": {
            "workload": f"{G} groups x {k} x {L} B per GPU: parity encode + single-loss "
                        f"recover (BASELINE configs[1]+[2])",
            "groups_per_gpu": G, "k": k, "L": L,
            "parallelism": f"group-shard x{world} (no collective)",
        },
        "roofline": None,
        "verified": verified,
    }
    if enc_s:
        enc_gbs = bytes_encode / enc_s / 1e9
        rec_gbs = bytes_recover / rec_s / 1e9
        line["roofline"] = {
            "bound": "hbm",
            "kernel": kernel or fixed_kernel_name(k, False),
            "achieved": round(enc_gbs, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(enc_gbs / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "algorithmic_bytes_per_launch": bytes_encode,
            "avg_launch_us": round(enc_s * 1e6, 2),
        }
        line["encode_GiBps"] = round(bytes_encode / enc_s / 2**30, 2)
        line["recover_GiBps"] = round(bytes_recover / rec_s / 2**30, 2)
        line["recover_roofline_frac"] = round(rec_gbs / HBM_PEAK_GBS, 4)
    return line


def bench_inslot(work, steps, verify=True):
    """the in-slot recover (qfec_recover_inslot_batch) on the
    same rows and the same 14,850 B per group as the headline recover -- the
    redundancy placed in each group's lost row m, so the lost packet is the
    XOR of the k rows (one contiguous stream).  Out of place (into `out`) and
    in place (into row m; an involution, so an even number of launches leaves
    the redundancy there).  The rows are restored afterwards (untimed)."""
    torch, G, k, L = work.torch, work.G, work.k, work.L
    r3 = work.rows.view(G, k, L)
    idx = torch.arange(G, device=work.dev)
    m = work.miss.long()
    lost = r3[idx, m].clone()
    r3[idx, m] = work.par.view(G, L)  # the redundancy into the lost slot
    work.out.fill_(0x5A)
    work.synchronize()
    res = {"bytes_per_launch": G * (k * L + L),
           "note": "recover with the redundancy in the lost row: k rows read + L written per "
                   "group, the headline recover's algorithmic bytes"}
    for tag, out in (("out_of_place", work.out), ("in_place", None)):
        work.ctx.recover_inslot(work.rows, work.miss, k, L, G, out)  # warm (in place: twice)
        if out is None:
            work.ctx.recover_inslot(work.rows, work.miss, k, L, G, out)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
        ev[0].record(work.stream)
        for i in range(steps):
            work.ctx.recover_inslot(work.rows, work.miss, k, L, G, out)
            ev[i + 1].record(work.stream)
        work.synchronize()
        us = float(np.mean([ev[i].elapsed_time(ev[i + 1]) for i in range(steps)])) * 1e3
        res[tag] = {"us": round(us, 2),
                    "frac": round(res["bytes_per_launch"] / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                    "GiBps": round(res["bytes_per_launch"] / (us * 1e-6) / 2**30, 2),
                    "phased": work.ctx.last_fixed_phased() == 1}
    ok = None
    if verify:
        # out of place: every group's revived row; in place (even count): the
        # redundancy is back; one more in-place call revives into the rows
        ok = bool(torch.equal(work.out.view(G, L), lost)) and \
            bool(torch.equal(r3[idx, m], work.par.view(G, L)))
        work.ctx.recover_inslot(work.rows, work.miss, k, L, G, None)
        work.synchronize()
        ok = ok and bool(torch.equal(r3[idx, m], lost))
    r3[idx, m] = lost  # the original rows (untimed)
    work.synchronize()
    del lost
    res["verified"] = ok
    res["kernel"] = fixed_kernel_name(k, res["out_of_place"]["phased"]) + \
        " (in place: the INPL form, stores into row m)"
    return res


def bench_phase_beside_service(work, reps=6):
    """the headline encode (phased) on context A while a
    connection thread keeps context B's small-batch worker resident (the
    reference's model, one thread per QuicConnection, quic_connection.h:14):
    a native thread owning B (qfec_debug_service_feed) warms its worker at
    each turn's start and flushes one-group mapped batches back to back.  A's
    phased grid leaves B's 8 CUs out (qfec_capi.cpp other_service_cus), so no
    launch abandons its meetings.  Reported: A's encode frac (HIP events on
    A's stream), the same launches without B, A's grids, abandoned launches,
    B's batches meanwhile and whether A's parity equals the uncontended
    steps' parity."""
    from libquic_amd import qfec
    torch, ctx, s = work.torch, work.ctx, work.stream
    k, L, G = work.k, work.L, work.G
    want = work.par.clone()
    # each timed launch is queued behind a ~10 ms spin kernel on its stream,
    # so the events bracket the kernel alone, whatever the host thread does
    # between enqueueing the first event and the launch
    c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    c0.record(s)
    torch.cuda._sleep(1 << 24)
    c1.record(s)
    c1.synchronize()
    spin = max(1 << 20, int((1 << 24) * 10.0 / max(c0.elapsed_time(c1), 1e-3)))
    spins = []

    def encodes(grids):
        secs = []
        for _ in range(reps):
            es, e0, e1 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            es.record(s)
            torch.cuda._sleep(spin)
            e0.record(s)
            ctx.encode(work.rows, k, L, G, work.par)
            e1.record(s)
            grids.append(ctx.last_phase_grid())
            e1.synchronize()
            secs.append(e0.elapsed_time(e1) / 1e3)
            spins.append(es.elapsed_time(e0))
        return float(np.mean(secs[1:])) if len(secs) > 1 else float(secs[0])

    alone = encodes([])  # the same launches without the other context
    b = qfec.Context(work.dev.index)
    try:
        b.debug_service_feed(True)  # (back once its first batch is done)
        before = ctx.phase_abandons()
        grids = []
        w0 = time.perf_counter()
        try:
            enc = encodes(grids)
        finally:
            fed = b.debug_service_feed(False)
        wall = time.perf_counter() - w0
        bst = b.debug_service()
        launches, rotations = bst["launches"], bst.get("rotations")
    finally:
        b.close()
    work.synchronize()
    same = bool(torch.equal(work.par, want))
    del want
    return {"encode_frac": round(work.bytes_encode / enc / 1e9 / HBM_PEAK_GBS, 4),
            "encode_us": round(enc * 1e6, 2),
            "alone_encode_frac": round(work.bytes_encode / alone / 1e9 / HBM_PEAK_GBS, 4),
            "grids": grids,
            "ncu": torch.cuda.get_device_properties(work.dev.index).multi_processor_count,
            "abandoned": ctx.phase_abandons() - before,
            "service_jobs_meanwhile": fed["jobs"], "service_wrong": fed["wrong"],
            "service_launches": launches, "service_rotations": rotations,
            "service_us_per_job": round(wall / max(fed["jobs"], 1) * 1e6, 2),
            "spin_ms": [round(x, 1) for x in spins],
            "parity_equal_uncontended": same,
            "note": "context A's phased encode of the headline batch while a native thread owning "
                    "context B warms its small-batch worker and flushes one-group mapped batches "
                    "back to back (qfec_debug_service_feed); mean of the last reps-1 launches"}


def measured_traffic(G, k, L, phased=False):
    """PMC bytes per encode launch (tools/pmc.sh -> profiles/traffic_latest.json),
    when that run measured this shape with the same kernel (phased or one-pass)."""
    tpath = os.path.join(ROOT, "profiles", "traffic_latest.json")
    if os.path.exists(tpath):
        with open(tpath) as f:
            tj = json.load(f)
        names = " ".join(tj.get("kernels", {}).get("encode", []))
        same_kernel = ("phase_xor_kernel" in names) == phased if names else not phased
        if tj.get("groups") == G and tj.get("k") == k and tj.get("L") == L and same_kernel:
            return tj.get("encode_hbm_bytes_per_launch")
    return None


def _progress(msg):
    """One stderr line per leg (a long default run keeps producing output)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def _cpulist(text):
    cpus = set()
    for part in text.strip().split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        cpus.update(range(int(a), int(b or a) + 1))
    return cpus


def numa_bind(torch, idx):
    """Pin this rank's host threads to the NUMA node of its GPU (N>1, VERDICT r4
    item 4): the pinned host buffers of the host-memory legs are placed by
    first touch, so allocating them from a thread on the GPU's node keeps each
    GPU's PCIe traffic on its own socket's memory.  Only CPUs this process may
    use are taken (a cgroup share may hold none of the node's: then nothing is
    changed, and the line says so)."""
    try:
        p = torch.cuda.get_device_properties(idx)
        addr = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
        with open(f"/sys/bus/pci/devices/{addr}/numa_node") as f:
            node = int(f.read())
        if node < 0:
            return {"pci": addr, "numa_node": None, "pinned_cpus": 0}
        with open(f"/sys/devices/system/node/node{node}/cpulist") as f:
            cpus = _cpulist(f.read())
        use = cpus & os.sched_getaffinity(0)
        if use:
            os.sched_setaffinity(0, use)
        return {"pci": addr, "numa_node": node, "pinned_cpus": len(use)}
    except Exception as e:  # no sysfs / no torch field: report, do not fail the run
        return {"error": f"{type(e).__name__}: {e}"}


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv):
    """`python bench.py --gpus N` without a launcher: start N rank processes of
    this script (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set), one per GPU,
    and return the worst exit code.  This parent process never imports torch
    and never touches a GPU; rank 0 prints the JSON line."""
    import signal
    import subprocess
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv],
                                      env=env))
    rc = 0
    try:
        pending = list(procs)
        while pending:
            for p in list(pending):
                code = p.poll()
                if code is None:
                    continue
                pending.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code
                    for q in pending:  # a dead rank leaves the others in a collective
                        q.send_signal(signal.SIGTERM)
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    args = parse(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        if args.gpus > 1:
            return launch_ranks(args.gpus, argv)
        world = 1
    else:
        world = int(env_world)
        if world != args.gpus:
            print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
            return 2
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.groups < 1 or not 1 <= args.k <= 255 or not 1 <= args.L <= 1452 or args.steps < 1:
        print(f"bench.py[rank {rank}]: invalid workload groups={args.groups} k={args.k} "
              f"L={args.L} steps={args.steps}", file=sys.stderr)
        return 2

    import torch
    import torch.distributed as dist

    if args.beside_only:  # the beside-service leg on its own (a child of the default run)
        torch.cuda.set_device(0)
        work = HipFixedWorkload(torch, torch.device("cuda", 0), 0, args.groups, args.k, args.L)
        work.step()
        work.synchronize()
        if work.ctx.last_fixed_phased() != 1:
            print(json.dumps({"phase_beside_service": None, "note": "batch not phased"}), flush=True)
        else:
            print(json.dumps({"phase_beside_service": bench_phase_beside_service(work)}), flush=True)
        work.ctx.close()
        return 0

    if args.protect_only:  # instruction-count runs of the protection kernels
        from libquic_amd import qfec
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        ctx = qfec.Context(0)
        stream = torch.cuda.current_stream()
        ctx.set_stream(stream)
        res = bench_protect(ctx, torch, dev, stream, args.groups, args.k, args.L, reps=1, cpu=False)
        print(json.dumps({"protect": res}), flush=True)
        ctx.close()
        return 0

    cpu = args.cpu_workload
    # QFEC_BENCH_SHARE_DEVICE=1 (tests only): every rank on cuda:0, so the N>1
    # path runs on a one-GPU box (weak scaling is then not meaningful).
    share = os.environ.get("QFEC_BENCH_SHARE_DEVICE") == "1"
    if world > 1:
        # The shards exchange nothing (independent FEC groups): the control
        # plane — the timing barrier, the max of the elapsed time, the gather
        # of per-rank results — runs over gloo on CPU tensors, so the path
        # needs no RCCL (north_star: no collective).
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo")
    if not cpu:
        torch.cuda.set_device(0 if (world == 1 or share) else local)
    dev = None if cpu else torch.device("cuda", torch.cuda.current_device())
    numa = numa_bind(torch, dev.index) if (world > 1 and not cpu) else None

    def barrier():
        if world > 1:
            dist.barrier()

    def reduce_max(x):
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def gather(obj):
        if world == 1:
            return [obj]
        out = [None] * world
        dist.all_gather_object(out, obj)
        return out

    k, L, G = args.k, args.L, args.groups
    g0 = rank * G  # contiguous group shard per rank: no collective on the data path
    if cpu:
        work = CpuStandInWorkload(g0, G, k, L)
    else:
        work = HipFixedWorkload(torch, dev, g0, G, k, L, cached=args.cached,
                                one_pass=args.one_pass)
    elapsed, events = timed_steps(work, args.steps, args.warmup, barrier, reduce_max)
    enc_s, rec_s = work.kernel_seconds(events)
    verified = None if args.no_verify else work.verify()
    per_rank = gather({"rank": rank, "g0": g0, "groups": G, "enc_s": enc_s, "rec_s": rec_s,
                       "verified": verified,
                       "digests": work.digests() if (cpu or args.digests) else None,
                       "device": None if cpu else torch.cuda.current_device()})
    if enc_s:  # the roofline of the slowest rank's encode launch
        enc_s = max(r["enc_s"] for r in per_rank)
        rec_s = max(r["rec_s"] for r in per_rank)
    if verified is not None:
        verified = all(r["verified"] for r in per_rank)
    phased = phased_used(work, cpu)
    line = result_line(world, args.steps, args.warmup, elapsed, G, k, L, work.bytes_encode,
                       work.bytes_recover, enc_s, rec_s,
                       measured_traffic(G, k, L, phased), verified,
                       kernel=fixed_kernel_name(k, phased))
    if line["roofline"] and phased:
        # phased launches that gave up their meetings (should be 0 on an idle GPU)
        line["roofline"]["phase_abandons"] = work.ctx.phase_abandons()
    if world > 1 and line["roofline"]:
        fr = [work.bytes_encode / r["enc_s"] / 1e9 / HBM_PEAK_GBS for r in per_rank]
        line["roofline"]["per_rank_frac"] = {"min": round(min(fr), 4), "max": round(max(fr), 4)}
    if world > 1:
        line["control_plane"] = "gloo (CPU tensors): barrier, max, gather; no data collective"
    if world > 1 and not cpu and not args.no_e2e and not args.profile_only:
        # the host-memory path on every rank at once: each
        # GPU's pinned buffers on its own NUMA node, its own PCIe link
        barrier()
        e2e = bench_e2e(work.ctx, torch, k, L)
        e2e["rank"], e2e["numa"] = rank, numa
        per = gather(e2e)
        enc = [r["encode_GiBps"] for r in per]
        zc = [r["zero_copy"]["encode_GiBps"] for r in per]
        line["e2e_pinned_host"] = {
            "per_rank": [{kk: r.get(kk) for kk in ("rank", "encode_GiBps", "recover_GiBps",
                                                    "verified", "numa")} |
                         {"zero_copy_encode_GiBps": r["zero_copy"]["encode_GiBps"]} for r in per],
            "aggregate_encode_GiBps": round(sum(enc), 2),
            "aggregate_zero_copy_encode_GiBps": round(sum(zc), 2),
            "min_rank_encode_GiBps": min(enc),
            "verified": all(r["verified"] and r["zero_copy"]["verified"] for r in per),
            "note": "QFEC_PTR_HOST / QFEC_PTR_MAPPED legs run concurrently on every rank "
                    "(barrier-started); aggregate = sum of the per-rank rates; each rank's host "
                    "threads and pinned buffers on its GPU's NUMA node (numa)"}
    if cpu:
        line["data"] = "synthetic; --cpu-workload numpy stand-in (test of the rank path, not a measurement)"
        line["dtype"] = "u8"
    if cpu or args.digests:
        line["shards"] = [{"rank": r["rank"], "g0": r["g0"], "groups": r["groups"],
                           "device": r["device"], "verified": r["verified"],
                           "digests": r["digests"]} for r in per_rank]
    if share and world > 1:
        line["note_shared_device"] = ("QFEC_BENCH_SHARE_DEVICE: all ranks on cuda:0 (a test of the "
                                      "N>1 path, not a scaling measurement)")

    extras = rank == 0 and world == 1 and not cpu and not args.profile_only
    if rank == 0 and world == 1 and not cpu and args.profile_only and not args.no_ragged:
        # the ragged kernels' launches for the rocprofv3 runs (tools/pmc.sh)
        work.release()
        line["ragged"] = bench_ragged(work.ctx, torch, dev, work.stream, steps=3)
    if extras and not args.one_pass and phased:
        # the same steps with the one-pass kernel (QFEC_ONE_PASS), same buffers
        work.one_pass = True
        _, ev1 = timed_steps(work, args.steps, 1, barrier, reduce_max)
        e1, r1 = work.kernel_seconds(ev1)
        line["one_pass"] = {
            "kernel": fixed_kernel_name(k, False),
            "encode_frac": round(work.bytes_encode / e1 / 1e9 / HBM_PEAK_GBS, 4),
            "recover_frac": round(work.bytes_recover / r1 / 1e9 / HBM_PEAK_GBS, 4),
            "encode_us": round(e1 * 1e6, 2), "recover_us": round(r1 * 1e6, 2),
            "verified": None if args.no_verify else work.verify(),
            "note": "QFEC_ONE_PASS: the one-pass fixed kernel on the same buffers, same steps "
                    "(its rate depends on the buffers' DRAM placement, DESIGN.md §4)"}
        work.one_pass = False
    if extras and not args.one_pass:
        line["recover_inslot"] = bench_inslot(work, max(4, args.steps // 2 * 2),
                                              verify=not args.no_verify)
    if extras and not args.one_pass and phased and not args.no_beside_service:
        # in a child process under a time limit: the leg runs two contexts and
        # a native feeder thread, and a stall there must not cost the line
        _progress("phase beside service")
        import subprocess
        cmd = [sys.executable, os.path.abspath(__file__), "--beside-only", "--groups", str(G),
               "--k", str(k), "--L", str(L)]
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=240)
            js = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
            line["phase_beside_service"] = (json.loads(js[-1])["phase_beside_service"] if js else
                                            {"error": f"rc {r.returncode}", "stderr": r.stderr[-400:]})
        except subprocess.TimeoutExpired:
            line["phase_beside_service"] = {"error": "timed out (240 s)"}
        _progress("phase beside service done")
    if extras and not args.no_ceilings:
        line["ceilings"] = bench_ceilings(work.ctx, torch, work.rows, work.stream)
        if line["roofline"]:  # the encode kernel against this box's measured streaming read
            line["ceilings"]["encode_frac_of_read_ceiling"] = round(
                line["roofline"]["achieved"] / line["ceilings"]["read_GBps"], 4)
    # The CPU baseline: rank 0 at N=1 only, after the timed region, over the
    # same workload (an N>1 line carries cpu_baseline null: the N=1 line has it).
    host_rows = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.profile_only:
        host_rows = work.host_rows()
    if extras:
        work.release()
        ctx, stream = work.ctx, work.stream
        _progress("fixed-shape timed steps done")
        if not args.no_ragged:
            line["ragged"] = bench_ragged(ctx, torch, dev, stream, steps=max(5, args.steps // 2))
            line["ragged_packed"] = bench_ragged(ctx, torch, dev, stream,
                                                 steps=max(5, args.steps // 2), align=1, slot=1452)
        _progress("ragged done")
        if not args.no_protect:
            line["protect"] = bench_protect(ctx, torch, dev, stream, G, k, L,
                                            cpu=not args.no_cpu_baseline)
            if line.get("ceilings"):  # NULL encrypt is a copy + hash: its own roofline
                cp = line["ceilings"]["copy_GBps"]
                pr = line["protect"]
                pr["encrypt_frac_of_copy_ceiling"] = round(
                    pr["encrypt_hbm_frac"] * HBM_PEAK_GBS / cp, 4)
                pr["decrypt_scratch_out_frac_of_copy_ceiling"] = round(
                    pr["decrypt_scratch_out_hbm_frac"] * HBM_PEAK_GBS / cp, 4)
        _progress("protect done")
        if not args.no_entropy:
            line["entropy"] = bench_entropy(ctx, torch, dev, stream,
                                            cpu=not args.no_cpu_baseline)
        _progress("entropy done")
        # the fused leg before the host-pointer leg: that one creates the
        # context's staging streams, and the fewer streams the process has,
        # the likelier each copy direction gets a hardware queue of its own
        if not args.no_fused:
            line["e2e_fec_gcm"] = bench_fused(ctx, torch, dev, stream, k, L,
                                              cpu=not args.no_cpu_baseline)
        _progress("fused e2e done")
        if not args.no_e2e:
            line["e2e_pinned_host"] = bench_e2e(ctx, torch, k, L)
        _progress("e2e done")
        if not args.no_connection:
            line["connection"] = bench_connection(cpu=not args.no_cpu_baseline)
            _progress("connection flush done")
            line["connection_e2e"] = bench_connection_e2e()
    if host_rows is not None:
        _progress("cpu baseline")
        line["cpu_baseline"] = cpu_baseline(host_rows, G, k, L, args.cpu_seconds,
                                            args.cpu_threads)
        del host_rows
    line.setdefault("cpu_baseline", None)
    line["summary"] = line_summary(line)  # last: the driver keeps the line's last 2 KB
    barrier()
    if rank == 0:
        print(json.dumps(line), flush=True)
    if not cpu:
        work.ctx.close()
    if world > 1:
        dist.destroy_process_group()
    return 0


def line_summary(line):
    """The legs' headline numbers, compact, as the LAST key of the line: the
    driver keeps the last 2,000 characters of stdout, and the full legs
    (connection_e2e, ceilings, protect, ...) are longer than that."""
    def g(d, *path):
        for p in path:
            if not isinstance(d, dict) or p not in d:
                return None
            d = d[p]
        return d
    s = {"encode_frac": g(line, "roofline", "frac"),
         "recover_frac": line.get("recover_roofline_frac"),
         "traffic": g(line, "roofline", "traffic"),
         "kernel_phased": (g(line, "roofline", "kernel") or "").startswith("phase_xor_kernel")}
    for leg in ("one_pass", "ragged", "ragged_packed"):
        if isinstance(line.get(leg), dict):
            s[leg] = {kk: line[leg].get(kk) for kk in ("encode_frac", "recover_frac")}
    pb = line.get("phase_beside_service")
    if isinstance(pb, dict):
        s["phase_beside_service"] = {kk: pb.get(kk) for kk in
                                     ("encode_frac", "alone_encode_frac", "abandoned")}
    ri = line.get("recover_inslot")
    if isinstance(ri, dict):
        s["recover_inslot_frac"] = {kk: g(ri, kk, "frac") for kk in ("out_of_place", "in_place")}
    if isinstance(line.get("ceilings"), dict):
        s["encode_frac_of_read_ceiling"] = line["ceilings"].get("encode_frac_of_read_ceiling")
    pr = line.get("protect")
    if isinstance(pr, dict):
        s["null_encrypt_hbm_frac"] = pr.get("encrypt_hbm_frac")
        s["null_decrypt_scratch_out_hbm_frac"] = pr.get("decrypt_scratch_out_hbm_frac")
    for leg, key in (("e2e_pinned_host", "encode_GiBps"), ("e2e_fec_gcm", "payload_GiBps")):
        if isinstance(line.get(leg), dict):
            s[f"{leg}_{key}"] = line[leg].get(key, line[leg].get("aggregate_" + key))
    fg = line.get("e2e_fec_gcm")
    if isinstance(fg, dict):
        s["e2e_fec_gcm_link_frac_of_duplex_ceiling"] = fg.get("link_frac_of_duplex_ceiling")
        cbv = g(fg, "cpu_baseline", "value")
        if cbv:
            s["e2e_fec_gcm_vs_cpu"] = round(fg["payload_GiBps"] / cbv, 2)
    ce = line.get("connection_e2e")
    if isinstance(ce, dict) and ce.get("runs"):
        s["connection_e2e_host_us_per_group"] = {
            str(r["connections"]): r.get("gpu_host_us_per_group") for r in ce["runs"]}
    cb = line.get("cpu_baseline")
    if isinstance(cb, dict):
        s["cpu_baseline"] = {kk: cb.get(kk) for kk in ("value", "unit", "cores", "kind")}
    return s


def ragged_alg_bytes(G=1 << 20):
    """Algorithmic bytes of one encode / one recover launch
    over bench_ragged's batch: encode reads every packet and writes
    parity_len; recover reads the received packets and the parity and writes
    parity_len."""
    from libquic_amd import synth
    ks, ptr, ln, off = synth.ragged_layout(0, G, 5, 15, 64, 1350, SEED_RAGGED)
    plen_max = np.maximum.reduceat(ln, ptr[:-1].astype(np.int64))
    miss = synth.drop_indices(SEED_DROP, np.arange(G, dtype=np.uint64), ks).astype(np.uint8)
    lens_sum = float(ln.astype(np.float64).sum())
    pl_sum = float(plen_max.astype(np.float64).sum())
    miss_len = float(ln[ptr[:-1].astype(np.int64) + miss.astype(np.int64)].astype(np.float64).sum())
    return lens_sum + pl_sum, (lens_sum - miss_len) + 2 * pl_sum


RAGGED_ALIGN, RAGGED_SLOT = 16, 1536  # the default ragged line's layout


def ragged_layout_tag(align=RAGGED_ALIGN, slot=RAGGED_SLOT):
    return f"align{align}_slot{slot}"


def bench_ragged(ctx, torch, dev, stream, steps=10, G=1 << 20, align=RAGGED_ALIGN,
                 slot=RAGGED_SLOT):
    """configs[3]: ragged batch, k 5-15, len 64-1350 (device-resident).

    align=16 / slot=1536 (the default line): payloads on 16-B boundaries, as
    the host side's payload arena lays them out (quic_fec_group.cc
    PayloadArena::Alloc), parity / revived rows in 128-B-aligned slots.
    align=1 / slot=1452: byte-packed payloads and kMaxPacketSize slots (the
    `ragged_packed` line).  Same groups, lengths and algorithmic bytes."""
    from libquic_amd import synth
    gs = np.arange(G, dtype=np.uint64)
    ks, ptr, ln, off = synth.ragged_layout(0, G, 5, 15, 64, 1350, SEED_RAGGED, align=align)
    total = int(off[-1]) + int(ln[-1])
    plen_max = np.maximum.reduceat(ln, ptr[:-1].astype(np.int64))
    miss = synth.drop_indices(SEED_DROP, gs, ks).astype(np.uint8)
    t_off = torch.from_numpy(off.view(np.int64)).to(dev)
    t_len = torch.from_numpy(ln.view(np.int16)).to(dev)
    t_ptr = torch.from_numpy(ptr.view(np.int32)).to(dev)
    poff = np.arange(G, dtype=np.uint64) * np.uint64(slot)
    t_poff = torch.from_numpy(poff.view(np.int64)).to(dev)
    t_miss = torch.from_numpy(miss).to(dev)
    data = torch.empty(total, dtype=torch.uint8, device=dev)
    ctx.synth_ragged(data, t_off, t_len, t_ptr, 0, G, SEED_RAGGED)
    par = torch.empty(G * slot, dtype=torch.uint8, device=dev)
    plen = torch.empty(G, dtype=torch.int16, device=dev)
    out = torch.empty(G * slot, dtype=torch.uint8, device=dev)

    def run(ev=None):
        if ev:
            ev[0].record(stream)
        ctx.encode_ragged(data, t_off, t_len, t_ptr, G, par, t_poff, plen)
        if ev:
            ev[1].record(stream)
        ctx.recover_ragged(data, t_off, t_len, t_ptr, G, par, t_poff, plen, t_miss, out, t_poff)
        if ev:
            ev[2].record(stream)

    run()  # warm
    ctx.sync()
    par.fill_(0xA5)  # poison: the check below sees only what the timed steps wrote
    out.fill_(0x5A)
    plen.fill_(0)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
    torch.cuda.synchronize()
    for s in range(steps):
        run(evs[s])
    torch.cuda.synchronize()
    enc = np.mean([e[0].elapsed_time(e[1]) for e in evs]) / 1e3
    rec = np.mean([e[1].elapsed_time(e[2]) for e in evs]) / 1e3
    # verify the last timed step: parity lengths, the revived packet of a
    # sample of groups (zero tail to parity_len), parity XOR rows == 0 there
    ok = np.array_equal(plen.cpu().numpy().view(np.uint16), plen_max)
    out_h = out.cpu().numpy()
    par_h = par.cpu().numpy()
    data_h = data.cpu().numpy()
    for g in np.random.default_rng(0).choice(G, 256, replace=False):
        p = int(ptr[g]) + int(miss[g])
        o, l_ = int(off[p]), int(ln[p])
        pl = int(plen_max[g])
        seg = out_h[g * slot: g * slot + pl]
        ok = ok and np.array_equal(seg[:l_], data_h[o:o + l_]) and not seg[l_:].any()
        acc = par_h[g * slot: g * slot + pl].copy()
        for q in range(int(ptr[g]), int(ptr[g + 1])):
            acc[:int(ln[q])] ^= data_h[int(off[q]):int(off[q]) + int(ln[q])]
        ok = ok and not acc.any()
    b_enc, b_rec = ragged_alg_bytes(G)
    traffic = None
    tpath = os.path.join(ROOT, "profiles", "traffic_latest.json")
    if os.path.exists(tpath):
        with open(tpath) as f:
            tj = json.load(f)
        ent = tj.get("ragged_by_layout", {}).get(ragged_layout_tag(align, slot))
        if tj.get("ragged_groups") == G and ent:
            traffic = {kd: ent.get(kd) for kd in ("encode", "recover")}
            traffic["source"] = ("profiles/traffic_latest.json (PMC FETCH_SIZE + WRITE_SIZE, run "
                                 f"{ent.get('source')})")
    layout = ("packed CSR (byte offsets)" if align == 1 else
              f"CSR, payloads on {align}-B boundaries (the payload arena's layout)")
    return {"groups": G, "k": "5-15", "len": "64-1350", "layout": layout,
            "parity_slot_bytes": slot,
            "encode_GiBps": round(b_enc / enc / 2**30, 2),
            "recover_GiBps": round(b_rec / rec / 2**30, 2),
            "encode_frac": round(b_enc / enc / 1e9 / HBM_PEAK_GBS, 4),
            "recover_frac": round(b_rec / rec / 1e9 / HBM_PEAK_GBS, 4),
            "encode_us": round(enc * 1e6, 1), "recover_us": round(rec * 1e6, 1),
            "hbm_traffic_over_algorithmic": traffic, "verified": bool(ok),
            "kernel": "ragged_block_kernel<RECOVER, 4, 8> (4 waves x 8 groups per block, one flat window space; aligned last windows loaded in place)"}


def _time_on(torch, stream, fn, reps):
    """Mean ms of fn() over reps, HIP events on `stream` (the kernels' stream)."""
    fn()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def bench_ceilings(ctx, torch, buf, stream, reps=5):
    """Measured streaming ceilings on this GPU: nt read of the
    whole rows buffer and an nt copy of half of it into the other half."""
    n = buf.numel()
    half = (n // 2) & ~15
    ms_r = _time_on(torch, stream, lambda: ctx.stream_probe(buf, n, buf, copy=False), reps)
    ms_c = _time_on(torch, stream, lambda: ctx.stream_probe(buf, half, buf[half:], copy=True),
                    reps)
    return {"read_GBps": round(n / ms_r / 1e6, 1), "copy_GBps": round(2 * half / ms_c / 1e6, 1),
            "read_frac_of_peak": round(n / ms_r / 1e6 / HBM_PEAK_GBS, 4),
            "note": "nt 16-B streaming kernels (qfec_stream_probe), bytes moved / time"}


def bench_protect(ctx, torch, dev, stream, G, k, L, hdr=22, reps=5, cpu=True):
    """Packet protection around FEC (ENCRYPTION_NONE, FNV-1a-128 tag): every
    data packet of the headline workload (G x k packets of L bytes, a
    `hdr`-byte header each) encrypted and decrypted in one batch each."""
    n = G * k
    rec = hdr + L
    data = torch.empty(n * rec, dtype=torch.uint8, device=dev)
    # payload bytes from the counter-based generator (k rows of L at stride rec)
    ctx.synth_fixed(data[hdr:], k, L, 0, G, SEED_FIXED, row_stride=rec, group_stride=k * rec)
    ar = torch.arange(n, dtype=torch.int64, device=dev)
    # header of packet p = the hdr bytes in front of its payload (the synth
    # generator left them untouched: fill them with a pattern)
    data.view(n, rec)[:, :hdr] = (ar.view(n, 1) * 131 + torch.arange(hdr, device=dev)).to(torch.uint8)
    ad_off = ar * rec
    pt_off = ad_off + hdr
    ad_len = torch.full((n,), hdr, dtype=torch.int16, device=dev)
    pt_len = torch.full((n,), L, dtype=torch.int16, device=dev)
    out = torch.empty(n * (L + 12), dtype=torch.uint8, device=dev)
    out_off = ar * (L + 12)
    ms_e = _time_on(torch, stream, lambda: ctx.null_encrypt(data, ad_off, ad_len, pt_off, pt_len, n,
                                                            out, out_off), reps)
    # in place, as QuicPacketCreator::EncryptInPlace calls it: [header |
    # payload | 12 spare] records, the tag written over the payload start and
    # the payload shifted right by 12 (the kernel's in-place ordering rule)
    ip_rec = hdr + L + 12
    ip = torch.empty(n * ip_rec, dtype=torch.uint8, device=dev)
    ipv = ip.view(n, ip_rec)
    ipv[:, :rec] = data.view(n, rec)
    ip_ad, ip_pt = ar * ip_rec, ar * ip_rec + hdr
    ctx.null_encrypt(ip, ip_ad, ad_len, ip_pt, pt_len, n, ip, ip_pt)  # from fresh plaintext
    ctx.sync()
    verified_ip = torch.equal(ipv[:, hdr:], out.view(n, L + 12))
    ms_ip = _time_on(torch, stream, lambda: ctx.null_encrypt(ip, ip_ad, ad_len, ip_pt, pt_len, n,
                                                             ip, ip_pt), reps)
    del ip, ipv
    # out of place on payload-aligned records: a host batcher that places each
    # record so that its payload starts on a 16-B boundary on both sides
    # ([pad 10 | header 22 | payload] in, [pad 4 | tag 12 | payload] out, 1,376-B
    # records) — the layout study of DESIGN.md §9 on the bench's batch
    AS = (rec + 10 + 15) // 16 * 16
    al_in = torch.empty(n * AS, dtype=torch.uint8, device=dev)
    al_in.view(n, AS)[:, 10:10 + rec] = data.view(n, rec)
    al_out = torch.empty(n * AS, dtype=torch.uint8, device=dev)
    al_ad, al_pt, al_oo = ar * AS + 10, ar * AS + 10 + hdr, ar * AS + 4
    ctx.null_encrypt(al_in, al_ad, ad_len, al_pt, pt_len, n, al_out, al_oo)
    ctx.sync()
    verified_al = torch.equal(al_out.view(n, AS)[:, 4:4 + L + 12], out.view(n, L + 12))
    ms_al = _time_on(torch, stream, lambda: ctx.null_encrypt(al_in, al_ad, ad_len, al_pt, pt_len,
                                                             n, al_out, al_oo), reps)
    del al_in, al_out
    # decrypt: [header | ciphertext] records
    crec = hdr + L + 12
    cat = torch.empty(n * crec, dtype=torch.uint8, device=dev)
    cv = cat.view(n, crec)
    cv[:, :hdr] = data.view(n, rec)[:, :hdr]
    cv[:, hdr:] = out.view(n, L + 12)
    del out
    ct_len = torch.full((n,), L + 12, dtype=torch.int16, device=dev)
    dout = torch.empty(n * L, dtype=torch.uint8, device=dev)
    ok = torch.zeros(n, dtype=torch.uint8, device=dev)
    c_ad_off, c_ct_off, d_out_off = ar * crec, ar * crec + hdr, ar * L
    ms_d = _time_on(torch, stream, lambda: ctx.null_decrypt(cat, c_ad_off, ad_len, c_ct_off,
                                                            ct_len, n, dout, d_out_off, ok), reps)
    ctx.sync()
    verified = bool(ok.all()) and torch.equal(dout.view(n, L), data.view(n, rec)[:, hdr:])
    # the one-pass decrypt (QFEC_SCRATCH_OUTPUT: a failed packet's output may
    # hold its unverified plaintext, as in QuicFramer's scratch buffer)
    dout.fill_(0)
    ok.zero_()
    ms_d1 = _time_on(torch, stream, lambda: ctx.null_decrypt(
        cat, c_ad_off, ad_len, c_ct_off, ct_len, n, dout, d_out_off, ok, scratch_out=True), reps)
    ctx.sync()
    verified = verified and bool(ok.all()) and torch.equal(dout.view(n, L),
                                                           data.view(n, rec)[:, hdr:])
    # ChaCha20-Poly1305 (one key, packet numbers 1..n): seal -> out (ct || tag),
    # open of [header | ct || tag] records
    key = torch.arange(32, dtype=torch.uint8, device=dev) * 7 + 1
    pre = torch.tensor([0xA0, 0xA1, 0xA2, 0xA3], dtype=torch.uint8, device=dev)
    kidx = torch.zeros(n, dtype=torch.int32, device=dev)
    pn = ar + 1
    out = torch.empty(n * (L + 12), dtype=torch.uint8, device=dev)
    ms_cs = _time_on(torch, stream, lambda: ctx.chacha20poly1305_seal(
        key, pre, kidx, pn, None, data, ad_off, ad_len, pt_off, pt_len, n, out, out_off), reps)
    cv[:, hdr:] = out.view(n, L + 12)
    del out
    ms_co = _time_on(torch, stream, lambda: ctx.chacha20poly1305_open(
        key, pre, kidx, pn, None, cat, c_ad_off, ad_len, c_ct_off, ct_len, n, dout, d_out_off,
        ok), reps)
    ctx.sync()
    verified_c = bool(ok.all()) and torch.equal(dout.view(n, L), data.view(n, rec)[:, hdr:])
    dout.fill_(0)
    ok.zero_()
    ms_co1 = _time_on(torch, stream, lambda: ctx.chacha20poly1305_open(
        key, pre, kidx, pn, None, cat, c_ad_off, ad_len, c_ct_off, ct_len, n, dout, d_out_off,
        ok, scratch_out=True), reps)
    ctx.sync()
    verified_c = verified_c and bool(ok.all()) and torch.equal(dout.view(n, L),
                                                               data.view(n, rec)[:, hdr:])
    # AES-128-GCM-12 (one key: every wave key-uniform, the Shoup-table GHASH path)
    gkey = torch.arange(16, dtype=torch.uint8, device=dev) * 11 + 3
    out = torch.empty(n * (L + 12), dtype=torch.uint8, device=dev)
    ms_gs = _time_on(torch, stream, lambda: ctx.aes128gcm_seal(
        gkey, pre, kidx, pn, None, data, ad_off, ad_len, pt_off, pt_len, n, out, out_off), reps)
    cv[:, hdr:] = out.view(n, L + 12)
    del out
    ok.zero_()
    ms_go = _time_on(torch, stream, lambda: ctx.aes128gcm_open(
        gkey, pre, kidx, pn, None, cat, c_ad_off, ad_len, c_ct_off, ct_len, n, dout, d_out_off,
        ok), reps)
    ctx.sync()
    verified_g = bool(ok.all()) and torch.equal(dout.view(n, L), data.view(n, rec)[:, hdr:])
    dout.fill_(0)
    ok.zero_()
    ms_go1 = _time_on(torch, stream, lambda: ctx.aes128gcm_open(
        gkey, pre, kidx, pn, None, cat, c_ad_off, ad_len, c_ct_off, ct_len, n, dout, d_out_off,
        ok, scratch_out=True), reps)
    ctx.sync()
    verified_g = verified_g and bool(ok.all()) and torch.equal(dout.view(n, L),
                                                               data.view(n, rec)[:, hdr:])
    b_enc = n * (hdr + L + L + 12)  # read header + payload, write tag + payload
    b_dec = n * (hdr + L + 12 + L)
    res = {"packets": n, "header": hdr, "payload": L,
           "encrypt_GiBps": round(b_enc / (ms_e / 1e3) / 2**30, 2),
           "decrypt_GiBps": round(b_dec / (ms_d / 1e3) / 2**30, 2),
           "decrypt_scratch_out_GiBps": round(b_dec / (ms_d1 / 1e3) / 2**30, 2),
           "decrypt_scratch_out_hbm_frac": round(b_dec / (ms_d1 / 1e3) / 8e12, 4),
           "encrypt_hashed_GBps": round(n * (hdr + L) / (ms_e / 1e3) / 1e9, 1),
           "encrypt_hbm_frac": round(b_enc / (ms_e / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
           "encrypt_in_place_GiBps": round(b_enc / (ms_ip / 1e3) / 2**30, 2),
           "encrypt_in_place_hbm_frac": round(b_enc / (ms_ip / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
           "encrypt_in_place_verified": verified_ip,
           "encrypt_aligned_records_GiBps": round(b_enc / (ms_al / 1e3) / 2**30, 2),
           "encrypt_aligned_records_hbm_frac": round(b_enc / (ms_al / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
           "encrypt_aligned_records_verified": verified_al,
           "encrypt_aligned_records_layout": ("out of place, payloads on 16-B boundaries on both "
                                              f"sides ({AS}-B records)"),
           "encrypt_us": round(ms_e * 1e3, 1), "decrypt_us": round(ms_d * 1e3, 1),
           "bound": "memory pipeline of the packed layout's unaligned payload loads (stores 16-B aligned on a 128-B line grid; VALU busy ~0.6: serial FNV-1a-128 per packet, 3 bytes per multiply, VALU-only bound ~3.9 TB/s hashed)",
           "verified": verified,
           "chacha20poly1305": {
               "seal_GiBps": round(b_enc / (ms_cs / 1e3) / 2**30, 2),
               "open_GiBps": round(b_dec / (ms_co / 1e3) / 2**30, 2),
               "open_scratch_out_GiBps": round(b_dec / (ms_co1 / 1e3) / 2**30, 2),
               "seal_payload_GBps": round(n * L / (ms_cs / 1e3) / 1e9, 1),
               "seal_us": round(ms_cs * 1e3, 1), "open_us": round(ms_co * 1e3, 1),
               "verified": verified_c},
           "aes128gcm": {
               "seal_GiBps": round(b_enc / (ms_gs / 1e3) / 2**30, 2),
               "open_GiBps": round(b_dec / (ms_go / 1e3) / 2**30, 2),
               "open_scratch_out_GiBps": round(b_dec / (ms_go1 / 1e3) / 2**30, 2),
               "seal_payload_GBps": round(n * L / (ms_gs / 1e3) / 1e9, 1),
               "seal_us": round(ms_gs * 1e3, 1), "open_us": round(ms_go * 1e3, 1),
               "verified": verified_g}}
    def targs(k):  # the kernel's template arguments
        return [x.strip() for x in k.split("<", 1)[1].rsplit(">", 1)[0].split(",")] if "<" in k else []

    def gcm(open_, onepass):
        return lambda k: ("aes128gcm_kernel" in k and targs(k)[1] == ("true" if open_ else "false")
                          and (len(targs(k)) > 6 and targs(k)[6] == "true") == onepass)

    res["issue_bound"] = {
        "null_encrypt": _issue_bound(lambda k: "null_encrypt_staged" in k, n, ms_e),
        "null_decrypt": _issue_bound(lambda k: "null_decrypt_staged" in k, n, ms_d),
        "null_decrypt_scratch_out": _issue_bound(lambda k: "null_decrypt_onepass" in k, n, ms_d1),
        "chacha20poly1305_seal": _issue_bound(lambda k: "c20p1305_seal" in k, n, ms_cs),
        "chacha20poly1305_open": _issue_bound(
            lambda k: "c20p1305_open" in k and targs(k)[1:2] != ["true"], n, ms_co),
        "chacha20poly1305_open_scratch_out": _issue_bound(
            lambda k: "c20p1305_open" in k and targs(k)[1:2] == ["true"], n, ms_co1),
        "aes128gcm_seal": _issue_bound(gcm(False, False), n, ms_gs),
        "aes128gcm_open": _issue_bound(gcm(True, False), n, ms_go),
        "aes128gcm_open_scratch_out": _issue_bound(gcm(True, True), n, ms_go1),
        "note": "fraction of kernel time the VALU / LDS / scalar units were busy (PMC)"}
    del cat, dout, data
    torch.cuda.empty_cache()
    if cpu:
        res["cpu_baseline"] = cpu_protect_baseline(hdr, L)
    return res


def _issue_bound(kernel_pred, n, ms):
    """Compute-roofline fractions of a protection kernel, from the PMC passes
    in profiles/protect_insts_latest.json (tools/pmc_protect.sh): the
    fraction of the kernel's time the CUs' VALU / LDS / scalar units were
    busy (rocprofv3's VALUBusy definition) and its wave instructions per
    packet.  A VALU-bound kernel sits near valu_busy = 1."""
    path = os.path.join(ROOT, "profiles", "protect_insts_latest.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        pj = json.load(f)
    for name, kd in pj.get("kernels", {}).items():
        if kernel_pred(name):
            pp = kd.get("per_packet", {})
            r = {"kernel": name,
                 "valu_insts_per_packet": round(pp.get("SQ_INSTS_VALU", 0.0), 1),
                 "lds_insts_per_packet": round(pp.get("SQ_INSTS_LDS", 0.0), 1),
                 "source": "profiles/protect_insts_latest.json"}
            for u in ("valu", "lds", "salu"):
                if f"{u}_busy" in kd:
                    r[f"{u}_busy"] = round(kd[f"{u}_busy"], 4)
            r.update(_stall_picture(name))
            return r
    return None


def _stall_picture(name):
    """the kernel's issue fractions against the CU's issue
    ceilings (SIMD-32: a wave64 VALU instruction issues in 2 cycles, 2 per CU
    per cycle; a 64-lane ds_read_b32 moves 256 B at 128 B per CU per cycle,
    0.5 per CU per cycle) and where its waves' cycles go (PMC:
    tools/pmc_aead_stall.sh -> profiles/round5/aead_stall.json, kept as
    profiles/aead_stall_latest.json: the round directories do not travel to
    the GPU box)."""
    path = os.path.join(ROOT, "profiles", "aead_stall_latest.json")
    if not os.path.exists(path):
        return {}
    with open(path) as f:
        kd = json.load(f).get("kernels", {}).get(name)
    if not kd:
        return {}
    keys = ("valu_issue_frac", "lds_issue_frac", "waves_per_simd", "active_any_frac",
            "wait_any_frac", "wait_inst_any_frac", "wait_lds_frac")
    return {"stall": {k: round(kd[k], 3) for k in keys if k in kd} |
            {"source": "profiles/aead_stall_latest.json (= round5/aead_stall.json)"}}


def cpu_protect_baseline(hdr, L, n=1 << 16, seconds=4.0):
    res = _cpu_null_baseline(hdr, L, n, seconds)
    res["chacha20poly1305"] = _cpu_aead_baseline("chacha20poly1305", hdr, L, n // 4, seconds)
    res["aes128gcm"] = _cpu_aead_baseline("aes128gcm", hdr, L, n // 4, seconds)
    return res


def _cpu_aead_baseline(aead, hdr, L, n, seconds):
    """AEAD seal on the host cores: the reference's own Aes128Gcm12Encrypter /
    ChaCha20Poly1305Encrypter over BoringSSL built WITH its x86-64 assembly
    (oracle/_ref/libref_aead_asm.so: AES-NI + PCLMULQDQ, SIMD ChaCha20 and
    Poly1305), or the vector-pinned scalar C restatement where that build is
    absent (kind "port")."""
    from oracle import oracle_c as OC
    from oracle import ref_quic
    threads = _cpu_share()
    rec = hdr + L
    rng = np.random.default_rng(2)
    data = rng.integers(0, 256, n * rec, dtype=np.uint8)
    ar = np.arange(n, dtype=np.uint64)
    ad_off, pt_off = ar * np.uint64(rec), ar * np.uint64(rec) + np.uint64(hdr)
    ad_len = np.full(n, hdr, np.uint16)
    pt_len = np.full(n, L, np.uint16)
    out_off = ar * np.uint64(L + 12)
    keys = np.arange(32 if aead == "chacha20poly1305" else 16, dtype=np.uint8)
    kind, what = "port", "scalar C restatement pinned by BoringSSL's vectors"
    seal = OC.quic_c20p1305_encrypt_batch if aead == "chacha20poly1305" \
        else OC.quic_aes128gcm_encrypt_batch
    feats = None
    if ref_quic.asm_available():
        feats = ref_quic.asm_cpu_features()
        kind = "reference"
        what = ("the reference's EncryptPacket over BoringSSL with its x86-64 assembly, "
                f"CPU features {sorted(k for k, v in feats.items() if v)}")

        def seal(keys, pre, kidx, pn, path, *rest, threads, out):
            return ref_quic.asm_seal_batch(aead, keys, pre, kidx, pn, *rest, threads=threads,
                                           out=out)
    name = "ChaCha20-Poly1305" if aead == "chacha20poly1305" else "AES-128-GCM-12"
    obuf = np.zeros(n * (L + 12), np.uint8)  # reused: no page faults in the timed loop
    pre = np.arange(4, dtype=np.uint8)
    kidx = np.zeros(n, np.uint32)
    pn = ar + np.uint64(1)

    def run(th, budget):
        seal(keys, pre, kidx, pn, None, data, ad_off, ad_len, pt_off, pt_len, out_off,
             n * (L + 12), threads=th, out=obuf)  # untimed
        t0, reps = time.perf_counter(), 0
        while time.perf_counter() - t0 < budget:
            seal(keys, pre, kidx, pn, None, data, ad_off, ad_len, pt_off, pt_len, out_off,
                 n * (L + 12), threads=th, out=obuf)
            reps += 1
        el = time.perf_counter() - t0
        return reps * n * (hdr + L + L + 12) / el / 2**30, reps
    mt, reps = run(threads, seconds / 2)
    st, _ = run(1, seconds / 4)
    return {"value": round(mt, 3), "unit": "GiB/s", "cores": threads, "threads": threads,
            "kind": kind, "single_core_value": round(st, 3),
            "sample": f"{name} seal of {n} packets ({hdr}+{L} B), {reps} passes on {threads} "
                      f"threads ({what})"}


def _cpu_null_baseline(hdr, L, n, seconds):
    """NullEncrypter::EncryptPacket on the host cores: the reference's own
    null_encrypter.cc + quic_utils.cc (oracle/_ref) when present, else the
    reference-pinned C restatement."""
    from oracle import oracle_c as OC
    from oracle import ref_quic
    enc, kind, what = OC.null_encrypt_batch, "port", "restatement pinned against the reference build"
    if ref_quic.available():
        enc, kind, what = ref_quic.null_encrypt_batch, "reference", \
            "the reference's NullEncrypter compiled from its sources"
    threads = _cpu_share()
    rec = hdr + L
    rng = np.random.default_rng(1)
    data = rng.integers(0, 256, n * rec, dtype=np.uint8)
    ar = np.arange(n, dtype=np.uint64)
    ad_off, pt_off = ar * np.uint64(rec), ar * np.uint64(rec) + np.uint64(hdr)
    ad_len = np.full(n, hdr, np.uint16)
    pt_len = np.full(n, L, np.uint16)
    out_off = ar * np.uint64(L + 12)
    obuf = np.zeros(n * (L + 12), np.uint8)  # reused: no page faults in the timed loop

    def run(th):
        t0, reps = time.perf_counter(), 0
        while True:
            enc(data, ad_off, ad_len, pt_off, pt_len, out_off, n * (L + 12), threads=th,
                out=obuf)
            reps += 1
            el = time.perf_counter() - t0
            if el >= seconds / 2:
                return reps * n * (hdr + L + L + 12) / el / 2**30, reps
    mt, reps_mt = run(threads)
    st, _ = run(1)
    return {"value": round(mt, 3), "unit": "GiB/s", "cores": threads, "kind": kind,
            "single_core_value": round(st, 3),
            "sample": f"NULL encrypt of {n} packets ({hdr}+{L} B), {reps_mt} passes on "
                      f"{threads} threads ({what})"}


def entropy_workload(C, W, seed=7):
    """C connections x W-packet windows of sent-packet entropy hashes (random
    entropy bits, hash = flag << (pn % 8)), one ack per connection with two
    missing intervals and its true claimed hash (host numpy; the claim is what
    the peer would send)."""
    rng = np.random.default_rng(seed)
    pn0 = rng.integers(1, 1 << 30, C).astype(np.uint64)
    flags = rng.integers(0, 2, (C, W)).astype(np.uint8)
    e = (flags << ((pn0[:, None] + np.arange(W, dtype=np.uint64)) % np.uint64(8))
         .astype(np.uint8)).astype(np.uint8)
    base = rng.integers(0, 256, C).astype(np.uint8)
    cum = np.bitwise_xor.accumulate(e, axis=1) ^ base[:, None]
    off = np.sort(rng.integers(0, W, (C, 4)), axis=1)  # window offsets of 2 intervals
    off[:, 1] += 1
    off[:, 3] += 1
    off[:, 2] = np.maximum(off[:, 2], off[:, 1])
    off[:, 3] = np.maximum(off[:, 3], off[:, 2] + 1)
    off = np.minimum(off, W)
    largest_off = np.full(C, W - 1)
    rows = np.arange(C)

    def at(o):  # cumulative through window offset o-1 (o = 0: the base)
        return np.where(o > 0, cum[rows, np.maximum(o - 1, 0)], base)
    claimed = cum[rows, largest_off] ^ at(off[:, 1]) ^ at(off[:, 0]) ^ at(off[:, 3]) ^ at(off[:, 2])
    lo = (pn0[:, None] + off[:, [0, 2]].astype(np.uint64)).reshape(-1)
    hi = (pn0[:, None] + off[:, [1, 3]].astype(np.uint64)).reshape(-1)
    return {"entropy": e.reshape(-1), "conn_ptr": np.arange(C + 1, dtype=np.uint64) * np.uint64(W),
            "first_pn": pn0, "cum_base": base, "ack_conn": rows.astype(np.uint32),
            "largest": pn0 + largest_off.astype(np.uint64), "claimed": claimed.astype(np.uint8),
            "range_ptr": (np.arange(C + 1) * 2).astype(np.uint32), "range_lo": lo,
            "range_hi": hi, "cum": cum.reshape(-1)}


def bench_entropy(ctx, torch, dev, stream, C=1 << 20, W=128, reps=10, cpu=True):
    """cumulative entropy of every sent packet of 2^20
    connections (128-packet windows) + validation of one ack per connection
    (two missing intervals each), device-resident."""
    d = entropy_workload(C, W)

    def dv(a):
        sig = {1: np.uint8, 4: np.int32, 8: np.int64}[a.dtype.itemsize]
        return torch.from_numpy(np.ascontiguousarray(a).view(sig)).to(dev)
    t = {k: dv(v) for k, v in d.items() if k != "cum"}
    cum = torch.empty(C * W, dtype=torch.uint8, device=dev)
    ok = torch.zeros(C, dtype=torch.uint8, device=dev)
    scan = lambda: ctx.entropy_cumulative(t["entropy"], t["conn_ptr"], t["cum_base"], C, cum,  # noqa: E731
                                          n_packets=C * W)
    val = lambda: ctx.entropy_validate(cum, t["conn_ptr"], t["first_pn"], t["cum_base"], C,  # noqa: E731
                                       t["ack_conn"], t["largest"], t["claimed"], t["range_ptr"],
                                       t["range_lo"], t["range_hi"], C, ok)
    ms_s = _time_on(torch, stream, scan, reps)
    ms_v = _time_on(torch, stream, val, reps)
    ctx.sync()
    verified = bool(ok.all()) and np.array_equal(cum.cpu().numpy(), d["cum"])
    # algorithmic bytes: scan reads 1 B + writes 1 B per packet (+ 9 B/connection
    # of pointers and base); validation reads 8+8+4+1 B per ack, 16 B per
    # interval, 4 cumulative bytes + 2 window pointers (16 B) and writes 1 B
    b_scan = C * W * 2 + C * 9
    b_val = C * (8 + 8 + 4 + 1 + 4 + 2 * 16 + 4 + 16 + 8 + 1 + 1)
    res = {"connections": C, "window": W, "acks": C,
           "cumulative_GBps": round(b_scan / (ms_s / 1e3) / 1e9, 1),
           "cumulative_us": round(ms_s * 1e3, 1),
           "cumulative_Gpackets_per_s": round(C * W / (ms_s / 1e3) / 1e9, 2),
           "validate_us": round(ms_v * 1e3, 1),
           "validate_Macks_per_s": round(C / (ms_v / 1e3) / 1e6, 1),
           "validate_GBps": round(b_val / (ms_v / 1e3) / 1e9, 1),
           "bound": "hbm (1-byte hashes; scan: 2 B/packet)", "verified": verified}
    del t, cum, ok
    torch.cuda.empty_cache()
    if cpu:
        res["cpu_baseline"] = _cpu_entropy_baseline(d, C)
    return res


def _cpu_entropy_baseline(d, C, n=1 << 16, seconds=3.0):
    """Oracle (reference-pinned restatement of QuicSentEntropyManager's
    cumulative / IsValidEntropy walk) on one host core over a sample."""
    from oracle import oracle_c as OC
    W = int(d["conn_ptr"][1])
    sub = {"entropy": d["entropy"][:n * W], "conn_ptr": d["conn_ptr"][:n + 1],
           "first_pn": d["first_pn"][:n], "cum_base": d["cum_base"][:n],
           "ack_conn": d["ack_conn"][:n], "largest": d["largest"][:n],
           "claimed": d["claimed"][:n], "range_ptr": d["range_ptr"][:n + 1],
           "range_lo": d["range_lo"][:2 * n], "range_hi": d["range_hi"][:2 * n]}
    t0, reps = time.perf_counter(), 0
    while time.perf_counter() - t0 < seconds:
        cum = OC.entropy_cumulative_batch(sub["entropy"], sub["conn_ptr"], sub["cum_base"])
        OC.entropy_validate_batch(cum, sub["conn_ptr"], sub["first_pn"], sub["cum_base"],
                                  sub["ack_conn"], sub["largest"], sub["claimed"],
                                  sub["range_ptr"], sub["range_lo"], sub["range_hi"])
        reps += 1
    el = time.perf_counter() - t0
    return {"value": round(reps * n * W / el / 1e9, 3), "unit": "Gpackets/s (cumulative + validate)",
            "cores": 1, "kind": "port",
            "sample": f"oracle over {n} connections x {W} packets + {n} acks, {reps} passes "
                      f"(restatement pinned against the reference's QuicSentEntropyManager; "
                      f"the reference runs it per connection on the connection thread)"}


def bench_connection(cpu=True):
    """Connection layer (QuicFecEncodeBatch / QuicFecReviveBatch::Flush through
    the host-pointer ragged path): us per Flush and groups/s at 1, 64, 4096,
    65536 groups of 10 x 1350 B, beside the reference's per-connection CPU
    accumulate on one core (tests/cpp/bench_connection.cc)."""
    import subprocess
    exe = os.path.join(ROOT, "tests", "cpp", "build", "bench_connection")
    if not os.path.exists(exe):
        return {"error": f"{exe} not built"}
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        return {"error": (r.stderr or r.stdout)[-400:]}
    res = json.loads(r.stdout.strip().splitlines()[-1])
    res["note"] = ("one Flush = CSR build + one ragged launch reading the groups' payloads in "
                   "place from the pinned payload arena (QFEC_PTR_MAPPED) + the redundancy / "
                   "revived views (wall, median); up to 256 groups the index tables are read in "
                   "place too and the host spins on a completion flag the kernel's last "
                   "workgroup stores (latency path), above that they are staged to the device; "
                   "batches of up to 64 groups go to the resident small-batch service, which each "
                   "rep's turn start warms (qfec_service_warm) before the batch is assembled "
                   "(encode_build_us), as an event loop does; "
                   "cpu_1core = the oracle's per-group XorBuffers accumulate (the reference's "
                   "connection-thread path), one core"
                   + ("" if cpu else "; cpu legs requested off but always run"))
    return res


def bench_connection_e2e():
    """The FEC path inside the patched reference QuicConnection (VERDICT r2
    next-round 2): client/server pairs of the reference's own QuicConnection
    at QUIC_VERSION_31 (integration/connection_shim.cc, simulated clock, 1 ms
    loop turns, one data packet in about two 10-packet groups dropped), every
    connection on ONE QuicFecBatcher: once per turn one encode + one revive
    launch for all of them, queued asynchronously (QFEC_ASYNC) and completed at
    the next turn.  Per connection count: the connection thread's FEC cost per
    group (the batcher's launch + completion time over the groups it encoded
    and revived) against the historical connection-thread path — every
    protected packet XORed into its group's accumulator at send time
    (XorBuffers), timed on the same packets on one core (the receive side
    folded every packet again; not counted)."""
    spec_path = os.path.join(ROOT, "integration", "conn_harness.py")
    import importlib.util
    spec = importlib.util.spec_from_file_location("conn_harness", spec_path)
    h = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(h)
    if not os.path.exists(h.LIB):
        return {"error": f"{h.LIB} not built (built where /root/reference is)"}
    res = {"workload": "reference QuicConnection pairs, v31, groups of 10, ~1 loss per 2 "
                       "groups, NULL encryption, simulated 1 ms turns", "runs": []}
    # one untimed run first, at the largest connection count: the process's
    # first launches and the growth of this thread's pinned payload arena
    # (32-MiB hipHostMalloc slabs, reused once drained) are not per-group costs
    h.run(n_pairs=4096, group_size=10, drop_every=2, stream_len=20_000, batched=True,
          require_gpu=True)
    def host_per_group(r):
        return (r["fec_host_us"] - r["fec_wait_us"]) / max(1, r["groups_encoded"] +
                                                             r["groups_revived"])

    for n, stream in ((1, 400_000), (64, 100_000), (4096, 20_000)):
        # three runs, the median one reported (a run has 4-300 launches: one
        # slow launch moves a single run's per-group figure by tens of percent)
        rs = []
        for _ in range(3):
            t0 = time.perf_counter()
            r = h.run(n_pairs=n, group_size=10, drop_every=2, stream_len=stream, batched=True,
                      require_gpu=True)
            rs.append((host_per_group(r), time.perf_counter() - t0, r))
        rs.sort(key=lambda x: x[0])
        _, wall, r = rs[1]
        spread = [round(x[0], 3) for x in rs]
        groups = r["groups_encoded"] + r["groups_revived"]
        enc = max(1, r["groups_encoded"])
        res["runs"].append({
            "connections": n, "stream_bytes": stream, "streams_ok": r["streams_ok"],
            "connected": r["connected"], "turns": r["turns"], "launches": r["launches"],
            "groups_encoded": r["groups_encoded"], "groups_revived": r["groups_revived"],
            "dropped": r["dropped"], "retransmitted": r["retransmitted"],
            "groups_per_launch": round(groups / max(1, r["launches"]), 1),
            # connection-thread work per group: the launch (index tables +
            # queueing) and the completion, without the time blocked waiting
            # for the device (a polling loop does other work then)
            "gpu_host_us_per_group": round((r["fec_host_us"] - r["fec_wait_us"]) / max(1, groups), 3),
            "gpu_host_us_per_group_3runs": spread,
            "gpu_wait_us_per_launch": round(r["fec_wait_us"] / max(1, r["launches"]), 2),
            "launch_us_per_launch": round(r["fec_launch_us"] / max(1, r["launches"]), 2),
            # of the launch: CSR tables / C-ABI calls per group; the slowest launch
            "tables_us_per_group": round(r["fec_tables_us"] / max(1, groups), 3),
            "capi_us_per_group": round(r["fec_call_us"] / max(1, groups), 3),
            "launch_us_max": round(r["fec_launch_us_max"], 1),
            "arena_slabs_allocated": r["slabs_allocated"],
            "payloads_copied": r["payloads_copied"], "payloads_adopted": r["payloads_adopted"],
            "cpu_1core_us_per_group": round(r["cpu_xor_us"] / enc, 3),
            "callbacks_incl_us_per_group": round(r["fec_wall_us"] / max(1, groups), 3),
            "run_s": round(wall, 2), "status": r["status"], "detail": r["detail"]})
    return res


def bench_fused(ctx0, torch, dev, stream, k, L, G=1 << 18, hdr=22, cg=16384, slots=3, cpu=True):
    """Host memory in, host memory out, FEC + packet protection on the device
    with ONE PCIe crossing each way:
    per chunk of cg groups, H2D of the plaintext payloads + headers, FEC encode
    (qfec_encode_batch) into the slot, AES-128-GCM-12 seal of every data packet
    AND every FEC packet (qfec_aes128gcm_seal_batch), D2H of the ciphertexts;
    chunks rotate over `slots` streams so copies overlap compute.  Rate =
    plaintext payload bytes / wall time (pinned host buffers)."""
    from libquic_amd import qfec
    assert G % cg == 0
    nchunk = G // cg
    npk = cg * (k + 1)                      # packets per chunk: data, then FEC
    rows_b, par_b, hdr_b = cg * k * L, cg * L, npk * hdr
    host_rows = torch.empty(G * k * L, dtype=torch.uint8).pin_memory()
    d = torch.empty(G * k * L, dtype=torch.uint8, device=dev)
    ctx0.synth_fixed(d, k, L, 0, G, SEED_FIXED)
    ctx0.sync()
    host_rows.copy_(d)
    del d
    torch.cuda.empty_cache()
    ar = torch.arange(G * (k + 1), dtype=torch.int64)
    host_hdr = ((ar.view(-1, 1) * 131 + torch.arange(hdr)) & 0xFF).to(torch.uint8).reshape(-1)
    host_hdr = host_hdr.pin_memory()
    host_out = torch.empty(G * (k + 1) * (L + 12), dtype=torch.uint8).pin_memory()
    # per-chunk packet tables (identical for every chunk), device-resident
    q = torch.arange(npk, dtype=torch.int64, device=dev)
    in_off = torch.where(q < cg * k, q * L, rows_b + (q - cg * k) * L)
    ad_off = rows_b + par_b + q * hdr
    ad_len = torch.full((npk,), hdr, dtype=torch.int16, device=dev)
    in_len = torch.full((npk,), L, dtype=torch.int16, device=dev)
    out_off = q * (L + 12)
    kidx = torch.zeros(npk, dtype=torch.int32, device=dev)
    grp = torch.where(q < cg * k, q // k, q - cg * k)
    idx = torch.where(q < cg * k, q % k, torch.full_like(q, k))
    key = torch.arange(16, dtype=torch.uint8, device=dev) * 11 + 3
    pre = torch.tensor([0xA0, 0xA1, 0xA2, 0xA3], dtype=torch.uint8, device=dev)
    pn = [((c * cg + grp) * (k + 1) + idx + 1) for c in range(nchunk)]  # per chunk
    # streams (and a context on each): slot i's stream in the slot schedule;
    # the duplex schedule's H2D / compute / D2H streams are streams 0 / 1 / 2
    # -- no more streams than the process's hardware queues (4 with the default
    # stream): a stream that shares a queue with another runs behind its work
    nst = max(3, slots)
    streams = [torch.cuda.Stream(device=dev) for _ in range(nst)]
    ctxs = []
    for st in streams:
        c = qfec.Context(dev.index)
        c.set_stream(st)
        ctxs.append(c)
    S = []
    for s in range(slots):
        S.append({"stream": streams[s], "ctx": ctxs[s],
                  "buf": torch.empty(rows_b + par_b + hdr_b, dtype=torch.uint8, device=dev),
                  "out": torch.empty(npk * (L + 12), dtype=torch.uint8, device=dev)})

    def chunk(c, direct_out=False):
        s = S[c % slots]
        buf, out = s["buf"], s["out"]
        ob = npk * (L + 12)
        with torch.cuda.stream(s["stream"]):
            buf[:rows_b].copy_(host_rows[c * rows_b:(c + 1) * rows_b], non_blocking=True)
            buf[rows_b + par_b:].copy_(host_hdr[c * hdr_b:(c + 1) * hdr_b], non_blocking=True)
            s["ctx"].encode(buf[:rows_b], k, L, cg, buf[rows_b:rows_b + par_b])
            if direct_out:
                # the seal kernel writes the ciphertexts straight into pinned host
                # memory (device-mapped): no D2H copy, the link's two directions
                # carried by the copy engine (in) and the kernel's stores (out)
                s["ctx"].aes128gcm_seal(key, pre, kidx, pn[c], None, buf, ad_off, ad_len, in_off,
                                        in_len, npk, host_out[c * ob:(c + 1) * ob], out_off)
            else:
                s["ctx"].aes128gcm_seal(key, pre, kidx, pn[c], None, buf, ad_off, ad_len, in_off,
                                        in_len, npk, out, out_off)
                host_out[c * ob:(c + 1) * ob].copy_(out, non_blocking=True)

    # Duplex form (round 4): ONE stream per copy
    # direction and one compute stream, ordered by events.  The link carries
    # H2D and D2H at once only when each direction's copies sit in a queue of
    # their own (tools/tune/pcie_duplex.hip: one copy each way on two streams
    # 97 GB/s combined; the same bytes as 64-MiB chunks over 8 streams 64 GB/s,
    # as the slot form's 3 streams that each copy in, compute and copy out).
    h2d_st, cmp_st, d2h_st = streams[0], streams[1], streams[2]
    cctx = ctxs[1]
    ev = {n: [torch.cuda.Event() for _ in range(slots)]
          for n in ("in", "done", "buf_free", "out_free")}

    seq = [0]  # chunks issued so far (slot = seq % slots; the first `slots` wait for nothing)

    def chunk_duplex(c):
        i = seq[0] % slots
        first = seq[0] < slots
        seq[0] += 1
        buf, out = S[i]["buf"], S[i]["out"]
        ob = npk * (L + 12)
        with torch.cuda.stream(h2d_st):
            if not first:
                h2d_st.wait_event(ev["buf_free"][i])  # compute of chunk c - slots read buf
            buf[:rows_b].copy_(host_rows[c * rows_b:(c + 1) * rows_b], non_blocking=True)
            buf[rows_b + par_b:].copy_(host_hdr[c * hdr_b:(c + 1) * hdr_b], non_blocking=True)
            ev["in"][i].record(h2d_st)
        with torch.cuda.stream(cmp_st):
            cmp_st.wait_event(ev["in"][i])
            if not first:
                cmp_st.wait_event(ev["out_free"][i])  # D2H of chunk c - slots read out
            cctx.encode(buf[:rows_b], k, L, cg, buf[rows_b:rows_b + par_b])
            cctx.aes128gcm_seal(key, pre, kidx, pn[c], None, buf, ad_off, ad_len, in_off, in_len,
                                npk, out, out_off)
            ev["buf_free"][i].record(cmp_st)
            ev["done"][i].record(cmp_st)
        with torch.cuda.stream(d2h_st):
            d2h_st.wait_event(ev["done"][i])
            host_out[c * ob:(c + 1) * ob].copy_(out, non_blocking=True)
            ev["out_free"][i].record(d2h_st)

    # Two-stream duplex form: copies in AND the kernels on one stream, copies
    # out on the other -- a compute stream of its own can land on a hardware
    # queue shared with a copy stream in a process that has created many
    # streams (the full bench: 53 GB/s there against 92 in a fresh process),
    # and the kernels (~0.2 ms per chunk) cost the inbound queue little.
    in_st, out_st = streams[0], streams[2]
    cctx0 = ctxs[0]

    def chunk_duplex2(c):
        i = seq[0] % slots
        first = seq[0] < slots
        seq[0] += 1
        buf, out = S[i]["buf"], S[i]["out"]
        ob = npk * (L + 12)
        with torch.cuda.stream(in_st):
            buf[:rows_b].copy_(host_rows[c * rows_b:(c + 1) * rows_b], non_blocking=True)
            buf[rows_b + par_b:].copy_(host_hdr[c * hdr_b:(c + 1) * hdr_b], non_blocking=True)
            if not first:
                in_st.wait_event(ev["out_free"][i])  # D2H of chunk c - slots read out
            cctx0.encode(buf[:rows_b], k, L, cg, buf[rows_b:rows_b + par_b])
            cctx0.aes128gcm_seal(key, pre, kidx, pn[c], None, buf, ad_off, ad_len, in_off, in_len,
                                 npk, out, out_off)
            ev["done"][i].record(in_st)
        with torch.cuda.stream(out_st):
            out_st.wait_event(ev["done"][i])
            host_out[c * ob:(c + 1) * ob].copy_(out, non_blocking=True)
            ev["out_free"][i].record(out_st)

    def timed_duplex(chunk_fn=None):
        chunk_duplex_ = chunk_fn or chunk_duplex
        seq[0] = 0
        for c in range(min(slots, nchunk)):  # warm
            chunk_duplex_(c)
        torch.cuda.synchronize()
        host_out.fill_(0)
        reps = 2
        t0 = time.perf_counter()
        for _ in range(reps):
            for c in range(nchunk):
                chunk_duplex_(c)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps

    def verify_chunks():
        """chunk 0 and the last chunk: open on the device, plaintext == rows,
        FEC plaintext == XOR of the group's rows"""
        ok = True
        vs = S[0]
        torch.cuda.synchronize()
        for c in (0, nchunk - 1):
            # torch's copies and the context's launches on the SAME stream (the
            # open kernel must not read `cat` before the copies have filled it)
            with torch.cuda.stream(vs["stream"]):
                ob = npk * (L + 12)
                ct = host_out[c * ob:(c + 1) * ob].to(dev)
                vb = vs["buf"]
                vb[rows_b + par_b:].copy_(host_hdr[c * hdr_b:(c + 1) * hdr_b])
                cat = torch.empty(hdr_b + ob, dtype=torch.uint8, device=dev)
                cat[:hdr_b] = vb[rows_b + par_b:]
                cat[hdr_b:] = ct
                pt = torch.empty(npk * L, dtype=torch.uint8, device=dev)
                okv = torch.zeros(npk, dtype=torch.uint8, device=dev)
                vs["ctx"].aes128gcm_open(key, pre, kidx, pn[c], None, cat, q * hdr, ad_len,
                                         hdr_b + q * (L + 12), (in_len + 12).to(torch.int16), npk, pt,
                                         q * L, okv)
                vs["ctx"].sync()
                rows_c = host_rows[c * rows_b:(c + 1) * rows_b].to(dev)
                par_c = rows_c.view(cg, k, L)[:, 0].clone()
                for i in range(1, k):
                    par_c ^= rows_c.view(cg, k, L)[:, i]
                ok = ok and bool(okv.all()) and torch.equal(pt[:rows_b], rows_c) and \
                    torch.equal(pt[rows_b:], par_c.reshape(-1))
        torch.cuda.synchronize()
        return ok

    def timed(direct_out):
        for c in range(min(slots, nchunk)):  # warm (contexts, kernels)
            chunk(c, direct_out)
        torch.cuda.synchronize()
        host_out.fill_(0)
        reps = 2
        t0 = time.perf_counter()
        for _ in range(reps):
            for c in range(nchunk):
                chunk(c, direct_out)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps

    # the link's both-ways ceiling, measured here: 1 GiB each way at once, one
    # stream per direction (tools/tune/pcie_duplex.hip: 94-97 GB/s with SDMA)
    nb = 1 << 30
    din = torch.empty(nb, dtype=torch.uint8, device=dev)
    dout = torch.empty(nb, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    duplex_ceiling = 0.0
    for _ in range(3):
        t0 = time.perf_counter()
        with torch.cuda.stream(streams[0]):
            din.copy_(host_rows[:nb], non_blocking=True)
        with torch.cuda.stream(streams[2]):
            host_out[:nb].copy_(dout, non_blocking=True)
        torch.cuda.synchronize()
        duplex_ceiling = max(duplex_ceiling, 2 * nb / (time.perf_counter() - t0) / 1e9)
    del din, dout
    torch.cuda.empty_cache()
    wall_direct = timed(True)
    ok_direct = verify_chunks()
    wall_slots = timed(False)
    ok_slots = verify_chunks()
    wall_duplex3 = timed_duplex(chunk_duplex)
    ok_duplex3 = verify_chunks()
    wall_duplex2 = timed_duplex(chunk_duplex2)
    ok_duplex2 = verify_chunks()
    two = wall_duplex2 <= wall_duplex3
    wall_duplex, ok_duplex = (wall_duplex2, ok_duplex2) if two else (wall_duplex3, ok_duplex3)
    for c in ctxs:
        c.close()
    # the leg's figure: the better of the two copy schedules
    duplex_best = wall_duplex <= wall_slots
    wall, ok = (wall_duplex, ok_duplex) if duplex_best else (wall_slots, ok_slots)
    payload = G * k * L
    res = {"groups": G, "chunk_groups": cg, "slots": slots, "header": hdr,
           "payload_GiBps": round(payload / wall / 2**30, 2),
           "wall_ms": round(wall * 1e3, 2),
           "pcie_h2d_bytes": G * k * L + G * (k + 1) * hdr,
           "pcie_d2h_bytes": G * (k + 1) * (L + 12),
           "verified": bool(ok),
           "schedule": "duplex" if duplex_best else "slots",
           "pcie_duplex_ceiling_GBps": round(duplex_ceiling, 1),
           "link_frac_of_duplex_ceiling": round((G * k * L + G * (k + 1) * hdr +
                                                 G * (k + 1) * (L + 12)) / wall / 1e9 /
                                                duplex_ceiling, 3),
           "duplex": {"payload_GiBps": round(payload / wall_duplex / 2**30, 2),
                      "wall_ms": round(wall_duplex * 1e3, 2), "verified": bool(ok_duplex),
                      "streams": 2 if two else 3,
                      "two_stream_GiBps": round(payload / wall_duplex2 / 2**30, 2),
                      "three_stream_GiBps": round(payload / wall_duplex3 / 2**30, 2),
                      "verified_both": bool(ok_duplex2 and ok_duplex3),
                      "link_GBps_combined": round((G * k * L + G * (k + 1) * hdr +
                                                   G * (k + 1) * (L + 12)) / wall_duplex / 1e9, 1),
                      "note": "each copy direction on a stream of its own (2 streams: the "
                              "kernels on the inbound one; 3: a compute stream between), "
                              "events between them"},
           "slots": {"payload_GiBps": round(payload / wall_slots / 2**30, 2),
                     "wall_ms": round(wall_slots * 1e3, 2), "verified": bool(ok_slots),
                     "note": "3 streams, each: H2D, encode + seal, D2H"},
           "direct_out": {"payload_GiBps": round(payload / wall_direct / 2**30, 2),
                          "wall_ms": round(wall_direct * 1e3, 2), "verified": bool(ok_direct),
                          "note": "the seal kernel stores the ciphertexts into pinned host "
                                  "memory itself (no D2H copy)"},
           "note": "pinned host plaintext -> H2D -> FEC encode + AES-128-GCM-12 seal of data and "
                   "FEC packets -> D2H ciphertext; one PCIe crossing each way"}
    del host_rows, host_out, host_hdr, S
    torch.cuda.empty_cache()
    if cpu:
        res["cpu_baseline"] = _cpu_fused_baseline(k, L, hdr)
    return res


def _cpu_fused_baseline(k, L, hdr, n=4096, seconds=4.0):
    """The same work on the host cores: FEC encode (oracle, word-wise XOR) +
    AES-128-GCM-12 seal of every data and FEC packet (the reference's own
    BoringSSL aes.c + gcm.c from oracle/_ref when present, else the port)."""
    from oracle import oracle_c as OC
    from oracle import ref_quic
    threads = _cpu_share()
    npk = n * (k + 1)
    rows_b, par_b = n * k * L, n * L
    buf = np.zeros(rows_b + par_b + npk * hdr, np.uint8)
    buf[:rows_b] = OC.synth_fixed(SEED_FIXED, 0, n, k, L)
    q = np.arange(npk, dtype=np.uint64)
    in_off = np.where(q < n * k, q * np.uint64(L), np.uint64(rows_b) + (q - np.uint64(n * k)) * np.uint64(L)).astype(np.uint64)
    ad_off = np.uint64(rows_b + par_b) + q * np.uint64(hdr)
    ad_len = np.full(npk, hdr, np.uint16)
    in_len = np.full(npk, L, np.uint16)
    out_off = q * np.uint64(L + 12)
    keys = np.arange(16, dtype=np.uint8)
    pre = np.arange(4, dtype=np.uint8)
    kidx = np.zeros(npk, np.uint32)
    pn = q + np.uint64(1)
    obuf = np.zeros(npk * (L + 12), np.uint8)
    kind, what = "port", "oracle FEC + scalar C AES-GCM restatement"
    seal = OC.quic_aes128gcm_encrypt_batch
    if ref_quic.asm_available():
        kind = "reference"
        what = ("oracle FEC + the reference's Aes128Gcm12Encrypter over BoringSSL with its "
                "x86-64 assembly (AES-NI, PCLMULQDQ)")

        def seal(keys, pre, kidx, pn, path, *rest, threads, out):
            return ref_quic.asm_seal_batch("aes128gcm", keys, pre, kidx, pn, *rest,
                                           threads=threads, out=out)
    lib = OC.lib()

    def once():
        assert lib.qo_encode_fixed_mt(OC._p(buf), k, L, n, OC._p(buf[rows_b:]), threads) == 0
        seal(keys, pre, kidx, pn, None, buf, ad_off, ad_len, in_off, in_len, out_off,
             npk * (L + 12), threads=threads, out=obuf)
    once()
    t0, reps = time.perf_counter(), 0
    while time.perf_counter() - t0 < seconds:
        once()
        reps += 1
    el = time.perf_counter() - t0
    return {"value": round(reps * n * k * L / el / 2**30, 3), "unit": "GiB/s of payload",
            "cores": threads, "kind": kind,
            "sample": f"{n} groups x {k} x {L} B: FEC encode + seal of {npk} packets, {reps} "
                      f"passes on {threads} threads ({what})"}


def bench_e2e(ctx, torch, k, L, G=1 << 18):
    """Host-resident path: pinned host rows -> H2D -> kernel -> D2H (QFEC_PTR_HOST)."""
    rows = torch.empty(G * k * L, dtype=torch.uint8).pin_memory()
    # fill from the device generator (plumbing) to avoid a slow host fill
    d = torch.empty(G * k * L, dtype=torch.uint8, device="cuda")
    ctx.synth_fixed(d, k, L, 0, G, SEED_FIXED)
    ctx.sync()
    rows.copy_(d)
    del d
    par = torch.empty(G * L, dtype=torch.uint8).pin_memory()
    out = torch.empty(G * L, dtype=torch.uint8).pin_memory()
    miss = drop_indices(0, G, k)
    ctx.encode(rows, k, L, G, par, host=True)  # warm (allocates staging)
    reps = 3
    t0 = time.perf_counter()
    for _ in range(reps):
        ctx.encode(rows, k, L, G, par, host=True)
    t_enc = (time.perf_counter() - t0) / reps
    t0 = time.perf_counter()
    for _ in range(reps):
        ctx.recover(rows, par, miss, k, L, G, out, host=True)
    t_rec = (time.perf_counter() - t0) / reps
    r3 = rows.numpy().reshape(G, k, L)
    ok = np.array_equal(out.numpy().reshape(G, L)[:4096], r3[np.arange(4096), miss[:4096]])
    # zero-copy (QFEC_PTR_MAPPED): the kernels read the pinned rows / parity and
    # write their outputs in host memory in place, no staging
    par.fill_(0)
    out.fill_(0)
    ctx.encode(rows, k, L, G, par, mapped=True)  # warm
    t0 = time.perf_counter()
    for _ in range(reps):
        ctx.encode(rows, k, L, G, par, mapped=True)
    t_enc_m = (time.perf_counter() - t0) / reps
    t0 = time.perf_counter()
    for _ in range(reps):
        ctx.recover(rows, par, miss, k, L, G, out, mapped=True)
    t_rec_m = (time.perf_counter() - t0) / reps
    ok_m = np.array_equal(out.numpy().reshape(G, L)[-4096:], r3[np.arange(G - 4096, G),
                                                                 miss[-4096:]])
    b = G * (k * L + L)
    return {"groups": G, "encode_GiBps": round(b / t_enc / 2**30, 2),
            "recover_GiBps": round(b / t_rec / 2**30, 2),
            "pcie_bytes_encode": G * (k * L + L), "verified": bool(ok),
            "zero_copy": {"encode_GiBps": round(b / t_enc_m / 2**30, 2),
                          "recover_GiBps": round(b / t_rec_m / 2**30, 2), "verified": bool(ok_m),
                          "note": "QFEC_PTR_MAPPED: kernels read/write the pinned host buffers "
                                  "in place over PCIe"},
            "note": "algorithmic bytes / wall time, pinned host buffers, 3-slot H2D/kernel/D2H"}


if __name__ == "__main__":
    sys.exit(main())
