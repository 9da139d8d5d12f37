"""CPU multi-rank test of bench.py's N>1 path (gloo, world_size 2).

The FEC groups are independent, so the multi-GPU design is a contiguous group
shard per rank (g0 = rank * G) with no collective on the data path; the only
collectives are the timing barrier and the max-over-ranks of the elapsed time.
This test runs exactly that skeleton (bench.timed_steps / bench.result_line)
in two gloo processes, with the oracle standing in for the GPU (test
infrastructure), and checks that the shards tile the global group range and
reproduce the single-process result group for group.
"""
import json
import os
import socket
import subprocess
import sys
import textwrap

import numpy as np

from conftest import ROOT

WORKER = textwrap.dedent(r"""
    import json, os, sys
    sys.path.insert(0, os.environ["QFEC_ROOT"])
    import numpy as np
    import torch
    import torch.distributed as dist
    import bench
    from oracle import oracle_c as OC

    class CpuOracleWorkload:
        # same shard assignment and step structure as bench.HipFixedWorkload
        def __init__(self, g0, G, k, L):
            self.g0, self.G, self.k, self.L = g0, G, k, L
            self.rows = OC.synth_fixed(bench.SEED_FIXED, g0, G, k, L)
            self.miss = bench.drop_indices(g0, G, k)
            self.par = np.zeros(G * L, np.uint8)
            self.out = np.zeros(G * L, np.uint8)
            self.bytes_encode = G * (k * L + L)
            self.bytes_recover = G * ((k - 1) * L + 2 * L)
            self.steps = 0
        def new_events(self):
            return None
        def step(self, ev=None):
            lib = OC.lib()
            assert lib.qo_encode_fixed_mt(OC._p(self.rows), self.k, self.L, self.G,
                                          OC._p(self.par), 1) == 0
            assert lib.qo_recover_fixed_mt(OC._p(self.rows), OC._p(self.par), OC._p(self.miss),
                                           self.k, self.L, self.G, OC._p(self.out), 1) == 0
            self.steps += 1
        def synchronize(self):
            pass

    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    G, k, L = int(os.environ["QFEC_G"]), 10, 1350
    work = CpuOracleWorkload(rank * G, G, k, L)

    def barrier():
        dist.barrier()

    def reduce_max(x):
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    local = []
    def reduce_max_record(x):
        local.append(x)
        return reduce_max(x)

    elapsed, _ = bench.timed_steps(work, 3, 1, barrier, reduce_max_record)
    d = torch.tensor([OC.group_digest(work.par, G, L, L), OC.group_digest(work.out, G, L, L)],
                     dtype=torch.float64)  # carried as raw bits below
    digests = [int(OC.group_digest(work.par, G, L, L)), int(OC.group_digest(work.out, G, L, L))]
    gathered = [None] * world
    dist.all_gather_object(gathered, {"rank": rank, "g0": work.g0, "G": G, "digests": digests,
                                      "local_elapsed": local[0], "steps": work.steps})
    if rank == 0:
        line = bench.result_line(world, 3, 1, elapsed, G, k, L, work.bytes_encode,
                                 work.bytes_recover)
        print("RESULT " + json.dumps({"line": line, "ranks": gathered, "elapsed": elapsed}))
    dist.destroy_process_group()
""")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_rank_gloo_shards():
    G = 256
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="2",
                   RANK=str(r), LOCAL_RANK=str(r), QFEC_ROOT=ROOT, QFEC_G=str(G),
                   OMP_NUM_THREADS="1")
        procs.append(subprocess.Popen([sys.executable, "-c", WORKER], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        o, e = p.communicate(timeout=300)
        assert p.returncode == 0, e
        outs.append(o)
    res = json.loads([l for l in outs[0].splitlines() if l.startswith("RESULT ")][0][7:])
    ranks = sorted(res["ranks"], key=lambda r: r["rank"])
    # shards tile [0, 2G) contiguously, every rank ran warmup + K steps
    assert [r["g0"] for r in ranks] == [0, G]
    assert all(r["steps"] == 4 for r in ranks)
    # elapsed is the max over ranks
    assert abs(res["elapsed"] - max(r["local_elapsed"] for r in ranks)) < 1e-9
    # the JSON line aggregates all ranks' bytes over the max time
    line = res["line"]
    assert line["n_gpus"] == 2 and line["scaling"] == "weak"
    want = 2 * 3 * G * 14850 * 2 / 2**30 / res["elapsed"]
    assert abs(line["value"] - round(want, 2)) < 0.02
    # each shard reproduces the single-process computation of its group range
    from oracle import oracle_c as OC
    import bench
    k, L = 10, 1350
    rows = OC.synth_fixed(bench.SEED_FIXED, 0, 2 * G, k, L)
    rc, par = OC.encode_fixed(rows, k, L, 2 * G)
    miss = bench.drop_indices(0, 2 * G, k)
    rc2, out = OC.recover_fixed(rows, par, miss, k, L, 2 * G)
    assert rc == 0 and rc2 == 0
    for r in ranks:
        sl = slice(r["g0"] * L, (r["g0"] + G) * L)
        assert r["digests"][0] == OC.group_digest(np.ascontiguousarray(par[sl]), G, L, L)
        assert r["digests"][1] == OC.group_digest(np.ascontiguousarray(out[sl]), G, L, L)


def test_shard_ranges_disjoint_for_8_ranks():
    # bench assigns g0 = rank * G: 8 ranks x 2^20 groups cover [0, 2^23) exactly
    G = 1 << 20
    starts = [r * G for r in range(8)]
    assert starts == sorted(starts) and starts[-1] + G == 8 * G
    # drop indices of a shard equal the global sequence's slice
    import bench
    a = bench.drop_indices(3 * 1000, 1000, 10)
    b = bench.drop_indices(0, 4000, 10)[3000:]
    assert np.array_equal(a, b)
