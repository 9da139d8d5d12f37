"""Debug: a two-group job behind a split job whose followers are held
(test_no_rotation_while_a_split_job_waits_for_late_followers), polled with
a deadline instead of a blocking wait; prints the service state."""
import sys, os, time
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from libquic_amd import qfec
from test_hip_mapped import _mapped_case

def run(bound, n_small, hold):
    ctx = qfec.Context(0)
    z, want_l = _mapped_case(40, g0=96000, kmin=2, kmax=12, lmin=16, lmax=1350, seed=23)
    z1, want_1 = _mapped_case(n_small, g0=97000, kmin=2, kmax=12, lmin=16, lmax=1350, seed=24)
    data, data1 = qfec.HostBuffer(len(z["data"])), qfec.HostBuffer(len(z1["data"]))
    data.array[:] = z["data"]; data1.array[:] = z1["data"]
    par, par1 = qfec.HostBuffer(z["parity"].size), qfec.HostBuffer(z1["parity"].size)
    ctx.debug_service_resident(bound)
    ctx.debug_service(on=False); ctx.debug_service(on=True)
    ctx.debug_service_hold(hold)
    plen = np.zeros(40, np.uint16)
    ctx.encode_ragged(data.array, z["pkt_off"], z["pkt_len"], z["grp_ptr"], 40, par.array,
                      z["parity_off"], plen, mapped=True, async_=True)
    t = ctx.async_ticket()
    for it in range(3):
        plen1 = np.zeros(n_small, np.uint16)
        par1.array[:] = 0
        ctx.encode_ragged(data1.array, z1["pkt_off"], z1["pkt_len"], z1["grp_ptr"], n_small,
                          par1.array, z1["parity_off"], plen1, mapped=True, async_=True)
        t1 = ctx.async_ticket()
        deadline = time.perf_counter() + 1.0
        rc = 1
        while time.perf_counter() < deadline:
            rc = ctx.lib.qfec_complete_ticket(ctx.ctx, t1, 0)
            if rc != 1:
                break
        print(f"bound {bound} n {n_small} hold {hold} it {it}: small job rc {rc} service {ctx.debug_service()}", flush=True)
        if rc == 1:
            break
    ctx.debug_service_hold(False)
    if rc == 1:
        rc = ctx.complete_ticket(t1)
        print(f"  after release: rc {rc}", flush=True)
    print(f"  small exact {np.array_equal(par1.array, z1['parity'])}", flush=True)
    assert ctx.complete_ticket(t) == 0
    print(f"  split exact {np.array_equal(par.array, z['parity'])}", flush=True)
    ctx.debug_service_resident(2_000_000)
    for b in (data, data1, par, par1):
        b.close()
    ctx.close()

for bound, n, hold in [(2_000_000, 2, True), (0, 2, True), (0, 1, True), (0, 3, True)]:
    run(bound, n, hold)
