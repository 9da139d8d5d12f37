"""Prints the revived-packets channel of the patched reference QuicConnection
runs (integration/conn_harness.py) for the DESIGN.md §10.1 table: per
scenario, drops, revivals, revivals the sender saw in acks, retransmissions
(of revived packets, and after a revival report), protected packets with
entropy bit 1.  GPU box; writes one JSON line per scenario."""
import importlib.util
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location(
    "conn_harness", os.path.join(ROOT, "integration", "conn_harness.py"))
h = importlib.util.module_from_spec(spec)
spec.loader.exec_module(h)

KEYS = ("connected", "streams_ok", "data_packets_sent", "protected_entropy_set",
        "fec_packets_sent", "dropped", "revived", "revived_reported", "acks_with_revived",
        "retransmitted", "retransmitted_of_revived", "retransmitted_after_report", "turns")
for name, kw in [
        ("k10_unbatched", dict(n_pairs=4, group_size=10, drop_every=2, stream_len=300_000,
                               batched=False)),
        ("k10_batched", dict(n_pairs=4, group_size=10, drop_every=2, stream_len=300_000,
                             batched=True)),
        ("k2", dict(n_pairs=2, group_size=2, drop_every=3, stream_len=300_000, batched=True)),
        ("k255", dict(n_pairs=2, group_size=255, drop_every=1, stream_len=300_000,
                      batched=True)),
        ("reorder3", dict(n_pairs=4, group_size=10, drop_every=2, stream_len=300_000,
                          batched=True, reorder=3)),
        ("c64", dict(n_pairs=64, group_size=10, drop_every=2, stream_len=60_000,
                     batched=True))]:
    r = h.run(require_gpu=True, **kw)
    print(json.dumps({"scenario": name, **{k: r[k] for k in KEYS}, "detail": r["detail"]}),
          flush=True)
