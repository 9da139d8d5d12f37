#!/bin/bash
# Round 5: the small-batch service (inline tables) -- its GPU tests, then the
# bench's connection legs alone.
TAG=${1:-svc1}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_hip_service.py tests/test_hip_mapped.py tests/test_connection.py tests/test_connection_e2e.py tests/test_hip_ragged.py -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -n 40 "$OUT/pytest.log"; exit 1; }
tail -n 2 "$OUT/pytest.log"
timeout -k 10 240 python -u tools/svc_stamps.py > "$OUT/stamps.txt" 2>&1 || { tail -n 30 "$OUT/stamps.txt"; exit 1; }
cat "$OUT/stamps.txt"
timeout -k 10 600 python -u bench.py --groups 65536 --steps 2 --warmup 1 --no-ragged --no-protect --no-entropy --no-fused --no-e2e --no-ceilings --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -n 30 "$OUT/bench.err"; exit 1; }
python3 -c "
import json; l=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
for g in l['connection']['legs']: print(g['groups'], g['encode_flush_us'], g['revive_flush_us'], g['cpu_1core_encode_us'])
for r in l['connection_e2e']['runs']: print(r['connections'], r['gpu_host_us_per_group'], r['gpu_wait_us_per_launch'], r['capi_us_per_group'])
"
