#!/bin/bash
# A/B of two libqfec.so builds (tools/ab/old.so, tools/ab/new.so) on the
# bench's connection legs, alternating old/new twice in one box session.
# Usage: tools/ab_svc.sh <tag>
TAG=${1:-ab}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cp libquic_amd/libqfec.so "$OUT/orig.so"
for round in 1 2; do
  for v in old new; do
    cp tools/ab/$v.so libquic_amd/libqfec.so
    timeout -k 10 300 python -u bench.py --groups 65536 --steps 2 --warmup 1 --no-ragged --no-protect --no-entropy --no-fused --no-e2e --no-ceilings --no-cpu-baseline > "$OUT/bench_${v}_$round.json" 2> "$OUT/bench_${v}_$round.err" || { cp "$OUT/orig.so" libquic_amd/libqfec.so; tail -n 20 "$OUT/bench_${v}_$round.err"; exit 1; }
    python3 -c "
import json; l=json.loads(open('$OUT/bench_${v}_$round.json').read().strip().splitlines()[-1])
print('$v', $round, [(g['groups'], g['encode_flush_us'], g['revive_flush_us']) for g in l['connection']['legs']][:2], [(r['connections'], r['gpu_host_us_per_group'], r['gpu_wait_us_per_launch']) for r in l['connection_e2e']['runs']][:2])
"
  done
done
cp "$OUT/orig.so" libquic_amd/libqfec.so
