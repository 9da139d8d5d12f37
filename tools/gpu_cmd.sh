mkdir -p gpurun_out/pal
timeout -k 10 400 python -u bench.py --protect-only > gpurun_out/pal/bench_protect.json 2> gpurun_out/pal/bench_protect.err; rc=$?; python - <<'PY'
import json
d=json.loads(open('gpurun_out/pal/bench_protect.json').read().strip().splitlines()[-1])
p=d.get('protect', d)
print({k:v for k,v in p.items() if k.startswith('encrypt')})
PY
exit $rc
