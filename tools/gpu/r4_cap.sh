set -o pipefail
out="gpurun_out/$1"
mkdir -p "$out"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > "$out/gpu_tests.log" 2>&1 || { tail -20 "$out/gpu_tests.log"; exit 1; }
tail -1 "$out/gpu_tests.log"
timeout -k 10 300 python3 bench.py --no-cpu-baseline --users 6040 --items 3706 --positives 575000 --factor 64 > "$out/ml1m.log" 2>&1 &&
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 > "$out/k20.log" 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1
rc=$?
for f in ml1m k20; do python3 -c "
import json
d=json.loads(open('$out/$f.log').read().strip().splitlines()[-1]); r=d['roofline']
print('$f', d['value'], r['avg_us_per_step'], r['frac'])
"; done
tail -1 "$out/smoke.log"
exit $rc
