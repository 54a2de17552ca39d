# the other shapes on the final tree: C5 (one GPU), B=8192, the ml-1m shape at d=64; exact and local
set -o pipefail
out="gpurun_out/$1"
mkdir -p "$out"
run() {  # name, timeout, args...
  local n="$1" to="$2"; shift 2
  timeout -k 10 "$to" python3 bench.py --no-cpu-baseline "$@" > "$out/$n.log" 2>&1 || { tail -5 "$out/$n.log"; return 1; }
  python3 -c "
import json
d=json.loads(open('$out/$n.log').read().strip().splitlines()[-1]); r=d['roofline']
print('$n', d['value'], r['avg_us_per_step'], r['frac'])
"
}
run c5_exact 900 --users 10000000 --items 100000000 --positives 150000000 --factor 256 --steps 1000 --warmup 100 &&
run b8192_exact 300 --batch-size 8192 &&
run b8192_local 300 --batch-size 8192 --semantics local &&
run ml1m_exact 300 --users 6040 --items 3706 --positives 575000 --factor 64 &&
run ml1m_local 300 --users 6040 --items 3706 --positives 575000 --factor 64 --semantics local
