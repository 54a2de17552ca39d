# bench.py lines at the other shapes: C5 on one GPU (10M x 100M, d = 256), B = 8192, the ml-1m
# shape at d = 64; exact and local.   gpurun --timeout 1200 -- 'bash tools/gpu/shapes.sh <tag> [names]'
set -o pipefail
out="gpurun_out/$1"
only="${2:-c5_exact,c5_local,b8192_exact,b8192_local,ml1m_exact,ml1m_local}"
mkdir -p "$out"
C5="--users 10000000 --items 100000000 --positives 150000000 --factor 256"
ML1M="--users 6040 --items 3706 --positives 575000 --factor 64"
run() {  # name, timeout, args...
  local n="$1" to="$2"; shift 2
  [[ ",$only," == *",$n,"* ]] || return 0
  timeout -k 10 "$to" python3 bench.py --no-cpu-baseline --no-relaxed "$@" > "$out/$n.log" 2>&1 || { tail -n 5 "$out/$n.log"; return 1; }
  python3 -c "
import json
d=json.loads(open('$out/$n.log').read().strip().splitlines()[-1]); r=d['roofline']
print('$n', d['value'], r['avg_us_per_step'], r['frac'])
" | tee -a "$out/shapes.txt"
}
run c5_exact 900 $C5 --steps 1000 --warmup 100 &&
run c5_local 900 $C5 --semantics local --steps 1024 --warmup 256 &&
run b8192_exact 300 --batch-size 8192 &&
run b8192_local 300 --batch-size 8192 --semantics local &&
run ml1m_exact 300 $ML1M &&
run ml1m_local 300 $ML1M --semantics local
