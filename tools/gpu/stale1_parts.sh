# Per-rank components of the sharded runner at world 1 (no link time), for the 8-GPU projection
# of DESIGN.md §6c: rocprofv3 --stats of bench.py --sharded for the exact runner (forced at world
# 1: BPRMF_DIST_W1_RUNNER=1) and the stale1 runner, at the C3 shape (ml-20m, d = 128) and at the
# C5 per-rank shape (1/8 of C5's users, all 100M items, d = 256).
#   gpurun --timeout 1200 -- 'bash tools/gpu/stale1_parts.sh <tag> [c3|c5|c3,c5]'
set -o pipefail
tag="$1"; which="${2:-c3,c5}"
R=${GRAFT_REPO_ROOT:-$(pwd)}
out="$R/gpurun_out/$tag"
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
C5="--users 1250000 --items 100000000 --positives 18750000 --factor 256"
run() {  # name, env, args...
  local n="$1" env="$2"; shift 2
  ( [ -n "$env" ] && export $env
    timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$out/prof_$n" -o run --output-format csv \
      -- python3 "$R/bench.py" --sharded --no-cpu-baseline --no-relaxed "$@" > "$out/$n.log" 2>&1 ) ||
    { tail -n 8 "$out/$n.log"; return 1; }
  grep -h '^{' "$out/$n.log" | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']
print('$n', d['value'], d['ms_per_step'], r['avg_us_per_step'])" | tee -a "$out/parts.txt"
  python3 "$R/tools/kstats.py" $(find "$out/prof_$n" -name '*kernel_stats.csv' | head -n 1) | tee -a "$out/parts.txt"
}
ok=0
if [[ ",$which," == *",c3,"* ]]; then
  run c3_exact BPRMF_DIST_W1_RUNNER=1 --steps 1000 --warmup 100 &&
  run c3_stale1 "" --semantics stale1 --steps 1000 --warmup 100 || ok=1
fi
if [ $ok -eq 0 ] && [[ ",$which," == *",c5,"* ]]; then
  run c5_exact BPRMF_DIST_W1_RUNNER=1 $C5 --steps 600 --warmup 60 &&
  run c5_stale1 "" --semantics stale1 $C5 --steps 600 --warmup 60 || ok=1
fi
exit $ok
