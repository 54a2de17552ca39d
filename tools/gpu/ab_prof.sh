# A/B of library variants at the driver's settings (bench.py --steps 20 --warmup 5), on one box:
# per variant and repeat, one rocprofv3 --kernel-trace --stats run (per-kernel averages) and one
# plain bench.py run (the driver's clock).  Variants run interleaved, so box drift hits all alike.
#   gpurun --timeout 1200 -- 'bash tools/gpu/ab_prof.sh <tag> <repeats> "name:ENV=v,ENV2=v" ...'
# a variant's ENV list may name BPRMF_DIAG_LIB=<path> (a diagnostic build of the library).
set -o pipefail
tag="$1"; reps="$2"; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
out="$R/gpurun_out/$tag"
mkdir -p "$out"
export TMPDIR=/tmp
for r in $(seq 1 "$reps"); do
  for spec in "$@"; do
    name="${spec%%:*}"; envs="${spec#*:}"
    ( [ "$envs" != "$spec" ] && [ -n "$envs" ] && for kv in ${envs//,/ }; do export "$kv"; done
      case "${BPRMF_DIAG_LIB:-/}" in /*) ;; *) export BPRMF_DIAG_LIB="$R/$BPRMF_DIAG_LIB" ;; esac
      cd /tmp &&
      timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/prof_${name}_$r" -o run \
        --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-relaxed \
        > "$out/prof_${name}_$r.log" 2>&1 &&
      cd "$R" &&
      timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-relaxed \
        > "$out/bench_${name}_$r.log" 2>&1 ) || { echo "variant $name rep $r failed"; tail -n 5 "$out/prof_${name}_$r.log" "$out/bench_${name}_$r.log"; exit 1; }
    st=$(find "$out/prof_${name}_$r" -name '*kernel_stats.csv' | head -n 1)
    echo "$name $r $(python3 tools/kstats.py --only k_fused_step,k_user_step,k_build_split,k_owner_diag "$st" | cut -d: -f2-) | bench $(grep '^{' "$out/bench_${name}_$r.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e8,4), "e8", d["ms_per_step"]*1e3, "us/step", d["roofline"]["avg_us_per_step"])')" | tee -a "$out/summary.txt"
  done
done
