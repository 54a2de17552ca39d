# A/B of the persistent step (BPRMF_PERSIST=1, step.hip k_persist_steps) against the fused launches
# at one batch size (bench.py --steps 20 --warmup 5): rocprofv3 kernel stats + bench line per variant.
#   gpurun -- 'bash tools/gpu/persist_ab.sh <tag> <batch> "name:ENV=v,..." ...'
set -o pipefail
tag="$1"; bs="$2"; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
out="$R/gpurun_out/$tag"
mkdir -p "$out"
export TMPDIR=/tmp
for spec in "$@"; do
  name="${spec%%:*}"; envs="${spec#*:}"
  ( [ "$envs" != "$spec" ] && [ -n "$envs" ] && for kv in ${envs//,/ }; do export "$kv"; done
    case "${BPRMF_DIAG_LIB:-/}" in /*) ;; *) export BPRMF_DIAG_LIB="$R/$BPRMF_DIAG_LIB" ;; esac
    cd /tmp &&
    timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/prof_$name" -o run --output-format csv \
      -- python3 "$R/bench.py" --steps 20 --warmup 5 --batch-size "$bs" --no-cpu-baseline --no-relaxed \
      > "$out/prof_$name.log" 2>&1 ) || { echo "variant $name failed"; tail -n 5 "$out/prof_$name.log"; exit 1; }
  st=$(find "$out/prof_$name" -name '*kernel_stats.csv' | head -n 1)
  echo "$name B=$bs $(python3 tools/kstats.py --only k_fused_step,k_user_step,k_build_split,k_persist_steps "$st" | cut -d: -f2-)" | tee -a "$out/summary.txt"
done
