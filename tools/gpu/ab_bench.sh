# A/B of library variants by bench.py lines only (exact value, relaxed_local, relaxed_local_hbm),
# variants interleaved per repeat on one box.
#   gpurun --timeout 1200 -- 'bash tools/gpu/ab_bench.sh <tag> <repeats> "name:ENV=v,..." ... [-- bench args]'
# a variant's ENV list may name BPRMF_DIAG_LIB=<path> (another build of the library).
set -o pipefail
tag="$1"; reps="$2"; shift 2
specs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do specs+=("$1"); shift; done
[ "$1" = "--" ] && shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
out="$R/gpurun_out/$tag"
mkdir -p "$out"
for r in $(seq 1 "$reps"); do
  for spec in "${specs[@]}"; do
    name="${spec%%:*}"; envs="${spec#*:}"
    ( [ "$envs" != "$spec" ] && [ -n "$envs" ] && for kv in ${envs//,/ }; do export "$kv"; done
      case "${BPRMF_DIAG_LIB:-/}" in /*) ;; *) export BPRMF_DIAG_LIB="$R/$BPRMF_DIAG_LIB" ;; esac
      timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" \
        > "$out/bench_${name}_$r.log" 2>&1 ) || { echo "variant $name rep $r failed"; tail -n 5 "$out/bench_${name}_$r.log"; exit 1; }
    echo "$name $r $(grep '^{' "$out/bench_${name}_$r.log" | python3 -c '
import json, sys
d = json.loads(sys.stdin.read())
parts = ["exact %.4ge8 %.2f us/step" % (d["value"] / 1e8, d["ms_per_step"] * 1e3)]
if d.get("roofline"):
    parts[0] += " kernels %.3f" % d["roofline"]["avg_us_per_step"]
for k in ("relaxed_local", "relaxed_local_hbm"):
    if k in d:
        parts.append("%s %.4ge9 %.3f us/step frac %.3f" % (k, d[k]["value"] / 1e9, d[k]["ms_per_step"] * 1e3, d[k]["roofline"]["frac"]))
print(" | ".join(parts))')" | tee -a "$out/summary.txt"
  done
done
