# World-1 step time of the sharded runner's forms, unprofiled, interleaved repeats (bench.py
# --sharded --steps 1000 --warmup 100): the exact runner (graphs), the exact IPC two-launch form,
# stale1 over IPC (the device-flag form) and stale1 over rccl (two streams).
#   gpurun --timeout 900 -- 'bash tools/gpu/stale1_ipc.sh <tag> [repeats]'
set -o pipefail
tag="$1"; reps="${2:-2}"
R=${GRAFT_REPO_ROOT:-$(pwd)}
out="$R/gpurun_out/$tag"
mkdir -p "$out"
args="--sharded --steps 1000 --warmup 100 --no-relaxed --no-profile --no-cpu-baseline"
variants=(
  "exact_runner|BPRMF_DIST_W1_RUNNER=1|"
  "exact_ipc2|BPRMF_DIST_W1_RUNNER=1 BPRMF_DIST_FUSE=1|--transport ipc"
  "stale1_ipc|BPRMF_DIST_FUSE=1|--semantics stale1 --transport ipc"
  "stale1_rccl||--semantics stale1 --transport rccl"
)
for r in $(seq 1 "$reps"); do
  for v in "${variants[@]}"; do
    IFS='|' read -r name envs extra <<< "$v"
    ( for kv in $envs; do export "$kv"; done
      timeout -k 10 200 python3 bench.py $args $extra > "$out/${name}_$r.log" 2>&1 ) ||
      { echo "$name rep $r failed"; tail -n 5 "$out/${name}_$r.log"; exit 1; }
    echo "$name $r $(grep '^{' "$out/${name}_$r.log" | python3 -c '
import json, sys
d = json.loads(sys.stdin.read())
print("%.4ge8 triplets/s %.2f us/step" % (d["value"] / 1e8, d["ms_per_step"] * 1e3))')" | tee -a "$out/summary.txt"
  done
done
