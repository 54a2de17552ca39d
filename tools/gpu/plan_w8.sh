# k_owner_plan at world 8 (in-process loopback shards on the one GPU, ml-20m per-rank shape) under
# rocprofv3, the lane-parallel plan and the sequential one (BPRMF_PLAN_LANES=0); sharded tests first.
#   gpurun --timeout 900 -- 'bash tools/gpu/plan_w8.sh <tag>'
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
tag="$1"
out="$R/gpurun_out/$tag"
mkdir -p "$out"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_ipc.py -m gpu -x -q --timeout 200 --timeout-method thread > "$out/sh_tests.log" 2>&1
rc=$?
tail -2 "$out/sh_tests.log"
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
  BPRMF_PLAN_LANES=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/p$v" -o run --output-format csv -- python3 "$R/tools/ubench_plan_w8.py" 8 20 3 > "$out/p$v.log" 2>&1 || { tail -20 "$out/p$v.log"; exit 1; }
  f=$(find "$out/p$v" -name '*kernel_stats.csv' | head -1)
  echo "BPRMF_PLAN_LANES=$v"; grep -E "owner_plan|pack_ids|build_split|own_max|pair_out" "$f" | cut -d, -f1-4 | sed 's/(.*)"//'
done
