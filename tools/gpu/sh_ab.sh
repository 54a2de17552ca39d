# A/B of sharded-path switches at world 1 (--sharded), driver settings, 3 runs each
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash tools/gpu/sh_ab.sh "ENV=.." "ENV=.."'
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3; do
  for v in "$@"; do
    env $v timeout -k 10 200 python bench.py --sharded --steps 20 --warmup 5 --no-cpu-baseline --no-profile > gpurun_out/sh_ab.log 2>&1 || { tail -5 gpurun_out/sh_ab.log; exit 1; }
    echo "[$v] $(grep '^{' gpurun_out/sh_ab.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
