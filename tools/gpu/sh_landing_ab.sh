# A/B at world 1 (--sharded): the plain runner path against the fused IPC forms over landing
# memory allocated uncached (default), fine-grained or plain.  gpurun -- bash tools/gpu/sh_landing_ab.sh
set -o pipefail
mkdir -p gpurun_out/sh4
n=0
for v in "X=0" "BPRMF_DIST_FUSE=1" "BPRMF_DIST_FUSE=1 BPRMF_DIST_LANDING=fine" "BPRMF_DIST_FUSE=1 BPRMF_DIST_LANDING=plain"; do
  n=$((n+1))
  env $v timeout -k 10 200 python bench.py --sharded --steps 2000 --warmup 100 --no-cpu-baseline > gpurun_out/sh4/w1_$n.log 2>&1 || { tail -5 gpurun_out/sh4/w1_$n.log; exit 1; }
  echo "[$v] $(grep '^{' gpurun_out/sh4/w1_$n.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_us_per_step"])')"
done
