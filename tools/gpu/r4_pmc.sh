# Round 4 PMC traffic (separate FETCH_SIZE / WRITE_SIZE passes, MI355X_MICROARCH.md HBM section):
# the exact fused step and the local mode's kernels, ml-20m shape; -> gpurun_out/<tag>/pmc_traffic.json
#   gpurun --timeout 900 -- 'bash tools/gpu/r4_pmc.sh <tag>'
set -o pipefail
tag="$1"
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p $O
cp $R/profiles/pmc_traffic.json $O/pmc_traffic.json
cd /tmp && export TMPDIR=/tmp
for mode in exact local; do
  extra=""
  [ $mode = local ] && extra="--semantics local --steps 192 --warmup 16"
  [ $mode = exact ] && extra="--steps 200 --warmup 20"
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $c -d $O/$mode/$c -o run --output-format csv -- python3 $R/bench.py $extra --no-cpu-baseline --no-profile > $O/$mode.$c.out 2>&1 || { tail -5 $O/$mode.$c.out; exit 1; }
  done
done
cd $R
python3 tools/pmc_traffic.py ml20m_d128_B4096 $O/exact/FETCH_SIZE $O/exact/WRITE_SIZE --out $O/pmc_traffic.json &&
python3 tools/pmc_traffic.py ml20m_d128_B4096_local $O/local/FETCH_SIZE $O/local/WRITE_SIZE --steps-per-launch 16 --out $O/pmc_traffic.json
