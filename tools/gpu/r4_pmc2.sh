# PMC traffic of the local mode's current kernels (128-step periods: every launch 128 steps),
# separate FETCH_SIZE / WRITE_SIZE passes -> gpurun_out/<tag>/pmc_traffic.json
set -o pipefail
tag="$1"
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p $O
cp $R/profiles/pmc_traffic.json $O/pmc_traffic.json
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c -d $O/local/$c -o run --output-format csv -- python3 $R/bench.py --semantics local --steps 256 --warmup 128 --no-cpu-baseline --no-profile > $O/local.$c.out 2>&1 || { tail -5 $O/local.$c.out; exit 1; }
done
cd $R
python3 tools/pmc_traffic.py ml20m_d128_B4096_local $O/local/FETCH_SIZE $O/local/WRITE_SIZE --steps-per-launch 128 --out $O/pmc_traffic.json
