#!/bin/bash
# GPU box: SQ counter passes (wave cycles split into issuing / parked / issue-stalled, and the
# instruction mix) over a short K=20 bench.py run; CSVs under gpurun_out/pmc_sq/<tag>/.
#   /usr/local/graft/bin/gpurun --timeout 600 -- 'bash tools/gpu/pmc_sq.sh <tag> [--ncf] [bench args]'
# (--ncf: over tools/bench_ncf.py, 100 steps, instead of bench.py)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
tag=$1; shift
O=$R/gpurun_out/pmc_sq/$tag
mkdir -p $O
prog=("$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-profile)
if [ "$1" = "--ncf" ]; then shift; prog=("$R/tools/bench_ncf.py" --no-cpu-baseline --steps 100 --warmup 10); fi
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU -d $O/p1 -o run --output-format csv -- python3 "${prog[@]}" "$@" > $O/p1.out 2>&1 || { tail -5 $O/p1.out; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d $O/p2 -o run --output-format csv -- python3 "${prog[@]}" "$@" > $O/p2.out 2>&1 || { tail -5 $O/p2.out; exit 1; }
cd $R && python3 tools/pmc_sq.py $O
