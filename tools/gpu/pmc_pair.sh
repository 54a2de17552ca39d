# SQ + cache-level counter passes (separate rocprofv3 --pmc runs) over one K=20 bench.py call per
# variant, summarised per kernel by tools/pmc_sq.py: the persistent step against the fused launches
# (wave wait share, L1 accesses and L1->L2 reads, L2 hits / misses, L2->fabric
# read requests of the gate polls).
#   gpurun --timeout 900 -- 'bash tools/gpu/pmc_pair.sh <tag> "fused:" "persist:BPRMF_PERSIST=1"'
set -o pipefail
tag="$1"; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc_pair/$tag
mkdir -p "$O"
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
P2="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"
for spec in "$@"; do
  name="${spec%%:*}"; envs="${spec#*:}"
  n=0; mkdir -p "$O/$name"
  for pass in "$P1" "$P2"; do
    n=$((n + 1))
    ( [ -n "$envs" ] && for kv in ${envs//,/ }; do export "$kv"; done
      cd /tmp &&
      timeout -s KILL 120 rocprofv3 --pmc $pass -d "$O/$name/p$n" -o run --output-format csv -- \
        python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-profile --no-relaxed \
        > "$O/$name/p$n.out" 2>&1 ) || { echo "variant $name pass $n failed"; tail -n 5 "$O/$name/p$n.out"; exit 1; }
  done
  echo "== $name"
  (cd "$R" && python3 tools/pmc_sq.py "$O/$name" | grep -E "k_fused_step|k_persist_steps|k_user_step|k_item_step") || exit 1
done
