# HR@10 / NDCG@10, the in-training and the final-table loss of the exact step and the relaxed
# modes, with the popularity baseline (tools/hr_modes.py): the planted-structure ml-20m shape and
# the F5 protocol, seeds 11-13.   gpurun --timeout 1200 -- 'bash tools/gpu/quality.sh <tag> [which] [modes]'
set -o pipefail
tag="$1"; which="${2:-planted,f5}"; modes="${3:-exact,local,hogwild}"
out="gpurun_out/$tag"
mkdir -p "$out"
timeout -k 10 1000 python -u tools/hr_modes.py --which "$which" --modes "$modes" --seeds 11,12,13 \
  --epochs 10 --users-eval 20000 > "$out/hr_modes.jsonl" 2> "$out/hr_modes.err" || { tail -n 20 "$out/hr_modes.err"; exit 1; }
cut -c1-330 "$out/hr_modes.jsonl"
