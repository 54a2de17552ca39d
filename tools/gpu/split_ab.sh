# Builder tests first (they compare the split builder bitwise with the one-workgroup and radix
# builds), then ubench_call A/B of the variants given, then the whole -m gpu suite.
#   gpurun --timeout 900 -- 'bash tools/gpu/split_ab.sh <tag> "ENV=a" "ENV=b" ...'
set -o pipefail
tag="$1"; shift
out="gpurun_out/$tag"
mkdir -p "$out"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "builder or split or replay or fused" > "$out/builder_tests.log" 2>&1
rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" "$out/builder_tests.log" | tail -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/ubench_call.py --ab "$@" > "$out/ab.log" 2>&1 || { tail -20 "$out/ab.log"; exit 1; }
cut -c1-330 "$out/ab.log"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1
rc=$?
tail -3 "$out/gpu_tests.log"
exit $rc
