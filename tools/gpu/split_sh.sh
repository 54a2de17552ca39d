# Split builder in the sharded runner: builder + sharded + IPC tests, world-1 sharded bench A/B,
# then the whole -m gpu suite.
#   gpurun --timeout 1200 -- 'bash tools/gpu/split_sh.sh <tag>'
set -o pipefail
tag="$1"
out="gpurun_out/$tag"
mkdir -p "$out"
timeout -k 10 400 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_ipc.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "split or builder or runner or ipc or sharded" > "$out/sh_tests.log" 2>&1
rc=$?
tail -3 "$out/sh_tests.log"
[ $rc -eq 0 ] || { grep -E "FAIL|Error|error" "$out/sh_tests.log" | head -20; exit $rc; }
bash tools/gpu/sh_w1.sh "$tag/shw1" "BPRMF_SPLIT_ITEMS=0" "X=1" "BPRMF_SPLIT_ITEMS=0" "X=1" || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1
rc=$?
tail -3 "$out/gpu_tests.log"
exit $rc
