set -o pipefail
L=$GRAFT_REPO_ROOT/recommend-lib_amd
mkdir -p gpurun_out/r3b_parts
for v in p8 p2; do
BPRMF_DIAG_LIB=$L/libbprmf_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "builder or split or replay" > gpurun_out/r3b_parts/t_$v.log 2>&1 || { tail -20 gpurun_out/r3b_parts/t_$v.log; exit 1; }
tail -1 gpurun_out/r3b_parts/t_$v.log
done
timeout -k 10 500 python -u tools/ubench_call.py --ab "X=1" "BPRMF_DIAG_LIB=$L/libbprmf_p8.so" "BPRMF_DIAG_LIB=$L/libbprmf_p2.so" "X=1" "BPRMF_DIAG_LIB=$L/libbprmf_p8.so" "BPRMF_DIAG_LIB=$L/libbprmf_p2.so" 2>&1 | cut -c1-330
