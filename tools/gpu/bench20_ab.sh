for v in "X=1" "BPRMF_DIAG_LIB=recommend-lib_amd/libbprmf_alt.so" "X=1" "BPRMF_DIAG_LIB=recommend-lib_amd/libbprmf_alt.so" "X=1" "BPRMF_DIAG_LIB=recommend-lib_amd/libbprmf_alt.so"; do
  env $v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-profile > gpurun_out/b3.log 2>&1 || exit 1
  echo "[$v] $(grep '^{' gpurun_out/b3.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
