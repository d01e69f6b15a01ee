# pipelined winner chain: parity of the fused path, then A/B timing
set -o pipefail
mkdir -p gpurun_out/r2m
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_hash_assign.py tests/test_gpu_update.py tests/test_gpu_multirank.py > gpurun_out/r2m/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r2m/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in base nopipe base nopipe; do
  if [ $v = base ]; then lib=crypto-recommendation_amd/liblshkm.so; else lib=crypto-recommendation_amd/liblshkm_$v.so; fi
  LSHKM_LIB=$PWD/$lib timeout -k 10 120 python tools/time_fused.py > gpurun_out/r2m/$v.txt 2>&1 || { tail -3 gpurun_out/r2m/$v.txt; exit 1; }
  echo "$v $(tail -1 gpurun_out/r2m/$v.txt)"
done
