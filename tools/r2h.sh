# hi-only kernel restructure: parity tests of the fused path, then timing vs variants
set -o pipefail
mkdir -p gpurun_out/r2h
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_hash_assign.py > gpurun_out/r2h/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r2h/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in base w8 w8nofence pair base; do
  if [ $v = base ]; then lib=crypto-recommendation_amd/liblshkm.so; else lib=crypto-recommendation_amd/liblshkm_$v.so; fi
  LSHKM_LIB=$PWD/$lib timeout -k 10 120 python tools/time_fused.py > gpurun_out/r2h/$v.txt 2>&1 || { tail -3 gpurun_out/r2h/$v.txt; exit 1; }
  echo "$v $(tail -1 gpurun_out/r2h/$v.txt)"
done
