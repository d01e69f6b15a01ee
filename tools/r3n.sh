# s_setprio variants of the hi-only kernel: chain priority 2 / no MFMA priority / both (fused-pass timing)
set -o pipefail
mkdir -p gpurun_out/r3o
LSHKM_LIB=$PWD/crypto-recommendation_amd/liblshkm_cp3.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_hash_assign.py > gpurun_out/r3o/pytest.log 2>&1; rc=$?; tail -1 gpurun_out/r3o/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in base cp3 cp3mp2 base cp3 cp3mp2; do
  if [ $v = base ]; then lib=crypto-recommendation_amd/liblshkm.so; else lib=crypto-recommendation_amd/liblshkm_$v.so; fi
  LSHKM_LIB=$PWD/$lib timeout -k 10 120 python tools/time_fused.py > gpurun_out/r3o/$v.txt 2>&1 || { tail -3 gpurun_out/r3o/$v.txt; exit 1; }
  echo "$v $(tail -1 gpurun_out/r3o/$v.txt | cut -c1-70)"
done
