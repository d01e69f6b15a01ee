# bound E before the centroid tiles, first chain loads before the certificate: parity, then timing vs the previous build
set -o pipefail
mkdir -p gpurun_out/r3b
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_hash_assign.py tests/test_gpu_f64.py tests/test_gpu_zero_vectors.py tests/test_gpu_multirank.py > gpurun_out/r3b/pytest.log 2>&1; rc=$?; tail -1 gpurun_out/r3b/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in prev base prev base prev base; do
  if [ $v = base ]; then lib=crypto-recommendation_amd/liblshkm.so; else lib=crypto-recommendation_amd/liblshkm_$v.so; fi
  LSHKM_LIB=$PWD/$lib timeout -k 10 120 python tools/time_fused.py > gpurun_out/r3b/$v.txt 2>&1 || { tail -3 gpurun_out/r3b/$v.txt; exit 1; }
  echo "$v $(tail -1 gpurun_out/r3b/$v.txt | cut -c1-80)"
done
