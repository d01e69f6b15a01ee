# scheduler strategies for fused.hip (max-ilp / max-memory-clause): hash-assign parity on each, then timing
set -o pipefail
mkdir -p gpurun_out/r3a
for v in ilp mclause; do
  LSHKM_LIB=$PWD/crypto-recommendation_amd/liblshkm_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_hash_assign.py > gpurun_out/r3a/pytest_$v.log 2>&1; rc=$?; echo "$v $(tail -1 gpurun_out/r3a/pytest_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for v in base ilp mclause base ilp mclause; do
  if [ $v = base ]; then lib=crypto-recommendation_amd/liblshkm.so; else lib=crypto-recommendation_amd/liblshkm_$v.so; fi
  LSHKM_LIB=$PWD/$lib timeout -k 10 120 python tools/time_fused.py > gpurun_out/r3a/$v.txt 2>&1 || { tail -3 gpurun_out/r3a/$v.txt; exit 1; }
  echo "$v $(tail -1 gpurun_out/r3a/$v.txt | cut -c1-90)"
done
