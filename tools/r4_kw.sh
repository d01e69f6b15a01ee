#!/bin/bash
# fp64 k-means update: segment window variants (parity + time), tools/r4_kw.sh
set -u
for v in ${KW_VARIANTS:-base w256 w128}; do
  if [ $v = base ]; then lib=crypto-recommendation_amd/liblshkm.so; else lib=crypto-recommendation_amd/liblshkm_$v.so; fi
  LSHKM_LIB=$PWD/$lib timeout -k 10 200 python -u -m pytest tests/test_gpu_update.py -m gpu -x -q -k f64 --timeout 120 --timeout-method thread > gpurun_out/kw_$v.log 2>&1
  rc=$?; echo "$v: $(tail -1 gpurun_out/kw_$v.log)"; [ $rc -eq 0 ] || { grep -E "^E " gpurun_out/kw_$v.log | head -5; exit $rc; }
  LSHKM_LIB=$PWD/$lib timeout -k 10 120 python tools/time_update64.py > gpurun_out/kw_t.log || exit 1; head -1 gpurun_out/kw_t.log
  LSHKM_LIB=$PWD/$lib timeout -k 10 120 python tools/time_update64.py > gpurun_out/kw_t.log || exit 1; head -1 gpurun_out/kw_t.log
done
