#!/bin/bash
# C3 whole-call timing: the K <= 256 pruned pass in the flat form (A/B): tools/r4_xpn.sh TAG
set -u
TAG=${1:?tag}
LSHKM_LIB=$PWD/crypto-recommendation_amd/liblshkm_xpn.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fast_dist.py tests/test_gpu_general_rows.py tests/test_gpu_hash_assign.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || { grep -E "^E |Error" gpurun_out/${TAG}_tests.log | head; exit $rc; }
bash tools/variants.sh "${TAG}_c3" base xpn || exit 1
