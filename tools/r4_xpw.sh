#!/bin/bash
# C5 fused call timing (the pruned exact pass inside) for the wide pruned-pass
# variants, alternated: tools/r4_xpw.sh TAG
set -u
TAG=${1:?tag}
timeout -k 10 300 python -u -m pytest tests/test_gpu_c5.py tests/test_gpu_general_rows.py -m gpu -x -q --timeout 120 --timeout-method thread -k "not full_size" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || { grep -E "^E |Error" gpurun_out/${TAG}_tests.log | head; exit $rc; }
TF_K=1024 bash tools/variants.sh "${TAG}_c5" base xpw4 xpw2 xpw0 || exit 1
