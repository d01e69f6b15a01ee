#!/bin/bash
# Headline-kernel variant check: hash/assign parity tests (incl. the fast
# distance), then fused-pass timing of the chain variants (alternating):
#   exact chain + LDS-DMA gather (default: f32 rows when exact) | fp64 rows gathered | register loads | fast distance
set -o pipefail
OUT=gpurun_out/${1:-r3h}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gather.py tests/test_gpu_hash_assign.py tests/test_gpu_c5.py tests/test_gpu_fast_dist.py > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in gather gather64 nogather fast; do
    case $v in gather) e="LSHKM_GATHER=1";; gather64) e="LSHKM_GATHER32=0";; nogather) e="LSHKM_GATHER=0";; fast) e="LSHKM_DIST=fast";; esac
    env $e timeout -k 10 120 python tools/time_fused.py > $OUT/$v.$rep.txt 2>&1 || exit 1
    echo "$v $(tail -1 $OUT/$v.$rep.txt | cut -d: -f2 | cut -c1-80)"
  done
done
