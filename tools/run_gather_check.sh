#!/bin/bash
# Gather-path check: hash/assign parity tests, then fused-pass timing with the
# LDS-DMA gather on and off (alternating), then TA/TD counters of the gather build.
set -o pipefail
OUT=gpurun_out/${1:-r3h}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_hash_assign.py tests/test_gpu_c5.py > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for g in 1 0; do
    LSHKM_GATHER=$g timeout -k 10 120 python tools/time_fused.py > $OUT/g$g.$rep.txt 2>&1 || exit 1
    echo "gather=$g $(tail -1 $OUT/g$g.$rep.txt | cut -d: -f2 | cut -c1-60)"
  done
done
bash tools/pmc_passes.sh ${1:-r3h}/pmc "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE GRBM_COUNT" "TD_TD_BUSY_sum TD_TC_STALL_sum" "TCP_TCP_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum"
