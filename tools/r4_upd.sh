#!/bin/bash
# k-means update on fp64 rows: parity of the segmented form, timings of the
# three forms, and a kernel-trace profile of the segmented one. tools/r4_upd.sh TAG
set -u
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_update.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [ $rc -eq 0 ] || { grep -E "^E |Error" "$OUT/tests.log" | head -20; exit $rc; }
for v in seg fx; do
  LSHKM_KM_PATH=$v timeout -k 10 120 python tools/time_update64.py || exit 1
done
LSHKM_KM_CHAIN=64 timeout -k 10 120 python tools/time_update64.py || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
LSHKM_KM_PATH=seg timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o upd -- python3 tools/time_update64.py > "$OUT/prof.log" 2>&1 || { tail -5 "$OUT/prof.log"; exit 1; }
f=$(find "$OUT/prof" -name "*kernel_stats.csv" | head -1); cut -d, -f1-8 "$f" | head -15
