#!/bin/bash
# A/B kernel stats of the recommender's terms phase (tools/time_terms.py) under
# the test build's switches: tools/terms_ab.sh TAG "ENV=VAL ..." ...
set -u
TAG=${1:?tag}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
i=0
for cfg in "$@"; do
  i=$((i + 1))
  (cd /tmp && export TMPDIR=/tmp LSHKM_LIB=$R/crypto-recommendation_amd/liblshkm_test.so && export $cfg && \
   { [ "${LIBV:-}" = "" ] || export LSHKM_LIB=$R/crypto-recommendation_amd/liblshkm_$LIBV.so; } && \
   timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ab$i" -o run -- \
     python3 "$R/tools/time_terms.py" > "$OUT/ab$i.txt" 2>&1)
  rc=$?; echo "[$cfg] rc=$rc $(grep cluster_terms "$OUT/ab$i.txt")"; [ $rc -eq 0 ] || exit $rc
  find "$OUT/ab$i" -name '*kernel_stats.csv' -exec python3 -c "
import csv,sys
for r in list(csv.DictReader(open(sys.argv[1])))[:6]: print('   ', r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1))" {} \;
done
