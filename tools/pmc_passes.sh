#!/bin/bash
# Separate rocprofv3 --pmc passes (one counter set each) over tools/time_fused.py:
#   tools/pmc_passes.sh TAG "C1 C2 ..." "C3 C4 ..." ...
# Summaries: python tools/sqsum.py "fused_hi_kernel<true, false, 0, 1>" gpurun_out/TAG/p*
set -u
TAG=${1:?tag}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
i=0
for set in "$@"; do
  i=$((i+1))
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set --output-format csv \
     -d "$OUT/p$i" -o run -- python3 "$R/tools/time_fused.py" > "$OUT/p$i.txt" 2> "$OUT/p$i.err")
  rc=$?; echo "pass $i ($set) rc=$rc"; [ $rc -eq 0 ] || { tail -3 "$OUT/p$i.err"; exit $rc; }
done
