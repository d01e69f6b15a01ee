#!/bin/bash
# Kernel-level timing of library variants: rocprofv3 --kernel-trace --stats over
# tools/time_fused.py per variant; prints the average duration of the headline
# kernel (and the fused-pass line).  tools/variants_prof.sh TAG base name1 ...
set -u
TAG=${1:?tag}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
for v in "$@"; do
  if [ "$v" = base ]; then lib=$R/crypto-recommendation_amd/liblshkm.so; else lib=$R/crypto-recommendation_amd/liblshkm_$v.so; fi
  (cd /tmp && export TMPDIR=/tmp LSHKM_LIB=$lib && timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv \
     -d "$OUT/$v" -o run -- python3 "$R/tools/time_fused.py" > "$OUT/$v.txt" 2> "$OUT/$v.err")
  rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -3 "$OUT/$v.err"; exit $rc; }
  python3 - "$OUT/$v" "$v" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
out = []
for r in csv.DictReader(open(f)):
    if "fused_hi_kernel" in r["Name"] or "hash_fixup" in r["Name"] or "fused_persistent" in r["Name"]:
        out.append(f"{r['Name'].split('(')[0].replace('void lshkm::', '')} {float(r['AverageNs']) / 1e3:.1f}us")
print(sys.argv[2] + ": " + "; ".join(out))
PY
done
