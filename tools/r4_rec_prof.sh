#!/bin/bash
# Kernel-trace profile of the C5 bench (recommend kernels): tools/r4_rec_prof.sh TAG
set -u
TAG=${1:?tag}; R=$(pwd); OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
   -d "$OUT/prof5" -o run -- python3 "$R/bench.py" --workload c5 --steps 3 --warmup 1 --no-cpu-baseline \
   > "$OUT/c5.json" 2> "$OUT/c5.err") || { tail -5 "$OUT/c5.err"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/prof5/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:12]:
    print(r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us", r["Percentage"])
PY
