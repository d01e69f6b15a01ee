#!/bin/bash
# terms-phase timing + SQ counters of rc_terms_kernel: tools/r4_terms_pmc.sh TAG
set -u
TAG=${1:?tag}; R=$(pwd); OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"
timeout -k 10 200 python tools/time_terms.py || exit 1
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU" \
           "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_BUSY_CYCLES"; do
  i=$((i+1))
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set --output-format csv \
     -d "$OUT/sq$i" -o run -- python3 "$R/tools/time_terms.py" > "$OUT/sq$i.log" 2>&1) || { tail -3 "$OUT/sq$i.log"; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/sq*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "rc_terms_kernel" in r.get("Kernel_Name", ""):
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(k, sorted(v)[len(v) // 2])
PY
