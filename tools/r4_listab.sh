#!/bin/bash
# LIST-refinement ablations (timing only): kernel averages of tools/time_fused.py per library build
set -u
R=$PWD
for v in "$@"; do
  if [ $v = base ]; then lib=$R/crypto-recommendation_amd/liblshkm.so; else lib=$R/crypto-recommendation_amd/liblshkm_$v.so; fi
  (cd /tmp && export TMPDIR=/tmp LSHKM_LIB=$lib && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
     -d $R/gpurun_out/listab_$v -o run -- python3 $R/tools/time_fused.py > $R/gpurun_out/listab_$v.log 2>&1) || { tail -5 gpurun_out/listab_$v.log; exit 1; }
  echo "== $v: $(grep fused gpurun_out/listab_$v.log | head -1)"
  python3 - "$R/gpurun_out/listab_$v" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if any(k in r["Name"] for k in ("persistent", "pruned", "fused_hi", "fixup")):
        print(f'{float(r["AverageNs"])/1e3:9.1f} us x{r["Calls"]:>4} {r["Name"][:70]}')
PY
done
