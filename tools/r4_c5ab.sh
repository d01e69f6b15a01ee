#!/bin/bash
# C5 hash+assign call A/B between library builds (same box): tools/r4_c5ab.sh VARIANT
set -u
V=${1:?variant}
OUT=gpurun_out/c5ab; mkdir -p $OUT
for i in 1 2; do
  for v in base $V; do
    if [ $v = base ]; then lib=crypto-recommendation_amd/liblshkm.so; else lib=crypto-recommendation_amd/liblshkm_$v.so; fi
    LSHKM_LIB=$PWD/$lib timeout -k 10 300 python bench.py --workload c5 --steps 5 --warmup 1 --no-cpu-baseline > $OUT/$v$i.json 2> $OUT/$v$i.err || { tail -5 $OUT/$v$i.err; exit 1; }
    python -c "
import json; b=json.loads(open('$OUT/$v$i.json').read().strip().splitlines()[-1]); c=b.get('c5', b)
print('$v', round(c['ms_per_step'], 3), 'fused pass', round(c['roofline']['kernel_ms'], 3))"
  done
done
