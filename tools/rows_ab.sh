#!/bin/bash
# bench_rows rows under two environments (same box): tools/rows_ab.sh TAG ROWS "ENV_A" "ENV_B"
set -o pipefail
OUT=gpurun_out/${1:?tag}; ROWS=${2:?rows}; A=${3:?env A}; B=${4:?env B}
mkdir -p $OUT
for v in A B; do
  if [ $v = A ]; then e="$A"; else e="$B"; fi
  env $e timeout -k 10 300 python tools/bench_rows.py --rows $ROWS --no-cpu > $OUT/rows_$v.jsonl 2> $OUT/rows_$v.err || { tail -3 $OUT/rows_$v.err; exit 1; }
  python3 -c "
import json
for l in open('$OUT/rows_$v.jsonl'):
    r = json.loads(l); print('$v ($e):', r['row'], round(r['gpu_s'] * 1e3, 3), 'ms')"
done
