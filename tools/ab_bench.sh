#!/bin/bash
# A/B of an environment switch on the C3 bench line (same box, alternating):
#   tools/ab_bench.sh TAG "ENV_A" "ENV_B" [reps]   e.g. "LSHKM_DEFER_JOIN=0" "LSHKM_DEFER_JOIN=1"
set -o pipefail
OUT=gpurun_out/${1:?tag}
A=${2:?env A}; B=${3:?env B}; REPS=${4:-2}
mkdir -p $OUT
for rep in $(seq 1 $REPS); do
  for v in A B; do
    if [ $v = A ]; then e="$A"; else e="$B"; fi
    env $e timeout -k 10 300 python bench.py --no-cpu-baseline --no-c5 > $OUT/$v.$rep.json 2> $OUT/$v.$rep.err || { tail -3 $OUT/$v.$rep.err; exit 1; }
    python3 -c "import json,sys; b=json.load(open('$OUT/$v.$rep.json')); print('$v ($e): %.4f ms/step, kernel %.4f ms' % (b['ms_per_step'], b['roofline']['kernel_ms']))"
  done
done
