#!/bin/bash
# usage: tools/c5_ab.sh TAG base name1 name2 ... (name = crypto-recommendation_amd/liblshkm_<name>.so)
# C5 A/B of library variants: bench.py --workload c5 per variant (each under its own limit)
set -u
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
for rep in 1 2; do
  for v in "$@"; do
    if [ "$v" = base ]; then lib=$PWD/crypto-recommendation_amd/liblshkm.so; else lib=$PWD/crypto-recommendation_amd/liblshkm_$v.so; fi
    LSHKM_LIB=$lib timeout -k 10 200 python bench.py --workload c5 --no-cpu-baseline --steps 8 --warmup 6 > "$OUT/$v.$rep.json" 2> "$OUT/$v.$rep.err" || { tail -3 "$OUT/$v.$rep.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$OUT/$v.$rep.json')); print('$v', round(d['ms_per_step'],3), round(d['km_sums_exchange_ms'],3))"
  done
done
