#!/bin/bash
# Fused-pass timing of library variants (tools/time_fused.py), twice each in
# alternation: tools/variants.sh TAG base name1 name2 ...  (base = liblshkm.so,
# name = crypto-recommendation_amd/liblshkm_<name>.so); each run under its own limit.
set -u
TAG=${1:?tag}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for rep in 1 2; do
  for v in "$@"; do
    if [ "$v" = base ]; then lib=crypto-recommendation_amd/liblshkm.so; else lib=crypto-recommendation_amd/liblshkm_$v.so; fi
    LSHKM_LIB=$PWD/$lib timeout -k 10 120 python tools/time_fused.py > "$OUT/$v.$rep.txt" 2>&1 || { tail -3 "$OUT/$v.$rep.txt"; exit 1; }
    echo "$v: $(tail -1 "$OUT/$v.$rep.txt" | cut -d: -f2 | cut -c1-60)"
  done
done
