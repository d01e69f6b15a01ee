#!/bin/bash
# Fused-pass timing of library variants (tools/time_fused.py), twice each in
# alternation: tools/variants.sh TAG base name1 name2 ...  (base = liblshkm.so,
# name = crypto-recommendation_amd/liblshkm_<name>.so; name@VAR=VALUE runs that
# library with one environment setting); each run under its own limit.
set -u
TAG=${1:?tag}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for rep in 1 2; do
  for vv in "$@"; do
    v=${vv%%@*}; ev=""; [ "$v" != "$vv" ] && ev=${vv#*@}
    if [ "$v" = base ]; then lib=crypto-recommendation_amd/liblshkm.so; else lib=crypto-recommendation_amd/liblshkm_$v.so; fi
    tagf=$(echo "$vv" | tr '@=' '__')
    env LSHKM_LIB=$PWD/$lib $ev timeout -k 10 120 python tools/time_fused.py > "$OUT/$tagf.$rep.txt" 2>&1 || { tail -3 "$OUT/$tagf.$rep.txt"; exit 1; }
    echo "$vv: $(tail -1 "$OUT/$tagf.$rep.txt" | cut -d: -f2- | cut -c1-150)"
  done
done
