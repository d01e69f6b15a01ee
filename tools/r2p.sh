# winner-chain prefetch depth: timing of the fused pass for CHAIN_PF 1 / 4 / 8
set -o pipefail
mkdir -p gpurun_out/r2p
for v in base pf4 pf8 base pf8; do
  if [ $v = base ]; then lib=crypto-recommendation_amd/liblshkm.so; else lib=crypto-recommendation_amd/liblshkm_$v.so; fi
  LSHKM_LIB=$PWD/$lib timeout -k 10 120 python tools/time_fused.py > gpurun_out/r2p/$v.txt 2>&1 || { tail -3 gpurun_out/r2p/$v.txt; exit 1; }
  echo "$v $(tail -1 gpurun_out/r2p/$v.txt)"
done
