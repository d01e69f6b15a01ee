# Timing of fused_hi_kernel ablation builds (results of the ablated builds are wrong by construction).
set -o pipefail
mkdir -p gpurun_out/r2g
for v in base nochain l2x nohash noctile l2xnochain computeonly base; do
  if [ $v = base ]; then lib=crypto-recommendation_amd/liblshkm.so; else lib=crypto-recommendation_amd/liblshkm_$v.so; fi
  LSHKM_LIB=$PWD/$lib timeout -k 10 120 python tools/time_fused.py > gpurun_out/r2g/$v.txt 2>&1 || { tail -3 gpurun_out/r2g/$v.txt; exit 1; }
  echo "$v $(tail -1 gpurun_out/r2g/$v.txt)"
done
