# k-means sums rows in flight: 16 vs 32 (update row timing)
set -o pipefail
mkdir -p gpurun_out/r2y
for v in base u32 base u32; do
  if [ $v = base ]; then lib=crypto-recommendation_amd/liblshkm.so; else lib=crypto-recommendation_amd/liblshkm_$v.so; fi
  LSHKM_LIB=$PWD/$lib timeout -k 10 200 python tools/bench_rows.py --rows update --no-cpu > gpurun_out/r2y/$v.txt 2>&1 || { tail -3 gpurun_out/r2y/$v.txt; exit 1; }
  echo "$v $(cut -c1-120 gpurun_out/r2y/$v.txt)"
done
