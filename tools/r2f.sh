set -o pipefail
mkdir -p gpurun_out/r2f
for v in base l2x l2xnochain nochain; do
  if [ $v = base ]; then lib=crypto-recommendation_amd/liblshkm.so; else lib=crypto-recommendation_amd/liblshkm_$v.so; fi
  LSHKM_LIB=$PWD/$lib timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r2f/$v.json 2> gpurun_out/r2f/$v.err || { tail -3 gpurun_out/r2f/$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r2f/$v.json'));print('$v', round(d['ms_per_step'],3), 'kernel', round(d['roofline']['kernel_ms'],3))"
done

