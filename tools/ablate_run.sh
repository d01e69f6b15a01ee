# Timing of ablation builds (results of nolo/nochain are wrong by construction).
set -o pipefail
mkdir -p gpurun_out/abl
for v in base nolo nochain nolonochain base; do
  if [ $v = base ]; then lib=crypto-recommendation_amd/liblshkm.so; else lib=crypto-recommendation_amd/liblshkm_$v.so; fi
  LSHKM_LIB=$PWD/$lib timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/abl/$v.json 2> gpurun_out/abl/$v.err || { tail -3 gpurun_out/abl/$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/abl/$v.json'));print('$v', round(d['ms_per_step'],3), 'kernel', round(d['roofline']['kernel_ms'],3), 'ambig', d['exactness']['assign_ambiguous_rows'])"
done
