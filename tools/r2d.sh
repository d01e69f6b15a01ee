set -o pipefail
mkdir -p gpurun_out/r2d
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r2d/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r2d/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0 1; do
  LSHKM_FUSED_HI=$v timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r2d/hi$v.json 2> gpurun_out/r2d/hi$v.err || { tail -3 gpurun_out/r2d/hi$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r2d/hi$v.json'));print('hi=$v', round(d['ms_per_step'],3), 'kernel', round(d['roofline']['kernel_ms'],3), d['exactness'])"
done
LSHKM_FUSED_HI=1 timeout -k 10 200 python bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r2d/c5.json 2> gpurun_out/r2d/c5.err || { tail -3 gpurun_out/r2d/c5.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r2d/c5.json'));print('c5', round(d['ms_per_step'],3), 'kernel', round(d['roofline']['kernel_ms'],3), d['exactness'])"
