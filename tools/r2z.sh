# two-image single launch at K = 1024: parity tests, C5 both forms, kernel profile and PMC traffic
set -o pipefail
mkdir -p gpurun_out/r2z
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_hash_assign.py tests/test_gpu_multirank.py tests/test_gpu_update.py tests/test_gpu_f64.py tests/test_gpu_zero_vectors.py > gpurun_out/r2z/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r2z/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0 1; do
  LSHKM_HI_TWO_IMAGE=$v timeout -k 10 200 python bench.py --workload c5 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r2z/c5_$v.json 2> gpurun_out/r2z/c5_$v.err || exit 1
  python3 -c "import json;b=json.load(open('gpurun_out/r2z/c5_$v.json'));print('TWO_IMAGE=$v', round(b['ms_per_step'],3), b['roofline']['kernel_ms'], b['exactness'])"
done
bash tools/gpu_run.sh r2z prof5 pmc5
