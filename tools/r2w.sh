# LIST refinement on/off (LSHKM_HI_LIST): parity with it off, then C3 / C5 timings both ways
set -o pipefail
mkdir -p gpurun_out/r2w
LSHKM_HI_LIST=0 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_hash_assign.py tests/test_gpu_update.py tests/test_gpu_f64.py > gpurun_out/r2w/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r2w/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0 1 0; do
  LSHKM_HI_LIST=$v timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r2w/c3_$v.json 2> gpurun_out/r2w/c3_$v.err || exit 1
  LSHKM_HI_LIST=$v timeout -k 10 200 python bench.py --workload c5 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r2w/c5_$v.json 2> gpurun_out/r2w/c5_$v.err || exit 1
  python3 -c "import json;a=json.load(open('gpurun_out/r2w/c3_$v.json'));b=json.load(open('gpurun_out/r2w/c5_$v.json'));print('LIST=$v', 'c3', round(a['ms_per_step'],3), a['roofline']['kernel_ms'], 'c5', round(b['ms_per_step'],3), b['exactness'])"
done
