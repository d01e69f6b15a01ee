# hash fix-up on a side stream beside the LIST refinement: parity, timing, C3 bench with kernel trace
set -o pipefail
mkdir -p gpurun_out/r3f
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_hash_assign.py tests/test_gpu_f64.py tests/test_gpu_zero_vectors.py tests/test_gpu_multirank.py tests/test_gpu_c1.py > gpurun_out/r3f/pytest.log 2>&1; rc=$?; tail -1 gpurun_out/r3f/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do timeout -k 10 120 python tools/time_fused.py 2>&1 | tail -1 | cut -c1-120 || exit 1; done
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r3f/bench.json 2> gpurun_out/r3f/bench.err || exit 1
python3 -c "import json;b=json.load(open('gpurun_out/r3f/bench.json'));print(b['ms_per_step'], b['value'], b['roofline']['kernel_ms'], b['roofline']['frac'])"
