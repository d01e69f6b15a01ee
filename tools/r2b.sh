set -o pipefail
mkdir -p gpurun_out/r2b
timeout -k 10 300 python -u -m pytest tests/test_gpu_f64.py tests/test_gpu_c1.py tests/test_compat.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r2b/f64.log 2>&1
rc=$?; tail -5 gpurun_out/r2b/f64.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/r2b/pytest.log 2>&1
rc=$?; tail -5 gpurun_out/r2b/pytest.log; exit $rc
