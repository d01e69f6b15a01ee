set -o pipefail
mkdir -p gpurun_out/r2c
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 500 --timeout-method thread > gpurun_out/r2c/mr.log 2>&1
rc=$?; tail -5 gpurun_out/r2c/mr.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r2c/c5.json 2> gpurun_out/r2c/c5.err
rc=$?; cat gpurun_out/r2c/c5.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/r2c/c5.err; exit $rc; }
timeout -k 10 400 python bench.py > gpurun_out/r2c/c3.json 2> gpurun_out/r2c/c3.err
rc=$?; cat gpurun_out/r2c/c3.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/r2c/c3.err; exit $rc; }
