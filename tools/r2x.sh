# whole-row k-means sums: update parity tests, then the update row and C5 under rocprof
set -o pipefail
mkdir -p gpurun_out/r2x
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_update.py tests/test_gpu_multirank.py tests/test_gpu_f64.py tests/test_gpu_c1.py > gpurun_out/r2x/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r2x/pytest.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r2x/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload c5 --steps 5 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r2x/bench5.json 2> $GRAFT_REPO_ROOT/gpurun_out/r2x/bench5.err; rc=$?; cut -c1-250 $GRAFT_REPO_ROOT/gpurun_out/r2x/bench5.json; grep km_ $GRAFT_REPO_ROOT/gpurun_out/r2x/prof/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-150; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 $GRAFT_REPO_ROOT/tools/bench_rows.py --rows update --no-cpu | cut -c1-300
