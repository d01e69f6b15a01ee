# cosine winner on both lane halves: cosine parity tests, then the cosine row
set -o pipefail
mkdir -p gpurun_out/r2o
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_hash_assign.py tests/test_gpu_zero_vectors.py tests/test_gpu_f64.py tests/test_gpu_c1.py tests/test_gpu_multirank.py > gpurun_out/r2o/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r2o/pytest.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r2o/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_rows.py --rows cosine --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/r2o/rows.jsonl 2> $GRAFT_REPO_ROOT/gpurun_out/r2o/rows.err; rc=$?; cat $GRAFT_REPO_ROOT/gpurun_out/r2o/rows.jsonl; head -6 $GRAFT_REPO_ROOT/gpurun_out/r2o/prof/run_kernel_stats.csv | cut -c1-120; exit $rc
