# windowed hypercube candidate copy: index tests, then the index rows under rocprof
set -o pipefail
mkdir -p gpurun_out/r2t
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_index.py tests/test_gpu_multirank.py > gpurun_out/r2t/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r2t/pytest.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r2t/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_rows.py --rows lsh,cube --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/r2t/rows.jsonl 2> $GRAFT_REPO_ROOT/gpurun_out/r2t/rows.err; rc=$?; cut -c1-500 $GRAFT_REPO_ROOT/gpurun_out/r2t/rows.jsonl; grep -E "cq_|lq_" $GRAFT_REPO_ROOT/gpurun_out/r2t/prof/run_kernel_stats.csv | cut -c1-120; exit $rc
