# double-double x87 chain in the exact cosine paths: full GPU suite, then the cosine rows under rocprof
set -o pipefail
mkdir -p gpurun_out/r2v
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2v/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r2v/pytest.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r2v/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_rows.py --rows cosine,recom --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/r2v/rows.jsonl 2> $GRAFT_REPO_ROOT/gpurun_out/r2v/rows.err; rc=$?; cut -c1-420 $GRAFT_REPO_ROOT/gpurun_out/r2v/rows.jsonl; head -14 $GRAFT_REPO_ROOT/gpurun_out/r2v/prof/run_kernel_stats.csv | cut -c1-110; exit $rc
