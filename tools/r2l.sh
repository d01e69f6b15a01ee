# cosine on the hi-only form: full GPU suite, cosine row under rocprof
set -o pipefail
mkdir -p gpurun_out/r2l
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2l/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r2l/pytest.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r2l/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_rows.py --rows cosine --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/r2l/rows.jsonl 2> $GRAFT_REPO_ROOT/gpurun_out/r2l/rows.err; rc=$?; cat $GRAFT_REPO_ROOT/gpurun_out/r2l/rows.jsonl; exit $rc
