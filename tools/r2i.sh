# MFMA hash: parity tests, then the index rows under rocprof
set -o pipefail
mkdir -p gpurun_out/r2i
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_hash_mfma.py tests/test_gpu_index.py > gpurun_out/r2i/pytest.log 2>&1; rc=$?; tail -5 gpurun_out/r2i/pytest.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r2i/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_rows.py --rows lsh,cube --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/r2i/rows.jsonl 2> $GRAFT_REPO_ROOT/gpurun_out/r2i/rows.err; rc=$?; cat $GRAFT_REPO_ROOT/gpurun_out/r2i/rows.jsonl; exit $rc
