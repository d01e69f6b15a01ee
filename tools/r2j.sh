# fix-up kernels with the row loaded once; fresh cube builds
set -o pipefail
mkdir -p gpurun_out/r2j
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_hash_mfma.py tests/test_gpu_index.py > gpurun_out/r2j/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r2j/pytest.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r2j/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_rows.py --rows lsh --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/r2j/rows.jsonl 2> $GRAFT_REPO_ROOT/gpurun_out/r2j/rows.err; rc=$?; cat $GRAFT_REPO_ROOT/gpurun_out/r2j/rows.jsonl; exit $rc
