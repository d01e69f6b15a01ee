# two-barrier radix downsweep: full GPU suite, then the index / update rows and C5 under rocprof
set -o pipefail
mkdir -p gpurun_out/r2s
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2s/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r2s/pytest.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r2s/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_rows.py --rows lsh,cube,update --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/r2s/rows.jsonl 2> $GRAFT_REPO_ROOT/gpurun_out/r2s/rows.err; rc=$?; cut -c1-330 $GRAFT_REPO_ROOT/gpurun_out/r2s/rows.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 $GRAFT_REPO_ROOT/bench.py --workload c5 --steps 5 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r2s/bench5.json 2> $GRAFT_REPO_ROOT/gpurun_out/r2s/bench5.err; rc=$?; cut -c1-300 $GRAFT_REPO_ROOT/gpurun_out/r2s/bench5.json; exit $rc
