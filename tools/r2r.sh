# per-instantiation wave counts of the hi-only kernel: parity tests, C5 and C3 benches with kernel profiles
set -o pipefail
mkdir -p gpurun_out/r2r
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_hash_assign.py tests/test_gpu_f64.py tests/test_gpu_zero_vectors.py tests/test_gpu_multirank.py tests/test_gpu_update.py > gpurun_out/r2r/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r2r/pytest.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r2r/prof5 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload c5 --steps 5 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r2r/bench5.json 2> $GRAFT_REPO_ROOT/gpurun_out/r2r/bench5.err; rc=$?; cut -c1-400 $GRAFT_REPO_ROOT/gpurun_out/r2r/bench5.json; head -8 $GRAFT_REPO_ROOT/gpurun_out/r2r/prof5/run_kernel_stats.csv | cut -c1-110; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r2r/bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/r2r/bench.err; rc=$?; cut -c1-300 $GRAFT_REPO_ROOT/gpurun_out/r2r/bench.json; exit $rc
