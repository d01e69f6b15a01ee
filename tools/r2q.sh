# 4-lane hash fix-ups: fused-path parity tests, timing, kernel profile
set -o pipefail
mkdir -p gpurun_out/r2q
true || timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_hash_assign.py tests/test_gpu_f64.py tests/test_gpu_zero_vectors.py > gpurun_out/r2q/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r2q/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in base s3 s2 base; do
  if [ $v = base ]; then lib=crypto-recommendation_amd/liblshkm.so; else lib=crypto-recommendation_amd/liblshkm_$v.so; fi
  LSHKM_LIB=$PWD/$lib timeout -k 10 120 python tools/time_fused.py > gpurun_out/r2q/$v.txt 2>&1 || { tail -3 gpurun_out/r2q/$v.txt; exit 1; }
  echo "$v $(tail -1 gpurun_out/r2q/$v.txt)"
done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r2q/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r2q/bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/r2q/bench.err; rc=$?; cat $GRAFT_REPO_ROOT/gpurun_out/r2q/bench.json; head -8 $GRAFT_REPO_ROOT/gpurun_out/r2q/prof/run_kernel_stats.csv | cut -c1-110; exit $rc
