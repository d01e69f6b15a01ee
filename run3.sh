set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/prof3
cd $R
timeout -k 10 300 python -m pytest tests/test_gpu_hash_assign.py -q -m gpu -p no:cacheprovider > gpurun_out/t3.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t3.log; if [ $rc -gt 1 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof3 -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $R/gpurun_out/bench3.json 2> $R/gpurun_out/bench3.err
echo "rocprof rc=$?"
