set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/prof
cd $R
timeout -k 10 300 python -m pytest tests/test_gpu_hash_assign.py -q -m gpu -p no:cacheprovider > gpurun_out/t2.log 2>&1
rc=$?; echo "pytest rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py > gpurun_out/bench1.json 2> gpurun_out/bench1.err
rc=$?; echo "bench rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $R/gpurun_out/bench_prof.json 2> $R/gpurun_out/bench_prof.err
echo "rocprof rc=$?"
