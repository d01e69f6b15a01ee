set -u
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -m pytest tests/test_gpu_index.py tests/test_gpu_hash_assign.py -q -m gpu -p no:cacheprovider > gpurun_out/t4.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/t4.log
