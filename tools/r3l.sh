# SQ counters and HBM fetch of the k-means++ row (one pass each)
set -o pipefail
mkdir -p gpurun_out/r3l
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r3l/sq -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_rows.py --rows kpp --no-cpu > /dev/null 2> $GRAFT_REPO_ROOT/gpurun_out/r3l/sq.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r3l/fetch -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_rows.py --rows kpp --no-cpu > /dev/null 2> $GRAFT_REPO_ROOT/gpurun_out/r3l/fetch.err || exit 1
echo done
