# k-means sums by exact fp64 adds; pruned exact pass up to K = 1024
set -o pipefail
mkdir -p gpurun_out/r2n
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2n/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r2n/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_run.sh r2n prof5 && head -8 gpurun_out/r2n/prof5/run_kernel_stats.csv | cut -c1-150 && python -c "import json;d=json.load(open('gpurun_out/r2n/bench_prof5.json'));print(d['ms_per_step'], d['roofline']['kernel_ms'], d['exactness'])"
timeout -k 10 200 python tools/bench_rows.py --rows update --no-cpu
