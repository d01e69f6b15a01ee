# wide pruned pass rows per wave 2 vs 4 (C5 bench, pruned kernel time from rocprof)
set -o pipefail
mkdir -p gpurun_out/r3g
for v in base wr4; do
  if [ $v = base ]; then lib=crypto-recommendation_amd/liblshkm.so; else lib=crypto-recommendation_amd/liblshkm_$v.so; fi
  (cd /tmp && export TMPDIR=/tmp && LSHKM_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r3g/$v -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload c5 --steps 5 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r3g/$v.json 2> $GRAFT_REPO_ROOT/gpurun_out/r3g/$v.err) || exit 1
  echo "$v $(python3 -c "import json;print(json.load(open('gpurun_out/r3g/$v.json'))['ms_per_step'])") $(grep assign_pruned gpurun_out/r3g/$v/run_kernel_stats.csv | cut -d, -f3-4)"
done
