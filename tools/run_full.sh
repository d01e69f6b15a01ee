#!/bin/bash
# Full GPU check: pytest -m gpu, then bench_rows for the given rows under rocprof
#   tools/run_full.sh TAG ROWS
set -o pipefail
T=${1:?tag}; ROWS=${2:-f64,update}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/$T/pytest.log; [ $rc -eq 0 ] || exit $rc
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$T/rows -o run -- python3 $R/tools/bench_rows.py --rows $ROWS --no-cpu > $R/gpurun_out/$T/rows.jsonl 2> $R/gpurun_out/$T/rows.err) || { tail -5 gpurun_out/$T/rows.err; exit 1; }
cut -c1-260 gpurun_out/$T/rows.jsonl
