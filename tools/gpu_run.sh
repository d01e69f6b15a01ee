#!/bin/bash
# GPU-box routine (run through gpurun from the repo root):
#   tools/gpu_run.sh TAG [tests|smoke|bench|benchq|prof|pmc|pmc5|prof5|sq|sq5|rows]...
# Each GPU step has its own time limit; the script stops at the first failure.
set -u
TAG=${1:?tag}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
for step in "$@"; do
  case $step in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
      rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || { echo "tests rc=$rc"; exit $rc; } ;;
    pyt)
      # a subset: TESTS="tests/test_a.py tests/test_b.py::name" tools/gpu_run.sh TAG pyt
      timeout -k 10 900 python -u -m pytest ${TESTS:?TESTS} -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pyt.log" 2>&1
      rc=$?; tail -3 "$OUT/pyt.log"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" "$OUT/pyt.log" | head -20; echo "pyt rc=$rc"; exit $rc; } ;;
    profn)
      # kernel stats of the C3 step and the C5 iteration on full-mantissa rows
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
         -d "$OUT/profn" -o run -- python3 "$R/bench.py" --data normal --steps 5 --warmup 2 --no-cpu-baseline \
         --no-exact-dist-line > "$OUT/bench_profn.json" 2> "$OUT/bench_profn.err")
      rc=$?; echo "profn rc=$rc"; [ $rc -eq 0 ] || exit $rc
      find "$OUT/profn" -name '*kernel_stats.csv' -exec head -14 {} \; ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
      rc=$?; tail -2 "$OUT/smoke.log"; [ $rc -eq 0 ] || { echo "smoke rc=$rc"; exit $rc; } ;;
    bench)
      timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
      rc=$?; cat "$OUT/bench.json"; [ $rc -eq 0 ] || { tail -5 "$OUT/bench.err"; exit $rc; } ;;
    benchq)
      timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err"
      rc=$?; cat "$OUT/bench.json"; [ $rc -eq 0 ] || { tail -5 "$OUT/bench.err"; exit $rc; } ;;
    prof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
         -d "$OUT/prof" -o run -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-c5 --no-normal-leg \
         > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err")
      rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
      find "$OUT/prof" -name '*kernel_stats.csv' -exec head -8 {} \; ;;
    pmc)
      for c in FETCH_SIZE WRITE_SIZE; do
        (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --pmc $c --output-format csv \
           -d "$OUT/pmc_$c" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-c5 --no-exact-dist-line --no-normal-leg \
           > "$OUT/pmc_$c.json" 2> "$OUT/pmc_$c.err")
        rc=$?; echo "pmc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
      done ;;
    pmc5)
      for c in FETCH_SIZE WRITE_SIZE; do
        (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --pmc $c --output-format csv \
           -d "$OUT/c5/pmc_$c" -o run -- python3 "$R/bench.py" --workload c5 --steps 2 --warmup 1 --no-cpu-baseline \
           > "$OUT/c5_pmc_$c.json" 2> "$OUT/c5_pmc_$c.err")
        rc=$?; echo "pmc5 $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
      done ;;
    prof5)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
         -d "$OUT/prof5" -o run -- python3 "$R/bench.py" --workload c5 --steps 5 --warmup 1 --no-cpu-baseline \
         > "$OUT/bench_prof5.json" 2> "$OUT/bench_prof5.err")
      rc=$?; echo "prof5 rc=$rc"; [ $rc -eq 0 ] || exit $rc ;;
    sq)
      i=0
      for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES" \
                 "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_SALU"; do
        i=$((i+1))
        (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --pmc $set --output-format csv \
           -d "$OUT/sq$i" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-c5 --no-exact-dist-line --no-normal-leg \
           > "$OUT/sq$i.json" 2> "$OUT/sq$i.err")
        rc=$?; echo "sq pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
      done ;;
    sq5)
      i=0
      for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES" \
                 "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_SALU"; do
        i=$((i+1))
        (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --pmc $set --output-format csv \
           -d "$OUT/c5sq$i" -o run -- python3 "$R/bench.py" --workload c5 --steps 2 --warmup 1 --no-cpu-baseline \
           > "$OUT/c5sq$i.json" 2> "$OUT/c5sq$i.err")
        rc=$?; echo "sq5 pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
      done ;;
    rows)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 1000 rocprofv3 --kernel-trace --stats --output-format csv \
         -d "$OUT/rows_prof" -o run -- python3 "$R/tools/bench_rows.py" \
         > "$OUT/rows.jsonl" 2> "$OUT/rows.err")
      rc=$?; echo "rows rc=$rc"; cat "$OUT/rows.jsonl"; [ $rc -eq 0 ] || { tail -5 "$OUT/rows.err"; exit $rc; } ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
