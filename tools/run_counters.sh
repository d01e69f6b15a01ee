#!/bin/bash
# Counter passes + phase timer of the default headline kernel (tools/time_fused.py)
set -o pipefail
T=${1:-r3k}
mkdir -p gpurun_out/$T
LSHKM_LIB=$PWD/crypto-recommendation_amd/liblshkm_prof.so timeout -k 10 120 python tools/time_fused.py > gpurun_out/$T/phases.txt 2>&1 || exit 1
grep PHASES gpurun_out/$T/phases.txt | tail -1
bash tools/pmc_passes.sh $T "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE GRBM_COUNT" "TD_TD_BUSY_sum TD_TC_STALL_sum" "TCP_TCP_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_SALU"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$T/rows -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_rows.py --rows lsh,cube,kpp,f64 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/$T/rows.jsonl 2> $GRAFT_REPO_ROOT/gpurun_out/$T/rows.err) || { tail -5 gpurun_out/$T/rows.err; exit 1; }
cat gpurun_out/$T/rows.jsonl | cut -c1-250
