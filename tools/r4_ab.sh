#!/bin/bash
# Round-4 A/B on one GPU box: parity of the opt-in kernels (16-row fused form,
# wide k-means chains), then timings. tools/r4_ab.sh TAG
set -u
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
LSHKM_CSR=onepass LSHKM_F16=1 LSHKM_KM_CHAIN=16 timeout -k 10 500 python -u -m pytest tests/test_gpu_fast_dist.py tests/test_gpu_hash_assign.py \
  tests/test_gpu_update.py tests/test_gpu_f64.py tests/test_gpu_recom.py tests/test_gpu_c5.py tests/test_gpu_index.py \
  tests/test_gpu_crec.py -k "not full_size" \
  -m gpu -x -q -s --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [ $rc -eq 0 ] || { grep -E "^E |Error" "$OUT/tests.log" | head -20; exit $rc; }
LSHKM_LIB=$PWD/crypto-recommendation_amd/liblshkm_h64.so LSHKM_F16=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_fast_dist.py \
  tests/test_gpu_hash_assign.py tests/test_gpu_c5.py -k "not full_size" -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/tests_h64.log" 2>&1
rc=$?; tail -3 "$OUT/tests_h64.log"; [ $rc -eq 0 ] || { grep -E "^E |Error" "$OUT/tests_h64.log" | head -20; exit $rc; }
LSHKM_KM_PATH=seg timeout -k 10 120 python tools/time_update64.py || exit 1
LSHKM_KM_CHAIN=16 timeout -k 10 120 python tools/time_update64.py || exit 1
timeout -k 10 120 python tools/time_update64.py || exit 1
LSHKM_CSR=onepass LSHKM_KM_CHAIN=16 timeout -k 10 300 python tools/bench_rows.py --rows lsh,cube,update --no-cpu > "$OUT/rows.jsonl" 2> "$OUT/rows.err" || { tail -5 "$OUT/rows.err"; exit 1; }
cut -c1-220 "$OUT/rows.jsonl"
LSHKM_CSR=radix timeout -k 10 300 python tools/bench_rows.py --rows lsh,cube --no-cpu > "$OUT/rows_radix.jsonl" 2> "$OUT/rows_radix.err" || { tail -5 "$OUT/rows_radix.err"; exit 1; }
cut -c1-220 "$OUT/rows_radix.jsonl"
bash tools/variants.sh "${TAG}_c3" base base@LSHKM_F16=1 h64@LSHKM_F16=1 w12@LSHKM_F16=1 nt0@LSHKM_F16=1 || exit 1
TF_K=1024 bash tools/variants.sh "${TAG}_c5" base base@LSHKM_F16=1 h64@LSHKM_F16=1 w12@LSHKM_F16=1 nt0@LSHKM_F16=1 || exit 1
