set -u
OUT=gpurun_out/r4k; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_crec.py tests/test_gpu_c5.py tests/test_gpu_multirank.py tests/test_gpu_recom.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAIL" $OUT/tests.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --workload c5 --steps 5 --warmup 1 --no-cpu-baseline > $OUT/c5.json 2> $OUT/c5.err || { tail -5 $OUT/c5.err; exit 1; }
python -c "
import json; b=json.loads(open('$OUT/c5.json').read().strip().splitlines()[-1]); c=b.get('c5', b)
print(c.get('value'), c.get('ms_per_step'), json.dumps(c.get('recommend'))[:600])"
