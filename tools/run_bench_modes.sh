#!/bin/bash
# bench.py in the default mode and with LSHKM_DIST=fast (C3 line + C5 object), no CPU baseline
set -o pipefail
OUT=gpurun_out/${1:-r3j}
mkdir -p $OUT
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -3 $OUT/bench_default.err; exit 1; }
LSHKM_DIST=fast timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_fast.json 2> $OUT/bench_fast.err || { tail -3 $OUT/bench_fast.err; exit 1; }
python3 - $OUT <<'PY'
import json, sys
for m in ("default", "fast"):
    b = json.load(open(f"{sys.argv[1]}/bench_{m}.json"))
    c5 = b["c5"]
    print(f"{m}: C3 {b['ms_per_step']:.3f} ms/step {b['value']:.3e} pts/s kernel {b['roofline']['kernel_ms']:.3f} ms "
          f"frac {b['roofline']['frac']:.3f} | C5 {c5['ms_per_step']:.3f} ms/step kernel {c5['roofline']['kernel_ms']:.3f} ms")
PY
