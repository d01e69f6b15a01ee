"""CPU baseline leg of bench.py: the C restatement (oracle/_ref/liboracle.so,
-O2, OpenMP over rows) timed on a bounded sample of the headline workload.
TEST / BASELINE INFRASTRUCTURE ONLY (never the thing measured on the GPU).
The thread count comes from OMP_NUM_THREADS (set by the caller before the
library loads). Prints one JSON line.

usage: python oracle/bench_port.py HASH_ROWS ASSIGN_ROWS K SEED"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import oracle  # noqa: E402

D, L, KF, W = 128, 5, 4, 0.4


def main():
    nh, na, K, seed = (int(a) for a in sys.argv[1:5])
    X = oracle.synth(seed, max(nh, na), D)
    V, t, r, _ = oracle.gen_lsh_euclid(12345, L, KF, D, np.float32(W))
    rows = (np.arange(K) * (na // K)).astype(np.int32)
    C = X[rows].astype(np.float64)
    oracle.lib()                                          # load before timing
    t0 = time.perf_counter()
    oracle.lsh_hash_euclid(X[:nh], V, t, np.float32(W), r, max(nh // 100, 1))
    t1 = time.perf_counter()
    oracle.lloyd_assign(X[:na], C, "euclidean", rows)
    t2 = time.perf_counter()
    print(json.dumps(dict(hash_pts=nh, hash_s=t1 - t0, assign_pts=na, assign_s=t2 - t1,
                          threads=int(os.environ.get("OMP_NUM_THREADS", "0") or 0))))


if __name__ == "__main__":
    main()
