"""bench.py's multi-rank launch on CPU: `--gpus N` starts N ranks itself (under
torch.distributed.run, before any GPU call), each rank sees WORLD_SIZE = N, and
the C5 exchange (sharding.allreduce_partials) and the max-over-ranks timing run
over gloo (--dry-run: no GPU work)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*argv):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *argv], env=env, capture_output=True,
                         text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]          # rank 0 alone prints
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [1, 2, 3])
def test_bench_spawns_ranks(n):
    res = _bench("--gpus", str(n), "--dry-run", "--steps", "2", "--warmup", "1", "--n", "1000", "--k", "64",
                 "--cpu-hash-sample", "2000", "--cpu-assign-sample", "400", "--cpu-port-hash-sample", "2000",
                 "--cpu-port-assign-sample", "400")
    assert res["dry_run"] and res["n_gpus"] == n and res["world_size"] == n and res["backend"] == "gloo"
    # rank 0 times the reference's CPU path in the same run at every N (after the final barrier)
    cb = res["cpu_baseline"]
    assert cb["value"] > 0 and cb["cores"] >= 1 and cb["kind"] in ("reference", "port"), cb
    assert "all_cores" in cb
    assert res["allreduce_ok"]
    assert [s["rank"] for s in res["shards"]] == list(range(n))
    assert sum(s["n"] for s in res["shards"]) == 1000 * n
    assert res["ms_per_step"] > 0


def test_bench_rejects_mismatched_world():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3", "--dry-run"], env=env,
                         capture_output=True, text=True, timeout=120)
    assert out.returncode != 0 and "WORLD_SIZE=2" in out.stderr
