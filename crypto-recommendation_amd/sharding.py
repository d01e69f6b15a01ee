"""Row sharding of the hot path across GPUs.

The reference is single-process; the contract that makes sharding exact is the
row order: bucket members, query unions and cluster chains are all ordered by
row index. With contiguous row shards [row0, row0 + n) in rank order:
  - hashes / bucket IDs / cluster IDs are per row: no exchange;
  - an LSH query's global result (a row-sorted set) is the concatenation of the
    per-shard results in shard order;
  - a hypercube query's result is, slot by slot (main bucket, then each probe
    bucket), the concatenation of the shards' members of that bucket;
  - k-means centers need the per-cluster sums: one all-reduce of K x d fp64 sums
    and K counts (fast mode; the exact-order chain would serialize the shards).
Pure host logic (numpy + torch.distributed); the compute is the HIP library.
"""
import numpy as np


def shard_range(n_total, world, rank):
    """Contiguous, near-equal row range of `rank`: (row0, n)."""
    base, rem = divmod(n_total, world)
    row0 = rank * base + min(rank, rem)
    return row0, base + (1 if rank < rem else 0)


def centroid_rows(n_total, K):
    """Initial centroid rows i * floor(N / K) (the bench's deterministic init)."""
    return np.arange(K, dtype=np.int64) * (n_total // K)


def local_src_rows(rows, row0, n):
    """Centroid-override rows (assignment.hpp:77-78) local to a shard, -1 elsewhere."""
    rows = np.asarray(rows, np.int64)
    inside = (rows >= row0) & (rows < row0 + n)
    return np.where(inside, rows - row0, -1).astype(np.int32)


def merge_lsh_results(parts):
    """parts: per-shard (ptr, idx_local, row0) in rank order -> global (ptr, idx)."""
    nq = len(parts[0][0]) - 1
    out, ptr = [], [0]
    for q in range(nq):
        for p, idx, row0 in parts:
            out.append(idx[p[q]:p[q + 1]].astype(np.int64) + row0)
        ptr.append(ptr[-1] + sum(p[q + 1] - p[q] for p, _, _ in parts))
    idx = np.concatenate(out) if out else np.zeros(0, np.int64)
    return np.asarray(ptr, np.int64), idx


def merge_cube_results(parts, slots):
    """parts: per-shard (slot_ptr[nq * slots + 1], idx_local, row0); slot-major merge."""
    nq = (len(parts[0][0]) - 1) // slots
    out, ptr = [], [0]
    for q in range(nq):
        for s in range(slots):
            e = q * slots + s
            for sp, idx, row0 in parts:
                out.append(idx[sp[e]:sp[e + 1]].astype(np.int64) + row0)
        ptr.append(sum(len(o) for o in out))
    idx = np.concatenate(out) if out else np.zeros(0, np.int64)
    return np.asarray(ptr, np.int64), idx


def allreduce_partials(sums, counts):
    """Sum the per-shard (sums, counts) over all ranks in place (RCCL on GPUs, gloo on CPU)."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(sums)
        dist.all_reduce(counts)
    return sums, counts
