"""Row sharding of the hot path across GPUs.

The reference is single-process; the contract that makes sharding exact is the
row order: bucket members, query unions and cluster chains are all ordered by
row index. With contiguous row shards [row0, row0 + n) in rank order:
  - hashes / bucket IDs / cluster IDs are per row: no exchange;
  - an LSH query's global result (a row-sorted set) is the concatenation of the
    per-shard results in shard order;
  - a hypercube query's result is, slot by slot (main bucket, then each probe
    bucket), the concatenation of the shards' members of that bucket;
  - k-means centers need the per-cluster sums, which the reference forms as ONE
    sequential chain per (cluster, dim) in row order: kmeans_sums_sharded gets
    that chain's value bit for bit from one all-gather of the K x d partial sums
    plus three all-reduces, wherever the chain provably never rounds (the global
    never-rounds test), and carries only the other chains rank to rank.
Host logic (numpy + torch.distributed); the compute is the HIP library.
Collectives: RCCL ("nccl") on GPU tensors; with the gloo backend (CPU tests,
or several ranks sharing one GPU) device tensors are staged through host
memory, since gloo's collectives run on host buffers.
"""
import numpy as np


def _dist():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        return dist
    return None


def _staged(dist, t):
    """(buffer the collective runs on, copy-back) for tensor t."""
    if t.is_cuda and dist.get_backend() == "gloo":
        h = t.cpu()
        return h, (lambda: t.copy_(h))
    return t, (lambda: None)


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


def merge_unseen(parts, k):
    """Global first-occurrence order of the EuclideanF coins.

    parts: per shard, in shard order, (f, h, global_first_row) arrays. Each
    (f, h) is kept at its smallest global key row * k + f -- the order in which
    the reference's single pass over the rows (HypercubeGen::generate, f = 0..k-1
    per row) first meets it -- and the entries come back sorted by that key."""
    if not parts:
        return (np.zeros(0, np.int32),) * 2
    f = np.concatenate([np.asarray(p[0], np.int64) for p in parts])
    h = np.concatenate([np.asarray(p[1], np.int64) for p in parts])
    key = np.concatenate([np.asarray(p[2], np.int64) for p in parts]) * k + f
    order = np.lexsort((key, h, f))                 # by (f, h), then key
    f, h, key = f[order], h[order], key[order]
    first = np.ones(len(f), bool)
    first[1:] = (f[1:] != f[:-1]) | (h[1:] != h[:-1])
    f, h, key = f[first], h[first], key[first]
    by_key = np.argsort(key, kind="stable")
    return f[by_key].astype(np.int32), h[by_key].astype(np.int32)


def cube_build_sharded(lk, cube, X_local, row0):
    """Build this rank's part of a euclidean hypercube with the coins the
    reference would draw over all ranks' rows in order: export the unseen
    (f, h), all-gather, merge in global first-occurrence order, draw on the
    host (identically on every rank), import, build. One KB-sized exchange."""
    import torch.distributed as dist
    f, h, r = cube.unseen(X_local)
    mine = (f, h, np.asarray(r, np.int64) + row0)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        parts = [None] * dist.get_world_size()
        dist.all_gather_object(parts, mine)
    else:
        parts = [mine]
    fs, hs = merge_unseen(parts, cube.k)
    state = cube.memo()[3]
    bits, state = lk.coins_draw(state, hs)
    cube.import_coins(fs, hs, bits, state)
    cube.build(X_local)


def chain_partials(local_fn, sums_like, counts_like):
    """Exact-order sharded k-means sums (SURVEY §8e "exact mode").

    Rank r receives the running (sums, counts) of rows [0, row0_r) from rank
    r-1, continues every per-(c, j) chain over its own rows in row order
    (``local_fn(carry_sums, carry_counts) -> (sums, counts)``, e.g.
    ``lshkm.kmeans_partial_carry``; the carry is None on rank 0), and hands the
    result to rank r+1: the reference's single sequential sum (update.hpp:45-58)
    bit for bit. The last rank broadcasts the totals. ``sums_like`` /
    ``counts_like`` are receive buffers of the right shape, dtype and device.
    Point-to-point hops of K*d*8 bytes (1 MiB at K=1024, d=128) over RCCL/xGMI."""
    dist = _dist()
    if dist is None:
        return local_fn(None, None)
    rank, world = dist.get_rank(), dist.get_world_size()

    def xfer(op, t, peer):
        b, back = _staged(dist, t)
        if op == "recv":
            dist.recv(b, src=peer)
            back()
        elif op == "send":
            dist.send(b, dst=peer)
        else:
            dist.broadcast(b, src=peer)
            back()

    carry_s = carry_c = None
    if rank > 0:
        carry_s, carry_c = sums_like, counts_like
        xfer("recv", carry_s, rank - 1)
        xfer("recv", carry_c, rank - 1)
    sums, counts = local_fn(carry_s, carry_c)
    if rank + 1 < world:
        xfer("send", sums, rank + 1)
        xfer("send", counts, rank + 1)
        sums, counts = sums_like, counts_like
    xfer("bcast", sums, world - 1)
    xfer("bcast", counts, world - 1)
    return sums, counts


def _all_gather_rows(dist, t):
    """[world, *t.shape] tensor of every rank's t, in rank order, on t's device."""
    world = dist.get_world_size()
    if t.is_cuda and dist.get_backend() != "gloo":
        out = t.new_empty((world,) + tuple(t.shape))
        dist.all_gather_into_tensor(out, t.contiguous())
        return out
    h = t.cpu()
    parts = [h.new_empty(h.shape) for _ in range(world)]
    dist.all_gather(parts, h)
    import torch
    return torch.stack(parts).to(t.device)


def kmeans_sums_sharded(ops, timing=None):
    """The reference's k-means sums (update.hpp:45-58: one sequential fp64 chain
    per (cluster, dim) over ALL rows in row order) from row shards, bit for bit,
    at all-reduce cost (lshkm_kmeans_shard_*, include/lshkm.h):
      1. ops.begin(): this rank's partial sums (any order), sums of |x|, the
         values' lowest / top bit positions, counts;
      2. all-gather the partial sums; all-reduce |x| sums and counts (SUM) and
         the bit positions (MIN) -- 1 + 3 collectives of ~K*d*8 bytes;
      3. ops.certify(): the never-rounds test on the GLOBAL values. Where it
         holds (every chain of the 2^-15-grid bench data; ~95 % of the chains of
         10K N(0,1) fp32 values), any order of fp64 adds is exact: the gathered
         partials' total IS the chain. The rest are flagged, identically on
         every rank;
      4. only if some chain is flagged: ops.prepare() forms their segment
         records on every rank at once, then ops.chain() composes them in rank
         order from the previous rank's running sums (point-to-point), and the
         last rank broadcasts the result.
    ops: lshkm.ShardSums (or a restatement with the same methods). Returns
    (sums, counts): the chains' values and the global counts, on every rank.
    timing: optional dict that receives the flagged-chain count."""
    dist = _dist()
    world, rank = (dist.get_world_size(), dist.get_rank()) if dist is not None else (1, 0)
    sums, asum, qt, counts = ops.begin()
    if dist is not None:
        gathered = _all_gather_rows(dist, sums)
        for t, op in ((asum, dist.ReduceOp.SUM), (counts, dist.ReduceOp.SUM), (qt, dist.ReduceOp.MIN)):
            b, back = _staged(dist, t)
            dist.all_reduce(b, op=op)
            back()
    else:
        gathered = sums.reshape((1,) + tuple(sums.shape))
    out, start, flag, mask, n_flagged = ops.certify(gathered, asum, qt, counts, world, rank)
    if timing is not None:
        timing["flagged"] = n_flagged
    if n_flagged:
        ops.prepare(start, flag, mask)      # carry-free: every rank at once
        carry = None
        if rank > 0:
            carry = ops.empty(tuple(out.shape), out.dtype)
            b, back = _staged(dist, carry)
            dist.recv(b, src=rank - 1)
            back()
        ops.chain(flag, mask, carry, out)
        if dist is not None:
            if rank + 1 < world:
                b, _ = _staged(dist, out)
                dist.send(b, dst=rank + 1)
            b, back = _staged(dist, out)
            dist.broadcast(b, src=world - 1)
            back()
    return out, counts


def allreduce_partials(sums, counts):
    """Sum the per-shard (sums, counts) over all ranks in place (RCCL on GPUs, gloo on CPU)."""
    dist = _dist()
    if dist is not None:
        for t in (sums, counts):
            b, back = _staged(dist, t)
            dist.all_reduce(b)
            back()
    return sums, counts


def recommend_terms(lk, ctx, X, x_mean, assign, K, U, u_mean, ucl, unk_ptr, unk_idx, csr=None):
    """Phase 1 of recommend_sharded (steps 1-2 below): this rank's similarities
    and prediction terms, all ranks at once. Returns the state recommend_chain
    continues from."""
    crow, crows = csr if csr is not None else lk.clusters(ctx, assign, K)
    # the terms form stages rows of <= 1016 B in 8-B units (lshkm_cluster_terms):
    # other rows (fp32 of odd d, fp64 of d >= 128) take the sims form, the same
    # rank-to-rank chain over lshkm_cluster_sims + lshkm_cluster_chain
    rb = X.shape[1] * X.element_size()
    if rb % 8 == 0 and rb <= 1016:
        soff, toff, sims, terms = lk.cluster_terms(ctx, X, x_mean, crow, crows, U, ucl, unk_ptr, unk_idx)
        return (lk.cluster_chain_terms, (ctx, u_mean, unk_ptr, unk_idx, soff, toff, sims, terms), ucl, unk_idx)
    soff, sims = lk.cluster_sims(ctx, X, crow, crows, U, ucl, unk_ptr)
    return (lk.cluster_chain, (ctx, X, x_mean, crow, crows, ucl, u_mean, unk_ptr, unk_idx, soff, sims), ucl, unk_idx)


def recommend_chain(ctx, state, n_top):
    """Phase 2 of recommend_sharded (step 3 below): the prediction sums carried
    rank to rank from recommend_terms' state; the result on every rank."""
    torch = ctx.torch
    chain, args, ucl, unk_idx = state
    dist = _dist()
    if dist is None:
        return chain(*args, carry=None, n_top=n_top)
    rank, world = dist.get_rank(), dist.get_world_size()
    nq, M = ucl.shape[0], unk_idx.shape[0]
    carry = None
    if rank > 0:
        carry = (ctx.empty((max(M, 1),), torch.float64), ctx.empty((nq,), torch.float64),
                 ctx.empty((nq,), torch.int64))
        for t in carry:
            b, back = _staged(dist, t)
            dist.recv(b, src=rank - 1)
            back()
    if rank + 1 < world:
        outs = chain(*args, carry=carry, n_top=None)
        for t in outs:
            b, _ = _staged(dist, t)
            dist.send(b, dst=rank + 1)
        out = ctx.empty((nq, n_top), torch.int32)
    else:
        out = chain(*args, carry=carry, n_top=n_top)
    b, back = _staged(dist, out)
    dist.broadcast(b, src=world - 1)
    back()
    return out


def recommend_sharded(lk, ctx, X, x_mean, assign, K, U, u_mean, ucl, unk_ptr, unk_idx, n_top, timing=None, csr=None):
    """The clustering recommender over row shards (main.cpp:260-269 on the
    sharded rows; get_top_N_recom's 3-argument overload, crypto_rec.hpp:327-345).

    A cluster's members lie on every rank, in row order = rank order, and the
    reference sums get_predicted_user_sim's terms over them in that order. Every
    rank holds the same query users (U rows, u_mean, their global clusters ucl,
    the unknown-index CSR) and its own rows (X, x_mean, assign):
      1. lshkm_clusters of the local assignment -> the local cluster CSR;
      2. lshkm_cluster_terms: every user's similarities to the local members of
         its cluster and its prediction terms sim * (x[index] - mean) -- the
         bulk of the work, all ranks at once;
      3. lshkm_cluster_chain_terms in rank order: rank r receives the running sums
         (one fp64 per (user, unknown index) + |sim| sum + member count per user)
         from rank r-1 over RCCL point-to-point, continues them over its
         members, and sends them on; the last rank finalizes (quicksort, first
         n_top) and broadcasts the [nq][n_top] result.
    Bit for bit lshkm_cluster_top_n over the concatenated rows. Returns the
    result on every rank (device tensor). timing: optional list that receives
    (ms of phases 1, 2+3) from CUDA events. csr: (crow, crows) of this
    assignment when the caller built it already (ShardedLloyd's sums)."""
    torch = ctx.torch
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)] if timing is not None else None
    if ev:
        ev[0].record()
    state = recommend_terms(lk, ctx, X, x_mean, assign, K, U, u_mean, ucl, unk_ptr, unk_idx, csr=csr)
    if ev:
        ev[1].record()
    out = recommend_chain(ctx, state, n_top)
    if ev:
        ev[2].record()
        torch.cuda.synchronize(ctx.dev)
        timing.append((ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2])))
    return out


def synth_recom_users(ctx, n_total, Q, d, seed):
    """The C5 recommend step's query users (bench / tests): Q rows spread over
    the whole job (rows i * floor(N / Q)), their known means (0: synthetic rows
    carry no ratings) and unknown sets {j : (7j + row) % 16 == 0}. Returns
    (rows numpy, U, u_mean, unk_ptr, unk_idx) device tensors, equal on every rank."""
    torch = ctx.torch
    rows = np.arange(Q, dtype=np.int64) * (n_total // Q)
    U = torch.stack([ctx.synth(seed, 1, d, row0=int(r))[0] for r in rows])
    u_mean = torch.zeros((Q,), dtype=torch.float64, device=ctx.dev)
    sets = [np.nonzero((7 * np.arange(d) + int(r)) % 16 == 0)[0].astype(np.int32) for r in rows]
    unk_ptr = torch.from_numpy(np.cumsum([0] + [len(s) for s in sets]).astype(np.int64)).to(ctx.dev)
    unk_idx = torch.from_numpy(np.concatenate(sets)).to(ctx.dev)
    return rows, U, u_mean, unk_ptr, unk_idx


def user_cluster_index(ctx, rows, row0, n):
    """(positions, local rows) of the users this rank owns, device tensors (or
    None when it owns none): user_clusters' gather, formed once per user set."""
    mine = (rows >= row0) & (rows < row0 + n)
    if not mine.any():
        return None
    torch = ctx.torch
    return (torch.from_numpy(np.nonzero(mine)[0]).to(ctx.dev),
            torch.from_numpy(rows[mine] - row0).to(ctx.dev))


def user_clusters(ctx, rows, assign_local, row0, n, index=False):
    """The users' clusters (main.cpp:261: user.getCluster()): the owning rank's
    assignment of each user row, all-reduced (one int32 per user). index: a
    user_cluster_index result for these rows (False: formed here)."""
    torch = ctx.torch
    Q = len(rows)
    if index is False:
        index = user_cluster_index(ctx, rows, row0, n)
    dist = _dist()
    if dist is None and index is not None and index[0].numel() == Q:
        return assign_local.index_select(0, index[1])        # every user local: one gather
    ucl = torch.zeros((Q,), dtype=torch.int32, device=ctx.dev)
    if index is not None:
        ucl[index[0]] = assign_local[index[1]]
    if dist is not None:
        b, back = _staged(dist, ucl)
        dist.all_reduce(b)
        back()
    return ucl


class ShardedLloyd:
    """One rank's part of the C5 iteration (main.cpp:96-103 with
    LSH hashing riding on the assignment pass): per step, on the rank's
    resident rows,
      lshkm_hash_assign   -- L x k hashes + bucket IDs + argmin over K centroids
      lshkm_clusters      -- the cluster CSR (shared with the recommend step)
      the k-means sums    -- mode "certified" (default): kmeans_sums_sharded,
        the reference's chains bit for bit at all-reduce cost over RCCL; mode
        "carry": every chain carried rank to rank (lshkm_kmeans_partial_carry,
        the shards' updates in series; kept as the cross-check)
      lshkm_kmeans_finalize -- means, the reference's continue test
    and the centers are replaced when k_means would replace them
    (update.hpp:63-80). X: this rank's rows [row0, row0 + n) of N_total."""

    MODES = ("certified", "carry")

    def __init__(self, lk, ctx, lsh, X, C0, src_rows, mode="certified", metric="euclidean", min_dist=0.0):
        torch = ctx.torch
        self.lk, self.ctx, self.lsh, self.X = lk, ctx, lsh, X
        if mode not in self.MODES:
            raise ValueError(f"unknown mode {mode!r} (one of {self.MODES})")
        self.mode, self.metric, self.min_dist = mode, metric, float(min_dist)
        n = X.shape[0]
        self.K, self.d = C0.shape
        self.C = C0.clone()
        self.src = None if src_rows is None else np.ascontiguousarray(src_rows, np.int32)
        e = ctx.empty
        if metric not in lk._METRIC:
            raise ValueError(f"unknown metric {metric!r}")
        # cosine indexes have no k-tuples (CosineGGen, cosine_g_gen.hpp:58-66)
        self.tuples = e((n, lsh.L, lsh.k), torch.int32) if lsh is not None and lsh.metric == lk.EUCLIDEAN else None
        self.bucket = e((n, lsh.L), torch.int32) if lsh is not None else None
        self.assign = e((n,), torch.int32)
        self.dist = e((n,), torch.float64)
        self.sums = e((self.K, self.d), torch.float64)
        self.counts = e((self.K,), torch.int64)
        self.cont = True
        self.timing = False       # True: HIP events around the sums + exchange (bench.py's breakdown)
        self.flagged = 0          # chains the last step's global never-rounds test flagged
        self.exchange_events = []
        self.recom = None         # enable_recommend(): the C5 recommend step after each update
        self.csr = None           # (crow, crows) of this iteration's assignment (recommend runs)
        self._rstream = None      # device rows: the recommend phase's stream (enable_recommend)
        self.rctx = None
        self._rs_pending = False  # recommend work on that stream not yet joined into torch's
        self._recom_out = None
        self._recom_ucl = None

    def step(self):
        import ctypes as C
        lk, ctx, X = self.lk, self.ctx, self.X
        p = lk._t_ptr
        src = None if self.src is None else self.src.ctypes.data_as(C.c_void_p)
        if self.lsh is not None:
            # the assignment metric is this iteration's (an index of either family
            # may ride along; the cosine index + cosine Lloyd is one pass)
            lk._ck(lk._fn("lshkm_hash_assign_metric", X)(self.lsh.h, p(X), X.shape[0], p(self.C), self.K,
                                                         lk._METRIC[self.metric], src,
                                                         p(self.tuples) if self.tuples is not None else None,
                                                         None, p(self.bucket), p(self.assign), p(self.dist)))
        else:
            lk.lloyd_assign(ctx, X, self.C, self.metric, self.src, self.assign, self.dist)
        # the previous step's recommend chain ran beside this assignment (it
        # reads none of its outputs); everything after waits for it
        self._join_recommend()
        # the recommend phase on its own stream (device rows): its similarities
        # and terms depend only on this assignment, so they run beside the
        # k-means sums, and each phase's host synchronisations wait for its own
        # stream only; the chain follows the finalize, and the stream joins
        # torch's before the step returns (host order keeps the ranks'
        # collectives in one order)
        rs = self._rstream if self.recom is not None else None
        rstate = None
        # the cluster CSR of this assignment serves the sums and the recommender
        self.csr = lk.clusters(ctx, self.assign, self.K) if self.mode != "carry" or self.recom is not None else None
        if rs is not None:
            torch = ctx.torch
            rs.wait_stream(torch.cuda.current_stream(ctx.dev))
            with torch.cuda.stream(rs):
                rstate = self._recommend_begin()
        if self.mode == "carry":
            def local(cs, cc):
                return lk.kmeans_partial_carry(ctx, X, self.assign, self.K, cs, cc)
            sums, counts = chain_partials(local, self.sums, self.counts)
        else:
            if self.timing:
                ev = [ctx.torch.cuda.Event(enable_timing=True) for _ in range(2)]
                ev[0].record()
            info = {}
            sums, counts = kmeans_sums_sharded(lk.ShardSums(ctx, X, self.csr, self.K), timing=info)
            self.flagged = info.get("flagged", 0)
            if self.timing:
                ev[1].record()
                self.exchange_events.append(ev)
        self.last_sums, self.last_counts = sums, counts     # this iteration's totals (either mode)
        Cn, cont = lk.kmeans_finalize(ctx, sums, counts, self.C, self.metric, self.min_dist)
        if cont:              # k_means replaces every center (update.hpp:70-79)
            self.C = Cn
            self.src = None   # the override applies to dataset-row centroids only
        self.cont = cont
        if rs is not None:
            torch = ctx.torch
            with torch.cuda.stream(rs):
                self._recommend_end(rstate)
            # joined by the next step after its assignment is enqueued, or by
            # the first read of recom_out / recom_ucl
            self._rs_pending = True
        elif self.recom is not None:
            self.recommend()
        return cont

    def enable_recommend(self, n_total, row0, Q, n_top=5, seed=0x5EED, x_mean=None):
        """Add the "k-means recommend" step of C5 (BASELINE configs[4]) to every
        iteration: Q query users spread over the whole job (synth_recom_users)
        get get_top_N_recom over their whole clusters (recommend_sharded). The
        users' clusters are this iteration's assignment (main.cpp:261)."""
        torch = self.ctx.torch
        n = self.X.shape[0]
        if x_mean is None:
            x_mean = torch.zeros((n,), dtype=torch.float64, device=self.ctx.dev)
        rows, U, um, up, ui = synth_recom_users(self.ctx, n_total, Q, self.d, seed)
        self.recom = dict(row0=row0, n_top=n_top, x_mean=x_mean, rows=rows, U=U, u_mean=um, unk_ptr=up, unk_idx=ui,
                          index=user_cluster_index(self.ctx, rows, row0, n))
        if self.X.is_cuda and self._rstream is None:
            # the recommend phase's stream and a library context on it (its own
            # workspaces: the two phases run at once)
            import ctypes as C
            self._rstream = torch.cuda.Stream(device=self.ctx.dev)
            self.rctx = self.lk.Context(self.ctx.device, use_torch_stream=False)
            self.lk._ck(self.lk.lib().lshkm_ctx_set_stream(self.rctx.h, C.c_void_p(self._rstream.cuda_stream)))
        self.recom_out = None
        self.recom_ucl = None
        self.recom_timing = None      # a list: (phase-1 ms, phase-2 ms) per step

    def _join_recommend(self):
        if self._rs_pending:
            self.ctx.torch.cuda.current_stream(self.ctx.dev).wait_stream(self._rstream)
            self._rs_pending = False

    @property
    def recom_out(self):
        """The last step's recommendations ([Q][n_top] int32, device)."""
        self._join_recommend()
        return self._recom_out

    @recom_out.setter
    def recom_out(self, v):
        self._recom_out = v

    @property
    def recom_ucl(self):
        """The last step's users' clusters (int32, device)."""
        self._join_recommend()
        return self._recom_ucl

    @recom_ucl.setter
    def recom_ucl(self, v):
        self._recom_ucl = v

    def _recommend_begin(self):
        """The users' clusters and phase 1 (recommend_terms) on the recommend
        stream; returns the state _recommend_end continues."""
        r, torch = self.recom, self.ctx.torch
        ev = None
        if self.recom_timing is not None:
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            ev[0].record()
        ucl = user_clusters(self.ctx, r["rows"], self.assign, r["row0"], self.X.shape[0], index=r["index"])
        self.recom_ucl = ucl
        state = recommend_terms(self.lk, self.rctx, self.X, r["x_mean"], self.assign, self.K, r["U"], r["u_mean"], ucl,
                                r["unk_ptr"], r["unk_idx"], csr=self.csr)
        if ev:
            ev[1].record()
        return state, ev

    def _recommend_end(self, begun):
        state, ev = begun
        self.recom_out = recommend_chain(self.rctx, state, self.recom["n_top"])
        if ev:
            ev[2].record()
            ev[2].synchronize()
            self.recom_timing.append((ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2])))

    def recommend(self):
        r = self.recom
        ucl = user_clusters(self.ctx, r["rows"], self.assign, r["row0"], self.X.shape[0], index=r["index"])
        self.recom_ucl = ucl
        self.recom_out = recommend_sharded(self.lk, self.ctx, self.X, r["x_mean"], self.assign, self.K, r["U"],
                                           r["u_mean"], ucl, r["unk_ptr"], r["unk_idx"], r["n_top"],
                                           timing=self.recom_timing, csr=getattr(self, "csr", None))
        return self.recom_out

    def exchange_ms(self):
        """Mean time (ms) of the sums and their exchange (kmeans_sums_sharded)
        over the timed steps (torch's stream, which the library context and RCCL
        share), then forget them."""
        if not self.exchange_events:
            return None
        self.ctx.torch.cuda.synchronize(self.ctx.dev)
        ms = sum(a.elapsed_time(b) for a, b in self.exchange_events) / len(self.exchange_events)
        self.exchange_events = []
        return ms
