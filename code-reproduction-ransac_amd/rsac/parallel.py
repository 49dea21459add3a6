"""Multi-GPU RANSAC: one process per GPU, torch.distributed (RCCL over xGMI on ROCm).

SURVEY.md §8e.  Two ways the hot path shards, both without moving point data:

* one problem's hypothesis space (C2, C5): rank r owns a contiguous range of hypothesis
  indices.  Hypothesis i is the Philox draw (seed, i), so the set scored does not depend
  on the GPU count.
  - Fixed budget (``sharded_best``): the only exchange is an all-reduce(MAX) of the packed key
    ``count << 32 | (0xFFFFFFFF - i)``: highest count, lowest index on ties -- the same winner as
    OpenCV's sequential "first strictly greater" loop (ptsetreg.cpp run()).  The winning model is
    re-derived from its index on every rank (one P3P solve), so no model broadcast is needed.
  - Adaptive (``sharded_ransac``, OpenCV's iteration semantics): each round's {status, count}
    rows are written on the device by every rank for its chunk, all-gathered into one device
    buffer (RCCL), and every rank runs the same sequential scan over it (rsac_scan_device: the
    improvements are listed on the device, the host applies the iteration bound), so best index,
    inlier count and iteration count equal the single-GPU rsac.pnp_ransac result.  With LO the
    scan stops at each new best, every rank re-derives the model from its index on its GPU and
    runs the same deterministic local optimisation.
* independent problems (C3, the K sweep of testpro-K.py:58-75, the location loop of
  main_v1.py:274): problems are split in contiguous chunks across ranks and a single all-gather
  of the fixed-size per-problem rows ends the call.

The evaluator is injectable: ``PnPShard`` runs the HIP kernels of this package; the CPU
tests drive the same code with the gloo backend and a restatement-backed evaluator.
"""
from __future__ import annotations

import time
from dataclasses import dataclass

import numpy as np
import torch
import torch.distributed as dist

from . import api

KEY_IDX_MASK = 0xFFFFFFFF
FIRST_ROUND = 256  # the single-GPU adaptive loop's first round (rsac_api.hip run_loop)
MIN_SHARE = 256  # hypotheses per rank and sharded round, at least (one first round's worth)
COLLECTIVES = 0  # data-path collectives issued by this module (the tests count them)


def shard(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous balanced split of range(n): (begin, count) of ``rank``."""
    base, rem = divmod(int(n), int(world))
    begin = rank * base + min(rank, rem)
    return begin, base + (1 if rank < rem else 0)


def chunk(n: int, rank: int, world: int) -> tuple[int, int, int]:
    """Contiguous split of range(n) in chunks of equal width w = ceil(n / world) (the last ones
    shorter or empty), the layout of an all-gather of equal-size tensors: (begin, count, w)."""
    w = -(-int(n) // int(world)) if n > 0 else 0
    b = min(rank * w, int(n))
    return b, max(0, min(w, int(n) - b)), w


def pack_key(count: int, index: int) -> int:
    """(count << 32) | (0xFFFFFFFF - low32(index)); 0 = no model."""
    if count <= 0:
        return 0
    return (int(count) << 32) | (KEY_IDX_MASK - (int(index) & KEY_IDX_MASK))


def unpack_key(key: int) -> tuple[int, int]:
    """-> (count, hypothesis index); the index is exact below 2**32 hypotheses."""
    return int(key) >> 32, KEY_IDX_MASK - (int(key) & KEY_IDX_MASK)


def best_key_of(counts, status, begin: int) -> int:
    """Packed key of the best hypothesis among per-hypothesis (status, counts) starting at ``begin``."""
    c = np.where(np.asarray(status) > 0, np.asarray(counts, np.int64), 0)
    if c.size == 0 or c.max() <= 0:
        return 0
    i = int(np.argmax(c))  # first maximum = lowest index
    return pack_key(int(c[i]), begin + i)


def _rank_world(group):
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    return 0, 1


def _comm_device(group):
    if dist.is_available() and dist.is_initialized() and dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def all_reduce_max_key(key: int, group=None) -> int:
    """Global best packed key (all-reduce MAX of one int64; keys are < 2**63)."""
    global COLLECTIVES
    _, world = _rank_world(group)
    if world == 1:
        return int(key)
    COLLECTIVES += 1
    t = torch.tensor([int(key)], dtype=torch.int64, device=_comm_device(group))
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return int(t.item())


def all_gather_chunks(t: torch.Tensor, group=None) -> torch.Tensor:
    """All-gather of equal-size tensors (one per rank, first axis = the rank's chunk) into one
    tensor in rank order, on the tensor's device (RCCL for device tensors, no host copy)."""
    global COLLECTIVES
    _, world = _rank_world(group)
    if world == 1:
        return t
    COLLECTIVES += 1
    dev = _comm_device(group)  # a gloo rehearsal on GPU tensors goes through the host
    src = t.to(dev).contiguous()
    out = torch.empty((world * src.shape[0],) + tuple(src.shape[1:]), dtype=src.dtype, device=dev)
    dist.all_gather_into_tensor(out, src, group=group)
    return out if out.device == t.device else out.to(t.device)


class PnPShard:
    """Evaluator of one PnP problem on this rank's GPU (points uploaded once, kept resident)."""

    def __init__(self, points2D, points3D, K, reproj_thresh: float = 30.0, seed: int = 0x5EED, device=None):
        dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        self.p2 = torch.as_tensor(np.asarray(points2D, np.float64).reshape(-1, 2), device=dev)
        self.p3 = torch.as_tensor(np.asarray(points3D, np.float64).reshape(-1, 3), device=dev)
        self.K = np.asarray(K, np.float64).reshape(3, 3)
        self.thr = float(reproj_thresh)
        self.seed = int(seed)
        self.n = self.p3.shape[0]

    def range_key(self, begin: int, count: int) -> int:
        key, _ = api.evaluate_range(self.p2, self.p3, self.K, begin, count, self.thr, seed=self.seed)
        return max(int(key), 0)  # -1 = no model in the range

    def hypotheses(self, begin: int, count: int):
        st, cn, _ = api.hypotheses("pnp", self.p3, self.p2, self.K, begin, count, self.thr, seed=self.seed)
        return st, cn

    def round_rows(self, begin: int, count: int, width: int) -> torch.Tensor:
        """{status, count} int32 rows of hypotheses [begin, begin + count), padded to ``width``
        rows, on this GPU (written by the kernels, nothing waits)."""
        rows = torch.zeros((max(width, 1), 2), dtype=torch.int32, device=self.p3.device)
        if count > 0:
            api.hypothesis_rows(self.p2, self.p3, self.K, begin, count, self.thr, rows, seed=self.seed)
        return rows[:width]

    def first_round(self, max_iters: int, confidence: float, lo: bool):
        """The single-GPU adaptive loop's first round on this rank alone (rsac_pnp_ransac_first_round:
        the device's speculative finish, one synchronisation) -> (done, model12 or None, Scan,
        LO refits that raised the count)."""
        done, R, t, _, scan, info = api.pnp_ransac_first_round(self.p2, self.p3, self.K, max_iters, self.thr,
                                                               confidence=confidence, seed=self.seed, refine=False,
                                                               lo=lo)
        model = None if R is None else np.concatenate([np.asarray(R).reshape(9), np.asarray(t).reshape(3)])
        return done, model, scan, info.lo_improvements

    def model(self, index: int) -> np.ndarray:
        """(R 9 row-major, t 3) of hypothesis ``index``, re-derived on this GPU from its Philox counter."""
        key = torch.tensor([pack_key(1, index)], dtype=torch.int64, device=self.p3.device)
        m, _ = api.winner(self.p2, self.p3, self.K, key, self.thr, seed=self.seed, with_mask=False)
        return m.cpu().numpy()

    def local_opt(self, model12, count: int):
        """LO-RANSAC step on this rank's copy of the points (identical on every rank)
        -> (model12, inlier count, refits that raised it)."""
        return api.local_opt(self.p2, self.p3, self.K, model12, self.thr)

    def mask(self, model12) -> np.ndarray:
        m, _ = api.pose_mask(self.p2, self.p3, self.K, model12, self.thr)
        return np.asarray(m.cpu() if torch.is_tensor(m) else m, bool)


@dataclass
class ShardedResult:
    best: int  # global hypothesis index, -1 = no model
    n_inliers: int
    iters: int  # hypotheses consumed by the (adaptive) scan
    model: np.ndarray | None  # (R 9, t 3)
    lo_improvements: int = 0


def sharded_best(ev, n_total: int, group=None) -> ShardedResult:
    """Fixed budget (adaptive off): best of hypotheses [0, n_total) over all ranks."""
    rank, world = _rank_world(group)
    b, c = shard(n_total, rank, world)
    key = ev.range_key(b, c) if c > 0 else 0
    g = all_reduce_max_key(key, group)
    if g == 0:
        return ShardedResult(-1, 0, n_total, None)
    cnt, idx = unpack_key(g)
    return ShardedResult(idx, cnt, n_total, ev.model(idx))


def _round_rows(ev, begin: int, count: int, width: int, device) -> torch.Tensor:
    if hasattr(ev, "round_rows"):
        return ev.round_rows(begin, count, width)
    rows = torch.zeros((width, 2), dtype=torch.int32, device=device)
    if count > 0:
        st, cn = ev.hypotheses(begin, count)
        rows[:count, 0] = torch.as_tensor(np.asarray(st, np.int32))
        rows[:count, 1] = torch.as_tensor(np.asarray(cn, np.int32))
    return rows


def _scan_round(ev, scan, rows, hr: int, lo: bool, best_model, n_lo: int):
    """Scan one round's {status, count} rows (hypothesis order) -> (best_model, n_lo)."""
    if not lo:
        scan.step_rows(rows, hr)
        return best_model, n_lo
    pos = 0
    while not scan.done and pos < hr:
        pos += scan.step_rows(rows[pos:], hr - pos, stop_on_improve=True)
        if scan.improved:
            m0 = ev.model(scan.best)
            m, cnt, steps = ev.local_opt(m0, scan.max_good)
            n_lo += steps
            best_model = m if cnt > scan.max_good else m0
            scan.raise_count(cnt)
    return best_model, n_lo


def sharded_ransac(ev, max_iters: int, confidence: float = 0.99, round_size: int = 4096, group=None,
                   model_points: int = 4, lo: bool = False) -> ShardedResult:
    """Adaptive RANSAC (OpenCV iteration semantics) with each round's hypotheses split over ranks.

    Round 1 is the single-GPU loop's first round (FIRST_ROUND hypotheses), run redundantly on
    every rank with no collective (PnPShard: rsac_pnp_ransac_first_round, the device's speculative
    finish); most scans end there (C2, C5), so a multi-GPU call costs what a one-GPU call does.
    Later rounds double from max(2 FIRST_ROUND, MIN_SHARE x ranks) up to max(round_size,
    MIN_SHARE x ranks) and are split over the ranks: every rank writes the {status, count} rows
    of its chunk (on its GPU for PnPShard), one all-gather assembles the round in hypothesis order
    on every rank, and every rank scans it identically (device-listed improvements for GPU rows).
    lo=True: LO-RANSAC (BASELINE.json configs[4]); the scan stops at every new best, every rank
    runs the same (deterministic) local optimisation on its copy of the points, and the scan
    continues with the raised count -- the single-GPU rsac.pnp_ransac(lo=True) result.
    """
    rank, world = _rank_world(group)
    dev = _comm_device(group)
    best_model = None
    n_lo = 0
    if hasattr(ev, "first_round"):
        done, best_model, scan, n_lo = ev.first_round(max_iters, confidence, lo)
        if done:
            if scan.best < 0:
                return ShardedResult(-1, 0, scan.iters, None)
            return ShardedResult(scan.best, scan.max_good, scan.iters, best_model, n_lo)
    else:
        scan = api.Scan(max_iters, ev.n, confidence, model_points)
        hr = min(FIRST_ROUND, max_iters, scan.niters)
        best_model, n_lo = _scan_round(ev, scan, _round_rows(ev, 0, hr, hr, dev), hr, lo, best_model, n_lo)
    hb = scan.iters
    cur = max(2 * FIRST_ROUND, MIN_SHARE * world)
    cap = max(int(round_size), MIN_SHARE * world)
    while not scan.done and hb < max_iters:
        hr = min(cur, max_iters - hb, scan.niters - hb)
        cur = min(2 * cur, cap)
        b, c, w = chunk(hr, rank, world)
        full = all_gather_chunks(_round_rows(ev, hb + b, c, w, dev), group)  # rank order = hypothesis order
        best_model, n_lo = _scan_round(ev, scan, full, hr, lo, best_model, n_lo)
        hb += hr
    if scan.best < 0:
        return ShardedResult(-1, 0, scan.iters, None)
    model = best_model if lo else ev.model(scan.best)
    return ShardedResult(scan.best, scan.max_good, scan.iters, model, n_lo)


def sharded_batched(run_local, n_problems: int, group=None):
    """Independent problems split in contiguous chunks over ranks.

    ``run_local(begin, count)`` solves problems [begin, begin + count) on this rank and returns a
    (count, W) float64 array (numpy or a torch tensor, e.g. status, n_inliers, R 9, t 3); the
    call returns the (n_problems, W) rows of all ranks, identical on every rank (a torch tensor
    on the communication device, all-gathered without a host round trip for device rows).
    """
    rank, world = _rank_world(group)
    b, c, w = chunk(n_problems, rank, world)
    local = run_local(b, c)
    local = torch.as_tensor(local, dtype=torch.float64)
    if local.ndim != 2 or local.shape[0] != c:
        raise ValueError("run_local must return one row per problem")
    dev = _comm_device(group)
    padded = torch.zeros((max(w, 1), local.shape[1]), dtype=torch.float64, device=dev)
    padded[:c] = local.to(dev)
    return all_gather_chunks(padded[:w], group)[:n_problems]


def pnp_batched_rows(points2D, points3D, offsets, Ks, n_iters: int = 5000, reproj_thresh: float = 30.0, **kw):
    """run_local for sharded_batched over rsac.pnp_ransac_batched_rows: the problems'
    concatenated points (device tensors stay on the device) and offsets; rows (ok, n_inliers,
    R 9, t 3) written on this rank's GPU by the library, so the all-gather takes them from HBM."""
    off = np.asarray(offsets, np.int64)

    def run(begin, count):
        if count == 0:
            return torch.zeros((0, 14), dtype=torch.float64)
        o0, o1 = int(off[begin]), int(off[begin + count])
        rows, _ = api.pnp_ransac_batched_rows(points2D[o0:o1], points3D[o0:o1], off[begin:begin + count + 1] - o0,
                                              np.asarray(Ks)[begin:begin + count], n_iters, reproj_thresh, **kw)
        return rows

    return run


# ---------------------------------------------------------------------------------------------
# the multi-GPU legs of bench.py (BASELINE.json configs[2], configs[4], ms-to-best at N GPUs);
# the CPU rehearsal test drives the same functions with gloo and restatement-backed evaluators
# ---------------------------------------------------------------------------------------------
def _barrier_time(fn, group=None, sync=None):
    """fn() between barriers (+ device synchronisation); -> (result, max over ranks of the wall time)."""
    _, world = _rank_world(group)
    if world > 1:
        dist.barrier(group=group)
    if sync:
        sync()
    t = time.perf_counter()
    out = fn()
    if sync:
        sync()
    dt = time.perf_counter() - t
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=_comm_device(group))
        dist.all_reduce(tt, op=dist.ReduceOp.MAX, group=group)
        dt = float(tt.item())
    return out, dt


def c3_problem_shards(run_local, n_problems: int, group=None, sync=None, repeats: int = 3):
    """C3 across the ranks: problem chunks solved locally, one all-gather of the rows.
    -> (rows (n_problems, W) on the comm device, median wall seconds over `repeats`, max over ranks)."""
    walls = []
    rows = None
    for _ in range(max(1, repeats)):
        rows, dt = _barrier_time(lambda: sharded_batched(run_local, n_problems, group), group, sync)
        walls.append(dt)
    return rows, float(np.median(walls))


def adaptive_shards(ev, max_iters: int, confidence: float = 0.99, round_size: int = 4096, lo: bool = False,
                    group=None, sync=None, repeats: int = 3):
    """C5 (lo=True) / ms-to-best (lo=False) across the ranks with sharded_ransac.
    -> (ShardedResult, median wall seconds, max over ranks)."""
    walls = []
    res = None
    for _ in range(max(1, repeats)):
        res, dt = _barrier_time(lambda: sharded_ransac(ev, max_iters, confidence, round_size, group, lo=lo), group,
                                sync)
        walls.append(dt)
    return res, float(np.median(walls))


def comm_report(n_problems: int = 0, n_hyps: int = 0, group=None, sync=None, samples: int = 50) -> dict:
    """What an N > 1 bench line needs to describe itself: the process-group backend
    (nccl = RCCL), the world size the backend reports, the median latency of an 8-byte (one int64)
    all-reduce(MAX) -- the exchange of the hypothesis-shard and adaptive paths -- over `samples`
    timed calls after 5 untimed ones (each synchronised, max over ranks), and every rank's share:
    its C3-style problem chunk (chunk(), the all-gather layout) and its hypothesis shard
    (shard())."""
    rank, world = _rank_world(group)
    backend = dist.get_backend(group) if (dist.is_available() and dist.is_initialized()) else "none"
    dev = _comm_device(group)
    t = torch.zeros(1, dtype=torch.int64, device=dev)
    lat = []
    for i in range(5 + max(1, samples)):
        if world > 1:
            dist.barrier(group=group)
        if sync:
            sync()
        t0 = time.perf_counter()
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        if sync:
            sync()
        dt = time.perf_counter() - t0
        if i >= 5:
            lat.append(dt)
    us = float(np.median(lat)) * 1e6
    if world > 1:
        tt = torch.tensor([us], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX, group=group)
        us = float(tt.item())
    return {"backend": backend, "world_size": world, "rank": rank, "allreduce_8b_us": us,
            "allreduce_samples": max(1, samples),
            "problem_shares": [list(chunk(n_problems, r, world)[:2]) for r in range(world)],
            "hypothesis_shares": [list(shard(n_hyps, r, world)) for r in range(world)]}
