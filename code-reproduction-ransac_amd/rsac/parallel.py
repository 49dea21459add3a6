"""Multi-GPU RANSAC: one process per GPU, torch.distributed (RCCL over xGMI on ROCm).

SURVEY.md §8e.  Two ways the hot path shards, both without moving point data:

* one problem's hypothesis space (C2, C5): rank r owns a contiguous range of hypothesis
  indices.  Hypothesis i is the Philox draw (seed, i), so the set scored does not depend
  on the GPU count.  The only exchange is an all-reduce(MAX) of the packed key
  ``count << 32 | (0xFFFFFFFF - i)``: highest count, lowest index on ties -- the same
  winner as OpenCV's sequential "first strictly greater" loop (ptsetreg.cpp run()).  The
  winning model is re-derived from its index on every rank (one P3P solve), so no model
  broadcast is needed.
* independent problems (C3, the K sweep of testpro-K.py:58-75, the location loop of
  main_v1.py:274): problems are split contiguously across ranks and a single all-gather
  of the fixed-size per-problem results ends the call.

The adaptive loop (``sharded_ransac``) keeps OpenCV's iteration-count semantics exactly:
each round's per-hypothesis counts are gathered from every rank and every rank runs the
same sequential scan (rsac_scan), so best index, inlier count and iteration count equal
the single-GPU rsac.pnp_ransac result for the same seed.

The evaluator is injectable: ``PnPShard`` runs the HIP kernels of this package; the CPU
tests drive the same code with the gloo backend and a restatement-backed evaluator.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch
import torch.distributed as dist

from . import api

KEY_IDX_MASK = 0xFFFFFFFF


def shard(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous balanced split of range(n): (begin, count) of ``rank``."""
    base, rem = divmod(int(n), int(world))
    begin = rank * base + min(rank, rem)
    return begin, base + (1 if rank < rem else 0)


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
    if dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def all_reduce_max_key(key: int, group=None) -> int:
    """Global best packed key (all-reduce MAX of one int64; keys are < 2**63)."""
    _, world = _rank_world(group)
    if world == 1:
        return int(key)
    t = torch.tensor([int(key)], dtype=torch.int64, device=_comm_device(group))
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return int(t.item())


def _all_gather_rows(arr: np.ndarray, group) -> list[np.ndarray]:
    """All-gather of a ragged first axis (pads to the longest, one collective for sizes + one for data)."""
    _, world = _rank_world(group)
    if world == 1:
        return [arr]
    dev = _comm_device(group)
    n = torch.tensor([arr.shape[0]], dtype=torch.int64, device=dev)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(s.item()) for s in sizes]
    m = max(sizes)
    pad = np.zeros((m,) + arr.shape[1:], arr.dtype)
    pad[:arr.shape[0]] = arr
    t = torch.from_numpy(pad).to(dev)
    outs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(outs, t, group=group)
    return [o.cpu().numpy()[:s] for o, s in zip(outs, sizes)]


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

    def model(self, index: int) -> np.ndarray:
        """(R 9 row-major, t 3) of hypothesis ``index``, re-derived from its Philox counter."""
        _, _, m = api.hypotheses("pnp", self.p3, self.p2, self.K, index, 1, self.thr, seed=self.seed)
        return m[0, :12].copy()

    def local_opt(self, model12, count: int):
        """LO-RANSAC step on this rank's copy of the points (identical on every rank)."""
        m, c, _ = api.local_opt(self.p2, self.p3, self.K, model12, self.thr)
        return m, c

    def mask(self, model12) -> np.ndarray:
        m, _ = api.pose_mask(self.p2, self.p3, self.K, model12, self.thr)
        return np.asarray(m.cpu() if torch.is_tensor(m) else m, bool)


@dataclass
class ShardedResult:
    best: int  # global hypothesis index, -1 = no model
    n_inliers: int
    iters: int  # hypotheses consumed by the (adaptive) scan
    model: np.ndarray | None  # (R 9, t 3)


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


def sharded_ransac(ev, max_iters: int, confidence: float = 0.99, round_size: int = 4096, group=None,
                   model_points: int = 4, lo: bool = False) -> ShardedResult:
    """Adaptive RANSAC (OpenCV iteration semantics) with each round's hypotheses split over ranks.

    lo=True: LO-RANSAC (BASELINE.json configs[4]); the scan stops at every new best, every rank
    runs the same (deterministic) local optimisation on its copy of the points, and the scan
    continues with the raised count -- the single-GPU rsac.pnp_ransac(lo=True) result.
    """
    rank, world = _rank_world(group)
    scan = api.Scan(max_iters, ev.n, confidence, model_points)
    hb = 0
    best_model = None
    while not scan.done and hb < max_iters:
        hr = min(int(round_size), max_iters - hb, scan.niters - hb)
        b, c = shard(hr, rank, world)
        st, cn = ev.hypotheses(hb + b, c) if c > 0 else (np.zeros(0, np.int8), np.zeros(0, np.int32))
        rows = np.zeros((c, 2), np.int32)
        rows[:, 0] = st
        rows[:, 1] = cn
        full = np.concatenate(_all_gather_rows(rows, group))  # rank order = hypothesis order
        if not lo:
            scan.step(full[:, 1], full[:, 0].astype(np.int8))
        else:
            pos = 0
            while not scan.done and pos < hr:
                pos += scan.step_until_best(full[pos:, 1], full[pos:, 0].astype(np.int8))
                if scan.improved:
                    m, cnt = ev.local_opt(ev.model(scan.best), scan.max_good)
                    best_model = m if cnt > scan.max_good else ev.model(scan.best)
                    scan.raise_count(cnt)
        hb += hr
    if scan.best < 0:
        return ShardedResult(-1, 0, scan.iters, None)
    model = best_model if lo else ev.model(scan.best)
    return ShardedResult(scan.best, scan.max_good, scan.iters, model)


def sharded_batched(run_local, n_problems: int, group=None):
    """Independent problems split contiguously over ranks.

    ``run_local(begin, count)`` solves problems [begin, begin + count) on this rank and returns a
    (count, W) float64 array of fixed-size results (e.g. status, n_inliers, R 9, t 3); the call
    returns the (n_problems, W) array of all ranks, identical on every rank.
    """
    rank, world = _rank_world(group)
    b, c = shard(n_problems, rank, world)
    local = np.asarray(run_local(b, c), np.float64)
    if local.ndim != 2 or local.shape[0] != c:
        raise ValueError("run_local must return one row per problem")
    return np.concatenate(_all_gather_rows(local, group))


def pnp_batched_rows(points2D_list, points3D_list, K_list, n_iters: int = 5000, reproj_thresh: float = 30.0, **kw):
    """run_local for sharded_batched over rsac.pnp_ransac_batched: rows (ok, n_inliers, R 9, t 3)."""

    def run(begin, count):
        rows = np.zeros((count, 14))
        if count == 0:
            return rows
        sl = slice(begin, begin + count)
        res = api.pnp_ransac_batched(points2D_list[sl], points3D_list[sl], K_list[sl], n_iters, reproj_thresh, **kw)
        for i, (R, t, _, ninl) in enumerate(res):
            if R is not None:
                rows[i, 0] = 1
                rows[i, 1] = ninl
                rows[i, 2:11] = R.reshape(9)
                rows[i, 11:14] = t
        return rows

    return run
