"""Multi-rank driver (rsac/parallel.py) on CPU: world_size 2 over gloo, with an evaluator backed by
the CPU restatement (the GPU evaluator PnPShard is exercised in test_gpu_parity.py).

Checks that hypothesis sharding + all-reduce(MAX) of the packed key, the gathered adaptive scan,
and the problem-sharded all-gather give exactly the single-process results.
"""
from __future__ import annotations

import json
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import pyoracle as O
from rsac import parallel as par
from rsac import synth


class OracleShard:
    """Evaluator with PnPShard's interface, computed by oracle/ (test infrastructure)."""

    def __init__(self, pr, thr=30.0, seed=0x5EED):
        self.soa = O.soa_pnp(pr["points3d"], pr["points2d"])
        self.cam = O.cam_from_K(pr["K"])
        self.thr, self.seed = thr, seed
        self.n = len(self.soa[0])

    def hypotheses(self, begin, count):
        counts, status = O.pnp_hypotheses(self.soa, self.cam, self.thr, self.seed, count, hyp0=begin)
        return status, counts

    def range_key(self, begin, count):
        st, cn = self.hypotheses(begin, count)
        return par.best_key_of(cn, st, begin)

    def model(self, index):
        _, _, m = O.pnp_hypotheses(self.soa, self.cam, self.thr, self.seed, 1, hyp0=index, models=True)
        return m[0, :12].copy()

    def local_opt(self, model12, count):
        R, t, c, steps = O.pnp_local_opt(self.soa, self.cam, self.thr, model12[:9], model12[9:12], count)
        return np.concatenate([R.reshape(9), t]), c, steps


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pr = synth.pnp_problem(600, 0.6, seed=21)
        ev = OracleShard(pr)
        best = par.sharded_best(ev, 3001)
        c0 = par.COLLECTIVES
        ada = par.sharded_ransac(ev, 5000, 0.99, round_size=100)
        c1 = par.COLLECTIVES
        ada2 = par.sharded_ransac(OracleShard(synth.pnp_problem(800, 0.75, seed=22)), 5000, 0.99, round_size=700)
        c2 = par.COLLECTIVES
        lo = par.sharded_ransac(OracleShard(synth.pnp_problem(1500, 0.8, seed=8)), 5000, 0.99, round_size=97, lo=True)
        c3 = par.COLLECTIVES
        lo1 = par.sharded_ransac(OracleShard(synth.pnp_problem(700, 0.5, seed=23)), 5000, 0.99, round_size=97, lo=True)
        c4 = par.COLLECTIVES
        # problem sharding: 5 problems over the ranks, rows computed locally from the restatement
        probs = [synth.pnp_problem(300, 0.4, seed=s) for s in range(5)]

        def run_local(b, c):
            rows = np.zeros((c, 3))
            for i in range(c):
                p = probs[b + i]
                r = O.pnp_ransac(p["points3d"], p["points2d"], p["K"], 30.0, 0.99, 400)
                rows[i] = (b + i, r["best"], r["n_inliers"])
            return rows

        rows = par.sharded_batched(run_local, len(probs))
        res = {"best": [best.best, best.n_inliers, best.model.tolist()],
               "ada": [ada.best, ada.n_inliers, ada.iters, ada.model.tolist()],
               "ada2": [ada2.best, ada2.n_inliers, ada2.iters, ada2.model.tolist()],
               "lo": [lo.best, lo.n_inliers, lo.iters, lo.model.tolist()],
               "lo1": [lo1.best, lo1.n_inliers, lo1.iters, lo1.model.tolist()],
               "collectives": [c1 - c0, c2 - c1, c3 - c2, c4 - c3],
               "rows": rows.tolist()}
        json.dump(res, open(os.path.join(out_dir, f"rank{rank}.json"), "w"))
    finally:
        dist.destroy_process_group()


@pytest.fixture(scope="module")
def gloo_results(tmp_path_factory):
    d = tmp_path_factory.mktemp("gloo")
    mp.spawn(_worker, args=(2, _free_port(), str(d)), nprocs=2, join=True)
    return [json.load(open(d / f"rank{r}.json")) for r in range(2)]


def test_ranks_agree(gloo_results):
    assert gloo_results[0] == gloo_results[1]


def test_sharded_best_equals_single_process(gloo_results):
    pr = synth.pnp_problem(600, 0.6, seed=21)
    ev = OracleShard(pr)
    st, cn = ev.hypotheses(0, 3001)
    key = par.best_key_of(cn, st, 0)
    cnt, idx = par.unpack_key(key)
    b, n, model = gloo_results[0]["best"]
    assert (b, n) == (idx, cnt)
    # lowest index among the maxima (OpenCV's first strictly-greater winner)
    good = np.where(st > 0, cn, 0)
    assert idx == int(np.flatnonzero(good == good.max())[0])
    np.testing.assert_array_equal(model, ev.model(idx))


@pytest.mark.parametrize("key,n,outl,seed", [("ada", 600, 0.6, 21), ("ada2", 800, 0.75, 22)])
def test_sharded_adaptive_equals_sequential_loop(gloo_results, key, n, outl, seed):
    pr = synth.pnp_problem(n, outl, seed=seed)
    ref = O.pnp_ransac(pr["points3d"], pr["points2d"], pr["K"], 30.0, 0.99, 5000)
    b, cnt, iters, model = gloo_results[0][key]
    assert (b, cnt, iters) == (ref["best"], ref["n_inliers"], ref["iters"])
    np.testing.assert_array_equal(np.array(model[:9]).reshape(3, 3), ref["R"])
    np.testing.assert_array_equal(model[9:], ref["t"])


@pytest.mark.parametrize("key,n,outl,seed", [("lo", 1500, 0.8, 8), ("lo1", 700, 0.5, 23)])
def test_sharded_lo_ransac_equals_sequential_loop(gloo_results, key, n, outl, seed):
    pr = synth.pnp_problem(n, outl, seed=seed)
    ref = O.pnp_ransac_lo(pr["points3d"], pr["points2d"], pr["K"], 30.0, 0.99, 5000)
    b, cnt, iters, model = gloo_results[0][key]
    assert (b, cnt, iters) == (ref["best"], ref["n_inliers"], ref["iters"])
    np.testing.assert_array_equal(np.array(model[:9]).reshape(3, 3), ref["R"])
    np.testing.assert_array_equal(model[9:], ref["t"])


def test_sharded_first_round_runs_without_collectives(gloo_results):
    """Round 1 (FIRST_ROUND hypotheses) runs redundantly on every rank: a scan that ends inside it
    issues no collective at all; one that goes on all-gathers once per later round."""
    iters = {k: gloo_results[0][k][2] for k in ("ada", "ada2", "lo", "lo1")}
    coll = dict(zip(("ada", "ada2", "lo", "lo1"), gloo_results[0]["collectives"]))
    for k, it in iters.items():
        if it <= par.FIRST_ROUND:
            assert coll[k] == 0, (k, it, coll[k])
        else:
            assert coll[k] >= 1, (k, it, coll[k])
    # both kinds of scan are exercised
    assert min(iters.values()) <= par.FIRST_ROUND < max(iters.values())
    assert iters["ada"] <= par.FIRST_ROUND and iters["ada2"] > par.FIRST_ROUND


def test_problem_shards_gather_in_order(gloo_results):
    rows = np.array(gloo_results[0]["rows"])
    assert rows[:, 0].tolist() == list(range(5))
    for i in range(5):
        p = synth.pnp_problem(300, 0.4, seed=i)
        r = O.pnp_ransac(p["points3d"], p["points2d"], p["K"], 30.0, 0.99, 400)
        assert rows[i, 1:].tolist() == [r["best"], r["n_inliers"]]


@pytest.mark.parametrize("n,world", [(0, 2), (1, 2), (7, 3), (4096, 8), (100001, 8)])
def test_shard_partition(n, world):
    parts = [par.shard(n, r, world) for r in range(world)]
    assert sum(c for _, c in parts) == n
    pos = 0
    for b, c in parts:
        assert b == pos
        pos += c
    assert max(c for _, c in parts) - min(c for _, c in parts) <= 1


def test_key_packing_orders_like_sequential_scan():
    assert par.pack_key(10, 5) > par.pack_key(10, 6) > par.pack_key(9, 0) > par.pack_key(0, 0) == 0
    assert par.unpack_key(par.pack_key(1234, 98765)) == (1234, 98765)


def test_scan_matches_restatement():
    rng = np.random.default_rng(5)
    counts = rng.integers(0, 500, 3000).astype(np.int32)
    status = rng.choice(np.array([0, 1], np.int8), 3000, p=[0.2, 0.8])
    ref = O.scan(counts, status, 1000, 4, 0.99, 3000)
    import rsac
    sc = rsac.Scan(3000, 1000, 0.99, 4)
    for b in range(0, 3000, 700):  # round boundaries must not matter
        if sc.done:
            break
        sc.step(counts[b:b + 700], status[b:b + 700])
    assert (sc.best, sc.max_good, sc.iters) == ref
