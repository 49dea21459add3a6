"""CPU rehearsal of bench.py's multi-GPU legs: `torch.distributed.run
--nproc-per-node 2` with gloo runs tests/dist_rehearsal.py, which calls the rsac.parallel functions
bench.py uses at N > 1 (C3 problem chunks + all-gather, C5 sharded LO-RANSAC, the sharded adaptive
ms-to-best loop) on restatement-backed evaluators.  The two ranks must agree, and give the
single-process results: per-problem rows for C3; best, inlier count, iterations and LO
improvements for C5 (orc_pnp_ransac_lo) and the adaptive loop (orc_pnp_ransac)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import pyoracle as O
from rsac import synth

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import dist_rehearsal as W  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def ranks(tmp_path_factory):
    d = tmp_path_factory.mktemp("rehearsal")
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(HERE, "dist_rehearsal.py"), str(d)]
    subprocess.run(cmd, check=True, env=env, timeout=600, cwd=os.path.dirname(HERE))
    return [json.load(open(d / f"rank{r}.json")) for r in range(2)]


def test_ranks_agree(ranks):
    assert ranks[0] == ranks[1]


def test_comm_report_describes_the_line(ranks):
    """bench.py's multi_gpu.comm: backend, world size as the backend reports
    it, the timed 8-byte all-reduce, each rank's problem and hypothesis share."""
    c = ranks[0]["comm"]
    assert c["backend"] == "gloo" and c["world_size"] == 2 and c["allreduce_samples"] == 10
    assert c["problem_shares"] == [[0, 8], [8, 8]]
    assert c["hypothesis_shares"] == [[0, 500], [500, 500]]


def test_comm_report_single_process():
    from rsac import parallel as par
    c = par.comm_report(10, 7, samples=3)
    assert (c["backend"], c["world_size"], c["rank"]) == ("none", 1, 0)
    assert c["problem_shares"] == [[0, 10]] and c["hypothesis_shares"] == [[0, 7]] and c["allreduce_8b_us"] >= 0


def test_c3_rows_equal_single_process(ranks):
    rows = np.array(ranks[0]["c3"])
    assert rows.shape == (W.C3_PROBLEMS, 14)
    for i, s in enumerate(range(1, W.C3_PROBLEMS + 1)):
        p = synth.pnp_problem(W.C3_POINTS, 0.5, seed=s)
        r = O.pnp_ransac(p["points3d"], p["points2d"], p["K"], 30.0, 0.99, W.C3_HYPS)
        assert rows[i, 0] == (r["best"] >= 0) and rows[i, 1] == r["n_inliers"]
        np.testing.assert_array_equal(rows[i, 2:11], r["R"].reshape(9))
        np.testing.assert_array_equal(rows[i, 11:14], r["t"])


def test_c5_sharded_lo_equals_single_process(ranks):
    p = synth.pnp_problem(W.C5_POINTS, 0.5, seed=3)
    ref = O.pnp_ransac_lo(p["points3d"], p["points2d"], p["K"], 30.0, 0.99, 5000)
    best, ninl, iters, nlo, model = ranks[0]["c5"]
    assert (best, ninl, iters, nlo) == (ref["best"], ref["n_inliers"], ref["iters"], ref["lo_improvements"])
    np.testing.assert_array_equal(np.array(model[:9]).reshape(3, 3), ref["R"])
    np.testing.assert_array_equal(model[9:], ref["t"])


def test_sharded_adaptive_equals_single_process(ranks):
    p = synth.pnp_problem(3000, 0.7, seed=12)
    ref = O.pnp_ransac(p["points3d"], p["points2d"], p["K"], 30.0, 0.99, 5000)
    best, ninl, iters, model = ranks[0]["ada"]
    assert (best, ninl, iters) == (ref["best"], ref["n_inliers"], ref["iters"])
    np.testing.assert_array_equal(np.array(model[:9]).reshape(3, 3), ref["R"])
