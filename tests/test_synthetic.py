"""the NumPy restatement of the reference's synthetic
ARC-TopK / EF21 study (oracle/synthetic.py) reproduces the reference's committed result
files bit for bit -- a known-answer check of the algorithm family (block energy
ranking on the exact mean and on a Gaussian sketch, EF21 momentum variants)."""
import csv
import os

import numpy as np
import pytest

from oracle import synthetic as S

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "synthetic")


def _load(name):
    with open(os.path.join(HERE, name)) as f:
        rows = list(csv.reader(f))
    cols = rows[0][1:]
    data = np.array([[float(x) for x in r[1:]] for r in rows[1:]])
    return cols, data


@pytest.fixture(scope="module")
def study():
    return S.run_study()  # the full 1000-iteration study, ~12 s


@pytest.mark.parametrize("which", ["dist.csv", "loss.csv"])
def test_study_matches_reference_results(study, which):
    cols, ref = _load(which)
    got = study[0] if which == "dist.csv" else study[1]
    assert sorted(cols) == sorted(got)
    for j, name in enumerate(cols):
        a = np.asarray(got[name])
        assert a.shape == ref[:, j].shape, name
        assert np.array_equal(a, ref[:, j]), (name, float(np.abs(a - ref[:, j]).max()))


def test_study_claim_arc_beats_local_topk(study):
    """The study's point, from the trajectories: ARC-TopK (shared blocks from the mean's
    energy) converges where per-node top-k blocks stall."""
    d = study[0]
    for opt in S.OPTIMIZERS:
        assert d[f"{opt}_ArcTopK"][-1] < 0.1 * d[f"{opt}_Local TopK"][-1]
        assert d[f"{opt}_ArcTopK-Sketch"][-1] < 0.1 * d[f"{opt}_Local TopK"][-1]


def test_compressor_keeps_k_blocks_shared_across_nodes():
    np.random.seed(0)
    g = np.random.randn(1, 4, 200 * 10)
    for name in ("Random Block", "ArcTopK", "ArcTopK-Sketch"):
        out = S.COMPRESSORS[name](g, 200, 0.05).reshape(1, 4, 200, 10)
        kept = np.any(out != 0, axis=-1)
        assert kept.sum(axis=-1).tolist() == [[10] * 4]
        assert np.all(kept[:, :1] == kept)  # same blocks on every node
    out = S.c_local_topk_blocks(g, 200, 0.05).reshape(1, 4, 200, 10)
    assert np.all(np.any(out != 0, axis=-1).sum(axis=-1) == 10)
