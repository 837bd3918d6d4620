"""TEST INFRASTRUCTURE ONLY -- never imported by the product path.

NumPy restatement of the reference's synthetic convergence study
(synthetic_release/main.py), SURVEY.md section 8 row f4: a shift-coupled quadratic
objective over ``num_nodes`` workers, block compressors (none / random blocks /
per-node top-k blocks / ARC-TopK on the exact mean / ARC-TopK on a Gaussian sketch of
the mean) and the two EF21 momentum optimizers.  Pinned by the reference's own
committed result files (tests/golden/synthetic/*.csv): the distance-to-optimum and
loss trajectories must agree bit for bit (same NumPy global RNG stream, same float64
operation order).

Conventions of the study (they differ from the DDP hook): the gradient of one node is
viewed as [m blocks, ncols], K = max(1, min(ceil(mu * m), m)) blocks are kept, and
ARC-TopK ranks blocks by the energy of the node MEAN (an exact all-reduce), or of the
mean projected on R ~ N(0, 1)^{ncols x sketch_dim} drawn from the global stream.
"""
import math

import numpy as np


class ShiftedObjective:
    """Objective of main.py:15-180 (RobustShiftedObjective).

    Noise blocks 0..noise_blocks-1 of node i are pulled to xi_i + gamma_i * w_s, where
    w_s is the signal block; half of the nodes have (+noise_scale, +gamma), the other
    half (-noise_scale, -gamma).  The signal block is pulled to ``signal_scale``.
    """

    def __init__(self, num_nodes, dim, block_size, noise_blocks, signal_block, noise_scale,
                 signal_scale, gamma):
        self.num_nodes, self.dim, self.bs = num_nodes, dim, block_size
        self.noise_blocks, self.signal_block = noise_blocks, signal_block
        self.signal_scale = signal_scale
        self.scale = 1.0 / max(1, noise_blocks)
        half = num_nodes // 2
        nd = noise_blocks * block_size
        self.shifts = np.zeros((num_nodes, dim))
        self.gammas = np.zeros((num_nodes, dim))
        self.shifts[:half, :nd] = noise_scale
        self.shifts[half:, :nd] = -noise_scale
        self.gammas[:half, :nd] = gamma
        self.gammas[half:, :nd] = -gamma
        # optimum from the first noise block's statistics (main.py:52-90)
        xi0, g0 = self.shifts[:, :block_size], self.gammas[:, :block_size]
        w_s = (signal_scale - np.mean(g0 * xi0)) / (1.0 + np.mean(g0 ** 2))
        w_n = np.mean(xi0) + np.mean(g0) * w_s
        self.w_star = np.zeros(dim)
        self.w_star[self._sl(signal_block)] = w_s
        self.w_star[:nd] = w_n

    def _sl(self, b):
        return slice(b * self.bs, (b + 1) * self.bs)

    def grads(self, w, noise_std=0.0):
        """[1, nodes, dim] per-node gradients (main.py:97-140)."""
        nodes, bs, nb = self.num_nodes, self.bs, self.noise_blocks
        sig = self._sl(self.signal_block)
        w_s = np.broadcast_to(w[sig], (nodes, bs))
        nd = nb * bs
        xi = self.shifts[:, :nd].reshape(nodes, nb, bs)
        gam = self.gammas[:, :nd].reshape(nodes, nb, bs)
        wn = np.broadcast_to(w[:nd].reshape(1, nb, bs), (nodes, nb, bs))
        resid = wn - (xi + gam * w_s[:, None, :])
        out = np.zeros((1, nodes, self.dim))
        out[0, :, :nd] = (resid * self.scale).reshape(nodes, nd)
        # the reference accumulates the cross term block by block from zero: a running
        # (sequential) sum, which cumsum reproduces bit for bit
        cross = np.cumsum((resid * (-gam)) * self.scale, axis=1)[:, -1, :]
        out[0, :, sig] = (w_s - self.signal_scale) + cross
        if np.isnan(out).any():
            out = np.nan_to_num(out, nan=0.0, posinf=1e5, neginf=-1e5)
        if noise_std > 0:
            out += np.random.normal(loc=0.0, scale=noise_std, size=out.shape)
        return out

    def loss(self, w):
        """Global loss averaged over nodes (main.py:142-177)."""
        sig = self._sl(self.signal_block)
        w_s = w[sig]
        loss_s = 0.5 * np.sum((w_s - self.signal_scale) ** 2)
        nd = self.noise_blocks * self.bs
        target = self.shifts[:, :nd] + self.gammas[:, :nd] * np.tile(np.tile(w_s, self.noise_blocks),
                                                                     (self.num_nodes, 1))
        sq = np.sum((w[:nd] - target) ** 2, axis=1)
        return loss_s + self.scale * 0.5 * np.mean(sq)

    def dist(self, w):
        return np.linalg.norm(w - self.w_star)


def _keep(m, mu):
    return max(1, min(int(math.ceil(mu * m)), m))


def c_none(g, m, mu, **_):
    return g


def c_random_blocks(g, m, mu, **_):
    """K random blocks, shared by every node of a run (main.py:200-219)."""
    runs, nodes, d = g.shape
    v = g.reshape(runs, nodes, m, d // m)
    out = np.zeros_like(v)
    for r in range(runs):
        blocks = np.random.choice(m, _keep(m, mu), replace=False)
        out[r, :, blocks, :] = v[r, :, blocks, :]
    return out.reshape(runs, nodes, d)


def c_local_topk_blocks(g, m, mu, **_):
    """Each node keeps its own K highest-energy blocks (main.py:185-198)."""
    runs, nodes, d = g.shape
    v = g.reshape(runs, nodes, m, d // m)
    k = _keep(m, mu)
    idx = np.argpartition(np.sum(v ** 2, axis=-1), -k, axis=-1)[..., -k:]
    mask = np.zeros((runs, nodes, m), dtype=bool)
    np.put_along_axis(mask, idx, True, axis=-1)
    return np.where(mask[..., None], v, 0.0).reshape(runs, nodes, d)


def _shared_blocks(g, energy, m, mu):
    runs, nodes, d = g.shape
    v = g.reshape(runs, nodes, m, d // m)
    k = _keep(m, mu)
    idx = np.argpartition(energy, -k, axis=1)[:, -k:]
    mask = np.zeros((runs, m), dtype=bool)
    np.put_along_axis(mask, idx, True, axis=1)
    return np.where(mask[:, None, :, None], v, 0.0).reshape(runs, nodes, d)


def c_arctopk(g, m, mu, **_):
    """Blocks ranked by the energy of the node mean (main.py:221-232)."""
    runs, nodes, d = g.shape
    mean = np.mean(g.reshape(runs, nodes, m, d // m), axis=1)
    return _shared_blocks(g, np.sum(mean * mean, axis=2), m, mu)


def c_arctopk_sketch(g, m, mu, sketch_dim=2, **_):
    """Blocks ranked by the energy of mean @ R, R ~ N(0,1) [ncols, sketch_dim] (:234-264)."""
    runs, nodes, d = g.shape
    mean = np.mean(g.reshape(runs, nodes, m, d // m), axis=1)
    R = np.random.randn(runs, d // m, sketch_dim)
    P = np.matmul(mean, R)
    return _shared_blocks(g, np.sum(P * P, axis=2), m, mu)


COMPRESSORS = {
    "No Compressor": c_none,
    "Random Block": c_random_blocks,
    "Local TopK": c_local_topk_blocks,
    "ArcTopK": c_arctopk,
    "ArcTopK-Sketch": c_arctopk_sketch,
}
OPTIMIZERS = ("EF21-MSGD", "EF21 Double Momentum")


class EF21Momentum:
    """EF21 with one (MSGD) or two (double) momentum buffers, cold start (:267-320)."""

    def __init__(self, mode, compressor, shape, m, mu, eta, sketch_dim=2):
        if mode not in OPTIMIZERS:
            raise ValueError(f"Unknown mode: {mode}")
        self.mode, self.comp, self.m, self.mu, self.eta = mode, compressor, m, mu, eta
        self.sketch_dim = sketch_dim
        self.v = np.zeros(shape)
        self.u = np.zeros(shape)
        self.e = np.zeros(shape)

    def step(self, g):
        self.v = self.eta * self.v + g
        target = self.v
        if self.mode == "EF21 Double Momentum":
            self.u = self.eta * self.u + self.v
            target = self.u
        self.e = self.e + self.comp(target - self.e, self.m, self.mu, sketch_dim=self.sketch_dim)
        return self.e


# the study's configuration (main.py:326-356)
STUDY = dict(num_nodes=10, dim=2000, blocks=200, block_size=10, mu=0.05, noise_blocks=150,
             noise_scale=100.0, signal_scale=1.0, gamma=5.0, lr=0.001, steps=1000, beta=0.5,
             sketch_dim=2, noise_std=0.001, seed=42)


def run_study(steps=None, compressors=None, optimizers=OPTIMIZERS, **over):
    """Distance and loss trajectories per "<optimizer>_<compressor>" (main.py:322-413)."""
    cfg = dict(STUDY, **over)
    steps = cfg["steps"] if steps is None else steps
    np.random.seed(cfg["seed"])
    obj = ShiftedObjective(cfg["num_nodes"], cfg["dim"], cfg["block_size"], cfg["noise_blocks"],
                           cfg["noise_blocks"], cfg["noise_scale"], cfg["signal_scale"],
                           cfg["gamma"])
    names = list(COMPRESSORS) if compressors is None else list(compressors)
    dists, losses = {}, {}
    for opt_mode in optimizers:
        for name in names:
            np.random.seed(cfg["seed"])
            w = np.zeros(cfg["dim"])
            opt = EF21Momentum(opt_mode, COMPRESSORS[name], (1, cfg["num_nodes"], cfg["dim"]),
                               cfg["blocks"], cfg["mu"], cfg["beta"], cfg["sketch_dim"])
            dd, ll = [], []
            for t in range(steps):
                upd = np.mean(opt.step(obj.grads(w, noise_std=cfg["noise_std"])), axis=1).flatten()
                w -= cfg["lr"] * upd
                dist, loss = obj.dist(w), obj.loss(w)
                dd.append(dist)
                ll.append(loss)
                if dist > 1e5 or np.isnan(dist):  # diverged: pad like the reference
                    dd.extend([dist] * (steps - t - 1))
                    ll.extend([loss] * (steps - t - 1))
                    break
            dists[f"{opt_mode}_{name}"] = dd
            losses[f"{opt_mode}_{name}"] = ll
    return dists, losses
