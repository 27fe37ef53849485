"""MultiHover reset distribution (MultiHoverAviary.reset, MH:75-110).

The reference draws from numpy's global MT19937; the build draws from Philox, so
RNG streams cannot match (SURVEY §7 hard-3).  This checks the *distribution*: an
independent numpy restatement of the reference's rejection sampler vs the oracle
(which the GPU kernel matches bit for bit, tests/test_gpu_parity.py), with a
two-sample KS test per coordinate and the acceptance-rate implied spacing.
"""
import numpy as np
import pytest
from scipy import stats

import qs_oracle

L = 0.0397
ORIG = lambda D: np.stack([np.arange(D) * 4 * L, np.arange(D) * 4 * L, np.full(D, 0.025 / 2 + 0.1)], 1)


def reference_reset(D, rng):
    orig = ORIG(D)
    xyz = orig + rng.uniform(-0.25, 0.25, (D, 3))
    xyz[:, 2] = np.clip(xyz[:, 2], 0.1, 1.0)
    while True:
        dists = np.linalg.norm(xyz[:, None, :] - xyz[None, :, :], axis=2)
        np.fill_diagonal(dists, np.inf)
        if not np.any(dists < 0.5) and not np.any(xyz[:, 2] < 0.1):
            return xyz
        xyz = orig + rng.uniform(-0.25, 0.25, (D, 3))
        xyz[:, 2] = np.clip(xyz[:, 2], 0.1, 1.0)


@pytest.mark.parametrize("D", [2, 3])
def test_reset_distribution_matches_reference_sampler(D):
    n = 1500
    rng = np.random.default_rng(7)
    ref = np.stack([reference_reset(D, rng) for _ in range(n)])
    s = qs_oracle.OracleSim(task="multihover", num_envs=n, num_drones=D, act="rpm", precision=8)
    obs = s.reset(99)
    ours = obs[:, :, :3].astype(np.float64)
    for d in range(D):
        for k in range(3):
            p = stats.ks_2samp(ref[:, d, k].astype(np.float32), ours[:, d, k]).pvalue   # obs are float32
            assert p > 1e-3, (d, k, p)
    # every draw satisfies the rejection constraints
    dd = np.linalg.norm(ours[:, :, None, :] - ours[:, None, :, :], axis=3) + np.eye(D) * 9
    assert dd.min() >= 0.5 - 1e-6
    assert ours[:, :, 2].min() >= 0.1 - 1e-7
