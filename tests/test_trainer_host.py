"""Host-side trainer logic that needs no GPU."""
import numpy as np
import pytest
import torch


def _holder(bits, reference_compat):
    holder = type("H", (), {})()
    holder._reasons = torch.as_tensor(bits)
    holder.reference_compat = reference_compat
    return holder


def test_termination_counts_from_reason_bits():
    """MAPPO._termination_counts with reference_compat=False: one count per
    (drone, reason) at the terminal states of a rollout, under the reference
    counter's keys (mappo.py:720-735: 'crashed' -> crash, 'flipped' -> flip,
    'out of bounds' -> out_of_bounds)."""
    from gym_pybullet_drones_amd.mappo.mappo import MAPPO
    rng = np.random.default_rng(0)
    T, E, D = 7, 5, 3
    bits = rng.integers(0, 8, size=(T, E, D)).astype(np.uint8)
    bits[rng.random((T, E)) < 0.7] = 0   # most envs do not end at a step
    got = MAPPO._termination_counts(_holder(bits, False))
    want = {}
    for b in bits.reshape(-1):
        for name, mask in (("crash", 1), ("flip", 2), ("out_of_bounds", 4)):
            if b & mask:
                want[name] = want.get(name, 0) + 1
    assert dict(got) == want


def test_termination_counts_reference_compat_is_empty():
    """reference_compat: the reference's vectorised loop reads the info of the
    auto-reset (subproc_vec_env.py:195-205), whose termination_reasons
    MultiHoverAviary.reset has cleared (MH:109), so its counter stays empty."""
    from gym_pybullet_drones_amd.mappo.mappo import MAPPO
    bits = np.full((3, 4, 2), 7, dtype=np.uint8)
    assert dict(MAPPO._termination_counts(_holder(bits, True))) == {}


def test_mappo_utils_match_their_definitions():
    """mappo/utils.py:6-13: normalize_tensor and explained_variance (re-exported
    from the package like the reference's module)."""
    from gym_pybullet_drones_amd.mappo import explained_variance, normalize_tensor
    rng = np.random.default_rng(3)
    x = rng.normal(2.0, 3.0, size=(50, 4))
    got = normalize_tensor(torch.as_tensor(x)).numpy()
    np.testing.assert_allclose(got, (x - x.mean()) / (x.std(ddof=1) + 1e-8), rtol=1e-12)
    np.testing.assert_allclose(normalize_tensor(x).numpy(), got, rtol=0)   # numpy input
    y = rng.normal(size=200)
    yp = y + 0.1 * rng.normal(size=200)
    ev = float(explained_variance(torch.as_tensor(yp), torch.as_tensor(y)))
    assert ev == pytest.approx(1 - np.var(y - yp, ddof=1) / np.var(y, ddof=1), rel=1e-12)
    with pytest.raises(AssertionError):
        explained_variance(torch.zeros(2, 2), torch.zeros(2, 2))


def test_fused_mlp_row_limits():
    """The fused MLP paths (MLP.forward inference, _TanhMLP3) take a batch only
    within the qs_mlp3_* launchers' limits (csrc/learner.hip: K > 0, K·256·4 and
    K·I·4 below 2^31); anything else falls back to the GEMM path instead of
    raising QS_E_INVALID."""
    from gym_pybullet_drones_amd.mappo.agent import _m3_shape_ok
    assert not _m3_shape_ok(0, 27)
    assert _m3_shape_ok(1, 27)
    assert _m3_shape_ok(2 ** 21 - 1, 27) and not _m3_shape_ok(2 ** 21, 27)      # 262 144 envs x 8 drones
    assert not _m3_shape_ok(2 ** 19, 1024) and _m3_shape_ok(2 ** 19 - 1, 1024)


def test_reward_std_normalizer_matches_reference_restatement():
    """RewardStdNormalizer (normalization.py:123-160) against a numpy restatement
    of the reference with its own dtypes: float64 rewards (MultiHoverAviary's
    numpy reward), the return tracked in float64 (np.zeros_like of the reward),
    its float64 running moments, the reward scaled (not centred) and clipped,
    the return cleared on done.  A float32 reward (this port's rollout buffer)
    gives the same float64 return.  Off in both reference trainer configs
    (learn_mappo.py / env_select_learn_mappo.py: norm_reward False), kept for
    the MAPPO constructor's norm_reward switch."""
    import numpy as np
    import torch
    from gym_pybullet_drones_amd.mappo.normalization import RewardStdNormalizer
    rng = np.random.default_rng(4)
    E, gamma = 64, 0.99
    for dt in (np.float64, np.float32):
        norm = RewardStdNormalizer(gamma=gamma, clip=10.0, epsilon=1e-8, device="cpu")
        mean, var, count, ret = 0.0, 1.0, 1e-4, None
        for t in range(40):
            x = (rng.normal(size=E) * 0.3 - 1.0).astype(dt)
            dones = rng.random(E) < 0.05
            got = norm(torch.as_tensor(x), torch.as_tensor(dones)).numpy()
            # the reference (numpy): its reward is float64
            x64 = x.astype(np.float64)
            ret = np.zeros_like(x64) if ret is None else ret
            ret = ret * gamma + x64
            assert ret.dtype == np.float64
            bm, bv, bc = ret.mean(0), ret.var(0), E
            delta = bm - mean
            tot = count + bc
            mean, var, count = (mean + delta * bc / tot,
                                (var * count + bv * bc + delta * delta * count * bc / (count + bc)) / (count + bc),
                                bc + count)
            ret[dones] = 0
            want = np.clip(x64 / np.sqrt(var + 1e-8), -10.0, 10.0).astype(dt)
            assert norm.ret.dtype == torch.float64
            np.testing.assert_array_equal(norm.ret.numpy(), ret)
            np.testing.assert_allclose(float(norm.rms.var), var, rtol=1e-12)
            np.testing.assert_allclose(got, want, rtol=1e-6, atol=0)
        assert got.dtype == dt


def test_rms_hip_path_only_for_matching_columns():
    """The HIP normaliser kernels index the float64 statistics by column, so a
    batch takes them only when its rows have the normaliser's shape; other
    shapes (an unbatched (D, O) obs, a 2-D (E·D, O) batch for a (D, O)
    normaliser) take the broadcasting torch expressions.  Checked
    on the guard itself (no GPU here) with a stand-in device batch."""
    import torch
    from gym_pybullet_drones_amd.mappo.normalization import RunningMeanStd
    rms = RunningMeanStd(shape=(3, 5))

    class Batch:   # what _hip_ok reads of a CUDA tensor
        is_cuda, dtype = True, torch.float32

        def __init__(self, *shape):
            self.shape = shape

        def dim(self):
            return len(self.shape)

        def numel(self):
            n = 1
            for s in self.shape:
                n *= s
            return n

    assert rms._hip_ok(Batch(64, 3, 5))        # (E, D, O)
    assert rms._hip_ok(Batch(64, 15))          # (E, D·O)
    assert not rms._hip_ok(Batch(3, 5))        # unbatched (D, O)
    assert not rms._hip_ok(Batch(192, 5))      # (E·D, O)
    assert not rms._hip_ok(Batch(0, 3, 5))
    assert not rms._hip_ok(torch.zeros(4, 3, 5))   # CPU tensor
