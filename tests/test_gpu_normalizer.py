"""The rollout's observation normaliser on the HIP kernels qs_rms_update /
qs_rms_normalize (csrc/normalizer.hip), through the C-ABI, against a numpy
float64 restatement of safe_control_gym/math_and_models/normalization.py:13-120.

* running statistics after a sequence of updates: 1e-12 relative (the batch
  moments are float64 sums in another order than numpy's);
* the normalised output from the kernel's own statistics: bit for bit (the same
  float64 expression, correctly rounded division and square root, float32 out);
* the multi-rank form ([Σx | Σx² | n] for the all-reduce) and shapes with one
  row, one column and more than 256 columns.
"""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


class _NpRMS:
    """normalization.py:13-60 (numpy, float64)."""

    def __init__(self, shape, epsilon=1e-4):
        self.mean, self.var, self.count = np.zeros(shape), np.ones(shape), epsilon

    def update(self, arr):
        bm, bv, bc = arr.mean(0), arr.var(0), arr.shape[0]
        delta = bm - self.mean
        tot = self.count + bc
        new_mean = self.mean + delta * bc / tot
        m2 = self.var * self.count + bv * bc + delta * delta * self.count * bc / (self.count + bc)
        self.mean, self.var, self.count = new_mean, m2 / (self.count + bc), bc + self.count


@pytest.mark.parametrize("shape", [(1, 12), (16, 4, 27), (8192, 5, 27), (1000, 432), (37, 300), (4099, 1)])
def test_rms_update_and_normalize_match_numpy(shape):
    from gym_pybullet_drones_amd.mappo.normalization import MeanStdNormalizer
    rng = np.random.default_rng(sum(shape))
    norm = MeanStdNormalizer(shape=shape[1:], clip=10.0, epsilon=1e-8, device="cuda")
    ref = _NpRMS(shape[1:])
    for k in range(3):
        # obs-like columns: offsets and scales that differ per column, a few outliers to clip
        x = (rng.normal(size=shape) * rng.uniform(0.01, 3.0, size=shape[1:]) + rng.uniform(-5, 5, size=shape[1:]))
        x = x.astype(np.float32)
        if k == 2:
            x.reshape(-1)[:: 97] *= 1e3
        xd = torch.as_tensor(x, device="cuda")
        out = torch.empty_like(xd)
        y = norm(xd, out=out)
        assert y is out
        ref.update(x.astype(np.float64))
        np.testing.assert_allclose(norm.rms.mean.cpu().numpy(), ref.mean, rtol=1e-12, atol=1e-13, err_msg=f"mean {k}")
        np.testing.assert_allclose(norm.rms.var.cpu().numpy(), ref.var, rtol=1e-12, atol=1e-13, err_msg=f"var {k}")
        assert float(norm.rms.count) == ref.count
        # the output from the device's own statistics: the same float64 expression
        m, v = norm.rms.mean.cpu().numpy(), norm.rms.var.cpu().numpy()
        want = np.clip((x.astype(np.float64) - m) / np.sqrt(v + 1e-8), -10.0, 10.0).astype(np.float32)
        np.testing.assert_array_equal(y.cpu().numpy(), want, err_msg=f"normalised {k}")
    # read-only: no statistics update, output only
    norm.set_read_only()
    before = norm.rms.mean.clone()
    y2 = norm(xd)
    assert torch.equal(norm.rms.mean, before) and y2.dtype == torch.float32
    np.testing.assert_array_equal(y2.cpu().numpy(), y.cpu().numpy())


def test_rms_sums_for_the_rank_exchange():
    """sums != NULL: this rank's [Σx | Σx² | n] (float64), statistics untouched."""
    from gym_pybullet_drones_amd import _lib as L
    rng = np.random.default_rng(5)
    R, C = 3001, 140
    x = (rng.normal(size=(R, C)) * 2 + 1).astype(np.float32)
    xd = torch.as_tensor(x, device="cuda")
    lib = L.load()
    work = torch.zeros(int(lib.qs_rms_work_bytes(R, C)), dtype=torch.uint8, device="cuda")
    buf = torch.zeros(2 * C + 1, dtype=torch.float64, device="cuda")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    L.check(lib.qs_rms_update(R, C, L.ptr(xd), None, None, None, L.ptr(buf), L.ptr(work), st), "qs_rms_update")
    b = buf.cpu().numpy()
    x64 = x.astype(np.float64)
    np.testing.assert_allclose(b[:C], x64.sum(0), rtol=1e-12)
    np.testing.assert_allclose(b[C:2 * C], (x64 * x64).sum(0), rtol=1e-12)
    assert b[2 * C] == R
    assert int(work[:4].view(torch.int32)[0]) == 0   # the launch leaves its counter zero


def test_rms_update_is_replay_deterministic():
    """Fixed reduction orders: the same batch from the same statistics gives the same bits."""
    from gym_pybullet_drones_amd.mappo.normalization import RunningMeanStd
    rng = np.random.default_rng(9)
    x = torch.as_tensor(rng.normal(size=(8192, 135)).astype(np.float32), device="cuda")
    outs = []
    for _ in range(2):
        r = RunningMeanStd(shape=(135,), device="cuda")
        r.update(x)
        r.update(x * 2)
        outs.append((r.mean.clone(), r.var.clone()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


def test_rms_rejects_bad_arguments():
    from gym_pybullet_drones_amd import _lib as L
    lib = L.load()
    with pytest.raises(L.QuadSwarmError, match="qs_rms_update"):
        L.check(lib.qs_rms_update(0, 4, None, None, None, None, None, None, None), "qs_rms_update")
    with pytest.raises(L.QuadSwarmError, match="qs_rms_normalize"):
        L.check(lib.qs_rms_normalize(4, 0, None, None, None, 1e-8, 10.0, None, None), "qs_rms_normalize")


@pytest.mark.parametrize("batch", [(4, 27), (8, 1, 27)])
def test_rms_mismatched_shape_takes_the_broadcasting_path(batch):
    """A batch whose rows are not the normaliser's shape — an unbatched (D, O)
    obs, or (E, 1, O) rows for a (D, O) normaliser — must not reach the
    kernels (they would index mean / var by the batch's column count): it takes
    the torch expressions, whose results equal the same expressions on the CPU
    (numpy broadcasting in the reference)."""
    from gym_pybullet_drones_amd.mappo.normalization import MeanStdNormalizer
    rng = np.random.default_rng(13)
    D, O = 4, 27
    norms = [MeanStdNormalizer(shape=(D, O), clip=10.0, epsilon=1e-8, device=dev) for dev in ("cuda", "cpu")]
    for k in range(2):
        x = (rng.normal(size=batch) * 2 + 0.5).astype(np.float32)
        y = [n(torch.as_tensor(x, device=n.rms.mean.device)) for n in norms]
        np.testing.assert_allclose(norms[0].rms.mean.cpu().numpy(), norms[1].rms.mean.numpy(), rtol=1e-12)
        np.testing.assert_allclose(norms[0].rms.var.cpu().numpy(), norms[1].rms.var.numpy(), rtol=1e-12)
        np.testing.assert_allclose(y[0].cpu().numpy(), y[1].numpy(), rtol=1e-6)
