"""Device-resident observation/reward normalisers.

Same semantics as safe_control_gym/math_and_models/normalization.py:13-160
(RunningMeanStd parallel-moment merge in float64, MeanStdNormalizer, and the
return-based RewardStdNormalizer), on the device so the rollout never leaves
HBM.  A float32 batch on the GPU takes the HIP kernels qs_rms_update (column
moments and the running merge in one launch) and qs_rms_normalize
(csrc/normalizer.hip); other inputs (CPU tensors of the gloo tests, the
float64 returns of RewardStdNormalizer) use the same formulas as torch ops.
With torch.distributed initialised, batch moments are merged across ranks
(sum / sum-of-squares all-reduce) so every shard normalises with the global
statistics.
"""
import ctypes

import numpy as np
import torch
import torch.distributed as tdist

from .. import _lib as L
from . import collectives


def _dist_on():
    return tdist.is_available() and tdist.is_initialized() and tdist.get_world_size() > 1


class RunningMeanStd:
    def __init__(self, epsilon=1e-4, shape=(), device="cpu"):
        self.mean = torch.zeros(shape, dtype=torch.float64, device=device)
        self.var = torch.ones(shape, dtype=torch.float64, device=device)
        self.count = torch.full((), epsilon, dtype=torch.float64, device=device)

    def _hip_ok(self, arr):
        """The HIP kernels take a float32 device batch whose rows are exactly this
        normaliser's shape (C = numel / rows = mean.numel(): the kernels index the
        float64 statistics by column).  Anything else — an unbatched (D, O) obs, a
        2-D (E·D, O) batch for a (D, O) normaliser — takes the torch expressions,
        which broadcast like the reference's numpy."""
        return (arr.is_cuda and arr.dtype == torch.float32 and arr.dim() >= 1 and arr.shape[0] > 0
                and arr.numel() // arr.shape[0] == self.mean.numel())

    def _work(self, R, C):
        key = (R, C)
        if getattr(self, '_wkey', None) != key:
            n = int(L.load().qs_rms_work_bytes(R, C))
            self._wbuf = torch.zeros(n, dtype=torch.uint8, device=self.mean.device)
            self._wkey = key
        return self._wbuf

    def update(self, arr):
        if self._hip_ok(arr):
            self._update_hip(arr)
            return
        x = arr.to(torch.float64)
        n = float(x.shape[0])   # a host constant: no host-to-device copy (the step is graph-captured)
        s1 = x.sum(0)
        s2 = (x * x).sum(0)
        if _dist_on():
            buf = torch.cat([s1.reshape(-1), s2.reshape(-1), torch.full((1,), n, dtype=torch.float64, device=x.device)])
            collectives.all_reduce(buf)
            k = s1.numel()
            s1, s2, n = buf[:k].view_as(s1), buf[k:2 * k].view_as(s2), buf[2 * k]
            batch_mean = s1 / n
            batch_var = s2 / n - batch_mean * batch_mean
        else:
            batch_mean = x.mean(0)
            batch_var = x.var(0, unbiased=False)     # np.var
        self.update_from_moments(batch_mean, batch_var, n)

    def _update_hip(self, arr):
        """qs_rms_update: the batch's column moments merged into the statistics in
        one launch (one rank); with several ranks the kernel writes this rank's
        [Σx | Σx² | n], which are all-reduced and merged as in update()."""
        x = arr.contiguous()
        R = int(x.shape[0])
        C = x.numel() // R
        lib = L.load()
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        work = self._work(R, C)
        if not _dist_on():
            L.check(lib.qs_rms_update(R, C, L.ptr(x), L.ptr(self.mean), L.ptr(self.var), L.ptr(self.count), None,
                                      L.ptr(work), st), "qs_rms_update")
            return
        buf = torch.empty(2 * C + 1, dtype=torch.float64, device=x.device)
        L.check(lib.qs_rms_update(R, C, L.ptr(x), None, None, None, L.ptr(buf), L.ptr(work), st), "qs_rms_update")
        collectives.all_reduce(buf)
        shape = self.mean.shape
        s1, s2, n = buf[:C].view(shape), buf[C:2 * C].view(shape), buf[2 * C]
        batch_mean = s1 / n
        self.update_from_moments(batch_mean, s2 / n - batch_mean * batch_mean, n)

    def update_from_moments(self, batch_mean, batch_var, batch_count):
        """normalization.py:42-60.  The statistics are updated in place, so a
        captured rollout graph reads and writes the same tensors on every replay."""
        delta = batch_mean - self.mean
        tot_count = self.count + batch_count
        new_mean = self.mean + delta * batch_count / tot_count
        m_a = self.var * self.count
        m_b = batch_var * batch_count
        m_2 = m_a + m_b + delta * delta * self.count * batch_count / (self.count + batch_count)
        new_var = m_2 / (self.count + batch_count)
        self.var.copy_(new_var)
        self.mean.copy_(new_mean)
        self.count.copy_(batch_count + self.count)

    def snapshot(self):
        return self.mean.clone(), self.var.clone(), self.count.clone()

    def restore(self, snap):
        for dst, src in zip((self.mean, self.var, self.count), snap):
            dst.copy_(src)


class BaseNormalizer:
    def __init__(self, read_only=False):
        self.read_only = read_only

    def set_read_only(self):
        self.read_only = True

    def unset_read_only(self):
        self.read_only = False

    def __call__(self, x, *args, **kwargs):
        return x

    def state_dict(self):
        return {}

    def load_state_dict(self, _):
        pass


class MeanStdNormalizer(BaseNormalizer):
    def __init__(self, shape=(), read_only=False, clip=10.0, epsilon=1e-8, device="cpu"):
        super().__init__(read_only)
        self.rms = RunningMeanStd(shape=shape, device=device)
        self.clip = clip
        self.epsilon = epsilon

    def __call__(self, x, out=None):
        if not self.read_only:
            self.rms.update(x)
        if self.rms._hip_ok(x) and (out is None or (out.dtype == torch.float32 and out.is_contiguous()
                                                      and out.numel() == x.numel())):
            # qs_rms_normalize: the same float64 expression, float32 out, one launch
            xc = x.contiguous()
            R = int(xc.shape[0])
            y = torch.empty_like(xc) if out is None else out
            st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
            L.check(L.load().qs_rms_normalize(R, xc.numel() // R, L.ptr(xc), L.ptr(self.rms.mean), L.ptr(self.rms.var),
                                              float(self.epsilon), float(self.clip), L.ptr(y), st), "qs_rms_normalize")
            return y
        y = torch.clamp((x.to(torch.float64) - self.rms.mean) / torch.sqrt(self.rms.var + self.epsilon),
                        -self.clip, self.clip)
        if out is not None:
            out.copy_(y)
            return out
        return y.to(torch.float32)

    def state_dict(self):
        return {'mean': self.rms.mean.cpu().numpy(), 'var': self.rms.var.cpu().numpy()}

    def load_state_dict(self, saved):
        # in place: a captured rollout graph keeps reading these tensors
        dev = self.rms.mean.device
        self.rms.mean.copy_(torch.as_tensor(np.asarray(saved['mean']), dtype=torch.float64, device=dev))
        self.rms.var.copy_(torch.as_tensor(np.asarray(saved['var']), dtype=torch.float64, device=dev))


class RewardStdNormalizer(MeanStdNormalizer):
    def __init__(self, gamma=0.99, read_only=False, clip=10.0, epsilon=1e-8, device="cpu"):
        super().__init__((), read_only, clip, epsilon, device)
        self.gamma = gamma
        self.ret = None

    def __call__(self, x, dones):
        """normalization.py:147-160: the discounted return (np.zeros_like(x) of the
        reference's float64 rewards — MultiHoverAviary._computeReward's numpy
        state arithmetic — so float64 here whatever the reward's dtype), its
        moments feed the running statistics, and the reward is only scaled."""
        if not self.read_only:
            if self.ret is None:
                self.ret = torch.zeros_like(x, dtype=torch.float64)
            self.ret = self.ret * self.gamma + x.to(torch.float64)
            self.rms.update(self.ret.reshape(-1))
            self.ret = torch.where(dones.bool(), torch.zeros_like(self.ret), self.ret)
        x64 = x.to(torch.float64)
        return torch.clamp(x64 / torch.sqrt(self.rms.var + self.epsilon), -self.clip, self.clip).to(x.dtype)
