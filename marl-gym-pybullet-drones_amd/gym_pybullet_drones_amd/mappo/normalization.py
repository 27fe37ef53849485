"""Device-resident observation/reward normalisers.

Same semantics as safe_control_gym/math_and_models/normalization.py:13-160
(RunningMeanStd parallel-moment merge in float64, MeanStdNormalizer, and the
return-based RewardStdNormalizer), computed with torch on the GPU so the rollout
never leaves HBM.  With torch.distributed initialised, batch moments are merged
across ranks (sum / sum-of-squares all-reduce) so every shard normalises with
the global statistics.
"""
import numpy as np
import torch
import torch.distributed as tdist


def _dist_on():
    return tdist.is_available() and tdist.is_initialized() and tdist.get_world_size() > 1


class RunningMeanStd:
    def __init__(self, epsilon=1e-4, shape=(), device="cpu"):
        self.mean = torch.zeros(shape, dtype=torch.float64, device=device)
        self.var = torch.ones(shape, dtype=torch.float64, device=device)
        self.count = torch.full((), epsilon, dtype=torch.float64, device=device)

    def update(self, arr):
        x = arr.to(torch.float64)
        n = float(x.shape[0])   # a host constant: no host-to-device copy (the step is graph-captured)
        s1 = x.sum(0)
        s2 = (x * x).sum(0)
        if _dist_on():
            buf = torch.cat([s1.reshape(-1), s2.reshape(-1), torch.full((1,), n, dtype=torch.float64, device=x.device)])
            tdist.all_reduce(buf)
            k = s1.numel()
            s1, s2, n = buf[:k].view_as(s1), buf[k:2 * k].view_as(s2), buf[2 * k]
            batch_mean = s1 / n
            batch_var = s2 / n - batch_mean * batch_mean
        else:
            batch_mean = x.mean(0)
            batch_var = x.var(0, unbiased=False)     # np.var
        self.update_from_moments(batch_mean, batch_var, n)

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
        x64 = x.to(torch.float64)
        if not self.read_only:
            if self.ret is None:
                self.ret = torch.zeros_like(x64)
            self.ret = self.ret * self.gamma + x64
            self.rms.update(self.ret.reshape(-1))
            self.ret = torch.where(dones.bool(), torch.zeros_like(self.ret), self.ret)
        return torch.clamp(x64 / torch.sqrt(self.rms.var + self.epsilon), -self.clip, self.clip).to(x.dtype)
