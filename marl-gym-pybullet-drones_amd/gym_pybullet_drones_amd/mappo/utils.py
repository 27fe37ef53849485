"""The MAPPO package's two statistics helpers (gym_pybullet_drones/mappo/utils.py:6-13).

Both keep the reference's arithmetic (unbiased torch variance, epsilon added to the
standard deviation) and accept numpy arrays as well as tensors; tensors stay on
their device, so a call on rollout-buffer views does not synchronise the host.
"""
import numpy as np
import torch


def _as_tensor(x):
    return x if torch.is_tensor(x) else torch.as_tensor(np.asarray(x))


def normalize_tensor(tensor, epsilon=1e-8):
    """utils.py:6-8: zero mean, unit (unbiased) standard deviation."""
    t = _as_tensor(tensor)
    centred = t - t.mean()
    return centred / (t.std() + epsilon)


def explained_variance(y_pred, y_true):
    """utils.py:10-13: 1 − Var(y_true − y_pred) / Var(y_true) of two 1-D series
    (a 0-d tensor; NaN/inf when y_true is constant, as in the reference)."""
    yp, yt = _as_tensor(y_pred), _as_tensor(y_true)
    if yt.dim() != 1 or yp.dim() != 1:
        raise AssertionError("explained_variance takes 1-D y_pred and y_true")
    resid_var = torch.var(yt - yp)
    return 1 - resid_var / torch.var(yt)
