"""Host-side trainer logic that needs no GPU."""
import numpy as np
import torch


def test_termination_counts_from_reason_bits():
    """MAPPO._termination_counts: one count per (drone, reason) at the terminal
    states of a rollout, under the reference counter's keys (mappo.py:720-735:
    'crashed' -> crash, 'flipped' -> flip, 'out of bounds' -> out_of_bounds)."""
    from gym_pybullet_drones_amd.mappo.mappo import MAPPO
    rng = np.random.default_rng(0)
    T, E, D = 7, 5, 3
    bits = rng.integers(0, 8, size=(T, E, D)).astype(np.uint8)
    bits[rng.random((T, E)) < 0.7] = 0   # most envs do not end at a step
    holder = type("H", (), {})()
    holder._reasons = torch.as_tensor(bits)
    got = MAPPO._termination_counts(holder)
    want = {}
    for b in bits.reshape(-1):
        for name, mask in (("crash", 1), ("flip", 2), ("out_of_bounds", 4)):
            if b & mask:
                want[name] = want.get(name, 0) + 1
    assert dict(got) == want
