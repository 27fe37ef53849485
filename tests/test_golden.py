"""The oracle reproduces the committed golden vectors (tests/golden/make_golden.py)."""
import os

import numpy as np
import pytest

import qs_oracle

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = np.load(os.path.join(HERE, "golden", "oracle_golden.npz"))


def _cases():
    import sys
    sys.path.insert(0, os.path.join(HERE, "golden"))
    import make_golden
    return make_golden


@pytest.mark.parametrize("name", ["mh_rpm_d4", "mh_onedpid_d8", "mh_vel_d3", "spiral_vel_d5", "mh_dw_d16",
                                  "mh_onedpid_d8_pyb"])
def test_oracle_reproduces_golden(name):
    mg = _cases()
    s = qs_oracle.OracleSim(num_envs=mg.E, precision=8, **mg.CASES[name])
    np.testing.assert_array_equal(s.reset(mg.SEED), GOLD[f"{name}/obs0"])
    for t in range(mg.STEPS):
        r = s.step(None)
        np.testing.assert_array_equal(r["actions"], GOLD[f"{name}/actions"][t])
        np.testing.assert_array_equal(r["terminated"], GOLD[f"{name}/terminated"][t])
        np.testing.assert_array_equal(r["truncated"], GOLD[f"{name}/truncated"][t])
        np.testing.assert_allclose(r["obs"], GOLD[f"{name}/obs"][t], rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(r["reward"], GOLD[f"{name}/reward"][t], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(s.get_state(0), GOLD[f"{name}/state"], rtol=1e-10, atol=1e-10)
    np.testing.assert_array_equal(s.get_state(1), GOLD[f"{name}/env"])
