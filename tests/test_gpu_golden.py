"""The HIP kernel (fp64 and fp32, through the C-ABI) replays the committed golden vectors."""
import os
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = np.load(os.path.join(HERE, "golden", "oracle_golden.npz"))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_golden as mg  # noqa: E402


@pytest.mark.parametrize("precision", [8, 4])
@pytest.mark.parametrize("name", list(mg.CASES))
def test_kernel_replays_golden(name, precision):
    from gym_pybullet_drones_amd.envs import QuadSwarm
    from gym_pybullet_drones_amd.utils.enums import Physics
    kw = dict(mg.CASES[name])
    aux = kw.pop("aux", ())
    phys = Physics.PYB if kw.pop("physics", "dyn") == "pyb" else Physics.DYN
    sw = QuadSwarm(num_envs=mg.E, precision=precision, physics=phys, aux=aux, **kw)
    # reset obs: fp64 to float32 rounding; fp32 kernel within 2e-6 (hardware sin/cos of
    # the Spiral phase, ~1e-6 absolute)
    np.testing.assert_allclose(sw.reset(mg.SEED).cpu().numpy(), GOLD[f"{name}/obs0"],
                               atol=1e-7 if precision == 8 else 2e-6)
    act = torch.zeros((mg.E, sw.num_drones, sw.act_dim), device=sw.device)
    steps = mg.STEPS if precision == 8 else 10   # fp32: short open-loop horizon
    atol = 2e-6 if precision == 8 else 2e-3
    for t in range(steps):
        r = sw.step(None, actions_out=act)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(act.cpu().numpy(), GOLD[f"{name}/actions"][t])
        np.testing.assert_array_equal(r.terminated.cpu().numpy(), GOLD[f"{name}/terminated"][t])
        np.testing.assert_array_equal(r.truncated.cpu().numpy(), GOLD[f"{name}/truncated"][t])
        np.testing.assert_allclose(r.obs.cpu().numpy(), GOLD[f"{name}/obs"][t], rtol=atol, atol=atol)
    sw.close()
