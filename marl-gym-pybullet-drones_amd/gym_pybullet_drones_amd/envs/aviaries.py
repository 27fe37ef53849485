"""Gymnasium-shaped single-env facades with the reference class names.

`MultiHoverAviary` / `SpiralFormationAviary` keep the constructor signature,
spaces, attributes and the 5-tuple `step` of the reference classes
(envs/MultiHoverAviary.py:12-285, envs/SpiralAviary.py:20-205,
envs/BaseAviary.py:220-383) over an E=1 slice of the HIP QuadSwarm with the
vec-env auto-reset disabled (BaseAviary.step never resets by itself).
gymnasium is not installed here, so the class is duck-typed.

Physics defaults to Physics.PYB like the reference (MH:18, SP:26): the kernel's
restatement of Bullet's step (parity unpinned against pybullet).
"""
import numpy as np
import torch

from .. import _lib as L
from ..utils.enums import ActionType, DroneModel, ObservationType, Physics
from .swarm import QuadSwarm


class _SingleEnvAviary:
    TASK = None

    def __init__(self, drone_model=DroneModel.CF2X, num_drones=2, neighbourhood_radius=np.inf, initial_xyzs=None,
                 initial_rpys=None, physics=Physics.PYB, pyb_freq=240, ctrl_freq=30, gui=False, record=False,
                 obs=ObservationType.KIN, act=ActionType.RPM, device=None, precision=4, **task_kw):
        if gui or record:
            raise NotImplementedError("GUI/recording are out of scope (SURVEY §2)")
        if ObservationType(obs) != ObservationType.KIN:
            raise NotImplementedError("only ObservationType.KIN is implemented")
        if initial_rpys is not None and np.any(np.asarray(initial_rpys) != 0):
            raise NotImplementedError("non-zero initial_rpys are not supported by the MultiHover/Spiral tasks here")
        self.swarm = QuadSwarm(task=self.TASK, num_envs=1, num_drones=num_drones, act=act, physics=physics,
                               pyb_freq=pyb_freq, ctrl_freq=ctrl_freq, precision=precision, device=device,
                               initial_xyzs=initial_xyzs, autoreset=False, drone_model=drone_model, **task_kw)
        from ..vec_env.vec_env import action_space_for, observation_space_for
        self.observation_space = observation_space_for(self.swarm)
        self.action_space = action_space_for(self.swarm)
        self.NUM_DRONES = num_drones
        self.NEIGHBOURHOOD_RADIUS = neighbourhood_radius
        self.DRONE_MODEL = DroneModel(drone_model)
        self.PHYSICS = Physics(physics)
        self.OBS_TYPE = ObservationType(obs)
        self.ACT_TYPE = ActionType(act)
        self.PYB_FREQ = pyb_freq
        self.CTRL_FREQ = ctrl_freq
        self.PYB_STEPS_PER_CTRL = pyb_freq // ctrl_freq
        self.CTRL_TIMESTEP = 1.0 / ctrl_freq
        self.PYB_TIMESTEP = 1.0 / pyb_freq
        self.ACTION_BUFFER_SIZE = ctrl_freq // 2
        self.EPISODE_LEN_SEC = self.swarm.episode_len_sec
        self._started = False
        self._vec_spec = dict(task=self.TASK, num_drones=num_drones, act=ActionType(act), physics=Physics(physics),
                              pyb_freq=pyb_freq, ctrl_freq=ctrl_freq, precision=precision, drone_model=self.DRONE_MODEL,
                              initial_xyzs=None if initial_xyzs is None else np.asarray(initial_xyzs, np.float64),
                              **task_kw)
        self.swarm.reset(0)

    def vec_spec(self):
        """Constructor kwargs that rebuild this env as a batched SwarmVecEnv (used by MAPPO
        in place of make_vec_envs(env_func, ...), vectorized_env/__init__.py:42-66)."""
        return dict(self._vec_spec)

    @property
    def step_counter(self):
        return int(self.swarm.get_state(L.STATE_ENV)[L.E_STEP_COUNTER, 0].item())

    def _state(self):
        return self.swarm.get_state(L.STATE_AGENT).double().cpu().numpy()

    @property
    def pos(self):
        return self._state()[L.F_POS:L.F_POS + 3].T.copy()

    @property
    def quat(self):
        return self._state()[L.F_QUAT:L.F_QUAT + 4].T.copy()

    @property
    def vel(self):
        return self._state()[L.F_VEL:L.F_VEL + 3].T.copy()

    def _info(self, reasons=()):
        raise NotImplementedError

    def reset(self, seed=None, options=None):
        """seed is ignored, as in the reference (BaseAviary.py:243)."""
        obs = self.swarm.reset_envs(None)
        self._started = True
        return obs[0].cpu().numpy(), self._info(0)

    def step(self, action):
        sc = self.step_counter
        a = torch.as_tensor(np.asarray(action, np.float32)).reshape(1, self.NUM_DRONES, self.swarm.act_dim)
        r = self.swarm.step(a.to(self.swarm.device).contiguous(), want_reasons=True)
        obs = r.obs[0].cpu().numpy()
        term = bool(r.terminated[0].item())
        trunc = bool(r.truncated[0].item())
        from ..vec_env.vec_env import _reasons_strings
        reasons = _reasons_strings(r.reasons[0].cpu().numpy(), obs) if self.swarm.task == "multihover" else []
        return obs, float(r.reward[0].item()), term, trunc, self._info(sc, reasons)

    def close(self):
        self.swarm.close()

    def render(self, mode="human", close=False):
        p = self.pos
        for i in range(self.NUM_DRONES):
            print(f"[INFO] drone {i} x {p[i, 0]:+06.2f}, y {p[i, 1]:+06.2f}, z {p[i, 2]:+06.2f}")


class MultiHoverAviary(_SingleEnvAviary):
    """MultiHoverAviary.py:7-285 (ctrl_freq 30, EPISODE_LEN_SEC 8)."""
    TASK = "multihover"

    def __init__(self, drone_model=DroneModel.CF2X, num_drones=2, neighbourhood_radius=np.inf, initial_xyzs=None,
                 initial_rpys=None, physics=Physics.PYB, pyb_freq=240, ctrl_freq=30, gui=False, record=False,
                 obs=ObservationType.KIN, act=ActionType.RPM, **kw):
        super().__init__(drone_model, num_drones, neighbourhood_radius, initial_xyzs, initial_rpys, physics,
                         pyb_freq, ctrl_freq, gui, record, obs, act, **kw)

    @property
    def TARGET_POS(self):
        return self._state()[L.F_TARGET:L.F_TARGET + 3].T.copy()

    def _info(self, sc, reasons=()):
        return {"answer": 42, "termination_reasons": list(reasons)}


class SpiralFormationAviary(_SingleEnvAviary):
    """SpiralAviary.py:9-205 (ctrl_freq 48, EPISODE_LEN_SEC 12, ActionType.VEL)."""
    TASK = "spiral"

    def __init__(self, drone_model=DroneModel.CF2X, num_drones=3, neighbourhood_radius=np.inf, initial_xyzs=None,
                 initial_rpys=None, physics=Physics.PYB, pyb_freq=240, ctrl_freq=48, gui=False, record=False,
                 obs=ObservationType.KIN, act=ActionType.VEL, spiral_radius=0.4, spiral_period=10.0,
                 height_rate=0.05, target_center=np.array([0.0, 0.0, 0.0]), **kw):
        self.R = spiral_radius
        self.PERIOD = spiral_period
        self.OMEGA = 2 * np.pi / spiral_period
        self.VZ = height_rate
        self.CENTER = np.asarray(target_center, np.float64)
        super().__init__(drone_model, num_drones, neighbourhood_radius, initial_xyzs, initial_rpys, physics,
                         pyb_freq, ctrl_freq, gui, record, obs, act, spiral_radius=spiral_radius,
                         spiral_period=spiral_period, height_rate=height_rate,
                         target_center=tuple(self.CENTER), **kw)

    def _info(self, sc, reasons=()):
        return {"time": sc / self.PYB_FREQ, "omega": self.OMEGA, "radius": self.R}


class _MarlAviary(_SingleEnvAviary):
    """Base of the three BaseRLAviary MARL tasks without a custom reset: KIN obs,
    EPISODE_LEN_SEC 8, ctrl_freq 30, ActionType.RPM, info {"answer": 42}."""

    def __init__(self, drone_model=DroneModel.CF2X, num_drones=2, neighbourhood_radius=np.inf, initial_xyzs=None,
                 initial_rpys=None, physics=Physics.PYB, pyb_freq=240, ctrl_freq=30, gui=False, record=False,
                 obs=ObservationType.KIN, act=ActionType.RPM, **kw):
        super().__init__(drone_model, num_drones, neighbourhood_radius, initial_xyzs, initial_rpys, physics,
                         pyb_freq, ctrl_freq, gui, record, obs, act, **kw)

    def _info(self, sc, reasons=()):
        return {"answer": 42}


class FlockAviary(_MarlAviary):
    """FlockAviary.py:7-199: alignment + flock speed - spacing penalty - spacing variance;
    never terminates; truncated out of a 10 m box or tilted."""
    TASK = "flock"


class MeetupAviary(_MarlAviary):
    """MeetupAviary.py:6-164: pairs (i, D-1-i) meet; terminates when all pairs are within 0.1 m."""
    TASK = "meetup"


class LeaderFollowerAviary(_MarlAviary):
    """LeaderFollowerAviary.py:6-157: drone 0 hovers at (0, 0, 0.5), the others match its height."""
    TASK = "leaderfollower"
