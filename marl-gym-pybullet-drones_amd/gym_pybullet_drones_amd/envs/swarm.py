"""QuadSwarm: the device-resident batch of (env × drone) quadrotors.

Thin host object over the C-ABI handle (include/quadswarm.h).  It owns no
physics: every call is one launch of the HIP step kernel on the caller's
current stream, with inputs and outputs as torch tensors resident in HBM
(zero-copy — their data pointers are passed straight through).

Reference semantics it implements (paths relative to gym_pybullet_drones/):
  BaseAviary.step/reset                envs/BaseAviary.py:220-383
  BaseRLAviary action/obs types        envs/BaseRLAviary.py:132-319
  MultiHoverAviary task                envs/MultiHoverAviary.py:12-285
  SpiralFormationAviary task           envs/SpiralAviary.py:20-205
  SubprocVecEnv worker auto-reset      safe_control_gym/envs/env_wrappers/
                                       vectorized_env/subproc_vec_env.py:188-206
"""
import ctypes
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from .. import _lib as L
from ..utils.enums import ActionType, DroneModel, Physics

_ACT = {ActionType.RPM: L.ACT_RPM, ActionType.PID: L.ACT_PID, ActionType.VEL: L.ACT_VEL,
        ActionType.ONE_D_RPM: L.ACT_ONE_D_RPM, ActionType.ONE_D_PID: L.ACT_ONE_D_PID}
# Physics → (integrator, aux force bits) (enums.py:13-21, BA:352-367).
_PHYS = {Physics.DYN: (L.PHYS_DYN, 0), Physics.PYB: (L.PHYS_PYB, 0),
         Physics.PYB_GND: (L.PHYS_PYB, L.AUX_GND), Physics.PYB_DRAG: (L.PHYS_PYB, L.AUX_DRAG),
         Physics.PYB_DW: (L.PHYS_PYB, L.AUX_DW),
         Physics.PYB_GND_DRAG_DW: (L.PHYS_PYB, L.AUX_GND | L.AUX_DRAG | L.AUX_DW)}
_AUX_NAMES = {"gnd": L.AUX_GND, "drag": L.AUX_DRAG, "dw": L.AUX_DW}
TASKS = {"multihover": L.TASK_MULTIHOVER, "spiral": L.TASK_SPIRAL, "flock": L.TASK_FLOCK, "meetup": L.TASK_MEETUP,
         "leaderfollower": L.TASK_LEADERFOLLOWER}


@dataclass
class StepResult:
    obs: torch.Tensor          # (E, D, O) float32, post auto-reset
    reward: torch.Tensor       # (E,) float32/float64
    terminated: torch.Tensor   # (E,) uint8
    truncated: torch.Tensor    # (E,) uint8
    terminal_obs: Optional[torch.Tensor] = None
    reasons: Optional[torch.Tensor] = None
    actions: Optional[torch.Tensor] = None


def grid_layout(num_drones, spacing=1.0, z=0.5):
    """Centred square-ish grid (SURVEY §7 hard-2 deviation for D >= 6): the
    reference's diagonal 4L layout (BaseAviary.py:194-197) cannot pass its own
    0.5 m rejection test for D >= 6, so the large-D configs use explicit
    initial_xyzs with `spacing` >= 1 m (acceptance 1 with the ±0.25 m noise)."""
    cols = int(np.ceil(np.sqrt(num_drones)))
    rows = int(np.ceil(num_drones / cols))
    out = []
    for i in range(num_drones):
        r, c = divmod(i, cols)
        out.append([(c - (cols - 1) / 2) * spacing, (r - (rows - 1) / 2) * spacing, z])
    return np.asarray(out, np.float64)


def _as_enum(x, enum):
    return x if isinstance(x, enum) else enum(x)


class QuadSwarm:
    """Batch of `num_envs` envs of `num_drones` drones (DroneModel.CF2X, the
    MAPPO tasks' model, or CF2P) on one GPU."""

    def __init__(self, task="multihover", num_envs=1, num_drones=2, act=ActionType.RPM, physics=Physics.DYN,
                 pyb_freq=240, ctrl_freq=None, precision=4, device=None, env_offset=0, initial_xyzs=None,
                 episode_len_sec=None, autoreset=True, drone_model=DroneModel.CF2X,
                 spiral_radius=0.4, spiral_period=10.0, height_rate=0.05, target_center=(0.0, 0.0, 0.0),
                 aux=(), inkernel_reset_search=False):
        """inkernel_reset_search: run MultiHover's whole reset rejection loop inside
        the step kernel instead of the deferred search launch (validation form).
        aux: extra force models ("gnd", "drag", "dw") added on top of `physics`;
        with Physics.DYN this is the build-defined DYN + aux combination (SURVEY §8
        physics-mode note), e.g. C5's DYN + downwash."""
        if task not in TASKS:
            raise ValueError(f"unknown task {task!r}")
        act = _as_enum(act, ActionType)
        physics = _as_enum(physics, Physics)
        drone_model = _as_enum(drone_model, DroneModel)
        # CF2X and CF2P: the models DSLPIDControl accepts (DSLPIDControl.py:34-36);
        # CF2P's inertia, props, torques and mixer ride on QS_FLAG_CF2P
        if drone_model not in (DroneModel.CF2X, DroneModel.CF2P):
            raise NotImplementedError("DroneModel.CF2X and CF2P are implemented (RACE has no DSL PID, "
                                      "DSLPIDControl.py:34-36)")
        if any(a not in _AUX_NAMES for a in aux):
            raise ValueError(f"unknown aux force model in {aux!r} (gnd, drag, dw)")
        if not torch.cuda.is_available():
            raise L.QuadSwarmError("QuadSwarm needs a ROCm GPU: the step runs only as a HIP kernel (no CPU path)")
        self.lib = L.load()
        self.task = task
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        if ctrl_freq is None:
            ctrl_freq = 48 if task == "spiral" else 30           # SP:28; MH:20 and the other MARL tasks
        if episode_len_sec is None:
            episode_len_sec = 12.0 if task == "spiral" else 8.0       # SP:39; MH:58 and the other MARL tasks
        spec = L.QsSpec()
        spec.task = TASKS[task]
        spec.num_envs = int(num_envs)
        spec.num_drones = int(num_drones)
        spec.act_type = _ACT[act]
        phys_id, aux_bits = _PHYS[physics]
        spec.physics = phys_id
        spec.aux_forces = aux_bits | sum(_AUX_NAMES[a] for a in set(aux))
        spec.pyb_freq = int(pyb_freq)
        spec.ctrl_freq = int(ctrl_freq)
        spec.precision = int(precision)
        spec.flags = ((0 if autoreset else L.FLAG_NO_AUTORESET) | (L.FLAG_INKERNEL_RESET_SEARCH if inkernel_reset_search else 0)
                      | (L.FLAG_CF2P if drone_model == DroneModel.CF2P else 0))
        spec.env_offset = int(env_offset)
        spec.episode_len_sec = float(episode_len_sec)
        self._xyz_keep = None
        if initial_xyzs is not None:
            xyz = np.ascontiguousarray(np.asarray(initial_xyzs, np.float64))
            if xyz.shape != (num_drones, 3):
                raise ValueError("invalid initial_xyzs, try initial_xyzs.reshape(NUM_DRONES,3)")  # BA:198-201
            self._xyz_keep = xyz
            spec.initial_xyzs = xyz.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
        spec.spiral_radius, spec.spiral_period, spec.height_rate = spiral_radius, spiral_period, height_rate
        for i in range(3):
            spec.target_center[i] = float(target_center[i])
        self.spec = spec
        self.act_type, self.physics, self.drone_model = act, physics, drone_model
        self._h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            L.check(self.lib.qs_create(ctypes.byref(spec), self.device.index, ctypes.byref(self._h)), "qs_create")
        dims = L.QsDims()
        L.check(self.lib.qs_get_dims(self._h, ctypes.byref(dims)), "qs_get_dims")
        self.dims = dims
        self.num_envs, self.num_drones, self.num_agents = dims.num_envs, dims.num_drones, dims.num_agents
        self.act_dim, self.obs_dim, self.hist_len = dims.act_dim, dims.obs_dim, dims.hist_len
        self.substeps = dims.substeps
        self.precision = dims.precision
        self.rdtype = torch.float64 if self.precision == 8 else torch.float32
        self.pyb_freq, self.ctrl_freq = int(pyb_freq), int(ctrl_freq)
        self.episode_len_sec = float(episode_len_sec)
        self.env_offset = int(env_offset)
        E, D, O = self.num_envs, self.num_drones, self.obs_dim
        kw = dict(device=self.device)
        self.obs = torch.zeros((E, D, O), dtype=torch.float32, **kw)
        self.reward = torch.zeros(E, dtype=self.rdtype, **kw)
        self.terminated = torch.zeros(E, dtype=torch.uint8, **kw)
        self.truncated = torch.zeros(E, dtype=torch.uint8, **kw)
        self.terminal_obs = torch.zeros((E, D, O), dtype=torch.float32, **kw)
        self.reasons = torch.zeros((E, D), dtype=torch.uint8, **kw)
        self.seed = 0
        self.reset_generation = 0   # qs_reset count: the device episode counters restart at each

    # ------------------------------------------------------------------ utils
    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def close(self):
        if getattr(self, "_h", None):
            torch.cuda.synchronize(self.device)
            self.lib.qs_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -------------------------------------------------------------- stepping
    def reset(self, seed=0, obs: Optional[torch.Tensor] = None):
        """Construct-time reset of every env (episode 0 draws); returns obs."""
        self.seed = int(seed)
        out = self.obs if obs is None else obs
        L.check(self.lib.qs_reset(self._h, ctypes.c_uint64(self.seed), L.ptr(out), self._stream()), "qs_reset")
        self.reset_generation += 1
        return out

    def reset_envs(self, mask: Optional[torch.Tensor] = None, obs: Optional[torch.Tensor] = None):
        """env.reset() (MultiHoverAviary.reset semantics) for envs with mask != 0."""
        if mask is not None:
            assert mask.dtype == torch.uint8 and mask.numel() == self.num_envs and mask.is_contiguous()
        out = self.obs if obs is None else obs
        L.check(self.lib.qs_reset_envs(self._h, L.ptr(mask), L.ptr(out), self._stream()), "qs_reset_envs")
        return out

    def step(self, actions: Optional[torch.Tensor] = None, *, obs=None, reward=None, terminated=None,
             truncated=None, terminal_obs=None, reasons=None, actions_out=None, want_terminal=False,
             want_reasons=False) -> StepResult:
        """One control step of every env.  actions: (E, D, A) float32 on device, or None
        for the synthetic random policy (Philox U(-1,1))."""
        if actions is not None:
            if (actions.dtype != torch.float32 or not actions.is_contiguous() or actions.device != self.device
                    or actions.numel() != self.num_agents * self.act_dim):
                raise ValueError(f"actions must be a contiguous float32 ({self.num_envs},{self.num_drones},"
                                 f"{self.act_dim}) tensor on {self.device}")
        obs = self.obs if obs is None else obs
        reward = self.reward if reward is None else reward
        terminated = self.terminated if terminated is None else terminated
        truncated = self.truncated if truncated is None else truncated
        # the kernel writes whole rows through these pointers: refuse a buffer it would overrun
        for t, dt, n, what in ((obs, torch.float32, self.num_agents * self.obs_dim, "obs"),
                               (reward, self.rdtype, self.num_envs, "reward"),
                               (terminated, torch.uint8, self.num_envs, "terminated"),
                               (truncated, torch.uint8, self.num_envs, "truncated")):
            if t.dtype != dt or not t.is_contiguous() or t.numel() < n or t.device != self.device:
                raise ValueError(f"{what} must be a contiguous {dt} tensor of >= {n} elements on {self.device}")
        if want_terminal and terminal_obs is None:
            terminal_obs = self.terminal_obs
        if want_reasons and reasons is None:
            reasons = self.reasons
        so = L.QsStepOut(L.ptr(obs), L.ptr(reward), L.ptr(terminated), L.ptr(truncated), L.ptr(terminal_obs),
                         L.ptr(reasons), L.ptr(actions_out))
        L.check(self.lib.qs_step(self._h, L.ptr(actions), ctypes.byref(so), self._stream()), "qs_step")
        return StepResult(obs, reward, terminated, truncated, terminal_obs, reasons, actions_out)

    # ------------------------------------------------------------ state I/O
    def _state_buf(self, block):
        kw = dict(device=self.device)
        if block == L.STATE_AGENT:
            return torch.zeros((L.AGENT_FIELDS, self.num_agents), dtype=self.rdtype, **kw)
        if block == L.STATE_ENV:
            return torch.zeros((L.ENV_FIELDS, self.num_envs), dtype=torch.int32, **kw)
        if block == L.STATE_HISTORY:
            return torch.zeros((self.hist_len, self.num_agents, self.act_dim), dtype=torch.float32, **kw)
        if block == L.STATE_EP_RETURN:
            return torch.zeros(self.num_envs, dtype=torch.float64, **kw)
        raise ValueError(block)

    def get_state(self, block=L.STATE_AGENT) -> torch.Tensor:
        buf = self._state_buf(block)
        L.check(self.lib.qs_state_io(self._h, block, L.ptr(buf), 0, self._stream()), "qs_state_io(get)")
        return buf

    def set_state(self, block, value):
        buf = self._state_buf(block)
        buf.copy_(torch.as_tensor(value).reshape(buf.shape).to(buf.dtype))
        L.check(self.lib.qs_state_io(self._h, block, L.ptr(buf), 1, self._stream()), "qs_state_io(set)")
        torch.cuda.current_stream(self.device).synchronize()

    def episode_log(self, cap=1 << 16):
        """(records ndarray[EPISODE_DTYPE] of the most recent ≤cap completed episodes, total ever)."""
        dst = torch.empty(max(cap, 1) * L.EPISODE_DTYPE.itemsize, dtype=torch.uint8, device=self.device)
        total, written = ctypes.c_int64(0), ctypes.c_int64(0)
        L.check(self.lib.qs_episode_log(self._h, L.ptr(dst) if cap > 0 else None, cap, ctypes.byref(total),
                                        ctypes.byref(written), self._stream()), "qs_episode_log")
        n = written.value   # fewer than min(total, cap) when rings dropped episodes
        recs = dst[: n * L.EPISODE_DTYPE.itemsize].cpu().numpy().view(L.EPISODE_DTYPE)
        order = np.lexsort((recs["env"], recs["seq"]))   # the reference's env-loop order per step
        return recs[order], total.value

    def reset_error(self):
        v = ctypes.c_int(0)
        L.check(self.lib.qs_reset_error(self._h, ctypes.byref(v)), "qs_reset_error")
        return v.value
