"""ctypes binding of the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module; it is the parity checker, never the product path.  Parity status:
"parity unpinned" against the reference (see qs_oracle.cpp header and
DESIGN.md §Oracle).
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libqs_oracle.so")

TASK = {"multihover": 0, "spiral": 1, "flock": 2, "meetup": 3, "leaderfollower": 4}
ACT = {"rpm": 0, "pid": 1, "vel": 2, "one_d_rpm": 3, "one_d_pid": 4}
AUX = {"gnd": 1, "drag": 2, "dw": 4}
AGENT_FIELDS = 29
ENV_FIELDS = 4


class QsSpec(ctypes.Structure):
    _fields_ = [
        ("task", ctypes.c_int32), ("num_envs", ctypes.c_int32), ("num_drones", ctypes.c_int32),
        ("act_type", ctypes.c_int32), ("physics", ctypes.c_int32), ("aux_forces", ctypes.c_uint32),
        ("pyb_freq", ctypes.c_int32), ("ctrl_freq", ctypes.c_int32), ("precision", ctypes.c_int32),
        ("flags", ctypes.c_uint32), ("env_offset", ctypes.c_int64), ("episode_len_sec", ctypes.c_double),
        ("initial_xyzs", ctypes.POINTER(ctypes.c_double)), ("spiral_radius", ctypes.c_double),
        ("spiral_period", ctypes.c_double), ("height_rate", ctypes.c_double),
        ("target_center", ctypes.c_double * 3),
    ]


class QsDims(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "num_envs", "num_drones", "num_agents", "act_dim", "obs_dim", "hist_len", "substeps",
        "precision", "agent_fields", "env_fields")]


class QsStepOut(ctypes.Structure):
    _fields_ = [("obs", ctypes.c_void_p), ("reward", ctypes.c_void_p), ("terminated", ctypes.c_void_p),
                ("truncated", ctypes.c_void_p), ("terminal_obs", ctypes.c_void_p), ("reasons", ctypes.c_void_p),
                ("actions_out", ctypes.c_void_p)]


class QsEpisodeRec(ctypes.Structure):
    _fields_ = [("ret", ctypes.c_double), ("len", ctypes.c_int32), ("env", ctypes.c_int32), ("seq", ctypes.c_int64)]


EPISODE_DTYPE = np.dtype([("ret", "<f8"), ("len", "<i4"), ("env", "<i4"), ("seq", "<i8")])

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        vp, i32, i64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
        L.qso_last_error.restype = ctypes.c_char_p
        L.qso_create.argtypes = [ctypes.POINTER(QsSpec), ctypes.POINTER(vp)]
        L.qso_destroy.argtypes = [vp]
        L.qso_get_dims.argtypes = [vp, ctypes.POINTER(QsDims)]
        L.qso_reset.argtypes = [vp, ctypes.c_uint64, vp]
        L.qso_step.argtypes = [vp, vp, ctypes.POINTER(QsStepOut), i32]
        L.qso_run_random.argtypes = [vp, i32, i32]
        L.qso_reset_envs.argtypes = [vp, vp, vp]
        L.qso_state_io.argtypes = [vp, i32, vp, i32]
        L.qso_episode_log.argtypes = [vp, vp, i64]
        L.qso_episode_log.restype = i64
        L.qso_reset_error.argtypes = [vp]
        L.qso_philox4x32_10.argtypes = [vp, vp, vp]
        L.qso_quat_to_matrix.argtypes = [vp, vp]
        L.qso_euler_from_quat.argtypes = [vp, vp]
        L.qso_integrate_q.argtypes = [vp, vp, ctypes.c_double]
        L.qso_constants.argtypes = [vp]
        L.qso_dsl_pid.argtypes = [vp, vp, vp, vp, vp, vp, vp, ctypes.c_double, vp]
        L.qso_gae.argtypes = [i32, i64, vp, vp, vp, vp, vp, ctypes.c_double, i32, ctypes.c_double, vp, vp]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def make_spec(task="multihover", num_envs=1, num_drones=2, act="rpm", aux=(), physics="dyn", ctrl_freq=None, pyb_freq=240,
              precision=8, env_offset=0, episode_len_sec=None, initial_xyzs=None, autoreset=True,
              spiral_radius=0.4, spiral_period=10.0, height_rate=0.05, target_center=(0.0, 0.0, 0.0),
              drone_model="cf2x"):
    s = QsSpec()
    s.task = TASK[task]
    s.num_envs = num_envs
    s.num_drones = num_drones
    s.act_type = ACT[act]
    s.physics = {"pyb": 0, "dyn": 1}[physics]
    s.aux_forces = sum(AUX[a] for a in aux)
    s.pyb_freq = pyb_freq
    s.ctrl_freq = ctrl_freq if ctrl_freq is not None else (48 if task == "spiral" else 30)
    s.precision = precision
    s.flags = (0 if autoreset else 1) | {"cf2x": 0, "cf2p": 4}[str(getattr(drone_model, "value", drone_model))]   # QS_FLAG_CF2P
    s.env_offset = env_offset
    s.episode_len_sec = episode_len_sec if episode_len_sec is not None else (12.0 if task == "spiral" else 8.0)
    keep = None
    if initial_xyzs is not None:
        keep = np.ascontiguousarray(np.asarray(initial_xyzs, dtype=np.float64).reshape(num_drones, 3))
        s.initial_xyzs = keep.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
    s.spiral_radius = spiral_radius
    s.spiral_period = spiral_period
    s.height_rate = height_rate
    for i in range(3):
        s.target_center[i] = target_center[i]
    return s, keep


class OracleSim:
    """Host-side vectorised env with the same semantics as the HIP qs_handle."""

    def __init__(self, **kw):
        self._spec, self._keep = make_spec(**kw)
        self._h = ctypes.c_void_p()
        rc = lib().qso_create(ctypes.byref(self._spec), ctypes.byref(self._h))
        if rc != 0:
            raise ValueError(lib().qso_last_error().decode())
        d = QsDims()
        lib().qso_get_dims(self._h, ctypes.byref(d))
        self.dims = d
        self.E, self.D, self.N = d.num_envs, d.num_drones, d.num_agents
        self.A, self.O, self.H, self.S = d.act_dim, d.obs_dim, d.hist_len, d.substeps
        self.precision = d.precision
        self.rdtype = np.float64 if self.precision == 8 else np.float32

    def close(self):
        if self._h:
            lib().qso_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset(self, seed=0):
        obs = np.zeros((self.E, self.D, self.O), np.float32)
        lib().qso_reset(self._h, seed, _p(obs))
        return obs

    def step(self, actions=None, nthreads=1):
        E, D, O, A = self.E, self.D, self.O, self.A
        out = dict(obs=np.zeros((E, D, O), np.float32), reward=np.zeros(E, self.rdtype),
                   terminated=np.zeros(E, np.uint8), truncated=np.zeros(E, np.uint8),
                   terminal_obs=np.zeros((E, D, O), np.float32), reasons=np.zeros((E, D), np.uint8),
                   actions=np.zeros((E, D, A), np.float32))
        so = QsStepOut(_p(out["obs"]), _p(out["reward"]), _p(out["terminated"]), _p(out["truncated"]),
                       _p(out["terminal_obs"]), _p(out["reasons"]), _p(out["actions"]))
        act = None
        if actions is not None:
            act = np.ascontiguousarray(np.asarray(actions, np.float32).reshape(E, D, A))
        lib().qso_step(self._h, _p(act), ctypes.byref(so), nthreads)
        return out

    def reset_envs(self, mask=None):
        obs = np.zeros((self.E, self.D, self.O), np.float32)
        m = None if mask is None else np.ascontiguousarray(np.asarray(mask, np.uint8).reshape(self.E))
        lib().qso_reset_envs(self._h, _p(m), _p(obs))
        return obs

    def run_random(self, steps, nthreads):
        lib().qso_run_random(self._h, steps, nthreads)

    def get_state(self, block):
        buf = self._alloc(block)
        lib().qso_state_io(self._h, block, _p(buf), 0)
        return buf

    def set_state(self, block, buf):
        want = self._alloc(block)
        buf = np.ascontiguousarray(np.asarray(buf, dtype=want.dtype).reshape(want.shape))
        lib().qso_state_io(self._h, block, _p(buf), 1)

    def _alloc(self, block):
        if block == 0:
            return np.zeros((AGENT_FIELDS, self.N), self.rdtype)
        if block == 1:
            return np.zeros((ENV_FIELDS, self.E), np.int32)
        if block == 2:
            return np.zeros((self.H, self.N, self.A), np.float32)
        if block == 3:
            return np.zeros(self.E, np.float64)
        raise ValueError(block)

    def episode_log(self, cap=1 << 20):
        dst = np.zeros(cap, EPISODE_DTYPE)
        total = lib().qso_episode_log(self._h, _p(dst), cap)
        return dst[:min(total, cap)], total

    def reset_error(self):
        return lib().qso_reset_error(self._h)


# ---- unit-level helpers -----------------------------------------------------
def philox(ctr, key):
    c = np.asarray(ctr, np.uint32)
    k = np.asarray(key, np.uint32)
    o = np.zeros(4, np.uint32)
    lib().qso_philox4x32_10(_p(c), _p(k), _p(o))
    return o


def quat_to_matrix(q):
    q = np.asarray(q, np.float64)
    m = np.zeros(9)
    lib().qso_quat_to_matrix(_p(q), _p(m))
    return m.reshape(3, 3)


def euler_from_quat(q):
    q = np.asarray(q, np.float64)
    r = np.zeros(3)
    lib().qso_euler_from_quat(_p(q), _p(r))
    return r


def integrate_q(q, w, dt):
    q = np.array(q, np.float64)
    w = np.asarray(w, np.float64)
    lib().qso_integrate_q(_p(q), _p(w), dt)
    return q


def constants():
    o = np.zeros(8)
    lib().qso_constants(_p(o))
    keys = ["GRAVITY", "HOVER_RPM", "MAX_RPM", "MAX_THRUST", "GND_EFF_H_CLIP", "SPEED_LIMIT", "L_SQRT2", "INIT_Z"]
    return dict(zip(keys, o))


def dsl_pid(pid_state, cur_pos, cur_quat, cur_vel, target_pos, target_rpy=(0, 0, 0), target_vel=(0, 0, 0),
            ctrl_dt=1 / 30):
    st = np.array(pid_state, np.float64)
    rpm = np.zeros(4)
    a = [np.asarray(x, np.float64) for x in (cur_pos, cur_quat, cur_vel, target_pos, target_rpy, target_vel)]
    lib().qso_dsl_pid(_p(st), *[_p(x) for x in a], ctrl_dt, _p(rpm))
    return rpm, st


def gae(rews, vals, masks, terminal_vals, last_val, gamma=0.99, use_gae=True, lam=0.95):
    """rews/vals/masks/terminal_vals [T][N] float32, last_val [N] float32 → (rets, advs) float64."""
    arrs = [np.ascontiguousarray(np.asarray(x, np.float32)) for x in (rews, vals, masks, terminal_vals)]
    lv = np.ascontiguousarray(np.asarray(last_val, np.float32).reshape(-1))
    T = arrs[0].shape[0]
    N = int(np.prod(arrs[0].shape[1:]))
    rets = np.zeros((T, N))
    advs = np.zeros((T, N))
    lib().qso_gae(T, N, *[_p(x) for x in arrs], _p(lv), gamma, int(use_gae), lam, _p(rets), _p(advs))
    shape = arrs[0].shape
    return rets.reshape(shape), advs.reshape(shape)
