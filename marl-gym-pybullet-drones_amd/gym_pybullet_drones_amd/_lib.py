"""ctypes binding of libquadswarm.so — the C-ABI declared in include/quadswarm.h.

This is exactly the binding a maintainer would add on the reference side
(INTEGRATION.md): plain pointers, sizes and a hipStream_t, no torch types.
The library must be built in-tree (``__graft_entry__.build()``); importing the
product path without it raises — there is no CPU fallback.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("QS_DEV_LIB") or os.path.join(_HERE, "lib", "libquadswarm.so")   # QS_DEV_LIB: dev variant builds

QS_OK = 0
TASK_MULTIHOVER, TASK_SPIRAL, TASK_FLOCK, TASK_MEETUP, TASK_LEADERFOLLOWER = 0, 1, 2, 3, 4
ACT_RPM, ACT_PID, ACT_VEL, ACT_ONE_D_RPM, ACT_ONE_D_PID = 0, 1, 2, 3, 4
PHYS_PYB, PHYS_DYN = 0, 1
AUX_GND, AUX_DRAG, AUX_DW = 1, 2, 4
AGENT_FIELDS, ENV_FIELDS = 29, 4
STATE_AGENT, STATE_ENV, STATE_HISTORY, STATE_EP_RETURN = 0, 1, 2, 3
FLAG_NO_AUTORESET = 1
FLAG_INKERNEL_RESET_SEARCH = 2
FLAG_CF2P = 4   # DroneModel.CF2P (include/quadswarm.h QS_FLAG_CF2P)
REASON_CRASH, REASON_FLIP, REASON_OOB, REASON_ZRANGE = 1, 2, 4, 8

# agent field offsets (include/quadswarm.h)
F_POS, F_QUAT, F_VEL, F_RPY_RATES, F_LAST_RPM = 0, 3, 7, 10, 13
F_PID_INT_POS, F_PID_INT_RPY, F_PID_LAST_RPY, F_TARGET = 17, 20, 23, 26
E_STEP_COUNTER, E_EPISODE, E_TOTAL_STEPS, E_EP_LEN = 0, 1, 2, 3


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


EPISODE_DTYPE = np.dtype([("ret", "<f8"), ("len", "<i4"), ("env", "<i4"), ("seq", "<i8")])

# Every symbol include/quadswarm.h declares (tests check the .so exports them).
ABI_VERSION = 4   # include/quadswarm.h QS_ABI_VERSION
EXPORTS = ("qs_create", "qs_destroy", "qs_last_error", "qs_abi_version", "qs_get_dims", "qs_reset",
           "qs_reset_envs", "qs_step", "qs_state_io", "qs_episode_log", "qs_reset_error", "qs_calib_copy",
           # include/qs_learner.h
           "qs_gae", "qs_adam_gated", "qs_adam_commit", "qs_ppo_heads", "qs_ppo_heads_work_bytes",
           "qs_mlp_bias_tanh", "qs_mlp_bwd_blocks", "qs_mlp_tanh_bwd", "qs_mlp_sum_partials",
           "qs_mlp_sum_partials_multi", "qs_adam_step", "qs_mlp3_tiles", "qs_mlp3_pack_floats",
           "qs_mlp3_pack", "qs_mlp3_fwd", "qs_mlp3_fwd_rows", "qs_mlp3_fwd_group_rows", "qs_mlp3_bwd", "qs_mlp_wgrad", "qs_mlp_wgrad_chunks", "qs_adam_multi",
           "qs_adam_multi_pack", "qs_mlp_sum_adam", "qs_mlp_sum_adam_work_bytes", "qs_mlp3f_tiles", "qs_mlp3f_pack_floats", "qs_mlp3f_work_bytes",
           "qs_mlp3f_pack", "qs_mlp3f_actor", "qs_mlp3f_actor_w1", "qs_value_head", "qs_mlp_wgrad_x_chunks", "qs_mlp_wgrad_x",
           "qs_wgrad_rm", "qs_learner_last_error", "qs_rms_work_bytes", "qs_rms_update", "qs_rms_normalize",
           "qs_rms_last_error", "qs_mlp3_value_work_bytes", "qs_mlp3_fwd_rows_value", "qs_policy_sample", "qs_rollout_record", "qs_rollout_last_error", "qs_ppo_small_work_bytes", "qs_ppo_small_step", "qs_ppo_small_last_error",
           "qs_ppo_small_layout", "qs_ppo_critic_tiles", "qs_wgrad_t", "qs_ppo_small_grads", "qs_ppo_small_adam")
QS_PACK_F16 = 1 << 16   # pack_I flag: a qs_mlp3f_pack image (include/qs_learner.h)
QS_PACK_W2T = 1 << 17   # pack_I flag: a [256][256] W2ᵀ copy (include/qs_learner.h)
QS_PPO_SMALL_LAYOUT_N = 29   # include/qs_learner.h: entries qs_ppo_small_layout writes
QS_PPO_SMALL_MAX_ROWS = 16384   # include/qs_learner.h: mb·D at most on qs_ppo_small_step / _grads

_lib = None


class QsMlp256(ctypes.Structure):
    """include/qs_learner.h qs_mlp256: one 256-wide tanh MLP inside its flat Adam buffers."""
    _fields_ = [("params", ctypes.c_void_p), ("exp_avg", ctypes.c_void_p), ("exp_avg_sq", ctypes.c_void_p),
                ("step", ctypes.c_void_p), ("w2t", ctypes.c_void_p),
                ("w1", ctypes.c_int64), ("b1", ctypes.c_int64), ("w2", ctypes.c_int64), ("b2", ctypes.c_int64),
                ("w3", ctypes.c_int64), ("b3", ctypes.c_int64), ("logstd", ctypes.c_int64),
                ("in_", ctypes.c_int32), ("out", ctypes.c_int32),
                ("lr", ctypes.c_float), ("beta1", ctypes.c_float), ("beta2", ctypes.c_float), ("eps", ctypes.c_float),
                ("w1p", ctypes.c_void_p)]


class QuadSwarmError(RuntimeError):
    pass


def load():
    """Load libquadswarm.so (after torch, so both share one HIP runtime)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise QuadSwarmError(
            f"{LIB_PATH} is missing: build the HIP extension first "
            "(python -c 'import __graft_entry__ as g; g.build()'). There is no CPU fallback.")
    try:
        import torch  # noqa: F401  (registers libamdhip64.so.7 first)
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    vp, i32, i64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
    L.qs_last_error.restype = ctypes.c_char_p
    L.qs_abi_version.restype = i32
    if L.qs_abi_version() != ABI_VERSION:   # a stale build: its signatures differ from the argtypes below
        raise QuadSwarmError(f"{LIB_PATH} has ABI version {L.qs_abi_version()}, this package binds "
                             f"{ABI_VERSION}: rebuild the HIP extension")
    L.qs_create.argtypes = [ctypes.POINTER(QsSpec), i32, ctypes.POINTER(vp)]
    L.qs_destroy.argtypes = [vp]
    L.qs_get_dims.argtypes = [vp, ctypes.POINTER(QsDims)]
    L.qs_reset.argtypes = [vp, ctypes.c_uint64, vp, vp]
    L.qs_reset_envs.argtypes = [vp, vp, vp, vp]
    L.qs_step.argtypes = [vp, vp, ctypes.POINTER(QsStepOut), vp]
    L.qs_state_io.argtypes = [vp, i32, vp, i32, vp]
    L.qs_episode_log.argtypes = [vp, vp, i64, ctypes.POINTER(i64), ctypes.POINTER(i64), vp]
    L.qs_reset_error.argtypes = [vp, ctypes.POINTER(i32)]
    L.qs_calib_copy.argtypes = [vp, vp, i64, vp]
    L.qs_gae.argtypes = [ctypes.c_int32, i64, vp, vp, vp, vp, vp, ctypes.c_double, ctypes.c_double, ctypes.c_int32,
                         vp, vp, vp]
    f32 = ctypes.c_float
    L.qs_adam_gated.argtypes = [i64, vp, vp, vp, vp, vp, f32, f32, f32, f32, vp, f32, vp]
    L.qs_adam_commit.argtypes = [vp, vp, f32, vp]
    L.qs_ppo_heads.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, vp, vp, vp, f32, vp, vp, vp, vp, vp,
                               f32, f32, vp, vp, vp, vp, vp, vp, vp]
    L.qs_ppo_heads_work_bytes.argtypes = [ctypes.c_int32, ctypes.c_int32]
    L.qs_mlp_bias_tanh.argtypes = [i64, ctypes.c_int32, vp, vp, vp, ctypes.c_int32, vp, vp, vp, vp]
    L.qs_mlp_bwd_blocks.argtypes = [i64]
    L.qs_mlp_tanh_bwd.argtypes = [i64, ctypes.c_int32, vp, vp, ctypes.c_int32, vp, vp, vp, vp, vp]
    L.qs_mlp_sum_partials.argtypes = [ctypes.c_int32, i64, vp, vp, i64, vp, i64, vp, vp]
    L.qs_mlp_sum_partials_multi.argtypes = [ctypes.c_int32, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.qs_adam_step.argtypes = [i64, vp, vp, vp, vp, vp, f32, f32, f32, f32, vp, f32, vp, vp]
    L.qs_adam_multi.argtypes = [ctypes.c_int32] + [vp] * 14
    L.qs_mlp3_tiles.argtypes = [i64, i32]
    L.qs_mlp3_pack_floats.argtypes = [ctypes.c_int32]
    L.qs_mlp3_pack.argtypes = [ctypes.c_int32, ctypes.c_int32, vp, vp, vp, vp]
    L.qs_mlp3_fwd.argtypes = [i64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32] + [vp] * 10
    L.qs_mlp3_bwd.argtypes = [i64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32] + [vp] * 10
    L.qs_mlp3_fwd_rows.argtypes = [i64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32] + [vp] * 12
    L.qs_mlp_wgrad_chunks.argtypes = [i64, ctypes.c_int32, ctypes.c_int32]
    L.qs_mlp_wgrad_chunks.restype = ctypes.c_int32
    L.qs_mlp_wgrad.argtypes = [i64, ctypes.c_int32, ctypes.c_int32, vp, vp, ctypes.c_int32, ctypes.c_int32, vp, vp]
    L.qs_mlp3_fwd_group_rows.argtypes = [i64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, vp, vp,
                                         ctypes.c_int32] + [vp] * 9
    L.qs_adam_multi_pack.argtypes = [ctypes.c_int32] + [vp] * 16 + [ctypes.c_int32, vp, vp]
    L.qs_mlp_sum_adam.argtypes = [ctypes.c_int32] + [vp] * 9 + [ctypes.c_int32] + [vp] * 18
    L.qs_mlp3f_tiles.argtypes = [i64]
    L.qs_mlp3f_pack_floats.argtypes = [ctypes.c_int32]
    L.qs_mlp3f_work_bytes.argtypes = [i64]
    L.qs_mlp3f_pack.argtypes = [ctypes.c_int32, vp, vp, vp, vp]
    L.qs_mlp3f_actor.argtypes = ([i64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32] + [vp] * 8 + [f32] + [vp] * 3
                                 + [f32, f32] + [vp] * 12)
    L.qs_mlp3f_actor_w1.argtypes = ([i64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32] + [vp] * 8 + [f32] + [vp] * 3
                                    + [f32, f32] + [vp] * 13)
    L.qs_value_head.argtypes = [ctypes.c_int32, ctypes.c_int32] + [vp] * 7
    L.qs_mlp_wgrad_x_chunks.argtypes = [i64, ctypes.c_int32]
    L.qs_mlp_wgrad_x.argtypes = [i64, ctypes.c_int32, ctypes.c_int32, vp, ctypes.c_int32, vp, vp, vp]
    L.qs_wgrad_rm.argtypes = [i64, ctypes.c_int32, ctypes.c_int32, vp, vp, ctypes.c_int32, vp, vp]
    L.qs_learner_last_error.restype = ctypes.c_char_p
    L.qs_rms_last_error.restype = ctypes.c_char_p
    L.qs_rollout_last_error.restype = ctypes.c_char_p
    L.qs_mlp3_value_work_bytes.argtypes = [i64]
    L.qs_mlp3_fwd_rows_value.argtypes = [i64, ctypes.c_int32, ctypes.c_int32] + [vp] * 16
    L.qs_policy_sample.argtypes = [i64, ctypes.c_int32, vp, vp, f32, f32, ctypes.c_int32, vp, vp, vp, vp]
    L.qs_rollout_record.argtypes = [i64] + [vp] * 7
    L.qs_ppo_small_last_error.restype = ctypes.c_char_p
    L.qs_ppo_small_work_bytes.argtypes = [ctypes.c_int32] * 5
    L.qs_ppo_small_layout.argtypes = [ctypes.c_int32] * 5 + [vp, ctypes.c_int32]
    L.qs_ppo_critic_tiles.argtypes = [ctypes.c_int32, ctypes.c_int32, vp, vp, vp, ctypes.POINTER(QsMlp256), vp, vp, vp]
    L.qs_wgrad_t.argtypes = [i64, i64, ctypes.c_int32, ctypes.c_int32, vp, vp, ctypes.c_int32, vp, vp]
    L.qs_ppo_small_step.argtypes = ([ctypes.c_int32, ctypes.c_int32] + [vp] * 6 + [f32, f32, f32, ctypes.c_int32, f32]
                                    + [ctypes.POINTER(QsMlp256)] * 2 + [vp] * 4)
    L.qs_ppo_small_grads.argtypes = ([ctypes.c_int32, ctypes.c_int32] + [vp] * 6 + [f32, f32, f32]
                                     + [ctypes.POINTER(QsMlp256)] * 2 + [vp] * 6)
    L.qs_ppo_small_adam.argtypes = ([ctypes.c_int32, ctypes.c_int32] + [ctypes.POINTER(QsMlp256)] * 2 + [vp] * 2
                                    + [f32, ctypes.c_int32, f32] + [vp] * 3)
    L.qs_rms_work_bytes.argtypes = [i64, ctypes.c_int32]
    L.qs_rms_update.argtypes = [i64, ctypes.c_int32] + [vp] * 7
    L.qs_rms_normalize.argtypes = [i64, ctypes.c_int32, vp, vp, vp, ctypes.c_double, ctypes.c_double, vp, vp]
    for name in EXPORTS:
        if name not in ("qs_last_error", "qs_learner_last_error", "qs_rms_last_error", "qs_ppo_small_last_error",
                        "qs_rollout_last_error"):
            getattr(L, name).restype = i32
    L.qs_ppo_heads_work_bytes.restype = i64
    L.qs_mlp3_pack_floats.restype = i64
    L.qs_mlp3f_pack_floats.restype = i64
    L.qs_mlp3f_work_bytes.restype = i64
    L.qs_mlp_sum_adam_work_bytes.restype = i64
    L.qs_rms_work_bytes.restype = i64
    L.qs_mlp3_value_work_bytes.restype = i64
    L.qs_ppo_small_work_bytes.restype = i64
    L.qs_mlp_sum_adam_work_bytes.argtypes = []
    _lib = L
    return L


def check(rc, what=""):
    if rc != QS_OK:
        lib = load()
        if what.startswith("qs_rms"):
            msg = lib.qs_rms_last_error()
        elif what.startswith(("qs_policy_sample", "qs_rollout")):
            msg = lib.qs_rollout_last_error()
        elif what.startswith(("qs_ppo_small", "qs_ppo_critic", "qs_wgrad_t")):
            msg = lib.qs_ppo_small_last_error()
        elif what.startswith(("qs_gae", "qs_adam", "qs_ppo", "qs_mlp", "qs_wgrad", "qs_value")):
            msg = lib.qs_learner_last_error()
        else:
            msg = lib.qs_last_error()
        raise QuadSwarmError(f"{what} failed (rc={rc}): {msg.decode() if msg else ''}")


def ptr(t):
    """Device pointer of a torch tensor (or None)."""
    return None if t is None else ctypes.c_void_p(t.data_ptr())
