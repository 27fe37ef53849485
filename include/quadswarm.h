/*
 * quadswarm.h — C-ABI of the MI355X-native batched quadrotor-swarm step.
 *
 * This is the drop-in boundary for the reference's per-control-step drone
 * update.  In the reference that boundary is the pybullet
 * CPython extension plus the Python env classes that drive it:
 *
 *   reference interface replaced                        entry point here
 *   --------------------------------------------------  ------------------
 *   BaseAviary.__init__ (+ _parseURDFParameters)         qs_create
 *     gym_pybullet_drones/envs/BaseAviary.py:25-216, 985-1017
 *   BaseAviary.reset / MultiHoverAviary.reset            qs_reset
 *     BaseAviary.py:220-255, MultiHoverAviary.py:75-110
 *   BaseAviary.step (preprocess → PYB_STEPS_PER_CTRL     qs_step
 *     substeps → readback → obs/reward/term/trunc)
 *     BaseAviary.py:259-383, BaseRLAviary.py:160-239, 284-319,
 *     DSLPIDControl.py:82-259, MultiHoverAviary.py:128-268,
 *     SpiralAviary.py:82-196
 *   worker.step_env auto-reset                           qs_step (in-kernel)
 *     safe_control_gym/.../subproc_vec_env.py:188-206
 *   p.resetBasePositionAndOrientation / getBase*         qs_state_io
 *     BaseAviary.py:509-519, 865-875 (state injection / readback)
 *   VecRecordEpisodeStatistics.step_wait                 qs_episode_log
 *     safe_control_gym/.../record_episode_statistics.py:144-172
 *   BaseAviary.close (p.disconnect)                      qs_destroy
 *
 * Conventions
 *  - All array arguments of qs_reset/qs_step/qs_state_io/qs_episode_log are
 *    DEVICE pointers (HBM, from hipMalloc or a torch tensor's data_ptr()).
 *    `stream` is a hipStream_t passed as void*; every call is stream-ordered
 *    and asynchronous unless documented otherwise.
 *  - Agent index a = env * num_drones + drone.  Observation layout is
 *    [env][drone][obs_dim] float32 (the reference's per-env (D, O) float32
 *    obs stacked over envs, BaseRLAviary.py:315-319, SpiralAviary.py:146).
 *  - Actions are float32 [env][drone][act_dim] (the trainer's dtype).
 *  - Rewards are `real` = float (precision 4) or double (precision 8).
 *  - Errors: every function returns 0 on success or a negative QS_E_* code;
 *    qs_last_error() returns a thread-local message.  Nothing calls exit().
 *  - Threading: a handle is bound to one device, is not re-entrant, and must
 *    be used from one host thread at a time (one handle per rank).
 */
#ifndef QUADSWARM_H
#define QUADSWARM_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QS_ABI_VERSION 4   /* 2: qs_episode_log reports the records it wrote; 3: qs_ppo_small_layout takes
                              the caller's entry count; 4: QS_FLAG_CF2P */

/* ---- status codes ------------------------------------------------------ */
#define QS_OK 0
#define QS_E_INVALID (-1)   /* bad argument / unsupported configuration     */
#define QS_E_HIP (-2)       /* HIP runtime error (message has the HIP text)  */
#define QS_E_NOMEM (-3)     /* device allocation failed                      */
#define QS_E_STATE (-4)     /* handle in wrong state (e.g. step before reset) */

/* ---- enums mirroring gym_pybullet_drones/utils/enums.py:3-48 ------------ */
typedef enum {
  QS_TASK_MULTIHOVER = 0, /* MultiHoverAviary.py                          */
  QS_TASK_SPIRAL = 1,     /* SpiralAviary.py (SpiralFormationAviary)      */
  QS_TASK_FLOCK = 2,      /* FlockAviary.py                               */
  QS_TASK_MEETUP = 3,     /* MeetupAviary.py                              */
  QS_TASK_LEADERFOLLOWER = 4 /* LeaderFollowerAviary.py                   */
} qs_task;

typedef enum {            /* ActionType (enums.py:35-41)                   */
  QS_ACT_RPM = 0,
  QS_ACT_PID = 1,         /* waypoint via _calculateNextStep (BA:1108-1150) */
  QS_ACT_VEL = 2,
  QS_ACT_ONE_D_RPM = 3,
  QS_ACT_ONE_D_PID = 4
} qs_action_type;

typedef enum {            /* Physics (enums.py:13-21)                      */
  QS_PHYS_PYB = 0,        /* Bullet's step of BaseAviary._physics forces
                             (BA:679-711, 369-370), restated */
  QS_PHYS_DYN = 1         /* BaseAviary._dynamics (BA:815-892)            */
} qs_physics;

/* Extra force models: BaseAviary._groundEffect (BA:715-750), _drag
 * (BA:754-781), _downwash (BA:785-811).  With QS_PHYS_PYB they give the
 * reference's PYB_GND / PYB_DRAG / PYB_DW / PYB_GND_DRAG_DW; with
 * QS_PHYS_DYN they are added to the DYN force/torque sum (build-defined
 * combination, SURVEY §8 "Physics-mode note").                           */
#define QS_AUX_GND 1u
#define QS_AUX_DRAG 2u
#define QS_AUX_DW 4u

/* qs_spec.flags */
#define QS_FLAG_NO_AUTORESET 1u  /* single-env facade: BaseAviary.step never
                                    resets by itself (BaseAviary.py:259-383) */
#define QS_FLAG_INKERNEL_RESET_SEARCH 2u  /* MultiHover layouts that can reject:
                                    run the whole reset rejection loop
                                    (MultiHoverAviary.py:83-102) inside the
                                    step kernel, no deferred search launch
                                    (the validation form of the deferred one) */
#define QS_FLAG_CF2P 4u  /* DroneModel.CF2P, the + configuration (cf2p.urdf:
                                    inertia and prop links on the axes;
                                    BaseAviary.py:852-853 torques,
                                    DSLPIDControl.py:54-60 mixer); default
                                    DroneModel.CF2X */

typedef struct qs_spec {
  int32_t task;          /* qs_task                                        */
  int32_t num_envs;      /* E on this device (the rank's shard)            */
  int32_t num_drones;    /* D                                              */
  int32_t act_type;      /* qs_action_type                                 */
  int32_t physics;       /* qs_physics                                     */
  uint32_t aux_forces;   /* OR of QS_AUX_*                                 */
  int32_t pyb_freq;      /* 240 (BA:32)                                    */
  int32_t ctrl_freq;     /* MultiHover 30 (MH:20), Spiral 48 (SP:28)       */
  int32_t precision;     /* 4 = fp32 state/math, 8 = fp64 state/math       */
  uint32_t flags;        /* OR of QS_FLAG_*                                 */
  int64_t env_offset;    /* global id of env 0 (multi-GPU shard offset)    */
  double episode_len_sec;/* MH 8 (MH:58), SP 12 (SP:39)                    */
  /* [D][3] initial positions, or NULL for the reference default:
   *   MultiHover: diagonal grid x=y=i*4L, z=0.1125 (BA:194-197)
   *   Spiral: circle radius R at z=0.3 (SP:47-53)                         */
  const double* initial_xyzs;
  /* Spiral parameters (SP:33-45); ignored for MultiHover. */
  double spiral_radius;  /* 0.4  */
  double spiral_period;  /* 10.0 */
  double height_rate;    /* 0.05 */
  double target_center[3];
} qs_spec;

/* Derived sizes (BRL:66, 141-147, 262-277; SP:105-113). */
typedef struct qs_dims {
  int32_t num_envs, num_drones, num_agents;  /* N = E*D                   */
  int32_t act_dim;        /* A                                            */
  int32_t obs_dim;        /* O = 12 + H*A (+11 Spiral)                    */
  int32_t hist_len;       /* H = ctrl_freq // 2                           */
  int32_t substeps;       /* PYB_STEPS_PER_CTRL                           */
  int32_t precision;      /* 4 or 8                                       */
  int32_t agent_fields;   /* QS_AGENT_FIELDS                              */
  int32_t env_fields;     /* QS_ENV_FIELDS                                */
} qs_dims;

/* Per-agent state, structure-of-arrays [field][N] in `real` precision.
 * This is what BaseAviary keeps in pybullet + its numpy arrays
 * (BA:471-477, 509-519), plus DSLPIDControl's integrators
 * (DSLPIDControl.py:73-78) and MultiHover's TARGET_POS (MH:106).        */
enum {
  QS_F_POS = 0,        /* 3: x y z (world)                                */
  QS_F_QUAT = 3,       /* 4: x y z w (pybullet order, NOT renormalised)   */
  QS_F_VEL = 7,        /* 3: world linear velocity                        */
  QS_F_RPY_RATES = 10, /* 3: body angular rates, DYN (BA:477, 877)        */
  QS_F_LAST_RPM = 13,  /* 4: last_clipped_action (BA:372, 468)            */
  QS_F_PID_INT_POS = 17, /* 3: integral_pos_e (PID:190-192)               */
  QS_F_PID_INT_RPY = 20, /* 3: integral_rpy_e (PID:249-251)               */
  QS_F_PID_LAST_RPY = 23,/* 3: last_rpy (PID:247-248)                     */
  QS_F_TARGET = 26,    /* 3: MultiHover TARGET_POS (MH:72, 106)           */
  QS_AGENT_FIELDS = 29
};

/* Per-env int32 state [field][E]. */
enum {
  QS_E_STEP_COUNTER = 0, /* BaseAviary.step_counter (PYB steps, BA:382)   */
  QS_E_EPISODE = 1,      /* episodes started by this env (RNG counter)    */
  QS_E_TOTAL_STEPS = 2,  /* control steps ever taken (history ring head)  */
  QS_E_EP_LEN = 3,       /* VecRecordEpisodeStatistics.episode_length     */
  QS_ENV_FIELDS = 4
};

typedef enum {
  QS_STATE_AGENT = 0,    /* real  [QS_AGENT_FIELDS][N]                     */
  QS_STATE_ENV = 1,      /* int32 [QS_ENV_FIELDS][E]                       */
  QS_STATE_HISTORY = 2,  /* float [H][N][A] action ring (BRL:66-67, 187)   */
  QS_STATE_EP_RETURN = 3 /* double [E] episode_return accumulator          */
} qs_state_block;

/* Termination reason bits (MultiHoverAviary._computeTerminated MH:216-241). */
#define QS_REASON_CRASH 1u   /* z < 0.03                                  */
#define QS_REASON_FLIP 2u    /* |roll| > 1.2 or |pitch| > 1.2             */
#define QS_REASON_OOB 4u     /* |x| > 3 or |y| > 3                         */
#define QS_REASON_ZRANGE 8u  /* Spiral: z < 0.05 or z > 3 (SP:185-191)    */

typedef struct qs_handle qs_handle;

/* Optional outputs of one control step. Every pointer may be NULL. */
typedef struct qs_step_out {
  float* obs;            /* [E][D][O] float32 (post auto-reset obs)        */
  void* reward;          /* [E] real                                      */
  uint8_t* terminated;   /* [E]                                           */
  uint8_t* truncated;    /* [E]                                           */
  float* terminal_obs;   /* [E][D][O]: obs before auto-reset; only rows of
                            envs with terminated|truncated are written     */
  uint8_t* reasons;      /* [E][D] QS_REASON_* bits at the terminal state  */
  float* actions_out;    /* [E][D][A]: copy of the actions consumed
                            (useful with the random policy)                */
} qs_step_out;

/* Random policy: when `actions` is NULL, qs_step draws i.i.d. U(-1,1)
 * actions from Philox4x32-10(key=seed, counter=(env_total_steps,
 * global_env, 0, (1<<24)|drone)) — the synthetic workload of SURVEY §8(d). */

int qs_create(const qs_spec* spec, int device, qs_handle** out);
int qs_destroy(qs_handle* h);
const char* qs_last_error(void);
int qs_abi_version(void);
int qs_get_dims(const qs_handle* h, qs_dims* out);

/* Reset every env (episode 0 draws), as MAPPO.reset → VecEnv.reset does
 * (mappo.py:147-167).  Writes the initial obs if obs != NULL.  PID state,
 * action history and episode counters are zeroed only here (the reference
 * never resets them inside an episode boundary). */
int qs_reset(qs_handle* h, uint64_t seed, float* obs, void* stream);

/* env.reset() for the envs with mask[e] != 0 (mask: device uint8 [E], NULL =
 * all): MultiHoverAviary.reset semantics (MH:75-110) — new episode draw,
 * step_counter = 0; PID integrators and the action history persist, as in
 * the reference.  Writes obs rows of the reset envs if obs != NULL. */
int qs_reset_envs(qs_handle* h, const uint8_t* mask, float* obs, void* stream);

/* One control step of every env: the reference's BaseAviary.step for all
 * envs + the worker's auto-reset.  actions: [E][D][A] float32 or NULL. */
int qs_step(qs_handle* h, const float* actions, const qs_step_out* out,
            void* stream);

/* Copy a state block between the handle and `buf` (device pointer).
 * dir = 0: handle → buf (get), dir = 1: buf → handle (set). */
int qs_state_io(qs_handle* h, int block, void* buf, int dir, void* stream);

/* Completed-episode log: a ring per env (max(8, 65536 / num_envs) slots,
 * appended in-kernel on done, no atomics).  Each record: {double return;
 * int32 length; int32 env; int64 seq}: seq = the step index at which it
 * completed.  qs_episode_log merges the rings in (seq, env) order — the
 * order the reference's env loop logs them — copies up to `cap` most-recent
 * records to `dst` (device) and writes the total number of episodes ever
 * logged to *total and the number of records written to dst to *written
 * (host, synchronous; written may be NULL): fewer than min(total, cap) when
 * rings dropped episodes.  The selection runs on the device
 * (a seq-distance histogram, then a compaction): O(cap) records cross to the
 * host, and cap = 0 reads back the total alone.  An env that completes more episodes
 * than its ring holds between two reads keeps only its latest ones. */
typedef struct qs_episode_rec {
  double ret;
  int32_t len;
  int32_t env;
  int64_t seq;
} qs_episode_rec;
int qs_episode_log(qs_handle* h, qs_episode_rec* dst, int64_t cap,
                   int64_t* total, int64_t* written, void* stream);

/* 1 if an in-kernel reset rejection search hit its try cap (2^24) since the
 * last qs_reset (synchronous). */
int qs_reset_error(qs_handle* h, int* out);

/* Diagnostics: a dword-per-lane copy with the same access pattern as the
 * step kernel's SoA loads/stores; used to calibrate rocprofv3 FETCH_SIZE /
 * WRITE_SIZE on gfx950 (MI355X_MICROARCH.md §HBM). */
int qs_calib_copy(float* dst, const float* src, int64_t n, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* QUADSWARM_H */
