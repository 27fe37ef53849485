"""Benchmark: agent-steps/s of the batched quadrotor-swarm control step on MI355X.

Workload (BASELINE.json configs[2], the metric's config, fits one GPU):
MultiHover, 8 drones, 16 384 envs per GPU, ActionType.ONE_D_PID (learn_mappo.py
default), Physics.DYN, fp32, synthetic random-policy rollout (Philox U(-1,1)
actions drawn in-kernel), obs written into an on-device rollout
buffer slot each step.  A "step" = one control step of every env on the rank
(one fused HIP launch: action→PID→8 substeps→obs/reward/done/auto-reset).

Steady state: after the reset the envs' episode clocks are staggered uniformly
over the 242-step MultiHover episode (578 for Spiral), as in a long-running
vectorised rollout whose envs have drifted apart, so any timed window of K steps
holds K/242 of the envs' truncations and auto-resets.  The default K = 484 is two
full episodes; `--steps K` is honoured exactly.

Multi-GPU: `python bench.py --gpus N` (no WORLD_SIZE in the environment) starts
`torch.distributed.run --nproc-per-node N` on this script as a child process
before anything touches a GPU, and exits with its status; under torchrun (the
driver's form) each rank runs directly.  Envs are sharded (weak scaling, 16 384
envs per rank, global env ids offset by rank) with no data-path collective;
value = all ranks' agent-steps ÷ max-over-ranks wall time.

Extra JSON fields:
  pyb           the same rollout under Physics.PYB (the kernel's restatement of
                Bullet's step, the reference's training default).
  mappo         full MAPPO on the same C3 envs (BASELINE config 3) with the
                reference's rollout length T = 256 (learn_mappo.py:665): agent-steps/s
                of MAPPO.train_step = T-step rollout with the shared actor + simulator,
                last value, GAE, advantage normalisation and the PPO update
                (10 epochs x T·E/mini_batch_size minibatches, centralized critic) —
                SURVEY §8(d)'s "full MAPPO" figure; with N ranks the gradients are
                all-reduced.  `learner_roofline`: the update's algorithmic fp32 FLOP
                (MLP forward + backward, counted in DESIGN.md §4c) ÷ its device time
                vs the 157.3 TFLOP/s fp32 MFMA peak.
  mappo_t32     the same with T = 32 (round-1 leg, kept for comparison).
  roofline      the step kernel: §8(d) algorithmic bytes per agent-step (418 B,
                C3 ONE_D_PID) × agents per launch ÷ mean launch time from HIP
                events on the launch stream, vs 8 TB/s.
  configs       the other BASELINE.json configs (C2, C3 with ActionType.VEL, C4
                Spiral, C5 16-drone with the O(D²) downwash under Physics.PYB_DW),
                each a random-policy rollout on one GPU: agent-steps/s, kernel ms
                and roofline fraction with that config's §8(d) bytes per agent-step.
  cpu_baseline  the oracle (C++ CPU restatement of the reference semantics,
                fp64 like the reference) on 176 envs (README's 22-worker
                topology) timed on this host, rank 0 only.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "marl-gym-pybullet-drones_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from gym_pybullet_drones_amd.envs.swarm import grid_layout  # noqa: E402

METRIC = "agent-steps/sec, MultiHover 8-drone MAPPO @ 1/2/4/8 GPU vs PyBullet CPU"


def bytes_per_agent_step(act="one_d_pid", task="multihover", D=8, precision=4):
    """SURVEY §8(d)'s algorithmic HBM bytes per agent-step, per field, with each
    field in the step kernel's own buffer type (csrc/step_kernel.h Params): the
    agent state st, the MultiHover target and the reward are `real` (float32, or
    float64 in the precision-8 build); the action, the action history and the
    obs are float32 in both builds (BRL:307-319 emits a float32 obs once the
    history holds float32 actions).  Per drone: action A read; state S read +
    written (S = 29 with the PID state of the PID action types, else 20); target
    3 read (MultiHover only); history H·A (the H−1 older entries read, one
    written); obs O written.  Per env, over its D drones: the step counter
    read + written (8 B), the reward, two flag bytes."""
    real = 8 if precision == 8 else 4
    A = {"one_d_pid": 1, "one_d_rpm": 1, "rpm": 4, "vel": 4, "pid": 3}[act]
    H = 24 if task == "spiral" else 15            # ctrl 48 Hz / 30 Hz: BRL:66 (SURVEY §8 derived sizes)
    O = 12 + H * A + (11 if task == "spiral" else 0)
    S = 29 if act in ("one_d_pid", "vel", "pid") else 20
    target = 3 * real if task != "spiral" else 0
    per_drone = 4 * A + 2 * S * real + target + 4 * H * A + 4 * O
    per_env = 8 + real + 2
    return per_drone + per_env / D


BYTES_PER_AGENT_STEP = {a: bytes_per_agent_step(a) for a in ("one_d_pid", "vel", "rpm")}   # D = 8: 417.75 / 789.75 / 717.75
HBM_PEAK_GBS = 8000.0
CPU_WORKERS = 22   # the reference's num_workers (README.md:38-39: 22 workers x 8 envs)
FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: f32-input MFMA = the f32 vector rate
EPISODE_STEPS = {"multihover": 242, "spiral": 578}   # SURVEY §8 derived sizes


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=484, help="timed control steps (default: two MultiHover episodes)")
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--envs", type=int, default=16384, help="envs per GPU")
    p.add_argument("--drones", type=int, default=8)
    p.add_argument("--act", default="one_d_pid")
    p.add_argument("--slots", type=int, default=32, help="rollout-buffer slots the obs ring cycles through")
    p.add_argument("--graph-steps", type=int, default=512, help="control steps per captured HIP graph of the sim legs")
    p.add_argument("--no-stagger", action="store_true", help="start every env at episode step 0")
    p.add_argument("--rehearse", type=int, default=16,
                   help="untimed passes of the timed window's graphs right before it (a 20-step window measured "
                        "10.85 -> 10.28 us per step at 16: the first window after the setup ran cold; 256 passes "
                        "measured slower, the sustained-load clock)")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample length")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--mappo", type=int, default=1, help="also time full MAPPO train steps (0 = skip)")
    p.add_argument("--pyb", type=int, default=1, help="also time the rollout under Physics.PYB (0 = skip)")
    p.add_argument("--fp64", type=int, default=1,
                   help="also time the headline rollout in float64, the reference's own precision (0 = skip)")
    p.add_argument("--configs", type=int, default=1, help="also time BASELINE configs C2, C3-VEL, C4, C5 (N=1 only)")
    p.add_argument("--mappo-steps", type=int, default=256, help="rollout_steps T of the MAPPO leg (learn_mappo.py:665)")
    p.add_argument("--mappo-mb", type=int, default=4096, help="mini_batch_size (env-timesteps) of the MAPPO legs")
    p.add_argument("--mappo-iters", type=int, default=2, help="timed train steps (after one warm-up)")
    p.add_argument("--mappo-t32", type=int, default=1, help="also time the T=32 MAPPO leg (0 = skip)")
    p.add_argument("--mappo-configs", default="C4,C5,ref",
                   help="also time these MAPPO_LEGS trainer configs at N=1 ('' = none)")
    p.add_argument("--wgrad", default="", help="learner weight gradients on the MFMA qs_mlp_wgrad kernel (w1,w2; '' = GEMMs)")
    p.add_argument("--splitk", default="", help="learner split-K chunk rows per weight-gradient shape, 'KxM=rows,...'")
    p.add_argument("--side-stream", type=int, default=1, help="learner: critic kernels on a second stream (0 = one stream)")
    p.add_argument("--w1-stream", type=int, default=1, help="learner: actor dW1 GEMM on a third stream beside dW2")
    p.add_argument("--fused-max-a", type=int, default=None,
                   help="learner: widest actor output on the fused actor kernel (default: the agent's _F16_MAX_A)")
    p.add_argument("--critic-tiles", type=int, default=0,
                   help="learner: the critic on qs_ppo_critic_tiles + qs_wgrad_t (0 = qs_mlp3w kernels + GEMMs)")
    p.add_argument("--small-rows", type=int, default=None,
                   help="learner: minibatches of at most this many actor rows on qs_ppo_small_step (0 = never)")
    p.add_argument("--critic-adam-side", type=int, default=0,
                   help="learner: the critic's sums + Adam on the side stream (0 = one launch after the join)")
    p.add_argument("--strong", type=int, default=1,
                   help="with N > 1 ranks: also time SURVEY §8(e)'s strong partitions of configs 3-5 (0 = skip)")
    p.add_argument("--rank-shapes", default="C3/2,C3/4,C3/8,C4/4,C5/8",
                   help="N = 1: one rank's share of these STRONG_LEGS partitions ('name/G'), timed through the "
                        "exchange path on a world-1 group ('' = skip)")
    p.add_argument("--assumed-allreduce-us", type=float, default=30.0,
                   help="G-GPU all-reduce latency assumed in the rank-shape projections (and twice it)")
    p.add_argument("--dry-run", action="store_true", help="rank plumbing only: gloo on CPU, stand-in steps, no GPU")
    p.add_argument("--dry-ms", type=float, default=2.0, help="--dry-run: ms per stand-in step of rank 0 (rank r: (1+r)x)")
    return p.parse_args()


def progress(msg):
    """A progress line on stderr (the JSON line alone goes to stdout)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n):
    """--gpus N without a launcher: run N ranks of this script under torchrun as a
    child process (never an exec) and return its exit status.  Nothing here has
    touched a GPU."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


class Ranks:
    """The bench's rank plumbing: the torchrun environment, the process group (RCCL;
    gloo on CPU tensors for --dry-run), barrier + device-sync fences around a timed
    window, and the MAX of a duration over ranks."""

    def __init__(self, dry=False):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.dry = dry
        self.dist = None
        if not dry:
            torch.cuda.set_device(self.local)
        if self.world > 1:
            import torch.distributed as dist
            if dry:
                dist.init_process_group("gloo")
            else:
                dist.init_process_group("nccl", device_id=torch.device("cuda", self.local))
            self.dist = dist

    def sync(self):
        if not self.dry:
            torch.cuda.synchronize()

    def fence(self):
        """Every rank's queued work done, then all ranks together."""
        self.sync()
        if self.dist:
            # the barrier is itself device work under RCCL: drain it too (one rank
            # has nothing to wait for, so its window ends at the first sync)
            self.dist.barrier()
            self.sync()

    def max(self, seconds):
        if not self.dist:
            return seconds
        t = torch.tensor([seconds], dtype=torch.float64, device="cpu" if self.dry else "cuda")
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def close(self):
        if self.dist:
            # every MAPPO leg released its HIP graphs (MAPPO.close -> release_graphs:
            # they hold captured RCCL all-reduces, which must not outlive the
            # communicator); drain the device before it goes
            self.sync()
            self.dist.destroy_process_group()


def dry_leg(args, ranks):
    """--dry-run: the rank plumbing of a sim leg with no GPU (gloo, CPU).  Each
    control step is a CPU stand-in that takes (1 + rank)·--dry-ms: the fences make
    every rank's window hold the slowest rank's work, and the reported time is the
    MAX of the ranks' windows (tests/test_bench_ranks.py checks both)."""
    def busy(sec):
        t_end = time.perf_counter() + sec
        while time.perf_counter() < t_end:
            pass
    per_step = (1 + ranks.rank) * args.dry_ms * 1e-3
    for _ in range(args.warmup):
        busy(per_step)
    ranks.fence()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        busy(per_step)
    ranks.fence()
    mine = time.perf_counter() - t0
    every = [mine]
    if ranks.dist:   # each rank's own window, reported beside the max
        t = [torch.zeros(1, dtype=torch.float64) for _ in range(ranks.world)]
        ranks.dist.all_gather(t, torch.tensor([mine], dtype=torch.float64))
        every = [float(x) for x in t]
    return every, ranks.max(mine)


def _ppid(pid):
    with open(f"/proc/{pid}/stat") as f:
        return int(f.read().rsplit(")", 1)[1].split()[1])


def cpu_baseline(args, seconds, task="multihover", D=None, act=None, physics="dyn", aux=(), extra22=False):
    """The oracle (C++ restatement of the reference step, fp64) timed on this host's
    cores at the reference's 176 envs (README.md:38-39: 22 workers x 8 envs) on the
    same task, D, action type and physics as a GPU leg (BASELINE.md:36): a bounded
    sample of about `seconds`."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import qs_oracle
    D = D or args.drones
    act = act or args.act
    # the reference topology: 22 workers x 8 envs (README.md:38-39, BASELINE.md:35-37)
    # on at most the CPUs this process may use: min(22, affinity CPUs, the cgroup
    # quota) OpenMP threads (22 threads on a 16-CPU quota were
    # throttled, which understated the CPU path); `extra22` also times 22 threads
    # oversubscribed, as a labelled extra
    host = host_cpu()
    threads = max(1, min(CPU_WORKERS, host["nproc"] or CPU_WORKERS,
                         int(host["cpu_quota"]) if host["cpu_quota"] else CPU_WORKERS))
    E = 176
    ophys, oaux = ("pyb", ("dw",)) if physics == "pyb_dw" else (physics, tuple(aux))
    kw = dict(initial_xyzs=grid_layout(D)) if task == "multihover" and D >= 6 else {}
    sim = qs_oracle.OracleSim(task=task, num_envs=E, num_drones=D, act=act, precision=8, physics=ophys, aux=oaux,
                              **kw)
    sim.reset(0)
    sim.run_random(2, threads)   # warm the thread pool
    # doubling chunks until the budget is spent: a step's cost changes over an
    # episode (C2's resets run the rejection loop), so no calibration from the first steps
    steps, chunk, dt = 0, 4, 0.0
    while dt < seconds:
        t0 = time.perf_counter()
        sim.run_random(chunk, threads)
        dc = time.perf_counter() - t0
        dt += dc
        steps += chunk
        # next chunk: double, but no longer than the rest of the budget at the last chunk's rate
        chunk = max(1, min(2 * chunk, int((seconds - dt) / max(dc / chunk, 1e-9)) + 1))
    out22 = None
    if extra22 and threads < CPU_WORKERS:   # the 22-worker topology oversubscribed (labelled extra)
        s22, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < seconds / 3:
            sim.run_random(8, CPU_WORKERS)
            s22 += 8
        out22 = {"value": E * D * s22 / (time.perf_counter() - t0), "threads": CPU_WORKERS,
                 "note": "22 OpenMP threads on fewer CPUs (oversubscribed): not the baseline"}
    sim.close()
    host["threads"] = threads
    host["oversubscribed"] = threads > min(host["nproc"] or threads, host["cpu_quota"] or threads)
    out = {"value": E * D * steps / dt, "unit": "agent-steps/s", "cores": threads, "kind": "port",
           "host": host,
           "sample": f"C++ oracle (CPU restatement of the reference step, fp64, not PyBullet), {task} {E} envs x "
                     f"{D} drones ({CPU_WORKERS} reference workers' envs), {act}, "
                     f"{physics}{'+' + '+'.join(aux) if aux else ''}, {steps} random-policy "
                     f"ctrl steps, OpenMP {threads} threads (this process's CPU share), {dt:.1f} s"}
    if out22:
        out["oversubscribed_22"] = out22
    return out


def host_cpu():
    """The CPU the baseline ran on (BASELINE.md:37): model name and the logical
    CPUs this process may use (os.cpu_count() reports the whole machine's)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), None)
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count()
    quota = None
    try:   # cgroup v2 CPU quota ("max" = none): the box's CPU share
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        quota = None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        pass
    return {"cpu_model": model, "nproc": usable, "machine_cpus": os.cpu_count(), "cpu_quota": quota,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def pmc_traffic(E, D, act, precision=4):
    """HBM bytes per step-kernel launch from the newest committed PMC summary of this
    workload (profiles/rNN_pmc_traffic*.json: FETCH_SIZE/WRITE_SIZE passes, calibrated;
    scripts/gpu_prof.sh, scripts/r05_pmc64.sh).  The counters need rocprofv3 around
    the process, so the bench reports the committed measurement of the same kernel
    and names its source.  precision 8: the fp64 kernel's summary."""
    import glob
    best = None
    want = {"envs": E, "drones": D, "act": act}
    if precision != 4:
        want["precision"] = precision
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic*.json"))):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("workload") == want:
            best = (f, d)
    if best is None:
        return None, None
    return best[1]["step_traffic_bytes"], os.path.relpath(best[0], ROOT)


# BASELINE.json configs other than the headline one, each timed as its own
# random-policy rollout on one rank (bytes per agent-step: SURVEY §8(d)).
EXTRA_CONFIGS = {
    "C2": dict(task="multihover", drones=4, envs=4096, act="rpm", physics="dyn", aux=(),
               bytes=bytes_per_agent_step("rpm", "multihover", 4),
               label="MultiHover 4-drone x 4096 envs, ActionType.RPM, Physics.DYN"),
    "C3_vel": dict(task="multihover", drones=8, envs=16384, act="vel", physics="dyn", aux=(),
                   bytes=bytes_per_agent_step("vel", "multihover", 8),
                   label="MultiHover 8-drone x 16384 envs, ActionType.VEL, Physics.DYN"),
    "C4": dict(task="spiral", drones=5, envs=8192, act="vel", physics="dyn", aux=(),
               bytes=bytes_per_agent_step("vel", "spiral", 5),
               label="Spiral 5-drone x 8192 envs, ActionType.VEL, Physics.DYN"),
    "C5": dict(task="multihover", drones=16, envs=8192, act="one_d_pid", physics="pyb_dw", aux=(),
               bytes=bytes_per_agent_step("one_d_pid", "multihover", 16),
               label="MultiHover 16-drone x 8192 envs, ActionType.ONE_D_PID, Physics.PYB_DW (O(D^2) downwash)"),
}


def stagger_episodes(sw, task):
    """Spread the envs' episode clocks uniformly over one episode (steady state of a
    long vectorised rollout): env e starts at control step ⌊e·L/E⌋ of its episode."""
    from gym_pybullet_drones_amd import _lib as L
    E, L_ep = sw.num_envs, EPISODE_STEPS.get(task, 242)
    env = sw.get_state(L.STATE_ENV).clone()
    phase = (torch.arange(E, device=env.device, dtype=torch.int64) * L_ep // E).to(torch.int32)
    env[L.E_STEP_COUNTER] = phase * sw.substeps
    env[L.E_EP_LEN] = phase
    sw.set_state(L.STATE_ENV, env)


def sim_leg(args, ranks, physics="dyn", task="multihover", E=None, D=None, act=None, aux=(), precision=4):
    """The timed random-policy rollout: exactly `args.steps` control steps of E envs
    per rank, as replays of HIP graphs of step launches (one per rollout-buffer slot).
    Returns (agent-steps/s over all ranks, max-over-ranks seconds, mean step-kernel
    ms on the launch stream, steps, resets inside the timed window)."""
    from gym_pybullet_drones_amd.envs import QuadSwarm
    from gym_pybullet_drones_amd.utils.enums import Physics
    E = args.envs if E is None else E
    D = args.drones if D is None else D
    act = args.act if act is None else act
    phys = {"dyn": Physics.DYN, "pyb": Physics.PYB, "pyb_dw": Physics.PYB_DW}[physics]
    layout = grid_layout(D) if (D >= 6 and task == "multihover") else None
    sw = QuadSwarm(task, num_envs=E, num_drones=D, act=act, precision=precision, physics=phys, aux=aux,
                   initial_xyzs=layout, env_offset=ranks.rank * E)
    O, A = sw.obs_dim, sw.act_dim
    slots = max(1, min(args.slots, args.steps))
    obs_buf = torch.empty((slots, E, D, O), dtype=torch.float32, device=sw.device)
    act_buf = torch.empty((slots, E, D, A), dtype=torch.float32, device=sw.device)
    rew_buf = torch.empty((slots, E), dtype=sw.reward.dtype, device=sw.device)   # the kernel's `real`
    te_buf = torch.zeros((slots, E), dtype=torch.uint8, device=sw.device)
    tr_buf = torch.zeros((slots, E), dtype=torch.uint8, device=sw.device)
    sw.reset(0, obs=obs_buf[0])
    if not args.no_stagger:
        stagger_episodes(sw, task)
    done_count = torch.zeros((), dtype=torch.int64, device=sw.device)

    def step(k):
        sw.step(None, obs=obs_buf[k], reward=rew_buf[k], terminated=te_buf[k], truncated=tr_buf[k],
                actions_out=act_buf[k])

    for t in range(args.warmup):
        step(t % slots)
    torch.cuda.synchronize()
    # The rollout loop is captured as HIP graphs of up to --graph-steps step launches
    # each (the obs ring cycling through its `slots` buffers inside a graph), so that
    # exactly `steps` run: a window of 484 steps is one replay, not 16 (each graph
    # boundary cost ~9 µs of idle device time between the replays)
    # (no collective inside the window's graph: the fences' eager barriers stay on the default group)
    gsteps = max(1, min(args.graph_steps, args.steps))
    n_full, rem = divmod(args.steps, gsteps)
    stream = torch.cuda.Stream()
    graphs = []
    for n in ([gsteps] if n_full else []) + ([rem] if rem else []):
        g = torch.cuda.CUDAGraph()
        # thread_local: with N ranks the RCCL watchdog thread may query the fences' events during the capture
        with torch.cuda.graph(g, stream=stream, capture_error_mode="thread_local"):
            for k in range(n):
                step(k % slots)
        graphs.append((g, n))
    torch.cuda.synchronize()
    # one untimed replay of each graph: a graph's first launch also uploads it to
    # the device (at --steps 20 that upload was 2 µs of every timed step)
    for g, _ in graphs:
        g.replay()
    torch.cuda.synchronize()
    plan = [graphs[0]] * n_full + ([graphs[-1]] if rem else [])
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in plan]
    cur = torch.cuda.current_stream()
    for a, b in ev:   # a torch Event creates its HIP event at its first record: not inside the window
        a.record(cur)
        b.record(cur)
    # --rehearse untimed passes of the window itself (the same events and replays)
    # right before it, so the timed pass is not the first after the setup's idle
    # device; the episodes they end are not counted
    _, ended0 = sw.episode_log(cap=0)
    for _ in range(args.rehearse):
        for (g, n), (a, b) in zip(plan, ev):
            a.record(cur)
            g.replay()
            b.record(cur)
    ranks.fence()
    _, ended_r = sw.episode_log(cap=0)   # (episodes the rehearsals ended: not the window's)
    ranks.fence()
    t0 = time.perf_counter()
    for (g, n), (a, b) in zip(plan, ev):
        a.record(cur)
        g.replay()
        b.record(cur)
    ranks.fence()
    elapsed = time.perf_counter() - t0
    # mean step-kernel duration on the launch stream: graph time / launches per graph
    kern_ms = float(sum(a.elapsed_time(b) for a, b in ev)) / args.steps
    elapsed = ranks.max(elapsed)
    # sanity of the window: every reset succeeded, outputs finite, episodes ended in it
    assert sw.reset_error() == 0
    assert torch.isfinite(obs_buf).all()
    _, ended1 = sw.episode_log(cap=0)
    del graphs, plan
    sw.close()
    return E * D * ranks.world * args.steps / elapsed, elapsed, kern_ms, args.steps, int(ended1 - ended_r)


def mappo_flops(T, E, D, O, A, H=256, epochs=10):
    """Algorithmic fp32 FLOP of one MAPPO train step: the update's
    MLP forward + backward over epochs × T·E env-timesteps (actor on D agent rows of
    O inputs each, centralized critic on one row of D·O), and the rollout's actor
    forwards.  2 FLOP per MAC; the first layer has no input gradient."""
    actor_row = 2 * (2 * O * H + 3 * H * H + 3 * H * A)
    critic_row = 2 * (2 * D * O * H + 3 * H * H + 3 * H)
    update = epochs * T * E * (D * actor_row + critic_row)
    rollout = T * E * D * 2 * (O * H + H * H + H * A)
    return update, rollout


# MAPPO trainer configurations beside the headline leg (C3 envs, learn_mappo.py
# hyper-parameters): the reference's other trainer script on the Spiral config,
# the 16-drone PYB_DW config, and the reference's own learner shape (176 envs,
# mini_batch_size 32).  Keys: MAPPO constructor overrides + the env.
LEARN_MAPPO = dict(clip_param=0.2, entropy_coef=0.005, action_scale=0.25, clip_obs=100)   # learn_mappo.py:207-216
MAPPO_LEGS = {
    # env_select_learn_mappo.py:262-283: T=64, mini_batch_size 32 (here 4 096 env-timesteps, as the
    # headline leg), clip 0.1, entropy 5e-4, action_scale 0.4, norm_obs (reference_compat off: the
    # rollout graph; the compat quirk re-normalises done steps on the host)
    "C4": dict(task="spiral", drones=5, envs=8192, act="vel", physics="dyn", T=64, mb=4096, norm_obs=True,
               clip_param=0.1, entropy_coef=0.0005, action_scale=0.4, clip_obs=10, reference_compat=False,
               label="Spiral 5-drone x 8192 envs, VEL, DYN; env_select_learn_mappo.py:262-283"),
    "C5": dict(task="multihover", drones=16, envs=8192, act="one_d_pid", physics="pyb_dw", T=256, mb=4096,
               **LEARN_MAPPO, label="MultiHover 16-drone x 8192 envs, ONE_D_PID, PYB_DW; learn_mappo.py:196-216"),
    # learn_mappo.py:196-216 at the README's 176 envs: 1 408 minibatches of 32 env-timesteps per epoch
    "ref": dict(task="multihover", drones=8, envs=176, act="one_d_pid", physics="dyn", T=256, mb=32,
                **LEARN_MAPPO, label="MultiHover 8-drone x 176 envs, ONE_D_PID, DYN, mini_batch_size 32 (the reference's "
                      "learner shape, README.md:38-39, learn_mappo.py:196-216)"),
}


# SURVEY §8(e)'s partitions of BASELINE.json configs 3-5 over the ranks of a run
# (strong scaling: the global env batch and the global minibatch are fixed, each
# rank holds 1/G of both and the gradients are all-reduced per minibatch).  At
# G = 8 the C3 and C5 legs are exactly configs[2] and configs[4]; at G = 4 the
# C4 leg is configs[3].
STRONG_LEGS = {
    "C3": dict(task="multihover", drones=8, global_envs=16384, act="one_d_pid", physics="dyn", T=256,
               global_mb=4096, **LEARN_MAPPO,
               label="MultiHover 8-drone x 16384 envs (BASELINE configs[2]); learn_mappo.py:196-216"),
    "C4": dict(task="spiral", drones=5, global_envs=8192, act="vel", physics="dyn", T=64, global_mb=4096,
               norm_obs=True, clip_param=0.1, entropy_coef=0.0005, action_scale=0.4, clip_obs=10,
               reference_compat=False,
               label="Spiral 5-drone x 8192 envs (BASELINE configs[3]); env_select_learn_mappo.py:262-283"),
    "C5": dict(task="multihover", drones=16, global_envs=8192, act="one_d_pid", physics="pyb_dw", T=256,
               global_mb=4096, **LEARN_MAPPO,
               label="MultiHover 16-drone x 8192 envs, PYB_DW (BASELINE configs[4]); learn_mappo.py:196-216"),
}
STRONG_SIM = {"C3": ("one_d_pid", "dyn", "multihover", 8, 16384, bytes_per_agent_step("one_d_pid", "multihover", 8)),
              "C4": ("vel", "dyn", "spiral", 5, 8192, bytes_per_agent_step("vel", "spiral", 5)),
              "C5": ("one_d_pid", "pyb_dw", "multihover", 16, 8192, bytes_per_agent_step("one_d_pid", "multihover", 16))}


def leg_plan(args, world):
    """The legs a run of `world` ranks times, in order: (kind, name, scaling, per-rank
    envs, per-rank mini_batch_size or None).  world 1: the headline, PYB, the MAPPO
    legs (C3 at T = 256 and 32, the C4 / C5 / reference-shape trainer configs) and
    the other BASELINE configs' rollouts.  world > 1: the headline and the MAPPO C3
    leg weak-scaled (16 384 envs per rank, as at world 1), the C4 / C5 trainer and
    rollout legs weak-scaled beside them, and §8(e)'s strong partitions of
    configs 3-5 (STRONG_LEGS / STRONG_SIM)."""
    plan = [("sim", "headline", "weak", args.envs, None)]
    if args.fp64:
        plan.append(("sim", "fp64", "weak", args.envs, None))
    if args.pyb:
        plan.append(("sim", "pyb", "weak", args.envs, None))
    if args.mappo:
        plan.append(("mappo", "C3", "weak", args.envs, args.mappo_mb))
        if args.mappo_t32 and world == 1:
            plan.append(("mappo", "C3_t32", "weak", args.envs, args.mappo_mb))
        for k in filter(None, args.mappo_configs.split(",")):
            if k in MAPPO_LEGS and (world == 1 or k != "ref"):   # ref: the 1-GPU reference shape
                plan.append(("mappo", k, "weak", MAPPO_LEGS[k]["envs"], MAPPO_LEGS[k]["mb"]))
        if world > 1 and args.strong:
            for k, c in STRONG_LEGS.items():
                if c["global_envs"] % world == 0 and c["global_mb"] % world == 0:
                    plan.append(("mappo", k, "strong", c["global_envs"] // world, c["global_mb"] // world))
        if world == 1 and args.rank_shapes:
            plan.append(("mappo", "rank_shapes", "rank-shape", None, None))   # one rank of G, timed on one GPU
    if args.configs:
        for k, c in EXTRA_CONFIGS.items():
            plan.append(("sim", k, "weak", c["envs"], None))
        if world > 1 and args.strong:
            for k, c in STRONG_SIM.items():
                if c[4] % world == 0:
                    plan.append(("sim", k, "strong", c[4] // world, None))
    return plan


def mappo_leg(args, ranks, T, cfg=None, rank_shape=None):
    """Full MAPPO train steps: by default on the bench's C3 envs (learn_mappo.py:196-216
    hyper-parameters, hidden 256, opt_epochs 10; minibatch scaled to the ~100x larger
    env batch), or one of MAPPO_LEGS.  rank_shape G: one rank's share of a STRONG_LEGS
    partition over G ranks, timed on this rank through the exchange path (the
    gradient all-reduce on the world-1 process group, _force_allreduce)."""
    from gym_pybullet_drones_amd.envs import MultiHoverAviary, SpiralFormationAviary
    from gym_pybullet_drones_amd.mappo import MAPPO
    from gym_pybullet_drones_amd.utils.enums import ActionType, Physics
    cfg = dict(cfg or dict(task="multihover", drones=args.drones, envs=args.envs, act=args.act, physics="dyn",
                           T=T, mb=args.mappo_mb, **LEARN_MAPPO))
    scaling = "weak"
    if "global_envs" in cfg:   # a strong partition (STRONG_LEGS): 1/G of the envs and of the minibatch per rank
        G = rank_shape or ranks.world
        cfg["envs"], cfg["mb"] = cfg.pop("global_envs") // G, cfg.pop("global_mb") // G
        scaling = "strong"
    D, E, T, mb = cfg.pop("drones"), cfg.pop("envs"), cfg.pop("T"), cfg.pop("mb")
    task, phys, label = cfg.pop("task"), cfg.pop("physics"), cfg.pop("label", None)
    act = {"one_d_pid": ActionType.ONE_D_PID, "vel": ActionType.VEL, "rpm": ActionType.RPM}[cfg.pop("act")]
    physics = {"dyn": Physics.DYN, "pyb": Physics.PYB, "pyb_dw": Physics.PYB_DW}[phys]
    if task == "spiral":
        env_func = lambda seed=0: SpiralFormationAviary(num_drones=D, act=act, physics=physics)
    else:
        env_func = lambda seed=0: MultiHoverAviary(num_drones=D, act=act, physics=physics,
                                                   initial_xyzs=grid_layout(D) if D >= 6 else None)
    m = MAPPO(env_func, training=True, seed=0, hidden_dim=256, actor_lr=3e-4, critic_lr=1e-3,
              rollout_steps=T, rollout_batch_size=E, opt_epochs=10,
              mini_batch_size=mb, output_dir="/tmp/qs_bench_mappo", **cfg)
    m.agent._force_allreduce = bool(rank_shape)
    m.agent.side_stream = bool(args.side_stream)
    m.agent.critic_adam_side = bool(args.critic_adam_side)
    m.agent.critic_tiles = bool(args.critic_tiles)
    from gym_pybullet_drones_amd.mappo import agent as agent_mod
    from gym_pybullet_drones_amd.mappo.agent import _F16Work, _M3Work, _SPLITK_MIN_ROWS
    if args.small_rows is not None:
        agent_mod._SMALL_MAX_ROWS = int(args.small_rows)
    if args.fused_max_a is not None:
        agent_mod._F16_MAX_A = int(args.fused_max_a)
    _F16Work.w1_stream = bool(args.w1_stream)
    _M3Work.wgrad = tuple(w for w in args.wgrad.split(",") if w)
    for item in filter(None, args.splitk.split(",")):   # "KxM=rows": split-K chunk rows of a weight gradient
        km, rows = item.split("=")
        k, mm = km.split("x")
        _SPLITK_MIN_ROWS[(int(k), int(mm))] = int(rows)
    m.reset()
    progress(f"mappo leg {label or 'C3'}{f' (one rank of {rank_shape})' if rank_shape else ''}: T={T} E={E} D={D} "
             f"mb={mb}, warm-up train step")
    m.train_step()   # warm-up: graph capture (with N ranks the all-reduce is captured too), lazy kernel loads
    m.time_phases = True
    ranks.fence()
    phases = []
    t0 = time.perf_counter()
    for _ in range(args.mappo_iters):
        phases.append(m.train_step()['phase_ms'])
        progress(f"  train step {len(phases)}: {phases[-1]}")
    ranks.fence()
    dt = ranks.max((time.perf_counter() - t0) / args.mappo_iters)
    O, A = m.obs_dim, m.agent.ac.act_dim
    world = ranks.world
    graphed = world == 1 or m.agent.graph_collectives
    rollout_graph = m._rollout_graph is not None
    fused_actor = type(getattr(m.agent, "_ws_actor", None)).__name__ == "_F16Work"
    if getattr(m.agent, "_sm_key", None) is not None:
        learner_path = ("qs_ppo_small_grads + all-reduce + qs_ppo_small_adam" if (world > 1 or rank_shape) else
                        "qs_ppo_small_step (16-row tiles, 2-3 launches per minibatch)")
    else:
        fold = fused_actor and getattr(m.agent._ws_actor, "pw1f", None) is not None
        learner_path = (("qs_mlp3f_actor_w1 (dW1 folded) + bmm dW2" if fold else "qs_mlp3f_actor + bmm dW2")
                        if fused_actor else "qs_mlp3 actor") + (
            " | critic qs_ppo_critic_tiles + qs_wgrad_t" if type(getattr(m.agent, "_ws_critic", None)).__name__
            == "_CriticTiles" else " | critic qs_mlp3w + GEMMs")
    exchange = int(m.agent._reduce_buf.numel())   # [critic grads | actor grads | approx_kl] floats
    m.close()
    ph = {k: float(np.mean([p[k] for p in phases])) for k in phases[0]}
    upd_flop, roll_flop = mappo_flops(T, E, D, O, A)
    upd_tflops = upd_flop / (ph["update"] * 1e-3) / 1e12
    return {"value": T * E * D * world / dt, "unit": "agent-steps/s", "ms_per_train_step": dt * 1e3,
            "train_steps": args.mappo_iters, "phase_ms": ph, "exchange_floats": exchange,
            "learner_roofline": {"bound": "mfma", "achieved": upd_tflops, "peak": FP32_MFMA_PEAK_TFLOPS,
                                 "unit": "TFLOP/s", "frac": upd_tflops / FP32_MFMA_PEAK_TFLOPS,
                                 "flop_per_update": upd_flop, "rollout_actor_flop": roll_flop,
                                 "train_step_tflops": (upd_flop + roll_flop) / dt / 1e12,
                                 "what": "PPO update: MLP fwd+bwd FLOP / update device time, fp32"},
            "config": {"workload": label, "scaling": scaling, "global_envs": E * world,
                       "global_mini_batch_size": mb * world, "rollout_steps": T, "envs_per_gpu": E, "drones": D,
                       "obs_dim": O,
                       "act_dim": A, "hidden": 256, "opt_epochs": 10, "mini_batch_size": mb,
                       "minibatches_per_epoch": T * E // mb, "fused_actor_kernel": fused_actor,
                       "learner_path": learner_path,
                       "overrides": cfg or None,
                       "reference": "learn_mappo.py: T=256, 176 envs, mini_batch_size 32 (1408 minibatches/epoch)",
                       "graphs": ("rollout + " if rollout_graph else "") + ("update" if graphed else ""),
                       "grad_allreduce": ("one fused all-reduce per minibatch" + (", captured in the update graph"
                                                                                   if graphed else ""))
                       if (world > 1 or rank_shape) else None}}


def world1_group():
    """A world-1 RCCL process group (N = 1 runs), so the rank-shape legs take the
    multi-rank exchange path (_force_allreduce) with its all-reduce captured."""
    import torch.distributed as dist
    if not dist.is_initialized():
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{free_port()}", rank=0, world_size=1,
                                device_id=torch.device("cuda", torch.cuda.current_device()))
        return True
    return False


def allreduce_us(n, reps=10, per_graph=20):
    """Mean device time of one all-reduce (sum) of n float32 on the current group,
    as the update graph issues it: `per_graph` all-reduces captured in a HIP graph,
    replayed `reps` times between HIP events."""
    import torch.distributed as dist
    buf = torch.zeros(n, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            dist.all_reduce(buf, async_op=True).wait()   # (eager: the event on the group's own stream)
    torch.cuda.current_stream().wait_stream(s)
    from gym_pybullet_drones_amd.mappo.collectives import capture_collectives, collective_group
    g = torch.cuda.CUDAGraph()
    # the captured all-reduces on the capture group, as the update graph issues them (mappo/collectives.py)
    with capture_collectives(), torch.cuda.graph(g, capture_error_mode="thread_local"):
        for _ in range(per_graph):
            dist.all_reduce(buf, group=collective_group())
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / (reps * per_graph)
    del g
    return us


def rank_shapes_leg(args, ranks, c3_one_gpu=None):
    """SURVEY §8(e)'s per-rank strong shapes timed on ONE GPU through the exchange
    path: C3 at G = 2 / 4 / 8, C4 at 4, C5 at 8 (--rank-shapes).
    Each is one rank's MAPPO train step (E/G envs, mini_batch_size/G, the gradient
    all-reduce on a world-1 group, captured in the update graph).  The G-rank
    projection replaces the world-1 all-reduce measured here by an assumed G-GPU
    xGMI all-reduce latency (--assumed-allreduce-us; not measurable on one GPU):
    value(G) = T·E·D / (train step + minibatches·(assumed − measured world-1)),
    and against the 1-GPU global configuration (the 'mappo' leg) its speed-up."""
    own = world1_group()
    out = {}
    try:
        for item in filter(None, args.rank_shapes.split(",")):
            name, G = item.split("/")
            G = int(G)
            cfg = STRONG_LEGS[name]
            r = mappo_leg(args, ranks, cfg["T"], cfg, rank_shape=G)
            c = r["config"]
            n_upd = 10 * c["minibatches_per_epoch"]
            out[item] = {"workload": f"{c['workload']}: one rank of {G}", "G": G, "envs_per_rank": c["envs_per_gpu"],
                         "mini_batch_per_rank": c["mini_batch_size"],
                         "actor_rows_per_minibatch": c["mini_batch_size"] * c["drones"],
                         "learner_path": c["learner_path"], "phase_ms": r["phase_ms"],
                         "ms_per_train_step": r["ms_per_train_step"],
                         "us_per_minibatch": r["phase_ms"]["update"] * 1e3 / n_upd,
                         "minibatches_per_update": n_upd, "exchange_floats": r.get("exchange_floats")}
            ar1 = allreduce_us(r["exchange_floats"])
            out[item]["allreduce_us_world1"] = ar1
            t_step = r["ms_per_train_step"] * 1e-3
            agent_steps = c["rollout_steps"] * c["envs_per_gpu"] * G * c["drones"]
            proj = {}
            for ar in (args.assumed_allreduce_us, 2 * args.assumed_allreduce_us):
                t = t_step + n_upd * (ar - ar1) * 1e-6
                proj[f"allreduce_{ar:g}us"] = {"value": agent_steps / t, "ms_per_train_step": t * 1e3}
                if name == "C3" and c3_one_gpu:
                    proj[f"allreduce_{ar:g}us"]["speedup_vs_1gpu"] = agent_steps / t / c3_one_gpu
                    proj[f"allreduce_{ar:g}us"]["efficiency"] = agent_steps / t / c3_one_gpu / G
            out[item]["projected_G_ranks"] = proj
    finally:
        if own:
            import torch.distributed as dist
            torch.cuda.synchronize()
            dist.destroy_process_group()
    return out


VALU_ISSUE_PEAK = 1024 * 2.4e9 / 2   # wave64 VALU instr/s: 1024 SIMDs, one per 2 cycles (the fp32 vector rate)


def valu_roofline(name, kernel_ms):
    """VALU bound of a config's step kernel: its VALU issue cycles per launch
    (profiles/r02_valu.json: SQ_INSTS_VALU, transcendentals at 4x) over the
    SIMD-cycles of the measured launch time."""
    path = os.path.join(ROOT, "profiles", "r02_valu.json")
    try:
        with open(path) as f:
            k = json.load(f)["kernels"].get(name)
    except (OSError, ValueError):
        return None
    if not k:
        return None
    cycles = k["valu_cycles_per_launch"]
    avail = 1024 * 2.4e9 * kernel_ms * 1e-3
    return {"bound": "valu", "achieved": cycles / 2 / (kernel_ms * 1e-3), "peak": VALU_ISSUE_PEAK,
            "unit": "wave64 VALU instr/s (2-cycle issue, transcendentals 8)", "frac": cycles / avail,
            "valu_lane_instr_per_agent_step": k["valu_lane_instr_per_agent_step"],
            "source": "profiles/r02_valu.json"}


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    # stdout carries the one JSON line: whatever the libraries print there (RCCL's
    # version banner at its first communicator) goes to stderr instead
    out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
    ranks = Ranks(dry=args.dry_run)
    world, rank = ranks.world, ranks.rank
    if args.dry_run:
        every, elapsed = dry_leg(args, ranks)
        if rank == 0:
            print(json.dumps({
                "metric": METRIC + " [dry run: CPU stand-in steps, no GPU]", "value": args.steps * world / elapsed,
                "unit": "stand-in steps/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": elapsed / args.steps * 1e3, "rank_ms_per_step": [e / args.steps * 1e3 for e in every],
                "dry_run": {"pid": os.getpid(), "ppid": os.getppid(), "pppid": _ppid(os.getppid()),
                            "backend": "gloo" if world > 1 else None},
                "legs": [{"kind": k, "name": n, "scaling": sc, "envs_per_rank": e, "mini_batch_per_rank": m}
                         for k, n, sc, e, m in leg_plan(args, world)]}), file=out, flush=True)
        ranks.close()
        return
    E, D = args.envs, args.drones
    progress("headline rollout leg")
    value, elapsed, kern_ms, steps, eps_done = sim_leg(args, ranks, "dyn")
    bpas = bytes_per_agent_step(args.act, "multihover", D)
    nbytes = bpas * E * D
    achieved = nbytes / (kern_ms * 1e-3) / 1e9
    pyb = fp64 = mappo = mappo32 = mappo_cfgs = configs = rank_shapes = None
    mappo_strong, configs_strong = {}, {}
    for kind, name, scaling, e_rank, mb_rank in leg_plan(args, world)[1:]:
        if kind == "sim" and name == "fp64":   # the headline rollout in the reference's float64
            progress("headline rollout leg, float64")
            fv, fel, fk, _, _ = sim_leg(args, ranks, "dyn", precision=8)
            b64 = bytes_per_agent_step(args.act, "multihover", D, precision=8)
            t64, t64_src = pmc_traffic(E, D, args.act, precision=8)
            fp64 = {"value": fv, "unit": "agent-steps/s", "kernel_ms": fk, "ms_per_step": fel / args.steps * 1e3,
                    "dtype": "f64", "roofline_frac": b64 * E * D / (fk * 1e-3) / 1e9 / HBM_PEAK_GBS,
                    "bytes_per_agent_step": b64,
                    "traffic": t64, "traffic_unit": "bytes per launch (HBM, PMC)", "traffic_source": t64_src,
                    "algorithmic_bytes_per_launch": b64 * E * D,
                    "what": "the same C3 rollout with every state field, target, reward and the physics in float64 "
                            "(the reference's numpy precision); action, history and obs float32 as in the kernel's "
                            "buffers (bench.bytes_per_agent_step)"}
        elif kind == "sim" and name == "pyb":   # the same rollout under Physics.PYB (the reference's training default)
            pv, _, pk, _, _ = sim_leg(args, ranks, "pyb")
            pyb = {"value": pv, "unit": "agent-steps/s", "kernel_ms": pk,
                   "roofline_frac": nbytes / (pk * 1e-3) / 1e9 / HBM_PEAK_GBS}
            if rank == 0 and world == 1 and not args.no_cpu_baseline:
                pyb["cpu_baseline"] = cpu_baseline(args, args.cpu_seconds / 4, physics="pyb")
        elif kind == "mappo" and name == "rank_shapes":
            rank_shapes = rank_shapes_leg(args, ranks, mappo["value"] if mappo else None)
        elif kind == "mappo" and scaling == "strong":
            mappo_strong[name] = mappo_leg(args, ranks, STRONG_LEGS[name]["T"], STRONG_LEGS[name])
            # the real G-GPU all-reduce of the exchange buffer, as the update graph issues it
            mappo_strong[name]["allreduce_us"] = allreduce_us(mappo_strong[name]["exchange_floats"])
        elif kind == "mappo" and name == "C3":
            mappo = mappo_leg(args, ranks, args.mappo_steps)
        elif kind == "mappo" and name == "C3_t32":
            mappo32 = mappo_leg(args, ranks, 32)
        elif kind == "mappo":   # the other trainer configs, per-GPU sizes
            mappo_cfgs = mappo_cfgs or {}
            mappo_cfgs[name] = mappo_leg(args, ranks, MAPPO_LEGS[name]["T"], MAPPO_LEGS[name])
        elif kind == "sim" and scaling == "strong":
            act, phys, task, D_, glob, byts = STRONG_SIM[name]
            progress(f"config leg {name} (strong: {glob} envs over {world} ranks)")
            v, el, km, st, ne = sim_leg(args, ranks, phys, task, e_rank, D_, act, ())
            nb = byts * e_rank * D_
            configs_strong[name] = {"workload": f"{task} {D_}-drone x {glob} envs over {world} ranks "
                                                f"({e_rank} per rank), {act}, {phys}", "scaling": "strong",
                                    "value": v, "unit": "agent-steps/s", "kernel_ms": km,
                                    "bytes_per_agent_step": byts, "roofline_frac": nb / (km * 1e-3) / 1e9 / HBM_PEAK_GBS,
                                    "episodes_ended_in_timed_window_rank0": ne}
        elif kind == "sim":   # the other BASELINE configs, per-GPU sizes
            c = EXTRA_CONFIGS[name]
            progress(f"config leg {name}")
            v, el, km, st, ne = sim_leg(args, ranks, c["physics"], c["task"], c["envs"], c["drones"],
                                        c["act"], c["aux"])
            nb = c["bytes"] * c["envs"] * c["drones"]
            configs = configs or {}
            configs[name] = {"workload": c["label"], "scaling": "weak", "value": v, "unit": "agent-steps/s",
                             "kernel_ms": km, "bytes_per_agent_step": c["bytes"],
                             "roofline_frac": nb / (km * 1e-3) / 1e9 / HBM_PEAK_GBS,
                             "episodes_ended_in_timed_window": ne}
            vr = valu_roofline(name, km)
            if vr:
                configs[name]["valu_roofline"] = vr
            if rank == 0 and world == 1 and not args.no_cpu_baseline:
                # BASELINE.md:36: the CPU restatement of the same config (rank 0 at N=1 only)
                configs[name]["cpu_baseline"] = cpu_baseline(args, args.cpu_seconds / 4, c["task"], c["drones"],
                                                             c["act"], c["physics"], c["aux"])
    if rank == 0:
        cpu = None if (args.no_cpu_baseline or world > 1) else cpu_baseline(args, args.cpu_seconds, extra22=True)
        traffic, traffic_src = pmc_traffic(E, D, args.act)
        line = {
            "metric": METRIC, "value": value, "unit": "agent-steps/s", "n_gpus": world, "steps": steps,
            "warmup": args.warmup, "ms_per_step": elapsed / steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": f"MultiHover {D}-drone x {E} envs/GPU, ActionType.{args.act.upper()}, "
                                   "Physics.DYN, random-policy rollout (C3 env config; MAPPO learner in the "
                                   "'mappo' field)",
                       "envs_per_gpu": E, "drones": D, "total_envs": E * world, "act": args.act,
                       "physics": "dyn", "parallelism": f"env-shard x{world}", "precision": "fp32",
                       "episode_phases": "uniform over 242 steps" if not args.no_stagger else "synchronised",
                       "episodes_ended_in_timed_window_rank0": eps_done},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_unit": "bytes per launch (HBM, PMC)", "traffic_source": traffic_src,
                         "algorithmic_bytes_per_launch": nbytes,
                         "kernel_ms": kern_ms, "bytes_per_agent_step": bpas},
            "timing": {"wall_ms_per_step": elapsed / steps * 1e3, "event_ms_per_step": kern_ms,
                       "fixed_wall_us_per_window": (elapsed / steps * 1e3 - kern_ms) * steps * 1e3,
                       "untimed_rehearsals": args.rehearse,
                       "what": "wall: barrier + device sync on both sides of the K steps (the value); event: HIP "
                               "events around the graph replays on the launch stream (the roofline's kernel time); "
                               "the window's graphs are replayed untimed `untimed_rehearsals` times right before it "
                               "(their episodes not counted)"},
            "cpu_baseline": cpu,
            "fp64": fp64,
            "pyb": pyb,
            "mappo": mappo,
            "mappo_t32": mappo32,
            "mappo_configs": mappo_cfgs,
            "mappo_rank_shapes": rank_shapes,
            "configs": configs,
        }
        if world > 1:
            line["mappo_strong"] = mappo_strong or None
            line["configs_strong"] = configs_strong or None
        print(json.dumps(line), file=out, flush=True)
    ranks.close()


if __name__ == "__main__":
    main()
