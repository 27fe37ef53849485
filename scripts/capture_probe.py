"""Dev probe: graph captures of the update (its all-reduce
captured) right after eager all-reduces on a world-1 RCCL group, no sleep.

  python scripts/capture_probe.py capture N   # the product path (mappo/collectives.py)
  python scripts/capture_probe.py default N   # synchronous eager all-reduces and the captured one on the
                                              # default group (round 5's hazard, without its drain)

Before each capture, eager all-reduces run with the graphs' default capture
stream current (the stream the next capture uses: a synchronous collective
records its end event on the current stream).  Prints one line per capture;
an abort of the process (hipErrorCapturedEvent from the RCCL watchdog) is the
hazard."""
import os
import socket
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "marl-gym-pybullet-drones_amd"))
from gym_pybullet_drones_amd import _lib as L  # noqa: E402
from gym_pybullet_drones_amd.mappo import agent as agent_mod  # noqa: E402
from gym_pybullet_drones_amd.mappo import collectives  # noqa: E402
from gym_pybullet_drones_amd.mappo.agent import MAPPOAgent  # noqa: E402
from gym_pybullet_drones_amd.mappo.buffer import MAPPOBuffer  # noqa: E402
from gym_pybullet_drones_amd.utils.spaces import Box  # noqa: E402


def main():
    mode, n = sys.argv[1], int(sys.argv[2])
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    if mode == "default":   # every all-reduce synchronous on the default group
        collectives.all_reduce = lambda t: dist.all_reduce(t)
    agent_mod._SMALL_MAX_ROWS = L.QS_PPO_SMALL_MAX_ROWS
    D, O, A, T, E = 8, 27, 1, 16, 512
    osp, asp = Box(-np.inf * np.ones((D, O)), np.inf * np.ones((D, O))), Box(-np.ones((D, A)), np.ones((D, A)))
    agent = MAPPOAgent(osp, asp, hidden_dim=256, opt_epochs=1, mini_batch_size=512, entropy_coef=0.005,
                       target_kl=1e9, device="cuda", small=True)
    agent._force_allreduce = True
    buf = MAPPOBuffer(osp, asp, T, E, include_global_state=True, device="cuda")
    for t in (buf.next_obs_slots, buf.act, buf.logp, buf.ret_env, buf.adv_env):
        t.normal_()
    buf.t, buf.full = 0, True
    x = torch.ones(1 << 16, device="cuda")
    agent._capture(buf, 1)   # (creates the graphs' default capture stream)
    cs = torch.cuda.graph.default_capture_stream
    for i in range(n):
        with torch.cuda.stream(cs):
            for _ in range(4):
                collectives.all_reduce(x)
        t0 = time.perf_counter()
        agent._capture(buf, int(os.environ.get("QS_CAPTURE_K", "400")))   # a capture window of K minibatch iterations (~70 ms at 400)
        agent._graph.replay()
        print(f"{mode} capture {i}: {1e3 * (time.perf_counter() - t0):.1f} ms", flush=True)
    torch.cuda.synchronize()
    agent.release_graphs()
    dist.destroy_process_group()
    print(f"{mode}: {n} captures OK", flush=True)


if __name__ == "__main__":
    main()
