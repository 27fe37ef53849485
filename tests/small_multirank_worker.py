"""One rank of tests/test_gpu_small_multirank.py (not collected by pytest).

Every rank shares cuda:0 and the gloo backend (gloo all-reduces CUDA tensors
through the host; RCCL refuses two ranks on one device).  Rank r holds envs
[r·E/G, (r+1)·E/G) of a global rollout built from one seeded CPU generator and
runs the tile path's multi-rank minibatch steps (qs_ppo_small_grads → gloo
all-reduce → qs_ppo_small_adam) over its local minibatches; the parameters,
Adam moments and step counts it ends with are saved for the parent to compare
with one rank stepping the union of the ranks' minibatches.

usage: small_multirank_worker.py RANK WORLD PORT OUT E T D MB [GATE_CLOSED]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "marl-gym-pybullet-drones_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    rank, world, port, out = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    E, T, D, MB = (int(x) for x in sys.argv[5:9])
    gate_closed = len(sys.argv) > 9 and sys.argv[9] == "1"
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        import small_multirank_case as case
        agent, buf = case.build(E, T, D, rank=rank, world=world, gate_closed=gate_closed)
        assert dist.get_world_size() == world
        acc = torch.zeros(4, dtype=torch.float64, device="cuda")
        for idx in case.local_minibatches(E // world, T, MB // world):
            agent._step_minibatch(buf, idx.cuda(), acc)
        torch.cuda.synchronize()
        assert agent._sm_key is not None, "the tile path did not take the minibatch"
        torch.save({k: v.cpu() for k, v in case.snapshot(agent).items()} | {"acc": acc.cpu()}, out)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
