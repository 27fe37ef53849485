"""bench.py's N-rank path on CPU (gloo): `--gpus 2` launches torchrun as a child
process (never an exec), both ranks time the window between barrier fences, and
rank 0 reports the MAX over ranks with n_gpus = 2 (bench.py Ranks / dry_leg)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run_bench(*extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    p = subprocess.Popen([sys.executable, os.path.join(ROOT, "bench.py"), *extra], cwd=ROOT, env=env,
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    out, err = p.communicate(timeout=240)
    assert p.returncode == 0, err[-3000:]
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out   # rank 0 alone prints the line
    return p.pid, json.loads(lines[0])


def test_bench_two_ranks_max_over_ranks():
    dry_ms, steps = 20.0, 6
    launcher, line = _run_bench("--gpus", "2", "--dry-run", "--dry-ms", str(dry_ms), "--steps", str(steps),
                                "--warmup", "1")
    assert line["n_gpus"] == 2 and line["steps"] == steps
    # rank 1's stand-in step takes 2 x dry_ms: the barrier fences make rank 0's own
    # window hold rank 1's work too, and the reported time is the MAX of the windows
    per_rank = line["rank_ms_per_step"]
    assert len(per_rank) == 2
    # (10 % for the barrier-exit skew between the ranks: rank 0's own step is 1 x dry_ms)
    assert min(per_rank) >= 0.9 * 2 * dry_ms
    assert line["ms_per_step"] == max(per_rank)
    assert line["value"] == pytest.approx(2 / (line["ms_per_step"] * 1e-3), rel=1e-9)
    # rank 0 runs in a torchrun child of the launcher: its grandparent is the
    # process we started, and it is a different process (no exec)
    d = line["dry_run"]
    assert d["backend"] == "gloo"
    assert d["pid"] != launcher and d["ppid"] != launcher
    assert d["pppid"] == launcher


def test_bench_one_rank_dry_run():
    launcher, line = _run_bench("--dry-run", "--dry-ms", "1", "--steps", "3", "--warmup", "0")
    assert line["n_gpus"] == 1 and line["dry_run"]["pid"] == launcher and line["dry_run"]["backend"] is None


def test_bench_two_ranks_lists_strong_legs():
    """At N > 1 the bench also times SURVEY §8(e)'s strong partitions of BASELINE
    configs 3-5 (global envs and global minibatch fixed, 1/G per rank), beside the
    weak-scaled legs; the dry run lists the plan a GPU run of that size executes."""
    _, line = _run_bench("--gpus", "2", "--dry-run", "--dry-ms", "1", "--steps", "2", "--warmup", "0")
    legs = {(g["kind"], g["name"], g["scaling"]): g for g in line["legs"]}
    for name, envs in (("C3", 16384), ("C4", 8192), ("C5", 8192)):
        m = legs[("mappo", name, "strong")]
        assert m["envs_per_rank"] == envs // 2 and m["mini_batch_per_rank"] == 4096 // 2
        assert legs[("sim", name, "strong")]["envs_per_rank"] == envs // 2
    assert legs[("mappo", "C3", "weak")]["envs_per_rank"] == 16384   # the weak legs stay, labelled
    assert ("mappo", "C4", "weak") in legs and ("mappo", "C5", "weak") in legs
    assert ("mappo", "ref", "weak") not in legs   # the 1-GPU reference learner shape
    _, one = _run_bench("--dry-run", "--dry-ms", "1", "--steps", "2", "--warmup", "0")
    assert not any(g["scaling"] == "strong" for g in one["legs"])
    assert ("mappo", "ref", "weak") in {(g["kind"], g["name"], g["scaling"]) for g in one["legs"]}
    # N = 1: the per-rank strong shapes, each timed on one GPU through the exchange path
    assert ("mappo", "rank_shapes", "rank-shape") in {(g["kind"], g["name"], g["scaling"]) for g in one["legs"]}
    assert not any(g["name"] == "rank_shapes" for g in line["legs"])


def test_bytes_per_agent_step_matches_survey():
    """bench.bytes_per_agent_step reproduces SURVEY §8(d)'s per-config figures
    (C2 720, C3 418 / VEL 790, C4 1111, C5 418 B, rounded there) and prices the
    precision-8 build with float32 action, history and obs (the kernel's buffer
    types) and float64 state, target and reward: 662.25 B for C3, not 2 x 418."""
    import bench
    b = bench.bytes_per_agent_step
    assert round(b("rpm", "multihover", 4)) == 720
    assert round(b("one_d_pid", "multihover", 8)) == 418
    assert round(b("vel", "multihover", 8)) == 790
    assert round(b("vel", "spiral", 5)) == 1111
    assert abs(b("one_d_pid", "multihover", 16) - 418) < 1.2   # (SURVEY: "= C3 per agent"; per-env bytes / 16)
    assert b("one_d_pid", "multihover", 8, precision=8) == 4 + 2 * 29 * 8 + 3 * 8 + 15 * 4 + 27 * 4 + 18 / 8
