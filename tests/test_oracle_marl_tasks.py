"""Flock / Meetup / LeaderFollower reward, termination and truncation in the oracle
(SURVEY §8(f) next-4), each expected value computed here by hand from the reference
text: FlockAviary.py:74-186, MeetupAviary.py:71-151, LeaderFollowerAviary.py:71-144."""
import numpy as np
import pytest

import qs_oracle as Q

F_POS, F_QUAT, F_VEL, F_W = 0, 3, 7, 10


def _sim(task, D, pos, vel=None, quat=None, **kw):
    s = Q.OracleSim(task=task, num_envs=1, num_drones=D, act="rpm", precision=8, physics="dyn",
                    initial_xyzs=pos, autoreset=False, **kw)
    s.reset(0)
    st = s.get_state(0)
    st[:] = 0
    st[F_POS:F_POS + 3] = np.asarray(pos, np.float64).T
    st[F_QUAT + 3] = 1
    if quat is not None:
        st[F_QUAT:F_QUAT + 4] = np.asarray(quat, np.float64).T
    if vel is not None:
        st[F_VEL:F_VEL + 3] = np.asarray(vel, np.float64).T
    s.set_state(0, st)
    return s


def _one_step(s, D):
    """Zero action = hover rpm: with level drones the state after one DYN step is the
    injected one moved by v·t only (no net force); read it back for the expected value."""
    out = s.step(np.zeros((1, D, 4), np.float32))
    st = s.get_state(0)
    return out, st[F_POS:F_POS + 3].T, st[F_VEL:F_VEL + 3].T


def flock_expected(p, v):
    D = len(p)
    n = np.linalg.norm(v, axis=1)
    ali = 0.0
    for i in range(D):
        for j in range(D):
            if j != i:
                ali += (v[i] @ v[j]) / (n[i] + 1e-3) / (n[j] + 1e-3)
    ali = ali / (D * (D - 1)) if D > 1 else 0.0
    speed = np.linalg.norm(v.mean(axis=0))
    sp = np.array([min(np.linalg.norm(p[j] - p[i]) for j in range(D) if j != i) for i in range(D)])
    mean, var = sp.mean(), sp.var()
    pen = 0.0 if 1.0 < mean < 3.0 else min(abs(mean - 1.0), abs(mean - 3.0))
    return ali + speed - pen - var


@pytest.mark.parametrize("spread", [0.5, 2.0, 4.0])
def test_flock_reward(spread):
    pos = [[0, 0, 1.0], [spread, 0.3, 1.0], [0.2, spread, 1.1]]
    vel = [[0.3, 0.1, 0.0], [0.25, -0.05, 0.02], [-0.1, 0.2, 0.0]]
    s = _sim("flock", 3, pos, vel)
    out, p, v = _one_step(s, 3)
    assert out["reward"][0] == pytest.approx(flock_expected(p, v), rel=1e-12, abs=1e-12)
    assert out["terminated"][0] == 0 and out["truncated"][0] == 0


def test_meetup_reward_and_success():
    pos = [[0, 0, 1.0], [1.0, 0.5, 1.2], [2.0, 0, 1.0], [0.5, 0.5, 1.0]]
    s = _sim("meetup", 4, pos)
    out, p, _ = _one_step(s, 4)
    want = sum(-1 * np.linalg.norm(p[i] - p[3 - i]) ** 2 * 2 for i in range(2))
    assert out["reward"][0] == pytest.approx(want, rel=1e-12)
    assert out["terminated"][0] == 0
    # every pair within 0.1 m ⇒ terminated (MeetupAviary.py:97-117)
    s = _sim("meetup", 4, [[0, 0, 1.0], [1, 0, 1.0], [1.05, 0, 1.0], [0.02, 0, 1.0]])
    out, _, _ = _one_step(s, 4)
    assert out["terminated"][0] == 1


def test_leaderfollower_reward():
    pos = [[0.2, -0.1, 0.7], [1.0, 0.5, 1.2], [-0.5, 0.3, 0.4]]
    s = _sim("leaderfollower", 3, pos)
    out, p, _ = _one_step(s, 3)
    want = -np.linalg.norm(np.array([0, 0, 0.5]) - p[0]) ** 2
    for i in (1, 2):
        want += -(1 / 3) * np.linalg.norm(np.array([p[i, 0], p[i, 1], p[0, 2]]) - p[i]) ** 2
    assert out["reward"][0] == pytest.approx(want, rel=1e-12)
    assert out["terminated"][0] == 0


@pytest.mark.parametrize("task,pos,trunc", [
    ("flock", [[0, 0, 1.0], [10.5, 0, 1.0]], 1), ("flock", [[0, 0, 1.0], [9.5, 0, 9.5]], 0),
    ("meetup", [[0, 0, 1.0], [0, 5.5, 1.0]], 1), ("meetup", [[0, 0, 0.05], [1, 0, 1.0]], 1),
    ("meetup", [[0, 0, 1.0], [1, 0, 2.9]], 0),
    ("leaderfollower", [[0, 0, 1.0], [2.2, 0, 1.0]], 1), ("leaderfollower", [[0, 0, 1.0], [1.9, 0, 1.9]], 0),
])
def test_box_truncation(task, pos, trunc):
    s = _sim(task, 2, pos)
    out, _, _ = _one_step(s, 2)
    assert out["truncated"][0] == trunc


@pytest.mark.parametrize("task", ["flock", "meetup", "leaderfollower"])
def test_tilt_truncation(task):
    r = 0.45   # |roll| > 0.4
    s = _sim(task, 2, [[0, 0, 1.0], [1, 0, 1.0]], quat=[[0, 0, 0, 1], [np.sin(r / 2), 0, 0, np.cos(r / 2)]])
    out, _, _ = _one_step(s, 2)
    assert out["truncated"][0] == 1
    assert out["terminated"][0] == 0


def test_marl_reset_is_deterministic_init():
    """BaseAviary.reset puts the drones back at INIT_XYZS (no noise, BA:245-255)."""
    pos = [[0.1, 0.2, 1.0], [1.1, 0.2, 1.0]]
    s = Q.OracleSim(task="flock", num_envs=2, num_drones=2, act="rpm", precision=8, initial_xyzs=pos)
    o0 = s.reset(7)
    np.testing.assert_array_equal(o0[0, :, 0:3], np.asarray(pos, np.float32))
    np.testing.assert_array_equal(o0[1, :, 0:3], np.asarray(pos, np.float32))
