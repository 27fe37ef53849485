"""Known answers for the oracle's drone–drone contact in Physics.PYB.

The reference's Bullet world keeps every drone's collision cylinder live
(assets/cf2x.urdf:31-36, BaseAviary.py:484-491; the collision-filter disable at
BaseAviary.py:500-503 is commented out), so drones that meet push each other
apart.  The restatement (oracle drone_contacts) is inelastic and
frictionless with equal masses: after a contact the pair is separated along the
axis of the smaller penetration and both drones carry the mean of their
velocity components on that axis.  Expected values derived by hand.
"""
import numpy as np

import qs_oracle as Q

F_POS, F_QUAT, F_VEL, F_W, F_TGT = 0, 3, 7, 10, 26
R_CYL, H_CYL = 0.06, 0.0125


def _sim(D=2):
    s = Q.OracleSim(task="multihover", num_envs=1, num_drones=D, act="one_d_rpm", precision=8, physics="pyb",
                    initial_xyzs=[[float(i), 0.0, 1.0] for i in range(D)], autoreset=False)
    s.reset(0)
    return s


def _inject(s, pos, vel):
    st = s.get_state(0)
    st[:] = 0
    for d, (p, v) in enumerate(zip(pos, vel)):
        st[F_POS:F_POS + 3, d] = p
        st[F_QUAT + 3, d] = 1.0
        st[F_VEL:F_VEL + 3, d] = v
        st[F_TGT:F_TGT + 3, d] = p
    s.set_state(0, st)


def _hover(s, steps=1):
    for _ in range(steps):
        s.step(np.zeros((1, s.D, 1), np.float32))   # ONE_D_RPM a = 0: hover rpm on every motor
    return s.get_state(0)


def test_head_on_horizontal_contact():
    """Two level drones 0.2 m apart closing at 2 m/s each: within one control step
    (8 substeps of 1/240 s) their gap would shrink by 0.13 m, below 2r = 0.12 m.
    After the contact they touch (centre distance 2r, no overlap), share the
    mean x velocity (zero by symmetry), and the total momentum is unchanged."""
    s = _sim()
    _inject(s, [(-0.1, 0, 1), (0.1, 0, 1)], [(2, 0, 0), (-2, 0, 0)])
    st = _hover(s)
    x0, x1 = st[F_POS, 0], st[F_POS, 1]
    assert x1 - x0 >= 2 * R_CYL - 1e-12
    assert x1 - x0 < 2 * R_CYL + 2 * 2 * (1 / 240)   # in contact at the last substep, or one substep apart
    np.testing.assert_allclose(st[F_VEL, 0] + st[F_VEL, 1], 0.0, atol=1e-12)   # momentum
    assert abs(st[F_VEL, 0]) < 1e-12 and abs(st[F_VEL, 1]) < 1e-12            # inelastic: relative velocity gone
    np.testing.assert_allclose(st[F_POS + 1], 0.0, atol=1e-15)                 # no tangential effect
    np.testing.assert_allclose(st[F_POS, 0], -st[F_POS, 1], atol=1e-12)        # symmetric


def test_oblique_contact_keeps_tangential_velocity():
    """Drone 1 passes drone 0 with an x offset: only the velocity component along
    the centre line is averaged, the tangential component is untouched, momentum
    is conserved, and the pair ends with no overlap."""
    s = _sim()
    _inject(s, [(0.0, 0.0, 1.0), (0.02, 0.2, 1.0)], [(0, 0, 0), (0.5, -3.0, 0)])
    st = _hover(s)
    p0, p1 = st[F_POS:F_POS + 2, 0], st[F_POS:F_POS + 2, 1]
    v0, v1 = st[F_VEL:F_VEL + 2, 0], st[F_VEL:F_VEL + 2, 1]
    assert np.hypot(*(p1 - p0)) >= 2 * R_CYL - 1e-12
    # total horizontal momentum: only the (small) damping acts besides the contact
    free = _sim(D=1)
    _inject(free, [(0.02, 0.2, 1.0)], [(0.5, -3.0, 0)])
    vf = _hover(free)[F_VEL:F_VEL + 2, 0]
    assert np.linalg.norm((v0 + v1) - vf) < 0.02 * np.linalg.norm(vf)
    n = (p1 - p0) / np.hypot(*(p1 - p0))
    assert (v1 - v0) @ n >= -1e-12   # not approaching along the centre line any more
    assert abs(v0 @ np.array([-n[1], n[0]])) < 0.2 * abs(v1 @ np.array([-n[1], n[0]]))   # drone 0 got no shove sideways


def test_vertical_stack_contact():
    """Drone 1 falls at 1 m/s onto drone 0 from 0.03 m above (the two flat
    cylinders are 2h = 0.025 m tall together): the vertical gap stays >= 2h and
    both end with the same vertical velocity (momentum shared)."""
    s = _sim()
    _inject(s, [(0.0, 0.0, 1.0), (0.0, 0.0, 1.03)], [(0, 0, 0), (0, 0, -1.0)])
    st = _hover(s)
    dz = st[F_POS + 2, 1] - st[F_POS + 2, 0]
    assert dz >= 2 * H_CYL - 1e-12
    np.testing.assert_allclose(st[F_VEL + 2, 0], st[F_VEL + 2, 1], atol=1e-12)
    np.testing.assert_allclose(st[F_POS:F_POS + 2], 0.0, atol=1e-15)


def test_no_contact_when_apart():
    """Drones that never come within 2r move exactly as alone (the contact pass is a no-op)."""
    s = _sim()
    _inject(s, [(-0.2, 0, 1), (0.2, 0, 1)], [(1, 0, 0), (-1, 0, 0)])   # gap 0.4 - 0.067 stays > 0.12
    st = _hover(s)
    a = _sim(D=1)
    _inject(a, [(-0.2, 0, 1)], [(1, 0, 0)])
    np.testing.assert_array_equal(st[:, 0], _hover(a)[:, 0])
