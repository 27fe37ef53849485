"""The C-ABI libraries load and export every symbol their headers declare (no GPU calls)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared(header):
    src = open(os.path.join(ROOT, "include", header)).read()
    return sorted(set(re.findall(r"^(?:int|const char\*|void)\s+(qs_\w+)\s*\(", src, re.M)))


def test_quadswarm_exports_every_declared_symbol():
    from gym_pybullet_drones_amd import _lib
    assert os.path.exists(_lib.LIB_PATH), "build the extension first (__graft_entry__.build())"
    lib = ctypes.CDLL(_lib.LIB_PATH)
    names = declared("quadswarm.h") + declared("qs_learner.h")
    assert len(names) >= 16
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) <= set(_lib.EXPORTS)
    lib.qs_abi_version.restype = ctypes.c_int
    assert lib.qs_abi_version() == _lib.ABI_VERSION == 4


def test_create_rejects_bad_spec_without_gpu_work():
    """Argument validation runs before any device call (reference raises ValueError, BA:79-80)."""
    from gym_pybullet_drones_amd import _lib as L
    lib = L.load()
    spec = L.QsSpec()
    spec.task, spec.num_envs, spec.num_drones, spec.act_type, spec.physics = 0, 4, 2, 0, 1
    spec.pyb_freq, spec.ctrl_freq, spec.precision = 240, 7, 4     # 240 % 7 != 0
    h = ctypes.c_void_p()
    assert lib.qs_create(ctypes.byref(spec), 0, ctypes.byref(h)) == -1
    assert b"divisible" in lib.qs_last_error()
    spec.ctrl_freq, spec.num_drones = 30, 7                         # default layout, D >= 6
    assert lib.qs_create(ctypes.byref(spec), 0, ctypes.byref(h)) == -1
    assert b"D >= 6" in lib.qs_last_error()
    spec.num_drones, spec.flags = 2, L.FLAG_CF2P << 1               # a flag this ABI does not define
    assert lib.qs_create(ctypes.byref(spec), 0, ctypes.byref(h)) == -1
    assert b"bad flags" in lib.qs_last_error()


def test_drone_models():
    """CF2X and CF2P are accepted (QS_FLAG_CF2P); RACE, which has no DSL PID
    (DSLPIDControl.py:34-36), is refused before any device work."""
    from gym_pybullet_drones_amd.envs.swarm import QuadSwarm
    from gym_pybullet_drones_amd.utils.enums import DroneModel
    with pytest.raises(NotImplementedError):
        QuadSwarm(num_envs=1, num_drones=2, drone_model=DroneModel.RACE)
    import qs_oracle
    s, _ = qs_oracle.make_spec(drone_model=DroneModel.CF2P)
    assert s.flags & 4 and not qs_oracle.make_spec(drone_model="cf2x")[0].flags & 4


def test_oracle_exports():
    import qs_oracle
    lib = qs_oracle.lib()
    for n in ("qso_create", "qso_reset", "qso_step", "qso_state_io", "qso_reset_envs", "qso_gae", "qso_dsl_pid"):
        assert hasattr(lib, n)


def test_ctypes_records_match_the_headers(tmp_path):
    """The ctypes mirrors of the C-ABI records (qs_spec, qs_mlp256) have the headers'
    size and field offsets: a C program built with gcc against include/*.h prints
    them (a field added on one side only would shift every later field)."""
    import subprocess
    from gym_pybullet_drones_amd import _lib as L
    recs = {"qs_spec": L.QsSpec, "qs_dims": L.QsDims, "qs_step_out": L.QsStepOut, "qs_mlp256": L.QsMlp256}
    ctype_name = {"in_": "in"}   # Python keyword renamed in the mirror
    lines = ["#include <stddef.h>", "#include <stdio.h>", '#include "quadswarm.h"', '#include "qs_learner.h"',
             "int main(void) {"]
    for rec, cls in recs.items():
        lines.append(f'  printf("{rec} size %zu\\n", sizeof({rec}));')
        for f in cls._fields_:
            name = ctype_name.get(f[0], f[0])
            lines.append(f'  printf("{rec} {f[0]} %zu\\n", offsetof({rec}, {name}));')
    lines.append('  printf("qs_episode_rec size %zu\\n", sizeof(qs_episode_rec));')
    for name in L.EPISODE_DTYPE.names:   # the numpy view of the episode-log records
        lines.append(f'  printf("qs_episode_rec {name} %zu\\n", offsetof(qs_episode_rec, {name}));')
    lines += ["  return 0;", "}"]
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines) + "\n")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = {}
    for line in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.splitlines():
        rec, field, val = line.split()
        got[(rec, field)] = int(val)
    for rec, cls in recs.items():
        assert got[(rec, "size")] == ctypes.sizeof(cls), rec
        for f in cls._fields_:
            assert got[(rec, f[0])] == getattr(cls, f[0]).offset, (rec, f[0])
    assert got[("qs_episode_rec", "size")] == L.EPISODE_DTYPE.itemsize
    for name in L.EPISODE_DTYPE.names:
        assert got[("qs_episode_rec", name)] == L.EPISODE_DTYPE.fields[name][1], name


def test_tile_layouts_at_the_per_rank_shapes():
    """qs_ppo_small_layout (host code, no GPU): the tile path's row blocks per net
    at SURVEY §8(e)'s per-rank shapes — 16-row tiles while both nets fit one
    round of the 256 CUs, then 32- and 48-row actor tiles with the critic's kept
    at 16 rows while they still fit, and the weight gradients'
    K-chunks (64×64 tiles in 64-row steps, s_chunks' launch estimate)."""
    from gym_pybullet_drones_amd import _lib as L
    lib = L.load()
    off = (ctypes.c_int64 * L.QS_PPO_SMALL_LAYOUT_N)()

    def lay(mb, D, Ia, Ic, A):
        assert lib.qs_ppo_small_layout(mb, D, Ia, Ic, A, off, len(off)) == 0
        return dict(nA=off[16], nC=off[17], KaP=off[18], KcP=off[19], Sa=off[27], Sc=off[28])

    # the reference's learner shape: 256 actor rows, 32 critic rows, 16-row tiles
    assert lay(32, 8, 27, 216, 1) == dict(nA=16, nC=2, KaP=256, KcP=32, Sa=1, Sc=1)
    # C3 at G = 8: 288 16-row tiles would take two rounds: 32-row actor tiles, 16-row critic tiles
    assert lay(512, 8, 27, 216, 1) == dict(nA=128, nC=32, KaP=4096, KcP=512, Sa=8, Sc=1)
    # C3 at G = 4: 48-row actor tiles (171, padded to 8 208 rows)
    assert lay(1024, 8, 27, 216, 1) == dict(nA=171, nC=64, KaP=8208, KcP=1024, Sa=9, Sc=2)
    # C5 at G = 8: a narrow actor at 48 rows beside the 432-wide critic at 16
    assert lay(512, 16, 27, 432, 1) == dict(nA=171, nC=32, KaP=8208, KcP=512, Sa=10, Sc=1)
    # C4 at G = 4: the four-output actor at 32 rows beside the 595-wide critic at 16 (one round)
    d = lay(1024, 5, 119, 595, 4)
    assert (d["nA"], d["nC"], d["KaP"], d["KcP"]) == (160, 64, 5120, 1024)


def test_small_layout_writes_only_the_callers_entries():
    """qs_ppo_small_layout writes min(n_off, QS_PPO_SMALL_LAYOUT_N)
    entries — a caller sized for fewer (an older contract) is never overrun."""
    from gym_pybullet_drones_amd import _lib as L
    lib = L.load()
    buf = (ctypes.c_int64 * 40)(*([-7] * 40))
    assert lib.qs_ppo_small_layout(512, 8, 27, 216, 1, buf, 23) == 0
    assert all(buf[i] != -7 for i in range(23)) and all(buf[i] == -7 for i in range(23, 40))
    full = (ctypes.c_int64 * L.QS_PPO_SMALL_LAYOUT_N)()
    assert lib.qs_ppo_small_layout(512, 8, 27, 216, 1, full, len(full)) == 0
    assert list(buf[:23]) == list(full[:23])
    assert lib.qs_ppo_small_layout(512, 8, 27, 216, 1, full, 0) != 0   # no room: refused
