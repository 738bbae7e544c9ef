"""The oracle's flavor-B goal scenarios (oracle/quadswarm_oracle_scen.c) replayed against the reference.

tests/golden/scen_*.npz were recorded from the reference's own scenario classes by
tools/gen_golden_scen.py (every Generator / np.random draw in call order, goals after reset() and after
every step()).  Replaying the tape, the oracle must reproduce every goal: this pins the scenario
restatement that the GPU kernels are then compared with draw-for-draw (tests/test_gpu_parity_scen.py).
"""
import ctypes
import glob
import os

import numpy as np
import pytest

import oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")
FILES = sorted(glob.glob(os.path.join(GOLD, "scen_*.npz")))


def _params(n, mode_name):
    p = O.default_params(num_agents=n, num_envs=1)
    p.control_dt = 0.01        # sim_freq 200, 2 substeps -> control_freq 100
    p.spawn_box = 2.0          # QuadrotorSingle.box (quadrotor_single.py:218)
    p.scenario_b = O.SC_MIX if mode_name == "mix" else O.SC_MODES.index(mode_name)
    return p


@pytest.mark.parametrize("path", FILES, ids=[os.path.basename(f)[5:-4] for f in FILES])
def test_scenario_replays_reference(path):
    g = np.load(path)
    name = os.path.basename(path)[5:-4]
    mode = name.rsplit("_n", 1)[0]
    n, T = int(g["n"]), int(g["T"])
    p = _params(n, mode)
    draws = O.ScenDraws(tape=g["tape"])
    sc = O.OrScen()
    goals = np.zeros((n, 3))
    recs, ticks = g["goals"], g["ticks"]
    k = 0
    for r, want_mode in enumerate(g["modes"]):
        O.lib().or_scen_reset(ctypes.byref(p), ctypes.byref(sc), draws.ref, O.dptr(goals))
        assert sc.mode == want_mode, f"reset {r}: mode {sc.mode} vs reference {want_mode}"
        assert ticks[k] == 0
        np.testing.assert_allclose(goals, recs[k], rtol=0, atol=1e-10, err_msg=f"reset {r}")
        k += 1
        for t in range(1, T + 1):
            prev = goals.copy()
            O.lib().or_scen_step(ctypes.byref(p), ctypes.byref(sc), t, draws.ref, O.dptr(goals))
            if k < len(ticks) and ticks[k] == t:
                np.testing.assert_allclose(goals, recs[k], rtol=0, atol=1e-10, err_msg=f"reset {r} tick {t}")
                k += 1
            else:
                np.testing.assert_array_equal(goals, prev, err_msg=f"reset {r} tick {t}: goals moved, reference kept them")
    assert k == len(ticks)
    assert draws.s.tape_pos == len(g["tape"]) and not draws.s.overrun, "draw count differs from the reference"


def test_generate_goals_formations():
    """Every formation of generate_goals (base.py:42-116) for layer counts 1..2, incl. sphere with n < 3."""
    c = np.array([0.5, -1.0, 2.0])
    g = np.zeros((40, 3))
    for f in range(8):
        for n in (1, 2, 8, 9, 17, 32):
            m = O.lib().or_generate_goals(f, n, 50 if f in (4, 5, 6) else 8, 0.7, 0.3, O.dptr(c), O.dptr(g))
            assert m == (max(n, 3) if f == 3 else n)
            assert np.isfinite(g[:m]).all()
            if f in (4, 5, 6, 7):   # grid / cube are centred on the formation centre
                np.testing.assert_allclose(g[:n].mean(0), c, atol=1e-12)
