"""GPU parity of the flavor-B goal scenarios: the HIP kernels' scenario reset / step
(qs_flavor_b.h scen_reset / scen_step, run by each env's lead lane on LDS goal tables) against the oracle
(oracle/quadswarm_oracle_scen.c, itself replayed against the reference's scenario classes in
tests/test_oracle_golden_scen.py).  Same Philox draws; fp32 vs fp64.

Tolerances: goals and scenario floats 2e-5 abs after a reset / one step from an identical state (the
float formation geometry: sin/cos on the hardware units, ~1e-6); integer scenario state (mode, formation,
period, increase flag) identical; observations / rewards as in test_gpu_parity.py (2e-4).  Free-running
goals over 700 steps: 1e-2 (fp32 accumulation of ep_lissajous3D / dynamic_formations).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no HIP device", allow_module_level=True)

import oracle as O  # noqa: E402
from parity_utils import (assert_obs_match, crowd, oracle_params, oracle_to_gpu, scen_gpu_to_oracle,  # noqa: E402
                          scen_oracle_to_gpu)
from quadswarm_amd import QuadSwarmConfig  # noqa: E402
from quadswarm_amd import _native as NAT  # noqa: E402
from quadswarm_amd.env import QuadSwarmEnv  # noqa: E402

MODES = ["mix", "static_diff_goal", "ep_lissajous3D", "ep_rand_bezier", "dynamic_same_goal", "dynamic_diff_goal",
         "dynamic_formations", "swap_goals", "swarm_vs_swarm", "run_away"]


def make_pair(mode, E=128, N=8, seed=11, **kw):
    cfg = QuadSwarmConfig(num_envs=E, num_agents=N, neighbor_visible_num=min(6, N - 1),
                          neighbor_obs_type="pos_vel" if N > 1 else "none", quads_mode=mode, seed=seed, **kw)
    return cfg, QuadSwarmEnv(cfg), O.OracleEnv(oracle_params(cfg), seed=seed)


def np_(t):
    return t.double().cpu().numpy()


def goals_of(oenv):
    return np.array([oenv.drones[g].goal[:] for g in range(oenv.E * oenv.N)])


def check_scen_state(env, oenv, atol=2e-5):
    es, ef = env.env_state.cpu().numpy(), NAT.env_f_rows(np_(env.env_f))
    for e in range(env.E):
        sc = oenv.envs[e].scen
        got_i = es[NAT.E_SC_MODE:NAT.E_SC_MODE + 4, e]
        assert list(got_i) == [sc.mode, sc.formation, sc.period, sc.increase], f"env {e}"
        want_f = [sc.size, sc.lo, sc.hi, sc.layer, sc.speed]
        np.testing.assert_allclose(ef[NAT.ENVF_SC_SIZE:NAT.ENVF_SC_SIZE + 5, e], want_f, atol=atol, err_msg=f"env {e}")
        np.testing.assert_allclose(ef[NAT.ENVF_SC_CENTER:NAT.ENVF_SC_CENTER + 3, e], sc.center[:], atol=atol)
        np.testing.assert_allclose(ef[NAT.ENVF_SC_C1:NAT.ENVF_SC_C1 + 3, e], sc.c1[:], atol=atol)
        np.testing.assert_allclose(ef[NAT.ENVF_SC_C2:NAT.ENVF_SC_C2 + 3, e], sc.c2[:], atol=atol)


@pytest.mark.parametrize("mode", MODES)
def test_reset_goals_match_oracle(mode):
    N = 8 if mode != "mix" else 8
    cfg, env, oenv = make_pair(mode, E=256, N=N)
    obs = np_(env.reset())
    want = oenv.reset()
    np.testing.assert_allclose(np_(env.state[NAT.F_GOAL:NAT.F_GOAL + 3]).T, goals_of(oenv), atol=2e-5)
    np.testing.assert_allclose(obs, want, atol=5e-5, rtol=1e-5)
    check_scen_state(env, oenv)
    if mode == "mix":   # all nine QUADS_MODE_LIST scenarios occur
        assert len(set(env.env_state[NAT.E_SC_MODE].cpu().numpy().tolist())) == 9


@pytest.mark.parametrize("mode", MODES)
def test_scenario_events_from_identical_state(mode):
    """Every env placed two ticks before its next scenario event, then stepped across it from the
    oracle's state (re-synced every step): new goals, the obs goal of envs whose state-update flag is
    set (impulses, crowd()) and rewards all match."""
    cfg, env, oenv = make_pair(mode, E=128, N=8, episode_duration=15.0)
    env.reset()
    oenv.reset()
    # spawns are clipped to the room (swarm_vs_swarm centres reach the walls): a drone resting exactly on a
    # wall makes crashed_wall hinge on the fp32/fp64 sign of a ~0 velocity, so move them inside first;
    # crowd() then sends drones through walls deliberately
    for g in range(oenv.E * oenv.N):
        for c in range(2):
            oenv.drones[g].pos[c] = float(np.clip(oenv.drones[g].pos[c], -4.6, 4.6))
    rng = np.random.default_rng(21)
    crowd(oenv, rng, frac_pairs=0.4, walls=True)
    for e in range(oenv.E):
        sc = oenv.envs[e].scen
        per = {O.SC_MODES.index("ep_rand_bezier"): 500, O.SC_MODES.index("run_away"): 100}.get(sc.mode, sc.period)
        oenv.envs[e].tick = max(per - 2, 1) if e % 5 else oenv.envs[e].tick   # crowd() left some at ep_len
    changed = 0
    for t in range(5):
        oracle_to_gpu(oenv, env)
        scen_oracle_to_gpu(oenv, env)
        g0 = goals_of(oenv)
        a = rng.uniform(-1, 1, (env.I, 4)).astype(np.float32)
        obs, rew, done, term = env.step(torch.from_numpy(a).cuda())
        w_obs, w_rew, w_done, w_term = oenv.step(a.astype(np.float64))
        np.testing.assert_array_equal(done.cpu().numpy().astype(bool), w_done)
        np.testing.assert_allclose(np_(env.state[NAT.F_GOAL:NAT.F_GOAL + 3]).T, goals_of(oenv), atol=2e-5,
                                   err_msg=f"step {t} goals")
        np.testing.assert_allclose(np_(rew), w_rew, atol=2e-4, rtol=1e-4)
        assert_obs_match(np_(obs), w_obs, oenv, 18, cfg.k_neighbors)
        if w_done.any():
            np.testing.assert_allclose(np_(term)[w_done], w_term[w_done], atol=2e-4, rtol=1e-4)
        check_scen_state(env, oenv)
        changed += int((np.abs(goals_of(oenv) - g0).max(1) > 1e-9).sum())
    if mode not in ("static_diff_goal",):
        assert changed > 0, "no scenario event was exercised"


@pytest.mark.parametrize("mode", ["mix", "ep_lissajous3D", "ep_rand_bezier", "dynamic_formations", "swarm_vs_swarm"])
def test_free_running_goals(mode):
    """Goals do not depend on the (chaotic) drone states: free-running 700 steps, the GPU's goals stay on
    the oracle's through several events, curve samples and formation bounces."""
    cfg, env, oenv = make_pair(mode, E=64, N=8, seed=5)
    env.reset()
    oenv.reset()
    a = np.full((env.I, 4), -0.2, np.float32)
    at = torch.from_numpy(a).cuda()
    for t in range(700):
        env.step(at)
        oenv.step(a.astype(np.float64))
        if t % 100 == 99:
            np.testing.assert_allclose(np_(env.state[NAT.F_GOAL:NAT.F_GOAL + 3]).T, goals_of(oenv), atol=1e-2,
                                       err_msg=f"step {t}")


def test_mix_full_size_invariants():
    """4096 envs x 8 drones in mix mode: every env reset draws a scenario, goals and spawns stay finite and
    inside the room; a full episode later every env has reset once and re-drawn."""
    cfg = QuadSwarmConfig(num_envs=4096, num_agents=8, quads_mode="mix", episode_duration=0.2, seed=3)
    env = QuadSwarmEnv(cfg)
    env.reset()
    m0 = env.env_state[NAT.E_SC_MODE].cpu().numpy()
    cnt = np.bincount(m0, minlength=9)
    assert cnt.min() > 4096 / 9 * 0.7 and cnt.max() < 4096 / 9 * 1.3, cnt
    a = torch.zeros(env.I, 4, device="cuda")
    for _ in range(cfg.ep_len + 1):
        env.step(a)
    torch.cuda.synchronize()
    assert (env.env_state[NAT.E_EPISODE].cpu().numpy() == 2).all()
    g = np_(env.state[NAT.F_GOAL:NAT.F_GOAL + 3]).T
    assert np.isfinite(g).all() and np.abs(g[:, :2]).max() < 6 and g[:, 2].min() > -1 and g[:, 2].max() < 11
    assert not (env.env_state[NAT.E_SC_MODE].cpu().numpy() == m0).all()
