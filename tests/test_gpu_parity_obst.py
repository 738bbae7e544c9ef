"""GPU parity for the obstacle rows: SDF obs, pillar collisions and
impulses, obstacle maps and the mix of o_random / o_static_same_goal spawns -- the HIP step through
the C ABI against the CPU oracle (identical Philox draws) and the reference's noise-free flight.

Tolerances as tests/test_gpu_parity.py (fp32 GPU vs fp64 oracle).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no HIP device", allow_module_level=True)

import oracle as O  # noqa: E402
from parity_utils import assert_obs_match, crowd, gpu_to_oracle, oracle_params, oracle_to_gpu  # noqa: E402
from quadswarm_amd import QuadSwarmConfig, _native as NAT  # noqa: E402
from quadswarm_amd.env import QuadSwarmEnv  # noqa: E402


def make_pair(E=256, N=8, seed=21, **kw):
    cfg = QuadSwarmConfig.c4(num_envs=E, num_agents=N, seed=seed, **kw)
    env = QuadSwarmEnv(cfg)
    oenv = O.OracleEnv(oracle_params(cfg), seed=seed)
    return cfg, env, oenv


def np_(t):
    return t.double().cpu().numpy()


def obstacles_of(oenv):
    return np.array([[[oenv.envs[e].obst[o][0], oenv.envs[e].obst[o][1]] for o in range(oenv.envs[e].n_obst)]
                     for e in range(oenv.E)])


@pytest.mark.parametrize("mode", ["mix", "o_random", "o_static_same_goal"])
def test_reset_matches_oracle(mode):
    cfg, env, oenv = make_pair(quads_mode=mode)
    obs = np_(env.reset())
    want = oenv.reset()
    np.testing.assert_array_equal(np_(env.obstacles), obstacles_of(oenv))
    np.testing.assert_allclose(obs, want, atol=2e-5, rtol=1e-5)
    pos = np.array([oenv.drones[g].pos[:] for g in range(env.I)])
    np.testing.assert_allclose(np_(env.drone_fields()["pos"]), pos, atol=2e-6)
    goal = np.array([oenv.drones[g].goal[:] for g in range(env.I)])
    np.testing.assert_allclose(np_(env.drone_fields()["goal"]), goal, atol=2e-6)
    if mode == "mix":   # both scenario modes appear
        modes = {int(oenv.envs[e].obst_mode) for e in range(oenv.E)}
        assert modes == {0, 1}


def aim_at_obstacles(oenv, rng):
    """Send the first three drones of every env at a pillar (collisions + impulses)."""
    N = oenv.N
    for e in range(oenv.E):
        ev = oenv.envs[e]
        for i in range(min(3, N)):
            d = oenv.drones[e * N + i]
            o = ev.obst[(i + e) % ev.n_obst]
            ang = rng.uniform(-np.pi, np.pi)
            d.pos[0], d.pos[1] = o[0] + 0.4 * np.cos(ang), o[1] + 0.4 * np.sin(ang)
            d.vel[0], d.vel[1] = -2.0 * np.cos(ang), -2.0 * np.sin(ang)


@pytest.mark.parametrize("N", [8, 4])
def test_one_step_from_identical_state(N):
    cfg, env, oenv = make_pair(E=2048 // N, N=N, episode_duration=0.3)
    env.reset()
    oenv.reset()
    rng = np.random.default_rng(4)
    crowd(oenv, rng, walls=False)
    aim_at_obstacles(oenv, rng)
    K = cfg.k_neighbors
    so = NAT.SELF_OBS_DIM[NAT.OBS_REPR[cfg.obs_repr]]
    stats = dict(done=0, obst=0)
    for t in range(12):
        oracle_to_gpu(oenv, env)
        a = rng.uniform(-1, 1, (env.I, 4)).astype(np.float32)
        obs, rew, done, term = env.step(torch.from_numpy(a).cuda())
        w_obs, w_rew, w_done, w_term = oenv.step(a.astype(np.float64))
        np.testing.assert_array_equal(done.cpu().numpy().astype(bool), w_done)
        np.testing.assert_allclose(np_(rew), w_rew, atol=2e-4, rtol=1e-4)
        g_obs = np_(obs)
        # SDF block (last 9) compared directly; self + neighbour parts through the tie-aware check
        np.testing.assert_allclose(g_obs[:, -9:], w_obs[:, -9:], atol=2e-4, rtol=1e-4)
        assert_obs_match(g_obs[:, :-9], w_obs[:, :-9], oenv, so, K)
        if w_done.any():
            np.testing.assert_allclose(np_(term)[w_done][:, -9:], w_term[w_done][:, -9:], atol=2e-4, rtol=1e-4)
            np.testing.assert_array_equal(np_(env.obstacles), obstacles_of(oenv))   # new maps after resets
        stats["done"] += int(w_done.sum())
        stats["obst"] += int((w_rew < -2.0).sum())
        pos = np.array([oenv.drones[g].pos[:] for g in range(env.I)])
        vel = np.array([oenv.drones[g].vel[:] for g in range(env.I)])
        np.testing.assert_allclose(np_(env.drone_fields()["pos"]), pos, atol=2e-5)
        np.testing.assert_allclose(np_(env.drone_fields()["vel"]), vel, atol=5e-4, rtol=1e-4)
        gpu_to_oracle(env, oenv)
    assert stats["done"] > 0 and stats["obst"] > 0


def test_reference_quiet_flight_with_obstacles(golden):
    """The reference's noise-free 8-drone flight among 12 pillars (obst_traj_quiet), replayed on the GPU
    until the first random event (a collision at step 89 draws impulse noise)."""
    g = golden("obst_traj_quiet")
    n, k = int(g["n"]), int(g["k"])
    cfg = QuadSwarmConfig.c4(num_envs=1, num_agents=n, sense_noise=None, thrust_noise_ratio=0.0, use_downwash=False,
                             episode_duration=15.0, collision_smooth_max_penalty=10.0)
    env = QuadSwarmEnv(cfg)
    oenv = O.OracleEnv(oracle_params(cfg), seed=0)
    for i in range(n):
        d = oenv.drones[i]
        O.set_drone(d, pos=g["init_pos"][i], vel=g["init_vel"][i], rot=g["init_rot"][i], omega=g["init_omega"][i],
                    thrust_rot_damp=g["init_rd"][i], thrust_cmds_damp=g["init_cd"][i], ou=g["init_ou"][i],
                    goal=g["init_goal"][i])
        d.since_last_svd = float(g["init_since"][i])
        for a in range(3):
            oenv.envs[0].obs_vel[i][a] = g["init_env_vel"][i][a]
    ob = g["init_obst"]
    oenv.envs[0].n_obst = len(ob)
    for o in range(len(ob)):
        oenv.envs[0].obst[o][0], oenv.envs[0].obst[o][1] = ob[o][0], ob[o][1]
    oenv.envs[0].tick = int(g["init_tick"])
    oracle_to_gpu(oenv, env)
    first_event = int(np.argwhere(g["rew"] < -1)[0, 0]) if (g["rew"] < -1).any() else len(g["actions"])
    assert first_event > 50
    for t in range(first_event):
        a = torch.from_numpy(np.ascontiguousarray(g["actions"][t], dtype=np.float32)).cuda()
        obs, rew, done, _ = env.step(a)
        got = np_(obs)
        np.testing.assert_allclose(got[:, -9:], g["obs"][t][:, -9:], atol=2e-3, err_msg=f"sdf step {t}")
        np.testing.assert_allclose(got[:, :19], g["obs"][t][:, :19], atol=2e-3, err_msg=f"self step {t}")
        np.testing.assert_allclose(np_(rew), g["rew"][t], atol=1e-3)


def test_full_size_c4_properties():
    cfg = QuadSwarmConfig.c4(num_envs=4096, num_agents=8, seed=5, episode_duration=0.5)
    env = QuadSwarmEnv(cfg)
    obs = env.reset()
    assert obs.shape == (32768, 40) and torch.isfinite(obs).all()
    ob = env.obstacles.cpu().numpy()
    assert ob.shape == (4096, 12, 2)
    # pillars sit on distinct cell centres of the 8x8 area
    assert np.all(np.abs(ob) <= 3.5) and np.all((ob + 3.5) == np.round(ob + 3.5))
    for e in range(0, 4096, 97):
        assert len({tuple(x) for x in ob[e]}) == 12
    # drones spawn in free cells (never inside a pillar) within the 0.1 m spawn box
    pos = env.drone_fields()["pos"].cpu().numpy().reshape(4096, 8, 3)
    dmin = np.linalg.norm(pos[:, :, None, :2] - ob[:, None, :, :], axis=-1).min(-1)
    assert dmin.min() > 0.5 - 0.1 * np.sqrt(2) - 1e-5
    rng = torch.Generator(device="cuda").manual_seed(0)
    dones = 0
    for t in range(60):
        a = torch.rand(env.I, 4, device="cuda", generator=rng) * 2 - 1
        obs, rew, done, term = env.step(a)
        assert torch.isfinite(obs).all()
        dones += int(done.sum())
    assert dones == 32768   # ep_len 50: every env reset once inside the run


# ---------------------------------------------------------------- obstacle domain randomisation
DR_RUN = dict(replay_buffer_sample_prob=0.75, domain_random=True, obst_density_random=True, obst_size_random=True,
              obst_density_min=0.05, obst_density_max=0.2, obst_size_min=0.3, obst_size_max=0.6)   # obst_domain_random.py
DR_ZERO = dict(DR_RUN, obst_density_min=0.0, obst_size_min=0.0)   # 0.0 choices: falsy, the env keeps its value


def assert_obstacles_match(env, oenv):
    """Per env: the domain-randomisation indices, then the env's first n pillar slots."""
    es = env.env_state.cpu().numpy()
    ob = np_(env.obstacles)
    for e in range(oenv.E):
        ev = oenv.envs[e]
        assert (int(es[NAT.E_OBST_M, e]), int(es[NAT.E_OBST_SZ, e])) == (ev.obst_mi, ev.obst_si), e
        want = np.array([[ev.obst[o][0], ev.obst[o][1]] for o in range(ev.n_obst)])
        np.testing.assert_array_equal(ob[e, :ev.n_obst], want)


@pytest.mark.parametrize("dr", [DR_RUN, DR_ZERO], ids=["run", "zero_choices"])
def test_domain_random_resets_match_oracle(dr):
    cfg, env, oenv = make_pair(E=512, **dr)
    assert env.obstacles.shape[1] == cfg.max_obstacles
    for r in range(3):   # explicit resets: each draws a (density, size) pair per env (wrapper.reset)
        obs = np_(env.reset())
        want = oenv.reset()
        assert_obstacles_match(env, oenv)
        np.testing.assert_allclose(obs, want, atol=2e-5, rtol=1e-5)
    counts = {oenv.envs[e].n_obst for e in range(oenv.E)}
    sizes = {oenv.envs[e].obst_si for e in range(oenv.E)}
    assert len(counts) >= 3 and len(sizes) >= 3


def test_domain_random_steps_from_identical_state():
    """Fused auto-resets draw new (density, size) pairs (the replay wrapper's new_episode); SDF obs, pillar
    hits and impulses use each env's own pillar count and radius."""
    cfg, env, oenv = make_pair(E=256, episode_duration=0.3, **DR_RUN)
    env.reset()
    oenv.reset()
    rng = np.random.default_rng(7)
    crowd(oenv, rng, walls=False)
    aim_at_obstacles(oenv, rng)
    K = cfg.k_neighbors
    so = NAT.SELF_OBS_DIM[NAT.OBS_REPR[cfg.obs_repr]]
    stats = dict(done=0, obst=0)
    for t in range(12):
        oracle_to_gpu(oenv, env)
        a = rng.uniform(-1, 1, (env.I, 4)).astype(np.float32)
        obs, rew, done, term = env.step(torch.from_numpy(a).cuda())
        w_obs, w_rew, w_done, w_term = oenv.step(a.astype(np.float64))
        np.testing.assert_array_equal(done.cpu().numpy().astype(bool), w_done)
        np.testing.assert_allclose(np_(rew), w_rew, atol=2e-4, rtol=1e-4)
        g_obs = np_(obs)
        np.testing.assert_allclose(g_obs[:, -9:], w_obs[:, -9:], atol=2e-4, rtol=1e-4)
        assert_obs_match(g_obs[:, :-9], w_obs[:, :-9], oenv, so, K)
        assert_obstacles_match(env, oenv)
        stats["done"] += int(w_done.sum())
        stats["obst"] += int((w_rew < -2.0).sum())
        gpu_to_oracle(env, oenv)
    assert stats["done"] > 0 and stats["obst"] > 0


# ---------------------------------------------------------------- the obstacle maps' dynamic scenarios
# o_swap_goals / o_ep_rand_bezier / o_dynamic_same_goal (scenarios/obstacles/, QUADS_MODE_LIST_OBSTACLES_TEST): the
# oracle's restatement is pinned to the reference's own classes by tests/test_oracle_golden_oscen.py; here the GPU
# matches it draw for draw (Philox) at reset and across the scenario's events.
OSCEN = ["o_swap_goals", "o_ep_rand_bezier", "o_dynamic_same_goal"]


def _scen_rows(env):
    es = env.env_state.cpu().numpy()
    ef = NAT.env_f_rows(env.env_f.double().cpu().numpy())
    return es, ef


def assert_scen_match(env, oenv, atol=2e-5):
    from parity_utils import OR_TO_GPU_MODE
    es, ef = _scen_rows(env)
    for e in range(oenv.E):
        sc = oenv.envs[e].scen
        assert int(es[NAT.E_SC_MODE, e]) == OR_TO_GPU_MODE[sc.mode], e
        assert int(es[NAT.E_SC_PERIOD, e]) == sc.period, e
        assert int(es[NAT.E_SC_FORM, e]) == sc.formation, e
        np.testing.assert_allclose(ef[NAT.ENVF_SC_CENTER:NAT.ENVF_SC_CENTER + 3, e], sc.center[:], atol=atol)
        np.testing.assert_allclose([ef[NAT.ENVF_SC_SIZE, e], ef[NAT.ENVF_SC_LAYER, e]], [sc.size, sc.layer], atol=1e-6)


def goals_of(oenv):
    return np.array([oenv.drones[g].goal[:] for g in range(oenv.E * oenv.N)])


@pytest.mark.parametrize("N", [8, 2])
@pytest.mark.parametrize("mode", OSCEN)
def test_dynamic_scenario_reset_matches_oracle(mode, N):
    cfg, env, oenv = make_pair(E=512, N=N, quads_mode=mode, neighbor_visible_num=min(2, N - 1))
    obs = np_(env.reset())
    want = oenv.reset()
    np.testing.assert_array_equal(np_(env.obstacles), obstacles_of(oenv))
    np.testing.assert_allclose(obs, want, atol=2e-5, rtol=1e-5)
    pos = np.array([oenv.drones[g].pos[:] for g in range(env.I)])
    np.testing.assert_allclose(np_(env.drone_fields()["pos"]), pos, atol=2e-6)
    np.testing.assert_allclose(np_(env.drone_fields()["goal"]), goals_of(oenv), atol=2e-5)
    assert_scen_match(env, oenv)
    periods = {oenv.envs[e].scen.period for e in range(oenv.E)}
    assert len(periods) > 10 if mode != "o_ep_rand_bezier" else periods == {1}
    if mode == "o_swap_goals":   # the formation draws cover several formations
        assert len({oenv.envs[e].scen.formation for e in range(oenv.E)}) >= 5


@pytest.mark.parametrize("mode", OSCEN)
def test_dynamic_scenario_steps_from_identical_state(mode):
    """Steps across the scenario's events from identical states: every env's tick is set a few ticks before its next
    event (the swap / resample period, the bezier curve's 6 s boundary, tick 1), goals, rewards, obs and the scenario
    record compared after every step."""
    from parity_utils import scen_gpu_to_oracle, scen_oracle_to_gpu
    N = 8
    cfg, env, oenv = make_pair(E=256, N=N, quads_mode=mode, episode_duration=15.0)
    env.reset()
    oenv.reset()
    rng = np.random.default_rng(11)
    for e in range(oenv.E):   # the next event within 0..5 steps (tick 0 -> the tick-1 event)
        ev = oenv.envs[e]
        per = 600 if mode == "o_ep_rand_bezier" else ev.scen.period
        ev.tick = 0 if e % 4 == 0 else max(per * (1 + e % 2) - int(rng.integers(1, 6)), 0)
    K = cfg.k_neighbors
    so = NAT.SELF_OBS_DIM[NAT.OBS_REPR[cfg.obs_repr]]
    moved = 0
    for t in range(10):
        oracle_to_gpu(oenv, env)
        scen_oracle_to_gpu(oenv, env)
        g0 = goals_of(oenv)
        a = (rng.uniform(-1, 1, (env.I, 4)) * 0.2 + 0.05).astype(np.float32)
        obs, rew, done, term = env.step(torch.from_numpy(a).cuda())
        w_obs, w_rew, w_done, w_term = oenv.step(a.astype(np.float64))
        np.testing.assert_array_equal(done.cpu().numpy().astype(bool), w_done)
        np.testing.assert_allclose(np_(env.drone_fields()["goal"]), goals_of(oenv), atol=2e-5, err_msg=f"step {t}")
        np.testing.assert_allclose(np_(rew), w_rew, atol=2e-4, rtol=1e-4)
        g_obs = np_(obs)
        np.testing.assert_allclose(g_obs[:, -9:], w_obs[:, -9:], atol=2e-4, rtol=1e-4)
        assert_obs_match(g_obs[:, :-9], w_obs[:, :-9], oenv, so, K)
        assert_scen_match(env, oenv)
        moved += int((np.abs(goals_of(oenv) - g0).max(axis=1) > 1e-6).sum())
        gpu_to_oracle(env, oenv)
        scen_gpu_to_oracle(env, oenv)
    assert moved > env.I // 4, moved   # the events happened in the window


@pytest.mark.parametrize("mode", OSCEN)
def test_full_size_dynamic_scenarios(mode):
    """4096 x 8 under each mode: finite obs, goals inside the room (the bezier goal inside its shrunk box), goals that
    move, the episode stats' scenario name of the reference's class."""
    from quadswarm_amd.stats import SCENARIO_NAMES
    cfg = QuadSwarmConfig.c4(num_envs=4096, num_agents=8, seed=9, quads_mode=mode, episode_duration=7.0)
    env = QuadSwarmEnv(cfg)
    env.reset()
    g0 = env.drone_fields()["goal"].clone()
    rng = torch.Generator(device="cuda").manual_seed(3)
    for t in range(700):
        a = torch.rand(env.I, 4, device="cuda", generator=rng) * 2 - 1
        obs, rew, done, term = env.step(a)
    assert torch.isfinite(obs).all()
    g = env.drone_fields()["goal"]
    assert torch.isfinite(g).all() and (g[:, :2].abs() <= 5.0).all() and (g[:, 2] >= 0.0).all()
    frac_moved = float(((g - g0).abs().max(dim=1).values > 1e-6).float().mean())
    assert frac_moved > 0.5, frac_moved
    es = env.env_state.cpu().numpy()
    ids = set(es[NAT.E_SC_MODE].tolist())
    assert ids == {19 + OSCEN.index(mode)} and SCENARIO_NAMES[ids.pop()] == mode
