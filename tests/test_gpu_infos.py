"""Per-step infos on the GPU (config step_infos): the reward components the step kernels write (buffers.rew_info)
against the oracle's (pinned to the reference's own infos dicts by tests/golden/traj_n8info, obst_traj_c4info and
a_traj_n4info), the VecEnv surface built from them, and the native (device) VecEnv mode making no host sync.

Reference: flavor B infos[i]["rewards"] -- gym_art/quadrotor_multi/quadrotor_single.py:79-105, 371 and
quadrotor_multi.py:642-651; flavor A infos[i]["goal_dist"] -- quadrotor_single_rewards.py:457.
Tolerances (fp32 GPU vs fp64 oracle, identical state before every step): the continuous components within
1e-5 abs + 1e-5 rel on rows with no impulse and no contact, 2e-4 on eventful rows; the discrete ones
(on_floor, collision / pillar raw terms) identical.
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no HIP device", allow_module_level=True)

import oracle as O  # noqa: E402
from conftest import GOLDEN  # noqa: E402
from parity_utils import (crowd, gpu_to_oracle_a, oracle_params, oracle_params_a, oracle_to_gpu,  # noqa: E402
                          oracle_to_gpu_a)
from quadswarm_amd import QuadSwarmConfig  # noqa: E402
from quadswarm_amd import _native as N_  # noqa: E402
from quadswarm_amd.env import QuadSwarmEnv  # noqa: E402
from quadswarm_amd.infos import REWARD_KEYS_B, REWARD_KEYS_OBST  # noqa: E402
from quadswarm_amd.vec_env import GpuQuadVecEnv  # noqa: E402
from test_gpu_parity import eventful_rows  # noqa: E402
from test_gpu_parity_a import _perturb  # noqa: E402
from test_gpu_parity_obst import aim_at_obstacles  # noqa: E402

DISCRETE = [N_.RI_CRASH, N_.RI_QUADCOL, N_.RI_OBST]
CONT = [N_.RI_DIST, N_.RI_EFFORT, N_.RI_ORIENT, N_.RI_SPIN, N_.RI_PROX]


def np_(t):
    return t.double().cpu().numpy()


def ocomp(oenv):
    return np.array([list(oenv.drones[g].rinfo) for g in range(oenv.E * oenv.N)]).T


def check_components(env, oenv, quiet, t):
    got, want = np_(env.rew_info), ocomp(oenv)
    np.testing.assert_array_equal(got[DISCRETE], want[DISCRETE], err_msg=f"step {t} discrete components")
    np.testing.assert_allclose(got[CONT], want[CONT], atol=2e-4, rtol=1e-4, err_msg=f"step {t} components")
    if quiet.any():
        np.testing.assert_allclose(got[CONT][:, quiet], want[CONT][:, quiet], atol=1e-5, rtol=1e-5,
                                   err_msg=f"step {t} quiet components")
    return want


@pytest.mark.parametrize("N,K,obst", [(8, 6, False), (1, 0, False), (32, 6, False), (8, 2, True)])
def test_reward_components_match_oracle(N, K, obst):
    E = 2048 // N
    if obst:
        cfg = QuadSwarmConfig.c4(num_envs=E, num_agents=N, seed=21, episode_duration=0.3, step_infos=True)
    else:
        cfg = QuadSwarmConfig(num_envs=E, num_agents=N, neighbor_visible_num=K if N > 1 else 0,
                              neighbor_obs_type="pos_vel" if N > 1 else "none", seed=7, episode_duration=0.5,
                              step_infos=True)
    env = QuadSwarmEnv(cfg)
    oenv = O.OracleEnv(oracle_params(cfg), seed=cfg.seed)
    env.reset()
    oenv.reset()
    rng = np.random.default_rng(3)
    crowd(oenv, rng, walls=not obst)
    if obst:
        aim_at_obstacles(oenv, rng)
    seen = np.zeros(N_.NRI, int)
    for t in range(10):
        oracle_to_gpu(oenv, env)
        floor_before = np.array([oenv.drones[g].on_floor != 0 for g in range(env.I)])
        a = rng.uniform(-1, 1, (env.I, 4)).astype(np.float32)
        env.step(torch.from_numpy(a).cuda())
        w_obs, w_rew, w_done, _ = oenv.step(a.astype(np.float64))
        quiet = ~eventful_rows(oenv, floor_before, w_done)
        want = check_components(env, oenv, quiet, t)
        seen += (want != 0).sum(1)
    # every term was exercised (the pillar term only with obstacles, the pair terms only with neighbours)
    # (crowd() drives drones into the floor only in envs of 3 or more drones)
    need = [N_.RI_DIST, N_.RI_EFFORT, N_.RI_ORIENT, N_.RI_SPIN] + ([N_.RI_CRASH] if N >= 3 and not obst else []) + \
        ([N_.RI_QUADCOL, N_.RI_PROX] if N > 1 else []) + ([N_.RI_OBST] if obst else [])
    assert (seen[need] > 0).all(), seen


def test_goal_dist_matches_oracle_flavor_a():
    cfg = QuadSwarmConfig.sb_train(num_envs=256, num_agents=8, neighbor_obs_type="dist_angle", seed=11,
                                   step_infos=True)
    env = QuadSwarmEnv(cfg)
    oenv = O.OracleEnvA(oracle_params_a(cfg), seed=11)
    oenv.set_capture_radius(cfg.initial_capture_radius)
    env.reset()
    oenv.reset()
    rng = np.random.default_rng(5)
    n_done = 0
    for t in range(6):
        _perturb(oenv, cfg, rng, t)
        oracle_to_gpu_a(oenv, env)
        a = rng.uniform(-1.2, 1.2, (env.I, 2)).astype(np.float32)
        env.step(torch.from_numpy(a).cuda())
        _, _, w_done, _, _ = oenv.step(a.astype(np.float64))
        np.testing.assert_allclose(np_(env.rew_info[N_.RI_GOAL_DIST]), ocomp(oenv)[O.RI_GOAL_DIST], atol=3e-5,
                                   rtol=1e-5, err_msg=f"goal_dist step {t}")
        n_done += int(w_done.sum())
        gpu_to_oracle_a(env, oenv)
    assert n_done > 0   # the done rows report the pre-reset distance


@pytest.mark.parametrize("flavor", ["B", "A"])
def test_step_infos_leave_the_step_unchanged(flavor):
    """The components are extra stores only: obs, rewards, dones and the whole state are bitwise those of a
    handle without them."""
    outs = []
    for on in (False, True):
        if flavor == "B":
            cfg = QuadSwarmConfig(num_envs=256, num_agents=8, seed=2, episode_duration=0.2, step_infos=on)
        else:
            cfg = QuadSwarmConfig.sb_train(num_envs=256, num_agents=8, seed=2, episode_duration=0.4, step_infos=on)
        env = QuadSwarmEnv(cfg)
        env.reset()
        g = torch.Generator(device="cuda").manual_seed(1)
        acc = []
        for _ in range(30):
            a = torch.rand(env.I, cfg.act_dim, device="cuda", generator=g) * 2 - 1
            obs, rew, done, _ = env.step(a)
            acc += [obs.clone(), rew.clone(), done.clone()]
        acc += [env.state.clone(), env.istate.clone(), env.env_state.clone()]
        outs.append(acc)
        env.close()
    for x, y in zip(*outs):
        assert torch.equal(x, y)


def _infokeys(name):
    return json.load(open(os.path.join(GOLDEN, name)))["rewards_keys"]


@pytest.mark.parametrize("obst", [False, True])
def test_vec_env_rewards_infos(obst):
    """Every agent row of every step carries the reference's infos["rewards"] keys (the fixtures' own key sets),
    and the terms add up to the step's reward like compute_reward_weighted + the swarm terms do."""
    if obst:
        cfg = QuadSwarmConfig.c4(num_envs=32, num_agents=8, seed=3, episode_duration=0.1)
        keys = _infokeys("obst_traj_c4info_infokeys.json")
        assert sorted(keys) == sorted(REWARD_KEYS_B + REWARD_KEYS_OBST)
    else:
        cfg = QuadSwarmConfig(num_envs=32, num_agents=8, seed=3, episode_duration=0.1)
        keys = _infokeys("traj_n8info_infokeys.json")
    venv = GpuQuadVecEnv(cfg)
    venv.reset()
    rng = np.random.default_rng(0)
    n_done = 0
    for t in range(15):
        _, rew, dones, infos = venv.step(rng.uniform(-1, 1, (256, 4)).astype(np.float32))
        for i in range(0, 256, 7):
            r = infos[i]["rewards"]
            assert sorted(r) == sorted(keys)
            total = (r["rew_pos"] + r["rew_action"] + r["rew_crash"] + r["rew_orient"] + r["rew_spin"] +
                     r["rew_quadcol"] + r["rew_proximity"] + r.get("rew_quadcol_obstacle", 0.0))
            assert total == pytest.approx(float(rew[i]), abs=2e-6, rel=1e-5)
            assert r["rewraw_pos"] == pytest.approx(r["rew_pos"] / venv.env.reward_coefficients()["pos"])
        for i in np.flatnonzero(dones):
            assert {"terminal_observation", "rewards", "episode_extra_stats"} <= set(infos[int(i)])
            n_done += 1
    assert n_done > 0
    venv.close()


def test_vec_env_goal_dist_infos_flavor_a():
    venv = GpuQuadVecEnv(QuadSwarmConfig.sb_train(num_envs=16, num_agents=4, seed=1))
    venv.reset()
    venv.env_method("set_capture_radius", 0.0, indices=list(range(8, 16)))
    _, _, dones, infos = venv.step(np.zeros((64, 2), np.float32))
    gd = venv.env.rew_info[N_.RI_GOAL_DIST].cpu().numpy()
    for i in range(64):
        assert infos[i]["rewards"] == {} and infos[i]["goal_dist"] == pytest.approx(float(gd[i]))
        assert ("terminal_observation" in infos[i]) == bool(dones[i])
    assert dones[:32].any()
    venv.close()


@pytest.mark.parametrize("flavor", ["B", "A"])
def test_native_step_makes_no_host_sync(flavor):
    """Native mode (as_torch): a step issues no synchronising device-to-host transfer (torch's sync debug mode
    raises on any); the lazily built infos resolve on read, and refuse once the next step has run."""
    if flavor == "B":
        cfg = QuadSwarmConfig(num_envs=64, num_agents=8, seed=4, episode_duration=0.05)
    else:
        cfg = QuadSwarmConfig.sb_train(num_envs=64, num_agents=4, seed=4, episode_duration=0.4)
    venv = GpuQuadVecEnv(cfg, as_torch=True)
    venv.reset()
    a = torch.zeros(venv.num_envs, cfg.act_dim, device="cuda")
    venv.step(a)   # allocator warm-up outside the checked region
    torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode("error")
    try:
        for _ in range(20):
            obs, rew, done, infos = venv.step(a)
    finally:
        torch.cuda.set_sync_debug_mode(0)
    assert obs.is_cuda and rew.is_cuda and done.is_cuda and len(infos) == venv.num_envs
    rows = infos.done_rows   # resolves now (one host read)
    np.testing.assert_array_equal(rows, np.flatnonzero(done.cpu().numpy()))
    key = "rewards" if flavor == "B" else "goal_dist"
    assert key in infos[0]
    stale = venv.step(a)[3]
    venv.step(a)
    with pytest.raises(RuntimeError, match="older step"):
        stale[0]
    venv.close()


def test_native_mode_raises_on_nan_reward():
    venv = GpuQuadVecEnv(QuadSwarmConfig(num_envs=8, num_agents=8, seed=1), as_torch=True)
    venv.reset()
    a = torch.zeros(64, 4, device="cuda")
    venv.step(a)
    a[3, 1] = float("nan")
    venv.step(a)
    a[3, 1] = 0.0
    with pytest.raises(ValueError, match="reward is Nan"):
        for _ in range(50):   # the stream-ordered counter copy is read once it has landed
            venv.step(a)
            torch.cuda.synchronize()
    venv.close()


def test_vec_env_nan_check_resyncs_after_counter_reset():
    """A counter reset through the underlying env (not the VecEnv) must not hide a later NaN reward."""
    venv = GpuQuadVecEnv(QuadSwarmConfig(num_envs=8, num_agents=8, seed=1))
    venv.reset()
    a = np.zeros((64, 4), np.float32)
    a[3, 1] = np.nan
    with pytest.raises(ValueError):
        venv.step(a)
    with pytest.raises(ValueError):
        venv.step(a)   # a second NaN reward is a new increase
    venv.env.reset_counters()
    venv.step(np.zeros((64, 4), np.float32))   # the counter dropped to 0: resynchronised, no raise
    with pytest.raises(ValueError):
        venv.step(a)
    venv.close()
