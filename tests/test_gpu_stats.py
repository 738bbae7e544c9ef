"""episode_extra_stats on the GPU (quadrotor_multi.py:555-656 accumulators, :739-831 the dicts at done).

* the step kernel's accumulators and done rows against the oracle's (which test_oracle_golden.py pins to the
  reference's own dicts on the n8stats trajectory), re-syncing the GPU to the oracle every step, so every
  collision / wall / floor / ceiling / settle / final-window / distance path is compared on identical states;
* the counters do not perturb the step: obs / rewards / physics bitwise equal with episode_stats off;
* GpuQuadVecEnv's infos carry the reference's keys (and the replay wrapper's, quad_experience_replay.py:124-137).
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
from parity_utils import crowd, oracle_params, oracle_to_gpu  # noqa: E402
from quadswarm_amd import QuadSwarmConfig  # noqa: E402
from quadswarm_amd import _native as N_  # noqa: E402
from quadswarm_amd import stats as S  # noqa: E402
from quadswarm_amd.env import QuadSwarmEnv  # noqa: E402
from quadswarm_amd.vec_env import GpuQuadVecEnv  # noqa: E402

COUNT_COLS = [S.ES_COL, S.ES_ROOM, S.ES_FLOOR, S.ES_WALL, S.ES_CEIL, S.ES_COL_SETTLE, S.ES_COL_FINAL, S.ES_OCOL,
              S.ES_OCOL_SETTLE, S.ES_O35, S.ES_O5, S.ES_SCEN]


def _oracle_rows(oenv, e):
    """The oracle's [N, NES] stats rows of env e after its done step (env counters + per-drone distances)."""
    N = oenv.N
    base = np.array(oenv.envs[e].ep_stats[:], dtype=np.float64)
    rows = np.repeat(base[None], N, 0)
    for i in range(N):
        d = oenv.drones[e * N + i]
        rows[i, S.ES_D1], rows[i, S.ES_D3], rows[i, S.ES_D5] = d.ep_dist[0], d.ep_dist[1], d.ep_dist[2]
    return rows


def test_episode_stats_match_oracle():
    E, N = 128, 8
    cfg = QuadSwarmConfig(num_envs=E, num_agents=N, neighbor_visible_num=6, seed=4)
    env = QuadSwarmEnv(cfg)
    assert env.estats is not None
    oenv = O.OracleEnv(oracle_params(cfg), seed=4)
    env.reset()
    oenv.reset()
    rng = np.random.default_rng(11)
    ep = cfg.ep_len
    for e in range(E):       # the last ~2 s of the episode: past the 1.5 s grace, inside every distance window
        oenv.envs[e].tick = ep - 200 + (e % 37)
    n_done_envs, seen = 0, np.zeros(len(COUNT_COLS))
    for t in range(200):
        if t % 20 == 0:
            crowd(oenv, rng, frac_pairs=0.6)
            for e in range(E):       # crowd() parks every 5th env at its last tick: undo that here
                if oenv.envs[e].tick >= ep:
                    oenv.envs[e].tick = ep - 1 - (e % 50)
        oracle_to_gpu(oenv, env)
        a = rng.uniform(-1, 1, (env.I, 4)).astype(np.float32)
        _, _, done, _ = env.step(torch.from_numpy(a).cuda())
        _, _, w_done, _ = oenv.step(a.astype(np.float64))
        done = done.cpu().numpy().astype(bool)
        np.testing.assert_array_equal(done, w_done)
        envs = np.flatnonzero(w_done.reshape(E, N)[:, 0])
        if not len(envs):
            continue
        est = env.estats.double().cpu().numpy()
        for e in envs:
            got, want = est[e * N:(e + 1) * N], _oracle_rows(oenv, e)
            np.testing.assert_array_equal(got[:, COUNT_COLS], want[:, COUNT_COLS], err_msg=f"step {t} env {e}")
            for c in (S.ES_SUCCESS, S.ES_DEADLOCK, S.ES_COLRATE, S.ES_NCOLRATE, S.ES_OCOLRATE):
                np.testing.assert_allclose(got[:, c], want[:, c], rtol=1e-6, atol=1e-7, err_msg=f"{t} {e} col {c}")
            np.testing.assert_allclose(got[:, [S.ES_D1, S.ES_D3, S.ES_D5]], want[:, [S.ES_D1, S.ES_D3, S.ES_D5]],
                                       rtol=2e-5, atol=2e-5, err_msg=f"step {t} env {e}")
            seen += got[0, COUNT_COLS] != 0
            n_done_envs += 1
    assert n_done_envs >= E
    # the episodes exercised collisions (all / after settle / final 5 s), room, floor, wall and ceiling hits
    for k, c in enumerate(COUNT_COLS[:7]):
        assert seen[k] > 0, c


@pytest.mark.parametrize("over", [{}, dict(quads_mode="mix", replay_buffer_sample_prob=0.75)])
def test_stats_leave_the_step_unchanged(over):
    def mk(st):
        return QuadSwarmEnv(QuadSwarmConfig(num_envs=128, num_agents=8, seed=6, episode_duration=0.6,
                                            episode_stats=st, **over))
    on, off = mk(True), mk(False)
    assert on.estats is not None and off.estats is None
    assert torch.equal(on.reset(), off.reset())
    g = torch.Generator(device="cuda").manual_seed(3)
    for t in range(150):
        a = (torch.rand(on.I, 4, device="cuda", generator=g) * 2 - 1).contiguous()
        r_on = [x.clone() for x in on.step(a)]
        r_off = [x.clone() for x in off.step(a)]
        for x, y in zip(r_on, r_off):
            assert torch.equal(x, y), t
    assert torch.equal(on.state[:N_.F_DRING], off.state[:N_.F_DRING])


def _ref_keys():
    ev = json.load(open(os.path.join(GOLDEN, "traj_n8stats_stats.json")))["events"]
    return sorted(ev[0]["agents"][0])


@pytest.mark.parametrize("replay", [False, True])
def test_vec_env_infos_carry_reference_keys(replay):
    over = dict(quads_mode="mix", replay_buffer_sample_prob=0.75) if replay else {}
    venv = GpuQuadVecEnv(QuadSwarmConfig(num_envs=32, num_agents=8, seed=1, episode_duration=0.3, **over))
    venv.reset()
    rng = np.random.default_rng(0)
    n_done = 0
    for t in range(70):
        _, _, dones, infos = venv.step(rng.uniform(-1, 1, (256, 4)).astype(np.float32))
        for i in np.flatnonzero(dones):
            x = infos[int(i)]["episode_extra_stats"]
            keys = sorted(k for k in x if not k.startswith("replay/"))
            if not replay:
                assert keys == _ref_keys()
            else:   # mix names its scenario per episode ("<scenario>/..." keys); a replayed one reports 2 counts
                if "num_collisions_replay" in x:
                    assert keys == ["num_collisions_obst_replay", "num_collisions_replay"]
                else:
                    sc = {k.split("/")[0] for k in keys if "/" in k and not k.startswith("metric/")}
                    assert len(sc) == 1 and sc <= set(S.SCENARIO_NAMES.values()), sc
                    name = next(iter(sc))
                    assert keys == sorted(k.replace("static_same_goal/", name + "/") for k in _ref_keys())
                rk = sorted(k for k in x if k.startswith("replay/"))
                assert rk == sorted(["replay/replay_rate", "replay/new_episode_rate", "replay/replay_buffer_size",
                                     "replay/avg_replayed", "replay/obst_density", "replay/obst_size"])
                assert 0.0 <= x["replay/replay_rate"] <= 1.0
                assert x["replay/replay_rate"] + x["replay/new_episode_rate"] == pytest.approx(1.0)
            assert all(np.isfinite(v) for v in x.values())
            n_done += 1
    assert n_done == 2 * 256
    assert venv.counters() == {"nonfinite_obs": 0, "nonfinite_rew": 0, "nonfinite_state": 0}
    venv.close()


def test_vec_env_raises_on_nan_reward():
    venv = GpuQuadVecEnv(QuadSwarmConfig(num_envs=8, num_agents=8, seed=1))
    venv.reset()
    a = np.zeros((64, 4), np.float32)
    venv.step(a)
    a[3, 1] = np.nan
    with pytest.raises(ValueError, match="reward is Nan"):
        venv.step(a)
    assert venv.counters()["nonfinite_rew"] == 1
    venv.close()


@pytest.mark.parametrize("E,N", [(128, 8), (8, 128)])
def test_flavor_a_episode_stats_match_oracle(E, N):
    """Flavor A (quadrotor_multi_rewards.py:649-720 per tick, :886-969 at done): the A kernel's per-tick collision
    and room bookkeeping against the oracle's (pinned to the reference's dicts by a_traj_n8stats), from identical
    states every step; pairs 5 cm apart and drones driven into the ceiling / floor keep every counter busy.
    N = 128: the env spans a 4-wave workgroup (128-bit collision rows, the counters' LDS collectives)."""
    from parity_utils import gpu_to_oracle_a, oracle_params_a, oracle_to_gpu_a
    cfg = QuadSwarmConfig.sb_train(num_envs=E, num_agents=N, neighbor_obs_type="dist_angle", seed=4,
                                   episode_duration=3.0, neighbor_visible_num=7 if N > 8 else -1)
    env = QuadSwarmEnv(cfg)
    assert env.estats is not None
    oenv = O.OracleEnvA(oracle_params_a(cfg), seed=4)
    oenv.set_capture_radius(0.0)
    env.reset()
    oenv.reset()
    ep = cfg.ep_len
    top = float(cfg.room_dims[2])
    for e in range(E):
        oenv.envs[e].tick = ep - 120 + 8 * (e % 7)     # past the grace period, episodes end over ~15 steps
        oenv.envs[e].capture_radius = 0.0
    rng = np.random.default_rng(5)
    n_done, seen = 0, np.zeros(len(COUNT_COLS))
    for t in range(24):
        for e in range(E):
            dr = [oenv.drones[e * N + i] for i in range(N)]
            if t % 3 == 0:
                for c in range(3):
                    dr[1].pos[c] = dr[0].pos[c] + (0.05 if c == 0 else 0.0)
                dr[4].pos[2], dr[4].vel[2] = top - 0.02, 2.0
                dr[5].pos[2], dr[5].vel[2] = 0.06, -2.0
        oracle_to_gpu_a(oenv, env)
        a = rng.uniform(-1, 1, (env.I, 2)).astype(np.float32)
        _, _, done, _ = env.step(torch.from_numpy(a).cuda())
        _, _, w_done, _, _ = oenv.step(a.astype(np.float64))
        np.testing.assert_array_equal(done.cpu().numpy().astype(bool), w_done, err_msg=f"step {t}")
        est = env.estats.double().cpu().numpy()
        for e in np.flatnonzero(w_done.reshape(E, N)[:, 0]):
            got, want = est[e * N:(e + 1) * N], _oracle_rows(oenv, e)
            np.testing.assert_array_equal(got[:, COUNT_COLS], want[:, COUNT_COLS], err_msg=f"step {t} env {e}")
            for c in (S.ES_SUCCESS, S.ES_DEADLOCK, S.ES_COLRATE, S.ES_NCOLRATE, S.ES_OCOLRATE):
                np.testing.assert_allclose(got[:, c], want[:, c], rtol=1e-6, atol=1e-7, err_msg=f"{t} {e} col {c}")
            assert np.isnan(got[:, [S.ES_D1, S.ES_D3, S.ES_D5]]).all()     # np.mean of the empty list
            assert (got[:, S.ES_SCEN] == 18).all()                          # dynamic_repulsive
            seen += got[0, COUNT_COLS] != 0
            n_done += 1
        gpu_to_oracle_a(env, oenv)
    assert n_done >= E
    for k, c in enumerate(COUNT_COLS[:7]):
        if c not in (S.ES_FLOOR, S.ES_WALL):
            assert seen[k] > 0, c


def test_flavor_a_vec_env_infos():
    venv = GpuQuadVecEnv(QuadSwarmConfig.sb_train(num_envs=16, num_agents=4, seed=1, episode_duration=0.4,
                                                  initial_capture_radius=0.0))
    venv.reset()
    rng = np.random.default_rng(0)
    n_done = 0
    for t in range(12):
        _, _, dones, infos = venv.step(rng.uniform(-1, 1, (64, 2)).astype(np.float32))
        for i in np.flatnonzero(dones):
            x = infos[int(i)]["episode_extra_stats"]
            assert "dynamic_repulsive/num_collisions" in x and np.isnan(x["distance_to_goal_1s"])
            n_done += 1
    assert n_done >= 64
    venv.close()
