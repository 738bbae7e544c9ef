"""BASELINE.json configs 1 and 2 at the sizes it names (C3 / C4 / C5 have their own full-size tests in
test_gpu_parity.py, test_gpu_parity_obst.py and test_gpu_c5.py).

C1 -- "single_quad scenario, 1 env ... via swarm_rl.sb_train + SB3 PPO": sb_train builds its vec env from a
QuadrotorEnvConfig (swarm_rl/sb_train.py:50-51, global_cfg.py:7-190) and trains PPO on it (:54-68).  Here the
config is the reference dataclass's own field set and defaults (tests/golden/quadrotor_env_config.json) with one
env of one drone, built through make_vec_env, stepped through the VecEnv surface, and trained for one PPO
iteration by the GPU trainer.  The SB3 side is parity-unpinned (SB3 is not importable here): the
iteration is checked for its bookkeeping and finiteness, not against SB3's numbers.

C2 -- "single_quad x 16384 parallel envs on 1 MI355X": flavor B, one drone per env, obs 18 (runs/single_quad/
baseline.py); a whole episode at full size (the tick-1501 boundary, finiteness, the obs clip box, the spawn
box), and the oracle at full size: the reset and 5 free-running steps from it (identical Philox draws).
"""
import json
import os
import types

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no HIP device", allow_module_level=True)

import oracle as O  # noqa: E402
from conftest import GOLDEN  # noqa: E402
from parity_utils import oracle_params  # noqa: E402
from quadswarm_amd import QuadSwarmConfig  # noqa: E402
from quadswarm_amd.env import QuadSwarmEnv  # noqa: E402
from quadswarm_amd.ppo import PolicyConfig, PPOConfig, PPOTrainer, SwarmActorCritic  # noqa: E402
from quadswarm_amd.vec_env import make_vec_env  # noqa: E402


def reference_cfg(**over):
    """A QuadrotorEnvConfig stand-in carrying the reference dataclass's field set and defaults."""
    d = json.load(open(os.path.join(GOLDEN, "quadrotor_env_config.json")))
    d.update(over)
    return types.SimpleNamespace(**d)


@pytest.mark.parametrize("flavor", ["A", "B"])
def test_c1_single_env_single_drone_through_make_vec_env_and_ppo(flavor):
    if flavor == "A":   # what sb_train builds (dim_mode 2D_horizontal): the PID pre-controller env
        ref = reference_cfg(num_envs=1, num_agents=1, seed=5)
    else:               # runs/single_quad/baseline.py: flavor B, xyz_vxyz_R_omega, no neighbours
        ref = reference_cfg(num_envs=1, num_agents=1, seed=5, dim_mode="3D", obs_repr="xyz_vxyz_R_omega",
                            neighbor_obs_type="none", quads_mode="static_same_goal", room_dims=[10, 10, 10],
                            episode_duration=15.0)
    venv = make_vec_env(ref)
    cfg = venv.cfg
    assert cfg.flavor == flavor and cfg.num_envs == 1 and cfg.num_agents == 1 and venv.num_envs == 1
    obs = venv.reset()
    assert obs.shape == (1, cfg.obs_dim) == (1, venv.observation_space.shape[0])
    assert venv.reset_infos == (({"success": False},) if flavor == "A" else ({},))
    rng = np.random.default_rng(0)
    for _ in range(40):
        obs, rew, dones, infos = venv.step(rng.uniform(-1, 1, (1, cfg.act_dim)).astype(np.float32))
        assert obs.shape == (1, cfg.obs_dim) and rew.shape == (1,) and dones.shape == (1,) and len(infos) == 1
        assert np.isfinite(obs).all() and np.isfinite(rew).all()
        assert ("goal_dist" in infos[0]) if flavor == "A" else ("rewards" in infos[0])
    # one PPO iteration of sb_train's settings (n_steps 512, 10 epochs, batch 1024 -> one minibatch of 512)
    torch.manual_seed(0)
    pc = PolicyConfig.sb_train(cfg) if flavor == "A" else PolicyConfig.for_env(cfg, rnn_size=64)
    pol = SwarmActorCritic(pc).cuda()
    tr = PPOTrainer(venv.env, pol, PPOConfig(n_steps=512, batch_size=1024, n_epochs=10), seed=1)
    w0 = [p.detach().clone() for p in pol.parameters()]
    stats = tr.learn_iteration()
    assert tr.num_timesteps == 512
    assert stats["n_updates"] == 10
    assert all(np.isfinite(v) for k, v in stats.items() if k != "explained_variance")
    assert torch.isfinite(tr.storage.obs).all() and torch.isfinite(tr.storage.advantages).all()
    assert any(not torch.equal(p, q) for p, q in zip(pol.parameters(), w0))
    venv.close()


def test_c2_full_size_episode():
    """16384 single drones: the whole 1500-tick episode and the fused auto-reset of every env at tick 1501."""
    cfg = QuadSwarmConfig(num_envs=16384, num_agents=1, neighbor_obs_type="none")
    assert cfg.obs_dim == 18
    env = QuadSwarmEnv(cfg)
    obs = env.reset()
    assert obs.shape == (16384, 18)
    a = torch.empty(16384, 4, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(0)
    n_done_steps = 0
    room = torch.tensor([10.0, 10.0, 10.0], device="cuda")
    for t in range(cfg.ep_len + 3):
        a.uniform_(-1, 1, generator=g)
        obs, rew, done, term = env.step(a)
        if done.any():
            assert bool(done.all())          # synchronised episodes end together
            assert t == cfg.ep_len           # tick > ep_len: the 1501st step
            assert torch.isfinite(term).all()
            n_done_steps += 1
            f = env.drone_fields()          # static_same_goal spawn box around the goal (0, 0, 2), at rest
            pos = f["pos"]
            assert (pos[:, 0:2].abs() <= 2.0 + 1e-5).all() and (pos[:, 2] >= 0.75 - 1e-6).all()
            assert (pos[:, 2] <= 4.0 + 1e-5).all() and (f["vel"] == 0).all() and (f["omega"] == 0).all()
            assert (env.env_state[0] == 0).all()
        if t % 100 == 0 or done.any():
            assert torch.isfinite(obs).all() and torch.isfinite(rew).all()
            assert (obs[:, 0:3].abs() <= room + 0.1).all()           # pos - goal inside the room (+ noise)
            assert (obs[:, 6:15].abs() <= 1.0 + 1e-3).all()           # rotation entries
            assert (obs[:, 15:18].abs() <= 40.0 + 1e-2).all()         # omega clip (quadrotor_dynamics.py:567)
            # every cost term is >= 0 except the orientation term -R[2][2] >= -1 (quadrotor_single.py:45-51)
            assert (rew <= cfg.dt * 1.0 + 1e-6).all()
    assert n_done_steps == 1
    assert env.counters() == {"nonfinite_obs": 0, "nonfinite_rew": 0, "nonfinite_state": 0}


def test_c2_full_size_against_oracle():
    """The full 16384-env shard against the oracle: reset obs row for row, then 5 free-running steps from that
    reset with the same actions (identical Philox draws) within the free-running tolerance."""
    cfg = QuadSwarmConfig(num_envs=16384, num_agents=1, neighbor_obs_type="none", seed=9)
    env = QuadSwarmEnv(cfg)
    oenv = O.OracleEnv(oracle_params(cfg), seed=9)
    np.testing.assert_allclose(env.reset().double().cpu().numpy(), oenv.reset(), atol=2e-5, rtol=1e-5)
    rng = np.random.default_rng(1)
    for t in range(5):
        a = rng.uniform(-1, 1, (16384, 4)).astype(np.float32)
        obs, rew, done, _ = env.step(torch.from_numpy(a).cuda())
        w_obs, w_rew, w_done, _ = oenv.step(a.astype(np.float64), nthreads=8)
        np.testing.assert_array_equal(done.cpu().numpy().astype(bool), w_done)
        np.testing.assert_allclose(obs.double().cpu().numpy(), w_obs, atol=2e-3, err_msg=f"obs step {t}")
        np.testing.assert_allclose(rew.double().cpu().numpy(), w_rew, atol=2e-4, err_msg=f"rew step {t}")
