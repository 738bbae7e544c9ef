"""CPU tests of the GPU-PPO path's host logic: the policy mirror of
ActorCriticPolicyCustomSeparateWeights / QuadMultiEncoder, the squashed-Gaussian log-prob, the GAE
restatement (known answers), the flat gradient bucket, and one PPO iteration on a CPU stand-in env
(with the oracle GAE injected -- the product default is the HIP kernel, which has no CPU path).
"""
import numpy as np
import pytest
import torch

import ppo_oracle as PO
from quadswarm_amd import QuadSwarmConfig
from quadswarm_amd import _native as NAT
from quadswarm_amd.ppo import (FlatGradBucket, NeighborAttention, PolicyConfig, PPOConfig, PPOTrainer,
                               SwarmActorCritic, gae, squashed_log_prob)


# ---------------------------------------------------------------- GAE known answers
def test_gae_known_answer_no_dones():
    # T=3, one column, gamma=0.5, lambda=1: A_t = sum_k (0.5)^k delta_{t+k}, delta_t = r_t + 0.5 V_{t+1} - V_t
    r, v = np.array([[1.0], [2.0], [3.0]]), np.array([[0.5], [1.0], [2.0]])
    adv, ret = PO.gae_np(r, v, np.zeros((3, 1)), np.array([4.0]), np.array([0.0]), gamma=0.5, gae_lambda=1.0)
    d = [1 + 0.5 * 1.0 - 0.5, 2 + 0.5 * 2.0 - 1.0, 3 + 0.5 * 4.0 - 2.0]
    want = [d[0] + 0.5 * d[1] + 0.25 * d[2], d[1] + 0.5 * d[2], d[2]]
    np.testing.assert_allclose(adv[:, 0], want, rtol=1e-15)
    np.testing.assert_allclose(ret[:, 0], np.array(want) + v[:, 0], rtol=1e-15)


def test_gae_episode_boundaries_cut_bootstrap():
    rng = np.random.default_rng(0)
    T, I = 6, 4
    r, v = rng.normal(size=(T, I)), rng.normal(size=(T, I))
    starts = np.zeros((T, I))
    starts[3, 1] = 1           # column 1: an episode ends after step 2
    adv, _ = PO.gae_np(r, v, starts, np.zeros(I), np.ones(I), 0.99, 0.95)
    # last step: done -> no bootstrap
    np.testing.assert_allclose(adv[-1], r[-1] - v[-1], rtol=1e-14)
    # column 1 before the boundary only sees steps 0..2
    a1, _ = PO.gae_np(r[:3, 1:2], v[:3, 1:2], starts[:3, 1:2], np.zeros(1), np.ones(1), 0.99, 0.95)
    np.testing.assert_allclose(adv[:3, 1], a1[:, 0], rtol=1e-14)


def test_gae_product_path_refuses_cpu_tensors():
    z = torch.zeros(2, 3)
    with pytest.raises(NAT.QuadSwarmError):
        gae(z, z, z.to(torch.uint8), z[0], z[0].to(torch.uint8))


# ---------------------------------------------------------------- distribution
def test_squashed_log_prob_matches_restatement():
    torch.manual_seed(0)
    mean = torch.randn(64, 2, dtype=torch.float64)
    log_std = torch.tensor([0.3, -0.7], dtype=torch.float64)
    a = torch.tanh(mean + torch.randn_like(mean) * log_std.exp())
    a[0, 0] = 1.0                    # saturated action: clamp path
    got = squashed_log_prob(mean, log_std, a).numpy()
    want = PO.squashed_logp_np(mean.numpy(), log_std.numpy(), a.numpy())
    np.testing.assert_allclose(got, want, rtol=1e-9, atol=1e-9)


# ---------------------------------------------------------------- policy
def sb_cfg(**kw):
    env_cfg = QuadSwarmConfig.sb_train(num_envs=4, num_agents=8)
    return env_cfg, PolicyConfig.sb_train(env_cfg, **kw)


def test_policy_dims_and_param_count():
    env_cfg, pc = sb_cfg()
    assert (pc.self_obs_dim, pc.neighbor_obs_dim, pc.num_use_neighbor_obs, pc.act_dim) == (7, 3, 7, 2)
    pol = SwarmActorCritic(pc)
    obs = torch.randn(5, env_cfg.obs_dim)
    a, v, lp = pol(obs)
    assert a.shape == (5, 2) and v.shape == (5, 1) and lp.shape == (5,)
    assert a.abs().max() <= 1
    # hand count (per tower): self 7*128+128 + 128*128+128; attention embed (10*128+128)+(128^2+128),
    # value 2*(128^2+128), attention 256*128+128 + 128^2+128 + 128+1; ff 256*256+256; core 256*128+128 + 5*(128^2+128)
    H = 128
    lin = lambda i, o: i * o + o  # noqa: E731
    tower = (lin(7, H) + lin(H, H) + lin(10, H) + lin(H, H) + 2 * lin(H, H) + lin(2 * H, H) + lin(H, H) + lin(H, 1)
             + lin(2 * H, 2 * H) + lin(2 * H, H) + 5 * lin(H, H))
    want = 2 * tower + lin(H, 2) + 2 + lin(H, 1)
    assert sum(p.numel() for p in pol.parameters()) == want


def test_attention_row_pairing_quirk():
    """Row j of the attention input pairs neighbour (j // K, j % K) with agent j % B's self obs and the
    mean embedding of agent j % B (Tensor.repeat tiling, quad_multi_model.py:84-91)."""
    _, pc = sb_cfg()
    torch.manual_seed(1)
    att = NeighborAttention(pc).double()
    B, K = 3, pc.num_use_neighbor_obs
    so = torch.randn(B, pc.self_obs_dim, dtype=torch.float64)
    nb = torch.randn(B, K, pc.neighbor_obs_dim, dtype=torch.float64)
    got = att(so, nb)
    rows = nb.reshape(B * K, -1)
    e = torch.stack([att.embedding_mlp(torch.cat((so[j % B], rows[j]))) for j in range(B * K)])
    h = att.neighbor_value_mlp(e)
    em = e.view(B, K, -1).mean(1)
    s = torch.stack([att.attention_mlp(torch.cat((e[j], em[j % B]))) for j in range(B * K)]).view(B, K)
    w = torch.softmax(s, 1).view(B * K, 1)
    want = (w * h).view(B, K, -1).sum(1)
    torch.testing.assert_close(got, want, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("B", [1, 5])
def test_attention_split_weights_equal_concatenated(B):
    """The split-weight evaluation (per-agent halves of the two concatenating layers computed once per
    agent) is the reference's concatenated forward: same outputs and same parameter gradients at fp64."""
    _, pc = sb_cfg()
    torch.manual_seed(2)
    att = NeighborAttention(pc).double()
    K = pc.num_use_neighbor_obs
    so = torch.randn(B, pc.self_obs_dim, dtype=torch.float64)
    nb = torch.randn(B, K, pc.neighbor_obs_dim, dtype=torch.float64)
    outs, grads = [], []
    for split in (False, True):
        att.split = split
        att.zero_grad()
        y = att(so, nb)
        (y * torch.linspace(-1, 1, y.numel(), dtype=torch.float64).view_as(y)).sum().backward()
        outs.append(y.detach())
        grads.append(torch.cat([p.grad.flatten() for p in att.parameters()]))
    torch.testing.assert_close(outs[1], outs[0], rtol=1e-12, atol=1e-12)
    torch.testing.assert_close(grads[1], grads[0], rtol=1e-10, atol=1e-12)


def test_initialisation_follows_reference():
    """Only action_net / value_net are xavier-initialised (type(layer) == nn.Linear check); log_std = 0."""
    _, pc = sb_cfg(policy_init_gain=1.0)
    torch.manual_seed(0)
    pol = SwarmActorCritic(pc)
    assert torch.all(pol.log_std == 0)
    bound = np.sqrt(6.0 / (128 + 1))            # xavier_uniform bound for value_net (fan 128 -> 1)
    assert pol.value_net.weight.abs().max() <= bound
    # default nn.Linear init (kaiming_uniform a=sqrt 5) on the encoders: bound 1/sqrt(fan_in)
    w = pol.actor_encoder.self_encoder[0].weight
    assert w.abs().max() <= 1 / np.sqrt(7) + 1e-7


@pytest.mark.parametrize("enc", ["mean_embed", "mlp", "no_encoder"])
def test_other_neighbor_encoders_and_obstacles(enc):
    env_cfg = QuadSwarmConfig.c4(num_envs=2, num_agents=8)
    pc = PolicyConfig.for_env(env_cfg, neighbor_encoder_type=enc, rnn_size=32, neighbor_hidden_size=16,
                              obst_hidden_size=8, act_dim=4)
    assert pc.obstacle_obs_dim == 9 and pc.num_use_neighbor_obs == 2
    pol = SwarmActorCritic(pc)
    a, v, lp = pol(torch.randn(6, env_cfg.obs_dim))
    assert a.shape == (6, 4) and torch.isfinite(lp).all()


# ---------------------------------------------------------------- gradient bucket
def test_flat_bucket_views_and_clip():
    _, pc = sb_cfg(rnn_num_layers=2)
    torch.manual_seed(0)
    pol = SwarmActorCritic(pc)
    ref = SwarmActorCritic(pc)
    ref.load_state_dict(pol.state_dict())
    bucket = FlatGradBucket(pol.parameters())
    obs = torch.randn(16, 28)
    act = torch.rand(16, 2) * 1.8 - 0.9
    for m in (pol, ref):
        v, lp, _ = m.evaluate_actions(obs, act)
        (v.square().mean() - lp.mean()).backward()
    assert bucket.check_bound()
    for p, q in zip(pol.parameters(), ref.parameters()):
        torch.testing.assert_close(p.grad, q.grad)
    n1 = bucket.clip_norm_(0.5)
    n2 = torch.nn.utils.clip_grad_norm_(list(ref.parameters()), 0.5)
    torch.testing.assert_close(n1, n2)
    for p, q in zip(pol.parameters(), ref.parameters()):
        torch.testing.assert_close(p.grad, q.grad)


# ---------------------------------------------------------------- one PPO iteration on a CPU stand-in env
class ToyEnv:
    """Point-mass stand-in (CPU torch) with the QuadSwarmEnv step surface: obs [I, od], reward = -|x|,
    episodes of 5 steps."""

    def __init__(self, I=32, od=28, act_dim=2, seed=0):
        self.I, self.obs_dim, self.act_dim = I, od, act_dim
        self.g = torch.Generator().manual_seed(seed)
        self.t = 0
        self.x = torch.zeros(I, od)

    def reset(self):
        self.x = torch.randn(self.I, self.obs_dim, generator=self.g)
        self.t = 0
        return self.x

    def step(self, a):
        self.x = self.x.clone()
        self.x[:, :2] += 0.1 * a
        rew = -self.x[:, :2].norm(dim=1)
        self.t += 1
        done = torch.full((self.I,), int(self.t % 5 == 0), dtype=torch.uint8)
        if self.t % 5 == 0:
            self.x = torch.randn(self.I, self.obs_dim, generator=self.g)
        return self.x, rew, done, self.x


def gae_oracle_torch(r, v, s, lv, ld, gamma, lam, adv, ret):
    a, rt = PO.gae_np(r.numpy(), v.numpy(), s.numpy(), lv.numpy(), ld.numpy(), gamma, lam)
    adv.copy_(torch.from_numpy(a))
    ret.copy_(torch.from_numpy(rt))


def test_ppo_iteration_on_cpu_standin():
    torch.manual_seed(0)
    _, pc = sb_cfg(rnn_num_layers=2, rnn_size=32, neighbor_hidden_size=16)
    pol = SwarmActorCritic(pc)
    env = ToyEnv()
    tr = PPOTrainer(env, pol, PPOConfig(n_steps=10, batch_size=64, n_epochs=2), device="cpu",
                    gae_fn=gae_oracle_torch)
    w0 = [p.detach().clone() for p in pol.parameters()]
    stats = tr.learn_iteration()
    assert tr.num_timesteps == 10 * 32
    assert stats["n_updates"] == 2 * 5
    assert all(np.isfinite(v) for v in stats.values())
    # first-step episode_starts are ones (SB3 after reset), then the stand-in's every-5-step dones
    st = tr.storage
    assert st.episode_starts[0].all() and st.episode_starts[5].all() and not st.episode_starts[1].any()
    a, _ = PO.gae_np(st.rewards.numpy(), st.values.numpy(), st.episode_starts.numpy(), tr.last_values.numpy(),
                     tr.last_done.numpy())
    np.testing.assert_allclose(st.advantages.numpy(), a, rtol=1e-5, atol=1e-5)
    assert any(not torch.equal(p, q) for p, q in zip(pol.parameters(), w0))
    assert tr.bucket.check_bound()
