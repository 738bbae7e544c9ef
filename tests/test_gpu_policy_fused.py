"""The fused rollout forward (quadswarm_amd/policy_fused.py, csrc/qs_policy.h) against the torch module it
replaces: QuadNeighborhoodEncoderAttention (swarm_rl/models/quad_multi_model.py:44-101, ppo.py
NeighborAttention with the reference's j % B row pairing) and the whole SwarmActorCritic forward.

Tolerance: both sides are fp32; they differ only in the summation order of the 256-term (128-term) dot
products (matrix cores vs hipBLASLt) and of the K-row sums, ~1e-6 relative per layer; the encoder outputs
are tanh-bounded averages, so 5e-5 absolute is far above that and far below any real defect (a wrong
row pairing, weight layout or softmax row moves outputs by ~1e-1)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no HIP device", allow_module_level=True)

from quadswarm_amd import QuadSwarmConfig  # noqa: E402
from quadswarm_amd.env import QuadSwarmEnv  # noqa: E402
from quadswarm_amd.policy_fused import FusedRolloutPolicy, supports  # noqa: E402
from quadswarm_amd.ppo import PolicyConfig, PPOConfig, PPOTrainer, SwarmActorCritic  # noqa: E402

ATOL = 5e-5

CASES = {
    # C3's policy (bench e2e_settings flavor B): obs 54 = 18 self + 6 x 6 neighbours, H 256
    "c3": dict(self_obs_dim=18, neighbor_obs_dim=6, num_use_neighbor_obs=6, rnn_size=256, neighbor_hidden_size=256),
    # sb_train's (flavor A): 7 self + 7 x 3, H 128, 6 x 128 core
    "a8": dict(self_obs_dim=7, neighbor_obs_dim=3, num_use_neighbor_obs=7, rnn_size=128, neighbor_hidden_size=128,
               rnn_type="full", rnn_num_layers=6),
    "k1": dict(self_obs_dim=18, neighbor_obs_dim=6, num_use_neighbor_obs=1, rnn_size=256, neighbor_hidden_size=256),
    "k64": dict(self_obs_dim=18, neighbor_obs_dim=6, num_use_neighbor_obs=64, rnn_size=128, neighbor_hidden_size=128),
    "k31obst": dict(self_obs_dim=18, neighbor_obs_dim=6, num_use_neighbor_obs=31, obstacle_obs_dim=9, rnn_size=256,
                    neighbor_hidden_size=256, obst_hidden_size=256),
}


def make_policy(case, seed=0):
    torch.manual_seed(seed)
    pc = PolicyConfig(act_dim=4, **CASES[case])
    pol = SwarmActorCritic(pc).cuda().eval()
    # the default Linear init keeps every tanh in its linear range; widen the weights so that the kernels'
    # nonlinear regime and the softmax are exercised too
    with torch.no_grad():
        for enc in (pol.actor_encoder, pol.critic_encoder):
            for m in enc.neighbor_encoder.modules():
                if isinstance(m, torch.nn.Linear):
                    m.weight.mul_(3.0)
                    m.bias.uniform_(-0.5, 0.5)
    return pol


def obs_for(pc, B, seed=1):
    g = torch.Generator(device="cuda").manual_seed(seed)
    od = pc.self_obs_dim + pc.neighbor_obs_dim * pc.num_use_neighbor_obs + pc.obstacle_obs_dim
    return torch.randn(B, od, device="cuda", generator=g) * 2.0


PRECISIONS = ["fp32", "x3"]


@pytest.mark.parametrize("precision", PRECISIONS)
@pytest.mark.parametrize("case,B", [("c3", 4096), ("c3", 1003), ("a8", 2050), ("k1", 777), ("k64", 130),
                                    ("k31obst", 257)])
def test_neighbor_encodings_match_torch(case, B, precision):
    """x3 (split f16 products, csrc/qs_policy_x3.h) is held to the same bound as the fp32 matrix cores."""
    pol = make_policy(case)
    assert supports(pol)
    fp = FusedRolloutPolicy(pol, precision=precision)
    obs = obs_for(pol.cfg, B)
    got = fp.neighbor_encodings(obs).clone()
    so, K = pol.cfg.self_obs_dim, pol.cfg.num_use_neighbor_obs
    nbr = obs[:, so:so + K * pol.cfg.neighbor_obs_dim].reshape(B, K, -1)
    with torch.no_grad():
        for i, enc in enumerate((pol.actor_encoder, pol.critic_encoder)):
            want = enc.neighbor_encoder(obs[:, :so], nbr)
            err = (got[i] - want).abs().max().item()
            assert err < ATOL, (case, B, i, err)
            assert want.abs().max().item() > 0.05   # a non-trivial output


@pytest.mark.parametrize("precision", PRECISIONS)
@pytest.mark.parametrize("case", ["c3", "a8", "k31obst"])
def test_fused_forward_matches_policy(case, precision):
    pol = make_policy(case, seed=3)
    fp = FusedRolloutPolicy(pol, precision=precision)
    obs = obs_for(pol.cfg, 3000, seed=4)
    a_f, v_f, lp_f = fp(obs, deterministic=True)
    with torch.no_grad():
        a_t, v_t, lp_t = pol(obs, deterministic=True)
    assert (a_f - a_t).abs().max().item() < 2e-4
    assert (v_f - v_t).abs().max().item() < 2e-4
    assert (fp.predict_values(obs) - v_t).abs().max().item() < 2e-4
    # weights changed in place (an optimizer step): refresh() picks them up
    with torch.no_grad():
        for p in pol.parameters():
            p.add_(0.01 * torch.randn_like(p))
        a_t2, v_t2, _ = pol(obs, deterministic=True)
    fp.refresh()
    a_f2, v_f2, _ = fp(obs, deterministic=True)
    assert (a_f2 - a_t2).abs().max().item() < 2e-4 and (v_f2 - v_t2).abs().max().item() < 2e-4


def test_trainer_rollout_uses_fused_forward():
    cfg = QuadSwarmConfig(num_envs=64, num_agents=8)
    env = QuadSwarmEnv(cfg)
    torch.manual_seed(0)
    pol = SwarmActorCritic(PolicyConfig.for_env(cfg, rnn_size=256, neighbor_hidden_size=256)).cuda()
    tr = PPOTrainer(env, pol, PPOConfig(n_steps=16, batch_size=256, n_epochs=1), seed=0)
    assert tr.fused is not None
    calls = []
    orig = tr.fused.neighbor_encodings
    tr.fused.neighbor_encodings = lambda obs: calls.append(1) or orig(obs)
    tr.collect_rollouts()
    assert len(calls) == 16 + 1      # every step + the last values
    assert torch.isfinite(tr.storage.values).all() and torch.isfinite(tr.storage.log_probs).all()
    # the stored values are the torch module's values of the stored obs (same weights during the rollout)
    pol.eval()
    with torch.no_grad():
        for t in (0, 7, 15):
            v = pol.predict_values(tr.storage.obs[t]).view(-1)
            assert (v - tr.storage.values[t]).abs().max().item() < 2e-4
    stats = tr.train()
    assert np.isfinite(stats["loss"])


@pytest.mark.parametrize("precision", PRECISIONS)
@pytest.mark.parametrize("case", ["c3", "a8"])
def test_fused_rollout_log_probs_match_evaluate_actions(case, precision):
    """The rollout stores the fused path's log-probs; PPO's first epoch divides the torch module's
    evaluate_actions log-probs of the same (obs, actions) by them.  At a small std (exp(log_std) = 0.05, a late
    training stage) the log-prob amplifies a mean difference by z / std, so this bounds the ratio PPO sees
    before any update: |exp(lp_torch - lp_fused) - 1| (the clip range is 0.2)."""
    import math
    pol = make_policy(case, seed=5)
    with torch.no_grad():
        pol.log_std.fill_(math.log(0.05))
    fp = FusedRolloutPolicy(pol, precision=precision)
    obs = obs_for(pol.cfg, 4096, seed=6)
    torch.manual_seed(7)
    a_f, v_f, lp_f = fp(obs)
    with torch.no_grad():
        v_t, lp_t, _ = pol.evaluate_actions(obs, a_f)
    dev = (torch.exp(lp_t - lp_f) - 1).abs()
    print(f"{case} {precision}: ratio deviation max {dev.max().item():.3e} mean {dev.mean().item():.3e}")
    assert dev.max().item() < 2e-3 and dev.mean().item() < 2e-4
    assert (v_t.view(-1) - v_f.view(-1)).abs().max().item() < 2e-4


@pytest.mark.parametrize("precision", PRECISIONS)
@pytest.mark.parametrize("case", ["c3", "a8", "c4"])
def test_fused_policy_matches_reference_fixture(case, precision):
    """The fused rollout forward against the reference's own policy module: tests/golden/policy_<case> (written by
    tools/gen_golden_policy.py from swarm_rl/models/ActorCriticPolicyCustom.py + quad_multi_model.py), weights
    loaded under the reference's parameter names."""
    from test_policy_reference import load_case, reference_weights
    meta, data, pc = load_case(case)
    pol = SwarmActorCritic(pc).cuda().eval()
    pol.load_reference_state_dict(reference_weights(meta, torch.float32))
    assert supports(pol)
    fp = FusedRolloutPolicy(pol, precision=precision)
    obs = torch.from_numpy(data["obs"].astype(np.float32)).cuda()
    nbr = fp.neighbor_encodings(obs)
    for i, tw in enumerate(("actor", "critic")):
        err = np.abs(nbr[i].cpu().numpy() - data[f"{tw}_nbr64"]).max()
        print(f"{case} {precision} {tw}: max |encoder - reference fp64| {err:.2e}")
        assert err < ATOL, (case, tw, err)
    a, v, lp = fp(obs, deterministic=True)
    np.testing.assert_allclose(a.cpu().numpy(), data["det_actions32"], rtol=0, atol=2e-4)
    np.testing.assert_allclose(v.cpu().numpy(), data["det_values32"], rtol=1e-4, atol=2e-4)
    np.testing.assert_allclose(lp.cpu().numpy(), data["det_log_prob32"], rtol=1e-4, atol=2e-3)
    np.testing.assert_allclose(fp.predict_values(obs).cpu().numpy(), data["pv_values32"], rtol=1e-4, atol=2e-4)
