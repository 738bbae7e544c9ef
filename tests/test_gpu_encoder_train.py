"""The PPO update's fused attention encoders (quadswarm_amd/encoder_train.py, csrc/qs_policy_train.h) against the torch
module's autograd: forward outputs, the gradients of every encoder parameter for a random upstream gradient, and the
whole PPO loss / gradient bucket of a minibatch.

Weights: the reference-pinned fixtures' (tests/golden/policy_c3 / policy_a8: the reference's own
ActorCriticPolicyCustomSeparateWeights built by tools/gen_golden_policy.py; every tanh in its nonlinear range) and a
widened random policy for K = 1 / partial blocks.  Reference: the same module in fp64.  The fused path's products are
fp32-equivalent (three f16 products, ~7e-7 relative); torch's fp32 autograd is the yardstick: the fused gradients'
error against fp64 (max |g - g64| / max |g64| per tensor) must stay within 1e-4 and within 8x of torch fp32's own
error (+1e-6), the outputs within 5e-5 (the rollout kernels' bound)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no HIP device", allow_module_level=True)

from quadswarm_amd.encoder_train import (FusedAttentionTrain, _pow2_scales, col_scales, col_stats,  # noqa: E402
                                         colmax_scales, dw0_x3, dw_x3, tower_params)
from quadswarm_amd.ppo import PolicyConfig, SwarmActorCritic  # noqa: E402


def fixture_policy(case):
    from test_policy_reference import load_case, reference_weights
    meta, data, pc = load_case(case)
    pol = SwarmActorCritic(pc).cuda()
    pol.load_reference_state_dict(reference_weights(meta, torch.float32))
    return pol


def random_policy(K, H=256, seed=0):
    torch.manual_seed(seed)
    pol = SwarmActorCritic(PolicyConfig(self_obs_dim=18, neighbor_obs_dim=6, num_use_neighbor_obs=K, rnn_size=H,
                                        neighbor_hidden_size=H, act_dim=4)).cuda()
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


def torch_encodings(pol, obs):
    so, K = pol.cfg.self_obs_dim, pol.cfg.num_use_neighbor_obs
    nbr = obs[:, so:so + K * pol.cfg.neighbor_obs_dim].reshape(obs.shape[0], K, -1)
    return [enc.neighbor_encoder(obs[:, :so], nbr) for enc in (pol.actor_encoder, pol.critic_encoder)]


def rel_err(a, b):
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


@pytest.mark.parametrize("case,B", [("c3", 3000), ("a8", 2050), ("k1", 777), ("k6", 131)])
def test_encoder_gradients_match_torch(case, B):
    pol = fixture_policy(case) if case in ("c3", "a8") else random_policy(int(case[1:]), H=256 if case == "k6" else 128)
    obs = obs_for(pol.cfg, B, seed=3)
    H = pol.cfg.neighbor_hidden_size
    g = torch.Generator(device="cuda").manual_seed(9)
    G = [torch.randn(B, H, device="cuda", generator=g) * 1e-3 for _ in range(2)]   # dL/d out, a PPO-like scale
    params = [p for enc in (pol.actor_encoder, pol.critic_encoder) for p in tower_params(enc)]

    def grads_of(outs):
        loss = sum((o * gi).sum() for o, gi in zip(outs, G))
        return torch.autograd.grad(loss, params)

    fused = FusedAttentionTrain(pol)
    out_f = fused.encodings(obs)
    g_f = grads_of(out_f)
    out_t = torch_encodings(pol, obs)
    g_t = grads_of(out_t)
    pol64 = SwarmActorCritic(pol.cfg).cuda().double()
    pol64.load_state_dict(pol.state_dict())
    params64 = [p for enc in (pol64.actor_encoder, pol64.critic_encoder) for p in tower_params(enc)]
    out64 = torch_encodings(pol64, obs.double())
    g64 = torch.autograd.grad(sum((o * gi.double()).sum() for o, gi in zip(out64, G)), params64)
    for i in range(2):
        err = (out_f[i].double() - out64[i]).abs().max().item()
        assert err < 5e-5, (case, "out", i, err)
    names = ["e1_w", "e1_b", "e2_w", "e2_b", "v1_w", "v1_b", "v2_w", "v2_b", "a1_w", "a1_b", "a2_w", "a2_b", "a3_w",
             "a3_b"] * 2
    worst = 0.0
    for n, a, b, c in zip(names, g_f, g_t, g64):
        if n == "a3_b":   # the softmax is shift-invariant: the score bias' gradient is 0 (rounding noise in fp64 too)
            ref = max(x.abs().max().item() for x in g64)
            assert a.abs().max().item() < 1e-6 * ref and b.abs().max().item() < 1e-6 * ref, (case, n)
            continue
        ef, et = rel_err(a.double(), c), rel_err(b.double(), c)
        worst = max(worst, ef)
        assert ef < 1e-4 and ef < 8 * et + 1e-6, (case, n, ef, et)
    print(f"{case} B={B}: worst relative gradient error fused {worst:.2e}")


@pytest.mark.parametrize("case", ["c3", "a8"])
def test_ppo_loss_gradient_bucket_matches_torch(case):
    """The whole PPO minibatch step as PPOTrainer.train runs it: evaluate_actions with the fused encoders (nbr=...)
    and the self encoder's first layer and the feed_forward on the matrix cores (l0=..., ff=...) vs the torch module --
    values, log-probs and every parameter's gradient."""
    pol = fixture_policy(case)
    B = 2048
    obs = obs_for(pol.cfg, B, seed=5)
    g = torch.Generator(device="cuda").manual_seed(6)
    act = torch.rand(B, pol.cfg.act_dim, device="cuda", generator=g) * 1.6 - 0.8
    adv = torch.randn(B, device="cuda", generator=g)

    def loss_of(v, lp):
        return -(adv * torch.exp(lp - lp.detach())).mean() + 0.5 * (v.view(-1) ** 2).mean()

    fused = FusedAttentionTrain(pol)
    v_f, lp_f, _ = pol.evaluate_actions(obs, act, nbr=fused.encodings(obs), l0=fused.self_layer0,
                                        ff=fused.feed_forward)
    gf = torch.autograd.grad(loss_of(v_f, lp_f), list(pol.parameters()), allow_unused=True)
    v_t, lp_t, _ = pol.evaluate_actions(obs, act)
    gt = torch.autograd.grad(loss_of(v_t, lp_t), list(pol.parameters()), allow_unused=True)
    assert (v_f - v_t).abs().max().item() < 2e-4
    assert (lp_f - lp_t).abs().max().item() < 2e-3
    flat_f = torch.cat([(a if a is not None else torch.zeros_like(p)).flatten() for a, p in zip(gf, pol.parameters())])
    flat_t = torch.cat([(a if a is not None else torch.zeros_like(p)).flatten() for a, p in zip(gt, pol.parameters())])
    rel = ((flat_f - flat_t).norm() / flat_t.norm()).item()
    print(f"{case}: |g_fused - g_torch| / |g_torch| = {rel:.2e}")
    assert rel < 1e-4


def test_trainer_update_x3_runs_and_tracks_fp32():
    """PPOTrainer(update_precision='x3') on a device env: the same iteration from the same state as the fp32 update
    ends at nearly the same weights."""
    from quadswarm_amd import QuadSwarmConfig
    from quadswarm_amd.env import QuadSwarmEnv
    from quadswarm_amd.ppo import PPOConfig, PPOTrainer
    cfg = QuadSwarmConfig(num_envs=64, num_agents=8, seed=2)
    res, w0 = [], None
    for prec in ("fp32", "x3"):
        env = QuadSwarmEnv(cfg)
        torch.manual_seed(0)
        pol = SwarmActorCritic(PolicyConfig.for_env(cfg, rnn_size=256, neighbor_hidden_size=256)).cuda()
        tr = PPOTrainer(env, pol, PPOConfig(n_steps=16, batch_size=1024, n_epochs=1), seed=0, update_precision=prec)
        w0 = torch.cat([p.detach().flatten() for p in pol.parameters()])
        tr.collect_rollouts()
        stats = tr.train()
        assert np.isfinite(stats["loss"])
        res.append(torch.cat([p.detach().flatten() for p in pol.parameters()]))
        env.close()
    # Adam's first steps are ~lr sign(g): a gradient element near 0 may flip between the two, so the bound is on the
    # mean change and on 2.5 lr for the maximum
    d = (res[0] - res[1]).abs()
    step = (res[0] - w0).abs().mean().item()
    print(f"|w_fp32 - w_x3| after one update: max {d.max().item():.2e} mean {d.mean().item():.2e} (mean step {step:.2e})")
    assert d.max().item() <= 2.5e-4 and d.mean().item() < 0.02 * step


@pytest.mark.parametrize("H,R", [(256, 100003), (128, 777), (256, 16)])
def test_dw_x3_matches_fp64(H, R):
    """qs_attn_dw_x3: G^T A over R rows (a tail that is not a multiple of the 16-row step, column scales spanning
    2^-20 .. 2^4) against fp64 and torch's fp32 GEMM."""
    g = torch.Generator(device="cuda").manual_seed(R)
    G = torch.randn(R, H, device="cuda", generator=g) * torch.exp2(torch.linspace(-20, 4, H, device="cuda"))
    A = torch.tanh(torch.randn(R, H, device="cuda", generator=g) * 2)
    want = G.double().t().mm(A.double())
    got, sums = dw_x3(G, A, sums=True)
    assert torch.equal(got, dw_x3(G, A))
    # the column sums from the same pass (the bias gradients; ABI 15)
    G64 = G.double()
    assert ((sums.double() - G64.sum(0)).abs() / G64.abs().sum(0)).max().item() < 1e-6
    t32 = G.t().mm(A)
    # per output row n (column n of G has its own scale): relative to the row's magnitude
    scale = want.abs().amax(1, keepdim=True).clamp_min(1e-300)
    e_x3 = ((got.double() - want).abs() / scale).max().item()
    e_32 = ((t32.double() - want).abs() / scale).max().item()
    print(f"H={H} R={R}: dW relative error x3 {e_x3:.2e}, torch fp32 {e_32:.2e}")
    assert e_x3 < 1e-5 and e_x3 < 8 * e_32 + 1e-6


@pytest.mark.parametrize("H,B,K,parts", [(256, 4099, 6, None), (128, 777, 1, 5), (256, 300, 7, 4096)])
def test_colstats_matches_torch(H, B, K, parts):
    """qs_colstats: the column scales (bitwise those of col_scales), the column sums and the layer-0 weight gradient
    sum_j G_j^T [nbr_j | self_{j % B}] against torch in fp64, on ragged part splits (empty trailing parts)."""
    g = torch.Generator(device="cuda").manual_seed(B)
    so, nd = 18, 6
    R = B * K
    G = torch.randn(R, H, device="cuda", generator=g) * torch.exp2(torch.linspace(-20, 4, H, device="cuda"))
    obs = torch.randn(B, so + K * nd + 3, device="cuda", generator=g)
    gs, sums, gx = col_stats(G, obs, B, K, so, nd, nd + so, parts=parts)
    assert torch.equal(gs, col_scales(G))
    G64 = G.double()
    want_sum = G64.sum(0)
    assert ((sums.double() - want_sum).abs() / G64.abs().sum(0)).max().item() < 1e-6
    nbr = obs[:, so:so + K * nd].reshape(R, nd).double()
    slf = obs[:, :so].double().repeat(K, 1)
    X = torch.cat((nbr, slf), dim=1)
    want_x = X.t().mm(G64)                      # [nd + so, H]
    scale = (X.abs().t().mm(G64.abs())).clamp_min(1e-300)
    assert ((gx.double() - want_x).abs() / scale).max().item() < 1e-6
    # row weights: sum_r w_r G[r, :] (the score layer's weight gradient form)
    w = torch.randn(R, device="cuda", generator=g)
    _, wsum, _ = col_stats(G, row_w=w, parts=parts)
    want_w = (w.double()[:, None] * G64).sum(0)
    assert ((wsum.double() - want_w).abs() / (w.double().abs()[:, None] * G64.abs()).sum(0)).max().item() < 1e-6
    # a non-finite column gets scale 1 (and the sums carry the NaN)
    G[5, 3] = float("nan")
    gs2, sums2, _ = col_stats(G)
    assert gs2[3].item() == 1.0 and torch.isnan(sums2[3]) and torch.equal(gs2[4:], gs[4:])


def test_fused_update_falls_back_when_a_weight_leaves_the_x3_range():
    """a weight beyond the split-f16 packing range (|w| >= 255.9) makes encodings() return None (the
    caller's torch autograd path) instead of raising mid-training; back in range, the fused path returns."""
    import warnings
    pol = random_policy(6, H=128, seed=5)
    f = FusedAttentionTrain(pol)
    obs = obs_for(pol.cfg, 200)
    assert f.encodings(obs) is not None
    ne = pol.actor_encoder.neighbor_encoder
    with torch.no_grad():
        old = ne.embedding_mlp[2].weight[1, 2].item()
        ne.embedding_mlp[2].weight[1, 2] = 400.0
    with warnings.catch_warnings(record=True) as rec:
        warnings.simplefilter("always")
        assert f.encodings(obs) is None
    assert any("torch fp32" in str(r.message) for r in rec)
    with torch.no_grad():
        ne.embedding_mlp[2].weight[1, 2] = old
    out = f.encodings(obs)
    ref = torch_encodings(pol, obs)
    assert out is not None and max(rel_err(o, r) for o, r in zip(out, ref)) < 5e-5


@pytest.mark.parametrize("case,B", [("c3", 3000), ("k1", 777)])
def test_backward_column_statistics(case, B):
    """The column statistics the backward kernels form where the gradients are (ABI 15): over the blocks, colmax rows
    1..4 equal torch's max |g| of dv1_pre, da2_pre, da1_pre, de2_pre bitwise (a max is exact), row 0 (dh_pre,
    overwritten by de1_pre later) that of w_j dout[a] (1 - h^2) from the saved tensors; the per-block partials of
    sum_j dscore_j a2_j sum to torch's product."""
    pol = fixture_policy(case) if case == "c3" else random_policy(1, H=128)
    obs = obs_for(pol.cfg, B, seed=4)
    H, K = pol.cfg.neighbor_hidden_size, pol.cfg.num_use_neighbor_obs
    g = torch.Generator(device="cuda").manual_seed(11)
    G = [torch.randn(B, H, device="cuda", generator=g) * 1e-3 for _ in range(2)]
    fused = FusedAttentionTrain(pol)
    outs = fused.encodings(obs)
    params = fused.params()
    torch.autograd.grad(sum((o * gi).sum() for o, gi in zip(outs, G)), params)
    torch.cuda.synchronize()
    for i, b in enumerate(fused.runner.buf):
        cm = b["colmax"].amax(1)   # [6, n_blocks, H] -> the maxima over the blocks
        assert torch.equal(colmax_scales(b["colmax"]), _pow2_scales(cm))   # qs_colmax_reduce
        for row, name in ((1, "dv1_pre"), (2, "da2_pre"), (3, "da1_pre"), (4, "de2p")):
            assert torch.equal(cm[row], b[name].abs().amax(0)), (case, i, name)
        w, h = b["w"], b["h"]
        dh = (G[i].repeat_interleave(K, 0) * w[:, None]) * (1 - h * h)
        assert ((cm[0] - dh.abs().amax(0)).abs() <= 1e-6 * dh.abs().amax(0)).all(), (case, i, "dh_pre")
        want = b["dscore"].double()[None, :].mm(b["a2"].double())[0]
        got = b["a3w_part"].sum(0).double()
        scale = b["dscore"].double().abs()[None, :].mm(b["a2"].double().abs())[0].clamp_min(1e-300)
        assert ((got - want).abs() / scale).max().item() < 1e-6, (case, i, "a3w")


@pytest.mark.parametrize("H,B,K,parts,nd", [(256, 4099, 6, 512, 6), (128, 777, 1, 5, 6), (256, 300, 7, 4096, 6),
                                             (256, 5000, 1, 512, 0)])
def test_dw0_x3_matches_fp64(H, B, K, parts, nd):
    """qs_attn_dw0_x3: layer 0's weight gradient sum_j G_j^T [self_{j % B} | nbr_j] (the reference's column order)
    and the bias gradient against fp64, on ragged part splits (empty trailing parts) and column scales spanning
    2^-20 .. 2^4; nd = 0, K = 1: the self encoder's first layer."""
    g = torch.Generator(device="cuda").manual_seed(B + K)
    so = 18
    R = B * K
    G = torch.randn(R, H, device="cuda", generator=g) * torch.exp2(torch.linspace(-20, 4, H, device="cuda"))
    obs = torch.randn(B, so + K * nd + 3, device="cuda", generator=g) * 3
    got, sums = dw0_x3(G, obs, B, K, so, nd, parts=parts)
    nbr = obs[:, so:so + K * nd].reshape(R, nd).double()
    slf = obs[:, :so].double().repeat(K, 1)
    X = torch.cat((slf, nbr), dim=1)
    G64 = G.double()
    want = G64.t().mm(X)                          # [H, so + nd]
    scale = G64.abs().t().mm(X.abs()).clamp_min(1e-300)
    err = ((got.double() - want).abs() / scale).max().item()
    print(f"H={H} B={B} K={K}: layer-0 dW relative error {err:.2e}")
    assert err < 2e-6
    assert ((sums.double() - G64.sum(0)).abs() / G64.abs().sum(0)).max().item() < 1e-6


@pytest.mark.parametrize("M,K,N", [(1000, 512, 512), (4097, 256, 256), (64, 512, 1024)])
def test_linear_tanh_x3_matches_fp64(M, K, N):
    """qs_linear_tanh_x3 (the feed_forward's Linear + Tanh on the split-f16 matrix cores) against fp64 on tanh-range
    inputs, ragged row counts."""
    from quadswarm_amd.policy_fused import linear_tanh_x3, pack_linear_x3
    g = torch.Generator(device="cuda").manual_seed(M + K + N)
    x = torch.tanh(torch.randn(M, K, device="cuda", generator=g) * 2)
    w = torch.randn(N, K, device="cuda", generator=g) / K ** 0.5
    b = torch.randn(N, device="cuda", generator=g) * 0.1
    got = linear_tanh_x3(x, pack_linear_x3(w), b)
    want = torch.tanh(x.double().mm(w.double().t()) + b.double())
    t32 = torch.tanh(torch.nn.functional.linear(x, w, b))
    e_x3 = (got.double() - want).abs().max().item()
    e_32 = (t32.double() - want).abs().max().item()
    print(f"M={M} K={K} N={N}: max |err| x3 {e_x3:.2e}, torch fp32 {e_32:.2e}")
    assert e_x3 < 2e-6 and e_x3 < 8 * e_32 + 1e-6


@pytest.mark.parametrize("M,N", [(4097, 512), (65, 256)])
def test_linear_tanh_cat_x3_is_the_concatenated_layer(M, N):
    """qs_linear_tanh_cat_x3 on two [M, 256] parts is bitwise qs_linear_tanh_x3 on their concatenation, and the
    cat-free autograd node's gradients match the concatenated one's."""
    from quadswarm_amd.encoder_train import _FeedForwardCatFn, _FeedForwardFn
    from quadswarm_amd.policy_fused import linear_tanh_cat_x3, linear_tanh_x3, pack_linear_x3
    g = torch.Generator(device="cuda").manual_seed(M + N)
    x0 = torch.tanh(torch.randn(M, 256, device="cuda", generator=g) * 2)
    x1 = torch.tanh(torch.randn(M, 256, device="cuda", generator=g) * 2)
    w = torch.randn(N, 512, device="cuda", generator=g) / 512 ** 0.5
    b = torch.randn(N, device="cuda", generator=g) * 0.1
    pw, pwt = pack_linear_x3(w), pack_linear_x3(w.t())
    assert torch.equal(linear_tanh_cat_x3(x0, x1, pw, b), linear_tanh_x3(torch.cat((x0, x1), 1), pw, b))
    G = torch.randn(M, N, device="cuda", generator=g) * 1e-2
    a0, a1, wa, ba = (t.clone().requires_grad_() for t in (x0, x1, w, b))
    ga = torch.autograd.grad((_FeedForwardCatFn.apply(a0, a1, wa, ba, pw, pwt) * G).sum(), (a0, a1, wa, ba))
    c0, c1, wc, bc = (t.clone().requires_grad_() for t in (x0, x1, w, b))
    gc = torch.autograd.grad((_FeedForwardFn.apply(torch.cat((c0, c1), 1), wc, bc, pw, pwt) * G).sum(), (c0, c1, wc, bc))
    for u, v in zip(ga, gc):
        assert torch.equal(u, v)


@pytest.mark.parametrize("M,K,N", [(4097, 256, 256), (1000, 512, 512)])
def test_linear_bias_x3_matches_fp64(M, K, N):
    """qs_linear_bias_x3 (the score layer's mean half P = e_mean A_m^T + b_a1) against fp64 on tanh-range inputs,
    ragged row counts, relative to the row's |x| |w| products."""
    from quadswarm_amd.policy_fused import linear_bias_x3, pack_linear_x3
    g = torch.Generator(device="cuda").manual_seed(M + K + N + 1)
    x = torch.tanh(torch.randn(M, K, device="cuda", generator=g) * 2)
    w = torch.randn(N, K, device="cuda", generator=g) / K ** 0.5
    b = torch.randn(N, device="cuda", generator=g) * 0.1
    got = linear_bias_x3(x, pack_linear_x3(w), b)
    want = x.double().mm(w.double().t()) + b.double()
    scale = x.double().abs().mm(w.double().abs().t()) + b.double().abs()
    err = ((got.double() - want).abs() / scale).max().item()
    e32 = ((torch.nn.functional.linear(x, w, b).double() - want).abs() / scale).max().item()
    print(f"M={M} K={K} N={N}: relative error x3 {err:.2e}, torch fp32 {e32:.2e}")
    assert err < 2e-6


@pytest.mark.parametrize("S,M,N", [(6, 4099, 256), (7, 777, 512), (1, 64, 256), (5, 1, 256)])
def test_slab_sum_stats(S, M, N):
    """qs_slab_sum_stats (dP[b] = sum_k da1_pre[k B + b]): the sum against fp64, the row scales bitwise those of
    _pow2_scales over the result's rows, the block maxima's max bitwise torch's, a non-finite value -> +inf / scale 1."""
    from quadswarm_amd.encoder_train import _pow2_scales, slab_sum_stats
    g0 = torch.Generator(device="cuda").manual_seed(S * M + N)
    G = torch.randn(S * M, N, device="cuda", generator=g0) * torch.exp2(torch.linspace(-14, 4, S * M, device="cuda"))[:, None]
    if M > 7:
        G[(S - 1) * M + 7, 5] = float("nan")
    out = torch.full((M, N), 7.0, device="cuda")
    rs = torch.empty(M, device="cuda")
    cp = torch.empty(1, (M + 63) // 64, N, device="cuda")
    slab_sum_stats(G, S, out, rs, cp)
    want = G.double().view(S, M, N).sum(0)
    fin = torch.isfinite(want)
    scale = G.double().abs().view(S, M, N).sum(0)
    assert ((out.double() - want).abs() <= 8e-7 * scale)[fin].all()
    assert (~torch.isfinite(out) == ~fin).all()
    m = out.abs()
    m[~torch.isfinite(out)] = float("inf")
    assert torch.equal(rs, _pow2_scales(m.amax(1)))
    assert torch.equal(cp[0].amax(0), m.amax(0))


def test_dw_x3_on_column_slices():
    """qs_dw_x3_ld: the 256 x 256 blocks of a [512, 512] weight gradient from column slices of [R, 512] rows (the
    feed_forward's backward), against fp64."""
    g = torch.Generator(device="cuda").manual_seed(5)
    R = 20011
    G = torch.randn(R, 512, device="cuda", generator=g) * torch.exp2(torch.linspace(-10, 3, 512, device="cuda"))
    A = torch.tanh(torch.randn(R, 512, device="cuda", generator=g) * 2)
    want = G.double().t().mm(A.double())
    for zn in range(2):
        for zk in range(2):
            got, sums = dw_x3(G[:, 256 * zn:256 * (zn + 1)], A[:, 256 * zk:256 * (zk + 1)], sums=True)
            w = want[256 * zn:256 * (zn + 1), 256 * zk:256 * (zk + 1)]
            scale = w.abs().amax(1, keepdim=True).clamp_min(1e-300)
            assert ((got.double() - w).abs() / scale).max().item() < 1e-5, (zn, zk)
            G64 = G[:, 256 * zn:256 * (zn + 1)].double()
            assert ((sums.double() - G64.sum(0)).abs() / G64.abs().sum(0)).max().item() < 1e-6


@pytest.mark.parametrize("M,K,N", [(3001, 512, 512), (700, 256, 256)])
def test_linear_rows_x3_matches_fp64(M, K, N):
    """qs_linear_rows_x3 (the backward's dX = G W): gradient rows spanning 2^-20 .. 2^6 in magnitude, each at its
    power-of-two scale, against fp64 (relative to each row's magnitude)."""
    from quadswarm_amd.encoder_train import _pow2_scales
    from quadswarm_amd.policy_fused import linear_rows_x3, pack_linear_x3
    g = torch.Generator(device="cuda").manual_seed(M + K)
    x = torch.randn(M, K, device="cuda", generator=g) * torch.exp2(torch.linspace(-20, 6, M, device="cuda"))[:, None]
    w = torch.randn(N, K, device="cuda", generator=g) / K ** 0.5
    rs = _pow2_scales(x.abs().amax(1))
    got = linear_rows_x3(x, rs, pack_linear_x3(w), N)
    want = x.double().mm(w.double().t())
    scale = (x.double().abs().mm(w.double().abs().t())).clamp_min(1e-300)
    err = ((got.double() - want).abs() / scale).max().item()
    print(f"M={M} K={K} N={N}: dX relative error {err:.2e}")
    assert err < 2e-6


@pytest.mark.parametrize("M,N", [(4099, 512), (777, 256)])
def test_tanh_grad_stats(M, N):
    """qs_tanh_grad_stats: gp = g (1 - y^2) (to an fma's rounding), the row scales bitwise those of _pow2_scales over
    gp's rows, the per-block column maxima's max bitwise torch's, a non-finite value -> +inf / scale 1."""
    import ctypes
    from quadswarm_amd import _native as NAT
    from quadswarm_amd.encoder_train import _pow2_scales
    g0 = torch.Generator(device="cuda").manual_seed(M)
    g = torch.randn(M, N, device="cuda", generator=g0) * torch.exp2(torch.linspace(-12, 3, M, device="cuda"))[:, None]
    y = torch.tanh(torch.randn(M, N, device="cuda", generator=g0))
    g[7, 5] = float("inf")
    gp = torch.empty_like(g)
    rs = torch.empty(M, device="cuda")
    nb = (M + 63) // 64
    cp = torch.empty(nb, N, device="cuda")
    NAT.check(NAT.lib().qs_tanh_grad_stats(ctypes.c_void_p(g.data_ptr()), ctypes.c_void_p(y.data_ptr()),
                                           ctypes.c_void_p(gp.data_ptr()), ctypes.c_void_p(rs.data_ptr()),
                                           ctypes.c_void_p(cp.data_ptr()), M, N, None), "qs_tanh_grad_stats")
    want = g * (1 - y * y)
    fin = torch.isfinite(want)
    assert ((gp - want).abs() <= 2e-7 * g.abs())[fin].all()   # (1 - y^2) may be one fma apart
    m = gp.abs()
    m[~torch.isfinite(gp)] = float("inf")
    assert torch.equal(rs, _pow2_scales(m.amax(1)))
    assert torch.equal(cp.amax(0), m.amax(0))
