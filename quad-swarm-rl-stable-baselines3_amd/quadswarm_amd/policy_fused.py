"""Fused rollout forward of the attention policy: the no-grad evaluation that SB3's
collect_rollouts makes of ActorCriticPolicyCustomSeparateWeights (swarm_rl/models/ActorCriticPolicyCustom.py:
515-536) once per step, with both towers' attention neighbour encoders (QuadNeighborhoodEncoderAttention,
swarm_rl/models/quad_multi_model.py:44-101) run by the HIP kernels of csrc/qs_policy.h through the C ABI
(qs_attn_embed / qs_attn_pool) instead of ~20 torch GEMM + tanh launches per tower.

Per step, for the actor and the critic tower at once (one launch per stage):
  HIP     e1 (self and neighbour halves of layer 0), e2 rows, mean_K(e2)   (qs_attn_embed)
  HIP     P = mean_K(e2) W_a1[:, H:]^T + b_a1 (x3, H 256; else torch)   [B, H]
  HIP     value path, attention path, softmax over K, pooled out    (qs_attn_pool)
  torch   self encoder, feed_forward, core, decoder, heads          (small per-agent GEMMs)
The result is the same function as the torch module (fp32 throughout; only the summation order of the
GEMMs differs: tests/test_gpu_policy_fused.py bounds it).  Training (the PPO update with autograd) keeps
the torch module.
"""
import ctypes

import torch

from . import _native as NAT


def pack_mfma_weight(w):
    """[N, Kd] fp32 weight -> the matrix-core operand layout of qs_attn_tower (quadswarm.h):
    packed[ct][g][l][u] = W[32 ct + (l & 31)][(l >> 5) Kd/2 + 4 g + u]."""
    n, kd = w.shape
    assert n % 32 == 0 and kd % 8 == 0, (n, kd)
    return w.detach().float().contiguous().view(n // 32, 32, 2, kd // 8, 4).permute(0, 3, 2, 1, 4).contiguous()


X3_SW = 256.0   # weight scale of the split-f16 packing (csrc/qs_policy_x3.h X3_SW)
X3_SIN = 16.0   # raw-observation scale of the x3 layer-0 inputs (csrc/qs_policy_x3.h X3_SIN)
F16_MAX = 65504.0


def pack_mfma_weight_x3(w):
    """[N, Kd] fp32 weight -> the split-f16 operand layout of qs_attn_embed_x3 / qs_attn_pool_x3 (quadswarm.h):
    packed[ct][s][l] = 8 halves of hi(256 W[32 ct + (l & 31)][16 s + 8 (l >> 5) + j]), then the 8 lo halves,
    hi = f16(256 w), lo = f16(256 w - hi).  Returned as an int16 tensor [N/32, Kd/16, 64, 2, 8].
    Raises ValueError for a weight with |256 w| beyond the f16 range (it would pack as +-inf)."""
    n, kd = w.shape
    assert n % 32 == 0 and kd % 16 == 0, (n, kd)
    ws = w.detach().float() * X3_SW
    if not bool(ws.abs().amax() < F16_MAX):   # NaN fails too
        raise ValueError(f"x3 packing: max |w| = {float(w.detach().abs().amax()):.4g} is outside the split-f16 range "
                         f"(< {F16_MAX / X3_SW:.4g})")
    hi = ws.half()
    lo = (ws - hi.float()).half()

    def lay(x):   # [n, kd] -> [ct, s, h, r, j] -> [ct, s, l = 32 h + r, j]
        return x.contiguous().view(n // 32, 32, kd // 16, 2, 8).permute(0, 2, 3, 1, 4).reshape(n // 32, kd // 16, 64, 8)
    return torch.stack((lay(hi), lay(lo)), dim=3).contiguous().view(torch.int16)


def pack_mfma_weights_x3(ws):
    """pack_mfma_weight_x3 of several weights at once: those of one shape packed as one batch, the range of all of
    them checked with one host read (the update packs 22 matrices per minibatch).  Same layout, same ValueError."""
    groups = {}
    for i, w in enumerate(ws):
        groups.setdefault(tuple(w.shape), []).append(i)
    out = [None] * len(ws)
    scaled = {}
    peak = []
    for shape, idx in groups.items():
        n, kd = shape
        assert n % 32 == 0 and kd % 16 == 0, shape
        x = torch.stack([ws[i].detach().float() for i in idx]) * X3_SW
        scaled[shape] = x
        peak.append(x.abs().amax())
    if not bool(torch.stack(peak).amax() < F16_MAX):   # NaN fails too
        m = max(float(w.detach().abs().amax()) for w in ws)
        raise ValueError(f"x3 packing: max |w| = {m:.4g} is outside the split-f16 range (< {F16_MAX / X3_SW:.4g})")
    for shape, idx in groups.items():
        n, kd = shape
        x = scaled[shape]
        hi = x.half()
        lo = (x - hi.float()).half()
        g = len(idx)

        def lay(t):   # [g, n, kd] -> [g, ct, s, h, r, j] -> [g, ct, s, l = 32 h + r, j]
            return t.view(g, n // 32, 32, kd // 16, 2, 8).permute(0, 1, 3, 4, 2, 5).reshape(g, n // 32, kd // 16, 64, 8)
        packed = torch.stack((lay(hi), lay(lo)), dim=4).contiguous().view(torch.int16)
        for j, i in enumerate(idx):
            out[i] = packed[j]
    return out


def pack_linear_x3(w):
    """[N, K] fp32 weight (N a multiple of 256, K 256 or 512) -> the operand of qs_linear_tanh_x3: the packs of its
    256 x 256 blocks W[256 z .., 256 p ..] in (z, p) order, one contiguous int16 tensor.  ValueError out of range."""
    n, k = w.shape
    assert n % 256 == 0 and k in (256, 512), (n, k)
    blocks = [w[256 * z:256 * (z + 1), 256 * p:256 * (p + 1)] for z in range(n // 256) for p in range(k // 256)]
    return torch.stack(pack_mfma_weights_x3(blocks)).contiguous()


def ff_supported(lin):
    """Can qs_linear_tanh_x3 evaluate this feed_forward Linear?"""
    return lin.in_features in (256, 512) and lin.out_features % 256 == 0 and 256 <= lin.out_features <= 1024


def self_l2_supported(se):
    """The self encoder's second Linear + Tanh (Sequential(Linear, Tanh, Linear, Tanh), tanh inputs) on
    qs_linear_tanh_x3?"""
    return (len(se) == 4 and isinstance(se[1], torch.nn.Tanh) and isinstance(se[3], torch.nn.Tanh)
            and isinstance(se[2], torch.nn.Linear) and ff_supported(se[2]))


def linear_tanh_x3(x, packed, bias, out=None):
    """tanh(x W^T + b) for x [M, K] (|x| <= 1: tanh outputs) on the split-f16 matrix cores (qs_linear_tanh_x3)."""
    M, K = x.shape
    N = bias.shape[0]
    y = out if out is not None else torch.empty(M, N, dtype=torch.float32, device=x.device)
    st = ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream)
    assert x.is_contiguous() and packed.is_contiguous() and bias.is_contiguous() and y.is_contiguous()
    NAT.check(NAT.lib().qs_linear_tanh_x3(ctypes.c_void_p(x.data_ptr()), M, K, ctypes.c_void_p(packed.data_ptr()),
                                          packed.numel() * packed.element_size(), ctypes.c_void_p(bias.data_ptr()),
                                          ctypes.c_void_p(y.data_ptr()), N, st),
              "qs_linear_tanh_x3")
    return y


def linear_tanh_cat_x3(x0, x1, packed, bias, out=None):
    """tanh([x0 | x1] W^T + b) for x0, x1 [M, 256] (|x| <= 1) without forming the concatenation (qs_linear_tanh_cat_x3);
    packed = pack_linear_x3(W) for W [N, 512]."""
    M = x0.shape[0]
    N = bias.shape[0]
    assert x0.shape == (M, 256) and x1.shape == (M, 256)
    y = out if out is not None else torch.empty(M, N, dtype=torch.float32, device=x0.device)
    assert x0.is_contiguous() and x1.is_contiguous() and packed.is_contiguous() and bias.is_contiguous() and y.is_contiguous()
    st = ctypes.c_void_p(torch.cuda.current_stream(x0.device).cuda_stream)
    NAT.check(NAT.lib().qs_linear_tanh_cat_x3(ctypes.c_void_p(x0.data_ptr()), ctypes.c_void_p(x1.data_ptr()), M,
                                              ctypes.c_void_p(packed.data_ptr()), packed.numel() * packed.element_size(),
                                              ctypes.c_void_p(bias.data_ptr()), ctypes.c_void_p(y.data_ptr()), N, st),
              "qs_linear_tanh_cat_x3")
    return y


def cat_free(parts):
    """Two contiguous [M, 256] parts: qs_linear_tanh_cat_x3 reads them in place of their concatenation."""
    return (len(parts) == 2 and all(p.dim() == 2 and p.shape[1] == 256 and p.is_contiguous() for p in parts)
            and parts[0].shape[0] == parts[1].shape[0])


def linear_bias_x3(x, packed, bias, out=None):
    """x W^T + b for x [M, K] (|x| <= 1) on the split-f16 matrix cores (qs_linear_bias_x3: qs_linear_tanh_x3 without
    the tanh); the attention score layer's mean half P = e_mean A_m^T + b_a1."""
    M, K = x.shape
    N = bias.shape[0]
    y = out if out is not None else torch.empty(M, N, dtype=torch.float32, device=x.device)
    assert x.is_contiguous() and packed.is_contiguous() and bias.is_contiguous() and y.is_contiguous()
    st = ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream)
    NAT.check(NAT.lib().qs_linear_bias_x3(ctypes.c_void_p(x.data_ptr()), M, K, ctypes.c_void_p(packed.data_ptr()),
                                          packed.numel() * packed.element_size(), ctypes.c_void_p(bias.data_ptr()),
                                          ctypes.c_void_p(y.data_ptr()), N, st),
              "qs_linear_bias_x3")
    return y


def linear_rows_x3(x, row_scale, packed, n_out, out=None):
    """x W^T for rows x [M, K] of any magnitude (their power-of-two scales row_scale [M]: _pow2_scales of the row
    maxima) on the split-f16 matrix cores (qs_linear_rows_x3); packed = pack_linear_x3(W) for W [n_out, K]."""
    M, K = x.shape
    y = out if out is not None else torch.empty(M, n_out, dtype=torch.float32, device=x.device)
    assert x.is_contiguous() and row_scale.is_contiguous() and packed.is_contiguous() and y.is_contiguous()
    st = ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream)
    NAT.check(NAT.lib().qs_linear_rows_x3(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(row_scale.data_ptr()), M, K,
                                          ctypes.c_void_p(packed.data_ptr()), packed.numel() * packed.element_size(),
                                          ctypes.c_void_p(y.data_ptr()), n_out, st),
              "qs_linear_rows_x3")
    return y


def supports(policy):
    """Can the fused kernels evaluate this policy's encoders?"""
    c = policy.cfg
    return (c.neighbor_encoder_type == "attention" and c.num_use_neighbor_obs >= 1 and
            c.neighbor_hidden_size in (128, 256) and 1 <= c.neighbor_obs_dim <= 16 and
            c.num_use_neighbor_obs <= 64 and c.self_obs_dim + c.neighbor_obs_dim <= 32 and c.nonlinearity == "tanh")


class FusedRolloutPolicy:
    """forward(obs) / predict_values(obs) of a SwarmActorCritic with the fused neighbour encoders.
    refresh() re-packs the weights: call it whenever the policy's parameters changed (PPOTrainer does,
    once per rollout)."""

    PRECISIONS = ("fp32", "x3")

    def __init__(self, policy, precision="fp32"):
        """precision "fp32": fp32 operands on the fp32 matrix cores (v_mfma_f32_32x32x2f32); "x3": every fp32 product
        as three f16 products (hi/lo split, fp32 accumulation, ~7e-7 relative per product) on the f16 matrix cores
        (csrc/qs_policy_x3.h), 5.3x the contraction rate."""
        if precision not in self.PRECISIONS:
            raise ValueError(f"precision must be one of {self.PRECISIONS}")
        self.precision = precision
        self.packed_precision = None   # what refresh() packed: precision, or fp32 when x3 weights are out of range
        self._obs_absmax = None        # running max |obs| the x3 layer 0 has seen since the last check_inputs()
        if not supports(policy):
            raise ValueError("fused rollout forward: needs the tanh attention encoder with hidden size 128 or 256")
        self.policy = policy
        self.cfg = policy.cfg
        self.H = self.cfg.neighbor_hidden_size
        self.K = self.cfg.num_use_neighbor_obs
        self.nd = self.cfg.neighbor_obs_dim
        self.so = self.cfg.self_obs_dim
        self.encs = (policy.actor_encoder, policy.critic_encoder)
        self.L = NAT.lib()
        self.B = None
        self.packed = None
        self.towers = (NAT.QsAttnTower * NAT.ATTN_MAX_TOWERS)()

    # ---- weights / buffers ----
    def refresh(self):
        """Re-pack the weights.  x3: a weight outside the split-f16 range (|w| >= 255.9) would become +-inf; the
        towers are then packed (and evaluated) in fp32 until a later refresh finds every weight in range again."""
        prec = self.precision
        if prec == "x3":
            lim = F16_MAX / X3_SW
            big = max(float(m.weight.detach().abs().amax()) for enc in self.encs
                      for m in (enc.neighbor_encoder.embedding_mlp[0], enc.neighbor_encoder.embedding_mlp[2],
                                enc.neighbor_encoder.neighbor_value_mlp[0], enc.neighbor_encoder.neighbor_value_mlp[2],
                                enc.neighbor_encoder.attention_mlp[0], enc.neighbor_encoder.attention_mlp[2]))
            if not big < lim:
                import warnings
                warnings.warn(f"x3 rollout encoders: max |w| = {big:.4g} >= {lim:.4g} (f16 range); packing fp32")
                prec = "fp32"
        self.packed_precision = prec
        self._pack(prec)

    def check_inputs(self):
        """x3 only: raise if an observation given to the encoders since the last call was beyond the split-f16 range
        of layer 0 (|obs| >= 4094 packs as +-inf), i.e. the outputs of those calls are not the fp32 function.
        Non-finite observations are left to the env's non-finite guard.  One host sync (PPOTrainer: per rollout)."""
        m, self._obs_absmax = self._obs_absmax, None
        if m is None:
            return
        v = float(m)
        if v == v and v != float("inf") and v * X3_SIN >= F16_MAX:
            raise ValueError(f"x3 rollout encoders: an observation reached |obs| = {v:.4g} >= {F16_MAX / X3_SIN:.4g}, "
                             "beyond the split-f16 range of layer 0; use rollout_precision='fp32'")

    def _pack(self, prec):
        H, so = self.H, self.so
        pack = pack_mfma_weight_x3 if prec == "x3" else pack_mfma_weight
        packed = []
        for enc in self.encs:
            ne = enc.neighbor_encoder
            emb, val, att = ne.embedding_mlp, ne.neighbor_value_mlp, ne.attention_mlp
            w0 = emb[0].weight.detach()
            w_e1 = torch.zeros(H, 32, dtype=torch.float32, device=w0.device)   # [neighbour | self | 0]
            w_e1[:, :self.nd] = w0[:, so:]
            w_e1[:, self.nd:self.nd + so] = w0[:, :so]
            packed.append(dict(
                w_e1p=pack(w_e1), b_e1=emb[0].bias.detach(),
                w_e2p=pack(emb[2].weight), b_e2=emb[2].bias.detach(),
                w_v1p=pack(val[0].weight), b_v1=val[0].bias.detach(),
                w_v2p=pack(val[2].weight), b_v2=val[2].bias.detach(),
                w_a1ep=pack(att[0].weight[:, :H]), w_a1m=att[0].weight[:, H:].detach().contiguous(),
                b_a1=att[0].bias.detach().contiguous(),
                w_a2p=pack(att[2].weight), b_a2=att[2].bias.detach(),
                w_a3=att[4].weight.detach().reshape(-1).contiguous(), b_a3=float(att[4].bias.detach().item())))
            if prec == "x3" and H == 256:   # P = e_mean A_m^T + b_a1 on qs_linear_bias_x3 (|e_mean| <= 1)
                packed[-1].update(w_a1mp=pack_linear_x3(att[0].weight[:, H:].detach()))
            ff = enc.feed_forward[0]
            if prec == "x3" and ff_supported(ff) and float(ff.weight.detach().abs().amax()) < F16_MAX / X3_SW:
                packed[-1].update(w_ffp=pack_linear_x3(ff.weight.detach()), b_ff=ff.bias.detach().contiguous())
            se = enc.self_encoder
            if (prec == "x3" and self_l2_supported(se)
                    and float(se[2].weight.detach().abs().amax()) < F16_MAX / X3_SW):
                packed[-1].update(w_s2p=pack_linear_x3(se[2].weight.detach()), b_s2=se[2].bias.detach().contiguous())
        self.packed = packed
        self._bind()

    def _alloc(self, B, dev):
        H, K, T = self.H, self.K, len(self.encs)
        z = lambda *s: torch.empty(*s, dtype=torch.float32, device=dev)  # noqa: E731
        self.B = B
        self.P = z(T, B, H)
        self.e2, self.e_mean, self.out = z(T, B * K, H), z(T, B, H), z(T, B, H)
        self._bind()

    def _bind(self):
        if self.packed is None or self.B is None:
            return
        p = lambda t: t.data_ptr()  # noqa: E731
        for i, w in enumerate(self.packed):
            t = self.towers[i]
            t.w_e1p, t.b_e1 = p(w["w_e1p"]), p(w["b_e1"])
            t.w_e2p, t.b_e2 = p(w["w_e2p"]), p(w["b_e2"])
            t.e2, t.e_mean, t.P = p(self.e2[i]), p(self.e_mean[i]), p(self.P[i])
            t.w_v1p, t.b_v1, t.w_v2p, t.b_v2 = p(w["w_v1p"]), p(w["b_v1"]), p(w["w_v2p"]), p(w["b_v2"])
            t.w_a1ep, t.w_a2p, t.b_a2, t.w_a3 = p(w["w_a1ep"]), p(w["w_a2p"]), p(w["b_a2"]), p(w["w_a3"])
            t.b_a3, t.out = w["b_a3"], p(self.out[i])

    # ---- forward ----
    @torch.no_grad()
    def neighbor_encodings(self, obs):
        """[T, B, H]: both towers' QuadNeighborhoodEncoderAttention outputs (the tensor is reused by the next call)."""
        assert obs.is_cuda and obs.dtype == torch.float32 and obs.dim() == 2
        obs = obs.contiguous()
        B = obs.shape[0]
        if self.packed is None:
            self.refresh()
        if self.B != B:
            self._alloc(B, obs.device)
        so, H, K = self.so, self.H, self.K
        st = ctypes.c_void_p(torch.cuda.current_stream(obs.device).cuda_stream)
        x3 = self.packed_precision == "x3"
        if x3:   # the range check of the layer-0 inputs, on the device (read by check_inputs)
            m = obs.abs().amax()
            self._obs_absmax = m if self._obs_absmax is None else torch.maximum(self._obs_absmax, m)
        embed, pool = (self.L.qs_attn_embed_x3, self.L.qs_attn_pool_x3) if x3 else (self.L.qs_attn_embed, self.L.qs_attn_pool)
        NAT.check(embed(ctypes.c_void_p(obs.data_ptr()), obs.shape[1], so, so, B, K, self.nd, H,
                        self.towers, len(self.encs), st), "qs_attn_embed")
        for i, w in enumerate(self.packed):
            if "w_a1mp" in w:
                linear_bias_x3(self.e_mean[i], w["w_a1mp"], w["b_a1"], out=self.P[i])
            else:
                torch.addmm(w["b_a1"], self.e_mean[i], w["w_a1m"].t(), out=self.P[i])
        NAT.check(pool(B, K, H, self.towers, len(self.encs), st), "qs_attn_pool")
        return self.out

    def _encode(self, enc, obs, nbr_out, w=None):
        so, na = self.so, enc.all_neighbor_obs_size
        se = enc.self_encoder
        if w is not None and "w_s2p" in w:   # x3: the second Linear + Tanh (tanh inputs) as one kernel
            parts = [linear_tanh_x3(se[1](se[0](obs[:, :so])), w["w_s2p"], w["b_s2"]), nbr_out]
        else:
            parts = [se(obs[:, :so]), nbr_out]
        if enc.obstacle_encoder is not None:
            parts.append(enc.obstacle_encoder(obs[:, so + na:]))
        if w is not None and "w_ffp" in w and cat_free(parts):   # x3, [self | neighbour] read in place
            return linear_tanh_cat_x3(parts[0], parts[1], w["w_ffp"], w["b_ff"])
        x = torch.cat(parts, dim=1)
        if w is not None and "w_ffp" in w:   # x3: the feed_forward's Linear + Tanh as one kernel (|x| <= 1: tanh rows)
            return linear_tanh_x3(x, w["w_ffp"], w["b_ff"])
        return enc.feed_forward(x)

    @torch.no_grad()
    def forward(self, obs, deterministic=False):
        """SwarmActorCritic.forward: (actions, values [B, 1], log_prob [B])."""
        from .ppo import squashed_log_prob
        pol = self.policy
        nbr = self.neighbor_encodings(obs)
        a_lat = pol.actor_decoder(pol.actor_core(self._encode(pol.actor_encoder, obs, nbr[0], self.packed[0])))
        mean = pol.action_net(a_lat)
        values = pol.value_net(pol.critic_decoder(pol.critic_core(self._encode(pol.critic_encoder, obs, nbr[1],
                                                                               self.packed[1]))))
        if deterministic:
            actions = torch.tanh(mean)
        else:
            actions = torch.tanh(mean + torch.randn_like(mean) * pol.log_std.exp())
        return actions, values, squashed_log_prob(mean, pol.log_std, actions)

    __call__ = forward

    @torch.no_grad()
    def predict_values(self, obs):
        pol = self.policy
        nbr = self.neighbor_encodings(obs)
        return pol.value_net(pol.critic_decoder(pol.critic_core(self._encode(pol.critic_encoder, obs, nbr[1],
                                                                             self.packed[1]))))
