"""The PPO update's attention neighbour encoders on the split-f16 matrix cores (the update side).

PPO.train (as PPOTrainer.train restates it) evaluates ActorCriticPolicyCustomSeparateWeights on every minibatch with
autograd (swarm_rl/models/ActorCriticPolicyCustom.py:538-566); 89 % of a C3 update is the two towers'
QuadNeighborhoodEncoderAttention (swarm_rl/models/quad_multi_model.py:44-101): per neighbour row five H x H layers
with tanh, forward and backward, ~20 hipBLASLt GEMMs and as many elementwise tanh / tanh-backward passes per tower.
Here both towers' encoders are one autograd node (FusedAttentionTrain), whose forward and backward are the HIP
kernels of csrc/qs_policy_train.h through the C ABI:

  forward   qs_attn_embed_train_x3 (e1, e2, mean_K e2), P = mean A_m^T + b_a1 (qs_linear_bias_x3), qs_attn_pool_train_x3 (a1, a2,
            softmax, v1, h, pooled out) -- the rollout's x3 kernels plus the saved activations
  backward  qs_attn_bwd1_x3: the value chain (dh_pre -> dv1_pre -> dL/de2) and the attention chain (dscore ->
            da2_pre -> da1_pre -> dL/de2) of every 64-row block on the matrix cores, tanh derivatives in the epilogues;
            dP (qs_slab_sum_stats) and dL/d e_mean (qs_linear_rows_x3): the grid-wide per-agent terms, [B, H];
            qs_attn_bwd2_x3: dL/de2 -> de2_pre -> de1_pre;
            the weight gradients dW = grad^T act over the B K rows on the same split-f16 matrix cores (qs_attn_dw_x3:
            split over row ranges, per-column power-of-two scales of the gradient, the parts summed by torch), the
            biases as column sums, the small [B]-row terms (dA_m, the self half of layer 0) as torch GEMMs.
Every contraction of the kernels is an fp32 product carried as three f16 products (hi/lo split, fp32 accumulation,
~7e-7 relative per product; the backward's rows with their own power-of-two scales), i.e. fp32-equivalent; the
gradients match the torch module's fp32 autograd within fp32 reassociation (tests/test_gpu_encoder_train.py).
"""
import ctypes

import torch

from . import _native as NAT
from .policy_fused import (F16_MAX, X3_SIN, X3_SW, cat_free, ff_supported, linear_bias_x3,  # noqa: F401
                           linear_rows_x3, linear_tanh_cat_x3, linear_tanh_x3, pack_mfma_weight_x3, pack_mfma_weights_x3,
                           self_l2_supported, supports)

_PARAMS = ("e1_w", "e1_b", "e2_w", "e2_b", "v1_w", "v1_b", "v2_w", "v2_b", "a1_w", "a1_b", "a2_w", "a2_b", "a3_w", "a3_b")


def tower_params(enc):
    """The 14 parameters of one tower's NeighborAttention, in _PARAMS order."""
    ne = enc.neighbor_encoder
    emb, val, att = ne.embedding_mlp, ne.neighbor_value_mlp, ne.attention_mlp
    return [emb[0].weight, emb[0].bias, emb[2].weight, emb[2].bias, val[0].weight, val[0].bias, val[2].weight,
            val[2].bias, att[0].weight, att[0].bias, att[2].weight, att[2].bias, att[4].weight, att[4].bias]


def _pow2_scales(m):
    """Power-of-two scales s with s m in [2^13, 2^14) (1 where m is 0 or not finite), built from their exponent bits:
    they must be exact powers of two (torch.ldexp goes through pow on the device and is not), else the kernel's f16
    hi / lo split of s G is taken from a rounded product and near-tie elements lose an ulp of the hi half."""
    _, e = torch.frexp(m)
    k = (14 - e.to(torch.int32)).clamp(-126, 127)
    s = ((k + 127) << 23).view(torch.float32)
    return torch.where((m > 0) & torch.isfinite(m), s, torch.ones_like(m)).contiguous()


def col_scales(G):
    """Per-column power-of-two scales of a gradient [R, H] for qs_attn_dw_x3: s_n |G[:, n]| in [2^13, 2^14) (1 for an
    all-zero or non-finite column)."""
    return _pow2_scales(G.abs().amax(0))


def col_stats(G, obs=None, B=0, K=0, nbr_off=0, nd=0, nx=0, parts=None, row_w=None):
    """One pass over G [R, H] (qs_colstats): (the dW column scales, the column sums sum_r w_r G[r, :] (row_w = w [R],
    default 1), and with obs the layer-0 weight gradient sum_r G[r, :]^T X(r, :) as [nx, H] -- X the encoder's layer-0
    input of row r, neighbour features first, then the self features -- or None)."""
    R, H = G.shape
    parts = parts or max(1, min(2048, (R + 255) // 256))
    z = lambda *sh: torch.empty(*sh, dtype=torch.float32, device=G.device)  # noqa: E731
    pmx, psm = z(parts, H), z(parts, H)
    px = z(parts, nx, H) if nx else None
    st = ctypes.c_void_p(torch.cuda.current_stream(G.device).cuda_stream)
    NAT.check(NAT.lib().qs_colstats(ctypes.c_void_p(G.data_ptr()), R, H,
                                    ctypes.c_void_p(row_w.data_ptr() if row_w is not None else 0),
                                    ctypes.c_void_p(obs.data_ptr() if obs is not None else 0),
                                    obs.shape[1] if obs is not None else 0, nbr_off, B, K, nd, nx,
                                    ctypes.c_void_p(pmx.data_ptr()), ctypes.c_void_p(psm.data_ptr()),
                                    ctypes.c_void_p(px.data_ptr() if px is not None else 0), parts, st),
              "qs_colstats")
    return _pow2_scales(pmx.amax(0)), psm.sum(0), (px.sum(0) if px is not None else None)


def colmax_scales(part_max):
    """dW column scales from per-block column maxima [n_stats, n_blocks, H] (qs_attn_train.colmax rows): the max over
    the blocks (qs_colmax_reduce), then the power-of-two scales -> [n_stats, H]."""
    ns, nb, H = part_max.shape
    out = torch.empty(ns, H, dtype=torch.float32, device=part_max.device)
    st = ctypes.c_void_p(torch.cuda.current_stream(part_max.device).cuda_stream)
    NAT.check(NAT.lib().qs_colmax_reduce(ctypes.c_void_p(part_max.data_ptr()), ns, nb, H, ctypes.c_void_p(out.data_ptr()),
                                         st), "qs_colmax_reduce")
    return _pow2_scales(out)


def dw_x3(G, A, parts=256, out=None, gs=None, sums=False):
    """G^T A ([H, H]) over the rows of G, A [R, H] (|A| <= 1) on the split-f16 matrix cores (qs_attn_dw_x3), the row
    range split over `parts` blocks and the parts summed here.  gs: G's column scales (col_scales / col_stats).
    sums: also G's column sums from the same pass (returns (dW, sums))."""
    R, H = G.shape
    assert G.stride(1) == 1 and A.stride(1) == 1 and A.shape == G.shape   # rows may be slices of wider ones
    parts = max(1, min(parts, (R + 15) // 16))
    buf = torch.empty(parts, H, H, dtype=torch.float32, device=G.device)
    psum = torch.empty(parts, H, dtype=torch.float32, device=G.device) if sums else None
    if gs is None:
        gs = col_scales(G)
    gs = gs.contiguous()
    st = ctypes.c_void_p(torch.cuda.current_stream(G.device).cuda_stream)
    NAT.check(NAT.lib().qs_dw_x3_ld(ctypes.c_void_p(G.data_ptr()), G.stride(0), ctypes.c_void_p(A.data_ptr()),
                                    A.stride(0), ctypes.c_void_p(gs.data_ptr()), R, H, ctypes.c_void_p(buf.data_ptr()),
                                    ctypes.c_void_p(psum.data_ptr() if sums else 0), parts, st),
              "qs_dw_x3_ld")
    dW = torch.sum(buf, dim=0, out=out)
    return (dW, psum.sum(0)) if sums else dW


def dw0_x3(G, obs, B, K, so, nd, gs=None, parts=512):
    """Layer 0's weight gradient sum_j G_j^T x0_j ([H, nd + so], in the reference's column order [self | neighbour])
    and the bias gradient sum_j G_j, x0_j = [nbr_j | self_{j % B}] gathered from `obs` (the forward's pairing), on the
    split-f16 matrix cores (qs_attn_dw0_x3; gs: G's column scales, col_scales by default)."""
    R, H = G.shape
    parts = max(1, min(parts, (R + 15) // 16))
    buf = torch.empty(parts, H, 32, dtype=torch.float32, device=G.device)
    psum = torch.empty(parts, H, dtype=torch.float32, device=G.device)
    if gs is None:
        gs = col_scales(G)
    st = ctypes.c_void_p(torch.cuda.current_stream(G.device).cuda_stream)
    NAT.check(NAT.lib().qs_attn_dw0_x3(ctypes.c_void_p(G.data_ptr()), ctypes.c_void_p(gs.data_ptr()),
                                       ctypes.c_void_p(obs.data_ptr()), obs.shape[1], so, so, B, K, nd, H,
                                       ctypes.c_void_p(buf.data_ptr()), ctypes.c_void_p(psum.data_ptr()), parts, st),
              "qs_attn_dw0_x3")
    dW = buf.sum(0)
    return torch.cat((dW[:, nd:nd + so], dW[:, :nd]), dim=1), psum.sum(0)


def slab_sum_stats(G, n_slabs, out, row_scale, col_part):
    """out [M, N] = sum_s G[s M + m] for G [n_slabs M, N] (qs_slab_sum_stats: dP[b] = sum_k da1_pre[k B + b]), with
    out's row scales [M] and per-64-row-block column maxima [1, ceil(M / 64), N] in the same pass."""
    M, N = out.shape
    assert G.is_contiguous() and G.shape == (n_slabs * M, N) and out.is_contiguous()
    assert row_scale.shape == (M,) and col_part.shape == (1, (M + 63) // 64, N)
    st = ctypes.c_void_p(torch.cuda.current_stream(G.device).cuda_stream)
    NAT.check(NAT.lib().qs_slab_sum_stats(ctypes.c_void_p(G.data_ptr()), n_slabs, M, N, ctypes.c_void_p(out.data_ptr()),
                                          ctypes.c_void_p(row_scale.data_ptr()), ctypes.c_void_p(col_part.data_ptr()),
                                          st), "qs_slab_sum_stats")
    return out


class _Runner:
    """Buffers and launches for one policy's towers (reused across minibatches of the same size)."""

    def __init__(self, policy):
        c = policy.cfg
        self.H, self.K, self.nd, self.so = c.neighbor_hidden_size, c.num_use_neighbor_obs, c.neighbor_obs_dim, c.self_obs_dim
        self.encs = (policy.actor_encoder, policy.critic_encoder)
        self.T = len(self.encs)
        self.L = NAT.lib()
        self.B = None
        self.towers = (NAT.QsAttnTower * NAT.ATTN_MAX_TOWERS)()
        self.trains = (NAT.QsAttnTrain * NAT.ATTN_MAX_TOWERS)()
        self.pending = False
        self.lin_packed = {}   # id(Linear) -> its qs_linear_tanh_x3 operand, packed with this minibatch's weights
        self.dw_x3 = True   # the weight gradients on the split-f16 matrix cores (else torch fp32 GEMMs)

    def dw(self, G, A, gs=None):
        """(dW = G^T A over the B K rows (A: tanh outputs), the bias gradient sum_r G[r, :]).  gs: G's column scales
        from the maxima the kernels that wrote G formed (colmax_scales): then one pass over G and A (the sums from the
        dW pass), else a column-statistics pass first."""
        if not self.dw_x3:
            return G.t().mm(A), G.sum(0)
        if gs is not None:
            return dw_x3(G, A, gs=gs, sums=True)
        gs, sums, _ = col_stats(G)
        return dw_x3(G, A, gs=gs), sums

    def _alloc(self, B, dev):
        H, T, R = self.H, self.T, B * self.K
        z = lambda *s: torch.empty(*s, dtype=torch.float32, device=dev)  # noqa: E731
        self.B = B
        mu = (64 // self.K) * self.K                 # the kernels' row blocks (qs_policy.h MROWS = 64)
        nblk = (R + mu - 1) // mu
        self.buf = [dict(e1=z(R, H), e2=z(R, H), a1=z(R, H), a2=z(R, H), v1=z(R, H), h=z(R, H), w=z(R),
                         e_mean=z(B, H), P=z(B, H), dh_pre=z(R, H), dv1_pre=z(R, H), da2_pre=z(R, H),
                         da1_pre=z(R, H), de2p=z(R, H), dscore=z(R), dem=z(B, H),
                         colmax=z(NAT.ATTN_NCOLMAX, nblk, H), a3w_part=z(nblk, H),
                         dP=z(B, H), dP_rs=z(B), dP_cm=z(1, (B + 63) // 64, H)) for _ in range(T)]

    def _pack(self, params):
        """x3-pack the towers' weights (forward operands and the backward's transposes; both towers' 22 matrices as
        one batched pack with one range check), bind every pointer."""
        H, so, nd = self.H, self.so, self.nd
        p = lambda t: t.data_ptr()  # noqa: E731
        self.keep = []
        names = ("w_e1p", "w_e2p", "w_v1p", "w_v2p", "w_a1ep", "w_a2p", "w_v2tp", "w_v1tp", "w_a2tp", "w_a1etp",
                 "w_e2tp")
        ws, mats = [], []
        for i in range(self.T):
            w = dict(zip(_PARAMS, params[14 * i:14 * i + 14]))
            w_e1 = torch.zeros(H, 32, dtype=torch.float32, device=w["e1_w"].device)   # [neighbour | self | 0]
            w_e1[:, :nd] = w["e1_w"][:, so:]
            w_e1[:, nd:nd + so] = w["e1_w"][:, :so]
            ws.append(w)
            mats += [w_e1, w["e2_w"], w["v1_w"], w["v2_w"], w["a1_w"][:, :H], w["a2_w"], w["v2_w"].t(), w["v1_w"].t(),
                     w["a2_w"].t(), w["a1_w"][:, :H].t(), w["e2_w"].t()]
        # the score layer's mean half A_m (P's forward) and A_m^T (dL/d e_mean) for the x3 linear kernels (H 256)
        am_span = None
        if H == 256 and self.dw_x3:
            am_span = len(mats)
            for w in ws:
                mats += [w["a1_w"][:, H:], w["a1_w"][:, H:].t()]
        # the feed_forward Linears' and the self encoders' second Linears' 256 x 256 blocks ride along
        # (FusedAttentionTrain.feed_forward: Linear + Tanh of tanh inputs on qs_linear_tanh_x3)
        lins = [enc.feed_forward[0] for enc in self.encs if ff_supported(enc.feed_forward[0])]
        lins += [enc.self_encoder[2] for enc in self.encs if self_l2_supported(enc.self_encoder)]
        spans = []
        for f in lins:
            for w in (f.weight, f.weight.t()):   # the forward's W and the backward's dX operand W^T
                blocks = [w[256 * z:256 * (z + 1), 256 * q:256 * (q + 1)] for z in range(w.shape[0] // 256)
                          for q in range(w.shape[1] // 256)]
                spans.append((len(mats), len(blocks)))
                mats += blocks
        packed = pack_mfma_weights_x3(mats)
        self.lin_packed = {id(f): tuple(torch.stack(packed[a:a + n]).contiguous() for a, n in spans[2 * i:2 * i + 2])
                           for i, f in enumerate(lins)}
        self.am_packed = ([(packed[am_span + 2 * i][None].contiguous(), packed[am_span + 2 * i + 1][None].contiguous())
                           for i in range(self.T)] if am_span is not None else None)
        for i in range(self.T):
            w, b = ws[i], self.buf[i]
            k = dict(zip(names, packed[len(names) * i:len(names) * (i + 1)]))
            k.update(b_e1=w["e1_b"].detach().contiguous(), b_e2=w["e2_b"].detach().contiguous(),
                     b_v1=w["v1_b"].detach().contiguous(), b_v2=w["v2_b"].detach().contiguous(),
                     b_a2=w["a2_b"].detach().contiguous(), w_a3=w["a3_w"].detach().reshape(-1).contiguous(),
                     a_m=w["a1_w"][:, H:].detach().contiguous(), b_a1=w["a1_b"].detach().contiguous())
            self.keep.append(k)
            t = self.towers[i]
            t.w_e1p, t.b_e1, t.w_e2p, t.b_e2 = p(k["w_e1p"]), p(k["b_e1"]), p(k["w_e2p"]), p(k["b_e2"])
            t.e2, t.e_mean, t.P = p(b["e2"]), p(b["e_mean"]), p(b["P"])   # t.out: per forward
            t.w_v1p, t.b_v1, t.w_v2p, t.b_v2 = p(k["w_v1p"]), p(k["b_v1"]), p(k["w_v2p"]), p(k["b_v2"])
            t.w_a1ep, t.w_a2p, t.b_a2, t.w_a3 = p(k["w_a1ep"]), p(k["w_a2p"]), p(k["b_a2"]), p(k["w_a3"])
            t.b_a3 = float(w["a3_b"].detach().item())
            r = self.trains[i]
            for n in ("e1", "a1", "a2", "v1", "h", "w", "dh_pre", "dv1_pre", "da2_pre", "da1_pre", "dscore", "de2p", "dem",
                      "colmax", "a3w_part"):
                setattr(r, n, p(b[n]))
            r.de2_pre = p(b["de2p"])      # in place: bwd2 reads de2p[j] and writes de2_pre[j] on the same lane
            r.de1_pre = p(b["dh_pre"])    # dh_pre's last reader (dW_v2) runs before bwd2
            for n in ("w_v2tp", "w_v1tp", "w_a2tp", "w_a1etp", "w_e2tp"):
                setattr(r, n, p(k[n]))

    def stream(self, dev):
        return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)

    @torch.no_grad()
    def forward(self, obs, params):
        B = obs.shape[0]
        if self.B != B:
            self._alloc(B, obs.device)
        self._pack(params)
        self.obs = obs
        self.params = params
        H, K, so, st = self.H, self.K, self.so, self.stream(obs.device)
        NAT.check(self.L.qs_attn_embed_train_x3(ctypes.c_void_p(obs.data_ptr()), obs.shape[1], so, so, B, K, self.nd, H,
                                                self.towers, self.trains, self.T, st), "qs_attn_embed_train_x3")
        for i in range(self.T):   # P = e_mean A_m^T + b_a1 (|e_mean| <= 1: a mean of tanh rows)
            if self.am_packed is not None:
                linear_bias_x3(self.buf[i]["e_mean"], self.am_packed[i][0], self.keep[i]["b_a1"], out=self.buf[i]["P"])
            else:   # A_m contiguous: the strided slice picks a 4x slower GEMM
                torch.addmm(params[14 * i + 9], self.buf[i]["e_mean"], self.keep[i]["a_m"].t(), out=self.buf[i]["P"])
        # the pooled outputs into fresh tensors (autograd owns them; no copy out of a reused buffer)
        outs = [torch.empty(B, H, dtype=torch.float32, device=obs.device) for _ in range(self.T)]
        for i in range(self.T):
            self.towers[i].out = outs[i].data_ptr()
        NAT.check(self.L.qs_attn_pool_train_x3(B, K, H, self.towers, self.trains, self.T, st), "qs_attn_pool_train_x3")
        self.pending = True
        return outs

    @torch.no_grad()
    def backward(self, douts):
        if not self.pending:
            raise RuntimeError("FusedAttentionTrain: backward without a pending forward (buffers reused)")
        B, H, K, so, nd = self.B, self.H, self.K, self.so, self.nd
        obs, params = self.obs, self.params
        st = self.stream(obs.device)
        d = []
        for i in range(self.T):
            g = douts[i]
            d.append(torch.zeros(B, H, device=obs.device) if g is None else g.contiguous())
            self.trains[i].dout = d[i].data_ptr()
        NAT.check(self.L.qs_attn_bwd1_x3(B, K, H, self.towers, self.trains, self.T, st), "qs_attn_bwd1_x3")
        grads = [None] * (14 * self.T)
        for i in range(self.T):
            b, w0 = self.buf[i], 14 * i
            gsc = colmax_scales(b["colmax"][:4])   # the gradients' column scales (per-block maxima from backward 1)
            gi = {}
            gi["v2_w"], gi["v2_b"] = self.dw(b["dh_pre"], b["v1"], gsc[0])
            gi["v1_w"], gi["v1_b"] = self.dw(b["dv1_pre"], b["e2"], gsc[1])
            gi["a2_w"], gi["a2_b"] = self.dw(b["da2_pre"], b["a1"], gsc[2])
            # sum_j dscore_j a2_j: backward 1's per-block partial sums
            gi["a3_w"] = b["a3w_part"].sum(0).view(1, -1) if self.dw_x3 else b["dscore"].view(1, -1).mm(b["a2"])
            gi["a3_b"] = b["dscore"].sum().view(1)
            dA_e, gi["a1_b"] = self.dw(b["da1_pre"], b["e2"], gsc[3])   # a1_b = sum_j da1_pre_j = sum_b dP_b
            if self.am_packed is not None:
                # dP[b] = sum of the rows j with j % B == b (the repeat tiling) with its row scales and column maxima,
                # dL/d e_mean = dP A_m on the x3 layer at those row scales, dA_m = dP^T e_mean (|e_mean| <= 1)
                dP = slab_sum_stats(b["da1_pre"], K, b["dP"], b["dP_rs"], b["dP_cm"])
                dA_m = self.dw(dP, b["e_mean"], colmax_scales(b["dP_cm"])[0])[0]
                linear_rows_x3(dP, b["dP_rs"], self.am_packed[i][1], H, out=b["dem"])
            else:
                dP = b["da1_pre"].view(K, B, H).sum(0)                 # rows j with j % B == b (the repeat tiling)
                dA_m = self.dw(dP, b["e_mean"])[0]
                torch.mm(dP, self.keep[i]["a_m"], out=b["dem"])        # dL/d e_mean
            gi["a1_w"] = torch.cat((dA_e, dA_m), dim=1)
            for n in gi:
                grads[w0 + _PARAMS.index(n)] = gi[n]
        NAT.check(self.L.qs_attn_bwd2_x3(B, K, H, self.towers, self.trains, self.T, st), "qs_attn_bwd2_x3")
        self_obs = obs[:, :so]
        nbr_rows = obs[:, so:so + K * nd].reshape(B * K, nd)
        for i in range(self.T):
            b, w0 = self.buf[i], 14 * i
            de2_pre, de1_pre = b["de2p"], b["dh_pre"]
            gsc2 = colmax_scales(b["colmax"][4:])   # de2_pre's and de1_pre's (backward 2)
            grads[w0 + 2], grads[w0 + 3] = self.dw(de2_pre, b["e1"], gsc2[0])
            # embedding_mlp[0] on cat(self_{j % B}, nbr_j): both halves and the bias gradient in one pass over
            # de1_pre with the layer-0 rows gathered as the forward gathers them
            if self.dw_x3:
                grads[w0], grads[w0 + 1] = dw0_x3(de1_pre, obs, B, K, so, nd, gs=gsc2[1])
            else:
                g_self = de1_pre.view(K, B, H).sum(0).t().mm(self_obs)
                grads[w0] = torch.cat((g_self, de1_pre.t().mm(nbr_rows)), dim=1)
                grads[w0 + 1] = de1_pre.sum(0)
        self.pending = False
        self.obs = self.params = None
        return grads


class _AttnTrainFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, runner, obs, *params):
        ctx.runner = runner
        return tuple(runner.forward(obs, params))

    @staticmethod
    def backward(ctx, *douts):
        return (None, None) + tuple(ctx.runner.backward(douts))


class _SelfLayer0Fn(torch.autograd.Function):
    """The self encoder's first Linear (self_obs [B, so] -> [B, R]) with its weight gradient on the split-f16 matrix
    cores: forward F.linear; backward dW = G^T self_obs by qs_attn_dw0_x3 (rows = agents: K 1, no neighbour
    features; G's column scales and the bias gradient from one column-statistics pass) in place of the skinny
    [R x B] x [B x so] GEMM.  No input gradient (observations)."""

    @staticmethod
    def forward(ctx, obs, weight, bias, so):
        ctx.save_for_backward(obs)
        ctx.so = so
        return torch.nn.functional.linear(obs[:, :so], weight, bias)

    @staticmethod
    def backward(ctx, g):
        (obs,) = ctx.saved_tensors
        g = g.contiguous()
        gs, sums, _ = col_stats(g)
        dW, db = dw0_x3(g, obs, obs.shape[0], 1, ctx.so, 0, gs=gs)
        return None, dW, sums, None


def _tanh_grad_stats(g, y):
    """gp = g (1 - y^2) with its row scales and its dW column scales (qs_tanh_grad_stats + qs_colmax_reduce)."""
    M, N = y.shape
    g = g.contiguous()
    gp = torch.empty(M, N, dtype=torch.float32, device=g.device)
    rs = torch.empty(M, dtype=torch.float32, device=g.device)
    cpart = torch.empty(1, (M + 63) // 64, N, dtype=torch.float32, device=g.device)
    st = ctypes.c_void_p(torch.cuda.current_stream(g.device).cuda_stream)
    NAT.check(NAT.lib().qs_tanh_grad_stats(ctypes.c_void_p(g.data_ptr()), ctypes.c_void_p(y.data_ptr()),
                                           ctypes.c_void_p(gp.data_ptr()), ctypes.c_void_p(rs.data_ptr()),
                                           ctypes.c_void_p(cpart.data_ptr()), M, N, st), "qs_tanh_grad_stats")
    return gp, rs, colmax_scales(cpart)[0]


class _FeedForwardFn(torch.autograd.Function):
    """QuadMultiEncoder.feed_forward (Linear + Tanh; also the self encoder's second layer) on the split-f16 matrix
    cores: forward qs_linear_tanh_x3 (|x| <= 1: tanh outputs); backward gp = g (1 - y^2) with its row scales and
    column maxima (qs_tanh_grad_stats), then dW = gp^T x by 256 x 256 blocks (qs_dw_x3_ld) and dX = gp W
    (qs_linear_rows_x3)."""

    @staticmethod
    def forward(ctx, x, weight, bias, packed, packed_t):
        y = linear_tanh_x3(x, packed, bias.detach())
        ctx.save_for_backward(x, weight, y)
        ctx.packed_t = packed_t
        return y

    @staticmethod
    def backward(ctx, g):
        x, weight, y = ctx.saved_tensors
        N, K = weight.shape
        gp, rs, gs = _tanh_grad_stats(g, y)
        # the weight gradient gp^T x on the split-f16 matrix cores by 256 x 256 blocks (x: tanh range), the bias
        # gradient from the same passes
        dW = torch.empty(N, K, dtype=torch.float32, device=g.device)
        db = torch.empty(N, dtype=torch.float32, device=g.device)
        for zn in range(N // 256):
            for zk in range(K // 256):
                r = dw_x3(gp[:, 256 * zn:256 * (zn + 1)], x[:, 256 * zk:256 * (zk + 1)], gs=gs[256 * zn:256 * (zn + 1)],
                          sums=True)
                dW[256 * zn:256 * (zn + 1), 256 * zk:256 * (zk + 1)] = r[0]
                if zk == 0:
                    db[256 * zn:256 * (zn + 1)] = r[1]
        # dX = gp W with each row at its power-of-two scale
        dx = linear_rows_x3(gp, rs, ctx.packed_t, K)
        return dx, dW, db, None, None


class _FeedForwardCatFn(torch.autograd.Function):
    """_FeedForwardFn on the concatenation [x0 | x1] of two [M, 256] encodings without forming it: the forward reads both
    (qs_linear_tanh_cat_x3), the backward's dX halves are two N = 256 products on W^T's row blocks (each contiguous:
    no split copies of a [M, 512] gradient) and dW's column blocks take x0 / x1 directly."""

    @staticmethod
    def forward(ctx, x0, x1, weight, bias, packed, packed_t):
        y = linear_tanh_cat_x3(x0, x1, packed, bias.detach())
        ctx.save_for_backward(x0, x1, weight, y)
        ctx.packed_t = packed_t
        return y

    @staticmethod
    def backward(ctx, g):
        x0, x1, weight, y = ctx.saved_tensors
        N = weight.shape[0]
        gp, rs, gs = _tanh_grad_stats(g, y)
        dW = torch.empty(N, 512, dtype=torch.float32, device=g.device)
        db = torch.empty(N, dtype=torch.float32, device=g.device)
        for zn in range(N // 256):
            for zk, x in enumerate((x0, x1)):
                r = dw_x3(gp[:, 256 * zn:256 * (zn + 1)], x, gs=gs[256 * zn:256 * (zn + 1)], sums=True)
                dW[256 * zn:256 * (zn + 1), 256 * zk:256 * (zk + 1)] = r[0]
                if zk == 0:
                    db[256 * zn:256 * (zn + 1)] = r[1]
        # dX = gp W: W^T's packed blocks are z-major over its 512 rows, (N / 256) blocks per 256 rows
        nb = N // 256
        pt = ctx.packed_t
        dx0 = linear_rows_x3(gp, rs, pt[:nb], 256) if ctx.needs_input_grad[0] else None
        dx1 = linear_rows_x3(gp, rs, pt[nb:2 * nb], 256) if ctx.needs_input_grad[1] else None
        return dx0, dx1, dW, db, None, None


class FusedAttentionTrain:
    """Both towers' neighbour-encoder outputs for the PPO update as one autograd node on the HIP kernels:
    encodings(obs) -> [actor [B, H], critic [B, H]] (SwarmActorCritic.evaluate_actions(obs, actions, nbr=...)).  One
    backward per forward (the activations live in reused buffers)."""

    def __init__(self, policy):
        if not supports(policy):
            raise ValueError("fused update: needs the tanh attention encoder with hidden size 128 or 256")
        self.policy = policy
        self.runner = _Runner(policy)

    def params(self):
        return [p for enc in self.runner.encs for p in tower_params(enc)]

    def feed_forward(self, lin, x):
        """tanh(lin(x)) for a tower's feed_forward Linear or its self encoder's second Linear, x a tanh-range input or
        the list of the encoder's parts to concatenate (QuadMultiEncoder.forward's ff hook): the x3 kernel when this
        minibatch's encodings packed it (_FeedForwardCatFn on two [B, 256] parts, else _FeedForwardFn), else torch."""
        packed = self.runner.lin_packed.get(id(lin))
        if isinstance(x, (list, tuple)):   # the encoder's [self | neighbour (| obstacle)] parts
            if packed is not None and lin.in_features == 512 and cat_free(x):
                return _FeedForwardCatFn.apply(x[0], x[1], lin.weight, lin.bias, packed[0], packed[1])
            x = torch.cat(x, dim=1) if len(x) > 1 else x[0]
        if packed is not None and x.is_contiguous():
            return _FeedForwardFn.apply(x, lin.weight, lin.bias, packed[0], packed[1])
        return torch.tanh(lin(x))

    def self_layer0(self, lin, obs):
        """The self encoder's first Linear of one tower on the full observation rows (QuadMultiEncoder.forward's l0
        hook), its weight gradient on the matrix cores (_SelfLayer0Fn).  obs: the minibatch [B, obs_dim] (inside the
        split-f16 range: obs_in_range)."""
        so = self.runner.so
        if lin.out_features not in (128, 256) or so > 32:   # the kernel's shapes; else torch
            return lin(obs[:, :so])
        return _SelfLayer0Fn.apply(obs.contiguous(), lin.weight, lin.bias, so)

    def obs_in_range(self, obs):
        """True when every value of `obs` (e.g. the whole rollout storage, once per update) is inside the split-f16
        range of layer 0 (|obs| < 4094: s = 16, f16 max 65504).  Beyond it the x3 split packs +-inf and the
        gradients become NaN; PPOTrainer then runs that update's encoders on the torch autograd path.  Non-finite
        values are left to the env's non-finite guard.  One host sync."""
        v = float(obs.abs().amax())
        ok = not (v == v and v != float("inf") and v * X3_SIN >= F16_MAX)
        if not ok:
            self._warn(f"an observation reached |obs| = {v:.4g} >= {F16_MAX / X3_SIN:.4g}")
        return ok

    def _warn(self, why):
        import warnings
        warnings.warn(f"fused x3 update: {why}, beyond the split-f16 range; this update's encoders run in torch fp32")

    def encodings(self, obs):
        """Both towers' encoder outputs, or None (the caller's torch autograd path) when a weight left the split-f16
        range (|w| >= 255.9: pack_mfma_weight_x3 refuses it before any kernel runs), as FusedRolloutPolicy.refresh
        falls back to fp32 for the rollout."""
        assert obs.is_cuda and obs.dtype == torch.float32 and obs.dim() == 2
        try:
            return list(_AttnTrainFn.apply(self.runner, obs.contiguous(), *self.params()))
        except ValueError as e:
            self._warn(str(e))
            return None
