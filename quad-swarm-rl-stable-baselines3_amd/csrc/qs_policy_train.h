// qs_policy_train.h -- the PPO update's attention neighbour encoder on the split-f16 matrix cores: the forward with
// the activations the backward needs saved, and the backward's two row-block chains (the update side).
//
// QuadNeighborhoodEncoderAttention (swarm_rl/models/quad_multi_model.py:44-101) as qs_policy.h writes it, per
// neighbour row j (row j = agent j / K, neighbour j % K; self / e_mean of agent j % B -- the reference's pairing):
//   e1 = tanh(x0_j W_e1^T + b_e1)        x0_j = [nbr_j | self_{j % B}]
//   e2 = tanh(e1 W_e2^T + b_e2)          e_mean[a] = mean_k e2[a K + k]
//   a1 = tanh(e2 A_e^T + P[j % B])       P = e_mean A_m^T + b_a1
//   a2 = tanh(a1 W_a2^T + b_a2)          score = a2 . w3 + b3,  w = softmax over the agent's K rows
//   v1 = tanh(e2 W_v1^T + b_v1),  h = tanh(v1 W_v2^T + b_v2),  out[a] = sum_k w h
// Backward, with dout = dL/d out [B, H] (t' = 1 - t^2 the tanh derivative at the saved output t):
//   dh_pre  = w_j dout[a] h'                        dw_j = h_j . dout[a]
//   dv1_pre = (dh_pre W_v2) v1'                     dscore_j = w_j (dw_j - sum_k w_k dw_k)
//   da2_pre = dscore_j w3 a2'                       da1_pre = (da2_pre W_a2) a1'
//   de2p    = dv1_pre W_v1 + da1_pre A_e            (kernel 1: attn_bwd1_x3_kernel)
//   dP[b]   = sum_{j % B = b} da1_pre_j,  dem = dP A_m                       (torch, [B, H])
//   de2_pre = (de2p + dem[j / K] / K) e2'           de1_pre = (de2_pre W_e2) e1'   (kernel 2: attn_bwd2_x3_kernel)
// and the weight gradients as GEMMs over the rows of the saved pairs (dW_v2 = dh_pre^T v1, ...; torch / hipBLASLt).
//
// Every contraction is mfma_layer_x3 (qs_policy_x3.h: x = (hi + lo) / s, three f16 products per fp32 product, fp32
// accumulation).  The backward's tiles hold gradients, whose magnitudes are not bounded like tanh outputs: each
// row gets its own power-of-two scale s_i (its max |x| into [2^13, 2^14) -- exact, the products come back divided by
// s_i), the row maxima reduced over the wave (rows staged from HBM: a row is one wave's 64 lanes) or over the four
// waves through LDS (rows staged from the accumulators, in the barrier every layer has anyway).  The weights' range
// is checked by the packer (policy_fused.pack_mfma_weight_x3).  Block geometry, row pairing and packing as in
// qs_policy.h / qs_policy_x3.h; the W^T operands of the backward GEMMs are packed like any weight (of W^T).
#pragma once
#include <type_traits>

#include "qs_policy_x3.h"

namespace qs {
namespace pol {

#ifndef QS_BWD1_BR2
#define QS_BWD1_BR2 8   // rows per batch of bwd1's second staging (de2p's value part is live: 64 VGPRs)
#endif

struct Trains {
    qs_attn_train t[QS_ATTN_MAX_TOWERS];
};

// power-of-two scale of a row with max |x| = mx: s mx in [2^13, 2^14) (1 for an all-zero or non-finite row)
__device__ __forceinline__ float row_scale(float mx) {
    if (!(mx > 0.f) || !(mx <= 3.0e38f)) return 1.f;
    return __builtin_amdgcn_ldexpf(1.f, 14 - __builtin_amdgcn_frexp_expf(mx));
}
// wave reductions (every lane active): DPP inside each 16-lane row (quad swaps, then row rotations by 4 and 8), then
// the four rows' lane-0 values through readlane -- no LDS round trips (a __shfl_xor butterfly is six ds_bpermute)
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float rdl(float v, int l) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}
__device__ __forceinline__ float wave_sum(float v) {
    v += dppf<0xB1>(v);    // quad_perm [1, 0, 3, 2]
    v += dppf<0x4E>(v);    // quad_perm [2, 3, 0, 1]
    v += dppf<0x124>(v);   // row_ror 4
    v += dppf<0x128>(v);   // row_ror 8
    return (rdl(v, 0) + rdl(v, 16)) + (rdl(v, 32) + rdl(v, 48));
}
__device__ __forceinline__ float wave_max(float v) {
    v = fmaxf(v, dppf<0xB1>(v));
    v = fmaxf(v, dppf<0x4E>(v));
    v = fmaxf(v, dppf<0x124>(v));
    v = fmaxf(v, dppf<0x128>(v));
    return fmaxf(fmaxf(rdl(v, 0), rdl(v, 16)), fmaxf(rdl(v, 32), rdl(v, 48)));
}
__device__ __forceinline__ float4 ld4g(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4g(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
__device__ __forceinline__ float absmax4(float4 v) { return fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))); }
__device__ __forceinline__ float4 f4_scale(float4 v, float s) { return make_float4(s * v.x, s * v.y, s * v.z, s * v.w); }
__device__ __forceinline__ float4 f4_dtanh(float4 g, float4 t) {   // g (1 - t^2)
    return make_float4(g.x * (1.f - t.x * t.x), g.y * (1.f - t.y * t.y), g.z * (1.f - t.z * t.z), g.w * (1.f - t.w * t.w));
}

// column maxima of the gradients (qs_attn_train.colmax, dW's column scales): running max |x| (+inf once an x is not
// finite); every block writes its own row of maxima (plain stores: atomics from every block to the same H addresses
// serialise -- measured 2.6x slower backward kernels), the host takes the max over the blocks
__device__ __forceinline__ float absmax_acc(float m, float x) {
    const float a = fabsf(x);
    return a <= 3.4028235e38f ? fmaxf(m, a) : __builtin_inff();
}
__device__ __forceinline__ float4 absmax_acc4(float4 m, float4 v) {
    return make_float4(absmax_acc(m.x, v.x), absmax_acc(m.y, v.y), absmax_acc(m.z, v.z), absmax_acc(m.w, v.w));
}
__device__ __forceinline__ float4 max4(float4 a, float4 b) {
    return make_float4(fmaxf(a.x, b.x), fmaxf(a.y, b.y), fmaxf(a.z, b.z), fmaxf(a.w, b.w));
}
// accumulator-layout maxima m[c][g] (column acc_n0(wave, c, g, lane) + j over the lane's rows) -> the block's maxima of
// the wave's columns in dst[n]: over the 16 lanes of each lane row by DPP, then rows 0 + 1 and 2 + 3 (row_bcast 15:
// lanes 16 and 48 hold the 32 rows of their column sets), stored by those two lanes
template <int H>
__device__ __forceinline__ void colmax_store_acc(float* dst, float4 (&m)[Geo<H>::CT][4], int wave, int lane) {
#pragma unroll
    for (int c = 0; c < Geo<H>::CT; ++c)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            float v[4] = {m[c][g].x, m[c][g].y, m[c][g].z, m[c][g].w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                v[j] = fmaxf(v[j], dppf<0xB1>(v[j]));
                v[j] = fmaxf(v[j], dppf<0x4E>(v[j]));
                v[j] = fmaxf(v[j], dppf<0x124>(v[j]));
                v[j] = fmaxf(v[j], dppf<0x128>(v[j]));
                const int b = __builtin_bit_cast(int, v[j]);
                v[j] = fmaxf(v[j], __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(b, b, 0x142, 0xA, 0xF, false)));
            }
            if (lane == 16 || lane == 48) {
                const int n0 = acc_n0<H>(wave, c, g, lane);
#pragma unroll
                for (int j = 0; j < 4; ++j) dst[n0 + j] = v[j];
            }
        }
}
struct NoStat {
    template <typename A>
    __device__ void operator()(int, float4, const A&) const {}
};

// Rows staged from HBM: wave w takes rows w, w + 4, ...; lane l < H/4 the row's columns 4l .. 4l+3, BR rows at a time:
// ld(r, c4) -> the row's HBM operands (unconditional loads: an unused row reads the block's first row), issued for
// all BR rows before any is used, so a batch waits out one memory latency, not BR (a load behind a per-row branch, or
// behind the previous row's stores, waits for everything in flight); val(r, c4, on, aux) -> the row's float4 (0 for
// unused rows), called by every lane of the wave (it may reduce over the wave) with on = the lane holds columns (c4 is
// clamped for the others, whose value is dropped); sink(r, c4, v) sees the lane's value (e.g. stores it); the tile
// gets s_r v and RS[r] = 1 / s_r; stat(r, v, aux) sees every row's value (e.g. accumulates column statistics).
template <int H, int BR, typename Ld, typename Val, typename Sink, typename Stat = NoStat>
__device__ __forceinline__ void stage_rows_scaled(const TileX3& X, float* RS, int wave, int lane, Ld ld, Val val, Sink sink,
                                                  Stat stat = NoStat()) {
    constexpr int L4 = H / 4;
    static_assert((MROWS / NWAVE) % BR == 0, "whole batches of rows per wave");
    const bool on = lane < L4;
    const int c4 = on ? lane : 0;
    for (int r0 = wave; r0 < MROWS; r0 += NWAVE * BR) {
        decltype(ld(0, 0)) aux[BR];
#pragma unroll
        for (int u = 0; u < BR; ++u) aux[u] = ld(r0 + u * NWAVE, c4);
        float4 v[BR];
        float m[BR];
#pragma unroll
        for (int u = 0; u < BR; ++u) {
            v[u] = val(r0 + u * NWAVE, c4, on, aux[u]);
            if (!on) v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
            stat(r0 + u * NWAVE, v[u], aux[u]);
            m[u] = absmax4(v[u]);
        }
#pragma unroll
        for (int u = 0; u < BR; ++u) m[u] = wave_max(m[u]);
#pragma unroll
        for (int u = 0; u < BR; ++u) {
            const int r = r0 + u * NWAVE;
            if (on) sink(r, lane, v[u]);
            const float s = row_scale(m[u]);
            if (on) X.put4(r, 4 * lane, f4_scale(v[u], s));
            if (lane == 0) RS[r] = 1.f / s;
        }
    }
}

// the HBM values [RT][CT][4] of a row-major [R, H] array at the lane's accumulator positions (rows of unused tile
// slots read the block's first row), all loads issued back to back
template <int H, typename Ok>
__device__ __forceinline__ void load_acc_rows(const float* __restrict__ src, long row0, Ok okrow, int wave, int lane,
                                             float4 (&v)[RT][Geo<H>::CT][4]) {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
        const int i = acc_i(rt, lane);
        const float* p = src + (row0 + (okrow(i) ? i : 0)) * H;
#pragma unroll
        for (int c = 0; c < Geo<H>::CT; ++c)
#pragma unroll
            for (int g = 0; g < 4; ++g) v[rt][c][g] = ld4g(p + acc_n0<H>(wave, c, g, lane));
    }
}

// Rows staged from a layer's accumulators (acc -> y in place by f(i, n0, acc4, aux4) -> float4, aux: the HBM operand
// at the same positions, loaded by the caller with load_acc_rows): per-row max over the four waves through RMX, then
// the scaled tile.  Contains the barrier between the layer's last tile read and the tile's overwrite.  RS[i] (read by
// f) is replaced by the new row's 1 / s.
template <int H, typename F>
__device__ __forceinline__ void stage_acc_scaled(const TileX3& X, f32x16 (&acc)[RT][Geo<H>::CT], float* RS, float* RMX,
                                                 int wave, int lane, const float4 (&aux)[RT][Geo<H>::CT][4], F f,
                                                 float4 (&cm)[Geo<H>::CT][4]) {
    constexpr int CT = Geo<H>::CT;
#pragma unroll
    for (int c = 0; c < CT; ++c)
#pragma unroll
        for (int g = 0; g < 4; ++g) cm[c][g] = make_float4(0.f, 0.f, 0.f, 0.f);
    float mx[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
        const int i = acc_i(rt, lane);
        float m = 0.f;
#pragma unroll
        for (int c = 0; c < CT; ++c)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const float4 y = f(i, acc_n0<H>(wave, c, g, lane), acc4(acc[rt][c], g), aux[rt][c][g]);
                cm[c][g] = absmax_acc4(cm[c][g], y);
                acc[rt][c][4 * g] = y.x; acc[rt][c][4 * g + 1] = y.y;
                acc[rt][c][4 * g + 2] = y.z; acc[rt][c][4 * g + 3] = y.w;
                m = fmaxf(m, absmax4(y));
            }
        mx[rt] = fmaxf(m, __shfl_xor(m, 32));
    }
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
        if (lane < 32) RMX[wave * MROWS + acc_i(rt, lane)] = mx[rt];
    __syncthreads();   // every wave has read the tile (and RS), RMX complete
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
        const int i = acc_i(rt, lane);
        const float m = fmaxf(fmaxf(RMX[i], RMX[MROWS + i]), fmaxf(RMX[2 * MROWS + i], RMX[3 * MROWS + i]));
        const float s = row_scale(m);
#pragma unroll
        for (int c = 0; c < CT; ++c)
#pragma unroll
            for (int g = 0; g < 4; ++g) X.put4(i, acc_n0<H>(wave, c, g, lane), f4_scale(acc4(acc[rt][c], g), s));
        if (wave == 0 && lane < 32) RS[i] = 1.f / s;
    }
}

// ------------------------------------------------------------------------------------------------------------------
// forward with saves: attn_embed_x3_kernel + e1; attn_pool_x3_kernel + a1, a2, v1, h, w (qs_policy_x3.h, same math)
// ------------------------------------------------------------------------------------------------------------------
template <int H>
__global__ __launch_bounds__(NTHR, 2) __attribute__((amdgpu_waves_per_eu(2, 2))) void attn_embed_train_x3_kernel(
    const float* __restrict__ obs, int stride, int so, int off, int B, int K, int nd, Towers tw, Trains trs) {
    constexpr int LDH = GeoX3<H>::LDH, LD0 = GeoX3<KD0>::LDH, CT = Geo<H>::CT;
    extern __shared__ float4 smem4[];
    _Float16* xh = reinterpret_cast<_Float16*>(smem4);
    const TileX3 X{xh, xh + MROWS * LDH, LDH};
    const TileX3 X0{xh + 2 * MROWS * LDH, xh + 2 * MROWS * LDH + MROWS * LD0, LD0};
    float* BI = reinterpret_cast<float*>(xh + 2 * MROWS * LDH + 2 * MROWS * LD0);
    const qs_attn_tower& t = tw.t[blockIdx.y];
    const qs_attn_train& tr = trs.t[blockIdx.y];
    const int AB = MROWS / K, MU = AB * K;
    const long R = (long)B * K, row0 = (long)blockIdx.x * MU;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    QS_STAMP_DECL
    QS_RTSTAMP(12);
    QS_STAMP(0);
    for (int n = tid; n < H; n += NTHR) {
        BI[n] = t.b_e1[n];
        BI[H + n] = t.b_e2[n];
    }
    gather_rows0(obs, stride, so, off, B, K, nd, row0, MU, R, tid, [&](int r, int c, float v) { X0.put(r, c, X3_SIN * v); });
    __syncthreads();
    QS_STAMP(1);
    f32x16 acc[RT][CT];
    mfma_layer_x3<H, KD0, true, false>(X0, reinterpret_cast<const uint4*>(t.w_e1p), acc, wave, lane);
    QS_STAMP(2);
    const auto qe2 = mfma_prefetch_x3<H>(reinterpret_cast<const uint4*>(t.w_e2p), wave, lane);   // ahead of e1's stores
    store_tanh_x3<H>(X, acc, 1.f / (X3_SIN * X3_SW), wave, lane,
                     [&](int i, int n0) {
                         return (i < MU && row0 + i < R) ? lds4(BI + n0) : make_float4(0.f, 0.f, 0.f, 0.f);
                     },
                     [&](int i, int n0, float4 y) {
                         if (i < MU && row0 + i < R) st4g(tr.e1 + (row0 + i) * H + n0, y);
                     });
    __syncthreads();
    QS_STAMP(3);
    mfma_layer_x3<H, H, true, QS_EMBED_PIN != 0>(X, reinterpret_cast<const uint4*>(t.w_e2p), acc, wave, lane, qe2);
    __syncthreads();
    QS_STAMP(4);
    embed_e2_epilogue<H>(acc, BI + H, t.e2, t.e_mean, smem4, row0, MU, R, B, K, AB, wave, lane, tid);
    QS_STAMP(5);
    QS_STAMP(6);
    QS_RTSTAMP(13);
    if (blockIdx.y == 0) QS_STAMP_FLUSH();
}


template <int H>
__global__ __launch_bounds__(NTHR, 2) __attribute__((amdgpu_waves_per_eu(2, 2))) void attn_pool_train_x3_kernel(
    int B, int K, Towers tw, Trains trs) {
    constexpr int LDH = GeoX3<H>::LDH, CT = Geo<H>::CT;
    extern __shared__ float4 smem4[];
    _Float16* xh = reinterpret_cast<_Float16*>(smem4);
    const TileX3 X{xh, xh + MROWS * LDH, LDH};
    float* SC = reinterpret_cast<float*>(xh + 2 * MROWS * LDH);
    float* WT = SC + MROWS;
    float* A3 = WT + 2 * MROWS;
    const qs_attn_tower& t = tw.t[blockIdx.y];
    const qs_attn_train& tr = trs.t[blockIdx.y];
    const int AB = MROWS / K, MU = AB * K;
    const long R = (long)B * K, row0 = (long)blockIdx.x * MU;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    constexpr float SS = X3_SX * X3_SW, iSS = 1.f / SS;
    QS_STAMP_DECL
    QS_RTSTAMP(12);
    QS_STAMP(0);
    for (int n = tid; n < H; n += NTHR) {
        A3[n] = t.w_a3[n];
        A3[H + n] = t.b_a2[n];
        A3[2 * H + n] = t.b_v1[n];
        A3[3 * H + n] = t.b_v2[n];
    }
    auto okrow = [&](int i) { return i < MU && row0 + i < R; };
    f32x16 acc[RT][CT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
        const int i = acc_i(rt, lane);
        const int j = (int)row0 + i;
        const float okf = okrow(i) ? 1.f : 0.f;
        const float* pr = t.P + (size_t)(okrow(i) ? j % B : 0) * H;
#pragma unroll
        for (int c = 0; c < CT; ++c)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                float4 v = *reinterpret_cast<const float4*>(pr + acc_n0<H>(wave, c, g, lane));
                v = make_float4(v.x * okf, v.y * okf, v.z * okf, v.w * okf);
                acc[rt][c][4 * g] = SS * v.x; acc[rt][c][4 * g + 1] = SS * v.y;
                acc[rt][c][4 * g + 2] = SS * v.z; acc[rt][c][4 * g + 3] = SS * v.w;
            }
    }
    load_rows_x3<H>(X, t.e2, row0, MU, R, tid);
    __syncthreads();
    QS_STAMP(1);
    mfma_layer_x3<H, H, false>(X, reinterpret_cast<const uint4*>(t.w_a1ep), acc, wave, lane);
#if QS_POOL_V1_EARLY
    f32x16 accv[RT][CT];   // neighbor_value_mlp's first layer on the same e2 tile (attn_pool_x3_kernel)
    mfma_layer_x3<H>(X, reinterpret_cast<const uint4*>(t.w_v1p), accv, wave, lane);
#endif
    __syncthreads();
    QS_STAMP(2);
    store_tanh_x3<H>(X, acc, iSS, wave, lane, ZeroInit(), [&](int i, int n0, float4 y) {
        if (okrow(i)) st4g(tr.a1 + (row0 + i) * H + n0, y);
    });
    __syncthreads();
    QS_STAMP(3);
    mfma_layer_x3<H>(X, reinterpret_cast<const uint4*>(t.w_a2p), acc, wave, lane);
    QS_STAMP(4);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {   // a2 (the rollout kernel keeps it in the score's registers only)
        const int i = acc_i(rt, lane);
        if (!okrow(i)) continue;
#pragma unroll
        for (int c = 0; c < CT; ++c)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int n0 = acc_n0<H>(wave, c, g, lane);
                const float4 b = lds4(A3 + H + n0);
                st4g(tr.a2 + (row0 + i) * H + n0,
                     make_float4(tanh_fast(fmaf(acc[rt][c][4 * g], iSS, b.x)), tanh_fast(fmaf(acc[rt][c][4 * g + 1], iSS, b.y)),
                                 tanh_fast(fmaf(acc[rt][c][4 * g + 2], iSS, b.z)), tanh_fast(fmaf(acc[rt][c][4 * g + 3], iSS, b.w))));
            }
    }
    float* SCP = A3 + 4 * H;
    score_partials<H>(acc, iSS, A3, A3 + H, SCP, wave, lane);
    __syncthreads();
    QS_STAMP(5);
    if (tid < MROWS) SC[tid] = ((SCP[tid] + SCP[MROWS + tid]) + (SCP[2 * MROWS + tid] + SCP[3 * MROWS + tid])) + t.b_a3;
    __syncthreads();
    if (tid < AB) {
        const int base = tid * K;
        float m = SC[base];
        for (int k = 1; k < K; ++k) m = fmaxf(m, SC[base + k]);
        float s = 0.f;
        for (int k = 0; k < K; ++k) {
            const float x = expf(SC[base + k] - m);
            WT[base + k] = x;
            s += x;
        }
        for (int k = 0; k < K; ++k) WT[base + k] = WT[base + k] / s;
    }
#if QS_POOL_V1_EARLY
    __syncthreads();   // WT complete (the tile is free since the score barrier)
    if (tid < MU && row0 + tid < R) tr.w[row0 + tid] = WT[tid];
    QS_STAMP(6);
    QS_STAMP(7);
    store_tanh_x3<H>(X, accv, iSS, wave, lane, [&](int, int n0) { return lds4(A3 + 2 * H + n0); },
                     [&](int i, int n0, float4 y) {
                         if (okrow(i)) st4g(tr.v1 + (row0 + i) * H + n0, y);
                     });
    __syncthreads();
#else
    load_rows_x3<H>(X, t.e2, row0, MU, R, tid);
    __syncthreads();
    if (tid < MU && row0 + tid < R) tr.w[row0 + tid] = WT[tid];
    QS_STAMP(6);
    mfma_layer_x3<H>(X, reinterpret_cast<const uint4*>(t.w_v1p), acc, wave, lane);
    __syncthreads();
    QS_STAMP(7);
    store_tanh_x3<H>(X, acc, iSS, wave, lane, [&](int, int n0) { return lds4(A3 + 2 * H + n0); },
                     [&](int i, int n0, float4 y) {
                         if (okrow(i)) st4g(tr.v1 + (row0 + i) * H + n0, y);
                     });
    __syncthreads();
#endif
    QS_STAMP(8);
    mfma_layer_x3<H>(X, reinterpret_cast<const uint4*>(t.w_v2p), acc, wave, lane);
    __syncthreads();
    QS_STAMP(9);
    float* Y = reinterpret_cast<float*>(smem4);
    constexpr int LDY = H + 4;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
        const int i = acc_i(rt, lane);
        const float wi = i < MU ? WT[i] : 0.f;
#pragma unroll
        for (int c = 0; c < CT; ++c)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int n0 = acc_n0<H>(wave, c, g, lane);
                const float4 b = lds4(A3 + 3 * H + n0);
                const float4 h = make_float4(tanh_fast(fmaf(acc[rt][c][4 * g], iSS, b.x)), tanh_fast(fmaf(acc[rt][c][4 * g + 1], iSS, b.y)),
                                             tanh_fast(fmaf(acc[rt][c][4 * g + 2], iSS, b.z)), tanh_fast(fmaf(acc[rt][c][4 * g + 3], iSS, b.w)));
                if (okrow(i)) st4g(tr.h + (row0 + i) * H + n0, h);
                *reinterpret_cast<float4*>(Y + i * LDY + n0) = make_float4(wi * h.x, wi * h.y, wi * h.z, wi * h.w);
            }
    }
    __syncthreads();
    QS_STAMP(10);
    for (int e = tid; e < AB * H; e += NTHR) {   // (float4-wide as the rollout kernel: 4 spilled registers here)
        const int a = e / H, n = e - a * H;
        const long agent = row0 / K + a;
        if (agent < B) {
            float s = 0.f;
            for (int k = 0; k < K; ++k) s += Y[(a * K + k) * LDY + n];
            t.out[agent * H + n] = s;
        }
    }
    QS_STAMP(11);
    QS_RTSTAMP(13);
    if (blockIdx.y == 0) QS_STAMP_FLUSH();
}


// ------------------------------------------------------------------------------------------------------------------
// backward
// ------------------------------------------------------------------------------------------------------------------
template <int H>
constexpr size_t bwd_fixed_lds_bytes() {   // split tile + WT, DW, SC, RS (MROWS each) + RMX (4 MROWS) + w3 (H)
    return (size_t)(2 * MROWS * GeoX3<H>::LDH) * 2 + (size_t)(8 * MROWS + H) * 4;
}

// kernel 1: value chain (dh_pre -> dv1_pre -> de2 part) and attention chain (dscore -> da2_pre -> da1_pre -> de2 part);
// dynamic LDS: bwd_fixed_lds_bytes<H>() + max(MROWS / K, 2 NWAVE) H floats (the block's dout rows, then the column
// statistics' scratch); kernel 2: bwd_fixed_lds_bytes<H>() + NWAVE H floats
template <int H>
constexpr size_t bwd1_lds_bytes(int K) {
    return bwd_fixed_lds_bytes<H>() + (size_t)(MROWS / K > 2 * NWAVE ? MROWS / K : 2 * NWAVE) * H * 4;
}
template <int H>
constexpr size_t bwd2_lds_bytes() { return bwd_fixed_lds_bytes<H>() + (size_t)NWAVE * H * 4; }
template <int H>
__global__ __launch_bounds__(NTHR, 2) void attn_bwd1_x3_kernel(int B, int K, Towers tw, Trains trs) {
    constexpr int LDH = GeoX3<H>::LDH, CT = Geo<H>::CT, L4 = H / 4;
    extern __shared__ float4 smem4[];
    _Float16* xh = reinterpret_cast<_Float16*>(smem4);
    const TileX3 X{xh, xh + MROWS * LDH, LDH};
    float* WT = reinterpret_cast<float*>(xh + 2 * MROWS * LDH);
    float* DW = WT + MROWS;
    float* SC = DW + MROWS;
    float* RS = SC + MROWS;
    float* RMX = RS + MROWS;
    float* W3 = RMX + NWAVE * MROWS;
    float* DO = W3 + H;   // [max(AB, 8) H]: the block's dout rows (stage 1), then the column statistics' scratch
    const qs_attn_tower& t = tw.t[blockIdx.y];
    const qs_attn_train& tr = trs.t[blockIdx.y];
    const int AB = MROWS / K, MU = AB * K;
    const long R = (long)B * K, row0 = (long)blockIdx.x * MU, a0 = row0 / K;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    auto okrow = [&](int i) { return i < MU && row0 + i < R; };
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    QS_STAMP_DECL
    QS_RTSTAMP(12);
    QS_STAMP(0);
    for (int e = tid; e < AB * L4; e += NTHR) {
        const int a = e / L4, c4 = e - a * L4;
        reinterpret_cast<float4*>(DO)[e] = (a0 + a < B) ? ld4g(tr.dout + (a0 + a) * H + 4 * c4) : z4;
    }
    for (int n = tid; n < H; n += NTHR) W3[n] = t.w_a3[n];
    if (tid < MROWS) WT[tid] = okrow(tid) ? tr.w[row0 + tid] : 0.f;
    __syncthreads();
    QS_STAMP(1);
    float4 cmr = z4, aw = z4;   // column maxima / sum dscore a2 of the lane's columns over the wave's rows
    // dw_j = h_j . dout[a] and dh_pre = w_j dout[a] (1 - h^2): wave-owned rows
    auto rowp = [&](const float* a, int r, int c4) { return a + (row0 + (okrow(r) ? r : 0)) * H + 4 * c4; };
    stage_rows_scaled<H, MROWS / NWAVE>(X, RS, wave, lane, [&](int r, int c4) { return ld4g(rowp(tr.h, r, c4)); },
                         [&](int r, int c4, bool on, float4 h) {
                             if (!okrow(r)) return z4;
                             const float4 d = lds4(DO + (r / K) * H + 4 * c4);
                             const float dw = wave_sum(on ? h.x * d.x + h.y * d.y + h.z * d.z + h.w * d.w : 0.f);
                             if (lane == 0) DW[r] = dw;
                             return f4_dtanh(f4_scale(d, WT[r]), h);
                         },
                         [&](int r, int c4, float4 v) {
                             if (okrow(r)) st4g(tr.dh_pre + (row0 + r) * H + 4 * c4, v);
                         },
                         [&](int, float4 v, const float4&) { cmr = absmax_acc4(cmr, v); });
    __syncthreads();
    // the waves' column maxima of dh_pre into the scratch (dout is no longer read); merged after the next barrier
    if (lane < L4) *reinterpret_cast<float4*>(DO + wave * H + 4 * lane) = cmr;
    QS_STAMP(2);
    const size_t nblk = gridDim.x;
    auto cm_row = [&](int k) { return tr.colmax + ((size_t)k * nblk + blockIdx.x) * H; };
    f32x16 acc[RT][CT];
    constexpr float iSW = 1.f / X3_SW;
    // dv1_pre = (dh_pre W_v2) (1 - v1^2)
    float4 aux[RT][CT][4];
    load_acc_rows<H>(tr.v1, row0, okrow, wave, lane, aux);   // in flight during the layer's MFMAs
    mfma_layer_x3<H>(X, reinterpret_cast<const uint4*>(tr.w_v2tp), acc, wave, lane);
    QS_STAMP(3);
    float4 cma[CT][4];
    stage_acc_scaled<H>(X, acc, RS, RMX, wave, lane, aux, [&](int i, int n0, float4 a, float4 v1) {
        if (!okrow(i)) return z4;
        const float4 y = f4_dtanh(f4_scale(a, RS[i] * iSW), v1);
        st4g(tr.dv1_pre + (row0 + i) * H + n0, y);
        return y;
    }, cma);
    if (tr.colmax) {
        colmax_store_acc<H>(cm_row(1), cma, wave, lane);
        for (int n = tid; n < H; n += NTHR)
            cm_row(0)[n] = fmaxf(fmaxf(DO[n], DO[H + n]), fmaxf(DO[2 * H + n], DO[3 * H + n]));
    }
    __syncthreads();
    // de2p = dv1_pre W_v1 + (the attention chain's part, below): the value part stays in registers until then, so
    // de2p is written once (a store, reload and store of 1.6 GB per tower before)
    QS_STAMP(4);
    mfma_layer_x3<H>(X, reinterpret_cast<const uint4*>(tr.w_v1tp), acc, wave, lane);
    f32x16 dev[RT][CT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
        const float sc = RS[acc_i(rt, lane)] * iSW;
#pragma unroll
        for (int c = 0; c < CT; ++c)
#pragma unroll
            for (int r = 0; r < 16; ++r) dev[rt][c][r] = acc[rt][c][r] * sc;
    }
    // dscore_j = w_j (dw_j - sum_k w_k dw_k) over the agent's K rows
    if (tid < MROWS) {
        float s = 0.f;
        if (tid < MU) {
            const int base = (tid / K) * K;
            for (int k = 0; k < K; ++k) s += WT[base + k] * DW[base + k];
        }
        const float ds = okrow(tid) ? WT[tid] * (DW[tid] - s) : 0.f;
        SC[tid] = ds;
        if (okrow(tid)) tr.dscore[row0 + tid] = ds;
    }
    QS_STAMP(5);
    __syncthreads();   // SC complete; every wave has read the tile and RS
    QS_STAMP(6);
    cmr = z4;
    // da2_pre = dscore_j w3 (1 - a2^2)
    stage_rows_scaled<H, QS_BWD1_BR2>(X, RS, wave, lane, [&](int r, int c4) { return ld4g(rowp(tr.a2, r, c4)); },
                         [&](int r, int c4, bool, float4 a2) {
                             if (!okrow(r)) return z4;
                             return f4_dtanh(f4_scale(lds4(W3 + 4 * c4), SC[r]), a2);
                         },
                         [&](int r, int c4, float4 v) {
                             if (okrow(r)) st4g(tr.da2_pre + (row0 + r) * H + 4 * c4, v);
                         },
                         [&](int r, float4 v, const float4& a2) {
                             cmr = absmax_acc4(cmr, v);
                             aw = f4_add(aw, f4_scale(a2, SC[r]));   // SC = 0 on unused rows
                         });
    if (lane < L4) {   // the scratch was last read before the dscore barrier
        *reinterpret_cast<float4*>(DO + wave * H + 4 * lane) = cmr;
        *reinterpret_cast<float4*>(DO + (NWAVE + wave) * H + 4 * lane) = aw;
    }
    __syncthreads();
    // da1_pre = (da2_pre W_a2) (1 - a1^2)
    QS_STAMP(7);
    mfma_layer_x3<H>(X, reinterpret_cast<const uint4*>(tr.w_a2tp), acc, wave, lane);
    QS_STAMP(8);
    load_acc_rows<H>(tr.a1, row0, okrow, wave, lane, aux);   // after the layer (de2p's value part holds 64 VGPRs)
    stage_acc_scaled<H>(X, acc, RS, RMX, wave, lane, aux, [&](int i, int n0, float4 a, float4 a1) {
        if (!okrow(i)) return z4;
        const float4 y = f4_dtanh(f4_scale(a, RS[i] * iSW), a1);
        st4g(tr.da1_pre + (row0 + i) * H + n0, y);
        return y;
    }, cma);
    if (tr.colmax) {
        colmax_store_acc<H>(cm_row(3), cma, wave, lane);
        for (int n = tid; n < H; n += NTHR)
            cm_row(2)[n] = fmaxf(fmaxf(DO[n], DO[H + n]), fmaxf(DO[2 * H + n], DO[3 * H + n]));
    }
    if (tr.a3w_part)
        for (int n = tid; n < H; n += NTHR)
            tr.a3w_part[(size_t)blockIdx.x * H + n] =
                (DO[NWAVE * H + n] + DO[(NWAVE + 1) * H + n]) + (DO[(NWAVE + 2) * H + n] + DO[(NWAVE + 3) * H + n]);
    __syncthreads();
    // de2p += da1_pre A_e
    QS_STAMP(9);
    mfma_layer_x3<H>(X, reinterpret_cast<const uint4*>(tr.w_a1etp), acc, wave, lane);
    QS_STAMP(10);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
        const int i = acc_i(rt, lane);
        if (!okrow(i)) continue;
        const float sc = RS[i] * iSW;
#pragma unroll
        for (int c = 0; c < CT; ++c)
#pragma unroll
            for (int g = 0; g < 4; ++g)
                st4g(tr.de2p + (row0 + i) * H + acc_n0<H>(wave, c, g, lane),
                     f4_add(acc4(dev[rt][c], g), f4_scale(acc4(acc[rt][c], g), sc)));
    }
    QS_STAMP(11);
    QS_RTSTAMP(13);
    if (blockIdx.y == 0) QS_STAMP_FLUSH();
}


// kernel 2: de2_pre = (de2p + dem[j / K] / K) (1 - e2^2) -> de1_pre = (de2_pre W_e2) (1 - e1^2)
template <int H>
__global__ __launch_bounds__(NTHR, 2) void attn_bwd2_x3_kernel(int B, int K, Towers tw, Trains trs) {
    constexpr int LDH = GeoX3<H>::LDH, CT = Geo<H>::CT;
    extern __shared__ float4 smem4[];
    _Float16* xh = reinterpret_cast<_Float16*>(smem4);
    const TileX3 X{xh, xh + MROWS * LDH, LDH};
    float* RS = reinterpret_cast<float*>(xh + 2 * MROWS * LDH);
    float* RMX = RS + MROWS;
    float* SCR = RMX + NWAVE * MROWS;   // [NWAVE][H] the waves' column maxima of de2_pre
    const qs_attn_tower& t = tw.t[blockIdx.y];
    const qs_attn_train& tr = trs.t[blockIdx.y];
    const int AB = MROWS / K, MU = AB * K;
    const long R = (long)B * K, row0 = (long)blockIdx.x * MU;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    auto okrow = [&](int i) { return i < MU && row0 + i < R; };
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    const float invK = 1.f / (float)K;
    float4 cmr = z4;   // column maxima of de2_pre over the wave's rows
    struct Ops {
        float4 g, m, e;
    };
    stage_rows_scaled<H, 8>(X, RS, wave, lane,
                            [&](int r, int c4) {
                                const long j = row0 + (okrow(r) ? r : 0);
                                return Ops{ld4g(tr.de2p + j * H + 4 * c4), ld4g(tr.dem + (j / K) * H + 4 * c4),
                                           ld4g(t.e2 + j * H + 4 * c4)};
                            },
                            [&](int r, int, bool, const Ops& o) {
                                if (!okrow(r)) return z4;
                                return f4_dtanh(f4_add(o.g, f4_scale(o.m, invK)), o.e);
                            },
                            [&](int r, int c4, float4 v) {
                                if (okrow(r)) st4g(tr.de2_pre + (row0 + r) * H + 4 * c4, v);
                            },
                            [&](int, float4 v, const Ops&) { cmr = absmax_acc4(cmr, v); });
    if (lane < H / 4) *reinterpret_cast<float4*>(SCR + wave * H + 4 * lane) = cmr;
    __syncthreads();
    if (tr.colmax)
        for (int n = tid; n < H; n += NTHR)
            tr.colmax[((size_t)4 * gridDim.x + blockIdx.x) * H + n] =
                fmaxf(fmaxf(SCR[n], SCR[H + n]), fmaxf(SCR[2 * H + n], SCR[3 * H + n]));
    f32x16 acc[RT][CT];
    constexpr float iSW = 1.f / X3_SW;
    float4 e1[RT][CT][4];
    load_acc_rows<H>(tr.e1, row0, okrow, wave, lane, e1);   // in flight during the layer's MFMAs
    mfma_layer_x3<H>(X, reinterpret_cast<const uint4*>(tr.w_e2tp), acc, wave, lane);
    float4 cma[CT][4];
#pragma unroll
    for (int c = 0; c < CT; ++c)
#pragma unroll
        for (int g = 0; g < 4; ++g) cma[c][g] = z4;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
        const int i = acc_i(rt, lane);
        if (!okrow(i)) continue;
        const float sc = RS[i] * iSW;
#pragma unroll
        for (int c = 0; c < CT; ++c)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const float4 y = f4_dtanh(f4_scale(acc4(acc[rt][c], g), sc), e1[rt][c][g]);
                st4g(tr.de1_pre + (row0 + i) * H + acc_n0<H>(wave, c, g, lane), y);
                cma[c][g] = absmax_acc4(cma[c][g], y);
            }
    }
    if (tr.colmax) colmax_store_acc<H>(tr.colmax + ((size_t)5 * gridDim.x + blockIdx.x) * H, cma, wave, lane);
    (void)RMX;
}

}  // namespace pol
}  // namespace qs

namespace qs {
namespace pol {

// ------------------------------------------------------------------------------------------------------------------
// weight gradients: part[b] = G[rows of b]^T A[rows of b] (split-K over the B K rows; torch sums the parts)
// G: [R, H] pre-activation gradients with a power-of-two scale per column (gs[n], |G[:, n]| gs[n] < 2^14: the
// column's scale factors out of dW[n, :]); A: [R, H] tanh outputs (|a| <= 1, scale X3_SX).  Both split into f16
// hi / lo, three MFMAs per product as mfma_layer_x3.  A block's 16-row step: the 16 x H tiles of G and A staged
// TRANSPOSED in LDS ([n][r] / [k][r], 16 r + 8 padding halves per row), so that a lane's MFMA operand -- 8 consecutive
// rows r of one column -- is one ds_read_b128; wave w owns output rows n in [w H/4, (w+1) H/4), all H columns k.
// Staging: thread t owns column t % H and rows (t / H) RPT .. of the step (coalesced 4-byte row loads; its column's
// rows leave as ds_write_b128 at a 48-byte column stride, conflict-free); the next step's rows are loaded into
// registers while the current step's MFMAs run (double-buffered tiles), which are issued product by product over
// all 16 (H = 256) output tiles (no back-to-back dependent MFMAs).
// ------------------------------------------------------------------------------------------------------------------
constexpr int DW_STEP = 16, DW_LDR = DW_STEP + 8;   // rows per step; LDS row stride in halves (48 B)

template <int H>
constexpr size_t dw_lds_bytes() { return (size_t)2 * 4 * H * DW_LDR * 2; }   // 2 buffers x {Gh, Gl, Ah, Al}

#ifndef QS_DW_RING
#define QS_DW_RING 2   // steps of rows in flight in registers ahead of the MFMAs (1: the next step only)
#endif

// threads of a dW block: one wave per 32 output rows n (H = 256: 8 waves, 128 accumulator registers each -- room for
// the two-step register ring; H = 128: 4 waves)
template <int H>
constexpr int dw_threads() { return 64 * (H / 32); }

template <int H>
__global__ __launch_bounds__(dw_threads<H>(), 1) void dw_x3_kernel(const float* __restrict__ G, const float* __restrict__ A,
                                                        const float* __restrict__ gs, long R, int steps_per_block,
                                                        float* __restrict__ part, float* __restrict__ part_sum,
                                                        int ldg, int lda) {
    constexpr int DWT = dw_threads<H>();
    constexpr int NT = 1, KT = H / 32, TPC = DWT / H, RPT = DW_STEP / TPC;   // threads per column, rows each
    constexpr int RING = QS_DW_RING;
    static_assert(RPT % 8 == 0, "a thread's rows leave as whole 8-row (16-byte) groups");
    static_assert(RING == 1 || RING == 2, "one or two steps in flight");
    extern __shared__ float4 smem4[];
    _Float16* lds = reinterpret_cast<_Float16*>(smem4);
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int sc = tid % H, sr = (tid / H) * RPT;   // staging: column, first row of the step
    const long r_begin = (long)blockIdx.x * steps_per_block * DW_STEP;
    auto buf = [&](int b, int which) { return lds + ((size_t)b * 4 + which) * H * DW_LDR; };   // 0 Gh 1 Gl 2 Ah 3 Al
    const float sg = gs[sc];
    // register ring: slot k % RING holds step k's rows from its load until it is staged (statically indexed: the
    // main loop is unrolled by RING)
    float gv[RING][RPT], av[RING][RPT];
    float csum = 0.f;   // the column's sum over the part's rows (the bias gradient's part; rows in order)
    // the block's rows through buffer descriptors (base = its first row, records = its rows that exist): a 32-bit
    // offset per load and the range check's zeros past R, no 64-bit address or select per row
    // (row strides ldg / lda in floats: G and A may be column slices of wider rows)
    const long r_end = r_begin + (long)steps_per_block * DW_STEP < R ? r_begin + (long)steps_per_block * DW_STEP : R;
    const long nrow = r_end > r_begin ? r_end - r_begin : 0;
    const auto rg = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(G + r_begin * ldg), (short)0,
                                                      (int)(nrow * ldg * 4), 0x00020000);
    const auto ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(A + r_begin * lda), (short)0,
                                                      (int)(nrow * lda * 4), 0x00020000);
    const int voffg = (sr * ldg + sc) * 4, voffa = (sr * lda + sc) * 4;
    auto load = [&](auto SL, int s) {
        constexpr int sl = decltype(SL)::value;
        const int sog = s * DW_STEP * ldg * 4, soa = s * DW_STEP * lda * 4;   // (a step past the rows reads zeros)
#pragma unroll
        for (int u = 0; u < RPT; ++u) {
            gv[sl][u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rg, voffg + u * ldg * 4, sog, 0));
            av[sl][u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ra, voffa + u * lda * 4, soa, 0));
        }
    };
    auto stage = [&](auto SL, int b) {
        constexpr int sl = decltype(SL)::value;
#pragma unroll
        for (int o = 0; o < RPT; o += 8) {
            f16x8 gh, gl, ah, al;
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                csum += gv[sl][o + u];
                const float g = sg * gv[sl][o + u], a = X3_SX * av[sl][o + u];
                gh[u] = (_Float16)g;
                gl[u] = (_Float16)(g - (float)gh[u]);
                ah[u] = (_Float16)a;
                al[u] = (_Float16)(a - (float)ah[u]);
            }
            const int off = sc * DW_LDR + sr + o;
            *reinterpret_cast<f16x8*>(buf(b, 0) + off) = gh;
            *reinterpret_cast<f16x8*>(buf(b, 1) + off) = gl;
            *reinterpret_cast<f16x8*>(buf(b, 2) + off) = ah;
            *reinterpret_cast<f16x8*>(buf(b, 3) + off) = al;
        }
    };
    f32x16 acc[NT][KT];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int k = 0; k < KT; ++k)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[t][k][r] = 0.f;
    const int aoff = (lane & 31) * DW_LDR + (lane >> 5) * 8;
    auto mfmas = [&](int b) {
        f16x8 gh[NT], gl[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const int n0 = (wave * NT + t) * 32;
            gh[t] = *reinterpret_cast<const f16x8*>(buf(b, 0) + n0 * DW_LDR + aoff);
            gl[t] = *reinterpret_cast<const f16x8*>(buf(b, 1) + n0 * DW_LDR + aoff);
        }
        // A's columns as the first operand, G's as the second: the result tile is [k][n], i.e. a lane holds output
        // row n = lane & 31 (the layout of the store below; qs_policy.h acc_i / acc_n0).  A's fragments stream one
        // column tile ahead (a 32x32x16 MFMA chain on one accumulator issues at the full rate: no operand hoard)
        f16x8 ahn = *reinterpret_cast<const f16x8*>(buf(b, 2) + aoff);
        f16x8 aln = *reinterpret_cast<const f16x8*>(buf(b, 3) + aoff);
#pragma unroll
        for (int k = 0; k < KT; ++k) {
            const f16x8 ah = ahn, al = aln;
            if (k + 1 < KT) {
                ahn = *reinterpret_cast<const f16x8*>(buf(b, 2) + (k + 1) * 32 * DW_LDR + aoff);
                aln = *reinterpret_cast<const f16x8*>(buf(b, 3) + (k + 1) * 32 * DW_LDR + aoff);
            }
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                acc[t][k] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, gh[t], acc[t][k], 0, 0, 0);
                acc[t][k] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, gl[t], acc[t][k], 0, 0, 0);
                acc[t][k] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, gh[t], acc[t][k], 0, 0, 0);
            }
        }
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, RING - 1>;
    if constexpr (RING == 1) {
        load(I0{}, 0);
        stage(I0{}, 0);
        __syncthreads();
        for (int s = 0; s < steps_per_block; ++s) {
            const int b = s & 1;
            if (s + 1 < steps_per_block) load(I0{}, s + 1);   // next rows in flight during this step's MFMAs
            mfmas(b);
            if (s + 1 < steps_per_block) stage(I0{}, b ^ 1);   // the other buffer: last read two steps ago
            __syncthreads();
        }
    } else {
        // step k's rows: loaded at iteration k - 2 into slot k % 2, staged at iteration k - 1 into LDS buffer k % 2,
        // multiplied at iteration k
        load(I0{}, 0);
        load(I1{}, 1);
        stage(I0{}, 0);
        __syncthreads();
        auto iter = [&](auto SL, int s) {   // SL = s % 2
            constexpr int sl = decltype(SL)::value;
            using Cur = std::integral_constant<int, sl>;
            using Nxt = std::integral_constant<int, sl ^ 1>;
            if (s + 2 < steps_per_block) load(Cur{}, s + 2);   // slot s % 2 was staged last iteration
            mfmas(sl);
            if (s + 1 < steps_per_block) stage(Nxt{}, sl ^ 1);
            __syncthreads();
        };
        for (int s = 0; s < steps_per_block; s += 2) {
            iter(I0{}, s);
            if (s + 1 < steps_per_block) iter(I1{}, s + 1);
        }
    }
    if (part_sum) {   // the TPC threads of a column through LDS (the staging buffers are free after the loop's barrier)
        float* cs = reinterpret_cast<float*>(smem4);
        cs[tid] = csum;
        __syncthreads();
        if (tid < H) {
            float v = cs[tid];
#pragma unroll
            for (int q = 1; q < TPC; ++q) v += cs[q * H + tid];
            part_sum[(size_t)blockIdx.x * H + tid] = v;
        }
    }
    // acc[t][k] register 4g + j: output row n = (wave NT + t) 32 + (lane & 31), column k 32 + 8 g + 4 (lane >> 5) + j
    float* out = part + (size_t)blockIdx.x * H * H;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const int n = (wave * NT + t) * 32 + (lane & 31);
        const float inv = 1.f / (gs[n] * X3_SX);
#pragma unroll
        for (int k = 0; k < KT; ++k)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int col = k * 32 + 8 * g + 4 * (lane >> 5);
                *reinterpret_cast<float4*>(out + (size_t)n * H + col) =
                    make_float4(acc[t][k][4 * g] * inv, acc[t][k][4 * g + 1] * inv, acc[t][k][4 * g + 2] * inv,
                                acc[t][k][4 * g + 3] * inv);
            }
    }
}

// ------------------------------------------------------------------------------------------------------------------
// layer 0's weight gradient (qs_attn_dw0_x3): part[b] = G[rows of b]^T X[rows of b], X the layer-0 input rows
// gathered from the observations (row r = agent r / K, slot r % K: [nbr (nd) | self of agent r % B (so) | 0], KD0 = 32
// columns -- the forward's gather_rows0), G = de1_pre [R, H] with its column scales gs (|G[:, n]| gs[n] < 2^14), X at
// the forward's layer-0 scale X3_SIN; the column sums of G (the bias gradient's parts) from the same pass.  The
// structure of dw_x3_kernel with A = the gathered X: 16-row steps, G's tile and X's 32 columns staged transposed as
// f16 hi / lo, double-buffered; per wave NT 32 x 32 output tiles (rows n of the wave's range, the 32 X columns).
// ------------------------------------------------------------------------------------------------------------------
template <int H>
constexpr size_t dw0_lds_bytes() { return (size_t)2 * (2 * H + 2 * KD0) * DW_LDR * 2; }

template <int H>
__global__ __launch_bounds__(NTHR, 2) void dw0_x3_kernel(const float* __restrict__ G, const float* __restrict__ gs,
                                                         const float* __restrict__ obs, int stride, int so, int off,
                                                         int B, int K, int nd, long R, int steps_per_block,
                                                         float* __restrict__ part, float* __restrict__ part_sum) {
    constexpr int NT = H / 128, TPC = NTHR / H, RPT = DW_STEP / TPC;
    constexpr int XR = DW_STEP * KD0 / NTHR;   // X values per thread and step (2): column tid % KD0, consecutive rows
    static_assert(RPT % 8 == 0 && XR == 2, "staging shapes");
    extern __shared__ float4 smem4[];
    _Float16* lds = reinterpret_cast<_Float16*>(smem4);
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int sc = tid % H, sr = (tid / H) * RPT;
    const int xc = tid % KD0, xr = (tid / KD0) * XR;
    const long r_begin = (long)blockIdx.x * steps_per_block * DW_STEP;
    constexpr size_t BUF = (size_t)(2 * H + 2 * KD0) * DW_LDR;   // halves per buffer: Gh, Gl [H][24], Xh, Xl [32][24]
    auto gbuf = [&](int b, int which) { return lds + b * BUF + (size_t)which * H * DW_LDR; };
    auto xbuf = [&](int b, int which) { return lds + b * BUF + (size_t)2 * H * DW_LDR + (size_t)which * KD0 * DW_LDR; };
    const float sg = gs[sc];
    // two steps in flight in a register ring (slot k % 2; the loop is unrolled by 2), G through a buffer descriptor
    // over the block's rows (as dw_x3_kernel)
    float gv[2][RPT], xv[2][XR];
    float csum = 0.f;
    const long r_end = r_begin + (long)steps_per_block * DW_STEP < R ? r_begin + (long)steps_per_block * DW_STEP : R;
    const int nbytes = r_end > r_begin ? (int)((r_end - r_begin) * H * 4) : 0;
    const auto rg = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(G + r_begin * H), (short)0, nbytes, 0x00020000);
    const int voff = (sr * H + sc) * 4;
    auto load = [&](auto SL, int s) {
        constexpr int sl = decltype(SL)::value;
        const int soff = s * DW_STEP * H * 4;
#pragma unroll
        for (int u = 0; u < RPT; ++u)
            gv[sl][u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rg, voff + u * H * 4, soff, 0));
#pragma unroll
        for (int u = 0; u < XR; ++u) {   // gather_rows0's indexing (unconditional loads, zeroed by a product)
            const long r = r_begin + (long)s * DW_STEP + xr + u;
            const bool ok = r < R && s < steps_per_block && xc < nd + so;
            const long j = ok ? r : 0;
            const long a = j / K;
            const long idx = xc < nd ? a * stride + off + (j - a * K) * nd + xc : (j % B) * stride + (xc < nd + so ? xc - nd : 0);
            xv[sl][u] = obs[idx] * (ok ? 1.f : 0.f);
        }
    };
    auto stage = [&](auto SL, int b) {
        constexpr int sl = decltype(SL)::value;
#pragma unroll
        for (int o = 0; o < RPT; o += 8) {
            f16x8 gh, gl;
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                csum += gv[sl][o + u];
                const float g = sg * gv[sl][o + u];
                gh[u] = (_Float16)g;
                gl[u] = (_Float16)(g - (float)gh[u]);
            }
            const int off8 = sc * DW_LDR + sr + o;
            *reinterpret_cast<f16x8*>(gbuf(b, 0) + off8) = gh;
            *reinterpret_cast<f16x8*>(gbuf(b, 1) + off8) = gl;
        }
        typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
        f16x2 h2, l2;
#pragma unroll
        for (int u = 0; u < XR; ++u) {
            const float x = X3_SIN * xv[sl][u];
            h2[u] = (_Float16)x;
            l2[u] = (_Float16)(x - (float)h2[u]);
        }
        *reinterpret_cast<f16x2*>(xbuf(b, 0) + xc * DW_LDR + xr) = h2;
        *reinterpret_cast<f16x2*>(xbuf(b, 1) + xc * DW_LDR + xr) = l2;
    };
    f32x16 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
    const int aoff = (lane & 31) * DW_LDR + (lane >> 5) * 8;
    auto mfmas = [&](int b) {
        f16x8 gh[NT], gl[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const int n0 = (wave * NT + t) * 32;
            gh[t] = *reinterpret_cast<const f16x8*>(gbuf(b, 0) + n0 * DW_LDR + aoff);
            gl[t] = *reinterpret_cast<const f16x8*>(gbuf(b, 1) + n0 * DW_LDR + aoff);
        }
        const f16x8 xh = *reinterpret_cast<const f16x8*>(xbuf(b, 0) + aoff);
        const f16x8 xl = *reinterpret_cast<const f16x8*>(xbuf(b, 1) + aoff);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, gh[t], acc[t], 0, 0, 0);
            acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, gl[t], acc[t], 0, 0, 0);
            acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(xl, gh[t], acc[t], 0, 0, 0);
        }
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    load(I0{}, 0);
    load(I1{}, 1);
    stage(I0{}, 0);
    __syncthreads();
    auto iter = [&](auto SL, int s) {   // SL = s % 2: step s in LDS buffer s % 2, step s + 1 in slot (s + 1) % 2
        constexpr int sl = decltype(SL)::value;
        if (s + 2 < steps_per_block) load(std::integral_constant<int, sl>{}, s + 2);
        mfmas(sl);
        if (s + 1 < steps_per_block) stage(std::integral_constant<int, sl ^ 1>{}, sl ^ 1);
        __syncthreads();
    };
    for (int s = 0; s < steps_per_block; s += 2) {
        iter(I0{}, s);
        if (s + 1 < steps_per_block) iter(I1{}, s + 1);
    }
    if (part_sum) {
        float* cs = reinterpret_cast<float*>(smem4);
        cs[tid] = csum;
        __syncthreads();
        if (tid < H) {
            float v = cs[tid];
#pragma unroll
            for (int q = 1; q < TPC; ++q) v += cs[q * H + tid];
            part_sum[(size_t)blockIdx.x * H + tid] = v;
        }
    }
    // acc[t] register 4g + j: output row n = (wave NT + t) 32 + (lane & 31), X column 8 g + 4 (lane >> 5) + j
    float* out = part + (size_t)blockIdx.x * H * KD0;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const int n = (wave * NT + t) * 32 + (lane & 31);
        const float inv = 1.f / (gs[n] * X3_SIN);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int col = 8 * g + 4 * (lane >> 5);
            *reinterpret_cast<float4*>(out + (size_t)n * KD0 + col) =
                make_float4(acc[t][4 * g] * inv, acc[t][4 * g + 1] * inv, acc[t][4 * g + 2] * inv, acc[t][4 * g + 3] * inv);
        }
    }
}

// ------------------------------------------------------------------------------------------------------------------
// the maxima over the blocks of the backward's per-block column maxima (qs_colmax_reduce): block (s, c, q) takes
// stat s, 64 columns c, every CM_CHUNKS-th row chunk q; thread (r, n): column 64 c + n, rows r, r + 4, ... of the
// chunk (a row's 64 columns are one 256-byte read per wave); the four row lanes through LDS, then one unsigned-bits
// atomic max per column and block into out (zeroed by the launcher; maxima of non-negative floats, order-free)
// ------------------------------------------------------------------------------------------------------------------
constexpr int CM_CHUNKS = 16;
__global__ __launch_bounds__(256) void colmax_reduce_kernel(const float* __restrict__ part, int nblk, int H,
                                                            float* __restrict__ out) {
    __shared__ float red[256];
    const int s = blockIdx.z, c = blockIdx.y, q = blockIdx.x;
    const int n = threadIdx.x & 63, r = threadIdx.x >> 6, col = 64 * c + n;
    const long rows_per = (nblk + CM_CHUNKS - 1) / CM_CHUNKS;
    const long r0 = q * rows_per, r1 = r0 + rows_per < nblk ? r0 + rows_per : nblk;
    float m = 0.f;
    if (col < H) {
        const float* p = part + (size_t)s * nblk * H + col;
#pragma unroll 4
        for (long b = r0 + r; b < r1; b += 4) m = fmaxf(m, p[b * H]);   // inf stays inf; the entries are >= 0
    }
    red[threadIdx.x] = m;
    __syncthreads();
    if (r == 0 && col < H) {
        m = fmaxf(fmaxf(red[n], red[64 + n]), fmaxf(red[128 + n], red[192 + n]));
        atomicMax(reinterpret_cast<unsigned int*>(out) + (size_t)s * H + col, __float_as_uint(m));
    }
}

// ------------------------------------------------------------------------------------------------------------------
// tanh backward with the statistics the x3 backward needs (qs_tanh_grad_stats): gp = g (1 - y^2) for [M, N] rows,
// each row's power-of-two scale (row_scale: max |gp_r| s in [2^13, 2^14), 1 for a zero or non-finite row) and the
// block's column maxima (col_part [n_blocks][N]: +inf where a value is not finite) -- one pass instead of torch's
// tanh_backward and two max-abs reductions.  Block = 64 rows, wave w its rows w, w + 4, ...; lane l the columns
// 4 (l + 64 f) .. + 3, f < N / 256, TG_BR rows' loads in flight at a time.
// ------------------------------------------------------------------------------------------------------------------
constexpr int TG_BR = 4;
template <int NF>
__global__ __launch_bounds__(NTHR) void tanh_grad_stats_kernel(const float* __restrict__ g, const float* __restrict__ y,
                                                               float* __restrict__ gp, float* __restrict__ row_scale,
                                                               float* __restrict__ col_part, long M) {
    constexpr int N = 256 * NF;
    __shared__ float4 cm_lds[NWAVE][64 * NF];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const long row0 = (long)blockIdx.x * MROWS;
    float4 cm[NF];
#pragma unroll
    for (int f = 0; f < NF; ++f) cm[f] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int r0 = wave; r0 < MROWS; r0 += NWAVE * TG_BR) {
        float4 gv[TG_BR][NF], yv[TG_BR][NF];
#pragma unroll
        for (int u = 0; u < TG_BR; ++u) {
            const long r = row0 + r0 + u * NWAVE;
            const long rr = r < M ? r : 0;   // unconditional loads (row 0 stands in past M)
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                gv[u][f] = ld4g(g + rr * N + 4 * (lane + 64 * f));
                yv[u][f] = ld4g(y + rr * N + 4 * (lane + 64 * f));
            }
        }
#pragma unroll
        for (int u = 0; u < TG_BR; ++u) {
            const long r = row0 + r0 + u * NWAVE;
            float m = 0.f;
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                const float4 v = f4_dtanh(gv[u][f], yv[u][f]);
                if (r < M) {
                    st4g(gp + r * N + 4 * (lane + 64 * f), v);
                    cm[f] = absmax_acc4(cm[f], v);
                    m = absmax_acc(m, v.x);
                    m = absmax_acc(m, v.y);
                    m = absmax_acc(m, v.z);
                    m = absmax_acc(m, v.w);
                }
            }
            m = wave_max(m);   // (inf stays inf: row_scale -> 1)
            if (lane == 0 && r < M) row_scale[r] = qs::pol::row_scale(m);
        }
    }
#pragma unroll
    for (int f = 0; f < NF; ++f) cm_lds[wave][lane + 64 * f] = cm[f];
    __syncthreads();
    for (int c4 = tid; c4 < N / 4; c4 += NTHR) {
        float4 m = cm_lds[0][c4];
#pragma unroll
        for (int w = 1; w < NWAVE; ++w) m = max4(m, cm_lds[w][c4]);
        *reinterpret_cast<float4*>(col_part + (size_t)blockIdx.x * N + 4 * c4) = m;
    }
}

// ------------------------------------------------------------------------------------------------------------------
// A sum over slabs with the same statistics (qs_slab_sum_stats): out[m] = sum_{s < S} G[s M + m] for [M, N] rows -- the
// score layer's mean-half gradient dP[b] = sum_k da1_pre[k B + b] (quad_multi_model.py:90-92 pairs attention row j
// with agent j % B through the repeat tiling) -- with each out row's power-of-two scale and the block's column maxima
// as qs_tanh_grad_stats (for qs_linear_rows_x3 and qs_dw_x3_ld).  The slabs SS_U at a time with unconditional loads
// (the last slab stands in past S and is not added); SS_BR rows per wave in flight.
// ------------------------------------------------------------------------------------------------------------------
constexpr int SS_BR = 4, SS_U = 4;
template <int NF>
__global__ __launch_bounds__(NTHR) void slab_sum_stats_kernel(const float* __restrict__ G, int S, float* __restrict__ out,
                                                              float* __restrict__ row_scale, float* __restrict__ col_part,
                                                              long M) {
    constexpr int N = 256 * NF;
    __shared__ float4 cm_lds[NWAVE][64 * NF];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const long row0 = (long)blockIdx.x * MROWS;
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 cm[NF];
#pragma unroll
    for (int f = 0; f < NF; ++f) cm[f] = z4;
    for (int r0 = wave; r0 < MROWS; r0 += NWAVE * SS_BR) {
        float4 sum[SS_BR][NF];
#pragma unroll
        for (int u = 0; u < SS_BR; ++u)
#pragma unroll
            for (int f = 0; f < NF; ++f) sum[u][f] = z4;
        for (int s0 = 0; s0 < S; s0 += SS_U) {
            float4 v[SS_U][SS_BR][NF];
#pragma unroll
            for (int q = 0; q < SS_U; ++q) {
                const long s = s0 + q < S ? s0 + q : S - 1;
#pragma unroll
                for (int u = 0; u < SS_BR; ++u) {
                    const long r = row0 + r0 + u * NWAVE;
                    const long rr = r < M ? r : 0;   // unconditional loads (row 0 stands in past M)
#pragma unroll
                    for (int f = 0; f < NF; ++f) v[q][u][f] = ld4g(G + (s * M + rr) * N + 4 * (lane + 64 * f));
                }
            }
#pragma unroll
            for (int q = 0; q < SS_U; ++q)
                if (s0 + q < S)
#pragma unroll
                    for (int u = 0; u < SS_BR; ++u)
#pragma unroll
                        for (int f = 0; f < NF; ++f) sum[u][f] = f4_add(sum[u][f], v[q][u][f]);
        }
#pragma unroll
        for (int u = 0; u < SS_BR; ++u) {
            const long r = row0 + r0 + u * NWAVE;
            float m = 0.f;
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                const float4 x = sum[u][f];
                if (r < M) {
                    st4g(out + r * N + 4 * (lane + 64 * f), x);
                    cm[f] = absmax_acc4(cm[f], x);
                    m = absmax_acc(m, x.x);
                    m = absmax_acc(m, x.y);
                    m = absmax_acc(m, x.z);
                    m = absmax_acc(m, x.w);
                }
            }
            m = wave_max(m);
            if (lane == 0 && r < M) row_scale[r] = qs::pol::row_scale(m);
        }
    }
#pragma unroll
    for (int f = 0; f < NF; ++f) cm_lds[wave][lane + 64 * f] = cm[f];
    __syncthreads();
    for (int c4 = tid; c4 < N / 4; c4 += NTHR) {
        float4 m = cm_lds[0][c4];
#pragma unroll
        for (int w = 1; w < NWAVE; ++w) m = max4(m, cm_lds[w][c4]);
        *reinterpret_cast<float4*>(col_part + (size_t)blockIdx.x * N + 4 * c4) = m;
    }
}

// ------------------------------------------------------------------------------------------------------------------
// column reductions of a gradient G [R, H] (qs_colstats): block p walks rows [p rows_per, (p+1) rows_per), thread n
// owns column n (blockDim = H): a coalesced row of H floats per step, max |g|, sum w_r g (w: optional row weights)
// and, with NX > 0, sum g X(r, c) with the layer-0 input X of row r = q K + m (neighbour m of agent q; self row
// r % B).  X is gathered a chunk of CH rows at a time into LDS by the whole block (each value once), then read as
// LDS broadcasts by every column's thread.  The bias gradients, the dW column scales, the layer-0 weight gradient
// and the score layer's weight gradient (w = dscore) in one pass each; an empty trailing part writes identities.
// ------------------------------------------------------------------------------------------------------------------
template <int NX>
__global__ __launch_bounds__(256) void colstats_kernel(const float* __restrict__ G, long R, int H, long rows_per,
                                                       const float* __restrict__ rw, const float* __restrict__ obs,
                                                       int stride, int nbr_off, int B, int K, int nd, int nx,
                                                       float* __restrict__ pmx, float* __restrict__ psm,
                                                       float* __restrict__ px) {
    constexpr int CH = 64;   // rows per staged chunk of X
    __shared__ float xs_lds[NX > 0 ? CH * NX : 1];
    const int n = threadIdx.x;
    const long r0 = (long)blockIdx.x * rows_per, r1 = r0 + rows_per < R ? r0 + rows_per : R;
    float mx = 0.f, sm = 0.f, xs[NX > 0 ? NX : 1];
#pragma unroll
    for (int c = 0; c < (NX > 0 ? NX : 1); ++c) xs[c] = 0.f;
    bool bad = false;
    if constexpr (NX == 0) {
#pragma unroll 8
        for (long r = r0; r < r1; ++r) {
            const float g = G[r * H + n];
            const float a = fabsf(g);
            mx = fmaxf(mx, a);
            bad |= !(a <= 3.4028235e38f);
            sm += rw ? rw[r] * g : g;
        }
    } else {
        for (long c0 = r0; c0 < r1; c0 += CH) {
            const int rows = (int)(r1 - c0 < CH ? r1 - c0 : CH);
            __syncthreads();   // the previous chunk's X has been read
            for (int e = n; e < rows * nx; e += H) {   // 32-bit index arithmetic (the launcher checks R < 2^31)
                const int i = e / nx, c = e - i * nx;
                const int r = (int)c0 + i, q = r / K;
                xs_lds[i * NX + c] = c < nd ? obs[(long)q * stride + nbr_off + (r - q * K) * nd + c]
                                            : obs[(long)(r % B) * stride + (c - nd)];
            }
            __syncthreads();
#pragma unroll 4
            for (int i = 0; i < rows; ++i) {
                const float g = G[(c0 + i) * H + n];
                const float a = fabsf(g);
                mx = fmaxf(mx, a);
                bad |= !(a <= 3.4028235e38f);
                sm += rw ? rw[c0 + i] * g : g;
                const float* xr = xs_lds + i * NX;
#pragma unroll
                for (int c = 0; c < NX; ++c)
                    if (c < nx) xs[c] = fmaf(g, xr[c], xs[c]);
            }
        }
    }
    pmx[(long)blockIdx.x * H + n] = bad ? __builtin_inff() : mx;
    psm[(long)blockIdx.x * H + n] = sm;
    if constexpr (NX > 0) {
#pragma unroll
        for (int c = 0; c < NX; ++c)
            if (c < nx) px[((long)blockIdx.x * nx + c) * H + n] = xs[c];
    }
}

}  // namespace pol
}  // namespace qs
