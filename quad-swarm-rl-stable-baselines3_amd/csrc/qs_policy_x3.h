// qs_policy_x3.h -- the fused attention-encoder forward of qs_policy.h with every fp32 product split over the
// f16 matrix cores (precision QS_ATTN_X3).
//
// Same function, same two kernels, same block structure (64 neighbour rows per block, 4 waves, wave w owning
// output columns [w H/4, (w+1) H/4)); what changes is the contraction.  Each fp32 operand x is carried as two
// f16 values, hi = f16(s x) and lo = f16(s x - hi) with a power-of-two scale s (activations 2^8, raw obs 2^4,
// weights 2^8: the scale keeps hi normal for the values that matter; lo goes subnormal only where x itself is so
// small that its lo half is below f16's normal range, i.e. where the dropped bits are below fp32's own rounding of
// the products), so x = (hi + lo) / s to 2^-22 relative, and
//   x . w = (hi_x hi_w + hi_x lo_w + lo_x hi_w) / (s_x s_w)   (+ the dropped lo_x lo_w, < 2^-22 relative)
// with every f16 x f16 product exact in the fp32 accumulator (11 + 11 bits).  Three v_mfma_f32_32x32x16_f16 per
// 32 x 32 x 16 step replace eight v_mfma_f32_32x32x2f32 (32 vs 64 cycles each): 5.3x the fp32 matrix rate at a
// per-product error of ~7e-7 relative (fp32's own rounding: 6e-8), i.e. the fp32 GEMM emulated on the f16 matrix
// cores the way split-precision ("3 x f16") GEMMs do.  Accumulation, biases, tanh, softmax and pooling stay fp32.
//
// LDS: the block's activation tile as two f16 tiles (hi, lo) [64][H + 8] -- the same 67 KB as the fp32 tile, so
// two blocks still share a CU; the A operand of a 16-deep step is one ds_read_b128 per tile and 32-row half.
// Weights: packed per (32-column tile ct, 16-deep step s, lane l): 8 hi halves then 8 lo halves of
// W[32 ct + (l & 31)][16 s + 8 (l >> 5) .. + 7] * 2^8 -- two global_load_dwordx4 per lane and step, 2 KB
// contiguous per wave (policy_fused.pack_mfma_weight_x3).
#pragma once
#include "qs_policy.h"

namespace qs {
namespace pol {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

#ifndef QS_EMBED_PIN
#define QS_EMBED_PIN 1   // the embed kernels' H x H layer with the scheduling fences of mfma_layer_x3 (PIN)
#endif

#ifndef QS_POOL_V1_EARLY
#define QS_POOL_V1_EARLY 1   // pool kernels: value layer 1 on the first e2 tile (no second e2 load; 64 more live registers)
#endif

constexpr float X3_SX = 256.f;        // activation scale (tanh outputs, e2 rows)
constexpr float X3_SIN = 16.f;        // raw observation scale (layer 0 inputs)
constexpr float X3_SW = 256.f;        // weight scale (policy_fused.pack_mfma_weight_x3)
// range: f16 overflows at 65504, i.e. |w| >= 65504 / X3_SW = 255.9 or |obs| >= 65504 / X3_SIN = 4094 would become
// +-inf.  tanh outputs are < 1; policy_fused checks the weights at every refresh (and packs fp32 if any is out of
// range) and the observations it was given once per rollout (FusedRolloutPolicy.check_inputs).

template <int KD>
struct GeoX3 {
    static constexpr int LDH = KD + 8;   // f16 row stride: 16-B rotation per row, ds_read_b128 of 16 rows conflict-free
    static constexpr int S = KD / 16;    // 16-deep steps
};

// one tile pair: element (i, n) -> hi / lo halves
struct TileX3 {
    _Float16* h;
    _Float16* l;
    int ld;
    __device__ __forceinline__ void put(int i, int n, float ys) const {   // ys = s x (already scaled)
        const _Float16 a = (_Float16)ys;
        h[i * ld + n] = a;
        l[i * ld + n] = (_Float16)(ys - (float)a);
    }
    __device__ __forceinline__ float get(int i, int n) const {   // s x
        return (float)h[i * ld + n] + (float)l[i * ld + n];
    }
    // four consecutive elements (n0 % 4 == 0): one 8-byte LDS store per half
    __device__ __forceinline__ void put4(int i, int n0, float4 ys) const {
        typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
        const f16x4 a = {(_Float16)ys.x, (_Float16)ys.y, (_Float16)ys.z, (_Float16)ys.w};
        const f16x4 b = {(_Float16)(ys.x - (float)a[0]), (_Float16)(ys.y - (float)a[1]), (_Float16)(ys.z - (float)a[2]),
                         (_Float16)(ys.w - (float)a[3])};
        *reinterpret_cast<f16x4*>(h + i * ld + n0) = a;
        *reinterpret_cast<f16x4*>(l + i * ld + n0) = b;
    }
};

// A layer's first two 16-deep weight steps (the queue mfma_layer_x3 starts from).  Issued by the caller ahead of an
// epilogue's HBM stores (mfma_prefetch_x3, then the stores, then the layer), the layer's first MFMAs wait for these
// loads alone: the memory counter retires in order, so weight loads issued after a burst of stores wait for every
// store's completion (one full HBM write latency per layer, measured on the update's kernels).
template <int H, int KD = H>
struct WQueue {
    uint4 bh0[Geo<H>::CT], bl0[Geo<H>::CT], bh1[Geo<H>::CT], bl1[Geo<H>::CT];
};
template <int H, int KD = H>
__device__ __forceinline__ const uint4* wlane_base(const uint4* __restrict__ Wp, int wave, int lane) {
    // lane's 32 B of (ct, s): uint4 index ((ct S + s) 64 + lane) 2 + {0: hi, 1: lo}
    return Wp + ((size_t)(wave * Geo<H>::CT) * GeoX3<KD>::S * 64 + lane) * 2;
}
template <int H, int KD = H>
__device__ __forceinline__ WQueue<H, KD> mfma_prefetch_x3(const uint4* __restrict__ Wp, int wave, int lane) {
    constexpr int CT = Geo<H>::CT, S = GeoX3<KD>::S;
    const uint4* wb = wlane_base<H, KD>(Wp, wave, lane);
    auto wld = [&](int c, int s, int part) { return wb[((size_t)(c * S + s) * 64) * 2 + part]; };
    WQueue<H, KD> q;
#pragma unroll
    for (int c = 0; c < CT; ++c) {
        q.bh0[c] = wld(c, 0, 0);
        q.bl0[c] = wld(c, 0, 1);
        q.bh1[c] = S > 1 ? wld(c, 1, 0) : q.bh0[c];
        q.bl1[c] = S > 1 ? wld(c, 1, 1) : q.bl0[c];
    }
    return q;
}

// acc = (Xh + Xl)(Wh + Wl)^T for the block's 64 rows (dropping Xl Wl), scaled by s_x s_w; starting from the weight
// queue q (mfma_prefetch_x3 of the same Wp)
// PIN: fence the MFMA block of each step with scheduling barriers (below); measured per kernel
template <int H, int KD = H, bool ZERO = true, bool PIN = true>
__device__ __forceinline__ void mfma_layer_x3(const TileX3& X, const uint4* __restrict__ Wp, f32x16 (&acc)[RT][Geo<H>::CT],
                                              int wave, int lane, const WQueue<H, KD>& q) {
    constexpr int CT = Geo<H>::CT, S = GeoX3<KD>::S;
    if constexpr (ZERO) {
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int c = 0; c < CT; ++c)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[rt][c][r] = 0.f;
    }
    const int aoff = (lane & 31) * X.ld + (lane >> 5) * 8;
    const uint4* wb = wlane_base<H, KD>(Wp, wave, lane);
    auto wld = [&](int c, int s, int part) { return wb[((size_t)(c * S + s) * 64) * 2 + part]; };
    auto ald = [&](const _Float16* t, int rt, int s) {
        return *reinterpret_cast<const f16x8*>(t + aoff + rt * 32 * X.ld + 16 * s);
    };
    uint4 bh0[CT], bl0[CT], bh1[CT], bl1[CT];
#pragma unroll
    for (int c = 0; c < CT; ++c) {
        bh0[c] = q.bh0[c];
        bl0[c] = q.bl0[c];
        bh1[c] = q.bh1[c];
        bl1[c] = q.bl1[c];
    }
    f16x8 ahn[RT], aln[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
        ahn[rt] = ald(X.h, rt, 0);
        aln[rt] = ald(X.l, rt, 0);
    }
    for (int s = 0; s < S; ++s) {
        f16x8 ah[RT], al[RT], bh[CT], bl[CT];
#pragma unroll
        for (int c = 0; c < CT; ++c) {   // weights: two steps in flight ahead of the MFMAs
            bh[c] = __builtin_bit_cast(f16x8, bh0[c]);
            bl[c] = __builtin_bit_cast(f16x8, bl0[c]);
            bh0[c] = bh1[c];
            bl0[c] = bl1[c];
            if (s + 2 < S) {
                bh1[c] = wld(c, s + 2, 0);
                bl1[c] = wld(c, s + 2, 1);
            }
        }
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {   // activations: one step ahead (the LDS latency off the MFMA chain)
            ah[rt] = ahn[rt];
            al[rt] = aln[rt];
            if (s + 1 < S) {
                ahn[rt] = ald(X.h, rt, s + 1);
                aln[rt] = ald(X.l, rt, s + 1);
            }
        }
        // keep the queue where it is written: left alone, the scheduler sinks each load next to its first MFMA
        // (and reuses one register for every LDS read), which waits out the full latency at each step
        if constexpr (PIN) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int c = 0; c < CT; ++c) {
                // weights as A, activations as B: the result tile is [output column][row] (qs_policy.h acc_i / acc_n0)
                acc[rt][c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(bh[c], ah[rt], acc[rt][c], 0, 0, 0);
                acc[rt][c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(bl[c], ah[rt], acc[rt][c], 0, 0, 0);
                acc[rt][c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(bh[c], al[rt], acc[rt][c], 0, 0, 0);
            }
        if constexpr (PIN) __builtin_amdgcn_sched_barrier(0);
    }
}

template <int H, int KD = H, bool ZERO = true, bool PIN = true>
__device__ __forceinline__ void mfma_layer_x3(const TileX3& X, const uint4* __restrict__ Wp, f32x16 (&acc)[RT][Geo<H>::CT],
                                              int wave, int lane) {
    mfma_layer_x3<H, KD, ZERO, PIN>(X, Wp, acc, wave, lane, mfma_prefetch_x3<H, KD>(Wp, wave, lane));
}

// Y = tanh(acc / (s_x s_w) + bias4(i, n0)), stored scaled by X3_SX as hi / lo; out(i, n0, y4) also receives the
// fp32 values (four consecutive columns of row i)
struct NoOut {
    __device__ void operator()(int, int, float4) const {}
};
template <int H, typename Bias4, typename Out = NoOut>
__device__ __forceinline__ void store_tanh_x3(const TileX3& Y, const f32x16 (&acc)[RT][Geo<H>::CT], float inv, int wave,
                                              int lane, Bias4 bias4, Out out = NoOut()) {
    constexpr int CT = Geo<H>::CT;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
        const int i = acc_i(rt, lane);
#pragma unroll
        for (int c = 0; c < CT; ++c)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int n0 = acc_n0<H>(wave, c, g, lane);
                const float4 b = bias4(i, n0);
                const float4 y = make_float4(tanh_fast(fmaf(acc[rt][c][4 * g], inv, b.x)),
                                             tanh_fast(fmaf(acc[rt][c][4 * g + 1], inv, b.y)),
                                             tanh_fast(fmaf(acc[rt][c][4 * g + 2], inv, b.z)),
                                             tanh_fast(fmaf(acc[rt][c][4 * g + 3], inv, b.w)));
                out(i, n0, y);
                Y.put4(i, n0, make_float4(X3_SX * y.x, X3_SX * y.y, X3_SX * y.z, X3_SX * y.w));   // (exact: 2^8)
            }
    }
}

// The embedding's last epilogue: e2 = tanh(acc / (s_x s_w) + b_e2) to HBM (rows < MU of the data) and as fp32 into
// LDS (over the split tile: call after the barrier that follows the layer's last tile read), then e_mean[agent] = (sum_k
// e2 rows of the agent) / K (torch's mean: the sum in k order, times 1 / K) as float4 per thread.
template <int H>
__device__ __forceinline__ void embed_e2_epilogue(const f32x16 (&acc)[RT][Geo<H>::CT], const float* bias, float* e2,
                                                  float* e_mean, float4* smem4, long row0, int MU, long R, int B, int K,
                                                  int AB, int wave, int lane, int tid) {
    constexpr int CT = Geo<H>::CT, LDY = H + 4;
    static_assert(MROWS * (H + 4) * 4 <= 2 * MROWS * GeoX3<H>::LDH * 2, "fp32 tile fits the split tile's bytes");
    float* Y = reinterpret_cast<float*>(smem4);
    constexpr float inv_s = 1.f / (X3_SX * X3_SW);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
        const int i = acc_i(rt, lane);
#pragma unroll
        for (int c = 0; c < CT; ++c)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int n0 = acc_n0<H>(wave, c, g, lane);
                const float4 b = lds4(bias + n0);
                const float4 y = make_float4(tanh_fast(fmaf(acc[rt][c][4 * g], inv_s, b.x)),
                                             tanh_fast(fmaf(acc[rt][c][4 * g + 1], inv_s, b.y)),
                                             tanh_fast(fmaf(acc[rt][c][4 * g + 2], inv_s, b.z)),
                                             tanh_fast(fmaf(acc[rt][c][4 * g + 3], inv_s, b.w)));
                if (i < MU && row0 + i < R) *reinterpret_cast<float4*>(e2 + (row0 + i) * H + n0) = y;
                *reinterpret_cast<float4*>(Y + i * LDY + n0) = y;
            }
    }
    __syncthreads();
    const float inv = 1.f / (float)K;
    constexpr int H4 = H / 4;
    for (int e = tid; e < AB * H4; e += NTHR) {
        const int a = e / H4, c4 = e - a * H4;
        const long agent = row0 / K + a;
        if (agent < B) {
            float4 s = lds4(Y + (a * K) * LDY + 4 * c4);
            for (int k = 1; k < K; ++k) {
                const float4 v = lds4(Y + (a * K + k) * LDY + 4 * c4);
                s = make_float4(s.x + v.x, s.y + v.y, s.z + v.z, s.w + v.w);
            }
            *reinterpret_cast<float4*>(e_mean + agent * H + 4 * c4) = make_float4(s.x * inv, s.y * inv, s.z * inv, s.w * inv);
        }
    }
}

template <int H>
constexpr size_t embed_x3_lds_bytes() {
    return (size_t)(2 * MROWS * GeoX3<H>::LDH + 2 * MROWS * GeoX3<KD0>::LDH) * 2 + (size_t)2 * H * 4;
}
template <int H>
constexpr size_t pool_x3_lds_bytes() {
    return (size_t)(2 * MROWS * GeoX3<H>::LDH) * 2 + (size_t)(3 * MROWS + 4 * H + NWAVE * MROWS) * 4;
}

// attn_embed_kernel with the split-f16 contraction (same inputs, same outputs: e2 rows and means in fp32)
template <int H>
__global__ __launch_bounds__(NTHR, 2) __attribute__((amdgpu_waves_per_eu(2, 2))) void attn_embed_x3_kernel(const float* __restrict__ obs, int stride, int so,
                                                               int off, int B, int K, int nd, Towers tw) {
    constexpr int LDH = GeoX3<H>::LDH, LD0 = GeoX3<KD0>::LDH, CT = Geo<H>::CT;
    extern __shared__ float4 smem4[];
    _Float16* xh = reinterpret_cast<_Float16*>(smem4);
    const TileX3 X{xh, xh + MROWS * LDH, LDH};
    const TileX3 X0{xh + 2 * MROWS * LDH, xh + 2 * MROWS * LDH + MROWS * LD0, LD0};
    float* BI = reinterpret_cast<float*>(xh + 2 * MROWS * LDH + 2 * MROWS * LD0);   // b_e1, b_e2
    const qs_attn_tower& t = tw.t[blockIdx.y];
    const int AB = MROWS / K, MU = AB * K;
    const long R = (long)B * K, row0 = (long)blockIdx.x * MU;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    for (int n = tid; n < H; n += NTHR) {
        BI[n] = t.b_e1[n];
        BI[H + n] = t.b_e2[n];
    }
    // layer 0's input rows [nbr_j (nd) | self_{j % B} (so) | 0 ...], row j = agent j / K, slot j % K; self half from
    // agent j % B (the reference's row pairing)
    gather_rows0(obs, stride, so, off, B, K, nd, row0, MU, R, tid, [&](int r, int c, float v) { X0.put(r, c, X3_SIN * v); });
    __syncthreads();
    f32x16 acc[RT][CT];
    mfma_layer_x3<H, KD0, true, false>(X0, reinterpret_cast<const uint4*>(t.w_e1p), acc, wave, lane);
    store_tanh_x3<H>(X, acc, 1.f / (X3_SIN * X3_SW), wave, lane, [&](int i, int n0) {
        return (i < MU && row0 + i < R) ? lds4(BI + n0) : make_float4(0.f, 0.f, 0.f, 0.f);
    });
    __syncthreads();
    mfma_layer_x3<H, H, true, QS_EMBED_PIN != 0>(X, reinterpret_cast<const uint4*>(t.w_e2p), acc, wave, lane);
    __syncthreads();   // every wave has read the tile
    // e2 to HBM straight from the epilogue (fp32 tanh values) and into an fp32 tile over the split tile's bytes
    // (the last layer: the split tile is not read again), whose rows the per-agent means then read as float4
    embed_e2_epilogue<H>(acc, BI + H, t.e2, t.e_mean, smem4, row0, MU, R, B, K, AB, wave, lane, tid);
}

// the block's e2 rows (fp32, HBM) into the split tile (zero rows past the data)
template <int H>
__device__ __forceinline__ void load_rows_x3(const TileX3& X, const float* __restrict__ src, long row0, int MU, long R,
                                             int tid) {
    constexpr int NV = MROWS * (H / 4) / NTHR;
    float4 v[NV];
#pragma unroll
    for (int u = 0; u < NV; ++u) {
        const int e = tid + u * NTHR, r = e / (H / 4), c4 = e - r * (H / 4);
        const long j = row0 + r;
        const bool ok = r < MU && j < R;
        const float okf = ok ? 1.f : 0.f;
        v[u] = reinterpret_cast<const float4*>(src + (ok ? j : 0) * H)[c4];   // unconditional (see the P loads)
        v[u] = make_float4(v[u].x * okf, v[u].y * okf, v[u].z * okf, v[u].w * okf);
    }
#pragma unroll
    for (int u = 0; u < NV; ++u) {
        const int e = tid + u * NTHR, r = e / (H / 4), c4 = e - r * (H / 4);
        X.put4(r, 4 * c4, make_float4(X3_SX * v[u].x, X3_SX * v[u].y, X3_SX * v[u].z, X3_SX * v[u].w));
    }
}

// attn_pool_kernel with the split-f16 contraction
template <int H>
__global__ __launch_bounds__(NTHR, 2) __attribute__((amdgpu_waves_per_eu(2, 2))) void attn_pool_x3_kernel(int B, int K, Towers tw) {
    constexpr int LDH = GeoX3<H>::LDH, CT = Geo<H>::CT;
    extern __shared__ float4 smem4[];
    _Float16* xh = reinterpret_cast<_Float16*>(smem4);
    const TileX3 X{xh, xh + MROWS * LDH, LDH};
    float* SC = reinterpret_cast<float*>(xh + 2 * MROWS * LDH);
    float* WT = SC + MROWS;
    float* A3 = WT + 2 * MROWS;                      // attention_mlp[4].weight, then b_a2, b_v1, b_v2
    const qs_attn_tower& t = tw.t[blockIdx.y];
    const int AB = MROWS / K, MU = AB * K;
    const long R = (long)B * K, row0 = (long)blockIdx.x * MU;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    constexpr float SS = X3_SX * X3_SW, iSS = 1.f / SS;
    for (int n = tid; n < H; n += NTHR) {
        A3[n] = t.w_a3[n];
        A3[H + n] = t.b_a2[n];
        A3[2 * H + n] = t.b_v1[n];
        A3[3 * H + n] = t.b_v2[n];
    }
    // attention_mlp: a1 = tanh(e2 A_e^T + P[j % B]): the accumulators start at P (scaled like the products)
    f32x16 acc[RT][CT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
        const int i = acc_i(rt, lane);
        const int j = (int)row0 + i;
        const bool ok = i < MU && j < R;
        const float okf = ok ? 1.f : 0.f;
        const float* pr = t.P + (size_t)(ok ? j % B : 0) * H;
#pragma unroll
        for (int c = 0; c < CT; ++c)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                // loaded unconditionally (row 0 stands in for an unused row) and zeroed by a product: a
                // conditional load (or a select the compiler sinks back into a branch) costs a branch + a full
                // wait per load, 16 serial HBM latencies
                float4 v = *reinterpret_cast<const float4*>(pr + acc_n0<H>(wave, c, g, lane));
                v = make_float4(v.x * okf, v.y * okf, v.z * okf, v.w * okf);
                acc[rt][c][4 * g] = SS * v.x; acc[rt][c][4 * g + 1] = SS * v.y;
                acc[rt][c][4 * g + 2] = SS * v.z; acc[rt][c][4 * g + 3] = SS * v.w;
            }
    }
    load_rows_x3<H>(X, t.e2, row0, MU, R, tid);
    __syncthreads();
    mfma_layer_x3<H, H, false>(X, reinterpret_cast<const uint4*>(t.w_a1ep), acc, wave, lane);
#if QS_POOL_V1_EARLY
    // neighbor_value_mlp's first layer on the same e2 tile (its pre-activations held until the tile is free again)
    f32x16 accv[RT][CT];
    mfma_layer_x3<H>(X, reinterpret_cast<const uint4*>(t.w_v1p), accv, wave, lane);
#endif
    __syncthreads();
    store_tanh_x3<H>(X, acc, iSS, wave, lane, ZeroInit());
    __syncthreads();
    mfma_layer_x3<H>(X, reinterpret_cast<const uint4*>(t.w_a2p), acc, wave, lane);
    // score = a2 . a3 + b_a3 from the accumulators (a2 is not stored)
    float* SCP = A3 + 4 * H;
    score_partials<H>(acc, iSS, A3, A3 + H, SCP, wave, lane);
    __syncthreads();
    if (tid < MROWS) SC[tid] = ((SCP[tid] + SCP[MROWS + tid]) + (SCP[2 * MROWS + tid] + SCP[3 * MROWS + tid])) + t.b_a3;
    __syncthreads();
    if (tid < AB) {   // softmax over the agent's K rows
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
    store_tanh_x3<H>(X, accv, iSS, wave, lane, [&](int, int n0) { return lds4(A3 + 2 * H + n0); });
    __syncthreads();
#else
    // neighbor_value_mlp on the e2 rows again (L2 / Infinity Cache)
    load_rows_x3<H>(X, t.e2, row0, MU, R, tid);
    __syncthreads();
    mfma_layer_x3<H>(X, reinterpret_cast<const uint4*>(t.w_v1p), acc, wave, lane);
    __syncthreads();
    store_tanh_x3<H>(X, acc, iSS, wave, lane, [&](int, int n0) { return lds4(A3 + 2 * H + n0); });
    __syncthreads();
#endif
    mfma_layer_x3<H>(X, reinterpret_cast<const uint4*>(t.w_v2p), acc, wave, lane);
    __syncthreads();
    // the weighted h rows into a plain fp32 tile over the same LDS (the split tile is no longer read)
    float* Y = reinterpret_cast<float*>(smem4);
    constexpr int LDY = H + 4;
    static_assert(MROWS * (H + 4) * 4 <= 2 * MROWS * GeoX3<H>::LDH * 2, "fp32 tile fits the split tile's bytes");
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
                *reinterpret_cast<float4*>(Y + i * LDY + n0) =
                    make_float4(wi * tanh_fast(fmaf(acc[rt][c][4 * g], iSS, b.x)),
                                wi * tanh_fast(fmaf(acc[rt][c][4 * g + 1], iSS, b.y)),
                                wi * tanh_fast(fmaf(acc[rt][c][4 * g + 2], iSS, b.z)),
                                wi * tanh_fast(fmaf(acc[rt][c][4 * g + 3], iSS, b.w)));
            }
    }
    __syncthreads();
    for (int e = tid; e < AB * (H / 4); e += NTHR) {   // the agent's weighted rows summed in k order, float4 wide
        const int a = e / (H / 4), c4 = e - a * (H / 4);
        const long agent = row0 / K + a;
        if (agent < B) {
            float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
            for (int k = 0; k < K; ++k) s = f4_add(s, lds4(Y + (a * K + k) * LDY + 4 * c4));
            *reinterpret_cast<float4*>(t.out + agent * H + 4 * c4) = s;
        }
    }
}

}  // namespace pol
}  // namespace qs

namespace qs {
namespace pol {

// ------------------------------------------------------------------------------------------------------------------
// The encoder's feed_forward (quad_multi_model.py:250-353 QuadMultiEncoder: Linear(2R -> 2R) + Tanh on the
// concatenated [self | neighbour] encodings) on the split-f16 matrix cores: Y[:, 256 z + n] = tanh(X W^T + b) for
// X [M, 256 P] with |x| <= 1 (tanh outputs and the attention's softmax-weighted tanh rows), one 64-row block per
// (row tile, output half z): the input's P 256-column slices pass through one split tile in turn, accumulating in
// the same registers; weights packed per (z, p) as pack_mfma_weight_x3 of W[256 z .., 256 p ..].
// ------------------------------------------------------------------------------------------------------------------
// ROWS (the backward's dX = G W for gradient rows G of any magnitude): no bias and no activation, row r of X staged
// at its power-of-two scale rs[r] (max |x_r| rs[r] in [2^13, 2^14): exact, it factors out of the row's products),
// Y = acc / (rs[r] s_w).  ACT false (the attention score layer's mean half P = e_mean A_m^T + b_a1): bias, no tanh.
// The input's column slice p is read from X (p = 0) or X1 (p = 1) with row stride ldx: one [M, 512] input is X, X + 256,
// ldx 512; the feed_forward's [self | neighbour] encodings are two [M, 256] tensors (X, X1, ldx 256: no concatenation).
template <int P, bool ROWS = false, bool ACT = true>
__global__ __launch_bounds__(NTHR, 2) __attribute__((amdgpu_waves_per_eu(2, 2))) void linear_tanh_x3_kernel(
    const float* __restrict__ X, const float* __restrict__ X1, long ldx, long M, const uint4* __restrict__ Wp,
    const float* __restrict__ bias, float* __restrict__ Y, int N, const float* __restrict__ rs = nullptr) {
    constexpr int H = 256, LDH = GeoX3<H>::LDH, CT = Geo<H>::CT, NV = MROWS * (H / 4) / NTHR;
    constexpr size_t WBLK = (size_t)H * H * 2 * 2 / 16;   // uint4 per packed 256 x 256 block: hi + lo f16 halves
    extern __shared__ float4 smem4[];
    _Float16* xh = reinterpret_cast<_Float16*>(smem4);
    const TileX3 T{xh, xh + MROWS * LDH, LDH};
    float* BI = reinterpret_cast<float*>(xh + 2 * MROWS * LDH);
    const long row0 = (long)blockIdx.x * MROWS;
    const int z = blockIdx.y, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    float* RSI = BI + H;        // ROWS: 1 / (rs[r] s_w) of the block's rows
    float* RSX = RSI + MROWS;   // ROWS: rs[r] (0 past M)
    if constexpr (ROWS) {
        if (tid < MROWS) {
            const float r = row0 + tid < M ? rs[row0 + tid] : 0.f;
            RSX[tid] = r;
            RSI[tid] = r > 0.f ? 1.f / (r * X3_SW) : 0.f;
        }
        __syncthreads();
    } else {
        for (int n = tid; n < H; n += NTHR) BI[n] = bias[256 * z + n];
    }
    f32x16 acc[RT][CT];
    float4 v[NV];
    auto load = [&](int p) {   // unconditional loads (row 0 stands in past M), zeroed when put
#pragma unroll
        for (int u = 0; u < NV; ++u) {
            const int e = tid + u * NTHR, r = e / (H / 4), c4 = e - r * (H / 4);
            v[u] = *reinterpret_cast<const float4*>((p == 0 ? X : X1) + (row0 + r < M ? row0 + r : 0) * ldx + 4 * c4);
        }
    };
    auto put = [&]() {
#pragma unroll
        for (int u = 0; u < NV; ++u) {
            const int e = tid + u * NTHR, r = e / (H / 4), c4 = e - r * (H / 4);
            const float sx = ROWS ? RSX[r] : (row0 + r < M ? X3_SX : 0.f);
            T.put4(r, 4 * c4, make_float4(sx * v[u].x, sx * v[u].y, sx * v[u].z, sx * v[u].w));
        }
    };
    load(0);
    put();
    __syncthreads();
#pragma unroll
    for (int p = 0; p < P; ++p) {
        if (p + 1 < P) load(p + 1);   // the next slice in flight during this one's MFMAs
        const uint4* wp = Wp + ((size_t)z * P + p) * WBLK;
        if (p == 0)
            mfma_layer_x3<H, H, true>(T, wp, acc, wave, lane);
        else
            mfma_layer_x3<H, H, false>(T, wp, acc, wave, lane);
        if (p + 1 < P) {
            __syncthreads();   // every wave has read the tile
            put();
            __syncthreads();
        }
    }
    constexpr float iSS = 1.f / (X3_SX * X3_SW);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
        const int i = acc_i(rt, lane);
        if (row0 + i >= M) continue;
        const float si = ROWS ? RSI[i] : 0.f;
#pragma unroll
        for (int c = 0; c < CT; ++c)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int n0 = acc_n0<H>(wave, c, g, lane);
                float4 y;
                if constexpr (ROWS) {
                    y = make_float4(acc[rt][c][4 * g] * si, acc[rt][c][4 * g + 1] * si, acc[rt][c][4 * g + 2] * si,
                                    acc[rt][c][4 * g + 3] * si);
                } else {
                    const float4 b = lds4(BI + n0);
                    y = make_float4(fmaf(acc[rt][c][4 * g], iSS, b.x), fmaf(acc[rt][c][4 * g + 1], iSS, b.y),
                                    fmaf(acc[rt][c][4 * g + 2], iSS, b.z), fmaf(acc[rt][c][4 * g + 3], iSS, b.w));
                    if constexpr (ACT) y = make_float4(tanh_fast(y.x), tanh_fast(y.y), tanh_fast(y.z), tanh_fast(y.w));
                }
                *reinterpret_cast<float4*>(Y + (row0 + i) * N + 256 * z + n0) = y;
            }
    }
}
constexpr size_t linear_x3_lds_bytes() { return (size_t)(2 * MROWS * GeoX3<256>::LDH) * 2 + (size_t)(256 + 2 * MROWS) * 4; }

}  // namespace pol
}  // namespace qs
