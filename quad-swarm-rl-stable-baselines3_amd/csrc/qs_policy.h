// qs_policy.h -- fused no-grad forward of the rollout policy's attention neighbour encoder.
//
// QuadNeighborhoodEncoderAttention (swarm_rl/models/quad_multi_model.py:44-101) as the rollout evaluates it
// once per tower (actor, critic) and step: per neighbour row j of the [B*K, nd] neighbour block
//   e1 = tanh([nbr_j | self_{j % B}] [W_n | W_s]^T + b_e1)   embedding_mlp[0] on the concatenated row
//   e2 = tanh(e1 W_e2^T + b_e2)                               embedding_mlp[2]
//   a1 = tanh(e2 A_e^T + P[j % B]),  P = mean_K(e2) A_m^T + b_a1  (attention_mlp[0], split: per agent)
//   a2 = tanh(a1 A2^T + b_a2),  score = a2 . a3 + b_a3
//   h  = tanh(tanh(e2 V1^T + c1) V2^T + c2)                   neighbor_value_mlp
//   out[b] = sum_k softmax_k(score[bK + k]) h[bK + k]
// (the row pairing j % B is the reference's Tensor.repeat tiling, ppo.py NeighborAttention).
//
// Two kernels, because P of agent j % B needs the mean embedding of agents another block computes:
//   attn_embed_kernel : e1, e2 -> e2 rows and mean_K(e2) per agent to HBM
//   attn_pool_kernel  : e2 rows -> a1, a2, score, softmax, then h weighted and pooled -> out [B, H]
// (torch forms P between them: a [B, H] x [H, H] GEMM).
//
// A block owns 64 neighbour rows (AB = 64 / K whole agents, MU = AB K rows used) and keeps them in LDS as
// ONE [64][H + 4] fp32 tile (67 KB at H = 256: two blocks per CU, so one block's epilogues, barriers and
// loads overlap the other's matrix-core work); each layer's output stays in the accumulators until every
// wave has read the tile, then overwrites it.  A layer is a 64 x H x Kd fp32 GEMM on the matrix cores,
// v_mfma_f32_32x32x2f32, wave w owning output columns [w H/4, (w+1) H/4).  The contraction index is
// permuted so that lane half hf covers k in [hf Kd/2, (hf+1) Kd/2): one ds_read_b128 of a row gives a lane
// its A operand for 4 MFMA steps, and the weights are pre-packed (quadswarm.h qs_attn_tower, policy_fused.py
// pack_mfma_weight) so that one global_load_dwordx4 per lane gives its B operand for 4 steps, 1 KB
// contiguous per wave-instruction.  Activations never leave the CU between layers; bias + tanh are applied
// to the accumulators as they are written back to LDS.  fp32 throughout (the reference trains in fp32);
// tanh is 1 - 2 / (exp(2x) + 1) on the hardware exp2 / rcp (absolute error < 3e-7 against tanhf).
// Roofline: the matrix cores (157 TF fp32 dense): 5 H^2 + 32 H MACs per neighbour row and tower.
#pragma once
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#include <stdint.h>
#endif
#include "quadswarm.h"

namespace qs {
namespace pol {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int MROWS = 64;            // neighbour rows per block
constexpr int RT = MROWS / 32;       // 32-row MFMA tiles
constexpr int NWAVE = 4;
constexpr int NTHR = 64 * NWAVE;
constexpr int MAX_ND = 16;           // neighbour features per row (the reference's largest is 6)
constexpr int KD0 = 32;              // embedding layer 0's input: nd + so <= 32 (the reference's largest is 30)
constexpr int LD0 = KD0 + 4;

template <int H>
struct Geo {
    static_assert(H == 128 || H == 256, "hidden size 128 or 256");
    static constexpr int LD = H + 4;             // LDS row stride in floats: ds_read_b128 of 32 rows conflict-free
    static constexpr int CT = H / (32 * NWAVE);  // 32-column output tiles per wave
    static constexpr int G = H / 8;              // float4 groups along k: 4 MFMA steps each
};

struct Towers {
    qs_attn_tower t[QS_ATTN_MAX_TOWERS];
};

// tanh x = 1 - 2 / (exp(2x) + 1): +-1 at the extremes (exp2 -> inf / 0), NaN in -> NaN out
__device__ __forceinline__ float tanh_fast(float x) {
    const float e = __builtin_amdgcn_exp2f(x * 2.8853900817779268f);   // 2 log2(e)
    return 1.f - 2.f * __builtin_amdgcn_rcpf(e + 1.f);
}

__device__ __forceinline__ float f4at(const float4& v, int u) {
    return u == 0 ? v.x : (u == 1 ? v.y : (u == 2 ? v.z : v.w));
}

// acc = X W^T for the block's 64 rows (X: LDS [64][LD]); W packed: float4 index ((ct G + g) 64 + lane) holds
// W[ct 32 + (lane & 31)][(lane >> 5) H/2 + 4g .. + 3].
struct ZeroInit {
    __device__ float4 operator()(int, int) const { return make_float4(0.f, 0.f, 0.f, 0.f); }
};
// (init(i, n): the accumulators' starting value, e.g. a per-row bias; 0 by default)
// KD: the contraction size (the layer's input width; the tile X has row stride KD + 4).  ZERO: start the
// accumulators at 0 (else they keep what the caller put there, e.g. a per-row bias loaded early)
template <int H, int KD = H, bool ZERO = true>
__device__ __forceinline__ void mfma_layer(const float* X, const float4* __restrict__ Wp, f32x16 (&acc)[RT][Geo<H>::CT],
                                           int wave, int lane) {
    static_assert(KD % 16 == 0, "contraction in float4 groups per lane half");
    constexpr int CT = Geo<H>::CT, G = KD / 8, LD = KD + 4;
    if constexpr (ZERO) {
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int c = 0; c < CT; ++c)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[rt][c][r] = 0.f;
    }
    const float* xa = X + (lane & 31) * LD + (lane >> 5) * (KD / 2);
    const float4* wb = Wp + (size_t)(wave * CT) * G * 64 + lane;
    float4 b0[CT], b1[CT];
#pragma unroll
    for (int c = 0; c < CT; ++c) {
        b0[c] = wb[(size_t)(c * G + 0) * 64];
        b1[c] = G > 1 ? wb[(size_t)(c * G + 1) * 64] : b0[c];
    }
    float4 an[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) an[rt] = *reinterpret_cast<const float4*>(xa + rt * 32 * LD);
    for (int g = 0; g < G; ++g) {
        float4 b[CT], a[RT];
#pragma unroll
        for (int c = 0; c < CT; ++c) {   // weights: two groups in flight ahead of the MFMAs
            b[c] = b0[c];
            b0[c] = b1[c];
            if (g + 2 < G) b1[c] = wb[(size_t)(c * G + g + 2) * 64];
        }
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {   // activations: one group ahead
            a[rt] = an[rt];
            if (g + 1 < G) an[rt] = *reinterpret_cast<const float4*>(xa + rt * 32 * LD + 4 * (g + 1));
        }
        __builtin_amdgcn_sched_barrier(0);   // keep the loads ahead of the MFMAs (qs_policy_x3.h mfma_layer_x3)
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                for (int c = 0; c < CT; ++c)
                    acc[rt][c] = __builtin_amdgcn_mfma_f32_32x32x2f32(f4at(b[c], u), f4at(a[rt], u), acc[rt][c], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
    }
}

// Layer 0's input rows of a block (MROWS x KD0): [nbr_j (nd) | self_{j % B} (so) | 0 ...], row j = agent j / K, slot
// j % K (the reference's row pairing), through put(r, c, v).  Every lane's loads are issued unconditionally, back to
// back: a predicated load compiles to a branch and a full wait per element (8 serial HBM latencies per lane).  The
// padding columns read the row's own self word and are zeroed by a product (finite unless the row itself is not);
// rows past the data read obs[0] and are never used.  (row indices < 2^31: qs_attn_embed checks B K H)
template <typename Put>
__device__ __forceinline__ void gather_rows0(const float* __restrict__ obs, int stride, int so, int off, int B, int K,
                                             int nd, long row0, int MU, long R, int tid, Put put) {
    constexpr int NV = MROWS * KD0 / NTHR;
    float v[NV];
#pragma unroll
    for (int u = 0; u < NV; ++u) {
        const int e = tid + u * NTHR, r = e / KD0, c = e - r * KD0;
        const int j = (int)row0 + r;
        const bool okr = r < MU && j < R;
        const int a = j / K;
        const size_t self = (size_t)(j % B) * stride;
        const size_t idx = c < nd ? (size_t)a * stride + off + (size_t)(j - a * K) * nd + c
                                  : self + (c < nd + so ? c - nd : 0);
        v[u] = obs[okr ? idx : 0] * (c < nd + so ? 1.f : 0.f);
    }
#pragma unroll
    for (int u = 0; u < NV; ++u) {
        const int e = tid + u * NTHR;
        put(e / KD0, e % KD0, v[u]);
    }
}

// The weights are the MFMA's A operand and the activations its B operand, so a 32 x 32 result tile is
// [output column][row]: the block row i is on the lane, and registers 4g .. 4g + 3 of tile (rt, c) hold four
// consecutive output columns n0 .. n0 + 3 -- an epilogue writes them as one float4 (or four packed halves).
__device__ __forceinline__ int acc_i(int rt, int lane) { return rt * 32 + (lane & 31); }
template <int H>
__device__ __forceinline__ int acc_n0(int wave, int c, int g, int lane) {
    return (wave * Geo<H>::CT + c) * 32 + 8 * g + 4 * (lane >> 5);
}
__device__ __forceinline__ float4 f4_add(float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
__device__ __forceinline__ float4 f4_tanh(float4 a) {
    return make_float4(tanh_fast(a.x), tanh_fast(a.y), tanh_fast(a.z), tanh_fast(a.w));
}
__device__ __forceinline__ float4 acc4(const f32x16& a, int g) { return make_float4(a[4 * g], a[4 * g + 1], a[4 * g + 2], a[4 * g + 3]); }

// Y[i][n0 .. n0 + 3] = tanh(acc + bias4(i, n0)) into LDS
template <int H, typename Bias4>
__device__ __forceinline__ void store_tanh(float* Y, const f32x16 (&acc)[RT][Geo<H>::CT], int wave, int lane, Bias4 bias4) {
    constexpr int CT = Geo<H>::CT, LD = Geo<H>::LD;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
        const int i = acc_i(rt, lane);
#pragma unroll
        for (int c = 0; c < CT; ++c)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int n0 = acc_n0<H>(wave, c, g, lane);
                *reinterpret_cast<float4*>(Y + i * LD + n0) = f4_tanh(f4_add(acc4(acc[rt][c], g), bias4(i, n0)));
            }
    }
}
__device__ __forceinline__ float4 lds4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// score = tanh(acc * inv + b_a2) . a3 straight from the a2 layer's accumulators (a2 itself is never stored): this
// lane's part of row i's dot, summed with the other lane half (same row, other columns); SCP[wave][i] = the wave's
// column range.  The caller adds the 4 waves' parts after a barrier.
template <int H>
__device__ __forceinline__ void score_partials(const f32x16 (&acc)[RT][Geo<H>::CT], float inv, const float* a3,
                                               const float* ba2, float* SCP, int wave, int lane) {
    constexpr int CT = Geo<H>::CT;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
        float p = 0.f;
#pragma unroll
        for (int c = 0; c < CT; ++c)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int n0 = acc_n0<H>(wave, c, g, lane);
                const float4 b = lds4(ba2 + n0), w = lds4(a3 + n0);
                p = fmaf(tanh_fast(fmaf(acc[rt][c][4 * g], inv, b.x)), w.x, p);
                p = fmaf(tanh_fast(fmaf(acc[rt][c][4 * g + 1], inv, b.y)), w.y, p);
                p = fmaf(tanh_fast(fmaf(acc[rt][c][4 * g + 2], inv, b.z)), w.z, p);
                p = fmaf(tanh_fast(fmaf(acc[rt][c][4 * g + 3], inv, b.w)), w.w, p);
            }
        p += __shfl_xor(p, 32);
        if (lane < 32) SCP[wave * MROWS + acc_i(rt, lane)] = p;
    }
}

template <int H>
constexpr size_t embed_lds_bytes() { return (size_t)(MROWS * Geo<H>::LD + MROWS * LD0 + 2 * H) * 4; }
template <int H>
constexpr size_t pool_lds_bytes() { return (size_t)(MROWS * Geo<H>::LD + 3 * MROWS + 4 * H + NWAVE * MROWS) * 4; }

// e1 -> e2 for the block's rows (both layers on the matrix cores); e2 rows and the per-agent mean of e2 to HBM
template <int H>
__global__ __launch_bounds__(NTHR, 2) void attn_embed_kernel(const float* __restrict__ obs, int stride, int so,
                                                            int off, int B, int K, int nd, Towers tw) {
    constexpr int LD = Geo<H>::LD, CT = Geo<H>::CT;
    extern __shared__ float4 smem4[];
    float* X = reinterpret_cast<float*>(smem4);
    float* X0 = X + MROWS * LD;   // layer 0's input rows
    float* BI = X0 + MROWS * LD0;  // b_e1, b_e2
    const qs_attn_tower& t = tw.t[blockIdx.y];
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
    // layer 0's input rows [nbr_j (nd) | self_{j % B} (so) | 0 ...] (KD0 wide): row j = agent j / K, slot j % K;
    // its self half comes from agent j % B (the reference's row pairing)
    gather_rows0(obs, stride, so, off, B, K, nd, row0, MU, R, tid, [&](int r, int c, float v) { X0[r * LD0 + c] = v; });
    __syncthreads();
    QS_STAMP(1);
    f32x16 acc[RT][CT];
    {   // e1 = tanh([nbr | self] [W_n | W_s]^T + b_e1): a KD0-deep layer on the matrix cores
        mfma_layer<H, KD0>(X0, reinterpret_cast<const float4*>(t.w_e1p), acc, wave, lane);
        store_tanh<H>(X, acc, wave, lane, [&](int i, int n0) {
            return (i < MU && row0 + i < R) ? lds4(BI + n0) : make_float4(0.f, 0.f, 0.f, 0.f);
        });
    }
    __syncthreads();
    QS_STAMP(2);
    mfma_layer<H>(X, reinterpret_cast<const float4*>(t.w_e2p), acc, wave, lane);
    QS_STAMP(3);
    __syncthreads();   // every wave has read the tile
    store_tanh<H>(X, acc, wave, lane, [&](int, int n0) { return lds4(BI + H + n0); });
    __syncthreads();
    QS_STAMP(4);
    for (int e = tid; e < MROWS * (H / 4); e += NTHR) {
        const int r = e / (H / 4), c4 = e - r * (H / 4);
        const long j = row0 + r;
        if (r < MU && j < R)
            reinterpret_cast<float4*>(t.e2 + j * H)[c4] = *reinterpret_cast<const float4*>(X + r * LD + 4 * c4);
    }
    const float inv = 1.f / (float)K;   // torch's mean: the sum times 1 / K
    for (int e = tid; e < AB * H; e += NTHR) {
        const int a = e / H, n = e - a * H;
        const long agent = row0 / K + a;
        if (agent < B) {
            float s = 0.f;
            for (int k = 0; k < K; ++k) s += X[(a * K + k) * LD + n];
            t.e_mean[agent * H + n] = s * inv;
        }
    }
    QS_STAMP(5);
    QS_RTSTAMP(13);
    QS_STAMP_FLUSH();
}

// the block's e2 rows into the tile (zero rows past the data)
template <int H>
__device__ __forceinline__ void load_rows(float* X, const float* __restrict__ src, long row0, int MU, long R, int tid) {
    constexpr int LD = Geo<H>::LD, NV = MROWS * (H / 4) / NTHR;   // float4 per thread, all loads in flight
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
        *reinterpret_cast<float4*>(X + r * LD + 4 * c4) = v[u];
    }
}

// e2 rows -> attention path (a1, a2, score, softmax over each agent's K rows), then the value path h, whose
// accumulators are weighted and summed straight into out = sum_k w_k h_k (no second accumulator set live)
template <int H>
__global__ __launch_bounds__(NTHR, 2) void attn_pool_kernel(int B, int K, Towers tw) {
    constexpr int LD = Geo<H>::LD, CT = Geo<H>::CT;
    extern __shared__ float4 smem4[];
    float* X = reinterpret_cast<float*>(smem4);
    float* SC = X + MROWS * LD;
    float* WT = SC + MROWS;
    float* A3 = WT + 2 * MROWS;                      // attention_mlp[4].weight, then b_a2, b_v1, b_v2
    const qs_attn_tower& t = tw.t[blockIdx.y];
    const int AB = MROWS / K, MU = AB * K;
    const long R = (long)B * K, row0 = (long)blockIdx.x * MU;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    QS_STAMP_DECL
    QS_RTSTAMP(12);
    QS_STAMP(0);
    for (int n = tid; n < H; n += NTHR) {
        A3[n] = t.w_a3[n];
        A3[H + n] = t.b_a2[n];
        A3[2 * H + n] = t.b_v1[n];
        A3[3 * H + n] = t.b_v2[n];
    }
    // attention_mlp: a1 = tanh(e2 A_e^T + P[j % B]); the per-agent half (with its bias) is the accumulators'
    // start, loaded with the block's e2 rows so that both latencies overlap
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
                acc[rt][c][4 * g] = v.x; acc[rt][c][4 * g + 1] = v.y;
                acc[rt][c][4 * g + 2] = v.z; acc[rt][c][4 * g + 3] = v.w;
            }
    }
    load_rows<H>(X, t.e2, row0, MU, R, tid);
    __syncthreads();
    QS_STAMP(1);
    mfma_layer<H, H, false>(X, reinterpret_cast<const float4*>(t.w_a1ep), acc, wave, lane);
    QS_STAMP(2);
    __syncthreads();
    store_tanh<H>(X, acc, wave, lane, ZeroInit());
    __syncthreads();
    QS_STAMP(3);
    mfma_layer<H>(X, reinterpret_cast<const float4*>(t.w_a2p), acc, wave, lane);
    QS_STAMP(4);
    // score = a2 . a3 + b_a3 from the accumulators (a2 is not stored)
    float* SCP = A3 + 4 * H;
    score_partials<H>(acc, 1.f, A3, A3 + H, SCP, wave, lane);
    __syncthreads();
    QS_STAMP(5);
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
    // neighbor_value_mlp on the e2 rows again (L2 / Infinity Cache): h1 -> tile, h -> weighted into the tile
    load_rows<H>(X, t.e2, row0, MU, R, tid);
    __syncthreads();
    QS_STAMP(6);
    mfma_layer<H>(X, reinterpret_cast<const float4*>(t.w_v1p), acc, wave, lane);
    QS_STAMP(7);
    __syncthreads();
    store_tanh<H>(X, acc, wave, lane, [&](int, int n0) { return lds4(A3 + 2 * H + n0); });
    __syncthreads();
    QS_STAMP(8);
    mfma_layer<H>(X, reinterpret_cast<const float4*>(t.w_v2p), acc, wave, lane);
    QS_STAMP(9);
    __syncthreads();
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
        const int i = acc_i(rt, lane);
        const float wi = i < MU ? WT[i] : 0.f;
#pragma unroll
        for (int c = 0; c < CT; ++c)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int n0 = acc_n0<H>(wave, c, g, lane);
                const float4 h = f4_tanh(f4_add(acc4(acc[rt][c], g), lds4(A3 + 3 * H + n0)));
                *reinterpret_cast<float4*>(X + i * LD + n0) = make_float4(wi * h.x, wi * h.y, wi * h.z, wi * h.w);
            }
    }
    __syncthreads();
    for (int e = tid; e < AB * H; e += NTHR) {
        const int a = e / H, n = e - a * H;
        const long agent = row0 / K + a;
        if (agent < B) {
            float s = 0.f;
            for (int k = 0; k < K; ++k) s += X[(a * K + k) * LD + n];
            t.out[agent * H + n] = s;
        }
    }
    QS_STAMP(10);
    QS_RTSTAMP(13);
    QS_STAMP_FLUSH();
}

}  // namespace pol
}  // namespace qs
