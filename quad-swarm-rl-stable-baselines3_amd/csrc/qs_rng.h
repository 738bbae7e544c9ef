// qs_rng.h -- counter-based RNG for the swarm step (Philox4x32-10, Salmon et al. SC'11).
//
// Every random draw of the reference (numba_utils.py:101-105 OU, sensor_noise.py:234-261,
// collisions/*.py impulses, quadrotor_dynamics.py:624 floor flip, quadrotor_single.py:409,454 reset)
// becomes a pure function of (seed, drone id, stream, step counter, index): results do not depend
// on the launch geometry or on how many GPUs the envs are sharded over.
//   key     = {drone global id, seed}
//   counter = {block = index / 4, stream id, step_lo, step_hi}
// Normals: Box-Muller on word pairs (0,1) and (2,3) of a block -> 4 normals per block.
// Uniforms: stream | QS_UNIF_BIT, one word per draw.  The CPU oracle uses the same numbering.
#pragma once
#ifndef __HIPCC_RTC__   // hipRTC (qs_specialize) provides these itself
#include <hip/hip_runtime.h>
#include <stdint.h>
#endif

namespace qs {

enum : uint32_t {
    S_OU = 1, S_FLOOR = 2, S_SENSOR = 3, S_PAIR = 4, S_WALL = 5, S_CEIL = 6, S_DW = 7, S_DWPAIR = 8,
    S_RESET = 9, S_RESET_YAW = 10, S_RESET_SENSOR = 11, S_OBST = 12,
    // flavor A: camera pixel noise (normals 0 = u1, 1 = u2; | neighbour j << 8), spawn / heading draws
    S_CAM = 13, S_CAM_SEL = 14, S_SELF_CAM = 15, S_RESET_A = 16, S_SCEN = 17, S_RESET_CAM = 18,
    S_RESET_CAM_SEL = 19, S_RESET_SELF_CAM = 20,
    // obstacles: per-env map (partial Fisher-Yates uniforms) and scenario draws (mode, cells, goal z)
    S_OBSTMAP = 21, S_OSCEN = 22,
    // flavor-B goal scenarios, per env (key = drone 0): one word per draw in call order
    S_SCN = 23, S_SCN_RESET = 24,
    // obstacle domain randomisation, per env (key = drone 0): uniform 0 density choice, 1 size choice
    S_DR = 26,
    UNIF_BIT = 0x80
};

struct Rng {
    uint32_t seed, ctr_lo, ctr_hi;
};

struct W4 {
    uint32_t w[4];
};

__device__ __forceinline__ W4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        // one v_mad_u64_u32 per product instead of a v_mul_hi_u32 + v_mul_lo_u32 pair
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    W4 o;
    o.w[0] = c0; o.w[1] = c1; o.w[2] = c2; o.w[3] = c3;
    return o;
}

__device__ __forceinline__ W4 block(const Rng& r, uint32_t id, uint32_t stream, uint32_t blk) {
    return philox(blk, stream, r.ctr_lo, r.ctr_hi, id, r.seed);
}

// (0,1), exact in fp32: 24 high bits + half ulp
__device__ __forceinline__ float u01(uint32_t x) { return ((float)(x >> 8) + 0.5f) * (1.0f / 16777216.0f); }

// Box-Muller on the hardware transcendentals: v_log_f32 (log2), v_sqrt_f32, and v_sin/v_cos_f32,
// which take their argument in revolutions (sin(2 pi x)), exactly the Box-Muller angle.
__device__ __forceinline__ void box_muller(uint32_t a, uint32_t b, float& z0, float& z1) {
    const float rr = __builtin_amdgcn_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u01(a)));  // -2 ln u
    const float ub = u01(b);
    z0 = rr * __builtin_amdgcn_cosf(ub);
    z1 = rr * __builtin_amdgcn_sinf(ub);
}

// 4 normals of block blk
__device__ __forceinline__ void normals4(const Rng& r, uint32_t id, uint32_t stream, uint32_t blk, float* z) {
    const W4 q = block(r, id, stream, blk);
    box_muller(q.w[0], q.w[1], z[0], z[1]);
    box_muller(q.w[2], q.w[3], z[2], z[3]);
}

// word k of a block without a dynamically indexed private array (which would live in scratch)
__device__ __forceinline__ uint32_t word_of(const W4& q, uint32_t k) {
    return k == 0 ? q.w[0] : (k == 1 ? q.w[1] : (k == 2 ? q.w[2] : q.w[3]));
}
__device__ __forceinline__ float pick4(const float* z, uint32_t k) {
    return k == 0 ? z[0] : (k == 1 ? z[1] : (k == 2 ? z[2] : z[3]));
}

__device__ __forceinline__ float normal1(const Rng& r, uint32_t id, uint32_t stream, uint32_t idx) {
    float z[4];
    normals4(r, id, stream, idx >> 2, z);
    return pick4(z, idx & 3);
}

// 4 uniforms of block blk of stream | UNIF_BIT
__device__ __forceinline__ void uniforms4(const Rng& r, uint32_t id, uint32_t stream, uint32_t blk, float* u) {
    const W4 q = block(r, id, stream | UNIF_BIT, blk);
#pragma unroll
    for (int i = 0; i < 4; ++i) u[i] = u01(q.w[i]);
}

__device__ __forceinline__ float uniform1(const Rng& r, uint32_t id, uint32_t stream, uint32_t idx) {
    const W4 q = block(r, id, stream | UNIF_BIT, idx >> 2);
    return u01(word_of(q, idx & 3));
}

}  // namespace qs
