// qs_flavor_b.h -- flavor-B kernels (quadrotor_multi.QuadrotorEnvMulti: raw motor commands, shaped
// rewards, drone/room impulses, pos_vel neighbour obs, in-env auto-reset).  Included by qs_step.hip.
#pragma once
#include "qs_common.h"
#include "qs_scen.h"
#include "qs_replay.h"

#ifndef QS_SCW_LATE
#define QS_SCW_LATE 0   // A/B: the scenario record's loads after the drone state's (default: before)
#endif
#ifndef QS_SCW_SKIP
#define QS_SCW_SKIP 0   // diagnostic only (wrong results): no scenario-record loads, every env reads as static
#endif
#ifndef QS_PAIR_ROUNDS
#define QS_PAIR_ROUNDS 1   // drone-pair impulses in rounds of disjoint pairs (else one pair per iteration)
#endif

namespace qs {

// ---------------------------------------------------------------------------------------------
// observations
// ---------------------------------------------------------------------------------------------
// sensor noise (add_noise_numba sensor_noise.py:172-218) + state_xyz_vxyz_R_omega[_floor|_wall]
// (get_state.py:226-292), written to an LDS row.
// z = the 12 normals of the stream's blocks 0..2 (drawn by the caller, possibly on other sub-lanes)
__device__ __forceinline__ void self_obs_z(const KP& kp, const Drone& d, const float* z, const Rng& rng, uint32_t gid, uint32_t stream,
                           float* out) {
    float np_[3], nv[3], no[3], nr[9];
    if (kp.sense) {
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            np_[i] = d.pos[i] + kp.pos_std * z[i];
            nv[i] = d.vel[i] + kp.vel_std * z[3 + i];
            no[i] = d.om[i] + kp.gyro * z[6 + i];
        }
        float th[3] = {0.f, 0.f, 0.f};
        if (kp.pos_unif != 0.f || kp.vel_unif != 0.f || kp.quat_unif != 0.f) {
            float u[12];
            uniforms4(rng, gid, stream, 0, u);
            uniforms4(rng, gid, stream, 1, u + 4);
            uniforms4(rng, gid, stream, 2, u + 8);
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                np_[i] += -kp.pos_unif + 2.f * kp.pos_unif * u[i];
                nv[i] += -kp.vel_unif + 2.f * kp.vel_unif * u[3 + i];
                th[i] = -kp.quat_unif + 2.f * kp.quat_unif * u[6 + i];
            }
        }
        if (kp.quat_std != 0.f) {   // normals 9..11 (block 2, words 1..3)
#pragma unroll
            for (int i = 0; i < 3; ++i) th[i] = kp.quat_std * z[9 + i] + th[i];
        }
        // quat_from_small_angle (sensor_noise.py:11-23)
        const float q2 = (th[0] * th[0] + th[1] * th[1] + th[2] * th[2]) * 0.25f;
        float qt[4];
        if (q2 < 1.f) {
            qt[0] = fsqrt(1.f - q2); qt[1] = th[0] * 0.5f; qt[2] = th[1] * 0.5f; qt[3] = th[2] * 0.5f;
        } else {
            const float w = rsqrtf(1.f + q2), f = 0.5f * w;
            qt[0] = w; qt[1] = th[0] * f; qt[2] = th[1] * f; qt[3] = th[2] * f;
        }
        const float qn = frcp(fsqrt(qt[0] * qt[0] + qt[1] * qt[1] + qt[2] * qt[2] + qt[3] * qt[3]));
#pragma unroll
        for (int i = 0; i < 4; ++i) qt[i] *= qn;
        // rot2quat (sensor_noise.py:34-63)
        const float* R = d.rot;
        float q[4];
        const float tr = R[0] + R[4] + R[8];
        if (tr > 0.f) {
            const float S = fsqrt(tr + 1.f) * 2.f, iS = frcp(S);
            q[0] = 0.25f * S; q[1] = (R[7] - R[5]) * iS; q[2] = (R[2] - R[6]) * iS; q[3] = (R[3] - R[1]) * iS;
        } else if (R[0] > R[4] && R[0] > R[8]) {
            const float S = fsqrt(1.f + R[0] - R[4] - R[8]) * 2.f, iS = frcp(S);
            q[0] = (R[7] - R[5]) * iS; q[1] = 0.25f * S; q[2] = (R[1] + R[3]) * iS; q[3] = (R[2] + R[6]) * iS;
        } else if (R[4] > R[8]) {
            const float S = fsqrt(1.f + R[4] - R[0] - R[8]) * 2.f, iS = frcp(S);
            q[0] = (R[2] - R[6]) * iS; q[1] = (R[1] + R[3]) * iS; q[2] = 0.25f * S; q[3] = (R[5] + R[7]) * iS;
        } else {
            const float S = fsqrt(1.f + R[8] - R[0] - R[4]) * 2.f, iS = frcp(S);
            q[0] = (R[3] - R[1]) * iS; q[1] = (R[2] + R[6]) * iS; q[2] = (R[5] + R[7]) * iS; q[3] = 0.25f * S;
        }
        // quatXquat + quat2R (quad_utils.py:146-174)
        const float w = q[0] * qt[0] - q[1] * qt[1] - q[2] * qt[2] - q[3] * qt[3];
        const float x = q[0] * qt[1] + q[1] * qt[0] - q[2] * qt[3] + q[3] * qt[2];
        const float y = q[0] * qt[2] + q[1] * qt[3] + q[2] * qt[0] - q[3] * qt[1];
        const float zz = q[0] * qt[3] - q[1] * qt[2] + q[2] * qt[1] + q[3] * qt[0];
        nr[0] = 1.f - 2.f * y * y - 2.f * zz * zz; nr[1] = 2.f * x * y - 2.f * zz * w; nr[2] = 2.f * x * zz + 2.f * y * w;
        nr[3] = 2.f * x * y + 2.f * zz * w; nr[4] = 1.f - 2.f * x * x - 2.f * zz * zz; nr[5] = 2.f * y * zz - 2.f * x * w;
        nr[6] = 2.f * x * zz - 2.f * y * w; nr[7] = 2.f * y * zz + 2.f * x * w; nr[8] = 1.f - 2.f * x * x - 2.f * y * y;
    } else {
#pragma unroll
        for (int i = 0; i < 3; ++i) { np_[i] = d.pos[i]; nv[i] = d.vel[i]; no[i] = d.om[i]; }
#pragma unroll
        for (int i = 0; i < 9; ++i) nr[i] = d.rot[i];
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        out[i] = np_[i] - d.goal[i];
        out[3 + i] = nv[i];
        out[15 + i] = no[i];
    }
#pragma unroll
    for (int i = 0; i < 9; ++i) out[6 + i] = nr[i];
    if (kp.obs_repr == QS_OBS_XYZ_VXYZ_R_OMEGA_FLOOR) out[18] = np_[2];
    if (kp.obs_repr == QS_OBS_XYZ_VXYZ_R_OMEGA_WALL) {
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            out[18 + i] = clampf(np_[i] - kp.room_lo[i], 0.f, 5.f);
            out[21 + i] = clampf(kp.room_hi[i] - np_[i], 0.f, 5.f);
        }
    }
}

__device__ __forceinline__ void self_obs(const KP& kp, const Drone& d, const Rng& rng, uint32_t gid, uint32_t stream,
                                         float* out) {
    float z[12];
    if (kp.sense) {
        normals4(rng, gid, stream, 0, z);
        normals4(rng, gid, stream, 1, z + 4);
        normals4(rng, gid, stream, 2, z + 8);
    }
    self_obs_z(kp, d, z, rng, gid, stream, out);
}

__device__ __forceinline__ void xch_put(float4* xch, int lane, const float* P, const float* V) {
    xch[2 * lane] = make_float4(P[0], P[1], P[2], 0.f);
    xch[2 * lane + 1] = make_float4(V[0], V[1], V[2], 0.f);
}

// pos_vel neighbour obs: neighborhood_indices (quadrotor_multi.py:344-375) + extend_obs_space
// clip (:328-342).  Key = |[rel_pos, rel_vel]| clamped at 0.01 (compared squared, clamp 1e-4);
// stable (index) tie-break like numpy's insertion sort; k == N-1 keeps index order (all keys 0).
// Reads the exchange tile (caller has synchronised).  With Q sub-lanes per drone, sub-lane q owns
// the candidates j = q + Q t: it builds their keys, gathers the other sub-lanes' keys by DPP, ranks
// its own candidates and writes those that land among the K nearest.  Only write == true stores.
template <int NPAD, int Q>
__device__ __forceinline__ void neighbor_obs(const KP& kp, const float4* xch, int dbase, int di, int q, const float* P, const float* V,
                             bool write, float* out) {
    constexpr int PJ = (NPAD + Q - 1) / Q;   // candidates per sub-lane
    constexpr bool KEEP = PJ <= 8;           // keep the relative vectors in VGPRs between passes
    float key[PJ];
    float rel[KEEP ? PJ : 1][6];
    const bool sorted = kp.K < kp.N - 1;
#pragma unroll
    for (int t = 0; t < PJ; ++t) {
        const int j = q + Q * t;
        const int jj = j < NPAD ? j : NPAD - 1;
        const float4 pj = xch[2 * (dbase + jj)], vj = xch[2 * (dbase + jj) + 1];
        const float r[6] = {pj.x - P[0], pj.y - P[1], pj.z - P[2], vj.x - V[0], vj.y - V[1], vj.z - V[2]};
        const float s = r[0] * r[0] + r[1] * r[1] + r[2] * r[2] + r[3] * r[3] + r[4] * r[4] + r[5] * r[5];
        const bool valid = (j != di) && (j < kp.N);
        key[t] = valid ? (sorted ? fmaxf(s, 1e-4f) : 0.f) : __builtin_inff();
        if (KEEP) {
#pragma unroll
            for (int c = 0; c < 6; ++c) rel[KEEP ? t : 0][c] = r[c];
        }
    }
    float allk_[Q == 1 || NPAD >= 64 ? 1 : PJ * Q];   // key of candidate m = q' + Q t' (sub-lane q', slot t')
    float* allk = Q == 1 || NPAD >= 64 ? key : allk_;
#pragma unroll
    for (int t = 0; t < PJ; ++t) {
        if constexpr (Q == 1 || NPAD >= 64) {   // (the K-pass selection below needs no gathered keys)
        } else if constexpr (Q == 2) {
            allk[2 * t] = qbc<2, 0>(key[t]);
            allk[2 * t + 1] = qbc<2, 1>(key[t]);
        } else {
            allk[4 * t] = qbc<4, 0>(key[t]);
            allk[4 * t + 1] = qbc<4, 1>(key[t]);
            allk[4 * t + 2] = qbc<4, 2>(key[t]);
            allk[4 * t + 3] = qbc<4, 3>(key[t]);
        }
    }
    if (!write) return;
    const float vm = 2.f * kp.vxyz_max;
    const bool pairs = ((kp.so_dim | kp.obs_dim) & 1) == 0;   // 8-byte aligned slots: ds_write_b64
    if constexpr (NPAD >= 64) {
        // 128-drone envs and the sub-lane (multi-wave) envs always take this path (k = N - 1 keys are all 0: the
        // passes pick index order, as the ranking does); their ranking is not compiled
        if (NPAD > 64 || Q > 1 || (sorted && kp.K <= 16)) {
            // many candidates, few neighbours: K passes of a (key, index) minimum above the previous pick instead
            // of ranking every candidate against all the others -- the same strict (key, index) order, so the
            // same neighbours in the same slots.  With 2 sub-lanes each scans its candidates j = q + 2 m and the
            // pair's two minima meet by one DPP swap.
            float pk = -1.f;
            int pjx = -1;
            for (int r = 0; r < kp.K; ++r) {
                float bk = __builtin_inff();
                int bj = NPAD;
#pragma unroll
                for (int m = 0; m < PJ; ++m) {
                    const int j = q + Q * m;
                    const bool above = key[m] > pk || (key[m] == pk && j > pjx);
                    const bool below = key[m] < bk;   // j ascending: the first of equal keys wins
                    if (above && below) { bk = key[m]; bj = j; }
                }
                if constexpr (Q == 2) {
                    const float ok = dpp_f<quad_perm(1, 0, 3, 2)>(bk);
                    const int oj = dpp_i<quad_perm(1, 0, 3, 2)>(bj);
                    if (ok < bk || (ok == bk && oj < bj)) { bk = ok; bj = oj; }
                }
                if (bk == __builtin_inff()) break;
                pk = bk;
                pjx = bj;
                if (Q > 1 && q != 0) continue;   // the pair's first sub-lane writes the slot
                const float4 pj = xch[2 * (dbase + bj)], vj = xch[2 * (dbase + bj) + 1];
                const float o0 = clampf(pj.x - P[0], -kp.room_range[0], kp.room_range[0]);
                const float o1 = clampf(pj.y - P[1], -kp.room_range[1], kp.room_range[1]);
                const float o2 = clampf(pj.z - P[2], -kp.room_range[2], kp.room_range[2]);
                const float o3 = clampf(vj.x - V[0], -vm, vm), o4 = clampf(vj.y - V[1], -vm, vm);
                const float o5 = clampf(vj.z - V[2], -vm, vm);
                float* o = out + kp.so_dim + r * 6;
                o[0] = o0; o[1] = o1; o[2] = o2; o[3] = o3; o[4] = o4; o[5] = o5;
            }
            return;
        }
    }
    if constexpr (NPAD < 64 || (NPAD == 64 && Q == 1)) {
#pragma unroll
    for (int t = 0; t < PJ; ++t) {
        const int j = q + Q * t;
        int rank = 0;
#pragma unroll
        for (int m = 0; m < PJ * Q; ++m) rank += (allk[m] < key[t]) || (m < j && allk[m] == key[t]);
        if (key[t] != __builtin_inff() && rank < kp.K) {
            float r[6];
            if (KEEP) {
#pragma unroll
                for (int c = 0; c < 6; ++c) r[c] = rel[KEEP ? t : 0][c];
            } else {
                const float4 pj = xch[2 * (dbase + j)], vj = xch[2 * (dbase + j) + 1];
                r[0] = pj.x - P[0]; r[1] = pj.y - P[1]; r[2] = pj.z - P[2];
                r[3] = vj.x - V[0]; r[4] = vj.y - V[1]; r[5] = vj.z - V[2];
            }
            const float o0 = clampf(r[0], -kp.room_range[0], kp.room_range[0]);
            const float o1 = clampf(r[1], -kp.room_range[1], kp.room_range[1]);
            const float o2 = clampf(r[2], -kp.room_range[2], kp.room_range[2]);
            const float o3 = clampf(r[3], -vm, vm), o4 = clampf(r[4], -vm, vm), o5 = clampf(r[5], -vm, vm);
            float* o = out + kp.so_dim + rank * 6;
            if (pairs) {
                float2* o2p = reinterpret_cast<float2*>(o);
                o2p[0] = make_float2(o0, o1);
                o2p[1] = make_float2(o2, o3);
                o2p[2] = make_float2(o4, o5);
            } else {
                o[0] = o0; o[1] = o1; o[2] = o2; o[3] = o3; o[4] = o4; o[5] = o5;
            }
        }
    }
    }
}

// ---------------------------------------------------------------------------------------------
// interactions
// ---------------------------------------------------------------------------------------------
// compute_new_vel (collisions/utils.py:7-20)
__device__ __forceinline__ void new_vel(float maxv, float* v, const float* sh, float ratio) {
    const float n0 = v[0] + sh[0], n1 = v[1] + sh[1], n2 = v[2] + sh[2];
    const float mag = fsqrt(n0 * n0 + n1 * n1 + n2 * n2);
    const float inv = frcp(mag == 0.f ? 1e-5f : mag);
    const float nm = fminf(mag * ratio, maxv);
    v[0] += n0 * inv * nm - v[0];
    v[1] += n1 * inv * nm - v[1];
    v[2] += n2 * inv * nm - v[2];
}

// perform_collision_between_drones (collisions/quadrotors.py:23-59) for the pair (1 = lower id).
// Both drones of the pair evaluate it with identical inputs and draws (key = lower drone, stream j):
// z = normals 0..27 (blocks 0..6: the 3 rejection tries use normals t*9 .. t*9+8), u = uniforms 0..7.
__device__ __forceinline__ void collide_pair(const float* p1, float* v1, float* w1, const float* p2, float* v2, float* w2,
                             const float* z, const float* u) {
    float n[3] = {p1[0] - p2[0], p1[1] - p2[1], p1[2] - p2[2]};
    const float m = fsqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
    const float im = frcp(m == 0.f ? 1e-5f : m);
    n[0] *= im; n[1] *= im; n[2] *= im;
    const float v1n = v1[0] * n[0] + v1[1] * n[1] + v1[2] * n[2];
    const float v2n = v2[0] * n[0] + v2[1] * n[1] + v2[2] * n[2];
    float vc[3], s1[3], s2[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) { vc[i] = (v2n - v1n) * n[i]; s1[i] = vc[i]; s2[i] = -vc[i]; }
#pragma unroll
    for (int t = 0; t < 3; ++t) {  // "make sure new vel direction would be opposite" rejection, 3 tries
        float d1 = 0.f, d2 = 0.f;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const float cons = 0.8f * z[t * 9 + i], a = 0.15f * z[t * 9 + 3 + i], bb = 0.15f * z[t * 9 + 6 + i];
            s1[i] = vc[i] + (cons + a);
            s2[i] = -vc[i] + (-cons + bb);
            d1 += (v1[i] + s1[i]) * n[i];
            d2 += (v2[i] + s2[i]) * n[i];
        }
        if (d1 > 0.f && 0.f > d2) break;
    }
    const float mx = fmaxf(fsqrt(v1[0] * v1[0] + v1[1] * v1[1] + v1[2] * v1[2]),
                           fsqrt(v2[0] * v2[0] + v2[1] * v2[1] + v2[2] * v2[2]));
    new_vel(mx, v1, s1, 0.2f + 0.6f * u[0]);
    new_vel(mx, v2, s2, 0.2f + 0.6f * u[1]);
    // compute_new_omega (collisions/utils.py:23-33), magn_scale 20
    const float om = 20.f * 3.14159265358979f;
    float w[3] = {-1.f + 2.f * u[2], -1.f + 2.f * u[3], -1.f + 2.f * u[4]};
    const float wm = fsqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
    const float iw = frcp(wm == 0.f ? 1e-5f : wm);
    const float mg = om * 0.5f + (om - om * 0.5f) * u[5];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const float x = w[i] * iw * mg;
        w1[i] += x;
        w2[i] -= x;
    }
}

// perform_collision_with_wall (collisions/room.py:6-44) / _with_ceiling (:91-113); u = uniforms 0..11
// of stream S_WALL / S_CEIL
__device__ __forceinline__ void collide_room(const KP& kp, Drone& d, const float* u, bool wall) {
    const float sp = fsqrt(d.vel[0] * d.vel[0] + d.vel[1] * d.vel[1] + d.vel[2] * d.vel[2]);
    const float real = clampf(0.2f * sp + (0.8f * sp - 0.2f * sp) * u[0], 0.1f, 6.0f);
    float dir[3] = {-1.f + 2.f * u[1], -1.f + 2.f * u[2], -1.f + 2.f * u[3]};
    int ow;
    if (wall) {
        if (d.pos[0] == kp.room_lo[0]) dir[0] = 0.1f + 0.9f * u[4];
        else if (d.pos[0] == kp.room_hi[0]) dir[0] = -1.f + 0.9f * u[4];
        if (d.pos[1] == kp.room_lo[1]) dir[1] = 0.1f + 0.9f * u[5];
        else if (d.pos[1] == kp.room_hi[1]) dir[1] = -1.f + 0.9f * u[5];
        dir[2] = -1.f + 0.5f * u[6];
        ow = 7;
    } else {
        dir[2] = -1.f + 0.5f * u[4];
        ow = 5;
    }
    const float idm = frcp(fsqrt(dir[0] * dir[0] + dir[1] * dir[1] + dir[2] * dir[2]) + 1e-5f);
    float w[3] = {-1.f + 2.f * u[ow], -1.f + 2.f * u[ow + 1], -1.f + 2.f * u[ow + 2]};
    const float iw = frcp(fsqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]) + 1e-5f);
    const float om = 20.f * 3.14159265358979f;
    const float mg = om * 0.5f + (om - om * 0.5f) * u[ow + 3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        d.vel[i] = real * (dir[i] * idm);
        d.om[i] += w[i] * iw * mg;
    }
}

// ---------------------------------------------------------------------------------------------
// reset (QuadrotorSingle._reset quadrotor_single.py:401-469): spawn = spawn point + U(-box, box)^3
// (static_same_goal: the goal, box 2; obstacle scenarios: a free grid cell, box 0.1)
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void reset_drone(const KP& kp, Drone& d, const Rng& rng, uint32_t gid, const float* spawn,
                            const float* goal) {
    float u[4];
    uniforms4(rng, gid, S_RESET, 0, u);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        d.goal[i] = goal[i];
        d.pos[i] = (-kp.spawn_box + 2.f * kp.spawn_box * u[i]) + spawn[i];
        d.vel[i] = 0.f;
        d.om[i] = 0.f;
    }
    if (d.pos[2] < 0.75f) d.pos[2] = 0.75f;
    // randyaw rejection until the body x axis points within 60 deg of the origin (:454-456)
    float tx = -d.pos[0], ty = -d.pos[1];
    const float tn = fsqrt(tx * tx + ty * ty);
    const bool degenerate = tn < 1e-5f;
    tx = degenerate ? 0.f : tx / tn;
    ty = degenerate ? 0.f : ty / tn;
    float yaw = 0.f;
    for (uint32_t blk = 0; blk < 64; ++blk) {
        float y[4];
        uniforms4(rng, gid, S_RESET_YAW, blk, y);
        bool found = false;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if (found) continue;
            const float cand = -3.14159265358979f + 6.28318530717959f * y[i];
            float s, c;
            sincos_hw(cand, &s, &c);
            yaw = cand;
            if (c * tx + s * ty >= 0.5f || degenerate) found = true;
        }
        if (found) break;
    }
    yaw_rot(yaw, d.rot);
#pragma unroll
    for (int k = 0; k < 4; ++k) { d.rd[k] = 0.f; d.cd[k] = 0.f; }
    d.flags = 0;
    d.prev = 0;
    d.prevx = 0;
}

// ---------------------------------------------------------------------------------------------
// obstacles: pillars on an n x n grid of 1 m cells, xy only
// ---------------------------------------------------------------------------------------------
// (cell_xy: grid cell -> cell centre, qs_scen.h)


// partial Fisher-Yates (the first k of a random permutation of 0..n-1): the Philox stand-in for
// np.random.choice(n, k, replace=False); a: LDS scratch of n bytes, out: k picks
__device__ __forceinline__ void choose_k(const Rng& r, uint32_t id, uint32_t st, uint32_t u0, int n, int k, uint8_t* a, uint8_t* out) {
    for (int i = 0; i < n; ++i) a[i] = (uint8_t)i;
    for (int i = 0; i < k; ++i) {
        int j = i + ufloor(ubits(r, id, st, u0 + (uint32_t)i), n - i);
        j = min(j, n - 1);
        const uint8_t t = a[i];
        a[i] = a[j];
        a[j] = t;
        out[i] = a[i];
    }
}

// per-env reset scratch in LDS (QS_OBST_SCRATCH bytes per env)
constexpr int QS_OBST_SCRATCH = 400;
struct ObstScratch {
    uint8_t perm[64], map[64], fr[64], dp[64], sp[32], gl[32], ids[64];
    float ez;
    int mode;     // 0 o_random, 1 o_static_same_goal, 2 o_swap_goals, 3 o_ep_rand_bezier, 4 o_dynamic_same_goal
    int mi, si;   // domain randomisation: the env's pillar count / size table indices (in: current, out: new)
};
// the episode_extra_stats scenario id of an obstacle mode (quadswarm_amd.stats: 16 o_random, 17 o_static_same_goal,
// 19 o_swap_goals, 20 o_ep_rand_bezier, 21 o_dynamic_same_goal; 18 is flavor A's dynamic_repulsive)
__device__ __forceinline__ int obst_stats_id(int mode) { return mode < 2 ? 16 + mode : 17 + mode; }

// The env's pillar geometry: count, radius, collision threshold (arm + radius).  Without domain
// randomisation these are the (specialised) constants; with it, the env's table entries.
struct OGeo {
    int m;
    float r, thr;
};
__device__ __forceinline__ OGeo ogeo(const KP& kp, int mi, int si) {
    if (!kp.dr) return OGeo{kp.M, kp.obst_r, kp.obst_thr};
    return OGeo{kp.dr_m[mi], kp.dr_r[si], kp.dr_thr[si]};
}
static_assert(sizeof(ObstScratch) <= QS_OBST_SCRATCH, "obstacle scratch");

// the max_square_area_center cell of the env's map (Scenario_o_base, o_base.py:125-153): dp's first row and column
// start as the map itself, the centre is (i - (s-1)//2, j - (s-1)//2)
__device__ __forceinline__ int obst_max_square_cell(ObstScratch* sc, int n) {
    const int nn = n * n;
    for (int c = 0; c < nn; ++c) sc->dp[c] = 0;
    for (int j = 0; j < n; ++j) sc->dp[j] = sc->map[j];
    for (int i = 0; i < n; ++i) sc->dp[i * n] = sc->map[i * n];
    int ms = 0, cx = 0, cy = 0;
    for (int i = 1; i < n; ++i)
        for (int j = 1; j < n; ++j)
            if (sc->map[i * n + j] == 0) {
                const int v = min(min(sc->dp[(i - 1) * n + j], sc->dp[i * n + j - 1]), sc->dp[(i - 1) * n + j - 1]) + 1;
                sc->dp[i * n + j] = (uint8_t)v;
                if (v > ms) { ms = v; cx = i - (ms - 1) / 2; cy = j - (ms - 1) / 2; }
            }
    return cx * n + cy;
}

// Obstacle map + scenario of one env (quadrotor_multi.py:405-426, 449-452; scenarios/mix.py:78-99;
// o_random.py:26-51; o_static_same_goal.py:28-48; o_base.py:58-153; the dynamic modes o_swap_goals.py:27-52,
// o_ep_rand_bezier.py:55-103, o_dynamic_same_goal.py:31-51).  One lane per env runs it; the other lanes of the env
// read sp/gl/mode/ez (and, dynamic modes, their goal rows in gtab) after a barrier.  Writes the env's obstacle list;
// for the dynamic modes also `so`, the scenario record (stored by the caller) -- the draws of their scenario
// parameters are one Philox word each on stream S_SCN_RESET (key: the env's drone 0), in this order:
//   o_swap_goals          duration U(4, 6), formation, size, layer dist, end z U(1.5, 3), the goals' shuffle
//   o_ep_rand_bezier      end cell (choice of the free cells), end z U(0.75, 3)
//   o_dynamic_same_goal   duration U(4, 6), end z U(1.5, 3)
// (the reference's o_ep_rand_bezier also samples 10 trajectory points it never uses: not drawn here).
__device__ __forceinline__ void obstacle_reset_env(const KP& kp, const Rng& r, uint32_t genv, ObstScratch* sc, float2* ob,
                                                   Scen* so = nullptr, float* gtab = nullptr) {
    if (kp.dr) {   // the replay wrapper's reset: np.random.choice of density, then of size (quad_experience_replay.py:106-118)
        if (kp.dr_nm > 0) {
            const int c = ufloor(ubits(r, genv, S_DR, 0), kp.dr_nm);
            if (kp.dr_m[c + 1] >= 0) sc->mi = c + 1;   // a 0.0 density is falsy: keep (quadrotor_multi.py:443)
        }
        if (kp.dr_ns > 0) {
            const int c = ufloor(ubits(r, genv, S_DR, 1), kp.dr_ns);
            if (kp.dr_r[c + 1] > 0.f) sc->si = c + 1;
        }
    }
    const int n = kp.obst_n, nn = n * n, M = ogeo(kp, sc->mi, sc->si).m, N = kp.N;
    for (int c = 0; c < nn; ++c) sc->map[c] = 0;
    choose_k(r, genv, S_OBSTMAP, 0, nn, M, sc->perm, sc->ids);
    for (int o = 0; o < M; ++o) {
        sc->map[sc->ids[o]] = 1;
        ob[o] = cell_xy(sc->ids[o], n);
    }
    int mode = kp.obst_scen == 0 ? (int)(ubits(r, genv, S_OSCEN, 0) >> 31) : kp.obst_scen - 1;
    int F = 0;
    for (int c = 0; c < nn; ++c)
        if (!sc->map[c]) sc->fr[F++] = (uint8_t)c;
    choose_k(r, genv, S_OSCEN, 1, F, N, sc->perm, sc->sp);
    for (int i = 0; i < N; ++i) sc->sp[i] = sc->fr[sc->sp[i]];
    if (mode == 0) {   // o_random: own goal cell per drone
        choose_k(r, genv, S_OSCEN, 1 + (uint32_t)N, F, N, sc->perm, sc->gl);
        for (int i = 0; i < N; ++i) sc->gl[i] = sc->fr[sc->gl[i]];
    } else if (mode == 1) {   // o_static_same_goal: Scenario_o_base.max_square_area_center (o_base.py:125-153)
        const int cell = obst_max_square_cell(sc, n);
        for (int i = 0; i < N; ++i) sc->gl[i] = (uint8_t)cell;
        sc->ez = 1.5f + 1.5f * uniform1(r, genv, S_OSCEN, 2 * (uint32_t)N + 1);
    } else if (so != nullptr && gtab != nullptr) {   // the dynamic modes: goals into gtab rows, the record into so
        Scen& s = *so;
        s = Scen{};
        s.mode = obst_stats_id(mode);
        SDraw sd = sdraw(r, genv, S_SCN_RESET);
        const float cf = 1.f / kp.cdt;
        if (mode == 3) {   // o_ep_rand_bezier: end point = generate_pos_obst_map(); the curve is sampled at tick 1
            const float2 xy = cell_xy(sc->fr[sd_int(sd, 0, F)], n);
            s.c[0] = xy.x; s.c[1] = xy.y; s.c[2] = sd_uniform(sd, 0.75f, 3.f);
            s.period = (int)(0.01f * cf);
            for (int i = 0; i < N; ++i)
                for (int k = 0; k < 3; ++k) gtab[4 * i + k] = s.c[k];
        } else {
            s.period = (int)(sd_uniform(sd, 4.f, 6.f) * cf);   // duration_time ~ U(4, 6)
            if (mode == 2) {   // o_swap_goals: a formation (update_formation_and_relate_param) around the centre
                Scen f{};
                f.mode = SC_O_SWAP_GOALS;
                sc_update_formation(kp, f, sd);
                s.form = f.form; s.lo = f.lo; s.hi = f.hi; s.size = f.size; s.layer = f.layer;
            }
            const float2 xy = cell_xy(obst_max_square_cell(sc, n), n);   // max_square_area_center()
            s.c[0] = xy.x; s.c[1] = xy.y; s.c[2] = sd_uniform(sd, 1.5f, 3.f);
            if (mode == 2) {   // generate_goals(num_agents, formation_center, layer_dist), np.random.shuffle(goals)
                const int m = sc_generate(s.form, sc_num(kp), sc_per_layer(s.form), s.size, s.layer, s.c, gtab);
                sd_shuffle(sd, gtab, m);
                // a sphere of N < 3 drones has 3 goal rows: the scenario keeps the ones no drone takes in c1 / c2
                for (int k = 0; k < 3; ++k) {
                    if (m > N) s.c1[k] = gtab[4 * N + k];
                    if (m > N + 1) s.c2[k] = gtab[4 * (N + 1) + k];
                }
            } else {           // o_dynamic_same_goal: every drone's goal is the end point
                for (int i = 0; i < N; ++i)
                    for (int k = 0; k < 3; ++k) gtab[4 * i + k] = s.c[k];
            }
        }
    }
    sc->mode = mode;
}

// spawn point and goal of drone `di` after obstacle_reset_env (o_base.py:81-92: z ~ U(1, 3)); the dynamic modes'
// goals are gtab's rows
__device__ __forceinline__ void obstacle_spawn_goal(const KP& kp, const ObstScratch* sc, int di, const Rng& r,
                                                    uint32_t gid, float* spawn, float* goal, const float* gtab = nullptr) {
    float u[4];
    uniforms4(r, gid, S_RESET, 0, u);   // u[3] = start z, block 1 word 0 = goal z
    const float2 s = cell_xy(sc->sp[di], kp.obst_n), g = cell_xy(sc->gl[di], kp.obst_n);
    spawn[0] = s.x; spawn[1] = s.y; spawn[2] = 1.f + 2.f * u[3];
    if (sc->mode >= 2 && gtab != nullptr) {
        for (int k = 0; k < 3; ++k) goal[k] = gtab[4 * di + k];
        return;
    }
    goal[0] = g.x; goal[1] = g.y;
    goal[2] = sc->mode == 0 ? 1.f + 2.f * uniform1(r, gid, S_RESET, 4) : sc->ez;
}


// get_surround_sdfs (obstacles/utils.py:4-27)
__device__ __forceinline__ void sdf_obs(const KP& kp, const OGeo& og, const float2* ob, float x, float y, float* out) {
    const float res = kp.sdf_res;
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b) {
            const float gx = x + (float)(a - 1) * res, gy = y + (float)(b - 1) * res;
            float m2 = 1.0e4f;   // (100 m)^2
            for (int o = 0; o < og.m; ++o) {
                const float dx = gx - ob[o].x, dy = gy - ob[o].y;
                m2 = fminf(m2, dx * dx + dy * dy);
            }
            out[a * 3 + b] = fsqrt(m2) - og.r;
        }
}

// the same 9 points dealt over the drone's Q sub-lanes (point p on sub-lane p % Q), each written to its
// slot of the drone's obs row by the sub-lane that computed it: the same arithmetic per point
template <int Q>
__device__ __forceinline__ void sdf_obs_q(const KP& kp, const OGeo& og, const float2* ob, float x, float y, float* out,
                                          int q) {
    const float res = kp.sdf_res;
#pragma unroll
    for (int t = 0; t < (9 + Q - 1) / Q; ++t) {
        const int p = q + Q * t;
        if (p >= 9) continue;
        const int a = p / 3, b = p % 3;
        const float gx = x + (float)(a - 1) * res, gy = y + (float)(b - 1) * res;
        float m2 = 1.0e4f;   // (100 m)^2
        for (int o = 0; o < og.m; ++o) {
            const float dx = gx - ob[o].x, dy = gy - ob[o].y;
            m2 = fminf(m2, dx * dx + dy * dy);
        }
        out[p] = fsqrt(m2) - og.r;
    }
}

// collision_detection (obstacles/utils.py:30-43): first obstacle within arm + radius
__device__ __forceinline__ int obst_detect(const OGeo& og, const float2* ob, float x, float y) {
    for (int o = 0; o < og.m; ++o) {
        const float dx = x - ob[o].x, dy = y - ob[o].y;
        if (fsqrt(dx * dx + dy * dy) <= og.thr) return o;
    }
    return -1;
}

// the same test dealt over the drone's Q sub-lanes: sub-lane q scans pillars q, q + Q, ... and the smallest
// index hit over the sub-lanes (DPP min) is the first pillar of the sequential scan
template <int Q>
__device__ __forceinline__ int obst_detect_q(const OGeo& og, const float2* ob, float x, float y, int q) {
    int first = 0x7fffffff;
    for (int o = q; o < og.m; o += Q) {
        const float dx = x - ob[o].x, dy = y - ob[o].y;
        if (fsqrt(dx * dx + dy * dy) <= og.thr) {
            first = o;
            break;
        }
    }
    if constexpr (Q >= 2) first = min(first, dpp_i<quad_perm(1, 0, 3, 2)>(first));
    if constexpr (Q >= 4) first = min(first, dpp_i<quad_perm(2, 3, 0, 1)>(first));
    return first == 0x7fffffff ? -1 : first;
}

// perform_collision_with_obstacle (collisions/obstacles.py:23-50); Philox indices as the oracle's:
// z = normals 0..19 of S_OBST (try t uses t*6 .. t*6+5), u = uniforms 0..7
__device__ __forceinline__ void collide_obstacle(const KP& kp, const OGeo& og, Drone& d, float ox, float oy,
                                                 const float* z, const float* u) {
    float n[3] = {d.pos[0] - ox, d.pos[1] - oy, 0.f};
    const float nm = fsqrt(n[0] * n[0] + n[1] * n[1]);
    const float inm = frcp(nm == 0.f ? 1e-5f : nm);
    n[0] *= inm; n[1] *= inm;
    const float vm = fsqrt(d.vel[0] * d.vel[0] + d.vel[1] * d.vel[1] + d.vel[2] * d.vel[2]);
    const float nv[3] = {vm * n[0], vm * n[1], 0.f};
    float noise[3] = {0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 3; ++t) {
        float tmp[3], dt_ = 0.f;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            tmp[c] = 0.1f * z[t * 6 + c] + 0.05f * z[t * 6 + 3 + c];
            dt_ += (nv[c] + tmp[c]) * n[c];
        }
        if (dt_ > 0.f) {
            noise[0] = tmp[0]; noise[1] = tmp[1]; noise[2] = tmp[2];
            break;
        }
    }
    const float dz = d.pos[2] - kp.obst_z;
    const bool inside = fsqrt(nm * nm + dz * dz) < og.r;
    float sh[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) sh[c] = nv[c] - d.vel[c] + noise[c];
    new_vel(vm, d.vel, sh, inside ? 1.f : 0.2f + 0.6f * u[0]);
    const float om = 3.14159265358979f;   // compute_new_omega(magn_scale=1.0)
    float w[3] = {-1.f + 2.f * u[1], -1.f + 2.f * u[2], -1.f + 2.f * u[3]};
    const float wm = fsqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
    const float iw = frcp(wm == 0.f ? 1e-5f : wm);
    const float mg = om * 0.5f + (om - om * 0.5f) * u[4];
#pragma unroll
    for (int c = 0; c < 3; ++c) d.om[c] += w[c] * iw * mg;
}

// LDS of a launch with `slots` drone rows per workgroup: obs tile [slots, obs_dim] | exchange tile
// [slots x 2 float4] | 64 words | obstacle tiles [EPB, M] float2 | obstacle reset scratch [EPB]
// (qs_lds_bytes() in qs_step.hip sizes it)
__device__ __forceinline__ float2* obst_tile(float* lds, const KP& kp, int slots) {
    return reinterpret_cast<float2*>(lds + slots * kp.obs_dim + slots * 8 + 64);
}
// the goal-scenario tables (qs_scen.h scen_tab): after the obstacle tiles and reset scratch in obstacle kernels
template <bool OBST>
__device__ __forceinline__ float* scen_tab_b(float* lds, const KP& kp, int slots, int epb) {
    return scen_tab(lds, kp, slots) + (OBST ? epb * (2 * kp.M + QS_OBST_SCRATCH / 4) : 0);
}

// Geometry of the flavor-B step kernel: Q lanes per drone (Q * NPAD <= 64), EPB envs per wave.
// Cooperative state load / store of the Q sub-lanes of a drone (flavor-B step).  The drone's state words
// (33 fp32 fields QS_F_POS .. QS_F_GOAL, then the NIW int fields QS_I_* a swarm of its size uses: 2 for
// single drones, 3 up to 32, 4 up to 64, 6 at 128 -- StepGeo::NIW) are dealt over the sub-lanes:
// instruction t moves word t*Q + q on sub-lane q, so a wave instruction covers Q fields x its drones and
// the drone needs ceil(37 / Q) load / store instructions instead of 37.  Loaded words are broadcast to
// every sub-lane by DPP (every sub-lane holds the whole drone).  Addresses are b.st (SGPRs) + a 32-bit
// per-lane byte offset: the int fields are reached through their offset from b.st (istate follows state
// in the handle's workspace, qs_step.hip layout).
constexpr int DRONE_WORDS = QS_F_GOAL + 3 + 4;
// with episode_extra_stats on, the step also loads the drone's distance ring and window sums (fields
// QS_F_DRING .. QS_F_DSUM + 2) in the same batch: words DRONE_WORDS .. LOAD_WORDS - 1
constexpr int STAT_WORDS = 8;
constexpr int LOAD_WORDS = DRONE_WORDS + STAT_WORDS;

// 128-drone envs carry NIW = 6 istate words (the 128-bit collision row, QS_I_PREV_2 / _3): the drone's words
// are then the 33 fp32 fields, 6 int fields and the stats words
template <int NIW>
struct WordsOf {
    static constexpr int DW = QS_F_GOAL + 3 + NIW, LW = DW + STAT_WORDS;
};

template <int Q, int W, int T, int LW = LOAD_WORDS>
__device__ __forceinline__ void qbc_words(const uint32_t (&r)[T], uint32_t* wv) {
    if constexpr (W < LW && W / Q < T) {
        wv[W] = (uint32_t)__float_as_int(qbc<Q, W % Q>(__int_as_float((int)r[W / Q])));
        qbc_words<Q, W + 1, T, LW>(r, wv);
    }
}

template <int NIW = 4>
__device__ __forceinline__ uint32_t drone_word_off(const KP& kp, const Bufs& b, int w, uint32_t go) {
    constexpr int DW = WordsOf<NIW>::DW;
    const uint32_t I4 = (uint32_t)kp.I * 4u;
    const uint32_t ist0 = (uint32_t)((const char*)b.ist - (const char*)b.st);
    if (w >= DW) return (uint32_t)(QS_F_DRING + w - DW) * I4 + go;
    return (w < QS_F_GOAL + 3 ? (uint32_t)w * I4 : ist0 + (uint32_t)(w - QS_F_GOAL - 3) * I4) + go;
}

template <int Q, int NW = DRONE_WORDS>
struct DroneWords {
    static constexpr int T = (NW + Q - 1) / Q;
    uint32_t r[T];
};
// issue the sub-lane's state-word loads (no wait): the first nw <= NW words
template <int Q, int NW, int NIW = 4>
__device__ __forceinline__ void load_words_q(const KP& kp, const Bufs& b, int g, int q, DroneWords<Q, NW>& dw,
                                             int nw = NW) {
    const uint32_t go = (uint32_t)g * 4u;
#pragma unroll
    for (int t = 0; t < DroneWords<Q, NW>::T; ++t) {
        const int w = t * Q + q;
        dw.r[t] = w < nw ? *reinterpret_cast<const uint32_t*>((const char*)b.st + drone_word_off<NIW>(kp, b, w, go)) : 0u;
    }
}
// the drone on every sub-lane; stw (if given) gets the STAT_WORDS words as floats
// DEAL (Q = 4, QS_DEAL_MOTORS): the motor words 18..29 are the sub-lane's own motor's (no broadcast; see motors_dealt4)
template <int Q, int NW, int NIW = 4, bool DEAL = false>
__device__ __forceinline__ void unpack_words_q(const DroneWords<Q, NW>& dw, Drone& d, float* stw = nullptr, int q = 0) {
    constexpr int T = DroneWords<Q, NW>::T, DW = WordsOf<NIW>::DW;
    const uint32_t (&r)[T] = dw.r;
    uint32_t wv[T * Q > DW ? T * Q : DW];
    qbc_words<Q, 0, T, WordsOf<NIW>::LW>(r, wv);
    if constexpr (NW > DW) {
        if (stw) {
#pragma unroll
            for (int k = 0; k < STAT_WORDS; ++k) stw[k] = __int_as_float((int)wv[DW + k]);
        }
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        d.pos[i] = __int_as_float((int)wv[QS_F_POS + i]); d.vel[i] = __int_as_float((int)wv[QS_F_VEL + i]);
        d.om[i] = __int_as_float((int)wv[QS_F_OMEGA + i]); d.goal[i] = __int_as_float((int)wv[QS_F_GOAL + i]);
    }
#pragma unroll
    for (int i = 0; i < 9; ++i) d.rot[i] = __int_as_float((int)wv[QS_F_ROT + i]);
    if constexpr (DEAL) {
        static_assert(Q == 4, "dealt motors: one motor per sub-lane");
        // the sub-lane's word of field F: F + ((q - F) & 3), in register slot (that word) / 4 -- F / 4 or F / 4 + 1
        auto own = [&](int F) {
            const int t = (F + ((q - F) & 3)) >> 2;
            return __int_as_float((int)(t == F / 4 ? r[F / 4] : r[F / 4 + 1]));
        };
        const float rd = own(QS_F_ROT_DAMP), cd = own(QS_F_CMD_DAMP), ou = own(QS_F_OU);
#pragma unroll
        for (int i = 0; i < 4; ++i) { d.rd[i] = rd; d.cd[i] = cd; d.ou[i] = ou; }
    } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        d.rd[i] = __int_as_float((int)wv[QS_F_ROT_DAMP + i]);
        d.cd[i] = __int_as_float((int)wv[QS_F_CMD_DAMP + i]);
        d.ou[i] = __int_as_float((int)wv[QS_F_OU + i]);
    }
    }
    constexpr int IW = QS_F_GOAL + 3;
    d.svd = (int32_t)wv[IW + QS_I_SVD];
    d.flags = wv[IW + QS_I_FLAGS];
    d.prev = 0ull;
    d.prevx = 0ull;
    if constexpr (NIW > QS_I_PREV_LO) d.prev = (uint64_t)wv[IW + QS_I_PREV_LO];
    if constexpr (NIW > QS_I_PREV_HI) d.prev |= (uint64_t)wv[IW + QS_I_PREV_HI] << 32;
    if constexpr (NIW > QS_I_PREV_3) d.prevx = (uint64_t)wv[IW + QS_I_PREV_2] | ((uint64_t)wv[IW + QS_I_PREV_3] << 32);
}
template <int Q>
__device__ __forceinline__ void load_drone_q(const KP& kp, const Bufs& b, int g, int q, Drone& d) {
    DroneWords<Q> dw;
    load_words_q(kp, b, g, q, dw);
    unpack_words_q(dw, d);
}

// ST: also the stats words DRONE_WORDS + k whose bit k of stmask is set (stw = their values).
template <int Q, bool ST = false, int NIW = 4>
__device__ __forceinline__ void store_drone_q(const KP& kp, const Bufs& b, int g, int q, bool active, const Drone& d,
                                              const float* stw = nullptr, uint32_t stmask = 0u) {
    constexpr int DW = WordsOf<NIW>::DW, NW = ST ? WordsOf<NIW>::LW : DW;
    uint32_t wv[NW];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        wv[QS_F_POS + i] = (uint32_t)__float_as_int(d.pos[i]); wv[QS_F_VEL + i] = (uint32_t)__float_as_int(d.vel[i]);
        wv[QS_F_OMEGA + i] = (uint32_t)__float_as_int(d.om[i]); wv[QS_F_GOAL + i] = (uint32_t)__float_as_int(d.goal[i]);
    }
#pragma unroll
    for (int i = 0; i < 9; ++i) wv[QS_F_ROT + i] = (uint32_t)__float_as_int(d.rot[i]);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        wv[QS_F_ROT_DAMP + i] = (uint32_t)__float_as_int(d.rd[i]);
        wv[QS_F_CMD_DAMP + i] = (uint32_t)__float_as_int(d.cd[i]);
        wv[QS_F_OU + i] = (uint32_t)__float_as_int(d.ou[i]);
    }
    constexpr int IW = QS_F_GOAL + 3;
    wv[IW + QS_I_SVD] = (uint32_t)d.svd;
    wv[IW + QS_I_FLAGS] = d.flags;
    if constexpr (NIW > QS_I_PREV_LO) wv[IW + QS_I_PREV_LO] = (uint32_t)d.prev;
    if constexpr (NIW > QS_I_PREV_HI) wv[IW + QS_I_PREV_HI] = (uint32_t)(d.prev >> 32);
    if constexpr (NIW > QS_I_PREV_3) {
        wv[IW + QS_I_PREV_2] = (uint32_t)d.prevx;
        wv[IW + QS_I_PREV_3] = (uint32_t)(d.prevx >> 32);
    }
    if constexpr (ST) {
#pragma unroll
        for (int k = 0; k < STAT_WORDS; ++k) wv[DW + k] = (uint32_t)__float_as_int(stw[k]);
    }
    constexpr int T = (NW + Q - 1) / Q;
    const uint32_t go = (uint32_t)g * 4u;
    const __amdgpu_buffer_rsrc_t rs = qs_rsrc(b.st);
#pragma unroll
    for (int t = 0; t < T; ++t) {
        const int w = t * Q + q;
        uint32_t v = wv[t * Q];
#pragma unroll
        for (int k = 1; k < Q; ++k)
            if (q == k && t * Q + k < NW) v = wv[t * Q + k];
        const bool wr = w < DW || (w < NW && ((stmask >> (w - DW)) & 1u));
        if (active && wr) st_wt1(rs, drone_word_off<NIW>(kp, b, w, go), 0u, v);
    }
}

// Dealt motors (QS_DEAL_MOTORS, Q = 4): sub-lane q runs motor m = (q + 2) & 3 of its drone -- the motor whose
// rot_damp / cmd_damp / OU words (fields 18 + m, 22 + m, 26 + m: word w sits on sub-lane w % 4) that sub-lane already
// loads and stores, so they need no broadcast.  The drone's Drone::rd / cd / ou hold that motor's value in all four
// entries on the sub-lane (unpack_words_q<.., DEAL>, reset and the floor branch write every entry; the store takes word
// F + m from sub-lane q, i.e. the owner's copy).  The motor filter, its noise and its thrust run once per motor
// instead of four times per lane; thrust and the three torques are summed over the quad by qsum (DPP butterfly: every
// sub-lane gets the same bits, so the replicated rest of the substep stays bit-identical on the quad).  The sums are
// (m0 + m1) + (m2 + m3) instead of a running sum over the motors: fp32 reassociation, inside the parity tolerances
// (the oracle is float64).  Measured slower on C3 / C2 / C4 (7.20 -> 7.28, 5.04 -> 5.08, 9.72 -> 9.82 us,
// profiles/ab/r06_deal_motors_ab.txt; parity green either way): the quad sums lengthen the wave's dependency chain
// more than the replicated motor arithmetic costs in issue slots.  Off by default; -DQS_DEAL_MOTORS=1 for A/Bs.
#ifndef QS_DEAL_MOTORS
#define QS_DEAL_MOTORS 0
#endif
struct MotorK {   // the sub-lane's motor: thrust_max, the three torque-arm coefficients, torque_max * ccw
    float tmax, p0, p1, p2, tq;
};
__device__ __forceinline__ float sel4(int m, float a, float b, float c, float d) {
    return m == 0 ? a : (m == 1 ? b : (m == 2 ? c : d));
}
__device__ __forceinline__ MotorK motor_k(const KP& kp, int m) {
    MotorK k;
    k.tmax = sel4(m, kp.thrust_max[0], kp.thrust_max[1], kp.thrust_max[2], kp.thrust_max[3]);
    k.p0 = sel4(m, kp.pc0[0], kp.pc0[1], kp.pc0[2], kp.pc0[3]);
    k.p1 = sel4(m, kp.pc1[0], kp.pc1[1], kp.pc1[2], kp.pc1[3]);
    k.p2 = sel4(m, kp.pc2[0], kp.pc2[1], kp.pc2[2], kp.pc2[3]);
    k.tq = sel4(m, kp.torque_max[0] * kp.ccw[0], kp.torque_max[1] * kp.ccw[1], kp.torque_max[2] * kp.ccw[2],
                kp.torque_max[3] * kp.ccw[3]);
    return k;
}
// motors() for the sub-lane's motor (quadrotor_dynamics.py:511-533), the sums over the quad
__device__ __forceinline__ Torque motors_dealt4(const KP& kp, Drone& d, float cmd, float noise, const MotorK& mk) {
    float tau = cmd < d.cd[0] ? kp.tau_down : kp.tau_up;
    tau = fminf(tau, 1.0f);
    const float r = tau * (fsqrt(cmd) - d.rd[0]) + d.rd[0];
    const float c = clampf(r * r + cmd * noise, 0.f, 1.f);
#pragma unroll
    for (int k = 0; k < 4; ++k) { d.rd[k] = r; d.cd[k] = c; }
    const float th = mk.tmax * (kp.lin == 1.f ? c : (1.f - kp.lin) * c * c + kp.lin * c);
    Torque t;
    t.t0 = qsum<4>(mk.p0 * th);
    t.t1 = qsum<4>(mk.p1 * th);
    t.t2 = qsum<4>(mk.p2 * th + mk.tq * c);
    t.sum = qsum<4>(th);
    return t;
}
__device__ __forceinline__ void substep_dealt4(const KP& kp, Drone& d, float cmd, float noise, const MotorK& mk,
                                               const Rng& rng, uint32_t gid, int s) {
    const Torque tq = motors_dealt4(kp, d, cmd, noise, mk);
    {
        const RodCoef rc = rod_coef(kp, d.rot, d.om);
        float Rn[9];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            float dr[3];
            rod_row(rc, i, dr);
            rod_apply_row(dr, d.rot, Rn + 3 * i);
        }
#pragma unroll
        for (int i = 0; i < 9; ++i) d.rot[i] = Rn[i];
    }
    substep_tail(kp, d, tq, rng, gid, s);
}

// Sub-lanes per drone of the flavor-B step kernel (QS_QB; 64 / NPAD when an env would not fit a wave).
#ifndef QS_QB
#define QS_QB 4
#endif
template <int NPAD>
struct StepGeo {
    static constexpr int Q = NPAD * QS_QB <= 64 ? QS_QB : (NPAD >= 64 ? QS_QW : 64 / NPAD);
    static constexpr int LPE = NPAD * Q;            // lanes per env
    static constexpr int WGS = LPE > 64 ? LPE : 64; // threads per workgroup: one wave, or the env's waves
    static constexpr int EPB = WGS / LPE;           // envs per workgroup
    static constexpr int SLOTS = EPB * NPAD;        // drone slots per workgroup
    static constexpr bool WIDE = LPE > 64;          // the env spans the workgroup's waves (64 / 128 drones)
    static constexpr bool ROW2 = NPAD > 64;         // 128-bit collision rows (128-drone envs)
    // istate words a step moves per drone (WordsOf): SVD counter, flags, then the previous-collision row's
    // words that a partner can set -- none for single-drone envs, the low word up to 32 drones, both up to 64,
    // four for the 128-bit rows.  The words beyond stay 0 in memory (zeroed at creation) and are never moved.
    static constexpr int NIW = NPAD == 1 ? 2 : (NPAD <= 32 ? 3 : (ROW2 ? 6 : 4));
};

// Drone-drone impulses of an env that spans several waves: the new pairs in the reference's (i, j) order, one
// event per round.  Every drone posts its pos / vel / omega and its first pending partner to LDS tables (in the
// obs tile, unused until the obs phase), a collective finds the first drone i with a pending pair, lanes 0..8
// draw the pair's 9 Philox blocks (7 normal, 2 uniform), and the pair's lanes apply collide_pair -- the same
// draws and arithmetic as the one-wave loop of step_kernel.
template <int NPAD, class EC, class Row>
__device__ __forceinline__ void impulses_wide(const KP& kp, const Rng& rng, float* lds, EC& ec, Drone& d,
                                              Row pend, int env, int di, int q, int lane, bool& vchanged) {
    float4* pscr = reinterpret_cast<float4*>(lds);       // the pair's 9 blocks
    float4* tab = pscr + 16;                              // per drone: {pos}, {vel}, {omega}
    int* jt = reinterpret_cast<int*>(tab + 3 * NPAD);     // per drone: first pending partner, -1 = none
    for (;;) {
        const bool has = row_any(pend);
        if (q == 0) {
            tab[3 * di] = make_float4(d.pos[0], d.pos[1], d.pos[2], 0.f);
            tab[3 * di + 1] = make_float4(d.vel[0], d.vel[1], d.vel[2], 0.f);
            tab[3 * di + 2] = make_float4(d.om[0], d.om[1], d.om[2], 0.f);
            jt[di] = has ? row_ffs(pend) : -1;
        }
        const Row bal = ec.bits(has);   // its barrier also orders the table writes
        if (!row_any(bal)) break;
        const int istar = row_ffs(bal), jstar = jt[istar];
        const bool involved = di == istar || di == jstar;
        const int partner = di == istar ? jstar : istar;
        const float4 a = tab[3 * partner], bv = tab[3 * partner + 1], c = tab[3 * partner + 2];
        const float pp[3] = {a.x, a.y, a.z};
        float pv[3] = {bv.x, bv.y, bv.z}, pw[3] = {c.x, c.y, c.z};   // the partner's copy (collide_pair writes both)
        const uint32_t gi = kp.id0 + (uint32_t)(env * kp.N + istar);
        const uint32_t st = S_PAIR | ((uint32_t)jstar << 8);
        if (lane < 9) {
            const bool isn = lane < 7;
            const W4 w = block(rng, gi, isn ? st : (st | UNIF_BIT), (uint32_t)(isn ? lane : lane - 7));
            float v[4];
            if (isn) {
                box_muller(w.w[0], w.w[1], v[0], v[1]);
                box_muller(w.w[2], w.w[3], v[2], v[3]);
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) v[i] = u01(w.w[i]);
            }
            pscr[lane] = make_float4(v[0], v[1], v[2], v[3]);
        }
        lds_sync();
        if (involved) {
            float z[28], u[8];
#pragma unroll
            for (int k = 0; k < 9; ++k) {
                const float4 x = pscr[k];
                float* o = k < 7 ? z + 4 * k : u + 4 * (k - 7);
                o[0] = x.x; o[1] = x.y; o[2] = x.z; o[3] = x.w;
            }
            if (di == istar) collide_pair(d.pos, d.vel, d.om, pp, pv, pw, z, u);
            else collide_pair(pp, pv, pw, d.pos, d.vel, d.om, z, u);
        }
        vchanged |= involved;
        if (di == istar) row_clear(pend, jstar);
    }
}

template <int NPAD, bool OBST>
__global__ __launch_bounds__(StepGeo<NPAD>::WGS) void step_kernel(const KP* __restrict__ kpp, Bufs b, const RArgs* __restrict__ rargs) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    QS_BIND_KP(kpp);
    vptr_bufs<(NPAD <= 16)>(b);
    const uint32_t seed = kpm.seed;
    QS_STAMP_DECL
    QS_RTSTAMP(12);
    QS_STAMP(0);
    using G = StepGeo<NPAD>;
    constexpr int Q = G::Q, LPE = G::LPE, EPB = G::EPB, SLOTS = G::SLOTS, WGS = G::WGS, NIW = G::NIW;
    constexpr bool WIDE = G::WIDE;
    constexpr int LW = WordsOf<NIW>::LW, DW = WordsOf<NIW>::DW;
    using Row = typename RowOf<G::ROW2>::T;
    const int lane = threadIdx.x;
    const int el = lane / LPE, di = (lane % LPE) / Q, q = lane % Q;
    const int env0 = xcd_block((int)blockIdx.x, (int)gridDim.x) * EPB;
    const int env = env0 + el;
    const bool active = env < kp.E && di < kp.N;
    const bool lead = active && q == 0;   // the sub-lane that writes the drone's outputs
    const int g = active ? env * kp.N + di : 0;
    const uint32_t gid = kp.id0 + (uint32_t)g;
    const int lbase = el * LPE;           // first lane of the env
    const int dbase = el * NPAD;          // first drone slot of the env
    const int nenv_blk = min(EPB, kp.E - env0);
    const int rows = nenv_blk * kp.N;
    float* row = lds + (size_t)(el * kp.N + di) * kp.obs_dim;
    float4* xch = reinterpret_cast<float4*>(lds + SLOTS * kp.obs_dim);
    const uint64_t lmask = (LPE >= 64) ? ~0ull : ((1ull << LPE) - 1ull);
    // env-level collectives; WIDE: their LDS slots and the env counters' exchange in the 64 words after xch
    uint64_t* wscr = reinterpret_cast<uint64_t*>(lds + SLOTS * kp.obs_dim + SLOTS * 8);
    EnvColl<WIDE, G::ROW2, Q, WGS / 64> ec{lbase, lmask, wscr, 0};
    float2* otile = obst_tile(lds, kp, SLOTS);
    ObstScratch* oscr = reinterpret_cast<ObstScratch*>(otile + EPB * kp.M);
    const float2* myob = otile + el * kp.M;
    if (OBST)   // the block's obstacle lists -> LDS (ordered by the first lds_sync below)
        for (int k = lane; k < nenv_blk * kp.M; k += WGS) otile[k] = b.obst[(size_t)env0 * kp.M + k];

    // Every global load of the step is issued up front, back to back -- the action, the env's counters, the
    // drone's state words -- before anything waits: their HBM latencies overlap instead of adding up (the
    // scheduler otherwise sank the action load behind the state's waits).
    const float4 av = reinterpret_cast<const float4*>(b.act)[g];
    const int eidx = active ? env : 0;
    const int tick0 = b.env[QS_E_TICK * kp.E + eidx];
    const int episode = b.env[QS_E_EPISODE * kp.E + eidx];
    const int32_t ef0 = b.env[QS_E_FLAGS * kp.E + eidx];   // the env's flags (rewritten at the end of the step)
    // episode_extra_stats: the env's 11 counters QS_E_ST_COL.. dealt over its lanes (lane li holds li + LPE t)
    constexpr int NCNT = 11, CT = (NCNT + LPE - 1) / LPE;
    const int li = lane - lbase;
    const bool envok = env < kp.E;
    int cnt[CT];
    bool cdirty[CT];   // the counter changed this step: stored once, at the end of the step
    auto cnt_at = [&](int k) -> int32_t* { return b.env + (QS_E_ST_COL + k) * kp.E + env; };
    // a counter that no event of this configuration can increment stays 0: not loaded (drone-drone collisions
    // need a partner, the obstacle counters obstacles; with the specialised kernels these tests are constants)
    // (counters 0, 5, 6: drone-drone; 1-4: room; 7-10: obstacles -> the live ones are [cnt_lo, cnt_hi))
    const int cnt_lo = kp.N > 1 ? 0 : 1, cnt_hi = OBST ? NCNT : (kp.N > 1 ? 7 : 5);
    auto cnt_live = [&](int k) { return k >= cnt_lo && k < cnt_hi; };
#pragma unroll
    for (int t = 0; t < CT; ++t) {
        const int k = li + LPE * t;
        cnt[t] = (kp.stats && envok && k < NCNT && cnt_live(k)) ? *cnt_at(k) : 0;
        cdirty[t] = false;
    }
    int omi = 0, osi = 0;   // the env's domain-randomisation choice (QS_E_OBST_M / _SZ)
    if (OBST && kp.dr) { omi = b.env[QS_E_OBST_M * kp.E + eidx]; osi = b.env[QS_E_OBST_SZ * kp.E + eidx]; }
    // goal scenario: the env's scenario record (SC_WORDS words) dealt over its lanes -- word li + LPE t on lane li
    // -- loaded with the step's other loads and staged in LDS for scenario.step() after the forces
    const bool SCEN = !OBST && kp.scen_b >= 0;
    // the obstacle maps' dynamic scenarios (o_swap_goals, o_ep_rand_bezier, o_dynamic_same_goal): reset with the map
    // (obstacle_reset_env), stepped like the goal scenarios
    const bool OSCEN = OBST && kp.scen_b >= SC_O_SWAP_GOALS;
    const bool SCEN_STEP = (SCEN && kp.scen_b != SC_STATIC_DIFF_GOAL) || OSCEN;   // static_diff_goal's step() does nothing
    constexpr int SRW = (SC_WORDS + LPE - 1) / LPE;
    uint32_t scw[SRW];
    auto load_scw = [&]() {
#pragma unroll
        for (int t = 0; t < SRW; ++t) {
            const int w = li + LPE * t;
            scw[t] = (SCEN_STEP && !QS_SCW_SKIP && envok && w < SC_WORDS) ? scen_word(kp, b, env, w) : 0u;
        }
    };
#if !QS_SCW_LATE
    load_scw();
#endif
    Drone d;   // every sub-lane holds the whole drone
    DroneWords<Q, LW> dw;
    load_words_q<Q, LW, NIW>(kp, b, g, q, dw, kp.stats ? LW : DW);
#if QS_SCW_LATE
    // after the state words: the unpack's wait (in-order vmcnt) then does not include the record's 27 rows
    load_scw();
#endif
    __builtin_amdgcn_sched_barrier(0);
    const Rng rng = env_rng(seed, tick0, episode);
    // The step's regular draws: Philox block k of {OU 0, sensor 0, sensor 1, sensor 2} on sub-lane
    // k % Q, slot k / Q -- one block per lane for Q = 4 -- then broadcast by DPP.  They need only the env's
    // Philox counter {tick, episode}, the oldest of the step's loads: drawn while the drone's state words
    // are still in flight (the unpack below is the first wait on them).
    float zou[4], zs[12];
    {
        constexpr int ZT = (4 + Q - 1) / Q;   // blocks per sub-lane (Q = 8: sub-lanes 4-7 draw nothing)
        float zr[ZT][4] = {};
#pragma unroll
        for (int t = 0; t < ZT; ++t) {
            const int k = q + Q * t;
            if (k < 4 && (k == 0 || kp.sense))
                normals4(rng, gid, k == 0 ? S_OU : S_SENSOR, k == 0 ? 0u : (uint32_t)(k - 1), zr[t]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            zou[i] = qbc<Q, 0>(zr[0][i]);
            zs[i] = qbc<Q, 1 % Q>(zr[1 / Q][i]);
            zs[4 + i] = qbc<Q, 2 % Q>(zr[2 / Q][i]);
            zs[8 + i] = qbc<Q, 3 % Q>(zr[3 / Q][i]);
        }
    }

    QS_PRIO(11);
    __builtin_amdgcn_sched_barrier(0);
    float stw[STAT_WORDS];
    constexpr bool DEALM = QS_DEAL_MOTORS && Q == 4;
    unpack_words_q<Q, LW, NIW, DEALM>(dw, d, stw, q);
    float a[4] = {av.x, av.y, av.z, av.w};
    const int tick = tick0 + 1;
    const bool done = tick > kpm.ep_len;
    // episode_extra_stats (kp.stats): distance_to_goal's last entries and window sums of this drone (loaded
    // with the state words; consumed after the physics) -- the ring while it is still needed, the sums in
    // their windows
    float dring[5] = {0.f, 0.f, 0.f, 0.f, 0.f}, dsum[3] = {0.f, 0.f, 0.f};
    bool in_win[3] = {false, false, false};
    uint32_t stmask = 0u;   // the stats words (stw) the state store writes back
    if (kp.stats) {
        const int T = kpm.ep_len + 1;   // the entry count when the episode ends
#pragma unroll
        for (int k = 0; k < 3; ++k) in_win[k] = tick > T - kp.st_win[k];
        if (!(d.flags & QS_FL_REACHED) && tick >= 5) {
#pragma unroll
            for (int k = 0; k < 5; ++k) dring[k] = stw[k];
        }
#pragma unroll
        for (int k = 0; k < 3; ++k)
            if (in_win[k]) dsum[k] = stw[5 + k];
    }
    OGeo og = ogeo(kp, omi, osi);

    QS_STAMP(1);
    // ---- per-drone control + physics (QuadrotorSingle._step), replicated on the sub-lanes ----
    float rw = 0.f;
    bool floor_now = false;   // drone 0's on the env's flags: its rew_crash feeds the replay wrapper
    float rc_dist, rc_effort, rc_orient, rc_spin;   // compute_reward_weighted's raw terms (per-step infos)
    {
        if constexpr (DEALM) {   // the sub-lane's motor m (motors_dealt4)
            const int m = (q + 2) & 3;
            const float zm = sel4(m, zou[0], zou[1], zou[2], zou[3]), am = sel4(m, a[0], a[1], a[2], a[3]);
            const float ou = d.ou[0] + (kp.ou_theta * (kp.ou_mu - d.ou[0]) + kp.ou_sigma * zm);
#pragma unroll
            for (int k = 0; k < 4; ++k) d.ou[k] = ou;
            const float cmd = 0.5f * (clampf(am, -1.f, 1.f) + 1.f);
            const MotorK mk = motor_k(kp, m);
            for (int s = 0; s < kp.sim_steps; ++s) substep_dealt4(kp, d, cmd, ou, mk, rng, gid, s);
        } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) d.ou[k] = d.ou[k] + (kp.ou_theta * (kp.ou_mu - d.ou[k]) + kp.ou_sigma * zou[k]);
        float cmds[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) cmds[k] = 0.5f * (clampf(a[k], -1.f, 1.f) + 1.f);
        for (int s = 0; s < kp.sim_steps; ++s) substep(kp, d, cmds, d.ou, rng, gid, s);
        }
        // compute_reward_weighted (quadrotor_single.py:34-66)
        const float gx = d.goal[0] - d.pos[0], gy = d.goal[1] - d.pos[1], gz = d.goal[2] - d.pos[2];
        const bool on_floor = d.flags & QS_FL_ON_FLOOR;
        floor_now = on_floor;
        const float dist = fsqrt(gx * gx + gy * gy + gz * gz);
        if (kp.stats && active) {   // distance_to_goal[i].append(-rewraw_pos) and reached_goal (:651-655)
            // every sub-lane (the flags stay identical); the words reach HBM with the state's store burst
            const float v = kp.dt * dist;
            const int slot = tick % 5;
#pragma unroll
            for (int k = 0; k < 5; ++k) stw[k] = k == slot ? v : stw[k];
            stmask = 1u << slot;
#pragma unroll
            for (int k = 0; k < 3; ++k)
                if (in_win[k]) {
                    dsum[k] += v;
                    stw[5 + k] = dsum[k];
                    stmask |= 1u << (5 + k);
                }
            if (!(d.flags & QS_FL_REACHED) && tick >= 5) {
                // the last 5 entries are the whole ring (this step's in its slot), summed in slot order
                float m = 0.f;
#pragma unroll
                for (int k = 0; k < 5; ++k) m += k == slot ? v : dring[k];
                // approch_goal_metric: mean(m / dt over 5) < 0.5 as m < 2.5 dt (no IEEE division on the common path;
                // the two forms differ only within an ulp of the threshold)
                if (m < 2.5f * kp.dt) d.flags |= QS_FL_REACHED;
            }
        }
        rc_dist = dist;
        rc_effort = fsqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2] + a[3] * a[3]);
        rc_orient = on_floor ? 1.f : -d.rot[8];
        rc_spin = fsqrt(d.om[0] * d.om[0] + d.om[1] * d.om[1] + d.om[2] * d.om[2]);
        const float cost = kpm.rew_pos * dist + kpm.rew_effort * rc_effort + kpm.rew_crash * (on_floor ? 1.f : 0.f) +
                           kpm.rew_orient * rc_orient + kpm.rew_spin * rc_spin;
        rw = -kp.dt * cost;
    }

    QS_STAMP(2);
    QS_PRIO_DROP(21);
    // ---- swarm phase: collisions + proximity (quadrotor_multi.py:537-568, 608-622) ----
    Row cur{};
    float pen = 0.f;
    if (q == 0) xch_put(xch, dbase + di, d.pos, d.vel);
    lds_sync();
    if (kp.N > 1) {
        // sub-lane q tests the partners j = q + Q t (LDS reads issued back to back, branch-free
        // tests), then the drone's collision row and proximity sum are reduced over the sub-lanes
        constexpr int PJ = (NPAD + Q - 1) / Q;
        constexpr int CH = PJ < 16 ? PJ : 16;   // partners loaded per batch (bounds the VGPRs at N = 64)
        for (int t0 = 0; t0 < PJ; t0 += CH) {
            float4 pj[CH];
#pragma unroll
            for (int u = 0; u < CH; ++u) {
                const int j = q + Q * (t0 + u);
                pj[u] = xch[2 * (dbase + (j < NPAD ? j : NPAD - 1))];
            }
#pragma unroll
            for (int u = 0; u < CH; ++u) {
                const int j = q + Q * (t0 + u);
                const float dx = d.pos[0] - pj[u].x, dy = d.pos[1] - pj[u].y, dz = d.pos[2] - pj[u].z;
                const float dist = fsqrt(dx * dx + dy * dy + dz * dz);
                const bool ok = j != di && j < kp.N;
                row_set(cur, j, ok && dist <= kp.col_thr);
                const float pterm = kpm.prox_ratio * dist + kpm.prox_max;
                pen += (ok && dist <= kp.fall_thr) ? pterm : 0.f;   // pen >= 0: adding +0 is exact
            }
        }
        if constexpr (Q > 1) cur = qor<Q>(cur);
        pen = qsum<Q>(pen);
    }
    Row prow;
    row_of(d, prow);
    const Row newpairs = cur & ~prow;
    // setdiff1d(flat(cur), flat(prev)) and its ".any()" (drone 0 alone does not count)
    const bool uniq = active && row_any(cur) && !row_any(prow);
    const bool any_uniq = ec.any(uniq && di != 0 && q == 0);
    rw += kpm.quadcol * ((any_uniq && uniq) ? -1.f : 0.f);
    rw += -(kp.cdt * pen);
    // room: new wall / ceiling crashes vs the previous NEW lists (:390-403, :604-605)
    const bool wall_new = (d.flags & QS_FL_CRASH_WALL) && !(d.flags & QS_FL_PREV_WALL);
    const bool ceil_new = (d.flags & QS_FL_CRASH_CEIL) && !(d.flags & QS_FL_PREV_CEIL);
    d.flags = (d.flags & ~(uint32_t)(QS_FL_PREV_WALL | QS_FL_PREV_CEIL)) | (wall_new ? QS_FL_PREV_WALL : 0u) |
              (ceil_new ? QS_FL_PREV_CEIL : 0u);
    // obstacles (quadrotor_multi.py:570-589): first pillar hit, new vs the previous step's set
    int ohit = -1;
    bool onew = false;
    if (OBST) {
        ohit = (Q == 2 || Q == 4) ? obst_detect_q<Q>(og, myob, d.pos[0], d.pos[1], q) : obst_detect(og, myob, d.pos[0], d.pos[1]);
        onew = active && ohit >= 0 && !(d.flags & QS_FL_PREV_OBST);
        rw += kpm.quadcol_obst * (onew ? -1.f : 0.f);
        d.flags = (d.flags & ~(uint32_t)QS_FL_PREV_OBST) | (ohit >= 0 ? (uint32_t)QS_FL_PREV_OBST : 0u);
    }
    bool any_onew = false;   // curr_quad_col non-empty (quadrotor_multi.py:576)
    if (OBST) any_onew = ec.any(onew && q == 0);
    if (kp.stats) {   // episode_extra_stats counters (quadrotor_multi.py:555-566, 575-589, 599-606, 631-635)
        auto env_count = [&](bool x) { return ec.count(x && q == 0); };
        const bool settle = tick >= kp.st_settle;
        const bool cfloor = active && (d.flags & QS_FL_CRASH_FLOOR);
        const bool room_new = active && (cfloor || wall_new || ceil_new) && !(d.flags & QS_FL_PREV_ROOM);
        d.flags = (d.flags & ~(uint32_t)QS_FL_PREV_ROOM) | (room_new ? (uint32_t)QS_FL_PREV_ROOM : 0u);
        // every count below is zero unless one of these events happened somewhere in the wave (a new
        // collision, a first floor contact, a new wall / ceiling / room crash, a new pillar hit): one
        // wave-uniform test skips the per-env counting in the common step
        if (ec.wany(q == 0 && (uniq || cfloor || (active && (wall_new || ceil_new)) || room_new || (OBST && onew))))
        {
        const int col = env_count(uniq) / 2;   // len(last_step_unique_collisions) // 2
        if (col > 0 && settle && uniq) d.flags |= QS_FL_HIT_AGENT;
        const int nfl = env_count(cfloor), nw = env_count(active && wall_new), nc = env_count(active && ceil_new);
        const int nr = env_count(room_new);
        int oc = 0, o35 = 0, o5 = 0;
        if (OBST) {
            oc = env_count(onew);
            bool f35 = false, f5 = false;
            if (oc > 0 && settle && onew) {
                d.flags |= QS_FL_HIT_OBST;
                // the step's obs[qid][0:3]: the sensed position minus the goal (self obs before the forces)
                float rr = 0.f;
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    const float x = d.pos[c] + (kp.sense ? kp.pos_std * zs[c] : 0.f) - d.goal[c];
                    rr += x * x;
                }
                const float rd = fsqrt(rr);
                f35 = rd > 3.5f;
                f5 = rd > 5.f;
            }
            o35 = env_count(f35);
            o5 = env_count(f5);
        }
        const bool fin5 = kpm.ep_len - tick0 <= kp.st_final;   // time_remain <= collisions_final_grace_period_steps
        // counter QS_E_ST_COL + k lives on lane k (mod LPE) of the env: it adds its own increment (env-uniform
        // values from the ballots) and stores only when that changed it
#pragma unroll
        for (int t = 0; t < CT; ++t) {
            const int k = li + LPE * t;
            const bool os = OBST && oc > 0 && settle;
            const int inc = k == 0 ? col : k == 1 ? (settle ? nr : 0) : k == 2 ? (settle ? nfl : 0) :
                            k == 3 ? (settle ? nw : 0) : k == 4 ? (settle ? nc : 0) :
                            k == 5 ? (settle ? col : 0) : k == 6 ? (fin5 ? col : 0) : k == 7 ? oc :
                            k == 8 ? (os ? oc : 0) : k == 9 ? (os ? o35 : 0) : k == 10 ? (os ? o5 : 0) : 0;
            if (envok && k < NCNT && inc != 0) {
                cnt[t] += inc;
                cdirty[t] = true;
            }
        }
        }
    }

    QS_STAMP(3);
    QS_PRIO_DROP(22);
    // ---- random forces (:659-698), replicated on the sub-lanes ----
    bool vchanged = false;
    if (kp.downwash && kp.N > 1)   // perform_downwash (aerodynamics/downwash.py:4-51)
        vchanged = downwash_env<NPAD, Q>(kp, d, rng, gid, env, lbase, di, q, active,
                                         kp.obs_dim >= 8 ? reinterpret_cast<float4*>(lds) : nullptr, dbase);
    if (kp.collide) {
        // drone-drone impulses, pairs in (i, j) order; a wave-uniform loop over pending events.
        // Ballots read sub-lane 0 of each drone (bit lbase + i * Q).
        if constexpr (WIDE) {
            impulses_wide<NPAD>(kp, rng, lds, ec, d, active ? row_above(newpairs, di) : Row{}, env, di, q, lane, vchanged);
        } else {
        uint64_t pend = active ? row_above(newpairs, di) : 0ull;
#if QS_PAIR_ROUNDS
        // Rounds of disjoint pairs (round 5).  The reference applies the new pairs one by one in (i, j) order
        // (quadrotor_multi.py:671-676); a pair only reads and writes its two drones, so what matters is that every
        // pair sees its drones after all their earlier pairs.  A round takes every pending pair that is the earliest
        // pending pair of both its drones -- disjoint pairs, each already preceded by all of its drones' earlier
        // pairs -- and applies them at once: the same draws and arithmetic per pair as the one-pair loop below
        // (bitwise the same states), in as many rounds as the longest chain of pairs sharing drones instead of one
        // iteration per pair.  Per round: the env's pending rows and their columns through LDS (the obs tile is
        // free until the obs phase), the ready pairs' 9 Philox blocks drawn by the env's lanes (lane le: block
        // le % 9 of pair le / 9), up to LPE / 9 pairs (more wait a round).
        constexpr int PMAX = LPE / 9, TBL4 = (2 * NPAD + 3) / 4, STR4 = PMAX * 9 + TBL4;
        // only when some env of the wave has two or more pairs pending (else the one-pair loop takes one iteration)
        const uint64_t pbal = __ballot(pend != 0ull && q == 0);
        const bool multi = q == 0 && (__popcll(pend) >= 2 || __popcll((pbal >> lbase) & lmask) >= 2);
        if (PMAX > 0 && NPAD <= 32 && EPB * STR4 * 4 <= SLOTS * kp.obs_dim && __ballot(multi) != 0ull) {
            float4* pscr = reinterpret_cast<float4*>(lds) + el * STR4;
            uint32_t* pt = reinterpret_cast<uint32_t*>(pscr + PMAX * 9);   // [NPAD] the drones' pending rows
            uint32_t* ct = pt + NPAD;                                     // [NPAD] their columns (earlier owners)
            const int le = lane - lbase, pb = le / 9, kb = le - 9 * pb;
            for (;;) {
                const uint64_t bal = __ballot(pend != 0ull && q == 0);
                if (bal == 0ull) break;
                if (q == 0) pt[di] = (uint32_t)pend;
                lds_sync();
                uint32_t col = 0u;
#pragma unroll
                for (int i = 0; i < NPAD; ++i) col |= ((pt[i] >> di) & 1u) << i;
                if (q == 0) ct[di] = col;
                lds_sync();
                const int jf = pend ? (__ffsll((long long)pend) - 1) : 0;
                const int i0 = col ? (__ffs((int)col) - 1) : 0;
                // owner of a ready pair: nothing earlier of this drone pending, and (di, jf) is jf's earliest
                const bool own = pend != 0ull && col == 0u && (__ffs((int)ct[jf]) - 1) == di;
                // partner in a ready pair: its earliest pair is (i0, di) and i0 has nothing earlier pending
                const bool part = col != 0u && ct[i0] == 0u && (__ffs((int)pt[i0]) - 1) == di;
                const uint64_t re = (__ballot(own && q == 0) >> lbase) & lmask;   // ready owners (bit owner * Q)
                const int ow = own ? di : (part ? i0 : 0);
                const int rank = __popcll(re & ((1ull << (ow * Q)) - 1ull));
                const bool go = (own || part) && rank < PMAX;
                const int partner = own ? jf : (part ? i0 : di);
                float pp[3], pv[3], pw[3];
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    pp[c] = __shfl(d.pos[c], lbase + partner * Q + q);
                    pv[c] = __shfl(d.vel[c], lbase + partner * Q + q);
                    pw[c] = __shfl(d.om[c], lbase + partner * Q + q);
                }
                if (pb < PMAX && pb < __popcll(re)) {   // block kb of the round's pb-th pair
                    uint64_t m = re;
                    for (int k = 0; k < pb; ++k) m &= m - 1ull;
                    const int ob = (__ffsll((long long)m) - 1) / Q, oj = __ffs((int)pt[ob]) - 1;
                    const bool isn = kb < 7;
                    const uint32_t st = S_PAIR | ((uint32_t)oj << 8);
                    const W4 w = block(rng, kp.id0 + (uint32_t)(env * kp.N + ob), isn ? st : (st | UNIF_BIT),
                                       (uint32_t)(isn ? kb : kb - 7));
                    float v[4];
                    if (isn) {
                        box_muller(w.w[0], w.w[1], v[0], v[1]);
                        box_muller(w.w[2], w.w[3], v[2], v[3]);
                    } else {
#pragma unroll
                        for (int i = 0; i < 4; ++i) v[i] = u01(w.w[i]);
                    }
                    pscr[le] = make_float4(v[0], v[1], v[2], v[3]);
                }
                lds_sync();
                if (go) {
                    float z[28], u[8];
#pragma unroll
                    for (int k = 0; k < 9; ++k) {
                        const float4 x = pscr[rank * 9 + k];
                        float* o = k < 7 ? z + 4 * k : u + 4 * (k - 7);
                        o[0] = x.x; o[1] = x.y; o[2] = x.z; o[3] = x.w;
                    }
                    if (own) collide_pair(d.pos, d.vel, d.om, pp, pv, pw, z, u);
                    else collide_pair(pp, pv, pw, d.pos, d.vel, d.om, z, u);
                    vchanged = true;
                }
                lds_sync();   // the scratch and the tables are rewritten by the next round
                if (go && own) pend &= ~(1ull << jf);
            }
        }
#endif
        for (;;) {
            const uint64_t bal = __ballot(pend != 0ull && q == 0);
            if (bal == 0ull) break;
            const uint64_t eb = (bal >> lbase) & lmask;
            const int istar = eb ? (__ffsll((long long)eb) - 1) / Q : 0;
            const int myj = pend ? (__ffsll((long long)pend) - 1) : 0;
            const int jstar = __shfl(myj, lbase + istar * Q);
            const int partner = (di == istar) ? jstar : istar;
            float pp[3], pv[3], pw[3];
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                pp[c] = __shfl(d.pos[c], lbase + partner * Q + q);
                pv[c] = __shfl(d.vel[c], lbase + partner * Q + q);
                pw[c] = __shfl(d.om[c], lbase + partner * Q + q);
            }
            const bool involved = eb != 0 && (di == istar || di == jstar);
            vchanged |= involved;
            const uint32_t gi = kp.id0 + (uint32_t)(env * kp.N + istar);
            const uint32_t st = S_PAIR | ((uint32_t)jstar << 8);
            if constexpr (LPE >= 9) {
                // The env's lanes draw the pair's 9 Philox blocks (7 normal, 2 uniform) in ONE round, lane le
                // block le, and hand them to the pair's lanes through LDS (the obs tile is free until the obs
                // phase).  An event is rare, but the wave that has one is the launch's last: keep it short.
                float4* pscr = reinterpret_cast<float4*>(lds) + el * 9;
                const int le = lane - lbase;
                if (eb != 0 && le < 9) {
                    const bool isn = le < 7;
                    const W4 w = block(rng, gi, isn ? st : (st | UNIF_BIT), (uint32_t)(isn ? le : le - 7));
                    float v[4];
                    if (isn) {
                        box_muller(w.w[0], w.w[1], v[0], v[1]);
                        box_muller(w.w[2], w.w[3], v[2], v[3]);
                    } else {
#pragma unroll
                        for (int i = 0; i < 4; ++i) v[i] = u01(w.w[i]);
                    }
                    pscr[le] = make_float4(v[0], v[1], v[2], v[3]);
                }
                lds_sync();
                if (involved) {
                    float z[28], u[8];
#pragma unroll
                    for (int k = 0; k < 9; ++k) {
                        const float4 x = pscr[k];
                        float* o = k < 7 ? z + 4 * k : u + 4 * (k - 7);
                        o[0] = x.x; o[1] = x.y; o[2] = x.z; o[3] = x.w;
                    }
                    if (di == istar) collide_pair(d.pos, d.vel, d.om, pp, pv, pw, z, u);
                    else collide_pair(pp, pv, pw, d.pos, d.vel, d.om, z, u);
                }
                lds_sync();   // the scratch is rewritten by the next event
            } else if (involved) {   // both drones' sub-lanes draw the pair's 9 Philox blocks in parallel
                float z[28], u[8];
                qdraws<Q, 7, 2>(rng, gi, st, st, q, z, u);
                if (di == istar) collide_pair(d.pos, d.vel, d.om, pp, pv, pw, z, u);
                else collide_pair(pp, pv, pw, d.pos, d.vel, d.om, z, u);
            }
            if (eb != 0 && di == istar) pend &= ~(1ull << jstar);
        }
        }
        if (OBST && onew) {   // perform_collision_with_obstacle, drones in ascending order (:680-689)
            float z[20], u[8];
            qdraws<Q, 5, 2>(rng, gid, S_OBST, S_OBST, q, z, u);
            collide_obstacle(kp, og, d, myob[ohit].x, myob[ohit].y, z, u);
            vchanged = true;
        }
        if (active && (wall_new || ceil_new)) {
            float u[12];
            if (wall_new) {
                qdraws<Q, 0, 3>(rng, gid, S_WALL, S_WALL, q, nullptr, u);
                collide_room(kp, d, u, true);
            }
            if (ceil_new) {
                qdraws<Q, 0, 3>(rng, gid, S_CEIL, S_CEIL, q, nullptr, u);
                collide_room(kp, d, u, false);
            }
        }
        vchanged |= active && (wall_new || ceil_new);
    }
    row_keep(d, cur);

    // ---- scenario.step() (quadrotor_multi.py:700-701): new goals after the forces.  The reference's
    // observations keep the old goal unless the env's state-update flag (a downwash or impulse on any
    // drone, :659-698) makes it recompute them after the scenario step (:711-712). ----
    // Every lane of an env runs scenario.step() for its own drone (scen_step_lane: the same draws and scalars on
    // every lane, the drone's own goal row); envs whose scenario does nothing at this tick skip it, and the
    // scenario record is stored only where it changed.
    float obs_goal[3] = {d.goal[0], d.goal[1], d.goal[2]};
    float* stab = scen_tab_b<OBST>(lds, kp, SLOTS, EPB) + el * scen_stride<NPAD>();
    QS_STAMP(18);   // sub-phases of "impulses+scenario+state store" (slots 18-21)
    if (SCEN_STEP) {
        uint32_t* srec = reinterpret_cast<uint32_t*>(stab + 2 * (NPAD + 4) * 4);
        if (q == 0 && di < kp.N) { stab[4 * di] = d.goal[0]; stab[4 * di + 1] = d.goal[1]; stab[4 * di + 2] = d.goal[2]; }
#pragma unroll
        for (int t = 0; t < SRW; ++t) {
            const int w = li + LPE * t;
            if (envok && w < SC_WORDS) srec[w] = scw[t];
        }
        lds_sync();
        QS_STAMP(19);
        const bool sact = active && scen_acts(kp, (int)srec[0], (int)srec[2], tick);
        if (ec.wany(sact)) {
            bool via = false;
            int bz0 = 0;   // ep_rand_bezier: the first accepted try of its rejection loop, searched by the env's lanes
            if constexpr (!WIDE)
                if (kp.scen_b == SC_MIX || kp.scen_b == SC_EP_RAND_BEZIER || kp.scen_b == SC_O_EP_RAND_BEZIER) {
                    // scen_step_lane's period
                    const int steps = (int)((kp.scen_b == SC_O_EP_RAND_BEZIER ? 6.f : 5.f) * (1.f / kp.cdt));
                    // the env's active lanes (li < N Q) search; the padding lanes of an env with N < NPAD hold env
                    // 0's tick / Philox counter and idle
                    const int bm = sc_mode(kp, (int)srec[0]);
                    const bool bneed = active && (bm == SC_EP_RAND_BEZIER || bm == SC_O_EP_RAND_BEZIER) &&
                                       (tick % steps == 0 || tick == 1);
                    if (ec.wany(bneed))
                        bz0 = bz_first_parallel<LPE>(kp, srec, bneed, li, lbase, kp.N * Q, rng,
                                                     kp.id0 + (uint32_t)(env * kp.N), stab);
                }
            if (sact) {
                Scen sc;
                scen_from_words(srec, sc);
                SDraw sd = sdraw(rng, kp.id0 + (uint32_t)(env * kp.N), S_SCN);
                const OCtx oc{myob, og.m, kp.obst_n};
                const int ch = scen_step_lane(kp, sc, tick, sd, di, stab, stab + 4 * (NPAD + 4), d.goal, via, bz0,
                                              OBST ? &oc : nullptr);
                if (di == 0 && q == 0) {
                    if (ch == 2) scen_store(kp, b, env, sc);
                    else if (ch == 1) scen_store_size(kp, b, env, sc);
                }
            }
            QS_STAMP(20);
            if (ec.wany(via)) {   // the shuffled goals: table B's row of the drone
                lds_sync();
                if (via)
                    for (int k = 0; k < 3; ++k) d.goal[k] = stab[4 * (NPAD + 4) + 4 * di + k];
            }
        }
        const bool upd = ec.any(active && vchanged);
        if (upd)
            for (int k = 0; k < 3; ++k) obs_goal[k] = d.goal[k];
    }
    QS_STAMP(21);

    // The drone state is final here (unless its env resets below, which stores it again): storing it now
    // lets its write-through bytes drain while the observations are computed.
    if (kp.stats) store_drone_q<Q, true, NIW>(kp, b, g, q, active, d, stw, stmask);
    else store_drone_q<Q, false, NIW>(kp, b, g, q, active, d);
    if (lead) {
        b.rew[g] = rw;
        b.done[g] = done ? 1 : 0;
    }
    if (kp.rcomp && active) {   // per-step infos: the reward components (QS_RI_*), fields dealt over the sub-lanes
        const float rc[QS_NRI] = {rc_dist, rc_effort, floor_now ? 1.f : 0.f, rc_orient, rc_spin,
                                  (any_uniq && uniq) ? -1.f : 0.f, -(kp.cdt * pen), onew ? -1.f : 0.f};
#pragma unroll
        for (int t = 0; t < (QS_NRI + Q - 1) / Q; ++t) {
            float v = rc[t * Q];
#pragma unroll
            for (int k = 1; k < Q; ++k)
                if (q == k && t * Q + k < QS_NRI) v = rc[t * Q + k];
            if (t * Q + q < QS_NRI) b.rcomp[(size_t)(t * Q + q) * kp.I + g] = v;
        }
    }
    QS_STAMP(4);
    if (SCEN_STEP) QS_PRIO_DROP(23);   // goal-scenario kernels: c3mix 9.38 -> 9.30 us (C3 neutral-to-worse: kept)
    // ---- observations (post-impulse state; quadrotor_multi.py:704-720) ----
    const bool nbr = kp.neighbor == QS_NEIGHBOR_POS_VEL && kp.K > 0;
    if (nbr && ec.wany(vchanged)) {  // impulses changed velocities: refresh the tile
        lds_sync();
        if (q == 0) xch_put(xch, dbase + di, d.pos, d.vel);
        lds_sync();
    }
    QS_STAMP(5);
    if (lead) {
        Drone dv = d;   // the self obs measure against the goal the reference's observation saw
        for (int k = 0; k < 3; ++k) dv.goal[k] = obs_goal[k];
        self_obs_z(kp, dv, zs, rng, gid, S_SENSOR, row);
    }
    QS_STAMP(6);
    if (nbr) neighbor_obs<NPAD, Q>(kp, xch, dbase, di, q, d.pos, d.vel, active, row);
    if (OBST && active) sdf_obs_q<Q>(kp, og, myob, d.pos[0], d.pos[1], row + kp.obs_dim - 9, q);   // MultiObstacles.step
    QS_STAMP(7);
    // non-finite guard of the stepped drone and its reward (before a fused reset replaces the drone)
    const bool state_bad = lead && drone_nonfinite(d), rew_bad = lead && !(rw * 0.f == 0.f);

    // a WIDE workgroup holds one env: bit 0 = it finished
    const uint64_t dball = WIDE ? (ec.wany(active && done) ? 1ull : 0ull) : __ballot(active && done);
    if (dball) {  // rare: some env of this block finished -> terminal obs + fused auto-reset (:739-838)
        lds_sync();
        // terminal obs: the finished envs' rows (contiguous in the tile and in HBM), all lanes of the wave;
        // an env's done flag is its lead lane's bit of the ballot (no memory access)
        const int nrow = kp.N * kp.obs_dim;
        for (int e = 0; e < nenv_blk; ++e) {
            if (!((dball >> (e * LPE)) & 1ull)) continue;
            float* dst = b.term + (size_t)(env0 + e) * nrow;
            const float* src = lds + (size_t)e * nrow;
            for (int c = lane; c < nrow; c += WGS) dst[c] = src[c];
        }
        lds_sync();
        if (kp.stats) {   // the finished episode's episode_extra_stats rows (quadrotor_multi.py:739-831)
            // the env's counters from the lanes that hold them (every lane takes part in the permutes)
            float cv[NCNT];
            if constexpr (WIDE) {   // counter k lives on lane k (the first wave): through LDS words 16.. of wscr
                int* cx = reinterpret_cast<int*>(wscr + 8);
                if (li < NCNT) cx[li] = cnt[0];
                lds_sync();
#pragma unroll
                for (int k = 0; k < NCNT; ++k) cv[k] = (float)cx[k];
            } else {
#pragma unroll
                for (int k = 0; k < NCNT; ++k) cv[k] = (float)__shfl(cnt[k / LPE], lbase + k % LPE);
            }
            auto env_bits = [&](bool x) { return ec.bits(x && q == 0); };
            const Row hit_a = env_bits(active && (d.flags & QS_FL_HIT_AGENT));
            const Row hit_o = env_bits(active && (d.flags & QS_FL_HIT_OBST));
            const Row reach = env_bits(active && (d.flags & QS_FL_REACHED));
            const Row all = env_bits(active);
            if (active && done && q == 0) {
                const float n = (float)kp.N;
                const Row ok = all & ~hit_a & ~hit_o;   // logical_and(agent_col_agent, agent_col_obst)
                float* row = b.estats + (size_t)g * QS_NES;
                const int E = kp.E;
#pragma unroll
                for (int k = 0; k < NCNT; ++k) row[QS_ES_COL + k] = cv[k];
                row[QS_ES_SUCCESS] = (float)row_popc(ok & reach) / n;
                row[QS_ES_DEADLOCK] = (float)row_popc(ok & ~reach) / n;
                row[QS_ES_COLRATE] = 1.f - (float)row_popc(ok) / n;
                row[QS_ES_NCOLRATE] = 1.f - (float)row_popc(all & ~hit_a) / n;
                row[QS_ES_OCOLRATE] = 1.f - (float)row_popc(all & ~hit_o) / n;
                row[QS_ES_SCEN] = (OBST || SCEN) ? (float)b.env[QS_E_SC_MODE * E + env] : 0.f;
                const int T = kpm.ep_len + 1;
#pragma unroll
                for (int k = 0; k < 3; ++k) row[QS_ES_D1 + k] = dsum[k] / (float)min(kp.st_win[k], T) / kp.dt;
                const int32_t* rri = gptr<int32_t>(rargs->ri);
                row[QS_ES_REPLAY] = (rri != nullptr && rri[QS_R_SAVED * E + env]) ? 1.f : 0.f;
            }
            // QuadrotorEnvMulti.reset zeroes the statistics (:487-509): the drone's entries go out with the reset
            // drone's state store below, the env's counters from the lanes that hold them
#pragma unroll
            for (int t = 0; t < CT; ++t) {
                const int k = li + LPE * t;
                if (envok && done && k < NCNT && cnt_live(k)) {
                    cnt[t] = 0;
                    cdirty[t] = true;
                }
            }
        }
        float sv[3] = {d.vel[0], d.vel[1], d.vel[2]};  // QuadrotorEnvMulti.vel seen by the reset (:477)
        if (OBST) {   // new obstacle map + scenario per finished env (one lane each)
            if (active && done && di == 0 && q == 0) {
                oscr[el].mi = omi;
                oscr[el].si = osi;
                Scen so;
                obstacle_reset_env(kp, rng, kp.id0 + (uint32_t)(env * kp.N), oscr + el, otile + el * kp.M,
                                   OSCEN ? &so : nullptr, OSCEN ? stab : nullptr);
                if (kp.dr) {
                    b.env[QS_E_OBST_M * kp.E + env] = oscr[el].mi;
                    b.env[QS_E_OBST_SZ * kp.E + env] = oscr[el].si;
                }
                if (OSCEN) scen_store(kp, b, env, so);   // its mode word is the stats' scenario id
                else if (kp.stats) b.env[QS_E_SC_MODE * kp.E + env] = obst_stats_id(oscr[el].mode);   // the stats' name
            }
            lds_sync();
            if (active && done && kp.dr) og = ogeo(kp, oscr[el].mi, oscr[el].si);
        }
        if (SCEN) {   // scenario.reset() of every finished env (its lead lane), goals into the LDS table
            if (active && done && di == 0 && q == 0) {
                Scen sc;
                SDraw sd = sdraw(rng, gid, S_SCN_RESET);
                scen_reset(kp, sc, sd, stab, stab + 4 * (NPAD + 4));
                scen_store(kp, b, env, sc);
            }
            lds_sync();
        }
        if (active && done) {   // replicated: every sub-lane needs the new pose for the neighbour pass
            if (q == 0) {
                b.stale[0 * kp.I + g] = sv[0];
                b.stale[1 * kp.I + g] = sv[1];
                b.stale[2 * kp.I + g] = sv[2];
            }
            float spawn[3] = {kp.goal[0], kp.goal[1], kp.goal[2]}, goal[3] = {kp.goal[0], kp.goal[1], kp.goal[2]};
            if (OBST) obstacle_spawn_goal(kp, oscr + el, di, rng, gid, spawn, goal, OSCEN ? stab : nullptr);
            if (SCEN)   // spawn point = goal (quadrotor_multi.py:469-470)
                for (int k = 0; k < 3; ++k) spawn[k] = goal[k] = stab[4 * di + k];
            reset_drone(kp, d, rng, gid, spawn, goal);
        }
        if (kp.sense) {   // the reset obs' 3 sensor blocks dealt over the sub-lanes (all lanes: DPP)
            float zr[12], uu[1];
            qdraws<Q, 3, 0>(rng, gid, S_RESET_SENSOR, S_RESET_SENSOR, q, zr, uu);
            if (active && done && q == 0) self_obs_z(kp, d, zr, rng, gid, S_RESET_SENSOR, row);
        } else if (active && done && q == 0) {
            self_obs(kp, d, rng, gid, S_RESET_SENSOR, row);
        }
        // the reset drones' state (the stepped state was stored before the obs phase)
        if (kp.stats) {
            const float zero[STAT_WORDS] = {};
            store_drone_q<Q, true, NIW>(kp, b, g, q, active && done, d, zero, (1u << STAT_WORDS) - 1u);
        } else {
            store_drone_q<Q, false, NIW>(kp, b, g, q, active && done, d);
        }
        if (nbr) {
            if (q == 0) xch_put(xch, dbase + di, d.pos, sv);
            lds_sync();
            neighbor_obs<NPAD, Q>(kp, xch, dbase, di, q, d.pos, sv, active && done, row);
        }
        if (OBST && lead && done) {
            sdf_obs(kp, og, myob, d.pos[0], d.pos[1], row + kp.obs_dim - 9);   // MultiObstacles.reset
            if (di == 0)
                for (int o = 0; o < kp.M; ++o) b.obst[(size_t)env * kp.M + o] = myob[o];
        }
    }
    lds_sync();
    QS_STAMP(8);
    const int obs_bad = tile_store_v<tile_vecs<SLOTS, WGS>()>(lds, b.obs + (size_t)env0 * kp.N * kp.obs_dim, rows * kp.obs_dim,
                                                              lane, WGS);
    QS_STAMP(9);

    if (lead) {
        if (di == 0) {
            b.env[QS_E_TICK * kp.E + env] = done ? 0 : tick;
            if (done) b.env[QS_E_EPISODE * kp.E + env] = episode + 1;
            const int32_t ef = ef0;
            int32_t nf = done ? (ef | QS_EF_STALE) : (ef & ~QS_EF_STALE);
            // what the replay wrapper reads of this step (quad_experience_replay.py:161-163, quadrotor_multi.py:725)
            nf = (nf & ~(QS_EF_NEWCOL | QS_EF_FLOOR0)) | ((any_uniq || any_onew) ? QS_EF_NEWCOL : 0) |
                 (floor_now ? QS_EF_FLOOR0 : 0);
            if (nf != ef) b.env[QS_E_FLAGS * kp.E + env] = nf;
        }
    }
    // the env's episode counters that changed this step (a finished env's zeroed ones included), after every
    // other global access of the step: a store issued mid-step made the step's later memory waits wait for it
    if (kp.stats) {
#pragma unroll
        for (int t = 0; t < CT; ++t) {
            const int k = li + LPE * t;
            if (envok && k < NCNT && cdirty[t]) *cnt_at(k) = cnt[t];
        }
    }
    guard_count(b, obs_bad, rew_bad, state_bad);
    QS_STAMP(10);
    const RBufs r = load_rbufs(rargs);
    if (r.ri != nullptr) {   // experience replay on (uniform): ExperienceReplayWrapper.step of every env (:124-180)
        // the step's global stores above are read back by other lanes of the wave: workgroup-scope
        // release/acquire (one wave per workgroup, one L1)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (WIDE) lds_sync();   // the env's other wave has made its stores too
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        const RP rp = rargs->p;
        if (env < kp.E) replay_env<true>(kp, kpm, b, r, rp, seed, env, lane % LPE, LPE);
    }
    QS_STAMP(11);
    // slots 16 / 17: drones of the wave on the floor / in a drone collision this step
    QS_STAMP_NOTE(16, __builtin_popcountll(__ballot(active && q == 0 && (d.flags & QS_FL_ON_FLOOR))));
    QS_STAMP_NOTE(17, __builtin_popcountll(__ballot(active && q == 0 && row_any(cur))));
    QS_RTSTAMP(13);
    QS_STAMP_FLUSH();
}

// explicit reset of masked envs (QuadrotorEnvMulti.reset quadrotor_multi.py:440-517)
template <int NPAD, bool OBST>
__global__ __launch_bounds__(NPAD > 64 ? NPAD : 64) void reset_kernel(const KP* __restrict__ kpp, Bufs b) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    QS_BIND_KP(kpp);
    const uint32_t seed = kpm.seed;
    constexpr int WGS = NPAD > 64 ? NPAD : 64, EPB = WGS / NPAD, SLOTS = EPB * NPAD;   // one lane per drone
    constexpr bool WIDE = NPAD > 64;
    const int lane = threadIdx.x;
    const int el = lane / NPAD, di = lane % NPAD;
    const int env0 = blockIdx.x * EPB;
    const int env = env0 + el;
    const bool inr = env < kp.E && di < kp.N;
    const bool sel = inr && (b.mask == nullptr || b.mask[env] != 0);
    const int g = inr ? env * kp.N + di : 0;
    const int base = el * NPAD;
    const int eidx = inr ? env : 0;
    const int episode = b.env[QS_E_EPISODE * kp.E + eidx];
    const Rng rng = env_rng(seed, b.env[QS_E_TICK * kp.E + eidx], episode);
    float* row = lds + (size_t)(el * kp.N + di) * kp.obs_dim;
    Drone d;
    load_drone<WIDE>(kp, b, g, d);
    // stale QuadrotorEnvMulti.vel: the state's vel unless a reset already happened since the last step
    const bool stale_valid = inr && (b.env[QS_E_FLAGS * kp.E + env] & 1);
    float sv[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) sv[c] = stale_valid ? b.stale[c * kp.I + g] : d.vel[c];
    float2* otile = obst_tile(lds, kp, SLOTS);
    ObstScratch* oscr = reinterpret_cast<ObstScratch*>(otile + EPB * kp.M);
    float* stab = scen_tab_b<OBST>(lds, kp, SLOTS, EPB) + el * scen_stride<NPAD>();
    const bool OSCEN = OBST && kp.scen_b >= SC_O_SWAP_GOALS;
    if (OBST) {
        if (sel && di == 0) {
            oscr[el].mi = kp.dr ? b.env[QS_E_OBST_M * kp.E + env] : 0;
            oscr[el].si = kp.dr ? b.env[QS_E_OBST_SZ * kp.E + env] : 0;
            Scen so;
            obstacle_reset_env(kp, rng, kp.id0 + (uint32_t)(env * kp.N), oscr + el, otile + el * kp.M,
                               OSCEN ? &so : nullptr, OSCEN ? stab : nullptr);
            if (kp.dr) {
                b.env[QS_E_OBST_M * kp.E + env] = oscr[el].mi;
                b.env[QS_E_OBST_SZ * kp.E + env] = oscr[el].si;
            }
            if (OSCEN) scen_store(kp, b, env, so);
            else if (kp.stats) b.env[QS_E_SC_MODE * kp.E + env] = obst_stats_id(oscr[el].mode);
        }
        lds_sync();
    }
    const bool SCEN = !OBST && kp.scen_b >= 0;
    if (SCEN) {   // scenario.reset() (quadrotor_multi.py:449-459) by each selected env's lead lane
        if (sel && di == 0) {
            Scen sc;
            SDraw sd = sdraw(rng, kp.id0 + (uint32_t)g, S_SCN_RESET);
            scen_reset(kp, sc, sd, stab, stab + 4 * (NPAD + 4));
            scen_store(kp, b, env, sc);
        }
        lds_sync();
    }
    if (sel) {
        float spawn[3] = {kp.goal[0], kp.goal[1], kp.goal[2]}, goal[3] = {kp.goal[0], kp.goal[1], kp.goal[2]};
        if (OBST) obstacle_spawn_goal(kp, oscr + el, di, rng, kp.id0 + (uint32_t)g, spawn, goal, OSCEN ? stab : nullptr);
        if (SCEN)   // spawn point = goal (quadrotor_multi.py:469-470)
            for (int k = 0; k < 3; ++k) spawn[k] = goal[k] = stab[4 * di + k];
        reset_drone(kp, d, rng, kp.id0 + (uint32_t)g, spawn, goal);
        self_obs(kp, d, rng, kp.id0 + (uint32_t)g, S_RESET_SENSOR, row);
    }
    if (kp.neighbor == QS_NEIGHBOR_POS_VEL && kp.K > 0) {
        float4* xch = reinterpret_cast<float4*>(lds + SLOTS * kp.obs_dim);
        xch_put(xch, lane, d.pos, sv);
        lds_sync();
        neighbor_obs<NPAD, 1>(kp, xch, base, di, 0, d.pos, sv, sel, row);
    }
    if (OBST && sel) {
        const float2* myob = otile + el * kp.M;
        sdf_obs(kp, ogeo(kp, oscr[el].mi, oscr[el].si), myob, d.pos[0], d.pos[1], row + kp.obs_dim - 9);   // MultiObstacles.reset
        if (di == 0)
            for (int o = 0; o < kp.M; ++o) b.obst[(size_t)env * kp.M + o] = myob[o];
    }
    lds_sync();
    const int nenv_blk = min(EPB, kp.E - env0);
    for (int r = 0; r < nenv_blk * kp.N; ++r) {
        const int e = env0 + r / kp.N;
        if (b.mask != nullptr && b.mask[e] == 0) continue;
        for (int c = lane; c < kp.obs_dim; c += WGS)
            b.obs[(size_t)(env0 * kp.N + r) * kp.obs_dim + c] = lds[(size_t)r * kp.obs_dim + c];
    }
    if (sel) {
        store_drone<WIDE>(kp, b, g, d);
#pragma unroll
        for (int c = 0; c < 3; ++c) b.stale[c * kp.I + g] = sv[c];
        b.done[g] = 0;
        if (kp.stats) {   // QuadrotorEnvMulti.reset zeroes the episode statistics (quadrotor_multi.py:487-509)
#pragma unroll
            for (int k = 0; k < 5; ++k) b.st[(QS_F_DRING + k) * kp.I + g] = 0.f;
#pragma unroll
            for (int k = 0; k < 3; ++k) b.st[(QS_F_DSUM + k) * kp.I + g] = 0.f;
        }
        if (di == 0) {
            b.env[QS_E_TICK * kp.E + env] = 0;
            b.env[QS_E_EPISODE * kp.E + env] = episode + 1;
            b.env[QS_E_FLAGS * kp.E + env] |= 1;
            if (kp.stats)
                for (int k = 0; k < 11; ++k) b.env[(QS_E_ST_COL + k) * kp.E + env] = 0;
        }
    }
}

}  // namespace qs
