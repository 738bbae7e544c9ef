// qs_step.hip -- fused MI355X (gfx950) kernels for the quadrotor-swarm env step + the C ABI.
//
// Reference path replaced (priban42/quad-swarm-rl-stable-baselines3):
//   QuadrotorEnvMulti.step            gym_art/quadrotor_multi/quadrotor_multi.py:521-841
//   QuadrotorSingle._step / _reset    quadrotor_single.py:355-371 / :401-469
//   QuadrotorDynamics.step/step1_numba quadrotor_dynamics.py:215-221, :355-390, :504-656
//   RawControl.step                   quadrotor_control.py:53-57
//   SensorNoise.add_noise_numba       sensor_noise.py:172-261 ; get_state.py:226-292
//   collisions / room / downwash      collisions/quadrotors.py, collisions/room.py, aerodynamics/downwash.py
//
// Execution model: one lane per drone, all drones of an env inside one 64-lane
// wavefront (NPAD = next pow2 >= N lanes per env, 64/NPAD envs per wave), one wave per workgroup.
// Cross-drone work (collision matrix, proximity, neighbour top-k, impulses) uses wave shuffles, no
// LDS round trips and no barriers.  Observations are staged in LDS and written as contiguous
// 16-byte stores of the block's [rows, obs_dim] tile.  Everything is fp32; state is SoA in HBM.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <new>
#include <string>

#include "qs_rng.h"
#include "quadswarm.h"

namespace qs {

struct KP {
    int E, N, I, obs_dim, so_dim, K, neighbor, obs_repr, ep_len, sim_steps, svd_every, sense, downwash, collide;
    uint32_t id0;  // global id of drone 0 (RNG key offset)
    float dt, cdt, mass, inv_mass, inertia[3], inv_inertia[3];
    float thrust_max[4], torque_max[4], pc0[4], pc1[4], pc2[4], ccw[4];
    float tau_up, tau_down, lin, arm, grav, omega_max, vel_damp, dq, vxyz_max;
    float room_lo[3], room_hi[3], room_range[3];
    float ou_mu, ou_theta, ou_sigma;
    float pos_std, pos_unif, vel_std, vel_unif, gyro, quat_std, quat_unif;
    float col_thr, fall_thr, prox_ratio, prox_max;
    float rew_pos, rew_effort, rew_crash, rew_orient, rew_spin, quadcol;
    float spawn_box, goal[3];
};

struct Bufs {
    float* st;
    int32_t* ist;
    int32_t* env;
    float* stale;
    float* obs;
    float* term;
    float* rew;
    uint8_t* done;
    const float* act;
    const uint8_t* mask;
};

// Diagnostic phase stamps (build with -DQS_STAMPS=1 only; never in the shipped library): lane 0 of
// each block records s_memtime at phase boundaries; tools/phase_stamps.py reads them back.
#ifdef QS_STAMPS
__device__ uint64_t qs_dbg_stamps[65536 * 16];
#define QS_STAMP(k)                                                                                   \
    do {                                                                                              \
        uint64_t t_;                                                                                  \
        __builtin_amdgcn_sched_barrier(0);                                                            \
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
        __builtin_amdgcn_sched_barrier(0);                                                            \
        stamps_[k] = t_;                                                                              \
    } while (0)
#define QS_STAMP_FLUSH()                                                                              \
    do {                                                                                              \
        if (threadIdx.x == 0 && blockIdx.x < 65536)                                                   \
            for (int k_ = 0; k_ < 16; ++k_) qs_dbg_stamps[blockIdx.x * 16 + k_] = stamps_[k_];        \
    } while (0)
#define QS_STAMP_DECL uint64_t stamps_[16] = {0};
#else
#define QS_STAMP(k) do {} while (0)
#define QS_STAMP_FLUSH() do {} while (0)
#define QS_STAMP_DECL
#endif

struct Drone {
    float pos[3], vel[3], rot[9], om[3], rd[4], cd[4], ou[4], goal[3];
    int32_t svd;
    uint32_t flags;
    uint64_t prev;
};

__device__ __forceinline__ float clampf(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }
// single-instruction sqrt / reciprocal (v_sqrt_f32 / v_rcp_f32, ~1 ulp): the step is compared with the
// fp64 oracle at 1e-5..1e-4, far above these errors
__device__ __forceinline__ float fsqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
__device__ __forceinline__ float frcp(float x) { return __builtin_amdgcn_rcpf(x); }

// ---------------------------------------------------------------------------------------------
// state I/O (SoA, coalesced per field)
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void load_drone(const KP& kp, const Bufs& b, int g, Drone& d) {
    const float* s = b.st + g;
    const int I = kp.I;
#pragma unroll
    for (int i = 0; i < 3; ++i) { d.pos[i] = s[(QS_F_POS + i) * I]; d.vel[i] = s[(QS_F_VEL + i) * I]; }
#pragma unroll
    for (int i = 0; i < 9; ++i) d.rot[i] = s[(QS_F_ROT + i) * I];
#pragma unroll
    for (int i = 0; i < 3; ++i) { d.om[i] = s[(QS_F_OMEGA + i) * I]; d.goal[i] = s[(QS_F_GOAL + i) * I]; }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        d.rd[i] = s[(QS_F_ROT_DAMP + i) * I];
        d.cd[i] = s[(QS_F_CMD_DAMP + i) * I];
        d.ou[i] = s[(QS_F_OU + i) * I];
    }
    const int32_t* is = b.ist + g;
    d.svd = is[QS_I_SVD * I];
    d.flags = (uint32_t)is[QS_I_FLAGS * I];
    d.prev = (uint64_t)(uint32_t)is[QS_I_PREV_LO * I] | ((uint64_t)(uint32_t)is[QS_I_PREV_HI * I] << 32);
}

__device__ __forceinline__ void store_drone(const KP& kp, const Bufs& b, int g, const Drone& d) {
    float* s = b.st + g;
    const int I = kp.I;
#pragma unroll
    for (int i = 0; i < 3; ++i) { s[(QS_F_POS + i) * I] = d.pos[i]; s[(QS_F_VEL + i) * I] = d.vel[i]; }
#pragma unroll
    for (int i = 0; i < 9; ++i) s[(QS_F_ROT + i) * I] = d.rot[i];
#pragma unroll
    for (int i = 0; i < 3; ++i) { s[(QS_F_OMEGA + i) * I] = d.om[i]; s[(QS_F_GOAL + i) * I] = d.goal[i]; }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        s[(QS_F_ROT_DAMP + i) * I] = d.rd[i];
        s[(QS_F_CMD_DAMP + i) * I] = d.cd[i];
        s[(QS_F_OU + i) * I] = d.ou[i];
    }
    int32_t* is = b.ist + g;
    is[QS_I_SVD * I] = d.svd;
    is[QS_I_FLAGS * I] = (int32_t)d.flags;
    is[QS_I_PREV_LO * I] = (int32_t)(uint32_t)d.prev;
    is[QS_I_PREV_HI * I] = (int32_t)(uint32_t)(d.prev >> 32);
}

// ---------------------------------------------------------------------------------------------
// L1 physics: one substep == step1_numba (quadrotor_dynamics.py:355-390)
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void yaw_rot(float theta, float* R) {
    float s, c;
    sincosf(theta, &s, &c);
    R[0] = c; R[1] = -s; R[2] = 0.f;
    R[3] = s; R[4] = c; R[5] = 0.f;
    R[6] = 0.f; R[7] = 0.f; R[8] = 1.f;
}

// polar factor (u @ vh of the SVD, :554-558): Newton X <- (X + X^-T)/2; R is within ~1e-5 of
// orthonormal after 100 fp32 substeps, three iterations converge to fp32 precision.
__device__ __forceinline__ void polar3(float* x) {
#pragma unroll
    for (int it = 0; it < 3; ++it) {
        const float a = x[0], b = x[1], c = x[2], d = x[3], e = x[4], f = x[5], g = x[6], h = x[7], i = x[8];
        const float A = e * i - f * h, B = f * g - d * i, C = d * h - e * g;
        const float inv = frcp(a * A + b * B + c * C);
        const float cof[9] = {A, B, C, c * h - b * i, a * i - c * g, b * g - a * h, b * f - c * e, c * d - a * f,
                              a * e - b * d};
#pragma unroll
        for (int k = 0; k < 9; ++k) x[k] = 0.5f * (x[k] + cof[k] * inv);
    }
}

__device__ void substep(const KP& kp, Drone& d, const float* cmds, const float* noise, const Rng& rng, uint32_t gid,
                        int s) {
    const float dt = kp.dt;
    float thrusts[4], tq0 = 0.f, tq1 = 0.f, tq2 = 0.f, tsum = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // motor filter in sqrt space + multiplicative OU noise (:511-524)
        const float cmd = cmds[k];
        float tau = cmd < d.cd[k] ? kp.tau_down : kp.tau_up;
        tau = fminf(tau, 1.0f);
        d.rd[k] = tau * (fsqrt(cmd) - d.rd[k]) + d.rd[k];
        const float c = clampf(d.rd[k] * d.rd[k] + cmd * noise[k], 0.f, 1.f);
        d.cd[k] = c;
        thrusts[k] = kp.thrust_max[k] * ((1.f - kp.lin) * c * c + kp.lin * c);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // torques (:527-533)
        tq0 += kp.pc0[k] * thrusts[k];
        tq1 += kp.pc1[k] * thrusts[k];
        tq2 += kp.pc2[k] * thrusts[k] + kp.torque_max[k] * kp.ccw[k] * d.cd[k];
        tsum += thrusts[k];
    }
    float* R = d.rot;
    {  // Rodrigues with world-frame omega (:544-551):  dR = I + sin(a) K + (1 - cos a) K^2,
       // K = skew(w)/|w|, a = |w| dt.  Written as I + dt S(a^2) skew(w) + dt^2 C(a^2) (w w^T - |w|^2 I)
       // with S = sin(a)/a and C = (1 - cos a)/a^2: no sqrt, no division, no branch at w = 0 (where
       // the reference skips the update: dR = I exactly as the series gives).
        const float wx = R[0] * d.om[0] + R[1] * d.om[1] + R[2] * d.om[2];
        const float wy = R[3] * d.om[0] + R[4] * d.om[1] + R[5] * d.om[2];
        const float wz = R[6] * d.om[0] + R[7] * d.om[1] + R[8] * d.om[2];
        const float w2 = wx * wx + wy * wy + wz * wz;
        const float x = w2 * (dt * dt);
        float sf, cf;
        if (x < 0.36f) {  // a < 0.6: Taylor to a^8, truncation < 2e-10 (|omega| <= 40 per axis gives a <= 0.35)
            sf = dt * (1.f + x * (-1.f / 6.f + x * (1.f / 120.f + x * (-1.f / 5040.f + x * (1.f / 362880.f)))));
            cf = dt * dt * (0.5f + x * (-1.f / 24.f + x * (1.f / 720.f + x * (-1.f / 40320.f + x * (1.f / 3628800.f)))));
        } else {          // after collision kicks (|omega| up to ~100 rad/s before the clip)
            const float wn = fsqrt(w2), a = wn * dt;
            float sa, ca;
            sincosf(0.5f * a, &sa, &ca);
            sf = 2.f * sa * ca / wn;
            cf = 2.f * sa * sa / w2;
        }
        const float sx = sf * wx, sy = sf * wy, sz = sf * wz;
        const float d0 = 1.f - cf * w2;
        const float dR[9] = {d0 + cf * wx * wx, -sz + cf * wx * wy, sy + cf * wx * wz,
                             sz + cf * wx * wy, d0 + cf * wy * wy, -sx + cf * wy * wz,
                             -sy + cf * wx * wz, sx + cf * wy * wz, d0 + cf * wz * wz};
        float Rn[9];
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j)
                Rn[i * 3 + j] = dR[i * 3] * R[j] + dR[i * 3 + 1] * R[3 + j] + dR[i * 3 + 2] * R[6 + j];
#pragma unroll
        for (int i = 0; i < 9; ++i) R[i] = Rn[i];
    }
    if (++d.svd >= kp.svd_every) {  // since_last_svd > 0.5 s (:553-558)
        polar3(R);
        d.svd = 0;
    }
    {  // omega (:562-567)
        const float o0 = d.om[0], o1 = d.om[1], o2 = d.om[2];
        const float I0 = kp.inertia[0] * o0, I1 = kp.inertia[1] * o1, I2 = kp.inertia[2] * o2;
        const float c0 = -o1 * I2 + o2 * I1, c1 = -o2 * I0 + o0 * I2, c2 = -o0 * I1 + o1 * I0;
        const float od0 = kp.inv_inertia[0] * (c0 + tq0);
        const float od1 = kp.inv_inertia[1] * (c1 + tq1);
        const float od2 = kp.inv_inertia[2] * (c2 + tq2);
        const float dm0 = clampf(kp.dq * (o0 * o0), 0.f, 1.f), dm1 = clampf(kp.dq * (o1 * o1), 0.f, 1.f),
                    dm2 = clampf(kp.dq * (o2 * o2), 0.f, 1.f);
        d.om[0] = clampf(o0 + (1.f - dm0) * dt * od0, -kp.omega_max, kp.omega_max);
        d.om[1] = clampf(o1 + (1.f - dm1) * dt * od1, -kp.omega_max, kp.omega_max);
        d.om[2] = clampf(o2 + (1.f - dm2) * dt * od2, -kp.omega_max, kp.omega_max);
    }
    // position + room clip (:570, :367-374)
    float before[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        before[i] = d.pos[i] + dt * d.vel[i];
        d.pos[i] = clampf(before[i], kp.room_lo[i], kp.room_hi[i]);
    }
    uint32_t fl = d.flags & ~(uint32_t)(QS_FL_CRASH_FLOOR | QS_FL_CRASH_WALL | QS_FL_CRASH_CEIL);
    if (before[0] != d.pos[0] || before[1] != d.pos[1]) fl |= QS_FL_CRASH_WALL;
    if (before[2] > d.pos[2]) fl |= QS_FL_CRASH_CEIL;
    // floor (floor_interaction_numba :576-646, threshold = arm)
    float fx = R[2] * tsum, fy = R[5] * tsum, fz = R[8] * tsum;
    float ax, ay, az;
    if (d.pos[2] <= kp.arm) {
        d.pos[2] = kp.arm;
        if (fl & QS_FL_ON_FLOOR) {
            yaw_rot(atan2f(R[3], R[0] + 1e-6f), R);
            const float fric = 0.6f * (kp.mass * kp.grav - fz);
            const float vn = fsqrt(d.vel[0] * d.vel[0] + d.vel[1] * d.vel[1] + d.vel[2] * d.vel[2]);
            if (vn < 1e-6f) {
                float fxy = fsqrt(fx * fx + fy * fy);
                fxy = fmaxf(fxy - fric, 0.f);
                if (fxy == 0.f) {
                    fx = 0.f; fy = 0.f;
                } else {
                    float sa, ca;
                    sincosf(atan2f(fy, fx), &sa, &ca);
                    fx = fxy * ca; fy = fxy * sa;
                }
            } else {
                float sa, ca;
                sincosf(atan2f(d.vel[1], d.vel[0]), &sa, &ca);
                fx = fx - ca * fric;
                fy = fy - sa * fric;
            }
        } else {
            fl |= QS_FL_ON_FLOOR | QS_FL_CRASH_FLOOR;
#pragma unroll
            for (int i = 0; i < 3; ++i) { d.vel[i] = 0.f; d.om[i] = 0.f; }
            float theta = atan2f(R[3], R[0] + 1e-6f);
            if (R[8] < 0.f) theta = -3.14159265358979f + 6.28318530717959f * uniform1(rng, gid, S_FLOOR | ((uint32_t)s << 8), 0);
            yaw_rot(theta, R);
#pragma unroll
            for (int k = 0; k < 4; ++k) { d.cd[k] = 0.f; d.rd[k] = 0.f; }
        }
        ax = kp.inv_mass * fx;
        ay = kp.inv_mass * fy;
        az = fmaxf(-kp.grav + kp.inv_mass * fz, 0.f);
    } else {
        fl &= ~(uint32_t)QS_FL_ON_FLOOR;
        ax = kp.inv_mass * fx;
        ay = kp.inv_mass * fy;
        az = -kp.grav + kp.inv_mass * fz;
    }
    d.flags = fl;
    d.vel[0] = (1.f - kp.vel_damp) * d.vel[0] + dt * ax;  // (:652)
    d.vel[1] = (1.f - kp.vel_damp) * d.vel[1] + dt * ay;
    d.vel[2] = (1.f - kp.vel_damp) * d.vel[2] + dt * az;
}

// ---------------------------------------------------------------------------------------------
// observations
// ---------------------------------------------------------------------------------------------
// sensor noise (add_noise_numba sensor_noise.py:172-218) + state_xyz_vxyz_R_omega[_floor|_wall]
// (get_state.py:226-292), written to an LDS row.
__device__ void self_obs(const KP& kp, const Drone& d, const Rng& rng, uint32_t gid, uint32_t stream, float* out) {
    float np_[3], nv[3], no[3], nr[9];
    if (kp.sense) {
        float z[12];
        normals4(rng, gid, stream, 0, z);
        normals4(rng, gid, stream, 1, z + 4);
        normals4(rng, gid, stream, 2, z + 8);
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
        if (kp.quat_std != 0.f) {
            float zq[4];
            normals4(rng, gid, stream, 2, zq);  // normals 9..11 live in block 2, words 1..3
#pragma unroll
            for (int i = 0; i < 3; ++i) th[i] = kp.quat_std * zq[1 + i] + th[i];
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

// Neighbour exchange tile in LDS: lane l stores {pos, 0} at xch[2l] and {vel, 0} at xch[2l+1]; the
// drones of one env read each other's rows with broadcast ds_read_b128 (one wave per workgroup, so a
// workgroup barrier costs nothing but orders the LDS traffic).
// LDS-only workgroup barrier: workgroups are one wave, so this just orders LDS traffic.  Unlike
// __syncthreads() it does not wait for outstanding global stores (vmcnt) or fence global memory.
__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ void xch_put(float4* xch, int lane, const float* P, const float* V) {
    xch[2 * lane] = make_float4(P[0], P[1], P[2], 0.f);
    xch[2 * lane + 1] = make_float4(V[0], V[1], V[2], 0.f);
}

// pos_vel neighbour obs: neighborhood_indices (quadrotor_multi.py:344-375) + extend_obs_space
// clip (:328-342).  Key = |[rel_pos, rel_vel]| clamped at 0.01 (compared squared, clamp 1e-4);
// stable (index) tie-break like numpy's insertion sort; k == N-1 keeps index order (all keys 0).
// Reads the exchange tile (caller has synchronised); only lanes with write == true store.
template <int NPAD>
__device__ void neighbor_obs(const KP& kp, const float4* xch, int base, int di, const float* P, const float* V,
                             bool write, float* out) {
    constexpr bool KEEP = NPAD <= 8;  // small swarms keep the relative vectors in VGPRs between passes
    float key[NPAD];
    float rel[KEEP ? NPAD : 1][6];
    const bool sorted = kp.K < kp.N - 1;
#pragma unroll
    for (int j = 0; j < NPAD; ++j) {
        const float4 pj = xch[2 * (base + j)], vj = xch[2 * (base + j) + 1];
        const float r[6] = {pj.x - P[0], pj.y - P[1], pj.z - P[2], vj.x - V[0], vj.y - V[1], vj.z - V[2]};
        const float s = r[0] * r[0] + r[1] * r[1] + r[2] * r[2] + r[3] * r[3] + r[4] * r[4] + r[5] * r[5];
        const bool valid = (j != di) && (j < kp.N);
        key[j] = valid ? (sorted ? fmaxf(s, 1e-4f) : 0.f) : __builtin_inff();
        if (KEEP) {
#pragma unroll
            for (int c = 0; c < 6; ++c) rel[KEEP ? j : 0][c] = r[c];
        }
    }
    if (!write) return;
    const float vm = 2.f * kp.vxyz_max;
    const bool pairs = ((kp.so_dim | kp.obs_dim) & 1) == 0;   // 8-byte aligned slots: ds_write_b64
#pragma unroll
    for (int j = 0; j < NPAD; ++j) {
        int rank = 0;
#pragma unroll
        for (int m = 0; m < NPAD; ++m) rank += (key[m] < key[j]) || (m < j && key[m] == key[j]);
        if (key[j] != __builtin_inff() && rank < kp.K) {
            float r[6];
            if (KEEP) {
#pragma unroll
                for (int c = 0; c < 6; ++c) r[c] = rel[KEEP ? j : 0][c];
            } else {
                const float4 pj = xch[2 * (base + j)], vj = xch[2 * (base + j) + 1];
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
// Both lanes of the pair evaluate it with identical inputs and draws (key = lower drone, stream j).
__device__ void collide_pair(const float* p1, float* v1, float* w1, const float* p2, float* v2, float* w2,
                             const Rng& rng, uint32_t gid, uint32_t j) {
    const uint32_t st = S_PAIR | (j << 8);
    float n[3] = {p1[0] - p2[0], p1[1] - p2[1], p1[2] - p2[2]};
    const float m = fsqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
    const float im = frcp(m == 0.f ? 1e-5f : m);
    n[0] *= im; n[1] *= im; n[2] *= im;
    const float v1n = v1[0] * n[0] + v1[1] * n[1] + v1[2] * n[2];
    const float v2n = v2[0] * n[0] + v2[1] * n[1] + v2[2] * n[2];
    float vc[3], s1[3], s2[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) { vc[i] = (v2n - v1n) * n[i]; s1[i] = vc[i]; s2[i] = -vc[i]; }
    for (int t = 0; t < 3; ++t) {  // "make sure new vel direction would be opposite" rejection, 3 tries
        float z[12];  // normals t*9 .. t*9+8 lie in blocks (t*9)/4 .. (t*9+8)/4
        const uint32_t b0 = (uint32_t)(t * 9) >> 2, off = (uint32_t)(t * 9) & 3;
        normals4(rng, gid, st, b0, z);
        normals4(rng, gid, st, b0 + 1, z + 4);
        normals4(rng, gid, st, b0 + 2, z + 8);
        float d1 = 0.f, d2 = 0.f;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const float cons = 0.8f * z[off + i], a = 0.15f * z[off + 3 + i], bb = 0.15f * z[off + 6 + i];
            s1[i] = vc[i] + (cons + a);
            s2[i] = -vc[i] + (-cons + bb);
            d1 += (v1[i] + s1[i]) * n[i];
            d2 += (v2[i] + s2[i]) * n[i];
        }
        if (d1 > 0.f && 0.f > d2) break;
    }
    const float mx = fmaxf(fsqrt(v1[0] * v1[0] + v1[1] * v1[1] + v1[2] * v1[2]),
                           fsqrt(v2[0] * v2[0] + v2[1] * v2[1] + v2[2] * v2[2]));
    float u[8];
    uniforms4(rng, gid, st, 0, u);
    uniforms4(rng, gid, st, 1, u + 4);
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

// perform_collision_with_wall (collisions/room.py:6-44) / _with_ceiling (:91-113)
__device__ void collide_room(const KP& kp, Drone& d, const Rng& rng, uint32_t gid, bool wall) {
    const uint32_t st = wall ? S_WALL : S_CEIL;
    float u[12];
    uniforms4(rng, gid, st, 0, u);
    uniforms4(rng, gid, st, 1, u + 4);
    uniforms4(rng, gid, st, 2, u + 8);
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
// reset (QuadrotorSingle._reset quadrotor_single.py:401-469 with static_same_goal goals)
// ---------------------------------------------------------------------------------------------
__device__ void reset_drone(const KP& kp, Drone& d, const Rng& rng, uint32_t gid) {
    float u[4];
    uniforms4(rng, gid, S_RESET, 0, u);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        d.goal[i] = kp.goal[i];
        d.pos[i] = (-kp.spawn_box + 2.f * kp.spawn_box * u[i]) + d.goal[i];
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
            sincosf(cand, &s, &c);
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
}

// ---------------------------------------------------------------------------------------------
// block-level obs staging: LDS tile [rows, obs_dim] -> contiguous global rows
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void tile_store(const float* lds, float* dst, int nfloat, int lane) {
    // dst = first row of the block; rows are contiguous in HBM.  obs is 256-B aligned and a block owns
    // 64/NPAD*N rows, so the start is 16-B aligned whenever rows*obs_dim*4 is: b128 in, dwordx4 out.
    if ((((uintptr_t)dst) & 15) == 0) {
        const int nvec = nfloat >> 2;
        const float4* lv = reinterpret_cast<const float4*>(lds);
        float4* dv = reinterpret_cast<float4*>(dst);
        for (int v = lane; v < nvec; v += 64) dv[v] = lv[v];
        const int t = (nvec << 2) + lane;
        if (t < nfloat) dst[t] = lds[t];
    } else {
        for (int f = lane; f < nfloat; f += 64) dst[f] = lds[f];
    }
}

// ---------------------------------------------------------------------------------------------
// the fused step kernel
// ---------------------------------------------------------------------------------------------
// Philox counter of an env = {tick, episode}: unique for every step and reset of that env, resident
// with the env state (no global counter, no atomics), so a hipGraph replay of K steps draws K fresh
// streams and sharding envs over GPUs does not change any draw.
__device__ __forceinline__ Rng env_rng(uint32_t seed, int32_t tick, int32_t episode) {
    Rng r;
    r.seed = seed;
    r.ctr_lo = (uint32_t)tick;
    r.ctr_hi = (uint32_t)episode;
    return r;
}

template <int NPAD>
__global__ __launch_bounds__(64) void step_kernel(const KP* __restrict__ kpp, Bufs b, uint32_t seed) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const KP& kp = *kpp;
    QS_STAMP_DECL
    QS_STAMP(0);
    constexpr int EPB = 64 / NPAD;
    const int lane = threadIdx.x;
    const int el = lane / NPAD, di = lane % NPAD;
    const int env0 = blockIdx.x * EPB;
    const int env = env0 + el;
    const bool active = env < kp.E && di < kp.N;
    const int g = active ? env * kp.N + di : 0;
    const uint32_t gid = kp.id0 + (uint32_t)g;
    const int base = el * NPAD;
    const int nenv_blk = min(EPB, kp.E - env0);
    const int rows = nenv_blk * kp.N;
    float* row = lds + (size_t)(el * kp.N + di) * kp.obs_dim;
    float4* xch = reinterpret_cast<float4*>(lds + 64 * kp.obs_dim);

    Drone d;
    load_drone(kp, b, g, d);
    float a[4];
    {
        const float4 av = reinterpret_cast<const float4*>(b.act)[g];
        a[0] = av.x; a[1] = av.y; a[2] = av.z; a[3] = av.w;
    }
    const int eidx = active ? env : 0;
    const int tick0 = b.env[QS_E_TICK * kp.E + eidx];
    const int episode = b.env[QS_E_EPISODE * kp.E + eidx];
    const Rng rng = env_rng(seed, tick0, episode);
    const int tick = tick0 + 1;
    const bool done = tick > kp.ep_len;

    QS_STAMP(1);
    // ---- per-drone control + physics (QuadrotorSingle._step) ----
    float rw = 0.f;
    {
        float z[4];
        normals4(rng, gid, S_OU, 0, z);  // OUNoiseNumba.noise, once per control step (:216)
#pragma unroll
        for (int k = 0; k < 4; ++k) d.ou[k] = d.ou[k] + (kp.ou_theta * (kp.ou_mu - d.ou[k]) + kp.ou_sigma * z[k]);
        float cmds[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) cmds[k] = 0.5f * (clampf(a[k], -1.f, 1.f) + 1.f);
        for (int s = 0; s < kp.sim_steps; ++s) substep(kp, d, cmds, d.ou, rng, gid, s);
        // compute_reward_weighted (quadrotor_single.py:34-66)
        const float gx = d.goal[0] - d.pos[0], gy = d.goal[1] - d.pos[1], gz = d.goal[2] - d.pos[2];
        const bool on_floor = d.flags & QS_FL_ON_FLOOR;
        const float cost = kp.rew_pos * fsqrt(gx * gx + gy * gy + gz * gz) +
                           kp.rew_effort * fsqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2] + a[3] * a[3]) +
                           kp.rew_crash * (on_floor ? 1.f : 0.f) + kp.rew_orient * (on_floor ? 1.f : -d.rot[8]) +
                           kp.rew_spin * fsqrt(d.om[0] * d.om[0] + d.om[1] * d.om[1] + d.om[2] * d.om[2]);
        rw = -kp.dt * cost;
    }

    QS_STAMP(2);
    // ---- swarm phase: collisions + proximity (quadrotor_multi.py:537-568, 608-622) ----
    uint64_t cur = 0;
    float pen = 0.f;
    xch_put(xch, lane, d.pos, d.vel);
    lds_sync();
    if (kp.N > 1) {
#pragma unroll
        for (int j = 0; j < NPAD; ++j) {
            const float4 pj = xch[2 * (base + j)];
            const float dx = d.pos[0] - pj.x, dy = d.pos[1] - pj.y, dz = d.pos[2] - pj.z;
            const float dist = fsqrt(dx * dx + dy * dy + dz * dz);
            if (j != di && j < kp.N) {
                if (dist <= kp.col_thr) cur |= 1ull << j;
                if (dist <= kp.fall_thr) pen += kp.prox_ratio * dist + kp.prox_max;
            }
        }
    }
    const uint64_t newpairs = cur & ~d.prev;
    // setdiff1d(flat(cur), flat(prev)) and its ".any()" (drone 0 alone does not count)
    const bool uniq = active && cur != 0 && d.prev == 0;
    const uint64_t ub = __ballot(uniq && di != 0);
    const uint64_t gmask = (NPAD == 64) ? ~0ull : ((1ull << NPAD) - 1ull);
    const bool any_uniq = ((ub >> base) & gmask) != 0;
    rw += kp.quadcol * ((any_uniq && uniq) ? -1.f : 0.f);
    rw += -(kp.cdt * pen);
    // room: new wall / ceiling crashes vs the previous NEW lists (:390-403, :604-605)
    const bool wall_new = (d.flags & QS_FL_CRASH_WALL) && !(d.flags & QS_FL_PREV_WALL);
    const bool ceil_new = (d.flags & QS_FL_CRASH_CEIL) && !(d.flags & QS_FL_PREV_CEIL);
    d.flags = (d.flags & ~(uint32_t)(QS_FL_PREV_WALL | QS_FL_PREV_CEIL)) | (wall_new ? QS_FL_PREV_WALL : 0u) |
              (ceil_new ? QS_FL_PREV_CEIL : 0u);

    QS_STAMP(3);
    // ---- random forces (:659-698) ----
    bool vchanged = false;
    if (kp.downwash && kp.N > 1) {  // perform_downwash (aerodynamics/downwash.py:4-51)
        float dwu[4];
        uniforms4(rng, gid, S_DW, 0, dwu);
        const float an = -0.1f + 0.2f * dwu[0], wn = -0.01f + 0.02f * dwu[1];
        const float P0 = d.pos[0], P1 = d.pos[1], P2 = d.pos[2];
        for (int i = 0; i < NPAD; ++i) {
            const float zi0 = __shfl(d.rot[2], base + i), zi1 = __shfl(d.rot[5], base + i), zi2 = __shfl(d.rot[8], base + i);
            const float pi0 = __shfl(P0, base + i), pi1 = __shfl(P1, base + i), pi2 = __shfl(P2, base + i);
            const float ani = __shfl(an, base + i), wni = __shfl(wn, base + i);
            if (!active || i >= kp.N || i == di) continue;
            const float r0 = P0 - pi0, r1 = P1 - pi1, r2 = P2 - pi2;
            const float dist = fsqrt(r0 * r0 + r1 * r1 + r2 * r2);
            const float rz = r0 * zi0 + r1 * zi1 + r2 * zi2;
            const float rxy = fsqrt(dist * dist - rz * rz);
            if (-0.7f < rz && rz < 0.f && rxy < 0.1f) {
                const float acc = fmaxf((6.f / 17.f) * (-10.f * dist + 7.f) + ani, 1e-6f);
                const float wd = fmaxf(0.3f * (dist - 1.f) * (dist - 1.f) + wni, 1e-6f);
                float u[8];
                const uint32_t gi = kp.id0 + (uint32_t)(env * kp.N + i);
                uniforms4(rng, gi, S_DWPAIR | ((uint32_t)di << 8), 0, u);
                uniforms4(rng, gi, S_DWPAIR | ((uint32_t)di << 8), 1, u + 4);
                float nz[3] = {zi0 - 0.1f + 0.2f * u[0], zi1 - 0.1f + 0.2f * u[1], zi2 - 0.1f + 0.2f * u[2]};
                const float nm = fsqrt(nz[0] * nz[0] + nz[1] * nz[1] + nz[2] * nz[2]);
                const float inz = frcp(nm == 0.f ? 1e-6f : nm);
                float dw[3] = {-1.f + 2.f * u[3], -1.f + 2.f * u[4], -1.f + 2.f * u[5]};
                const float dm = fsqrt(dw[0] * dw[0] + dw[1] * dw[1] + dw[2] * dw[2]);
                const float idw = frcp(dm == 0.f ? 1e-6f : dm);
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    d.vel[c] += acc * (-(nz[c] * inz)) * kp.cdt;
                    d.om[c] += wd * (dw[c] * idw) * kp.cdt;
                }
                vchanged = true;
            }
        }
    }
    if (kp.collide) {
        // drone-drone impulses, pairs in (i, j) order; a wave-uniform loop over pending events
        uint64_t pend = active ? (newpairs & ~((2ull << di) - 1ull)) : 0ull;
        for (;;) {
            const uint64_t bal = __ballot(pend != 0ull);
            if (bal == 0ull) break;
            const uint64_t eb = (bal >> base) & gmask;
            const int istar = eb ? (__ffsll((long long)eb) - 1) : 0;
            const int myj = pend ? (__ffsll((long long)pend) - 1) : 0;
            const int jstar = __shfl(myj, base + istar);
            const int partner = (di == istar) ? jstar : istar;
            float pp[3], pv[3], pw[3];
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                pp[c] = __shfl(d.pos[c], base + partner);
                pv[c] = __shfl(d.vel[c], base + partner);
                pw[c] = __shfl(d.om[c], base + partner);
            }
            const bool involved = eb != 0 && (di == istar || di == jstar);
            vchanged |= involved;
            if (involved) {
                const uint32_t gi = kp.id0 + (uint32_t)(env * kp.N + istar);
                if (di == istar) collide_pair(d.pos, d.vel, d.om, pp, pv, pw, rng, gi, (uint32_t)jstar);
                else collide_pair(pp, pv, pw, d.pos, d.vel, d.om, rng, gi, (uint32_t)jstar);
            }
            if (eb != 0 && di == istar) pend &= ~(1ull << jstar);
        }
        if (active && wall_new) collide_room(kp, d, rng, gid, true);
        if (active && ceil_new) collide_room(kp, d, rng, gid, false);
        vchanged |= active && (wall_new || ceil_new);
    }
    d.prev = cur;

    QS_STAMP(4);
    // ---- observations (post-impulse state; quadrotor_multi.py:704-720) ----
    const bool nbr = kp.neighbor == QS_NEIGHBOR_POS_VEL && kp.K > 0;
    if (nbr && __ballot(vchanged)) {  // impulses changed velocities: refresh the tile
        lds_sync();
        xch_put(xch, lane, d.pos, d.vel);
        lds_sync();
    }
    QS_STAMP(5);
    if (active) self_obs(kp, d, rng, gid, S_SENSOR, row);
    QS_STAMP(6);
    if (nbr) neighbor_obs<NPAD>(kp, xch, base, di, d.pos, d.vel, active, row);
    QS_STAMP(7);

    const uint64_t dball = __ballot(active && done);
    if (dball) {  // rare: some env of this block finished -> terminal obs + fused auto-reset (:739-838)
        lds_sync();
        for (int r = 0; r < rows; ++r) {
            const int e = env0 + r / kp.N;
            if (b.env[QS_E_TICK * kp.E + e] + 1 <= kp.ep_len) continue;
            for (int c = lane; c < kp.obs_dim; c += 64)
                b.term[(size_t)(env0 * kp.N + r) * kp.obs_dim + c] = lds[(size_t)r * kp.obs_dim + c];
        }
        lds_sync();
        float sv[3] = {d.vel[0], d.vel[1], d.vel[2]};  // QuadrotorEnvMulti.vel seen by the reset (:477)
        if (active && done) {
            b.stale[0 * kp.I + g] = sv[0];
            b.stale[1 * kp.I + g] = sv[1];
            b.stale[2 * kp.I + g] = sv[2];
            reset_drone(kp, d, rng, gid);
            self_obs(kp, d, rng, gid, S_RESET_SENSOR, row);
        }
        if (nbr) {
            xch_put(xch, lane, d.pos, sv);
            lds_sync();
            neighbor_obs<NPAD>(kp, xch, base, di, d.pos, sv, active && done, row);
        }
    }
    lds_sync();
    QS_STAMP(8);
    tile_store(lds, b.obs + (size_t)env0 * kp.N * kp.obs_dim, rows * kp.obs_dim, lane);
    QS_STAMP(9);

    if (active) {
        store_drone(kp, b, g, d);
        b.rew[g] = rw;
        b.done[g] = done ? 1 : 0;
        if (di == 0) {
            b.env[QS_E_TICK * kp.E + env] = done ? 0 : tick;
            if (done) b.env[QS_E_EPISODE * kp.E + env] = episode + 1;
            const int32_t ef = b.env[QS_E_FLAGS * kp.E + env];
            const int32_t nf = done ? (ef | 1) : (ef & ~1);
            if (nf != ef) b.env[QS_E_FLAGS * kp.E + env] = nf;
        }
    }
    QS_STAMP(10);
    QS_STAMP(11);
    QS_STAMP_FLUSH();
}

// explicit reset of masked envs (QuadrotorEnvMulti.reset quadrotor_multi.py:440-517)
template <int NPAD>
__global__ __launch_bounds__(64) void reset_kernel(const KP* __restrict__ kpp, Bufs b, uint32_t seed) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const KP& kp = *kpp;
    constexpr int EPB = 64 / NPAD;
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
    load_drone(kp, b, g, d);
    // stale QuadrotorEnvMulti.vel: the state's vel unless a reset already happened since the last step
    const bool stale_valid = inr && (b.env[QS_E_FLAGS * kp.E + env] & 1);
    float sv[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) sv[c] = stale_valid ? b.stale[c * kp.I + g] : d.vel[c];
    if (sel) {
        reset_drone(kp, d, rng, kp.id0 + (uint32_t)g);
        self_obs(kp, d, rng, kp.id0 + (uint32_t)g, S_RESET_SENSOR, row);
    }
    if (kp.neighbor == QS_NEIGHBOR_POS_VEL && kp.K > 0) {
        float4* xch = reinterpret_cast<float4*>(lds + 64 * kp.obs_dim);
        xch_put(xch, lane, d.pos, sv);
        lds_sync();
        neighbor_obs<NPAD>(kp, xch, base, di, d.pos, sv, sel, row);
    }
    lds_sync();
    const int nenv_blk = min(EPB, kp.E - env0);
    for (int r = 0; r < nenv_blk * kp.N; ++r) {
        const int e = env0 + r / kp.N;
        if (b.mask != nullptr && b.mask[e] == 0) continue;
        for (int c = lane; c < kp.obs_dim; c += 64)
            b.obs[(size_t)(env0 * kp.N + r) * kp.obs_dim + c] = lds[(size_t)r * kp.obs_dim + c];
    }
    if (sel) {
        store_drone(kp, b, g, d);
#pragma unroll
        for (int c = 0; c < 3; ++c) b.stale[c * kp.I + g] = sv[c];
        b.done[g] = 0;
        if (di == 0) {
            b.env[QS_E_TICK * kp.E + env] = 0;
            b.env[QS_E_EPISODE * kp.E + env] = episode + 1;
            b.env[QS_E_FLAGS * kp.E + env] |= 1;
        }
    }
}

}  // namespace qs

// =============================================================================================
// C ABI
// =============================================================================================
struct qs_handle {
    qs_config cfg;
    qs::KP kp;
    qs_layout lay;
    int device;
    void* ws;
    bool owns_ws;
    int npad;
};

static thread_local std::string g_err;

static int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define QS_HIP(call)                                                                              \
    do {                                                                                          \
        hipError_t e_ = (call);                                                                   \
        if (e_ != hipSuccess) return fail(QS_E_HIP, std::string(#call ": ") + hipGetErrorString(e_)); \
    } while (0)

extern "C" int qs_abi_version(void) { return QS_ABI_VERSION; }

#ifdef QS_STAMPS
extern "C" int qs_debug_stamps(uint64_t* host, size_t n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(qs::qs_dbg_stamps), n * sizeof(uint64_t)) == hipSuccess ? 0 : -3;
}
#endif
extern "C" const char* qs_last_error(void) { return g_err.c_str(); }

extern "C" int qs_struct_sizes(size_t* c, size_t* l, size_t* b) {
    if (!c || !l || !b) return fail(QS_E_INVALID, "NULL argument");
    *c = sizeof(qs_config);
    *l = sizeof(qs_layout);
    *b = sizeof(qs_buffers);
    return QS_OK;
}

static int self_obs_dim(int repr) {
    return repr == QS_OBS_XYZ_VXYZ_R_OMEGA ? 18 : (repr == QS_OBS_XYZ_VXYZ_R_OMEGA_FLOOR ? 19 : 24);
}

static int validate(const qs_config* c) {
    if (!c) return fail(QS_E_INVALID, "config is NULL");
    if (c->abi_version != QS_ABI_VERSION) return fail(QS_E_INVALID, "config abi_version mismatch");
    if (c->num_envs < 1) return fail(QS_E_INVALID, "num_envs must be >= 1");
    if (c->num_agents < 1 || c->num_agents > QS_MAX_AGENTS)
        return fail(QS_E_UNSUPPORTED, "num_agents must be in [1, QS_MAX_AGENTS]");
    if (c->obs_repr < 0 || c->obs_repr > 2) return fail(QS_E_INVALID, "unknown obs_repr");
    if (c->neighbor_obs != QS_NEIGHBOR_NONE && c->neighbor_obs != QS_NEIGHBOR_POS_VEL)
        return fail(QS_E_UNSUPPORTED, "neighbor_obs type not implemented");
    if (c->neighbor_obs == QS_NEIGHBOR_POS_VEL && (c->k_neighbors < 1 || c->k_neighbors > c->num_agents - 1))
        return fail(QS_E_INVALID, "k_neighbors must be in [1, num_agents-1] for pos_vel");
    if (c->sim_steps < 1 || c->svd_every < 1 || c->ep_len < 0) return fail(QS_E_INVALID, "bad sim_steps/svd_every/ep_len");
    if ((long long)c->num_envs * c->num_agents > (1ll << 31) / 64) return fail(QS_E_INVALID, "too many drones");
    return QS_OK;
}

static qs_layout make_layout(const qs_config* c) {
    qs_layout L;
    memset(&L, 0, sizeof L);
    const size_t I = (size_t)c->num_envs * c->num_agents;
    const int od = self_obs_dim(c->obs_repr) + (c->neighbor_obs == QS_NEIGHBOR_POS_VEL ? 6 * c->k_neighbors : 0);
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    size_t o = 0;
    L.params = o; o = al(o + sizeof(qs::KP));
    L.state = o; o = al(o + sizeof(float) * QS_NF * I);
    L.istate = o; o = al(o + sizeof(int32_t) * QS_NI * I);
    L.env = o; o = al(o + sizeof(int32_t) * QS_NE * (size_t)c->num_envs);
    L.stale_vel = o; o = al(o + sizeof(float) * 3 * I);
    L.obs = o; o = al(o + sizeof(float) * I * od);
    L.term_obs = o; o = al(o + sizeof(float) * I * od);
    L.rew = o; o = al(o + sizeof(float) * I);
    L.done = o; o = al(o + I);
    L.total_bytes = o;
    L.obs_dim = od;
    L.num_drones = (int32_t)I;
    return L;
}

static qs::KP make_kp(const qs_config* c, const qs_layout& L) {
    qs::KP k;
    memset(&k, 0, sizeof k);
    k.E = c->num_envs; k.N = c->num_agents; k.I = L.num_drones; k.obs_dim = L.obs_dim;
    k.so_dim = self_obs_dim(c->obs_repr);
    k.neighbor = c->neighbor_obs;
    k.K = c->neighbor_obs == QS_NEIGHBOR_POS_VEL ? c->k_neighbors : 0;
    k.id0 = c->drone_id_offset;
    k.obs_repr = c->obs_repr; k.ep_len = c->ep_len; k.sim_steps = c->sim_steps; k.svd_every = c->svd_every;
    k.sense = c->sense_noise; k.downwash = c->use_downwash; k.collide = c->apply_collision_force;
    k.dt = c->dt; k.cdt = c->control_dt; k.mass = c->mass; k.inv_mass = (float)(1.0 / (double)c->mass);
    for (int i = 0; i < 3; ++i) {
        k.inertia[i] = c->inertia[i];
        k.inv_inertia[i] = (float)(1.0 / (double)c->inertia[i]);
        k.room_lo[i] = c->room_lo[i];
        k.room_hi[i] = c->room_hi[i];
        k.room_range[i] = c->room_hi[i] - c->room_lo[i];
        k.goal[i] = c->goal[i];
    }
    for (int j = 0; j < 4; ++j) {
        k.thrust_max[j] = c->thrust_max[j]; k.torque_max[j] = c->torque_max[j];
        k.pc0[j] = c->prop_cross[j][0]; k.pc1[j] = c->prop_cross[j][1]; k.pc2[j] = c->prop_cross[j][2];
        k.ccw[j] = c->prop_ccw[j];
    }
    k.tau_up = c->motor_tau_up; k.tau_down = c->motor_tau_down; k.lin = c->motor_linearity;
    k.arm = c->arm; k.grav = c->gravity; k.omega_max = c->omega_max; k.vel_damp = c->vel_damp;
    k.dq = c->damp_omega_quadratic; k.vxyz_max = c->vxyz_max;
    k.ou_mu = c->ou_mu; k.ou_theta = c->ou_theta; k.ou_sigma = c->ou_sigma;
    k.pos_std = c->pos_norm_std; k.pos_unif = c->pos_unif_range; k.vel_std = c->vel_norm_std;
    k.vel_unif = c->vel_unif_range; k.gyro = c->gyro_noise_density; k.quat_std = c->quat_norm_std;
    k.quat_unif = c->quat_unif_range;
    k.col_thr = c->collision_threshold; k.fall_thr = c->collision_falloff_threshold;
    k.prox_max = c->rew_quadcol_smooth_max;
    k.prox_ratio = c->collision_falloff_threshold > 0.f ? -c->rew_quadcol_smooth_max / c->collision_falloff_threshold : 0.f;
    k.rew_pos = c->rew_pos; k.rew_effort = c->rew_effort; k.rew_crash = c->rew_crash; k.rew_orient = c->rew_orient;
    k.rew_spin = c->rew_spin; k.quadcol = c->rew_quadcol_bin;
    k.spawn_box = c->spawn_box;
    return k;
}

extern "C" int qs_config_default(qs_config* c, int32_t num_envs, int32_t num_agents) {
    if (!c) return fail(QS_E_INVALID, "config is NULL");
    memset(c, 0, sizeof *c);
    c->abi_version = QS_ABI_VERSION;
    c->num_envs = num_envs;
    c->num_agents = num_agents;
    c->obs_repr = QS_OBS_XYZ_VXYZ_R_OMEGA;
    c->neighbor_obs = num_agents > 1 ? QS_NEIGHBOR_POS_VEL : QS_NEIGHBOR_NONE;
    c->k_neighbors = num_agents > 1 ? (num_agents - 1 < 6 ? num_agents - 1 : 6) : 0;
    c->ep_len = 1500;
    c->sim_steps = 2;
    c->svd_every = 100;
    c->sense_noise = 1;
    c->use_downwash = 0;
    c->apply_collision_force = 1;
    c->seed = 0;
    c->dt = 0.005f;
    c->control_dt = 0.01f;
    // Crazyflie (quad_models.py:1-42) through QuadLink (inertia.py:182-310), see quadswarm_amd/params.py
    const double mass = 0.028000000000000008;
    c->mass = (float)mass;
    c->inertia[0] = 1.3669232142857143e-05f; c->inertia[1] = 1.4356732142857143e-05f; c->inertia[2] = 2.656158333333334e-05f;
    const double tm = 9.81 * mass * 1.9 / 4.0;
    const float px[4] = {0.0325f, -0.0325f, -0.0325f, 0.0325f}, py[4] = {-0.0325f, -0.0325f, 0.0325f, 0.0325f};
    const float ccw[4] = {-1.f, 1.f, -1.f, 1.f};
    for (int k = 0; k < 4; ++k) {
        c->thrust_max[k] = (float)tm; c->torque_max[k] = (float)(0.006 * tm);
        c->prop_cross[k][0] = py[k]; c->prop_cross[k][1] = -px[k]; c->prop_cross[k][2] = 0.f; c->prop_ccw[k] = ccw[k];
    }
    c->motor_tau_up = c->motor_tau_down = (float)(4 * 0.005 / (0.15 + 1e-6));
    c->motor_linearity = 1.f;
    c->arm = 0.04596194077712559f; c->gravity = 9.81f; c->omega_max = 40.f; c->vel_damp = 0.f;
    c->damp_omega_quadratic = 0.f; c->vxyz_max = 3.f;
    c->room_lo[0] = -5.f; c->room_lo[1] = -5.f; c->room_lo[2] = 0.f;
    c->room_hi[0] = 5.f; c->room_hi[1] = 5.f; c->room_hi[2] = 10.f;
    c->ou_mu = 0.f; c->ou_theta = 0.15f; c->ou_sigma = 0.2f * 0.05f;
    c->pos_norm_std = 0.005f; c->vel_norm_std = 0.01f; c->gyro_noise_density = 0.000175f;
    c->collision_threshold = 2.f * c->arm; c->collision_falloff_threshold = 4.f * c->arm;
    c->rew_pos = 1.f; c->rew_effort = 0.05f; c->rew_crash = 1.f; c->rew_orient = 1.f; c->rew_spin = 0.1f;
    c->rew_quadcol_bin = 5.f; c->rew_quadcol_smooth_max = 10.f;
    c->spawn_box = 2.f; c->goal[0] = 0.f; c->goal[1] = 0.f; c->goal[2] = 2.f;
    return QS_OK;
}

extern "C" int qs_layout_query(const qs_config* c, qs_layout* out) {
    int rc = validate(c);
    if (rc) return rc;
    if (!out) return fail(QS_E_INVALID, "layout is NULL");
    *out = make_layout(c);
    return QS_OK;
}

static int npad_of(int n) {
    int p = 1;
    while (p < n) p <<= 1;
    return p;
}

extern "C" int qs_create(const qs_config* c, int dev, void* ws, qs_handle** out) {
    int rc = validate(c);
    if (rc) return rc;
    if (!out) return fail(QS_E_INVALID, "out handle is NULL");
    *out = nullptr;
    QS_HIP(hipSetDevice(dev));
    qs_handle* h = new (std::nothrow) qs_handle();
    if (!h) return fail(QS_E_NOMEM, "host allocation failed");
    h->cfg = *c;
    h->lay = make_layout(c);
    h->kp = make_kp(c, h->lay);
    h->device = dev;
    h->npad = npad_of(c->num_agents);
    if (ws) {
        if (((uintptr_t)ws & 255) != 0) { delete h; return fail(QS_E_INVALID, "workspace must be 256-byte aligned"); }
        h->ws = ws;
        h->owns_ws = false;
    } else {
        hipError_t e = hipMalloc(&h->ws, h->lay.total_bytes);
        if (e != hipSuccess) { delete h; return fail(QS_E_HIP, std::string("hipMalloc: ") + hipGetErrorString(e)); }
        h->owns_ws = true;
    }
    hipError_t e = hipMemset(h->ws, 0, h->lay.total_bytes);
    if (e == hipSuccess) e = hipMemcpy((char*)h->ws + h->lay.params, &h->kp, sizeof(qs::KP), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        if (h->owns_ws) (void)hipFree(h->ws);
        delete h;
        return fail(QS_E_HIP, std::string("workspace init: ") + hipGetErrorString(e));
    }
    *out = h;
    return QS_OK;
}

extern "C" int qs_destroy(qs_handle* h) {
    if (!h) return QS_OK;
    if (h->owns_ws && h->ws) {
        hipError_t e = hipFree(h->ws);
        delete h;
        if (e != hipSuccess) return fail(QS_E_HIP, std::string("hipFree: ") + hipGetErrorString(e));
        return QS_OK;
    }
    delete h;
    return QS_OK;
}

static qs::Bufs bufs_of(qs_handle* h) {
    char* w = (char*)h->ws;
    qs::Bufs b;
    b.st = (float*)(w + h->lay.state);
    b.ist = (int32_t*)(w + h->lay.istate);
    b.env = (int32_t*)(w + h->lay.env);
    b.stale = (float*)(w + h->lay.stale_vel);
    b.obs = (float*)(w + h->lay.obs);
    b.term = (float*)(w + h->lay.term_obs);
    b.rew = (float*)(w + h->lay.rew);
    b.done = (uint8_t*)(w + h->lay.done);
    b.act = nullptr;
    b.mask = nullptr;
    return b;
}

extern "C" int qs_buffers_get(qs_handle* h, qs_buffers* o) {
    if (!h || !o) return fail(QS_E_INVALID, "NULL argument");
    qs::Bufs b = bufs_of(h);
    o->state = b.st; o->istate = b.ist; o->env = b.env; o->stale_vel = b.stale;
    o->obs = b.obs; o->term_obs = b.term; o->rew = b.rew; o->done = b.done;
    return QS_OK;
}

static int launch(qs_handle* h, bool step, const float* act, const uint8_t* mask, hipStream_t s) {
    qs::Bufs b = bufs_of(h);
    b.act = act;
    b.mask = mask;
    const uint32_t seed = h->cfg.seed;
    const qs::KP* kpd = (const qs::KP*)((char*)h->ws + h->lay.params);
    const int epb = 64 / h->npad;
    const dim3 grid((unsigned)((h->kp.E + epb - 1) / epb)), block(64);
    const size_t shm = sizeof(float) * 64 * (size_t)h->kp.obs_dim + sizeof(float) * 64 * 8;  // obs tile + exchange
#define QS_LAUNCH(NP)                                                                                           \
    case NP:                                                                                                   \
        if (step) hipLaunchKernelGGL(qs::step_kernel<NP>, grid, block, shm, s, kpd, b, seed);                  \
        else hipLaunchKernelGGL(qs::reset_kernel<NP>, grid, block, shm, s, kpd, b, seed);                      \
        break;
    switch (h->npad) {
        QS_LAUNCH(1)
        QS_LAUNCH(2)
        QS_LAUNCH(4)
        QS_LAUNCH(8)
        QS_LAUNCH(16)
        QS_LAUNCH(32)
        default:
            return fail(QS_E_UNSUPPORTED, "num_agents not supported");
    }
#undef QS_LAUNCH
    QS_HIP(hipGetLastError());
    return QS_OK;
}

extern "C" int qs_reset(qs_handle* h, const uint8_t* d_mask, void* stream) {
    if (!h) return fail(QS_E_INVALID, "handle is NULL");
    QS_HIP(hipSetDevice(h->device));
    return launch(h, false, nullptr, d_mask, (hipStream_t)stream);
}

extern "C" int qs_step(qs_handle* h, const float* d_actions, void* stream) {
    if (!h || !d_actions) return fail(QS_E_INVALID, "NULL argument");
    if (((uintptr_t)d_actions & 15) != 0) return fail(QS_E_INVALID, "actions must be 16-byte aligned [I,4] fp32");
    QS_HIP(hipSetDevice(h->device));
    return launch(h, true, d_actions, nullptr, (hipStream_t)stream);
}

static float* param_slot(qs_handle* h, const char* key) {
    qs::KP& k = h->kp;
    struct { const char* n; float* p; } t[] = {
        {"rew_pos", &k.rew_pos}, {"rew_effort", &k.rew_effort}, {"rew_crash", &k.rew_crash},
        {"rew_orient", &k.rew_orient}, {"rew_spin", &k.rew_spin}, {"quadcol_bin", &k.quadcol},
        {"quadcol_bin_smooth_max", &k.prox_max}};
    for (auto& e : t)
        if (strcmp(e.n, key) == 0) return e.p;
    return nullptr;
}

static int upload_params(qs_handle* h) {
    QS_HIP(hipSetDevice(h->device));
    QS_HIP(hipDeviceSynchronize());   // launches in flight read the old block
    QS_HIP(hipMemcpy((char*)h->ws + h->lay.params, &h->kp, sizeof(qs::KP), hipMemcpyHostToDevice));
    return QS_OK;
}

// Parameters live in device memory (read by every launch), so a change also reaches launches that
// are replayed from a captured hipGraph.
extern "C" int qs_set_param(qs_handle* h, const char* key, double v) {
    if (!h || !key) return fail(QS_E_INVALID, "NULL argument");
    if (strcmp(key, "ep_len") == 0) { h->kp.ep_len = (int)v; h->cfg.ep_len = (int)v; return upload_params(h); }
    if (strcmp(key, "seed") == 0) { h->cfg.seed = (uint32_t)v; return QS_OK; }
    float* p = param_slot(h, key);
    if (!p) return fail(QS_E_INVALID, std::string("unknown param ") + key);
    *p = (float)v;
    if (strcmp(key, "quadcol_bin_smooth_max") == 0)
        h->kp.prox_ratio = h->kp.fall_thr > 0.f ? -h->kp.prox_max / h->kp.fall_thr : 0.f;
    return upload_params(h);
}

extern "C" int qs_get_param(qs_handle* h, const char* key, double* v) {
    if (!h || !key || !v) return fail(QS_E_INVALID, "NULL argument");
    if (strcmp(key, "ep_len") == 0) { *v = h->kp.ep_len; return QS_OK; }
    if (strcmp(key, "seed") == 0) { *v = h->cfg.seed; return QS_OK; }
    float* p = param_slot(h, key);
    if (!p) return fail(QS_E_INVALID, std::string("unknown param ") + key);
    *v = *p;
    return QS_OK;
}

// snapshot = the workspace from the state buffer up to (not including) the obs buffers; the env
// block holds tick + episode, i.e. the RNG counters, so a restored env replays the same draws
extern "C" size_t qs_state_bytes(qs_handle* h) {
    if (!h) return 0;
    return h->lay.obs - h->lay.state;
}

extern "C" int qs_get_state(qs_handle* h, void* dst, size_t bytes, void* stream) {
    if (!h || !dst) return fail(QS_E_INVALID, "NULL argument");
    if (bytes < qs_state_bytes(h)) return fail(QS_E_INVALID, "buffer too small");
    QS_HIP(hipSetDevice(h->device));
    QS_HIP(hipMemcpyAsync(dst, (char*)h->ws + h->lay.state, qs_state_bytes(h), hipMemcpyDeviceToHost,
                          (hipStream_t)stream));
    QS_HIP(hipStreamSynchronize((hipStream_t)stream));
    return QS_OK;
}

extern "C" int qs_set_state(qs_handle* h, const void* src, size_t bytes, void* stream) {
    if (!h || !src) return fail(QS_E_INVALID, "NULL argument");
    if (bytes < qs_state_bytes(h)) return fail(QS_E_INVALID, "buffer too small");
    QS_HIP(hipSetDevice(h->device));
    QS_HIP(hipMemcpyAsync((char*)h->ws + h->lay.state, src, qs_state_bytes(h), hipMemcpyHostToDevice,
                          (hipStream_t)stream));
    QS_HIP(hipStreamSynchronize((hipStream_t)stream));
    return QS_OK;
}
