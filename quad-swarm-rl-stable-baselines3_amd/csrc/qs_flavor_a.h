// qs_flavor_a.h -- flavor-A kernels: the env swarm_rl/sb_train.py trains on.
//
//   quadrotor_multi_rewards.QuadrotorEnvMulti.step   quadrotor_multi_rewards.py:630-991
//     8 x QuadrotorSingle._step                      quadrotor_single_rewards.py:418-452
//         Controller.update_vel_height_dir           Controller/Controller.py:76-101 (+ Position/Velocity/
//                                                    Acceleration/Attitude/Rate controllers, Mixer, Pid.py)
//         CustomPidControl.step + QuadrotorDynamics  quadrotor_control.py:90-94, quadrotor_dynamics.py:215-221
//     capture reward / dones                         quadrotor_multi_rewards.py:711-735, 882-988
//     perform_downwash per tick (use_downwash)       quadrotor_multi_rewards.py:810-815, aerodynamics/downwash.py
//     Scenario_dynamic_repulsive.step / reset        scenarios/dynamic_repulsive.py:37-74 (float-fixed)
//     any other quads_mode: create_scenario (:123)   the goal scenarios of qs_scen.h, step per tick (:848)
//     neighbour obs + camera model                   quadrotor_multi_rewards.py:238-476
//   SubprocVecEnvCustom worker reset on done         subproc_vec_env_custom.py:39-46 (reset_infos)
//
// Same execution model as flavor B (qs_flavor_b.h): one lane per drone, an env is an NPAD-lane
// segment of a 64-lane wave, one wave per workgroup.  The 8 controller+physics ticks of a step run in
// registers; an env that finishes mid-step (capture) idles for the remaining ticks, like the
// reference's `break`.  Cross-drone work per tick is one segment reduction (target repulsion) and
// two segment ballots (capture, done); neighbour features read an LDS exchange tile once per step.
#pragma once
#include "qs_common.h"
#include "qs_scen.h"

namespace qs {

constexpr float kPi = 3.14159265358979f;
constexpr float k2Pi = 6.28318530717959f;

struct Ctl {
    float pid[20];  // (last_error, integral) x {pos z, vel x y z, att x y z, rate x y z}
    float angle, angvel;
};

__device__ __forceinline__ void load_ctl(const KP& kp, const Bufs& b, int g, Ctl& c) {
    const float* s = b.st + g;
#pragma unroll
    for (int i = 0; i < 20; ++i) c.pid[i] = s[(QS_F_PID + i) * kp.I];
    c.angle = s[QS_F_ANGLE * kp.I];
    c.angvel = s[QS_F_ANGVEL * kp.I];
}

__device__ __forceinline__ void store_ctl(const KP& kp, const Bufs& b, int g, const Ctl& c) {
    float* s = b.st + g;
#pragma unroll
    for (int i = 0; i < 20; ++i) s[(QS_F_PID + i) * kp.I] = c.pid[i];
    s[QS_F_ANGLE * kp.I] = c.angle;
    s[QS_F_ANGVEL * kp.I] = c.angvel;
}

// sin(x) for 0 <= x < pi/2, odd Taylor series to x^11 (relative error < 1e-7 for small x, where the
// camera range r / sin(alpha/2) needs it)
__device__ __forceinline__ float sin_small(float x) {
    const float x2 = x * x;
    return x * (1.f + x2 * (-1.f / 6.f + x2 * (1.f / 120.f + x2 * (-1.f / 5040.f + x2 * (1.f / 362880.f + x2 * (-1.f / 39916800.f))))));
}

#ifndef QS_CAM_RCP
#define QS_CAM_RCP 1
#endif
#ifndef QS_CAM_SECTOR
#define QS_CAM_SECTOR 1
#endif
#ifndef QS_PID_MED3
#define QS_PID_MED3 1
#endif
#ifndef QS_A_DEAL_SENSE
#define QS_A_DEAL_SENSE 1
#endif
#ifndef QS_COL_FOLD
#define QS_COL_FOLD 1
#endif
#ifndef QS_ACT_FOLD
#define QS_ACT_FOLD 1
#endif

// (x + pi) % (2 pi) - pi with Python's modulo sign convention.  For r = x + pi in [-2 pi, 4 pi) -- every
// angle the step wraps -- fmodf(r, 2 pi) is r itself below 2 pi and r - 2 pi above (exact by Sterbenz), so
// the fast path gives fmodf's bits without its ~30-instruction loop; anything else (and NaN / inf) takes it.
// The common range as selects, the fmodf fallback as the only branch (rare, skipped by whole waves).
__device__ __forceinline__ float wrap_pi(float x) {
    const float r = x + kPi;
    float w = r >= k2Pi ? r - k2Pi : r;
    if (__builtin_expect(!(r >= -k2Pi && r < 2.f * k2Pi), 0)) w = fmodf(r, k2Pi);
    w = w < 0.f ? w + k2Pi : w;
    return w - kPi;
}

// u[k] = sub-lane (k % Q)'s v[k / Q]
template <int Q, int K = 0>
__device__ __forceinline__ void ctl_share(const float (&v)[4 / Q], float* u) {
    if constexpr (K < 4) {
        u[K] = qbc<Q, K % Q>(v[K / Q]);
        ctl_share<Q, K + 1>(v, u);
    }
}

// _pid_update_numba (Controller/Pid.py:6-26)
__device__ __forceinline__ float pid_update(const KP& kp, int k, float e, float* st) {
    const float diff = (e - st[0]) * kp.inv_dt;
    st[0] = e;
    float out = kp.pkp[k] * e + kp.pkd[k] * diff + kp.pki[k] * st[1];
    const float sat = kp.psat[k];
#if QS_PID_MED3
    // the clamp as one v_med3_f32 (the same value for every non-NaN out, -0 and +-inf included); NaN passes through
    // as in the reference's if / elif
    if (sat > 0.f) {
        const float c = __builtin_amdgcn_fmed3f(out, -sat, sat);
        out = out != out ? out : c;
    }
#else
    if (sat > 0.f) out = out >= sat ? sat : (out <= -sat ? -sat : out);
#endif
    const float aw = kp.paw[k];
    if (aw > 0.f && -aw < out && out < aw) st[1] += e * kp.dt;
    return out;
}

// Controller.update_vel_height_dir (Controller.py:76-101) -> Mixer output -> _step's reorder/arctan
// (quadrotor_single_rewards.py:436-437) -> CustomPidControl.step (quadrotor_control.py:90-94): the 4
// normalised thrust commands for QuadrotorDynamics.step.
// Q > 1: the drone's Q sub-lanes each take the atan of motors q, q + Q, ..., shared by DPP (bitwise the same)
template <int Q = 1>
__device__ __forceinline__ void controller(const KP& kp, const Drone& d, Ctl& c, float a0, float height, float* u,
                                           int q = 0) {
    c.angvel = a0;
    c.angle = wrap_pi(c.angle + a0 * kp.hrate);
    float sa, ca;
    sincos_hw(c.angle, &sa, &ca);
    // PositionController z (PositionController.py:62-77); x/y outputs are overwritten by the heading
    // velocity (:90) and their PID state never reaches an output, so they are not carried.
    const float vz = pid_update(kp, 0, height - d.pos[2], c.pid);
    const float vref[3] = {ca * kp.speed, sa * kp.speed, vz};
    float acc[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) acc[i] = pid_update(kp, 1 + i, vref[i] - d.vel[i], c.pid + 2 * (1 + i));
    // AccelerationController (AccelerationController.py:18-108), heading 0: the oblique projection of
    // (1,0,0) along z onto the plane normal to n is (1, 0, -n0/n2), i.e. x_des = (|n2|, 0, -n0 sgn n2)/|(n0,n2)|
    const float fd0 = acc[0] * kp.m_mass, fd1 = acc[1] * kp.m_mass, fd2 = acc[2] * kp.m_mass + kp.m_mass_g;
    const float ifn = rsqrtf(fd0 * fd0 + fd1 * fd1 + fd2 * fd2);
    const float n0 = fd0 * ifn, n1 = fd1 * ifn, n2 = fd2 * ifn;
    const float ixn = rsqrtf(n0 * n0 + n2 * n2);
    const float x0 = fabsf(n2) * ixn, x1 = 0.f, x2 = (n2 >= 0.f ? -n0 : n0) * ixn;
    float y0 = n1 * x2 - n2 * x1, y1 = n2 * x0 - n0 * x2, y2 = n0 * x1 - n1 * x0;
    const float iyn = rsqrtf(y0 * y0 + y1 * y1 + y2 * y2);
    y0 *= iyn; y1 *= iyn; y2 *= iyn;
    const float* R = d.rot;
    const float tf = fmaxf(fd0 * R[2] + fd1 * R[5] + fd2 * R[8], 0.f);
    // tf / kf4 as a product with the (constant-folded) reciprocal: ~1 ulp, no IEEE division in the tick loop
    const float thr = clampf((fsqrt(tf * frcp(kp.m_kf4)) - kp.m_min_rpm) * kp.m_inv_rpm, 0.f, 1.f);
    // AttitudeController (AttitudeController.py:60-82): e = vee(0.5 (Rd^T R - R^T Rd)); M = Rd^T R
    const float Rd0[3] = {x0, x1, x2}, Rd1[3] = {y0, y1, y2}, Rd2[3] = {n0, n1, n2};
    auto M = [&](const float* col, int j) { return col[0] * R[j] + col[1] * R[3 + j] + col[2] * R[6 + j]; };
    const float e0 = 0.5f * (M(Rd1, 2) - M(Rd2, 1));
    const float e1 = 0.5f * (M(Rd2, 0) - M(Rd0, 2));
    const float e2 = 0.5f * (M(Rd0, 1) - M(Rd1, 0));
    const float rate0 = pid_update(kp, 4, e0, c.pid + 8);
    const float rate1 = pid_update(kp, 5, e1, c.pid + 10);
    const float rate2 = pid_update(kp, 6, e2, c.pid + 12);
    // RateController (RateController.py:71-89)
    float cg[4];
    cg[0] = pid_update(kp, 7, rate0 - d.om[0], c.pid + 14) * kp.rate_scale;
    cg[1] = pid_update(kp, 8, rate1 - d.om[1], c.pid + 16) * kp.rate_scale;
    cg[2] = pid_update(kp, 9, rate2 - d.om[2], c.pid + 18) * kp.rate_scale;
    cg[3] = thr;
    // Mixer with desaturation (Mixer.py:70-111)
    const float* X = kp.mix;
    float m[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) m[i] = X[i * 4] * cg[0] + X[i * 4 + 1] * cg[1] + X[i * 4 + 2] * cg[2] + X[i * 4 + 3] * cg[3];
    const float mn = fminf(fminf(m[0], m[1]), fminf(m[2], m[3]));
    if (mn < 0.f) {
#pragma unroll
        for (int i = 0; i < 4; ++i) m[i] += -mn;
    }
    const float mx = fmaxf(fmaxf(m[0], m[1]), fmaxf(m[2], m[3]));
    if (mx > 1.f) {
        if (thr > 1e-2f) {
            const float isc = thr / ((m[0] + ((m[1] + m[2]) + m[3])) * 0.25f);
            cg[0] *= isc; cg[1] *= isc; cg[2] *= isc;
#pragma unroll
            for (int i = 0; i < 4; ++i)
                m[i] = X[i * 4] * cg[0] + X[i * 4 + 1] * cg[1] + X[i * 4 + 2] * cg[2] + X[i * 4 + 3] * cg[3];
        } else {
            const float im = 1.f / mx;
#pragma unroll
            for (int i = 0; i < 4; ++i) m[i] *= im;
        }
    }
    const float re[4] = {m[0], m[3], m[1], m[2]};
    if constexpr (Q == 1 || 4 % Q != 0) {
#pragma unroll
        for (int k = 0; k < 4; ++k) u[k] = 0.5f * (clampf(atanf(re[k] * 2.f - 1.f), -1.f, 1.f) + 1.f);
    } else {
        float v[4 / Q];
#pragma unroll
        for (int t = 0; t < 4 / Q; ++t) {
            float x = re[Q * t];
#pragma unroll
            for (int s = 1; s < Q; ++s)
                if (q == s) x = re[Q * t + s];
            v[t] = 0.5f * (clampf(atanf(x * 2.f - 1.f), -1.f, 1.f) + 1.f);
        }
        ctl_share<Q>(v, u);
    }
}

// (|p + v dt| - |p|) / dt without the fp32 cancellation: (2 p.v + dt |v|^2) / (|p + v dt| + |p|)
__device__ __forceinline__ float norm_rate(float p0, float p1, float v0, float v1, float dt, float pn) {
    const float q0 = p0 + v0 * dt, q1 = p1 + v1 * dt;
    const float den = fsqrt(q0 * q0 + q1 * q1) + pn;
    const float num = 2.f * (p0 * v0 + p1 * v1) + dt * (v0 * v0 + v1 * v1);
    return den > 0.f ? num * frcp(den) : 0.f;   // a reciprocal product (~1 ulp), no IEEE division per neighbour
}

// simulate_camera_measurement_vect (get_state.py:128-176 == quadrotor_multi_rewards.py:275-324) for one
// target; n1, n2: pixel noise.  circle_intersection_vect(c, r, c/2, |c|/2) in closed form: the chord
// distance a = r^2/|c|, midpoint c (1 - r^2/|c|^2), perpendicular (c1, -c0)/|c|.
__device__ __forceinline__ void camera(const KP& kp, float rx, float ry, float ga, float n1, float n2, float& dist, float& ang) {
    float s, c;
    sincos_hw(-ga, &s, &c);
    const float rp0 = c * rx - s * ry, rp1 = s * rx + c * ry;
#if QS_CAM_SECTOR
    // get_camera_angle (get_state.py:128-137) without the atan2: the camera whose axis k seg is nearest the
    // bearing is the one with the largest projection rp . (cos k seg, sin k seg) (the first on an exact tie; the
    // reference's round() differs only on the sector boundaries, where the features are ill-conditioned anyway).
    // The axes are computed once on the host (KP cam_cos / cam_sin): constants in the specialised kernels, loads
    // in the generic ones (no libm call in the candidate loop).
    const float seg = k2Pi / (float)kp.n_cam;
    float best = rp0, ca = 1.f, sa = 0.f, cam = 0.f;
    for (int k = 1; k < kp.n_cam; ++k) {
        const float ck = kp.cam_cos[k], sk = kp.cam_sin[k];
        const float pk = rp0 * ck + rp1 * sk;
        const bool gt = pk > best;
        best = gt ? pk : best;
        ca = gt ? ck : ca;
        sa = gt ? sk : sa;
        cam = gt ? (float)k * seg : cam;
    }
    s = -sa;   // sincos(-cam)
    c = ca;
#else
    float m = atan2f(rp1, rp0);   // fmodf(m, 2 pi) is m itself: |atan2| <= pi
    if (m < 0.f) m += k2Pi;
    const float seg = k2Pi / (float)kp.n_cam;
    const int ci = ((int)rintf(m / seg)) % kp.n_cam;
    const float cam = (float)ci * seg;
    sincos_hw(-cam, &s, &c);
#endif
    const float c0 = c * rp0 - s * rp1, c1 = s * rp0 + c * rp1;
    const float cn2 = c0 * c0 + c1 * c1, cn = fsqrt(cn2);
    const float r = kp.cam_r, r2 = r * r;
    const float pxs = kp.cam_w / (kp.cam_res * kp.cam_f);  // pixel -> tan(angle)
#if QS_CAM_RCP
    // the quotients as products with hardware reciprocals (~1 ulp each, like target_step): 1 / |c| once for
    // a, mf and the perpendicular; the camera index (m / seg above) keeps its IEEE division, since a rounding
    // flip there would move the segment.  0 / inf / NaN cases as the divisions give them (x * rcp(0) = +-inf,
    // 0 * rcp(0) = NaN)
    const float icn = frcp(cn);
    const float a = r2 * icn;
    // v_sqrt_f32 (~1 ulp) instead of the correctly-rounded sqrtf expansion; NaN when the target is inside the marker
    const float h = fsqrt(r2 - a * a);
    const float mf = 1.f - r2 * (icn * icn);
    const float mid0 = c0 * mf, mid1 = c1 * mf;
    const float pe0 = c1 * icn, pe1 = -c0 * icn;
    const float x10 = mid0 + h * pe0, x11 = mid1 + h * pe1;
    const float x20 = mid0 - h * pe0, x21 = mid1 - h * pe1;
    const float at1 = atanf(x11 * frcp(x10) + n1 * pxs), at2 = atanf(x21 * frcp(x20) + n2 * pxs);
    const float alpha = fabsf(at1 - at2);
    const float l = r * frcp(sin_small(0.5f * alpha));
#else
    const float a = r2 / cn;
    const float h = sqrtf(r2 - a * a);                   // NaN when the target is inside the marker
    const float mf = 1.f - r2 / cn2;
    const float mid0 = c0 * mf, mid1 = c1 * mf;
    const float pe0 = c1 / cn, pe1 = -c0 / cn;
    const float x10 = mid0 + h * pe0, x11 = mid1 + h * pe1;
    const float x20 = mid0 - h * pe0, x21 = mid1 - h * pe1;
    const float at1 = atanf(x11 / x10 + n1 * pxs), at2 = atanf(x21 / x20 + n2 * pxs);
    const float alpha = fabsf(at1 - at2);
    const float l = r / sin_small(0.5f * alpha);
#endif
    const float ar = wrap_pi(0.5f * (at1 + at2) + cam);
    dist = (l != l) ? 0.f : l;
    ang = (ar != ar) ? 0.f : ar;
}

// pos / vel sensor noise (sensor_noise.py:234-261, draws 0-5 of the 27; the rest do not reach a
// flavor-A observation)
// zpre: the 8 normals already drawn (the step kernel deals the two blocks over the drone's sub-lanes), or null
__device__ __forceinline__ void noisy_pos_vel(const KP& kp, const Drone& d, const Rng& rng, uint32_t gid,
                                              uint32_t st, float* np_, float* nv, const float* zpre = nullptr) {
#pragma unroll
    for (int i = 0; i < 3; ++i) { np_[i] = d.pos[i]; nv[i] = d.vel[i]; }
    if (!kp.sense) return;
    float z[8];
    if (zpre) {
#pragma unroll
        for (int i = 0; i < 8; ++i) z[i] = zpre[i];
    } else {
        normals4(rng, gid, st, 0, z);
        normals4(rng, gid, st, 1, z + 4);
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        np_[i] += kp.pos_std * z[i];
        nv[i] += kp.vel_std * z[3 + i];
    }
    if (kp.pos_unif != 0.f || kp.vel_unif != 0.f) {
        float u[8];
        uniforms4(rng, gid, st, 0, u);
        uniforms4(rng, gid, st, 1, u + 4);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            np_[i] += -kp.pos_unif + 2.f * kp.pos_unif * u[i];
            nv[i] += -kp.vel_unif + 2.f * kp.vel_unif * u[3 + i];
        }
    }
}

// flavor-A self observation (get_state.py:7-223)
__device__ __forceinline__ void self_obs_a(const KP& kp, const Drone& d, const Ctl& c, float gx, float gy, const Rng& rng,
                           uint32_t gid, uint32_t st_sensor, uint32_t st_cam, float* out, const float* zsense = nullptr) {
    float np_[3], nv[3];
    noisy_pos_vel(kp, d, rng, gid, st_sensor, np_, nv, zsense);
    const float dt = kp.dt;
    const float rp0 = gx - np_[0], rp1 = gy - np_[1];
    const float rd = fsqrt(rp0 * rp0 + rp1 * rp1);
    const float drd = norm_rate(rp0, rp1, nv[0], nv[1], dt, rd);
    const float ra = wrap_pi(atan2f(rp1, rp0) - c.angle);
    const float av = c.angvel, pr = av * ra;
    const float adot = -(pr > 0.f ? 1.f : (pr < 0.f ? -1.f : 0.f)) * fabsf(av);
    if (kp.obs_repr == QS_OBS_AW_AWDOT_DIST_DISTDOT_ANGLE_ANGLEDOT) {
        out[0] = c.angle; out[1] = av; out[2] = rd; out[3] = drd; out[4] = ra; out[5] = adot;
        return;
    }
    const float cd = fsqrt(np_[0] * np_[0] + np_[1] * np_[1]);
    out[0] = cd;
    out[1] = norm_rate(np_[0], np_[1], nv[0], nv[1], dt, cd);
    out[3] = drd;
    if (kp.obs_repr == QS_OBS_CDIST_CDISTDOT_DIST_DISTDOT_ANGLE_ANGLEDOT) {
        out[2] = rd; out[4] = ra; out[5] = adot;
    } else if (kp.obs_repr == QS_OBS_CDIST_CDISTDOT_DIST_DISTDOT_SANGLE_ANGLEDOT) {
        float s, co;
        sincos_hw(ra, &s, &co);
        out[2] = rd; out[4] = co; out[5] = s; out[6] = adot;
    } else {
        float n1 = 0.f, n2 = 0.f;
        if (kp.cam_px != 0.f) {
            float z[4];
            normals4(rng, gid, st_cam, 0, z);
            n1 = kp.cam_px * z[0];
            n2 = kp.cam_px * z[1];
        }
        float nd, na, s, co;
        camera(kp, rp0, rp1, c.angle, n1, n2, nd, na);
        sincos_hw(na, &s, &co);
        out[2] = clampf(nd, 0.f, 10.f); out[4] = co; out[5] = s; out[6] = adot;
    }
}

// exchange tile: lane l holds {pos, heading} at xch[2l] and {vel, 0} at xch[2l+1]
__device__ __forceinline__ void xch_put_a(float4* xch, int lane, const float* P, float H, const float* V) {
    xch[2 * lane] = make_float4(P[0], P[1], P[2], H);
    xch[2 * lane + 1] = make_float4(V[0], V[1], V[2], 0.f);
}

// get_rel_pos_vel_item for the pair (i = this lane, j): emits the features in the reference's order
// to sink(slot, value) (no private array: slots are runtime, the sink accumulates or writes LDS)
template <class Sink>
__device__ __forceinline__ void rel_features(const KP& kp, const float4& pj, const float4& vj, const float* P, float H,
                                             float aw, const float* V, const Rng& rng, uint32_t gid, uint32_t st,
                                             Sink&& sink) {
    const int m = kp.nfeat;
    const float r0 = pj.x - P[0], r1 = pj.y - P[1], r2 = pj.z - P[2];
    int n = 0;
    float na = 0.f;
    if (m & QS_NF_DIST) sink(n++, fsqrt(r0 * r0 + r1 * r1 + r2 * r2));
    if (m & QS_NF_NDIST) {
        float n1 = 0.f, n2 = 0.f;
        if (kp.cam_px != 0.f) {
            float z[4];
            normals4(rng, gid, st, 0, z);
            n1 = kp.cam_px * z[0];
            n2 = kp.cam_px * z[1];
        }
        float nd;
        camera(kp, r0, r1, aw, n1, n2, nd, na);
        sink(n++, clampf(nd, 0.f, 10.f));
    }
    if (m & (QS_NF_ANGLE | QS_NF_SANGLE)) {
        // atan2 of the 3-D-normalised vector (:365-367); undefined (NaN) for coincident drones
        const float pn = fsqrt(r0 * r0 + r1 * r1 + r2 * r2);
        const float ra = pn > 0.f ? wrap_pi(atan2f(r1, r0) - aw) : __builtin_nanf("");
        if (m & QS_NF_ANGLE) sink(n++, ra);
        if (m & QS_NF_SANGLE) { float s, c; sincos_hw(ra, &s, &c); sink(n++, c); sink(n++, s); }
    }
    if (m & QS_NF_NSANGLE) { float s, c; sincos_hw(na, &s, &c); sink(n++, c); sink(n++, s); }
    if (m & (QS_NF_HEADING | QS_NF_SHEADING)) {
        const float rh = wrap_pi(pj.w - H);
        if (m & QS_NF_HEADING) sink(n++, rh);
        if (m & QS_NF_SHEADING) { float s, c; sincos_hw(rh, &s, &c); sink(n++, c); sink(n++, s); }
    }
    if (m & (QS_NF_NPOS | QS_NF_POS)) { sink(n++, r0); sink(n++, r1); sink(n++, r2); }
    if (m & QS_NF_VEL) { sink(n++, vj.x - V[0]); sink(n++, vj.y - V[1]); sink(n++, vj.z - V[2]); }
}

// neighborhood_indices (:445-476) + extend_obs_space clip (:422-443).  k < N-1: selection by the norm
// of the feature vector (clamped at 0.01, stable, NaN last) with its own camera noise, then the
// selected pairs' features again with the obs-pass noise (the reference calls the camera twice).
// Q > 1: the drone's sub-lane q writes the neighbours j with j % Q == q (same draws, same slots).
template <int NPAD, int Q = 1>
__device__ __forceinline__ void neighbor_obs_a(const KP& kp, const float4* xch, int base, int di, const float* P, float H, float aw,
                               const float* V, const Rng& rng, uint32_t gid, bool reset, bool write, float* out,
                               int q = 0) {
    const bool sorted = kp.K < kp.N - 1;
    const uint32_t st_obs = reset ? S_RESET_CAM : S_CAM, st_sel = reset ? S_RESET_CAM_SEL : S_CAM_SEL;
    const int F = kp.nfd;
    float key[NPAD];
    if (sorted) {
#pragma unroll
        for (int j = 0; j < NPAD; ++j) {
            const bool valid = (j != di) && (j < kp.N);
            float s = 0.f;
            rel_features(kp, xch[2 * (base + j)], xch[2 * (base + j) + 1], P, H, aw, V, rng, gid,
                         st_sel | ((uint32_t)j << 8), [&](int, float v) { s += v * v; });
            key[j] = valid ? ((s != s) ? 3.0e38f : fmaxf(s, 1e-4f)) : __builtin_inff();
        }
    }
    if (!write) return;
    if constexpr (Q > 1) {
        if (!sorted) {   // every neighbour in index order: sub-lane q takes j = q, q + Q, ... (the same code path)
#pragma unroll
            for (int t = 0; t < (NPAD + Q - 1) / Q; ++t) {
                const int j = q + Q * t;
                const int rank = j < di ? j : j - 1;
                if (j != di && j < kp.N && rank < kp.K) {
                    float* o = out + kp.so_dim + rank * F;
                    rel_features(kp, xch[2 * (base + j)], xch[2 * (base + j) + 1], P, H, aw, V, rng, gid,
                                 st_obs | ((uint32_t)j << 8),
                                 [&](int k, float v) { o[k] = clampf(v, kp.nclip_lo[k], kp.nclip_hi[k]); });
                }
            }
            return;
        }
    }
#pragma unroll
    for (int j = 0; j < NPAD; ++j) {
        const bool valid = (j != di) && (j < kp.N);
        int rank;
        if (sorted) {
            rank = 0;
#pragma unroll
            for (int m = 0; m < NPAD; ++m) rank += (key[m] < key[j]) || (m < j && key[m] == key[j]);
        } else {
            rank = j < di ? j : j - 1;
        }
        if (valid && rank < kp.K && (Q == 1 || j % Q == q)) {
            float* o = out + kp.so_dim + rank * F;
            rel_features(kp, xch[2 * (base + j)], xch[2 * (base + j) + 1], P, H, aw, V, rng, gid,
                         st_obs | ((uint32_t)j << 8),
                         [&](int q, float v) { o[q] = clampf(v, kp.nclip_lo[q], kp.nclip_hi[q]); });
        }
    }
}

// neighbor_obs_a for the envs of more than 64 drones (k < N - 1 always selects there), without the NPAD-entry key
// array: sub-lane q evaluates the candidates j = q, q + Q, ... once each (camera with the selection noise) and keeps
// the k smallest (key, j) in a sorted register list by insertion; the Q lists are merged over DPP, so every
// sub-lane holds the env's k nearest in the order the rank formula of neighbor_obs_a gives (key, then index).
// Sub-lane q then writes slots q, q + Q, ... with the obs-pass noise.  k <= QS_A_KMAX (qs_step.hip validate).
#ifndef QS_A_KMAX
#define QS_A_KMAX 16
#endif
template <int NPAD, int Q = 1>
__device__ __forceinline__ void neighbor_obs_wide(const KP& kp, const float4* xch, int base, int di, const float* P, float H,
                                                  float aw, const float* V, const Rng& rng, uint32_t gid, bool reset,
                                                  bool write, float* out, int q = 0) {
    constexpr int KM = QS_A_KMAX;
    const uint32_t st_obs = reset ? S_RESET_CAM : S_CAM, st_sel = reset ? S_RESET_CAM_SEL : S_CAM_SEL;
    const int F = kp.nfd;
    float lk[KM];
    int lj[KM];
#pragma unroll
    for (int s = 0; s < KM; ++s) { lk[s] = __builtin_inff(); lj[s] = NPAD; }
    auto insert = [&](float ck, int cj) {
#pragma unroll
        for (int s = 0; s < KM; ++s) {
            if (s < kp.K) {   // a constant in specialised builds
                const bool lt = ck < lk[s] || (ck == lk[s] && cj < lj[s]);
                const float tk = lk[s];
                const int tj = lj[s];
                lk[s] = lt ? ck : tk;
                lj[s] = lt ? cj : tj;
                ck = lt ? tk : ck;
                cj = lt ? tj : cj;
            }
        }
    };
#pragma unroll 1
    for (int t = 0; t < NPAD / Q; ++t) {
        const int j = q + Q * t;
        const bool valid = (j != di) && (j < kp.N);
        float sq = 0.f;
        rel_features(kp, xch[2 * (base + j)], xch[2 * (base + j) + 1], P, H, aw, V, rng, gid, st_sel | ((uint32_t)j << 8),
                     [&](int, float v) { sq += v * v; });
        insert(valid ? ((sq != sq) ? 3.0e38f : fmaxf(sq, 1e-4f)) : __builtin_inff(), j);
    }
    if constexpr (Q == 2) {   // the pair's lists: each the k smallest of its half, merged into the union's k smallest
        float pk[KM];
        int pj[KM];
#pragma unroll
        for (int s = 0; s < KM; ++s) {
            pk[s] = dpp_f<quad_perm(1, 0, 3, 2)>(lk[s]);
            pj[s] = dpp_i<quad_perm(1, 0, 3, 2)>(lj[s]);
        }
#pragma unroll
        for (int s = 0; s < KM; ++s)
            if (s < kp.K) insert(pk[s], pj[s]);
    } else {
        static_assert(Q == 1, "one or two sub-lanes per drone");
    }
    if (!write) return;
#pragma unroll 1
    for (int t = 0; t * Q < kp.K; ++t) {
        const int slot = q + Q * t;
        int j = lj[0];
#pragma unroll
        for (int s = 1; s < KM; ++s) j = slot == s ? lj[s] : j;
        if (slot < kp.K && j < kp.N) {
            float* o = out + kp.so_dim + slot * F;
            rel_features(kp, xch[2 * (base + j)], xch[2 * (base + j) + 1], P, H, aw, V, rng, gid, st_obs | ((uint32_t)j << 8),
                         [&](int k, float v) { o[k] = clampf(v, kp.nclip_lo[k], kp.nclip_hi[k]); });
        }
    }
}

// segment (= env) helpers over the LPE = NPAD * Q lanes of an env (Q sub-lanes per drone)
template <int LPE>
__device__ __forceinline__ bool seg_any(bool x, int base) {
    const uint64_t gm = (LPE == 64) ? ~0ull : ((1ull << LPE) - 1ull);
    return ((__ballot(x) >> base) & gm) != 0ull;
}
// butterfly over the drones (lane distance Q .. LPE/2): every lane ends with the same bits, and the
// summation tree is the one-lane-per-drone tree whatever Q is
template <int NPAD, int Q = 1>
__device__ __forceinline__ float seg_sum(float v) {
    if constexpr (NPAD * Q == 16) {
        // the env is one 16-lane DPP row: the same tree by DPP instead of LDS permutes.  At lane distance
        // m the partner is any lane of the other half of the 2m-lane group (l ^ 1, l ^ 2 by quad_perm; 7 - l
        // by row_half_mirror; 15 - l by row_mirror); every lane of a group holds the same bits, and each add
        // is commutative, so every lane ends with the bits of the xor butterfly below
        if constexpr (Q <= 1) v += dpp_f<quad_perm(1, 0, 3, 2)>(v);
        if constexpr (Q <= 2) v += dpp_f<quad_perm(2, 3, 0, 1)>(v);
        if constexpr (Q <= 4) v += dpp_f<0x141>(v);   // row_half_mirror
        v += dpp_f<0x140>(v);                         // row_mirror
        return v;
    }
#pragma unroll
    for (int m = Q; m < NPAD * Q; m <<= 1) v += __shfl_xor(v, m);
    return v;
}

// Env collectives of flavor A.  An env inside one wave: segment ballots and the butterfly above.  An env that
// spans the workgroup's NW waves (WIDE: 128-drone envs): the drone ballots of EnvColl (qs_common.h) and float
// sums as a butterfly over each wave's drones whose NW partials meet in LDS and are added in wave order on every
// lane (the same bits everywhere; two alternating slots, so one barrier per collective).  Every lane of the
// workgroup makes the same calls.  Counts take x && q == 0 (one bit per drone in either form).
template <int NPAD, int Q>
struct EnvA {
    static constexpr int LPE = NPAD * Q;
    static constexpr bool WIDE = LPE > 64;
    static constexpr int NW = WIDE ? LPE / 64 : 1;
    EnvColl<WIDE, (NPAD > 64), Q, NW> ec;
    float* fscr;   // WIDE: 4 NW floats
    int fslot;
    __device__ __forceinline__ EnvA(int base, uint64_t* bscr, float* fs) : fscr(fs), fslot(0) {
        ec.lbase = base;
        ec.lmask = (LPE >= 64) ? ~0ull : ((1ull << LPE) - 1ull);
        ec.scr = bscr;
        ec.slot = 0;
    }
    __device__ __forceinline__ bool any(bool x) { return ec.any(x); }
    __device__ __forceinline__ int count(bool x) { return ec.count(x); }
    __device__ __forceinline__ bool wany(bool x) { return ec.wany(x); }
    __device__ __forceinline__ void sum2(float& a, float& b) {
        if constexpr (!WIDE) {
            a = seg_sum<NPAD, Q>(a);
            b = seg_sum<NPAD, Q>(b);
        } else {
#pragma unroll
            for (int m = Q; m < 64; m <<= 1) {
                a += __shfl_xor(a, m);
                b += __shfl_xor(b, m);
            }
            float* sc = fscr + 2 * NW * fslot;
            fslot ^= 1;
            const int w = threadIdx.x >> 6;
            if ((threadIdx.x & 63) == 0) {
                sc[w] = a;
                sc[NW + w] = b;
            }
            lds_sync();
            a = sc[0];
            b = sc[NW];
#pragma unroll
            for (int k = 1; k < NW; ++k) {
                a += sc[k];
                b += sc[NW + k];
            }
        }
    }
};

// Scenario_dynamic_repulsive.step (dynamic_repulsive.py:37-62): target flees the chasers (1/d each)
// and the arena edge, speed <= v_max.  Every lane of the env computes the same update.
template <class Env>
__device__ __forceinline__ void target_step(const KP& kp, float& tx, float& ty, const float* pos, bool contrib, Env& ev) {
    // the quotients as products with hardware reciprocals (~1 ulp; five IEEE divisions per tick otherwise)
    const float r0 = tx - pos[0], r1 = ty - pos[1];
    const float id2 = frcp(r0 * r0 + r1 * r1);
    float fx = contrib ? r0 * id2 : 0.f, fy = contrib ? r1 * id2 : 0.f;
    ev.sum2(fx, fy);
    const float de = fsqrt(tx * tx + ty * ty);
    const float iden = frcp(de * fmaxf(kp.arena - de, 0.1f));
    const float vx = fx - tx * iden, vy = fy - ty * iden;
    const float vs = fsqrt(vx * vx + vy * vy);
    const float sc = fminf(vs, kp.tgt_vmax) * frcp(vs) * kp.tgt_dt;
    tx = tx + vx * sc;
    ty = ty + vy * sc;
}

// QuadrotorEnvMulti.reset (quadrotor_multi_rewards.py:541-627) for the lanes of one env, including
// Scenario_dynamic_repulsive.reset (dynamic_repulsive.py:64-74, its step() sees the pre-reset chaser
// positions) and QuadrotorSingle._reset (quadrotor_single_rewards.py:480-549).  All lanes of the
// segment must call it (the target update is a segment reduction); `sel` lanes take the new state.
template <class Env>
__device__ __forceinline__ void reset_env_a(const KP& kp, Drone& d, Ctl& c, float& tx, float& ty, bool has_pos, bool active,
                            bool sel, const Rng& rng, uint32_t gid, uint32_t genv, Env& ev) {
    float ru[4], ue[4];
    uniforms4(rng, gid, S_RESET_A, 0, ru);
    if (kp.scenario == QS_SCEN_DYNAMIC_REPULSIVE) {
        uniforms4(rng, genv, S_SCEN, 0, ue);
        const float a = ue[1] - 0.5f, b = ue[2] - 0.5f, in = rsqrtf(a * a + b * b), tr = ue[3] * 3.f + 2.f;
        float ntx = a * in * tr, nty = b * in * tr;
        target_step(kp, ntx, nty, d.pos, active && has_pos, ev);
        if (sel) {
            tx = ntx;
            ty = nty;
            const float sa = ru[0] - 0.5f, sb = ru[1] - 0.5f, isn = rsqrtf(sa * sa + sb * sb), rad = ue[0] * 0.5f;
            d.goal[0] = tx; d.goal[1] = ty; d.goal[2] = fmaxf(kp.tgt_z, 0.25f);
            d.pos[0] = sa * isn * rad;
            d.pos[1] = sb * isn * rad;
        }
    } else if (sel) {   // static_same_goal, or a goal scenario (goal from scen_reset_a): spawn at the goal
        if (kp.scen_b < 0) { d.goal[0] = kp.goal[0]; d.goal[1] = kp.goal[1]; d.goal[2] = kp.goal[2]; }
        d.pos[0] = d.goal[0];
        d.pos[1] = d.goal[1];
    }
    if (!sel) return;
    d.pos[2] = fmaxf(d.goal[2], 0.75f);
    c.angle = (ru[2] - 0.5f) * k2Pi;
    {   // randyaw (quad_utils.py:228-230)
        float sy, cy;
        sincos_hw(-kPi + k2Pi * uniform1(rng, gid, S_RESET_YAW, 0), &sy, &cy);
        d.rot[0] = cy; d.rot[1] = -sy; d.rot[2] = 0.f;
        d.rot[3] = sy; d.rot[4] = cy; d.rot[5] = 0.f;
        d.rot[6] = 0.f; d.rot[7] = 0.f; d.rot[8] = 1.f;
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) { d.vel[i] = 0.f; d.om[i] = 0.f; }
#pragma unroll
    for (int k = 0; k < 4; ++k) { d.rd[k] = 0.f; d.cd[k] = 0.f; }
    d.flags = 0;
    d.prev = 0;   // prev_drone_collisions = [] (:606)
}

// drone-drone collision row of this lane's drone (calculate_collision_matrix, collisions/quadrotors.py:62-91)
// when the env is one 16-lane DPP row (8 drones x 2 sub-lanes): the row rotated by Q k lanes brings drone
// di + k (mod 8) -- its position and its index -- to this lane, no LDS round trip.  Squared distances
// against the squared threshold (the same order as |r| <= thr up to the last bit).
template <int Q, int K>
__device__ __forceinline__ void col_row16(const KP& kp, const Drone& d, int di, float thr2, uint32_t& cur) {
    if constexpr (K * Q < 16) {
        constexpr int C = 0x120 + K * Q;   // DPP row_ror:K*Q
        const float dx = d.pos[0] - dpp_f<C>(d.pos[0]), dy = d.pos[1] - dpp_f<C>(d.pos[1]);
        const float dz = d.pos[2] - dpp_f<C>(d.pos[2]);
        const int j = dpp_i<C>(di);
        // non-short-circuit: a select, not a branch per partner
        const bool hit = (j < kp.N) & (dx * dx + dy * dy + dz * dz <= thr2);
        cur |= hit ? (1u << j) : 0u;   // j < 16: the row's low word
        col_row16<Q, K + 1>(kp, d, di, thr2, cur);
    }
}

// The same row with the partners dealt over the drone's 2 sub-lanes: a rotation by 4k + 1 lanes brings drone
// di + 2k (its sub-lane 1) to sub-lane 0 and drone di + 2k + 1 (its sub-lane 0) to sub-lane 1, so 4
// rotations cover the 7 partners (and the drone itself once, skipped); the two halves are OR-ed by DPP.
template <int K>
__device__ __forceinline__ void col_row16_q2(const KP& kp, const Drone& d, int di, float thr2, uint32_t& cur) {
    if constexpr (K < 4) {
        constexpr int C = 0x120 + 4 * K + 1;   // DPP row_ror:4K+1
        const float dx = d.pos[0] - dpp_f<C>(d.pos[0]), dy = d.pos[1] - dpp_f<C>(d.pos[1]);
        const float dz = d.pos[2] - dpp_f<C>(d.pos[2]);
        const int j = dpp_i<C>(di);
        // only the K = 0 rotation can bring the drone itself (its own other sub-lane); with 8 drones every slot of the
        // row is a drone (constants in the specialised kernels: the two tests fold away)
        const bool self_ok = (QS_COL_FOLD && K != 0) || j != di;
        const bool in_env = (QS_COL_FOLD && kp.N == 8) || j < kp.N;
        const bool hit = self_ok & in_env & (dx * dx + dy * dy + dz * dz <= thr2);   // a select, not a branch
        cur |= hit ? (1u << j) : 0u;   // j < 8: the row's low word
        col_row16_q2<K + 1>(kp, d, di, thr2, cur);
    }
}

// scenario.reset() of the selected envs for the goal scenarios (:560, spawn_points None -> spawn at the
// goal, :569-573): the env's lead lane fills the LDS goal table (draw key = the env's drone 0, stream
// S_SCN_RESET) and stores the scenario state; every selected drone takes its goal.  Whole wave.
template <int NPAD>
__device__ __forceinline__ void scen_reset_a(const KP& kp, const Bufs& b, float* stab, int env, int di, bool lead_sel,
                                             bool sel, const Rng& rng, uint32_t genv, Drone& d) {
    if (lead_sel) {
        Scen sc;
        SDraw sd = sdraw(rng, genv, S_SCN_RESET);
        scen_reset(kp, sc, sd, stab, stab + 4 * (NPAD + 4));
        scen_store(kp, b, env, sc);
    }
    lds_sync();
    if (sel)
        for (int k = 0; k < 3; ++k) d.goal[k] = stab[4 * di + k];
    lds_sync();
}

// Step geometry of flavor A: Q sub-lanes per drone (QS_QA, 2 by default; 64 / NPAD when an env would
// not fit a wave).  4096 x 8 drones are then 1024 waves (one per SIMD) instead of 512.  The tick
// chain (controller, physics) is replicated on the sub-lanes; the divisible work is dealt over them:
// the per-tick OU blocks (sub-lane q draws tick t + q's block, DPP broadcast) and the neighbour
// features (neighbour j on sub-lane j % Q).  Reductions over the env keep the one-lane-per-drone tree.
#ifndef QS_QA
#define QS_QA 2
#endif
// tick (t + k)'s OU normals from sub-lane k: k = 0 -> z, k >= 1 -> zn[k - 1]
template <int Q, int K = 0>
__device__ __forceinline__ void qbc_ticks(const float (&zr)[4], float (&z)[4], float (&zn)[Q > 1 ? Q - 1 : 1][4]) {
    if constexpr (K < Q) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float v = qbc<Q, K>(zr[k]);
            if constexpr (K == 0) z[k] = v;
            else zn[K - 1][k] = v;
        }
        qbc_ticks<Q, K + 1>(zr, z, zn);
    }
}
template <int NPAD>
struct StepGeoA {
    // 128-drone envs: QS_QW sub-lanes, the env is a workgroup of 4 waves (one per SIMD at 256 envs)
    static constexpr int Q = NPAD * QS_QA <= 64 ? QS_QA : (NPAD > 64 ? QS_QW : 64 / NPAD);
    static constexpr int LPE = NPAD * Q;        // lanes per env
    static constexpr int WGS = LPE > 64 ? LPE : 64;   // threads per workgroup: one wave, or the env's waves
    static constexpr int EPB = WGS / LPE;       // envs per workgroup
    static constexpr int SLOTS = EPB * NPAD;    // drone slots (LDS rows) per workgroup
    static constexpr bool WIDE = LPE > 64;      // the env spans the workgroup's waves
};
// the explicit reset kernel: one lane per drone
template <int NPAD>
struct ResetGeoA {
    static constexpr int WGS = NPAD > 64 ? NPAD : 64;
    static constexpr int EPB = WGS / NPAD;
    static constexpr int SLOTS = EPB * NPAD;
};
// LDS words after the exchange tile (64 words before the scenario tables, qs_scen.h scen_tab): the env-finished
// flags (one per env of the workgroup), then for the multi-wave envs the collectives' scratch (EnvColl ballots at
// words 16-31, float sums at 32-47), the episode counters (48-58) and env drone 0's goal (60-62)
constexpr int QS_A_SCR_BITS = 16, QS_A_SCR_SUM = 32, QS_A_SCR_CNT = 48, QS_A_SCR_GOAL0 = 60;

template <int NPAD>
__global__ __launch_bounds__(StepGeoA<NPAD>::WGS) void step_kernel_a(const KP* __restrict__ kpp, Bufs b) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    QS_BIND_KP(kpp);
    const uint32_t seed = kpm.seed;
    // phase stamps (QS_STAMPS builds only): slot 0 loads, then summed over the ticks 1 controller, 2 OU draw,
    // 3 physics, 4 per-tick stats collisions, 5 capture / done, 6 downwash + target / scenario; after the loop
    // 7 counters + final obs, 8 done path, 9 obs tile + stores; 12 / 13 realtime wave start / end
    QS_STAMP_DECL
    QS_STAMP_ACC_DECL
    QS_RTSTAMP(12);
    QS_STAMP_MARK();
    using G = StepGeoA<NPAD>;
    constexpr int Q = G::Q, LPE = G::LPE, EPB = G::EPB, SLOTS = G::SLOTS, WGS = G::WGS;
    constexpr bool WIDE = G::WIDE;
    const int lane = threadIdx.x;
    const int el = lane / LPE, di = (lane % LPE) / Q, q = lane % Q;
    const int env0 = blockIdx.x * EPB;
    const int env = env0 + el;
    const bool active = env < kp.E && di < kp.N;
    const bool lead = active && q == 0;   // the sub-lane that writes the drone's outputs
    const int g = active ? env * kp.N + di : 0;
    const uint32_t gid = kp.id0 + (uint32_t)g;
    const int base = el * LPE;            // first lane of the env
    const int sbase = el * NPAD;          // first drone slot of the env
    const int nenv_blk = min(EPB, kp.E - env0);
    const int rows = nenv_blk * kp.N;
    float* row = lds + (size_t)(el * kp.N + di) * kp.obs_dim;
    float4* xch = reinterpret_cast<float4*>(lds + SLOTS * kp.obs_dim);
    int* efin = reinterpret_cast<int*>(lds + SLOTS * kp.obs_dim + SLOTS * 8);
    EnvA<NPAD, Q> ev(base, reinterpret_cast<uint64_t*>(efin + QS_A_SCR_BITS), reinterpret_cast<float*>(efin + QS_A_SCR_SUM));
    using Row = typename RowOf<(NPAD > 64)>::T;

    Drone d;
    load_drone<(NPAD > 64)>(kp, b, g, d);
    Ctl c;
    load_ctl(kp, b, g, c);
    const float a0 = reinterpret_cast<const float2*>(b.act)[g].x;
    const int eidx = active ? env : 0;
    int tick = b.env[QS_E_TICK * kp.E + eidx];
    const int episode = b.env[QS_E_EPISODE * kp.E + eidx];
    const int eflags = b.env[QS_E_FLAGS * kp.E + eidx];
    float tx = b.envf[QS_ENVF_TARGET_X * kp.E + eidx], ty = b.envf[QS_ENVF_TARGET_Y * kp.E + eidx];
    const float capr = b.envf[QS_ENVF_CAPTURE * kp.E + eidx];
    const bool repulsive = kp.scenario == QS_SCEN_DYNAMIC_REPULSIVE;
    const bool SCEN = kp.scen_b >= 0;   // a goal scenario of create_scenario: its state lives in the lead lane
    float* stab = scen_tab(lds, kp, SLOTS) + el * scen_stride<NPAD>();
    Scen sc;
    if (SCEN && active && di == 0 && q == 0) scen_load(kp, b, env, sc);

    // episode_extra_stats (kp.stats, quadrotor_multi_rewards.py:649-720, 886-969): the env's 11 counters
    // QS_E_ST_COL.. dealt over its lanes (lane li holds li + LPE t), kept in registers over the ticks
    constexpr int NCNT = 11, CT = (NCNT + LPE - 1) / LPE;
    const int li = lane - base;
    const bool envok = env < kp.E;
    int cnt[CT], cnt0[CT];
#pragma unroll
    for (int t = 0; t < CT; ++t) {
        const int k = li + LPE * t;
        cnt[t] = cnt0[t] = (kp.stats && envok && k < NCNT) ? b.env[(QS_E_ST_COL + k) * kp.E + env] : 0;
    }

    QS_STAMP_ACC(0);
    bool fin = false, success = eflags & QS_EF_SUCCESS;
    float rw = 0.f, gox = d.goal[0], goy = d.goal[1];
    float gdist = 0.f;   // infos[i]["goal_dist"] of the last executed tick (per-step infos, kp.rcomp)
    bool dn = false;
    float zn[Q > 1 ? Q - 1 : 1][4] = {};   // OU normals of the next Q - 1 ticks, drawn by sub-lanes 1 .. Q-1
    // Inside the tick loop `active` only masks the env-level collectives (each reads its own env's lanes) and the
    // env's LDS rows -- no global access: an env past E (a partial last block) computes values it never stores, so
    // the loop needs only the drone test, and none when the env's drones fill its lanes (a constant when specialised)
    const bool active_tick = QS_ACT_FOLD ? (kp.N == NPAD || di < kp.N) : active;
#pragma unroll 1   // 8 controller ticks: one copy of the body (I-cache), also when kp.ticks is a constant
    for (int sub = 0; sub < kp.ticks; ++sub) {
        const bool active = active_tick;
        if (fin) continue;   // the reference breaks out of its tick loop (:988); segment-uniform
        const Rng rng = env_rng(seed, tick, episode);
        float u[4];
        controller<Q>(kp, d, c, a0, d.goal[2], u, q);
        QS_STAMP_ACC(1);
        float z[4];   // QuadrotorDynamics.step: one OU draw per tick (:216)
        if constexpr (Q == 1) {
            normals4(rng, gid, S_OU, 0, z);
        } else if (sub % Q == 0) {   // wave-uniform: sub-lane q draws tick (tick + q)'s block
            float zr[4];
            normals4(env_rng(seed, tick + q, episode), gid, S_OU, 0, zr);
            qbc_ticks<Q>(zr, z, zn);
        } else {   // the next buffered tick, then shift the buffer (register moves, no dynamic index)
#pragma unroll
            for (int k = 0; k < 4; ++k) z[k] = zn[0][k];
#pragma unroll
            for (int t = 0; t + 1 < Q - 1; ++t)
#pragma unroll
                for (int k = 0; k < 4; ++k) zn[t][k] = zn[t + 1][k];
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) d.ou[k] = d.ou[k] + (kp.ou_theta * (kp.ou_mu - d.ou[k]) + kp.ou_sigma * z[k]);
        QS_STAMP_ACC(2);
        for (int s = 0; s < kp.sim_steps; ++s) substep(kp, d, u, d.ou, rng, gid, s);
        QS_STAMP_ACC(3);
        ++tick;
        if (kp.rcomp) {   // np.linalg.norm(self.dynamics.pos - self.goal) of this _step (quadrotor_single_rewards.py:457)
            const float gx = d.pos[0] - d.goal[0], gy = d.pos[1] - d.goal[1], gz = d.pos[2] - d.goal[2];
            gdist = fsqrt(gx * gx + gy * gy + gz * gz);
        }
        if (kp.stats) {   // collisions between drones and with the room (:649-720): bookkeeping only
            Row cur{};
            const float thr2 = kp.col_thr * kp.col_thr;
            if constexpr (LPE == 16 && NPAD * Q == 16) {   // (32-bit row words: the env's drones are < 16)
                uint32_t c32 = 0;
                if constexpr (Q == 2) {
                    col_row16_q2<0>(kp, d, di, thr2, c32);
                    c32 |= (uint32_t)dpp_i<quad_perm(1, 0, 3, 2)>((int)c32);   // qor<2> of the low word
                } else
                    col_row16<Q, 1>(kp, d, di, thr2, c32);
                cur = c32;
            } else {
                if (active && q == 0) xch[2 * (sbase + di)] = make_float4(d.pos[0], d.pos[1], d.pos[2], 0.f);
                lds_sync();
                constexpr int PJ = (NPAD + Q - 1) / Q;
                for (int t = 0; t < PJ; ++t) {
                    const int j = q + Q * t;
                    const float4 pj = xch[2 * (sbase + (j < NPAD ? j : NPAD - 1))];
                    const float dx = d.pos[0] - pj.x, dy = d.pos[1] - pj.y, dz = d.pos[2] - pj.z;
                    const bool hit = (j != di) & (j < kp.N) & (dx * dx + dy * dy + dz * dz <= thr2);
                    row_set(cur, j, hit);
                }
                cur = qor<Q>(cur);
                lds_sync();   // the tile is rewritten next tick
            }
            Row prevrow;
            row_of(d, prevrow);
            const bool uniq = active && row_any(cur) && !row_any(prevrow);   // setdiff1d(flat(cur), flat(prev))
            row_keep(d, cur);
            auto env_count = [&](bool x) { return ev.count(x && q == 0); };
            const bool settle = tick >= kp.st_settle;
            const bool fin5 = kpm.ep_len - (tick - 1) <= kp.st_final;   // time_remain (before tick += 1)
            const int col = env_count(uniq) / 2;
            if (col > 0 && settle && uniq) d.flags |= QS_FL_HIT_AGENT;
            const bool wall_new = (d.flags & QS_FL_CRASH_WALL) && !(d.flags & QS_FL_PREV_WALL);
            const bool ceil_new = (d.flags & QS_FL_CRASH_CEIL) && !(d.flags & QS_FL_PREV_CEIL);
            const bool cfloor = active && (d.flags & QS_FL_CRASH_FLOOR);
            const bool room_new = active && (cfloor || wall_new || ceil_new) && !(d.flags & QS_FL_PREV_ROOM);
            d.flags = (d.flags & ~(uint32_t)(QS_FL_PREV_WALL | QS_FL_PREV_CEIL | QS_FL_PREV_ROOM)) |
                      (wall_new ? QS_FL_PREV_WALL : 0u) | (ceil_new ? QS_FL_PREV_CEIL : 0u) |
                      (room_new ? (uint32_t)QS_FL_PREV_ROOM : 0u);
            if (ev.wany(cfloor || wall_new || ceil_new || room_new || col > 0)) {   // rare: something to count
                const int nfl = env_count(cfloor), nw = env_count(active && wall_new);
                const int nc = env_count(active && ceil_new), nr = env_count(room_new);
#pragma unroll
                for (int t = 0; t < CT; ++t) {
                    const int k = li + LPE * t;
                    cnt[t] += k == 0 ? col : k == 1 ? (settle ? nr : 0) : k == 2 ? (settle ? nfl : 0) :
                              k == 3 ? (settle ? nw : 0) : k == 4 ? (settle ? nc : 0) :
                              k == 5 ? (settle ? col : 0) : k == 6 ? (fin5 ? col : 0) : 0;
                }
            }
        }
        QS_STAMP_ACC(4);
        gox = d.goal[0];
        goy = d.goal[1];
        // capture reward (:711-735) against env 0's goal; dones (:882-988)
        float g0x = tx, g0y = ty;
        if (!repulsive) {
            if constexpr (WIDE) {   // env drone 0's goal through LDS (read before the next collective's barrier)
                float* g0 = reinterpret_cast<float*>(efin + QS_A_SCR_GOAL0);
                if (threadIdx.x == 0) {
                    g0[0] = d.goal[0];
                    g0[1] = d.goal[1];
                }
                lds_sync();
                g0x = g0[0];
                g0y = g0[1];
            } else {
                g0x = __shfl(d.goal[0], base);
                g0y = __shfl(d.goal[1], base);
            }
        }
        const float dx = g0x - d.pos[0], dy = g0y - d.pos[1];
        const float rel = fsqrt(dx * dx + dy * dy);
        const bool capi = capr > rel;
        const bool cap = ev.any(active && capi);
        const float captor = cap && capi ? kp.w_captor : 0.f;
        const float helper = cap && capr < rel ? kp.w_helper : 0.f;
        rw = ((0.f + captor) + helper) + kp.existence;
        dn = cap ? capi : (tick > kpm.ep_len);
        fin = ev.any(active && dn);
        success = success || cap;
        QS_STAMP_ACC(5);
        // perform_downwash once per tick with the control dt (:810-815); the reference then rebuilds the
        // tick's obs from the post-downwash state, which is what the final obs below read
        bool dwa = false;
        if (kp.downwash && kp.N > 1)
            dwa = downwash_env<NPAD, Q>(kp, d, rng, gid, env, base, di, q, active,
                                        kp.obs_dim >= 8 ? reinterpret_cast<float4*>(lds) : (WIDE ? xch : nullptr), sbase);
        if (repulsive) {   // scenario.step() (:797)
            target_step(kp, tx, ty, d.pos, active, ev);
            d.goal[0] = tx;
            d.goal[1] = ty;
        } else if (SCEN) {   // scenario.step() of a goal scenario (:848): the env's goal table in LDS
            if (active && q == 0)
                for (int k = 0; k < 3; ++k) stab[4 * di + k] = d.goal[k];
            lds_sync();
            // envok: `sc` is loaded only for envs < E (scen_load above); an env past E in a partial last block
            // runs the tick loop (QS_ACT_FOLD) but must not step a scenario from uninitialised registers
            if (active && envok && di == 0 && q == 0) {
                SDraw sd = sdraw(rng, gid, S_SCN);
                scen_step(kp, sc, tick, sd, stab, stab + 4 * (NPAD + 4));
            }
            lds_sync();
            if (active)
                for (int k = 0; k < 3; ++k) d.goal[k] = stab[4 * di + k];
        }
        // downwash anywhere in the env: the tick's obs are rebuilt after scenario.step (:848-859), i.e. they
        // see the moved goal
        if (kp.downwash && kp.N > 1 && ev.any(active && dwa)) {
            gox = d.goal[0];
            goy = d.goal[1];
        }
        QS_STAMP_ACC(6);
    }

    if (SCEN && active && di == 0 && q == 0 && !fin) scen_store(kp, b, env, sc);   // (a reset stores its own)
    if (kp.stats)
#pragma unroll
        for (int t = 0; t < CT; ++t) {
            const int k = li + LPE * t;
            if (envok && !fin && k < NCNT && cnt[t] != cnt0[t]) b.env[(QS_E_ST_COL + k) * kp.E + env] = cnt[t];
        }
    // ---- observations of the final tick (self obs of the last _step, neighbours after the loop) ----
    const Rng rng_last = env_rng(seed, tick - 1, episode);
    if (q == 0) xch_put_a(xch, sbase + di, d.pos, c.angle, d.vel);
    if (lane < EPB) efin[lane] = 0;
    lds_sync();
    if (fin && di == 0 && q == 0) efin[el] = 1;
#if QS_A_DEAL_SENSE
    if constexpr (Q == 2) {   // the sensor noise's two Philox blocks, one per sub-lane (bitwise the lead's draws)
        float zs[8];
        if (kp.sense) qdraws<Q, 2, 0>(rng_last, gid, S_SENSOR, 0, q, zs, nullptr);
        if (lead) self_obs_a(kp, d, c, gox, goy, rng_last, gid, S_SENSOR, S_SELF_CAM, row, zs);
    } else
#endif
    if (lead) self_obs_a(kp, d, c, gox, goy, rng_last, gid, S_SENSOR, S_SELF_CAM, row);
    if (kp.K > 0) {
        if constexpr (WIDE)
            neighbor_obs_wide<NPAD, Q>(kp, xch, sbase, di, d.pos, c.angle, c.angle, d.vel, rng_last, gid, false, active, row, q);
        else
            neighbor_obs_a<NPAD, Q>(kp, xch, sbase, di, d.pos, c.angle, c.angle, d.vel, rng_last, gid, false, active, row, q);
    }

    const bool state_bad = lead && drone_nonfinite(d), rew_bad = lead && !(rw * 0.f == 0.f);
    QS_STAMP_ACC(7);
    if (ev.wany(active && fin)) {  // some env finished: terminal obs + the worker's reset (subproc_vec_env_custom.py:42-46)
        lds_sync();
        for (int r = 0; r < rows; ++r) {
            if (!efin[r / kp.N]) continue;
            for (int q = lane; q < kp.obs_dim; q += WGS)
                b.term[(size_t)(env0 * kp.N + r) * kp.obs_dim + q] = lds[(size_t)r * kp.obs_dim + q];
        }
        lds_sync();
        if (kp.stats) {   // the finished episodes' episode_extra_stats rows (:886-969)
            float cv[NCNT];
            if constexpr (WIDE) {   // the counters live on lanes 0..10 of wave 0: through LDS
                int* cs = efin + QS_A_SCR_CNT;
                if (li < NCNT) cs[li] = cnt[0];
                lds_sync();
#pragma unroll
                for (int k = 0; k < NCNT; ++k) cv[k] = (float)cs[k];
            } else {
#pragma unroll
                for (int k = 0; k < NCNT; ++k) cv[k] = (float)__shfl(cnt[k / LPE], base + k % LPE);
            }
            auto env_bits = [&](bool x) { return ev.ec.bits(x && q == 0); };
            const Row hit_a = env_bits(active && (d.flags & QS_FL_HIT_AGENT));
            const Row all = env_bits(active);
            if (active && fin && q == 0) {
                const float n = (float)kp.N;
                const Row ok = all & ~hit_a;   // agent_col_obst stays 1 (no obstacles in flavor A)
                float* er = b.estats + (size_t)g * QS_NES;
#pragma unroll
                for (int k = 0; k < NCNT; ++k) er[QS_ES_COL + k] = cv[k];
                er[QS_ES_SUCCESS] = 0.f;                           // reached_goal is never set (:797-802)
                er[QS_ES_DEADLOCK] = (float)row_popc(ok) / n;
                er[QS_ES_COLRATE] = 1.f - (float)row_popc(ok) / n;
                er[QS_ES_NCOLRATE] = 1.f - (float)row_popc(all & ~hit_a) / n;
                er[QS_ES_OCOLRATE] = 0.f;
                er[QS_ES_SCEN] = repulsive ? 18.f : (SCEN ? (float)b.env[QS_E_SC_MODE * kp.E + env] : 0.f);
                const float nan = __builtin_nanf("");                  // np.mean of the empty distance list
                er[QS_ES_D1] = nan; er[QS_ES_D3] = nan; er[QS_ES_D5] = nan;
                er[QS_ES_REPLAY] = 0.f;
            }
#pragma unroll
            for (int t = 0; t < CT; ++t) {   // the episode statistics start over (:605-617)
                const int k = li + LPE * t;
                if (envok && fin && k < NCNT) b.env[(QS_E_ST_COL + k) * kp.E + env] = 0;
            }
            if (fin) row_keep(d, Row{});
        }
        const float sh = c.angle, sv[3] = {d.vel[0], d.vel[1], d.vel[2]};  // QuadrotorEnvMulti.heading / .vel
        const Rng rr = env_rng(seed, tick, episode);
        if (SCEN)
            scen_reset_a<NPAD>(kp, b, stab, env, di, active && fin && di == 0 && q == 0, active && fin, rr,
                               kp.id0 + (uint32_t)(env * kp.N), d);
        reset_env_a(kp, d, c, tx, ty, true, active, active && fin, rr, gid, kp.id0 + (uint32_t)(env * kp.N), ev);
        if (lead && fin) {
            self_obs_a(kp, d, c, d.goal[0], d.goal[1], rr, gid, S_RESET_SENSOR, S_RESET_SELF_CAM, row);
            b.stale[0 * kp.I + g] = sv[0];
            b.stale[1 * kp.I + g] = sv[1];
            b.stale[2 * kp.I + g] = sv[2];
            b.st[QS_F_HEADING * kp.I + g] = sh;
        }
        if (kp.K > 0) {
            if (q == 0) xch_put_a(xch, sbase + di, d.pos, sh, sv);
            lds_sync();
            if constexpr (WIDE)
                neighbor_obs_wide<NPAD, Q>(kp, xch, sbase, di, d.pos, sh, c.angle, sv, rr, gid, true, active && fin, row, q);
            else
                neighbor_obs_a<NPAD, Q>(kp, xch, sbase, di, d.pos, sh, c.angle, sv, rr, gid, true, active && fin, row, q);
        }
    }
    lds_sync();
    QS_STAMP_ACC(8);
    const int obs_bad = tile_store_v<tile_vecs<SLOTS, WGS>()>(lds, b.obs + (size_t)env0 * kp.N * kp.obs_dim, rows * kp.obs_dim,
                                                              lane, WGS);
    guard_count(b, obs_bad, rew_bad, state_bad);

    if (lead) {
        store_drone<(NPAD > 64)>(kp, b, g, d);
        store_ctl(kp, b, g, c);
        b.rew[g] = rw;
        b.done[g] = fin ? 1 : 0;
        if (kp.rcomp) b.rcomp[(size_t)QS_RI_GOAL_DIST * kp.I + g] = gdist;
        if (di == 0) {
            b.env[QS_E_TICK * kp.E + env] = fin ? 0 : tick;
            if (fin) b.env[QS_E_EPISODE * kp.E + env] = episode + 1;
            const int32_t nf = fin ? (QS_EF_STALE | QS_EF_HAS_POS) : ((eflags & ~QS_EF_STALE) | (success ? QS_EF_SUCCESS : 0));
            if (nf != eflags) b.env[QS_E_FLAGS * kp.E + env] = nf;
            if (repulsive) {
                b.envf[QS_ENVF_TARGET_X * kp.E + env] = tx;
                b.envf[QS_ENVF_TARGET_Y * kp.E + env] = ty;
            }
            b.rinfo[env] = fin ? (success ? 2 : 1) : 0;
        }
    }
    QS_STAMP_ACC(9);
    QS_RTSTAMP(13);
    QS_STAMP_FLUSH();
}

// explicit reset of masked envs (quadrotor_multi_rewards.QuadrotorEnvMulti.reset)
template <int NPAD>
__global__ __launch_bounds__(ResetGeoA<NPAD>::WGS) void reset_kernel_a(const KP* __restrict__ kpp, Bufs b) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    QS_BIND_KP(kpp);
    const uint32_t seed = kpm.seed;
    using G = ResetGeoA<NPAD>;
    constexpr int EPB = G::EPB, SLOTS = G::SLOTS, WGS = G::WGS;
    const int lane = threadIdx.x;
    const int el = lane / NPAD, di = lane % NPAD;
    const int env0 = blockIdx.x * EPB;
    const int env = env0 + el;
    const bool inr = env < kp.E && di < kp.N;
    const bool envsel = env < kp.E && (b.mask == nullptr || b.mask[env] != 0);
    const bool sel = inr && envsel;
    const int g = inr ? env * kp.N + di : 0;
    const uint32_t gid = kp.id0 + (uint32_t)g;
    const int base = el * NPAD;
    const int eidx = env < kp.E ? env : 0;
    const int episode = b.env[QS_E_EPISODE * kp.E + eidx];
    const int eflags = b.env[QS_E_FLAGS * kp.E + eidx];
    const Rng rng = env_rng(seed, b.env[QS_E_TICK * kp.E + eidx], episode);
    float* row = lds + (size_t)(el * kp.N + di) * kp.obs_dim;
    int* escr = reinterpret_cast<int*>(lds + SLOTS * kp.obs_dim + SLOTS * 8);
    EnvA<NPAD, 1> ev(base, reinterpret_cast<uint64_t*>(escr + QS_A_SCR_BITS), reinterpret_cast<float*>(escr + QS_A_SCR_SUM));
    Drone d;
    load_drone<(NPAD > 64)>(kp, b, g, d);
    Ctl c;
    load_ctl(kp, b, g, c);
    float tx = b.envf[QS_ENVF_TARGET_X * kp.E + eidx], ty = b.envf[QS_ENVF_TARGET_Y * kp.E + eidx];
    // stale QuadrotorEnvMulti.vel / .heading: last step's values unless a reset happened since
    const bool stale_valid = eflags & QS_EF_STALE;
    float sv[3], sh = stale_valid ? b.st[QS_F_HEADING * kp.I + g] : c.angle;
#pragma unroll
    for (int q = 0; q < 3; ++q) sv[q] = stale_valid ? b.stale[q * kp.I + g] : d.vel[q];
    const bool success = eflags & QS_EF_SUCCESS;
    if (kp.scen_b >= 0)
        scen_reset_a<NPAD>(kp, b, scen_tab(lds, kp, SLOTS) + el * scen_stride<NPAD>(), env, di, sel && di == 0, sel, rng,
                           kp.id0 + (uint32_t)(env * kp.N), d);
    reset_env_a(kp, d, c, tx, ty, eflags & QS_EF_HAS_POS, inr, sel, rng, gid, kp.id0 + (uint32_t)(env * kp.N), ev);
    if (sel) self_obs_a(kp, d, c, d.goal[0], d.goal[1], rng, gid, S_RESET_SENSOR, S_RESET_SELF_CAM, row);
    if (kp.K > 0) {
        float4* xch = reinterpret_cast<float4*>(lds + SLOTS * kp.obs_dim);
        xch_put_a(xch, lane, d.pos, sh, sv);
        lds_sync();
        if constexpr (NPAD > 64)
            neighbor_obs_wide<NPAD>(kp, xch, base, di, d.pos, sh, c.angle, sv, rng, gid, true, sel, row);
        else
            neighbor_obs_a<NPAD>(kp, xch, base, di, d.pos, sh, c.angle, sv, rng, gid, true, sel, row);
    }
    lds_sync();
    const int nenv_blk = min(EPB, kp.E - env0);
    for (int r = 0; r < nenv_blk * kp.N; ++r) {
        const int e = env0 + r / kp.N;
        if (b.mask != nullptr && b.mask[e] == 0) continue;
        for (int q = lane; q < kp.obs_dim; q += WGS)
            b.obs[(size_t)(env0 * kp.N + r) * kp.obs_dim + q] = lds[(size_t)r * kp.obs_dim + q];
    }
    if (env < kp.E && di == 0) b.rinfo[env] = envsel ? (success ? 2 : 1) : 0;
    if (sel) {
        store_drone<(NPAD > 64)>(kp, b, g, d);
        store_ctl(kp, b, g, c);
#pragma unroll
        for (int q = 0; q < 3; ++q) b.stale[q * kp.I + g] = sv[q];
        b.st[QS_F_HEADING * kp.I + g] = sh;
        b.done[g] = 0;
        if (di == 0) {
            b.env[QS_E_TICK * kp.E + env] = 0;
            b.env[QS_E_EPISODE * kp.E + env] = episode + 1;
            b.env[QS_E_FLAGS * kp.E + env] = QS_EF_STALE | QS_EF_HAS_POS;
            if (kp.stats)
                for (int k = 0; k < 11; ++k) b.env[(QS_E_ST_COL + k) * kp.E + env] = 0;
            b.envf[QS_ENVF_TARGET_X * kp.E + env] = tx;
            b.envf[QS_ENVF_TARGET_Y * kp.E + env] = ty;
        }
    }
}

}  // namespace qs
