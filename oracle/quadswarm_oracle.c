/* quadswarm_oracle.c -- float64 CPU restatement of the reference flavor-B swarm env step.
 *
 * TEST INFRASTRUCTURE ONLY (parity oracle + cpu_baseline "port" leg of bench.py).  Not linked
 * into, called by, or shipped with the product path.  See quadswarm_oracle.h for the RNG model.
 *
 * Reference = priban42/quad-swarm-rl-stable-baselines3; file:line citations are relative to its
 * root.  The numba kernels (@njit) are restated with the semantics NumPy gives them under the
 * harness in tools/refshim.py, which is how the golden fixtures in tests/golden were produced.
 */
#include "quadswarm_oracle.h"
#include <math.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define GRAV_C 9.81      /* quadrotor_dynamics.py:12 */
#define EPS_DYN 1e-6     /* quadrotor_dynamics.py:13 */
#define EPS_UTIL 1e-5    /* quad_utils.py:10 (collisions) */

/* ------------------------------------------------------------------------------------------ */
/* Philox4x32-10 (Salmon et al., "Parallel random numbers: as easy as 1, 2, 3", SC'11).       */
/* ------------------------------------------------------------------------------------------ */
static inline void mulhilo32(uint32_t a, uint32_t b, uint32_t* hi, uint32_t* lo) {
    uint64_t p = (uint64_t)a * (uint64_t)b;
    *hi = (uint32_t)(p >> 32);
    *lo = (uint32_t)p;
}

void or_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
    uint32_t k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; ++r) {
        uint32_t hi0, lo0, hi1, lo1;
        mulhilo32(0xD2511F53u, c0, &hi0, &lo0);
        mulhilo32(0xCD9E8D57u, c2, &hi1, &lo1);
        uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* u in (0,1): 24 high bits + half ulp; exactly representable in fp32 (GPU uses the same map) */
static inline double u01(uint32_t x) { return ((double)(x >> 8) + 0.5) * (1.0 / 16777216.0); }

static void philox_block(uint32_t seed, uint32_t id, uint32_t stream, uint64_t step, uint32_t block,
                         uint32_t out[4]) {
    uint32_t ctr[4] = {block, stream, (uint32_t)step, (uint32_t)(step >> 32)};
    uint32_t key[2] = {id, seed};
    or_philox4x32_10(ctr, key, out);
}

double or_philox_normal(uint32_t seed, uint32_t id, uint32_t stream, uint64_t step, uint32_t idx) {
    uint32_t w[4];
    philox_block(seed, id, stream, step, idx >> 2, w);
    int pair = (idx >> 1) & 1;
    double ua = u01(w[2 * pair]), ub = u01(w[2 * pair + 1]);
    double rr = sqrt(-2.0 * log(ua));
    double ang = 6.283185307179586 * ub;
    return (idx & 1) ? rr * sin(ang) : rr * cos(ang);
}

double or_philox_uniform(uint32_t seed, uint32_t id, uint32_t stream, uint64_t step, uint32_t idx) {
    uint32_t w[4];
    philox_block(seed, id, stream, step, idx >> 2, w);
    return u01(w[idx & 3]);
}

/* ---- draw source ---- */
static double tape_next(or_rng* r) {
    if (r->tape_pos >= r->tape_n) { r->overrun = 1; return 0.0; }
    return r->tape[r->tape_pos++];
}
static double spawn_next(or_rng* r) {
    if (r->spawn_pos >= r->spawn_n) { r->overrun = 1; return 0.0; }
    return r->spawn[r->spawn_pos++];
}
/* numpy normal(loc, scale) / uniform(low, high) */
static double rn(or_rng* r, uint32_t gid, uint32_t stream, uint32_t idx, double loc, double scale) {
    if (r->mode == OR_RNG_TAPE) return tape_next(r);
    return loc + scale * or_philox_normal(r->seed, gid, stream, r->step, idx);
}
static double ru(or_rng* r, uint32_t gid, uint32_t stream, uint32_t idx, double lo, double hi) {
    if (r->mode == OR_RNG_TAPE) return tape_next(r);
    return lo + (hi - lo) * or_philox_uniform(r->seed, gid, stream | OR_UNIF_BIT, r->step, idx);
}

double or_rn(or_rng* r, uint32_t gid, uint32_t stream, uint32_t idx, double loc, double scale) {
    return rn(r, gid, stream, idx, loc, scale);
}
double or_ru(or_rng* r, uint32_t gid, uint32_t stream, uint32_t idx, double lo, double hi) {
    return ru(r, gid, stream, idx, lo, hi);
}
double or_gnext(or_rng* r) { return spawn_next(r); }

/* ------------------------------------------------------------------------------------------ */
/* small linear algebra                                                                        */
/* ------------------------------------------------------------------------------------------ */
static inline double clipd(double x, double lo, double hi) { return x < lo ? lo : (x > hi ? hi : x); }
static inline double norm3(const double* v) { return sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); }
static inline double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static void matmul3(const double* a, const double* b, double* c) {
    double t[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) t[i * 3 + j] = a[i * 3] * b[j] + a[i * 3 + 1] * b[3 + j] + a[i * 3 + 2] * b[6 + j];
    memcpy(c, t, sizeof t);
}
static void yaw_rot(double theta, double* rot) {
    double c = cos(theta), s = sin(theta);
    double r[9] = {c, -s, 0., s, c, 0., 0., 0., 1.};
    memcpy(rot, r, sizeof r);
}

/* polar factor of rot == u @ vh of np.linalg.svd (quadrotor_dynamics.py:554-558); Newton
 * iteration X <- (X + X^-T)/2 converges to the same orthogonal factor for det > 0. */
void or_polar(double rot[9]) {
    double x[9];
    memcpy(x, rot, sizeof x);
    for (int it = 0; it < 60; ++it) {
        double a = x[0], b = x[1], c = x[2], d = x[3], e = x[4], f = x[5], g = x[6], h = x[7], i = x[8];
        double A = e * i - f * h, B = -(d * i - f * g), C = d * h - e * g;
        double det = a * A + b * B + c * C;
        /* inverse transpose = cofactor / det */
        double cof[9] = {A, B, C,
                         -(b * i - c * h), a * i - c * g, -(a * h - b * g),
                         b * f - c * e, -(a * f - c * d), a * e - b * d};
        double diff = 0.0;
        for (int k = 0; k < 9; ++k) {
            double nx = 0.5 * (x[k] + cof[k] / det);
            diff += fabs(nx - x[k]);
            x[k] = nx;
        }
        if (diff < 1e-16) break;
    }
    memcpy(rot, x, sizeof x);
}

/* ------------------------------------------------------------------------------------------ */
/* L1 physics                                                                                  */
/* ------------------------------------------------------------------------------------------ */
void or_params_default(or_params* p) {
    memset(p, 0, sizeof *p);
    p->scenario_b = OR_SC_NONE;
    /* crazyflie_params (quad_models.py:1-42) through QuadLink (inertia.py:182-310):
       values as the reference computes them (checked by tests/test_oracle_golden.py). */
    p->mass = 0.028000000000000008;
    p->inertia[0] = 1.3669232142857143e-05;
    p->inertia[1] = 1.4356732142857143e-05;
    p->inertia[2] = 2.656158333333334e-05;
    double tm = 9.81 * p->mass * 1.9 / 4.0;   /* quadrotor_dynamics.py:136 */
    double px[4] = {0.0325, -0.0325, -0.0325, 0.0325}, py[4] = {-0.0325, -0.0325, 0.0325, 0.0325};
    double ccw[4] = {-1., 1., -1., 1.};
    for (int k = 0; k < 4; ++k) {
        p->thrust_max[k] = tm;
        p->torque_max[k] = 0.006 * tm;
        p->prop_cross[k][0] = py[k];        /* cross(prop_pos, [0,0,1]) = (y, -x, 0) */
        p->prop_cross[k][1] = -px[k];
        p->prop_cross[k][2] = 0.0;
        p->prop_ccw[k] = ccw[k];
    }
    p->motor_tau_up = 4 * 0.005 / (0.15 + EPS_DYN);
    p->motor_tau_down = 4 * 0.005 / (0.15 + EPS_DYN);
    p->motor_linearity = 1.0;
    p->arm = 0.04596194077712559;
    p->gravity = 9.81;
    p->omega_max = 40.0;
    p->vel_damp = 0.0;
    p->damp_omega_quadratic = 0.0;
    p->dt = 0.005;
    p->sim_steps = 2;
    p->since_last_svd_limit = 0.5;
    p->room_lo[0] = -5; p->room_lo[1] = -5; p->room_lo[2] = 0;
    p->room_hi[0] = 5; p->room_hi[1] = 5; p->room_hi[2] = 10;
    p->ou_mu = 0.0; p->ou_theta = 0.15; p->ou_sigma = 0.2 * 0.05;
    p->sense_noise = 1;
    p->pos_norm_std = 0.005; p->pos_unif_range = 0.0;
    p->vel_norm_std = 0.01; p->vel_unif_range = 0.0;
    p->gyro_noise_density = 0.000175;
    p->quat_norm_std = 0.0; p->quat_unif_range = 0.0;
    p->acc_static_std = 0.002; p->acc_dyn_ratio = 0.005;
    p->num_agents = 8; p->num_envs = 1; p->ep_len = 1500;
    p->obs_repr = 0; p->k_neighbors = 6;
    p->collision_threshold = 2.0 * p->arm;
    p->collision_falloff_threshold = 4.0 * p->arm;
    p->control_dt = 0.01;
    p->rew_pos = 1.0; p->rew_effort = 0.05; p->rew_crash = 1.0; p->rew_orient = 1.0; p->rew_spin = 0.1;
    p->rew_quadcol_bin = 5.0; p->rew_quadcol_smooth_max = 10.0;
    p->use_downwash = 0; p->apply_collision_force = 1;
    p->spawn_box = 2.0;
    p->goal[0] = 0; p->goal[1] = 0; p->goal[2] = 2.0;
    /* obstacles off; C4 values when enabled (swarm_rl/runs/obstacles/quad_obstacle_baseline.py) */
    p->use_obstacles = 0; p->num_obstacles = 12; p->obst_area = 8; p->obst_scenario = 0;
    p->obst_size = 0.6; p->obst_z = 5.0; p->sdf_resolution = 0.1; p->rew_quadcol_bin_obst = 5.0;
}

/* OUNoiseNumba.noise (numba_utils.py:101-105): x <- x + theta(mu - x) + sigma randn(4) */
void or_ou_noise(const or_params* p, double ou[4], or_rng* r, uint32_t gid) {
    for (int k = 0; k < 4; ++k) {
        double z = rn(r, gid, OR_S_OU, (uint32_t)k, 0.0, 1.0);
        ou[k] = ou[k] + (p->ou_theta * (p->ou_mu - ou[k]) + p->ou_sigma * z);
    }
}

/* One physics substep == QuadrotorDynamics.step1_numba (quadrotor_dynamics.py:355-390):
 *   calculate_torque_integrate_rotations_and_update_omega (:504-573), room clip (:367-374),
 *   floor_interaction_numba (:576-646, threshold = arm), compute_velocity_and_acceleration (:649-656). */
void or_dyn_substep(const or_params* p, or_drone* d, const double cmds_in[4], const double thr_noise[4],
                    or_rng* r, uint32_t gid, int substep) {
    const double dt = p->dt;
    double cmds[4], thrusts[4], torque[3] = {0, 0, 0};
    double thrust_sum = 0.0;
    for (int k = 0; k < 4; ++k) {
        cmds[k] = clipd(cmds_in[k], 0.0, 1.0);                                   /* :511 */
        double tau = p->motor_tau_up;
        if (cmds[k] < d->thrust_cmds_damp[k]) tau = p->motor_tau_down;          /* :512-513 */
        if (tau > 1.0) tau = 1.0;                                                 /* :514 */
        double thrust_rot = pow(cmds[k], 0.5);                                    /* :517 */
        d->thrust_rot_damp[k] = tau * (thrust_rot - d->thrust_rot_damp[k]) + d->thrust_rot_damp[k];
        d->thrust_cmds_damp[k] = d->thrust_rot_damp[k] * d->thrust_rot_damp[k];  /* :519 */
        double noise = cmds[k] * thr_noise[k];                                    /* :522 */
        d->thrust_cmds_damp[k] = clipd(d->thrust_cmds_damp[k] + noise, 0.0, 1.0);
        double cd = d->thrust_cmds_damp[k];
        thrusts[k] = p->thrust_max[k] * ((1 - p->motor_linearity) * cd * cd + p->motor_linearity * cd);
    }
    for (int k = 0; k < 4; ++k) {                                                /* :527-533 */
        double t0 = p->prop_cross[k][0] * thrusts[k];
        double t1 = p->prop_cross[k][1] * thrusts[k];
        double t2 = p->prop_cross[k][2] * thrusts[k] + p->torque_max[k] * p->prop_ccw[k] * d->thrust_cmds_damp[k];
        torque[0] += t0; torque[1] += t1; torque[2] += t2;
    }
    for (int k = 0; k < 4; ++k) thrust_sum += thrusts[k];
    /* rotation: Rodrigues with world-frame omega (:544-551) */
    double* R = d->rot;
    double w[3];
    for (int i = 0; i < 3; ++i) w[i] = R[i * 3] * d->omega[0] + R[i * 3 + 1] * d->omega[1] + R[i * 3 + 2] * d->omega[2];
    double wn = norm3(w);
    if (wn != 0.0) {
        double K[9] = {0., -w[2] / wn, w[1] / wn, w[2] / wn, 0., -w[0] / wn, -w[1] / wn, w[0] / wn, 0.};
        double ang = wn * dt, sa = sin(ang), ca = 1.0 - cos(ang);
        double KK[9], dR[9];
        matmul3(K, K, KK);
        for (int i = 0; i < 9; ++i) dR[i] = ((i % 4 == 0) ? 1.0 : 0.0) + sa * K[i] + ca * KK[i];
        matmul3(dR, R, R);
    }
    d->since_last_svd += dt;                                                     /* :554-558 */
    if (d->since_last_svd > p->since_last_svd_limit) {
        or_polar(R);
        d->since_last_svd = 0.0;
    }
    /* omega update (:562-567) */
    const double* I = p->inertia;
    double o[3] = {d->omega[0], d->omega[1], d->omega[2]};
    double Io[3] = {I[0] * o[0], I[1] * o[1], I[2] * o[2]};
    double mo[3] = {-o[0], -o[1], -o[2]};
    double cr[3] = {mo[1] * Io[2] - mo[2] * Io[1], mo[2] * Io[0] - mo[0] * Io[2], mo[0] * Io[1] - mo[1] * Io[0]};
    for (int i = 0; i < 3; ++i) {
        double odot = (1.0 / I[i]) * (cr[i] + torque[i]);
        double damp = clipd(p->damp_omega_quadratic * (o[i] * o[i]), 0.0, 1.0);
        double on = o[i] + (1.0 - damp) * dt * odot;
        d->omega[i] = clipd(on, -p->omega_max, p->omega_max);
    }
    /* position (:570) and room clip (:367-374) */
    double before[3];
    for (int i = 0; i < 3; ++i) {
        d->pos[i] = d->pos[i] + dt * d->vel[i];
        before[i] = d->pos[i];
        d->pos[i] = clipd(d->pos[i], p->room_lo[i], p->room_hi[i]);
    }
    d->crashed_wall = (before[0] != d->pos[0]) || (before[1] != d->pos[1]);
    d->crashed_ceiling = before[2] > d->pos[2];
    /* floor_interaction_numba (:576-646), floor_threshold = self.arm (:385) */
    d->crashed_floor = 0;
    double acc[3];
    if (d->pos[2] <= p->arm) {
        d->pos[2] = p->arm;
        double force[3] = {R[2] * thrust_sum, R[5] * thrust_sum, R[8] * thrust_sum};
        if (d->on_floor) {
            double theta = atan2(R[3], R[0] + EPS_DYN);
            yaw_rot(theta, R);
            double fric = 0.6 * (p->mass * GRAV_C - force[2]);
            if (norm3(d->vel) < EPS_DYN) {
                double fxy = sqrt(force[0] * force[0] + force[1] * force[1]);
                fxy = fxy - fric > 0.0 ? fxy - fric : 0.0;
                if (fxy == 0.0) {
                    force[0] = 0.0; force[1] = 0.0;
                } else {
                    double fa = atan2(force[1], force[0]);
                    force[0] = fxy * cos(fa);
                    force[1] = fxy * sin(fa);
                }
            } else {
                double fa = atan2(d->vel[1], d->vel[0]);   /* numba sign (:608), see SURVEY §7 */
                force[0] = force[0] - cos(fa) * fric;
                force[1] = force[1] - sin(fa) * fric;
            }
        } else {
            d->on_floor = 1;
            d->crashed_floor = 1;
            for (int i = 0; i < 3; ++i) { d->vel[i] = 0.0; d->omega[i] = 0.0; }
            double theta = atan2(R[3], R[0] + EPS_DYN);
            if (R[8] < 0.0) theta = ru(r, gid, OR_S_FLOOR | ((uint32_t)substep << 8), 0, -M_PI, M_PI);
            yaw_rot(theta, R);
            for (int k = 0; k < 4; ++k) { d->thrust_cmds_damp[k] = 0.0; d->thrust_rot_damp[k] = 0.0; }
        }
        for (int i = 0; i < 3; ++i) acc[i] = (i == 2 ? -GRAV_C : 0.0) + (1.0 / p->mass) * force[i];
        if (acc[2] < 0.0) acc[2] = 0.0;
    } else {
        d->on_floor = 0;
        double force[3] = {R[2] * thrust_sum, R[5] * thrust_sum, R[8] * thrust_sum};
        for (int i = 0; i < 3; ++i) acc[i] = (i == 2 ? -GRAV_C : 0.0) + (1.0 / p->mass) * force[i];
    }
    for (int i = 0; i < 3; ++i) {
        d->acc[i] = acc[i];
        d->vel[i] = (1.0 - p->vel_damp) * d->vel[i] + dt * acc[i];             /* :652 */
    }
}

/* ------------------------------------------------------------------------------------------ */
/* sensor noise + self observation                                                             */
/* ------------------------------------------------------------------------------------------ */
/* rot2quat (sensor_noise.py:34-63) */
static void rot2quat(const double* R, double q[4]) {
    double tr = R[0] + R[4] + R[8];
    if (tr > 0) {
        double S = pow(tr + 1.0, 0.5) * 2;
        q[0] = 0.25 * S; q[1] = (R[7] - R[5]) / S; q[2] = (R[2] - R[6]) / S; q[3] = (R[3] - R[1]) / S;
    } else if (R[0] > R[4] && R[0] > R[8]) {
        double S = pow(1.0 + R[0] - R[4] - R[8], 0.5) * 2;
        q[0] = (R[7] - R[5]) / S; q[1] = 0.25 * S; q[2] = (R[1] + R[3]) / S; q[3] = (R[2] + R[6]) / S;
    } else if (R[4] > R[8]) {
        double S = pow(1.0 + R[4] - R[0] - R[8], 0.5) * 2;
        q[0] = (R[2] - R[6]) / S; q[1] = (R[1] + R[3]) / S; q[2] = 0.25 * S; q[3] = (R[5] + R[7]) / S;
    } else {
        double S = pow(1.0 + R[8] - R[0] - R[4], 0.5) * 2;
        q[0] = (R[3] - R[1]) / S; q[1] = (R[2] + R[6]) / S; q[2] = (R[5] + R[7]) / S; q[3] = 0.25 * S;
    }
}

/* add_noise_numba (sensor_noise.py:172-218) + add_noise_to_vel_acc_pos_omega_rot (:234-261).
 * Draw order is the reference's (27 draws); Philox indices: pos n0-2/u0-2, vel n3-5/u3-5,
 * omega n6-8, theta n9-11/u6-8, acc n12-17 (acc output unused by every obs repr). */
void or_sensor_noise(const or_params* p, const double pos[3], const double vel[3], const double rot[9],
                     const double omega[3], or_rng* r, uint32_t gid, uint32_t st,
                     double npos[3], double nvel[3], double nrot[9], double nomega[3]) {
    if (!p->sense_noise) {
        memcpy(npos, pos, 3 * sizeof(double)); memcpy(nvel, vel, 3 * sizeof(double));
        memcpy(nrot, rot, 9 * sizeof(double)); memcpy(nomega, omega, 3 * sizeof(double));
        return;
    }
    double a[3], b[3], theta[3];
    for (int i = 0; i < 3; ++i) a[i] = rn(r, gid, st, (uint32_t)i, 0.0, p->pos_norm_std);
    for (int i = 0; i < 3; ++i) b[i] = ru(r, gid, st, (uint32_t)i, -p->pos_unif_range, p->pos_unif_range);
    for (int i = 0; i < 3; ++i) npos[i] = pos[i] + a[i] + b[i];
    for (int i = 0; i < 3; ++i) a[i] = rn(r, gid, st, (uint32_t)(3 + i), 0.0, p->vel_norm_std);
    for (int i = 0; i < 3; ++i) b[i] = ru(r, gid, st, (uint32_t)(3 + i), -p->vel_unif_range, p->vel_unif_range);
    for (int i = 0; i < 3; ++i) nvel[i] = vel[i] + a[i] + b[i];
    for (int i = 0; i < 3; ++i) nomega[i] = omega[i] + rn(r, gid, st, (uint32_t)(6 + i), 0.0, p->gyro_noise_density);
    for (int i = 0; i < 3; ++i) a[i] = rn(r, gid, st, (uint32_t)(9 + i), 0.0, p->quat_norm_std);
    for (int i = 0; i < 3; ++i) b[i] = ru(r, gid, st, (uint32_t)(6 + i), -p->quat_unif_range, p->quat_unif_range);
    for (int i = 0; i < 3; ++i) theta[i] = a[i] + b[i];
    for (int i = 0; i < 6; ++i) (void)rn(r, gid, st, (uint32_t)(12 + i), 0.0, i < 3 ? p->acc_static_std : p->acc_dyn_ratio);
    /* quat_from_small_angle (sensor_noise.py:11-23) */
    double qs = (theta[0] * theta[0] + theta[1] * theta[1] + theta[2] * theta[2]);
    qs = sqrt(qs); qs = qs * qs / 4.0;
    double qt[4];
    if (qs < 1) {
        qt[0] = pow(1 - qs, 0.5); qt[1] = theta[0] * 0.5; qt[2] = theta[1] * 0.5; qt[3] = theta[2] * 0.5;
    } else {
        double w = 1.0 / pow(1 + qs, 0.5), f = 0.5 * w;
        qt[0] = w; qt[1] = theta[0] * f; qt[2] = theta[1] * f; qt[3] = theta[2] * f;
    }
    double qn = sqrt(qt[0] * qt[0] + qt[1] * qt[1] + qt[2] * qt[2] + qt[3] * qt[3]);
    for (int i = 0; i < 4; ++i) qt[i] /= qn;
    double q[4], nq[4];
    rot2quat(rot, q);
    /* quatXquat (quad_utils.py:163-174) */
    nq[0] = q[0] * qt[0] - q[1] * qt[1] - q[2] * qt[2] - q[3] * qt[3];
    nq[1] = q[0] * qt[1] + q[1] * qt[0] - q[2] * qt[3] + q[3] * qt[2];
    nq[2] = q[0] * qt[2] + q[1] * qt[3] + q[2] * qt[0] - q[3] * qt[1];
    nq[3] = q[0] * qt[3] - q[1] * qt[2] + q[2] * qt[1] + q[3] * qt[0];
    /* quat2R (quad_utils.py:146-151) */
    double w = nq[0], x = nq[1], y = nq[2], z = nq[3];
    nrot[0] = 1.0 - 2 * y * y - 2 * z * z; nrot[1] = 2 * x * y - 2 * z * w; nrot[2] = 2 * x * z + 2 * y * w;
    nrot[3] = 2 * x * y + 2 * z * w; nrot[4] = 1.0 - 2 * x * x - 2 * z * z; nrot[5] = 2 * y * z - 2 * x * w;
    nrot[6] = 2 * x * z - 2 * y * w; nrot[7] = 2 * y * z + 2 * x * w; nrot[8] = 1.0 - 2 * x * x - 2 * y * y;
}

static int self_obs_dim(const or_params* p) { return p->obs_repr == 0 ? 18 : (p->obs_repr == 1 ? 19 : 24); }

int or_obs_dim(const or_params* p) { return self_obs_dim(p) + 6 * p->k_neighbors + (p->use_obstacles ? 9 : 0); }

/* get_state.state_xyz_vxyz_R_omega[_floor|_wall] (get_state.py:226-292) */
static void self_obs(const or_params* p, const or_drone* d, or_rng* r, uint32_t gid, uint32_t st, double* out) {
    double np_[3], nv[3], nr[9], no[3];
    or_sensor_noise(p, d->pos, d->vel, d->rot, d->omega, r, gid, st, np_, nv, nr, no);
    for (int i = 0; i < 3; ++i) out[i] = np_[i] - d->goal[i];
    for (int i = 0; i < 3; ++i) out[3 + i] = nv[i];
    for (int i = 0; i < 9; ++i) out[6 + i] = nr[i];
    for (int i = 0; i < 3; ++i) out[15 + i] = no[i];
    if (p->obs_repr == 1) out[18] = np_[2];
    if (p->obs_repr == 2) {
        for (int i = 0; i < 3; ++i) out[18 + i] = clipd(np_[i] - p->room_lo[i], 0.0, 5.0);
        for (int i = 0; i < 3; ++i) out[21 + i] = clipd(p->room_hi[i] - np_[i], 0.0, 5.0);
    }
}

/* neighbour obs: neighborhood_indices (quadrotor_multi.py:344-375) + get_rel_pos_vel_item
 * (:275-319, pos_vel) + extend_obs_space clip (:328-342).  Sort key = norm of the 6-vector
 * [rel_pos, rel_vel] clamped at 0.01; numpy argsort on <=16 keys is insertion sort (stable). */
static void neighbor_obs(const or_params* p, const or_env* ev, double* obs, int obs_dim) {
    const int N = p->num_agents, K = p->k_neighbors, so = self_obs_dim(p);
    if (K <= 0) return;
    double rr[3], rv[3];
    for (int i = 0; i < 3; ++i) {
        rr[i] = p->room_hi[i] - p->room_lo[i];
        rv[i] = 2.0 * 3.0;          /* 2 * vxyz_max (quadrotor_single.py:296) */
    }
    for (int i = 0; i < N; ++i) {
        int idx[OR_MAXN], ord[OR_MAXN];
        double key[OR_MAXN], rel[OR_MAXN][6];
        int m = 0;
        for (int j = 0; j < N; ++j) {
            if (j == i) continue;
            for (int c = 0; c < 3; ++c) {
                rel[m][c] = ev->obs_pos[j][c] - ev->obs_pos[i][c];
                rel[m][3 + c] = ev->obs_vel[j][c] - ev->obs_vel[i][c];
            }
            idx[m] = j;
            m++;
        }
        for (int a = 0; a < m; ++a) ord[a] = a;
        if (K < N - 1) {
            for (int a = 0; a < m; ++a) {
                double s = 0.0;
                for (int c = 0; c < 6; ++c) s += rel[a][c] * rel[a][c];
                key[a] = sqrt(s);
                if (key[a] < 0.01) key[a] = 0.01;
            }
            /* stable insertion sort */
            for (int a = 1; a < m; ++a) {
                int v = ord[a], b = a - 1;
                while (b >= 0 && key[ord[b]] > key[v]) { ord[b + 1] = ord[b]; b--; }
                ord[b + 1] = v;
            }
        }
        double* row = obs + (size_t)i * obs_dim + so;
        for (int s = 0; s < K; ++s) {
            int a = ord[s];
            for (int c = 0; c < 3; ++c) row[s * 6 + c] = clipd(rel[a][c], -rr[c], rr[c]);
            for (int c = 0; c < 3; ++c) row[s * 6 + 3 + c] = clipd(rel[a][3 + c], -rv[c], rv[c]);
        }
        (void)idx;
    }
}

/* ------------------------------------------------------------------------------------------ */
/* collisions                                                                                  */
/* ------------------------------------------------------------------------------------------ */
/* compute_new_vel (collisions/utils.py:7-20) */
static void new_vel(double max_vel_magn, double vel[3], const double shift[3], double ratio) {
    double vn[3] = {vel[0] + shift[0], vel[1] + shift[1], vel[2] + shift[2]};
    double mag = norm3(vn);
    double den = mag == 0.0 ? mag + EPS_UTIL : mag;
    double dir[3] = {vn[0] / den, vn[1] / den, vn[2] / den};
    double nm = mag * ratio;
    if (nm > max_vel_magn) nm = max_vel_magn;
    for (int i = 0; i < 3; ++i) {
        double v = dir[i] * nm;
        double s = v - vel[i];
        vel[i] += s;
    }
}

/* compute_new_omega (collisions/utils.py:23-33): direction U(-1,1)^3, magnitude U(om/2, om) */
static void new_omega(or_rng* r, uint32_t gid, uint32_t st, uint32_t u0, double magn_scale, double out[3]) {
    double om = magn_scale * M_PI;
    double w[3];
    for (int i = 0; i < 3; ++i) w[i] = ru(r, gid, st, u0 + (uint32_t)i, -1.0, 1.0);
    double mag = norm3(w);
    double den = mag == 0.0 ? mag + EPS_UTIL : mag;
    double m2 = ru(r, gid, st, u0 + 3, om / 2, om);
    for (int i = 0; i < 3; ++i) out[i] = (w[i] / den) * m2;
}

/* perform_collision_between_drones (collisions/quadrotors.py:23-59).
 * Philox: key gid (lower drone), stream OR_S_PAIR | j<<8; normals try*9 + {0-2 cons, 3-5, 6-8};
 * uniforms 0 decay1, 1 decay2, 2-4 omega dir, 5 omega magnitude. */
void or_collide_drones(double pos1[3], double vel1[3], double omega1[3],
                       double pos2[3], double vel2[3], double omega2[3],
                       or_rng* r, uint32_t gid, uint32_t j) {
    uint32_t st = OR_S_PAIR | (j << 8);
    double n[3] = {pos1[0] - pos2[0], pos1[1] - pos2[1], pos1[2] - pos2[2]};
    double m = norm3(n);
    double den = m == 0.0 ? m + EPS_UTIL : m;
    for (int i = 0; i < 3; ++i) n[i] /= den;
    double v1n = dot3(vel1, n), v2n = dot3(vel2, n);
    double vc[3], s1[3], s2[3];
    for (int i = 0; i < 3; ++i) { vc[i] = (v2n - v1n) * n[i]; s1[i] = vc[i]; s2[i] = -vc[i]; }
    for (int t = 0; t < 3; ++t) {
        double cons[3], a[3], b[3];
        for (int i = 0; i < 3; ++i) cons[i] = rn(r, gid, st, (uint32_t)(t * 9 + i), 0.0, 0.8);
        for (int i = 0; i < 3; ++i) a[i] = rn(r, gid, st, (uint32_t)(t * 9 + 3 + i), 0.0, 0.15);
        for (int i = 0; i < 3; ++i) b[i] = rn(r, gid, st, (uint32_t)(t * 9 + 6 + i), 0.0, 0.15);
        double t1[3], t2[3];
        for (int i = 0; i < 3; ++i) {
            s1[i] = vc[i] + (cons[i] + a[i]);
            s2[i] = -vc[i] + (-cons[i] + b[i]);
            t1[i] = vel1[i] + s1[i];
            t2[i] = vel2[i] + s2[i];
        }
        double d1 = dot3(t1, n), d2 = dot3(t2, n);
        if (d1 > 0 && 0 > d2) break;
    }
    double n1 = norm3(vel1), n2 = norm3(vel2);
    double mx = n1 > n2 ? n1 : n2;
    double r1 = ru(r, gid, st, 0, 0.2, 0.8);
    new_vel(mx, vel1, s1, r1);
    double r2 = ru(r, gid, st, 1, 0.2, 0.8);
    new_vel(mx, vel2, s2, r2);
    double w[3];
    new_omega(r, gid, st, 2, 20.0, w);
    for (int i = 0; i < 3; ++i) { omega1[i] += w[i]; omega2[i] -= w[i]; }
}

/* perform_collision_with_wall (collisions/room.py:6-44).  Philox uniforms: 0 speed, 1-3 dir,
 * 4 x-override, 5 y-override, 6 z, 7-9 omega dir, 10 omega magnitude. */
void or_collide_wall(const or_params* p, or_drone* d, or_rng* r, uint32_t gid) {
    uint32_t st = OR_S_WALL;
    double sp = norm3(d->vel);
    double real = ru(r, gid, st, 0, 0.2 * sp, 0.8 * sp);
    real = clipd(real, 0.1, 6.0);
    int x0 = d->pos[0] == p->room_lo[0], x1 = d->pos[0] == p->room_hi[0];
    int y0 = d->pos[1] == p->room_lo[1], y1 = d->pos[1] == p->room_hi[1];
    double dir[3];
    for (int i = 0; i < 3; ++i) dir[i] = ru(r, gid, st, (uint32_t)(1 + i), -1.0, 1.0);
    if (x0) dir[0] = ru(r, gid, st, 4, 0.1, 1.0);
    else if (x1) dir[0] = ru(r, gid, st, 4, -1.0, -0.1);
    if (y0) dir[1] = ru(r, gid, st, 5, 0.1, 1.0);
    else if (y1) dir[1] = ru(r, gid, st, 5, -1.0, -0.1);
    dir[2] = ru(r, gid, st, 6, -1.0, -0.5);
    double dm = norm3(dir);
    for (int i = 0; i < 3; ++i) d->vel[i] = real * (dir[i] / (dm + 1e-5));
    double om = 20 * M_PI, w[3];
    for (int i = 0; i < 3; ++i) w[i] = ru(r, gid, st, (uint32_t)(7 + i), -1.0, 1.0);
    double wn = norm3(w) + 1e-5;
    for (int i = 0; i < 3; ++i) w[i] /= wn;
    double mg = ru(r, gid, st, 10, om / 2, om);
    for (int i = 0; i < 3; ++i) d->omega[i] += w[i] * mg;
}

/* perform_collision_with_ceiling (collisions/room.py:91-113).  Philox uniforms: 0 speed, 1-3 dir,
 * 4 z, 5-7 omega dir, 8 omega magnitude. */
void or_collide_ceiling(or_drone* d, or_rng* r, uint32_t gid) {
    uint32_t st = OR_S_CEIL;
    double sp = norm3(d->vel);
    double real = ru(r, gid, st, 0, 0.2 * sp, 0.8 * sp);
    real = clipd(real, 0.1, 6.0);
    double dir[3];
    for (int i = 0; i < 3; ++i) dir[i] = ru(r, gid, st, (uint32_t)(1 + i), -1.0, 1.0);
    dir[2] = ru(r, gid, st, 4, -1.0, -0.5);
    double dm = norm3(dir);
    for (int i = 0; i < 3; ++i) d->vel[i] = real * (dir[i] / (dm + 1e-5));
    double om = 20 * M_PI, w[3];
    for (int i = 0; i < 3; ++i) w[i] = ru(r, gid, st, (uint32_t)(5 + i), -1.0, 1.0);
    double wn = norm3(w) + 1e-5;
    for (int i = 0; i < 3; ++i) w[i] /= wn;
    double mg = ru(r, gid, st, 8, om / 2, om);
    for (int i = 0; i < 3; ++i) d->omega[i] += w[i] * mg;
}

/* perform_downwash (aerodynamics/downwash.py:4-51) + get_vel_omega_norm (:54-66).
 * Philox: key = source drone i; OR_S_DW uniforms 0 acc noise, 1 omega noise;
 * OR_S_DWPAIR | j<<8 uniforms 0-2 z-axis noise, 3-5 omega direction. */
int or_downwash(const or_params* p, or_drone* dr, int N, uint32_t gbase, or_rng* r) {
    int applied = 0;
    double P[OR_MAXN][3];
    for (int i = 0; i < N; ++i) for (int c = 0; c < 3; ++c) P[i][c] = dr[i].pos[c];
    for (int i = 0; i < N; ++i) {
        double z[3] = {dr[i].rot[2], dr[i].rot[5], dr[i].rot[8]};
        uint32_t gi = gbase + (uint32_t)i;
        double an = ru(r, gi, OR_S_DW, 0, -0.1, 0.1);
        double wnz = ru(r, gi, OR_S_DW, 1, -0.01, 0.01);
        for (int j = 0; j < N; ++j) {
            double rel[3] = {P[j][0] - P[i][0], P[j][1] - P[i][1], P[j][2] - P[i][2]};
            double dist = norm3(rel);
            double acc = (6.0 / 17.0) * (-10 * dist + 7) + an;
            if (acc < 1e-6) acc = 1e-6;
            double wd = 0.3 * (dist - 1) * (dist - 1) + wnz;
            if (wd < 1e-6) wd = 1e-6;
            double rz = dot3(rel, z);
            double rxy = sqrt(dist * dist - rz * rz);
            if (i == j) continue;
            if (-0.7 < rz && rz < 0 && rxy < 0.1) {
                uint32_t st = OR_S_DWPAIR | ((uint32_t)j << 8);
                double nz[3], dw[3];
                for (int c = 0; c < 3; ++c) nz[c] = z[c] + ru(r, gi, st, (uint32_t)c, -0.1, 0.1);
                double nm = norm3(nz);
                double den = nm == 0.0 ? nm + 1e-6 : nm;
                for (int c = 0; c < 3; ++c) dw[c] = ru(r, gi, st, (uint32_t)(3 + c), -1.0, 1.0);
                double dm = norm3(dw);
                double den2 = dm == 0.0 ? dm + 1e-6 : dm;
                for (int c = 0; c < 3; ++c) {
                    dr[j].vel[c] += acc * (-1.0 * (nz[c] / den)) * p->control_dt;
                    dr[j].omega[c] += wd * (dw[c] / den2) * p->control_dt;
                }
                applied = 1;
            }
        }
    }
    return applied;
}

/* ------------------------------------------------------------------------------------------ */
/* obstacles (flavor B)                                                            */
/* ------------------------------------------------------------------------------------------ */
/* get_cell_centers (obstacles/utils.py:46-58) as the env indexes it: grid cell (row, col) of the
 * n x n spawn area -> cell_centers[row + n*col] (quadrotor_multi.py:422, o_base.py:89-92) */
void or_cell_xy(int row, int col, int n, double out[2]) {
    const double h = (double)(n / 2);
    out[0] = (double)col + 0.5 - h;
    out[1] = (double)(n - 1 - row) + 0.5 - h;
}

/* the env's pillar diameter: MultiObstacles(obstacle_size=self.obst_size) of its last reset
 * (quadrotor_multi.py:445-450), i.e. the configured size or a domain-randomisation choice */
double or_env_obst_size(const or_params* p, const or_env* ev) {
    return ev->obst_si > 0 ? p->dr_sizes[ev->obst_si] : p->obst_size;
}

/* get_surround_sdfs (obstacles/utils.py:4-27): 3x3 grid at +-resolution, min distance - radius */
void or_obst_sdf(const or_params* p, const or_env* ev, const double xy[2], double out[9]) {
    const double res = p->sdf_resolution, rad = or_env_obst_size(p, ev) / 2.0;
    const double gx[3] = {xy[0] - res, xy[0], xy[0] + res}, gy[3] = {xy[1] - res, xy[1], xy[1] + res};
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) {
            double md = 100.0;
            for (int o = 0; o < ev->n_obst; ++o) {
                double dx = gx[a] - ev->obst[o][0], dy = gy[b] - ev->obst[o][1];
                double d = sqrt(dx * dx + dy * dy);
                if (d < md) md = d;
            }
            out[a * 3 + b] = md - rad;
        }
}

/* collision_detection (obstacles/utils.py:30-43): first obstacle within arm + radius (xy) */
int or_obst_detect(const or_params* p, const or_env* ev, const double xy[2]) {
    const double thr = p->arm + or_env_obst_size(p, ev) / 2.0;
    for (int o = 0; o < ev->n_obst; ++o) {
        double dx = xy[0] - ev->obst[o][0], dy = xy[1] - ev->obst[o][1];
        if (sqrt(dx * dx + dy * dy) <= thr) return o;
    }
    return -1;
}

/* perform_collision_with_obstacle (collisions/obstacles.py:23-50) with
 * compute_col_norm_and_new_vel_obst (:8-20).  Philox indices (stream OBST): normals t*6+0..2 (0.1),
 * t*6+3..5 (0.05) for try t; uniforms 0 decay ratio, 1-3 omega direction, 4 omega magnitude. */
static void collide_obstacle_sz(double size, or_drone* d, const double opos[3], or_rng* r,
                                uint32_t gid) {
    double n[3] = {d->pos[0] - opos[0], d->pos[1] - opos[1], 0.0};
    double nm = norm3(n);
    double den = nm == 0.0 ? nm + EPS_UTIL : nm;
    for (int c = 0; c < 3; ++c) n[c] /= den;
    const double vm = norm3(d->vel);
    double nv[3] = {vm * n[0], vm * n[1], vm * n[2]};
    double noise[3] = {0, 0, 0};
    for (int t = 0; t < 3; ++t) {
        double cons[3], tmp[3];
        for (int c = 0; c < 3; ++c) cons[c] = rn(r, gid, OR_S_OBST, (uint32_t)(t * 6 + c), 0.0, 0.1);
        for (int c = 0; c < 3; ++c) tmp[c] = cons[c] + rn(r, gid, OR_S_OBST, (uint32_t)(t * 6 + 3 + c), 0.0, 0.05);
        if ((nv[0] + tmp[0]) * n[0] + (nv[1] + tmp[1]) * n[1] + (nv[2] + tmp[2]) * n[2] > 0) {
            memcpy(noise, tmp, sizeof tmp);
            break;
        }
    }
    const double max_v = norm3(d->vel);
    double dp[3] = {d->pos[0] - opos[0], d->pos[1] - opos[1], d->pos[2] - opos[2]};
    const int inside = norm3(dp) < size / 2.0;
    double shift[3];
    for (int c = 0; c < 3; ++c) shift[c] = nv[c] - d->vel[c] + noise[c];
    double ratio = inside ? ru(r, gid, OR_S_OBST, 0, 1.0, 1.0) : ru(r, gid, OR_S_OBST, 0, 0.2, 0.8);
    new_vel(max_v, d->vel, shift, ratio);
    double w[3];
    new_omega(r, gid, OR_S_OBST, 1, 1.0, w);
    for (int c = 0; c < 3; ++c) d->omega[c] += w[c];
}

void or_collide_obstacle(const or_params* p, or_drone* d, const double opos[3], or_rng* r, uint32_t gid) {
    collide_obstacle_sz(p->obst_size, d, opos, r, gid);
}

/* Scenario_o_base.max_square_area_center (o_base.py:125-153), quirks included: dp's first row and
 * column start as the obstacle map itself, the centre is (i - (s-1)//2, j - (s-1)//2). */
void or_max_square_center(const unsigned char* map, int n, double out_xy[2]) {
    int dp[64][64];
    memset(dp, 0, sizeof dp);
    for (int j = 0; j < n; ++j) dp[0][j] = map[j];
    for (int i = 0; i < n; ++i) dp[i][0] = map[i * n];
    int ms = 0, cx = 0, cy = 0;
    for (int i = 1; i < n; ++i)
        for (int j = 1; j < n; ++j)
            if (map[i * n + j] == 0) {
                int a = dp[i - 1][j], b = dp[i][j - 1], c = dp[i - 1][j - 1];
                int m = a < b ? a : b;
                m = m < c ? m : c;
                dp[i][j] = m + 1;
                if (dp[i][j] > ms) {
                    ms = dp[i][j];
                    cx = i - (ms - 1) / 2;
                    cy = j - (ms - 1) / 2;
                }
            }
    /* cell_centers[cx + n*cy] */
    or_cell_xy(cx, cy, n, out_xy);
}

/* partial Fisher-Yates: the first k of a uniformly random permutation of 0..n-1 (Philox stand-in for
 * np.random.choice(n, k, replace=False), same distribution) */
static void choose_k(or_rng* r, uint32_t gid, uint32_t st, uint32_t u0, int n, int k, int* out) {
    int a[64];
    for (int i = 0; i < n; ++i) a[i] = i;
    for (int i = 0; i < k; ++i) {
        double u = or_philox_uniform(r->seed, gid, st | OR_UNIF_BIT, r->step, u0 + (uint32_t)i);
        int j = i + (int)(u * (double)(n - i));
        if (j > n - 1) j = n - 1;
        int t = a[i]; a[i] = a[j]; a[j] = t;
        out[i] = a[i];
    }
}

/* obstacle map + scenario for one env reset (quadrotor_multi.py:405-426, 449-452; scenarios/mix.py:78-99;
 * o_random.py:26-51; o_static_same_goal.py:28-48; o_base.py:58-92).  Fills per-drone spawn points
 * and goals. */
static void obstacle_reset(const or_params* p, or_env* ev, uint32_t gbase, or_rng* r, double spawn[][3],
                           double goal[][3]) {
    const int tape = r->mode == OR_RNG_TAPE;
    /* domain randomisation (quad_experience_replay.py:106-118, 206-214): the wrapper's reset picks
     * np.random.choice(obst_densities) then np.random.choice(obst_sizes) and hands them to env.reset
     * (quadrotor_multi.py:440-446).  Philox mode = the GPU's fused reset, which IS the wrapper's reset
     * (DR needs the wrapper, i.e. replay on).  Tape mode replays the bare env, whose in-env resets keep
     * the values: the caller sets obst_mi / obst_si as the wrapper chose them. */
    if (!tape && p->dr_n_counts > 0) {
        const int c = (int)(or_philox_uniform(r->seed, gbase, OR_S_DR | OR_UNIF_BIT, r->step, 0) * (double)p->dr_n_counts);
        if (p->dr_counts[c + 1] >= 0) ev->obst_mi = c + 1;
    }
    if (!tape && p->dr_n_sizes > 0) {
        const int c = (int)(or_philox_uniform(r->seed, gbase, OR_S_DR | OR_UNIF_BIT, r->step, 1) * (double)p->dr_n_sizes);
        if (p->dr_sizes[c + 1] > 0.0) ev->obst_si = c + 1;
    }
    const int n = p->obst_area, N = p->num_agents;
    const int M = ev->obst_mi > 0 ? p->dr_counts[ev->obst_mi] : p->num_obstacles;
    unsigned char map[64 * 64];
    memset(map, 0, sizeof map);
    int ids[64];
    if (tape) for (int o = 0; o < M; ++o) ids[o] = (int)tape_next(r);
    else choose_k(r, gbase, OR_S_OBSTMAP, 0, n * n, M, ids);
    ev->n_obst = M;
    for (int o = 0; o < M; ++o) {
        int rid = ids[o] / n, cid = ids[o] % n;
        map[rid * n + cid] = 1;
        or_cell_xy(rid, cid, n, ev->obst[o]);
    }
    int mode;
    if (p->obst_scenario == 0) mode = tape ? ((int)spawn_next(r)) % 2
                                           : (or_philox_uniform(r->seed, gbase, OR_S_OSCEN | OR_UNIF_BIT, r->step, 0) < 0.5 ? 0 : 1);
    else mode = p->obst_scenario - 1;
    ev->obst_mode = mode;
    int fr[64 * 64], F = 0;
    for (int i = 0; i < n * n; ++i) if (!map[i]) fr[F++] = i;   /* np.where(map == 0): row-major */
    int sp[OR_MAXN], gl[OR_MAXN];
    double sz[OR_MAXN], gz[OR_MAXN], ez = 0.0;
    if (mode == 0) {   /* o_random */
        if (tape) {
            for (int k = 0; k < 2 * N; ++k) { (void)tape_next(r); (void)tape_next(r); }   /* generate_pos_obst_map x2N */
            for (int i = 0; i < N; ++i) sp[i] = (int)tape_next(r);
            for (int i = 0; i < N; ++i) sz[i] = tape_next(r);
            for (int i = 0; i < N; ++i) gl[i] = (int)tape_next(r);
            for (int i = 0; i < N; ++i) gz[i] = tape_next(r);
            (void)tape_next(r);   /* duration_step */
        } else {
            choose_k(r, gbase, OR_S_OSCEN, 1, F, N, sp);
            choose_k(r, gbase, OR_S_OSCEN, 1 + (uint32_t)N, F, N, gl);
            for (int i = 0; i < N; ++i) {
                sz[i] = 1.0 + 2.0 * or_philox_uniform(r->seed, gbase + (uint32_t)i, OR_S_RESET | OR_UNIF_BIT, r->step, 3);
                gz[i] = 1.0 + 2.0 * or_philox_uniform(r->seed, gbase + (uint32_t)i, OR_S_RESET | OR_UNIF_BIT, r->step, 4);
            }
        }
        for (int i = 0; i < N; ++i) {
            int a = fr[sp[i]], b = fr[gl[i]];
            or_cell_xy(a / n, a % n, n, spawn[i]); spawn[i][2] = sz[i];
            or_cell_xy(b / n, b % n, n, goal[i]); goal[i][2] = gz[i];
        }
    } else if (mode >= 2) {   /* the dynamic modes (Philox: the GPU's obstacle_reset_env order) */
        choose_k(r, gbase, OR_S_OSCEN, 1, F, N, sp);
        for (int i = 0; i < N; ++i)
            sz[i] = 1.0 + 2.0 * or_philox_uniform(r->seed, gbase + (uint32_t)i, OR_S_RESET | OR_UNIF_BIT, r->step, 3);
        or_sdraw sd;
        memset(&sd, 0, sizeof sd);
        sd.mode = OR_RNG_PHILOX; sd.seed = r->seed; sd.key = gbase; sd.stream = OR_S_SCN_RESET; sd.step = r->step;
        or_oscen_reset(p, mode, &ev->scen, &sd, map, n, NULL, NULL, goal);
        for (int i = 0; i < N; ++i) {
            int a = fr[sp[i]];
            or_cell_xy(a / n, a % n, n, spawn[i]); spawn[i][2] = sz[i];
        }
    } else {           /* o_static_same_goal */
        if (tape) {
            (void)tape_next(r);   /* duration_time */
            for (int i = 0; i < N; ++i) sp[i] = (int)tape_next(r);
            for (int i = 0; i < N; ++i) sz[i] = tape_next(r);
            ez = tape_next(r);
        } else {
            choose_k(r, gbase, OR_S_OSCEN, 1, F, N, sp);
            for (int i = 0; i < N; ++i)
                sz[i] = 1.0 + 2.0 * or_philox_uniform(r->seed, gbase + (uint32_t)i, OR_S_RESET | OR_UNIF_BIT, r->step, 3);
            ez = 1.5 + 1.5 * or_philox_uniform(r->seed, gbase, OR_S_OSCEN | OR_UNIF_BIT, r->step, 2 * (uint32_t)N + 1);
        }
        double exy[2];
        or_max_square_center(map, n, exy);
        for (int i = 0; i < N; ++i) {
            int a = fr[sp[i]];
            or_cell_xy(a / n, a % n, n, spawn[i]); spawn[i][2] = sz[i];
            goal[i][0] = exy[0]; goal[i][1] = exy[1]; goal[i][2] = ez;
        }
    }
}

/* ------------------------------------------------------------------------------------------ */
/* env step / reset                                                                            */
/* ------------------------------------------------------------------------------------------ */
/* QuadrotorSingle._reset (quadrotor_single.py:401-469), static_same_goal goals
 * (scenarios/base.py:255-272 with formation size 0), QuadrotorEnvMulti.reset (quadrotor_multi.py:440-517) */
/* episode_extra_stats bookkeeping of one step (quadrotor_multi.py:555-566, 575-589, 599-606, 631-656).
 * tick = envs[0].tick after the drones' _step; time_remain = QuadrotorSingle.time_remain of the step. */
void or_episode_stats_step(const or_params* p, or_env* ev, or_drone* dr, int N, const int* in_cur, const int* in_prev,
                           const int* onew, const int* wall_new, const int* ceil_new, const double* dist_goal,
                           const double* obs, int od, int time_remain) {
    const double freq = 1.0 / p->control_dt;
    const int settle = (double)ev->tick >= 1.5 * freq;               /* collisions_grace_period_steps */
    /* collisions_curr_tick = len(last_step_unique_collisions) // 2 */
    int uniq = 0;
    for (int i = 0; i < N; ++i) uniq += in_cur[i] && !in_prev[i];
    const int cnt = uniq / 2;
    ev->st_col += cnt;
    if (cnt > 0 && settle) {
        ev->st_col_settle += cnt;
        for (int i = 0; i < N; ++i) if (in_cur[i] && !in_prev[i]) dr[i].hit_agent = 1;
    }
    if (cnt > 0 && (double)time_remain <= 5.0 * freq) ev->st_col_final += cnt;
    if (p->use_obstacles && onew) {
        int oc = 0;
        for (int i = 0; i < N; ++i) oc += onew[i];
        ev->st_ocol += oc;
        if (oc > 0 && settle) {
            ev->st_ocol_settle += oc;
            for (int i = 0; i < N; ++i)
                if (onew[i]) {
                    const double* q = obs + (size_t)i * od;   /* the step's obs[qid][0:3] (noisy pos - goal) */
                    const double rd = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2]);
                    if (rd > 3.5) ev->st_o35 += 1;
                    if (rd > 5.0) ev->st_o5 += 1;
                    dr[i].hit_obst = 1;
                }
        }
    }
    /* room: floor list (crashed_floor), new wall / ceiling lists; room list = their union minus the previous
     * step's room list (which it then becomes) */
    int nf = 0, nw = 0, nc = 0, nr = 0;
    for (int i = 0; i < N; ++i) {
        const int any = dr[i].crashed_floor || wall_new[i] || ceil_new[i];
        const int room = any && !dr[i].prev_room;
        dr[i].prev_room = room;
        nf += dr[i].crashed_floor != 0; nw += wall_new[i]; nc += ceil_new[i]; nr += room;
    }
    if (settle) { ev->st_room += nr; ev->st_floor += nf; ev->st_wall += nw; ev->st_ceil += nc; }
    /* distance_to_goal[i].append(dt * dist); reached_goal (mean of the last 5 entries / dt < 0.5); flavor A
     * never appends (quadrotor_multi_rewards.py:797-802 commented out): dist_goal NULL */
    if (!dist_goal) return;
    const int T = p->ep_len + 1;                                    /* the entry count when the episode ends */
    const int win[3] = {(int)(1.0 * freq), (int)(3.0 * freq), (int)(5.0 * freq)};
    for (int i = 0; i < N; ++i) {
        or_drone* d = &dr[i];
        const double v = p->dt * dist_goal[i];
        d->dring[ev->tick % 5] = v;
        for (int k = 0; k < 3; ++k) if (ev->tick > T - win[k]) d->dsum[k] += v;
        if (ev->tick >= 5 && !d->reached) {
            double m = 0.0;
            for (int j = 4; j >= 0; --j) m += d->dring[(ev->tick - j) % 5];   /* oldest first, like np.mean */
            if (m / 5.0 / p->dt < 0.5) d->reached = 1;                      /* approch_goal_metric */
        }
    }
}

/* the stats of the episode that just finished (quadrotor_multi.py:739-831), before the in-env reset */
void or_episode_stats_done(const or_params* p, or_env* ev, or_drone* dr, int N) {
    const double freq = 1.0 / p->control_dt;
    const int T = p->ep_len + 1;
    double* s = ev->ep_stats;
    memset(s, 0, sizeof ev->ep_stats);
    s[OR_ES_COL] = ev->st_col; s[OR_ES_ROOM] = ev->st_room; s[OR_ES_FLOOR] = ev->st_floor; s[OR_ES_WALL] = ev->st_wall;
    s[OR_ES_CEIL] = ev->st_ceil; s[OR_ES_COL_SETTLE] = ev->st_col_settle; s[OR_ES_COL_FINAL] = ev->st_col_final;
    s[OR_ES_OCOL] = ev->st_ocol; s[OR_ES_OCOL_SETTLE] = ev->st_ocol_settle; s[OR_ES_O35] = ev->st_o35;
    s[OR_ES_O5] = ev->st_o5;
    int n_ok = 0, n_succ = 0, n_dead = 0, n_ha = 0, n_ho = 0;
    for (int i = 0; i < N; ++i) {
        const int ok = !dr[i].hit_agent && !dr[i].hit_obst;   /* logical_and(agent_col_agent, agent_col_obst) */
        n_ok += ok; n_succ += ok && dr[i].reached; n_dead += ok && !dr[i].reached;
        n_ha += !dr[i].hit_agent; n_ho += !dr[i].hit_obst;
    }
    s[OR_ES_SUCCESS] = (double)n_succ / N;
    s[OR_ES_DEADLOCK] = (double)n_dead / N;
    s[OR_ES_COLRATE] = 1.0 - (double)n_ok / N;
    s[OR_ES_NCOLRATE] = 1.0 - (double)n_ha / N;
    s[OR_ES_OCOLRATE] = 1.0 - (double)n_ho / N;
    /* scenario ids of quadswarm_amd.stats: 16 + mode for o_random / o_static_same_goal, 17 + mode for the dynamic ones */
    s[OR_ES_SCEN] = p->use_obstacles ? (ev->obst_mode < 2 ? 16 : 17) + ev->obst_mode
                                     : (p->scenario_b == OR_SC_NONE ? 0 : ev->scen.mode);
    const int win[3] = {(int)(1.0 * freq), (int)(3.0 * freq), (int)(5.0 * freq)};
    for (int i = 0; i < N; ++i)
        for (int k = 0; k < 3; ++k) dr[i].ep_dist[k] = dr[i].dsum[k] / (double)(win[k] < T ? win[k] : T) / p->dt;
    ev->ep_done += 1;
}

void or_env_reset(const or_params* p, or_drone* drones, or_env* envs, int e, or_rng* r, double* obs) {
    const int N = p->num_agents, od = or_obs_dim(p);
    or_env* ev = &envs[e];
    r->step = ((uint64_t)ev->episode << 32) | (uint32_t)ev->tick;   /* env Philox counter */
    const uint32_t gbase = p->id_offset + (uint32_t)((size_t)e * N);
    double spawn[OR_MAXN][3], goal[OR_MAXN][3];
    if (p->use_obstacles) {
        obstacle_reset(p, ev, gbase, r, spawn, goal);
    } else if (p->scenario_b != OR_SC_NONE) {   /* scenario.reset(); spawn points = goals (:459-472) */
        or_sdraw sd;
        memset(&sd, 0, sizeof sd);
        sd.mode = OR_RNG_PHILOX; sd.seed = r->seed; sd.key = gbase; sd.stream = OR_S_SCN_RESET; sd.step = r->step;
        or_scen_reset(p, &ev->scen, &sd, goal);
        memcpy(spawn, goal, sizeof(double) * 3 * (size_t)N);
    } else {
        for (int i = 0; i < N; ++i)
            for (int c = 0; c < 3; ++c) spawn[i][c] = goal[i][c] = p->goal[c];
    }
    for (int i = 0; i < N; ++i) {
        or_drone* d = &drones[(size_t)e * N + i];
        uint32_t gid = gbase + (uint32_t)i;
        for (int c = 0; c < 3; ++c) d->goal[c] = goal[i][c];
        double xyz[3];
        for (int c = 0; c < 3; ++c) {
            double u = (r->mode == OR_RNG_TAPE) ? spawn_next(r)
                                                : -p->spawn_box + 2 * p->spawn_box *
                                                      or_philox_uniform(r->seed, gid, OR_S_RESET | OR_UNIF_BIT, r->step, (uint32_t)c);
            xyz[c] = u + spawn[i][c];
        }
        if (xyz[2] < 0.75) xyz[2] = 0.75;
        for (int c = 0; c < 3; ++c) { d->pos[c] = xyz[c]; d->vel[c] = 0.0; d->omega[c] = 0.0; d->acc[c] = 0.0; }
        /* randyaw rejection (quadrotor_single.py:454-456, quad_utils.py:228-230, to_xyhat :140-145) */
        double tx = -xyz[0], ty = -xyz[1];
        double tn = sqrt(tx * tx + ty * ty);
        if (tn < 0.00001) { tx = 0; ty = 0; } else { tx /= tn; ty /= tn; }
        for (uint32_t t = 0;; ++t) {
            double yaw = ru(r, gid, OR_S_RESET_YAW, t, -M_PI, M_PI);
            yaw_rot(yaw, d->rot);
            if (d->rot[0] * tx + d->rot[3] * ty >= 0.5) break;
            if (t >= 255 || tn < 0.00001 || r->overrun) break;   /* reference would loop forever */
        }
        for (int k = 0; k < 4; ++k) { d->thrust_cmds_damp[k] = 0.0; d->thrust_rot_damp[k] = 0.0; }
        d->on_floor = 0; d->crashed_floor = 0; d->crashed_wall = 0; d->crashed_ceiling = 0;
        d->prev_wall = 0; d->prev_ceiling = 0; d->prev_obst = 0;
        self_obs(p, d, r, gid, OR_S_RESET_SENSOR, obs + (size_t)i * od);
        for (int c = 0; c < 3; ++c) ev->obs_pos[i][c] = d->pos[c];
    }
    ev->tick = 0;
    ev->episode += 1;
    memset(ev->prev_pair_bits, 0, sizeof ev->prev_pair_bits);
    /* QuadrotorEnvMulti.reset zeroes the episode statistics (quadrotor_multi.py:487-509) */
    ev->st_col = ev->st_room = ev->st_floor = ev->st_wall = ev->st_ceil = ev->st_col_settle = ev->st_col_final = 0;
    ev->st_ocol = ev->st_ocol_settle = ev->st_o35 = ev->st_o5 = 0;
    for (int i = 0; i < N; ++i) {
        or_drone* d = &drones[(size_t)e * N + i];
        d->hit_agent = d->hit_obst = d->reached = d->prev_room = 0;
        memset(d->dring, 0, sizeof d->dring);
        memset(d->dsum, 0, sizeof d->dsum);
    }
    neighbor_obs(p, ev, obs, od);   /* uses fresh obs_pos and the stale obs_vel (:477) */
    if (p->use_obstacles)           /* MultiObstacles.reset (obstacles/obstacles.py:15-26) */
        for (int i = 0; i < N; ++i) or_obst_sdf(p, ev, ev->obs_pos[i], obs + (size_t)i * od + od - 9);
}

/* QuadrotorEnvMulti.step (quadrotor_multi.py:521-841) with QuadrotorSingle._step
 * (quadrotor_single.py:355-371), RawControl.step (quadrotor_control.py:53-57),
 * QuadrotorDynamics.step (quadrotor_dynamics.py:215-221), compute_reward_weighted (:34-92). */
void or_env_step(const or_params* p, or_drone* drones, or_env* envs, int e, const double* actions,
                 or_rng* r, double* obs, double* rew, unsigned char* done, double* term_obs) {
    const int N = p->num_agents, od = or_obs_dim(p);
    or_env* ev = &envs[e];
    or_drone* dr = &drones[(size_t)e * N];
    const uint32_t gbase = p->id_offset + (uint32_t)((size_t)e * N);
    const double* act = actions + (size_t)e * N * 4;
    double* o = obs + (size_t)e * N * od;
    double* rw = rew + (size_t)e * N;
    r->step = ((uint64_t)ev->episode << 32) | (uint32_t)ev->tick;   /* env Philox counter */
    const int time_remain = p->ep_len - ev->tick;                  /* QuadrotorSingle.time_remain (:361) */
    double dist_goal[OR_MAXN];

    for (int i = 0; i < N; ++i) {
        or_drone* d = &dr[i];
        uint32_t gid = gbase + (uint32_t)i;
        const double* a = act + i * 4;
        double cmds[4];
        for (int k = 0; k < 4; ++k) cmds[k] = 0.5 * (clipd(a[k], -1.0, 1.0) + 1.0);
        or_ou_noise(p, d->ou, r, gid);
        for (int s = 0; s < p->sim_steps; ++s) or_dyn_substep(p, d, cmds, d->ou, r, gid, s);
        /* reward (quadrotor_single.py:34-66) */
        double gp[3] = {d->goal[0] - d->pos[0], d->goal[1] - d->pos[1], d->goal[2] - d->pos[2]};
        dist_goal[i] = norm3(gp);
        double cost_pos = p->rew_pos * dist_goal[i];
        double an = sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2] + a[3] * a[3]);
        double cost_effort = p->rew_effort * an;
        double cost_orient = p->rew_orient * (d->on_floor ? 1.0 : -d->rot[8]);
        double cost_spin = p->rew_spin * pow(d->omega[0] * d->omega[0] + d->omega[1] * d->omega[1] + d->omega[2] * d->omega[2], 0.5);
        double cost_crash = p->rew_crash * (double)d->on_floor;
        double sum = cost_pos + cost_effort;
        sum += cost_crash; sum += cost_orient; sum += cost_spin;
        rw[i] = -p->dt * sum;
        /* compute_reward_weighted's raw terms (rew_info, quadrotor_single.py:79-105) */
        d->rinfo[OR_RI_DIST] = dist_goal[i];
        d->rinfo[OR_RI_EFFORT] = an;
        d->rinfo[OR_RI_CRASH] = (double)d->on_floor;
        d->rinfo[OR_RI_ORIENT] = d->on_floor ? 1.0 : -d->rot[8];
        d->rinfo[OR_RI_SPIN] = pow(d->omega[0] * d->omega[0] + d->omega[1] * d->omega[1] + d->omega[2] * d->omega[2], 0.5);
        if (i == 0) ev->last_floor0 = d->on_floor;
        self_obs(p, d, r, gid, OR_S_SENSOR, o + (size_t)i * od);
        for (int c = 0; c < 3; ++c) ev->obs_pos[i][c] = d->pos[c];
    }
    ev->tick += 1;
    int is_done = ev->tick > p->ep_len;

    /* 1) drone-drone collisions (quadrotor_multi.py:537-568, collisions/quadrotors.py:62-103) */
    unsigned char cur[OR_MAXN][OR_MAXN];
    memset(cur, 0, sizeof cur);
    double dist[OR_MAXN][OR_MAXN];
    int in_cur[OR_MAXN] = {0}, in_prev[OR_MAXN] = {0};
    for (int i = 0; i < N; ++i)
        for (int j = i + 1; j < N; ++j) {
            double dx = ev->obs_pos[i][0] - ev->obs_pos[j][0];
            double dy = ev->obs_pos[i][1] - ev->obs_pos[j][1];
            double dz = ev->obs_pos[i][2] - ev->obs_pos[j][2];
            dist[i][j] = pow(dx * dx + dy * dy + dz * dz, 0.5);
            if (dist[i][j] <= p->collision_threshold) { cur[i][j] = 1; in_cur[i] = in_cur[j] = 1; }
            if (ev->prev_pair_bits[i * OR_MAXN + j]) { in_prev[i] = in_prev[j] = 1; }
        }
    /* last_step_unique_collisions = setdiff1d(flat(cur), flat(prev)); penalty only if .any() */
    int any_nonzero = 0;
    for (int i = 0; i < N; ++i) if (in_cur[i] && !in_prev[i] && i != 0) any_nonzero = 1;
    double pen[OR_MAXN] = {0};
    int any_near = 0;
    double ratio = -p->rew_quadcol_smooth_max / p->collision_falloff_threshold;
    for (int i = 0; i < N; ++i)
        for (int j = i + 1; j < N; ++j)
            if (dist[i][j] <= p->collision_falloff_threshold) {
                double pe = ratio * dist[i][j] + p->rew_quadcol_smooth_max;
                pen[i] += pe; pen[j] += pe; any_near = 1;
            }
    /* 3) room (quadrotor_multi.py:390-403, 600-606) */
    int wall_new[OR_MAXN], ceil_new[OR_MAXN];
    for (int i = 0; i < N; ++i) {
        wall_new[i] = dr[i].crashed_wall && !dr[i].prev_wall;
        ceil_new[i] = dr[i].crashed_ceiling && !dr[i].prev_ceiling;
        dr[i].prev_wall = wall_new[i];
        dr[i].prev_ceiling = ceil_new[i];
    }
    /* 2) obstacles (quadrotor_multi.py:570-589): first obstacle hit per drone, new vs previous step */
    int ocol[OR_MAXN], onew[OR_MAXN];
    for (int i = 0; i < N; ++i) {
        ocol[i] = p->use_obstacles ? or_obst_detect(p, ev, ev->obs_pos[i]) : -1;
        onew[i] = ocol[i] >= 0 && !dr[i].prev_obst;
    }
    ev->last_col = any_nonzero;
    for (int i = 0; i < N; ++i) if (onew[i]) ev->last_col = 1;
    or_episode_stats_step(p, ev, dr, N, in_cur, in_prev, onew, wall_new, ceil_new, dist_goal, o, od, time_remain);
    for (int i = 0; i < N; ++i) {
        double rc = (any_nonzero && in_cur[i] && !in_prev[i]) ? -1.0 : 0.0;
        rw[i] += p->rew_quadcol_bin * rc;
        rw[i] += any_near ? -1.0 * (p->control_dt * pen[i]) : 0.0;
        if (p->use_obstacles) rw[i] += p->rew_quadcol_bin_obst * (onew[i] ? -1.0 : 0.0);
        /* the swarm terms of infos[i]["rewards"] (quadrotor_multi.py:642-651) */
        dr[i].rinfo[OR_RI_QUADCOL] = rc;
        dr[i].rinfo[OR_RI_PROX] = any_near ? -1.0 * (p->control_dt * pen[i]) : 0.0;
        dr[i].rinfo[OR_RI_OBST] = (p->use_obstacles && onew[i]) ? -1.0 : 0.0;
    }
    /* 3. random forces (quadrotor_multi.py:659-698) */
    int flag = 0;
    if (p->use_downwash) flag |= or_downwash(p, dr, N, gbase, r);
    if (p->apply_collision_force) {
        for (int i = 0; i < N; ++i)
            for (int j = i + 1; j < N; ++j)
                if (cur[i][j] && !ev->prev_pair_bits[i * OR_MAXN + j]) {
                    flag = 1;
                    or_collide_drones(dr[i].pos, dr[i].vel, dr[i].omega, dr[j].pos, dr[j].vel, dr[j].omega,
                                      r, gbase + (uint32_t)i, (uint32_t)j);
                }
        for (int i = 0; i < N; ++i)   /* 3) obstacles, curr_quad_col ascending (:680-689) */
            if (onew[i]) {
                flag = 1;
                const double op[3] = {ev->obst[ocol[i]][0], ev->obst[ocol[i]][1], p->obst_z};
                collide_obstacle_sz(or_env_obst_size(p, ev), &dr[i], op, r, gbase + (uint32_t)i);
            }
        for (int i = 0; i < N; ++i) if (wall_new[i]) { flag = 1; or_collide_wall(p, &dr[i], r, gbase + (uint32_t)i); }
        for (int i = 0; i < N; ++i) if (ceil_new[i]) { flag = 1; or_collide_ceiling(&dr[i], r, gbase + (uint32_t)i); }
    }
    for (int i = 0; i < N; ++i)
        for (int j = i + 1; j < N; ++j) ev->prev_pair_bits[i * OR_MAXN + j] = cur[i][j];
    for (int i = 0; i < N; ++i) dr[i].prev_obst = ocol[i] >= 0;
    /* 4. scenario.step() (:700-701): new goals; the observations above keep the old ones unless the
     * state-update flag makes the reference recompute them below */
    if ((p->scenario_b != OR_SC_NONE && !p->use_obstacles) || (p->use_obstacles && ev->obst_mode >= 2)) {
        or_sdraw sd;
        memset(&sd, 0, sizeof sd);
        sd.mode = OR_RNG_PHILOX; sd.seed = r->seed; sd.key = gbase; sd.stream = OR_S_SCN; sd.step = r->step;
        double g[OR_MAXN][3];
        for (int i = 0; i < N; ++i) memcpy(g[i], dr[i].goal, sizeof g[i]);
        if (p->use_obstacles) {   /* the map back from the pillar centres (or_cell_xy's inverse) */
            const int n = p->obst_area;
            const double h = (double)(n / 2);
            unsigned char map[64 * 64];
            memset(map, 0, sizeof map);
            for (int o = 0; o < ev->n_obst; ++o) {
                const int col = (int)lround(ev->obst[o][0] - 0.5 + h), row = n - 1 - (int)lround(ev->obst[o][1] - 0.5 + h);
                map[row * n + col] = 1;
            }
            or_oscen_step(p, &ev->scen, ev->tick, &sd, map, n, g);
        } else {
            or_scen_step(p, &ev->scen, ev->tick, &sd, g);
        }
        for (int i = 0; i < N; ++i) memcpy(dr[i].goal, g[i], sizeof g[i]);
    }
    /* 5. refresh and observations (:704-716) */
    for (int i = 0; i < N; ++i)
        for (int c = 0; c < 3; ++c) { ev->obs_pos[i][c] = dr[i].pos[c]; ev->obs_vel[i][c] = dr[i].vel[c]; }
    if (flag)
        for (int i = 0; i < N; ++i) self_obs(p, &dr[i], r, gbase + (uint32_t)i, OR_S_SENSOR, o + (size_t)i * od);
    neighbor_obs(p, ev, o, od);
    if (p->use_obstacles)   /* MultiObstacles.step (obstacles/obstacles.py:28-35) */
        for (int i = 0; i < N; ++i) or_obst_sdf(p, ev, ev->obs_pos[i], o + (size_t)i * od + od - 9);
    for (int i = 0; i < N; ++i) done[(size_t)e * N + i] = (unsigned char)is_done;
    if (is_done) {
        or_episode_stats_done(p, ev, dr, N);
        if (term_obs) memcpy(term_obs + (size_t)e * N * od, o, sizeof(double) * (size_t)N * od);
        ev->tick -= 1;                              /* the reset draws at the step's counter */
        or_env_reset(p, drones, envs, e, r, o);     /* in-env auto reset (:836) */
    }
}

void or_reset_all(const or_params* p, or_drone* drones, or_env* envs, uint32_t seed, double* obs) {
    const int od = or_obs_dim(p);
    for (int e = 0; e < p->num_envs; ++e) {
        or_rng r;
        memset(&r, 0, sizeof r);
        r.mode = OR_RNG_PHILOX; r.seed = seed;
        or_env_reset(p, drones, envs, e, &r, obs + (size_t)e * p->num_agents * od);
    }
}

void or_step_all(const or_params* p, or_drone* drones, or_env* envs, const double* actions, uint32_t seed,
                 double* obs, double* rew, unsigned char* done, double* term_obs, int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(static)
#endif
    for (int e = 0; e < p->num_envs; ++e) {
        or_rng r;
        memset(&r, 0, sizeof r);
        r.mode = OR_RNG_PHILOX; r.seed = seed;
        or_env_step(p, drones, envs, e, actions, &r, obs, rew, done, term_obs);
    }
    (void)nthreads;
}

void or_neighbor_obs(const or_params* p, const or_env* ev, double* obs, int obs_dim) {
    neighbor_obs(p, ev, obs, obs_dim);
}

int or_sizeof_params(void) { return (int)sizeof(or_params); }
int or_sizeof_drone(void) { return (int)sizeof(or_drone); }
int or_sizeof_env(void) { return (int)sizeof(or_env); }
int or_sizeof_rng(void) { return (int)sizeof(or_rng); }
