/* quadswarm_oracle_a.c -- CPU restatement of the reference's flavor-A swarm env step.
 *
 * TEST INFRASTRUCTURE ONLY (parity oracle and cpu_baseline "port"); the product never links it.
 *
 * Flavor A is what swarm_rl.sb_train trains on (sb3_quad_env.py:34-41):
 *   QuadrotorEnvMulti.step / reset     gym_art/quadrotor_multi/quadrotor_multi_rewards.py:541-991
 *   QuadrotorSingle._step / _reset     quadrotor_single_rewards.py:418-452 / :480-549
 *   Controller.update_vel_height_dir   Controller/Controller.py:76-101 and the Position / Velocity /
 *                                      Acceleration / Attitude / Rate controllers, Mixer, Pid.py
 *   CustomPidControl.step              quadrotor_control.py:90-94
 *   state_* (flavor-A reprs)           get_state.py:7-223
 *   neighbour obs + camera model       quadrotor_multi_rewards.py:238-476
 *   Scenario_dynamic_repulsive         scenarios/dynamic_repulsive.py:37-74 (float-fixed)
 * The physics under the controller is the same QuadrotorDynamics.step as flavor B
 * (or_ou_noise + or_dyn_substep in quadswarm_oracle.c).  float64 throughout, like the reference.
 */
#include <math.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "quadswarm_oracle.h"

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

static inline double clipd(double x, double lo, double hi) { return x < lo ? lo : (x > hi ? hi : x); }

/* Python / numpy float modulo (result has the divisor's sign) */
static double pymod(double x, double y) {
    double m = fmod(x, y);
    if (m != 0.0) {
        if ((y < 0) != (m < 0)) m += y;
    } else {
        m = copysign(0.0, y);
    }
    return m;
}
static inline double wrap_pi(double x) { return pymod(x + M_PI, 2 * M_PI) - M_PI; }
static inline double npsign(double x) { return x > 0 ? 1.0 : (x < 0 ? -1.0 : (x == x ? 0.0 : x)); }
/* np.nan_to_num(x, nan=0.0) */
static inline double nan_to_num(double x) {
    if (x != x) return 0.0;
    if (isinf(x)) return x > 0 ? 1.7976931348623157e308 : -1.7976931348623157e308;
    return x;
}

/* ------------------------------------------------------------------------------------------ */
/* constants                                                                                   */
/* ------------------------------------------------------------------------------------------ */
/* 4x4 inverse by Gauss-Jordan with partial pivoting (Mixer.calculate_allocation uses the
 * pseudo-inverse A^T (A A^T)^-1 of the square, invertible allocation matrix == A^-1) */
static int inv4(const double* a, double* out) {
    double m[4][8];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 8; ++j) m[i][j] = j < 4 ? a[i * 4 + j] : (j - 4 == i ? 1.0 : 0.0);
    for (int c = 0; c < 4; ++c) {
        int piv = c;
        for (int r = c + 1; r < 4; ++r)
            if (fabs(m[r][c]) > fabs(m[piv][c])) piv = r;
        if (m[piv][c] == 0.0) return -1;
        if (piv != c)
            for (int j = 0; j < 8; ++j) { double t = m[c][j]; m[c][j] = m[piv][j]; m[piv][j] = t; }
        double d = m[c][c];
        for (int j = 0; j < 8; ++j) m[c][j] /= d;
        for (int r = 0; r < 4; ++r)
            if (r != c) {
                double f = m[r][c];
                for (int j = 0; j < 8; ++j) m[r][j] -= f * m[c][j];
            }
    }
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) out[i * 4 + j] = m[i][4 + j];
    return 0;
}

void or_params_default_a(or_params* p) {
    or_params_default(p);
    p->flavor = 1;
    /* swarm_rl/global_cfg.py defaults (room 15x15x3, 30 s episodes) */
    p->room_lo[0] = -7.5; p->room_lo[1] = -7.5; p->room_lo[2] = 0.0;
    p->room_hi[0] = 7.5; p->room_hi[1] = 7.5; p->room_hi[2] = 3.0;
    p->ep_len = 3000;
    p->num_agents = 4;
    p->k_neighbors = 3;
    p->obs_repr_a = OR_OA_CDIST_SANGLE;
    p->nfeat = OR_NF_NDIST | OR_NF_NSANGLE;
    p->nfeat_dim = 3;
    p->ticks_per_step = 8;
    p->scenario_a = 1;
    p->nclip_lo[0] = -7.5; p->nclip_hi[0] = 7.5;
    for (int i = 1; i < 8; ++i) { p->nclip_lo[i] = -1.0; p->nclip_hi[i] = 1.0; }
    p->apply_collision_force = 0;   /* quadrotor_multi_rewards.py:203 */
    /* camera (global_cfg.py:14-18; simulate_camera_measurement_vect defaults fov 70, 640 px) */
    p->cam_size = 0.2; p->cam_focal = 0.035; p->cam_px_noise = 3.0; p->cam_fov_deg = 70.0; p->cam_res = 640.0;
    p->n_cameras = 3;
    /* Controller (Controller.py:24-29) */
    p->heading_rate = M_PI * 80 / 180;
    p->speed = 0.2;
    /* ModelParams defaults (MultirotorModel.py:10-50) */
    p->m_n_motors = 4; p->m_g = 9.81; p->m_mass = 0.028; p->m_kf = 0.00000000125;
    p->m_min_rpm = 1170.0; p->m_max_rpm = 13000;
    const double km = 0.0025, prop_r = 0.00015, arm = 0.04596, bh = 0.003, m = p->m_mass;
    const double Jd[3] = {m * (3.0 * arm * arm + bh * bh) / 12.0, m * (3.0 * arm * arm + bh * bh) / 12.0,
                          (m * arm * arm) / 2.0};
    /* PID gains: PositionController.py:13-19,51-56 (z only), VelocityController.py:19-26,57-66,
     * AttitudeController.py:11-18,45-55, RateController.py:11-17,48-66 (gains x J) */
    for (int k = 0; k < OR_NPID; ++k) {
        if (k == OR_PID_POS_Z) { p->pid_kp[k] = 4.1625; p->pid_kd[k] = 0.5473; p->pid_ki[k] = 0.0023; p->pid_sat[k] = 6.0; p->pid_aw[k] = 2.0; }
        else if (k < OR_PID_ATT) { p->pid_kp[k] = 2.4531; p->pid_kd[k] = 0.0003; p->pid_ki[k] = 0.0382; p->pid_sat[k] = 40.0; p->pid_aw[k] = 1.0; }
        else if (k < OR_PID_RATE) {
            p->pid_kp[k] = 11.2081; p->pid_kd[k] = 0.0490; p->pid_ki[k] = 0.0073;
            p->pid_sat[k] = (k == OR_PID_ATT + 2) ? 1.0 : 10.0; p->pid_aw[k] = 0.1;
        } else {
            const double J = Jd[k - OR_PID_RATE];
            p->pid_kp[k] = 3.1222 * J; p->pid_kd[k] = 0.0477 * J; p->pid_ki[k] = 0.0001 * J;
            p->pid_sat[k] = -1; p->pid_aw[k] = 1.0;
        }
    }
    p->rate_out_scale = 800.0;
    /* Mixer.calculate_allocation (Mixer.py:31-66) */
    double alloc[16] = {-0.707, 0.707, 0.707, -0.707, -0.707, 0.707, -0.707, 0.707,
                        -1.0, -1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0};
    for (int j = 0; j < 4; ++j) {
        alloc[0 * 4 + j] *= arm * p->m_kf;
        alloc[1 * 4 + j] *= arm * p->m_kf;
        alloc[2 * 4 + j] *= km * (3.0 * prop_r) * p->m_kf;
        alloc[3 * 4 + j] *= p->m_kf;
    }
    double inv[16];
    inv4(alloc, inv);
    for (int i = 0; i < 4; ++i) {
        double n = sqrt(inv[i * 4 + 0] * inv[i * 4 + 0] + inv[i * 4 + 1] * inv[i * 4 + 1]);
        if (n > 0) { inv[i * 4 + 0] /= n; inv[i * 4 + 1] /= n; }
        double v = inv[i * 4 + 2];
        inv[i * 4 + 2] = v > 1e-2 ? 1.0 : (v < -1e-2 ? -1.0 : 0.0);
        inv[i * 4 + 3] = 1.0;
    }
    memcpy(p->mixer, inv, sizeof inv);
    /* rewards (quadrotor_multi_rewards.py:716-724) */
    p->w_captor = 100; p->w_helper = 100; p->existence = -0.1;
    /* Scenario_dynamic_repulsive (scenarios/dynamic_repulsive.py:29-35, 52-55) */
    p->target_vmax = 0.5; p->target_dt = 1.0 / 200; p->arena_size = 5; p->target_z = 2;
}

int or_obs_dim_a(const or_params* p) {
    const int so = (p->obs_repr_a == OR_OA_CDIST_SANGLE || p->obs_repr_a == OR_OA_CDIST_NDIST_NSANGLE) ? 7 : 6;
    return so + p->k_neighbors * p->nfeat_dim;
}
static int self_dim_a(const or_params* p) { return or_obs_dim_a(p) - p->k_neighbors * p->nfeat_dim; }

/* ------------------------------------------------------------------------------------------ */
/* Controller                                                                                  */
/* ------------------------------------------------------------------------------------------ */
/* _pid_update_numba (Controller/Pid.py:6-26) */
double or_pid_update(double error, double* last_error, double* integral, double dt, double kp, double kd,
                     double ki, double sat, double aw) {
    double difference = (error - *last_error) / dt;
    *last_error = error;
    double output = kp * error + kd * difference + ki * (*integral);
    if (sat > 0) {
        if (output >= sat) output = sat;
        else if (output <= -sat) output = -sat;
    }
    if (aw > 0) {
        if (-aw < output && output < aw) *integral += error * dt;
    }
    return output;
}

static double pid(const or_params* p, or_drone* d, int k, double e, double dt) {
    return or_pid_update(e, &d->pid[2 * k], &d->pid[2 * k + 1], dt, p->pid_kp[k], p->pid_kd[k], p->pid_ki[k],
                         p->pid_sat[k], p->pid_aw[k]);
}

/* Controller.update_vel_height_dir (Controller.py:76-101): returns Mixer output (motors in [0,1]-ish).
 * The position PIDs for x and y run in the reference too, but their outputs are overwritten by the
 * heading velocity (:90) and their state never reaches any output, so they are not carried. */
void or_ctrl_a(const or_params* p, or_drone* d, double cmd0, double height, double motors[4]) {
    const double dt = p->dt;
    d->ang_vel = cmd0;
    d->angle = d->angle + d->ang_vel * dt * p->heading_rate;
    d->angle = pymod(d->angle + M_PI, 2 * M_PI) - M_PI;
    const double dir0 = cos(d->angle), dir1 = sin(d->angle);
    /* PositionController.get_control_signal (PositionController.py:62-77), z axis */
    double vz = pid(p, d, OR_PID_POS_Z, height - d->pos[2], dt);
    double vref[3] = {dir0 * p->speed, dir1 * p->speed, vz};
    /* VelocityController.get_control_signal (VelocityController.py:68-83) */
    double acc[3];
    for (int i = 0; i < 3; ++i) acc[i] = pid(p, d, OR_PID_VEL + i, vref[i] - d->vel[i], dt);
    /* AccelerationController.get_control_signal (AccelerationController.py:18-108), heading 0 */
    double fd[3] = {(acc[0] + 0.0) * p->m_mass, (acc[1] + 0.0) * p->m_mass, (acc[2] + p->m_g) * p->m_mass};
    double fn_ = sqrt(fd[0] * fd[0] + fd[1] * fd[1] + fd[2] * fd[2]);
    double n[3] = {fd[0] / fn_, fd[1] / fn_, fd[2] / fn_};
    double A2[3][2] = {{1.0 - n[0] * n[0], -n[0] * n[1]}, {-n[1] * n[0], 1.0 - n[1] * n[1]}, {-n[2] * n[0], -n[2] * n[1]}};
    double det2 = A2[0][0] * A2[1][1] - A2[0][1] * A2[1][0];
    double Binv[2][2] = {{A2[1][1] / det2, -A2[0][1] / det2}, {-A2[1][0] / det2, A2[0][0] / det2}};
    const double bxd0 = cos(0.0), bxd1 = sin(0.0);
    double co[2] = {Binv[0][0] * bxd0 + Binv[0][1] * bxd1, Binv[1][0] * bxd0 + Binv[1][1] * bxd1};
    double x[3];
    for (int i = 0; i < 3; ++i) x[i] = A2[i][0] * co[0] + A2[i][1] * co[1];
    double xn = sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]);
    for (int i = 0; i < 3; ++i) x[i] /= xn;
    double y[3] = {n[1] * x[2] - n[2] * x[1], n[2] * x[0] - n[0] * x[2], n[0] * x[1] - n[1] * x[0]};
    double yn = sqrt(y[0] * y[0] + y[1] * y[1] + y[2] * y[2]);
    for (int i = 0; i < 3; ++i) y[i] /= yn;
    double Rd[9] = {x[0], y[0], n[0], x[1], y[1], n[1], x[2], y[2], n[2]};
    const double* R = d->rot;
    double tf = fd[0] * R[2] + fd[1] * R[5] + fd[2] * R[8];
    tf = tf > 0 ? tf : 0;
    double throttle = (sqrt(tf / (p->m_kf * p->m_n_motors)) - p->m_min_rpm) / (p->m_max_rpm - p->m_min_rpm);
    throttle = throttle < 0.0 ? 0.0 : (throttle > 1.0 ? 1.0 : throttle);
    /* AttitudeController.get_control_signal (AttitudeController.py:60-82) */
    double E[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double a = 0, b = 0;
            for (int k = 0; k < 3; ++k) {
                a += Rd[k * 3 + i] * R[k * 3 + j];   /* (Rd^T R)_ij */
                b += R[k * 3 + i] * Rd[k * 3 + j];   /* (R^T Rd)_ij */
            }
            E[i * 3 + j] = 0.5 * (a - b);
        }
    double ev[3] = {(E[1 * 3 + 2] - E[2 * 3 + 1]) / 2.0, (E[2 * 3 + 0] - E[0 * 3 + 2]) / 2.0,
                    (E[0 * 3 + 1] - E[1 * 3 + 0]) / 2.0};
    double rate[3];
    for (int i = 0; i < 3; ++i) rate[i] = pid(p, d, OR_PID_ATT + i, ev[i], dt);
    /* RateController.get_control_signal (RateController.py:71-89) */
    double cg[4];
    for (int i = 0; i < 3; ++i) cg[i] = pid(p, d, OR_PID_RATE + i, rate[i] - d->omega[i], dt) * p->rate_out_scale;
    cg[3] = throttle;
    /* Mixer.get_control_signal (Mixer.py:70-111) with desaturation */
    const double* M = p->mixer;
    double mo[4];
    for (int i = 0; i < 4; ++i) mo[i] = M[i * 4 + 0] * cg[0] + M[i * 4 + 1] * cg[1] + M[i * 4 + 2] * cg[2] + M[i * 4 + 3] * cg[3];
    double mn = mo[0];
    for (int i = 1; i < 4; ++i) mn = mo[i] < mn ? mo[i] : mn;
    if (mn < 0.0)
        for (int i = 0; i < 4; ++i) mo[i] = mo[i] + fabs(mn);
    double mx = mo[0];
    for (int i = 1; i < 4; ++i) mx = mo[i] > mx ? mo[i] : mx;
    if (mx > 1.0) {
        if (cg[3] > 1e-2) {
            double scale = (mo[0] + ((mo[1] + mo[2]) + mo[3])) / 4.0 / cg[3];   /* np.mean: a0 + pairwise(a1..) */
            for (int i = 0; i < 3; ++i) cg[i] /= scale;
            for (int i = 0; i < 4; ++i) mo[i] = M[i * 4 + 0] * cg[0] + M[i * 4 + 1] * cg[1] + M[i * 4 + 2] * cg[2] + M[i * 4 + 3] * cg[3];
        } else {
            for (int i = 0; i < 4; ++i) mo[i] = mo[i] / mx;
        }
    }
    memcpy(motors, mo, sizeof mo);
}

/* QuadrotorSingle._step (quadrotor_single_rewards.py:436-441) + CustomPidControl.step
 * (quadrotor_control.py:90-94): reorder [0,3,1,2], x2-1, arctan, clip [-1,1], 0.5(a+1) */
void or_motors_to_cmds(const double m[4], double u[4]) {
    const double re[4] = {m[0], m[3], m[1], m[2]};
    for (int k = 0; k < 4; ++k) u[k] = 0.5 * (clipd(atan(re[k] * 2 - 1), -1.0, 1.0) + 1.0);
}

/* ------------------------------------------------------------------------------------------ */
/* camera model: simulate_camera_measurement_vect (get_state.py:128-176,                      */
/* quadrotor_multi_rewards.py:275-324) + circle_intersection_vect + get_camera_angle           */
/* n1, n2: the pixel noise added to u1_px / u2_px                                              */
/* ------------------------------------------------------------------------------------------ */
void or_camera(const or_params* p, double rx, double ry, double ga, double n1, double n2, double* dist,
               double* angle) {
    double c = cos(-ga), s = sin(-ga);
    double rp0 = c * rx - s * ry, rp1 = s * rx + c * ry;
    double ao = atan2(rp1, rp0);
    const double nc = (double)p->n_cameras;
    double idx = nearbyint(pymod(ao, 2 * M_PI) / (2 * M_PI / nc));
    long ci = (long)idx % (long)p->n_cameras;
    double cam = (double)ci * 2 * M_PI / nc;
    c = cos(-cam); s = sin(-cam);
    double c0 = c * rp0 - s * rp1, c1 = s * rp0 + c * rp1;
    double r = p->cam_size / 2, f = p->cam_focal;
    double w = 2 * tan((p->cam_fov_deg / 2) * M_PI / 180) * f;
    /* circle_intersection_vect(center, r, center/2, |center|/2) */
    double h0 = c0 / 2, h1 = c1 / 2;
    double r2 = sqrt(c0 * c0 + c1 * c1) / 2;
    double dd0 = h0 - c0, dd1 = h1 - c1;
    double d = sqrt(dd0 * dd0 + dd1 * dd1);
    double a = (r * r - r2 * r2 + d * d) / (2 * d);
    double h = sqrt(r * r - a * a);
    double rad0 = dd0 / d, rad1 = dd1 / d;
    double mid0 = c0 + a * rad0, mid1 = c1 + a * rad1;
    double pe0 = -rad1, pe1 = rad0;
    double x10 = mid0 + h * pe0, x11 = mid1 + h * pe1;
    double x20 = mid0 - h * pe0, x21 = mid1 - h * pe1;
    double u1 = x11 * f / x10, u2 = x21 * f / x20;
    double u1p = u1 * p->cam_res / w + n1, u2p = u2 * p->cam_res / w + n2;
    u1 = u1p * w / p->cam_res;
    u2 = u2p * w / p->cam_res;
    double at1 = atan(u1 / f), at2 = atan(u2 / f);
    double alpha = fabs(at1 - at2);
    double l = r / sin(alpha / 2);
    double acam = (at1 + at2) / 2;
    double arel = wrap_pi(acam + cam);
    *dist = nan_to_num(l);
    *angle = nan_to_num(arel);
}

static void cam_noise(const or_params* p, or_rng* r, uint32_t gid, uint32_t st, double* n1, double* n2) {
    if (r->mode == OR_RNG_TAPE) {
        *n1 = or_rn(r, gid, st, 0, 0.0, p->cam_px_noise);
        *n2 = or_rn(r, gid, st, 1, 0.0, p->cam_px_noise);
    } else if (p->cam_px_noise != 0.0) {
        *n1 = or_rn(r, gid, st, 0, 0.0, p->cam_px_noise);
        *n2 = or_rn(r, gid, st, 1, 0.0, p->cam_px_noise);
    } else {
        *n1 = 0.0; *n2 = 0.0;
    }
}

/* ------------------------------------------------------------------------------------------ */
/* self observation (get_state.py:7-223) with sensor noise (sensor_noise.py:172-261)           */
/* ------------------------------------------------------------------------------------------ */
void or_self_obs_a(const or_params* p, const or_drone* d, or_rng* r, uint32_t gid, uint32_t st_sensor,
                   uint32_t st_cam, double* out) {
    double np_[3], nv[3], nr[9], no[3];
    or_sensor_noise(p, d->pos, d->vel, d->rot, d->omega, r, gid, st_sensor, np_, nv, nr, no);
    const double dt = p->dt;
    double rp0 = d->goal[0] - np_[0], rp1 = d->goal[1] - np_[1];
    double rel_dist = sqrt(rp0 * rp0 + rp1 * rp1);
    double q0 = rp0 + nv[0] * dt, q1 = rp1 + nv[1] * dt;
    double dot_rel = (sqrt(q0 * q0 + q1 * q1) - rel_dist) / dt;
    double angle_world = d->angle;
    double rn0 = rp0 / rel_dist, rn1 = rp1 / rel_dist;
    double rel_angle = wrap_pi(atan2(rn1, rn0) - angle_world);
    double av = d->ang_vel;
    double angledot = -npsign(av * rel_angle) * fabs(av);
    if (p->obs_repr_a == OR_OA_AW) {
        out[0] = angle_world; out[1] = av; out[2] = rel_dist; out[3] = dot_rel; out[4] = rel_angle; out[5] = angledot;
        return;
    }
    double cd = sqrt(np_[0] * np_[0] + np_[1] * np_[1]);
    double c0 = np_[0] + nv[0] * dt, c1 = np_[1] + nv[1] * dt;
    double cdd = (sqrt(c0 * c0 + c1 * c1) - cd) / dt;
    out[0] = cd; out[1] = cdd; out[3] = dot_rel;
    if (p->obs_repr_a == OR_OA_CDIST_ANGLE) {
        out[2] = rel_dist; out[4] = rel_angle; out[5] = angledot;
    } else if (p->obs_repr_a == OR_OA_CDIST_SANGLE) {
        out[2] = rel_dist; out[4] = cos(rel_angle); out[5] = sin(rel_angle); out[6] = angledot;
    } else {
        double n1, n2, nd, na;
        cam_noise(p, r, gid, st_cam, &n1, &n2);
        or_camera(p, rp0, rp1, angle_world, n1, n2, &nd, &na);
        out[2] = clipd(nd, 0.0, 10.0); out[4] = cos(na); out[5] = sin(na); out[6] = angledot;
    }
}

/* ------------------------------------------------------------------------------------------ */
/* neighbour obs (quadrotor_multi_rewards.py:326-476)                                          */
/* ------------------------------------------------------------------------------------------ */
/* Test hooks (tests/parity_utils.py, per-feature conditioning of the GPU-vs-oracle comparison): when set,
 * the obs pass of or_neighbor_obs_a records the inputs of every (drone, slot) feature block in
 * or_nb_trace[(gid * OR_MAXN + slot) * OR_NB_TRACE_W] = {j, n1, n2, pr[3], vr[3], aw, h_i, h_j}, and the
 * selection pass the sort key of every candidate j in or_key_trace[gid * OR_MAXN + j]; the *_reset pair gets the passes of
 * the resets (the obs a finished env returns), the other pair those of the step (its terminal obs). */
double* or_nb_trace = NULL;
double* or_key_trace = NULL;
double* or_nb_trace_reset = NULL;
double* or_key_trace_reset = NULL;

/* get_rel_pos_vel_item for one (i, j) pair on explicit inputs: pr = pos_j - pos_i, aw = own heading angle,
 * hi / hj = the stale headings, vr = vel_j - vel_i; features in the reference's concatenation order */
int or_rel_features_x(const or_params* p, const double pr[3], double aw, double hi, double hj, const double vr[3],
                      double n1, double n2, double* f) {
    const int m = p->nfeat;
    double pn = sqrt(pr[0] * pr[0] + pr[1] * pr[1] + pr[2] * pr[2]);
    int n = 0;
    double nd = 0, na = 0;
    if (m & OR_NF_DIST) f[n++] = pn;
    if (m & OR_NF_NDIST) {
        or_camera(p, pr[0], pr[1], aw, n1, n2, &nd, &na);
        f[n++] = clipd(nd, 0.0, 10.0);
    }
    if (m & (OR_NF_ANGLE | OR_NF_SANGLE)) {
        double ra = wrap_pi(atan2(pr[1] / pn, pr[0] / pn) - aw);
        if (m & OR_NF_ANGLE) f[n++] = ra;
        if (m & OR_NF_SANGLE) { f[n++] = cos(ra); f[n++] = sin(ra); }
    }
    if (m & OR_NF_NSANGLE) { f[n++] = cos(na); f[n++] = sin(na); }
    if (m & (OR_NF_HEADING | OR_NF_SHEADING)) {
        double rh = wrap_pi(hj - hi);
        if (m & OR_NF_HEADING) f[n++] = rh;
        if (m & OR_NF_SHEADING) { f[n++] = cos(rh); f[n++] = sin(rh); }
    }
    if (m & OR_NF_NPOS) for (int c = 0; c < 3; ++c) f[n++] = pr[c];
    if (m & OR_NF_POS) for (int c = 0; c < 3; ++c) f[n++] = pr[c];
    if (m & OR_NF_VEL) for (int c = 0; c < 3; ++c) f[n++] = vr[c];
    return n;
}

static int rel_features(const or_params* p, const or_env* ev, const or_drone* dr, int i, int j, double n1,
                        double n2, double* f) {
    double pr[3], vr[3];
    for (int c = 0; c < 3; ++c) {
        pr[c] = ev->obs_pos[j][c] - ev->obs_pos[i][c];
        vr[c] = ev->obs_vel[j][c] - ev->obs_vel[i][c];
    }
    return or_rel_features_x(p, pr, dr[i].angle, ev->heading[i], ev->heading[j], vr, n1, n2, f);
}

/* neighborhood_indices (:445-476) + extend_obs_space (:422-443) with the clip box.  The camera is
 * evaluated twice when k < N-1 (selection pass, then obs pass on the selected ones), each with its
 * own pixel noise, like the reference.  In tape mode the draws come in the reference's order:
 * per drone, all u1 then all u2 of the pass (np.random.normal(size=n) twice). */
void or_neighbor_obs_a(const or_params* p, const or_env* ev, const or_drone* dr, or_rng* r, uint32_t gbase,
                       int reset, double* obs, int od) {
    const int N = p->num_agents, K = p->k_neighbors, F = p->nfeat_dim, so = self_dim_a(p);
    if (K <= 0) return;
    const int cam = (p->nfeat & OR_NF_NDIST) != 0;
    double* nbt = reset ? or_nb_trace_reset : or_nb_trace;
    double* kt = reset ? or_key_trace_reset : or_key_trace;
    const uint32_t st_obs = reset ? OR_S_RESET_CAM : OR_S_CAM, st_sel = reset ? OR_S_RESET_CAM_SEL : OR_S_CAM_SEL;
    int sel[OR_MAXN][OR_MAXN];
    for (int i = 0; i < N; ++i) {
        int c = 0;
        for (int j = 0; j < N; ++j) if (j != i) sel[i][c++] = j;
    }
    if (K < N - 1) {
        for (int i = 0; i < N; ++i) {
            double n1[OR_MAXN] = {0}, n2[OR_MAXN] = {0}, key[OR_MAXN];
            if (cam) {
                for (int c = 0; c < N - 1; ++c) cam_noise(p, r, gbase + (uint32_t)i, st_sel | ((uint32_t)sel[i][c] << 8), &n1[c], &n2[c]);
                if (r->mode == OR_RNG_TAPE) {   /* tape: n1 of all pairs, then n2 of all pairs */
                    double t[2 * OR_MAXN];
                    for (int c = 0; c < N - 1; ++c) { t[2 * c] = n1[c]; t[2 * c + 1] = n2[c]; }
                    for (int c = 0; c < N - 1; ++c) { n1[c] = t[c]; n2[c] = t[N - 1 + c]; }
                }
            }
            for (int c = 0; c < N - 1; ++c) {
                double f[8];
                int nf = rel_features(p, ev, dr, i, sel[i][c], n1[c], n2[c], f);
                double s = 0;
                for (int q = 0; q < nf; ++q) s += f[q] * f[q];
                double k = sqrt(s);
                key[c] = k > 0.01 ? k : (k == k ? 0.01 : k);
                if (kt) kt[(size_t)(gbase + (uint32_t)i) * OR_MAXN + sel[i][c]] = key[c];
            }
            /* argsort (insertion sort: stable; NaN sorts last) */
            int order[OR_MAXN];
            for (int c = 0; c < N - 1; ++c) order[c] = c;
            for (int a = 1; a < N - 1; ++a) {
                int v = order[a], b = a - 1;
                while (b >= 0 && (key[order[b]] > key[v] || (key[order[b]] != key[order[b]] && key[v] == key[v]))) {
                    order[b + 1] = order[b];
                    --b;
                }
                order[b + 1] = v;
            }
            int tmp[OR_MAXN];
            for (int c = 0; c < K; ++c) tmp[c] = sel[i][order[c]];
            for (int c = 0; c < K; ++c) sel[i][c] = tmp[c];
        }
    }
    for (int i = 0; i < N; ++i) {
        double n1[OR_MAXN] = {0}, n2[OR_MAXN] = {0};
        if (cam) {
            for (int c = 0; c < K; ++c) cam_noise(p, r, gbase + (uint32_t)i, st_obs | ((uint32_t)sel[i][c] << 8), &n1[c], &n2[c]);
            if (r->mode == OR_RNG_TAPE) {
                double t[2 * OR_MAXN];
                for (int c = 0; c < K; ++c) { t[2 * c] = n1[c]; t[2 * c + 1] = n2[c]; }
                for (int c = 0; c < K; ++c) { n1[c] = t[c]; n2[c] = t[K + c]; }
            }
        }
        double* o = obs + (size_t)i * od + so;
        for (int c = 0; c < K; ++c) {
            double f[8];
            if (nbt) {
                const int j = sel[i][c];
                double* t = nbt + ((size_t)(gbase + (uint32_t)i) * OR_MAXN + c) * OR_NB_TRACE_W;
                t[0] = j; t[1] = n1[c]; t[2] = n2[c];
                for (int q = 0; q < 3; ++q) {
                    t[3 + q] = ev->obs_pos[j][q] - ev->obs_pos[i][q];
                    t[6 + q] = ev->obs_vel[j][q] - ev->obs_vel[i][q];
                }
                t[9] = dr[i].angle; t[10] = ev->heading[i]; t[11] = ev->heading[j];
            }
            rel_features(p, ev, dr, i, sel[i][c], n1[c], n2[c], f);
            for (int q = 0; q < F; ++q) o[c * F + q] = clipd(f[q], p->nclip_lo[q], p->nclip_hi[q]);
        }
    }
}

/* ------------------------------------------------------------------------------------------ */
/* Scenario_dynamic_repulsive.step (scenarios/dynamic_repulsive.py:37-62)                      */
/* ------------------------------------------------------------------------------------------ */
void or_target_step(const or_params* p, or_env* ev, or_drone* dr) {
    const int N = p->num_agents;
    double af0 = 0, af1 = 0;
    if (ev->has_pos)
        for (int i = 0; i < N; ++i) {
            double r0 = -(dr[i].pos[0] - ev->target[0]), r1 = -(dr[i].pos[1] - ev->target[1]);
            double d = sqrt(r0 * r0 + r1 * r1);
            af0 += r0 / (d * d);
            af1 += r1 / (d * d);
        }
    double de = sqrt(ev->target[0] * ev->target[0] + ev->target[1] * ev->target[1]);
    double den = de * (p->arena_size - de > 0.1 ? p->arena_size - de : 0.1);
    double v0 = af0 + -ev->target[0] / den, v1 = af1 + -ev->target[1] / den;
    double vs = sqrt(v0 * v0 + v1 * v1);
    double m = vs < p->target_vmax ? vs : p->target_vmax;
    ev->target[0] = ev->target[0] + (v0 / vs) * m * p->target_dt;
    ev->target[1] = ev->target[1] + (v1 / vs) * m * p->target_dt;
    double z = p->target_z > 0.25 ? p->target_z : 0.25;
    for (int i = 0; i < N; ++i) {   /* generate_goals with formation size 0 (scenarios/base.py:41-66) */
        dr[i].goal[0] = ev->target[0]; dr[i].goal[1] = ev->target[1]; dr[i].goal[2] = z;
    }
}

/* ------------------------------------------------------------------------------------------ */
/* reset: QuadrotorEnvMulti.reset (quadrotor_multi_rewards.py:541-627) with                    */
/* Scenario_dynamic_repulsive.reset (dynamic_repulsive.py:64-74) and QuadrotorSingle._reset     */
/* (quadrotor_single_rewards.py:480-549)                                                       */
/* ------------------------------------------------------------------------------------------ */
void or_env_reset_a(const or_params* p, or_drone* drones, or_env* envs, int e, or_rng* r, double* obs,
                    unsigned char* reset_info) {
    const int N = p->num_agents, od = or_obs_dim_a(p);
    or_env* ev = &envs[e];
    or_drone* dr = &drones[(size_t)e * N];
    const uint32_t gbase = p->id_offset + (uint32_t)((size_t)e * N);
    r->step = ((uint64_t)ev->episode << 32) | (uint32_t)ev->tick;
    const int tape = r->mode == OR_RNG_TAPE;
    if (p->scenario_a == 1) {
        double dirs[OR_MAXN][2], rad, t0, t1, tr;
        if (tape) {
            for (int k = 0; k < 4; ++k) (void)or_gnext(r);   /* duration, formation, size, layer dist */
            for (int i = 0; i < N; ++i) { dirs[i][0] = or_gnext(r); dirs[i][1] = or_gnext(r); }
            rad = or_gnext(r); t0 = or_gnext(r); t1 = or_gnext(r); tr = or_gnext(r);
        } else {
            for (int i = 0; i < N; ++i) {
                dirs[i][0] = or_ru(r, gbase + (uint32_t)i, OR_S_RESET_A, 0, 0.0, 1.0);
                dirs[i][1] = or_ru(r, gbase + (uint32_t)i, OR_S_RESET_A, 1, 0.0, 1.0);
            }
            rad = or_ru(r, gbase, OR_S_SCEN, 0, 0.0, 1.0);
            t0 = or_ru(r, gbase, OR_S_SCEN, 1, 0.0, 1.0);
            t1 = or_ru(r, gbase, OR_S_SCEN, 2, 0.0, 1.0);
            tr = or_ru(r, gbase, OR_S_SCEN, 3, 0.0, 1.0);
        }
        double sp[OR_MAXN][2];   /* spawn_points[:, :2] */
        for (int i = 0; i < N; ++i) {
            double a = dirs[i][0] - 0.5, b = dirs[i][1] - 0.5, n = sqrt(a * a + b * b);
            sp[i][0] = (a / n) * (rad * 0.5);
            sp[i][1] = (b / n) * (rad * 0.5);
        }
        double a = t0 - 0.5, b = t1 - 0.5, n = sqrt(a * a + b * b);
        ev->target[0] = (a / n) * (tr * 3 + 2);
        ev->target[1] = (b / n) * (tr * 3 + 2);
        /* scenario.step() inside reset: the chasers are still at their pre-reset positions */
        or_target_step(p, ev, dr);
        for (int i = 0; i < N; ++i) { dr[i].pos[0] = sp[i][0]; dr[i].pos[1] = sp[i][1]; }
    } else {   /* static_same_goal: goals at the formation centre (size 0), spawn_points None -> spawn at the goal */
        double goal[OR_MAXN][3];
        if (p->scenario_b != OR_SC_NONE) {   /* any other create_scenario goal scenario (:123, :560) */
            or_sdraw sd;
            memset(&sd, 0, sizeof sd);
            sd.mode = OR_RNG_PHILOX; sd.seed = r->seed; sd.key = gbase; sd.stream = OR_S_SCN_RESET; sd.step = r->step;
            or_scen_reset(p, &ev->scen, &sd, goal);
        } else {
            for (int i = 0; i < N; ++i)
                for (int c = 0; c < 3; ++c) goal[i][c] = p->goal[c];
        }
        for (int i = 0; i < N; ++i) {
            for (int c = 0; c < 3; ++c) dr[i].goal[c] = goal[i][c];
            dr[i].pos[0] = dr[i].goal[0];
            dr[i].pos[1] = dr[i].goal[1];
        }
    }
    for (int i = 0; i < N; ++i) {
        or_drone* d = &dr[i];
        const uint32_t gid = gbase + (uint32_t)i;
        d->angle = ((tape ? or_gnext(r) : or_ru(r, gid, OR_S_RESET_A, 2, 0.0, 1.0)) - 0.5) * 2 * M_PI;
        double z = d->goal[2];
        if (z < 0.75) z = 0.75;
        d->pos[2] = z;
        for (int c = 0; c < 3; ++c) { d->vel[c] = 0.0; d->omega[c] = 0.0; d->acc[c] = 0.0; }
        double yaw = or_ru(r, gid, OR_S_RESET_YAW, 0, -M_PI, M_PI);   /* randyaw (quad_utils.py:228-230) */
        double cy = cos(yaw), sy = sin(yaw);
        double R[9] = {cy, -sy, 0, sy, cy, 0, 0, 0, 1};
        memcpy(d->rot, R, sizeof R);
        for (int k = 0; k < 4; ++k) { d->thrust_cmds_damp[k] = 0.0; d->thrust_rot_damp[k] = 0.0; }
        d->on_floor = 0; d->crashed_floor = 0; d->crashed_wall = 0; d->crashed_ceiling = 0;
        or_self_obs_a(p, d, r, gid, OR_S_RESET_SENSOR, OR_S_RESET_SELF_CAM, obs + (size_t)i * od);
        for (int c = 0; c < 3; ++c) ev->obs_pos[i][c] = d->pos[c];
    }
    ev->has_pos = 1;
    /* neighbours: fresh positions, stale QuadrotorEnvMulti.heading / .vel (:598-599) */
    or_neighbor_obs_a(p, ev, dr, r, gbase, 1, obs, od);
    if (reset_info) reset_info[e] = (unsigned char)(ev->success ? 2 : 1);
    ev->success = 0;
    ev->tick = 0;
    ev->episode += 1;
    /* the episode statistics start over (:605-617) */
    memset(ev->prev_pair_bits, 0, sizeof ev->prev_pair_bits);
    ev->st_col = ev->st_room = ev->st_floor = ev->st_wall = ev->st_ceil = ev->st_col_settle = ev->st_col_final = 0;
    ev->st_ocol = ev->st_ocol_settle = ev->st_o35 = ev->st_o5 = 0;
    for (int i = 0; i < N; ++i) {
        dr[i].hit_agent = dr[i].hit_obst = dr[i].reached = dr[i].prev_room = 0;
        dr[i].prev_wall = dr[i].prev_ceiling = 0;
    }
}

/* ------------------------------------------------------------------------------------------ */
/* step: QuadrotorEnvMulti.step (quadrotor_multi_rewards.py:630-991) + the SubprocVecEnvCustom */
/* worker's reset on done (subproc_vec_env_custom.py:33-46)                                    */
/* actions: [E*N, 2] (only a[0], the heading rate, is used: Controller.py:79)                  */
/* reset_info[e]: 0 = no reset, 1 = reset {"success": False}, 2 = reset {"success": True}     */
/* ------------------------------------------------------------------------------------------ */
void or_env_step_a(const or_params* p, or_drone* drones, or_env* envs, int e, const double* actions,
                   or_rng* r, double* obs, double* rew, unsigned char* done, double* term_obs,
                   unsigned char* reset_info) {
    const int N = p->num_agents, od = or_obs_dim_a(p);
    or_env* ev = &envs[e];
    or_drone* dr = &drones[(size_t)e * N];
    const uint32_t gbase = p->id_offset + (uint32_t)((size_t)e * N);
    const double* act = actions + (size_t)e * N * 2;
    double* o = obs + (size_t)e * N * od;
    double* rw = rew + (size_t)e * N;
    unsigned char* dn = done + (size_t)e * N;
    if (reset_info) reset_info[e] = 0;
    int any_done = 0;
    for (int sub = 0; sub < p->ticks_per_step && !any_done; ++sub) {
        r->step = ((uint64_t)ev->episode << 32) | (uint32_t)ev->tick;
        for (int i = 0; i < N; ++i) {
            or_drone* d = &dr[i];
            const uint32_t gid = gbase + (uint32_t)i;
            double motors[4], u[4];
            or_ctrl_a(p, d, act[i * 2], d->goal[2], motors);
            or_motors_to_cmds(motors, u);
            or_ou_noise(p, d->ou, r, gid);
            for (int s = 0; s < p->sim_steps; ++s) or_dyn_substep(p, d, u, d->ou, r, gid, s);
            {   /* infos[i]["goal_dist"] = |pos - goal| of this _step (quadrotor_single_rewards.py:457) */
                const double gd[3] = {d->pos[0] - d->goal[0], d->pos[1] - d->goal[1], d->pos[2] - d->goal[2]};
                d->rinfo[OR_RI_GOAL_DIST] = sqrt(gd[0] * gd[0] + gd[1] * gd[1] + gd[2] * gd[2]);
            }
            or_self_obs_a(p, d, r, gid, OR_S_SENSOR, OR_S_SELF_CAM, o + (size_t)i * od);
            for (int c = 0; c < 3; ++c) ev->obs_pos[i][c] = d->pos[c];
            ev->heading[i] = d->angle;
        }
        const int time_remain = p->ep_len - ev->tick;   /* QuadrotorSingle.time_remain, before tick += 1 */
        ev->tick += 1;
        const int tick_done = ev->tick > p->ep_len;
        /* 1. collisions between drones and with the room (:649-720) -- no forces (apply_collision_force is
         * False, :203), only the episode_extra_stats bookkeeping */
        {
            int in_cur[OR_MAXN] = {0}, in_prev[OR_MAXN] = {0}, wall_new[OR_MAXN], ceil_new[OR_MAXN];
            unsigned char cur[OR_MAXN * OR_MAXN];   /* the env's pair-bit layout (stride OR_MAXN) */
            memset(cur, 0, sizeof cur);
            for (int i = 0; i < N; ++i)
                for (int j = i + 1; j < N; ++j) {
                    const double dx = dr[i].pos[0] - dr[j].pos[0], dy = dr[i].pos[1] - dr[j].pos[1];
                    const double dz = dr[i].pos[2] - dr[j].pos[2];
                    if (sqrt(dx * dx + dy * dy + dz * dz) <= p->collision_threshold) {
                        cur[i * OR_MAXN + j] = 1; in_cur[i] = in_cur[j] = 1;
                    }
                    if (ev->prev_pair_bits[i * OR_MAXN + j]) in_prev[i] = in_prev[j] = 1;
                }
            memcpy(ev->prev_pair_bits, cur, sizeof cur);
            for (int i = 0; i < N; ++i) {   /* calculate_room_collision (:491-504): new wall / ceiling lists */
                wall_new[i] = dr[i].crashed_wall && !dr[i].prev_wall;
                ceil_new[i] = dr[i].crashed_ceiling && !dr[i].prev_ceiling;
                dr[i].prev_wall = wall_new[i];
                dr[i].prev_ceiling = ceil_new[i];
            }
            or_episode_stats_step(p, ev, dr, N, in_cur, in_prev, NULL, wall_new, ceil_new, NULL, NULL, od, time_remain);
        }
        /* capture reward (:711-735): xy distance of every drone to env 0's goal */
        double rel[OR_MAXN];
        int cap = 0;
        for (int i = 0; i < N; ++i) {
            double a = dr[0].goal[0] - dr[i].pos[0], b = dr[0].goal[1] - dr[i].pos[1];
            rel[i] = sqrt(a * a + b * b);
            if (ev->capture_radius > rel[i]) cap = 1;
        }
        for (int i = 0; i < N; ++i) {
            double captor = cap ? p->w_captor * (ev->capture_radius > rel[i] ? 1.0 : 0.0) : 0.0;
            double helper = cap ? p->w_helper * (ev->capture_radius < rel[i] ? 1.0 : 0.0) : 0.0;
            double x = 0.0;
            x += -0.0 * rel[i];
            x += captor;
            x += helper;
            x += p->existence;
            rw[i] = x;
            dn[i] = (unsigned char)(cap ? (ev->capture_radius > rel[i]) : tick_done);
            if (dn[i]) any_done = 1;
        }
        if (cap) ev->success = 1;
        /* perform_downwash with the control dt (:810-815); when it touched a drone the reference rebuilds the
         * tick's obs after scenario.step() (:848-859: state_vector, i.e. the moved goal and fresh sensor /
         * camera noise) */
        const int dw = p->use_downwash && N > 1 && or_downwash(p, dr, N, gbase, r);
        if (p->scenario_a == 1) {
            or_target_step(p, ev, dr);   /* scenario.step() (:797) */
        } else if (p->scenario_b != OR_SC_NONE) {   /* a goal scenario's step, every tick (:848) */
            or_sdraw sd;
            memset(&sd, 0, sizeof sd);
            sd.mode = OR_RNG_PHILOX; sd.seed = r->seed; sd.key = gbase; sd.stream = OR_S_SCN; sd.step = r->step;
            double g[OR_MAXN][3];
            for (int i = 0; i < N; ++i) memcpy(g[i], dr[i].goal, sizeof g[i]);
            or_scen_step(p, &ev->scen, ev->tick, &sd, g);
            for (int i = 0; i < N; ++i) memcpy(dr[i].goal, g[i], sizeof g[i]);
        }
        if (dw)
            for (int i = 0; i < N; ++i)
                or_self_obs_a(p, &dr[i], r, gbase + (uint32_t)i, OR_S_SENSOR, OR_S_SELF_CAM, o + (size_t)i * od);
        for (int i = 0; i < N; ++i)
            for (int c = 0; c < 3; ++c) { ev->obs_pos[i][c] = dr[i].pos[c]; ev->obs_vel[i][c] = dr[i].vel[c]; }
    }
    if (any_done) {
        for (int i = 0; i < N; ++i) dn[i] = 1;
        /* infos[i]["episode_extra_stats"] (:886-969): distance_to_goal is empty -> np.mean gives nan */
        or_episode_stats_done(p, ev, dr, N);
        if (p->scenario_a == 1) ev->ep_stats[OR_ES_SCEN] = 18;   /* Scenario_dynamic_repulsive */
        for (int i = 0; i < N; ++i) for (int k = 0; k < 3; ++k) dr[i].ep_dist[k] = NAN;
    }
    or_neighbor_obs_a(p, ev, dr, r, gbase, 0, o, od);
    if (any_done) {
        if (term_obs) memcpy(term_obs + (size_t)e * N * od, o, sizeof(double) * (size_t)N * od);
        or_env_reset_a(p, drones, envs, e, r, o, reset_info);
    }
}

void or_reset_all_a(const or_params* p, or_drone* drones, or_env* envs, uint32_t seed, double* obs,
                    unsigned char* reset_info) {
    const int od = or_obs_dim_a(p);
    for (int e = 0; e < p->num_envs; ++e) {
        or_rng r;
        memset(&r, 0, sizeof r);
        r.mode = OR_RNG_PHILOX; r.seed = seed;
        or_env_reset_a(p, drones, envs, e, &r, obs + (size_t)e * p->num_agents * od, reset_info);
    }
}

void or_step_all_a(const or_params* p, or_drone* drones, or_env* envs, const double* actions, uint32_t seed,
                   double* obs, double* rew, unsigned char* done, double* term_obs, unsigned char* reset_info,
                   int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(static)
#endif
    for (int e = 0; e < p->num_envs; ++e) {
        or_rng r;
        memset(&r, 0, sizeof r);
        r.mode = OR_RNG_PHILOX; r.seed = seed;
        or_env_step_a(p, drones, envs, e, actions, &r, obs, rew, done, term_obs, reset_info);
    }
    (void)nthreads;
}
