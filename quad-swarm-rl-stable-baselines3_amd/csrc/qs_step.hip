// qs_step.hip -- the C ABI (include/quadswarm.h) over the fused MI355X (gfx950) step kernels:
// flavor B in qs_flavor_b.h, flavor A in qs_flavor_a.h, shared device code in qs_common.h.
//
// Reference path replaced (priban42/quad-swarm-rl-stable-baselines3), flavor B:
//   QuadrotorEnvMulti.step            gym_art/quadrotor_multi/quadrotor_multi.py:521-841
//   QuadrotorSingle._step / _reset    quadrotor_single.py:355-371 / :401-469
//   QuadrotorDynamics.step/step1_numba quadrotor_dynamics.py:215-221, :355-390, :504-656
//   RawControl.step                   quadrotor_control.py:53-57
//   SensorNoise.add_noise_numba       sensor_noise.py:172-261 ; get_state.py:226-292
//   collisions / room / downwash      collisions/quadrotors.py, collisions/room.py, aerodynamics/downwash.py
// flavor A: see qs_flavor_a.h (quadrotor_multi_rewards.py, quadrotor_single_rewards.py, Controller/).
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

#include <math.h>

#include <hip/hiprtc.h>

#include <map>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "qs_rng.h"
#include "quadswarm.h"
#include "qs_common.h"
#include "qs_flavor_b.h"
#include "qs_flavor_a.h"
#include "qs_gae.h"
#include "qs_curriculum.h"
#include "qs_replay.h"
#include "qs_error.h"

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
    hipFunction_t jit_step = nullptr;    // qs_specialize: kernels compiled for this handle's parameters
    hipFunction_t jit_reset = nullptr;
    hipModule_t jit_mod = nullptr;       // their module
    int qb = QS_QB, qa = QS_QA;          // sub-lanes per drone of the step kernels in use (flavor B / A)
    // experience replay (qs_replay_enable): one device allocation holding every RBufs array
    void* rws = nullptr;
    bool rws_owned = false;
    qs::RBufs rb{};
    qs::RP rp{};
};

static thread_local std::string g_err;

// make h's device current; hipGetDevice is a thread-local read, hipSetDevice only when it differs
static hipError_t use_device(const qs_handle* h) {
    int cur = -1;
    if (hipGetDevice(&cur) == hipSuccess && cur == h->device) return hipSuccess;
    return hipSetDevice(h->device);
}

int qs_fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}
static int fail(int code, const std::string& msg) { return qs_fail(code, msg); }

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
    static const int d[7] = {18, 19, 24, 6, 6, 7, 7};   // quad_utils.py:30-38
    return (repr >= 0 && repr < 7) ? d[repr] : 0;
}

// floats per visible neighbour (quad_utils.py:40-58) and the flavor-A feature mask
static int neighbor_dim(int t) {
    static const int d[9] = {0, 6, 2, 3, 3, 3, 5, 3, 3};
    return (t >= 0 && t < 9) ? d[t] : 0;
}
static int neighbor_feats(int t) {
    using namespace qs;
    switch (t) {
        case QS_NEIGHBOR_POS_VEL: return QS_NF_POS | QS_NF_VEL;
        case QS_NEIGHBOR_DIST_ANGLE: return QS_NF_DIST | QS_NF_ANGLE;
        case QS_NEIGHBOR_DIST_SANGLE: return QS_NF_DIST | QS_NF_SANGLE;
        case QS_NEIGHBOR_NDIST_NSANGLE: return QS_NF_NDIST | QS_NF_NSANGLE;
        case QS_NEIGHBOR_DIST_ANGLE_HEADING: return QS_NF_DIST | QS_NF_ANGLE | QS_NF_HEADING;
        case QS_NEIGHBOR_DIST_SANGLE_SHEADING: return QS_NF_DIST | QS_NF_SANGLE | QS_NF_SHEADING;
        case QS_NEIGHBOR_POS: return QS_NF_POS;
        case QS_NEIGHBOR_NPOS: return QS_NF_NPOS;
        default: return 0;
    }
}

static int validate(const qs_config* c) {
    if (!c) return fail(QS_E_INVALID, "config is NULL");
    if (c->abi_version != QS_ABI_VERSION) return fail(QS_E_INVALID, "config abi_version mismatch");
    if (c->num_envs < 1) return fail(QS_E_INVALID, "num_envs must be >= 1");
    if (c->num_agents < 1 || c->num_agents > QS_MAX_AGENTS)
        return fail(QS_E_UNSUPPORTED, "num_agents must be in [1, QS_MAX_AGENTS]");
    if (c->flavor != QS_FLAVOR_B && c->flavor != QS_FLAVOR_A) return fail(QS_E_INVALID, "unknown flavor");
    if (c->neighbor_obs < 0 || c->neighbor_obs > QS_NEIGHBOR_NPOS) return fail(QS_E_INVALID, "unknown neighbor_obs");
    if (c->flavor == QS_FLAVOR_B) {
        if (c->obs_repr < 0 || c->obs_repr > 2) return fail(QS_E_INVALID, "obs_repr is not a flavor-B repr");
        if (c->neighbor_obs != QS_NEIGHBOR_NONE && c->neighbor_obs != QS_NEIGHBOR_POS_VEL)
            return fail(QS_E_UNSUPPORTED, "flavor B implements neighbor_obs none / pos_vel");
        if (c->use_obstacles) {
            if ((c->scenario < QS_SCEN_OBST_MIX || c->scenario > QS_SCEN_O_STATIC_SAME_GOAL) &&
                (c->scenario < QS_SCEN_O_SWAP_GOALS || c->scenario > QS_SCEN_O_DYNAMIC_SAME_GOAL))
                return fail(QS_E_UNSUPPORTED, "obstacles need scenario obst_mix / o_random / o_static_same_goal / "
                                              "o_swap_goals / o_ep_rand_bezier / o_dynamic_same_goal");
            if (c->obst_area < 1 || c->obst_area > 8) return fail(QS_E_UNSUPPORTED, "obst_area must be in [1, 8]");
            if (c->num_obstacles < 1 || c->num_obstacles + c->num_agents > c->obst_area * c->obst_area)
                return fail(QS_E_INVALID, "num_obstacles must leave a free cell per drone");
            if (c->obst_size <= 0.f || c->sdf_resolution <= 0.f) return fail(QS_E_INVALID, "bad obst_size / sdf_resolution");
            if (c->dr_num_counts < 0 || c->dr_num_counts > QS_MAX_DR_CHOICES || c->dr_num_sizes < 0 ||
                c->dr_num_sizes > QS_MAX_DR_CHOICES)
                return fail(QS_E_INVALID, "dr_num_counts / dr_num_sizes must be in [0, QS_MAX_DR_CHOICES]");
            for (int i = 0; i < c->dr_num_counts; ++i)
                if (c->dr_counts[i] != -1 &&
                    (c->dr_counts[i] < 1 || c->dr_counts[i] + c->num_agents > c->obst_area * c->obst_area))
                    return fail(QS_E_INVALID, "dr_counts entries: -1 (keep) or pillars leaving a free cell per drone");
            for (int i = 0; i < c->dr_num_sizes; ++i)
                if (!(c->dr_sizes[i] >= 0.f)) return fail(QS_E_INVALID, "dr_sizes entries must be >= 0 (0 = keep)");
        } else if (c->scenario != QS_SCEN_STATIC_SAME_GOAL &&
                   (c->scenario < QS_SCEN_MIX || c->scenario > QS_SCEN_RUN_AWAY)) {
            return fail(QS_E_UNSUPPORTED, "flavor B without obstacles: static_same_goal, mix or a goal scenario");
        } else if (c->scenario == QS_SCEN_RUN_AWAY && c->num_agents < 2) {
            return fail(QS_E_INVALID, "run_away needs at least 2 drones (run_away.py:16-27)");
        }
    } else {
        if (c->use_obstacles) return fail(QS_E_UNSUPPORTED, "flavor A with obstacles is not implemented");
        if (c->obs_repr < 3 || c->obs_repr > 6) return fail(QS_E_INVALID, "obs_repr is not a flavor-A repr");
        if (c->scenario != QS_SCEN_STATIC_SAME_GOAL && c->scenario != QS_SCEN_DYNAMIC_REPULSIVE &&
            (c->scenario < QS_SCEN_MIX || c->scenario > QS_SCEN_RUN_AWAY))
            return fail(QS_E_INVALID, "flavor A: static_same_goal, dynamic_repulsive or a goal scenario");
        if (c->scenario == QS_SCEN_RUN_AWAY && c->num_agents < 2)
            return fail(QS_E_INVALID, "run_away needs at least 2 drones (run_away.py:16-27)");
        if (c->ticks_per_step < 1) return fail(QS_E_INVALID, "ticks_per_step must be >= 1");
        if (c->n_cameras < 1 || c->n_cameras > 8) return fail(QS_E_INVALID, "n_cameras must be 1..8");
        // envs of more than 64 drones (multi-wave workgroups) select their neighbours by register insertion
        // (qs_flavor_a.h neighbor_obs_wide)
        if (c->num_agents > 64 && c->neighbor_obs != QS_NEIGHBOR_NONE && c->k_neighbors > QS_A_KMAX)
            return fail(QS_E_UNSUPPORTED, "flavor A with more than 64 drones: k_neighbors must be <= QS_A_KMAX (16)");
    }
    if (c->neighbor_obs != QS_NEIGHBOR_NONE && (c->k_neighbors < 1 || c->k_neighbors > c->num_agents - 1))
        return fail(QS_E_INVALID, "k_neighbors must be in [1, num_agents-1]");
    if (c->sim_steps < 1 || c->svd_every < 1 || c->ep_len < 0) return fail(QS_E_INVALID, "bad sim_steps/svd_every/ep_len");
    // The drone state is addressed by 32-bit byte offsets from the state buffer, and the step's state stores go
    // through a buffer descriptor of 0x7fffffff records (qs_rsrc): the last istate word, at most
    // 4 (QS_NF + QS_NI) I + 255 bytes from the state base, must stay inside it (I <= 7 669 584 drones).
    if (4ll * (QS_NF + QS_NI) * ((long long)c->num_envs * c->num_agents) + 256 > 0x7fffffffll)
        return fail(QS_E_INVALID, "too many drones: 4 (QS_NF + QS_NI) num_envs num_agents + 256 must stay below 2^31");
    return QS_OK;
}

static int npad_of(int n);
// a gfx950 workgroup may allocate the CU's whole 160 KB of LDS (64-drone envs with all 63 neighbours visible
// stage 64 rows of 396 floats)
static constexpr size_t QS_LDS_MAX = 160 * 1024;
static size_t shm_bytes(const qs_config& c, int obs_dim, int npad, bool step, int qb = QS_QB, int qa = QS_QA);
static int neighbor_dim(int t);

// pillar slots per env: the configured count, or the largest domain-randomisation choice
static int obst_slots(const qs_config* c) {
    int m = c->num_obstacles;
    for (int i = 0; i < c->dr_num_counts && i < QS_MAX_DR_CHOICES; ++i) m = c->dr_counts[i] > m ? c->dr_counts[i] : m;
    return m;
}

static qs_layout make_layout(const qs_config* c) {
    qs_layout L;
    memset(&L, 0, sizeof L);
    const size_t I = (size_t)c->num_envs * c->num_agents, E = (size_t)c->num_envs;
    const int od = self_obs_dim(c->obs_repr) +
                   (c->neighbor_obs != QS_NEIGHBOR_NONE ? neighbor_dim(c->neighbor_obs) * c->k_neighbors : 0) +
                   (c->use_obstacles ? 9 : 0);
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    size_t o = 0;
    L.params = o; o = al(al(o + sizeof(qs::KP)) + sizeof(qs::RArgs));   // KP, then the replay arguments (rargs_of)
    L.state = o; o = al(o + sizeof(float) * QS_NF * I);
    L.istate = o; o = al(o + sizeof(int32_t) * QS_NI * I);
    L.env = o; o = al(o + sizeof(int32_t) * QS_NE * E);
    L.env_f = o; o = al(o + sizeof(float) * QS_NENVF * E);
    L.obst = o; o = al(o + sizeof(float) * 2 * (c->use_obstacles ? (size_t)obst_slots(c) : 0) * E);
    L.stale_vel = o; o = al(o + sizeof(float) * 3 * I);
    L.obs = o; o = al(o + sizeof(float) * I * od);
    L.term_obs = o; o = al(o + sizeof(float) * I * od);
    L.rew = o; o = al(o + sizeof(float) * I);
    L.done = o; o = al(o + I);
    L.reset_info = o; o = al(o + E);
    L.stats = o; o = al(o + sizeof(uint64_t) * QS_NSTAT);
    L.estats = o; o = al(o + sizeof(float) * QS_NES * (c->episode_stats ? I : 0));
    L.rew_info = o; o = al(o + sizeof(float) * QS_NRI * (c->step_infos ? I : 0));
    L.total_bytes = o;
    L.obs_dim = od;
    L.num_drones = (int32_t)I;
    return L;
}

// 4x4 inverse (Gauss-Jordan, partial pivoting) for Mixer.calculate_allocation (Mixer.py:31-66): the
// pseudo-inverse A^T (A A^T)^-1 of the square invertible allocation matrix is A^-1
static void inv4(const double* a, double* out) {
    double m[4][8];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 8; ++j) m[i][j] = j < 4 ? a[i * 4 + j] : (j - 4 == i ? 1.0 : 0.0);
    for (int col = 0; col < 4; ++col) {
        int piv = col;
        for (int r = col + 1; r < 4; ++r)
            if (fabs(m[r][col]) > fabs(m[piv][col])) piv = r;
        for (int j = 0; j < 8; ++j) { const double t = m[col][j]; m[col][j] = m[piv][j]; m[piv][j] = t; }
        const double dv = m[col][col];
        for (int j = 0; j < 8; ++j) m[col][j] /= dv;
        for (int r = 0; r < 4; ++r)
            if (r != col) {
                const double f = m[r][col];
                for (int j = 0; j < 8; ++j) m[r][j] -= f * m[col][j];
            }
    }
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) out[i * 4 + j] = m[i][4 + j];
}

// flavor-A constants: Controller() builds every controller from the default ModelParams
// (Controller.py:16-29, MultirotorModel.py:10-50), independent of the env's dynamics params.
static void make_kp_a(const qs_config* c, qs::KP& k) {
    const double PI = 3.14159265358979323846;
    k.flavor = c->flavor; k.scenario = c->scenario; k.ticks = c->ticks_per_step;
    k.nfeat = neighbor_feats(c->neighbor_obs); k.nfd = neighbor_dim(c->neighbor_obs);
    k.n_cam = c->n_cameras;
    k.cam_r = 0.5f * c->cam_size; k.cam_f = c->cam_focal; k.cam_px = c->cam_px_noise; k.cam_res = c->cam_res;
    {   // the camera axes of qs::camera's sector pick, in the kernel's float arithmetic (seg = 2 pi / n in fp32)
        const float seg = 6.28318530717959f / (float)k.n_cam;
        for (int i = 0; i < 8; ++i) {
            k.cam_cos[i] = i < k.n_cam ? cosf((float)i * seg) : 1.f;
            k.cam_sin[i] = i < k.n_cam ? sinf((float)i * seg) : 0.f;
        }
    }
    k.cam_w = (float)(2.0 * tan((c->cam_fov_deg / 2.0) * PI / 180.0) * c->cam_focal);
    k.hrate = (float)((double)c->dt * (PI * 80.0 / 180.0));
    k.speed = 0.2f;
    k.inv_dt = (float)(1.0 / (double)c->dt);
    const double mass = 0.028, g = 9.81, kf = 0.00000000125, km = 0.0025, prop_r = 0.00015, arm = 0.04596,
                 bh = 0.003, min_rpm = 1170.0, max_rpm = 13000.0;
    const double J[3] = {mass * (3.0 * arm * arm + bh * bh) / 12.0, mass * (3.0 * arm * arm + bh * bh) / 12.0,
                         (mass * arm * arm) / 2.0};
    for (int i = 0; i < 10; ++i) {
        double kp_, kd_, ki_, sat, aw;
        if (i == 0) { kp_ = 4.1625; kd_ = 0.5473; ki_ = 0.0023; sat = 6.0; aw = 2.0; }           // PositionController z
        else if (i < 4) { kp_ = 2.4531; kd_ = 0.0003; ki_ = 0.0382; sat = 40.0; aw = 1.0; }      // VelocityController
        else if (i < 7) { kp_ = 11.2081; kd_ = 0.0490; ki_ = 0.0073; sat = i == 6 ? 1.0 : 10.0; aw = 0.1; }  // Attitude
        else { const double j = J[i - 7]; kp_ = 3.1222 * j; kd_ = 0.0477 * j; ki_ = 0.0001 * j; sat = -1; aw = 1.0; }  // Rate
        k.pkp[i] = (float)kp_; k.pkd[i] = (float)kd_; k.pki[i] = (float)ki_; k.psat[i] = (float)sat; k.paw[i] = (float)aw;
    }
    k.rate_scale = 800.f;
    double alloc[16] = {-0.707, 0.707, 0.707, -0.707, -0.707, 0.707, -0.707, 0.707,
                        -1.0, -1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0};
    for (int j = 0; j < 4; ++j) {
        alloc[j] *= arm * kf; alloc[4 + j] *= arm * kf;
        alloc[8 + j] *= km * (3.0 * prop_r) * kf; alloc[12 + j] *= kf;
    }
    double inv[16];
    inv4(alloc, inv);
    for (int i = 0; i < 4; ++i) {
        const double n = sqrt(inv[i * 4] * inv[i * 4] + inv[i * 4 + 1] * inv[i * 4 + 1]);
        if (n > 0) { inv[i * 4] /= n; inv[i * 4 + 1] /= n; }
        const double v = inv[i * 4 + 2];
        inv[i * 4 + 2] = v > 1e-2 ? 1.0 : (v < -1e-2 ? -1.0 : 0.0);
        inv[i * 4 + 3] = 1.0;
    }
    for (int i = 0; i < 16; ++i) k.mix[i] = (float)inv[i];
    k.m_mass = (float)mass; k.m_mass_g = (float)(mass * g); k.m_kf4 = (float)(kf * 4);
    k.m_min_rpm = (float)min_rpm; k.m_inv_rpm = (float)(1.0 / (max_rpm - min_rpm));
    k.w_captor = 100.f; k.w_helper = 100.f; k.existence = -0.1f;                  // quadrotor_multi_rewards.py:716-724
    k.tgt_vmax = 0.5f; k.tgt_dt = (float)(1.0 / 200); k.arena = 5.f; k.tgt_z = 2.f; // dynamic_repulsive.py:29-35,52-55
    // neighbour clip box = float32 observation-space Box (quadrotor_single_rewards.py:267-319)
    const float pi32 = (float)PI;
    int q = 0;
    auto put = [&](float lo, float hi) { if (q < 8) { k.nclip_lo[q] = lo; k.nclip_hi[q] = hi; ++q; } };
    const int m = k.nfeat;
    const float half = 0.5f * (c->room_hi[0] - c->room_lo[0]);
    if (m & qs::QS_NF_DIST) put(-half, half);
    if (m & qs::QS_NF_NDIST) put(-half, half);
    if (m & qs::QS_NF_ANGLE) put(-pi32, pi32);
    if (m & qs::QS_NF_SANGLE) { put(-1.f, 1.f); put(-1.f, 1.f); }
    if (m & qs::QS_NF_NSANGLE) { put(-1.f, 1.f); put(-1.f, 1.f); }
    if (m & qs::QS_NF_HEADING) put(-pi32, pi32);
    if (m & qs::QS_NF_SHEADING) { put(-1.f, 1.f); put(-1.f, 1.f); }
    if (m & (qs::QS_NF_NPOS | qs::QS_NF_POS))
        for (int i = 0; i < 3; ++i) put(-(c->room_hi[i] - c->room_lo[i]), c->room_hi[i] - c->room_lo[i]);
    if (m & qs::QS_NF_VEL)
        for (int i = 0; i < 3; ++i) put(-2.f * c->vxyz_max, 2.f * c->vxyz_max);
}

static qs::KP make_kp(const qs_config* c, const qs_layout& L) {
    qs::KP k;
    memset(&k, 0, sizeof k);
    k.E = c->num_envs; k.N = c->num_agents; k.I = L.num_drones; k.obs_dim = L.obs_dim;
    k.so_dim = self_obs_dim(c->obs_repr);
    k.neighbor = c->neighbor_obs;
    k.K = c->neighbor_obs != QS_NEIGHBOR_NONE ? c->k_neighbors : 0;
    k.id0 = c->drone_id_offset;
    k.seed = c->seed;
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
    k.mass_g = (float)((double)c->mass * (double)c->gravity);
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
    k.flavor = c->flavor;
    // goal scenarios (flavor B, no obstacles): QS_SCEN_MIX -> 10, QS_SCEN_STATIC_DIFF_GOAL.. -> 1..9
    k.scen_b = -1;
    if (!c->use_obstacles && c->scenario >= QS_SCEN_MIX && c->scenario <= QS_SCEN_RUN_AWAY)
        k.scen_b = c->scenario == QS_SCEN_MIX ? 10 : c->scenario - QS_SCEN_MIX;
    if (c->flavor == QS_FLAVOR_A) make_kp_a(c, k);
    k.rcomp = c->step_infos ? 1 : 0;
    if (c->episode_stats) {   // quadrotor_multi.py:156-161, 651-655, 761-774; quadrotor_multi_rewards.py:131-136
        double freq = 1.0 / (double)c->control_dt;   // control_freq (100 for the reference's 0.01 s)
        if (fabs(freq - (double)llround(freq)) < 1e-4) freq = (double)llround(freq);
        k.stats = 1;
        k.st_settle = (int)ceil(1.5 * freq - 1e-9);    // tick >= collisions_grace_period_steps
        k.st_final = (int)floor(5.0 * freq + 1e-9);    // time_remain <= collisions_final_grace_period_steps
        k.st_win[0] = (int)(1.0 * freq + 1e-9); k.st_win[1] = (int)(3.0 * freq + 1e-9); k.st_win[2] = (int)(5.0 * freq + 1e-9);
    }
    if (c->use_obstacles) {
        k.obst = 1; k.M = obst_slots(c); k.obst_n = c->obst_area;
        // 0 mix (o_random / o_static_same_goal), then the obstacle mode + 1: o_random, o_static_same_goal,
        // o_swap_goals, o_ep_rand_bezier, o_dynamic_same_goal; the dynamic ones also step as goal scenarios (scen_b)
        k.obst_scen = c->scenario == QS_SCEN_OBST_MIX ? 0 : (c->scenario == QS_SCEN_O_RANDOM ? 1 :
                      c->scenario == QS_SCEN_O_STATIC_SAME_GOAL ? 2 : 3 + (c->scenario - QS_SCEN_O_SWAP_GOALS));
        if (c->scenario >= QS_SCEN_O_SWAP_GOALS) k.scen_b = qs::SC_O_SWAP_GOALS + (c->scenario - QS_SCEN_O_SWAP_GOALS);
        k.obst_r = 0.5f * c->obst_size;
        k.obst_thr = (float)((double)c->arm + 0.5 * (double)c->obst_size);   // quad arm + pillar radius
        // domain randomisation tables: index 0 = the configured pillars, choice c = index c + 1
        k.dr_nm = c->dr_num_counts; k.dr_ns = c->dr_num_sizes;
        k.dr = (k.dr_nm > 0 || k.dr_ns > 0) ? 1 : 0;
        k.dr_m[0] = c->num_obstacles; k.dr_r[0] = k.obst_r; k.dr_thr[0] = k.obst_thr;
        for (int i = 0; i < k.dr_nm; ++i) k.dr_m[i + 1] = c->dr_counts[i];
        for (int i = 0; i < k.dr_ns; ++i) {
            const float sz = c->dr_sizes[i];
            k.dr_r[i + 1] = sz > 0.f ? 0.5f * sz : 0.f;   // 0 = a falsy 0.0 choice: keep the env's size
            k.dr_thr[i + 1] = sz > 0.f ? (float)((double)c->arm + 0.5 * (double)sz) : 0.f;
        }
        k.obst_z = 0.5f * c->room_hi[2];                                       // pillar centre (:423)
        k.sdf_res = c->sdf_resolution;
        k.quadcol_obst = c->rew_quadcol_bin_obst;
    }
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
    // flavor-A fields (used once flavor = QS_FLAVOR_A): swarm_rl/global_cfg.py:14-40
    c->flavor = QS_FLAVOR_B;
    c->scenario = QS_SCEN_STATIC_SAME_GOAL;
    c->ticks_per_step = 8;
    c->n_cameras = 3;
    c->capture_radius = 3.f;
    c->cam_size = 0.2f; c->cam_focal = 0.035f; c->cam_px_noise = 3.f; c->cam_fov_deg = 70.f; c->cam_res = 640.f;
    // obstacle fields (used once use_obstacles = 1): the C4 run (swarm_rl/runs/obstacles/quad_obstacle_baseline.py)
    c->use_obstacles = 0;
    c->num_obstacles = 12;
    c->obst_area = 8;
    c->obst_size = 0.6f;
    c->sdf_resolution = 0.1f;
    c->rew_quadcol_bin_obst = 5.f;
    return QS_OK;
}

// flavor A as swarm_rl/sb_train.py configures it (global_cfg.py + parameter_sweep :111-133): room
// 15x15x3, 30 s episodes (3000 ticks), cdist..sangle self obs, camera neighbours of all N-1 drones,
// dynamic_repulsive target, no drone/room impulses (quadrotor_multi_rewards.py:203).
extern "C" int qs_config_default_a(qs_config* c, int32_t num_envs, int32_t num_agents) {
    int rc = qs_config_default(c, num_envs, num_agents);
    if (rc) return rc;
    c->flavor = QS_FLAVOR_A;
    c->scenario = QS_SCEN_DYNAMIC_REPULSIVE;
    c->obs_repr = QS_OBS_CDIST_CDISTDOT_DIST_DISTDOT_SANGLE_ANGLEDOT;
    c->neighbor_obs = num_agents > 1 ? QS_NEIGHBOR_NDIST_NSANGLE : QS_NEIGHBOR_NONE;
    c->k_neighbors = num_agents > 1 ? num_agents - 1 : 0;
    c->ep_len = 3000;
    c->apply_collision_force = 0;
    c->room_lo[0] = -7.5f; c->room_lo[1] = -7.5f; c->room_lo[2] = 0.f;
    c->room_hi[0] = 7.5f; c->room_hi[1] = 7.5f; c->room_hi[2] = 3.f;
    c->cam_px_noise = 0.f;   // parameter_sweep (sb_train.py:139)
    return QS_OK;
}

static int check_lds(const qs_config* c) {
    const qs_layout L = make_layout(c);
    const int np = npad_of(c->num_agents);
    if (shm_bytes(*c, L.obs_dim, np, true) > QS_LDS_MAX || shm_bytes(*c, L.obs_dim, np, false) > QS_LDS_MAX)
        return fail(QS_E_UNSUPPORTED, "observation / obstacle tiles exceed the 160 KB of LDS of a workgroup");
    return QS_OK;
}

extern "C" int qs_layout_query(const qs_config* c, qs_layout* out) {
    int rc = validate(c);
    if (!rc) rc = check_lds(c);
    if (rc) return rc;
    if (!out) return fail(QS_E_INVALID, "layout is NULL");
    *out = make_layout(c);
    return QS_OK;
}

// Step launches give every drone Q lanes (qs::StepGeo for flavor B: QS_QB, qs::StepGeoA for A: QS_QA; fewer
// when an env would not fit a wave); resets one lane.  Specialised kernels may be compiled with another Q
// (qs_handle::qb / qa).
// flavor B (qs::StepGeo): QS_QW sub-lanes for the multi-wave 64 / 128-drone envs; flavor A (qs::StepGeoA): an
// env of up to 64 drones stays inside one wave, a 128-drone env takes QS_QW sub-lanes over 4 waves
static int step_lanes_per_drone(int npad, int q, bool flavor_a = false) {
    return npad * q <= 64 ? q : ((npad >= 64 && !flavor_a) || npad > 64 ? QS_QW : 64 / npad);
}
static_assert(qs::StepGeo<8>::Q == QS_QB && qs::StepGeo<32>::Q == 64 / 32 && qs::StepGeo<64>::Q == QS_QW &&
              qs::StepGeo<128>::Q == QS_QW && qs::StepGeo<128>::WGS == 128 * QS_QW && qs::StepGeoA<8>::Q == QS_QA &&
              qs::StepGeoA<32>::Q == 2 && qs::StepGeoA<64>::Q == 1 && qs::StepGeoA<128>::Q == QS_QW &&
              qs::StepGeoA<128>::WGS == 128 * QS_QW && qs::ResetGeoA<128>::WGS == 128 && qs::ResetGeoA<8>::EPB == 8,
              "step_lanes_per_drone");
// threads per workgroup: one wave, or (128-drone envs) the env's lanes
static int block_threads(const qs_config& c, int npad, bool step, int qb = QS_QB, int qa = QS_QA) {
    const int q = !step ? 1 : step_lanes_per_drone(npad, c.flavor == QS_FLAVOR_A ? qa : qb, c.flavor == QS_FLAVOR_A);
    return npad * q > 64 ? npad * q : 64;
}
static int envs_per_block(const qs_config& c, int npad, bool step, int qb = QS_QB, int qa = QS_QA) {
    const int q = !step ? 1 : step_lanes_per_drone(npad, c.flavor == QS_FLAVOR_A ? qa : qb, c.flavor == QS_FLAVOR_A);
    return block_threads(c, npad, step, qb, qa) / (npad * q);
}

// dynamic LDS of a launch with `slots` drone rows per workgroup: obs tile + neighbour exchange tile
// + 64 words (flavor-A flags) + obstacle tiles and per-env reset scratch (qs_flavor_b.h obst_tile)
static size_t shm_bytes(const qs_config& c, int obs_dim, int npad, bool step, int qb, int qa) {
    const size_t epb = (size_t)envs_per_block(c, npad, step, qb, qa), slots = epb * (size_t)npad;
    size_t b = sizeof(float) * slots * (size_t)obs_dim + sizeof(float) * slots * 8 + sizeof(float) * 64;
    if (c.use_obstacles) b += epb * (sizeof(float) * 2 * (size_t)obst_slots(&c) + (size_t)qs::QS_OBST_SCRATCH);
    const bool tables = c.use_obstacles ? c.scenario >= QS_SCEN_O_SWAP_GOALS
                                        : (c.scenario >= QS_SCEN_MIX && c.scenario <= QS_SCEN_RUN_AWAY);
    if (tables) b += epb * sizeof(float) * (2 * ((size_t)npad + 4) * 4 + 32);   // goal tables (qs::scen_stride)
    return b;
}

static int npad_of(int n) {
    int p = 1;
    while (p < n) p <<= 1;
    return p;
}

extern "C" int qs_create(const qs_config* c, int dev, void* ws, qs_handle** out) {
    int rc = validate(c);
    if (!rc) rc = check_lds(c);
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
    if (e == hipSuccess && c->flavor == QS_FLAVOR_A) {   // per-env capture radius (initial_capture_radius)
        std::vector<float> cr((size_t)c->num_envs, c->capture_radius);
        e = hipMemcpy((char*)h->ws + h->lay.env_f + sizeof(float) * QS_ENVF_CAPTURE * (size_t)c->num_envs, cr.data(),
                      sizeof(float) * cr.size(), hipMemcpyHostToDevice);
    }
    // the initialisation ran on the null stream: complete it before any (possibly non-blocking) stream
    // of the caller touches the workspace
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) {
        if (h->owns_ws) (void)hipFree(h->ws);
        delete h;
        return fail(QS_E_HIP, std::string("workspace init: ") + hipGetErrorString(e));
    }
    *out = h;
    return QS_OK;
}

// the step kernel's replay arguments in device memory, after the KP block (zeroed with the workspace: replay off)
static qs::RArgs* rargs_of(qs_handle* h) {
    return (qs::RArgs*)((char*)h->ws + h->lay.params + ((sizeof(qs::KP) + 255) & ~(size_t)255));
}
static hipError_t rargs_sync(qs_handle* h) {
    qs::RArgs a{};
    if (h->rws) {
        a.ri = (uint64_t)h->rb.ri; a.crash = (uint64_t)h->rb.crash; a.hist = (uint64_t)h->rb.hist;
        a.perm = (uint64_t)h->rb.perm; a.nrep = (uint64_t)h->rb.nrep; a.store = (uint64_t)h->rb.store;
    }
    a.p = h->rp;
    return hipMemcpy(rargs_of(h), &a, sizeof a, hipMemcpyHostToDevice);
}

static void replay_free(qs_handle* h) {
    if (h->rws && h->rws_owned) (void)hipFree(h->rws);
    h->rws = nullptr;
    h->rb = qs::RBufs{};
    if (h->ws) (void)rargs_sync(h);
}

extern "C" int qs_destroy(qs_handle* h) {
    if (!h) return QS_OK;
    replay_free(h);
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
    b.envf = (float*)(w + h->lay.env_f);
    b.obst = (float2*)(w + h->lay.obst);
    b.stale = (float*)(w + h->lay.stale_vel);
    b.obs = (float*)(w + h->lay.obs);
    b.term = (float*)(w + h->lay.term_obs);
    b.rew = (float*)(w + h->lay.rew);
    b.done = (uint8_t*)(w + h->lay.done);
    b.rinfo = (uint8_t*)(w + h->lay.reset_info);
    b.act = nullptr;
    b.mask = nullptr;
    b.stats = (unsigned long long*)(w + h->lay.stats);
    b.estats = (float*)(w + h->lay.estats);
    b.rcomp = (float*)(w + h->lay.rew_info);
    return b;
}

extern "C" int qs_buffers_get(qs_handle* h, qs_buffers* o) {
    if (!h || !o) return fail(QS_E_INVALID, "NULL argument");
    qs::Bufs b = bufs_of(h);
    o->state = b.st; o->istate = b.ist; o->env = b.env; o->env_f = b.envf; o->obst = (float*)b.obst; o->stale_vel = b.stale;
    o->obs = b.obs; o->term_obs = b.term; o->rew = b.rew; o->done = b.done; o->reset_info = b.rinfo;
    o->stats = (uint64_t*)b.stats;
    o->estats = h->cfg.episode_stats ? b.estats : nullptr;
    o->rew_info = h->cfg.step_infos ? b.rcomp : nullptr;
    return QS_OK;
}

static int launch(qs_handle* h, bool step, const float* act, const uint8_t* mask, hipStream_t s) {
    qs::Bufs b = bufs_of(h);
    b.act = act;
    b.mask = mask;
    const qs::KP* kpd = (const qs::KP*)((char*)h->ws + h->lay.params);
    const int epb = envs_per_block(h->cfg, h->npad, step, h->qb, h->qa);
    const dim3 grid((unsigned)((h->kp.E + epb - 1) / epb)), block((unsigned)block_threads(h->cfg, h->npad, step, h->qb, h->qa));
    const size_t shm = shm_bytes(h->cfg, h->kp.obs_dim, h->npad, step, h->qb, h->qa);
    const bool a = h->cfg.flavor == QS_FLAVOR_A, ob = h->kp.obst != 0;
    // the flavor-B step kernel runs the replay wrapper in its tail (qs_replay.h); rb.ri == NULL: replay off
    const qs::RArgs* ra = rargs_of(h);
    if (hipFunction_t f = step ? h->jit_step : h->jit_reset) {
        void* args[] = {(void*)&kpd, (void*)&b, (void*)&ra};   // the last one: B step only
        QS_HIP(hipModuleLaunchKernel(f, grid.x, 1, 1, block.x, 1, 1, (unsigned)shm, s, args, nullptr));
        return QS_OK;
    }
#define QS_LAUNCH(NP)                                                                                           \
    case NP:                                                                                                   \
        if (a) {                                                                                               \
            if (step) hipLaunchKernelGGL(qs::step_kernel_a<NP>, grid, block, shm, s, kpd, b);                  \
            else hipLaunchKernelGGL(qs::reset_kernel_a<NP>, grid, block, shm, s, kpd, b);                      \
        } else if (ob) {                                                                                       \
            if (step) hipLaunchKernelGGL((qs::step_kernel<NP, true>), grid, block, shm, s, kpd, b, ra);        \
            else hipLaunchKernelGGL((qs::reset_kernel<NP, true>), grid, block, shm, s, kpd, b);                \
        } else {                                                                                               \
            if (step) hipLaunchKernelGGL((qs::step_kernel<NP, false>), grid, block, shm, s, kpd, b, ra);       \
            else hipLaunchKernelGGL((qs::reset_kernel<NP, false>), grid, block, shm, s, kpd, b);               \
        }                                                                                                      \
        break;
    switch (h->npad) {
        QS_LAUNCH(1)
        QS_LAUNCH(2)
        QS_LAUNCH(4)
        QS_LAUNCH(8)
        QS_LAUNCH(16)
        QS_LAUNCH(32)
        QS_LAUNCH(64)
        case 128:   // flavor A, or flavor B without obstacles (validate)
            if (a) {
                if (step) hipLaunchKernelGGL(qs::step_kernel_a<128>, grid, block, shm, s, kpd, b);
                else hipLaunchKernelGGL(qs::reset_kernel_a<128>, grid, block, shm, s, kpd, b);
            } else {
                if (step) hipLaunchKernelGGL((qs::step_kernel<128, false>), grid, block, shm, s, kpd, b, ra);
                else hipLaunchKernelGGL((qs::reset_kernel<128, false>), grid, block, shm, s, kpd, b);
            }
            break;
        default:
            return fail(QS_E_UNSUPPORTED, "num_agents not supported");
    }
#undef QS_LAUNCH
    QS_HIP(hipGetLastError());
    return QS_OK;
}

// the replay wavefront per env after the step / reset kernel (qs_replay.h)
static int launch_replay(qs_handle* h, bool step, const uint8_t* mask, hipStream_t s) {
    qs::Bufs b = bufs_of(h);
    b.mask = mask;
    const qs::KP* kpd = (const qs::KP*)((char*)h->ws + h->lay.params);
    constexpr int epb = 256 / qs::RL;   // envs per workgroup
    const dim3 grid((unsigned)((h->kp.E + epb - 1) / epb)), block(256);
    if (step) hipLaunchKernelGGL(qs::replay_kernel<true>, grid, block, 0, s, kpd, b, h->rb, h->rp);
    else hipLaunchKernelGGL(qs::replay_kernel<false>, grid, block, 0, s, kpd, b, h->rb, h->rp);
    QS_HIP(hipGetLastError());
    return QS_OK;
}

static size_t snap_words(const qs_config* c, int obs_dim) {
    const size_t M = c->use_obstacles ? (size_t)obst_slots(c) : 0;
    const size_t N = (size_t)c->num_agents;
    return N * (QS_NF + QS_NI + 3 + (size_t)obs_dim) + QS_NE + QS_NENVF + 2 * M;
}

extern "C" int qs_replay_config_default(qs_replay_config* rc, float control_dt) {
    if (!rc || !(control_dt > 0.f)) return fail(QS_E_INVALID, "NULL config or control_dt <= 0");
    const double freq = 1.0 / (double)control_dt;      // control_freq (quadrotor_single.py: sim_freq / sim_steps)
    rc->sample_prob = 0.75f;                           // the reference's runs (runs/quad_multi_mix_baseline.py:17)
    rc->buffer_size = 20;
    rc->keep = 6;                                      // int(3.0 / 0.5)
    rc->steps_ago = 3;                                 // int(1.5 / 0.5)
    rc->cp_every = (int32_t)llround(0.5 * freq);
    rc->grace_ticks = (int32_t)floor(1.5 * freq + 1e-9);
    rc->min_gap_ticks = (int32_t)floor(5.0 * freq + 1e-9);
    rc->max_replays = 10;
    rc->hist_len = 100;
    rc->hist_min = 10;
    return QS_OK;
}

struct ReplayOffsets { size_t ri, crash, hist, perm, nrep, store, total; };
static ReplayOffsets replay_offsets(const qs_handle* h, const qs_replay_config* rc) {
    const size_t E = (size_t)h->cfg.num_envs, W = snap_words(&h->cfg, h->lay.obs_dim);
    const size_t slots = (size_t)rc->keep + (size_t)rc->buffer_size;
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    ReplayOffsets o;
    o.ri = 0;
    o.crash = al(o.ri + 4 * QS_NR * E);
    o.hist = al(o.crash + 8 * E);
    o.perm = al(o.hist + 8 * (size_t)rc->hist_len * E);
    o.nrep = al(o.perm + 4 * (size_t)rc->buffer_size * E);
    o.store = al(o.nrep + 4 * (size_t)rc->buffer_size * E);
    o.total = al(o.store + 4 * E * slots * W);
    return o;
}

static int replay_check(const qs_handle* h, const qs_replay_config* rc) {
    if (!h || !rc) return fail(QS_E_INVALID, "NULL argument");
    if (h->cfg.flavor != QS_FLAVOR_B) return fail(QS_E_UNSUPPORTED, "experience replay is implemented for flavor B");
    if (rc->buffer_size < 1 || rc->buffer_size > 1024 || rc->keep < 1 || rc->keep > 1024 || rc->steps_ago < 1 ||
        rc->cp_every < 1 || rc->max_replays < 1 || rc->hist_len < 1 || rc->hist_len > 4096 || rc->hist_min < 0 ||
        !(rc->sample_prob >= 0.f && rc->sample_prob <= 1.f))
        return fail(QS_E_INVALID, "replay config out of range");
    return QS_OK;
}

extern "C" int qs_replay_workspace_bytes(qs_handle* h, const qs_replay_config* rc, size_t* bytes) {
    int r = replay_check(h, rc);
    if (r) return r;
    if (!bytes) return fail(QS_E_INVALID, "NULL argument");
    *bytes = replay_offsets(h, rc).total;
    return QS_OK;
}

extern "C" int qs_replay_enable(qs_handle* h, const qs_replay_config* rc, void* d_workspace) {
    int r = replay_check(h, rc);
    if (r) return r;
    if (d_workspace && ((uintptr_t)d_workspace & 255) != 0) return fail(QS_E_INVALID, "workspace must be 256-byte aligned");
    QS_HIP(use_device(h));
    QS_HIP(hipDeviceSynchronize());
    replay_free(h);
    const size_t E = (size_t)h->cfg.num_envs, W = snap_words(&h->cfg, h->lay.obs_dim);
    const ReplayOffsets off = replay_offsets(h, rc);
    hipError_t e = hipSuccess;
    if (d_workspace) {
        h->rws = d_workspace;
        h->rws_owned = false;
    } else {
        e = hipMalloc(&h->rws, off.total);
        if (e != hipSuccess) { h->rws = nullptr; return fail(QS_E_HIP, std::string("hipMalloc(replay): ") + hipGetErrorString(e)); }
        h->rws_owned = true;
    }
    const size_t total = off.total;
    const size_t o_ri = off.ri, o_crash = off.crash, o_hist = off.hist, o_perm = off.perm, o_nrep = off.nrep,
                 o_store = off.store;
    char* w = (char*)h->rws;
    h->rb.ri = (int32_t*)(w + o_ri);
    h->rb.crash = (double*)(w + o_crash);
    h->rb.hist = (double*)(w + o_hist);
    h->rb.perm = (int32_t*)(w + o_perm);
    h->rb.nrep = (int32_t*)(w + o_nrep);
    h->rb.store = (uint32_t*)(w + o_store);
    h->rp.prob = rc->sample_prob;
    h->rp.bufsz = rc->buffer_size;
    h->rp.keep = rc->keep;
    h->rp.steps_ago = rc->steps_ago;
    h->rp.cp_every = rc->cp_every;
    h->rp.grace = rc->grace_ticks;
    h->rp.gap = rc->min_gap_ticks;
    h->rp.max_rep = rc->max_replays;
    h->rp.hist_len = rc->hist_len;
    h->rp.hist_min = rc->hist_min;
    h->rp.W = (int)W;
    // initial wrapper state: identity deque map, no last add, no restore / push yet
    std::vector<int32_t> ri((size_t)QS_NR * E, 0), perm((size_t)rc->buffer_size * E);
    for (size_t x = 0; x < E; ++x) {
        ri[QS_R_LAST_ADD * E + x] = qs::LAST_ADD_NONE;
        ri[QS_R_RESTORED * E + x] = -1;
        ri[QS_R_PUSHED * E + x] = -1;
    }
    for (int p = 0; p < rc->buffer_size; ++p)
        for (size_t x = 0; x < E; ++x) perm[(size_t)p * E + x] = p;
    e = hipMemset(h->rws, 0, total);
    if (e == hipSuccess) e = hipMemcpy(h->rb.ri, ri.data(), 4 * ri.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(h->rb.perm, perm.data(), 4 * perm.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = rargs_sync(h);            // the step kernel's replay arguments (replay on)
    if (e == hipSuccess) e = hipDeviceSynchronize();   // null-stream init complete before any caller stream
    if (e != hipSuccess) {
        replay_free(h);
        return fail(QS_E_HIP, std::string("replay init: ") + hipGetErrorString(e));
    }
    return QS_OK;
}

extern "C" int qs_replay_disable(qs_handle* h) {
    if (!h) return fail(QS_E_INVALID, "handle is NULL");
    QS_HIP(use_device(h));
    QS_HIP(hipDeviceSynchronize());
    replay_free(h);
    return QS_OK;
}

extern "C" int qs_replay_buffers_get(qs_handle* h, qs_replay_buffers* o) {
    if (!h || !o) return fail(QS_E_INVALID, "NULL argument");
    if (!h->rws) return fail(QS_E_INVALID, "replay is not enabled");
    o->ri = h->rb.ri;
    o->crash = h->rb.crash;
    o->hist = h->rb.hist;
    o->perm = h->rb.perm;
    o->nrep = h->rb.nrep;
    o->store = h->rb.store;
    o->snap_words = (size_t)h->rp.W;
    return QS_OK;
}

extern "C" int qs_reset(qs_handle* h, const uint8_t* d_mask, void* stream) {
    if (!h) return fail(QS_E_INVALID, "handle is NULL");
    QS_HIP(use_device(h));
    int rc = launch(h, false, nullptr, d_mask, (hipStream_t)stream);
    if (rc == QS_OK && h->rws) rc = launch_replay(h, false, d_mask, (hipStream_t)stream);
    return rc;
}

static int check_actions(const qs_handle* h, const float* d_actions) {
    if (!h || !d_actions) return fail(QS_E_INVALID, "NULL argument");
    if (h->cfg.flavor == QS_FLAVOR_A) {
        if (((uintptr_t)d_actions & 7) != 0) return fail(QS_E_INVALID, "actions must be 8-byte aligned [I,2] fp32");
    } else if (((uintptr_t)d_actions & 15) != 0) {
        return fail(QS_E_INVALID, "actions must be 16-byte aligned [I,4] fp32");
    }
    return QS_OK;
}

extern "C" int qs_step(qs_handle* h, const float* d_actions, void* stream) {
    if (int rc = check_actions(h, d_actions)) return rc;
    QS_HIP(use_device(h));
    // with replay on, the flavor-B step kernel runs the wrapper in its tail (no second launch)
    return launch(h, true, d_actions, nullptr, (hipStream_t)stream);
}

extern "C" int qs_step_n(qs_handle* h, const float* d_actions, int steps, void* stream) {
    if (steps < 1) return fail(QS_E_INVALID, "qs_step_n: steps < 1");
    if (int rc = check_actions(h, d_actions)) return rc;
    QS_HIP(use_device(h));
    for (int i = 0; i < steps; ++i)
        if (int rc = launch(h, true, d_actions, nullptr, (hipStream_t)stream)) return rc;
    return QS_OK;
}

extern "C" int qs_step_blocks(qs_handle* const* hs, int n, const float* const* d_actions, void* const* streams) {
    if (!hs || !d_actions || !streams || n < 1) return fail(QS_E_INVALID, "NULL argument or n < 1");
    for (int i = 0; i < n; ++i) {
        if (int rc = check_actions(hs[i], d_actions[i])) return rc;
        if (hs[i]->device != hs[0]->device) return fail(QS_E_INVALID, "qs_step_blocks: handles on different devices");
    }
    QS_HIP(use_device(hs[0]));
    for (int i = 0; i < n; ++i)
        if (int rc = launch(hs[i], true, d_actions[i], nullptr, (hipStream_t)streams[i])) return rc;
    return QS_OK;
}

extern "C" int qs_counters(qs_handle* h, qs_stats* out, void* stream) {
    if (!h || !out) return fail(QS_E_INVALID, "NULL argument");
    QS_HIP(use_device(h));
    uint64_t v[QS_NSTAT];
    QS_HIP(hipMemcpyAsync(v, (char*)h->ws + h->lay.stats, sizeof v, hipMemcpyDeviceToHost, (hipStream_t)stream));
    QS_HIP(hipStreamSynchronize((hipStream_t)stream));
    out->nonfinite_obs = v[QS_ST_OBS];
    out->nonfinite_rew = v[QS_ST_REW];
    out->nonfinite_state = v[QS_ST_STATE];
    out->reserved = 0;
    return QS_OK;
}

extern "C" int qs_counters_reset(qs_handle* h, void* stream) {
    if (!h) return fail(QS_E_INVALID, "NULL argument");
    QS_HIP(use_device(h));
    QS_HIP(hipMemsetAsync((char*)h->ws + h->lay.stats, 0, sizeof(uint64_t) * QS_NSTAT, (hipStream_t)stream));
    return QS_OK;
}

static float* param_slot(qs_handle* h, const char* key) {
    qs::KP& k = h->kp;
    struct { const char* n; float* p; } t[] = {
        {"rew_pos", &k.rew_pos}, {"rew_effort", &k.rew_effort}, {"rew_crash", &k.rew_crash},
        {"rew_orient", &k.rew_orient}, {"rew_spin", &k.rew_spin}, {"quadcol_bin", &k.quadcol},
        {"quadcol_bin_smooth_max", &k.prox_max}, {"quadcol_bin_obst", &k.quadcol_obst}};
    for (auto& e : t)
        if (strcmp(e.n, key) == 0) return e.p;
    return nullptr;
}

static int upload_params(qs_handle* h) {
    QS_HIP(use_device(h));
    QS_HIP(hipDeviceSynchronize());   // launches in flight read the old block
    QS_HIP(hipMemcpy((char*)h->ws + h->lay.params, &h->kp, sizeof(qs::KP), hipMemcpyHostToDevice));
    return QS_OK;
}

// Parameters live in device memory (read by every launch), so a change also reaches launches that
// are replayed from a captured hipGraph.
static int set_capture_radius(qs_handle* h, float v) {
    if (h->cfg.flavor != QS_FLAVOR_A) return fail(QS_E_INVALID, "capture_radius is a flavor-A parameter");
    QS_HIP(use_device(h));
    QS_HIP(hipDeviceSynchronize());
    std::vector<float> cr((size_t)h->cfg.num_envs, v);
    QS_HIP(hipMemcpy((char*)h->ws + h->lay.env_f + sizeof(float) * QS_ENVF_CAPTURE * (size_t)h->cfg.num_envs, cr.data(),
                     sizeof(float) * cr.size(), hipMemcpyHostToDevice));
    h->cfg.capture_radius = v;
    return QS_OK;
}

extern "C" int qs_set_param(qs_handle* h, const char* key, double v) {
    if (!h || !key) return fail(QS_E_INVALID, "NULL argument");
    if (strcmp(key, "capture_radius") == 0) return set_capture_radius(h, (float)v);
    if (strcmp(key, "ep_len") == 0) { h->kp.ep_len = (int)v; h->cfg.ep_len = (int)v; return upload_params(h); }
    if (strcmp(key, "seed") == 0) { h->kp.seed = h->cfg.seed = (uint32_t)v; return upload_params(h); }
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
    if (strcmp(key, "seed") == 0) { *v = h->kp.seed; return QS_OK; }
    if (strcmp(key, "capture_radius") == 0) {   // env 0's radius (set per env through buffers.env_f)
        if (h->cfg.flavor != QS_FLAVOR_A) return fail(QS_E_INVALID, "capture_radius is a flavor-A parameter");
        float r;
        QS_HIP(use_device(h));
        QS_HIP(hipMemcpy(&r, (char*)h->ws + h->lay.env_f + sizeof(float) * QS_ENVF_CAPTURE * (size_t)h->cfg.num_envs,
                         sizeof(float), hipMemcpyDeviceToHost));
        *v = r;
        return QS_OK;
    }
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
    QS_HIP(use_device(h));
    QS_HIP(hipMemcpyAsync(dst, (char*)h->ws + h->lay.state, qs_state_bytes(h), hipMemcpyDeviceToHost,
                          (hipStream_t)stream));
    QS_HIP(hipStreamSynchronize((hipStream_t)stream));
    return QS_OK;
}

extern "C" int qs_set_state(qs_handle* h, const void* src, size_t bytes, void* stream) {
    if (!h || !src) return fail(QS_E_INVALID, "NULL argument");
    if (bytes < qs_state_bytes(h)) return fail(QS_E_INVALID, "buffer too small");
    QS_HIP(use_device(h));
    QS_HIP(hipMemcpyAsync((char*)h->ws + h->lay.state, src, qs_state_bytes(h), hipMemcpyHostToDevice,
                          (hipStream_t)stream));
    QS_HIP(hipStreamSynchronize((hipStream_t)stream));
    return QS_OK;
}

// GAE over a device rollout (qs_gae.h); all pointers device memory, [T, I] time-major
extern "C" int qs_gae(const float* rewards, const float* values, const uint8_t* episode_starts,
                      const float* last_values, const uint8_t* last_dones, float* advantages, float* returns,
                      int32_t n_steps, int32_t n_cols, float gamma, float gae_lambda, void* stream) {
    if (!rewards || !values || !episode_starts || !last_values || !last_dones || !advantages || !returns)
        return fail(QS_E_INVALID, "NULL argument");
    if (n_steps < 1 || n_cols < 1) return fail(QS_E_INVALID, "n_steps and n_cols must be >= 1");
    const dim3 block(256), grid((unsigned)((n_cols + 255) / 256));
    hipLaunchKernelGGL(qs::gae_kernel, grid, block, 0, (hipStream_t)stream, rewards, values, episode_starts,
                       last_values, last_dones, advantages, returns, n_steps, n_cols, gamma, gae_lambda);
    QS_HIP(hipGetLastError());
    return QS_OK;
}

// capture-radius curriculum (qs_curriculum.h)
extern "C" int qs_curriculum_init(qs_curriculum* c, double initial_radius, double sr_threshold, double decay,
                                  int32_t window) {
    if (!c) return fail(QS_E_INVALID, "NULL argument");
    if (window < 1 || window > QS_CUR_MAX_WINDOW) return fail(QS_E_INVALID, "curriculum window must be 1..64");
    if (!(initial_radius > 0.0) || !(decay > 0.0)) return fail(QS_E_INVALID, "radius and decay must be > 0");
    memset(c, 0, sizeof *c);
    c->radius = initial_radius;
    c->sr_threshold = sr_threshold;
    c->decay = decay;
    c->window = window;
    return QS_OK;
}

extern "C" int qs_curriculum_step(qs_handle* h, qs_curriculum* d_cur, void* stream) {
    if (!h || !d_cur) return fail(QS_E_INVALID, "NULL argument");
    if (h->cfg.flavor != QS_FLAVOR_A) return fail(QS_E_INVALID, "the capture-radius curriculum is flavor A");
    QS_HIP(use_device(h));
    const uint8_t* ri = (const uint8_t*)((char*)h->ws + h->lay.reset_info);
    float* cap = (float*)((char*)h->ws + h->lay.env_f) + (size_t)QS_ENVF_CAPTURE * (size_t)h->cfg.num_envs;
    hipLaunchKernelGGL(qs::curriculum_kernel, dim3(1), dim3(qs::QS_CUR_THREADS), 0, (hipStream_t)stream, ri, cap,
                       (int)h->cfg.num_envs, (int)h->cfg.num_envs, d_cur);
    QS_HIP(hipGetLastError());
    return QS_OK;
}

extern "C" int qs_curriculum_step_all(qs_handle* h, const uint8_t* d_reset_all, int64_t n_all, qs_curriculum* d_cur,
                                      void* stream) {
    if (!h || !d_cur || !d_reset_all) return fail(QS_E_INVALID, "NULL argument");
    if (h->cfg.flavor != QS_FLAVOR_A) return fail(QS_E_INVALID, "the capture-radius curriculum is flavor A");
    if (n_all < (int64_t)h->cfg.num_envs || n_all > (int64_t)INT32_MAX)
        return fail(QS_E_INVALID, "n_all must cover at least the handle's envs (world * num_envs)");
    QS_HIP(use_device(h));
    float* cap = (float*)((char*)h->ws + h->lay.env_f) + (size_t)QS_ENVF_CAPTURE * (size_t)h->cfg.num_envs;
    hipLaunchKernelGGL(qs::curriculum_kernel, dim3(1), dim3(qs::QS_CUR_THREADS), 0, (hipStream_t)stream, d_reset_all,
                       cap, (int)n_all, (int)h->cfg.num_envs, d_cur);
    QS_HIP(hipGetLastError());
    return QS_OK;
}

// the kernel parameter block a config produces (host only; runtime specialisation / diagnostics)
extern "C" int qs_config_kp_words(const qs_config* c, uint32_t* out, size_t n_words) {
    if (!c || !out) return fail(QS_E_INVALID, "NULL argument");
    int rc = validate(c);
    if (rc) return rc;
    if (n_words < sizeof(qs::KP) / 4) return fail(QS_E_INVALID, "buffer too small for the parameter block");
    const qs::KP k = make_kp(c, make_layout(c));
    memcpy(out, &k, sizeof(qs::KP));
    return (int)(sizeof(qs::KP) / 4);
}

// ---------------------------------------------------------------------------------------------
// Runtime specialisation (hipRTC).  The step/reset kernels are recompiled with this handle's whole
// parameter block as a compile-time constant (QS_JIT, qs_common.h bind_kp): physical constants fold
// into the instructions, config branches and unused feature paths vanish, and the kernel stops paying
// scalar-cache round trips for parameters.  Fields qs_set_param may change stay in device memory.
// Modules are cached per (device, parameter block, kernel) for the process lifetime.
// ---------------------------------------------------------------------------------------------
#include "qs_jit_sources.inc"

namespace {
struct JitEntry {
    hipModule_t mod = nullptr;
    hipFunction_t step = nullptr, reset = nullptr;
};
std::mutex g_jit_mu;
std::map<std::string, JitEntry> g_jit_cache;
}  // namespace

static std::string kernel_names(const qs_config* c, const qs::KP& kp, int npad, std::string* reset) {
    const std::string np = std::to_string(npad);
    if (c->flavor == QS_FLAVOR_A) {
        *reset = "qs::reset_kernel_a<" + np + ">";
        return "qs::step_kernel_a<" + np + ">";
    }
    const char* ob = kp.obst ? "true" : "false";
    *reset = "qs::reset_kernel<" + np + ", " + ob + ">";
    return "qs::step_kernel<" + np + ", " + ob + ">";
}

static std::string kp_words(const qs::KP& kp_in) {
    qs::KP kp = kp_in;
    kp.seed = 0;   // read per launch (KPM): one compiled module serves every seed
    std::string words;
    const uint32_t* w = reinterpret_cast<const uint32_t*>(&kp);
    char buf[16];
    for (size_t i = 0; i < sizeof(qs::KP) / 4; ++i) {
        snprintf(buf, sizeof buf, "0x%08xu,", w[i]);
        words += buf;
    }
    words.pop_back();
    return words;
}

static std::vector<std::string> jit_extra_opts() {
    std::vector<std::string> v;
    if (const char* e = getenv("QS_JIT_OPTS")) {
        std::string cur;
        for (const char* p = e;; ++p) {
            if (*p == ' ' || *p == '\0') {
                if (!cur.empty()) v.push_back(cur);
                cur.clear();
                if (!*p) break;
            } else {
                cur += *p;
            }
        }
    }
    return v;
}

// hipRTC compile of the step/reset kernels for one parameter block (host only)
static int jit_compile(const qs_config* c, const qs::KP& kp, int npad, int qb, int qa, std::vector<char>& code,
                       std::string& lstep, std::string& lreset) {
    std::string reset_name;
    const std::string step_name = kernel_names(c, kp, npad, &reset_name);
    std::string src =
        "typedef __hip_internal::uint8_t uint8_t;\n"
        "typedef __hip_internal::int8_t int8_t;\n"
        "typedef __hip_internal::uint16_t uint16_t;\n"
        "typedef __hip_internal::int16_t int16_t;\n"
        "typedef __hip_internal::uint32_t uint32_t;\n"
        "typedef __hip_internal::int32_t int32_t;\n"
        "typedef __hip_internal::uint64_t uint64_t;\n"
        "typedef __hip_internal::int64_t int64_t;\n"
        "typedef unsigned long uintptr_t;\n"
        "#define QS_JIT 1\n#define QS_QB " + std::to_string(qb) + "\n#define QS_QA " + std::to_string(qa) +
        "\n#define QS_QW " + std::to_string(QS_QW) + "\n#define QS_KP_WORDS " + kp_words(kp) + "\n";
    src += c->flavor == QS_FLAVOR_A ? "#include \"qs_flavor_a.h\"\n" : "#include \"qs_flavor_b.h\"\n";
    // the kernel sources embedded at build time, or (QS_JIT_SRC_DIR, kernel-variant A/B experiments) the same
    // header names read from that directory
    std::vector<std::string> dir_src;
    std::vector<const char*> hsrc(kJitHeaderSources, kJitHeaderSources + kJitNumHeaders);
    if (const char* dir = getenv("QS_JIT_SRC_DIR")) {
        for (int i = 0; i < kJitNumHeaders; ++i) {
            std::string path = std::string(dir) + "/" + kJitHeaderNames[i];
            FILE* f = fopen(path.c_str(), "rb");
            if (!f) return fail(QS_E_INVALID, "QS_JIT_SRC_DIR: cannot read " + path);
            std::string txt;
            char chunk[4096];
            for (size_t n; (n = fread(chunk, 1, sizeof chunk, f)) > 0;) txt.append(chunk, n);
            fclose(f);
            dir_src.push_back(txt);
        }
        // The host launches the directory's kernels with THIS library's argument list and workspace layout.  A
        // source tree of another ABI (e.g. round 4's step kernel, which still took the replay wrapper's pointers
        // as kernel arguments, under the ABI-13 host that passes them in the RArgs device block) reads its
        // pointers from the wrong kernarg offsets and faults (round 5, hipErrorIllegalAddress):
        // the directory's quadswarm.h must carry this library's QS_ABI_VERSION.
        int dir_abi = -1;
        for (int i = 0; i < kJitNumHeaders; ++i) {
            if (std::string(kJitHeaderNames[i]) != "quadswarm.h") continue;
            const std::string& t = dir_src[i];
            const size_t p = t.find("#define QS_ABI_VERSION");
            if (p != std::string::npos) dir_abi = atoi(t.c_str() + p + sizeof("#define QS_ABI_VERSION") - 1);
        }
        if (dir_abi != QS_ABI_VERSION)
            return fail(QS_E_INVALID, "QS_JIT_SRC_DIR: " + std::string(dir) + "/quadswarm.h has QS_ABI_VERSION " +
                                          std::to_string(dir_abi) + ", this library is ABI " +
                                          std::to_string(QS_ABI_VERSION) + " (kernel arguments would not match)");
        for (int i = 0; i < kJitNumHeaders; ++i) hsrc[i] = dir_src[i].c_str();
    }
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, src.c_str(), "qs_jit.hip", kJitNumHeaders, hsrc.data(), kJitHeaderNames) !=
        HIPRTC_SUCCESS)
        return fail(QS_E_HIP, "hiprtcCreateProgram failed");
    hiprtcAddNameExpression(prog, step_name.c_str());
    hiprtcAddNameExpression(prog, reset_name.c_str());
    std::vector<const char*> opts = {"--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=on",
                                     "-munsafe-fp-atomics"};
    // Code generation measured on MI355X (tools/opts_ab.sh, profiles/ab/r03_jit_opts_ab.txt; every variant
    // bitwise identical): the ILP-first machine scheduler for both flavors, and for flavor B no SLP packing
    // of fp32 math into v_pk_* (the packing's operand moves cost more issue slots than the pairs save at 2
    // waves per SIMD).  C3 8.69 -> 8.19 us, C5 15.2 -> 13.4, C4 12.0 -> 11.2, C2 5.69 -> 5.55, a8 27.2 -> 26.3.
    // Flavor A kept the packing in round 3; on the round-4 kernel it loses there too (a8 23.82 -> 23.60,
    // 23.69 -> 23.49 us, profiles/ab/r04_a8_noslp_ab.txt), so no flavor packs.
    opts.push_back("-mllvm");
    opts.push_back("-amdgpu-sched-strategy=max-ilp");
    opts.push_back("-fno-slp-vectorize");
    // Flavor A: fp32 denormals flushed (no denormal scaling around the transcendentals of the controller and the
    // camera model).  Bitwise identical digests on a8 and C3 / C2 (no denormal reaches a result), a8 21.31 -> 21.10
    // us, C3 / C2 neutral (profiles/ab/r06_fp_opts_ab.txt): flavor A only.
    if (c->flavor == QS_FLAVOR_A) opts.push_back("-fgpu-flush-denormals-to-zero");
    // (flavor A kept DPP permutes without bound_ctrl in round 3; on the round-4 kernel bound_ctrl is as good or
    // better there too, a8 23.54 -> 23.37, 23.48 -> 23.41 us, profiles/ab/r04_a8_dpp_bc_ab.txt: one form for both)
    // QS_JIT_OPTS: extra space-separated hipRTC options (kernel-variant experiments, e.g. -DQS_X=1).  The launch
    // geometry (sub-lanes per drone) is the host's: block_threads / envs_per_block size the launch from it, so a
    // kernel compiled with another QS_QB / QS_QA / QS_QW would index envs and LDS differently -- refused here.
    std::vector<std::string> extra = jit_extra_opts();
    for (const std::string& o : extra)
        for (const char* geo : {"QS_QB", "QS_QA", "QS_QW", "QS_JIT", "QS_KP_WORDS"})
            if (o.find(geo) != std::string::npos)
                return fail(QS_E_INVALID, std::string("QS_JIT_OPTS may not set ") + geo +
                                              " (launch geometry comes from the host; use the QS_QB / QS_QA env vars)");
    for (const std::string& o : extra) opts.push_back(o.c_str());
    const hiprtcResult rc = hiprtcCompileProgram(prog, (int)opts.size(), opts.data());
    if (rc != HIPRTC_SUCCESS) {
        size_t n = 0;
        hiprtcGetProgramLogSize(prog, &n);
        std::string log(n + 1, '\0');
        hiprtcGetProgramLog(prog, &log[0]);
        hiprtcDestroyProgram(&prog);
        return fail(QS_E_HIP, std::string("hipRTC compile failed: ") + hiprtcGetErrorString(rc) + "\n" + log);
    }
    const char *ls = nullptr, *lr = nullptr;
    hiprtcGetLoweredName(prog, step_name.c_str(), &ls);
    hiprtcGetLoweredName(prog, reset_name.c_str(), &lr);
    lstep = ls ? ls : "";
    lreset = lr ? lr : "";
    size_t code_n = 0;
    hiprtcGetCodeSize(prog, &code_n);
    code.resize(code_n);
    if (code_n) hiprtcGetCode(prog, code.data());
    hiprtcDestroyProgram(&prog);
    if (lstep.empty() || lreset.empty() || code.empty()) return fail(QS_E_HIP, "hipRTC produced no kernels");
    return QS_OK;
}

// sub-lanes per drone of the specialised step kernels: the build default, or QS_QB / QS_QA (1, 2, 4) from the
// environment (geometry experiments; the results are bitwise the same for every Q)
static void jit_lanes(int* qb, int* qa) {
    *qb = QS_QB;
    *qa = QS_QA;
    for (auto kv : {std::make_pair("QS_QB", qb), std::make_pair("QS_QA", qa)})
        if (const char* v = getenv(kv.first)) {
            const int x = atoi(v);
            if (x == 1 || x == 2 || x == 4 || (x == 8 && kv.second == qb)) *kv.second = x;   // 8: single-drone envs
        }
}

extern "C" int qs_specialize(qs_handle* h, int enable) {
    if (!h) return fail(QS_E_INVALID, "NULL handle");
    if (!enable) {
        h->jit_step = h->jit_reset = nullptr;
        h->jit_mod = nullptr;
        h->qb = QS_QB;
        h->qa = QS_QA;
        return QS_OK;
    }
    QS_HIP(use_device(h));
    int qb, qa;
    jit_lanes(&qb, &qa);
    if (shm_bytes(h->cfg, h->lay.obs_dim, h->npad, true, qb, qa) > QS_LDS_MAX)
        return fail(QS_E_UNSUPPORTED, "QS_QB / QS_QA geometry exceeds the 160 KB of LDS of a workgroup");
    std::string rn;
    const std::string key = std::to_string(h->device) + "|" + kernel_names(&h->cfg, h->kp, h->npad, &rn) + "|" +
                            std::to_string(qb) + "," + std::to_string(qa) + "|" +
                            (getenv("QS_JIT_OPTS") ? getenv("QS_JIT_OPTS") : "") + "|" +
                            (getenv("QS_JIT_SRC_DIR") ? getenv("QS_JIT_SRC_DIR") : "") + "|" + kp_words(h->kp);
    std::lock_guard<std::mutex> lock(g_jit_mu);
    auto it = g_jit_cache.find(key);
    if (it == g_jit_cache.end()) {
        std::vector<char> code;
        std::string lstep, lreset;
        if (int rc = jit_compile(&h->cfg, h->kp, h->npad, qb, qa, code, lstep, lreset)) return rc;
        JitEntry e;
        QS_HIP(hipModuleLoadData(&e.mod, code.data()));
        QS_HIP(hipModuleGetFunction(&e.step, e.mod, lstep.c_str()));
        QS_HIP(hipModuleGetFunction(&e.reset, e.mod, lreset.c_str()));
        it = g_jit_cache.emplace(key, e).first;
    }
    h->jit_step = it->second.step;
    h->jit_reset = it->second.reset;
    h->jit_mod = it->second.mod;
    h->qb = qb;
    h->qa = qa;
    return QS_OK;
}

// host-only check that a config's specialised kernels compile; returns the code-object size in bytes
extern "C" long long qs_specialize_compile(const qs_config* c) {
    if (!c) return fail(QS_E_INVALID, "NULL argument");
    if (int rc = validate(c)) return rc;
    const qs::KP kp = make_kp(c, make_layout(c));
    std::vector<char> code;
    std::string ls, lr;
    int qb, qa;
    jit_lanes(&qb, &qa);
    if (int rc = jit_compile(c, kp, npad_of(c->num_agents), qb, qa, code, ls, lr)) return rc;
    if (const char* dump = getenv("QS_JIT_DUMP")) {   // diagnostics: write the code object for llvm-objdump
        if (FILE* f = fopen(dump, "wb")) {
            fwrite(code.data(), 1, code.size(), f);
            fclose(f);
        }
    }
    return (long long)code.size();
}

// 1 when the handle launches specialised kernels
extern "C" int qs_is_specialized(const qs_handle* h) { return h && h->jit_step ? 1 : 0; }

#ifdef QS_STAMPS
// diagnostics build only: the phase stamps of the kernels this handle launches (tools/phase_stamps.py); a
// specialised handle's kernels write the copy of qs_dbg_stamps in their own hipRTC module
extern "C" int qs_debug_stamps_h(qs_handle* h, uint64_t* host, size_t n) {
    if (!h || !host) return fail(QS_E_INVALID, "NULL argument");
    QS_HIP(use_device(h));
    QS_HIP(hipDeviceSynchronize());
    if (!h->jit_mod) return qs_debug_stamps(host, n);
    hipDeviceptr_t p = nullptr;
    size_t bytes = 0;
    QS_HIP(hipModuleGetGlobal(&p, &bytes, h->jit_mod, "_ZN2qs13qs_dbg_stampsE"));
    QS_HIP(hipMemcpyDtoH(host, p, n * sizeof(uint64_t) < bytes ? n * sizeof(uint64_t) : bytes));
    return QS_OK;
}
#endif
