// qs_common.h -- device-side building blocks shared by the flavor-B and flavor-A step kernels:
// kernel parameters, SoA state I/O, the QuadrotorDynamics substep (quadrotor_dynamics.py:355-656),
// LDS staging helpers and the per-env Philox counter.  Included by qs_step.hip only.
#pragma once
#ifndef __HIPCC_RTC__   // hipRTC (qs_specialize) provides these itself
#include <hip/hip_runtime.h>
#include <stdint.h>
#endif

#include "qs_rng.h"
#include "quadswarm.h"

namespace qs {

// flavor-A neighbour features (get_rel_pos_vel_item, quadrotor_multi_rewards.py:326-420), in the
// reference's concatenation order
enum : int {
    QS_NF_DIST = 1, QS_NF_NDIST = 2, QS_NF_ANGLE = 4, QS_NF_SANGLE = 8, QS_NF_NSANGLE = 16,
    QS_NF_HEADING = 32, QS_NF_SHEADING = 64, QS_NF_NPOS = 128, QS_NF_POS = 256, QS_NF_VEL = 512
};

struct KP {
    int E, N, I, obs_dim, so_dim, K, neighbor, obs_repr, ep_len, sim_steps, svd_every, sense, downwash, collide;
    uint32_t id0;  // global id of drone 0 (RNG key offset)
    uint32_t seed; // Philox seed: read per launch through KPM (qs_set_param("seed") reaches captured graphs)
    float dt, cdt, mass, inv_mass, inertia[3], inv_inertia[3];
    float thrust_max[4], torque_max[4], pc0[4], pc1[4], pc2[4], ccw[4];
    float tau_up, tau_down, lin, arm, grav, omega_max, vel_damp, dq, vxyz_max;
    float mass_g;   // mass * gravity rounded once on the host (the floor friction: the same bits in both builds)
    float room_lo[3], room_hi[3], room_range[3];
    float ou_mu, ou_theta, ou_sigma;
    float pos_std, pos_unif, vel_std, vel_unif, gyro, quat_std, quat_unif;
    float col_thr, fall_thr, prox_ratio, prox_max;
    float rew_pos, rew_effort, rew_crash, rew_orient, rew_spin, quadcol;
    float spawn_box, goal[3];
    // ---- flavor A (quadrotor_multi_rewards + Controller/), host-derived in make_kp ----
    int flavor, scenario, ticks, nfeat, nfd, n_cam;
    float cam_r, cam_f, cam_px, cam_w, cam_res;      // marker radius, focal, pixel sigma, sensor width, px
    float cam_cos[8], cam_sin[8];                     // camera k's axis (cos, sin of k 2 pi / n_cam), host-computed
    float hrate;                                      // dt * MAX_ANGULAR_RATE (Controller.py:29,81)
    float speed, inv_dt;
    float pkp[10], pkd[10], pki[10], psat[10], paw[10];
    float rate_scale, mix[16];
    float m_mass_g, m_mass, m_kf4, m_min_rpm, m_inv_rpm;   // m*g, m, kf*n_motors, min rpm, 1/(max-min)
    float w_captor, w_helper, existence;
    float tgt_vmax, tgt_dt, arena, tgt_z;
    float nclip_lo[8], nclip_hi[8];
    // ---- obstacles (flavor B) ----
    int obst, M, obst_n, obst_scen;                 // on, pillar slots per env, grid side, scenario
    float obst_r, obst_thr, obst_z, sdf_res, quadcol_obst;
    // obstacle domain randomisation (replay wrapper reset): index 0 = configured, choice c = index c + 1;
    // dr_m -1 / dr_r 0 = a falsy 0.0 choice that keeps the env's current value
    int dr, dr_nm, dr_ns, dr_m[9];
    float dr_r[9], dr_thr[9];
    // ---- flavor-B goal scenarios: -1 = the fixed static_same_goal goal, 0..9 a scenario, 10 = mix ----
    int scen_b;
    // ---- episode_extra_stats (flavor B): on; collisions_grace_period_steps (ticks >= settle count), the
    // final-5-s window (time_remain <= final), distance windows of 1 / 3 / 5 s in ticks ----
    int stats, st_settle, st_final, st_win[3];
    // ---- per-step reward components (qs_config.step_infos): the step writes buffers.rew_info
    int rcomp;
};

// The fields qs_set_param may change after creation, read once per launch into registers (uniform):
// kernels use `kpm.` for them so that neither build re-loads them inside loops.
struct KPM {
    int ep_len;
    uint32_t seed;
    float rew_pos, rew_effort, rew_crash, rew_orient, rew_spin, quadcol, prox_max, prox_ratio, quadcol_obst;
};
__device__ __forceinline__ KPM load_kpm(const KP* __restrict__ p) {
    KPM m;
    m.ep_len = p->ep_len;
    m.seed = p->seed;
    m.rew_pos = p->rew_pos;
    m.rew_effort = p->rew_effort;
    m.rew_crash = p->rew_crash;
    m.rew_orient = p->rew_orient;
    m.rew_spin = p->rew_spin;
    m.quadcol = p->quadcol;
    m.prox_max = p->prox_max;
    m.prox_ratio = p->prox_ratio;
    m.quadcol_obst = p->quadcol_obst;
    return m;
}

// Runtime specialisation (qs_specialize, hipRTC): the whole parameter block is a compile-time constant
// object, so every physical constant folds into the instructions and config branches vanish.
#ifdef QS_JIT
struct KPWords { uint32_t w[sizeof(KP) / 4]; };
static_assert(sizeof(KP) % 4 == 0, "KP must be a whole number of words");
__device__ constexpr KP kKP = __builtin_bit_cast(KP, KPWords{{QS_KP_WORDS}});
#define QS_BIND_KP(p)               \
    const KP& kp = kKP;             \
    const KPM kpm = load_kpm(p);    \
    (void)kpm
#else
#define QS_BIND_KP(p)               \
    const KP& kp = *(p);            \
    const KPM kpm = load_kpm(p);    \
    (void)kpm
#endif

struct Bufs {
    float* st;
    int32_t* ist;
    int32_t* env;
    float* envf;
    float2* obst;     // [E, M] obstacle xy
    float* stale;
    float* obs;
    float* term;
    float* rew;
    uint8_t* done;
    uint8_t* rinfo;
    const float* act;
    const uint8_t* mask;
    unsigned long long* stats;   // [QS_NSTAT] non-finite guard counters (qs_counters)
    float* estats;               // [I, QS_NES] episode_extra_stats rows of finished envs
    float* rcomp;                // [QS_NRI, I] the step's reward components (kp.rcomp)
};

// The buffer pointers as VGPR values (QS_VPTR): a step kernel's uniform state outgrows the 102 SGPRs, and the
// compiler then loads the kernel's pointer arguments in small batches, each waited for and spilled to VGPR lanes
// before the next (five kernarg round trips at the start of the flavor-B mix kernel).  Moving them to VGPRs at
// entry issues every argument load at once, waits once, and keeps them out of the SGPR budget (2 VGPRs each; the
// per-lane addresses are VGPR arithmetic anyway).
#ifndef QS_VPTR
#define QS_VPTR 0   // measured slower on every flavor-B config (round 5: C3 8.00 vs 7.47 us); kept for A/B
#endif
template <class T, bool ON = true>
__device__ __forceinline__ void vptr(T*& p) {
#if QS_VPTR
    if constexpr (!ON) return;
    uint64_t x = reinterpret_cast<uint64_t>(p);
    asm volatile("" : "+v"(x));
    // back through a global (address space 1) pointer: the accesses stay global_* (a plain cast would make them
    // generic -> flat_*)
    typedef __attribute__((address_space(1))) T GT;
    p = (T*)(reinterpret_cast<GT*>(x));
#else
    (void)p;
#endif
}
// ON: the kernels whose VGPR budget has the room (flavor B up to 16 drone slots: 181 -> 226 VGPRs at C3, still two
// waves per SIMD; the 32-slot kernel would cross 256 and lose its second wave)
template <bool ON>
__device__ __forceinline__ void vptr_bufs(Bufs& b) {
    vptr<float, ON>(b.st); vptr<int32_t, ON>(b.ist); vptr<int32_t, ON>(b.env); vptr<float, ON>(b.envf);
    vptr<float2, ON>(b.obst); vptr<float, ON>(b.stale); vptr<float, ON>(b.obs); vptr<float, ON>(b.term);
    vptr<float, ON>(b.rew); vptr<uint8_t, ON>(b.done); vptr<uint8_t, ON>(b.rinfo); vptr<const float, ON>(b.act);
    vptr<const uint8_t, ON>(b.mask); vptr<unsigned long long, ON>(b.stats); vptr<float, ON>(b.estats);
    vptr<float, ON>(b.rcomp);
}

// Diagnostic phase stamps (build with -DQS_STAMPS=1 only; never in the shipped library): lane 0 of
// each block records s_memtime at phase boundaries; tools/phase_stamps.py reads them back.  A stamp waits
// for nothing but its own counter read: a phase's time includes the memory waits its own code has.
#ifdef QS_STAMPS
constexpr int QS_NSTAMP = 32;   // slots per block
__device__ uint64_t qs_dbg_stamps[65536 * QS_NSTAMP];
#define QS_STAMP(k)                                                                                   \
    do {                                                                                              \
        uint64_t t_;                                                                                  \
        __builtin_amdgcn_sched_barrier(0);                                                            \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");               \
        __builtin_amdgcn_sched_barrier(0);                                                            \
        stamps_[k] = t_;                                                                              \
    } while (0)
// realtime (100 MHz, chip-wide) stamps in slots 12 (wave start) / 13 (wave end) for the launch timeline
#define QS_RTSTAMP(k)                                                                                 \
    do {                                                                                              \
        uint64_t t_;                                                                                  \
        asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");                \
        stamps_[k] = t_;                                                                              \
    } while (0)
// slots 14 / 15: the wave's HW_ID (wave slot, SIMD, CU, SH, SE) and XCC_ID registers (where it ran)
#define QS_STAMP_FLUSH()                                                                              \
    do {                                                                                              \
        uint32_t hw_, xcc_;                                                                           \
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw_));                            \
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc_));                          \
        stamps_[14] = hw_;                                                                            \
        stamps_[15] = xcc_;                                                                           \
        if (threadIdx.x == 0 && blockIdx.x < 65536)                                                   \
            for (int k_ = 0; k_ < QS_NSTAMP; ++k_) qs_dbg_stamps[blockIdx.x * QS_NSTAMP + k_] = stamps_[k_]; \
    } while (0)
#define QS_STAMP_DECL uint64_t stamps_[QS_NSTAMP] = {0};
// a wave-uniform value in slot k (16..31): what the wave's drones were doing
#define QS_STAMP_NOTE(k, v) do { stamps_[k] = (uint64_t)(v); } while (0)
// accumulating form (phases inside a loop, flavor A's tick loop): slot k += cycles since the previous mark
#define QS_STAMP_ACC_DECL uint64_t stamp_last_ = 0;
#define QS_STAMP_MARK()                                                                               \
    do {                                                                                              \
        __builtin_amdgcn_sched_barrier(0);                                                            \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(stamp_last_)::"memory");          \
        __builtin_amdgcn_sched_barrier(0);                                                            \
    } while (0)
#define QS_STAMP_ACC(k)                                                                               \
    do {                                                                                              \
        uint64_t t_;                                                                                  \
        __builtin_amdgcn_sched_barrier(0);                                                            \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");                   \
        __builtin_amdgcn_sched_barrier(0);                                                            \
        stamps_[k] += t_ - stamp_last_;                                                               \
        stamp_last_ = t_;                                                                             \
    } while (0)
#else
#define QS_STAMP_ACC_DECL
#define QS_STAMP_NOTE(k, v) do {} while (0)
#define QS_STAMP_MARK() do {} while (0)
#define QS_STAMP_ACC(k) do {} while (0)
#define QS_STAMP(k) do {} while (0)
#define QS_RTSTAMP(k) do {} while (0)
#define QS_STAMP_FLUSH() do {} while (0)
#define QS_STAMP_DECL
#endif

// Two waves share each SIMD (C3: 2048 one-wave workgroups), and VALU issue goes to the older one first: it
// ends ~1.1 us before its partner (profiles/r03_stamps_c3_s2.txt, by wave slot), and the launch ends with the
// younger waves.  The younger wave (wave slot != 0) takes the issue priority once the older one has drawn
// its Philox blocks -- mark 11, between the draws and the first wait on the state loads -- so the pair
// finishes together: C3 8.16 -> 7.77 us (profiles/ab/r03_prio_ab.txt; marks after the loads / physics
// gain less, priority from the start loses).  -DQS_PRIO_AT=-1 turns it off for A/Bs.
#ifndef QS_PRIO_AT
#define QS_PRIO_AT 11
#endif
#if QS_PRIO_AT >= 0
#define QS_PRIO(k)                                                                                    \
    do {                                                                                              \
        if ((k) == QS_PRIO_AT) {                                                                      \
            uint32_t hw_;                                                                             \
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw_));                        \
            if (hw_ & 0xFu) __builtin_amdgcn_s_setprio(1);                                            \
        }                                                                                             \
    } while (0)
#else
#define QS_PRIO(k) do {} while (0)
#endif
// The younger wave drops the priority again at mark QS_PRIO_END (-1: keeps it to the end); marks 21 (after the
// physics), 22 (after the collisions), 23 (after the impulses / scenario / state store) of the flavor-B step.
// Round 5 (profiles/ab/r05_prio_end_ab.txt): 23 in the goal-scenario kernels only (c3mix 9.38 -> 9.30 us; C3 and
// the earlier marks lose)
#ifndef QS_PRIO_END
#define QS_PRIO_END 23
#endif
#if QS_PRIO_AT >= 0 && QS_PRIO_END >= 0
#define QS_PRIO_DROP(k)                                                                               \
    do {                                                                                              \
        if ((k) == QS_PRIO_END) {                                                                     \
            uint32_t hw_;                                                                             \
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw_));                        \
            if (hw_ & 0xFu) __builtin_amdgcn_s_setprio(0);                                            \
        }                                                                                             \
    } while (0)
#else
#define QS_PRIO_DROP(k) do {} while (0)
#endif

struct Drone {
    float pos[3], vel[3], rot[9], om[3], rd[4], cd[4], ou[4], goal[3];
    int32_t svd;
    uint32_t flags;
    uint64_t prev;    // previous-collision row, partners 0..63 (bit j = partner j)
    uint64_t prevx;   // partners 64..127 (128-drone envs only; zero otherwise)
};

// ---------------------------------------------------------------------------------------------
// Non-finite guard (qs_counters): the reference raises on a NaN reward
// (quadrotor_single.py:87-90); the batched step counts non-finite observations, rewards and drone
// states per launch instead.  x * 0 is 0 for finite x and NaN for NaN / inf, so a chain of fma(x, 0, acc)
// and one compare tests a whole vector.  The common case costs one ballot; atomics only when something
// is non-finite.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ float fin_acc(float acc, float x) { return __builtin_fmaf(x, 0.f, acc); }
__device__ __forceinline__ bool drone_nonfinite(const Drone& d) {
    float a = 0.f;
#pragma unroll
    for (int i = 0; i < 3; ++i) { a = fin_acc(a, d.pos[i]); a = fin_acc(a, d.vel[i]); a = fin_acc(a, d.om[i]); }
#pragma unroll
    for (int i = 0; i < 9; ++i) a = fin_acc(a, d.rot[i]);
    return !(a == 0.f);
}
__device__ __forceinline__ void guard_count(const Bufs& b, int obs_bad, bool rew_bad, bool state_bad) {
    if (__ballot(obs_bad != 0 || rew_bad || state_bad) == 0ull) return;
    if (obs_bad) atomicAdd(b.stats + QS_ST_OBS, (unsigned long long)obs_bad);
    if (rew_bad) atomicAdd(b.stats + QS_ST_REW, 1ull);
    if (state_bad) atomicAdd(b.stats + QS_ST_STATE, 1ull);
}

__device__ __forceinline__ float clampf(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }
// single-instruction sqrt / reciprocal (v_sqrt_f32 / v_rcp_f32, ~1 ulp): the step is compared with the
// fp64 oracle at 1e-5..1e-4, far above these errors
__device__ __forceinline__ float fsqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
__device__ __forceinline__ float frcp(float x) { return __builtin_amdgcn_rcpf(x); }

// sin / cos of a bounded angle on the hardware units (v_sin/v_cos_f32, abs error < 4e-7 on [-pi, pi]):
// libm sincosf carries a Payne-Hanek path whose private array lands in scratch
__device__ __forceinline__ void sincos_hw(float x, float* s, float* c) {
    *s = __sinf(x);
    *c = __cosf(x);
}
// ---------------------------------------------------------------------------------------------
// state I/O (SoA, coalesced per field)
// ---------------------------------------------------------------------------------------------
// SoA field f of drone g as (uniform field base, 32-bit byte offset g * 4): the base lives in SGPRs and
// every field shares one offset VGPR, so the loads/stores use the saddr form (global_load_dword v, voff,
// s[base]) instead of one 64-bit VGPR address per field.
template <typename T>
__device__ __forceinline__ T ld_field(const T* base, int f, int I, uint32_t boff) {
    return *reinterpret_cast<const T*>(reinterpret_cast<const char*>(base + (size_t)f * (size_t)I) + boff);
}

// WIDE: the 128-drone envs' collision row (istate words QS_I_PREV_2 / _3 too)
template <bool WIDE = false>
__device__ __forceinline__ void load_drone(const KP& kp, const Bufs& b, int g, Drone& d) {
    const float* s = b.st;
    const int I = kp.I;
    const uint32_t bo = (uint32_t)g * 4u;
#pragma unroll
    for (int i = 0; i < 3; ++i) { d.pos[i] = ld_field(s, QS_F_POS + i, I, bo); d.vel[i] = ld_field(s, QS_F_VEL + i, I, bo); }
#pragma unroll
    for (int i = 0; i < 9; ++i) d.rot[i] = ld_field(s, QS_F_ROT + i, I, bo);
#pragma unroll
    for (int i = 0; i < 3; ++i) { d.om[i] = ld_field(s, QS_F_OMEGA + i, I, bo); d.goal[i] = ld_field(s, QS_F_GOAL + i, I, bo); }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        d.rd[i] = ld_field(s, QS_F_ROT_DAMP + i, I, bo);
        d.cd[i] = ld_field(s, QS_F_CMD_DAMP + i, I, bo);
        d.ou[i] = ld_field(s, QS_F_OU + i, I, bo);
    }
    const int32_t* is = b.ist;
    d.svd = ld_field(is, QS_I_SVD, I, bo);
    d.flags = (uint32_t)ld_field(is, QS_I_FLAGS, I, bo);
    d.prev = (uint64_t)(uint32_t)ld_field(is, QS_I_PREV_LO, I, bo) |
             ((uint64_t)(uint32_t)ld_field(is, QS_I_PREV_HI, I, bo) << 32);
    d.prevx = WIDE ? (uint64_t)(uint32_t)ld_field(is, QS_I_PREV_2, I, bo) |
                         ((uint64_t)(uint32_t)ld_field(is, QS_I_PREV_3, I, bo) << 32)
                   : 0ull;
}

// Write-through (sc1) stores: the bytes leave the XCD's L2 during the kernel instead of being
// written back by the end-of-kernel release (MI355X_MICROARCH "boundary": + dirty bytes / 6 TB/s).
// They are raw buffer stores with the sc1 cache-policy bit (aux 16): compiler-visible builtins, so the
// hazard recognizer schedules the wait states of the SGPR descriptor like for any other store.
#ifndef QS_WT_OBS
#define QS_WT_OBS 1
#endif
#ifndef QS_WT_STATE
#define QS_WT_STATE 1
#endif
constexpr int QS_AUX_SC1 = 16;
typedef uint32_t qs_v4u __attribute__((ext_vector_type(4)));
// buffer descriptor over a uniform base (raw, stride 0, 32-bit offsets; gfx950 dword3 0x00020000)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t qs_rsrc(const void* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
}
// 16-B store at byte offset voff (per lane) of a uniform base
__device__ __forceinline__ void st_wt4(__amdgpu_buffer_rsrc_t r, uint32_t voff, float4 v) {
    const qs_v4u x = {(uint32_t)__float_as_int(v.x), (uint32_t)__float_as_int(v.y), (uint32_t)__float_as_int(v.z),
                      (uint32_t)__float_as_int(v.w)};
    __builtin_amdgcn_raw_buffer_store_b128(x, r, (int)voff, 0, QS_WT_OBS ? QS_AUX_SC1 : 0);
}
// 4-B store of word `v` at (uniform soff + per-lane voff) bytes from the descriptor's base
#ifndef QS_STATE_AUX   // cache policy of the state stores: sc1 (write-through), or QS_STATE_AUX=2 (nt) / 0 (plain)
#define QS_STATE_AUX (QS_WT_STATE ? QS_AUX_SC1 : 0)
#endif
__device__ __forceinline__ void st_wt1(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, uint32_t v) {
    __builtin_amdgcn_raw_buffer_store_b32(v, r, (int)voff, (int)soff, QS_STATE_AUX);
}
// field f of a SoA array at (uniform base, lane byte offset): the field offset rides in soffset
template <typename T>
__device__ __forceinline__ void st_field(T* base, int f, int I, uint32_t boff, T v) {
    uint32_t w;
    __builtin_memcpy(&w, &v, 4);
    st_wt1(qs_rsrc(base), boff, (uint32_t)f * (uint32_t)I * 4u, w);
}

template <bool WIDE = false>
__device__ __forceinline__ void store_drone(const KP& kp, const Bufs& b, int g, const Drone& d) {
    float* s = b.st;
    const int I = kp.I;
    const uint32_t bo = (uint32_t)g * 4u;
#pragma unroll
    for (int i = 0; i < 3; ++i) { st_field(s, QS_F_POS + i, I, bo, d.pos[i]); st_field(s, QS_F_VEL + i, I, bo, d.vel[i]); }
#pragma unroll
    for (int i = 0; i < 9; ++i) st_field(s, QS_F_ROT + i, I, bo, d.rot[i]);
#pragma unroll
    for (int i = 0; i < 3; ++i) { st_field(s, QS_F_OMEGA + i, I, bo, d.om[i]); st_field(s, QS_F_GOAL + i, I, bo, d.goal[i]); }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        st_field(s, QS_F_ROT_DAMP + i, I, bo, d.rd[i]);
        st_field(s, QS_F_CMD_DAMP + i, I, bo, d.cd[i]);
        st_field(s, QS_F_OU + i, I, bo, d.ou[i]);
    }
    int32_t* is = b.ist;
    st_field(is, QS_I_SVD, I, bo, d.svd);
    st_field(is, QS_I_FLAGS, I, bo, (int32_t)d.flags);
    st_field(is, QS_I_PREV_LO, I, bo, (int32_t)(uint32_t)d.prev);
    st_field(is, QS_I_PREV_HI, I, bo, (int32_t)(uint32_t)(d.prev >> 32));
    if (WIDE) {
        st_field(is, QS_I_PREV_2, I, bo, (int32_t)(uint32_t)d.prevx);
        st_field(is, QS_I_PREV_3, I, bo, (int32_t)(uint32_t)(d.prevx >> 32));
    }
}

// ---------------------------------------------------------------------------------------------
// L1 physics: one substep == step1_numba (quadrotor_dynamics.py:355-390)
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void yaw_rot(float theta, float* R) {
    float s, c;
    sincos_hw(theta, &s, &c);
    R[0] = c; R[1] = -s; R[2] = 0.f;
    R[3] = s; R[4] = c; R[5] = 0.f;
    R[6] = 0.f; R[7] = 0.f; R[8] = 1.f;
}

// yaw_rot(atan2(y, x)) without trigonometry: cos / sin of atan2(y, x) are x / |(x, y)| and y / |(x, y)|
// (for (x, y) = (+-0, +-0): atan2 = 0 or +-pi by the signs, cos = +-1, sin = +-0)
__device__ __forceinline__ void yaw_rot_xy(float x, float y, float* R) {
    const float h2 = x * x + y * y;
    float c, s;
    if (h2 > 0.f) {
        const float r = __builtin_amdgcn_rsqf(h2);
        c = x * r;
        s = y * r;
    } else {   // h2 == 0, or NaN: arctan2 of a NaN is NaN, and so are its cos / sin (the state stays non-finite)
        c = h2 == 0.f ? __builtin_copysignf(1.f, x) : h2;
        s = h2 == 0.f ? __builtin_copysignf(0.f, y) : h2;
    }
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

// The substep in three pieces (motors -> torques, Rodrigues attitude update, the rest).  Every sub-lane of a
// drone runs all of it: dealing the motors and the Rodrigues rows over the sub-lanes measured slower (the DPP
// exchanges cost more issue slots than the replicated arithmetic).
struct Torque {
    float t0, t1, t2, sum;   // body torque, total thrust
};

// motor filter in sqrt space + multiplicative OU noise (:511-524) and torques (:527-533), all 4 motors
__device__ __forceinline__ Torque motors(const KP& kp, Drone& d, const float* cmds, const float* noise) {
    float thrusts[4];
    Torque t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float cmd = cmds[k];
        float tau = cmd < d.cd[k] ? kp.tau_down : kp.tau_up;
        tau = fminf(tau, 1.0f);
        d.rd[k] = tau * (fsqrt(cmd) - d.rd[k]) + d.rd[k];
        const float c = clampf(d.rd[k] * d.rd[k] + cmd * noise[k], 0.f, 1.f);
        d.cd[k] = c;
        // c in [0, 1]: with lin == 1 (every reference config) the quadratic term is exactly +0, so the
        // branch (folded in specialised builds) changes no bits -- it only drops the 0 * c * c work
        thrusts[k] = kp.thrust_max[k] * (kp.lin == 1.f ? c : (1.f - kp.lin) * c * c + kp.lin * c);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // zero arm coefficients add exactly +-0: skipped
        if (kp.pc0[k] != 0.f) t.t0 += kp.pc0[k] * thrusts[k];
        if (kp.pc1[k] != 0.f) t.t1 += kp.pc1[k] * thrusts[k];
        if (kp.pc2[k] != 0.f) t.t2 += kp.pc2[k] * thrusts[k];
        t.t2 += kp.torque_max[k] * kp.ccw[k] * d.cd[k];
        t.sum += thrusts[k];
    }
    return t;
}

// Rodrigues with world-frame omega (:544-551):  dR = I + sin(a) K + (1 - cos a) K^2, K = skew(w)/|w|,
// a = |w| dt.  Written as I + dt S(a^2) skew(w) + dt^2 C(a^2) (w w^T - |w|^2 I) with S = sin(a)/a and
// C = (1 - cos a)/a^2: no sqrt, no division, no branch at w = 0 (where the reference skips the update:
// dR = I exactly as the series gives).  rod_coef gives w, sx sy sz = S w, cf = C, d0 = 1 - C |w|^2.
struct RodCoef {
    float w[3], s[3], cf, d0;
};
__device__ __forceinline__ RodCoef rod_coef(const KP& kp, const float* R, const float* om) {
    const float dt = kp.dt;
    RodCoef r;
    r.w[0] = R[0] * om[0] + R[1] * om[1] + R[2] * om[2];
    r.w[1] = R[3] * om[0] + R[4] * om[1] + R[5] * om[2];
    r.w[2] = R[6] * om[0] + R[7] * om[1] + R[8] * om[2];
    const float w2 = r.w[0] * r.w[0] + r.w[1] * r.w[1] + r.w[2] * r.w[2];
    const float x = w2 * (dt * dt);
    // a < 0.6: Taylor to a^8, truncation < 2e-10 (|omega| <= 40 per axis gives a <= 0.35); computed on every lane, the
    // rare lanes past it overwrite it (one masked block instead of an if / else)
    float sf = dt * (1.f + x * (-1.f / 6.f + x * (1.f / 120.f + x * (-1.f / 5040.f + x * (1.f / 362880.f)))));
    float cf = dt * dt * (0.5f + x * (-1.f / 24.f + x * (1.f / 720.f + x * (-1.f / 40320.f + x * (1.f / 3628800.f)))));
    if (!(x < 0.36f)) {   // after collision kicks (|omega| up to ~100 rad/s before the clip)
        const float wn = fsqrt(w2), a = wn * dt;
        float sa, ca;
        sincos_hw(0.5f * a, &sa, &ca);
        sf = 2.f * sa * ca / wn;
        cf = 2.f * sa * sa / w2;
    }
    r.s[0] = sf * r.w[0]; r.s[1] = sf * r.w[1]; r.s[2] = sf * r.w[2];
    r.cf = cf;
    r.d0 = 1.f - cf * w2;
    return r;
}
// row i of dR
__device__ __forceinline__ void rod_row(const RodCoef& r, int i, float* o) {
    const float wi = r.w[i], cw = r.cf * wi;
    // skew(s) row i: [0, -s2, s1] / [s2, 0, -s0] / [-s1, s0, 0], diagonal d0
    const float a0 = i == 0 ? r.d0 : (i == 1 ? r.s[2] : -r.s[1]);
    const float a1 = i == 0 ? -r.s[2] : (i == 1 ? r.d0 : r.s[0]);
    const float a2 = i == 0 ? r.s[1] : (i == 1 ? -r.s[0] : r.d0);
    o[0] = a0 + cw * r.w[0];
    o[1] = a1 + cw * r.w[1];
    o[2] = a2 + cw * r.w[2];
}
// row i of dR @ R
__device__ __forceinline__ void rod_apply_row(const float* dr, const float* R, float* o) {
#pragma unroll
    for (int j = 0; j < 3; ++j) o[j] = dr[0] * R[j] + dr[1] * R[3 + j] + dr[2] * R[6 + j];
}

__device__ __forceinline__ void substep_tail(const KP& kp, Drone& d, const Torque& tq, const Rng& rng, uint32_t gid,
                                             int s);

// one substep == step1_numba (quadrotor_dynamics.py:355-390), everything on this lane
__device__ __forceinline__ void substep(const KP& kp, Drone& d, const float* cmds, const float* noise, const Rng& rng, uint32_t gid,
                        int s) {
    const Torque tq = motors(kp, d, cmds, noise);
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

// polar re-orthonormalisation, omega, position + room clip, floor, velocity (:553-656)
__device__ __forceinline__ void substep_tail(const KP& kp, Drone& d, const Torque& tq, const Rng& rng, uint32_t gid,
                                             int s) {
    const float dt = kp.dt;
    float* R = d.rot;
    const float tq0 = tq.t0, tq1 = tq.t1, tq2 = tq.t2, tsum = tq.sum;
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
        // rotational damping (dq = 0 in every reference config: 1 - dm == 1 exactly)
        const float dm0 = kp.dq != 0.f ? clampf(kp.dq * (o0 * o0), 0.f, 1.f) : 0.f,
                    dm1 = kp.dq != 0.f ? clampf(kp.dq * (o1 * o1), 0.f, 1.f) : 0.f,
                    dm2 = kp.dq != 0.f ? clampf(kp.dq * (o2 * o2), 0.f, 1.f) : 0.f;
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
    float az;
    const float azf = -kp.grav + kp.inv_mass * fz;
    const bool low = d.pos[2] <= kp.arm;
    fl = low ? fl : (fl & ~(uint32_t)QS_FL_ON_FLOOR);
    if (low) {
        d.pos[2] = kp.arm;
        if (fl & QS_FL_ON_FLOOR) {   // resting on the floor: the common case of an untrained swarm
            // rot = yaw_rot(arctan2(R10, R00 + EPS)) and the friction directions cos / sin of arctan2 as
            // normalised components (no atan2 / sin / cos)
            yaw_rot_xy(R[0] + 1e-6f, R[3], R);
            const float fric = 0.6f * (kp.mass_g - fz);
            const float vn = fsqrt(d.vel[0] * d.vel[0] + d.vel[1] * d.vel[1] + d.vel[2] * d.vel[2]);
            if (vn < 1e-6f) {
                const float f2 = fx * fx + fy * fy, fm = fsqrt(f2);
                const float fxy = fmaxf(fm - fric, 0.f);
                if (fxy == 0.f) {
                    fx = 0.f; fy = 0.f;
                } else {   // fm > fric >= 0
                    const float k = fxy * __builtin_amdgcn_rsqf(f2);
                    fx = k * fx; fy = k * fy;
                }
            } else {
                const float v2 = d.vel[0] * d.vel[0] + d.vel[1] * d.vel[1];
                float ca, sa;
                if (v2 > 0.f) {
                    const float r = __builtin_amdgcn_rsqf(v2);
                    ca = d.vel[0] * r;
                    sa = d.vel[1] * r;
                } else {
                    ca = __builtin_copysignf(1.f, d.vel[0]);
                    sa = __builtin_copysignf(0.f, d.vel[1]);
                }
                fx = fx - ca * fric;
                fy = fy - sa * fric;
            }
        } else {
            fl |= QS_FL_ON_FLOOR | QS_FL_CRASH_FLOOR;
#pragma unroll
            for (int i = 0; i < 3; ++i) { d.vel[i] = 0.f; d.om[i] = 0.f; }
            if (R[8] < 0.f) {   // upside down: a random yaw
                uint32_t gid_ = gid;   // opaque: keeps the Philox key schedule out of the common path
                asm volatile("" : "+v"(gid_));
                yaw_rot(-3.14159265358979f + 6.28318530717959f * uniform1(rng, gid_, S_FLOOR | ((uint32_t)s << 8), 0), R);
            } else {            // yaw_rot(arctan2(R10, R00 + EPS)) as normalised components, like the resting case
                yaw_rot_xy(R[0] + 1e-6f, R[3], R);
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) { d.cd[k] = 0.f; d.rd[k] = 0.f; }
        }
        az = fmaxf(azf, 0.f);
    } else {
        az = azf;
    }
    const float ax = kp.inv_mass * fx, ay = kp.inv_mass * fy;
    d.flags = fl;
    d.vel[0] = (1.f - kp.vel_damp) * d.vel[0] + dt * ax;  // (:652)
    d.vel[1] = (1.f - kp.vel_damp) * d.vel[1] + dt * ay;
    d.vel[2] = (1.f - kp.vel_damp) * d.vel[2] + dt * az;
}


// Neighbour exchange tile in LDS: lane l stores {pos, 0} at xch[2l] and {vel, 0} at xch[2l+1]; the
// drones of one env read each other's rows with broadcast ds_read_b128 (one wave per workgroup, so a
// workgroup barrier costs nothing but orders the LDS traffic).
// LDS-only workgroup barrier: workgroups are one wave, so this just orders LDS traffic.  Unlike
// __syncthreads() it does not wait for outstanding global stores (vmcnt) or fence global memory.
__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// ---------------------------------------------------------------------------------------------
// sub-lanes: the flavor-B step kernel gives each drone Q consecutive lanes (a quad for Q = 4, a
// pair for Q = 2).  The drone's physics runs replicated on all Q lanes (bit-identical), while the
// divisible work -- Philox blocks, partner tests, neighbour candidates -- is dealt over them and
// exchanged through DPP quad permutes (a VALU modifier: no LDS round trip).  Every helper below
// must be called with all Q lanes of the drone active (quad-uniform control flow).
// ---------------------------------------------------------------------------------------------
// QS_DPP_BC: bound_ctrl on (an out-of-range / disabled source lane reads 0 -- the same value as the old = 0
// form, so bitwise the same results) lets the compiler fold the permute into its consumer (v_sub_f32_dpp ...)
// more often: C3 7.74 -> 7.64 us (profiles/ab/r03_dpp_bc_ab.txt); flavor A kept it off in round 3 and takes it
// since round 4 (a8 23.54 -> 23.37 us, profiles/ab/r04_a8_dpp_bc_ab.txt)
#ifndef QS_DPP_BC
#define QS_DPP_BC 1
#endif
template <int CTRL>
__device__ __forceinline__ int dpp_i(int x) { return __builtin_amdgcn_update_dpp(0, x, CTRL, 0xF, 0xF, QS_DPP_BC != 0); }
template <int CTRL>
__device__ __forceinline__ float dpp_f(float x) { return __int_as_float(dpp_i<CTRL>(__float_as_int(x))); }
constexpr int quad_perm(int a, int b, int c, int d) { return a | (b << 2) | (c << 4) | (d << 6); }

// Q = 8 (single-drone envs): the drone's 8 lanes are two quads of a 16-lane DPP row; the other quad's lane
// (lane ^ 4) comes by row_shl:4 (lower quad) or row_shr:4 (upper quad)
constexpr int DPP_ROW_SHL4 = 0x104, DPP_ROW_SHR4 = 0x114;
__device__ __forceinline__ int xquad_i(int x) {
    const int up = dpp_i<DPP_ROW_SHL4>(x), dn = dpp_i<DPP_ROW_SHR4>(x);
    return (__lane_id() & 4) ? dn : up;
}
__device__ __forceinline__ float xquad_f(float x) { return __int_as_float(xquad_i(__float_as_int(x))); }
// value of sub-lane K of this lane's drone
template <int Q, int K>
__device__ __forceinline__ float qbc(float x) {
    static_assert(K < Q, "sub-lane");
    static_assert(Q == 1 || Q == 2 || Q == 4 || Q == 8, "sub-lanes per drone");
    if constexpr (Q == 1) return x;
    else if constexpr (Q == 2) return dpp_f<quad_perm(K, K, 2 + K, 2 + K)>(x);
    else if constexpr (Q == 4) return dpp_f<quad_perm(K, K, K, K)>(x);
    else {   // lane K % 4 of each quad, then the quad that holds sub-lane K
        const float v = dpp_f<quad_perm(K % 4, K % 4, K % 4, K % 4)>(x);
        const float o = xquad_f(v);
        return ((__lane_id() & 4) != 0) == (K >= 4) ? v : o;
    }
}
// sum over the drone's sub-lanes: every lane gets the same bits ((a+b)+(c+d) == (c+d)+(a+b))
template <int Q>
__device__ __forceinline__ float qsum(float x) {
    if constexpr (Q >= 2) x += dpp_f<quad_perm(1, 0, 3, 2)>(x);
    if constexpr (Q >= 4) x += dpp_f<quad_perm(2, 3, 0, 1)>(x);
    if constexpr (Q >= 8) x += xquad_f(x);
    return x;
}
// compile-time walk over the blocks of qdraws: block K lives on sub-lane K % Q, slot K / Q
template <int Q, int K, int NN, int NU, int T>
__device__ __forceinline__ void qdraws_gather(const float (&v)[T][4], float* z, float* u) {
    if constexpr (K < NN + NU) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float x = qbc<Q, K % Q>(v[K / Q][i]);
            if constexpr (K < NN) z[4 * K + i] = x;
            else u[4 * (K - NN) + i] = x;
        }
        qdraws_gather<Q, K + 1, NN, NU, T>(v, z, u);
    }
}

template <int Q>
__device__ __forceinline__ uint64_t qor(uint64_t m) {
    int lo = (int)(uint32_t)m, hi = (int)(uint32_t)(m >> 32);
    if constexpr (Q >= 2) { lo |= dpp_i<quad_perm(1, 0, 3, 2)>(lo); hi |= dpp_i<quad_perm(1, 0, 3, 2)>(hi); }
    if constexpr (Q >= 4) { lo |= dpp_i<quad_perm(2, 3, 0, 1)>(lo); hi |= dpp_i<quad_perm(2, 3, 0, 1)>(hi); }
    if constexpr (Q >= 8) { lo |= xquad_i(lo); hi |= xquad_i(hi); }
    return (uint64_t)(uint32_t)lo | ((uint64_t)(uint32_t)hi << 32);
}

// NN normal blocks (stream sn) and NU uniform blocks (stream su | UNIF_BIT) of one Philox key,
// dealt over the Q sub-lanes (block k on sub-lane k % Q) and broadcast: z[4 NN], u[4 NU] on all of
// them.  Every lane runs the same Philox + Box-Muller instructions (no divergence on the kind).
template <int Q, int NN, int NU>
__device__ __forceinline__ void qdraws(const Rng& r, uint32_t id, uint32_t sn, uint32_t su, int q, float* z, float* u) {
    constexpr int L = NN + NU, T = (L + Q - 1) / Q;
    float v[T][4];
#pragma unroll
    for (int t = 0; t < T; ++t) {
        const int k = q + Q * t;
        const bool isn = k < NN;
        const W4 w = block(r, id, isn ? sn : (su | UNIF_BIT), (uint32_t)(isn ? k : k - NN));
        float n[4];
        box_muller(w.w[0], w.w[1], n[0], n[1]);
        box_muller(w.w[2], w.w[3], n[2], n[3]);
#pragma unroll
        for (int i = 0; i < 4; ++i) v[t][i] = isn ? n[i] : u01(w.w[i]);
    }
    qdraws_gather<Q, 0, NN, NU, T>(v, z, u);
}

// XCD-aware block order: workgroups are dealt round-robin over the 8 XCDs (block b on XCD b % 8), so
// consecutive blocks -- whose SoA fields share 128-B lines when a block covers only 64 B of a field --
// would pull the same line into two L2s.  Hand each XCD a contiguous run of logical blocks instead.
__device__ __forceinline__ int xcd_block(int b, int nblocks) {
    return (nblocks & 7) ? b : (b & 7) * (nblocks >> 3) + (b >> 3);
}

// Sub-lanes per drone of an env that spans several waves (64- and 128-drone envs): with 2, a 512-env
// 64-drone shard or a 256-env 128-drone shard is 1024 waves, one per SIMD.
#ifndef QS_QW
#define QS_QW 2
#endif

// ---- collision rows: bit j = partner drone j; 64 bits, or two words for the 128-drone envs ----
struct Row128 {
    uint64_t lo, hi;
};
__device__ __forceinline__ Row128 operator|(Row128 a, Row128 b) { return Row128{a.lo | b.lo, a.hi | b.hi}; }
__device__ __forceinline__ Row128 operator&(Row128 a, Row128 b) { return Row128{a.lo & b.lo, a.hi & b.hi}; }
__device__ __forceinline__ Row128 operator~(Row128 a) { return Row128{~a.lo, ~a.hi}; }
template <bool WIDE> struct RowOf { using T = uint64_t; };
template <> struct RowOf<true> { using T = Row128; };
__device__ __forceinline__ bool row_any(uint64_t r) { return r != 0ull; }
__device__ __forceinline__ bool row_any(Row128 r) { return (r.lo | r.hi) != 0ull; }
__device__ __forceinline__ int row_popc(uint64_t r) { return __popcll(r); }
__device__ __forceinline__ int row_popc(Row128 r) { return __popcll(r.lo) + __popcll(r.hi); }
__device__ __forceinline__ int row_ffs(uint64_t r) { return __ffsll((long long)r) - 1; }   // r != 0
__device__ __forceinline__ int row_ffs(Row128 r) {
    return r.lo ? __ffsll((long long)r.lo) - 1 : 64 + __ffsll((long long)r.hi) - 1;
}
__device__ __forceinline__ void row_set(uint64_t& r, int j, bool c) { r |= c ? (1ull << j) : 0ull; }
__device__ __forceinline__ void row_set(Row128& r, int j, bool c) {
    if (j < 64) r.lo |= c ? (1ull << j) : 0ull;
    else r.hi |= c ? (1ull << (j - 64)) : 0ull;
}
__device__ __forceinline__ void row_clear(uint64_t& r, int j) { r &= ~(1ull << j); }
__device__ __forceinline__ void row_clear(Row128& r, int j) {
    if (j < 64) r.lo &= ~(1ull << j);
    else r.hi &= ~(1ull << (j - 64));
}
// the partners above drone di (pairs (di, j > di))
__device__ __forceinline__ uint64_t row_above(uint64_t r, int di) { return r & ~((2ull << di) - 1ull); }
__device__ __forceinline__ Row128 row_above(Row128 r, int di) {
    return di < 64 ? Row128{r.lo & ~((2ull << di) - 1ull), r.hi} : Row128{0ull, r.hi & ~((2ull << (di - 64)) - 1ull)};
}
template <int Q>
__device__ __forceinline__ Row128 qor(Row128 r) { return Row128{qor<Q>(r.lo), qor<Q>(r.hi)}; }
__device__ __forceinline__ void row_of(const Drone& d, uint64_t& r) { r = d.prev; }
__device__ __forceinline__ void row_of(const Drone& d, Row128& r) { r = Row128{d.prev, d.prevx}; }
__device__ __forceinline__ void row_keep(Drone& d, uint64_t r) { d.prev = r; }
__device__ __forceinline__ void row_keep(Drone& d, Row128 r) { d.prev = r.lo; d.prevx = r.hi; }

// the drones' bits of a wave ballot with Q = 2 sub-lanes per drone: bit i = lane 2i or 2i + 1 (32 bits)
__device__ __forceinline__ uint64_t compact_pairs(uint64_t b) {
    uint64_t x = (b | (b >> 1)) & 0x5555555555555555ull;
    x = (x | (x >> 1)) & 0x3333333333333333ull;
    x = (x | (x >> 2)) & 0x0F0F0F0F0F0F0F0Full;
    x = (x | (x >> 4)) & 0x00FF00FF00FF00FFull;
    x = (x | (x >> 8)) & 0x0000FFFF0000FFFFull;
    return (x | (x >> 16)) & 0x00000000FFFFFFFFull;
}

// Env-level collectives of the step kernel over a predicate of the env's lanes (callers pass x && q == 0 to
// count drones).  An env inside one wave: a ballot of the env's lane segment (drone i at bit i Q).  An env that
// spans the workgroup's NW waves (WIDE: 64 drones x 2 sub-lanes, 128 drones x 1 or 2): each wave's ballot,
// reduced to its drones (bit i = drone i of the env), through an LDS slot and a workgroup barrier; the slots
// alternate so that one barrier per collective suffices.  Every lane of the workgroup must make the same calls.
template <bool WIDE, bool ROW2 = false, int Q = 1, int NW = 1>
struct EnvColl {
    using Row = typename RowOf<ROW2>::T;
    int lbase;
    uint64_t lmask;
    uint64_t* scr;   // WIDE: 2 NW words of LDS
    int slot;
    __device__ __forceinline__ Row bits(bool x) {
        if constexpr (!WIDE) {
            return (__ballot(x) >> lbase) & lmask;
        } else {
            static_assert(Q == 1 || Q == 2, "sub-lanes of a multi-wave env");
            constexpr int DPW = 64 / Q;   // drones per wave
            const uint64_t bw = Q == 2 ? compact_pairs(__ballot(x)) : __ballot(x);
            uint64_t* s = scr + NW * slot;
            slot ^= 1;
            if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = bw;
            lds_sync();
            uint64_t w[2] = {0ull, 0ull};
#pragma unroll
            for (int k = 0; k < NW; ++k) w[(k * DPW) >> 6] |= s[k] << ((k * DPW) & 63);
            if constexpr (ROW2) return Row128{w[0], w[1]};
            else return w[0];
        }
    }
    __device__ __forceinline__ bool any(bool x) { return row_any(bits(x)); }
    __device__ __forceinline__ int count(bool x) { return row_popc(bits(x)); }
    // uniform over the launch's unit of lockstep (the wave, or the WIDE workgroup): guards work that has barriers
    __device__ __forceinline__ bool wany(bool x) {
        if constexpr (!WIDE) return __ballot(x) != 0ull;
        else return any(x);
    }
};

// ---------------------------------------------------------------------------------------------
// block-level obs staging: LDS tile [rows, obs_dim] -> contiguous global rows
// ---------------------------------------------------------------------------------------------
// Returns how many of the values this lane stored are non-finite (the obs guard of qs_counters).
__device__ __forceinline__ int tile_store(const float* lds, float* dst, int nfloat, int lane, int nthr = 64) {
    // dst = first row of the block; rows are contiguous in HBM.  obs is 256-B aligned and a block owns
    // 64/NPAD*N rows, so the start is 16-B aligned whenever rows*obs_dim*4 is: b128 in, dwordx4 out.
    int bad = 0;
    if ((((uintptr_t)dst) & 15) == 0) {
        const int nvec = nfloat >> 2;
        const float4* lv = reinterpret_cast<const float4*>(lds);
        const __amdgpu_buffer_rsrc_t r = qs_rsrc(dst);
        for (int v = lane; v < nvec; v += nthr) {
            const float4 x = lv[v];
            st_wt4(r, (uint32_t)v * 16u, x);
            if (!(fin_acc(fin_acc(fin_acc(x.x * 0.f, x.y), x.z), x.w) == 0.f))
                bad += !(x.x * 0.f == 0.f) + !(x.y * 0.f == 0.f) + !(x.z * 0.f == 0.f) + !(x.w * 0.f == 0.f);
        }
        const int t = (nvec << 2) + lane;
        if (t < nfloat) {
            dst[t] = lds[t];
            bad += !(lds[t] * 0.f == 0.f);
        }
    } else {
        for (int f = lane; f < nfloat; f += nthr) {
            dst[f] = lds[f];
            bad += !(lds[f] * 0.f == 0.f);
        }
    }
    return bad;
}

// float4 per lane of a block's obs tile (`slots` rows of obs_dim floats over `nthr` lanes): a compile-time bound in
// the specialised kernels (obs_dim is a constant there), 0 in the generic ones (tile_store's loop)
template <int SLOTS, int NTHR>
__device__ constexpr int tile_vecs() {
#ifdef QS_JIT
    return (SLOTS * kKP.obs_dim / 4 + NTHR - 1) / NTHR;
#else
    return 0;
#endif
}

// tile_store with every float4 read of the lane issued back to back before the stores: one LDS wait for the tile
// instead of one per vector (the loop above waits on each read before its store).  Reads past the tile are
// clamped to its last vector (stored by its own lane only); the non-finite count is the loop's, taken exactly in
// the rare branch.  V = tile_vecs<>() bounds the vectors per lane; a larger tile falls back to the loop.
#ifndef QS_TILE_BATCH
#define QS_TILE_BATCH 1
#endif
template <int V>
__device__ __forceinline__ int tile_store_v(const float* lds, float* dst, int nfloat, int lane, int nthr) {
    const int nvec = nfloat >> 2;
    if (!QS_TILE_BATCH || V <= 0 || V > 8 || (((uintptr_t)dst) & 15) != 0 || nvec < 1 || nvec > V * nthr)
        return tile_store(lds, dst, nfloat, lane, nthr);
    const float4* lv = reinterpret_cast<const float4*>(lds);
    const __amdgpu_buffer_rsrc_t r = qs_rsrc(dst);
    float4 x[V > 0 ? V : 1];
#pragma unroll
    for (int i = 0; i < V; ++i) x[i] = lv[min(lane + i * nthr, nvec - 1)];
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < V; ++i) {
        const int v = lane + i * nthr;
        if (v < nvec) st_wt4(r, (uint32_t)v * 16u, x[i]);
        acc = fin_acc(fin_acc(fin_acc(fin_acc(acc, x[i].x), x[i].y), x[i].z), x[i].w);
    }
    int bad = 0;
    if (!(acc == 0.f)) {   // some value is inf / NaN (a clamped copy included): count the tile's own exactly
#pragma unroll
        for (int i = 0; i < V; ++i)
            if (lane + i * nthr < nvec)
                bad += !(x[i].x * 0.f == 0.f) + !(x[i].y * 0.f == 0.f) + !(x[i].z * 0.f == 0.f) + !(x[i].w * 0.f == 0.f);
    }
    const int t = (nvec << 2) + lane;
    if (t < nfloat) {
        dst[t] = lds[t];
        bad += !(lds[t] * 0.f == 0.f);
    }
    return bad;
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

// perform_downwash (aerodynamics/downwash.py:4-51) on this lane's drone, for one control step of kp.cdt:
// every other drone i of the env (read by __shfl from its sub-lane q, lanes lbase + i Q + q) whose
// z-axis points at it from above within 0.7 m and 0.1 m sideways pushes it down and spins it, with the
// source's per-step noise (stream S_DW of drone i) and the pair's draws (stream S_DWPAIR | this drone).
// Every lane of the env segment must execute it (the permutes read the env's lanes).  True when applied.
// dwt: an LDS scratch of 2 float4 per drone slot of the workgroup (the obs tile, which is not in use
// yet when the forces run); dbase = the env's first slot.  The sources' {z axis, noise} and {pos, noise} go
// through it -- 2 ds_write_b128 + 2 broadcast ds_read_b128 per source instead of 8 LDS permutes.
template <int NPAD, int Q>
__device__ __forceinline__ bool downwash_env(const KP& kp, Drone& d, const Rng& rng, uint32_t gid, int env, int lbase,
                                             int di, int q, bool active, float4* dwt = nullptr, int dbase = 0) {
    bool vchanged = false;
    float dwu[4];
    uniforms4(rng, gid, S_DW, 0, dwu);
    const float an = -0.1f + 0.2f * dwu[0], wn = -0.01f + 0.02f * dwu[1];
    const float P0 = d.pos[0], P1 = d.pos[1], P2 = d.pos[2];
    if (dwt) {
        if (q == 0) {
            dwt[2 * (dbase + di)] = make_float4(d.rot[2], d.rot[5], d.rot[8], an);
            dwt[2 * (dbase + di) + 1] = make_float4(P0, P1, P2, wn);
        }
        lds_sync();
    }
    for (int i = 0; i < NPAD; ++i) {
        float zi0, zi1, zi2, pi0, pi1, pi2, ani, wni;
        if (dwt) {
            const float4 a = dwt[2 * (dbase + i)], b = dwt[2 * (dbase + i) + 1];
            zi0 = a.x; zi1 = a.y; zi2 = a.z; ani = a.w;
            pi0 = b.x; pi1 = b.y; pi2 = b.z; wni = b.w;
        } else {
            const int src = lbase + i * Q + q;
            zi0 = __shfl(d.rot[2], src); zi1 = __shfl(d.rot[5], src); zi2 = __shfl(d.rot[8], src);
            pi0 = __shfl(P0, src); pi1 = __shfl(P1, src); pi2 = __shfl(P2, src);
            ani = __shfl(an, src); wni = __shfl(wn, src);
        }
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
    if (dwt) lds_sync();   // the scratch is the obs tile: every read done before it is written
    return vchanged;
}

}  // namespace qs
