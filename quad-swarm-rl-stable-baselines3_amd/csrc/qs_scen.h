// qs_scen.h -- the goal scenarios of gym_art/quadrotor_multi/scenarios/ on the device, shared by the
// flavor-B step / reset kernels (quadrotor_multi.py) and the flavor-A ones (quadrotor_multi_rewards.py:123,
// create_scenario).  Mirrors oracle/quadswarm_oracle_scen.c.
#pragma once
#include "qs_common.h"

namespace qs {

__device__ __forceinline__ uint32_t ubits(const Rng& r, uint32_t id, uint32_t st, uint32_t idx) {
    return word_of(block(r, id, st | UNIF_BIT, idx >> 2), idx & 3);
}
// floor(u * m) exactly for u = ((w >> 8) + 0.5) / 2^24 (the oracle evaluates it in double, exactly)
__device__ __forceinline__ int ufloor(uint32_t w, int m) {
    return (int)((((uint64_t)(w >> 8) * 2u + 1u) * (uint64_t)m) >> 25);
}

// ---------------------------------------------------------------------------------------------
// goal scenarios (gym_art/quadrotor_multi/scenarios/).  The env's lead lane runs
// them serially (a reset, or an event every 4-6 s; per step only for ep_lissajous3D / ep_rand_bezier /
// dynamic_formations) on goal tables in LDS (4 floats per drone); the drones then read their goal.
// Mirrors oracle/quadswarm_oracle_scen.c draw for draw: Philox key = the env's drone 0, stream S_SCN
// (step) / S_SCN_RESET (reset), one 32-bit word per draw in call order.
// ---------------------------------------------------------------------------------------------
enum { SC_STATIC_SAME_GOAL = 0, SC_STATIC_DIFF_GOAL, SC_EP_LISSAJOUS3D, SC_EP_RAND_BEZIER, SC_DYNAMIC_SAME_GOAL,
       SC_DYNAMIC_DIFF_GOAL, SC_DYNAMIC_FORMATIONS, SC_SWAP_GOALS, SC_SWARM_VS_SWARM, SC_RUN_AWAY, SC_MIX,
       // the obstacle maps' dynamic scenarios (scenarios/obstacles/, QUADS_MODE_LIST_OBSTACLES_TEST utils.py:18-20):
       // reset with the env's map by obstacle_reset_env (qs_flavor_b.h), stepped by scen_step_lane
       SC_O_SWAP_GOALS, SC_O_EP_RAND_BEZIER, SC_O_DYNAMIC_SAME_GOAL };
enum { F_CIRCLE_H = 0, F_CIRCLE_XZ, F_CIRCLE_YZ, F_SPHERE, F_GRID_H, F_GRID_XZ, F_GRID_YZ, F_CUBE };

struct Scen {
    int mode, form, period, inc;
    float size, lo, hi, layer, speed, c[3], bz[9], c1[3], c2[3];
};

static_assert(QS_ENVF_SC_C2 + 3 - QS_ENVF_SC_SIZE == QS_SC_NF, "the scenario float block");
// the env's scenario float k (row QS_ENVF_SC_SIZE + k) in the env-major block (quadswarm.h QS_SC_NF)
__device__ __forceinline__ float* scf(float* f, int E, int env, int row) {
    return f + (size_t)QS_ENVF_SC_SIZE * E + (size_t)QS_SC_NF * env + (row - QS_ENVF_SC_SIZE);
}
__device__ __forceinline__ void scen_load(const KP& kp, const Bufs& b, int env, Scen& s) {
    const int E = kp.E;
    s.mode = b.env[QS_E_SC_MODE * E + env]; s.form = b.env[QS_E_SC_FORM * E + env];
    s.period = b.env[QS_E_SC_PERIOD * E + env]; s.inc = b.env[QS_E_SC_INC * E + env];
    const float* f = scf(b.envf, E, env, QS_ENVF_SC_SIZE);   // the env's 23 floats, row order
    s.size = f[0]; s.lo = f[1]; s.hi = f[2]; s.layer = f[3]; s.speed = f[4];
    for (int i = 0; i < 3; ++i) {
        s.c[i] = f[QS_ENVF_SC_CENTER - QS_ENVF_SC_SIZE + i];
        s.c1[i] = f[QS_ENVF_SC_C1 - QS_ENVF_SC_SIZE + i];
        s.c2[i] = f[QS_ENVF_SC_C2 - QS_ENVF_SC_SIZE + i];
    }
    for (int i = 0; i < 9; ++i) s.bz[i] = f[QS_ENVF_SC_BEZIER - QS_ENVF_SC_SIZE + i];
}
__device__ __forceinline__ void scen_store(const KP& kp, const Bufs& b, int env, const Scen& s) {
    const int E = kp.E;
    b.env[QS_E_SC_MODE * E + env] = s.mode; b.env[QS_E_SC_FORM * E + env] = s.form;
    b.env[QS_E_SC_PERIOD * E + env] = s.period; b.env[QS_E_SC_INC * E + env] = s.inc;
    float* f = scf(b.envf, E, env, QS_ENVF_SC_SIZE);
    f[0] = s.size; f[1] = s.lo; f[2] = s.hi; f[3] = s.layer; f[4] = s.speed;
    for (int i = 0; i < 3; ++i) {
        f[QS_ENVF_SC_CENTER - QS_ENVF_SC_SIZE + i] = s.c[i];
        f[QS_ENVF_SC_C1 - QS_ENVF_SC_SIZE + i] = s.c1[i];
        f[QS_ENVF_SC_C2 - QS_ENVF_SC_SIZE + i] = s.c2[i];
    }
    for (int i = 0; i < 9; ++i) f[QS_ENVF_SC_BEZIER - QS_ENVF_SC_SIZE + i] = s.bz[i];
}

// draw source: one Philox word per draw, the last block cached (draws are sequential)
struct SDraw {
    Rng r;
    uint32_t key, stream, k, blk;
    W4 w;
};
__device__ __forceinline__ SDraw sdraw(const Rng& r, uint32_t key, uint32_t stream) {
    SDraw s;
    s.r = r; s.key = key; s.stream = stream | UNIF_BIT; s.k = 0; s.blk = 0xFFFFFFFFu;
    return s;
}
__device__ __forceinline__ uint32_t sd_word(SDraw& s) {
    const uint32_t k = s.k++;
    if ((k >> 2) != s.blk) {
        s.blk = k >> 2;
        s.w = block(s.r, s.key, s.stream, s.blk);
    }
    return word_of(s.w, k & 3);
}
__device__ __forceinline__ float sd_uniform(SDraw& s, float lo, float hi) { return lo + (hi - lo) * u01(sd_word(s)); }
__device__ __forceinline__ int sd_int(SDraw& s, int lo, int hi) { return lo + ufloor(sd_word(s), hi - lo); }
// One try of ep_rand_bezier's rejection loop (ep_rand_bezier.py:20-33): 6 uniforms + 1 integer = 7 words from sd's
// position, so try i reads words 7 i .. 7 i + 6 of the step's scenario stream (the loop draws nothing else first).
// np_: the candidate's two control points [c][j]; returns whether both lie inside the shrunk bounds.
constexpr int BZ_WORDS = 7, BZ_MAX_TRIES = 1024;
// o_ep_rand_bezier accepts ~0.6 % of its tries (its z band is 0.5 m wide): ~160 on average, beyond 1024 for ~0.2 % of
// the resamples -- its bound is 8192 ((0.994)^8192 ~ 4e-22), searched by the env's lanes in parallel
constexpr int BZ_MAX_TRIES_O = 8192;
// o_dynamic_same_goal's rejection loop (a free cell within 4 m of the end point): bounded here
constexpr int ODS_MAX_TRIES = 4096;
__device__ __forceinline__ bool bz_try(SDraw& sd, const float* hi, const float* lo, float mx, const float* g,
                                       float (&np_)[3][2]) {
    float u[6];   // uniform(size=(2, 3)).reshape(3, 2): [c][j] = flat 2c + j
    for (int k = 0; k < 6; ++k) u[k] = sd_uniform(sd, -hi[k % 3], hi[k % 3]);
    // np.random.randint(min_dist, max_dist + 1) with float bounds: numpy truncates both (randint(2.5, 6) draws 2..5)
    const float mag = (float)sd_int(sd, (int)(mx * 0.5f), (int)floorf(mx) + 1);
    bool ok = true;
    for (int j = 0; j < 2; ++j) {
        const float v0 = u[j], v1 = u[2 + j], v2 = u[4 + j];
        const float sc = mag / fsqrt(v0 * v0 + v1 * v1 + v2 * v2);
        np_[0][j] = v0 * sc + g[0]; np_[1][j] = v1 * sc + g[1]; np_[2][j] = v2 * sc + g[2];
        for (int k = 0; k < 3; ++k) ok = ok && np_[k][j] > lo[k] + 0.5f && np_[k][j] < hi[k] - 0.5f;
    }
    return ok;
}
// the bounds of the tries for a formation of size `size`: ep_rand_bezier.py:13-19, or (obst) o_ep_rand_bezier.py:19-28
// (max_dist min(5, .), z in [1.5, 3.0])
__device__ __forceinline__ float bz_bounds(const KP& kp, float size, float* hi, float* lo, bool obst = false) {
    float rd[3];
    for (int k = 0; k < 3; ++k) rd[k] = kp.room_hi[k] - kp.room_lo[k] - size;
    const float mx = fminf(fmaxf(fmaxf(rd[0], rd[1]), rd[2]), obst ? 5.f : 30.f);
    hi[0] = rd[0] * 0.5f; hi[1] = rd[1] * 0.5f; hi[2] = obst ? 3.f : rd[2];
    lo[0] = -hi[0]; lo[1] = -hi[1]; lo[2] = obst ? 1.5f : 0.f;
    return mx;
}

// ---------------------------------------------------------------------------------------------
// obstacle maps: pillars on an n x n grid of 1 m cells (quadrotor_multi.py:405-426, obstacles/utils.py:46-58)
// ---------------------------------------------------------------------------------------------
// grid cell (row, col) -> cell_centers[row + n*col]
__device__ __forceinline__ float2 cell_xy(int cell, int n) {
    const int row = cell / n, col = cell % n;
    const float h = (float)(n / 2);
    return make_float2((float)col + 0.5f - h, (float)(n - 1 - row) + 0.5f - h);
}
// the env's map as its pillar list (the block's LDS copy): m pillars on the n x n grid
struct OCtx {
    const float2* ob;
    int m, n;
};
// Scenario_o_base.generate_pos_obst_map's cell (o_base.py:58-72): free_space[k] of np.where(obstacle_map == 0), i.e.
// the k-th free cell in row-major order, as its centre; the occupied cells come back from the pillar centres
// (cell_xy's inverse: small half-integers, exact)
__device__ __forceinline__ float2 o_free_cell(const OCtx& oc, int k) {
    const int n = oc.n;
    const float h = (float)(n / 2);
    uint64_t occ = 0ull;
    for (int o = 0; o < oc.m; ++o) {
        const int col = (int)(oc.ob[o].x - 0.5f + h), row = n - 1 - (int)(oc.ob[o].y - 0.5f + h);
        occ |= 1ull << (row * n + col);
    }
    int c = 0;
    for (; c < n * n; ++c)
        if (!((occ >> c) & 1ull) && k-- == 0) break;
    return cell_xy(min(c, n * n - 1), n);
}
// Generator.shuffle as Fisher-Yates from the top over LDS rows g[4 i ..]
__device__ __forceinline__ void sd_shuffle(SDraw& s, float* g, int n) {
    for (int i = n - 1; i >= 1; --i) {
        const int j = sd_int(s, 0, i + 1);
        for (int c = 0; c < 3; ++c) {
            const float t = g[4 * i + c];
            g[4 * i + c] = g[4 * j + c];
            g[4 * j + c] = t;
        }
    }
}

// sin / cos of any angle on the hardware units, reduced to [-0.5, 0.5] revolutions first
__device__ __forceinline__ float sin_any(float x) {
    const float r = x * 0.15915494309189535f;
    return __builtin_amdgcn_sinf(r - rintf(r));
}
__device__ __forceinline__ float cos_any(float x) {
    const float r = x * 0.15915494309189535f;
    return __builtin_amdgcn_cosf(r - rintf(r));
}

// The drone count as a run-time value: in the specialised build kp.N is a constant, and the compiler would
// constant-fold the hardware transcendentals of the formation geometry exactly (sin / cos / log2 / exp2 of
// constant arguments) where the generic build evaluates them on the approximate hardware units.
__device__ __forceinline__ int sc_num(const KP& kp) {
    int n = kp.N;
    asm volatile("" : "+v"(n));
    return n;
}

// QUADS_PARAMS_DICT (utils.py:33-53)
__device__ __forceinline__ void sc_mode_params(int mode, int& nform, float& low, float& high) {
    if (mode == SC_STATIC_DIFF_GOAL || mode == SC_DYNAMIC_DIFF_GOAL || mode == SC_SWARM_VS_SWARM || mode == SC_RUN_AWAY) {
        nform = 8; low = 0.25f; high = 0.5f;
    } else if (mode == SC_SWAP_GOALS) {
        nform = 8; low = 0.4f; high = 0.8f;
    } else if (mode == SC_O_SWAP_GOALS) {   // QUADS_FORMATION_LIST_OBSTACLES has 7 entries: index into QUADS_FORMATION_LIST
        nform = 7; low = 0.4f; high = 0.8f;
    } else if (mode == SC_DYNAMIC_FORMATIONS) {
        nform = 8; low = 0.f; high = 1.0f;
    } else {
        nform = 1; low = 0.f; high = 0.f;
    }
}
__device__ __forceinline__ int sc_per_layer(int f) { return (f == F_GRID_H || f == F_GRID_XZ || f == F_GRID_YZ) ? 50 : 8; }
__device__ __forceinline__ void sc_grid_dims(int num, int& d1, int& d2) {   // get_grid_dim_number (utils.py:124-136)
    // floor(sqrt(num) + 1e-6) is the integer square root for every num this sees (a non-square's root is over 1e-6
    // below the next integer up to num ~ 1e11): integer arithmetic, folded away when num is a JIT constant
    int g = 0;
    while ((g + 1) * (g + 1) <= num) ++g;
    while (g > 1 && num % g != 0) --g;
    d1 = g;
    d2 = num / g;
}
__device__ __forceinline__ void sc_by_formation(int f, float p0, float p1, float layer, float* g) {   // utils.py:164-175
    if (f == F_CIRCLE_H || f == F_GRID_H) { g[0] = p0; g[1] = p1; g[2] = layer; }
    else if (f == F_CIRCLE_XZ || f == F_GRID_XZ) { g[0] = p0; g[1] = layer; g[2] = p1; }
    else { g[0] = layer; g[1] = p0; g[2] = p1; }
}

// QuadrotorScenario.generate_goals (base.py:42-116) into LDS rows; returns the goal count (sphere >= 3)
__device__ int sc_generate(int f, int n, int per_layer, float size, float layer, const float* c, float* g) {
    if (f <= F_CIRCLE_YZ) {
        const int whole = n / per_layer, rest = n % per_layer;
        for (int i = 0; i < n; ++i) {
            const int cur = n <= per_layer ? n : ((i / per_layer) < whole ? per_layer : rest);
            const float rev = (float)(i % cur) / (float)cur;   // degree / 2 pi
            float* gi = g + 4 * i;
            sc_by_formation(f, size * __builtin_amdgcn_cosf(rev), size * __builtin_amdgcn_sinf(rev),
                            (float)(i / per_layer) * layer, gi);
            gi[0] += c[0]; gi[1] += c[1]; gi[2] += c[2];
        }
        return n;
    }
    if (f == F_SPHERE) {   // generate_points (utils.py:87-103)
        const int m = n < 3 ? 3 : n;
        const float x = 0.1f + 1.2f * (float)m;
        const float start = -1.f + 1.f / ((float)m - 1.f), inc = (2.f - 2.f / ((float)m - 1.f)) / ((float)m - 1.f);
        for (int j = 0; j < m; ++j) {
            const float s = start + (float)j * inc;
            const float sg = s > 0.f ? 1.f : (s < 0.f ? -1.f : 0.f);
            const float a = s * x, bb = 1.5707963267948966f * sg * (1.f - fsqrt(1.f - fabsf(s)));
            const float cb = cos_any(bb);
            float* gj = g + 4 * j;
            gj[0] = size * (cos_any(a) * cb) + c[0];
            gj[1] = size * (sin_any(a) * cb) + c[1];
            gj[2] = size * sin_any(bb) + c[2];
        }
        return m;
    }
    if (f == F_CUBE) {
        // int(np.power(n, 1/3)) as float64 rounds it: 27 ** (1/3) = 2.9999999999999996 -> 2, 64 ** (1/3) -> 3,
        // 125 ** (1/3) = 4.999999999999999 -> 4 (the steps over n <= 128, QS_MAX_AGENTS)
        const int fd = n < 8 ? 1 : (n < 28 ? 2 : (n < 65 ? 3 : (n < 126 ? 4 : 5)));
        for (int i = 0; i < n; ++i) {
            float* gi = g + 4 * i;
            gi[0] = c[2] + size * (float)(i / (fd * fd));
            gi[1] = size * (float)((i / fd) % fd);
            gi[2] = size * (float)(i % fd);
        }
    } else {   // grid
        int d1, d2, r1 = 1, r2 = 1;
        sc_grid_dims(n <= per_layer ? n : per_layer, d1, d2);
        if (n > per_layer && n % per_layer) sc_grid_dims(n % per_layer, r1, r2);
        const int whole = n / per_layer;
        for (int i = 0; i < n; ++i) {
            const int L = i / per_layer;
            const bool full = n <= per_layer || L < whole;
            const int a = full ? d1 : r1, b2 = full ? d2 : r2;
            sc_by_formation(f, size * (float)(i % b2), size * (float)((i / b2) % a), (float)L * layer, g + 4 * i);
        }
    }
    float mean[3] = {0.f, 0.f, 0.f};
    for (int i = 0; i < n; ++i)
        for (int k = 0; k < 3; ++k) mean[k] += g[4 * i + k];
    for (int k = 0; k < 3; ++k) mean[k] /= (float)n;
    for (int i = 0; i < n; ++i)
        for (int k = 0; k < 3; ++k) g[4 * i + k] = g[4 * i + k] - mean[k] + c[k];
    return n;
}

// update_formation_and_relate_param (base.py:126-139) with get_formation_range (utils.py:139-161)
__device__ void sc_update_formation(const KP& kp, Scen& s, SDraw& sd) {
    int nform;
    float low, high;
    sc_mode_params(s.mode, nform, low, high);
    s.form = sd_int(sd, 0, nform);
    const int pl = sc_per_layer(s.form);
    if (s.form <= F_CIRCLE_YZ) {   // get_circle_radius: 0.5 dist / sin(pi / per_layer)
        const float k = 0.5f / __builtin_amdgcn_sinf(0.5f / (float)pl);
        s.lo = low * k; s.hi = high * k;
    } else if (s.form == F_SPHERE) {   // get_sphere_radius
        const int n = s.mode == SC_SWARM_VS_SWARM ? sc_num(kp) / 2 : sc_num(kp);
        const float ratio = (1.75388487222762f - 0.0920858134405214f) /
                                (1.f + exp2f(0.860487305801679f * __log2f((float)n / 10.3632729642351f))) +
                            0.0920858134405214f;
        s.lo = low / ratio; s.hi = high / ratio;
    } else {
        s.lo = low; s.hi = high;
    }
    s.size = sd_uniform(sd, s.lo, s.hi);
    s.layer = sd_uniform(sd, s.lo, s.hi);
}

// get_z_value (utils.py:178-189)
__device__ float sc_z_value(const KP& kp, const Scen& s, SDraw& sd) {
    const float box = kp.spawn_box;
    const float z = sd_uniform(sd, -0.5f * box, 0.5f * box) + 2.0f;
    float lb = 0.25f;
    if (s.form == F_SPHERE || s.form == F_CIRCLE_XZ || s.form == F_CIRCLE_YZ) lb = s.size + 0.25f;
    else if (s.form == F_GRID_XZ || s.form == F_GRID_YZ) {
        int d1, d2;
        sc_grid_dims(min(kp.N, sc_per_layer(s.form)), d1, d2);
        lb = (float)d1 * s.size + 0.25f;
    }
    return fmaxf(z, lb);
}

// swarm_vs_swarm create_formations (swarm_vs_swarm.py:49-54) [+ update_goals' shuffles]; tmp: scratch rows
__device__ void sc_vs_formations(const KP& kp, Scen& s, float* g, float* tmp, bool shuffle, SDraw& sd) {
    const int N = sc_num(kp), pl = sc_per_layer(s.form);
    const int n1 = sc_generate(s.form, N / 2, pl, s.size, s.layer, s.c1, g);
    if (shuffle) sd_shuffle(sd, g, n1);
    const int n2 = sc_generate(s.form, N - N / 2, pl, s.size, s.layer, s.c2, tmp);
    if (shuffle) sd_shuffle(sd, tmp, n2);
    for (int i = 0; i < n2 && n1 + i < N; ++i)
        for (int k = 0; k < 3; ++k) g[4 * (n1 + i) + k] = tmp[4 * i + k];
}

// Scenario_mix.reset (mix.py:79-99) -> <scenario>.__init__ + .reset: the N goals into g
__device__ void scen_reset(const KP& kp, Scen& s, SDraw& sd, float* g, float* tmp) {
    s = Scen{};   // a fresh Scenario_* object per reset (mix.py:88)
    const int N = sc_num(kp);
    const float cf = 1.f / kp.cdt;
    s.mode = kp.scen_b == SC_MIX ? sd_int(sd, 0, N == 1 ? 5 : 9) : kp.scen_b;
    s.period = (int)(5.f * cf);
    s.inc = 0;
    if (s.mode == SC_DYNAMIC_FORMATIONS) {   // dynamic_formations.py:9-16, 42-48
        s.speed = sd_uniform(sd, 1.f, 3.f);
        s.inc = sd_uniform(sd, 0.f, 1.f) < 0.5f;
        s.speed = sd_uniform(sd, 1.f, 3.f);
    } else if (s.mode == SC_DYNAMIC_SAME_GOAL || s.mode == SC_DYNAMIC_DIFF_GOAL || s.mode == SC_SWAP_GOALS ||
               s.mode == SC_SWARM_VS_SWARM) {
        s.period = (int)(sd_uniform(sd, 4.f, 6.f) * cf);
    }
    sc_update_formation(kp, s, sd);
    const int pl = sc_per_layer(s.form);
    if (s.mode == SC_SWARM_VS_SWARM) {   // swarm_vs_swarm.py:125-139, formation_centers :11-47
        const float box = kp.spawn_box;
        const float x = sd_uniform(sd, -box, box), y = sd_uniform(sd, -box, box);
        s.c1[0] = x; s.c1[1] = y; s.c1[2] = sc_z_value(kp, s, sd);
        const float dist = sd_uniform(sd, box / 4.f, box);
        const float phi = sd_uniform(sd, -3.14159265358979f, 3.14159265358979f);
        const float th = sd_uniform(sd, -1.5707963267948966f, 1.5707963267948966f);
        s.c2[0] = s.c1[0] + dist * (sin_any(th) * cos_any(phi));
        s.c2[1] = s.c1[1] + dist * (sin_any(th) * sin_any(phi));
        s.c2[2] = s.c1[2] + dist * cos_any(th);
        const int f = s.form;
        const int ax = (f == F_CIRCLE_H || f == F_GRID_H) ? 2 : (f == F_CIRCLE_XZ || f == F_GRID_XZ) ? 1
                     : (f == F_CIRCLE_YZ || f == F_GRID_YZ) ? 0 : -1;
        if (ax >= 0) {
            const float dd = s.c2[ax] - s.c1[ax];
            if (fabsf(dd) < s.lo) s.c2[ax] = (dd > 0.f ? 1.f : (dd < 0.f ? -1.f : 0.f)) * s.lo + s.c1[ax];
        }
        sc_vs_formations(kp, s, g, tmp, false, sd);
        for (int k = 0; k < 3; ++k) s.c[k] = (s.c1[k] + s.c2[k]) * 0.5f;
        return;
    }
    if (s.mode == SC_EP_LISSAJOUS3D) {   // ep_lissajous3D.py:31-38, no shuffle
        s.c[0] = -2.f; s.c[1] = 0.f; s.c[2] = 2.f;
        sc_generate(s.form, N, pl, s.size, 0.f, s.c, g);
        return;
    }
    s.c[0] = 0.f; s.c[1] = 0.f; s.c[2] = 2.f;   // reset / standard_reset (base.py:144-173)
    const int m = sc_generate(s.form, N, pl, s.size, s.layer, s.c, g);
    sd_shuffle(sd, g, m);
}

// <scenario>.step() after the drones stepped (quadrotor_multi.py:700-701), tick = envs[0].tick
__device__ void scen_step(const KP& kp, Scen& s, int tick, SDraw& sd, float* g, float* tmp) {
    const int N = sc_num(kp);
    const float box = kp.spawn_box, cf = 1.f / kp.cdt;
    const int pl = sc_per_layer(s.form);
    const bool ev = s.period > 0 && tick % s.period == 0 && tick > 0;
    if (s.mode == SC_DYNAMIC_SAME_GOAL) {   // dynamic_same_goal.py:16-29
        if (!ev) return;
        const float x = sd_uniform(sd, -box, box), y = sd_uniform(sd, -box, box);
        const float z = fmaxf(sd_uniform(sd, -0.5f * box, 0.5f * box) + 2.f, 0.25f);
        s.c[0] = x; s.c[1] = y; s.c[2] = z;
        sc_generate(s.form, N, pl, s.size, 0.f, s.c, g);
    } else if (s.mode == SC_DYNAMIC_DIFF_GOAL) {   // dynamic_diff_goal.py:13-40
        if (!ev) return;
        const float x = sd_uniform(sd, -box, box), y = sd_uniform(sd, -box, box);
        const float z = sc_z_value(kp, s, sd);
        s.c[0] = x; s.c[1] = y; s.c[2] = z;
        sc_update_formation(kp, s, sd);
        const int m = sc_generate(s.form, N, sc_per_layer(s.form), s.size, s.layer, s.c, tmp);
        sd_shuffle(sd, tmp, m);
        for (int i = 0; i < 4 * N; ++i) g[i] = tmp[i];
    } else if (s.mode == SC_SWAP_GOALS) {   // swap_goals.py:12-25
        if (ev) sd_shuffle(sd, g, N);
    } else if (s.mode == SC_DYNAMIC_FORMATIONS) {   // dynamic_formations.py:18-40
        if (s.size <= -s.hi) {
            s.inc = 1;
            s.speed = sd_uniform(sd, 1.f, 3.f);
        } else if (s.size >= s.hi) {
            s.inc = 0;
            s.speed = sd_uniform(sd, 1.f, 3.f);
        }
        s.size += (s.inc ? 0.001f : -0.001f) * s.speed;
        sc_generate(s.form, N, pl, s.size, s.layer, s.c, g);
    } else if (s.mode == SC_EP_LISSAJOUS3D) {   // ep_lissajous3D.py:8-26 (accumulates on goals[0])
        const float t = (float)tick / cf;
        const float nx = 0.03f * sin_any(t) + g[0], ny = 0.01f * sin_any(2.f * t + 90.f) + g[1],
                    nz = 0.01f * cos_any(2.f * t + 90.f) + g[2];
        for (int i = 0; i < N; ++i) { g[4 * i] = nx; g[4 * i + 1] = ny; g[4 * i + 2] = nz; }
    } else if (s.mode == SC_EP_RAND_BEZIER) {   // ep_rand_bezier.py:6-47
        const int steps = (int)(5.f * cf);
        const int t = tick % steps;
        float hi[3], lo[3];
        const float mx = bz_bounds(kp, s.size, hi, lo);
        if (t == 0 || tick == 1) {
            float np_[3][2];
            for (int tries = 0;; ++tries)   // the reference loops without a bound
                if (bz_try(sd, hi, lo, mx, g, np_) || tries >= BZ_MAX_TRIES - 1) break;
            for (int k = 0; k < 3; ++k) {
                s.bz[k] = g[k];
                s.bz[3 + k] = np_[k][0];
                s.bz[6 + k] = np_[k][1];
            }
        }
        if (t != 0 && tick > 1) {   // interp[:, t] of the degree-2 Bezier (bezier's Bernstein evaluation)
            const float sp = t == steps - 1 ? 1.f : (float)t * (1.f / (float)(steps - 1));
            const float l1 = 1.f - sp;
            float pt[3];
            for (int k = 0; k < 3; ++k) pt[k] = (l1 * s.bz[k] + 2.f * sp * s.bz[3 + k]) * l1 + sp * sp * s.bz[6 + k];
            for (int i = 0; i < N; ++i) { g[4 * i] = pt[0]; g[4 * i + 1] = pt[1]; g[4 * i + 2] = pt[2]; }
        }
    } else if (s.mode == SC_SWARM_VS_SWARM) {   // swarm_vs_swarm.py:56-76
        if (!ev) return;
        for (int k = 0; k < 3; ++k) {
            const float t3 = s.c1[k];
            s.c1[k] = s.c2[k];
            s.c2[k] = t3;
        }
        sc_update_formation(kp, s, sd);
        sc_vs_formations(kp, s, g, tmp, true, sd);
    } else if (s.mode == SC_RUN_AWAY) {   // run_away.py:16-27
        if (tick % (int)(1.f * cf) == 0 && tick > 0 && N >= 2) {
            const int a = sd_int(sd, 1, N), b2 = sd_int(sd, 1, N);
            float ga[3], gb[3];
            for (int k = 0; k < 3; ++k) { ga[k] = g[4 * a + k]; gb[k] = g[4 * b2 + k]; }
            for (int k = 0; k < 3; ++k) { g[k] = ga[k]; g[4 + k] = gb[k]; }
        }
    }
}

// ---------------------------------------------------------------------------------------------
// scenario.step() on every lane of the env at once (flavor-B step kernel).  scen_step above runs the
// reference's loops over the env's drones on the env's lead lane while the env's other lanes wait; here every
// lane runs the same scalar code (the same Philox words, the same formation scalars) and computes only its
// own drone's goal: generate_goals' row of the drone (sc_row), the cube / grid centring by a running sum over
// the rows (the same rows in the same order, the sums bitwise the lead lane's), and a Generator.shuffle as the
// drone's row tracked through the swaps (sd_track) instead of swapping a table.  Bitwise the same goals and
// scenario state as scen_step (and so oracle/quadswarm_oracle_scen.c draw for draw).
// ---------------------------------------------------------------------------------------------

// generate_goals' row i before the cube / grid centring (circle and sphere rows are final) -- sc_generate's
// per-row expressions
__device__ __forceinline__ void sc_row(int f, int n, int per_layer, float size, float layer, const float* c, int i,
                                       float* gi) {
    // n: the row count as an integer constant of the specialised kernel where the JIT knows it (index arithmetic
    // only: exact, folded); per_layer is sc_per_layer(f), a literal in each branch (8 circles, 50 grids); the
    // sphere's float geometry takes n through an opaque copy (sc_num: no constant-folded transcendentals)
    (void)per_layer;
    if (f <= F_CIRCLE_YZ) {
        constexpr int PL = 8;
        int idx = i, cur = n;   // n <= 8 (one layer): i % n = i
        if (n > PL) {
            const int whole = n / PL, rest = n % PL;
            cur = (i / PL) < whole ? PL : rest;
            idx = i % cur;
        }
        const float rev = (float)idx / (float)cur;
        sc_by_formation(f, size * __builtin_amdgcn_cosf(rev), size * __builtin_amdgcn_sinf(rev),
                        (float)(i / PL) * layer, gi);
        gi[0] += c[0]; gi[1] += c[1]; gi[2] += c[2];
    } else if (f == F_SPHERE) {
        int m = n < 3 ? 3 : n;
        asm volatile("" : "+v"(m));
        const float x = 0.1f + 1.2f * (float)m;
        const float start = -1.f + 1.f / ((float)m - 1.f), inc = (2.f - 2.f / ((float)m - 1.f)) / ((float)m - 1.f);
        const float s = start + (float)i * inc;
        const float sg = s > 0.f ? 1.f : (s < 0.f ? -1.f : 0.f);
        const float a = s * x, bb = 1.5707963267948966f * sg * (1.f - fsqrt(1.f - fabsf(s)));
        const float cb = cos_any(bb);
        gi[0] = size * (cos_any(a) * cb) + c[0];
        gi[1] = size * (sin_any(a) * cb) + c[1];
        gi[2] = size * sin_any(bb) + c[2];
    } else if (f == F_CUBE) {
        const int fd = n < 8 ? 1 : (n < 28 ? 2 : (n < 65 ? 3 : (n < 126 ? 4 : 5)));
        gi[0] = c[2] + size * (float)(i / (fd * fd));
        gi[1] = size * (float)((i / fd) % fd);
        gi[2] = size * (float)(i % fd);
    } else {
        constexpr int PL = 50;
        int d1, d2, r1 = 1, r2 = 1;
        sc_grid_dims(n <= PL ? n : PL, d1, d2);
        if (n > PL && n % PL) sc_grid_dims(n % PL, r1, r2);
        const int whole = n / PL, L = i / PL;
        const bool full = n <= PL || L < whole;
        const int a = full ? d1 : r1, b2 = full ? d2 : r2;
        sc_by_formation(f, size * (float)(i % b2), size * (float)((i / b2) % a), (float)L * layer, gi);
    }
}
// sc_generate's row count (a sphere has at least 3 points)
__device__ __forceinline__ int sc_count(int f, int n) { return (f == F_SPHERE && n < 3) ? 3 : n; }

// the centring of cube / grid formations (sc_generate's mean): rows 0..n-1 summed in order, each row from
// running counters (the divisions of sc_row only where a grid's last, partial layer starts)
__device__ __forceinline__ void sc_center(int f, int n, int per_layer, float size, float layer, const float* c,
                                          float* gi) {
    if (f <= F_CIRCLE_YZ || f == F_SPHERE) return;
    float mean[3] = {0.f, 0.f, 0.f};
    if (f == F_CUBE) {
        const int fd = n < 8 ? 1 : (n < 28 ? 2 : (n < 65 ? 3 : (n < 126 ? 4 : 5)));
        int u = 0, v = 0, w = 0;   // j % fd, (j / fd) % fd, j / fd^2
        for (int j = 0; j < n; ++j) {
            float gj[3];   // sc_row's cube row j, one statement per coordinate as there (same contraction)
            gj[0] = c[2] + size * (float)w;
            gj[1] = size * (float)v;
            gj[2] = size * (float)u;
            mean[0] += gj[0]; mean[1] += gj[1]; mean[2] += gj[2];
            if (++u == fd) { u = 0; if (++v == fd) { v = 0; ++w; } }
        }
    } else {
        (void)per_layer;
        constexpr int PL = 50;   // sc_per_layer of the grids
        int d1, d2, r1 = 1, r2 = 1;
        sc_grid_dims(n <= PL ? n : PL, d1, d2);
        if (n > PL && n % PL) sc_grid_dims(n % PL, r1, r2);
        const int whole = n / PL;
        int L = 0, jl = 0, a = d1, b2 = d2, u = 0, v = 0;   // layer, index in layer, j % b2, (j / b2) % a
        float s0 = 0.f, s1 = 0.f, sl = 0.f;
        for (int j = 0; j < n; ++j) {
            if (jl == PL) {
                ++L;
                jl = 0;
                const bool full = n <= per_layer || L < whole;
                a = full ? d1 : r1;
                b2 = full ? d2 : r2;
                u = j % b2;
                v = (j / b2) % a;
            }
            // the row's three terms summed per term and placed by the formation's axes after the loop: each
            // coordinate's sum sees the same values in the same order as sc_generate's (no branch per row)
            const float p0 = size * (float)u, p1 = size * (float)v, pl = (float)L * layer;   // rounded products:
            s0 += p0;                                                                          // separate statements
            s1 += p1;                                                                          // (no contraction
            sl += pl;                                                                          // into FMAs)
            ++jl;
            if (++u == b2) { u = 0; if (++v == a) v = 0; }
        }
        sc_by_formation(f, s0, s1, sl, mean);
    }
    for (int k = 0; k < 3; ++k) mean[k] /= (float)n;
    for (int k = 0; k < 3; ++k) gi[k] = gi[k] - mean[k] + c[k];
}

// where row `pos` of an n-row table ends after sd_shuffle (Fisher-Yates from the top), consuming the same words
__device__ __forceinline__ int sd_track(SDraw& s, int pos, int n) {
    for (int i = n - 1; i >= 1; --i) {
        const int j = sd_int(s, 0, i + 1);
        pos = pos == i ? j : (pos == j ? i : pos);
    }
    return pos;
}

// the env's scenario: the record's mode under quads_mode=mix, else the config's (a constant of the specialised
// kernel, so that its step code is the only one compiled in)
__device__ __forceinline__ int sc_mode(const KP& kp, int rec_mode) { return kp.scen_b == SC_MIX ? rec_mode : kp.scen_b; }

// does scenario.step() change anything at this tick (scen_step's branches)
__device__ __forceinline__ bool scen_acts(const KP& kp, int mode, int period, int tick) {
    mode = sc_mode(kp, mode);
    const bool ev = period > 0 && tick % period == 0 && tick > 0;
    switch (mode) {
        case SC_DYNAMIC_SAME_GOAL: case SC_DYNAMIC_DIFF_GOAL: case SC_SWAP_GOALS: case SC_SWARM_VS_SWARM: return ev;
        case SC_RUN_AWAY: return tick % (int)(1.f * (1.f / kp.cdt)) == 0 && tick > 0 && kp.N >= 2;
        case SC_EP_LISSAJOUS3D: case SC_EP_RAND_BEZIER: case SC_DYNAMIC_FORMATIONS: return true;
        case SC_O_SWAP_GOALS: return ev;
        case SC_O_EP_RAND_BEZIER: return true;
        case SC_O_DYNAMIC_SAME_GOAL: return (period > 0 && tick % period == 0) || tick == 1;
        default: return false;
    }
}

// the scenario record of an env as 27 words (scen_load's fields): 0-3 mode, form, period, inc (env rows
// QS_E_SC_MODE..); 4-26 the env's env-major env_f run QS_ENVF_SC_SIZE.. (size lo hi layer speed c[3] bz[9] c1[3] c2[3])
constexpr int SC_WORDS = 27;
__device__ __forceinline__ uint32_t scen_word(const KP& kp, const Bufs& b, int env, int w) {
    return w < 4 ? (uint32_t)b.env[(QS_E_SC_MODE + w) * kp.E + env]
                 : __float_as_uint(*scf(b.envf, kp.E, env, QS_ENVF_SC_SIZE + w - 4));
}
__device__ __forceinline__ void scen_from_words(const uint32_t* r, Scen& s) {
    s.mode = (int)r[0]; s.form = (int)r[1]; s.period = (int)r[2]; s.inc = (int)r[3];
    s.size = __uint_as_float(r[4]); s.lo = __uint_as_float(r[5]); s.hi = __uint_as_float(r[6]);
    s.layer = __uint_as_float(r[7]); s.speed = __uint_as_float(r[8]);
    for (int i = 0; i < 3; ++i) {
        s.c[i] = __uint_as_float(r[9 + i]);
        s.c1[i] = __uint_as_float(r[21 + i]);
        s.c2[i] = __uint_as_float(r[24 + i]);
    }
    for (int i = 0; i < 9; ++i) s.bz[i] = __uint_as_float(r[12 + i]);
}

// scen_step for drone di's lane.  ta: the env's goals (rows of 4 floats) as the step left them (read by the modes
// that use other drones' goals); tb: the shuffled goals (the shuffling modes write their drones' rows there and
// set via_tab: the new goal is tb's row di after a barrier).  goal: in, the drone's goal; out, its new goal.
// Returns what of the scenario record changed: 0 nothing, 1 size / inc / speed, 2 more (the whole record).
// oc: the env's obstacle map (the obstacle scenarios only).
__device__ __forceinline__ int scen_step_lane(const KP& kp, Scen& s, int tick, SDraw& sd, int di, const float* ta,
                                              float* tb, float* goal, bool& via_tab, int bz_first = 0,
                                              const OCtx* oc = nullptr) {
    const int N = kp.N;   // index arithmetic (a constant of the specialised kernel); float geometry: sc_row / sc_num
    const float box = kp.spawn_box, cf = 1.f / kp.cdt;
    const int pl = sc_per_layer(s.form);
    const bool ev = s.period > 0 && tick % s.period == 0 && tick > 0;
    via_tab = false;
    const int mode = sc_mode(kp, s.mode);
    if (mode == SC_DYNAMIC_SAME_GOAL) {   // dynamic_same_goal.py:16-29
        if (!ev) return 0;
        const float x = sd_uniform(sd, -box, box), y = sd_uniform(sd, -box, box);
        const float z = fmaxf(sd_uniform(sd, -0.5f * box, 0.5f * box) + 2.f, 0.25f);
        s.c[0] = x; s.c[1] = y; s.c[2] = z;
        sc_row(s.form, N, pl, s.size, 0.f, s.c, di, goal);
        sc_center(s.form, N, pl, s.size, 0.f, s.c, goal);
        return 2;
    } else if (mode == SC_DYNAMIC_DIFF_GOAL) {   // dynamic_diff_goal.py:13-40
        if (!ev) return 0;
        const float x = sd_uniform(sd, -box, box), y = sd_uniform(sd, -box, box);
        const float z = sc_z_value(kp, s, sd);
        s.c[0] = x; s.c[1] = y; s.c[2] = z;
        sc_update_formation(kp, s, sd);
        const int f = s.form, pl2 = sc_per_layer(f), m = sc_count(f, N);
        const SDraw s0 = sd;   // the shuffle's words, for every row of the generated table
        for (int r = di; r < m; r += N) {
            float gr[3];
            sc_row(f, N, pl2, s.size, s.layer, s.c, r, gr);
            sc_center(f, N, pl2, s.size, s.layer, s.c, gr);
            SDraw t = s0;
            const int p = sd_track(t, r, m);
            if (p < N) { tb[4 * p] = gr[0]; tb[4 * p + 1] = gr[1]; tb[4 * p + 2] = gr[2]; }
        }
        via_tab = true;
        return 2;
    } else if (mode == SC_SWAP_GOALS) {   // swap_goals.py:12-25
        if (!ev) return 0;
        const int p = sd_track(sd, di, N);
        tb[4 * p] = goal[0]; tb[4 * p + 1] = goal[1]; tb[4 * p + 2] = goal[2];
        via_tab = true;
        return 0;
    } else if (mode == SC_DYNAMIC_FORMATIONS) {   // dynamic_formations.py:18-40
        if (s.size <= -s.hi) {
            s.inc = 1;
            s.speed = sd_uniform(sd, 1.f, 3.f);
        } else if (s.size >= s.hi) {
            s.inc = 0;
            s.speed = sd_uniform(sd, 1.f, 3.f);
        }
        s.size += (s.inc ? 0.001f : -0.001f) * s.speed;
        sc_row(s.form, N, pl, s.size, s.layer, s.c, di, goal);
        sc_center(s.form, N, pl, s.size, s.layer, s.c, goal);
        return 1;
    } else if (mode == SC_EP_LISSAJOUS3D) {   // ep_lissajous3D.py:8-26 (accumulates on goals[0])
        const float t = (float)tick / cf;
        const float nx = 0.03f * sin_any(t) + ta[0], ny = 0.01f * sin_any(2.f * t + 90.f) + ta[1],
                    nz = 0.01f * cos_any(2.f * t + 90.f) + ta[2];
        goal[0] = nx; goal[1] = ny; goal[2] = nz;
        return 0;
    } else if (mode == SC_EP_RAND_BEZIER || mode == SC_O_EP_RAND_BEZIER) {
        // ep_rand_bezier.py:6-47; o_ep_rand_bezier.py:14-53 (6 s curves, max_dist min(5, .), z in [1.5, 3])
        const bool ob = mode == SC_O_EP_RAND_BEZIER;
        const int steps = (int)((ob ? 6.f : 5.f) * cf);
        const int t = tick % steps;
        float hi[3], lo[3];
        const float mx = bz_bounds(kp, s.size, hi, lo, ob);
        int ch = 0;
        if (t == 0 || tick == 1) {
            // the rejection loop from try bz_first on (the first try any lane of the env found accepted, or 0): the
            // tries before it are rejected, so the loop ends on the same try as one from 0 would
            float np_[3][2];
            const int cap = ob ? BZ_MAX_TRIES_O : BZ_MAX_TRIES;
            sd.k += (uint32_t)(BZ_WORDS * bz_first);
            for (int tries = bz_first;; ++tries)   // the reference loops without a bound
                if (bz_try(sd, hi, lo, mx, ta, np_) || tries >= cap - 1) break;
            for (int k = 0; k < 3; ++k) {
                s.bz[k] = ta[k];
                s.bz[3 + k] = np_[k][0];
                s.bz[6 + k] = np_[k][1];
            }
            ch = 2;
        }
        if (t != 0 && tick > 1) {   // interp[:, t] of the degree-2 Bezier (bezier's Bernstein evaluation)
            const float sp = t == steps - 1 ? 1.f : (float)t * (1.f / (float)(steps - 1));
            const float l1 = 1.f - sp;
            for (int k = 0; k < 3; ++k) goal[k] = (l1 * s.bz[k] + 2.f * sp * s.bz[3 + k]) * l1 + sp * sp * s.bz[6 + k];
        }
        return ch;
    } else if (mode == SC_SWARM_VS_SWARM) {   // swarm_vs_swarm.py:56-76 (sc_vs_formations with the shuffles)
        if (!ev) return 0;
        for (int k = 0; k < 3; ++k) {
            const float t3 = s.c1[k];
            s.c1[k] = s.c2[k];
            s.c2[k] = t3;
        }
        sc_update_formation(kp, s, sd);
        const int f = s.form, pl2 = sc_per_layer(f);
        const int h1 = N / 2, h2 = N - N / 2, m1 = sc_count(f, h1), m2 = sc_count(f, h2);
        for (int rr = di; rr < m1 + m2; rr += N) {   // group 1's rows, then group 2's
            const bool g2 = rr >= m1;
            const int r = g2 ? rr - m1 : rr, n = g2 ? h2 : h1;
            const float* cc = g2 ? s.c2 : s.c1;
            float gr[3];
            sc_row(f, n, pl2, s.size, s.layer, cc, r, gr);
            sc_center(f, n, pl2, s.size, s.layer, cc, gr);
            SDraw t = sd;
            if (g2) t.k += (uint32_t)(m1 - 1);   // group 1's shuffle words come first
            const int p = sd_track(t, r, g2 ? m2 : m1);
            const int slot = g2 ? m1 + p : p;
            if (slot < N) { tb[4 * slot] = gr[0]; tb[4 * slot + 1] = gr[1]; tb[4 * slot + 2] = gr[2]; }
        }
        via_tab = true;
        return 2;
    } else if (mode == SC_O_SWAP_GOALS) {   // o_swap_goals.py:14-24: np.random.shuffle(self.goals) every 4-6 s
        if (!ev) return 0;
        if (s.form == F_SPHERE && N < 3) {   // 3 goal rows (generate_points): the 1-2 no drone holds are c1 / c2
            int idx[3] = {0, 1, 2};
            for (int i = 2; i >= 1; --i) {
                const int j = sd_int(sd, 0, i + 1);
                const int t = idx[i];
                idx[i] = idx[j];
                idx[j] = t;
            }
            float old[3][3];
            for (int r = 0; r < 3; ++r)
                for (int k = 0; k < 3; ++k) old[r][k] = r < N ? ta[4 * r + k] : (r == N ? s.c1[k] : s.c2[k]);
            for (int k = 0; k < 3; ++k) {
                goal[k] = old[idx[di]][k];
                s.c1[k] = old[idx[N]][k];
                if (N + 1 < 3) s.c2[k] = old[idx[N + 1]][k];
            }
            return 2;
        }
        const int p = sd_track(sd, di, N);
        tb[4 * p] = goal[0]; tb[4 * p + 1] = goal[1]; tb[4 * p + 2] = goal[2];
        via_tab = true;
        return 0;
    } else if (mode == SC_O_DYNAMIC_SAME_GOAL) {   // o_dynamic_same_goal.py:17-29
        if (!((s.period > 0 && tick % s.period == 0) || tick == 1)) return 0;
        // generate_pos_obst_map() until the new goal is within max_dist = 4 of the end point: one free cell (choice of
        // len(free_space)) and z ~ U(0.75, 3) per try, 2 words
        const int F = oc->n * oc->n - oc->m;
        float ng[3];
        for (int tries = 0;; ++tries) {   // the reference loops without a bound
            const float2 xy = o_free_cell(*oc, sd_int(sd, 0, F));
            ng[0] = xy.x; ng[1] = xy.y; ng[2] = sd_uniform(sd, 0.75f, 3.f);
            const float dx = s.c[0] - ng[0], dy = s.c[1] - ng[1], dz = s.c[2] - ng[2];
            if (!(fsqrt(dx * dx + dy * dy + dz * dz) > 4.f) || tries >= ODS_MAX_TRIES - 1) break;
        }
        for (int k = 0; k < 3; ++k) s.c[k] = goal[k] = ng[k];
        return 2;
    } else if (mode == SC_RUN_AWAY) {   // run_away.py:16-27
        if (tick % (int)(1.f * cf) == 0 && tick > 0 && N >= 2) {
            const int a = sd_int(sd, 1, N), b2 = sd_int(sd, 1, N);
            const int src = di == 0 ? a : b2;
            if (di < 2) { goal[0] = ta[4 * src]; goal[1] = ta[4 * src + 1]; goal[2] = ta[4 * src + 2]; }
        }
        return 0;
    }
    return 0;
}
// ep_rand_bezier's rejection loop over the env's lanes: the env's LA active lanes (li < LA) evaluate tries li,
// li + LA, ... (each try's 7 words sit at a fixed offset of the stream), a ballot of their lane segment finds the
// first accepted try; returns it (the same on the env's lanes), or BZ_MAX_TRIES - 1 when none of the first
// BZ_MAX_TRIES - 1 tries is accepted, i.e. where the serial loop stops.  `need`: this lane's env resamples at this
// tick (false on other lanes: they idle through the rounds).  An env that needed ~300 tries held its wave (and the
// launch) for ~340 us serially (c3mix, ticks 1 / 500 / 1000).
template <int LPE>
__device__ __forceinline__ int bz_first_parallel(const KP& kp, const uint32_t* srec, bool need, int li, int lbase,
                                                 int LA, const Rng& r, uint32_t key, const float* ta) {
    static_assert(LPE <= 64, "the env's lanes inside one wave");
    const uint64_t seg = LA >= 64 ? ~0ull : ((1ull << LA) - 1ull);
    float hi[3], lo[3];
    const bool ob = kp.scen_b == SC_O_EP_RAND_BEZIER;
    const int cap = ob ? BZ_MAX_TRIES_O : BZ_MAX_TRIES;
    const float mx = bz_bounds(kp, __uint_as_float(srec[4]), hi, lo, ob);
    int found = need ? -1 : 0;
    for (int rd = 0;; ++rd) {
        const int tr = rd * LA + li;
        bool ok = false;
        if (found < 0 && tr < cap) {
            SDraw t = sdraw(r, key, S_SCN);
            t.k = (uint32_t)(BZ_WORDS * tr);
            float np_[3][2];
            ok = bz_try(t, hi, lo, mx, ta, np_);
        }
        const uint64_t m = (__ballot(ok) >> lbase) & seg;
        if (found < 0 && m) found = min(rd * LA + (int)__ffsll((long long)m) - 1, cap - 1);
        if (found < 0 && (rd + 1) * LA >= cap - 1) found = cap - 1;
        if (__ballot(found < 0) == 0ull) break;
    }
    return found;
}

__device__ __forceinline__ void scen_store_size(const KP& kp, const Bufs& b, int env, const Scen& s) {
    b.env[QS_E_SC_INC * kp.E + env] = s.inc;
    *scf(b.envf, kp.E, env, QS_ENVF_SC_SIZE) = s.size;
    *scf(b.envf, kp.E, env, QS_ENVF_SC_SPEED) = s.speed;
}

// LDS goal tables of the env (2 x (NPAD + 4) rows of 4 floats), after the obs / exchange tiles, then the env's
// scenario record (SC_WORDS words, padded to 32; the flavor-B step kernel's copy for scen_step_lane)
template <int NPAD>
constexpr int scen_stride() { return 2 * (NPAD + 4) * 4 + 32; }
__device__ __forceinline__ float* scen_tab(float* lds, const KP& kp, int slots) {
    return lds + slots * kp.obs_dim + slots * 8 + 64;
}

}  // namespace qs
