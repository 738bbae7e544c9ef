/* quadswarm_oracle_scen.c -- TEST INFRASTRUCTURE: float64 restatement of the flavor-B goal scenarios
 * (gym_art/quadrotor_multi/scenarios/) for the CPU parity oracle.  Never shipped, never measured.
 *
 * Every function cites the reference lines it restates.  Draws come from an or_sdraw source: either a
 * TAPE (the values the reference drew, in call order: Generator.integers / .uniform / .shuffle as the
 * resulting permutation, np.random.uniform / .randint; tools/gen_golden_scen.py records them) or Philox
 * (keyed like the GPU kernels: key {env id, seed}, counter {index / 4, stream | UNIF, tick, episode},
 * one 32-bit word per draw, drawn in call order), so the GPU is compared draw-for-draw with this file in
 * Philox mode and this file is pinned to the reference in tape mode.
 */
#include <math.h>
#include <string.h>

#include "quadswarm_oracle.h"

/* QUADS_FORMATION_LIST (scenarios/utils.py:24-25) */
enum { F_CIRCLE_H = 0, F_CIRCLE_XZ, F_CIRCLE_YZ, F_SPHERE, F_GRID_H, F_GRID_XZ, F_GRID_YZ, F_CUBE };

/* ---------------------------------------------------------------------------------------------- */
/* draws                                                                                           */
/* ---------------------------------------------------------------------------------------------- */
static double sd_next(or_sdraw* s) {
    if (s->tape_pos < s->tape_n) return s->tape[s->tape_pos++];
    s->overrun = 1;
    return 0.0;
}
static uint32_t sd_word(or_sdraw* s) {
    const uint32_t k = s->count++;
    const uint32_t ctr[4] = {k >> 2, s->stream | OR_UNIF_BIT, (uint32_t)s->step, (uint32_t)(s->step >> 32)};
    const uint32_t key[2] = {s->key, s->seed};
    uint32_t w[4];
    or_philox4x32_10(ctr, key, w);
    return w[k & 3];
}
/* Generator.uniform(lo, hi) / np.random.uniform(lo, hi) */
double or_sd_uniform(or_sdraw* s, double lo, double hi) {
    if (s->mode == OR_RNG_TAPE) return sd_next(s);
    const uint32_t w = sd_word(s);
    return lo + (hi - lo) * (((double)(w >> 8) + 0.5) * (1.0 / 16777216.0));
}
/* Generator.integers(lo, hi) / np.random.randint(lo, hi): lo <= x < hi, floor(u m) computed exactly */
int or_sd_int(or_sdraw* s, int lo, int hi) {
    if (s->mode == OR_RNG_TAPE) return (int)sd_next(s);
    const uint32_t w = sd_word(s);
    const uint64_t m = (uint64_t)(hi - lo);
    return lo + (int)((((uint64_t)(w >> 8) * 2u + 1u) * m) >> 25);
}
/* Generator.shuffle(goals[0..n)): tape = the resulting permutation (new[i] = old[perm[i]]); Philox =
 * Fisher-Yates from the top (i = n-1 .. 1, j = floor(u (i+1))), the order numpy's shuffle walks */
void or_sd_shuffle(or_sdraw* s, double (*g)[3], int n) {
    if (s->mode == OR_RNG_TAPE) {
        double tmp[OR_MAXN][3];
        memcpy(tmp, g, sizeof(double) * 3 * (size_t)n);
        for (int i = 0; i < n; ++i) {
            const int p = (int)sd_next(s);
            for (int c = 0; c < 3; ++c) g[i][c] = tmp[p][c];
        }
        return;
    }
    for (int i = n - 1; i >= 1; --i) {
        const int j = or_sd_int(s, 0, i + 1);
        for (int c = 0; c < 3; ++c) {
            const double t = g[i][c];
            g[i][c] = g[j][c];
            g[j][c] = t;
        }
    }
}

/* ---------------------------------------------------------------------------------------------- */
/* formations (scenarios/utils.py, scenarios/base.py)                                              */
/* ---------------------------------------------------------------------------------------------- */
/* QUADS_PARAMS_DICT (utils.py:33-53): formations to draw from, [low, high] */
static void mode_params(int mode, int* nform, double* low, double* high) {
    const double arm = 0.05;   /* quad_arm_size, utils.py:32 */
    switch (mode) {
        case OR_SC_STATIC_DIFF_GOAL: case OR_SC_DYNAMIC_DIFF_GOAL: case OR_SC_SWARM_VS_SWARM: case OR_SC_RUN_AWAY:
            *nform = 8; *low = 5 * arm; *high = 10 * arm; return;
        case OR_SC_SWAP_GOALS: *nform = 8; *low = 8 * arm; *high = 16 * arm; return;
        /* QUADS_FORMATION_LIST_OBSTACLES (7 entries) indexes QUADS_FORMATION_LIST (update_formation_and_max_agent_per_layer) */
        case OR_SC_O_SWAP_GOALS: *nform = 7; *low = 8 * arm; *high = 16 * arm; return;
        case OR_SC_DYNAMIC_FORMATIONS: *nform = 8; *low = 0.0; *high = 20 * arm; return;
        default: *nform = 1; *low = 0.0; *high = 0.0; return;   /* ['circle_horizontal'], [0, 0] */
    }
}

/* update_formation_and_max_agent_per_layer (utils.py:56-70) */
static int per_layer_of(int f) { return (f == F_GRID_H || f == F_GRID_XZ || f == F_GRID_YZ) ? 50 : 8; }

/* get_grid_dim_number (utils.py:124-136) */
static void grid_dims(int num, int* d1, int* d2) {
    int g = (int)floor(sqrt((double)num));
    while (g > 1) {
        if (num % g == 0) break;
        --g;
    }
    *d1 = g;
    *d2 = num / g;
}

static double circle_radius(int num, double dist) { return (0.5 * dist) / sin((2 * M_PI / num) / 2); }  /* :117-121 */
static double sphere_radius(int num, double dist) {                                                      /* :106-114 */
    const double A = 1.75388487222762, B = 0.860487305801679, C = 10.3632729642351, D = 0.0920858134405214;
    return dist / ((A - D) / (1 + pow(num / C, B)) + D);
}

/* get_formation_range (utils.py:139-161) */
static void formation_range(int mode, int f, int num_agents, double low, double high, int per_layer, double* lo,
                            double* hi) {
    const int n = mode == OR_SC_SWARM_VS_SWARM ? num_agents / 2 : num_agents;
    if (f <= F_CIRCLE_YZ) { *lo = circle_radius(per_layer, low); *hi = circle_radius(per_layer, high); }
    else if (f == F_SPHERE) { *lo = sphere_radius(n, low); *hi = sphere_radius(n, high); }
    else { *lo = low; *hi = high; }
}

/* get_goal_by_formation (utils.py:164-175) */
static void by_formation(int f, double p0, double p1, double layer, double* g) {
    if (f == F_CIRCLE_H || f == F_GRID_H) { g[0] = p0; g[1] = p1; g[2] = layer; }
    else if (f == F_CIRCLE_XZ || f == F_GRID_XZ) { g[0] = p0; g[1] = layer; g[2] = p1; }
    else { g[0] = layer; g[1] = p0; g[2] = p1; }
}

/* QuadrotorScenario.generate_goals (base.py:42-116).  Returns the number of goals written: the sphere
 * formation makes at least 3 (generate_points, utils.py:87-103). */
int or_generate_goals(int f, int n, int per_layer, double size, double layer_dist, const double* center,
                      double (*g)[3]) {
    if (f <= F_CIRCLE_YZ) {
        const int whole = n / per_layer, rest = n % per_layer;
        for (int i = 0; i < n; ++i) {
            const int cur = n <= per_layer ? n : ((i / per_layer) < whole ? per_layer : rest);
            const double deg = 2 * M_PI * (i % cur) / cur;
            by_formation(f, size * cos(deg), size * sin(deg), (i / per_layer) * layer_dist, g[i]);
            for (int c = 0; c < 3; ++c) g[i][c] += center[c];
        }
        return n;
    }
    if (f == F_SPHERE) {
        const int m = n < 3 ? 3 : n;
        const double x = 0.1 + 1.2 * m;
        const double start = -1. + 1. / (m - 1.);
        const double inc = (2. - 2. / (m - 1.)) / (m - 1.);
        for (int j = 0; j < m; ++j) {
            const double s = start + j * inc;
            const double sg = s > 0 ? 1.0 : (s < 0 ? -1.0 : 0.0);
            const double a = s * x, b = M_PI / 2. * sg * (1. - sqrt(1. - fabs(s)));
            const double pt[3] = {cos(a) * cos(b), sin(a) * cos(b), sin(b)};
            for (int c = 0; c < 3; ++c) g[j][c] = size * pt[c] + center[c];
        }
        return m;
    }
    if (f == F_CUBE) {
        const int fd = (int)pow((double)n, 1.0 / 3);
        for (int i = 0; i < n; ++i) {
            g[i][0] = center[2] + size * (i / (fd * fd));
            g[i][1] = size * ((i / fd) % fd);
            g[i][2] = size * (i % fd);
        }
    } else {   /* grid */
        int d1, d2, r1 = 1, r2 = 1;
        grid_dims(n <= per_layer ? n : per_layer, &d1, &d2);
        if (n > per_layer && n % per_layer) grid_dims(n % per_layer, &r1, &r2);
        const int whole = n / per_layer;
        for (int i = 0; i < n; ++i) {
            const int L = i / per_layer;
            const int full = n <= per_layer || L < whole;
            const int a = full ? d1 : r1, b = full ? d2 : r2;
            by_formation(f, size * (i % b), size * ((i / b) % a), L * layer_dist, g[i]);
        }
    }
    double mean[3] = {0, 0, 0};   /* np.mean(goals, axis=0) */
    for (int i = 0; i < n; ++i)
        for (int c = 0; c < 3; ++c) mean[c] += g[i][c];
    for (int c = 0; c < 3; ++c) mean[c] /= n;
    for (int i = 0; i < n; ++i)
        for (int c = 0; c < 3; ++c) g[i][c] = g[i][c] - mean[c] + center[c];
    return n;
}

/* update_formation_and_relate_param (base.py:126-139) + update_layer_dist (utils.py:73-78) */
static void update_formation(const or_params* p, or_scen* sc, or_sdraw* s) {
    int nform;
    double low, high;
    mode_params(sc->mode, &nform, &low, &high);
    sc->formation = or_sd_int(s, 0, nform);
    sc->per_layer = per_layer_of(sc->formation);
    formation_range(sc->mode, sc->formation, p->num_agents, low, high, sc->per_layer, &sc->lo, &sc->hi);
    sc->size = or_sd_uniform(s, sc->lo, sc->hi);
    sc->layer = or_sd_uniform(s, sc->lo, sc->hi);
}

/* get_z_value (utils.py:178-189), np.random */
static double z_value(int n, int per_layer, double box, int f, double size, or_sdraw* s) {
    const double z = or_sd_uniform(s, -0.5 * box, 0.5 * box) + 2.0;
    double lb = 0.25;
    if (f == F_SPHERE || f == F_CIRCLE_XZ || f == F_CIRCLE_YZ) lb = size + 0.25;
    else if (f == F_GRID_XZ || f == F_GRID_YZ) {
        int d1, d2;
        grid_dims(n < per_layer ? n : per_layer, &d1, &d2);
        lb = d1 * size + 0.25;
    }
    return z > lb ? z : lb;
}

/* Scenario_swarm_vs_swarm.create_formations (swarm_vs_swarm.py:49-54) [+ the shuffles of update_goals
 * :66-71]: goals_1 (N // 2 around c1) then goals_2 (the rest around c2); surplus sphere points spill */
static void vs_formations(const or_params* p, or_scen* sc, double (*g)[3], int shuffle, or_sdraw* s) {
    double g1[OR_MAXN][3], g2[OR_MAXN][3];
    const int N = p->num_agents;
    const int n1 = or_generate_goals(sc->formation, N / 2, sc->per_layer, sc->size, sc->layer, sc->c1, g1);
    const int n2 = or_generate_goals(sc->formation, N - N / 2, sc->per_layer, sc->size, sc->layer, sc->c2, g2);
    if (shuffle) {
        or_sd_shuffle(s, g1, n1);
        or_sd_shuffle(s, g2, n2);
    }
    int k = 0;
    for (int i = 0; i < n1 && k < N; ++i, ++k) memcpy(g[k], g1[i], sizeof g1[i]);
    for (int i = 0; i < n2 && k < N; ++i, ++k) memcpy(g[k], g2[i], sizeof g2[i]);
}

/* ---------------------------------------------------------------------------------------------- */
/* reset: Scenario_mix.reset (mix.py:79-99) -> <scenario>.__init__ + .reset; writes the N goals      */
/* ---------------------------------------------------------------------------------------------- */
void or_scen_reset(const or_params* p, or_scen* sc, or_sdraw* s, double (*g)[3]) {
    const int N = p->num_agents;
    memset(sc, 0, sizeof *sc);   /* a fresh Scenario_* object per reset (mix.py:88) */
    const double cf = 1.0 / p->control_dt;                 /* control_freq (quadrotor_single.py:160) */
    sc->mode = p->scenario_b == OR_SC_MIX ? or_sd_int(s, 0, N == 1 ? 5 : 9) : p->scenario_b;  /* mix.py:46-56, 82 */
    double tmp[OR_MAXN][3];
    sc->period = (int)(5.0 * cf);                          /* __init__: duration_time = 5.0 */
    switch (sc->mode) {
        case OR_SC_DYNAMIC_FORMATIONS:                     /* dynamic_formations.py:9-16 (__init__), 42-48 */
            sc->speed = or_sd_uniform(s, 1.0, 3.0);
            sc->increase = or_sd_uniform(s, 0.0, 1.0) < 0.5;
            sc->speed = or_sd_uniform(s, 1.0, 3.0);
            break;
        case OR_SC_DYNAMIC_SAME_GOAL: case OR_SC_DYNAMIC_DIFF_GOAL: case OR_SC_SWAP_GOALS: case OR_SC_SWARM_VS_SWARM:
            sc->period = (int)(or_sd_uniform(s, 4.0, 6.0) * cf);
            break;
        default: break;
    }
    update_formation(p, sc, s);
    if (sc->mode == OR_SC_SWARM_VS_SWARM) {               /* swarm_vs_swarm.py:125-139, formation_centers :11-47 */
        const double box = p->spawn_box, dlow = sc->lo;
        const double x = or_sd_uniform(s, -box, box), y = or_sd_uniform(s, -box, box);
        const double z = z_value(N, sc->per_layer, box, sc->formation, sc->size, s);
        sc->c1[0] = x; sc->c1[1] = y; sc->c1[2] = z;
        const double dist = or_sd_uniform(s, box / 4, box);
        const double phi = or_sd_uniform(s, -M_PI, M_PI), th = or_sd_uniform(s, -0.5 * M_PI, 0.5 * M_PI);
        sc->c2[0] = sc->c1[0] + dist * (sin(th) * cos(phi));
        sc->c2[1] = sc->c1[1] + dist * (sin(th) * sin(phi));
        sc->c2[2] = sc->c1[2] + dist * cos(th);
        const int f = sc->formation;
        const int ax = (f == F_CIRCLE_H || f == F_GRID_H) ? 2 : (f == F_CIRCLE_XZ || f == F_GRID_XZ) ? 1
                     : (f == F_CIRCLE_YZ || f == F_GRID_YZ) ? 0 : -1;
        if (ax >= 0) {
            const double d = sc->c2[ax] - sc->c1[ax];
            if (fabs(d) < dlow) sc->c2[ax] = (d > 0 ? 1.0 : (d < 0 ? -1.0 : 0.0)) * dlow + sc->c1[ax];
        }
        vs_formations(p, sc, g, 0, s);
        for (int c = 0; c < 3; ++c) sc->center[c] = (sc->c1[c] + sc->c2[c]) / 2;
        return;
    }
    if (sc->mode == OR_SC_EP_LISSAJOUS3D) {                /* ep_lissajous3D.py:31-38: no shuffle */
        sc->center[0] = -2.0; sc->center[1] = 0.0; sc->center[2] = 2.0;
        or_generate_goals(sc->formation, N, sc->per_layer, sc->size, 0.0, sc->center, tmp);
        memcpy(g, tmp, sizeof(double) * 3 * (size_t)N);
        return;
    }
    /* QuadrotorScenario.reset / standard_reset (base.py:144-173) */
    sc->center[0] = 0.0; sc->center[1] = 0.0; sc->center[2] = 2.0;
    const int m = or_generate_goals(sc->formation, N, sc->per_layer, sc->size, sc->layer, sc->center, tmp);
    or_sd_shuffle(s, tmp, m);
    memcpy(g, tmp, sizeof(double) * 3 * (size_t)N);
}

/* bezier.Curve(nodes, degree=2).evaluate_multi -- third-party `bezier` (unpinned, absent here): its
 * Bernstein evaluation (evaluate_multi_barycentric with lambda1 = 1 - s, lambda2 = s) */
static void bezier2(const double (*nd)[3], double s, double* out) {
    const double l1 = 1.0 - s, l2 = s;
    for (int c = 0; c < 3; ++c) {
        double r = l1 * nd[0][c];
        r += 2.0 * l2 * nd[1][c];
        r *= l1;
        r += l2 * l2 * nd[2][c];
        out[c] = r;
    }
}

/* ---------------------------------------------------------------------------------------------- */
/* step: <scenario>.step() after the drones stepped (quadrotor_multi.py:700-701), tick = envs[0].tick */
/* ---------------------------------------------------------------------------------------------- */
void or_scen_step(const or_params* p, or_scen* sc, int tick, or_sdraw* s, double (*g)[3]) {
    const int N = p->num_agents;
    const double box = p->spawn_box, cf = 1.0 / p->control_dt;
    double tmp[OR_MAXN][3];
    switch (sc->mode) {
        case OR_SC_DYNAMIC_SAME_GOAL:                      /* dynamic_same_goal.py:16-29 (np.random) */
            if (tick % sc->period == 0 && tick > 0) {
                const double x = or_sd_uniform(s, -box, box), y = or_sd_uniform(s, -box, box);
                double z = or_sd_uniform(s, -0.5 * box, 0.5 * box) + 2.0;
                z = z > 0.25 ? z : 0.25;
                sc->center[0] = x; sc->center[1] = y; sc->center[2] = z;
                or_generate_goals(sc->formation, N, sc->per_layer, sc->size, 0.0, sc->center, tmp);
                memcpy(g, tmp, sizeof(double) * 3 * (size_t)N);
            }
            return;
        case OR_SC_DYNAMIC_DIFF_GOAL:                      /* dynamic_diff_goal.py:13-40 */
            if (tick % sc->period == 0 && tick > 0) {
                const double x = or_sd_uniform(s, -box, box), y = or_sd_uniform(s, -box, box);
                const double z = z_value(N, sc->per_layer, box, sc->formation, sc->size, s);
                sc->center[0] = x; sc->center[1] = y; sc->center[2] = z;
                update_formation(p, sc, s);
                const int m = or_generate_goals(sc->formation, N, sc->per_layer, sc->size, sc->layer, sc->center, tmp);
                or_sd_shuffle(s, tmp, m);
                memcpy(g, tmp, sizeof(double) * 3 * (size_t)N);
            }
            return;
        case OR_SC_SWAP_GOALS:                             /* swap_goals.py:12-25 */
            if (tick % sc->period == 0 && tick > 0) or_sd_shuffle(s, g, N);
            return;
        case OR_SC_DYNAMIC_FORMATIONS:                     /* dynamic_formations.py:18-40 */
            if (sc->size <= -sc->hi) {
                sc->increase = 1;
                sc->speed = or_sd_uniform(s, 1.0, 3.0);
            } else if (sc->size >= sc->hi) {
                sc->increase = 0;
                sc->speed = or_sd_uniform(s, 1.0, 3.0);
            }
            if (sc->increase) sc->size += 0.001 * sc->speed;
            else sc->size -= 0.001 * sc->speed;
            or_generate_goals(sc->formation, N, sc->per_layer, sc->size, sc->layer, sc->center, tmp);
            memcpy(g, tmp, sizeof(double) * 3 * (size_t)N);
            return;
        case OR_SC_EP_LISSAJOUS3D: {                       /* ep_lissajous3D.py:8-26 (accumulates on goals[0]) */
            const double t = tick / cf;
            const double x = 0.03 * sin(t), y = 0.01 * sin(2 * t + 90), z = 0.01 * cos(2 * t + 90);
            const double nx = x + g[0][0], ny = y + g[0][1], nz = z + g[0][2];
            for (int i = 0; i < N; ++i) { g[i][0] = nx; g[i][1] = ny; g[i][2] = nz; }
            return;
        }
        case OR_SC_EP_RAND_BEZIER: {                       /* ep_rand_bezier.py:6-47 (np.random) */
            const int steps = (int)(5 * cf);
            const int t = tick % steps;
            const double rd[3] = {p->room_hi[0] - p->room_lo[0] - sc->size, p->room_hi[1] - p->room_lo[1] - sc->size,
                                  p->room_hi[2] - p->room_lo[2] - sc->size};
            double mx = rd[0] > rd[1] ? rd[0] : rd[1];
            mx = mx > rd[2] ? mx : rd[2];
            const double max_dist = mx < 30 ? mx : 30, min_dist = max_dist / 2;
            if (t == 0 || tick == 1) {
                const double lo[3] = {-rd[0] / 2, -rd[1] / 2, 0}, hi[3] = {rd[0] / 2, rd[1] / 2, rd[2]};
                double np_[3][2];
                for (int tries = 0;; ++tries) {
                    /* uniform(low=-high, high=high, size=(2, 3)).reshape(3, 2): element [c][j] is flat 2c + j,
                     * drawn with the bounds of column (2c + j) % 3; node j = column j */
                    double u[6];
                    for (int k = 0; k < 6; ++k) u[k] = or_sd_uniform(s, -hi[k % 3], hi[k % 3]);
                    /* np.random.randint(min_dist, max_dist + 1): numpy truncates float bounds */
                    const double mag = (double)or_sd_int(s, (int)min_dist, (int)floor(max_dist) + 1);
                    int ok = 1;
                    for (int j = 0; j < 2; ++j) {
                        const double v[3] = {u[j], u[2 + j], u[4 + j]};
                        const double nrm = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
                        for (int q = 0; q < 3; ++q) {
                            np_[q][j] = v[q] * mag / nrm + g[0][q];
                            if (!(np_[q][j] > lo[q] + 0.5 && np_[q][j] < hi[q] - 0.5)) ok = 0;
                        }
                    }
                    if (ok || tries >= 1023 || s->overrun) break;   /* the reference loops without a bound */
                }
                for (int q = 0; q < 3; ++q) {
                    sc->bz[0][q] = g[0][q];
                    sc->bz[1][q] = np_[q][0];
                    sc->bz[2][q] = np_[q][1];
                }
            }
            if (t != 0 && tick > 1) {                      /* interp[:, t], pts = linspace(0, 1, steps) */
                double pt[3];
                bezier2((const double(*)[3])sc->bz, t == steps - 1 ? 1.0 : t * (1.0 / (steps - 1)), pt);
                for (int i = 0; i < N; ++i) memcpy(g[i], pt, sizeof pt);
            }
            return;
        }
        case OR_SC_SWARM_VS_SWARM:                         /* swarm_vs_swarm.py:56-76 */
            if (tick % sc->period == 0 && tick > 0) {
                double t3[3];
                memcpy(t3, sc->c1, sizeof t3);
                memcpy(sc->c1, sc->c2, sizeof t3);
                memcpy(sc->c2, t3, sizeof t3);
                update_formation(p, sc, s);
                vs_formations(p, sc, g, 1, s);
            }
            return;
        case OR_SC_RUN_AWAY:                               /* run_away.py:16-27 (np.random) */
            if (tick % (int)(1.0 * cf) == 0 && tick > 0) {
                const int a = or_sd_int(s, 1, N), b = or_sd_int(s, 1, N);
                double ga[3], gb[3];
                memcpy(ga, g[a], sizeof ga);
                memcpy(gb, g[b], sizeof gb);
                memcpy(g[0], ga, sizeof ga);
                memcpy(g[1], gb, sizeof gb);
            }
            return;
        default:
            return;   /* static_same_goal, static_diff_goal */
    }
}

/* ---------------------------------------------------------------------------------------------- */
/* the obstacle maps' dynamic scenarios (scenarios/obstacles/o_swap_goals.py, o_ep_rand_bezier.py,   */
/* o_dynamic_same_goal.py; o_base.py).  free_space = np.where(map == 0): cells in row-major order;  */
/* cell (x, y) of free_space -> cell_centers[x + n y] (or_cell_xy(x, y)).                          */
/* ---------------------------------------------------------------------------------------------- */
static int free_cells(const unsigned char* map, int n, int* fr) {
    int F = 0;
    for (int c = 0; c < n * n; ++c) if (!map[c]) fr[F++] = c;
    return F;
}
/* Scenario_o_base.max_square_area_center's cell centre (o_base.py:125-153), z drawn by the caller */
static void max_square_xy(const unsigned char* map, int n, double xy[2]) { or_max_square_center(map, n, xy); }

/* generate_pos_obst_map_2 (o_base.py:74-88): np.random.choice(range(F), N, replace=False), then one
 * np.random.uniform(1, 3) per drone (tape mode only) */
static void tape_spawns(or_sdraw* s, int N, int* sp_cells, double* sp_z, const int* fr) {
    for (int i = 0; i < N; ++i) sp_cells[i] = fr[(int)or_sd_uniform(s, 0, 0)];
    for (int i = 0; i < N; ++i) sp_z[i] = or_sd_uniform(s, 1.0, 3.0);
}

void or_oscen_reset(const or_params* p, int omode, or_scen* sc, or_sdraw* s, const unsigned char* map, int n,
                    int* sp_cells, double* sp_z, double (*g)[3]) {
    const int N = p->num_agents, tape = s->mode == OR_RNG_TAPE;
    const double cf = 1.0 / p->control_dt;
    int fr[64 * 64];
    const int F = free_cells(map, n, fr);
    memset(sc, 0, sizeof *sc);
    sc->mode = omode == 2 ? OR_SC_O_SWAP_GOALS : (omode == 3 ? OR_SC_O_EP_RAND_BEZIER : OR_SC_O_DYNAMIC_SAME_GOAL);
    double xy[2];
    if (omode == 3) {                                      /* o_ep_rand_bezier.py:55-103 */
        sc->period = (int)(0.01 * cf);
        if (tape) tape_spawns(s, N, sp_cells, sp_z, fr);
        /* end_point = generate_pos_obst_map() (o_base.py:58-72) */
        const int c = fr[tape ? (int)or_sd_uniform(s, 0, 0) : or_sd_int(s, 0, F)];
        or_cell_xy(c / n, c % n, n, xy);
        sc->center[0] = xy[0]; sc->center[1] = xy[1]; sc->center[2] = or_sd_uniform(s, 0.75, 3.0);
        if (tape) {   /* the 10 trajectory points it samples and never uses (:79-96): replay their draws */
            int pts[10], np_ = 0, Fc = F;
            double cc[64][2];
            for (int i = 0; i < n * n; ++i) or_cell_xy(i % n, i / n, n, cc[i]);   /* cell_centers[i] */
            while (np_ < 10 && !s->overrun) {
                const int idx = (int)or_sd_uniform(s, 0, 0);   /* np.random.choice(len(free_space)) */
                int far = 0;
                for (int k = 0; k < np_; ++k) {
                    const double dx = cc[pts[k]][0] - cc[idx][0], dy = cc[pts[k]][1] - cc[idx][1];
                    if (sqrt(dx * dx + dy * dy) > 4.0) far = 1;
                }
                if (far) continue;
                pts[np_++] = idx;
                --Fc;
            }
            (void)Fc;
            update_formation(p, sc, s);                    /* circle_horizontal, size 0 */
        }
        for (int i = 0; i < N; ++i) memcpy(g[i], sc->center, sizeof sc->center);
        return;
    }
    sc->period = (int)(or_sd_uniform(s, 4.0, 6.0) * cf);  /* duration_time ~ U(4, 6) */
    if (omode == 2) {                                      /* o_swap_goals.py:27-52 */
        update_formation(p, sc, s);
        if (tape) tape_spawns(s, N, sp_cells, sp_z, fr);
        max_square_xy(map, n, xy);
        sc->center[0] = xy[0]; sc->center[1] = xy[1]; sc->center[2] = or_sd_uniform(s, 1.5, 3.0);
        double tmp[OR_MAXN][3];
        const int m = or_generate_goals(sc->formation, N, sc->per_layer, sc->size, sc->layer, sc->center, tmp);
        or_sd_shuffle(s, tmp, m);                          /* np.random.shuffle(self.goals) */
        memcpy(g, tmp, sizeof(double) * 3 * (size_t)N);
        /* a sphere of N < 3 drones has 3 goals: the scenario keeps the rows no drone takes (they are shuffled
         * back in at the next swap) -- in c1 / c2 */
        if (m > N) memcpy(sc->c1, tmp[N], sizeof sc->c1);
        if (m > N + 1) memcpy(sc->c2, tmp[N + 1], sizeof sc->c2);
        return;
    }
    /* o_dynamic_same_goal.py:31-51 */
    if (tape) tape_spawns(s, N, sp_cells, sp_z, fr);
    max_square_xy(map, n, xy);
    sc->center[0] = xy[0]; sc->center[1] = xy[1]; sc->center[2] = or_sd_uniform(s, 1.5, 3.0);
    if (tape) update_formation(p, sc, s);                  /* circle_horizontal, size 0 */
    for (int i = 0; i < N; ++i) memcpy(g[i], sc->center, sizeof sc->center);
}

void or_oscen_step(const or_params* p, or_scen* sc, int tick, or_sdraw* s, const unsigned char* map, int n,
                   double (*g)[3]) {
    const int N = p->num_agents, tape = s->mode == OR_RNG_TAPE;
    const double cf = 1.0 / p->control_dt;
    int fr[64 * 64];
    const int F = free_cells(map, n, fr);
    switch (sc->mode) {
        case OR_SC_O_SWAP_GOALS:                           /* o_swap_goals.py:14-24 */
            if (tick % sc->period == 0 && tick > 0) {      /* np.random.shuffle(self.goals): all of its rows */
                const int m = (sc->formation == 3 && N < 3) ? 3 : N;   /* F_SPHERE: generate_points makes >= 3 */
                double t[OR_MAXN + 2][3];
                memcpy(t, g, sizeof(double) * 3 * (size_t)N);
                if (m > N) memcpy(t[N], sc->c1, sizeof sc->c1);
                if (m > N + 1) memcpy(t[N + 1], sc->c2, sizeof sc->c2);
                or_sd_shuffle(s, t, m);
                memcpy(g, t, sizeof(double) * 3 * (size_t)N);
                if (m > N) memcpy(sc->c1, t[N], sizeof sc->c1);
                if (m > N + 1) memcpy(sc->c2, t[N + 1], sizeof sc->c2);
            }
            return;
        case OR_SC_O_DYNAMIC_SAME_GOAL:                    /* o_dynamic_same_goal.py:17-29 */
            if (tick % sc->period == 0 || tick == 1) {
                double ng[3];
                for (int tries = 0;; ++tries) {            /* generate_pos_obst_map() until within max_dist = 4 */
                    const int c = fr[tape ? (int)or_sd_uniform(s, 0, 0) : or_sd_int(s, 0, F)];
                    double xy[2];
                    or_cell_xy(c / n, c % n, n, xy);
                    ng[0] = xy[0]; ng[1] = xy[1]; ng[2] = or_sd_uniform(s, 0.75, 3.0);
                    const double d[3] = {sc->center[0] - ng[0], sc->center[1] - ng[1], sc->center[2] - ng[2]};
                    if (!(sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]) > 4.0) || tries >= 4095 || s->overrun) break;
                }
                memcpy(sc->center, ng, sizeof ng);
                for (int i = 0; i < N; ++i) memcpy(g[i], ng, sizeof ng);
            }
            return;
        case OR_SC_O_EP_RAND_BEZIER: {                     /* o_ep_rand_bezier.py:14-53 */
            const int steps = (int)(6 * cf);
            const int t = tick % steps;
            const double rd[3] = {p->room_hi[0] - p->room_lo[0] - sc->size, p->room_hi[1] - p->room_lo[1] - sc->size,
                                  p->room_hi[2] - p->room_lo[2] - sc->size};
            double mx = rd[0] > rd[1] ? rd[0] : rd[1];
            mx = mx > rd[2] ? mx : rd[2];
            const double max_dist = mx < 5 ? mx : 5, min_dist = max_dist / 2;
            if (t == 0 || tick == 1) {
                const double lo[3] = {-rd[0] / 2, -rd[1] / 2, 1.5}, hi[3] = {rd[0] / 2, rd[1] / 2, 3.0};
                double np_[3][2];
                for (int tries = 0;; ++tries) {
                    double u[6];
                    for (int k = 0; k < 6; ++k) u[k] = or_sd_uniform(s, -hi[k % 3], hi[k % 3]);
                    const double mag = (double)or_sd_int(s, (int)min_dist, (int)floor(max_dist) + 1);
                    int ok = 1;
                    for (int j = 0; j < 2; ++j) {
                        const double v[3] = {u[j], u[2 + j], u[4 + j]};
                        const double nrm = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
                        for (int q = 0; q < 3; ++q) {
                            np_[q][j] = v[q] * mag / nrm + g[0][q];
                            if (!(np_[q][j] > lo[q] + 0.5 && np_[q][j] < hi[q] - 0.5)) ok = 0;
                        }
                    }
                    if (ok || tries >= 8191 || s->overrun) break;   /* the reference loops without a bound */
                }
                for (int q = 0; q < 3; ++q) {
                    sc->bz[0][q] = g[0][q];
                    sc->bz[1][q] = np_[q][0];
                    sc->bz[2][q] = np_[q][1];
                }
            }
            if (t != 0 && tick > 1) {
                double pt[3];
                bezier2((const double(*)[3])sc->bz, t == steps - 1 ? 1.0 : t * (1.0 / (steps - 1)), pt);
                for (int i = 0; i < N; ++i) memcpy(g[i], pt, sizeof pt);
            }
            return;
        }
        default:
            return;
    }
}
