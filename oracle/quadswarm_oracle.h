/* quadswarm_oracle.h -- CPU restatement of the reference's swarm env step (flavors B and A).
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity oracle (and the bench's cpu_baseline "port"
 * leg).  The product path (HIP kernels behind include/quadswarm.h) never links or calls it.
 *
 * Every function cites the reference file:line it restates (paths relative to the reference
 * root, priban42/quad-swarm-rl-stable-baselines3).  Arithmetic is float64, like the reference.
 *
 * Random draws come from an or_rng:
 *   OR_RNG_PHILOX : counter-based Philox4x32-10, keyed exactly like the GPU kernel
 *                   (key = {drone global id, seed}, counter = {block, stream, env tick, env episode}),
 *                   so GPU fp32 and oracle fp64 consume identical underlying draws.
 *   OR_RNG_TAPE   : replays values recorded from the reference's own np.random calls, in the
 *                   reference's call order (tools/gen_golden.py), so the oracle can be pinned
 *                   bit-for-bit against the reference on full noisy trajectories.
 */
#ifndef QUADSWARM_ORACLE_H
#define QUADSWARM_ORACLE_H
/* drones per env: the largest swarm the build steps (QS_MAX_AGENTS, the paper's 128 quads, paper/fps_compare.py:7) */
#define OR_MAXN 128
#include <stdint.h>

/* OR_F32: the same sources as an fp32 twin (liboracle_f32.so, built with -fsingle-precision-constant),
 * used only as the bench's fp32 cpu_baseline leg ("C++ restatement, fp32, same SoA").
 * Every double becomes float and <tgmath.h> maps the libm calls to their float versions.  Parity
 * tests use the fp64 build only. */
#ifdef OR_F32
#include <math.h>
#include <omp.h>
#include <string.h>
#include <tgmath.h>
#undef I   /* complex.h's imaginary unit (pulled in by tgmath.h) */
#define double float
#endif

#ifdef __cplusplus
extern "C" {
#endif

/* ---- Philox stream ids (shared numbering with the HIP kernel, csrc/qs_rng.h) ---- */
enum {
    OR_S_OU = 1,          /* OU thrust noise: 4 normals                      */
    OR_S_FLOOR = 2,       /* floor flip yaw: 1 uniform; | substep << 8        */
    OR_S_SENSOR = 3,      /* sensor noise: normals pos 0-2, vel 3-5, omega 6-8 */
    OR_S_PAIR = 4,        /* drone-drone impulse, key = lower id; | j << 8    */
    OR_S_WALL = 5,
    OR_S_CEIL = 6,
    OR_S_DW = 7,          /* downwash per-source scalars                     */
    OR_S_DWPAIR = 8,      /* downwash per applied pair; | j << 8              */
    OR_S_RESET = 9,       /* spawn uniforms 0-2                               */
    OR_S_RESET_YAW = 10,  /* yaw rejection uniforms                           */
    OR_S_RESET_SENSOR = 11,
    OR_S_OBST = 12,
    /* flavor A */
    OR_S_CAM = 13,        /* neighbour camera pixel noise (obs pass): normals 0 (u1), 1 (u2); | j << 8 */
    OR_S_CAM_SEL = 14,    /* same, neighbour-selection pass (k < N-1)          */
    OR_S_SELF_CAM = 15,   /* ndist self obs: normals 0, 1                       */
    OR_S_RESET_A = 16,    /* per drone: uniforms 0-1 spawn direction, 2 heading */
    OR_S_SCEN = 17,       /* per env (key = drone 0): uniforms 0 spawn radius, 1-2 target dir, 3 target radius */
    OR_S_RESET_CAM = 18,
    OR_S_RESET_CAM_SEL = 19,
    OR_S_RESET_SELF_CAM = 20,
    /* obstacles (flavor B) */
    OR_S_OBSTMAP = 21,    /* per env: uniforms 0..M-1 partial Fisher-Yates over the grid cells     */
    OR_S_OSCEN = 22,      /* per env: uniform 0 mode, 1..N spawn cells, N+1..2N goal cells, 2N+1 goal z */
    /* flavor-B goal scenarios (quadswarm_oracle_scen.c): per env (key = drone 0), one word per draw in call order */
    OR_S_SCN = 23,        /* scenario.step() draws                                                  */
    OR_S_SCN_RESET = 24,  /* mix mode + scenario __init__ / reset draws                             */
    OR_S_DR = 26,         /* per env (key = drone 0): uniform 0 density choice, 1 size choice (wrapper reset) */
    OR_UNIF_BIT = 0x80    /* uniform draws use stream | OR_UNIF_BIT           */
};

/* flavor-A neighbour features, in get_rel_pos_vel_item order (quadrotor_multi_rewards.py:326-420) */
enum {
    OR_NF_DIST = 1, OR_NF_NDIST = 2, OR_NF_ANGLE = 4, OR_NF_SANGLE = 8, OR_NF_NSANGLE = 16,
    OR_NF_HEADING = 32, OR_NF_SHEADING = 64, OR_NF_NPOS = 128, OR_NF_POS = 256, OR_NF_VEL = 512
};
/* flavor-A self obs reprs (get_state.py:7-223) */
enum { OR_OA_AW = 0, OR_OA_CDIST_ANGLE = 1, OR_OA_CDIST_SANGLE = 2, OR_OA_CDIST_NDIST_NSANGLE = 3 };
/* flavor-A PIDs, state layout or_drone.pid[2*k] = last_error, [2*k+1] = integral */
enum { OR_PID_POS_Z = 0, OR_PID_VEL = 1, OR_PID_ATT = 4, OR_PID_RATE = 7, OR_NPID = 10 };

enum { OR_RNG_PHILOX = 0, OR_RNG_TAPE = 1 };

typedef struct {
    int mode;
    uint32_t seed;
    uint64_t step;          /* Philox counter words 2,3 = {tick, episode}; set per env by the env calls */
    /* tape mode */
    const double* tape;      /* np.random legacy draws (global stream)          */
    long tape_n, tape_pos;
    const double* spawn;     /* Generator draws used for spawn positions        */
    long spawn_n, spawn_pos;
    int overrun;             /* set when a tape ran dry                         */
} or_rng;

/* Physical + env parameters (host-derived, mirrors QuadrotorDynamics.update_model
 * quadrotor_dynamics.py:106-168 and QuadrotorEnvMulti.__init__ quadrotor_multi.py:26-227). */
typedef struct {
    double mass, inertia[3];
    double thrust_max[4], torque_max[4], prop_cross[4][3], prop_ccw[4];
    double motor_tau_up, motor_tau_down, motor_linearity;
    double arm, gravity, omega_max, vel_damp, damp_omega_quadratic;
    double dt;                 /* 1/sim_freq = 0.005                                 */
    int sim_steps;             /* physics substeps per control tick (2)              */
    double since_last_svd_limit;
    double room_lo[3], room_hi[3];
    double ou_mu, ou_theta, ou_sigma;
    int sense_noise;           /* 0 = bypass                                          */
    double pos_norm_std, pos_unif_range, vel_norm_std, vel_unif_range;
    double gyro_noise_density, quat_norm_std, quat_unif_range, acc_static_std, acc_dyn_ratio;
    /* env */
    int num_agents, num_envs, ep_len;
    int obs_repr;              /* 0 xyz_vxyz_R_omega(18) 1 +floor(19) 2 +wall(24)     */
    int k_neighbors;           /* visible neighbours (0 = none)                       */
    double collision_threshold, collision_falloff_threshold, control_dt;
    double rew_pos, rew_effort, rew_crash, rew_orient, rew_spin;
    double rew_quadcol_bin, rew_quadcol_smooth_max;
    int use_downwash, apply_collision_force;
    double spawn_box;          /* QuadrotorSingle.box = 2.0                           */
    double goal[3];            /* static_same_goal formation centre (0,0,2)            */
    uint32_t id_offset;        /* global id of drone 0 (Philox key), for sharded runs    */
    /* ---- flavor A: quadrotor_multi_rewards.py / quadrotor_single_rewards.py / Controller/ ---- */
    int flavor;                /* 0 = B (quadrotor_multi.py), 1 = A                     */
    int obs_repr_a;            /* OR_OA_*                                                */
    int nfeat;                 /* OR_NF_* mask of the neighbour obs type                 */
    int nfeat_dim;             /* floats per visible neighbour                           */
    int ticks_per_step;        /* 8 single-env ticks per QuadrotorEnvMulti.step (:636)    */
    int scenario_a;            /* 0 = goals/spawns left as set (tests), 1 = dynamic_repulsive */
    double nclip_lo[8], nclip_hi[8];   /* neighbour obs clip box per feature (float32 Box) */
    double cam_size, cam_focal, cam_px_noise, cam_fov_deg, cam_res;
    int n_cameras;
    double heading_rate;       /* Controller.MAX_ANGULAR_RATE = pi*80/180                */
    double speed;              /* fixed 0.2 m/s (Controller.py:88)                       */
    double pid_kp[OR_NPID], pid_kd[OR_NPID], pid_ki[OR_NPID], pid_sat[OR_NPID], pid_aw[OR_NPID];
    double rate_out_scale;     /* RateController output x800                             */
    double mixer[16];          /* Mixer.allocation_matrix_inv, row-major 4x4             */
    double m_mass, m_g, m_kf, m_min_rpm, m_max_rpm;
    int m_n_motors;
    double w_captor, w_helper, existence;
    double target_vmax, target_dt, arena_size, target_z;
    /* ---- obstacles (flavor B): quadrotor_multi.py:128-140, 405-426; obstacles/; scenarios/obstacles/ ---- */
    int use_obstacles;
    int num_obstacles;         /* int(density * area_l * area_w)                          */
    int obst_area;             /* spawn area side (8), 1 m grid cells                     */
    int obst_scenario;         /* 0 = mix (o_random / o_static_same_goal), 1 = o_random, 2 = o_static_same_goal,
                                  3 = o_swap_goals, 4 = o_ep_rand_bezier, 5 = o_dynamic_same_goal (obstacle mode + 1) */
    double obst_size;          /* diameter (0.6); radius = size / 2                        */
    double obst_z;             /* pillar centre z = room height / 2 (only the 3-D inside test) */
    double sdf_resolution;     /* 0.1                                                      */
    double rew_quadcol_bin_obst;
    /* ---- flavor-B goal scenarios (scenarios/ files): OR_SC_NONE = the fixed static_same_goal goal ---- */
    int scenario_b;
    /* ---- obstacle domain randomisation (ExperienceReplayWrapper, quad_experience_replay.py:76-87, 106-118,
     * 206-214; env side quadrotor_multi.py:440-450).  Index 0 of each table is the configured value
     * (num_obstacles / obst_size); choice c of the wrapper's np.arange list is index c + 1.  A choice whose
     * density or size is 0.0 is falsy at quadrotor_multi.py:443-446 and keeps the env's current value:
     * dr_counts[c + 1] = -1, dr_sizes[c + 1] = 0. ---- */
    int dr_n_counts, dr_counts[9];
    int dr_n_sizes;
    double dr_sizes[9];
} or_params;

/* flavor-B scenarios, QUADS_MODE_LIST order (scenarios/utils.py:7-10) + run_away; OR_SC_MIX draws one per
 * reset (scenarios/mix.py) */
enum { OR_SC_NONE = -1, OR_SC_STATIC_SAME_GOAL = 0, OR_SC_STATIC_DIFF_GOAL, OR_SC_EP_LISSAJOUS3D,
       OR_SC_EP_RAND_BEZIER, OR_SC_DYNAMIC_SAME_GOAL, OR_SC_DYNAMIC_DIFF_GOAL, OR_SC_DYNAMIC_FORMATIONS,
       OR_SC_SWAP_GOALS, OR_SC_SWARM_VS_SWARM, OR_SC_RUN_AWAY, OR_SC_MIX,
       /* the obstacle maps' dynamic scenarios (scenarios/obstacles/, QUADS_MODE_LIST_OBSTACLES_TEST) */
       OR_SC_O_SWAP_GOALS, OR_SC_O_EP_RAND_BEZIER, OR_SC_O_DYNAMIC_SAME_GOAL };

/* per-env scenario state (the attributes of the reference's Scenario_* object) */
typedef struct {
    int mode, formation, per_layer, period, increase;
    double size, lo, hi, layer, speed;   /* formation_size, lowest/highest_formation_size, layer_dist, control_speed */
    double center[3];                    /* formation_center                                     */
    double bz[3][3];                     /* ep_rand_bezier curve nodes (goals[0], new_pos[:, 0], new_pos[:, 1]) */
    double c1[3], c2[3];                 /* swarm_vs_swarm goal_center_1 / _2                    */
} or_scen;

/* scenario draw source: tape (reference values in call order) or Philox (see quadswarm_oracle_scen.c) */
typedef struct {
    int mode;                            /* OR_RNG_PHILOX / OR_RNG_TAPE */
    uint32_t seed, key, stream, count;
    uint64_t step;
    const double* tape;
    long tape_n, tape_pos;
    int overrun;
} or_sdraw;

/* Per-drone state (QuadrotorDynamics attributes + QuadrotorSingle bookkeeping). */
typedef struct {
    double pos[3], vel[3], rot[9], omega[3], acc[3];
    double thrust_rot_damp[4], thrust_cmds_damp[4];
    double ou[4];
    double since_last_svd;
    int on_floor, crashed_floor, crashed_wall, crashed_ceiling;
    int prev_wall, prev_ceiling;   /* quadrotor_multi.py:604-605 (stores the NEW lists)   */
    double goal[3];
    /* flavor A: Controller state (PIDs that reach an output, heading, last command) */
    double pid[2 * OR_NPID];
    double angle, ang_vel;
    int prev_obst;             /* in prev_obst_quad_collisions (quadrotor_multi.py:585) */
    /* episode_extra_stats (flavor B, quadrotor_multi.py:153-216, 541-657): agent_col_agent / agent_col_obst
     * cleared (hit_* = 1), reached_goal, in prev_crashed_room; distance_to_goal[i] kept as its last 5
     * entries (ring by tick % 5) and its sums over the final 100 / 300 / 500 entries of the episode */
    int hit_agent, hit_obst, reached, prev_room;
    double dring[5];
    double dsum[3];
    double ep_dist[3];         /* distance_to_goal_1s / _3s / _5s of the last finished episode */
    /* the step's per-drone reward components (OR_RI_*): the raw terms behind infos[i]["rewards"]
     * (quadrotor_single.py:34-105, quadrotor_multi.py:608-651); flavor A: OR_RI_GOAL_DIST = infos[i]["goal_dist"]
     * of the last executed tick (quadrotor_single_rewards.py:457) */
    double rinfo[8];
} or_drone;
enum { OR_RI_DIST = 0, OR_RI_EFFORT, OR_RI_CRASH, OR_RI_ORIENT, OR_RI_SPIN, OR_RI_QUADCOL, OR_RI_PROX, OR_RI_OBST,
       OR_NRI, OR_RI_GOAL_DIST = 0 };

/* env-level episode_extra_stats values of a finished episode (quadrotor_multi.py:739-831), the GPU's
 * qs estats columns (include/quadswarm.h QS_ES_*) */
enum { OR_ES_COL = 0, OR_ES_ROOM, OR_ES_FLOOR, OR_ES_WALL, OR_ES_CEIL, OR_ES_COL_SETTLE, OR_ES_COL_FINAL,
       OR_ES_OCOL, OR_ES_OCOL_SETTLE, OR_ES_O35, OR_ES_O5, OR_ES_SUCCESS, OR_ES_DEADLOCK, OR_ES_COLRATE,
       OR_ES_NCOLRATE, OR_ES_OCOLRATE, OR_ES_SCEN, OR_ES_D1, OR_ES_D3, OR_ES_D5, OR_ES_REPLAY, OR_NES = 24 };

typedef struct {
    int tick;
    uint32_t episode;   /* resets so far; with tick it is the env's Philox counter {tick, episode} */
    unsigned char prev_pair_bits[OR_MAXN * OR_MAXN];  /* [i*OR_MAXN+j], i<j: pair collided at the previous step */
    double obs_pos[OR_MAXN][3], obs_vel[OR_MAXN][3];  /* QuadrotorEnvMulti.pos / .vel (neighbour obs) */
    /* flavor A */
    double heading[OR_MAXN];                      /* QuadrotorEnvMulti.heading (stale across resets) */
    double target[2];                        /* Scenario_dynamic_repulsive.pos                  */
    double capture_radius;
    int success;                             /* episode_success                                 */
    int has_pos;                             /* dynamics.pos exists (hasattr check, :38)        */
    /* obstacles */
    int n_obst;
    double obst[64][2];                      /* MultiObstacles.pos_arr xy, in generation order   */
    int obst_mode;                           /* 0 o_random, 1 o_static_same_goal, 2 o_swap_goals, 3 o_ep_rand_bezier,
                                                4 o_dynamic_same_goal (2..4 keep their state in scen) */
    or_scen scen;                            /* flavor-B goal scenario (p->scenario_b != OR_SC_NONE) */
    /* what the experience-replay wrapper reads of the last step (quad_experience_replay.py:161-163,
     * quadrotor_multi.py:725): a new drone collision (.any() of the ids) or obstacle hit; drone 0 on the floor */
    int last_col, last_floor0;
    /* obstacle domain randomisation: the env's current (obst_density, obst_size) as table indices
     * (0 = the configured values) */
    int obst_mi, obst_si;
    /* episode_extra_stats accumulators of the running episode (quadrotor_multi.py:153-171, 487-509):
     * collisions_per_episode, _room_, _floor_, _wall_, _ceiling_, collisions_after_settle, collisions_final_5s,
     * obst_quad_collisions_per_episode, _after_settle, distance_to_goal_3_5, distance_to_goal_5 */
    int st_col, st_room, st_floor, st_wall, st_ceil, st_col_settle, st_col_final;
    int st_ocol, st_ocol_settle, st_o35, st_o5;
    int ep_done;                 /* episodes finished (ep_stats holds the last one's values) */
    double ep_stats[OR_NES];
} or_env;

/* ---- low level pieces (exported for per-function golden tests) ---- */
void or_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
double or_philox_normal(uint32_t seed, uint32_t id, uint32_t stream, uint64_t step, uint32_t idx);
double or_philox_uniform(uint32_t seed, uint32_t id, uint32_t stream, uint64_t step, uint32_t idx);

void or_params_default(or_params* p);
void or_dyn_substep(const or_params* p, or_drone* d, const double cmds[4], const double thr_noise[4],
                    or_rng* r, uint32_t gid, int substep);
void or_ou_noise(const or_params* p, double ou[4], or_rng* r, uint32_t gid);
void or_sensor_noise(const or_params* p, const double pos[3], const double vel[3], const double rot[9],
                     const double omega[3], or_rng* r, uint32_t gid, uint32_t stream,
                     double npos[3], double nvel[3], double nrot[9], double nomega[3]);
void or_polar(double rot[9]);
void or_collide_drones(double pos1[3], double vel1[3], double omega1[3],
                       double pos2[3], double vel2[3], double omega2[3],
                       or_rng* r, uint32_t gid, uint32_t j);
void or_collide_wall(const or_params* p, or_drone* d, or_rng* r, uint32_t gid);
int or_downwash(const or_params* p, or_drone* dr, int N, uint32_t gbase, or_rng* r);   /* 1 when applied */
/* episode_extra_stats accumulators (quadrotor_multi.py:555-656) and the done row (:739-831); flavor A passes
 * dist_goal = NULL (it never appends distance_to_goal) and onew = NULL (no obstacles) */
void or_episode_stats_step(const or_params* p, or_env* ev, or_drone* dr, int N, const int* in_cur, const int* in_prev,
                           const int* onew, const int* wall_new, const int* ceil_new, const double* dist_goal,
                           const double* obs, int od, int time_remain);
void or_episode_stats_done(const or_params* p, or_env* ev, or_drone* dr, int N);
void or_collide_ceiling(or_drone* d, or_rng* r, uint32_t gid);

/* ---- whole env (flavor B, QuadrotorEnvMulti quadrotor_multi.py) ---- */
/* state arrays are num_envs*num_agents drones and num_envs envs. obs is [E*N, obs_dim]. */
int or_obs_dim(const or_params* p);
void or_env_reset(const or_params* p, or_drone* drones, or_env* envs, int env_idx, or_rng* r,
                  double* obs /* rows of this env */);
void or_env_step(const or_params* p, or_drone* drones, or_env* envs, int env_idx, const double* actions,
                 or_rng* r, double* obs, double* rew, unsigned char* done, double* term_obs);
/* batched helpers (Philox mode, OpenMP over envs) */
void or_reset_all(const or_params* p, or_drone* drones, or_env* envs, uint32_t seed, double* obs);
void or_step_all(const or_params* p, or_drone* drones, or_env* envs, const double* actions,
                 uint32_t seed, double* obs, double* rew, unsigned char* done,
                 double* term_obs, int nthreads);

void or_neighbor_obs(const or_params* p, const or_env* ev, double* obs, int obs_dim);

/* obstacles: get_surround_sdfs (obstacles/utils.py:4-27), collision_detection (:30-43),
 * perform_collision_with_obstacle (collisions/obstacles.py:23-50), max_square_area_center (o_base.py:125-153) */
void or_obst_sdf(const or_params* p, const or_env* ev, const double xy[2], double out[9]);
int or_obst_detect(const or_params* p, const or_env* ev, const double xy[2]);
void or_collide_obstacle(const or_params* p, or_drone* d, const double opos[3], or_rng* r, uint32_t gid);
double or_env_obst_size(const or_params* p, const or_env* ev);
void or_max_square_center(const unsigned char* map, int n, double out_xy[2]);
void or_cell_xy(int row, int col, int n, double out_xy[2]);

/* ---- flavor-B goal scenarios (quadswarm_oracle_scen.c) ---- */
double or_sd_uniform(or_sdraw* s, double lo, double hi);
int or_sd_int(or_sdraw* s, int lo, int hi);
void or_sd_shuffle(or_sdraw* s, double (*g)[3], int n);
int or_generate_goals(int formation, int n, int per_layer, double size, double layer_dist, const double* center,
                      double (*g)[3]);
void or_scen_reset(const or_params* p, or_scen* sc, or_sdraw* s, double (*goals)[3]);
void or_scen_step(const or_params* p, or_scen* sc, int tick, or_sdraw* s, double (*goals)[3]);
/* the obstacle maps' dynamic scenarios (quadswarm_oracle_scen.c): omode 2 o_swap_goals, 3 o_ep_rand_bezier,
 * 4 o_dynamic_same_goal; map = the n x n occupancy (row-major).  Tape mode reads the reference's whole reset draw
 * sequence (spawn cells and heights included: sp_cells / sp_z out); Philox mode draws only the scenario's words
 * (S_SCN_RESET order of csrc/qs_flavor_b.h obstacle_reset_env) and leaves the spawns to the caller. */
void or_oscen_reset(const or_params* p, int omode, or_scen* sc, or_sdraw* s, const unsigned char* map, int n,
                    int* sp_cells, double* sp_z, double (*goals)[3]);
void or_oscen_step(const or_params* p, or_scen* sc, int tick, or_sdraw* s, const unsigned char* map, int n,
                   double (*goals)[3]);

/* ---- flavor A (quadrotor_multi_rewards.QuadrotorEnvMulti) ---- */
void or_params_default_a(or_params* p);     /* Controller/ModelParams constants, camera, rewards */
double or_pid_update(double error, double* last_error, double* integral, double dt, double kp, double kd,
                     double ki, double sat, double aw);
void or_ctrl_a(const or_params* p, or_drone* d, double cmd0, double height, double motors[4]);
void or_motors_to_cmds(const double motors[4], double u[4]);
void or_camera(const or_params* p, double rx, double ry, double global_angle, double n1, double n2,
               double* dist, double* angle);
void or_self_obs_a(const or_params* p, const or_drone* d, or_rng* r, uint32_t gid, uint32_t st_sensor,
                   uint32_t st_cam, double* out);
int or_rel_features_x(const or_params* p, const double pr[3], double aw, double hi, double hj, const double vr[3],
                      double n1, double n2, double* f);
#define OR_NB_TRACE_W 12
extern double* or_nb_trace;    /* test hooks: see quadswarm_oracle_a.c */
extern double* or_key_trace;
extern double* or_nb_trace_reset;
extern double* or_key_trace_reset;
void or_neighbor_obs_a(const or_params* p, const or_env* ev, const or_drone* dr, or_rng* r, uint32_t gbase,
                       int reset, double* obs, int obs_dim);
void or_target_step(const or_params* p, or_env* ev, or_drone* dr);
void or_env_reset_a(const or_params* p, or_drone* drones, or_env* envs, int e, or_rng* r, double* obs,
                    unsigned char* reset_info);
void or_env_step_a(const or_params* p, or_drone* drones, or_env* envs, int e, const double* actions,
                   or_rng* r, double* obs, double* rew, unsigned char* done, double* term_obs,
                   unsigned char* reset_info);
void or_reset_all_a(const or_params* p, or_drone* drones, or_env* envs, uint32_t seed, double* obs,
                    unsigned char* reset_info);
void or_step_all_a(const or_params* p, or_drone* drones, or_env* envs, const double* actions, uint32_t seed,
                   double* obs, double* rew, unsigned char* done, double* term_obs, unsigned char* reset_info,
                   int nthreads);
int or_obs_dim_a(const or_params* p);

/* internal draw helpers shared by the flavor files */
double or_rn(or_rng* r, uint32_t gid, uint32_t stream, uint32_t idx, double loc, double scale);
double or_ru(or_rng* r, uint32_t gid, uint32_t stream, uint32_t idx, double lo, double hi);
double or_gnext(or_rng* r);   /* next Generator draw (tape mode: the "spawn"/gtape stream) */

/* sizes for ctypes */
int or_sizeof_params(void);
int or_sizeof_drone(void);
int or_sizeof_env(void);
int or_sizeof_rng(void);

#ifdef __cplusplus
}
#endif
#endif
