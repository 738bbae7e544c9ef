/* quadswarm.h -- C ABI of the MI355X-native quadrotor-swarm environment step (libquadswarm.so).
 *
 * Drop-in boundary for the reference's env-stepping path
 * (priban42/quad-swarm-rl-stable-baselines3), two env flavors:
 *   flavor B (raw motor control, shaped rewards):
 *   - qs_step   replaces QuadrotorEnvMulti.step        gym_art/quadrotor_multi/quadrotor_multi.py:521-841
 *               as driven per env by SubprocVecEnvCustom  swarm_rl/env_wrappers/subproc_vec_env_custom.py:141-153
 *               (worker loop :33-52: step, terminal_observation, auto-reset)
 *   - qs_reset  replaces QuadrotorEnvMulti.reset       quadrotor_multi.py:440-517
 *               (SubprocVecEnvCustom.reset :155-164)
 *   flavor A (what swarm_rl/sb_train.py trains: PID pre-controller, pursuit of a repulsive target):
 *   - qs_step   replaces quadrotor_multi_rewards.QuadrotorEnvMulti.step  quadrotor_multi_rewards.py:630-991
 *               (8 QuadrotorSingle._step ticks, quadrotor_single_rewards.py:418-452, Controller/Controller.py:76-101)
 *               plus the worker's reset on done (subproc_vec_env_custom.py:39-46) with reset_infos
 *   - qs_reset  replaces quadrotor_multi_rewards.QuadrotorEnvMulti.reset   quadrotor_multi_rewards.py:541-627
 *   - qs_set_param("capture_radius") replaces set_capture_radius         quadrotor_multi_rewards.py:212-213
 *   - qs_set_param replaces rew_coeff updates          swarm_rl/env_wrappers/reward_shaping.py:70-76,110-118
 *   - qs_get_state/qs_set_state: env snapshot/restore (no reference equivalent; checkpoint + parity)
 *   - qs_curriculum_step replaces CurriculumCallback._on_step          swarm_rl/custom_callbacks.py:441-468
 *   - qs_curriculum_step_all: the same over every data-parallel rank's envs   custom_callbacks.py:452-462
 *   - qs_attn_*_train_x3 / qs_attn_bwd{1,2}_x3: the PPO update's attention encoder forward + backward
 *                                              (QuadNeighborhoodEncoderAttention, quad_multi_model.py:44-101,
 *                                              under PPO.train's loss.backward)
 * The Python mirror of the reference's VecEnv surface (quadswarm_amd.vec_env.GpuQuadVecEnv) calls
 * these through ctypes; INTEGRATION.md shows the binding.
 *
 * Conventions: plain C types only; every call returns 0 on success or a negative QS_E* code and sets a
 * thread-local message readable with qs_last_error().  HIP errors are surfaced, never aborted on.
 * One handle = one HIP device; calls are asynchronous on the caller's stream (hipStream_t passed as
 * void*; NULL = the default stream) and a handle is not re-entrant.
 */
#ifndef QUADSWARM_H
#define QUADSWARM_H

#ifndef __HIPCC_RTC__
#include <stddef.h>
#include <stdint.h>
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define QS_ABI_VERSION 15
#define QS_MAX_AGENTS 128           /* drones per env: up to 64 inside one 64-lane wavefront, 128 = a two-wave
                                       workgroup per env (flavor B without obstacles; paper/fps_compare.py:7) */
#define QS_MAX_DR_CHOICES 8         /* entries per obstacle domain-randomisation list */

enum qs_status {
    QS_OK = 0,
    QS_E_INVALID = -1,              /* bad argument / config                          */
    QS_E_UNSUPPORTED = -2,          /* config outside what the kernels implement      */
    QS_E_HIP = -3,                  /* HIP runtime error (message has the HIP string) */
    QS_E_NOMEM = -4,
};

enum qs_flavor {
    QS_FLAVOR_B = 0,                   /* quadrotor_multi.QuadrotorEnvMulti: 4 raw motor commands    */
    QS_FLAVOR_A = 1,                   /* quadrotor_multi_rewards.QuadrotorEnvMulti: [heading rate, _] */
};

enum qs_obs_repr {                  /* quad_utils.py:30-38 (QUADS_OBS_REPR) */
    QS_OBS_XYZ_VXYZ_R_OMEGA = 0,       /* 18, flavor B */
    QS_OBS_XYZ_VXYZ_R_OMEGA_FLOOR = 1, /* 19, flavor B */
    QS_OBS_XYZ_VXYZ_R_OMEGA_WALL = 2,  /* 24, flavor B */
    QS_OBS_AW_AWDOT_DIST_DISTDOT_ANGLE_ANGLEDOT = 3,             /* 6, flavor A */
    QS_OBS_CDIST_CDISTDOT_DIST_DISTDOT_ANGLE_ANGLEDOT = 4,       /* 6, flavor A */
    QS_OBS_CDIST_CDISTDOT_DIST_DISTDOT_SANGLE_ANGLEDOT = 5,      /* 7, flavor A */
    QS_OBS_CDIST_CDISTDOT_NDIST_DISTDOT_NSANGLE_ANGLEDOT = 6,    /* 7, flavor A (camera model) */
};

enum qs_neighbor_obs {              /* quad_utils.py:40-58 (QUADS_NEIGHBOR_OBS_TYPE) */
    QS_NEIGHBOR_NONE = 0,
    QS_NEIGHBOR_POS_VEL = 1,           /* 6 per visible neighbour (both flavors) */
    QS_NEIGHBOR_DIST_ANGLE = 2,        /* 2, flavor A */
    QS_NEIGHBOR_DIST_SANGLE = 3,       /* 3, flavor A */
    QS_NEIGHBOR_NDIST_NSANGLE = 4,     /* 3, flavor A, camera model */
    QS_NEIGHBOR_DIST_ANGLE_HEADING = 5,    /* 3, flavor A */
    QS_NEIGHBOR_DIST_SANGLE_SHEADING = 6,  /* 5, flavor A */
    QS_NEIGHBOR_POS = 7,               /* 3, flavor A */
    QS_NEIGHBOR_NPOS = 8,              /* 3, flavor A (the reference discards its noise) */
};

enum qs_scenario {
    QS_SCEN_STATIC_SAME_GOAL = 0,      /* scenarios/static_same_goal.py (flavor A: spawn at the goal)  */
    QS_SCEN_DYNAMIC_REPULSIVE = 1,     /* scenarios/dynamic_repulsive.py, flavor A only (float-fixed)  */
    /* flavor B with obstacles (use_obstacles = 1): scenarios/mix.py over QUADS_MODE_LIST_OBSTACLES */
    QS_SCEN_OBST_MIX = 2,              /* o_random or o_static_same_goal, drawn per reset (mix.py:78-99) */
    QS_SCEN_O_RANDOM = 3,              /* scenarios/obstacles/o_random.py                              */
    QS_SCEN_O_STATIC_SAME_GOAL = 4,    /* scenarios/obstacles/o_static_same_goal.py                    */
    /* flavor B without obstacles: the goal scenarios of scenarios/ (one .py each), QUADS_MODE_LIST order + run_away */
    QS_SCEN_MIX = 5,                   /* one of the 9 below (5 for one drone) drawn per reset, mix.py  */
    QS_SCEN_STATIC_DIFF_GOAL = 6,      /* static_diff_goal.py                                          */
    QS_SCEN_EP_LISSAJOUS3D = 7,        /* ep_lissajous3D.py                                            */
    QS_SCEN_EP_RAND_BEZIER = 8,        /* ep_rand_bezier.py                                            */
    QS_SCEN_DYNAMIC_SAME_GOAL = 9,     /* dynamic_same_goal.py                                         */
    QS_SCEN_DYNAMIC_DIFF_GOAL = 10,    /* dynamic_diff_goal.py                                         */
    QS_SCEN_DYNAMIC_FORMATIONS = 11,   /* dynamic_formations.py                                        */
    QS_SCEN_SWAP_GOALS = 12,           /* swap_goals.py                                                */
    QS_SCEN_SWARM_VS_SWARM = 13,       /* swarm_vs_swarm.py                                            */
    QS_SCEN_RUN_AWAY = 14,             /* run_away.py                                                  */
    /* flavor B with obstacles: the maps' dynamic scenarios (QUADS_MODE_LIST_OBSTACLES_TEST, scenarios/utils.py:18-20;
     * the reference reaches them through create_scenario, scenarios/mix.py:24-36) -- ABI 14 */
    QS_SCEN_O_SWAP_GOALS = 15,         /* scenarios/obstacles/o_swap_goals.py                          */
    QS_SCEN_O_EP_RAND_BEZIER = 16,     /* scenarios/obstacles/o_ep_rand_bezier.py                      */
    QS_SCEN_O_DYNAMIC_SAME_GOAL = 17,  /* scenarios/obstacles/o_dynamic_same_goal.py                   */
};

/* Environment + physical configuration.  Physical constants are derived on the host exactly like
 * QuadrotorDynamics.update_model (quadrotor_dynamics.py:106-168); quadswarm_amd.params does it for
 * Python callers, qs_config_default() fills the Crazyflie values for C callers. */
typedef struct qs_config {
    int32_t abi_version;            /* must be QS_ABI_VERSION */
    int32_t num_envs;               /* E */
    int32_t num_agents;             /* N, 1..QS_MAX_AGENTS */
    int32_t obs_repr;               /* enum qs_obs_repr */
    int32_t neighbor_obs;           /* enum qs_neighbor_obs */
    int32_t k_neighbors;            /* visible neighbours (0..N-1); N-1 = all, no sorting */
    int32_t ep_len;                 /* int(ep_time / (dt * sim_steps)); done when tick > ep_len */
    int32_t sim_steps;              /* physics substeps per control tick (2) */
    int32_t svd_every;              /* substeps between polar re-orthonormalisations (100) */
    int32_t sense_noise;            /* 0: SensorNoise(bypass=True); 1: default noise */
    int32_t use_downwash;
    int32_t apply_collision_force;
    uint32_t seed;
    uint32_t drone_id_offset;       /* global id of drone 0 (RNG key): env shards on several GPUs draw
                                       exactly what one big env would (DESIGN.md multi-GPU) */
    float dt;                       /* 1 / sim_freq (0.005) */
    float control_dt;               /* dt * sim_steps (0.01) */
    /* rigid body */
    float mass, inertia[3];
    float thrust_max[4], torque_max[4], prop_cross[4][3], prop_ccw[4];
    float motor_tau_up, motor_tau_down, motor_linearity;
    float arm, gravity, omega_max, vel_damp, damp_omega_quadratic, vxyz_max;
    float room_lo[3], room_hi[3];
    /* noise */
    float ou_mu, ou_theta, ou_sigma;
    float pos_norm_std, pos_unif_range, vel_norm_std, vel_unif_range;
    float gyro_noise_density, quat_norm_std, quat_unif_range;
    /* rewards / collisions */
    float collision_threshold, collision_falloff_threshold;
    float rew_pos, rew_effort, rew_crash, rew_orient, rew_spin;
    float rew_quadcol_bin, rew_quadcol_smooth_max;
    /* static_same_goal scenario */
    float spawn_box, goal[3];
    /* ---- flavor A (ignored for flavor B) ---- */
    int32_t flavor;                 /* enum qs_flavor */
    int32_t scenario;               /* enum qs_scenario */
    int32_t ticks_per_step;         /* QuadrotorSingle._step calls per env step (8, :636) */
    int32_t n_cameras;              /* camera model (global_cfg.py:14-18) */
    float capture_radius;           /* initial_capture_radius (global_cfg.py:37); per env at run time */
    float cam_size, cam_focal, cam_px_noise, cam_fov_deg, cam_res;
    /* ---- obstacles (flavor B; quadrotor_multi.py:128-140, quad_obstacle_baseline.py) ---- */
    int32_t use_obstacles;
    int32_t num_obstacles;          /* int(obst_density * area^2), the pillars per env (C4: 12) */
    int32_t obst_area;              /* spawn area side in 1 m cells (8); area^2 <= 64 */
    float obst_size;                /* pillar diameter (0.6) */
    float sdf_resolution;           /* 0.1 (obstacles/obstacles.py:12) */
    float rew_quadcol_bin_obst;     /* quadcol_bin_obst reward coefficient */
    /* ---- obstacle domain randomisation: the experience-replay wrapper's reset draws one entry of each list
     * per new episode and hands it to env.reset (quad_experience_replay.py:76-87, 106-118, 206-214;
     * quadrotor_multi.py:440-450).  0 entries = off.  dr_counts[c] = int(area^2 * density_c) pillars, -1 for a
     * 0.0 density (falsy there: the env keeps its current value); dr_sizes[c] = pillar diameter, 0 = keep.
     * The env's current choice is part of its state (QS_E_OBST_M / QS_E_OBST_SZ), so replays restore it. */
    int32_t dr_num_counts;
    int32_t dr_counts[QS_MAX_DR_CHOICES];
    int32_t dr_num_sizes;
    float dr_sizes[QS_MAX_DR_CHOICES];
    /* ---- episode_extra_stats (flavor B; quadrotor_multi.py:153-216, 541-657, 739-831): 1 = the step kernels
     * keep the reference's per-episode counters and write each finished env's rows to buffers.estats ---- */
    int32_t episode_stats;
    /* ---- per-step infos (quadrotor_single.py:79-105, 371; quadrotor_multi.py:642-651; flavor A
     * quadrotor_single_rewards.py:457): 1 = every step writes each drone's reward components to
     * buffers.rew_info (QS_RI_*), from which the host builds infos[i]["rewards"] / infos[i]["goal_dist"] ---- */
    int32_t step_infos;
} qs_config;

/* Device buffers of a handle.  State is structure-of-arrays: field f of drone g lives at
 * state[f * I + g] with I = E * N (fp32), istate[f * I + g] (int32).  Observations are row-major
 * [I, obs_dim] fp32 so a torch tensor can consume them zero-copy. */
enum qs_state_field {
    QS_F_POS = 0, QS_F_VEL = 3, QS_F_ROT = 6, QS_F_OMEGA = 15, QS_F_ROT_DAMP = 18, QS_F_CMD_DAMP = 22,
    QS_F_OU = 26, QS_F_GOAL = 30,
    /* flavor A: Controller PIDs as (last_error, integral) pairs in the order position z, velocity
     * x y z, attitude x y z, rate x y z; heading angle and last heading-rate command; the
     * QuadrotorEnvMulti.heading value a reset sees (stale, like stale_vel) */
    QS_F_PID = 33, QS_F_ANGLE = 53, QS_F_ANGVEL = 54, QS_F_HEADING = 55,
    /* episode_extra_stats (flavor B): distance_to_goal[i] as its last 5 entries (dt * |goal - pos|, ring by
     * tick % 5) and its sums over the final 100 / 300 / 500 entries of the episode */
    QS_F_DRING = 56, QS_F_DSUM = 61,
    QS_NF = 64
};
/* QS_I_PREV_*: the drone's previous-collision row, bit j = partner j, 32 bits per word (PREV_2 / PREV_3 are
 * used by 128-drone envs only) */
enum qs_istate_field { QS_I_SVD = 0, QS_I_FLAGS = 1, QS_I_PREV_LO = 2, QS_I_PREV_HI = 3, QS_I_PREV_2 = 4, QS_I_PREV_3 = 5,
                       QS_NI = 6 };
enum qs_drone_flags {
    QS_FL_ON_FLOOR = 1, QS_FL_PREV_WALL = 2, QS_FL_PREV_CEIL = 4,
    QS_FL_CRASH_FLOOR = 8, QS_FL_CRASH_WALL = 16, QS_FL_CRASH_CEIL = 32,
    QS_FL_PREV_OBST = 64,           /* in prev_obst_quad_collisions (quadrotor_multi.py:585) */
    /* episode_extra_stats: in prev_crashed_room (:606); agent_col_agent / agent_col_obst cleared (:563, :589);
     * reached_goal (:652-655) */
    QS_FL_PREV_ROOM = 128, QS_FL_HIT_AGENT = 256, QS_FL_HIT_OBST = 512, QS_FL_REACHED = 1024
};
/* per env: tick, flags, episode.  {tick, episode} is the env's Philox counter: every step and reset
 * of an env draws a fresh stream.  Flavor A counts QuadrotorSingle ticks (8 per step). */
enum qs_env_field {
    QS_E_TICK = 0, QS_E_FLAGS = 1, QS_E_EPISODE = 2,
    /* flavor-B goal scenario of the env's episode (the reference's Scenario_* attributes): scenario
     * (QUADS_MODE_LIST index), formation (QUADS_FORMATION_LIST index), control_step_for_sec,
     * increase_formation_size */
    QS_E_SC_MODE = 3, QS_E_SC_FORM = 4, QS_E_SC_PERIOD = 5, QS_E_SC_INC = 6,
    /* obstacle domain randomisation: the env's pillar count / size as 1 + its list entry, 0 = configured */
    QS_E_OBST_M = 7, QS_E_OBST_SZ = 8,
    /* episode_extra_stats counters of the running episode (quadrotor_multi.py:153-171): collisions_per_episode,
     * collisions_room / floor / wall / ceiling_per_episode, collisions_after_settle, collisions_final_5s,
     * obst_quad_collisions_per_episode, obst_quad_collisions_after_settle, distance_to_goal_3_5, _5 */
    QS_E_ST_COL = 9, QS_E_ST_ROOM = 10, QS_E_ST_FLOOR = 11, QS_E_ST_WALL = 12, QS_E_ST_CEIL = 13,
    QS_E_ST_COL_SETTLE = 14, QS_E_ST_COL_FINAL = 15, QS_E_ST_OCOL = 16, QS_E_ST_OCOL_SETTLE = 17,
    QS_E_ST_O35 = 18, QS_E_ST_O5 = 19,
    QS_NE = 20
};
/* columns of a buffers.estats row (one per drone of a finished env, written by the step that ends the episode):
 * the env's counters, the agent rates, the scenario (QUADS_MODE_LIST index, 16 + mode for the obstacle
 * scenarios), the drone's own distance_to_goal_1s / 3s / 5s and whether the episode was a replay
 * (saved_in_replay_buffer).  quadswarm_amd.stats turns a row into the reference's dict. */
enum qs_estat {
    QS_ES_COL = 0, QS_ES_ROOM = 1, QS_ES_FLOOR = 2, QS_ES_WALL = 3, QS_ES_CEIL = 4, QS_ES_COL_SETTLE = 5,
    QS_ES_COL_FINAL = 6, QS_ES_OCOL = 7, QS_ES_OCOL_SETTLE = 8, QS_ES_O35 = 9, QS_ES_O5 = 10,
    QS_ES_SUCCESS = 11, QS_ES_DEADLOCK = 12, QS_ES_COLRATE = 13, QS_ES_NCOLRATE = 14, QS_ES_OCOLRATE = 15,
    QS_ES_SCEN = 16, QS_ES_D1 = 17, QS_ES_D3 = 18, QS_ES_D5 = 19, QS_ES_REPLAY = 20,
    QS_NES = 24
};
/* rows of buffers.rew_info [QS_NRI, I] (config step_infos), written by every step before a fused reset.  Flavor B:
 * compute_reward_weighted's raw terms (quadrotor_single.py:34-66) -- |goal - pos|, |action|, on_floor, the
 * orientation term (1 on the floor, else -R[2][2]), |omega| -- then the swarm terms (quadrotor_multi.py:608-651):
 * rew_collisions_raw (-1 for a drone in last_step_unique_collisions, else 0), the proximity reward
 * (-control_dt * penalty) and the obstacle raw term (-1 on a new pillar hit).  infos[i]["rewards"] is these times the
 * reward coefficients and dt (quadswarm_amd.infos).  Flavor A: row 0 = |pos - goal| after the last executed
 * tick (infos[i]["goal_dist"]). */
enum qs_rinfo {
    QS_RI_DIST = 0, QS_RI_EFFORT = 1, QS_RI_CRASH = 2, QS_RI_ORIENT = 3, QS_RI_SPIN = 4, QS_RI_QUADCOL = 5,
    QS_RI_PROX = 6, QS_RI_OBST = 7, QS_NRI = 8,
    QS_RI_GOAL_DIST = 0             /* flavor A */
};
enum qs_env_flags {
    QS_EF_STALE = 1,                /* stale_vel / QS_F_HEADING hold QuadrotorEnvMulti.vel / .heading */
    QS_EF_SUCCESS = 2,              /* flavor A episode_success (a capture happened this episode)     */
    QS_EF_HAS_POS = 4,              /* drones have been placed once (dynamic_repulsive.py:38 hasattr) */
    /* written by every flavor-B step, read by the replay kernel: */
    QS_EF_NEWCOL = 8,               /* last_step_unique_collisions.any() or curr_quad_col non-empty
                                       (quad_experience_replay.py:161-163) */
    QS_EF_FLOOR0 = 16,              /* drone 0 on the floor after the step (its rew_crash, quadrotor_multi.py:725) */
};
/* per env float state [QS_NENVF, E] (flavor A): target position of the dynamic_repulsive scenario and
 * the env's capture radius (set_capture_radius acts per env, custom_callbacks.py:455-462) */
enum qs_env_ffield {
    QS_ENVF_TARGET_X = 0, QS_ENVF_TARGET_Y = 1, QS_ENVF_CAPTURE = 2,
    /* flavor-B goal scenario: formation_size, lowest/highest_formation_size, layer_dist, control_speed,
     * formation_center xyz, ep_rand_bezier curve nodes (3 x xyz), swarm_vs_swarm goal centres (2 x xyz) */
    QS_ENVF_SC_SIZE = 3, QS_ENVF_SC_LO = 4, QS_ENVF_SC_HI = 5, QS_ENVF_SC_LAYER = 6, QS_ENVF_SC_SPEED = 7,
    QS_ENVF_SC_CENTER = 8, QS_ENVF_SC_BEZIER = 11, QS_ENVF_SC_C1 = 20, QS_ENVF_SC_C2 = 23,
    QS_NENVF = 26
};
/* The scenario floats (rows QS_ENVF_SC_SIZE .. QS_ENVF_SC_C2 + 2, QS_SC_NF of them) are stored ENV-MAJOR inside
 * their block (ABI 13): field k = row - QS_ENVF_SC_SIZE of env e at env_f[QS_ENVF_SC_SIZE * E + QS_SC_NF * e + k],
 * so that an env's record is one 92-byte run (the step kernel loads it with one instruction over the env's lanes:
 * 2-3 cache lines per wave instead of one per field).  The other env_f rows stay [row][E]. */
#define QS_SC_NF 23

typedef struct qs_layout {          /* byte offsets inside one workspace allocation */
    size_t params;                  /* kernel parameter block (device copy of the config + runtime params) */
    size_t state, istate, env, env_f, obst, stale_vel, obs, term_obs, rew, done, reset_info, stats, estats,
        rew_info, total_bytes;
    int32_t obs_dim, num_drones;
} qs_layout;

typedef struct qs_buffers {         /* device pointers (valid for the handle's lifetime) */
    float* state;                   /* [QS_NF, I] */
    int32_t* istate;                /* [QS_NI, I] */
    int32_t* env;                   /* [QS_NE, E] */
    float* env_f;                   /* [QS_NENVF, E] */
    float* obst;                    /* [E, M, 2] pillar xy (MultiObstacles.pos_arr order); M = num_obstacles, or
                                       the largest dr_counts entry (an env uses its first QS_E_OBST_M slots) */
    float* stale_vel;               /* [3, I]  QuadrotorEnvMulti.vel as last seen by a reset */
    float* obs;                     /* [I, obs_dim] */
    float* term_obs;                /* [I, obs_dim] rows of envs that finished this step */
    float* rew;                     /* [I] */
    uint8_t* done;                  /* [I] */
    uint8_t* reset_info;            /* [E] 0: no reset this call; 1: reset, {"success": False}; 2: True */
    uint64_t* stats;                /* [QS_NSTAT] non-finite guard counters (qs_counters)              */
    float* estats;                  /* [I, QS_NES] episode_extra_stats rows of the envs that finished (config
                                       episode_stats; rows of other envs keep their previous contents)   */
    float* rew_info;                /* [QS_NRI, I] the last step's reward components (config step_infos), or NULL */
} qs_buffers;

/* Non-finite guard.  The reference raises ValueError on a NaN reward (gym_art/quadrotor_multi/
 * quadrotor_single.py:87-90); a batched step cannot raise per env, so every step kernel counts what it
 * produced non-finite -- observation values written, rewards, drone states after the step (before a
 * fused reset replaces them) -- into device counters (one ballot per wave; atomics only on a hit).
 * The counters accumulate across launches (also inside captured graphs) until qs_counters_reset. */
enum qs_stat { QS_ST_OBS = 0, QS_ST_REW = 1, QS_ST_STATE = 2, QS_NSTAT = 4 };
typedef struct qs_stats {
    uint64_t nonfinite_obs;         /* observation values (obs rows of every step)                      */
    uint64_t nonfinite_rew;         /* rewards                                                          */
    uint64_t nonfinite_state;       /* drones whose pos / vel / rotation / omega was non-finite          */
    uint64_t reserved;
} qs_stats;

typedef struct qs_handle qs_handle;

int qs_abi_version(void);
const char* qs_last_error(void);
/* sizeof(qs_config), sizeof(qs_layout), sizeof(qs_buffers): lets FFI callers check struct mirrors. */
int qs_struct_sizes(size_t* config, size_t* layout, size_t* buffers);

/* Crazyflie + flavor-B defaults (values of quad_models.py:1-42 via QuadLink, SF quad_utils.py). */
int qs_config_default(qs_config* cfg, int32_t num_envs, int32_t num_agents);
/* Flavor-A defaults as swarm_rl/sb_train.py trains (global_cfg.py, sb_train.py:111-139): dynamic_repulsive,
 * cdist_cdistdot_dist_distdot_sangle_angledot, ndist_nsangle of all N-1 neighbours, pixel noise 0. */
int qs_config_default_a(qs_config* cfg, int32_t num_envs, int32_t num_agents);
int qs_layout_query(const qs_config* cfg, qs_layout* out);

/* d_workspace: NULL -> the library allocates (and frees) layout.total_bytes on hip_device;
 * otherwise caller-owned device memory of at least layout.total_bytes, 256-byte aligned. */
int qs_create(const qs_config* cfg, int hip_device, void* d_workspace, qs_handle** out);
int qs_destroy(qs_handle* h);
int qs_buffers_get(qs_handle* h, qs_buffers* out);

/* Reset the envs whose byte in d_env_mask[E] is non-zero (NULL = all); writes obs rows of those envs. */
int qs_reset(qs_handle* h, const uint8_t* d_env_mask, void* stream);
/* One control step for every env.  d_actions: flavor B [I, 4] fp32 raw policy output (clipped
 * inside, 16-byte aligned); flavor A [I, 2] fp32 (8-byte aligned, a[0] = heading rate, unclipped
 * like the reference).  Writes obs, rew, done; envs that finished (tick > ep_len, or a capture in
 * flavor A) are reset in the same launch, their final observation goes to term_obs, obs holds the
 * reset observation and reset_info[e] says so (SubprocVecEnvCustom semantics). */
int qs_step(qs_handle* h, const float* d_actions, void* stream);
/* `steps` back-to-back qs_step launches on `stream` with the same action buffer, from one C call (no
 * host language between the launches): the benchmark's launch loop, the eager equivalent of a captured
 * graph of `steps` steps.  Each launch is a whole step; the actions are the caller's buffer as it is
 * when each launch runs (a policy writing new actions orders itself on the same stream). */
int qs_step_n(qs_handle* h, const float* d_actions, int steps, void* stream);
/* qs_step of n handles (env blocks of one device, e.g. a GPU's shard split into blocks that overlap on
 * separate streams): handle i steps with d_actions[i] on streams[i].  One C call, one device check. */
int qs_step_blocks(qs_handle* const* hs, int n, const float* const* d_actions, void* const* streams);

/* Non-finite guard counters (qs_stats) accumulated since creation / the last qs_counters_reset.
 * qs_counters synchronises `stream` and copies them to the host; qs_counters_reset zeroes them
 * asynchronously on `stream`. */
int qs_counters(qs_handle* h, qs_stats* out, void* stream);
int qs_counters_reset(qs_handle* h, void* stream);

/* Runtime-tunable scalars: "rew_pos", "rew_effort", "rew_crash", "rew_orient", "rew_spin",
 * "quadcol_bin", "quadcol_bin_smooth_max", "quadcol_bin_obst", "ep_len", "seed", "capture_radius" (flavor A, all envs;
 * write buffers.env_f[QS_ENVF_CAPTURE * E + e] for one env). */
int qs_set_param(qs_handle* h, const char* key, double value);
int qs_get_param(qs_handle* h, const char* key, double* value);

/* Host snapshot of the whole env state (state, istate, env incl. RNG counters, env_f, stale_vel): bytes =
 * qs_state_bytes(); round-trips exactly through qs_set_state. Synchronises the stream. */
size_t qs_state_bytes(qs_handle* h);
int qs_get_state(qs_handle* h, void* host_dst, size_t bytes, void* stream);
int qs_set_state(qs_handle* h, const void* host_src, size_t bytes, void* stream);

/* Runtime specialisation: recompile this handle's step/reset kernels with hipRTC, its whole parameter
 * block baked in as constants (parameters qs_set_param can change stay live).  enable = 0 returns to the
 * generic kernels.  Results are the generic kernels' (tests/test_gpu_specialize.py).  Compiled modules
 * are cached per process.  No reference counterpart (the reference's numba JIT specialises on types only). */
int qs_specialize(qs_handle* h, int enable);
int qs_is_specialized(const qs_handle* h);
/* Host-only: compile a config's specialised kernels without a device (build check); returns the
 * code-object size in bytes or a negative error. */
long long qs_specialize_compile(const qs_config* cfg);

/* The kernel parameter block a config produces, as 32-bit words (host only, no device needed).
 * Returns the word count or a negative error. */
int qs_config_kp_words(const qs_config* cfg, uint32_t* out, size_t n_words);

/* ---- Experience replay on device: ExperienceReplayWrapper + ReplayBuffer
 *      (gym_art/quadrotor_multi/quad_experience_replay.py:16-216, applied by swarm_rl/env_wrappers/quad_utils.py:68-71
 *      when replay_buffer_sample_prob > 0; the reference's swarm runs use 0.75) and the env-side bookkeeping it
 *      reads (quadrotor_multi.py:182-185, 382-388, 461-465, 722-725).  Flavor B.
 * Per env: a ring of `keep` checkpoints (env snapshot + its obs) saved every cp_every ticks while the env is
 * active and not a replay; on a new drone/obstacle collision after the grace period the checkpoint
 * steps_ago back becomes an event of the env's buffer (bufsz slots, replaced round-robin once full); when an
 * episode ends the env restarts from a random event with probability sample_prob (events replayed max_replays
 * times are dropped).  Runs as a second kernel inside qs_step / qs_reset once enabled, on the same stream.
 * Draws: Philox stream S_REPLAY (25) keyed by drone 0 of the env at the env's new {tick, episode}: word 0 is
 * the sample_prob uniform, word 1 the event index.  A replayed env keeps its new episode counter, so its
 * noise draws are fresh (the reference's numba RNG is global, not part of the copied env). */
typedef struct qs_replay_config {
    float sample_prob;              /* replay_buffer_sample_prob */
    int32_t buffer_size;            /* ReplayBuffer buffer_size (20, :17)                                   */
    int32_t keep;                   /* max_episode_checkpoints_to_keep = int(3.0 / cp_step_size) (6, :88)   */
    int32_t steps_ago;              /* int(save_time_before_collision_sec / cp_step_size) (3, :170)         */
    int32_t cp_every;               /* cp_step_size_freq = 0.5 s * control_freq, in ticks (50, :20)         */
    int32_t grace_ticks;            /* collisions_grace_period_seconds * control_freq (150, :163)           */
    int32_t min_gap_ticks;          /* 5 * control_freq (500, :167)                                          */
    int32_t max_replays;            /* cleanup() keeps events replayed fewer times (10, :51)                 */
    int32_t hist_len;               /* crashes_in_recent_episodes maxlen (100, quadrotor_multi.py:184)      */
    int32_t hist_min;               /* can_drones_fly needs this many episodes (10, :387)                    */
} qs_replay_config;

/* per-env replay integers [QS_NR, E] */
enum qs_replay_field {
    QS_R_ACTIVE = 0,                /* activate_replay_buffer                       */
    QS_R_SAVED = 1,                 /* saved_in_replay_buffer                       */
    QS_R_CK_N = 2, QS_R_CK_HEAD = 3,    /* episode_checkpoints: length, next ring slot */
    QS_R_BUF_N = 4, QS_R_BUF_IDX = 5,   /* len(replay_buffer.buffer), buffer_idx       */
    QS_R_LAST_ADD = 6,              /* last_tick_added_to_buffer (-1e9 = none)      */
    QS_R_EPISODES = 7,              /* episode_counter                              */
    QS_R_REPLAYED = 8,              /* replayed_events                              */
    QS_R_INDEX_ERR = 9,             /* the reference's IndexError (:171-173), counted */
    QS_R_HIST_N = 10, QS_R_HIST_HEAD = 11,   /* crashes_in_recent_episodes ring       */
    QS_R_RESTORED = 12,             /* buffer slot restored by the last call, -1 = none */
    QS_R_PUSHED = 13,               /* buffer slot written by the last call, -1 = none  */
    QS_NR = 14
};

typedef struct qs_replay_buffers {  /* device pointers, valid while replay is enabled */
    int32_t* ri;                    /* [QS_NR, E]                                                    */
    double* crash;                  /* [E] crashes_last_episode                                       */
    double* hist;                   /* [hist_len, E] crashes_in_recent_episodes (ring)                */
    int32_t* perm;                  /* [buffer_size, E] deque position -> slot (positions >= BUF_N: free) */
    int32_t* nrep;                  /* [buffer_size, E] num_replayed per slot                          */
    uint32_t* store;                /* [E, keep + buffer_size, snap_words]: ring slots, then buffer slots */
    size_t snap_words;              /* words per snapshot: per drone (QS_NF + QS_NI + 3 + obs_dim) fields
                                       drone-minor, then env ints QS_NE, env floats QS_NENVF, obstacle xy
                                       2M, obs rows N x obs_dim */
} qs_replay_buffers;

/* The reference's values for a control period control_dt (quad_experience_replay.py:17-20, 88-92, 163-170). */
int qs_replay_config_default(qs_replay_config* rc, float control_dt);
/* Device bytes the replay state of this handle + config needs. */
int qs_replay_workspace_bytes(qs_handle* h, const qs_replay_config* rc, size_t* bytes);
/* Initialises the replay state in d_workspace (caller-owned device memory of qs_replay_workspace_bytes,
 * 256-byte aligned; NULL: the library allocates it).  Replay off again: qs_replay_disable or qs_destroy. */
int qs_replay_enable(qs_handle* h, const qs_replay_config* rc, void* d_workspace);
int qs_replay_disable(qs_handle* h);
int qs_replay_buffers_get(qs_handle* h, qs_replay_buffers* out);

/* Generalized advantage estimation over a device-resident rollout (replaces stable_baselines3
 * RolloutBuffer.compute_returns_and_advantage, the PPO of swarm_rl/sb_train.py:53-64).  Arrays are
 * [n_steps, n_cols] fp32 / u8, time-major; episode_starts[t] = done of step t-1; last_* = after the
 * final step.  Asynchronous on `stream`. */
int qs_gae(const float* d_rewards, const float* d_values, const uint8_t* d_episode_starts,
           const float* d_last_values, const uint8_t* d_last_dones, float* d_advantages, float* d_returns,
           int32_t n_steps, int32_t n_cols, float gamma, float gae_lambda, void* stream);

/* Fused no-grad forward of the rollout policy's attention neighbour encoder (replaces the torch evaluation of
 * QuadNeighborhoodEncoderAttention, swarm_rl/models/quad_multi_model.py:44-101, inside
 * ActorCriticPolicyCustomSeparateWeights.forward during SB3 collect_rollouts).  One tower = one encoder's
 * weights and buffers; up to QS_ATTN_MAX_TOWERS towers (actor, critic) per launch.  H (hidden size) is 128
 * or 256; K (neighbours per agent) 1..64; nd (features per neighbour) 1..16.  Every pointer is device
 * memory, fp32, row-major.  The [H, Kd] weights are passed PACKED for the matrix cores: packed[ct][g][l][u]
 * = W[32 ct + (l & 31)][(l >> 5) Kd/2 + 4 g + u] for ct < H/32, g < Kd/8, l < 64, u < 4
 * (quadswarm_amd.policy_fused.pack_mfma_weight).  Stage 1 (qs_attn_embed) writes e2 and e_mean; the caller
 * forms P = e_mean A_m^T + b_a1; stage 2 (qs_attn_pool) writes out.  Asynchronous on `stream`. */
#define QS_ATTN_MAX_TOWERS 2
typedef struct qs_attn_tower {
    /* stage 1: embedding_mlp */
    const float* w_e1p;    /* packed [H, 32]: [embedding_mlp[0].weight[:, so:] (nd) | [:, :so] (so) | 0] */
    const float* b_e1;     /* [H] */
    const float* w_e2p;    /* packed embedding_mlp[2].weight */
    const float* b_e2;     /* [H] */
    float* e2;             /* [B*K, H] out: embeddings e_i (row j = agent j / K, neighbour j % K) */
    float* e_mean;         /* [B, H] out: mean over the agent's K rows */
    /* stage 2: neighbor_value_mlp + attention_mlp + softmax pooling */
    const float* P;        /* [B, H] e_mean @ W_a1[:, H:]^T + b_a1 */
    const float* w_v1p;    /* packed neighbor_value_mlp[0].weight */
    const float* b_v1;
    const float* w_v2p;    /* packed neighbor_value_mlp[2].weight */
    const float* b_v2;
    const float* w_a1ep;   /* packed attention_mlp[0].weight[:, :H] */
    const float* w_a2p;    /* packed attention_mlp[2].weight */
    const float* b_a2;
    const float* w_a3;     /* [H] attention_mlp[4].weight */
    float b_a3;            /* attention_mlp[4].bias */
    float* out;            /* [B, H] out: the attention-weighted value embedding per agent */
} qs_attn_tower;
/* obs: [B, obs_stride] rows; agent b's self features are obs[b * obs_stride + 0 .. self_dim), its neighbour
 * block obs[b * obs_stride + nbr_off ...], K x nd; nd + self_dim <= 32. */
int qs_attn_embed(const float* d_obs, int32_t obs_stride, int32_t self_dim, int32_t nbr_off, int32_t B, int32_t K,
                  int32_t nd, int32_t H, const qs_attn_tower* towers, int32_t n_towers, void* stream);
int qs_attn_pool(int32_t B, int32_t K, int32_t H, const qs_attn_tower* towers, int32_t n_towers, void* stream);
/* The same two stages with every fp32 product of the contractions split over the f16 matrix cores (ABI 11):
 * x = (hi + lo) / s with hi = f16(s x), lo = f16(s x - hi), and x w = (hi_x hi_w + hi_x lo_w + lo_x hi_w) / (s_x s_w)
 * accumulated in fp32 (per-product error ~7e-7 relative; biases, tanh, softmax, pooling fp32).  The towers' w_*p then
 * point to weights packed for v_mfma_f32_32x32x16_f16 (quadswarm_amd.policy_fused.pack_mfma_weight_x3): per
 * 32-column tile ct, 16-deep step s and lane l, 8 f16 of hi(256 W[32 ct + (l & 31)][16 s + 8 (l >> 5) + j]) then
 * the 8 matching lo halves; every other pointer as above. */
int qs_attn_embed_x3(const float* d_obs, int32_t obs_stride, int32_t self_dim, int32_t nbr_off, int32_t B, int32_t K,
                     int32_t nd, int32_t H, const qs_attn_tower* towers, int32_t n_towers, void* stream);
int qs_attn_pool_x3(int32_t B, int32_t K, int32_t H, const qs_attn_tower* towers, int32_t n_towers, void* stream);

/* The PPO update's attention encoder (ABI 12; SURVEY §8 f4, the update side; qs_policy_train.h): the x3 forward with
 * the activations the backward needs saved, and the backward's two row-block chains.  Per tower, next to its
 * qs_attn_tower (x3-packed weights, e2 / e_mean / P / out as for qs_attn_embed_x3 / qs_attn_pool_x3), fp32 [B*K, H]
 * unless noted (row j = agent j / K, neighbour j % K). */
typedef struct qs_attn_train {
    float* e1; float* a1; float* a2; float* v1; float* h;   /* forward: the tanh outputs (embedding 0, attention 0/2,
                                                               value 0/2) */
    float* w;              /* forward: [B*K] the softmax weights */
    const float* dout;     /* backward 1: [B, H] dL/d out */
    const float* dem;      /* backward 2: [B, H] dL/d e_mean = (sum over rows j % B = b of da1_pre_j) A_m */
    const void* w_v2tp; const void* w_v1tp; const void* w_a2tp; const void* w_a1etp; const void* w_e2tp;
                           /* x3-packed TRANSPOSED weights: W_v2^T, W_v1^T, W_a2^T, attention_mlp[0].weight[:, :H]^T, W_e2^T */
    float* dh_pre; float* dv1_pre; float* da2_pre; float* da1_pre;   /* backward 1 outputs: pre-activation gradients */
    float* dscore;         /* backward 1: [B*K] dL/d score */
    float* de2p;           /* backward 1: dL/d e2 without the e_mean term */
    float* de2_pre; float* de1_pre;                                  /* backward 2 outputs */
    /* ABI 15 (both may be NULL: not written): the gradients' column statistics, formed where the gradients are, per
     * row block of the kernels (n_blocks = ceil(B K / (floor(64 / K) K)), block b = rows [b m, (b + 1) m), m =
     * floor(64 / K) K):
     * colmax: [QS_ATTN_NCOLMAX][n_blocks][H] max |g| over the block's rows per column (+inf when a g is not finite)
     *   of dh_pre, dv1_pre, da2_pre, da1_pre (backward 1), de2_pre and de1_pre (backward 2) -- their max over the
     *   blocks gives dW's column scales (qs_attn_dw_x3 / qs_attn_dw0_x3 col_scale);
     * a3w_part: [n_blocks][H] the block's sum of dscore_j a2_j (the score layer's weight gradient is the sum over
     *   the blocks). */
    float* colmax;
    float* a3w_part;
} qs_attn_train;
#define QS_ATTN_NCOLMAX 6   /* colmax rows: 0 dh_pre, 1 dv1_pre, 2 da2_pre, 3 da1_pre, 4 de2_pre, 5 de1_pre */
int qs_attn_embed_train_x3(const float* d_obs, int32_t obs_stride, int32_t self_dim, int32_t nbr_off, int32_t B, int32_t K,
                           int32_t nd, int32_t H, const qs_attn_tower* towers, const qs_attn_train* trains,
                           int32_t n_towers, void* stream);
int qs_attn_pool_train_x3(int32_t B, int32_t K, int32_t H, const qs_attn_tower* towers, const qs_attn_train* trains,
                          int32_t n_towers, void* stream);
int qs_attn_bwd1_x3(int32_t B, int32_t K, int32_t H, const qs_attn_tower* towers, const qs_attn_train* trains,
                    int32_t n_towers, void* stream);
int qs_attn_bwd2_x3(int32_t B, int32_t K, int32_t H, const qs_attn_tower* towers, const qs_attn_train* trains,
                    int32_t n_towers, void* stream);
/* A weight gradient G^T A over R rows on the split-f16 matrix cores, split over n_parts row ranges:
 * part[p] = G[rows of p]^T A[rows of p] ([n_parts, H, H] fp32; dW = the sum over p).  G [R, H] (pre-activation
 * gradients) with a power-of-two scale per column, col_scale[n] |G[:, n]| < 2^14; A [R, H] with |A| <= 1 (tanh).
 * part_sum (ABI 15; NULL: not written): [n_parts, H] the column sums of G over each part's rows (the bias gradient
 * is their sum over p) from the same pass. */
int qs_attn_dw_x3(const float* G, const float* A, const float* col_scale, int64_t R, int32_t H, float* part,
                  float* part_sum, int32_t n_parts, void* stream);
/* qs_attn_dw_x3 on column slices of wider rows (ABI 15): row strides ldg / lda (floats, H .. 4096) -- e.g. the 256 x
 * 256 blocks of the feed_forward's [512, 512] weight gradient. */
int qs_dw_x3_ld(const float* G, int32_t ldg, const float* A, int32_t lda, const float* col_scale, int64_t R, int32_t H,
                float* part, float* part_sum, int32_t n_parts, void* stream);
/* The encoder's feed_forward on the split-f16 matrix cores (ABI 15; quad_multi_model.py QuadMultiEncoder
 * feed_forward = Linear + Tanh): Y [M, N] = tanh(X W^T + bias) for X [M, K] fp32 with |x| <= 1 (tanh outputs), K 256
 * or 512, N a multiple of 256 (<= 1024); w_packed: for each 256-row block z of W and 256-column slice p (z-major), the
 * pack of W[256 z .., 256 p ..] as the attention weights are packed (qs_attn_tower); w_bytes its size (checked:
 * (N / 256) (K / 256) 262 144 bytes). */
int qs_linear_tanh_x3(const float* X, int64_t M, int32_t K, const void* w_packed, int64_t w_bytes, const float* bias,
                      float* Y, int32_t N, void* stream);
/* qs_linear_tanh_x3 with K = 512 on the concatenation [X0 | X1] of two [M, 256] row-major tensors (ABI 15; the
 * feed_forward's input torch.cat((embeddings, neighborhood_embedding), 1), quad_multi_model.py:342, without
 * forming it); w_packed / w_bytes as qs_linear_tanh_x3 for W [N, 512]. */
int qs_linear_tanh_cat_x3(const float* X0, const float* X1, int64_t M, const void* w_packed, int64_t w_bytes,
                          const float* bias, float* Y, int32_t N, void* stream);
/* Y [M, N] = X W^T for rows X [M, K] of any magnitude (ABI 15; the feed_forward's backward dX = G W with the packed
 * W^T): row r staged at its power-of-two scale row_scale[r] (max |X[r, :]| row_scale[r] < 2^14 -- the
 * qs_attn_dw_x3 column-scale rule applied to rows), no bias, no activation; K, N, w_packed / w_bytes as
 * qs_linear_tanh_x3. */
int qs_linear_rows_x3(const float* X, const float* row_scale, int64_t M, int32_t K, const void* w_packed, int64_t w_bytes,
                      float* Y, int32_t N, void* stream);
/* Y [M, N] = X W^T + bias for X [M, K] fp32 with |x| <= 1 on the split-f16 matrix cores (ABI 15; the attention
 * score layer's mean half P = e_mean A_m^T + b_a1, quad_multi_model.py:90-93 -- attention_mlp[0] on the repeated
 * neighbour-embedding mean): qs_linear_tanh_x3 without the tanh; K, N, w_packed / w_bytes as qs_linear_tanh_x3. */
int qs_linear_bias_x3(const float* X, int64_t M, int32_t K, const void* w_packed, int64_t w_bytes, const float* bias,
                      float* Y, int32_t N, void* stream);
/* out [M, N] = sum_{s < n_slabs} G[s M + m, :] for G [n_slabs M, N] (ABI 15; the backward's dP[b] = sum_k
 * da1_pre[k B + b] of the repeat tiling, quad_multi_model.py:90-92), with out's row scales (row_scale [M]) and per
 * 64-row block column maxima (col_part [ceil(M / 64)][N]) as qs_tanh_grad_stats; N 256 or 512. */
int qs_slab_sum_stats(const float* G, int32_t n_slabs, int64_t M, int32_t N, float* out, float* row_scale,
                      float* col_part, void* stream);
/* tanh backward with its x3 statistics (ABI 15): gp = g (1 - y^2) for [M, N] rows (N 256 or 512), row_scale [M] the
 * power-of-two scale of each gp row (qs_linear_rows_x3's), col_part [ceil(M / 64)][N] per 64-row block column maxima
 * of |gp| (qs_colmax_reduce -> qs_dw_x3_ld's column scales); +inf marks a non-finite value. */
int qs_tanh_grad_stats(const float* g, const float* y, float* gp, float* row_scale, float* col_part, int64_t M, int32_t N,
                       void* stream);
/* The maxima over the blocks of per-block column maxima (ABI 15; qs_attn_train.colmax rows): out[s][n] =
 * max_b part_max[s][b][n] for s < n_stats (entries >= 0, +inf propagates), part_max [n_stats][n_blocks][H]. */
int qs_colmax_reduce(const float* part_max, int32_t n_stats, int32_t n_blocks, int32_t H, float* out, void* stream);
/* Layer 0's weight gradient (ABI 15): part[p] = G[rows of p]^T X[rows of p] ([n_parts, H, 32] fp32; the sum over p
 * is the gradient of embedding layer 0's weight in the kernels' column order [neighbour (nd) | self (self_dim) | 0])
 * with X the layer-0 input rows the forward gathers (row r = agent r / K, neighbour r % K of that agent's block at
 * nbr_off, self features of agent r % B -- the reference's repeat pairing, quad_multi_model.py:44-101), G = de1_pre
 * [B K, H] with col_scale as qs_attn_dw_x3, |obs| < 4094 (the forward's split-f16 range); part_sum (NULL: not
 * written): [n_parts, H] G's column sums (the bias gradient's parts).  nd + self_dim <= 32; nd = 0 with K = 1: the self
 * features alone (the self encoder's first layer, rows = agents). */
int qs_attn_dw0_x3(const float* G, const float* col_scale, const float* d_obs, int32_t obs_stride, int32_t self_dim,
                   int32_t nbr_off, int32_t B, int32_t K, int32_t nd, int32_t H, float* part, float* part_sum,
                   int32_t n_parts, void* stream);
/* Column reductions of a gradient G [R, H] in one pass over its rows (ABI 13; the update's bias gradients, the dW
 * column scales and layer 0's weight gradient, in place of torch's abs / amax / sum / skinny-GEMM passes), split
 * over n_parts row ranges, per part p and column n:
 *   part_max[p, n] = max |G[r, n]| (NaN / inf propagate), part_sum[p, n] = sum w[r] G[r, n] (row_w = w, or
 *   NULL for w = 1: with row_w the dscore of the attention rows and G = a2 it is the score layer's weight gradient),
 *   part_x[p, c, n] = sum G[r, n] X(r, c) for c < nx (nx <= QS_COLSTATS_MAX_X; part_x may be NULL when nx = 0) with
 *   the layer-0 input of row r = k B + b of the attention encoder's repeat tiling (quad_multi_model.py:44-101):
 *   X(r, c) = obs[(r / K) * obs_stride + nbr_off + (r % K) * nd + c] for c < nd (neighbour k of row r / K, the
 *   reshape of the neighbour block), obs[(r % B) * obs_stride + c - nd] for nd <= c < nx (self.repeat(K, 1)).
 * H is 128 or 256. */
#define QS_COLSTATS_MAX_X 32
int qs_colstats(const float* G, int64_t R, int32_t H, const float* row_w, const float* d_obs, int32_t obs_stride,
                int32_t nbr_off, int32_t B, int32_t K, int32_t nd, int32_t nx, float* part_max, float* part_sum,
                float* part_x, int32_t n_parts, void* stream);

/* sb_train's capture-radius curriculum on the device (ABI 11; replaces CurriculumCallback._on_step,
 * swarm_rl/custom_callbacks.py:441-468, which SB3 runs after every VecEnv step).  Flavor A.  The callback's state
 * is a qs_curriculum in DEVICE memory; qs_curriculum_step, enqueued after a qs_step, records the outcome of every
 * env that step reset (buffers.reset_info, env order) into the window, re-evaluates the success rate when any env
 * was reset and, when it exceeds sr_threshold, multiplies the radius by decay, writes it to every env's
 * env_f[QS_ENVF_CAPTURE] row (set_capture_radius) and clears the window.  Nothing is read back: the host copies
 * the struct when it wants to log or checkpoint (n_shrinks / history name the reference's curriculum
 * checkpoints).  fp64 arithmetic like the reference's numpy / Python floats. */
#define QS_CUR_MAX_WINDOW 64
#define QS_CUR_MAX_HIST 64
typedef struct qs_curriculum {
    double radius;                  /* current_capture_radius (initial_capture_radius at the start)      */
    double success_rate;            /* sucess_rate: the window mean at the last step that reset an env    */
    double sr_threshold;            /* cfg.capture_radius_sr                                              */
    double decay;                   /* cfg.capture_radius_decay                                           */
    int64_t window_i;               /* window_i: outcomes recorded so far                                 */
    int32_t window;                 /* window_size (40 in the reference), 1..QS_CUR_MAX_WINDOW            */
    int32_t n_shrinks;              /* radius reductions so far                                           */
    double past[QS_CUR_MAX_WINDOW]; /* past_successes (first `window` entries)                            */
    double history[QS_CUR_MAX_HIST];/* radius after reduction k, at k % QS_CUR_MAX_HIST                   */
} qs_curriculum;
/* Fill a host struct with the reference's initial values (window cleared); copy it to device memory yourself. */
int qs_curriculum_init(qs_curriculum* host, double initial_radius, double sr_threshold, double decay, int32_t window);
/* One curriculum update for the step just enqueued on `stream` (d_cur: device qs_curriculum). */
int qs_curriculum_step(qs_handle* h, qs_curriculum* d_cur, void* stream);
/* The same update over the reset outcomes of ALL data-parallel ranks (ABI 12; SURVEY §8e, custom_callbacks.py:452-462
 * iterating the whole VecEnv's reset_infos): d_reset_all holds n_all = world * num_envs reset_info bytes in global env
 * order (rank r's handle owns envs [r * num_envs, (r + 1) * num_envs), e.g. an all-gather of every rank's
 * buffers.reset_info); every rank runs it with the same bytes, so every rank's d_cur evolves identically, and the
 * new radius is written to THIS handle's envs. */
int qs_curriculum_step_all(qs_handle* h, const uint8_t* d_reset_all, int64_t n_all, qs_curriculum* d_cur, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* QUADSWARM_H */
