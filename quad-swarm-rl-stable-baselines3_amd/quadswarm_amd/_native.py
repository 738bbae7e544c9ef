"""ctypes binding of libquadswarm.so (include/quadswarm.h).

The HIP library is the only implementation of the step: if it is missing or cannot be loaded this
module raises instead of falling back to anything else.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("QUADSWARM_LIB", os.path.join(HERE, "lib", "libquadswarm.so"))

ABI_VERSION = 15
MAX_AGENTS = 128
A_KMAX = 16   # flavor A, more than 64 drones: visible neighbours (qs_flavor_a.h QS_A_KMAX)
MAX_DR_CHOICES = 8
F, I32, U32, U64, SZ = ctypes.c_float, ctypes.c_int32, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_size_t

# enum values (quadswarm.h)
FLAVOR_B, FLAVOR_A = 0, 1
OBS_REPR = {"xyz_vxyz_R_omega": 0, "xyz_vxyz_R_omega_floor": 1, "xyz_vxyz_R_omega_wall": 2,
            "aw_awdot_dist_distdot_angle_angledot": 3, "cdist_cdistdot_dist_distdot_angle_angledot": 4,
            "cdist_cdistdot_dist_distdot_sangle_angledot": 5, "cdist_cdistdot_ndist_distdot_nsangle_angledot": 6}
OBS_REPR_B = (0, 1, 2)
OBS_REPR_A = (3, 4, 5, 6)
SELF_OBS_DIM = {0: 18, 1: 19, 2: 24, 3: 6, 4: 6, 5: 7, 6: 7}
NEIGHBOR_NONE, NEIGHBOR_POS_VEL = 0, 1
NEIGHBOR = {"none": 0, "pos_vel": 1, "dist_angle": 2, "dist_sangle": 3, "ndist_nsangle": 4, "dist_angle_heading": 5,
            "dist_sangle_sheading": 6, "pos": 7, "npos": 8}
NEIGHBOR_DIM = {0: 0, 1: 6, 2: 2, 3: 3, 4: 3, 5: 3, 6: 5, 7: 3, 8: 3}
SCENARIO = {"static_same_goal": 0, "dynamic_repulsive": 1, "obst_mix": 2, "o_random": 3, "o_static_same_goal": 4,
            "o_swap_goals": 15, "o_ep_rand_bezier": 16, "o_dynamic_same_goal": 17}
# flavor B with obstacles: quads_mode -> qs_scenario (scenarios/obstacles/; the dynamic three: ABI 14)
SCENARIO_OBST = {"mix": 2, "o_random": 3, "o_static_same_goal": 4, "o_swap_goals": 15, "o_ep_rand_bezier": 16,
                 "o_dynamic_same_goal": 17}
# flavor B without obstacles: quads_mode -> qs_scenario (the goal scenarios of gym_art/quadrotor_multi/scenarios/)
SCENARIO_B = {"static_same_goal": 0, "mix": 5, "static_diff_goal": 6, "ep_lissajous3D": 7, "ep_rand_bezier": 8,
              "dynamic_same_goal": 9, "dynamic_diff_goal": 10, "dynamic_formations": 11, "swap_goals": 12,
              "swarm_vs_swarm": 13, "run_away": 14}
F_POS, F_VEL, F_ROT, F_OMEGA, F_ROT_DAMP, F_CMD_DAMP, F_OU, F_GOAL = 0, 3, 6, 15, 18, 22, 26, 30
F_PID, F_ANGLE, F_ANGVEL, F_HEADING = 33, 53, 54, 55
F_DRING, F_DSUM, NF = 56, 61, 64
I_SVD, I_FLAGS, I_PREV_LO, I_PREV_HI, I_PREV_2, I_PREV_3, NI = 0, 1, 2, 3, 4, 5, 6   # rows 4, 5: 128-drone envs
FL_ON_FLOOR, FL_PREV_WALL, FL_PREV_CEIL, FL_CRASH_FLOOR, FL_CRASH_WALL, FL_CRASH_CEIL = 1, 2, 4, 8, 16, 32
FL_PREV_OBST = 64
FL_PREV_ROOM, FL_HIT_AGENT, FL_HIT_OBST, FL_REACHED = 128, 256, 512, 1024
E_TICK, E_FLAGS, E_EPISODE = 0, 1, 2
E_SC_MODE, E_SC_FORM, E_SC_PERIOD, E_SC_INC = 3, 4, 5, 6
E_OBST_M, E_OBST_SZ = 7, 8
E_ST_COL, NE_ST, NE = 9, 11, 20     # episode_extra_stats counters QS_E_ST_COL .. QS_E_ST_O5
EF_STALE, EF_SUCCESS, EF_HAS_POS, EF_NEWCOL, EF_FLOOR0 = 1, 2, 4, 8, 16
ENVF_TARGET_X, ENVF_TARGET_Y, ENVF_CAPTURE = 0, 1, 2
ENVF_SC_SIZE, ENVF_SC_LO, ENVF_SC_HI, ENVF_SC_LAYER, ENVF_SC_SPEED = 3, 4, 5, 6, 7
ENVF_SC_CENTER, ENVF_SC_BEZIER, ENVF_SC_C1, ENVF_SC_C2, NENVF = 8, 11, 20, 23, 26
SC_NF = 23   # the scenario floats ENVF_SC_SIZE .. ENVF_SC_C2 + 2, stored env-major inside their block (QS_SC_NF)


def env_f_rows(env_f):
    """A numpy copy of an env_f array [NENVF, E] with the env-major scenario block as [row][E] rows like the others
    (row ENVF_SC_SIZE + k = scenario float k of every env)."""
    E = env_f.shape[1]
    out = env_f.copy()
    out[ENVF_SC_SIZE:ENVF_SC_SIZE + SC_NF] = env_f[ENVF_SC_SIZE:ENVF_SC_SIZE + SC_NF].reshape(E, SC_NF).T
    return out


def env_f_from_rows(rows):
    """The inverse of env_f_rows: [row][E] scenario rows back into the device's env-major block (numpy)."""
    E = rows.shape[1]
    out = rows.copy()
    out[ENVF_SC_SIZE:ENVF_SC_SIZE + SC_NF] = rows[ENVF_SC_SIZE:ENVF_SC_SIZE + SC_NF].T.reshape(SC_NF, E)
    return out


class QsConfig(ctypes.Structure):
    _fields_ = [
        ("abi_version", I32), ("num_envs", I32), ("num_agents", I32), ("obs_repr", I32), ("neighbor_obs", I32),
        ("k_neighbors", I32), ("ep_len", I32), ("sim_steps", I32), ("svd_every", I32), ("sense_noise", I32),
        ("use_downwash", I32), ("apply_collision_force", I32), ("seed", U32), ("drone_id_offset", U32),
        ("dt", F), ("control_dt", F),
        ("mass", F), ("inertia", F * 3),
        ("thrust_max", F * 4), ("torque_max", F * 4), ("prop_cross", (F * 3) * 4), ("prop_ccw", F * 4),
        ("motor_tau_up", F), ("motor_tau_down", F), ("motor_linearity", F),
        ("arm", F), ("gravity", F), ("omega_max", F), ("vel_damp", F), ("damp_omega_quadratic", F), ("vxyz_max", F),
        ("room_lo", F * 3), ("room_hi", F * 3),
        ("ou_mu", F), ("ou_theta", F), ("ou_sigma", F),
        ("pos_norm_std", F), ("pos_unif_range", F), ("vel_norm_std", F), ("vel_unif_range", F),
        ("gyro_noise_density", F), ("quat_norm_std", F), ("quat_unif_range", F),
        ("collision_threshold", F), ("collision_falloff_threshold", F),
        ("rew_pos", F), ("rew_effort", F), ("rew_crash", F), ("rew_orient", F), ("rew_spin", F),
        ("rew_quadcol_bin", F), ("rew_quadcol_smooth_max", F),
        ("spawn_box", F), ("goal", F * 3),
        ("flavor", I32), ("scenario", I32), ("ticks_per_step", I32), ("n_cameras", I32),
        ("capture_radius", F), ("cam_size", F), ("cam_focal", F), ("cam_px_noise", F), ("cam_fov_deg", F), ("cam_res", F),
        ("use_obstacles", I32), ("num_obstacles", I32), ("obst_area", I32), ("obst_size", F), ("sdf_resolution", F),
        ("rew_quadcol_bin_obst", F),
        ("dr_num_counts", I32), ("dr_counts", I32 * MAX_DR_CHOICES), ("dr_num_sizes", I32),
        ("dr_sizes", F * MAX_DR_CHOICES),
        ("episode_stats", I32),
        ("step_infos", I32),
    ]


class QsLayout(ctypes.Structure):
    _fields_ = [("params", SZ), ("state", SZ), ("istate", SZ), ("env", SZ), ("env_f", SZ), ("obst", SZ), ("stale_vel", SZ),
                ("obs", SZ),
                ("term_obs", SZ), ("rew", SZ), ("done", SZ), ("reset_info", SZ), ("stats", SZ), ("estats", SZ),
                ("rew_info", SZ), ("total_bytes", SZ),
                ("obs_dim", I32),
                ("num_drones", I32)]


class QsBuffers(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("state", "istate", "env", "env_f", "obst", "stale_vel", "obs", "term_obs",
                                               "rew", "done", "reset_info", "stats", "estats", "rew_info")]


# per-step reward components, rows of buffers.rew_info (qs_rinfo)
RI_DIST, RI_EFFORT, RI_CRASH, RI_ORIENT, RI_SPIN, RI_QUADCOL, RI_PROX, RI_OBST, NRI = range(9)
RI_GOAL_DIST = 0   # flavor A

# non-finite guard counters (qs_stat / qs_stats)
ST_OBS, ST_REW, ST_STATE, NSTAT = 0, 1, 2, 4


class QsStats(ctypes.Structure):
    _fields_ = [("nonfinite_obs", U64), ("nonfinite_rew", U64), ("nonfinite_state", U64), ("reserved", U64)]


class QsReplayConfig(ctypes.Structure):
    _fields_ = [("sample_prob", F), ("buffer_size", I32), ("keep", I32), ("steps_ago", I32), ("cp_every", I32),
                ("grace_ticks", I32), ("min_gap_ticks", I32), ("max_replays", I32), ("hist_len", I32), ("hist_min", I32)]


class QsReplayBuffers(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("ri", "crash", "hist", "perm", "nrep", "store")] + [("snap_words", SZ)]


# qs_replay_field
R_ACTIVE, R_SAVED, R_CK_N, R_CK_HEAD, R_BUF_N, R_BUF_IDX, R_LAST_ADD, R_EPISODES, R_REPLAYED, R_INDEX_ERR = range(10)
R_HIST_N, R_HIST_HEAD, R_RESTORED, R_PUSHED, NR = 10, 11, 12, 13, 14


ATTN_MAX_TOWERS = 2
ATTN_NCOLMAX = 6          # qs_attn_train.colmax rows (QS_ATTN_NCOLMAX)


class QsAttnTower(ctypes.Structure):
    """qs_attn_tower (device pointers of one attention-encoder tower, quadswarm.h)."""
    _fields_ = [(n, ctypes.c_void_p) for n in ("w_e1p", "b_e1", "w_e2p", "b_e2", "e2", "e_mean", "P", "w_v1p", "b_v1",
                                                "w_v2p", "b_v2", "w_a1ep", "w_a2p", "b_a2", "w_a3")] + \
               [("b_a3", F), ("out", ctypes.c_void_p)]


class QsAttnTrain(ctypes.Structure):
    """qs_attn_train (the PPO update's saved activations and gradients of one tower, quadswarm.h)."""
    _fields_ = [(n, ctypes.c_void_p) for n in ("e1", "a1", "a2", "v1", "h", "w", "dout", "dem", "w_v2tp", "w_v1tp",
                                                "w_a2tp", "w_a1etp", "w_e2tp", "dh_pre", "dv1_pre", "da2_pre", "da1_pre",
                                                "dscore", "de2p", "de2_pre", "de1_pre", "colmax", "a3w_part")]


CUR_MAX_WINDOW = CUR_MAX_HIST = 64


class QsCurriculum(ctypes.Structure):
    """qs_curriculum (the device-side CurriculumCallback state, quadswarm.h)."""
    _fields_ = [("radius", ctypes.c_double), ("success_rate", ctypes.c_double), ("sr_threshold", ctypes.c_double),
                ("decay", ctypes.c_double), ("window_i", ctypes.c_int64), ("window", I32), ("n_shrinks", I32),
                ("past", ctypes.c_double * CUR_MAX_WINDOW), ("history", ctypes.c_double * CUR_MAX_HIST)]


class QuadSwarmError(RuntimeError):
    pass


# every symbol include/quadswarm.h declares (tests check the library exports all of them)
EXPORTS = ["qs_abi_version", "qs_last_error", "qs_struct_sizes", "qs_config_default", "qs_config_default_a",
           "qs_layout_query", "qs_create", "qs_destroy",
           "qs_buffers_get", "qs_reset", "qs_step", "qs_step_n", "qs_step_blocks", "qs_counters", "qs_counters_reset",
           "qs_set_param",
           "qs_get_param", "qs_state_bytes", "qs_get_state", "qs_set_state", "qs_gae",
           "qs_specialize", "qs_is_specialized", "qs_config_kp_words", "qs_specialize_compile",
           "qs_replay_config_default", "qs_replay_workspace_bytes", "qs_replay_enable", "qs_replay_disable", "qs_replay_buffers_get",
           "qs_attn_embed", "qs_attn_pool", "qs_attn_embed_x3", "qs_attn_pool_x3", "qs_curriculum_init",
           "qs_curriculum_step", "qs_curriculum_step_all", "qs_attn_embed_train_x3", "qs_attn_pool_train_x3",
           "qs_attn_bwd1_x3", "qs_attn_bwd2_x3", "qs_attn_dw_x3", "qs_attn_dw0_x3", "qs_colmax_reduce", "qs_colstats",
           "qs_linear_tanh_x3", "qs_dw_x3_ld", "qs_linear_rows_x3",
           "qs_tanh_grad_stats", "qs_linear_bias_x3", "qs_slab_sum_stats",
           "qs_linear_tanh_cat_x3"]

_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise QuadSwarmError(f"libquadswarm.so not found at {LIB_PATH}; build it with __graft_entry__.build() "
                             "or `make -C quad-swarm-rl-stable-baselines3_amd`")
    L = ctypes.CDLL(LIB_PATH)
    P, V = ctypes.POINTER, ctypes.c_void_p
    sig = {
        "qs_abi_version": ([], I32), "qs_last_error": ([], ctypes.c_char_p),
        "qs_struct_sizes": ([P(SZ), P(SZ), P(SZ)], I32),
        "qs_config_default": ([P(QsConfig), I32, I32], I32), "qs_config_default_a": ([P(QsConfig), I32, I32], I32),
        "qs_layout_query": ([P(QsConfig), P(QsLayout)], I32),
        "qs_create": ([P(QsConfig), ctypes.c_int, V, P(V)], I32), "qs_destroy": ([V], I32),
        "qs_buffers_get": ([V, P(QsBuffers)], I32), "qs_reset": ([V, V, V], I32), "qs_step": ([V, V, V], I32),
        "qs_step_n": ([V, V, ctypes.c_int, V], I32),
        "qs_step_blocks": ([P(V), ctypes.c_int, P(V), P(V)], I32),
        "qs_counters": ([V, P(QsStats), V], I32), "qs_counters_reset": ([V, V], I32),
        "qs_set_param": ([V, ctypes.c_char_p, ctypes.c_double], I32),
        "qs_get_param": ([V, ctypes.c_char_p, P(ctypes.c_double)], I32),
        "qs_state_bytes": ([V], SZ), "qs_get_state": ([V, V, SZ, V], I32), "qs_set_state": ([V, V, SZ, V], I32),
        "qs_gae": ([V, V, V, V, V, V, V, I32, I32, F, F, V], I32),
        "qs_specialize": ([V, I32], I32), "qs_is_specialized": ([V], I32),
        "qs_config_kp_words": ([P(QsConfig), V, SZ], I32),
        "qs_specialize_compile": ([P(QsConfig)], ctypes.c_longlong),
        "qs_replay_config_default": ([P(QsReplayConfig), F], I32),
        "qs_replay_workspace_bytes": ([V, P(QsReplayConfig), P(SZ)], I32),
        "qs_replay_enable": ([V, P(QsReplayConfig), V], I32), "qs_replay_disable": ([V], I32),
        "qs_replay_buffers_get": ([V, P(QsReplayBuffers)], I32),
        "qs_attn_embed": ([V, I32, I32, I32, I32, I32, I32, I32, P(QsAttnTower), I32, V], I32),
        "qs_attn_pool": ([I32, I32, I32, P(QsAttnTower), I32, V], I32),
        "qs_attn_embed_x3": ([V, I32, I32, I32, I32, I32, I32, I32, P(QsAttnTower), I32, V], I32),
        "qs_attn_pool_x3": ([I32, I32, I32, P(QsAttnTower), I32, V], I32),
        "qs_curriculum_init": ([V, ctypes.c_double, ctypes.c_double, ctypes.c_double, I32], I32),
        "qs_curriculum_step": ([V, V, V], I32),
        "qs_curriculum_step_all": ([V, V, ctypes.c_int64, V, V], I32),
        "qs_attn_embed_train_x3": ([V, I32, I32, I32, I32, I32, I32, I32, P(QsAttnTower), P(QsAttnTrain), I32, V], I32),
        "qs_attn_pool_train_x3": ([I32, I32, I32, P(QsAttnTower), P(QsAttnTrain), I32, V], I32),
        "qs_attn_bwd1_x3": ([I32, I32, I32, P(QsAttnTower), P(QsAttnTrain), I32, V], I32),
        "qs_attn_bwd2_x3": ([I32, I32, I32, P(QsAttnTower), P(QsAttnTrain), I32, V], I32),
        "qs_attn_dw_x3": ([V, V, V, ctypes.c_int64, I32, V, V, I32, V], I32),
        "qs_colstats": ([V, ctypes.c_int64, I32, V, V, I32, I32, I32, I32, I32, I32, V, V, V, I32, V], I32),
        "qs_attn_dw0_x3": ([V, V, V, I32, I32, I32, I32, I32, I32, I32, V, V, I32, V], I32),
        "qs_colmax_reduce": ([V, I32, I32, I32, V, V], I32),
        "qs_linear_tanh_x3": ([V, ctypes.c_int64, I32, V, ctypes.c_int64, V, V, I32, V], I32),
        "qs_dw_x3_ld": ([V, I32, V, I32, V, ctypes.c_int64, I32, V, V, I32, V], I32),
        "qs_linear_rows_x3": ([V, V, ctypes.c_int64, I32, V, ctypes.c_int64, V, I32, V], I32),
        "qs_tanh_grad_stats": ([V, V, V, V, V, ctypes.c_int64, I32, V], I32),
        "qs_linear_bias_x3": ([V, ctypes.c_int64, I32, V, ctypes.c_int64, V, V, I32, V], I32),
        "qs_slab_sum_stats": ([V, I32, ctypes.c_int64, I32, V, V, V, V], I32),
        "qs_linear_tanh_cat_x3": ([V, V, ctypes.c_int64, V, ctypes.c_int64, V, V, I32, V], I32),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes, fn.restype = args, res
    if L.qs_abi_version() != ABI_VERSION:
        raise QuadSwarmError("libquadswarm ABI version mismatch")
    c, lay, b = SZ(), SZ(), SZ()
    L.qs_struct_sizes(ctypes.byref(c), ctypes.byref(lay), ctypes.byref(b))
    want = (ctypes.sizeof(QsConfig), ctypes.sizeof(QsLayout), ctypes.sizeof(QsBuffers))
    if (c.value, lay.value, b.value) != want:
        raise QuadSwarmError(f"struct mirror mismatch: C {(c.value, lay.value, b.value)} vs ctypes {want}")
    _lib = L
    return L


def check(rc, what=""):
    if rc != 0:
        msg = lib().qs_last_error().decode(errors="replace")
        raise QuadSwarmError(f"{what}: {msg} (code {rc})")
