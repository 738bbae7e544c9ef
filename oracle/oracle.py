"""ctypes binding of the CPU parity oracle (oracle/quadswarm_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg.  The product package never imports this module.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# QS_ORACLE_F32=1 (set only by bench.py's cpu_baseline subprocess): the fp32 twin of the same sources
F32 = os.environ.get("QS_ORACLE_F32") == "1"
LIB_PATH = os.path.join(HERE, "_build", "liboracle_f32.so" if F32 else "liboracle.so")

D = ctypes.c_float if F32 else ctypes.c_double
FT = np.float32 if F32 else np.float64
I = ctypes.c_int


class OrParams(ctypes.Structure):
    _fields_ = [
        ("mass", D), ("inertia", D * 3),
        ("thrust_max", D * 4), ("torque_max", D * 4), ("prop_cross", (D * 3) * 4), ("prop_ccw", D * 4),
        ("motor_tau_up", D), ("motor_tau_down", D), ("motor_linearity", D),
        ("arm", D), ("gravity", D), ("omega_max", D), ("vel_damp", D), ("damp_omega_quadratic", D),
        ("dt", D), ("sim_steps", I), ("since_last_svd_limit", D),
        ("room_lo", D * 3), ("room_hi", D * 3),
        ("ou_mu", D), ("ou_theta", D), ("ou_sigma", D),
        ("sense_noise", I),
        ("pos_norm_std", D), ("pos_unif_range", D), ("vel_norm_std", D), ("vel_unif_range", D),
        ("gyro_noise_density", D), ("quat_norm_std", D), ("quat_unif_range", D),
        ("acc_static_std", D), ("acc_dyn_ratio", D),
        ("num_agents", I), ("num_envs", I), ("ep_len", I), ("obs_repr", I), ("k_neighbors", I),
        ("collision_threshold", D), ("collision_falloff_threshold", D), ("control_dt", D),
        ("rew_pos", D), ("rew_effort", D), ("rew_crash", D), ("rew_orient", D), ("rew_spin", D),
        ("rew_quadcol_bin", D), ("rew_quadcol_smooth_max", D),
        ("use_downwash", I), ("apply_collision_force", I),
        ("spawn_box", D), ("goal", D * 3), ("id_offset", ctypes.c_uint32),
        # flavor A
        ("flavor", I), ("obs_repr_a", I), ("nfeat", I), ("nfeat_dim", I), ("ticks_per_step", I),
        ("scenario_a", I), ("nclip_lo", D * 8), ("nclip_hi", D * 8),
        ("cam_size", D), ("cam_focal", D), ("cam_px_noise", D), ("cam_fov_deg", D), ("cam_res", D),
        ("n_cameras", I), ("heading_rate", D), ("speed", D),
        ("pid_kp", D * 10), ("pid_kd", D * 10), ("pid_ki", D * 10), ("pid_sat", D * 10), ("pid_aw", D * 10),
        ("rate_out_scale", D), ("mixer", D * 16),
        ("m_mass", D), ("m_g", D), ("m_kf", D), ("m_min_rpm", D), ("m_max_rpm", D), ("m_n_motors", I),
        ("w_captor", D), ("w_helper", D), ("existence", D),
        ("target_vmax", D), ("target_dt", D), ("arena_size", D), ("target_z", D),
        ("use_obstacles", I), ("num_obstacles", I), ("obst_area", I), ("obst_scenario", I),
        ("obst_size", D), ("obst_z", D), ("sdf_resolution", D), ("rew_quadcol_bin_obst", D),
        ("scenario_b", I),
        ("dr_n_counts", I), ("dr_counts", I * 9), ("dr_n_sizes", I), ("dr_sizes", D * 9),
    ]


class OrScen(ctypes.Structure):   # or_scen: the attributes of the reference's Scenario_* object
    _fields_ = [("mode", I), ("formation", I), ("per_layer", I), ("period", I), ("increase", I),
                ("size", D), ("lo", D), ("hi", D), ("layer", D), ("speed", D),
                ("center", D * 3), ("bz", (D * 3) * 3), ("c1", D * 3), ("c2", D * 3)]


class OrSDraw(ctypes.Structure):  # or_sdraw: scenario draw source (tape or Philox)
    _fields_ = [("mode", I), ("seed", ctypes.c_uint32), ("key", ctypes.c_uint32), ("stream", ctypes.c_uint32),
                ("count", ctypes.c_uint32), ("step", ctypes.c_uint64), ("tape", ctypes.POINTER(D)),
                ("tape_n", ctypes.c_long), ("tape_pos", ctypes.c_long), ("overrun", I)]


# flavor-B scenarios (OR_SC_*): QUADS_MODE_LIST order (scenarios/utils.py:7-10) + run_away; mix = 10
SC_MODES = ["static_same_goal", "static_diff_goal", "ep_lissajous3D", "ep_rand_bezier", "dynamic_same_goal",
            "dynamic_diff_goal", "dynamic_formations", "swap_goals", "swarm_vs_swarm", "run_away"]
SC_NONE, SC_MIX = -1, 10
SC_O_SWAP_GOALS, SC_O_EP_RAND_BEZIER, SC_O_DYNAMIC_SAME_GOAL = 11, 12, 13   # the obstacle maps' dynamic scenarios
OSCEN_MODES = ["o_swap_goals", "o_ep_rand_bezier", "o_dynamic_same_goal"]  # obstacle modes 2, 3, 4
S_SCN, S_SCN_RESET = 23, 24
S_DR = 26


# reward components in or_drone.rinfo (OR_RI_*, quadswarm_oracle.h)
RI_DIST, RI_EFFORT, RI_CRASH, RI_ORIENT, RI_SPIN, RI_QUADCOL, RI_PROX, RI_OBST, NRI = range(9)
RI_GOAL_DIST = 0


class OrDrone(ctypes.Structure):
    _fields_ = [
        ("pos", D * 3), ("vel", D * 3), ("rot", D * 9), ("omega", D * 3), ("acc", D * 3),
        ("thrust_rot_damp", D * 4), ("thrust_cmds_damp", D * 4), ("ou", D * 4),
        ("since_last_svd", D),
        ("on_floor", I), ("crashed_floor", I), ("crashed_wall", I), ("crashed_ceiling", I),
        ("prev_wall", I), ("prev_ceiling", I),
        ("goal", D * 3),
        ("pid", D * 20), ("angle", D), ("ang_vel", D), ("prev_obst", I),
        ("hit_agent", I), ("hit_obst", I), ("reached", I), ("prev_room", I),
        ("dring", D * 5), ("dsum", D * 3), ("ep_dist", D * 3),
        ("rinfo", D * 8),   # the step's reward components (OR_RI_*, quadswarm_oracle.h)
    ]


MAXN = 128   # OR_MAXN (quadswarm_oracle.h): drones per env


class OrEnv(ctypes.Structure):
    _fields_ = [("tick", I), ("episode", ctypes.c_uint32), ("prev_pair_bits", ctypes.c_ubyte * (MAXN * MAXN)),
                ("obs_pos", (D * 3) * MAXN), ("obs_vel", (D * 3) * MAXN),
                ("heading", D * MAXN), ("target", D * 2), ("capture_radius", D), ("success", I), ("has_pos", I),
                ("n_obst", I), ("obst", (D * 2) * 64), ("obst_mode", I), ("scen", OrScen),
                ("last_col", I), ("last_floor0", I), ("obst_mi", I), ("obst_si", I),
                ("st_col", I), ("st_room", I), ("st_floor", I), ("st_wall", I), ("st_ceil", I), ("st_col_settle", I),
                ("st_col_final", I), ("st_ocol", I), ("st_ocol_settle", I), ("st_o35", I), ("st_o5", I),
                ("ep_done", I), ("ep_stats", D * 24)]


# episode_extra_stats (flavor B, quadrotor_multi.py:739-831): env-level columns of or_env.ep_stats (the GPU's
# estats columns QS_ES_*), and the reference's key names; scenario ids: QUADS_MODE_LIST order (scenarios/utils.py)
# for the goal scenarios, 16 + mode for the obstacle scenarios
ES_COL, ES_ROOM, ES_FLOOR, ES_WALL, ES_CEIL, ES_COL_SETTLE, ES_COL_FINAL = range(7)
ES_OCOL, ES_OCOL_SETTLE, ES_O35, ES_O5 = 7, 8, 9, 10
ES_SUCCESS, ES_DEADLOCK, ES_COLRATE, ES_NCOLRATE, ES_OCOLRATE, ES_SCEN, ES_D1, ES_D3, ES_D5, ES_REPLAY, NES = \
    11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 24


class OrRng(ctypes.Structure):
    _fields_ = [("mode", I), ("seed", ctypes.c_uint32), ("step", ctypes.c_uint64),
                ("tape", ctypes.POINTER(D)), ("tape_n", ctypes.c_long), ("tape_pos", ctypes.c_long),
                ("spawn", ctypes.POINTER(D)), ("spawn_n", ctypes.c_long), ("spawn_pos", ctypes.c_long),
                ("overrun", I)]


RNG_PHILOX, RNG_TAPE = 0, 1
S_SENSOR, S_RESET_SENSOR = 3, 11


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.POINTER
        L.or_params_default.argtypes = [P(OrParams)]
        L.or_dyn_substep.argtypes = [P(OrParams), P(OrDrone), P(D), P(D), P(OrRng), ctypes.c_uint32, I]
        L.or_ou_noise.argtypes = [P(OrParams), P(D), P(OrRng), ctypes.c_uint32]
        L.or_sensor_noise.argtypes = [P(OrParams), P(D), P(D), P(D), P(D), P(OrRng), ctypes.c_uint32,
                                      ctypes.c_uint32, P(D), P(D), P(D), P(D)]
        L.or_polar.argtypes = [P(D)]
        L.or_collide_drones.argtypes = [P(D)] * 6 + [P(OrRng), ctypes.c_uint32, ctypes.c_uint32]
        L.or_collide_wall.argtypes = [P(OrParams), P(OrDrone), P(OrRng), ctypes.c_uint32]
        L.or_collide_ceiling.argtypes = [P(OrDrone), P(OrRng), ctypes.c_uint32]
        L.or_obs_dim.argtypes = [P(OrParams)]
        L.or_env_reset.argtypes = [P(OrParams), P(OrDrone), P(OrEnv), I, P(OrRng), P(D)]
        L.or_env_step.argtypes = [P(OrParams), P(OrDrone), P(OrEnv), I, P(D), P(OrRng), P(D), P(D),
                                  P(ctypes.c_ubyte), P(D)]
        L.or_reset_all.argtypes = [P(OrParams), P(OrDrone), P(OrEnv), ctypes.c_uint32, P(D)]
        L.or_step_all.argtypes = [P(OrParams), P(OrDrone), P(OrEnv), P(D), ctypes.c_uint32,
                                  P(D), P(D), P(ctypes.c_ubyte), P(D), I]
        L.or_neighbor_obs.argtypes = [P(OrParams), P(OrEnv), P(D), I]
        U8 = P(ctypes.c_ubyte)
        L.or_params_default_a.argtypes = [P(OrParams)]
        L.or_pid_update.argtypes = [D, P(D), P(D), D, D, D, D, D, D]
        L.or_pid_update.restype = D
        L.or_ctrl_a.argtypes = [P(OrParams), P(OrDrone), D, D, P(D)]
        L.or_motors_to_cmds.argtypes = [P(D), P(D)]
        L.or_camera.argtypes = [P(OrParams), D, D, D, D, D, P(D), P(D)]
        L.or_self_obs_a.argtypes = [P(OrParams), P(OrDrone), P(OrRng), ctypes.c_uint32, ctypes.c_uint32,
                                    ctypes.c_uint32, P(D)]
        L.or_neighbor_obs_a.argtypes = [P(OrParams), P(OrEnv), P(OrDrone), P(OrRng), ctypes.c_uint32, I, P(D), I]
        L.or_target_step.argtypes = [P(OrParams), P(OrEnv), P(OrDrone)]
        L.or_env_reset_a.argtypes = [P(OrParams), P(OrDrone), P(OrEnv), I, P(OrRng), P(D), U8]
        L.or_env_step_a.argtypes = [P(OrParams), P(OrDrone), P(OrEnv), I, P(D), P(OrRng), P(D), P(D), U8, P(D), U8]
        L.or_reset_all_a.argtypes = [P(OrParams), P(OrDrone), P(OrEnv), ctypes.c_uint32, P(D), U8]
        L.or_step_all_a.argtypes = [P(OrParams), P(OrDrone), P(OrEnv), P(D), ctypes.c_uint32, P(D), P(D), U8,
                                    P(D), U8, I]
        L.or_obs_dim_a.argtypes = [P(OrParams)]
        L.or_obst_sdf.argtypes = [P(OrParams), P(OrEnv), P(D), P(D)]
        L.or_obst_detect.argtypes = [P(OrParams), P(OrEnv), P(D)]
        L.or_collide_obstacle.argtypes = [P(OrParams), P(OrDrone), P(D), P(OrRng), ctypes.c_uint32]
        L.or_max_square_center.argtypes = [P(ctypes.c_ubyte), I, P(D)]
        L.or_cell_xy.argtypes = [I, I, I, P(D)]
        L.or_scen_reset.argtypes = [P(OrParams), P(OrScen), P(OrSDraw), P(D)]
        L.or_scen_step.argtypes = [P(OrParams), P(OrScen), I, P(OrSDraw), P(D)]
        L.or_oscen_reset.argtypes = [P(OrParams), I, P(OrScen), P(OrSDraw), P(ctypes.c_ubyte), I, P(I), P(D), P(D)]
        L.or_oscen_step.argtypes = [P(OrParams), P(OrScen), I, P(OrSDraw), P(ctypes.c_ubyte), I, P(D)]
        L.or_generate_goals.argtypes = [I, I, I, D, D, P(D), P(D)]
        L.or_generate_goals.restype = I
        L.or_philox4x32_10.argtypes = [P(ctypes.c_uint32), P(ctypes.c_uint32), P(ctypes.c_uint32)]
        L.or_philox_normal.argtypes = [ctypes.c_uint32] * 3 + [ctypes.c_uint64, ctypes.c_uint32]
        L.or_philox_normal.restype = D
        L.or_philox_uniform.argtypes = [ctypes.c_uint32] * 3 + [ctypes.c_uint64, ctypes.c_uint32]
        L.or_philox_uniform.restype = D
        for nm, st in [("or_sizeof_params", OrParams), ("or_sizeof_drone", OrDrone),
                       ("or_sizeof_env", OrEnv), ("or_sizeof_rng", OrRng)]:
            got = getattr(L, nm)()
            if got != ctypes.sizeof(st):
                raise RuntimeError(f"oracle ABI mismatch {nm}: C {got} vs ctypes {ctypes.sizeof(st)}")
        _lib = L
    return _lib


def dptr(a):
    return a.ctypes.data_as(ctypes.POINTER(D))


def default_params(**over):
    p = OrParams()
    lib().or_params_default(ctypes.byref(p))
    for k, v in over.items():
        setattr(p, k, v)
    return p


# flavor-A neighbour types: feature mask (OR_NF_*), floats per neighbour, clip-box components
NF = dict(dist=1, ndist=2, angle=4, sangle=8, nsangle=16, heading=32, sheading=64, npos=128, pos=256, vel=512)
A_NTYPES = {
    "dist_angle": ("dist angle", ["dist", "angle"]),
    "dist_sangle": ("dist sangle", ["dist", "sangle"]),
    "ndist_nsangle": ("ndist nsangle", ["dist", "sangle"]),
    "dist_angle_heading": ("dist angle heading", ["dist", "angle", "angle"]),
    "dist_sangle_sheading": ("dist sangle sheading", ["dist", "sangle", "sangle"]),
    "pos": ("pos", ["rxyz"]),
    "npos": ("npos", ["rxyz"]),
    "pos_vel": ("pos vel", ["rxyz", "rvxyz"]),
}
A_REPRS = ["aw_awdot_dist_distdot_angle_angledot", "cdist_cdistdot_dist_distdot_angle_angledot",
           "cdist_cdistdot_dist_distdot_sangle_angledot", "cdist_cdistdot_ndist_distdot_nsangle_angledot"]


def a_neighbor_box(ntype, room):
    """(mask, dim, lo[], hi[]) of a flavor-A neighbour type: the per-feature clip box is the float32
    observation-space Box of quadrotor_single_rewards.make_observation_space (:267-319)."""
    feats, comps = A_NTYPES[ntype]
    mask = sum(NF[f] for f in feats.split())
    rr = np.array(room, dtype=np.float64)
    box = {"dist": ([-rr[0] / 2], [rr[0] / 2]), "angle": ([-np.pi], [np.pi]), "sangle": ([-1.0, -1.0], [1.0, 1.0]),
           "rxyz": (list(-rr), list(rr)), "rvxyz": ([-6.0] * 3, [6.0] * 3)}
    lo, hi = [], []
    for c in comps:
        lo += box[c][0]
        hi += box[c][1]
    lo = np.array(lo, dtype=np.float32).astype(np.float64)
    hi = np.array(hi, dtype=np.float32).astype(np.float64)
    return mask, len(lo), lo, hi


def params_a(num_agents=4, num_envs=1, k=None, obs_repr="cdist_cdistdot_dist_distdot_sangle_angledot",
             ntype="ndist_nsangle", room=(15.0, 15.0, 3.0), **over):
    p = OrParams()
    lib().or_params_default_a(ctypes.byref(p))
    p.num_agents, p.num_envs = num_agents, num_envs
    p.k_neighbors = (num_agents - 1) if k is None or k == -1 else k
    p.obs_repr_a = A_REPRS.index(obs_repr)
    mask, dim, lo, hi = a_neighbor_box(ntype, room)
    p.nfeat, p.nfeat_dim = mask, dim
    for i in range(dim):
        p.nclip_lo[i], p.nclip_hi[i] = lo[i], hi[i]
    for i in range(3):
        p.room_lo[i] = -room[i] / 2 if i < 2 else 0.0
        p.room_hi[i] = room[i] / 2 if i < 2 else room[2]
    for kk, v in over.items():
        setattr(p, kk, v)
    return p


def params_from_golden(g, **over):
    """Physical constants exactly as the reference derived them (tests/golden/params.npz)."""
    p = default_params()
    p.mass = float(g["mass"])
    for i in range(3):
        p.inertia[i] = float(g["inertia"][i])
    for k in range(4):
        p.thrust_max[k] = float(g["thrust_max"][k])
        p.torque_max[k] = float(g["torque_max"][k])
        p.prop_ccw[k] = float(g["prop_ccw"][k])
        for c in range(3):
            p.prop_cross[k][c] = float(g["prop_cross"][k][c])
    p.arm = float(g["arm"])
    p.motor_tau_up = float(g["motor_tau_up"])
    p.motor_tau_down = float(g["motor_tau_down"])
    p.collision_threshold = 2.0 * p.arm
    p.collision_falloff_threshold = 4.0 * p.arm
    for k, v in over.items():
        setattr(p, k, v)
    return p


class TapeRng:
    """Holds the numpy arrays alive for an OrRng in tape mode."""

    def __init__(self, tape, spawn=None):
        self.tape = np.ascontiguousarray(tape, dtype=FT)
        self.spawn = np.ascontiguousarray(spawn if spawn is not None else np.zeros(1), dtype=FT)
        self.r = OrRng()
        self.r.mode = RNG_TAPE
        self.r.tape = dptr(self.tape)
        self.r.tape_n = len(tape)
        self.r.spawn = dptr(self.spawn)
        self.r.spawn_n = 0 if spawn is None else len(spawn)

    @property
    def ref(self):
        return ctypes.byref(self.r)


class ScenDraws:
    """A scenario draw source (or_sdraw): tape mode holds the numpy array alive; Philox mode keys a
    stream exactly like the GPU (key = env id, stream S_SCN / S_SCN_RESET, counter = env {tick, episode})."""

    def __init__(self, tape=None, seed=0, key=0, stream=S_SCN_RESET, step=0):
        self.s = OrSDraw()
        if tape is not None:
            self.tape = np.ascontiguousarray(tape, dtype=FT)
            self.s.mode = RNG_TAPE
            self.s.tape = dptr(self.tape)
            self.s.tape_n = len(self.tape)
        else:
            self.s.mode = RNG_PHILOX
            self.s.seed, self.s.key, self.s.stream, self.s.step = seed, key, stream, step

    @property
    def ref(self):
        return ctypes.byref(self.s)


def philox_rng(seed, step):
    r = OrRng()
    r.mode = RNG_PHILOX
    r.seed = seed
    r.step = step
    return r


def drones_array(n):
    return (OrDrone * n)()


def envs_array(n):
    return (OrEnv * n)()


def set_drone(d, **kw):
    for k, v in kw.items():
        f = getattr(d, k)
        if isinstance(f, ctypes.Array):
            flat = np.ravel(np.asarray(v, dtype=np.float64))
            for i, x in enumerate(flat):
                f[i] = x
        else:
            setattr(d, k, type(f)(v) if not isinstance(f, (int, float)) else (int(v) if isinstance(f, int) else float(v)))


def get_arr(field, shape=None):
    a = np.ctypeslib.as_array(field).astype(np.float64).copy()
    return a.reshape(shape) if shape else a


class OracleEnv:
    """Batched flavor-B env in Philox mode: the CPU baseline and the GPU parity checker."""

    def __init__(self, params, seed=0):
        self.p = params
        self.E, self.N = params.num_envs, params.num_agents
        self.obs_dim = lib().or_obs_dim(ctypes.byref(params))
        self.drones = drones_array(self.E * self.N)
        self.envs = envs_array(self.E)
        self.seed = seed

    def reset(self, mask=None):
        obs = np.zeros((self.E * self.N, self.obs_dim), dtype=FT)
        if mask is None:
            lib().or_reset_all(ctypes.byref(self.p), self.drones, self.envs, self.seed, dptr(obs))
        else:
            r = philox_rng(self.seed, 0)
            for e in np.flatnonzero(mask):
                rows = obs[e * self.N:(e + 1) * self.N]
                lib().or_env_reset(ctypes.byref(self.p), self.drones, self.envs, int(e), ctypes.byref(r), dptr(rows))
        return obs

    def step(self, actions, nthreads=0):
        a = np.ascontiguousarray(actions, dtype=FT).reshape(self.E * self.N, 4)
        obs = np.zeros((self.E * self.N, self.obs_dim), dtype=FT)
        term = np.zeros_like(obs)
        rew = np.zeros(self.E * self.N, dtype=FT)
        done = np.zeros(self.E * self.N, dtype=np.uint8)
        lib().or_step_all(ctypes.byref(self.p), self.drones, self.envs, dptr(a), self.seed,
                          dptr(obs), dptr(rew), done.ctypes.data_as(ctypes.POINTER(ctypes.c_ubyte)),
                          dptr(term), nthreads)
        return obs, rew, done.astype(bool), term


NB_TRACE_W = 12   # OR_NB_TRACE_W


class OracleEnvA:
    """Batched flavor-A env (quadrotor_multi_rewards) in Philox mode."""

    def __init__(self, params, seed=0):
        self.p = params
        self.E, self.N = params.num_envs, params.num_agents
        self.obs_dim = lib().or_obs_dim_a(ctypes.byref(params))
        self.drones = drones_array(self.E * self.N)
        self.envs = envs_array(self.E)
        self.seed = seed
        n = self.E * self.N + int(params.id_offset)
        # inputs of the last call's neighbour-obs passes per drone (or_nb_trace* / or_key_trace* of
        # quadswarm_oracle_a.c): trace["step"|"reset"][g, slot] = (j, pixel noise 1, 2, pr[3], vr[3], aw, h_i, h_j),
        # keys["step"|"reset"][g, j] = selection key (K < N-1); NaN where the call ran no such pass
        on = FT == np.float64
        self.trace = {k: np.full((n, MAXN, NB_TRACE_W), np.nan) for k in ("step", "reset")} if on else None
        self.keys = {k: np.full((n, MAXN), np.nan) for k in ("step", "reset")} if on else None

    def _traced(self, fn):
        if self.trace is None:
            return fn()
        ptrs = [(ctypes.c_void_p.in_dll(lib(), name), arr) for name, arr in (
            ("or_nb_trace", self.trace["step"]), ("or_key_trace", self.keys["step"]),
            ("or_nb_trace_reset", self.trace["reset"]), ("or_key_trace_reset", self.keys["reset"]))]
        for v, arr in ptrs:
            arr.fill(np.nan)
            v.value = arr.ctypes.data
        try:
            return fn()
        finally:
            for v, _ in ptrs:
                v.value = None

    def rel_features(self, pr, aw, hi, hj, vr, n1=0.0, n2=0.0):
        """or_rel_features_x: one neighbour's features (unclipped) on explicit inputs."""
        f = np.zeros(8)
        a, b = np.ascontiguousarray(pr, dtype=np.float64), np.ascontiguousarray(vr, dtype=np.float64)
        n = lib().or_rel_features_x(ctypes.byref(self.p), dptr(a), ctypes.c_double(aw), ctypes.c_double(hi),
                                    ctypes.c_double(hj), dptr(b), ctypes.c_double(n1), ctypes.c_double(n2), dptr(f))
        return f[:n]

    def set_capture_radius(self, r):
        for e in range(self.E):
            self.envs[e].capture_radius = float(r)

    def reset(self, mask=None):
        obs = np.zeros((self.E * self.N, self.obs_dim), dtype=FT)
        ri = np.zeros(self.E, dtype=np.uint8)
        u8 = ri.ctypes.data_as(ctypes.POINTER(ctypes.c_ubyte))
        def run():
            if mask is None:
                lib().or_reset_all_a(ctypes.byref(self.p), self.drones, self.envs, self.seed, dptr(obs), u8)
                return
            for e in np.flatnonzero(mask):
                r = philox_rng(self.seed, 0)
                rows = obs[e * self.N:(e + 1) * self.N]
                lib().or_env_reset_a(ctypes.byref(self.p), self.drones, self.envs, int(e), ctypes.byref(r),
                                     dptr(rows), u8)
        self._traced(run)
        return obs, ri

    def step(self, actions, nthreads=0):
        a = np.ascontiguousarray(actions, dtype=FT).reshape(self.E * self.N, 2)
        obs = np.zeros((self.E * self.N, self.obs_dim), dtype=FT)
        term = np.zeros_like(obs)
        rew = np.zeros(self.E * self.N, dtype=FT)
        done = np.zeros(self.E * self.N, dtype=np.uint8)
        ri = np.zeros(self.E, dtype=np.uint8)
        self._traced(lambda: lib().or_step_all_a(
            ctypes.byref(self.p), self.drones, self.envs, dptr(a), self.seed, dptr(obs), dptr(rew),
            done.ctypes.data_as(ctypes.POINTER(ctypes.c_ubyte)), dptr(term),
            ri.ctypes.data_as(ctypes.POINTER(ctypes.c_ubyte)), nthreads))
        return obs, rew, done.astype(bool), term, ri
