"""CPU-side checks of the C ABI: libquadswarm.so loads, exports every symbol include/quadswarm.h
declares, and its host-side logic (defaults, layout, validation, error reporting) behaves.  No
compute calls: this runs without a GPU."""
import ctypes
import os
import re

import numpy as np
import pytest

from quadswarm_amd import QuadSwarmConfig, _native as N
from quadswarm_amd.env import observation_bounds
from quadswarm_amd.params import dynamics_constants, svd_every

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, "include", "quadswarm.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(qs_\w+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    L = N.lib()
    syms = header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(L, s), f"libquadswarm.so does not export {s}"
    assert sorted(N.EXPORTS) == syms


def test_struct_mirrors_and_abi():
    L = N.lib()
    assert L.qs_abi_version() == N.ABI_VERSION
    c, lay, b = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
    assert L.qs_struct_sizes(ctypes.byref(c), ctypes.byref(lay), ctypes.byref(b)) == 0
    assert (c.value, lay.value, b.value) == (ctypes.sizeof(N.QsConfig), ctypes.sizeof(N.QsLayout),
                                             ctypes.sizeof(N.QsBuffers))


def test_config_default_matches_host_derivation():
    c = N.QsConfig()
    assert N.lib().qs_config_default(c, 4096, 8) == 0
    k = dynamics_constants()
    assert c.num_envs == 4096 and c.num_agents == 8 and c.k_neighbors == 6 and c.ep_len == 1500
    assert c.svd_every == svd_every() == 100
    np.testing.assert_allclose(c.mass, k["mass"], rtol=1e-7)
    np.testing.assert_allclose(list(c.inertia), k["inertia"], rtol=1e-7)
    np.testing.assert_allclose(list(c.thrust_max), k["thrust_max"], rtol=1e-7)
    np.testing.assert_allclose(c.arm, k["arm"], rtol=1e-7)
    cfg = QuadSwarmConfig(num_envs=4096).to_qs_config()
    for f in ("mass", "arm", "motor_tau_up", "ou_sigma", "collision_threshold", "ep_len", "k_neighbors"):
        assert getattr(cfg, f) == pytest.approx(getattr(c, f), rel=1e-6), f


@pytest.mark.parametrize("N_,K,repr_,od", [(8, 6, "xyz_vxyz_R_omega", 54), (1, 0, "xyz_vxyz_R_omega", 18),
                                          (8, 2, "xyz_vxyz_R_omega_floor", 31), (32, 6, "xyz_vxyz_R_omega", 54),
                                          (8, -1, "xyz_vxyz_R_omega_wall", 66), (128, 6, "xyz_vxyz_R_omega", 54),
                                          (128, 16, "xyz_vxyz_R_omega", 114)])
def test_layout(N_, K, repr_, od):
    cfg = QuadSwarmConfig(num_envs=100, num_agents=N_, neighbor_visible_num=K, obs_repr=repr_,
                          neighbor_obs_type="pos_vel" if N_ > 1 else "none")
    assert cfg.obs_dim == od
    lay = N.QsLayout()
    assert N.lib().qs_layout_query(cfg.to_qs_config(), lay) == 0
    assert lay.obs_dim == od and lay.num_drones == 100 * N_
    offs = [lay.params, lay.state, lay.istate, lay.env, lay.stale_vel, lay.obs, lay.term_obs, lay.rew, lay.done]
    assert all(o % 256 == 0 for o in offs) and offs == sorted(offs)
    assert lay.obs - lay.state >= 4 * (N.NF + N.NI + 3) * 100 * N_
    assert lay.total_bytes >= lay.done + 100 * N_


def test_validation_errors_are_reported():
    L = N.lib()
    c = QuadSwarmConfig(num_envs=4, num_agents=8).to_qs_config()
    lay = N.QsLayout()
    bad = N.QsConfig.from_buffer_copy(c)
    bad.k_neighbors = 9
    assert L.qs_layout_query(bad, lay) == -1
    assert b"k_neighbors" in L.qs_last_error()
    bad = N.QsConfig.from_buffer_copy(c)
    bad.num_agents = 129
    assert L.qs_layout_query(bad, lay) == -2
    # envs of 65..128 drones (multi-wave workgroups): flavor A keeps its k nearest in registers (k <= 16); the
    # obs tile must fit the LDS
    a = N.QsConfig.from_buffer_copy(QuadSwarmConfig.sb_train(num_envs=4, num_agents=8).to_qs_config())
    a.num_agents = 65
    assert L.qs_layout_query(a, lay) == 0
    a.k_neighbors = N.A_KMAX + 1
    assert L.qs_layout_query(a, lay) == -2 and b"QS_A_KMAX" in L.qs_last_error()
    with pytest.raises(ValueError):
        QuadSwarmConfig.sb_train(num_envs=2, num_agents=128).to_qs_config()   # all 127 neighbours visible
    QuadSwarmConfig.sb_train(num_envs=2, num_agents=128, neighbor_visible_num=7).to_qs_config()
    wide = N.QsConfig.from_buffer_copy(QuadSwarmConfig(num_envs=4, num_agents=128, neighbor_visible_num=127).to_qs_config())
    assert L.qs_layout_query(wide, lay) == -2 and b"LDS" in L.qs_last_error()
    # the state / istate byte offsets (32-bit, 2 GB buffer descriptor) bound the drone count: the largest
    # accepted shard still addresses its last istate word inside the descriptor, one more drone is refused
    limit = (0x7fffffff - 256) // (4 * (N.NF + N.NI))
    big = N.QsConfig.from_buffer_copy(QuadSwarmConfig(num_envs=limit, num_agents=1, neighbor_obs_type="none",
                                                      neighbor_visible_num=0).to_qs_config())
    assert L.qs_layout_query(big, lay) == 0
    assert 4 * (N.NF + N.NI) * lay.num_drones + 255 < 0x7fffffff
    assert lay.istate - lay.state + 4 * N.NI * lay.num_drones <= 0x7fffffff
    big.num_envs = limit + 1
    assert L.qs_layout_query(big, lay) == -1 and b"too many drones" in L.qs_last_error()
    big.num_envs, big.num_agents = limit // 8 + 1, 8
    big.neighbor_obs, big.k_neighbors = c.neighbor_obs, c.k_neighbors
    assert L.qs_layout_query(big, lay) == -1
    bad = N.QsConfig.from_buffer_copy(c)
    bad.abi_version = 99
    assert L.qs_layout_query(bad, lay) == -1
    with pytest.raises(N.QuadSwarmError):
        N.check(L.qs_layout_query(bad, lay), "qs_layout_query")


DR = dict(replay_buffer_sample_prob=0.75, domain_random=True, obst_density_random=True, obst_size_random=True)


def test_domain_random_config_and_layout():
    """Obstacle domain randomisation: on only with replay (the reference builds the wrapper only then),
    pillar slots = the largest count, tables in qs_config, bad entries rejected by the library."""
    L = N.lib()
    off = QuadSwarmConfig.c4(num_envs=16, domain_random=True, obst_density_random=True)   # no replay
    assert not off.domain_random_active and off.to_qs_config().dr_num_counts == 0
    cfg = QuadSwarmConfig.c4(num_envs=16, obst_density_max=0.35, **DR)
    dens, counts, sizes = cfg.domain_random_tables()
    assert counts == [3, 6, 9, 12, 16, 19] and cfg.max_obstacles == 19
    c = cfg.to_qs_config()
    assert c.dr_num_counts == 6 and list(c.dr_counts[:6]) == counts
    assert c.dr_num_sizes == 3 and np.allclose(list(c.dr_sizes[:3]), [0.3, 0.4, 0.5])
    lay, lay0 = N.QsLayout(), N.QsLayout()
    assert L.qs_layout_query(c, lay) == 0
    assert L.qs_layout_query(QuadSwarmConfig.c4(num_envs=16).to_qs_config(), lay0) == 0
    assert lay.stale_vel - lay.obst >= 8 * 19 * 16 > lay0.stale_vel - lay0.obst - 256
    for field, val in (("dr_num_counts", 9), ("dr_num_sizes", -1)):
        bad = N.QsConfig.from_buffer_copy(c)
        setattr(bad, field, val)
        assert L.qs_layout_query(bad, lay) == -1
    bad = N.QsConfig.from_buffer_copy(c)
    bad.dr_counts[0] = 60          # no free cell left for 8 drones
    assert L.qs_layout_query(bad, lay) == -1 and b"dr_counts" in L.qs_last_error()
    bad = N.QsConfig.from_buffer_copy(c)
    bad.dr_counts[0] = -1          # a 0.0 density choice: keep
    assert L.qs_layout_query(bad, lay) == 0
    with pytest.raises(ValueError):   # a density choice with 0 pillars
        QuadSwarmConfig.c4(num_envs=4, obst_density_min=0.01, obst_density_max=0.02, **DR).to_qs_config()


def test_config_rejects_unbuilt_or_mixed_flavors():
    with pytest.raises(ValueError):   # a flavor-A repr on a flavor-B env
        QuadSwarmConfig(obs_repr="cdist_cdistdot_dist_distdot_sangle_angledot").to_qs_config()
    with pytest.raises(NotImplementedError):   # not in QUADS_MODE_LIST (needs a trajectory csv)
        QuadSwarmConfig(quads_mode="ep_trajectory").to_qs_config()
    with pytest.raises(NotImplementedError):   # not a create_scenario mode of either flavor
        QuadSwarmConfig.sb_train(quads_mode="o_random").to_qs_config()
    # flavor A builds every goal scenario through create_scenario (quadrotor_multi_rewards.py:123)
    c = QuadSwarmConfig.sb_train(quads_mode="mix").to_qs_config()
    assert c.scenario == N.SCENARIO_B["mix"]
    lay = N.QsLayout()
    assert N.lib().qs_layout_query(ctypes.byref(c), ctypes.byref(lay)) == 0
    with pytest.raises(ValueError):
        QuadSwarmConfig(num_agents=1, quads_mode="run_away").to_qs_config()


@pytest.mark.parametrize("mode", sorted(N.SCENARIO_B))
def test_flavor_b_goal_scenarios_accepted(mode):
    """Every quads_mode of QUADS_MODE_LIST (+ mix, run_away) builds a flavor-B config; the C side keeps the
    layout and adds the goal tables to the LDS of the step kernel."""
    c = QuadSwarmConfig(num_envs=3, num_agents=8, quads_mode=mode).to_qs_config()
    assert c.scenario == N.SCENARIO_B[mode]
    lay = N.QsLayout()
    assert N.lib().qs_layout_query(ctypes.byref(c), ctypes.byref(lay)) == 0
    assert lay.obs_dim == 54
    assert QuadSwarmConfig.sb_train(use_downwash=True).to_qs_config().use_downwash == 1   # flavor A: per tick
    with pytest.raises(NotImplementedError):
        QuadSwarmConfig.sb_train(neighbor_obs_type="pos_vel_R").to_qs_config()


@pytest.mark.parametrize("N_,ntype,k,repr_,od", [
    (4, "ndist_nsangle", -1, "cdist_cdistdot_dist_distdot_sangle_angledot", 7 + 3 * 3),
    (8, "ndist_nsangle", -1, "cdist_cdistdot_dist_distdot_sangle_angledot", 7 + 7 * 3),
    (8, "dist_sangle_sheading", 3, "cdist_cdistdot_ndist_distdot_nsangle_angledot", 7 + 3 * 5),
    (8, "dist_angle", 6, "aw_awdot_dist_distdot_angle_angledot", 6 + 6 * 2),
    (8, "pos_vel", -1, "cdist_cdistdot_dist_distdot_angle_angledot", 6 + 7 * 6),
    (1, "none", -1, "cdist_cdistdot_dist_distdot_sangle_angledot", 7),
])
def test_layout_flavor_a(N_, ntype, k, repr_, od):
    """obs dims of flavor A (QUADS_OBS_REPR / QUADS_NEIGHBOR_OBS_TYPE, quad_utils.py:30-58) and the
    reference's own observation_space shape for the sb_train config."""
    cfg = QuadSwarmConfig.sb_train(num_envs=5, num_agents=N_, neighbor_obs_type=ntype, neighbor_visible_num=k,
                                   obs_repr=repr_)
    c = cfg.to_qs_config()
    lay = N.QsLayout()
    N.check(N.lib().qs_layout_query(c, lay))
    assert lay.obs_dim == od == cfg.obs_dim
    lo, hi = observation_bounds(cfg)
    assert lo.shape == (od,)
    assert lay.env_f >= lay.env and lay.stale_vel > lay.env_f and lay.reset_info > lay.done
    assert lay.total_bytes >= lay.reset_info + 5


def test_sb_train_observation_space_matches_reference():
    """Box bounds of the sb_train flavor-A config: 7 self + 3 per neighbour (cdist 0..7.5, cdistdot +-3,
    dist +-7.5, distdot +-3, sangle +-1, angledot +-40; neighbour dist +-7.5, sangle +-1)."""
    cfg = QuadSwarmConfig.sb_train(num_envs=1, num_agents=4)
    lo, hi = observation_bounds(cfg)
    np.testing.assert_allclose(lo[:7], [0, -3, -7.5, -3, -1, -1, -40])
    np.testing.assert_allclose(hi[:7], [7.5, 3, 7.5, 3, 1, 1, 40])
    np.testing.assert_allclose(lo[7:], [-7.5, -1, -1] * 3)


def test_config_default_a():
    c = N.QsConfig()
    N.check(N.lib().qs_config_default_a(c, 16, 8))
    assert c.flavor == N.FLAVOR_A and c.scenario == N.SCENARIO["dynamic_repulsive"]
    assert c.k_neighbors == 7 and c.neighbor_obs == N.NEIGHBOR["ndist_nsangle"] and c.ep_len == 3000
    assert c.apply_collision_force == 0 and c.ticks_per_step == 8 and c.cam_px_noise == 0.0
    mine = QuadSwarmConfig.sb_train(num_envs=16, num_agents=8).to_qs_config()
    for f in ("flavor", "scenario", "obs_repr", "neighbor_obs", "k_neighbors", "ep_len", "ticks_per_step",
              "n_cameras", "apply_collision_force"):
        assert getattr(mine, f) == getattr(c, f), f
    assert list(mine.room_hi) == list(c.room_hi)


def test_from_reference_cfg_flavor_a():
    class Cfg:  # swarm_rl/global_cfg.py QuadrotorEnvConfig defaults (flavor A, sb_train)
        num_agents = 4
        obs_repr = "cdist_cdistdot_dist_distdot_angle_angledot"
        episode_duration = 30.0
        neighbor_visible_num = -1
        neighbor_obs_type = "dist_angle"
        dim_mode = "2D_horizontal"
        quads_mode = "dynamic_repulsive"
        room_dims = [15, 15, 3]
        initial_capture_radius = 3.0
        pixel_noise_cam = 3.0
        thrust_noise_ratio = 0.3     # ignored by the reference's flavor A
        dynamics_change = None
        use_downwash = False
    c = QuadSwarmConfig.from_reference_cfg(Cfg(), num_envs=13)
    assert c.flavor == "A" and c.thrust_noise_ratio == 0.05 and not c.apply_collision_force
    assert c.obs_dim == 6 + 3 * 2 and c.ep_len == 3000
    q = c.to_qs_config()
    assert q.capture_radius == 3.0 and q.cam_px_noise == 3.0


def test_from_reference_cfg_names():
    class Cfg:  # swarm_rl/global_cfg.py field names
        num_agents = 8
        episode_duration = 15.0
        neighbor_visible_num = 6
        neighbor_obs_type = "pos_vel"
        obs_repr = "xyz_vxyz_R_omega"
        quads_mode = "static_same_goal"
        room_dims = [10, 10, 10]
        seed = None
    c = QuadSwarmConfig.from_reference_cfg(Cfg, num_envs=4096)
    assert c.num_envs == 4096 and c.ep_len == 1500 and c.obs_dim == 54 and c.seed == 0


def test_params_restatement_matches_reference(golden):
    g = golden("params")
    k = dynamics_constants()
    for f in ("mass", "inertia", "thrust_max", "torque_max", "prop_cross", "arm", "motor_tau_up", "motor_tau_down"):
        np.testing.assert_array_equal(np.asarray(k[f]), g[f])


def test_create_without_device_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    L = N.lib()
    h = ctypes.c_void_p()
    rc = L.qs_create(QuadSwarmConfig(num_envs=4, num_agents=8).to_qs_config(), 0, None, ctypes.byref(h))
    assert rc == -3 and not h.value
    assert L.qs_last_error()


@pytest.mark.parametrize("make", [lambda: QuadSwarmConfig(num_envs=64, num_agents=8, neighbor_visible_num=6),
                                  lambda: QuadSwarmConfig.c4(num_envs=64),
                                  lambda: QuadSwarmConfig.sb_train(num_envs=64, num_agents=4),
                                  lambda: QuadSwarmConfig(num_envs=64, num_agents=64, neighbor_visible_num=6),
                                  lambda: QuadSwarmConfig(num_envs=64, num_agents=1, neighbor_obs_type="none",
                                                          episode_stats=False)],
                         ids=["c3", "c4", "a4", "n64", "c2-nostats"])
def test_specialised_kernels_compile_on_the_host(make):
    """qs_specialize's hipRTC path (kernel source embedded in the .so, parameter block baked in)
    compiles for gfx950 without a device."""
    L = N.lib()
    n = L.qs_specialize_compile(make().to_qs_config())
    assert n > 10000, L.qs_last_error()


def test_config_kp_words():
    L = N.lib()
    buf = (ctypes.c_uint32 * 4096)()
    qc = QuadSwarmConfig(num_envs=64, num_agents=8).to_qs_config()
    n = L.qs_config_kp_words(qc, buf, 4096)
    assert 100 < n < 4096
    assert L.qs_config_kp_words(qc, buf, 10) < 0      # buffer too small
    # the parameter block starts with E, N, I, obs_dim
    assert list(buf[:4]) == [64, 8, 512, 54]


def _reference_env_config(**over):
    """The reference's own QuadrotorEnvConfig defaults (swarm_rl/global_cfg.py), as recorded by
    tools/gen_golden_a_replay.py into tests/golden/quadrotor_env_config.json."""
    import json
    import types
    with open(os.path.join(os.path.dirname(__file__), "golden", "quadrotor_env_config.json")) as f:
        d = json.load(f)
    d.update(over)
    return types.SimpleNamespace(**d)


def test_from_reference_cfg_real_field_set():
    ref = _reference_env_config()
    c = QuadSwarmConfig.from_reference_cfg(ref, num_envs=13)
    assert c.flavor == "A" and c.num_envs == 13 and c.num_agents == ref.num_agents
    assert c.obs_repr == ref.obs_repr and c.neighbor_obs_type == ref.neighbor_obs_type
    assert c.quads_mode == ref.quads_mode and tuple(c.room_dims) == tuple(ref.room_dims)
    # flavor A: the replay wrapper comes only from use_replay_buffer (sb3_quad_env.py:43-45), not from the
    # SF runs' replay_buffer_sample_prob (0.75 in the same dataclass)
    assert ref.replay_buffer_sample_prob == 0.75 and c.replay_buffer_sample_prob == 0.0
    q = c.to_qs_config()
    assert q.capture_radius == ref.initial_capture_radius and q.cam_px_noise == ref.pixel_noise_cam
    assert c.ep_len == int(ref.episode_duration * ref.sim_freq / ref.sim_steps)


def test_flavor_a_replay_refused_like_the_reference():
    """The reference's flavor-A replay stack raises KeyError('rew_crash') on its first step
    (tests/golden/a_replay_outcome.json, generated by running the reference's own wrapper + env)."""
    import json
    with open(os.path.join(os.path.dirname(__file__), "golden", "a_replay_outcome.json")) as f:
        rec = json.load(f)
    assert [c["n"] for c in rec["cases"]] == [8, 4, 2]
    for case in rec["cases"]:
        assert case["step_error"] == "KeyError: 'rew_crash'" and case["step_error_at"] == 0
    c = QuadSwarmConfig.from_reference_cfg(_reference_env_config(use_replay_buffer=True), num_envs=4)
    assert c.replay_buffer_sample_prob == 0.5
    with pytest.raises(KeyError, match="rew_crash"):
        c.to_qs_config()


def test_jit_opts_may_not_change_launch_geometry(monkeypatch):
    """The host sizes step launches from its own QS_QB / QS_QA / QS_QW (block_threads, envs_per_block); a hipRTC
    option that redefines them would compile kernels indexing envs and LDS for another geometry: refused."""
    L = N.lib()
    qc = QuadSwarmConfig(num_envs=64, num_agents=64, neighbor_visible_num=6).to_qs_config()
    for opt in ("-DQS_QW=1", "-DQS_QB=2", "-DQS_QA=4"):
        monkeypatch.setenv("QS_JIT_OPTS", "-DQS_FOO=1 " + opt)
        assert L.qs_specialize_compile(qc) == -1          # QS_E_INVALID
        assert opt[2:7] in L.qs_last_error().decode()


def test_jit_src_dir_of_another_abi_is_refused(monkeypatch, tmp_path):
    """QS_JIT_SRC_DIR (kernel-variant A/B) compiles the directory's headers but launches them with this library's
    kernel arguments: a tree whose quadswarm.h carries another QS_ABI_VERSION is refused before hipRTC runs
    (round 5's illegal address: round-4 sources under the ABI-13 host).  The current sources pass."""
    import shutil
    L = N.lib()
    qc = QuadSwarmConfig(num_envs=64, num_agents=8, neighbor_visible_num=6).to_qs_config()
    csrc = os.path.join(os.path.dirname(__file__), "..", "quad-swarm-rl-stable-baselines3_amd", "csrc")
    inc = os.path.join(os.path.dirname(__file__), "..", "include")
    for name in ("qs_rng.h", "qs_common.h", "qs_flavor_b.h", "qs_flavor_a.h", "qs_replay.h", "qs_scen.h"):
        shutil.copy(os.path.join(csrc, name), tmp_path / name)
    hdr = open(os.path.join(inc, "quadswarm.h")).read()
    abi = N.ABI_VERSION
    assert f"#define QS_ABI_VERSION {abi}\n" in hdr
    monkeypatch.setenv("QS_JIT_SRC_DIR", str(tmp_path))
    (tmp_path / "quadswarm.h").write_text(hdr)
    assert L.qs_specialize_compile(qc) > 10000, L.qs_last_error()
    (tmp_path / "quadswarm.h").write_text(hdr.replace(f"#define QS_ABI_VERSION {abi}\n",
                                                      f"#define QS_ABI_VERSION {abi - 2}\n"))
    assert L.qs_specialize_compile(qc) == -1          # QS_E_INVALID
    assert f"QS_ABI_VERSION {abi - 2}" in L.qs_last_error().decode()


def test_curriculum_init_fills_the_struct_mirror():
    """qs_curriculum_init (host only) writes exactly the mirrored struct: the reference's starting state of
    CurriculumCallback (custom_callbacks.py:442-451), a cleared window."""
    L = N.lib()
    n = ctypes.sizeof(N.QsCurriculum)
    raw = (ctypes.c_uint8 * (n + 64))(*([0xAB] * (n + 64)))
    assert L.qs_curriculum_init(raw, 0.5, 0.8, 0.9, 40) == 0
    assert bytes(raw[n:]) == b"\xab" * 64             # nothing written past the mirror's size
    c = N.QsCurriculum.from_buffer_copy(bytes(raw[:n]))
    assert (c.radius, c.sr_threshold, c.decay, c.window) == (0.5, 0.8, 0.9, 40)
    assert c.window_i == 0 and c.n_shrinks == 0 and c.success_rate == 0.0 and not any(c.past)
    assert L.qs_curriculum_init(raw, 0.5, 0.8, 0.9, 65) == -1
    assert L.qs_curriculum_init(raw, 0.0, 0.8, 0.9, 40) == -1


@pytest.mark.parametrize("mode", ["o_swap_goals", "o_ep_rand_bezier", "o_dynamic_same_goal"])
def test_obstacle_dynamic_scenarios_accepted(mode):
    """The obstacle maps' dynamic scenarios (ABI 14): accepted with obstacles, their qs_scenario values, a layout with
    the goal tables in the LDS budget, and specialised kernels that compile; refused without obstacles."""
    L = N.lib()
    c = QuadSwarmConfig.c4(num_envs=64, quads_mode=mode)
    qc = c.to_qs_config()
    assert qc.scenario == N.SCENARIO[mode] == {"o_swap_goals": 15, "o_ep_rand_bezier": 16, "o_dynamic_same_goal": 17}[mode]
    lay = N.QsLayout()
    assert L.qs_layout_query(qc, lay) == 0, L.qs_last_error()
    assert L.qs_specialize_compile(qc) > 10000, L.qs_last_error()
    with pytest.raises(NotImplementedError):
        QuadSwarmConfig(num_envs=4, num_agents=8, quads_mode=mode).to_qs_config()
