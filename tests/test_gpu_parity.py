"""GPU parity: the HIP step (libquadswarm.so through the C ABI) against the CPU oracle and the
reference's golden fixtures.  Needs an MI355X: every test is marked gpu.

Tolerances (fp32 GPU vs fp64 oracle, identical Philox draws):
  * one step from an identical state: rows with no impulse and no contact (quiet) within 1e-6 abs + 1e-5 rel
    on state and rewards, 2e-6 abs + 1e-5 rel on self obs; eventful rows (pair impulse, floor / wall / ceiling
    contact, reset) within 2e-4 abs on obs / rewards, 5e-4 on velocity; discrete outputs (done, collisions ->
    rewards) identical;
  * free-running 10 steps from the same reset: 2e-3 abs on obs;
  * reference noise-free golden trajectory (n8quiet, 300 steps): positions within 2e-3 m.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no HIP device", allow_module_level=True)

import oracle as O  # noqa: E402
from parity_utils import (assert_obs_match, crowd, gpu_to_oracle, oracle_params, oracle_state_arrays,  # noqa: E402
                          oracle_to_gpu)
from quadswarm_amd import QuadSwarmConfig  # noqa: E402
from quadswarm_amd import _native as N_  # noqa: E402
from quadswarm_amd.env import QuadSwarmEnv  # noqa: E402
from quadswarm_amd.vec_env import GpuQuadVecEnv  # noqa: E402


def make_pair(E=64, N=8, K=6, seed=7, **kw):
    cfg = QuadSwarmConfig(num_envs=E, num_agents=N, neighbor_visible_num=K,
                          neighbor_obs_type="pos_vel" if N > 1 else "none", seed=seed, **kw)
    env = QuadSwarmEnv(cfg)
    oenv = O.OracleEnv(oracle_params(cfg), seed=seed)
    return cfg, env, oenv


def np_(t):
    return t.double().cpu().numpy()


@pytest.mark.parametrize("N,K", [(8, 6), (8, 7), (1, 0), (4, 2), (32, 6), (64, 6), (64, 63)])
def test_reset_matches_oracle(N, K):
    E = 2048 // N
    cfg, env, oenv = make_pair(E=E, N=N, K=K if N > 1 else -1)
    obs = np_(env.reset())
    want = oenv.reset()
    np.testing.assert_allclose(obs, want, atol=2e-5, rtol=1e-5)
    fields = env.drone_fields()
    pos = np.array([oenv.drones[g].pos[:] for g in range(env.I)])
    np.testing.assert_allclose(np_(fields["pos"]), pos, atol=2e-6)


# per-substep tolerance of the survey for rows with no impulse and no contact; the loose band
# is kept for rows that took a pair impulse / were in contact with the floor, a wall or the ceiling / reset
QUIET_STATE = dict(atol=1e-6, rtol=1e-5)
QUIET_OBS = dict(atol=2e-6, rtol=1e-5)
# omega's increment is a sum of four motor torques that cancel: one motor's per-substep change of omega is
# ~ arm * thrust_max / I * dt ~ 2 rad/s, so fp32 rounding leaves ~1e-6 rad/s absolute whatever |omega| is
# (measured: 2.5e-6 worst over 12 steps x 2048 drones); the bound is 16 ulp of that per-motor increment
QUIET_OMEGA = dict(atol=16 * 2.0 * 2.0 ** -23, rtol=1e-5)


def eventful_rows(oenv, floor_before, done):
    """Drones of the step that collided (any pair bit set after the step: new collisions took an impulse),
    touched the floor (before or after), crashed into a wall / the ceiling, or were reset."""
    N = oenv.N
    ev = np.array(done, bool).copy()
    for e in range(oenv.E):
        bits = np.frombuffer(bytes(oenv.envs[e].prev_pair_bits), np.uint8).reshape(O.MAXN, O.MAXN)[:N, :N]
        hit = (bits | bits.T).any(1)
        for i in range(N):
            d = oenv.drones[e * N + i]
            ev[e * N + i] |= bool(hit[i] or floor_before[e * N + i] or d.on_floor or d.crashed_floor or
                                  d.crashed_wall or d.crashed_ceiling or d.prev_wall or d.prev_ceiling)
    return ev


def _close_rows(got, want, rows, what, atol, rtol):
    if rows.any():
        err = np.abs(got[rows] - want[rows]) - rtol * np.abs(want[rows])
        np.testing.assert_allclose(got[rows], want[rows], atol=atol, rtol=rtol,
                                   err_msg=f"{what}: worst excess {err.max():.3g}")


@pytest.mark.parametrize("N,K,dw,rep", [(8, 6, False, "xyz_vxyz_R_omega"), (8, 7, False, "xyz_vxyz_R_omega"),
                                         (1, 0, False, "xyz_vxyz_R_omega"), (8, 2, True, "xyz_vxyz_R_omega"),
                                         (32, 6, False, "xyz_vxyz_R_omega"), (64, 6, False, "xyz_vxyz_R_omega"),
                                         (64, 63, True, "xyz_vxyz_R_omega"), (8, 6, False, "xyz_vxyz_R_omega_wall"),
                                         (8, 6, False, "xyz_vxyz_R_omega_floor")])
def test_one_step_from_identical_state(N, K, dw, rep):
    """Re-sync the GPU to the oracle's fp64 state every step: per-step parity incl. every branch -- quiet rows
    (no impulse, no contact) at the per-substep tolerance, eventful rows in the loose band (counted)."""
    E = 2048 // N
    cfg, env, oenv = make_pair(E=E, N=N, K=K if N > 1 else -1, use_downwash=dw, episode_duration=0.5, obs_repr=rep)
    so = cfg.obs_dim - 6 * cfg.k_neighbors
    env.reset()
    oenv.reset()
    rng = np.random.default_rng(3)
    crowd(oenv, rng)
    stats = dict(done=0, wall=0, coll=0, quiet=0, eventful=0)
    for t in range(12):
        oracle_to_gpu(oenv, env)
        floor_before = np.array([oenv.drones[g].on_floor != 0 for g in range(env.I)])
        a = rng.uniform(-1, 1, (env.I, 4)).astype(np.float32)
        obs, rew, done, term = env.step(torch.from_numpy(a).cuda())
        w_obs, w_rew, w_done, w_term = oenv.step(a.astype(np.float64))
        np.testing.assert_array_equal(done.cpu().numpy().astype(bool), w_done)
        loud = eventful_rows(oenv, floor_before, w_done)
        quiet = ~loud
        stats["quiet"] += int(quiet.sum())
        stats["eventful"] += int(loud.sum())
        g_rew, g_obs = np_(rew), np_(obs)
        np.testing.assert_allclose(g_rew, w_rew, atol=2e-4, rtol=1e-4)
        _close_rows(g_rew, w_rew, quiet, f"step {t} quiet rew", **QUIET_STATE)
        assert_obs_match(g_obs, w_obs, oenv, so, cfg.k_neighbors)
        oc = np.r_[0:15, 18:so]        # the omega columns (15:18) carry omega's absolute bound
        _close_rows(g_obs[:, oc], w_obs[:, oc], quiet, f"step {t} quiet self obs", **QUIET_OBS)
        _close_rows(g_obs[:, 15:18], w_obs[:, 15:18], quiet, f"step {t} quiet obs omega", **QUIET_OMEGA)
        if rep.endswith("wall"):    # the six wall distances saw contacts (clipped at 0) this step
            stats["wall"] += int((w_obs[:, 18:24] == 0).any(1).sum())
        if w_done.any():
            np.testing.assert_allclose(np_(term)[w_done], w_term[w_done], atol=2e-4, rtol=1e-4)
        # what the replay wrapper reads of the step: new collision, drone 0 on the floor
        fl = env.env_state[N_.E_FLAGS].cpu().numpy()
        np.testing.assert_array_equal((fl & N_.EF_NEWCOL) != 0, [oenv.envs[e].last_col != 0 for e in range(E)])
        np.testing.assert_array_equal((fl & N_.EF_FLOOR0) != 0, [oenv.envs[e].last_floor0 != 0 for e in range(E)])
        stats["newcol"] = stats.get("newcol", 0) + int(((fl & N_.EF_NEWCOL) != 0).sum())
        stats["done"] += int(w_done.sum())
        stats["coll"] += int((w_rew < -0.5).sum())
        # states agree after the step too
        f = env.drone_fields()
        want = dict(zip(("pos", "vel", "rot", "omega"), oracle_state_arrays(oenv)))
        np.testing.assert_allclose(np_(f["pos"]), want["pos"], atol=2e-5)
        np.testing.assert_allclose(np_(f["vel"]), want["vel"], atol=5e-4, rtol=1e-4)
        for k in ("pos", "vel", "rot", "omega"):
            _close_rows(np_(f[k]).reshape(env.I, -1), want[k], quiet, f"step {t} quiet {k}",
                        **(QUIET_OMEGA if k == "omega" else QUIET_STATE))
    assert stats["done"] > 0
    assert stats["quiet"] > stats["eventful"] > 0, stats
    if rep.endswith("wall"):
        assert stats["wall"] > 0
    if N > 1:
        assert stats["coll"] > 0 and stats["newcol"] > 0


def test_free_run_matches_oracle():
    cfg, env, oenv = make_pair(E=256, N=8, K=6)
    np.testing.assert_allclose(np_(env.reset()), oenv.reset(), atol=2e-5)
    rng = np.random.default_rng(5)
    for t in range(10):
        a = rng.uniform(-1, 1, (env.I, 4)).astype(np.float32)
        obs, rew, done, _ = env.step(torch.from_numpy(a).cuda())
        w_obs, w_rew, w_done, _ = oenv.step(a.astype(np.float64))
        np.testing.assert_allclose(np_(obs), w_obs, atol=2e-3, rtol=1e-3)
        np.testing.assert_allclose(np_(rew), w_rew, atol=1e-3)


def test_reference_quiet_trajectory(golden):
    """Noise-free reference trajectory (tests/golden/traj_n8quiet.npz, 300 steps) replayed on the GPU.

    SURVEY §8c's long-horizon bound is position error <= 1e-3 m after 100 control ticks; the divergence curve
    (tools/divergence_curve.py, profiles/r03_divergence_curve.txt) measures 8.0e-6 m at tick 100 and 2.2e-5 m at
    most over the 178 airborne ticks, self obs 6.0e-5: the bounds below are 1e-4 m (and 2e-5 m up to tick 100),
    3e-4 on the self obs."""
    g = golden("traj_n8quiet")
    n = int(g["n"])
    cfg = QuadSwarmConfig(num_envs=1, num_agents=n, neighbor_visible_num=int(g["k"]), sense_noise=None,
                          thrust_noise_ratio=0.0, episode_duration=15.0)
    env = QuadSwarmEnv(cfg)
    env.reset()
    _load_initial_state(env, g, n)
    # Compare each drone while it is airborne.  All eight eventually drop to the floor (open-loop
    # near-hover actions); floor sliding switches friction direction on |v| < 1e-6 (quadrotor_dynamics
    # .py:593-611), which is ill-conditioned between fp32 and fp64, so contact phases are checked
    # only for sanity.
    airborne = np.ones(n, bool)
    compared = 0
    for t in range(len(g["actions"])):
        obs, rew, done, _ = env.step(torch.from_numpy(g["actions"][t].astype(np.float32)).cuda())
        o = np_(obs)
        assert not done.any() and np.isfinite(o).all()
        want = g["obs"][t]
        airborne &= (want[:, 2] + 2.0) > 0.3
        m = airborne
        np.testing.assert_allclose(o[m, 0:3], want[m, 0:3], atol=2e-5 if t < 100 else 1e-4, err_msg=f"step {t}")
        np.testing.assert_allclose(o[m, :18], want[m, :18], atol=3e-4, err_msg=f"step {t}")
        np.testing.assert_allclose(np_(rew)[m], g["rew"][t][m], atol=2e-4, err_msg=f"step {t}")
        if m.all():
            assert_neighbors_close(o[:, 18:], want[:, 18:], atol=2e-2)
        compared += int(m.sum())
        assert (o[:, 2] + 2.0 >= 0.0459).all()      # nobody sinks through the floor
    assert compared >= 8 * 60


def test_reference_wall_trajectory(golden):
    """xyz_vxyz_R_omega_wall (get_state.py:270-292): the reference's noise-free 4-drone flight
    (tests/golden/traj_n4wallquiet.npz, 150 steps) replayed on the GPU, wall distances included."""
    g = golden("traj_n4wallquiet")
    n = int(g["n"])
    cfg = QuadSwarmConfig(num_envs=1, num_agents=n, neighbor_visible_num=int(g["k"]), sense_noise=None,
                          thrust_noise_ratio=0.0, episode_duration=15.0, obs_repr="xyz_vxyz_R_omega_wall")
    assert cfg.obs_dim == g["obs"].shape[2] == 24 + 6 * int(g["k"])
    env = QuadSwarmEnv(cfg)
    env.reset()
    _load_initial_state(env, g, n)
    airborne = np.ones(n, bool)
    compared = 0
    for t in range(len(g["actions"])):
        obs, rew, done, _ = env.step(torch.from_numpy(g["actions"][t].astype(np.float32)).cuda())
        o = np_(obs)
        assert not done.any() and np.isfinite(o).all()
        want = g["obs"][t]
        airborne &= (want[:, 2] + 2.0) > 0.3
        m = airborne   # divergence curve: 1.1e-5 m at most, self obs 3.6e-5 (profiles/r03_divergence_curve.txt)
        np.testing.assert_allclose(o[m, 0:3], want[m, 0:3], atol=1e-4, err_msg=f"step {t}")
        np.testing.assert_allclose(o[m, :24], want[m, :24], atol=3e-4, err_msg=f"step {t}")
        # the wall block is the room distances of the position, clipped to [0, 5] (get_state.py:282-287)
        np.testing.assert_allclose(o[m, 18:24], want[m, 18:24], atol=2e-3, err_msg=f"step {t} walls")
        np.testing.assert_allclose(np_(rew)[m], g["rew"][t][m], atol=2e-4, err_msg=f"step {t}")
        compared += int(m.sum())
    assert compared >= n * 60


def _load_initial_state(env, g, n):
    st = env.state.cpu().numpy()
    for i in range(n):
        st[0:3, i], st[3:6, i] = g["init_pos"][i], g["init_vel"][i]
        st[6:15, i], st[15:18, i] = g["init_rot"][i].ravel(), g["init_omega"][i]
        st[18:22, i], st[22:26, i], st[26:30, i] = g["init_rd"][i], g["init_cd"][i], g["init_ou"][i]
        st[30:33, i] = g["init_goal"][i]
    env.state.copy_(torch.from_numpy(st))
    ist = env.istate.cpu().numpy()
    ist[0, :n] = np.round(g["init_since"] / 0.005).astype(np.int32)
    ist[1:, :n] = 0
    env.istate.copy_(torch.from_numpy(ist))
    env.env_state.zero_()


def assert_neighbors_close(got, want, atol):
    """Neighbour slots compared up to a permutation: after hundreds of fp32 steps two neighbours whose
    sort keys are within rounding of each other may trade slots (the reference sorts in fp64)."""
    got = got.reshape(len(got), -1, 6)
    want = want.reshape(len(want), -1, 6)
    for i in range(len(got)):
        d = np.abs(got[i][:, None, :] - want[i][None, :, :]).max(-1)   # [slot_got, slot_want]
        match = d.argmin(1)
        assert len(set(match.tolist())) == len(match), f"drone {i}: neighbour sets differ"
        assert d[np.arange(len(match)), match].max() <= atol, f"drone {i}: {d.min(1).max()}" 


def test_full_size_properties():
    """Headline config (4096 envs x 8 drones): episode boundary, finiteness, clip boxes."""
    cfg = QuadSwarmConfig(num_envs=4096, num_agents=8)
    env = QuadSwarmEnv(cfg)
    obs = env.reset()
    assert obs.shape == (32768, 54)
    a = torch.empty(32768, 4, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(0)
    n_done_steps = 0
    for t in range(cfg.ep_len + 3):
        a.uniform_(-1, 1, generator=g)
        obs, rew, done, term = env.step(a)
        if done.any():
            assert bool(done.all())          # synchronised episodes end together
            assert t == cfg.ep_len           # tick > ep_len: 1501st step
            assert torch.isfinite(term).all()
            n_done_steps += 1
            # the reset put every drone inside the static_same_goal spawn box, at rest
            f = env.drone_fields()
            pos = f["pos"]
            assert (pos[:, 0:2].abs() <= 2.0 + 1e-5).all() and (pos[:, 2] >= 0.75 - 1e-6).all()
            assert (pos[:, 2] <= 4.0 + 1e-5).all() and (f["vel"] == 0).all() and (f["omega"] == 0).all()
            assert (env.env_state[0] == 0).all()
        if t % 100 == 0 or done.any():
            assert torch.isfinite(obs).all() and torch.isfinite(rew).all()
            nb = obs[:, 18:].view(-1, 6, 6)
            assert (nb[:, :, 0:3].abs() <= 10.0).all() and (nb[:, :, 3:6].abs() <= 6.0).all()
            assert (obs[:, 6:15].abs() <= 1.0 + 1e-3).all()
    assert n_done_steps == 1


def test_deterministic_and_shard_invariant():
    """Same seed -> bitwise identical; two half-size shards with drone_id_offset == one big env."""
    cfg = QuadSwarmConfig(num_envs=128, num_agents=8, seed=11, episode_duration=0.3)
    a_env, b_env = QuadSwarmEnv(cfg), QuadSwarmEnv(cfg)
    s0 = QuadSwarmEnv(QuadSwarmConfig(num_envs=64, num_agents=8, seed=11, episode_duration=0.3))
    s1 = QuadSwarmEnv(QuadSwarmConfig(num_envs=64, num_agents=8, seed=11, episode_duration=0.3, drone_id_offset=512))
    outs = [e.reset().clone() for e in (a_env, b_env)]
    assert torch.equal(outs[0], outs[1])
    assert torch.equal(torch.cat([s0.reset(), s1.reset()]), outs[0])
    g = torch.Generator(device="cuda").manual_seed(1)
    for t in range(40):
        act = torch.rand(1024, 4, device="cuda", generator=g) * 2 - 1
        ra = [x.clone() for x in a_env.step(act)[:3]]
        rb = [x.clone() for x in b_env.step(act)[:3]]
        r0 = [x.clone() for x in s0.step(act[:512].contiguous())[:3]]
        r1 = [x.clone() for x in s1.step(act[512:].contiguous())[:3]]
        for x, y, p, q in zip(ra, rb, r0, r1):
            assert torch.equal(x, y)
            assert torch.equal(torch.cat([p, q]), x)


def test_state_snapshot_roundtrip():
    env = QuadSwarmEnv(QuadSwarmConfig(num_envs=32, num_agents=8, seed=2))
    env.reset()
    act = torch.rand(256, 4, device="cuda") * 2 - 1
    for _ in range(5):
        env.step(act)
    blob = env.get_state()
    first = [x.clone() for x in env.step(act)[:3]]
    env.set_state(blob)
    again = [x.clone() for x in env.step(act)[:3]]
    for x, y in zip(first, again):
        assert torch.equal(x, y)


def test_partial_reset_mask_matches_oracle():
    cfg, env, oenv = make_pair(E=64, N=8, K=6)
    env.reset()
    oenv.reset()
    a = np.random.default_rng(0).uniform(-1, 1, (env.I, 4)).astype(np.float32)
    env.step(torch.from_numpy(a).cuda())
    oenv.step(a.astype(np.float64))
    mask = np.zeros(64, np.uint8)
    mask[::3] = 1
    before = np_(env.obs).copy()
    gpu_to_oracle(env, oenv)   # oracle twin of the post-step state (incl. the envs' RNG counters)
    obs = np_(env.reset(mask))
    want = oenv.reset(mask)
    rows = np.repeat(mask.astype(bool), 8)
    np.testing.assert_array_equal(obs[~rows], before[~rows])
    np.testing.assert_allclose(obs[rows], want[rows], atol=2e-5, rtol=1e-5)
    f = env.drone_fields()
    assert (np_(f["vel"])[rows] == 0).all()
    assert (env.env_state[0].cpu().numpy()[mask.astype(bool)] == 0).all()


def test_vec_env_surface():
    venv = GpuQuadVecEnv(QuadSwarmConfig(num_envs=16, num_agents=8, episode_duration=0.05))
    assert venv.num_envs == 128
    obs = venv.reset()
    assert obs.shape == (128, 54) and obs.dtype == np.float32
    assert venv.observation_space.shape == (54,) and venv.action_space.shape == (4,)
    got_done = False
    for t in range(10):
        obs, rew, dones, infos = venv.step(np.random.uniform(-1, 1, (128, 4)).astype(np.float32))
        assert obs.shape == (128, 54) and rew.shape == (128,) and dones.dtype == bool and len(infos) == 128
        if dones.any():
            got_done = True
            i = int(np.flatnonzero(dones)[0])
            assert infos[i]["terminal_observation"].shape == (54,)
            assert venv.reset_infos[i // 8] == {}
        else:
            assert all(r is None for r in venv.reset_infos)
    assert got_done
    venv.close()
