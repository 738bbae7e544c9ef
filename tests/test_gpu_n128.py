"""128-drone envs (the paper's largest swarm, /root/reference/paper/fps_compare.py:7): an env spans the two waves of
a 128-lane workgroup (qs_flavor_b.h StepGeo<128>, EnvColl<true>, impulses_wide).  The oracle is pinned at this size
by the reference's own 128-drone tape (tests/golden/traj_n128k6.npz, test_oracle_golden.py) and neighbour
selections (neighbors128.npz); here the HIP path is compared with the oracle on the same Philox draws.

Tolerances are those of test_gpu_parity.py (fp32 GPU vs fp64 oracle): quiet rows at the per-substep bound,
eventful rows (impulses, contacts, resets) in the loose band."""
import os
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import oracle as O  # noqa: E402
from parity_utils import assert_obs_match, crowd, oracle_state_arrays, oracle_to_gpu  # noqa: E402
from quadswarm_amd import QuadSwarmConfig  # noqa: E402
from quadswarm_amd import _native as N_  # noqa: E402
from quadswarm_amd.env import QuadSwarmEnv  # noqa: E402
from test_gpu_parity import (QUIET_OBS, QUIET_OMEGA, QUIET_STATE, _close_rows, eventful_rows,  # noqa: E402
                             make_pair, np_)


@pytest.mark.parametrize("K", [6, 16])
def test_reset_matches_oracle_128(K):
    cfg, env, oenv = make_pair(E=16, N=128, K=K)
    obs = np_(env.reset())
    want = oenv.reset()
    np.testing.assert_allclose(obs, want, atol=2e-5, rtol=1e-5)
    pos = np.array([oenv.drones[g].pos[:] for g in range(env.I)])
    np.testing.assert_allclose(np_(env.drone_fields()["pos"]), pos, atol=2e-6)


@pytest.mark.parametrize("K,dw,stats", [(6, True, True), (16, False, False)])
def test_one_step_from_identical_state_128(K, dw, stats):
    """Per-step parity from a shared fp64 state (re-synced every step), crowded so that pairs collide: the
    128-bit collision rows, the two-wave impulse loop and the env collectives of the stats counters."""
    N, E = 128, 16
    cfg, env, oenv = make_pair(E=E, N=N, K=K, use_downwash=dw, episode_duration=0.1, episode_stats=stats)
    so = cfg.obs_dim - 6 * K
    env.reset()
    oenv.reset()
    rng = np.random.default_rng(4)
    crowd(oenv, rng)
    seen = dict(done=0, coll=0, newcol=0, quiet=0, eventful=0, hi=0)
    for t in range(12):
        oracle_to_gpu(oenv, env)
        floor_before = np.array([oenv.drones[g].on_floor != 0 for g in range(env.I)])
        a = rng.uniform(-1, 1, (env.I, 4)).astype(np.float32)
        obs, rew, done, term = env.step(torch.from_numpy(a).cuda())
        w_obs, w_rew, w_done, w_term = oenv.step(a.astype(np.float64))
        np.testing.assert_array_equal(done.cpu().numpy().astype(bool), w_done)
        loud = eventful_rows(oenv, floor_before, w_done)
        quiet = ~loud
        seen["quiet"] += int(quiet.sum())
        seen["eventful"] += int(loud.sum())
        g_rew, g_obs = np_(rew), np_(obs)
        np.testing.assert_allclose(g_rew, w_rew, atol=2e-4, rtol=1e-4)
        _close_rows(g_rew, w_rew, quiet, f"step {t} quiet rew", **QUIET_STATE)
        assert_obs_match(g_obs, w_obs, oenv, so, K)
        oc = np.r_[0:15, 18:so]
        _close_rows(g_obs[:, oc], w_obs[:, oc], quiet, f"step {t} quiet self obs", **QUIET_OBS)
        _close_rows(g_obs[:, 15:18], w_obs[:, 15:18], quiet, f"step {t} quiet obs omega", **QUIET_OMEGA)
        if w_done.any():
            np.testing.assert_allclose(np_(term)[w_done], w_term[w_done], atol=2e-4, rtol=1e-4)
        fl = env.env_state[N_.E_FLAGS].cpu().numpy()
        np.testing.assert_array_equal((fl & N_.EF_NEWCOL) != 0, [oenv.envs[e].last_col != 0 for e in range(E)])
        seen["newcol"] += int(((fl & N_.EF_NEWCOL) != 0).sum())
        seen["done"] += int(w_done.sum())
        seen["coll"] += int((w_rew < -0.5).sum())
        # the collision rows after the step: the GPU's 128-bit rows equal the oracle's pair bits
        ist = env.istate.cpu().numpy().view(np.uint32).astype(np.uint64)
        rows = ist[N_.I_PREV_LO] | (ist[N_.I_PREV_HI] << 32), ist[N_.I_PREV_2] | (ist[N_.I_PREV_3] << 32)
        for e in range(E):
            bits = np.frombuffer(bytes(oenv.envs[e].prev_pair_bits), np.uint8).reshape(O.MAXN, O.MAXN)[:N, :N]
            sym = (bits | bits.T).astype(bool)
            for half, r in enumerate(rows):
                got = (r[e * N:(e + 1) * N, None] >> np.arange(64, dtype=np.uint64)[None, :]) & np.uint64(1)
                np.testing.assert_array_equal(got.astype(bool), sym[:, 64 * half:64 * (half + 1)],
                                              err_msg=f"step {t} env {e} collision row words {2 * half}..")
            seen["hi"] += int(sym[:, 64:].any())
        f = env.drone_fields()
        want = dict(zip(("pos", "vel", "rot", "omega"), oracle_state_arrays(oenv)))
        np.testing.assert_allclose(np_(f["pos"]), want["pos"], atol=2e-5)
        np.testing.assert_allclose(np_(f["vel"]), want["vel"], atol=5e-4, rtol=1e-4)
        for k in ("pos", "vel", "rot", "omega"):
            _close_rows(np_(f[k]).reshape(env.I, -1), want[k], quiet, f"step {t} quiet {k}",
                        **(QUIET_OMEGA if k == "omega" else QUIET_STATE))
    assert seen["done"] > 0 and seen["coll"] > 0 and seen["newcol"] > 0, seen
    assert seen["hi"] > 0, "no collision among drones 64..127 was exercised"
    assert seen["quiet"] > seen["eventful"] > 0, seen


def test_full_size_properties_128():
    """256 envs x 128 drones (32 768 drones, the C3 drone count) over a whole episode: the tick-1501 boundary,
    finiteness, the clip boxes and the spawn box after the fused reset."""
    cfg = QuadSwarmConfig(num_envs=256, num_agents=128, neighbor_visible_num=6)
    env = QuadSwarmEnv(cfg)
    obs = env.reset()
    assert obs.shape == (32768, 54)
    a = torch.empty(32768, 4, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(1)
    n_done_steps = 0
    for t in range(cfg.ep_len + 3):
        a.uniform_(-1, 1, generator=g)
        obs, rew, done, term = env.step(a)
        if done.any():
            assert bool(done.all()) and t == cfg.ep_len
            assert torch.isfinite(term).all()
            n_done_steps += 1
            f = env.drone_fields()
            pos = f["pos"]
            assert (pos[:, 0:2].abs() <= 2.0 + 1e-5).all() and (pos[:, 2] >= 0.75 - 1e-6).all()
            assert (pos[:, 2] <= 4.0 + 1e-5).all() and (f["vel"] == 0).all() and (f["omega"] == 0).all()
            # the reset cleared every drone's collision row, all four words
            assert (env.istate[N_.I_PREV_LO:N_.I_PREV_3 + 1] == 0).all()
        if t % 100 == 0 or done.any():
            assert torch.isfinite(obs).all() and torch.isfinite(rew).all()
            nb = obs[:, 18:].view(-1, 6, 6)
            assert (nb[:, :, 0:3].abs() <= 10.0).all() and (nb[:, :, 3:6].abs() <= 6.0).all()
    assert n_done_steps == 1
    c = env.counters()
    assert c["nonfinite_obs"] == 0 and c["nonfinite_rew"] == 0 and c["nonfinite_state"] == 0


def test_specialized_matches_generic_128():
    """The hipRTC-specialised 128-drone kernels are bitwise the generic ones."""
    outs = []
    for spec in (False, True):
        cfg = QuadSwarmConfig(num_envs=32, num_agents=128, neighbor_visible_num=6, seed=5, episode_duration=0.2,
                              use_downwash=True, specialize=spec)
        env = QuadSwarmEnv(cfg)
        assert env.specialized == spec
        env.reset()
        a = torch.rand(env.I, 4, device="cuda", generator=torch.Generator(device="cuda").manual_seed(2)) * 2 - 1
        acc = []
        for _ in range(30):
            obs, rew, done, _ = env.step(a)
            acc += [obs.clone(), rew.clone()]
        acc += [env.state.clone(), env.istate.clone()]
        outs.append(acc)
    for x, y in zip(*outs):
        assert torch.equal(x, y)

