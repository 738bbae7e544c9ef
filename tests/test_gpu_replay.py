"""GPU experience replay (csrc/qs_replay.h) against the replay oracle (oracle/replay_oracle.py, pinned to the
reference's ExperienceReplayWrapper by tests/golden/replay_*.npz).

The oracle is driven by exactly what the GPU step produced (done, tick, the step's collision / floor flags and
the Philox draws of stream S_REPLAY), so the comparison is bit-exact over thousands of steps: every replay
integer (activation, checkpoint ring, event deque order, replay counts, last add tick, episode / replay
counters), the crash history, and the contents of every snapshot the kernel saves, writes to the buffer and
restores."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no HIP device", allow_module_level=True)

import ctypes  # noqa: E402

import oracle as O  # noqa: E402
from replay_oracle import FixedDraws, ReplayOracle  # noqa: E402
from quadswarm_amd import QuadSwarmConfig  # noqa: E402
from quadswarm_amd import _native as N  # noqa: E402
from quadswarm_amd.env import QuadSwarmEnv  # noqa: E402

S_REPLAY = 25


def host_views(env):
    """The live buffers a snapshot covers, on the host as 32-bit words."""
    v = dict(state=env.state.cpu().numpy().view(np.int32), istate=env.istate.cpu().numpy(),
             stale=env.stale_vel.cpu().numpy().view(np.int32), env=env.env_state.cpu().numpy(),
             envf=N.env_f_rows(env.env_f.cpu().numpy()).view(np.int32), obs=env.obs.cpu().numpy().view(np.int32))
    v["obst"] = env.obstacles.cpu().numpy().view(np.int32) if env.obstacles is not None else None
    return v


def pack_live(v, n, e):
    """env e's live state as the kernel's snapshot words (quadswarm.h qs_replay_buffers.snap_words)."""
    sl = slice(e * n, (e + 1) * n)
    parts = [v["state"][:, sl].ravel(), v["istate"][:, sl].ravel(), v["stale"][:, sl].ravel(), v["env"][:, e],
             v["envf"][:, e]]
    if v["obst"] is not None:
        parts.append(v["obst"][e].ravel())
    parts.append(v["obs"][sl].ravel())
    return np.concatenate(parts)


def philox_pair(seed, gid, tick, episode):
    step = (int(episode) << 32) | (int(tick) & 0xFFFFFFFF)
    L = O.lib()
    return (L.or_philox_uniform(seed, gid, S_REPLAY | 0x80, ctypes.c_uint64(step), 0),
            L.or_philox_uniform(seed, gid, S_REPLAY | 0x80, ctypes.c_uint64(step), 1))


@pytest.mark.parametrize("obst", [False, True])
def test_replay_matches_oracle(obst):
    E, n = 24, 8
    kw = dict(num_envs=E, num_agents=n, neighbor_visible_num=6 if not obst else 2, seed=11, episode_duration=1.0)
    cfg = QuadSwarmConfig.c4(**kw) if obst else QuadSwarmConfig(**kw)
    env = QuadSwarmEnv(cfg)
    qc = env.qcfg
    # the reference's rules at a 10x shorter time scale so that episodes, activation and events come quickly
    env.enable_replay(0.75, cp_every=5, grace_ticks=15, min_gap_ticks=20)
    rc, R = env.replay_config, env.replay
    W, keep, nod = R["snap_words"], rc.keep, n * env.obs_dim
    crash_unit = float(np.float32(qc.dt)) * float(np.float32(qc.rew_crash))
    ep_len = int(env.get_param("ep_len"))
    ros = [ReplayOracle(rc.sample_prob, rc.cp_every, rc.grace_ticks, rc.min_gap_ticks, bufsz=rc.buffer_size,
                        keep=keep, steps_ago=rc.steps_ago, max_rep=rc.max_replays) for _ in range(E)]
    # crowd the spawn so drones collide often: the static goal with a small spawn box
    env.reset()
    for ro in ros:
        ro.explicit_reset()
    rng = np.random.default_rng(0)
    counts = dict(saves=0, pushes=0, replays=0, active=0)
    for t in range(1400):
        # hover-ish actions with noise: drones stay airborne most of the time and bump into each other
        a = np.clip(rng.normal(0.0, 0.6, (env.I, 4)), -1, 1).astype(np.float32)
        if t % 40 == 0:
            st = env.state.cpu().numpy()
            for e in range(E):   # pull each env's drones together around drone 0
                for i in range(1, n):
                    g = e * n + i
                    st[0:3, g] = st[0:3, e * n] + rng.normal(0, 0.05, 3)
            env.state.copy_(torch.from_numpy(st))
        _, _, done, _ = env.step(torch.from_numpy(a).cuda())
        torch.cuda.synchronize()
        dn = done.cpu().numpy().reshape(E, n)[:, 0].astype(bool)
        es = env.env_state.cpu().numpy()
        ri = R["ri"].cpu().numpy()
        store = R["store"].cpu().numpy()
        perm, crash = R["perm"].cpu().numpy(), R["crash"].cpu().numpy()
        hv = host_views(env)
        for e in range(E):
            ro = ros[e]
            tick = ep_len + 1 if dn[e] else int(es[N.E_TICK, e])
            flags = int(es[N.E_FLAGS, e])
            col, fl0 = int((flags & N.EF_NEWCOL) != 0), int((flags & N.EF_FLOOR0) != 0)
            draws = None
            if dn[e]:   # a restored env's flags are the snapshot's; it was active, so they are not read
                draws = FixedDraws(*philox_pair(cfg.seed, e * n, 0, es[N.E_EPISODE, e]))
            ck_before = ro.ck_head
            live = None
            if not dn[e]:
                live = pack_live(hv, n, e)
            tok, restored = ro.step(tick, dn[e], col, fl0, crash_unit, draws, ("pending", t, e))
            # a checkpoint saved this step: the ring slot holds the live state (its obs is the live obs,
            # even when the same step then hands the event's obs to the policy)
            if not dn[e] and ro.ck_head != ck_before:
                slot = ck_before
                got = store[e, slot]
                if ro.pushed_slot < 0:
                    np.testing.assert_array_equal(got, live, err_msg=f"checkpoint t={t} e={e}")
                else:
                    np.testing.assert_array_equal(got[:W - nod], live[:W - nod], err_msg=f"checkpoint t={t} e={e}")
                ro.tok_ck[slot] = got.copy()
                counts["saves"] += 1
            if ro.pushed_slot >= 0:   # event written: buffer slot = the checkpoint, live obs = its obs
                np.testing.assert_array_equal(store[e, keep + ro.pushed_slot], tok, err_msg=f"push t={t} e={e}")
                np.testing.assert_array_equal(live[W - nod:], tok[W - nod:], err_msg=f"push obs t={t} e={e}")
                ro.tok_buf[ro.pushed_slot] = tok
                counts["pushes"] += 1
            if restored:              # replayed episode: live state = the event (its own episode counter kept)
                got = pack_live(hv, n, e)
                off = n * (N.NF + N.NI + 3) + N.E_EPISODE
                want = tok.copy()
                want[off] = got[off]
                np.testing.assert_array_equal(got, want, err_msg=f"restore t={t} e={e}")
                counts["replays"] += 1
            want_ri = [ro.active, ro.saved, ro.ck_n, ro.ck_head, ro.buf_n, ro.buf_idx, ro.last_add, ro.episodes,
                       ro.replayed, ro.index_err, len(ro.hist), None, ro.last_slot, ro.pushed_slot]
            for f, v in enumerate(want_ri):
                if v is not None:
                    assert ri[f, e] == v, (t, e, f, ri[f, e], v)
            assert list(perm[:, e]) == ro.perm, (t, e)
            assert crash[e] == ro.crash, (t, e)
        counts["active"] = int(ri[N.R_ACTIVE].sum())
    # the run covered activation, checkpoints, events and replays in every env family
    assert counts["active"] == E, counts
    assert counts["saves"] > 200 and counts["pushes"] > 20 and counts["replays"] > 20, counts
    assert int(R["ri"][N.R_INDEX_ERR].sum()) == 0
    env.close()


def test_replay_off_leaves_step_unchanged():
    """Enabling replay changes nothing before the first episode ends (no activation yet)."""
    cfg = QuadSwarmConfig(num_envs=64, num_agents=8, seed=3)
    a_env, b_env = QuadSwarmEnv(cfg), QuadSwarmEnv(cfg)
    b_env.enable_replay(0.75)
    a_env.reset()
    b_env.reset()
    rng = np.random.default_rng(1)
    for _ in range(20):
        a = torch.from_numpy(rng.uniform(-1, 1, (a_env.I, 4)).astype(np.float32)).cuda()
        oa, ra, _, _ = a_env.step(a)
        ob, rb, _, _ = b_env.step(a)
        assert torch.equal(oa, ob) and torch.equal(ra, rb)
    assert int(b_env.replay["ri"][N.R_HIST_N].max()) == 1   # the explicit reset's history entry
    b_env.disable_replay()
    assert b_env.replay is None
