"""Experience-replay oracle (oracle/replay_oracle.py) vs the reference's own ExperienceReplayWrapper
(gym_art/quadrotor_multi/quad_experience_replay.py), recorded by tools/gen_golden_replay.py."""
import os

import numpy as np
import pytest

from replay_oracle import LAST_ADD_NONE, ReplayOracle, TapeDraws

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("name", ["a", "b", "c"])
def test_replay_oracle_matches_reference_wrapper(name):
    with np.load(os.path.join(GOLD, f"replay_{name}.npz")) as z:
        g = {k: z[k] for k in z.files}   # NpzFile decompresses on every access
    cf = float(g["control_freq"])
    ro = ReplayOracle(float(g["prob"]), cp_every=int(0.5 * cf), grace=int(1.5 * cf), gap=int(5 * cf))
    draws = TapeDraws(g["tape"])
    ep_len, unit = int(g["ep_len"]), float(g["crash_unit"])
    ro.explicit_reset()
    prev = tuple(g["obs0"])
    next_id = [int(g["obs0"][0])]
    n_replays = 0
    for t in range(len(g["col"])):
        tick = int(prev[1]) + 1
        done = tick > ep_len
        obs = tuple(g["obs"][t])
        live = None if done else tuple(g["live"][t])
        tok, restored = ro.step(tick, done, int(g["col"][t]), int(g["floor0"][t]), unit, draws, live)
        if tok is not None:
            n_replays += restored
            assert obs == tok, (t, obs, tok)          # the replayed / pushed checkpoint's obs is returned
            if not restored:                          # the env itself continues from the live state
                obs = live
        elif done:
            assert obs[1] == 0 and obs[0] > next_id[0], (t, obs)   # a fresh reset
        next_id[0] = max(next_id[0], obs[0])
        prev = obs
        assert ro.active == g["active"][t] and ro.saved == g["saved"][t], t
        ck = [c[0] for c in ro.ck_tokens()]
        assert ck + [0] * (6 - len(ck)) == list(g["ck"][t]), t
        buf = [b[0] for b in ro.buf_tokens()]
        assert buf + [0] * (20 - len(buf)) == list(g["buf"][t]), t
        nr = ro.buf_nrep()
        assert nr + [-1] * (20 - len(nr)) == list(g["nrep"][t]), t
        assert ro.buf_idx == g["buf_idx"][t], t
        assert max(ro.last_add, LAST_ADD_NONE) == g["last_add"][t], t
        assert ro.replayed == g["replayed"][t] and ro.episodes == g["episodes"][t], t
        assert draws.pos == g["tape_pos"][t], t
    assert n_replays == g["replayed"][-1] > 50
    assert ro.index_err == 0


def test_replay_oracle_golden_coverage():
    """The fixtures exercise delayed activation, a full buffer (buffer_idx wrap) and cleanup drops."""
    a = np.load(os.path.join(GOLD, "replay_a.npz"))
    assert 200 < int(np.argmax(a["active"] > 0)) < 6000
    for n in "abc":
        g = np.load(os.path.join(GOLD, f"replay_{n}.npz"))
        assert (g["nrep"] >= 0).sum(1).max() == 20 and g["buf_idx"].max() == 19
    c = np.load(os.path.join(GOLD, "replay_c.npz"))
    size = (c["nrep"] >= 0).sum(1)
    assert (size[1:] < size[:-1]).sum() >= 5           # cleanup removed events replayed 10 times
    assert c["nrep"].max() == 9
