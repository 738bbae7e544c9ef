"""The flavor-B neighbour-block comparison (tests/parity_utils.py:assert_obs_match) on the CPU: it must accept the
oracle's own obs, accept a swap of two slots whose sort keys tie, and reject a wrong slot order, a duplicated
neighbour and a neighbour that is not among the K nearest.  The "GPU" obs here are the oracle's obs with the
slots deliberately permuted (reference: neighborhood_indices / extend_obs_space, quadrotor_multi.py:328-375)."""
import types

import numpy as np
import pytest

import oracle as O
import parity_utils as PU
from quadswarm_amd import QuadSwarmConfig

SO = 18


def stepped(N=8, K=6, E=6, seed=11):
    cfg = QuadSwarmConfig(num_envs=E, num_agents=N, neighbor_visible_num=K, neighbor_obs_type="pos_vel", seed=seed)
    oenv = O.OracleEnv(PU.oracle_params(cfg), seed=seed)
    oenv.reset()
    a = np.random.default_rng(seed).uniform(-1, 1, (E * N, 4))
    obs, _, _, _ = oenv.step(a)
    return oenv, np.asarray(obs, dtype=np.float64)


def untied_pair(oenv, obs, K, tol=1e-3):
    """(row, slot a, slot b) of two selected neighbours whose keys do not tie."""
    for r in range(len(obs)):
        e, i = divmod(r, oenv.N)
        keys, _, order = PU.neighbor_slots_b(oenv, e, i, K)
        for a in range(K - 1):
            if abs(keys[order[a]] - keys[order[a + 1]]) > tol * keys[order[a + 1]] + tol:
                return r, a, a + 1
    raise AssertionError("no untied pair")


def blk(x, r, s):
    return x[r, SO + 6 * s:SO + 6 * (s + 1)]


@pytest.mark.parametrize("N,K", [(8, 6), (8, 2), (32, 6)])
def test_oracle_obs_pass_without_excuses(N, K):
    oenv, obs = stepped(N, K, E=3)
    assert PU.assert_obs_match(obs.copy(), obs, oenv, SO, K) == 0


@pytest.mark.parametrize("N,K", [(8, 6), (32, 6)])
def test_permuted_slot_order_fails(N, K):
    oenv, obs = stepped(N, K, E=3)
    r, a, b = untied_pair(oenv, obs, K)
    got = obs.copy()
    blk(got, r, a)[:], blk(got, r, b)[:] = blk(obs, r, b), blk(obs, r, a)
    with pytest.raises(AssertionError, match="where the reference's sort puts"):
        PU.assert_obs_match(got, obs, oenv, SO, K)


def test_duplicated_neighbour_fails():
    oenv, obs = stepped()
    r, a, b = untied_pair(oenv, obs, 6)
    got = obs.copy()
    blk(got, r, b)[:] = blk(obs, r, a)
    with pytest.raises(AssertionError, match="distinct neighbours"):
        PU.assert_obs_match(got, obs, oenv, SO, 6)


def test_neighbour_outside_the_k_nearest_fails():
    oenv, obs = stepped(N=8, K=2)
    K = 2
    got = obs.copy()
    for r in range(len(obs)):
        e, i = divmod(r, oenv.N)
        keys, relc, order = PU.neighbor_slots_b(oenv, e, i, K)
        far = int(np.argsort(keys, kind="stable")[-2])      # the farthest real neighbour
        if keys[far] > 1.01 * keys[order[-1]] + 1e-3:
            blk(got, r, K - 1)[:] = relc[far]
            break
    with pytest.raises(AssertionError, match="where the reference's sort puts"):
        PU.assert_obs_match(got, obs, oenv, SO, K)


def test_unmatched_slot_fails():
    oenv, obs = stepped()
    got = obs.copy()
    blk(got, 5, 2)[:] += 0.5
    with pytest.raises(AssertionError, match="no neighbour"):
        PU.assert_obs_match(got, obs, oenv, SO, 6)


def fake_env(P, V, room=10.0):
    """A one-env stand-in carrying what the checker reads (obs positions / velocities, the room)."""
    ev = types.SimpleNamespace(obs_pos=P, obs_vel=V)
    p = types.SimpleNamespace(room_hi=[room / 2] * 3, room_lo=[-room / 2] * 3)
    return types.SimpleNamespace(N=len(P), envs=[ev], p=p)


def test_tied_keys_may_swap_and_are_counted():
    # drone 0 at the origin, drones 1 and 2 mirror images (equal keys), 3..5 farther out
    P = np.array([[0, 0, 2], [1, 0, 2], [-1, 0, 2], [0, 2, 2], [0, -3, 2], [4, 0, 2]], dtype=np.float64)
    V = np.zeros_like(P)
    oenv = fake_env(P, V)
    K = 3
    keys, relc, order = PU.neighbor_slots_b(oenv, 0, 0, K)
    assert order == [1, 2, 3]
    want = np.zeros((1, SO + 6 * K))
    want[0, SO:] = relc[order].ravel()
    got = want.copy()
    got[0, SO:SO + 12] = relc[[2, 1]].ravel()          # the tied pair swapped
    before = PU.EXCUSES_B["slot_order_tie"]
    assert PU.assert_obs_match(got, want, oenv, SO, K, max_excused=1) == 1
    assert PU.EXCUSES_B["slot_order_tie"] == before + 2
    # the same swap with the tie broken by 1 cm is a wrong order
    P2 = P.copy()
    P2[2, 0] = -1.01
    oenv2 = fake_env(P2, V)
    keys2, relc2, order2 = PU.neighbor_slots_b(oenv2, 0, 0, K)
    want2 = np.zeros((1, SO + 6 * K))
    want2[0, SO:] = relc2[order2].ravel()
    got2 = want2.copy()
    got2[0, SO:SO + 12] = relc2[[2, 1]].ravel()
    with pytest.raises(AssertionError, match="where the reference's sort puts"):
        PU.assert_obs_match(got2, want2, oenv2, SO, K)


def test_excused_rows_are_bounded():
    P = np.array([[0, 0, 2], [1, 0, 2], [-1, 0, 2], [0, 2, 2]], dtype=np.float64)
    oenv = fake_env(P, np.zeros_like(P))
    K = 2
    _, relc, order = PU.neighbor_slots_b(oenv, 0, 0, K)
    want = np.zeros((1, SO + 6 * K))
    want[0, SO:] = relc[order].ravel()
    got = want.copy()
    got[0, SO:] = relc[[2, 1]].ravel()
    with pytest.raises(AssertionError, match="excused by sort-key ties"):
        PU.assert_obs_match(got, want, oenv, SO, K, max_excused=0)
