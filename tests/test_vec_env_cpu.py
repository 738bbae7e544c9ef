"""GpuQuadVecEnv's host-side infos (no GPU): StepInfos rows are memoised mutable dicts, so a wrapper's in-place
writes stick (SB3 VecNormalize rewrites infos[i]["terminal_observation"]; the reference's replay wrapper adds
keys), and terminal observations are indexed in done-row order."""
import numpy as np
import pytest

from quadswarm_amd.vec_env import StepInfos


@pytest.mark.parametrize("mode", ["plain", "goal_dist"])
def test_step_infos_rows_are_memoised_and_mutable(mode):
    n = 6
    term = np.arange(2 * 3, dtype=np.float32).reshape(2, 3)          # rows 2 and 5 finished
    gd = np.linspace(0.0, 1.0, n) if mode == "goal_dist" else None
    inf = StepInfos(n, [2, 5], term, [{"num_collisions": 1}, {"num_collisions": 2}], None, gd)
    np.testing.assert_array_equal(inf[2]["terminal_observation"], term[0])
    np.testing.assert_array_equal(inf[5]["terminal_observation"], term[1])
    assert inf[5]["episode_extra_stats"] == {"num_collisions": 2}
    for i in range(n):
        row = inf[i]
        assert inf[i] is row and inf[i - n] is row                     # the same dict on every read
        row["added_by_wrapper"] = i
        assert inf[i]["added_by_wrapper"] == i
    inf[2]["terminal_observation"] = np.zeros(3, np.float32)          # VecNormalize-style rewrite
    assert not inf[2]["terminal_observation"].any()
    assert ("terminal_observation" in inf[0]) is False
    if mode == "goal_dist":
        assert inf[3]["goal_dist"] == pytest.approx(gd[3]) and inf[3]["rewards"] == {}
    assert [r["added_by_wrapper"] for r in inf[1:4]] == [1, 2, 3]
    with pytest.raises(IndexError):
        inf[n]


def test_step_infos_lazy_resolve_once():
    calls = []

    def resolve():
        calls.append(1)
        return np.array([1]), np.ones((1, 2), np.float32), None, None, None
    inf = StepInfos(3, resolve=resolve)
    assert calls == []
    r = inf[1]
    assert inf[1] is r and calls == [1]
    assert list(inf.done_rows) == [1] and calls == [1]
