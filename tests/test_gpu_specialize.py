"""qs_specialize (hipRTC kernels with the parameter block baked in as constants) against the generic
kernels through the C ABI: same seeds, same actions, every output and the whole state compared over
episodes with resets.  The specialised path is what bench.py measures, so it is held to the generic
kernels' results -- which tests/test_gpu_parity*.py hold to the oracle.

Bitwise: both builds contract multiply-adds only inside source expressions (-ffp-contract=on), and
constant folding under IEEE semantics (no reassociation) does not change a result.  (With the
backend's cross-statement contraction the two builds fused different pairs and drifted by an ulp.)
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no HIP device", allow_module_level=True)

from quadswarm_amd import QuadSwarmConfig  # noqa: E402
from quadswarm_amd.env import QuadSwarmEnv  # noqa: E402

CONFIGS = {
    "c3": lambda: QuadSwarmConfig(num_envs=512, num_agents=8, neighbor_visible_num=6, episode_duration=0.3, seed=4),
    "c4": lambda: QuadSwarmConfig.c4(num_envs=512, episode_duration=0.3, seed=4),
    "c2": lambda: QuadSwarmConfig(num_envs=2048, num_agents=1, neighbor_visible_num=0, neighbor_obs_type="none",
                                  episode_duration=0.3, seed=4),
    "a8": lambda: QuadSwarmConfig.sb_train(num_envs=256, num_agents=8, seed=4, episode_duration=0.6,
                                           initial_capture_radius=1.0),
    "a4cam": lambda: QuadSwarmConfig.sb_train(num_envs=256, num_agents=4, seed=4, neighbor_visible_num=2,
                                              episode_duration=0.6),
    "n32": lambda: QuadSwarmConfig(num_envs=64, num_agents=32, neighbor_visible_num=6, episode_duration=0.3, seed=4),
}


def assert_same(a, b, what):
    a, b = a.cpu(), b.cpu()
    if torch.equal(a, b) or (a.is_floating_point() and torch.equal(torch.nan_to_num(a, 7.0), torch.nan_to_num(b, 7.0))
                             and torch.equal(a.isnan(), b.isnan())):
        return
    d = (a.double() - b.double()).abs().nan_to_num(1e9)
    raise AssertionError(f"{what}: not bitwise equal, max |diff| {d.max().item():.3g} at {int(d.argmax())}")


@pytest.mark.parametrize("name", sorted(CONFIGS))
def test_specialised_matches_generic(name):
    cfg = CONFIGS[name]()
    cfg.specialize = False
    gen = QuadSwarmEnv(cfg)
    spc = QuadSwarmEnv(CONFIGS[name]())
    spc.specialize(True)
    assert spc.specialized and not gen.specialized
    o1, o2 = gen.reset(), spc.reset()
    assert_same(o2, o1, "reset obs")
    g = torch.Generator(device="cuda").manual_seed(11)
    dones = 0
    for t in range(40):
        a = (torch.rand(gen.I, gen.act_dim, device="cuda", generator=g) * 2 - 1).contiguous()
        if t == 20:   # a runtime parameter change reaches the specialised kernel too
            for e in (gen, spc):
                e.set_param("rew_pos" if cfg.flavor == "B" else "ep_len", 2.0 if cfg.flavor == "B" else 40)
        r1 = gen.step(a)
        r2 = spc.step(a)
        for x, y, w in zip(r2, r1, ("obs", "rew", "done", "term")):
            assert_same(x, y, f"{w} step {t}")
        dones += int(r1[2].sum())
    assert_same(spc.state, gen.state, "state")
    assert torch.equal(spc.istate, gen.istate) and torch.equal(spc.env_state, gen.env_state)
    assert dones > 0


def test_specialise_toggle_and_cache():
    cfg = CONFIGS["c3"]()
    e = QuadSwarmEnv(cfg)
    assert e.specialized            # the default
    e.specialize(True)
    e.specialize(False)
    assert not e.specialized
    e.specialize(True)       # second time from the process cache
    assert e.specialized
