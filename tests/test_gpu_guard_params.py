"""Boundary behaviour of the C ABI that sits around the step kernels:

* the non-finite guard (qs_counters): the reference raises on a NaN reward (quadrotor_single.py:87-90);
  the batched step counts non-finite rewards, drone states and observation values instead, exactly;
* runtime parameters live in device memory, so they reach launches replayed from captured hipGraphs:
  the Philox seed (qs_set_param("seed"), GpuQuadVecEnv.seed) and the reward coefficients, including the
  rew_crash the fused experience-replay tail reads (specialised == generic kernels, bitwise);
* bench.py's launch path (env blocks built under their own non-blocking streams, graphs of min(--graph,
  --steps) steps plus a remainder graph) gives the one handle's results bitwise.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no HIP device", allow_module_level=True)

from quadswarm_amd import QuadSwarmConfig  # noqa: E402
from quadswarm_amd import _native as N  # noqa: E402
from quadswarm_amd.env import QuadSwarmEnv  # noqa: E402


def _acts(env, g):
    return (torch.rand(env.I, env.act_dim, device="cuda", generator=g) * 2 - 1).contiguous()


@pytest.mark.parametrize("flavor", ["B", "A"])
def test_nonfinite_guard_counts(flavor):
    if flavor == "B":
        cfg = QuadSwarmConfig(num_envs=64, num_agents=8, neighbor_visible_num=6, seed=2)
    else:
        cfg = QuadSwarmConfig.sb_train(num_envs=64, num_agents=8, seed=2)
    env = QuadSwarmEnv(cfg)
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(1)
    for _ in range(5):
        env.step(_acts(env, g))
    assert env.counters() == {"nonfinite_obs": 0, "nonfinite_rew": 0, "nonfinite_state": 0}

    if flavor == "B":
        # a NaN action: RawControl clips it away from the motors (fmax(NaN, -1) = -1), but the effort
        # term of compute_reward_weighted reads the raw action -> exactly one NaN reward
        a = _acts(env, g)
        a[77, 2] = float("nan")
        _, rew, _, _ = env.step(a)
        torch.cuda.synchronize()
        assert torch.isnan(rew).sum().item() == 1
        assert env.counters() == {"nonfinite_obs": 0, "nonfinite_rew": 1, "nonfinite_state": 0}
    env.reset_counters()
    assert env.counters() == {"nonfinite_obs": 0, "nonfinite_rew": 0, "nonfinite_state": 0}

    # a drone whose attitude went non-finite (a non-finite position or velocity is sanitised by the room
    # clip and the wall bounce, like in the reference): counted as a state, its reward (flavor B's orient
    # term reads R22; flavor A's capture reward does not), and every non-finite obs value the step wrote
    g0 = 8 * 5 + 3
    env.state[N.F_ROT + 4, g0] = float("nan")
    a = _acts(env, g)
    obs, rew, _, _ = env.step(a)
    torch.cuda.synchronize()
    c = env.counters()
    want_obs = int((~torch.isfinite(obs)).sum().item())
    assert c["nonfinite_state"] == int((~torch.isfinite(env.state[:N.F_ROT_DAMP])).any(0).sum().item()) >= 1
    # (flavor B: the NaN attitude makes the thrust NaN, the room clip puts the drone on the floor, whose
    # reset of the attitude to yaw-only leaves R22 = 1: the reward stays finite, as in the reference)
    assert c["nonfinite_rew"] == int((~torch.isfinite(rew)).sum().item())
    assert c["nonfinite_obs"] == want_obs >= (1 if flavor == "B" else 0)
    # only the poisoned env is affected
    bad_envs = set((torch.nonzero(~torch.isfinite(obs).all(1)).flatten() // 8).tolist())
    assert bad_envs <= {5}


def test_guard_counts_inside_graph():
    cfg = QuadSwarmConfig(num_envs=32, num_agents=8, seed=9)
    env = QuadSwarmEnv(cfg)
    env.reset()
    a = _acts(env, torch.Generator(device="cuda").manual_seed(2))
    a[5, 0] = float("nan")    # one NaN reward per step
    env.step(a)
    torch.cuda.synchronize()
    env.reset_counters()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for _ in range(4):
            env.step(a)
    gr.replay()
    gr.replay()
    torch.cuda.synchronize()
    assert env.counters()["nonfinite_rew"] == 8


@pytest.mark.parametrize("flavor", ["B", "A"])
def test_seed_change_reaches_captured_graph(flavor):
    mk = (lambda **k: QuadSwarmConfig(num_envs=64, num_agents=8, **k)) if flavor == "B" else \
        (lambda **k: QuadSwarmConfig.sb_train(num_envs=64, num_agents=8, **k))
    x = QuadSwarmEnv(mk(seed=0))
    x.reset()
    y = QuadSwarmEnv(mk(seed=7))
    y.set_state(x.get_state())
    a = _acts(x, torch.Generator(device="cuda").manual_seed(4))
    x.step(a)
    torch.cuda.synchronize()
    y.set_state(x.get_state())
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for _ in range(3):
            x.step(a)
    x.set_param("seed", 7)          # after the capture
    assert x.get_param("seed") == 7
    gr.replay()
    for _ in range(3):
        y.step(a)
    torch.cuda.synchronize()
    assert torch.equal(x.obs, y.obs) and torch.equal(x.state, y.state) and torch.equal(x.rew, y.rew)


@pytest.mark.parametrize("mode,prob", [("mix", 0.75), ("mix", 0.0), ("static_same_goal", 0.75)])
def test_specialised_replay_tail_reads_live_rew_crash(mode, prob):
    def mk(spec):
        return QuadSwarmConfig(num_envs=128, num_agents=8, seed=3, episode_duration=1.0, quads_mode=mode,
                               replay_buffer_sample_prob=prob, specialize=spec)
    gen, spc = QuadSwarmEnv(mk(False)), QuadSwarmEnv(mk(True))
    assert spc.specialized and not gen.specialized
    for e in (gen, spc):
        e.reset()
        e.set_param("rew_crash", 3.0)
    g = torch.Generator(device="cuda").manual_seed(8)
    first = None
    for t in range(250):
        a = (0.1 * _acts(gen, g) - 0.9).contiguous()   # low thrust: drones reach the floor (rew_crash)
        for e in (gen, spc):
            e.step(a)
        if first is None:
            for k in ("state", "obs", "rew"):
                x, y = getattr(gen, k), getattr(spc, k)
                same = (x == y) | (torch.isnan(x) & torch.isnan(y))
                if not bool(same.all()):
                    bad = torch.nonzero(~same)[:6].tolist()
                    first = (t, k, bad, [(float(x[tuple(i)]), float(y[tuple(i)])) for i in bad[:3]])
                    break
    torch.cuda.synchronize()
    if prob > 0:
        assert (gen.replay["hist"] != 0).any()
        for k in ("ri", "crash", "hist", "perm", "nrep"):
            assert torch.equal(gen.replay[k], spc.replay[k]), k
    assert first is None, first


@pytest.mark.parametrize("steps,chunk", [(25, 20), (20, 100)])
def test_bench_block_graphs_equal_one_handle(steps, chunk):
    import bench

    dev = torch.device("cuda", 0)
    E, S, Nd = 256, 4, 8
    kw = dict(num_envs=E, num_agents=Nd, neighbor_visible_num=6, seed=0, episode_duration=0.1)
    one = QuadSwarmEnv(QuadSwarmConfig(**kw))
    one.reset()
    actions = _acts(one, torch.Generator(device="cuda").manual_seed(1234))
    streams, destroy = bench.raw_streams(torch, dev, S, spare=3)
    stream = torch.cuda.current_stream(dev)
    entries = []
    Eb = E // S
    for s in range(S):
        st = streams[s]
        st.wait_stream(stream)
        with torch.cuda.stream(st):
            eb = QuadSwarmEnv(QuadSwarmConfig(**dict(kw, num_envs=Eb, drone_id_offset=s * Eb * Nd)))
            eb.reset()
        entries.append((eb, actions[s * Eb * Nd:(s + 1) * Eb * Nd].contiguous(), st))
    torch.cuda.synchronize()
    blocks = bench.Blocks(torch, dev, entries, min(chunk, steps))
    blocks.prepare([steps])
    ev = blocks.timed(steps, stream)
    for _ in range(steps):
        one.step(actions)
    torch.cuda.synchronize()
    assert ev[0].elapsed_time(ev[1]) > 0
    assert blocks.replays == (2 if steps % min(chunk, steps) else 1)
    assert torch.equal(torch.cat([e.obs for e, _, _ in entries]), one.obs)
    assert torch.equal(torch.cat([e.state for e, _, _ in entries], 1), one.state)
    assert torch.equal(torch.cat([e.rew for e, _, _ in entries]), one.rew)
    for e, _, _ in entries:
        e.close()
    destroy()
