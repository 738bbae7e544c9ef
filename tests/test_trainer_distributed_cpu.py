"""world_size-2 gloo tests of the rank-correct training hooks (VERDICT r04 "missing #1"):

* DeviceCurriculum under data parallelism: the two ranks see different episode outcomes, all-gather them every env
  step (rank-major = the global env order of the reference's one VecEnv) and both end with exactly the window,
  success rate, radius and reduction count that the reference's CurriculumCallback._on_step
  (swarm_rl/custom_callbacks.py:441-468, restated in oracle/curriculum_oracle.py) computes over the concatenated
  outcomes; every env of both ranks carries that radius.  The curriculum update itself is the host restatement
  here (no HIP device on CPU; the HIP kernel, qs_curriculum_step / _step_all, is checked against the same
  restatement in tests/test_gpu_trainer.py) -- what is tested is the gather and that every rank runs the same update.
* num_timesteps counts both ranks' agents (learn(total_timesteps) stops at the global count).
* a collective checkpoint (one file, both ranks' env shards) loaded into fresh trainers on both ranks reproduces
  the next iteration bitwise; a checkpoint of another world size is refused.

CPU stand-in env (flavor-A surface: reset_info, set_capture_radius, get/set_state) + oracle GAE."""
import io
import os
import socket
import struct

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from curriculum_oracle import CurriculumOracle
from quadswarm_amd import _native as NAT
from quadswarm_amd.callbacks import CheckpointCallback, DeviceCurriculum, TrainerCallback
from quadswarm_amd.ppo import PPOConfig, PPOTrainer, SwarmActorCritic
from test_ppo_cpu import gae_oracle_torch, sb_cfg


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _Cfg:
    flavor = "A"


class ToyEnvA:
    """E envs x N agents; every env ends an episode after its own length (3..7 steps, per rank and env) with a
    success pattern that differs between ranks; reset_info as the device env writes it (0 none, 1 / 2)."""

    def __init__(self, E=6, N=4, od=28, rank=0, seed=0):
        self.E, self.N, self.I, self.obs_dim, self.act_dim = E, N, E * N, od, 2
        self.cfg = _Cfg()
        self.rank = rank
        self.g = torch.Generator().manual_seed(seed)
        self.t = np.zeros(E, dtype=np.int64)
        self.ep = np.zeros(E, dtype=np.int64)
        self.x = torch.zeros(self.I, od)
        self.reset_info = torch.zeros(E, dtype=torch.uint8)
        self.capture = np.full(E, np.nan)
        self.obs = None

    def _len(self, e):
        return 3 + (e * 7 + self.rank * 3 + int(self.ep[e])) % 5

    def reset(self):
        self.x = torch.randn(self.I, self.obs_dim, generator=self.g)
        self.t[:] = 0
        self.reset_info.zero_()
        return self.x

    def step(self, a):
        self.x = self.x.clone()
        self.x[:, :2] += 0.1 * a
        rew = -self.x[:, :2].norm(dim=1)
        self.t += 1
        done = np.zeros(self.I, dtype=np.uint8)
        ri = np.zeros(self.E, dtype=np.uint8)
        for e in range(self.E):
            if self.t[e] >= self._len(e):
                # rank 0 succeeds mostly on even episodes, rank 1 mostly on odd ones
                ok = (int(self.ep[e]) + e + self.rank) % 3 != 0 if self.rank == 0 else (int(self.ep[e]) * 5 + e) % 4 == 1
                ri[e] = 2 if ok else 1
                done[e * self.N:(e + 1) * self.N] = 1
                self.t[e] = 0
                self.ep[e] += 1
                self.x[e * self.N:(e + 1) * self.N] = torch.randn(self.N, self.obs_dim, generator=self.g)
        self.reset_info.copy_(torch.from_numpy(ri))
        return self.x, rew, torch.from_numpy(done), self.x

    def set_capture_radius(self, v):
        self.capture[:] = v

    def get_state(self):
        b = io.BytesIO()
        gs = self.g.get_state().numpy().tobytes()
        b.write(struct.pack("<q", len(gs)) + gs)
        for arr in (self.t, self.ep, self.capture, self.x.numpy(), self.reset_info.numpy()):
            raw = np.ascontiguousarray(arr).tobytes()
            b.write(struct.pack("<q", len(raw)) + raw)
        return b.getvalue()

    def set_state(self, blob):
        off = 0

        def take():
            nonlocal off
            (n,) = struct.unpack_from("<q", blob, off)
            off += 8
            r = blob[off:off + n]
            off += n
            return r
        self.g.set_state(torch.frombuffer(bytearray(take()), dtype=torch.uint8))
        self.t = np.frombuffer(take(), dtype=np.int64).copy()
        self.ep = np.frombuffer(take(), dtype=np.int64).copy()
        self.capture = np.frombuffer(take(), dtype=np.float64).copy()
        self.x = torch.from_numpy(np.frombuffer(take(), dtype=np.float32).copy()).view(self.I, self.obs_dim)
        self.reset_info = torch.from_numpy(np.frombuffer(take(), dtype=np.uint8).copy())

    def get_param(self, k):
        raise NAT.QuadSwarmError(k)


def host_curriculum_step(trainer, state, reset_all):
    """The curriculum update on the host (oracle restatement) on the qs_curriculum struct bytes `state`, writing the
    new radius into this rank's envs -- what qs_curriculum_step_all does on the device."""
    c = NAT.QsCurriculum.from_buffer_copy(bytes(state.numpy().tobytes()))
    o = CurriculumOracle(c.radius, c.sr_threshold, c.decay, c.window)
    o.past[:] = list(c.past)[:c.window]
    o.window_i, o.success_rate = c.window_i, c.success_rate
    rows = (reset_all if reset_all is not None else trainer.env.reset_info).numpy()
    if o.step(rows.tolist()):
        c.history[c.n_shrinks % NAT.CUR_MAX_HIST] = o.radius
        c.n_shrinks += 1
        trainer.env.set_capture_radius(np.float32(o.radius))
    c.radius, c.success_rate, c.window_i = o.radius, o.success_rate, o.window_i
    for k in range(c.window):
        c.past[k] = o.past[k]
    state.copy_(torch.frombuffer(bytearray(bytes(c)), dtype=torch.uint8))


class Rows(TrainerCallback):
    def __init__(self):
        self.rows = []

    def on_step(self, ctx):
        self.rows.append(ctx.reset_info.clone())
        return True


def _trainer(rank, seed, n_steps=8):
    torch.manual_seed(100 * seed + rank)     # different init per rank: the trainer broadcasts rank 0's
    _, pc = sb_cfg(rnn_num_layers=2, rnn_size=32, neighbor_hidden_size=16)
    pol = SwarmActorCritic(pc)
    env = ToyEnvA(rank=rank, seed=seed * 10 + rank)
    tr = PPOTrainer(env, pol, PPOConfig(n_steps=n_steps, batch_size=48, n_epochs=1), device="cpu",
                    gae_fn=gae_oracle_torch, seed=7 + rank)
    return env, tr


def _guarded(fn):
    """A failing rank reports its exception instead of leaving the parent waiting on the queue."""
    def run(rank, *a):
        q = a[-1]
        try:
            fn(rank, *a)
        except BaseException as e:   # noqa: BLE001
            import traceback
            q.put((rank, "error", traceback.format_exc()))
            raise
    return run


def _get(q, n):
    out = [q.get(timeout=300) for _ in range(n)]
    errs = [r for r in out if len(r) == 3 and r[1] == "error"]
    assert not errs, errs[0][2]
    return sorted(out, key=lambda r: r[0])


def _curriculum_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    env, tr = _trainer(rank, seed=1)
    cur = DeviceCurriculum(capture_radius_sr=0.4, capture_radius_decay=0.9, initial_capture_radius=2.0,
                           window_size=10, verbose=0, step_fn=host_curriculum_step)
    rec = Rows()
    # 5 iterations x 8 steps x (2 ranks x 24 agents)
    tr.learn(5 * 8 * world * env.I, callback=[cur, rec])
    rows = torch.stack(rec.rows)                       # [steps, E] this rank's outcomes
    allr = [torch.empty_like(rows) for _ in range(world)]
    dist.all_gather(allr, rows)
    c = cur.read()
    q.put((rank, tr.num_timesteps, tr.env_steps, [r.numpy() for r in allr],
           dict(radius=c.radius, success_rate=c.success_rate, window_i=c.window_i, n_shrinks=c.n_shrinks,
                past=list(c.past)[:c.window]), env.capture.copy()))
    dist.barrier()
    dist.destroy_process_group()


def _guarded_curriculum(*a):
    _guarded(_curriculum_worker)(*a)


def test_two_rank_curriculum_is_one_curriculum_over_all_envs():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_guarded_curriculum, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = _get(q, 2)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, ts0, steps0, rows, c0, cap0), (_, ts1, steps1, _, c1, cap1) = res
    assert steps0 == steps1 == 40
    assert ts0 == ts1 == 40 * 2 * 24                 # global num_timesteps: both ranks' agents
    r0, r1 = rows
    assert not np.array_equal(r0, r1)                # the ranks saw different outcomes
    # the reference's one callback over the global env order (rank 0's envs, then rank 1's), step by step
    o = CurriculumOracle(2.0, 0.4, 0.9, window=10)
    for t in range(r0.shape[0]):
        o.step(np.concatenate([r0[t], r1[t]]).tolist())
    assert len(o.history) >= 2                        # the radius shrank more than once
    for c in (c0, c1):
        assert c["n_shrinks"] == len(o.history) and c["window_i"] == o.window_i
        assert c["radius"] == o.radius and c["success_rate"] == o.success_rate
        assert c["past"] == list(o.past)
    assert (cap0 == np.float32(o.radius)).all() and (cap1 == np.float32(o.radius)).all()
    # a curriculum per rank (the defect this fixes) would have diverged on these outcomes
    own = [CurriculumOracle(2.0, 0.4, 0.9, window=10) for _ in range(2)]
    for t in range(r0.shape[0]):
        own[0].step(r0[t].tolist())
        own[1].step(r1[t].tolist())
    assert (own[0].radius, own[0].window_i) != (own[1].radius, own[1].window_i)


def _resume_worker(rank, world, port, path, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n_steps = 8
    env, tr = _trainer(rank, seed=2, n_steps=n_steps)
    cur = DeviceCurriculum(0.6, 0.9, 2.0, window_size=10, verbose=0, step_fn=host_curriculum_step)
    ck = CheckpointCallback(save_freq=n_steps, save_path=path, name_prefix="quad_swarm")
    per_it = n_steps * world * env.I
    tr.learn(2 * per_it, callback=[cur, ck])
    want_w = torch.cat([p.detach().flatten() for p in tr.policy.parameters()])
    want_env = env.get_state()
    want_rew = tr.storage.rewards.clone()
    want_cur = bytes(cur.read())

    env2, tr2 = _trainer(rank, seed=9, n_steps=n_steps)      # other weights and env draws
    cur2 = DeviceCurriculum(0.6, 0.9, 2.0, window_size=10, verbose=0, step_fn=host_curriculum_step)
    ck2 = CheckpointCallback(save_freq=n_steps, save_path=os.path.join(path, "b"), name_prefix="quad_swarm")
    c = tr2.load(ck.saved[0], callbacks=[cur2, ck2])
    loaded = (c["world_size"], len(c["shards"]), [s["rank"] for s in c["shards"]], tr2.num_timesteps)
    tr2.learn(2 * per_it, callback=[cur2, ck2])
    got_w = torch.cat([p.detach().flatten() for p in tr2.policy.parameters()])
    ok = dict(weights=torch.equal(want_w, got_w), env=env2.get_state() == want_env,
              rewards=torch.equal(want_rew, tr2.storage.rewards), curriculum=bytes(cur2.read()) == want_cur)
    q.put((rank, [os.path.basename(p) for p in ck.saved], loaded, ok))
    dist.barrier()
    dist.destroy_process_group()


def _guarded_resume(*a):
    _guarded(_resume_worker)(*a)


def test_two_rank_checkpoint_resume_is_bitwise(tmp_path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_guarded_resume, args=(r, 2, port, str(tmp_path), q)) for r in range(2)]
    for p in procs:
        p.start()
    res = _get(q, 2)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    per_it = 8 * 2 * 24
    for rank, saved, loaded, ok in res:
        assert saved == [f"quad_swarm_{per_it}_steps.pt", f"quad_swarm_{2 * per_it}_steps.pt"]
        assert loaded == (2, 2, [0, 1], per_it)
        assert all(ok.values()), (rank, ok)
    # one file per checkpoint (rank 0 writes it), holding both shards; a single-rank trainer refuses it
    assert sorted(os.listdir(tmp_path)) == sorted(["b", f"quad_swarm_{2 * per_it}_steps.pt", f"quad_swarm_{per_it}_steps.pt"])
    env, tr = _trainer(0, seed=2)
    try:
        tr.load(str(tmp_path / f"quad_swarm_{per_it}_steps.pt"))
    except ValueError as e:
        assert "2 ranks" in str(e)
    else:
        raise AssertionError("a 2-rank checkpoint loaded into a 1-rank trainer")


def _eval_worker(rank, world, port, path, q):
    """only rank 0 has an eval env (EvalCallback's documented data-parallel use); DeviceCurriculum must
    still give every rank an evaluator, or rank 0's evaluation broadcast / best-model save would wait forever."""
    from quadswarm_amd.callbacks import EvalCallback
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n_steps = 8
    env, tr = _trainer(rank, seed=3, n_steps=n_steps)
    eenv = ToyEnvA(E=2, N=4, rank=0, seed=77) if rank == 0 else None
    cur = DeviceCurriculum(0.6, 0.9, 2.0, window_size=10, verbose=0, step_fn=host_curriculum_step,
                           eval_env=eenv, eval_freq=4, n_eval_episodes=4)
    ev = EvalCallback(eenv, n_eval_episodes=4, eval_freq=n_steps, best_model_save_path=os.path.join(path, "best"),
                      verbose=0)
    seen = []

    class Watch(TrainerCallback):
        def on_iteration_end(self, trainer):
            seen.append((trainer.num_timesteps, len(ev.best_saved), os.path.exists(os.path.join(path, "best",
                                                                                               "best_model.pt"))))
    tr.learn(3 * n_steps * world * env.I, callback=[cur, ev, Watch()])
    sd = cur.state_dict()
    q.put((rank, cur.evaluator is not None, sorted(sd), sd.get("eval"), ev.state_dict(), seen))
    dist.barrier()
    dist.destroy_process_group()


def _guarded_eval(*a):
    _guarded(_eval_worker)(*a)


def test_two_rank_evaluation_with_an_eval_env_on_rank_0_only(tmp_path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_guarded_eval, args=(r, 2, port, str(tmp_path), q)) for r in range(2)]
    for p in procs:
        p.start()
    res = _get(q, 2)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, has0, keys0, cev0, ev0, seen0), (_, has1, keys1, cev1, ev1, seen1) = res
    assert has0 and has1                         # rank 1 got an evaluator without an eval env
    assert keys0 == keys1 == ["eval", "qs_curriculum", "seen"]
    assert cev0 == cev1 and cev0["n_calls"] == 3 * 8    # same evaluation count and broadcast rewards
    assert ev0 == ev1 and np.isfinite(ev0["best_mean_reward"])
    # the best model is written at an iteration boundary (collective), visible to both ranks there
    assert seen0 == seen1 and seen0[0][1] == 1 and seen0[0][2]
