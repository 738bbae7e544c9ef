#!/usr/bin/env python
"""Diagnostic: per-phase cycle budget of a step kernel from s_memtime stamps (QS_STAMPS build).

    make -C quad-swarm-rl-stable-baselines3_amd stamps && python tools/phase_stamps.py [config]

The stamps library compiles the specialised (hipRTC) kernels with -DQS_STAMPS=1, i.e. the kernels the bench runs
plus the stamps.  Flavor B stamps phase boundaries (slots 0-11); flavor A sums each phase of its 8-tick loop over
the ticks (slots 0-9).  Slots 12 / 13 are the wave's s_memrealtime start / end (the launch timeline).  A stamp
waits for its own counter read only (s_waitcnt lgkmcnt(0)): read the SHARES; the total runs a little long."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("QUADSWARM_LIB", os.path.join(ROOT, "quad-swarm-rl-stable-baselines3_amd", "quadswarm_amd", "lib",
                                           "libquadswarm_stamps.so"))
os.environ["QS_JIT_OPTS"] = (os.environ.get("QS_JIT_OPTS", "") + " -DQS_STAMPS=1").strip()
sys.path.insert(0, os.path.join(ROOT, "quad-swarm-rl-stable-baselines3_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

NAMES_B = ["launch->loads issued", "loads + draws", "OU+physics+reward", "collisions+proximity",
           "impulses+scenario+state store", "tile refresh", "self obs (sensor noise)", "neighbour obs", "done path+sync",
           "obs tile store", "env ints + guard", "replay tail"]
NAMES_A = ["loads", "controller (x ticks)", "OU draw (x ticks)", "physics 2 substeps (x ticks)",
           "stats collisions (x ticks)", "capture + done (x ticks)", "downwash/target/scenario (x ticks)",
           "counters + final obs", "done path", "obs tile + stores"]


def main():
    import bench
    from quadswarm_amd import _native as N
    from quadswarm_amd.env import QuadSwarmEnv

    config = sys.argv[1] if len(sys.argv) > 1 else "c3"
    cfg = bench.make_cfg(bench.CONFIGS[config], seed=0, specialize=True)
    env = QuadSwarmEnv(cfg)
    assert env.specialized, "the stamps run on the specialised kernels"
    env.reset()
    a = torch.rand(env.I, cfg.act_dim, device="cuda") * 2 - 1
    for _ in range(60):
        env.step(a)
    torch.cuda.synchronize()
    L = N.lib()
    L.qs_debug_stamps_h.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    npad = 1 << (cfg.num_agents - 1).bit_length()
    qd = 2 if cfg.flavor == "A" else 4
    q = qd if npad * qd <= 64 else 64 // npad
    epb = 64 // (npad * q)
    nb = min((cfg.num_envs + epb - 1) // epb, 65536)
    buf = np.zeros(65536 * 16, np.uint64)
    assert L.qs_debug_stamps_h(env._h, buf.ctypes.data, buf.size) == 0, L.qs_last_error()
    st = buf.reshape(65536, 16)[:nb].astype(np.int64)
    rt = st[:, 12:14]
    t0 = rt[:, 0].min()
    s_, e_ = (rt[:, 0] - t0) * 10, (rt[:, 1] - t0) * 10   # ns (s_memrealtime = 100 MHz)
    print(f"{config}: {nb} waves; launch timeline (ns from the first wave's start): start p50 {np.median(s_):.0f} "
          f"p90 {np.percentile(s_, 90):.0f} max {s_.max():.0f}; end p10 {np.percentile(e_, 10):.0f} p50 "
          f"{np.median(e_):.0f} p90 {np.percentile(e_, 90):.0f} max {e_.max():.0f}; wave lifetime p50 "
          f"{np.median(e_ - s_):.0f}")
    if cfg.flavor == "A":
        d = st[:, :10]
        names = NAMES_A
    else:
        d = np.diff(st[:, :12], axis=1)
        names = NAMES_B[1:]
    tot = d.sum(1)
    print(f"wave cycles between the first and last stamp: median {np.median(tot):.0f}  p90 {np.percentile(tot, 90):.0f}")
    for k, name in enumerate(names):
        print(f"  {name:36s} {np.median(d[:, k]):8.0f} cycles  {100 * np.median(d[:, k]) / np.median(tot):5.1f} %")
    slow = np.argsort(e_)[-max(1, nb // 100):]   # the last 1 % of waves to finish: what holds the launch open
    print(f"slowest 1% of waves (end >= {e_[slow].min():.0f} ns): cycles median {np.median(tot[slow]):.0f}, "
          f"start ns median {np.median(s_[slow]):.0f}")
    for k, name in enumerate(names):
        print(f"  {name:36s} {np.median(d[slow, k]):8.0f} cycles (max {d[slow, k].max():.0f})")


if __name__ == "__main__":
    main()
