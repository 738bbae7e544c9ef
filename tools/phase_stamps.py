#!/usr/bin/env python
"""Diagnostic: per-phase cycle budget of a step kernel from s_memtime stamps (QS_STAMPS build).

    make -C quad-swarm-rl-stable-baselines3_amd stamps && python tools/phase_stamps.py [config [quads_mode]]

The stamps library compiles the specialised (hipRTC) kernels with -DQS_STAMPS=1, i.e. the kernels the bench runs
plus the stamps.  Flavor B stamps phase boundaries (slots 0-11); flavor A sums each phase of its 8-tick loop over
the ticks (slots 0-9).  Slots 12 / 13 are the wave's s_memrealtime start / end (the launch timeline), 14 / 15 its HW_ID / XCC_ID.  A stamp
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
    over = dict(bench.CONFIGS[config])
    if len(sys.argv) > 2:   # a goal scenario for the swarm configs (bench.py --quads-mode)
        over["quads_mode"] = sys.argv[2]
    cfg = bench.make_cfg(over, seed=0, specialize=True)
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
    q = qd if npad * qd <= 64 else (2 if npad >= 64 and cfg.flavor == "B" else 64 // npad)   # StepGeo / StepGeoA
    epb = max(64, npad * q) // (npad * q)
    nb = min((cfg.num_envs + epb - 1) // epb, 65536)
    NS = 32   # slots per block (QS_NSTAMP)
    buf = np.zeros(65536 * NS, np.uint64)
    assert L.qs_debug_stamps_h(env._h, buf.ctypes.data, buf.size) == 0, L.qs_last_error()
    st = buf.reshape(65536, NS)[:nb].astype(np.int64)
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
    sub = None
    if cfg.flavor == "B" and (st[:, 18] != 0).any():   # the scenario sub-phases (slots 18-21)
        # slots 19 / 20 are stamped only inside the scenario step: a kernel without one leaves them 0
        s19 = np.where(st[:, 19] != 0, st[:, 19], st[:, 18])
        seq = np.stack([st[:, 3], st[:, 18], s19, st[:, 21], st[:, 4]], axis=1)
        sub = np.diff(seq, axis=1)
        s20 = np.where(st[:, 20] != 0, st[:, 20] - s19, 0)
        sub = np.concatenate([sub, s20[:, None]], axis=1)
        sub_names = ["  forces/impulses", "  scen: tables + sync", "  scen: step (+ via)", "  state store",
                     "  (of which scen step proper)"]
    print(f"wave cycles between the first and last stamp: median {np.median(tot):.0f}  p90 {np.percentile(tot, 90):.0f}")
    for k, name in enumerate(names):
        print(f"  {name:36s} {np.median(d[:, k]):8.0f} cycles  {100 * np.median(d[:, k]) / np.median(tot):5.1f} %")
    if sub is not None:
        for k, name in enumerate(sub_names):
            print(f"  {name:36s} median {np.median(sub[:, k]):8.0f}  p90 {np.percentile(sub[:, k], 90):8.0f}  max "
                  f"{sub[:, k].max():8.0f} cycles")
    # where the waves ran: HW_ID (gfx9 layout: wave slot 3:0, SIMD 5:4, CU 11:8, SH 12, SE 15:13) + XCC_ID
    hw, xcc = st[:, 14], st[:, 15] & 0xF
    simd_key = (xcc << 16) | (((hw >> 8) & 0xFF) << 2) | ((hw >> 4) & 3)
    cu_key = simd_key >> 2
    for name, key in (("SIMD", simd_key), ("CU", cu_key)):
        u, inv, cnt = np.unique(key, return_inverse=True, return_counts=True)
        per = cnt[inv]   # waves sharing this wave's SIMD / CU
        line = ", ".join(f"{c} waves: {np.sum(cnt == c)} {name}s (wave end p50 {np.median(e_[per == c]):.0f} ns, "
                         f"max {e_[per == c].max():.0f})" for c in np.unique(cnt))
        print(f"waves per {name} ({len(u)} {name}s used): {line}")
    slot = hw & 0xF
    print("wave end by wave slot (ns): " + ", ".join(
        f"slot {s}: {np.sum(slot == s)} waves, start p50 {np.median(s_[slot == s]):.0f}, end p50 "
        f"{np.median(e_[slot == s]):.0f} p99 {np.percentile(e_[slot == s], 99):.0f} max {e_[slot == s].max():.0f}"
        for s in np.unique(slot)))
    print("wave end by XCD (ns): " + ", ".join(f"{x}: p50 {np.median(e_[xcc == x]):.0f} max {e_[xcc == x].max():.0f}"
                                              for x in np.unique(xcc)))
    slow = np.argsort(e_)[-max(1, nb // 100):]
    if cfg.flavor == "B":   # slots 16 / 17: the wave's drones on the floor / in a drone collision
        fl, co = st[:, 16], st[:, 17]
        print(f"drones per wave on the floor: mean {fl.mean():.2f} (slowest 1%: {fl[slow].mean():.2f}); in a "
              f"collision: mean {co.mean():.3f} (slowest 1%: {co[slow].mean():.3f})")
        for c in np.unique(fl)[:8]:
            print(f"  {c} on the floor: {np.sum(fl == c)} waves, end p50 {np.median(e_[fl == c]):.0f} ns")   # the last 1 % of waves to finish: what holds the launch open
    print(f"slowest 1% of waves (end >= {e_[slow].min():.0f} ns): cycles median {np.median(tot[slow]):.0f}, "
          f"start ns median {np.median(s_[slow]):.0f}")
    for k, name in enumerate(names):
        print(f"  {name:36s} {np.median(d[slow, k]):8.0f} cycles (max {d[slow, k].max():.0f})")
    if sub is not None:
        for k, name in enumerate(sub_names):
            print(f"  {name:36s} {np.median(sub[slow, k]):8.0f} cycles (max {sub[slow, k].max():.0f})")


if __name__ == "__main__":
    main()
