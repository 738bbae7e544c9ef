#!/usr/bin/env python
"""Diagnostic: per-phase cycle shares of the step kernel from s_memtime stamps (QS_STAMPS build).

    make -C quad-swarm-rl-stable-baselines3_amd stamps && python tools/phase_stamps.py
Stamps force memory waits at phase boundaries, so read the SHARES, not the total."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("QUADSWARM_LIB", os.path.join(ROOT, "quad-swarm-rl-stable-baselines3_amd", "quadswarm_amd", "lib",
                                           "libquadswarm_stamps.so"))
sys.path.insert(0, os.path.join(ROOT, "quad-swarm-rl-stable-baselines3_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from quadswarm_amd import QuadSwarmConfig, _native as N  # noqa: E402
from quadswarm_amd.env import QuadSwarmEnv  # noqa: E402

NAMES = ["launch->loads issued", "loads + draws", "OU+physics+reward", "collisions+proximity",
         "impulses+scenario+state store", "tile refresh", "self obs (sensor noise)", "neighbour obs", "done path+sync",
         "obs tile store", "env ints + guard", "replay tail"]


def main():
    cfg = QuadSwarmConfig(num_envs=int(os.environ.get("QS_E", 4096)), num_agents=int(os.environ.get("QS_N", 8)),
                          specialize=False)   # the stamps live in the generic kernels of this build
    env = QuadSwarmEnv(cfg)
    env.reset()
    a = torch.rand(env.I, 4, device="cuda") * 2 - 1
    for _ in range(60):
        env.step(a)
    torch.cuda.synchronize()
    L = N.lib()
    L.qs_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    npad = 1 << (cfg.num_agents - 1).bit_length()
    epb = 64 // (npad * min(4, 64 // npad))          # flavor-B step geometry (qs::StepGeo, QS_QB = 4)
    nb = min((cfg.num_envs + epb - 1) // epb, 65536)
    buf = np.zeros(65536 * 16, np.uint64)
    assert L.qs_debug_stamps(buf.ctypes.data, buf.size) == 0
    rt = buf.reshape(65536, 16)[:nb, 12:14].astype(np.int64)
    t0 = rt[:, 0].min()
    s_, e_ = (rt[:, 0] - t0) * 10, (rt[:, 1] - t0) * 10   # ns (s_memrealtime = 100 MHz)
    print(f"launch timeline (ns from first wave start): start p50 {np.median(s_):.0f} p90 {np.percentile(s_, 90):.0f} "
          f"max {s_.max():.0f}; end p10 {np.percentile(e_, 10):.0f} p50 {np.median(e_):.0f} p90 "
          f"{np.percentile(e_, 90):.0f} max {e_.max():.0f}; wave lifetime p50 {np.median(e_ - s_):.0f}")
    st = buf.reshape(65536, 16)[:nb, :12].astype(np.int64)
    d = np.diff(st, axis=1)
    tot = st[:, 11] - st[:, 0]
    print(f"blocks {nb}; wave lifetime cycles: median {np.median(tot):.0f}  p90 {np.percentile(tot, 90):.0f}")
    print(f"block start skew (cycles): {st[:, 0].max() - st[:, 0].min()}; end skew {st[:, 11].max() - st[:, 11].min()}")
    for k in range(11):
        print(f"  {NAMES[k + 1]:28s} {np.median(d[:, k]):8.0f} cycles  {100 * np.median(d[:, k]) / np.median(tot):5.1f} %")
    slow = np.argsort(e_)[-max(1, nb // 100):]   # the last 1 % of waves to finish: what holds the launch open
    print(f"slowest 1% of waves (end >= {e_[slow].min():.0f} ns): lifetime cycles median {np.median(tot[slow]):.0f}, "
          f"start ns median {np.median(s_[slow]):.0f}")
    for k in range(11):
        print(f"  {NAMES[k + 1]:28s} {np.median(d[slow, k]):8.0f} cycles (max {d[slow, k].max():.0f})")


if __name__ == "__main__":
    main()
