#!/usr/bin/env python
"""Diagnostic: per-phase cycle shares of the step kernel from s_memtime stamps (QS_STAMPS build).

    make -C quad-swarm-rl-stable-baselines3_amd stamps && python tools/phase_stamps.py
Stamps force memory waits at phase boundaries, so read the SHARES, not the total."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["QUADSWARM_LIB"] = os.path.join(ROOT, "quad-swarm-rl-stable-baselines3_amd", "quadswarm_amd", "lib",
                                           "libquadswarm_stamps.so")
sys.path.insert(0, os.path.join(ROOT, "quad-swarm-rl-stable-baselines3_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from quadswarm_amd import QuadSwarmConfig, _native as N  # noqa: E402
from quadswarm_amd.env import QuadSwarmEnv  # noqa: E402

NAMES = ["launch->loads issued", "state loads", "OU+physics+reward", "collisions+proximity", "forces/impulses",
         "tile refresh", "self obs (sensor noise)", "neighbour obs", "done path+sync", "obs tile store",
         "state stores", "counter atomic"]


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
    nb = (cfg.num_envs + (64 // 8) - 1) // (64 // 8) if cfg.num_agents == 8 else 512
    buf = np.zeros(65536 * 16, np.uint64)
    assert L.qs_debug_stamps(buf.ctypes.data, buf.size) == 0
    st = buf.reshape(65536, 16)[:nb, :12].astype(np.int64)
    d = np.diff(st, axis=1)
    tot = st[:, 11] - st[:, 0]
    print(f"blocks {nb}; wave lifetime cycles: median {np.median(tot):.0f}  p90 {np.percentile(tot, 90):.0f}")
    print(f"block start skew (cycles): {st[:, 0].max() - st[:, 0].min()}; end skew {st[:, 11].max() - st[:, 11].min()}")
    for k in range(11):
        print(f"  {NAMES[k + 1]:28s} {np.median(d[:, k]):8.0f} cycles  {100 * np.median(d[:, k]) / np.median(tot):5.1f} %")


if __name__ == "__main__":
    main()
