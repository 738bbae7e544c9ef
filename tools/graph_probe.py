#!/usr/bin/env python
"""Where a short bench run's time goes: wall and HIP-event time of consecutive replays of one captured
20-step hipGraph of the C3 step in a fresh process, with and without hipGraphUpload before the first
replay, then again after ~0.3 s of back-to-back steps (GPU clock ramp).  Diagnostic only.

    python tools/graph_probe.py [--upload] [--steps 20]
"""
import argparse
import ctypes
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "quad-swarm-rl-stable-baselines3_amd"))
sys.path.insert(0, os.path.join(HERE, ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--upload", action="store_true")
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    import torch
    import bench
    from quadswarm_amd.env import QuadSwarmEnv
    dev = torch.device("cuda:0")
    cfg = bench.make_cfg(bench.CONFIGS["c3"], seed=0, specialize=True)
    env = QuadSwarmEnv(cfg, device=dev)
    I = cfg.num_envs * cfg.num_agents
    acts = (torch.rand(I, 4, device=dev, generator=torch.Generator(device=dev).manual_seed(1234)) * 2 - 1).contiguous()
    env.reset()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(args.steps):
            env.step(acts)
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    if args.upload:
        hip = ctypes.CDLL("libamdhip64.so")
        rc = hip.hipGraphUpload(ctypes.c_void_p(g.raw_cuda_graph_exec()), ctypes.c_void_p(stream.cuda_stream))
        torch.cuda.synchronize()
        print("upload rc", rc)

    def one(tag):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record(stream)
        g.replay()
        e1.record(stream)
        torch.cuda.synchronize()
        w = (time.perf_counter() - t0) * 1e6 / args.steps
        print(f"{tag}: wall {w:.2f} us/step, events {e0.elapsed_time(e1) * 1e3 / args.steps:.2f} us/step", flush=True)

    def loop(tag):   # the same steps from one C call (qs_step_n) instead of a graph replay
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record(stream)
        env.step_n(acts, args.steps)
        e1.record(stream)
        torch.cuda.synchronize()
        w = (time.perf_counter() - t0) * 1e6 / args.steps
        print(f"{tag}: wall {w:.2f} us/step, events {e0.elapsed_time(e1) * 1e3 / args.steps:.2f} us/step", flush=True)

    for k in range(6):
        one(f"fresh replay {k}")
    for k in range(6):
        loop(f"C loop {k}")
    for k in range(3):
        one(f"replay again {k}")
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
        g.replay()
    torch.cuda.synchronize()
    for k in range(4):
        one(f"after 0.3 s busy, replay {k}")
    time.sleep(0.5)
    for k in range(3):
        one(f"after 0.5 s idle, replay {k}")


if __name__ == "__main__":
    main()
