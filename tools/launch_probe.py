#!/usr/bin/env python
"""Launch-path A/B for a short timed window (the driver's 20 steps): the same C3 steps issued as
  graph      one captured 20-step hipGraph replayed through torch (bench.py's path)
  rawgraph   the same executable graph launched with hipGraphLaunch directly (no torch wrapper)
  eager      20 launches from one C call (qs_step_n)
  e1+g19     1 eager launch, then a 19-step graph (the graph's launch preparation overlaps the first kernel)
  e2+g18     2 eager launches, then an 18-step graph
each round-robin over several repetitions, with wall / HIP-event times and the host time of each call.  Diagnostic.

    python tools/launch_probe.py [--reps 8]
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
    ap.add_argument("--config", default="c3")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=8)
    args = ap.parse_args()
    import torch
    import bench
    from quadswarm_amd.env import QuadSwarmEnv
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    cfg = bench.make_cfg(bench.CONFIGS[args.config], seed=0, specialize=True)
    env = QuadSwarmEnv(cfg, device=dev)
    I = cfg.num_envs * cfg.num_agents
    acts = (torch.rand(I, cfg.act_dim, device=dev, generator=torch.Generator(device=dev).manual_seed(1234)) * 2
            - 1).contiguous()
    env.reset()
    stream = torch.cuda.current_stream(dev)
    hip = ctypes.CDLL("libamdhip64.so")
    K = args.steps
    graphs = {}

    def graph(n):
        if n not in graphs:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(n):
                    env.step(acts)
            torch.cuda.synchronize(dev)
            rc = hip.hipGraphUpload(ctypes.c_void_p(g.raw_cuda_graph_exec()), ctypes.c_void_p(stream.cuda_stream))
            assert rc == 0
            graphs[n] = g
        return graphs[n]

    for n in (K, K - 1, K - 2):
        graph(n)
    torch.cuda.synchronize(dev)

    def raw_launch(g):
        rc = hip.hipGraphLaunch(ctypes.c_void_p(g.raw_cuda_graph_exec()), ctypes.c_void_p(stream.cuda_stream))
        assert rc == 0

    variants = {
        "graph": lambda: graph(K).replay(),
        "rawgraph": lambda: raw_launch(graph(K)),
        "eager": lambda: env.step_n(acts, K),
        "e1+g19": lambda: (env.step(acts), raw_launch(graph(K - 1))),
        "e2+g18": lambda: (env.step_n(acts, 2), raw_launch(graph(K - 2))),
    }
    res = {k: [] for k in variants}
    for k, f in variants.items():   # warm every path once
        f()
    torch.cuda.synchronize(dev)
    for _ in range(args.reps):
        for k, f in variants.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            e0.record(stream)
            t1 = time.perf_counter()
            f()
            t2 = time.perf_counter()
            e1.record(stream)
            t3 = time.perf_counter()
            torch.cuda.synchronize(dev)
            t4 = time.perf_counter()
            res[k].append(((t4 - t0) * 1e6, e0.elapsed_time(e1) * 1e3, (t1 - t0) * 1e6, (t2 - t1) * 1e6,
                           (t3 - t2) * 1e6, (t4 - t3) * 1e6))
    print(f"{'variant':10s} {'wall':>8s} {'events':>8s} {'rec0':>6s} {'launch':>7s} {'rec1':>6s} {'sync':>7s}  (us, "
          f"median of {args.reps}, {K} steps)")
    for k, rows in res.items():
        med = [sorted(c)[len(c) // 2] for c in zip(*rows)]
        print(f"{k:10s} {med[0]:8.2f} {med[1]:8.2f} {med[2]:6.2f} {med[3]:7.2f} {med[4]:6.2f} {med[5]:7.2f}", flush=True)


if __name__ == "__main__":
    main()
