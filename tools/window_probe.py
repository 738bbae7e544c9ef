#!/usr/bin/env python
"""Where the driver's short bench window goes (VERDICT r05 "do this" #5): the C3 step run exactly as
`bench.py --gpus 1 --steps 20 --warmup 5` runs it (fresh env, reset, graphs of 20 and 5 steps captured and uploaded,
5 warm-up replays' worth of steps, then one timed 20-step replay bracketed by HIP events and the wall clock), followed
by the controls that split its excess over the steady-state step time into named parts:

  repeat     the same 20-step replay again, back to back, continuing the same episode (cold first replay vs state)
  reset      a fresh reset on a warm device, then warm-up 5 + timed 20 (the post-reset state on a warm device)
  empty      the timed region with no work (event records + synchronize): the fixed host cost
  one        a 1-step graph in the timed region
  chunks     2000 steps in 100-step replays with events per replay: step time against episode progress

Diagnostic only; prints one line per measurement and a JSON summary.

    python tools/window_probe.py [--config c3]
"""
import argparse
import json
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
    ap.add_argument("--warmup", type=int, default=5)
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
    run = bench.Blocks(torch, dev, [(env, acts, stream)], min(100, args.steps))
    run.prepare([args.warmup, args.steps, 1])
    run.upload()
    out = {}

    def region(tag, n, work=True):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        e0.record(stream)
        if work:
            run.run(n)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        wall = (time.perf_counter() - t0) * 1e6
        ev = e0.elapsed_time(e1) * 1e3
        print(f"{tag:28s} wall {wall:8.2f} us  events {ev:8.2f} us  ({n} steps: wall {wall / max(n, 1):6.3f}, "
              f"events {ev / max(n, 1):6.3f} us/step)", flush=True)
        out.setdefault(tag, []).append({"wall_us": round(wall, 2), "events_us": round(ev, 2), "steps": n})
        return wall, ev

    # 1. the driver's window, exactly
    run.run(args.warmup)
    torch.cuda.synchronize(dev)
    region("driver window", args.steps)
    # 2. the same replay again, continuing the episode
    for _ in range(5):
        region("repeat", args.steps)
    # 3. fixed cost of the region
    for _ in range(5):
        region("empty", 0, work=False)
    for _ in range(5):
        region("one step", 1)
    # 4. post-reset on a warm device
    for _ in range(3):
        env.reset()
        run.run(args.warmup)
        torch.cuda.synchronize(dev)
        region("reset+warm5 window", args.steps)
    # 5. step time against episode progress (100-step replays after a reset)
    env.reset()
    run2 = bench.Blocks(torch, dev, [(env, acts, stream)], 100)
    run2.prepare([100])
    run2.upload()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
    torch.cuda.synchronize(dev)
    for a, b in evs:
        a.record(stream)
        run2.run(100)
        b.record(stream)
    torch.cuda.synchronize(dev)
    chunks = [round(a.elapsed_time(b) * 10, 3) for a, b in evs]    # us per step
    print("chunks of 100 steps after a reset (us/step):", chunks, flush=True)
    out["chunks_us_per_step"] = chunks
    print(json.dumps(out))


if __name__ == "__main__":
    main()
