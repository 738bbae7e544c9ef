"""Experiment: split one GPU's env shard into S blocks on S HIP streams.

Each block is its own handle (drone_id_offset keyed, so the union draws exactly what one big env
would, see tests/test_gpu_*shard*).  Per block, step t+1 only waits for step t of the same block, so
one block's next launch can fill the CUs the other block's tail wave leaves idle.
Usage: python tools/exp_streams.py --config c3 --splits 1 2 4 --steps 2000
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "quad-swarm-rl-stable-baselines3_amd"))

import bench  # noqa: E402


def new_stream(torch, dev, kind):
    if kind == "hi":
        return torch.cuda.Stream(dev, priority=-1)
    if kind == "raw":
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so")
        p = ctypes.c_void_p()
        assert hip.hipStreamCreateWithFlags(ctypes.byref(p), ctypes.c_uint(1)) == 0  # hipStreamNonBlocking
        return torch.cuda.ExternalStream(p.value, device=dev)
    return torch.cuda.Stream(dev)


def measure(torch, QuadSwarmEnv, kw, S, steps, warmup, chunk, dev, kind="pool"):
    cfg0 = bench.make_cfg(kw, seed=0, specialize=True)
    E, N = cfg0.num_envs, cfg0.num_agents
    sizes = [E // S + (1 if s < E % S else 0) for s in range(S)]
    starts = [sum(sizes[:s]) for s in range(S)]
    envs, acts, streams, graphs = [], [], [], []
    gen = torch.Generator(device=dev).manual_seed(1234)
    actions = (torch.rand(E * N, cfg0.act_dim, device=dev, generator=gen) * 2.0 - 1.0).contiguous()
    for s in range(S):
        kws = dict(kw)
        kws["num_envs"] = sizes[s]
        cfg = bench.make_cfg(kws, seed=0, specialize=True)
        cfg.drone_id_offset = starts[s] * N
        st = new_stream(torch, dev, kind)
        with torch.cuda.stream(st):
            env = QuadSwarmEnv(cfg, device=dev)
            env.reset()
            a = actions[starts[s] * N:(starts[s] + sizes[s]) * N].contiguous()
            for _ in range(3):
                env.step(a)
        torch.cuda.synchronize(dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            for _ in range(chunk):
                env.step(a)
        torch.cuda.synchronize(dev)
        envs.append(env); acts.append(a); streams.append(st); graphs.append(g)

    def run(n):
        for _ in range(n // chunk):
            for s in range(S):
                with torch.cuda.stream(streams[s]):
                    graphs[s].replay()

    run(warmup)
    torch.cuda.synchronize(dev)
    main = torch.cuda.current_stream(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(main)
    for st in streams:
        st.wait_stream(main)
    run(steps)
    for st in streams:
        main.wait_stream(st)
    ev1.record(main)
    torch.cuda.synchronize(dev)
    us = ev0.elapsed_time(ev1) * 1e3 / steps
    return {"splits": S, "us_per_step": round(us, 3), "agent_steps_per_s": E * N / (us * 1e-6)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--splits", type=int, nargs="+", default=[1, 2, 4])
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--graph", type=int, default=100)
    ap.add_argument("--burn", type=int, default=0, help="streams created and used once before the blocks'")
    ap.add_argument("--kind", default="pool", choices=["pool", "hi", "raw"])
    args = ap.parse_args()
    import torch
    from quadswarm_amd.env import QuadSwarmEnv
    dev = torch.device("cuda", 0)
    kw = bench.CONFIGS[args.config]
    burnt = []
    for _ in range(args.burn):
        st = new_stream(torch, dev, args.kind)
        with torch.cuda.stream(st):
            torch.zeros(1, device=dev).add_(1)
        burnt.append(st)
    torch.cuda.synchronize(dev)
    for S in args.splits:
        r = measure(torch, QuadSwarmEnv, kw, S, args.steps, args.warmup, args.graph, dev, args.kind)
        r["config"] = args.config
        r["kind"] = args.kind
        r["burn"] = args.burn
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
