#!/usr/bin/env python
"""Benchmark: agent-steps/s of the fused HIP swarm step (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (one rank per GPU)

`python bench.py --gpus N` (N > 1) with no launcher around starts the second form itself as a child process
(before any HIP call) and relays rank 0's line; under a launcher WORLD_SIZE must equal --gpus (else exit 1).

A "step" = one QuadrotorEnvMulti.step of every env on the GPU (qs_step: physics x2 substeps,
collisions, proximity, impulses, neighbour top-k, sensor noise, obs, rewards, fused auto-reset),
actions read from a fixed device buffer of U(-1,1) draws (seed 1234), state resident in HBM.
Weak scaling: every rank owns its own 4096 envs x 8 drones (disjoint Philox key ranges), no
collective on the data path; value = all ranks' agent-steps / max-over-ranks wall time.

Besides the required fields the JSON line carries:
  roofline      algorithmic bytes per launch / HIP-event kernel time vs 8 TB/s
  cpu_baseline  the C oracle (oracle/, OpenMP over envs) on this host, bounded ~10 s sample
  end_to_end    SURVEY §8 d(ii): PPO agent-steps/s of the GPU trainer (quadswarm_amd/ppo.py) --
                rollout over the same env shard + HIP GAE + minibatch update with one RCCL all-reduce
                of the flat gradient bucket per minibatch (N>1), max-over-ranks wall time
"""
import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "quad-swarm-rl-stable-baselines3_amd"))

# BASELINE.json configs -> (envs per GPU, agents, visible neighbours, downwash); "a*" = flavor A as
# swarm_rl/sb_train.py trains it (QuadSwarmConfig.sb_train), capture radius at a late curriculum stage
CONFIGS = {
    "c2": dict(num_envs=16384, num_agents=1, neighbor_visible_num=0, neighbor_obs_type="none"),
    "c3": dict(num_envs=4096, num_agents=8, neighbor_visible_num=6, neighbor_obs_type="pos_vel"),
    "c4": dict(preset="c4", num_envs=4096, num_agents=8),
    # the reference's own swarm training run (swarm_rl/runs/quad_multi_mix_baseline.py): C3 with quads_mode=mix
    "c3mix": dict(num_envs=4096, num_agents=8, neighbor_visible_num=6, neighbor_obs_type="pos_vel", quads_mode="mix"),
    # ... with its experience replay (replay_buffer_sample_prob=0.75, quad_experience_replay.py on device)
    "c3mixr": dict(num_envs=4096, num_agents=8, neighbor_visible_num=6, neighbor_obs_type="pos_vel", quads_mode="mix",
                   replay_buffer_sample_prob=0.75),
    # C4 as the reference trains obstacle domain randomisation (runs/obstacles/obst_domain_random.py: replay 0.75,
    # per-episode pillar density in {0.05 .. 0.2} and size in {0.3, 0.4, 0.5})
    "c4dr": dict(preset="c4", num_envs=4096, num_agents=8, replay_buffer_sample_prob=0.75, domain_random=True,
                 obst_density_random=True, obst_size_random=True, obst_density_min=0.05, obst_density_max=0.2,
                 obst_size_min=0.3, obst_size_max=0.6),
    "c5": dict(num_envs=1024, num_agents=32, neighbor_visible_num=6, neighbor_obs_type="pos_vel"),
    "a8": dict(flavor="A", num_envs=4096, num_agents=8, initial_capture_radius=0.5),
    # 64-drone swarms (the paper's scaling axis, paper/fps_compare.py:7): one env per wave, one lane per drone
    "n64": dict(num_envs=512, num_agents=64, neighbor_visible_num=6, neighbor_obs_type="pos_vel"),
    # 128-drone swarms (the paper's largest, paper/fps_compare.py:7): one env per two-wave workgroup
    "n128": dict(num_envs=256, num_agents=128, neighbor_visible_num=6, neighbor_obs_type="pos_vel"),
    "a4": dict(flavor="A", num_envs=8192, num_agents=4, initial_capture_radius=0.5),
    # flavor A at the paper's largest swarm (paper/fps_compare.py:7): one env per 4-wave workgroup, k = 7
    "a128": dict(flavor="A", num_envs=256, num_agents=128, neighbor_visible_num=7, initial_capture_radius=0.5),
}
WORKLOAD = {"c2": "single_quad x 16384 envs", "c3": "8-drone swarm static_same_goal x 4096 envs (pos_vel k=6)",
            "n64": "64-drone swarm static_same_goal x 512 envs (pos_vel k=6)",
            "n128": "128-drone swarm static_same_goal x 256 envs (pos_vel k=6)",
            "c3mix": "8-drone swarm, quads_mode mix (the 9 goal scenarios of QUADS_MODE_LIST) x 4096 envs (pos_vel k=6)",
            "c3mixr": "8-drone swarm, quads_mode mix x 4096 envs (pos_vel k=6) + experience replay (p=0.75), the "
                      "reference's swarm run (runs/quad_multi_mix_baseline.py)",
            "c4": "8-drone swarm + obstacles x 4096 envs (12 pillars, SDF obs, pos_vel k=2, floor obs, downwash, "
                  "mix of o_random / o_static_same_goal)",
            "c4dr": "8-drone swarm + obstacles x 4096 envs with experience replay (p=0.75) and obstacle domain "
                    "randomisation (3-12 pillars of 0.3-0.5 m per episode), runs/obstacles/obst_domain_random.py",
            "c5": "32-drone swarm x 1024 envs per GPU (pos_vel k=6)",
            "a8": "flavor A (sb_train env: PID pre-controller x 8 ticks, dynamic_repulsive target, ndist_nsangle "
                  "camera neighbours k=7) 8 drones x 4096 envs, capture radius 0.5",
            "a4": "flavor A sb_train default 4 drones x 8192 envs (k=3), capture radius 0.5",
            "a128": "flavor A (sb_train env) 128 drones x 256 envs, camera neighbours k=7, capture radius 0.5"}


def make_cfg(kw, **extra):
    from quadswarm_amd import QuadSwarmConfig
    kw = dict(kw)
    if kw.pop("preset", None) == "c4":
        return QuadSwarmConfig.c4(**kw, **extra)
    if kw.pop("flavor", "B") == "A":
        return QuadSwarmConfig.sb_train(**kw, **extra)
    return QuadSwarmConfig(**kw, **extra)


HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table (spec)


def algorithmic_bytes_per_agent_step(obs_dim, n_agents, flavor="B", n_obst=0):
    """B = 4 (S_r + S_w + A + O + 1) + 1 with S_r = 33 persistent fp32 state
    (pos3 vel3 rot9 omega3 cmd_damp4 rot_damp4 OU4 goal3), S_w = 30, A = 4, O = obs_dim, +1 reward,
    +1 byte done.  C3: 489 B, C2: 345 B.
    Flavor A: S_r = S_w = 55 (+ PID 20, heading, heading rate; the goal moves with the target), A = 2,
    plus per env (tick/flags/episode r+w 24 B, target r+w 16 B, capture radius 4 B, reset_info 1 B) / N.
    A8 (obs 28): 570.6 B.  Obstacles add the env's pillar list once per env: 8 M / N (C4: 445 B)."""
    if flavor == "A":
        return 4 * (55 + 55 + 2 + obs_dim + 1) + 1 + 45.0 / n_agents
    return 4 * (33 + 30 + 4 + obs_dim + 1) + 1 + 8.0 * n_obst / n_agents


def state_bytes_per_agent_step(cfg):
    """Bytes a step moves per agent once the state the reference's step also carries is counted (§8d's formula leaves
    it out): per drone the istate words (SVD counter, flags, the collision-row words a swarm of N can set: 0 / 1 / 2 / 4
    for N = 1 / <= 32 / <= 64 / 128) read and written, and with episode_extra_stats on (the reference's default) the
    distance ring + window sums read (8 words) and one ring slot written; per env (divided by N) tick, episode and flags
    read, tick and flags written, and the episode counters no configuration leaves at 0 read (room 4, drone-drone 3
    when N > 1, obstacle 4 with obstacles).  Flavor B only (flavor A's §8d count already includes its env words).
    Returns (bytes per agent-step, read bytes per agent-step)."""
    n = cfg.num_agents
    npad = 1 << (n - 1).bit_length()
    niw = 2 if npad == 1 else (3 if npad <= 32 else (4 if npad <= 64 else 6))
    obst = cfg.num_obstacles if cfg.use_obstacles else 0
    base = algorithmic_bytes_per_agent_step(cfg.obs_dim, n, cfg.flavor, obst)
    base_read = 4 * (33 + 4) + 8.0 * obst / n
    stats = bool(cfg.episode_stats)
    ncnt = (4 + (3 if n > 1 else 0) + (4 if cfg.use_obstacles else 0)) if stats else 0
    drone_r = 4 * niw + (4 * 8 if stats else 0)
    drone_w = 4 * niw + (4 if stats else 0)
    env_r, env_w = 4 * (3 + ncnt), 4 * 2
    return base + drone_r + drone_w + (env_r + env_w) / n, base_read + drone_r + env_r / n


def cpu_worker(config, seconds):
    """One cpu_baseline leg, run as a child process (bench.py --cpu-worker): the C oracle on this host's cores,
    fp64 (liboracle.so) or its fp32 twin (liboracle_f32.so, QS_ORACLE_F32=1), OpenMP over envs with
    OMP_NUM_THREADS threads, on the same workload shape as the GPU line; time-bounded sample."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle as O
    from parity_utils import oracle_params, oracle_params_a

    threads = int(os.environ.get("OMP_NUM_THREADS", "1"))
    cfg = make_cfg(CONFIGS[config])
    if cfg.flavor == "A":
        env = O.OracleEnvA(oracle_params_a(cfg), seed=0)
        env.set_capture_radius(cfg.initial_capture_radius)
    else:
        env = O.OracleEnv(oracle_params(cfg), seed=0)
    env.reset()
    a = np.random.default_rng(1234).uniform(-1.0, 1.0, (cfg.num_envs * cfg.num_agents, cfg.act_dim))
    env.step(a, nthreads=threads)
    steps, t0 = 0, time.perf_counter()
    while True:
        env.step(a, nthreads=threads)
        steps += 1
        el = time.perf_counter() - t0
        if el >= seconds or steps >= 4000:
            break
    print(json.dumps({"value": round(steps * cfg.num_envs * cfg.num_agents / el, 1), "steps": steps,
                      "seconds": round(el, 2), "threads": threads, "fp32": O.F32}), flush=True)


def cpu_baseline(config, seconds=6.0):
    """SURVEY §8d CPU baseline: the oracle restatement on the GPU box's host cores, in three legs -- fp32
    on 1 thread, fp32 on all usable threads (the headline `value`), fp64 on all threads (the parity
    checker itself) -- each a child process with its own bounded sample."""
    cores = len(os.sched_getaffinity(0))
    cores = min(cores, int(os.environ.get("OMP_NUM_THREADS", cores)))
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    legs = {}
    for name, f32, th in (("fp32_1t", True, 1), (f"fp32_{cores}t", True, cores), (f"fp64_{cores}t", False, cores)):
        env = dict(os.environ, OMP_NUM_THREADS=str(th), QS_ORACLE_F32="1" if f32 else "0")
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--cpu-worker", "--config", config,
                            "--cpu-seconds", str(seconds)], env=env, capture_output=True, text=True, timeout=600)
        if r.returncode != 0:
            raise RuntimeError(f"cpu leg {name} failed: {r.stderr[-400:]}")
        legs[name] = json.loads(r.stdout.strip().splitlines()[-1])
    cfg = make_cfg(CONFIGS[config])
    head = legs[f"fp32_{cores}t"]
    return {"value": head["value"], "unit": "agent-steps/s", "cores": cores, "kind": "port",
            "precision": "fp32",
            "sample": f"{head['steps']} steps x {cfg.num_envs} envs x {cfg.num_agents} drones, the C oracle's fp32 twin "
                      f"(oracle/liboracle_f32.so), {cores} OpenMP threads, {head['seconds']} s on '{model}'",
            "legs": {k: {"value": v["value"], "threads": v["threads"], "steps": v["steps"], "seconds": v["seconds"]}
                     for k, v in legs.items()}}


def npad(n):
    p = 1
    while p < n:
        p <<= 1
    return p


def pmc_traffic(config):
    """HBM bytes per launch measured by rocprofv3 --pmc (profiles/pmc_<config>.json, written by
    tools/summarize_prof.py from separate FETCH_SIZE / WRITE_SIZE passes with the gfx950 correction), and where
    they come from (file, the tree they were taken on, reads / writes)."""
    p = os.path.join(ROOT, "profiles", f"pmc_{config}.json")
    if not os.path.exists(p):
        return None, None
    try:
        d = json.load(open(p))
        src = {"file": os.path.relpath(p, ROOT), "tree": d.get("tree"),
               "read_bytes": d.get("hbm_read_bytes_per_launch"), "write_bytes": d.get("hbm_write_bytes_per_launch"),
               "passes": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate runs, FETCH x2 (gfx950)",
               "correction": d.get("correction")}
        return d.get("hbm_bytes_per_launch"), src
    except Exception:
        return None, None


VALU_PEAK_TFLOPS = 157.3      # MI355X_MICROARCH.md chip table: FP32 vector (v_pk_fma_f32, 64 FLOP/clk/SIMD)


SIMDS = 1024                  # 256 CUs x 4 SIMDs


def valu_roofline(config, agents_per_launch, kernel_ms):
    """The VALU side of the step (flavor A is near the fp32-vector ridge; flavor B's waves are issue /
    latency-bound below the HBM roofline), from the committed PMC summary profiles/pmc_<config>.json
    (tools/summarize_prof.py):
      issue_frac   VALU instructions issued per wave / the wave's lifetime in quad-cycles (SQ_INSTS_VALU /
                   SQ_WAVE_CYCLES per wave; a wave64 VALU instruction occupies its SIMD for one quad-cycle)
      waves_per_simd, simd_issue_frac   SQ_WAVES / 1024 SIMDs, and that many waves' VALU issue against one wave's
                   lifetime: the share of the SIMD's VALU issue slots the launch uses (C3: 2 waves per SIMD)
      issue_floor_us   simd_issue_frac x this line's kernel time: the launch if every SIMD issued VALU back to back
                   (no memory / LDS / dependency wait); kernel_us / issue_floor_us is the latency factor
      flop         executed fp32 FLOP per launch = 64 lanes x (2 FMA + ADD + MUL + TRANS) instructions
                   (SQ_INSTS_VALU_{FMA,ADD,MUL,TRANS}_F32, the derived-counter formula of rocprofiler's
                   TOTAL_32_OPS without the integer and MFMA terms), per agent-step, and the rate at this
                   line's kernel time against the 157.3 TF fp32 vector peak (frac).  Executed, not algorithmic: the
                   chain replicated on a drone's sub-lanes counts once per sub-lane."""
    p = os.path.join(ROOT, "profiles", f"pmc_{config}.json")
    if not os.path.exists(p):
        return None
    try:
        d = json.load(open(p))
        pw, c = d.get("per_wave", {}), d.get("counters_per_launch", {})
        out = {"source": {"file": os.path.relpath(p, ROOT), "tree": d.get("tree")}}
        if "SQ_INSTS_VALU" in pw and "SQ_WAVE_CYCLES" in pw:
            out.update(valu_insts_per_wave=round(pw["SQ_INSTS_VALU"], 1),
                       wave_quad_cycles=round(pw["SQ_WAVE_CYCLES"], 1),
                       issue_frac=round(pw["SQ_INSTS_VALU"] / pw["SQ_WAVE_CYCLES"], 4))
            if "SQ_WAVES" in c:
                wps = c["SQ_WAVES"] / SIMDS
                sif = wps * pw["SQ_INSTS_VALU"] / pw["SQ_WAVE_CYCLES"]
                out.update(waves_per_simd=round(wps, 3), simd_issue_frac=round(sif, 4),
                           issue_floor_us=round(sif * kernel_ms * 1e3, 3))
            if "SQ_WAIT_ANY" in pw:
                out["wait_frac"] = round(pw["SQ_WAIT_ANY"] / pw["SQ_WAVE_CYCLES"], 4)
        keys = ("SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_TRANS_F32")
        if all(k in c for k in keys):
            flop = 64.0 * (2 * c[keys[0]] + c[keys[1]] + c[keys[2]] + c[keys[3]])
            tf = flop / (kernel_ms * 1e-3) / 1e12
            out.update(flop_per_launch=round(flop), flop_per_agent_step=round(flop / agents_per_launch, 1),
                       achieved_tflops=round(tf, 2), peak_tflops=VALU_PEAK_TFLOPS, frac=round(tf / VALU_PEAK_TFLOPS, 4))
            if "SQ_INSTS_VALU_FLOPS_FP32" in c:
                out["sq_insts_valu_flops_fp32_per_launch"] = round(c["SQ_INSTS_VALU_FLOPS_FP32"])
        return out
    except Exception:
        return None


# end-to-end PPO leg per workload family: policy / PPO settings of the reference run that trains it
#   flavor A: swarm_rl/sb_train.py parameter_sweep (SB3 PPO, global_cfg.py:21-29): n_steps 512, 10 epochs,
#             gamma 0.99, lambda 0.95, clip 0.2, max_grad_norm 0.5, lr 1e-4; attention encoder, 6x128 MLP core.
#             The reference's 12 envs x 4 agents x 512 steps / batch 1024 = 24 minibatches per epoch; the GPU
#             rollout is ~700x larger, so the minibatch is scaled to keep 24 minibatches per epoch.
#   flavor B: runs/quad_multi_mix_baseline.py (rollout 128, lambda 1.0, max_grad_norm 5.0, rnn 256,
#             attention 256, identity core, 1 pass per sample); 16 minibatches per rollout.
def e2e_settings(cfg):
    from quadswarm_amd.ppo import PolicyConfig, PPOConfig
    if cfg.flavor == "A":
        return PolicyConfig.sb_train(cfg), PPOConfig(), 24
    pc = PolicyConfig.for_env(cfg, rnn_size=256, neighbor_hidden_size=256, obst_hidden_size=256)
    return pc, PPOConfig(n_steps=128, n_epochs=1, gae_lambda=1.0, max_grad_norm=5.0), 16


def update_flops_per_sample(pol, obs_dim, act_dim, dev, rows=256, split=False):
    """FLOPs of one sample's PPO update (evaluate_actions forward + backward), counted by torch's
    FlopCounterMode (GEMM / addmm / bmm flops) on a small batch of the same policy.  split: also the share of the
    modules the fused x3 update runs on the f16 matrix cores: both towers' neighbour encoders, feed_forward and
    self encoder (all but its first layer's forward, 18 inputs, which stays in hipBLASLt like the heads)."""
    import torch
    from torch.utils.flop_counter import FlopCounterMode
    obs = torch.randn(rows, obs_dim, device=dev)
    act = torch.rand(rows, act_dim, device=dev) * 1.8 - 0.9
    with FlopCounterMode(display=False) as fc:
        v, lp, _ = pol.evaluate_actions(obs, act)
        (v.sum() + lp.sum()).backward()
    pol.zero_grad(set_to_none=False)
    total = fc.get_total_flops() / rows
    if not split:
        return total
    # the x3 share = everything but the heads (forward, dX, dW: 6 d_in d_out each) and the self encoders' first
    # layer forward (2 so R per tower; its dW is x3) -- FlopCounterMode's per-module keys nest and collide
    heads = sum(6 * m.in_features * m.out_features for m in (pol.action_net, pol.value_net))
    l0 = sum(2 * e.self_encoder[0].in_features * e.self_encoder[0].out_features
             for e in (pol.actor_encoder, pol.critic_encoder))
    return total, total - heads - l0


F16_DENSE_TFLOPS = 2500.0     # MI355X_MICROARCH.md: BF16 / F16 MFMA ~2.5 PF dense


def end_to_end(env, cfg, dev, world, iters, n_steps=None, log=None, fused=True, precision="fp32",
               update_precision="fp32"):
    """Timed PPO iterations (rollout + GAE + update) on the bench's env shard.  update_precision "x3": the update's
    attention encoders through the fused forward / backward kernels (encoder_train.py), else torch autograd."""
    import torch
    import torch.distributed as dist
    from quadswarm_amd.ppo import PPOTrainer, SwarmActorCritic, use_gemm_table

    pc, pcfg, n_mb = e2e_settings(cfg)
    tuned = use_gemm_table() if os.environ.get("PYTORCH_TUNABLEOP_TUNING") != "1" else "tuning"
    if n_steps:
        pcfg.n_steps = n_steps
    samples = pcfg.n_steps * env.I
    pcfg.batch_size = -(-samples // n_mb)
    torch.manual_seed(0)
    pol = SwarmActorCritic(pc).to(dev)
    from quadswarm_amd.policy_fused import supports
    upd = update_precision if (fused and supports(pol)) else "fp32"
    tr = PPOTrainer(env, pol, pcfg, seed=0, fused_rollout=fused, rollout_precision=precision, update_precision=upd)
    tr.reset()

    def sync():
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)

    # warm-up: one rollout + one epoch cut short (allocator, rocBLAS/hipBLASLt kernel selection)
    tr.collect_rollouts()
    tr.train(max_updates=3)
    sync()
    t_roll = t_train = 0.0
    t0 = time.perf_counter()
    stats = {}
    for it in range(iters):
        a = time.perf_counter()
        tr.collect_rollouts()
        torch.cuda.synchronize(dev)
        b = time.perf_counter()
        stats = tr.train()
        torch.cuda.synchronize(dev)
        t_roll += b - a
        t_train += time.perf_counter() - b
        if log:
            log(f"e2e iteration {it + 1}/{iters}: rollout {b - a:.2f} s, update {time.perf_counter() - b:.2f} s")
    sync()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el, t_roll, t_train], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el, t_roll, t_train = (float(x) for x in t.tolist())
    nparam = sum(p.numel() for p in pol.parameters())
    # the update's GEMM work against the fp32 matrix-core peak (MI355X_MICROARCH: 157.3 TF dense f32)
    fps, enc_fps = update_flops_per_sample(pol, env.obs_dim, env.act_dim, dev, split=True)
    upd_tf = fps * samples * pcfg.n_epochs / (t_train / iters) / 1e12
    # the ceiling of the update as it runs: with the fused x3 encoders their fp32-equivalent work is 3 f16 products per
    # fp32 product on the f16 matrix cores (2.5 PF / 3), the rest fp32 on hipBLASLt (157.3 TF); without, all fp32
    x3 = update_precision == "x3" and getattr(tr, "fused_update", None) is not None
    enc_peak = (F16_DENSE_TFLOPS / 3.0) if x3 else 157.3
    floor_s = samples * pcfg.n_epochs * (enc_fps / (enc_peak * 1e12) + (fps - enc_fps) / 157.3e12)
    tr.bucket.zero()
    return {
        "metric": "end-to-end PPO agent-steps/s (rollout + GAE + update; weak scaling, one gradient "
                  "all-reduce per minibatch)",
        "value": round(world * iters * samples / el, 1), "unit": "agent-steps/s", "iterations": iters,
        "s_per_iteration": round(el / iters, 3), "rollout_s": round(t_roll / iters, 3),
        "update_s": round(t_train / iters, 3),
        "n_steps": pcfg.n_steps, "n_epochs": pcfg.n_epochs, "batch_size_per_rank": pcfg.batch_size,
        "minibatches_per_epoch": n_mb, "policy_params": nparam,
        "policy": f"ActorCriticPolicyCustomSeparateWeights: {pc.neighbor_encoder_type} k={pc.num_use_neighbor_obs}, "
                  f"rnn {pc.rnn_size}, core {pc.rnn_type or 'identity'} x{pc.rnn_num_layers if pc.rnn_type else 0}, "
                  f"fp32 (torch/hipBLASLt GEMMs" + (f", rollout neighbour encoders + feed_forward / self-encoder layers: "
                                                    f"fused HIP MFMA kernels, {precision})"
                                                    if tr.fused is not None else ")"),
        "rollout_precision": precision if tr.fused is not None else "torch fp32",
        "update_precision": ("x3: fused HIP attention-encoder forward + backward (encoder_train.py), the encoders' "
                             "feed_forward / self-encoder layers and every dW on split-f16 MFMA; heads in torch fp32"
                             if upd == "x3" else "torch fp32 autograd (hipBLASLt)"),
        "gemm_table": tuned,
        "update_flop_per_sample": round(fps), "update_tflops": round(upd_tf, 2),
        # against the fp32 matrix-core peak only when the update runs there (x3 runs on the f16 matrix cores and
        # can pass 157 TF fp32-equivalent: its ceiling is update_ceiling)
        "update_frac_fp32_mfma_peak": None if x3 else round(upd_tf / 157.3, 3),
        "update_encoder_flop_share": round(enc_fps / fps, 3),
        "update_ceiling": {"encoders_tflops": round(enc_peak, 1), "rest_tflops": 157.3, "floor_s": round(floor_s, 4),
                           "frac": round(floor_s / (t_train / iters), 3),
                           "note": "x3 encoders + MLP layers: 3 f16 MFMA products per fp32 product at the 2.5 PF "
                                   "dense f16 peak; the rest (heads) fp32" if x3 else "all fp32 matrix cores"},
        "last_update": {k: (round(v, 6) if isinstance(v, float) else v) for k, v in stats.items()},
    }


class Blocks:
    """The GPU's env shard as S env blocks, each its own handle on its own HIP stream, stepped from
    captured hipGraphs (or eagerly through qs_step_blocks).  S = 1 is the one handle on torch's
    current stream."""

    def __init__(self, torch, dev, entries, chunk):
        self.torch, self.dev = torch, dev
        self.entries = entries      # [(env, actions, stream)]
        self.chunk = chunk
        self.graphs = {}            # (block, steps) -> CUDAGraph
        self.replays = self.eager_steps = 0

    def _graph(self, i, n):
        key = (i, n)
        if key not in self.graphs:
            eb, ab, st = self.entries[i]
            g = self.torch.cuda.CUDAGraph()
            # captured on the block's stream (one block: torch's capture side stream), replayed on it
            with self.torch.cuda.graph(g, stream=st if len(self.entries) > 1 else None):
                for _ in range(n):
                    eb.step(ab)
            self.torch.cuda.synchronize(self.dev)
            self.graphs[key] = g
        return self.graphs[key]

    def prepare(self, lengths):
        """capture every graph a run will replay before anything is timed"""
        for n in lengths:
            q, r = divmod(n, self.chunk) if self.chunk else (0, 0)
            for i in range(len(self.entries)):
                if q:
                    self._graph(i, self.chunk)
                if r:
                    self._graph(i, r)

    def run(self, n):
        from quadswarm_amd.env import step_blocks
        if not self.chunk:
            if len(self.entries) == 1:   # one handle: the n launches from one C call (qs_step_n)
                eb, ab, st = self.entries[0]
                with self.torch.cuda.stream(st):
                    eb.step_n(ab, n)
                self.eager_steps += n
                return
            envs = [e for e, _, _ in self.entries]
            acts = [a for _, a, _ in self.entries]
            sts = [s for _, _, s in self.entries]
            for _ in range(n):
                step_blocks(envs, acts, sts)
            self.eager_steps += n
            return
        q, r = divmod(n, self.chunk)
        for L, times in ((self.chunk, q), (r, 1 if r else 0)):
            for _ in range(times):
                for i, (_, _, st) in enumerate(self.entries):
                    with self.torch.cuda.stream(st):
                        self._graph(i, L).replay()
                self.replays += 1

    def upload(self):
        """hipGraphUpload every captured graph on its stream: the executable graph is made device-resident
        before anything is timed (otherwise its first replay, inside the timed region, pays the upload)."""
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so")
        for (i, _), g in self.graphs.items():
            st = self.entries[i][2]
            rc = hip.hipGraphUpload(ctypes.c_void_p(g.raw_cuda_graph_exec()), ctypes.c_void_p(st.cuda_stream))
            if rc != 0:
                raise RuntimeError(f"hipGraphUpload failed ({rc})")
        self.torch.cuda.synchronize(self.dev)

    def timed(self, n, stream, ev0=None, ev1=None):
        """n steps bracketed by HIP events (best created by the caller, outside any timed region) on `stream`
        (the blocks' streams join it on both sides; one handle runs on `stream` itself, so no cross-stream
        waits sit in the timed region)"""
        if ev0 is None:
            ev0, ev1 = self.torch.cuda.Event(enable_timing=True), self.torch.cuda.Event(enable_timing=True)
        joins = [st for _, _, st in self.entries if st is not stream]
        ev0.record(stream)
        for st in joins:
            st.wait_stream(stream)
        self.run(n)
        for st in joins:
            stream.wait_stream(st)
        ev1.record(stream)
        return ev0, ev1


def raw_streams(torch, dev, n, spare):
    """n non-blocking HIP streams (after `spare` streams used once: DESIGN.md §4, queue mapping)."""
    hip = ctypes.CDLL("libamdhip64.so")
    made = []

    def mk():
        p = ctypes.c_void_p()
        if hip.hipStreamCreateWithFlags(ctypes.byref(p), ctypes.c_uint(1)) != 0:  # hipStreamNonBlocking
            raise RuntimeError("hipStreamCreateWithFlags failed")
        made.append(p.value)
        return torch.cuda.ExternalStream(p.value, device=dev)
    for _ in range(spare):
        st = mk()
        with torch.cuda.stream(st):
            torch.zeros(1, device=dev).add_(1)
    torch.cuda.synchronize(dev)
    streams = [mk() for _ in range(n)]

    def destroy():
        torch.cuda.synchronize(dev)
        for p in made:
            hip.hipStreamDestroy(ctypes.c_void_p(p))
    return streams, destroy


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launcher_argv(argv, gpus, port):
    """The N-rank launch of this bench (one process per GPU, rendezvous on 127.0.0.1): what the driver runs for
    N > 1, started by `python bench.py --gpus N` itself when no launcher is around.  Replaces the reference's
    process-parallel envs (swarm_rl/env_wrappers/subproc_vec_env_custom.py:118-134) at GPU granularity."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def launch_ranks(argv, gpus):
    """Run the N ranks as a child process (nothing here has touched the GPU yet, so no exec), relay rank 0's
    JSON line as this process's last stdout line and return the child's exit code."""
    r = subprocess.run(launcher_argv(argv, gpus, free_port()), stdout=subprocess.PIPE, text=True)
    lines = r.stdout.splitlines()
    js = [ln for ln in lines if ln.startswith("{")]
    for ln in lines:
        if ln not in js:
            print(ln, file=sys.stderr, flush=True)
    for ln in js:
        print(ln, flush=True)
    return r.returncode


def launch_world(gpus, environ=None):
    """World size the bench runs at, checked against --gpus: under a launcher WORLD_SIZE must equal --gpus
    (a mismatch exits non-zero instead of reporting a line for a different GPU count)."""
    environ = os.environ if environ is None else environ
    if gpus < 1:
        raise SystemExit(f"bench.py: --gpus must be >= 1 (got {gpus})")
    world = int(environ.get("WORLD_SIZE", "1"))
    if world != gpus:
        raise SystemExit(f"bench.py: --gpus {gpus} but the launcher started {world} rank(s)")
    return world


def aggregate_ranks(agent_steps, seconds, world, device=None):
    """Weak-scaling aggregate: (sum of every rank's agent-steps, max-over-ranks seconds, per-rank agent-steps/s).
    One all_gather of two fp64 words per rank (RCCL on the GPU ranks, gloo in the CPU tests)."""
    if world == 1:
        return float(agent_steps), float(seconds), [float(agent_steps) / float(seconds)]
    import torch
    import torch.distributed as dist
    t = torch.tensor([float(agent_steps), float(seconds)], dtype=torch.float64, device=device)
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    rows = torch.stack(parts).cpu()
    return (float(rows[:, 0].sum()), float(rows[:, 1].max()),
            [float(a / s) for a, s in rows.tolist()])


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--graph", type=int, default=100, help="max steps per captured hipGraph (0 = eager launches)")
    ap.add_argument("--streams", type=int, default=0,
                    help="env blocks per GPU, each its own handle on its own HIP stream (default 1 = one handle, "
                         "the launch rocprofv3 profiles); with S > 1 the bench keeps the blocks only if an A/B "
                         "measures them faster than the one handle")
    ap.add_argument("--generic", action="store_true", help="generic kernels instead of qs_specialize (hipRTC)")
    ap.add_argument("--no-episode-stats", action="store_true",
                    help="A/B only: skip the episode_extra_stats accumulators the reference's step keeps")
    ap.add_argument("--quads-mode", default=None, help="A/B only: override the config's quads_mode (goal scenario)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=6.0, help="seconds per cpu_baseline leg (3 legs)")
    ap.add_argument("--cpu-worker", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--e2e-iters", type=int, default=2, help="timed PPO iterations for end_to_end (0 = skip)")
    ap.add_argument("--e2e-steps", type=int, default=0, help="override the PPO rollout length n_steps")
    ap.add_argument("--e2e-unfused", action="store_true",
                    help="A/B only: the rollout evaluates the torch policy module instead of the fused encoders")
    ap.add_argument("--e2e-precision", choices=["fp32", "x3"], default="x3",
                    help="fused rollout encoders: fp32 matrix cores, or each fp32 product as 3 f16 products with fp32 "
                         "accumulation (x3, the default: within 2e-7 of fp32 on the encoder outputs, DESIGN.md §4.6)")
    ap.add_argument("--e2e-update-precision", choices=["fp32", "x3"], default=None,
                    help="the update's attention encoders: torch fp32 autograd or the fused x3 forward / backward "
                         "kernels (default: --e2e-precision)")
    ap.add_argument("--host-sync", choices=["spin", "auto"], default="auto",
                    help="host wait of torch.cuda.synchronize(): spin (hipDeviceScheduleSpin) or HIP's default")
    args = ap.parse_args(argv)
    if args.cpu_worker:
        return cpu_worker(args.config, args.cpu_seconds)
    # --gpus N without a launcher: start the N ranks as a child (before any HIP call in this process)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        raise SystemExit(launch_ranks(argv, args.gpus))
    world = launch_world(args.gpus)

    if args.host_sync == "spin":   # before anything creates the device's context
        if ctypes.CDLL("libamdhip64.so").hipSetDeviceFlags(ctypes.c_uint(1)) != 0:   # hipDeviceScheduleSpin
            raise RuntimeError("hipSetDeviceFlags(hipDeviceScheduleSpin) failed")
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_dist = world > 1 or os.environ.get("QS_BENCH_DIST") == "1"   # QS_BENCH_DIST: RCCL path at N=1 (rehearsal)
    if use_dist:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but the process group has {dist.get_world_size()} ranks")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from quadswarm_amd.env import QuadSwarmEnv

    kw = CONFIGS[args.config]
    if args.no_episode_stats:
        kw = dict(kw, episode_stats=False)
    if args.quads_mode:
        kw = dict(kw, quads_mode=args.quads_mode)
    cfg = make_cfg(kw, seed=0, specialize=not args.generic)
    I = cfg.num_envs * cfg.num_agents
    cfg.drone_id_offset = rank * I
    env = QuadSwarmEnv(cfg, device=dev)
    gen = torch.Generator(device=dev).manual_seed(1234)
    actions = (torch.rand(I, cfg.act_dim, device=dev, generator=gen) * 2.0 - 1.0).contiguous()
    env.reset()
    stream = torch.cuda.current_stream(dev)
    # graphs of min(--graph, steps) steps, the remainder of a run in one more graph: every warm-up and
    # timed step of any --steps / --warmup is a graph replay (the driver runs --steps 20 --warmup 5)
    chunk = min(args.graph, args.steps) if args.graph > 0 else 0
    one = Blocks(torch, dev, [(env, actions, stream)], chunk)

    # Env blocks: envs are independent, so the shard is split into S blocks of E/S envs, each
    # its own handle keyed by its global drone ids (the union draws exactly what the one handle draws) on
    # its own HIP stream: one block's next launch fills the CUs another block's last waves leave idle.
    # Whether that pays depends on the config and on HIP's stream -> hardware-queue mapping, so it is
    # measured here against the one handle (same graphs, same step count) and kept only if faster.
    S = max(1, args.streams)
    if S > 1 and cfg.num_envs % S:
        S = 1
    blocks, destroy_streams, ab = None, None, None
    if S > 1:
        Eb = cfg.num_envs // S
        bstreams, destroy_streams = raw_streams(torch, dev, S, spare=3)
        entries = []
        for s_ in range(S):
            cb = make_cfg(dict(kw, num_envs=Eb), seed=0, specialize=not args.generic)
            cb.drone_id_offset = rank * I + s_ * Eb * cfg.num_agents
            st = bstreams[s_]
            st.wait_stream(stream)
            with torch.cuda.stream(st):
                eb = QuadSwarmEnv(cb, device=dev)
                eb.reset()
            entries.append((eb, actions[s_ * Eb * cfg.num_agents:(s_ + 1) * Eb * cfg.num_agents].contiguous(), st))
        torch.cuda.synchronize(dev)
        blocks = Blocks(torch, dev, entries, chunk)
        # A/B on the configuration's own graphs: 2 x max(chunk, 20) steps each, after one warm pass
        n_ab = max(chunk, 20) if chunk else 20
        for cand in (one, blocks):
            cand.prepare([n_ab])
            cand.run(n_ab)
        torch.cuda.synchronize(dev)
        times = {}
        for name, cand in (("one_handle", one), ("blocks", blocks)):
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            cand.timed(2 * n_ab, stream, *ev)
            torch.cuda.synchronize(dev)
            times[name] = ev[0].elapsed_time(ev[1]) * 1e3 / (2 * n_ab)
        if world > 1:   # every rank takes the same decision (rank 0's measurement)
            t = torch.tensor([times["one_handle"], times["blocks"]], device=dev, dtype=torch.float64)
            dist.broadcast(t, 0)
            times = {"one_handle": float(t[0]), "blocks": float(t[1])}
        ab = {k: round(v, 3) for k, v in times.items()}
        if times["blocks"] >= times["one_handle"]:
            S = 1
        ab["chosen"] = "blocks" if S > 1 else "one_handle"
    run = blocks if S > 1 else one
    run.replays = run.eager_steps = 0
    run.prepare([args.warmup, args.steps])
    if run.chunk:
        run.upload()

    run.run(args.warmup)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    # HIP events on the stream the launches are ordered on (graph replays and eager launches both go to
    # torch's current stream, or to the block streams that join it), bracketing the timed region: back to
    # back step kernels, so the average step time = span / K (rocprofv3 --kernel-trace, one handle, agrees)
    replays0, eager0 = run.replays, run.eager_steps
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    run.timed(args.steps, stream, ev0, ev1)
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    k_ms = ev0.elapsed_time(ev1) / args.steps
    timed_replays, timed_eager = run.replays - replays0, run.eager_steps - eager0
    if world > 1:
        dist.barrier()
    total_agent_steps, el, per_rank = aggregate_ranks(I * args.steps, el, world, dev)

    # the timed region's fixed cost, measured after it (untimed): the same event records and synchronize with no
    # step between them (median of 5) -- the wall the region pays whatever the kernel time
    empties = []
    for _ in range(5):
        e0_, e1_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        t0_ = time.perf_counter()
        e0_.record(stream)
        e1_.record(stream)
        torch.cuda.synchronize(dev)
        empties.append(((time.perf_counter() - t0_) * 1e6, e0_.elapsed_time(e1_) * 1e3))
    empty_wall, empty_ev = sorted(empties)[2]
    window = {"region_wall_us": round(el * 1e6, 2), "region_events_us": round(k_ms * args.steps * 1e3, 2),
              "host_side_us": round(el * 1e6 - k_ms * args.steps * 1e3, 2),
              "empty_region_wall_us": round(empty_wall, 2), "empty_region_events_us": round(empty_ev, 2),
              "note": "region wall = region events (graph launch latency + the step kernels) + host side (event "
                      "records, synchronize wake-up); tools/window_probe.py and profiles/r06/window_* split it "
                      "per launch"}

    # secondary: one eager launch of the one handle bracketed by its own events (includes the host launch gap)
    nk = min(200, max(20, args.steps // 10))
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(nk)]
    for s_ev, e_ev in evs:
        s_ev.record(stream)
        env.step(actions)
        e_ev.record(stream)
    torch.cuda.synchronize(dev)
    k_eager_ms = sum(s.elapsed_time(e) for s, e in evs) / nk
    guard = env.counters()

    e2e = None
    if args.e2e_iters > 0:
        log = (lambda m: print(m, file=sys.stderr, flush=True)) if rank == 0 else None
        try:
            e2e = end_to_end(env, cfg, dev, world, args.e2e_iters, args.e2e_steps or None, log,
                             fused=not args.e2e_unfused, precision=args.e2e_precision,
                             update_precision=args.e2e_update_precision or args.e2e_precision)
        except Exception as e:  # never let the PPO leg kill the env number
            if world > 1:
                raise
            e2e = {"error": repr(e)}

    if rank == 0:
        value = total_agent_steps / el
        bpa = algorithmic_bytes_per_agent_step(cfg.obs_dim, cfg.num_agents, cfg.flavor,
                                               cfg.num_obstacles if cfg.use_obstacles else 0)
        achieved = bpa * I / (k_ms * 1e-3) / 1e9
        traffic, traffic_src = pmc_traffic(args.config)
        if chunk:
            launch = f"{timed_replays} hipGraph replays ({timed_replays * len(run.entries)} graphs) for {args.steps} timed steps"
        else:
            launch = (f"eager: {timed_eager} launches from one qs_step_n call" if len(run.entries) == 1
                      else f"eager: {timed_eager} qs_step_blocks calls")
        if S > 1:
            launch += f", {S} env blocks of {cfg.num_envs // S} envs on {S} HIP streams"
        launch += ", specialised kernels (qs_specialize, hipRTC)" if env.specialized else ", generic kernels"
        out = {
            "metric": "agent-steps/sec, 8-drone swarm \u00d7 4096 envs, at 1/2/4/8 MI355X" if args.config == "c3"
            else f"agent-steps/sec, {WORKLOAD[args.config]}",
            "value": round(value, 1),
            "unit": "agent-steps/s",
            "n_gpus": world,
            "per_rank_agent_steps_per_s": [round(v, 1) for v in per_rank],
            "rccl_world_size": dist.get_world_size() if use_dist else None,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el * 1e3 / args.steps, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: U(-1,1) actions (seed 1234) from a fixed device buffer; Crazyflie constants; "
                    + ("dynamic_repulsive target and spawns (Philox seed 0)" if cfg.flavor == "A" else
                       "random 12-pillar maps + o_random/o_static_same_goal spawns (Philox seed 0)" if cfg.use_obstacles
                       else f"{cfg.quads_mode} goals and spawns (Philox seed 0)"),
            "config": {"workload": WORKLOAD[args.config], "envs_per_gpu": cfg.num_envs,
                       "agents_per_env": cfg.num_agents, "visible_neighbors": cfg.k_neighbors,
                       "obs_dim": cfg.obs_dim, "global_batch": world * I, "parallelism": f"env-shard x{world}",
                       "flavor": cfg.flavor, "episode_stats": bool(cfg.episode_stats), "launch": launch,
                       "blocks_ab_us_per_step": ab},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic,
                         "traffic_scope": "HBM bytes of one whole-shard step (PMC, one handle)",
                         "traffic_source": traffic_src,
                         "kernel": (f"qs::step_kernel_a<{npad(cfg.num_agents)}>" if cfg.flavor == "A" else
                                    f"qs::step_kernel<{npad(cfg.num_agents)}, {'true' if cfg.use_obstacles else 'false'}>"),
                         "kernel_us": round(k_ms * 1e3, 3),
                         "kernel_us_source": "HIP events on the launch stream over the timed region / steps"
                         + (f" (one step = {S} concurrent launches of {cfg.num_envs // S} envs; achieved = bytes per"
                            " step / step time, the aggregate rate of the overlapping launches)" if S > 1 else ""),
                         "launches_per_step": S,
                         "kernel_us_eager_single": round(k_eager_ms * 1e3, 3),
                         "bytes_per_agent_step": round(bpa, 1),
                         "bytes_per_agent_step_state_complete": (round(state_bytes_per_agent_step(cfg)[0], 1)
                                                                 if cfg.flavor == "B" else None),
                         # the PMC reads against the reads the step needs once its istate, stats ring and env
                         # words are counted (the FETCH x2 factor calibrated on the step's own load shape,
                         # tools/calib/fetch_calib read_sub64)
                         "read_ratio_state_complete": (round(traffic_src["read_bytes"] /
                                                             (state_bytes_per_agent_step(cfg)[1] * I), 3)
                                                       if cfg.flavor == "B" and traffic_src and
                                                       traffic_src.get("read_bytes") else None),
                         "bytes_per_launch": round(bpa * I / S),
                         "valu": valu_roofline(args.config, I, k_ms)},
            "window": window,
            "nonfinite_guard": guard,
            "cpu_baseline": None,
            "end_to_end": e2e,
        }
        if world == 1 and not args.no_cpu_baseline:
            try:
                out["cpu_baseline"] = cpu_baseline(args.config, seconds=args.cpu_seconds)
            except Exception as e:  # never let the baseline leg kill the GPU number
                out["cpu_baseline"] = {"error": repr(e)}
        print(json.dumps(out), flush=True)
    if blocks is not None:
        for eb, _, _ in blocks.entries:
            eb.close()
    env.close()
    if destroy_streams is not None:
        destroy_streams()
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
