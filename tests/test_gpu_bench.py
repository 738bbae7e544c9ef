"""bench.py at the driver's arguments (`--steps 20 --warmup 5`): every timed step is a hipGraph replay of the
specialised step kernel (no eager fallback), the line carries BASELINE.json's metric, and its roofline
figures are consistent with the measured kernel time."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_driver_arguments_replay_graphs():
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "1", "--steps", "20", "--warmup", "5",
                        "--no-cpu-baseline", "--e2e-iters", "0"], cwd=ROOT, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        base = json.load(f)
    assert line["metric"] == base["metric"] and line["unit"] == "agent-steps/s"
    assert line["n_gpus"] == 1 and line["steps"] == 20 and line["warmup"] == 5 and line["higher_is_better"]
    launch = line["config"]["launch"]
    assert launch.startswith("1 hipGraph replays") and "eager" not in launch and "specialised" in launch
    rf = line["roofline"]
    assert rf["bound"] == "hbm" and rf["peak"] == 8000.0 and 0.0 < rf["frac"] < 1.0
    assert rf["bytes_per_launch"] == 489 * 32768
    # achieved = algorithmic bytes per launch / the HIP-event kernel time
    assert abs(rf["achieved"] - rf["bytes_per_launch"] / (rf["kernel_us"] * 1e-6) / 1e9) <= 0.01 * rf["achieved"]
    # the wall-clock step (what `value` is computed from) includes the kernel
    assert line["ms_per_step"] * 1e3 >= 0.95 * rf["kernel_us"]
    assert abs(line["value"] - 32768 / (line["ms_per_step"] * 1e-3)) <= 0.01 * line["value"]
    assert line["nonfinite_guard"] == {"nonfinite_obs": 0, "nonfinite_rew": 0, "nonfinite_state": 0}


@pytest.mark.gpu
def test_step_n_equals_repeated_steps():
    """qs_step_n (the eager launch loop from one C call) == the same number of qs_step calls, bitwise."""
    import torch
    sys.path.insert(0, ROOT)
    import bench
    from quadswarm_amd.env import QuadSwarmEnv
    dev = torch.device("cuda:0")
    outs = []
    for use_n in (False, True):
        cfg = bench.make_cfg(dict(bench.CONFIGS["c3"], num_envs=64), seed=0, specialize=True)
        env = QuadSwarmEnv(cfg, device=dev)
        g = torch.Generator(device=dev).manual_seed(7)
        acts = (torch.rand(env.I, 4, device=dev, generator=g) * 2 - 1).contiguous()
        env.reset()
        if use_n:
            env.step_n(acts, 12)
        else:
            for _ in range(12):
                env.step(acts)
        torch.cuda.synchronize()
        outs.append((env.obs.clone(), env.rew.clone(), env.done.clone()))
        env.close()
    for a, b in zip(*outs):
        assert torch.equal(a, b)
