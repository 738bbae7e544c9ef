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
