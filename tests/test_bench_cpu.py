"""bench.py's multi-GPU entry on CPU: `--gpus N` starts N ranks through torch.distributed.run (argv checked,
the launch itself stubbed), a WORLD_SIZE / --gpus mismatch exits non-zero before touching a device, and the
line's aggregate (sum of the ranks' agent-steps / max-over-ranks seconds) is right at world size 2 (gloo)."""
import os
import socket
import subprocess
import sys

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_launcher_argv():
    argv = bench.launcher_argv(["--gpus", "8", "--steps", "20", "--warmup", "5"], 8, 29511)
    assert argv[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nnodes=1" in argv and "--nproc-per-node=8" in argv
    assert "--master-addr=127.0.0.1" in argv and "--master-port=29511" in argv
    i = argv.index(os.path.join(ROOT, "bench.py"))
    assert argv[i + 1:] == ["--gpus", "8", "--steps", "20", "--warmup", "5"]


def test_gpus_n_without_launcher_starts_ranks(monkeypatch):
    seen = {}

    class R:
        returncode = 3
        stdout = 'rank noise\n{"metric": "m", "n_gpus": 4}\n'

    def fake_run(cmd, **kw):
        seen["cmd"] = cmd
        return R()
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench.subprocess, "run", fake_run)
    with pytest.raises(SystemExit) as ex:
        bench.main(["--gpus", "4", "--steps", "7"])
    assert ex.value.code == 3                       # the child's exit code
    cmd = seen["cmd"]
    assert "--nproc-per-node=4" in cmd and cmd[-4:] == ["--gpus", "4", "--steps", "7"]


@pytest.mark.parametrize("world,gpus", [("2", "4"), ("4", "1"), ("1", "2")])
def test_world_gpus_mismatch_exits_nonzero(world, gpus):
    env = dict(os.environ, WORLD_SIZE=world, RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", gpus], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert f"--gpus {gpus} but the launcher started {world} rank" in r.stderr
    assert r.stdout.strip() == ""


def test_launch_world_checks():
    assert bench.launch_world(1, {}) == 1
    assert bench.launch_world(8, {"WORLD_SIZE": "8"}) == 8
    with pytest.raises(SystemExit):
        bench.launch_world(0, {})
    with pytest.raises(SystemExit):
        bench.launch_world(2, {"WORLD_SIZE": "1"})


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _agg_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, ROOT)
    import bench as b
    # rank r processed (r + 1) * 1000 agent-steps in (r + 2) seconds
    out = b.aggregate_ranks((rank + 1) * 1000, float(rank + 2), world, device="cpu")
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_aggregate_sum_over_max():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_agg_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in (0, 1):
        total, tmax, per_rank = got[r]
        assert total == 3000.0 and tmax == 3.0      # every rank sees the same aggregate
        assert per_rank == [500.0, 2000.0 / 3.0]
    assert bench.aggregate_ranks(500, 2.0, 1) == (500.0, 2.0, [250.0])


def test_state_complete_bytes():
    """The state-complete count adds to §8d's bytes what the reference's step also carries (istate words sized per
    swarm, the episode-stats words, the env words per drone): C2 / C3 / C5 / 128-drone values."""
    want = {"c2": (433.0, 216.0), "c3": (555.0, 197.0), "c5": (550.5, 193.25), "n128": (573.375, 204.3125)}
    for c, (b, r) in want.items():
        cfg = bench.make_cfg(bench.CONFIGS[c])
        got = bench.state_bytes_per_agent_step(cfg)
        assert abs(got[0] - b) < 1e-6 and abs(got[1] - r) < 1e-6, (c, got)
        base = bench.algorithmic_bytes_per_agent_step(cfg.obs_dim, cfg.num_agents, cfg.flavor)
        assert got[0] > base


def test_committed_pmc_reads_against_state_complete():
    """The committed round-5 PMC summaries (FETCH x2 calibrated on the step's own load shape,
    tools/calib/fetch_calib read_sub64) hold C2 / C3 reads within 10 % of the state-complete read count, as
    DESIGN.md states, and the pmc_traffic hand-off carries the correction's source."""
    for c in ("c2", "c3"):
        traffic, src = bench.pmc_traffic(c)
        assert traffic and src and src["correction"]["source"].endswith("read_sub64<true>"), (c, src)
        cfg = bench.make_cfg(bench.CONFIGS[c])
        ratio = src["read_bytes"] / (bench.state_bytes_per_agent_step(cfg)[1] * cfg.num_envs * cfg.num_agents)
        assert 1.0 <= ratio < 1.1, (c, ratio)


def test_every_bench_config_is_valid():
    """Every --config builds a configuration the C ABI accepts (layout query, no device): the sweep's configs,
    including the 128-drone flavor-A env (k = 7 <= QS_A_KMAX) and the obstacle / replay / mix variants."""
    from quadswarm_amd import _native as N
    L = N.lib()
    for name, kw in bench.CONFIGS.items():
        cfg = bench.make_cfg(kw)
        lay = N.QsLayout()
        assert L.qs_layout_query(cfg.to_qs_config(), lay) == 0, (name, L.qs_last_error())
        assert lay.obs_dim == cfg.obs_dim and lay.num_drones == cfg.num_envs * cfg.num_agents, name
