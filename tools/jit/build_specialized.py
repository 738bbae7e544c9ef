#!/usr/bin/env python
"""Experiment: build libquadswarm with the parameter block of one bench config baked in (-DQS_JIT).

    python tools/jit/build_specialized.py --config c3   -> quadswarm_amd/lib/libquadswarm_<config>_jit.so
Run the bench against it with QUADSWARM_LIB=<that .so> (same ABI)."""
import argparse
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "quad-swarm-rl-stable-baselines3_amd"))


def main():
    import bench
    from quadswarm_amd import _native as NAT
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--stamps", action="store_true", help="also -DQS_STAMPS=1 (tools/phase_stamps.py)")
    ap.add_argument("-D", dest="defines", action="append", default=[], help="extra -D macro (experiments)")
    ap.add_argument("--tag", default="", help="suffix of the output library name")
    a = ap.parse_args()
    cfg = bench.make_cfg(bench.CONFIGS[a.config], seed=0)
    qc = cfg.to_qs_config()
    buf = (ctypes.c_uint32 * 4096)()
    L = NAT.lib()
    L.qs_config_kp_words.argtypes = [ctypes.POINTER(NAT.QsConfig), ctypes.c_void_p, ctypes.c_size_t]
    n = L.qs_config_kp_words(qc, buf, 4096)
    assert n > 0, NAT.lib().qs_last_error()
    words = ",".join(f"0x{buf[i]:08x}u" for i in range(n))
    pkg = os.path.join(ROOT, "quad-swarm-rl-stable-baselines3_amd")
    out = os.path.join(pkg, "quadswarm_amd", "lib", f"libquadswarm_{a.config}_jit{'_stamps' if a.stamps else ''}{a.tag}.so")
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
           f"-I{ROOT}/include", f"-I{pkg}/csrc", "-munsafe-fp-atomics", "-ffp-contract=on", "-DQS_JIT", f"-DQS_KP_WORDS={words}",
           "-o", out, os.path.join(pkg, "csrc", "qs_step.hip"), "-lhiprtc"]
    if a.stamps:
        cmd.insert(-4, "-DQS_STAMPS=1")
    for d in a.defines:
        cmd.insert(-4, "-D" + d)
    subprocess.check_call(cmd)
    print(out)


if __name__ == "__main__":
    main()
