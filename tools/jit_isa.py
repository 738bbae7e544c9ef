#!/usr/bin/env python
"""Diagnostic: the ISA of a config's specialised step kernel (what qs_specialize compiles with hipRTC), built
offline with hipcc from the same sources and parameter words, plus instruction counts.

    python tools/jit_isa.py a8 [out.s]        (bench.py config names; QS_JIT_OPTS as for qs_specialize; QS_MODE=<quads_mode>)"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "quad-swarm-rl-stable-baselines3_amd")
sys.path.insert(0, PKG)
sys.path.insert(0, ROOT)


def main():
    import ctypes
    import bench
    from quadswarm_amd import _native as N
    config = sys.argv[1] if len(sys.argv) > 1 else "c3"
    out = sys.argv[2] if len(sys.argv) > 2 else f"/tmp/{config}_step.s"
    over = dict(bench.CONFIGS[config])
    if os.environ.get("QS_MODE"):   # a goal scenario for the swarm configs (bench.py --quads-mode)
        over["quads_mode"] = os.environ["QS_MODE"]
    cfg = bench.make_cfg(over, seed=0, specialize=True)
    qc = cfg.to_qs_config()
    L = N.lib()
    buf = (ctypes.c_uint32 * 8192)()
    n = L.qs_config_kp_words(qc, buf, 8192)
    assert n > 0, L.qs_last_error()
    words = list(buf[:n])
    seed_idx = 15   # KP.seed (id0 is word 14): zeroed as kp_words() does
    words[seed_idx] = 0
    npad = 1 << (cfg.num_agents - 1).bit_length()
    flavor_a = cfg.flavor == "A"
    kern = f"qs::step_kernel_a<{npad}>" if flavor_a else f"qs::step_kernel<{npad}, {'true' if cfg.use_obstacles else 'false'}>"
    sig = "(const qs::KP*, qs::Bufs)" if flavor_a else "(const qs::KP*, qs::Bufs, const qs::RArgs*)"
    src = (f"#define QS_JIT 1\n#define QS_QB {os.environ.get('QS_QB', 4)}\n#define QS_QA {os.environ.get('QS_QA', 2)}\n#define QS_KP_WORDS " +
           ",".join(f"0x{w:08x}u" for w in words) + "\n" +
           f'#include "{"qs_flavor_a.h" if flavor_a else "qs_flavor_b.h"}"\n' +
           f"template __global__ void {kern}{sig};\n")
    with tempfile.TemporaryDirectory() as d:
        f = os.path.join(d, "jit.hip")
        open(f, "w").write(src)
        # the hipRTC options of qs_step.hip jit_compile (scheduler, no SLP packing, flavor A's denormal flush)
        jit = ["-mllvm", "-amdgpu-sched-strategy=max-ilp", "-fno-slp-vectorize"] + \
            (["-fgpu-flush-denormals-to-zero"] if flavor_a else [])
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=on",
                        "-munsafe-fp-atomics", "--cuda-device-only", "-S"] + jit + ["-I",
                        os.environ.get("QS_JIT_SRC_DIR", os.path.join(PKG, "csrc")), "-I",
                        os.path.join(ROOT, "include"), f, "-o", out] + os.environ.get("QS_JIT_OPTS", "").split(),
                       check=True)
    text = open(out).read()
    body = text[text.index(".text"):]
    ins = [ln.split()[0] for ln in body.splitlines() if ln.startswith("\t") and not ln.startswith("\t.")
           and not ln.startswith("\t;")]
    cnt = {}
    for i in ins:
        k = "v_mfma" if i.startswith("v_mfma") else i.split("_")[0] + "_" if "_" in i else i
        cnt[k] = cnt.get(k, 0) + 1
    print(f"{config}: {kern}: {len(ins)} static instructions -> {out}")
    print("  " + ", ".join(f"{k}* {v}" for k, v in sorted(cnt.items(), key=lambda kv: -kv[1])[:10]))


if __name__ == "__main__":
    main()
