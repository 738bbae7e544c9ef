set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config c3 --steps 2000 --no-cpu-baseline --e2e-iters 0 > gpurun_out/jit_base.log 2>&1 && \
QUADSWARM_LIB=$PWD/quad-swarm-rl-stable-baselines3_amd/quadswarm_amd/lib/libquadswarm_c3_jit.so timeout -k 10 300 python bench.py --config c3 --steps 2000 --no-cpu-baseline --e2e-iters 0 > gpurun_out/jit_c3.log 2>&1
rc=$?
tail -1 gpurun_out/jit_base.log | cut -c1-400; tail -1 gpurun_out/jit_c3.log | cut -c1-400
exit $rc
