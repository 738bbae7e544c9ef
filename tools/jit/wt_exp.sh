set -u
mkdir -p gpurun_out
L=$PWD/quad-swarm-rl-stable-baselines3_amd/quadswarm_amd/lib
for rep in 1 2; do
for v in "" _wto _wtos; do
  QUADSWARM_LIB=$L/libquadswarm_c3_jit$v.so timeout -k 10 120 python bench.py --generic --steps 3000 --no-cpu-baseline --e2e-iters 0 > gpurun_out/wt$v.$rep.log 2>&1 || exit $?
  python -c "import json,sys; d=json.loads(open('gpurun_out/wt$v.$rep.log').read().strip().splitlines()[-1]); print('$v', $rep, d['ms_per_step']*1e3, d['roofline']['kernel_us'])"
done; done
