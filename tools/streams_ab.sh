cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/s_ab
for s in 1 4 2; do
  timeout -k 10 200 python bench.py --config c3 --steps 2000 --streams $s --no-cpu-baseline --e2e-iters 0 > gpurun_out/s_ab/c3_s$s.log 2>&1 || exit 1
  echo "S=$s $(tail -1 gpurun_out/s_ab/c3_s$s.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["roofline"]["kernel_us"], d["ms_per_step"], d["config"]["launch"], d["config"].get("blocks_ab_us_per_step"))')"
done
