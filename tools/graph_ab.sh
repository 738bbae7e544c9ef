# driver-argument bench (--steps 20 --warmup 5): hipGraph replays (default) vs eager launches (--graph 0), alternated
mkdir -p gpurun_out/ga
for r in 1 2 3; do
  for g in 100 0; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --e2e-iters 0 --graph $g > gpurun_out/ga/g$g-$r.log 2>&1 || exit $?
    echo "graph$g $r $(tail -1 gpurun_out/ga/g$g-$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_us"])')"
  done
done
