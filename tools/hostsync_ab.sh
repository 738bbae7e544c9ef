# driver-argument bench (--steps 20 --warmup 5) with the host wait spinning vs HIP's default, alternated
mkdir -p gpurun_out/hs
for r in 1 2 3; do
  for m in auto spin; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --e2e-iters 0 --host-sync $m > gpurun_out/hs/$m$r.log 2>&1 || exit $?
    echo "$m $r $(tail -1 gpurun_out/hs/$m$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_us"])')"
  done
done
