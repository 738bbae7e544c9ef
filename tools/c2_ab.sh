# C2 (16 384 single drones): sub-lanes per drone (QS_QB env: 4 default, 2, 1) and SLP vectorisation off, HIP events
mkdir -p gpurun_out/c2ab
for r in 1 2; do
  for v in q4 q2 q1 noslp; do
    case $v in
      q4) E="QS_QB=4" ;; q2) E="QS_QB=2" ;; q1) E="QS_QB=1" ;; noslp) E="QS_JIT_OPTS=-fno-slp-vectorize" ;;
    esac
    timeout -k 10 200 env $E python bench.py --config c2 --steps 2000 --no-cpu-baseline --e2e-iters 0 > gpurun_out/c2ab/$v$r.log 2>&1 || exit $?
    echo "c2 $v $r $(tail -1 gpurun_out/c2ab/$v$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_us"])')"
  done
done
