#!/bin/bash
# GPU-box sequences, one target per argument (smoke, tests, bench, profiles, A/Bs).  Every step runs under its own
# time limit and the script stops at the first step that exits non-zero (a failed test, an exception, a crash, a
# time limit: round 5 let an rc = 1 illegal-address exception pass and carried on).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a gpurun_out/steps.log
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
: > gpurun_out/steps.log
for s in "$@"; do
  case $s in
    smoke) step smoke 400 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) step gpu_tests 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    testsel) step gpu_tests_sel 900 python -u -m pytest ${TESTS:?TESTS=<test files>} -x -v --timeout 200 --timeout-method thread ;;
    testsall) step gpu_tests 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread ;;
    testsnew) step gpu_tests_new 600 python -u -m pytest tests/test_gpu_stats.py tests/test_gpu_guard_params.py tests/test_gpu_c5.py -v --timeout 200 --timeout-method thread ;;
    testspar) step gpu_tests_par 900 python -u -m pytest tests/test_gpu_stats.py tests/test_gpu_parity.py tests/test_gpu_parity_a.py -v --timeout 300 --timeout-method thread ;;
    benchdrv) step bench_driver 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    benchwarm)
      step bw_20_5 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --e2e-iters 0
      step bw_20_500 200 python bench.py --steps 20 --warmup 500 --no-cpu-baseline --e2e-iters 0
      step bw_2000 200 python bench.py --steps 2000 --warmup 50 --no-cpu-baseline --e2e-iters 0
      ;;
    benchst)
      step bst_on 200 python bench.py --steps 2000 --warmup 50 --no-cpu-baseline --e2e-iters 0
      step bst_off 200 python bench.py --steps 2000 --warmup 50 --no-cpu-baseline --e2e-iters 0 --no-episode-stats
      ;;
    ktst)
      export TMPDIR=/tmp
      step kt_on 300 rocprofv3 --kernel-trace -d gpurun_out/kt_on -o kt --output-format csv -- python bench.py --steps 200 --warmup 10 --no-cpu-baseline --e2e-iters 0
      step kt_off 300 rocprofv3 --kernel-trace -d gpurun_out/kt_off -o kt --output-format csv -- python bench.py --steps 200 --warmup 10 --no-cpu-baseline --e2e-iters 0 --no-episode-stats
      python tools/kt_summary.py gpurun_out/kt_on gpurun_out/kt_off > gpurun_out/kt_summary.txt 2>&1
      rm -f gpurun_out/kt_*/*/*kernel_trace.csv gpurun_out/kt_*/*kernel_trace.csv
      ;;
    benchn64) step bench_n64 300 python bench.py --config n64 --steps 1000 --cpu-seconds 5 --e2e-iters 0 ;;
    abstatsa)
      step a8_nost 300 python bench.py --config a8 --steps 1000 --no-cpu-baseline --e2e-iters 0 --no-episode-stats
      CONFIG=a8 STEPS=1000 step a8_ab 600 bash tools/ab_jit.sh base: nocol:-DQS_DIAG_A_NOCOL
      ;;
    statsa)
      step stats_a 600 python -u -m pytest tests/test_gpu_stats.py tests/test_gpu_parity_a.py -v --timeout 200 --timeout-method thread
      step a8_after 300 python bench.py --config a8 --steps 1000 --no-cpu-baseline --e2e-iters 0
      ;;
    par64) step gpu_tests_64 600 python -u -m pytest tests/test_gpu_parity.py -v -k "64" --timeout 300 --timeout-method thread ;;
    benchblocks) step bench_blocks 600 python bench.py --steps 2000 --streams 4 --no-cpu-baseline --e2e-iters 0 ;;
    bench) step bench 600 python bench.py ;;
    ppotests) step ppo_tests 600 python -m pytest tests/test_gpu_ppo.py -q -x ;;
    e2ea) step e2e_a8 600 python bench.py --config a8 --steps 500 --no-cpu-baseline --e2e-iters 1 --e2e-steps 64 ;;
    e2ec3p)    # C3 end to end, the rollout encoders in fp32 and split-f16 (x3)
      step e2e_c3_fp32 600 python bench.py --config c3 --steps 500 --no-cpu-baseline --e2e-iters 2 --e2e-precision fp32
      step e2e_c3_x3 600 python bench.py --config c3 --steps 500 --no-cpu-baseline --e2e-iters 2 --e2e-precision x3
      ;;
    polt) step pol_tests 600 python -u -m pytest tests/test_gpu_policy_fused.py tests/test_gpu_ppo.py tests/test_gpu_trainer.py -x -v --timeout 200 --timeout-method thread ;;
    e2ec3) step e2e_c3 600 python bench.py --config c3 --steps 500 --no-cpu-baseline --e2e-iters 1 ;;
    e2ea512) step e2e_a8_512 900 python bench.py --config a8 --steps 500 --no-cpu-baseline --e2e-iters 2 ;;
    benchgen) step bench_generic 300 python bench.py --generic --steps 2000 --e2e-iters 0 --no-cpu-baseline ;;
    benchspec) step bench_spec 300 python bench.py --steps 2000 --e2e-iters 0 --no-cpu-baseline ;;
    benchc2) step bench_c2 400 python bench.py --config c2 --steps 2000 --cpu-seconds 10 --e2e-iters 1 ;;
    benchc5) step bench_c5 400 python bench.py --config c5 --steps 1000 --cpu-seconds 10 --e2e-iters 1 ;;
    e2ea8) step e2e_a8_full 900 python bench.py --config a8 --steps 500 --no-cpu-baseline --e2e-iters 1 ;;
    benchfast) step bench 300 python bench.py --steps 1000 --cpu-seconds 5 ;;
    bencha) step bench_a8 400 python bench.py --config a8 --steps 1000 --cpu-seconds 10 --e2e-iters 0 ;;
    bencha4) step bench_a4 400 python bench.py --config a4 --steps 1000 --cpu-seconds 5 ;;
    benchc4) step bench_c4 400 python bench.py --config c4 --steps 1000 --cpu-seconds 10 --e2e-iters 0 ;;
    benchc3) step bench_c3 400 python bench.py --config c3 --steps 2000 --cpu-seconds 10 ;;
    replay) step gpu_replay 600 python -u -m pytest tests/test_gpu_replay.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread ;;
    benchmixr) step bench_c3mixr 400 python bench.py --config c3mixr --steps 2000 --cpu-seconds 5 --e2e-iters 0 ;;
    benchc4dr) step bench_c4dr 400 python bench.py --config c4dr --steps 1000 --cpu-seconds 5 --e2e-iters 0 ;;
    benchmix) step bench_c3mix 400 python bench.py --config c3mix --steps 2000 --cpu-seconds 10 --e2e-iters 0 ;;
    prof)
      export TMPDIR=/tmp
      step prof_kt 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kt -o kt --output-format csv -- python bench.py --steps 1000 --no-cpu-baseline --e2e-iters 0
      step prof_fetch 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_fetch -o f --output-format csv -- python bench.py --steps 100 --warmup 10 --no-cpu-baseline --graph 0 --e2e-iters 0 --streams 1
      step prof_write 400 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_write -o w --output-format csv -- python bench.py --steps 100 --warmup 10 --no-cpu-baseline --graph 0 --e2e-iters 0 --streams 1
      step prof_sq 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_LDS -d gpurun_out/prof_sq -o s --output-format csv -- python bench.py --steps 100 --warmup 10 --no-cpu-baseline --graph 0 --e2e-iters 0 --streams 1
      rm -f gpurun_out/prof_*/*kernel_trace.csv
      ;;
    sweep)
      for c in c2 c3 c3mix c3mixr c4 c4dr c5 a8 a128 n64 n128; do
        step sweep_$c 200 python bench.py --config $c --steps 1000 --no-cpu-baseline --e2e-iters 0
      done
      ;;
    profdrv)
      export TMPDIR=/tmp
      step profdrv_kt 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profdrv_kt -o kt --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --e2e-iters 0
      rm -f gpurun_out/profdrv_kt/*kernel_trace.csv
      ;;
    profa)
      export TMPDIR=/tmp
      step profa_kt 400 rocprofv3 --kernel-trace --stats -d gpurun_out/profa_kt -o kt --output-format csv -- python bench.py --config a8 --steps 1000 --no-cpu-baseline --e2e-iters 0
      step profa_fetch 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/profa_fetch -o f --output-format csv -- python bench.py --config a8 --steps 100 --warmup 10 --no-cpu-baseline --graph 0 --e2e-iters 0
      step profa_write 400 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/profa_write -o w --output-format csv -- python bench.py --config a8 --steps 100 --warmup 10 --no-cpu-baseline --graph 0 --e2e-iters 0
      step profa_sq 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_LDS -d gpurun_out/profa_sq -o s --output-format csv -- python bench.py --config a8 --steps 100 --warmup 10 --no-cpu-baseline --graph 0 --e2e-iters 0
      rm -f gpurun_out/profa_*/*kernel_trace.csv
      ;;
    profe2e)
      export TMPDIR=/tmp
      step profe2e_kt 600 rocprofv3 --kernel-trace --stats -d gpurun_out/profe2e_kt -o kt --output-format csv -- python bench.py --config a8 --steps 200 --no-cpu-baseline --e2e-iters 1 --e2e-steps 64
      step profe2e_c3_kt 600 rocprofv3 --kernel-trace --stats -d gpurun_out/profe2e_c3_kt -o kt --output-format csv -- python bench.py --config c3 --steps 200 --no-cpu-baseline --e2e-iters 1
      rm -f gpurun_out/profe2e_kt/*kernel_trace.csv gpurun_out/profe2e_c3_kt/*kernel_trace.csv
      ;;
    tune)
      step tune_a8 900 env PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_a8_%d.csv python bench.py --config a8 --steps 200 --no-cpu-baseline --e2e-iters 1 --e2e-steps 64
      step tuned_a8 600 env PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_a8_%d.csv python bench.py --config a8 --steps 200 --no-cpu-baseline --e2e-iters 1 --e2e-steps 64
      ;;
    tunec3)
      step tune_c3 1100 env PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_MAX_TUNING_ITERATIONS=20 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_c3_%d.csv python bench.py --config c3 --steps 200 --no-cpu-baseline --e2e-iters 1
      ;;
    tunea512)
      step tune_a512 1100 env PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_MAX_TUNING_ITERATIONS=20 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_a512_%d.csv python bench.py --config a8 --steps 200 --no-cpu-baseline --e2e-iters 1
      ;;
    profc4)
      export TMPDIR=/tmp
      step profc4_kt 400 rocprofv3 --kernel-trace --stats -d gpurun_out/profc4_kt -o kt --output-format csv -- python bench.py --config c4 --steps 1000 --no-cpu-baseline --e2e-iters 0
      step profc4_fetch 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/profc4_fetch -o f --output-format csv -- python bench.py --config c4 --steps 100 --warmup 10 --no-cpu-baseline --graph 0 --e2e-iters 0
      step profc4_write 400 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/profc4_write -o w --output-format csv -- python bench.py --config c4 --steps 100 --warmup 10 --no-cpu-baseline --graph 0 --e2e-iters 0
      step profc4_sq 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_LDS -d gpurun_out/profc4_sq -o s --output-format csv -- python bench.py --config c4 --steps 100 --warmup 10 --no-cpu-baseline --graph 0 --e2e-iters 0
      rm -f gpurun_out/profc4_*/*kernel_trace.csv
      ;;
    profcfg)   # CONFIG=<name>: kernel trace + FETCH / WRITE / SQ passes of one bench config
      export TMPDIR=/tmp
      C=${CONFIG:-c3}
      step prof_${C}_kt 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${C}_kt -o kt --output-format csv -- python bench.py --config $C --steps 1000 --no-cpu-baseline --e2e-iters 0
      step prof_${C}_fetch 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_${C}_fetch -o f --output-format csv -- python bench.py --config $C --steps 100 --warmup 10 --no-cpu-baseline --graph 0 --e2e-iters 0
      step prof_${C}_write 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_${C}_write -o w --output-format csv -- python bench.py --config $C --steps 100 --warmup 10 --no-cpu-baseline --graph 0 --e2e-iters 0
      step prof_${C}_sq 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_LDS -d gpurun_out/prof_${C}_sq -o s --output-format csv -- python bench.py --config $C --steps 100 --warmup 10 --no-cpu-baseline --graph 0 --e2e-iters 0
      step prof_${C}_flops 300 timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_WAVES -d gpurun_out/prof_${C}_flops -o fl --output-format csv -- python bench.py --config $C --steps 100 --warmup 10 --no-cpu-baseline --graph 0 --e2e-iters 0
      rm -f gpurun_out/prof_${C}_*/*kernel_trace.csv gpurun_out/prof_${C}_*/*/*kernel_trace.csv
      ;;
    sel2)      # QS_NBR_SELECT2 on 32-drone envs: bitwise digest A/B + timing A/B
      step sel2_dig0 200 python tools/bitwise_ab.py c5 60
      step sel2_dig1 200 env QS_JIT_OPTS=-DQS_NBR_SELECT2=1 python tools/bitwise_ab.py c5 60
      CONFIG=c5 STEPS=2000 step sel2_ab 600 bash tools/ab_jit.sh base: sel2:-DQS_NBR_SELECT2=1 base2: sel2b:-DQS_NBR_SELECT2=1
      ;;
    stamps) step stamps 300 python tools/phase_stamps.py ;;
    profpol)   # the rollout policy's kernels (C3): kernel trace + one PMC pass of MFMA counters on the fused encoders
      export TMPDIR=/tmp
      step profpol_kt 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profpol_kt -o kt --output-format csv -- python tools/rollout_prof.py c3
      step profpol_pmc 200 timeout -s KILL 180 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --kernel-include-regex attn -d gpurun_out/profpol_pmc -o p --output-format csv -- python tools/rollout_prof.py c3
      rm -f gpurun_out/profpol_*/*kernel_trace.csv gpurun_out/profpol_*/*/*kernel_trace.csv
      ;;
    profpol2)  # the fused encoders' instruction mix (one PMC pass)
      export TMPDIR=/tmp
      step profpol2_pmc 200 timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES --kernel-include-regex attn -d gpurun_out/profpol2_pmc -o p --output-format csv -- python tools/rollout_prof.py c3
      ;;
    n128) step gpu_tests_n128 900 python -u -m pytest tests/test_gpu_n128.py -x -v --timeout 300 --timeout-method thread ;;
    benchn128) step bench_n128 300 python bench.py --config n128 --steps 500 --cpu-seconds 5 --e2e-iters 0 ;;
    prioab)    # the younger-wave priority flip (QS_PRIO_AT, default 11) against off, per config
      for c in c3 c4 c3mix c5 c2; do
        CONFIG=$c STEPS=1000 step prioab_$c 300 bash tools/ab_jit.sh on: off:-DQS_PRIO_AT=-1 on2: off2:-DQS_PRIO_AT=-1
      done
      ;;
    calib)
      export TMPDIR=/tmp
      step calib_fetch 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/calib_fetch -o cf --output-format csv -- ./tools/calib/fetch_calib
      step calib_write 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/calib_write -o cw --output-format csv -- ./tools/calib/fetch_calib
      ;;
    final)     # the committed tree: smoke, the whole -m gpu suite, the default bench line
      step smoke_final 400 python -c "import __graft_entry__ as g; g.smoke()"
      step gpu_suite_final 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
      step bench_default 900 python bench.py
      ;;
    profall)   # CONFIGS (default "c3 c2 a8 c3mix c4 c5"): profcfg per config
      for c in ${CONFIGS:-c3 c2 a8 c3mix c4 c5}; do
        rm -rf gpurun_out/prof_${c}_*
        CONFIG=$c bash "$0" profcfg || exit $?
      done
      ;;
    stampsbc)  # phase stamps of C2 / C3 (the stamps library)
      for c in ${CONFIGS:-c2 c3}; do step stamps_$c 300 python tools/phase_stamps.py $c; done
      ;;
    modes)     # per-goal-scenario step time of the C3 swarm (MODES overrides the list)
      for m in ${MODES:-static_same_goal static_diff_goal ep_lissajous3D ep_rand_bezier dynamic_same_goal dynamic_diff_goal dynamic_formations swap_goals swarm_vs_swarm mix}; do
        step mode_$m 200 python bench.py --config c3mix --quads-mode $m --steps 1000 --no-cpu-baseline --e2e-iters 0
      done
      ;;
    scenbit)   # scenario kernels bitwise against a base source tree (BASE, same ABI), then the scenario parity tests
      step scen_bitwise 400 python tools/scen_bitwise.py ${BASE:-tools/jit/base_r06} 1600
      step scen_tests 400 python -u -m pytest tests/test_gpu_parity_scen.py -q --timeout 200 --timeout-method thread
      ;;
    polab)     # policy-kernel A/B: one C3 end-to-end iteration under a kernel trace per library (LIBS="name ...",
               # quadswarm_amd/lib/ab/libquadswarm_<name>.so from tools/build_pol_variant.sh; "base" = the in-tree library)
      export TMPDIR=/tmp
      for v in ${LIBS:?LIBS=<variant names>}; do
        if [ "$v" = base ]; then unset QUADSWARM_LIB; else
          export QUADSWARM_LIB=$PWD/quad-swarm-rl-stable-baselines3_amd/quadswarm_amd/lib/ab/libquadswarm_$v.so; fi
        step polab_$v 500 rocprofv3 --kernel-trace --stats -d gpurun_out/polab_$v -o e2e --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --e2e-iters 1
        python3 tools/kstats.py gpurun_out/polab_$v 40 > gpurun_out/polab_${v}_summary.txt 2>&1
        python3 tools/e2e_split.py gpurun_out/polab_$v --top 40 > gpurun_out/polab_${v}_split.txt 2>&1
        find gpurun_out/polab_$v -name "*kernel_trace.csv" -delete
      done
      unset QUADSWARM_LIB
      ;;
    e2eprof)   # kernel trace of one C3 end-to-end PPO iteration (where update_s goes)
      export TMPDIR=/tmp
      step e2eprof_kt 500 rocprofv3 --kernel-trace --stats -d gpurun_out/e2eprof -o e2e --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --e2e-iters 1
      python3 tools/kstats.py gpurun_out/e2eprof > gpurun_out/e2eprof_summary.txt 2>&1
      find gpurun_out/e2eprof -name "*kernel_trace.csv" -delete
      ;;
    a8e2e)     # flavor-A end to end (sb_train settings, n_steps 64) with the fused update vs torch fp32
      for up in x3 fp32; do
        step a8_e2e_$up 500 python bench.py --config a8 --steps 100 --no-cpu-baseline --e2e-iters 1 --e2e-steps 64 --e2e-update-precision $up
      done
      ;;
    torchrun1) # the N > 1 launch path rehearsed at world size 1: RCCL initialised (QS_BENCH_DIST=1)
      step bench_torchrun1 600 env QS_BENCH_DIST=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 2000 --no-cpu-baseline
      ;;
    window)    # the driver's 20-step window: its split (tools/window_probe.py) and a per-dispatch trace of the driver command
      export TMPDIR=/tmp
      step window_probe 300 python tools/window_probe.py
      rm -rf gpurun_out/window_kt
      step window_kt 300 rocprofv3 --kernel-trace --stats -d gpurun_out/window_kt -o kt --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --e2e-iters 0
      python3 tools/dispatch_summary.py gpurun_out/window_kt --all > gpurun_out/window_dispatch.txt 2>&1
      find gpurun_out/window_kt -name "*kernel_trace.csv" -delete
      ;;
    abjit)     # interleaved A/B of a kernel macro: CONFIGS, AB="tag:-DX=0 tag2:" (twice each, in order)
      for c in ${CONFIGS:-c3}; do
        CONFIG=$c STEPS=${STEPS:-2000} step abjit_$c 900 bash tools/ab_jit.sh ${AB:?AB=tag:defs ...} ${AB}
      done
      ;;
    absrc)     # bitwise digest + timing A/B against a base kernel tree: CONFIGS, BASE (default tools/jit/base_r06)
      for c in ${CONFIGS:-c3}; do
        CONFIG=$c STEPS=${STEPS:-2000} ROUNDS=${ROUNDS:-1} step absrc_$c 900 bash tools/ab_src.sh base:${BASE:-tools/jit/base_r06} new:
      done
      ;;
    launch)    # launch-path A/B of the driver's 20-step window (tools/launch_probe.py)
      step launch_probe 300 python tools/launch_probe.py --reps 10
      ;;
    mixtrace)  # per-dispatch trace of c3mix (the slow-launch outlier)
      export TMPDIR=/tmp
      rm -rf gpurun_out/mixtrace_kt
      step mixtrace_kt 300 rocprofv3 --kernel-trace --stats -d gpurun_out/mixtrace_kt -o kt --output-format csv -- python bench.py --config c3mix --steps 1000 --no-cpu-baseline --e2e-iters 0
      python3 tools/dispatch_summary.py gpurun_out/mixtrace_kt > gpurun_out/mixtrace_dispatch.txt 2>&1
      python3 tools/dispatch_summary.py gpurun_out/mixtrace_kt --match reset_kernel >> gpurun_out/mixtrace_dispatch.txt 2>&1
      find gpurun_out/mixtrace_kt -name "*kernel_trace.csv" -delete
      ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
