set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r05
timeout -k 10 400 python tools/scen_bitwise.py tools/jit/base_r04 1600 > gpurun_out/r05/scen_bitwise.log 2>&1; rc=$?; tail -30 gpurun_out/r05/scen_bitwise.log; [ $rc -gt 1 ] && exit $rc
MODES="static_diff_goal dynamic_formations dynamic_diff_goal swarm_vs_swarm mix" PMC=0 timeout -k 10 300 bash tools/r05_modes.sh || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity_scen.py tests/test_gpu_trainer.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r05/tests_scen_trainer.log 2>&1; rc=$?; tail -15 gpurun_out/r05/tests_scen_trainer.log; exit $rc
