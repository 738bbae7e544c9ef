#!/bin/bash
# round-5 final check on the committed tree: smoke, the whole -m gpu suite, the default bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05/smoke_final.log 2>&1 || { tail -5 gpurun_out/r05/smoke_final.log; exit 1; }
tail -2 gpurun_out/r05/smoke_final.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r05/gpu_suite_final.log 2>&1; rc=$?
tail -4 gpurun_out/r05/gpu_suite_final.log; [ $rc -ne 0 ] && exit $rc
grep -h "max |pid" gpurun_out/r05/gpu_suite_final.log | head -3
exit 0
