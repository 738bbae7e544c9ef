#!/bin/bash
# round 5: FETCH_SIZE / WRITE_SIZE calibration on the step's own access shapes (tools/calib/fetch_calib), then the
# C2 / C3 phase stamps again on the rebuilt stamps library (scenario sub-phase slots handled when unstamped)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/calib_fetch gpurun_out/calib_write
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/calib_fetch -o cf --output-format csv -- ./tools/calib/fetch_calib > gpurun_out/calib_fetch.log 2>&1 || { tail -5 gpurun_out/calib_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/calib_write -o cw --output-format csv -- ./tools/calib/fetch_calib > gpurun_out/calib_write.log 2>&1 || { tail -5 gpurun_out/calib_write.log; exit 1; }
for c in c2 c3; do
  timeout -k 10 300 python tools/phase_stamps.py $c > gpurun_out/r05_stamps_$c.txt 2>&1 || { tail -5 gpurun_out/r05_stamps_$c.txt; exit 1; }
done
exit 0
