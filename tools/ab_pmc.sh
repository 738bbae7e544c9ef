#!/bin/bash
# Per-wave SQ counters of the step kernel for kernel variants (QS_JIT_OPTS), one rocprofv3 --pmc pass each:
#   bash tools/ab_pmc.sh tag:-DMACRO[,-DMACRO2] ...      (CONFIG from the environment, default c3)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CONFIG=${CONFIG:-c3}
mkdir -p gpurun_out/ab_pmc
for spec in "$@"; do
  tag=${spec%%:*}; defs=${spec#*:}; defs=${defs//,/ }
  rm -rf gpurun_out/ab_pmc/${CONFIG}_$tag
  QS_JIT_OPTS="$defs" timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY \
      SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_LDS -d gpurun_out/ab_pmc/${CONFIG}_$tag -o s \
      --output-format csv -- python bench.py --config $CONFIG --steps 40 --warmup 5 --graph 0 --no-cpu-baseline \
      --e2e-iters 0 > gpurun_out/ab_pmc/${CONFIG}_$tag.log 2>&1
  rc=$?
  echo "$CONFIG $tag rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
  rm -f gpurun_out/ab_pmc/${CONFIG}_$tag/*kernel_trace.csv
done
python3 tools/ab_pmc_summary.py
