#!/bin/bash
# round-5 GPU check 24: C2 / c3mix with the branch-light substep (the library) against the previous substep
# (tools/jit/old = the kernel headers with qs_common.h of 34f65c1): bitwise digests + interleaved timing
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for c in c2 c3mix; do
  CONFIG=$c STEPS=2000 ROUNDS=2 timeout -k 10 500 bash tools/ab_src.sh new: old:tools/jit/old || exit $?
done
