#!/bin/bash
# round-5 GPU check 20: flavor A's per-tick collision row with the partner tests that are constants folded away
# (QS_COL_FOLD; tools/jit/cf = the working tree's kernel headers) against the library's embedded sources: bitwise
# digests + interleaved timing, a8 (3 rounds)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CONFIG=a8 STEPS=2000 ROUNDS=3 timeout -k 10 600 bash tools/ab_src.sh base: cf:tools/jit/cf || exit $?
