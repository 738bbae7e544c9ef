#!/bin/bash
# round-5 GPU check 21: flavor A's tick loop without the env-range test in its `active` mask (QS_ACT_FOLD;
# tools/jit/af = the working tree's kernel headers) against the library's embedded sources: bitwise digests +
# interleaved timing, a8 (3 rounds) and a4
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CONFIG=a8 STEPS=2000 ROUNDS=3 timeout -k 10 600 bash tools/ab_src.sh base: af:tools/jit/af || exit $?
CONFIG=a4 STEPS=2000 ROUNDS=1 timeout -k 10 400 bash tools/ab_src.sh base: af:tools/jit/af || exit $?
