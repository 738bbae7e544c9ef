#!/bin/bash
# round-5 GPU check 18: flavor A's neighbour pass with the exchange rows read back to back outside the divergent
# per-neighbour blocks (QS_NBR_HOIST; tools/jit/nh = the working tree's kernel headers) against the library's embedded
# sources: bitwise digests + interleaved timing, a8 / a4
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for c in a8 a4; do
  CONFIG=$c STEPS=2000 ROUNDS=2 timeout -k 10 500 bash tools/ab_src.sh base: nh:tools/jit/nh || exit $?
done
