#!/bin/bash
# round-5 GPU check 23: the physics substep with fewer divergent blocks (Rodrigues' Taylor coefficients on every lane,
# the rare large-angle lanes overwriting them; the floor branch's acceleration after it; tools/jit/rb = a copy of the
# kernel headers with that change) against the library: bitwise digests + interleaved timing, a8 / C3
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for c in a8 c3; do
  CONFIG=$c STEPS=2000 ROUNDS=2 timeout -k 10 500 bash tools/ab_src.sh base: rb:tools/jit/rb || exit $?
done
