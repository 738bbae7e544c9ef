#!/bin/bash
# A/B builds of the policy translation unit: links quadswarm_amd/lib/ab/libquadswarm_<name>.so from the env object
# (build/qs_step.o, `make`) and csrc/qs_policy_api.hip compiled with the given -D flags.  Selected at run time by
# QUADSWARM_LIB (gpu_check.sh polab).
#   bash tools/build_pol_variant.sh <name> [-DFLAG=V ...]
set -eu
cd "$(dirname "$0")/../quad-swarm-rl-stable-baselines3_amd"
name=$1; shift
mkdir -p build quadswarm_amd/lib/ab
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../include -Icsrc -munsafe-fp-atomics -ffp-contract=on \
  -Wall -Wno-unused-result "$@" -c -o "build/pol_$name.o" csrc/qs_policy_api.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "quadswarm_amd/lib/ab/libquadswarm_$name.so" build/qs_step.o \
  "build/pol_$name.o" -lhiprtc
echo "built quadswarm_amd/lib/ab/libquadswarm_$name.so"
