# 32-drone neighbour picks (QS_NBR_PICK32) A/B: digests (HEAD headers vs this tree, pick on), then timing
B=$PWD/tools/jit/base_h
mkdir -p gpurun_out
( QS_JIT_SRC_DIR=$B timeout -k 10 150 python tools/bitwise_ab.py c5 30 && timeout -k 10 150 python tools/bitwise_ab.py c5 30 && QS_JIT_OPTS=-DQS_NBR_PICK32=1 timeout -k 10 150 python tools/bitwise_ab.py c5 30 && QS_JIT_SRC_DIR=$B timeout -k 10 150 python tools/bitwise_ab.py c3 30 && timeout -k 10 150 python tools/bitwise_ab.py c3 30 ) > gpurun_out/pick_dig.log 2>&1 || exit $?
CONFIG=c5 STEPS=1000 timeout -k 10 400 bash tools/ab_jit.sh base: pick:-DQS_NBR_PICK32=1 base2: pick2:-DQS_NBR_PICK32=1
