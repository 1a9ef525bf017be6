#!/bin/bash
# Round-5 closing run: the build, smoke, the whole GPU suite and the default bench on the
# final tree, then one client's warm 7B round (pinned model_0, 3 rounds) drawn from the
# torch_cpu stream and from the default "auto" stream (torch_rocm on the GPU).
set -o pipefail
bash tools/gpu.sh r05f smoke pytestall bench || exit $?
OUT=gpurun_out/r05f
timeout -k 10 600 python -u harness/c5_round.py --rounds 3 --warm --placement pinned > $OUT/10_c5_torch_cpu.json 2> $OUT/10_c5_torch_cpu.err \
  && FKS_STREAM_MODE=auto timeout -k 10 600 python -u harness/c5_round.py --rounds 3 --warm --placement pinned > $OUT/11_c5_auto.json 2> $OUT/11_c5_auto.err
