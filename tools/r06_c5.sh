#!/bin/bash
# Round 6: the C5 client round on both streams with the D2H leg (the path ends in host
# memory), pinned model_0, 3 rounds, warm.  Output: gpurun_out/r06_c5/
OUT=gpurun_out/r06_c5
mkdir -p $OUT
FKS_STREAM_MODE=auto timeout -k 10 600 python -u harness/c5_round.py --rounds 3 --warm --placement pinned --d2h \
  > $OUT/c5_auto_d2h.json 2> $OUT/c5_auto_d2h.err \
  && FKS_STREAM_MODE=torch_cpu timeout -k 10 600 python -u harness/c5_round.py --rounds 3 --warm --placement pinned --d2h \
  > $OUT/c5_torch_cpu_d2h.json 2> $OUT/c5_torch_cpu_d2h.err
