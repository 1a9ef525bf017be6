#!/bin/bash
# C5 measurements, round 2 (repo root on the GPU box): one client, LLaMA-7B bf16, warm
# aggregator (all 4096 seeds replayed), 151 local steps; model_0 placements and drivers.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${TAG:-r02}
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python3 -u harness/c5_round.py --warm --k 4096 --steps 151 "$@" > gpurun_out/${TAG}_c5_$n.json 2> gpurun_out/${TAG}_c5_$n.err || { tail -5 gpurun_out/${TAG}_c5_$n.err; exit 9; }
  tail -c 700 gpurun_out/${TAG}_c5_$n.json; echo
}
run host --rounds 1 --placement host
run pinned --rounds 2 --placement pinned
run device --rounds 1 --placement device
run trainer_wire --rounds 2 --placement pinned --driver trainer --wire
