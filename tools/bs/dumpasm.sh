#!/bin/bash
# Device ISA of one slice kernel instantiation -> /tmp/bs.s; prints where scratch
# (spill) traffic sits relative to barriers and branches.
#   tools/bs/dumpasm.sh [MODE] [FULL(0|1)] [extra hipcc flags]
cd "$(dirname "$0")/../.." || exit 1
MODE=${1:-3}
FULL=${2:-1}
shift 2 2>/dev/null
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-gpu-flush-denormals-to-zero \
  -fhip-fp32-correctly-rounded-divide-sqrt -Iinclude -Ifate-llm_amd/csrc "$@" --cuda-device-only -S \
  fate-llm_amd/csrc/fks_device.hip -o /tmp/fks_dev.s 2>/dev/null
SYM="_ZN3fks12_GLOBAL__N_119fks_apply_bs_kernelILi${MODE}ELb$([ "$FULL" = 1 ] && echo 1 || echo 0)EEEvNS_11ApplyBsArgsE"
awk -v s="$SYM:" '$1 == s {on = 1} on {print} on && /s_endpgm/ {exit}' /tmp/fks_dev.s > /tmp/bs.s
echo "lines: $(wc -l < /tmp/bs.s)"
grep -n 'scratch_\|s_barrier\|s_cbranch\|^\.LBB' /tmp/bs.s | awk '{print $1, $2, $3}' | uniq -c -f1 | head -120
