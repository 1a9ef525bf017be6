#!/bin/bash
# Register/scratch usage of the slice kernel instantiations (compile only, no GPU):
#   tools/bs/resusage.sh [extra hipcc flags]
cd "$(dirname "$0")/../.." || exit 1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-gpu-flush-denormals-to-zero \
  -fhip-fp32-correctly-rounded-divide-sqrt -Iinclude -Ifate-llm_amd/csrc "$@" -c fate-llm_amd/csrc/fks_device.hip \
  -o /tmp/fks_dev_ru.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  grep -A12 'fks_apply_bs' | grep -E 'Function Name|VGPRs:|VGPRs Spill|SGPRs Spill|ScratchSize' |
  sed -e 's/.*remark: *//' -e 's/ \[-Rpass.*//'
