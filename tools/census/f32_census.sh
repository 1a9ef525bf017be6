#!/bin/bash
# Census of the fp32 19-seed kernel (fks_apply_kernel<FKS_F32, kModeUpdateWd, FULL>, the C4
# 70B chain) by removal: the main loop's static VALU count of the in-tree kernel and of
# wrong-value variants with one part of the z pipeline replaced by an identity
# (compile-only; tools/census/isa_census.py counts).  Per block the loop serves 19 seeds x
# one Box-Muller pair per lane.
cd "$(dirname "$0")/../.." || exit 1
SYM=fks_apply_kernelILi0ELi3ELb1ELb0E
run() {  # name, python edit of the source
  python - "$2" > /tmp/census_src.hip <<'PY'
import sys
s = open("fate-llm_amd/csrc/fks_device.hip").read()
exec(sys.argv[1])
sys.stdout.write(s)
PY
  cp /tmp/census_src.hip fate-llm_amd/csrc/.census_tmp.hip
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-gpu-flush-denormals-to-zero \
    -fhip-fp32-correctly-rounded-divide-sqrt -Iinclude -Ifate-llm_amd/csrc --cuda-device-only -S \
    fate-llm_amd/csrc/.census_tmp.hip -o /tmp/census.s 2>/dev/null
  rm -f fate-llm_amd/csrc/.census_tmp.hip
  printf '%-28s ' "$1"
  python tools/census/isa_census.py /tmp/census.s $SYM --top 0 | sed -n 2p
}
run in-tree 'pass'
run sqrt=raw_v_sqrt 's = s.replace("__device__ __forceinline__ float radius_sqrt(float x) { return sqrtf(x); }", "__device__ __forceinline__ float radius_sqrt(float x) { return __builtin_amdgcn_sqrtf(x); }")'
run sqrt=identity 's = s.replace("__device__ __forceinline__ float radius_sqrt(float x) { return sqrtf(x); }", "__device__ __forceinline__ float radius_sqrt(float x) { return x; }")'
run log=identity 's = s.replace("const float radius = radius_sqrt(-2.0f * cephes_logf(1.0f - d1));", "const float radius = radius_sqrt(-2.0f * (1.0f - d1));")'
run sincos=identity 's = s.replace("  cephes_sincosf_nonneg(6.28318548202514648438f * d2, s, c);\n  z1", "  s = d2; c = 6.28318548202514648438f * d2;\n  z1")'
run temper=identity 's = s.replace("  const u32x2_t t = temper_pair_u24(w);\n  const float d1", "  const u32x2_t t = w;\n  const float d1")'
run z=raw_words 's = s.replace("  const u32x2_t t = temper_pair_u24(w);\n  const float d1 = (float)t.x * (1.0f / 16777216.0f);\n  const float d2 = (float)t.y * (1.0f / 16777216.0f);\n  const float radius = radius_sqrt(-2.0f * cephes_logf(1.0f - d1));\n  float s, c;\n  cephes_sincosf_nonneg(6.28318548202514648438f * d2, s, c);\n  z1 = __fmaf_rn(radius, c, 0.0f);\n  z2 = __fmaf_rn(radius, s, 0.0f);", "  z1 = __uint_as_float(r1); z2 = __uint_as_float(r2);")'
run twist=none 's = s.replace("      twist_all(plan, nseeds);  // the raw words of stream block b", "      (void)plan;")'
