"""Build an A/B variant of the device code from a text patch of csrc/fks_device.hip
(timing experiments; the patched source stays under fate-llm_amd/build/, never in tree):
  python tools/r03/mkvariant.py [--base FILE] NAME 'old1' 'new1' ['old2' 'new2' ...]
-> fate-llm_amd/build/libfks_NAME.so (each `old` must occur exactly once; --base: patch
another copy of the device source instead of csrc/fks_device.hip)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = os.path.join(ROOT, "fate-llm_amd")


def main():
    args = sys.argv[1:]
    base = os.path.join(PKG, "csrc", "fks_device.hip")
    if args[0] == "--base":
        base, args = args[1], args[2:]
    name, pairs = args[0], args[1:]
    src = open(base).read()
    for old, new in zip(pairs[0::2], pairs[1::2]):
        n = src.count(old)
        if n != 1:
            raise SystemExit(f"{name}: {n} matches for {old[:80]!r}")
        src = src.replace(old, new)
    out = os.path.join(PKG, "build", f"fks_device_{name}.hip")
    open(out, "w").write(src)
    flags = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-gpu-flush-denormals-to-zero",
             "-fhip-fp32-correctly-rounded-divide-sqrt", "-Wno-unused-function", "-I" + os.path.join(ROOT, "include"),
             "-I" + os.path.join(PKG, "csrc")]
    obj = out[:-4] + ".o"
    subprocess.run(["/opt/rocm/bin/hipcc"] + flags + ["-c", out, "-o", obj], check=True)
    bid = os.path.join(PKG, "build", f"bid_{name}.cpp")
    open(bid, "w").write('extern "C" const char* fks_build_id(void) { return "variant-%s"; }\n' % name)
    subprocess.run(["/opt/rocm/bin/hipcc", "-fPIC", "-c", bid, "-o", bid[:-4] + ".o"], check=True)
    b = os.path.join(PKG, "build")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-o", os.path.join(b, f"libfks_{name}.so"),
                    obj, os.path.join(b, "fks_capi.o"), os.path.join(b, "fks_gf2.o"), os.path.join(b, "fks_tables.o"),
                    bid[:-4] + ".o"], check=True)
    print(f"built fate-llm_amd/build/libfks_{name}.so")


if __name__ == "__main__":
    main()
