"""Per-dispatch averages of the jump kernel's counters from tools/gpu_pmc2.sh passes
(gpurun_out/pmc2_<variant>_*), with the issue fractions the DESIGN notes quote.
python tools/r03/jump_pmc_show.py [variant]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pmc2_show import load  # noqa: E402


def main():
    v = sys.argv[1] if len(sys.argv) > 1 else "full"
    d = load(v, lambda n: "fks_jump_kernel" in n)
    for k in sorted(d):
        print(f"{k:26s} {d[k]:16.6g}")
    wc = d.get("SQ_WAVE_CYCLES")
    if wc:
        for k in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY",
                  "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_MISC"):
            if k in d:
                print(f"{k + ' / wave cycles':40s} {d[k] / wc:.4f}")
    if "SQ_INSTS_VALU" in d and "SQ_INSTS_SALU" in d:
        print(f"{'SALU / VALU instructions':40s} {d['SQ_INSTS_SALU'] / d['SQ_INSTS_VALU']:.4f}")


if __name__ == "__main__":
    main()
