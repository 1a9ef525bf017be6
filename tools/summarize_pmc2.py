"""Summarise the rocprofv3 --pmc passes of tools/gpu_pmc2.sh for the full 32-seed slice
kernel launch (fks_apply_bs_kernel<MODE, true>) into profiles/pmc_apply_<tag>.json:
  python tools/summarize_pmc2.py <tag> <variant> <params> <seeds_per_launch> [kernel] [elt]
kernel: the launch to count, a substring of its name (default the full slice-kernel
launch; tools/gpu_pmc_f32.sh passes the full 19-seed fp32 kernel); elt: bytes per param.
Each pass is its own process (dispatch ids restart), so counters are averaged per
dispatch within a pass, then merged across passes."""
import collections
import csv
import glob
import json
import sys

KERNEL = "fks_apply_bs_kernel<"


def _match(name, kernel):
    if kernel:
        return kernel in name
    return KERNEL in name and "true>" in name


def per_pass(path, kernel=None):
    vals = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    dur = {}
    for r in csv.DictReader(open(path)):
        if _match(r["Kernel_Name"], kernel):
            vals[r["Counter_Name"]] += float(r["Counter_Value"])
            disp[r["Counter_Name"]].add(r["Dispatch_Id"])
            dur[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    out = {k: vals[k] / len(disp[k]) for k in vals}
    if dur:
        out["duration_ns"] = sum(dur.values()) / len(dur)
    return out, max((len(d) for d in disp.values()), default=0)


def main(tag, variant, params, seeds, kernel=None, elt=2):
    c = {}
    n_disp = {}
    for f in sorted(glob.glob(f"gpurun_out/pmc2_{variant}_*/**/*counter_collection.csv", recursive=True)):
        d, n = per_pass(f, kernel)
        for k, v in d.items():
            c.setdefault(k, []).append(v)
        n_disp[f] = n
    c = {k: sum(v) / len(v) for k, v in c.items()}  # GRBM_GUI_ACTIVE appears in several passes
    units = params * seeds
    clk_cycles = c["GRBM_GUI_ACTIVE"] / 8  # summed over the 8 XCDs
    try:
        build_id = open(f"gpurun_out/pmc2_{variant}_buildid").read().strip()
    except OSError:
        build_id = None
    out = {
        # fks_build_id() of the profiled libfks.so: bench.py uses these counters only for
        # a library with the same device code
        "build_id": build_id,
        "source": f"rocprofv3 --pmc passes (tools/perf_one.py, {params} params of {elt} B, "
                  f"{seeds}-seed launches), variant {variant}; dispatches per pass {sorted(set(n_disp.values()))}",
        "kernel": kernel or "fks_apply_bs_kernel<MODE,true>", "seeds_per_full_launch": seeds, "params": params,
        "per_launch": c,
        "valu_lane_ops_per_seed_param": c["SQ_INSTS_VALU"] * 64 / units,
        "valu_instr_per_wave_seed": c["SQ_INSTS_VALU"] / (units / 128),
        # gfx950 counts SQ_ACTIVE_INST_VALU as one quad-cycle per VALU instruction
        "valu_active_frac": c["SQ_ACTIVE_INST_VALU"] * 4 / 1024 / clk_cycles,
        "valu_dual_issue_frac": c.get("SQ_ACTIVE_INST_VALU2", 0.0) / c["SQ_INSTS_VALU"],
        "wait_any_frac": c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"],
        "wait_inst_any_frac": c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"],
        "lds_bank_conflict_frac": (c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"] if c.get("SQ_LDS_IDX_ACTIVE") else None),
        # LDS-array cycles (conflicts included) per CU-cycle, 256 CUs
        "lds_active_frac": (c["SQ_LDS_IDX_ACTIVE"] / 256 / clk_cycles if c.get("SQ_LDS_IDX_ACTIVE") else None),
        "clock_cycles_per_launch": clk_cycles,
        # effective clock (MI355X_MICROARCH.md: GRBM_GUI_ACTIVE / 8 / wall time); profiled
        # passes run slightly slower than unprofiled ones
        "clock_ghz": clk_cycles / c["duration_ns"],
    }
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        # gfx950: FETCH_SIZE reports 1/2 of a wide streaming read's bytes (MI355X_MICROARCH.md)
        hbm = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
        out["hbm_bytes_per_launch_corrected"] = hbm
        out["hbm_bytes_per_param_per_launch"] = hbm / params
        out["algorithmic_bytes_per_param_per_launch"] = 2.0 * elt
    print(json.dumps(out, indent=1))
    with open(f"profiles/pmc_apply_{tag}.json", "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]),
         sys.argv[5] if len(sys.argv) > 5 else None, int(sys.argv[6]) if len(sys.argv) > 6 else 2)
