"""Per-dispatch counters of the small-K apply kernel (fks_apply_kernel<DT, MODE, false,
true>: the ZO step's K <= 4 passes) from tools/gpu_pmc_smallk.sh, per mode, into
profiles/pmc_smallk_<tag>.json:  python tools/summarize_pmc_smallk.py <tag> <variant>"""
import collections
import csv
import glob
import json
import re
import sys

PARAMS = 6_738_415_616
MODES = {"1": "perturb", "5": "perturb_update", "0": "update", "3": "update_wd", "4": "update_nowd",
         "1_store": "perturb_storing_z_indices", "replay_1": "perturb_replay", "replay_5": "perturb_update_replay",
         "replay_3": "update_wd_replay", "replay_4": "update_nowd_replay", "replay_0": "update_replay"}


def main(tag, variant):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(f"gpurun_out/pmcsk_{variant}_*/**/*counter_collection.csv", recursive=True)):
        vals = collections.defaultdict(lambda: collections.defaultdict(float))
        dur = collections.defaultdict(dict)
        for r in csv.DictReader(open(f)):
            m = re.search(r"(fks_apply_kernel<1, (\d+), false, true>|fks_small2_kernel<1, (\d+)(?:, (\d))?>|"
                          r"fks_zreplay_kernel<(\d+)>)", r["Kernel_Name"])
            if not m:
                continue
            if m.group(5):
                mode = "replay_" + m.group(5)
            elif m.group(3):
                mode = m.group(3) + ("_store" if m.group(4) == "1" else "")
            else:
                mode = m.group(2)
            vals[mode][(r["Counter_Name"], r["Dispatch_Id"])] += float(r["Counter_Value"])
            dur[mode][r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        for mode, d in vals.items():
            by = collections.defaultdict(list)
            for (name, _), v in d.items():
                by[name].append(v)
            for name, v in by.items():
                per[mode][name].append(sum(v) / len(v))
            per[mode]["duration_ns"].append(sum(dur[mode].values()) / len(dur[mode]))
    out = {"source": f"rocprofv3 --pmc, tools/perf_smallk.py on the LLaMA-7B bf16 layout ({PARAMS} params), "
                     f"variant {variant}", "modes": {}}
    for mode, d in per.items():
        c = {k: sum(v) / len(v) for k, v in d.items()}
        cyc = c["GRBM_GUI_ACTIVE"] / 8
        rec = {"per_launch": c, "duration_ms_profiled": c["duration_ns"] / 1e6, "clock_ghz": cyc / c["duration_ns"],
               "valu_instr_per_param": c["SQ_INSTS_VALU"] * 64 / PARAMS,
               "valu_active_frac": c["SQ_ACTIVE_INST_VALU"] * 4 / 1024 / cyc,
               "wait_any_frac": c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"],
               "lds_bank_conflict_frac": c["SQ_LDS_BANK_CONFLICT"] / max(c["SQ_LDS_IDX_ACTIVE"], 1)}
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            hbm = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
            rec["hbm_bytes_per_launch_corrected"] = hbm
            rec["hbm_bytes_per_param"] = hbm / PARAMS
            rec["hbm_GBps_profiled"] = hbm / c["duration_ns"]
        out["modes"][MODES.get(mode, mode)] = rec
    print(json.dumps(out, indent=1))
    with open(f"profiles/pmc_smallk_{tag}.json", "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
