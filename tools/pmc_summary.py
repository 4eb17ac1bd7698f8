"""Per-kernel summary of rocprofv3 --pmc passes (tools/gpu_round.sh bmmpmc / t16pmc).

    python tools/pmc_summary.py gpurun_out/bmmpmcA gpurun_out/bmmpmcB > summary.json

Every counter is averaged per dispatch over the kernel (grid size kept in the key: one kernel
template runs several shapes). Derived ratios, where the counters are present:
  lds_conflict_per_lds_active = SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS
  mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (SQ_BUSY_CYCLES x 4 SIMDs)    (per-SE busy scaled; rough)
  wait_frac = SQ_WAIT_ANY / SQ_WAVE_CYCLES
"""
import collections
import csv
import glob
import json
import os
import sys


def load(d):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in glob.glob(os.path.join(d, "*counter_collection.csv")):
        for r in csv.DictReader(open(path)):
            name = r["Kernel_Name"].split("(")[0]
            name = name.replace("void ", "").replace("lfk::", "")
            key = f"{name} grid={r['Grid_Size']}"
            per[key][(r["Dispatch_Id"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    out = {}
    for key, vals in per.items():
        by_counter = collections.defaultdict(list)
        for (disp, ctr), v in vals.items():
            by_counter[ctr].append(sum(v))  # a dispatch's value summed over its dimensions
        out[key] = {c: sum(v) / len(v) for c, v in by_counter.items()}
        out[key]["dispatches"] = max(len(v) for v in by_counter.values())
    return out


def main(dirs):
    merged = collections.defaultdict(dict)
    for d in dirs:
        for k, v in load(d).items():
            disp = v.pop("dispatches")
            merged[k].update(v)
            merged[k][f"dispatches_{os.path.basename(d.rstrip('/'))}"] = disp
    for k, v in merged.items():
        if v.get("SQ_ACTIVE_INST_LDS"):
            v["lds_conflict_per_lds_active"] = round(v.get("SQ_LDS_BANK_CONFLICT", 0.0) / v["SQ_ACTIVE_INST_LDS"], 3)
        if v.get("SQ_BUSY_CYCLES") and "SQ_VALU_MFMA_BUSY_CYCLES" in v:
            v["mfma_busy"] = round(v["SQ_VALU_MFMA_BUSY_CYCLES"] / (4 * v["SQ_BUSY_CYCLES"]), 3)
        if v.get("SQ_WAVE_CYCLES") and "SQ_WAIT_ANY" in v:
            v["wait_frac"] = round(v["SQ_WAIT_ANY"] / v["SQ_WAVE_CYCLES"], 3)
    top = sorted(merged.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0.0) * max(
        [n for c, n in kv[1].items() if c.startswith("dispatches_")] or [1]))
    json.dump({"dirs": dirs, "kernels": {k: {c: round(x, 3) if isinstance(x, float) else x for c, x in v.items()}
                                         for k, v in top[:25]}}, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1:])
