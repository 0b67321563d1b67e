"""Summarise rocprofv3 PMC CSVs (gpurun_out/prof/pmc_*) for one kernel: mean
counter value per dispatch, plus derived rates.  Usage:
  python scripts/pmc_summary.py gpurun_out/prof [kernel-substring] > summary.json"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(prof_dir, pat):
    per = defaultdict(list)
    meta = {}
    for f in sorted(glob.glob(os.path.join(prof_dir, "pmc_*", "*counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            if pat not in r["Kernel_Name"]:
                continue
            per[r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta = {k: r[k] for k in ("Kernel_Name", "Grid_Size", "Workgroup_Size",
                                      "LDS_Block_Size", "VGPR_Count", "SGPR_Count",
                                      "Scratch_Size")}
    return {k: sum(v) / len(v) for k, v in per.items()}, {k: len(v) for k, v in per.items()}, meta


def main():
    prof = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else "heap_predict_kernel"
    c, n, meta = load(prof, pat)
    d = {"kernel": meta, "dispatches": n, "counters": c}
    der = {}
    if "FETCH_SIZE" in c:
        # gfx950: FETCH_SIZE (KB) reads half the bytes of a wide streaming read
        # (MI355X_MICROARCH.md, HBM); report raw and x2-corrected
        der["fetch_bytes_raw"] = c["FETCH_SIZE"] * 1024
        der["fetch_bytes_corrected_x2"] = c["FETCH_SIZE"] * 1024 * 2
    if "WRITE_SIZE" in c:
        der["write_bytes"] = c["WRITE_SIZE"] * 1024
    if "SQ_LDS_BANK_CONFLICT" in c and "SQ_LDS_IDX_ACTIVE" in c and c["SQ_LDS_IDX_ACTIVE"]:
        der["lds_bank_conflict_rate"] = c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"]
    if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
        tot = c["TCC_HIT_sum"] + c["TCC_MISS_sum"]
        der["l2_hit_rate"] = c["TCC_HIT_sum"] / tot if tot else None
    if "SQ_INSTS_VALU" in c and "SQ_WAVES" in c:
        der["valu_insts_per_wave"] = c["SQ_INSTS_VALU"] / c["SQ_WAVES"]
        der["lds_insts_per_wave"] = c.get("SQ_INSTS_LDS", 0) / c["SQ_WAVES"]
        der["salu_insts_per_wave"] = c.get("SQ_INSTS_SALU", 0) / c["SQ_WAVES"]
    if "SQ_WAVE_CYCLES" in c:
        wc = c["SQ_WAVE_CYCLES"]
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
            if k in c and wc:
                der[k.lower() + "_frac_of_wave_cycles"] = c[k] / wc
    if "GRBM_GUI_ACTIVE" in c:
        der["gui_active_cycles_per_xcd"] = c["GRBM_GUI_ACTIVE"] / 8
    d["derived"] = der
    print(json.dumps(d, indent=1))


if __name__ == "__main__":
    main()
