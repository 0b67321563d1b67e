"""Condense the rocprofv3 PMC passes of scripts/pmc_passes.sh into the
per-launch figures bench.py's roofline reads (profiles/pmc_c2.json).

Usage: python scripts/make_pmc_json.py PROF_DIR KERNEL_SUBSTR WORKLOAD ROWS LAYOUT \
           MODEL_BYTES OUT.json [SOURCE_NAME]

FETCH_SIZE is doubled: on gfx950 it reports half the bytes of a streaming
read, for 16-byte AND 4-byte lanes alike (calibrated on this box:
profiles/r2_fetch_calib.csv, scripts/micro/fetch_calib.hip; MI355X_MICROARCH.md
HBM section for the 16-byte case).
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import load  # noqa: E402


def main():
    prof, pat, workload, rows, layout, model_bytes, out = sys.argv[1:8]
    source = sys.argv[8] if len(sys.argv) > 8 else prof
    c, n, meta = load(prof, pat)
    res = {"workload": workload, "layout": layout, "rows": int(rows),
           "kernel": meta.get("Kernel_Name"), "dispatches": n.get("SQ_INSTS_VALU"),
           "valu_insts_per_launch": c["SQ_INSTS_VALU"],
           "waves_per_launch": c.get("SQ_WAVES"),
           "valu_insts_per_wave": c["SQ_INSTS_VALU"] / c["SQ_WAVES"],
           "lds_insts_per_launch": c.get("SQ_INSTS_LDS"),
           "vmem_insts_per_launch": c.get("SQ_INSTS_VMEM_RD"),
           "model_bytes": int(model_bytes), "source": source}
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        res["fetch_bytes_raw"] = c["FETCH_SIZE"] * 1024
        res["fetch_bytes_x2"] = c["FETCH_SIZE"] * 2048
        res["write_bytes"] = c["WRITE_SIZE"] * 1024
        res["hbm_bytes_per_launch"] = res["fetch_bytes_x2"] + res["write_bytes"]
    if "GRBM_GUI_ACTIVE" in c:
        res["gui_active_cycles_per_xcd"] = c["GRBM_GUI_ACTIVE"] / 8
    for k in ("SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "TCC_HIT_sum", "TCC_MISS_sum",
              "TA_BUSY_avr", "SQ_WAIT_ANY", "SQ_WAVE_CYCLES"):
        if k in c:
            res[k] = c[k]
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
