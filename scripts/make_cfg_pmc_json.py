"""Condense the PMC passes of scripts/r2_cfgprof.sh (one config, one kernel,
1M-row launches) into the per-launch figures bench.py's c3 / c4 roofline keys
scale by rows: VALU wave-instructions, LDS-array cycles, TD busy cycles (the
vector memory data path a node gather occupies), and HBM bytes.

Usage: python scripts/make_cfg_pmc_json.py PROF_DIR KERNEL_SUBSTR WORKLOAD LAYOUT ROWS OUT.json
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import load  # noqa: E402


def main():
    prof, pat, workload, layout, rows, out = sys.argv[1:7]
    c, n, meta = load(prof, pat)
    res = {"workload": workload, "layout": layout, "rows": int(rows),
           "kernel": meta.get("Kernel_Name"), "vgprs": meta.get("VGPR_Count"),
           "lds_block_bytes": meta.get("LDS_Block_Size"),
           "valu_insts_per_launch": c["SQ_INSTS_VALU"],
           "lds_insts_per_launch": c.get("SQ_INSTS_LDS"),
           "vmem_insts_per_launch": c.get("SQ_INSTS_VMEM_RD"),
           "lds_idx_active_per_launch": c.get("SQ_LDS_IDX_ACTIVE"),
           "lds_bank_conflict_frac": (c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"]
                                      if c.get("SQ_LDS_IDX_ACTIVE") else None),
           "td_busy_per_launch": c.get("TD_TD_BUSY_sum"),
           "tcp_accesses_per_launch": c.get("TCP_TOTAL_CACHE_ACCESSES_sum"),
           "waves_per_launch": c.get("SQ_WAVES"),
           "wait_frac": c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"] if c.get("SQ_WAVE_CYCLES") else None,
           "gui_active_cycles_per_xcd": c["GRBM_GUI_ACTIVE"] / 8 if "GRBM_GUI_ACTIVE" in c else None,
           "source": prof}
    if "TCC_HIT_sum" in c:
        res["l2_hit_rate"] = c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        # FETCH_SIZE x2 on gfx950 (profiles/r2_fetch_calib.csv)
        res["hbm_bytes_per_launch"] = c["FETCH_SIZE"] * 2048 + c["WRITE_SIZE"] * 1024
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
