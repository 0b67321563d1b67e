"""Condense the rocprofv3 passes of scripts/kernel_pmc.sh (one workload, one
kernel) into the per-launch figures bench.py prices its rooflines with
(profiles/r3_<workload>_pmc.json):

  * counters: mean per dispatch of the kernel (name substring), FETCH_SIZE x 2
    (gfx950 counts half the bytes of a streaming read: MI355X_MICROARCH.md
    HBM; profiles/r2_fetch_calib.csv) + WRITE_SIZE as HBM bytes;
  * the profiled run's own cycles: each pass that carries GRBM_GUI_ACTIVE
    gives GUI_ACTIVE / 8 cycles per XCD per launch beside its kernel
    durations (its --kernel-trace), so every resource is priced on the
    cycles of the pass that counted it, never on another run's time, and the
    clock it ran at is those cycles / that duration (MI355X_MICROARCH.md
    "DVFS give-back").

Usage: python scripts/make_pmc_json.py PROF_DIR KERNEL_SUBSTR WORKLOAD LAYOUT ROWS OUT.json
           [--walk-step NAME] [--walk-id N] [--model-bytes N] [--source TEXT]

--walk-id is ti_forest_info.walk of the profiled binned-heap launch: bench.py
matches it (and the kernel name) against the launch it prices.
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def load_pass(d, pat):
    """(mean counter value per dispatch, mean kernel ns) of one pass dir."""
    per = defaultdict(list)
    meta = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if pat not in r["Kernel_Name"]:
                continue
            per[r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta = {k: r.get(k) for k in ("Kernel_Name", "LDS_Block_Size", "VGPR_Count",
                                          "SGPR_Count", "Grid_Size", "Workgroup_Size")}
    durs = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if pat in r["Kernel_Name"]:
                durs.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    # the first dispatch is the warm-up of kernel_workload.py: drop it when
    # there are more
    if len(durs) > 1:
        durs = durs[1:]
    c = {k: sum(v[1:] if len(v) > 1 else v) / max(1, len(v) - (1 if len(v) > 1 else 0))
         for k, v in per.items()}
    return c, (sum(durs) / len(durs) if durs else None), meta


def main():
    p = argparse.ArgumentParser()
    p.add_argument("prof")
    p.add_argument("kernel")
    p.add_argument("workload")
    p.add_argument("layout")
    p.add_argument("rows", type=int)
    p.add_argument("out")
    p.add_argument("--walk-step", default=None)
    p.add_argument("--walk-id", type=int, default=None)
    p.add_argument("--model-bytes", type=int, default=0)
    p.add_argument("--source", default=None)
    a = p.parse_args()
    passes = {}
    for d in sorted(glob.glob(os.path.join(a.prof, "pmc_*"))):
        passes[os.path.basename(d)] = load_pass(d, a.kernel)
    c = {}
    meta = {}
    for name, (cc, _, m) in passes.items():
        c.update({k: v for k, v in cc.items() if k != "GRBM_GUI_ACTIVE"})
        meta = meta or m

    def cycles(name):
        cc, ns, _ = passes.get(name, ({}, None, {}))
        g = cc.get("GRBM_GUI_ACTIVE")
        return (g / 8 if g else None), ns

    res = {"workload": a.workload, "layout": a.layout, "rows": a.rows,
           "kernel": meta.get("Kernel_Name"), "vgprs": meta.get("VGPR_Count"),
           "sgprs": meta.get("SGPR_Count"), "walk_step": a.walk_step, "walk_id": a.walk_id,
           "model_bytes": a.model_bytes,
           "valu_insts_per_launch": c.get("SQ_INSTS_VALU"),
           "waves_per_launch": c.get("SQ_WAVES"),
           "valu_insts_per_wave": (c["SQ_INSTS_VALU"] / c["SQ_WAVES"]
                                   if c.get("SQ_WAVES") else None),
           "lds_insts_per_launch": c.get("SQ_INSTS_LDS"),
           "salu_insts_per_launch": c.get("SQ_INSTS_SALU"),
           "vmem_insts_per_launch": c.get("SQ_INSTS_VMEM_RD"),
           "lds_idx_active_per_launch": c.get("SQ_LDS_IDX_ACTIVE"),
           "lds_bank_conflict_frac": (c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"]
                                      if c.get("SQ_LDS_IDX_ACTIVE") else None),
           "td_busy_per_launch": c.get("TD_TD_BUSY_sum"),
           "ta_busy_avr_per_launch": c.get("TA_BUSY_avr"),
           "tcp_accesses_per_launch": c.get("TCP_TOTAL_CACHE_ACCESSES_sum"),
           "wait_frac": c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"] if c.get("SQ_WAVE_CYCLES") else None,
           "active_inst_frac": (c["SQ_ACTIVE_INST_ANY"] / c["SQ_WAVE_CYCLES"]
                                if c.get("SQ_WAVE_CYCLES") else None),
           "source": a.source or a.prof}
    for name, key in (("pmc_a", "valu"), ("pmc_b", "lds"), ("pmc_t", "td")):
        cyc, ns = cycles(name)
        res[f"{key}_pass_cycles_per_xcd"] = cyc
        res[f"{key}_pass_kernel_ns"] = ns
    cyc, ns = cycles("pmc_a")
    res["gui_active_cycles_per_xcd"] = cyc
    res["profiled_kernel_ns"] = ns
    res["profiled_clock_GHz"] = cyc / ns if cyc and ns else None
    if "TCC_HIT_sum" in c:
        res["l2_hit_rate"] = c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
    if "FETCH_SIZE" in c:
        res["fetch_bytes_raw"] = c["FETCH_SIZE"] * 1024
        res["fetch_bytes_x2"] = c["FETCH_SIZE"] * 2048
    if "WRITE_SIZE" in c:
        res["write_bytes"] = c["WRITE_SIZE"] * 1024
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        res["hbm_bytes_per_launch"] = res["fetch_bytes_x2"] + res["write_bytes"]
    if c.get("SQ_WAVES") and c.get("SQ_WAVE_CYCLES") and cyc:
        # resident waves per SIMD on average: wave-cycles (quad-cycles x 4)
        # over 1,024 SIMDs x the kernel's cycles
        res["waves_per_simd"] = c["SQ_WAVE_CYCLES"] * 4 / (1024 * cyc)
    res["counters"] = c
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "counters"}))


if __name__ == "__main__":
    main()
