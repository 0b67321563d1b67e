"""bench.py's roofline keys from the committed PMC passes (the
headline roofline went to null when the pass's free-text walk label changed).
The identity that ties a pass to a launch is the workload, rows, layout, the
launched kernel's name and the integer walk id (ti_forest_info.walk)."""
import os

import pytest

import bench

PMC_C2 = bench.pmc_path("c2")
# ti_forest_info of the C2 forest on the current build: binned heap (3), the
# fixed-layout walk with the scalar-loaded root (2)
C2_INFO = {"layout": 3, "walk": 2, "bottom": 0}


def test_c2_roofline_from_committed_pmc_pass():
    rf = bench.roofline(0.7226, 1_000_000, C2_INFO, PMC_C2)
    assert "error" not in rf, rf.get("error")
    assert rf["bound"] == "lds_array"
    pmc = bench.load_pmc(PMC_C2)        # LDS-array cycles / (256 CUs x the pass's cycles)
    want = pmc["lds_idx_active_per_launch"] / (256 * pmc["lds_pass_cycles_per_xcd"])
    assert rf["frac"] == pytest.approx(want, rel=1e-12) and 0.5 < rf["frac"] < 0.9
    assert rf["achieved"] == pytest.approx(rf["frac"] * 2.4, rel=1e-9)
    assert rf["traffic"] and rf["traffic"] > rf["hbm_compulsory_bytes"]
    assert 0 < rf["lds_bank_conflict_frac"] < 0.5
    assert rf["valu"]["frac"] > 0 and rf["hbm_compulsory_frac"] > 0
    assert "bheap_fix_kernel" in rf["pmc_kernel"] and rf["kernel"] == "bheap_fix_kernel"


@pytest.mark.parametrize("info,why", [
    ({"layout": 3, "walk": 1, "bottom": 0}, "walk id"),
    ({"layout": 3, "walk": 0, "bottom": 0}, "kernel"),
    ({"layout": 0, "walk": 0, "bottom": 0}, "layout"),
])
def test_c2_roofline_mismatch_says_why(info, why):
    rf = bench.roofline(0.7226, 1_000_000, info, PMC_C2)
    assert rf["frac"] is None and why in rf["error"]
    assert rf["hbm_compulsory_frac"] > 0


@pytest.mark.parametrize("key,info,bound", [
    ("c3", {"layout": 9, "bottom": 3}, "td_busy"),
    ("c3_f64", {"layout": 9, "bottom": 3}, "td_busy"),
    ("c3_maxbin", {"layout": 9, "bottom": 1}, "lds_array"),
    ("c4", {"layout": 8}, "td_busy"),
])
def test_config_rooflines_from_committed_pmc_passes(key, info, bound):
    path = bench.pmc_path(key)
    rf = bench.config_roofline(5.0, 1_000_000, info, key, path)
    assert "error" not in rf, rf.get("error")
    assert rf["bound"] == bound and 0 < rf["frac"] <= 1.0
    assert rf["lds_bank_conflict_frac"] is not None and rf["traffic"]


def test_config_roofline_wrong_kernel():
    path = bench.pmc_path("c3_maxbin")
    rf = bench.config_roofline(5.0, 1_000_000, {"layout": 9, "bottom": 0}, "c3_maxbin", path)
    assert rf["frac"] is None and "t8explicit_predict_kernel" in rf["error"]
