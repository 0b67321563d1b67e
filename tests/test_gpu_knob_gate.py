"""libtreeinfer's layout / kernel A/B switches are
developer knobs, read only under TI_DEV_KNOBS=1, so a serving worker that
inherits a stray variable still runs the default kernels (the reference
plugin's one knob is nthread, python/xgbserver/xgbserver/model.py:38).
Without the gate, setting them leaves ti_forest_info unchanged; with it, they
take effect (so the test would notice a gate that blocks everything)."""
import pytest

from kfserving_amd.engine import DeviceForest
from kfserving_amd.formats.xgboost_format import forest_from_raw_trees, synthetic_complete_trees

pytestmark = pytest.mark.gpu

KNOBS = {"TI_FORCE_LAYOUT": "heap", "TI_BHEAP_FIX": "0", "TI_TX_TOP": "3", "TI_LX_ILP": "4",
         "TI_RX_B8": "0", "TI_COVER_ORDER": "0", "TI_HOST_REGISTER": "1"}


def _info(f):
    d = DeviceForest(f, [0])
    try:
        return d.info()
    finally:
        d.close()


def test_ab_knobs_need_the_dev_gate(monkeypatch):
    trees, ti = synthetic_complete_trees(40, 8, 28, seed=3)
    f = forest_from_raw_trees(trees, ti, 28, 0, 0.0, "binary:logistic")
    monkeypatch.delenv("TI_DEV_KNOBS", raising=False)
    for k in KNOBS:
        monkeypatch.delenv(k, raising=False)
    default = _info(f)
    for k, v in KNOBS.items():
        monkeypatch.setenv(k, v)
    assert _info(f) == default                  # no gate: the same kernels and image
    monkeypatch.setenv("TI_DEV_KNOBS", "0")
    assert _info(f) == default
    monkeypatch.setenv("TI_DEV_KNOBS", "1")
    forced = _info(f)
    assert forced["layout"] == 0 and default["layout"] == 3   # float-compare heap, forced
