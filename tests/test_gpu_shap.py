"""TreeSHAP contributions on the GPU (TI_OUTPUT_CONTRIB) against the float64
restatement oracle/shap_ref.py (itself pinned by brute-force Shapley values,
tests/test_shap_oracle.py), plus the efficiency property sum(phi) + bias ==
margin at sizes the oracle cannot reach.

Tolerances: float64-accumulating forests (LightGBM, sklearn) 1e-9 relative to
the row's largest contribution; float32 forests (XGBoost) accumulate in
float64 on the device and round once to float32, so 1e-6 of the row scale
(xgboost's own pred_contribs accumulates in float32 and sits further away)."""
import os
import tempfile

import numpy as np
import pytest

from kfserving_amd.engine import (OPT_SHAP_TABLE_MB, OPT_SHAP_TABLE_ROWS, DeviceForest,
                                  TreeInferError)
from kfserving_amd.forest import OUT_CONTRIB, OUT_MARGIN, TI_F32
from kfserving_amd.formats import load_lightgbm_model, load_xgboost_model
from kfserving_amd.formats import lightgbm_format as lf
from kfserving_amd.formats import xgboost_format as xf
from kfserving_amd.formats.sklearn_format import forest_from_sklearn
from oracle import shap_ref

pytestmark = pytest.mark.gpu


def _xgb(n_trees, depth, F, seed, K=0):
    trees, ti = xf.synthetic_complete_trees(n_trees, depth, F, seed=seed, num_class=K)
    obj = "multi:softprob" if K else "binary:logistic"
    return xf.forest_from_raw_trees(trees, ti, F, K, 0.5, obj)


def _lgb(n_trees, leaves, F, seed, K=1):
    trees = lf.synthetic_leafwise_trees(n_trees, leaves, F, seed=seed)
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "m.txt")
        obj = f"multiclass num_class:{K}" if K > 1 else "binary sigmoid:1"
        lf.write_lightgbm_text(p, trees, F, obj, num_class=K)
        return load_lightgbm_model(p)


def _sk(kind):
    from sklearn.ensemble import (GradientBoostingRegressor, RandomForestClassifier,
                                  RandomForestRegressor)
    rng = np.random.default_rng(3)
    X = rng.standard_normal((400, 6)).astype(np.float32)
    y = (X[:, 0] > 0).astype(int) + (X[:, 1] > 0.5).astype(int)
    if kind == "rf-clf":
        est = RandomForestClassifier(n_estimators=8, max_depth=6, random_state=0).fit(X, y)
    elif kind == "rf-reg":
        est = RandomForestRegressor(n_estimators=8, max_depth=7, random_state=0).fit(
            X, X[:, 0] * 2 + X[:, 2])
    else:
        est = GradientBoostingRegressor(n_estimators=20, max_depth=4, random_state=0).fit(
            X, X[:, 0] * 2 - X[:, 3])
    return forest_from_sklearn(est)


def _rows(f, n, seed, nan=True):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, f.n_features))
    if nan:
        X[rng.random(X.shape) < 0.08] = np.nan
    X[rng.random(X.shape) < 0.08] = 0.0
    return X.astype(np.float32) if f.input_dtype == TI_F32 else X


def _check(f, X, got):
    want = shap_ref.contributions(f, np.asarray(X, dtype=np.float64))
    assert got.shape == want.shape
    rel = 1e-6 if f.accum_dtype == TI_F32 else 1e-9
    scale = np.maximum(np.abs(want).max(axis=1, keepdims=True), 1.0)
    err = np.abs(got.astype(np.float64) - want) / scale
    assert err.max() <= rel, f"max scaled error {err.max():.3g}"


@pytest.mark.parametrize("make,nan", [
    (lambda: _xgb(24, 6, 10, seed=1), True),
    (lambda: _xgb(12, 4, 8, seed=2, K=3), True),
    (lambda: _lgb(12, 31, 10, seed=3), True),
    (lambda: _lgb(9, 15, 8, seed=4, K=3), True),
    (lambda: _sk("rf-clf"), True),
    (lambda: _sk("rf-reg"), True),
    (lambda: _sk("gb-reg"), False),
], ids=["xgb", "xgb-multiclass", "lgb-zero-missing", "lgb-multiclass", "sk-rf-clf",
        "sk-rf-reg", "sk-gb-reg"])
@pytest.mark.parametrize("kernel", ["table", "arith"])
def test_contributions_match_oracle(make, nan, kernel):
    """Both TreeSHAP kernels against the oracle: the coefficient table (small
    batches) and the extend / unwind arithmetic (batches over
    TI_OPT_SHAP_TABLE_ROWS), forced per forest."""
    f = make()
    X = _rows(f, 130, seed=11, nan=nan)        # 130 rows: two full 64-row blocks + a ragged one
    dev = DeviceForest(f, [0])
    dev.set_option(OPT_SHAP_TABLE_ROWS, 1 << 30 if kernel == "table" else 0)
    got = dev.predict(X, OUT_CONTRIB)
    _check(f, X, got)
    info = dev.info()
    if kernel == "arith":
        assert info["shap_table"] == 0          # never needed, never built
    elif f.accum_dtype == TI_F32:               # xgboost: paths of <= 8 features
        assert info["shap_table"] == 1 and info["shap_table_bytes"] > 0


def test_table_and_arithmetic_bit_identical_c2_shape():
    """The C2-shape forest (500 x depth 8, 28 features) at 4,096 rows: the
    table kernel's contributions are the arithmetic kernel's, bit for bit (the
    table holds the same float32 expressions in the same order)."""
    f = _xgb(500, 8, 28, seed=21)
    X = _rows(f, 4096, seed=22)
    dev = DeviceForest(f, [0])
    tab = dev.predict(X, OUT_CONTRIB)
    info = dev.info()
    assert info["shap_table"] == 1, info
    assert info["shap_table_build_ms"] > 0
    print(f"C2-shape table: {info['shap_table_bytes'] / 2**20:.0f} MiB built in "
          f"{info['shap_table_build_ms']:.0f} ms")
    dev.set_option(OPT_SHAP_TABLE_ROWS, 0)
    arith = dev.predict(X, OUT_CONTRIB)
    assert np.array_equal(tab, arith)
    # (the numpy oracle is minutes at this forest size: tests above pin both
    # kernels against it on smaller forests)


@pytest.mark.parametrize("how", ["fault", "cap0", "cap_small"])
def test_table_failure_falls_back_to_arithmetic(how, monkeypatch):
    """The table is optional: an allocation/launch failure (injected) or a size
    cap it exceeds leaves the extend / unwind kernel serving the batch, with
    the same contributions, and no error for the caller."""
    f = _xgb(40, 6, 12, seed=23)
    X = _rows(f, 300, seed=24)
    ref = DeviceForest(f, [0])
    ref.set_option(OPT_SHAP_TABLE_ROWS, 0)
    want = ref.predict(X, OUT_CONTRIB)
    dev = DeviceForest(f, [0])
    if how == "fault":
        monkeypatch.setenv("TI_SHAP_TABLE_FAULT", "1")
    else:
        dev.set_option(OPT_SHAP_TABLE_MB, 0 if how == "cap0" else 1)
    got = dev.predict(X, OUT_CONTRIB)
    assert dev.info()["shap_table"] == -1
    assert np.array_equal(got, want)
    monkeypatch.delenv("TI_SHAP_TABLE_FAULT", raising=False)
    assert np.array_equal(dev.predict(X, OUT_CONTRIB), want)    # still served, no retry


def test_set_option_rejects_bad_values():
    dev = DeviceForest(_xgb(4, 3, 5, seed=9), [0])
    with pytest.raises(TreeInferError, match="unknown option"):
        dev.set_option(99, 1)
    with pytest.raises(TreeInferError, match=">= 0"):
        dev.set_option(OPT_SHAP_TABLE_ROWS, -1)


def test_deep_lightgbm_paths():
    """255-leaf leaf-wise trees: paths of 20+ unique features (LDS per lane grows
    with the longest path)."""
    f = _lgb(4, 255, 40, seed=8)
    X = _rows(f, 70, seed=12)
    _check(f, X, DeviceForest(f, [0]).predict(X, OUT_CONTRIB))


def test_chunked_forest_20_classes():
    """K > 16: parts write their [rows, kc * (F + 1)] blocks into place."""
    f = _xgb(40, 3, 6, seed=5, K=20)
    X = _rows(f, 65, seed=13)
    got = DeviceForest(f, [0]).predict(X, OUT_CONTRIB)
    assert got.shape == (65, 20 * 7)
    _check(f, X, got)


def test_reference_iris_fixtures(golden):
    for name in ("xgb_iris_legacy_082.bst", "xgb_iris_binf_1x.bst"):
        f = load_xgboost_model(os.path.join(golden, name))
        X = np.random.default_rng(1).uniform(0, 8, (100, f.n_features)).astype(np.float32)
        _check(f, X, DeviceForest(f, [0]).predict(X, OUT_CONTRIB))
    f = load_lightgbm_model(os.path.join(golden, "lgb_iris_v3.txt"))
    X = np.random.default_rng(2).uniform(0, 8, (100, f.n_features))
    _check(f, X, DeviceForest(f, [0]).predict(X, OUT_CONTRIB))


@pytest.mark.parametrize("make", [lambda: _xgb(200, 8, 28, seed=6),
                                  lambda: _lgb(100, 63, 50, seed=7, K=3)],
                         ids=["xgb-c2-shape", "lgb-multiclass"])
def test_efficiency_at_scale(make):
    """sum over features + bias == margin, per row and group, on 50k rows."""
    f = make()
    X = _rows(f, 50_000, seed=14)
    dev = DeviceForest(f, [0])
    c = dev.predict(X, OUT_CONTRIB).astype(np.float64).reshape(len(X), f.n_groups, -1)
    m = dev.predict(X, OUT_MARGIN).astype(np.float64).reshape(len(X), f.n_groups)
    tol = 2e-4 if f.accum_dtype == TI_F32 else 1e-9
    np.testing.assert_allclose(c.sum(axis=2), m, rtol=tol, atol=tol)


def test_forest_without_covers_is_unsupported():
    f = _xgb(4, 3, 5, seed=9)
    f.cover = None
    with pytest.raises(TreeInferError, match="covers"):
        DeviceForest(f, [0]).predict(np.zeros((3, 5), np.float32), OUT_CONTRIB)


def test_plugin_explain(golden):
    from kfserving_amd.xgbserver import XGBoostModel
    f = load_xgboost_model(os.path.join(golden, "xgb_iris_legacy_082.bst"))
    model = XGBoostModel("m", "", 1, booster=f)
    rows = [[6.8, 2.8, 4.8, 1.4], [6.0, 3.4, 4.5, 1.6]]
    out = model.explain({"instances": rows})["explanations"]
    want = shap_ref.contributions(
        f, np.asarray(rows, np.float32)).reshape(2, f.n_groups, f.n_features + 1)
    got = np.asarray(out)
    assert got.shape == (want.shape if f.n_groups > 1 else (2, f.n_features + 1))
    np.testing.assert_allclose(got.reshape(want.shape), want, rtol=1e-5, atol=1e-6)
