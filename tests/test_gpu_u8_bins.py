"""Layout 9 with u8 bins (treeinfer_kernels.h RxBins<true>): forests whose
features have at most 254 distinct thresholds (126 with LightGBM's zero rule)
bin to one byte, four features a word, NaN as bin 0.  Every case is checked
bit for bit against the C restatement of lightgbm 2.3.1's predict loop
(oracle/c/tree_port.c) and against the u16 image of the same forest
(TI_RX_B8=0), on float32 and float64 inputs, with NaN, +-0, LightGBM's
|x| <= 1e-35 zero map, +-inf and values exactly at a threshold."""
import os
import tempfile

import numpy as np
import pytest

from kfserving_amd.engine import DeviceForest
from kfserving_amd.forest import MISSING_NAN, MISSING_NONE, MISSING_ZERO, OUT_LEAF, OUT_MARGIN
from kfserving_amd.formats import load_lightgbm_model
from kfserving_amd.formats import lightgbm_format as lf
from oracle import port

pytestmark = pytest.mark.gpu

TEXPLICIT = 9


def _forest(trees, F):
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "model.txt")
        lf.write_lightgbm_text(p, trees, F, "binary sigmoid:1")
        return load_lightgbm_model(p)


def _device(forest, monkeypatch, b8: bool):
    monkeypatch.setenv("TI_RX_B8", "1" if b8 else "0")
    dev = DeviceForest(forest, [0])
    monkeypatch.delenv("TI_RX_B8")
    return dev


def _inputs(trees, rows, F, seed, special_frac=0.03, at_frac=0.05):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((rows, F))
    thr = np.concatenate([np.asarray(t["threshold"], dtype=np.float64) for t in trees])
    pick = rng.random(X.shape)
    X = np.where(pick < at_frac, thr[rng.integers(0, len(thr), X.shape)], X)
    sp = np.array([np.nan, 0.0, -0.0, 1e-36, -1e-40, 1e-35, 2e-35, np.inf, -np.inf])
    m = rng.random(X.shape) < special_frac
    X[m] = sp[rng.integers(0, len(sp), m.sum())]
    return X


def _lone_leaf(value=0.25):
    z = np.zeros(0, dtype=np.int64)
    return {"split_feature": z, "threshold": np.zeros(0), "decision_type": z, "left_child": z,
            "right_child": z, "leaf_value": np.array([value]), "leaf_count": np.array([10]),
            "internal_count": z}


@pytest.mark.parametrize("top", [1, 3, 6, 9])
@pytest.mark.parametrize("tx8", [1, 0])
def test_u8_bottoms_every_top_depth(monkeypatch, top, tx8):
    """Layout 9's two u8 bottoms (TI_TX8=1: compact u32 nodes with their
    children side by side, leaves looping on themselves; 0: layout 7's
    records) at top depths that end above, inside and below the trees, with a
    one-split tree and a lone leaf among them, NaN / zero / 1e-36 rows in some
    tiles: margins and leaf ids bit-exact against the C port."""
    monkeypatch.setenv("TI_TX_TOP", str(top))
    monkeypatch.setenv("TI_TX8", str(tx8))
    mts = (MISSING_NONE, MISSING_ZERO, MISSING_NAN)
    trees = lf.synthetic_maxbin_trees(29, 255, 30, seed=top, max_bin=125, missing_types=mts)
    trees.insert(5, lf.synthetic_maxbin_trees(1, 2, 30, seed=99, max_bin=125)[0])
    trees.insert(11, _lone_leaf())
    f = _forest(trees, 30)
    dev = DeviceForest(f, [0])
    assert dev.info()["layout"] == TEXPLICIT and dev.info()["bin_bits"] == 8
    X = _inputs(trees, 3001, 30, seed=top + 7, special_frac=0.02)
    X[:1024][~np.isfinite(X[:1024])] = 0.5           # fast tiles first
    X[:1024][X[:1024] == 0] = 0.5
    for Xi in (X, X.astype(np.float32)):
        want = port.lgb_predict_raw(trees, 1, 30, Xi.astype(np.float64))[:, 0]
        assert np.array_equal(dev.predict(Xi, OUT_MARGIN), want)
    monkeypatch.setenv("TI_FORCE_LAYOUT", "rexplicit")
    ref = DeviceForest(f, [0])
    X32 = X.astype(np.float32)
    assert np.array_equal(dev.predict(X32, OUT_LEAF), ref.predict(X32, OUT_LEAF))


@pytest.mark.parametrize("missing", ["none", "all"])
def test_maxbin_u8_matches_port_and_u16(monkeypatch, missing):
    mts = (MISSING_NONE,) if missing == "none" else (MISSING_NONE, MISSING_ZERO, MISSING_NAN)
    # the zero rule doubles the bins (<= 126 thresholds) and adds {-denorm_min, 0}
    # to every zero-missing feature's thresholds: 124 edges + 2
    max_bin = 255 if missing == "none" else 125
    trees = lf.synthetic_maxbin_trees(60, 255, 40, seed=3, max_bin=max_bin, missing_types=mts)
    f = _forest(trees, 40)
    d8 = _device(f, monkeypatch, True)
    d16 = _device(f, monkeypatch, False)
    assert d8.info()["layout"] == TEXPLICIT and d8.info()["bin_bits"] == 8
    assert d16.info()["layout"] == TEXPLICIT and d16.info()["bin_bits"] == 16
    X = _inputs(trees, 5003, 40, seed=11)
    X[:1536][~np.isfinite(X[:1536])] = 0.25          # fast tiles first (512-row u8 tiles)
    X[:1536][X[:1536] == 0] = 0.25
    for Xi in (X, X.astype(np.float32)):
        want = port.lgb_predict_raw(trees, 1, 40, Xi.astype(np.float64))[:, 0]
        got = d8.predict(Xi, OUT_MARGIN)
        assert np.array_equal(got, want)
        assert np.array_equal(got, d16.predict(Xi, OUT_MARGIN))
        assert np.array_equal(d8.predict(Xi, OUT_LEAF), d16.predict(Xi, OUT_LEAF))


@pytest.mark.parametrize("rows", [1, 511, 513, 2048])
def test_u8_ragged_tiles(monkeypatch, rows):
    trees = lf.synthetic_maxbin_trees(30, 127, 24, seed=rows)
    f = _forest(trees, 24)
    d8 = _device(f, monkeypatch, True)
    assert d8.info()["bin_bits"] == 8
    X = _inputs(trees, rows, 24, seed=rows + 5)
    want = port.lgb_predict_raw(trees, 1, 24, X)[:, 0]
    assert np.array_equal(d8.predict(X, OUT_MARGIN), want)


@pytest.mark.parametrize("n_trees,bits", [(20, 8), (40, 16)])
def test_u8_limit(monkeypatch, n_trees, bits):
    """At the u8 limit: 20 trees on max_bin-256 edges put 254 distinct
    thresholds on a feature (bin 255 is reachable, NaN is 0), 40 trees put
    255, which does not fit u8, so the forest keeps u16 bins.  Same answers."""
    trees = lf.synthetic_maxbin_trees(n_trees, 255, 4, seed=1, max_bin=256)   # 255 bin edges
    f = _forest(trees, 4)
    counts = [len(np.unique(np.concatenate([np.asarray(t["threshold"])[np.asarray(
        t["split_feature"]) == j] for t in trees]))) for j in range(4)]
    assert max(counts) == (254 if bits == 8 else 255)
    dev = _device(f, monkeypatch, True)
    assert dev.info()["layout"] == TEXPLICIT and dev.info()["bin_bits"] == bits
    X = _inputs(trees, 3000, 4, seed=2)
    X[:, 0] = np.where(np.arange(3000) % 7 == 0, 9.0, X[:, 0])       # above every edge: top bin
    assert np.array_equal(dev.predict(X, OUT_MARGIN), port.lgb_predict_raw(trees, 1, 4, X)[:, 0])


def test_c3_maxbin_full_float64():
    """c3_maxbin at C3 shape (1000 trees x 255 leaves, 100 features): 200k
    float64 rows, the dtype lgbserver feeds (lgbserver/model.py:46-51), bit
    exact against the C restatement on layout 9 with u8 bins."""
    trees = lf.synthetic_maxbin_trees(1000, 255, 100, seed=1)
    dev = DeviceForest(_forest(trees, 100), [0])
    assert dev.info()["layout"] == TEXPLICIT and dev.info()["bin_bits"] == 8
    X = _inputs(trees, 200_000, 100, seed=5, special_frac=0.01)
    want = port.lgb_predict_raw(trees, 1, 100, X)[:, 0]
    assert np.array_equal(dev.predict(X, OUT_MARGIN), want)
    X32 = X[:50_000].astype(np.float32)
    assert np.array_equal(dev.predict(X32, OUT_MARGIN),
                          port.lgb_predict_raw(trees, 1, 100, X32.astype(np.float64))[:, 0])


def _lgb_to_xgb_raw(t):
    """A LightGBM tree dict as XGBoost RegTree arrays (internal nodes 0..n-1,
    then the leaves; default_left from decision_type bit 1): an irregular,
    deep, <= 255-leaf tree with a float32 accumulator."""
    sf = np.asarray(t["split_feature"], np.int64)
    n_int = sf.shape[0]
    lv = np.asarray(t["leaf_value"], np.float64)
    n = n_int + lv.shape[0]
    cleft = np.full(n, -1, np.int32)
    cright = np.full(n, -1, np.int32)
    fix = lambda c: c if c >= 0 else n_int + (~c)          # noqa: E731
    for i in range(n_int):
        cleft[i] = fix(int(t["left_child"][i]))
        cright[i] = fix(int(t["right_child"][i]))
    dl = (np.asarray(t["decision_type"], np.int64) >> 1) & 1
    sindex = np.zeros(n, np.uint32)
    sindex[:n_int] = sf.astype(np.uint32) | (dl.astype(np.uint32) << 31)
    value = np.zeros(n, np.float32)
    value[:n_int] = np.asarray(t["threshold"], np.float64).astype(np.float32)
    value[n_int:] = (lv * 0.1).astype(np.float32)
    return {"cleft": cleft, "cright": cright, "sindex": sindex, "value": value}


@pytest.mark.parametrize("tx8", [1, 0])
def test_u8_multiclass_lightgbm(monkeypatch, tx8):
    """K = 3 output groups on u8 bins (the deferred leaf adds of the
    compact bottom land in tree_group t mod 3), raw scores and leaf ids bit
    exact against the C port."""
    monkeypatch.setenv("TI_TX8", str(tx8))
    trees = lf.synthetic_maxbin_trees(45, 200, 20, seed=31)
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "model.txt")
        lf.write_lightgbm_text(p, trees, 20, "multiclass num_class:3", num_class=3)
        f = load_lightgbm_model(p)
    dev = DeviceForest(f, [0])
    info = dev.info()
    assert info["layout"] == TEXPLICIT and info["bin_bits"] == 8 and info["bottom"] == tx8
    X = _inputs(trees, 2500, 20, seed=32, special_frac=0.01)
    for Xi in (X, X.astype(np.float32)):
        want = port.lgb_predict_raw(trees, 3, 20, Xi.astype(np.float64))
        assert np.array_equal(dev.predict(Xi, OUT_MARGIN), want)


@pytest.mark.parametrize("tx8", [1, 0])
def test_u8_float32_accumulator_xgboost(monkeypatch, tx8):
    """a float32-accumulating forest (XGBoost, 4-byte leaf table of
    the compact bottom) on u8 bins: deep irregular trees of <= 255 leaves with
    at most 254 distinct thresholds a feature; margins bit-exact against the
    xgboost restatement."""
    from kfserving_amd.formats.xgboost_format import forest_from_raw_trees
    from oracle import xgb_ref
    monkeypatch.setenv("TI_TX8", str(tx8))
    lt = lf.synthetic_maxbin_trees(40, 255, 16, seed=33)
    raw = [_lgb_to_xgb_raw(t) for t in lt]
    ti = np.zeros(len(raw), np.int32)
    f = forest_from_raw_trees(raw, ti, 16, 0, 0.0, "binary:logistic")
    ref = xgb_ref.from_raw_trees(raw, ti, 16, 0, 0.0, "binary:logistic")
    dev = DeviceForest(f, [0])
    info = dev.info()
    assert info["layout"] == TEXPLICIT and info["bin_bits"] == 8 and info["bottom"] == tx8
    X = _inputs(lt, 3000, 16, seed=34, special_frac=0.01).astype(np.float32)
    assert np.array_equal(dev.predict(X, OUT_MARGIN), xgb_ref.predict(ref, X, output_margin=True))
    assert np.array_equal(dev.predict(X, OUT_LEAF), xgb_ref.leaf_index(ref, X))


def test_u8_vector_leaves_sklearn_classifier(monkeypatch):
    """vector leaves (leaf_width = K) through the compact bottom's
    ordinal table: a sklearn RandomForestClassifier, 3 classes, depth up to 14,
    <= 200 leaves a tree, features of <= 60 distinct values (u8 bins);
    predict_proba bit-exact against sklearn itself and the u16 image."""
    from sklearn.ensemble import RandomForestClassifier
    from kfserving_amd.forest import OUT_PREDICT
    from kfserving_amd.formats.sklearn_format import forest_from_sklearn
    rng = np.random.default_rng(35)
    Xt = rng.integers(0, 60, (4000, 12)).astype(np.float32)
    y = ((Xt[:, 0] + Xt[:, 1] * 0.5 + rng.normal(0, 8, 4000)) // 30).astype(int) % 3
    est = RandomForestClassifier(n_estimators=12, max_depth=14, max_leaf_nodes=200,
                                 random_state=0).fit(Xt, y)
    f = forest_from_sklearn(est)
    monkeypatch.setenv("TI_FORCE_LAYOUT", "texplicit")
    d8 = _device(f, monkeypatch, True)
    d16 = _device(f, monkeypatch, False)
    info = d8.info()
    assert info["layout"] == TEXPLICIT and info["bin_bits"] == 8 and info["bottom"] == 1, info
    X = rng.integers(-2, 62, (3000, 12)).astype(np.float32)
    X[rng.random(X.shape) < 0.01] = np.nan
    want = est.predict_proba(X)
    got = d8.predict(X, OUT_MARGIN)                  # a classifier's margin: the mean proba
    np.testing.assert_array_equal(got.reshape(want.shape), want)
    assert np.array_equal(got, d16.predict(X, OUT_MARGIN))
    assert np.array_equal(d8.predict(X, OUT_PREDICT), est.predict(X).astype(np.float64))
    assert np.array_equal(d8.predict(X, OUT_LEAF), d16.predict(X, OUT_LEAF))
