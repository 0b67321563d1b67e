"""GPU parity: libtreeinfer (through the C ABI) vs the oracle / sklearn itself.

Bar (BASELINE.json north_star): bit-exact leaf indices and class labels;
margins and probabilities within 1e-5 relative.  Where the accumulation order
is the library's own (XGBoost float32 sequential sum, LightGBM / sklearn
float64 sequential sum) the margins are compared bit-exactly.
"""
import json
import os
import tempfile

import numpy as np
import pytest

from kfserving_amd.engine import DeviceForest, TreeInferError
from kfserving_amd.forest import OUT_LEAF, OUT_MARGIN, OUT_PREDICT
from kfserving_amd.formats import (load_lightgbm_model, load_tree_arrays, load_xgboost_model)
from kfserving_amd.formats import lightgbm_format as lf
from kfserving_amd.formats import xgboost_format as xf
from oracle import lgb_ref, port, xgb_ref

pytestmark = pytest.mark.gpu

RTOL = 1e-5   # north_star tolerance for transformed outputs


def _model_dir(golden, fname, target="model.bst"):
    d = tempfile.mkdtemp()
    os.symlink(os.path.join(golden, fname), os.path.join(d, target))
    return d


def _iris_instances(golden):
    with open(os.path.join(golden, "iris_input.json")) as fh:
        return json.load(fh)["instances"]


# ------------------------------------------------------------ known answers
def test_xgbserver_known_answers(golden):
    from kfserving_amd.xgbserver import XGBoostModel
    model = XGBoostModel("model", _model_dir(golden, "xgb_iris_legacy_082.bst"), 1)
    model.load()
    # python/xgbserver/xgbserver/test_model.py:42-44
    assert model.predict({"instances": [[5.1, 3.5, 1.4, 0.2]]})["predictions"] == [0]
    # test/e2e/predictor/test_xgboost.py:67-68
    assert model.predict({"instances": _iris_instances(golden)})["predictions"] == [1, 1]
    m2 = XGBoostModel("m2", _model_dir(golden, "xgb_iris_binf_1x.bst"), 1)
    m2.load()
    assert m2.predict({"instances": _iris_instances(golden)})["predictions"] == [1.0, 1.0]


def test_lgbserver_known_answers(golden):
    from kfserving_amd.lgbserver import LightGBMModel
    model = LightGBMModel("model", _model_dir(golden, "lgb_iris_v3.txt"), 1)
    model.load()
    request = {"x": {0: 1.1}, 'sepal_width_(cm)': {0: 3.5}, 'petal_length_(cm)': {0: 1.4},
               'petal_width_(cm)': {0: 0.2}, 'sepal_length_(cm)': {0: 5.1}}
    response = model.predict({"inputs": [request, request]})
    assert np.argmax(response["predictions"][0]) == 0       # lgbserver/test_model.py:43-47
    with open(os.path.join(golden, "iris_input_v3.json")) as fh:
        res = model.predict(json.load(fh))
    assert res["predictions"][0][0] > 0.5                    # test_lightgbm.py:65-67
    m = lgb_ref.read_lgb_text(os.path.join(golden, "lgb_iris_v3.txt"))
    want = lgb_ref.predict(m, lgb_ref.rows_from_inputs(m, [request]))
    np.testing.assert_allclose(response["predictions"][0], want[0], rtol=RTOL)


# ---------------------------------------------------------------- fixtures
@pytest.mark.parametrize("name", ["xgb_iris_legacy_082.bst", "xgb_iris_binf_1x.bst"])
def test_xgb_fixture_full_iris(golden, name):
    from sklearn.datasets import load_iris
    path = os.path.join(golden, name)
    f = load_xgboost_model(path)
    m = xgb_ref.read_xgb_binary(path)
    X = load_iris()["data"].astype(np.float32)
    dev = DeviceForest(f, [0])
    assert np.array_equal(dev.predict(X, OUT_MARGIN), xgb_ref.predict(m, X, output_margin=True))
    assert np.array_equal(dev.predict(X, OUT_PREDICT), xgb_ref.predict(m, X))
    assert np.array_equal(dev.predict(X, OUT_LEAF), xgb_ref.leaf_index(m, X))


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_lgb_fixture_full_iris(golden, dtype):
    from sklearn.datasets import load_iris
    path = os.path.join(golden, "lgb_iris_v3.txt")
    f = load_lightgbm_model(path)
    m = lgb_ref.read_lgb_text(path)
    X = load_iris()["data"].astype(dtype)
    dev = DeviceForest(f, [0])
    Xd = X.astype(np.float64)
    assert np.array_equal(dev.predict(X, OUT_MARGIN), lgb_ref.predict(m, Xd, raw_score=True))
    np.testing.assert_allclose(dev.predict(X, OUT_PREDICT), lgb_ref.predict(m, Xd), rtol=RTOL)
    assert np.array_equal(dev.predict(X, OUT_LEAF), lgb_ref.leaf_index(m, Xd))


# -------------------------------------------------------- synthetic goldens
def test_xgb_synthetic_golden(golden):
    g = np.load(os.path.join(golden, "xgb_synth.npz"))
    trees, ti = xf.synthetic_complete_trees(40, 8, 28, seed=1)
    dev = DeviceForest(xf.forest_from_raw_trees(trees, ti, 28, 0, 0.0, "binary:logistic"), [0])
    assert np.array_equal(dev.predict(g["X"], OUT_MARGIN), g["margin"])
    np.testing.assert_allclose(dev.predict(g["X"], OUT_PREDICT), g["prob"], rtol=RTOL)
    assert np.array_equal(dev.predict(g["X"], OUT_LEAF), g["leaf"])
    trees3, ti3 = xf.synthetic_complete_trees(30, 6, 28, seed=2, num_class=3)
    dev3 = DeviceForest(xf.forest_from_raw_trees(trees3, ti3, 28, 3, 0.5, "multi:softprob"), [0])
    assert np.array_equal(dev3.predict(g["X"], OUT_MARGIN), g["margin3"])
    np.testing.assert_allclose(dev3.predict(g["X"], OUT_PREDICT), g["prob3"], rtol=RTOL)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_lgb_synthetic_golden(golden, tmp_path, dtype):
    g = np.load(os.path.join(golden, "lgb_synth.npz"))
    trees = lf.synthetic_leafwise_trees(20, 63, 28, seed=3)
    p = str(tmp_path / "model.txt")
    lf.write_lightgbm_text(p, trees, 28, "binary sigmoid:1")
    dev = DeviceForest(load_lightgbm_model(p), [0])
    X = g["X"].astype(dtype)
    if dtype == np.float64:
        raw, prob, leaf = g["raw"], g["prob"], g["leaf"]
    else:
        lm = lgb_ref.read_lgb_text(p)
        Xd = X.astype(np.float64)
        raw, prob, leaf = (lgb_ref.predict(lm, Xd, raw_score=True), lgb_ref.predict(lm, Xd),
                           lgb_ref.leaf_index(lm, Xd))
    assert np.array_equal(dev.predict(X, OUT_MARGIN), raw)
    np.testing.assert_allclose(dev.predict(X, OUT_PREDICT), prob, rtol=RTOL)
    assert np.array_equal(dev.predict(X, OUT_LEAF), leaf)


# ------------------------------------------------- LightGBM categorical splits
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_lgb_categorical_known_answers_gpu(golden, dtype):
    """Hand-computed Tree::CategoricalDecision answers (tests/test_formats.py)."""
    from tests.test_formats import CAT_KA_C, CAT_KA_WANT
    f = load_lightgbm_model(os.path.join(golden, "lgb_categorical_ka.txt"))
    c = np.array(CAT_KA_C)
    want = np.array(CAT_KA_WANT)
    dev = DeviceForest(f, [0])
    assert dev.info()["layout"] == 1
    for xval, w in ((0.0, want), (1.0, np.where(want == 10, 10, 30.))):
        X = np.stack([c, np.full_like(c, xval)], axis=1).astype(dtype)
        assert np.array_equal(dev.predict(X, OUT_MARGIN), w)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("layout", ["heap", "explicit"])
def test_lgb_categorical_synthetic_gpu(tmp_path, dtype, layout):
    trees = lf.synthetic_leafwise_trees(60, 31, 12, seed=21)
    lf.add_categorical_splits(trees, [0, 3, 7], n_categories=300, seed=22)
    p = str(tmp_path / "model.txt")
    lf.write_lightgbm_text(p, trees, 12, "multiclass num_class:3", num_class=3)
    f = load_lightgbm_model(p)
    m = lgb_ref.read_lgb_text(p)
    rng = np.random.default_rng(23)
    n = 5000
    X = rng.standard_normal((n, 12))
    for j in (0, 3, 7):
        X[:, j] = rng.integers(-5, 320, size=n) + rng.choice([0, 0.5, 0.999], size=n)
        X[rng.random(n) < 0.05, j] = np.nan
        X[rng.random(n) < 0.01, j] = 3e9
    X = X.astype(dtype)
    dev = _dev_with_layout(f, layout)   # categorical forests always run explicit
    assert dev.info()["layout"] == 1
    Xd = X.astype(np.float64)
    assert np.array_equal(dev.predict(X, OUT_LEAF), lgb_ref.leaf_index(m, Xd))
    assert np.array_equal(dev.predict(X, OUT_MARGIN), lgb_ref.predict(m, Xd, raw_score=True))
    np.testing.assert_allclose(dev.predict(X, OUT_PREDICT), lgb_ref.predict(m, Xd), rtol=RTOL)


def test_lgbserver_categorical_plugin(tmp_path):
    from kfserving_amd.lgbserver import LightGBMModel
    trees = lf.synthetic_leafwise_trees(10, 15, 4, seed=31)
    lf.add_categorical_splits(trees, [1], n_categories=40, seed=32)
    lf.write_lightgbm_text(str(tmp_path / "model.bst"), trees, 4, "binary sigmoid:1",
                           feature_names=["a", "cat", "b", "c"])
    model = LightGBMModel("m", str(tmp_path), 1)
    model.load()
    req = {"a": {0: 0.3, 1: -1.0}, "cat": {0: 7, 1: 12}, "b": {0: 0.0, 1: 2.0}, "c": {0: 1.0, 1: 0.5}}
    got = model.predict({"inputs": [req]})["predictions"]
    m = lgb_ref.read_lgb_text(str(tmp_path / "model.bst"))
    np.testing.assert_allclose(got, lgb_ref.predict(m, lgb_ref.rows_from_inputs(m, [req])), rtol=RTOL)


def test_sklearn_goldens_bit_exact(golden):
    f = load_tree_arrays(os.path.join(golden, "sk_rf_reg_model.npz"))
    g = np.load(os.path.join(golden, "sk_rf_reg.npz"))
    dev = DeviceForest(f, [0])
    assert dev.info()["layout"] in (1, 6, 8, 9)   # depth-16 trees: a record layout
    assert np.array_equal(dev.predict(g["X"], OUT_PREDICT), g["predict"])
    assert np.array_equal(dev.predict(g["X"], OUT_LEAF), g["apply"])
    fc = load_tree_arrays(os.path.join(golden, "sk_rf_clf_model.npz"))
    gc = np.load(os.path.join(golden, "sk_rf_clf.npz"))
    devc = DeviceForest(fc, [0])
    assert np.array_equal(devc.predict(gc["X"], OUT_MARGIN), gc["predict_proba"])
    lab = fc.meta["classes"].take(devc.predict(gc["X"], OUT_PREDICT).astype(np.int64))
    assert np.array_equal(lab, gc["predict"])


def test_sklearnserver_plugin(golden, tmp_path):
    import shutil
    from kfserving_amd.sklearnserver import SKLearnModel
    shutil.copy(os.path.join(golden, "sk_rf_clf_model.npz"), str(tmp_path / "model.npz"))
    model = SKLearnModel("m", str(tmp_path))
    assert model.load()
    gc = np.load(os.path.join(golden, "sk_rf_clf.npz"))
    X = np.nan_to_num(gc["X"][:64])
    from oracle import sk_ref
    from tests.test_oracle import _sk_trees
    trees, z = _sk_trees(os.path.join(golden, "sk_rf_clf_model.npz"))
    want = sk_ref.predict_classifier(trees, X, z["classes"]).tolist()
    assert model.predict({"instances": X.tolist()})["predictions"] == want


# ---------------------------------------------------------------- edge cases
@pytest.fixture(scope="module")
def c2_small():
    trees, ti = xf.synthetic_complete_trees(50, 8, 28, seed=21)
    ref = xgb_ref.from_raw_trees(trees, ti, 28, 0, 0.0, "binary:logistic")
    dev = DeviceForest(xf.forest_from_raw_trees(trees, ti, 28, 0, 0.0, "binary:logistic"), [0])
    return trees, ti, ref, dev


@pytest.mark.parametrize("rows", [0, 1, 63, 255, 256, 257, 1000, 4099])
def test_ragged_row_counts(c2_small, rows):
    _, _, ref, dev = c2_small
    X = np.random.default_rng(rows).standard_normal((rows, 28)).astype(np.float32)
    got = dev.predict(X, OUT_MARGIN)
    assert got.shape == (rows,)
    if rows:
        assert np.array_equal(got, xgb_ref.predict(ref, X, output_margin=True))


def test_specials_nan_inf_zero_denormal(c2_small):
    _, _, ref, dev = c2_small
    rng = np.random.default_rng(5)
    X = rng.standard_normal((2000, 28)).astype(np.float32)
    specials = np.array([np.nan, np.inf, -np.inf, 0.0, -0.0, 1e-45, -1e-45, 1e-38],
                        dtype=np.float32)
    mask = rng.random(X.shape) < 0.2
    X[mask] = specials[rng.integers(0, len(specials), mask.sum())]
    assert np.array_equal(dev.predict(X, OUT_MARGIN), xgb_ref.predict(ref, X, output_margin=True))
    assert np.array_equal(dev.predict(X, OUT_LEAF), xgb_ref.leaf_index(ref, X))


def test_fewer_columns_read_as_missing(c2_small):
    _, _, ref, dev = c2_small
    X = np.random.default_rng(6).standard_normal((300, 20)).astype(np.float32)
    Xp = np.concatenate([X, np.full((300, 8), np.nan, np.float32)], axis=1)
    assert np.array_equal(dev.predict(X, OUT_MARGIN), xgb_ref.predict(ref, Xp, output_margin=True))


def test_xgb_list_path_zero_is_missing(golden):
    """xgbserver with a JSON list: 0 -> missing, NaN -> right (DMatrix(list), 0.82)."""
    from kfserving_amd.xgbserver import XGBoostModel
    trees, ti = xf.synthetic_complete_trees(20, 6, 8, seed=8)
    model = XGBoostModel("m", "", 1, booster=xf.forest_from_raw_trees(trees, ti, 8, 0, 0.0,
                                                                        "binary:logistic"))
    ref = xgb_ref.from_raw_trees(trees, ti, 8, 0, 0.0, "binary:logistic")
    rng = np.random.default_rng(9)
    X = rng.standard_normal((200, 8))
    X[rng.random(X.shape) < 0.2] = 0.0
    X[rng.random(X.shape) < 0.1] = np.nan
    got = np.array(model.predict({"instances": X.tolist()})["predictions"], dtype=np.float32)
    np.testing.assert_allclose(got, xgb_ref.predict(ref, X.astype(np.float32), missing="csr"),
                               rtol=RTOL)


def test_device_path_with_row_stride(c2_small):
    torch = pytest.importorskip("torch")
    _, _, ref, dev = c2_small
    X = np.random.default_rng(7).standard_normal((777, 32)).astype(np.float32)
    xt = torch.from_numpy(X).cuda()
    out = torch.empty(777, dtype=torch.float32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    dev.predict_device(xt.data_ptr(), 0, 777, 28, 32, OUT_MARGIN, out.data_ptr(), 777,
                       stream=stream)
    torch.cuda.synchronize()
    want = xgb_ref.predict(ref, np.ascontiguousarray(X[:, :28]), output_margin=True)
    assert np.array_equal(out.cpu().numpy(), want)


def test_row_sharding_across_slots(c2_small):
    trees, ti, ref, _ = c2_small
    dev2 = DeviceForest(xf.forest_from_raw_trees(trees, ti, 28, 0, 0.0, "binary:logistic"),
                        [0, 0])
    X = np.random.default_rng(8).standard_normal((10001, 28)).astype(np.float32)
    assert np.array_equal(dev2.predict(X, OUT_MARGIN), xgb_ref.predict(ref, X, output_margin=True))


def test_errors_are_loud(c2_small):
    _, _, _, dev = c2_small
    with pytest.raises(TreeInferError):
        dev.predict_device(0, 0, 10, 28, 28, OUT_MARGIN, 0, 10)   # null pointers
    with pytest.raises(TreeInferError):
        dev.predict_device(1, 7, 10, 28, 28, OUT_MARGIN, 1, 10)   # bad dtype


# ------------------------------------------------------ full-size properties
def test_c2_full_size_matches_c_port():
    """BASELINE config C2 at full size: 500 depth-8 trees, 28 features, 1M rows.
    Every margin bit-exact against the C/OpenMP restatement of xgboost 0.82."""
    trees, ti = xf.synthetic_complete_trees(500, 8, 28, seed=0)
    dev = DeviceForest(xf.forest_from_raw_trees(trees, ti, 28, 0, 0.0, "binary:logistic"), [0])
    assert dev.info()["layout"] in (0, 3) and dev.info()["depth"] == 8
    rng = np.random.default_rng(0)
    X = rng.standard_normal((1_000_000, 28), dtype=np.float32)
    X[rng.random(X.shape, dtype=np.float32) < 0.01] = np.nan
    got = dev.predict(X, OUT_MARGIN)
    want = port.xgb_predict(trees, ti, 1, 0.0, 28, X)[:, 0]
    assert np.array_equal(got, want)
    prob = dev.predict(X, OUT_PREDICT)
    np.testing.assert_allclose(prob, 1.0 / (1.0 + np.exp(-want.astype(np.float64))), rtol=RTOL)


def test_c2_hist_full_size_matches_c_port():
    """The bench's `c2_hist` key at full size: C2's trees with thresholds on
    253 quantile bin bounds (u8 bins, the fixed walk's u8 instance and its
    cover-permuted image), 1M rows with 1 % NaN: every margin bit-exact
    against the C restatement of xgboost 0.82."""
    trees, ti = xf.synthetic_complete_trees(500, 8, 28, seed=0, max_bin=254)
    dev = DeviceForest(xf.forest_from_raw_trees(trees, ti, 28, 0, 0.0, "binary:logistic"), [0])
    info = dev.info()
    assert info["layout"] == 3 and info["bin_bits"] == 8 and info["walk"] == 2
    rng = np.random.default_rng(4)
    X = rng.standard_normal((1_000_000, 28), dtype=np.float32)
    X[rng.random(X.shape, dtype=np.float32) < 0.01] = np.nan
    assert np.array_equal(dev.predict(X, OUT_MARGIN), port.xgb_predict(trees, ti, 1, 0.0, 28, X)[:, 0])


def test_leafwise_lgb_full_property():
    """Config C3 shape (1000 trees x 255 leaves, 100 features) on 200k rows:
    raw scores bit-exact against the C restatement of lightgbm 2.3.1."""
    trees = lf.synthetic_leafwise_trees(1000, 255, 100, seed=1)
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "model.txt")
        lf.write_lightgbm_text(p, trees, 100, "binary sigmoid:1")
        f = load_lightgbm_model(p)
    dev = DeviceForest(f, [0])
    X = np.random.default_rng(2).standard_normal((200_000, 100)).astype(np.float32)
    got = dev.predict(X, OUT_MARGIN)
    want = port.lgb_predict_raw(trees, 1, 100, X.astype(np.float64))[:, 0]
    assert np.array_equal(got, want)


def test_leafwise_lgb_full_float64_specials():
    """lgbserver's own dtype at C3 shape: the reference predicts a float64
    DataFrame (python/lgbserver/lgbserver/model.py:46-51), so C3 traffic runs
    the float64 bin view.  1000 trees x 255 leaves, 100 features, 250k float64
    rows with NaN, +-0, 1e-36 / -1e-36 (LightGBM's |x| <= 1e-35 zero map),
    1e-35 itself and values that differ from a threshold only past float32
    precision, on the default layout (9): raw scores bit-exact against the C
    restatement, probabilities within 1e-5."""
    trees = lf.synthetic_leafwise_trees(1000, 255, 100, seed=1)
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "model.txt")
        lf.write_lightgbm_text(p, trees, 100, "binary sigmoid:1")
        f = load_lightgbm_model(p)
    dev = DeviceForest(f, [0])
    assert dev.info()["layout"] == LAYOUT_ID["texplicit"]
    rng = np.random.default_rng(5)
    X = rng.standard_normal((250_000, 100))
    thr = np.concatenate([t["threshold"] for t in trees])
    pick = rng.random(X.shape)
    at = thr[rng.integers(0, len(thr), X.shape)]
    X = np.where(pick < 0.05, at, X)                                  # exactly at a threshold
    X = np.where((pick >= 0.05) & (pick < 0.08), at + np.abs(at) * 1e-12, X)   # float64-only gap
    sp = np.array([np.nan, 0.0, -0.0, 1e-36, -1e-36, 1e-35, 2e-35])
    m = rng.random(X.shape) < 0.02
    X[m] = sp[rng.integers(0, len(sp), m.sum())]
    want = port.lgb_predict_raw(trees, 1, 100, X)[:, 0]
    assert np.array_equal(dev.predict(X, OUT_MARGIN), want)
    np.testing.assert_allclose(dev.predict(X[:20_000], OUT_PREDICT),
                               1.0 / (1.0 + np.exp(-want[:20_000])), rtol=RTOL)


# ------------------------------------------------- every layout, same forest
def _dev_with_layout(forest, layout):
    old = os.environ.get("TI_FORCE_LAYOUT")
    os.environ["TI_FORCE_LAYOUT"] = layout
    try:
        return DeviceForest(forest, [0])
    finally:
        if old is None:
            del os.environ["TI_FORCE_LAYOUT"]
        else:
            os.environ["TI_FORCE_LAYOUT"] = old


LAYOUT_ID = {"heap": 0, "explicit": 1, "bheap": 3, "rexplicit": 6, "lexplicit": 7,
             "hexplicit": 8, "texplicit": 9}


@pytest.mark.parametrize("layout", ["bheap", "heap", "explicit", "rexplicit", "lexplicit",
                                    "hexplicit", "texplicit"])
def test_xgb_golden_every_layout(golden, layout):
    g = np.load(os.path.join(golden, "xgb_synth.npz"))
    trees, ti = xf.synthetic_complete_trees(40, 8, 28, seed=1)
    dev = _dev_with_layout(xf.forest_from_raw_trees(trees, ti, 28, 0, 0.0, "binary:logistic"),
                           layout)
    assert dev.info()["layout"] == LAYOUT_ID[layout]
    assert np.array_equal(dev.predict(g["X"], OUT_MARGIN), g["margin"])
    assert np.array_equal(dev.predict(g["X"], OUT_LEAF), g["leaf"])
    trees3, ti3 = xf.synthetic_complete_trees(30, 6, 28, seed=2, num_class=3)
    dev3 = _dev_with_layout(xf.forest_from_raw_trees(trees3, ti3, 28, 3, 0.5, "multi:softprob"),
                            layout)
    assert np.array_equal(dev3.predict(g["X"], OUT_MARGIN), g["margin3"])
    np.testing.assert_allclose(dev3.predict(g["X"], OUT_PREDICT), g["prob3"], rtol=RTOL)


@pytest.mark.parametrize("layout", ["explicit", "rexplicit", "lexplicit", "hexplicit",
                                    "texplicit"])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_lgb_golden_every_layout(golden, tmp_path, layout, dtype):
    g = np.load(os.path.join(golden, "lgb_synth.npz"))
    trees = lf.synthetic_leafwise_trees(20, 63, 28, seed=3)
    p = str(tmp_path / "model.txt")
    lf.write_lightgbm_text(p, trees, 28, "binary sigmoid:1")
    f = load_lightgbm_model(p)
    dev = _dev_with_layout(f, layout)
    assert dev.info()["layout"] == LAYOUT_ID[layout]
    lm = lgb_ref.read_lgb_text(p)
    X = g["X"].astype(dtype)
    Xd = X.astype(np.float64)
    assert np.array_equal(dev.predict(X, OUT_MARGIN), lgb_ref.predict(lm, Xd, raw_score=True))
    assert np.array_equal(dev.predict(X, OUT_LEAF), lgb_ref.leaf_index(lm, Xd))


@pytest.mark.parametrize("layout", ["bheap", "heap", "explicit", "rexplicit", "lexplicit",
                                    "hexplicit", "texplicit"])
def test_lgb_iris_fixture_every_layout(golden, layout):
    from sklearn.datasets import load_iris
    path = os.path.join(golden, "lgb_iris_v3.txt")
    dev = _dev_with_layout(load_lightgbm_model(path), layout)
    m = lgb_ref.read_lgb_text(path)
    X = load_iris()["data"]
    assert np.array_equal(dev.predict(X, OUT_MARGIN), lgb_ref.predict(m, X, raw_score=True))


@pytest.mark.parametrize("layout", ["explicit", "rexplicit", "lexplicit", "hexplicit",
                                    "texplicit"])
def test_sklearn_classifier_every_layout(golden, layout):
    fc = load_tree_arrays(os.path.join(golden, "sk_rf_clf_model.npz"))
    gc = np.load(os.path.join(golden, "sk_rf_clf.npz"))
    dev = _dev_with_layout(fc, layout)
    assert dev.info()["layout"] == LAYOUT_ID[layout]
    assert np.array_equal(dev.predict(gc["X"], OUT_MARGIN), gc["predict_proba"])
    assert np.array_equal(dev.predict(gc["X"], OUT_LEAF), gc["apply"])


@pytest.mark.parametrize("layout", ["rexplicit", "lexplicit", "hexplicit", "texplicit"])
@pytest.mark.parametrize("rows", [1, 255, 257, 3000])
def test_record_zero_missing_and_specials(rows, layout):
    """The record layouts (nodes gathered from global memory / staged in LDS)
    on leaf-wise trees with every missing type: the zero rule runs on a
    dedicated bin of exact 0 (after the |x| <= 1e-35 map)."""
    trees = lf.synthetic_leafwise_trees(41, 255, 40, seed=7)
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "model.txt")
        lf.write_lightgbm_text(p, trees, 40, "binary sigmoid:1")
        f = load_lightgbm_model(p)
    dev = _dev_with_layout(f, layout)
    assert dev.info()["layout"] == LAYOUT_ID[layout]
    rng = np.random.default_rng(rows + 1)
    X = rng.standard_normal((rows, 40))
    sp = np.array([np.nan, 0.0, -0.0, 1e-40, -1e-36, 1e-35, 2e-35, np.inf, -np.inf])
    mask = rng.random(X.shape) < 0.15
    X[mask] = sp[rng.integers(0, len(sp), mask.sum())]
    want = port.lgb_predict_raw(trees, 1, 40, X)[:, 0]
    assert np.array_equal(dev.predict(X, OUT_MARGIN), want)
    X32 = X.astype(np.float32)
    assert np.array_equal(dev.predict(X32, OUT_MARGIN),
                          port.lgb_predict_raw(trees, 1, 40, X32.astype(np.float64))[:, 0])


@pytest.mark.parametrize("layout", ["rexplicit", "lexplicit", "hexplicit", "texplicit"])
@pytest.mark.parametrize("special", ["nan", "zero", "tiny", "none"])
def test_record_layouts_fast_and_slow_tiles(layout, special):
    """Layouts 6 to 9 walk tiles without NaN (and, for zero-missing forests,
    without exact zeros) with the 2-VALU rank step and the rest with the full
    rule: specials confined to a few rows put both kinds of tile in one batch,
    and every tile must agree with the C port bit for bit."""
    trees = lf.synthetic_leafwise_trees(45, 255, 40, seed=11)
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "model.txt")
        lf.write_lightgbm_text(p, trees, 40, "binary sigmoid:1")
        f = load_lightgbm_model(p)
    dev = _dev_with_layout(f, layout)
    assert dev.info()["layout"] == LAYOUT_ID[layout]
    rng = np.random.default_rng(17)
    X = rng.standard_normal((2000, 40))
    v = {"nan": np.nan, "zero": 0.0, "tiny": 1e-36, "none": None}[special]
    if v is not None:
        X[700:705, rng.integers(0, 40, 5)] = v   # tile 2 (256-row tiles) only
        X[1999, 3] = v                           # and the ragged last tile
    want = port.lgb_predict_raw(trees, 1, 40, X)[:, 0]
    assert np.array_equal(dev.predict(X, OUT_MARGIN), want)
    X32 = X.astype(np.float32)
    assert np.array_equal(dev.predict(X32, OUT_MARGIN),
                          port.lgb_predict_raw(trees, 1, 40, X32.astype(np.float64))[:, 0])
    # a forest without zero-missing nodes (XGBoost): NaN tiles only
    xt, xti = xf.synthetic_complete_trees(30, 9, 40, seed=4)
    xfo = xf.forest_from_raw_trees(xt, xti, 40, 0, 0.0, "binary:logistic")
    dx = _dev_with_layout(xfo, layout)
    assert dx.info()["layout"] == LAYOUT_ID[layout]
    assert np.array_equal(dx.predict(X32, OUT_MARGIN), port.xgb_predict(xt, xti, 1, 0.0, 40, X32)[:, 0])


@pytest.mark.parametrize("layout,top", [("hexplicit", 1), ("hexplicit", 3), ("hexplicit", 6),
                                        ("hexplicit", 10), ("texplicit", 1), ("texplicit", 4),
                                        ("texplicit", 6), ("texplicit", 9)])
def test_heap_top_depths(layout, top, monkeypatch):
    """Layouts 8 and 9 at several top depths: the heap top ends above, inside
    and below the trees' leaves (leaf-wise trees of every missing type, padding
    under shallow leaves, bottom entries that are leaves or internal nodes),
    the stage holds one ILP group or several, and a tree ends in its top."""
    monkeypatch.setenv("TI_HX_TOP", str(top))
    monkeypatch.setenv("TI_TX_TOP", str(top))
    monkeypatch.setenv("TI_HX_STAGE", "16" if top <= 6 else "4")
    monkeypatch.setenv("TI_HX_ILP", "8" if top <= 6 else "4")
    trees = lf.synthetic_leafwise_trees(37, 255, 40, seed=13)
    trees.append(lf.synthetic_leafwise_trees(1, 2, 40, seed=14)[0])   # a 1-split tree
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "model.txt")
        lf.write_lightgbm_text(p, trees, 40, "binary sigmoid:1")
        f = load_lightgbm_model(p)
    dev = _dev_with_layout(f, layout)
    assert dev.info()["layout"] == LAYOUT_ID[layout]
    rng = np.random.default_rng(top)
    X = rng.standard_normal((3001, 40))
    sp = np.array([np.nan, 0.0, -0.0, 1e-40, np.inf, -np.inf])
    mask = rng.random(X.shape) < 0.02
    X[mask] = sp[rng.integers(0, len(sp), mask.sum())]
    X[:1024][np.isnan(X[:1024])] = 0.5   # fast tiles first
    X[:1024][X[:1024] == 0] = 0.5
    want = port.lgb_predict_raw(trees, 1, 40, X)[:, 0]
    assert np.array_equal(dev.predict(X, OUT_MARGIN), want)
    X32 = X.astype(np.float32)
    assert np.array_equal(dev.predict(X32, OUT_MARGIN),
                          port.lgb_predict_raw(trees, 1, 40, X32.astype(np.float64))[:, 0])
    lm_leaf = dev.predict(X32, OUT_LEAF)
    ref = _dev_with_layout(f, "rexplicit")
    assert np.array_equal(lm_leaf, ref.predict(X32, OUT_LEAF))


# ------------------------------------------------- sklearn GradientBoosting
def test_sklearn_gradient_boosting_gpu_bit_exact(tmp_path):
    from tests.test_formats import _gb_models
    from kfserving_amd.formats.sklearn_format import forest_from_sklearn
    X, reg, binc, mult, zero = _gb_models()
    Xt = np.random.default_rng(2).standard_normal((3000, 7)).astype(np.float32)
    for est in (reg, zero):
        dev = DeviceForest(forest_from_sklearn(est), [0])
        assert np.array_equal(dev.predict(Xt, OUT_PREDICT), est.predict(Xt))
    for est in (binc, mult):
        f = forest_from_sklearn(est)
        dev = DeviceForest(f, [0])
        want = est.decision_function(Xt)
        assert np.array_equal(dev.predict(Xt, OUT_MARGIN).reshape(want.shape), want)
        lab = f.meta["classes"].take(dev.predict(Xt, OUT_PREDICT).astype(np.int64))
        assert np.array_equal(lab, est.predict(Xt))
    # through the sklearnserver plugin, loading a joblib file as the reference does
    import joblib
    from kfserving_amd.sklearnserver import SKLearnModel
    joblib.dump(mult, str(tmp_path / "model.joblib"))
    model = SKLearnModel("gb", str(tmp_path))
    assert model.load()
    got = model.predict({"instances": Xt[:64].tolist()})["predictions"]
    assert got == est.predict(Xt[:64]).tolist()
    with pytest.raises(Exception, match="NaN"):
        model.predict({"instances": [[float("nan")] * 7]})


@pytest.mark.parametrize("layout", ["rexplicit", "lexplicit", "hexplicit", "texplicit"])
def test_cover_order_changes_layout_only(golden, layout, monkeypatch):
    """Hot-nodes-first slots (cover_order / leaf_order) against breadth-first
    slots (TI_COVER_ORDER=0) and a forest without covers: probabilities and
    leaf ids identical on every record layout (vector leaves through the
    leaf tables, whose numbering follows the slot order)."""
    fc = load_tree_arrays(os.path.join(golden, "sk_rf_clf_model.npz"))
    gc = np.load(os.path.join(golden, "sk_rf_clf.npz"))
    outs = []
    for setting in ("1", "0", "none"):
        monkeypatch.setenv("TI_COVER_ORDER", "0" if setting == "0" else "1")
        f = fc
        if setting == "none":
            import copy
            f = copy.copy(fc)
            f.cover = None
        dev = _dev_with_layout(f, layout)
        assert dev.info()["layout"] == LAYOUT_ID[layout]
        outs.append((dev.predict(gc["X"], OUT_MARGIN), dev.predict(gc["X"], OUT_LEAF)))
    for m, leaf in outs:
        assert np.array_equal(m, gc["predict_proba"]) and np.array_equal(leaf, gc["apply"])
