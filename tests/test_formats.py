"""Loaders -> canonical forest, checked on CPU against the oracle through the
canonical-semantics evaluator (tests/canon_eval.py)."""
import json
import os

import numpy as np
import pytest

from kfserving_amd.forest import OUT_LEAF, OUT_MARGIN, OUT_PREDICT, round_down_f32
from kfserving_amd.formats import (forest_from_sklearn, load_lightgbm_model, load_tree_arrays,
                                   load_xgboost_model, parse_xgboost_bytes)
from kfserving_amd.formats import xgboost_format as xf
from kfserving_amd.formats import lightgbm_format as lf
from kfserving_amd.tree_model import lgb_matrix_from_inputs, xgb_matrix_from_list
from oracle import lgb_ref, xgb_ref
from tests import canon_eval


def _iris():
    from sklearn.datasets import load_iris
    return load_iris()["data"]


@pytest.mark.parametrize("name", ["xgb_iris_legacy_082.bst", "xgb_iris_binf_1x.bst"])
def test_xgb_fixture_canonical_matches_oracle(golden, name):
    path = os.path.join(golden, name)
    f = load_xgboost_model(path)
    assert f.meta["trailing_bytes"] == 0
    m = xgb_ref.read_xgb_binary(path)
    X = _iris().astype(np.float32)
    assert f.n_trees == 100 and f.n_groups == 10
    np.testing.assert_array_equal(canon_eval.predict(f, X, OUT_MARGIN),
                                  xgb_ref.predict(m, X, output_margin=True))
    np.testing.assert_array_equal(canon_eval.predict(f, X, OUT_PREDICT), xgb_ref.predict(m, X))
    np.testing.assert_array_equal(canon_eval.predict(f, X, OUT_LEAF), xgb_ref.leaf_index(m, X))


def test_lgb_fixture_canonical_matches_oracle(golden):
    path = os.path.join(golden, "lgb_iris_v3.txt")
    f = load_lightgbm_model(path)
    m = lgb_ref.read_lgb_text(path)
    X = _iris()
    np.testing.assert_array_equal(canon_eval.predict(f, X, OUT_MARGIN),
                                  lgb_ref.predict(m, X, raw_score=True))
    np.testing.assert_allclose(canon_eval.predict(f, X, OUT_PREDICT), lgb_ref.predict(m, X),
                               rtol=1e-12)
    np.testing.assert_array_equal(canon_eval.predict(f, X, OUT_LEAF), lgb_ref.leaf_index(m, X))
    # float32 input path: exact via round_down_f32 thresholds
    X32 = X.astype(np.float32)
    np.testing.assert_array_equal(canon_eval.predict(f, X32, OUT_MARGIN),
                                  lgb_ref.predict(m, X32.astype(np.float64), raw_score=True))


def test_lgb_synthetic_missing_types(golden):
    g = np.load(os.path.join(golden, "lgb_synth.npz"))
    trees = lf.synthetic_leafwise_trees(20, 63, 28, seed=3)
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "model.txt")
        lf.write_lightgbm_text(p, trees, 28, "binary sigmoid:1")
        f = load_lightgbm_model(p)
        m = lgb_ref.read_lgb_text(p)
    np.testing.assert_array_equal(canon_eval.predict(f, g["X"], OUT_MARGIN), g["raw"])
    np.testing.assert_array_equal(lgb_ref.predict(m, g["X"], raw_score=True), g["raw"])
    np.testing.assert_array_equal(canon_eval.predict(f, g["X"], OUT_LEAF), g["leaf"])


CAT_KA_C = [1, 3, 3.7, 33, 33.99, 2, 0, -0.5, -1, 32, 64, float("nan"), 1e10, -1e10, 1e-36]
CAT_KA_WANT = [10, 10, 10, 10, 10, 20, 20, 20, 20, 20, 20, 20, 20, 20, 20.]


def test_lgb_categorical_known_answers(golden):
    """Hand-computed Tree::CategoricalDecision answers: the bitset {1, 3, 33}
    (words 0b1010, 0b10); trunc toward zero; NaN / negative / past-the-bitset
    / out-of-int-range go right (to the numerical split on x <= 0.5,
    default-left so NaN x goes left)."""
    p = os.path.join(golden, "lgb_categorical_ka.txt")
    f = load_lightgbm_model(p)
    assert f.has_categorical and f.cat_bits.tolist() == [10, 2]
    c = np.array(CAT_KA_C)
    want = np.array(CAT_KA_WANT)
    X = np.stack([c, np.zeros_like(c)], axis=1)
    m = lgb_ref.read_lgb_text(p)
    np.testing.assert_array_equal(lgb_ref.predict(m, X), want)
    np.testing.assert_array_equal(canon_eval.predict(f, X, OUT_MARGIN), want)
    X[:, 1] = 1.0
    want2 = np.where(want == 10, 10, 30.)
    np.testing.assert_array_equal(canon_eval.predict(f, X, OUT_MARGIN), want2)
    np.testing.assert_array_equal(canon_eval.predict(f, X.astype(np.float32), OUT_MARGIN), want2)


def test_lgb_categorical_synthetic_matches_oracle(tmp_path):
    trees = lf.synthetic_leafwise_trees(30, 31, 12, seed=11)
    lf.add_categorical_splits(trees, [0, 3, 7], n_categories=70, seed=12)
    p = str(tmp_path / "model.txt")
    lf.write_lightgbm_text(p, trees, 12, "multiclass num_class:3", num_class=3)
    f = load_lightgbm_model(p)
    m = lgb_ref.read_lgb_text(p)
    assert f.has_categorical
    rng = np.random.default_rng(5)
    X = rng.standard_normal((3000, 12))
    for j in (0, 3, 7):
        X[:, j] = rng.integers(-3, 80, size=3000) + rng.choice([0, 0.25, 0.999], size=3000)
        X[rng.random(3000) < 0.05, j] = np.nan
    np.testing.assert_array_equal(canon_eval.predict(f, X, OUT_LEAF), lgb_ref.leaf_index(m, X))
    np.testing.assert_array_equal(canon_eval.predict(f, X, OUT_MARGIN),
                                  lgb_ref.predict(m, X, raw_score=True))


def test_lgb_categorical_bad_index(golden, tmp_path):
    p = tmp_path / "bad.txt"
    text = open(os.path.join(golden, "lgb_categorical_ka.txt")).read()
    p.write_text(text.replace("threshold=0 0.5", "threshold=1 0.5"))
    with pytest.raises(lf.LightGBMFormatError):
        load_lightgbm_model(str(p))


def test_xgb_writers_roundtrip(tmp_path):
    trees, ti = xf.synthetic_complete_trees(12, 5, 10, seed=4, num_class=3)
    pb = str(tmp_path / "m.bst")
    pj = str(tmp_path / "m.json")
    pu = str(tmp_path / "m.ubj")
    xf.write_legacy_binary(pb, trees, ti, 10, 3, 0.5, "multi:softprob")
    xf.write_json_model(pj, trees, ti, 10, 3, 0.5, "multi:softprob")
    xf.write_ubj_model(pu, trees, ti, 10, 3, 0.5, "multi:softprob")
    fb, fj, fu = load_xgboost_model(pb), load_xgboost_model(pj), load_xgboost_model(pu)
    assert fu.meta["format"] == "ubj" and fj.meta["format"] == "json"
    for k in ("feature", "threshold", "flags", "left", "right", "leaf_value", "tree_group"):
        assert np.array_equal(getattr(fu, k), getattr(fj, k)), k
    m = xgb_ref.read_xgb_binary(pb)
    rng = np.random.default_rng(0)
    X = rng.standard_normal((300, 10)).astype(np.float32)
    X[rng.random(X.shape) < 0.05] = np.nan
    want = xgb_ref.predict(m, X, output_margin=True)
    np.testing.assert_array_equal(canon_eval.predict(fb, X, OUT_MARGIN), want)
    np.testing.assert_array_equal(canon_eval.predict(fj, X, OUT_MARGIN), want)  # base 0.5 identity
    # .ubj carries version 1.6: xgboost >= 1.4 starts the sum at base_score
    # (base first), so margins match within float32 rounding, not bitwise
    assert fu.base_first and not fb.base_first
    np.testing.assert_allclose(canon_eval.predict(fu, X, OUT_MARGIN), want, rtol=1e-6)


def test_ubjson_roundtrip_values():
    from kfserving_amd.formats import ubjson
    doc = {"a": [1, 2.5, "x", True, None, {"b": []}], "f": np.arange(300, dtype=np.float32),
           "i": np.arange(5, dtype=np.int32), "s": "é" * 300}
    back = ubjson.loads(ubjson.dumps(doc))
    assert back["a"] == [1, 2.5, "x", True, None, {"b": []}] and back["s"] == doc["s"]
    assert np.array_equal(back["f"], doc["f"]) and back["f"].dtype == np.float32
    assert np.array_equal(back["i"], doc["i"])
    with pytest.raises(ubjson.UBJSONError):
        ubjson.loads(b"[$d#U\x05\x00")


def test_xgb_threshold_encoding_edges():
    s = np.array([0.0, -0.0, 1.0, np.float32(1e-45), np.inf, -np.inf], dtype=np.float32)
    t = xf.xgb_threshold(s)
    xs = np.array([0.0, -0.0, 1.0, np.float32(1e-45), 0.99999994, np.inf, -np.inf, 3.0],
                  dtype=np.float32)
    for si, ti in zip(s, t):
        assert np.array_equal(xs < si, xs.astype(np.float64) <= ti), (si, ti)


def test_round_down_f32_exact():
    rng = np.random.default_rng(1)
    t = np.concatenate([rng.standard_normal(1000), [3.1500000000000004, 1e300, -1e300, 0.0,
                                                    np.inf, -np.inf, 1e-45, 5e-324]])
    r = round_down_f32(t)
    x = np.concatenate([r, np.nextafter(r, np.float32(np.inf)), rng.standard_normal(1000).astype(np.float32)])
    for ti, ri in zip(t, r):
        assert np.array_equal(x.astype(np.float64) <= ti, x <= ri)


def test_sklearn_arrays_roundtrip(golden):
    f = load_tree_arrays(os.path.join(golden, "sk_rf_reg_model.npz"))
    g = np.load(os.path.join(golden, "sk_rf_reg.npz"))
    np.testing.assert_array_equal(canon_eval.predict(f, g["X"], OUT_PREDICT), g["predict"])
    np.testing.assert_array_equal(canon_eval.predict(f, g["X"], OUT_LEAF), g["apply"])
    fc = load_tree_arrays(os.path.join(golden, "sk_rf_clf_model.npz"))
    gc = np.load(os.path.join(golden, "sk_rf_clf.npz"))
    np.testing.assert_array_equal(canon_eval.predict(fc, gc["X"], OUT_MARGIN), gc["predict_proba"])
    lab = fc.meta["classes"].take(canon_eval.predict(fc, gc["X"], OUT_PREDICT).astype(int))
    np.testing.assert_array_equal(lab, gc["predict"])


def test_sklearn_live_estimator():
    from sklearn.ensemble import ExtraTreesRegressor
    rng = np.random.default_rng(2)
    X = rng.standard_normal((400, 6)).astype(np.float32)
    y = X[:, 0] - X[:, 1] ** 2
    est = ExtraTreesRegressor(n_estimators=5, random_state=0).fit(X, y)
    f = forest_from_sklearn(est)
    np.testing.assert_array_equal(canon_eval.predict(f, X, OUT_PREDICT), est.predict(X))


def test_xgb_list_semantics():
    X = xgb_matrix_from_list([[0.0, 1.5, float("nan"), -0.0]])
    assert np.isnan(X[0, 0]) and X[0, 1] == np.float32(1.5) and np.isinf(X[0, 2])
    assert np.isnan(X[0, 3])
    assert xgb_matrix_from_list([1.0, 2.0]).shape == (1, 2)


def test_lgb_inputs_by_name():
    names = ["a", "b", "c"]
    X = lgb_matrix_from_inputs([{"c": [3.0], "a": [1.0], "x": [9.0]}], names)
    assert X.shape == (1, 3) and X[0, 0] == 1.0 and np.isnan(X[0, 1]) and X[0, 2] == 3.0
    X = lgb_matrix_from_inputs([{"a": {"0": 1.0}, "b": {"0": 2}, "c": {"0": 3}}] * 2, names)
    assert X.tolist() == [[1.0, 2.0, 3.0], [1.0, 2.0, 3.0]]


def test_malformed_xgb_rejected():
    with pytest.raises(ValueError):
        parse_xgboost_bytes(b"\x00" * 100)


# ----------------------------------------------- sklearn GradientBoosting
def _gb_models():
    from sklearn.ensemble import GradientBoostingClassifier, GradientBoostingRegressor
    rng = np.random.default_rng(0)
    X = rng.standard_normal((600, 7)).astype(np.float32)
    y = X[:, 0] * 2 + np.sin(X[:, 1]) + 0.1 * rng.standard_normal(600)
    reg = GradientBoostingRegressor(n_estimators=25, max_depth=4, learning_rate=0.07,
                                    random_state=0).fit(X, y)
    binc = GradientBoostingClassifier(n_estimators=20, max_depth=3, random_state=0) \
        .fit(X, (y > 0.3).astype(int))
    mult = GradientBoostingClassifier(n_estimators=15, max_depth=3, random_state=0) \
        .fit(X, np.digitize(y, [-1.0, 0.0, 1.5]))
    zero = GradientBoostingRegressor(n_estimators=10, max_depth=3, init="zero",
                                     random_state=0).fit(X, y)
    return X, reg, binc, mult, zero


def test_sklearn_gradient_boosting_restated_bit_exact():
    """canonical forest (numpy evaluator) == sklearn's own decision_function / predict"""
    from kfserving_amd.formats.sklearn_format import forest_from_sklearn
    from kfserving_amd.forest import OUT_MARGIN, OUT_PREDICT
    X, reg, binc, mult, zero = _gb_models()
    Xt = np.random.default_rng(1).standard_normal((500, 7)).astype(np.float32)
    Xt[:5] = X[:5]
    for est in (reg, zero):
        f = forest_from_sklearn(est)
        assert np.array_equal(canon_eval.predict(f, Xt, OUT_PREDICT), est.predict(Xt))
    for est in (binc, mult):
        f = forest_from_sklearn(est)
        raw = canon_eval.predict(f, Xt, OUT_MARGIN)
        want = est.decision_function(Xt)
        assert np.array_equal(raw.reshape(want.shape), want)
        lab = f.meta["classes"].take(canon_eval.predict(f, Xt, OUT_PREDICT).astype(np.int64))
        assert np.array_equal(lab, est.predict(Xt))


def test_sklearn_request_checks_in_float32(golden, tmp_path):
    """sklearn converts X to float32 before its finiteness check, so a finite
    float64 beyond the float32 range is rejected like infinity."""
    import shutil
    from kfserving_amd.sklearnserver import SKLearnModel
    shutil.copy(os.path.join(golden, "sk_rf_reg_model.npz"), str(tmp_path / "model.npz"))
    model = SKLearnModel("sk", str(tmp_path))
    assert model.load()
    row = [0.5] * model._forest.n_features
    model.request_matrix({"instances": [row]})
    for v in (1e39, -1e39, float("inf")):
        with pytest.raises(ValueError, match="infinity or a value too large"):
            model.request_matrix({"instances": [[v] + row[1:]]})


def test_lgb_inputs_dtype_rules():
    """Columns pandas would not type as numbers fail lightgbm's dtype check
    (numeric strings, all-None columns); None beside numbers reads NaN."""
    X = lgb_matrix_from_inputs([{"a": [1, 2.5], "b": [None, 3]}], ["a", "b"])
    assert np.isnan(X[0, 1]) and X[1, 1] == 3
    for bad in ([{"a": ["1.5"], "b": [1]}], [{"a": [None], "b": [1]}]):
        with pytest.raises(ValueError, match="dtypes"):
            lgb_matrix_from_inputs(bad, ["a", "b"])
