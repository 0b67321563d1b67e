"""The oracle is pinned before it is trusted: every known answer the reference
holds for this path, sklearn's own outputs, and C-port == numpy restatement."""
import json
import os

import numpy as np
import pytest

from oracle import lgb_ref, port, sk_ref, xgb_ref


def _ka(golden):
    with open(os.path.join(golden, "known_answers.json")) as fh:
        return json.load(fh)


def _iris(golden):
    with open(os.path.join(golden, "iris_input.json")) as fh:
        return np.array(json.load(fh)["instances"])


def test_xgb_legacy_known_answers(golden):
    m = xgb_ref.read_xgb_binary(os.path.join(golden, "xgb_iris_legacy_082.bst"))
    ka = _ka(golden)
    # python/xgbserver/xgbserver/test_model.py:42-44
    assert xgb_ref.predict(m, np.array(ka["xgb_legacy_X0"]["instances"])).tolist() == [0]
    # test/e2e/predictor/test_xgboost.py:67-68
    assert xgb_ref.predict(m, _iris(golden)).tolist() == [1, 1]


def test_xgb_binf_known_answer(golden):
    m = xgb_ref.read_xgb_binary(os.path.join(golden, "xgb_iris_binf_1x.bst"))
    assert m.major_version == 1
    # docs/samples/v1beta1/xgboost/README.md:178
    assert xgb_ref.predict(m, _iris(golden)).tolist() == [1.0, 1.0]


def test_lgb_known_answers(golden):
    m = lgb_ref.read_lgb_text(os.path.join(golden, "lgb_iris_v3.txt"))
    assert len(m.trees) == 300 and m.num_tree_per_iteration == 3
    ka = _ka(golden)
    rows = lgb_ref.rows_from_inputs(m, ka["lgb_dict_row"]["inputs"])
    p = lgb_ref.predict(m, rows)
    assert int(np.argmax(p[0])) == 0        # lgbserver/test_model.py:43-47
    with open(os.path.join(golden, "iris_input_v3.json")) as fh:
        v3 = json.load(fh)["inputs"]
    assert lgb_ref.predict(m, lgb_ref.rows_from_inputs(m, v3))[0][0] > 0.5  # test_lightgbm.py:65-67


def _sk_trees(path):
    z = np.load(path, allow_pickle=False)
    keys = ("children_left", "children_right", "feature", "threshold", "missing_go_to_left",
            "value")
    return [{k: z[f"t{i}_{k}"] for k in keys} for i in range(int(z["n_trees"]))], z


def test_sklearn_restatement_matches_sklearn(golden):
    trees, _ = _sk_trees(os.path.join(golden, "sk_rf_reg_model.npz"))
    g = np.load(os.path.join(golden, "sk_rf_reg.npz"))
    assert np.array_equal(sk_ref.apply(trees, g["X"]), g["apply"])
    assert np.array_equal(sk_ref.predict_regressor(trees, g["X"]), g["predict"])   # bit-exact
    trees, z = _sk_trees(os.path.join(golden, "sk_rf_clf_model.npz"))
    g = np.load(os.path.join(golden, "sk_rf_clf.npz"))
    assert np.array_equal(sk_ref.predict_proba(trees, g["X"], 3), g["predict_proba"])
    assert np.array_equal(sk_ref.predict_classifier(trees, g["X"], z["classes"]), g["predict"])


def test_synthetic_goldens_reproduce(golden):
    from kfserving_amd.formats.xgboost_format import synthetic_complete_trees
    g = np.load(os.path.join(golden, "xgb_synth.npz"))
    trees, ti = synthetic_complete_trees(40, 8, 28, seed=1)
    m = xgb_ref.from_raw_trees(trees, ti, 28, 0, 0.0, "binary:logistic")
    assert np.array_equal(xgb_ref.predict(m, g["X"], output_margin=True), g["margin"])


def test_c_port_matches_numpy_restatement(golden):
    from kfserving_amd.formats.lightgbm_format import synthetic_leafwise_trees
    from kfserving_amd.formats.xgboost_format import synthetic_complete_trees
    rng = np.random.default_rng(3)
    X = rng.standard_normal((500, 28)).astype(np.float32)
    X[rng.random(X.shape) < 0.02] = np.nan
    trees, ti = synthetic_complete_trees(30, 8, 28, seed=9)
    m = xgb_ref.from_raw_trees(trees, ti, 28, 0, 0.0, "binary:logistic")
    got = port.xgb_predict(trees, ti, 1, 0.0, 28, X)[:, 0]
    assert np.array_equal(got, xgb_ref.predict(m, X, output_margin=True))
    lt = synthetic_leafwise_trees(10, 31, 28, seed=4)
    lm = lgb_ref.from_raw_trees(lt, 28, "binary sigmoid:1")
    Xd = X.astype(np.float64)
    assert np.array_equal(port.lgb_predict_raw(lt, 1, 28, Xd)[:, 0],
                          lgb_ref.predict(lm, Xd, raw_score=True))
    trees_sk, _ = _sk_trees(os.path.join(golden, "sk_rf_reg_model.npz"))
    g = np.load(os.path.join(golden, "sk_rf_reg.npz"))
    assert np.array_equal(port.sk_predict(trees_sk, 1, 64, g["X"])[:, 0], g["predict"])


@pytest.mark.parametrize("missing", ["nan", "csr"])
def test_xgb_missing_modes_differ_only_on_zero_and_nan(missing):
    from kfserving_amd.formats.xgboost_format import synthetic_complete_trees
    trees, ti = synthetic_complete_trees(5, 4, 4, seed=2)
    m = xgb_ref.from_raw_trees(trees, ti, 4, 0, 0.0, "binary:logistic")
    X = np.array([[0.5, -0.3, 1.2, 2.0]], dtype=np.float32)
    a = xgb_ref.predict(m, X, output_margin=True, missing=missing)
    b = xgb_ref.predict(m, X, output_margin=True)
    assert np.array_equal(a, b)
