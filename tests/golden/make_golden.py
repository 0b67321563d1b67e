"""Regenerate the committed golden vectors under tests/golden/.

Run from the repo root:  python tests/golden/make_golden.py

* sk_rf_reg.npz / sk_rf_clf.npz -- sklearn 1.7.2 itself (the library the
  reference's sklearnserver calls at python/sklearnserver/sklearnserver/
  model.py:50): seeded RandomForest{Regressor,Classifier} fitted here, their
  raw tree arrays (no pickle), inputs with NaNs, and sklearn's own
  predict / predict_proba / apply outputs (n_jobs=1, estimator order).
* xgb_synth.npz / lgb_synth.npz -- seeded synthetic XGBoost (complete depth 8,
  binary:logistic and multi:softprob) and LightGBM (leaf-wise, all three
  missing types) models with the oracle restatement's outputs
  ("parity unpinned vs library": xgboost / lightgbm are not installed).
* known_answers.json -- the reference's own known answers for this path.

The reference fixture files copied next to this script (data, not source):
  xgb_iris_legacy_082.bst <- python/xgbserver/xgbserver/example_model/model/model.bst
  xgb_iris_binf_1x.bst    <- docs/samples/v1beta1/xgboost/model.bst
  lgb_iris_v3.txt         <- python/lgbserver/lgbserver/example_model/model/model.bst
  iris_input.json         <- test/e2e/data/iris_input.json
  iris_input_v3.json      <- test/e2e/data/iris_input_v3.json
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))


def sklearn_goldens():
    from sklearn.ensemble import RandomForestClassifier, RandomForestRegressor
    from kfserving_amd.formats.sklearn_format import save_tree_arrays

    rng = np.random.default_rng(7)
    # regressor: 64 features, depth 16, trained with missing values
    Xtr = rng.standard_normal((3000, 64)).astype(np.float32)
    ytr = np.sin(Xtr[:, 0] * 2) + Xtr[:, 1] * Xtr[:, 2] + 0.1 * rng.standard_normal(3000)
    Xtr[rng.random(Xtr.shape) < 0.02] = np.nan
    reg = RandomForestRegressor(n_estimators=8, max_depth=16, max_features=1 / 3,
                                random_state=0, n_jobs=1).fit(Xtr, ytr)
    X = rng.standard_normal((2048, 64)).astype(np.float32)
    X[rng.random(X.shape) < 0.01] = np.nan
    X[5] = 0.0
    save_tree_arrays(os.path.join(HERE, "sk_rf_reg_model.npz"), reg)
    np.savez_compressed(os.path.join(HERE, "sk_rf_reg.npz"), X=X, predict=reg.predict(X),
                        apply=reg.apply(X).astype(np.int32))
    # classifier: 16 features, 3 classes, string-free integer labels
    Xc = rng.standard_normal((2000, 16)).astype(np.float32)
    yc = (Xc[:, 0] > 0).astype(int) + (Xc[:, 1] > 0.5).astype(int)
    Xc[rng.random(Xc.shape) < 0.02] = np.nan
    clf = RandomForestClassifier(n_estimators=8, max_depth=12, random_state=0,
                                 n_jobs=1).fit(Xc, yc)
    Xq = rng.standard_normal((2048, 16)).astype(np.float32)
    Xq[rng.random(Xq.shape) < 0.01] = np.nan
    save_tree_arrays(os.path.join(HERE, "sk_rf_clf_model.npz"), clf)
    np.savez_compressed(os.path.join(HERE, "sk_rf_clf.npz"), X=Xq, predict=clf.predict(Xq),
                        predict_proba=clf.predict_proba(Xq),
                        apply=clf.apply(Xq).astype(np.int32))


def synthetic_goldens():
    from kfserving_amd.formats.lightgbm_format import synthetic_leafwise_trees
    from kfserving_amd.formats.xgboost_format import synthetic_complete_trees
    from oracle import lgb_ref, xgb_ref

    rng = np.random.default_rng(11)
    X = rng.standard_normal((2000, 28)).astype(np.float32)
    X[rng.random(X.shape) < 0.01] = np.nan
    X[3] = 0.0
    trees, ti = synthetic_complete_trees(40, 8, 28, seed=1)
    m = xgb_ref.from_raw_trees(trees, ti, 28, 0, 0.0, "binary:logistic")
    trees3, ti3 = synthetic_complete_trees(30, 6, 28, seed=2, num_class=3)
    m3 = xgb_ref.from_raw_trees(trees3, ti3, 28, 3, 0.5, "multi:softprob")
    np.savez_compressed(os.path.join(HERE, "xgb_synth.npz"), X=X,
                        margin=xgb_ref.predict(m, X, output_margin=True),
                        prob=xgb_ref.predict(m, X),
                        leaf=xgb_ref.leaf_index(m, X).astype(np.int32),
                        margin3=xgb_ref.predict(m3, X, output_margin=True),
                        prob3=xgb_ref.predict(m3, X))
    lt = synthetic_leafwise_trees(20, 63, 28, seed=3)
    lm = lgb_ref.from_raw_trees(lt, 28, "binary sigmoid:1")
    Xd = X.astype(np.float64)
    Xd[7, :5] = 1e-40
    np.savez_compressed(os.path.join(HERE, "lgb_synth.npz"), X=Xd,
                        raw=lgb_ref.predict(lm, Xd, raw_score=True),
                        prob=lgb_ref.predict(lm, Xd),
                        leaf=lgb_ref.leaf_index(lm, Xd).astype(np.int32))


def known_answers():
    ka = {
        "xgb_legacy_X0": {"model": "xgb_iris_legacy_082.bst",
                          "instances": [[5.1, 3.5, 1.4, 0.2]], "predictions": [0],
                          "source": "python/xgbserver/xgbserver/test_model.py:42-44"},
        "xgb_legacy_iris": {"model": "xgb_iris_legacy_082.bst", "input": "iris_input.json",
                            "predictions": [1, 1],
                            "source": "test/e2e/predictor/test_xgboost.py:67-68"},
        "xgb_binf_iris": {"model": "xgb_iris_binf_1x.bst", "input": "iris_input.json",
                          "predictions": [1.0, 1.0],
                          "source": "docs/samples/v1beta1/xgboost/README.md:178"},
        "lgb_dict_row": {"model": "lgb_iris_v3.txt",
                         "inputs": [{"x": {"0": 1.1}, "sepal_width_(cm)": {"0": 3.5},
                                     "petal_length_(cm)": {"0": 1.4},
                                     "petal_width_(cm)": {"0": 0.2},
                                     "sepal_length_(cm)": {"0": 5.1}}] * 2,
                         "argmax": 0, "source": "python/lgbserver/lgbserver/test_model.py:43-47"},
        "lgb_v3_input": {"model": "lgb_iris_v3.txt", "input": "iris_input_v3.json",
                         "p0_gt": 0.5, "source": "test/e2e/predictor/test_lightgbm.py:65-67"},
    }
    with open(os.path.join(HERE, "known_answers.json"), "w") as fh:
        json.dump(ka, fh, indent=1)


if __name__ == "__main__":
    known_answers()
    sklearn_goldens()
    synthetic_goldens()
    print("goldens written to", HERE)
