"""sklearn tree ensembles -> canonical :class:`~kfserving_amd.forest.Forest`.

Replaces the estimator the reference unpickles at
python/sklearnserver/sklearnserver/model.py:38 (``joblib.load``) and calls at
:50 (``self._model.predict``).  Supported: DecisionTree{Regressor,Classifier},
RandomForest{Regressor,Classifier}, ExtraTrees{Regressor,Classifier} with one
output, and GradientBoosting{Regressor,Classifier} (forest_from_gradient_boosting).

Predict semantics encoded (installed sklearn 1.7.2,
sklearn/tree/_tree.pyx:979-997 and sklearn/ensemble/_forest.py:723-736,
882-962, 1044-1085): X converted to float32; at a node, NaN goes to
``missing_go_to_left``'s side, otherwise left iff ``(double)x <= threshold``;
regressors sum ``value[leaf]`` in float64 in estimator order and divide by
n_estimators; classifiers do the same with the per-leaf class-fraction
vector and take the first argmax.
"""
from __future__ import annotations

from typing import Tuple

import numpy as np

from ..forest import (Forest, NODE_NAN_LEFT, TI_F32, TI_F64, T_ARGMAX, T_IDENTITY, T_STEP,
                      concat_trees)

TREE_LEAF = -1


def tree_arrays_from_sklearn(tree_) -> dict:
    """Raw arrays of a fitted ``sklearn.tree._tree.Tree``."""
    mgl = getattr(tree_, "missing_go_to_left", None)
    n = int(tree_.node_count)
    return {
        "children_left": np.asarray(tree_.children_left, dtype=np.int64),
        "children_right": np.asarray(tree_.children_right, dtype=np.int64),
        "feature": np.asarray(tree_.feature, dtype=np.int64),
        "threshold": np.asarray(tree_.threshold, dtype=np.float64),
        "missing_go_to_left": (np.asarray(mgl, dtype=np.uint8) if mgl is not None
                               else np.zeros(n, dtype=np.uint8)),
        "value": np.asarray(tree_.value, dtype=np.float64),
        "cover": np.asarray(tree_.weighted_n_node_samples, dtype=np.float64),
    }


def _canon_tree(arr: dict, classifier: bool, n_classes: int) -> dict:
    cl = arr["children_left"]
    cr = arr["children_right"]
    leaf = cl == TREE_LEAF
    n = cl.shape[0]
    value = arr["value"]
    if value.ndim != 3 or value.shape[1] != 1:
        raise ValueError("multi-output sklearn trees are not supported")
    lv = value[:, 0, :n_classes] if classifier else value[:, 0, :1]
    return {
        "feature": np.where(leaf, -1, arr["feature"]),
        "threshold": np.where(leaf, 0.0, arr["threshold"]),
        "flags": np.where(~leaf & (arr["missing_go_to_left"] != 0), NODE_NAN_LEFT, 0),
        "left": np.where(leaf, -1, cl),
        "right": np.where(leaf, -1, cr),
        "leaf_id": np.arange(n),
        "leaf_value": np.where(leaf[:, None], lv, 0.0),
        "cover": arr.get("cover"),
    }


def forest_from_tree_arrays(trees, n_features: int, classifier: bool, n_classes: int = 1,
                            average: bool = True, classes=None, kind: str = "") -> Forest:
    K = n_classes if classifier else 1
    canon = [_canon_tree(a, classifier, K) for a in trees]
    cat = concat_trees(canon, K)
    return Forest(
        n_features=int(n_features), n_groups=K, leaf_width=K, accum_dtype=TI_F64,
        base_first=True, lgb_zero_map=False,
        tree_offset=cat["tree_offset"], tree_group=np.zeros(len(trees), dtype=np.int32),
        feature=cat["feature"], threshold=cat["threshold"], flags=cat["flags"],
        left=cat["left"], right=cat["right"], leaf_id=cat["leaf_id"],
        leaf_value=cat["leaf_value"], base_margin=np.zeros(K), cover=cat["cover"],
        average_divisor=float(len(trees)) if average else 1.0,
        transform=T_ARGMAX if classifier else T_IDENTITY, transform_param=1.0,
        input_dtype=TI_F32, library="sklearn", objective=kind,
        meta={"classes": None if classes is None else np.asarray(classes)},
    ).contiguous()


def _estimators(est) -> Tuple[list, bool]:
    name = type(est).__name__
    if name in ("RandomForestRegressor", "ExtraTreesRegressor"):
        return list(est.estimators_), True
    if name in ("RandomForestClassifier", "ExtraTreesClassifier"):
        return list(est.estimators_), True
    if name in ("DecisionTreeRegressor", "DecisionTreeClassifier", "ExtraTreeRegressor",
                "ExtraTreeClassifier"):
        return [est], False
    raise TypeError(f"sklearn estimator {name} is not a supported tree ensemble "
                    "(RandomForest / ExtraTrees / DecisionTree)")


def forest_from_gradient_boosting(est) -> Forest:
    """GradientBoosting{Regressor,Classifier} (installed sklearn 1.7.2,
    ensemble/_gb.py:948-967 and _gradient_boosting.pyx:56-75, 164-205):

        raw[:, k] = init_raw[k];  for stage i, for k: raw[:, k] += learning_rate * value[leaf]

    in float64 with X converted to float32 and ``x <= threshold`` (NaN input is
    rejected by validate_data).  Each stage's K trees are output groups 0..K-1
    in stage order, and the leaf payload is ``learning_rate * value`` (the same
    double product the Cython loop forms), so the sums are bit-identical.  The
    init estimator must be 'zero' or a Dummy{Regressor,Classifier} (the
    default): its raw prediction is a constant per output, taken from the
    estimator itself.  predict: regressor raw; binary classifier raw >= 0
    (_gb.py:1612-1632, T_STEP); multiclass first argmax."""
    from sklearn.dummy import DummyClassifier, DummyRegressor
    init = est.init_
    if not (isinstance(init, str) and init == "zero") and \
            not isinstance(init, (DummyRegressor, DummyClassifier)):
        raise TypeError("GradientBoosting with a non-constant init estimator "
                        f"({type(init).__name__}) is not supported")
    stages = est.estimators_                       # [n_stages, K] DecisionTreeRegressor
    n_stages, K = stages.shape
    F = int(est.n_features_in_)
    base = np.asarray(est._raw_predict_init(np.zeros((1, F), dtype=np.float32))[0],
                      dtype=np.float64)
    lr = float(est.learning_rate)
    canon, groups = [], []
    for i in range(n_stages):
        for k in range(K):
            arr = tree_arrays_from_sklearn(stages[i, k].tree_)
            t = _canon_tree(arr, False, 1)
            t["flags"] = np.zeros_like(t["flags"])      # the GB traversal ignores missing_go_to_left
            leaf = t["feature"] < 0
            t["leaf_value"] = np.where(leaf[:, None], lr * arr["value"][:, 0, :1], 0.0)
            canon.append(t)
            groups.append(k)
    cat = concat_trees(canon, 1)
    classifier = hasattr(est, "classes_")
    if classifier:
        transform = T_STEP if K == 1 else T_ARGMAX
    else:
        transform = T_IDENTITY
    return Forest(
        n_features=F, n_groups=K, leaf_width=1, accum_dtype=TI_F64,
        base_first=True, lgb_zero_map=False,
        tree_offset=cat["tree_offset"], tree_group=np.asarray(groups, dtype=np.int32),
        feature=cat["feature"], threshold=cat["threshold"], flags=cat["flags"],
        left=cat["left"], right=cat["right"], leaf_id=cat["leaf_id"],
        leaf_value=cat["leaf_value"], base_margin=base, average_divisor=1.0, cover=cat["cover"],
        transform=transform, transform_param=1.0,
        input_dtype=TI_F32, library="sklearn", objective=type(est).__name__,
        meta={"classes": np.asarray(est.classes_) if classifier else None,
              "allow_nan": False},
    ).contiguous()


def forest_from_sklearn(est) -> Forest:
    """Flatten a fitted sklearn tree ensemble."""
    if type(est).__name__ in ("GradientBoostingRegressor", "GradientBoostingClassifier"):
        return forest_from_gradient_boosting(est)
    members, average = _estimators(est)
    if getattr(est, "n_outputs_", 1) != 1:
        raise ValueError("multi-output sklearn models are not supported")
    classifier = hasattr(est, "classes_")
    n_classes = int(est.n_classes_) if classifier else 1
    trees = [tree_arrays_from_sklearn(m.tree_) for m in members]
    return forest_from_tree_arrays(trees, est.n_features_in_, classifier, n_classes,
                                   average=average,
                                   classes=getattr(est, "classes_", None),
                                   kind=type(est).__name__)


def save_tree_arrays(path: str, est) -> None:
    """Store a fitted ensemble's raw tree arrays as .npz (no pickle)."""
    members, average = _estimators(est)
    classifier = hasattr(est, "classes_")
    payload = {
        "n_trees": np.int64(len(members)),
        "n_features": np.int64(est.n_features_in_),
        "classifier": np.int64(classifier),
        "average": np.int64(average),
        "n_classes": np.int64(est.n_classes_ if classifier else 1),
        "kind": np.array(type(est).__name__),
    }
    if classifier:
        payload["classes"] = np.asarray(est.classes_)
    for i, m in enumerate(members):
        for k, v in tree_arrays_from_sklearn(m.tree_).items():
            payload[f"t{i}_{k}"] = v
    np.savez_compressed(path, **payload)


def load_tree_arrays(path: str) -> Forest:
    """Inverse of :func:`save_tree_arrays` (numpy.load, allow_pickle=False)."""
    z = np.load(path, allow_pickle=False)
    T = int(z["n_trees"])
    keys = ("children_left", "children_right", "feature", "threshold", "missing_go_to_left",
            "value", "cover")
    trees = [{k: z[f"t{i}_{k}"] for k in keys if f"t{i}_{k}" in z.files} for i in range(T)]
    classifier = bool(int(z["classifier"]))
    return forest_from_tree_arrays(trees, int(z["n_features"]), classifier,
                                   int(z["n_classes"]), average=bool(int(z["average"])),
                                   classes=z["classes"] if "classes" in z.files else None,
                                   kind=str(z["kind"]))
