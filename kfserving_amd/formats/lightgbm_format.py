"""LightGBM text model (v2/v3) -> canonical :class:`~kfserving_amd.forest.Forest`.

Replaces ``lgb.Booster(params={"nthread": n}, model_file=.../model.bst)`` at
python/lgbserver/lgbserver/model.py:39-40 without importing lightgbm (the
reference pins lightgbm 2.3.1, python/lgbserver/setup.py:37).  Format as in
the fixture python/lgbserver/lgbserver/example_model/model/model.bst:1-12
(header), :12-28 (one ``Tree=`` block), :5412 (``end of trees``).

Predict semantics encoded (upstream lightgbm 2.3.1 ``Tree::NumericalDecision``
and ``GBDT::PredictRaw``): features read as float64; missing type None maps
NaN to 0.0, Zero sends |x| <= 1e-35 to the default child, NaN sends NaN to the
default child; otherwise left iff ``x <= threshold``; scores accumulated in
float64 in tree order, tree t feeding class t mod num_tree_per_iteration.

Categorical splits (``Tree::CategoricalDecision``, decision_type bit 0): the
node's threshold indexes ``cat_boundaries``; the row goes left iff bit
``(int)x`` is set in ``cat_threshold[cat_boundaries[c]:cat_boundaries[c+1]]``;
NaN, negative and out-of-range values go right.  Bitsets are concatenated
over the forest into ``Forest.cat_bits`` with per-node word offsets.
"""
from __future__ import annotations

from typing import Dict, List

import numpy as np

from ..forest import (Forest, MISSING_NAN, MISSING_NONE, MISSING_ZERO, NODE_CATEGORICAL,
                      NODE_NAN_LEFT, NODE_ZERO_FLIP, TI_F64, T_EXP, T_IDENTITY, T_LOG1PEXP,
                      T_SIGMOID, T_SIGNSQUARE, T_SOFTMAX, concat_trees)


class LightGBMFormatError(ValueError):
    pass


def _ints(s: str) -> np.ndarray:
    return np.array([int(v) for v in s.split()], dtype=np.int64) if s.strip() else \
        np.zeros(0, dtype=np.int64)


def _floats(s: str) -> np.ndarray:
    return np.array([float(v) for v in s.split()], dtype=np.float64) if s.strip() else \
        np.zeros(0, dtype=np.float64)


def objective_transform(objective: str):
    """(transform, param) of ObjectiveFunction::ConvertOutput for a model line."""
    parts = objective.split()
    name = parts[0] if parts else ""
    kv = {}
    flags = set()
    for p in parts[1:]:
        if ":" in p:
            k, v = p.split(":", 1)
            kv[k] = v
        else:
            flags.add(p)
    if name == "binary":
        return T_SIGMOID, float(kv.get("sigmoid", 1.0))
    if name in ("multiclass", "softmax"):
        return T_SOFTMAX, 1.0
    if name in ("multiclassova", "multiclass_ova", "ova", "ovr"):
        return T_SIGMOID, float(kv.get("sigmoid", 1.0))
    if name in ("cross_entropy", "xentropy"):
        return T_SIGMOID, 1.0
    if name in ("cross_entropy_lambda", "xentlambda"):
        return T_LOG1PEXP, 1.0
    if name in ("poisson", "gamma", "tweedie"):
        return T_EXP, 1.0
    if name in ("regression", "regression_l2", "l2", "mean_squared_error", "mse") and \
            "sqrt" in flags:
        return T_SIGNSQUARE, 1.0
    return T_IDENTITY, 1.0


def _node_flags(decision_type: np.ndarray, threshold: np.ndarray) -> np.ndarray:
    default_left = (decision_type & 2) != 0
    missing = (decision_type >> 2) & 3
    zero_left = 0.0 <= threshold             # where a NaN->0 / zero input lands
    nan_left = np.where(missing == MISSING_NONE, zero_left, default_left)
    zero_flip = (missing == MISSING_ZERO) & (default_left != zero_left)
    flags = np.where(nan_left, NODE_NAN_LEFT, 0) | np.where(zero_flip, NODE_ZERO_FLIP, 0)
    # categorical nodes: Tree::CategoricalDecision (NaN / negative -> right)
    cat = (decision_type & 1) != 0
    flags = np.where(cat, NODE_CATEGORICAL, flags)
    if np.any((missing != MISSING_NONE) & (missing != MISSING_ZERO) & (missing != MISSING_NAN)):
        raise LightGBMFormatError("unknown missing type")
    return flags.astype(np.uint8)


def _tree(block: Dict[str, str]) -> dict:
    num_leaves = int(block["num_leaves"])
    leaf_value = _floats(block["leaf_value"])
    if leaf_value.shape[0] != num_leaves:
        raise LightGBMFormatError("leaf_value length != num_leaves")
    if block.get("is_linear", "0").strip() not in ("", "0"):
        raise LightGBMFormatError("linear trees are not supported")
    leaf_count = _floats(block["leaf_count"]) if "leaf_count" in block else None
    if num_leaves == 1:
        return {"feature": np.array([-1]), "threshold": np.zeros(1), "flags": np.zeros(1),
                "left": np.array([-1]), "right": np.array([-1]), "leaf_id": np.array([0]),
                "leaf_value": leaf_value.reshape(1, 1),
                "cover": None if leaf_count is None else leaf_count[:1]}
    n_int = num_leaves - 1
    feat = _ints(block["split_feature"])
    thr = _floats(block["threshold"])
    dt = _ints(block["decision_type"])
    lc = _ints(block["left_child"])
    rc = _ints(block["right_child"])
    for name, arr in (("split_feature", feat), ("threshold", thr), ("decision_type", dt),
                      ("left_child", lc), ("right_child", rc)):
        if arr.shape[0] != n_int:
            raise LightGBMFormatError(f"{name} length != num_leaves - 1")
    n = n_int + num_leaves
    # canonical numbering: internal nodes 0..n_int-1, leaf j at n_int + j
    left = np.where(lc >= 0, lc, n_int + ~lc)
    right = np.where(rc >= 0, rc, n_int + ~rc)
    cat_off = np.full(n, -1, dtype=np.int64)
    cat_nw = np.zeros(n, dtype=np.int32)
    cat_words = np.zeros(0, dtype=np.uint32)
    if int(block.get("num_cat", "0")) > 0:
        bounds = _ints(block["cat_boundaries"])
        cat_words = np.array([int(v) for v in block["cat_threshold"].split()], dtype=np.uint32)
        is_cat = (dt & 1) != 0
        ci = thr[is_cat].astype(np.int64)
        if ci.size and (ci.min() < 0 or ci.max() + 1 >= bounds.shape[0]):
            raise LightGBMFormatError("categorical threshold index out of range")
        cat_off[:n_int][is_cat] = bounds[ci]
        cat_nw[:n_int][is_cat] = bounds[ci + 1] - bounds[ci]
    return {
        "feature": np.concatenate([feat, np.full(num_leaves, -1)]),
        "threshold": np.concatenate([thr, np.zeros(num_leaves)]),
        "flags": np.concatenate([_node_flags(dt, thr), np.zeros(num_leaves, dtype=np.uint8)]),
        "left": np.concatenate([left, np.full(num_leaves, -1)]),
        "right": np.concatenate([right, np.full(num_leaves, -1)]),
        "leaf_id": np.concatenate([np.full(n_int, -1), np.arange(num_leaves)]),
        "leaf_value": np.concatenate([np.zeros(n_int), leaf_value]).reshape(n, 1),
        "cat_offset": cat_off, "cat_nwords": cat_nw, "cat_words": cat_words,
        # data counts (LightGBM's own SHAP weights children by them)
        "cover": (np.concatenate([_floats(block["internal_count"]), leaf_count])
                  if leaf_count is not None and "internal_count" in block else None),
    }


def parse_lightgbm_text(text: str) -> Forest:
    lines = text.splitlines()
    header: Dict[str, str] = {}
    flags_present = set()
    i = 0
    while i < len(lines) and not lines[i].startswith("Tree="):
        line = lines[i].strip()
        if "=" in line:
            k, v = line.split("=", 1)
            header[k.strip()] = v.strip()
        elif line:
            flags_present.add(line)
        i += 1
    if "version" not in header and "tree" not in flags_present:
        raise LightGBMFormatError("not a LightGBM text model")
    blocks: List[Dict[str, str]] = []
    cur = None
    for line in lines[i:]:
        s = line.strip()
        if s.startswith("Tree="):
            cur = {}
            blocks.append(cur)
        elif s == "end of trees":
            break
        elif cur is not None and "=" in s:
            k, v = s.split("=", 1)
            cur[k] = v
    if not blocks:
        raise LightGBMFormatError("model has no trees")
    trees = [_tree(b) for b in blocks]
    cat = concat_trees(trees, 1)
    # concatenate per-tree bitsets; node offsets become global word offsets
    cat_bits, cat_offset, cat_nwords = None, None, None
    if any(t.get("cat_words") is not None and t["cat_words"].size for t in trees):
        base, words, offs, nws = 0, [], [], []
        for t in trees:
            o = t["cat_offset"].copy()
            o[o >= 0] += base
            offs.append(o)
            nws.append(t["cat_nwords"])
            words.append(t["cat_words"])
            base += t["cat_words"].size
        cat_bits = np.concatenate(words).astype(np.uint32)
        cat_offset = np.concatenate(offs)
        cat_nwords = np.concatenate(nws).astype(np.int32)
    ntpi = int(header.get("num_tree_per_iteration", header.get("num_class", "1")))
    K = max(1, ntpi)
    n_features = int(header.get("max_feature_idx", "-1")) + 1
    used = cat["feature"][cat["feature"] >= 0]
    if used.size:
        n_features = max(n_features, int(used.max()) + 1)
    objective = header.get("objective", "")
    transform, tparam = objective_transform(objective)
    average = "average_output" in flags_present or header.get("average_output") is not None
    n_iter = len(trees) // K
    names = header.get("feature_names", "").split() or None
    return Forest(
        n_features=max(n_features, 1), n_groups=K, leaf_width=1, accum_dtype=TI_F64,
        base_first=True, lgb_zero_map=True,
        tree_offset=cat["tree_offset"],
        tree_group=(np.arange(len(trees)) % K).astype(np.int32),
        feature=cat["feature"], threshold=cat["threshold"], flags=cat["flags"],
        left=cat["left"], right=cat["right"], leaf_id=cat["leaf_id"],
        leaf_value=cat["leaf_value"], base_margin=np.zeros(K), cover=cat["cover"],
        average_divisor=float(n_iter) if average and n_iter > 0 else 1.0,
        transform=transform, transform_param=tparam, input_dtype=TI_F64,
        library="lightgbm", objective=objective, feature_names=names,
        meta={"version": header.get("version", ""), "num_class": int(header.get("num_class", 1))},
        cat_bits=cat_bits, cat_offset=cat_offset, cat_nwords=cat_nwords,
    ).contiguous()


def load_lightgbm_model(path: str) -> Forest:
    with open(path, "r") as fh:
        return parse_lightgbm_text(fh.read())


# ------------------------------------------------------------------ writer
def _fmt(v: float) -> str:
    return repr(float(v))


def write_lightgbm_text(path: str, trees: List[dict], n_features: int, objective: str,
                        num_class: int = 1, feature_names=None) -> None:
    """Write a LightGBM v3 text model (subset the loader reads).

    ``trees`` hold LightGBM Tree arrays: ``split_feature, threshold,
    decision_type, left_child, right_child`` (negative = ~leaf) and
    ``leaf_value``.  Used for the synthetic leaf-wise benchmark models.
    """
    names = feature_names or [f"Column_{j}" for j in range(n_features)]
    out = ["tree", "version=v3", f"num_class={num_class}",
           f"num_tree_per_iteration={num_class if num_class > 1 else 1}",
           "label_index=0", f"max_feature_idx={n_features - 1}", f"objective={objective}",
           "feature_names=" + " ".join(names), "feature_infos=" + " ".join(["none"] * n_features),
           "tree_sizes=" + " ".join(["0"] * len(trees)), ""]
    for i, t in enumerate(trees):
        nl = len(t["leaf_value"])
        out.append(f"Tree={i}")
        out.append(f"num_leaves={nl}")
        cb = t.get("cat_boundaries")
        out.append(f"num_cat={0 if cb is None else len(cb) - 1}")
        if nl > 1:
            out.append("split_feature=" + " ".join(str(int(v)) for v in t["split_feature"]))
            out.append("split_gain=" + " ".join("1" for _ in t["split_feature"]))
            out.append("threshold=" + " ".join(_fmt(v) for v in t["threshold"]))
            out.append("decision_type=" + " ".join(str(int(v)) for v in t["decision_type"]))
            out.append("left_child=" + " ".join(str(int(v)) for v in t["left_child"]))
            out.append("right_child=" + " ".join(str(int(v)) for v in t["right_child"]))
        if cb is not None and len(cb) > 1:
            out.append("cat_boundaries=" + " ".join(str(int(v)) for v in cb))
            out.append("cat_threshold=" + " ".join(str(int(v)) for v in t["cat_threshold"]))
        out.append("leaf_value=" + " ".join(_fmt(v) for v in t["leaf_value"]))
        if "leaf_count" in t:
            out.append("leaf_count=" + " ".join(str(int(v)) for v in t["leaf_count"]))
            if nl > 1:
                out.append("internal_count=" + " ".join(str(int(v)) for v in t["internal_count"]))
        out.append("shrinkage=1")
        out.append("")
        out.append("")
    out.append("end of trees")
    out.append("")
    with open(path, "w") as fh:
        fh.write("\n".join(out))


def add_categorical_splits(trees: List[dict], cat_features, n_categories: int, seed: int,
                           frac: float = 0.5) -> List[dict]:
    """Turn a fraction of the splits on ``cat_features`` into categorical
    splits (decision_type bit 0, threshold = index into cat_boundaries) with
    random bitsets over ``n_categories`` values -- the shape lightgbm 2.3.1
    writes (Tree::SplitCategorical): each bitset is just long enough for its
    highest category."""
    rng = np.random.default_rng(seed)
    cat_features = np.asarray(cat_features)
    for t in trees:
        if len(t["leaf_value"]) <= 1:
            continue
        feat = np.asarray(t["split_feature"]).copy()
        thr = np.asarray(t["threshold"], dtype=np.float64).copy()
        dt = np.asarray(t["decision_type"]).copy()
        bounds, words = [0], []
        for i in range(feat.shape[0]):
            if rng.random() >= frac:
                continue
            feat[i] = cat_features[rng.integers(0, cat_features.shape[0])]
            members = np.nonzero(rng.random(n_categories) < 0.4)[0]
            if members.size == 0:
                members = np.array([int(rng.integers(0, n_categories))])
            nw = int(members.max()) // 32 + 1
            bits = np.zeros(nw, dtype=np.uint64)
            for m in members:
                bits[m // 32] |= np.uint64(1) << np.uint64(m % 32)
            thr[i] = len(bounds) - 1
            dt[i] = 1 | (int(dt[i]) & 2) | (int(rng.integers(0, 3)) << 2)
            words.extend(int(w) for w in bits)
            bounds.append(bounds[-1] + nw)
        if len(bounds) > 1:
            t.update(split_feature=feat, threshold=thr, decision_type=dt,
                     cat_boundaries=np.asarray(bounds), cat_threshold=np.asarray(words))
    return trees


def synthetic_leafwise_trees(n_trees: int, num_leaves: int, n_features: int, seed: int,
                             missing_types=(MISSING_NONE, MISSING_ZERO, MISSING_NAN)) -> List[dict]:
    """Seeded leaf-wise trees: grow by splitting a
    random current leaf until ``num_leaves``; thresholds ~ N(0,1) as float64,
    decision_type draws default_left and a missing type; leaf / internal
    counts are those of a seeded N(0,1) sample (plus one per leaf)."""
    rng = np.random.default_rng(seed)
    crng = np.random.default_rng([seed, 7919])
    trees = []
    mts = np.asarray(missing_types)
    for _ in range(n_trees):
        n_int = num_leaves - 1
        feat = rng.integers(0, n_features, size=n_int)
        thr = rng.standard_normal(n_int)
        dl = rng.integers(0, 2, size=n_int)
        mt = mts[rng.integers(0, len(mts), size=n_int)]
        dtype_ = (dl << 1) | (mt << 2)
        left = np.zeros(n_int, dtype=np.int64)
        right = np.zeros(n_int, dtype=np.int64)
        # leaves as (parent, side); start: root split with two leaves 0, 1
        leaf_owner = [(0, 0), (0, 1)]
        left[0], right[0] = ~0, ~1
        for node in range(1, n_int):
            j = int(rng.integers(0, len(leaf_owner)))   # split leaf j
            parent, side = leaf_owner[j]
            if side == 0:
                left[parent] = node
            else:
                right[parent] = node
            new_leaf = len(leaf_owner)
            leaf_owner[j] = (node, 0)
            leaf_owner.append((node, 1))
            left[node] = ~j
            right[node] = ~new_leaf
        # counts as training would leave them: the rows of a seeded N(0,1)
        # sample that reach each leaf (+ 1: leaf-wise growth never leaves one
        # empty), from the counts' own stream (the trees are unchanged)
        Xs = crng.standard_normal((2000, n_features))
        node = np.zeros(Xs.shape[0], dtype=np.int64)
        rows = np.arange(Xs.shape[0])
        while (node >= 0).any():
            live = node >= 0
            nd = node[live]
            go_left = Xs[rows[live], feat[nd]] <= thr[nd]
            node[live] = np.where(go_left, left[nd], right[nd])
        leaf_count = np.bincount(~node, minlength=num_leaves).astype(np.int64) + 1
        internal_count = np.zeros(n_int, dtype=np.int64)

        def count(c):
            if c < 0:
                return int(leaf_count[~c])
            internal_count[c] = count(int(left[c])) + count(int(right[c]))
            return int(internal_count[c])
        count(0)
        trees.append({"split_feature": feat, "threshold": thr, "decision_type": dtype_,
                      "left_child": left, "right_child": right,
                      "leaf_value": rng.uniform(-0.05, 0.05, size=num_leaves),
                      "leaf_count": leaf_count, "internal_count": internal_count})
    return trees


def synthetic_maxbin_trees(n_trees: int, num_leaves: int, n_features: int, seed: int,
                           max_bin: int = 255,
                           missing_types=(MISSING_NONE,)) -> List[dict]:
    """Seeded leaf-wise trees shaped like a LightGBM model trained at
    ``max_bin`` on N(0,1) features (the C3 variant ``c3_maxbin``; VERDICT r2
    asked for it beside the i.i.d.-threshold generator above):

    * thresholds are bin upper bounds: the ``max_bin - 1`` N(0,1) quantiles
      ``Phi^-1(k / max_bin)``, k = 1 .. max_bin - 1, as LightGBM's histogram
      binning of such a feature gives (so at most max_bin - 1 = 254 distinct
      thresholds per feature, as in a trained model);
    * every split is drawn inside the interval its feature still spans at the
      leaf being split, so intervals nest along a path and neither child is
      empty (LightGBM never splits off an empty side);
    * the leaf to split is drawn with probability proportional to its N(0,1)
      mass (the rows it holds: a split's gain grows with them), which makes
      the paths the data takes deeper than uniform leaf choice does;
    * missing type None (a feature without NaN in training; NaN reads as 0.0)
      unless ``missing_types`` says otherwise; default_left ~ Bernoulli(1/2).
    """
    from math import erf, sqrt
    from statistics import NormalDist
    nd = NormalDist()
    edges = np.array([nd.inv_cdf(k / max_bin) for k in range(1, max_bin)])   # max_bin - 1 bounds
    cdf = np.concatenate([[0.0], np.array([0.5 * (1 + erf(e / sqrt(2))) for e in edges]), [1.0]])
    rng = np.random.default_rng([seed, 255])
    crng = np.random.default_rng([seed, 7919])
    mts = np.asarray(missing_types)
    trees = []
    B = max_bin
    for _ in range(n_trees):
        n_int = num_leaves - 1
        feat = np.zeros(n_int, dtype=np.int64)
        thr = np.zeros(n_int)
        left = np.zeros(n_int, dtype=np.int64)
        right = np.zeros(n_int, dtype=np.int64)
        # a leaf: (parent, side, lo[F], hi[F]) -- the bins [lo, hi) the leaf spans
        leaves = [(-1, 0, np.zeros(n_features, dtype=np.int64), np.full(n_features, B, np.int64))]
        mass = [1.0]
        for node in range(n_int):
            m = np.asarray(mass)
            j = int(rng.choice(len(leaves), p=m / m.sum()))
            parent, side, lo, hi = leaves[j]
            splittable = np.nonzero(hi - lo >= 2)[0]
            f = int(splittable[rng.integers(0, len(splittable))])
            b = int(rng.integers(lo[f], hi[f] - 1))          # left: [lo, b], right: [b + 1, hi)
            feat[node], thr[node] = f, edges[b]
            if parent >= 0:
                if side == 0:
                    left[parent] = node
                else:
                    right[parent] = node
            lhi, rlo = hi.copy(), lo.copy()
            lhi[f], rlo[f] = b + 1, b + 1
            frac_l = (cdf[b + 1] - cdf[lo[f]]) / max(cdf[hi[f]] - cdf[lo[f]], 1e-300)
            leaves[j] = (node, 0, lo, lhi)
            leaves.append((node, 1, rlo, hi))
            mass.append(mass[j] * (1.0 - frac_l))
            mass[j] *= frac_l
        for k, (parent, side, _, _) in enumerate(leaves):   # leaf k = ~k
            if side == 0:
                left[parent] = ~k
            else:
                right[parent] = ~k
        dl = rng.integers(0, 2, size=n_int)
        mt = mts[rng.integers(0, len(mts), size=n_int)]
        leaf_count = np.maximum(1, np.round(np.asarray(mass) * 1e6)).astype(np.int64)
        internal_count = np.zeros(n_int, dtype=np.int64)

        def count(c):
            if c < 0:
                return int(leaf_count[~c])
            internal_count[c] = count(int(left[c])) + count(int(right[c]))
            return int(internal_count[c])
        count(0)
        trees.append({"split_feature": feat, "threshold": thr,
                      "decision_type": (dl << 1) | (mt << 2),
                      "left_child": left, "right_child": right,
                      "leaf_value": crng.uniform(-0.05, 0.05, size=num_leaves),
                      "leaf_count": leaf_count, "internal_count": internal_count})
    return trees
