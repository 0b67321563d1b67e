"""XGBoost model files -> canonical :class:`~kfserving_amd.forest.Forest`.

Replaces ``xgb.Booster(params={"nthread": n}, model_file=.../model.bst)`` at
python/xgbserver/xgbserver/model.py:38-39 without importing xgboost.  Reads:

* the legacy binary written by xgboost <= 0.90 (the reference pins 0.82,
  python/xgbserver/setup.py:37; fixture python/xgbserver/xgbserver/
  example_model/model/model.bst),
* the 1.x binary with the ``binf`` magic (fixture docs/samples/v1beta1/
  xgboost/model.bst), and
* the JSON model (xgboost >= 1.0 ``save_model("*.json")``) and its UBJSON
  form (xgboost >= 1.6 default ``.ubj``).

Predict semantics encoded (upstream xgboost 0.82 ``RegTree::GetNext`` /
``CPUPredictor::PredValue``): go left iff ``x < split`` in float32, a missing
value takes the node's default child, leaves summed in float32 in tree order
per output group from 0 and then added to the base margin.
"""
from __future__ import annotations

import base64
import json
import struct
from typing import List, Optional, Tuple

import numpy as np

from ..forest import (Forest, NODE_NAN_LEFT, TI_F32, T_ARGMAX, T_EXP, T_HINGE, T_IDENTITY,
                      T_SIGMOID, T_SOFTMAX, concat_trees)

# on-disk structs of the legacy / binf binary (little endian)
_LEARNER_PARAM = 136       # LearnerModelParam
_GBTREE_PARAM = 160        # GBTreeModelParam
_TREE_PARAM = 148          # TreeParam
_NODE_DTYPE = np.dtype([("parent", "<i4"), ("cleft", "<i4"), ("cright", "<i4"),
                        ("sindex", "<u4"), ("info", "<f4")])        # 20 B
_STAT_BYTES = 16           # RTreeNodeStat
_DELETED = 0xFFFFFFFF

_SIGMOID_OBJ = ("binary:logistic", "reg:logistic")
_LOGIT_BASE_OBJ = ("binary:logistic", "reg:logistic", "binary:logitraw")
_EXP_OBJ = ("count:poisson", "reg:gamma", "reg:tweedie", "survival:cox", "survival:aft")


class XGBoostFormatError(ValueError):
    pass


class _Reader:
    def __init__(self, buf: bytes, pos: int = 0):
        self.buf = buf
        self.pos = pos

    def take(self, n: int) -> bytes:
        if self.pos + n > len(self.buf):
            raise XGBoostFormatError(f"truncated model: need {n} bytes at offset {self.pos}")
        b = self.buf[self.pos:self.pos + n]
        self.pos += n
        return b

    def unpack(self, fmt: str):
        return struct.unpack(fmt, self.take(struct.calcsize(fmt)))

    def string(self) -> str:
        (n,) = self.unpack("<Q")
        if n > len(self.buf):
            raise XGBoostFormatError("implausible string length")
        return self.take(n).decode("utf-8", "replace")


def objective_transform(objective: str) -> int:
    if objective in _SIGMOID_OBJ:
        return T_SIGMOID
    if objective == "multi:softmax":
        return T_ARGMAX
    if objective == "multi:softprob":
        return T_SOFTMAX
    if objective == "binary:hinge":
        return T_HINGE
    if objective in _EXP_OBJ:
        return T_EXP
    return T_IDENTITY


def prob_to_margin(objective: str, base_score: float) -> float:
    """ObjFunction::ProbToMargin in float32 (applied to xgboost >= 1.0 models)."""
    b = np.float32(base_score)
    with np.errstate(divide="ignore", invalid="ignore"):
        if objective in _LOGIT_BASE_OBJ:
            return float(-np.log(np.float32(1.0) / b - np.float32(1.0)))
        if objective in ("count:poisson", "reg:gamma", "reg:tweedie"):
            return float(np.log(b))
    return float(b)


def xgb_threshold(split: np.ndarray) -> np.ndarray:
    """x < t (float32)  <=>  x <= nextafterf(t, -inf); t = -inf never goes left."""
    s = np.asarray(split, dtype=np.float32)
    t = np.nextafter(s, np.float32(-np.inf)).astype(np.float64)
    t[np.isneginf(s)] = np.nan
    t[np.isnan(s)] = np.nan
    return t


_STAT_DTYPE = np.dtype([("loss_chg", "<f4"), ("sum_hess", "<f4"), ("base_weight", "<f4"),
                        ("leaf_child_cnt", "<i4")])


def _tree_from_arrays(cleft, cright, sindex, value, deleted=None, sum_hess=None) -> dict:
    cleft = np.asarray(cleft, dtype=np.int32)
    cright = np.asarray(cright, dtype=np.int32)
    sindex = np.asarray(sindex, dtype=np.uint32)
    value = np.asarray(value, dtype=np.float32)
    n = cleft.shape[0]
    leaf = cleft == -1
    if deleted is not None:
        leaf = leaf | deleted
    feature = np.where(leaf, -1, (sindex & 0x7FFFFFFF).astype(np.int64)).astype(np.int32)
    default_left = (sindex >> 31) != 0
    threshold = np.where(leaf, 0.0, xgb_threshold(value))
    flags = np.where(~leaf & default_left, NODE_NAN_LEFT, 0).astype(np.uint8)
    return {
        "feature": feature,
        "threshold": threshold,
        "flags": flags,
        "left": np.where(leaf, -1, cleft).astype(np.int32),
        "right": np.where(leaf, -1, cright).astype(np.int32),
        "leaf_id": np.arange(n, dtype=np.int32),
        "leaf_value": np.where(leaf, value, np.float32(0)).astype(np.float64).reshape(n, 1),
        # RTreeNodeStat::sum_hess, the cover TreeSHAP weights children by
        "cover": None if sum_hess is None else np.asarray(sum_hess, dtype=np.float32)
        .astype(np.float64),
    }


def _assemble(trees: List[dict], tree_info: np.ndarray, num_feature: int, num_group: int,
              base_score: float, objective: str, base_is_margin: bool, base_first: bool,
              version: Tuple[int, int, int], feature_names=None, fmt: str = "") -> Forest:
    cat = concat_trees(trees, 1)
    used = cat["feature"][cat["feature"] >= 0]
    n_features = max(int(num_feature), int(used.max()) + 1 if used.size else 1)
    K = max(1, int(num_group))
    margin = base_score if base_is_margin else prob_to_margin(objective, base_score)
    base = np.full(K, float(np.float32(margin)), dtype=np.float64)
    tinfo = np.asarray(tree_info, dtype=np.int32)
    if tinfo.shape[0] != len(trees):
        raise XGBoostFormatError("tree_info length does not match the number of trees")
    return Forest(
        n_features=n_features, n_groups=K, leaf_width=1, accum_dtype=TI_F32,
        base_first=base_first, lgb_zero_map=False,
        tree_offset=cat["tree_offset"], tree_group=tinfo,
        feature=cat["feature"], threshold=cat["threshold"], flags=cat["flags"],
        left=cat["left"], right=cat["right"], leaf_id=cat["leaf_id"],
        leaf_value=cat["leaf_value"], base_margin=base, cover=cat["cover"],
        transform=objective_transform(objective), transform_param=1.0,
        input_dtype=TI_F32, library="xgboost", objective=objective,
        feature_names=feature_names,
        meta={"format": fmt, "version": version, "base_score": base_score},
    ).contiguous()


def _parse_binary(buf: bytes, pos: int, fmt: str) -> Forest:
    r = _Reader(buf, pos)
    lp = r.take(_LEARNER_PARAM)
    base_score, num_feature, num_class, extra_attrs, eval_metrics, major, minor = \
        struct.unpack_from("<fIiiiii", lp, 0)
    objective = r.string()
    gbm = r.string()
    if gbm not in ("gbtree", "dart"):
        raise XGBoostFormatError(f"booster '{gbm}' is not a tree ensemble")
    gp = r.take(_GBTREE_PARAM)
    num_trees, num_roots, g_num_feature, _pad, _pbuf, num_output_group, size_leaf_vector = \
        struct.unpack_from("<iiiiqii", gp, 0)
    if size_leaf_vector != 0:
        raise XGBoostFormatError("size_leaf_vector != 0 is not supported")
    trees = []
    for _ in range(num_trees):
        tp = r.take(_TREE_PARAM)
        t_roots, num_nodes, num_deleted, _max_depth, _nf, t_slv = struct.unpack_from("<6i", tp, 0)
        if num_nodes <= 0:
            raise XGBoostFormatError("tree with no nodes")
        nodes = np.frombuffer(r.take(_NODE_DTYPE.itemsize * num_nodes), dtype=_NODE_DTYPE)
        stats = np.frombuffer(r.take(_STAT_BYTES * num_nodes), dtype=_STAT_DTYPE)
        if t_slv != 0:
            (nlv,) = r.unpack("<Q")
            r.take(4 * nlv)
        deleted = nodes["sindex"] == _DELETED
        trees.append(_tree_from_arrays(nodes["cleft"], nodes["cright"], nodes["sindex"],
                                       nodes["info"], deleted, stats["sum_hess"]))
    tree_info = np.frombuffer(r.take(4 * num_trees), dtype="<i4") if num_trees else np.zeros(0)
    if gbm == "dart":
        (nw,) = r.unpack("<Q")
        weights = np.frombuffer(r.take(4 * nw), dtype="<f4")
        for t, w in zip(trees, weights):     # Dart::Pred: weight_drop[i] * leaf (float32)
            lv = t["leaf_value"][:, 0].astype(np.float32) * np.float32(w)
            t["leaf_value"] = lv.astype(np.float64).reshape(-1, 1)
    attrs = {}
    if extra_attrs != 0 and r.pos < len(buf):
        (na,) = r.unpack("<Q")
        for _ in range(na):
            k = r.string()
            attrs[k] = r.string()
    version = (major, minor, 0)
    # xgboost < 1.0 stores base_score already in margin space; >= 1.0 stores the
    # user value and applies ProbToMargin at load (LearnerIO::LoadModel).
    base_is_margin = major < 1
    # xgboost >= 1.0 deprecates num_output_group in favour of the learner's num_class
    num_group = max(1, num_output_group, num_class)
    f = _assemble(trees, tree_info, num_feature, num_group, base_score, objective,
                  base_is_margin=base_is_margin, base_first=False, version=version, fmt=fmt)
    f.meta["attributes"] = attrs
    f.meta["trailing_bytes"] = len(buf) - r.pos
    return f


def _json_num(v) -> float:
    if isinstance(v, list):
        v = v[0]
    return float(v)


def _parse_json(doc: dict) -> Forest:
    learner = doc["learner"]
    lmp = learner["learner_model_param"]
    base_score = _json_num(lmp.get("base_score", 0.5))
    num_class = int(_json_num(lmp.get("num_class", 0)))
    num_feature = int(_json_num(lmp.get("num_feature", 0)))
    objective = learner["objective"]["name"]
    gb = learner["gradient_booster"]
    name = gb["name"]
    weights = None
    if name == "gbtree":
        model = gb["model"]
    elif name == "dart":
        model = gb["gbtree"]["model"]
        weights = np.asarray(gb["weight_drop"], dtype=np.float32)
    else:
        raise XGBoostFormatError(f"booster '{name}' is not a tree ensemble")
    trees = []
    for i, jt in enumerate(model["trees"]):
        if any(int(s) != 0 for s in jt.get("split_type", [])):
            raise XGBoostFormatError("categorical splits are not supported yet")
        cleft = np.asarray(jt["left_children"], dtype=np.int32)
        dl = np.asarray(jt["default_left"], dtype=np.uint32) & 1
        sindex = np.asarray(jt["split_indices"], dtype=np.uint32) | (dl << 31)
        t = _tree_from_arrays(cleft, jt["right_children"], sindex, jt["split_conditions"],
                              sum_hess=jt.get("sum_hessian"))
        if weights is not None:
            lv = t["leaf_value"][:, 0].astype(np.float32) * weights[i]
            t["leaf_value"] = lv.astype(np.float64).reshape(-1, 1)
        trees.append(t)
    version = tuple(int(v) for v in doc.get("version", [1, 0, 0]))
    K = max(1, num_class)
    names = learner.get("feature_names") or None
    return _assemble(trees, model["tree_info"], num_feature, K, base_score, objective,
                     base_is_margin=False, base_first=version >= (1, 4, 0), version=version,
                     feature_names=names, fmt="json")


def parse_xgboost_bytes(buf: bytes) -> Forest:
    if buf[:4] == b"binf":
        return _parse_binary(buf, 4, "binf")
    if buf[:4] == b"bs64":
        return _parse_binary(base64.b64decode(buf[4:]), 0, "legacy-b64")
    head = buf.lstrip()[:1]
    if head == b"{":
        # JSON text continues with whitespace or a quoted key; UBJSON with a
        # length marker ('U', 'i', 'l', ...) or a container header ('$', '#')
        if buf[1:2] in (b'"', b" ", b"\n", b"\r", b"\t", b"}"):
            try:
                doc = json.loads(buf.decode("utf-8"))
            except (UnicodeDecodeError, json.JSONDecodeError) as e:
                raise XGBoostFormatError(f"malformed JSON model: {e}") from e
            return _parse_json(doc)
        from . import ubjson
        try:
            doc = ubjson.loads(buf)
        except (ubjson.UBJSONError, KeyError, UnicodeDecodeError) as e:
            raise XGBoostFormatError(f"malformed UBJSON model: {e}") from e
        f = _parse_json(doc)
        f.meta["format"] = "ubj"
        return f
    return _parse_binary(buf, 0, "legacy")


def load_xgboost_model(path: str) -> Forest:
    with open(path, "rb") as fh:
        return parse_xgboost_bytes(fh.read())


# ------------------------------------------------------------------ writers
def write_legacy_binary(path: str, trees: List[dict], tree_info, num_feature: int,
                        num_class: int, base_score: float, objective: str) -> None:
    """Write an xgboost-0.82 legacy binary model.

    ``trees`` hold XGBoost RegTree arrays: ``cleft, cright, sindex`` (bit 31 =
    default_left) and ``value`` (split condition or leaf value).  Used for the
    synthetic benchmark models; the layout is the one
    the loader above reads and that fixture #1 follows.
    """
    out = bytearray()
    lp = bytearray(_LEARNER_PARAM)
    struct.pack_into("<fIiii", lp, 0, base_score, num_feature, num_class, 0, 0)
    out += lp
    for s in (objective, "gbtree"):
        b = s.encode()
        out += struct.pack("<Q", len(b)) + b
    num_group = max(1, num_class)
    gp = bytearray(_GBTREE_PARAM)
    struct.pack_into("<iiiiqii", gp, 0, len(trees), 1, num_feature, 0, 0, num_group, 0)
    out += gp
    for t in trees:
        n = len(t["cleft"])
        tp = bytearray(_TREE_PARAM)
        struct.pack_into("<6i", tp, 0, 1, n, 0, 0, num_feature, 0)
        out += tp
        nodes = np.zeros(n, dtype=_NODE_DTYPE)
        nodes["cleft"] = t["cleft"]
        nodes["cright"] = t["cright"]
        nodes["sindex"] = t["sindex"]
        nodes["info"] = t["value"]
        parent = np.full(n, -1, dtype=np.int64)
        for i in range(n):
            if t["cleft"][i] != -1:
                parent[t["cleft"][i]] = i | (1 << 31)
                parent[t["cright"][i]] = i
        nodes["parent"] = parent.astype(np.uint32).view(np.int32)
        out += nodes.tobytes()
        stats = np.zeros(n, dtype=_STAT_DTYPE)
        if "sum_hess" in t:
            stats["sum_hess"] = t["sum_hess"]
        out += stats.tobytes()
    out += np.asarray(tree_info, dtype="<i4").tobytes()
    with open(path, "wb") as fh:
        fh.write(bytes(out))


def json_model_doc(trees: List[dict], tree_info, num_feature: int, num_class: int,
                   base_score: float, objective: str, version=(1, 3, 0), arrays=False) -> dict:
    """The xgboost >= 1.0 JSON model document (subset the loader reads);
    ``arrays=True`` keeps numpy arrays (for the UBJSON writer)."""
    jt = []
    for i, t in enumerate(trees):
        n = len(t["cleft"])
        conv = (lambda a, dt: np.asarray(a, dtype=dt)) if arrays else \
            (lambda a, dt: [dt(v).item() for v in np.asarray(a, dtype=dt)])
        jt.append({
            "id": i,
            "left_children": conv(t["cleft"], np.int32),
            "right_children": conv(t["cright"], np.int32),
            "split_indices": conv(np.asarray(t["sindex"]) & 0x7FFFFFFF, np.int32),
            "default_left": conv(np.asarray(t["sindex"]) >> 31, np.uint8),
            "split_conditions": conv(t["value"], np.float32),
            "sum_hessian": conv(t.get("sum_hess", np.zeros(n)), np.float32),
            "tree_param": {"num_nodes": str(n), "num_feature": str(num_feature),
                           "size_leaf_vector": "0"},
        })
    return {
        "version": list(version),
        "learner": {
            "attributes": {},
            "feature_names": [],
            "learner_model_param": {"base_score": repr(float(base_score)),
                                    "num_class": str(num_class),
                                    "num_feature": str(num_feature)},
            "objective": {"name": objective},
            "gradient_booster": {"name": "gbtree", "model": {
                "gbtree_model_param": {"num_trees": str(len(trees)), "size_leaf_vector": "0"},
                "tree_info": np.asarray(tree_info, dtype=np.int32) if arrays
                else [int(v) for v in tree_info],
                "trees": jt}},
        },
    }


def write_ubj_model(path: str, trees: List[dict], tree_info, num_feature: int, num_class: int,
                    base_score: float, objective: str, version=(1, 6, 0)) -> None:
    """Write the model as xgboost >= 1.6 UBJSON."""
    from . import ubjson
    doc = json_model_doc(trees, tree_info, num_feature, num_class, base_score, objective,
                         version, arrays=True)
    with open(path, "wb") as fh:
        fh.write(ubjson.dumps(doc))


def write_json_model(path: str, trees: List[dict], tree_info, num_feature: int, num_class: int,
                     base_score: float, objective: str, version=(1, 3, 0)) -> None:
    """Write the same model as xgboost >= 1.0 JSON (subset the loader reads)."""
    doc = json_model_doc(trees, tree_info, num_feature, num_class, base_score, objective, version)
    with open(path, "w") as fh:
        json.dump(doc, fh)


def synthetic_complete_trees(n_trees: int, depth: int, n_features: int, seed: int,
                             num_class: int = 0, max_bin: int = 0) -> Tuple[List[dict], np.ndarray]:
    """Seeded complete depth-``depth`` XGBoost trees.

    feature ~ U{0..F-1}, threshold ~ N(0,1) rounded to float32, default_left ~
    Bernoulli(1/2), leaf ~ U(-0.05, 0.05) float32; nodes numbered in heap order;
    sum_hess (the covers) from a seeded N(0,1) sample.  ``max_bin`` > 0 snaps
    every threshold to the nearest of the max_bin - 1 N(0,1) quantile edges
    Phi^-1(k / max_bin), as xgboost's hist / approx tree methods place splits
    on histogram bin bounds (at most max_bin - 1 distinct thresholds a
    feature: u8 bins in the engine); the draws are the same either way.
    """
    edges = None
    if max_bin > 0:
        from statistics import NormalDist
        nd = NormalDist()
        edges = np.array([nd.inv_cdf(k / max_bin) for k in range(1, max_bin)], dtype=np.float32)
    rng = np.random.default_rng(seed)
    crng = np.random.default_rng([seed, 7919])   # covers: own stream, trees unchanged
    n_int = (1 << depth) - 1
    n = 2 * n_int + 1
    trees = []
    for _ in range(n_trees):
        cleft = np.full(n, -1, dtype=np.int32)
        cright = np.full(n, -1, dtype=np.int32)
        idx = np.arange(n_int)
        cleft[:n_int] = 2 * idx + 1
        cright[:n_int] = 2 * idx + 2
        feat = rng.integers(0, n_features, size=n_int).astype(np.uint32)
        dl = rng.integers(0, 2, size=n_int).astype(np.uint32)
        sindex = np.zeros(n, dtype=np.uint32)
        sindex[:n_int] = feat | (dl << 31)
        value = np.zeros(n, dtype=np.float32)
        value[:n_int] = rng.standard_normal(n_int).astype(np.float32)
        if edges is not None:
            value[:n_int] = edges[np.abs(value[:n_int, None] - edges[None, :]).argmin(axis=1)]
        value[n_int:] = rng.uniform(-0.05, 0.05, size=n - n_int).astype(np.float32)
        # covers as training on N(0,1) rows leaves them: the logistic hessian
        # sum p(1 - p) ~ 0.25 per row of a seeded N(0,1) sample reaching each
        # leaf (+ 1 row: no empty leaf), a parent the float32 sum of its
        # children; from the covers' own stream (the trees are unchanged)
        Xs = crng.standard_normal((2000, n_features)).astype(np.float32)
        node = np.zeros(Xs.shape[0], dtype=np.int64)
        for _ in range(depth):
            go_left = ~(Xs[np.arange(Xs.shape[0]), feat[node]] >= value[node])   # x < t or NaN
            node = np.where(go_left, cleft[node], cright[node])
        hess = np.zeros(n, dtype=np.float32)
        hess[n_int:] = (0.25 * (np.bincount(node - n_int, minlength=n - n_int) + 1)).astype(np.float32)
        for i in range(n_int - 1, -1, -1):
            hess[i] = hess[2 * i + 1] + hess[2 * i + 2]
        trees.append({"cleft": cleft, "cright": cright, "sindex": sindex, "value": value,
                      "sum_hess": hess})
    K = max(1, num_class)
    tree_info = (np.arange(n_trees) % K).astype(np.int32)
    return trees, tree_info


def forest_from_raw_trees(trees: List[dict], tree_info, num_feature: int, num_class: int,
                          base_score: float, objective: str, legacy: bool = True) -> Forest:
    """Canonical forest straight from RegTree arrays (what the writers store)."""
    canon = [_tree_from_arrays(t["cleft"], t["cright"], t["sindex"], t["value"],
                              sum_hess=t.get("sum_hess")) for t in trees]
    return _assemble(canon, tree_info, num_feature, max(1, num_class), base_score, objective,
                     base_is_margin=legacy, base_first=False,
                     version=(0, 82, 0) if legacy else (1, 3, 0), fmt="raw")
