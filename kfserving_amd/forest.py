"""Canonical structure-of-arrays forest handed to libtreeinfer (treeinfer.h).

Every loader (XGBoost legacy binary / binf / JSON, LightGBM text v3, sklearn
tree ensembles) flattens its model into this one library-agnostic form.  The
split rule is normalised to ``left iff x <= threshold`` plus two per-node flag
bits (NaN direction, LightGBM zero flip) -- see the comment block at the top of
include/treeinfer.h for how each library's comparison maps onto it.

This replaces the trained-model handles the reference plugins keep:
``xgb.Booster`` (python/xgbserver/xgbserver/model.py:38-39), ``lgb.Booster``
(python/lgbserver/lgbserver/model.py:39-40) and the unpickled sklearn
estimator (python/sklearnserver/sklearnserver/model.py:38).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

# element types (treeinfer.h)
TI_F32 = 0
TI_F64 = 1
TI_I32 = 2

# node flags
NODE_NAN_LEFT = 0x01
NODE_ZERO_FLIP = 0x02
NODE_CATEGORICAL = 0x04

# transforms
T_IDENTITY = 0
T_SIGMOID = 1
T_SOFTMAX = 2
T_ARGMAX = 3
T_HINGE = 4
T_EXP = 5
T_SIGNSQUARE = 6
T_LOG1PEXP = 7
T_STEP = 8          # x >= 0 -> 1 (sklearn binary GradientBoostingClassifier.predict)

# output kinds
OUT_MARGIN = 0
OUT_PREDICT = 1
OUT_LEAF = 2
OUT_CONTRIB = 3     # TreeSHAP contributions [rows, K * (F + 1)], bias last per group

# LightGBM missing types (decision_type bits 2-3)
MISSING_NONE = 0
MISSING_ZERO = 1
MISSING_NAN = 2

# outputs per row; the library splits forests of more than 16 groups into
# parts of at most 16 (treeinfer.hip, create_chunked)
MAX_GROUPS = 1 << 20


@dataclass
class Forest:
    """A tree ensemble in the engine's canonical SoA form.

    Node arrays are concatenated over trees; ``left``/``right`` are tree-local
    indices (-1 for leaves).  ``leaf_value`` is ``[n_nodes, leaf_width]``
    (rows of internal nodes are ignored).
    """

    n_features: int
    n_groups: int
    leaf_width: int
    accum_dtype: int                 # TI_F32 | TI_F64
    base_first: bool
    lgb_zero_map: bool
    tree_offset: np.ndarray          # int64 [T+1]
    tree_group: np.ndarray           # int32 [T]
    feature: np.ndarray              # int32 [N]
    threshold: np.ndarray            # float64 [N]
    flags: np.ndarray                # uint8 [N]
    left: np.ndarray                 # int32 [N]
    right: np.ndarray                # int32 [N]
    leaf_id: np.ndarray              # int32 [N]
    leaf_value: np.ndarray           # float64 [N, leaf_width]
    base_margin: np.ndarray          # float64 [K]
    average_divisor: float = 1.0
    transform: int = T_IDENTITY
    transform_param: float = 1.0
    input_dtype: int = TI_F32        # how the plugin feeds X (xgb/sk: f32, lgb: f64)
    # categorical splits (LightGBM): node goes left iff bit trunc(x) is set in
    # cat_bits[cat_offset[n] : cat_offset[n] + cat_nwords[n]]
    cat_bits: Optional[np.ndarray] = None       # uint32 [W]
    cat_offset: Optional[np.ndarray] = None     # int64 [N]
    cat_nwords: Optional[np.ndarray] = None     # int32 [N]
    # node covers (xgboost sum_hess, LightGBM data counts, sklearn weighted
    # samples): the node weights of TreeSHAP contributions (OUT_CONTRIB)
    cover: Optional[np.ndarray] = None          # float64 [N]
    library: str = ""
    objective: str = ""
    feature_names: Optional[List[str]] = None
    meta: Dict[str, object] = field(default_factory=dict)

    @property
    def n_trees(self) -> int:
        return int(self.tree_offset.shape[0] - 1)

    @property
    def n_nodes(self) -> int:
        return int(self.feature.shape[0])

    def tree_slice(self, t: int) -> slice:
        return slice(int(self.tree_offset[t]), int(self.tree_offset[t + 1]))

    def depths(self) -> np.ndarray:
        """Max leaf depth of each tree (root = depth 0)."""
        out = np.zeros(self.n_trees, dtype=np.int32)
        for t in range(self.n_trees):
            s = self.tree_slice(t)
            feat, lft, rgt = self.feature[s], self.left[s], self.right[s]
            depth = np.full(feat.shape[0], -1, dtype=np.int32)
            depth[0] = 0
            frontier = np.array([0], dtype=np.int64)
            d = 0
            while frontier.size:
                internal = frontier[feat[frontier] >= 0]
                if internal.size == 0:
                    break
                d += 1
                frontier = np.concatenate([lft[internal], rgt[internal]]).astype(np.int64)
                depth[frontier] = d
            out[t] = depth.max()
        return out

    def validate(self) -> None:
        """Cheap structural checks before the forest crosses the C ABI."""
        T = self.n_trees
        N = self.n_nodes
        if T <= 0:
            raise ValueError("forest has no trees")
        if not (1 <= self.n_groups <= MAX_GROUPS):
            raise ValueError(f"n_groups={self.n_groups} outside [1, {MAX_GROUPS}]")
        if self.leaf_width not in (1, self.n_groups):
            raise ValueError("leaf_width must be 1 or n_groups")
        if self.tree_offset[0] != 0 or self.tree_offset[-1] != N:
            raise ValueError("tree_offset does not cover the node arrays")
        for name, arr in (("threshold", self.threshold), ("flags", self.flags),
                          ("left", self.left), ("right", self.right), ("leaf_id", self.leaf_id)):
            if arr.shape[0] != N:
                raise ValueError(f"{name} has {arr.shape[0]} entries, expected {N}")
        if self.leaf_value.shape != (N, self.leaf_width):
            raise ValueError("leaf_value must be [n_nodes, leaf_width]")
        if self.base_margin.shape != (self.n_groups,):
            raise ValueError("base_margin must be [n_groups]")
        internal = self.feature >= 0
        if np.any(self.feature[internal] >= self.n_features):
            raise ValueError("split feature index >= n_features")
        if self.cover is not None and self.cover.shape[0] != N:
            raise ValueError("cover must be [n_nodes]")
        cat = internal & ((self.flags & NODE_CATEGORICAL) != 0)
        if cat.any():
            if self.cat_bits is None or self.cat_offset is None or self.cat_nwords is None:
                raise ValueError("categorical nodes without bitsets")
            end = self.cat_offset[cat] + self.cat_nwords[cat]
            if np.any(self.cat_offset[cat] < 0) or np.any(end > self.cat_bits.shape[0]):
                raise ValueError("categorical bitset out of range")

    def contiguous(self) -> "Forest":
        """Return self with every array C-contiguous in the ABI's dtypes."""
        self.tree_offset = np.ascontiguousarray(self.tree_offset, dtype=np.int64)
        self.tree_group = np.ascontiguousarray(self.tree_group, dtype=np.int32)
        self.feature = np.ascontiguousarray(self.feature, dtype=np.int32)
        self.threshold = np.ascontiguousarray(self.threshold, dtype=np.float64)
        self.flags = np.ascontiguousarray(self.flags, dtype=np.uint8)
        self.left = np.ascontiguousarray(self.left, dtype=np.int32)
        self.right = np.ascontiguousarray(self.right, dtype=np.int32)
        self.leaf_id = np.ascontiguousarray(self.leaf_id, dtype=np.int32)
        self.leaf_value = np.ascontiguousarray(
            np.asarray(self.leaf_value, dtype=np.float64).reshape(self.n_nodes, self.leaf_width))
        self.base_margin = np.ascontiguousarray(self.base_margin, dtype=np.float64)
        if self.cover is not None:
            self.cover = np.ascontiguousarray(self.cover, dtype=np.float64)
        if self.cat_bits is not None:
            self.cat_bits = np.ascontiguousarray(self.cat_bits, dtype=np.uint32)
            self.cat_offset = np.ascontiguousarray(self.cat_offset, dtype=np.int64)
            self.cat_nwords = np.ascontiguousarray(self.cat_nwords, dtype=np.int32)
        return self

    def tree_subset(self, t0: int, t1: int, keep_base: bool = True) -> "Forest":
        """Trees [t0, t1) as a forest of their own (same features, groups,
        transform and divisor); base margin zeroed unless ``keep_base`` -- one
        rank's shard in the tree-sharded mode (tree_shard.py)."""
        import dataclasses
        if not (0 <= t0 < t1 <= self.n_trees):
            raise ValueError(f"bad tree range [{t0}, {t1}) of {self.n_trees}")
        s = slice(int(self.tree_offset[t0]), int(self.tree_offset[t1]))
        cut = lambda a: None if a is None else np.ascontiguousarray(a[s])   # noqa: E731
        return dataclasses.replace(
            self, tree_offset=self.tree_offset[t0:t1 + 1] - self.tree_offset[t0],
            tree_group=np.ascontiguousarray(self.tree_group[t0:t1]),
            feature=cut(self.feature), threshold=cut(self.threshold), flags=cut(self.flags),
            left=cut(self.left), right=cut(self.right), leaf_id=cut(self.leaf_id),
            leaf_value=cut(self.leaf_value), cover=cut(self.cover),
            cat_offset=cut(self.cat_offset), cat_nwords=cut(self.cat_nwords),
            base_margin=(self.base_margin.copy() if keep_base
                         else np.zeros_like(self.base_margin)),
            meta=dict(self.meta))

    @property
    def has_categorical(self) -> bool:
        return bool(np.any((self.flags & NODE_CATEGORICAL) != 0))

    def output_width(self, kind: int) -> int:
        if kind == OUT_LEAF:
            return self.n_trees
        if kind == OUT_CONTRIB:
            return self.n_groups * (self.n_features + 1)
        if kind == OUT_PREDICT and self.transform == T_ARGMAX:
            return 1
        return self.n_groups

    def output_dtype(self, kind: int):
        if kind == OUT_LEAF:
            return np.int32
        return np.float32 if self.accum_dtype == TI_F32 else np.float64


def concat_trees(trees: List[dict], leaf_width: int) -> Dict[str, np.ndarray]:
    """Concatenate per-tree node dicts into the SoA arrays of :class:`Forest`.

    Each tree dict holds equal-length arrays ``feature, threshold, flags,
    left, right, leaf_id`` and ``leaf_value`` of shape [n, leaf_width].
    """
    sizes = [int(t["feature"].shape[0]) for t in trees]
    offset = np.zeros(len(trees) + 1, dtype=np.int64)
    np.cumsum(sizes, out=offset[1:])
    cat = {}
    for key, dt in (("feature", np.int32), ("threshold", np.float64), ("flags", np.uint8),
                    ("left", np.int32), ("right", np.int32), ("leaf_id", np.int32)):
        cat[key] = np.concatenate([np.asarray(t[key], dtype=dt) for t in trees])
    cat["leaf_value"] = np.concatenate(
        [np.asarray(t["leaf_value"], dtype=np.float64).reshape(-1, leaf_width) for t in trees])
    if all(t.get("cover") is not None for t in trees):
        cat["cover"] = np.concatenate([np.asarray(t["cover"], dtype=np.float64) for t in trees])
    else:
        cat["cover"] = None
    cat["tree_offset"] = offset
    return cat


def round_down_f32(t: np.ndarray) -> np.ndarray:
    """Largest float32 <= t (elementwise, NaN preserved).

    For every float32 x: ``x <= t`` (in float64) iff ``x <= round_down_f32(t)``.
    """
    t = np.asarray(t, dtype=np.float64)
    with np.errstate(over="ignore", invalid="ignore"):
        f = t.astype(np.float32)
        up = f.astype(np.float64) > t
        f[up] = np.nextafter(f[up], np.float32(-np.inf))
    return f
