"""Fit the C4 model once and cache it for bench.py / the GPU tests.

BASELINE.json configs[3] / SURVEY.md 8(d) C4: sklearn
RandomForestRegressor(n_estimators=200, max_depth=16, max_features=1/3,
random_state=0) fitted on N(0,1) [200k x 64] with the nonlinear target below
(~6.9k nodes per tree).  The fit takes minutes, so it is not redone inside
every bench run: this script writes

  bench_data/c4_rf200_d16.npz         raw tree arrays (save_tree_arrays, no pickle)
  bench_data/c4_rf200_d16_check.npz   4,096 seeded rows (1 % NaN) with sklearn's
                                      own predict() and apply() outputs on them

bench_data/ is git-ignored (about 25 MB) but not gpurun-ignored, so it travels
to the GPU box with the tree.  bench.py falls back to fitting a smaller
forest when the file is absent and says so in its output.

Usage: python scripts/make_c4_model.py [--jobs N]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT_DIR = os.path.join(ROOT, "bench_data")
MODEL = os.path.join(OUT_DIR, "c4_rf200_d16.npz")
CHECK = os.path.join(OUT_DIR, "c4_rf200_d16_check.npz")


def training_set(rows: int, seed: int = 0):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((rows, 64)).astype(np.float32)
    y = np.sin(2 * X[:, 0]) + X[:, 1] * X[:, 2] + X[:, 3] ** 2 + 0.1 * rng.standard_normal(rows)
    return X, y


def fit(rows: int, jobs: int, n_estimators: int = 200):
    from sklearn.ensemble import RandomForestRegressor
    X, y = training_set(rows)
    return RandomForestRegressor(n_estimators=n_estimators, max_depth=16, max_features=1 / 3,
                                 random_state=0, n_jobs=jobs).fit(X, y)


def sklearn_estimator(path: str = MODEL):
    """sklearn's own RandomForestRegressor rebuilt from the cached tree arrays
    (no pickle, no refit): each member's ``tree_`` is restored through
    ``Tree.__setstate__`` from the arrays the fit produced, so ``predict`` is
    the library's own code on the fitted model (bench.py's C4 CPU baseline).
    The node fields predict never reads (impurity, sample counts) are zero;
    ``weighted_n_node_samples`` is the cached cover.  check() proves the
    rebuilt estimator answers exactly what the fitted one did."""
    from sklearn.ensemble import RandomForestRegressor
    from sklearn.tree import DecisionTreeRegressor
    from sklearn.tree._tree import Tree
    z = np.load(path, allow_pickle=False)
    T, F = int(z["n_trees"]), int(z["n_features"])
    est = RandomForestRegressor(n_estimators=T, max_depth=16, max_features=1 / 3, random_state=0)
    members = []
    for i in range(T):
        left = z[f"t{i}_children_left"]
        n = left.shape[0]
        nodes = np.zeros(n, dtype=[("left_child", "<i8"), ("right_child", "<i8"),
                                   ("feature", "<i8"), ("threshold", "<f8"),
                                   ("impurity", "<f8"), ("n_node_samples", "<i8"),
                                   ("weighted_n_node_samples", "<f8"),
                                   ("missing_go_to_left", "u1")])
        nodes["left_child"] = left
        nodes["right_child"] = z[f"t{i}_children_right"]
        nodes["feature"] = z[f"t{i}_feature"]
        nodes["threshold"] = z[f"t{i}_threshold"]
        nodes["missing_go_to_left"] = z[f"t{i}_missing_go_to_left"]
        if f"t{i}_cover" in z.files:
            nodes["weighted_n_node_samples"] = z[f"t{i}_cover"]
        value = np.ascontiguousarray(z[f"t{i}_value"], dtype=np.float64)
        depth = _depth(left, nodes["right_child"])
        tree = Tree(F, np.array([1], dtype=np.intp), 1)
        tree.__setstate__({"max_depth": depth, "node_count": n, "nodes": nodes, "values": value})
        m = DecisionTreeRegressor(max_depth=16, max_features=1 / 3)
        m.tree_ = tree
        m.n_features_in_ = F
        m.n_outputs_ = 1
        m.max_features_ = max(1, int(F / 3))
        members.append(m)
    est.estimators_ = members
    est.estimator_ = DecisionTreeRegressor()
    est.n_features_in_ = F
    est.n_outputs_ = 1
    return est


def _depth(left, right) -> int:
    depth = np.zeros(left.shape[0], dtype=np.int64)
    for j in range(left.shape[0]):     # children follow their parent in sklearn's order
        if left[j] >= 0:
            depth[left[j]] = depth[right[j]] = depth[j] + 1
    return int(depth.max())


def check(est) -> bool:
    """The rebuilt estimator's predict on the cached check rows equals the
    fitted estimator's, bit for bit (single thread: estimator order)."""
    z = np.load(CHECK, allow_pickle=False)
    est.set_params(n_jobs=1)
    return bool(np.array_equal(est.predict(z["X"]), z["predict"]))


def check_rows(n: int = 4096, seed: int = 2):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, 64)).astype(np.float32)
    X[rng.random(X.shape) < 0.01] = np.nan
    return X


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--jobs", type=int, default=os.cpu_count())
    p.add_argument("--fit-rows", type=int, default=200_000)
    a = p.parse_args()
    from kfserving_amd.formats.sklearn_format import save_tree_arrays
    os.makedirs(OUT_DIR, exist_ok=True)
    t0 = time.perf_counter()
    est = fit(a.fit_rows, a.jobs)
    print(f"fit {time.perf_counter() - t0:.1f} s, "
          f"{sum(e.tree_.node_count for e in est.estimators_) / 200:.0f} nodes/tree", flush=True)
    save_tree_arrays(MODEL, est)
    X = check_rows()
    est.set_params(n_jobs=1)   # estimator order: the summation order the engine reproduces
    np.savez_compressed(CHECK, X=X, predict=est.predict(X), apply=est.apply(X).astype(np.int32),
                        fit_rows=np.int64(a.fit_rows))
    print("wrote", MODEL, CHECK)


if __name__ == "__main__":
    main()
