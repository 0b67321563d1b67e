import os, sys, tempfile, json
import numpy as np
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from kfserving_amd.engine import DeviceForest
from kfserving_amd.forest import OUT_LEAF, OUT_MARGIN
from kfserving_amd.formats import load_lightgbm_model
from kfserving_amd.formats import lightgbm_format as lf
trees = lf.synthetic_leafwise_trees(41, 255, 40, seed=7)
with tempfile.TemporaryDirectory() as d:
    p = os.path.join(d, "model.txt")
    lf.write_lightgbm_text(p, trees, 40, "binary sigmoid:1")
    f = load_lightgbm_model(p)
def mk(v):
    os.environ["TI_TX16"] = v
    dv = DeviceForest(f, [0]); del os.environ["TI_TX16"]; return dv
d16, drec = mk("1"), mk("0")
print("info16", {k: d16.info()[k] for k in ("layout", "bottom", "tree_ilp", "n_stages", "top_depth")})
print("inforec", {k: drec.info()[k] for k in ("layout", "bottom", "tree_ilp", "n_stages", "top_depth")})
sp_all = {"nan": [np.nan], "zero": [0.0, -0.0, 1e-40, -1e-36, 1e-35], "tiny": [2e-35], "inf": [np.inf, -np.inf]}
for name, sp in list(sp_all.items()) + [("all", sum(sp_all.values(), []))]:
    for dt in (np.float64, np.float32):
        rng = np.random.default_rng(256)
        X = rng.standard_normal((255, 40))
        sp = np.array(sp)
        m = rng.random(X.shape) < 0.15
        X[m] = sp[rng.integers(0, len(sp), m.sum())]
        X = X.astype(dt)
        a, b = d16.predict(X, OUT_MARGIN), drec.predict(X, OUT_MARGIN)
        la, lb = d16.predict(X, OUT_LEAF), drec.predict(X, OUT_LEAF)
        bad = np.nonzero(a != b)[0]
        badl = np.argwhere(la != lb)
        print(name, dt.__name__, "rows differing", len(bad), "leaf mismatches", len(badl), badl[:5].tolist())
        if len(badl) and name == "all":
            r, t = badl[0]
            print(" row", r, "tree", t, "t16 leaf", la[r, t], "rec leaf", lb[r, t])
            tr = trees[t]
            node = 0; path = []
            while node >= 0:
                fe = tr["split_feature"][node]; th = tr["threshold"][node]; dtp = tr["decision_type"][node]
                x = float(X[r, fe])
                path.append((node, int(fe), float(th), int(dtp), x))
                # lightgbm rule (missing types), via the oracle's logic is complex: print only
                break
            print(" root", path)
