"""C4 layout 8: distinct lines of 4-byte records with children side by side
(plus the leaf-value gather they need) against the 8-byte cover-ordered
records.  Usage: python scripts/sim/c4_4byte_records.py"""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench
f = bench.c4_forest()[0]
T = f.n_trees; to = f.tree_offset
rng = np.random.default_rng(2)
R = 2048
X = rng.standard_normal((R, 64)).astype(np.float32)
D0 = 8
cur = 0; new = 0; newval = 0; ninstr = 0; maxlw = 0
for t in range(T):
    a, b = to[t], to[t+1]
    feat = f.feature[a:b]; thr = f.threshold[a:b]; L = f.left[a:b]; Rr = f.right[a:b]; cov = f.cover[a:b]
    n = b - a
    levels = []; level = [0]; depth = np.zeros(n, np.int64); d = 0
    while level:
        level = sorted(level, key=lambda v: -cov[v]); levels.append(level)
        nxt = []
        for v in level:
            depth[v] = d
            if feat[v] >= 0: nxt += [L[v], Rr[v]]
        level = nxt; d += 1
    # current: internal slots level-ordered, then leaves level-ordered (8 B)
    slot = np.zeros(n, np.int64); k = 0
    for lv in levels:
        for v in lv:
            if feat[v] >= 0: slot[v] = k; k += 1
    for lv in levels:
        for v in lv:
            if feat[v] < 0: slot[v] = k; k += 1
    # new: 4-B records, children pairs adjacent, pairs ordered by parent's position (level order by cover)
    pos = np.zeros(n, np.int64); p = 1  # root at pos 0 (pad 1)
    p = 2
    for lv in levels:
        for v in lv:
            if feat[v] >= 0:
                pos[L[v]] = p; pos[Rr[v]] = p + 1; p += 2
    lvals = [v for lv in levels for v in lv if feat[v] < 0]
    lidx = np.zeros(n, np.int64)
    for i, v in enumerate(lvals): lidx[v] = i
    node = np.zeros(R, np.int64); paths = [node.copy()]
    for s in range(40):
        isint = feat[node] >= 0
        if not isint.any(): break
        x = X[np.arange(R), np.maximum(feat[node], 0)].astype(np.float64)
        node = np.where(isint, np.where(x <= thr[node], L[node], Rr[node]), node)
        paths.append(node.copy())
    P = np.array(paths); dep = depth[P]
    for w in range(R // 64):
        cols = slice(w*64, w*64+64)
        for s in range(D0, P.shape[0]):
            act = dep[s, cols] == s
            if not act.any(): continue
            nd = P[s, cols][act]
            ninstr += 1
            cur += len(np.unique(slot[nd] * 8 // 128))
            new += len(np.unique(pos[nd] * 4 // 128))
        fin = P[-1, cols]
        newval += len(np.unique(lidx[fin] * 8 // 128))
print("gathers", ninstr, "cur lines", cur, "new 4B lines", new, "+ value gathers lines", newval, "ratio", (new + newval) / cur)
