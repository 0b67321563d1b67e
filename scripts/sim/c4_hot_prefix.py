"""C4 layout 8: lines saved by an LDS cache of the first H records of each
bottom level.  Usage: python scripts/sim/c4_hot_prefix.py"""
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
res = {}
for H in (0, 8, 16, 32):
    res[H] = [0, 0]
for t in range(T):
    a, b = to[t], to[t+1]
    feat = f.feature[a:b]; thr = f.threshold[a:b]; L = f.left[a:b]; Rr = f.right[a:b]; cov = f.cover[a:b]
    n = b - a
    level = [0]; depth = np.zeros(n, np.int64); internal = []; leaves = []
    istart = {}; lstart = {}; d = 0
    levels = []
    while level:
        level = sorted(level, key=lambda v: -cov[v])
        levels.append(level)
        nxt = []
        for v in level:
            depth[v] = d
            if feat[v] >= 0: nxt += [L[v], Rr[v]]
        level = nxt; d += 1
    slot = np.zeros(n, np.int64); rank_in_level = np.zeros(n, np.int64)
    k = 0
    for lv in levels:
        r = 0
        for v in lv:
            if feat[v] >= 0: slot[v] = k; k += 1; rank_in_level[v] = r; r += 1
    for lv in levels:
        r = 0
        for v in lv:
            if feat[v] < 0: slot[v] = k; k += 1; rank_in_level[v] = r; r += 1
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
            for H in res:
                cold = rank_in_level[nd] >= H
                res[H][0] += len(np.unique(slot[nd[cold]] * 8 // 128))
                res[H][1] += (~cold).sum()
tot_lanes = None
for H in res:
    print(f"H {H}: lines {res[H][0]}  ({res[H][0]/res[0][0]:.2f} of H=0), hot lane-gathers {res[H][1]}")
