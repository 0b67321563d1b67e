"""Distinct 128-byte lines per 64-lane bottom gather of layout 8 on the C4
forest over N(0,1) rows (a gather costs its distinct lines):
breadth-first slots vs slots by cover within each level.
Usage: python scripts/sim/c4_gather_lines.py SORT MIX LEAFBFS  (e.g. 1 0 0)"""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench
f = bench.c4_forest()[0]
T = f.n_trees
to = f.tree_offset
rng = np.random.default_rng(2)
R = 4096
X = rng.standard_normal((R, 64)).astype(np.float32)
D0 = 8
SORT = int(sys.argv[1]); MIX = int(sys.argv[2]); LEAFBFS = int(sys.argv[3])
cur_lines = 0; alt_lines = 0; alt2_lines = 0; n_instr = 0; n_instr_alt = 0
for t in range(T):
    a, b = to[t], to[t+1]
    feat = f.feature[a:b]; thr = f.threshold[a:b]; L = f.left[a:b]; Rr = f.right[a:b]
    n = b - a
    # BFS order
    order = [0]; depth = {0: 0}; i = 0
    while i < len(order):
        v = order[i]; i += 1
        if feat[v] >= 0:
            for c in (L[v], Rr[v]):
                depth[c] = depth[v] + 1; order.append(c)
    cov = f.cover[a:b]
    import itertools
    # within each level, hottest (largest cover) first
    order = sorted(order, key=lambda v: (depth[v], -cov[v])) if SORT else order
    internal = [v for v in order if feat[v] >= 0]
    leaves = [v for v in order if feat[v] < 0]
    if LEAFBFS:
        bfs = [0]; j = 0
        while j < len(bfs):
            v = bfs[j]; j += 1
            if feat[v] >= 0: bfs += [L[v], Rr[v]]
        leaves = [v for v in bfs if feat[v] < 0]
    slot = np.zeros(n, np.int64)
    if MIX:
        for k, v in enumerate(order): slot[v] = k
    else:
        for k, v in enumerate(internal): slot[v] = k
        for k, v in enumerate(leaves): slot[v] = len(internal) + k
    islot = np.zeros(n, np.int64); lslot = np.zeros(n, np.int64)
    for k, v in enumerate(internal): islot[v] = k
    for k, v in enumerate(leaves): lslot[v] = k
    # paths
    node = np.zeros(R, np.int64)
    paths = [node.copy()]
    for d in range(40):
        isint = feat[node] >= 0
        if not isint.any(): break
        x = X[np.arange(R), np.maximum(feat[node], 0)].astype(np.float64)
        go_left = x <= thr[node]
        nxt = np.where(go_left, L[node], Rr[node])
        node = np.where(isint, nxt, node)
        paths.append(node.copy())
    P = np.array(paths)   # [steps, R]
    # gathers of the bottom: records fetched at depth >= D0 (node at depth D0 is the first gather)
    dep = np.vectorize(depth.get)(P)
    for w in range(R // 64):
        cols = slice(w*64, w*64+64)
        for s in range(D0, P.shape[0]):
            nodes = P[s, cols]; dd = dep[s, cols]
            prev = P[s-1, cols]
            # a lane gathers at step s if it moved (node at depth s exactly == s)
            act = dd == s
            if s == D0: act = dd == D0
            if not act.any(): continue
            nd = nodes[act]
            n_instr += 1
            cur_lines += len(np.unique(slot[nd] * 8 // 128))
            isl = feat[nd] >= 0
            li = np.unique(islot[nd[isl]] * 4 // 128); ll = np.unique(lslot[nd[~isl]] * 8 // 128)
            alt_lines += len(li) + len(ll)
            n_instr_alt += (len(li) > 0) + (len(ll) > 0)
print('sort',SORT,'mix',MIX,"instr", n_instr, "cur lines/instr", cur_lines / n_instr, "alt lines total ratio", alt_lines / cur_lines, "alt instr", n_instr_alt)
