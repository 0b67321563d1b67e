"""C4 layout 8's bottom: distinct 128-byte lines and gather instructions of
today's 8-byte records (cover-ordered, one gather per level) against 16-byte
two-level blocks (a node, its two children and the base of its up to four
grandchild blocks, stored as contiguous quads; one gather per two levels, plus
one leaf-value gather when the path ends), over N(0,1) rows, lockstep per
64-lane wave as the kernel walks (a gather is one wave instruction; its cost
is its distinct lines).
Usage: python scripts/sim/c4_block2.py [trees]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402

f = bench.c4_forest()[0]
T = int(sys.argv[1]) if len(sys.argv) > 1 else 40
to = f.tree_offset
rng = np.random.default_rng(2)
R = 2048
X = rng.standard_normal((R, 64)).astype(np.float32)
D0 = 8
cur_l = cur_i = 0
blk_l = blk_i = 0
val_l = val_i = 0
for t in range(T):
    a, b = to[t], to[t + 1]
    feat = f.feature[a:b]; thr = f.threshold[a:b]; L = f.left[a:b]; Rr = f.right[a:b]
    cov = f.cover[a:b]
    n = b - a
    depth = np.zeros(n, np.int64)
    levels = []
    level = [0]; d = 0
    while level:
        level = sorted(level, key=lambda v: -cov[v]); levels.append(level)
        nxt = []
        for v in level:
            depth[v] = d
            if feat[v] >= 0:
                nxt += [L[v], Rr[v]]
        level = nxt; d += 1
    # today: internal slots level by level by cover, then leaves (8 B each)
    slot = np.zeros(n, np.int64); k = 0
    for lv in levels:
        for v in lv:
            if feat[v] >= 0:
                slot[v] = k; k += 1
    for lv in levels:
        for v in lv:
            if feat[v] < 0:
                slot[v] = k; k += 1
    # blocks rooted at depths D0, D0 + 2, ...: a block's grandchild blocks are a
    # contiguous quad; quads numbered in order of their parent block, parent
    # blocks taken level by level by cover (so hot quads come first)
    bpos = {}
    roots = [v for v in levels[D0]] if len(levels) > D0 else []
    roots = [v for v in roots if feat[v] >= 0]
    p = 0
    for v in roots:
        bpos[v] = p; p += 1
    frontier = roots
    while frontier:
        nxt = []
        for v in sorted(frontier, key=lambda u: bpos[u]):
            for c in (L[v], Rr[v]):
                if feat[c] < 0:
                    continue
                for g in (L[c], Rr[c]):
                    if feat[g] >= 0:
                        bpos[g] = p; p += 1; nxt.append(g)
        frontier = nxt
    leaves = [v for lv in levels for v in lv if feat[v] < 0]
    lidx = {v: i for i, v in enumerate(leaves)}
    # paths
    node = np.zeros(R, np.int64); paths = [node.copy()]
    for s in range(64):
        isint = feat[node] >= 0
        if not isint.any():
            break
        x = X[np.arange(R), np.maximum(feat[node], 0)].astype(np.float64)
        node = np.where(isint, np.where(x <= thr[node], L[node], Rr[node]), node)
        paths.append(node.copy())
    P = np.array(paths); dep = depth[P]
    for w in range(R // 64):
        cols = slice(w * 64, w * 64 + 64)
        for s in range(D0, P.shape[0]):
            act = dep[s, cols] == s
            if not act.any():
                continue
            nd = P[s, cols][act]
            cur_i += 1
            cur_l += len(np.unique(slot[nd] * 8 // 128))
            # a block gather at even offsets below D0, for lanes on an internal node
            if (s - D0) % 2 == 0:
                ib = nd[feat[nd] >= 0]
                if len(ib):
                    blk_i += 1
                    blk_l += len(np.unique(np.array([bpos[v] for v in ib]) * 16 // 128))
        fin = P[-1, cols]
        fin = fin[depth[fin] > D0]   # paths that reached the bottom
        if len(fin):
            val_i += 1
            val_l += len(np.unique(np.array([lidx[v] for v in fin]) * 8 // 128))
print({"trees": T, "today": {"gathers": cur_i, "lines": cur_l},
       "block2": {"gathers": blk_i + val_i, "lines": blk_l + val_l,
                  "block_gathers": blk_i, "value_gathers": val_i},
       "ratio_lines": (blk_l + val_l) / cur_l, "ratio_gathers": (blk_i + val_i) / cur_i})
