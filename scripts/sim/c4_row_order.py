"""Distinct 128-byte lines per 64-lane bottom gather of layout 8 on the C4
forest over N(0,1) rows, with the rows of each tile in arrival order or
sorted within the tile by a key (the slot of the leaf a row reaches in the
first K trees, lexicographic).  Slots are the kernel's: level by level, by
cover within a level, internal nodes and leaves mixed (cover_order).
Usage: python scripts/sim/c4_row_order.py [TREES] [TILE]"""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench

f = bench.c4_forest()[0]
to = f.tree_offset
NT = int(sys.argv[1]) if len(sys.argv) > 1 else 24
TILE = int(sys.argv[2]) if len(sys.argv) > 2 else 256
rng = np.random.default_rng(2)
R = 4096
X = rng.standard_normal((R, 64)).astype(np.float32)
D0 = 8


def tree(t):
    a, b = to[t], to[t + 1]
    feat = f.feature[a:b]; thr = f.threshold[a:b]; L = f.left[a:b]; Rr = f.right[a:b]
    cov = f.cover[a:b]
    n = b - a
    depth = np.zeros(n, np.int64)
    order = [0]; i = 0
    while i < len(order):
        v = order[i]; i += 1
        if feat[v] >= 0:
            for c in (L[v], Rr[v]):
                depth[c] = depth[v] + 1; order.append(c)
    order = sorted(order, key=lambda v: (depth[v], -cov[v]))
    slot = np.zeros(n, np.int64)
    for k, v in enumerate(order): slot[v] = k
    node = np.zeros(R, np.int64)
    paths = [node.copy()]
    for _ in range(40):
        isint = feat[node] >= 0
        if not isint.any(): break
        x = X[np.arange(R), np.maximum(feat[node], 0)].astype(np.float64)
        nxt = np.where(x <= thr[node], L[node], Rr[node])
        node = np.where(isint, nxt, node)
        paths.append(node.copy())
    P = np.array(paths)
    return slot, depth, P


trees = [tree(t) for t in range(NT)]


def lines(perm, skip=4):
    # the key trees (the first 4) are not counted: their own gain is the key's
    tot = 0; n = 0
    for slot, depth, P in trees[skip:]:
        Pp = P[:, perm]
        dep = depth[Pp]
        for w in range(R // 64):
            cols = slice(w * 64, w * 64 + 64)
            for s in range(D0, Pp.shape[0]):
                act = dep[s, cols] == s
                if not act.any(): continue
                n += 1
                tot += len(np.unique(slot[Pp[s, cols][act]] * 8 // 128))
    return tot / n, n


ident = np.arange(R)
base, nb = lines(ident)
print("arrival order: %.2f lines a gather, %d gathers" % (base, nb))
perm = []
for t0 in range(0, R, TILE):
    rows = np.arange(t0, t0 + TILE)
    P0 = trees[0][2]
    key = trees[0][0][P0[min(D0, P0.shape[0] - 1), rows]]
    perm.append(rows[np.argsort(key, kind="stable")])
perm = np.concatenate(perm)
v, n = lines(perm)
print("sorted by the slot tree 0's heap top selects (depth %d, tiles of %d): %.2f lines a gather (%.1f %%)"
      % (D0, TILE, v, 100 * (v * n / (base * nb) - 1)))
for K in (1, 2, 4):
    perm = []
    for t0 in range(0, R, TILE):
        rows = np.arange(t0, t0 + TILE)
        keys = [trees[k][0][trees[k][2][-1, rows]] for k in range(K)]
        perm.append(rows[np.lexsort(keys[::-1])])
    perm = np.concatenate(perm)
    v, n = lines(perm)
    print("sorted by the leaf slots of the first %d trees (tiles of %d): %.2f lines a gather, %d gathers (%.1f %%)"
          % (K, TILE, v, n, 100 * (v * n / (base * nb) - 1)))
