"""c3_maxbin's compact u8 bottom (t8explicit_predict_kernel, plan_tx8): LDS
cycles of the walk's reads, per the MI355X_MICROARCH.md LDS table
(ds_read_b64: two 32-lane groups, bank (a/4) mod 64, an 8-byte pair is one
of 32 slots a 256-byte row; ds_read_u8 / ds_read_b32: two groups, conflict-free
here or (a/4) mod 32), with the bottom's pair indices numbered as plan_tx8
numbers them (breadth-first, each level by cover) or bank-aware (greedy: the
pairs read most go to the least-loaded slots, counted on a training sample).

A lane at an internal bottom node reads the pair of that node's children; a
lane at a leaf re-reads the pair it sits in, i.e. its parent's children pair
(the compact bottom's self loop), every step until its group of ILP trees
ends.  Usage: python scripts/sim/c3_maxbin_banks.py [n_trees]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from kfserving_amd.formats import lightgbm_format as lf   # noqa: E402

D0, ILP, TREES_PER_STAGE, R = 6, 4, 12, 512
STAGE_OFF = 51216            # the bin image of a 512-row u8 tile at F = 100, aligned


def tree_nodes(t):
    """node ids: internal i -> i, leaf j -> n_int + j"""
    n_int = len(t["split_feature"])
    L = lambda c: int(c) if c >= 0 else n_int + ~int(c)
    left = np.array([L(c) for c in t["left_child"]])
    right = np.array([L(c) for c in t["right_child"]])
    cover = np.concatenate([t["internal_count"], t["leaf_count"]]).astype(np.float64)
    return n_int, t["split_feature"], t["threshold"], left, right, cover


def plan(t, pair_order=None):
    """plan_tx8's positions: the top's cut (left to right), padded even, then
    breadth-first children, each level's internal nodes by cover.  Returns
    (entries, kpair, pos_of, n_pos) with kpair[v] the pair index of internal
    node v's children.  pair_order (optional): a map v -> pair index to use
    instead of the breadth-first numbering (a permutation of the same set)."""
    n_int, feat, thr, left, right, cover = tree_nodes(t)
    ents, st = [], [(0, 0)]
    while st:
        v, l = st.pop()
        if l == D0 or v >= n_int:
            ents.append(v)
            continue
        st.append((right[v], l + 1))
        st.append((left[v], l + 1))
    ordr = list(ents) + ([-1] if len(ents) & 1 else [])
    half = len(ordr) // 2
    kpair = {}
    lvl = [v for v in ents if v < n_int]
    k = 0
    while lvl:
        lvl.sort(key=lambda v: -cover[v])
        nxt = []
        for v in lvl:
            kpair[v] = half + k
            k += 1
            for c in (left[v], right[v]):
                if c < n_int:
                    nxt.append(c)
        lvl = nxt
    if pair_order is not None:
        kpair = dict(pair_order)
    n_pos = 2 * (half + k)
    pos = np.full(n_int + n_int + 1, -1)
    for p, v in enumerate(ordr):
        if v >= 0 and pos[v] < 0:
            pos[v] = p
    for v, kp in kpair.items():
        pos[left[v]], pos[right[v]] = 2 * kp, 2 * kp + 1
    return ents, kpair, pos, n_pos, half


def walk(trees, plans, X, count=None):
    """LDS cycles of the walk over rows X (a multiple of 64), tree groups of
    ILP in stages of TREES_PER_STAGE.  count: dict (tree, pair) -> reads, filled."""
    cyc = ideal = 0
    T = len(trees)
    nt = [tree_nodes(t) for t in trees]
    # byte offsets in the stage (plan_tx8: top 8 << D0 bytes + 4 B a position, 16-aligned)
    sizes = [(8 << D0) + ((p[3] * 4 + 15) & ~15) for p in plans]
    off = np.concatenate([[0], np.cumsum(sizes)])
    for s0 in range(0, T, TREES_PER_STAGE):
        for g0 in range(s0, min(s0 + TREES_PER_STAGE, T), ILP):
            grp = list(range(g0, min(g0 + ILP, T)))
            for w0 in range(0, X.shape[0], 64):
                xs = X[w0:w0 + 64]
                node = {}
                for q in grp:
                    n_int, feat, thr, left, right, cover = nt[q]
                    base = STAGE_OFF + off[q] - off[s0]
                    v = np.zeros(64, np.int64)
                    idx = np.ones(64, np.int64)
                    for l in range(D0):     # the heap top: pair reads at base + 8 idx
                        inside = v < n_int
                        cyc_q = 0
                        for h in (0, 32):
                            a = base + 8 * idx[h:h + 32]
                            u = np.unique(a)
                            cyc_q += np.bincount((u // 8) % 32, minlength=32).max()
                        cyc += cyc_q + 2          # + the bin read
                        ideal += 4
                        go_r = np.zeros(64, bool)
                        vi = v[inside]
                        go_r[inside] = ~(xs[np.arange(64)[inside], feat[vi]] <= thr[vi])
                        idx = 2 * idx + go_r
                        v = np.where(inside, np.where(go_r, right[np.minimum(v, n_int - 1)],
                                                      left[np.minimum(v, n_int - 1)]), v)
                    node[q] = v
                while True:
                    if all((node[q] >= nt[q][0]).all() for q in grp):
                        break
                    for q in grp:
                        n_int, feat, thr, left, right, cover = nt[q]
                        ents, kpair, pos, n_pos, half = plans[q]
                        base = STAGE_OFF + off[q] - off[s0] + (8 << D0)
                        v = node[q]
                        pr = np.array([kpair[x] if x < n_int else pos[x] // 2 for x in v])
                        if count is not None:
                            for x in v:
                                if x < n_int:
                                    count[(q, x)] = count.get((q, x), 0) + 1
                                else:
                                    count[(q, ('leaf', x))] = count.get((q, ('leaf', x)), 0) + 1
                        for h in (0, 32):
                            a = base + 8 * pr[h:h + 32]
                            u = np.unique(a)
                            cyc += np.bincount((u // 8) % 32, minlength=32).max()
                        cyc += 2
                        ideal += 4
                        inside = v < n_int
                        if inside.any():
                            vi = v[inside]
                            go_r = ~(xs[np.arange(64)[inside], feat[vi]] <= thr[vi])
                            v = v.copy()
                            v[inside] = np.where(go_r, right[vi], left[vi])
                        node[q] = v
    return cyc, ideal


def bank_aware(t, q, plan0, count, stage_base_mod):
    """Greedy: internal bottom nodes by read mass (their own reads plus their
    leaf children's), each to the free pair index whose 8-byte slot has the
    least mass so far."""
    n_int, feat, thr, left, right, cover = tree_nodes(t)
    ents, kpair, pos, n_pos, half = plan0
    mass = {}
    for v in kpair:
        m = count.get((q, v), 0)
        for c in (left[v], right[v]):
            if c >= n_int:
                m += count.get((q, ("leaf", c)), 0)
        mass[v] = m
    free = sorted(kpair.values())
    load = np.zeros(32)
    for p in range(half):    # the entries' pairs are fixed: leaves among them load their slot
        for v in ents[2 * p:2 * p + 2]:
            if v >= n_int:
                load[(stage_base_mod // 8 + p) % 32] += count.get((q, ("leaf", v)), 0)
    out = {}
    for v in sorted(mass, key=lambda v: -mass[v]):
        slots = np.array([(stage_base_mod // 8 + k) % 32 for k in free])
        j = int(np.argmin(load[slots] * 1e6 + np.arange(len(free))))
        out[v] = free.pop(j)
        load[slots[j]] += mass[v]
    return out


def main():
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 48
    trees = lf.synthetic_maxbin_trees(T, 255, 100, seed=1)
    X_train = np.random.default_rng(100).standard_normal((2048, 100))
    X_eval = np.random.default_rng(200).standard_normal((2048, 100))
    plans = [plan(t) for t in trees]
    c0, i0 = walk(trees, plans, X_eval)
    print(f"plan_tx8 order: LDS cycles {c0}, conflict-free {i0}, conflicts {1 - i0 / c0:.3f} of cycles")
    count = {}
    walk(trees, plans, X_train, count)
    sizes = [(8 << D0) + ((p[3] * 4 + 15) & ~15) for p in plans]
    off = np.concatenate([[0], np.cumsum(sizes)])
    plans2 = []
    for q, t in enumerate(trees):
        s0 = (q // TREES_PER_STAGE) * TREES_PER_STAGE
        bm = (STAGE_OFF + off[q] - off[s0] + (8 << D0)) % 256
        plans2.append(plan(t, bank_aware(t, q, plans[q], count, bm)))
    c1, i1 = walk(trees, plans2, X_eval)
    print(f"bank-aware:     LDS cycles {c1}, conflict-free {i1}, conflicts {1 - i1 / c1:.3f} of cycles"
          f" ({c1 / c0 - 1:+.3f})")


if __name__ == "__main__":
    main()
