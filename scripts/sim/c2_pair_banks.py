"""C2 fixed walk: LDS cycles per 32-lane group of a ds_read_b64 pair read
(64 banks, MI355X_MICROARCH.md LDS) with heap-ordered vs cover-permuted
pair slots.  Usage: python scripts/sim/c2_pair_banks.py"""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from kfserving_amd.formats import xgboost_format as xf
trees, ti = xf.synthetic_complete_trees(100, 8, 28, seed=0)
rng = np.random.default_rng(1000)
R = 4096
X = rng.standard_normal((R, 28)).astype(np.float32)
tot = {0: 0, 1: 0}; n = 0
for t in trees:
    cl, cr, si, val, hs = t['cleft'], t['cright'], t['sindex'], t['value'], t['sum_hess']
    feat = si & 0x7FFFFFFF
    # heap index h (1-based) <-> node id v = h - 1
    # permutation per level by hess desc
    pi = np.zeros(256, np.int64)
    for lo in [1 << l for l in range(8)]:
        hs_l = hs[np.arange(lo, 2 * lo) - 1]
        order = np.argsort(-hs_l, kind='stable')
        pi[lo + order] = lo + np.arange(lo)
    h = np.ones(R, np.int64)
    for l in range(8):
        v = h - 1
        x = X[np.arange(R), feat[v]]
        right = ~(x < val[v])
        # pair read of node h at level l (levels 1..7 read from LDS; level 0 is scalar)
        if l >= 1:
            for perm in (0, 1):
                p = pi[h] if perm else h
                dw = 2 * p                      # dword index of the pair
                for g in range(R // 32):
                    d = np.unique(dw[g*32:(g+1)*32])
                    banks = np.concatenate([d % 64, (d + 1) % 64])
                    tot[perm] += np.bincount(banks, minlength=64).max()
            n += R // 32
        h = 2 * h + right
print("avg LDS cycles per 32-lane group of a pair read: plain %.3f, permuted %.3f (1.0 = conflict-free)"
      % (tot[0] / n, tot[1] / n))
