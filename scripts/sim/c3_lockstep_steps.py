"""Layout 9 bottoms: lockstep tree-steps per wave (a group runs for its
deepest lane and tree) against per-lane progress over a stage's trees, on
the C3 and c3_maxbin forests.
Usage: python scripts/sim/c3_lockstep_steps.py maxbin|iid"""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from kfserving_amd.formats import lightgbm_format as lf
which = sys.argv[1]
trees = (lf.synthetic_maxbin_trees if which == 'maxbin' else lf.synthetic_leafwise_trees)(1000, 255, 100, seed=1)
rng = np.random.default_rng(3)
R = 2048
X = rng.standard_normal((R, 100))
D0 = 6
depths = np.zeros((len(trees), R), np.int64)
for ti, t in enumerate(trees):
    sf = np.asarray(t['split_feature']); thr = np.asarray(t['threshold'], float)
    L = np.asarray(t['left_child']); Rr = np.asarray(t['right_child'])
    node = np.zeros(R, np.int64); d = np.zeros(R, np.int64)
    live = np.ones(R, bool)
    while live.any():
        nd = node[live]
        x = X[np.arange(R)[live], sf[nd]]
        nxt = np.where(x <= thr[nd], L[nd], Rr[nd])
        node[live] = nxt; d[live] += 1
        live = node >= 0
    depths[ti] = d
bot = np.maximum(depths - D0, 0)   # bottom steps per (tree,row)
print(which, "mean depth", depths.mean(), "mean bottom", bot.mean())
for ILP, S in ((4, 12), (7, 7)):
    lock = 0; lane = 0; lane2 = 0
    for w in range(R // 64):
        b = bot[:, w*64:(w+1)*64]
        for s0 in range(0, len(trees), S):
            st = b[s0:s0+S]
            # lockstep: groups of ILP trees, each group runs max over lanes & trees (+1 exit pass)
            for g in range(0, st.shape[0], ILP):
                lock += st[g:g+ILP].max() + 1
            # per-lane progress, ILP chains over the stage's trees (round robin)
            ch = [st[c::ILP].sum(axis=0) for c in range(ILP)]
            lane += max(c.max() for c in ch) + 1
    print(f"ILP {ILP} stage {S}: lockstep steps/wave {lock/(R//64):.0f}  per-lane chains {lane/(R//64):.0f}  ratio {lane/lock:.2f}")
print("--- LDS tree-step instructions per wave (steps x width)")
for S in (7, 12):
    for ILP in (4, 7) if S == 7 else (4,):
        lock = 0
        for w in range(R // 64):
            b = bot[:, w*64:(w+1)*64]
            for s0 in range(0, len(trees), S):
                st = b[s0:s0+S]
                for g in range(0, st.shape[0], ILP):
                    lock += (st[g:g+ILP].max() + 1) * ILP
        print(f"S {S} lockstep ILP {ILP}: {lock/(R//64):.0f}")
    for C in (1, 2, 3, 4):
        lane = 0
        for w in range(R // 64):
            b = bot[:, w*64:(w+1)*64]
            for s0 in range(0, len(trees), S):
                st = b[s0:s0+S]
                ch = [st[c::C].sum(axis=0) for c in range(C)]
                lane += (max(c.max() for c in ch) + 1) * C
        print(f"S {S} per-lane C {C}: {lane/(R//64):.0f}")
print("--- lockstep tree-steps, S=12 stage")
for ILP in (1, 2, 3, 4, 6):
    lock = 0; steps = 0
    for w in range(R // 64):
        b = bot[:, w*64:(w+1)*64]
        for s0 in range(0, len(trees), 12):
            st = b[s0:s0+12]
            for g in range(0, st.shape[0], ILP):
                m = st[g:g+ILP].max() + 1
                lock += m * ILP; steps += m
    print(f"ILP {ILP}: tree-steps/wave {lock/(R//64):.0f}, loop passes/wave {steps/(R//64):.0f}")
