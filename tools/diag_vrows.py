"""Diagnostic: model statistics of the fused path (optionally vs the oracle).

usage: diag_vrows.py KEY_BITS ROWS STEPS [oracle]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401
from difacto_amd import data as D  # noqa: E402
from difacto_amd import hotpath as H  # noqa: E402

kb = int(sys.argv[1]) if len(sys.argv) > 1 else 20
B = int(sys.argv[2]) if len(sys.argv) > 2 else 50000
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 8
use_oracle = len(sys.argv) > 4
cfg = dict(V_dim=16, V_threshold=0, l1=0, lr=.1, V_lr=.01)
c = H.Context(0, max_keys=1 << kb, max_vrows=1 << kb, **cfg)
st = H.Store(c)
up = None
if use_oracle:
    from oracle import oracle as O
    up = O.Updater(**cfg)
for step in range(steps):
    blk = D.synthetic(B, 39, 1 << kb, seed=500 + step)
    pc = step < steps - 2
    H.train_step(c, H.DeviceRowBlock(c, blk), H.kTraining, push_cnt=pc)
    p = H.progress(c)
    s = st.stats()
    msg = "%d loss %.4f keys %d vrows %d seed %d" % (step, p["loss"], s["n_keys"], s["n_vrows"],
                                                     s["seed"])
    if up is not None:
        loss, auc = up.train_step(blk.offs, blk.ids, blk.vals, blk.labels, push_cnt=pc)
        msg += " | oracle loss %.4f keys %d seed %d" % (loss, up.size(), up.seed)
    print(msg, flush=True)
