"""C++ split driver over its RCCL transport at world size 1: phase marks of a few steps
(forced exchange and solo).  usage: python tools/split_store_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from difacto_amd import data as D  # noqa: E402
from difacto_amd import dist as DI  # noqa: E402
from difacto_amd import hotpath as H  # noqa: E402

for force in (True, False):
    for pipelined in (True, False):
        ctx = H.Context(0, max_keys=1 << 18, push_agg="sum", V_dim=16, V_threshold=0, l1=0)
        sh = DI.Shard(ctx, 1)
        st = DI.SplitStore([sh], pipelined=pipelined,
                           rccl=(0, 1, DI.SplitStore.rccl_ids(), force))
        st.set_marks([4, 5])
        for s in range(6):
            blk = D.synthetic(20000, 39, 1 << 20, seed=s)
            st.submit([H.DeviceRowBlock(ctx, blk)], H.kTraining, push_cnt=s == 0)
        st.flush()
        print("force", force, "pipelined", pipelined, st.take_marks(), H.progress(ctx),
              flush=True)
        st.close()
        ctx.close()
