"""CPU test double of difacto_amd.dist.Shard built from the oracle, so the sharded step's
orchestration (difacto_amd.dist.sharded_step over TorchComm / gloo) runs with world_size > 1
in this container.  It speaks the same record layout as the C-ABI (include/difacto_amd.h):
pulled records [V(d) | w | live | 0 | 0], gradient records [gV(d) | gw | live | 0 | 0]."""
from types import SimpleNamespace

import numpy as np
import torch

from oracle import oracle as O
from oracle.dist_oracle import owner_bounds

kTraining = 3


class CpuShard:
    def __init__(self, nranks, **kw):
        self.nranks = int(nranks)
        self.up = O.Updater(**kw)
        self.d = self.up.V_dim
        self.S = self.d + 4
        self.ctx = SimpleNamespace(V_dim=self.d)
        self.agg_sum = False  # the mock serves push_agg=ranks (one Update per pushing worker)
        self.losses, self.aucs = [], []
        self.wslot = [None, None]
        self.oslot = [{}, {}]

    # worker (per step slot, like the device Shard)
    def localize(self, blk, want_cnt, slot=0, max_index=(1 << 64) - 1):
        uniq, cnt, col = O.localize(blk.offs, blk.ids, max_index)
        splits = [int(s) for s in np.diff(owner_bounds(uniq, self.nranks))]
        keys = torch.from_numpy(uniq.view(np.int64).copy())
        self.wslot[slot] = (uniq, col, (keys, torch.from_numpy(cnt.copy()) if want_cnt else None,
                                        splits))

    def localize_wait(self, slot=0):
        return self.wslot[slot][2]

    def fwd_bwd(self, blk, pulled, job_type, slot=0, pred=None):
        d, S = self.d, self.S
        uniq, col = self.wslot[slot][:2]
        U = len(uniq)
        rec = pulled.numpy().reshape(U, S)
        live = rec[:, d + 1] != 0 if d > 0 else np.zeros(U, bool)
        lens = (1 + d * live).astype(np.int32)
        vals = np.concatenate([np.concatenate([[rec[u, d]], rec[u, :d]]) if live[u]
                               else rec[u, d:d + 1] for u in range(U)]).astype(np.float32) \
            if U else np.zeros(0, np.float32)
        wp, vp = O.get_pos(lens) if d > 0 else (None, None)
        p = O.fm_predict(blk.offs, col, blk.vals, vals, wp, vp, d)
        self.losses.append(O.evaluate(blk.labels, p))
        self.aucs.append(O.auc(blk.labels, p))
        if pred is not None:
            pred.copy_(torch.from_numpy(p))
        if job_type != kTraining:
            return None
        g = O.fm_calcgrad(blk.offs, col, blk.vals, blk.labels, blk.weights, vals, wp, vp, U, d,
                          p)
        out = np.zeros((U, S), np.float32)
        for u in range(U):
            q = wp[u] if d > 0 else u
            out[u, d] = g[q]
            if live[u]:
                out[u, :d] = g[vp[u]:vp[u] + d]
                out[u, d + 1] = 1.0
        return torch.from_numpy(out.ravel())

    # server
    def owner_begin(self, recv_keys, recv_splits, recv_cnt=None, slot=0):
        keys = recv_keys.numpy().view(np.uint64)
        offs = np.concatenate([[0], np.cumsum(recv_splits)]).astype(np.int64)
        o = self.oslot[slot]
        o["rkeys"] = [keys[offs[r]:offs[r + 1]] for r in range(self.nranks)]
        o["roffs"] = offs
        if recv_cnt is not None:
            cnt = recv_cnt.numpy()
            for r in range(self.nranks):
                if offs[r + 1] > offs[r]:
                    self.up.update(o["rkeys"][r], O.Updater.kFeaCount, cnt[offs[r]:offs[r + 1]])

    def owner_pull(self, slot=0):
        d, S = self.d, self.S
        o = self.oslot[slot]
        R = int(o["roffs"][-1])
        rec = np.zeros((R, S), np.float32)
        o["rlive"] = []
        for r, keys in enumerate(o["rkeys"]):
            live = np.zeros(len(keys), bool)
            if len(keys):
                v, l = self.up.get(keys)
                p = 0
                for i in range(len(keys)):
                    row = o["roffs"][r] + i
                    rec[row, d] = v[p]
                    if d > 0 and l[i] > 1:
                        rec[row, :d] = v[p + 1:p + 1 + d]
                        rec[row, d + 1] = 1.0
                        live[i] = True
                        p += 1 + d
                    else:
                        p += 1
            o["rlive"].append(live)
        return torch.from_numpy(rec.ravel())

    def owner_push(self, recv_grads, slot=0):
        d, S = self.d, self.S
        o = self.oslot[slot]
        rec = recv_grads.numpy().reshape(-1, S)
        for r, keys in enumerate(o["rkeys"]):
            if not len(keys):
                continue
            rows = rec[o["roffs"][r]:o["roffs"][r + 1]]
            live = rows[:, d + 1] != 0 if d > 0 else np.zeros(len(keys), bool)
            assert np.array_equal(live, o["rlive"][r])  # the push carries what was pulled
            vals = np.concatenate([np.concatenate([[rows[i, d]], rows[i, :d]]) if live[i]
                                   else rows[i, d:d + 1] for i in range(len(keys))])
            lens = (1 + d * live).astype(np.int32) if d > 0 else None
            self.up.update(keys, O.Updater.kGradient, vals.astype(np.float32), lens)
