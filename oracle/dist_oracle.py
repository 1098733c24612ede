"""CPU restatement of the key-range-sharded store step (KVStoreDist), built from the oracle.

TEST INFRASTRUCTURE ONLY (see oracle.py).  N SGDUpdater restatements play the N servers of
src/store/kvstore_dist.h: server g owns the keys with floor(key * N / 2^64) == g and applies
every worker push as one Update call (HandlePush, kvstore_dist.h:158-165) and answers pulls
with Get (HandlePull, :167-175).  Each worker runs SGDLearner::IterateData's executor
(src/sgd/sgd_learner.cc:272-317) on its own batch: Localizer::Compact, the epoch-0 kFeaCount
push (waited on, :304-307), Pull, Predict, Evaluate, AUC, CalcGrad, Push.  The schedule is
bulk synchronous with pushes applied in worker-rank order: all count pushes, then all pulls,
then all gradient pushes.
"""
import numpy as np

from . import oracle as O


def owner_of(keys, nranks):
    k = np.asarray(keys, dtype=np.uint64)
    hi = k >> np.uint64(32)
    lo = k & np.uint64(0xFFFFFFFF)
    n = np.uint64(nranks)
    return ((hi * n + ((lo * n) >> np.uint64(32))) >> np.uint64(32)).astype(np.int64)


def owner_bounds(uniq, nranks):
    """sorted unique keys -> [N+1] boundaries of each owner's contiguous range"""
    return np.searchsorted(owner_of(uniq, nranks), np.arange(nranks + 1)).astype(np.int64)


def value_bounds(lens, bounds):
    """value offsets (pull/push layout) of key boundaries"""
    if lens is None:
        return bounds.copy()
    cum = np.concatenate([[0], np.cumsum(lens, dtype=np.int64)])
    return cum[bounds]


class ShardedOracle:
    def __init__(self, nranks, **kw):
        self.N = int(nranks)
        self.up = [O.Updater(**kw) for _ in range(self.N)]
        self.d = self.up[0].V_dim

    def step(self, blocks, push_cnt=False, train=True, max_index=(1 << 64) - 1):
        """blocks: one data.RowBlock per worker.  -> [(loss, auc*n, pred)] per worker"""
        N, d = self.N, self.d
        assert len(blocks) == N
        loc = []
        for blk in blocks:
            uniq, cnt, col = O.localize(blk.offs, blk.ids, max_index, want_cnt=True)
            loc.append((uniq, cnt, col, owner_bounds(uniq, N)))
        if push_cnt and d > 0:
            for g in range(N):
                for r in range(N):
                    uniq, cnt, _, bd = loc[r]
                    if bd[g + 1] > bd[g]:
                        self.up[g].update(uniq[bd[g]:bd[g + 1]], O.Updater.kFeaCount,
                                          cnt[bd[g]:bd[g + 1]])
        pulled = []
        for r in range(N):
            uniq, _, _, bd = loc[r]
            vs, ls = [], []
            for g in range(N):
                if bd[g + 1] > bd[g]:
                    v, l = self.up[g].get(uniq[bd[g]:bd[g + 1]])
                    vs.append(v)
                    ls.append(l)
            vals = np.concatenate(vs) if vs else np.zeros(0, np.float32)
            lens = (np.concatenate(ls) if ls else np.zeros(0, np.int32)) if d > 0 else None
            pulled.append((vals, lens))
        out, grads = [], []
        for r in range(N):
            blk = blocks[r]
            uniq, _, col, _ = loc[r]
            vals, lens = pulled[r]
            wp, vp = O.get_pos(lens) if d > 0 else (None, None)
            pred = O.fm_predict(blk.offs, col, blk.vals, vals, wp, vp, d)
            loss = O.evaluate(blk.labels, pred)
            a = O.auc(blk.labels, pred)
            out.append((loss, a, pred))
            if train:
                grads.append(O.fm_calcgrad(blk.offs, col, blk.vals, blk.labels, blk.weights, vals,
                                           wp, vp, len(uniq), d, pred))
        if train:
            for g in range(N):
                for r in range(N):
                    uniq, _, _, bd = loc[r]
                    if bd[g + 1] == bd[g]:
                        continue
                    lens = pulled[r][1]
                    vb = value_bounds(lens, bd)
                    self.up[g].update(uniq[bd[g]:bd[g + 1]], O.Updater.kGradient,
                                      grads[r][vb[g]:vb[g + 1]],
                                      None if lens is None else lens[bd[g]:bd[g + 1]])
        return out

    def owner(self, key):
        return int(owner_of(np.array([key], np.uint64), self.N)[0])

    def entry(self, key):
        return self.up[self.owner(key)].entry(key)
