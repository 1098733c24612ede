"""CPU restatement of the key-range-sharded store step (KVStoreDist), built from the oracle.

TEST INFRASTRUCTURE ONLY (see oracle.py).  N SGDUpdater restatements play the N servers of
src/store/kvstore_dist.h: server g owns the keys with floor(key * N / 2^64) == g and applies
every worker push as one Update call (HandlePush, kvstore_dist.h:158-165) and answers pulls
with Get (HandlePull, :167-175).  Each worker runs SGDLearner::IterateData's executor
(src/sgd/sgd_learner.cc:272-317) on its own batch: Localizer::Compact, the epoch-0 kFeaCount
push (waited on, :304-307), Pull, Predict, Evaluate, AUC, CalcGrad, Push.
ShardedOracle.step is bulk synchronous with pushes applied in worker-rank order: all count
pushes, then all pulls, then all gradient pushes (push_agg=ranks).  AggOracle is the
push_agg=sum semantics (one Update per key on the workers' summed gradients: one reference
step over the concatenated batches).  StaleOracle is the pipelined (1-step-stale) schedule of
either.
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

    # the step in phases: the bulk-synchronous step runs them in order; the pipelined
    # (1-step-stale) schedule runs begin(t+1), pull(t+1) before push(t) (StaleOracle)
    def begin(self, blocks, push_cnt=False, max_index=(1 << 64) - 1):
        """every worker's Localizer::Compact, then the kFeaCount pushes (server order: for each
        server, the workers in rank order)"""
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
        return {"blocks": blocks, "loc": loc}

    def pull(self, st):
        N, d = self.N, self.d
        pulled = []
        for r in range(N):
            uniq, _, _, bd = st["loc"][r]
            vs, ls = [], []
            for g in range(N):
                if bd[g + 1] > bd[g]:
                    v, l = self.up[g].get(uniq[bd[g]:bd[g + 1]])
                    vs.append(v)
                    ls.append(l)
            vals = np.concatenate(vs) if vs else np.zeros(0, np.float32)
            lens = (np.concatenate(ls) if ls else np.zeros(0, np.int32)) if d > 0 else None
            pulled.append((vals, lens))
        st["pulled"] = pulled

    def compute(self, st, train=True):
        """every worker's Predict / Evaluate / AUC (/ CalcGrad) on its pulled values"""
        d = self.d
        out, grads = [], []
        for r in range(self.N):
            blk = st["blocks"][r]
            uniq, _, col, _ = st["loc"][r]
            vals, lens = st["pulled"][r]
            wp, vp = O.get_pos(lens) if d > 0 else (None, None)
            pred = O.fm_predict(blk.offs, col, blk.vals, vals, wp, vp, d)
            out.append((O.evaluate(blk.labels, pred), O.auc(blk.labels, pred), pred))
            if train:
                grads.append(O.fm_calcgrad(blk.offs, col, blk.vals, blk.labels, blk.weights, vals,
                                           wp, vp, len(uniq), d, pred))
        st["grads"] = grads if train else None
        return out

    def push(self, st):
        """the kGradient pushes: for each server, the workers in rank order"""
        N = self.N
        for g in range(N):
            for r in range(N):
                uniq, _, _, bd = st["loc"][r]
                if bd[g + 1] == bd[g]:
                    continue
                lens = st["pulled"][r][1]
                vb = value_bounds(lens, bd)
                self.up[g].update(uniq[bd[g]:bd[g + 1]], O.Updater.kGradient,
                                  st["grads"][r][vb[g]:vb[g + 1]],
                                  None if lens is None else lens[bd[g]:bd[g + 1]])

    def step(self, blocks, push_cnt=False, train=True, max_index=(1 << 64) - 1):
        """blocks: one data.RowBlock per worker.  -> [(loss, auc*n, pred)] per worker"""
        st = self.begin(blocks, push_cnt, max_index)
        self.pull(st)
        out = self.compute(st, train)
        if train:
            self.push(st)
        return out

    def owner(self, key):
        return int(owner_of(np.array([key], np.uint64), self.N)[0])

    def entry(self, key):
        return self.up[self.owner(key)].entry(key)


class AggOracle:
    """push_agg=sum (SURVEY.md §8(e)'s synchronous semantics): a step over N workers is one
    reference step over the concatenation of their batches.  The N servers together hold
    exactly one SGDUpdater's model (a key's state lives on its owner, and InitV draws are
    ranked over all owners in key order, so one rand_r stream serves them all); this oracle
    therefore keeps one Updater:
      begin   every worker's Localizer::Compact; a count push adds, per key of the union, the
              workers' counts (= the concatenated batch's Localizer count), in key order
      pull    every worker's Get of its own keys from the same state
      push    per key of the union the workers' gradients summed in rank order (float32, the
              order the owner adds the received records), then ONE Update in key order
    Same interface as ShardedOracle (begin / pull / compute / push / step / entry)."""

    def __init__(self, nranks, **kw):
        self.N = int(nranks)
        self.one = O.Updater(**kw)
        self.up = [self.one]
        self.d = self.one.V_dim

    def begin(self, blocks, push_cnt=False, max_index=(1 << 64) - 1):
        d = self.d
        assert len(blocks) == self.N
        loc = []
        for blk in blocks:
            uniq, cnt, col = O.localize(blk.offs, blk.ids, max_index, want_cnt=True)
            loc.append((uniq, cnt, col, owner_bounds(uniq, self.N)))
        if push_cnt and d > 0:
            keys, cnts = self._union([l[0] for l in loc], [l[1] for l in loc], 1)
            if len(keys):
                self.one.update(keys, O.Updater.kFeaCount, cnts)
        return {"blocks": blocks, "loc": loc}

    @staticmethod
    def _union(keys, rows, width):
        """union of the workers' sorted keys and their rows of `width` floats summed in rank
        order (float32 adds, starting from the first worker's row)"""
        allk = np.concatenate(keys) if keys else np.zeros(0, np.uint64)
        uk = np.unique(allk)
        acc = np.zeros((len(uk), width), np.float32)
        seen = np.zeros(len(uk), bool)
        for k, r in zip(keys, rows):
            if len(k) == 0:
                continue
            idx = np.searchsorted(uk, k)
            r = np.asarray(r, np.float32).reshape(len(k), width)
            first = ~seen[idx]
            acc[idx[first]] = r[first]
            acc[idx[~first]] = (acc[idx[~first]] + r[~first]).astype(np.float32)
            seen[idx] = True
        return uk, acc.reshape(-1) if width == 1 else acc

    def pull(self, st):
        st["pulled"] = [self.one.get(l[0]) for l in st["loc"]]

    compute = ShardedOracle.compute

    def push(self, st):
        d = self.d
        keys, rows, lens_u = [], [], None
        for r in range(self.N):
            uniq = st["loc"][r][0]
            vals, lens = st["pulled"][r]
            g = st["grads"][r]
            # each key's gradient as a full [gw | gV(d)] row (gV zero unless V was pulled)
            full = np.zeros((len(uniq), 1 + d), np.float32)
            if d > 0:
                wp, vp = O.get_pos(lens)
                full[:, 0] = g[wp]
                live = lens > 1
                if np.any(live):
                    full[live, 1:] = g[vp[live][:, None] + np.arange(d)]
            else:
                full[:, 0] = g
            keys.append(uniq)
            rows.append(full)
        uk, acc = self._union(keys, rows, 1 + d)
        if len(uk) == 0:
            return
        if d == 0:  # acc is one float per key
            self.one.update(uk, O.Updater.kGradient, acc)
            return
        # lens of the union keys: what the workers pulled (every worker pulled the same state)
        lens_u = np.ones(len(uk), np.int32)
        for r in range(self.N):
            uniq = st["loc"][r][0]
            lens = st["pulled"][r][1]
            lens_u[np.searchsorted(uk, uniq)] = lens
        parts = []
        for i in range(len(uk)):
            parts.append(acc[i] if lens_u[i] > 1 else acc[i, :1])
        self.one.update(uk, O.Updater.kGradient, np.concatenate(parts), lens_u)

    step = ShardedOracle.step

    def entry(self, key):
        return self.one.entry(key)


class StaleOracle:
    """The pipelined schedule of the sharded store (difacto_amd.dist.ShardedPipeline): step
    t+1's count pushes and pulls are answered before step t's gradient pushes are applied,
    i.e. every pull is at most one step stale.  This is one of the schedules the reference's
    asynchronous KVStoreDist allows with two batches in flight per worker
    (sgd_learner.cc:310-312, kvstore_dist.h:137-150), made deterministic:
        begin(t), pull(t), push(t-1), compute(t), ..., push(T-1) at flush()."""

    def __init__(self, nranks, agg="ranks", **kw):
        self.so = AggOracle(nranks, **kw) if agg == "sum" else ShardedOracle(nranks, **kw)
        self.N, self.up, self.d = self.so.N, self.so.up, self.so.d
        self.pending = None

    def submit(self, blocks, push_cnt=False, train=True, max_index=(1 << 64) - 1):
        st = self.so.begin(blocks, push_cnt, max_index)
        self.so.pull(st)
        self.flush()
        out = self.so.compute(st, train)
        if train:
            self.pending = st
        return out

    def flush(self):
        if self.pending is not None:
            self.so.push(self.pending)
            self.pending = None

    def entry(self, key):
        return self.so.entry(key)



class SplitStaleOracle:
    """The split store's 1-step-stale schedule (GpuSplitStore pipelined = 2, dist.SplitStore
    stale=True) on push_agg=sum: on every GPU the owner forward of step t+1
    runs before the backward of step t, so step t's exchanges travel beside the other step's
    compute.  Per step:
        begin(t+1)            count push, as AggOracle (before step t's update)
        forward(t+1)          predictions from the model after update t-1 (one step stale)
        update(t)             step t's gradient: p and XV_ from its (stale) forward, the
                              gradient's layout and the diag(XXp) V term from the model as it
                              is now (the owner's backward reads V when it runs), summed over
                              the workers per key and applied once (oracle.fm_calcgrad_stale)
    flush() applies the last pending update.  Deterministic; one of the schedules the
    reference's asynchronous KVStoreDist allows with two batches in flight per worker
    (sgd_learner.cc:310-312, kvstore_dist.h:137-150), with the server's current V in the
    gradient's V term instead of the worker's pulled copy."""

    def __init__(self, nranks, **kw):
        self.so = AggOracle(nranks, **kw)
        self.N, self.one, self.d = self.so.N, self.so.one, self.so.d
        self.up = self.so.up
        self.pending = None

    def submit(self, blocks, push_cnt=False, train=True, max_index=(1 << 64) - 1):
        st = self.so.begin(blocks, push_cnt, max_index)
        self.so.pull(st)
        out = []
        for r in range(self.N):
            blk = st["blocks"][r]
            uniq, _, col, _ = st["loc"][r]
            vals, lens = st["pulled"][r]
            wp, vp = O.get_pos(lens) if self.d > 0 else (None, None)
            pred = O.fm_predict(blk.offs, col, blk.vals, vals, wp, vp, self.d)
            out.append((O.evaluate(blk.labels, pred), O.auc(blk.labels, pred), pred))
        st["preds"] = [o[2] for o in out]
        self.flush()
        if train:
            self.pending = st
        return out

    def flush(self):
        st, self.pending = self.pending, None
        if st is None:
            return
        d = self.d
        grads, now = [], []
        for r in range(self.N):
            blk = st["blocks"][r]
            uniq, _, col, _ = st["loc"][r]
            fv, fl = st["pulled"][r]
            bv, bl = self.one.get(uniq)  # the model as the backward reads it
            if d > 0:
                _, fvp = O.get_pos(fl)
                bwp, bvp = O.get_pos(bl)
            else:
                fvp = bwp = bvp = None
            grads.append(O.fm_calcgrad_stale(blk.offs, col, blk.vals, blk.labels, blk.weights,
                                             fv, fvp, bv, bwp, bvp, len(uniq), d,
                                             st["preds"][r]))
            now.append((bv, bl if d > 0 else None))
        st["pulled"], st["grads"] = now, grads
        self.so.push(st)

    def entry(self, key):
        return self.so.entry(key)
