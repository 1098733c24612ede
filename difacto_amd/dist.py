"""Key-range-sharded model store over N GPUs: KVStoreDist (src/store/kvstore_dist.h) as one
process per GPU exchanging keys, pulled records and gradient records with all-to-all-v
collectives (torch.distributed: RCCL over xGMI on GPUs, gloo on CPU).

Every rank is a worker (its own minibatch, SGDLearner::IterateData's executor,
src/sgd/sgd_learner.cc:201-317) and the server of the keys k with floor(k * N / 2^64) ==
rank; keys are nibble-reversed feature ids, so ranges are balanced.  A step is bulk
synchronous — every pull is answered before any push, pushes are applied in worker-rank
order — which is the deterministic schedule of the reference's (unimplemented) sync_mode;
each server applies one Update per pushing worker like HandlePush (kvstore_dist.h:158-165).

The device phases are the C-ABI's dfx_dist_* calls (include/difacto_amd.h); this module is
only the orchestration between them.  ``Comm`` abstracts the exchange so the same step runs
over torch.distributed (one shard per process) or, for single-GPU tests, over N shards held
by one process (``LoopbackComm``).
"""
import ctypes

import torch

from . import _lib
from ._lib import check
from .hotpath import MAX_INDEX, kTraining, _p


def owner_of(keys_u64, nranks):
    """host restatement of the owner rule for numpy uint64 keys (tests, tools)"""
    import numpy as np
    k = np.asarray(keys_u64, dtype=np.uint64)
    hi = (k >> np.uint64(32)).astype(np.uint64)
    lo = (k & np.uint64(0xFFFFFFFF)).astype(np.uint64)
    n = np.uint64(nranks)
    # floor(k * n / 2^64) = floor((hi * n + floor(lo * n / 2^32)) / 2^32)
    return ((hi * n + ((lo * n) >> np.uint64(32))) >> np.uint64(32)).astype(np.int64)


class Shard:
    """One rank's device context in the sharded store: worker and key-range server."""

    def __init__(self, ctx, nranks):
        self.ctx = ctx
        self.nranks = int(nranks)
        self.S = _lib.lib().dfx_dist_record_floats(ctx.h)
        self._U = 0
        self._R = 0

    # worker ---------------------------------------------------------------------------------
    def localize(self, dblk, want_cnt, max_index=MAX_INDEX):
        ctx = self.ctx
        n = max(dblk.nnz, 1)
        keys = torch.empty(n, dtype=torch.int64, device=ctx.device)
        cnt = torch.empty(n, dtype=torch.float32, device=ctx.device) if want_cnt else None
        splits = (ctypes.c_int64 * self.nranks)()
        U = ctypes.c_int64(0)
        b = dblk.as_batch()
        check(_lib.lib().dfx_dist_localize(ctx.h, ctypes.byref(b), ctypes.c_uint64(max_index),
                                           self.nranks, _p(keys), _p(cnt), splits,
                                           ctypes.byref(U)))
        self._U = U.value
        return keys[:self._U], (cnt[:self._U] if want_cnt else None), list(splits)

    def fwd_bwd(self, dblk, pulled, job_type, pred=None):
        ctx = self.ctx
        grads = None
        if job_type == kTraining:
            grads = torch.empty(max(self._U * self.S, 1), dtype=torch.float32, device=ctx.device)
        b = dblk.as_batch()
        check(_lib.lib().dfx_dist_fwd_bwd(ctx.h, ctypes.byref(b), _p(pulled), int(job_type),
                                          _p(grads), _p(pred)))
        return None if grads is None else grads[:self._U * self.S]

    # server ---------------------------------------------------------------------------------
    def owner_begin(self, recv_keys, recv_splits, recv_cnt=None):
        offs = [0]
        for s in recv_splits:
            offs.append(offs[-1] + int(s))
        self._R = offs[-1]
        arr = (ctypes.c_int64 * len(offs))(*offs)
        check(_lib.lib().dfx_dist_owner_begin(self.ctx.h, _p(recv_keys), arr, self.nranks,
                                              _p(recv_cnt)))

    def owner_pull(self):
        vals = torch.empty(max(self._R * self.S, 1), dtype=torch.float32, device=self.ctx.device)
        check(_lib.lib().dfx_dist_owner_pull(self.ctx.h, _p(vals)))
        return vals[:self._R * self.S]

    def owner_push(self, recv_grads):
        check(_lib.lib().dfx_dist_owner_push(self.ctx.h, _p(recv_grads)))


class TorchComm:
    """Exchange over torch.distributed; this process holds one shard (its rank).

    device: where the count exchange lives (the GPU for nccl/RCCL, cpu for gloo).
    stage_cpu: route device tensors through host memory (gloo between processes that share
    one GPU — the single-GPU test box; RCCL needs one GPU per rank)."""

    def __init__(self, group=None, device=None, stage_cpu=False):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.device = device
        self.stage_cpu = stage_cpu

    def exchange_counts(self, send_splits):
        (s,) = send_splits
        t = torch.tensor(s, dtype=torch.int64, device=self.device)
        out = torch.empty_like(t)
        self.dist.all_to_all_single(out, t, group=self.group)
        return [out.tolist()]

    def alltoallv(self, tensors, send_splits, recv_splits, row=1):
        (x,), (ss,), (rs,) = tensors, send_splits, recv_splits
        home = x.device
        x = x[:sum(ss) * row]
        if self.stage_cpu:
            x = x.cpu()
        out = torch.empty(sum(rs) * row, dtype=x.dtype, device=x.device)
        self.dist.all_to_all_single(out, x.contiguous(),
                                    output_split_sizes=[int(r) * row for r in rs],
                                    input_split_sizes=[int(s) * row for s in ss],
                                    group=self.group)
        return [out.to(home) if self.stage_cpu else out]

    def allreduce_sum(self, values):
        (v,) = values
        t = torch.tensor(v, dtype=torch.float64, device=self.device)
        self.dist.all_reduce(t, group=self.group)
        return [t.tolist()]


class LoopbackComm:
    """N shards held by one process (tests on one GPU); the exchange is a device copy."""

    def __init__(self, world):
        self.world = int(world)

    def exchange_counts(self, send_splits):
        return [[send_splits[r][g] for r in range(self.world)] for g in range(self.world)]

    def alltoallv(self, tensors, send_splits, recv_splits, row=1):
        offs = []
        for r in range(self.world):
            o = [0]
            for s in send_splits[r]:
                o.append(o[-1] + int(s) * row)
            offs.append(o)
        out = []
        for g in range(self.world):
            parts = [tensors[r][offs[r][g]:offs[r][g + 1]] for r in range(self.world)]
            out.append(torch.cat(parts) if parts else tensors[g][:0])
        return out

    def allreduce_sum(self, values):
        tot = [sum(v[i] for v in values) for i in range(len(values[0]))]
        return [list(tot) for _ in values]


PHASES = ("localize", "xchg_keys", "owner_begin", "owner_pull", "xchg_pull", "fwd_bwd",
          "xchg_grads", "owner_push")


def sharded_step(shards, dblks, comm, job_type=kTraining, push_cnt=False, max_index=MAX_INDEX,
                 preds=None, mark=None):
    """One synchronous step of the sharded store.  shards / dblks (/ preds): this process's
    shards and their batches (one each under torch.distributed, N under LoopbackComm).
    push_cnt: epoch-0 Update(kFeaCount) (sgd_learner.cc:272, 304-307); ignored when V_dim == 0
    like the reference's do_embedding_.  mark(i): called after phase PHASES[i] is issued
    (and with -1 first), e.g. to record stream events."""
    mark = mark or (lambda i: None)
    mark(-1)
    n = len(shards)
    want_cnt = bool(push_cnt) and shards[0].ctx.V_dim > 0
    loc = [shards[i].localize(dblks[i], want_cnt, max_index) for i in range(n)]
    mark(0)
    send = [l[2] for l in loc]
    recv = comm.exchange_counts(send)
    rkeys = comm.alltoallv([l[0] for l in loc], send, recv)
    rcnt = comm.alltoallv([l[1] for l in loc], send, recv) if want_cnt else [None] * n
    mark(1)
    for i in range(n):
        shards[i].owner_begin(rkeys[i], recv[i], rcnt[i])
    mark(2)
    S = shards[0].S
    vals = [s.owner_pull() for s in shards]
    mark(3)
    pulled = comm.alltoallv(vals, recv, send, S)
    mark(4)
    grads = [shards[i].fwd_bwd(dblks[i], pulled[i], job_type, preds[i] if preds else None)
             for i in range(n)]
    mark(5)
    if job_type == kTraining:
        rgrads = comm.alltoallv(grads, send, recv, S)
        mark(6)
        for i in range(n):
            shards[i].owner_push(rgrads[i])
    else:
        mark(6)
    mark(7)
    return [sum(s) for s in recv]  # keys served per shard (for accounting)
