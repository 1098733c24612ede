"""Key-range-sharded model store over N GPUs: KVStoreDist (src/store/kvstore_dist.h) as one
process per GPU exchanging keys, pulled records and gradient records with all-to-all-v
collectives (torch.distributed: RCCL over xGMI on GPUs, gloo on CPU).

Every rank is a worker (its own minibatch, SGDLearner::IterateData's executor,
src/sgd/sgd_learner.cc:201-317) and the server of the keys k with floor(k * N / 2^64) ==
rank; keys are nibble-reversed feature ids, so ranges are balanced.  A step is bulk
synchronous — every pull is answered before any push — which is the deterministic schedule
of the reference's (unimplemented) sync_mode.  With push_agg=sum (the default) a step is one
reference step over the concatenation of the workers' batches: one Update
per key on the summed gradient; with push_agg=ranks each server applies one Update per
pushing worker in rank order like HandlePush (kvstore_dist.h:158-165).

The device phases are the C-ABI's dfx_dist_* calls (include/difacto_amd.h); this module is
only the orchestration between them.  ``Comm`` abstracts the exchange so the same step runs
over torch.distributed (one shard per process) or, for single-GPU tests, over N shards held
by one process (``LoopbackComm``).
"""
import ctypes
import time

import torch

from . import _lib
from ._lib import check
from .hotpath import MAX_INDEX, kTraining, kValidation, _p  # noqa: F401


def owner_of(keys_u64, nranks):
    """host restatement of the owner rule for numpy uint64 keys (tests, tools)"""
    import numpy as np
    k = np.asarray(keys_u64, dtype=np.uint64)
    hi = (k >> np.uint64(32)).astype(np.uint64)
    lo = (k & np.uint64(0xFFFFFFFF)).astype(np.uint64)
    n = np.uint64(nranks)
    # floor(k * n / 2^64) = floor((hi * n + floor(lo * n / 2^32)) / 2^32)
    return ((hi * n + ((lo * n) >> np.uint64(32))) >> np.uint64(32)).astype(np.int64)


def model_name(prefix, rank, it=-1):
    """SGDLearner::ModelName (sgd_learner.h:65-69): every server saves / loads its own part"""
    name = str(prefix)
    if it >= 0:
        name += "_iter-%d" % it
    return name + "_part-%d" % rank


class Shard:
    """One rank's device context in the sharded store: worker and key-range server.  Every
    call takes the step slot (0 or 1) whose buffers it uses; two steps can be in flight.
    The context's push_agg kwarg picks the update semantics (include/difacto_amd.h): sum (one
    Update per key on the workers' summed gradients, InitV ranked over all owners) or ranks
    (one Update per pushing worker, KVStoreDist's HandlePush)."""

    def __init__(self, ctx, nranks):
        self.ctx = ctx
        self.nranks = int(nranks)
        self.S = _lib.lib().dfx_dist_record_floats(ctx.h)
        self.agg_sum = _lib.lib().dfx_dist_push_agg_sum(ctx.h) == 1
        self._U = [0, 0]
        self._R = [0, 0]
        # the Localizer lane writes these; they live until the slot's fwd_bwd
        self._keys = [None, None]
        self._cnt = [None, None]
        self._want_cnt = [False, False]
        self._split = [None, None]
        self._split_R = [0, 0]
        self._pstream = None

    def _slot_buffers(self, slot, n, want_cnt):
        dev = self.ctx.device
        grow = self._keys[slot] is None or self._keys[slot].numel() < n
        grow = grow or (want_cnt and (self._cnt[slot] is None or self._cnt[slot].numel() < n))
        if grow:
            if self._keys[slot] is not None and torch.device(dev).type == "cuda":
                torch.cuda.synchronize(dev)  # the old buffers may still be in use on a lane
            cap = max(n, 1) + max(n, 1) // 8
            self._keys[slot] = torch.empty(cap, dtype=torch.int64, device=dev)
            self._cnt[slot] = torch.empty(cap, dtype=torch.float32, device=dev)
        return self._keys[slot], (self._cnt[slot] if want_cnt else None)

    # worker ---------------------------------------------------------------------------------
    def localize(self, dblk, want_cnt, slot=0, max_index=MAX_INDEX):
        """issue Localizer::Compact of the batch on the Localizer lane (asynchronous)"""
        keys, cnt = self._slot_buffers(slot, dblk.nnz, want_cnt)
        self._want_cnt[slot] = want_cnt
        b = dblk.as_batch()
        check(_lib.lib().dfx_dist_localize(self.ctx.h, ctypes.byref(b),
                                           ctypes.c_uint64(max_index), self.nranks, slot,
                                           _p(keys), _p(cnt)))

    def localize_wait(self, slot=0):
        """-> (sorted unique keys, their counts or None, keys per owner rank)"""
        splits = (ctypes.c_int64 * self.nranks)()
        U = ctypes.c_int64(0)
        check(_lib.lib().dfx_dist_localize_wait(self.ctx.h, slot, self.nranks, splits,
                                                ctypes.byref(U)))
        self._U[slot] = U.value
        cnt = self._cnt[slot][:U.value] if self._want_cnt[slot] else None
        return self._keys[slot][:U.value], cnt, list(splits)

    def fwd_bwd(self, dblk, pulled, job_type, slot=0, pred=None):
        ctx = self.ctx
        U = self._U[slot]
        grads = None
        if job_type == kTraining:
            grads = torch.empty(max(U * self.S, 1), dtype=torch.float32, device=ctx.device)
        b = dblk.as_batch()
        check(_lib.lib().dfx_dist_fwd_bwd(ctx.h, slot, ctypes.byref(b), _p(pulled),
                                          int(job_type), _p(grads), _p(pred)))
        return None if grads is None else grads[:U * self.S]

    # server ---------------------------------------------------------------------------------
    def owner_begin(self, recv_keys, recv_splits, recv_cnt=None, slot=0):
        offs = [0]
        for s in recv_splits:
            offs.append(offs[-1] + int(s))
        self._R[slot] = offs[-1]
        arr = (ctypes.c_int64 * len(offs))(*offs)
        check(_lib.lib().dfx_dist_owner_begin(self.ctx.h, slot, _p(recv_keys), arr,
                                              self.nranks, _p(recv_cnt)))

    def owner_pull(self, slot=0):
        R = self._R[slot]
        vals = torch.empty(max(R * self.S, 1), dtype=torch.float32, device=self.ctx.device)
        check(_lib.lib().dfx_dist_owner_pull(self.ctx.h, slot, _p(vals)))
        return vals[:R * self.S]

    def owner_push(self, recv_grads, slot=0):
        check(_lib.lib().dfx_dist_owner_push(self.ctx.h, slot, _p(recv_grads)))

    # the literal north_star exchange (rsag_step) ------------------------------------------
    def union(self, runs, run_offs):
        """-> (sorted union of the runs, union position of every run item, owner bounds of the
        union (host list, nranks + 1))"""
        R = int(run_offs[-1])
        dev = self.ctx.device
        uni = torch.empty(max(R, 1), dtype=torch.int64, device=dev)
        upos = torch.empty(max(R, 1), dtype=torch.int32, device=dev)
        offs = (ctypes.c_int64 * len(run_offs))(*[int(o) for o in run_offs])
        bounds = (ctypes.c_int64 * (self.nranks + 1))()
        n = ctypes.c_int64(0)
        check(_lib.lib().dfx_dist_union(self.ctx.h, _p(runs), offs, len(run_offs) - 1,
                                        self.nranks, _p(uni), _p(upos), bounds,
                                        ctypes.byref(n)))
        return uni[:n.value], upos[:R], list(bounds)

    def union_rows(self, keys, upos, bounds, M, width, to_union, src, dst):
        bd = (ctypes.c_int64 * len(bounds))(*bounds)
        check(_lib.lib().dfx_dist_union_rows(self.ctx.h, _p(keys), _p(upos), keys.numel(), bd,
                                             self.nranks, int(M), int(width), int(to_union),
                                             _p(src), _p(dst)))

    # push_agg=sum: InitV ranked over all owners (after a count push and after every push)
    def initv_local(self, slot=0):
        """-> device int64[1]: this owner's InitV request count"""
        out = torch.empty(1, dtype=torch.int64, device=self.ctx.device)
        check(_lib.lib().dfx_dist_initv_local(self.ctx.h, slot, _p(out)))
        return out

    def initv_draw(self, counts_all, rank, slot=0):
        check(_lib.lib().dfx_dist_initv_draw(self.ctx.h, slot, _p(counts_all), int(rank),
                                             self.nranks))

    # owner-computes split (csrc/split.hip) ---------------------------------------------------
    def split_partition(self, dblk, slot=0, max_index=MAX_INDEX, want_x=False):
        """issue the partition of the batch's nnz by owner (asynchronous); values travel for
        valued data (want_x: binary data too, as 1s)"""
        dev = self.ctx.device
        b = dblk.as_batch()
        B, nnz = int(dblk.size), int(dblk.nnz)
        # the partition runs on a torch stream of its own and its outputs are allocated there,
        # so the allocator reuses them only behind it; readers on other streams are recorded by
        # the drivers
        if self._pstream is None and torch.device(dev).type == "cuda":
            self._pstream = torch.cuda.Stream(device=dev, priority=-1)
            check(_lib.lib().dfx_ctx_set_lane_stream(self.ctx.h, 2,
                                                     ctypes.c_void_p(self._pstream.cuda_stream)))
        with torch.cuda.stream(self._pstream):
            keys = torch.empty(max(nnz, 1), dtype=torch.int64, device=dev)
            x = (torch.empty(max(nnz, 1), dtype=torch.float32, device=dev)
                 if (b.value or want_x) else None)
            rc = torch.empty(max(self.nranks * B, 1), dtype=torch.int32, device=dev)
        check(_lib.lib().dfx_split_partition(self.ctx.h, slot, ctypes.byref(b),
                                             ctypes.c_uint64(max_index), self.nranks, _p(keys),
                                             _p(x), _p(rc)))
        self._split[slot] = (keys, x, rc, B)

    def split_partition_wait(self, slot=0):
        """-> (keys grouped by owner, their values or None, nnz per (owner, row) [N * B], keys
        per owner, B)"""
        splits = (ctypes.c_int64 * self.nranks)()
        check(_lib.lib().dfx_split_partition_wait(self.ctx.h, slot, self.nranks, splits))
        keys, x, rc, B = self._split[slot]
        return keys, x, rc[:self.nranks * B], list(splits), B

    def split_owner_begin(self, keys, x, row_cnt, rows_per_rank, keys_per_rank, job_type,
                          push_cnt, slot=0, lane=False):
        """row_cnt: the received per-row counts (scanned in place)"""
        rows = (ctypes.c_int64 * self.nranks)(*[int(v) for v in rows_per_rank])
        kpr = (ctypes.c_int64 * self.nranks)(*[int(v) for v in keys_per_rank])
        self._split_R[slot] = sum(int(v) for v in rows_per_rank)
        check(_lib.lib().dfx_split_owner_begin(self.ctx.h, slot, _p(keys), _p(x), _p(row_cnt),
                                               rows, kpr, self.nranks, int(job_type),
                                               int(bool(push_cnt)), int(bool(lane))))

    def split_owner_forward(self, slot=0):
        R = self._split_R[slot]
        PS = _lib.lib().dfx_split_part_floats(self.ctx.h, self.nranks)
        part = torch.empty(max(R * PS, 1), dtype=torch.float32, device=self.ctx.device)
        check(_lib.lib().dfx_split_owner_forward(self.ctx.h, slot, _p(part)))
        return part[:R * PS]

    def split_combine(self, dblk, parts, part_rows, slot=0, pred=None, pxv=None):
        """-> the batch's [XV*p | p | 0 0 0] rows (into pxv when given, part_rows rows)"""
        PX = _lib.lib().dfx_split_pxv_floats(self.ctx.h)
        if pxv is None:
            pxv = torch.zeros(max(int(part_rows) * PX, 1), dtype=torch.float32,
                              device=self.ctx.device)
        b = dblk.as_batch()
        check(_lib.lib().dfx_split_combine(self.ctx.h, slot, ctypes.byref(b), _p(parts),
                                           int(part_rows), self.nranks, _p(pxv), _p(pred)))
        return pxv

    def split_owner_backward(self, pxv, slot=0):
        check(_lib.lib().dfx_split_owner_backward(self.ctx.h, slot, _p(pxv)))

    def split_owner_stats(self, slot=0):
        """-> (rows, keys, unique keys) of the owner's last begin"""
        r, k, u = ctypes.c_int64(0), ctypes.c_int64(0), ctypes.c_int64(0)
        check(_lib.lib().dfx_split_owner_stats(self.ctx.h, slot, ctypes.byref(r),
                                               ctypes.byref(k), ctypes.byref(u)))
        return r.value, k.value, u.value

    def split_initv_local(self, slot=0):
        out = torch.empty(1, dtype=torch.int64, device=self.ctx.device)
        check(_lib.lib().dfx_split_initv_local(self.ctx.h, slot, _p(out)))
        return out

    def split_initv_draw(self, counts_all, rank, slot=0):
        check(_lib.lib().dfx_split_initv_draw(self.ctx.h, slot, _p(counts_all), int(rank),
                                              self.nranks))

    # model files (SGDLearner::SaveLoadModel, sgd_learner.cc:180-196) ---------------------------
    def save(self, prefix, rank, save_aux=False, it=-1):
        """this server's part, in SGDUpdater::Save's format (flush a pipeline first)"""
        self.ctx.sync()
        check(_lib.lib().dfx_store_save(self.ctx.h, model_name(prefix, rank, it).encode(),
                                        int(save_aux)))

    def load(self, prefix, rank, it=-1, saved_ranks=None):
        """this server's part.  saved_ranks (the number of servers that saved the model, when
        it differs from this run's): read every part and keep the keys this rank owns"""
        if saved_ranks is None or saved_ranks == self.nranks:
            check(_lib.lib().dfx_store_load(self.ctx.h, model_name(prefix, rank, it).encode()))
            return
        for r in range(int(saved_ranks)):
            check(_lib.lib().dfx_store_load_part(self.ctx.h, model_name(prefix, r, it).encode(),
                                                 int(rank), self.nranks))


class _Done:
    """an exchange that completed when it was issued"""

    def __init__(self, out):
        self.out = out

    def wait(self):
        return self.out


class TorchComm:
    """Exchange over torch.distributed; this process holds one shard (its rank).

    device: the shard's device (the count exchange always goes through host memory).
    stage_cpu: route device tensors through host memory (gloo between processes that share
    one GPU — the single-GPU test box; RCCL needs one GPU per rank).

    With the nccl (RCCL) backend the exchanges are asynchronous: records and gradients go
    over the default group, keys over a second communicator issued from an idle stream, so
    that step t+1's key exchange neither queues behind step t's gradient exchange nor waits
    for the compute stream; the split counts go over a gloo group on the host."""

    def __init__(self, group=None, device=None, stage_cpu=False, force_collectives=False,
                 comm_priority="high"):
        """force_collectives: run every exchange as a collective even at world size 1 (whose
        exchanges are otherwise the inputs themselves) — exercises the RCCL paths on one GPU.
        comm_priority: "high" runs RCCL's kernels on high-priority streams, like the
        Localizer lanes beside them: on normal-priority streams their blocks wait behind the
        lanes' for CU slots while the compute stream waits for the exchange"""
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.solo = self.world == 1 and not force_collectives
        self.rank = dist.get_rank(group)
        self.device = device
        self.stage_cpu = stage_cpu
        self.nccl = dist.get_backend(group) == "nccl"
        if self.nccl:
            ranks = list(range(self.world))
            opts = None
            if comm_priority == "high":
                opts = dist.ProcessGroupNCCL.Options()
                opts.is_high_priority_stream = True
                if group is None:
                    self.group = dist.new_group(ranks, backend="nccl", pg_options=opts)
            self.kgroup = dist.new_group(ranks, backend="nccl", pg_options=opts)
            self.cgroup = dist.new_group(ranks, backend="gloo")
            self.kstream = torch.cuda.Stream(device=device)
            # communicators up before the first grouped send/recv, which need not involve
            # every rank
            if self.world > 1:
                dist.barrier(group=self.group)
                dist.barrier(group=self.kgroup)
        else:
            self.kgroup = self.cgroup = group

    def ranks(self):
        return [self.rank]

    def exchange_counts(self, send_splits):
        """the split counts (a host round trip: the receivers size their buffers).  RCCL: one
        all-to-all of N int64 on the key communicator's idle stream, read back into host
        memory — no host-side (gloo / TCP) collective in the step; gloo: all_gather"""
        (s,) = send_splits
        if self.nccl and not self.solo:
            with torch.cuda.stream(self.kstream):
                t = torch.tensor(s, dtype=torch.int64, device=self.device)
                out = torch.empty(self.world, dtype=torch.int64, device=self.device)
                self.dist.all_to_all_single(out, t, group=self.kgroup)
                return [out.cpu().tolist()]
        t = torch.tensor(s, dtype=torch.int64)
        out = [torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t, group=self.cgroup)
        return [[int(o[self.rank]) for o in out]]

    def exchange_counts2(self, send):
        """send[0]: this rank's 2N ints [a_0 .. a_{N-1}, b_0 .. b_{N-1}] (a_g, b_g for peer g)
        -> [[a from every peer .., b from every peer ..]] (one host round trip)"""
        (s,) = send
        N = self.world
        pairs = [[int(s[g]), int(s[N + g])] for g in range(N)]
        if self.nccl and not self.solo:
            with torch.cuda.stream(self.kstream):
                t = torch.tensor(pairs, dtype=torch.int64, device=self.device).reshape(-1)
                out = torch.empty(2 * N, dtype=torch.int64, device=self.device)
                self.dist.all_to_all_single(out, t, group=self.kgroup)
                o = out.cpu().tolist()
        elif not self.solo:
            t = torch.tensor(pairs, dtype=torch.int64).reshape(-1)
            outs = [torch.empty_like(t) for _ in range(N)]
            self.dist.all_gather(outs, t, group=self.cgroup)
            o = []
            for g in range(N):
                o += outs[g].tolist()[2 * self.rank:2 * self.rank + 2]
        else:
            o = pairs[0]
        return [[o[2 * g] for g in range(N)] + [o[2 * g + 1] for g in range(N)]]

    def allgather_rows(self, tensors, M, row):
        """the north_star's all-gather: every rank's first rows (up to M rows of `row`
        elements, padded to M) -> [world * M * row], rank-major"""
        (x,) = tensors
        buf = torch.zeros(M * row, dtype=x.dtype, device=x.device)
        buf[:x.numel()] = x
        if self.solo:
            return [buf]
        if self.stage_cpu:
            out = [torch.empty(M * row, dtype=x.dtype) for _ in range(self.world)]
            self.dist.all_gather(out, buf.cpu(), group=self.group)
            return [torch.cat(out).to(x.device)]
        out = torch.empty(self.world * M * row, dtype=x.dtype, device=x.device)
        self.dist.all_gather_into_tensor(out, buf, group=self.group)
        return [out]

    def reduce_scatter_sum(self, tensors, M, row):
        """the north_star's reduce-scatter: every rank's [world * M * row] buffer summed, rank
        g receiving chunk g"""
        (x,) = tensors
        if self.solo:
            return [x]
        if self.stage_cpu:  # gloo has no reduce-scatter: all-reduce, keep this rank's chunk
            t = x.cpu()
            self.dist.all_reduce(t, group=self.group)
            c = M * row
            return [t[self.rank * c:(self.rank + 1) * c].to(x.device)]
        out = torch.empty(M * row, dtype=x.dtype, device=x.device)
        self.dist.reduce_scatter_tensor(out, x, group=self.group)
        return [out]

    def allgather_i64(self, tensors):
        """every rank's device int64[1] -> device int64[world] in rank order (stream-ordered
        on the current stream: no host round trip)"""
        (t,) = tensors
        if self.solo:
            return [t]
        if self.stage_cpu:
            out = [torch.empty(1, dtype=torch.int64) for _ in range(self.world)]
            self.dist.all_gather(out, t.cpu(), group=self.group)
            return [torch.cat(out).to(t.device)]
        out = torch.empty(self.world, dtype=torch.int64, device=t.device)
        self.dist.all_gather_into_tensor(out, t, group=self.group)
        return [out]

    def _a2a(self, x, ss, rs, row, group, async_op):
        """all-to-all-v of rows of `row` elements: ss[p] rows to rank p, rs[p] rows from it.
        One process alone: the input itself.  RCCL: one all_to_all_single.  gloo (tests,
        ranks sharing a GPU): grouped point-to-point transfers with the peers and a copy of
        this rank's own part."""
        home = x.device
        x = x[:sum(ss) * row]
        if self.stage_cpu:
            x = x.cpu()
        x = x.contiguous()
        if self.solo:
            return (x.to(home) if self.stage_cpu else x), None
        if self.nccl:
            # one all-to-all-v call (RCCL groups the per-peer sends / receives in C++): a
            # Python-side P2POp per peer costs tens of microseconds of host time each, which at
            # 8 ranks (14 transfers, three exchanges a step) approaches the step itself
            out = torch.empty(sum(int(b) for b in rs) * row, dtype=x.dtype, device=x.device)
            work = self.dist.all_to_all_single(
                out, x, output_split_sizes=[int(b) * row for b in rs],
                input_split_sizes=[int(a) * row for a in ss], group=group, async_op=async_op)
            return out, work
        so, ro = [0], [0]
        for a, b in zip(ss, rs):
            so.append(so[-1] + int(a) * row)
            ro.append(ro[-1] + int(b) * row)
        out = torch.empty(ro[-1], dtype=x.dtype, device=x.device)
        ops = []
        for p in range(self.world):
            if p == self.rank:
                continue
            if so[p + 1] > so[p]:
                ops.append(self.dist.P2POp(self.dist.isend, x[so[p]:so[p + 1]], p, group=group))
            if ro[p + 1] > ro[p]:
                ops.append(self.dist.P2POp(self.dist.irecv, out[ro[p]:ro[p + 1]], p, group=group))
        works = self.dist.batch_isend_irecv(ops) if ops else []
        me = self.rank
        if so[me + 1] > so[me]:
            out[ro[me]:ro[me + 1]].copy_(x[so[me]:so[me + 1]])
        work = _Works(works)
        if not async_op:
            work.wait()
            work = None
        if self.stage_cpu:
            out = out.to(home)
        return out, work

    def alltoallv(self, tensors, send_splits, recv_splits, row=1):
        return self.alltoallv_async(tensors, send_splits, recv_splits, row).wait()

    def alltoallv_async(self, tensors, send_splits, recv_splits, row=1):
        """-> handle whose wait() returns [received tensor] (the current stream then waits
        for the exchange)"""
        (x,), (ss,), (rs,) = tensors, send_splits, recv_splits
        if not self.nccl:
            return _Done([self._a2a(x, ss, rs, row, self.group, False)[0]])
        out, work = self._a2a(x, ss, rs, row, self.group, True)
        return _Work(work, [out])

    def alltoallv_keys_async(self, tensors, send_splits, recv_splits, row=1):
        """the key exchange: its inputs are complete (the host joined the Localizer lane), so
        it is issued from an idle stream over the second communicator"""
        (x,), (ss,), (rs,) = tensors, send_splits, recv_splits
        if not self.nccl:
            return _Done([self._a2a(x, ss, rs, row, self.kgroup, False)[0]])
        with torch.cuda.stream(self.kstream):
            out, work = self._a2a(x, ss, rs, row, self.kgroup, True)
        return _Work(work, [out], foreign=True)

    def allreduce_sum(self, values):
        (v,) = values
        t = torch.tensor(v, dtype=torch.float64)
        self.dist.all_reduce(t, group=self.cgroup)
        return [t.tolist()]


class _Works:
    """the transfers of one grouped exchange"""

    def __init__(self, works):
        self.works = works

    def wait(self):
        for w in self.works:
            w.wait()


class _Work:
    def __init__(self, work, out, foreign=False):
        self.work, self.out, self.foreign = work, out, foreign

    def wait(self):
        if self.work is not None:
            self.work.wait()  # the current stream waits for the exchange
        if self.foreign:
            # allocated on the exchange's own stream, read on this one: keep the caching
            # allocator from handing the memory out again before this stream is past its use
            s = torch.cuda.current_stream()
            for o in self.out:
                o.record_stream(s)
        return self.out


class LoopbackComm:
    """N shards held by one process (tests on one GPU); the exchange is a device copy."""

    def __init__(self, world):
        self.world = int(world)

    def ranks(self):
        return list(range(self.world))

    def allgather_i64(self, tensors):
        allc = torch.cat([t.reshape(1) for t in tensors])
        return [allc for _ in tensors]

    def allgather_rows(self, tensors, M, row):
        bufs = []
        for x in tensors:
            b = torch.zeros(M * row, dtype=x.dtype, device=x.device)
            b[:x.numel()] = x
            bufs.append(b)
        allb = torch.cat(bufs)
        return [allb for _ in tensors]

    def reduce_scatter_sum(self, tensors, M, row):
        acc = tensors[0].clone()
        for x in tensors[1:]:
            acc += x  # float32, in rank order
        c = M * row
        return [acc[g * c:(g + 1) * c] for g in range(self.world)]

    def exchange_counts(self, send_splits):
        return [[send_splits[r][g] for r in range(self.world)] for g in range(self.world)]

    def exchange_counts2(self, send):
        N = self.world
        return [[send[r][g] for r in range(N)] + [send[r][N + g] for r in range(N)]
                for g in range(N)]

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

    def alltoallv_async(self, tensors, send_splits, recv_splits, row=1):
        return _Done(self.alltoallv(tensors, send_splits, recv_splits, row))

    alltoallv_keys_async = alltoallv_async

    def allreduce_sum(self, values):
        tot = [sum(v[i] for v in values) for i in range(len(values[0]))]
        return [list(tot) for _ in values]


def _initv(shards, comm, slot):
    """push_agg=sum: rank the owners' InitV requests over all owners (a tiny all-gather of
    their counts, on the device) and draw them"""
    if not shards[0].agg_sum or shards[0].ctx.V_dim <= 0:
        return
    cnt = [sh.initv_local(slot) for sh in shards]
    allc = comm.allgather_i64(cnt)
    for sh, a, r in zip(shards, allc, comm.ranks()):
        sh.initv_draw(a, r, slot)


PHASES = ("localize", "xchg_keys", "owner_begin", "owner_pull", "xchg_pull", "fwd_bwd",
          "xchg_grads", "owner_push")
# ShardedPipeline.submit's marks: the previous step's push sits between the pull and the
# forward/backward, which starts after the record exchange
PIPE_PHASES = ("localize", "xchg_keys", "owner_begin", "owner_pull", "owner_push_prev",
               "xchg_pull+fwd_bwd", "xchg_grads_issue", "end")


def sharded_step(shards, dblks, comm, job_type=kTraining, push_cnt=False, max_index=MAX_INDEX,
                 preds=None, mark=None):
    """One bulk-synchronous step of the sharded store (oracle: ShardedOracle.step).  shards /
    dblks (/ preds): this process's shards and their batches (one each under
    torch.distributed, N under LoopbackComm).  push_cnt: epoch-0 Update(kFeaCount)
    (sgd_learner.cc:272, 304-307); ignored when V_dim == 0 like the reference's
    do_embedding_.  mark(i): called after phase PHASES[i] is issued (and with -1 first), e.g.
    to record stream events."""
    mark = mark or (lambda i: None)
    mark(-1)
    n = len(shards)
    want_cnt = bool(push_cnt) and shards[0].ctx.V_dim > 0
    for i in range(n):
        shards[i].localize(dblks[i], want_cnt, 0, max_index)
    loc = [shards[i].localize_wait(0) for i in range(n)]
    mark(0)
    send = [l[2] for l in loc]
    recv = comm.exchange_counts(send)
    rkeys = comm.alltoallv([l[0] for l in loc], send, recv)
    rcnt = comm.alltoallv([l[1] for l in loc], send, recv) if want_cnt else [None] * n
    mark(1)
    for i in range(n):
        shards[i].owner_begin(rkeys[i], recv[i], rcnt[i], 0)
    if want_cnt:
        _initv(shards, comm, 0)
    mark(2)
    S = shards[0].S
    vals = [s.owner_pull(0) for s in shards]
    mark(3)
    pulled = comm.alltoallv(vals, recv, send, S)
    mark(4)
    grads = [shards[i].fwd_bwd(dblks[i], pulled[i], job_type, 0, preds[i] if preds else None)
             for i in range(n)]
    mark(5)
    if job_type == kTraining:
        rgrads = comm.alltoallv(grads, send, recv, S)
        mark(6)
        for i in range(n):
            shards[i].owner_push(rgrads[i], 0)
        _initv(shards, comm, 0)
    else:
        mark(6)
    mark(7)
    return [sum(s) for s in recv]  # keys served per shard (for accounting)


def rsag_step(shards, dblks, comm, job_type=kTraining, push_cnt=False, max_index=MAX_INDEX,
              preds=None):
    """One bulk-synchronous step over the north_star's literal collectives:
    an all-gather of the workers' keys forms the sorted union, every owner pulls its union
    slice, an all-gather of the union-indexed records serves every worker's pull, and a
    reduce-scatter of union-indexed gradient rows (and, in epoch 0, counts) hands each owner
    the workers' summed rows of its slice — one Update per key (push_agg=sum semantics, oracle
    AggOracle).  The measured baseline beside the all-to-all-v schedule: its exchanges move
    union-sized, padded buffers instead of only the keys each worker touches."""
    n = len(shards)
    N = shards[0].nranks
    assert all(sh.agg_sum for sh in shards), "rsag_step needs push_agg=sum"
    want_cnt = bool(push_cnt) and shards[0].ctx.V_dim > 0
    for i in range(n):
        shards[i].localize(dblks[i], want_cnt, 0, max_index)
    loc = [shards[i].localize_wait(0) for i in range(n)]
    dev = shards[0].ctx.device
    # 1. every worker's key count, then its keys (padded to the largest), all-gathered
    cnts = comm.allgather_i64([torch.tensor([l[0].numel()], dtype=torch.int64, device=dev)
                               for l in loc])
    Us = [int(v) for v in cnts[0].cpu().tolist()]
    Umax = max(max(Us), 1)
    allk = comm.allgather_rows([l[0] for l in loc], Umax, 1)
    run_offs = [0]
    for u in Us:
        run_offs.append(run_offs[-1] + u)
    S = shards[0].S
    outs = []
    for i in range(n):
        r = comm.ranks()[i]
        ak = allk[i]
        runs = torch.cat([ak[g * Umax:g * Umax + Us[g]] for g in range(N)])
        uni, upos, bounds = shards[i].union(runs, run_offs)
        outs.append((uni, upos[run_offs[r]:run_offs[r + 1]], bounds))
    bounds = outs[0][2]
    M = max(max(bounds[g + 1] - bounds[g] for g in range(N)), 1)
    ranks = comm.ranks()
    own = [outs[i][0][bounds[ranks[i]]:bounds[ranks[i] + 1]] for i in range(n)]
    # 2. epoch 0: the workers' counts, union-indexed and reduce-scattered to the owners
    rcnt = [None] * n
    if want_cnt:
        bufs = []
        for i in range(n):
            b = torch.zeros(N * M, dtype=torch.float32, device=dev)
            shards[i].union_rows(loc[i][0], outs[i][1], bounds, M, 1, 1, loc[i][1], b)
            bufs.append(b)
        rcnt = comm.reduce_scatter_sum(bufs, M, 1)
    for i in range(n):
        R = own[i].numel()
        shards[i].owner_begin(own[i], [R] + [0] * (N - 1),
                              rcnt[i][:R] if want_cnt else None, 0)
    if want_cnt:
        _initv(shards, comm, 0)
    # 3. the owners' records of their slices, all-gathered (union-indexed)
    recs = comm.allgather_rows([sh.owner_pull(0) for sh in shards], M, S)
    grads = []
    for i in range(n):
        U = loc[i][0].numel()
        pulled = torch.empty(max(U * S, 1), dtype=torch.float32, device=dev)
        shards[i].union_rows(loc[i][0], outs[i][1], bounds, M, S, 0, recs[i], pulled)
        grads.append(shards[i].fwd_bwd(dblks[i], pulled[:U * S], job_type, 0,
                                       preds[i] if preds else None))
    if job_type != kTraining:
        return
    # 4. union-indexed gradient rows, reduce-scattered: each owner gets the summed rows
    bufs = []
    for i in range(n):
        b = torch.zeros(N * M * S, dtype=torch.float32, device=dev)
        shards[i].union_rows(loc[i][0], outs[i][1], bounds, M, S, 1, grads[i], b)
        bufs.append(b)
    rg = comm.reduce_scatter_sum(bufs, M, S)
    for i in range(n):
        shards[i].owner_push(rg[i][:own[i].numel() * S], 0)
    _initv(shards, comm, 0)


def _keep(tensors, stream):
    """tell the allocator that `stream` uses these (device) tensors: a buffer freed on the host
    is handed out again only after that stream's work queued so far"""
    for t in tensors:
        if t is not None and t.device.type == "cuda":
            t.record_stream(stream)


def _split_initv(shards, comm, slot):
    """InitV of the split owners' requests, ranked over all owners (a tiny device all-gather)"""
    if shards[0].ctx.V_dim <= 0:
        return
    cnt = [sh.split_initv_local(slot) for sh in shards]
    allc = comm.allgather_i64(cnt)
    for sh, a, r in zip(shards, allc, comm.ranks()):
        sh.split_initv_draw(a, r, slot)


SPLIT_PHASES = ("partition", "xchg_keys", "owner_begin", "owner_forward", "xchg_parts",
                "combine", "xchg_pxv", "owner_backward")


def split_step(shards, dblks, comm, job_type=kTraining, push_cnt=False, max_index=MAX_INDEX,
               preds=None, mark=None):
    """One bulk-synchronous step of the owner-computes split (csrc/split.hip; oracle:
    AggOracle.step, the single reference updater on the concatenated batch).  Every worker is
    padded to M = the largest batch's rows with empty rows, so the row-sized collectives are
    equal-size: the partials an all-to-all of M rows per owner, the [XV*p | p] rows an
    all-gather.  mark(i): called after phase SPLIT_PHASES[i] is issued (and with -1 first)."""
    mark = mark or (lambda i: None)
    mark(-1)
    n = len(shards)
    N = shards[0].nranks
    want_cnt = bool(push_cnt) and job_type == kTraining and shards[0].ctx.V_dim > 0
    for i in range(n):
        shards[i].split_partition(dblks[i], 0, max_index)
    part = [sh.split_partition_wait(0) for sh in shards]
    mark(0)
    # keys per owner, every worker's row count and whether its rows carry values, in one host
    # exchange (bit 40 of the row count: valued)
    send = [p[3] + [p[4] | ((p[1] is not None) << 40)] * N for p in part]
    both = comm.exchange_counts2(send)
    recv = [b[:N] for b in both]
    M = max(max(int(v) & ((1 << 40) - 1) for v in b[N:]) for b in both)
    M = max(M, 1)
    valued = any(int(v) >> 40 for v in both[0][N:])
    rkeys = comm.alltoallv([p[0] for p in part], [p[3] for p in part], recv)
    if valued:  # binary workers send 1s beside a valued worker
        xs = [p[1] if p[1] is not None else
              torch.ones(max(p[0].numel(), 1), dtype=torch.float32, device=p[0].device)
              for p in part]
        rx = comm.alltoallv(xs, [p[3] for p in part], recv)
    else:
        rx = [None] * n
    # nnz per (owner, row), padded to M rows per owner
    rcs = []
    for p in part:
        rc, B = p[2], p[4]
        if B < M:
            pad = torch.zeros(N * M, dtype=torch.int32, device=rc.device)
            pad.view(N, M)[:, :B] = rc.view(N, B)
            rc = pad
        rcs.append(rc)
    rrc = comm.alltoallv(rcs, [[M] * N] * n, [[M] * N] * n)
    cur = torch.cuda.current_stream() if torch.device(shards[0].ctx.device).type == "cuda" \
        else None
    if cur is not None:  # the partition's buffers (its own stream) are read here
        for p in part:
            _keep(p[:3], cur)
    mark(1)
    for i in range(n):
        shards[i].split_owner_begin(rkeys[i], rx[i], rrc[i], [M] * N, recv[i], job_type,
                                    want_cnt, 0)
    if want_cnt:
        _split_initv(shards, comm, 0)
    mark(2)
    PS = _lib.lib().dfx_split_part_floats(shards[0].ctx.h, shards[0].nranks)
    parts = [sh.split_owner_forward(0) for sh in shards]
    mark(3)
    rparts = comm.alltoallv(parts, [[M] * N] * n, [[M] * N] * n, PS)
    mark(4)
    pxv = [shards[i].split_combine(dblks[i], rparts[i], M, 0, preds[i] if preds else None)
           for i in range(n)]
    mark(5)
    if job_type == kTraining:
        PX = _lib.lib().dfx_split_pxv_floats(shards[0].ctx.h)
        allp = comm.allgather_rows(pxv, M, PX)
        mark(6)
        for i in range(n):
            shards[i].split_owner_backward(allp[i], 0)
        _split_initv(shards, comm, 0)
    else:
        mark(6)
    mark(7)
    return [sum(r) for r in recv]  # keys received per owner (for accounting)


# SplitPipeline's main-stream marks (the next step's begin runs on the lanes)
SPLIT_PIPE_PHASES = ("owner_forward", "xchg_parts", "combine", "xchg_pxv", "owner_backward",
                     "initv", "end", "end2")


class SplitPipeline:
    """The owner-computes split (split_step's results exactly: every forward reads the model
    after the previous step's update) with the fused step's overlap: submit(batch t+1) issues
    batch t+1's partition on the Localizer lanes, then step t's forward, partial exchange,
    combine, record all-gather and backward on the context stream, then batch t+1's key
    exchange and owner Localizer (owner_begin, lane = 1) on the lanes, which run beside step
    t's main-stream work.  A count push (epoch 0) or a step without a backward touches the
    table in owner_begin, so that begin runs on the context stream after step t's update.
    flush() runs the last step.  A batch must stay alive until the submit after the one that
    took it (or flush())."""

    AHEAD = 2  # steps the host may run ahead of the context stream

    def __init__(self, shards, comm, max_index=MAX_INDEX):
        self.shards, self.comm, self.max_index = shards, comm, max_index
        self.slot = 0
        self.pending = None
        self.done = []  # one event per step's main-stream work: bounds the host's run-ahead
        self.throttle_s = 0.0  # host seconds spent waiting on that bound
        # the contexts' Localizer lanes become torch streams (high priority, like the
        # library's own): torch's allocator tracks the exchange buffers used on them, and the
        # streams outlive the contexts
        self.lanes = []
        for sh in shards:
            ln = torch.cuda.Stream(device=sh.ctx.device, priority=-1)
            check(_lib.lib().dfx_ctx_set_lane_stream(sh.ctx.h, 0, ctypes.c_void_p(ln.cuda_stream)))
            self.lanes.append(ln)

    def submit(self, dblks, job_type=kTraining, push_cnt=False, preds=None, mark=None):
        s = self.slot
        self.slot ^= 1
        want_cnt = bool(push_cnt) and job_type == kTraining and self.shards[0].ctx.V_dim > 0
        for i, sh in enumerate(self.shards):
            sh.split_partition(dblks[i], s, self.max_index)
        if self.pending is not None:
            self._main(self.pending, mark)
        self.pending = self._begin(s, dblks, job_type, want_cnt, preds)

    def flush(self, mark=None):
        if self.pending is not None:
            self._main(self.pending, mark)
            self.pending = None

    def _begin(self, s, dblks, job_type, want_cnt, preds):
        shards, comm = self.shards, self.comm
        n, N = len(shards), shards[0].nranks
        part = [sh.split_partition_wait(s) for sh in shards]
        send = [p[3] + [p[4] | ((p[1] is not None) << 40)] * N for p in part]
        both = comm.exchange_counts2(send)
        recv = [b[:N] for b in both]
        M = max(1, max(max(int(v) & ((1 << 40) - 1) for v in b[N:]) for b in both))
        valued = any(int(v) >> 40 for v in both[0][N:])
        lane = not want_cnt and job_type == kTraining
        main = torch.cuda.current_stream()
        # the exchanges feed the owners' Localizer: issue them (and wait for them) on the lane
        with torch.cuda.stream(self.lanes[0] if lane else main):
            rcs = []
            for p in part:
                rc, B = p[2], p[4]
                if B < M:
                    pad = torch.zeros(N * M, dtype=torch.int32, device=rc.device)
                    pad.view(N, M)[:, :B] = rc.view(N, B)
                    rc = pad
                rcs.append(rc)
            hk = comm.alltoallv_keys_async([p[0] for p in part], [p[3] for p in part], recv)
            hr = comm.alltoallv_keys_async(rcs, [[M] * N] * n, [[M] * N] * n)
            if valued:
                xs = [p[1] if p[1] is not None else
                      torch.ones(max(p[0].numel(), 1), dtype=torch.float32, device=p[0].device)
                      for p in part]
                hx = comm.alltoallv_keys_async(xs, [p[3] for p in part], recv)
            rkeys, rrc = hk.wait(), hr.wait()
            rx = hx.wait() if valued else [None] * n
            for p in part:  # the partition's buffers (its own stream) are read here
                _keep(p[:3], torch.cuda.current_stream())
            if lane and n > 1:  # loopback: every lane waits for the exchange on lane 0
                ev = torch.cuda.Event()
                ev.record()
                for ln in self.lanes[1:]:
                    ln.wait_event(ev)
        for i in range(n):
            # the owner Localizer (lane) and the forward (context stream) read the received keys
            # / values; at world size 1 they are the partition's own buffers
            _keep((rkeys[i], rx[i]), main)
            if lane:
                _keep((rkeys[i], rx[i], rrc[i]), self.lanes[i])
            shards[i].split_owner_begin(rkeys[i], rx[i], rrc[i], [M] * N, recv[i], job_type,
                                        want_cnt, s, lane)
        if want_cnt:
            _split_initv(shards, comm, s)
        return (s, dblks, job_type, preds, M, rkeys, rx, part)

    def _main(self, q, mark):
        mark = mark or (lambda i: None)
        s, dblks, job_type, preds, M, _, _, _ = q
        shards, comm = self.shards, self.comm
        n, N = len(shards), shards[0].nranks
        mark(-1)
        PS = _lib.lib().dfx_split_part_floats(shards[0].ctx.h, shards[0].nranks)
        parts = [sh.split_owner_forward(s) for sh in shards]
        mark(0)
        rparts = comm.alltoallv(parts, [[M] * N] * n, [[M] * N] * n, PS)
        mark(1)
        pxv = [shards[i].split_combine(dblks[i], rparts[i], M, s, preds[i] if preds else None)
               for i in range(n)]
        mark(2)
        if job_type == kTraining:
            PX = _lib.lib().dfx_split_pxv_floats(shards[0].ctx.h)
            allp = comm.allgather_rows(pxv, M, PX)
            mark(3)
            for i in range(n):
                shards[i].split_owner_backward(allp[i], s)
            mark(4)
            _split_initv(shards, comm, s)
        else:
            mark(3)
            mark(4)
        mark(5)
        mark(6)
        mark(7)
        if torch.device(shards[0].ctx.device).type == "cuda":
            ev = torch.cuda.Event()
            ev.record()
            self.done.append(ev)
            t = time.perf_counter()
            while len(self.done) > self.AHEAD:
                self.done.pop(0).synchronize()
            self.throttle_s += time.perf_counter() - t


class ShardedPipeline:
    """The pipelined (1-step-stale) schedule of the sharded store (oracle: StaleOracle).

    submit(batch t+1) issues batch t+1's Localizer on its lane and then runs step t, whose
    Localizer was issued one submit earlier:
      host             join step t's Localizer; exchange the split counts
      exchange         keys(t) (+ counts) to their owners
      main stream      owner_begin(t), owner_pull(t)       beside step t-1's gradient exchange
      exchange         records(t) back to the workers
      main stream      owner_push(t-1)                    beside the record exchange
      main stream      fwd_bwd(t); exchange gradients(t)  (pending until the next step)
    so every pull is answered before the previous step's push: pulls are at most one step
    stale, the reference's two batches in flight against an asynchronous server
    (sgd_learner.cc:310-312, kvstore_dist.h:137-150).  flush() runs the queued step and the
    last push.  A step's predictions / progress are complete after the submit that follows
    it (or flush()); its batch must stay alive until then and one submit longer."""

    def __init__(self, shards, comm, max_index=MAX_INDEX):
        self.shards, self.comm, self.max_index = shards, comm, max_index
        self.slot = 0
        self.queue = []
        self.pending = None

    def submit(self, dblks, job_type=kTraining, push_cnt=False, preds=None, mark=None):
        s = self.slot
        self.slot ^= 1
        want_cnt = bool(push_cnt) and self.shards[0].ctx.V_dim > 0
        for i, sh in enumerate(self.shards):
            sh.localize(dblks[i], want_cnt, s, self.max_index)
        self.queue.append((s, dblks, job_type, want_cnt, preds))
        if len(self.queue) > 1:
            self._step(self.queue.pop(0), mark)

    def flush(self, mark=None):
        """run the queued step and apply the last push"""
        while self.queue:
            self._step(self.queue.pop(0), mark)
        self._push_pending()

    def _step(self, q, mark):
        mark = mark or (lambda i: None)
        s, dblks, job_type, want_cnt, preds = q
        shards, comm = self.shards, self.comm
        n = len(shards)
        mark(-1)
        loc = [shards[i].localize_wait(s) for i in range(n)]
        mark(0)
        send = [l[2] for l in loc]
        recv = comm.exchange_counts(send)
        hk = comm.alltoallv_keys_async([l[0] for l in loc], send, recv)
        hc = comm.alltoallv_keys_async([l[1] for l in loc], send, recv) if want_cnt else None
        rkeys = hk.wait()
        rcnt = hc.wait() if hc else [None] * n
        mark(1)
        for i in range(n):
            shards[i].owner_begin(rkeys[i], recv[i], rcnt[i], s)
        if want_cnt:
            _initv(shards, comm, s)
        mark(2)
        S = shards[0].S
        vals = [sh.owner_pull(s) for sh in shards]
        mark(3)
        hr = comm.alltoallv_async(vals, recv, send, S)
        self._push_pending()
        mark(4)
        pulled = hr.wait()
        grads = [shards[i].fwd_bwd(dblks[i], pulled[i], job_type, s, preds[i] if preds else None)
                 for i in range(n)]
        mark(5)
        if job_type == kTraining:
            self.pending = (s, comm.alltoallv_async(grads, send, recv, S), dblks)
        mark(6)
        mark(7)

    def _push_pending(self):
        if self.pending is None:
            return
        s, hg, _ = self.pending
        self.pending = None
        rgrads = hg.wait()
        for i, sh in enumerate(self.shards):
            sh.owner_push(rgrads[i], s)
        _initv(self.shards, self.comm, s)


class SplitStore:
    """The owner-computes split driven from C++ (libdfx_dist.so, host/split_host.cc): the
    schedule of split_step (pipelined=False) or SplitPipeline (pipelined=True) without the
    interpreter between the launches — the same results bit for bit.

    Loopback: SplitStore(shards) drives N shards held by this process (one GPU).  RCCL:
    SplitStore([shard], rccl=(rank, nranks, ids, force_exchange)), one shard per process,
    ids = SplitStore.rccl_ids() made on rank 0 and handed to every rank by the caller.

    stale=True (pipelined): the 1-step-stale schedule — step t+1's owner forward runs before
    step t's backward, so each step's partial exchange and row gather travel beside the other
    step's compute (oracle: dist_oracle.SplitStaleOracle; push_agg=sum).  EXPERIMENTAL and
    parity unpinned by the reference, which has no such schedule: the gradient takes the stale
    forward's p / XV*p but the diag(XXp) V term from the owner's current V.  One slice only
    (set_slices(k > 1) raises).

    Batches must stay alive until the second submit after the one that took them (the store
    keeps them), a pipelined step's predictions / progress are complete after the next submit
    (or flush())."""

    MARKS = 7  # main-stream boundaries (dfx_split_store_set_marks)
    PHASES = ("owner_forward", "xchg_parts", "combine", "xchg_pxv", "owner_backward", "initv")

    def __init__(self, shards, pipelined=True, max_index=MAX_INDEX, rccl=None, stale=False):
        D = _lib.dist_lib()
        self.n = len(shards)
        mode = 2 if stale else int(bool(pipelined))
        self.shards = shards
        h = ctypes.c_void_p()
        if rccl is None:
            arr = (ctypes.c_void_p * self.n)(*[sh.ctx.h for sh in shards])
            _lib.dist_check(D.dfx_split_store_create_loopback(arr, self.n, mode, max_index,
                                                              ctypes.byref(h)))
        else:
            if self.n != 1:
                raise ValueError("SplitStore over RCCL holds one shard per process")
            rank, nranks, ids, force = rccl
            buf = ctypes.create_string_buffer(bytes(ids), len(ids))
            _lib.dist_check(D.dfx_split_store_create_rccl(
                shards[0].ctx.h, int(rank), int(nranks), buf, int(bool(force)), mode, max_index,
                ctypes.byref(h)))
        self.h = h
        self._live = []

    @staticmethod
    def rccl_ids():
        """fresh communicator ids (rank 0), as bytes for the caller's rendezvous"""
        D = _lib.dist_lib()
        k = D.dfx_dist_rccl_comms()
        buf = ctypes.create_string_buffer(k * D.dfx_dist_rccl_id_bytes())
        _lib.dist_check(D.dfx_dist_rccl_ids(k, buf))
        return buf.raw

    @staticmethod
    def rccl_ids_size():
        """bytes of rccl_ids() (every rank allocates its receive buffer with it)"""
        D = _lib.dist_lib()
        return D.dfx_dist_rccl_comms() * D.dfx_dist_rccl_id_bytes()

    def set_slices(self, k):
        """rows of a step in k slices (the exchanges of one slice beside the next slice's
        compute; 0: the driver's default, one slice)"""
        _lib.dist_check(_lib.dist_lib().dfx_split_store_set_slices(self.h, int(k)))

    def submit(self, dblks, job_type=kTraining, push_cnt=False, preds=None):
        D = _lib.dist_lib()
        bs = (_lib.Batch * self.n)(*[b.as_batch() for b in dblks])
        pp = None
        if preds is not None:
            pp = (ctypes.c_void_p * self.n)(*[p.data_ptr() if p is not None else None
                                              for p in preds])
        _lib.dist_check(D.dfx_split_store_submit(self.h, bs, int(job_type), int(bool(push_cnt)),
                                                 pp))
        self._live.append((dblks, preds))
        del self._live[:-3]

    def flush(self):
        _lib.dist_check(_lib.dist_lib().dfx_split_store_flush(self.h))

    def throttle_seconds(self):
        v = ctypes.c_double(0)
        _lib.dist_check(_lib.dist_lib().dfx_split_store_throttle_seconds(self.h, ctypes.byref(v)))
        return v.value

    def set_marks(self, boundaries):
        mask = 0
        for b in boundaries:
            mask |= 1 << int(b)
        _lib.dist_check(_lib.dist_lib().dfx_split_store_set_marks(self.h, mask))

    def take_marks(self):
        """-> {phase: (summed ms, steps)} of the marked steps"""
        ms = (ctypes.c_double * (self.MARKS - 1))()
        st = (ctypes.c_int64 * (self.MARKS - 1))()
        _lib.dist_check(_lib.dist_lib().dfx_split_store_take_marks(self.h, ms, st))
        return {p: (ms[i], st[i]) for i, p in enumerate(self.PHASES)}

    def close(self):
        if self.h:
            _lib.dist_check(_lib.dist_lib().dfx_split_store_destroy(self.h))
            self.h = None
            self._live = []

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
