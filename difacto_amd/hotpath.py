"""Python mirror of DiFacto's plugin interfaces for the hot path, over libdifacto_amd.so.

Names, argument meaning and error behaviour follow the reference's C++ interfaces so the
parity tests read like its gtests:

    Localizer.compact          src/data/localizer.h:41-51
    FMLoss.predict/calc_grad   src/loss/fm_loss.h:56-203 (LogitLoss == FMLoss with V_dim 0)
    Loss.evaluate, auc         include/difacto/loss.h:57-66, src/loss/bin_class_metric.h:35-57
    Store.pull/push            include/difacto/store.h:44-75 over SGDUpdater::Get/Update
    Store.save/load/dump       src/sgd/sgd_updater.h:84-139
    train_step                 SGDLearner::IterateData's per-batch executor (fused)

Device buffers are torch tensors (torch is the allocator and stream provider only); u64
keys travel as int64 tensors holding the same bits, u32 as int32.  Every call goes through
the C-ABI; a failing status raises DfxError (the reference would LOG(FATAL)).
"""
import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import check

kFeaCount, kWeight, kGradient = 1, 2, 3
kTraining, kValidation, kPrediction = 3, 4, 5
MAX_INDEX = (1 << 64) - 1


def _p(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _kwstr(kwargs):
    return ",".join("%s=%s" % (k, v) for k, v in kwargs.items()).encode()


class Context:
    """One device context: a stream, the device model store and a scratch workspace.

    kwargs are the reference .conf keys (lr, V_dim, V_lr, l1, l2, V_threshold, ...) plus
    max_keys / max_vrows for the device hash table.  Like the reference's Loss objects a
    context is not thread-safe.
    """

    def __init__(self, device=0, **kwargs):
        self.device = torch.device("cuda", device)
        self.kwargs = dict(kwargs)
        h = ctypes.c_void_p()
        # strict: a misspelt or retired kwarg raises instead of running the default
        check(_lib.lib().dfx_ctx_create(device, _kwstr(dict(kwargs, strict=1)), ctypes.byref(h)))
        self.h = h
        self.V_dim = _lib.lib().dfx_ctx_vdim(h)
        self.use_current_stream()

    def use_current_stream(self):
        s = torch.cuda.current_stream(self.device)
        check(_lib.lib().dfx_ctx_set_stream(self.h, ctypes.c_void_p(s.cuda_stream)))

    def set_input_stream(self, stream):
        """batches of train_step are produced on this torch stream (None: the context's)"""
        check(_lib.lib().dfx_ctx_set_input_stream(
            self.h, None if stream is None else ctypes.c_void_p(stream.cuda_stream)))

    def close(self):
        if getattr(self, "h", None):
            _lib.lib().dfx_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def sync(self):
        check(_lib.lib().dfx_sync(self.h))

    def reserve(self, max_rows, max_nnz):
        check(_lib.lib().dfx_reserve(self.h, int(max_rows), int(max_nnz)))

    # ---- helpers -------------------------------------------------------------------------
    def tensor(self, a, dtype):
        """host numpy array -> device tensor of ``dtype`` (u64 -> int64 bits, u32 -> int32)."""
        if a is None:
            return None
        a = np.ascontiguousarray(a)
        if a.dtype == np.uint64:
            a = a.view(np.int64)
        elif a.dtype == np.uint32:
            a = a.view(np.int32)
        return torch.from_numpy(a.copy()).to(self.device, dtype=dtype)


class DeviceRowBlock:
    """dmlc::RowBlock<feaid_t> resident on the device (BatchReader output)."""

    def __init__(self, ctx, blk):
        self.size = blk.size
        self.nnz = blk.nnz
        self.offs = ctx.tensor(blk.offs, torch.int64)
        self.ids = ctx.tensor(blk.ids, torch.int64)
        self.vals = ctx.tensor(blk.vals, torch.float32)
        self.labels = ctx.tensor(blk.labels, torch.float32)
        self.weights = ctx.tensor(blk.weights, torch.float32)

    def as_batch(self):
        return _lib.Batch(self.size, self.nnz, _p(self.offs), _p(self.ids), _p(self.vals),
                          _p(self.labels), _p(self.weights))


def u64(t):
    """device int64 tensor holding u64 bits -> numpy uint64"""
    return t.cpu().numpy().view(np.uint64)


def u32(t):
    return t.cpu().numpy().view(np.uint32)


class Localizer:
    """Localizer (src/data/localizer.h:16-95): uint64 ids -> sorted unique reversed keys,
    float counts and a u32-remapped CSR.  Compact returns (col, uniq, cnt) device tensors; the
    compacted block's offsets/values/labels are the input's."""

    def __init__(self, ctx, max_index=MAX_INDEX):
        self.ctx = ctx
        self.max_index = max_index

    def compact(self, dblk, want_cnt=True):
        ctx = self.ctx
        nnz = dblk.nnz
        uniq = torch.empty(max(nnz, 1), dtype=torch.int64, device=ctx.device)
        cnt = torch.empty(max(nnz, 1), dtype=torch.float32, device=ctx.device) if want_cnt else None
        col = torch.empty(max(nnz, 1), dtype=torch.int32, device=ctx.device)
        n = ctypes.c_int64(0)
        check(_lib.lib().dfx_localize(ctx.h, dblk.size, nnz, _p(dblk.offs), _p(dblk.ids),
                                      ctypes.c_uint64(self.max_index), _p(uniq), _p(cnt),
                                      _p(col), ctypes.byref(n)))
        U = n.value
        return col[:nnz], uniq[:U], (cnt[:U] if want_cnt else None)


class FMLoss:
    """FMLoss (src/loss/fm_loss.h); V_dim == 0 is LogitLoss (src/loss/logit_loss.h)."""

    def __init__(self, ctx, V_dim=0):
        self.ctx = ctx
        self.V_dim = int(V_dim)

    def predict(self, dblk, col, weights, w_pos, V_pos, pred, n_cols):
        """pred += forward(X, weights) — accumulates like the reference."""
        check(_lib.lib().dfx_fm_predict(self.ctx.h, dblk.size, dblk.nnz, _p(dblk.offs), _p(col),
                                        _p(dblk.vals), _p(weights), _p(w_pos), _p(V_pos),
                                        int(n_cols), self.V_dim, _p(pred)))

    def calc_grad(self, dblk, col, weights, w_pos, V_pos, pred, grad, n_cols):
        """grad += backward(X, weights, pred) — grad must be pre-zeroed like the reference."""
        check(_lib.lib().dfx_fm_calcgrad(self.ctx.h, dblk.size, dblk.nnz, _p(dblk.offs), _p(col),
                                         _p(dblk.vals), _p(dblk.labels), _p(dblk.weights),
                                         _p(weights), _p(w_pos), _p(V_pos), int(n_cols),
                                         self.V_dim, _p(pred), _p(grad)))

    def evaluate(self, label, pred):
        out = ctypes.c_double(0)
        check(_lib.lib().dfx_evaluate(self.ctx.h, pred.numel(), _p(label), _p(pred),
                                      ctypes.byref(out)))
        return out.value


def auc(ctx, label, pred):
    """BinClassMetric::AUC, returned as AUC * n like the reference."""
    out = ctypes.c_double(0)
    check(_lib.lib().dfx_auc(ctx.h, pred.numel(), _p(label), _p(pred), ctypes.byref(out)))
    return out.value


def get_pos(ctx, lens):
    n = lens.numel()
    w = torch.empty(max(n, 1), dtype=torch.int32, device=ctx.device)
    v = torch.empty(max(n, 1), dtype=torch.int32, device=ctx.device)
    check(_lib.lib().dfx_get_pos(ctx.h, n, _p(lens), _p(w), _p(v)))
    return w[:n], v[:n]


class Store:
    """The device model store: Store push/pull over the SGDUpdater (FTRL w, AdaGrad V,
    V_threshold lazy InitV)."""

    def __init__(self, ctx):
        self.ctx = ctx

    def pull(self, keys):
        ctx = self.ctx
        n = keys.numel()
        d = ctx.V_dim
        vals = torch.empty(max(n * (1 + d), 1), dtype=torch.float32, device=ctx.device)
        lens = torch.empty(max(n, 1), dtype=torch.int32, device=ctx.device) if d > 0 else None
        nv = ctypes.c_int64(0)
        check(_lib.lib().dfx_store_pull(ctx.h, _p(keys), n, _p(vals), _p(lens), ctypes.byref(nv)))
        return vals[:nv.value], (lens[:n] if d > 0 else None)

    def push(self, keys, val_type, vals, lens=None):
        check(_lib.lib().dfx_store_push(self.ctx.h, _p(keys), keys.numel(), int(val_type),
                                        _p(vals), vals.numel(), _p(lens)))

    def save(self, path, save_aux=True):
        check(_lib.lib().dfx_store_save(self.ctx.h, str(path).encode(), int(save_aux)))

    def load(self, path):
        check(_lib.lib().dfx_store_load(self.ctx.h, str(path).encode()))

    def dump(self, path, dump_aux=False, need_reverse=False):
        check(_lib.lib().dfx_store_dump(self.ctx.h, str(path).encode(), int(dump_aux),
                                        int(need_reverse)))

    def stats(self):
        nk, nv, nw = ctypes.c_int64(0), ctypes.c_int64(0), ctypes.c_double(0)
        seed = ctypes.c_uint32(0)
        check(_lib.lib().dfx_store_stats(self.ctx.h, ctypes.byref(nk), ctypes.byref(nv),
                                         ctypes.byref(nw), ctypes.byref(seed)))
        return {"n_keys": nk.value, "n_vrows": nv.value, "new_w": nw.value, "seed": seed.value}

    def evaluate(self):
        pen, nnz = ctypes.c_double(0), ctypes.c_int64(0)
        check(_lib.lib().dfx_store_evaluate(self.ctx.h, ctypes.byref(pen), ctypes.byref(nnz)))
        return pen.value, nnz.value

    def probe_stats(self):
        """-> (mean probe distance, longest probe distance, table capacity)"""
        m, mx, cap = ctypes.c_double(0), ctypes.c_int64(0), ctypes.c_int64(0)
        check(_lib.lib().dfx_store_probe_stats(self.ctx.h, ctypes.byref(m), ctypes.byref(mx),
                                               ctypes.byref(cap)))
        return m.value, mx.value, cap.value

    def reserve(self, n_keys, n_vrows):
        check(_lib.lib().dfx_store_reserve(self.ctx.h, int(n_keys), int(n_vrows)))

    def entry(self, key):
        d = self.ctx.V_dim
        st = (ctypes.c_float * 4)()
        V = (ctypes.c_float * max(2 * d, 1))()
        hv, found = ctypes.c_int(0), ctypes.c_int(0)
        check(_lib.lib().dfx_store_entry(self.ctx.h, ctypes.c_uint64(int(key)), st, V,
                                         ctypes.byref(hv), ctypes.byref(found)))
        if not found.value:
            return None
        return (np.array(st, np.float32),
                np.array(V, np.float32)[:2 * d].copy() if hv.value else None)


def train_step(ctx, dblk, job_type=kTraining, push_cnt=False, max_index=MAX_INDEX, pred=None):
    """One fused minibatch (localize -> [feacnt] -> pull -> predict -> eval -> AUC ->
    calcgrad -> push).  Progress accumulates on the device; read it with progress()."""
    b = dblk.as_batch()
    check(_lib.lib().dfx_train_step(ctx.h, ctypes.byref(b), int(job_type), int(bool(push_cnt)),
                                    ctypes.c_uint64(max_index), _p(pred)))


# main-stream phases of dfx_train_step (the Localizer runs on its own lane; "localize" is
# the part of it the main stream waits for)
PHASES = ("localize", "probe_pull", "feacnt", "forward", "eval_auc", "backward_update", "initv")


def prof_enable(ctx, max_steps, phases=None):
    """time the next max_steps dfx_train_step calls: every phase and the lanes, or only the
    named phases (e.g. ("backward_update",): fewer events, less added latency)"""
    if phases is None:
        check(_lib.lib().dfx_prof_enable(ctx.h, int(max_steps)))
        return
    mask = 0
    for p in phases:
        m = PHASES.index(p)
        mask |= 3 << m
    check(_lib.lib().dfx_prof_enable_marks(ctx.h, int(max_steps), mask))


def prof_read(ctx):
    """-> ({phase: summed ms}, recorded steps, mean U per step)"""
    ms = (ctypes.c_double * 7)()
    n = ctypes.c_int(0)
    mu = ctypes.c_double(0)
    check(_lib.lib().dfx_prof_read(ctx.h, ms, ctypes.byref(n), ctypes.byref(mu)))
    return dict(zip(PHASES, list(ms))), n.value, mu.value


def prof_counts(ctx):
    """per step since the last call (or prof_read): mean unique keys, keys with live V and
    their occurrences; and the batches the bucket Localizer placed by its hot-key map; resets"""
    out = (ctypes.c_double * 4)()
    check(_lib.lib().dfx_prof_counts(ctx.h, out))
    r = dict(zip(("U", "U_V", "occ_V"), list(out)))
    r["lb_map_steps"] = int(out[3])
    return r


def prof_host(ctx):
    """host seconds dfx_train_step calls waited (capacity guard) since the last call, waits"""
    out = (ctypes.c_double * 2)()
    if not hasattr(_lib.lib(), "dfx_prof_host"):  # an older library under A/B (DFX_LIB_PATH)
        return {"wait_s": 0.0, "waits": 0}
    check(_lib.lib().dfx_prof_host(ctx.h, out))
    return {"wait_s": out[0], "waits": int(out[1])}


def prof_lanes(ctx):
    """after prof_read: mean ms per batch of the Localizer lane, its start / end relative to
    the main stream reaching the batch, and the AUC lane"""
    out = (ctypes.c_double * 4)()
    check(_lib.lib().dfx_prof_lanes(ctx.h, out))
    return dict(zip(("loc_ms", "loc_start_rel_ms", "loc_end_rel_ms", "auc_ms"), list(out)))


def progress(ctx, reset=True):
    p = _lib.Progress()
    check(_lib.lib().dfx_progress_read(ctx.h, ctypes.byref(p), int(reset)))
    return {"nrows": p.nrows, "loss": p.loss, "auc": p.auc, "penalty": p.penalty,
            "nnz_w": p.nnz_w}
