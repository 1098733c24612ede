"""ctypes view of oracle/liboracle.so — the CPU restatement of DiFacto's hot path.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
``cpu_baseline`` leg, never by the product package (difacto_amd/).  See oracle.cc for
what each function restates (reference file:line) and how parity is pinned.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "liboracle.so")
_lib = None

u64p = ctypes.POINTER(ctypes.c_uint64)
u32p = ctypes.POINTER(ctypes.c_uint32)
i32p = ctypes.POINTER(ctypes.c_int32)
f32p = ctypes.POINTER(ctypes.c_float)
f64p = ctypes.POINTER(ctypes.c_double)


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        L = ctypes.CDLL(_LIB)
        L.orc_reverse_bytes.restype = ctypes.c_uint64
        L.orc_reverse_bytes.argtypes = [ctypes.c_uint64]
        L.orc_localize.restype = ctypes.c_int64
        L.orc_localize.argtypes = [ctypes.c_int64, u64p, u64p, ctypes.c_uint64, u64p, f32p, u32p]
        L.orc_fm_predict.restype = None
        L.orc_fm_predict.argtypes = [ctypes.c_int64, u64p, u32p, f32p, f32p, i32p, i32p,
                                     ctypes.c_int, f32p]
        L.orc_fm_calcgrad.restype = None
        L.orc_fm_calcgrad.argtypes = [ctypes.c_int64, u64p, u32p, f32p, f32p, f32p, f32p, i32p,
                                      i32p, ctypes.c_int64, ctypes.c_int, f32p, f32p]
        L.orc_fm_calcgrad_stale.restype = None
        L.orc_fm_calcgrad_stale.argtypes = [ctypes.c_int64, u64p, u32p, f32p, f32p, f32p, f32p,
                                            i32p, f32p, i32p, i32p, ctypes.c_int64, ctypes.c_int,
                                            f32p, f32p]
        L.orc_evaluate.restype = ctypes.c_double
        L.orc_evaluate.argtypes = [ctypes.c_int64, f32p, f32p]
        L.orc_auc.restype = ctypes.c_float
        L.orc_auc.argtypes = [ctypes.c_int64, f32p, f32p]
        L.orc_get_pos.restype = None
        L.orc_get_pos.argtypes = [ctypes.c_int64, i32p, i32p, i32p]
        L.orc_updater_create.restype = ctypes.c_void_p
        L.orc_updater_create.argtypes = [ctypes.c_char_p]
        L.orc_updater_destroy.argtypes = [ctypes.c_void_p]
        L.orc_updater_vdim.argtypes = [ctypes.c_void_p]
        L.orc_updater_seed.restype = ctypes.c_uint
        L.orc_updater_seed.argtypes = [ctypes.c_void_p]
        L.orc_updater_new_w.restype = ctypes.c_float
        L.orc_updater_new_w.argtypes = [ctypes.c_void_p]
        L.orc_updater_size.restype = ctypes.c_int64
        L.orc_updater_size.argtypes = [ctypes.c_void_p]
        L.orc_updater_get.restype = ctypes.c_int64
        L.orc_updater_get.argtypes = [ctypes.c_void_p, u64p, ctypes.c_int64, f32p, i32p]
        L.orc_updater_update.restype = ctypes.c_int
        L.orc_updater_update.argtypes = [ctypes.c_void_p, u64p, ctypes.c_int64, ctypes.c_int, f32p,
                                         ctypes.c_int64, i32p]
        L.orc_updater_penalty.restype = ctypes.c_double
        L.orc_updater_penalty.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64)]
        L.orc_updater_entry.restype = ctypes.c_int
        L.orc_updater_entry.argtypes = [ctypes.c_void_p, ctypes.c_uint64, f32p, f32p,
                                        ctypes.POINTER(ctypes.c_int)]
        L.orc_updater_dump.restype = ctypes.c_int
        L.orc_updater_dump.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int,
                                       ctypes.c_int]
        L.orc_updater_save.restype = ctypes.c_int
        L.orc_updater_save.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int]
        L.orc_updater_load.restype = ctypes.c_int
        L.orc_updater_load.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
        L.orc_train_step.restype = ctypes.c_int
        L.orc_train_step.argtypes = [ctypes.c_void_p, ctypes.c_int64, u64p, u64p, f32p, f32p, f32p,
                                     ctypes.c_uint64, ctypes.c_int, ctypes.c_int, f64p, f32p]
        L.orc_rand_r.restype = ctypes.c_int
        L.orc_rand_r.argtypes = [ctypes.POINTER(ctypes.c_uint)]
        L.orc_last_error.restype = ctypes.c_char_p
        _lib = L
    return _lib


def _p(a, t):
    if a is None:
        return None
    return a.ctypes.data_as(t)


def _c(a, dt):
    return None if a is None else np.ascontiguousarray(a, dtype=dt)


def reverse_bytes(x):
    return lib().orc_reverse_bytes(int(x))


def localize(offs, ids, max_index=(1 << 64) - 1, want_cnt=True):
    """Localizer::Compact -> (uniq u64[U], cnt f32[U] or None, col u32[nnz])."""
    offs = _c(offs, np.uint64)
    ids = _c(ids, np.uint64)
    B = len(offs) - 1
    nnz = int(offs[-1]) if B > 0 else 0
    uniq = np.zeros(max(nnz, 1), np.uint64)
    cnt = np.zeros(max(nnz, 1), np.float32)
    col = np.zeros(max(nnz, 1), np.uint32)
    U = lib().orc_localize(B, _p(offs, u64p), _p(ids, u64p), ctypes.c_uint64(max_index),
                           _p(uniq, u64p), _p(cnt, f32p), _p(col, u32p))
    return uniq[:U].copy(), (cnt[:U].copy() if want_cnt else None), col[:nnz].copy()


def fm_predict(offs, col, val, weights, w_pos, V_pos, V_dim, pred=None):
    offs = _c(offs, np.uint64)
    col = _c(col, np.uint32)
    val = _c(val, np.float32)
    weights = _c(weights, np.float32)
    w_pos = _c(w_pos, np.int32)
    V_pos = _c(V_pos, np.int32)
    B = len(offs) - 1
    out = np.zeros(B, np.float32) if pred is None else np.array(pred, np.float32, copy=True)
    lib().orc_fm_predict(B, _p(offs, u64p), _p(col, u32p), _p(val, f32p), _p(weights, f32p),
                         _p(w_pos, i32p), _p(V_pos, i32p), int(V_dim), _p(out, f32p))
    return out


def fm_calcgrad(offs, col, val, label, rweight, weights, w_pos, V_pos, ncol, V_dim, pred,
                grad=None):
    offs = _c(offs, np.uint64)
    col = _c(col, np.uint32)
    val = _c(val, np.float32)
    label = _c(label, np.float32)
    rweight = _c(rweight, np.float32)
    weights = _c(weights, np.float32)
    w_pos = _c(w_pos, np.int32)
    V_pos = _c(V_pos, np.int32)
    pred = _c(pred, np.float32)
    B = len(offs) - 1
    out = np.zeros(len(weights), np.float32) if grad is None else np.array(grad, np.float32, copy=True)
    lib().orc_fm_calcgrad(B, _p(offs, u64p), _p(col, u32p), _p(val, f32p), _p(label, f32p),
                          _p(rweight, f32p), _p(weights, f32p), _p(w_pos, i32p), _p(V_pos, i32p),
                          int(ncol), int(V_dim), _p(pred, f32p), _p(out, f32p))
    return out


def fm_calcgrad_stale(offs, col, val, label, rweight, fw_weights, fw_V_pos, bw_weights, bw_w_pos,
                      bw_V_pos, ncol, V_dim, pred):
    """CalcGrad of a 1-step-stale split step (oracle.cc CalcGradStale): p and XV_ from the
    forward's (older) model, the gradient's layout and diag(XXp) V from the model the update
    reads.  Returns the gradient in the bw layout."""
    offs = _c(offs, np.uint64)
    col = _c(col, np.uint32)
    val = _c(val, np.float32)
    label = _c(label, np.float32)
    rweight = _c(rweight, np.float32)
    fw_weights = _c(fw_weights, np.float32)
    fw_V_pos = _c(fw_V_pos, np.int32)
    bw_weights = _c(bw_weights, np.float32)
    bw_w_pos = _c(bw_w_pos, np.int32)
    bw_V_pos = _c(bw_V_pos, np.int32)
    pred = _c(pred, np.float32)
    B = len(offs) - 1
    out = np.zeros(len(bw_weights), np.float32)
    lib().orc_fm_calcgrad_stale(B, _p(offs, u64p), _p(col, u32p), _p(val, f32p),
                                _p(label, f32p), _p(rweight, f32p), _p(fw_weights, f32p),
                                _p(fw_V_pos, i32p), _p(bw_weights, f32p), _p(bw_w_pos, i32p),
                                _p(bw_V_pos, i32p), int(ncol), int(V_dim), _p(pred, f32p),
                                _p(out, f32p))
    return out


def evaluate(label, pred):
    label = _c(label, np.float32)
    pred = _c(pred, np.float32)
    return lib().orc_evaluate(len(pred), _p(label, f32p), _p(pred, f32p))


def auc(label, pred):
    label = _c(label, np.float32)
    pred = _c(pred, np.float32)
    return lib().orc_auc(len(pred), _p(label, f32p), _p(pred, f32p))


def auc_stable_ties(label, pred):
    """BinClassMetric::AUC (bin_class_metric.h:35-57) with ties between equal predictions
    kept in input order.  The reference sorts with the unstable std::sort, so its value on
    tied predictions (e.g. the all-zero first batch, or clipped +-20) is unspecified; the
    device path breaks ties by input order, and tie-heavy checks compare against this."""
    label = np.asarray(label, np.float32)
    pred = np.asarray(pred, np.float32) + np.float32(0.0)
    n = len(pred)
    lab = (label[np.argsort(pred, kind="stable")] > 0).astype(np.float64)
    before = np.cumsum(lab) - lab
    area = float(before[lab == 0].sum())
    P = float(lab.sum())
    if P == 0 or P == n:
        return 1.0
    area /= P * (n - P)
    return (1 - area if area < 0.5 else area) * n


def has_ties(pred):
    p = np.asarray(pred, np.float32) + np.float32(0.0)
    return len(np.unique(p)) != len(p)


def get_pos(lens):
    lens = _c(lens, np.int32)
    n = len(lens)
    w = np.zeros(n, np.int32)
    v = np.zeros(n, np.int32)
    lib().orc_get_pos(n, _p(lens, i32p), _p(w, i32p), _p(v, i32p))
    return w, v


class Updater:
    """SGDUpdater restated (FTRL w, AdaGrad V, rand_r InitV) on std::unordered_map."""

    kFeaCount, kWeight, kGradient = 1, 2, 3

    def __init__(self, **kw):
        s = ",".join("%s=%s" % (k, v) for k, v in kw.items())
        self.h = lib().orc_updater_create(s.encode())
        self.V_dim = lib().orc_updater_vdim(self.h)

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_updater_destroy(self.h)
            self.h = None

    @property
    def seed(self):
        return lib().orc_updater_seed(self.h)

    @property
    def new_w(self):
        return lib().orc_updater_new_w(self.h)

    def size(self):
        return lib().orc_updater_size(self.h)

    def get(self, keys):
        keys = _c(keys, np.uint64)
        U = len(keys)
        d = self.V_dim
        vals = np.zeros(max(U * (1 + d), 1), np.float32)
        lens = np.zeros(max(U, 1), np.int32) if d > 0 else None
        n = lib().orc_updater_get(self.h, _p(keys, u64p), U, _p(vals, f32p), _p(lens, i32p))
        return vals[:n].copy(), (lens[:U].copy() if d > 0 else None)

    def update(self, keys, typ, vals, lens=None):
        keys = _c(keys, np.uint64)
        vals = _c(vals, np.float32)
        lens = _c(lens, np.int32)
        rc = lib().orc_updater_update(self.h, _p(keys, u64p), len(keys), int(typ), _p(vals, f32p),
                                      len(vals), _p(lens, i32p))
        if rc != 0:
            raise RuntimeError(lib().orc_last_error().decode())

    def entry(self, key):
        st = np.zeros(4, np.float32)
        V = np.zeros(max(2 * self.V_dim, 1), np.float32)
        hv = ctypes.c_int(0)
        ok = lib().orc_updater_entry(self.h, ctypes.c_uint64(int(key)), _p(st, f32p), _p(V, f32p),
                                     ctypes.byref(hv))
        if not ok:
            return None
        return st, (V[:2 * self.V_dim].copy() if hv.value else None)

    def penalty(self):
        n = ctypes.c_int64(0)
        v = lib().orc_updater_penalty(self.h, ctypes.byref(n))
        return v, n.value

    def save(self, path, save_aux=True):
        if lib().orc_updater_save(self.h, path.encode(), int(save_aux)) != 0:
            raise RuntimeError(lib().orc_last_error().decode())

    def dump(self, path, dump_aux=False, need_reverse=False):
        """SGDUpdater::Dump (sgd_updater.h:108-139): text, one line per non-empty entry"""
        if lib().orc_updater_dump(self.h, path.encode(), int(dump_aux), int(need_reverse)) != 0:
            raise RuntimeError(lib().orc_last_error().decode())

    def load(self, path):
        if lib().orc_updater_load(self.h, path.encode()) != 0:
            raise RuntimeError(lib().orc_last_error().decode())

    def train_step(self, offs, ids, val, label, rweight=None, max_index=(1 << 64) - 1,
                   push_cnt=False, train=True, want_pred=False):
        offs = _c(offs, np.uint64)
        ids = _c(ids, np.uint64)
        val = _c(val, np.float32)
        label = _c(label, np.float32)
        rweight = _c(rweight, np.float32)
        B = len(offs) - 1
        out = np.zeros(3, np.float64)
        pred = np.zeros(max(B, 1), np.float32) if want_pred else None
        rc = lib().orc_train_step(self.h, B, _p(offs, u64p), _p(ids, u64p), _p(val, f32p),
                                  _p(label, f32p), _p(rweight, f32p), ctypes.c_uint64(max_index),
                                  int(push_cnt), int(train), _p(out, f64p), _p(pred, f32p))
        if rc != 0:
            raise RuntimeError(lib().orc_last_error().decode())
        if want_pred:
            return out[0], out[1], pred[:B].copy()
        return out[0], out[1]


def rand_r_seq(seed, n):
    s = ctypes.c_uint(seed)
    out = [lib().orc_rand_r(ctypes.byref(s)) for _ in range(n)]
    return out, s.value
