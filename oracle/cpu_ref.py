"""ctypes view of oracle/libcpuref.so — the reference's CPU hot path WITH its threading
(cpu_ref.cc: OpenMP row / column splits, ParallelSort, the two-thread IterateData pipeline).

MEASUREMENT / TEST INFRASTRUCTURE ONLY: bench.py's ``cpu_baseline`` leg times it on the host
cores; tests/test_oracle.py checks it against oracle.cc.  Never imported by difacto_amd/.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "libcpuref.so")
_lib = None

u64p = ctypes.POINTER(ctypes.c_uint64)
f32p = ctypes.POINTER(ctypes.c_float)
f64p = ctypes.POINTER(ctypes.c_double)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            subprocess.check_call(["make", "-s", "-C", _HERE])
        L = ctypes.CDLL(_LIB)
        L.cref_create.restype = ctypes.c_void_p
        L.cref_create.argtypes = [ctypes.c_char_p]
        L.cref_destroy.argtypes = [ctypes.c_void_p]
        L.cref_size.restype = ctypes.c_int64
        L.cref_size.argtypes = [ctypes.c_void_p]
        L.cref_seed.restype = ctypes.c_uint
        L.cref_seed.argtypes = [ctypes.c_void_p]
        L.cref_step.restype = None
        L.cref_step.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, u64p, u64p, f32p,
                                f32p, ctypes.c_int, ctypes.c_int, f64p, f32p]
        L.cref_iterate.restype = ctypes.c_double
        L.cref_iterate.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                   ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(u64p),
                                   ctypes.POINTER(u64p), ctypes.POINTER(f32p),
                                   ctypes.POINTER(f32p), f64p]
        L.cref_max_threads.restype = ctypes.c_int
        L.cref_phases.restype = None
        L.cref_phases.argtypes = [f64p]
        _lib = L
    return _lib


def _p(a, t):
    return None if a is None else a.ctypes.data_as(t)


class CpuRef:
    """SGDLearner local mode on the CPU with blk_nthreads = nthreads"""

    def __init__(self, nthreads, **kw):
        self.nt = int(nthreads)
        self.h = lib().cref_create(",".join("%s=%s" % kv for kv in kw.items()).encode())

    def close(self):
        if self.h:
            lib().cref_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def size(self):
        return lib().cref_size(self.h)

    @property
    def seed(self):
        return lib().cref_seed(self.h)

    def step(self, blk, push_cnt=False, train=True, want_pred=False):
        out = np.zeros(3, np.float64)
        pred = np.zeros(blk.size, np.float32) if want_pred else None
        lib().cref_step(self.h, self.nt, blk.size, _p(blk.offs, u64p), _p(blk.ids, u64p),
                        _p(blk.vals, f32p), _p(blk.labels, f32p), int(push_cnt), int(train),
                        _p(out, f64p), _p(pred, f32p))
        return (out[0], out[1], pred) if want_pred else (out[0], out[1])

    def iterate(self, blocks):
        """one pass over the batches in the reference's pipeline (no count push); returns
        (seconds, loss, auc*n, nrows)"""
        n = len(blocks)
        B = (ctypes.c_int64 * n)(*[b.size for b in blocks])
        offs = (u64p * n)(*[_p(b.offs, u64p) for b in blocks])
        ids = (u64p * n)(*[_p(b.ids, u64p) for b in blocks])
        has_val = any(b.vals is not None for b in blocks)
        val = (f32p * n)(*[_p(b.vals, f32p) for b in blocks]) if has_val else None
        lab = (f32p * n)(*[_p(b.labels, f32p) for b in blocks])
        out = np.zeros(3, np.float64)
        dt = lib().cref_iterate(self.h, self.nt, n, B, offs, ids, val, lab, _p(out, f64p))
        return dt, out[0], out[1], out[2]


PHASES = ("localize", "get", "predict", "evaluate_auc", "calcgrad", "update")


def phases():
    """wall seconds per phase since the last call (then reset)"""
    out = np.zeros(6, np.float64)
    lib().cref_phases(_p(out, f64p))
    return dict(zip(PHASES, out.tolist()))


def host_cores():
    return lib().cref_max_threads()
