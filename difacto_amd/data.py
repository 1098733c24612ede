"""Host-side batch producers: the libsvm reader and the synthetic generators.

The reference keeps reading and batching on the CPU (BASELINE.json north_star); this
module is the thin CSR producer that feeds the device path.  A batch is a
``RowBlock<feaid_t>`` in the reference's layout (dmlc RowBlock, include/difacto/base.h):

    offs   u64[B+1]   (size_t offsets, offs[0] == 0)
    ids    u64[nnz]   (raw feature ids)
    vals   f32[nnz] or None   (None == binary: BatchReader drops all-1 values,
                               src/reader/batch_reader.cc:71-73)
    labels f32[B]
"""
import numpy as np


class RowBlock:
    __slots__ = ("offs", "ids", "vals", "labels", "weights")

    def __init__(self, offs, ids, vals, labels, weights=None):
        self.offs = np.ascontiguousarray(offs, dtype=np.uint64)
        self.ids = np.ascontiguousarray(ids, dtype=np.uint64)
        self.vals = None if vals is None else np.ascontiguousarray(vals, dtype=np.float32)
        self.labels = np.ascontiguousarray(labels, dtype=np.float32)
        self.weights = None if weights is None else np.ascontiguousarray(weights, dtype=np.float32)

    @property
    def size(self):
        return len(self.offs) - 1

    @property
    def nnz(self):
        return int(self.offs[-1]) if self.size > 0 else 0

    def slice(self, begin, end):
        o0, o1 = int(self.offs[begin]), int(self.offs[end])
        return RowBlock(self.offs[begin:end + 1] - self.offs[begin], self.ids[o0:o1],
                        None if self.vals is None else self.vals[o0:o1], self.labels[begin:end],
                        None if self.weights is None else self.weights[begin:end])

    def drop_binary_values(self):
        """BatchReader::Next's binary detection (batch_reader.cc:71-73)."""
        if self.vals is not None and np.all(self.vals == 1):
            self.vals = None
        return self


def concat(blocks):
    offs = [np.zeros(1, np.uint64)]
    base = 0
    for b in blocks:
        offs.append(b.offs[1:] + np.uint64(base))
        base += b.nnz
    vals = None
    if any(b.vals is not None for b in blocks):
        vals = np.concatenate([b.vals if b.vals is not None else np.ones(b.nnz, np.float32)
                               for b in blocks])
    return RowBlock(np.concatenate(offs), np.concatenate([b.ids for b in blocks]), vals,
                    np.concatenate([b.labels for b in blocks]))


def read_libsvm(path):
    """Minimal libsvm reader (label idx:val ...), the format of tests/data."""
    offs = [0]
    ids = []
    vals = []
    labels = []
    with open(path) as f:
        for line in f:
            tok = line.split()
            if not tok:
                continue
            labels.append(float(tok[0]))
            for t in tok[1:]:
                k, v = t.split(":")
                ids.append(int(k))
                vals.append(float(v))
            offs.append(len(ids))
    return RowBlock(np.array(offs, np.uint64), np.array(ids, np.uint64),
                    np.array(vals, np.float32), np.array(labels, np.float32))


def synthetic(rows, nnz_per_row, key_space, binary=True, pos_frac=0.25, seed=42, zipf=None,
              ragged=False):
    """Criteo/LR/Zipf-shaped synthetic batches (SURVEY.md §8(d) inputs).

    keys ~ U[0, key_space) (or Zipf(s) over [1, key_space] when ``zipf`` is set), labels
    +1 with probability ``pos_frac`` else -1, values U(0,1] unless binary.
    ``ragged`` draws row lengths in [0, 2*nnz_per_row] (empty rows included).
    """
    rng = np.random.default_rng(seed)
    if ragged:
        lens = rng.integers(0, 2 * nnz_per_row + 1, size=rows)
    else:
        lens = np.full(rows, nnz_per_row)
    offs = np.zeros(rows + 1, np.uint64)
    offs[1:] = np.cumsum(lens)
    nnz = int(offs[-1])
    if zipf is None:
        ids = rng.integers(0, key_space, size=nnz, dtype=np.uint64)
    else:
        ids = zipf_keys(rng, nnz, zipf, key_space)
    vals = None if binary else (1.0 - rng.random(nnz, dtype=np.float32)).astype(np.float32)
    labels = np.where(rng.random(rows) < pos_frac, 1.0, -1.0).astype(np.float32)
    return RowBlock(offs, ids, vals, labels)


_ZIPF_CDF = {}


def zipf_keys(rng, n, s, key_space):
    """Zipf(s) over ranks 1..key_space by inverse CDF.  The CDF table is exact up to 2^25
    ranks (C5: Zipf(1.1) over [1, 2^24] uses the whole table); beyond that the tail's mass is
    the continuous power-law integral and tail ranks are drawn by inverting it."""
    m = int(min(key_space, 1 << 25))
    key = (m, s)
    if key not in _ZIPF_CDF:
        ranks = np.arange(1, m + 1, dtype=np.float64)
        _ZIPF_CDF[key] = np.cumsum(ranks ** (-s))
    head = _ZIPF_CDF[key]
    tail = 0.0
    if key_space > m:  # integral of x^-s over [m + 1/2, key_space + 1/2]
        a, b = m + 0.5, key_space + 0.5
        tail = (a ** (1 - s) - b ** (1 - s)) / (s - 1)
    total = head[-1] + tail
    u = rng.random(n) * total
    out = (np.searchsorted(head, u) + 1).astype(np.uint64)
    t = u > head[-1]
    if np.any(t):  # invert the tail integral
        a = m + 0.5
        r = a ** (1 - s) - (u[t] - head[-1]) * (s - 1)
        x = np.floor(r ** (1.0 / (1 - s)) + 0.5)
        out[t] = np.clip(x, m + 1, key_space).astype(np.uint64)
    return out
