"""The owner side of the sharded step at N shards, on one GPU (loopback shards in one process):
N workers' batches of the bench's shape (B rows x 39 binary nnz over 2^24 keys), so each owner
receives N sorted runs of ~U/N keys — the merge, find-or-insert, pull and push an 8-GPU run
makes per GPU.  Run under `rocprofv3 --kernel-trace --stats` to read per-kernel times.
usage: owner_bench.py [N] [B] [steps]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from difacto_amd import dist as DI  # noqa: E402
from difacto_amd import hotpath as H  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 6
    k, kb = 39, 24
    dev = torch.device("cuda", 0)
    per = (1 << kb) // N
    ctxs = [H.Context(0, V_dim=16, V_threshold=0, l1=0, lr=.1, V_lr=.01, max_keys=per,
                      max_vrows=per + per // 8 + 4096) for _ in range(N)]
    shards = [DI.Shard(c, N) for c in ctxs]
    comm = DI.LoopbackComm(N)
    g = torch.Generator(device=dev)

    def batch(seed):
        g.manual_seed(seed)
        blk = type("B", (), {})()
        blk.size, blk.nnz = B, B * k
        ids = torch.randint(0, 1 << kb, (B * k,), device=dev, generator=g, dtype=torch.int64)
        offs = torch.arange(0, B * k + 1, k, device=dev, dtype=torch.int64)
        lab = torch.where(torch.rand(B, device=dev, generator=g) < .25, 1.0, -1.0)
        return _Dev(offs, ids, lab.to(torch.float32))

    # count-push steps until the key space is covered (as bench.py's epoch 0), so the timed
    # steps run in the steady state: every key present, no inserts
    warm = max(1, -(-int(4.6 * (1 << kb)) // (N * B * k)))
    for s in range(warm + steps):
        dbs = [batch(1000 * s + r) for r in range(N)]
        DI.sharded_step(shards, dbs, comm, H.kTraining, push_cnt=(s < warm))
        torch.cuda.synchronize()
        print("step", s, "warm" if s < warm else "", flush=True)
    print("owner_bench N=%d B=%d steps=%d done" % (N, B, steps))


class _Dev:
    def __init__(self, offs, ids, labels):
        self.offs, self.ids, self.labels = offs, ids, labels
        self.size = labels.numel()
        self.nnz = ids.numel()
        self.vals = None
        self.weights = None

    def as_batch(self):
        import ctypes
        from difacto_amd import _lib
        return _lib.Batch(self.size, self.nnz, ctypes.c_void_p(self.offs.data_ptr()),
                          ctypes.c_void_p(self.ids.data_ptr()), None,
                          ctypes.c_void_p(self.labels.data_ptr()), None)


if __name__ == "__main__":
    main()
