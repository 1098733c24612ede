"""RCCL collective latency through torch.distributed at world size N (default 1): per call
of a small all-gather, an all-to-all of a step's partials and an all-gather of its [XV*p | p]
rows, queued back to back on the current stream, and the host time per call.
usage: torchrun --nproc-per-node 1 tools/rccl_lat.py"""
import os
import time

import torch
import torch.distributed as dist


def main():
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist.init_process_group("nccl", device_id=dev)
    w = dist.get_world_size()
    cases = {
        "allgather_8B": (torch.zeros(1, dtype=torch.int64, device=dev),
                         torch.zeros(w, dtype=torch.int64, device=dev), "ag"),
        "alltoall_14MB": (torch.zeros(100000 * 36, device=dev),
                          torch.zeros(100000 * 36, device=dev), "a2a"),
        "allgather_8MB": (torch.zeros(100000 * 20, device=dev),
                          torch.zeros(w * 100000 * 20, device=dev), "ag"),
    }
    for name, (x, y, kind) in cases.items():
        for it in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            n = 50
            for _ in range(n):
                if kind == "ag":
                    dist.all_gather_into_tensor(y, x)
                else:
                    dist.all_to_all_single(y, x)
            t_host = time.perf_counter() - t0
            torch.cuda.synchronize()
            t = time.perf_counter() - t0
        if dist.get_rank() == 0:
            print("%-14s %8.1f us/call GPU-bound, host %6.1f us/call" % (name, t / n * 1e6,
                                                                          t_host / n * 1e6))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
