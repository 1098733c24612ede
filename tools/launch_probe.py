"""Host launch cost probe: time N tiny kernel launches before / after torch.distributed
(nccl) init, to find what slows hipLaunchKernel in the sharded bench."""
import os, sys, time
import torch
import torch.distributed as dist

def probe(tag, x, n=2000):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        x.add_(1.0)
    te = time.perf_counter() - t
    torch.cuda.synchronize()
    print("%-40s %.2f us/launch" % (tag, te / n * 1e6), flush=True)

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
x = torch.zeros(16, device=dev)
probe("plain", x)
s = torch.cuda.Stream(); 
with torch.cuda.stream(s): probe("side stream", x)
os.environ.setdefault("MASTER_ADDR", "127.0.0.1"); os.environ.setdefault("MASTER_PORT", "29533")
os.environ.setdefault("RANK", "0"); os.environ.setdefault("WORLD_SIZE", "1")
mode = sys.argv[1] if len(sys.argv) > 1 else "nccl"
if mode == "nccl":
    dist.init_process_group("nccl", device_id=dev)
else:
    dist.init_process_group("gloo")
probe("after init " + mode, x)
dist.barrier()
probe("after barrier", x)
g = dist.new_group([0], backend="gloo")
probe("after gloo group", x)
t = torch.tensor([1]); dist.all_gather([torch.empty_like(t)], t, group=g)
probe("after gloo all_gather", x)
dist.destroy_process_group()
probe("after destroy", x)
