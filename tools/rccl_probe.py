"""Probe: can RCCL run two ranks on one device (the 1-GPU box), so that bench.py's `nccl` branch
(MCPT_BENCH_SHARE_GPU=1) can be rehearsed end to end?  One all_reduce and one point-to-point
send / recv of a device tensor, as parallel.gather_film_to_root does.

Usage: python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \\
           --master-port 29561 tools/rccl_probe.py
"""
import os
import sys

import torch
import torch.distributed as dist


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count()
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
    x = torch.full((4,), float(rank + 1), device="cuda")
    dist.all_reduce(x)
    ok = bool(torch.all(x == world * (world + 1) / 2))
    if rank == 1:
        dist.send(torch.arange(8, dtype=torch.float32, device="cuda"), dst=0)
    elif rank == 0:
        buf = torch.empty(8, dtype=torch.float32, device="cuda")
        dist.recv(buf, src=1)
        ok = ok and bool(torch.equal(buf.cpu(), torch.arange(8, dtype=torch.float32)))
    torch.cuda.synchronize()
    dist.barrier()
    print(f"rank {rank}: device {dev} of {torch.cuda.device_count()}, backend {dist.get_backend()}, ok={ok}", flush=True)
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
