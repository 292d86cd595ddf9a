"""Probe: can two ranks share the box's single GPU over RCCL ("nccl")? If so, the multi-rank bench path (device
broadcast, MIN all-reduce of the frame-equality table, the per-step all-gather) can execute on RCCL here.

  python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 \
      tools/probes/rccl_same_gpu.py
"""
import os

import torch
import torch.distributed as dist


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", device_id=dev)
    x = torch.full((4,), float(rank + 1), device=dev)
    g = torch.empty(4 * world, device=dev)
    dist.all_gather_into_tensor(g, x)
    m = torch.tensor([rank + 3], device=dev, dtype=torch.int32)
    dist.all_reduce(m, op=dist.ReduceOp.MIN)
    b = torch.full((2,), float(rank), device=dev)
    dist.broadcast(b, src=0)
    torch.cuda.synchronize()
    print(f"rank {rank}: gather {g.tolist()} min {m.item()} bcast {b.tolist()}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
