"""Probe: can two RCCL ranks share ONE GPU (torchrun --nproc-per-node 2, both
on cuda:0)?  Each rank all-reduces its rank id and prints the sum; NCCL's
own rule is one rank per device, so a refusal is the expected answer.
    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 tools/rccl_dup_probe.py"""
import os

import torch
import torch.distributed as dist

torch.cuda.set_device(0)
dist.init_process_group("nccl")
t = torch.tensor([float(dist.get_rank())], device="cuda")
dist.all_reduce(t)
torch.cuda.synchronize()
print(f"rank {dist.get_rank()}: all_reduce sum {t.item()} (world {dist.get_world_size()}, "
      f"LOCAL_RANK {os.environ.get('LOCAL_RANK')})", flush=True)
dist.destroy_process_group()
