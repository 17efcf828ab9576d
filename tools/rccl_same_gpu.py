"""Probe: can two RCCL ranks share one GPU on this box (rehearsal of the nccl path on a 1-GPU machine)?
usage: python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 tools/rccl_same_gpu.py"""
import os

import torch
import torch.distributed as dist

rank = int(os.environ['RANK'])
torch.cuda.set_device(0)
dist.init_process_group('nccl', device_id=torch.device('cuda', 0))
t = torch.full((1024,), float(rank + 1), device='cuda')
dist.all_reduce(t)
torch.cuda.synchronize()
print(f'rank {rank}: all_reduce -> {float(t[0])} (expect 3.0)', flush=True)
dist.destroy_process_group()
