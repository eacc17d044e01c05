"""Can two ranks of one RCCL process group share the box's single GPU?  (If so, the N > 1 bench / exchange
path can be exercised over real RCCL on the one-GPU box.)  torchrun --nproc-per-node 2 tools/rccl_same_gpu_probe.py"""
import os
import torch
import torch.distributed as dist

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda:0"))
t = torch.full((1024,), float(rank + 1), device="cuda")
dist.all_reduce(t)
g = torch.empty(world, device="cuda")
dist.all_gather_into_tensor(g, torch.tensor([float(rank)], device="cuda"))
torch.cuda.synchronize()
print(f"rank {rank}: all_reduce {t[0].item()} (expect {world * (world + 1) / 2}), all_gather {g.tolist()}", flush=True)
dist.destroy_process_group()
