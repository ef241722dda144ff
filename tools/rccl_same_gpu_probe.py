# Probe: can two ranks share one GPU over RCCL (backend "nccl")? Run with
#   torchrun --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 tools/rccl_same_gpu_probe.py
import os, torch, torch.distributed as dist
r = int(os.environ["RANK"]); w = int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda:0"))
x = torch.full((1 << 20,), float(r + 1), device="cuda:0")
dist.all_reduce(x)
torch.cuda.synchronize()
print("rank", r, "sum", x[0].item(), flush=True)
dist.destroy_process_group()
