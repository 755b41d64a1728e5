"""Does torch.distributed (nccl = RCCL) all-reduce torch.uint64 with MAX natively? (1 rank)"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "rust-crdt_amd"))
import torch
import torch.distributed as dist

torch.cuda.set_device(0)
dist.init_process_group("nccl", init_method="tcp://127.0.0.1:29533", rank=0, world_size=1,
                        device_id=torch.device("cuda:0"))
from crdts_hip import replica

print("native_u64_max:", replica.native_u64_max(torch.device("cuda:0")))
t = torch.arange(10, dtype=torch.int64, device="cuda")
replica.dense_allreduce_max(t)
print("ok", t.tolist())
dist.destroy_process_group()
