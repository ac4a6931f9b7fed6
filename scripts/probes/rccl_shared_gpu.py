"""Can RCCL run several ranks on ONE GPU (the 1-GPU box)?  Spawns N ranks on
cuda:0 with the nccl backend and all-reduces; prints the outcome.  Used to
decide whether multi-rank RCCL paths (PS=1 Worker=2) can be exercised on a
single MI355X."""
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def run(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    t = torch.full((1 << 20,), float(rank + 1), device="cuda")
    dist.all_reduce(t)
    torch.cuda.synchronize()
    print(f"rank {rank}: all_reduce -> {float(t[0])} (want {world * (world + 1) / 2})", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.spawn(run, args=(world, port), nprocs=world, join=True)
    print("shared-GPU RCCL ok")
