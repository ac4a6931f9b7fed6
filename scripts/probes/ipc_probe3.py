import os, sys, socket
import torch, torch.distributed as dist, torch.multiprocessing as mp
sys.path.insert(0, os.getcwd())

def w(rank, port, world):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tf_operator_amd.parallel.ipc import IpcAllReduce
    ar = IpcAllReduce(slot_bytes=4 << 20, timeout_ms=5000)
    for n in (8, 1000, 4096, 65536, 131072, 262144, 262147):
        for dt in (torch.float32, torch.bfloat16):
            parts = [torch.arange(n, dtype=torch.float32) * 0.001 * (r + 1) for r in range(world)]
            t = parts[rank].to(dt).cuda()
            ar(t)
            torch.cuda.synchronize()
            want = sum(p.to(dt).float() for p in parts)
            got = t.float().cpu()
            bad = ((got - want).abs() > 0.02 * (want.abs() + 1)).nonzero().flatten()
            if rank == 0:
                print(f"world {world} n {n} {dt}: bad {len(bad)} first {bad[:4].tolist()} "
                      f"got {got[bad[:2]].tolist()} want {want[bad[:2]].tolist()}", flush=True)
    dist.barrier()

if __name__ == "__main__":
    world = int(sys.argv[1])
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    mp.spawn(w, args=(port, world), nprocs=world)
