import os, sys, socket
import torch, torch.distributed as dist, torch.multiprocessing as mp
sys.path.insert(0, os.getcwd())

def w(rank, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    from tf_operator_amd.parallel.ipc import IpcAllReduce
    ar = IpcAllReduce(slot_bytes=1 << 20, timeout_ms=5000)
    print("rank", rank, "bufs", [hex(ar.bufs[i] or 0) for i in range(2)], "flags", [hex(ar.flags[i] or 0) for i in range(2)], flush=True)
    for it in range(3):
        t = torch.full((8,), float(rank + 1 + 10 * it), device="cuda")
        ar(t)
        torch.cuda.synchronize()
        print("rank", rank, "it", it, t.tolist(), "err", int(ar.err.item()), flush=True)
    dist.barrier()

if __name__ == "__main__":
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    mp.spawn(w, args=(port,), nprocs=2)
