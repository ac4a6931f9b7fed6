import os, sys, socket
import torch, torch.distributed as dist, torch.multiprocessing as mp
sys.path.insert(0, os.getcwd())

def w(rank, port, sync):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    from tf_operator_amd.parallel.ipc import IpcAllReduce
    ar = IpcAllReduce(slot_bytes=4 << 20, timeout_ms=5000)
    bad = 0
    for it in range(12):
        for n, dt in ((1000, torch.bfloat16), (262147, torch.float32), (1 << 20, torch.bfloat16)):
            g = torch.Generator(device="cpu").manual_seed(1000 * it + n)
            parts = [torch.randn(n, generator=g) for _ in range(2)]
            t = parts[rank].to(dt).cuda()
            ar(t)
            if sync:
                torch.cuda.synchronize()
            want = sum(p.to(dt).float() for p in parts)
            got = t.float().cpu()
            e = float((got - want).abs().max())
            if e > 0.05 and bad < 4:
                bad += 1
                idx = int((got - want).abs().argmax())
                print(f"rank {rank} sync {sync} it {it} n {n} dt {dt} maxerr {e:.3f} at {idx}: got {got[idx]:.3f} want {want[idx]:.3f} mine {parts[rank][idx]:.3f} other {parts[1-rank][idx]:.3f}", flush=True)
    print(f"rank {rank} sync {sync} bad {bad} err {int(ar.err.item())}", flush=True)
    dist.barrier()

if __name__ == "__main__":
    sync = int(sys.argv[1])
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    mp.spawn(w, args=(port, sync), nprocs=2)
