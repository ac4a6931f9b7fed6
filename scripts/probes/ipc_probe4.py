import os, sys, socket
import torch, torch.distributed as dist, torch.multiprocessing as mp
sys.path.insert(0, os.getcwd())

def w(rank, port, mode):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    from tf_operator_amd.parallel.ipc import IpcAllReduce
    ar = IpcAllReduce(slot_bytes=4 << 20, timeout_ms=5000)
    n = 262147
    for it in range(3):
        g = torch.Generator(device="cpu").manual_seed(77 + it)
        parts = [torch.randn(n, generator=g) for _ in range(2)]
        if mode == "h2d":
            t = parts[rank].cuda()
        elif mode == "h2d_sync":
            t = parts[rank].cuda(); torch.cuda.synchronize()
        else:
            t = torch.empty(n, device="cuda"); t.copy_(parts[rank]); torch.cuda.synchronize()
        before = t.clone().cpu()
        ar(t)
        torch.cuda.synchronize()
        got = t.cpu()
        want = parts[0] + parts[1]
        bad = ((got - want).abs() > 1e-3).nonzero().flatten()
        ok_in = torch.equal(before, parts[rank])
        if rank == 0:
            msg = f"mode {mode} it {it}: input ok {ok_in} bad {len(bad)}"
            if len(bad):
                i = int(bad[0])
                msg += f" first {i} got {got[i]:.4f} want {want[i]:.4f} p0 {parts[0][i]:.4f} p1 {parts[1][i]:.4f}"
                # does got match p0+p1 of another index?
                m = ((parts[0] + parts[1]) - got[i]).abs().argmin()
                msg += f" nearest-sum-index {int(m)} (delta {int(m) - i})"
            print(msg, flush=True)
    dist.barrier()

if __name__ == "__main__":
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    mp.spawn(w, args=(port, sys.argv[1]), nprocs=2)
