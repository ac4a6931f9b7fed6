"""Device-to-device copy rate of a copy engine (hipMemcpyDeviceToDeviceNoCU,
toa_emulate_copy_nocu) against the ring-kernel stand-in at full speed, on
this GPU: what the SDMA all-gather arm of parallel/emulate.py moves per
second when nothing else runs."""
import json
import sys

import torch

sys.path.insert(0, ".")
from tf_operator_amd.ops import _lib  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    out = {}
    for mb in (16, 256, 1024):
        n = mb << 20
        src = torch.empty(n, dtype=torch.uint8, device=dev)
        dst = torch.empty(n, dtype=torch.uint8, device=dev)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for name, fn in (("sdma", lambda: _lib.call("toa_emulate_copy_nocu", _lib.ptr(src), _lib.ptr(dst), n,
                                                     _lib.stream(src))),
                         ("ring32_unpaced", lambda: _lib.call("toa_emulate_xfer", _lib.ptr(src), _lib.ptr(dst), n, 32,
                                                              0.0, _lib.stream(src)))):
            fn()
            torch.cuda.synchronize()
            ev[0].record()
            for _ in range(5):
                fn()
            ev[1].record()
            torch.cuda.synchronize()
            ms = ev[0].elapsed_time(ev[1]) / 5
            out[f"{name}_{mb}MiB_GBps"] = round(n / ms / 1e6, 1)
        del src, dst
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
