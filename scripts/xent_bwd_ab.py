"""Cross-entropy backward at the bench shape (24576 rows x 128256 vocab,
bf16 logits) with 1, 2 or 4 chunks of 8 per thread per round
(toa_xent_set_unroll), interleaved rounds in one process; outputs compared
bit for bit.

    python scripts/xent_bwd_ab.py [--rows 24576] [--vocab 128256] [--rounds 6]
"""
import argparse
import json
import statistics
import sys

import torch

sys.path.insert(0, ".")
from tf_operator_amd.ops import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=24576)
    ap.add_argument("--vocab", type=int, default=128256)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    R, V = a.rows, a.vocab
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    logits = (torch.randn(R, V, device=dev) * 2).to(torch.bfloat16)
    tgt = torch.randint(0, V, (R,), device=dev)
    lse = torch.logsumexp(logits.float(), dim=1).contiguous()
    gout = torch.ones(1, device=dev)
    nval = torch.full((1,), float(R), device=dev)
    outs = {u: torch.empty_like(logits) for u in (1, 2, 4)}

    def run(u):
        _lib.call("toa_xent_set_unroll", u)
        _lib.call("toa_xent_bwd", 0, _lib.ptr(logits), _lib.ptr(tgt), _lib.ptr(lse), _lib.ptr(gout), _lib.ptr(nval),
                  _lib.ptr(outs[u]), R, V, V, -100, _lib.stream(logits))

    times = {u: [] for u in outs}
    for r in range(a.rounds):
        for u in (outs if r % 2 == 0 else list(outs)[::-1]):
            run(u)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                run(u)
            e1.record()
            torch.cuda.synchronize()
            times[u].append(e0.elapsed_time(e1) / a.reps)
    _lib.call("toa_xent_set_unroll", 2)
    nbytes = 2 * R * V * 2
    out = {f"u{u}": {"ms": round(statistics.median(t), 4), "TBps": round(nbytes / statistics.median(t) / 1e9, 2)}
           for u, t in times.items()}
    out["bit_identical"] = all(torch.equal(outs[1], outs[u]) for u in (2, 4))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
