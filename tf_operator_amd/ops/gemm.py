"""Row-major bf16 GEMM entry points of the training step.

    linear_fwd(x, w)           y  = x w^T            [M,K] x [N,K] -> [M,N]
    linear_dgrad(dy, w)        dx = dy w             [M,N] x [N,K] -> [M,K]
    wgrad_acc_(g, dy, x)       g += dy^T x           (beta = 1, in place)

The forward / data-gradient forms run on the hand-written assembly kernel
(the default, ``TOA_GEMM=asm``) or on the hipBLASLt layer (csrc/hip/gemm.hip,
one column-major call per form, see there for the transposition algebra;
``TOA_GEMM=nosk``); the weight gradient on the assembly NT kernel
(csrc/asm/wgrad_gen.py), with the HIP NT kernel (csrc/hip/wgrad.hip) as its
fallback.
The per-form solution tables measured by ``scripts/tune_gemm.py`` on an
MI355X are stored next to this file, keyed by the hipBLASLt build.

Modes (``TOA_GEMM``):

* ``asm``: the hand-written gfx950 assembly GEMM (csrc/asm/gemm_gen.py,
  launched from csrc/hip/gemm_asm.hip) for every forward / data-gradient
  GEMM whose shape it takes (M, N multiples of 256, K a multiple of 64 and
  >= 128 -- all Llama forms), with the Llama MLP's SwiGLU fused into the
  gate|up projection's epilogue and its backward into the down projection's
  data gradient (``ops.llm.swiglu_mlp``); anything else as ``nosk``.  No
  hipBLASLt table to load, so nothing to prewarm for these forms.
  ``hip`` is an alias (it named the round-3 HIP TN kernel this replaced).
* ``torch``: torch.matmul, i.e. hipBLASLt's own heuristic.  Per-form
  winners picked in isolation were 2-22 % faster alone, yet the full
  Llama-3-8B step was ~1.3 % SLOWER with them (profiles/r1_gemm_*).
* ``tuned``: the measured per-form table (``gemm_tuning_gfx950.json``).
* ``nosk``: the fastest solution per form among those that are NOT
  stream-K (``gemm_tuning_gfx950_nosk.json``, ``scripts/tune_gemm.py
  --exclude-streamk``).  Stream-K kernels hold one workgroup per CU for the
  whole GEMM, so a collective on another stream gets no CU until it ends
  (profiles/r2_sk_contention; +6.7 % vs +3.4 % under emulated world-8
  ZeRO-1 traffic, profiles/r3_overlap).
* ``auto`` (the default): resolved by :func:`resolve_auto` when the trainer
  starts, to ``asm``.
"""
from __future__ import annotations

import atexit
import ctypes
import json
import os
import threading
import weakref

import torch

from . import _lib

_HERE = os.path.dirname(os.path.abspath(__file__))
TABLE = os.path.join(_HERE, "gemm_tuning_gfx950.json")
TABLE_NOSK = os.path.join(_HERE, "gemm_tuning_gfx950_nosk.json")
_MODE = os.environ.get("TOA_GEMM", "auto")
if _MODE == "hip":
    _MODE = "asm"
_installed = False


def mode() -> str:
    return _MODE


def set_mode(m: str):
    """Select the GEMM policy for this process (before the first GEMM)."""
    global _MODE, _installed
    if m not in ("auto", "torch", "tuned", "nosk", "hip", "asm"):
        raise ValueError(f"unknown GEMM mode {m!r}")
    _MODE = "asm" if m == "hip" else m
    _installed = False


def resolve_auto(world: int = 1) -> str:
    """``auto`` -> ``asm`` (an explicit TOA_GEMM is kept).  Returns the mode
    in force.  The assembly kernel with the library-form slot map, the
    per-shape tile order and the fused SwiGLU epilogues wins in-model: the
    Llama-3-8B step is 5.5 +- 1.6 ms faster than on ``nosk`` (12 ABBA rounds
    in one process, profiles/r5_asm_gemm/inmodel_abba12.log; 9.4 ms less kernel time
    under rocprofv3, profiles/r5_prof1).  Like ``nosk`` it never holds the
    whole chip (one workgroup per tile, no stream-K), so the data-parallel
    collectives overlap it.  Round 4 measured the other way (946.3 vs 930.1
    ms, profiles/r4_wgrad/inmodel_ab.log), before those changes."""
    del world
    if _MODE == "auto":
        set_mode("asm")
    return _MODE


def hipblaslt_build() -> str:
    """Identity of the hipBLASLt library solution indices belong to."""
    for d in ("/opt/rocm/lib", os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib")):
        p = os.path.join(d, "libhipblaslt.so")
        if os.path.exists(p):
            return os.path.basename(os.path.realpath(p))
    return "unknown"


def _install():
    global _installed
    if _installed:
        return
    _installed = True
    if _lib.has("toa_gemm_set_no_streamk"):
        _lib.call("toa_gemm_set_no_streamk", int(_MODE in ("nosk", "asm")))
    table = TABLE_NOSK if _MODE in ("nosk", "asm") else TABLE
    if not os.path.exists(table):
        return
    with open(table) as f:
        tab = json.load(f)
    if tab.get("hipblaslt") != hipblaslt_build():
        return
    for e in tab.get("entries", []):
        if e.get("index", -1) >= 0:
            _lib.call("toa_gemm_set_algo", e["ta"], e["tb"], e["m"], e["n"], e["k"], e["lda"], e["ldb"], e["ldc"],
                      e["beta_nz"], e.get("out_f32", 0), e["index"])


_prewarm_thread = None
_prewarm_dev = None


def prewarm(device=None, background: bool = True):
    """Resolve the installed table's plans (hipBLASLt handle, solution
    lookup, support checks: ~0.47 s of host work, mostly code-object loading,
    at the first GEMM -- profiles/r3_first) ahead of the first step.  With
    `background` it runs on a helper thread -- ctypes drops the GIL, so the
    caller initialises the process group and the model meanwhile -- and the
    thread is returned (the GEMM layer's lock orders the first real GEMM
    after it).  Idempotent; None when the policy uses no table."""
    global _prewarm_thread, _prewarm_dev
    if _MODE not in ("tuned", "nosk") or not _lib.has("toa_gemm_prewarm"):
        return None
    dev = None if device is None else torch.device(device).index
    dev = torch.cuda.current_device() if dev is None else dev
    if _prewarm_thread is not None:
        if _prewarm_dev != dev:
            # started for another device (a caller guessed LOCAL_RANK): the
            # handle it built is not this replica's -- fail loudly
            raise RuntimeError(f"GEMM prewarm ran on cuda:{_prewarm_dev}, trainer binds cuda:{dev}")
        return _prewarm_thread
    _install()
    _prewarm_dev = dev

    def work():
        torch.cuda.set_device(dev)
        _lib.call_ret("toa_gemm_prewarm")

    if not background:
        work()
        return None
    _prewarm_thread = threading.Thread(target=work, name="toa-gemm-prewarm", daemon=True)
    _prewarm_thread.start()
    # the first step no longer waits for it (first_step), so a one-step job
    # can reach interpreter exit while it is inside the HIP / hipBLASLt
    # loaders; a daemon thread killed there takes the process down with a
    # non-zero exit (profiles/r4_fresh2: a one-step probe job Failed after
    # "done: 1 steps").  Join it at exit instead.
    atexit.register(_join_prewarm)
    return _prewarm_thread


def _join_prewarm(timeout: float = 120.0):
    t = _prewarm_thread
    if t is not None and t.is_alive():
        t.join(timeout)


def prewarm_early():
    """Start :func:`prewarm` at process start, on this replica's GPU (the
    device train/dist.py binds: TOA_LOCAL_DEVICE, the pod-resources
    allocation, else LOCAL_RANK), before the process group and the model
    exist.  No-op off the GPU, for the ``torch`` policy, or without the HIP
    library."""
    if not torch.cuda.is_available():
        return None
    resolve_auto()
    from ..train import dist as tdist

    try:
        local = tdist.local_device_index()
    except Exception:  # noqa: BLE001 - e.g. grpc.RpcError (kubelet socket down), ImportError (no grpcio)
        return None  # the trainer's own init (train/dist.py) hits the same lookup and reports it
    if local >= torch.cuda.device_count():
        return None
    return prewarm(torch.device("cuda", local))


def _ok(*ts):
    if _MODE not in ("tuned", "nosk", "asm") or not _lib.has("toa_gemm"):
        return False
    for t in ts:
        if not (t.is_cuda and t.dtype == torch.bfloat16 and t.dim() == 2 and t.stride(1) == 1):
            return False
    return _lib.use_hip(ts[0])


def _gemm(ta, tb, m, n, k, a, lda, b, ldb, c, ldc, beta):
    _install()
    _lib.call("toa_gemm", ta, tb, m, n, k, _lib.ptr(a), lda, _lib.ptr(b), ldb, _lib.ptr(c), ldc, float(beta),
              int(c.dtype == torch.float32), _lib.stream(c))


_asm_first = False

# GEMMs of a GPU training step that left the hand-written kernels for the
# library (hipBLASLt / torch.matmul) under the ``asm`` policy, per (op, shape):
# a user's TFJob at, say, seq 4000 would otherwise run the library for every
# GEMM without a trace.  Warned once per shape on stderr; the bench record
# carries the counts (``gemm_fallbacks``).
_FALLBACKS: dict = {}
_fallback_lock = threading.Lock()


def _fallback(op: str, shape, target: str, why: str):
    key = f"{op} {'x'.join(str(int(d)) for d in shape)} -> {target}"
    with _fallback_lock:
        n = _FALLBACKS.get(key, 0)
        _FALLBACKS[key] = n + 1
    if n == 0:
        import sys

        print(f"[toa.gemm] WARNING: {key} ({why}); later calls of this shape are counted, not logged",
              file=sys.stderr, flush=True)


def fallbacks() -> dict:
    """{"op MxNxK -> target": calls} since the process started (or reset)."""
    with _fallback_lock:
        return dict(_FALLBACKS)


def reset_fallbacks():
    with _fallback_lock:
        _FALLBACKS.clear()


def _why_not_asm(x2: torch.Tensor, w: torch.Tensor, n_mult: int = 256) -> str:
    M, K = x2.shape
    N = w.shape[0]
    if x2.dtype != torch.bfloat16 or w.dtype != torch.bfloat16:
        return f"dtype {x2.dtype}/{w.dtype}, not bf16"
    if M % 256 or N % n_mult:
        return f"M={M} / N={N} not multiples of 256 (tokens per micro-batch x seq, output features)"
    if K % 64 or K < 128:
        return f"K={K} not a multiple of 64 >= 128"
    return "layout: non-unit column stride, unaligned rows or base"


class first_step:
    """Context of a trainer's FIRST step under the hipBLASLt policies: every
    forward / data-gradient GEMM the assembly kernel takes runs on it, so the
    step does not wait for the hipBLASLt plans that :func:`prewarm` is still
    loading on its helper thread (profiles/r4_fresh: model_init ->
    first forward issued 0.48-0.63 s without it).  Deterministic: the first
    step always takes this path, whatever the helper thread's progress, and
    later steps never do.  The MLP stays unfused (ops.llm.swiglu_mlp keys on
    the policy)."""

    def __init__(self, on: bool = True):
        # TOA_GEMM_TN_FIRST=0: the first step stays on the steady-state policy
        self.on = (bool(on) and _MODE in ("nosk", "tuned") and _lib.has("toa_gemm_asm")
                   and os.environ.get("TOA_GEMM_TN_FIRST", "1") != "0")

    def __enter__(self):
        global _asm_first
        self.prev, _asm_first = _asm_first, self.on or _asm_first
        return self

    def __exit__(self, *exc):
        global _asm_first
        _asm_first = self.prev
        return False


def _asm_shape_ok(x2: torch.Tensor, w: torch.Tensor, n_mult: int = 256) -> bool:
    """Operands the assembly GEMM takes (csrc/hip/gemm_asm.hip checks the
    same and refuses anything else): bf16 GPU rows with unit column stride,
    16-byte aligned rows, M and N multiples of 256 (n_mult), K a multiple of
    64 and >= 128."""
    if not (_MODE == "asm" or _asm_first) or not _lib.has("toa_gemm_asm"):
        return False
    if not (x2.is_cuda and x2.dtype == w.dtype == torch.bfloat16 and x2.dim() == 2 and w.dim() == 2):
        return False
    if x2.stride(1) != 1 or w.stride(1) != 1 or x2.stride(0) % 8 or w.stride(0) % 8:
        return False
    M, K = x2.shape
    N = w.shape[0]
    return (M % 256 == 0 and N % n_mult == 0 and K % 64 == 0 and K >= 128 and w.shape[1] == K
            and x2.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0 and _lib.use_hip(x2))


def linear_fwd(x2: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    if _asm_shape_ok(x2, w):
        M, N = x2.shape[0], w.shape[0]
        y = torch.empty(M, N, device=x2.device, dtype=x2.dtype)
        _lib.call("toa_gemm_asm", _lib.ptr(x2), x2.stride(0), _lib.ptr(w), w.stride(0), _lib.ptr(y), N, M, N,
                  x2.shape[1], _lib.stream(x2))
        return y
    lib_ok = _ok(x2, w)
    if _MODE == "asm" and x2.is_cuda and x2.dim() == 2 and w.dim() == 2:
        _fallback("fwd", (x2.shape[0], w.shape[0], x2.shape[1]), "hipBLASLt" if lib_ok else "torch.matmul",
                  _why_not_asm(x2, w))
    if not lib_ok:
        return torch.matmul(x2, w.t())
    M, K = x2.shape
    N = w.shape[0]
    y = torch.empty(M, N, device=x2.device, dtype=x2.dtype)
    _gemm(1, 0, N, M, K, w, w.stride(0), x2, x2.stride(0), y, N, 0.0)
    return y


def linear_dgrad(dy2: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    wt = getattr(w, "_toa_wt", None)
    if wt is not None:  # W^T kept by ops.wt.TransposedWeights: dx = dy (W^T)^T, the forward's form
        return linear_fwd(dy2, wt)
    lib_ok = _ok(dy2, w)
    if _MODE == "asm" and dy2.is_cuda and dy2.dim() == 2 and w.dim() == 2:
        _fallback("dgrad", (dy2.shape[0], w.shape[1], dy2.shape[1]), "hipBLASLt" if lib_ok else "torch.matmul",
                  "no transposed weight copy (ops/wt.py) for this weight")
    if not lib_ok:
        return torch.matmul(dy2, w)
    M, N = dy2.shape
    K = w.shape[1]
    dx = torch.empty(M, K, device=dy2.device, dtype=dy2.dtype)
    _gemm(0, 0, K, M, N, w, w.stride(0), dy2, dy2.stride(0), dx, K, 0.0)
    return dx


def swiglu_gate_up(x2: torch.Tensor, wgu: torch.Tensor):
    """(gu, s) = (x Wgu^T, silu(gate) * up) from ONE assembly GEMM with the
    SwiGLU in its epilogue; None when the kernel cannot take the shapes."""
    if not (_asm_shape_ok(x2, wgu, n_mult=2) and (wgu.shape[0] // 2) % 128 == 0):
        return None
    M, F = x2.shape[0], wgu.shape[0] // 2
    gu = torch.empty(M, 2 * F, device=x2.device, dtype=x2.dtype)
    s = torch.empty(M, F, device=x2.device, dtype=x2.dtype)
    _lib.call("toa_gemm_asm_swiglu", _lib.ptr(x2), x2.stride(0), _lib.ptr(wgu), wgu.stride(0), _lib.ptr(gu), 2 * F,
              _lib.ptr(s), F, M, F, x2.shape[1], _lib.stream(x2))
    return gu, s


def swiglu_down_dgrad(d2: torch.Tensor, wd: torch.Tensor, gu: torch.Tensor):
    """dgu = SwiGLU-backward(gu, ds = d2 Wd) from ONE assembly GEMM on the
    transposed weight copy (ops/wt.py) with the SwiGLU backward in its
    epilogue (ds is never stored); None when the kernel cannot take it."""
    wdt = getattr(wd, "_toa_wt", None)
    if wdt is None or not (_asm_shape_ok(d2, wdt) and gu.is_contiguous() and gu.shape[1] == 2 * wdt.shape[0]
                           and gu.data_ptr() % 16 == 0):
        return None
    M, F = d2.shape[0], wdt.shape[0]
    dgu = torch.empty_like(gu)
    _lib.call("toa_gemm_asm_swiglu_bwd", _lib.ptr(d2), d2.stride(0), _lib.ptr(wdt), wdt.stride(0), _lib.ptr(gu),
              2 * F, _lib.ptr(dgu), 2 * F, M, F, d2.shape[1], _lib.stream(d2))
    return dgu


_ws = {}
HIP_ERROR_INVALID_VALUE = 1
# weight-gradient kernel: the assembly NT kernel (csrc/asm/wgrad_gen.py;
# 1.30-1.50 PF/s at the Llama forms, 1-12 % faster than the HIP kernel and
# bit-identical to it, profiles/r4_wgrad/) where the library carries it, else
# the HIP kernel (csrc/hip/wgrad.hip).  set_wgrad_kernel switches it for
# in-process A/B runs (scripts/wgrad_inmodel_ab.py).
_WGRAD_KERNEL = None


def wgrad_kernel() -> str:
    """``asm`` (default where the library carries it) or ``hip``;
    ``TOA_WGRAD=hip`` forces the HIP kernel without a code change."""
    global _WGRAD_KERNEL
    if _WGRAD_KERNEL is None:
        forced = os.environ.get("TOA_WGRAD", "")
        if forced not in ("", "asm", "hip"):
            raise ValueError(f"TOA_WGRAD={forced!r}: expected asm or hip")
        _WGRAD_KERNEL = forced or ("asm" if _lib.has("toa_wgrad_asm") else "hip")
    return _WGRAD_KERNEL


def set_wgrad_kernel(name: str):
    """asm | hip | asm_v1 (the round-4 assembly schedule, bit-identical: the
    round-to-round A/B of scripts/wgrad_inmodel_ab.py)."""
    global _WGRAD_KERNEL
    if name not in ("asm", "hip", "asm_v1"):
        raise ValueError(f"unknown weight-gradient kernel {name!r}")
    _WGRAD_KERNEL = name


def _workspace(dev, nbytes):
    """Split-K partials scratch, one per (device, stream): a weight gradient
    on a side stream (ops.llm set_mlp_overlap) must not share it with one on
    the main stream."""
    key = (dev, torch.cuda.current_stream(dev).stream_id if torch.device(dev).type == "cuda" else 0)
    t = _ws.get(key)
    if t is None or t.numel() * 4 < nbytes:
        t = torch.empty((nbytes + 3) // 4, device=dev, dtype=torch.float32)
        _ws[key] = t
    return t


def wgrad_hip_ok(g, dy2, x2) -> bool:
    """Shapes/layouts csrc/hip/wgrad.hip takes: bf16, 256-multiple output
    dims, token count a multiple of 64, unit column stride."""
    if not _lib.has("toa_wgrad"):
        return False
    if not (dy2.is_cuda and g.dtype == dy2.dtype == x2.dtype == torch.bfloat16 and g.is_contiguous()):
        return False
    if dy2.dim() != 2 or x2.dim() != 2 or dy2.stride(1) != 1 or x2.stride(1) != 1:
        return False
    T, N = dy2.shape
    K = x2.shape[1]
    return (N % 256 == 0 and K % 256 == 0 and T % 128 == 0 and T >= 1024 and dy2.stride(0) % 8 == 0
            and x2.stride(0) % 8 == 0 and dy2.data_ptr() % 16 == 0 and x2.data_ptr() % 16 == 0
            and g.data_ptr() % 16 == 0 and tuple(g.shape) == (N, K))


class SumsqSession:
    """The clipping norm from partials the weight-gradient kernels write as
    they produce the gradients (no separate pass over the 16 GB of bf16
    gradients at Llama-3-8B): every 2-D weight in `params` whose gradient
    the assembly kernel produces gets a fixed region of `buf`, 256 floats per
    256 x 256 output tile (wgrad_gen.py KARG "sq"; the split-K tail tiles via
    the reduce kernel).  norm_sq() sums the whole buffer in one fixed-order
    pass when every region was written this step and adds the squares of the
    flat ranges outside the regions (embeddings, norm weights); otherwise it
    falls back to the full pass over the gradient.  Only for an unsharded,
    unreduced world-1 update: the partials are of this rank's gradient.
    Differs from the full pass only in summation order and in squaring the
    fp32 tile values before their bf16 rounding."""

    def __init__(self, flat, params):
        self.flat = flat
        want = {id(p) for p in params}
        self.regions = {}      # grad view data_ptr -> (offset in buf, floats, [N, K])
        off = 0
        covered = []
        for sgm in flat.segments:
            p = sgm.param
            if id(p) not in want or p.dim() != 2 or p.shape[0] % 256 or p.shape[1] % 256:
                continue
            n = (p.shape[0] // 256) * (p.shape[1] // 256) * 256
            self.regions[p.main_grad.data_ptr()] = (off, n, tuple(p.shape))
            covered.append((sgm.offset, sgm.offset + sgm.numel))
            off += n
        self.buf = torch.zeros(max(off, 4), device=flat.device, dtype=torch.float32)
        # the flat ranges no region covers, as contiguous runs
        covered.sort()
        self.rest, pos = [], 0
        for a, b in covered:
            if a > pos:
                self.rest.append((pos, a))
            pos = max(pos, b)
        if pos < flat.numel:
            self.rest.append((pos, flat.numel))
        # the small rest ranges (norm weights) in one launch: offsets / lengths on the device
        small = [(a, b - a) for a, b in self.rest if b - a < (1 << 20)]
        self.rest = [(a, b) for a, b in self.rest if b - a >= (1 << 20)]
        self.small = None
        if small and flat.grad.dtype == torch.bfloat16 and len(small) <= 32768:
            t = torch.tensor(small, dtype=torch.int64).t().contiguous().to(flat.device)
            self.small = (t[0], t[1], len(small))
        elif small:
            self.rest = sorted(self.rest + [(a, a + n) for a, n in small])
        self.written = set()
        self.hits = 0           # steps served from the partials (tests, diagnostics)

    def owns(self, g) -> bool:
        return g.data_ptr() in self.regions

    def arm(self, g) -> bool:
        """Point the next weight-gradient launch at g's region."""
        off, n, shape = self.regions[g.data_ptr()]
        if tuple(g.shape) != shape:
            return False
        _lib.call("toa_wgrad_asm_set_sumsq", self.buf.data_ptr() + 4 * off)
        return True

    def norm_sq(self, out, ws):
        """out[0] = the squared gradient norm; the written set is cleared."""
        f = self.flat
        s = _lib.stream(f.grad)
        full = len(self.written) == len(self.regions)
        self.written = set()
        if not full:
            _lib.call("toa_sumsq", _lib.ptr(f.grad), f.grad.numel(), int(f.grad.dtype == torch.bfloat16),
                      _lib.ptr(ws), _lib.ptr(out), 0, s)
            return out
        self.hits += 1
        _lib.call("toa_sum_f32", _lib.ptr(self.buf), self.buf.numel(), _lib.ptr(ws), _lib.ptr(out), 0, s)
        esz = f.grad.element_size()
        for a, b in self.rest:
            _lib.call("toa_sumsq", f.grad.data_ptr() + esz * a, b - a, int(f.grad.dtype == torch.bfloat16),
                      _lib.ptr(ws), _lib.ptr(out), 1, s)
        if self.small is not None:
            offs, lens, n = self.small
            _lib.call("toa_sumsq_ranges", _lib.ptr(f.grad), _lib.ptr(offs), _lib.ptr(lens), n, _lib.ptr(ws),
                      _lib.ptr(out), 1, s)
        return out


_SESSIONS = weakref.WeakSet()   # live SumsqSession objects (each held by its trainer's optimizer)


def _session_for(g):
    for sess in _SESSIONS:
        if sess.owns(g):
            return sess
    return None


def wgrad_hip_(g, dy2, x2, beta=1.0, split=None):
    """g[N,K] (+)= dy2[T,N]^T x2[T,K] on the hand-written MFMA kernel.
    split=None: the kernel's auto plan (whole-K waves, only the tail tiles
    cut into K-pieces); an int: every tile cut into `split` pieces."""
    _lib.use_hip(dy2)
    T, N = dy2.shape
    K = x2.shape[1]
    split = 0 if split is None else int(split)
    nbytes = int(_lib.call_ret("toa_wgrad_workspace", N, K, T, split))
    ws = _workspace(dy2.device, nbytes) if nbytes > 0 else None
    args = (_lib.ptr(dy2), dy2.stride(0), _lib.ptr(x2), x2.stride(0), _lib.ptr(g), K, _lib.ptr(ws),
            N, K, T, int(split), int(beta != 0.0), _lib.stream(dy2))
    kern = wgrad_kernel()
    if kern in ("asm", "asm_v1"):
        sess = _session_for(g) if _SESSIONS else None
        armed = sess is not None and sess.arm(g)
        try:
            rc = (_lib.call_ret("toa_wgrad_asm", *args) if kern == "asm"
                  else _lib.call_ret("toa_wgrad_asm_variant", 1, *args))
        finally:
            if armed:
                _lib.call("toa_wgrad_asm_set_sumsq", None)   # one-shot: never left for another launch
        if rc == 0:
            if armed:
                sess.written.add(g.data_ptr())
            return g
        if rc != HIP_ERROR_INVALID_VALUE:
            raise RuntimeError(f"toa_wgrad_asm failed: hipError {rc}")
        # a shape / layout the assembly kernel's launcher refuses (it checks
        # before launching): the HIP kernel shares its split plan and reduce
    _lib.call("toa_wgrad", *args)
    return g


def wgrad_acc_(g: torch.Tensor, dy2: torch.Tensor, x2: torch.Tensor, beta: float = 1.0):
    """g[N,K] = beta*g + dy2[M,N]^T @ x2[M,K]  (in place; g bf16 or fp32)."""
    if beta in (0.0, 1.0) and wgrad_hip_ok(g, dy2, x2):
        return wgrad_hip_(g, dy2, x2, beta)
    if dy2.is_cuda and g.dtype == torch.bfloat16 and dy2.dim() == 2 and x2.dim() == 2:
        T, N = dy2.shape
        _fallback("wgrad", (N, x2.shape[1], T), "hipBLASLt" if _ok(dy2, x2) else "torch.mm",
                  "output dims not multiples of 256, tokens not a multiple of 128 (>= 1024), or layout")
    if (g.dtype == torch.float32 and dy2.dtype == x2.dtype == torch.bfloat16 and g.is_cuda and g.is_contiguous()
            and dy2.stride(1) == 1 and x2.stride(1) == 1 and _lib.has("toa_gemm")):
        # fp32 master-gradient accumulation (small payloads): one hipBLASLt call
        # with bf16 inputs, fp32 C/D and beta = 1 -- no bf16 temporary, cast or add
        M, N = dy2.shape
        K = x2.shape[1]
        _gemm(0, 1, K, N, M, x2, x2.stride(0), dy2, dy2.stride(0), g, K, beta)
        return g
    if not (_ok(dy2, x2) and g.is_contiguous() and g.dtype in (torch.bfloat16, torch.float32)):
        if beta == 0.0:
            g.copy_(torch.mm(dy2.t(), x2))
        elif g.dtype == dy2.dtype:
            g.addmm_(dy2.t(), x2)
        else:
            g.add_(torch.mm(dy2.t(), x2).to(g.dtype))
        return g
    M, N = dy2.shape
    K = x2.shape[1]
    _gemm(0, 1, K, N, M, x2, x2.stride(0), dy2, dy2.stride(0), g, K, beta)
    return g


def form_keys(T: int, shapes: dict) -> list:
    """The (ta, tb, m, n, k, lda, ldb, ldc, beta_nz) forms of linear layers
    `shapes` = {name: (K, N)} at T tokens (forward, dgrad, wgrad)."""
    out = []
    for name, (K, N) in shapes.items():
        out.append((name, "fwd", (1, 0, N, T, K, K, K, N, 0)))
        out.append((name, "dgrad", (0, 0, K, T, N, K, N, K, 0)))
        # dgrad on the transposed weight copy (ops/wt.py, the default): the forward's form
        out.append((name, "dgrad_wt", (1, 0, K, T, N, N, N, K, 0)))
        out.append((name, "wgrad", (0, 1, K, N, T, K, N, K, 1)))
    return out


def kernel_name(key) -> str:
    """hipBLASLt kernel a form currently runs through this layer ("" if none)."""
    if not _lib.has("toa_gemm_kernel_name"):
        return ""
    buf = ctypes.create_string_buffer(512)
    _lib.call_ret("toa_gemm_kernel_name", *key, 0, buf, 512)
    return buf.value.decode(errors="replace")


def current_algo(key) -> int:
    return _lib.call_ret("toa_gemm_current_algo", *key, 0) if _lib.has("toa_gemm_current_algo") else -1


def tune_form(key, device="cuda", exclude_streamk=False):
    """Time all hipBLASLt solutions for one form on scratch buffers
    (optionally only the non-stream-K ones)."""
    ta, tb, m, n, k, lda, ldb, ldc, beta_nz = key
    a_rows, a_cols = (m, k) if not ta else (k, m)   # column-major op(A) source dims
    b_rows, b_cols = (k, n) if not tb else (n, k)
    # column-major X (rows x cols, ld) == row-major tensor [cols, ld]
    A = torch.randn(a_cols, lda, device=device, dtype=torch.bfloat16)
    B = torch.randn(b_cols, ldb, device=device, dtype=torch.bfloat16)
    C = torch.zeros(n, ldc, device=device, dtype=torch.bfloat16)
    del a_rows, b_rows
    bi, bms, dms, nt = ctypes.c_int(-1), ctypes.c_float(0), ctypes.c_float(0), ctypes.c_int(0)
    rc = _lib.call_ret("toa_gemm_tune", ta, tb, m, n, k, _lib.ptr(A), lda, _lib.ptr(B), ldb, _lib.ptr(C), ldc,
                       float(beta_nz), 0, _lib.stream(C), ctypes.byref(bi), ctypes.byref(bms), ctypes.byref(dms),
                       ctypes.byref(nt), int(bool(exclude_streamk)))
    if rc != 0:
        raise RuntimeError(f"toa_gemm_tune failed ({rc}) for {key}")
    return bi.value, bms.value, dms.value, nt.value


def save_table(entries: list, path: str = TABLE):
    with open(path, "w") as f:
        json.dump({"hipblaslt": hipblaslt_build(), "arch": "gfx950", "entries": entries}, f, indent=1)
