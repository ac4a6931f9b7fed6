// Host side of the hand-written gfx950 assembly GEMMs (csrc/asm/gemm_gen.py).
//
// The build (tf_operator_amd/_build.py) generates the assembly, assembles and
// links it into a code object and embeds the bytes here (toa_asm_blob.inc),
// so the kernels live inside libtoa_hip.so like every other kernel: the
// module is loaded from memory once per device on first use, and launches go
// through hipModuleLaunchKernel on the caller's stream (graph-capturable).
//
//   toa_gemm_asm              C[M][N]  = X[M][K] W[N][K]^T
//   toa_gemm_asm_swiglu       gu = X Wgu^T (Wgu = [gate; up], F rows each),
//                             s = silu(gate) * up              (one launch)
//   toa_gemm_asm_swiglu_bwd   dgu = SwiGLU'(gu) applied to ds = dY WdT^T
//                             (ds never stored)                  (one launch)
//
// Shapes: M, N multiples of 256 (F of 128 forward / 256 backward), K a
// multiple of 64 and >= 128, row strides multiples of 8 elements, 16-byte
// aligned bases.  Anything else returns hipErrorInvalidValue before a launch
// (callers fall back to another GEMM), so the kernel never sees a shape whose
// tiles it does not cover.  The 80-byte argument block matches KARG in
// gemm_gen.py (and csrc/asm/host_args.py, which the CPU emulator tests use).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>

#include "toa_common.h"

namespace {

#include "toa_asm_blob.inc"  // const unsigned char toa_asm_blob[]; size_t toa_asm_blob_len

constexpr int kMaxDev = 64;
enum { K_PLAIN = 0, K_SWIGLU_FWD = 1, K_SWIGLU_BWD = 2, K_PROBE = 3, K_TRACE = 4, K_TIMING = 5, K_TIMING2 = 6,
       K_WGRAD = 7, K_V1 = 8, K_WGRAD_V1 = 16, K_ATTN_FWD = 17, K_ATTN_D1 = 18, K_ATTN_T1 = 23,
       K_ATTN_DKDV = 26, K_DKDV_D1 = 27, K_DKDV_T1 = 34, K_SWIGLU_FWD_R4 = 41, K_SWIGLU_BWD_R4 = 42, K_SWBWD_V1 = 43, K_PLAIN_V9 = 48, K_DKDV_S7 = 49, K_DKDV_D8 = 50, K_DKDV_S8 = 51, K_SWFWD_P1 = 52, K_SWBWD_P1 = 53, K_ROPE = 54, K_DELTA = 55, K_RESADD = 56, K_N = 57 };
// K_V1 .. K_N - 1: the A/B arms of the plain kernel (gemm_gen.py PLAIN_VARIANTS)
const char* kNames[K_N] = {"toa_gemm_tn_asm_plain",    "toa_gemm_tn_asm_swiglu_fwd", "toa_gemm_tn_asm_swiglu_bwd",
                           "toa_gemm_tn_asm_probe",    "toa_gemm_tn_asm_trace",      "toa_gemm_tn_asm_timing",
                           "toa_gemm_tn_asm_timing2",  "toa_wgrad_nt_asm",           "toa_gemm_tn_asm_plain_v1",
                           "toa_gemm_tn_asm_plain_v2", "toa_gemm_tn_asm_plain_v3", "toa_gemm_tn_asm_plain_v4",
                           "toa_gemm_tn_asm_plain_v5", "toa_gemm_tn_asm_plain_v6", "toa_gemm_tn_asm_plain_v7",
                           "toa_gemm_tn_asm_plain_v8", "toa_wgrad_nt_asm_v1",       "toa_attn_fwd_asm",
                           // K_ATTN_D1 ..: attn_gen.py VARIANTS (diagnostic arms, wrong outputs by design)
                           "toa_attn_fwd_asm_d1",      "toa_attn_fwd_asm_d2",        "toa_attn_fwd_asm_d3",
                           "toa_attn_fwd_asm_d4",      "toa_attn_fwd_asm_d5",        "toa_attn_fwd_asm_t1",
                           "toa_attn_fwd_asm_c1",      "toa_attn_fwd_asm_t2",        "toa_attn_dkdv_asm",
                           // K_DKDV_D1 ..: attn_bwd_gen.py VARIANTS (diagnostic arms, wrong outputs by design)
                           "toa_attn_dkdv_asm_d1",     "toa_attn_dkdv_asm_d2",       "toa_attn_dkdv_asm_d3",
                           "toa_attn_dkdv_asm_d4",     "toa_attn_dkdv_asm_d5",       "toa_attn_dkdv_asm_d6",
                           "toa_attn_dkdv_asm_d7",     "toa_attn_dkdv_asm_t1",
                           // schedule-parameter arms (correct outputs)
                           "toa_attn_dkdv_asm_s1",     "toa_attn_dkdv_asm_s2",       "toa_attn_dkdv_asm_s3",
                           "toa_attn_dkdv_asm_s4",     "toa_attn_dkdv_asm_s5",       "toa_attn_dkdv_asm_s6",
                           // the round-4 SwiGLU epilogues (drain per row block): in-model A/B arms
                           "toa_gemm_tn_asm_swiglu_fwd_r4", "toa_gemm_tn_asm_swiglu_bwd_r4",
                           // K_SWBWD_V1 ..: gemm_gen.py SWIGLU_BWD_VARIANTS (diagnostic arms, wrong outputs by design)
                           "toa_gemm_tn_asm_swiglu_bwd_b1", "toa_gemm_tn_asm_swiglu_bwd_b2",
                           "toa_gemm_tn_asm_swiglu_bwd_b3", "toa_gemm_tn_asm_swiglu_bwd_b4",
                           "toa_gemm_tn_asm_swiglu_bwd_b5",
                           // the plain kernel's ninth A/B arm (after the table above was laid out)
                           "toa_gemm_tn_asm_plain_v9",
                           // the dK/dV kernel's arm s7 (attn_bwd_gen.py VARIANTS, appended)
                           "toa_attn_dkdv_asm_s7", "toa_attn_dkdv_asm_d8", "toa_attn_dkdv_asm_s8",
                           // the persistent fused SwiGLU GEMMs (gemm_gen.py SWIGLU_PERSIST_VARIANTS)
                           "toa_gemm_tn_asm_swiglu_fwd_p1", "toa_gemm_tn_asm_swiglu_bwd_p1",
                           // the fused-QKV projection with RoPE + head-major relayout (gemm_gen.py epilogue_rope)
                           "toa_gemm_tn_asm_rope",
                           // the output projection's data gradient with the attention delta (epilogue_delta)
                           "toa_gemm_tn_asm_delta",
                           // C = X W^T + R (epilogue_resadd: the output projection's residual add)
                           "toa_gemm_tn_asm_resadd"};

struct DevModule {
  std::once_flag once;
  hipError_t err = hipSuccess;
  hipModule_t mod = nullptr;
  hipFunction_t fn[K_N] = {};
};
DevModule g_mod[kMaxDev];

hipFunction_t get_fn(int which, hipError_t* err) {
  int dev = 0;
  if ((*err = hipGetDevice(&dev)) != hipSuccess) return nullptr;
  if (dev < 0 || dev >= kMaxDev) {
    *err = hipErrorInvalidDevice;
    return nullptr;
  }
  DevModule& m = g_mod[dev];
  std::call_once(m.once, [&m]() {
    m.err = hipModuleLoadData(&m.mod, toa_asm_blob);
    for (int i = 0; m.err == hipSuccess && i < K_N; ++i) m.err = hipModuleGetFunction(&m.fn[i], m.mod, kNames[i]);
  });
  *err = m.err;
  return m.err == hipSuccess ? m.fn[which] : nullptr;
}

struct __attribute__((packed)) Args {
  uint64_t X, W, C, S;
  uint32_t ldx, ldw, ldc, lds;  // bytes
  uint32_t ktiles, tiles_m, tiles_n, xq, xr, per_group;
  uint32_t fw, fc;  // swiglu: up-half row offset in W (bytes) / column offset in gu (bytes)
  uint32_t map;     // tile order: log2 group | 16 = column groups walk the rows (gemm_gen.py KARG)
  uint32_t grid;    // persistent kernels: the workgroup count
  uint32_t phase;   // first-wave start offsets: n | log2 g << 16 (gemm_gen.py phase_delay; 0 = off)
  uint32_t pad;
};
static_assert(sizeof(Args) == 96, "kernarg block must match csrc/asm/gemm_gen.py KARG_BYTES");

constexpr uint32_t kMapDefault = 2;  // groups of 4 row tiles walk the column tiles
constexpr uint32_t kMapWalkCols = 16;

bool ld_ok(int64_t ld, int64_t min_cols) { return ld >= min_cols && ld % 8 == 0 && ld * 2 * 256 < (1ll << 32); }
bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// The plain kernel's A/B arms by variant number 1.. (gemm_gen.py
// PLAIN_VARIANTS): kernel id, and whether it walks several tiles per
// workgroup (SCHED "persist": its grid is one workgroup per CU).
constexpr int kNumPlainVariants = 9;
constexpr int kVariantFn[kNumPlainVariants] = {K_V1,     K_V1 + 1, K_V1 + 2, K_V1 + 3,  K_V1 + 4,
                                               K_V1 + 5, K_V1 + 6, K_V1 + 7, K_PLAIN_V9};
constexpr bool kVariantPersist[kNumPlainVariants] = {false, false, true, false, false, false, false, true, true};
constexpr unsigned kPersistGrid = 256;

// First-wave start offsets per kernel family (plain / SwiGLU forward /
// SwiGLU backward): the phase word of gemm_gen.py phase_delay.  Set by
// toa_gemm_asm_set_phase (in-process A/B) or TOA_ASM_PHASE_{PLAIN,FWD,BWD}.
uint32_t g_phase[3] = {0, 0, 0};
std::once_flag g_phase_env;

uint32_t phase_word(int which) {
  std::call_once(g_phase_env, [] {
    const char* names[3] = {"TOA_ASM_PHASE_PLAIN", "TOA_ASM_PHASE_FWD", "TOA_ASM_PHASE_BWD"};
    for (int i = 0; i < 3; ++i) {
      const char* e = getenv(names[i]);
      if (e && *e) g_phase[i] = (uint32_t)strtoul(e, nullptr, 0);
    }
  });
  if (which == K_PLAIN) return g_phase[0];
  if (which == K_SWIGLU_FWD || which == K_SWIGLU_FWD_R4) return g_phase[1];
  if (which == K_SWIGLU_BWD || which == K_SWIGLU_BWD_R4) return g_phase[2];
  return 0;
}

int launch(int which, const Args& a, hipStream_t stream, unsigned grid = 0) {
  hipError_t err;
  hipFunction_t fn = get_fn(which, &err);
  if (!fn) return (int)err;
  Args k = a;
  if (which != K_DELTA) k.phase = phase_word(which);   // (the delta kernel's bytes 88..95 are a pointer)
  size_t sz = sizeof(k);
  void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &k, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
  const unsigned nwg = grid ? grid : a.tiles_m * a.tiles_n;
  if (grid) k.grid = grid;  // the persistent kernels read their grid size here
  return (int)hipModuleLaunchKernel(fn, nwg, 1, 1, 256, 1, 1, 0, stream, nullptr, cfg);
}

// Tile order (kernarg `map`) per shape, from the in-process form sweeps
// (profiles/r5_lib2, r5_lib3; scripts/asm_gemm_bench.py --maps).  Both orders
// keep 256 tiles in flight that share their operand strips through each
// XCD's L2 and the Infinity Cache; what differs is how many distinct strips
// the chip streams per k-step.  With a long reduction (K >= 8192: the down
// projection, the wide data gradients) a strip is 4-65 MB, and column groups
// of 4 tiles walking the rows (map 18) stream fewer of them: +1.5..3 % at
// down.fwd / gate_up.dgrad / lm_head.dgrad.  At K = 4096..6144 row groups of
// 4 (map 2) are as fast or 0.5..1 % faster.  Override: TOA_ASM_TILE_MAP.
int g_map_forced = -2;  // -2: TOA_ASM_TILE_MAP not read yet; -1: the per-shape rule

uint32_t tile_map(uint32_t tiles_m, uint32_t tiles_n, uint32_t ktiles) {
  if (g_map_forced == -2) {
    const char* e = getenv("TOA_ASM_TILE_MAP");
    const int v = (e && *e) ? atoi(e) : -1;
    g_map_forced = (v >= 0 && v < 32 && (v & 15) <= 6) ? v : -1;
  }
  const int forced = g_map_forced;
  if (forced >= 0) return (uint32_t)forced;
  (void)tiles_m;
  (void)tiles_n;
  return ktiles >= 128 ? (kMapWalkCols | 2) : kMapDefault;
}

Args base_args(const void* X, int64_t ldx, const void* W, int64_t ldw, void* C, int64_t ldc, int M, int tiles_n,
               int K) {
  Args a;
  memset(&a, 0, sizeof(a));
  a.X = (uint64_t)X;
  a.W = (uint64_t)W;
  a.C = (uint64_t)C;
  a.ldx = (uint32_t)(ldx * 2);
  a.ldw = (uint32_t)(ldw * 2);
  a.ldc = (uint32_t)(ldc * 2);
  a.ktiles = (uint32_t)(K / 64);
  a.tiles_m = (uint32_t)(M / 256);
  a.tiles_n = (uint32_t)tiles_n;
  const uint32_t nwg = a.tiles_m * a.tiles_n;
  a.xq = nwg >> 3;
  a.xr = nwg & 7;
  a.per_group = 8 * a.tiles_n;
  a.map = tile_map(a.tiles_m, a.tiles_n, a.ktiles);
  return a;
}

bool common_ok(int M, int K, int64_t ldx, int64_t ldw, const void* X, const void* W) {
  return M > 0 && M % 256 == 0 && K >= 128 && K % 64 == 0 && ld_ok(ldx, K) && ld_ok(ldw, K) && al16(X) && al16(W) &&
         (int64_t)(M / 256) < (1 << 20);
}

}  // namespace

// A/B: the first-wave start offsets of one kernel family (0 plain, 1 SwiGLU
// forward, 2 SwiGLU backward): word = n | log2 g << 16, each first-wave
// workgroup sleeping ((b >> 3) mod g) * n * 512 cycles (0 = off).
extern "C" int toa_gemm_asm_set_phase(int kind, unsigned word) {
  if (kind < 0 || kind > 2 || (word >> 20) != 0) return (int)hipErrorInvalidValue;
  phase_word(K_PLAIN);  // env defaults read first, so an explicit setting wins
  g_phase[kind] = word;
  return 0;
}

// A/B: force the TN kernels' tile order (a map word) for every launch, -1 =
// the per-shape rule (tile_map).
extern "C" int toa_gemm_asm_set_map(int map) {
  if (map < -1 || map >= 32 || (map >= 0 && (map & 15) > 6)) return (int)hipErrorInvalidValue;
  g_map_forced = map;
  return 0;
}

extern "C" int toa_gemm_asm_available() {
  hipError_t err;
  return get_fn(K_PLAIN, &err) != nullptr ? 1 : 0;
}

// Persistent plain kernel (PLAIN_VARIANTS v3: a workgroup per CU walks its
// tiles, the next tile's first k-tiles staged under the current epilogue).
// In isolation it is 1.5-2.8 % faster at the qkv / o forward and data-gradient
// forms (K <= 6144, N <= 6144; profiles/r6_defer), but in the model the step
// is the same (-0.3 +- 0.8 ms, 8 ABBA rounds, profiles/r6_persist): the chip
// runs these GEMMs at its power cap, so fewer stalls become a lower clock.  So
// the rule (-1) keeps one workgroup per tile everywhere; toa_gemm_asm_set_persist
// / TOA_ASM_PERSIST force the persistent form for the forms above (1) or off (0).
int g_persist = -2;
bool use_persist(int N, int K) {
  if (g_persist == -2) {
    const char* e = getenv("TOA_ASM_PERSIST");
    g_persist = (e && *e) ? (atoi(e) ? 1 : 0) : -1;
  }
  return g_persist == 1 && K <= 6144 && N <= 6144;
}

extern "C" int toa_gemm_asm(const bf16_t* X, int64_t ldx, const bf16_t* W, int64_t ldw, bf16_t* C, int64_t ldc, int M,
                            int N, int K, hipStream_t stream) {
  if (!common_ok(M, K, ldx, ldw, X, W) || N <= 0 || N % 256 || !ld_ok(ldc, N) || !al16(C))
    return (int)hipErrorInvalidValue;
  Args a = base_args(X, ldx, W, ldw, C, ldc, M, N / 256, K);
  if (use_persist(N, K)) {
    const unsigned tiles = a.tiles_m * a.tiles_n;
    return launch(kVariantFn[2], a, stream, tiles < kPersistGrid ? tiles : kPersistGrid);
  }
  return launch(K_PLAIN, a, stream);
}

extern "C" int toa_gemm_asm_set_persist(int v) {
  if (v < -1 || v > 1) return (int)hipErrorInvalidValue;
  g_persist = v;
  return 0;
}

// A/B: variant v of the plain kernel (0 = the product kernel, 1.. = the arms
// gemm_gen.py PLAIN_VARIANTS lists), same arguments and checks as toa_gemm_asm.
extern "C" int toa_gemm_asm_variant(int v, const bf16_t* X, int64_t ldx, const bf16_t* W, int64_t ldw, bf16_t* C,
                                    int64_t ldc, int M, int N, int K, hipStream_t stream) {
  if (v < 0 || v > kNumPlainVariants || !common_ok(M, K, ldx, ldw, X, W) || N <= 0 || N % 256 || !ld_ok(ldc, N) ||
      !al16(C) || (v == 9 && K < 192))
    return (int)hipErrorInvalidValue;
  Args a = base_args(X, ldx, W, ldw, C, ldc, M, N / 256, K);
  if (v > 0 && kVariantPersist[v - 1]) {
    const unsigned tiles = a.tiles_m * a.tiles_n;
    return launch(kVariantFn[v - 1], a, stream, tiles < kPersistGrid ? tiles : kPersistGrid);
  }
  return launch(v == 0 ? K_PLAIN : kVariantFn[v - 1], a, stream);
}

// A/B: the product kernel with an explicit tile order (kernarg `map`, see
// tile_map) instead of the per-shape choice.
extern "C" int toa_gemm_asm_map(int map, const bf16_t* X, int64_t ldx, const bf16_t* W, int64_t ldw, bf16_t* C,
                                int64_t ldc, int M, int N, int K, hipStream_t stream) {
  if (map < 0 || map >= 32 || (map & 15) > 6 || !common_ok(M, K, ldx, ldw, X, W) || N <= 0 || N % 256 ||
      !ld_ok(ldc, N) || !al16(C))
    return (int)hipErrorInvalidValue;
  Args a = base_args(X, ldx, W, ldw, C, ldc, M, N / 256, K);
  a.map = (uint32_t)map;
  return launch(K_PLAIN, a, stream);
}

// Diagnostic: the product kernel with s_memtime stamps (csrc/asm/gemm_gen.py
// SCHED["timing"]); per workgroup and wave, 8 dwords at out + 32 (4 wg + wave):
// three accumulated stretches, start -> loop end, epilogue (shader clocks),
// k-tiles, workgroup id, 0.  which = 1: the stretches are the vmcnt wait, the
// X-free and the W-free barrier; which = 2: the X-DMA, W-DMA and bare-MFMA
// stretches of the main loop.
extern "C" int toa_gemm_asm_timing(int which, void* out, const bf16_t* X, int64_t ldx, const bf16_t* W, int64_t ldw,
                                   bf16_t* C, int64_t ldc, int M, int N, int K, hipStream_t stream) {
  if (!common_ok(M, K, ldx, ldw, X, W) || N <= 0 || N % 256 || !ld_ok(ldc, N) || !al16(C) || !out || !al16(out) ||
      (which != 1 && which != 2))
    return (int)hipErrorInvalidValue;
  Args a = base_args(X, ldx, W, ldw, C, ldc, M, N / 256, K);
  a.S = (uint64_t)out;
  return launch(which == 1 ? K_TIMING : K_TIMING2, a, stream);
}

// Diagnostic: the plain kernel ending after `stage` (1 = prologue DMA landed,
// 2 = main loop done, 0 = everything), for bisecting a hardware fault.
extern "C" int toa_gemm_asm_stage(int stage, const bf16_t* X, int64_t ldx, const bf16_t* W, int64_t ldw, bf16_t* C,
                                  int64_t ldc, int M, int N, int K, hipStream_t stream) {
  if (!common_ok(M, K, ldx, ldw, X, W) || N <= 0 || N % 256 || !ld_ok(ldc, N) || !al16(C) || stage < 0 || stage > 2)
    return (int)hipErrorInvalidValue;
  Args a = base_args(X, ldx, W, ldw, C, ldc, M, N / 256, K);
  a.fc = (uint32_t)stage;
  return launch(K_PLAIN, a, stream);
}

// Diagnostic: host-coherent memory for the trace kernel (readable by the host
// even after a device fault has poisoned the context).
extern "C" void* toa_host_coherent_alloc(size_t bytes) {
  void* p = nullptr;
  if (hipHostMalloc(&p, bytes, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) return nullptr;
  memset(p, 0, bytes);
  return p;
}
extern "C" int toa_host_free(void* p) { return (int)hipHostFree(p); }

// Diagnostic: the plain kernel with progress markers (csrc/asm/gemm_gen.py
// trace_mark) written system-coherently into `trace_host` (32 B per
// workgroup and wave): after a fault, how far every wave got.
extern "C" int toa_gemm_asm_trace(void* trace_host, const bf16_t* X, int64_t ldx, const bf16_t* W, int64_t ldw,
                                  bf16_t* C, int64_t ldc, int M, int N, int K, hipStream_t stream) {
  if (!common_ok(M, K, ldx, ldw, X, W) || N <= 0 || N % 256 || !ld_ok(ldc, N) || !al16(C) || !trace_host)
    return (int)hipErrorInvalidValue;
  void* dev = nullptr;
  hipError_t e = hipHostGetDevicePointer(&dev, trace_host, 0);
  if (e != hipSuccess) return (int)e;
  Args a = base_args(X, ldx, W, ldw, C, ldc, M, N / 256, K);
  a.S = (uint64_t)dev;
  return launch(K_TRACE, a, stream);
}

// Diagnostic: the plain kernel's prologue on the same arguments, every
// workgroup b dumping its registers into out + b * 8704 B (csrc/asm/gemm_gen.py
// probe_kernel).  `out` goes in the S slot and a magic value in fw / fc: an
// argument block that arrives corrupted stores nothing.
extern "C" int toa_gemm_asm_probe(void* out, const bf16_t* X, int64_t ldx, const bf16_t* W, int64_t ldw, bf16_t* C,
                                  int64_t ldc, int M, int N, int K, hipStream_t stream) {
  if (!common_ok(M, K, ldx, ldw, X, W) || N <= 0 || N % 256 || !ld_ok(ldc, N) || !al16(C) || !al16(out))
    return (int)hipErrorInvalidValue;
  Args a = base_args(X, ldx, W, ldw, C, ldc, M, N / 256, K);
  a.S = (uint64_t)out;
  a.fw = 0x626F7270u;
  a.fc = 0x31657461u;
  hipError_t err;
  hipFunction_t fn = get_fn(K_PROBE, &err);
  if (!fn) return (int)err;
  size_t sz = sizeof(a);
  void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &a, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
  return (int)hipModuleLaunchKernel(fn, a.tiles_m * a.tiles_n, 1, 1, 256, 1, 1, 0, stream, nullptr, cfg);
}

// Weight gradient on the assembly NT kernel (csrc/asm/wgrad_gen.py), the
// contract of toa_wgrad (csrc/hip/wgrad.hip): C[M][N] (+)= A[K][M]^T B[K][N],
// split == 0 the auto plan (whole-K tiles for whole waves of 256 CUs, the tail
// cut into k-pieces), split >= 1 every tile cut into `split` pieces; the
// pieces' fp32 partials (workspace W, toa_wgrad_workspace bytes) are summed in
// a fixed order by wgrad.hip's reduce kernel.
extern "C" int toa_wgrad_split(int M, int N, int K);
extern "C" int toa_wgrad_reduce_map(const float* W, bf16_t* C, int64_t ldc, int M, int N, int full, int rem,
                                    int split, int beta, unsigned map, hipStream_t stream);
extern "C" int toa_wgrad_reduce_map_sq(const float* W, bf16_t* C, int64_t ldc, int M, int N, int full, int rem,
                                       int split, int beta, unsigned map, float* sq, hipStream_t stream);

// Gradient-norm partials of the NEXT weight-gradient launch (one-shot; the
// launch consumes it): per tile 256 floats at (tm tiles_n + tn) 256 -- the
// whole-K tiles from the assembly kernel's epilogue (wgrad_gen.py KARG "sq"),
// the k-piece tiles from the reduce kernel.  ops/gemm.py SumsqSession.
static float* g_wgrad_sq = nullptr;
extern "C" int toa_wgrad_asm_set_sumsq(float* sq) {
  g_wgrad_sq = sq;
  return 0;
}

static int wgrad_asm_launch(int which, const bf16_t* A, int64_t lda, const bf16_t* B, int64_t ldb, bf16_t* C,
                            int64_t ldc, float* W, int M, int N, int K, int split, int beta, hipStream_t stream);

// Tile order of the weight-gradient kernel (wgrad_gen.py, the TN kernels'
// map encoding), per shape from the in-process sweep of round 6
// (profiles/r6_wmap; scripts/asm_gemm_bench.py --wgrad --wgrad-maps):
//   * 3 = groups of 8 row (dW row) tiles walking the column tiles: the
//     round-4/5 order, kept where nothing measured faster (qkv, o, down);
//   * tall outputs (tiles_m >= 4 tiles_n) with at most 8 waves of tiles
//     (gate|up: 112 x 16): 18 = groups of 4 COLUMN tiles walking all the row
//     tiles, 3.85 vs 3.97 ms (-3.2 %);
//   * tall outputs with many waves (lm_head: 501 x 16): 2 = row groups of
//     4, 17.50 vs 17.86 ms (-2.0 %).
// toa_wgrad_asm_set_map forces one (in-process A/B; -1 = this rule), as does
// TOA_WGRAD_TILE_MAP.
static int g_wgrad_map_forced = -2;  // -2: TOA_WGRAD_TILE_MAP not read yet
static uint32_t wgrad_tile_map(int tiles_m, int tiles_n) {
  if (g_wgrad_map_forced == -2) {
    const char* e = getenv("TOA_WGRAD_TILE_MAP");
    const int v = (e && *e) ? atoi(e) : -1;
    g_wgrad_map_forced = (v >= 0 && v < 32 && (v & 15) <= 6) ? v : -1;
  }
  if (g_wgrad_map_forced >= 0) return (uint32_t)g_wgrad_map_forced;
  const int64_t tiles = (int64_t)tiles_m * tiles_n;
  if (tiles_m >= 4 * tiles_n) return tiles <= 8 * 256 ? 18u : 2u;
  return 3u;
}
extern "C" int toa_wgrad_asm_set_map(int map) {
  if (map < -1 || map >= 32 || (map >= 0 && (map & 15) > 6)) return (int)hipErrorInvalidValue;
  g_wgrad_map_forced = map;
  return 0;
}

extern "C" int toa_wgrad_asm(const bf16_t* A, int64_t lda, const bf16_t* B, int64_t ldb, bf16_t* C, int64_t ldc,
                             float* W, int M, int N, int K, int split, int beta, hipStream_t stream) {
  return wgrad_asm_launch(K_WGRAD, A, lda, B, ldb, C, ldc, W, M, N, K, split, beta, stream);
}

// A/B: variant v of the weight-gradient kernel (0 = product, 1 = the round-4
// schedule: "spread" slot map, accumulators zeroed before the prologue DMA).
extern "C" int toa_wgrad_asm_variant(int v, const bf16_t* A, int64_t lda, const bf16_t* B, int64_t ldb, bf16_t* C,
                                     int64_t ldc, float* W, int M, int N, int K, int split, int beta,
                                     hipStream_t stream) {
  if (v < 0 || v > 1) return (int)hipErrorInvalidValue;
  return wgrad_asm_launch(v ? K_WGRAD_V1 : K_WGRAD, A, lda, B, ldb, C, ldc, W, M, N, K, split, beta, stream);
}

static int wgrad_asm_launch(int which, const bf16_t* A, int64_t lda, const bf16_t* B, int64_t ldb, bf16_t* C,
                            int64_t ldc, float* W, int M, int N, int K, int split, int beta, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0 || M % 256 || N % 256 || split < 0 || split > 4 || !ld_ok(lda, M) ||
      !ld_ok(ldb, N) || !ld_ok(ldc, N) || !al16(A) || !al16(B) || !al16(C) || (lda * 2) * 64 >= (1ll << 31) ||
      (ldb * 2) * 64 >= (1ll << 31))
    return (int)hipErrorInvalidValue;
  const int tiles = (M / 256) * (N / 256);
  int full;
  if (split == 0) {
    split = toa_wgrad_split(M, N, K);
    full = split > 1 ? tiles - tiles % 256 : tiles;
  } else {
    full = split == 1 ? tiles : 0;
  }
  const int rem = tiles - full;
  if (K % (64 * split) || K / split < 128 || (split > 1 && (W == nullptr || !al16(W))) ||
      (int64_t)split * rem >= (1 << 14))
    return (int)hipErrorInvalidValue;
  Args a;
  memset(&a, 0, sizeof(a));
  a.X = (uint64_t)A;
  a.W = (uint64_t)B;
  a.C = (uint64_t)C;
  a.S = (uint64_t)W;
  a.ldx = (uint32_t)(lda * 2);
  a.ldw = (uint32_t)(ldb * 2);
  a.ldc = (uint32_t)(ldc * 2);
  a.lds = (uint32_t)(beta ? 1 : 0);
  a.ktiles = (uint32_t)(K / 64);
  a.tiles_m = (uint32_t)(M / 256);
  a.tiles_n = (uint32_t)(N / 256);
  a.xq = (uint32_t)full;
  a.xr = (uint32_t)rem;
  a.per_group = (uint32_t)split;
  a.map = wgrad_tile_map(M / 256, N / 256);
  float* sq = g_wgrad_sq;
  g_wgrad_sq = nullptr;
  memcpy(&a.phase, &sq, sizeof(sq));   // bytes 88..95: wgrad_gen.py KARG "sq"
  hipError_t err;
  hipFunction_t fn = get_fn(which, &err);
  if (!fn) return (int)err;
  size_t sz = sizeof(a);
  void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &a, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
  const unsigned nwg = (unsigned)(full + (split > 1 ? rem * split : 0));
  err = hipModuleLaunchKernel(fn, nwg, 1, 1, 256, 1, 1, 0, stream, nullptr, cfg);
  if (err != hipSuccess) return (int)err;
  if (split > 1 && rem > 0) return toa_wgrad_reduce_map_sq(W, C, ldc, M, N, full, rem, split, beta, a.map, sq, stream);
  return 0;
}

// Causal flash-attention forward (csrc/asm/attn_gen.py), the contract of
// toa_attn_fwd (csrc/hip/attention.hip) for the shapes this kernel takes:
// head dim 128, S % 256 == 0, causal (flags bit 0), flags bit 1 = O as
// [B, S, H, D].  One workgroup of 4 waves per (256-row query block, head,
// batch); the 80-byte argument block matches attn_gen.py KARG.
struct __attribute__((packed)) AttnArgs {
  uint64_t q, k, v, o, lse;
  uint32_t B, H, Hk, S;
  float c;  // scale * log2(e)
  uint32_t flags, nqb, rep, g8, pad;
  uint64_t dbg;  // the timing arm's records (attn_gen.py timing_store)
};
static_assert(sizeof(AttnArgs) == 88, "kernarg block must match csrc/asm/attn_gen.py KARG_BYTES");

static int attn_fwd_asm_launch(int which, const bf16_t* q, const bf16_t* k, const bf16_t* v, bf16_t* o, float* lse,
                               int B, int H, int Hk, int S, int D, int flags, float scale, hipStream_t stream,
                               void* dbg = nullptr);

extern "C" int toa_attn_fwd_asm(const bf16_t* q, const bf16_t* k, const bf16_t* v, bf16_t* o, float* lse, int B,
                                int H, int Hk, int S, int D, int flags, float scale, hipStream_t stream) {
  return attn_fwd_asm_launch(K_ATTN_FWD, q, k, v, o, lse, B, H, Hk, S, D, flags, scale, stream);
}

// Diagnostic: arm v (1.. = attn_gen.py VARIANTS, 0 = the product kernel),
// same contract; the arms' outputs are wrong by design (timing only).
extern "C" int toa_attn_fwd_asm_variant(int v, const bf16_t* q, const bf16_t* k, const bf16_t* v_, bf16_t* o,
                                        float* lse, int B, int H, int Hk, int S, int D, int flags, float scale,
                                        hipStream_t stream) {
  if (v < 0 || v > K_ATTN_DKDV - K_ATTN_D1 || K_ATTN_D1 + v - 1 == K_ATTN_T1 || K_ATTN_D1 + v - 1 == K_ATTN_DKDV - 1)
    return (int)hipErrorInvalidValue;  // the timing arms take toa_attn_fwd_asm_timing
  return attn_fwd_asm_launch(v ? K_ATTN_D1 + v - 1 : K_ATTN_FWD, q, k, v_, o, lse, B, H, Hk, S, D, flags, scale,
                             stream);
}

// Diagnostic: the product kernel with s_memtime stamps (attn_gen.py
// timing_store): 8 dwords per (workgroup, wave) at dbg + 32 (4 wg + wave) --
// prologue / loop / epilogue shader cycles, tiles, query block, rescales.
// which = 1: the product schedule's timing arm, 2: the group-placed one's.
extern "C" int toa_attn_fwd_asm_timing(int which, void* dbg, const bf16_t* q, const bf16_t* k, const bf16_t* v,
                                       bf16_t* o, float* lse, int B, int H, int Hk, int S, int D, int flags,
                                       float scale, hipStream_t stream) {
  if (!dbg || !al16(dbg) || (which != 1 && which != 2)) return (int)hipErrorInvalidValue;
  return attn_fwd_asm_launch(which == 1 ? K_ATTN_T1 : K_ATTN_DKDV - 1, q, k, v, o, lse, B, H, Hk, S, D, flags, scale, stream,
                             dbg);
}

static int attn_fwd_asm_launch(int which, const bf16_t* q, const bf16_t* k, const bf16_t* v, bf16_t* o, float* lse,
                               int B, int H, int Hk, int S, int D, int flags, float scale, hipStream_t stream,
                               void* dbg) {
  if (D != 128 || !(flags & 1) || B <= 0 || H <= 0 || Hk <= 0 || H % Hk || S <= 0 || S % 256 || !al16(q) ||
      !al16(k) || !al16(v) || !al16(o) || ((uintptr_t)lse & 3))
    return (int)hipErrorInvalidValue;
  const int64_t nwg = (int64_t)(S / 256) * H * B;
  // the kernel's block-coordinate division works below 2^24; row indices
  // (b H + h) S + q and (b S + q) H + h are 32-bit
  if (nwg >= (1 << 24) || (int64_t)B * H * S >= (1ll << 32) || (int64_t)S * 256 >= (1ll << 31))
    return (int)hipErrorInvalidValue;
  hipError_t err;
  hipFunction_t fn = get_fn(which, &err);
  if (!fn) return (int)err;
  AttnArgs a;
  memset(&a, 0, sizeof(a));
  a.q = (uint64_t)q;
  a.k = (uint64_t)k;
  a.v = (uint64_t)v;
  a.o = (uint64_t)o;
  a.lse = (uint64_t)lse;
  a.B = (uint32_t)B;
  a.H = (uint32_t)H;
  a.Hk = (uint32_t)Hk;
  a.S = (uint32_t)S;
  a.c = scale * 1.4426950408889634f;
  a.flags = (uint32_t)(flags & 3);
  a.nqb = (uint32_t)(S / 256);
  a.rep = (uint32_t)(H / Hk);
  a.g8 = ((int64_t)B * Hk) % 8 == 0 ? 1u : 0u;
  a.dbg = (uint64_t)dbg;
  size_t sz = sizeof(a);
  void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &a, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
  return (int)hipModuleLaunchKernel(fn, (unsigned)nwg, 1, 1, 256, 1, 1, 0, stream, nullptr, cfg);
}

// In-model A/B (scripts/wgrad_inmodel_ab.py epi=r4): 1 = the fused SwiGLU
// GEMMs run the round-4 epilogues (every row block drained); 0 = the
// software-pipelined ones (csrc/asm/gemm_gen.py epilogue_swiglu_bwd_pipe).
static int g_epi_r4 = 0;
extern "C" int toa_gemm_asm_set_epi_variant(int v) {
  if (v < 0 || v > 1) return (int)hipErrorInvalidValue;
  g_epi_r4 = v;
  return 0;
}

// Persistent fused SwiGLU GEMMs (gemm_gen.py SWIGLU_PERSIST_VARIANTS: a
// workgroup per CU walks its tiles, the next tile's first k-tiles staged
// before the current tile's epilogue).  bit 0: the forward, bit 1: the
// backward.  Set by toa_gemm_asm_set_swiglu_persist or TOA_ASM_SWIGLU_PERSIST.
static int g_swiglu_persist = -1;
static int swiglu_persist() {
  if (g_swiglu_persist < 0) {
    const char* e = getenv("TOA_ASM_SWIGLU_PERSIST");
    g_swiglu_persist = (e && *e) ? (atoi(e) & 3) : 0;
  }
  return g_swiglu_persist;
}
extern "C" int toa_gemm_asm_set_swiglu_persist(int v) {
  if (v < 0 || v > 3) return (int)hipErrorInvalidValue;
  g_swiglu_persist = v;
  return 0;
}
static int launch_swiglu(int which, int persist_bit, const Args& a, hipStream_t stream) {
  if (!g_epi_r4 && (swiglu_persist() & persist_bit)) {
    const unsigned tiles = a.tiles_m * a.tiles_n;
    return launch(which == K_SWIGLU_FWD ? K_SWFWD_P1 : K_SWBWD_P1, a, stream,
                  tiles < kPersistGrid ? tiles : kPersistGrid);
  }
  return launch(which, a, stream);
}

extern "C" int toa_gemm_asm_swiglu(const bf16_t* X, int64_t ldx, const bf16_t* Wgu, int64_t ldw, bf16_t* GU,
                                   int64_t ldgu, bf16_t* S, int64_t lds_, int M, int F, int K, hipStream_t stream) {
  if (!common_ok(M, K, ldx, ldw, X, Wgu) || F <= 0 || F % 128 || !ld_ok(ldgu, 2 * F) || !ld_ok(lds_, F) || !al16(GU) ||
      !al16(S) || (int64_t)F * ldw * 2 + 128 * ldw * 2 >= (1ll << 32))
    return (int)hipErrorInvalidValue;
  Args a = base_args(X, ldx, Wgu, ldw, GU, ldgu, M, F / 128, K);
  a.S = (uint64_t)S;
  a.lds = (uint32_t)(lds_ * 2);
  a.fw = (uint32_t)((int64_t)F * ldw * 2);
  a.fc = (uint32_t)(F * 2);
  return g_epi_r4 ? launch(K_SWIGLU_FWD_R4, a, stream) : launch_swiglu(K_SWIGLU_FWD, 1, a, stream);
}

extern "C" int toa_gemm_asm_swiglu_bwd(const bf16_t* dY, int64_t ldy, const bf16_t* WdT, int64_t ldw,
                                       const bf16_t* GU, int64_t ldgu, bf16_t* dGU, int64_t lddgu, int M, int F, int K,
                                       hipStream_t stream) {
  if (!common_ok(M, K, ldy, ldw, dY, WdT) || F <= 0 || F % 256 || !ld_ok(ldgu, 2 * F) || !ld_ok(lddgu, 2 * F) ||
      !al16(GU) || !al16(dGU))
    return (int)hipErrorInvalidValue;
  Args a = base_args(dY, ldy, WdT, ldw, dGU, lddgu, M, F / 256, K);
  a.S = (uint64_t)GU;
  a.lds = (uint32_t)(ldgu * 2);
  a.fc = (uint32_t)(F * 2);
  return g_epi_r4 ? launch(K_SWIGLU_BWD_R4, a, stream) : launch_swiglu(K_SWIGLU_BWD, 2, a, stream);
}

// The fused-QKV projection x Wqkv^T written as RoPE-rotated, head-major
// q | k | v (gemm_gen.py epilogue_rope; replaces toa_rope_fwd): out =
// [B Hq S 128 | B Hkv S 128 | B Hkv S 128] bf16, cossin = cos | sin [2][S][64]
// fp32.  N = (Hq + 2 Hkv) 128 must be a multiple of 256, S of 256, M of S.
extern "C" int toa_gemm_asm_rope(const bf16_t* X, int64_t ldx, const bf16_t* W, int64_t ldw, bf16_t* out,
                                 const float* cossin, int M, int K, int S, int Hq, int Hkv, hipStream_t stream) {
  const int64_t N = (int64_t)(Hq + 2 * Hkv) * 128;
  if (!common_ok(M, K, ldx, ldw, X, W) || Hq <= 0 || Hkv <= 0 || Hq > 4096 || Hkv > 4096 || N % 256 || S <= 0 ||
      S % 256 || M % S || !al16(out) || !al16(cossin) || (int64_t)M * N * 2 >= (1ll << 32) ||
      (int64_t)S * 512 + 128 * 256 >= (1ll << 32))
    return (int)hipErrorInvalidValue;
  Args a = base_args(X, ldx, W, ldw, out, 0, M, (int)(N / 256), K);
  a.S = (uint64_t)cossin;
  a.fw = (uint32_t)S;
  a.fc = (uint32_t)(Hq | (Hkv << 16));
  return launch(K_ROPE, a, stream);
}

// dX = dY Wt^T (the plain TN kernel's C) with the attention backward's
// delta fused (gemm_gen.py epilogue_delta): ndelta[(b H + h) S + s] =
// -sum_d bf16(dX)[t][128 h + d] O[t][128 h + d]; O laid out like dX (row
// stride ldc), N = H 128.  toa_attn_bwd_rope then skips its delta pass.
extern "C" int toa_gemm_asm_delta(const bf16_t* X, int64_t ldx, const bf16_t* W, int64_t ldw, bf16_t* C, int64_t ldc,
                                  const bf16_t* O, float* ndelta, int M, int N, int K, int S, int H,
                                  hipStream_t stream) {
  if (!common_ok(M, K, ldx, ldw, X, W) || N <= 0 || N % 256 || !ld_ok(ldc, N) || !al16(C) || !al16(O) ||
      ndelta == nullptr || ((uintptr_t)ndelta & 3) || H <= 0 || (int64_t)H * 128 != N || S <= 0 || S % 256 || M % S)
    return (int)hipErrorInvalidValue;
  Args a = base_args(X, ldx, W, ldw, C, ldc, M, N / 256, K);
  a.S = (uint64_t)O;
  a.fw = (uint32_t)S;
  a.fc = (uint32_t)H;
  memcpy(&a.phase, &ndelta, sizeof(ndelta));   // bytes 88..95
  return launch(K_DELTA, a, stream);
}

// C = X W^T + R, R bf16 laid out like C (gemm_gen.py epilogue_resadd).
extern "C" int toa_gemm_asm_resadd(const bf16_t* X, int64_t ldx, const bf16_t* W, int64_t ldw, bf16_t* C, int64_t ldc,
                                   const bf16_t* R, int M, int N, int K, hipStream_t stream) {
  if (!common_ok(M, K, ldx, ldw, X, W) || N <= 0 || N % 256 || !ld_ok(ldc, N) || !al16(C) || !al16(R))
    return (int)hipErrorInvalidValue;
  Args a = base_args(X, ldx, W, ldw, C, ldc, M, N / 256, K);
  a.S = (uint64_t)R;
  return launch(K_RESADD, a, stream);
}

// DIAGNOSTIC: arm v (1..) of the fused SwiGLU backward (gemm_gen.py
// SWIGLU_BWD_VARIANTS: the main loop alone, no loads, no math, no stores),
// same arguments and checks as toa_gemm_asm_swiglu_bwd; v = 0 the product.
extern "C" int toa_gemm_asm_swiglu_bwd_variant(int v, const bf16_t* dY, int64_t ldy, const bf16_t* WdT, int64_t ldw,
                                               const bf16_t* GU, int64_t ldgu, bf16_t* dGU, int64_t lddgu, int M,
                                               int F, int K, hipStream_t stream) {
  if (v < 0 || v > K_PLAIN_V9 - K_SWBWD_V1 || !common_ok(M, K, ldy, ldw, dY, WdT) || F <= 0 || F % 256 ||
      !ld_ok(ldgu, 2 * F) || !ld_ok(lddgu, 2 * F) || !al16(GU) || !al16(dGU))
    return (int)hipErrorInvalidValue;
  Args a = base_args(dY, ldy, WdT, ldw, dGU, lddgu, M, F / 256, K);
  a.S = (uint64_t)GU;
  a.lds = (uint32_t)(ldgu * 2);
  a.fc = (uint32_t)(F * 2);
  return launch(v == 0 ? K_SWIGLU_BWD : K_SWBWD_V1 + v - 1, a, stream);
}

// Causal flash-attention dK / dV backward of the dS form (csrc/asm/attn_bwd_gen.py),
// the contract of attention.hip's attn_bwd_dkdv_ds_kernel for the shapes this
// kernel takes: head dim 128, S % 256 == 0; nlse2 / ndelta the delta pass's
// -lse log2(e) / -delta rows; ds the dQ GEMM's packed dS blocks.  flags bit 0:
// dO as [B, S, H, D]; bit 1: RoPE -- dK rotated back with cos / sin [S, 64]
// and dK / dV written into the k / v parts of d(qkv) rows [B S, H3 D] (dk ==
// dv == dqkv).  One workgroup of 4 waves per (128-key block, kv head, batch),
// heaviest key blocks first; the 144-byte argument block matches KARG there.
struct __attribute__((packed)) DkdvArgs {
  uint64_t q, k, v, dout, nlse2, ndelta, dk, dv, ds, cosv, sinv, dbg;
  uint32_t B, H, Hk, S;
  float scale, c;  // scale, scale * log2(e)
  uint32_t flags, rep, nkb, H3, pad[2];
};
static_assert(sizeof(DkdvArgs) == 144, "kernarg block must match csrc/asm/attn_bwd_gen.py KARG_BYTES");

static int attn_dkdv_launch(int which, const bf16_t* q, const bf16_t* k, const bf16_t* v, const bf16_t* dout,
                            const float* nlse2, const float* ndelta, bf16_t* dk, bf16_t* dv, bf16_t* ds, int B, int H,
                            int Hk, int S, int D, float scale, int flags, const float* cosv, const float* sinv, int H3,
                            hipStream_t stream, void* dbg = nullptr);

// In-model A/B: toa_attn_dkdv_asm_set_arm(1) runs the packed-VALU arm (s7,
// the round-5 form) in place of the product kernel; 0 = the product.
static int g_dkdv_arm = 0;
extern "C" int toa_attn_dkdv_asm_set_arm(int v) {
  if (v < 0 || v > 1) return (int)hipErrorInvalidValue;
  g_dkdv_arm = v;
  return 0;
}

extern "C" int toa_attn_dkdv_asm(const bf16_t* q, const bf16_t* k, const bf16_t* v, const bf16_t* dout,
                                 const float* nlse2, const float* ndelta, bf16_t* dk, bf16_t* dv, bf16_t* ds, int B,
                                 int H, int Hk, int S, int D, float scale, int flags, const float* cosv,
                                 const float* sinv, int H3, hipStream_t stream) {
  return attn_dkdv_launch(g_dkdv_arm ? K_DKDV_S7 : K_ATTN_DKDV, q, k, v, dout, nlse2, ndelta, dk, dv, ds, B, H, Hk, S,
                          D, scale, flags, cosv, sinv, H3, stream);
}

// Diagnostic: arm v (1.. = attn_bwd_gen.py VARIANTS, 0 = the product kernel),
// same contract; the arms' outputs are wrong by design (timing only).
extern "C" int toa_attn_dkdv_asm_variant(int v, const bf16_t* q, const bf16_t* k, const bf16_t* v_,
                                         const bf16_t* dout, const float* nlse2, const float* ndelta, bf16_t* dk,
                                         bf16_t* dv, bf16_t* ds, int B, int H, int Hk, int S, int D, float scale,
                                         int flags, const float* cosv, const float* sinv, int H3, hipStream_t stream) {
  // arms 1..14 sit at K_DKDV_D1.., arms 15.. (s7, d8, s8) were appended from K_DKDV_S7
  constexpr int kDkdvArms = K_SWIGLU_FWD_R4 - K_DKDV_D1;
  if (v < 0 || v > kDkdvArms + (K_DKDV_S8 - K_DKDV_S7 + 1) || (v && v <= kDkdvArms && K_DKDV_D1 + v - 1 == K_DKDV_T1))
    return (int)hipErrorInvalidValue;  // the timing arm takes its own entry
  const int which = v == 0 ? K_ATTN_DKDV : (v <= kDkdvArms ? K_DKDV_D1 + v - 1 : K_DKDV_S7 + v - kDkdvArms - 1);
  return attn_dkdv_launch(which, q, k, v_, dout, nlse2, ndelta, dk, dv, ds, B, H, Hk, S, D, scale, flags, cosv, sinv,
                          H3, stream);
}

// Diagnostic: the product kernel with s_memtime stamps (attn_bwd_gen.py
// timing_store): 8 dwords per (workgroup, wave) at dbg + 32 (4 wg + wave) --
// loop cycles (lo, hi), steps, key block.
extern "C" int toa_attn_dkdv_asm_timing(void* dbg, const bf16_t* q, const bf16_t* k, const bf16_t* v,
                                        const bf16_t* dout, const float* nlse2, const float* ndelta, bf16_t* dk,
                                        bf16_t* dv, bf16_t* ds, int B, int H, int Hk, int S, int D, float scale,
                                        int flags, const float* cosv, const float* sinv, int H3, hipStream_t stream) {
  if (!dbg || !al16(dbg)) return (int)hipErrorInvalidValue;
  return attn_dkdv_launch(K_DKDV_T1, q, k, v, dout, nlse2, ndelta, dk, dv, ds, B, H, Hk, S, D, scale, flags, cosv,
                          sinv, H3, stream, dbg);
}

static int attn_dkdv_launch(int which, const bf16_t* q, const bf16_t* k, const bf16_t* v, const bf16_t* dout,
                            const float* nlse2, const float* ndelta, bf16_t* dk, bf16_t* dv, bf16_t* ds, int B, int H,
                            int Hk, int S, int D, float scale, int flags, const float* cosv, const float* sinv, int H3,
                            hipStream_t stream, void* dbg) {
  const bool rope = (flags & 2) != 0;
  if (D != 128 || B <= 0 || H <= 0 || Hk <= 0 || H % Hk || S <= 0 || S % 256 || !al16(q) || !al16(k) || !al16(v) ||
      !al16(dout) || !al16(dk) || !al16(dv) || !al16(ds) || ((uintptr_t)nlse2 & 3) || ((uintptr_t)ndelta & 3) ||
      (flags & ~3) || (rope && (!cosv || !sinv || !al16(cosv) || !al16(sinv) || H3 != H + 2 * Hk)))
    return (int)hipErrorInvalidValue;
  const int64_t nb = S / 32, nblk = nb * (nb + 1) / 2;
  const int64_t nwg = (int64_t)(S / 128) * B * Hk;
  // 32-bit offsets inside the kernel: dS blocks of one batch, dO / Q rows of
  // one batch, d(qkv) rows; block-coordinate division below 2^24
  if (nwg >= (1 << 24) || (int64_t)H * nblk * 2048 >= (1ll << 32) || (int64_t)S * H * 256 >= (1ll << 31) ||
      (int64_t)B * S * (rope ? H3 : Hk) * 256 >= (1ll << 40))
    return (int)hipErrorInvalidValue;
  hipError_t err;
  hipFunction_t fn = get_fn(which, &err);
  if (!fn) return (int)err;
  DkdvArgs a;
  memset(&a, 0, sizeof(a));
  a.q = (uint64_t)q;
  a.k = (uint64_t)k;
  a.v = (uint64_t)v;
  a.dout = (uint64_t)dout;
  a.nlse2 = (uint64_t)nlse2;
  a.ndelta = (uint64_t)ndelta;
  a.dk = (uint64_t)dk;
  a.dv = (uint64_t)dv;
  a.ds = (uint64_t)ds;
  a.cosv = (uint64_t)cosv;
  a.sinv = (uint64_t)sinv;
  a.B = (uint32_t)B;
  a.H = (uint32_t)H;
  a.Hk = (uint32_t)Hk;
  a.S = (uint32_t)S;
  a.scale = scale;
  a.c = scale * 1.4426950408889634f;
  a.flags = (uint32_t)flags;
  a.rep = (uint32_t)(H / Hk);
  a.nkb = (uint32_t)(S / 128);
  a.H3 = (uint32_t)(rope ? H3 : 0);
  a.dbg = (uint64_t)dbg;
  size_t sz = sizeof(a);
  void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &a, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
  return (int)hipModuleLaunchKernel(fn, (unsigned)nwg, 1, 1, 256, 1, 1, 0, stream, nullptr, cfg);
}
