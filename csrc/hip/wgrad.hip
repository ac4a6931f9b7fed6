// Weight-gradient GEMM on MFMA (the "NT" form of a column-major BLAS):
//
//     C[M][N] (+)= sum_k A[k][m] * B[k][n]          (bf16 in, fp32 accumulate)
//
// with A = dY [T][M] (row stride lda), B = X [T][N] (ldb), C = dW [M][N] (ldc),
// so dW = dY^T X without materialising a transpose.  Both operands are
// contiguous along the OUTPUT dims, not along the reduction: the form
// hipBLASLt is weakest at on gfx950 (1.0-1.17 PF/s against 1.54 PF/s for the
// forward's TN form, profiles/r1_gemm_tuning_coldcache.log) and 30 % of the
// Llama-3-8B step.
//
// Here both tiles are staged into LDS unchanged with global_load_lds (no
// register round trip, overlapped with the previous k-step's MFMAs), and
// the MFMA operands come out of LDS transposed by ds_read_b64_tr_b16 (guide
// T10) -- the same LDS bandwidth as the ds_read_b128 row reads of a TN kernel.
//
//   workgroup: 8 waves (2 M x 4 N), tile 256 x 256, 32 k per phase, 4 LDS
//              stages, the two wave rows staggered by one barrier
//   wave:      128 x 64 of C = 8 x 4 v_mfma_f32_16x16x32_bf16 tiles
//   operands:  swapped (B fragment first) so each lane's accumulator holds 4
//              consecutive n of one row m -> 8-byte read-modify-write stores
//   split-K:   only the tiles that would leave the last wave of 256 CUs
//              part-empty are split: the first `full` tiles (whole waves)
//              run over the whole K and store bf16 directly; the `rem` tail
//              tiles are cut into `split` K-pieces that fill the last wave.
//              Their fp32 partials go to a tile-major workspace and
//              wgrad_tile_reduce_kernel adds them in a fixed order
//              (deterministic, no float atomics).  Full tiles are launched
//              first, so the pieces fill in behind them.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "toa_common.h"

#define WG_BM 256
#define WG_BN 256
#define WG_BK 32                     // k rows per stage (one phase)
#define WG_ROWB 512                  // one LDS row = 256 bf16
#define WG_TILE (WG_BK * WG_ROWB)    // 16 KiB per operand per stage
#define WG_STAGE (2 * WG_TILE)       // A + B
#define WG_NSTAGE 4                  // 4 stages = 128 KiB
// s_waitcnt immediates (gfx9 encoding, expcnt/lgkmcnt left at max)
#define WG_VMCNT0 0x0F70
#define WG_VMCNT4 0x0F74

typedef __attribute__((ext_vector_type(8))) short wg_s16x8;
typedef __attribute__((ext_vector_type(4))) short wg_s16x4;

// Chunk c (16 B, 0..31) of LDS row r lives at chunk position c ^ wg_f(r).  A
// transposed read takes 32 contiguous bytes from each of 8 rows (r0..r0+3 and
// r0+8..r0+11, r0 % 16 in {0, 4}); the XOR puts those 8 segments in 8
// distinct 32-byte bank slots, so every read is conflict-free.
__device__ __forceinline__ int wg_f(int r) { return ((r & 3) | ((r & 8) >> 1)) << 1; }
__device__ __forceinline__ int wg_off(int r, int c) { return r * WG_ROWB + ((c ^ wg_f(r)) << 4); }

__device__ __forceinline__ wg_s16x4 wg_tr(const char* lds, int byte_off) {
  typedef __attribute__((address_space(3))) wg_s16x4 lds_t;
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_t*)(lds + byte_off));
}

// One 32 x 256 operand tile -> LDS stage image: 16 wave-instructions of
// 1 KiB (two rows each); wave w issues rows 4w .. 4w+3.  global_load_lds
// writes lane-linearly, so the swizzle is applied to the SOURCE chunk
// (goff[u]: this lane's element offset, precomputed; g: wave-uniform base,
// so the load uses the scalar-base + 32-bit-offset form).
__device__ __forceinline__ int wg_goff(int64_t ld, int wave, int lane, int u) {
  const int r = 4 * wave + 2 * u + (lane >> 5);
  return (int)(r * ld) + ((lane & 31) ^ wg_f(r)) * 8;
}

__device__ __forceinline__ void wg_stage(const bf16_t* __restrict__ g, const int* goff, char* lds_tile, int wave) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    char* dst = lds_tile + (4 * wave + 2 * u) * WG_ROWB;  // wave-uniform
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(g + (uint32_t)goff[u]),
                                     (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
  }
}

// 16x16x32 operand fragment of rows k0..k0+31 and 16 columns starting at col0:
// lane l gets image[k0 + 8(l>>4) + j][col0 + (l & 15)], j = 0..7.
__device__ __forceinline__ wg_s16x8 wg_frag(const char* img, int k0, int col0, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int r = k0 + 8 * g + q;
  const int c = (col0 >> 3) + (p >> 1);
  const int b = 8 * (p & 1);
  const wg_s16x4 lo = wg_tr(img, wg_off(r, c) + b);
  const wg_s16x4 hi = wg_tr(img, wg_off(r + 4, c) + b);
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

__device__ __forceinline__ int wg_xcd_remap(int bid, int nwg) {
  // bijective XCD grouping (guide §5): consecutive ids land on one XCD's L2
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// tile index -> (tm, tn): group-M order (8 row tiles per group) for L2 reuse
// of the B strips
__device__ __forceinline__ void wg_tile_coords(int tile, int tiles_m, int tiles_n, int* tm, int* tn) {
  const int per_group = 8 * tiles_n, group = tile / per_group, first_m = group * 8;
  const int gsz = min(tiles_m - first_m, 8);
  *tm = first_m + (tile - group * per_group) % gsz;
  *tn = (tile - group * per_group) / gsz;
}

// The tile order of the assembly NT kernel's `map` word (csrc/asm/wgrad_gen.py,
// the TN kernels' encoding): groups of 2^lg tiles of the grouped dimension
// (rows; columns when bit 4 is set) walk the other one.  map 3 is
// wg_tile_coords' order.
__device__ __forceinline__ void wg_tile_coords_map(int tile, int tiles_m, int tiles_n, unsigned map, int* tm,
                                                   int* tn) {
  const int lg = (int)(map & 15u);
  const bool walk = (map >> 4) & 1u;
  const int a_n = walk ? tiles_n : tiles_m, b_n = walk ? tiles_m : tiles_n;
  const int per = b_n << lg, group = tile / per, within = tile - group * per;
  const int first = group << lg, gsz = min(a_n - first, 1 << lg);
  const int ta = first + within % gsz, tb = within / gsz;
  *tm = walk ? tb : ta;
  *tn = walk ? ta : tb;
}

__global__ __launch_bounds__(512, 1) void wgrad_nt_kernel(const bf16_t* __restrict__ A, int64_t lda,
                                                          const bf16_t* __restrict__ B, int64_t ldb,
                                                          bf16_t* __restrict__ C, int64_t ldc, float* __restrict__ W,
                                                          int M, int N, int K, int full, int split, int beta) {
  // Four DISTINCT LDS objects, one per stage, and a loop unrolled by four so
  // every access names its buffer statically: hipcc's wait-count pass then
  // knows a ds_read of one stage cannot alias the LDS-DMA still filling
  // another and emits no vmcnt(0) before it (with one array, or a runtime
  // stage index, it drains the prefetch before every phase's first read).
  __shared__ __attribute__((aligned(1024))) char sb0[WG_STAGE];
  __shared__ __attribute__((aligned(1024))) char sb1[WG_STAGE];
  __shared__ __attribute__((aligned(1024))) char sb2[WG_STAGE];
  __shared__ __attribute__((aligned(1024))) char sb3[WG_STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int tiles_m = M / WG_BM, tiles_n = N / WG_BN, tiles = tiles_m * tiles_n;
  const int rem = tiles - full;
  // blocks [0, full): whole-K tiles; [full, full + rem * split): K-pieces of the tail tiles
  const bool piece = (int)blockIdx.x >= full;
  int tile, s = 0, j = 0;
  if (!piece) {
    tile = wg_xcd_remap(blockIdx.x, full);
  } else {
    const int w2 = wg_xcd_remap(blockIdx.x - full, rem * split);
    s = w2 / rem;
    j = w2 - s * rem;
    tile = full + j;
  }
  int tm, tn;
  wg_tile_coords(tile, tiles_m, tiles_n, &tm, &tn);
  const int kc = piece ? K / split : K, k_begin = s * kc, np = kc / WG_BK;

  const bf16_t* Ab = A + (int64_t)k_begin * lda + (int64_t)tm * WG_BM;
  const bf16_t* Bb = B + (int64_t)k_begin * ldb + (int64_t)tn * WG_BN;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Staggered phases (guide §5 template): wave row wm = 1 runs one barrier
  // behind wm = 0, and every phase is  [ds_reads + LDS-DMA] barrier [MFMAs]
  // barrier.  Each SIMD holds one wave of each row, so while one computes
  // its 32 MFMAs the other reads its next fragments.  LDS-DMA runs two
  // phases ahead; a wave retires its DMA of phase p+1 (vmcnt(4): only the
  // phase p+2 one may stay in flight) before the barrier that precedes the
  // first read of phase p+1 (both rows wait before their first barrier of
  // a phase: exact for the lagging row, one barrier early for the leading
  // one), and restages a buffer only two phases after its last read (4
  // buffers: the lagging row finished it by then).
  const bool lag = wm == 1;
  int ga[2], gb[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    ga[u] = wg_goff(lda, wave, lane, u);
    gb[u] = wg_goff(ldb, wave, lane, u);
  }
  auto sync = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  auto phase = [&](const char* cur, char* pre, int p) {
    wg_s16x8 bf[4], af[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) bf[j] = wg_frag(cur + WG_TILE, 0, wn * 64 + 16 * j, lane);
#pragma unroll
    for (int i = 0; i < 8; ++i) af[i] = wg_frag(cur, 0, wm * 128 + 16 * i, lane);
    // past the end the last stage is re-fetched into a buffer nobody reads
    // again: keeps the DMA count per phase constant (no branches, vmcnt(4))
    const int q = min(p + 2, np - 1);
    wg_stage(Ab + (int64_t)q * WG_BK * lda, ga, pre, wave);
    wg_stage(Bb + (int64_t)q * WG_BK * ldb, gb, pre + WG_TILE, wave);
    __builtin_amdgcn_s_waitcnt(WG_VMCNT4);  // my DMA of phase p+1 retired
    sync();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j], af[i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    sync();
  };

  wg_stage(Ab, ga, sb0, wave);
  wg_stage(Bb, gb, sb0 + WG_TILE, wave);
  wg_stage(Ab + (int64_t)WG_BK * lda, ga, sb1, wave);
  wg_stage(Bb + (int64_t)WG_BK * ldb, gb, sb1 + WG_TILE, wave);
  __builtin_amdgcn_s_waitcnt(WG_VMCNT4);  // phase 0's DMA retired
  sync();
  if (lag) sync();
  for (int p = 0; p < np; p += 4) {
    phase(sb0, sb2, p);
    phase(sb1, sb3, p + 1);
    phase(sb2, sb0, p + 2);
    phase(sb3, sb1, p + 3);
  }
  if (!lag) sync();
  __builtin_amdgcn_s_waitcnt(WG_VMCNT0);  // no LDS-DMA left in flight at exit

  // epilogue: lane holds C[m][n .. n+3], m = row16 + (lane & 15), n = col16 + 4 (lane >> 4)
  const int mrow = tm * WG_BM + wm * 128 + (lane & 15);
  const int ncol = tn * WG_BN + wn * 64 + 4 * (lane >> 4);
  if (!piece) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        bf16_t* p = C + (int64_t)(mrow + 16 * i) * ldc + ncol + 16 * j;
        f32x4 v = acc[i][j];
        if (beta) {
          const uint2 o = *(const uint2*)p;
          v[0] += __uint_as_float(o.x << 16);
          v[1] += __uint_as_float(o.x & 0xffff0000u);
          v[2] += __uint_as_float(o.y << 16);
          v[3] += __uint_as_float(o.y & 0xffff0000u);
        }
        uint2 w;
        w.x = pack2(v[0], v[1]);
        w.y = pack2(v[2], v[3]);
        *(uint2*)p = w;
      }
  } else {
    // tile-major fp32 partial: [split][rem][256][256]
    float* ws = W + ((int64_t)s * rem + j) * (WG_BM * WG_BN);
    const int lrow = wm * 128 + (lane & 15), lcol = wn * 64 + 4 * (lane >> 4);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) *(f32x4*)(ws + (lrow + 16 * i) * WG_BN + lcol + 16 * jj) = acc[i][jj];
  }
}

// Tail tile j of `rem`: C = (beta ? C : 0) + sum_s W[s][j], summed in split order.
// sq != nullptr: each thread also stores the sum of squares of its fp32
// results at sq[(tm tiles_n + tn) 256 + thread] -- the tile's slots in the
// gradient-norm partials the assembly kernel writes for whole-K tiles.
__global__ __launch_bounds__(256) void wgrad_tile_reduce_kernel(const float* __restrict__ W, bf16_t* __restrict__ C,
                                                                int64_t ldc, int M, int N, int full, int rem,
                                                                int split, int beta, unsigned map,
                                                                float* __restrict__ sq) {
  const int j = blockIdx.x;
  int tm, tn;
  wg_tile_coords_map(full + j, M / WG_BM, N / WG_BN, map, &tm, &tn);
  float ss = 0.f;
  for (int e = threadIdx.x; e < WG_BM * WG_BN / 8; e += 256) {
    const int row = e / (WG_BN / 8), col = (e % (WG_BN / 8)) * 8;
    bf16_t* p = C + (int64_t)(tm * WG_BM + row) * ldc + tn * WG_BN + col;
    float acc[8];
    if (beta) {
      unpack8(ld16(p), acc);
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] = 0.f;
    }
    for (int s = 0; s < split; ++s) {
      const f32x4* w = (const f32x4*)(W + ((int64_t)s * rem + j) * (WG_BM * WG_BN) + row * WG_BN + col);
      const f32x4 a = w[0], b = w[1];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        acc[q] += a[q];
        acc[4 + q] += b[q];
      }
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) ss = fmaf(acc[q], acc[q], ss);
    st16(p, pack8(acc));
  }
  if (sq != nullptr) sq[((int64_t)tm * (N / WG_BN) + tn) * 256 + threadIdx.x] = ss;
}

static bool wg_split_ok(int K, int s) { return K % (4 * WG_BK * s) == 0 && K / s >= 16 * WG_BK; }

// The launch plan: `full` whole-K tiles (whole waves of the 256 CUs, one
// workgroup per CU: 128 KiB LDS) and the tail tiles cut into `split` pieces
// so the last wave is as full as possible.  No tail: split 1.
static void wg_plan(int M, int N, int K, int* full, int* split) {
  const int tiles = (M / WG_BM) * (N / WG_BN);
  const int rem = tiles % 256;
  *full = tiles - rem;
  *split = 1;
  if (rem == 0) return;
  int best = 1;
  for (int s = 2; s <= 4; ++s)
    if (rem * s <= 256 && wg_split_ok(K, s)) best = s;
  if (best == 1) {  // nothing to split: the tail runs whole
    *full = tiles;
    return;
  }
  *split = best;
}

// The reduce kernel of a split plan, for the assembly NT kernel
// (csrc/hip/gemm_asm.hip toa_wgrad_asm), which writes the same tile-major
// fp32 partials.
// map: the tile order the pieces were computed in (wg_tile_coords_map).
extern "C" int toa_wgrad_reduce_map_sq(const float* W, bf16_t* C, int64_t ldc, int M, int N, int full, int rem,
                                       int split, int beta, unsigned map, float* sq, hipStream_t stream) {
  if (rem <= 0 || split < 2 || W == nullptr || map >= 32u || (map & 15u) > 6u) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(wgrad_tile_reduce_kernel, dim3(rem), dim3(256), 0, stream, W, C, ldc, M, N, full, rem, split, beta,
                     map, sq);
  return (int)hipGetLastError();
}

extern "C" int toa_wgrad_reduce_map(const float* W, bf16_t* C, int64_t ldc, int M, int N, int full, int rem,
                                    int split, int beta, unsigned map, hipStream_t stream) {
  return toa_wgrad_reduce_map_sq(W, C, ldc, M, N, full, rem, split, beta, map, nullptr, stream);
}

extern "C" int toa_wgrad_reduce(const float* W, bf16_t* C, int64_t ldc, int M, int N, int full, int rem, int split,
                                int beta, hipStream_t stream) {
  return toa_wgrad_reduce_map(W, C, ldc, M, N, full, rem, split, beta, 3u, stream);
}

// Auto plan's split factor (1 = no split-K at all).
extern "C" int toa_wgrad_split(int M, int N, int K) {
  int full, split;
  wg_plan(M, N, K, &full, &split);
  return split;
}

// Bytes of fp32 workspace toa_wgrad needs: split == 0 = the auto plan, else
// `split` K-pieces for every tile.
extern "C" int64_t toa_wgrad_workspace(int M, int N, int K, int split) {
  const int tiles = (M / WG_BM) * (N / WG_BN);
  int full = 0;
  if (split == 0) wg_plan(M, N, K, &full, &split);
  else full = split == 1 ? tiles : 0;
  return split > 1 ? (int64_t)split * (tiles - full) * WG_BM * WG_BN * 4 : 0;
}

// dW[M][N] (+)= dY[K][M]^T X[K][N].  M, N multiples of 256, K of 128 * split,
// row strides multiples of 8 elements, 16-byte aligned bases.  split == 0:
// the auto plan (whole-K waves + a split tail); split >= 1: every tile cut
// into `split` K-pieces (1 = none).
extern "C" int toa_wgrad(const bf16_t* A, int64_t lda, const bf16_t* B, int64_t ldb, bf16_t* C, int64_t ldc,
                         float* W, int M, int N, int K, int split, int beta, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0 || M % WG_BM || N % WG_BN || split < 0 || (lda | ldb | ldc) % 8)
    return (int)hipErrorInvalidValue;
  const int tiles = (M / WG_BM) * (N / WG_BN);
  int full;
  if (split == 0) {
    wg_plan(M, N, K, &full, &split);
  } else {
    full = split == 1 ? tiles : 0;
  }
  if (K % (4 * WG_BK * split) || (split > 1 && W == nullptr) || (split == 1 && full != tiles))
    return (int)hipErrorInvalidValue;
  const int rem = tiles - full;
  const int nwg = full + (split > 1 ? rem * split : 0);
  hipLaunchKernelGGL(wgrad_nt_kernel, dim3(nwg), dim3(512), 0, stream, A, lda, B, ldb, C, ldc, W, M, N, K, full, split,
                     beta);
  if (split > 1 && rem > 0)
    hipLaunchKernelGGL(wgrad_tile_reduce_kernel, dim3(rem), dim3(256), 0, stream, W, C, ldc, M, N, full, rem, split,
                       beta, 3u, (float*)nullptr);
  return (int)hipGetLastError();
}
