// bf16 matrix transpose: dst[C][R] = src[R][C]^T.
//
// Used to keep a transposed copy W^T of every linear weight, refreshed once
// per optimizer step, so the backward's data gradient dX = dY W runs as the
// same "x w^T" GEMM form as the forward (hipBLASLt's fastest form on gfx950:
// 1.44-1.58 PF/s against 1.1-1.4 PF/s for the dY W form it replaces,
// profiles/r1_gemm_tuning_coldcache.log).
//
// Pure data movement, HBM bound: one wave moves one 64 x 64 tile in
// registers, no LDS.  Lane (rb, cb) = (lane >> 3, lane & 7) owns the 8 x 8
// block at rows 8 rb.., cols 8 cb..: it loads 8 rows of 16 B (the 8 lanes
// of one rb read 128 contiguous bytes of a row), transposes the block in
// registers (v_perm byte selects), and stores 8 rows of 16 B of dst (the 8
// lanes of one cb write 128 contiguous bytes).  All 8 loads are issued
// before the first store; loads and stores non-temporal (W^T is read next
// in the backward, long after any cache would have kept it).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "toa_common.h"

// tr8x8: toa_common.h (shared with the fused AdamW + W^T kernel, optim.hip)

__global__ __launch_bounds__(256) void transpose_bf16_kernel(const bf16_t* __restrict__ src, int64_t lds_,
                                                             bf16_t* __restrict__ dst, int64_t ldd, int R, int C) {
  const int lane = threadIdx.x & 63;
  const int rb = lane >> 3, cb = lane & 7;
  const int tiles_c = C >> 6;
  const int64_t ntiles = (int64_t)(R >> 6) * tiles_c;
  const int64_t wstride = (int64_t)gridDim.x * (blockDim.x >> 6);
  for (int64_t t = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); t < ntiles; t += wstride) {
    const int tr = (int)(t / tiles_c), tc = (int)(t - (int64_t)tr * tiles_c);
    const int r0 = tr * 64 + 8 * rb, c0 = tc * 64 + 8 * cb;
    u32x4 in[8], out[8];
    const bf16_t* s = src + (int64_t)r0 * lds_ + c0;
#pragma unroll
    for (int i = 0; i < 8; ++i) in[i] = __builtin_nontemporal_load((const u32x4*)(s + i * lds_));
    tr8x8(in, out);
    bf16_t* d = dst + (int64_t)c0 * ldd + r0;
#pragma unroll
    for (int j = 0; j < 8; ++j) __builtin_nontemporal_store(out[j], (u32x4*)(d + j * ldd));
  }
}

// LDS-staged form for R, C multiples of 128: a workgroup moves one 128 x 128
// tile per round.  Global loads: 16 lanes read one source row's 256
// contiguous bytes; LDS image: row r at 256 r bytes, its 16-byte chunk c at
// chunk c ^ ((r >> 3) & 15) (XOR swizzle: the writes and the transposed
// 8 x 8 block reads below are both conflict-free); each thread then reads
// the 8 x 8 block at rows 8a.., chunk b (a = tid & 15, b = tid >> 4),
// transposes it in registers and stores 8 destination rows of 16 B, the 16
// lanes of one b writing 256 contiguous bytes of a destination row.  Both
// HBM sides move 256-byte runs instead of the register kernel's 128.
__global__ __launch_bounds__(256) void transpose_bf16_lds_kernel(const bf16_t* __restrict__ src, int64_t lds_,
                                                                 bf16_t* __restrict__ dst, int64_t ldd, int R, int C) {
  __shared__ u32x4 tile[128 * 16];
  const int tid = threadIdx.x;
  const int tiles_c = C >> 7;
  const int64_t ntiles = (int64_t)(R >> 7) * tiles_c;
  const int lr = tid >> 4, lc = tid & 15;   // load: row lr + 16 p, chunk lc
  const int a = tid & 15, b = tid >> 4;     // store: source rows 8a.., chunk b
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int tr = (int)(t / tiles_c), tc = (int)(t - (int64_t)tr * tiles_c);
    const int64_t r0 = (int64_t)tr * 128, c0 = (int64_t)tc * 128;
    u32x4 v[8];
#pragma unroll
    for (int p = 0; p < 8; ++p)
      v[p] = __builtin_nontemporal_load((const u32x4*)(src + (r0 + lr + 16 * p) * lds_ + c0 + 8 * lc));
    __syncthreads();   // the previous round's reads of the tile are done
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      const int r = lr + 16 * p;
      tile[r * 16 + (lc ^ ((r >> 3) & 15))] = v[p];
    }
    __syncthreads();
    u32x4 in[8], out[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) in[i] = tile[(8 * a + i) * 16 + (b ^ a)];
    tr8x8(in, out);
    bf16_t* d = dst + (c0 + 8 * b) * ldd + r0 + 8 * a;
#pragma unroll
    for (int j = 0; j < 8; ++j) __builtin_nontemporal_store(out[j], (u32x4*)(d + j * ldd));
  }
}

// 1: the LDS-staged kernel where it applies; 0: the register kernel.  Measured
// (profiles/r6_stream/transpose.log): the down projection 0.0523 -> 0.0476 ms,
// gate|up -2 %, qkv / o +2..3 %, lm_head equal; 5.90 vs 6.07 ms per step.
static int g_transpose_variant = 1;
extern "C" int toa_transpose_set_variant(int v) {
  if (v < 0 || v > 1) return (int)hipErrorInvalidValue;
  g_transpose_variant = v;
  return 0;
}

// dst[C][R] (row stride ldd) = src[R][C]^T (row stride lds).  R, C multiples
// of 64, strides multiples of 8 elements, 16-byte aligned bases.
extern "C" int toa_transpose_bf16(const bf16_t* src, int64_t lds_, bf16_t* dst, int64_t ldd, int R, int C,
                                  hipStream_t stream) {
  if (R <= 0 || C <= 0 || R % 64 || C % 64 || lds_ % 8 || ldd % 8 || lds_ < C || ldd < R)
    return (int)hipErrorInvalidValue;
  if (g_transpose_variant == 1 && R % 128 == 0 && C % 128 == 0) {
    const int64_t tiles128 = (int64_t)(R / 128) * (C / 128);
    const int blocks = (int)(tiles128 < 16384 ? tiles128 : 16384);
    hipLaunchKernelGGL(transpose_bf16_lds_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, src, lds_, dst, ldd, R,
                       C);
    return (int)hipGetLastError();
  }
  const int64_t tiles = (int64_t)(R / 64) * (C / 64);
  int64_t blocks = (tiles + 3) / 4;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(transpose_bf16_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, src, lds_, dst, ldd, R, C);
  return (int)hipGetLastError();
}
