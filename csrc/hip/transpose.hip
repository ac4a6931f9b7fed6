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

// 8 x 8 block of 16-bit values: row i = 4 dwords, element (i, j) in dword
// j/2, half j&1.  Returns the transposed block in the same format.
__device__ __forceinline__ void tr8x8(const u32x4* in, u32x4* out) {
#pragma unroll
  for (int j = 0; j < 8; j += 2) {
    // out row j   = in[0..7] element j
    // out row j+1 = in[0..7] element j+1
    const int d = j >> 1;
#pragma unroll
    for (int i = 0; i < 8; i += 2) {
      const uint32_t a = in[i][d], b = in[i + 1][d];
      // low halves of a, b -> (a.lo | b.lo << 16); high halves -> (a.hi | b.hi << 16)
      out[j][i >> 1] = __builtin_amdgcn_perm(b, a, 0x05040100u);
      out[j + 1][i >> 1] = __builtin_amdgcn_perm(b, a, 0x07060302u);
    }
  }
}

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

// dst[C][R] (row stride ldd) = src[R][C]^T (row stride lds).  R, C multiples
// of 64, strides multiples of 8 elements, 16-byte aligned bases.
extern "C" int toa_transpose_bf16(const bf16_t* src, int64_t lds_, bf16_t* dst, int64_t ldd, int R, int C,
                                  hipStream_t stream) {
  if (R <= 0 || C <= 0 || R % 64 || C % 64 || lds_ % 8 || ldd % 8 || lds_ < C || ldd < R)
    return (int)hipErrorInvalidValue;
  const int64_t tiles = (int64_t)(R / 64) * (C / 64);
  int64_t blocks = (tiles + 3) / 4;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(transpose_bf16_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, src, lds_, dst, ldd, R, C);
  return (int)hipGetLastError();
}
