// Shared device helpers for the tf_operator_amd CDNA4 (gfx950) kernels.
//
// Conventions used by every kernel in this directory:
//   * bf16 tensors travel as raw 16-bit words (uint16_t) and are loaded/stored
//     8 at a time (16 B per lane, one global_load_dwordx4) -- CDNA guide G13:
//     hipcc never auto-vectorises bf16.
//   * wave64 everywhere: block sizes are multiples of 64, reductions use
//     64-lane shuffles.
//   * every launcher is `extern "C" int toa_*(..., hipStream_t)` returning the
//     hipError_t of the launch, so Python binds them with ctypes and no torch
//     headers are involved in the device build.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#define TOA_WAVE 64

typedef uint16_t bf16_t;
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;

__device__ __forceinline__ float bf2f(bf16_t u) {
  return __uint_as_float(((uint32_t)u) << 16);
}

// Round-to-nearest-even; at -O3 hipcc lowers the __hip_bfloat16 conversion to
// v_cvt_pk_bf16_f32 which also keeps NaNs NaN (MI355X_MICROARCH correctness table).
__device__ __forceinline__ bf16_t f2bf(float f) {
  __hip_bfloat16 h = __float2bfloat16(f);
  return *reinterpret_cast<bf16_t*>(&h);
}

// 8 x bf16 <-> 8 x f32, packed in one 16-byte vector.
__device__ __forceinline__ void unpack8(const u32x4 v, float* f) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(v[i] << 16);
    f[2 * i + 1] = __uint_as_float(v[i] & 0xffff0000u);
  }
}

__device__ __forceinline__ u32x4 pack8(const float* f) {
  u32x4 v;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[i] = (uint32_t)f2bf(f[2 * i]) | ((uint32_t)f2bf(f[2 * i + 1]) << 16);
  }
  return v;
}

__device__ __forceinline__ u32x4 ld16(const void* p) {
  return *reinterpret_cast<const u32x4*>(p);
}
__device__ __forceinline__ void st16(void* p, u32x4 v) {
  *reinterpret_cast<u32x4*>(p) = v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x a multiple of 64 (<= 1024). `red` needs
// blockDim.x/64 floats of LDS. Result broadcast to every thread.
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}

// Online-softmax pair merge: (m, s) <- (m, s) (+) (m2, s2)
__device__ __forceinline__ void lse_merge(float& m, float& s, float m2, float s2) {
  float mn = fmaxf(m, m2);
  if (mn == -INFINITY) return;
  s = s * __expf(m - mn) + s2 * __expf(m2 - mn);
  m = mn;
}

// two floats -> packed bf16x2, round-to-nearest-even (one v_cvt_pk_bf16_f32)
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  typedef __bf16 b2 __attribute__((ext_vector_type(2)));
  const f2 v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, b2));  // one v_cvt_pk_bf16_f32
}

// Grid size for memory-bound grid-stride kernels: cap at 256 CUs x 8 blocks
// (CDNA guide G11).
// Kernel-variant switch for in-process A/B of the streaming kernels
// (defined in optim.hip, set by toa_set_stream_variant).
int toa_stream_variant();

static inline int toa_stream_grid(int64_t work_items, int block) {
  int64_t g = (work_items + block - 1) / block;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}

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

