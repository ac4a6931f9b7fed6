// Fused dense-layer kernels for the bundled MNIST / estimator payloads
// (SURVEY K1/K2/K3/K8/K9/K12):
//
//   toa_gemm_bias_act : Y = drop(act(X . W^T + b))   bf16 MFMA (32x32x16), fp32
//                       accumulate, bias + ReLU/GELU + inverted dropout in the
//                       epilogue (dropout mask = counter hash of (seed, row, col):
//                       nothing stored, backward regenerates it)
//   toa_bias_act_bwd  : dZ = dY * act'(.) * mask/keep ; db = colsum(dZ)
//   toa_dropout_fwd   : standalone inverted dropout (same hash)
//   toa_accuracy      : #rows with argmax(logits) == label
//
// GEMM geometry: 256-thread workgroup = 2x2 waves, 64x64 output tile, each
// wave one 32x32 MFMA accumulator; K stepped 32 at a time through LDS with
// 80-byte padded rows (conflict-free 16-B fragment reads); arbitrary M, N, K
// (zero-filled edges; 16-byte loads when K % 8 == 0).
#include "toa_common.h"

typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;

__device__ __forceinline__ uint32_t hash3(uint64_t seed, uint64_t idx) {
  // splitmix64 of (seed ^ idx * golden) -> 32 bits (stateless per element)
  uint64_t z = seed + 0x9E3779B97F4A7C15ull * (idx + 1);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (uint32_t)(z >> 32);
}

__device__ __forceinline__ bool keep_elem(uint64_t seed, uint64_t idx, uint32_t thresh) {
  return hash3(seed, idx) < thresh;
}

__device__ __forceinline__ float act_fwd(int act, float z) {
  if (act == 1) return z > 0.f ? z : 0.f;
  if (act == 2) return 0.5f * z * (1.f + erff(z * 0.7071067811865476f));
  return z;
}

#define PADB 80  // padded LDS row: 32 bf16 (64 B) + 16 B

template <bool VEC, bool OUT_BF16>
__global__ __launch_bounds__(256) void gemm_bias_act_kernel(const bf16_t* __restrict__ X, const bf16_t* __restrict__ W,
                                                            const void* __restrict__ bias, int bias_bf16,
                                                            void* __restrict__ Y, int M, int N, int K, int act,
                                                            float keep_prob, uint64_t seed) {
  __shared__ __attribute__((aligned(16))) char sA[64 * PADB];
  __shared__ __attribute__((aligned(16))) char sB[64 * PADB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
  f32x16 acc;
#pragma unroll
  for (int j = 0; j < 16; ++j) acc[j] = 0.f;
  // loader: thread -> (row = tid / 4, 8-element chunk = tid % 4) of a 64 x 32 tile
  const int lrow = tid >> 2, lch = tid & 3;
  for (int k0 = 0; k0 < K; k0 += 32) {
    const int kk = k0 + lch * 8;
    u32x4 va = {0, 0, 0, 0}, vb = {0, 0, 0, 0};
    const int am = m0 + lrow, bn = n0 + lrow;
    if (VEC) {
      if (am < M && kk < K) va = ld16(X + (int64_t)am * K + kk);
      if (bn < N && kk < K) vb = ld16(W + (int64_t)bn * K + kk);
    } else {
      bf16_t ta[8], tb[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        ta[j] = (am < M && kk + j < K) ? X[(int64_t)am * K + kk + j] : (bf16_t)0;
        tb[j] = (bn < N && kk + j < K) ? W[(int64_t)bn * K + kk + j] : (bf16_t)0;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        va[j] = (uint32_t)ta[2 * j] | ((uint32_t)ta[2 * j + 1] << 16);
        vb[j] = (uint32_t)tb[2 * j] | ((uint32_t)tb[2 * j + 1] << 16);
      }
    }
    __syncthreads();
    *(u32x4*)(sA + lrow * PADB + lch * 16) = va;
    *(u32x4*)(sB + lrow * PADB + lch * 16) = vb;
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8 af = __builtin_bit_cast(bf16x8, *(const u32x4*)(sA + (wm * 32 + r) * PADB + ks * 32 + hh * 16));
      const bf16x8 bfr = __builtin_bit_cast(bf16x8, *(const u32x4*)(sB + (wn * 32 + r) * PADB + ks * 32 + hh * 16));
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bfr, acc, 0, 0, 0);
    }
  }
  // epilogue: C[m][n], n = column on the lane, 16 rows per lane
  const int n = n0 + wn * 32 + r;
  if (n >= N) return;
  const float bv = bias == nullptr ? 0.f : (bias_bf16 ? bf2f(((const bf16_t*)bias)[n]) : ((const float*)bias)[n]);
  const uint32_t thresh = (uint32_t)fminf(keep_prob * 4294967296.f, 4294967295.f);
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int m = m0 + wm * 32 + (j & 3) + 8 * (j >> 2) + 4 * hh;
    if (m >= M) continue;
    float y = act_fwd(act, acc[j] + bv);
    if (keep_prob < 1.f) y = keep_elem(seed, (uint64_t)m * N + n, thresh) ? y / keep_prob : 0.f;
    if (OUT_BF16)
      ((bf16_t*)Y)[(int64_t)m * N + n] = f2bf(y);
    else
      ((float*)Y)[(int64_t)m * N + n] = y;
  }
}

extern "C" int toa_gemm_bias_act(int out_bf16, const bf16_t* X, const bf16_t* W, const void* bias, void* Y,
                                 int M, int N, int K, int act, int bias_bf16, int has_dropout, int _unused,
                                 hipStream_t stream) {
  (void)has_dropout;
  (void)_unused;
  dim3 grid((N + 63) / 64, (M + 63) / 64);
  const bool vec = K % 8 == 0;
#define L(V, O)                                                                                          \
  hipLaunchKernelGGL((gemm_bias_act_kernel<V, O>), grid, dim3(256), 0, stream, X, W, bias, bias_bf16, Y, \
                     M, N, K, act, 1.f, (uint64_t)0)
  if (vec) { if (out_bf16) L(true, true); else L(true, false); }
  else { if (out_bf16) L(false, true); else L(false, false); }
#undef L
  return (int)hipGetLastError();
}

extern "C" int toa_gemm_bias_act_dropout(int out_bf16, const bf16_t* X, const bf16_t* W, const void* bias, void* Y,
                                         int M, int N, int K, int act, int bias_bf16, float keep_prob,
                                         uint64_t seed, hipStream_t stream) {
  dim3 grid((N + 63) / 64, (M + 63) / 64);
  const bool vec = K % 8 == 0;
#define L(V, O)                                                                                          \
  hipLaunchKernelGGL((gemm_bias_act_kernel<V, O>), grid, dim3(256), 0, stream, X, W, bias, bias_bf16, Y, \
                     M, N, K, act, keep_prob, seed)
  if (vec) { if (out_bf16) L(true, true); else L(true, false); }
  else { if (out_bf16) L(false, true); else L(false, false); }
#undef L
  return (int)hipGetLastError();
}

// dZ = dY * act'(.) * mask / keep ; db[n] = sum_m dZ[m][n].  Y is the stored
// forward output (post act/dropout); for GELU the pre-activation Z is needed.
template <typename T>
__global__ __launch_bounds__(256) void bias_act_bwd_kernel(const T* __restrict__ dY, const T* __restrict__ Yo,
                                                           const T* __restrict__ Zpre, T* __restrict__ dZ,
                                                           float* __restrict__ db, int M, int N, int act,
                                                           float keep_prob, uint64_t seed) {
  // block = 32 columns x 8 row groups; each thread walks every 8th row (the
  // loads are independent, so the unrolled loop keeps several in flight),
  // then the 8 partial column sums meet in LDS
  __shared__ float red[8][33];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int n = blockIdx.x * 32 + tx;
  const uint32_t thresh = (uint32_t)fminf(keep_prob * 4294967296.f, 4294967295.f);
  float acc = 0.f;
  if (n < N) {
#pragma unroll 4
    for (int m = ty; m < M; m += 8) {
      const int64_t i = (int64_t)m * N + n;
      float g = sizeof(T) == 2 ? bf2f(((const bf16_t*)dY)[i]) : ((const float*)dY)[i];
      if (keep_prob < 1.f) g = keep_elem(seed, (uint64_t)i, thresh) ? g / keep_prob : 0.f;
      if (act == 1) {
        const float y = sizeof(T) == 2 ? bf2f(((const bf16_t*)Yo)[i]) : ((const float*)Yo)[i];
        if (!(y > 0.f)) g = 0.f;
      } else if (act == 2) {
        const float z = sizeof(T) == 2 ? bf2f(((const bf16_t*)Zpre)[i]) : ((const float*)Zpre)[i];
        const float cdf = 0.5f * (1.f + erff(z * 0.7071067811865476f));
        const float pdf = 0.3989422804014327f * __expf(-0.5f * z * z);
        g *= cdf + z * pdf;
      }
      if (sizeof(T) == 2)
        ((bf16_t*)dZ)[i] = f2bf(g);
      else
        ((float*)dZ)[i] = g;
      acc += g;
    }
  }
  red[ty][tx] = acc;
  __syncthreads();
  if (ty == 0 && n < N && db != nullptr) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) t += red[k][tx];  // fixed order: deterministic
    db[n] = t;
  }
}

extern "C" int toa_bias_act_bwd(int dtype, const void* dY, const void* Y, void* dZ, float* db, int M, int N, int act,
                                hipStream_t stream) {
  dim3 grid((N + 31) / 32);
  if (dtype == 0)
    hipLaunchKernelGGL(bias_act_bwd_kernel<bf16_t>, grid, dim3(256), 0, stream, (const bf16_t*)dY, (const bf16_t*)Y,
                       (const bf16_t*)nullptr, (bf16_t*)dZ, db, M, N, act, 1.f, (uint64_t)0);
  else
    hipLaunchKernelGGL(bias_act_bwd_kernel<float>, grid, dim3(256), 0, stream, (const float*)dY, (const float*)Y,
                       (const float*)nullptr, (float*)dZ, db, M, N, act, 1.f, (uint64_t)0);
  return (int)hipGetLastError();
}

extern "C" int toa_bias_act_dropout_bwd(int dtype, const void* dY, const void* Y, const void* Zpre, void* dZ,
                                        float* db, int M, int N, int act, float keep_prob, uint64_t seed,
                                        hipStream_t stream) {
  dim3 grid((N + 31) / 32);
  if (dtype == 0)
    hipLaunchKernelGGL(bias_act_bwd_kernel<bf16_t>, grid, dim3(256), 0, stream, (const bf16_t*)dY, (const bf16_t*)Y,
                       (const bf16_t*)Zpre, (bf16_t*)dZ, db, M, N, act, keep_prob, seed);
  else
    hipLaunchKernelGGL(bias_act_bwd_kernel<float>, grid, dim3(256), 0, stream, (const float*)dY, (const float*)Y,
                       (const float*)Zpre, (float*)dZ, db, M, N, act, keep_prob, seed);
  return (int)hipGetLastError();
}

// standalone inverted dropout; mask regenerated from (seed, index)
template <typename T>
__global__ __launch_bounds__(256) void dropout_kernel(const T* __restrict__ x, T* __restrict__ y, int64_t n,
                                                      float keep_prob, uint64_t seed, uint64_t offset) {
  const uint32_t thresh = (uint32_t)fminf(keep_prob * 4294967296.f, 4294967295.f);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const bool keep = keep_elem(seed, offset + (uint64_t)i, thresh);
    if (sizeof(T) == 2) {
      const float v = bf2f(((const bf16_t*)x)[i]);
      ((bf16_t*)y)[i] = f2bf(keep ? v / keep_prob : 0.f);
    } else {
      const float v = ((const float*)x)[i];
      ((float*)y)[i] = keep ? v / keep_prob : 0.f;
    }
  }
}

extern "C" int toa_dropout_fwd(int dtype, const void* x, void* y, void* _mask_unused, int64_t n, float keep_prob,
                               uint64_t seed, uint64_t offset, hipStream_t stream) {
  (void)_mask_unused;
  const int grid = toa_stream_grid(n, 256);
  if (dtype == 0)
    hipLaunchKernelGGL(dropout_kernel<bf16_t>, dim3(grid), dim3(256), 0, stream, (const bf16_t*)x, (bf16_t*)y, n,
                       keep_prob, seed, offset);
  else
    hipLaunchKernelGGL(dropout_kernel<float>, dim3(grid), dim3(256), 0, stream, (const float*)x, (float*)y, n,
                       keep_prob, seed, offset);
  return (int)hipGetLastError();
}

// one wave per row: argmax over C columns (first max wins), compare to label
template <typename T>
__global__ __launch_bounds__(256) void accuracy_kernel(const T* __restrict__ logits, const int64_t* __restrict__ lab,
                                                       int* __restrict__ correct, int rows, int C) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  float best = -INFINITY;
  int bi = 0x7fffffff;
  for (int c = lane; c < C; c += 64) {
    const float v = sizeof(T) == 2 ? bf2f(((const bf16_t*)logits)[(int64_t)row * C + c])
                                   : ((const float*)logits)[(int64_t)row * C + c];
    if (v > best) { best = v; bi = c; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ob = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
  }
  if (lane == 0 && bi == (int)lab[row]) atomicAdd(correct, 1);
}

extern "C" int toa_accuracy(int dtype, const void* logits, const int64_t* labels, int* correct, int rows, int C,
                            hipStream_t stream) {
  dim3 grid((rows + 3) / 4);
  if (dtype == 0)
    hipLaunchKernelGGL(accuracy_kernel<bf16_t>, grid, dim3(256), 0, stream, (const bf16_t*)logits, labels, correct,
                       rows, C);
  else
    hipLaunchKernelGGL(accuracy_kernel<float>, grid, dim3(256), 0, stream, (const float*)logits, labels, correct,
                       rows, C);
  return (int)hipGetLastError();
}
