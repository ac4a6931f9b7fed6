// Fused optimizer kernels over FLAT parameter storage (gfx950).
//
// Design (MI355X-first): every trainable parameter of a model lives in one
// contiguous bf16 buffer (compute copy), with matching contiguous fp32 master /
// exp_avg / exp_avg_sq buffers and one contiguous bf16 gradient buffer.  An
// optimizer step is therefore ONE streaming kernel over N elements instead of
// a multi-tensor launch list: 16 B bf16 loads, 2x16 B fp32 loads per stream,
// grid capped at 2048 blocks and grid-strided (CDNA guide G11/G13).  Gradient
// clipping reads the global grad-norm^2 from device memory, so the step never
// synchronises with the host.
//
// Reference parity: the reference payload's Adam (examples/v1/dist-mnist/
// dist_mnist.py:194,208 ; multi_worker_strategy-with-keras.py:56) -- SURVEY K5.
#include "toa_common.h"

#include <algorithm>

// ---------------------------------------------------------------------------
// sum of squares of a bf16 (or fp32) vector, two-pass deterministic reduction
// ---------------------------------------------------------------------------
template <bool BF16>
__global__ __launch_bounds__(256) void sumsq_partial_kernel(const void* __restrict__ x, int64_t n,
                                                            float* __restrict__ partial) {
  __shared__ float red[4];
  float acc = 0.f;
  const int64_t n8 = n / 8;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8;
       i += (int64_t)gridDim.x * blockDim.x) {
    float f[8];
    if (BF16) {
      unpack8(ld16((const bf16_t*)x + i * 8), f);
    } else {
      f32x4 a = *((const f32x4*)x + 2 * i), b = *((const f32x4*)x + 2 * i + 1);
      f[0] = a[0]; f[1] = a[1]; f[2] = a[2]; f[3] = a[3];
      f[4] = b[0]; f[5] = b[1]; f[6] = b[2]; f[7] = b[3];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) acc = fmaf(f[j], f[j], acc);
  }
  // tail (n % 8) handled by block 0
  if (blockIdx.x == 0) {
    for (int64_t i = n8 * 8 + threadIdx.x; i < n; i += blockDim.x) {
      float f = BF16 ? bf2f(((const bf16_t*)x)[i]) : ((const float*)x)[i];
      acc = fmaf(f, f, acc);
    }
  }
  float t = block_sum(acc, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = t;
}

__global__ __launch_bounds__(256) void sum_partials_kernel(const float* __restrict__ partial, int np,
                                                           float* __restrict__ out, int accumulate) {
  __shared__ float red[4];
  float acc = 0.f;
  for (int i = threadIdx.x; i < np; i += blockDim.x) acc += partial[i];
  float t = block_sum(acc, red);
  if (threadIdx.x == 0) out[0] = accumulate ? out[0] + t : t;
}

// Plain sum of an fp32 vector, the same two passes (the gradient-norm
// partials that the weight-gradient kernels write, ops/gemm.py SumsqSession).
__global__ __launch_bounds__(256) void sum_partial_kernel(const float* __restrict__ x, int64_t n,
                                                          float* __restrict__ partial) {
  __shared__ float red[4];
  float acc = 0.f;
  const int64_t n4 = n / 4;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const f32x4 a = *((const f32x4*)x + i);
    acc += (a[0] + a[1]) + (a[2] + a[3]);
  }
  if (blockIdx.x == 0)
    for (int64_t i = n4 * 4 + threadIdx.x; i < n; i += blockDim.x) acc += x[i];
  float t = block_sum(acc, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = t;
}

extern "C" int toa_sum_f32(const float* x, int64_t n, float* workspace, float* out, int accumulate,
                           hipStream_t stream) {
  if (n <= 0 || ((uintptr_t)x & 15)) return (int)hipErrorInvalidValue;
  const int64_t n4 = n / 4 > 0 ? n / 4 : 1;
  const int grid = (int)std::min<int64_t>((n4 + 255) / 256, 32768);
  hipLaunchKernelGGL(sum_partial_kernel, dim3(grid), dim3(256), 0, stream, x, n, workspace);
  hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(256), 0, stream, workspace, grid, out, accumulate);
  return (int)hipGetLastError();
}

// Sum of squares over many small ranges of one bf16 vector in one launch
// (the clipping norm's rest after the weight-gradient partials: the norm
// weights between the linear weights, ops/gemm.SumsqSession): workgroup b
// sums range b (offs[b], lens[b]) into partial[b], then one sum, added to
// out.  Deterministic: fixed ranges, fixed order.
__global__ __launch_bounds__(256) void sumsq_ranges_kernel(const bf16_t* __restrict__ x,
                                                           const int64_t* __restrict__ offs,
                                                           const int64_t* __restrict__ lens,
                                                           float* __restrict__ partial) {
  __shared__ float red[4];
  const int64_t o = offs[blockIdx.x], n = lens[blockIdx.x];
  float acc = 0.f;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    const float f = bf2f(x[o + i]);
    acc = fmaf(f, f, acc);
  }
  float t = block_sum(acc, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = t;
}

extern "C" int toa_sumsq_ranges(const bf16_t* x, const int64_t* offs, const int64_t* lens, int n, float* workspace,
                                float* out, int accumulate, hipStream_t stream) {
  if (n <= 0 || n > 32768) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(sumsq_ranges_kernel, dim3(n), dim3(256), 0, stream, x, offs, lens, workspace);
  hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(256), 0, stream, workspace, n, out, accumulate);
  return (int)hipGetLastError();
}

// workspace must hold >= TOA_SUMSQ_WS (32768) floats.  Grid: one 8-element
// chunk per thread up to 32768 blocks (the flat AdamW's measurement: a grid
// capped at 2048 blocks left each thread looping, 5-6 % slower per byte).
extern "C" int toa_sumsq(const void* x, int64_t n, int is_bf16, float* workspace, float* out,
                         int accumulate, hipStream_t stream) {
  const int64_t n8 = n / 8 > 0 ? n / 8 : 1;
  const int grid = (int)std::min<int64_t>((n8 + 255) / 256, 32768);
  if (is_bf16)
    hipLaunchKernelGGL(sumsq_partial_kernel<true>, dim3(grid), dim3(256), 0, stream, x, n, workspace);
  else
    hipLaunchKernelGGL(sumsq_partial_kernel<false>, dim3(grid), dim3(256), 0, stream, x, n, workspace);
  hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(256), 0, stream, workspace, grid, out, accumulate);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// AdamW on flat buffers.
//   g_eff = grad * grad_scale * clip,   clip = min(1, max_norm / (||grad*grad_scale|| + 1e-6))
//   m = b1 m + (1-b1) g ; v = b2 v + (1-b2) g^2
//   p = p - lr * ( m/bc1 / (sqrt(v/bc2) + eps) + wd * p )      (decoupled decay)
//   param_bf16 = bf16(p)
// grad may be bf16 or fp32.  n must be a multiple of 8 (flat buffers are
// padded to 64 elements by the Python side).
// ---------------------------------------------------------------------------
// Every stream is touched exactly once per step (28 B / parameter, far
// beyond the 256 MB Infinity Cache at Llama-3-8B), so NT = 1 issues the
// loads and stores non-temporal: nothing of the optimizer sweep is kept in
// L2 / MALL that the next step's GEMMs would have to evict.
template <typename T>
__device__ __forceinline__ T ld_s(const T* p, bool nt) {
  return nt ? __builtin_nontemporal_load(p) : *p;
}
template <typename T>
__device__ __forceinline__ void st_s(T* p, T v, bool nt) {
  if (nt)
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}

// The clipped gradient scale and (graph-replayable form) the bias
// corrections.
__device__ __forceinline__ float adam_prologue(float b1, float b2, float grad_scale, const float* norm_sq,
                                               float max_norm, const int* step_dev, float& inv_bc1,
                                               float& inv_sqrt_bc2) {
  if (step_dev != nullptr) {  // graph-replayable form: the step count lives on the device
    const float st = (float)step_dev[0];
    inv_bc1 = 1.f / (1.f - powf(b1, st));
    inv_sqrt_bc2 = 1.f / sqrtf(1.f - powf(b2, st));
  }
  float scale = grad_scale;
  if (norm_sq != nullptr && max_norm > 0.f) {
    float nrm = sqrtf(norm_sq[0]) * grad_scale;
    float c = max_norm / (nrm + 1e-6f);
    scale *= (c < 1.f ? c : 1.f);
  }
  return scale;
}

// One parameter's update.
__device__ __forceinline__ void adam_elem(float g, float& p, float& m, float& v, float scale, float b1, float b2,
                                          float omb1, float omb2, float lr, float lrwd, float eps, float inv_bc1,
                                          float inv_sqrt_bc2) {
  const float gj = g * scale;
  m = fmaf(b1, m, omb1 * gj);
  v = fmaf(b2, v, omb2 * gj * gj);
  const float denom = sqrtf(v) * inv_sqrt_bc2 + eps;
  p = p - lr * (m * inv_bc1) / denom - lrwd * p;
}

template <bool GRAD_BF16, bool NT>
__global__ __launch_bounds__(256) void adamw_flat_kernel(float* __restrict__ master, bf16_t* __restrict__ param,
                                                         void* __restrict__ grad, int zero_grad, float* __restrict__ m,
                                                         float* __restrict__ v, int64_t n8, float lr, float b1,
                                                         float b2, float eps, float wd, float inv_bc1,
                                                         float inv_sqrt_bc2, float grad_scale,
                                                         const float* __restrict__ norm_sq, float max_norm,
                                                         const int* __restrict__ step_dev) {
  const float scale = adam_prologue(b1, b2, grad_scale, norm_sq, max_norm, step_dev, inv_bc1, inv_sqrt_bc2);
  const float omb1 = 1.f - b1, omb2 = 1.f - b2, lrwd = lr * wd;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8;
       i += (int64_t)gridDim.x * blockDim.x) {
    float g[8], p[8], mm[8], vv[8];
    if (GRAD_BF16) {
      unpack8(ld_s((const u32x4*)grad + i, NT), g);
      if (zero_grad) st16((bf16_t*)grad + i * 8, u32x4{0, 0, 0, 0});
    } else {
      f32x4 a = ld_s((const f32x4*)grad + 2 * i, NT), b = ld_s((const f32x4*)grad + 2 * i + 1, NT);
      g[0] = a[0]; g[1] = a[1]; g[2] = a[2]; g[3] = a[3];
      g[4] = b[0]; g[5] = b[1]; g[6] = b[2]; g[7] = b[3];
      if (zero_grad) {
        *((f32x4*)grad + 2 * i) = f32x4{0.f, 0.f, 0.f, 0.f};
        *((f32x4*)grad + 2 * i + 1) = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
    f32x4* pm = (f32x4*)master + 2 * i;
    f32x4* mv = (f32x4*)m + 2 * i;
    f32x4* vvp = (f32x4*)v + 2 * i;
    f32x4 p0 = ld_s(pm, NT), p1 = ld_s(pm + 1, NT), m0 = ld_s(mv, NT), m1 = ld_s(mv + 1, NT),
          v0 = ld_s(vvp, NT), v1 = ld_s(vvp + 1, NT);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      p[j] = p0[j]; p[j + 4] = p1[j];
      mm[j] = m0[j]; mm[j + 4] = m1[j];
      vv[j] = v0[j]; vv[j + 4] = v1[j];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
      adam_elem(g[j], p[j], mm[j], vv[j], scale, b1, b2, omb1, omb2, lr, lrwd, eps, inv_bc1, inv_sqrt_bc2);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      p0[j] = p[j]; p1[j] = p[j + 4];
      m0[j] = mm[j]; m1[j] = mm[j + 4];
      v0[j] = vv[j]; v1[j] = vv[j + 4];
    }
    st_s(pm, p0, NT); st_s(pm + 1, p1, NT);
    st_s(mv, m0, NT); st_s(mv + 1, m1, NT);
    st_s(vvp, v0, NT); st_s(vvp + 1, v1, NT);
    if (param != nullptr) st_s((u32x4*)param + i, pack8(p), NT);
  }
}

// ---------------------------------------------------------------------------
// AdamW over one 2-D weight [R][C] of the flat buffers (R, C multiples of
// 128, bf16 gradient) that also writes the weight's transposed bf16 copy
// W^T [C][R] (row stride ldt) in the same pass -- the copy the data-gradient
// GEMMs read (ops/wt.py).  The separate refresh re-read the bf16 weight the
// update had just written (2 B / parameter); here the fresh bf16 values go
// through a 128 x 128 LDS tile (the XOR-swizzled image of transpose.hip's
// LDS kernel) and out as 256-byte runs of W^T.  Per element the arithmetic is
// adam_elem, as in adamw_flat_kernel: bit-identical master / m / v / weight.
// A workgroup walks 128 x 128 tiles; each pass of its 256 threads updates
// 16 rows x 128 columns (16 lanes per 256-byte row).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void adamw_wt_kernel(float* __restrict__ master, bf16_t* __restrict__ param,
                                                       bf16_t* __restrict__ grad, int zero_grad,
                                                       float* __restrict__ m, float* __restrict__ v,
                                                       bf16_t* __restrict__ wt, int64_t ldt, int R, int C, float lr,
                                                       float b1, float b2, float eps, float wd, float inv_bc1,
                                                       float inv_sqrt_bc2, float grad_scale,
                                                       const float* __restrict__ norm_sq, float max_norm) {
  __shared__ u32x4 tile[128 * 16];
  const float scale = adam_prologue(b1, b2, grad_scale, norm_sq, max_norm, nullptr, inv_bc1, inv_sqrt_bc2);
  const float omb1 = 1.f - b1, omb2 = 1.f - b2, lrwd = lr * wd;
  const int tid = threadIdx.x;
  const int lr_ = tid >> 4, lc = tid & 15;   // update: row lr_ + 16 p, chunk lc
  const int a = tid & 15, bq = tid >> 4;     // transposed store: rows 8a.., chunk bq
  const int tiles_c = C >> 7;
  const int64_t ntiles = (int64_t)(R >> 7) * tiles_c;
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int tr = (int)(t / tiles_c), tc = (int)(t - (int64_t)tr * tiles_c);
    const int64_t r0 = (int64_t)tr * 128, c0 = (int64_t)tc * 128;
    __syncthreads();   // the previous tile's transposed reads are done
#pragma unroll 1
    for (int pp = 0; pp < 8; pp += 2) {
      u32x4 gb[2];
      f32x4 pv[2][2], mv[2][2], vv[2][2];
      int64_t e8[2];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int r = lr_ + 16 * (pp + q);
        e8[q] = ((r0 + r) * C + c0) / 8 + lc;   // 8-element chunk index in the weight
        gb[q] = ld_s((const u32x4*)grad + e8[q], true);
        pv[q][0] = ld_s((const f32x4*)master + 2 * e8[q], true);
        pv[q][1] = ld_s((const f32x4*)master + 2 * e8[q] + 1, true);
        mv[q][0] = ld_s((const f32x4*)m + 2 * e8[q], true);
        mv[q][1] = ld_s((const f32x4*)m + 2 * e8[q] + 1, true);
        vv[q][0] = ld_s((const f32x4*)v + 2 * e8[q], true);
        vv[q][1] = ld_s((const f32x4*)v + 2 * e8[q] + 1, true);
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int r = lr_ + 16 * (pp + q);
        float g[8], p[8];
        unpack8(gb[q], g);
        if (zero_grad) st16(grad + e8[q] * 8, u32x4{0, 0, 0, 0});
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float pp_ = pv[q][h][j], mm = mv[q][h][j], vq = vv[q][h][j];
            adam_elem(g[4 * h + j], pp_, mm, vq, scale, b1, b2, omb1, omb2, lr, lrwd, eps, inv_bc1, inv_sqrt_bc2);
            pv[q][h][j] = pp_;
            mv[q][h][j] = mm;
            vv[q][h][j] = vq;
            p[4 * h + j] = pp_;
          }
        st_s((f32x4*)master + 2 * e8[q], pv[q][0], true);
        st_s((f32x4*)master + 2 * e8[q] + 1, pv[q][1], true);
        st_s((f32x4*)m + 2 * e8[q], mv[q][0], true);
        st_s((f32x4*)m + 2 * e8[q] + 1, mv[q][1], true);
        st_s((f32x4*)v + 2 * e8[q], vv[q][0], true);
        st_s((f32x4*)v + 2 * e8[q] + 1, vv[q][1], true);
        const u32x4 pk = pack8(p);
        st_s((u32x4*)param + e8[q], pk, true);
        tile[r * 16 + (lc ^ ((r >> 3) & 15))] = pk;
      }
    }
    __syncthreads();
    u32x4 in[8], out[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) in[i] = tile[(8 * a + i) * 16 + (bq ^ a)];
    tr8x8(in, out);
    bf16_t* d = wt + (c0 + 8 * bq) * ldt + r0 + 8 * a;
#pragma unroll
    for (int j = 0; j < 8; ++j) __builtin_nontemporal_store(out[j], (u32x4*)(d + j * ldt));
  }
}

extern "C" int toa_adamw_wt(float* master, bf16_t* param, bf16_t* grad, int zero_grad, float* m, float* v,
                            bf16_t* wt, int64_t ldt, int R, int C, float lr, float beta1, float beta2, float eps,
                            float weight_decay, int step, float grad_scale, const float* norm_sq, float max_norm,
                            hipStream_t stream) {
  if (R <= 0 || C <= 0 || R % 128 || C % 128 || ldt < R || ldt % 8 || ((uintptr_t)master & 15) ||
      ((uintptr_t)m & 15) || ((uintptr_t)v & 15) || ((uintptr_t)grad & 15) || ((uintptr_t)param & 15) ||
      ((uintptr_t)wt & 15) || step < 1)
    return (int)hipErrorInvalidValue;
  const float inv_bc1 = 1.f / (1.f - powf(beta1, (float)step));
  const float inv_sqrt_bc2 = 1.f / sqrtf(1.f - powf(beta2, (float)step));
  const int64_t tiles = (int64_t)(R / 128) * (C / 128);
  const int grid = (int)(tiles < 16384 ? tiles : 16384);
  hipLaunchKernelGGL(adamw_wt_kernel, dim3(grid), dim3(256), 0, stream, master, param, grad, zero_grad, m, v, wt, ldt,
                     R, C, lr, beta1, beta2, eps, weight_decay, inv_bc1, inv_sqrt_bc2, grad_scale, norm_sq, max_norm);
  return (int)hipGetLastError();
}

// Variant switch for in-process A/B (scripts/stream_ab.py,
// scripts/adamw_grid_bench.py): bit 0 = the non-temporal AdamW, bit 1 = the
// row-structured non-temporal SwiGLU, bits 8.. = AdamW grid cap / 1024 (0:
// toa_stream_grid's 2048).  Defaults from A/Bs on MI355X: AdamW NT
// (profiles/r2_stream_ab/), SwiGLU rows+NT fwd 0.404 -> 0.373 ms and bwd
// 0.723 -> 0.653 ms at T = 24576, F = 14336; and the AdamW grid at one
// 8-element chunk per thread (cap 255K blocks, above any Llama-3-8B launch):
// 1.247 -> 1.174 ms for one layer's 218M parameters against the round-2 16K
// cap (profiles/r5_adamw/).  All arms bit-identical.
static int g_stream_variant = 1 | 2 | (255 << 8);
int toa_stream_variant() { return g_stream_variant; }
extern "C" int toa_set_stream_variant(int v) {
  const int old = g_stream_variant;
  g_stream_variant = v;
  return old;
}

// grad_flags: bit 0 = grad is bf16 (else fp32); bit 1 = zero the gradient
// after reading it (the next step's zero_grad pass, fused).
static int adamw_launch(float* master, bf16_t* param, void* grad, int grad_flags, float* m, float* v, int64_t n,
                        float lr, float beta1, float beta2, float eps, float weight_decay, int step, float grad_scale,
                        const float* norm_sq, float max_norm, const int* step_dev, hipStream_t stream) {
  if (n % 8 != 0) return (int)hipErrorInvalidValue;
  const int64_t n8 = n / 8;
  const float bc1 = 1.f - powf(beta1, (float)step);
  const float bc2 = 1.f - powf(beta2, (float)step);
  const float inv_bc1 = 1.f / bc1, inv_sqrt_bc2 = 1.f / sqrtf(bc2);
  int grid = toa_stream_grid(n8, 256);
  const int cap = (g_stream_variant >> 8) * 1024;
  if (cap > 0 && n8 >= (int64_t)(1 << 20)) grid = (int)std::min<int64_t>(std::max<int64_t>((n8 + 255) / 256, 1), cap);
  const int zero_grad = (grad_flags >> 1) & 1;
  // non-temporal only for sweeps far beyond the caches: a small model's whole
  // optimizer state (MNIST: 2.2 MB) stays L2-resident between graph replays; 8M+ parameters per launch
  const bool nt = (g_stream_variant & 1) && n8 >= (int64_t)(1 << 20);
  auto k = (grad_flags & 1) ? (nt ? adamw_flat_kernel<true, true> : adamw_flat_kernel<true, false>)
                            : (nt ? adamw_flat_kernel<false, true> : adamw_flat_kernel<false, false>);
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, stream, master, param, grad, zero_grad, m, v, n8, lr, beta1, beta2,
                     eps, weight_decay, inv_bc1, inv_sqrt_bc2, grad_scale, norm_sq, max_norm, step_dev);
  return (int)hipGetLastError();
}

extern "C" int toa_adamw_flat(float* master, bf16_t* param, void* grad, int grad_flags, float* m,
                              float* v, int64_t n, float lr, float beta1, float beta2, float eps,
                              float weight_decay, int step, float grad_scale, const float* norm_sq,
                              float max_norm, hipStream_t stream) {
  return adamw_launch(master, param, grad, grad_flags, m, v, n, lr, beta1, beta2, eps, weight_decay, step, grad_scale,
                      norm_sq, max_norm, nullptr, stream);
}

// Same update with the step count read from device memory (step_dev[0], the
// step being taken): a captured HIP graph replays it with fresh bias
// corrections.  toa_step_inc advances the counter inside the same graph.
extern "C" int toa_adamw_flat_dstep(float* master, bf16_t* param, void* grad, int grad_flags, float* m, float* v,
                                    int64_t n, float lr, float beta1, float beta2, float eps, float weight_decay,
                                    const int* step_dev, float grad_scale, const float* norm_sq, float max_norm,
                                    hipStream_t stream) {
  if (step_dev == nullptr) return (int)hipErrorInvalidValue;
  return adamw_launch(master, param, grad, grad_flags, m, v, n, lr, beta1, beta2, eps, weight_decay, 1, grad_scale,
                      norm_sq, max_norm, step_dev, stream);
}

__global__ void step_inc_kernel(int* step) { step[0] += 1; }

extern "C" int toa_step_inc(int* step, hipStream_t stream) {
  hipLaunchKernelGGL(step_inc_kernel, dim3(1), dim3(1), 0, stream, step);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Plain SGD with momentum over flat fp32 params (the estimator example's
// optimizer) -- fp32 params, fp32 grads.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void sgd_flat_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                       float* __restrict__ buf, int64_t n, float lr,
                                                       float momentum, float wd) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float gi = g[i] + wd * p[i];
    if (buf != nullptr) {
      float b = momentum * buf[i] + gi;
      buf[i] = b;
      gi = b;
    }
    p[i] -= lr * gi;
  }
}

extern "C" int toa_sgd_flat(float* p, const float* g, float* momentum_buf, int64_t n, float lr, float momentum,
                            float weight_decay, hipStream_t stream) {
  int grid = toa_stream_grid(n, 256);
  hipLaunchKernelGGL(sgd_flat_kernel, dim3(grid), dim3(256), 0, stream, p, g, momentum_buf, n, lr, momentum,
                     weight_decay);
  return (int)hipGetLastError();
}

// bf16 <-> fp32 flat casts (used to (re)materialise the compute copy after a
// checkpoint load and to zero/scale gradient buckets).
__global__ __launch_bounds__(256) void cast_f32_bf16_kernel(const float* __restrict__ x, bf16_t* __restrict__ y,
                                                            int64_t n8) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    f32x4 a = *((const f32x4*)x + 2 * i), b = *((const f32x4*)x + 2 * i + 1);
    float f[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
    st16(y + i * 8, pack8(f));
  }
}

extern "C" int toa_cast_f32_to_bf16(const float* x, bf16_t* y, int64_t n, hipStream_t stream) {
  if (n % 8 != 0) return (int)hipErrorInvalidValue;
  int grid = toa_stream_grid(n / 8, 256);
  hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3(grid), dim3(256), 0, stream, x, y, n / 8);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// A stream whose kernels may only use some of the CUs
// (hipExtStreamCreateWithCUMask): the overlapped AdamW (FlatAdamW overlap,
// TOA_OPT_CUS) runs its memory-bound update on a few CUs beside the
// compute-bound GEMMs instead of taking every CU a finished GEMM workgroup
// frees.  mode 0: CUs 0 .. n-1 of the mask; mode 1: n CUs spread evenly over
// the mask (which bit is which XCD is the driver's mapping: the probe
// scripts/cu_mask_probe.py measures both).
// ---------------------------------------------------------------------------
extern "C" int toa_stream_create_cu_mask(int mode, int n, void** out) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return (int)e;
  int total = 0;
  e = hipDeviceGetAttribute(&total, hipDeviceAttributeMultiprocessorCount, dev);
  if (e != hipSuccess) return (int)e;
  if (out == nullptr || n <= 0 || n > total || total > 1024 || (mode != 0 && mode != 1))
    return (int)hipErrorInvalidValue;
  uint32_t mask[32] = {};
  const int words = (total + 31) / 32;
  for (int i = 0; i < n; ++i) {
    const int cu = mode == 0 ? i : (int)((int64_t)i * total / n);
    mask[cu / 32] |= 1u << (cu % 32);
  }
  hipStream_t s = nullptr;
  e = hipExtStreamCreateWithCUMask(&s, (uint32_t)words, mask);
  if (e != hipSuccess) return (int)e;
  *out = (void*)s;
  return 0;
}

extern "C" int toa_stream_destroy(void* s) { return (int)hipStreamDestroy((hipStream_t)s); }
