// Training-mode BatchNorm for channels-last (NHWC) activations on gfx950,
// with the ReLU and the residual add of a ResNet bottleneck fused in:
//
//     y = act(x * scale[c] + shift[c] (+ res)),  scale = gamma / sqrt(var + eps),
//                                                 shift = beta - mean * scale
//
// x / res / y / dy are [R][C] row-major (R = N*H*W, C contiguous), bf16 or
// fp32; gamma / beta / running stats bf16 or fp32; statistics and all
// reductions in fp32.  C % 8 == 0, C <= 2048 (a thread owns 8 consecutive
// channels = one 16-B bf16 vector).
//
// Forward (3 launches): per-workgroup partial sums of (x - pivot) and
// (x - pivot)^2 (pivot = row 0 of x, the shifted-data variance form: no
// E[x^2] - E[x]^2 cancellation for large means), a finalize kernel that
// also updates the running statistics, and the elementwise apply.
// Backward (3 launches): partial sums of dy' and dy' * xhat where dy' is dy
// masked by the saved output's sign (ReLU), finalize to dgamma / dbeta, then
//     dx = scale * (dy' - dbeta / R - xhat * dgamma / R)   and  dres = dy'.
// Every reduction sums partials in a fixed order: deterministic, no atomics.
//
// The library path (PyTorch's batch_norm_collect_statistics /
// batch_norm_backward_reduce for channels-last bf16) ran these reductions at
// a fraction of HBM bandwidth and kept ReLU / add as separate passes
// (profiles/r2_resnet).
#include "toa_common.h"

#define BN_THREADS 256

template <typename T>
__device__ __forceinline__ void ld8(const T* p, float* f);
template <>
__device__ __forceinline__ void ld8<bf16_t>(const bf16_t* p, float* f) { unpack8(ld16(p), f); }
template <>
__device__ __forceinline__ void ld8<float>(const float* p, float* f) {
  const f32x4 a = *(const f32x4*)p, b = *((const f32x4*)p + 1);
  f[0] = a[0]; f[1] = a[1]; f[2] = a[2]; f[3] = a[3];
  f[4] = b[0]; f[5] = b[1]; f[6] = b[2]; f[7] = b[3];
}
template <typename T>
__device__ __forceinline__ void st8(T* p, const float* f);
template <>
__device__ __forceinline__ void st8<bf16_t>(bf16_t* p, const float* f) { st16(p, pack8(f)); }
template <>
__device__ __forceinline__ void st8<float>(float* p, const float* f) {
  *(f32x4*)p = f32x4{f[0], f[1], f[2], f[3]};
  *((f32x4*)p + 1) = f32x4{f[4], f[5], f[6], f[7]};
}
template <typename P>
__device__ __forceinline__ float ldp(const P* p, int i);
template <>
__device__ __forceinline__ float ldp<float>(const float* p, int i) { return p[i]; }
template <>
__device__ __forceinline__ float ldp<bf16_t>(const bf16_t* p, int i) { return bf2f(p[i]); }
template <typename P>
__device__ __forceinline__ void stp(P* p, int i, float v);
template <>
__device__ __forceinline__ void stp<float>(float* p, int i, float v) { p[i] = v; }
template <>
__device__ __forceinline__ void stp<bf16_t>(bf16_t* p, int i, float v) { p[i] = f2bf(v); }
// dgamma / dbeta store: gdt 0 = bf16, 1 = fp32; acc: add into what is there
// (the flat fp32 gradient buffer, main_grad) instead of overwriting
__device__ __forceinline__ void st_grad(void* p, int gdt, int acc, int i, float v) {
  if (gdt == 1) {
    float* q = (float*)p;
    q[i] = acc ? q[i] + v : v;
  } else {
    bf16_t* q = (bf16_t*)p;
    q[i] = f2bf(acc ? bf2f(q[i]) + v : v);
  }
}

// Block geometry: CG = C/8 channel groups across the threads of a row,
// RPI = 256 / CG rows per block iteration (threads >= RPI*CG idle).
struct BnGeo {
  int cg, rpi;
  __device__ __forceinline__ BnGeo(int C) : cg(C >> 3), rpi(BN_THREADS / (C >> 3)) {}
};

// Sum the per-thread partials of the RPI row-threads of each channel through
// LDS and write one [2][C] fp32 partial per workgroup.
__device__ __forceinline__ void bn_block_partial(const float* a, const float* b, int C, float* __restrict__ out,
                                                 float* lds) {
  const BnGeo g(C);
  const int t = threadIdx.x, ro = t / g.cg, cgi = t - ro * g.cg;
  if (ro < g.rpi) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      lds[ro * C + cgi * 8 + j] = a[j];
      lds[BN_THREADS * 8 + ro * C + cgi * 8 + j] = b[j];
    }
  }
  __syncthreads();
  for (int c = t; c < C; c += BN_THREADS) {
    float sa = 0.f, sb = 0.f;
    for (int r = 0; r < g.rpi; ++r) {
      sa += lds[r * C + c];
      sb += lds[BN_THREADS * 8 + r * C + c];
    }
    out[c] = sa;
    out[C + c] = sb;
  }
}

template <typename T>
__global__ __launch_bounds__(BN_THREADS) void bn_stats_partial_kernel(const T* __restrict__ x, int64_t R, int C,
                                                                       float* __restrict__ ws) {
  __shared__ float lds[2 * BN_THREADS * 8];
  const BnGeo g(C);
  const int t = threadIdx.x, ro = t / g.cg, cgi = t - ro * g.cg;
  float s[8] = {}, q[8] = {}, piv[8];
  ld8(x + cgi * 8, piv);  // pivot: row 0
  if (ro < g.rpi) {
    for (int64_t r = (int64_t)blockIdx.x * g.rpi + ro; r < R; r += (int64_t)gridDim.x * g.rpi) {
      float v[8];
      ld8(x + r * C + cgi * 8, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[j] - piv[j];
        s[j] += d;
        q[j] = fmaf(d, d, q[j]);
      }
    }
  }
  bn_block_partial(s, q, C, ws + (int64_t)blockIdx.x * 2 * C, lds);
}

// Sum the nb [2][C] workgroup partials for the 8 channels [c8, c8+8): 256
// threads = 8 channels x 32 partial strides (independent loads in flight),
// then a 32-way LDS reduction.  Returns the two sums in thread (ch, 0).
__device__ __forceinline__ bool bn_sum_partials(const float* __restrict__ ws, int nb, int C, int c8, float* out_a,
                                                float* out_b) {
  __shared__ float red[2][32][8];
  const int t = threadIdx.x, ch = t & 7, pr = t >> 3;
  float a = 0.f, b = 0.f;
  for (int i = pr; i < nb; i += 32) {
    a += ws[(int64_t)i * 2 * C + c8 + ch];
    b += ws[(int64_t)i * 2 * C + C + c8 + ch];
  }
  red[0][pr][ch] = a;
  red[1][pr][ch] = b;
  __syncthreads();
  if (pr != 0) return false;
  a = 0.f;
  b = 0.f;
  for (int i = 0; i < 32; ++i) {  // fixed order: deterministic
    a += red[0][i][ch];
    b += red[1][i][ch];
  }
  *out_a = a;
  *out_b = b;
  return true;
}

// stats[0..C) = mean, stats[C..2C) = invstd, stats[2C..4C) = scale, shift
// (saved for backward);
// sc[0..C) = scale, sc[C..2C) = shift; running stats updated with momentum
// (unbiased variance), as torch.nn.BatchNorm2d does.
template <typename T, typename P>
__global__ __launch_bounds__(BN_THREADS) void bn_finalize_kernel(const T* __restrict__ x, const float* __restrict__ ws,
                                                                  int nb, int64_t R, int C, const P* __restrict__ gamma,
                                                                  const P* __restrict__ beta, P* __restrict__ rmean,
                                                                  P* __restrict__ rvar, float momentum, float eps,
                                                                  float* __restrict__ stats, float* __restrict__ sc) {
  // one workgroup per 8 channels
  float s, q;
  if (!bn_sum_partials(ws, nb, C, blockIdx.x * 8, &s, &q)) return;
  const int c = blockIdx.x * 8 + (threadIdx.x & 7);
  float piv[8];
  ld8(x + (c & ~7), piv);
  const float inv_r = 1.f / (float)R;
  const float dm = s * inv_r;
  const float var = fmaxf(q * inv_r - dm * dm, 0.f);
  const float mean = piv[c & 7] + dm;
  const float invstd = rsqrtf(var + eps);
  stats[c] = mean;
  stats[C + c] = invstd;
  const float gm = gamma ? ldp(gamma, c) : 1.f, bt = beta ? ldp(beta, c) : 0.f;
  sc[c] = gm * invstd;
  sc[C + c] = bt - mean * gm * invstd;
  stats[2 * C + c] = sc[c];  // kept for the backward's ReLU mask (mask mode 2)
  stats[3 * C + c] = sc[C + c];
  if (rmean) {
    const float unb = R > 1 ? var * (float)R / (float)(R - 1) : var;
    stp(rmean, c, (1.f - momentum) * ldp(rmean, c) + momentum * mean);
    stp(rvar, c, (1.f - momentum) * ldp(rvar, c) + momentum * unb);
  }
}

// eval mode: scale / shift from the running statistics
template <typename P>
__global__ __launch_bounds__(BN_THREADS) void bn_eval_coeffs_kernel(int C, const P* __restrict__ gamma,
                                                                     const P* __restrict__ beta,
                                                                     const P* __restrict__ rmean,
                                                                     const P* __restrict__ rvar, float eps,
                                                                     float* __restrict__ sc) {
  const int c = blockIdx.x * BN_THREADS + threadIdx.x;
  if (c >= C) return;
  const float gm = gamma ? ldp(gamma, c) : 1.f, bt = beta ? ldp(beta, c) : 0.f;
  const float s = gm * rsqrtf(ldp(rvar, c) + eps);
  sc[c] = s;
  sc[C + c] = bt - ldp(rmean, c) * s;
}

template <typename T>
__global__ __launch_bounds__(BN_THREADS) void bn_apply_kernel(const T* __restrict__ x, const T* __restrict__ res,
                                                              T* __restrict__ y, const float* __restrict__ sc,
                                                              int64_t n8, int C, int relu) {
  for (int64_t i = (int64_t)blockIdx.x * BN_THREADS + threadIdx.x; i < n8; i += (int64_t)gridDim.x * BN_THREADS) {
    const int c0 = (int)((i * 8) % C);
    float v[8], r[8];
    ld8(x + i * 8, v);
    if (res) ld8(res + i * 8, r);
    const f32x4 s0 = *(const f32x4*)(sc + c0), s1 = *(const f32x4*)(sc + c0 + 4);
    const f32x4 h0 = *(const f32x4*)(sc + C + c0), h1 = *(const f32x4*)(sc + C + c0 + 4);
    const float sv[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
    const float hv[8] = {h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float o = fmaf(v[j], sv[j], hv[j]);
      if (res) o += r[j];
      v[j] = relu ? fmaxf(o, 0.f) : o;
    }
    st8(y + i * 8, v);
  }
}

// ---------------------------------------------------------------------------
// backward
// ---------------------------------------------------------------------------
// ReLU mask of the backward: mode 0 none, 1 from the saved output y (a
// residual was added before the ReLU), 2 recomputed from x with the forward's
// own fmaf(x, scale, shift) -- bit-identical sign, and one tensor less to read.
template <typename T>
__device__ __forceinline__ void bn_mask(int mode, const T* __restrict__ y, int64_t off, const float* v,
                                        const float* sc, const float* sh, float* d) {
  if (mode == 1) {
    float o[8];
    ld8(y + off, o);
#pragma unroll
    for (int j = 0; j < 8; ++j) d[j] = o[j] > 0.f ? d[j] : 0.f;
  } else if (mode == 2) {
#pragma unroll
    for (int j = 0; j < 8; ++j) d[j] = fmaf(v[j], sc[j], sh[j]) > 0.f ? d[j] : 0.f;
  }
}

template <typename T>
__global__ __launch_bounds__(BN_THREADS) void bn_bwd_partial_kernel(const T* __restrict__ dy,
                                                                    const T* __restrict__ x,
                                                                    const T* __restrict__ y, int mask,
                                                                    const float* __restrict__ stats, int64_t R, int C,
                                                                    float* __restrict__ ws) {
  __shared__ float lds[2 * BN_THREADS * 8];
  const BnGeo g(C);
  const int t = threadIdx.x, ro = t / g.cg, cgi = t - ro * g.cg;
  float sd[8] = {}, sx[8] = {}, mu[8], is[8], sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    mu[j] = stats[cgi * 8 + j];
    is[j] = stats[C + cgi * 8 + j];
    sc[j] = stats[2 * C + cgi * 8 + j];
    sh[j] = stats[3 * C + cgi * 8 + j];
  }
  if (ro < g.rpi) {
    for (int64_t r = (int64_t)blockIdx.x * g.rpi + ro; r < R; r += (int64_t)gridDim.x * g.rpi) {
      float d[8], v[8];
      ld8(dy + r * C + cgi * 8, d);
      ld8(x + r * C + cgi * 8, v);
      bn_mask(mask, y, r * C + cgi * 8, v, sc, sh, d);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sd[j] += d[j];
        sx[j] = fmaf(d[j], (v[j] - mu[j]) * is[j], sx[j]);
      }
    }
  }
  bn_block_partial(sd, sx, C, ws + (int64_t)blockIdx.x * 2 * C, lds);
}

// g[0..C) = dbeta (sum dy'), g[C..2C) = dgamma (sum dy' xhat), fp32; the
// parameter gradients are also written in the parameters' dtype.  k[0..3C)
// are the per-channel coefficients of the input gradient,
//     dx = k1 dy' + k2 x + k3,   k1 = gamma invstd,  k2 = -k1 invstd dgamma / R,
//                                k3 = k1 (mean invstd dgamma - dbeta) / R
template <typename P>
__global__ __launch_bounds__(BN_THREADS) void bn_bwd_finalize_kernel(const float* __restrict__ ws, int nb, int64_t R,
                                                                      int C, const float* __restrict__ stats,
                                                                      const P* __restrict__ gamma,
                                                                      float* __restrict__ g, float* __restrict__ k,
                                                                      void* __restrict__ dgamma,
                                                                      void* __restrict__ dbeta, int gdt, int acc) {
  float a, b;  // one workgroup per 8 channels
  if (!bn_sum_partials(ws, nb, C, blockIdx.x * 8, &a, &b)) return;
  const int c = blockIdx.x * 8 + (threadIdx.x & 7);
  g[c] = a;
  g[C + c] = b;
  if (dbeta) st_grad(dbeta, gdt, acc, c, a);
  if (dgamma) st_grad(dgamma, gdt, acc, c, b);
  const float inv_r = 1.f / (float)R, mean = stats[c], is = stats[C + c];
  const float k1 = (gamma ? ldp(gamma, c) : 1.f) * is;
  k[c] = k1;
  k[C + c] = -k1 * is * b * inv_r;
  k[2 * C + c] = k1 * (mean * is * b - a) * inv_r;
}

__device__ __forceinline__ void ld8f(const float* p, float* f) { ld8<float>(p, f); }

template <typename T>
__global__ __launch_bounds__(BN_THREADS) void bn_bwd_apply_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                                  const T* __restrict__ y, int mask,
                                                                  const float* __restrict__ stats,
                                                                  const float* __restrict__ k, int64_t n8, int C,
                                                                  T* __restrict__ dx, T* __restrict__ dres) {
  for (int64_t i = (int64_t)blockIdx.x * BN_THREADS + threadIdx.x; i < n8; i += (int64_t)gridDim.x * BN_THREADS) {
    const int c0 = (int)((i * 8) % C);
    float d[8], v[8], k1[8], k2[8], k3[8];
    ld8(dy + i * 8, d);
    ld8(x + i * 8, v);
    if (mask == 2) {
      float sc[8], sh[8];
      ld8f(stats + 2 * C + c0, sc);
      ld8f(stats + 3 * C + c0, sh);
      bn_mask(2, y, i * 8, v, sc, sh, d);
    } else {
      bn_mask(mask, y, i * 8, v, nullptr, nullptr, d);
    }
    if (dres) st8(dres + i * 8, d);
    ld8f(k + c0, k1);
    ld8f(k + C + c0, k2);
    ld8f(k + 2 * C + c0, k3);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = fmaf(k1[j], d[j], fmaf(k2[j], v[j], k3[j]));
    st8(dx + i * 8, v);
  }
}

// ---------------------------------------------------------------------------
// launchers.  dtype: 0 = bf16, 1 = fp32 (activations); pdtype: same codes for
// gamma / beta / running stats.  ws: fp32 workspace of toa_bn_ws_floats().
// ---------------------------------------------------------------------------
static int bn_blocks(int64_t R, int C) {
  const int rpi = BN_THREADS / (C / 8);
  int64_t nb = (R + (int64_t)rpi * 16 - 1) / ((int64_t)rpi * 16);  // >= 16 rows per thread
  return (int)(nb < 1 ? 1 : (nb > 1024 ? 1024 : nb));
}
static bool bn_shape_ok(int64_t R, int C) { return R > 0 && C >= 8 && C % 8 == 0 && C <= 8 * BN_THREADS; }
static int bn_grid(int64_t n8) {
  int64_t b = (n8 + BN_THREADS - 1) / BN_THREADS;
  return (int)(b > 8192 ? 8192 : (b < 1 ? 1 : b));
}

extern "C" int64_t toa_bn_ws_floats(int64_t R, int C) { return (int64_t)bn_blocks(R, C) * 2 * C + 6 * C; }

#define BN_DISPATCH(dtype, pdtype, CALL)           \
  do {                                             \
    if ((dtype) == 0 && (pdtype) == 0) {           \
      using T = bf16_t; using P = bf16_t; CALL;    \
    } else if ((dtype) == 0 && (pdtype) == 1) {    \
      using T = bf16_t; using P = float; CALL;     \
    } else if ((dtype) == 1 && (pdtype) == 1) {    \
      using T = float; using P = float; CALL;      \
    } else {                                       \
      using T = float; using P = bf16_t; CALL;     \
    }                                              \
  } while (0)

// training forward: writes y, stats (mean, invstd: 2C fp32), updates running stats (may be null)
extern "C" int toa_bn_fwd_train(int dtype, int pdtype, const void* x, const void* res, void* y, int64_t R, int C,
                                const void* gamma, const void* beta, void* rmean, void* rvar, float momentum,
                                float eps, int relu, float* stats, float* ws, hipStream_t st) {
  if (!bn_shape_ok(R, C)) return (int)hipErrorInvalidValue;
  const int nb = bn_blocks(R, C);
  float* sc = ws + (int64_t)nb * 2 * C;
  BN_DISPATCH(dtype, pdtype, {
    hipLaunchKernelGGL(bn_stats_partial_kernel<T>, dim3(nb), dim3(BN_THREADS), 0, st, (const T*)x, R, C, ws);
    hipLaunchKernelGGL((bn_finalize_kernel<T, P>), dim3(C / 8), dim3(BN_THREADS), 0, st,
                       (const T*)x, ws, nb, R, C, (const P*)gamma, (const P*)beta, (P*)rmean, (P*)rvar, momentum,
                       eps, stats, sc);
    hipLaunchKernelGGL(bn_apply_kernel<T>, dim3(bn_grid(R * C / 8)), dim3(BN_THREADS), 0, st, (const T*)x,
                       (const T*)res, (T*)y, sc, R * C / 8, C, relu);
  });
  return (int)hipGetLastError();
}

extern "C" int toa_bn_fwd_eval(int dtype, int pdtype, const void* x, const void* res, void* y, int64_t R, int C,
                               const void* gamma, const void* beta, const void* rmean, const void* rvar, float eps,
                               int relu, float* ws, hipStream_t st) {
  if (!bn_shape_ok(R, C)) return (int)hipErrorInvalidValue;
  BN_DISPATCH(dtype, pdtype, {
    hipLaunchKernelGGL(bn_eval_coeffs_kernel<P>, dim3((C + BN_THREADS - 1) / BN_THREADS), dim3(BN_THREADS), 0, st, C,
                       (const P*)gamma, (const P*)beta, (const P*)rmean, (const P*)rvar, eps, ws);
    hipLaunchKernelGGL(bn_apply_kernel<T>, dim3(bn_grid(R * C / 8)), dim3(BN_THREADS), 0, st, (const T*)x,
                       (const T*)res, (T*)y, ws, R * C / 8, C, relu);
  });
  return (int)hipGetLastError();
}

// backward: y = the forward output when relu was fused (its sign is the
// mask), else null; dres (may be null) receives dy' for a fused residual
// mask: 0 no ReLU, 1 ReLU mask from y (the saved output), 2 from x and the
// saved scale / shift (y unused)
// dgamma / dbeta: gdtype 0 = bf16, 1 = fp32; accumulate = add into them
extern "C" int toa_bn_bwd(int dtype, int pdtype, const void* dy, const void* x, const void* y, int mask,
                          const float* stats,
                          const void* gamma, int64_t R, int C, void* dx, void* dres, void* dgamma, void* dbeta,
                          int gdtype, int accumulate, float* ws, hipStream_t st) {
  if (!bn_shape_ok(R, C) || mask < 0 || mask > 2 || (mask == 1 && !y) || gdtype < 0 || gdtype > 1)
    return (int)hipErrorInvalidValue;
  const int nb = bn_blocks(R, C);
  float* g = ws + (int64_t)nb * 2 * C;
  float* k = g + 2 * C;
  BN_DISPATCH(dtype, pdtype, {
    hipLaunchKernelGGL(bn_bwd_partial_kernel<T>, dim3(nb), dim3(BN_THREADS), 0, st, (const T*)dy, (const T*)x,
                       (const T*)y, mask, stats, R, C, ws);
    hipLaunchKernelGGL(bn_bwd_finalize_kernel<P>, dim3(C / 8), dim3(BN_THREADS), 0, st,
                       ws, nb, R, C, stats, (const P*)gamma, g, k, dgamma, dbeta, gdtype, accumulate);
    hipLaunchKernelGGL(bn_bwd_apply_kernel<T>, dim3(bn_grid(R * C / 8)), dim3(BN_THREADS), 0, st, (const T*)dy,
                       (const T*)x, (const T*)y, mask, stats, k, R * C / 8, C, (T*)dx, (T*)dres);
  });
  return (int)hipGetLastError();
}
