// RMSNorm / LayerNorm forward + backward for gfx950.
//
// Layout: one 64-lane wave owns one row; a 256-thread workgroup owns 4 rows.
// Each lane holds CH chunks of 8 elements (16 B bf16 / 32 B fp32 loads), so a
// 4096-wide row is 8 vector loads per lane with the whole row in registers:
// one HBM read + one HBM write per element in the forward (CDNA guide G13,
// Appendix B "Reduction").  The forward optionally fuses the residual add
// (h = x + r, y = norm(h)) so the transformer residual stream is touched once.
// The backward streams rows grid-strided, keeps the weight-gradient partial
// of its columns in registers across rows, reduces the 4 waves through LDS
// and writes one fp32 partial row per workgroup; a second tiny kernel sums the
// partials (deterministic, no float atomics -- guide G12).
//
// Reference parity: SURVEY K19 (LayerNorm/RMSNorm north-star additions).
#include "toa_common.h"

template <typename T>
struct Vec8;
template <>
struct Vec8<bf16_t> {
  static __device__ __forceinline__ void load(const bf16_t* p, float* f) { unpack8(ld16(p), f); }
  static __device__ __forceinline__ void store(bf16_t* p, const float* f) { st16(p, pack8(f)); }
};
template <>
struct Vec8<float> {
  static __device__ __forceinline__ void load(const float* p, float* f) {
    f32x4 a = *(const f32x4*)p, b = *((const f32x4*)p + 1);
    f[0] = a[0]; f[1] = a[1]; f[2] = a[2]; f[3] = a[3];
    f[4] = b[0]; f[5] = b[1]; f[6] = b[2]; f[7] = b[3];
  }
  static __device__ __forceinline__ void store(float* p, const float* f) {
    f32x4 a = {f[0], f[1], f[2], f[3]}, b = {f[4], f[5], f[6], f[7]};
    *(f32x4*)p = a;
    *((f32x4*)p + 1) = b;
  }
};

// ---------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------
template <typename T, int CH, bool RMS>
__global__ __launch_bounds__(256) void norm_fwd_kernel(const T* __restrict__ x, const T* __restrict__ res,
                                                       T* __restrict__ h_out, const T* __restrict__ w,
                                                       const T* __restrict__ b, T* __restrict__ y,
                                                       float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                       int rows, int cols, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nch = cols >> 3;
  const T* xr = x + (int64_t)row * cols;
  float v[CH][8];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
      Vec8<T>::load(xr + ch * 8, v[c]);
      if (res != nullptr) {
        float r[8];
        Vec8<T>::load(res + (int64_t)row * cols + ch * 8, r);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] += r[j];
        Vec8<T>::store(h_out + (int64_t)row * cols + ch * 8, v[c]);
        // re-read the rounded value so the statistics match what backward sees
        Vec8<T>::load(h_out + (int64_t)row * cols + ch * 8, v[c]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) s += RMS ? v[c][j] * v[c][j] : v[c][j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[c][j] = 0.f;
    }
  }
  float mean = 0.f, rstd;
  if (RMS) {
    s = wave_sum(s);
    rstd = rsqrtf(s / cols + eps);
  } else {
    mean = wave_sum(s) / cols;
    float q = 0.f;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int ch = lane + c * 64;
      if (ch < nch) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float d = v[c][j] - mean;
          q += d * d;
        }
      }
    }
    q = wave_sum(q);
    rstd = rsqrtf(q / cols + eps);
  }
  T* yr = y + (int64_t)row * cols;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
      float wv[8], o[8];
      Vec8<T>::load(w + ch * 8, wv);
      if (!RMS && b != nullptr) {
        float bv[8];
        Vec8<T>::load(b + ch * 8, bv);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (v[c][j] - mean) * rstd * wv[j] + bv[j];
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (v[c][j] - mean) * rstd * wv[j];
      }
      Vec8<T>::store(yr + ch * 8, o);
    }
  }
  if (lane == 0) {
    rstd_out[row] = rstd;
    if (!RMS) mean_out[row] = mean;
  }
}

// ---------------------------------------------------------------------------
// backward: dx (+ optional extra gradient added, e.g. residual-stream grad),
// per-workgroup fp32 partials of dw (and db for LayerNorm).
// partial layout: [gridDim.x][cols] for dw, then [gridDim.x][cols] for db.
// ---------------------------------------------------------------------------
// A/B knobs (scripts/norm_bench.py, profiles/r2_norm): keep the row in
// registers between the two passes below this CH; resident workgroups per CU
#ifndef NORM_KEEP_BELOW
#define NORM_KEEP_BELOW 8
#endif
#ifndef NORM_NT_SINGLE
#define NORM_NT_SINGLE 1
#endif
#ifndef NORM_BWD_WG_PER_CU
#define NORM_BWD_WG_PER_CU 3
#endif

template <typename T, int CH, bool RMS>
__global__ __launch_bounds__(256) void norm_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ h,
                                                       const T* __restrict__ w, const float* __restrict__ mean_in,
                                                       const float* __restrict__ rstd_in,
                                                       const T* __restrict__ dadd, T* __restrict__ dx,
                                                       float* __restrict__ partial, int rows, int cols) {
  extern __shared__ __attribute__((aligned(16))) float lds[];  // [4][512] (+[4][512] for db)
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nch = cols >> 3;
  // register budget at CH=8 (4096 cols): dw partial 64 + db partial 64 (LN only)
  // + x-hat 64 + dy 64; the weight is re-read per row (8 KB, L1/L2 resident).
  float dwacc[CH][8];
  float dbacc[CH][8];
#pragma unroll
  for (int c = 0; c < CH; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) { dwacc[c][j] = 0.f; dbacc[c][j] = 0.f; }
  for (int row = blockIdx.x * 4 + wid; row < rows; row += gridDim.x * 4) {
    const float rstd = rstd_in[row];
    const float mean = RMS ? 0.f : mean_in[row];
    // At CH >= 8 the row is NOT kept in registers between the two passes: the
    // second pass re-reads h / dy (L2 / Infinity-Cache hits) so the kernel
    // stays at ~100 VGPRs (4 waves/SIMD) instead of 256 (1 wave/SIMD).
    constexpr bool KEEP = CH < NORM_KEEP_BELOW;
    float xh[KEEP ? CH : 1][8], d[KEEP ? CH : 1][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int ch = lane + c * 64;
      const int cc = KEEP ? c : 0;
      if (ch < nch) {
        float wv[8];
        Vec8<T>::load(h + (int64_t)row * cols + ch * 8, xh[cc]);
        Vec8<T>::load(dy + (int64_t)row * cols + ch * 8, d[cc]);
        Vec8<T>::load(w + ch * 8, wv);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xh[cc][j] = (xh[cc][j] - mean) * rstd;
          const float g = d[cc][j] * wv[j];
          s1 = fmaf(g, xh[cc][j], s1);
          s2 += g;
          dwacc[c][j] = fmaf(d[cc][j], xh[cc][j], dwacc[c][j]);
          if (!RMS) dbacc[c][j] += d[cc][j];
        }
      } else if (KEEP) {
#pragma unroll
        for (int j = 0; j < 8; ++j) { xh[cc][j] = 0.f; d[cc][j] = 0.f; }
      }
    }
    s1 = wave_sum(s1) / cols;
    if (!RMS) s2 = wave_sum(s2) / cols;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int ch = lane + c * 64;
      if (ch < nch) {
        float o[8], wv[8];
        const int cc = KEEP ? c : 0;
        if (!KEEP) {
          Vec8<T>::load(h + (int64_t)row * cols + ch * 8, xh[0]);
          Vec8<T>::load(dy + (int64_t)row * cols + ch * 8, d[0]);
#pragma unroll
          for (int j = 0; j < 8; ++j) xh[0][j] = (xh[0][j] - mean) * rstd;
        }
        Vec8<T>::load(w + ch * 8, wv);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float g = d[cc][j] * wv[j];
          o[j] = RMS ? (g - xh[cc][j] * s1) * rstd : (g - s2 - xh[cc][j] * s1) * rstd;
        }
        if (dadd != nullptr) {
          float a[8];
          if (NORM_NT_SINGLE && sizeof(T) == 2)
            unpack8(__builtin_nontemporal_load((const u32x4*)(dadd + (int64_t)row * cols + ch * 8)), a);
          else
            Vec8<T>::load(dadd + (int64_t)row * cols + ch * 8, a);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] += a[j];
        }
        // single-use streams (dadd, dx) non-temporal: they leave the L2 to
        // the h / dy rows the second pass re-reads
        if (NORM_NT_SINGLE && sizeof(T) == 2)
          __builtin_nontemporal_store(pack8(o), (u32x4*)(dx + (int64_t)row * cols + ch * 8));
        else
          Vec8<T>::store(dx + (int64_t)row * cols + ch * 8, o);
      }
    }
  }
  // reduce the 4 waves' column partials through LDS, one 512-column chunk at a
  // time: 8 KB of LDS (16 KB for LayerNorm) instead of 64 KB for a 4096-wide
  // row, so LDS no longer caps the kernel at 2 workgroups per CU
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int ch = lane + c * 64;
    if (c) __syncthreads();
    if (ch < nch) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        lds[wid * 512 + lane * 8 + j] = dwacc[c][j];
        if (!RMS) lds[4 * 512 + wid * 512 + lane * 8 + j] = dbacc[c][j];
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int lc = threadIdx.x + k * 256, col = c * 512 + lc;
      if (col < cols) {
        partial[(int64_t)blockIdx.x * cols + col] = lds[lc] + lds[512 + lc] + lds[1024 + lc] + lds[1536 + lc];
        if (!RMS)
          partial[(int64_t)gridDim.x * cols + (int64_t)blockIdx.x * cols + col] =
              lds[2048 + lc] + lds[2560 + lc] + lds[3072 + lc] + lds[3584 + lc];
      }
    }
  }
}

// out[c] (+)= sum_b partial[b][c]; out dtype bf16 (out_bf16=1) or fp32.
// One 512-thread workgroup per 64-column strip: wave w sums partial rows
// b = w (mod 8) with 4 independent accumulators (coalesced 256-B rows), then
// the 8 wave sums meet in LDS in a fixed order (deterministic).  The old
// one-thread-per-column loop ran 16 workgroups on 256 CUs, latency-bound.
__global__ __launch_bounds__(512) void col_reduce_kernel(const float* __restrict__ partial, int nb, int cols,
                                                         void* __restrict__ out, int out_bf16, int accumulate) {
  __shared__ float red[8][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + lane;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (col < cols) {
    int b = wave;
    for (; b + 24 < nb; b += 32) {
      a0 += partial[(int64_t)b * cols + col];
      a1 += partial[(int64_t)(b + 8) * cols + col];
      a2 += partial[(int64_t)(b + 16) * cols + col];
      a3 += partial[(int64_t)(b + 24) * cols + col];
    }
    for (; b < nb; b += 8) a0 += partial[(int64_t)b * cols + col];
  }
  red[wave][lane] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (wave != 0 || col >= cols) return;
  float t = 0.f;
#pragma unroll
  for (int w = 0; w < 8; ++w) t += red[w][lane];
  if (out_bf16) {
    bf16_t* o = (bf16_t*)out;
    if (accumulate) t += bf2f(o[col]);
    o[col] = f2bf(t);
  } else {
    float* o = (float*)out;
    o[col] = accumulate ? o[col] + t : t;
  }
}

static inline int pick_ch(int cols) {
  int need = (cols / 8 + 63) / 64;
  if (need <= 1) return 1;
  if (need <= 2) return 2;
  if (need <= 4) return 4;
  if (need <= 8) return 8;
  if (need <= 16) return 16;
  return -1;
}

#define TOA_NORM_DISPATCH(CHV, ...)          \
  switch (CHV) {                             \
    case 1: { constexpr int CH = 1; __VA_ARGS__; break; } \
    case 2: { constexpr int CH = 2; __VA_ARGS__; break; } \
    case 4: { constexpr int CH = 4; __VA_ARGS__; break; } \
    case 8: { constexpr int CH = 8; __VA_ARGS__; break; } \
    case 16: { constexpr int CH = 16; __VA_ARGS__; break; } \
    default: return (int)hipErrorInvalidValue; \
  }

// RMSNorm form for bf16 rows of 2048-multiple width up to 8192: 1 = one row
// per workgroup (rms_fwd_row_kernel / rms_bwd_row_kernel, the default), 0 =
// one row per wave (norm_fwd_kernel / norm_bwd_kernel, every other shape).
// toa_norm_set_row pins a form for in-process tests (-1 = the default).
static int g_norm_row = 1;
// Forward row kernel's grid cap in workgroups (toa_norm_set_fwd_cap for A/B).
// One row per workgroup, no cap: 0.1488 -> 0.1381 ms at 24576 x 4096 against
// the old 2048-workgroup grid-stride (scripts/rms_fwd_grid_ab.py,
// profiles/r5_grid/rms_fwd.log); outputs identical.
static const int kNormFwdCapDefault = 1 << 30;
static int g_norm_fwd_cap = kNormFwdCapDefault;
extern "C" int toa_norm_set_fwd_cap(int c) {
  g_norm_fwd_cap = c > 0 ? c : kNormFwdCapDefault;
  return 0;
}
static int norm_row_form() { return g_norm_row; }
extern "C" int toa_norm_set_row(int v) {
  g_norm_row = v < 0 ? 1 : (v ? 1 : 0);
  return 0;
}

// RMSNorm forward (+ residual add), one row per workgroup (bf16, cols a
// multiple of 2048, at most 8192): each wave a contiguous quarter of the row,
// the sum of squares across the waves through a double-buffered LDS pair (one
// barrier per row), the weight loaded once per workgroup, and h rounded to
// bf16 in registers (the value backward re-reads) instead of re-loaded from
// the store just made.  Grid-stride over rows.
template <int CPL>
__global__ __launch_bounds__(256) void rms_fwd_row_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ res,
                                                          bf16_t* __restrict__ h_out, const bf16_t* __restrict__ w,
                                                          bf16_t* __restrict__ y, float* __restrict__ rstd_out,
                                                          int rows, int cols, float eps) {
  __shared__ float red[2][4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int col0 = wid * (cols >> 2);
  float wv[CPL][8];
#pragma unroll
  for (int c = 0; c < CPL; ++c) Vec8<bf16_t>::load(w + col0 + (c * 64 + lane) * 8, wv[c]);
  const float inv_cols = 1.f / (float)cols;
  int par = 0;
  for (int row = blockIdx.x; row < rows; row += gridDim.x, par ^= 1) {
    const int64_t base = (int64_t)row * cols + col0;
    float v[CPL][8];
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const int64_t off = base + (c * 64 + lane) * 8;
      Vec8<bf16_t>::load(x + off, v[c]);
      if (res != nullptr) {
        float r[8];
        Vec8<bf16_t>::load(res + off, r);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] += r[j];
        const u32x4 hv = pack8(v[c]);
        st16(h_out + off, hv);
        unpack8(hv, v[c]);  // the rounded values: what backward reads back
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) s = fmaf(v[c][j], v[c][j], s);
    }
    s = wave_sum(s);
    if (lane == 0) red[par][wid] = s;
    __syncthreads();
    const float rstd = rsqrtf((red[par][0] + red[par][1] + red[par][2] + red[par][3]) * inv_cols + eps);
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = v[c][j] * rstd * wv[c][j];
      Vec8<bf16_t>::store(y + base + (c * 64 + lane) * 8, o);
    }
    if (threadIdx.x == 0) rstd_out[row] = rstd;
  }
}

template <typename T, bool RMS>
static int norm_fwd_launch(const void* x, const void* res, void* h_out, const void* w, const void* b, void* y,
                           float* mean, float* rstd, int rows, int cols, float eps, hipStream_t s) {
  if (cols % 8 != 0) return (int)hipErrorInvalidValue;
  int chv = pick_ch(cols);
  if (RMS && sizeof(T) == 2 && cols % 2048 == 0 && cols <= 8192 && norm_row_form()) {
    const int nb = rows < g_norm_fwd_cap ? rows : g_norm_fwd_cap;  // grid-stride over rows beyond the cap
    const bf16_t *x16 = (const bf16_t*)x, *r16 = (const bf16_t*)res, *w16 = (const bf16_t*)w;
    bf16_t *h16 = (bf16_t*)h_out, *y16 = (bf16_t*)y;
    switch (cols / 2048) {
      case 1: hipLaunchKernelGGL(rms_fwd_row_kernel<1>, dim3(nb), dim3(256), 0, s, x16, r16, h16, w16, y16, rstd, rows,
                                 cols, eps); break;
      case 2: hipLaunchKernelGGL(rms_fwd_row_kernel<2>, dim3(nb), dim3(256), 0, s, x16, r16, h16, w16, y16, rstd, rows,
                                 cols, eps); break;
      case 3: hipLaunchKernelGGL(rms_fwd_row_kernel<3>, dim3(nb), dim3(256), 0, s, x16, r16, h16, w16, y16, rstd, rows,
                                 cols, eps); break;
      default: hipLaunchKernelGGL(rms_fwd_row_kernel<4>, dim3(nb), dim3(256), 0, s, x16, r16, h16, w16, y16, rstd,
                                  rows, cols, eps); break;
    }
    return (int)hipGetLastError();
  }
  dim3 grid((rows + 3) / 4), block(256);
  TOA_NORM_DISPATCH(chv, hipLaunchKernelGGL((norm_fwd_kernel<T, CH, RMS>), grid, block, 0, s, (const T*)x,
                                            (const T*)res, (T*)h_out, (const T*)w, (const T*)b, (T*)y, mean, rstd,
                                            rows, cols, eps));
  return (int)hipGetLastError();
}

// RMSNorm backward, one row per workgroup (bf16, cols a multiple of 2048, at
// most 8192): the row's 4 waves each own a contiguous quarter of the columns
// (CPL 16-byte chunks per lane), so h and dy stay in registers between the
// two halves of the row (no second read) and the weight, the same for every
// row, is loaded once.  The row sum crosses the waves through LDS, double
// buffered so one barrier per row suffices (row k + 2 rewrites row k's slot
// only after every wave has passed row k + 1's barrier, i.e. read row k's).
// Each wave's dW partials cover its own columns: written straight to
// partial[blockIdx.x][cols] for col_reduce_kernel, no LDS reduction.
template <int CPL>
__global__ __launch_bounds__(256) void rms_bwd_row_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ h,
                                                          const bf16_t* __restrict__ w,
                                                          const float* __restrict__ rstd_in,
                                                          const bf16_t* __restrict__ dadd, bf16_t* __restrict__ dx,
                                                          float* __restrict__ partial, int rows, int cols) {
  __shared__ float red[2][4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int col0 = wid * (cols >> 2);  // this wave's quarter
  float wv[CPL][8], dw[CPL][8];
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    Vec8<bf16_t>::load(w + col0 + (c * 64 + lane) * 8, wv[c]);
#pragma unroll
    for (int j = 0; j < 8; ++j) dw[c][j] = 0.f;
  }
  const float inv_cols = 1.f / (float)cols;
  int par = 0;
  for (int row = blockIdx.x; row < rows; row += gridDim.x, par ^= 1) {
    const float rstd = rstd_in[row];
    const int64_t base = (int64_t)row * cols + col0;
    float xh[CPL][8], g[CPL][8];
    float s1 = 0.f;
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      float d[8];
      Vec8<bf16_t>::load(h + base + (c * 64 + lane) * 8, xh[c]);
      Vec8<bf16_t>::load(dy + base + (c * 64 + lane) * 8, d);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        xh[c][j] *= rstd;
        g[c][j] = d[j] * wv[c][j];
        s1 = fmaf(g[c][j], xh[c][j], s1);
        dw[c][j] = fmaf(d[j], xh[c][j], dw[c][j]);
      }
    }
    s1 = wave_sum(s1);
    if (lane == 0) red[par][wid] = s1;
    __syncthreads();
    s1 = (red[par][0] + red[par][1] + red[par][2] + red[par][3]) * inv_cols;
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const int64_t off = base + (c * 64 + lane) * 8;
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (g[c][j] - xh[c][j] * s1) * rstd;
      if (dadd != nullptr) {
        float a[8];
        unpack8(__builtin_nontemporal_load((const u32x4*)(dadd + off)), a);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] += a[j];
      }
      __builtin_nontemporal_store(pack8(o), (u32x4*)(dx + off));
    }
  }
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    float* pp = partial + (int64_t)blockIdx.x * cols + col0 + (c * 64 + lane) * 8;
    *(f32x4*)pp = f32x4{dw[c][0], dw[c][1], dw[c][2], dw[c][3]};
    *((f32x4*)pp + 1) = f32x4{dw[c][4], dw[c][5], dw[c][6], dw[c][7]};
  }
}

// number of workgroups the backward uses (=> partial rows); caller sizes the
// partial workspace as nb * cols * (RMS ? 1 : 2) floats.
extern "C" int toa_norm_bwd_blocks(int rows, int cols) {
  // ~154 VGPRs at <= 4096 columns: 3 workgroups (12 waves) resident per CU on 256 CUs
  int nb = (rows + 3) / 4;
  int cap = cols > 4096 ? 256 : 256 * NORM_BWD_WG_PER_CU;
  return nb < cap ? nb : cap;
}

template <typename T, bool RMS>
static int norm_bwd_launch(const void* dy, const void* h, const void* w, const float* mean, const float* rstd,
                           const void* dadd, void* dx, float* partial, void* dw, int dw_bf16, void* db,
                           int db_bf16, int accumulate, int rows, int cols, hipStream_t s) {
  if (cols % 8 != 0) return (int)hipErrorInvalidValue;
  int chv = pick_ch(cols);
  int nb = toa_norm_bwd_blocks(rows, cols);
  size_t lds = (size_t)4 * 512 * sizeof(float) * (RMS ? 1 : 2);
  if (RMS && sizeof(T) == 2 && cols % 2048 == 0 && cols <= 8192 && norm_row_form()) {
    const bf16_t *dy16 = (const bf16_t*)dy, *h16 = (const bf16_t*)h, *w16 = (const bf16_t*)w,
                 *a16 = (const bf16_t*)dadd;
    bf16_t* dx16 = (bf16_t*)dx;
    switch (cols / 2048) {
      case 1: hipLaunchKernelGGL(rms_bwd_row_kernel<1>, dim3(nb), dim3(256), 0, s, dy16, h16, w16, rstd, a16, dx16,
                                 partial, rows, cols); break;
      case 2: hipLaunchKernelGGL(rms_bwd_row_kernel<2>, dim3(nb), dim3(256), 0, s, dy16, h16, w16, rstd, a16, dx16,
                                 partial, rows, cols); break;
      case 3: hipLaunchKernelGGL(rms_bwd_row_kernel<3>, dim3(nb), dim3(256), 0, s, dy16, h16, w16, rstd, a16, dx16,
                                 partial, rows, cols); break;
      default: hipLaunchKernelGGL(rms_bwd_row_kernel<4>, dim3(nb), dim3(256), 0, s, dy16, h16, w16, rstd, a16,
                                  dx16, partial, rows, cols); break;
    }
  } else {
    TOA_NORM_DISPATCH(chv, hipLaunchKernelGGL((norm_bwd_kernel<T, CH, RMS>), dim3(nb), dim3(256), lds, s,
                                              (const T*)dy, (const T*)h, (const T*)w, mean, rstd, (const T*)dadd,
                                              (T*)dx, partial, rows, cols));
  }
  dim3 rg((cols + 63) / 64);
  if (dw != nullptr)
    hipLaunchKernelGGL(col_reduce_kernel, rg, dim3(512), 0, s, partial, nb, cols, dw, dw_bf16, accumulate);
  if (!RMS && db != nullptr)
    hipLaunchKernelGGL(col_reduce_kernel, rg, dim3(512), 0, s, partial + (int64_t)nb * cols, nb, cols, db,
                       db_bf16, accumulate);
  return (int)hipGetLastError();
}

// dtype: 0 = bf16, 1 = fp32
extern "C" int toa_rmsnorm_fwd(int dtype, const void* x, const void* res, void* h_out, const void* w, void* y,
                               float* rstd, int rows, int cols, float eps, hipStream_t s) {
  return dtype == 0 ? norm_fwd_launch<bf16_t, true>(x, res, h_out, w, nullptr, y, nullptr, rstd, rows, cols, eps, s)
                    : norm_fwd_launch<float, true>(x, res, h_out, w, nullptr, y, nullptr, rstd, rows, cols, eps, s);
}

extern "C" int toa_rmsnorm_bwd(int dtype, const void* dy, const void* h, const void* w, const float* rstd,
                               const void* dadd, void* dx, float* partial, void* dw, int dw_bf16, int accumulate,
                               int rows, int cols, hipStream_t s) {
  return dtype == 0 ? norm_bwd_launch<bf16_t, true>(dy, h, w, nullptr, rstd, dadd, dx, partial, dw, dw_bf16,
                                                    nullptr, 0, accumulate, rows, cols, s)
                    : norm_bwd_launch<float, true>(dy, h, w, nullptr, rstd, dadd, dx, partial, dw, dw_bf16, nullptr,
                                                   0, accumulate, rows, cols, s);
}

extern "C" int toa_layernorm_fwd(int dtype, const void* x, const void* res, void* h_out, const void* w,
                                 const void* b, void* y, float* mean, float* rstd, int rows, int cols, float eps,
                                 hipStream_t s) {
  return dtype == 0 ? norm_fwd_launch<bf16_t, false>(x, res, h_out, w, b, y, mean, rstd, rows, cols, eps, s)
                    : norm_fwd_launch<float, false>(x, res, h_out, w, b, y, mean, rstd, rows, cols, eps, s);
}

extern "C" int toa_layernorm_bwd(int dtype, const void* dy, const void* h, const void* w, const float* mean,
                                 const float* rstd, const void* dadd, void* dx, float* partial, void* dw,
                                 int dw_bf16, void* db, int db_bf16, int accumulate, int rows, int cols,
                                 hipStream_t s) {
  return dtype == 0 ? norm_bwd_launch<bf16_t, false>(dy, h, w, mean, rstd, dadd, dx, partial, dw, dw_bf16, db,
                                                     db_bf16, accumulate, rows, cols, s)
                    : norm_bwd_launch<float, false>(dy, h, w, mean, rstd, dadd, dx, partial, dw, dw_bf16, db,
                                                    db_bf16, accumulate, rows, cols, s);
}
