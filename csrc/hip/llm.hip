// Transformer elementwise / reduction kernels for the Llama-family trainer
// (gfx950): RoPE (+ head-major relayout + GQA expansion), SwiGLU, and the
// vocab-parallel-free fused softmax cross-entropy.
//
// All are HBM-bound; each moves bf16 data 16 B per lane (guide G13) and does
// its layout change in the same pass, so no separate transpose/contiguous()
// kernels run around them.
//
// Reference parity: SURVEY K19 north-star additions (Llama-3-8B) and K4
// (`dist_mnist.py:192` clip+log+mul+reduce_sum cross entropy).
#include "toa_common.h"

#include <algorithm>

// ---------------------------------------------------------------------------
// RoPE.  qkv: [T = B*S, (Hq + 2*Hkv) * D] (output of the fused QKV GEMM).
// Writes q: [B, Hq, S, D], k / v: [B, Hkv*rep, S, D] (rep = kv replication
// factor: Hq/Hkv to feed an MHA attention kernel, 1 to keep GQA packed).
// cos/sin: [S, D/2] fp32.  Llama rotate-half convention: pair (i, i + D/2).
// Work unit = one (token, qkv-head, 8-wide pair chunk).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void rope_fwd_kernel(const bf16_t* __restrict__ qkv, const float* __restrict__ cosv,
                                                       const float* __restrict__ sinv, bf16_t* __restrict__ q,
                                                       bf16_t* __restrict__ k, bf16_t* __restrict__ v, int B, int S,
                                                       int Hq, int Hkv, int D, int rep) {
  const int half = D / 2, cpd = half / 8;  // 8-wide chunks per half-head
  const int H3 = Hq + 2 * Hkv;
  const int64_t units = (int64_t)B * S * H3 * cpd;
  const int Hk = Hkv * rep;
  for (int64_t u = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; u < units; u += (int64_t)gridDim.x * blockDim.x) {
    const int c = u % cpd;
    const int64_t r = u / cpd;
    const int h = r % H3;
    const int64_t t = r / H3;
    const int s = t % S, b = t / S;
    const bf16_t* src = qkv + t * (int64_t)(H3 * D) + h * D + c * 8;
    u32x4 x1v = ld16(src), x2v = ld16(src + half);
    if (h >= Hq + Hkv) {  // V: copy into every replica
      const int g = h - Hq - Hkv;
      for (int rr = 0; rr < rep; ++rr) {
        bf16_t* dst = v + (((int64_t)b * Hk + g * rep + rr) * S + s) * D + c * 8;
        st16(dst, x1v);
        st16(dst + half, x2v);
      }
      continue;
    }
    float x1[8], x2[8], y1[8], y2[8];
    unpack8(x1v, x1);
    unpack8(x2v, x2);
    const float* cp = cosv + (int64_t)s * half + c * 8;
    const float* sp = sinv + (int64_t)s * half + c * 8;
    f32x4 c0 = *(const f32x4*)cp, c1 = *(const f32x4*)(cp + 4);
    f32x4 s0 = *(const f32x4*)sp, s1 = *(const f32x4*)(sp + 4);
    float cs[8] = {c0[0], c0[1], c0[2], c0[3], c1[0], c1[1], c1[2], c1[3]};
    float sn[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      y1[j] = x1[j] * cs[j] - x2[j] * sn[j];
      y2[j] = x2[j] * cs[j] + x1[j] * sn[j];
    }
    u32x4 o1 = pack8(y1), o2 = pack8(y2);
    if (h < Hq) {
      bf16_t* dst = q + (((int64_t)b * Hq + h) * S + s) * D + c * 8;
      st16(dst, o1);
      st16(dst + half, o2);
    } else {
      const int g = h - Hq;
      for (int rr = 0; rr < rep; ++rr) {
        bf16_t* dst = k + (((int64_t)b * Hk + g * rep + rr) * S + s) * D + c * 8;
        st16(dst, o1);
        st16(dst + half, o2);
      }
    }
  }
}

// Backward: dq/dk/dv in head-major layout (dk/dv with `rep` replicas) ->
// dqkv [T, (Hq+2Hkv)*D]; replica gradients are summed, rotation inverted.
__global__ __launch_bounds__(256) void rope_bwd_kernel(const bf16_t* __restrict__ dq, const bf16_t* __restrict__ dk,
                                                       const bf16_t* __restrict__ dv, const float* __restrict__ cosv,
                                                       const float* __restrict__ sinv, bf16_t* __restrict__ dqkv,
                                                       int B, int S, int Hq, int Hkv, int D, int rep) {
  const int half = D / 2, cpd = half / 8;
  const int H3 = Hq + 2 * Hkv;
  const int64_t units = (int64_t)B * S * H3 * cpd;
  const int Hk = Hkv * rep;
  for (int64_t u = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; u < units; u += (int64_t)gridDim.x * blockDim.x) {
    const int c = u % cpd;
    const int64_t r = u / cpd;
    const int h = r % H3;
    const int64_t t = r / H3;
    const int s = t % S, b = t / S;
    float y1[8], y2[8];
    if (h < Hq) {
      const bf16_t* src = dq + (((int64_t)b * Hq + h) * S + s) * D + c * 8;
      unpack8(ld16(src), y1);
      unpack8(ld16(src + half), y2);
    } else {
      const bool isv = h >= Hq + Hkv;
      const int g = isv ? h - Hq - Hkv : h - Hq;
      const bf16_t* base = isv ? dv : dk;
#pragma unroll
      for (int j = 0; j < 8; ++j) { y1[j] = 0.f; y2[j] = 0.f; }
      for (int rr = 0; rr < rep; ++rr) {
        const bf16_t* src = base + (((int64_t)b * Hk + g * rep + rr) * S + s) * D + c * 8;
        float a1[8], a2[8];
        unpack8(ld16(src), a1);
        unpack8(ld16(src + half), a2);
#pragma unroll
        for (int j = 0; j < 8; ++j) { y1[j] += a1[j]; y2[j] += a2[j]; }
      }
      if (isv) {
        bf16_t* dst = dqkv + t * (int64_t)(H3 * D) + h * D + c * 8;
        st16(dst, pack8(y1));
        st16(dst + half, pack8(y2));
        continue;
      }
    }
    const float* cp = cosv + (int64_t)s * half + c * 8;
    const float* sp = sinv + (int64_t)s * half + c * 8;
    f32x4 c0 = *(const f32x4*)cp, c1 = *(const f32x4*)(cp + 4);
    f32x4 s0 = *(const f32x4*)sp, s1 = *(const f32x4*)(sp + 4);
    float cs[8] = {c0[0], c0[1], c0[2], c0[3], c1[0], c1[1], c1[2], c1[3]};
    float sn[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
    float x1[8], x2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      x1[j] = y1[j] * cs[j] + y2[j] * sn[j];
      x2[j] = y2[j] * cs[j] - y1[j] * sn[j];
    }
    bf16_t* dst = dqkv + t * (int64_t)(H3 * D) + h * D + c * 8;
    st16(dst, pack8(x1));
    st16(dst + half, pack8(x2));
  }
}

extern "C" int toa_rope_fwd(const bf16_t* qkv, const float* cosv, const float* sinv, bf16_t* q, bf16_t* k, bf16_t* v,
                            int B, int S, int Hq, int Hkv, int D, int rep, hipStream_t stream) {
  if (D % 16 != 0 || Hq % Hkv != 0) return (int)hipErrorInvalidValue;
  int64_t units = (int64_t)B * S * (Hq + 2 * Hkv) * (D / 16);
  // one unit per thread (a 2048-block cap left each thread 18 units at the bench shape)
  const unsigned grid = (unsigned)std::max<int64_t>((units + 255) / 256, 1);
  hipLaunchKernelGGL(rope_fwd_kernel, dim3(grid), dim3(256), 0, stream, qkv, cosv, sinv, q, k,
                     v, B, S, Hq, Hkv, D, rep);
  return (int)hipGetLastError();
}

extern "C" int toa_rope_bwd(const bf16_t* dq, const bf16_t* dk, const bf16_t* dv, const float* cosv,
                            const float* sinv, bf16_t* dqkv, int B, int S, int Hq, int Hkv, int D, int rep,
                            hipStream_t stream) {
  if (D % 16 != 0 || Hq % Hkv != 0) return (int)hipErrorInvalidValue;
  int64_t units = (int64_t)B * S * (Hq + 2 * Hkv) * (D / 16);
  hipLaunchKernelGGL(rope_bwd_kernel, dim3(toa_stream_grid(units, 256)), dim3(256), 0, stream, dq, dk, dv, cosv,
                     sinv, dqkv, B, S, Hq, Hkv, D, rep);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// SwiGLU: gu [T, 2F] (gate | up) -> out [T, F] = silu(gate) * up
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void swiglu_fwd_kernel(const bf16_t* __restrict__ gu, bf16_t* __restrict__ out,
                                                         int64_t T, int F) {
  const int fc = F / 8;
  const int64_t units = T * fc;
  for (int64_t u = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; u < units; u += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = u / fc;
    const int c = u % fc;
    const bf16_t* row = gu + t * 2 * F;
    float g[8], up[8], o[8];
    unpack8(ld16(row + c * 8), g);
    unpack8(ld16(row + F + c * 8), up);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = g[j] / (1.f + __expf(-g[j])) * up[j];
    st16(out + t * F + c * 8, pack8(o));
  }
}

__global__ __launch_bounds__(256) void swiglu_bwd_kernel(const bf16_t* __restrict__ dout, const bf16_t* __restrict__ gu,
                                                         bf16_t* __restrict__ dgu, int64_t T, int F) {
  const int fc = F / 8;
  const int64_t units = T * fc;
  for (int64_t u = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; u < units; u += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = u / fc;
    const int c = u % fc;
    const bf16_t* row = gu + t * 2 * F;
    float g[8], up[8], d[8], dg[8], du[8];
    unpack8(ld16(row + c * 8), g);
    unpack8(ld16(row + F + c * 8), up);
    unpack8(ld16(dout + t * F + c * 8), d);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float sg = 1.f / (1.f + __expf(-g[j]));
      const float silu = g[j] * sg;
      du[j] = d[j] * silu;
      dg[j] = d[j] * up[j] * sg * (1.f + g[j] * (1.f - sg));
    }
    st16(dgu + t * 2 * F + c * 8, pack8(dg));
    st16(dgu + t * 2 * F + F + c * 8, pack8(du));
  }
}

// Row-structured forms: workgroup per row (grid-strided over rows), threads
// over the row's 16-B chunks -- no 64-bit divide per chunk -- with
// non-temporal loads/stores (every byte is touched once; the 1-3 GB streams
// are far beyond the Infinity Cache).  Selected by toa_set_stream_variant
// bit 1 (in-process A/B, scripts/stream_ab.py).
__global__ __launch_bounds__(256) void swiglu_fwd_rows_kernel(const bf16_t* __restrict__ gu, bf16_t* __restrict__ out,
                                                              int64_t T, int F) {
  const int fc = F / 8;
  for (int64_t t = blockIdx.x; t < T; t += gridDim.x) {
    const u32x4* row = (const u32x4*)(gu + t * 2 * F);
    u32x4* orow = (u32x4*)(out + t * F);
    for (int c = threadIdx.x; c < fc; c += blockDim.x) {
      float g[8], up[8], o[8];
      unpack8(__builtin_nontemporal_load(row + c), g);
      unpack8(__builtin_nontemporal_load(row + fc + c), up);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = g[j] / (1.f + __expf(-g[j])) * up[j];
      __builtin_nontemporal_store(pack8(o), orow + c);
    }
  }
}

__global__ __launch_bounds__(256) void swiglu_bwd_rows_kernel(const bf16_t* __restrict__ dout,
                                                              const bf16_t* __restrict__ gu, bf16_t* __restrict__ dgu,
                                                              int64_t T, int F) {
  const int fc = F / 8;
  for (int64_t t = blockIdx.x; t < T; t += gridDim.x) {
    const u32x4* row = (const u32x4*)(gu + t * 2 * F);
    const u32x4* drow = (const u32x4*)(dout + t * F);
    u32x4* orow = (u32x4*)(dgu + t * 2 * F);
    for (int c = threadIdx.x; c < fc; c += blockDim.x) {
      float g[8], up[8], d[8], dg[8], du[8];
      unpack8(__builtin_nontemporal_load(row + c), g);
      unpack8(__builtin_nontemporal_load(row + fc + c), up);
      unpack8(__builtin_nontemporal_load(drow + c), d);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float sg = 1.f / (1.f + __expf(-g[j]));
        const float silu = g[j] * sg;
        du[j] = d[j] * silu;
        dg[j] = d[j] * up[j] * sg * (1.f + g[j] * (1.f - sg));
      }
      __builtin_nontemporal_store(pack8(dg), orow + c);
      __builtin_nontemporal_store(pack8(du), orow + fc + c);
    }
  }
}

static inline int rows_grid(int64_t T) { return (int)std::min<int64_t>(std::max<int64_t>(T, 1), 4096); }

extern "C" int toa_swiglu_fwd(const bf16_t* gu, bf16_t* out, int64_t T, int F, hipStream_t stream) {
  if (F % 8 != 0) return (int)hipErrorInvalidValue;
  if (toa_stream_variant() & 2)
    hipLaunchKernelGGL(swiglu_fwd_rows_kernel, dim3(rows_grid(T)), dim3(256), 0, stream, gu, out, T, F);
  else
    hipLaunchKernelGGL(swiglu_fwd_kernel, dim3(toa_stream_grid(T * (F / 8), 256)), dim3(256), 0, stream, gu, out, T,
                       F);
  return (int)hipGetLastError();
}

extern "C" int toa_swiglu_bwd(const bf16_t* dout, const bf16_t* gu, bf16_t* dgu, int64_t T, int F,
                              hipStream_t stream) {
  if (F % 8 != 0) return (int)hipErrorInvalidValue;
  if (toa_stream_variant() & 2)
    hipLaunchKernelGGL(swiglu_bwd_rows_kernel, dim3(rows_grid(T)), dim3(256), 0, stream, dout, gu, dgu, T, F);
  else
    hipLaunchKernelGGL(swiglu_bwd_kernel, dim3(toa_stream_grid(T * (F / 8), 256)), dim3(256), 0, stream, dout, gu,
                       dgu, T, F);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Cross entropy over a (large) vocabulary, one workgroup per row.
//   forward : loss[row] = lse(row) - x[row, target],  lse saved   (1 HBM read)
//   backward: dx = (softmax - onehot) * (*grad_out / *n_valid)    (1 read, 1 write,
//             may run in place over the logits buffer)
// Rows whose target == ignore_index get loss 0 and zero gradient.
// logits dtype: bf16 (0) or fp32 (1).
// ---------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ void ld8(const T* p, float* f);
template <>
__device__ __forceinline__ void ld8<bf16_t>(const bf16_t* p, float* f) { unpack8(ld16(p), f); }
template <>
__device__ __forceinline__ void ld8<float>(const float* p, float* f) {
  f32x4 a = *(const f32x4*)p, b = *((const f32x4*)p + 1);
  f[0] = a[0]; f[1] = a[1]; f[2] = a[2]; f[3] = a[3];
  f[4] = b[0]; f[5] = b[1]; f[6] = b[2]; f[7] = b[3];
}
template <typename T>
__device__ __forceinline__ void st8(T* p, const float* f);
template <>
__device__ __forceinline__ void st8<bf16_t>(bf16_t* p, const float* f) { st16(p, pack8(f)); }
template <>
__device__ __forceinline__ void st8<float>(float* p, const float* f) {
  f32x4 a = {f[0], f[1], f[2], f[3]}, b = {f[4], f[5], f[6], f[7]};
  *(f32x4*)p = a;
  *((f32x4*)p + 1) = b;
}
template <typename T>
__device__ __forceinline__ float ld1(const T* p);
template <>
__device__ __forceinline__ float ld1<bf16_t>(const bf16_t* p) { return bf2f(*p); }
template <>
__device__ __forceinline__ float ld1<float>(const float* p) { return *p; }

template <typename T>
__global__ __launch_bounds__(512) void xent_fwd_kernel(const T* __restrict__ logits, const int64_t* __restrict__ tgt,
                                                       float* __restrict__ loss, float* __restrict__ lse_out,
                                                       int V, int64_t ldx, int ignore_index) {
  __shared__ float sm[8], ss[8];
  const int64_t row = blockIdx.x;
  const T* x = logits + row * ldx;
  const int64_t target = tgt[row];
  float m = -INFINITY, s = 0.f;
  const int v8 = (V % 8 == 0 && ldx % 8 == 0) ? V / 8 : 0;
  for (int i = threadIdx.x; i < v8; i += blockDim.x) {
    float f[8];
    ld8<T>(x + i * 8, f);
    float mx = f[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) mx = fmaxf(mx, f[j]);
    float mn = fmaxf(m, mx);
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += __expf(f[j] - mn);
    s = s * __expf(m - mn) + acc;
    m = mn;
  }
  for (int i = v8 * 8 + threadIdx.x; i < V; i += blockDim.x) {
    float f = ld1<T>(x + i);
    float mn = fmaxf(m, f);
    s = s * __expf(m - mn) + __expf(f - mn);
    m = mn;
  }
  // wave reduce of (m, s)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    lse_merge(m, s, m2, s2);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { sm[wid] = m; ss[wid] = s; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = sm[0], Ssum = ss[0];
    for (int i = 1; i < (int)(blockDim.x >> 6); ++i) lse_merge(M, Ssum, sm[i], ss[i]);
    const float lse = M + __logf(Ssum);
    lse_out[row] = lse;
    if (target == ignore_index || target < 0 || target >= V)
      loss[row] = 0.f;
    else
      loss[row] = lse - ld1<T>(x + target);
  }
}

// U chunks of 8 per thread per round, all U loads issued before the first
// store: one 16-B load in flight per thread (U = 1, the round-5 loop) left
// the sweep at 5.1 TB/s.  toa_xent_set_unroll picks U (A/B; bit-identical).
template <typename T, int U>
__global__ __launch_bounds__(512) void xent_bwd_kernel(const T* __restrict__ logits, const int64_t* __restrict__ tgt,
                                                       const float* __restrict__ lse_in,
                                                       const float* __restrict__ grad_out,
                                                       const float* __restrict__ n_valid, T* __restrict__ dx, int V,
                                                       int64_t ldx, int ignore_index) {
  const int64_t row = blockIdx.x;
  const T* x = logits + row * ldx;
  T* d = dx + row * ldx;
  const int64_t target = tgt[row];
  const bool ign = target == ignore_index || target < 0 || target >= V;
  const float scale = ign ? 0.f : grad_out[0] / fmaxf(n_valid[0], 1.f);
  const float lse = lse_in[row];
  const int v8 = (V % 8 == 0 && ldx % 8 == 0) ? V / 8 : 0;
  const int nb = blockDim.x;
  int i = threadIdx.x;
  for (; i + (U - 1) * nb < v8; i += U * nb) {
    float f[U][8];
#pragma unroll
    for (int u = 0; u < U; ++u) ld8<T>(x + (int64_t)(i + u * nb) * 8, f[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int c = i + u * nb;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float p = __expf(f[u][j] - lse);
        if (c * 8 + j == target) p -= 1.f;
        f[u][j] = p * scale;
      }
      st8<T>(d + (int64_t)c * 8, f[u]);
    }
  }
  for (; i < v8; i += nb) {
    float f[8];
    ld8<T>(x + (int64_t)i * 8, f);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float p = __expf(f[j] - lse);
      if (i * 8 + j == target) p -= 1.f;
      f[j] = p * scale;
    }
    st8<T>(d + (int64_t)i * 8, f);
  }
  for (int k = v8 * 8 + threadIdx.x; k < V; k += nb) {
    float p = __expf(ld1<T>(x + k) - lse);
    if (k == target) p -= 1.f;
    if (sizeof(T) == 2)
      ((bf16_t*)d)[k] = f2bf(p * scale);
    else
      ((float*)d)[k] = p * scale;
  }
}

static int g_xent_unroll = 2;   // measured: 2.493 (1) -> 2.323 (2) -> 2.404 ms (4) at 24576 x 128256 (profiles/r6_stream)
extern "C" int toa_xent_set_unroll(int u) {
  if (u != 1 && u != 2 && u != 4) return (int)hipErrorInvalidValue;
  g_xent_unroll = u;
  return 0;
}

extern "C" int toa_xent_fwd(int dtype, const void* logits, const int64_t* tgt, float* loss, float* lse, int64_t rows,
                            int V, int64_t ldx, int ignore_index, hipStream_t stream) {
  if (dtype == 0)
    hipLaunchKernelGGL(xent_fwd_kernel<bf16_t>, dim3(rows), dim3(512), 0, stream, (const bf16_t*)logits, tgt, loss,
                       lse, V, ldx, ignore_index);
  else
    hipLaunchKernelGGL(xent_fwd_kernel<float>, dim3(rows), dim3(512), 0, stream, (const float*)logits, tgt, loss, lse,
                       V, ldx, ignore_index);
  return (int)hipGetLastError();
}

extern "C" int toa_xent_bwd(int dtype, const void* logits, const int64_t* tgt, const float* lse,
                            const float* grad_out, const float* n_valid, void* dx, int64_t rows, int V, int64_t ldx,
                            int ignore_index, hipStream_t stream) {
  if (dtype == 0) {
    auto k = g_xent_unroll == 4 ? xent_bwd_kernel<bf16_t, 4>
                                : (g_xent_unroll == 2 ? xent_bwd_kernel<bf16_t, 2> : xent_bwd_kernel<bf16_t, 1>);
    hipLaunchKernelGGL(k, dim3(rows), dim3(512), 0, stream, (const bf16_t*)logits, tgt, lse, grad_out, n_valid,
                       (bf16_t*)dx, V, ldx, ignore_index);
  } else {
    hipLaunchKernelGGL((xent_bwd_kernel<float, 1>), dim3(rows), dim3(512), 0, stream, (const float*)logits, tgt, lse,
                       grad_out, n_valid, (float*)dx, V, ldx, ignore_index);
  }
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Embedding backward without float atomics: the token ids arrive sorted
// (stable sort, so equal ids keep their original order).  Workgroup i owns
// the run of equal ids starting at position i (every other workgroup exits
// at once), sums those rows of dy in fp32 in a fixed order and adds the sum
// into the gradient row once.  Deterministic, and the bf16 gradient gets one
// rounding per step instead of one per occurrence.
__global__ __launch_bounds__(256) void embed_bwd_kernel(const int64_t* __restrict__ sorted,
                                                       const int64_t* __restrict__ perm,
                                                       const bf16_t* __restrict__ dy, void* __restrict__ grad,
                                                       int grad_f32, int64_t n, int dim) {
  const int64_t i = blockIdx.x;
  const int64_t tok = sorted[i];
  if (i > 0 && sorted[i - 1] == tok) return;
  for (int c = threadIdx.x * 8; c < dim; c += 256 * 8) {
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    for (int64_t r = i; r < n && sorted[r] == tok; ++r) {
      float f[8];
      unpack8(ld16(dy + perm[r] * dim + c), f);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += f[j];
    }
    if (grad_f32) {
      float* g = (float*)grad + tok * dim + c;
      f32x4 a = *(f32x4*)g, b = *(f32x4*)(g + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        a[j] += acc[j];
        b[j] += acc[4 + j];
      }
      *(f32x4*)g = a;
      *(f32x4*)(g + 4) = b;
    } else {
      bf16_t* g = (bf16_t*)grad + tok * dim + c;
      float old[8];
      unpack8(ld16(g), old);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += old[j];
      st16(g, pack8(acc));
    }
  }
}

// sorted/perm: int64 [n] (torch.sort(stable=True) of the ids); dy bf16 [n, dim];
// grad bf16 or fp32 [vocab, dim]; dim % 8 == 0.
extern "C" int toa_embed_bwd(const int64_t* sorted, const int64_t* perm, const bf16_t* dy, void* grad, int grad_f32,
                             int64_t n, int dim, hipStream_t stream) {
  if (dim % 8 != 0 || n <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(embed_bwd_kernel, dim3((unsigned)n), dim3(256), 0, stream, sorted, perm, dy, grad, grad_f32, n,
                     dim);
  return (int)hipGetLastError();
}
