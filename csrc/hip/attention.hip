// Causal flash attention for gfx950 (bf16 in/out, fp32 accumulate), with
// native GQA (K/V stay packed per kv-head; no repeat_interleave copies).
//
// Layouts: q [B, H, S, D], o/dO [B, H, S, D] or [B, S, H, D] (flag bit 1),
// k/v [B, Hk, S, D], lse [B, H, S] (natural log), D = 64 or 128 (template;
// LDS rows of 2D bytes = D/8 16-byte chunks), any S >= 1.  Forward / dQ:
// one workgroup = 8 waves = a 256-row query block of one (batch, head);
// wave w owns 32 query rows.  K/V tiles of 64 keys are staged
// global -> registers -> LDS (double buffered, loads of tile t+1 in flight
// while tile t is computed -- guide T14), K in a 16-way XOR-swizzled
// row-major image read with ds_read_b128 (conflict-free for the 32x32 MFMA
// operand pattern, guide T2), V row-major with a 4-row XOR swizzle read by
// ds_read_b64_tr_b16 (hardware transpose for the PV operand, guide T10).
//
// MFMA orientation (guide §3 "accumulator tile as next operand"):
//   S^T[key][q] = K . Q^T      v_mfma_f32_32x32x16_bf16, A = K frag, B = Q frag
//   -> each lane owns ONE query row (column q = lane&31) and 16 of the 64 key
//      scores (its partner lane l^32 owns the other 16 of each 32-key half), so
//      the online softmax row max/sum is lane-local + one cross-half shuffle;
//   O^T[d][q] += V^T . P^T     the S^T accumulator registers, converted to
//      bf16, ARE the B operand (k permutation handled by the V^T read order).
// Softmax in the exp2 domain with the scale folded in; causal tiles beyond a
// wave's last row are skipped wave-uniformly; blocks are launched
// heaviest-first for load balance.
//
// Backward (S % 256 == 0, default): a delta pass, dK/dV (workgroup per
// 128-key block, sweeping the GQA group's query heads) which also stores dS,
// and dQ as a GEMM over the stored dS; otherwise two kernels: dQ (which also
// computes delta = rowsum(dO*O)), then dK/dV.  No float atomics:
// deterministic.
//
// Ragged S (S % 64 != 0): every row index that feeds a LOAD is clamped to
// S - 1, so tiles past the end re-read the last row instead of branching
// around loads (a per-load select makes hipcc wait vmcnt(0) per element).
// That is exact for causal attention: a padded key sits after every real
// query (the diagonal mask removes it), a padded query's outputs are never
// stored, and in dK/dV a padded query row gets lse = +inf, i.e. p = 0.
#include <cstdlib>
#include <cstring>

#include "toa_common.h"

typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(4))) short bf16x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;

#define LOG2E 1.4426950408889634f
#define EXP2(x) __builtin_amdgcn_exp2f(x)
#define RESCALE_THR 8.0f  // guide T13: defer the O rescale while the row max grows < 2^8

__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x8 as_bf16x8(u32x4 v) { return __builtin_bit_cast(bf16x8, v); }

// LDS tile geometry: 64 keys x D bf16, rows of ROWB = 2D bytes = NCH chunks
// of 16 B (D = 128: 256-B rows, 16 chunks; D = 64: 128-B rows, 8 chunks).
#define TK 64
template <int D>
struct AG {
  static constexpr int NCH = D / 8;     // 16-B chunks per row
  static constexpr int ROWB = 2 * D;    // bytes per row
  static constexpr int NS = D / 16;     // k-steps of a 32x32x16 MFMA over d
  static constexpr int ND = D / 32;     // 32-row d tiles of an O^T / dK^T accumulator
  static constexpr int TILEB = TK * ROWB;
};

// K image: chunk c of row `key` stored at chunk position c ^ (key & (NCH-1))
template <int D>
__device__ __forceinline__ int k_off(int key, int chunk) {
  return key * AG<D>::ROWB + ((chunk ^ (key & (AG<D>::NCH - 1))) << 4);
}
// V image (read transposed): chunk c of row `key` at c ^ ((key & 3) << 2) (D = 128) / << 1 (D = 64)
template <int D>
__device__ __forceinline__ int v_off(int key, int chunk) {
  return key * AG<D>::ROWB + ((chunk ^ ((key & 3) << (D == 128 ? 2 : 1))) << 4);
}

// LDS-DMA through the buffer path (MUBUF `buffer_load ... lds`) instead of
// global_load_lds: hipcc's wait-count pass counts a pending FLAT-encoded
// LDS-DMA against both the VM and the LGKM counters and then waits
// lgkmcnt(0) before every LDS read that follows it; with the MUBUF form the
// reads keep counted lgkmcnt(N) waits, so fragments can be read ahead of the
// MFMAs that use them.  base: the tensor slice the offsets are relative to.
// (__device__ helpers, not macros in the kernel bodies: the host pass of a
// kernel template that names these builtins drops the kernel's launch stub)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ void buf_dma16(__amdgpu_buffer_rsrc_t r, uint32_t voff, void* lds, int aux = 0) {
  if (aux)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, 0, 0, 2);
  else
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, 0, 0, 0);
}
__device__ __forceinline__ void buf_dma4(__amdgpu_buffer_rsrc_t r, uint32_t voff, void* lds) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 4, voff, 0, 0, 0);
}
#define BUF_DMA(BYTES, rsrc, voff, lds) buf_dma##BYTES((rsrc), (voff), (lds))

// the shader clock after the wave's outstanding LDS / scalar reads retire
__device__ __forceinline__ unsigned long long memtime_sync() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

// an empty asm on a value: hipcc must assume it changed here, so work
// derived from it is not hoisted above this point (a __device__ helper: the
// host pass never sees the VGPR constraint)
__device__ __forceinline__ void opaque_v(int& x) { asm volatile("" : "+v"(x)); }

typedef short __attribute__((ext_vector_type(4))) s16x4;
__device__ __forceinline__ bf16x4 tr_read(const char* lds_base, int byte_off) {
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  lds_s16x4* p = (lds_s16x4*)(lds_base + byte_off);
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(p);
}

// ---------------------------------------------------------------------------
// forward: workgroup = 8 waves = a 256-row query block of one (batch, head);
// wave w owns rows 32w..32w+31, two waves per SIMD.  One 64-key K/V tile in
// LDS feeds all 8 waves (half the L2->LDS traffic of two 4-wave blocks).
// ---------------------------------------------------------------------------
#define FWD_QB 256
#define FWD_WAVES 8

__device__ __forceinline__ uint32_t cvt_pk(float a, float b) { return pack2(a, b); }

// combine a value with the partner lane's (l ^ 32) by v_permlane32_swap
// (vdst's upper half <-> vsrc's lower half; with both = v, lane l < 32 ends
// with {v[l], v[l+32]} and lane l >= 32 with {v[l-32], v[l]}).  Inline asm:
// the builtin with identical operands gets folded to a single result.
__device__ __forceinline__ void xhalf_pair(float v, float& a, float& b) {
  a = v;
  b = v;
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
}
__device__ __forceinline__ float xhalf_max(float v) {
  float a, b;
  xhalf_pair(v, a, b);
  return fmaxf(a, b);
}
__device__ __forceinline__ float xhalf_sum(float v) {
  float a, b;
  xhalf_pair(v, a, b);
  return a + b;
}

// Softmax VALU trimmed to what the MFMA gaps can hide (guide §5.5 T12 and
// MI355X_MICROARCH 'vector-instruction ISSUE cost': at two waves per SIMD the
// issue port, not the MFMA pipe, bounded these kernels):
//  * row max as two independent v_max3_f32 chains;
//  * scale-and-subtract and the row sum on PAIRS of scores with
//    v_pk_fma_f32 / v_pk_add_f32 (consecutive accumulator registers).
typedef __attribute__((ext_vector_type(2))) float f32x2;
// max over the 32 scores of sc[0], sc[1] (one lane's row half): two
// independent chains the compiler turns into v_max3_f32
__device__ __forceinline__ float rowmax32(const f32x16& a, const f32x16& b) {
  float m0 = fmaxf(a[0], a[1]), m1 = fmaxf(b[0], b[1]);
#pragma unroll
  for (int j = 2; j < 16; ++j) {
    m0 = fmaxf(m0, a[j]);
    m1 = fmaxf(m1, b[j]);
  }
  return fmaxf(m0, m1);
}
__device__ __forceinline__ f32x2 pk_fma(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }

#ifndef ATTN_WIDE_STORE
#define ATTN_WIDE_STORE 1
#endif
// Epilogue store of one 32x32 accumulator tile's row (guide T21): lane l and
// l^32 own the same row; `a` / `b` are this lane's packed bf16x4 of column
// groups 2k and 2k+1 (cols 16k + 8*g' + 4*hh).  One v_permlane32_swap per
// dword leaves lanes < 32 with cols 16k..16k+7 and lanes >= 32 with
// 16k+8..16k+15: one 16-B store per lane instead of two 8-B ones.
__device__ __forceinline__ void store_pair16(bf16_t* row, int col16k, int hh, uint2 a, uint2 b) {
#if ATTN_WIDE_STORE
  const auto r0 = __builtin_amdgcn_permlane32_swap(a.x, b.x, false, false);
  const auto r1 = __builtin_amdgcn_permlane32_swap(a.y, b.y, false, false);
  *(uint4*)(row + col16k + 8 * hh) = make_uint4(r0[0], r1[0], r0[1], r1[1]);
#else
  *(uint2*)(row + col16k + 4 * hh) = a;
  *(uint2*)(row + col16k + 8 + 4 * hh) = b;
#endif
}

// Offset of row (b, h, s) of O / dO: [B, H, S, D] (head-major, like Q) or, with
// bshd, [B, S, H, D] -- the layout the output projection consumes, so the
// model needs no transpose copy of O forward or of dO backward.
template <int D>
__device__ __forceinline__ int64_t o_off(int b, int h, int s, int H, int S, int bshd) {
  return bshd ? (((int64_t)b * S + s) * H + h) * D : (((int64_t)b * H + h) * S + s) * D;
}

// XCD-aware block order: the hardware deals workgroups to the 8 XCDs round
// robin, so give every XCD whole (batch, kv-head) groups -- their K/V stay
// in that XCD's L2 across the GQA heads and query blocks -- and walk each
// XCD's share heaviest (most keys) first.
__device__ __forceinline__ void fwd_block_coords(int pid, int nqb, int B, int H, int Hk, int* qb, int* h, int* b) {
  const int rep = H / Hk, G = B * Hk;
  if ((G & 7) == 0) {
    const int xcd = pid & 7, slot = pid >> 3, gper = G >> 3;
    const int per_rank = gper * rep;
    const int rank = slot / per_rank, w = slot - rank * per_rank;
    const int gi = w / rep, hr = w - gi * rep;
    const int grp = xcd * gper + gi;
    *b = grp / Hk;
    *h = (grp - *b * Hk) * rep + hr;
    *qb = nqb - 1 - rank;
  } else {
    const int per = H * B, rank = pid / per, w = pid - rank * per;
    *qb = nqb - 1 - rank;
    *h = w % H;
    *b = w / H;
  }
}

template <int D, bool TAIL>
__global__ __launch_bounds__(512, 1) void attn_fwd_kernel(const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K,
                                                          const bf16_t* __restrict__ V, bf16_t* __restrict__ O,
                                                          float* __restrict__ LSE, int B, int H, int Hk, int S,
                                                          float scale_log2, int o_bshd) {
  using G = AG<D>;
  constexpr int ROWB = G::ROWB, NCH = G::NCH, NS = G::NS, ND = G::ND, TILEB = G::TILEB;
  constexpr int NL = TK * NCH / 512;  // 16-B chunks of K (and of V) per thread per tile
  extern __shared__ __attribute__((aligned(16))) char smem[];  // 2 x (K tile + V tile)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int nqb = (S + FWD_QB - 1) / FWD_QB;
  int qb, h, b;
  fwd_block_coords(blockIdx.x, nqb, B, H, Hk, &qb, &h, &b);
  const int hk = h / (H / Hk);
  const int64_t qoff = ((int64_t)(b * H + h) * S) * D;
  const int64_t koff = ((int64_t)(b * Hk + hk) * S) * D;
  const int q0 = qb * FWD_QB + wave * 32;  // first row of this wave
  const bool live = q0 < S;                // wave has at least one real row
  const int myq = q0 + r;                  // the query row this lane owns (>= S: padding)
  const int myq_ld = TAIL ? min(myq, S - 1) : myq;
  const int kend = min(S, (qb + 1) * FWD_QB);
  const int ntiles = (kend + TK - 1) / TK;
  const int t_diag = live ? (q0 + 31) / TK : -1;  // this wave's last (masked) tile

  // Q fragments: Q[myq][16s + 8hh .. +7], s = 0..NS-1
  bf16x8 qf[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s)
    qf[s] = live ? as_bf16x8(ld16(Q + qoff + (int64_t)myq_ld * D + 16 * s + 8 * hh)) : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};

  // lane-constant LDS read offsets (buffer / half / k-step parts are immediates)
  int kro[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) kro[s] = k_off<D>(r, 2 * s + hh);
  // V^T: key = 32n + 16s' + 4hh + qq (+8), column block 32dt + 16(g&1) + 4pp
  int vro[ND];
  {
    const int g = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) vro[dt] = v_off<D>(4 * hh + qq, 4 * dt + 2 * (g & 1) + (pp >> 1)) + (pp & 1) * 8;
  }

  f32x16 acc[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i)
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[i][j] = 0.f;
  float m_run = -INFINITY, l_run = 0.f;

  // staging: 512 threads x NL x (16 B of K + 16 B of V) = one 64-key tile
  u32x4 stk[NL], stv[NL];
  auto gload = [&](int t) {
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int e = tid + 512 * i;
      const int key = e / NCH, c = e % NCH;
      const int64_t gidx = koff + (int64_t)(TAIL ? min(t * TK + key, S - 1) : t * TK + key) * D + c * 8;
      stk[i] = ld16(K + gidx);
      stv[i] = ld16(V + gidx);
    }
  };
  auto swrite = [&](int buf) {
    char* kb = smem + buf * 2 * TILEB;
    char* vb = kb + TILEB;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int e = tid + 512 * i;
      const int key = e / NCH, c = e % NCH;
      *(u32x4*)(kb + k_off<D>(key, c)) = stk[i];
      *(u32x4*)(vb + v_off<D>(key, c)) = stv[i];
    }
  };

  auto compute = [&](int t, int buf, bool mask) {
    const char* kb = smem + buf * 2 * TILEB;
    const char* vb = kb + TILEB;
    // ---- S^T = K Q^T : two 32-key halves (first MFMA of each chain starts from 0)
    f32x16 sc[2];
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const f32x16 z = {};
      sc[n] = mfma32(as_bf16x8(*(const u32x4*)(kb + kro[0] + 32 * ROWB * n)), qf[0], z);
#pragma unroll
      for (int s = 1; s < NS; ++s)
        sc[n] = mfma32(as_bf16x8(*(const u32x4*)(kb + kro[s] + 32 * ROWB * n)), qf[s], sc[n]);
    }
    // ---- causal mask (diagonal tile only) and row max of the raw scores
    if (mask) {
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const int key = t * TK + 32 * n + (j & 3) + 8 * (j >> 2) + 4 * hh;
          if (key > myq) sc[n][j] = -INFINITY;
        }
    }
    float mx = rowmax32(sc[0], sc[1]);
    mx = xhalf_max(mx) * scale_log2;
    // T13: rescale O / l only when some row's max grew by more than THR
    if (__any(mx > m_run + RESCALE_THR)) {
      const float m_new = fmaxf(m_run, mx);
      const float alpha = (m_run == -INFINITY) ? 0.f : EXP2(m_run - m_new);
      l_run *= alpha;
      m_run = m_new;
#pragma unroll
      for (int i = 0; i < ND; ++i)
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[i][j] *= alpha;
    }
    // ---- P = exp2(s*c - m) packed straight into the PV B operand
    f32x2 ls;
    const f32x2 c2 = {scale_log2, scale_log2}, nm2 = {-m_run, -m_run};
    uint32_t pw[2][8];
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int j = 0; j < 16; j += 2) {
        f32x2 x = pk_fma(f32x2{sc[n][j], sc[n][j + 1]}, c2, nm2);
        x[0] = EXP2(x[0]);
        x[1] = EXP2(x[1]);
        ls = (n == 0 && j == 0) ? x : ls + x;
        pw[n][j >> 1] = cvt_pk(x[0], x[1]);
      }
    l_run += ls[0] + ls[1];
    // ---- O^T += V^T P^T (k permutation of the accumulator handled by the V^T read order)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        u32x4 w;
        w[0] = pw[n][4 * s + 0];
        w[1] = pw[n][4 * s + 1];
        w[2] = pw[n][4 * s + 2];
        w[3] = pw[n][4 * s + 3];
        const bf16x8 pf = as_bf16x8(w);
        const int kb0 = (32 * n + 16 * s) * ROWB;
#pragma unroll
        for (int dt = 0; dt < ND; ++dt) {
          const bf16x4 va = tr_read(vb, vro[dt] + kb0);
          const bf16x4 vbv = tr_read(vb, vro[dt] + kb0 + 8 * ROWB);
          const bf16x8 vf = __builtin_shufflevector(va, vbv, 0, 1, 2, 3, 4, 5, 6, 7);
          acc[dt] = mfma32(vf, pf, acc[dt]);
        }
      }
  };
  auto step = [&](int t, int buf) {
    if (t + 1 < ntiles) gload(t + 1);
    if (t < t_diag) compute(t, buf, false);
    else if (t == t_diag) compute(t, buf, true);
    if (t + 1 < ntiles) swrite(buf ^ 1);
    __syncthreads();
  };

  gload(0);
  swrite(0);
  // Retire the Q loads HERE.  Left to itself the compiler sinks them past the
  // barrier; the loop then inherits "Q pending" and, vmcnt being in-order,
  // its first MFMA waits on the K/V prefetch of the same iteration.
#pragma unroll
  for (int s = 0; s < NS; ++s) asm volatile("" ::"v"(qf[s]));
  __syncthreads();
  int t = 0;
  for (; t + 1 < ntiles; t += 2) {  // unrolled by 2: buffer offsets become immediates
    step(t, 0);
    step(t + 1, 1);
  }
  if (t < ntiles) step(t, 0);

  if (!live || (TAIL && myq >= S)) return;
  // ---- epilogue: O = O^T / l  (lane owns query row myq; d rows from the C map)
  const float l_tot = xhalf_sum(l_run);
  const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
  bf16_t* orow = O + o_off<D>(b, h, myq, H, S, o_bshd);
#pragma unroll
  for (int dt = 0; dt < ND; ++dt)
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      uint2 w[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int g = 2 * k + u;
        w[u].x = cvt_pk(acc[dt][4 * g + 0] * inv, acc[dt][4 * g + 1] * inv);
        w[u].y = cvt_pk(acc[dt][4 * g + 2] * inv, acc[dt][4 * g + 3] * inv);
      }
      store_pair16(orow, 32 * dt + 16 * k, hh, w[0], w[1]);
    }
  if (hh == 0) LSE[(int64_t)(b * H + h) * S + myq] = (m_run + log2f(l_tot)) * 0.6931471805599453f;
}

// Forward with LDS-DMA staging (S % 256 == 0; the default): the same
// body as attn_fwd_kernel, the K / V tiles brought in by global_load_lds
// into two distinct LDS objects instead of register staging + ds_write
// (the change that took the dK/dV kernel from 2.19 to 1.97 ms).
template <int D>
__global__ __launch_bounds__(512, 1) void attn_fwd_gl_kernel(const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K,
                                                          const bf16_t* __restrict__ V, bf16_t* __restrict__ O,
                                                          float* __restrict__ LSE, int B, int H, int Hk, int S,
                                                          float scale_log2, int o_bshd) {
  using G = AG<D>;
  constexpr int ROWB = G::ROWB, NCH = G::NCH, NS = G::NS, ND = G::ND, TILEB = G::TILEB;
  constexpr bool TAIL = false;
  // two (K tile + V tile) buffers, distinct LDS objects (a read of one then
  // never waits on the LDS-DMA filling the other)
  __shared__ __attribute__((aligned(1024))) char kv0[2 * TILEB];
  __shared__ __attribute__((aligned(1024))) char kv1[2 * TILEB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int nqb = (S + FWD_QB - 1) / FWD_QB;
  int qb, h, b;
  fwd_block_coords(blockIdx.x, nqb, B, H, Hk, &qb, &h, &b);
  const int hk = h / (H / Hk);
  const int64_t qoff = ((int64_t)(b * H + h) * S) * D;
  const int64_t koff = ((int64_t)(b * Hk + hk) * S) * D;
  const int q0 = qb * FWD_QB + wave * 32;  // first row of this wave
  const bool live = q0 < S;                // wave has at least one real row
  const int myq = q0 + r;                  // the query row this lane owns (>= S: padding)
  const int myq_ld = TAIL ? min(myq, S - 1) : myq;
  const int kend = min(S, (qb + 1) * FWD_QB);
  const int ntiles = (kend + TK - 1) / TK;
  const int t_diag = live ? (q0 + 31) / TK : -1;  // this wave's last (masked) tile

  // Q fragments: Q[myq][16s + 8hh .. +7], s = 0..NS-1
  bf16x8 qf[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s)
    qf[s] = live ? as_bf16x8(ld16(Q + qoff + (int64_t)myq_ld * D + 16 * s + 8 * hh)) : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};

  // lane-constant LDS read offsets (buffer / half / k-step parts are immediates)
  int kro[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) kro[s] = k_off<D>(r, 2 * s + hh);
  // V^T: key = 32n + 16s' + 4hh + qq (+8), column block 32dt + 16(g&1) + 4pp
  int vro[ND];
  {
    const int g = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) vro[dt] = v_off<D>(4 * hh + qq, 4 * dt + 2 * (g & 1) + (pp >> 1)) + (pp & 1) * 8;
  }

  f32x16 acc[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i)
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[i][j] = 0.f;
  float m_run = -INFINITY, l_run = 0.f;

  // K / V tiles by LDS-DMA: 1-KB piece pt of a tile covers keys RPP pt ..
  // + RPP - 1; waves 0-3 fetch K, 4-7 V, PW pieces each; the lane's 16 B land
  // at chunk position lane % NCH of key RPP pt + lane / NCH, so it loads the
  // chunk the k_off / v_off image keeps there
  constexpr int RPP = 1024 / ROWB, PW = TILEB / 1024 / 4;
  const int lkey = lane / NCH, lpos = lane % NCH;
  const int kcol = (lpos ^ (lkey & (NCH - 1))) << 3;  // k_off at D = 64; at 128 XOR (4 (pt & 3)) << 3 per piece
  const int vcol = (lpos ^ ((lkey & 3) << (D == 128 ? 2 : 1))) << 3;
  auto stage = [&](int t, int buf) {
    char* st = buf ? kv1 : kv0;
    const bf16_t* base = (wave < 4 ? K : V) + koff + (int64_t)t * TK * D;
    if (wave < 4) {
#pragma unroll
      for (int u = 0; u < PW; ++u) {
        const int pt = PW * wave + u;
        const int col = D == 128 ? kcol ^ ((4 * (pt & 3)) << 3) : kcol;
        __builtin_amdgcn_global_load_lds(
            (const __attribute__((address_space(1))) void*)(base + (uint32_t)((RPP * pt + lkey) * D + col)),
            (__attribute__((address_space(3))) void*)(st + pt * 1024), 16, 0, 0);
      }
    } else {
#pragma unroll
      for (int u = 0; u < PW; ++u) {
        const int pt = PW * (wave - 4) + u;
        __builtin_amdgcn_global_load_lds(
            (const __attribute__((address_space(1))) void*)(base + (uint32_t)((RPP * pt + lkey) * D + vcol)),
            (__attribute__((address_space(3))) void*)(st + TILEB + pt * 1024), 16, 0, 0);
      }
    }
  };

  auto compute = [&](int t, int buf, bool mask) {
    const char* kb = buf ? kv1 : kv0;
    const char* vb = kb + TILEB;
    // ---- S^T = K Q^T : two 32-key halves (first MFMA of each chain starts from 0)
    f32x16 sc[2];
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const f32x16 z = {};
      sc[n] = mfma32(as_bf16x8(*(const u32x4*)(kb + kro[0] + 32 * ROWB * n)), qf[0], z);
#pragma unroll
      for (int s = 1; s < NS; ++s)
        sc[n] = mfma32(as_bf16x8(*(const u32x4*)(kb + kro[s] + 32 * ROWB * n)), qf[s], sc[n]);
    }
    // ---- causal mask (diagonal tile only) and row max of the raw scores
    if (mask) {
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const int key = t * TK + 32 * n + (j & 3) + 8 * (j >> 2) + 4 * hh;
          if (key > myq) sc[n][j] = -INFINITY;
        }
    }
    float mx = rowmax32(sc[0], sc[1]);
    mx = xhalf_max(mx) * scale_log2;
    // T13: rescale O / l only when some row's max grew by more than THR
    if (__any(mx > m_run + RESCALE_THR)) {
      const float m_new = fmaxf(m_run, mx);
      const float alpha = (m_run == -INFINITY) ? 0.f : EXP2(m_run - m_new);
      l_run *= alpha;
      m_run = m_new;
#pragma unroll
      for (int i = 0; i < ND; ++i)
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[i][j] *= alpha;
    }
    // ---- P = exp2(s*c - m) packed straight into the PV B operand
    f32x2 ls;
    const f32x2 c2 = {scale_log2, scale_log2}, nm2 = {-m_run, -m_run};
    uint32_t pw[2][8];
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int j = 0; j < 16; j += 2) {
        f32x2 x = pk_fma(f32x2{sc[n][j], sc[n][j + 1]}, c2, nm2);
        x[0] = EXP2(x[0]);
        x[1] = EXP2(x[1]);
        ls = (n == 0 && j == 0) ? x : ls + x;
        pw[n][j >> 1] = cvt_pk(x[0], x[1]);
      }
    l_run += ls[0] + ls[1];
    // ---- O^T += V^T P^T (k permutation of the accumulator handled by the V^T read order)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        u32x4 w;
        w[0] = pw[n][4 * s + 0];
        w[1] = pw[n][4 * s + 1];
        w[2] = pw[n][4 * s + 2];
        w[3] = pw[n][4 * s + 3];
        const bf16x8 pf = as_bf16x8(w);
        const int kb0 = (32 * n + 16 * s) * ROWB;
#pragma unroll
        for (int dt = 0; dt < ND; ++dt) {
          const bf16x4 va = tr_read(vb, vro[dt] + kb0);
          const bf16x4 vbv = tr_read(vb, vro[dt] + kb0 + 8 * ROWB);
          const bf16x8 vf = __builtin_shufflevector(va, vbv, 0, 1, 2, 3, 4, 5, 6, 7);
          acc[dt] = mfma32(vf, pf, acc[dt]);
        }
      }
  };
  auto step = [&](int t, int buf) {
    if (t + 1 < ntiles) stage(t + 1, buf ^ 1);
    if (t < t_diag) compute(t, buf, false);
    else if (t == t_diag) compute(t, buf, true);
    // my DMA retired, then everyone's (the next step reads buf ^ 1 and restages buf)
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  };

  stage(0, 0);
  // Q loads and the first tile's DMA retired before the loop
#pragma unroll
  for (int s = 0; s < NS; ++s) asm volatile("" ::"v"(qf[s]));
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  int t = 0;
  for (; t + 1 < ntiles; t += 2) {  // unrolled by 2: buffer offsets become immediates
    step(t, 0);
    step(t + 1, 1);
  }
  if (t < ntiles) step(t, 0);

  if (!live) return;
  // ---- epilogue: O = O^T / l  (lane owns query row myq; d rows from the C map)
  const float l_tot = xhalf_sum(l_run);
  const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
  bf16_t* orow = O + o_off<D>(b, h, myq, H, S, o_bshd);
#pragma unroll
  for (int dt = 0; dt < ND; ++dt)
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      uint2 w[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int g = 2 * k + u;
        w[u].x = cvt_pk(acc[dt][4 * g + 0] * inv, acc[dt][4 * g + 1] * inv);
        w[u].y = cvt_pk(acc[dt][4 * g + 2] * inv, acc[dt][4 * g + 3] * inv);
      }
      store_pair16(orow, 32 * dt + 16 * k, hh, w[0], w[1]);
    }
  if (hh == 0) LSE[(int64_t)(b * H + h) * S + myq] = (m_run + log2f(l_tot)) * 0.6931471805599453f;
}


// One image for row reads (ds_read_b128, 32x32x16 A/B operand) AND
// transposed reads (ds_read_b64_tr_b16): guide T10 layout (b),
// D = 128: chunk' = chunk ^ (((row & 3) << 2) | ((row >> 2) & 3));
// D = 64 (8 chunks): chunk' = chunk ^ (((row & 3) << 1) | ((row >> 2) & 1)).
// The XOR depends on row & 15 only, so offsets of rows 16k apart differ by
// exactly 16k rows (the row-block parts of every read are immediates).
template <int D>
__device__ __forceinline__ int rt_off(int row, int chunk) {
  const int swz = D == 128 ? (((row & 3) << 2) | ((row >> 2) & 3)) : (((row & 3) << 1) | ((row >> 2) & 1));
  return row * AG<D>::ROWB + ((chunk ^ swz) << 4);
}

// ---------------------------------------------------------------------------
// dK / dV: workgroup = 8 waves = 128 keys of one (batch, kv head).  Wave w
// owns keys 32(w&3)..+31 of the block (key on the MFMA lane) and query half
// m = w>>2 of every 64-row query tile, so two waves accumulate partial dK^T /
// dV^T for the same keys over disjoint query rows; they are summed through
// LDS at the end.  K/V of the block live in LDS (not registers): the
// accumulators (128) + one sub-tile's working set fit 256 VGPRs, i.e. two
// waves per SIMD, which is what hides the LDS and softmax latency.
//   S = Q K^T, dP = dO V^T - delta   (A = Q / dO row reads, B = K / V row reads)
//   dV^T += dO^T P, dK^T += Q^T dS   (A = transposed reads, B = the accumulators)
// The block sweeps every query head of the GQA group and every causal tile.
// ---------------------------------------------------------------------------
template <int D>
struct DKV {
  static constexpr int QBUF = 2 * TK * AG<D>::ROWB + 512;  // Q tile, dO tile, lse, -delta
  static constexpr int KVB = 128 * AG<D>::ROWB;             // K (or V) of the 128-key block
  static constexpr int LDS = 2 * QBUF + 2 * KVB;
};

template <int D, bool TAIL>
__global__ __launch_bounds__(512, 1) void attn_bwd_dkdv_kernel(
    const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V,
    const bf16_t* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ DELTA,
    bf16_t* __restrict__ dK, bf16_t* __restrict__ dV, int B, int H, int Hk, int S, float scale,
    float scale_log2, int o_bshd) {
  using G = AG<D>;
  constexpr int ROWB = G::ROWB, NCH = G::NCH, NS = G::NS, ND = G::ND, TILEB = G::TILEB;
  constexpr int QBUF = DKV<D>::QBUF, KVB = DKV<D>::KVB;
  constexpr int NLQ = TK * NCH / 512, NLK = 128 * NCH / 512;
  // [Q/dO/lse/-delta buffer 0][buffer 1][K][V]
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* kimg = smem + 2 * QBUF;
  char* vimg = kimg + KVB;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int kg = wave & 3, m = wave >> 2;
  // (b, hk) fastest
  // heaviest first: key block kb sees S / 64 - 2 kb query tiles, so kb = 0
  // leads (largest-first keeps the last wave of workgroups short: a
  // simulated 800 vs 912 tile-units makespan at the bench shape)
  const int kb = (int)(blockIdx.x / (B * Hk));
  const int bh = blockIdx.x % (B * Hk);
  const int b = bh / Hk, hk = bh % Hk;
  const int rep = H / Hk;
  const int kw = kb * 128 + kg * 32;  // first key of this wave
  const int mykey = kw + r;
  const int64_t koff = ((int64_t)(b * Hk + hk) * S) * D;

  // K / V of the block -> LDS (rt_off image: row reads give the B operands)
#pragma unroll
  for (int i = 0; i < NLK; ++i) {
    const int e = tid + 512 * i;
    const int row = e / NCH, c = e % NCH;
    const int64_t g = koff + (int64_t)(TAIL ? min(kb * 128 + row, S - 1) : kb * 128 + row) * D + c * 8;
    *(u32x4*)(kimg + rt_off<D>(row, c)) = ld16(K + g);
    *(u32x4*)(vimg + rt_off<D>(row, c)) = ld16(V + g);
  }
  f32x16 dk[ND], dv[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i)
#pragma unroll
    for (int j = 0; j < 16; ++j) { dk[i][j] = 0.f; dv[i][j] = 0.f; }

  int rro[NS], tro[ND], tro8[ND];
  {
#pragma unroll
    for (int s = 0; s < NS; ++s) rro[s] = rt_off<D>(r, 2 * s + hh);
    const int g = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) {
      const int c = 4 * dt + 2 * (g & 1) + (pp >> 1);
      tro[dt] = rt_off<D>(4 * hh + qq, c) + (pp & 1) * 8;
      tro8[dt] = rt_off<D>(4 * hh + qq + 8, c) + (pp & 1) * 8;
    }
  }

  const int qt0 = (kb * 128) / 64;  // first causal 64-row query tile
  const int nqt = (S + TK - 1) / TK - qt0;
  const int total = nqt * rep;
  u32x4 sq[NLQ], sdo[NLQ];
  float slse = 0.f, sdel = 0.f;
  auto gload = [&](int it) {
    const int hq = hk * rep + it / nqt;
    const int qt = qt0 + it % nqt;
    const int64_t qoff = ((int64_t)(b * H + hq) * S) * D;
#pragma unroll
    for (int i = 0; i < NLQ; ++i) {
      const int e = tid + 512 * i;
      const int row = e / NCH, c = e % NCH;
      const int qr = TAIL ? min(qt * 64 + row, S - 1) : qt * 64 + row;
      sq[i] = ld16(Q + qoff + (int64_t)qr * D + c * 8);
      sdo[i] = ld16(dO + o_off<D>(b, hq, qr, H, S, o_bshd) + c * 8);
    }
    if (tid < 64) {
      const int q = qt * 64 + tid;
      const int64_t li = (int64_t)(b * H + hq) * S + (TAIL ? min(q, S - 1) : q);
      const float x = LSE[li];  // scaled at swrite: consuming it here would wait on the whole prefetch
      slse = (!TAIL || q < S) ? x : INFINITY;  // padded query row: p = exp2(. - inf) = 0
      sdel = DELTA[li];
    }
  };
  auto swrite = [&](int buf) {
    char* qb_ = smem + buf * QBUF;
    char* ob = qb_ + TILEB;
    float* lb = (float*)(qb_ + 2 * TILEB);
#pragma unroll
    for (int i = 0; i < NLQ; ++i) {
      const int e = tid + 512 * i;
      const int row = e / NCH, c = e % NCH;
      *(u32x4*)(qb_ + rt_off<D>(row, c)) = sq[i];
      *(u32x4*)(ob + rt_off<D>(row, c)) = sdo[i];
    }
    if (tid < 64) {
      lb[tid] = -(slse * LOG2E);  // the exp2 argument's addend (pk_fma); padded rows: -inf -> p = 0
      lb[64 + tid] = -sdel;
    }
  };

  auto subtile = [&](int buf, int qs, bool mask) {
    const char* qi = smem + buf * QBUF;
    const char* oi = qi + TILEB;
    const float* lb = (const float*)(qi + 2 * TILEB);
    f32x16 nd;
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const f32x4 d4 = *(const f32x4*)(lb + 64 + 32 * m + 8 * g4 + 4 * hh);
#pragma unroll
      for (int j = 0; j < 4; ++j) nd[4 * g4 + j] = d4[j];
    }
    const f32x16 z = {};
    f32x16 sc = z, dp = nd;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const bf16x8 qa = as_bf16x8(*(const u32x4*)(qi + rro[s] + 32 * ROWB * m));
      const bf16x8 kf = as_bf16x8(*(const u32x4*)(kimg + rro[s] + 32 * ROWB * kg));
      sc = mfma32(qa, kf, sc);
      const bf16x8 oa = as_bf16x8(*(const u32x4*)(oi + rro[s] + 32 * ROWB * m));
      const bf16x8 vf = as_bf16x8(*(const u32x4*)(vimg + rro[s] + 32 * ROWB * kg));
      dp = mfma32(oa, vf, dp);
    }
    // (scalar VALU here: the packed forms need aligned register pairs, and at
    // 256 VGPRs with resident dK^T / dV^T accumulators that spills in the loop)
    uint32_t pw[8], sw[8];
#pragma unroll
    for (int j = 0; j < 16; j += 2) {
      const f32x4 l4 = *(const f32x4*)(lb + 32 * m + 8 * (j >> 2) + 4 * hh);  // -lse * log2(e)
      float p0 = EXP2(fmaf(sc[j], scale_log2, l4[j & 3]));
      float p1 = EXP2(fmaf(sc[j + 1], scale_log2, l4[(j + 1) & 3]));
      if (mask) {
        const int q = qs + (j & 3) + 8 * (j >> 2) + 4 * hh;
        if (q < mykey) p0 = 0.f;
        if (q + 1 < mykey) p1 = 0.f;
      }
      pw[j >> 1] = pack2(p0, p1);
      sw[j >> 1] = pack2(p0 * dp[j], p1 * dp[j + 1]);
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      u32x4 a, c;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        a[i] = pw[4 * s2 + i];
        c[i] = sw[4 * s2 + i];
      }
      const bf16x8 pb = as_bf16x8(a), sb = as_bf16x8(c);
      const int rb = (32 * m + 16 * s2) * ROWB;
#pragma unroll
      for (int dt = 0; dt < ND; ++dt) {
        const bf16x4 o0 = tr_read(oi, tro[dt] + rb), o1 = tr_read(oi, tro8[dt] + rb);
        dv[dt] = mfma32((bf16x8)__builtin_shufflevector(o0, o1, 0, 1, 2, 3, 4, 5, 6, 7), pb, dv[dt]);
        const bf16x4 q0 = tr_read(qi, tro[dt] + rb), q1 = tr_read(qi, tro8[dt] + rb);
        dk[dt] = mfma32((bf16x8)__builtin_shufflevector(q0, q1, 0, 1, 2, 3, 4, 5, 6, 7), sb, dk[dt]);
      }
    }
  };
  auto step = [&](int it, int buf) {
    if (it + 1 < total) gload(it + 1);
    const int qs = (qt0 + it % nqt) * 64 + 32 * m;
    if (qs > kw) subtile(buf, qs, false);        // strictly below this wave's diagonal
    else if (qs == kw) subtile(buf, qs, true);  // the diagonal sub-tile
    if (it + 1 < total) swrite(buf ^ 1);
    __syncthreads();
  };

  gload(0);
  swrite(0);
  __syncthreads();
  int it = 0;
  for (; it + 1 < total; it += 2) {  // unrolled by 2: buffer offsets become immediates
    step(it, 0);
    step(it + 1, 1);
  }
  if (it < total) step(it, 0);
  // sum the two query halves' partials: waves m = 1 park theirs in LDS
  // (4 waves x 2 x 64 lanes x 16 ND floats; Q/dO/K/V are dead)
  constexpr int RW = ND * 16 * 64;  // floats per (wave, dk|dv)
  float* red = (float*)smem;
  if (m == 1) {
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
      for (int j = 0; j < 16; j += 4) {
        *(f32x4*)(red + (kg * 2 + 0) * RW + (dt * 16 + j) * 64 + lane * 4) =
            f32x4{dk[dt][j], dk[dt][j + 1], dk[dt][j + 2], dk[dt][j + 3]};
        *(f32x4*)(red + (kg * 2 + 1) * RW + (dt * 16 + j) * 64 + lane * 4) =
            f32x4{dv[dt][j], dv[dt][j + 1], dv[dt][j + 2], dv[dt][j + 3]};
      }
  }
  __syncthreads();
  if (m == 1 || (TAIL && mykey >= S)) return;
#pragma unroll
  for (int dt = 0; dt < ND; ++dt)
#pragma unroll
    for (int j = 0; j < 16; j += 4) {
      const f32x4 a = *(const f32x4*)(red + (kg * 2 + 0) * RW + (dt * 16 + j) * 64 + lane * 4);
      const f32x4 c = *(const f32x4*)(red + (kg * 2 + 1) * RW + (dt * 16 + j) * 64 + lane * 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        dk[dt][j + i] += a[i];
        dv[dt][j + i] += c[i];
      }
    }
  // store: lane owns key `mykey`, d rows 32dt + 8g + 4hh + (0..3)
  bf16_t* dkr = dK + koff + (int64_t)mykey * D;
  bf16_t* dvr = dV + koff + (int64_t)mykey * D;
#pragma unroll
  for (int dt = 0; dt < ND; ++dt)
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      uint2 a[2], c[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int g = 2 * k + u;
        a[u].x = pack2(dk[dt][4 * g + 0] * scale, dk[dt][4 * g + 1] * scale);
        a[u].y = pack2(dk[dt][4 * g + 2] * scale, dk[dt][4 * g + 3] * scale);
        c[u].x = pack2(dv[dt][4 * g + 0], dv[dt][4 * g + 1]);
        c[u].y = pack2(dv[dt][4 * g + 2], dv[dt][4 * g + 3]);
      }
      store_pair16(dkr, 32 * dt + 16 * k, hh, a[0], a[1]);
      store_pair16(dvr, 32 * dt + 16 * k, hh, c[0], c[1]);
    }
}

// ---------------------------------------------------------------------------
// dQ: same geometry as the forward (8 waves x 32 query rows, XCD-aware
// heaviest-first blocks, 64-key K/V tiles shared by all waves, query on the
// lane).  Per tile: S^T = K Q^T and dP^T = V dO^T (K, V row reads), then
// dS^T = P^T (dP^T - delta) feeds dQ^T += K^T dS^T (K transposed reads) as
// the B operand straight from the accumulator.  K and V share the
// one-image-two-ways layout (rt_off).
// ---------------------------------------------------------------------------
template <int D, bool TAIL>
__global__ __launch_bounds__(512, 1) void attn_bwd_dq_kernel(
    const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V,
    const bf16_t* __restrict__ dO, const bf16_t* __restrict__ O, const float* __restrict__ LSE,
    float* __restrict__ DELTA, bf16_t* __restrict__ dQ, int B, int H, int Hk, int S, float scale, float scale_log2,
    int o_bshd) {
  using G = AG<D>;
  constexpr int ROWB = G::ROWB, NCH = G::NCH, NS = G::NS, ND = G::ND, TILEB = G::TILEB;
  constexpr int NL = TK * NCH / 512;
  extern __shared__ __attribute__((aligned(16))) char smem[];  // 2 x (K tile + V tile)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int nqb = (S + FWD_QB - 1) / FWD_QB;
  int qb, h, b;
  fwd_block_coords(blockIdx.x, nqb, B, H, Hk, &qb, &h, &b);
  const int hk = h / (H / Hk);
  const int64_t qoff = ((int64_t)(b * H + h) * S) * D;
  const int64_t koff = ((int64_t)(b * Hk + hk) * S) * D;
  const int q0 = qb * FWD_QB + wave * 32;
  const bool live = q0 < S;
  const int myq = q0 + r;
  const int myq_ld = TAIL ? min(myq, S - 1) : myq;
  const int kend = min(S, (qb + 1) * FWD_QB);
  const int ntiles = (kend + TK - 1) / TK;
  const int t_diag = live ? (q0 + 31) / TK : -1;

  bf16x8 qf[NS], of[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    qf[s] = live ? as_bf16x8(ld16(Q + qoff + (int64_t)myq_ld * D + 16 * s + 8 * hh)) : bf16x8{};
    of[s] = live ? as_bf16x8(ld16(dO + o_off<D>(b, h, myq_ld, H, S, o_bshd) + 16 * s + 8 * hh)) : bf16x8{};
  }
  const float lse2 = live ? LSE[(int64_t)(b * H + h) * S + myq_ld] * LOG2E : 0.f;
  // delta = rowsum(dO * O), computed here (the lane already holds its half of
  // the dO row) and published for the dK/dV kernel that runs next
  float del = 0.f;
  if (live) {
    float part = 0.f;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      float a[8], g[8];
      unpack8(ld16(O + o_off<D>(b, h, myq_ld, H, S, o_bshd) + 16 * s + 8 * hh), a);
      unpack8(__builtin_bit_cast(u32x4, of[s]), g);
#pragma unroll
      for (int j = 0; j < 8; ++j) part = fmaf(a[j], g[j], part);
    }
    del = xhalf_sum(part);
    if (hh == 0 && (!TAIL || myq < S)) DELTA[(int64_t)(b * H + h) * S + myq] = del;
  }
  f32x16 acc[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i)
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[i][j] = 0.f;

  int rro[NS], tro[ND], tro8[ND];
  {
#pragma unroll
    for (int s = 0; s < NS; ++s) rro[s] = rt_off<D>(r, 2 * s + hh);
    const int g = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) {
      const int c = 4 * dt + 2 * (g & 1) + (pp >> 1);
      tro[dt] = rt_off<D>(4 * hh + qq, c) + (pp & 1) * 8;
      tro8[dt] = rt_off<D>(4 * hh + qq + 8, c) + (pp & 1) * 8;
    }
  }

  u32x4 stk[NL], stv[NL];
  auto gload = [&](int t) {
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int e = tid + 512 * i;
      const int key = e / NCH, c = e % NCH;
      const int64_t gidx = koff + (int64_t)(TAIL ? min(t * TK + key, S - 1) : t * TK + key) * D + c * 8;
      stk[i] = ld16(K + gidx);
      stv[i] = ld16(V + gidx);
    }
  };
  auto swrite = [&](int buf) {
    char* kb = smem + buf * 2 * TILEB;
    char* vb = kb + TILEB;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int e = tid + 512 * i;
      const int key = e / NCH, c = e % NCH;
      *(u32x4*)(kb + rt_off<D>(key, c)) = stk[i];
      *(u32x4*)(vb + rt_off<D>(key, c)) = stv[i];
    }
  };
  auto compute = [&](int t, int buf, bool mask) {
    const char* kb = smem + buf * 2 * TILEB;
    const char* vb = kb + TILEB;
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const f32x16 z = {};
      f32x16 sc = mfma32(as_bf16x8(*(const u32x4*)(kb + rro[0] + 32 * ROWB * n)), qf[0], z);
      f32x16 dp = mfma32(as_bf16x8(*(const u32x4*)(vb + rro[0] + 32 * ROWB * n)), of[0], z);
#pragma unroll
      for (int s = 1; s < NS; ++s) {
        sc = mfma32(as_bf16x8(*(const u32x4*)(kb + rro[s] + 32 * ROWB * n)), qf[s], sc);
        dp = mfma32(as_bf16x8(*(const u32x4*)(vb + rro[s] + 32 * ROWB * n)), of[s], dp);
      }
      uint32_t sw[8];
      const f32x2 c2 = {scale_log2, scale_log2}, nl2 = {-lse2, -lse2}, del2 = {del, del};
#pragma unroll
      for (int j = 0; j < 16; j += 2) {
        const f32x2 x = pk_fma(f32x2{sc[j], sc[j + 1]}, c2, nl2);
        float p0 = EXP2(x[0]);
        float p1 = EXP2(x[1]);
        if (mask) {
          const int key = t * TK + 32 * n + (j & 3) + 8 * (j >> 2) + 4 * hh;
          if (key > myq) p0 = 0.f;
          if (key + 1 > myq) p1 = 0.f;
        }
        const f32x2 d = (f32x2{dp[j], dp[j + 1]} - del2) * f32x2{p0, p1};
        sw[j >> 1] = pack2(d[0], d[1]);
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        u32x4 w;
#pragma unroll
        for (int i = 0; i < 4; ++i) w[i] = sw[4 * s2 + i];
        const bf16x8 sb = as_bf16x8(w);
        const int rb = 32 * n + 16 * s2;
#pragma unroll
        for (int dt = 0; dt < ND; ++dt) {
          const bf16x4 a = tr_read(kb, tro[dt] + rb * ROWB);
          const bf16x4 c = tr_read(kb, tro8[dt] + rb * ROWB);
          acc[dt] = mfma32((bf16x8)__builtin_shufflevector(a, c, 0, 1, 2, 3, 4, 5, 6, 7), sb, acc[dt]);
        }
      }
    }
  };
  auto step = [&](int t, int buf) {
    if (t + 1 < ntiles) gload(t + 1);
    if (t < t_diag) compute(t, buf, false);
    else if (t == t_diag) compute(t, buf, true);
    if (t + 1 < ntiles) swrite(buf ^ 1);
    __syncthreads();
  };

  gload(0);
  swrite(0);
#pragma unroll
  for (int s = 0; s < NS; ++s) asm volatile("" ::"v"(qf[s]), "v"(of[s]));  // retire resident loads (see fwd)
  asm volatile("" ::"v"(lse2), "v"(del));
  __syncthreads();
  int t = 0;
  for (; t + 1 < ntiles; t += 2) {
    step(t, 0);
    step(t + 1, 1);
  }
  if (t < ntiles) step(t, 0);

  if (!live || (TAIL && myq >= S)) return;
  bf16_t* qrow = dQ + qoff + (int64_t)myq * D;
#pragma unroll
  for (int dt = 0; dt < ND; ++dt)
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      uint2 w[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int g = 2 * k + u;
        w[u].x = pack2(acc[dt][4 * g + 0] * scale, acc[dt][4 * g + 1] * scale);
        w[u].y = pack2(acc[dt][4 * g + 2] * scale, acc[dt][4 * g + 3] * scale);
      }
      store_pair16(qrow, 32 * dt + 16 * k, hh, w[0], w[1]);
    }
}

// ---------------------------------------------------------------------------
// Backward with dS through HBM (TOA_ATTN_BWD=ds): the dK/dV kernel already
// forms dS = P * (dP - delta) for every (32-query, 32-key) block at or below
// the diagonal; the dS form's dK/dV kernel also stores them (bf16, 2 KB per
// block of 16-byte (key, 8-query) chunks, chunk (k, g') at g' * 512 + k * 16
// bytes, so each store instruction writes 1 KB contiguous; the blocks of one
// (batch, head) packed lower-triangular: block (qi, ki) at qi (qi + 1) / 2 + ki).  dQ = scale * dS K is
// then a plain GEMM over those blocks -- the split form's dQ kernel recomputes
// S and dP for it (3 of the backward's 7 executed S^2 D products; this form
// executes 5).  The dS round trip is 2 x 3.2 GB at the Llama-3-8B shape; the
// GEMM streams it once.  delta = rowsum(dO * O) moves to its own pass, since
// the dK/dV kernel now runs first.
// ---------------------------------------------------------------------------
template <int D>
__global__ __launch_bounds__(256) void attn_delta_kernel(const bf16_t* __restrict__ O, const bf16_t* __restrict__ dO,
                                                         const float* __restrict__ LSE, float* __restrict__ NDELTA,
                                                         float* __restrict__ NLSE2, int rows, int H, int S,
                                                         int o_bshd) {
  constexpr int LPR = D / 8;  // lanes per row, 16 B each
  const int lin = blockIdx.x * (256 / LPR) + (int)threadIdx.x / LPR;
  const int c = threadIdx.x % LPR;
  if (lin >= rows) return;  // whole LPR-lane groups leave together
  // O / dO in [B, S, H, D]: walk the rows in (b, s, h) order, so a wave's
  // loads are contiguous (in (b, h, s) order they sit H * D apart)
  int s, bh;
  if (o_bshd) {
    const int h = lin % H, bs = lin / H;
    s = bs % S;
    bh = (bs / S) * H + h;
  } else {
    s = lin % S;
    bh = lin / S;
  }
  const int row = bh * S + s;
  const int64_t off = o_off<D>(bh / H, bh % H, s, H, S, o_bshd) + c * 8;
  float a[8], g[8];
  unpack8(ld16(O + off), a);
  unpack8(ld16(dO + off), g);
  float part = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) part = fmaf(a[j], g[j], part);
#pragma unroll
  for (int m = LPR / 2; m >= 1; m >>= 1) part += __shfl_xor(part, m, LPR);
  if (c == 0) {
    NDELTA[row] = -part;              // the dP accumulators' initial value
    NLSE2[row] = -(LSE[row] * LOG2E);  // the exp2 argument's addend
  }
}

// RoPE backward on a lane's accumulator tiles, in place (the fused
// rope + attention backward, toa_attn_bwd_rope): element j of tile dt is
// d = 32 dt + 8 (j / 4) + 4 hh + j % 4, its rotation partner d + D / 2 sits in
// tile dt + ND / 2 of the same lane; dx1 = dy1 c + dy2 s, dx2 = dy2 c - dy1 s
// with c / s = cos / sin[position][d], after scaling by `scale`.
template <int D>
__device__ __forceinline__ void rope_bwd_acc(f32x16 (&a)[D / 32], const float* __restrict__ cs,
                                             const float* __restrict__ sn, int hh, float scale) {
  constexpr int HALF = D / 64;
#pragma unroll
  for (int dt = 0; dt < HALF; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 c = *(const f32x4*)(cs + 32 * dt + 8 * g + 4 * hh);
      const f32x4 sv = *(const f32x4*)(sn + 32 * dt + 8 * g + 4 * hh);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float y1 = a[dt][4 * g + e] * scale, y2 = a[dt + HALF][4 * g + e] * scale;
        a[dt][4 * g + e] = y1 * c[e] + y2 * sv[e];
        a[dt + HALF][4 * g + e] = y2 * c[e] - y1 * sv[e];
      }
    }
}

// the same with the lane's cos / sin values loaded beforehand (rope_cs_load)
template <int D>
__device__ __forceinline__ void rope_cs_load(f32x4 (&c)[D / 64][4], f32x4 (&sv)[D / 64][4],
                                             const float* __restrict__ cs, const float* __restrict__ sn, int hh) {
#pragma unroll
  for (int dt = 0; dt < D / 64; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      c[dt][g] = *(const f32x4*)(cs + 32 * dt + 8 * g + 4 * hh);
      sv[dt][g] = *(const f32x4*)(sn + 32 * dt + 8 * g + 4 * hh);
    }
}
template <int D>
__device__ __forceinline__ void rope_bwd_acc(f32x16 (&a)[D / 32], const f32x4 (&c)[D / 64][4],
                                             const f32x4 (&sv)[D / 64][4], float scale) {
  constexpr int HALF = D / 64;
#pragma unroll
  for (int dt = 0; dt < HALF; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float y1 = a[dt][4 * g + e] * scale, y2 = a[dt + HALF][4 * g + e] * scale;
        a[dt][4 * g + e] = y1 * c[dt][g][e] + y2 * sv[dt][g][e];
        a[dt + HALF][4 * g + e] = y2 * c[dt][g][e] - y1 * sv[dt][g][e];
      }
}

template <int D>
struct DQG {
  static constexpr int KT = TK * AG<D>::ROWB;  // one 64-key K tile
  static constexpr int DSW = 4096;             // per wave and tile: two 32 x 32 dS blocks
  static constexpr int STAGE = KT + 8 * DSW;   // 48 KB (D = 128) / 40 KB (D = 64)
  static constexpr int NKP = KT / 1024 / 8;    // K LDS-DMA pieces per wave and tile
};

// dQ^T[d][q] = sum_key K^T[d][key] dS^T[key][q] for one (batch, head) and a
// 256-row query block: 8 waves x 32 query rows, 64-key tiles, v_mfma 32x32x16
// with the accumulator of the split dQ kernel (query on the lane, so its
// epilogue is reused).  Everything reaches LDS by LDS-DMA in a 3-slot ring
// (guide §5 "Pipelining across barriers": counted vmcnt, raw s_barrier, one
// distinct LDS object per slot so no read waits on another slot's DMA):
//  * the K tile, shared by the 8 waves, in the rt_off image (source-swizzled);
//    the A operand comes out of it by transposed reads, as in the split kernel;
//  * each wave's own two dS blocks, copied verbatim; a transposed read of a
//    block's (key, 4-query) pieces gives the B operand (query on the lane, 4
//    keys per read; the key order matches the K^T read's, as in the split
//    kernel).
template <int D, bool ROPE = false>
__global__ __launch_bounds__(512, 1) void attn_bwd_dqg_kernel(const bf16_t* __restrict__ K,
                                                              const bf16_t* __restrict__ dS, bf16_t* __restrict__ dQ,
                                                              int B, int H, int Hk, int S, float scale,
                                                              const float* __restrict__ cosv = nullptr,
                                                              const float* __restrict__ sinv = nullptr, int H3 = 0) {
  using G = AG<D>;
  constexpr int ROWB = G::ROWB, NCH = G::NCH, ND = G::ND;
  constexpr int KT = DQG<D>::KT, NKP = DQG<D>::NKP;
  __shared__ __attribute__((aligned(1024))) char s0[DQG<D>::STAGE];
  __shared__ __attribute__((aligned(1024))) char s1[DQG<D>::STAGE];
  __shared__ __attribute__((aligned(1024))) char s2[DQG<D>::STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hh = lane >> 5;
  const int nqb = S / FWD_QB;
  int qb, h, b;
  fwd_block_coords(blockIdx.x, nqb, B, H, Hk, &qb, &h, &b);
  const int hk = h / (H / Hk);
  const int nb = S >> 5;
  const int qi = qb * 8 + wave;    // this wave's 32-row query block
  const int tdiag = qi >> 1;       // its last 64-key tile
  const int ntiles = (qb + 1) * 4;  // the workgroup's causal key range
  const bf16_t* kbase = K + ((int64_t)(b * Hk + hk) * S) * D;
  const bf16_t* dsrow = dS + (((int64_t)(b * H + h) * (nb * (nb + 1) / 2) + (int64_t)qi * (qi + 1) / 2) << 10);

  // K tile pieces: wave w fills rows (w NKP + u) * rows_per_piece ..; the
  // lane's 16 B land at chunk position lane % NCH, so it loads the chunk the
  // rt_off image keeps there
  constexpr int RPP = 1024 / ROWB;
  int kgo[NKP];
#pragma unroll
  for (int u = 0; u < NKP; ++u) {
    const int row = (wave * NKP + u) * RPP + lane / NCH, cpos = lane % NCH;
    const int swz = D == 128 ? (((row & 3) << 2) | ((row >> 2) & 3)) : (((row & 3) << 1) | ((row >> 2) & 1));
    kgo[u] = row * D + ((cpos ^ swz) << 3);
  }
  // dS blocks as stored: 16-byte chunk (key k, queries 8g' .. + 7) at
  // g' * 512 + k * 16.  In LDS the keys of chunk row g' rotate by 4g' (chunk
  // (k, g') at g' * 512 + ((k + 4g') & 31) * 16), which makes the transposed
  // reads below conflict-free; the rotation is applied to the DMA's source
  // chunks: LDS chunk j = 64 half + lane holds (k = ((j & 31) - 4g') & 31, g' = j >> 5).
  int dsg[2];
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    const int gq = 2 * half + (lane >> 5);
    dsg[half] = (32 * gq + (((lane & 31) - 4 * gq) & 31)) * 8;
  }
  auto stage_k = [&](int t, char* st) {  // this wave's pieces of K tile t (shared by the workgroup)
#pragma unroll
    for (int u = 0; u < NKP; ++u)
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(kbase + (int64_t)t * TK * D + (uint32_t)kgo[u]),
          (__attribute__((address_space(3))) void*)(st + (wave * NKP + u) * 1024), 16, 0, 0);
  };
  auto stage_s = [&](int t, char* st) {  // this wave's own dS blocks 2t, 2t + 1 (clamped to the diagonal)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int ki = min(2 * t + (v >> 1), qi);
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(dsrow + ((int64_t)ki << 10) + (uint32_t)dsg[v & 1]),
          (__attribute__((address_space(3))) void*)(st + KT + wave * DQG<D>::DSW + v * 1024), 16, 0,
          2 /* nt: read once; leave L2 to the K tiles */);
    }
  };

  int tro[ND], tro8[ND];
  {
    const int g = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) {
      const int c = 4 * dt + 2 * (g & 1) + (pp >> 1);
      tro[dt] = rt_off<D>(4 * hh + qq, c) + (pp & 1) * 8;
      tro8[dt] = rt_off<D>(4 * hh + qq + 8, c) + (pp & 1) * 8;
    }
  }
  // dS^T operand: group lane 4q + p reads key R = 16 s2 + 8 e + 4 hh + q,
  // queries 16 (g & 1) + 4p .. + 3 = half (p & 1) of chunk g' = 2 (g & 1) + (p >> 1)
  int dso[2][2];
  {
    const int gq = 2 * ((lane >> 4) & 1) + ((lane & 3) >> 1), q = (lane >> 2) & 3;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int e = 0; e < 2; ++e)
        dso[s2][e] = gq * 512 + ((16 * s2 + 8 * e + 4 * hh + q + 4 * gq) & 31) * 16 + (lane & 1) * 8;
  }

  f32x16 acc[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i)
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[i][j] = 0.f;
  // the epilogue's cos / sin rows loaded ahead of the main loop, so their
  // latency hides under it instead of following it
  f32x4 rcs[D / 64][4], rsn[D / 64][4];
  if constexpr (ROPE)
    rope_cs_load<D>(rcs, rsn, cosv + (int64_t)(qi * 32 + r) * (D / 2), sinv + (int64_t)(qi * 32 + r) * (D / 2), hh);

  auto compute = [&](int t, const char* st) {
    const char* dimg = st + KT + wave * DQG<D>::DSW;
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      if (n == 1 && 2 * t + 1 > qi) break;  // above the diagonal: never stored
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x4 lo = tr_read(dimg + n * 2048, dso[s2][0]);
        const bf16x4 hi = tr_read(dimg + n * 2048, dso[s2][1]);
        const bf16x8 sb = (bf16x8)__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        const int rb = (32 * n + 16 * s2) * ROWB;
#pragma unroll
        for (int dt = 0; dt < ND; ++dt) {
          const bf16x4 a = tr_read(st, tro[dt] + rb), c = tr_read(st, tro8[dt] + rb);
          acc[dt] = mfma32((bf16x8)__builtin_shufflevector(a, c, 0, 1, 2, 3, 4, 5, 6, 7), sb, acc[dt]);
        }
      }
    }
  };
  auto sync = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  // The K tiles are shared, so they are restaged only behind a barrier; a
  // wave's dS slot is its own, so it is refilled as soon as the wave has
  // read it -- dS runs three tiles ahead, K two.  Per-wave issue order:
  // dS0 K0 dS1 K1 dS2 | K2 dS3 | K3 dS4 | ...; at tile t, K t and dS t are
  // retired once only dS t+1, K t+1 and dS t+2 (2 x 4 + NKP pieces) may
  // still be in flight.  Past the end the last tile is re-fetched into a
  // slot nobody reads (constant DMA count).
  auto it = [&](int t, const char* cur, char* kpre) {
    __builtin_amdgcn_s_waitcnt(0x0F70 | (8 + NKP));
    sync();  // every wave's K pieces of t landed; every wave done with K t - 1
    stage_k(min(t + 2, ntiles - 1), kpre);
    if (t <= tdiag) compute(t, cur);
    stage_s(min(t + 3, ntiles - 1), (char*)cur);
  };
  stage_s(0, s0);
  stage_k(0, s0);
  stage_s(1, s1);
  stage_k(1, s1);
  stage_s(2, s2);
  // whole rounds of three (the extra tiles compute nothing): a conditional
  // it() would let hipcc's wait-count pass see a path on which the slot
  // about to be read was just restaged, and wait vmcnt(0) before every read
  for (int t = 0; t < ntiles; t += 3) {
    it(t, s0, s2);
    it(t + 1, s1, s0);
    it(t + 2, s2, s1);
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);  // no LDS-DMA in flight at exit

  const int myq = qi * 32 + r;
  bf16_t* qrow = dQ + ((int64_t)(b * H + h) * S + myq) * D;
  float osc = scale;
  if constexpr (ROPE) {  // rotate back and write the q part of d(qkv) row (b, myq)
    rope_bwd_acc<D>(acc, rcs, rsn, scale);
    qrow = dQ + ((int64_t)b * S + myq) * H3 * D + h * D;
    osc = 1.f;
  }
#pragma unroll
  for (int dt = 0; dt < ND; ++dt)
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      uint2 w[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int g = 2 * k + u;
        w[u].x = pack2(acc[dt][4 * g + 0] * osc, acc[dt][4 * g + 1] * osc);
        w[u].y = pack2(acc[dt][4 * g + 2] * osc, acc[dt][4 * g + 3] * osc);
      }
      store_pair16(qrow, 32 * dt + 16 * k, hh, w[0], w[1]);
    }
}

// dK / dV of the dS form: the split form's dK/dV kernel (same workgroup /
// wave geometry and the same sub-tile body) with
//  * the Q / dO tiles and their -lse log2(e) / -delta rows (from the delta
//    pass) brought in by LDS-DMA into two distinct LDS objects (no register
//    staging: 16 VGPRs and the ds_write pass freed; guide §5 "Pipelining
//    across barriers"), and
//  * every (32-query, 32-key) dS block stored for the dQ GEMM (layout at
//    attn_bwd_dqg_kernel), between the sub-tile's two MFMA halves so the
//    stores drain under the second half.
// The sub-tile reads its LDS fragments one MFMA pair ahead of their use
// (round 4: counted lgkmcnt waits, which the buffer-path DMA makes possible;
// 2.13 -> 1.93 ms at the bench shape, profiles/r4_attn).  Each step ends with
// its own DMA retired and a barrier; the wave's two dS stores, issued after
// the DMA, drain under the next step (vmcnt(2)).  LSE / DELTA here are the
// delta pass's -lse log2(e) / -delta rows.  S % 256 == 0 only (no ragged
// tiles).  TIMED: per wave, s_memtime sums of issue time and step-end wait
// time (scripts/attn_bwd_ab.py --timing).
template <int D, bool ROPE = false, bool TIMED = false>
__global__ __launch_bounds__(512, 1) void attn_bwd_dkdv_ds_kernel(
    const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V,
    const bf16_t* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ DELTA,
    bf16_t* __restrict__ dK, bf16_t* __restrict__ dV, bf16_t* __restrict__ dS, int B, int H, int Hk, int S,
    float scale, float scale_log2, int o_bshd,
    const float* __restrict__ cosv = nullptr, const float* __restrict__ sinv = nullptr, int H3 = 0,
    unsigned long long* __restrict__ tstat = nullptr) {
  using G = AG<D>;
  constexpr int ROWB = G::ROWB, NCH = G::NCH, NS = G::NS, ND = G::ND, TILEB = G::TILEB;
  constexpr int QBUF = DKV<D>::QBUF, KVB = DKV<D>::KVB;
  constexpr int NLK = 128 * NCH / 512;
  // Q/dO/lse/-delta buffers 0 and 1, K and V: distinct LDS objects, so
  // hipcc's wait-count pass knows a read of one buffer cannot alias the
  // LDS-DMA filling the other (with one array it waits vmcnt(0) before the
  // first transposed read of every sub-tile)
  __shared__ __attribute__((aligned(1024))) char qd0[QBUF];
  __shared__ __attribute__((aligned(1024))) char qd1[QBUF];
  __shared__ __attribute__((aligned(1024))) char kv[2 * KVB];
  char* kimg = kv;
  char* vimg = kv + KVB;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int kg = wave & 3, m = wave >> 2;
  // (b, hk) fastest
  // heaviest first: key block kb sees S / 64 - 2 kb query tiles, so kb = 0
  // leads (largest-first keeps the last wave of workgroups short: a
  // simulated 800 vs 912 tile-units makespan at the bench shape)
  const int kb = (int)(blockIdx.x / (B * Hk));
  const int bh = blockIdx.x % (B * Hk);
  const int b = bh / Hk, hk = bh % Hk;
  const int rep = H / Hk;
  const int kw = kb * 128 + kg * 32;  // first key of this wave
  const int mykey = kw + r;
  const int64_t koff = ((int64_t)(b * Hk + hk) * S) * D;

  // K / V of the block -> LDS (rt_off image: row reads give the B operands)
#pragma unroll
  for (int i = 0; i < NLK; ++i) {
    const int e = tid + 512 * i;
    const int row = e / NCH, c = e % NCH;
    const int64_t g = koff + (int64_t)(kb * 128 + row) * D + c * 8;
    *(u32x4*)(kimg + rt_off<D>(row, c)) = ld16(K + g);
    *(u32x4*)(vimg + rt_off<D>(row, c)) = ld16(V + g);
  }
  f32x16 dk[ND], dv[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i)
#pragma unroll
    for (int j = 0; j < 16; ++j) { dk[i][j] = 0.f; dv[i][j] = 0.f; }

  int rro[NS], tro[ND], tro8[ND];
  {
#pragma unroll
    for (int s = 0; s < NS; ++s) rro[s] = rt_off<D>(r, 2 * s + hh);
    const int g = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) {
      const int c = 4 * dt + 2 * (g & 1) + (pp >> 1);
      tro[dt] = rt_off<D>(4 * hh + qq, c) + (pp & 1) * 8;
      tro8[dt] = rt_off<D>(4 * hh + qq + 8, c) + (pp & 1) * 8;
    }
  }

  const int qt0 = (kb * 128) / 64;  // first causal 64-row query tile
  const int nqt = (S + TK - 1) / TK - qt0;
  const int total = nqt * rep;
  // Q / dO tiles by LDS-DMA (no register staging): 1-KB piece pt of a tile
  // covers rows RPP pt .. + RPP - 1; waves 0-3 fetch Q, 4-7 dO, PW pieces
  // each.  The lane's 16 B land at chunk position lane % NCH of row
  // RPP pt + lane / NCH, so it loads the chunk the rt_off image keeps there
  // (the swizzle's row-block part is (pt & 3) << 3 elements at D = 128, 0 at 64).
  constexpr int RPP = 1024 / ROWB, PPT = TILEB / 1024, PW = PPT / 4;
  const int lrow = lane / NCH;
  const int lswz = D == 128 ? (lrow & 3) << 2 : ((lrow & 3) << 1) | ((lrow >> 2) & 1);
  const int lcol = ((lane % NCH) ^ lswz) << 3;
  auto stage = [&](int it, int buf) {
    const int hq = hk * rep + it / nqt;
    const int qt = qt0 + it % nqt;
    char* st = buf ? qd1 : qd0;
    if (wave < 4) {
      const auto rs = buf_rsrc(Q + ((int64_t)(b * H + hq) * S + qt * 64) * D);
#pragma unroll
      for (int u = 0; u < PW; ++u) {
        const int pt = PW * wave + u;
        const int col = D == 128 ? lcol ^ ((pt & 3) << 3) : lcol;
        BUF_DMA(16, rs, (uint32_t)((RPP * pt + lrow) * D + col) * 2, st + pt * 1024);
      }
    } else {
      const int rstr = o_bshd ? H * D : D;  // dO row stride (elements)
      const auto rs = buf_rsrc(dO + o_off<D>(b, hq, qt * 64, H, S, o_bshd));
#pragma unroll
      for (int u = 0; u < PW; ++u) {
        const int pt = PW * (wave - 4) + u;
        const int col = D == 128 ? lcol ^ ((pt & 3) << 3) : lcol;
        BUF_DMA(16, rs, (uint32_t)((RPP * pt + lrow) * rstr + col) * 2, st + TILEB + pt * 1024);
      }
    }
    if (wave == 0) {  // -lse log2e and -delta rows (the delta pass wrote them): 256 B each
      const int64_t li = (int64_t)(b * H + hq) * S + qt * 64;
      BUF_DMA(4, buf_rsrc(LSE + li), lane * 4, st + 2 * TILEB);
      BUF_DMA(4, buf_rsrc(DELTA + li), lane * 4, st + 2 * TILEB + 256);
    }
  };

  // one (32-query, 32-key) sub-tile: S / dP, P and dS, dV^T / dK^T, the dS
  // block stored.  Two fragment sets per operand stream, so each LDS read is
  // issued one MFMA pair before its MFMA (counted lgkmcnt waits instead of a
  // lgkmcnt(0) before every MFMA); the -lse rows are read under the last
  // S / dP pair.
  auto subtile = [&](int buf, int qs, bool mask, bf16_t* dsb) {
    const char* qi = buf ? qd1 : qd0;
    const char* oi = qi + TILEB;
    const float* lb = (const float*)(qi + 2 * TILEB);
    // D = 128: the operand offsets from 4 per-lane values instead of 16
    // registers (rro[s] = rb + 32 (s ^ rc), tro[dt] = tb + 64 (dt ^ qq),
    // tro8 = tro + d8); the empty asm keeps hipcc from hoisting the 16 back
    // out of the loop
    int rb = 0, rc = 0, tb = 0, d8 = 0, tq = 0;
    if constexpr (D == 128) {
      const int swz = ((r & 3) << 2) | ((r >> 2) & 3);
      rb = r * ROWB + ((hh ^ (swz & 1)) << 4);
      rc = swz >> 1;
      tq = (lane & 15) >> 2;
      tb = tro[0] - (tq << 6);
      d8 = tro8[0] - tro[0];
      opaque_v(rb);
      opaque_v(rc);
      opaque_v(tb);
      opaque_v(d8);
      opaque_v(tq);
    }
    auto rro_at = [&](int s) { return D == 128 ? rb + ((s ^ rc) << 5) : rro[s]; };
    auto tro_at = [&](int dt) { return D == 128 ? tb + ((dt ^ tq) << 6) : tro[dt]; };
    auto tro8_at = [&](int dt) { return D == 128 ? tb + ((dt ^ tq) << 6) + d8 : tro8[dt]; };
    f32x16 dp;
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const f32x4 d4 = *(const f32x4*)(lb + 64 + 32 * m + 8 * g4 + 4 * hh);
#pragma unroll
      for (int j = 0; j < 4; ++j) dp[4 * g4 + j] = d4[j];
    }
    f32x16 sc = {};
    // S / dP: the (Q, K) and (dO, V) fragment pairs of step s + 1 are read
    // while the MFMAs of step s issue, staggered by half a step (the Q/K pair
    // of s + 1 before S(s), the dO/V pair before dP(s)): 24 fragment
    // registers, two MFMAs of cover for every read
    bf16x8 qk[2][2], ov[2][2];
    auto ldqk = [&](int s, bf16x8(&f)[2]) {
      const int o = rro_at(s);
      f[0] = as_bf16x8(*(const u32x4*)(qi + o + 32 * ROWB * m));
      f[1] = as_bf16x8(*(const u32x4*)(kimg + o + 32 * ROWB * kg));
    };
    auto ldov = [&](int s, bf16x8(&f)[2]) {
      const int o = rro_at(s);
      f[0] = as_bf16x8(*(const u32x4*)(oi + o + 32 * ROWB * m));
      f[1] = as_bf16x8(*(const u32x4*)(vimg + o + 32 * ROWB * kg));
    };
    f32x4 l4[4];
    ldqk(0, qk[0]);
    ldov(0, ov[0]);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      if (s + 1 < NS) ldqk(s + 1, qk[(s + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
      sc = mfma32(qk[s & 1][0], qk[s & 1][1], sc);
      __builtin_amdgcn_sched_barrier(0);
      if (s + 1 < NS) {
        ldov(s + 1, ov[(s + 1) & 1]);
      } else {
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) l4[g4] = *(const f32x4*)(lb + 32 * m + 8 * g4 + 4 * hh);  // -lse * log2(e)
      }
      __builtin_amdgcn_sched_barrier(0);
      dp = mfma32(ov[s & 1][0], ov[s & 1][1], dp);
      __builtin_amdgcn_sched_barrier(0);
    }
    // P and dS (scalar VALU: a register-pair form measured 3 % slower per
    // step, profiles/r4_attn/r4_batch): elements 0-7 (the first 16-query
    // half, s2 = 0) here, 8-15 between the s2 = 0 MFMAs below, whose issue
    // they overlap (1.2 % fewer cycles per step, profiles/r4_attn/r4_attn6).
    uint32_t pw[8], sw[8];
    auto expair = [&](int j) {
      float p0 = EXP2(fmaf(sc[j], scale_log2, l4[j >> 2][j & 3]));
      float p1 = EXP2(fmaf(sc[j + 1], scale_log2, l4[j >> 2][(j + 1) & 3]));
      if (mask) {
        const int q = qs + (j & 3) + 8 * (j >> 2) + 4 * hh;
        if (q < mykey) p0 = 0.f;
        if (q + 1 < mykey) p1 = 0.f;
      }
      pw[j >> 1] = pack2(p0, p1);
      sw[j >> 1] = pack2(p0 * dp[j], p1 * dp[j + 1]);
    };
#pragma unroll
    for (int j = 0; j < 8; j += 2) expair(j);
    // dV^T / dK^T: 8 (s2, dt) pairs of MFMAs, the transposed reads one pair ahead
    bf16x4 ft[2][4];
    auto ldt = [&](int i, bf16x4(&f)[4]) {
      const int s2 = i / ND, dt = i % ND;
      const int rbo = (32 * m + 16 * s2) * ROWB;
      const int o = tro_at(dt) + rbo, o8 = tro8_at(dt) + rbo;
      f[0] = tr_read(oi, o);
      f[1] = tr_read(oi, o8);
      f[2] = tr_read(qi, o);
      f[3] = tr_read(qi, o8);
    };
    ldt(0, ft[0]);
#pragma unroll
    for (int i = 0; i < 2 * ND; ++i) {
      const int s2 = i / ND, dt = i % ND;
      u32x4 a, c;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        a[e] = pw[4 * s2 + e];
        c[e] = sw[4 * s2 + e];
      }
      if (i + 1 < 2 * ND) ldt(i + 1, ft[(i + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
      const bf16x4* f = ft[i & 1];
      dv[dt] = mfma32((bf16x8)__builtin_shufflevector(f[0], f[1], 0, 1, 2, 3, 4, 5, 6, 7), as_bf16x8(a), dv[dt]);
      dk[dt] = mfma32((bf16x8)__builtin_shufflevector(f[2], f[3], 0, 1, 2, 3, 4, 5, 6, 7), as_bf16x8(c), dk[dt]);
      if (i < ND) {  // elements 8-15, 4 / ND pairs under each s2 = 0 MFMA pair
#pragma unroll
        for (int e = 0; e < 4 / ND; ++e) expair(8 + 2 * (i * (4 / ND) + e));
      }
      __builtin_amdgcn_sched_barrier(0);
      if (i == ND - 1) {  // dS chunks (as in `subtile`), draining under the second half
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const auto x = __builtin_amdgcn_permlane32_swap(sw[4 * k], sw[4 * k + 2], false, false);
          const auto y = __builtin_amdgcn_permlane32_swap(sw[4 * k + 1], sw[4 * k + 3], false, false);
          __builtin_nontemporal_store(u32x4{x[0], y[0], x[1], y[1]}, (u32x4*)(dsb + (2 * k + hh) * 256 + r * 8));
        }
      }
    }
  };

  unsigned long long t_issue = 0, t_wait = 0;
  auto stamp = [&]() { return memtime_sync(); };
  auto step = [&](int it, int buf) {
    unsigned long long t0 = 0, t1 = 0;
    if constexpr (TIMED) t0 = stamp();
    if (it + 1 < total) stage(it + 1, buf ^ 1);
    const int qs = (qt0 + it % nqt) * 64 + 32 * m;
    const int hq = hk * rep + it / nqt, qb32 = qs >> 5, nb = S >> 5;
    bf16_t* dsb = dS + (int64_t)(b * H + hq) * (nb * (nb + 1) / 2) * 1024 + ((uint32_t)(qb32 * (qb32 + 1) / 2 + (kw >> 5)) << 10);
    if (qs > kw) subtile(buf, qs, false, dsb);        // strictly below this wave's diagonal
    else if (qs == kw) subtile(buf, qs, true, dsb);  // the diagonal sub-tile
    if constexpr (TIMED) t1 = stamp();
    if (qs < kw) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no stores this step
    asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if constexpr (TIMED) {
      const unsigned long long t2 = stamp();
      t_issue += t1 - t0;
      t_wait += t2 - t1;
    }
  };

  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  int it = 0;
  for (; it + 1 < total; it += 2) {  // unrolled by 2: buffer offsets become immediates
    step(it, 0);
    step(it + 1, 1);
  }
  if (it < total) step(it, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the last dS stores
  if constexpr (TIMED) {
    if (lane == 0) {
      unsigned long long* o = tstat + ((int64_t)blockIdx.x * 8 + wave) * 4;
      o[0] = t_issue;
      o[1] = t_wait;
      o[2] = (unsigned long long)total;
      o[3] = 0;
    }
  }

  // sum the two query halves' partials: waves m = 1 park theirs in LDS
  // (dK^T partials in kv, dV^T in qd0 / qd1: ND 16 64 floats per wave)
  constexpr int RW = ND * 16 * 64;
  float* rdk = (float*)kv + kg * RW;
  float* rdv = (float*)(kg < 2 ? qd0 : qd1) + (kg & 1) * RW;
  if (m == 1) {
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
      for (int j = 0; j < 16; j += 4) {
        *(f32x4*)(rdk + (dt * 16 + j) * 64 + lane * 4) = f32x4{dk[dt][j], dk[dt][j + 1], dk[dt][j + 2], dk[dt][j + 3]};
        *(f32x4*)(rdv + (dt * 16 + j) * 64 + lane * 4) = f32x4{dv[dt][j], dv[dt][j + 1], dv[dt][j + 2], dv[dt][j + 3]};
      }
  }
  __syncthreads();
  if (m == 1) return;
#pragma unroll
  for (int dt = 0; dt < ND; ++dt)
#pragma unroll
    for (int j = 0; j < 16; j += 4) {
      const f32x4 a = *(const f32x4*)(rdk + (dt * 16 + j) * 64 + lane * 4);
      const f32x4 c = *(const f32x4*)(rdv + (dt * 16 + j) * 64 + lane * 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        dk[dt][j + i] += a[i];
        dv[dt][j + i] += c[i];
      }
    }
  // store: lane owns key `mykey`, d rows 32dt + 8g + 4hh + (0..3)
  bf16_t* dkr = dK + koff + (int64_t)mykey * D;
  bf16_t* dvr = dV + koff + (int64_t)mykey * D;
  float ksc = scale;
  if constexpr (ROPE) {  // rotate dK back; dK / dV go to the k / v parts of d(qkv) row (b, mykey)
    rope_bwd_acc<D>(dk, cosv + (int64_t)mykey * (D / 2), sinv + (int64_t)mykey * (D / 2), hh, scale);
    bf16_t* row = dK + ((int64_t)b * S + mykey) * H3 * D;
    dkr = row + (H + hk) * D;
    dvr = row + (H + Hk + hk) * D;
    ksc = 1.f;
  }
#pragma unroll
  for (int dt = 0; dt < ND; ++dt)
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      uint2 a[2], c[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int g = 2 * k + u;
        a[u].x = pack2(dk[dt][4 * g + 0] * ksc, dk[dt][4 * g + 1] * ksc);
        a[u].y = pack2(dk[dt][4 * g + 2] * ksc, dk[dt][4 * g + 3] * ksc);
        c[u].x = pack2(dv[dt][4 * g + 0], dv[dt][4 * g + 1]);
        c[u].y = pack2(dv[dt][4 * g + 2], dv[dt][4 * g + 3]);
      }
      store_pair16(dkr, 32 * dt + 16 * k, hh, a[0], a[1]);
      store_pair16(dvr, 32 * dt + 16 * k, hh, c[0], c[1]);
    }
}

// Backward form: 1 = dS through HBM (default where S % 256 == 0: the
// Llama-3-8B step 987.9 -> 978.1 ms, profiles/r3_attn_ds), 0 = split (dQ
// recomputes S / dP; ragged S always).  TOA_ATTN_BWD=split|ds, or
// toa_attn_set_bwd_variant (-1: back to the environment's choice).
static int g_bwd_variant = -1;
static int attn_bwd_variant() {
  if (g_bwd_variant < 0) {
    const char* e = getenv("TOA_ATTN_BWD");
    g_bwd_variant = (e && e[0] == 's' && e[1] == 'p') ? 0 : 1;
  }
  return g_bwd_variant;
}
extern "C" int toa_attn_set_bwd_variant(int v) {
  if (v < -1 || v > 1) return (int)hipErrorInvalidValue;
  g_bwd_variant = v;
  return 0;
}
// A/B instrumentation (scripts/attn_bwd_ab.py --timing): when set, the dS
// form's dK/dV kernel writes per-wave {issue cycles, step-end wait cycles,
// steps, 0} (u64) at tstat[(block * 8 + wave) * 4]
static unsigned long long* g_attn_tstat = nullptr;
extern "C" int toa_attn_set_bwd_timing(void* tstat) {
  g_attn_tstat = (unsigned long long*)tstat;
  return 0;
}
// dK / dV of the dS form on the assembly kernel (csrc/asm/attn_bwd_gen.py, host
// side csrc/hip/gemm_asm.hip): D = 128, the default there.  TOA_ATTN_DKDV=hip,
// or toa_attn_set_dkdv_variant(0), keeps attn_bwd_dkdv_ds_kernel (A/B, tests);
// 1 forces the assembly kernel, -1 returns to the environment's choice.
extern "C" int toa_attn_dkdv_asm(const bf16_t* q, const bf16_t* k, const bf16_t* v, const bf16_t* dout,
                                 const float* nlse2, const float* ndelta, bf16_t* dk, bf16_t* dv, bf16_t* ds, int B,
                                 int H, int Hk, int S, int D, float scale, int flags, const float* cosv,
                                 const float* sinv, int H3, hipStream_t stream);
static int g_dkdv_variant = -1;
extern "C" int toa_attn_set_dkdv_variant(int v) {
  if (v < -1 || v > 1) return (int)hipErrorInvalidValue;
  g_dkdv_variant = v;
  return 0;
}
static bool attn_dkdv_asm_on() {
  static const bool env_on = [] {
    const char* e = getenv("TOA_ATTN_DKDV");
    return !(e && strcmp(e, "hip") == 0);
  }();
  return g_dkdv_variant == 1 || (g_dkdv_variant < 0 && env_on);
}

template <int D, bool ROPE>
static void dkdv_ds_launch(hipStream_t stream, const bf16_t* q, const bf16_t* k, const bf16_t* v, const bf16_t* dout,
                           const float* nlse2, const float* delta, bf16_t* dk, bf16_t* dv, bf16_t* ds, int B, int H,
                           int Hk, int S, float scale, int o_bshd, const float* cosv, const float* sinv, int H3) {
  if (D == 128 && !g_attn_tstat && attn_dkdv_asm_on()) {
    // a refused shape (never one the dS form takes) falls through to the HIP kernel
    if (toa_attn_dkdv_asm(q, k, v, dout, nlse2, delta, dk, dv, ds, B, H, Hk, S, D, scale, o_bshd | (ROPE ? 2 : 0),
                          cosv, sinv, H3, stream) == 0)
      return;
  }
  const dim3 grid((S / 128) * B * Hk), block(512);
  if (g_attn_tstat)
    hipLaunchKernelGGL((attn_bwd_dkdv_ds_kernel<D, ROPE, true>), grid, block, 0, stream, q, k, v, dout, nlse2, delta,
                       dk, dv, ds, B, H, Hk, S, scale, scale * LOG2E, o_bshd, cosv, sinv, H3, g_attn_tstat);
  else
    hipLaunchKernelGGL((attn_bwd_dkdv_ds_kernel<D, ROPE>), grid, block, 0, stream, q, k, v, dout, nlse2, delta, dk,
                       dv, ds, B, H, Hk, S, scale, scale * LOG2E, o_bshd, cosv, sinv, H3, nullptr);
}
static bool attn_bwd_uses_ds(int S) { return attn_bwd_variant() >= 1 && S % FWD_QB == 0; }
// [dS blocks][-lse log2e rows]; the -delta rows go to the caller's delta buffer
static int64_t attn_ds_blocks_bytes(int B, int H, int S) {
  const int64_t nb = S / 32;
  return (int64_t)B * H * (nb * (nb + 1) / 2) * 2048;
}
static int64_t attn_ds_bytes(int B, int H, int S) {
  return attn_ds_blocks_bytes(B, H, S) + (int64_t)B * H * S * 4 + 2048;
}
// Workspace toa_attn_bwd needs (its `ws` argument) under the current form; 0 = none.
extern "C" int64_t toa_attn_bwd_ws_bytes(int B, int H, int S, int D) {
  (void)D;
  return attn_bwd_uses_ds(S) ? attn_ds_bytes(B, H, S) : 0;
}

template <int D, bool TAIL>
static void attn_set_lds_limits() {
  static bool done = false;
  if (done) return;
  (void)hipFuncSetAttribute((const void*)attn_fwd_kernel<D, TAIL>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            4 * AG<D>::TILEB);
  (void)hipFuncSetAttribute((const void*)attn_bwd_dkdv_kernel<D, TAIL>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            DKV<D>::LDS);
  (void)hipFuncSetAttribute((const void*)attn_bwd_dq_kernel<D, TAIL>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            4 * AG<D>::TILEB);
  done = true;
}

// Forward form: 1 = LDS-DMA staged K/V (where S % 256 == 0: 0.868 -> 0.811
// ms at the bench shape, bit-identical, profiles/r3_attn_ds), 0 = register
// staged (ragged S always), 2 = the assembly kernel (csrc/asm/attn_gen.py;
// D = 128, S % 256 == 0 -- the default there unless TOA_ATTN_FWD=hip).
// toa_attn_set_fwd_variant pins a form for in-process tests / A/B (-1: back
// to the default).
static int g_fwd_variant = -1;
static int attn_fwd_variant() { return g_fwd_variant == 0 ? 0 : 1; }
extern "C" int toa_attn_set_fwd_variant(int v) {
  if (v < -1 || v > 2) return (int)hipErrorInvalidValue;
  g_fwd_variant = v;
  return 0;
}

template <int D, bool TAIL>
static int attn_fwd_launch(const bf16_t* q, const bf16_t* k, const bf16_t* v, bf16_t* o, float* lse, int B, int H,
                           int Hk, int S, int o_bshd, float scale, hipStream_t stream) {
  attn_set_lds_limits<D, TAIL>();
  const int nqb = (S + FWD_QB - 1) / FWD_QB;
  if constexpr (!TAIL) {
    if (attn_fwd_variant() == 1) {
      hipLaunchKernelGGL((attn_fwd_gl_kernel<D>), dim3(nqb * H * B), dim3(64 * FWD_WAVES), 0, stream, q, k, v, o, lse,
                         B, H, Hk, S, scale * LOG2E, o_bshd);
      return (int)hipGetLastError();
    }
  }
  hipLaunchKernelGGL((attn_fwd_kernel<D, TAIL>), dim3(nqb * H * B), dim3(64 * FWD_WAVES), 4 * AG<D>::TILEB, stream, q, k, v,
                     o, lse, B, H, Hk, S, scale * LOG2E, o_bshd);
  return (int)hipGetLastError();
}

template <int D, bool TAIL>
static int attn_bwd_launch(const bf16_t* q, const bf16_t* k, const bf16_t* v, const bf16_t* o, const bf16_t* dout,
                           const float* lse, float* delta, void* ws, bf16_t* dq, bf16_t* dk, bf16_t* dv, int B, int H,
                           int Hk, int S, int o_bshd, float scale, hipStream_t stream) {
  attn_set_lds_limits<D, TAIL>();
  if constexpr (!TAIL) {
    if (attn_bwd_uses_ds(S)) {
      if (ws == nullptr) return (int)hipErrorInvalidValue;
      bf16_t* ds = (bf16_t*)ws;
      float* nlse2 = (float*)((char*)ws + attn_ds_blocks_bytes(B, H, S));
      const int rows = B * H * S;
      hipLaunchKernelGGL((attn_delta_kernel<D>), dim3((rows + 256 / (D / 8) - 1) / (256 / (D / 8))), dim3(256), 0,
                         stream, o, dout, lse, delta, nlse2, rows, H, S, o_bshd);
      dkdv_ds_launch<D, false>(stream, q, k, v, dout, nlse2, delta, dk, dv, ds, B, H, Hk, S, scale, o_bshd, nullptr,
                               nullptr, 0);
      hipLaunchKernelGGL((attn_bwd_dqg_kernel<D>), dim3((S / FWD_QB) * H * B), dim3(512), 0, stream, k, ds, dq, B, H,
                         Hk, S, scale, nullptr, nullptr, 0);
      return (int)hipGetLastError();
    }
  }
  // dQ first: it also computes delta = rowsum(dO * O), which dK/dV then reads
  hipLaunchKernelGGL((attn_bwd_dq_kernel<D, TAIL>), dim3(((S + FWD_QB - 1) / FWD_QB) * H * B), dim3(64 * FWD_WAVES),
                     4 * AG<D>::TILEB, stream, q, k, v, dout, o, lse, delta, dq, B, H, Hk, S, scale, scale * LOG2E,
                     o_bshd);
  hipLaunchKernelGGL((attn_bwd_dkdv_kernel<D, TAIL>), dim3(((S + 127) / 128) * B * Hk), dim3(512), DKV<D>::LDS, stream,
                     q, k, v, dout, lse, delta, dk, dv, B, H, Hk, S, scale, scale * LOG2E, o_bshd);
  return (int)hipGetLastError();
}

static bool attn_shape_ok(int B, int H, int Hk, int S, int D, int flags) {
  return (D == 64 || D == 128) && B > 0 && S > 0 && Hk > 0 && H % Hk == 0 && (flags & 1);
}

// The assembly forward (csrc/asm/attn_gen.py, host side csrc/hip/gemm_asm.hip)
// takes D = 128, S % 256 == 0; TOA_ATTN_FWD=hip keeps the HIP kernel (A/B).
extern "C" int toa_attn_fwd_asm(const bf16_t* q, const bf16_t* k, const bf16_t* v, bf16_t* o, float* lse, int B,
                                int H, int Hk, int S, int D, int flags, float scale, hipStream_t stream);
static bool attn_fwd_asm_on() {
  static const bool env_on = [] {
    const char* e = getenv("TOA_ATTN_FWD");
    return !(e && strcmp(e, "hip") == 0);
  }();
  return g_fwd_variant == 2 || (g_fwd_variant < 0 && env_on);
}

// flags: bit 0 causal (required), bit 1 O / dO in [B, S, H, D] (else [B, H, S, D]).
extern "C" int toa_attn_fwd(const bf16_t* q, const bf16_t* k, const bf16_t* v, bf16_t* o, float* lse, int B, int H,
                            int Hk, int S, int D, int flags, float scale, hipStream_t stream) {
  if (!attn_shape_ok(B, H, Hk, S, D, flags)) return (int)hipErrorInvalidValue;
  if (D == 128 && S % 256 == 0 && attn_fwd_asm_on()) {
    // the assembly launcher refuses (hipErrorInvalidValue) what it cannot
    // run -- unaligned q/k/v/o, 32-bit size limits, a module that did not
    // load -- before touching the stream: those inputs take the HIP kernel,
    // as the dK/dV path does (dkdv_ds_launch)
    const int rc = toa_attn_fwd_asm(q, k, v, o, lse, B, H, Hk, S, D, flags, scale, stream);
    if (rc != (int)hipErrorInvalidValue) return rc;
  }
  const int o_bshd = (flags >> 1) & 1;
  // S % 256 == 0: every 256-row block and 64-key tile is full, no clamping
  const bool tail = S % FWD_QB != 0;
#define TOA_ATTN_FWD(DD, TT) attn_fwd_launch<DD, TT>(q, k, v, o, lse, B, H, Hk, S, o_bshd, scale, stream)
#ifdef TOA_ATTN_D128_ONLY
  if (D != 128) return (int)hipErrorInvalidValue;
  return tail ? TOA_ATTN_FWD(128, true) : TOA_ATTN_FWD(128, false);
#else
  if (D == 128) return tail ? TOA_ATTN_FWD(128, true) : TOA_ATTN_FWD(128, false);
  return tail ? TOA_ATTN_FWD(64, true) : TOA_ATTN_FWD(64, false);
#endif
#undef TOA_ATTN_FWD
}

// ws: toa_attn_bwd_ws_bytes(B, H, S, D) bytes (may be null when that is 0); dq/dk/dv bf16.
extern "C" int toa_attn_bwd(const bf16_t* q, const bf16_t* k, const bf16_t* v, const bf16_t* o, const bf16_t* dout,
                            const float* lse, float* delta, void* ws, bf16_t* dq, bf16_t* dk, bf16_t* dv, int B,
                            int H, int Hk, int S, int D, int flags, float scale, hipStream_t stream) {
  if (!attn_shape_ok(B, H, Hk, S, D, flags)) return (int)hipErrorInvalidValue;
  const int o_bshd = (flags >> 1) & 1;
  const bool tail = S % FWD_QB != 0;
#define TOA_ATTN_BWD(DD, TT) \
  attn_bwd_launch<DD, TT>(q, k, v, o, dout, lse, delta, ws, dq, dk, dv, B, H, Hk, S, o_bshd, scale, stream)
#ifdef TOA_ATTN_D128_ONLY
  if (D != 128) return (int)hipErrorInvalidValue;
  return tail ? TOA_ATTN_BWD(128, true) : TOA_ATTN_BWD(128, false);
#else
  if (D == 128) return tail ? TOA_ATTN_BWD(128, true) : TOA_ATTN_BWD(128, false);
  return tail ? TOA_ATTN_BWD(64, true) : TOA_ATTN_BWD(64, false);
#endif
#undef TOA_ATTN_BWD
}

// Fused RoPE + attention backward (the dS form only: S % 256 == 0, packed
// K/V = one copy per kv head): d(qkv) [B*S, (H + 2 Hk) * D] straight from the
// dQ GEMM's and the dK/dV kernel's epilogues, rotated back with cos / sin
// [S, D / 2] -- no dq / dk / dv tensors and no RoPE backward pass (the
// inverse of toa_rope_fwd).  hipErrorNotSupported when the dS form is off or
// the shape is not one it takes; the caller then runs toa_attn_bwd +
// toa_rope_bwd.  ws: toa_attn_bwd_ws_bytes(B, H, S, D) bytes.
// -lse log2(e) rows alone: the delta pass's other output, when the delta rows
// came from the output projection's data-gradient GEMM (toa_gemm_asm_delta).
__global__ __launch_bounds__(256) void attn_nlse2_kernel(const float* __restrict__ LSE, float* __restrict__ NLSE2,
                                                         int rows) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < rows) NLSE2[i] = -(LSE[i] * LOG2E);
}

// flags bit 2: `delta` already holds the -delta rows (toa_gemm_asm_delta).
extern "C" int toa_attn_bwd_rope(const bf16_t* q, const bf16_t* k, const bf16_t* v, const bf16_t* o,
                                 const bf16_t* dout, const float* lse, float* delta, void* ws, const float* cosv,
                                 const float* sinv, bf16_t* dqkv, int B, int H, int Hk, int S, int D, int flags,
                                 float scale, hipStream_t stream) {
  if (!attn_shape_ok(B, H, Hk, S, D, flags)) return (int)hipErrorInvalidValue;
  if (!attn_bwd_uses_ds(S)) return (int)hipErrorNotSupported;
  if (ws == nullptr || dqkv == nullptr || cosv == nullptr || sinv == nullptr) return (int)hipErrorInvalidValue;
  const int o_bshd = (flags >> 1) & 1;
  const int H3 = H + 2 * Hk;
  bf16_t* ds = (bf16_t*)ws;
  float* nlse2 = (float*)((char*)ws + attn_ds_blocks_bytes(B, H, S));
  const int rows = B * H * S;
#define TOA_ATTN_BWD_ROPE(DD)                                                                                    \
  do {                                                                                                           \
    if (flags & 4)                                                                                               \
      hipLaunchKernelGGL(attn_nlse2_kernel, dim3((rows + 255) / 256), dim3(256), 0, stream, lse, nlse2, rows);   \
    else                                                                                                         \
      hipLaunchKernelGGL((attn_delta_kernel<DD>), dim3((rows + 256 / (DD / 8) - 1) / (256 / (DD / 8))),          \
                         dim3(256), 0, stream, o, dout, lse, delta, nlse2, rows, H, S, o_bshd);                  \
    dkdv_ds_launch<DD, true>(stream, q, k, v, dout, nlse2, delta, dqkv, dqkv, ds, B, H, Hk, S, scale, o_bshd,  \
                             cosv, sinv, H3);                                                                   \
    hipLaunchKernelGGL((attn_bwd_dqg_kernel<DD, true>), dim3((S / FWD_QB) * H * B), dim3(512), 0, stream, k, ds, \
                       dqkv, B, H, Hk, S, scale, cosv, sinv, H3);                                               \
  } while (0)
#ifdef TOA_ATTN_D128_ONLY
  if (D != 128) return (int)hipErrorInvalidValue;
  TOA_ATTN_BWD_ROPE(128);
#else
  if (D == 128)
    TOA_ATTN_BWD_ROPE(128);
  else
    TOA_ATTN_BWD_ROPE(64);
#endif
#undef TOA_ATTN_BWD_ROPE
  return (int)hipGetLastError();
}
