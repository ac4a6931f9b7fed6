// Causal flash attention for gfx950 (bf16 in/out, fp32 accumulate), with
// native GQA (K/V stay packed per kv-head; no repeat_interleave copies).
//
// Layouts: q [B, H, S, D], o/dO [B, H, S, D] or [B, S, H, D] (flag bit 1),
// k/v [B, Hk, S, D], lse [B, H, S] (natural log), D = 128.  Forward / dQ:
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
// Backward = two kernels: dQ (which also computes delta = rowsum(dO*O)),
// then dK/dV (workgroup per 128-key block, sweeping the GQA group's query
// heads).  No float atomics: deterministic.
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

// LDS tile geometry: 64 keys x 128 d bf16 = 16 KB, rows of 256 B = 16 chunks of 16 B.
#define TK 64
#define ROWB 256

// K image: chunk c of row `key` stored at chunk position c ^ (key & 15)
__device__ __forceinline__ int k_off(int key, int chunk) { return key * ROWB + ((chunk ^ (key & 15)) << 4); }
// V image: chunk c of row `key` stored at chunk position c ^ ((key & 3) << 2)
__device__ __forceinline__ int v_off(int key, int chunk) { return key * ROWB + ((chunk ^ ((key & 3) << 2)) << 4); }

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

// Offset of row (b, h, s) of O / dO: [B, H, S, D] (head-major, like Q) or, with
// bshd, [B, S, H, D] -- the layout the output projection consumes, so the
// model needs no transpose copy of O forward or of dO backward.
__device__ __forceinline__ int64_t o_off(int b, int h, int s, int H, int S, int bshd) {
  return bshd ? (((int64_t)b * S + s) * H + h) * 128 : (((int64_t)b * H + h) * S + s) * 128;
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

template <int D>
__global__ __launch_bounds__(512, 1) void attn_fwd_kernel(const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K,
                                                          const bf16_t* __restrict__ V, bf16_t* __restrict__ O,
                                                          float* __restrict__ LSE, int B, int H, int Hk, int S,
                                                          float scale_log2, int o_bshd) {
  static_assert(D == 128, "D=128 path");
  extern __shared__ __attribute__((aligned(16))) char smem[];  // 2 x (K 16KB + V 16KB)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int nqb = (S + FWD_QB - 1) / FWD_QB;
  int qb, h, b;
  fwd_block_coords(blockIdx.x, nqb, B, H, Hk, &qb, &h, &b);
  const int hk = h / (H / Hk);
  const int64_t qoff = ((int64_t)(b * H + h) * S) * D;
  const int64_t koff = ((int64_t)(b * Hk + hk) * S) * D;
  const int q0 = qb * FWD_QB + wave * 32;  // first row of this wave
  const bool live = q0 < S;                // S % 128 == 0: a wave is all in or all out
  const int myq = q0 + r;                  // the query row this lane owns
  const int kend = min(S, (qb + 1) * FWD_QB);
  const int ntiles = kend / TK;
  const int t_diag = live ? (q0 + 31) / TK : -1;  // this wave's last (masked) tile

  // Q fragments: Q[myq][16s + 8hh .. +7], s = 0..7
  bf16x8 qf[8];
#pragma unroll
  for (int s = 0; s < 8; ++s)
    qf[s] = live ? as_bf16x8(ld16(Q + qoff + (int64_t)myq * D + 16 * s + 8 * hh)) : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};

  // lane-constant LDS read offsets (buffer / half / k-step parts are immediates)
  // K: k_off(32n + r, 2s + hh) = r*256 + ((2s ^ x) << 4) + 8192 n,  x = hh ^ (r & 15)
  int kro[8];
  {
    const int x = hh ^ (r & 15);
#pragma unroll
    for (int s = 0; s < 8; ++s) kro[s] = r * ROWB + (((2 * s) ^ x) << 4);
  }
  // V^T: key = 32n + 16s' + 4hh + qq (+8), column block 32dt + 16(g&1) + 4pp
  int vro[4];
  {
    const int g = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
      vro[dt] = (4 * hh + qq) * ROWB + ((4 * (dt ^ qq) + 2 * (g & 1) + (pp >> 1)) << 4) + (pp & 1) * 8;
  }

  f32x16 acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[i][j] = 0.f;
  float m_run = -INFINITY, l_run = 0.f;

  // staging: 512 threads x (2 x 16 B of K + 2 x 16 B of V) = one 64-key tile
  u32x4 stk[2], stv[2];
  auto gload = [&](int t) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = tid + 512 * i;
      const int key = e >> 4, c = e & 15;
      const int64_t gidx = koff + (int64_t)(t * TK + key) * D + c * 8;
      stk[i] = ld16(K + gidx);
      stv[i] = ld16(V + gidx);
    }
  };
  auto swrite = [&](int buf) {
    char* kb = smem + buf * 32768;
    char* vb = kb + 16384;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = tid + 512 * i;
      const int key = e >> 4, c = e & 15;
      *(u32x4*)(kb + k_off(key, c)) = stk[i];
      *(u32x4*)(vb + v_off(key, c)) = stv[i];
    }
  };

  auto compute = [&](int t, int buf, bool mask) {
    const char* kb = smem + buf * 32768;
    const char* vb = kb + 16384;
    // ---- S^T = K Q^T : two 32-key halves (first MFMA of each chain starts from 0)
    f32x16 sc[2];
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const f32x16 z = {};
      sc[n] = mfma32(as_bf16x8(*(const u32x4*)(kb + kro[0] + 8192 * n)), qf[0], z);
#pragma unroll
      for (int s = 1; s < 8; ++s)
        sc[n] = mfma32(as_bf16x8(*(const u32x4*)(kb + kro[s] + 8192 * n)), qf[s], sc[n]);
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
    float mx = sc[0][0];
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int j = 0; j < 16; ++j) mx = fmaxf(mx, sc[n][j]);
    mx = xhalf_max(mx) * scale_log2;
    // T13: rescale O / l only when some row's max grew by more than THR
    if (__any(mx > m_run + RESCALE_THR)) {
      const float m_new = fmaxf(m_run, mx);
      const float alpha = (m_run == -INFINITY) ? 0.f : EXP2(m_run - m_new);
      l_run *= alpha;
      m_run = m_new;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[i][j] *= alpha;
    }
    // ---- P = exp2(s*c - m) packed straight into the PV B operand
    float ls = 0.f;
    uint32_t pw[2][8];
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int j = 0; j < 16; j += 2) {
        const float p0 = EXP2(fmaf(sc[n][j], scale_log2, -m_run));
        const float p1 = EXP2(fmaf(sc[n][j + 1], scale_log2, -m_run));
        ls += p0 + p1;
        pw[n][j >> 1] = cvt_pk(p0, p1);
      }
    l_run += ls;
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
        for (int dt = 0; dt < 4; ++dt) {
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
  for (int s = 0; s < 8; ++s) asm volatile("" ::"v"(qf[s]));
  __syncthreads();
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
  bf16_t* orow = O + o_off(b, h, myq, H, S, o_bshd);
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d = 32 * dt + 8 * g + 4 * hh;
      uint2 w;
      w.x = cvt_pk(acc[dt][4 * g + 0] * inv, acc[dt][4 * g + 1] * inv);
      w.y = cvt_pk(acc[dt][4 * g + 2] * inv, acc[dt][4 * g + 3] * inv);
      *(uint2*)(orow + d) = w;
    }
  if (hh == 0) LSE[(int64_t)(b * H + h) * S + myq] = (m_run + log2f(l_tot)) * 0.6931471805599453f;
}

// One image for row reads (ds_read_b128, 32x32x16 A/B operand) AND
// transposed reads (ds_read_b64_tr_b16): guide T10 layout (b),
// chunk' = chunk ^ (((row & 3) << 2) | ((row >> 2) & 3)).
__device__ __forceinline__ int rt_off(int row, int chunk) {
  return row * ROWB + ((chunk ^ (((row & 3) << 2) | ((row >> 2) & 3))) << 4);
}

// A-operand fragment of X^T . Y where X is a row-major [rows][128] bf16 LDS
// image read transposed: lane (r, hh) gets X[rows rb + 4hh + (0..3)][32dt + r]
// and X[rows rb + 8 + 4hh + (0..3)][32dt + r]  (the permuted k order that
// matches a C-layout accumulator used as the B operand).
__device__ __forceinline__ bf16x8 tr_frag(const char* img, int rb, int dt, int lane) {
  const int g = lane >> 4, i16 = lane & 15, hh = lane >> 5;
  const int qq = i16 >> 2, pp = i16 & 3;
  const int col = 32 * dt + 16 * (g & 1) + 4 * pp;
  const int ra = rb + 4 * hh + qq;
  const bf16x4 a = tr_read(img, rt_off(ra, col >> 3) + (col & 7) * 2);
  const bf16x4 b = tr_read(img, rt_off(ra + 8, col >> 3) + (col & 7) * 2);
  bf16x8 f;
  f[0] = a[0]; f[1] = a[1]; f[2] = a[2]; f[3] = a[3];
  f[4] = b[0]; f[5] = b[1]; f[6] = b[2]; f[7] = b[3];
  return f;
}

__device__ __forceinline__ bf16x8 pack_frag(const f32x16& x, int s) {
  u32x4 w;
  w[0] = pack2(x[8 * s + 0], x[8 * s + 1]);
  w[1] = pack2(x[8 * s + 2], x[8 * s + 3]);
  w[2] = pack2(x[8 * s + 4], x[8 * s + 5]);
  w[3] = pack2(x[8 * s + 6], x[8 * s + 7]);
  return as_bf16x8(w);
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
#define DKV_QBUF (32768 + 512)
#define DKV_LDS (2 * DKV_QBUF + 65536)

__global__ __launch_bounds__(512, 1) void attn_bwd_dkdv_kernel(
    const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V,
    const bf16_t* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ DELTA,
    bf16_t* __restrict__ dK, bf16_t* __restrict__ dV, int B, int H, int Hk, int S, float scale,
    float scale_log2, int o_bshd) {
  // [Q/dO/lse/-delta buffer 0][buffer 1][K 32K][V 32K]
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* kimg = smem + 2 * DKV_QBUF;
  char* vimg = kimg + 32768;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int kg = wave & 3, m = wave >> 2;
  // heaviest (most query tiles) key blocks first; (b, hk) fastest
  const int nkb = S / 128;
  const int kb = nkb - 1 - (int)(blockIdx.x / (B * Hk));
  const int bh = blockIdx.x % (B * Hk);
  const int b = bh / Hk, hk = bh % Hk;
  const int rep = H / Hk;
  const int kw = kb * 128 + kg * 32;  // first key of this wave
  const int mykey = kw + r;
  const int64_t koff = ((int64_t)(b * Hk + hk) * S) * 128;

  // K / V of the block -> LDS (rt_off image: row reads give the B operands)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int e = tid + 512 * i;
    const int row = e >> 4, c = e & 15;
    const int64_t g = koff + (int64_t)(kb * 128 + row) * 128 + c * 8;
    *(u32x4*)(kimg + rt_off(row, c)) = ld16(K + g);
    *(u32x4*)(vimg + rt_off(row, c)) = ld16(V + g);
  }
  f32x16 dk[4], dv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 16; ++j) { dk[i][j] = 0.f; dv[i][j] = 0.f; }

  int rro[8], tro[4], tro8[4];
  {
    const int swz = ((r & 3) << 2) | ((r >> 2) & 3);
#pragma unroll
    for (int s = 0; s < 8; ++s) rro[s] = r * ROWB + (((2 * s + hh) ^ swz) << 4);
    const int g = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
    const int lo = 2 * (g & 1) + (pp >> 1);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      tro[dt] = (4 * hh + qq) * ROWB + ((4 * (dt ^ qq) + (lo ^ hh)) << 4) + (pp & 1) * 8;
      tro8[dt] = (4 * hh + qq + 8) * ROWB + ((4 * (dt ^ qq) + (lo ^ ((hh + 2) & 3))) << 4) + (pp & 1) * 8;
    }
  }

  const int qt0 = (kb * 128) / 64;  // first causal 64-row query tile
  const int nqt = S / 64 - qt0;
  const int total = nqt * rep;
  u32x4 sq[2], sdo[2];
  float slse = 0.f, sdel = 0.f;
  auto gload = [&](int it) {
    const int hq = hk * rep + it / nqt;
    const int qt = qt0 + it % nqt;
    const int64_t qoff = ((int64_t)(b * H + hq) * S) * 128;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = tid + 512 * i;
      const int row = e >> 4, c = e & 15;
      const int64_t g = qoff + (int64_t)(qt * 64 + row) * 128 + c * 8;
      sq[i] = ld16(Q + g);
      sdo[i] = ld16(dO + o_off(b, hq, qt * 64 + row, H, S, o_bshd) + c * 8);
    }
    if (tid < 64) {
      const int64_t li = (int64_t)(b * H + hq) * S + qt * 64 + tid;
      slse = LSE[li];  // scaled at swrite: consuming it here would wait on the whole prefetch
      sdel = DELTA[li];
    }
  };
  auto swrite = [&](int buf) {
    char* qb_ = smem + buf * DKV_QBUF;
    char* ob = qb_ + 16384;
    float* lb = (float*)(qb_ + 32768);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = tid + 512 * i;
      const int row = e >> 4, c = e & 15;
      *(u32x4*)(qb_ + rt_off(row, c)) = sq[i];
      *(u32x4*)(ob + rt_off(row, c)) = sdo[i];
    }
    if (tid < 64) {
      lb[tid] = slse * LOG2E;
      lb[64 + tid] = -sdel;
    }
  };

  auto subtile = [&](int buf, int qs, bool mask) {
    const char* qi = smem + buf * DKV_QBUF;
    const char* oi = qi + 16384;
    const float* lb = (const float*)(qi + 32768);
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
    for (int s = 0; s < 8; ++s) {
      const bf16x8 qa = as_bf16x8(*(const u32x4*)(qi + rro[s] + 8192 * m));
      const bf16x8 kf = as_bf16x8(*(const u32x4*)(kimg + rro[s] + 8192 * kg));
      sc = mfma32(qa, kf, sc);
      const bf16x8 oa = as_bf16x8(*(const u32x4*)(oi + rro[s] + 8192 * m));
      const bf16x8 vf = as_bf16x8(*(const u32x4*)(vimg + rro[s] + 8192 * kg));
      dp = mfma32(oa, vf, dp);
    }
    uint32_t pw[8], sw[8];
#pragma unroll
    for (int j = 0; j < 16; j += 2) {
      const f32x4 l4 = *(const f32x4*)(lb + 32 * m + 8 * (j >> 2) + 4 * hh);
      float p0 = EXP2(fmaf(sc[j], scale_log2, -l4[j & 3]));
      float p1 = EXP2(fmaf(sc[j + 1], scale_log2, -l4[(j + 1) & 3]));
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
      for (int dt = 0; dt < 4; ++dt) {
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
  float* red = (float*)smem;  // 4 waves x 2 x 64 lanes x 64 floats = 128 KB, Q/dO/K/V are dead
  if (m == 1) {
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int j = 0; j < 16; j += 4) {
        *(f32x4*)(red + ((kg * 2 + 0) * 64 * 64) + (dt * 16 + j) * 64 + lane * 4) =
            f32x4{dk[dt][j], dk[dt][j + 1], dk[dt][j + 2], dk[dt][j + 3]};
        *(f32x4*)(red + ((kg * 2 + 1) * 64 * 64) + (dt * 16 + j) * 64 + lane * 4) =
            f32x4{dv[dt][j], dv[dt][j + 1], dv[dt][j + 2], dv[dt][j + 3]};
      }
  }
  __syncthreads();
  if (m == 1) return;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int j = 0; j < 16; j += 4) {
      const f32x4 a = *(const f32x4*)(red + ((kg * 2 + 0) * 64 * 64) + (dt * 16 + j) * 64 + lane * 4);
      const f32x4 c = *(const f32x4*)(red + ((kg * 2 + 1) * 64 * 64) + (dt * 16 + j) * 64 + lane * 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        dk[dt][j + i] += a[i];
        dv[dt][j + i] += c[i];
      }
    }
  // store: lane owns key `mykey`, d rows 32dt + 8g + 4hh + (0..3)
  bf16_t* dkr = dK + koff + (int64_t)mykey * 128;
  bf16_t* dvr = dV + koff + (int64_t)mykey * 128;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d = 32 * dt + 8 * g + 4 * hh;
      uint2 a, c;
      a.x = pack2(dk[dt][4 * g + 0] * scale, dk[dt][4 * g + 1] * scale);
      a.y = pack2(dk[dt][4 * g + 2] * scale, dk[dt][4 * g + 3] * scale);
      c.x = pack2(dv[dt][4 * g + 0], dv[dt][4 * g + 1]);
      c.y = pack2(dv[dt][4 * g + 2], dv[dt][4 * g + 3]);
      *(uint2*)(dkr + d) = a;
      *(uint2*)(dvr + d) = c;
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
__global__ __launch_bounds__(512, 1) void attn_bwd_dq_kernel(
    const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V,
    const bf16_t* __restrict__ dO, const bf16_t* __restrict__ O, const float* __restrict__ LSE,
    float* __restrict__ DELTA, bf16_t* __restrict__ dQ, int B, int H, int Hk, int S, float scale, float scale_log2,
    int o_bshd) {
  extern __shared__ __attribute__((aligned(16))) char smem[];  // 2 x (K 16K + V 16K)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int nqb = (S + FWD_QB - 1) / FWD_QB;
  int qb, h, b;
  fwd_block_coords(blockIdx.x, nqb, B, H, Hk, &qb, &h, &b);
  const int hk = h / (H / Hk);
  const int64_t qoff = ((int64_t)(b * H + h) * S) * 128;
  const int64_t koff = ((int64_t)(b * Hk + hk) * S) * 128;
  const int q0 = qb * FWD_QB + wave * 32;
  const bool live = q0 < S;
  const int myq = q0 + r;
  const int kend = min(S, (qb + 1) * FWD_QB);
  const int ntiles = kend / TK;
  const int t_diag = live ? (q0 + 31) / TK : -1;

  bf16x8 qf[8], of[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    qf[s] = live ? as_bf16x8(ld16(Q + qoff + (int64_t)myq * 128 + 16 * s + 8 * hh)) : bf16x8{};
    of[s] = live ? as_bf16x8(ld16(dO + o_off(b, h, myq, H, S, o_bshd) + 16 * s + 8 * hh)) : bf16x8{};
  }
  const float lse2 = live ? LSE[(int64_t)(b * H + h) * S + myq] * LOG2E : 0.f;
  // delta = rowsum(dO * O), computed here (the lane already holds its half of
  // the dO row) and published for the dK/dV kernel that runs next
  float del = 0.f;
  if (live) {
    float part = 0.f;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      float a[8], g[8];
      unpack8(ld16(O + o_off(b, h, myq, H, S, o_bshd) + 16 * s + 8 * hh), a);
      unpack8(__builtin_bit_cast(u32x4, of[s]), g);
#pragma unroll
      for (int j = 0; j < 8; ++j) part = fmaf(a[j], g[j], part);
    }
    del = xhalf_sum(part);
    if (hh == 0) DELTA[(int64_t)(b * H + h) * S + myq] = del;
  }
  f32x16 acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[i][j] = 0.f;

  int rro[8], tro[4], tro8[4];
  {
    const int swz = ((r & 3) << 2) | ((r >> 2) & 3);
#pragma unroll
    for (int s = 0; s < 8; ++s) rro[s] = r * ROWB + (((2 * s + hh) ^ swz) << 4);
    const int g = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
    const int lo = 2 * (g & 1) + (pp >> 1);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      tro[dt] = (4 * hh + qq) * ROWB + ((4 * (dt ^ qq) + (lo ^ hh)) << 4) + (pp & 1) * 8;
      tro8[dt] = (4 * hh + qq + 8) * ROWB + ((4 * (dt ^ qq) + (lo ^ ((hh + 2) & 3))) << 4) + (pp & 1) * 8;
    }
  }

  u32x4 stk[2], stv[2];
  auto gload = [&](int t) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = tid + 512 * i;
      const int key = e >> 4, c = e & 15;
      const int64_t gidx = koff + (int64_t)(t * TK + key) * 128 + c * 8;
      stk[i] = ld16(K + gidx);
      stv[i] = ld16(V + gidx);
    }
  };
  auto swrite = [&](int buf) {
    char* kb = smem + buf * 32768;
    char* vb = kb + 16384;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = tid + 512 * i;
      const int key = e >> 4, c = e & 15;
      *(u32x4*)(kb + rt_off(key, c)) = stk[i];
      *(u32x4*)(vb + rt_off(key, c)) = stv[i];
    }
  };
  auto compute = [&](int t, int buf, bool mask) {
    const char* kb = smem + buf * 32768;
    const char* vb = kb + 16384;
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const f32x16 z = {};
      f32x16 sc = mfma32(as_bf16x8(*(const u32x4*)(kb + rro[0] + 8192 * n)), qf[0], z);
      f32x16 dp = mfma32(as_bf16x8(*(const u32x4*)(vb + rro[0] + 8192 * n)), of[0], z);
#pragma unroll
      for (int s = 1; s < 8; ++s) {
        sc = mfma32(as_bf16x8(*(const u32x4*)(kb + rro[s] + 8192 * n)), qf[s], sc);
        dp = mfma32(as_bf16x8(*(const u32x4*)(vb + rro[s] + 8192 * n)), of[s], dp);
      }
      uint32_t sw[8];
#pragma unroll
      for (int j = 0; j < 16; j += 2) {
        float p0 = EXP2(fmaf(sc[j], scale_log2, -lse2));
        float p1 = EXP2(fmaf(sc[j + 1], scale_log2, -lse2));
        if (mask) {
          const int key = t * TK + 32 * n + (j & 3) + 8 * (j >> 2) + 4 * hh;
          if (key > myq) p0 = 0.f;
          if (key + 1 > myq) p1 = 0.f;
        }
        sw[j >> 1] = pack2(p0 * (dp[j] - del), p1 * (dp[j + 1] - del));
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        u32x4 w;
#pragma unroll
        for (int i = 0; i < 4; ++i) w[i] = sw[4 * s2 + i];
        const bf16x8 sb = as_bf16x8(w);
        const int rb = 32 * n + 16 * s2;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
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
  for (int s = 0; s < 8; ++s) asm volatile("" ::"v"(qf[s]), "v"(of[s]));  // retire resident loads (see fwd)
  asm volatile("" ::"v"(lse2), "v"(del));
  __syncthreads();
  int t = 0;
  for (; t + 1 < ntiles; t += 2) {
    step(t, 0);
    step(t + 1, 1);
  }
  if (t < ntiles) step(t, 0);

  if (!live) return;
  bf16_t* qrow = dQ + qoff + (int64_t)myq * 128;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d = 32 * dt + 8 * g + 4 * hh;
      uint2 w;
      w.x = pack2(acc[dt][4 * g + 0] * scale, acc[dt][4 * g + 1] * scale);
      w.y = pack2(acc[dt][4 * g + 2] * scale, acc[dt][4 * g + 3] * scale);
      *(uint2*)(qrow + d) = w;
    }
}

static void attn_set_lds_limits() {
  static bool done = false;
  if (done) return;
  (void)hipFuncSetAttribute((const void*)attn_fwd_kernel<128>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
  (void)hipFuncSetAttribute((const void*)attn_bwd_dkdv_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, DKV_LDS);
  (void)hipFuncSetAttribute((const void*)attn_bwd_dq_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
  done = true;
}

// flags: bit 0 causal (required), bit 1 O / dO in [B, S, H, D] (else [B, H, S, D]).
extern "C" int toa_attn_fwd(const bf16_t* q, const bf16_t* k, const bf16_t* v, bf16_t* o, float* lse, int B, int H,
                            int Hk, int S, int D, int flags, float scale, hipStream_t stream) {
  if (D != 128 || S % 128 != 0 || H % Hk != 0 || !(flags & 1)) return (int)hipErrorInvalidValue;
  const int o_bshd = (flags >> 1) & 1;
  attn_set_lds_limits();
  const int nqb = (S + FWD_QB - 1) / FWD_QB;
  hipLaunchKernelGGL(attn_fwd_kernel<128>, dim3(nqb * H * B), dim3(64 * FWD_WAVES), 65536, stream, q, k, v, o, lse,
                     B, H, Hk, S, scale * LOG2E, o_bshd);
  return (int)hipGetLastError();
}

// dq_acc is unused (kept in the ABI for an atomic-dQ variant); dq/dk/dv bf16.
extern "C" int toa_attn_bwd(const bf16_t* q, const bf16_t* k, const bf16_t* v, const bf16_t* o, const bf16_t* dout,
                            const float* lse, float* delta, float* dq_acc, bf16_t* dq, bf16_t* dk, bf16_t* dv, int B,
                            int H, int Hk, int S, int D, int flags, float scale, hipStream_t stream) {
  (void)dq_acc;
  if (D != 128 || S % 128 != 0 || H % Hk != 0 || !(flags & 1)) return (int)hipErrorInvalidValue;
  const int o_bshd = (flags >> 1) & 1;
  attn_set_lds_limits();
  const int64_t rows = (int64_t)B * H * S;
  (void)rows;
  // dQ first: it also computes delta = rowsum(dO * O), which dK/dV then reads
  hipLaunchKernelGGL(attn_bwd_dq_kernel, dim3(((S + FWD_QB - 1) / FWD_QB) * H * B), dim3(64 * FWD_WAVES), 65536,
                     stream, q, k, v, dout, o, lse, delta, dq, B, H, Hk, S, scale, scale * LOG2E, o_bshd);
  hipLaunchKernelGGL(attn_bwd_dkdv_kernel, dim3((S / 128) * B * Hk), dim3(512), DKV_LDS, stream, q, k, v, dout, lse,
                     delta, dk, dv, B, H, Hk, S, scale, scale * LOG2E, o_bshd);
  return (int)hipGetLastError();
}
