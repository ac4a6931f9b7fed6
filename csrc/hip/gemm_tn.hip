// Forward / data-gradient GEMM on MFMA (the "TN" form) with fused epilogues:
//
//     C[M][N] = sum_k A[m][k] * B[n][k]          (bf16 in, fp32 accumulate)
//
// A = X [M][K] (row stride lda), B = W [N][K] (ldb): y = x W^T, and the data
// gradient on the transposed weight copy (ops/wt.py) has the same form.
// Both operands are contiguous along the reduction, so every MFMA operand
// fragment is ONE ds_read_b128 of a row (the weight-gradient kernel,
// wgrad.hip, needs two transposed reads per fragment).
//
//   workgroup: 8 waves (2 M x 4 N), tile 256 x 256, 32 k per phase, 4 LDS
//              stages filled by global_load_lds two phases ahead, the two
//              wave rows staggered by one barrier (guide §5 template)
//   wave:      128 x 64 of C = 8 x 4 v_mfma_f32_16x16x32_bf16 tiles
//   operands:  swapped (B fragment first): each lane's accumulator holds 4
//              consecutive n of one row m -> 8-byte stores
//   grid:      one workgroup per tile, not persistent: a collective kernel
//              on another stream takes CUs as tiles retire (parallel/zero.py,
//              profiles/r3_overlap) instead of waiting for the whole GEMM
//
// Epilogues (the element-wise work the Llama MLP does around these GEMMs):
//   TN_PLAIN        C (bf16)
//   TN_SWIGLU_FWD   gate|up projection: the workgroup's 256 columns are 128
//                   gate columns [c, c+128) and the SAME 128 up columns
//                   [F+c, F+c+128) (the B-row map below; W keeps its [gate |
//                   up] layout), each wave holding 32 gate + 32 up columns of
//                   the same 32 hidden units, so it writes gu (saved for
//                   backward) AND s = silu(gate) * up for the down projection
//                   -- no separate SwiGLU pass re-reading gu
//   TN_SWIGLU_BWD   data gradient of the down projection: C = ds is never
//                   stored; the epilogue reads gate / up from gu and writes
//                   dgu = [ds * up * silu'(gate) | ds * silu(gate)]
#include <hip/hip_runtime.h>

#include <cstdint>

#include "toa_common.h"

#define TN_BM 256
#define TN_BN 256
#define TN_BK 32                   // k per stage (one phase)
#define TN_ROWB 64                 // one LDS row = 32 bf16 of k
#define TN_TILE (TN_BM * TN_ROWB)  // 16 KiB per operand per stage
#define TN_STAGE (2 * TN_TILE)
#define TN_VMCNT0 0x0F70
#define TN_VMCNT4 0x0F74

enum { TN_PLAIN = 0, TN_SWIGLU_FWD = 1, TN_SWIGLU_BWD = 2 };

typedef __attribute__((ext_vector_type(8))) short tn_s16x8;

// Chunk c (16 B, 0..3) of LDS row r lives at chunk position c ^ tn_f(r).  A
// fragment read takes chunk (lane >> 4) of rows r0 + (lane & 15): with the XOR
// the 16 lanes of every ds_read_b128 lane group hit 16 distinct 16-byte bank
// slots (plain rows are 2-way).
__device__ __forceinline__ int tn_f(int r) { return ((r >> 3) & 1) << 1; }
__device__ __forceinline__ int tn_off(int r, int c) { return r * TN_ROWB + ((c ^ tn_f(r)) << 4); }

// 16x16x32 operand fragment of rows row0..row0+15, all 32 k of the stage:
// lane l gets image[row0 + (l & 15)][8 (l >> 4) .. +7].
__device__ __forceinline__ tn_s16x8 tn_frag(const char* img, int row0, int lane) {
  const int r = row0 + (lane & 15);
  return *(const tn_s16x8*)(img + tn_off(r, lane >> 4));
}

// B-row map: tile row t of column tile tn -> row of B.  Plain: tn * 256 + t.
// SwiGLU forward (f = F, the up half's offset): wave block w = t / 64 holds
// gate rows c + 32w .. +31 then the same up rows, c = tn * 128.
// (relative to the column tile's first row: tn * 256, or tn * 128 for SwiGLU)
__device__ __forceinline__ int tn_brow(int t, int f) {
  if (f == 0) return t;
  const int w = t >> 6, u = t & 63;
  return 32 * w + (u & 31) + (u >= 32 ? f : 0);
}

// Lane's source element offset (from the tile's first row) for staging LDS
// row t, chunk (lane & 3) of the image (the swizzle goes on the SOURCE: LDS-DMA
// writes lane-linearly, guide §5.4 rule 21); `src_row` = the row of the
// operand, relative to the wave-uniform base.
__device__ __forceinline__ uint32_t tn_goff(int64_t ld, int t, int src_row, int lane) {
  const int chunk = (lane & 3) ^ tn_f(t);
  return (uint32_t)(src_row * ld + 8 * chunk);
}

// one 16-row (1 KiB) global_load_lds per u: LDS rows 32 wave + 16 u + (lane >> 2);
// g = wave-uniform base (tile start + k offset): the scalar-base + 32-bit-offset form
__device__ __forceinline__ void tn_stage(const bf16_t* __restrict__ g, const uint32_t* goff, char* lds_tile, int wave) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    char* dst = lds_tile + (32 * wave + 16 * u) * TN_ROWB;  // wave-uniform
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(g + goff[u]),
                                     (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
  }
}

__device__ __forceinline__ int tn_xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// tile index -> (tm, tn): groups of 8 row tiles walk the column tiles, so a
// group's 8 A strips and the current B strip stay in the XCD's L2
__device__ __forceinline__ void tn_tile_coords(int tile, int tiles_m, int tiles_n, int* tm, int* tn) {
  const int per_group = 8 * tiles_n, group = tile / per_group, first_m = group * 8;
  const int gsz = min(tiles_m - first_m, 8);
  *tm = first_m + (tile - group * per_group) % gsz;
  *tn = (tile - group * per_group) / gsz;
}

__device__ __forceinline__ float tn_silu(float g) { return g / (1.f + __expf(-g)); }

// Epilogue shared by both main loops: acc[i][j] holds C[m][n .. n+3] of the
// wave's 128 x 64 block, m = wave row 0 + 16 i + (lane & 15), n = wave column 0
// + 16 j + 4 (lane >> 4).
template <int EPI>
__device__ __forceinline__ void tn_epilogue(f32x4 (&acc)[8][4], int tm, int tn, int wm, int wn, int lane,
                                            bf16_t* __restrict__ C, int64_t ldc, bf16_t* __restrict__ S,
                                            int64_t lds_, const bf16_t* __restrict__ GU, int64_t ldgu, int F) {
  const int m0 = tm * TN_BM + wm * 128 + (lane & 15);
  const int nl = 4 * (lane >> 4);
  if (EPI == TN_PLAIN) {
    const int n0 = tn * TN_BN + wn * 64 + nl;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        uint2 w;
        w.x = pack2(acc[i][j][0], acc[i][j][1]);
        w.y = pack2(acc[i][j][2], acc[i][j][3]);
        *(uint2*)(C + (int64_t)(m0 + 16 * i) * ldc + n0 + 16 * j) = w;
      }
  } else if (EPI == TN_SWIGLU_FWD) {
    // j = 0, 1: gate units h0 + 16 j; j = 2, 3: the same units' up values
    const int h0 = tn * (TN_BN / 2) + 32 * wn + nl;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      bf16_t* crow = C + (int64_t)(m0 + 16 * i) * ldc;
      bf16_t* srow = S + (int64_t)(m0 + 16 * i) * lds_;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const f32x4 g = acc[i][j], u = acc[i][j + 2];
        uint2 wg, wu, ws;
        wg.x = pack2(g[0], g[1]);
        wg.y = pack2(g[2], g[3]);
        wu.x = pack2(u[0], u[1]);
        wu.y = pack2(u[2], u[3]);
        // s from the bf16-rounded gate / up: the values backward re-reads from gu
        const float g0 = __uint_as_float(wg.x << 16), g1 = __uint_as_float(wg.x & 0xffff0000u);
        const float g2 = __uint_as_float(wg.y << 16), g3 = __uint_as_float(wg.y & 0xffff0000u);
        const float u0 = __uint_as_float(wu.x << 16), u1 = __uint_as_float(wu.x & 0xffff0000u);
        const float u2 = __uint_as_float(wu.y << 16), u3 = __uint_as_float(wu.y & 0xffff0000u);
        ws.x = pack2(tn_silu(g0) * u0, tn_silu(g1) * u1);
        ws.y = pack2(tn_silu(g2) * u2, tn_silu(g3) * u3);
        const int h = h0 + 16 * j;
        *(uint2*)(crow + h) = wg;
        *(uint2*)(crow + F + h) = wu;
        *(uint2*)(srow + h) = ws;
      }
    }
  } else {  // TN_SWIGLU_BWD: C = ds (never stored) -> dgu
    const int n0 = tn * TN_BN + wn * 64 + nl;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const bf16_t* gurow = GU + (int64_t)(m0 + 16 * i) * ldgu;
      bf16_t* drow = C + (int64_t)(m0 + 16 * i) * ldc;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int h = n0 + 16 * j;
        const uint2 gw = *(const uint2*)(gurow + h), uw = *(const uint2*)(gurow + F + h);
        float g[4] = {__uint_as_float(gw.x << 16), __uint_as_float(gw.x & 0xffff0000u), __uint_as_float(gw.y << 16),
                      __uint_as_float(gw.y & 0xffff0000u)};
        float u[4] = {__uint_as_float(uw.x << 16), __uint_as_float(uw.x & 0xffff0000u), __uint_as_float(uw.y << 16),
                      __uint_as_float(uw.y & 0xffff0000u)};
        // ds rounded to bf16 first: the value the unfused path stores
        float d[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) d[e] = bf2f(f2bf(acc[i][j][e]));
        float dg[4], du[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float sg = 1.f / (1.f + __expf(-g[e]));
          du[e] = d[e] * g[e] * sg;
          dg[e] = d[e] * u[e] * sg * (1.f + g[e] * (1.f - sg));
        }
        uint2 wdg, wdu;
        wdg.x = pack2(dg[0], dg[1]);
        wdg.y = pack2(dg[2], dg[3]);
        wdu.x = pack2(du[0], du[1]);
        wdu.y = pack2(du[2], du[3]);
        *(uint2*)(drow + h) = wdg;
        *(uint2*)(drow + F + h) = wdu;
      }
    }
  }
}

template <int EPI, int DIST>
__global__ __launch_bounds__(512, 1) void gemm_tn_kernel(const bf16_t* __restrict__ A, int64_t lda,
                                                         const bf16_t* __restrict__ B, int64_t ldb,
                                                         bf16_t* __restrict__ C, int64_t ldc,
                                                         bf16_t* __restrict__ S, int64_t lds_,
                                                         const bf16_t* __restrict__ GU, int64_t ldgu, int M, int N,
                                                         int K, int F) {
  // one LDS object per stage, loop unrolled by four: every access names its
  // buffer statically (see wgrad.hip: a runtime stage index makes hipcc drain
  // the LDS-DMA prefetch before every phase's first read)
  __shared__ __attribute__((aligned(1024))) char sb0[TN_STAGE];
  __shared__ __attribute__((aligned(1024))) char sb1[TN_STAGE];
  __shared__ __attribute__((aligned(1024))) char sb2[TN_STAGE];
  __shared__ __attribute__((aligned(1024))) char sb3[TN_STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int tiles_m = M / TN_BM, tiles_n = N / TN_BN;
  int tm, tn;
  tn_tile_coords(tn_xcd_remap(blockIdx.x, tiles_m * tiles_n), tiles_m, tiles_n, &tm, &tn);
  const int np = K / TN_BK;
  const int fmap = EPI == TN_SWIGLU_FWD ? F : 0;

  const bf16_t* Ab = A + (int64_t)tm * TN_BM * lda;
  const bf16_t* Bb = B + (int64_t)tn * (fmap ? TN_BN / 2 : TN_BN) * ldb;
  uint32_t ga[2], gb[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int t = 32 * wave + 16 * u + (lane >> 2);
    ga[u] = tn_goff(lda, t, t, lane);
    gb[u] = tn_goff(ldb, t, tn_brow(t, fmap), lane);
  }

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const bool lag = wm == 1;
  auto sync = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  // phase p: fragments of stage p (this buffer), LDS-DMA of stage p + DIST
  // into the buffer stage p + DIST - 4 used, wait for this wave's DMA of stage
  // p + 1, barrier, 32 MFMAs, barrier (the wgrad.hip schedule).  DIST = 3
  // gives each stage two phases of flight instead of one; the buffer it
  // refills was read in phase p - 1, by the lagging wave row one barrier
  // after the leading row, so every phase retires its reads (lgkmcnt(0))
  // before its first barrier.
  auto phase = [&](const char* cur, char* pre, int p) {
    tn_s16x8 bf[4], af[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) bf[j] = tn_frag(cur + TN_TILE, wn * 64 + 16 * j, lane);
#pragma unroll
    for (int i = 0; i < 8; ++i) af[i] = tn_frag(cur, wm * 128 + 16 * i, lane);
    const int q = min(p + DIST, np - 1);  // past the end: re-fetch into a buffer nobody reads again
    tn_stage(Ab + q * TN_BK, ga, pre, wave);
    tn_stage(Bb + q * TN_BK, gb, pre + TN_TILE, wave);
    if (DIST == 2)
      __builtin_amdgcn_s_waitcnt(TN_VMCNT4);
    else
      __builtin_amdgcn_s_waitcnt(0x0078);  // vmcnt(8) lgkmcnt(0)
    sync();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j], af[i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    sync();
  };

  tn_stage(Ab, ga, sb0, wave);
  tn_stage(Bb, gb, sb0 + TN_TILE, wave);
  tn_stage(Ab + TN_BK, ga, sb1, wave);
  tn_stage(Bb + TN_BK, gb, sb1 + TN_TILE, wave);
  if (DIST == 3) {
    tn_stage(Ab + 2 * TN_BK, ga, sb2, wave);
    tn_stage(Bb + 2 * TN_BK, gb, sb2 + TN_TILE, wave);
    __builtin_amdgcn_s_waitcnt(0x0F78);  // vmcnt(8): stage 0 landed
  } else {
    __builtin_amdgcn_s_waitcnt(TN_VMCNT4);
  }
  sync();
  if (lag) sync();
  for (int p = 0; p < np; p += 4) {
    if (DIST == 2) {
      phase(sb0, sb2, p);
      phase(sb1, sb3, p + 1);
      phase(sb2, sb0, p + 2);
      phase(sb3, sb1, p + 3);
    } else {
      phase(sb0, sb3, p);
      phase(sb1, sb0, p + 1);
      phase(sb2, sb1, p + 2);
      phase(sb3, sb2, p + 3);
    }
  }
  if (!lag) sync();
  __builtin_amdgcn_s_waitcnt(TN_VMCNT0);

  tn_epilogue<EPI>(acc, tm, tn, wm, wn, lane, C, ldc, S, lds_, GU, ldgu, F);
}

// ---------------------------------------------------------------------------
// Full-line form (the default): LDS rows of 64 k = 128 B, so every LDS-DMA
// piece is 8 rows x one whole 128-B line of each (the 32-k kernel above
// fetches 16 half lines per piece: twice the TA / L2 requests per byte --
// guide §5 "Projection GEMM at M = 256" item 3, and what hipBLASLt's
// MT256x256x64 does).  Two 64-KiB stages hold two 64-k tiles.  The phases
// stay 32 k deep (12 ds_read_b128 + 32 MFMAs per wave, two barriers, wave
// rows staggered by one barrier: the schedule the weight-gradient kernel
// measured best): phase (t, h) computes k-half h of tile t, and the first
// half-phase of tile t issues tile t + 1's whole DMA into the other stage
// (8 pieces per wave), which the second half-phase waits for.
//
//   RAW: tile t + 1 is waited (vmcnt(0), every issuing wave) before phase
//        (t, 1)'s first barrier and first read in phase (t + 1, 0).
//   WAR: the DMA of phase (t, 0) overwrites the stage tile t - 1 was read
//        from in phase (t - 1, 1); the lagging wave row issues those reads
//        one barrier later than the leading row issues the DMA, so phase
//        (., 1) retires its own reads (lgkmcnt(0)) before its first barrier.
//
// Swizzle: 16-B chunk c of LDS row r sits at chunk c ^ ((r >> 1) & 7); the 16
// lanes of each ds_read_b128 lane group then read 16 distinct 16-B bank slots
// (2 rows per 256-B bank row), for either k half.
#define TN64_ROWB 128
#define TN64_TILE (TN_BM * TN64_ROWB)  // 32 KiB per operand per stage
#define TN64_STAGE (2 * TN64_TILE)
#define TN_WAIT_ALL 0x0070             // vmcnt(0) lgkmcnt(0)

__device__ __forceinline__ int tn64_off(int r, int c) { return r * TN64_ROWB + ((c ^ ((r >> 1) & 7)) << 4); }

// lane's source offset (elements, from the operand tile's first row) for
// LDS row t, chunk position (lane & 7)
__device__ __forceinline__ uint32_t tn64_goff(int64_t ld, int t, int src_row, int lane) {
  const int chunk = (lane & 7) ^ ((t >> 1) & 7);
  return (uint32_t)(src_row * ld + 8 * chunk);
}

// one operand's 256-row tile: 32 pieces of 8 rows, 4 per wave (rows 32 wave +
// 8 u + (lane >> 3))
__device__ __forceinline__ void tn64_stage(const bf16_t* __restrict__ g, const uint32_t* goff, char* lds_tile,
                                           int wave) {
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    char* dst = lds_tile + (32 * wave + 8 * u) * TN64_ROWB;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(g + goff[u]),
                                     (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
  }
}

template <int EPI, int MODE>
__global__ __launch_bounds__(512, 1) void gemm_tn64_kernel(const bf16_t* __restrict__ A, int64_t lda,
                                                           const bf16_t* __restrict__ B, int64_t ldb,
                                                           bf16_t* __restrict__ C, int64_t ldc,
                                                           bf16_t* __restrict__ S, int64_t lds_,
                                                           const bf16_t* __restrict__ GU, int64_t ldgu, int M, int N,
                                                           int K, int F) {
  // two distinct LDS objects, every access names its stage statically
  __shared__ __attribute__((aligned(1024))) char sb0[TN64_STAGE];
  __shared__ __attribute__((aligned(1024))) char sb1[TN64_STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int tiles_m = M / TN_BM, tiles_n = N / TN_BN;
  int tm, tn;
  tn_tile_coords(tn_xcd_remap(blockIdx.x, tiles_m * tiles_n), tiles_m, tiles_n, &tm, &tn);
  const int nt = K / 64;
  // ROT: every tile starts its k loop at its own tile offset, so the
  // workgroups in flight fetch different k windows (their rows are K * 2
  // bytes apart: in lockstep, all of them would hit the same L2 channels)
  // MODE 2: tile t + 1's DMA goes out between phase (t, 0)'s MFMAs instead of
  // ahead of its barrier (the MFMA segment has idle issue slots; ahead of the
  // barrier, 8 pieces' issue can outlast the partner wave's MFMAs)
  const int rot = MODE == 1 ? (tm * 5 + tn * 3) % nt : 0;
  const int fmap = EPI == TN_SWIGLU_FWD ? F : 0;

  const bf16_t* Ab = A + (int64_t)tm * TN_BM * lda;
  const bf16_t* Bb = B + (int64_t)tn * (fmap ? TN_BN / 2 : TN_BN) * ldb;
  uint32_t ga[4], gb[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int t = 32 * wave + 8 * u + (lane >> 3);
    ga[u] = tn64_goff(lda, t, t, lane);
    gb[u] = tn64_goff(ldb, t, tn_brow(t, fmap), lane);
  }
  // fragment offsets: rows row0 + (lane & 15), chunk 4 h + (lane >> 4); row0
  // is a multiple of 16, so the swizzle term depends on the lane only
  const int fr = lane & 15;
  const int foff0 = fr * TN64_ROWB + (((lane >> 4) ^ ((fr >> 1) & 7)) << 4);
  const int foff1 = fr * TN64_ROWB + (((4 + (lane >> 4)) ^ ((fr >> 1) & 7)) << 4);

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const bool lag = wm == 1;
  auto sync = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  // one 32-k phase: fragments of k-half h of `cur`; h == 0 issues tile t + 1
  // into `nxt` (past the end: tile t again, into the stage nobody reads any
  // more), h == 1 waits for it and retires its own reads
  auto phase = [&](const char* cur, char* nxt, int t, int h) {
    const int foff = h ? foff1 : foff0;
    tn_s16x8 bf[4], af[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) bf[j] = *(const tn_s16x8*)(cur + TN64_TILE + (wn * 64 + 16 * j) * TN64_ROWB + foff);
#pragma unroll
    for (int i = 0; i < 8; ++i) af[i] = *(const tn_s16x8*)(cur + (wm * 128 + 16 * i) * TN64_ROWB + foff);
    int q = min(t + 1, nt - 1) + rot;
    q = (q >= nt ? q - nt : q) * 64;
    if (h == 0 && MODE != 2) {
      tn64_stage(Ab + q, ga, nxt, wave);
      tn64_stage(Bb + q, gb, nxt + TN64_TILE, wave);
    } else if (h == 1) {
      __builtin_amdgcn_s_waitcnt(TN_WAIT_ALL);
    }
    sync();
    __builtin_amdgcn_s_setprio(1);
    if (h == 0 && MODE == 2) {
      // fragments must have landed before the first MFMA
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_sched_barrier(0);
      tn64_stage(Ab + q, ga, nxt, wave);
      tn64_stage(Bb + q, gb, nxt + TN64_TILE, wave);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j], af[i], acc[i][j], 0, 0, 0);
    if (h == 0 && MODE == 2) {
#pragma unroll
      for (int g = 0; g < 8; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);  // MFMA
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM (LDS-DMA)
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
    }
    __builtin_amdgcn_s_setprio(0);
    sync();
  };

  tn64_stage(Ab + rot * 64, ga, sb0, wave);
  tn64_stage(Bb + rot * 64, gb, sb0 + TN64_TILE, wave);
  __builtin_amdgcn_s_waitcnt(TN_WAIT_ALL);
  sync();
  if (lag) sync();
  for (int t = 0; t < nt; t += 2) {
    phase(sb0, sb1, t, 0);
    phase(sb0, sb1, t, 1);
    phase(sb1, sb0, t + 1, 0);
    phase(sb1, sb0, t + 1, 1);
  }
  if (!lag) sync();
  __builtin_amdgcn_s_waitcnt(TN_WAIT_ALL);
  tn_epilogue<EPI>(acc, tm, tn, wm, wn, lane, C, ldc, S, lds_, GU, ldgu, F);
}

// ---------------------------------------------------------------------------
// One wave per SIMD (variant 2): 4 waves (2 M x 2 N), 128 x 128 of C per wave
// = 8 x 8 v_mfma_f32_16x16x32_bf16 tiles (64 f32x4 accumulators, 256
// registers: AGPRs).  Per 32-k phase a wave reads 16 fragments for 64 MFMAs
// (0.25 ds_read_b128 per MFMA against 0.375 with 8 waves of 128 x 64): less
// LDS energy per FLOP, which is what the clock under sustained MFMA load
// follows (MI355X_MICROARCH 'DVFS give-back'; profiles/r2_gemm_pmc: the
// library's 1-wave-per-SIMD 128 x 128 kernel holds a ~6 % higher clock).
// With no partner wave, the next phase's fragments are read into a second
// register set between this phase's MFMAs, and tile t + 1's LDS-DMA (16
// pieces per wave) goes out between the MFMAs of phase (t, 0).
//
// Phase (t, h): wait for the reads of its own fragments (issued during the
// previous phase) -- and for h == 1 this wave's DMA of tile t + 1 -- then ONE
// barrier, then 64 MFMAs with the reads of the next phase's fragments (for
// h == 1 those are tile t + 1's, from the other stage, landed behind the
// barrier) and for h == 0 tile t + 1's DMA between them.
//   WAR: the DMA of phase (t, 0) overwrites the stage of tile t - 1, whose
//        last reads (phase (t - 1, 1)'s fragments) were retired before the
//        barrier of phase (t - 1, 1).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void tn4_stage(const bf16_t* __restrict__ g, const uint32_t* goff, char* lds_tile,
                                          int wave, int half) {
#pragma unroll
  for (int u = 4 * half; u < 4 * half + 4; ++u) {
    char* dst = lds_tile + (64 * wave + 8 * u) * TN64_ROWB;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(g + goff[u]),
                                     (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
  }
}

__global__ __launch_bounds__(256, 1) void gemm_tn4w_kernel(const bf16_t* __restrict__ A, int64_t lda,
                                                           const bf16_t* __restrict__ B, int64_t ldb,
                                                           bf16_t* __restrict__ C, int64_t ldc, int M, int N, int K) {
  __shared__ __attribute__((aligned(1024))) char sb0[TN64_STAGE];
  __shared__ __attribute__((aligned(1024))) char sb1[TN64_STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int tiles_m = M / TN_BM, tiles_n = N / TN_BN;
  int tm, tn;
  tn_tile_coords(tn_xcd_remap(blockIdx.x, tiles_m * tiles_n), tiles_m, tiles_n, &tm, &tn);
  const int nt = K / 64;

  const bf16_t* Ab = A + (int64_t)tm * TN_BM * lda;
  const bf16_t* Bb = B + (int64_t)tn * TN_BN * ldb;
  uint32_t ga[8], gb[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int t = 64 * wave + 8 * u + (lane >> 3);
    ga[u] = tn64_goff(lda, t, t, lane);
    gb[u] = tn64_goff(ldb, t, t, lane);
  }
  const int fr = lane & 15;
  const int foff0 = fr * TN64_ROWB + (((lane >> 4) ^ ((fr >> 1) & 7)) << 4);
  const int foff1 = fr * TN64_ROWB + (((4 + (lane >> 4)) ^ ((fr >> 1) & 7)) << 4);
  const int arow = wm * 128 * TN64_ROWB, brow = TN64_TILE + wn * 128 * TN64_ROWB;

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto sync = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  auto rd = [&](const char* img, int off) { return *(const tn_s16x8*)(img + off); };
  // One phase: MFMAs of row block i (8, on fragment a[i] and the 8 B
  // fragments b), then a[i] <- the next phase's row block i and bn[i] <- its
  // B fragment i (from `nimg`, k half `nfoff`), and in DMA phases two of tile
  // t + 1's 16 LDS-DMA pieces: A is refilled in place, B double-buffered
  // (b / bn swap names between phases), 96 fragment registers in all.
  auto phase = [&](tn_s16x8(&a)[8], tn_s16x8(&b)[8], tn_s16x8(&bn)[8], const char* nimg, int nfoff, bool dma,
                   char* dimg, int t, bool waitdma) {
    if (waitdma)
      __builtin_amdgcn_s_waitcnt(TN_WAIT_ALL);
    else
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    sync();
    const int q = min(t + 1, nt - 1) * 64;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0);
      a[i] = rd(nimg, arow + 16 * i * TN64_ROWB + nfoff);
      bn[i] = rd(nimg, brow + 16 * i * TN64_ROWB + nfoff);
      if (dma) {
        const bf16_t* g = i < 4 ? Ab + q : Bb + q;
        char* d = i < 4 ? dimg : dimg + TN64_TILE;
        const uint32_t* go = i < 4 ? ga : gb;
        const int u = 2 * (i & 3);
#pragma unroll
        for (int v = u; v < u + 2; ++v)
          __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(g + go[v]),
                                           (__attribute__((address_space(3))) void*)(d + (64 * wave + 8 * v) *
                                                                                      TN64_ROWB),
                                           16, 0, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // DS read
      if (dma) __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);  // VMEM (LDS-DMA)
    }
  };

  tn_s16x8 a[8], b0[8], b1[8];
  tn4_stage(Ab, ga, sb0, wave, 0);
  tn4_stage(Ab, ga, sb0, wave, 1);
  tn4_stage(Bb, gb, sb0 + TN64_TILE, wave, 0);
  tn4_stage(Bb, gb, sb0 + TN64_TILE, wave, 1);
  __builtin_amdgcn_s_waitcnt(TN_WAIT_ALL);
  sync();
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a[i] = rd(sb0, arow + 16 * i * TN64_ROWB + foff0);
    b0[i] = rd(sb0, brow + 16 * i * TN64_ROWB + foff0);
  }
  for (int t = 0; t < nt; t += 2) {
    phase(a, b0, b1, sb0, foff1, true, sb1, t, false);
    phase(a, b1, b0, sb1, foff0, false, nullptr, t, true);
    phase(a, b0, b1, sb1, foff1, true, sb0, t + 1, false);
    phase(a, b1, b0, sb0, foff0, false, nullptr, t + 1, true);
  }
  __builtin_amdgcn_s_waitcnt(TN_WAIT_ALL);

  // epilogue: acc[i][j] = C[m][n .. n+3], m = 16 i + (lane & 15), n = 16 j + 4 (lane >> 4)
  const int m0 = tm * TN_BM + wm * 128 + (lane & 15);
  const int n0 = tn * TN_BN + wn * 128 + 4 * (lane >> 4);
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      uint2 w;
      w.x = pack2(acc[i][j][0], acc[i][j][1]);
      w.y = pack2(acc[i][j][2], acc[i][j][3]);
      *(uint2*)(C + (int64_t)(m0 + 16 * i) * ldc + n0 + 16 * j) = w;
    }
}

// ---------------------------------------------------------------------------
// Full lines AND a deeper prefetch (variant 6): the 160 KiB of LDS as a ring
// of five 32-KiB operand slots, each one operand's 64-k tile (256 rows x 128
// B, the full-line image of gemm_tn64_kernel).  Operand tiles go through the
// ring in the order A0 B0 A1 B1 A2 ..., slot = position % 5, so 2.5 tiles are
// resident: the two being read, the next one, and half of the one after.
// Phase (t, 0) issues B(t+1) and A(t+2) into the slots tile t - 1 freed;
// phase (t, 1) retires A(t+1) and B(t+1) (vmcnt(4): only A(t+2) may stay in
// flight) and its own reads (the lagging wave row reads tile t - 1's slots
// one barrier after the leading row refills them) before its first barrier.
// B gets the full-line kernel's two phases from issue to first read, A four.
// The slot pattern repeats every 5 tiles: the loop body is 5 tiles, and the
// K % 320 remainder runs the first tiles of the same body.
// ---------------------------------------------------------------------------
template <int EPI>
__global__ __launch_bounds__(512, 1) void gemm_tn5_kernel(const bf16_t* __restrict__ A, int64_t lda,
                                                          const bf16_t* __restrict__ B, int64_t ldb,
                                                          bf16_t* __restrict__ C, int64_t ldc,
                                                          bf16_t* __restrict__ S, int64_t lds_,
                                                          const bf16_t* __restrict__ GU, int64_t ldgu, int M, int N,
                                                          int K, int F) {
  __shared__ __attribute__((aligned(1024))) char r0[TN64_TILE];
  __shared__ __attribute__((aligned(1024))) char r1[TN64_TILE];
  __shared__ __attribute__((aligned(1024))) char r2[TN64_TILE];
  __shared__ __attribute__((aligned(1024))) char r3[TN64_TILE];
  __shared__ __attribute__((aligned(1024))) char r4[TN64_TILE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int tiles_m = M / TN_BM, tiles_n = N / TN_BN;
  int tm, tn;
  tn_tile_coords(tn_xcd_remap(blockIdx.x, tiles_m * tiles_n), tiles_m, tiles_n, &tm, &tn);
  const int nt = K / 64;
  const int fmap = EPI == TN_SWIGLU_FWD ? F : 0;

  const bf16_t* Ab = A + (int64_t)tm * TN_BM * lda;
  const bf16_t* Bb = B + (int64_t)tn * (fmap ? TN_BN / 2 : TN_BN) * ldb;
  uint32_t ga[4], gb[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int t = 32 * wave + 8 * u + (lane >> 3);
    ga[u] = tn64_goff(lda, t, t, lane);
    gb[u] = tn64_goff(ldb, t, tn_brow(t, fmap), lane);
  }
  const int fr = lane & 15;
  const int foff0 = fr * TN64_ROWB + (((lane >> 4) ^ ((fr >> 1) & 7)) << 4);
  const int foff1 = fr * TN64_ROWB + (((4 + (lane >> 4)) ^ ((fr >> 1) & 7)) << 4);

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const bool lag = wm == 1;
  auto sync = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  // phase (t, h): fragments of k-half h from slots (ai, bi); h == 0 issues
  // B(t+1) into `nb` and A(t+2) into `na` (past the end: the last tile again,
  // into slots nobody reads any more)
  auto phase = [&](const char* ai, const char* bi, char* nb, char* na, int t, int h) {
    const int foff = h ? foff1 : foff0;
    tn_s16x8 bf[4], af[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) bf[j] = *(const tn_s16x8*)(bi + (wn * 64 + 16 * j) * TN64_ROWB + foff);
#pragma unroll
    for (int i = 0; i < 8; ++i) af[i] = *(const tn_s16x8*)(ai + (wm * 128 + 16 * i) * TN64_ROWB + foff);
    if (h == 0) {
      tn64_stage(Bb + min(t + 1, nt - 1) * 64, gb, nb, wave);
      tn64_stage(Ab + min(t + 2, nt - 1) * 64, ga, na, wave);
    } else {
      __builtin_amdgcn_s_waitcnt(0x0074);  // vmcnt(4) lgkmcnt(0)
    }
    sync();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j], af[i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    sync();
  };
  // tile t = 5 g + j reads A from slot 2j % 5, B from (2j + 1) % 5 and
  // refills (2j + 3) % 5 with B(t+1), (2j + 4) % 5 with A(t+2)
#define TN5_TILE(AI, BI, NB, NA, T) \
  phase(AI, BI, NB, NA, T, 0);      \
  phase(AI, BI, NB, NA, T, 1);

  tn64_stage(Ab, ga, r0, wave);
  tn64_stage(Bb, gb, r1, wave);
  tn64_stage(Ab + min(1, nt - 1) * 64, ga, r2, wave);
  __builtin_amdgcn_s_waitcnt(0x0F74);  // vmcnt(4): A0, B0 landed
  sync();
  if (lag) sync();
  const int ng = nt / 5, rem = nt - 5 * ng;
  int t = 0;
  for (int g = 0; g < ng; ++g, t += 5) {
    TN5_TILE(r0, r1, r3, r4, t)
    TN5_TILE(r2, r3, r0, r1, t + 1)
    TN5_TILE(r4, r0, r2, r3, t + 2)
    TN5_TILE(r1, r2, r4, r0, t + 3)
    TN5_TILE(r3, r4, r1, r2, t + 4)
  }
  if (rem > 0) { TN5_TILE(r0, r1, r3, r4, t) }
  if (rem > 1) { TN5_TILE(r2, r3, r0, r1, t + 1) }
  if (rem > 2) { TN5_TILE(r4, r0, r2, r3, t + 2) }
  if (rem > 3) { TN5_TILE(r1, r2, r4, r0, t + 3) }
#undef TN5_TILE
  if (!lag) sync();
  __builtin_amdgcn_s_waitcnt(TN_WAIT_ALL);
  tn_epilogue<EPI>(acc, tm, tn, wm, wn, lane, C, ldc, S, lds_, GU, ldgu, F);
}

// main loop: 1 = full-line 64-k stages, 8 waves (default), 0 = the 32-k
// kernel, 2 = one wave per SIMD (plain epilogue only; the SwiGLU epilogues
// stay on 1), 3 = 1 with a per-tile k rotation, 4 = 1 with the DMA between
// the MFMAs, 5 = 0 with the DMA three stages ahead, 6 = full lines in a
// five-slot ring (gemm_tn5_kernel).  TOA_GEMM_TN_VARIANT selects; toa_gemm_tn_set_variant for A/B
static int g_tn_variant = -1;
static int tn_variant() {
  if (g_tn_variant < 0) {
    const char* e = getenv("TOA_GEMM_TN_VARIANT");
    g_tn_variant = (e && e[0] >= '0' && e[0] <= '6') ? e[0] - '0' : 1;
  }
  return g_tn_variant;
}
extern "C" int toa_gemm_tn_set_variant(int v) {
  g_tn_variant = (v < 0 || v > 6) ? -1 : v;
  return 0;
}

template <int EPI>
static void tn_launch(dim3 grid, hipStream_t stream, const bf16_t* A, int64_t lda, const bf16_t* B, int64_t ldb,
                      bf16_t* C, int64_t ldc, bf16_t* S, int64_t lds_, const bf16_t* GU, int64_t ldgu, int M, int N,
                      int K, int F) {
  const int v = tn_variant();
  if (v == 2 && EPI == TN_PLAIN)
    hipLaunchKernelGGL(gemm_tn4w_kernel, grid, dim3(256), 0, stream, A, lda, B, ldb, C, ldc, M, N, K);
  else if (v == 4)
    hipLaunchKernelGGL((gemm_tn64_kernel<EPI, 2>), grid, dim3(512), 0, stream, A, lda, B, ldb, C, ldc, S, lds_, GU,
                       ldgu, M, N, K, F);
  else if (v == 3)
    hipLaunchKernelGGL((gemm_tn64_kernel<EPI, 1>), grid, dim3(512), 0, stream, A, lda, B, ldb, C, ldc, S, lds_, GU,
                       ldgu, M, N, K, F);
  else if (v)
    hipLaunchKernelGGL((gemm_tn64_kernel<EPI, 0>), grid, dim3(512), 0, stream, A, lda, B, ldb, C, ldc, S, lds_, GU, ldgu, M,
                       N, K, F);
  else if (v == 6)
    hipLaunchKernelGGL(gemm_tn5_kernel<EPI>, grid, dim3(512), 0, stream, A, lda, B, ldb, C, ldc, S, lds_, GU, ldgu, M,
                       N, K, F);
  else if (v == 5)
    hipLaunchKernelGGL((gemm_tn_kernel<EPI, 3>), grid, dim3(512), 0, stream, A, lda, B, ldb, C, ldc, S, lds_, GU, ldgu,
                       M, N, K, F);
  else
    hipLaunchKernelGGL((gemm_tn_kernel<EPI, 2>), grid, dim3(512), 0, stream, A, lda, B, ldb, C, ldc, S, lds_, GU, ldgu, M,
                       N, K, F);
}

static bool tn_shape_ok(int M, int N, int K, int64_t lda, int64_t ldb) {
  return M > 0 && N > 0 && K > 0 && M % TN_BM == 0 && N % TN_BN == 0 && K % (4 * TN_BK) == 0 && lda % 8 == 0 &&
         ldb % 8 == 0;
}

// C[M][N] = A[M][K] B[N][K]^T.  M, N multiples of 256, K of 128, strides of
// 8 elements, 16-byte aligned bases.
extern "C" int toa_gemm_tn(const bf16_t* A, int64_t lda, const bf16_t* B, int64_t ldb, bf16_t* C, int64_t ldc, int M,
                           int N, int K, hipStream_t stream) {
  if (!tn_shape_ok(M, N, K, lda, ldb) || ldc % 4) return (int)hipErrorInvalidValue;
  tn_launch<TN_PLAIN>(dim3((M / TN_BM) * (N / TN_BN)), stream, A, lda, B, ldb, C, ldc, nullptr, 0, nullptr, 0, M, N,
                      K, 0);
  return (int)hipGetLastError();
}

// gu[M][2F] = X[M][K] Wgu[2F][K]^T (Wgu = [gate; up]) and s[M][F] =
// silu(gate) * up.  F a multiple of 128.
extern "C" int toa_gemm_tn_swiglu(const bf16_t* X, int64_t ldx, const bf16_t* Wgu, int64_t ldw, bf16_t* GU,
                                  int64_t ldgu, bf16_t* S, int64_t lds_, int M, int F, int K, hipStream_t stream) {
  if (F % (TN_BN / 2) || !tn_shape_ok(M, 2 * F, K, ldx, ldw) || ldgu % 4 || lds_ % 4)
    return (int)hipErrorInvalidValue;
  tn_launch<TN_SWIGLU_FWD>(dim3((M / TN_BM) * (2 * F / TN_BN)), stream, X, ldx, Wgu, ldw, GU, ldgu, S, lds_, nullptr, 0,
                           M, 2 * F, K, F);
  return (int)hipGetLastError();
}

// dgu[M][2F] = swiglu'(gu) applied to ds = dY[M][K] WdT[F][K]^T (ds itself is
// not stored).  F a multiple of 256.
extern "C" int toa_gemm_tn_swiglu_bwd(const bf16_t* dY, int64_t ldy, const bf16_t* WdT, int64_t ldw,
                                      const bf16_t* GU, int64_t ldgu, bf16_t* dGU, int64_t lddgu, int M, int F, int K,
                                      hipStream_t stream) {
  if (!tn_shape_ok(M, F, K, ldy, ldw) || ldgu % 4 || lddgu % 4) return (int)hipErrorInvalidValue;
  tn_launch<TN_SWIGLU_BWD>(dim3((M / TN_BM) * (F / TN_BN)), stream, dY, ldy, WdT, ldw, dGU, lddgu, nullptr, 0, GU, ldgu,
                           M, F, K, F);
  return (int)hipGetLastError();
}
