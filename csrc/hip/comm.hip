// One-shot all-reduce on IPC-mapped peer buffers.
//
// For the latency-bound messages of the small payloads (MNIST MLP / Keras
// CNN gradients are 0.3-0.4 MB) a ring pays 2(N-1) link hops.  Here every
// rank exposes a fine-grained staging buffer and a flag array through
// hipIpcGetMemHandle; a call is
//   1. copy:    local input -> my staging slot (this call's half of a 2-deep ring)
//   2. barrier: publish the call's epoch into every peer's flag array
//               (system-scope release), wait until all peers published it
//               (bounded spin: a missing peer sets an error flag, never hangs)
//   3. reduce:  out[i] = sum over ranks of staging[r][i], reading the 7 peers
//               directly over xGMI (one hop, all links busy at once).
// The ring is two slots deep: a rank can only reach barrier e after its
// reduce of e-1 finished, so slot (e+1)&1 is never overwritten while a peer
// still reads it.  Large messages stay on RCCL (bandwidth-bound: channel
// spreading over the 7 links is what matters there).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

#include "toa_common.h"

#define TOA_MAX_RANKS 8

struct IpcPeers {
  void* buf[TOA_MAX_RANKS];         // staging buffers (2 slots each), mapped
  unsigned* flags[TOA_MAX_RANKS];   // flag arrays [TOA_MAX_RANKS] per rank, mapped
};

__global__ void ipc_copy_kernel(const char* __restrict__ src, char* __restrict__ dst, int64_t nbytes) {
  const int64_t n16 = nbytes / 16;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (int64_t)gridDim.x * blockDim.x)
    ((u32x4*)dst)[i] = ((const u32x4*)src)[i];
  if (blockIdx.x == 0 && threadIdx.x < (nbytes & 15)) dst[n16 * 16 + threadIdx.x] = src[n16 * 16 + threadIdx.x];
}

// one wave: lane r < world publishes to / waits on rank r
__global__ void ipc_barrier_kernel(IpcPeers peers, int rank, int world, unsigned epoch, unsigned* err,
                                   long long timeout_cycles) {
  const int r = threadIdx.x;
  __threadfence_system();  // the copy kernel's writes are visible before the flag
  if (r < world) {
    __hip_atomic_store(peers.flags[r] + rank, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    const long long t0 = wall_clock64();
    unsigned* mine = peers.flags[rank] + r;
    while (__hip_atomic_load(mine, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < epoch) {
      if (wall_clock64() - t0 > timeout_cycles) {
        atomicOr(err, 1u << r);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __threadfence_system();
}

template <typename T>
__global__ void ipc_reduce_kernel(IpcPeers peers, int world, int64_t slot_off, T* __restrict__ out, int64_t n) {
  constexpr int V = 16 / sizeof(T);
  const int64_t nv = n / V;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (int64_t)gridDim.x * blockDim.x) {
    float acc[V];
#pragma unroll
    for (int j = 0; j < V; ++j) acc[j] = 0.f;
    for (int r = 0; r < world; ++r) {  // fixed rank order: every rank gets bit-identical sums
      const u32x4 v = ((const u32x4*)((const char*)peers.buf[r] + slot_off))[i];
      if constexpr (sizeof(T) == 2) {
        float f[8];
        unpack8(v, f);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += f[j];
      } else {
        // whole-vector bit_cast: hipcc (ROCm 7.2) miscompiles bit_cast of
        // single ext_vector elements in this loop (all lanes got element 0)
        const f32x4 fv = __builtin_bit_cast(f32x4, v);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] += fv[j];
      }
    }
    u32x4 o;
    if constexpr (sizeof(T) == 2) {
      o = pack8(acc);
    } else {
      o = __builtin_bit_cast(u32x4, f32x4{acc[0], acc[1], acc[2], acc[3]});
    }
    ((u32x4*)out)[i] = o;
  }
  // tail (n not a multiple of V)
  for (int64_t i = nv * V + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float a = 0.f;
    for (int r = 0; r < world; ++r) {
      const T* p = (const T*)((const char*)peers.buf[r] + slot_off);
      if constexpr (sizeof(T) == 2) a += bf2f(p[i]); else a += (float)p[i];
    }
    if constexpr (sizeof(T) == 2) out[i] = f2bf(a); else out[i] = (T)a;
  }
}

// fine-grained (coherent across the xGMI fabric) allocation
extern "C" int toa_ipc_alloc(int64_t bytes, void** ptr) {
  const char* fg = getenv("TOA_IPC_FINEGRAINED");
  if (fg != nullptr && fg[0] == '0') {
    if (hipMalloc(ptr, (size_t)bytes) != hipSuccess) return 1;
  } else if (hipExtMallocWithFlags(ptr, (size_t)bytes, hipDeviceMallocFinegrained) != hipSuccess) {
    return 1;
  }
  return (int)hipMemset(*ptr, 0, (size_t)bytes);
}

extern "C" int toa_ipc_free(void* ptr) { return (int)hipFree(ptr); }

extern "C" int toa_ipc_get_handle(void* ptr, void* handle64) {
  return (int)hipIpcGetMemHandle((hipIpcMemHandle_t*)handle64, ptr);
}

extern "C" int toa_ipc_open_handle(const void* handle64, void** ptr) {
  hipIpcMemHandle_t h;
  __builtin_memcpy(&h, handle64, sizeof(h));
  return (int)hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess);
}

extern "C" int toa_ipc_close_handle(void* ptr) { return (int)hipIpcCloseMemHandle(ptr); }

extern "C" int toa_ipc_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }

// bufs / flags: `world` device pointers (own ones at [rank]); slot_bytes:
// capacity of one of the two slots.  dtype 0 bf16, 1 fp32.  err: device
// uint32 that gets bit r set if rank r never arrived (timeout_ms).
extern "C" int toa_allreduce_oneshot(void* const* bufs, void* const* flags, int rank, int world, int dtype,
                                     const void* in, void* out, int64_t n, int64_t slot_bytes, unsigned epoch,
                                     unsigned* err, int timeout_ms, hipStream_t stream) {
  if (world < 1 || world > TOA_MAX_RANKS || rank < 0 || rank >= world) return (int)hipErrorInvalidValue;
  const int64_t esz = dtype == 0 ? 2 : 4;
  const int64_t bytes = n * esz;
  if (bytes > slot_bytes) return (int)hipErrorInvalidValue;
  IpcPeers p;
  for (int r = 0; r < TOA_MAX_RANKS; ++r) {
    p.buf[r] = r < world ? bufs[r] : nullptr;
    p.flags[r] = r < world ? (unsigned*)flags[r] : nullptr;
  }
  const int64_t slot_off = (int64_t)(epoch & 1) * slot_bytes;
  const int blocks = (int)std::min<int64_t>(256, (bytes / 16 + 255) / 256 + 1);
  hipLaunchKernelGGL(ipc_copy_kernel, dim3(blocks), dim3(256), 0, stream, (const char*)in,
                     (char*)bufs[rank] + slot_off, bytes);
  // wall_clock64 runs at 100 MHz on gfx9
  hipLaunchKernelGGL(ipc_barrier_kernel, dim3(1), dim3(64), 0, stream, p, rank, world, epoch, err,
                     (long long)timeout_ms * 100000ll);
  if (dtype == 0)
    hipLaunchKernelGGL(ipc_reduce_kernel<bf16_t>, dim3(blocks), dim3(256), 0, stream, p, world, slot_off,
                       (bf16_t*)out, n);
  else
    hipLaunchKernelGGL(ipc_reduce_kernel<float>, dim3(blocks), dim3(256), 0, stream, p, world, slot_off,
                       (float*)out, n);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Collective traffic emulator (parallel/emulate.py): what one rank's RCCL
// reduce-scatter / all-gather kernel does to THIS GPU at world N, on a
// one-GPU box.  RCCL's ring kernel occupies `nblocks` workgroups (one per
// channel, 256 threads) for the whole collective, streams (N-1)/N of the
// bucket through HBM, and lasts as long as the xGMI links need for it.  The
// emulator moves the same bytes (src -> a scratch dst) with the same
// workgroup count and paces every workgroup to the link rate: a workgroup
// that covered `done` bytes of its share waits until t0 + done / rate
// (s_memrealtime, 100 MHz) before its next 64 KiB chunk.  A workgroup that
// is dispatched late (CUs held by a GEMM) starts its clock late, so the
// emulated collective stretches exactly as a real one whose peers wait for
// this rank would.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void emu_xfer_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                       int64_t n16, int64_t ticks_per_mib) {
  const int64_t per = (n16 + gridDim.x - 1) / gridDim.x;
  const int64_t lo = (int64_t)blockIdx.x * per;
  const int64_t hi = lo + per < n16 ? lo + per : n16;
  constexpr int64_t CHUNK = 4096;  // 16-B vectors: 64 KiB per workgroup step
  const long long t0 = wall_clock64();
  for (int64_t c = lo; c < hi; c += CHUNK) {
    const int64_t e = c + CHUNK < hi ? c + CHUNK : hi;
    for (int64_t i = c + threadIdx.x; i < e; i += 256) dst[i] = src[i];
    if (ticks_per_mib > 0) {
      // bytes of this workgroup's share done so far -> earliest allowed time
      const long long due = t0 + (long long)(((e - lo) * 16 * ticks_per_mib) >> 20);
      while (wall_clock64() < due) __builtin_amdgcn_s_sleep(8);
    }
  }
}

// Move `nbytes` (multiple of 16) from src to dst on `nblocks` workgroups,
// paced to `gbps` GB/s for the whole transfer (0 = unpaced).
extern "C" int toa_emulate_xfer(const void* src, void* dst, int64_t nbytes, int nblocks, double gbps,
                                hipStream_t stream) {
  if (nbytes <= 0) return 0;
  if (nbytes % 16 || nblocks <= 0) return (int)hipErrorInvalidValue;
  // per-workgroup rate = gbps / nblocks; ticks of the 100 MHz clock per MiB of a share
  const int64_t ticks_per_mib = gbps > 0 ? (int64_t)(1e8 * (double)(1 << 20) * nblocks / (gbps * 1e9)) : 0;
  hipLaunchKernelGGL(emu_xfer_kernel, dim3(nblocks), dim3(256), 0, stream, (const u32x4*)src, (u32x4*)dst,
                     nbytes / 16, ticks_per_mib);
  return (int)hipGetLastError();
}

// One-GPU emulation of a CU-free all-gather (verdict r4 item 5): the bytes a
// rank pulls from its peers, moved by a copy engine (hipMemcpyDeviceToDeviceNoCU:
// SDMA, no workgroup on any CU) instead of a ring kernel's workgroups.  A copy
// engine cannot be paced: it runs at its own rate, which
// scripts/overlap_emulation.py reports next to the assumed bus rate.
extern "C" int toa_emulate_copy_nocu(const void* src, void* dst, int64_t nbytes, hipStream_t stream) {
  if (nbytes <= 0) return 0;
  return (int)hipMemcpyAsync(dst, src, (size_t)nbytes, hipMemcpyDeviceToDeviceNoCU, stream);
}

// ---------------------------------------------------------------------------
// Copy-engine all-gather of the ZeRO-1 weights (parallel/pull_gather.py):
// after a rank's AdamW has written its shard of a bucket it publishes the
// step's epoch in its own IPC-exported flag word for that bucket (system-
// scope release: the update's writes are visible to the peers' copy
// engines first); each rank's copy stream waits until every peer published
// the epoch (bounded spin: a missing peer sets its error bit, never hangs),
// then pulls the peers' shards with hipMemcpyDeviceToDeviceNoCU (SDMA, no
// workgroup on any CU -- the GEMMs of the forward keep every CU).
// ---------------------------------------------------------------------------
struct PeerFlags {
  unsigned* f[TOA_MAX_RANKS];  // each rank's flag array, mapped (own one at [rank])
};

__global__ void flag_publish_kernel(unsigned* flag, unsigned epoch) {
  __threadfence_system();
  __hip_atomic_store(flag, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void flags_wait_kernel(PeerFlags peers, int idx, int rank, int world, unsigned epoch, unsigned* err,
                                  long long timeout_cycles) {
  const int r = threadIdx.x;
  // a peer already marked lost (an earlier bucket's wait timed out) is not
  // waited for again: a lost peer costs one timeout per run, not one per bucket
  if (r < world && r != rank && !(__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & (1u << r))) {
    const long long t0 = wall_clock64();
    while (__hip_atomic_load(peers.f[r] + idx, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < epoch) {
      if (wall_clock64() - t0 > timeout_cycles) {
        atomicOr(err, 1u << r);
        break;
      }
      __builtin_amdgcn_s_sleep(4);
    }
  }
  __threadfence_system();
}

extern "C" int toa_flag_publish(void* flag, unsigned epoch, hipStream_t stream) {
  if (!flag) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(flag_publish_kernel, dim3(1), dim3(1), 0, stream, (unsigned*)flag, epoch);
  return (int)hipGetLastError();
}

// flags: `world` device pointers (each rank's flag array); waits for entry
// idx of every peer's array to reach epoch.  err: bit r set on a timeout.
extern "C" int toa_flags_wait(void* const* flags, int idx, int rank, int world, unsigned epoch, unsigned* err,
                              int timeout_ms, hipStream_t stream) {
  if (world < 1 || world > TOA_MAX_RANKS || rank < 0 || rank >= world || idx < 0 || !err)
    return (int)hipErrorInvalidValue;
  PeerFlags p;
  for (int r = 0; r < TOA_MAX_RANKS; ++r) p.f[r] = r < world ? (unsigned*)flags[r] : nullptr;
  hipLaunchKernelGGL(flags_wait_kernel, dim3(1), dim3(64), 0, stream, p, idx, rank, world, epoch, err,
                     (long long)timeout_ms * 100000ll);  // wall_clock64: 100 MHz
  return (int)hipGetLastError();
}

// The owner's half of the copy-engine reduce-scatter
// (parallel/pull_gather.PullReduceScatter): dst[i] <- bf16(dst[i] + src[0][i]
// + ... + src[nsl - 1][i]), summed in fp32 in that order and rounded once;
// src slices `stride` elements apart (the peers' pulled slices, staged).
// n a multiple of 8, 16-byte aligned.  HBM-bound: 8 elements per thread.
__global__ __launch_bounds__(256) void sum_slices_bf16_kernel(bf16_t* __restrict__ dst, const bf16_t* __restrict__ src,
                                                              int nsl, int64_t stride, int64_t n8) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    float acc[8], f[8];
    unpack8(ld16(dst + i * 8), acc);
    for (int k = 0; k < nsl; ++k) {
      unpack8(__builtin_nontemporal_load((const u32x4*)(src + k * stride) + i), f);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += f[j];
    }
    st16(dst + i * 8, pack8(acc));
  }
}

extern "C" int toa_sum_slices_bf16(bf16_t* dst, const bf16_t* src, int nsl, int64_t stride, int64_t n,
                                   hipStream_t stream) {
  if (n <= 0) return 0;
  if (n % 8 || stride % 8 || nsl < 0 || (((uintptr_t)dst | (uintptr_t)src) & 15)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(sum_slices_bf16_kernel, dim3(toa_stream_grid(n / 8, 256)), dim3(256), 0, stream, dst, src, nsl,
                     stride, n / 8);
  return (int)hipGetLastError();
}

// A copy on a copy engine (SDMA): peer-mapped source, local destination.
extern "C" int toa_copy_nocu(const void* src, void* dst, int64_t nbytes, hipStream_t stream) {
  if (nbytes <= 0) return 0;
  return (int)hipMemcpyAsync(dst, src, (size_t)nbytes, hipMemcpyDeviceToDeviceNoCU, stream);
}
