// All-reduce by direct peer reads over xGMI: the small-message path of the communication layer
// (the FedAvg / FedSGD weighted reduce C13 of a 1.2M-parameter MnistCnn is
// 4.8 MB, VFL / pipeline messages are KBs — sizes where ring all-reduce is latency-bound).
//
// Every rank owns ONE uncached device allocation (hipExtMallocWithFlags(hipDeviceMallocUncached)),
// exported with hipIpcGetMemHandle and mapped by every peer (hipIpcOpenMemHandle), so a kernel on
// rank r can load and store any peer's buffer; uncached memory keeps no stale copy in any XCD's
// L2 on either side. Layout of one rank's allocation:
//   [signal words: 2 phases x IPC_MAXB blocks x IPC_MAXR sources, uint32]  (IPC_SIG_BYTES)
//   [epoch counter {epoch, ticket}]
//   parity slot 0: [data: cap bytes][result: cap bytes]   parity slot 1: [data][result]
//
// One launch per all-reduce (graph-capturable: the epoch lives on the device, the last block of
// a launch advances it). Block b of every rank handles the same element ranges:
//   one-shot (small n): copy my range into my data slot -> barrier -> sum the range over all
//     ranks' data slots, in rank order 0..W-1 (so every rank gets bit-identical results) -> out.
//     Per GPU (W-1)*n*4 bytes cross xGMI, spread over all 7 links at once.
//   two-shot (larger n): shards of n/W; copy-in -> barrier -> reduce MY shard's range from every
//     rank (reduce-scatter) into my result slot -> barrier -> gather every shard's range from its
//     owner's result slot (all-gather). 2*(W-1)/W*n*4 bytes per GPU.
// Barriers are per block: block b signals block b of every peer (system-scope store into the
// peer's signal words) and spins on its own words with a wall-clock bound (s_memrealtime,
// 100 MHz): a missing peer sets the error word and the kernel exits instead of hanging the GPU.
// Parity slots: a rank's copy-in of call e+1 cannot overwrite data a slower peer still reads for
// call e (one-shot has no second barrier).
#include "ddl_common.h"

#include <cstring>

#define IPC_MAXR 8
#define IPC_MAXB 64
#define IPC_SIG_BYTES (2 * IPC_MAXB * IPC_MAXR * 4)
#define IPC_HDR_BYTES 65536  // signal words + epoch counter, rounded up

struct IpcArgs {
  char* base[IPC_MAXR];  // each rank's mapped allocation (base[rank] = my own)
  const float* in;
  float* out;            // may alias in
  long long n;           // fp32 elements
  long long cap;         // bytes per data / result slot
  int* err;              // device word, set to 1 on a barrier timeout
  long long timeout;     // s_memrealtime ticks (100 MHz)
  int rank, world, two_shot;
};

__device__ __forceinline__ unsigned* ipc_sig(char* base, int phase, int blk, int src) {
  return (unsigned*)base + (phase * IPC_MAXB + blk) * IPC_MAXR + src;
}
__device__ __forceinline__ unsigned* ipc_epoch(char* base) { return (unsigned*)(base + IPC_SIG_BYTES); }
__device__ __forceinline__ float* ipc_data(char* base, unsigned epoch, long long cap) {
  return (float*)(base + IPC_HDR_BYTES + (long long)(epoch & 1u) * 2 * cap);
}

// Block-level cross-rank barrier for (phase, this block): every wave drains its stores, one
// lane per peer publishes `epoch` into that peer's signal word for (phase, block, my rank) and
// polls my own word for (phase, block, peer) until it has reached `epoch`. The compare is
// wrap-safe and monotonic (>=, not ==): back-to-back all-reduces without a host sync let a fast
// peer overwrite its word with epoch+1 before a slow block here has seen epoch — which also
// proves the peer passed this barrier.
__device__ void ipc_barrier(const IpcArgs& a, int phase, unsigned epoch) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int t = threadIdx.x;
  if (t < a.world) {
    __threadfence_system();
    __hip_atomic_store(ipc_sig(a.base[t], phase, blockIdx.x, a.rank), epoch, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    unsigned* mine = ipc_sig(a.base[a.rank], phase, blockIdx.x, t);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while ((int)(__hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
      __builtin_amdgcn_s_sleep(2);
      if ((long long)(__builtin_amdgcn_s_memrealtime() - t0) > a.timeout) {
        __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
    __threadfence_system();
  }
  __syncthreads();
}

// dst[i] = src[i] for i in [lo, hi)  (lo % 4 == 0; 16-B vectors, scalar tail)
__device__ __forceinline__ void ipc_copy(float* dst, const float* src, long long lo, long long hi) {
  const long long hi4 = lo + ((hi - lo) & ~3LL);
  for (long long i = lo + 4 * threadIdx.x; i < hi4; i += 4 * blockDim.x)
    *(float4*)(dst + i) = *(const float4*)(src + i);
  for (long long i = hi4 + threadIdx.x; i < hi; i += blockDim.x) dst[i] = src[i];
}

// out[i] = sum_r src_r[i] (rank order; my own term from `mine`)
__device__ __forceinline__ void ipc_sum(const IpcArgs& a, unsigned epoch, const float* mine,
                                        float* out, float* out2, long long lo, long long hi) {
  const long long hi4 = lo + ((hi - lo) & ~3LL);
  for (long long i = lo + 4 * threadIdx.x; i < hi4; i += 4 * blockDim.x) {
    float4 v[IPC_MAXR];
#pragma unroll
    for (int r = 0; r < IPC_MAXR; ++r)
      if (r < a.world)
        v[r] = *(const float4*)((r == a.rank ? mine : ipc_data(a.base[r], epoch, a.cap)) + i);
    float4 s = v[0];
#pragma unroll
    for (int r = 1; r < IPC_MAXR; ++r)
      if (r < a.world) { s.x += v[r].x; s.y += v[r].y; s.z += v[r].z; s.w += v[r].w; }
    *(float4*)(out + i) = s;
    if (out2) *(float4*)(out2 + i) = s;
  }
  for (long long i = hi4 + threadIdx.x; i < hi; i += blockDim.x) {
    float s = 0.f;
    for (int r = 0; r < a.world; ++r)
      s += (r == a.rank ? mine : ipc_data(a.base[r], epoch, a.cap))[i];
    out[i] = s;
    if (out2) out2[i] = s;
  }
}

__global__ __launch_bounds__(256) void ipc_allreduce_kernel(IpcArgs a) {
  char* me = a.base[a.rank];
  unsigned* ectr = ipc_epoch(me);
  const unsigned epoch = __hip_atomic_load(ectr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) + 1u;
  float* my_data = ipc_data(me, epoch, a.cap);
  const int nb = gridDim.x, b = blockIdx.x;
  if (!a.two_shot) {
    long long per = ((a.n + nb - 1) / nb + 3) & ~3LL;
    const long long lo = min(a.n, b * per), hi = min(a.n, lo + per);
    ipc_copy(my_data, a.in, lo, hi);
    ipc_barrier(a, 0, epoch);
    ipc_sum(a, epoch, a.in, a.out, nullptr, lo, hi);
  } else {
    const long long S = ((a.n + a.world - 1) / a.world + 3) & ~3LL;  // shard
    const long long per = ((S + nb - 1) / nb + 3) & ~3LL;             // block's part of a shard
    for (int p = 0; p < a.world; ++p) {
      const long long lo = min(a.n, p * S + min(S, b * per));
      const long long hi = min(a.n, min((p + 1) * S, p * S + min(S, (b + 1) * per)));
      ipc_copy(my_data, a.in, lo, hi);
    }
    ipc_barrier(a, 0, epoch);
    {
      const int p = a.rank;
      const long long lo = min(a.n, p * S + min(S, b * per));
      const long long hi = min(a.n, min((p + 1) * S, p * S + min(S, (b + 1) * per)));
      float* my_res = (float*)((char*)my_data + a.cap);
      // reduce-scatter of my shard into my result slot (and straight into out)
      ipc_sum(a, epoch, a.in, my_res, a.out, lo, hi);
    }
    ipc_barrier(a, 1, epoch);
    for (int p = 0; p < a.world; ++p) {
      if (p == a.rank) continue;
      const long long lo = min(a.n, p * S + min(S, b * per));
      const long long hi = min(a.n, min((p + 1) * S, p * S + min(S, (b + 1) * per)));
      const float* res = (const float*)((const char*)ipc_data(a.base[p], epoch, a.cap) + a.cap);
      ipc_copy(a.out, res, lo, hi);
    }
  }
  // advance the device epoch once every block of this launch has read it
  __syncthreads();
  if (threadIdx.x == 0) {
    if (__hip_atomic_fetch_add(ectr + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)nb - 1) {
      __hip_atomic_store(ectr + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ectr, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

DDL_API int ddl_ipc_args_size() { return (int)sizeof(IpcArgs); }
DDL_API int ddl_ipc_header_bytes() { return IPC_HDR_BYTES; }
DDL_API int ddl_ipc_max_blocks() { return IPC_MAXB; }

// one uncached allocation: header + 2 parity slots x (data + result) of `cap` bytes each
DDL_API int ddl_ipc_malloc(long long cap, void** out) {
  if (cap <= 0 || cap % 16) return (int)hipErrorInvalidValue;
  const size_t bytes = (size_t)IPC_HDR_BYTES + 4 * (size_t)cap;
  hipError_t e = hipExtMallocWithFlags(out, bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  e = hipMemset(*out, 0, bytes);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  return (int)e;
}
DDL_API int ddl_ipc_free(void* p) { return (int)hipFree(p); }
DDL_API int ddl_ipc_get_handle(void* p, void* handle64) {
  hipIpcMemHandle_t h;
  hipError_t e = hipIpcGetMemHandle(&h, p);
  if (e != hipSuccess) return (int)e;
  static_assert(sizeof(h) <= 64, "handle size");
  memcpy(handle64, &h, sizeof(h));
  return 0;
}
DDL_API int ddl_ipc_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }
DDL_API int ddl_ipc_open(const void* handle64, void** out) {
  hipIpcMemHandle_t h;
  memcpy(&h, handle64, sizeof(h));
  return (int)hipIpcOpenMemHandle(out, h, hipIpcMemLazyEnablePeerAccess);
}
DDL_API int ddl_ipc_close(void* p) { return (int)hipIpcCloseMemHandle(p); }

DDL_API int ddl_ipc_allreduce(const IpcArgs* a, int nblocks, hipStream_t s) {
  if (a->world < 1 || a->world > IPC_MAXR || a->rank < 0 || a->rank >= a->world) return (int)hipErrorInvalidValue;
  if (a->n < 0 || a->n * 4 > a->cap || nblocks < 1 || nblocks > IPC_MAXB) return (int)hipErrorInvalidValue;
  if (((uintptr_t)a->in | (uintptr_t)a->out) & 15) return (int)hipErrorInvalidValue;
  for (int r = 0; r < a->world; ++r)
    if (!a->base[r]) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(ipc_allreduce_kernel, dim3(nblocks), dim3(256), 0, s, *a);
  return (int)hipGetLastError();
}
