// Federated aggregation kernels.
//
//   ddl_weighted_sum   : out[i] (+)= sum_g coeff[g] * src[g][i]   — FedAvg / FedSGD weighted
//                        reduce over the clients resident on this GPU (reference
//                        hfl_complete.py:291-299, 370-378 do this with torch.stack(...).sum(0)
//                        on the host); the cross-GPU part is one RCCL all-reduce of `out`.
//   ddl_broadcast_rows : dst[g][i] = src[i] (+ bf16 shadow) — server -> client weight download
//                        (hfl_complete.py:323-325) without leaving HBM.
//   ddl_gram_f32       : G = (X - c)(X - c)^T on the exact-fp32 MFMA (v_mfma_f32_16x16x4_f32),
//                        split over the coordinate axis, K <= 128 clients, deterministic —
//                        pairwise distances for Krum / multi-Krum (Blanchard et al. 2017)
//                        [north-star, absent in reference].
//   ddl_coord_select   : coordinate-wise median / trimmed mean over K <= 128 client vectors by an
//                        in-register bitonic sort per coordinate (Yin et al. 2018) [north-star].
#include "ddl_common.h"

__global__ void weighted_sum_kernel(const float* __restrict__ src, long long ld,
                                    const float* __restrict__ coeff, int G, long long n,
                                    float* __restrict__ out, int accumulate) {
  // every product rounded on its own, then added: hipcc contracts a * b + c into an fma by default
  // (also through __fmul_rn / __fadd_rn, whose header bodies carry the contract flag), which made the
  // G-row single-process sum differ from per-rank partials summed across ranks
#pragma clang fp contract(off)
  // float4 path only when every row start and the output are 16-B aligned (a sub-slice of a
  // flat buffer passed as `out` / `src` need not be)
  const bool vec = (ld % 4) == 0 && (((uintptr_t)out | (uintptr_t)src) & 15) == 0;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t * 4 < n;
       t += (long long)gridDim.x * blockDim.x) {
    const long long e = t * 4;
    if (e + 4 <= n && vec) {
      float4 acc = accumulate ? *(const float4*)(out + e) : make_float4(0, 0, 0, 0);
      // products rounded, then added in client order (no fused multiply-add): the same bits as
      // clients spread over ranks (each rank's product, then the all-reduce add) for 2 ranks, and
      // the reference's sum of n_k/n-scaled state dicts (hfl_complete.py:370-378)
      for (int g = 0; g < G; ++g) {
        const float c = coeff[g];
        const float4 v = *(const float4*)(src + g * ld + e);
        acc.x = acc.x + c * v.x; acc.y = acc.y + c * v.y;  // no contraction: see the pragma
        acc.z = acc.z + c * v.z; acc.w = acc.w + c * v.w;
      }
      *(float4*)(out + e) = acc;
    } else {
      for (long long k = e; k < min(n, e + 4); ++k) {
        float acc = accumulate ? out[k] : 0.f;
        for (int g = 0; g < G; ++g) acc = acc + coeff[g] * src[g * ld + k];
        out[k] = acc;
      }
    }
  }
}

DDL_API int ddl_weighted_sum(const float* src, long long ld, const float* coeff, int G, long long n,
                             float* out, int accumulate, hipStream_t s) {
  hipLaunchKernelGGL(weighted_sum_kernel, dim3(grid_for((n + 3) / 4, 256)), dim3(256), 0, s, src,
                     ld, coeff, G, n, out, accumulate);
  return (int)hipGetLastError();
}

__global__ void broadcast_rows_kernel(const float* __restrict__ src, float* __restrict__ dst,
                                      long long ld, int G, long long n, bf16_t* __restrict__ shadow,
                                      long long sld) {
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n;
       e += (long long)gridDim.x * blockDim.x) {
    const float v = src[e];
    const bf16_t b = f2bf(v);
    for (int g = 0; g < G; ++g) {
      dst[g * ld + e] = v;
      if (shadow) shadow[g * sld + e] = b;
    }
  }
}

DDL_API int ddl_broadcast_rows(const float* src, float* dst, long long ld, int G, long long n,
                               void* shadow, long long sld, hipStream_t s) {
  hipLaunchKernelGGL(broadcast_rows_kernel, dim3(grid_for(n, 256)), dim3(256), 0, s, src, dst, ld,
                     G, n, (bf16_t*)shadow, sld);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Gram on exact-fp32 MFMA. X [K][n] (row stride ld), optional center c [n] subtracted on load.
// Block = 256 threads = 4 waves; the block owns a slice of the coordinate axis and computes the
// upper-triangular 16x16 tiles of its partial KP x KP Gram (KP = K rounded up to 16, <= 128; the
// Gram is symmetric, so only ti <= tj tiles: 36 instead of 64 at KP = 128), tiles dealt round-robin
// over the waves. Partials go to a per-block slice of `part` with plain stores, and
// gram_reduce_kernel sums the slices in block order: the K x K result is bit-reproducible (no
// float atomics), which Krum's argsort of scores needs to pick the same clients on every run.
// Staging: LDS tile [KP][CHUNK] fp32 with a +1 float pad per row (conflict-free column reads).
// Chunks of the coordinate axis: 256 columns for KP <= 32 (a small Gram has little MFMA work per
// chunk, so each barrier round should move more bytes), 64 above. The next chunk's elements are
// loaded into registers while the current chunk's MFMAs run (one chunk of prefetch).
constexpr int GRAM_CHUNK = 64;  // the workspace sizing granule (gram_blocks)
template <int KP> constexpr int gram_chunk() { return KP <= 32 ? 256 : 64; }

__host__ __device__ inline int gram_blocks_cap(int KP) { return KP <= 64 ? 1024 : 512; }

template <int KP>
__global__ __launch_bounds__(256) void gram_f32_kernel(const float* __restrict__ X, long long ld,
                                                       const float* __restrict__ center, int K,
                                                       long long n, float* __restrict__ part) {
  constexpr int CH = gram_chunk<KP>();
  constexpr int LDW = CH + 1;
  constexpr int NT = KP / 16;
  constexpr int TILES = NT * (NT + 1) / 2;
  constexpr int TPW = (TILES + 3) / 4;  // tiles per wave
  constexpr int PER = KP * CH / 256;    // staged elements per thread
  __shared__ float tile[KP * LDW];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  int ti_[TPW], tj_[TPW];
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    int idx = wid + 4 * t, ti = 0;
    while (ti < NT && idx >= NT - ti) { idx -= NT - ti; ++ti; }
    ti_[t] = ti;            // ti == NT: this wave has no tile in slot t
    tj_[t] = ti + idx;
  }
  f4v acc[TPW];
#pragma unroll
  for (int i = 0; i < TPW; ++i) acc[i] = (f4v){0.f, 0.f, 0.f, 0.f};
  float nxt[PER];
  auto fetch = [&](long long c0) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int e = tid + i * 256, r = e / CH, c = e - r * CH;
      const long long col = c0 + c;
      float v = 0.f;
      if (r < K && col < n) v = X[r * ld + col] - (center ? center[col] : 0.f);
      nxt[i] = v;
    }
  };
  const long long stride = (long long)gridDim.x * CH;
  long long c0 = (long long)blockIdx.x * CH;
  if (c0 < n) fetch(c0);
  for (; c0 < n; c0 += stride) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int e = tid + i * 256, r = e / CH, c = e - r * CH;
      tile[r * LDW + c] = nxt[i];
    }
    __syncthreads();
    if (c0 + stride < n) fetch(c0 + stride);  // in flight during this chunk's MFMAs
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
      if (ti_[t] < NT) {
        const float* ra = tile + (ti_[t] * 16 + (lane & 15)) * LDW + (lane >> 4);
        const float* rb = tile + (tj_[t] * 16 + (lane & 15)) * LDW + (lane >> 4);
#pragma unroll
        for (int k = 0; k < CH; k += 4)
          // A[i][k] lane: i = lane&15, k = lane>>4 ; B[k][j] lane: j = lane&15, k = lane>>4
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(ra[k], rb[k], acc[t], 0, 0, 0);
      }
    }
  }
  float* mine = part + (long long)blockIdx.x * KP * KP;
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    if (ti_[t] < NT) {
      const int j = tj_[t] * 16 + (lane & 15);
#pragma unroll
      for (int e = 0; e < 4; ++e) mine[(ti_[t] * 16 + 4 * (lane >> 4) + e) * KP + j] = acc[t][e];
    }
  }
}

// out[i][j] = sum over the blocks' partials of the stored tile holding (i, j) or (j, i): one
// block per output element, thread t adding blocks t, t + 256, ... in order, then a fixed LDS tree
// -- a fixed summation order, so the result is bit-reproducible (no float atomics)
__global__ __launch_bounds__(256) void gram_reduce_kernel(const float* __restrict__ part, int blocks, int K,
                                                          int KP, float* __restrict__ out) {
  __shared__ float red[256];
  const int e = blockIdx.x;
  int i = e / K, j = e - (e / K) * K;
  if ((i >> 4) > (j >> 4)) { const int t = i; i = j; j = t; }
  const float* p = part + i * KP + j;
  float s = 0.f;
  for (int b = threadIdx.x; b < blocks; b += 256) s += p[(long long)b * KP * KP];
  red[threadIdx.x] = s;
  __syncthreads();
#pragma unroll
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[e] = red[0];
}

static int gram_kp(int K) { return K <= 16 ? 16 : K <= 32 ? 32 : K <= 48 ? 48 : K <= 64 ? 64 : K <= 96 ? 96 : 128; }

static int gram_blocks(int K, long long n) {
  return grid_for((n + GRAM_CHUNK - 1) / GRAM_CHUNK, 1, gram_blocks_cap(gram_kp(K)));
}

// floats of scratch `ddl_gram_f32` needs for K clients over n coordinates (0: K unsupported)
DDL_API long long ddl_gram_f32_workspace(int K, long long n) {
  if (K < 1 || K > 128 || n < 1) return 0;
  const long long kp = gram_kp(K);
  return (long long)gram_blocks(K, n) * kp * kp;
}

DDL_API int ddl_gram_f32(const float* X, long long ld, const float* center, int K, long long n,
                         float* part, long long part_cap, float* out, hipStream_t s) {
  if (K < 1 || K > 128 || n < 1 || part_cap < ddl_gram_f32_workspace(K, n)) return (int)hipErrorInvalidValue;
  const int blocks = gram_blocks(K, n);
  switch (gram_kp(K)) {
#define GRAM_CASE(KP_) \
    case KP_: hipLaunchKernelGGL(gram_f32_kernel<KP_>, dim3(blocks), dim3(256), 0, s, X, ld, center, K, n, part); break;
    GRAM_CASE(16) GRAM_CASE(32) GRAM_CASE(48) GRAM_CASE(64) GRAM_CASE(96) GRAM_CASE(128)
#undef GRAM_CASE
    default: return (int)hipErrorInvalidValue;
  }
  hipLaunchKernelGGL(gram_reduce_kernel, dim3(K * K), dim3(256), 0, s, part, blocks, K, gram_kp(K), out);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// coordinate-wise selection: mode 0 = median (mean of the two middle values for even K),
// mode 1 = trimmed mean dropping `trim` smallest and `trim` largest.
template <int KP>
__device__ __forceinline__ void bitonic_sort(float (&v)[KP]) {
#pragma unroll
  for (int k = 2; k <= KP; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
#pragma unroll
      for (int i = 0; i < KP; ++i) {
        const int l = i ^ j;
        if (l > i) {
          const bool up = ((i & k) == 0);
          const float a = v[i], b = v[l];
          if ((a > b) == up) { v[i] = b; v[l] = a; }
        }
      }
    }
  }
}

// ascending sort of a bitonic sequence (the half-cleaner cascade)
template <int N>
__device__ __forceinline__ void bitonic_merge(float (&v)[N]) {
#pragma unroll
  for (int j = N >> 1; j > 0; j >>= 1) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int l = i ^ j;
      if (l > i) {
        const float a = v[i], b = v[l];
        v[i] = fminf(a, b);
        v[l] = fmaxf(a, b);
      }
    }
  }
}

// Register-resident sort of KP <= 128 values. Above 64 the network is split: two 64-sorts, one
// cross compare (a[i] vs b[63-i] leaves every a <= every b, both halves bitonic) and two 64-merges,
// so each unrolled loop nest stays small enough to be fully unrolled and the array never leaves
// VGPRs (a single 128-wide network is only partially unrolled and falls back to scratch memory).
template <int KP>
__device__ __forceinline__ void sort_values(float (&v)[KP]) {
  if constexpr (KP <= 64) {
    bitonic_sort<KP>(v);
  } else {
    constexpr int H = KP / 2;
    float (&a)[H] = *reinterpret_cast<float (*)[H]>(v);
    float (&b)[H] = *reinterpret_cast<float (*)[H]>(v + H);
    bitonic_sort<H>(a);
    bitonic_sort<H>(b);
#pragma unroll
    for (int i = 0; i < H; ++i) {
      const float x = a[i], y = b[H - 1 - i];
      a[i] = fminf(x, y);
      b[H - 1 - i] = fmaxf(x, y);
    }
    bitonic_merge<H>(a);
    bitonic_merge<H>(b);
  }
}

template <int KP>
__global__ __launch_bounds__(256) void coord_select_kernel(const float* __restrict__ X, long long ld, int K, long long n,
                                    int mode, int trim, float* __restrict__ out) {
  // one coordinate per thread, no grid-stride loop: a loop would hoist the per-rank selection
  // masks (loop-invariant) out of it and spill ~KP lane masks from the SGPR file
  const long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (e < n) {
    float v[KP];
    const float* p = X + e;  // walk the rows by pointer increments: no per-row 64-bit offsets
#pragma unroll
    for (int i = 0; i < KP; ++i) {
      v[i] = (i < K) ? *p : INFINITY;
      p += (i + 1 < K) ? ld : 0;
    }
    sort_values<KP>(v);
    float r;
    if (mode == 0) {
      const int a = (K - 1) / 2, b = K / 2;
      float va = 0.f, vb = 0.f;
#pragma unroll
      for (int i = 0; i < KP; ++i) {
        if (i == a) va = v[i];
        if (i == b) vb = v[i];
      }
      r = 0.5f * (va + vb);
    } else {
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < KP; ++i)
        if (i >= trim && i < K - trim) s += v[i];
      r = s / (float)(K - 2 * trim);
    }
    out[e] = r;
  }
}

DDL_API int ddl_coord_select(const float* X, long long ld, int K, long long n, int mode, int trim,
                             float* out, hipStream_t s) {
  if (K < 1 || (mode == 1 && K - 2 * trim < 1)) return (int)hipErrorInvalidValue;
  const long long blocks = (n + 255) / 256;
  if (blocks > 0x7fffffffLL) return (int)hipErrorInvalidValue;
#define SEL_CASE(KP_) \
  if (K <= KP_) { \
    hipLaunchKernelGGL(coord_select_kernel<KP_>, dim3(blocks), dim3(256), 0, s, X, ld, K, n, mode, trim, out); \
    return (int)hipGetLastError(); \
  }
  SEL_CASE(8) SEL_CASE(16) SEL_CASE(32) SEL_CASE(64) SEL_CASE(128)
#undef SEL_CASE
  return (int)hipErrorInvalidValue;
}

// ---------------------------------------------------------------------------------------------
// Robust aggregation glue (round 6): the coordinate-sharded rules' all-to-all send buffer in one
// pass, and Krum's scoring / selection / winners' mean on the device without torch sort glue.
//
// send[w][g][s] = rows[g][w * S + s] for g < G and w * S + s < P, else 0 (g < gmax): client rows
// [G][P] (row stride ld) cut into W coordinate shards of S, zero-padded to gmax rows per rank.
__global__ void pack_shards_kernel(const float* __restrict__ rows, long long ld, int G, long long P,
                                   int W, long long S, int gmax, float* __restrict__ send) {
  const long long n = (long long)W * gmax * S;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n;
       e += (long long)gridDim.x * blockDim.x) {
    const long long s = e % S, wg = e / S;
    const int g = (int)(wg % gmax), w = (int)(wg / gmax);
    const long long c = (long long)w * S + s;
    send[e] = (g < G && c < P) ? rows[g * ld + c] : 0.f;
  }
}

DDL_API int ddl_pack_shards(const float* rows, long long ld, int G, long long P, int W, long long S,
                            int gmax, float* send, hipStream_t st) {
  if (W < 1 || S < 1 || gmax < 1 || G > gmax || (long long)W * S < P) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(pack_shards_kernel, dim3(grid_for((long long)W * gmax * S, 256)), dim3(256), 0, st,
                     rows, ld, G, P, W, S, gmax, send);
  return (int)hipGetLastError();
}

// Krum (Blanchard et al. 2017) from the K x K Gram of the client updates: d2[i][j] = g_ii + g_jj -
// 2 g_ij (clamped at 0), score_i = sum of the nb smallest d2[i][j], j != i (ascending order, as a
// sort would add them), sel = the m clients of least score (exact ties to the smaller key: the
// client's global order, so the choice does not depend on the rank layout; default the index). One block, a thread per
// client: its row sorted in registers by the bitonic network above.
template <int KP>
__global__ __launch_bounds__(128) void krum_select_kernel(const float* __restrict__ gram, int K, int nb,
                                                          int m, const int* __restrict__ keys,
                                                          float* __restrict__ scores, int* __restrict__ sel) {
#pragma clang fp contract(off)
  __shared__ float sc[128];
  const int i = threadIdx.x;
  if (i < K) {
    float v[KP];
    const float gii = gram[i * K + i];
#pragma unroll
    for (int j = 0; j < KP; ++j) {
      float d = INFINITY;
      if (j < K && j != i) d = fmaxf(gii + gram[j * K + j] - 2.f * gram[i * K + j], 0.f);
      v[j] = d;
    }
    sort_values<KP>(v);
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < KP; ++j)
      if (j < nb) s += v[j];
    sc[i] = s;
    if (scores) scores[i] = s;
  }
  __syncthreads();
  if (i < K) {
    const float s = sc[i];
    int rank = 0;
    const int ki = keys ? keys[i] : i;
    for (int j = 0; j < K; ++j) rank += (sc[j] < s || (sc[j] == s && (keys ? keys[j] : j) < ki)) ? 1 : 0;
    if (rank < m) sel[rank] = i;
  }
}

DDL_API int ddl_krum_select(const float* gram, int K, int nb, int m, const int* keys, float* scores, int* sel,
                            hipStream_t st) {
  if (K < 1 || K > 128 || nb < 1 || nb > K - 1 + (K == 1) || m < 1 || m > K) return (int)hipErrorInvalidValue;
#define KRUM_CASE(KP_) \
  if (K <= KP_) { \
    hipLaunchKernelGGL(krum_select_kernel<KP_>, dim3(1), dim3(128), 0, st, gram, K, nb, m, keys, scores, sel); \
    return (int)hipGetLastError(); \
  }
  KRUM_CASE(8) KRUM_CASE(16) KRUM_CASE(32) KRUM_CASE(64) KRUM_CASE(128)
#undef KRUM_CASE
  return (int)hipErrorInvalidValue;
}

// out[e] = sum_t (1/m) * X[sel[t]][e], t = 0 .. m-1 in selection order (products rounded, then
// added: the same bits as weighted_sum over the gathered rows)
__global__ void mean_rows_idx_kernel(const float* __restrict__ X, long long ld, const int* __restrict__ sel,
                                     int m, long long n, float* __restrict__ out) {
#pragma clang fp contract(off)
  const float c = 1.f / (float)m;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n;
       e += (long long)gridDim.x * blockDim.x) {
    float acc = 0.f;
    for (int t = 0; t < m; ++t) acc = acc + c * X[(long long)sel[t] * ld + e];
    out[e] = acc;
  }
}

DDL_API int ddl_mean_rows_idx(const float* X, long long ld, const int* sel, int m, long long n, float* out,
                              hipStream_t st) {
  if (m < 1 || n < 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(mean_rows_idx_kernel, dim3(grid_for(n, 256)), dim3(256), 0, st, X, ld, sel, m, n, out);
  return (int)hipGetLastError();
}
