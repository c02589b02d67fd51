// Reference-precision (fp32) kernels of the tiny-LLaMA path (reference lab/tutorial_1b: simplellm
// LLama trained in fp32 — stock modules, Adam, no autocast, intro_PP_1F1B_MB.py:16-46,
// intro_DP_GA.py:16-31). The projections, FFN and LM head run as 1x1 convolutions on the X6 /
// exact-fp32 conv engine (conv_f32.hip); this file holds the rest of the block, fp32 in and out:
//
//   ddl_embf_fwd / bwd    row gather; the backward is DETERMINISTIC: one wave per vocabulary row
//                         scans the token ids (staged in LDS) and adds the matching dY rows in token
//                         order (no float atomics; untouched rows are not written)
//   ddl_rmsf_fwd / bwd    one wave per row (rstd saved); d(gamma) partials per block, folded in a
//                         fixed block order by ddl_rmsf_fold (accumulates into the grad)
//   ddl_swiglu_f32_*      h = silu(a) * b over the fused [a | b] projection
//   ddl_attnf_fwd         causal attention with interleaved RoPE applied as K / Q are staged; four
//                         lanes per query row split the head dimension (dot products finish with
//                         two DPP quad exchanges), online softmax in the exp2 domain, log2-sum-exp
//                         saved
//   ddl_attnf_bwd_dq      recomputes P from the saved lse; delta = rowsum(dO * O) computed here
//   ddl_attnf_bwd_dkdv    one workgroup per 64 keys sweeps the later query tiles (no atomics);
//                         both backward kernels write the un-rotated gradients straight into the
//                         fused dQKV buffer
//   ddl_cevf_rows / fold  vocabulary cross-entropy: per-row loss + d(logits) at unit scale from
//                         one block per row, row losses folded in a fixed order
//   ddl_scale_f32         x *= *g unless *g == 1 (device scalar: no host sync)
#include "ddl_common.h"

// ---------------------------------------------------------------------------------------------
// sum over the 4 lanes of a quad (DPP quad_perm, no LDS traffic); every lane gets the same bits
__device__ __forceinline__ float quad_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, true));  // [1,0,3,2]
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, true));  // [2,3,0,1]
  return v;
}

// ---------------------------------------------------------------------------------------------
// embedding
__global__ void embf_fwd_kernel(const int* __restrict__ idx, const float* __restrict__ w,
                                float* __restrict__ y, int T, int D) {
  const long long n = (long long)T * D;
  GSTRIDE_LOOP(e, n) {
    const int t = (int)(e / D), d = (int)(e - (long long)t * D);
    y[e] = w[(long long)idx[t] * D + d];
  }
}

// Block = 4 waves x EMB_RPW vocabulary rows each; the token ids go through LDS in chunks.
constexpr int EMB_RPW = 4, EMB_CHUNK = 4096, EMB_MAXK = 16;  // D <= 64 * EMB_MAXK
__global__ __launch_bounds__(256) void embf_bwd_kernel(const int* __restrict__ idx,
                                                       const float* __restrict__ dy,
                                                       float* __restrict__ dw, int T, int D, int V,
                                                       int pad_idx) {
  __shared__ int sid[EMB_CHUNK];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int v0 = (blockIdx.x * 4 + wv) * EMB_RPW;
  float acc[EMB_RPW][EMB_MAXK];
  bool hit[EMB_RPW];
#pragma unroll
  for (int r = 0; r < EMB_RPW; ++r) {
    hit[r] = false;
#pragma unroll
    for (int k = 0; k < EMB_MAXK; ++k) acc[r][k] = 0.f;
  }
  const int nk = (D + 63) / 64;
  for (int c0 = 0; c0 < T; c0 += EMB_CHUNK) {
    const int cn = min(EMB_CHUNK, T - c0);
    __syncthreads();
    for (int i = threadIdx.x; i < cn; i += 256) sid[i] = idx[c0 + i];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < EMB_RPW; ++r) {
      const int v = v0 + r;
      if (v >= V || v == pad_idx) continue;
      for (int i0 = 0; i0 < cn; i0 += 64) {
        const int i = i0 + lane;
        unsigned long long m = __ballot(i < cn && sid[i] == v);
        while (m) {
          const int t = c0 + i0 + __builtin_ctzll(m);
          m &= m - 1;
          hit[r] = true;
          const float* src = dy + (long long)t * D;
#pragma unroll
          for (int k = 0; k < EMB_MAXK; ++k)
            if (k < nk && lane + 64 * k < D) acc[r][k] += src[lane + 64 * k];
        }
      }
    }
  }
#pragma unroll
  for (int r = 0; r < EMB_RPW; ++r) {
    const int v = v0 + r;
    if (!hit[r] || v >= V) continue;
    float* dst = dw + (long long)v * D;
#pragma unroll
    for (int k = 0; k < EMB_MAXK; ++k)
      if (k < nk && lane + 64 * k < D) dst[lane + 64 * k] += acc[r][k];
  }
}

// Block = RB consecutive vocabulary rows accumulated in LDS; the token ids go through LDS in
// chunks, wave 0 compacts a chunk's matching tokens in token order, and the block adds their dy
// rows in that order (8 rows' loads in flight) — per element the same adds, in the same order, as
// embf_bwd_kernel, whose waves each rescanned every id for 4 rows (210 us at 8192 tokens x 32k
// vocabulary; this kernel scans the ids once per RB rows).
constexpr int EMBR_CHUNK = 2048, EMBR_MAXJ = 4;  // D <= 256 * EMBR_MAXJ
__global__ __launch_bounds__(256) void embf_bwd_rows_kernel(const int* __restrict__ idx,
                                                            const float* __restrict__ dy,
                                                            float* __restrict__ dw, int T, int D, int V,
                                                            int pad_idx, int RB) {
  extern __shared__ float emb_smem[];
  float* acc = emb_smem;                    // [RB][D]
  int* sid = (int*)(acc + RB * D);          // ids of the chunk
  int* lt = sid + EMBR_CHUNK;               // matched tokens, token order
  int* lr = lt + EMBR_CHUNK;                // their rows (id - v0)
  __shared__ int nmatch;
  __shared__ unsigned long long hits;
  const int tid = threadIdx.x, lane = tid & 63;
  const int v0 = blockIdx.x * RB;
  for (int e = tid; e < RB * D; e += 256) acc[e] = 0.f;
  if (tid == 0) hits = 0ull;
  for (int c0 = 0; c0 < T; c0 += EMBR_CHUNK) {
    const int cn = min(EMBR_CHUNK, T - c0);
    __syncthreads();
    int ids[EMBR_CHUNK / 256];
#pragma unroll
    for (int q = 0; q < EMBR_CHUNK / 256; ++q) {
      const int i = tid + 256 * q;
      ids[q] = i < cn ? idx[c0 + i] : -1;
    }
#pragma unroll
    for (int q = 0; q < EMBR_CHUNK / 256; ++q) sid[tid + 256 * q] = ids[q];
    __syncthreads();
    if (tid < 64) {  // wave 0: ordered compaction of the matches
      int n = 0;
      unsigned long long h = 0ull;
      for (int i0 = 0; i0 < cn; i0 += 64) {
        const int i = i0 + lane;
        const int v = i < cn ? sid[i] : -1;
        const bool m = v >= v0 && v < v0 + RB && v < V && v != pad_idx;
        const unsigned long long b = __ballot(m);
        if (m) {
          const int pos = n + __popcll(b & ((1ull << lane) - 1ull));
          lt[pos] = c0 + i;
          lr[pos] = v - v0;
          h |= 1ull << (v - v0);
        }
        n += __popcll(b);
      }
      if (lane == 0) nmatch = n;  // (every lane holds n; each ORs in the rows it matched)
      atomicOr(&hits, h);
    }
    __syncthreads();
    const int n = nmatch;
    for (int b0 = 0; b0 < n; b0 += 8) {
      float val[8][EMBR_MAXJ];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int t = b0 + q < n ? lt[b0 + q] : -1;
#pragma unroll
        for (int j = 0; j < EMBR_MAXJ; ++j) {
          const int d = tid + 256 * j;
          val[q][j] = (t >= 0 && d < D) ? dy[(long long)t * D + d] : 0.f;
        }
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        if (b0 + q >= n) break;
        const int r = lr[b0 + q];
#pragma unroll
        for (int j = 0; j < EMBR_MAXJ; ++j) {
          const int d = tid + 256 * j;
          if (d < D) acc[r * D + d] += val[q][j];
        }
      }
    }
  }
  __syncthreads();
  const unsigned long long h = hits;
  for (int r = 0; r < RB; ++r) {
    if (!((h >> r) & 1ull)) continue;
    float* dst = dw + (long long)(v0 + r) * D;
    for (int d = tid; d < D; d += 256) dst[d] += acc[r * D + d];
  }
}

DDL_API int ddl_embf_fwd(const int* idx, const float* w, float* y, int T, int D, hipStream_t s) {
  if (T < 1 || D < 1) return 0;
  hipLaunchKernelGGL(embf_fwd_kernel, dim3(grid_for((long long)T * D, 256)), dim3(256), 0, s, idx, w, y, T, D);
  return (int)hipGetLastError();
}

DDL_API int ddl_embf_bwd(const int* idx, const float* dy, float* dw, int T, int D, int V, int pad_idx,
                         hipStream_t s) {
  if (D > 64 * EMB_MAXK || D < 1) return (int)hipErrorInvalidValue;
  if (T < 1) return 0;
  // rows per block: the largest power of two <= 64 whose LDS accumulators fit 40 KB (with the id
  // and match lists: <= 64 KB of dynamic LDS)
  int RB = 64;
  while (RB > 1 && RB * D * 4 > 40 * 1024) RB >>= 1;
  if (D <= 256 * EMBR_MAXJ && RB >= 8) {
    const size_t lds = (size_t)RB * D * 4 + 3 * EMBR_CHUNK * 4;
    hipLaunchKernelGGL(embf_bwd_rows_kernel, dim3((V + RB - 1) / RB), dim3(256), lds, s, idx, dy, dw, T, D, V,
                       pad_idx, RB);
    return (int)hipGetLastError();
  }
  const int rows_per_block = 4 * EMB_RPW;
  hipLaunchKernelGGL(embf_bwd_kernel, dim3((V + rows_per_block - 1) / rows_per_block), dim3(256), 0, s, idx, dy,
                     dw, T, D, V, pad_idx);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// RMSNorm: y = x * rstd * g, rstd = 1 / sqrt(mean(x^2) + eps). One wave per row; a lane keeps its
// float4 slices of the row in registers (D % 4 == 0, D <= 256 * RMS_MAXV).
constexpr int RMS_MAXV = 8;
__global__ __launch_bounds__(256) void rmsf_fwd_kernel(const float* __restrict__ x, const float* __restrict__ g,
                                                       float* __restrict__ y, float* __restrict__ rstd, int T,
                                                       int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= T) return;
  const int D4 = D / 4;
  const float4* xr = (const float4*)(x + (long long)row * D);
  float4 v[RMS_MAXV];
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < RMS_MAXV; ++k) {
    const int c = lane + 64 * k;
    v[k] = c < D4 ? xr[c] : make_float4(0.f, 0.f, 0.f, 0.f);
    ss += v[k].x * v[k].x + v[k].y * v[k].y + v[k].z * v[k].z + v[k].w * v[k].w;
  }
  ss = wave_sum(ss);
  const float r = 1.f / sqrtf(ss / (float)D + eps);
  if (lane == 0) rstd[row] = r;
  float4* yr = (float4*)(y + (long long)row * D);
  const float4* g4 = (const float4*)g;
#pragma unroll
  for (int k = 0; k < RMS_MAXV; ++k) {
    const int c = lane + 64 * k;
    if (c < D4) {
      const float4 gg = g4[c];
      yr[c] = make_float4(v[k].x * r * gg.x, v[k].y * r * gg.y, v[k].z * r * gg.z, v[k].w * r * gg.w);
    }
  }
}

// dx = r*g*dy - x * r^3 * sum(g*dy*x) / D (+ dres);  part[block][d] = sum over the block's rows of
// dy*x*r (fixed row order per wave, waves combined in a fixed order). KV float4 slots per lane
// (D <= 256 * KV); a wave loads RG rows' x / dy before using any of them, so RG rows' loads are in
// flight at once (one row at a time waited a full HBM round trip per row: 18.9 us at T = 8192).
template <int KV, int RMS_RG = 8 / KV>
__global__ __launch_bounds__(256) void rmsf_bwd_kernel(const float* __restrict__ x, const float* __restrict__ g,
                                                       const float* __restrict__ rstd,
                                                       const float* __restrict__ dy,
                                                       const float* __restrict__ dres, float* __restrict__ dx,
                                                       float* __restrict__ part, int T, int D, int rows_per_block) {
  __shared__ float4 sdg[4][64 * KV];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int D4 = D / 4;
  const float4* g4 = (const float4*)g;
  float4 dg[KV], gg[KV];
#pragma unroll
  for (int k = 0; k < KV; ++k) {
    const int c = lane + 64 * k;
    dg[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    gg[k] = c < D4 ? g4[c] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  const int r0 = blockIdx.x * rows_per_block, r1 = min(T, r0 + rows_per_block);
  for (int rb = r0 + wv; rb < r1; rb += 4 * RMS_RG) {
    float4 xv[RMS_RG][KV], dv[RMS_RG][KV];
    float r[RMS_RG];
#pragma unroll
    for (int i = 0; i < RMS_RG; ++i) {
      const int row = rb + 4 * i;
      const bool rin = row < r1;
      const float4* xr = (const float4*)(x + (long long)row * D);
      const float4* dr = (const float4*)(dy + (long long)row * D);
      r[i] = rin ? rstd[row] : 0.f;
#pragma unroll
      for (int k = 0; k < KV; ++k) {
        const int c = lane + 64 * k;
        const bool in = rin && c < D4;
        xv[i][k] = in ? xr[c] : make_float4(0.f, 0.f, 0.f, 0.f);
        dv[i][k] = in ? dr[c] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
#pragma unroll
    for (int i = 0; i < RMS_RG; ++i) {
      const int row = rb + 4 * i;
      if (row >= r1) break;  // wave-uniform
      float sm = 0.f;
#pragma unroll
      for (int k = 0; k < KV; ++k)
        sm += gg[k].x * dv[i][k].x * xv[i][k].x + gg[k].y * dv[i][k].y * xv[i][k].y +
              gg[k].z * dv[i][k].z * xv[i][k].z + gg[k].w * dv[i][k].w * xv[i][k].w;
      sm = wave_sum(sm);
      const float rr = r[i];
      const float c3 = rr * rr * rr * sm / (float)D;
      float4* out = (float4*)(dx + (long long)row * D);
      const float4* rs = dres ? (const float4*)(dres + (long long)row * D) : nullptr;
#pragma unroll
      for (int k = 0; k < KV; ++k) {
        const int c = lane + 64 * k;
        if (c >= D4) continue;
        float4 o = make_float4(rr * gg[k].x * dv[i][k].x - xv[i][k].x * c3, rr * gg[k].y * dv[i][k].y - xv[i][k].y * c3,
                               rr * gg[k].z * dv[i][k].z - xv[i][k].z * c3, rr * gg[k].w * dv[i][k].w - xv[i][k].w * c3);
        if (rs) {
          const float4 q = rs[c];
          o.x += q.x; o.y += q.y; o.z += q.z; o.w += q.w;
        }
        out[c] = o;
        dg[k].x += dv[i][k].x * xv[i][k].x * rr; dg[k].y += dv[i][k].y * xv[i][k].y * rr;
        dg[k].z += dv[i][k].z * xv[i][k].z * rr; dg[k].w += dv[i][k].w * xv[i][k].w * rr;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < KV; ++k) sdg[wv][lane + 64 * k] = dg[k];
  __syncthreads();
  float4* p = (float4*)(part + (long long)blockIdx.x * D);
  for (int c = threadIdx.x; c < D4; c += 256) {
    float4 a = sdg[0][c];
#pragma unroll
    for (int w = 1; w < 4; ++w) {
      const float4 b = sdg[w][c];
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
    p[c] = a;
  }
}

// d(gamma) fold: a block per 16 columns, 16 slices per column (slice s sums the partials of blocks
// s, s + 16, ... in order, every load of a thread in flight at once), then the slices in a fixed
// tree order: deterministic. One thread per column summing all partials serially ran on 2
// workgroups at D = 288 (8.4 us).
constexpr int RMSF_FOLD_COLS = 16, RMSF_FOLD_SLICES = 16;
__global__ __launch_bounds__(256) void rmsf_fold_kernel(const float* __restrict__ part, float* __restrict__ dg, int nb,
                                                        int D, int accumulate) {
  __shared__ float red[RMSF_FOLD_SLICES][RMSF_FOLD_COLS];
  const int cl = threadIdx.x % RMSF_FOLD_COLS, sl = threadIdx.x / RMSF_FOLD_COLS;
  const int d = blockIdx.x * RMSF_FOLD_COLS + cl;
  float s = 0.f;
  if (d < D) {
    int b = sl;
    for (; b + 7 * RMSF_FOLD_SLICES < nb; b += 8 * RMSF_FOLD_SLICES) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = part[(long long)(b + j * RMSF_FOLD_SLICES) * D + d];
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[j];
    }
    for (; b < nb; b += RMSF_FOLD_SLICES) s += part[(long long)b * D + d];
  }
  red[sl][cl] = s;
  __syncthreads();
#pragma unroll
  for (int h = RMSF_FOLD_SLICES / 2; h > 0; h >>= 1) {
    if (sl < h) red[sl][cl] += red[sl + h][cl];
    __syncthreads();
  }
  if (sl == 0 && d < D) dg[d] = accumulate ? dg[d] + red[0][cl] : red[0][cl];
}

DDL_API int ddl_rmsf_fwd(const float* x, const float* g, float* y, float* rstd, int T, int D, float eps,
                         hipStream_t s) {
  if (D % 4 || D > 256 * RMS_MAXV) return (int)hipErrorInvalidValue;
  if (T < 1) return 0;
  hipLaunchKernelGGL(rmsf_fwd_kernel, dim3((T + 3) / 4), dim3(256), 0, s, x, g, y, rstd, T, D, eps);
  return (int)hipGetLastError();
}

// blocks of the backward grid for T rows (the d(gamma) partial buffer holds nb x D floats)
DDL_API int ddl_rmsf_blocks(int T) {
  // ~512 workgroups (two per CU) at large T: each wave then holds its rows' loads in flight at once
  const int rpb = T <= 2048 ? 4 : ((T + 511) / 512 + 3) / 4 * 4;
  return (T + rpb - 1) / rpb;
}

DDL_API int ddl_rmsf_bwd(const float* x, const float* g, const float* rstd, const float* dy, const float* dres,
                         float* dx, float* part, float* dg, int accumulate, int T, int D, hipStream_t s) {
  if (D % 4 || D > 256 * RMS_MAXV) return (int)hipErrorInvalidValue;
  if (T < 1) return 0;
  const int nb = ddl_rmsf_blocks(T);
  const int rpb = (T + nb - 1) / nb;
  const int kv = (D / 4 + 63) / 64;
  if (kv <= 2)
    hipLaunchKernelGGL(rmsf_bwd_kernel<2>, dim3(nb), dim3(256), 0, s, x, g, rstd, dy, dres, dx, part, T, D, rpb);
  else if (kv <= 4)
    hipLaunchKernelGGL(rmsf_bwd_kernel<4>, dim3(nb), dim3(256), 0, s, x, g, rstd, dy, dres, dx, part, T, D, rpb);
  else
    hipLaunchKernelGGL(rmsf_bwd_kernel<RMS_MAXV>, dim3(nb), dim3(256), 0, s, x, g, rstd, dy, dres, dx, part, T, D,
                       rpb);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || !dg) return (int)e;
  hipLaunchKernelGGL(rmsf_fold_kernel, dim3((D + RMSF_FOLD_COLS - 1) / RMSF_FOLD_COLS), dim3(256), 0, s, part, dg, nb,
                     D, accumulate);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// SwiGLU over ab [T][2F] = [a | b]  ->  h [T][F]
__device__ __forceinline__ float sigm(float a) { return 1.f / (1.f + expf(-a)); }

__global__ void swiglu_f32_fwd_kernel(const float* __restrict__ ab, float* __restrict__ h, int T, int F) {
  const long long n = (long long)T * F;
  GSTRIDE_LOOP(e, n) {
    const long long t = e / F, f = e - t * F;
    const float a = ab[t * 2 * F + f], b = ab[t * 2 * F + F + f];
    h[e] = a * sigm(a) * b;
  }
}

__global__ void swiglu_f32_bwd_kernel(const float* __restrict__ ab, const float* __restrict__ dh,
                                      float* __restrict__ dab, int T, int F) {
  const long long n = (long long)T * F;
  GSTRIDE_LOOP(e, n) {
    const long long t = e / F, f = e - t * F;
    const float a = ab[t * 2 * F + f], b = ab[t * 2 * F + F + f], d = dh[e];
    const float sg = sigm(a), si = a * sg;
    dab[t * 2 * F + f] = d * b * sg * (1.f + a * (1.f - sg));
    dab[t * 2 * F + F + f] = d * si;
  }
}

DDL_API int ddl_swiglu_f32_fwd(const float* ab, float* h, int T, int F, hipStream_t s) {
  if (T < 1 || F < 1) return 0;
  hipLaunchKernelGGL(swiglu_f32_fwd_kernel, dim3(grid_for((long long)T * F, 256)), dim3(256), 0, s, ab, h, T, F);
  return (int)hipGetLastError();
}

DDL_API int ddl_swiglu_f32_bwd(const float* ab, const float* dh, float* dab, int T, int F, hipStream_t s) {
  if (T < 1 || F < 1) return 0;
  hipLaunchKernelGGL(swiglu_f32_bwd_kernel, dim3(grid_for((long long)T * F, 256)), dim3(256), 0, s, ab, dh, dab,
                     T, F);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Causal attention, fp32. qkv [B][S][3][H][HD], o / dO [B][S][H][HD], lse / delta [B][H][S]
// (lse in the log2 domain of the scaled scores), cos / sin [S][HD/2] (interleaved pairs). HD a
// multiple of 16. A workgroup owns 64 rows of one (b, h), 16 per wave; every product runs on the
// exact-fp32 MFMA (see "MFMA attention" below). Reference: the LLaMA of the labs trains in fp32
// (lab/tutorial_1b/PP/1F1B/intro_PP_1F1B_MB.py:16-46).
constexpr float LOG2E = 1.4426950408889634f;
constexpr int ATT_R = 64;

template <int DPT>
__device__ __forceinline__ void load_slice(const float* p, float (&v)[DPT]) {
#pragma unroll
  for (int m = 0; m < DPT; m += 4) {
    const float4 f = *(const float4*)(p + m);
    v[m] = f.x; v[m + 1] = f.y; v[m + 2] = f.z; v[m + 3] = f.w;
  }
}
template <int DPT>
__device__ __forceinline__ void store_slice(float* p, const float (&v)[DPT]) {
#pragma unroll
  for (int m = 0; m < DPT; m += 4) *(float4*)(p + m) = make_float4(v[m], v[m + 1], v[m + 2], v[m + 3]);
}
// rotate dims d0.. of a row at position pos in place (dir = +1 forward, -1 inverse: the gradient)
template <int DPT>
__device__ __forceinline__ void rope_slice(float (&v)[DPT], const float* cs, const float* sn, int d0, int dir) {
#pragma unroll
  for (int m = 0; m < DPT; m += 2) {
    const float c = cs[(d0 + m) >> 1], s = dir * sn[(d0 + m) >> 1];
    const float a = v[m], b = v[m + 1];
    v[m] = a * c - b * s;
    v[m + 1] = a * s + b * c;
  }
}

// Stage rows r0..r0+63 of one (b, h) into LDS img[64][HD] (rows >= S zero), optionally rotated.
template <int HD>
__device__ __forceinline__ void stage_rows(float* img, const float* base, long long rstride, int r0, int S,
                                           const float* cosb, const float* sinb, bool rope) {
  constexpr int N4 = ATT_R * HD / 4;
  for (int e = threadIdx.x; e < N4; e += 256) {
    const int r = e / (HD / 4), d = (e - r * (HD / 4)) * 4;
    const int row = r0 + r;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (row < S) {
      v = *(const float4*)(base + row * rstride + d);
      if (rope) {
        const float* cs = cosb + (long long)row * (HD / 2) + d / 2;
        const float* sn = sinb + (long long)row * (HD / 2) + d / 2;
        const float a0 = v.x * cs[0] - v.y * sn[0], a1 = v.x * sn[0] + v.y * cs[0];
        const float b0 = v.z * cs[1] - v.w * sn[1], b1 = v.z * sn[1] + v.w * cs[1];
        v = make_float4(a0, a1, b0, b1);
      }
    }
    *(float4*)(img + r * HD + d) = v;
  }
}

// ---- MFMA attention (exact fp32 products: v_mfma_f32_16x16x4_f32, the fmaf-chain of fp32) ----
// A wave owns 16 rows (queries, or keys in the dK/dV kernel) of a 64-row workgroup tile; the
// other side is staged 64 rows at a time in LDS (RoPE applied while staging), rows padded to
// HD + 4 floats (conflict-free: 16 rows x 4-float chunks cover the 64 banks). Operand maps of the
// 16x16x4 MFMA: lane l = 16g + n supplies A[m = n][k = g], B[k = g][n]; D holds rows 4g + i,
// column n. The MFMA sums its 4 k-slots in any order, so a product may assign its reduction index
// to (slot g, step j) freely as long as A and B agree:
//   * reductions over the head dim use d = (HD/4) g + j: each lane reads HD/4 CONTIGUOUS dims
//     (float4 LDS reads; its own row's slice kept in registers);
//   * reductions over keys / queries use the index 4g + j of the preceding product's D layout,
//     so P / dS feed the next MFMA straight from their registers (register j), no transpose.
// Forward and dQ compute S^T = K Q^T (D: key 4g+i, query n: the softmax runs down a column —
// 4 values in-lane + two xor-shuffles — and the per-query statistics are one value per lane);
// dK/dV computes S = Q K^T (D: query 4g+i, key n).
typedef float f4m __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f4m mfma4(float a, float b, f4m c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }
__device__ __forceinline__ float colmax(float v) {  // over the 4 lane groups of a column
  v = fmaxf(v, __shfl_xor(v, 16));
  return fmaxf(v, __shfl_xor(v, 32));
}
__device__ __forceinline__ float colsum(float v) {
  v += __shfl_xor(v, 16);
  return v + __shfl_xor(v, 32);
}

// Stage rows r0..r0+63 of one (b, h) into LDS img[64][HD + 4] (rows >= S zero), optionally rotated.
template <int HD>
__device__ __forceinline__ void stage_rows_p(float* img, const float* base, long long rstride, int r0, int S,
                                             const float* cosb, const float* sinb, bool rope) {
  constexpr int N4 = ATT_R * HD / 4, HP = HD + 4;
  for (int e = threadIdx.x; e < N4; e += 256) {
    const int r = e / (HD / 4), d = (e - r * (HD / 4)) * 4;
    const int row = r0 + r;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (row < S) {
      v = *(const float4*)(base + row * rstride + d);
      if (rope) {
        const float* cs = cosb + (long long)row * (HD / 2) + d / 2;
        const float* sn = sinb + (long long)row * (HD / 2) + d / 2;
        const float a0 = v.x * cs[0] - v.y * sn[0], a1 = v.x * sn[0] + v.y * cs[0];
        const float b0 = v.z * cs[1] - v.w * sn[1], b1 = v.z * sn[1] + v.w * cs[1];
        v = make_float4(a0, a1, b0, b1);
      }
    }
    *(float4*)(img + r * HP + d) = v;
  }
}

// Stage rows r0..r0+63 of one (b, h) TRANSPOSED into LDS imgT[HD][ATT_R + 4] (rows >= S zero), so
// a lane reads 4 consecutive rows of one dim as one float4 (accum_rows_t).
template <int HD>
__device__ __forceinline__ void stage_rows_t(float* imgT, const float* base, long long rstride, int r0, int S,
                                             const float* cosb = nullptr, const float* sinb = nullptr,
                                             bool rope = false) {
  constexpr int N4 = ATT_R * HD / 4, KP = ATT_R + 4;
  for (int e = threadIdx.x; e < N4; e += 256) {
    const int r = e % ATT_R, d = (e / ATT_R) * 4;  // consecutive threads: consecutive rows
    const int row = r0 + r;
    float4 v = row < S ? *(const float4*)(base + row * rstride + d) : make_float4(0.f, 0.f, 0.f, 0.f);
    if (rope && row < S) {
      const float* cs = cosb + (long long)row * (HD / 2) + d / 2;
      const float* sn = sinb + (long long)row * (HD / 2) + d / 2;
      const float a0 = v.x * cs[0] - v.y * sn[0], a1 = v.x * sn[0] + v.y * cs[0];
      const float b0 = v.z * cs[1] - v.w * sn[1], b1 = v.z * sn[1] + v.w * cs[1];
      v = make_float4(a0, a1, b0, b1);
    }
    imgT[(d + 0) * KP + r] = v.x;
    imgT[(d + 1) * KP + r] = v.y;
    imgT[(d + 2) * KP + r] = v.z;
    imgT[(d + 3) * KP + r] = v.w;
  }
}

// accum_rows over a transposed tile: acc[db] += sum_j tileT[16 db + n][rb + 4g + j] * w_j, the four
// rows of a lane in one float4 read (accum_rows: one scalar LDS read per MFMA)
template <int HD>
__device__ __forceinline__ void accum_rows_t(f4m (&acc)[HD / 16], const float* tileT, int rb, const float (&w)[4],
                                             int g, int n) {
  constexpr int KP = ATT_R + 4;
#pragma unroll
  for (int db = 0; db < HD / 16; ++db) {
    const float4 t = *(const float4*)(tileT + (16 * db + n) * KP + rb + 4 * g);
    acc[db] = mfma4(t.x, w[0], acc[db]);
    acc[db] = mfma4(t.y, w[1], acc[db]);
    acc[db] = mfma4(t.z, w[2], acc[db]);
    acc[db] = mfma4(t.w, w[3], acc[db]);
  }
}

// a lane's own slice: row `row` (clamped), dims [(HD/4) g, (HD/4)(g+1)), optionally rotated
template <int HD>
__device__ __forceinline__ void own_slice(float (&v)[HD / 4], const float* base, long long rstride, int row, int g,
                                          const float* cosb, const float* sinb, bool rope) {
  constexpr int DQ = HD / 4;
  load_slice<DQ>(base + row * rstride + g * DQ, v);
  if (rope) rope_slice<DQ>(v, cosb + (long long)row * (HD / 2), sinb + (long long)row * (HD / 2), g * DQ, 1);
}

// one 16x16 block of X Y^T over the head dim: A rows from LDS (row-major, padded), B = own slice
template <int HD>
__device__ __forceinline__ f4m dot_block(const float* arow, const float (&bv)[HD / 4], int g) {
  constexpr int DQ = HD / 4;
  f4m c = (f4m){0.f, 0.f, 0.f, 0.f};
  const float* a = arow + g * DQ;
#pragma unroll
  for (int j = 0; j < DQ; j += 4) {
    const float4 av = *(const float4*)(a + j);
    c = mfma4(av.x, bv[j], c);
    c = mfma4(av.y, bv[j + 1], c);
    c = mfma4(av.z, bv[j + 2], c);
    c = mfma4(av.w, bv[j + 3], c);
  }
  return c;
}

// acc[db] += T^T-block: sum over the 16 rows r = 4g + j of an LDS tile (rows rb..rb+15) of
// tile[r][16 db + n] * w_j (w = the lane's D-layout values of the preceding product)
template <int HD>
__device__ __forceinline__ void accum_rows(f4m (&acc)[HD / 16], const float* tile, int rb, const float (&w)[4], int g,
                                           int n) {
  constexpr int HP = HD + 4;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float* r = tile + (rb + 4 * g + j) * HP + n;
#pragma unroll
    for (int db = 0; db < HD / 16; ++db) acc[db] = mfma4(r[16 * db], w[j], acc[db]);
  }
}

// store D-layout blocks (d = 16 db + 4 g + i of row `row`), optionally scaled / inverse-rotated
template <int HD>
__device__ __forceinline__ void store_blocks(float* dst, f4m (&acc)[HD / 16], int g, float mul, const float* cs,
                                             const float* sn) {
#pragma unroll
  for (int db = 0; db < HD / 16; ++db) {
    const int d = 16 * db + 4 * g;
    float v[4] = {acc[db][0] * mul, acc[db][1] * mul, acc[db][2] * mul, acc[db][3] * mul};
    if (cs) {
#pragma unroll
      for (int i = 0; i < 4; i += 2) {
        const float c = cs[(d + i) >> 1], sv = -sn[(d + i) >> 1];
        const float a = v[i], b = v[i + 1];
        v[i] = a * c - b * sv;
        v[i + 1] = a * sv + b * c;
      }
    }
    *(float4*)(dst + d) = make_float4(v[0], v[1], v[2], v[3]);
  }
}

template <int HD>
__global__ __launch_bounds__(256) void attnf_fwd_kernel(const float* __restrict__ qkv, float* __restrict__ o,
                                                        float* __restrict__ lse, const float* __restrict__ cosb,
                                                        const float* __restrict__ sinb, int S, int H,
                                                        float sl2) {
  constexpr int HP = HD + 4, NDB = HD / 16, KP = ATT_R + 4;
  __shared__ __attribute__((aligned(16))) float Ks[ATT_R * HP], Vt[HD * KP];
  int qb, h, b;
  xcd_spread_block(qb, h, b);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, n = lane & 15;
  const int q = qb * ATT_R + 16 * w + n, qc = min(q, S - 1);
  const long long rs = 3LL * H * HD;
  const float* qbase = qkv + (long long)b * S * rs + (long long)h * HD;
  const float* kbase = qbase + (long long)H * HD;
  const float* vbase = qbase + 2LL * H * HD;
  float qf[HD / 4];
  own_slice<HD>(qf, qbase, rs, qc, g, cosb, sinb, true);
  f4m oacc[NDB];
#pragma unroll
  for (int db = 0; db < NDB; ++db) oacc[db] = (f4m){0.f, 0.f, 0.f, 0.f};
  float mx = -INFINITY, l = 0.f;
  for (int kt = 0; kt <= qb; ++kt) {
    __syncthreads();
    stage_rows_p<HD>(Ks, kbase, rs, kt * ATT_R, S, cosb, sinb, true);
    stage_rows_t<HD>(Vt, vbase, rs, kt * ATT_R, S);
    __syncthreads();
    // the tile's 16-key sub-tiles at or below this wave's diagonal: all scores first, then one
    // max / sum exchange per 64-key tile (per 16-key sub-tile: four cross-lane shuffles each)
    const int nu = kt < qb ? 4 : w + 1;
    float sc[4][4], tmax = -INFINITY;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (u < nu) {
        const f4m st = dot_block<HD>(Ks + (16 * u + n) * HP, qf, g);  // S^T[key 4g+i][query n]
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int key = kt * ATT_R + 16 * u + 4 * g + i;
          sc[u][i] = (key <= q && key < S) ? st[i] * sl2 : -INFINITY;
          tmax = fmaxf(tmax, sc[u][i]);
        }
      }
    }
    const float nm = fmaxf(mx, colmax(tmax));  // finite: key 0 is valid for every query
    const float corr = exp2f(mx - nm);
    float p[4][4], ps = 0.f;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (u < nu) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          p[u][i] = exp2f(sc[u][i] - nm);
          ps += p[u][i];
        }
      }
    }
    l = l * corr + colsum(ps);
    mx = nm;
#pragma unroll
    for (int db = 0; db < NDB; ++db) oacc[db] *= corr;
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (u < nu) accum_rows_t<HD>(oacc, Vt, 16 * u, p[u], g, n);  // O^T[d][query n] += V^T P^T
  }
  if (q >= S) return;
  store_blocks<HD>(o + ((long long)(b * S + q) * H + h) * HD, oacc, g, 1.f / l, nullptr, nullptr);
  if (g == 0) lse[((long long)b * H + h) * S + q] = mx + log2f(l);
}

// dQ (and delta = rowsum(dO * O)): a wave's 16 queries over the key tiles 0..qb
template <int HD>
__global__ __launch_bounds__(256) void attnf_bwd_dq_kernel(const float* __restrict__ qkv, const float* __restrict__ o,
                                                           const float* __restrict__ dout,
                                                           const float* __restrict__ lse, float* __restrict__ delta,
                                                           float* __restrict__ dqkv, const float* __restrict__ cosb,
                                                           const float* __restrict__ sinb, int S, int H, float sl2,
                                                           float scale) {
  constexpr int HP = HD + 4, NDB = HD / 16, DQ = HD / 4;
  __shared__ __attribute__((aligned(16))) float Ks[ATT_R * HP], Vs[ATT_R * HP];
  int qb, h, b;
  xcd_spread_block(qb, h, b);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, n = lane & 15;
  const int q = qb * ATT_R + 16 * w + n, qc = min(q, S - 1);
  const long long rs = 3LL * H * HD, ors = (long long)H * HD;
  const float* qbase = qkv + (long long)b * S * rs + (long long)h * HD;
  const float* kbase = qbase + (long long)H * HD;
  const float* vbase = qbase + 2LL * H * HD;
  const float* obase = o + (long long)b * S * ors + (long long)h * HD;
  const float* dbase = dout + (long long)b * S * ors + (long long)h * HD;
  float qf[DQ], df[DQ], of[DQ];
  own_slice<HD>(qf, qbase, rs, qc, g, cosb, sinb, true);
  own_slice<HD>(df, dbase, ors, qc, g, cosb, sinb, false);
  own_slice<HD>(of, obase, ors, qc, g, cosb, sinb, false);
  float dl = 0.f;
#pragma unroll
  for (int j = 0; j < DQ; ++j) dl += df[j] * of[j];
  dl = colsum(dl);
  const long long li = ((long long)b * H + h) * S + qc;
  const float L = lse[li];
  if (g == 0 && q < S) delta[li] = dl;
  f4m dq[NDB];
#pragma unroll
  for (int db = 0; db < NDB; ++db) dq[db] = (f4m){0.f, 0.f, 0.f, 0.f};
  for (int kt = 0; kt <= qb; ++kt) {
    __syncthreads();
    stage_rows_p<HD>(Ks, kbase, rs, kt * ATT_R, S, cosb, sinb, true);
    stage_rows_p<HD>(Vs, vbase, rs, kt * ATT_R, S, cosb, sinb, false);
    __syncthreads();
    const int nu = kt < qb ? 4 : w + 1;
    for (int u = 0; u < nu; ++u) {
      const f4m st = dot_block<HD>(Ks + (16 * u + n) * HP, qf, g);   // S^T
      const f4m dpt = dot_block<HD>(Vs + (16 * u + n) * HP, df, g);  // dP^T = V dO^T
      float ds[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int key = kt * ATT_R + 16 * u + 4 * g + i;
        const float pv = (key <= q && key < S) ? exp2f(st[i] * sl2 - L) : 0.f;
        ds[i] = pv * (dpt[i] - dl);
      }
      accum_rows<HD>(dq, Ks, 16 * u, ds, g, n);  // dQ^T[d][query n] += K^T dS^T
    }
  }
  if (q >= S) return;
  store_blocks<HD>(dqkv + (long long)(b * S + q) * rs + (long long)h * HD, dq, g, scale,
                   cosb + (long long)q * (HD / 2), sinb + (long long)q * (HD / 2));
}

// dK, dV: a wave's 16 keys over the query tiles kb..end (causal: queries >= key)
template <int HD>
__global__ __launch_bounds__(256) void attnf_bwd_dkdv_kernel(const float* __restrict__ qkv,
                                                             const float* __restrict__ dout,
                                                             const float* __restrict__ lse,
                                                             const float* __restrict__ delta,
                                                             float* __restrict__ dqkv, const float* __restrict__ cosb,
                                                             const float* __restrict__ sinb, int S, int H, float sl2,
                                                             float scale) {
  constexpr int HP = HD + 4, NDB = HD / 16, DQ = HD / 4;
  __shared__ __attribute__((aligned(16))) float Qs[ATT_R * HP], Ds[ATT_R * HP];
  __shared__ float Ls[ATT_R], Dl[ATT_R];
  int kb, h, b;
  xcd_spread_block(kb, h, b);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, n = lane & 15;
  const int key = kb * ATT_R + 16 * w + n, kc = min(key, S - 1);
  const long long rs = 3LL * H * HD, ors = (long long)H * HD;
  const float* qbase = qkv + (long long)b * S * rs + (long long)h * HD;
  const float* kbase = qbase + (long long)H * HD;
  const float* vbase = qbase + 2LL * H * HD;
  const float* dbase = dout + (long long)b * S * ors + (long long)h * HD;
  const long long lrow = ((long long)b * H + h) * S;
  float kf[DQ], vf[DQ];
  own_slice<HD>(kf, kbase, rs, kc, g, cosb, sinb, true);
  own_slice<HD>(vf, vbase, rs, kc, g, cosb, sinb, false);
  f4m dk[NDB], dv[NDB];
#pragma unroll
  for (int db = 0; db < NDB; ++db) dk[db] = dv[db] = (f4m){0.f, 0.f, 0.f, 0.f};
  const int nqt = (S + ATT_R - 1) / ATT_R;
  for (int qt = kb; qt < nqt; ++qt) {
    __syncthreads();
    stage_rows_p<HD>(Qs, qbase, rs, qt * ATT_R, S, cosb, sinb, true);
    stage_rows_p<HD>(Ds, dbase, ors, qt * ATT_R, S, cosb, sinb, false);
    if (threadIdx.x < ATT_R) {
      const int qi = qt * ATT_R + threadIdx.x;
      Ls[threadIdx.x] = qi < S ? lse[lrow + qi] : 0.f;
      Dl[threadIdx.x] = qi < S ? delta[lrow + qi] : 0.f;
    }
    __syncthreads();
    for (int u = (qt == kb ? w : 0); u < 4; ++u) {  // 16-query sub-tiles at or below the diagonal
      const f4m sv = dot_block<HD>(Qs + (16 * u + n) * HP, kf, g);   // S[query 4g+i][key n]
      const f4m dpv = dot_block<HD>(Ds + (16 * u + n) * HP, vf, g);  // dP = dO V^T
      float p[4], ds[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 16 * u + 4 * g + i, qi = qt * ATT_R + r;
        p[i] = (qi >= key && qi < S) ? exp2f(sv[i] * sl2 - Ls[r]) : 0.f;
        ds[i] = p[i] * (dpv[i] - Dl[r]);
      }
      accum_rows<HD>(dv, Ds, 16 * u, p, g, n);   // dV^T[d][key n] += dO^T P
      accum_rows<HD>(dk, Qs, 16 * u, ds, g, n);  // dK^T[d][key n] += Q^T dS
    }
  }
  if (key >= S) return;
  float* dst = dqkv + (long long)(b * S + key) * rs + (long long)h * HD;
  store_blocks<HD>(dst + (long long)H * HD, dk, g, scale, cosb + (long long)key * (HD / 2),
                   sinb + (long long)key * (HD / 2));
  store_blocks<HD>(dst + 2LL * H * HD, dv, g, 1.f, nullptr, nullptr);
}

#define ATT_HD_SWITCH(HDV, CALL) \
  switch (HDV) {                 \
    case 16: CALL(16); break;    \
    case 32: CALL(32); break;    \
    case 48: CALL(48); break;    \
    case 64: CALL(64); break;    \
    case 96: CALL(96); break;    \
    case 128: CALL(128); break;  \
    default: return (int)hipErrorInvalidValue; \
  }

DDL_API int ddl_attnf_fwd(const float* qkv, float* o, float* lse, const float* cosb, const float* sinb, int B, int S,
                          int H, int HD, float scale, hipStream_t s) {
  if (B < 1 || S < 1 || H < 1) return 0;
  const dim3 grid((S + ATT_R - 1) / ATT_R, H, B);
  const float sl2 = scale * LOG2E;
#define ATT_FWD(D) hipLaunchKernelGGL(attnf_fwd_kernel<D>, grid, dim3(256), 0, s, qkv, o, lse, cosb, sinb, S, H, sl2)
  ATT_HD_SWITCH(HD, ATT_FWD)
#undef ATT_FWD
  return (int)hipGetLastError();
}

DDL_API int ddl_attnf_bwd(const float* qkv, const float* o, const float* dout, const float* lse, float* delta,
                          float* dqkv, const float* cosb, const float* sinb, int B, int S, int H, int HD, float scale,
                          hipStream_t s) {
  if (B < 1 || S < 1 || H < 1) return 0;
  const dim3 grid((S + ATT_R - 1) / ATT_R, H, B);
  const float sl2 = scale * LOG2E;
#define ATT_DQ(D)                                                                                                 \
  hipLaunchKernelGGL(attnf_bwd_dq_kernel<D>, grid, dim3(256), 0, s, qkv, o, dout, lse, delta, dqkv, cosb, sinb, S, \
                     H, sl2, scale)
  ATT_HD_SWITCH(HD, ATT_DQ)
#undef ATT_DQ
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
#define ATT_DKV(D)                                                                                             \
  hipLaunchKernelGGL(attnf_bwd_dkdv_kernel<D>, grid, dim3(256), 0, s, qkv, dout, lse, delta, dqkv, cosb, sinb, \
                     S, H, sl2, scale)
  ATT_HD_SWITCH(HD, ATT_DKV)
#undef ATT_DKV
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Vocabulary cross-entropy, fp32 logits [R][V] (row stride ld), int32 labels. One block per row:
// pass 1 max / sum-exp, pass 2 d = (softmax - onehot) * (*inv); rowloss[r] = lse - z[label]
// (0 for ignored rows, whose gradient row is zero).
__device__ __forceinline__ void block_maxsum(float& m, float& s, float* sm) {
  // merge (m, s) pairs: wave level, then the 4 waves in a fixed order
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o), s2 = __shfl_xor(s, o);
    const float nm = fmaxf(m, m2);
    s = (nm == -INFINITY) ? 0.f : s * exp2f(m - nm) + s2 * exp2f(m2 - nm);
    m = nm;
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) { sm[w] = m; sm[4 + w] = s; }
  __syncthreads();
  m = sm[0]; s = sm[4];
  for (int k = 1; k < 4; ++k) {
    const float m2 = sm[k], s2 = sm[4 + k], nm = fmaxf(m, m2);
    s = (nm == -INFINITY) ? 0.f : s * exp2f(m - nm) + s2 * exp2f(m2 - nm);
    m = nm;
  }
}

__global__ __launch_bounds__(256) void cevf_rows_kernel(const float* __restrict__ z, const int* __restrict__ labels,
                                                        int V, long long ld, const float* __restrict__ inv,
                                                        int ignore_index, float* __restrict__ rowloss,
                                                        float* __restrict__ dz, long long ldd) {
  __shared__ float sm[8];
  const int row = blockIdx.x;
  const float* zr = z + row * ld;
  const int lab = labels[row];
  float m = -INFINITY, s = 0.f;
  const bool vec = (V % 4 == 0) && (ld % 4 == 0);
  if (vec) {
    for (int c = threadIdx.x; c < V / 4; c += 256) {
      const float4 v = ((const float4*)zr)[c];
      const float x[4] = {v.x * LOG2E, v.y * LOG2E, v.z * LOG2E, v.w * LOG2E};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float nm = fmaxf(m, x[k]);
        s = s * exp2f(m - nm) + exp2f(x[k] - nm);
        m = nm;
      }
    }
  } else {
    for (int c = threadIdx.x; c < V; c += 256) {
      const float x = zr[c] * LOG2E, nm = fmaxf(m, x);
      s = s * exp2f(m - nm) + exp2f(x - nm);
      m = nm;
    }
  }
  block_maxsum(m, s, sm);
  const float lse2 = m + log2f(s);  // log2 domain
  const bool valid = lab != ignore_index && lab >= 0 && lab < V;
  if (threadIdx.x == 0) rowloss[row] = valid ? (lse2 / LOG2E - zr[lab]) : 0.f;
  if (!dz) return;
  const float k = valid ? *inv : 0.f;
  float* dr = dz + row * ldd;
  for (int c = threadIdx.x; c < V; c += 256) {
    const float p = exp2f(zr[c] * LOG2E - lse2);
    dr[c] = (p - (c == lab ? 1.f : 0.f)) * k;
  }
}

// Rows of up to 1024 * NV4 logits held in registers: one HBM read of z instead of two (the
// streaming kernel above re-reads a 128 KB row after its sum pass, from HBM at 32k vocab).
template <int NV4>
__global__ __launch_bounds__(256) void cevf_rows_reg_kernel(const float* __restrict__ z,
                                                            const int* __restrict__ labels, int V, long long ld,
                                                            const float* __restrict__ inv, int ignore_index,
                                                            float* __restrict__ rowloss, float* __restrict__ dz,
                                                            long long ldd) {
  __shared__ float sm[8];
  const int row = blockIdx.x;
  const float* zr = z + row * ld;
  const int lab = labels[row];
  const int n4 = V >> 2;
  float4 v[NV4];
#pragma unroll
  for (int j = 0; j < NV4; ++j) {
    const int c = threadIdx.x + j * 256;
    v[j] = c < n4 ? ((const float4*)zr)[c] : make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
  }
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < NV4; ++j) mx = fmaxf(mx, fmaxf(fmaxf(v[j].x, v[j].y), fmaxf(v[j].z, v[j].w)));
  float m = mx * LOG2E, s = 0.f;
  if (mx != -INFINITY) {
#pragma unroll
    for (int j = 0; j < NV4; ++j)
      s += (exp2f(v[j].x * LOG2E - m) + exp2f(v[j].y * LOG2E - m)) +
           (exp2f(v[j].z * LOG2E - m) + exp2f(v[j].w * LOG2E - m));
  }
  block_maxsum(m, s, sm);
  const float lse2 = m + log2f(s);
  const bool valid = lab != ignore_index && lab >= 0 && lab < V;
  if (threadIdx.x == 0) rowloss[row] = valid ? (lse2 / LOG2E - zr[lab]) : 0.f;
  if (!dz) return;
  const float k = valid ? *inv : 0.f;
  float4* dr = (float4*)(dz + row * ldd);
#pragma unroll
  for (int j = 0; j < NV4; ++j) {
    const int c = threadIdx.x + j * 256;
    if (c < n4) {
      const int b = 4 * c;
      float4 p;
      p.x = (exp2f(v[j].x * LOG2E - lse2) - (b == lab ? 1.f : 0.f)) * k;
      p.y = (exp2f(v[j].y * LOG2E - lse2) - (b + 1 == lab ? 1.f : 0.f)) * k;
      p.z = (exp2f(v[j].z * LOG2E - lse2) - (b + 2 == lab ? 1.f : 0.f)) * k;
      p.w = (exp2f(v[j].w * LOG2E - lse2) - (b + 3 == lab ? 1.f : 0.f)) * k;
      dr[c] = p;
    }
  }
}

__global__ __launch_bounds__(256) void cevf_fold_kernel(const float* __restrict__ rowloss, int R,
                                                        const float* __restrict__ inv, float* __restrict__ loss) {
  __shared__ float sm[4];
  float s = 0.f;
  for (int r = threadIdx.x; r < R; r += 256) s += rowloss[r];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) loss[0] = (((sm[0] + sm[1]) + sm[2]) + sm[3]) * (*inv);
}

DDL_API int ddl_cevf(const float* z, const int* labels, int R, int V, long long ld, const float* inv,
                     int ignore_index, float* rowloss, float* loss, float* dz, long long ldd, hipStream_t s) {
  if (R < 1 || V < 1) return (int)hipErrorInvalidValue;
  const bool vec = V % 4 == 0 && ld % 4 == 0 && (!dz || ldd % 4 == 0) && ((uintptr_t)z & 15) == 0 &&
                   ((uintptr_t)dz & 15) == 0;
  const int n4 = V / 4;
  if (vec && n4 <= 256 * 8)
    hipLaunchKernelGGL(cevf_rows_reg_kernel<8>, dim3(R), dim3(256), 0, s, z, labels, V, ld, inv, ignore_index,
                       rowloss, dz, ldd);
  else if (vec && n4 <= 256 * 16)
    hipLaunchKernelGGL(cevf_rows_reg_kernel<16>, dim3(R), dim3(256), 0, s, z, labels, V, ld, inv, ignore_index,
                       rowloss, dz, ldd);
  else if (vec && n4 <= 256 * 32)
    hipLaunchKernelGGL(cevf_rows_reg_kernel<32>, dim3(R), dim3(256), 0, s, z, labels, V, ld, inv, ignore_index,
                       rowloss, dz, ldd);
  else
    hipLaunchKernelGGL(cevf_rows_kernel, dim3(R), dim3(256), 0, s, z, labels, V, ld, inv, ignore_index, rowloss,
                       dz, ldd);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(cevf_fold_kernel, dim3(1), dim3(256), 0, s, rowloss, R, inv, loss);
  return (int)hipGetLastError();
}

__global__ void scale_f32_kernel(float* __restrict__ x, long long n, const float* __restrict__ g) {
  const float s = *g;
  if (s == 1.f) return;
  GSTRIDE_LOOP(i, n) x[i] *= s;
}

DDL_API int ddl_scale_f32(float* x, long long n, const float* g, hipStream_t s) {
  if (n < 1) return 0;
  hipLaunchKernelGGL(scale_f32_kernel, dim3(grid_for(n, 256, 4096)), dim3(256), 0, s, x, n, g);
  return (int)hipGetLastError();
}
