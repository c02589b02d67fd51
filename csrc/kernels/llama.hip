// Kernels of the tiny-LLaMA used by the data/pipeline-parallel tutorials (reference
// lab/tutorial_1b: simplellm LLama dmodel=288, 6 heads x 48, 6 layers, seq 256, vocab ~32k).
//
//   ddl_embedding_fwd/bwd : row gather (bf16 out) / fp32 atomic scatter-add into the grad
//   ddl_rmsnorm_fwd/bwd   : one wave per row, rstd saved, gamma grad reduced per block then atomics
//   ddl_swiglu_fwd/bwd    : h = silu(a) * b over the fused [a | b] projection
//   ddl_add               : bf16 residual add
//   ddl_attn_fwd/bwd      : causal flash attention on the gfx950 16x16x32 bf16 MFMA (head_dim
//                           32/48/64/128; a 16-dim remainder zero-padded to 32) with RoPE applied
//                           as q / k tiles are staged
//                           (so RoPE costs no HBM pass), online softmax, log-sum-exp saved;
//                           backward recomputes P in two kernels (dQ; dK+dV) and writes the
//                           un-rotated gradients straight into the fused dQKV buffer.
// The projections / FFN / LM head run on the MFMA implicit-GEMM conv kernel.
#include "ddl_common.h"

// ---------------------------------------------------------------------------------------------
__global__ void embedding_fwd_kernel(const int* __restrict__ idx, const float* __restrict__ w,
                                     bf16_t* __restrict__ y, int T, int D) {
  const int DC = D / 4;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < (long long)T * DC;
       t += (long long)gridDim.x * blockDim.x) {
    const int row = (int)(t / DC), c = (int)(t % DC) * 4;
    const float4 v = *(const float4*)(w + (long long)idx[row] * D + c);
    i2v o;
    o[0] = (int)pack_bf2(v.x, v.y);
    o[1] = (int)pack_bf2(v.z, v.w);
    *(i2v*)(y + (long long)row * D + c) = o;
  }
}
__global__ void embedding_bwd_kernel(const int* __restrict__ idx, const bf16_t* __restrict__ dy,
                                     float* __restrict__ dw, int T, int D, int pad_idx) {
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < (long long)T * D;
       t += (long long)gridDim.x * blockDim.x) {
    const int row = (int)(t / D), c = (int)(t % D);
    const int tok = idx[row];
    if (tok == pad_idx) continue;
    atomicAdd(dw + (long long)tok * D + c, bf2f(dy[t]));
  }
}
DDL_API int ddl_embedding_fwd(const int* idx, const float* w, void* y, int T, int D, hipStream_t s) {
  if (D % 4) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(embedding_fwd_kernel, dim3(grid_for((long long)T * D / 4, 256)), dim3(256), 0,
                     s, idx, w, (bf16_t*)y, T, D);
  return (int)hipGetLastError();
}
DDL_API int ddl_embedding_bwd(const int* idx, const void* dy, float* dw, int T, int D, int pad_idx,
                              hipStream_t s) {
  hipLaunchKernelGGL(embedding_bwd_kernel, dim3(grid_for((long long)T * D, 256)), dim3(256), 0, s,
                     idx, (const bf16_t*)dy, dw, T, D, pad_idx);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// RMSNorm: one wave per row, D <= 64*8*MAXC
template <int MAXC>
__global__ __launch_bounds__(256) void rmsnorm_fwd_kernel(const bf16_t* __restrict__ x,
                                                          const float* __restrict__ g,
                                                          bf16_t* __restrict__ y,
                                                          float* __restrict__ rstd, int T, int D,
                                                          float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= T) return;
  const int NC = D / 8;
  float v[MAXC][8];
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + 64 * c;
    if (ch < NC) {
      unpack8(*(const i4v*)(x + (long long)row * D + ch * 8), v[c]);
#pragma unroll
      for (int k = 0; k < 8; ++k) ss += v[c][k] * v[c][k];
    }
  }
  ss = wave_sum(ss);
  const float r = rsqrtf(ss / D + eps);
  if (lane == 0) rstd[row] = r;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + 64 * c;
    if (ch < NC) {
      float o[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = v[c][k] * r * g[ch * 8 + k];
      *(i4v*)(y + (long long)row * D + ch * 8) = pack8(o);
    }
  }
}

// dx = r*g*dy - x * r^3 * sum(g*dy*x)/D ; dg += sum_rows dy * x * r
// A lane owns the same channels in every row it visits, so gamma stays in registers and d(gamma)
// accumulates in registers across the wave's rows; the 4 waves meet once in LDS and each block
// adds one row of D partial sums into the fp32 grad buffer (per-row LDS atomics from 4 waves on
// the same D addresses: 12.5 us for 2048 x 288; now 9.1 us).
template <int MAXC>
__global__ __launch_bounds__(256) void rmsnorm_bwd_kernel(const bf16_t* __restrict__ x,
                                                          const float* __restrict__ g,
                                                          const float* __restrict__ rstd,
                                                          const bf16_t* __restrict__ dy,
                                                          const bf16_t* __restrict__ dres,
                                                          bf16_t* __restrict__ dx,
                                                          float* __restrict__ dg, int T, int D) {
  extern __shared__ float dg_part[];  // [4][D]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int NC = D / 8;
  float gv[MAXC][8], acc[MAXC][8];
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + 64 * c;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      gv[c][k] = ch < NC ? g[ch * 8 + k] : 0.f;
      acc[c][k] = 0.f;
    }
  }
  // Rows are software-pipelined: the next row's x / dy / rstd loads are issued before the current
  // row's wave reduction, so a wave pays one HBM latency for its whole row sweep.
  const int stride = gridDim.x * 4;
  int row = blockIdx.x * 4 + w;
  float xv[MAXC][8], dv[MAXC][8], xn[MAXC][8], dn[MAXC][8];
  float r = 0.f, rn = 0.f;
  auto load_row = [&](int rr, float (*xa)[8], float (*da)[8]) {
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int ch = lane + 64 * c;
      if (ch < NC) {
        unpack8(*(const i4v*)(x + (long long)rr * D + ch * 8), xa[c]);
        unpack8(*(const i4v*)(dy + (long long)rr * D + ch * 8), da[c]);
      }
    }
  };
  if (row < T) {
    load_row(row, xv, dv);
    r = rstd[row];
  }
  for (; row < T; row += stride) {
    const int nrow = row + stride;
    if (nrow < T) {
      load_row(nrow, xn, dn);
      rn = rstd[nrow];
    }
    float dot = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int ch = lane + 64 * c;
      if (ch < NC) {
#pragma unroll
        for (int k = 0; k < 8; ++k) dot += gv[c][k] * dv[c][k] * xv[c][k];
      }
    }
    dot = wave_sum(dot) / D;
    const float r3 = r * r * r * dot;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int ch = lane + 64 * c;
      if (ch < NC) {
        float o[8];
        if (dres) unpack8(*(const i4v*)(dres + (long long)row * D + ch * 8), o);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          o[k] = (dres ? o[k] : 0.f) + r * gv[c][k] * dv[c][k] - xv[c][k] * r3;
          acc[c][k] += dv[c][k] * xv[c][k] * r;
        }
        *(i4v*)(dx + (long long)row * D + ch * 8) = pack8(o);
      }
    }
#pragma unroll
    for (int c = 0; c < MAXC; ++c)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        xv[c][k] = xn[c][k];
        dv[c][k] = dn[c][k];
      }
    r = rn;
  }
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + 64 * c;
    if (ch < NC) {
#pragma unroll
      for (int k = 0; k < 8; ++k) dg_part[w * D + ch * 8 + k] = acc[c][k];
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < D; i += 256)
    atomicAdd(dg + i, (dg_part[i] + dg_part[D + i]) + (dg_part[2 * D + i] + dg_part[3 * D + i]));
}

// Rows per wave of the backward grid; 0 = automatic. The d(gamma) atomics (one per block per
// column) contend on D addresses, so the grid is capped near 256 blocks and the software-pipelined
// row sweep absorbs the rest. Measured (scripts/rmsnorm_sweep.py, profiles/rmsnorm_bwd_sweep_r1.log):
//   T=2048: 1/2/4/8 rows per wave = 16.6/10.7/9.1/10.8 us;  T=8192: 54.4/31.4/18.9/15.8 us.
static int g_rmsnorm_bwd_rows_per_wave = 0;
DDL_API int ddl_rmsnorm_bwd_set_rows(int rows) {
  if (rows >= 0 && rows <= 64) g_rmsnorm_bwd_rows_per_wave = rows;
  return g_rmsnorm_bwd_rows_per_wave;
}

DDL_API int ddl_rmsnorm_fwd(const void* x, const float* g, void* y, float* rstd, int T, int D,
                            float eps, hipStream_t s) {
  if (D % 8 || D > 64 * 8 * 4) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(rmsnorm_fwd_kernel<4>, dim3((T + 3) / 4), dim3(256), 0, s, (const bf16_t*)x, g,
                     (bf16_t*)y, rstd, T, D, eps);
  return (int)hipGetLastError();
}
// dres (nullable): gradient arriving through the residual branch of the same x, added into dx
// (the residual fork of a pre-norm block; saves the separate gradient-sum pass).
DDL_API int ddl_rmsnorm_bwd(const void* x, const float* g, const float* rstd, const void* dy,
                            const void* dres, void* dx, float* dg, int T, int D, hipStream_t s) {
  if (D % 8 || D > 64 * 8 * 4) return (int)hipErrorInvalidValue;
  int rows = g_rmsnorm_bwd_rows_per_wave;
  if (rows <= 0) rows = (T + 1023) / 1024 > 4 ? (T + 1023) / 1024 : 4;
  const int blocks = grid_for(T, 4 * rows, 1 << 20);
  hipLaunchKernelGGL(rmsnorm_bwd_kernel<4>, dim3(blocks), dim3(256), 4 * D * sizeof(float), s,
                     (const bf16_t*)x, g, rstd, (const bf16_t*)dy, (const bf16_t*)dres, (bf16_t*)dx, dg, T, D);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// SwiGLU over ab [T][2F] = [a | b]  ->  h [T][F]
__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }
__global__ void swiglu_fwd_kernel(const bf16_t* __restrict__ ab, bf16_t* __restrict__ h, int T, int F) {
  const int FC = F / 8;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < (long long)T * FC;
       t += (long long)gridDim.x * blockDim.x) {
    const long long row = t / FC;
    const int c = (int)(t % FC) * 8;
    float a[8], b[8], o[8];
    unpack8(*(const i4v*)(ab + row * 2 * F + c), a);
    unpack8(*(const i4v*)(ab + row * 2 * F + F + c), b);
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = a[k] * sigm(a[k]) * b[k];
    *(i4v*)(h + row * F + c) = pack8(o);
  }
}
__global__ void swiglu_bwd_kernel(const bf16_t* __restrict__ ab, const bf16_t* __restrict__ dh,
                                  bf16_t* __restrict__ dab, int T, int F) {
  const int FC = F / 8;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < (long long)T * FC;
       t += (long long)gridDim.x * blockDim.x) {
    const long long row = t / FC;
    const int c = (int)(t % FC) * 8;
    float a[8], b[8], d[8], da[8], db[8];
    unpack8(*(const i4v*)(ab + row * 2 * F + c), a);
    unpack8(*(const i4v*)(ab + row * 2 * F + F + c), b);
    unpack8(*(const i4v*)(dh + row * F + c), d);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float sg = sigm(a[k]);
      const float silu = a[k] * sg;
      db[k] = d[k] * silu;
      da[k] = d[k] * b[k] * sg * (1.f + a[k] * (1.f - sg));
    }
    *(i4v*)(dab + row * 2 * F + c) = pack8(da);
    *(i4v*)(dab + row * 2 * F + F + c) = pack8(db);
  }
}
DDL_API int ddl_swiglu_fwd(const void* ab, void* h, int T, int F, hipStream_t s) {
  if (F % 8) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(swiglu_fwd_kernel, dim3(grid_for((long long)T * F / 8, 256)), dim3(256), 0, s,
                     (const bf16_t*)ab, (bf16_t*)h, T, F);
  return (int)hipGetLastError();
}
DDL_API int ddl_swiglu_bwd(const void* ab, const void* dh, void* dab, int T, int F, hipStream_t s) {
  if (F % 8) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(swiglu_bwd_kernel, dim3(grid_for((long long)T * F / 8, 256)), dim3(256), 0, s,
                     (const bf16_t*)ab, (const bf16_t*)dh, (bf16_t*)dab, T, F);
  return (int)hipGetLastError();
}

__global__ void add_kernel(const bf16_t* __restrict__ a, const bf16_t* __restrict__ b,
                           bf16_t* __restrict__ y, long long n8) {
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < n8;
       t += (long long)gridDim.x * blockDim.x) {
    float x[8], z[8];
    unpack8(*(const i4v*)(a + t * 8), x);
    unpack8(*(const i4v*)(b + t * 8), z);
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] += z[k];
    *(i4v*)(y + t * 8) = pack8(x);
  }
}
DDL_API int ddl_add(const void* a, const void* b, void* y, long long n, hipStream_t s) {
  if (n % 8) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(add_kernel, dim3(grid_for(n / 8, 256)), dim3(256), 0, s, (const bf16_t*)a,
                     (const bf16_t*)b, (bf16_t*)y, n / 8);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Causal attention on gfx950's double-rate MFMA (v_mfma_f32_16x16x32_bf16, fp32 accumulate; a
// head-dim remainder of 16, e.g. HD = 48 = 32 + 16, is zero-padded to one more x32).
// qkv: [B][S][3][H][HD] bf16 (the fused projection output), o / dout: [B][S][H][HD], lse / delta:
// [B][H][S] fp32, RoPE tables cos/sin [S][HD/2] fp32 (interleaved pairs (2i, 2i+1)), applied as
// tiles are staged. A workgroup owns 64 query rows (forward, dQ) or 64 key rows (dK/dV), each of
// its 4 waves 16 of them, and steps over the other side 32 rows at a time. Every product is
// oriented so that the softmax-side tiles an MFMA produces are directly the B operand of the next:
//   forward : S^T = K Q^T (keys x queries)  -> P^T   -> O^T  += V^T P^T
//   dQ      : S^T = K Q^T, dP^T = V dO^T    -> dS^T  -> dQ^T += K^T dS^T
//   dK, dV  : S = Q K^T,   dP = dO V^T      -> P, dS -> dV^T += dO^T P, dK^T += Q^T dS
// A 32-row step computes two 16x16 score tiles (rows 0-15 and 16-31 of the step); lane l holds
// rows 4(l/16)+i of the first and 16+4(l/16)+i of the second. The x32 MFMA sums over its k slots
// in any order as long as A and B agree, so the B operand of the follow-on product is just the
// 8 values the lane holds — k slot (g = l/16, j) := step row 4g+j (j < 4) or 16+4g+j-4 (j >= 4) —
// and the A operand (a transposed V / K / dO / Q image in LDS) is read at those same rows: two
// 8-byte reads per lane. No computed tile is ever transposed or shuffled through LDS.
// Online softmax in the exp2 domain; the backward recomputes P from the saved log-sum-exp
// (flash-attention 2).
constexpr int AT = 64;   // rows per workgroup tile
constexpr int AST = 32;  // rows per inner step (one x32 MFMA k-extent)
constexpr float LOG2E = 1.4426950408889634f;

__device__ __forceinline__ f4v mma32(s8v a, s8v b, f4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ s4v bf4(float a, float b, float c, float d) {
  s4v r;
  r[0] = (short)f2bf(a);
  r[1] = (short)f2bf(b);
  r[2] = (short)f2bf(c);
  r[3] = (short)f2bf(d);
  return r;
}
__device__ __forceinline__ s8v cat8(s4v a, s4v b) {
  return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}
__device__ __forceinline__ s8v bf8(const float* v) {
  return cat8(bf4(v[0], v[1], v[2], v[3]), bf4(v[4], v[5], v[6], v[7]));
}

// dims d0..d0+3 (d0 % 4 == 0) of one row, RoPE-rotated when cs != nullptr
__device__ __forceinline__ void row4(const bf16_t* row, const float* cs, const float* sn, int d0,
                                     float* v) {
  const i2v raw = *(const i2v*)(row + d0);
  v[0] = lo_bf((uint32_t)raw[0]);
  v[1] = hi_bf((uint32_t)raw[0]);
  v[2] = lo_bf((uint32_t)raw[1]);
  v[3] = hi_bf((uint32_t)raw[1]);
  if (cs) {
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const float c = cs[d0 / 2 + p], s = sn[d0 / 2 + p], x0 = v[2 * p], x1 = v[2 * p + 1];
      v[2 * p] = x0 * c - x1 * s;
      v[2 * p + 1] = x0 * s + x1 * c;
    }
  }
}

// inverse rotation of a gradient's dims d0..d0+3 and bf16 store
__device__ __forceinline__ void store4_unrot(bf16_t* dst, const float* cs, const float* sn, int d0,
                                             const f4v& g, bool rot) {
  float r[4] = {g[0], g[1], g[2], g[3]};
  if (rot) {
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const float c = cs[d0 / 2 + p], s = sn[d0 / 2 + p], g0 = g[2 * p], g1 = g[2 * p + 1];
      r[2 * p] = g0 * c + g1 * s;
      r[2 * p + 1] = -g0 * s + g1 * c;
    }
  }
  i2v v;
  v[0] = (int)pack_bf2(r[0], r[1]);
  v[1] = (int)pack_bf2(r[2], r[3]);
  *(i2v*)(dst + d0) = v;
}

// LDS images: row-major [64][HDP+8] with HDP = HD rounded up to 32 (16-byte aligned rows for the
// x32 A reads; dims HD..HDP-1 are staged as zeros, so a head-dim remainder of 16 runs as one x32
// MFMA with a zero upper half — the same cycles as a 16x16x16 on gfx950, and every head-dim
// product is one MFMA shape) and transposed [HD][64+8] (8-byte reads at 4g and 16+4g of a step
// land on distinct bank pairs).
template <int HD> struct AttnLds {
  static constexpr int HDP = (HD + 31) / 32 * 32;
  static constexpr int KP = HDP + 8, VP = AT + 8;
  static constexpr int D32 = HDP / 32, NT = HD / 16;
};

// Stage rows r0..r0+63 (row t at src + t*rs) into LDS (row-major and/or transposed); rows >= S
// and the row-major image's dims HD..HDP-1 are zeros. A thread owns a 4-row x 4-dim block: four
// 8-byte row reads, then (transposed image) a 4x4 register transpose and four 8-byte writes of 4
// consecutive rows per dim — a quarter of the LDS write instructions of per-element stores.
template <int HD>
__device__ __forceinline__ void stage_rows(const bf16_t* src, long long rs, int r0, int S,
                                           const float* rcos, const float* rsin, bf16_t* rm,
                                           bf16_t* tr) {
  constexpr int C4 = HD / 4, KP = AttnLds<HD>::KP, VP = AttnLds<HD>::VP, HDP = AttnLds<HD>::HDP;
  for (int e = threadIdx.x; e < (AT / 4) * C4; e += 256) {
    const int rq = e / C4, d0 = (e - rq * C4) * 4, rb = 4 * rq;
    float v[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int t = r0 + rb + j;
#pragma unroll
      for (int k = 0; k < 4; ++k) v[j][k] = 0.f;
      if (t < S)
        row4(src + (long long)t * rs, rcos ? rcos + (long long)t * (HD / 2) : nullptr,
             rsin ? rsin + (long long)t * (HD / 2) : nullptr, d0, v[j]);
      if (rm) *(s4v*)(rm + (rb + j) * KP + d0) = bf4(v[j][0], v[j][1], v[j][2], v[j][3]);
    }
    if (tr) {
#pragma unroll
      for (int k = 0; k < 4; ++k) *(s4v*)(tr + (d0 + k) * VP + rb) = bf4(v[0][k], v[1][k], v[2][k], v[3][k]);
    }
  }
  if constexpr (HDP > HD) {
    if (rm) {
      constexpr int Z4 = (HDP - HD) / 4;
      for (int e = threadIdx.x; e < AT * Z4; e += 256) {
        const int r = e / Z4, d0 = HD + (e - r * Z4) * 4;
        *(s4v*)(rm + r * KP + d0) = s4v{0, 0, 0, 0};
      }
    }
  }
}

// One row's B fragments over the (zero-padded) head dimension: chunk c holds dims 32c + 8g + j;
// zeros when !valid or past HD.
template <int HD> struct RowFrag {
  s8v c[AttnLds<HD>::D32];
};

template <int HD>
__device__ __forceinline__ void row_frags(const bf16_t* row, const float* cs, const float* sn,
                                          int lg, bool valid, RowFrag<HD>& f) {
#pragma unroll
  for (int c = 0; c < AttnLds<HD>::D32; ++c) {
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const int d0 = 32 * c + 8 * lg;
    if (valid && d0 < HD) row4(row, cs, sn, d0, v);
    if (valid && d0 + 4 < HD) row4(row, cs, sn, d0 + 4, v + 4);
    f.c[c] = bf8(v);
  }
}

// acc += A(16 rows of a row-major LDS image, this lane's row at `arow`) . f over the head dim
template <int HD>
__device__ __forceinline__ f4v dot_hd(const bf16_t* arow, const RowFrag<HD>& f, int lg, f4v acc) {
#pragma unroll
  for (int c = 0; c < AttnLds<HD>::D32; ++c) acc = mma32(*(const s8v*)(arow + 32 * c + 8 * lg), f.c[c], acc);
  return acc;
}

// A operand over a 32-row step from a transposed image row: k slots (g, j) -> rows 4g+j, 16+4g+j
__device__ __forceinline__ s8v step_frag(const bf16_t* trow, int lg) {
  return cat8(*(const s4v*)(trow + 4 * lg), *(const s4v*)(trow + 16 + 4 * lg));
}

template <int HD>
__global__ __launch_bounds__(256) void attn_fwd_kernel(const bf16_t* __restrict__ qkv,
                                                       bf16_t* __restrict__ o,
                                                       float* __restrict__ lse,
                                                       const float* __restrict__ rcos,
                                                       const float* __restrict__ rsin, int S, int H,
                                                       float scale) {
  using L = AttnLds<HD>;
  constexpr int NT = L::NT, KP = L::KP, VP = L::VP;
  __shared__ __attribute__((aligned(16))) bf16_t Ks[AT * KP];
  __shared__ __attribute__((aligned(16))) bf16_t Vt[HD * VP];
  int qt, h, b;
  xcd_spread_block(qt, h, b);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, lq = lane & 15, lg = lane >> 4;
  const long long rs = 3LL * H * HD, ro = (long long)H * HD;
  const bf16_t* base = qkv + (long long)b * S * rs + h * HD;
  const int q = qt * AT + wv * 16 + lq, qmax = qt * AT + wv * 16 + 15;
  const bool qv = q < S;
  const float sl2 = scale * LOG2E;
  RowFrag<HD> qf;
  row_frags<HD>(base + (long long)q * rs, rcos + (long long)q * (HD / 2),
                rsin + (long long)q * (HD / 2), lg, qv, qf);
  f4v acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f4v{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;
  for (int kt = 0; kt <= qt; ++kt) {
    __syncthreads();
    stage_rows<HD>(base + ro, rs, kt * AT, S, rcos, rsin, Ks, nullptr);
    stage_rows<HD>(base + 2 * ro, rs, kt * AT, S, nullptr, nullptr, nullptr, Vt);
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < AT / AST; ++ks) {
      const int key0 = kt * AT + ks * AST;
      if (key0 > qmax || key0 >= S) break;  // wave-uniform: the causal / sequence edge
      const f4v s0 = dot_hd<HD>(Ks + (ks * AST + lq) * KP, qf, lg, f4v{0.f, 0.f, 0.f, 0.f});
      const f4v s1 = dot_hd<HD>(Ks + (ks * AST + 16 + lq) * KP, qf, lg, f4v{0.f, 0.f, 0.f, 0.f});
      float x[8], mx = -INFINITY;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int key = key0 + (i < 4 ? 4 * lg + i : 16 + 4 * lg + i - 4);
        x[i] = (key <= q && key < S) ? (i < 4 ? s0[i] : s1[i - 4]) * sl2 : -INFINITY;
        mx = fmaxf(mx, x[i]);
      }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mn = fmaxf(m, mx);
      const float corr = (mn == -INFINITY) ? 1.f : exp2f(m - mn);
      float p[8], ps = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        p[i] = (x[i] == -INFINITY) ? 0.f : exp2f(x[i] - mn);
        ps += p[i];
      }
      ps += __shfl_xor(ps, 16, 64);
      ps += __shfl_xor(ps, 32, 64);
      l = l * corr + ps;
      m = mn;
      const s8v pb = bf8(p);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        acc[t] *= corr;
        acc[t] = mma32(step_frag(Vt + (16 * t + lq) * VP + ks * AST, lg), pb, acc[t]);
      }
    }
  }
  if (qv) {
    const float inv = 1.f / l;
    bf16_t* op = o + ((long long)b * S + q) * ro + h * HD;
#pragma unroll
    for (int t = 0; t < NT; ++t) store4_unrot(op, nullptr, nullptr, 16 * t + 4 * lg, acc[t] * inv, false);
    if (lg == 0) lse[((long long)b * H + h) * S + q] = (m + log2f(l)) * 0.6931471805599453f;
  }
}

// dQ (+ delta = rowsum(dO * O)), un-rotated into dqkv's q slot
template <int HD>
__global__ __launch_bounds__(256) void attn_bwd_dq_kernel(
    const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ o, const bf16_t* __restrict__ dout,
    const float* __restrict__ lse, float* __restrict__ delta, bf16_t* __restrict__ dqkv,
    const float* __restrict__ rcos, const float* __restrict__ rsin, int S, int H, float scale) {
  using L = AttnLds<HD>;
  constexpr int NT = L::NT, KP = L::KP, VP = L::VP;
  __shared__ __attribute__((aligned(16))) bf16_t Ks[AT * KP];
  __shared__ __attribute__((aligned(16))) bf16_t Vs[AT * KP];
  __shared__ __attribute__((aligned(16))) bf16_t Kt[HD * VP];
  int qt, h, b;
  xcd_spread_block(qt, h, b);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, lq = lane & 15, lg = lane >> 4;
  const long long rs = 3LL * H * HD, ro = (long long)H * HD;
  const bf16_t* base = qkv + (long long)b * S * rs + h * HD;
  const int q = qt * AT + wv * 16 + lq, qmax = qt * AT + wv * 16 + 15;
  const bool qv = q < S;
  const float sl2 = scale * LOG2E;
  const float* cs = rcos + (long long)q * (HD / 2);
  const float* sn = rsin + (long long)q * (HD / 2);
  RowFrag<HD> qf, df;
  row_frags<HD>(base + (long long)q * rs, cs, sn, lg, qv, qf);
  const bf16_t* orow = o + ((long long)b * S + q) * ro + h * HD;
  const bf16_t* drow = dout + ((long long)b * S + q) * ro + h * HD;
  row_frags<HD>(drow, nullptr, nullptr, lg, qv, df);
  float dd = 0.f;
  if (qv) {  // delta = rowsum(dO * O): this lane's quarter of the head dims, then the wave sum
#pragma unroll
    for (int d0 = 4 * lg; d0 < HD; d0 += 16) {
      float dv[4], ov[4];
      row4(drow, nullptr, nullptr, d0, dv);
      row4(orow, nullptr, nullptr, d0, ov);
      dd += dv[0] * ov[0] + dv[1] * ov[1] + dv[2] * ov[2] + dv[3] * ov[3];
    }
  }
  dd += __shfl_xor(dd, 16, 64);
  dd += __shfl_xor(dd, 32, 64);
  if (qv && lg == 0) delta[((long long)b * H + h) * S + q] = dd;
  const float L2 = qv ? lse[((long long)b * H + h) * S + q] * LOG2E : 0.f;
  f4v acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f4v{0.f, 0.f, 0.f, 0.f};
  for (int kt = 0; kt <= qt; ++kt) {
    __syncthreads();
    stage_rows<HD>(base + ro, rs, kt * AT, S, rcos, rsin, Ks, Kt);
    stage_rows<HD>(base + 2 * ro, rs, kt * AT, S, nullptr, nullptr, Vs, nullptr);
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < AT / AST; ++ks) {
      const int key0 = kt * AT + ks * AST;
      if (key0 > qmax || key0 >= S) break;
      const f4v z = {0.f, 0.f, 0.f, 0.f};
      const f4v s0 = dot_hd<HD>(Ks + (ks * AST + lq) * KP, qf, lg, z);
      const f4v s1 = dot_hd<HD>(Ks + (ks * AST + 16 + lq) * KP, qf, lg, z);
      const f4v p0 = dot_hd<HD>(Vs + (ks * AST + lq) * KP, df, lg, z);
      const f4v p1 = dot_hd<HD>(Vs + (ks * AST + 16 + lq) * KP, df, lg, z);
      float ds[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int key = key0 + (i < 4 ? 4 * lg + i : 16 + 4 * lg + i - 4);
        const float sv = i < 4 ? s0[i] : s1[i - 4], dp = i < 4 ? p0[i] : p1[i - 4];
        const float pr = (qv && key <= q && key < S) ? exp2f(sv * sl2 - L2) : 0.f;
        ds[i] = pr * (dp - dd) * scale;
      }
      const s8v db = bf8(ds);
#pragma unroll
      for (int t = 0; t < NT; ++t)
        acc[t] = mma32(step_frag(Kt + (16 * t + lq) * VP + ks * AST, lg), db, acc[t]);
    }
  }
  if (qv) {
    bf16_t* out = dqkv + ((long long)b * S + q) * rs + h * HD;
#pragma unroll
    for (int t = 0; t < NT; ++t) store4_unrot(out, cs, sn, 16 * t + 4 * lg, acc[t], true);
  }
}

// dK, dV: a workgroup owns 64 keys and walks the query tiles at or after them
template <int HD>
__global__ __launch_bounds__(256) void attn_bwd_dkv_kernel(
    const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ dout, const float* __restrict__ lse,
    const float* __restrict__ delta, bf16_t* __restrict__ dqkv, const float* __restrict__ rcos,
    const float* __restrict__ rsin, int S, int H, float scale) {
  using L = AttnLds<HD>;
  constexpr int NT = L::NT, KP = L::KP, VP = L::VP;
  __shared__ __attribute__((aligned(16))) bf16_t Qs[AT * KP];
  __shared__ __attribute__((aligned(16))) bf16_t Ds[AT * KP];
  __shared__ __attribute__((aligned(16))) bf16_t Qt[HD * VP];
  __shared__ __attribute__((aligned(16))) bf16_t Dt[HD * VP];
  __shared__ float Ls[AT], Dl[AT];
  int kt, h, b;
  xcd_spread_block(kt, h, b);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, lq = lane & 15, lg = lane >> 4;
  const long long rs = 3LL * H * HD, ro = (long long)H * HD;
  const bf16_t* base = qkv + (long long)b * S * rs + h * HD;
  const bf16_t* dbase = dout + (long long)b * S * ro + h * HD;
  const int key = kt * AT + wv * 16 + lq, kmin = kt * AT + wv * 16;
  const bool kv = key < S;
  const float sl2 = scale * LOG2E;
  const float* cs = rcos + (long long)key * (HD / 2);
  const float* sn = rsin + (long long)key * (HD / 2);
  RowFrag<HD> kf, vf;
  row_frags<HD>(base + ro + (long long)key * rs, cs, sn, lg, kv, kf);
  row_frags<HD>(base + 2 * ro + (long long)key * rs, nullptr, nullptr, lg, kv, vf);
  f4v dk[NT], dv[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) dk[t] = dv[t] = f4v{0.f, 0.f, 0.f, 0.f};
  for (int qt = kt; qt * AT < S; ++qt) {
    __syncthreads();
    stage_rows<HD>(base, rs, qt * AT, S, rcos, rsin, Qs, Qt);
    stage_rows<HD>(dbase, ro, qt * AT, S, nullptr, nullptr, Ds, Dt);
    for (int e = threadIdx.x; e < AT; e += 256) {
      const int qi = qt * AT + e;
      Ls[e] = qi < S ? lse[((long long)b * H + h) * S + qi] * LOG2E : 0.f;
      Dl[e] = qi < S ? delta[((long long)b * H + h) * S + qi] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int qs = 0; qs < AT / AST; ++qs) {
      const int q0 = qt * AT + qs * AST;
      if (q0 >= S) break;
      if (q0 + AST - 1 < kmin) continue;  // every query of the step precedes every key of the wave
      const f4v z = {0.f, 0.f, 0.f, 0.f};
      const f4v s0 = dot_hd<HD>(Qs + (qs * AST + lq) * KP, kf, lg, z);
      const f4v s1 = dot_hd<HD>(Qs + (qs * AST + 16 + lq) * KP, kf, lg, z);
      const f4v d0 = dot_hd<HD>(Ds + (qs * AST + lq) * KP, vf, lg, z);
      const f4v d1 = dot_hd<HD>(Ds + (qs * AST + 16 + lq) * KP, vf, lg, z);
      float p[8], ds[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int r = qs * AST + (i < 4 ? 4 * lg + i : 16 + 4 * lg + i - 4), qi = qt * AT + r;
        const float sv = i < 4 ? s0[i] : s1[i - 4], dp = i < 4 ? d0[i] : d1[i - 4];
        p[i] = (kv && qi >= key && qi < S) ? exp2f(sv * sl2 - Ls[r]) : 0.f;
        ds[i] = p[i] * (dp - Dl[r]) * scale;
      }
      const s8v pb = bf8(p), db = bf8(ds);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        dv[t] = mma32(step_frag(Dt + (16 * t + lq) * VP + qs * AST, lg), pb, dv[t]);
        dk[t] = mma32(step_frag(Qt + (16 * t + lq) * VP + qs * AST, lg), db, dk[t]);
      }
    }
  }
  if (kv) {
    bf16_t* ko = dqkv + ((long long)b * S + key) * rs + ro + h * HD;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      store4_unrot(ko, cs, sn, 16 * t + 4 * lg, dk[t], true);
      store4_unrot(ko + ro, nullptr, nullptr, 16 * t + 4 * lg, dv[t], false);
    }
  }
}

#define ATTN_DISPATCH(KERNEL, ...)                                                       \
  switch (HD) {                                                                          \
    case 32: hipLaunchKernelGGL(KERNEL<32>, __VA_ARGS__); break;                         \
    case 48: hipLaunchKernelGGL(KERNEL<48>, __VA_ARGS__); break;                         \
    case 64: hipLaunchKernelGGL(KERNEL<64>, __VA_ARGS__); break;                         \
    case 128: hipLaunchKernelGGL(KERNEL<128>, __VA_ARGS__); break;                       \
    default: return (int)hipErrorInvalidValue;                                           \
  }

DDL_API int ddl_attn_fwd(const void* qkv, void* o, float* lse, const float* rcos, const float* rsin,
                         int B, int S, int H, int HD, float scale, hipStream_t s) {
  dim3 grid((S + AT - 1) / AT, H, B);
  ATTN_DISPATCH(attn_fwd_kernel, grid, dim3(256), 0, s, (const bf16_t*)qkv, (bf16_t*)o, lse, rcos,
                rsin, S, H, scale)
  return (int)hipGetLastError();
}

DDL_API int ddl_attn_bwd(const void* qkv, const void* o, const void* dout, const float* lse,
                         float* delta, void* dqkv, const float* rcos, const float* rsin, int B, int S,
                         int H, int HD, float scale, hipStream_t s) {
  dim3 grid((S + AT - 1) / AT, H, B);
  ATTN_DISPATCH(attn_bwd_dq_kernel, grid, dim3(256), 0, s, (const bf16_t*)qkv, (const bf16_t*)o,
                (const bf16_t*)dout, lse, delta, (bf16_t*)dqkv, rcos, rsin, S, H, scale)
  ATTN_DISPATCH(attn_bwd_dkv_kernel, grid, dim3(256), 0, s, (const bf16_t*)qkv, (const bf16_t*)dout,
                lse, delta, (bf16_t*)dqkv, rcos, rsin, S, H, scale)
  return (int)hipGetLastError();
}
