// Kernels of the tiny-LLaMA used by the data/pipeline-parallel tutorials (reference
// lab/tutorial_1b: simplellm LLama dmodel=288, 6 heads x 48, 6 layers, seq 256, vocab ~32k).
//
//   ddl_embedding_fwd/bwd : row gather (bf16 out) / fp32 atomic scatter-add into the grad
//   ddl_rmsnorm_fwd/bwd   : one wave per row, rstd saved, gamma grad reduced per block then atomics
//   ddl_swiglu_fwd/bwd    : h = silu(a) * b over the fused [a | b] projection
//   ddl_add               : bf16 residual add
//   ddl_attn_fwd/bwd      : causal attention with RoPE applied on the fly to q and k (so RoPE costs
//                           no HBM pass), online softmax, log-sum-exp saved; backward recomputes P
//                           (flash-attention style) in two kernels (dQ; dK+dV) and writes the
//                           un-rotated gradients straight into the fused dQKV buffer.
// Attention is VALU fp32 (head_dim 48 is not an MFMA K multiple and S=256 makes it ~1% of the
// model's FLOPs); the projections / FFN / LM head run on the MFMA implicit-GEMM kernel.
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
template <int MAXC>
__global__ __launch_bounds__(256) void rmsnorm_bwd_kernel(const bf16_t* __restrict__ x,
                                                          const float* __restrict__ g,
                                                          const float* __restrict__ rstd,
                                                          const bf16_t* __restrict__ dy,
                                                          bf16_t* __restrict__ dx,
                                                          float* __restrict__ dg, int T, int D) {
  extern __shared__ float dg_acc[];  // [D]
  for (int i = threadIdx.x; i < D; i += 256) dg_acc[i] = 0.f;
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int NC = D / 8;
  for (int row = blockIdx.x * 4 + w; row < T; row += gridDim.x * 4) {
    float xv[MAXC][8], dv[MAXC][8];
    float dot = 0.f;
    const float r = rstd[row];
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int ch = lane + 64 * c;
      if (ch < NC) {
        unpack8(*(const i4v*)(x + (long long)row * D + ch * 8), xv[c]);
        unpack8(*(const i4v*)(dy + (long long)row * D + ch * 8), dv[c]);
#pragma unroll
        for (int k = 0; k < 8; ++k) dot += g[ch * 8 + k] * dv[c][k] * xv[c][k];
      }
    }
    dot = wave_sum(dot) / D;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int ch = lane + 64 * c;
      if (ch < NC) {
        float o[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          o[k] = r * g[ch * 8 + k] * dv[c][k] - xv[c][k] * r * r * r * dot;
          atomicAdd(&dg_acc[ch * 8 + k], dv[c][k] * xv[c][k] * r);
        }
        *(i4v*)(dx + (long long)row * D + ch * 8) = pack8(o);
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < D; i += 256) atomicAdd(dg + i, dg_acc[i]);
}

DDL_API int ddl_rmsnorm_fwd(const void* x, const float* g, void* y, float* rstd, int T, int D,
                            float eps, hipStream_t s) {
  if (D % 8 || D > 64 * 8 * 4) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(rmsnorm_fwd_kernel<4>, dim3((T + 3) / 4), dim3(256), 0, s, (const bf16_t*)x, g,
                     (bf16_t*)y, rstd, T, D, eps);
  return (int)hipGetLastError();
}
DDL_API int ddl_rmsnorm_bwd(const void* x, const float* g, const float* rstd, const void* dy, void* dx,
                            float* dg, int T, int D, hipStream_t s) {
  if (D % 8 || D > 64 * 8 * 4) return (int)hipErrorInvalidValue;
  const int blocks = grid_for(T, 16, 512);
  hipLaunchKernelGGL(rmsnorm_bwd_kernel<4>, dim3(blocks), dim3(256), D * sizeof(float), s,
                     (const bf16_t*)x, g, rstd, (const bf16_t*)dy, (bf16_t*)dx, dg, T, D);
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
// Causal attention. qkv: [B][S][3][H][HD] bf16 (the fused projection output), o: [B][S][H][HD],
// lse: [B][H][S] fp32, rope: cos/sin tables [S][HD/2] fp32 (interleaved pairs (2i, 2i+1)).
// Block = 64 query rows x 4 lanes per row (each lane owns HD/4 dims); K/V tiles of 64 keys in LDS.
constexpr int QT = 64;

template <int HD>
__device__ __forceinline__ void load_rot(const bf16_t* __restrict__ src, const float* __restrict__ cs,
                                         const float* __restrict__ sn, int d0, float* out, bool rot) {
  constexpr int DL = HD / 4;
#pragma unroll
  for (int k = 0; k < DL; k += 2) {
    const float x0 = bf2f(src[d0 + k]), x1 = bf2f(src[d0 + k + 1]);
    if (rot) {
      const int pi = (d0 + k) >> 1;
      const float c = cs[pi], s = sn[pi];
      out[k] = x0 * c - x1 * s;
      out[k + 1] = x0 * s + x1 * c;
    } else {
      out[k] = x0;
      out[k + 1] = x1;
    }
  }
}

template <int HD>
__global__ __launch_bounds__(256) void attn_fwd_kernel(const bf16_t* __restrict__ qkv,
                                                       bf16_t* __restrict__ o,
                                                       float* __restrict__ lse,
                                                       const float* __restrict__ rcos,
                                                       const float* __restrict__ rsin, int S, int H,
                                                       float scale) {
  constexpr int DL = HD / 4;
  __shared__ float Ks[QT][HD + 1], Vs[QT][HD + 1];
  const int b = blockIdx.z, h = blockIdx.y, q0 = blockIdx.x * QT;
  const int tid = threadIdx.x, qi = q0 + tid / 4, sub = tid & 3, d0 = sub * DL;
  const long long rs = 3LL * H * HD;  // token stride in qkv
  const bf16_t* base = qkv + (long long)b * S * rs;
  float q[DL], acc[DL];
  const bool valid = qi < S;
  if (valid)
    load_rot<HD>(base + (long long)qi * rs + 0 * H * HD + h * HD, rcos + (long long)qi * (HD / 2),
                 rsin + (long long)qi * (HD / 2), d0, q, true);
#pragma unroll
  for (int k = 0; k < DL; ++k) { acc[k] = 0.f; if (!valid) q[k] = 0.f; }
  float m = -INFINITY, l = 0.f;
  const int kend = min(S, q0 + QT);
  for (int k0 = 0; k0 < kend; k0 += QT) {
    __syncthreads();
    for (int e = tid; e < QT * (HD / 2); e += 256) {
      const int kr = e / (HD / 2), p = e % (HD / 2), kj = k0 + kr;
      float kx0 = 0, kx1 = 0, vx0 = 0, vx1 = 0;
      if (kj < S) {
        const bf16_t* kp = base + (long long)kj * rs + 1 * H * HD + h * HD + 2 * p;
        const bf16_t* vp = base + (long long)kj * rs + 2 * H * HD + h * HD + 2 * p;
        const float c = rcos[(long long)kj * (HD / 2) + p], s = rsin[(long long)kj * (HD / 2) + p];
        const float a0 = bf2f(kp[0]), a1 = bf2f(kp[1]);
        kx0 = a0 * c - a1 * s;
        kx1 = a0 * s + a1 * c;
        vx0 = bf2f(vp[0]);
        vx1 = bf2f(vp[1]);
      }
      Ks[kr][2 * p] = kx0; Ks[kr][2 * p + 1] = kx1;
      Vs[kr][2 * p] = vx0; Vs[kr][2 * p + 1] = vx1;
    }
    __syncthreads();
    const int jmax = min(QT, kend - k0);
    for (int jj = 0; jj < jmax; ++jj) {
      const int kj = k0 + jj;
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < DL; ++k) s += q[k] * Ks[jj][d0 + k];
      s += __shfl_xor(s, 1, 64);
      s += __shfl_xor(s, 2, 64);
      s *= scale;
      if (kj > qi) s = -INFINITY;
      const float mn = fmaxf(m, s);
      const float corr = (m == -INFINITY) ? 0.f : __expf(m - mn);
      const float p = (s == -INFINITY) ? 0.f : __expf(s - mn);
      l = l * corr + p;
#pragma unroll
      for (int k = 0; k < DL; ++k) acc[k] = acc[k] * corr + p * Vs[jj][d0 + k];
      m = mn;
    }
  }
  if (valid) {
    const float inv = 1.f / l;
    bf16_t* op = o + ((long long)b * S + qi) * H * HD + h * HD + d0;
#pragma unroll
    for (int k = 0; k < DL; ++k) op[k] = f2bf(acc[k] * inv);
    if (sub == 0) lse[((long long)b * H + h) * S + qi] = m + __logf(l);
  }
}

// dQ (+ delta = rowsum(dO*O)), un-rotated into dqkv's q slot
template <int HD>
__global__ __launch_bounds__(256) void attn_bwd_dq_kernel(
    const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ o, const bf16_t* __restrict__ dout,
    const float* __restrict__ lse, float* __restrict__ delta, bf16_t* __restrict__ dqkv,
    const float* __restrict__ rcos, const float* __restrict__ rsin, int S, int H, float scale) {
  constexpr int DL = HD / 4;
  __shared__ float Ks[QT][HD + 1], Vs[QT][HD + 1];
  const int b = blockIdx.z, h = blockIdx.y, q0 = blockIdx.x * QT;
  const int tid = threadIdx.x, qi = q0 + tid / 4, sub = tid & 3, d0 = sub * DL;
  const long long rs = 3LL * H * HD;
  const bf16_t* base = qkv + (long long)b * S * rs;
  const bool valid = qi < S;
  float q[DL], dq[DL], dov[DL];
  float D = 0.f, L = 0.f;
  if (valid) {
    load_rot<HD>(base + (long long)qi * rs + h * HD, rcos + (long long)qi * (HD / 2),
                 rsin + (long long)qi * (HD / 2), d0, q, true);
    const bf16_t* op = o + ((long long)b * S + qi) * H * HD + h * HD + d0;
    const bf16_t* dp = dout + ((long long)b * S + qi) * H * HD + h * HD + d0;
#pragma unroll
    for (int k = 0; k < DL; ++k) {
      dov[k] = bf2f(dp[k]);
      D += dov[k] * bf2f(op[k]);
    }
    L = lse[((long long)b * H + h) * S + qi];
  } else {
#pragma unroll
    for (int k = 0; k < DL; ++k) { q[k] = 0.f; dov[k] = 0.f; }
  }
  D += __shfl_xor(D, 1, 64);
  D += __shfl_xor(D, 2, 64);
  if (valid && sub == 0) delta[((long long)b * H + h) * S + qi] = D;
#pragma unroll
  for (int k = 0; k < DL; ++k) dq[k] = 0.f;
  const int kend = min(S, q0 + QT);
  for (int k0 = 0; k0 < kend; k0 += QT) {
    __syncthreads();
    for (int e = tid; e < QT * (HD / 2); e += 256) {
      const int kr = e / (HD / 2), p = e % (HD / 2), kj = k0 + kr;
      float kx0 = 0, kx1 = 0, vx0 = 0, vx1 = 0;
      if (kj < S) {
        const bf16_t* kp = base + (long long)kj * rs + 1 * H * HD + h * HD + 2 * p;
        const bf16_t* vp = base + (long long)kj * rs + 2 * H * HD + h * HD + 2 * p;
        const float c = rcos[(long long)kj * (HD / 2) + p], s = rsin[(long long)kj * (HD / 2) + p];
        const float a0 = bf2f(kp[0]), a1 = bf2f(kp[1]);
        kx0 = a0 * c - a1 * s;
        kx1 = a0 * s + a1 * c;
        vx0 = bf2f(vp[0]);
        vx1 = bf2f(vp[1]);
      }
      Ks[kr][2 * p] = kx0; Ks[kr][2 * p + 1] = kx1;
      Vs[kr][2 * p] = vx0; Vs[kr][2 * p + 1] = vx1;
    }
    __syncthreads();
    const int jmax = min(QT, kend - k0);
    for (int jj = 0; jj < jmax; ++jj) {
      const int kj = k0 + jj;
      float s = 0.f, dpv = 0.f;
#pragma unroll
      for (int k = 0; k < DL; ++k) {
        s += q[k] * Ks[jj][d0 + k];
        dpv += dov[k] * Vs[jj][d0 + k];
      }
      s += __shfl_xor(s, 1, 64);
      s += __shfl_xor(s, 2, 64);
      dpv += __shfl_xor(dpv, 1, 64);
      dpv += __shfl_xor(dpv, 2, 64);
      const float p = (kj > qi || !valid) ? 0.f : __expf(s * scale - L);
      const float ds = p * (dpv - D) * scale;
#pragma unroll
      for (int k = 0; k < DL; ++k) dq[k] += ds * Ks[jj][d0 + k];
    }
  }
  if (valid) {
    bf16_t* out = dqkv + ((long long)b * S + qi) * rs + h * HD + d0;
    const float* cs = rcos + (long long)qi * (HD / 2);
    const float* sn = rsin + (long long)qi * (HD / 2);
#pragma unroll
    for (int k = 0; k < DL; k += 2) {  // inverse rotation (transpose)
      const int pi = (d0 + k) >> 1;
      const float c = cs[pi], s = sn[pi];
      out[k] = f2bf(dq[k] * c + dq[k + 1] * s);
      out[k + 1] = f2bf(-dq[k] * s + dq[k + 1] * c);
    }
  }
}

// dK, dV: block = 64 keys x 4 lanes, loop over query tiles >= key tile
template <int HD>
__global__ __launch_bounds__(256) void attn_bwd_dkv_kernel(
    const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ dout, const float* __restrict__ lse,
    const float* __restrict__ delta, bf16_t* __restrict__ dqkv, const float* __restrict__ rcos,
    const float* __restrict__ rsin, int S, int H, float scale) {
  constexpr int DL = HD / 4;
  __shared__ float Qs[QT][HD + 1], Ds[QT][HD + 1];
  __shared__ float Ls[QT], Dl[QT];
  const int b = blockIdx.z, h = blockIdx.y, k0 = blockIdx.x * QT;
  const int tid = threadIdx.x, kj = k0 + tid / 4, sub = tid & 3, d0 = sub * DL;
  const long long rs = 3LL * H * HD;
  const bf16_t* base = qkv + (long long)b * S * rs;
  const bool valid = kj < S;
  float kv[DL], vv[DL], dk[DL], dv[DL];
  if (valid) {
    load_rot<HD>(base + (long long)kj * rs + 1 * H * HD + h * HD, rcos + (long long)kj * (HD / 2),
                 rsin + (long long)kj * (HD / 2), d0, kv, true);
    load_rot<HD>(base + (long long)kj * rs + 2 * H * HD + h * HD, nullptr, nullptr, d0, vv, false);
  } else {
#pragma unroll
    for (int k = 0; k < DL; ++k) { kv[k] = 0.f; vv[k] = 0.f; }
  }
#pragma unroll
  for (int k = 0; k < DL; ++k) { dk[k] = 0.f; dv[k] = 0.f; }
  for (int q0 = k0; q0 < S; q0 += QT) {
    __syncthreads();
    for (int e = tid; e < QT * (HD / 2); e += 256) {
      const int qr = e / (HD / 2), p = e % (HD / 2), qi = q0 + qr;
      float x0 = 0, x1 = 0, g0 = 0, g1 = 0;
      if (qi < S) {
        const bf16_t* qp = base + (long long)qi * rs + h * HD + 2 * p;
        const bf16_t* dp = dout + ((long long)b * S + qi) * H * HD + h * HD + 2 * p;
        const float c = rcos[(long long)qi * (HD / 2) + p], s = rsin[(long long)qi * (HD / 2) + p];
        const float a0 = bf2f(qp[0]), a1 = bf2f(qp[1]);
        x0 = a0 * c - a1 * s;
        x1 = a0 * s + a1 * c;
        g0 = bf2f(dp[0]);
        g1 = bf2f(dp[1]);
      }
      Qs[qr][2 * p] = x0; Qs[qr][2 * p + 1] = x1;
      Ds[qr][2 * p] = g0; Ds[qr][2 * p + 1] = g1;
    }
    for (int e = tid; e < QT; e += 256) {
      const int qi = q0 + e;
      Ls[e] = qi < S ? lse[((long long)b * H + h) * S + qi] : 0.f;
      Dl[e] = qi < S ? delta[((long long)b * H + h) * S + qi] : 0.f;
    }
    __syncthreads();
    const int imax = min(QT, S - q0);
    for (int ii = 0; ii < imax; ++ii) {
      const int qi = q0 + ii;
      float s = 0.f, dpv = 0.f;
#pragma unroll
      for (int k = 0; k < DL; ++k) {
        s += Qs[ii][d0 + k] * kv[k];
        dpv += Ds[ii][d0 + k] * vv[k];
      }
      s += __shfl_xor(s, 1, 64);
      s += __shfl_xor(s, 2, 64);
      dpv += __shfl_xor(dpv, 1, 64);
      dpv += __shfl_xor(dpv, 2, 64);
      const float p = (qi < kj || !valid) ? 0.f : __expf(s * scale - Ls[ii]);
      const float ds = p * (dpv - Dl[ii]) * scale;
#pragma unroll
      for (int k = 0; k < DL; ++k) {
        dv[k] += p * Ds[ii][d0 + k];
        dk[k] += ds * Qs[ii][d0 + k];
      }
    }
  }
  if (valid) {
    bf16_t* ko = dqkv + ((long long)b * S + kj) * rs + 1 * H * HD + h * HD + d0;
    bf16_t* vo = dqkv + ((long long)b * S + kj) * rs + 2 * H * HD + h * HD + d0;
    const float* cs = rcos + (long long)kj * (HD / 2);
    const float* sn = rsin + (long long)kj * (HD / 2);
#pragma unroll
    for (int k = 0; k < DL; k += 2) {
      const int pi = (d0 + k) >> 1;
      const float c = cs[pi], s = sn[pi];
      ko[k] = f2bf(dk[k] * c + dk[k + 1] * s);
      ko[k + 1] = f2bf(-dk[k] * s + dk[k + 1] * c);
      vo[k] = f2bf(dv[k]);
      vo[k + 1] = f2bf(dv[k + 1]);
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
  dim3 grid((S + QT - 1) / QT, H, B);
  ATTN_DISPATCH(attn_fwd_kernel, grid, dim3(256), 0, s, (const bf16_t*)qkv, (bf16_t*)o, lse, rcos,
                rsin, S, H, scale)
  return (int)hipGetLastError();
}

DDL_API int ddl_attn_bwd(const void* qkv, const void* o, const void* dout, const float* lse,
                         float* delta, void* dqkv, const float* rcos, const float* rsin, int B, int S,
                         int H, int HD, float scale, hipStream_t s) {
  dim3 grid((S + QT - 1) / QT, H, B);
  ATTN_DISPATCH(attn_bwd_dq_kernel, grid, dim3(256), 0, s, (const bf16_t*)qkv, (const bf16_t*)o,
                (const bf16_t*)dout, lse, delta, (bf16_t*)dqkv, rcos, rsin, S, H, scale)
  ATTN_DISPATCH(attn_bwd_dkv_kernel, grid, dim3(256), 0, s, (const bf16_t*)qkv, (const bf16_t*)dout,
                lse, delta, (bf16_t*)dqkv, rcos, rsin, S, H, scale)
  return (int)hipGetLastError();
}
