// Training-mode BatchNorm for NHWC bf16 activations with per-client (group) statistics.
//
// Forward statistics are produced by the conv epilogue (conv_igemm.hip, `stats` pointer: fp32
// per-channel sum / sum-of-squares accumulated from the MFMA accumulators), so BN forward here is
//   bn_finalize : stats -> (scale, shift, mean, rstd) + running-stat update   (G*C threads)
//   bn_apply    : y = act(x*scale + shift [+ r*rscale + rshift | + r])       (one HBM pass)
// which also fuses the ResNet residual join (identity or projected shortcut) and the ReLU.
// Backward is two passes:
//   bn_bwd_reduce : sum(dy_m), sum(dy_m * xhat)   with dy_m = dy * (y > 0) recomputed in-register
//   bn_bwd_apply  : dx = gamma*rstd*(dy_m - sum_dy/M - xhat*sum_dyx/M)   (+ emits dy_m if asked)
// The reduce pass accumulates d(gamma), d(beta) directly into the fp32 flat grad buffer.
//
// Reference parity: nn.BatchNorm1d/2d semantics (momentum 0.1, eps 1e-5, unbiased running var)
// used by the VAE models (reference lab/tutorial_2a/generative-modeling.py:21-45,
// lab/tutorial_2b/exercise_3.py:17-81) and the north-star ResNets.
#include "ddl_common.h"

struct BNArgs {
  const float* stats;    // [G][2C]: sum | sumsq   (finalize input)
  const float* gamma;    // [G][C] (group stride gs_param)
  const float* beta;
  float* running_mean;   // [G][C] (group stride gs_buf), nullable
  float* running_var;
  float* scale;          // [G][C] contiguous scratch outputs
  float* shift;
  float* mean;
  float* rstd;
  long long gs_param, gs_buf;
  int G, C;
  long long count;       // M = N*H*W per group
  float eps, momentum;
  int training, reserved;
};

__global__ void bn_finalize_kernel(BNArgs a) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.G * a.C) return;
  const int g = i / a.C, c = i - g * a.C;
  float mean, var;
  if (a.training) {
    const float* st = a.stats + (long long)g * 2 * a.C;
    const double M = (double)a.count;
    const double m = st[c] / M;
    double v = st[a.C + c] / M - m * m;
    if (v < 0) v = 0;
    mean = (float)m;
    var = (float)v;
    if (a.running_mean) {
      const long long o = (long long)g * a.gs_buf + c;
      const float unb = a.count > 1 ? (float)(v * M / (M - 1.0)) : (float)v;
      a.running_mean[o] = (1.f - a.momentum) * a.running_mean[o] + a.momentum * mean;
      a.running_var[o] = (1.f - a.momentum) * a.running_var[o] + a.momentum * unb;
    }
  } else {
    const long long o = (long long)g * a.gs_buf + c;
    mean = a.running_mean[o];
    var = a.running_var[o];
  }
  const float rs = rsqrtf(var + a.eps);
  const long long po = (long long)g * a.gs_param + c;
  const float ga = a.gamma ? a.gamma[po] : 1.f, be = a.beta ? a.beta[po] : 0.f;
  a.scale[i] = ga * rs;
  a.shift[i] = be - mean * ga * rs;
  a.mean[i] = mean;
  a.rstd[i] = rs;
}

DDL_API int ddl_bn_finalize(const BNArgs* a, hipStream_t s) {
  const int n = a->G * a->C;
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((n + 255) / 256), dim3(256), 0, s, *a);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// y = act(x*scale[c] + shift[c] + residual_term)     residual_term = r*rs[c]+rb[c] | r | 0
// act: 0 none, 1 relu, 2 leaky(0.01)
__global__ void bn_apply_kernel(const bf16_t* __restrict__ x, const float* __restrict__ scale,
                                const float* __restrict__ shift, const bf16_t* __restrict__ r,
                                const float* __restrict__ rscale, const float* __restrict__ rshift,
                                bf16_t* __restrict__ y, long long per_group, int C, int G, int act) {
  const long long chunks_pg = per_group / 8;
  const long long total = chunks_pg * G;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int g = (int)(t / chunks_pg);
    const long long e = t * 8;
    const int c0 = (int)((e - (long long)g * per_group) % C);
    const float* sc = scale + (long long)g * C + c0;
    const float* sh = shift + (long long)g * C + c0;
    float v[8];
    unpack8(*(const i4v*)(x + e), v);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = v[k] * sc[k] + sh[k];
    if (r) {
      float rv[8];
      unpack8(*(const i4v*)(r + e), rv);
      if (rscale) {
        const float* rsc = rscale + (long long)g * C + c0;
        const float* rsh = rshift + (long long)g * C + c0;
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] += rv[k] * rsc[k] + rsh[k];
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] += rv[k];
      }
    }
    if (act == 1) {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = fmaxf(v[k], 0.f);
    } else if (act == 2) {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = v[k] > 0.f ? v[k] : 0.01f * v[k];
    }
    *(i4v*)(y + e) = pack8(v);
  }
}

static int grid_for(long long work, int block) {
  long long b = (work + block - 1) / block;
  if (b > 4096) b = 4096;
  if (b < 1) b = 1;
  return (int)b;
}

DDL_API int ddl_bn_apply(const void* x, const float* scale, const float* shift, const void* r,
                         const float* rscale, const float* rshift, void* y, long long per_group,
                         int C, int G, int act, hipStream_t s) {
  if (C % 8 || per_group % C) return (int)hipErrorInvalidValue;
  const long long chunks = per_group / 8 * G;
  hipLaunchKernelGGL(bn_apply_kernel, dim3(grid_for(chunks, 256)), dim3(256), 0, s,
                     (const bf16_t*)x, scale, shift, (const bf16_t*)r, rscale, rshift, (bf16_t*)y,
                     per_group, C, G, act);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Backward reduce: per (g, c): s0 = sum dy_m, s1 = sum dy_m * xhat ; dy_m = dy * (ymask > 0)
// Thread layout: TPR = C/8 threads per pixel row (one 16-B chunk each), RPI = 256/TPR rows per
// iteration; partial sums folded through LDS, one atomic pair per (block, channel).
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ ymask, const bf16_t* __restrict__ x,
    const float* __restrict__ mean, const float* __restrict__ rstd, float* __restrict__ sums,
    float* __restrict__ dgamma, float* __restrict__ dbeta, long long gs_param, long long M, int C) {
  __shared__ float red[256 * 17];
  const int g = blockIdx.y;
  const int TPR = C / 8, RPI = 256 / TPR;
  const int tid = threadIdx.x;
  const int cc = tid % TPR, row = tid / TPR;
  const bool active = row < RPI;
  float s0[8], s1[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) s0[k] = s1[k] = 0.f;
  const long long base = (long long)g * M * C;
  const float* mu = mean + (long long)g * C + cc * 8;
  const float* rs = rstd + (long long)g * C + cc * 8;
  float m8[8], r8[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { m8[k] = mu[k]; r8[k] = rs[k]; }
  if (active) {
    for (long long p = (long long)blockIdx.x * RPI + row; p < M; p += (long long)gridDim.x * RPI) {
      const long long e = base + p * C + cc * 8;
      float d[8], xv[8];
      unpack8(*(const i4v*)(dy + e), d);
      unpack8(*(const i4v*)(x + e), xv);
      if (ymask) {
        float yv[8];
        unpack8(*(const i4v*)(ymask + e), yv);
#pragma unroll
        for (int k = 0; k < 8; ++k) if (!(yv[k] > 0.f)) d[k] = 0.f;
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        s0[k] += d[k];
        s1[k] += d[k] * (xv[k] - m8[k]) * r8[k];
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    red[tid * 17 + k] = s0[k];
    red[tid * 17 + 8 + k] = s1[k];
  }
  __syncthreads();
  if (tid < TPR) {
    float t0[8], t1[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) t0[k] = t1[k] = 0.f;
    for (int rr = 0; rr < RPI; ++rr) {
      const int src = rr * TPR + tid;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        t0[k] += red[src * 17 + k];
        t1[k] += red[src * 17 + 8 + k];
      }
    }
    float* sg = sums + (long long)g * 2 * C;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int c = tid * 8 + k;
      atomicAdd(sg + c, t0[k]);
      atomicAdd(sg + C + c, t1[k]);
      if (dbeta) atomicAdd(dbeta + (long long)g * gs_param + c, t0[k]);
      if (dgamma) atomicAdd(dgamma + (long long)g * gs_param + c, t1[k]);
    }
  }
}

DDL_API int ddl_bn_bwd_reduce(const void* dy, const void* ymask, const void* x, const float* mean,
                              const float* rstd, float* sums, float* dgamma, float* dbeta,
                              long long gs_param, long long M, int C, int G, hipStream_t s) {
  if (C % 8 || C / 8 > 256) return (int)hipErrorInvalidValue;
  const int RPI = 256 / (C / 8);
  long long want = (M + (long long)RPI * 16 - 1) / ((long long)RPI * 16);  // >=16 rows/thread
  long long cap = (1024 + G - 1) / G;
  if (cap < 4) cap = 4;
  if (want > cap) want = cap;
  if (want < 1) want = 1;
  hipLaunchKernelGGL(bn_bwd_reduce_kernel, dim3((unsigned)want, G), dim3(256), 0, s,
                     (const bf16_t*)dy, (const bf16_t*)ymask, (const bf16_t*)x, mean, rstd, sums,
                     dgamma, dbeta, gs_param, M, C);
  return (int)hipGetLastError();
}

__global__ void bn_bwd_apply_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ ymask,
                                    const bf16_t* __restrict__ x, const float* __restrict__ mean,
                                    const float* __restrict__ rstd, const float* __restrict__ gamma,
                                    long long gs_param, const float* __restrict__ sums,
                                    bf16_t* __restrict__ dx, bf16_t* __restrict__ dym_out,
                                    long long M, int C, int G) {
  const long long per_group = M * C;
  const long long chunks_pg = per_group / 8;
  const long long total = chunks_pg * G;
  const float invM = 1.f / (float)M;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int g = (int)(t / chunks_pg);
    const long long e = t * 8;
    const int c0 = (int)((e - (long long)g * per_group) % C);
    float d[8], xv[8];
    unpack8(*(const i4v*)(dy + e), d);
    unpack8(*(const i4v*)(x + e), xv);
    if (ymask) {
      float yv[8];
      unpack8(*(const i4v*)(ymask + e), yv);
#pragma unroll
      for (int k = 0; k < 8; ++k) if (!(yv[k] > 0.f)) d[k] = 0.f;
    }
    if (dym_out) *(i4v*)(dym_out + e) = pack8(d);
    const float* sg = sums + (long long)g * 2 * C;
    float o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int c = c0 + k;
      const float mu = mean[(long long)g * C + c], rs = rstd[(long long)g * C + c];
      const float ga = gamma ? gamma[(long long)g * gs_param + c] : 1.f;
      const float xh = (xv[k] - mu) * rs;
      o[k] = ga * rs * (d[k] - sg[c] * invM - xh * sg[C + c] * invM);
    }
    *(i4v*)(dx + e) = pack8(o);
  }
}

DDL_API int ddl_bn_bwd_apply(const void* dy, const void* ymask, const void* x, const float* mean,
                             const float* rstd, const float* gamma, long long gs_param,
                             const float* sums, void* dx, void* dym_out, long long M, int C, int G,
                             hipStream_t s) {
  if (C % 8) return (int)hipErrorInvalidValue;
  const long long chunks = M * C / 8 * G;
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(grid_for(chunks, 256)), dim3(256), 0, s,
                     (const bf16_t*)dy, (const bf16_t*)ymask, (const bf16_t*)x, mean, rstd, gamma,
                     gs_param, sums, (bf16_t*)dx, (bf16_t*)dym_out, M, C, G);
  return (int)hipGetLastError();
}

DDL_API int ddl_bn_args_size() { return (int)sizeof(BNArgs); }
