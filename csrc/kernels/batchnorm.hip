// Training-mode BatchNorm for NHWC bf16 activations with per-client (group) statistics.
//
// Forward statistics are produced by the conv epilogue (conv_igemm.hip, `stats` pointer: fp32
// per-channel sum / sum-of-squares accumulated from the MFMA accumulators), so BN forward here is
//   bn_finalize : stats -> (scale, shift, mean, rstd) + running-stat update   (G*C threads)
//   bn_apply    : y = act(x*scale + shift [+ r*rscale + rshift | + r])       (one HBM pass)
// which also fuses the ResNet residual join (identity or projected shortcut) and the ReLU.
// Backward is three launches:
//   bn_bwd_reduce : s0 = sum(dy_m), s1 = sum(dy_m * xhat)  (dy_m = dy * (y > 0) recomputed)
//   bn_bwd_coef   : per channel  dx = A*dy_m + B*x + Cc     (folds gamma, rstd, mean, s0, s1)
//   bn_bwd_apply  : one HBM pass  (+ emits dy_m for the residual branch if asked)
// The reduce pass accumulates d(gamma), d(beta) directly into the fp32 flat grad buffer.
//
// Streaming layout shared by all passes: a 256-thread block covers RPI = 256/(C/8) pixel rows, each
// thread owns one fixed 8-channel chunk (its per-channel coefficients stay in registers, no index
// division inside the loop), blockIdx.y = client group.
//
// Reference parity: nn.BatchNorm1d/2d semantics (momentum 0.1, eps 1e-5, unbiased running var)
// used by the VAE models (reference lab/tutorial_2a/generative-modeling.py:21-45,
// lab/tutorial_2b/exercise_3.py:17-81) and the north-star ResNets.
#include "ddl_common.h"

#define BN_NSTRIPE 32  // stats / backward-partial stripes (== ops.functional.BN_STRIPES)

struct BNArgs {
  const float* stats;    // [G][stripes][2C]: sum | sumsq per stripe   (finalize input)
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
  int training, stripes;  // stripes <= 1: plain [G][2C]
};

// Stripe fold shared by finalize / fold_coef: a 256-thread block owns 32 channels of one group;
// thread (sg, cl) sums stripes sg, sg+8, ... then the 8 partial sums of each channel meet in LDS.
// Returns the totals on threads with sg == 0. The stripe count is a template constant so every
// load is issued before the first add: one memory round trip (the atomics that filled the stripes
// ran at the memory side, so these reads miss in L2), not one per stripe pair.
template <int NSTR>
__device__ __forceinline__ void stripe_fold(const float* __restrict__ base, int ns, int C, int c,
                                            bool valid, float* red, float& t0, float& t1) {
  constexpr int PER = (NSTR + 7) / 8;
  const int sg = threadIdx.x >> 5, cl = threadIdx.x & 31;
  float v0[PER], v1[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int k = sg + 8 * j;
    const bool ok = valid && k < NSTR && k < ns;
    v0[j] = ok ? base[(long long)k * 2 * C + c] : 0.f;
    v1[j] = ok ? base[(long long)k * 2 * C + C + c] : 0.f;
  }
  float a0 = 0.f, a1 = 0.f;
#pragma unroll
  for (int j = 0; j < PER; ++j) { a0 += v0[j]; a1 += v1[j]; }
  red[sg * 64 + cl] = a0;
  red[sg * 64 + 32 + cl] = a1;
  __syncthreads();
  t0 = t1 = 0.f;
  if (sg == 0) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      t0 += red[k * 64 + cl];
      t1 += red[k * 64 + 32 + cl];
    }
  }
}

__device__ __forceinline__ void bn_finalize_body(const BNArgs& a, float* red) {
  const int g = blockIdx.y, c = blockIdx.x * 32 + (threadIdx.x & 31);
  const bool valid = c < a.C;
  const bool lead = (threadIdx.x >> 5) == 0 && valid;
  // everything the tail reads is loaded up front, alongside the stripe fold's loads
  const long long po = (long long)g * a.gs_param + c, o = (long long)g * a.gs_buf + c;
  const float ga = (lead && a.gamma) ? a.gamma[po] : 1.f, be = (lead && a.beta) ? a.beta[po] : 0.f;
  const bool rs_io = lead && a.running_mean;
  const float rm0 = rs_io ? a.running_mean[o] : 0.f, rv0 = rs_io ? a.running_var[o] : 0.f;
  float mean, var;
  if (a.training) {
    float s1f, s2f;
    const float* base = a.stats + (long long)g * (a.stripes > 1 ? a.stripes : 1) * 2 * a.C;
    stripe_fold<BN_NSTRIPE>(base, a.stripes > 1 ? a.stripes : 1, a.C, c, valid, red, s1f, s2f);
    if (!lead) return;
    const double M = (double)a.count;
    const double m = (double)s1f / M;
    double v = (double)s2f / M - m * m;
    if (v < 0) v = 0;
    mean = (float)m;
    var = (float)v;
    if (a.running_mean) {
      const float unb = a.count > 1 ? (float)(v * M / (M - 1.0)) : (float)v;
      a.running_mean[o] = (1.f - a.momentum) * rm0 + a.momentum * mean;
      a.running_var[o] = (1.f - a.momentum) * rv0 + a.momentum * unb;
    }
  } else {
    if (!lead) return;
    mean = rm0;
    var = rv0;
  }
  const int i = g * a.C + c;
  const float rs = rsqrtf(var + a.eps);
  a.scale[i] = ga * rs;
  a.shift[i] = be - mean * ga * rs;
  a.mean[i] = mean;
  a.rstd[i] = rs;
}

__global__ __launch_bounds__(256) void bn_finalize_kernel(BNArgs a) {
  __shared__ float red[8 * 64];
  bn_finalize_body(a, red);
}

// Two independent BatchNorms in one launch (blockIdx.z): a residual block's output BN and its
// projected shortcut's BN, whose statistics are both complete once the two convs have run.
__global__ __launch_bounds__(256) void bn_finalize2_kernel(BNArgs a, BNArgs b) {
  __shared__ float red[8 * 64];
  bn_finalize_body(blockIdx.z ? b : a, red);
}

DDL_API int ddl_bn_finalize(const BNArgs* a, hipStream_t s) {
  if (a->stripes > BN_NSTRIPE) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((a->C + 31) / 32, a->G), dim3(256), 0, s, *a);
  return (int)hipGetLastError();
}

DDL_API int ddl_bn_finalize2(const BNArgs* a, const BNArgs* b, hipStream_t s) {
  if (a->stripes > BN_NSTRIPE || b->stripes > BN_NSTRIPE || a->G != b->G) return (int)hipErrorInvalidValue;
  const int C = a->C > b->C ? a->C : b->C;
  hipLaunchKernelGGL(bn_finalize2_kernel, dim3((C + 31) / 32, a->G, 2), dim3(256), 0, s, *a, *b);
  return (int)hipGetLastError();
}

__device__ __forceinline__ void load8f(const float* p, float* v) {
  const float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

// blocks per group for a streaming pass over M rows with RPI rows per block-iteration
static unsigned stream_blocks(long long M, int RPI, int G, int rows_per_thread) {
  long long want = (M + (long long)RPI * rows_per_thread - 1) / ((long long)RPI * rows_per_thread);
  long long cap = (2048 + G - 1) / G;
  if (cap < 8) cap = 8;
  if (want > cap) want = cap;
  if (want < 1) want = 1;
  return (unsigned)want;
}

// Grid of a striped reduce pass: every block ends with 2C fp32 atomics into the stripes, and with
// wide channels the device-wide atomic rate, not HBM, bounds the pass (ResNet-50: a 2048-channel
// reduce over 7x7 maps took 100 us in 784 blocks, 3.2M atomics, for 50 MB of input). So the
// grid is also capped at ~512K atomics per launch; each block then sweeps more rows, 4 rows'
// loads in flight per thread (REDUCE_UNROLL).
static unsigned reduce_blocks(long long M, int RPI, int G, int C) {
  unsigned b = stream_blocks(M, RPI, G, 16);
  long long cap = (512LL * 1024) / (2LL * C * G);
  if (cap < 8) cap = 8;
  if (b > cap) b = (unsigned)cap;
  return b;
}
constexpr int REDUCE_UNROLL = 4;

// ---------------------------------------------------------------------------------------------
// y = act(x*scale[c] + shift[c] + residual_term)     residual_term = r*rs[c]+rb[c] | r | 0
// act: 0 none, 1 relu, 2 leaky(0.01), 3 leaky(0.2) (DCGAN)
__global__ __launch_bounds__(256) void bn_apply_kernel(
    const bf16_t* __restrict__ x, const float* __restrict__ scale, const float* __restrict__ shift,
    const bf16_t* __restrict__ r, const float* __restrict__ rscale, const float* __restrict__ rshift,
    bf16_t* __restrict__ y, long long M, int C, int act) {
  const int g = blockIdx.y;
  const int TPR = C >> 3, RPI = 256 / TPR;
  const int cc = threadIdx.x % TPR, row = threadIdx.x / TPR;
  if (row >= RPI) return;
  float sc[8], sh[8], rsc[8], rsh[8];
  load8f(scale + (long long)g * C + cc * 8, sc);
  load8f(shift + (long long)g * C + cc * 8, sh);
  if (rscale) {
    load8f(rscale + (long long)g * C + cc * 8, rsc);
    load8f(rshift + (long long)g * C + cc * 8, rsh);
  }
  const long long base = (long long)g * M * C + cc * 8;
  // RB rows per thread per pass, all loads issued before any use: a few-client grid gives each
  // thread ~4 rows, which a one-row loop paid as 4 dependent memory round trips
  constexpr int RB = 4;
  const long long stride = (long long)gridDim.x * RPI;
  for (long long p0 = (long long)blockIdx.x * RPI + row; p0 < M; p0 += stride * RB) {
    i4v xv[RB], rv[RB];
#pragma unroll
    for (int b = 0; b < RB; ++b) {
      const long long p = p0 + b * stride;
      const long long e = base + (p < M ? p : p0) * C;
      xv[b] = *(const i4v*)(x + e);
      if (r) rv[b] = *(const i4v*)(r + e);
    }
#pragma unroll
    for (int b = 0; b < RB; ++b) {
      const long long p = p0 + b * stride;
      if (p >= M) break;
      const long long e = base + p * C;
      float v[8];
      unpack8(xv[b], v);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = v[k] * sc[k] + sh[k];
      if (r) {
        float rr[8];
        unpack8(rv[b], rr);
        if (rscale) {
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] += rr[k] * rsc[k] + rsh[k];
        } else {
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] += rr[k];
        }
      }
      if (act == 1) {
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = fmaxf(v[k], 0.f);
      } else if (act == 2) {
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = v[k] > 0.f ? v[k] : 0.01f * v[k];
      } else if (act == 3) {
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = v[k] > 0.f ? v[k] : 0.2f * v[k];
      }
      *(i4v*)(y + e) = pack8(v);
    }
  }
}

DDL_API int ddl_bn_apply(const void* x, const float* scale, const float* shift, const void* r,
                         const float* rscale, const float* rshift, void* y, long long per_group,
                         int C, int G, int act, hipStream_t s) {
  if (C % 8 || C / 8 > 256 || per_group % C) return (int)hipErrorInvalidValue;
  const long long M = per_group / C;
  const int RPI = 256 / (C / 8);
  hipLaunchKernelGGL(bn_apply_kernel, dim3(stream_blocks(M, RPI, G, 4), G), dim3(256), 0, s,
                     (const bf16_t*)x, scale, shift, (const bf16_t*)r, rscale, rshift, (bf16_t*)y,
                     M, C, act);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Backward reduce: per (g, c): s0 = sum dy_m, s1 = sum dy_m * xhat ; dy_m = dy * (ymask > 0).
// Each block folds its rows through LDS (log-depth tree), then adds into stripe
// (blockIdx.x % NSTRIPE) of part[G][NSTRIPE][2C]; bn_fold sums the stripes into sums[G][2C] and
// d(beta) += s0, d(gamma) += s1 (one thread per channel, no contended atomics).
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ ymask, const bf16_t* __restrict__ x,
    const float* __restrict__ mean, const float* __restrict__ rstd, float* __restrict__ part,
    long long M, int C) {
  __shared__ float red[256 * 17];
  const int g = blockIdx.y;
  const int TPR = C / 8, RPI = 256 / TPR;
  const int tid = threadIdx.x;
  const int cc = tid % TPR, row = tid / TPR;
  const bool active = row < RPI;
  float s0[8], s1[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) s0[k] = s1[k] = 0.f;
  float m8[8], r8[8];
  load8f(mean + (long long)g * C + cc * 8, m8);
  load8f(rstd + (long long)g * C + cc * 8, r8);
  const long long base = (long long)g * M * C + cc * 8;
  if (active) {
    const long long stride = (long long)gridDim.x * RPI;
    for (long long p0 = (long long)blockIdx.x * RPI + row; p0 < M; p0 += stride * REDUCE_UNROLL) {
      i4v rd[REDUCE_UNROLL], rx[REDUCE_UNROLL], rm[REDUCE_UNROLL];
#pragma unroll
      for (int u = 0; u < REDUCE_UNROLL; ++u) {  // all loads first: 4 rows in flight
        const long long p = p0 + u * stride;
        if (p < M) {
          const long long e = base + p * C;
          rd[u] = *(const i4v*)(dy + e);
          rx[u] = *(const i4v*)(x + e);
          if (ymask) rm[u] = *(const i4v*)(ymask + e);
        }
      }
#pragma unroll
      for (int u = 0; u < REDUCE_UNROLL; ++u) {
        if (p0 + u * stride >= M) break;
        float d[8], xv[8];
        unpack8(rd[u], d);
        unpack8(rx[u], xv);
        if (ymask) {
          float yv[8];
          unpack8(rm[u], yv);
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
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    red[tid * 17 + k] = s0[k];
    red[tid * 17 + 8 + k] = s1[k];
  }
  __syncthreads();
  int top = 1;
  while (top < RPI) top <<= 1;
  for (int half = top >> 1; half > 0; half >>= 1) {  // RPI need not be a power of two (C = 96 ...)
    if (row < half && row + half < RPI) {
      const float* o = red + (tid + half * TPR) * 17;
      float* m = red + tid * 17;
#pragma unroll
      for (int k = 0; k < 16; ++k) m[k] += o[k];
    }
    __syncthreads();
  }
  if (row == 0) {
    float* pg = part + ((long long)g * BN_NSTRIPE + blockIdx.x % BN_NSTRIPE) * 2 * C;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      atomicAdd(pg + cc * 8 + k, red[tid * 17 + k]);
      atomicAdd(pg + C + cc * 8 + k, red[tid * 17 + 8 + k]);
    }
  }
}

__global__ void bn_fold_kernel(const float* __restrict__ part, float* __restrict__ sums,
                               float* __restrict__ dgamma, float* __restrict__ dbeta,
                               long long gs_param, int C, int G) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= G * C) return;
  const int g = i / C, c = i - g * C;
  const float* pg = part + (long long)g * BN_NSTRIPE * 2 * C;
  float t0 = 0.f, t1 = 0.f;
#pragma unroll 8
  for (int k = 0; k < BN_NSTRIPE; ++k) {
    t0 += pg[(long long)k * 2 * C + c];
    t1 += pg[(long long)k * 2 * C + C + c];
  }
  sums[(long long)g * 2 * C + c] = t0;
  sums[(long long)g * 2 * C + C + c] = t1;
  if (dbeta) dbeta[(long long)g * gs_param + c] += t0;
  if (dgamma) dgamma[(long long)g * gs_param + c] += t1;
}

// part: zeroed [G][BN_NSTRIPE][2C] scratch; sums: [G][2C] output
DDL_API int ddl_bn_bwd_reduce(const void* dy, const void* ymask, const void* x, const float* mean,
                              const float* rstd, float* part, float* sums, float* dgamma,
                              float* dbeta, long long gs_param, long long M, int C, int G,
                              hipStream_t s) {
  if (C % 8 || C / 8 > 256) return (int)hipErrorInvalidValue;
  const int RPI = 256 / (C / 8);
  hipLaunchKernelGGL(bn_bwd_reduce_kernel, dim3(reduce_blocks(M, RPI, G, C), G), dim3(256), 0, s,
                     (const bf16_t*)dy, (const bf16_t*)ymask, (const bf16_t*)x, mean, rstd, part,
                     M, C);
  hipLaunchKernelGGL(bn_fold_kernel, dim3((G * C + 255) / 256), dim3(256), 0, s, part, sums, dgamma,
                     dbeta, gs_param, C, G);
  return (int)hipGetLastError();
}

DDL_API int ddl_bn_nstripe() { return BN_NSTRIPE; }

// dx = gamma*rstd*(dy_m - s0/M - xhat*s1/M) = A*dy_m + B*x + Cc
__global__ void bn_bwd_coef_kernel(const float* __restrict__ mean, const float* __restrict__ rstd,
                                   const float* __restrict__ gamma, long long gs_param,
                                   const float* __restrict__ sums, float* __restrict__ coef,
                                   long long M, int C, int G) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= G * C) return;
  const int g = i / C, c = i - g * C;
  const float invM = 1.f / (float)M;
  const float mu = mean[i], rs = rstd[i];
  const float ga = gamma ? gamma[(long long)g * gs_param + c] : 1.f;
  const float s0 = sums[(long long)g * 2 * C + c], s1 = sums[(long long)g * 2 * C + C + c];
  const float A = ga * rs;
  const float B = -A * rs * s1 * invM;
  coef[(long long)g * 3 * C + c] = A;
  coef[(long long)g * 3 * C + C + c] = B;
  coef[(long long)g * 3 * C + 2 * C + c] = -A * s0 * invM - B * mu;
}

__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ ymask, const bf16_t* __restrict__ x,
    const float* __restrict__ coef, bf16_t* __restrict__ dx, bf16_t* __restrict__ dym_out,
    long long M, int C) {
  const int g = blockIdx.y;
  const int TPR = C >> 3, RPI = 256 / TPR;
  const int cc = threadIdx.x % TPR, row = threadIdx.x / TPR;
  if (row >= RPI) return;
  float A[8], B[8], Cc[8];
  const float* cg = coef + (long long)g * 3 * C + cc * 8;
  load8f(cg, A);
  load8f(cg + C, B);
  load8f(cg + 2 * C, Cc);
  const long long base = (long long)g * M * C + cc * 8;
  constexpr int RB = 4;  // rows per thread per pass, loads first (see bn_apply_kernel)
  const long long stride = (long long)gridDim.x * RPI;
  for (long long p0 = (long long)blockIdx.x * RPI + row; p0 < M; p0 += stride * RB) {
    i4v dv[RB], xv[RB], mv[RB];
#pragma unroll
    for (int b = 0; b < RB; ++b) {
      const long long p = p0 + b * stride;
      const long long e = base + (p < M ? p : p0) * C;
      dv[b] = *(const i4v*)(dy + e);
      xv[b] = *(const i4v*)(x + e);
      if (ymask) mv[b] = *(const i4v*)(ymask + e);
    }
#pragma unroll
    for (int b = 0; b < RB; ++b) {
      const long long p = p0 + b * stride;
      if (p >= M) break;
      const long long e = base + p * C;
      float d[8], xf[8];
      unpack8(dv[b], d);
      unpack8(xv[b], xf);
      if (ymask) {
        float yv[8];
        unpack8(mv[b], yv);
#pragma unroll
        for (int k = 0; k < 8; ++k) if (!(yv[k] > 0.f)) d[k] = 0.f;
      }
      if (dym_out) *(i4v*)(dym_out + e) = pack8(d);
      float o[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = A[k] * d[k] + B[k] * xf[k] + Cc[k];
      *(i4v*)(dx + e) = pack8(o);
    }
  }
}

DDL_API int ddl_bn_bwd_apply(const void* dy, const void* ymask, const void* x, const float* mean,
                             const float* rstd, const float* gamma, long long gs_param,
                             const float* sums, float* coef_ws, void* dx, void* dym_out,
                             long long M, int C, int G, hipStream_t s) {
  if (C % 8 || C / 8 > 256) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(bn_bwd_coef_kernel, dim3((G * C + 255) / 256), dim3(256), 0, s, mean, rstd,
                     gamma, gs_param, sums, coef_ws, M, C, G);
  const int RPI = 256 / (C / 8);
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(stream_blocks(M, RPI, G, 4), G), dim3(256), 0, s,
                     (const bf16_t*)dy, (const bf16_t*)ymask, (const bf16_t*)x, coef_ws,
                     (bf16_t*)dx, (bf16_t*)dym_out, M, C);
  return (int)hipGetLastError();
}

DDL_API int ddl_bn_args_size() { return (int)sizeof(BNArgs); }

// ---------------------------------------------------------------------------------------------
// Standalone forward statistics (for producers without the conv epilogue: transposed convs,
// linears of the GAN / tabular nets): stats[g][stripe][c] += sum x, [..][C + c] += sum x^2
// (stats is [G][BN_NSTRIPE][2C], finalize with stripes = BN_NSTRIPE).
// Same streaming layout; the RPI rows of one block are folded through LDS, one atomic per channel
// per block.
__global__ __launch_bounds__(256) void bn_stats_kernel(const bf16_t* __restrict__ x,
                                                       float* __restrict__ stats, long long M, int C) {
  __shared__ float red[256 * 16];
  const int g = blockIdx.y;
  const int TPR = C >> 3, RPI = 256 / TPR;
  const int cc = threadIdx.x % TPR, row = threadIdx.x / TPR;
  float s1[8] = {}, s2[8] = {};
  if (row < RPI) {
    const long long base = (long long)g * M * C + cc * 8;
    const long long stride = (long long)gridDim.x * RPI;
    for (long long p0 = (long long)blockIdx.x * RPI + row; p0 < M; p0 += stride * REDUCE_UNROLL) {
      i4v rv[REDUCE_UNROLL];
#pragma unroll
      for (int u = 0; u < REDUCE_UNROLL; ++u)
        if (p0 + u * stride < M) rv[u] = *(const i4v*)(x + base + (p0 + u * stride) * C);
#pragma unroll
      for (int u = 0; u < REDUCE_UNROLL; ++u) {
        if (p0 + u * stride >= M) break;
        float v[8];
        unpack8(rv[u], v);
#pragma unroll
        for (int k = 0; k < 8; ++k) { s1[k] += v[k]; s2[k] += v[k] * v[k]; }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) { red[threadIdx.x * 16 + k] = s1[k]; red[threadIdx.x * 16 + 8 + k] = s2[k]; }
  __syncthreads();
  if (row == 0) {
    for (int r = 1; r < RPI; ++r) {
      const float* o = red + (r * TPR + cc) * 16;
#pragma unroll
      for (int k = 0; k < 8; ++k) { s1[k] += o[k]; s2[k] += o[8 + k]; }
    }
    float* st = stats + ((long long)g * BN_NSTRIPE + blockIdx.x % BN_NSTRIPE) * 2 * C + cc * 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) { atomicAdd(st + k, s1[k]); atomicAdd(st + C + k, s2[k]); }
  }
}

DDL_API int ddl_bn_stats(const void* x, float* stats, long long M, int C, int G, hipStream_t s) {
  if (C % 8 || C / 8 > 256) return (int)hipErrorInvalidValue;
  const int RPI = 256 / (C / 8);
  hipLaunchKernelGGL(bn_stats_kernel, dim3(reduce_blocks(M, RPI, G, C), G), dim3(256), 0, s,
                     (const bf16_t*)x, stats, M, C);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Whole BN backward in three launches: striped reduce -> per-channel fold (d(beta) += s0,
// d(gamma) += s1, dx coefficients) -> one apply pass.
__device__ __forceinline__ void bn_fold_coef_body(
    const float* __restrict__ part, float* __restrict__ dgamma, float* __restrict__ dbeta,
    long long gs_param, const float* __restrict__ mean, const float* __restrict__ rstd,
    const float* __restrict__ gamma, float* __restrict__ coef, long long M, int C, float* red) {
  const int g = blockIdx.y, c = blockIdx.x * 32 + (threadIdx.x & 31);
  const bool valid = c < C;
  const bool lead = (threadIdx.x >> 5) == 0 && valid;
  const int i = g * C + c;
  const long long po = (long long)g * gs_param + c;
  // the tail's inputs load with the stripe fold's (one round trip)
  const float mu = lead ? mean[i] : 0.f, rs = lead ? rstd[i] : 0.f;
  const float ga = (lead && gamma) ? gamma[po] : 1.f;
  const float db0 = (lead && dbeta) ? dbeta[po] : 0.f, dg0 = (lead && dgamma) ? dgamma[po] : 0.f;
  float s0, s1;
  stripe_fold<BN_NSTRIPE>(part + (long long)g * BN_NSTRIPE * 2 * C, BN_NSTRIPE, C, c, valid, red, s0, s1);
  if (!lead) return;
  if (dbeta) dbeta[po] = db0 + s0;
  if (dgamma) dgamma[po] = dg0 + s1;
  const float invM = 1.f / (float)M;
  const float A = ga * rs;
  const float B = -A * rs * s1 * invM;
  coef[(long long)g * 3 * C + c] = A;
  coef[(long long)g * 3 * C + C + c] = B;
  coef[(long long)g * 3 * C + 2 * C + c] = -A * s0 * invM - B * mu;
}

__global__ __launch_bounds__(256) void bn_fold_coef_kernel(
    const float* __restrict__ part, float* __restrict__ dgamma, float* __restrict__ dbeta,
    long long gs_param, const float* __restrict__ mean, const float* __restrict__ rstd,
    const float* __restrict__ gamma, float* __restrict__ coef, long long M, int C, int G) {
  __shared__ float red[8 * 64];
  bn_fold_coef_body(part, dgamma, dbeta, gs_param, mean, rstd, gamma, coef, M, C, red);
}

// ---------------------------------------------------------------------------------------------
// Two BatchNorm backwards that share their (already masked) input gradient dy: a residual block's
// output BN and its projected shortcut's BN, both fed by the block's output gradient. One fold
// launch (blockIdx.z) and one apply pass that reads dy once and writes both input gradients.
struct BNBwdArgs {
  const void* x;         // BN input [G][M][C] bf16
  const float* mean;     // [G][C]
  const float* rstd;
  const float* gamma;    // [G][C] (group stride gs_param), nullable
  float* dgamma;         // nullable
  float* dbeta;
  const float* part;     // complete striped reduce sums [G][BN_NSTRIPE][2C]
  float* coef;           // [G][3C] scratch
  void* dx;              // [G][M][C] bf16 output
  long long gs_param;
};

__global__ __launch_bounds__(256) void bn_fold_coef2_kernel(BNBwdArgs a, BNBwdArgs b, long long M, int C) {
  __shared__ float red[8 * 64];
  const BNBwdArgs& t = blockIdx.z ? b : a;
  bn_fold_coef_body(t.part, t.dgamma, t.dbeta, t.gs_param, t.mean, t.rstd, t.gamma, t.coef, M, C, red);
}

__global__ __launch_bounds__(256) void bn_bwd_apply2_kernel(const bf16_t* __restrict__ dy, BNBwdArgs a,
                                                            BNBwdArgs b, long long M, int C) {
  const int g = blockIdx.y;
  const int TPR = C >> 3, RPI = 256 / TPR;
  const int cc = threadIdx.x % TPR, row = threadIdx.x / TPR;
  if (row >= RPI) return;
  float Aa[8], Ba[8], Ca[8], Ab[8], Bb[8], Cb[8];
  const float* ca = a.coef + (long long)g * 3 * C + cc * 8;
  const float* cb = b.coef + (long long)g * 3 * C + cc * 8;
  load8f(ca, Aa); load8f(ca + C, Ba); load8f(ca + 2 * C, Ca);
  load8f(cb, Ab); load8f(cb + C, Bb); load8f(cb + 2 * C, Cb);
  const bf16_t* __restrict__ xa = (const bf16_t*)a.x;
  const bf16_t* __restrict__ xb = (const bf16_t*)b.x;
  bf16_t* __restrict__ dxa = (bf16_t*)a.dx;
  bf16_t* __restrict__ dxb = (bf16_t*)b.dx;
  const long long base = (long long)g * M * C + cc * 8;
  constexpr int RB = 4;
  const long long stride = (long long)gridDim.x * RPI;
  for (long long p0 = (long long)blockIdx.x * RPI + row; p0 < M; p0 += stride * RB) {
    i4v dv[RB], av[RB], bv[RB];
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const long long p = p0 + r * stride;
      const long long e = base + (p < M ? p : p0) * C;
      dv[r] = *(const i4v*)(dy + e);
      av[r] = *(const i4v*)(xa + e);
      bv[r] = *(const i4v*)(xb + e);
    }
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const long long p = p0 + r * stride;
      if (p >= M) break;
      const long long e = base + p * C;
      float d[8], xf[8], o[8];
      unpack8(dv[r], d);
      unpack8(av[r], xf);
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = Aa[k] * d[k] + Ba[k] * xf[k] + Ca[k];
      *(i4v*)(dxa + e) = pack8(o);
      unpack8(bv[r], xf);
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = Ab[k] * d[k] + Bb[k] * xf[k] + Cb[k];
      *(i4v*)(dxb + e) = pack8(o);
    }
  }
}

DDL_API int ddl_bn_bwd_args_size() { return (int)sizeof(BNBwdArgs); }

DDL_API int ddl_bn_backward2(const void* dy, const BNBwdArgs* a, const BNBwdArgs* b, long long M, int C,
                             int G, hipStream_t s) {
  if (C % 8 || C / 8 > 256) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(bn_fold_coef2_kernel, dim3((C + 31) / 32, G, 2), dim3(256), 0, s, *a, *b, M, C);
  const int RPI = 256 / (C / 8);
  hipLaunchKernelGGL(bn_bwd_apply2_kernel, dim3(stream_blocks(M, RPI, G, 4), G), dim3(256), 0, s,
                     (const bf16_t*)dy, *a, *b, M, C);
  return (int)hipGetLastError();
}

// striped reduce sums only (part zeroed [G][BN_NSTRIPE][2C]): s0 = sum dy_m, s1 = sum dy_m * xhat
DDL_API int ddl_bn_bwd_reduce_part(const void* dy, const void* ymask, const void* x, const float* mean,
                                   const float* rstd, float* part, long long M, int C, int G, hipStream_t s) {
  if (C % 8 || C / 8 > 256) return (int)hipErrorInvalidValue;
  const int RPI = 256 / (C / 8);
  hipLaunchKernelGGL(bn_bwd_reduce_kernel, dim3(reduce_blocks(M, RPI, G, C), G), dim3(256), 0, s,
                     (const bf16_t*)dy, (const bf16_t*)ymask, (const bf16_t*)x, mean, rstd, part, M, C);
  return (int)hipGetLastError();
}

// part: zeroed [G][BN_NSTRIPE][2C]; coef: [G][3C] scratch
// do_reduce = 0: `part` was already filled by the producer of dy (conv dgrad epilogue with the
// fused BN reduce), so the backward is two launches.
DDL_API int ddl_bn_backward(const void* dy, const void* ymask, const void* x, const float* mean,
                            const float* rstd, const float* gamma, long long gs_param, float* part,
                            float* coef, float* dgamma, float* dbeta, void* dx, void* dym_out,
                            long long M, int C, int G, int do_reduce, hipStream_t s) {
  if (C % 8 || C / 8 > 256) return (int)hipErrorInvalidValue;
  const int RPI = 256 / (C / 8);
  if (do_reduce) hipLaunchKernelGGL(bn_bwd_reduce_kernel, dim3(reduce_blocks(M, RPI, G, C), G), dim3(256), 0, s,
                     (const bf16_t*)dy, (const bf16_t*)ymask, (const bf16_t*)x, mean, rstd, part,
                     M, C);
  hipLaunchKernelGGL(bn_fold_coef_kernel, dim3((C + 31) / 32, G), dim3(256), 0, s, part, dgamma,
                     dbeta, gs_param, mean, rstd, gamma, coef, M, C, G);
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(stream_blocks(M, RPI, G, 4), G), dim3(256), 0, s,
                     (const bf16_t*)dy, (const bf16_t*)ymask, (const bf16_t*)x, coef, (bf16_t*)dx,
                     (bf16_t*)dym_out, M, C);
  return (int)hipGetLastError();
}
