// Tabular / small-MLP kernels (heart-disease split-NN, tabular VAE, VFL-VAE, HeartDiseaseNN):
// exact fp32 (the reference trains these nets in fp32; reference lab/tutorial_2a/*.py,
// lab/tutorial_2b/*.py), latency-bound shapes (<= 1,025 rows, <= 256 features).
//
//   gemm_f32      C = act(op(A) op(B) + bias) (+ C)   on v_mfma_f32_16x16x4f32 (exact fp32),
//                 arbitrary M, N, K and strides (so x W^T, dY W and dY^T X are one kernel);
//                 LDS-staged 32x32 block tile, 4 waves x one 16x16 MFMA tile each
//   bias_act_bwd  dZ = dY * act'(Y)  and  db += colsum(dZ)         (one pass)
//   bn1d_fwd      BatchNorm1d training/eval + fused ReLU / LeakyReLU (two-pass fp32 statistics,
//                 running-stat update with unbiased variance, torch semantics)
//   bn1d_bwd      dX, d(gamma), d(beta) from the saved output (activation mask) and input
//   ce_soft_f32   softmax CE with probability targets or hard labels, mean, fused gradient
//   reparam       z = mu + eps * exp(logvar / 2), eps ~ N(0,1) from Philox (Box-Muller), eps kept
#include "ddl_common.h"

__device__ __forceinline__ float act_f(float v, int act, float slope) {
  return act == 1 ? fmaxf(v, 0.f) : (act == 2 ? (v > 0.f ? v : slope * v) : v);
}
__device__ __forceinline__ float act_grad_from_out(float y, int act, float slope) {
  return act == 1 ? (y > 0.f ? 1.f : 0.f) : (act == 2 ? (y > 0.f ? 1.f : slope) : 1.f);
}

// ---------------------------------------------------------------------------------------------
struct GemmF32Args {
  const float* A; const float* B; float* C; const float* bias;
  long long sam, sak, sbk, sbn, ldc;  // element strides: A(m,k) = A[m*sam + k*sak], ...
  int M, N, K, act, accumulate, reserved;
  float slope, alpha;
};

__global__ __launch_bounds__(256) void gemm_f32_kernel(GemmF32Args a) {
  constexpr int BM = 32, BN = 32, KC = 32, LD = KC + 1;
  __shared__ float As[BM * LD], Bs[BN * LD];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int wm = (wid >> 1) * 16, wn = (wid & 1) * 16;
  f4v acc = {0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < a.K; k0 += KC) {
    __syncthreads();
    for (int e = tid; e < BM * KC; e += 256) {
      const int r = e / KC, kk = e - r * KC;
      const int m = m0 + r, k = k0 + kk, n = n0 + r;
      As[r * LD + kk] = (m < a.M && k < a.K) ? a.A[m * a.sam + k * a.sak] : 0.f;
      Bs[r * LD + kk] = (n < a.N && k < a.K) ? a.B[k * a.sbk + n * a.sbn] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < KC; k += 4) {
      const float av = As[(wm + (lane & 15)) * LD + k + (lane >> 4)];
      const float bv = Bs[(wn + (lane & 15)) * LD + k + (lane >> 4)];
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc, 0, 0, 0);
    }
  }
  // C/D layout: col = lane & 15, rows 4*(lane >> 4) + i
  const int n = n0 + wn + (lane & 15);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + wm + 4 * (lane >> 4) + i;
    if (m < a.M && n < a.N) {
      float v = a.alpha * acc[i] + (a.bias ? a.bias[n] : 0.f);
      v = act_f(v, a.act, a.slope);
      float* dst = a.C + m * a.ldc + n;
      *dst = a.accumulate ? *dst + v : v;
    }
  }
}

DDL_API int ddl_gemm_f32(const GemmF32Args* a, hipStream_t s) {
  if (a->M <= 0 || a->N <= 0 || a->K <= 0) return 0;
  dim3 grid((a->N + 31) / 32, (a->M + 31) / 32);
  hipLaunchKernelGGL(gemm_f32_kernel, grid, dim3(256), 0, s, *a);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// dZ = dY * act'(Y) ; db[n] += sum_m dZ[m][n]. Block = 32 columns x 8 row groups.
__global__ __launch_bounds__(256) void bias_act_bwd_kernel(const float* __restrict__ dy,
                                                           const float* __restrict__ y,
                                                           float* __restrict__ dz,
                                                           float* __restrict__ db, int M, int N,
                                                           int act, float slope) {
  __shared__ float red[8 * 32];
  const int c = blockIdx.x * 32 + (threadIdx.x & 31), rg = threadIdx.x >> 5;
  float s = 0.f;
  if (c < N)
    for (int m = rg; m < M; m += 8) {
      const long long o = (long long)m * N + c;
      const float g = dy[o] * (y ? act_grad_from_out(y[o], act, slope) : 1.f);
      if (dz) dz[o] = g;
      s += g;
    }
  red[rg * 32 + (threadIdx.x & 31)] = s;
  __syncthreads();
  if (rg == 0 && c < N && db) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) t += red[k * 32 + threadIdx.x];
    db[c] += t;
  }
}

DDL_API int ddl_bias_act_bwd(const float* dy, const float* y, float* dz, float* db, int M, int N,
                             int act, float slope, hipStream_t s) {
  hipLaunchKernelGGL(bias_act_bwd_kernel, dim3((N + 31) / 32), dim3(256), 0, s, dy, y, dz, db, M, N,
                     act, slope);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// BatchNorm1d over [M][C] fp32, block = 32 channels x 8 row groups (LDS reduce), fused act.
__device__ __forceinline__ float block_col_sum(float v, float* red) {
  const int cl = threadIdx.x & 31, rg = threadIdx.x >> 5;
  __syncthreads();
  red[rg * 32 + cl] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) t += red[k * 32 + cl];
  return t;  // every thread of the column gets the total
}

__global__ __launch_bounds__(256) void bn1d_fwd_kernel(
    const float* __restrict__ x, const float* __restrict__ gamma, const float* __restrict__ beta,
    float* __restrict__ rmean, float* __restrict__ rvar, float* __restrict__ y,
    float* __restrict__ mean_out, float* __restrict__ rstd_out, int M, int C, int training,
    float momentum, float eps, int act, float slope) {
  __shared__ float red[8 * 32];
  const int c = blockIdx.x * 32 + (threadIdx.x & 31), rg = threadIdx.x >> 5;
  const bool ok = c < C;
  float mean, var;
  if (training) {
    float s = 0.f;
    if (ok)
      for (int m = rg; m < M; m += 8) s += x[(long long)m * C + c];
    mean = block_col_sum(s, red) / (float)M;
    float q = 0.f;
    if (ok)
      for (int m = rg; m < M; m += 8) {
        const float d = x[(long long)m * C + c] - mean;
        q += d * d;
      }
    var = block_col_sum(q, red) / (float)M;
    if (ok && rg == 0 && rmean) {
      const float unb = M > 1 ? var * (float)M / (float)(M - 1) : var;
      rmean[c] = (1.f - momentum) * rmean[c] + momentum * mean;
      rvar[c] = (1.f - momentum) * rvar[c] + momentum * unb;
    }
  } else {
    mean = ok ? rmean[c] : 0.f;
    var = ok ? rvar[c] : 1.f;
  }
  if (!ok) return;
  const float rs = rsqrtf(var + eps);
  const float ga = gamma ? gamma[c] : 1.f, be = beta ? beta[c] : 0.f;
  if (rg == 0) {
    if (mean_out) mean_out[c] = mean;
    if (rstd_out) rstd_out[c] = rs;
  }
  for (int m = rg; m < M; m += 8) {
    const long long o = (long long)m * C + c;
    y[o] = act_f((x[o] - mean) * rs * ga + be, act, slope);
  }
}

DDL_API int ddl_bn1d_fwd(const float* x, const float* gamma, const float* beta, float* rmean,
                         float* rvar, float* y, float* mean_out, float* rstd_out, int M, int C,
                         int training, float momentum, float eps, int act, float slope,
                         hipStream_t s) {
  hipLaunchKernelGGL(bn1d_fwd_kernel, dim3((C + 31) / 32), dim3(256), 0, s, x, gamma, beta, rmean,
                     rvar, y, mean_out, rstd_out, M, C, training, momentum, eps, act, slope);
  return (int)hipGetLastError();
}

// dy_m = dy * act'(y) ; xhat = (x - mean) * rstd ; dbeta = sum dy_m ; dgamma = sum dy_m xhat
// dx = gamma * rstd * (dy_m - dbeta / M - xhat * dgamma / M)      (training-mode statistics)
__global__ __launch_bounds__(256) void bn1d_bwd_kernel(
    const float* __restrict__ dy, const float* __restrict__ y, const float* __restrict__ x,
    const float* __restrict__ mean, const float* __restrict__ rstd, const float* __restrict__ gamma,
    float* __restrict__ dx, float* __restrict__ dgamma, float* __restrict__ dbeta, int M, int C,
    int act, float slope, int training) {
  __shared__ float red[8 * 32];
  const int c = blockIdx.x * 32 + (threadIdx.x & 31), rg = threadIdx.x >> 5;
  const bool ok = c < C;
  const float mu = ok ? mean[c] : 0.f, rs = ok ? rstd[c] : 0.f;
  float s0 = 0.f, s1 = 0.f;
  if (ok)
    for (int m = rg; m < M; m += 8) {
      const long long o = (long long)m * C + c;
      const float g = dy[o] * act_grad_from_out(y[o], act, slope);
      s0 += g;
      s1 += g * (x[o] - mu) * rs;
    }
  s0 = block_col_sum(s0, red);
  s1 = block_col_sum(s1, red);
  if (!ok) return;
  if (rg == 0) {
    if (dbeta) dbeta[c] += s0;
    if (dgamma) dgamma[c] += s1;
  }
  const float ga = gamma ? gamma[c] : 1.f;
  const float invM = 1.f / (float)M;
  for (int m = rg; m < M; m += 8) {
    const long long o = (long long)m * C + c;
    const float g = dy[o] * act_grad_from_out(y[o], act, slope);
    const float xh = (x[o] - mu) * rs;
    // eval mode (running statistics): the normalisation is a fixed affine map
    dx[o] = training ? ga * rs * (g - s0 * invM - xh * s1 * invM) : ga * rs * g;
  }
}

DDL_API int ddl_bn1d_bwd(const float* dy, const float* y, const float* x, const float* mean,
                         const float* rstd, const float* gamma, float* dx, float* dgamma,
                         float* dbeta, int M, int C, int act, float slope, int training, hipStream_t s) {
  hipLaunchKernelGGL(bn1d_bwd_kernel, dim3((C + 31) / 32), dim3(256), 0, s, dy, y, x, mean, rstd,
                     gamma, dx, dgamma, dbeta, M, C, act, slope, training);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Softmax CE on fp32 logits [M][C]: one wave per row, each lane over columns lane, lane + 64, ...
// targets: probabilities [M][C] (the VFL float one-hot) or labels [M] (int).
// loss (fp32 scalar) += mean; dlogits = (p * sum(t) - t) / M
__global__ __launch_bounds__(256) void ce_f32_kernel(const float* __restrict__ logits,
                                                     const float* __restrict__ targets,
                                                     const int* __restrict__ labels, int M, int C,
                                                     float* __restrict__ loss,
                                                     float* __restrict__ dlogits) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const float* lg = logits + (long long)row * C;
  float mx = -INFINITY;
  for (int c = lane; c < C; c += 64) mx = fmaxf(mx, lg[c]);
  mx = wave_max(mx);
  float se = 0.f, tsum = 0.f, tl = 0.f;
  for (int c = lane; c < C; c += 64) {
    const float v = lg[c];
    se += __expf(v - mx);
    const float t = targets ? targets[(long long)row * C + c] : (labels[row] == c ? 1.f : 0.f);
    tsum += t;
    tl += t * v;
  }
  se = wave_sum(se);
  tsum = wave_sum(tsum);
  tl = wave_sum(tl);
  const float lse = mx + __logf(se);
  if (dlogits) {
    for (int c = lane; c < C; c += 64) {
      const float t = targets ? targets[(long long)row * C + c] : (labels[row] == c ? 1.f : 0.f);
      dlogits[(long long)row * C + c] = (__expf(lg[c] - mx) / se * tsum - t) / (float)M;
    }
  }
  if (lane == 0) atomicAdd(loss, (tsum * lse - tl) / (float)M);
}

DDL_API int ddl_ce_f32(const float* logits, const float* targets, const int* labels, int M, int C,
                       float* loss, float* dlogits, hipStream_t s) {
  if (C < 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(ce_f32_kernel, dim3((M + 3) / 4), dim3(256), 0, s, logits, targets, labels, M,
                     C, loss, dlogits);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// z = mu + eps * exp(0.5 * logvar); eps from Philox(seed, offset + element) via Box-Muller.
__global__ void reparam_kernel(const float* __restrict__ mu, const float* __restrict__ lv,
                               float* __restrict__ eps, float* __restrict__ z, long long n,
                               unsigned long long seed, unsigned long long offset) {
  const uint2 key = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
  GSTRIDE_LOOP(i, n) {
    const unsigned long long c = offset + (unsigned long long)i;
    const uint4 r = philox4x32(make_uint4((uint32_t)c, (uint32_t)(c >> 32), 0x2545F491u, 0), key);
    const float u1 = fmaxf(u32_to_unit(r.x), 1e-12f), u2 = u32_to_unit(r.y);
    const float e = sqrtf(-2.f * __logf(u1)) * __cosf(6.28318530718f * u2);
    eps[i] = e;
    z[i] = mu[i] + e * __expf(0.5f * lv[i]);
  }
}

DDL_API int ddl_reparam(const float* mu, const float* lv, float* eps, float* z, long long n,
                        unsigned long long seed, unsigned long long offset, hipStream_t s) {
  hipLaunchKernelGGL(reparam_kernel, dim3(grid_for(n, 256)), dim3(256), 0, s, mu, lv, eps, z, n, seed,
                     offset);
  return (int)hipGetLastError();
}

DDL_API int ddl_gemm_f32_args_size() { return (int)sizeof(GemmF32Args); }
