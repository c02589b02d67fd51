// Reference-precision (fp32) BatchNorm / global-pool / classifier-head passes for NHWC fp32
// activations [G][M][C] (G = co-resident clients), the companions of conv_f32.hip.
//
// Every reduction here is DETERMINISTIC: partial sums go to per-block slots [G][S][2][C] with
// plain stores (no float atomics, no zero-fill launch) and are folded in a fixed order (double
// accumulation) by the consumer. Together with conv_f32.hip this makes a training step of the
// fp32 path bitwise reproducible run to run (the reference pins cudnn.deterministic,
// lab/tutorial_1a/hfl_complete.py:17).
//
//   bnf_finalize  : stats slots -> (scale, shift, mean, rstd) + running statistics (1 or 2 BNs)
//   bnf_apply     : y = act(x*scale + shift [+ r*rscale + rshift | + r])       (one HBM pass)
//   bnf_reduce    : s0 = sum dy_m, s1 = sum dy_m * xhat  -> slots      (dy_m = dy * (ymask > 0))
//   bnf_backward  : [reduce] -> fold (d(beta) += s0, d(gamma) += s1, dx coefficients) -> apply
//   bnf_backward2 : two BNs sharing dy (block output BN + projection-shortcut BN)
//   bnf_stats     : standalone forward statistics -> slots
//   avgpoolf_bwd_bn / headf_train : the ResNet classifier head (pool -> FC -> softmax CE -> FC
//                   grads -> pool backward masked by the last block's ReLU + that BN's reduce)
//
// Streaming layout: a 256-thread block covers RPI = 256 / (C/4) rows, each thread a fixed
// 4-channel float4 chunk; blockIdx.y = client group.
//
// Reference parity: nn.BatchNorm2d training semantics (momentum 0.1, eps 1e-5, unbiased running
// variance) of the north-star ResNets; nn.AdaptiveAvgPool2d + nn.Linear + F.cross_entropy.
#include "ddl_common.h"

struct BNFArgs {  // BNArgs (batchnorm.hip) + tile_rows; stats = [G][stripes][2][C] slots
  const float* stats;
  const float* gamma;
  const float* beta;
  float* running_mean;
  float* running_var;
  float* scale;
  float* shift;
  float* mean;
  float* rstd;
  long long gs_param, gs_buf;
  int G, C;
  long long count;
  float eps, momentum;
  int training, stripes;
  int tile_rows;  // > 0: slot i holds (sum, M2 about its own mean) of min(tile_rows, count - i*tile_rows) rows
  int pad_;
};

// Fixed-order fold of S slots of one group: thread (sg, cl) of a FOLD_T-thread block owning 32
// channels sums slots sg, sg+NSG, ... in double (NSG = FOLD_T / 32 slot groups); the NSG partials
// meet in LDS and are added in group order. Totals on sg == 0. (A 1024-thread block keeps 32 slot
// streams in flight per channel: the fold is latency-bound on its few blocks — 2 for C = 64 — and
// ran ~10 us per launch with 8 groups at one client per GPU.)
constexpr int FOLD_T = 1024, NSG = FOLD_T / 32;
__device__ __forceinline__ void slot_fold(const float* __restrict__ base, int S, int C, int c, bool valid,
                                          double* red, double& t0, double& t1) {
  const int sg = threadIdx.x >> 5, cl = threadIdx.x & 31;
  double a0 = 0.0, a1 = 0.0;
  if (valid) {
    int k = sg;
    for (; k + 7 * NSG < S; k += 8 * NSG) {  // 8 slots' loads in flight per thread, added in slot order
      float xs[8], ys[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        xs[j] = base[(long long)(k + j * NSG) * 2 * C + c];
        ys[j] = base[(long long)(k + j * NSG) * 2 * C + C + c];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        a0 += xs[j];
        a1 += ys[j];
      }
    }
    for (; k < S; k += NSG) {
      a0 += base[(long long)k * 2 * C + c];
      a1 += base[(long long)k * 2 * C + C + c];
    }
  }
  red[sg * 64 + cl] = a0;
  red[sg * 64 + 32 + cl] = a1;
  __syncthreads();
  t0 = t1 = 0.0;
  if (sg == 0) {
#pragma unroll 8
    for (int k = 0; k < NSG; ++k) {
      t0 += red[k * 64 + cl];
      t1 += red[k * 64 + 32 + cl];
    }
  }
}

// Chan's parallel merge of per-tile (sum, M2) slots, fixed order, in double, ONE slot pass:
// mean = sum S0 / M, M2 = sum M2_i + (sum S0_i^2 / n_i - (sum S0)^2 / M), n_i = min(rows, M - i * rows)
// (the between-tile term sum n_i (mean_i - mean)^2 expanded: in double its cancellation costs
// ~1e-16 * mean^2 / var relative, where the two-pass form waited out a second round of slot loads).
// red: NSG * 96 doubles.
__device__ __forceinline__ void slot_fold_chan(const float* __restrict__ base, int S, int C, int c, bool valid,
                                               double* red, long long M, int rows, double& mean, double& m2) {
  const int sg = threadIdx.x >> 5, cl = threadIdx.x & 31;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0;
  if (valid) {
    auto term = [&](int k, float s0, float q) {
      a0 += s0;
      a1 += q;
      const long long rem = M - (long long)k * rows;
      const double n = (double)(rem < rows ? rem : rows);
      if (n > 0.0) a2 += (double)s0 * (double)s0 / n;
    };
    int k = sg;
    for (; k + 7 * NSG < S; k += 8 * NSG) {  // 8 slots' loads in flight per thread, added in slot order
      float xs[8], ys[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        xs[j] = base[(long long)(k + j * NSG) * 2 * C + c];
        ys[j] = base[(long long)(k + j * NSG) * 2 * C + C + c];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) term(k + j * NSG, xs[j], ys[j]);
    }
    for (; k < S; k += NSG) term(k, base[(long long)k * 2 * C + c], base[(long long)k * 2 * C + C + c]);
  }
  red[sg * 96 + cl] = a0;
  red[sg * 96 + 32 + cl] = a1;
  red[sg * 96 + 64 + cl] = a2;
  __syncthreads();
  mean = m2 = 0.0;
  if (sg == 0) {
    double t0 = 0.0, t1 = 0.0, t2 = 0.0;
    for (int j = 0; j < NSG; ++j) {
      t0 += red[j * 96 + cl];
      t1 += red[j * 96 + 32 + cl];
      t2 += red[j * 96 + 64 + cl];
    }
    mean = t0 / (double)M;
    m2 = t1 + (t2 - t0 * t0 / (double)M);
  }
}

__device__ __forceinline__ void bnf_finalize_body(const BNFArgs& a, double* red) {
  const int g = blockIdx.y, c = blockIdx.x * 32 + (threadIdx.x & 31);
  const bool valid = c < a.C;
  const bool lead = (threadIdx.x >> 5) == 0 && valid;
  const long long po = (long long)g * a.gs_param + c, o = (long long)g * a.gs_buf + c;
  const float ga = (lead && a.gamma) ? a.gamma[po] : 1.f, be = (lead && a.beta) ? a.beta[po] : 0.f;
  const bool rs_io = lead && a.running_mean;
  const float rm0 = rs_io ? a.running_mean[o] : 0.f, rv0 = rs_io ? a.running_var[o] : 0.f;
  float mean, var;
  if (a.training) {
    const double M = (double)a.count;
    double m, v;
    if (a.tile_rows > 0) {
      double m2;
      slot_fold_chan(a.stats + (long long)g * a.stripes * 2 * a.C, a.stripes, a.C, c, valid, red, a.count,
                     a.tile_rows, m, m2);
      if (!lead) return;
      v = m2 / M;
    } else {
      double s1, s2;
      slot_fold(a.stats + (long long)g * a.stripes * 2 * a.C, a.stripes, a.C, c, valid, red, s1, s2);
      if (!lead) return;
      m = s1 / M;
      v = s2 / M - m * m;
    }
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
  const float rs = 1.f / sqrtf(var + a.eps);
  a.scale[i] = ga * rs;
  a.shift[i] = be - mean * ga * rs;
  a.mean[i] = mean;
  a.rstd[i] = rs;
}

__global__ __launch_bounds__(FOLD_T) void bnf_finalize_kernel(BNFArgs a, BNFArgs b) {
  __shared__ double red[NSG * 96];  // slot_fold_chan's three partials (slot_fold uses the first 64)
  bnf_finalize_body(blockIdx.z ? b : a, red);
}

DDL_API int ddl_bnf_finalize(const BNFArgs* a, const BNFArgs* b, hipStream_t s) {
  if (a->training && a->stripes < 1) return (int)hipErrorInvalidValue;
  const int nbn = b ? 2 : 1;
  if (b && (b->G != a->G || (b->training && b->stripes < 1))) return (int)hipErrorInvalidValue;
  const int C = (b && b->C > a->C) ? b->C : a->C;
  hipLaunchKernelGGL(bnf_finalize_kernel, dim3((C + 31) / 32, a->G, nbn), dim3(FOLD_T), 0, s, *a, b ? *b : *a);
  return (int)hipGetLastError();
}
DDL_API int ddl_bnf_args_size() { return (int)sizeof(BNFArgs); }

// Channel tiling of the streaming passes: a 256-thread block covers RPI = 256 / TPR rows of
// TPR = min(C/4, 256) float4 chunks; wider rows (C = 2048: ResNet-50's last stage) loop over
// NCH = C / (4 * TPR) channel chunks of 1024 (each chunk's bytes are disjoint: no extra traffic).
__device__ __host__ __forceinline__ int f_tpr(int C) { return (C >> 2) < 256 ? (C >> 2) : 256; }
static inline bool f_chan_ok(int C) { return C % 4 == 0 && ((C >> 2) <= 256 || (C >> 2) % 256 == 0); }

// blocks per group of a streaming pass
static unsigned fstream_blocks(long long M, int RPI, int G, int rows_per_thread) {
  long long want = (M + (long long)RPI * rows_per_thread - 1) / ((long long)RPI * rows_per_thread);
  long long cap = (2048 + G - 1) / G;
  if (cap < 8) cap = 8;
  if (want > cap) want = cap;
  if (want < 1) want = 1;
  return (unsigned)want;
}

__device__ __forceinline__ float4 ld4(const float* p) { return *(const float4*)p; }
__device__ __forceinline__ float4 fma4(float4 x, float4 a, float4 b) {
  return make_float4(x.x * a.x + b.x, x.y * a.y + b.y, x.z * a.z + b.z, x.w * a.w + b.w);
}
__device__ __forceinline__ float4 act4(float4 v, int act) {
  if (act == 1) return make_float4(fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f));
  if (act == 2 || act == 3) {
    const float sl = act == 2 ? 0.01f : 0.2f;
    return make_float4(v.x > 0.f ? v.x : sl * v.x, v.y > 0.f ? v.y : sl * v.y, v.z > 0.f ? v.z : sl * v.z,
                       v.w > 0.f ? v.w : sl * v.w);
  }
  return v;
}
__device__ __forceinline__ float4 mask4(float4 d, float4 m) {
  return make_float4(m.x > 0.f ? d.x : 0.f, m.y > 0.f ? d.y : 0.f, m.z > 0.f ? d.z : 0.f, m.w > 0.f ? d.w : 0.f);
}

// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void bnf_apply_kernel(
    const float* __restrict__ x, const float* __restrict__ scale, const float* __restrict__ shift,
    const float* __restrict__ r, const float* __restrict__ rscale, const float* __restrict__ rshift,
    float* __restrict__ y, long long M, int C, int act) {
  const int g = blockIdx.y;
  const int TPR = f_tpr(C), RPI = 256 / TPR, NCH = (C >> 2) / TPR;
  const int row = threadIdx.x / TPR;
  if (row >= RPI) return;
  for (int ch = 0; ch < NCH; ++ch) {
  const int cc = threadIdx.x % TPR + ch * TPR;
  const float4 sc = ld4(scale + (long long)g * C + cc * 4), sh = ld4(shift + (long long)g * C + cc * 4);
  float4 rsc = make_float4(1.f, 1.f, 1.f, 1.f), rsh = make_float4(0.f, 0.f, 0.f, 0.f);
  if (rscale) {
    rsc = ld4(rscale + (long long)g * C + cc * 4);
    rsh = ld4(rshift + (long long)g * C + cc * 4);
  }
  const long long base = (long long)g * M * C + cc * 4;
  constexpr int RB = 4;
  const long long stride = (long long)gridDim.x * RPI;
  for (long long p0 = (long long)blockIdx.x * RPI + row; p0 < M; p0 += stride * RB) {
    float4 xv[RB], rv[RB];
#pragma unroll
    for (int b = 0; b < RB; ++b) {
      const long long p = p0 + b * stride;
      const long long e = base + (p < M ? p : p0) * C;
      xv[b] = ld4(x + e);
      if (r) rv[b] = ld4(r + e);
    }
#pragma unroll
    for (int b = 0; b < RB; ++b) {
      const long long p = p0 + b * stride;
      if (p >= M) break;
      float4 v = fma4(xv[b], sc, sh);
      if (r) {
        const float4 t = fma4(rv[b], rsc, rsh);
        v.x += t.x; v.y += t.y; v.z += t.z; v.w += t.w;
      }
      *(float4*)(y + base + p * C) = act4(v, act);
    }
  }
  }
}

DDL_API int ddl_bnf_apply(const float* x, const float* scale, const float* shift, const float* r,
                          const float* rscale, const float* rshift, float* y, long long per_group, int C, int G,
                          int act, hipStream_t s) {
  if (!f_chan_ok(C) || per_group % C) return (int)hipErrorInvalidValue;
  const long long M = per_group / C;
  const int RPI = 256 / f_tpr(C);
  hipLaunchKernelGGL(bnf_apply_kernel, dim3(fstream_blocks(M, RPI, G, 4), G), dim3(256), 0, s, x, scale, shift, r,
                     rscale, rshift, y, M, C, act);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Reduce: s0 = sum dy_m, s1 = sum dy_m * (x - mean) * rstd over this block's rows -> slot
// blockIdx.x of part [G][gridDim.x][2][C]. MODE 0: BN backward reduce; MODE 1: forward statistics
// of x (s0 = sum x, s1 = sum x^2; dy / mean / rstd unused).
template <int MODE>
__global__ __launch_bounds__(256) void bnf_reduce_kernel(
    const float* __restrict__ dy, const float* __restrict__ ymask, const float* __restrict__ x,
    const float* __restrict__ mean, const float* __restrict__ rstd, float* __restrict__ part, long long M, int C) {
  __shared__ float red[256 * 8];
  const int g = blockIdx.y;
  const int TPR = f_tpr(C), RPI = 256 / TPR, NCH = (C >> 2) / TPR;
  const int tid = threadIdx.x, row = tid / TPR;
  for (int ch = 0; ch < NCH; ++ch) {
  const int cc = tid % TPR + ch * TPR;
  if (ch) __syncthreads();  // the previous chunk's LDS fold is done
  float4 s0 = make_float4(0.f, 0.f, 0.f, 0.f), s1 = s0;
  if (row < RPI) {
    float4 m4 = s0, r4 = s0;
    if (MODE == 0) {
      m4 = ld4(mean + (long long)g * C + cc * 4);
      r4 = ld4(rstd + (long long)g * C + cc * 4);
    }
    const long long base = (long long)g * M * C + cc * 4;
    const long long stride = (long long)gridDim.x * RPI;
    constexpr int U = 4;
    for (long long p0 = (long long)blockIdx.x * RPI + row; p0 < M; p0 += stride * U) {
      float4 rd[U], rx[U], rm[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long p = p0 + u * stride;
        if (p < M) {
          const long long e = base + p * C;
          rx[u] = ld4(x + e);
          if (MODE == 0) {
            rd[u] = ld4(dy + e);
            if (ymask) rm[u] = ld4(ymask + e);
          }
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (p0 + u * stride >= M) break;
        if (MODE == 0) {
          float4 d = rd[u];
          if (ymask) d = mask4(d, rm[u]);
          s0.x += d.x; s0.y += d.y; s0.z += d.z; s0.w += d.w;
          s1.x += d.x * ((rx[u].x - m4.x) * r4.x);
          s1.y += d.y * ((rx[u].y - m4.y) * r4.y);
          s1.z += d.z * ((rx[u].z - m4.z) * r4.z);
          s1.w += d.w * ((rx[u].w - m4.w) * r4.w);
        } else {
          const float4 v = rx[u];
          s0.x += v.x; s0.y += v.y; s0.z += v.z; s0.w += v.w;
          s1.x += v.x * v.x; s1.y += v.y * v.y; s1.z += v.z * v.z; s1.w += v.w * v.w;
        }
      }
    }
  }
  *(float4*)(red + tid * 8) = s0;
  *(float4*)(red + tid * 8 + 4) = s1;
  __syncthreads();
  if (row == 0) {
    for (int r = 1; r < RPI; ++r) {
      const float* o = red + (r * TPR + tid % TPR) * 8;
      s0.x += o[0]; s0.y += o[1]; s0.z += o[2]; s0.w += o[3];
      s1.x += o[4]; s1.y += o[5]; s1.z += o[6]; s1.w += o[7];
    }
    float* pg = part + ((long long)g * gridDim.x + blockIdx.x) * 2 * C + cc * 4;
    *(float4*)pg = s0;
    *(float4*)(pg + C) = s1;
  }
  }
}

// slots (= blocks per group) of a reduce pass over M rows: a pure function of the shape
DDL_API int ddl_bnf_reduce_slots(long long M, int C, int G) {
  if (!f_chan_ok(C)) return -1;
  const int RPI = 256 / f_tpr(C);
  long long want = (M + (long long)RPI * 16 - 1) / ((long long)RPI * 16);
  long long cap = (2048 + G - 1) / G;
  if (cap > 256) cap = 256;
  if (want > cap) want = cap;
  return (int)(want < 1 ? 1 : want);
}

// part: [G][S][2][C] with S = ddl_bnf_reduce_slots(M, C, G) (written, not accumulated)
DDL_API int ddl_bnf_reduce(const float* dy, const float* ymask, const float* x, const float* mean, const float* rstd,
                           float* part, long long M, int C, int G, hipStream_t s) {
  const int S = ddl_bnf_reduce_slots(M, C, G);
  if (S < 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(bnf_reduce_kernel<0>, dim3(S, G), dim3(256), 0, s, dy, ymask, x, mean, rstd, part, M, C);
  return (int)hipGetLastError();
}

DDL_API int ddl_bnf_stats(const float* x, float* stats, long long M, int C, int G, hipStream_t s) {
  const int S = ddl_bnf_reduce_slots(M, C, G);
  if (S < 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(bnf_reduce_kernel<1>, dim3(S, G), dim3(256), 0, s, (const float*)nullptr,
                     (const float*)nullptr, x, (const float*)nullptr, (const float*)nullptr, stats, M, C);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// fold: d(beta) += s0, d(gamma) += s1, coef = (A, B, Cc) with dx = A*dy_m + B*x + Cc
struct BNFBwdArgs {  // same layout as BNBwdArgs (batchnorm.hip) + the slot count
  const float* x;
  const float* mean;
  const float* rstd;
  const float* gamma;
  float* dgamma;
  float* dbeta;
  const float* part;
  float* coef;
  float* dx;
  long long gs_param;
  int slots;
  int pad0_;
  double* fold_ws;  // two-level fold: per-slot-block partials [S / FB_SB][2][C] (null: one-level fold)
  int* tickets;     // two-level fold in ONE launch: zeroed arrival counters [2][G][C/32] (null: two launches)
};

__device__ __forceinline__ void bnf_fold_body(const BNFBwdArgs& t, long long M, int C, double* red) {
  const int g = blockIdx.y, c = blockIdx.x * 32 + (threadIdx.x & 31);
  const bool valid = c < C;
  const bool lead = (threadIdx.x >> 5) == 0 && valid;
  const int i = g * C + c;
  const long long po = (long long)g * t.gs_param + c;
  const float mu = lead ? t.mean[i] : 0.f, rs = lead ? t.rstd[i] : 0.f;
  const float ga = (lead && t.gamma) ? t.gamma[po] : 1.f;
  const float db0 = (lead && t.dbeta) ? t.dbeta[po] : 0.f, dg0 = (lead && t.dgamma) ? t.dgamma[po] : 0.f;
  double s0, s1;
  slot_fold(t.part + (long long)g * t.slots * 2 * C, t.slots, C, c, valid, red, s0, s1);
  if (!lead) return;
  if (t.dbeta) t.dbeta[po] = db0 + (float)s0;
  if (t.dgamma) t.dgamma[po] = dg0 + (float)s1;
  const double invM = 1.0 / (double)M;
  const double A = (double)ga * rs;
  const double B = -A * rs * s1 * invM;
  t.coef[(long long)g * 3 * C + c] = (float)A;
  t.coef[(long long)g * 3 * C + C + c] = (float)B;
  t.coef[(long long)g * 3 * C + 2 * C + c] = (float)(-A * s0 * invM - B * mu);
}

__global__ __launch_bounds__(FOLD_T) void bnf_fold_kernel(BNFBwdArgs a, BNFBwdArgs b, long long M, int C) {
  __shared__ double red[NSG * 64];
  bnf_fold_body(blockIdx.z ? b : a, M, C, red);
}

// Two-level fixed-order fold for many slots (the fp32 step at 8 clients: S = 800 per BN). Level 1:
// 256-thread blocks (8 slot streams x 32 channels) each reduce FB_SB consecutive slots, all 2 x 8
// loads of a thread in flight at once, into a double partial per block; level 2 adds the partials in
// block order and derives the coefficients. Both levels are small blocks that fit beside the
// side-stream WGRAD's resident workgroups (the one-level fold's 1024-thread blocks waited for a
// whole CU to drain: ~100 us per fold inside the overlapped backward).
#ifndef BNF_FB_SB
#define BNF_FB_SB 64
#endif
constexpr int FB_SG = 8, FB_SB = BNF_FB_SB;

__global__ __launch_bounds__(256) void bnf_fold_part_kernel(BNFBwdArgs a, BNFBwdArgs b, int C, int nb) {
  const BNFBwdArgs& t = blockIdx.z ? b : a;
  __shared__ double red[FB_SG * 64];
  const int g = blockIdx.y, cg = blockIdx.x / nb, sb = blockIdx.x - cg * nb;
  const int sg = threadIdx.x >> 5, cl = threadIdx.x & 31, c = cg * 32 + cl;
  const int S = t.slots;
  const float* base = t.part + (long long)g * S * 2 * C;
  constexpr int PER = FB_SB / FB_SG;
  float x0[PER], x1[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int k = sb * FB_SB + sg + j * FB_SG;
    const bool ok = c < C && k < S;
    x0[j] = ok ? base[(long long)k * 2 * C + c] : 0.f;
    x1[j] = ok ? base[(long long)k * 2 * C + C + c] : 0.f;
  }
  double a0 = 0.0, a1 = 0.0;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    a0 += x0[j];
    a1 += x1[j];
  }
  red[sg * 64 + cl] = a0;
  red[sg * 64 + 32 + cl] = a1;
  __syncthreads();
  if (sg == 0 && c < C) {
    double t0 = 0.0, t1 = 0.0;
#pragma unroll
    for (int k = 0; k < FB_SG; ++k) {
      t0 += red[k * 64 + cl];
      t1 += red[k * 64 + 32 + cl];
    }
    double* w = t.fold_ws + ((long long)g * nb + sb) * 2 * C;
    w[c] = t0;
    w[C + c] = t1;
  }
}

__global__ __launch_bounds__(256) void bnf_fold_fin_kernel(BNFBwdArgs a, BNFBwdArgs b, long long M, int C, int nb) {
  const BNFBwdArgs& t = blockIdx.z ? b : a;
  const int g = blockIdx.y, c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  double s0 = 0.0, s1 = 0.0;
  const double* w = t.fold_ws + (long long)g * nb * 2 * C;
  int k = 0;
  for (; k + 8 <= nb; k += 8) {  // loads ahead, added in block order (as bnf_fold_one_kernel)
    double y0[8], y1[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      y0[j] = w[(long long)(k + j) * 2 * C + c];
      y1[j] = w[(long long)(k + j) * 2 * C + C + c];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s0 += y0[j];
      s1 += y1[j];
    }
  }
  for (; k < nb; ++k) {
    s0 += w[(long long)k * 2 * C + c];
    s1 += w[(long long)k * 2 * C + C + c];
  }
  const int i = g * C + c;
  const long long po = (long long)g * t.gs_param + c;
  const float mu = t.mean[i], rs = t.rstd[i];
  const float ga = t.gamma ? t.gamma[po] : 1.f;
  if (t.dbeta) t.dbeta[po] = t.dbeta[po] + (float)s0;
  if (t.dgamma) t.dgamma[po] = t.dgamma[po] + (float)s1;
  const double invM = 1.0 / (double)M;
  const double A = (double)ga * rs;
  const double B = -A * rs * s1 * invM;
  t.coef[(long long)g * 3 * C + c] = (float)A;
  t.coef[(long long)g * 3 * C + C + c] = (float)B;
  t.coef[(long long)g * 3 * C + 2 * C + c] = (float)(-A * s0 * invM - B * mu);
}

// The two levels in ONE launch: every level-1 block publishes its double partials write-through
// (relaxed agent-scope atomic stores: sc1, no release fence), drains them, and arrives on its
// (BN, group, channel group) counter; the last block to arrive acquires and folds the partials in
// block order — the sums and coefficients of bnf_fold_fin, bit for bit — then returns the counter
// to zero for the next launch. One launch and one kernel boundary fewer per BN backward.
__global__ __launch_bounds__(256) void bnf_fold_one_kernel(BNFBwdArgs a, BNFBwdArgs b, long long M, int C, int nb) {
  const BNFBwdArgs& t = blockIdx.z ? b : a;
  __shared__ double red[FB_SG * 64];
  __shared__ int is_last;
  const int g = blockIdx.y, cg = blockIdx.x / nb, sb = blockIdx.x - cg * nb;
  const int sg = threadIdx.x >> 5, cl = threadIdx.x & 31, c = cg * 32 + cl;
  const int S = t.slots;
  const float* base = t.part + (long long)g * S * 2 * C;
  constexpr int PER = FB_SB / FB_SG;
  float x0[PER], x1[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int k = sb * FB_SB + sg + j * FB_SG;
    const bool ok = c < C && k < S;
    x0[j] = ok ? base[(long long)k * 2 * C + c] : 0.f;
    x1[j] = ok ? base[(long long)k * 2 * C + C + c] : 0.f;
  }
  double a0 = 0.0, a1 = 0.0;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    a0 += x0[j];
    a1 += x1[j];
  }
  red[sg * 64 + cl] = a0;
  red[sg * 64 + 32 + cl] = a1;
  __syncthreads();
  double* const wsb = t.fold_ws + (long long)g * nb * 2 * C;
  if (sg == 0 && c < C) {
    double t0 = 0.0, t1 = 0.0;
#pragma unroll
    for (int k = 0; k < FB_SG; ++k) {
      t0 += red[k * 64 + cl];
      t1 += red[k * 64 + 32 + cl];
    }
    double* w = wsb + (long long)sb * 2 * C;
    __hip_atomic_store((unsigned long long*)(w + c), __double_as_longlong(t0), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store((unsigned long long*)(w + C + c), __double_as_longlong(t1), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  // Hand-off (cdna_hip_programming.md 'Projection GEMM at M = 256' item 2, the sc1 form): the
  // partials above are agent-scope atomic stores (write-through, no release fence needed), every
  // storing wave drains them before the workgroup's one relaxed agent-scope arrival, and the last
  // arriver acquires (agent fence) before its plain loads. Counters are per device and shared by
  // all folds, so every fold must run on one stream (functional_f32._fold_tickets).
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains before the arrival
  __syncthreads();
  if (threadIdx.x == 0) {
    int* ctr = t.tickets + ((long long)blockIdx.z * gridDim.y + g) * ((C + 31) / 32) + cg;
    const int prev = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    is_last = prev == nb - 1;
    if (is_last) {
      __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (!is_last || sg != 0 || c >= C) return;
  double s0 = 0.0, s1 = 0.0;
  int k = 0;
  for (; k + 8 <= nb; k += 8) {  // 16 loads in flight, added in block order (one at a time they
    double y0[8], y1[8];          // made the last block's fold a chain of load latencies)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      y0[j] = wsb[(long long)(k + j) * 2 * C + c];
      y1[j] = wsb[(long long)(k + j) * 2 * C + C + c];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s0 += y0[j];
      s1 += y1[j];
    }
  }
  for (; k < nb; ++k) {
    s0 += wsb[(long long)k * 2 * C + c];
    s1 += wsb[(long long)k * 2 * C + C + c];
  }
  const int i = g * C + c;
  const long long po = (long long)g * t.gs_param + c;
  const float mu = t.mean[i], rs = t.rstd[i];
  const float ga = t.gamma ? t.gamma[po] : 1.f;
  if (t.dbeta) t.dbeta[po] = t.dbeta[po] + (float)s0;
  if (t.dgamma) t.dgamma[po] = t.dgamma[po] + (float)s1;
  const double invM = 1.0 / (double)M;
  const double A = (double)ga * rs;
  const double B = -A * rs * s1 * invM;
  t.coef[(long long)g * 3 * C + c] = (float)A;
  t.coef[(long long)g * 3 * C + C + c] = (float)B;
  t.coef[(long long)g * 3 * C + 2 * C + c] = (float)(-A * s0 * invM - B * mu);
}

// ints of arrival counters a one-launch fold of up to two BNs with C channels and G groups uses
DDL_API long long ddl_bnf_fold_tickets(int C, int G) { return 2LL * G * ((C + 31) / 32); }

// doubles of fold workspace a BN backward with S slots needs (two-level fold)
DDL_API long long ddl_bnf_fold_ws(int S, int C, int G) {
  const int nb = (S + FB_SB - 1) / FB_SB;
  return (long long)G * nb * 2 * C;
}

__global__ __launch_bounds__(256) void bnf_bwd_apply_kernel(
    const float* __restrict__ dy, const float* __restrict__ ymask, BNFBwdArgs a, BNFBwdArgs b, int two,
    float* __restrict__ dym_out, long long M, int C) {
  const int g = blockIdx.y;
  const int TPR = f_tpr(C), RPI = 256 / TPR, NCH = (C >> 2) / TPR;
  const int row = threadIdx.x / TPR;
  if (row >= RPI) return;
  for (int ch = 0; ch < NCH; ++ch) {
  const int cc = threadIdx.x % TPR + ch * TPR;
  const float* ca = a.coef + (long long)g * 3 * C + cc * 4;
  const float4 Aa = ld4(ca), Ba = ld4(ca + C), Ca = ld4(ca + 2 * C);
  float4 Ab = Aa, Bb = Ba, Cb = Ca;
  if (two) {
    const float* cb = b.coef + (long long)g * 3 * C + cc * 4;
    Ab = ld4(cb); Bb = ld4(cb + C); Cb = ld4(cb + 2 * C);
  }
  const long long base = (long long)g * M * C + cc * 4;
  constexpr int RB = 4;
  const long long stride = (long long)gridDim.x * RPI;
  for (long long p0 = (long long)blockIdx.x * RPI + row; p0 < M; p0 += stride * RB) {
    float4 dv[RB], xa[RB], xb[RB], mv[RB];
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const long long p = p0 + r * stride;
      const long long e = base + (p < M ? p : p0) * C;
      dv[r] = ld4(dy + e);
      xa[r] = ld4(a.x + e);
      if (two) xb[r] = ld4(b.x + e);
      if (ymask) mv[r] = ld4(ymask + e);
    }
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const long long p = p0 + r * stride;
      if (p >= M) break;
      const long long e = base + p * C;
      float4 d = dv[r];
      if (ymask) d = mask4(d, mv[r]);
      if (dym_out) *(float4*)(dym_out + e) = d;
      float4 o;
      o.x = Aa.x * d.x + Ba.x * xa[r].x + Ca.x;
      o.y = Aa.y * d.y + Ba.y * xa[r].y + Ca.y;
      o.z = Aa.z * d.z + Ba.z * xa[r].z + Ca.z;
      o.w = Aa.w * d.w + Ba.w * xa[r].w + Ca.w;
      *(float4*)(a.dx + e) = o;
      if (two) {
        o.x = Ab.x * d.x + Bb.x * xb[r].x + Cb.x;
        o.y = Ab.y * d.y + Bb.y * xb[r].y + Cb.y;
        o.z = Ab.z * d.z + Bb.z * xb[r].z + Cb.z;
        o.w = Ab.w * d.w + Bb.w * xb[r].w + Cb.w;
        *(float4*)(b.dx + e) = o;
      }
    }
  }
  }
}

DDL_API int ddl_bnf_bwd_args_size() { return (int)sizeof(BNFBwdArgs); }

// One BN backward (b == null) or two sharing the already-masked dy. With do_reduce, a's part
// (S = ddl_bnf_reduce_slots slots) is produced here from (dy, ymask, a.x); otherwise every part
// holds `slots` complete partial sums from dy's producer.
DDL_API int ddl_bnf_backward(const float* dy, const float* ymask, const BNFBwdArgs* ap, const BNFBwdArgs* bp,
                             float* dym_out, long long M, int C, int G, int do_reduce, hipStream_t s) {
  if (!f_chan_ok(C)) return (int)hipErrorInvalidValue;
  BNFBwdArgs a = *ap;
  if (do_reduce) {
    a.slots = ddl_bnf_reduce_slots(M, C, G);
    hipLaunchKernelGGL(bnf_reduce_kernel<0>, dim3(a.slots, G), dim3(256), 0, s, dy, ymask, a.x, a.mean, a.rstd,
                       (float*)a.part, M, C);
  }
  if (a.slots < 1 || (bp && bp->slots < 1)) return (int)hipErrorInvalidValue;
  const int two = bp ? 1 : 0;
  const BNFBwdArgs b = bp ? *bp : a;
  if (a.fold_ws && (!two || b.fold_ws)) {
    // one grid for both BNs: nb of the larger; blocks past a BN's own slots add exact zeros
    const int sm = two && b.slots > a.slots ? b.slots : a.slots;
    const int nb = (sm + FB_SB - 1) / FB_SB;
    if (a.tickets) {
      hipLaunchKernelGGL(bnf_fold_one_kernel, dim3((C + 31) / 32 * nb, G, 1 + two), dim3(256), 0, s, a, b, M, C, nb);
    } else {
      hipLaunchKernelGGL(bnf_fold_part_kernel, dim3((C + 31) / 32 * nb, G, 1 + two), dim3(256), 0, s, a, b, C, nb);
      hipLaunchKernelGGL(bnf_fold_fin_kernel, dim3((C + 255) / 256, G, 1 + two), dim3(256), 0, s, a, b, M, C, nb);
    }
  } else {
    hipLaunchKernelGGL(bnf_fold_kernel, dim3((C + 31) / 32, G, 1 + two), dim3(FOLD_T), 0, s, a, b, M, C);
  }
  // coefficient-only mode (a.dx == null): the consumer applies A * dy + B * x + C itself (the halo
  // DGRAD's operand transform, conv_x6h.hip dyb_*), no apply pass
  if (!a.dx && (!two || !b.dx) && !dym_out) return (int)hipGetLastError();
  const int RPI = 256 / f_tpr(C);
  hipLaunchKernelGGL(bnf_bwd_apply_kernel, dim3(fstream_blocks(M, RPI, G, 4), G), dim3(256), 0, s, dy, ymask, a, b,
                     two, dym_out, M, C);
  return (int)hipGetLastError();
}

// out = A * dy + B * x + C per channel (coef [G][3][C]): the BN backward's apply from folded
// coefficients, for a consumer that cannot apply it on the fly
__global__ __launch_bounds__(256) void bnf_coef_apply_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                             const float* __restrict__ coef, float* __restrict__ out,
                                                             long long M, int C) {
  const int g = blockIdx.y, C4 = C >> 2;
  const long long n4 = M * C4;
  const float* cf = coef + (long long)g * 3 * C;
  const long long base = (long long)g * M * C;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < n4; t += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(t % C4) * 4;
    const float4 d = ld4(dy + base + t * 4), v = ld4(x + base + t * 4);
    const float4 A = ld4(cf + c), B = ld4(cf + C + c), K = ld4(cf + 2 * C + c);
    *(float4*)(out + base + t * 4) = make_float4(A.x * d.x + B.x * v.x + K.x, A.y * d.y + B.y * v.y + K.y,
                                                 A.z * d.z + B.z * v.z + K.z, A.w * d.w + B.w * v.w + K.w);
  }
}

DDL_API int ddl_bnf_coef_apply(const float* dy, const float* x, const float* coef, float* out, long long M, int C,
                               int G, hipStream_t s) {
  if (C % 4 || G < 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(bnf_coef_apply_kernel, dim3(grid_for(M * C / 4, 256, 4096), G), dim3(256), 0, s, dy, x, coef, out,
                     M, C);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Global average pool backward fused with the reduce of the BN that produced the pooled input
// x = relu(bn(c) + r): dx = dy / HW * (x > 0); slots as bnf_reduce (rows = N*HW pixels).
__global__ __launch_bounds__(256) void avgpoolf_bwd_bn_kernel(
    const float* __restrict__ dy, const float* __restrict__ x, const float* __restrict__ c,
    const float* __restrict__ mean, const float* __restrict__ rstd, float* __restrict__ dx,
    float* __restrict__ part, int N, int HW, int C) {
  __shared__ float red[256 * 8];
  const int g = blockIdx.y;
  const int TPR = f_tpr(C), RPI = 256 / TPR, NCH = (C >> 2) / TPR;
  const int tid = threadIdx.x, row = tid / TPR;
  const long long M = (long long)N * HW;
  const float inv = 1.f / HW;
  for (int ch = 0; ch < NCH; ++ch) {
  const int cc = tid % TPR + ch * TPR;
  if (ch) __syncthreads();  // the previous chunk's LDS fold is done
  float4 s0 = make_float4(0.f, 0.f, 0.f, 0.f), s1 = s0;
  if (row < RPI) {
    const float4 m4 = ld4(mean + (long long)g * C + cc * 4), r4 = ld4(rstd + (long long)g * C + cc * 4);
    const long long stride = (long long)gridDim.x * RPI;
    constexpr int U = 4;
    for (long long p0 = (long long)blockIdx.x * RPI + row; p0 < M; p0 += stride * U) {
      float4 rd[U], rx[U], rc[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long p = p0 + u * stride;
        if (p < M) {
          const long long e = ((long long)g * M + p) * C + cc * 4;
          rd[u] = ld4(dy + ((long long)g * N + p / HW) * C + cc * 4);
          rx[u] = ld4(x + e);
          rc[u] = ld4(c + e);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long p = p0 + u * stride;
        if (p >= M) break;
        const long long e = ((long long)g * M + p) * C + cc * 4;
        float4 d = make_float4(rd[u].x * inv, rd[u].y * inv, rd[u].z * inv, rd[u].w * inv);
        d = mask4(d, rx[u]);
        s0.x += d.x; s0.y += d.y; s0.z += d.z; s0.w += d.w;
        s1.x += d.x * ((rc[u].x - m4.x) * r4.x);
        s1.y += d.y * ((rc[u].y - m4.y) * r4.y);
        s1.z += d.z * ((rc[u].z - m4.z) * r4.z);
        s1.w += d.w * ((rc[u].w - m4.w) * r4.w);
        *(float4*)(dx + e) = d;
      }
    }
  }
  *(float4*)(red + tid * 8) = s0;
  *(float4*)(red + tid * 8 + 4) = s1;
  __syncthreads();
  if (row == 0) {
    for (int r = 1; r < RPI; ++r) {
      const float* o = red + (r * TPR + tid % TPR) * 8;
      s0.x += o[0]; s0.y += o[1]; s0.z += o[2]; s0.w += o[3];
      s1.x += o[4]; s1.y += o[5]; s1.z += o[6]; s1.w += o[7];
    }
    float* pg = part + ((long long)g * gridDim.x + blockIdx.x) * 2 * C + cc * 4;
    *(float4*)pg = s0;
    *(float4*)(pg + C) = s1;
  }
  }
}

// part: [G][S][2][C], S = ddl_bnf_reduce_slots(N * HW, C, G)
DDL_API int ddl_avgpoolf_bwd_bn(const float* dy, const float* x, const float* c, const float* mean, const float* rstd,
                                float* dx, float* part, int G, int N, int HW, int C, hipStream_t s) {
  const int S = ddl_bnf_reduce_slots((long long)N * HW, C, G);
  if (S < 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(avgpoolf_bwd_bn_kernel, dim3(S, G), dim3(256), 0, s, dy, x, c, mean, rstd, dx, part, N, HW, C);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Classifier head, fp32 and deterministic, in two launches:
//   headf_train_kernel : one workgroup per sample: pool x -> logits (W rows staged in LDS) ->
//                        softmax CE (per-sample loss / hit to scratch) -> d logits -> d pooled ->
//                        dx (masked by x > 0 with BN fusion; that BN's reduce into slot n)
//   headf_wgrad_kernel : dW[k][c] += sum_n dl[n][k] pooled[n][c] (n in order), db, and the
//                        group's loss / correct count (sums in sample order: no atomics)
struct HeadFArgs {
  const float* x;      // [G][N][HW][C]
  const float* w;      // group g at g * w_gs: [Kp][C] fp32 (the Linear's master weight)
  const float* b;      // [Kp] fp32 at g * b_gs (null: no bias)
  const int* labels;   // [G][N]
  float* loss;         // [G] = scale * sum of the rows' CE
  int* correct;        // [G] = #(argmax == label) (null: off)
  float* dw;           // [Kp][C] at g * dw_gs, accumulated
  float* db;           // [Kp] at g * db_gs, accumulated (null: no bias)
  float* dx;           // [G][N][HW][C]
  const float* c;      // BN fusion (null: plain pool backward): the BN's input [G][N][HW][C]
  const float* mean;   // [G][C]
  const float* rstd;   // [G][C]
  float* part;         // [G][N][2][C]: slot n = (sum dx, sum dx * (c - mean) * rstd) of sample n
  float* pooled;       // scratch [G][N][C]
  float* dlog;         // scratch [G][N][64]
  float* row_loss;     // scratch [G][N]
  int* row_hit;        // scratch [G][N]
  long long w_gs, b_gs, dw_gs, db_gs;
  int G, N, HW, C, ncls;
  float scale;
};

__global__ __launch_bounds__(256) void headf_train_kernel(HeadFArgs a) {
  extern __shared__ float hsm[];
  const int C = a.C, TPR = C / 4, RP = 256 / TPR, HW = a.HW, g = blockIdx.y, n = blockIdx.x;
  float* pooled = hsm;         // [C]
  float* dp = pooled + C;      // [C] d pooled / HW
  float* zl = dp + C;          // [64] logits, then d logits
  float* rb = zl + 64;         // [2][RP][C] row partials (RP * C == 1024)
  float* wl = rb + 2048;       // [ncls][C]
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, cc = tid % TPR, row = tid / TPR;
  const float inv = 1.f / HW;
  const long long rowg = (long long)g * a.N + n;
  const float* wg = a.w + g * a.w_gs;
  const bool bn = a.c != nullptr;
  const long long base = rowg * HW * C + cc * 4;
  for (int t = tid; t < a.ncls * TPR; t += 256) *(float4*)(wl + t * 4) = ld4(wg + t * 4);
  const int y = a.labels[rowg];
  const float bias = (a.b && lane < a.ncls) ? a.b[g * a.b_gs + lane] : 0.f;
  // 1. pool (pixels in order per thread, then the RP row partials in order)
  {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (row < RP)
      for (int p = row; p < HW; p += RP) {
        const float4 v = ld4(a.x + base + (long long)p * C);
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
      }
    if (row < RP) *(float4*)(rb + row * C + cc * 4) = acc;
  }
  __syncthreads();
  for (int t = tid; t < C; t += 256) {
    float v = 0.f;
    for (int r = 0; r < RP; ++r) v += rb[r * C + t];
    pooled[t] = v * inv;
  }
  __syncthreads();
  // 2. logits: one wave per class, lanes over channels (fixed shuffle tree)
  for (int k = wv; k < a.ncls; k += 4) {
    float acc = 0.f;
    for (int c = lane; c < C; c += 64) acc += pooled[c] * wl[k * C + c];
    acc = wave_sum(acc);
    if (lane == 0) zl[k] = acc;
  }
  __syncthreads();
  // 3. softmax CE on wave 0, one lane per class
  if (wv == 0) {
    const bool on = lane < a.ncls;
    const float z = on ? zl[lane] + bias : -INFINITY;
    float mx = z;
    int am = on ? lane : 0x7fffffff;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {  // argmax, first max wins (torch.argmax)
      const float om = __shfl_xor(mx, o, 64);
      const int oa = __shfl_xor(am, o, 64);
      if (om > mx || (om == mx && oa < am)) { mx = om; am = oa; }
    }
    const float e = on ? expf(z - mx) : 0.f;
    const float lse = mx + logf(wave_sum(e));
    const float zy = __shfl(z, y, 64);
    const float d = on ? a.scale * (expf(z - lse) - (lane == y ? 1.f : 0.f)) : 0.f;
    zl[lane] = d;
    a.dlog[rowg * 64 + lane] = d;
    if (lane == 0) {
      a.row_loss[rowg] = (lse - zy) * a.scale;
      a.row_hit[rowg] = am == y ? 1 : 0;
    }
  }
  for (int t = tid; t < C; t += 256) a.pooled[rowg * C + t] = pooled[t];
  __syncthreads();
  // 4. d pooled = dl . W / HW
  for (int c = tid; c < C; c += 256) {
    float acc = 0.f;
    for (int k = 0; k < a.ncls; ++k) acc += zl[k] * wl[k * C + c];
    dp[c] = acc * inv;
  }
  __syncthreads();
  // 5. pool backward (+ the BN's ReLU mask and its reduce for slot n)
  if (row >= RP) return;
  const float4 d0 = ld4(dp + cc * 4);
  float4 s0 = make_float4(0.f, 0.f, 0.f, 0.f), s1 = s0, m4 = s0, r4 = s0;
  if (bn) {
    m4 = ld4(a.mean + (long long)g * C + cc * 4);
    r4 = ld4(a.rstd + (long long)g * C + cc * 4);
  }
  for (int p = row; p < HW; p += RP) {
    const long long e = base + (long long)p * C;
    float4 d = d0;
    if (bn) {
      const float4 xv = ld4(a.x + e), cv = ld4(a.c + e);
      d = mask4(d, xv);
      s0.x += d.x; s0.y += d.y; s0.z += d.z; s0.w += d.w;
      s1.x += d.x * ((cv.x - m4.x) * r4.x);
      s1.y += d.y * ((cv.y - m4.y) * r4.y);
      s1.z += d.z * ((cv.z - m4.z) * r4.z);
      s1.w += d.w * ((cv.w - m4.w) * r4.w);
    }
    *(float4*)(a.dx + e) = d;
  }
  if (!bn) return;
  __syncthreads();  // every thread with row < RP reaches this (rows >= RP returned above: RP * TPR == 256)
  *(float4*)(rb + row * C + cc * 4) = s0;
  *(float4*)(rb + 1024 + row * C + cc * 4) = s1;
  __syncthreads();
  if (row == 0) {
    for (int r = 1; r < RP; ++r) {
      const float4 o0 = ld4(rb + r * C + cc * 4), o1 = ld4(rb + 1024 + r * C + cc * 4);
      s0.x += o0.x; s0.y += o0.y; s0.z += o0.z; s0.w += o0.w;
      s1.x += o1.x; s1.y += o1.y; s1.z += o1.z; s1.w += o1.w;
    }
    float* pg = a.part + (rowg * 2) * C + cc * 4;
    *(float4*)pg = s0;
    *(float4*)(pg + C) = s1;
  }
}

// grid (C / 64, ceil(ncls / 4), G): a wave per (class, 64 channels). Sample sums in sample order
// with 16 samples' loads in flight (one at a time, the 100-sample loops waited ~60 us on latency).
__global__ __launch_bounds__(256) void headf_wgrad_kernel(HeadFArgs a) {
  const int g = blockIdx.z, tid = threadIdx.x;
  const int c = blockIdx.x * 64 + (tid & 63), k = blockIdx.y * 4 + (tid >> 6);
  const float* pl = a.pooled + (long long)g * a.N * a.C;
  const float* dl = a.dlog + (long long)g * a.N * 64;
  const int N = a.N;
  if (blockIdx.x == 0 && blockIdx.y == 0 && tid < 64) {
    if (a.db && tid < a.ncls) {
      float s = 0.f;
      int n = 0;
      for (; n + 16 <= N; n += 16) {
        float v[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = dl[(n + j) * 64 + tid];
#pragma unroll
        for (int j = 0; j < 16; ++j) s += v[j];
      }
      for (; n < N; ++n) s += dl[n * 64 + tid];
      a.db[g * a.db_gs + tid] += s;
    }
    if (tid == 0) {
      float l = 0.f;
      int h = 0;
      int n = 0;
      const float* rl = a.row_loss + (long long)g * N;
      const int* rh = a.row_hit + (long long)g * N;
      for (; n + 16 <= N; n += 16) {
        float v[16];
        int hv[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) { v[j] = rl[n + j]; hv[j] = rh[n + j]; }
#pragma unroll
        for (int j = 0; j < 16; ++j) { l += v[j]; h += hv[j]; }
      }
      for (; n < N; ++n) { l += rl[n]; h += rh[n]; }
      a.loss[g] = l;
      if (a.correct) a.correct[g] = h;
    }
  }
  if (c >= a.C || k >= a.ncls) return;
  float acc = 0.f;
  int n = 0;
  for (; n + 16 <= N; n += 16) {
    float d[16], x[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      d[j] = dl[(n + j) * 64 + k];
      x[j] = pl[(long long)(n + j) * a.C + c];
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) acc += d[j] * x[j];
  }
  for (; n < N; ++n) acc += dl[n * 64 + k] * pl[(long long)n * a.C + c];
  a.dw[g * a.dw_gs + c + (long long)k * a.C] += acc;
}

DDL_API int ddl_headf_args_size() { return (int)sizeof(HeadFArgs); }

DDL_API int ddl_headf_train(const HeadFArgs* ap, hipStream_t s) {
  const HeadFArgs& a = *ap;
  if (a.C % 4 || a.C / 4 > 256 || 256 % (a.C / 4) || a.ncls < 1 || a.ncls > 64 || a.N < 1 || a.G < 1 ||
      a.HW < 1 || !a.pooled || !a.dlog || !a.row_loss || !a.row_hit)
    return (int)hipErrorInvalidValue;
  const int RP = 256 / (a.C / 4);
  if (RP * a.C > 1024) return (int)hipErrorInvalidValue;
  const size_t lds = (size_t)(2 * a.C + 64 + 2048 + a.ncls * a.C) * 4;
  if (lds > 64 * 1024) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(headf_train_kernel, dim3(a.N, a.G), dim3(256), lds, s, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(headf_wgrad_kernel, dim3((a.C + 63) / 64, (a.ncls + 3) / 4, a.G), dim3(256), 0, s, a);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Deterministic per-channel column sum (bias gradients): out[g][c] (+ g * gs) += sum_m x[g][m][c]
// via per-block slots (bnf_reduce_kernel<1>) and a fixed-order fold — the fp32 twin of
// nn_ops.hip's atomic channel_sum.
__global__ __launch_bounds__(FOLD_T) void bnf_colsum_fold_kernel(const float* __restrict__ part, int S, float* out,
                                                                 long long gs, int C) {
  __shared__ double red[NSG * 64];
  const int g = blockIdx.y, c = blockIdx.x * 32 + (threadIdx.x & 31);
  const bool valid = c < C;
  double s0, s1;
  slot_fold(part + (long long)g * S * 2 * C, S, C, c, valid, red, s0, s1);
  if ((threadIdx.x >> 5) == 0 && valid) out[(long long)g * gs + c] += (float)s0;
}

// part: scratch [G][S][2][C], S = ddl_bnf_reduce_slots(M, C, G)
DDL_API int ddl_bnf_channel_sum(const float* x, float* out, long long gs, float* part, long long M, int C, int G,
                                hipStream_t s) {
  const int S = ddl_bnf_reduce_slots(M, C, G);
  if (S < 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(bnf_reduce_kernel<1>, dim3(S, G), dim3(256), 0, s, (const float*)nullptr,
                     (const float*)nullptr, x, (const float*)nullptr, (const float*)nullptr, part, M, C);
  hipLaunchKernelGGL(bnf_colsum_fold_kernel, dim3((C + 31) / 32, G), dim3(FOLD_T), 0, s, (const float*)part, S, out,
                     gs, C);
  return (int)hipGetLastError();
}
