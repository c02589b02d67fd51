// Implicit-GEMM convolution on CDNA4 MFMA (v_mfma_f32_16x16x32_bf16), NHWC bf16, fp32 accumulate.
//
// One templated kernel family covers the three products of a conv layer (and of a Linear layer,
// which is the R=S=H=W=1 special case):
//
//   FWD   : y [q=(n,p,q)][p=k]         = sum_{(r,s,c)}  W[k][(r,s,c)]     * X[pix(q,r,s)][c]
//   DGRAD : dx[q=(n,h,w)][p=c]         = sum_{(r,s,k)}  W[k][(r,s,c)]     * dY[pix'(q,r,s)][k]
//   WGRAD : dW[p=k][q=(r,s,c)]        += sum_{(n,p,q)}  dY[(n,p,q)][k]    * X[pix(n,p,q,r,s)][c]
//
// Every mode is written as D[p][q] = sum_k Pop[p][k] * Qop[q][k] with the MFMA A operand = Pop,
// B operand = Qop, so the accumulator lane layout (lane holds 4 consecutive p for one q) gives
// 8-byte contiguous NHWC stores in FWD/DGRAD and 64-byte row segments for the fp32 WGRAD atomics.
//
// Operands are staged global -> registers -> LDS (register staging: the implicit-GEMM gathers
// are predicated / zero-filled per 16-byte chunk, which an LDS-DMA cannot express) into a
// double-buffered LDS ring with one barrier per K-step. Two LDS images are used:
//   * K-major  ([BK/32][rows][32] bf16, 16-B chunk XOR swizzle, fragment = one ds_read_b128)
//     for operands whose reduction index is memory-contiguous (weights / activations in FWD,
//     dY in DGRAD);
//   * MN-major ([BK][cols] bf16, 16-B chunk XOR swizzle, fragment = two ds_read_b64_tr_b16)
//     for operands whose *output* index is contiguous (W in DGRAD, dY and X in WGRAD). The
//     gfx950 transpose read turns them into K-contiguous MFMA fragments with no extra pass.
// Both swizzles are conflict-free for the fragment reads (derivation in docs/KERNELS.md).
//
// Each workgroup is 4 waves (2x2) computing a BP x BQ tile; blockIdx.z = client group,
// blockIdx.y = split-K slice (WGRAD), blockIdx.x = tile id remapped XCD-aware.
//
// Reference parity: replaces the stock nn.Conv2d / nn.Linear calls of MnistCnn
// (reference lab/tutorial_1a/hfl_complete.py:43-61) and the ResNet convs of the
// north-star configs.
#include "ddl_common.h"

struct ConvArgs {
  const void* x;         // [G][N][H][W][C] bf16
  const void* w;         // [G][K][R][S][C] bf16
  const void* dy;        // [G][N][P][Q][K] bf16
  void* out;             // FWD y bf16 | DGRAD dx bf16 | WGRAD dw fp32
  float* stats;          // FWD: per-channel [sum(K), sumsq(K)] fp32 accumulators (optional)
  const float* bias;     // FWD: [K] fp32 (optional)
  const void* residual;  // DGRAD: bf16 added to dx (optional), same layout as out
  const void* mask;      // DGRAD: dx *= (mask > 0) (optional), same layout as out
  long long x_gs, w_gs, dy_gs, out_gs, bias_gs, stats_gs;
  int G, N, H, W, C, K, R, S, P, Q, stride, pad;
  int relu, accumulate, split_k, reserved;
};

enum { MODE_FWD = 0, MODE_DGRAD = 1, MODE_WGRAD = 2 };

__device__ __forceinline__ int km_swz(int row) { return (4 - ((row >> 2) & 3)) & 3; }
template <int COLS>
__device__ __forceinline__ int mn_swz(int k) {
  if constexpr (COLS >= 128)
    return 2 * ((k & 3) | (((k >> 3) & 1) << 2));
  else
    return 2 * (((k >> 1) & 1) | (((k >> 3) & 1) << 1));
}
template <int ROWS>
__device__ __forceinline__ int km_off(int row, int kc) {
  return (kc >> 2) * ROWS * 64 + row * 64 + (((kc & 3) ^ km_swz(row)) << 4);
}
template <int COLS>
__device__ __forceinline__ int mn_off(int krow, int cc) {
  return krow * COLS * 2 + ((cc ^ mn_swz<COLS>(krow)) << 4);
}

typedef __attribute__((address_space(3))) s4v lds_s4v;

template <int ROWS>
__device__ __forceinline__ s8v km_frag(const char* lds, int rb, int u, int lane) {
  const int row = rb + (lane & 15);
  const int off = u * ROWS * 64 + row * 64 + (((lane >> 4) ^ km_swz(row)) << 4);
  return *(const s8v*)(lds + off);
}
template <int COLS>
__device__ __forceinline__ s8v mn_frag(const char* lds, int cb, int u, int lane) {
  const int g = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
  const int col = cb + 4 * p4;
  const int cc = col >> 3, half = (col >> 2) & 1;
  const int k1 = u * 32 + 8 * g + q4, k2 = k1 + 4;
  const char* a1 = lds + k1 * COLS * 2 + ((cc ^ mn_swz<COLS>(k1)) << 4) + half * 8;
  const char* a2 = lds + k2 * COLS * 2 + ((cc ^ mn_swz<COLS>(k2)) << 4) + half * 8;
  s4v r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)a1);
  s4v r2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)a2);
  s8v r;
  r[0] = r1[0]; r[1] = r1[1]; r[2] = r1[2]; r[3] = r1[3];
  r[4] = r2[0]; r[5] = r2[1]; r[6] = r2[2]; r[7] = r2[3];
  return r;
}

__device__ __forceinline__ i4v ld16(const bf16_t* p) { return *(const i4v*)p; }
__device__ __forceinline__ i4v zero16() { i4v z = {0, 0, 0, 0}; return z; }

template <int MODE, int BP, int BQ, int BK>
__global__ __launch_bounds__(256) void conv_igemm_kernel(ConvArgs a) {
  constexpr int P_BYTES = BP * BK * 2, Q_BYTES = BQ * BK * 2, STAGE = P_BYTES + Q_BYTES;
  constexpr int WP = BP / 2, WQ = BQ / 2, TP = WP / 16, TQ = WQ / 16;
  // operand image kinds
  constexpr bool P_KMAJOR = (MODE == MODE_FWD);
  constexpr bool Q_KMAJOR = (MODE != MODE_WGRAD);
  // load partitioning
  constexpr int KCPR = BK / 8;                        // 16B chunks per K-major row
  constexpr int P_NL = P_KMAJOR ? BP * KCPR / 256 : BK * (BP / 8) / 256;
  constexpr int Q_NL = Q_KMAJOR ? BQ * KCPR / 256 : BK * (BQ / 8) / 256;
  static_assert(P_NL >= 1 && Q_NL >= 1, "tile too small for 256 threads");

  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wp = wid >> 1, wq = wid & 1;
  const int g = blockIdx.z;
  const int H = a.H, W = a.W, C = a.C, K = a.K, R = a.R, S = a.S, P = a.P, Q = a.Q;
  const int st = a.stride, pd = a.pad;
  const int RSC = R * S * C;

  int Pd, Qd;
  long long Kr;
  if constexpr (MODE == MODE_FWD) { Pd = K; Qd = a.N * P * Q; Kr = RSC; }
  else if constexpr (MODE == MODE_DGRAD) { Pd = C; Qd = a.N * H * W; Kr = (long long)R * S * K; }
  else { Pd = K; Qd = RSC; Kr = (long long)a.N * P * Q; }

  const int ntp = (Pd + BP - 1) / BP;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int p0 = (tile % ntp) * BP, q0 = (tile / ntp) * BQ;
  const int nk_total = (int)((Kr + BK - 1) / BK);
  const int per = (nk_total + gridDim.y - 1) / gridDim.y;
  const int kt0 = blockIdx.y * per;
  const int kt1 = min(nk_total, kt0 + per);
  if (kt0 >= kt1) return;

  const bf16_t* X = (const bf16_t*)a.x + (long long)g * a.x_gs;
  const bf16_t* Wt = (const bf16_t*)a.w + (long long)g * a.w_gs;
  const bf16_t* DY = (const bf16_t*)a.dy + (long long)g * a.dy_gs;

  // ---------------- per-thread loader state ----------------
  // K-major loaders: fixed chunk column kc, rows r_i = tid/KCPR + i*(256/KCPR)
  const int kc = tid % KCPR;
  const int krow0 = tid / KCPR;
  constexpr int KRSTEP = 256 / KCPR;
  // Q K-major gather precompute (FWD: X rows = output pixels; DGRAD: dY rows = input pixels)
  int qb[Q_KMAJOR ? Q_NL : 1], qh[Q_KMAJOR ? Q_NL : 1], qw[Q_KMAJOR ? Q_NL : 1];
  // MN-major loaders: fixed column chunk cc, rows k_i = tid/CPR + i*(256/CPR)
  constexpr int P_CPR = BP / 8, Q_CPR = BQ / 8;
  const int p_cc = tid % P_CPR, p_kr0 = tid / P_CPR;
  const int q_cc = tid % Q_CPR, q_kr0 = tid / Q_CPR;
  // WGRAD X-gather column precompute
  int wg_r = 0, wg_s = 0, wg_c = 0;
  bool wg_cvalid = false;

  if constexpr (Q_KMAJOR) {
#pragma unroll
    for (int i = 0; i < Q_NL; ++i) {
      const int qq = q0 + krow0 + i * KRSTEP;
      if (qq < Qd) {
        if constexpr (MODE == MODE_FWD) {
          const int n = qq / (P * Q), rem = qq - n * (P * Q);
          const int op = rem / Q, oq = rem - op * Q;
          qb[i] = n * H * W;
          qh[i] = op * st - pd;
          qw[i] = oq * st - pd;
        } else {
          const int n = qq / (H * W), rem = qq - n * (H * W);
          const int h = rem / W, w = rem - h * W;
          qb[i] = n * P * Q;
          qh[i] = h + pd;
          qw[i] = w + pd;
        }
      } else {
        qb[i] = 0;
        qh[i] = -(1 << 28);
        qw[i] = -(1 << 28);
      }
    }
  }
  if constexpr (MODE == MODE_WGRAD) {
    const int col = q0 + q_cc * 8;
    wg_cvalid = col < Qd;
    const int rs = col / C;
    wg_c = col - rs * C;
    wg_r = rs / S;
    wg_s = rs - wg_r * S;
  }

  i4v rp[P_NL], rq[Q_NL];

  auto load_tiles = [&](int kt) {
    const long long kg = (long long)kt * BK;
    // ---- P operand ----
    if constexpr (MODE == MODE_FWD) {  // W K-major rows = out channels
#pragma unroll
      for (int i = 0; i < P_NL; ++i) {
        const int kk = p0 + krow0 + i * KRSTEP;
        rp[i] = (kk < K) ? ld16(Wt + (long long)kk * RSC + kg + kc * 8) : zero16();
      }
    } else if constexpr (MODE == MODE_DGRAD) {  // W MN-major: rows = reduction (k), cols = c
      const int rs = (int)(kg / K);
      const int k0 = (int)(kg - (long long)rs * K);
      const int c = p0 + p_cc * 8;
#pragma unroll
      for (int i = 0; i < P_NL; ++i) {
        const int kr = p_kr0 + i * (256 / P_CPR);
        rp[i] = (c < C) ? ld16(Wt + (long long)(k0 + kr) * RSC + rs * C + c) : zero16();
      }
    } else {  // WGRAD: dY MN-major rows = pixels, cols = out channels
      const int kch = p0 + p_cc * 8;
#pragma unroll
      for (int i = 0; i < P_NL; ++i) {
        const long long pix = kg + p_kr0 + i * (256 / P_CPR);
        rp[i] = (pix < Kr && kch < K) ? ld16(DY + pix * K + kch) : zero16();
      }
    }
    // ---- Q operand ----
    if constexpr (MODE == MODE_FWD) {  // X gather K-major
      const int rs = (int)(kg / C);
      const int c = (int)(kg - (long long)rs * C) + kc * 8;
      const int r = rs / S, s = rs - r * S;
#pragma unroll
      for (int i = 0; i < Q_NL; ++i) {
        const int ih = qh[i] + r, iw = qw[i] + s;
        const bool ok = (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
        rq[i] = ok ? ld16(X + ((long long)(qb[i] + ih * W + iw)) * C + c) : zero16();
      }
    } else if constexpr (MODE == MODE_DGRAD) {  // dY gather K-major
      const int rs = (int)(kg / K);
      const int k0 = (int)(kg - (long long)rs * K) + kc * 8;
      const int r = rs / S, s = rs - r * S;
#pragma unroll
      for (int i = 0; i < Q_NL; ++i) {
        int ph = qh[i] - r, pw = qw[i] - s;
        bool ok = ph >= 0 && pw >= 0;
        if (st > 1) {
          ok = ok && (ph % st == 0) && (pw % st == 0);
          ph /= st;
          pw /= st;
        }
        ok = ok && ph < P && pw < Q;
        rq[i] = ok ? ld16(DY + ((long long)(qb[i] + ph * Q + pw)) * K + k0) : zero16();
      }
    } else {  // WGRAD: X gather MN-major rows = pixels (n,p,q), cols = (r,s,c)
#pragma unroll
      for (int i = 0; i < Q_NL; ++i) {
        const long long pix = kg + q_kr0 + i * (256 / Q_CPR);
        bool ok = wg_cvalid && pix < Kr;
        i4v v = zero16();
        if (ok) {
          const int pi = (int)pix;
          const int n = pi / (P * Q), rem = pi - n * (P * Q);
          const int op = rem / Q, oq = rem - op * Q;
          const int ih = op * st - pd + wg_r, iw = oq * st - pd + wg_s;
          if ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W)
            v = ld16(X + ((long long)(n * H + ih) * W + iw) * C + wg_c);
        }
        rq[i] = v;
      }
    }
  };

  auto store_tiles = [&](int buf) {
    char* Ps = smem + buf * STAGE;
    char* Qs = Ps + P_BYTES;
    if constexpr (P_KMAJOR) {
#pragma unroll
      for (int i = 0; i < P_NL; ++i) *(i4v*)(Ps + km_off<BP>(krow0 + i * KRSTEP, kc)) = rp[i];
    } else {
#pragma unroll
      for (int i = 0; i < P_NL; ++i) *(i4v*)(Ps + mn_off<BP>(p_kr0 + i * (256 / P_CPR), p_cc)) = rp[i];
    }
    if constexpr (Q_KMAJOR) {
#pragma unroll
      for (int i = 0; i < Q_NL; ++i) *(i4v*)(Qs + km_off<BQ>(krow0 + i * KRSTEP, kc)) = rq[i];
    } else {
#pragma unroll
      for (int i = 0; i < Q_NL; ++i) *(i4v*)(Qs + mn_off<BQ>(q_kr0 + i * (256 / Q_CPR), q_cc)) = rq[i];
    }
  };

  f4v acc[TP][TQ];
#pragma unroll
  for (int i = 0; i < TP; ++i)
#pragma unroll
    for (int j = 0; j < TQ; ++j) acc[i][j] = (f4v){0.f, 0.f, 0.f, 0.f};

  load_tiles(kt0);
  store_tiles(0);
  __syncthreads();

  for (int kt = kt0; kt < kt1; ++kt) {
    const int cur = (kt - kt0) & 1;
    const bool more = kt + 1 < kt1;
    if (more) load_tiles(kt + 1);  // issue next tile's global loads before the MFMAs
    const char* Ps = smem + cur * STAGE;
    const char* Qs = Ps + P_BYTES;
#pragma unroll
    for (int u = 0; u < BK / 32; ++u) {
      s8v pf[TP], qf[TQ];
#pragma unroll
      for (int i = 0; i < TP; ++i) {
        if constexpr (P_KMAJOR) pf[i] = km_frag<BP>(Ps, wp * WP + i * 16, u, lane);
        else pf[i] = mn_frag<BP>(Ps, wp * WP + i * 16, u, lane);
      }
#pragma unroll
      for (int j = 0; j < TQ; ++j) {
        if constexpr (Q_KMAJOR) qf[j] = km_frag<BQ>(Qs, wq * WQ + j * 16, u, lane);
        else qf[j] = mn_frag<BQ>(Qs, wq * WQ + j * 16, u, lane);
      }
#pragma unroll
      for (int i = 0; i < TP; ++i)
#pragma unroll
        for (int j = 0; j < TQ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pf[i], qf[j], acc[i][j], 0, 0, 0);
    }
    if (more) store_tiles(cur ^ 1);
    __syncthreads();
  }

  // ---------------- epilogue ----------------
  const int lq = lane & 15, lp = 4 * (lane >> 4);
  if constexpr (MODE == MODE_FWD || MODE == MODE_DGRAD) {
    bf16_t* O = (bf16_t*)a.out + (long long)g * a.out_gs;
    const int ldo = Pd;  // NHWC: channel contiguous
    const float* bias = a.bias ? a.bias + (long long)g * a.bias_gs : nullptr;
    const bf16_t* res = a.residual ? (const bf16_t*)a.residual + (long long)g * a.out_gs : nullptr;
    const bf16_t* msk = a.mask ? (const bf16_t*)a.mask + (long long)g * a.out_gs : nullptr;
    float* stats = a.stats ? a.stats + (long long)g * a.stats_gs : nullptr;
#pragma unroll
    for (int i = 0; i < TP; ++i) {
      const int p = p0 + wp * WP + i * 16 + lp;
      float bsum[4] = {0.f, 0.f, 0.f, 0.f}, bsq[4] = {0.f, 0.f, 0.f, 0.f};
      float bv[4] = {0.f, 0.f, 0.f, 0.f};
      if (bias && p < Pd) {
#pragma unroll
        for (int e = 0; e < 4; ++e) bv[e] = bias[p + e];
      }
#pragma unroll
      for (int j = 0; j < TQ; ++j) {
        const int q = q0 + wq * WQ + j * 16 + lq;
        if (p < Pd && q < Qd) {
          float v[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = acc[i][j][e] + bv[e];
          const long long o = (long long)q * ldo + p;
          if (res) {
            const i2v rv = *(const i2v*)(res + o);
            v[0] += lo_bf((uint32_t)rv[0]); v[1] += hi_bf((uint32_t)rv[0]);
            v[2] += lo_bf((uint32_t)rv[1]); v[3] += hi_bf((uint32_t)rv[1]);
          }
          if (msk) {
            const i2v mv = *(const i2v*)(msk + o);
            if (!(lo_bf((uint32_t)mv[0]) > 0.f)) v[0] = 0.f;
            if (!(hi_bf((uint32_t)mv[0]) > 0.f)) v[1] = 0.f;
            if (!(lo_bf((uint32_t)mv[1]) > 0.f)) v[2] = 0.f;
            if (!(hi_bf((uint32_t)mv[1]) > 0.f)) v[3] = 0.f;
          }
          if (a.relu) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
          }
          i2v ov;
          ov[0] = (int)pack_bf2(v[0], v[1]);
          ov[1] = (int)pack_bf2(v[2], v[3]);
          *(i2v*)(O + o) = ov;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            bsum[e] += v[e];
            bsq[e] += v[e] * v[e];
          }
        }
      }
      if (MODE == MODE_FWD && stats) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float s = bsum[e], s2 = bsq[e];
#pragma unroll
          for (int o = 1; o < 16; o <<= 1) {
            s += __shfl_xor(s, o, 64);
            s2 += __shfl_xor(s2, o, 64);
          }
          bsum[e] = s;
          bsq[e] = s2;
        }
        if (lq == 0 && p < Pd) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            atomicAdd(stats + p + e, bsum[e]);
            atomicAdd(stats + K + p + e, bsq[e]);
          }
        }
      }
    }
  } else {  // WGRAD: dW[p=k][q=rsc] fp32
    float* O = (float*)a.out + (long long)g * a.out_gs;
    const bool atomic = a.accumulate || gridDim.y > 1;
#pragma unroll
    for (int i = 0; i < TP; ++i) {
#pragma unroll
      for (int j = 0; j < TQ; ++j) {
        const int q = q0 + wq * WQ + j * 16 + lq;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int p = p0 + wp * WP + i * 16 + lp + e;
          if (p < Pd && q < Qd) {
            float* dst = O + (long long)p * Qd + q;
            if (atomic) atomicAdd(dst, acc[i][j][e]);
            else *dst = acc[i][j][e];
          }
        }
      }
    }
  }
}

template <int MODE, int BP, int BQ, int BK>
static hipError_t launch_cfg(const ConvArgs& a, int Pd, int Qd, int splits, hipStream_t stream) {
  const int ntp = (Pd + BP - 1) / BP, ntq = (Qd + BQ - 1) / BQ;
  dim3 grid(ntp * ntq, splits, a.G);
  hipLaunchKernelGGL((conv_igemm_kernel<MODE, BP, BQ, BK>), grid, dim3(256), 0, stream, a);
  return hipGetLastError();
}

template <int MODE>
static hipError_t dispatch(const ConvArgs& a, int Pd, int Qd, int bp, int bq, int bk, int splits,
                           hipStream_t s) {
#define DDL_CFG(BP_, BQ_, BK_) \
  if (bp == BP_ && bq == BQ_ && bk == BK_) return launch_cfg<MODE, BP_, BQ_, BK_>(a, Pd, Qd, splits, s);
  DDL_CFG(64, 64, 32) DDL_CFG(64, 64, 64) DDL_CFG(64, 128, 32) DDL_CFG(64, 128, 64)
  DDL_CFG(128, 64, 32) DDL_CFG(128, 64, 64) DDL_CFG(128, 128, 32) DDL_CFG(128, 128, 64)
#undef DDL_CFG
  return hipErrorInvalidValue;
}

static int num_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  return cus;
}

// Validates the layout contract shared by all three modes.
static bool conv_shapes_ok(const ConvArgs& a) {
  if (a.G <= 0 || a.N <= 0 || a.C % 32 || a.K % 32 || a.R <= 0 || a.S <= 0) return false;
  if (a.stride <= 0 || a.pad < 0) return false;
  if (a.P != (a.H + 2 * a.pad - a.R) / a.stride + 1) return false;
  if (a.Q != (a.W + 2 * a.pad - a.S) / a.stride + 1) return false;
  return a.P > 0 && a.Q > 0;
}

// tile override: cfg = bp | bq<<8 | bk<<16 | splits<<24 (0 = heuristic); used by the autotuner.
DDL_API int ddl_conv_fwd(const ConvArgs* ap, int cfg, hipStream_t stream) {
  const ConvArgs& a = *ap;
  if (!conv_shapes_ok(a)) return (int)hipErrorInvalidValue;
  const int Pd = a.K, Qd = a.N * a.P * a.Q;
  int bp = a.K >= 128 ? 128 : 64, bq = 128, bk = (a.C % 64 == 0) ? 64 : 32;
  if (cfg) { bp = cfg & 0xff; bq = (cfg >> 8) & 0xff; bk = (cfg >> 16) & 0xff; }
  return (int)dispatch<MODE_FWD>(a, Pd, Qd, bp, bq, bk, 1, stream);
}

DDL_API int ddl_conv_dgrad(const ConvArgs* ap, int cfg, hipStream_t stream) {
  const ConvArgs& a = *ap;
  if (!conv_shapes_ok(a)) return (int)hipErrorInvalidValue;
  const int Pd = a.C, Qd = a.N * a.H * a.W;
  int bp = a.C >= 128 ? 128 : 64, bq = 128, bk = (a.K % 64 == 0) ? 64 : 32;
  if (cfg) { bp = cfg & 0xff; bq = (cfg >> 8) & 0xff; bk = (cfg >> 16) & 0xff; }
  if (bk > 32 && (a.K % bk)) return (int)hipErrorInvalidValue;
  return (int)dispatch<MODE_DGRAD>(a, Pd, Qd, bp, bq, bk, 1, stream);
}

DDL_API int ddl_conv_wgrad(const ConvArgs* ap, int cfg, hipStream_t stream) {
  const ConvArgs& a = *ap;
  if (!conv_shapes_ok(a)) return (int)hipErrorInvalidValue;
  const int Pd = a.K, Qd = a.R * a.S * a.C;
  const long long Kr = (long long)a.N * a.P * a.Q;
  int bp = a.K >= 128 ? 128 : 64, bq = Qd >= 128 ? 128 : 64, bk = 64;
  if (cfg) { bp = cfg & 0xff; bq = (cfg >> 8) & 0xff; bk = (cfg >> 16) & 0xff; }
  // wgrad gathers X by 8-channel chunks inside one (r,s) tap
  if (a.C % 8) return (int)hipErrorInvalidValue;
  const long long tiles = (long long)((Pd + bp - 1) / bp) * ((Qd + bq - 1) / bq) * a.G;
  const long long nk = (Kr + bk - 1) / bk;
  int splits = (cfg >> 24) & 0xff;
  if (!splits) {
    // aim for ~2 waves of workgroups over the CUs, keep >= 8 K-steps per split
    long long want = (2LL * num_cus() + tiles - 1) / tiles;
    long long maxs = nk / 8 > 0 ? nk / 8 : 1;
    splits = (int)(want < maxs ? want : maxs);
    if (splits < 1) splits = 1;
    if (splits > 255) splits = 255;
  }
  if (splits > 1 && !a.accumulate) return (int)hipErrorInvalidValue;  // needs zeroed fp32 output
  return (int)dispatch<MODE_WGRAD>(a, Pd, Qd, bp, bq, bk, splits, stream);
}

DDL_API int ddl_conv_args_size() { return (int)sizeof(ConvArgs); }
