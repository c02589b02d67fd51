// Shared pieces of the reference-precision (fp32) convolution kernels: the launch-argument block,
// per-block geometry, the exact 3-way bf16 operand split of the X6 engine and the fused epilogue.
//
// Two kernel families include this header:
//   * conv_f32.hip  — register-staged implicit GEMM, 16x16 MFMA tiles (exact fp32 MFMA or X6);
//   * conv_x6h.hip  — halo-staged X6 FWD / stride-1 DGRAD, 32x32x16 bf16 MFMA tiles, pre-split
//                     weights.
// The epilogue is written once against an accumulator LAYOUT policy: each lane holds "quads" of
// four consecutive output channels p for one output row q; the policy says which (p, q) a quad is
// and how many lanes share one p set (the width of the q reduction for BN statistics).
#pragma once
#include "ddl_common.h"

struct ConvF32Args {
  const float* x;         // [G][N][H][W][C]                    (group stride x_gs)
  const float* w;         // [G][K][R][S][C]                    (w_gs)
  const float* dy;        // [G][N][P][Q][K]                    (dy_gs)
  float* out;             // FWD y [G][N][P][Q][K] | DGRAD dx [G][N][H][W][C] | WGRAD dw like w (out_gs)
  float* stats;           // FWD: [G][slots][2][K] (sum, sumsq) | DGRAD with bn_x: [G][slots][2][C]
  const float* bias;      // FWD [G][K] (bias_gs)
  const float* residual;  // FWD / DGRAD: added (layout of out; DGRAD res_sub 2: compact grid, res_gs)
  const float* mask;      // DGRAD: dx *= (mask > 0) (layout of out)
  const float* in_scale;  // X operand transform (FWD / WGRAD): [G][C] contiguous
  const float* in_shift;
  const float* bn_x;      // DGRAD BN-backward reduce: the preceding BN's input (layout of out)
  const float* bn_mean;   // [G][C]
  const float* bn_rstd;
  const float* mask_scale;  // DGRAD: keep dx where bn_x * mask_scale + mask_shift > 0
  const float* mask_shift;
  float* partial;         // split-K workspace
  long long partial_cap;  // floats at `partial`
  long long x_gs, w_gs, dy_gs, out_gs, bias_gs, res_gs;
  int G, N, H, W, C, K, R, S, P, Q, stride, pad;
  int relu, accumulate, split_k, res_sub, in_relu;
  int slots;              // stats / BN-reduce slots per group (filled by the launcher)
  float gscale;           // WGRAD: out = (accumulate ? out : 0) + gscale * dW
  // conv_x6h: the weights pre-split into the X6 operand image (ddl_x6_split_weights), FWD layout
  // [G][K][R][S][C] or DGRAD layout [G][C][R][S][K], 8 bytes per element (group stride ws_gs bytes)
  const void* wsplit;
  long long ws_gs;
  // DGRAD (conv_x6h): the dY operand is the BN backward of the following BN, applied on the fly:
  // dY' = A[k] * dy + B[k] * dyb_x + C[k] with dyb_coef [G][3][K] (A | B | C) and dyb_x the BN's
  // input (layout of dy); dyb_out (nullable) receives dY' (each element written once: the first
  // P tile, core halo pixels) for the same layer's WGRAD
  const float* dyb_x;
  const float* dyb_coef;
  float* dyb_out;
  // WGRAD split-K (conv_f32.hip): one arrival counter per (group, tile), zero between launches;
  // the last slice's workgroup folds the slices in slice order (no reduce launch). Null: reduce pass
  int* tickets;
  long long tickets_cap;
};

enum { F_FWD = 0, F_DGRAD = 1, F_WGRAD = 2 };

struct FDiv {
  uint32_t m;
  int s;
};
__host__ __device__ inline FDiv mk_fdiv(uint32_t d) {
  FDiv f;
  if (d <= 1) { f.m = 0; f.s = 0; return f; }
  int l = 0;
  while ((1u << l) < d) ++l;
  f.m = (uint32_t)((((1ull << 32) * ((1ull << l) - d)) / d) + 1);
  f.s = l;
  return f;
}
__device__ __forceinline__ int fdv(int x, FDiv f) {
  if (f.s == 0) return x;
  const uint32_t t = __umulhi((uint32_t)x, f.m);
  return (int)((t + (((uint32_t)x - t) >> 1)) >> (f.s - 1));
}

// Per-block problem geometry (shared by the main kernels and the split-K epilogue kernel).
struct FGeo {
  int Pd, Qd, Kr, nph, phase, split, nsplit, g, p0, q0, tq;
  int pa, pb, Hs, Ws, r0, s0, Rn, Sn;
};

template <int MODE, int BP, int BQ>
__device__ __forceinline__ FGeo fgeo(const ConvF32Args& a, int bx, int by, int g, int gy) {
  FGeo o;
  o.nph = (MODE == F_DGRAD && a.stride == 2) ? 4 : 1;
  o.phase = by % o.nph;
  o.split = by / o.nph;
  o.nsplit = gy / o.nph;
  o.g = g;
  o.pa = o.pb = o.r0 = o.s0 = 0;
  o.Hs = a.H; o.Ws = a.W; o.Rn = a.R; o.Sn = a.S;
  if (MODE == F_FWD) {
    o.Pd = a.K; o.Qd = a.N * a.P * a.Q; o.Kr = a.R * a.S * a.C;
  } else if (MODE == F_DGRAD) {
    o.Pd = a.C;
    if (o.nph == 4) {
      o.pa = o.phase >> 1; o.pb = o.phase & 1;
      o.Hs = (a.H - o.pa + 1) >> 1; o.Ws = (a.W - o.pb + 1) >> 1;
      o.r0 = (o.pa + a.pad) & 1; o.s0 = (o.pb + a.pad) & 1;
      o.Rn = (a.R - o.r0 + 1) >> 1; o.Sn = (a.S - o.s0 + 1) >> 1;
    }
    o.Qd = a.N * o.Hs * o.Ws;
    o.Kr = o.Rn * o.Sn * a.K;
  } else {
    o.Pd = a.K; o.Qd = a.R * a.S * a.C; o.Kr = a.N * a.P * a.Q;
  }
  const int ntp = (o.Pd + BP - 1) / BP;
  o.p0 = (bx % ntp) * BP;
  o.tq = bx / ntp;
  o.q0 = o.tq * BQ;
  return o;
}

// ------------------------------------------------------------------------- accumulator layouts
// A workgroup is 4 waves, 2 x 2 over the BP x BQ tile; wave (wp, wq) owns rows wp*BP/2 .. and
// columns wq*BQ/2 .. . Each lane holds NPQ x NQ quads; quad (i, j) = D[p .. p+3][q] with
//   p = wp * BP/2 + poff(i, lane),  q = wq * BQ/2 + qoff(j, lane).
// QL lanes (the low bits of the lane id) share one set of p and differ in q.
template <int BP, int BQ>
struct Lay16 {  // v_mfma_*_16x16x*: acc[ti][tj] = one quad, lane: q = lane & 15, p = 4 * (lane >> 4)
  static constexpr int NPQ = BP / 32, NQ = BQ / 32, QL = 16;
  static __device__ __forceinline__ int poff(int i, int lane) { return i * 16 + 4 * (lane >> 4); }
  static __device__ __forceinline__ int qoff(int j, int lane) { return j * 16 + (lane & 15); }
};
template <int BP, int BQ>
struct Lay32 {  // v_mfma_f32_32x32x16_bf16: acc[ti][tj] = 16 floats = 4 quads (gg = v >> 2),
                // lane: q = lane & 31, p = 8 * gg + 4 * (lane >> 5)
  static constexpr int NPQ = BP / 16, NQ = BQ / 64, QL = 32;
  static __device__ __forceinline__ int poff(int i, int lane) {
    return (i >> 2) * 32 + 8 * (i & 3) + 4 * (lane >> 5);
  }
  static __device__ __forceinline__ int qoff(int j, int lane) { return j * 32 + (lane & 31); }
};

// ------------------------------------------------------------------------------------ epilogue
// FWD: y = [relu](acc + bias + residual), per-tile BN statistics (sum, M2 about the tile mean) to
// the tile's slot. DGRAD: dx = mask(acc + residual), with bn_x the BN-backward partial sums
// (sum dy, sum dy * xhat) to the tile's slot. WGRAD: out = (accumulate ? out : 0) + gscale * acc.
// `red`: >= 4 * BP floats of LDS (free: the main loop is over, all waves past its last barrier).
template <int MODE, int BP, int BQ, class L>
__device__ __forceinline__ void fepi(const ConvF32Args& a, const FGeo& o, f4v (&acc)[L::NPQ][L::NQ], float* red) {
  constexpr int WP = BP / 2, WQ = BQ / 2, NP = L::NPQ, NQ = L::NQ, QL = L::QL;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wp = wid >> 1, wq = wid & 1;
  const int g = o.g;
  if constexpr (MODE == F_WGRAD) {
    const int RSC = o.Qd;
    float* outg = a.out + (long long)g * a.out_gs;
#pragma unroll
    for (int i = 0; i < NP; ++i)
#pragma unroll
      for (int j = 0; j < NQ; ++j) {
        const int q = o.q0 + wq * WQ + L::qoff(j, lane);
        if (q >= RSC) continue;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int p = o.p0 + wp * WP + L::poff(i, lane) + v;
          if (p >= o.Pd) continue;
          float* d = outg + (long long)p * RSC + q;
          const float base = a.accumulate ? *d : 0.f;
          *d = base + a.gscale * acc[i][j][v];
        }
      }
    return;
  }
  const bool want_stats = a.stats != nullptr;
  const bool dg_stats = MODE == F_DGRAD && want_stats && a.bn_x;
  const int Pd = o.Pd;
  float* outg = a.out + (long long)g * a.out_gs;
  // per-q geometry of this lane (output pixel of each q column)
  long long pix[NQ];
  int hq[NQ], wqq[NQ], nq_[NQ];
  bool qv[NQ];
  const FDiv dpq = mk_fdiv((uint32_t)(o.Hs * o.Ws)), dq = mk_fdiv((uint32_t)o.Ws);
#pragma unroll
  for (int j = 0; j < NQ; ++j) {
    const int q = o.q0 + wq * WQ + L::qoff(j, lane);
    qv[j] = q < o.Qd;
    pix[j] = q;
    hq[j] = wqq[j] = nq_[j] = 0;
    if (MODE == F_DGRAD) {
      const int nn = fdv(q, dpq);
      const int rem = q - nn * o.Hs * o.Ws;
      const int ii = fdv(rem, dq), jj = rem - ii * o.Ws;
      const int hh = o.nph == 4 ? 2 * ii + o.pa : ii;
      const int ww = o.nph == 4 ? 2 * jj + o.pb : jj;
      nq_[j] = nn; hq[j] = hh; wqq[j] = ww;
      pix[j] = ((long long)nn * a.H + hh) * a.W + ww;
    }
  }
  // Quad rows (i) outer, q columns (j) inner: per-channel constants are loaded once per quad row
  // and the BN partial sums of a row are reduced across lanes right away (no per-row arrays live).
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int p = o.p0 + wp * WP + L::poff(i, lane);
    const bool pv = p < Pd;
    float bia[4], bm[4], br[4], ms[4], mh[4];
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      bia[v] = (MODE == F_FWD && a.bias && pv) ? a.bias[(long long)g * a.bias_gs + p + v] : 0.f;
      bm[v] = (MODE == F_DGRAD && a.bn_x && pv) ? a.bn_mean[(long long)g * Pd + p + v] : 0.f;
      br[v] = (MODE == F_DGRAD && a.bn_x && pv) ? a.bn_rstd[(long long)g * Pd + p + v] : 0.f;
      ms[v] = (MODE == F_DGRAD && a.mask_scale && pv) ? a.mask_scale[(long long)g * Pd + p + v] : 0.f;
      mh[v] = (MODE == F_DGRAD && a.mask_scale && pv) ? a.mask_shift[(long long)g * Pd + p + v] : 0.f;
    }
    float s0[4] = {0.f, 0.f, 0.f, 0.f}, s1[4] = {0.f, 0.f, 0.f, 0.f};
    // every operand load of the row is issued before any is used (a load behind a use or a
    // branch waits out the previous one's latency: conv_x6h.hip's DGRAD epilogue ran ~4x its bytes'
    // time that way). Lanes without an element read element 0 of the group and drop the value.
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 rr[NQ], mm[NQ], xx[NQ];
    long long ee[NQ];
#pragma unroll
    for (int j = 0; j < NQ; ++j) ee[j] = (qv[j] && pv) ? pix[j] * Pd + p : 0;
    const long long gofs = (long long)g * a.out_gs;
    if (a.residual && (MODE == F_FWD || a.res_sub != 2)) {
#pragma unroll
      for (int j = 0; j < NQ; ++j) rr[j] = *(const float4*)(a.residual + gofs + ee[j]);
    } else if (MODE == F_DGRAD && a.residual) {  // compact grid: even (h, w) only
      const int Hc = (a.H + 1) >> 1, Wc = (a.W + 1) >> 1;
#pragma unroll
      for (int j = 0; j < NQ; ++j) {
        const bool on = qv[j] && pv && ((hq[j] | wqq[j]) & 1) == 0;
        const long long re = on ? (((long long)nq_[j] * Hc + (hq[j] >> 1)) * Wc + (wqq[j] >> 1)) * Pd + p : 0;
        rr[j] = *(const float4*)(a.residual + (long long)g * a.res_gs + re);
        if (!on) rr[j] = z4;
      }
    }
    if (MODE == F_DGRAD && a.mask) {
#pragma unroll
      for (int j = 0; j < NQ; ++j) mm[j] = *(const float4*)(a.mask + gofs + ee[j]);
    }
    if (MODE == F_DGRAD && a.bn_x) {
#pragma unroll
      for (int j = 0; j < NQ; ++j) xx[j] = *(const float4*)(a.bn_x + gofs + ee[j]);
    }
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
      if (!qv[j] || !pv) continue;
      const long long e = ee[j];
      float v4[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if (MODE == F_FWD) {
#pragma unroll
        for (int v = 0; v < 4; ++v) v4[v] += bia[v];
        if (a.residual) {
          v4[0] += rr[j].x; v4[1] += rr[j].y; v4[2] += rr[j].z; v4[3] += rr[j].w;
        }
        if (a.relu) {
#pragma unroll
          for (int v = 0; v < 4; ++v) v4[v] = fmaxf(v4[v], 0.f);
        }
        if (want_stats) {
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            s0[v] += v4[v];
            acc[i][j][v] = v4[v];  // kept for the centred second pass below
          }
        }
      } else {  // DGRAD
        if (a.residual) {
          v4[0] += rr[j].x; v4[1] += rr[j].y; v4[2] += rr[j].z; v4[3] += rr[j].w;
        }
        if (a.mask) {
          const float4 m = mm[j];
          if (!(m.x > 0.f)) v4[0] = 0.f;
          if (!(m.y > 0.f)) v4[1] = 0.f;
          if (!(m.z > 0.f)) v4[2] = 0.f;
          if (!(m.w > 0.f)) v4[3] = 0.f;
        }
        if (a.bn_x) {
          const float xs[4] = {xx[j].x, xx[j].y, xx[j].z, xx[j].w};
          if (a.mask_scale) {
#pragma unroll
            for (int v = 0; v < 4; ++v)
              if (!(xs[v] * ms[v] + mh[v] > 0.f)) v4[v] = 0.f;
          }
          if (want_stats) {
#pragma unroll
            for (int v = 0; v < 4; ++v) {
              s0[v] += v4[v];
              s1[v] += v4[v] * ((xs[v] - bm[v]) * br[v]);
            }
          }
        }
      }
      *(float4*)(outg + e) = make_float4(v4[0], v4[1], v4[2], v4[3]);
    }
    // this quad row's partial sums over the tile's q -> red (FWD: sums only; M2 below)
    if ((MODE == F_FWD && want_stats) || dg_stats) {
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        float x0 = s0[v], x1 = s1[v];
#pragma unroll
        for (int o2 = 1; o2 < QL; o2 <<= 1) {
          x0 += __shfl_xor(x0, o2, 64);
          if (MODE == F_DGRAD) x1 += __shfl_xor(x1, o2, 64);
        }
        if ((lane & (QL - 1)) == 0) {
          const int pl = wp * WP + L::poff(i, lane) + v;
          red[(wq * BP + pl) * 2] = x0;
          if (MODE == F_DGRAD) red[(wq * BP + pl) * 2 + 1] = x1;
        }
      }
    }
  }
  if (!want_stats || (MODE == F_DGRAD && !a.bn_x)) return;
  if constexpr (MODE == F_FWD) {
    // Forward BN statistics of this tile as (sum, M2 = sum of squared deviations from the TILE
    // mean): two passes over the register-resident outputs, merged across tiles in bnf_finalize
    // with Chan's formula. A single-pass (sum, sum of squares) loses the variance to cancellation
    // when |mean| >> std (deep layers of ResNet-50: 1e-5 relative error in rstd).
    const int nq = min(BQ, o.Qd - o.q0);  // valid rows of this tile
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const bool pv = o.p0 + wp * WP + L::poff(i, lane) < Pd;
      float mu[4], s1[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int pl = wp * WP + L::poff(i, lane) + v;
        mu[v] = (red[pl * 2] + red[(BP + pl) * 2]) / (float)nq;
      }
#pragma unroll
      for (int j = 0; j < NQ; ++j) {
        if (!qv[j] || !pv) continue;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const float d = acc[i][j][v] - mu[v];
          s1[v] += d * d;
        }
      }
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        float x1 = s1[v];
#pragma unroll
        for (int o2 = 1; o2 < QL; o2 <<= 1) x1 += __shfl_xor(x1, o2, 64);
        if ((lane & (QL - 1)) == 0) red[(wq * BP + wp * WP + L::poff(i, lane) + v) * 2 + 1] = x1;
      }
    }
    __syncthreads();
    if (tid < BP && o.p0 + tid < Pd) {
      const int slot = o.phase * (a.slots / o.nph) + o.tq;
      float* st = a.stats + ((long long)g * a.slots + slot) * 2 * Pd + o.p0 + tid;
      st[0] = red[tid * 2] + red[(BP + tid) * 2];
      st[Pd] = red[tid * 2 + 1] + red[(BP + tid) * 2 + 1];
    }
    return;
  }
  __syncthreads();
  if (tid < BP && o.p0 + tid < Pd) {
    const float t0 = red[tid * 2] + red[(BP + tid) * 2];
    const float t1 = red[tid * 2 + 1] + red[(BP + tid) * 2 + 1];
    const int slot = o.phase * (a.slots / o.nph) + o.tq;
    float* st = a.stats + ((long long)g * a.slots + slot) * 2 * Pd + o.p0 + tid;
    st[0] = t0;
    st[Pd] = t1;
  }
}

// zero stats slot of a tile that has no work (q0 beyond a smaller DGRAD phase)
template <int MODE, int BP>
__device__ __forceinline__ void fzero_slot(const ConvF32Args& a, const FGeo& o) {
  if (MODE == F_WGRAD || !a.stats || (MODE == F_DGRAD && !a.bn_x)) return;
  const int tid = threadIdx.x;
  if (tid < BP && o.p0 + tid < o.Pd) {
    const int slot = o.phase * (a.slots / o.nph) + o.tq;
    float* st = a.stats + ((long long)o.g * a.slots + slot) * 2 * o.Pd + o.p0 + tid;
    st[0] = 0.f;
    st[o.Pd] = 0.f;
  }
}

// FWD / DGRAD split-K: sum the slices in slice order, then the same epilogue as the main kernel.
template <int MODE, int BP, int BQ>
__global__ __launch_bounds__(256) void convf32_splitk_epilogue(ConvF32Args a) {
  constexpr int WP = BP / 2, WQ = BQ / 2, TP = WP / 16, TQ = WQ / 16;
  __shared__ float red[2 * BP * 2];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wp = wid >> 1, wq = wid & 1;
  const int nph = (MODE == F_DGRAD && a.stride == 2) ? 4 : 1;
  const FGeo o = fgeo<MODE, BP, BQ>(a, blockIdx.x, blockIdx.y, blockIdx.z, nph * a.split_k);
  if (o.q0 >= o.Qd || o.p0 >= o.Pd) {
    fzero_slot<MODE, BP>(a, o);
    return;
  }
  const long long qmax = (long long)a.slots / nph * BQ;
  const long long slice = (long long)a.G * nph * qmax * o.Pd;
  const float* base = a.partial + ((long long)o.g * nph + o.phase) * qmax * o.Pd;
  // slice-outer: each slice's TP x TQ fragment loads are in flight together (fragment-outer, every
  // load of a fragment's slice chain waited on the previous add); per fragment the adds still run
  // in slice order, so the sum is bitwise the same
  f4v acc[TP][TQ];
  bool ok[TP][TQ];
  const float* src[TP][TQ];
#pragma unroll
  for (int ti = 0; ti < TP; ++ti)
#pragma unroll
    for (int tj = 0; tj < TQ; ++tj) {
      const int q = o.q0 + wq * WQ + tj * 16 + (lane & 15);
      const int p = o.p0 + wp * WP + ti * 16 + 4 * (lane >> 4);
      ok[ti][tj] = q < o.Qd && p < o.Pd;
      src[ti][tj] = base + (ok[ti][tj] ? (long long)q * o.Pd + p : 0);
      acc[ti][tj] = (f4v){0.f, 0.f, 0.f, 0.f};
    }
  for (int k = 0; k < a.split_k; ++k) {
    f4v v[TP][TQ];
#pragma unroll
    for (int ti = 0; ti < TP; ++ti)
#pragma unroll
      for (int tj = 0; tj < TQ; ++tj)
        v[ti][tj] = ok[ti][tj] ? *(const f4v*)(src[ti][tj] + k * slice) : (f4v){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ti = 0; ti < TP; ++ti)
#pragma unroll
      for (int tj = 0; tj < TQ; ++tj) acc[ti][tj] += v[ti][tj];
  }
  fepi<MODE, BP, BQ, Lay16<BP, BQ>>(a, o, acc, red);
}


// ------------------------------------------------------------------------------------ X6 split
// fp32 products on the bf16 MFMA (X6). Every fp32 operand value splits EXACTLY into three bf16
// pieces by truncation, x = xh + xm + xl (xh: the top 8 significand bits, xm the next 8, xl the
// last 8 — each remainder is exact in fp32 and the last fits bf16 exactly). Of the nine piece
// products the six down to 2^-16 relative are kept (hh, hm, mh, hl, lh, mm); the dropped ml, lm,
// ll are <= 2^-24 relative, the size of one fp32 rounding, and every bf16 x bf16 product is exact
// in the fp32 accumulator. A 4-deep chunk of reduction values becomes two 16-byte MFMA operand
// halves, (h0..h3 | m0..m3) and (l0..l3 | h0..h3); per chunk three MFMA slot pairings
//   A (l | h) . B (h | m) = lh + hm      A (h | m) . B (l | h) = hl + mh      A (h | m) . B (h | m) = hh + mm
// give the six products.
__device__ __forceinline__ void split3(float4 v, s4v& h, s4v& m, s4v& l) {
  const float x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t u = __float_as_uint(x[i]);
    const float r1 = x[i] - __uint_as_float(u & 0xFFFF0000u);
    const uint32_t um = __float_as_uint(r1);
    const float r2 = r1 - __uint_as_float(um & 0xFFFF0000u);
    h[i] = (short)(u >> 16);
    m[i] = (short)(um >> 16);
    l[i] = (short)(__float_as_uint(r2) >> 16);
  }
}
__device__ __forceinline__ void split1(float x, uint16_t& h, uint16_t& m, uint16_t& l) {
  const uint32_t u = __float_as_uint(x);
  const float r1 = x - __uint_as_float(u & 0xFFFF0000u);
  const uint32_t um = __float_as_uint(r1);
  const float r2 = r1 - __uint_as_float(um & 0xFFFF0000u);
  h = (uint16_t)(u >> 16);
  m = (uint16_t)(um >> 16);
  l = (uint16_t)(__float_as_uint(r2) >> 16);
}
__device__ __forceinline__ s8v cat44(s4v a, s4v b) {
  return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}
