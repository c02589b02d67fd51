// Reference-precision (fp32) implicit-GEMM convolution, NHWC fp32, in two product engines:
//   * exact: CDNA4's fp32 MFMA (v_mfma_f32_16x16x4_f32: fp32 operands, fp32 accumulate, bitwise
//     an fmaf chain);
//   * X6: fp32 products as six bf16 piece products on the double-rate v_mfma_f32_16x16x32_bf16
//     (exact 3-way operand split, dropped terms <= one fp32 rounding; see split3) — 2.7x fewer
//     MFMA cycles per step, same loads / LDS images / epilogues / determinism.
//
// The reference trains every model in fp32 (stock nn.Conv2d / nn.Linear, reference
// lab/tutorial_1a/hfl_complete.py:39-80); this is the kernel family behind the framework's fp32
// precision mode, which the headline benchmark runs. Same three products as the bf16 family
// (conv_igemm.hip), D[p][q] = sum_k Pop[p][k] * Qop[q][k]:
//
//   FWD   : y [q=(n,ho,wo)][p=k]    = sum_{(r,s,c)} W[k][(r,s,c)]    * X[pix(q,r,s)][c]
//   DGRAD : dx[q=(n,h,w)][p=c]      = sum_{(r,s,k)} W[k][(r,s,c)]    * dY[pix'(q,r,s)][k]
//   WGRAD : dW[p=k][q=(r,s,c)]     (+)= sum_{(n,ho,wo)} dY[pix][k]   * X[pix(r,s)][c]
//
// Design (fp32 MFMA issues at 1/16 of the bf16 rate, so the kernel is compute-bound from a much
// lower arithmetic intensity and needs no LDS-DMA rings or halo staging):
//   * 256-thread workgroup, 2x2 waves over a BP x BQ tile (64/128 each), 16-deep reduction steps;
//     each wave owns (BP/2) x (BQ/2) as 16x16 MFMA tiles (up to 16 independent accumulators);
//   * operands are register-prefetched one step ahead with 16-byte global loads and stored to a
//     double-buffered LDS image [rows][16 floats] whose 16-B chunk c of row r sits at
//     c ^ ((r >> 2) & 2): every fragment is ONE ds_read_b128 (4 reduction indices = the 4 MFMA
//     sub-steps, the same permutation of k on both operands) and conflict-free for the b128 lane
//     groups; MN-major sources (contiguous along p or q) are transposed 4 x KU in registers;
//   * one barrier per step; XCD-aware block order (consecutive tiles of one split / phase /
//     client share an XCD's L2);
//   * operand-side BatchNorm: with in_scale/in_shift the X operand is relu(x * scale + shift) on
//     in-image pixels (zero padding stays zero), so a BN+ReLU output that feeds only a conv is
//     never materialised (FWD reads the BN input, WGRAD recomputes it);
//   * DETERMINISTIC by construction — no floating-point atomics anywhere:
//       - FWD BN statistics and the DGRAD epilogue's BN-backward reduce are written per q-tile into
//         their own slot [G][slots][2][Pd] (plain stores, no zero-fill), folded in fixed order;
//       - split-K (grids too small to fill 256 CUs) stores fp32 partial slices that a second
//         kernel sums in slice order before the epilogue / the weight update;
//       - WGRAD's (out = out + gscale * dW) has exactly one writer per element (gscale = -lr on
//         the master weights is plain SGD fused into the backward).
//   * stride-2 DGRAD runs as four sub-pixel phases (no MFMA on taps that miss every output);
//     larger strides (none in the model zoo) run unphased with a per-tap divisibility test.
#include "conv_f32_core.h"
#include <cstdlib>

// operand prefetch depth in steps (register sets): 2 or 3
#ifndef F32_PREFETCH
#define F32_PREFETCH 2
#endif

constexpr int FBK = 16;

__device__ __forceinline__ int fswz(int row) { return (row >> 2) & 2; }
__device__ __forceinline__ int lds_off(int row, int ch) { return row * 16 + ((ch ^ fswz(row)) << 2); }

// ------------------------------------------------------------------------------------ X6 math
// fp32 products on the bf16 MFMA (X6 = 1). Every fp32 operand value splits EXACTLY into three
// bf16 pieces by truncation, x = xh + xm + xl (xh: the top 8 significand bits, xm the next 8, xl
// the last 8 — each remainder is exact in fp32 and the last fits bf16 exactly). Of the nine piece
// products the six down to 2^-16 relative are kept (hh, hm, mh, hl, lh, mm); the dropped ml, lm,
// ll are <= 2^-24 relative, the size of one fp32 rounding, and every bf16 x bf16 product is exact
// in the fp32 accumulator.
// The split happens ONCE, when a thread stores its loaded values to LDS: a 4-deep k chunk of a
// row becomes 32 bytes, two 16-byte halves (h | m) and (l | h), so every MFMA operand is one
// ds_read_b128 and the inner loop has no conversion work (splitting the fragments after the LDS
// read instead cost 253 VALU instructions per step against 24 MFMAs: VALU-bound). A 16-deep
// step is 16 k values x 6 piece pairs = three v_mfma_f32_16x16x32_bf16 per 16x16 tile (lane group
// g = k values 4g..4g+3):
//   A (l | h) . B (h | m) = lh + hm      A (h | m) . B (l | h) = hl + mh      A (h | m) . B (h | m) = hh + mm
// 48 MFMA cycles per tile-step instead of 128 for four v_mfma_f32_16x16x4_f32. Each step's three
// MFMAs start from a zero accumulator and are added to the running sum with one IEEE add: the bf16
// MFMA's internal accumulation is not a round-to-nearest fp32 chain, and over a 10^5-deep WGRAD
// reduction its bias would reach 1e-3 relative.
// LDS image: row r holds 4 chunks x 8 dwords; chunk c's half h sits at dword
//   r*32 + 8*(c ^ f(r)) + 4*(h ^ g(r)),  f = b1 << 1, g = b0 ^ b2  (bits of r)
// which makes both halves' fragment reads conflict-free for the four ds_read_b128 lane groups AND
// the K-major ds_write_b128 stores (8-lane groups = rows 2m, 2m+1 x 4 chunks) conflict-free (the
// previous swizzle left those stores 2-way; found by exhaustive search over XOR-linear swizzles).
__device__ __forceinline__ int x6_off(int row, int ch, int half) {  // dwords
  const int f = row & 2;                     // (b1 << 1)
  const int g = (row ^ (row >> 2)) & 1;      // b0 ^ b2
  return row * 32 + 8 * (ch ^ f) + 4 * (half ^ g);
}

// ------------------------------------------------------------------------------------ main kernel
template <int MODE, int BP, int BQ, int X6>
__global__ __launch_bounds__(256, (X6 && BP * BQ <= 64 * 128) ? 3 : 2) void convf32_kernel(ConvF32Args a) {
  constexpr int WP = BP / 2, WQ = BQ / 2, TP = WP / 16, TQ = WQ / 16;
  constexpr int RW = X6 ? 32 : 16;              // dwords per image row (X6: 3 bf16 pieces + dup)
  constexpr int SP = BP * RW, SQ = BQ * RW;     // dwords per operand image
  constexpr int UPK = BP / 64, UQK = BQ / 64;    // K-major units (float4) per thread
  constexpr int KUP = BP / 64, KUQ = BQ / 64;    // MN-major reductions per unit (4 rows x KU)
  __shared__ float4 smem4[(2 * (SP + SQ)) / 4];
  float* smem = (float*)smem4;
  __shared__ float xform[2 * 512];               // in_scale | in_shift (C <= 512)

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wp = wid >> 1, wq = wid & 1;
  const int gx = gridDim.x, gy = gridDim.y, gz = gridDim.z;
  const int lin = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  const int u = xcd_remap(lin, gx * gy * gz);
  const int bx = u % gx, by = (u / gx) % gy, g = u / (gx * gy);
  const FGeo o = fgeo<MODE, BP, BQ>(a, bx, by, g, gy);
  const bool split_store = a.split_k > 1;
  if (o.q0 >= o.Qd || o.p0 >= o.Pd) {
    // an empty tile's statistics slot is zeroed once (by the epilogue launch without tickets)
    if (!split_store || (a.tickets && o.split == 0)) fzero_slot<MODE, BP>(a, o);
    return;
  }
  const int nk = (o.Kr + FBK - 1) / FBK;
  const int per = (nk + o.nsplit - 1) / o.nsplit;
  const int kt0 = o.split * per, kt1 = min(nk, kt0 + per);

  const int H = a.H, W = a.W, C = a.C, K = a.K, S = a.S, P = a.P, Q = a.Q, st = a.stride, pd = a.pad;
  const float* X = a.x + (long long)g * a.x_gs;
  const float* Wt = a.w + (long long)g * a.w_gs;
  const float* DY = a.dy + (long long)g * a.dy_gs;
  const bool xf = (MODE != F_DGRAD) && a.in_scale != nullptr;
  if (xf) {
    for (int i = tid; i < C; i += 256) {
      xform[i] = a.in_scale[(long long)g * C + i];
      xform[512 + i] = a.in_shift[(long long)g * C + i];
    }
  }
  const bool xrelu = a.in_relu != 0;

  // ----------------------------------------------------------- per-thread operand bookkeeping
  // P operand
  int pk_row[UPK], pk_ch[UPK];  // FWD K-major units
  int pm_rg = 0, pm_kp = 0;     // DGRAD / WGRAD MN-major unit
  if constexpr (MODE == F_FWD) {
#pragma unroll
    for (int i = 0; i < UPK; ++i) {
      const int uu = tid + 256 * i;
      pk_row[i] = uu >> 2;
      pk_ch[i] = uu & 3;
    }
  } else {
    pm_kp = tid % (16 / KUP);
    pm_rg = tid / (16 / KUP);
  }
  // Q operand
  int qk_row[UQK], qk_ch[UQK], qk_n[UQK], qk_hb[UQK], qk_wb[UQK];
  int qm_rg = 0, qm_kp = 0, qm_r = 0, qm_s = 0, qm_c = 0;
  bool qm_ok = false;
  float qm_sc[4] = {1.f, 1.f, 1.f, 1.f}, qm_sh[4] = {0.f, 0.f, 0.f, 0.f};
  if constexpr (MODE != F_WGRAD) {
    const FDiv dpq = mk_fdiv((uint32_t)(MODE == F_FWD ? P * Q : o.Hs * o.Ws));
    const FDiv dq = mk_fdiv((uint32_t)(MODE == F_FWD ? Q : o.Ws));
    const int PQ = MODE == F_FWD ? P * Q : o.Hs * o.Ws, QQ = MODE == F_FWD ? Q : o.Ws;
#pragma unroll
    for (int i = 0; i < UQK; ++i) {
      const int uu = tid + 256 * i;
      qk_row[i] = uu >> 2;
      qk_ch[i] = uu & 3;
      const int q = o.q0 + qk_row[i];
      if (q < o.Qd) {
        const int n = fdv(q, dpq), rem = q - n * PQ;
        const int y = fdv(rem, dq), xq = rem - y * QQ;
        qk_n[i] = n;
        if (MODE == F_FWD) {
          qk_hb[i] = y * st - pd;
          qk_wb[i] = xq * st - pd;
        } else {  // DGRAD: (h + pad, w + pad) of the input pixel
          qk_hb[i] = (o.nph == 4 ? 2 * y + o.pa : y) + pd;
          qk_wb[i] = (o.nph == 4 ? 2 * xq + o.pb : xq) + pd;
        }
      } else {
        qk_n[i] = -1;
        qk_hb[i] = qk_wb[i] = 0;
      }
    }
  } else {
    qm_kp = tid % (16 / KUQ);
    qm_rg = tid / (16 / KUQ);
    const int q = o.q0 + 4 * qm_rg;
    qm_ok = q < o.Qd;
    if (qm_ok) {
      const int tap = q / C;
      qm_c = q - tap * C;
      qm_r = tap / S;
      qm_s = tap - qm_r * S;
    }
  }
  if (xf) __syncthreads();
  if constexpr (MODE == F_WGRAD) {
    if (xf && qm_ok) {
#pragma unroll
      for (int v = 0; v < 4; ++v) { qm_sc[v] = xform[qm_c + v]; qm_sh[v] = xform[512 + qm_c + v]; }
    }
  }
  const FDiv dpix = mk_fdiv((uint32_t)(P * Q)), dpq1 = mk_fdiv((uint32_t)Q);

  // ----------------------------------------------------------- global -> registers (step kt)
  // Raw buffer loads through per-group descriptors: an invalid element (padding tap, tile
  // overhang, past the last reduction index) gets an offset beyond the descriptor's range and
  // reads as zero — no branches around the loads. The operand-side BN is applied at LDS-store
  // time (after the step's MFMAs), so it never waits on the loads it transforms.
  constexpr unsigned OOB = 0xFFFFFFF0u;
  const __amdgpu_buffer_rsrc_t rX = __builtin_amdgcn_make_buffer_rsrc(
      (void*)X, 0, (int)((long long)a.N * H * W * C * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t rW = __builtin_amdgcn_make_buffer_rsrc(
      (void*)Wt, 0, (int)((long long)K * a.R * S * C * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t rD = __builtin_amdgcn_make_buffer_rsrc(
      (void*)DY, 0, (int)((long long)a.N * P * Q * K * 4), 0x00020000);
  auto bload = [&](const __amdgpu_buffer_rsrc_t& rs, unsigned off) -> float4 {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
    return __builtin_bit_cast(float4, v);
  };
  // PF register sets of prefetched operands (PF = F32_PREFETCH, 2 or 3): the loads of step kt + PF
  // are issued while step kt computes and steps kt + 1 .. kt + PF - 1 wait in the other sets to be
  // stored — PF steps of MFMA work cover the load latency (one step of the X6 engine's MFMAs does
  // not cover an L2 miss under load).
  constexpr int PF = F32_PREFETCH;
  float4 rpA[2], rqA[2], rpB[2], rqB[2], rpC[2], rqC[2];
  bool qvA[2] = {false, false}, qvB[2] = {false, false}, qvC[2] = {false, false};  // real (in-image) X data
  auto load_step = [&](int kt, float4 (&rp)[2], float4 (&rq)[2], bool (&qv)[2]) {
    const int kk0 = kt * FBK;
    // P operand
    if constexpr (MODE == F_FWD) {
#pragma unroll
      for (int i = 0; i < UPK; ++i) {
        const int p = o.p0 + pk_row[i];
        rp[i] = bload(rW, p < o.Pd ? (unsigned)(p * o.Kr + kk0 + 4 * pk_ch[i]) * 4u : OOB);
      }
    } else if constexpr (MODE == F_DGRAD) {
      const int tap = kk0 / K, k0 = kk0 - tap * K;
      const int ir = tap / o.Sn, is = tap - ir * o.Sn;
      const int r = o.r0 + (st == 2 ? 2 : 1) * ir, s = o.s0 + (st == 2 ? 2 : 1) * is;
      const int c = o.p0 + 4 * pm_rg;
#pragma unroll
      for (int j = 0; j < KUP; ++j) {
        const int k = k0 + pm_kp * KUP + j;
        rp[j] = bload(rW, c < C ? (unsigned)(((k * a.R + r) * S + s) * C + c) * 4u : OOB);
      }
    } else {  // WGRAD: dY rows = channels k
      const int kch = o.p0 + 4 * pm_rg;
#pragma unroll
      for (int j = 0; j < KUP; ++j) {
        const int pix = kk0 + pm_kp * KUP + j;
        rp[j] = bload(rD, (pix < o.Kr && kch < K) ? (unsigned)(pix * K + kch) * 4u : OOB);
      }
    }
    // Q operand
    if constexpr (MODE == F_FWD) {
      const int tap = kk0 / C, c0 = kk0 - tap * C;
      const int r = tap / S, s = tap - r * S;
#pragma unroll
      for (int i = 0; i < UQK; ++i) {
        const int h = qk_hb[i] + r, w = qk_wb[i] + s;
        const bool ok = qk_n[i] >= 0 && (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
        qv[i] = ok;
        rq[i] = bload(rX, ok ? (unsigned)(((qk_n[i] * H + h) * W + w) * C + c0 + 4 * qk_ch[i]) * 4u : OOB);
      }
    } else if constexpr (MODE == F_DGRAD) {
      const int tap = kk0 / K, k0 = kk0 - tap * K;
      const int ir = tap / o.Sn, is = tap - ir * o.Sn;
      const int r = o.r0 + (st == 2 ? 2 : 1) * ir, s = o.s0 + (st == 2 ? 2 : 1) * is;
#pragma unroll
      for (int i = 0; i < UQK; ++i) {
        int ho = qk_hb[i] - r, wo = qk_wb[i] - s;
        bool hit = true;
        if (st == 2) {
          ho >>= 1;  // exact: the phase's taps keep (h + pad - r) even
          wo >>= 1;
        } else if (st > 2) {  // unphased: only the taps that land on an output position
          hit = ho >= 0 && wo >= 0 && ho % st == 0 && wo % st == 0;
          ho /= st;
          wo /= st;
        }
        const bool ok = hit && qk_n[i] >= 0 && (unsigned)ho < (unsigned)P && (unsigned)wo < (unsigned)Q;
        rq[i] = bload(rD, ok ? (unsigned)(((qk_n[i] * P + ho) * Q + wo) * K + k0 + 4 * qk_ch[i]) * 4u : OOB);
      }
    } else {  // WGRAD: X rows = (r, s, c)
#pragma unroll
      for (int j = 0; j < KUQ; ++j) {
        const int pix = kk0 + qm_kp * KUQ + j;
        const int n = fdv(pix, dpix), rem = pix - n * P * Q;
        const int ho = fdv(rem, dpq1), wo = rem - ho * Q;
        const int h = ho * st - pd + qm_r, w = wo * st - pd + qm_s;
        const bool ok = qm_ok && pix < o.Kr && (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
        qv[j] = ok;
        rq[j] = bload(rX, ok ? (unsigned)(((n * H + h) * W + w) * C + qm_c) * 4u : OOB);
      }
    }
  };
  // operand-side BN of the X operand (FWD / WGRAD): relu(x * scale + shift) on real pixels only
  auto xform4 = [&](float4 v, const float* sc, const float* sh) {
    v.x = v.x * sc[0] + sh[0];
    v.y = v.y * sc[1] + sh[1];
    v.z = v.z * sc[2] + sh[2];
    v.w = v.w * sc[3] + sh[3];
    if (xrelu) { v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f); }
    return v;
  };
  // ----------------------------------------------------------- registers -> LDS image
  auto store_mn = [&](float* img, int rg, int kp, int KU, const float4* v) {
#pragma unroll
    for (int j4 = 0; j4 < 4; ++j4) {
      const int row = 4 * rg + j4;
      const int kk = kp * KU;
      float* d = img + row * 16 + (((kk >> 2) ^ fswz(row)) << 2) + (kk & 3);
      const float e0 = j4 == 0 ? v[0].x : j4 == 1 ? v[0].y : j4 == 2 ? v[0].z : v[0].w;
      if (KU == 2) {
        const float e1 = j4 == 0 ? v[1].x : j4 == 1 ? v[1].y : j4 == 2 ? v[1].z : v[1].w;
        *(float2*)d = make_float2(e0, e1);
      } else {
        *d = e0;
      }
    }
  };
  // X6: registers -> split LDS image (see split3 / x6_off)
  auto store_k6 = [&](float* img, int row, int ch, float4 v) {
    s4v h, m, l;
    split3(v, h, m, l);
    *(s8v*)(img + x6_off(row, ch, 0)) = cat44(h, m);
    *(s8v*)(img + x6_off(row, ch, 1)) = cat44(l, h);
  };
  auto store_mn6 = [&](float* img, int rg, int kp, int KU, const float4* v) {
#pragma unroll
    for (int j4 = 0; j4 < 4; ++j4) {
      const int row = 4 * rg + j4;
      const int kk = kp * KU, ch = kk >> 2, pos = kk & 3;
      uint16_t* h0 = (uint16_t*)(img + x6_off(row, ch, 0)) + pos;  // (h | m) half
      uint16_t* h1 = (uint16_t*)(img + x6_off(row, ch, 1)) + pos;  // (l | h) half
      const float e0 = j4 == 0 ? v[0].x : j4 == 1 ? v[0].y : j4 == 2 ? v[0].z : v[0].w;
      uint16_t ah, am, al;
      split1(e0, ah, am, al);
      if (KU == 2) {
        const float e1 = j4 == 0 ? v[1].x : j4 == 1 ? v[1].y : j4 == 2 ? v[1].z : v[1].w;
        uint16_t bh, bm, bl;
        split1(e1, bh, bm, bl);
        *(uint32_t*)h0 = (uint32_t)ah | ((uint32_t)bh << 16);
        *(uint32_t*)(h0 + 4) = (uint32_t)am | ((uint32_t)bm << 16);
        *(uint32_t*)h1 = (uint32_t)al | ((uint32_t)bl << 16);
        *(uint32_t*)(h1 + 4) = (uint32_t)ah | ((uint32_t)bh << 16);
      } else {
        h0[0] = ah;
        h0[4] = am;
        h1[0] = al;
        h1[4] = ah;
      }
    }
  };
  auto store_step = [&](int buf, int kt, float4 (&rp)[2], float4 (&rq)[2], const bool (&qv)[2]) {
    float* Ps = smem + buf * (SP + SQ);
    float* Qs = Ps + SP;
    if constexpr (MODE == F_FWD) {
#pragma unroll
      for (int i = 0; i < UPK; ++i) {
        if constexpr (X6) store_k6(Ps, pk_row[i], pk_ch[i], rp[i]);
        else *(float4*)(Ps + lds_off(pk_row[i], pk_ch[i])) = rp[i];
      }
    } else {
      if constexpr (X6) store_mn6(Ps, pm_rg, pm_kp, KUP, rp);
      else store_mn(Ps, pm_rg, pm_kp, KUP, rp);
    }
    if constexpr (MODE == F_FWD) {
      if (xf) {
        const int kk0 = kt * FBK, c0 = kk0 - (kk0 / C) * C;
#pragma unroll
        for (int i = 0; i < UQK; ++i) {
          const int c = c0 + 4 * qk_ch[i];
          if (qv[i]) rq[i] = xform4(rq[i], xform + c, xform + 512 + c);
        }
      }
    } else if constexpr (MODE == F_WGRAD) {
      if (xf) {
#pragma unroll
        for (int j = 0; j < KUQ; ++j)
          if (qv[j]) rq[j] = xform4(rq[j], qm_sc, qm_sh);
      }
    }
    if constexpr (MODE != F_WGRAD) {
#pragma unroll
      for (int i = 0; i < UQK; ++i) {
        if constexpr (X6) store_k6(Qs, qk_row[i], qk_ch[i], rq[i]);
        else *(float4*)(Qs + lds_off(qk_row[i], qk_ch[i])) = rq[i];
      }
    } else {
      if constexpr (X6) store_mn6(Qs, qm_rg, qm_kp, KUQ, rq);
      else store_mn(Qs, qm_rg, qm_kp, KUQ, rq);
    }
  };

  f4v acc[TP][TQ];
#pragma unroll
  for (int i = 0; i < TP; ++i)
#pragma unroll
    for (int j = 0; j < TQ; ++j) acc[i][j] = (f4v){0.f, 0.f, 0.f, 0.f};

  auto step = [&](int kt, float4 (&cp)[2], float4 (&cq)[2], bool (&cv)[2], float4 (&np)[2],
                  float4 (&nq)[2], bool (&nv)[2]) {
    // cp/cq/cv: step kt + 1 (loaded PF - 1 iterations ago); np/nq/nv receive step kt + PF
    const int cur = (kt - kt0) & 1;
    if (kt + PF < kt1) load_step(kt + PF, np, nq, nv);
    const float* Ps = smem + cur * (SP + SQ);
    const float* Qs = Ps + SP;
    if constexpr (X6) {
      s8v a0[TP], a1[TP], b0[TQ], b1[TQ];
#pragma unroll
      for (int ti = 0; ti < TP; ++ti) {
        const int R = wp * WP + ti * 16 + (lane & 15);
        a0[ti] = *(const s8v*)(Ps + x6_off(R, lane >> 4, 0));
        a1[ti] = *(const s8v*)(Ps + x6_off(R, lane >> 4, 1));
      }
#pragma unroll
      for (int tj = 0; tj < TQ; ++tj) {
        const int R = wq * WQ + tj * 16 + (lane & 15);
        b0[tj] = *(const s8v*)(Qs + x6_off(R, lane >> 4, 0));
        b1[tj] = *(const s8v*)(Qs + x6_off(R, lane >> 4, 1));
      }
#pragma unroll
      for (int ti = 0; ti < TP; ++ti)
#pragma unroll
        for (int tj = 0; tj < TQ; ++tj) {
          f4v c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[ti], b0[tj], (f4v){0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[ti], b1[tj], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[ti], b0[tj], c, 0, 0, 0);
          // four scalar v_add_f32 (this file builds with -fno-slp-vectorize): a packed
          // v_pk_add_f32 issued beside MFMAs costs more than two plain adds
#pragma unroll
          for (int v = 0; v < 4; ++v) acc[ti][tj][v] = acc[ti][tj][v] + c[v];
        }
    } else {
      float4 af[TP], bfr[TQ];
#pragma unroll
      for (int ti = 0; ti < TP; ++ti)
        af[ti] = *(const float4*)(Ps + lds_off(wp * WP + ti * 16 + (lane & 15), lane >> 4));
#pragma unroll
      for (int tj = 0; tj < TQ; ++tj)
        bfr[tj] = *(const float4*)(Qs + lds_off(wq * WQ + tj * 16 + (lane & 15), lane >> 4));
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
        for (int ti = 0; ti < TP; ++ti)
#pragma unroll
          for (int tj = 0; tj < TQ; ++tj) {
            const float av = s4 == 0 ? af[ti].x : s4 == 1 ? af[ti].y : s4 == 2 ? af[ti].z : af[ti].w;
            const float bv = s4 == 0 ? bfr[tj].x : s4 == 1 ? bfr[tj].y : s4 == 2 ? bfr[tj].z : bfr[tj].w;
            acc[ti][tj] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[ti][tj], 0, 0, 0);
          }
    }
    if (kt + 1 < kt1) store_step(cur ^ 1, kt + 1, cp, cq, cv);
    __syncthreads();
  };
  if (kt0 < kt1) {
    load_step(kt0, rpA, rqA, qvA);
    if (kt0 + 1 < kt1) load_step(kt0 + 1, rpB, rqB, qvB);
    if constexpr (PF == 3) {
      if (kt0 + 2 < kt1) load_step(kt0 + 2, rpC, rqC, qvC);
    }
    store_step(0, kt0, rpA, rqA, qvA);
    __syncthreads();
    if constexpr (PF == 3) {
      // set of step k = (k - kt0) % 3: A, B, C
      for (int kt = kt0; kt < kt1; kt += 3) {
        step(kt, rpB, rqB, qvB, rpA, rqA, qvA);
        if (kt + 1 < kt1) step(kt + 1, rpC, rqC, qvC, rpB, rqB, qvB);
        if (kt + 2 < kt1) step(kt + 2, rpA, rqA, qvA, rpC, rqC, qvC);
      }
    } else {
      for (int kt = kt0; kt < kt1; kt += 2) {
        step(kt, rpB, rqB, qvB, rpA, rqA, qvA);
        if (kt + 1 < kt1) step(kt + 1, rpA, rqA, qvA, rpB, rqB, qvB);
      }
    }
  }

  if (split_store) {
    // raw partial sums of this split slice: FWD / DGRAD [split][G][nph][Qd_max][Pd]; WGRAD [split][G][Pd][Qd]
#pragma unroll
    for (int ti = 0; ti < TP; ++ti)
#pragma unroll
      for (int tj = 0; tj < TQ; ++tj) {
        const int q = o.q0 + wq * WQ + tj * 16 + (lane & 15);
        const int p = o.p0 + wp * WP + ti * 16 + 4 * (lane >> 4);
        if (q >= o.Qd || p >= o.Pd) continue;
        if constexpr (MODE == F_WGRAD) {
          float* d = a.partial + ((long long)o.split * a.G + g) * o.Pd * o.Qd;
#pragma unroll
          for (int v = 0; v < 4; ++v)
            if (p + v < o.Pd) d[(long long)(p + v) * o.Qd + q] = acc[ti][tj][v];
        } else {
          const long long qmax = (long long)a.slots / o.nph * BQ;  // rows per phase (tile-padded)
          float* d = a.partial + (((long long)o.split * a.G + g) * o.nph + o.phase) * qmax * o.Pd;
          *(float4*)(d + (long long)q * o.Pd + p) = make_float4(acc[ti][tj][0], acc[ti][tj][1],
                                                                acc[ti][tj][2], acc[ti][tj][3]);
        }
      }
    if (a.tickets) {
      // the last slice to arrive at this (group, phase, tile) folds all slices, in slice order, and
      // runs the epilogue (no reduce / epilogue launch): the partial stores are released
      // device-wide before the arrival counts, and acquired (L1 / L2 invalidated) by the folding
      // workgroup after it sees the count complete
      __threadfence();
      __syncthreads();
      int* const last = (int*)smem;
      int* const ticket = a.tickets + ((long long)g * o.nph + o.phase) * gx + bx;
      if (tid == 0) *last = atomicAdd(ticket, 1) == o.nsplit - 1;
      __syncthreads();
      if (!*last) return;
      __threadfence();
      if constexpr (MODE != F_WGRAD) {
        // the split-K epilogue kernel's fold (convf32_splitk_epilogue), in this tile's registers
        const long long qmax = (long long)a.slots / o.nph * BQ;
        const long long slice = (long long)a.G * o.nph * qmax * o.Pd;
        const float* base = a.partial + ((long long)g * o.nph + o.phase) * qmax * o.Pd;
#pragma unroll
        for (int ti = 0; ti < TP; ++ti)
#pragma unroll
          for (int tj = 0; tj < TQ; ++tj) {
            const int q = o.q0 + wq * WQ + tj * 16 + (lane & 15);
            const int p = o.p0 + wp * WP + ti * 16 + 4 * (lane >> 4);
            f4v sm = (f4v){0.f, 0.f, 0.f, 0.f};
            if (q < o.Qd && p < o.Pd) {
              const float* src = base + (long long)q * o.Pd + p;
              for (int k = 0; k < o.nsplit; ++k) {
                const float4 v = *(const float4*)(src + k * slice);
                sm[0] += v.x; sm[1] += v.y; sm[2] += v.z; sm[3] += v.w;
              }
            }
            acc[ti][tj] = sm;
          }
        __syncthreads();  // the flag word in smem is epilogue scratch from here on
        if (tid == 0) *ticket = 0;
        fepi<MODE, BP, BQ, Lay16<BP, BQ>>(a, o, acc, smem);
        return;
      } else {
        const long long per = (long long)o.Pd * o.Qd;
        const float* src = a.partial + (long long)g * per;
        float* dst = a.out + (long long)g * a.out_gs;
        for (int e = tid; e < BP * (BQ / 4); e += 256) {
          const int p = o.p0 + e / (BQ / 4), q = o.q0 + 4 * (e % (BQ / 4));
          if (p >= o.Pd || q >= o.Qd) continue;
          const long long off = (long long)p * o.Qd + q;
          float4 sum = make_float4(0.f, 0.f, 0.f, 0.f);
          for (int k = 0; k < o.nsplit; ++k) {
            const float4 v = *(const float4*)(src + (long long)k * a.G * per + off);
            sum.x += v.x; sum.y += v.y; sum.z += v.z; sum.w += v.w;
          }
          float4 b = a.accumulate ? *(const float4*)(dst + off) : make_float4(0.f, 0.f, 0.f, 0.f);
          b.x += a.gscale * sum.x; b.y += a.gscale * sum.y; b.z += a.gscale * sum.z; b.w += a.gscale * sum.w;
          *(float4*)(dst + off) = b;
        }
        if (tid == 0) *ticket = 0;  // ready for the next launch (and graph replay)
      }
    }
    return;
  }
  fepi<MODE, BP, BQ, Lay16<BP, BQ>>(a, o, acc, smem);
}

// WGRAD split-K: out = (accumulate ? out : 0) + gscale * sum_k partial[k] (slice order).
// V floats per thread (4: float4 lanes for big outputs; 1: small outputs, e.g. a 64-channel 3x3
// dW at one client, 36,864 floats over 128 slices, which as float4 threads filled only 36
// workgroups and ran 30-70 us latency-bound). The slice loads are issued 8 at a time ahead of the
// adds, which still run in slice order: the sum is bitwise the sequential one.
template <int V>
__global__ __launch_bounds__(256) void convf32_wgrad_reduce(const float* __restrict__ part, float* out,
                                                            long long out_gs, int G, long long nv,
                                                            int splits, int accumulate, float gscale) {
  typedef float vec __attribute__((ext_vector_type(V)));
  const long long per = nv * V;
  GSTRIDE_LOOP(t, (long long)G * nv) {
    const long long g = t / nv, i = (t - g * nv) * V;
    vec s = (vec)(0.f);
    const float* src = part + g * per + i;
    const long long sstride = (long long)G * per;
    int k = 0;
    for (; k + 8 <= splits; k += 8) {
      vec v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = *(const vec*)(src + (long long)(k + j) * sstride);
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[j];
    }
    for (; k < splits; ++k) s += *(const vec*)(src + (long long)k * sstride);
    float* d = out + g * out_gs + i;
    vec b = accumulate ? *(const vec*)d : (vec)(0.f);
    b += gscale * s;
    *(vec*)d = b;
  }
}

static void launch_wgrad_reduce(const float* part, float* out, long long out_gs, int G, long long n, int splits,
                                int accumulate, float gscale, hipStream_t s) {
  // float4 lanes once that still gives >= 2 workgroups per CU, scalar lanes below
  // (DDL_WGRAD_REDUCE_V4_MIN overrides the float4 threshold, in float4 lanes: A/B timing)
  static const long long v4_min = [] {
    const char* e = getenv("DDL_WGRAD_REDUCE_V4_MIN");
    return e ? atoll(e) : 512LL * 256;
  }();
  if ((long long)G * (n / 4) >= v4_min)
    hipLaunchKernelGGL(convf32_wgrad_reduce<4>, dim3(grid_for((long long)G * (n / 4), 256)), dim3(256), 0, s, part,
                       out, out_gs, G, n / 4, splits, accumulate, gscale);
  else
    hipLaunchKernelGGL(convf32_wgrad_reduce<1>, dim3(grid_for((long long)G * n, 256)), dim3(256), 0, s, part, out,
                       out_gs, G, n, splits, accumulate, gscale);
}

// the same fold for other WGRAD producers of [split][G][Pd][Qd] slices (conv_x6hw.hip)
DDL_API int ddl_convf32_wgrad_reduce(const float* part, float* out, long long out_gs, int G, long long n, int splits,
                                     int accumulate, float gscale, hipStream_t s) {
  if (n % 4) return (int)hipErrorInvalidValue;
  launch_wgrad_reduce(part, out, out_gs, G, n, splits, accumulate, gscale, s);
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------------------------ launchers
static void fdims(const ConvF32Args& a, int mode, long long& Pd, long long& Qd, long long& Qmax, long long& Kr,
                  int& nph) {
  nph = (mode == F_DGRAD && a.stride == 2) ? 4 : 1;
  if (mode == F_FWD) { Pd = a.K; Qd = Qmax = (long long)a.N * a.P * a.Q; Kr = (long long)a.R * a.S * a.C; }
  else if (mode == F_DGRAD) {
    Pd = a.C;
    const int Hs = nph == 4 ? (a.H + 1) >> 1 : a.H, Ws = nph == 4 ? (a.W + 1) >> 1 : a.W;
    Qd = Qmax = (long long)a.N * Hs * Ws;
    Kr = (long long)a.R * a.S * a.K;
  } else { Pd = a.K; Qd = Qmax = (long long)a.R * a.S * a.C; Kr = (long long)a.N * a.P * a.Q; }
}

// slots per group of the stats / BN-reduce buffer this launch writes (tile config cfg)
DDL_API long long ddl_convf32_slots(const ConvF32Args* ap, int mode, int cfg) {
  long long Pd, Qd, Qmax, Kr;
  int nph;
  fdims(*ap, mode, Pd, Qd, Qmax, Kr, nph);
  const int bq = ((cfg >> 8) & 0xff) * 16;
  if (bq <= 0) return -1;
  return nph * ((Qmax + bq - 1) / bq);
}

// floats of split-K workspace a launch needs (0: none)
DDL_API long long ddl_convf32_workspace(const ConvF32Args* ap, int mode, int cfg) {
  if (ap->split_k <= 1) return 0;
  long long Pd, Qd, Qmax, Kr;
  int nph;
  fdims(*ap, mode, Pd, Qd, Qmax, Kr, nph);
  const int bq = ((cfg >> 8) & 0xff) * 16;
  if (mode == F_WGRAD) return (long long)ap->split_k * ap->G * Pd * Qd;
  const long long qm = (Qmax + bq - 1) / bq * bq;
  return (long long)ap->split_k * ap->G * nph * qm * Pd;
}

template <int MODE, int BP, int BQ, int X6>
static int launch_tile(ConvF32Args a, hipStream_t s) {
  long long Pd, Qd, Qmax, Kr;
  int nph;
  fdims(a, MODE, Pd, Qd, Qmax, Kr, nph);
  const long long ntp = (Pd + BP - 1) / BP, ntq = (Qmax + BQ - 1) / BQ;
  a.slots = (int)(nph * ntq);
  const int split = a.split_k < 1 ? 1 : a.split_k;
  a.split_k = split;
  if (split > 1) {
    const long long need = MODE == F_WGRAD ? (long long)split * a.G * Pd * Qd
                                           : (long long)split * a.G * nph * ntq * BQ * Pd;
    if (!a.partial || need > a.partial_cap) return (int)hipErrorInvalidValue;
  }
  const dim3 grid((unsigned)(ntp * ntq), (unsigned)(nph * split), (unsigned)a.G);
  if (split == 1 || (long long)a.G * nph * ntp * ntq > a.tickets_cap) a.tickets = nullptr;
  hipLaunchKernelGGL((convf32_kernel<MODE, BP, BQ, X6>), grid, dim3(256), 0, s, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || split == 1 || a.tickets) return (int)e;
  if (MODE == F_WGRAD) {
    launch_wgrad_reduce((const float*)a.partial, a.out, a.out_gs, a.G, Pd * Qd, split, a.accumulate, a.gscale, s);
  } else {
    hipLaunchKernelGGL((convf32_splitk_epilogue<MODE, BP, BQ>), dim3((unsigned)(ntp * ntq), nph, a.G),
                       dim3(256), 0, s, a);
  }
  return (int)hipGetLastError();
}

// cfg = bp/16 | (bq/16) << 8 | x6 << 16 (x6: fp32 products on the bf16 MFMA, see split3)
template <int MODE, int X6>
static int launch_math(const ConvF32Args& a, int bp, int bq, hipStream_t s) {
  if (bp == 64 && bq == 64) return launch_tile<MODE, 64, 64, X6>(a, s);
  if (bp == 64 && bq == 128) return launch_tile<MODE, 64, 128, X6>(a, s);
  if (bp == 128 && bq == 64) return launch_tile<MODE, 128, 64, X6>(a, s);
  if (bp == 128 && bq == 128) return launch_tile<MODE, 128, 128, X6>(a, s);
  return (int)hipErrorInvalidValue;
}

template <int MODE>
static int launch_mode(const ConvF32Args& a, int cfg, hipStream_t s) {
  const int bp = (cfg & 0xff) * 16, bq = ((cfg >> 8) & 0xff) * 16;
  return (cfg >> 16) & 1 ? launch_math<MODE, 1>(a, bp, bq, s) : launch_math<MODE, 0>(a, bp, bq, s);
}

DDL_API int ddl_convf32(const ConvF32Args* ap, int mode, int cfg, hipStream_t s) {
  const ConvF32Args& a = *ap;
  if (a.G < 1 || a.N < 1 || a.C < 1 || a.K < 1 || a.stride < 1) return (int)hipErrorInvalidValue;
  if (a.C > 512 && a.in_scale) return (int)hipErrorInvalidValue;
  // per-group operands are addressed with 32-bit byte offsets (buffer descriptors)
  const long long lim = (1LL << 31) - 64;
  if ((long long)a.N * a.H * a.W * a.C * 4 > lim || (long long)a.K * a.R * a.S * a.C * 4 > lim ||
      (long long)a.N * a.P * a.Q * a.K * 4 > lim)
    return (int)hipErrorInvalidValue;
  if (mode == F_FWD) {
    if (a.C % 16 || a.K % 4) return (int)hipErrorInvalidValue;
    return launch_mode<F_FWD>(a, cfg, s);
  }
  if (mode == F_DGRAD) {
    if (a.K % 16 || a.C % 4) return (int)hipErrorInvalidValue;
    return launch_mode<F_DGRAD>(a, cfg, s);
  }
  if (mode == F_WGRAD) {
    if (a.C % 4 || a.K % 4) return (int)hipErrorInvalidValue;
    if (!a.accumulate && a.gscale != 1.f) return (int)hipErrorInvalidValue;
    return launch_mode<F_WGRAD>(a, cfg, s);
  }
  return (int)hipErrorInvalidValue;
}

DDL_API int ddl_convf32_args_size() { return (int)sizeof(ConvF32Args); }
