// Halo-staged X6 fp32 convolution: FWD and stride-1 DGRAD of "same" 3x3 (pad 1) and 1x1 convs,
// NHWC fp32, on v_mfma_f32_32x32x16_bf16.
//
// The reference trains in fp32 (stock nn.Conv2d, reference lab/tutorial_1a/hfl_complete.py:43-53;
// the ResNet-18 of the FedAvg headline config is built from the same layer). This is the hot path
// of the framework's fp32 mode for the layers it covers; conv_f32.hip keeps stride-2 DGRAD, WGRAD
// and any geometry this kernel declines (ddl_x6h_ok).
//
// Why a second fp32 kernel. The register-staged implicit GEMM of conv_f32.hip is issue-bound on
// the X6 engine: per 16-deep reduction step a wave spends ~350 issue cycles splitting freshly
// loaded operands into bf16 pieces (9 loads of every activation pixel, once per tap) beside the
// 384 cycles its 16x16x32 MFMAs hold the issue port, against 768 cycles of MFMA work. Here:
//   * 32x32x16 MFMAs hold the vector issue port 8 of 32 cycles instead of 8 of 16;
//   * the activation (Q) operand is staged ONCE per 16-channel chunk as a halo image — the tile's
//     output rows plus a one-pixel border, split into the X6 pieces once — and the R x S taps read
//     it as shifted windows (a uniform LDS offset per tap: the image is padded, not swizzled);
//   * the weight (P) operand arrives pre-split (ddl_x6_split_weights: 8 bytes per element, the
//     exact LDS operand image) and is DMA'd global -> LDS (no VGPRs, no VALU work).
// Per tap-step a 64x64 wave tile issues 24 MFMAs (768 cycles) beside 64 accumulator adds,
// 16 fragment reads and 4 weight DMA pieces; the halo split (~1.5 loads per thread per step for a
// 3x3 conv) is amortised over the 9 taps.
//
// Tile: 4 waves (2 x 2) over BP output channels x 128 output pixels. The 128 pixels are TR = 128/OW
// consecutive output rows: within one image (TR <= OH) or TR/OH whole images (OH < TR); each
// image segment of the tile has its own (rows + R - 1) x (OW + S - 1) halo. Reduction order: 16
// channel chunk (outer) x tap (inner); split-K slices split the chunks.
// Deterministic: fixed reduction order, per-step IEEE accumulation of the three-MFMA chains (the
// bf16 MFMA's own accumulation is not round-to-nearest, see conv_f32.hip), plain stores only.
#include "conv_f32_core.h"

namespace {

constexpr int BQH = 128;    // output pixels per tile
constexpr int HSTR = 144;   // halo image bytes per pixel: 16 channels x 8 B + 16 B pad (bank spread)
constexpr int PSTR = 128;   // weight image bytes per row (16 channels x 8 B, 16-B granule XOR swizzle)
constexpr int HPMAX = 288;  // halo pixels per tile (4 x 4 images: 8 x 6 x 6)
constexpr unsigned OOB = 0xFFFFFFF0u;

struct HaloGeo {
  int lgW;      // log2 OW (output pixels per row)
  int SR;       // output rows per image segment of the tile
  int HR, HC;   // halo rows / cols per segment
  int HP;       // halo pixels per tile
  int OH;       // output rows per image
  int SH, SW, SC;  // source (X for FWD, dY for DGRAD) height, width, channels
  int Pd;       // output channels (K for FWD, C for DGRAD)
};

typedef float f16v __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float4 bload4(const __amdgpu_buffer_rsrc_t& rs, unsigned off) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
}

template <int MODE, int BP, int RS>
__global__ __launch_bounds__(256, 2) void convx6h_kernel(ConvF32Args a, HaloGeo hg) {
  constexpr int T = RS * RS;                 // taps
  constexpr int PD = (RS - 1) / 2;           // pad
  constexpr int WP = BP / 2, TI = WP / 32, TJ = 2;
  constexpr int UP = BP / 32;                // weight LDS-DMA pieces (1 KiB) per wave per step
  constexpr int NUH = (HPMAX * 4 + 255) / 256;  // halo units (pixel x 4-channel chunk) per thread
  constexpr int PIMG = BP * PSTR;            // bytes per weight image
  constexpr bool XF_OK = MODE == F_FWD;
  __shared__ __attribute__((aligned(16))) char smem[2 * PIMG + HPMAX * HSTR];
  __shared__ float xform[XF_OK ? 1024 : 1];
  char* const pimg = smem;
  char* const himg = smem + 2 * PIMG;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wp = wid >> 1, wq = wid & 1;
  const int gx = gridDim.x, gy = gridDim.y, gz = gridDim.z;
  const int lin = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  const int u = xcd_remap(lin, gx * gy * gz);
  const int bx = u % gx, by = (u / gx) % gy, g = u / (gx * gy);
  const FGeo o = fgeo<MODE, BP, BQH>(a, bx, by, g, gy);
  const bool split_store = a.split_k > 1;
  if (o.q0 >= o.Qd || o.p0 >= o.Pd) {
    if (!split_store) fzero_slot<MODE, BP>(a, o);
    return;
  }
  const int SC = hg.SC, Pd = hg.Pd;
  const int ncc = SC >> 4;
  const int per = (ncc + o.nsplit - 1) / o.nsplit;
  const int cc0 = o.split * per, cc1 = min(ncc, cc0 + per);

  const bool xf = XF_OK && a.in_scale != nullptr;
  if constexpr (XF_OK) {
    if (xf) {
      for (int i = tid; i < SC; i += 256) {
        xform[i] = a.in_scale[(long long)g * SC + i];
        xform[512 + i] = a.in_shift[(long long)g * SC + i];
      }
    }
  }
  const bool xrelu = a.in_relu != 0;

  // ---------------------------------------------------------------- buffer descriptors
  const float* src = MODE == F_FWD ? a.x + (long long)g * a.x_gs : a.dy + (long long)g * a.dy_gs;
  const long long src_bytes = (long long)a.N * hg.SH * hg.SW * SC * 4;
  const __amdgpu_buffer_rsrc_t rS = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, (int)src_bytes, 0x00020000);
  const char* wsp = (const char*)a.wsplit + (long long)g * a.ws_gs;
  const __amdgpu_buffer_rsrc_t rW = __builtin_amdgcn_make_buffer_rsrc(
      (void*)wsp, 0, (int)((long long)Pd * T * SC * 8), 0x00020000);

  // ---------------------------------------------------------------- halo bookkeeping
  // unit i of this thread: halo pixel hp = uu >> 2, 4-channel chunk ch = uu & 3
  const int nunits = hg.HP * 4;
  const int t0 = o.q0 >> hg.lgW;  // first output row (over n, oh) of the tile
  unsigned hoff[NUH];             // source byte offset at chunk 0 (OOB: padding / beyond N)
  int hlds[NUH];                  // LDS byte offset of the unit (-1: no unit)
#pragma unroll
  for (int i = 0; i < NUH; ++i) {
    const int uu = tid + 256 * i;
    hoff[i] = OOB;
    hlds[i] = -1;
    if (uu < nunits) {
      const int hp = uu >> 2, ch = uu & 3;
      const int segpix = hg.HR * hg.HC;
      const int seg = hp / segpix, rem = hp - seg * segpix;
      const int hi = rem / hg.HC, hj = rem - hi * hg.HC;
      const int ts = t0 + seg * hg.SR;
      const int n = ts / hg.OH, r0 = ts - n * hg.OH;
      const int sr = r0 + hi - PD, sc = hj - PD;
      if (n < a.N && (unsigned)sr < (unsigned)hg.SH && (unsigned)sc < (unsigned)hg.SW)
        hoff[i] = (unsigned)((((long long)n * hg.SH + sr) * hg.SW + sc) * SC + ch * 4) * 4u;
      hlds[i] = hp * HSTR + ch * 32;
    }
  }
  float4 hreg[NUH];
  auto halo_load = [&](int cc) {
#pragma unroll
    for (int i = 0; i < NUH; ++i) hreg[i] = bload4(rS, hoff[i] == OOB ? OOB : hoff[i] + (unsigned)cc * 64u);
  };
  auto halo_store = [&](int cc) {
#pragma unroll
    for (int i = 0; i < NUH; ++i) {
      if (hlds[i] < 0) continue;
      float4 v = hreg[i];
      if constexpr (XF_OK) {
        if (xf && hoff[i] != OOB) {  // operand-side BN + ReLU on real pixels (padding stays 0)
          const int c = cc * 16 + ((tid + 256 * i) & 3) * 4;
          v.x = v.x * xform[c] + xform[512 + c];
          v.y = v.y * xform[c + 1] + xform[512 + c + 1];
          v.z = v.z * xform[c + 2] + xform[512 + c + 2];
          v.w = v.w * xform[c + 3] + xform[512 + c + 3];
          if (xrelu) { v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f); }
        }
      }
      s4v h, m, l;
      split3(v, h, m, l);
      *(s8v*)(himg + hlds[i]) = cat44(h, m);
      *(s8v*)(himg + hlds[i] + 16) = cat44(l, h);
    }
  };

  // ---------------------------------------------------------------- weight (P operand) staging
  // LDS-DMA (buffer_load ... lds, 1 KiB per wave-instruction, lane-linear destination): piece i of
  // wave wsc covers image bytes (wsc + 4 i) KiB = rows 8 (wsc + 4 i) .. +7; a lane fetches the
  // logical granule that the XOR swizzle places at its destination (gl = physical ^ swizzle).
  const int wsc = __builtin_amdgcn_readfirstlane(wid);
  unsigned woff[UP];
#pragma unroll
  for (int i = 0; i < UP; ++i) {
    const int row = (wsc + 4 * i) * 8 + (lane >> 3);
    const int gl = (lane & 7) ^ ((row >> 1) & 7);
    const int p = o.p0 + row;
    woff[i] = p < Pd ? (unsigned)((long long)p * T * SC * 8 + gl * 16) : OOB;
  }
  auto wload = [&](int buf, int cc, int t) {
    const int wtap = MODE == F_FWD ? t : T - 1 - t;  // DGRAD: the flipped kernel
    const unsigned add = (unsigned)(wtap * SC * 8 + cc * 128);
#pragma unroll
    for (int i = 0; i < UP; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rW, (__attribute__((address_space(3))) void*)(pimg + buf * PIMG + (wsc + 4 * i) * 1024), 16,
          woff[i] == OOB ? OOB : woff[i] + add, 0, 0, 0);
  };

  // ---------------------------------------------------------------- fragment addressing
  const int hh = lane >> 5;  // lane half: reduction values 4 * hh .. of each 8-deep k-group
  int aoff[TI][4];           // weight image byte offsets per (ti, granule pair index 2j + half)
#pragma unroll
  for (int ti = 0; ti < TI; ++ti) {
    const int row = wp * WP + ti * 32 + (lane & 31), sw = (row >> 1) & 7;
#pragma unroll
    for (int jh = 0; jh < 4; ++jh) {  // jh = 2 * j + half
      const int gl = 4 * (jh >> 1) + 2 * hh + (jh & 1);
      aoff[ti][jh] = row * PSTR + 16 * (gl ^ sw);
    }
  }
  int boff[TJ];  // halo image byte offsets of tap (0, 0)
#pragma unroll
  for (int tj = 0; tj < TJ; ++tj) {
    const int ql = wq * 64 + tj * 32 + (lane & 31);
    const int jj = ql & ((1 << hg.lgW) - 1), rowl = ql >> hg.lgW;
    const int seg = rowl / hg.SR, ii = rowl - seg * hg.SR;
    boff[tj] = ((seg * hg.HR + ii) * hg.HC + jj) * HSTR + hh * 32;
  }

  f16v acc[TI][TJ];
#pragma unroll
  for (int ti = 0; ti < TI; ++ti)
#pragma unroll
    for (int tj = 0; tj < TJ; ++tj) acc[ti][tj] = (f16v){};

  const int k0 = cc0 * T, k1 = cc1 * T;
  constexpr int HT = T >= 3 ? T - 3 : 0;  // tap at which the next chunk's halo loads are issued

  auto compute = [&](int buf, int t) {
    const char* P = pimg + buf * PIMG;
    const int dr = t / RS, ds = t - dr * RS;
    const int tapoff = (dr * hg.HC + ds) * HSTR;
    s8v a_hm[TI][2], a_lh[TI][2], b_hm[TJ][2], b_lh[TJ][2];
#pragma unroll
    for (int ti = 0; ti < TI; ++ti)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        a_hm[ti][j] = *(const s8v*)(P + aoff[ti][2 * j]);
        a_lh[ti][j] = *(const s8v*)(P + aoff[ti][2 * j + 1]);
      }
#pragma unroll
    for (int tj = 0; tj < TJ; ++tj)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const char* hb = himg + boff[tj] + tapoff + j * 64;
        b_hm[tj][j] = *(const s8v*)hb;
        b_lh[tj][j] = *(const s8v*)(hb + 16);
      }
#pragma unroll
    for (int ti = 0; ti < TI; ++ti)
#pragma unroll
      for (int tj = 0; tj < TJ; ++tj) {
        f16v c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_lh[ti][0], b_hm[tj][0], (f16v){}, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_hm[ti][0], b_lh[tj][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_hm[ti][0], b_hm[tj][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_lh[ti][1], b_hm[tj][1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_hm[ti][1], b_lh[tj][1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_hm[ti][1], b_hm[tj][1], c, 0, 0, 0);
#pragma unroll
        for (int v = 0; v < 16; ++v) acc[ti][tj][v] = acc[ti][tj][v] + c[v];
      }
  };

  if (k0 < k1) {
    // prologue: halo of chunk cc0 and the weights of step k0
    wload(0, cc0, 0);
    halo_load(cc0);
    halo_store(cc0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int cc = cc0, t = 0;
    for (int k = k0; k < k1; ++k) {
      const int buf = (k - k0) & 1;
      // step k + 1's weights into the other buffer (its last reader, step k - 1, is past the barrier)
      if (k + 1 < k1) wload(buf ^ 1, t == T - 1 ? cc + 1 : cc, t == T - 1 ? 0 : t + 1);
      if (t == HT && cc + 1 < cc1) halo_load(cc + 1);
      compute(buf, t);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (t == T - 1 && k + 1 < k1) {  // chunk boundary: every wave is done with this chunk's halo
        halo_store(cc + 1);
        __syncthreads();
      }
      if (++t == T) { t = 0; ++cc; }
    }
  }

  // ---------------------------------------------------------------- epilogue
  f4v quad[Lay32<BP, BQH>::NPQ][Lay32<BP, BQH>::NQ];
#pragma unroll
  for (int ti = 0; ti < TI; ++ti)
#pragma unroll
    for (int tj = 0; tj < TJ; ++tj)
#pragma unroll
      for (int gg = 0; gg < 4; ++gg)
        quad[ti * 4 + gg][tj] = (f4v){acc[ti][tj][4 * gg], acc[ti][tj][4 * gg + 1], acc[ti][tj][4 * gg + 2],
                                      acc[ti][tj][4 * gg + 3]};
  if (split_store) {
    // raw partial sums of this slice: [split][G][1][qmax][Pd] (the layout of conv_f32.hip)
    const long long qmax = (long long)a.slots * BQH;
    float* d = a.partial + ((long long)o.split * a.G + g) * qmax * Pd;
#pragma unroll
    for (int i = 0; i < Lay32<BP, BQH>::NPQ; ++i)
#pragma unroll
      for (int j = 0; j < Lay32<BP, BQH>::NQ; ++j) {
        const int q = o.q0 + wq * 64 + Lay32<BP, BQH>::qoff(j, lane);
        const int p = o.p0 + wp * WP + Lay32<BP, BQH>::poff(i, lane);
        if (q >= o.Qd || p >= Pd) continue;
        *(float4*)(d + (long long)q * Pd + p) = make_float4(quad[i][j][0], quad[i][j][1], quad[i][j][2], quad[i][j][3]);
      }
    return;
  }
  fepi<MODE, BP, BQH, Lay32<BP, BQH>>(a, o, quad, (float*)smem);
}

// Pre-split weights: FWD layout [G][K][T][C] (chunks of 4 input channels), DGRAD layout [G][C][T][K]
// (chunks of 4 output channels), 8 bytes per element: per 4-chunk (h0..h3 | m0..m3)(l0..l3 | h0..h3).
__global__ __launch_bounds__(256) void x6_split_weights_kernel(const float* __restrict__ w, char* out, int G, int K,
                                                               int T, int C, int layout, long long w_gs,
                                                               long long o_gs) {
  const long long per = (long long)K * T * C / 4;  // 4-chunks per group
  GSTRIDE_LOOP(t, (long long)G * per) {
    const long long g = t / per, e = t - g * per;
    float4 v;
    long long dst;
    if (layout == 0) {  // element (k, tap, c..c+3): contiguous in w
      v = *(const float4*)(w + g * w_gs + e * 4);
      dst = e * 4;
    } else {  // element (c, tap, k..k+3): w[k + i][tap][c]
      const int K4 = K / 4;
      const long long ct = e / K4;
      const int k = (int)(e - ct * K4) * 4;
      const int c = (int)(ct / T), tap = (int)(ct - (long long)c * T);
      const float* s = w + g * w_gs + ((long long)k * T + tap) * C + c;
      const long long ks = (long long)T * C;
      v = make_float4(s[0], s[ks], s[2 * ks], s[3 * ks]);
      dst = ((long long)c * T + tap) * K + k;
    }
    s4v h, m, l;
    split3(v, h, m, l);
    char* d = out + g * o_gs + dst * 8;
    *(s8v*)d = cat44(h, m);
    *(s8v*)(d + 16) = cat44(l, h);
  }
}

bool x6h_geo(const ConvF32Args& a, int mode, int bp, HaloGeo& h, int& rs) {
  if (mode != F_FWD && mode != F_DGRAD) return false;
  if (bp != 64 && bp != 128) return false;
  if (a.stride != 1 || a.R != a.S || (a.R != 1 && a.R != 3) || a.pad != (a.R - 1) / 2) return false;
  if (a.P != a.H || a.Q != a.W) return false;
  rs = a.R;
  const int OH = a.P, OW = a.Q;
  if (OW < 4 || OW > BQH || (OW & (OW - 1))) return false;
  int lg = 0;
  while ((1 << lg) < OW) ++lg;
  const int TR = BQH / OW;
  int SR;
  if (TR <= OH) {
    if (OH % TR) return false;
    SR = TR;
  } else {
    if (TR % OH) return false;
    SR = OH;
  }
  h.lgW = lg;
  h.SR = SR;
  h.HR = SR + a.R - 1;
  h.HC = OW + a.S - 1;
  h.HP = (TR / SR) * h.HR * h.HC;
  h.OH = OH;
  h.SH = a.H;
  h.SW = a.W;
  h.SC = mode == F_FWD ? a.C : a.K;
  h.Pd = mode == F_FWD ? a.K : a.C;
  if (h.HP > HPMAX || h.SC % 16 || h.Pd % 4) return false;
  if (mode == F_FWD && a.in_scale && a.C > 512) return false;
  if (mode == F_DGRAD && a.in_scale) return false;
  const long long lim = (1LL << 31) - 64;
  if ((long long)a.N * a.H * a.W * h.SC * 4 > lim || (long long)h.Pd * a.R * a.S * h.SC * 8 > lim) return false;
  return true;
}

template <int MODE, int BP, int RS>
int launch_x6h(ConvF32Args a, const HaloGeo& h, hipStream_t s) {
  const long long Pd = h.Pd, Qd = (long long)a.N * a.P * a.Q;
  const long long ntp = (Pd + BP - 1) / BP, ntq = (Qd + BQH - 1) / BQH;
  a.slots = (int)ntq;
  const int split = a.split_k < 1 ? 1 : a.split_k;
  a.split_k = split;
  if (split > 1) {
    const long long need = (long long)split * a.G * ntq * BQH * Pd;
    if (!a.partial || need > a.partial_cap) return (int)hipErrorInvalidValue;
  }
  const dim3 grid((unsigned)(ntp * ntq), (unsigned)split, (unsigned)a.G);
  hipLaunchKernelGGL((convx6h_kernel<MODE, BP, RS>), grid, dim3(256), 0, s, a, h);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || split == 1) return (int)e;
  hipLaunchKernelGGL((convf32_splitk_epilogue<MODE, BP, BQH>), dim3((unsigned)(ntp * ntq), 1, a.G), dim3(256), 0,
                     s, a);
  return (int)hipGetLastError();
}

template <int MODE>
int dispatch_x6h(const ConvF32Args& a, int bp, int rs, const HaloGeo& h, hipStream_t s) {
  if (rs == 3) return bp == 128 ? launch_x6h<MODE, 128, 3>(a, h, s) : launch_x6h<MODE, 64, 3>(a, h, s);
  return bp == 128 ? launch_x6h<MODE, 128, 1>(a, h, s) : launch_x6h<MODE, 64, 1>(a, h, s);
}

}  // namespace

// Can the halo kernel run this (mode, geometry) with BP = (cfg & 0xff) * 16?
DDL_API int ddl_x6h_ok(const ConvF32Args* ap, int mode, int cfg) {
  HaloGeo h;
  int rs;
  return x6h_geo(*ap, mode, (cfg & 0xff) * 16, h, rs) ? 1 : 0;
}

DDL_API int ddl_x6h(const ConvF32Args* ap, int mode, int cfg, hipStream_t s) {
  const ConvF32Args& a = *ap;
  HaloGeo h;
  int rs;
  const int bp = (cfg & 0xff) * 16;
  if (a.G < 1 || a.N < 1 || !a.wsplit || !x6h_geo(a, mode, bp, h, rs)) return (int)hipErrorInvalidValue;
  if (((cfg >> 8) & 0xff) * 16 != BQH) return (int)hipErrorInvalidValue;
  return mode == F_FWD ? dispatch_x6h<F_FWD>(a, bp, rs, h, s) : dispatch_x6h<F_DGRAD>(a, bp, rs, h, s);
}

// w [G][K][T][C] fp32 (group stride w_gs floats) -> out (group stride o_gs bytes, >= K*T*C*8)
DDL_API int ddl_x6_split_weights(const float* w, void* out, int G, int K, int T, int C, int layout,
                                 long long w_gs, long long o_gs, int pad_, hipStream_t s) {
  (void)pad_;
  if (G < 1 || K < 1 || T < 1 || C < 1 || (layout == 0 ? C % 4 : K % 4) || (w_gs % 4)) return (int)hipErrorInvalidValue;
  const long long work = (long long)G * K * T * C / 4;
  hipLaunchKernelGGL(x6_split_weights_kernel, dim3(grid_for(work, 256)), dim3(256), 0, s, w, (char*)out, G, K, T,
                     C, layout, w_gs, o_gs);
  return (int)hipGetLastError();
}
