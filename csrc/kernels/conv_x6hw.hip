// Halo-staged X6 WGRAD of stride-1 "same" 3x3 / 1x1 convolutions (fp32 operands on the bf16 MFMA).
//
// dW[k][r][s][c] = sum over output pixels q of dY[q][k] * X[q + (r - pd, s - pd)][c]. conv_f32.hip
// runs this as an implicit GEMM whose X operand rows are (tap, channel): every X value is loaded,
// split into its three bf16 pieces and transposed into LDS once PER TAP (9x), which makes that loop
// VALU-bound (~6 VALU per MFMA, MFMA busy 30-37 %, profiles/pmc_wgrad_r4.txt). Here a workgroup
// owns dW[k0:k0+64][all taps][c0:c0+32] and sweeps a slice of the pixel tiles; per tile of 128
// output pixels it stages
//   dY  [64 k][128 pixels]                        (planar h | m | l bf16, pixel-contiguous rows)
//   X   [32 c][tile rows + halo][tile cols + halo] (planar, one image row per LDS row)
// each ONCE (register transpose: a thread loads 8 pixels x 4 channels and writes each channel's 8
// pixels as one 16-byte LDS store per plane), and the 9 taps read shifted windows of the X image.
// MFMA v_mfma_f32_32x32x16_bf16 with the REDUCTION over pixels: lane l holds 8 consecutive pixels
// (l >> 5 selects which 8 of the step's 16) of row / column l & 31; a tap's window starts s
// elements into an LDS row, so its 16-byte reads are 2-byte aligned (gfx950 LDS serves them).
// Per 16-pixel step and (k block, tap): six piece products chained from zero, then ONE IEEE add
// into the fp32 accumulator (the halo FWD / DGRAD kernel's rounding discipline).
// 4 waves: wave w computes k block (w >> 1) (32 rows), all taps, over the even (w even) or odd
// pixel steps of every tile; the two halves are summed once at the end.
// Split-K over pixel tiles writes [split][G][K][R*S*C] partial slices for convf32_wgrad_reduce;
// unsplit launches apply out = (accumulate ? out : 0) + gscale * dW directly (direct SGD).
#include <cstdlib>

#include "ddl_common.h"
#include "conv_f32_core.h"

namespace {

typedef float f16v __attribute__((ext_vector_type(16)));  // 32x32 MFMA accumulator

constexpr int HW_BK = 64, HW_BC = 32, HW_TP = 128;  // k rows, channels, pixels per tile
constexpr int HW_KS = 136;                           // dY LDS row stride (elements): 272 B = 16 mod 256
constexpr unsigned HW_OOB = 0x80000000u;

struct HWGeo {
  int lgW;      // log2 output width (8..64)
  int SR;       // rows per image segment of a tile (min(128 / OW, OH))
  int NSEG;     // image segments per tile
  int HR, HCp;  // halo rows per segment (SR + R - 1), padded halo row length (elements, % 8 == 0)
  int CS;       // X LDS channel stride (elements)
  int ntile;    // pixel tiles per group
  int NUX;      // X staging units per thread
  int probe;    // timing probes (DDL_HW_PROBE, wrong results): 1 skip LDS staging, 2 skip MFMAs, 4 skip loads
};

// Prefetch loads straight into AGPRs (inline asm: the compiler neither sees nor waits on them).
// With compiler-visible loads the next tile's staging registers were copied into AGPRs right
// after issue to free VGPRs for the MFMA loop — a vmcnt wait that exposed the whole load latency
// at every tile (the DDL_HW_PROBE "no loads" probe ran 25 % faster). hw_wait() at the next tile's
// staging is the one wait, and pins every prefetch register behind it.
typedef int hw_rsrc __attribute__((ext_vector_type(4)));
__device__ __forceinline__ hw_rsrc hw_make_rsrc(const void* p, long long bytes) {
  const unsigned long long a = (unsigned long long)p;
  hw_rsrc r;
  r.x = (int)(unsigned)(a & 0xffffffffull);
  r.y = (int)(unsigned)((a >> 32) & 0xffffull);
  r.z = (int)bytes;
  r.w = 0x00020000;
  return r;
}
__device__ __forceinline__ void hw_load(f4v& d, const hw_rsrc& rs, unsigned off) {
  asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=a"(d) : "v"(off), "s"(rs) : "memory");
}

// 8 values -> the three bf16 planes of one 16-byte LDS row segment each
__device__ __forceinline__ void split8(const float (&v)[8], s8v& h, s8v& m, s8v& l) {
  s4v h0, m0, l0, h1, m1, l1;
  split3(make_float4(v[0], v[1], v[2], v[3]), h0, m0, l0);
  split3(make_float4(v[4], v[5], v[6], v[7]), h1, m1, l1);
  h = cat44(h0, h1);
  m = cat44(m0, m1);
  l = cat44(l0, l1);
}

template <int RS, int NUX>
__global__ __launch_bounds__(256, 1) void convx6hw_kernel(ConvF32Args a, HWGeo hg) {
  constexpr int T = RS * RS, PD = (RS - 1) / 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* const dyl = (bf16_t*)smem;                        // [3][64][HW_KS]
  bf16_t* const xl = dyl + 3 * HW_BK * HW_KS;               // [3][32][CS]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int OW = 1 << hg.lgW, TR = HW_TP >> hg.lgW;
  const int nct = a.C / HW_BC;
  const int k0 = (blockIdx.x / nct) * HW_BK, c0 = (blockIdx.x % nct) * HW_BC;
  const int split = blockIdx.y, nsplit = gridDim.y, g = blockIdx.z;
  const int per = (hg.ntile + nsplit - 1) / nsplit;
  const int t0 = split * per, t1 = min(hg.ntile, t0 + per);
  const int K = a.K, C = a.C, H = a.H, W = a.W;
  const long long npix = (long long)a.N * H * W;

  const hw_rsrc rD = hw_make_rsrc(a.dy + (long long)g * a.dy_gs, npix * K * 4);
  const hw_rsrc rX = hw_make_rsrc(a.x + (long long)g * a.x_gs, npix * C * 4);

  // ---- dY unit: channels k0 + 4 * (tid & 15) .. + 3, tile pixels 8 * (tid >> 4) .. + 7
  const int dkc = tid & 15, dpg = tid >> 4;
  // ---- X units: channels c0 + 4 * cg, halo row xr (over segments), halo columns 8 * xc .. + 7
  const int ncol8 = hg.HCp >> 3;
  const int nxu = 8 * hg.NSEG * hg.HR * ncol8;
  // operand-side BN of X (relu(x * scale + shift) on real pixels)
  const bool xf = a.in_scale != nullptr;
  float4 xsc[NUX], xsh[NUX];
#pragma unroll
  for (int u = 0; u < NUX; ++u) {
    xsc[u] = make_float4(1.f, 1.f, 1.f, 1.f);
    xsh[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    const int uu = tid + 256 * u;
    if (xf && uu < nxu) {
      const long long cc = (long long)g * C + c0 + 4 * (uu & 7);
      xsc[u] = *(const float4*)(a.in_scale + cc);
      xsh[u] = *(const float4*)(a.in_shift + cc);
    }
  }

  // per X unit: halo segment, halo row within it, 8-column group (fixed for the kernel)
  int useg[NUX], uhr[NUX], uxc[NUX], uoff[NUX];  // uoff: LDS element offset of the unit's first channel
  bool uvalid[NUX];
#pragma unroll
  for (int u = 0; u < NUX; ++u) {
    const int uu = tid + 256 * u, rest = uu >> 3;
    const int xc = rest % ncol8, xrr = rest / ncol8;  // halo row over segments
    useg[u] = xrr / hg.HR;
    uhr[u] = xrr - useg[u] * hg.HR;
    uxc[u] = xc;
    uoff[u] = 4 * (uu & 7) * hg.CS + xrr * hg.HCp + 8 * xc;
    uvalid[u] = uu < nxu;
  }
  f4v rd[8], rx[NUX][8];
  unsigned xok[NUX];  // bit j: halo pixel j of the unit is a real input pixel
  auto load_tile = [&](int tile) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int p = tile * HW_TP + dpg * 8 + j;
      hw_load(rd[j], rD, p < npix ? (unsigned)((p * K + k0 + 4 * dkc) * 4) : HW_OOB);
    }
    // first output row of the tile over (n, oh): tile rows are whole image rows, one (uniform)
    // division per tile; a segment past the first is a whole image (seg * SR == seg * P)
    const int row0 = tile * TR;
    const int n0 = row0 / a.P, oh0 = row0 - n0 * a.P;
#pragma unroll
    for (int u = 0; u < NUX; ++u) {
      xok[u] = 0;
      const int n = n0 + useg[u];
      const int ih = oh0 + uhr[u] - PD;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int iw = 8 * uxc[u] + j - PD;
        const bool ok = uvalid[u] && n < a.N && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
        xok[u] |= (ok ? 1u : 0u) << j;
        hw_load(rx[u][j], rX, ok ? (unsigned)((((n * H + ih) * W + iw) * C + c0 + 4 * (tid & 7)) * 4) : HW_OOB);
      }
    }
  };
  // split the loaded dY tile into its bf16 planes (splitting the next tile between the two compute
  // halves of the current one, to overlap that VALU work with MFMAs, was measured slower: the
  // extra live registers push the accumulators through AGPR moves)...
  s8v sd[4][3], sx[NUX][4][3];  // sx: split at write time (registers)
  auto hw_wait = [&]() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("" : "+a"(rd[j]));
#pragma unroll
    for (int u = 0; u < NUX; ++u)
#pragma unroll
      for (int j = 0; j < 8; ++j) asm volatile("" : "+a"(rx[u][j]));
  };
  auto split_tile = [&]() {
    // dY: channel ch of the unit -> row k = 4 dkc + ch, pixels 8 dpg .. + 7
#pragma unroll
    for (int ch = 0; ch < 4; ++ch) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = ch == 0 ? rd[j].x : ch == 1 ? rd[j].y : ch == 2 ? rd[j].z : rd[j].w;
      split8(v, sd[ch][0], sd[ch][1], sd[ch][2]);
    }
  };
  // ... and write it to LDS once the previous tile's fragment reads are done
  auto write_tile = [&]() {
#pragma unroll
    for (int ch = 0; ch < 4; ++ch) {
      bf16_t* d = dyl + (4 * dkc + ch) * HW_KS + 8 * dpg;
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) *(s8v*)(d + pl * HW_BK * HW_KS) = sd[ch][pl];
    }
#pragma unroll
    for (int u = 0; u < NUX; ++u) {
#pragma unroll
      for (int ch = 0; ch < 4; ++ch) {
        const float sc = ch == 0 ? xsc[u].x : ch == 1 ? xsc[u].y : ch == 2 ? xsc[u].z : xsc[u].w;
        const float sh = ch == 0 ? xsh[u].x : ch == 1 ? xsh[u].y : ch == 2 ? xsh[u].z : xsh[u].w;
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float e = ch == 0 ? rx[u][j].x : ch == 1 ? rx[u][j].y : ch == 2 ? rx[u][j].z : rx[u][j].w;
          if (xf && ((xok[u] >> j) & 1u)) {
            e = e * sc + sh;
            if (a.in_relu) e = fmaxf(e, 0.f);
          }
          v[j] = e;
        }
        split8(v, sx[u][ch][0], sx[u][ch][1], sx[u][ch][2]);
      }
    }
#pragma unroll
    for (int u = 0; u < NUX; ++u) {
      if (!uvalid[u]) continue;
#pragma unroll
      for (int ch = 0; ch < 4; ++ch) {
        bf16_t* d = xl + uoff[u] + ch * hg.CS;
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) *(s8v*)(d + pl * HW_BC * hg.CS) = sx[u][ch][pl];
      }
    }
  };

  // ---- fragments: wave (kb, kh): k block kb (32 rows), the steps ks = kh, kh + 2, .. of each tile,
  // ALL taps. lane l: row / column l & 31, pixels 8 (l >> 5) .. + 7. A tap row r is read as two
  // 16-byte-ALIGNED chunks per plane (halo columns pcol .. pcol + 15); the s = 1, 2 windows are
  // shifted out of those registers (misaligned ds_read_b128 run at a fraction of the LDS rate:
  // timing probes DDL_HW_PROBE, profiles/x6hw_wgrad_r4.txt)
  const int kb = wid >> 1, kh = wid & 1;
  const int arow = (kb * 32 + (lane & 31)) * HW_KS;
  // halo element offset of the lane's first pixel (tap (0, 0)) in step ks
  auto xbase = [&](int ks) {
    const int p = 16 * ks + 8 * (lane >> 5);
    const int prow = p >> hg.lgW, pcol = p & (OW - 1);
    const int seg = prow / hg.SR, r = prow - seg * hg.SR;
    return (lane & 31) * hg.CS + (seg * hg.HR + r) * hg.HCp + pcol;
  };
  f16v acc[T];
#pragma unroll
  for (int t = 0; t < T; ++t)
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[t][v] = 0.f;

  if (t0 < t1) {
    if (!(hg.probe & 4)) load_tile(t0);
    for (int tile = t0; tile < t1; ++tile) {
      __syncthreads();  // previous tile's fragment reads are done
      hw_wait();
      if (!(hg.probe & 1)) {
        split_tile();
        write_tile();
      }
      if (tile + 1 < t1 && !(hg.probe & 4)) load_tile(tile + 1);  // in flight during this tile's MFMAs
      __syncthreads();
      if (hg.probe & 2) continue;
#pragma unroll 1
      for (int ip = 0; ip < 2; ++ip) {
        // two own steps (ks = 4 ip + kh, 4 ip + 2 + kh) per chain: twelve piece products from
        // zero, then one IEEE add per tap (half the VALU adds of per-step chains)
        s8v ah[2], am[2], al[2];
        int xb[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int ks = 4 * ip + 2 * j + kh;
          xb[j] = xbase(ks);
          const bf16_t* ap = dyl + arow + 16 * ks + 8 * (lane >> 5);
          ah[j] = *(const s8v*)ap;
          am[j] = *(const s8v*)(ap + HW_BK * HW_KS);
          al[j] = *(const s8v*)(ap + 2 * HW_BK * HW_KS);
        }
#pragma unroll
        for (int r = 0; r < RS; ++r) {
          f16v c[RS];
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const bf16_t* bp = xl + xb[j] + r * hg.HCp;
            s8v bh[RS], bm[RS], bl[RS];
            const s8v h0 = *(const s8v*)bp, m0 = *(const s8v*)(bp + HW_BC * hg.CS),
                      l0 = *(const s8v*)(bp + 2 * HW_BC * hg.CS);
            bh[0] = h0; bm[0] = m0; bl[0] = l0;
            if constexpr (RS == 3) {
              const s8v h1 = *(const s8v*)(bp + 8), m1 = *(const s8v*)(bp + 8 + HW_BC * hg.CS),
                        l1 = *(const s8v*)(bp + 8 + 2 * HW_BC * hg.CS);
              bh[1] = __builtin_shufflevector(h0, h1, 1, 2, 3, 4, 5, 6, 7, 8);
              bm[1] = __builtin_shufflevector(m0, m1, 1, 2, 3, 4, 5, 6, 7, 8);
              bl[1] = __builtin_shufflevector(l0, l1, 1, 2, 3, 4, 5, 6, 7, 8);
              bh[2] = __builtin_shufflevector(h0, h1, 2, 3, 4, 5, 6, 7, 8, 9);
              bm[2] = __builtin_shufflevector(m0, m1, 2, 3, 4, 5, 6, 7, 8, 9);
              bl[2] = __builtin_shufflevector(l0, l1, 2, 3, 4, 5, 6, 7, 8, 9);
            }
            // the row's RS chains interleaved stage by stage
#pragma unroll
            for (int s2 = 0; s2 < RS; ++s2)
              c[s2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[j], bh[s2], j ? c[s2] : (f16v){}, 0, 0, 0);
#pragma unroll
            for (int s2 = 0; s2 < RS; ++s2) c[s2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[j], bl[s2], c[s2], 0, 0, 0);
#pragma unroll
            for (int s2 = 0; s2 < RS; ++s2) c[s2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[j], bm[s2], c[s2], 0, 0, 0);
#pragma unroll
            for (int s2 = 0; s2 < RS; ++s2) c[s2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[j], bm[s2], c[s2], 0, 0, 0);
#pragma unroll
            for (int s2 = 0; s2 < RS; ++s2) c[s2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[j], bh[s2], c[s2], 0, 0, 0);
#pragma unroll
            for (int s2 = 0; s2 < RS; ++s2) c[s2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[j], bh[s2], c[s2], 0, 0, 0);
          }
#pragma unroll
          for (int s2 = 0; s2 < RS; ++s2) {
#pragma unroll
            for (int v = 0; v < 16; ++v) acc[r * RS + s2][v] = acc[r * RS + s2][v] + c[s2][v];
          }
        }
      }
    }
  }

  // ---- the two step-parity halves of each k block: kh = 1 hands its sums to kh = 0 through LDS
  // (fixed order: deterministic), which adds and writes
  __syncthreads();
  float* const red = (float*)smem;  // [2 kb][T][16][64]
  if (kh == 1) {
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
      for (int v = 0; v < 16; ++v) red[((kb * T + t) * 16 + v) * 64 + lane] = acc[t][v];
  }
  __syncthreads();
  if (kh == 1) return;
#pragma unroll
  for (int t = 0; t < T; ++t)
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[t][v] = acc[t][v] + red[((kb * T + t) * 16 + v) * 64 + lane];

  // ---- epilogue: 32x32 block (kb, tap): col = lane & 31 (channel), row = 8 (v >> 2) + 4 (lane >> 5) + (v & 3)
  const long long qd = (long long)T * C;  // dW row length (taps x channels)
  const bool split_store = nsplit > 1;
  float* dst = split_store ? a.partial + ((long long)split * a.G + g) * K * qd : a.out + (long long)g * a.out_gs;
#pragma unroll
  for (int t = 0; t < T; ++t) {
    // the read-modify-write's 16 loads are all issued before the first use (one at a time, each
    // waited out, they serialised the unsplit epilogue)
    float old[16];
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      const int k = k0 + kb * 32 + 8 * (v >> 2) + 4 * (lane >> 5) + (v & 3);
      const long long off = (long long)k * qd + (long long)t * C + c0 + (lane & 31);
      old[v] = (!split_store && a.accumulate) ? dst[off] : 0.f;
    }
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      const int k = k0 + kb * 32 + 8 * (v >> 2) + 4 * (lane >> 5) + (v & 3);
      const long long off = (long long)k * qd + (long long)t * C + c0 + (lane & 31);
      dst[off] = split_store ? acc[t][v] : old[v] + a.gscale * acc[t][v];
    }
  }
}

}  // namespace

static bool hw_geo(const ConvF32Args& a, HWGeo& h, int& rs) {
  if (a.stride != 1 || a.R != a.S || (a.R != 1 && a.R != 3) || a.pad != (a.R - 1) / 2) return false;
  if (a.P != a.H || a.Q != a.W || a.K % HW_BK || a.C % HW_BC) return false;
  const int OW = a.Q, OH = a.P;
  if (OW < 8 || OW > HW_TP || (OW & (OW - 1))) return false;
  rs = a.R;
  int lg = 0;
  while ((1 << lg) < OW) ++lg;
  const int TR = HW_TP / OW;
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
  h.NSEG = TR / SR;
  h.HR = SR + a.R - 1;
  h.HCp = (OW + a.S - 1 + 7) / 8 * 8;
  const int img = h.NSEG * h.HR * h.HCp;
  h.CS = (img - 8 + 127) / 128 * 128 + 8;  // >= img, == 8 (mod 128): 16 B apart mod 256 B per channel
  const long long npix = (long long)a.N * a.P * a.Q;
  h.ntile = (int)((npix + HW_TP - 1) / HW_TP);
  const int nxu = 8 * h.NSEG * h.HR * (h.HCp / 8);
  h.NUX = (nxu + 255) / 256;
  if (h.NUX > 2) return false;
  static const int probe = getenv("DDL_HW_PROBE") ? atoi(getenv("DDL_HW_PROBE")) : 0;
  h.probe = probe;
  const long long lim = (1LL << 31) - 64;
  if (npix * a.C * 4 > lim || npix * a.K * 4 > lim) return false;
  return true;
}

static size_t hw_lds(const HWGeo& h, int T) {
  const size_t stage = (size_t)3 * (HW_BK * HW_KS + HW_BC * h.CS) * 2;
  const size_t red = (size_t)2 * T * 16 * 64 * 4;  // the epilogue's cross-wave sums
  return stage > red ? stage : red;
}

extern "C" __attribute__((visibility("default"))) int ddl_x6hw_ok(const ConvF32Args* ap) {
  HWGeo h;
  int rs;
  return hw_geo(*ap, h, rs) && hw_lds(h, rs * rs) <= 160 * 1024 ? 1 : 0;
}

// pixel tiles per group (the split-K planner's unit)
extern "C" __attribute__((visibility("default"))) int ddl_x6hw_tiles(const ConvF32Args* ap) {
  HWGeo h;
  int rs;
  return hw_geo(*ap, h, rs) ? h.ntile : 0;
}

template <int RS, int NUX>
static int launch_hw(const ConvF32Args& a, const HWGeo& h, hipStream_t s) {
  const int split = a.split_k < 1 ? 1 : a.split_k;
  const size_t lds = hw_lds(h, RS * RS);
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)convx6hw_kernel<RS, NUX>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        160 * 1024);
    attr_set = true;
  }
  const dim3 grid((unsigned)((a.K / HW_BK) * (a.C / HW_BC)), (unsigned)split, (unsigned)a.G);
  hipLaunchKernelGGL((convx6hw_kernel<RS, NUX>), grid, dim3(256), lds, s, a, h);
  return (int)hipGetLastError();
}

extern "C" __attribute__((visibility("default"))) int ddl_x6hw(const ConvF32Args* ap, hipStream_t s) {
  const ConvF32Args& a = *ap;
  HWGeo h;
  int rs;
  if (a.G < 1 || a.N < 1 || !hw_geo(a, h, rs) || hw_lds(h, rs * rs) > 160 * 1024) return (int)hipErrorInvalidValue;
  const int split = a.split_k < 1 ? 1 : a.split_k;
  if (split > 1) {
    const long long need = (long long)split * a.G * a.K * a.R * a.S * a.C;
    if (!a.partial || need > a.partial_cap) return (int)hipErrorInvalidValue;
  }
  int e;
  if (rs == 3) e = h.NUX == 1 ? launch_hw<3, 1>(a, h, s) : launch_hw<3, 2>(a, h, s);
  else e = h.NUX == 1 ? launch_hw<1, 1>(a, h, s) : launch_hw<1, 2>(a, h, s);
  return e;
}
