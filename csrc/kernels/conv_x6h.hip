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
#include <cstdlib>

constexpr int BQH = 128;    // output pixels per tile
// Operand images are PLANAR per 16-channel chunk: [h0..h15 | m0..m15 | l0..l15] (3 x 32 B), one
// plane per bf16 piece of the exact split, padded to 7 x 16 B so consecutive rows / pixels rotate
// over the 16 bank quads (7 is odd).
constexpr int HSTR = 112;   // halo image bytes per pixel
constexpr int PSTR = 112;   // weight image bytes per row
constexpr int PQ = 7;       // quads per pixel / row
constexpr int HBSMALL = 32768;  // halo image bytes, OW >= 8 (2 workgroups per CU at BP 128: 48 + 32 KiB)
constexpr int HBLARGE = 45056;  // OW = 4 (8 image segments of 6 x 6 pixels)
constexpr int NWB = 3;      // weight images in the LDS ring (DMA runs two steps ahead)
// Precision note: the bf16 MFMA's internal accumulation is biased (not round-to-nearest). Long
// chains into one accumulator (one per 16-channel chunk = 54 MFMAs) left a ~3e-6 relative
// SYSTEMATIC error in the conv outputs, which a BatchNorm backward's sum over 16k pixels (heavy
// cancellation) amplified to 1e-2 (scripts/debug_r18_grads.py, ResNet-18 layer1 bn1.bias). Here
// each 16-channel step is one chain whose value is large for exactly one accumulation (hh last),
// then one IEEE add — the rounding pattern of conv_f32.hip's X6 engine.
// Out-of-range buffer offset: any per-step scalar offset added to it stays >= the descriptor's
// num_records (< 2^31), so the load returns zeros without a per-step select.
constexpr unsigned OOB = 0x80000000u;

// Halo image layout: pixel (segment sg, row hi, col hj) at sg * SEGB + hi * ROWB + hj * HSTR bytes.
// HSTR = 7 quads (16 B) per pixel spreads the pixels of one row over the 16 bank quads; ROWB and
// SEGB are padded (host: halo_layout) so that the 16 lanes of every ds_read_b128 group — which
// span 1..8 output rows of the tile depending on OW — land on distinct bank quads (conflict-free
// for OW = 4, 16, 32; one 2-way pair for OW = 8 inside the 32 KiB budget).
struct HaloGeo {
  int lgW;      // log2 OW (output pixels per row)
  int SR;       // output rows per image segment of the tile
  int HR, HC;   // halo rows / cols per segment
  int HP;       // halo pixels per tile
  int OH;       // output rows per image
  int SH, SW, SC;  // source (X for FWD, dY for DGRAD) height, width, channels
  int Pd;       // output channels (K for FWD, C for DGRAD)
  int ROWB, SEGB, HBYTES;  // halo row / segment strides, image bytes
  int OWr;      // real output width (< 1 << lgW: rows padded to the power of two, PADW instances)
  int Qv;       // virtual output pixels N * OH * (1 << lgW) (the tiles run over these)
  int probe;    // timing probes (DDL_X6H_PROBE, WRONG results): 1 no weight DMA, 2 no halo loads, 4 no
                // fragment reads / MFMAs, 8 no epilogue, 16 no main-loop barriers, 32 no halo split / LDS stores, 64 return at
                // once, 128 no main loop
};

typedef float f16v __attribute__((ext_vector_type(16)));

template <int N>
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
// Workgroup barrier WITHOUT the release fence of __syncthreads (which waits for every outstanding
// vector-memory op, the in-flight weight DMA included): callers order LDS themselves (counted
// vmcnt for the DMA pieces, lgkmcnt(0) after ds_writes that other waves read).
__device__ __forceinline__ void cta_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ void wait_lds() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// One LDS-DMA piece (16 B per lane to lds + 16 * lane). Kept out of the kernel body: with the
// address-space cast inline in a __global__ template, the host pass silently drops the kernel's
// launch stub (the library then fails to load).
__device__ __forceinline__ void dma16(const __amdgpu_buffer_rsrc_t& rs, char* lds, unsigned off, unsigned soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)lds, 16, off, soff, 0, 0);
}

__device__ __forceinline__ float4 bload4(const __amdgpu_buffer_rsrc_t& rs, unsigned off, unsigned soff) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, soff, 0));
}

#ifndef X6H_DGRAD128_CHAIN
#define X6H_DGRAD128_CHAIN 3
#endif
#ifndef X6H_CHAIN
#define X6H_CHAIN 3
#endif
// X6H_TRANSPOSE 1: activations are the MFMA A operand (D[q][p], fepi_t); 0: weights are (D[p][q],
// the quads-of-channels epilogue fepi of conv_f32_core.h) — kept for A/B runs
#ifndef X6H_TRANSPOSE
#define X6H_TRANSPOSE 1
#endif

// Epilogue on the transposed accumulators (activations were the MFMA A operand): lane l of wave
// (wp, wq) holds channel p = wp * BP/2 + ti * 32 + (l & 31) of the pixels
// q = wq * 64 + tj * 32 + 8 * (r >> 2) + 4 * (l >> 5) + (r & 3), r = 0..15 (acc[ti][tj][r]).
// Every store / residual / mask load is one dword per lane with 32 consecutive channels per
// half-wave (full 128-B lines; the quads-of-channels layout of fepi wrote 32-B pieces of 32 lines
// per instruction), addressed as buffer ops: the lane's (q, p) byte offset in a VGPR and the
// element's uniform row offset (tj * 32 + 8 * (r >> 2) + (r & 3)) * Pd * 4 in the SCALAR offset, so
// an element costs one memory instruction and no address VALU; rows past Qd fall outside the
// descriptor's range (loads read 0, stores drop) and lanes past Pd carry the OOB offset. The BN
// statistics reduce over a lane's own 32 pixels before a single cross-half shuffle (fepi: a 5-step
// shuffle tree per channel quad). Same outputs and slot layout as fepi (conv_f32_core.h): FWD y =
// [relu](acc + bias + residual) with per-tile (sum, M2 about the tile mean); stride-1 DGRAD
// dx = mask(acc + residual) with the BN-backward sums.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const float* p, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ float bld1(const __amdgpu_buffer_rsrc_t& rs, unsigned off, unsigned soff) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, off, soff, 0));
}
__device__ __forceinline__ void bst1(float v, const __amdgpu_buffer_rsrc_t& rs, unsigned off, unsigned soff) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), rs, off, soff, 0);
}

// PADW: the image rows are padded to 1 << lgW pixels (OWr real): o.Qd counts VIRTUAL pixels, a
// pixel q is real when (q & (2^lgW - 1)) < OWr and sits at (q >> lgW) * OWr + that column; element
// offsets are per lane (no scalar row offset) and padding pixels are neither stored nor counted.
template <int MODE, int BP, bool PADW>
__device__ __forceinline__ void fepi_t(const ConvF32Args& a, const FGeo& o, f16v (&acc)[BP / 64][2], float* red,
                                       int lgW, int OWr) {
  constexpr int WP = BP / 2, TI = WP / 32, TJ = 2;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wp = wid >> 1, wq = wid & 1;
  const int g = o.g, Pd = o.Pd;
  const bool want_stats = a.stats != nullptr;
  const bool dg_stats = MODE == F_DGRAD && want_stats && a.bn_x;
  const long long gofs = (long long)g * a.out_gs;
  const long long nreal = PADW ? (long long)(o.Qd >> lgW) * OWr : (long long)o.Qd;
  const long long nbytes = nreal * Pd * 4;  // one group's output (host: < 2^31)
  const __amdgpu_buffer_rsrc_t rO = rsrc_of(a.out + gofs, nbytes);
  const bool res_full = a.residual && (MODE == F_FWD || a.res_sub != 2);
  const __amdgpu_buffer_rsrc_t rR = rsrc_of(res_full ? a.residual + gofs : a.out, nbytes);
  const __amdgpu_buffer_rsrc_t rM = rsrc_of(a.mask ? a.mask + gofs : a.out, nbytes);
  const __amdgpu_buffer_rsrc_t rX = rsrc_of(a.bn_x ? a.bn_x + gofs : a.out, nbytes);
  const int qb = o.q0 + wq * 64 + 4 * (lane >> 5);
  const bool full = o.q0 + BQH <= o.Qd;
  const unsigned rowb = (unsigned)Pd * 4u;
  // compact-grid residual (res_sub 2, the stride-2 shortcut's dX on even pixels)
  const __amdgpu_buffer_rsrc_t rC = rsrc_of(a.residual && !res_full ? a.residual + (long long)g * a.res_gs : a.out,
                                            nbytes / 4);
  const int Wc = (a.W + 1) >> 1;  // compact grid width
  const int wmask = (1 << lgW) - 1;
  // per element (e = 16 tj + r): virtual pixel qb + dq(e), its real index (PADW) and validity
  auto dq_of = [](int e) { return (e >> 4) * 32 + 8 * ((e & 15) >> 2) + (e & 3); };
  auto real_of = [&](int q) { return PADW ? (q >> lgW) * OWr + (q & wmask) : q; };
  auto valid_q = [&](int q) { return (full || q < o.Qd) && (!PADW || (q & wmask) < OWr); };
#pragma unroll
  for (int ti = 0; ti < TI; ++ti) {
    const int pl = wp * WP + ti * 32 + (lane & 31);
    const int p = o.p0 + pl;
    const bool pv = p < Pd;
    const unsigned vo = pv ? ((unsigned)qb * (unsigned)Pd + (unsigned)p) * 4u : OOB;
    // PADW: element e's byte offset (vector), padding pixels out of range
    auto voff = [&](int e) -> unsigned {
      const int q = qb + dq_of(e);
      return (pv && valid_q(q)) ? ((unsigned)real_of(q) * (unsigned)Pd + (unsigned)p) * 4u : OOB;
    };
    float bia = 0.f, bm = 0.f, br = 0.f, ms = 0.f, mh = 0.f;
    if (MODE == F_FWD && a.bias && pv) bia = a.bias[(long long)g * a.bias_gs + p];
    if (MODE == F_DGRAD && a.bn_x && pv) {
      bm = a.bn_mean[(long long)g * Pd + p];
      br = a.bn_rstd[(long long)g * Pd + p];
    }
    if (MODE == F_DGRAD && a.mask_scale && pv) {
      ms = a.mask_scale[(long long)g * Pd + p];
      mh = a.mask_shift[(long long)g * Pd + p];
    }
    // every operand load of a 16-element group is issued before any is used (a load behind a use,
    // or behind a branch, waits out the previous one's full latency: the residual + mask + BN
    // DGRAD epilogue ran ~4x the time of its bytes that way)
    float s0 = 0.f, s1 = 0.f;
    // EB elements per load batch (BP 128 DGRAD sits at the 256-VGPR edge: 8)
    constexpr int EB = (MODE == F_DGRAD && BP == 128) ? 8 : 16;
#pragma unroll
    for (int b0 = 0; b0 < TJ * 16; b0 += EB) {
      float rv[EB], mv[EB], xv[EB];
      unsigned ve[PADW ? EB : 1];
      if constexpr (PADW) {
#pragma unroll
        for (int i = 0; i < EB; ++i) ve[i] = voff(b0 + i);
      }
      // element i's (vector, scalar) offsets: scalar row offset on the dense layout, per-lane on PADW
      auto ld = [&](const __amdgpu_buffer_rsrc_t& rs, int i) {
        if constexpr (PADW) return bld1(rs, ve[i], 0u);
        else return bld1(rs, vo, (unsigned)dq_of(b0 + i) * rowb);
      };
      if (res_full) {
#pragma unroll
        for (int i = 0; i < EB; ++i) rv[i] = ld(rR, i);
      } else if (MODE == F_DGRAD && a.residual) {
        // compact grid (res_sub 2, H even: host-checked): pixel (t = n*H + h, w) reads compact element
        // ((t >> 1) * ceil(W/2) + (w >> 1)) when t and w are both even, else nothing (OOB)
#pragma unroll
        for (int i = 0; i < EB; ++i) {
          const int q = qb + dq_of(b0 + i);
          const int t = q >> lgW, w = q & wmask;
          const unsigned ci = (unsigned)((t >> 1) * Wc + (w >> 1));
          rv[i] = bld1(rC, (((t | w) & 1) == 0 && pv && valid_q(q)) ? (ci * (unsigned)Pd + (unsigned)p) * 4u : OOB, 0u);
        }
      }
      if (MODE == F_DGRAD && a.mask) {
#pragma unroll
        for (int i = 0; i < EB; ++i) mv[i] = ld(rM, i);
      }
      if (MODE == F_DGRAD && a.bn_x) {
#pragma unroll
        for (int i = 0; i < EB; ++i) xv[i] = ld(rX, i);
      }
#pragma unroll
      for (int i = 0; i < EB; ++i) {
        const int e = b0 + i, tj = e >> 4, r = e & 15;
        const int dq = dq_of(e);
        const bool ok = pv && valid_q(qb + dq);
        float v = acc[ti][tj][r];
        if (MODE == F_FWD) {
          v += bia;
          if (res_full) v += rv[i];
          if (a.relu) v = fmaxf(v, 0.f);
          if (want_stats) {
            s0 += ok ? v : 0.f;
            acc[ti][tj][r] = v;  // kept for the centred second pass
          }
        } else {
          if (a.residual) v += rv[i];
          if (a.mask && !(mv[i] > 0.f)) v = 0.f;
          if (a.bn_x) {
            const float xs = xv[i];
            if (a.mask_scale && !(xs * ms + mh > 0.f)) v = 0.f;
            if (want_stats && ok) {
              s0 += v;
              s1 += v * ((xs - bm) * br);
            }
          }
        }
        if constexpr (PADW) bst1(v, rO, ve[i], 0u);
        else bst1(v, rO, vo, (unsigned)dq * rowb);
      }
    }
    if ((MODE == F_FWD && want_stats) || dg_stats) {
      s0 += __shfl_xor(s0, 32, 64);
      if (MODE == F_DGRAD) s1 += __shfl_xor(s1, 32, 64);
      if (lane < 32) {
        red[(wq * BP + pl) * 2] = s0;
        if (MODE == F_DGRAD) red[(wq * BP + pl) * 2 + 1] = s1;
      }
    }
  }
  if (!want_stats || (MODE == F_DGRAD && !a.bn_x)) return;
  if constexpr (MODE == F_FWD) {
    // (sum, M2 about the tile mean), merged across tiles with Chan's formula in bnf_finalize
    const int nq = PADW ? (min(BQH, o.Qd - o.q0) >> lgW) * OWr : min(BQH, o.Qd - o.q0);  // valid pixels
    __syncthreads();
#pragma unroll
    for (int ti = 0; ti < TI; ++ti) {
      const int pl = wp * WP + ti * 32 + (lane & 31);
      const bool pv = o.p0 + pl < Pd;
      const float mu = (red[pl * 2] + red[(BP + pl) * 2]) / (float)nq;
      float m2 = 0.f;
#pragma unroll
      for (int tj = 0; tj < TJ; ++tj)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float d = acc[ti][tj][r] - mu;
          m2 += (pv && valid_q(qb + dq_of(tj * 16 + r))) ? d * d : 0.f;
        }
      m2 += __shfl_xor(m2, 32, 64);
      if (lane < 32) red[(wq * BP + pl) * 2 + 1] = m2;
    }
  }
  __syncthreads();
  if (tid < BP && o.p0 + tid < Pd) {
    const int slot = o.phase * (a.slots / o.nph) + o.tq;
    float* st = a.stats + ((long long)g * a.slots + slot) * 2 * Pd + o.p0 + tid;
    st[0] = red[tid * 2] + red[(BP + tid) * 2];
    st[Pd] = red[tid * 2 + 1] + red[(BP + tid) * 2 + 1];
  }
}

template <int MODE, int BP, int RS, int HB, bool PADW>
__global__ __launch_bounds__(256, 2) void convx6h_kernel(ConvF32Args a, HaloGeo hg) {
  constexpr int T = RS * RS;                 // taps
  constexpr int PD = (RS - 1) / 2;           // pad
  constexpr int WP = BP / 2, TI = WP / 32, TJ = 2;
  constexpr int UP = BP / 32;                // weight LDS-DMA pieces (1 KiB) per wave per step
  constexpr int HPM = HB == HBSMALL ? 208 : 288;   // halo pixel capacity (host-checked)
  constexpr int NUH = (HPM * 4 + 255) / 256;  // halo units (pixel x 4-channel chunk) per thread
  constexpr int PIMG = BP * 128;             // bytes per weight image slot (BP * 112 used)
  constexpr bool XF_OK = MODE == F_FWD;
  constexpr bool DYB_OK = MODE == F_DGRAD;
  __shared__ __attribute__((aligned(16))) char smem[NWB * PIMG + HB];
  char* const pimg = smem;
  char* const himg = smem + NWB * PIMG;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wp = wid >> 1, wq = wid & 1;
  const int gx = gridDim.x, gy = gridDim.y, gz = gridDim.z;
  const int lin = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  const int u = xcd_remap(lin, gx * gy * gz);
  const int bx = u % gx, by = (u / gx) % gy, g = u / (gx * gy);
  if (hg.probe & 64) return;  // launch / dispatch cost only
  FGeo o = fgeo<MODE, BP, BQH>(a, bx, by, g, gy);
  o.Qd = hg.Qv;  // tiles run over the virtual (row-padded) pixels; == N*P*Q unless PADW
  const bool split_store = a.split_k > 1;
  if (o.q0 >= o.Qd || o.p0 >= o.Pd) {
    if (!split_store) fzero_slot<MODE, BP>(a, o);
    return;
  }
  const int SC = hg.SC, Pd = hg.Pd;
  const int ncc = SC >> 4;
  const int per = (ncc + o.nsplit - 1) / o.nsplit;
  const int cc0 = o.split * per, cc1 = min(ncc, cc0 + per);

  // operand-side BN (FWD): every halo unit of this thread covers the same 4 channels of a chunk,
  // channels cc * 16 + 4 * (tid & 3) .. + 3: scale / shift loaded with the chunk's halo
  const bool xf = XF_OK && a.in_scale != nullptr;
  const bool xrelu = a.in_relu != 0;
  float4 xsc = make_float4(1.f, 1.f, 1.f, 1.f), xsh = make_float4(0.f, 0.f, 0.f, 0.f);
  // DGRAD: dY operand = the following BN's backward, A * dy + B * x_bn + C (per channel); the
  // first P tile also writes it out (dyb_out) for the layer's WGRAD
  const bool dyb = DYB_OK && a.dyb_coef != nullptr;
  const bool dyb_w = dyb && a.dyb_out != nullptr && o.p0 == 0;
  float4 dA = xsc, dB = xsh, dC = xsh;

  // ---------------------------------------------------------------- buffer descriptors
  const float* src = MODE == F_FWD ? a.x + (long long)g * a.x_gs : a.dy + (long long)g * a.dy_gs;
  const long long src_bytes = (long long)a.N * hg.SH * hg.SW * SC * 4;
  const __amdgpu_buffer_rsrc_t rS = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, (int)src_bytes, 0x00020000);
  const float* srcx = dyb ? a.dyb_x + (long long)g * a.dy_gs : src;
  const __amdgpu_buffer_rsrc_t rXb = __builtin_amdgcn_make_buffer_rsrc((void*)srcx, 0, (int)src_bytes, 0x00020000);
  float* dyo = dyb_w ? a.dyb_out + (long long)g * a.dy_gs : nullptr;
  const char* wsp = (const char*)a.wsplit + (long long)g * a.ws_gs;
  const __amdgpu_buffer_rsrc_t rW = __builtin_amdgcn_make_buffer_rsrc(
      (void*)wsp, 0, (int)((long long)Pd * T * SC * 6), 0x00020000);

  // ---------------------------------------------------------------- halo bookkeeping
  // unit i of this thread: halo pixel hp = uu >> 2, 4-channel chunk ch = uu & 3
  const int nunits = hg.HP * 4;
  const int t0 = o.q0 >> hg.lgW;  // first output row (over n, oh) of the tile
  unsigned hoff[NUH];             // source byte offset at chunk 0 (OOB: padding / beyond N)
  int hlds[NUH];                  // LDS byte offset of the unit (-1: no unit)
  unsigned own = 0;               // bit i: unit i is one of the tile's own (core) pixels
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
      if (hoff[i] != OOB && hi >= PD && hi < PD + hg.SR && hj >= PD && hj < PD + hg.OWr) own |= 1u << i;
      hlds[i] = seg * hg.SEGB + hi * hg.ROWB + hj * HSTR + ch * 8;
    }
  }
  float4 hreg[NUH];
  float4 hxb[DYB_OK ? NUH : 1];
  auto halo_load = [&](int cc) {
    if (hg.probe & 2) return;
#pragma unroll
    for (int i = 0; i < NUH; ++i) hreg[i] = bload4(rS, hoff[i], (unsigned)cc * 64u);
    if constexpr (DYB_OK) {
      if (dyb) {
#pragma unroll
        for (int i = 0; i < NUH; ++i) hxb[i] = bload4(rXb, hoff[i], (unsigned)cc * 64u);
        const float* cf = a.dyb_coef + (long long)g * 3 * SC + cc * 16 + 4 * (tid & 3);
        dA = *(const float4*)cf;
        dB = *(const float4*)(cf + SC);
        dC = *(const float4*)(cf + 2 * SC);
      }
    }
    if constexpr (XF_OK) {
      if (xf) {
        const long long c = (long long)g * SC + cc * 16 + 4 * (tid & 3);
        xsc = *(const float4*)(a.in_scale + c);
        xsh = *(const float4*)(a.in_shift + c);
      }
    }
  };
  auto halo_store = [&](int cc) {
    if (hg.probe & 32) return;
#pragma unroll
    for (int i = 0; i < NUH; ++i) {
      if (hlds[i] < 0) continue;
      float4 v = hreg[i];
      if constexpr (XF_OK) {
        if (xf && hoff[i] != OOB) {  // operand-side BN + ReLU on real pixels (padding stays 0)
          v.x = v.x * xsc.x + xsh.x;
          v.y = v.y * xsc.y + xsh.y;
          v.z = v.z * xsc.z + xsh.z;
          v.w = v.w * xsc.w + xsh.w;
          if (xrelu) { v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f); }
        }
      }
      if constexpr (DYB_OK) {
        if (dyb && hoff[i] != OOB) {  // BN backward of dY on real pixels (padding stays 0)
          const float4 xb = hxb[i];
          v.x = dA.x * v.x + dB.x * xb.x + dC.x;
          v.y = dA.y * v.y + dB.y * xb.y + dC.y;
          v.z = dA.z * v.z + dB.z * xb.z + dC.z;
          v.w = dA.w * v.w + dB.w * xb.w + dC.w;
          if (dyb_w && ((own >> i) & 1u)) *(float4*)(dyo + (hoff[i] + (unsigned)cc * 64u) / 4u) = v;
        }
      }
      s4v h, m, l;
      split3(v, h, m, l);
      *(s4v*)(himg + hlds[i]) = h;
      *(s4v*)(himg + hlds[i] + 32) = m;
      *(s4v*)(himg + hlds[i] + 64) = l;
    }
  };

  // ---------------------------------------------------------------- weight (P operand) staging
  // LDS-DMA (buffer_load ... lds, 1 KiB per wave-instruction, lane-linear destination): piece i of
  // wave wsc covers image bytes (wsc + 4 i) KiB, i.e. 16-B granule L = 64 (wsc + 4 i) + lane =
  // row L / 7, granule L % 7 (6 = the pad: nothing to fetch). The global source (pre-split
  // weights) holds the same 96 B per (row, tap, 16-channel chunk).
  const int wsc = __builtin_amdgcn_readfirstlane(wid);
  unsigned woff[UP];
#pragma unroll
  for (int i = 0; i < UP; ++i) {
    const int L = (wsc + 4 * i) * 64 + lane;
    const int row = L / PQ, gr = L - row * PQ;
    const int p = o.p0 + row;
    woff[i] = (row < BP && gr < 6 && p < Pd) ? (unsigned)((long long)p * T * SC * 6 + gr * 16) : OOB;
  }
  auto wload = [&](int buf, int cc, int t) {
    if (hg.probe & 1) return;
    const int wtap = MODE == F_FWD ? t : T - 1 - t;  // DGRAD: the flipped kernel
    const unsigned add = (unsigned)(wtap * SC * 6 + cc * 96);  // wave-uniform: the scalar offset
#pragma unroll
    for (int i = 0; i < UP; ++i) dma16(rW, pimg + buf * PIMG + (wsc + 4 * i) * 1024, woff[i], add);
  };

  // ---------------------------------------------------------------- fragment addressing
  const int hh = lane >> 5;  // lane half: channels 8 hh .. 8 hh + 7 of the 16-channel chunk
  int aoff[TI];              // weight image byte offset of the h plane (m: +32, l: +64)
#pragma unroll
  for (int ti = 0; ti < TI; ++ti) aoff[ti] = (wp * WP + ti * 32 + (lane & 31)) * PSTR + hh * 16;
  int boff[TJ];  // halo image byte offsets of tap (0, 0)
#pragma unroll
  for (int tj = 0; tj < TJ; ++tj) {
    const int ql = wq * 64 + tj * 32 + (lane & 31);
    const int jj = ql & ((1 << hg.lgW) - 1), rowl = ql >> hg.lgW;
    const int seg = rowl / hg.SR, ii = rowl - seg * hg.SR;
    boff[tj] = seg * hg.SEGB + ii * hg.ROWB + jj * HSTR + hh * 16;
  }

  f16v acc[TI][TJ];  // running sums: one IEEE add per 16-channel step
#pragma unroll
  for (int ti = 0; ti < TI; ++ti)
#pragma unroll
    for (int tj = 0; tj < TJ; ++tj) acc[ti][tj] = (f16v){};

  const int k0 = cc0 * T, k1 = cc1 * T;
  constexpr int HT = T >= 3 ? T - 3 : 0;  // tap at which the next chunk's halo loads are issued

  int bdr[RS][TJ];  // halo fragment bases per tap row
#pragma unroll
  for (int dr = 0; dr < RS; ++dr)
#pragma unroll
    for (int tj = 0; tj < TJ; ++tj) bdr[dr][tj] = boff[tj] + dr * hg.ROWB;
  // X6H_CHAIN (1 or 2): steps per chain before the IEEE add (unrolled-tap path only); the BP 128
  // DGRAD (dY BN-backward operand: twice the halo registers) keeps per-step chains, whose carried
  // chain registers would otherwise spill
  constexpr int CHAIN = (MODE == F_DGRAD && BP == 128 && HB == HBSMALL) ? X6H_DGRAD128_CHAIN : X6H_CHAIN;
  f16v cch[TI][TJ];
  auto compute = [&](int buf, int t, bool first = true, bool last = true) {
    if (hg.probe & 4) return;
    const char* P = pimg + buf * PIMG;
    const int dr = t / RS, ds = t - dr * RS;
    // one 16-channel step: A (weights) and B (activations) as three piece vectors each; the six
    // piece products in ONE chain, the five small ones first and hh last, so the chain's value is
    // large for exactly one (biased, non-round-to-nearest) MFMA accumulation before the IEEE add
    s8v ah[TI], am[TI], al[TI], bh[TJ], bm[TJ], bl[TJ];
#pragma unroll
    for (int ti = 0; ti < TI; ++ti) {
      ah[ti] = *(const s8v*)(P + aoff[ti]);
      am[ti] = *(const s8v*)(P + aoff[ti] + 32);
      al[ti] = *(const s8v*)(P + aoff[ti] + 64);
    }
#pragma unroll
    for (int tj = 0; tj < TJ; ++tj) {
      const char* hb = himg + bdr[dr][tj] + ds * HSTR;
      bh[tj] = *(const s8v*)hb;
      bm[tj] = *(const s8v*)(hb + 32);
      bl[tj] = *(const s8v*)(hb + 64);
    }
#pragma unroll
    for (int ti = 0; ti < TI; ++ti)
#pragma unroll
      for (int tj = 0; tj < TJ; ++tj) {
        // activations as the A operand: D[q][p], so a lane ends up holding ONE channel of 16 pixels
        // (fepi_t: coalesced stores, per-lane BN sums)
#if X6H_TRANSPOSE
#define X6MF(A, B, C) __builtin_amdgcn_mfma_f32_32x32x16_bf16(B, A, C, 0, 0, 0)
#else
#define X6MF(A, B, C) __builtin_amdgcn_mfma_f32_32x32x16_bf16(A, B, C, 0, 0, 0)
#endif
        f16v c = X6MF(al[ti], bh[tj], first ? (f16v){} : cch[ti][tj]);
        c = X6MF(ah[ti], bl[tj], c);
        c = X6MF(am[ti], bm[tj], c);
        c = X6MF(ah[ti], bm[tj], c);
        c = X6MF(am[ti], bh[tj], c);
        c = X6MF(ah[ti], bh[tj], c);
#undef X6MF
        if (last) {
#pragma unroll
          for (int v = 0; v < 16; ++v) acc[ti][tj][v] = acc[ti][tj][v] + c[v];
          // pin the adds to this step: otherwise they sink past the unrolled taps' barriers and
          // every step's chain result lives (in scratch) until the end of the chunk
          asm volatile("" : "+v"(acc[ti][tj]));
        } else {
          cch[ti][tj] = c;
        }
      }
  };

  if (k0 < k1 && !(hg.probe & 128)) {
    // Weight images: a ring of NWB = 3; the DMA of step k + 2 is issued at step k into slot
    // (k + 2) % 3, whose last reader (step k - 1) is past the barrier. vmcnt counts in issue order
    // (DMA pieces and the halo register loads together): at the end of step k, step k + 1's pieces
    // must have landed while step k + 2's (UP) and — between issue (tap HT) and use (chunk end) —
    // the next chunk's halo loads (NUH, +2 for the BN constants with xf; 2 NUH + 3 with the dY
    // BN-backward transform: dy, x_bn and the A | B | C constants) may still fly.
    auto step_of = [&](int kk, int& c, int& tt) { c = kk / T; tt = kk - c * T; };
    {
      int c1_, t1_;
      wload(0, cc0, 0);
      halo_load(cc0);
      if (k0 + 1 < k1) { step_of(k0 + 1, c1_, t1_); wload(1, c1_, t1_); }
      halo_store(cc0);
      wait_vm<0>();
      wait_lds();
      cta_barrier();
    }
    if constexpr (T % 3 == 0) {
      // taps unrolled: slot (tap % 3), DMA targets, halo timing and vmcnt counts are constants
      for (int cc = cc0; cc < cc1; ++cc) {
        const bool more = cc + 1 < cc1;
#pragma unroll
        for (int t = 0; t < T; ++t) {
          if (t + 2 < T) wload((t + 2) % 3, cc, t + 2);
          else if (more) wload((t + 2) % 3, cc + 1, t + 2 - T);
          if (t == HT && more) halo_load(cc + 1);
          if constexpr (CHAIN == 3) compute(t % 3, t, t % 3 == 0, t % 3 == 2);
          else if constexpr (CHAIN == 2) compute(t % 3, t, t % 2 == 0, t % 2 == 1 || t == T - 1);
          else compute(t % 3, t);
          // keep each step's MFMAs and adds inside the step: moved across the barrier into the next
          // step they pile up two steps' operands and chains and spill
          __builtin_amdgcn_sched_barrier(0);
          // (the BN-constant / x_bn loads of the halo exist only with xf / dyb: the counts must match
          // exactly — a larger count than issued would let a weight piece still be in flight)
          if (!more && t + 2 >= T) wait_vm<0>();
          else if (more && (t == HT || t == HT + 1) && HT + 1 < T - 1) {
            if (dyb) wait_vm<UP + 2 * NUH + 3>();
            else if (xf) wait_vm<UP + NUH + 2>();
            else wait_vm<UP + NUH>();
          } else wait_vm<UP>();
          if (!(hg.probe & 16)) cta_barrier();
          if (t == T - 1 && more) {  // chunk boundary: every wave is done with this chunk's halo
            halo_store(cc + 1);
            wait_lds();
            cta_barrier();
          }
        }
      }
    } else {
    int cc = cc0, t = 0, slot = 0;
    for (int k = k0; k < k1; ++k) {
      const bool issue2 = k + 2 < k1;
      if (issue2) {
        int c2, t2;
        step_of(k + 2, c2, t2);
        wload(slot == 0 ? 2 : slot - 1, c2, t2);  // (slot + 2) % 3
      }
      const bool hl = t == HT && cc + 1 < cc1;
      if (hl) halo_load(cc + 1);
      compute(slot, t);
      // retire step k + 1's pieces (and, at the chunk's last tap, the halo loads)
      const bool halo_fly = (HT < T - 1) && cc + 1 < cc1 && (t == HT || t == HT + 1);
      if (!issue2) wait_vm<0>();
      else if (halo_fly) {
        if (dyb) wait_vm<UP + 2 * NUH + 3>();
        else if (xf) wait_vm<UP + NUH + 2>();
        else wait_vm<UP + NUH>();
      } else wait_vm<UP>();
      cta_barrier();
      if (t == T - 1 && k + 1 < k1) {  // chunk boundary: every wave is done with this chunk's halo
        halo_store(cc + 1);
        wait_lds();
        cta_barrier();
      }
      if (++t == T) { t = 0; ++cc; }
      slot = slot == 2 ? 0 : slot + 1;
    }
    }
  }

  // ---------------------------------------------------------------- epilogue
  if (hg.probe & 8) {  // keep the accumulators live without storing them
    float sink = 0.f;
#pragma unroll
    for (int ti = 0; ti < TI; ++ti)
#pragma unroll
      for (int tj = 0; tj < TJ; ++tj) sink += acc[ti][tj][0] + acc[ti][tj][15];
    if (sink == 1.2345f) a.out[tid] = sink;
    return;
  }
#if !X6H_TRANSPOSE
  static_assert(!PADW, "row-padded halo tiles need the transposed epilogue");
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
#else
  if (split_store) {
    // raw partial sums of this slice: [split][G][1][qmax][Pd] (the layout of conv_f32.hip)
    const long long qmax = (long long)a.slots * BQH;
    float* d = a.partial + ((long long)o.split * a.G + g) * qmax * Pd;
#pragma unroll
    for (int ti = 0; ti < TI; ++ti) {
      const int p = o.p0 + wp * WP + ti * 32 + (lane & 31);
      if (p >= Pd) continue;
#pragma unroll
      for (int tj = 0; tj < TJ; ++tj)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int q = o.q0 + wq * 64 + tj * 32 + 8 * (r >> 2) + 4 * (lane >> 5) + (r & 3);
          if (q < o.Qd) d[(long long)q * Pd + p] = acc[ti][tj][r];
        }
    }
    return;
  }
  fepi_t<MODE, BP, PADW>(a, o, acc, (float*)smem, hg.lgW, hg.OWr);
#endif
}

// Many weights' split images in ONE launch (a training step's pre-split: every halo layer's FWD and
// DGRAD images of the step's weights, functional_f32.PresplitScope) instead of one launch per conv.
// Entry e owns blocks [blk0, blk0 + nblk); its blocks grid-stride over its 16-element chunks.
struct SplitDesc {
  const float* w;
  char* out;
  long long w_gs, o_gs;
  int G, K, T, C, layout, blk0, nblk, pad_;
};

// Work item u of one group -> the 16-element chunk it splits. Layout 0: chunk u (16 consecutive c
// of one (k, tap): contiguous reads). Layout 1: items run c fastest, u = ((k16 * T) + tap) * C + c,
// so the 16 strided reads w[k16*16 + i][tap][c] of consecutive items are coalesced; the item's
// output chunk is e = (c * T + tap) * K/16 + k16. Every chunk is written as six 16-byte stores.
__device__ __forceinline__ void split_chunk(const float* __restrict__ wg, char* og, long long u, int K, int T, int C,
                                            int layout) {
  float v[16];
  long long e;
  if (layout == 0) {
    e = u;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float4 f = *(const float4*)(wg + u * 16 + 4 * i);
      v[4 * i] = f.x; v[4 * i + 1] = f.y; v[4 * i + 2] = f.z; v[4 * i + 3] = f.w;
    }
  } else {
    const int K16 = K / 16;
    const int c = (int)(u % C);
    const long long kt = u / C;
    const int tap = (int)(kt % T), k16 = (int)(kt / T);
    const float* src = wg + ((long long)k16 * 16 * T + tap) * C + c;
    const long long ks = (long long)T * C;
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = src[i * ks];
    e = ((long long)c * T + tap) * K16 + k16;
  }
  s8v h[2], m[2], l[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    s4v h0, m0, l0, h1, m1, l1;
    split3(make_float4(v[8 * q], v[8 * q + 1], v[8 * q + 2], v[8 * q + 3]), h0, m0, l0);
    split3(make_float4(v[8 * q + 4], v[8 * q + 5], v[8 * q + 6], v[8 * q + 7]), h1, m1, l1);
    h[q] = cat44(h0, h1);
    m[q] = cat44(m0, m1);
    l[q] = cat44(l0, l1);
  }
  char* d = og + e * 96;
  *(s8v*)(d) = h[0];
  *(s8v*)(d + 16) = h[1];
  *(s8v*)(d + 32) = m[0];
  *(s8v*)(d + 48) = m[1];
  *(s8v*)(d + 64) = l[0];
  *(s8v*)(d + 80) = l[1];
}

// Pre-split weights: FWD layout [G][K][T][C] (16-channel chunks of the input channels), DGRAD
// layout [G][C][T][K] (16-channel chunks of the output channels), 6 bytes per element: per chunk
// the three bf16 planes [h0..h15 | m0..m15 | l0..l15] (the LDS operand image row of conv_x6h).
__global__ __launch_bounds__(256) void x6_split_weights_kernel(const float* __restrict__ w, char* out, int G, int K,
                                                               int T, int C, int layout, long long w_gs,
                                                               long long o_gs) {
  const long long per = (long long)K * T * C / 16;  // 16-chunks per group
  GSTRIDE_LOOP(t, (long long)G * per) {
    const long long g = t / per, u = t - g * per;
    split_chunk(w + g * w_gs, out + g * o_gs, u, K, T, C, layout);
  }
}

__global__ __launch_bounds__(256) void x6_split_weights_multi_kernel(const SplitDesc* __restrict__ descs, int n) {
  int lo = 0, hi = n - 1;  // the entry owning this block: last e with blk0 <= blockIdx.x
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (descs[mid].blk0 <= (int)blockIdx.x) lo = mid; else hi = mid - 1;
  }
  const SplitDesc d = descs[lo];
  const long long per = (long long)d.K * d.T * d.C / 16;
  const long long total = (long long)d.G * per;
  for (long long t = (long long)(blockIdx.x - d.blk0) * 256 + threadIdx.x; t < total; t += (long long)d.nblk * 256) {
    const long long g = t / per, u = t - g * per;
    split_chunk(d.w + g * d.w_gs, d.out + g * d.o_gs, u, d.K, d.T, d.C, d.layout);
  }
}

DDL_API int ddl_x6_split_desc_size() { return (int)sizeof(SplitDesc); }

// descs: device array of n SplitDesc (blk0 / nblk filled by the host), nblocks = total blocks
DDL_API int ddl_x6_split_weights_multi(const void* descs, int n, int nblocks, hipStream_t s) {
  if (n < 1 || nblocks < n) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(x6_split_weights_multi_kernel, dim3(nblocks), dim3(256), 0, s, (const SplitDesc*)descs, n);
  return (int)hipGetLastError();
}

// Halo row / segment strides (in 16-B quads): the fewest bank conflicts of the fragment reads
// (the 4 ds_read_b128 lane groups of a 32x32x16 B operand: lane l reads tile pixel l & 31, chunk
// half l >> 5), then the fewest bytes; within HBSMALL when any candidate fits.
static void halo_layout(HaloGeo& h) {
  static const int grp[2][16] = {{0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27},
                                 {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31}};
  const int OW = 1 << h.lgW, nseg = h.HP / (h.HR * h.HC);
  int best[4] = {1 << 30, 1 << 30, 0, 0};  // worst, total, rq, sq
  bool best_fit = false;
  for (int rq = PQ * h.HC; rq < PQ * h.HC + 16; ++rq)
    for (int sq = h.HR * rq; sq < h.HR * rq + 16; ++sq) {
      int worst = 0, tot = 0;
      for (int hh = 0; hh < 2; ++hh)
        for (int gi = 0; gi < 2; ++gi) {
          int cnt[16] = {0};
          for (int e = 0; e < 16; ++e) {
            const int q = grp[gi][e], row = q / OW, col = q % OW;
            const int seg = row / h.SR, ri = row % h.SR;
            ++cnt[(seg * sq + ri * rq + PQ * col + hh) & 15];
          }
          int m = 0;
          for (int c = 0; c < 16; ++c) m = cnt[c] > m ? cnt[c] : m;
          worst = m > worst ? m : worst;
          tot += m;
        }
      const int bytes = nseg * sq * 16;
      if (bytes > HBLARGE) continue;
      // the small-LDS instance also holds fewer halo units per thread (HPM 208, convx6h_kernel)
      const bool fit = bytes <= HBSMALL && h.HP <= 208;
      const int bbytes = nseg * best[3] * 16;
      bool better;
      if (fit != best_fit) better = fit;
      else if (worst != best[0]) better = worst < best[0];
      else if (tot != best[1]) better = tot < best[1];
      else better = bytes < bbytes;
      if (better) {
        best[0] = worst; best[1] = tot; best[2] = rq; best[3] = sq;
        best_fit = fit;
      }
    }
  h.ROWB = best[2] * 16;
  h.SEGB = best[3] * 16;
  h.HBYTES = best[3] ? nseg * h.SEGB : (1 << 30);  // no candidate fits: x6h_geo refuses
}

static bool x6h_geo(const ConvF32Args& a, int mode, int bp, HaloGeo& h, int& rs) {
  if (mode != F_FWD && mode != F_DGRAD) return false;
  if (bp != 64 && bp != 128) return false;
  if (a.stride != 1 || a.R != a.S || (a.R != 1 && a.R != 3) || a.pad != (a.R - 1) / 2) return false;
  if (a.P != a.H || a.Q != a.W) return false;
  rs = a.R;
  const int OH = a.P, OWr = a.Q;
  if (OWr < 4 || OWr > BQH) return false;
  int lg = 0;
  while ((1 << lg) < OWr) ++lg;
  const int OW = 1 << lg;  // rows padded to the power of two (PADW instances when OW != OWr)
  // a padded row's tile cannot be split over K: the split-K epilogue tiles the REAL pixels
  if (OW != OWr && a.split_k > 1) return false;
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
  h.OWr = OWr;
  h.Qv = a.N * OH * OW;
  h.SR = SR;
  h.HR = SR + a.R - 1;
  h.HC = OW + a.S - 1;
  h.HP = (TR / SR) * h.HR * h.HC;
  h.OH = OH;
  h.SH = a.H;
  h.SW = a.W;
  h.SC = mode == F_FWD ? a.C : a.K;
  h.Pd = mode == F_FWD ? a.K : a.C;
  if (h.HP > 288 || h.SC % 16 || h.Pd % 4) return false;
  if (mode == F_DGRAD && a.in_scale) return false;
  const long long lim = (1LL << 31) - 64;
  if ((long long)a.N * a.H * a.W * h.SC * 4 > lim || (long long)h.Pd * a.R * a.S * h.SC * 6 > lim) return false;
  if ((long long)a.N * a.P * a.Q * h.Pd * 4 > lim) return false;  // fepi_t: buffer-addressed output
  // fepi_t reads a compact-grid residual on even-height images only (split-K: the generic epilogue)
  if (mode == F_DGRAD && a.residual && a.res_sub == 2 && (a.H & 1) && a.split_k <= 1) return false;
  halo_layout(h);
  static const int probe = [] {
    const char* e = getenv("DDL_X6H_PROBE");
    return e ? atoi(e) : 0;
  }();
  h.probe = probe;
  // the instance is chosen by x6h_large(): a halo of more than 208 pixels (e.g. 64-wide images: two
  // rows of 66) runs on the large instance even when its bytes would fit the small one
  if (h.HBYTES > HBLARGE || h.HP > 288) return false;
  return true;
}

template <int MODE, int BP, int RS, int HB, bool PADW>
static int launch_x6h(ConvF32Args a, const HaloGeo& h, hipStream_t s) {
  const long long Pd = h.Pd, Qd = h.Qv;
  const long long ntp = (Pd + BP - 1) / BP, ntq = (Qd + BQH - 1) / BQH;
  a.slots = (int)ntq;
  const int split = a.split_k < 1 ? 1 : a.split_k;
  a.split_k = split;
  if (split > 1) {
    const long long need = (long long)split * a.G * ntq * BQH * Pd;
    if (!a.partial || need > a.partial_cap) return (int)hipErrorInvalidValue;
  }
  const dim3 grid((unsigned)(ntp * ntq), (unsigned)split, (unsigned)a.G);
  hipLaunchKernelGGL((convx6h_kernel<MODE, BP, RS, HB, PADW>), grid, dim3(256), 0, s, a, h);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || split == 1) return (int)e;
  hipLaunchKernelGGL((convf32_splitk_epilogue<MODE, BP, BQH>), dim3((unsigned)(ntp * ntq), 1, a.G), dim3(256), 0,
                     s, a);
  return (int)hipGetLastError();
}

template <int MODE, int HB, bool PADW>
static int dispatch_rs(const ConvF32Args& a, int bp, int rs, const HaloGeo& h, hipStream_t s) {
  if (rs == 3)
    return bp == 128 ? launch_x6h<MODE, 128, 3, HB, PADW>(a, h, s) : launch_x6h<MODE, 64, 3, HB, PADW>(a, h, s);
  return bp == 128 ? launch_x6h<MODE, 128, 1, HB, PADW>(a, h, s) : launch_x6h<MODE, 64, 1, HB, PADW>(a, h, s);
}
template <int MODE, int HB>
static int dispatch_hb(const ConvF32Args& a, int bp, int rs, const HaloGeo& h, hipStream_t s) {
  return h.OWr != (1 << h.lgW) ? dispatch_rs<MODE, HB, true>(a, bp, rs, h, s) : dispatch_rs<MODE, HB, false>(a, bp, rs, h, s);
}
static bool x6h_large(const HaloGeo& h) { return h.HBYTES > HBSMALL || h.HP > 208; }
template <int MODE>
static int dispatch_x6h(const ConvF32Args& a, int bp, int rs, const HaloGeo& h, hipStream_t s) {
  return x6h_large(h) ? dispatch_hb<MODE, HBLARGE>(a, bp, rs, h, s) : dispatch_hb<MODE, HBSMALL>(a, bp, rs, h, s);
}

// Statistics / BN-reduce slots of a halo launch (= its 128-pixel tiles per group: over the
// row-padded pixels when the width is not a power of two), -1 when the kernel declines it
DDL_API long long ddl_x6h_slots(const ConvF32Args* ap, int mode) {
  HaloGeo h;
  int rs;
  if (!x6h_geo(*ap, mode, 64, h, rs)) return -1;
  return ((long long)h.Qv + BQH - 1) / BQH;
}

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

// w [G][K][T][C] fp32 (group stride w_gs floats) -> out (group stride o_gs bytes, >= K*T*C*6)
DDL_API int ddl_x6_split_weights(const float* w, void* out, int G, int K, int T, int C, int layout,
                                 long long w_gs, long long o_gs, int pad_, hipStream_t s) {
  (void)pad_;
  if (G < 1 || K < 1 || T < 1 || C < 1 || (layout == 0 ? C % 16 : K % 16) || (w_gs % 4)) return (int)hipErrorInvalidValue;
  const long long work = (long long)G * K * T * C / 16;
  hipLaunchKernelGGL(x6_split_weights_kernel, dim3(grid_for(work, 256)), dim3(256), 0, s, w, (char*)out, G, K, T,
                     C, layout, w_gs, o_gs);
  return (int)hipGetLastError();
}
