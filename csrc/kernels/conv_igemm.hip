// Implicit-GEMM convolution on CDNA4 MFMA (v_mfma_f32_16x16x32_bf16), NHWC bf16, fp32 accumulate.
//
// One templated kernel family covers the three products of a conv layer (and of a Linear layer,
// which is the R=S=H=W=1 special case):
//
//   FWD   : y [q=(n,p,q)][p=k]         = sum_{(r,s,c)}  W[k][(r,s,c)]     * X[pix(q,r,s)][c]
//   DGRAD : dx[q=(n,h,w)][p=c]         = sum_{(r,s,k)}  W[k][(r,s,c)]     * dY[pix'(q,r,s)][k]
//   WGRAD : dW[p=k][q=(r,s,c)]        += sum_{(n,p,q)}  dY[(n,p,q)][k]    * X[pix(n,p,q,r,s)][c]
//
// Every mode is D[p][q] = sum_k Pop[p][k] * Qop[q][k] with the MFMA A operand = Pop, B = Qop, so
// the accumulator layout (lane holds 4 consecutive p for one q) gives 8-byte contiguous NHWC
// stores in FWD/DGRAD and 64-byte row segments for the fp32 WGRAD atomics.
//
// Operand staging: LDS-DMA (`buffer_load_dwordx4 ... lds`, 1 KiB per wave-instruction) into an
// NSTAGE-deep LDS ring, one raw s_barrier per K-step and COUNTED `s_waitcnt vmcnt(N)` so the next
// NSTAGE-2 stages stay in flight across the barrier (cdna_hip_programming.md §5 "Pipelining across
// barriers"). The implicit-GEMM gather is expressed purely through the per-lane SOURCE offset
// (lane base + one wave-uniform cursor term per K-step): padding / out-of-range taps use an
// offset past the buffer descriptor's range, which the hardware reads as zeros, and the LDS
// swizzles are applied by permuting which logical 16-byte chunk each lane fetches (the DMA
// destination is lane-linear). With >= 4 stages the next K-step's fragments are read from LDS
// while the current MFMAs run.
// Two LDS images:
//   * K-major  [BK/32][rows][32] bf16, 16-B chunk XOR swizzle -> one ds_read_b128 per fragment,
//     for operands whose reduction index is contiguous (W and X in FWD, dY in DGRAD);
//   * MN-major [BK][cols] bf16, 16-B chunk XOR swizzle -> two ds_read_b64_tr_b16 per fragment
//     (gfx950 transpose read), for operands whose output index is contiguous (W in DGRAD, dY and
//     X in WGRAD).
// Both swizzles are bank-conflict-free for the fragment reads.
// Workgroup = 4 waves (2x2) on a BP x BQ tile; grid (tile, split-K slice x stride-2 DGRAD phase,
// client group). The WHOLE linear block id is remapped XCD-aware (bx fastest), so every tile of
// one (group, slice, phase) lands on the same XCD and shares its L2: WGRAD's split-K slices read
// one pixel chunk of dY and X from all their tiles.
// Split-K: WGRAD adds fp32 partials atomically into the zeroed gradient; FWD / DGRAD (grids too
// small to fill the CUs: one client, deep layers) store per-split fp32 slices and a streaming
// epilogue kernel sums them and applies the fused epilogue (BN statistics / BN backward reduce).
//
// Reference parity: replaces the stock nn.Conv2d / nn.Linear of MnistCnn
// (reference lab/tutorial_1a/hfl_complete.py:43-61) and the ResNets of the north-star configs.
#include "ddl_common.h"

#include <cstdlib>

struct ConvArgs {
  const void* x;         // [G][N][H][W][C] bf16
  const void* w;         // [G][K][R][S][C] bf16
  const void* dy;        // [G][N][P][Q][K] bf16
  void* out;             // FWD y bf16 | DGRAD dx bf16 | WGRAD dw fp32
  float* stats;          // FWD: per-channel [sum(K), sumsq(K)] fp32 accumulators (optional)
  const float* bias;     // FWD: [K] fp32 (optional)
  const void* residual;  // DGRAD: bf16 added to dx (optional), same layout as out
  const void* mask;      // DGRAD: dx *= (mask > 0) (optional), same layout as out
  const void* zero;      // legacy zero page (padding now reads past the buffer descriptor's range)
  long long x_gs, w_gs, dy_gs, out_gs, bias_gs, stats_gs;
  int G, N, H, W, C, K, R, S, P, Q, stride, pad;
  int relu, accumulate, split_k;
  int stats_stripes;     // stats: q-tile t adds into stripe t % stripes of [stripes][2*Pd] (<=1: one)
  // DGRAD fused BatchNorm-backward reduce (optional): with bn_x set, `stats` receives per channel
  // (sum dy_m, sum dy_m * xhat) of the stored (masked, residual-added) output, xhat =
  // (bn_x - bn_mean) * bn_rstd — the reduce pass of the preceding BN's backward.
  const void* bn_x;      // BN input (the previous conv's output), same layout as out
  const float* bn_mean;  // [G][C]
  const float* bn_rstd;  // [G][C]
  // FWD / DGRAD split-K (small grids): with split_k > 1 the kernel stores raw fp32 partial sums
  // to partial[split][G][rows][Pd] and conv_splitk_epilogue applies the epilogue above.
  float* partial;
  long long partial_cap;  // floats available at `partial` (0: no split-K for FWD / DGRAD)
  // DGRAD: ReLU mask recomputed from the BN input instead of read: keep dx where
  // bn_x * mask_scale + mask_shift > 0 (the forward bn_apply's pre-activation; needs bn_x)
  const float* mask_scale;  // [G][C]
  const float* mask_shift;
  // DGRAD residual on the stride-2 subgrid (res_sub = 2): `residual` is compact
  // [G][N][ceil(H/2)][ceil(W/2)][C] (group stride res_gs) and adds to the dx pixels (2i, 2j) only —
  // the gradient of a 1x1 / stride-2 projection shortcut, computed without the 3/4 zero pixels.
  long long res_gs;
  int res_sub;
  // WGRAD: every dW contribution is multiplied by gscale before it is added. gscale = -lr with
  // `out` = the fp32 master weights applies a plain SGD step inside the backward ("direct SGD",
  // fl/local.py): no gradient buffer to zero or re-read for the conv weights.
  float gscale;
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

typedef __attribute__((address_space(3))) s4v lds_s4v;

// x / d for 0 <= x < 2^31 via a multiply-high (round-up method); built once per block.
struct FastDiv {
  uint32_t m;
  int s;  // 0 => d == 1
};
__device__ __forceinline__ FastDiv make_fdiv(uint32_t d) {
  FastDiv f;
  if (d <= 1) { f.m = 0; f.s = 0; return f; }
  const int l = 32 - __clz(d - 1);
  f.m = (uint32_t)((((1ull << 32) * ((1ull << l) - d)) / d) + 1);
  f.s = l;
  return f;
}
__device__ __forceinline__ int fdiv(int x, FastDiv f) {
  if (f.s == 0) return x;
  const uint32_t t = __umulhi((uint32_t)x, f.m);
  return (int)((t + (((uint32_t)x - t) >> 1)) >> (f.s - 1));
}

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

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void cta_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Wave-instruction geometry of one operand tile image (per K-step):
//   K-major  ROWS x BK : NI = ROWS*BK/512 instructions, instr j -> sub-tile u = j/(ROWS/16),
//                        rows 16*(j%(ROWS/16)) .. +15 ; lane L -> row +L/4, phys chunk L%4
//   MN-major BK x COLS : NI = BK*COLS/512, instr j -> k-rows (512/COLS)*j .. ; lane L ->
//                        k-row + L/(COLS/8), phys chunk L%(COLS/8)
// WLP = waves along P (1, 2 or 4; the other 4/WLP waves split Q). 2x2 is the default; 1x4 gives
// a 64-channel tile (layer-1 convs) 64x64 per wave instead of 32x(BQ/2).
//
// HALO (FWD / DGRAD of 3x3, stride 1, pad 1 convs whose BQ-pixel tile is whole image rows): the
// activation operand is NOT streamed per K-step. The reduction runs channel-block-major (32
// channels, then the 9 taps), and per channel block the tile's rows plus a one-pixel halo
// ((BQ/W + 2) x (W + 2) pixels x 32 channels) are DMA'd into LDS once; the 9 taps read shifted
// windows of that image. The 9x per-tap re-fetch of the activations through L2 -> LDS-DMA was the
// bound of the streamed kernel on the 32x32 / 16x16 layers (PMC: MFMA busy ~20%, L2 -> CU reads
// ~9x the activation bytes). The next block's halo is DMA'd one piece per K-step during taps
// NS-1 .. of the current block into the other of two halo buffers; the weight operand keeps
// the NS-deep per-step ring. Halo image: 64 B per pixel, 16-B chunk c stored at c ^ 2*((pixel>>2)&1):
// for the ds_read_b128 lane groups ({0-3,12-15,20-27}, ...) every window of 16 consecutive
// pixels, at any shift (every tap of a fragment on >= 16-wide rows), reads conflict-free.
//
// The kernel body is a device function over a VIRTUAL block id `lin` of a virtual (gx, gy, gz)
// grid, so that two convolutions can share one launch (conv_pair_kernel below); the plain
// conv_igemm_kernel passes its own linear block id and gridDim.
template <int MODE, int BP, int BQ, int BK, int NS, int WLP, bool HALO>
struct ConvTile {
  static constexpr bool HALO_FD = HALO && MODE != MODE_WGRAD;
  static constexpr bool HALO_W = HALO && MODE == MODE_WGRAD;
  static constexpr int P_BYTES = BP * BK * 2, Q_BYTES = HALO_W ? 2 * 4 * 1024 : BQ * BK * 2;
  static constexpr int HPW_MAX = HALO_FD ? (BQ >= 256 ? 10 - NS : (10 - NS < 4 ? 10 - NS : 4)) : 0;
  static constexpr int SMEM = HALO_FD ? NS * P_BYTES + 2 * HPW_MAX * 4 * 1024 : NS * (P_BYTES + Q_BYTES);
};

template <int MODE, int BP, int BQ, int BK, int NS, int WLP, bool HALO>
__device__ __forceinline__ void conv_body(const ConvArgs& a, char* smem, int lin, int gx, int gy,
                                          int gz) {
  constexpr bool HALO_FD = HALO && MODE != MODE_WGRAD;  // halo FWD / DGRAD (channel-block-major)
  constexpr bool HALO_W = HALO && MODE == MODE_WGRAD;   // halo WGRAD (per-step row window)
  constexpr int WPW = 2;  // halo WGRAD: window pieces per wave per stage
  constexpr int P_BYTES = BP * BK * 2, Q_BYTES = HALO_W ? WPW * 4 * 1024 : BQ * BK * 2;
  constexpr int STAGE = P_BYTES + Q_BYTES;
  static_assert(!HALO || (BK == 32 && NS >= 4), "halo: BK 32, >= 4 stages");
  static_assert(!HALO_W || (BP == 64 && BQ == 288 && WLP == 2), "halo WGRAD: 64 x (9 taps x 32) tiles");
  // halo pieces (1 KiB DMA wave-instructions) per wave: issued at taps NS-1 .. 8 of a block
  constexpr int HPW_MAX = HALO_FD ? (BQ >= 256 ? 10 - NS : (10 - NS < 4 ? 10 - NS : 4)) : 0;
  constexpr int HALO_BYTES = HPW_MAX * 4 * 1024;
  constexpr int SMEM_BYTES = HALO_FD ? NS * P_BYTES + 2 * HALO_BYTES : NS * STAGE;
  constexpr int WP = BP / WLP, WQ = BQ / (4 / WLP), TP = WP / 16, TQ = WQ / 16;
  static_assert(WLP == 1 || WLP == 2 || WLP == 4, "4 waves");
  constexpr bool P_KMAJOR = (MODE == MODE_FWD);
  constexpr bool Q_KMAJOR = (MODE != MODE_WGRAD);
  constexpr int P_NI = BP * BK / 512, Q_NI = BQ * BK / 512;  // wave-instructions per tile
  constexpr int P_PW = P_NI / 4, Q_PW = Q_NI / 4;            // per wave
  constexpr int LPS = P_PW + (HALO_W ? WPW : Q_PW);          // DMA instructions per wave per stage
  static_assert(P_PW >= 1 && Q_PW >= 1, "tile too small");
  static_assert(SMEM_BYTES == ConvTile<MODE, BP, BQ, BK, NS, WLP, HALO>::SMEM, "LDS size");

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wp = wid / (4 / WLP), wq = wid % (4 / WLP);
  // XCD-aware decode of the linear block id: the dispatcher deals workgroups round-robin over
  // the 8 XCDs; consecutive logical ids u share an XCD (and its L2).
  const int u = xcd_remap(lin, gx * gy * gz);
  // Stride-2 DGRAD keeps the per-phase remap of the tile index only (measured: grouping the
  // phases of a tile, or the tiles of a phase, on one XCD both lose 10-20% there).
  const bool per_phase = MODE == MODE_DGRAD && a.stride == 2;
  const int bx = per_phase ? xcd_remap(lin % gx, gx) : u % gx;
  const int by = per_phase ? (lin / gx) % gy : (u / gx) % gy;
  const int g = per_phase ? lin / (gx * gy) : u / (gx * gy);
  const int H = a.H, W = a.W, C = a.C, K = a.K, R = a.R, S = a.S, P = a.P, Q = a.Q;
  const int st = a.stride, pd = a.pad;
  const int RSC = R * S * C;

  int Pd, Qd, Kr;
  if constexpr (MODE == MODE_FWD) { Pd = K; Qd = a.N * P * Q; Kr = RSC; }
  else if constexpr (MODE == MODE_DGRAD) { Pd = C; Qd = a.N * H * W; Kr = R * S * K; }
  else { Pd = K; Qd = RSC; Kr = a.N * P * Q; }
  const FastDiv div_pq = make_fdiv(P * Q), div_q = make_fdiv(Q);

  // DGRAD at stride 2: sub-pixel phase decomposition. blockIdx.y = phase (a, b); the phase's
  // input pixels (2i+a, 2j+b) only receive taps r = r0 (mod 2), s = s0 (mod 2), so no MFMA or
  // DMA is spent on the 3/4 of (pixel, tap) pairs that hit no output position.
  int ph_a = 0, ph_b = 0, Hs = H, Ws = W, r0 = 0, s0 = 0, tstep = 1, Rn = R, Sn = S;
  constexpr bool PHASED_MODE = (MODE == MODE_DGRAD);
  const bool phased = PHASED_MODE && st == 2;
  const int nph = phased ? 4 : 1;
  if (phased) {
    ph_a = (by >> 1) & 1;
    ph_b = by & 1;
    Hs = (H - ph_a + 1) >> 1;
    Ws = (W - ph_b + 1) >> 1;
    r0 = (ph_a + pd) & 1;
    s0 = (ph_b + pd) & 1;
    Rn = (R - r0 + 1) >> 1;
    Sn = (S - s0 + 1) >> 1;
    tstep = 2;
    Qd = a.N * Hs * Ws;
    Kr = Rn * Sn * K;
  }

  const int ntp = (Pd + BP - 1) / BP;
  const int tile = bx;
  const int p0 = (tile % ntp) * BP, q0 = (tile / ntp) * BQ;
  if (q0 >= Qd) return;  // smaller phases of a phased launch
  const int nsplit = gy / nph, split = by / nph;
  const int nk_total = (Kr + BK - 1) / BK;
  const int per = (nk_total + nsplit - 1) / nsplit;
  const int kt0 = split * per;
  const int kt1 = min(nk_total, kt0 + per);
  if (kt0 >= kt1 && MODE == MODE_WGRAD) return;  // empty split-K slice (atomics: nothing to add)
  const int nk = max(0, kt1 - kt0);  // FWD/DGRAD with no taps still write (zero) outputs

  const bf16_t* X = (const bf16_t*)a.x + (long long)g * a.x_gs;
  const bf16_t* Wt = (const bf16_t*)a.w + (long long)g * a.w_gs;
  const bf16_t* DY = (const bf16_t*)a.dy + (long long)g * a.dy_gs;

  // ---------------- operand sources: buffer descriptors + per-lane base offsets ----------------
  // Every LDS-DMA is `buffer_load_dwordx4 ... offen lds` at byte offset (lane base + wave-uniform
  // cursor). Padding taps, tile overhang and the partial last WGRAD step use an offset beyond
  // the descriptor's range, which the hardware returns as zeros: no branches, no zero page.
  const unsigned x_bytes = (unsigned)((long long)a.N * H * W * C * 2);
  const unsigned w_bytes = (unsigned)((long long)K * RSC * 2);
  const unsigned dy_bytes = (unsigned)((long long)a.N * P * Q * K * 2);
  const __amdgpu_buffer_rsrc_t rX = __builtin_amdgcn_make_buffer_rsrc((void*)X, 0, (int)x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rW = __builtin_amdgcn_make_buffer_rsrc((void*)Wt, 0, (int)w_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rD = __builtin_amdgcn_make_buffer_rsrc((void*)DY, 0, (int)dy_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rP = (MODE == MODE_WGRAD) ? rD : rW;
  const __amdgpu_buffer_rsrc_t rQ = (MODE == MODE_DGRAD) ? rD : rX;
  constexpr unsigned OOB = 0xFFFFFFF0u;
  const int wsc = __builtin_amdgcn_readfirstlane(wid);  // wave id in an SGPR: LDS bases stay scalar

  // P operand: element offset = p_base[i] + wave-uniform cursor term; p_base < 0 = never valid
  int p_base[P_PW];
#pragma unroll
  for (int i = 0; i < P_PW; ++i) {
    const int j = wid + 4 * i;
    if constexpr (P_KMAJOR) {  // FWD weights [K][RSC]: row = output channel
      const int u = j / (BP / 16), rb = 16 * (j % (BP / 16));
      const int row = rb + lane / 4;
      const int col = u * 32 + (((lane & 3) ^ km_swz(row)) << 3);
      const int kk = p0 + row;
      p_base[i] = kk < K ? kk * RSC + col : -1;
    } else {
      constexpr int CPR = BP / 8, RPIN = 512 / BP;
      const int kr = RPIN * j + lane / CPR;                 // reduction row within the stage
      const int col = p0 + (((lane % CPR) ^ mn_swz<BP>(kr)) << 3);
      if constexpr (MODE == MODE_DGRAD)  // weights [k][(r,s)][c]: + t_c*RSC + (r*S+s)*C
        p_base[i] = col < C ? kr * RSC + col : -1;
      else  // WGRAD dY [pix][k]: + kg*K ; the pixel row must stay < Kr
        p_base[i] = col < K ? kr * K + col : -1;
    }
  }
  f4v acc[TP][TQ];
#pragma unroll
  for (int i = 0; i < TP; ++i)
#pragma unroll
    for (int j = 0; j < TQ; ++j) acc[i][j] = (f4v){0.f, 0.f, 0.f, 0.f};
  auto mfma_all = [&](const s8v* pf, const s8v* qf) {
#pragma unroll
    for (int ti = 0; ti < TP; ++ti)
#pragma unroll
      for (int tj = 0; tj < TQ; ++tj)
        acc[ti][tj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pf[ti], qf[tj], acc[ti][tj], 0, 0, 0);
  };

  if constexpr (HALO_FD) {
    // host contract (halo_ok): stride 1, R = S = 3, pad 1, P = H, Q = W, tiles of whole rows of
    // one image or of whole images, halo pieces per wave <= HPW_MAX; no split-K, no phases.
    // The tile is TRh whole rows of one image (BQ <= H*W) or BQ/(H*W) whole images; its halo
    // image holds one (TRh+2) x (W+2) segment per image covered.
    const int CRh = (MODE == MODE_FWD) ? C : K;  // channels of the staged activation
    const int ncb = CRh >> 5;
    const int W2 = W + 2, TRh = min(BQ / W, H);
    const int HS = (TRh + 2) * W2, TPX = TRh * W;  // halo / output pixels per segment
    const int hpx = (BQ / TPX) * HS;
    const int hpw = (((hpx + 15) >> 4) + 3) >> 2;  // pieces per wave
    const int img = q0 / (H * W);
    const int row0 = (q0 - img * H * W) / W;
    const int img_base = img * H * W;
    const __amdgpu_buffer_rsrc_t rA = (MODE == MODE_FWD) ? rX : rD;
    char* const halo0 = smem + NS * P_BYTES;

    // Everything per lane that does not change with the channel block is computed once, so the
    // K-steps (taps fully unrolled) carry no address arithmetic beyond a scalar base:
    //   hsrc[j]     source element offset (block 0) of this lane's 16 B of halo piece j, -1 = zero;
    //   qoff[r][t]  LDS byte offset, inside a halo image, of Q fragment t for tap r.
    int hsrc[HPW_MAX];
    {
      const FastDiv div_w2 = make_fdiv(W2), div_hs = make_fdiv(HS);
#pragma unroll
      for (int j = 0; j < HPW_MAX; ++j) {
        const int hp = (wsc + 4 * j) * 16 + (lane >> 2);
        const int seg = fdiv(hp, div_hs), sp = hp - seg * HS;
        const int hr = fdiv(sp, div_w2), hc = sp - hr * W2;
        const int h = row0 - 1 + hr, w = hc - 1;
        const int lc = (lane & 3) ^ (((hp >> 2) & 1) << 1);
        const bool ok = (j < hpw) & (hp < hpx) & ((unsigned)h < (unsigned)H) & ((unsigned)w < (unsigned)W);
        hsrc[j] = ok ? (img_base + seg * H * W + h * W + w) * CRh + lc * 8 : -1;
      }
    }
    int qoff[9][TQ];
#pragma unroll
    for (int t = 0; t < TQ; ++t) {
      const int lpix = wq * WQ + t * 16 + (lane & 15);
      const int seg = lpix / TPX, sp = lpix - seg * TPX;
      const int th = sp / W, tw = sp - th * W;
      const int hq = seg * HS + th * W2 + tw;
#pragma unroll
      for (int r = 0; r < 9; ++r) {
        const int tr = r / 3, ts = r % 3;
        const int hp = hq + ((MODE == MODE_FWD) ? tr * W2 + ts : (2 - tr) * W2 + (2 - ts));
        qoff[r][t] = hp * 64 + (((lane >> 4) ^ (((hp >> 2) & 1) << 1)) << 4);
      }
    }

    // DMA ops a stage issues per wave: its weight pieces + one halo piece at taps NS-1 .. NS-2+hpw
    auto stage_ops = [&](int s) {
      const int t = s % 9 - (NS - 1);
      return P_PW + ((t >= 0) & (t < hpw) ? 1 : 0);
    };
    // ops issued after stage s0 up to stage s1 (inclusive, clipped to the last stage)
    auto ops_between = [&](int s0, int s1, int nkk) {
      int n = 0;
      for (int s = s0 + 1; s <= s1 && s < nkk; ++s) n += stage_ops(s);
      return n;
    };
    // s_waitcnt vmcnt needs an immediate: dispatch the (wave-uniform) count
    auto wait_dyn = [&](int n) {
      switch (n) {
        case 0: wait_vm<0>(); break;
        case 1: wait_vm<1>(); break;
        case 2: wait_vm<2>(); break;
        case 3: wait_vm<3>(); break;
        case 4: wait_vm<4>(); break;
        case 5: wait_vm<5>(); break;
        case 6: wait_vm<6>(); break;
        case 7: wait_vm<7>(); break;
        default: wait_vm<0>(); break;  // conservative
      }
    };
    // stage (scb, stap): the weights of tap stap / channel block scb into ring slot `slot`, and
    // piece stap-(NS-1) of block scb+1's halo (taps NS-1.. only: the other halo buffer's last
    // reader, block scb-1, has then retired on every wave)
    auto issue_h = [&](int slot, int scb, int stap) {
      char* Ps = smem + slot * P_BYTES;
      const int pcur = (MODE == MODE_FWD) ? stap * C + scb * 32 : scb * 32 * RSC + stap * C;
#pragma unroll
      for (int i = 0; i < P_PW; ++i) {
        const unsigned off = p_base[i] >= 0 ? (unsigned)(p_base[i] + pcur) * 2u : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rP, (__attribute__((address_space(3))) void*)(Ps + (wsc + 4 * i) * 1024), 16, off, 0, 0, 0);
      }
      const int j = stap - (NS - 1);
      if (j >= 0 && j < HPW_MAX && j < hpw) {
        const int src = hsrc[j < HPW_MAX ? j : 0];
        const unsigned off = (src >= 0 && scb + 1 < ncb) ? (unsigned)(src + (scb + 1) * 32) * 2u : OOB;
        char* hb = halo0 + ((scb + 1) & 1) * HALO_BYTES + (wsc + 4 * j) * 1024;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (__attribute__((address_space(3))) void*)hb, 16, off,
                                                 0, 0, 0);
      }
    };
    auto load_frags_h = [&](int slot, const char* hb, int tap, s8v* pf, s8v* qf) {
      const char* Ps = smem + slot * P_BYTES;
#pragma unroll
      for (int t = 0; t < TP; ++t) {
        if constexpr (P_KMAJOR) pf[t] = km_frag<BP>(Ps, wp * WP + t * 16, 0, lane);
        else pf[t] = mn_frag<BP>(Ps, wp * WP + t * 16, 0, lane);
      }
#pragma unroll
      for (int t = 0; t < TQ; ++t) qf[t] = *(const s8v*)(hb + qoff[tap][t]);
    };

    const int nkh = ncb * 9;
    // prologue: block 0's halo, then stages 0 .. NS-2 (block 0, taps 0 .. NS-2)
#pragma unroll
    for (int j = 0; j < HPW_MAX; ++j) {
      if (j < hpw) {
        const unsigned off = hsrc[j] >= 0 ? (unsigned)hsrc[j] * 2u : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rA, (__attribute__((address_space(3))) void*)(halo0 + (wsc + 4 * j) * 1024), 16, off, 0, 0, 0);
      }
    }
#pragma unroll
    for (int s = 0; s < NS - 1; ++s) issue_h(s, 0, s);
    wait_dyn(ops_between(0, NS - 2, nkh));  // retire stage 0 (and the halo before it)
    cta_barrier();
    s8v pfA[TP], qfA[TQ], pfB[TP], qfB[TQ];
    load_frags_h(0, halo0, 0, pfA, qfA);
    for (int cb = 0; cb < ncb; ++cb) {
      const char* hb = halo0 + (cb & 1) * HALO_BYTES;
      const char* hbn = halo0 + ((cb + 1) & 1) * HALO_BYTES;
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int i = cb * 9 + tap;
        wait_dyn(ops_between(i + 1, i + NS - 2, nkh));  // retire stage i+1; stages i+2.. may fly
        cta_barrier();
        if (i + NS - 1 < nkh) {
          issue_h((i + NS - 1) % NS, cb + (tap + NS - 1) / 9, (tap + NS - 1) % 9);
        }
        // the next step's fragments (past the last step: a stale read, unused)
        load_frags_h((i + 1) % NS, tap == 8 ? hbn : hb, tap == 8 ? 0 : tap + 1, pfB, qfB);
        mfma_all(pfA, qfA);
#pragma unroll
        for (int t = 0; t < TP; ++t) pfA[t] = pfB[t];
#pragma unroll
        for (int t = 0; t < TQ; ++t) qfA[t] = qfB[t];
      }
    }
  } else {
  // Q operand
  int q_base[Q_PW], q_h[Q_PW], q_w[Q_PW];
#pragma unroll
  for (int i = 0; i < (HALO_W ? 0 : Q_PW); ++i) {
    const int j = wid + 4 * i;
    if constexpr (Q_KMAJOR) {
      const int u = j / (BQ / 16), rb = 16 * (j % (BQ / 16));
      const int row = rb + lane / 4;
      const int kd = u * 32 + (((lane & 3) ^ km_swz(row)) << 3);  // k offset within stage
      const int qq = q0 + row;
      if constexpr (MODE == MODE_FWD) {
        // X pixel (n, op*st - pd + r, oq*st - pd + s): + (t_r*W + t_s)*C + t_c
        const int n = qq / (P * Q), rem = qq - n * (P * Q);
        const int op = rem / Q, oq = rem - op * Q;
        q_h[i] = op * st - pd;
        q_w[i] = oq * st - pd;
        q_base[i] = ((n * H + q_h[i]) * W + q_w[i]) * C + kd;
      } else {
        // dY pixel (n, q_h - jr, q_w - js) for the jr-th / js-th tap of this phase
        const int n = qq / (Hs * Ws), rem = qq - n * (Hs * Ws);
        const int hi = rem / Ws, wi = rem - hi * Ws;
        if (st <= 2) {
          q_h[i] = hi + (ph_a + pd - r0) / st;
          q_w[i] = wi + (ph_b + pd - s0) / st;
          q_base[i] = ((n * P + q_h[i]) * Q + q_w[i]) * K + kd;
        } else {  // generic stride: recomputed per step (rare)
          q_h[i] = hi + pd;
          q_w[i] = wi + pd;
          q_base[i] = n * P * Q;
        }
      }
      if (qq >= Qd) q_h[i] = -(1 << 28);  // tile overhang: always out of range
      if constexpr (MODE == MODE_DGRAD) if (st > 2) q_w[i] = (q_w[i] & 0xffff) | (kd << 16);
    } else {  // WGRAD X gather MN-major: k-row = pixel, col = (r, s, c)
      constexpr int CPR = BQ / 8, RPIN = 512 / BQ;
      const int kr = RPIN * j + lane / CPR;
      const int col = q0 + (((lane % CPR) ^ mn_swz<BQ>(kr)) << 3);
      q_base[i] = kr;
      if (col < Qd) {
        const int rs = col / C;
        const int c = col - rs * C;
        const int r = rs / S;
        q_h[i] = r - pd;
        q_w[i] = ((rs - r * S - pd) & 0xffff) | (c << 16);  // packed (s - pad, c)
      } else {
        q_h[i] = -(1 << 28);
        q_w[i] = 0;
      }
    }
  }

  // WGRAD: per-lane output-pixel cursor (n, op, oq) of k-row kr, advanced by BK pixels per step
  // with constant carries (no divisions in the loop)
  int wn[MODE == MODE_WGRAD ? Q_PW : 1], wop[MODE == MODE_WGRAD ? Q_PW : 1],
      woq[MODE == MODE_WGRAD ? Q_PW : 1];
  int w_dn = 0, w_dp = 0, w_dq = 0;
  if constexpr (MODE == MODE_WGRAD && !HALO_W) {
    const int pq = P * Q;
    w_dn = BK / pq;
    w_dp = (BK - w_dn * pq) / Q;
    w_dq = BK - w_dn * pq - w_dp * Q;
#pragma unroll
    for (int i = 0; i < Q_PW; ++i) {
      const int pix = kt0 * BK + q_base[i];
      wn[i] = fdiv(pix, div_pq);
      const int rem = pix - wn[i] * pq;
      wop[i] = fdiv(rem, div_q);
      woq[i] = rem - wop[i] * Q;
    }
  }

  // Halo WGRAD (3x3 / stride 1 / pad 1, W in {8, 16, 32}; host: wgrad_halo_ok): a K-step is 32
  // output pixels = TRW = 32/W whole rows of one image; its activation operand is those rows plus
  // a one-pixel halo, (TRW+2) x (W+2) pixels x 32 channels, DMA'd once and read by all 9 taps of
  // the tile (64 output channels x 9 taps x 32 channels) as shifted windows, instead of one
  // gathered DMA per tap. Pixel rows are 64 B; 16-B chunk c at c ^ 2*((pixel>>3)&1) keeps the
  // transpose reads (8 pixels {0-3, 8-11} + shift per lane group) conflict-free for W >= 16.
  int w_lane[WPW], w_hr[WPW], w_ok[WPW], qadr[HALO_W ? TQ : 1][2];
  int wpix = 0, wrow = 0, TRW = 1;
  if constexpr (HALO_W) {
    TRW = 32 / W;
    const int W2 = W + 2, hpx = (TRW + 2) * W2, c0 = q0 / 9;
#pragma unroll
    for (int j = 0; j < WPW; ++j) {
      const int hp = (wsc + 4 * j) * 16 + (lane >> 2);
      const int hr = hp / W2, hc = hp - hr * W2;
      const int lc = (lane & 3) ^ (((hp >> 3) & 1) << 1);
      w_ok[j] = (hp < hpx) & (hc >= 1) & (hc <= W);
      w_hr[j] = hr - 1;
      w_lane[j] = ((hr - 1) * W + (hc - 1)) * C + c0 + lc * 8;
    }
    const int g4 = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
#pragma unroll
    for (int t = 0; t < TQ; ++t) {
      const int f = wq * TQ + t, tap = f >> 1, cb16 = f & 1;
      const int r = tap / 3, sx = tap - 3 * r;
      const int col = cb16 * 16 + 4 * p4, cc = col >> 3, half = (col >> 2) & 1;
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int k = 8 * g4 + q4 + 4 * e;
        const int tt = k / W, ww = k - tt * W;
        const int hp = (tt + r) * W2 + ww + sx;
        qadr[t][e] = hp * 64 + ((cc ^ (((hp >> 3) & 1) << 1)) << 4) + half * 8;
      }
    }
    wpix = kt0 * BK;
    wrow = (wpix % (H * W)) / W;
  }

  // reduction cursor for FWD/DGRAD: tap (t_r, t_s) [jr, js = tap index within the phase],
  // channel run t_c; issue() is called for consecutive K-steps, so it advances without divisions
  const int CR = (MODE == MODE_FWD) ? C : K;  // contiguous reduction run per tap
  int kg_run = kt0 * BK, t_r = 0, t_s = 0, t_c = 0, jr = 0, js = 0;
  if constexpr (MODE != MODE_WGRAD) {
    const int ti = kg_run / CR;  // tap index among the (phase's) valid taps
    t_c = kg_run - ti * CR;
    jr = ti / Sn;
    js = ti - jr * Sn;
    t_r = r0 + tstep * jr;
    t_s = s0 + tstep * js;
  }

  auto issue = [&](int slot) {
    char* Ps = smem + slot * STAGE;
    char* Qs = Ps + P_BYTES;
    const int kg = kg_run;
    // ---- P ----
    int pcur;  // wave-uniform element offset of this step
    if constexpr (MODE == MODE_FWD) pcur = kg;
    else if constexpr (MODE == MODE_DGRAD) pcur = t_c * RSC + (t_r * S + t_s) * C;
    else pcur = kg * K;
#pragma unroll
    for (int i = 0; i < P_PW; ++i) {
      bool ok = p_base[i] >= 0;
      if constexpr (MODE == MODE_WGRAD) {
        constexpr int RPIN = 512 / BP, CPR = BP / 8;
        ok = ok && (RPIN * (wid + 4 * i) + lane / CPR) < Kr - kg;
      }
      const unsigned off = ok ? (unsigned)(p_base[i] + pcur) * 2u : OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rP, (__attribute__((address_space(3))) void*)(Ps + (wsc + 4 * i) * 1024), 16, off, 0, 0, 0);
    }
    // ---- Q ----  (wave-uniform tap term computed once; per lane: add + range test + select)
    if constexpr (HALO_W) {
#pragma unroll
      for (int j = 0; j < WPW; ++j) {
        const bool ok = w_ok[j] && (unsigned)(wrow + w_hr[j]) < (unsigned)H;
        const unsigned off = ok ? (unsigned)(w_lane[j] + wpix * C) * 2u : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rX, (__attribute__((address_space(3))) void*)(Qs + (wsc + 4 * j) * 1024), 16, off, 0, 0, 0);
      }
      wpix += BK;
      wrow += TRW;
      if (wrow >= H) wrow = 0;
    }
    int qcur = 0;
    if constexpr (MODE == MODE_FWD) qcur = (t_r * W + t_s) * C + t_c;
    else if constexpr (MODE == MODE_DGRAD) qcur = t_c - (jr * Q + js) * K;
#pragma unroll
    for (int i = 0; i < (HALO_W ? 0 : Q_PW); ++i) {
      unsigned off = OOB;
      if constexpr (MODE == MODE_FWD) {
        const int ih = q_h[i] + t_r, iw = q_w[i] + t_s;
        const bool ok = ((unsigned)ih < (unsigned)H) & ((unsigned)iw < (unsigned)W);
        off = ok ? (unsigned)(q_base[i] + qcur) * 2u : OOB;
      } else if constexpr (MODE == MODE_DGRAD) {
        if (st <= 2) {
          const int ph = q_h[i] - jr, pw = q_w[i] - js;
          const bool ok = ((unsigned)ph < (unsigned)P) & ((unsigned)pw < (unsigned)Q);
          off = ok ? (unsigned)(q_base[i] + qcur) * 2u : OOB;
        } else {
          int ph = q_h[i] - t_r, pw = (q_w[i] & 0xffff) - t_s;
          const int kd = q_w[i] >> 16;
          if (ph >= 0 && pw >= 0 && ph % st == 0 && pw % st == 0) {
            ph /= st;
            pw /= st;
            if (ph < P && pw < Q) off = (unsigned)((q_base[i] + ph * Q + pw) * K + t_c + kd) * 2u;
          }
        }
      } else {
        const int sw = (int)(short)(q_w[i] & 0xffff), c = q_w[i] >> 16;
        const int ih = wop[i] * st + q_h[i], iw = woq[i] * st + sw;
        const bool ok = (q_base[i] < Kr - kg) & ((unsigned)ih < (unsigned)H) &
                        ((unsigned)iw < (unsigned)W);
        off = ok ? (unsigned)(((wn[i] * H + ih) * W + iw) * C + c) * 2u : OOB;
        // advance this lane's pixel by BK: (n, op, oq) += (w_dn, w_dp, w_dq) with carries
        int oq = woq[i] + w_dq;
        const int cq = oq >= Q;
        woq[i] = cq ? oq - Q : oq;
        int op = wop[i] + w_dp + cq;
        const int cp = op >= P;
        wop[i] = cp ? op - P : op;
        wn[i] += w_dn + cp;
      }
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rQ, (__attribute__((address_space(3))) void*)(Qs + (wsc + 4 * i) * 1024), 16, off, 0, 0, 0);
    }
    // advance the reduction cursor by one K-step
    kg_run += BK;
    if constexpr (MODE != MODE_WGRAD) {
      t_c += BK;
      if (t_c >= CR) {
        t_c = 0;
        t_s += tstep;
        ++js;
        if (t_s >= S) { t_s = s0; js = 0; t_r += tstep; ++jr; }
      }
    }
  };

  auto load_frags = [&](const char* Ps, int u, s8v* pf, s8v* qf) {
    const char* Qs = Ps + P_BYTES;
#pragma unroll
    for (int t = 0; t < TP; ++t) {
      if constexpr (P_KMAJOR) pf[t] = km_frag<BP>(Ps, wp * WP + t * 16, u, lane);
      else pf[t] = mn_frag<BP>(Ps, wp * WP + t * 16, u, lane);
    }
#pragma unroll
    for (int t = 0; t < TQ; ++t) {
      if constexpr (HALO_W) {
        s4v r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(Qs + qadr[t][0]));
        s4v r2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(Qs + qadr[t][1]));
        s8v r;
        r[0] = r1[0]; r[1] = r1[1]; r[2] = r1[2]; r[3] = r1[3];
        r[4] = r2[0]; r[5] = r2[1]; r[6] = r2[2]; r[7] = r2[3];
        qf[t] = r;
      } else if constexpr (Q_KMAJOR) qf[t] = km_frag<BQ>(Qs, wq * WQ + t * 16, u, lane);
      else qf[t] = mn_frag<BQ>(Qs, wq * WQ + t * 16, u, lane);
    }
  };
  // prologue: stages 0 .. NS-2 in flight
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nk) issue(s);

  if constexpr (NS >= 4 && BK == 32) {
    // Fragment prefetch: the fragments of K-step i+1 are read from LDS while the MFMAs of step i
    // run (two register sets). Stage i+1 is waited for one step early, so NS-3 stages stay in
    // flight across each barrier. WAR on the slot refilled at step i (stage i-1's): its fragments
    // were consumed by step i-1's MFMAs, which every wave issued before this step's barrier.
    // The prefetch read is unconditional (past the last step it reads a stale slot, unused) so
    // the compiler's lgkmcnt tracking stays exact: a conditional read would make it wait for the
    // freshly issued reads before the current MFMAs.
    s8v pfA[TP], qfA[TQ], pfB[TP], qfB[TQ];
    if (NS - 2 < nk) wait_vm<(NS - 2) * LPS>();
    else wait_vm<0>();
    cta_barrier();
    load_frags(smem, 0, pfA, qfA);
    for (int i = 0; i < nk; ++i) {
      if (i + NS - 2 < nk) wait_vm<(NS - 3) * LPS>();  // retire stage i+1 (stages i+2.. may fly)
      else wait_vm<0>();
      cta_barrier();
      if (i + NS - 1 < nk) issue((i + NS - 1) % NS);
      load_frags(smem + ((i + 1) % NS) * STAGE, 0, pfB, qfB);
      mfma_all(pfA, qfA);
#pragma unroll
      for (int t = 0; t < TP; ++t) pfA[t] = pfB[t];
#pragma unroll
      for (int t = 0; t < TQ; ++t) qfA[t] = qfB[t];
    }
  } else {
    for (int i = 0; i < nk; ++i) {
      // retire stage i: at most (stages issued after it) * LPS DMA ops may stay outstanding
      if constexpr (NS >= 3) {
        if (i + NS - 2 < nk) wait_vm<(NS - 2) * LPS>();
        else if (NS >= 4 && i + NS - 3 < nk) wait_vm<(NS >= 4 ? (NS - 3) * LPS : 0)>();
        else wait_vm<0>();
      } else {
        wait_vm<0>();
      }
      cta_barrier();  // stage i visible to all waves; slot of stage i-1 free for reuse
      if (i + NS - 1 < nk) issue((i + NS - 1) % NS);
      const char* Ps = smem + (i % NS) * STAGE;
      // within a stage, the next 32-deep fragments load while the current ones feed the MFMAs
      s8v pfA[TP], qfA[TQ], pfB[TP], qfB[TQ];
      load_frags(Ps, 0, pfA, qfA);
#pragma unroll
      for (int u = 0; u < BK / 32; u += 2) {
        if (u + 1 < BK / 32) load_frags(Ps, u + 1, pfB, qfB);
        mfma_all(pfA, qfA);
        if (u + 1 < BK / 32) {
          if (u + 2 < BK / 32) load_frags(Ps, u + 2, pfA, qfA);
          mfma_all(pfB, qfB);
        }
      }
    }
  }
  }  // !HALO

  // ---------------- epilogue ----------------
  const int lq = lane & 15, lp = 4 * (lane >> 4);
  if constexpr (MODE == MODE_FWD || MODE == MODE_DGRAD) {
    if (nsplit > 1) {  // raw fp32 partial slice [split][g][rows][Pd]; conv_splitk_epilogue finishes
      const long long rows = MODE == MODE_FWD ? (long long)a.N * P * Q : (long long)a.N * H * W;
      float* PO = a.partial + ((long long)split * a.G + g) * rows * Pd;
#pragma unroll
      for (int ti = 0; ti < TP; ++ti) {
        const int p = p0 + wp * WP + ti * 16 + lp;
#pragma unroll
        for (int tj = 0; tj < TQ; ++tj) {
          const int q = q0 + wq * WQ + tj * 16 + lq;
          if (p < Pd && q < Qd) {
            long long o = (long long)q * Pd + p;
            if (phased) {
              const int n = q / (Hs * Ws), rem = q - n * (Hs * Ws);
              const int hi = rem / Ws, wi = rem - hi * Ws;
              o = ((long long)(n * H + 2 * hi + ph_a) * W + 2 * wi + ph_b) * Pd + p;
            }
            *(f4v*)(PO + o) = acc[ti][tj];
          }
        }
      }
      return;
    }
    bf16_t* O = (bf16_t*)a.out + (long long)g * a.out_gs;
    const float* bias = a.bias ? a.bias + (long long)g * a.bias_gs : nullptr;
    const bool rsub = MODE == MODE_DGRAD && a.res_sub == 2;
    const bf16_t* res = a.residual ? (const bf16_t*)a.residual + (long long)g * (rsub ? a.res_gs : a.out_gs)
                                   : nullptr;
    const bf16_t* msk = a.mask ? (const bf16_t*)a.mask + (long long)g * a.out_gs : nullptr;
    // striped accumulation: blocks of different pixel tiles hit different copies, so the fp32
    // atomics of thousands of blocks do not serialise on the same few cache lines
    float* stats = a.stats ? a.stats + (long long)g * a.stats_gs +
                                 (a.stats_stripes > 1 ? (long long)((tile / ntp) % a.stats_stripes) * 2 * Pd : 0)
                           : nullptr;
    const bf16_t* bnx = (MODE == MODE_DGRAD && a.bn_x) ? (const bf16_t*)a.bn_x + (long long)g * a.out_gs
                                                        : nullptr;
    const bool want_stats = stats && (MODE == MODE_FWD || bnx);
    // LDS-restaged epilogue. The MFMA accumulator gives a lane 4 channels of one pixel, so a direct
    // epilogue moves 8 B per lane at a pixel stride (residual / mask / BN-input reads, output
    // stores): 4 instructions share every 128-B line. Instead, per 16-pixel strip of every wave
    // column (tj), the tile's fp32 accumulators go through LDS and come back as 8 consecutive
    // channels of one pixel per thread: 16-B coalesced loads / stores, and per-thread channel
    // chunks fixed across strips for the BN statistics.
    {
      constexpr int NPX = (4 / WLP) * 16;  // pixels per strip
      constexpr int LROW = BP + 4;         // fp32 row pitch (+16 B: conflict-free b128 writes)
      constexpr int NCH = BP / 8;          // 8-channel chunks per pixel
      constexpr int PSTEP = 256 / NCH;     // pixels per thread-iteration
      static_assert(NPX * LROW * 4 <= SMEM_BYTES && 256 * 16 * 4 <= SMEM_BYTES, "epilogue LDS");
      static_assert(256 % NCH == 0, "chunks");
      float* const et = (float*)smem;
      const int c8 = tid % NCH, prow = tid / NCH;
      const int p = p0 + c8 * 8;
      const bool pok = p < Pd;
      const bool mbn = bnx && a.mask_scale;  // mask from the BN input (no mask read)
      float bv[8], bmu[8], brs[8], msc[8], msh[8], s1[8], s2[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        bv[k] = (bias && pok) ? bias[p + k] : 0.f;
        bmu[k] = (bnx && pok) ? a.bn_mean[(long long)g * Pd + p + k] : 0.f;
        brs[k] = (bnx && pok) ? a.bn_rstd[(long long)g * Pd + p + k] : 0.f;
        msc[k] = (mbn && pok) ? a.mask_scale[(long long)g * Pd + p + k] : 0.f;
        msh[k] = (mbn && pok) ? a.mask_shift[(long long)g * Pd + p + k] : 0.f;
        s1[k] = s2[k] = 0.f;
      }
      // The strip's global inputs (BN input, residual, mask) are loaded one strip ahead, so their
      // HBM latency overlaps the LDS round trip and the previous strip's arithmetic instead of
      // being paid once per strip.
      constexpr int IT = (NPX + PSTEP - 1) / PSTEP;  // items per thread per strip
      auto item_off = [&](int tj, int it, long long& o) {
        const int px = prow + it * PSTEP;
        const int q = q0 + (px >> 4) * WQ + tj * 16 + (px & 15);
        if (px >= NPX || !pok || q >= Qd) return false;
        o = (long long)q * Pd + p;
        if (phased) {  // phase-local pixel (n, i, j) -> NHWC offset of (n, 2i+a, 2j+b)
          const int n = q / (Hs * Ws), rem = q - n * (Hs * Ws);
          const int hi2 = rem / Ws, wi = rem - hi2 * Ws;
          o = ((long long)(n * H + 2 * hi2 + ph_a) * W + 2 * wi + ph_b) * Pd + p;
        }
        return true;
      };
      // residual element offset of output item (tj, it) at offset o; false: no residual term there
      auto res_off = [&](int tj, int it, long long o, long long& ro) {
        ro = o;
        if (!rsub) return true;
        const int px = prow + it * PSTEP;
        const int q = q0 + (px >> 4) * WQ + tj * 16 + (px & 15);
        if (phased) {  // phase (0, 0)'s local pixel index is the compact index
          ro = (long long)q * Pd + p;
          return (ph_a | ph_b) == 0;
        }
        const int n = q / (H * W), rem = q - n * (H * W);
        const int h = rem / W, w = rem - h * W;
        ro = ((long long)(n * ((H + 1) >> 1) + (h >> 1)) * ((W + 1) >> 1) + (w >> 1)) * Pd + p;
        return ((h | w) & 1) == 0;
      };
      auto load_in = [&](int tj, i4v* X, i4v* R, i4v* M) {
#pragma unroll
        for (int it = 0; it < IT; ++it) {
          long long o = 0, ro = 0;
          const bool ok = item_off(tj, it, o);
          X[it] = (ok && bnx) ? *(const i4v*)(bnx + o) : (i4v){0, 0, 0, 0};
          R[it] = (ok && res && res_off(tj, it, o, ro)) ? *(const i4v*)(res + ro) : (i4v){0, 0, 0, 0};
          M[it] = (ok && msk) ? *(const i4v*)(msk + o) : (i4v){0, 0, 0, 0};
        }
      };
      i4v cX[IT], cR[IT], cM[IT];
      load_in(0, cX, cR, cM);
      __syncthreads();  // every wave is done with the main loop's LDS (ring, halo)
#pragma unroll
      for (int tj = 0; tj < TQ; ++tj) {
#pragma unroll
        for (int ti = 0; ti < TP; ++ti)
          *(f4v*)(et + (wq * 16 + lq) * LROW + wp * WP + ti * 16 + lp) = acc[ti][tj];
        i4v nX[IT], nR[IT], nM[IT];
        if (tj + 1 < TQ) load_in(tj + 1, nX, nR, nM);
        __syncthreads();
#pragma unroll
        for (int it = 0; it < IT; ++it) {
          long long o = 0;
          if (!item_off(tj, it, o)) continue;
          const int px = prow + it * PSTEP;
          const f4v lo = *(const f4v*)(et + px * LROW + c8 * 8);
          const f4v hi = *(const f4v*)(et + px * LROW + c8 * 8 + 4);
          float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] += bv[k];
          float t[8], xb[8];
          if (bnx) unpack8(cX[it], xb);
          if (res) {
            unpack8(cR[it], t);
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] += t[k];
          }
          if (msk) {
            unpack8(cM[it], t);
#pragma unroll
            for (int k = 0; k < 8; ++k) if (!(t[k] > 0.f)) v[k] = 0.f;
          } else if (mbn) {
#pragma unroll
            for (int k = 0; k < 8; ++k) if (!(xb[k] * msc[k] + msh[k] > 0.f)) v[k] = 0.f;
          }
          if (a.relu) {
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = fmaxf(v[k], 0.f);
          }
          *(i4v*)(O + o) = pack8(v);
          if (bnx) {
#pragma unroll
            for (int k = 0; k < 8; ++k) { s1[k] += v[k]; s2[k] += v[k] * ((xb[k] - bmu[k]) * brs[k]); }
          } else {
#pragma unroll
            for (int k = 0; k < 8; ++k) { s1[k] += v[k]; s2[k] += v[k] * v[k]; }
          }
        }
        __syncthreads();
        if (tj + 1 < TQ) {
#pragma unroll
          for (int it = 0; it < IT; ++it) { cX[it] = nX[it]; cR[it] = nR[it]; cM[it] = nM[it]; }
        }
      }
      if (want_stats) {
        // fold the partial sums of the PSTEP threads that share each channel chunk; value-major
        // layout [16][256] so both the stores and the folding reads are lane-consecutive (a
        // [256][16] image made every store 16-way bank-conflicted: 15-20% of the LDS cycles)
#pragma unroll
        for (int k = 0; k < 8; ++k) { et[k * 256 + tid] = s1[k]; et[(8 + k) * 256 + tid] = s2[k]; }
        __syncthreads();
        for (int j = tid; j < 2 * BP; j += 256) {
          const int chunk = j % NCH, kk = j / NCH;  // kk = which * 8 + channel-in-chunk
          const int which = kk >> 3, ch = chunk * 8 + (kk & 7);
          float sum = 0.f;
          for (int r = 0; r < PSTEP; ++r) sum += et[kk * 256 + r * NCH + chunk];
          if (p0 + ch < Pd) atomicAdd(stats + which * Pd + p0 + ch, sum);
        }
      }
    }
  } else {  // WGRAD: dW[p=k][q=rsc] fp32
    float* O = (float*)a.out + (long long)g * a.out_gs;
    const bool atomic = a.accumulate || gy > 1;
    const float gs = a.gscale;
#pragma unroll
    for (int ti = 0; ti < TP; ++ti) {
#pragma unroll
      for (int tj = 0; tj < TQ; ++tj) {
        // halo tiles: column fragment f = (tap, 16-channel half) of the tile's 32 channels
        const int q = HALO_W ? ((wq * TQ + tj) >> 1) * C + q0 / 9 + ((wq * TQ + tj) & 1) * 16 + lq
                             : q0 + wq * WQ + tj * 16 + lq;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int p = p0 + wp * WP + ti * 16 + lp + e;
          if (p < Pd && q < Qd) {
            float* dst = O + (long long)p * Qd + q;
            if (atomic) atomicAdd(dst, gs * acc[ti][tj][e]);
            else *dst = gs * acc[ti][tj][e];
          }
        }
      }
    }
  }
}

template <int MODE, int BP, int BQ, int BK, int NS, int WLP = 2, bool HALO = false>
__global__ __launch_bounds__(256) void conv_igemm_kernel(ConvArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[ConvTile<MODE, BP, BQ, BK, NS, WLP, HALO>::SMEM];
  conv_body<MODE, BP, BQ, BK, NS, WLP, HALO>(
      a, smem, blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z), gridDim.x, gridDim.y,
      gridDim.z);
}

// Split-K epilogue for FWD / DGRAD: out = epi(sum_s partial[s]) with the same fused terms as the
// conv epilogue (bias, residual, mask, relu, BN statistics or the BN backward reduce). Each thread
// owns one 8-channel chunk; per-block sums fold through LDS and go to stripe blockIdx.x % stripes.
#ifndef SPLITK_EPI_RB
#define SPLITK_EPI_RB 2
#endif
__global__ __launch_bounds__(256) void conv_splitk_epilogue_kernel(ConvArgs a, int mode, int Pd,
                                                                   long long rows, int nsplit) {
  __shared__ float red[256 * 16];
  const int g = blockIdx.y;
  const int TPR = Pd >> 3, RPI = 256 / TPR;
  const int cc = threadIdx.x % TPR, row = threadIdx.x / TPR, c0 = cc * 8;
  const long long slice = (long long)a.G * rows * Pd;
  const float* part = a.partial + (long long)g * rows * Pd + c0;
  bf16_t* O = (bf16_t*)a.out + (long long)g * a.out_gs + c0;
  const bool rsub = mode == MODE_DGRAD && a.res_sub == 2;  // compact stride-2 residual (ConvArgs)
  const bf16_t* res = a.residual ? (const bf16_t*)a.residual + (long long)g * (rsub ? a.res_gs : a.out_gs) + c0
                                 : nullptr;
  const bf16_t* msk = a.mask ? (const bf16_t*)a.mask + (long long)g * a.out_gs + c0 : nullptr;
  const bf16_t* bnx = (mode == MODE_DGRAD && a.bn_x) ? (const bf16_t*)a.bn_x + (long long)g * a.out_gs + c0
                                                      : nullptr;
  const bool want_stats = a.stats && (mode == MODE_FWD || bnx);
  const bool mbn = bnx && a.mask_scale;
  float bv[8] = {}, bmu[8] = {}, brs[8] = {}, msc[8] = {}, msh[8] = {}, s1[8] = {}, s2[8] = {};
  if (a.bias) {
#pragma unroll
    for (int k = 0; k < 8; ++k) bv[k] = a.bias[(long long)g * a.bias_gs + c0 + k];
  }
  if (bnx) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      bmu[k] = a.bn_mean[(long long)g * Pd + c0 + k];
      brs[k] = a.bn_rstd[(long long)g * Pd + c0 + k];
    }
  }
  if (mbn) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      msc[k] = a.mask_scale[(long long)g * Pd + c0 + k];
      msh[k] = a.mask_shift[(long long)g * Pd + c0 + k];
    }
  }
  // RB rows per thread per pass; the slices are summed SPB at a time with all RB x SPB loads
  // issued before any use (one memory round trip per SPB slices, not one per slice: the 1-client
  // deep layers run 4-8 slices and this kernel was latency-bound on the serial slice loop).
  constexpr int RB = SPLITK_EPI_RB, SPB = 4;
  const long long stride = (long long)gridDim.x * RPI;
  if (row < RPI) {
    for (long long r0 = (long long)blockIdx.x * RPI + row; r0 < rows; r0 += stride * RB) {
      float v[RB][8];
#pragma unroll
      for (int b = 0; b < RB; ++b)
#pragma unroll
        for (int k = 0; k < 8; ++k) v[b][k] = bv[k];
      long long eb[RB];
#pragma unroll
      for (int b = 0; b < RB; ++b) {
        const long long r = r0 + b * stride;
        eb[b] = (r < rows ? r : r0) * Pd;
      }
      // the bf16 side operands do not depend on the sums: issue them with the first slices
      i4v xres[RB], xmsk[RB], xbnx[RB];
#pragma unroll
      for (int b = 0; b < RB; ++b) {
        xres[b] = (i4v){0, 0, 0, 0};
        if (res) {
          long long ro = eb[b];
          bool ok = true;
          if (rsub) {  // row r = (n*H + h)*W + w of dx; the residual lives on even (h, w) only
            const long long r = eb[b] / Pd;
            const long long n = r / ((long long)a.H * a.W), rem = r - n * a.H * a.W;
            const int h = (int)(rem / a.W), w = (int)(rem - (long long)h * a.W);
            ok = ((h | w) & 1) == 0;
            ro = ((n * ((a.H + 1) >> 1) + (h >> 1)) * ((a.W + 1) >> 1) + (w >> 1)) * Pd;
          }
          if (ok) xres[b] = *(const i4v*)(res + ro);
        }
        if (msk) xmsk[b] = *(const i4v*)(msk + eb[b]);
        if (bnx) xbnx[b] = *(const i4v*)(bnx + eb[b]);
      }
      for (int sp0 = 0; sp0 < nsplit; sp0 += SPB) {
        f4v lo[SPB][RB], hi[SPB][RB];
#pragma unroll
        for (int j = 0; j < SPB; ++j) {
          const long long so = (long long)(sp0 + j < nsplit ? sp0 + j : sp0) * slice;
#pragma unroll
          for (int b = 0; b < RB; ++b) {
            lo[j][b] = *(const f4v*)(part + eb[b] + so);
            hi[j][b] = *(const f4v*)(part + eb[b] + so + 4);
          }
        }
#pragma unroll
        for (int j = 0; j < SPB; ++j) {
          if (sp0 + j >= nsplit) break;
#pragma unroll
          for (int b = 0; b < RB; ++b) {
            v[b][0] += lo[j][b][0]; v[b][1] += lo[j][b][1]; v[b][2] += lo[j][b][2]; v[b][3] += lo[j][b][3];
            v[b][4] += hi[j][b][0]; v[b][5] += hi[j][b][1]; v[b][6] += hi[j][b][2]; v[b][7] += hi[j][b][3];
          }
        }
      }
#pragma unroll
      for (int b = 0; b < RB; ++b) {
        const long long r = r0 + b * stride;
        if (r >= rows) break;
        const long long e = r * Pd;
        float t[8], xb[8];
        if (bnx) unpack8(xbnx[b], xb);
        if (res) {
          unpack8(xres[b], t);
#pragma unroll
          for (int k = 0; k < 8; ++k) v[b][k] += t[k];
        }
        if (msk) {
          unpack8(xmsk[b], t);
#pragma unroll
          for (int k = 0; k < 8; ++k) if (!(t[k] > 0.f)) v[b][k] = 0.f;
        } else if (mbn) {
#pragma unroll
          for (int k = 0; k < 8; ++k) if (!(xb[k] * msc[k] + msh[k] > 0.f)) v[b][k] = 0.f;
        }
        if (a.relu) {
#pragma unroll
          for (int k = 0; k < 8; ++k) v[b][k] = fmaxf(v[b][k], 0.f);
        }
        *(i4v*)(O + e) = pack8(v[b]);
        if (bnx) {
#pragma unroll
          for (int k = 0; k < 8; ++k) { s1[k] += v[b][k]; s2[k] += v[b][k] * ((xb[k] - bmu[k]) * brs[k]); }
        } else {
#pragma unroll
          for (int k = 0; k < 8; ++k) { s1[k] += v[b][k]; s2[k] += v[b][k] * v[b][k]; }
        }
      }
    }
  }
  if (!want_stats) return;
#pragma unroll
  for (int k = 0; k < 8; ++k) { red[k * 256 + threadIdx.x] = s1[k]; red[(8 + k) * 256 + threadIdx.x] = s2[k]; }
  __syncthreads();
  if (row != 0) return;
  for (int r = 1; r < RPI; ++r) {
    const int t = r * TPR + cc;
#pragma unroll
    for (int k = 0; k < 8; ++k) { s1[k] += red[k * 256 + t]; s2[k] += red[(8 + k) * 256 + t]; }
  }
  float* st = a.stats + (long long)g * a.stats_gs +
              (a.stats_stripes > 1 ? (long long)(blockIdx.x % a.stats_stripes) * 2 * Pd : 0) + c0;
#pragma unroll
  for (int k = 0; k < 8; ++k) { atomicAdd(st + k, s1[k]); atomicAdd(st + Pd + k, s2[k]); }
}

static hipError_t splitk_epilogue(const ConvArgs& a, int mode, int Pd, long long rows, int nsplit,
                                  hipStream_t s) {
  const int RPI = 256 / (Pd / 8);
  long long want = (rows + RPI * (long long)SPLITK_EPI_RB - 1) / (RPI * (long long)SPLITK_EPI_RB);
  const long long cap = (2048 + a.G - 1) / a.G;
  if (want > cap) want = cap;
  hipLaunchKernelGGL(conv_splitk_epilogue_kernel, dim3((unsigned)(want < 1 ? 1 : want), a.G), dim3(256), 0, s,
                     a, mode, Pd, rows, nsplit);
  return hipGetLastError();
}

template <int MODE, int BP, int BQ, int BK, int NS, int WLP = 2, bool HALO = false>
static hipError_t launch_cfg(const ConvArgs& a, int Pd, int Qd, int gy, hipStream_t stream) {
  const int ntp = (Pd + BP - 1) / BP, ntq = (Qd + BQ - 1) / BQ;
  dim3 grid(ntp * ntq, gy, a.G);
  hipLaunchKernelGGL((conv_igemm_kernel<MODE, BP, BQ, BK, NS, WLP, HALO>), grid, dim3(256), 0, stream, a);
  return hipGetLastError();
}

// Instantiated (tile, K-step, LDS stages). LDS = NS*(BP+BQ)*BK*2 bytes: the 4-stage BK=32 tiles
// (<= 64 KB) keep 2 workgroups per CU, which the per-layer sweep (scripts/conv_bench.py --sweep,
// profiles/conv_sweep_*.log) found fastest for every ResNet-18 shape.
template <int MODE>
static hipError_t dispatch(const ConvArgs& a, int Pd, int Qd, int bp, int bq, int bk, int ns, int gy,
                           hipStream_t s) {
#define DDL_CFG(BP_, BQ_, BK_, NS_) \
  if (bp == BP_ && bq == BQ_ && bk == BK_ && ns == NS_) \
    return launch_cfg<MODE, BP_, BQ_, BK_, NS_>(a, Pd, Qd, gy, s);
  DDL_CFG(64, 64, 32, 4) DDL_CFG(64, 128, 32, 4) DDL_CFG(128, 64, 32, 4) DDL_CFG(128, 128, 32, 4)
  DDL_CFG(128, 128, 32, 3) DDL_CFG(64, 128, 64, 3) DDL_CFG(128, 128, 64, 3) DDL_CFG(128, 128, 64, 2)
  DDL_CFG(64, 64, 64, 3) DDL_CFG(128, 64, 64, 3)
  // 256-wide tiles: 128x64 per wave (1.5x the MFMA work per LDS byte of a 64x64 wave tile)
  DDL_CFG(256, 128, 32, 3) DDL_CFG(128, 256, 32, 3) DDL_CFG(256, 128, 32, 2) DDL_CFG(128, 256, 32, 2)
  // deep rings for few-workgroup grids (one client): a 64-wide wave tile issues 4-8 MFMAs per
  // K-step, far less than one L2 round trip, so more K-steps must be in flight per workgroup
  DDL_CFG(64, 64, 32, 6) DDL_CFG(64, 64, 32, 8) DDL_CFG(64, 128, 32, 6) DDL_CFG(64, 128, 32, 8)
  DDL_CFG(128, 64, 32, 6) DDL_CFG(128, 128, 32, 6)
#undef DDL_CFG
  // 64-wide P tiles with the 4 waves side by side along Q (64x64 per wave); encoded as bp = 48
#define DDL_CFG1(BQ_, BK_, NS_) \
  if (bp == 48 && bq == BQ_ && bk == BK_ && ns == NS_) \
    return launch_cfg<MODE, 64, BQ_, BK_, NS_, 1>(a, Pd, Qd, gy, s);
  DDL_CFG1(256, 32, 4) DDL_CFG1(256, 64, 3) DDL_CFG1(256, 64, 2) DDL_CFG1(256, 32, 3)
#undef DDL_CFG1
  return hipErrorInvalidValue;
}

// Halo-staged 3x3 stride-1 FWD / DGRAD (BK = 32); bp = 48 again selects 64 with 1x4 waves.
template <int MODE>
static hipError_t dispatch_halo(const ConvArgs& a, int Pd, int Qd, int bp, int bq, int ns, hipStream_t s) {
#define DDL_HCFG(BP_, BQ_, NS_, BPE_, WLP_) \
  if (bp == BP_ && bq == BQ_ && ns == NS_) \
    return launch_cfg<MODE, BPE_, BQ_, 32, NS_, WLP_, true>(a, Pd, Qd, 1, s);
  DDL_HCFG(48, 256, 4, 64, 1) DDL_HCFG(48, 128, 4, 64, 1) DDL_HCFG(64, 128, 4, 64, 2)
  DDL_HCFG(128, 128, 4, 128, 2) DDL_HCFG(128, 256, 4, 128, 2) DDL_HCFG(48, 256, 5, 64, 1)
  DDL_HCFG(48, 128, 6, 64, 1) DDL_HCFG(128, 128, 6, 128, 2)
#undef DDL_HCFG
  return hipErrorInvalidValue;
}

// Halo eligibility (the kernel's HALO contract): 3x3 / stride 1 / pad 1 with same-size output,
// tiles of whole rows inside one image or of whole images, and a halo image that fits the pieces the taps of one
// channel block can issue (NS-1 .. 8) and the LDS buffer (4 pieces per wave at BQ 128).
static bool halo_ok(const ConvArgs& a, int bq, int ns) {
  if (a.stride != 1 || a.R != 3 || a.S != 3 || a.pad != 1 || a.P != a.H || a.Q != a.W) return false;
  const int hw = a.H * a.W;
  if (hw >= bq ? (bq % a.W || hw % bq) : bq % hw) return false;  // whole rows / whole images
  const int trh = bq / a.W < a.H ? bq / a.W : a.H;
  const int hpx = bq / (trh * a.W) * (trh + 2) * (a.W + 2);
  const int hpw = ((hpx + 15) / 16 + 3) / 4;
  const int cap = bq >= 256 ? 10 - ns : (10 - ns < 4 ? 10 - ns : 4);
  return hpw <= cap;
}

// DDL_CONV_HALO=0 disables the halo kernels' automatic use (explicit cfgs still run them)
static bool halo_auto() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("DDL_CONV_HALO");
    v = (e && e[0] == '0') ? 0 : 1;
  }
  return v == 1;
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
  if (a.stride <= 0 || a.pad < 0 || !a.zero) return false;
  if (a.P != (a.H + 2 * a.pad - a.R) / a.stride + 1) return false;
  if (a.Q != (a.W + 2 * a.pad - a.S) / a.stride + 1) return false;
  // 32-bit element offsets and buffer byte ranges (< the out-of-range sentinel 0xFFFFFFF0)
  if ((long long)a.N * a.H * a.W * (a.C > a.K ? a.C : a.K) >= (1LL << 31) - 64) return false;
  if ((long long)a.N * a.P * a.Q * (a.C > a.K ? a.C : a.K) >= (1LL << 31) - 64) return false;
  if ((long long)a.K * a.R * a.S * a.C >= (1LL << 31) - 64) return false;
  return a.P > 0 && a.Q > 0;
}

// cfg = bp/16 | (bq/16)<<8 | bk<<16 | ns<<24 (0 = heuristic); WGRAD split-K count in a.split_k
// (0 = auto). Python: ops.functional.conv_cfg(bp, bq, bk, ns).
static void decode_cfg(int cfg, int& bp, int& bq, int& bk, int& ns) {
  if (!cfg) return;
  bp = (cfg & 0xff) * 16;
  bq = ((cfg >> 8) & 0xff) * 16;
  bk = (cfg >> 16) & 0xff;
  ns = (cfg >> 24) & 0xff;  // bit 0x40: halo-staged kernel
  if (!(ns & 0x3f)) ns |= bk == 32 ? 4 : 3;
}

// Grid-size-aware fallback (G=1 sweep, profiles/conv_sweep_g1.log): when the tuned tile leaves
// CUs without a workgroup, a 64-wide tile (BK=64 when the reduction run allows) gets more CUs
// working: 64x128 while that gives >= 1 workgroup per CU, else 64x64. (At 1-2 workgroups per CU
// the big tile still wins: profiles/conv_sweep_r1d.log, layer 4 at G=8.)
static void small_grid_tiles(int Pd, long long Qd, int G, bool bk64_ok, int& bp, int& bq, int& bk,
                             int& ns) {
  auto tiles = [&](int p, int q) { return (long long)((Pd + p - 1) / p) * ((Qd + q - 1) / q) * G; };
  if (tiles(bp, bq) >= num_cus()) return;
  bk = bk64_ok ? 64 : 32;
  ns = bk64_ok ? 3 : 4;
  bp = 64;
  bq = tiles(64, 128) >= num_cus() ? 128 : 64;
}

// FWD / DGRAD split-K count: automatic only for unphased DGRAD (deep_only) with grids under one
// workgroup per CU — ~3 per CU from K-splits of >= 8 steps — bounded by the caller's partial
// workspace; split_k = 1 disables, > 1 forces (any mode).
static int fd_splits(const ConvArgs& a, int Pd, long long tiles, long long nk, long long out_elems,
                     bool deep_only) {
  if (!a.partial || a.split_k == 1 || Pd % 8 || Pd / 8 > 256) return 1;
  long long sp;
  if (a.split_k > 1) {
    sp = a.split_k;
  } else {
    // the extra pass moves (splits + 0.5) x 4 B per output and the split kernels are bandwidth-
    // bound like the unsplit ones, so it only pays for deep reductions on small outputs
    // (profiles/conv_split_g1.log: 1-client layer-4 DGRAD 48 -> 29-34 us; everything else loses)
    if (!deep_only || tiles >= num_cus() || out_elems * a.G > (1LL << 20) || nk < 48) return 1;
    sp = (3LL * num_cus() + tiles / 2) / tiles;
    if (sp > nk / 8) sp = nk / 8;
  }
  const long long fit = a.partial_cap / (out_elems * a.G);
  if (sp > fit) sp = fit;
  if (sp > 64) sp = 64;
  return sp > 1 ? (int)sp : 1;
}

// A resolved launch: which instantiation (tile code bp — 48 = 64 channels with the 4 waves
// along Q — bq, bk, ns, halo), its virtual grid (ntp * ntq, gy, G) and the FWD / DGRAD split-K
// epilogue (sp > 1). Every entry point plans first, so a single launch and a paired launch
// (ddl_conv_pair) of the same op run the same tile on the same grid.
struct ConvPlan {
  int mode, bp, bq, bk, ns, halo;
  int Pd, Qd, gy, sp;
  long long rows;
};

static int plan_bpe(const ConvPlan& p) { return p.bp == 48 ? 64 : p.bp; }
static int plan_blocks(const ConvPlan& p, int G) {
  const int bpe = plan_bpe(p);
  return ((p.Pd + bpe - 1) / bpe) * ((p.Qd + p.bq - 1) / p.bq) * p.gy * G;
}

static int plan_fwd(const ConvArgs& a, int cfg, ConvPlan& pl) {
  if (!conv_shapes_ok(a)) return (int)hipErrorInvalidValue;
  const int Pd = a.K, Qd = a.N * a.P * a.Q;
  // sweep-tuned (profiles/conv_sweep_r1.log): 128x128x64 / 2 stages for >=128 output channels
  int bp = 64, bq = 128, bk = 32, ns = 4;
  if (a.K >= 128 && a.C % 64 == 0) { bp = 128; bk = 64; ns = 2; }
  small_grid_tiles(Pd, Qd, a.G, a.C % 64 == 0, bp, bq, bk, ns);
  bool halo = false;
  if (cfg) {
    decode_cfg(cfg, bp, bq, bk, ns);
    halo = ns & 0x40;
    ns &= 0x3f;
  } else if (halo_auto()) {
    // sweep (profiles/conv_halo_sweep_r1_g8.log): 64 x 256 tiles, 4 waves along Q
    const long long ht = (long long)((Pd + 63) / 64) * (Qd / 256) * a.G;
    if (halo_ok(a, 256, 4) && ht >= num_cus()) { halo = true; bp = 48; bq = 256; bk = 32; ns = 4; }
  }
  pl = ConvPlan{MODE_FWD, bp, bq, bk, ns, halo, Pd, Qd, 1, 1, Qd};
  if (halo) return (!halo_ok(a, bq, ns) || bk != 32) ? (int)hipErrorInvalidValue : 0;
  if (a.C % bk) return (int)hipErrorInvalidValue;
  const int bpe = bp == 48 ? 64 : bp;
  const long long tiles = (long long)((Pd + bpe - 1) / bpe) * ((Qd + bq - 1) / bq) * a.G;
  pl.sp = fd_splits(a, Pd, tiles, ((long long)a.R * a.S * a.C + bk - 1) / bk, (long long)Qd * Pd, false);
  pl.gy = pl.sp;
  return 0;
}

static int plan_dgrad(const ConvArgs& a, int cfg, ConvPlan& pl) {
  if (!conv_shapes_ok(a)) return (int)hipErrorInvalidValue;
  // stride 2 runs as 4 sub-pixel phases (blockIdx.y); grid sized for the largest (phase 0,0)
  const bool phased = a.stride == 2;
  const int Pd = a.C;
  const int Qd = phased ? a.N * ((a.H + 1) / 2) * ((a.W + 1) / 2) : a.N * a.H * a.W;
  int bp = 64, bq = 128, bk = 32, ns = 4;
  if (a.C >= 128 && a.K % 64 == 0) { bp = 128; bk = 64; ns = 2; }
  small_grid_tiles(Pd, Qd * (phased ? 4 : 1), a.G, a.K % 64 == 0, bp, bq, bk, ns);
  bool halo = false;
  if (cfg) {
    decode_cfg(cfg, bp, bq, bk, ns);
    halo = ns & 0x40;
    ns &= 0x3f;
  } else if (halo_auto() && !phased) {
    // sweep (profiles/conv_halo_sweep_r1_g8.log): 64 x 128 tiles, 4 waves along Q
    const long long ht = (long long)((Pd + 63) / 64) * (Qd / 128) * a.G;
    if (halo_ok(a, 128, 4) && ht >= num_cus()) { halo = true; bp = 48; bq = 128; bk = 32; ns = 4; }
  }
  const long long rows = (long long)a.N * a.H * a.W;
  pl = ConvPlan{MODE_DGRAD, bp, bq, bk, ns, halo, Pd, Qd, 1, 1, rows};
  if (halo) return (phased || !halo_ok(a, bq, ns) || bk != 32) ? (int)hipErrorInvalidValue : 0;
  if (a.K % bk) return (int)hipErrorInvalidValue;
  const int nph = phased ? 4 : 1;
  const int bpe = bp == 48 ? 64 : bp;
  const long long tiles = (long long)((Pd + bpe - 1) / bpe) * ((Qd + bq - 1) / bq) * a.G * nph;
  // the (0, 0) phase has the most taps: ceil(R/2) x ceil(S/2) for pad-parity 0
  const int rn = phased ? (a.R - (a.pad & 1) + 1) / 2 : a.R, sn = phased ? (a.S - (a.pad & 1) + 1) / 2 : a.S;
  pl.sp = fd_splits(a, Pd, tiles, ((long long)rn * sn * a.K + bk - 1) / bk, rows * Pd, !phased);
  pl.gy = nph * pl.sp;
  return 0;
}

// Halo WGRAD contract: 3x3 / stride 1 / pad 1, same-size output, 32-pixel K-steps of whole rows.
static bool wgrad_halo_ok(const ConvArgs& a) {
  if (a.stride != 1 || a.R != 3 || a.S != 3 || a.pad != 1 || a.P != a.H || a.Q != a.W) return false;
  if (!(a.W == 8 || a.W == 16 || a.W == 32) || a.H % (32 / a.W)) return false;
  return a.K % 64 == 0 && a.C % 32 == 0;
}

static int plan_wgrad(const ConvArgs& a, int cfg, ConvPlan& pl) {
  if (!conv_shapes_ok(a)) return (int)hipErrorInvalidValue;
  const bool halo_cfg = cfg && (((cfg >> 24) & 0xff) & 0x40);
  bool halo_pick = false;
  if (!cfg && halo_auto() && a.accumulate && wgrad_halo_ok(a) && a.W >= 16) {
    // ~2 workgroups per CU, and only with >= 64 K-steps per split: the halo tile covers all 9
    // taps of 32 channels, so grids of few clients would need splits too short to pay for the
    // per-step row window (sweep: profiles/conv_wgrad_halo_r1.log; 8 clients: layer 1 155 ->
    // 102 us, layer 2 107 -> 100 us; 1 client and 8x8 layers stay streamed)
    const long long tiles = (long long)(a.K / 64) * (a.C / 32) * a.G;
    const long long nk = (long long)a.N * a.H * a.W / 32;
    const long long sp = (2LL * num_cus() + tiles - 1) / tiles;
    halo_pick = nk / sp >= 64;
  }
  if (halo_cfg || halo_pick) {  // halo tile: 64 x (9 taps x 32 channels)
    if (!wgrad_halo_ok(a) || (halo_cfg && ((cfg & 0xff) != 4 || ((cfg >> 8) & 0xff) != 18)))
      return (int)hipErrorInvalidValue;
    const long long tiles = (long long)(a.K / 64) * (a.C / 32) * a.G;
    const long long nk = (long long)a.N * a.H * a.W / 32;
    long long sp = a.split_k ? a.split_k : (2LL * num_cus() + tiles - 1) / tiles;
    if (sp > nk / 8) sp = nk / 8 > 0 ? nk / 8 : 1;
    if (sp > 1024) sp = 1024;
    if (sp > 1 && !a.accumulate) return (int)hipErrorInvalidValue;
    const int hns = halo_cfg ? ((cfg >> 24) & 0x3f) : 4;  // LDS stages (12 KiB each)
    if (hns < 4 || hns > 6) return (int)hipErrorInvalidValue;
    pl = ConvPlan{MODE_WGRAD, 64, 288, 32, hns, 1, a.K, a.R * a.S * a.C, (int)sp, 1, 0};
    return 0;
  }
  const int Pd = a.K, Qd = a.R * a.S * a.C;
  const long long Kr = (long long)a.N * a.P * a.Q;
  int bp = a.K >= 128 ? 128 : 64, bq = Qd >= 128 ? 128 : 64, bk = 32, ns = 4;
  if (a.K >= 128 && Qd >= 128) ns = 3;
  if (Qd < 128) { bp = 64; bq = 64; bk = 64; ns = 3; }
  // aim for ~2 waves of workgroups over the CUs, keep >= 16 K-steps per split
  auto auto_splits = [&](int p, int q, int k) {
    const long long tiles = (long long)((Pd + p - 1) / p) * ((Qd + q - 1) / q) * a.G;
    const long long nk = (Kr + k - 1) / k;
    long long want = (2LL * num_cus() + tiles - 1) / tiles;
    long long maxs = nk / 16 > 0 ? nk / 16 : 1;
    long long sp = want < maxs ? want : maxs;
    return (int)(sp < 1 ? 1 : (sp > 1024 ? 1024 : sp));
  };
  // few tiles and a shallow reduction (one client, deep layers: profiles/conv_sweep_g1.log): the
  // splits would be too short to fill the LDS pipeline, so trade split depth for 4x the tiles
  if (!cfg && ((Kr + bk - 1) / bk) / auto_splits(bp, bq, bk) < 32) { bp = 64; bq = 64; bk = 64; ns = 3; }
  decode_cfg(cfg, bp, bq, bk, ns);
  const int splits = a.split_k ? a.split_k : auto_splits(bp, bq, bk);
  if (splits > 1 && !a.accumulate) return (int)hipErrorInvalidValue;  // needs zeroed fp32 output
  pl = ConvPlan{MODE_WGRAD, bp, bq, bk, ns, 0, Pd, Qd, splits, 1, 0};
  return 0;
}

static int plan_mode(int mode, const ConvArgs& a, int cfg, ConvPlan& pl) {
  if (a.res_sub == 2 && (mode != MODE_DGRAD || !a.residual)) return (int)hipErrorInvalidValue;
  if (mode == MODE_FWD) return plan_fwd(a, cfg, pl);
  if (mode == MODE_DGRAD) return plan_dgrad(a, cfg, pl);
  if (mode == MODE_WGRAD) return plan_wgrad(a, cfg, pl);
  return (int)hipErrorInvalidValue;
}

template <int MODE>
static hipError_t launch_single(const ConvArgs& a, const ConvPlan& p, hipStream_t s) {
  if (p.halo) {
    if constexpr (MODE == MODE_WGRAD) {
      if (p.ns == 4) return launch_cfg<MODE_WGRAD, 64, 288, 32, 4, 2, true>(a, p.Pd, p.Qd, p.gy, s);
      if (p.ns == 5) return launch_cfg<MODE_WGRAD, 64, 288, 32, 5, 2, true>(a, p.Pd, p.Qd, p.gy, s);
      if (p.ns == 6) return launch_cfg<MODE_WGRAD, 64, 288, 32, 6, 2, true>(a, p.Pd, p.Qd, p.gy, s);
      return hipErrorInvalidValue;
    } else {
      return dispatch_halo<MODE>(a, p.Pd, p.Qd, p.bp, p.bq, p.ns, s);
    }
  }
  return dispatch<MODE>(a, p.Pd, p.Qd, p.bp, p.bq, p.bk, p.ns, p.gy, s);
}

static int launch_plan(const ConvArgs& a, const ConvPlan& p, hipStream_t s) {
  hipError_t e;
  if (p.mode == MODE_FWD) e = launch_single<MODE_FWD>(a, p, s);
  else if (p.mode == MODE_DGRAD) e = launch_single<MODE_DGRAD>(a, p, s);
  else e = launch_single<MODE_WGRAD>(a, p, s);
  return (int)e;
}

// FWD / DGRAD with fd split-K: the epilogue pass after the partial-sum kernel
static int finish_plan(const ConvArgs& a, const ConvPlan& p, hipStream_t s) {
  if (p.mode == MODE_WGRAD || p.sp <= 1) return 0;
  return (int)splitk_epilogue(a, p.mode, p.Pd, p.rows, p.sp, s);
}

static int run_mode(int mode, const ConvArgs* ap, int cfg, hipStream_t stream) {
  ConvPlan pl;
  int e = plan_mode(mode, *ap, cfg, pl);
  if (e) return e;
  e = launch_plan(*ap, pl, stream);
  if (e) return e;
  return finish_plan(*ap, pl, stream);
}

DDL_API int ddl_conv_fwd(const ConvArgs* ap, int cfg, hipStream_t stream) {
  return run_mode(MODE_FWD, ap, cfg, stream);
}
DDL_API int ddl_conv_dgrad(const ConvArgs* ap, int cfg, hipStream_t stream) {
  return run_mode(MODE_DGRAD, ap, cfg, stream);
}
DDL_API int ddl_conv_wgrad(const ConvArgs* ap, int cfg, hipStream_t stream) {
  return run_mode(MODE_WGRAD, ap, cfg, stream);
}

// ---------------------------------------------------------------------------------------------
// Paired launch: two independent convolutions of one layer in ONE grid — the DGRAD and WGRAD of
// a backward conv (both read dY), or the two FWD convs of a downsample block that are independent
// (its last 3x3 conv and the 1x1 projection shortcut on the block input). Few-client grids fill a fraction of the 256 CUs per op (1 client, 8x8
// layer: 200 DGRAD workgroups); pairing lets the second op's workgroups run in the first op's
// tail and idle CU slots instead of after it, without the cross-queue synchronisation a second
// stream costs inside a HIP graph (docs/KERNELS.md, dead ends). Blocks [0, nA8) run op A (nA
// rounded up to 8 so op B's virtual block ids keep their XCD residue), the rest op B; the LDS
// image is the larger of the two.
template <class TA, class TB>
__global__ __launch_bounds__(256) void conv_pair_kernel(ConvArgs a, ConvArgs b, int4 ga, int3 gb) {
  __shared__ __attribute__((aligned(16))) char smem[TA::SMEM > TB::SMEM ? TA::SMEM : TB::SMEM];
  const int bid = blockIdx.x;
  if (bid < ga.w) {
    if (bid < ga.x * ga.y * ga.z) TA::run(a, smem, bid, ga.x, ga.y, ga.z);
  } else {
    TB::run(b, smem, bid - ga.w, gb.x, gb.y, gb.z);
  }
}

template <int MODE, int BP, int BQ, int BK, int NS, int WLP, bool HALO>
struct TileOp : ConvTile<MODE, BP, BQ, BK, NS, WLP, HALO> {
  static constexpr int M = MODE, BPC = (WLP == 1 && BP == 64) ? 48 : BP, BQC = BQ, BKC = BK, NSC = NS;
  static constexpr bool H = HALO;
  __device__ __forceinline__ static void run(const ConvArgs& a, char* smem, int lin, int gx, int gy,
                                             int gz) {
    conv_body<MODE, BP, BQ, BK, NS, WLP, HALO>(a, smem, lin, gx, gy, gz);
  }
  static bool match(const ConvPlan& p) {
    return p.mode == MODE && p.bp == BPC && p.bq == BQ && p.bk == BK && p.ns == NS && (bool)p.halo == HALO;
  }
};

template <class TA, class TB>
static bool try_pair(const ConvArgs& a, const ConvPlan& pa, const ConvArgs& b, const ConvPlan& pb,
                     hipStream_t s, int& err) {
  if (!TA::match(pa) || !TB::match(pb)) return false;
  const int bpa = plan_bpe(pa), bpb = plan_bpe(pb);
  const int gxa = ((pa.Pd + bpa - 1) / bpa) * ((pa.Qd + pa.bq - 1) / pa.bq);
  const int gxb = ((pb.Pd + bpb - 1) / bpb) * ((pb.Qd + pb.bq - 1) / pb.bq);
  const int na = gxa * pa.gy * a.G, na8 = (na + 7) & ~7, nb = gxb * pb.gy * b.G;
  hipLaunchKernelGGL((conv_pair_kernel<TA, TB>), dim3(na8 + nb), dim3(256), 0, s, a, b,
                     make_int4(gxa, pa.gy, a.G, na8), make_int3(gxb, pb.gy, b.G));
  err = (int)hipGetLastError();
  return true;
}

// Tile menu of the paired kernels (instantiated combinations; ops/autotune.py mirrors it in
// PAIR_DGRAD / PAIR_WGRAD / PAIR_FWD). bp 48 = 64 channels, 4 waves along Q.
using DgH256 = TileOp<MODE_DGRAD, 64, 256, 32, 4, 1, true>;
using DgH128 = TileOp<MODE_DGRAD, 64, 128, 32, 4, 1, true>;
using Dg128x128k64 = TileOp<MODE_DGRAD, 128, 128, 64, 2, 2, false>;
using Dg64x128k64 = TileOp<MODE_DGRAD, 64, 128, 64, 3, 2, false>;
using Dg128x64k64 = TileOp<MODE_DGRAD, 128, 64, 64, 3, 2, false>;
using Dg48x256k64 = TileOp<MODE_DGRAD, 64, 256, 64, 2, 1, false>;
using Wg64x64k64 = TileOp<MODE_WGRAD, 64, 64, 64, 3, 2, false>;
using Wg128x64k64 = TileOp<MODE_WGRAD, 128, 64, 64, 3, 2, false>;
using Wg128x128k32 = TileOp<MODE_WGRAD, 128, 128, 32, 3, 2, false>;
using Wg128x128k64 = TileOp<MODE_WGRAD, 128, 128, 64, 2, 2, false>;
using Wg64x128k32 = TileOp<MODE_WGRAD, 64, 128, 32, 4, 2, false>;
// FWD + FWD: a block's last 3x3 conv (A) and its 1x1 projection shortcut (B)
using Fw64x64k64 = TileOp<MODE_FWD, 64, 64, 64, 3, 2, false>;
using Fw64x128k64 = TileOp<MODE_FWD, 64, 128, 64, 3, 2, false>;
using Fw128x128k32 = TileOp<MODE_FWD, 128, 128, 32, 3, 2, false>;
using Fw128x64k64 = TileOp<MODE_FWD, 128, 64, 64, 3, 2, false>;
using Fw64x128k32 = TileOp<MODE_FWD, 64, 128, 32, 4, 2, false>;

// The instantiated (A, B) combinations, applied to a macro P(TA, TB).
#define DDL_PAIR_LIST(P)                                                                          \
  P(DgH256, Wg64x64k64) P(DgH256, Wg128x64k64) P(DgH256, Wg128x128k32) P(DgH256, Wg128x128k64)   \
  P(DgH256, Wg64x128k32) P(DgH128, Wg64x64k64) P(DgH128, Wg128x64k64) P(DgH128, Wg128x128k32)    \
  P(DgH128, Wg128x128k64) P(DgH128, Wg64x128k32) P(Dg128x128k64, Wg64x64k64)                     \
  P(Dg128x128k64, Wg128x64k64) P(Dg128x128k64, Wg128x128k32) P(Dg128x128k64, Wg128x128k64)       \
  P(Dg128x128k64, Wg64x128k32) P(Dg64x128k64, Wg64x64k64) P(Dg64x128k64, Wg128x64k64)            \
  P(Dg64x128k64, Wg128x128k32) P(Dg64x128k64, Wg128x128k64) P(Dg64x128k64, Wg64x128k32)          \
  P(Dg128x64k64, Wg64x64k64) P(Dg128x64k64, Wg128x64k64) P(Dg128x64k64, Wg128x128k32)            \
  P(Dg128x64k64, Wg128x128k64) P(Dg128x64k64, Wg64x128k32) P(Dg48x256k64, Wg64x64k64)            \
  P(Dg48x256k64, Wg128x64k64) P(Dg48x256k64, Wg128x128k32) P(Dg48x256k64, Wg128x128k64)          \
  P(Dg48x256k64, Wg64x128k32)                                                                    \
  P(Fw64x64k64, Fw64x128k32) P(Fw64x64k64, Fw64x64k64) P(Fw64x64k64, Fw64x128k64)                \
  P(Fw64x128k64, Fw64x128k32) P(Fw64x128k64, Fw64x64k64) P(Fw64x128k64, Fw64x128k64)             \
  P(Fw128x128k32, Fw64x128k32) P(Fw128x128k32, Fw64x64k64) P(Fw128x128k32, Fw64x128k64)          \
  P(Fw128x64k64, Fw64x128k32) P(Fw128x64k64, Fw64x64k64) P(Fw128x64k64, Fw64x128k64)

static int pair_dispatch(const ConvArgs& a, const ConvPlan& pa, const ConvArgs& b, const ConvPlan& pb,
                         hipStream_t s) {
  int err = 0;
#define DDL_PAIR_TRY(TA, TB) \
  if (try_pair<TA, TB>(a, pa, b, pb, s, err)) return err;
  DDL_PAIR_LIST(DDL_PAIR_TRY)
#undef DDL_PAIR_TRY
  return -1;  // no paired instantiation for these tiles
}

// mode_a / mode_b: 0 FWD, 1 DGRAD, 2 WGRAD; cfg_* as the single-op entry points (0 = heuristic).
// Returns -1 (nothing launched) when the two plans have no paired kernel: the caller launches
// them one after the other instead.
DDL_API int ddl_conv_pair(const ConvArgs* ap, int mode_a, int cfg_a, const ConvArgs* bp, int mode_b,
                          int cfg_b, hipStream_t stream) {
  ConvPlan pa, pb;
  int e = plan_mode(mode_a, *ap, cfg_a, pa);
  if (e) return e;
  e = plan_mode(mode_b, *bp, cfg_b, pb);
  if (e) return e;
  e = pair_dispatch(*ap, pa, *bp, pb, stream);
  if (e) return e;
  e = finish_plan(*ap, pa, stream);
  if (e) return e;
  return finish_plan(*bp, pb, stream);
}

// Whether (mode_a, cfg_a) + (mode_b, cfg_b) on these shapes has a paired kernel (no launch).
DDL_API int ddl_conv_pair_supported(const ConvArgs* ap, int mode_a, int cfg_a, const ConvArgs* bp,
                                    int mode_b, int cfg_b) {
  ConvPlan pa, pb;
  if (plan_mode(mode_a, *ap, cfg_a, pa) || plan_mode(mode_b, *bp, cfg_b, pb)) return 0;
  bool ok = false;
#define DDL_PAIR_OK(TA, TB) ok = ok || (TA::match(pa) && TB::match(pb));
  DDL_PAIR_LIST(DDL_PAIR_OK)
#undef DDL_PAIR_OK
  return ok ? 1 : 0;
}

DDL_API int ddl_conv_args_size() { return (int)sizeof(ConvArgs); }
