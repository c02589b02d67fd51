// Reference-precision (fp32) GEMM on the bf16 MFMA: D[p][q] = sum_k A(p, k) * B(q, k), fp32 in, fp32
// out, every product exact to one fp32 rounding (X6, see conv_f32_core.h split3). The plain-GEMM
// products of the fp32 LLaMA (the tutorial_1b model: qkv / out-proj / SwiGLU FFN / LM head linears,
// FWD, DGRAD and WGRAD; reference lab/tutorial_1b/PP/1F1B/intro_PP_1F1B_MB.py:16-46,
// lab/tutorial_1b/DP/gradient_aggr/intro_DP_GA.py:27-28,47-51) run here instead of a vendor GEMM.
//
// Operands are PRE-SPLIT "planes": an fp32 matrix X[R][C] becomes three bf16 matrices h, m, l of the
// same shape (x = h + m + l exactly; x6_planes_kernel below), stored plane after plane, each
// zero-padded to whole 32-row / 32-column multiples (a partial last reduction stage reads zeros). A GEMM
// operand reads them in whichever orientation the product needs, without a transpose pass:
//   * K-major (the reduction index is the contiguous one: X[p][k]) -> LDS image [plane][rows][16 k],
//     fragments by ds_read_b64;
//   * MN-major (the output index is contiguous: X[k][p]) -> LDS image [plane][16 k][cols], fragments
//     by the gfx950 transpose read ds_read_b64_tr_b16.
// So each tensor of a linear layer is split ONCE and serves all three products (x: FWD K-major,
// WGRAD MN-major; W: FWD K-major, DGRAD MN-major; dY: DGRAD K-major, WGRAD MN-major).
//
// Per 16-deep reduction step and 16x16 tile, three v_mfma_f32_16x16x32_bf16 (lane group g = the
// four k values 4g..4g+3, fragment halves assembled in registers from the plane reads):
//   A (l | h) . B (h | m) = lh + hm      A (h | m) . B (l | h) = hl + mh      A (h | m) . B (h | m) = hh + mm
// chained from zero (smallest products first) over four steps (64 reduction values), then ONE IEEE
// add into the fp32 accumulator (the rounding discipline of conv_f32.hip / conv_x6h.hip: the
// MFMA's internal sum is not an RNE fp32 chain, so chains stay short).
//
// Staging: LDS-DMA (buffer_load_dwordx4 ... lds, 1 KiB per wave-instruction, lane-linear destination,
// 16-B chunk XOR swizzles applied by permuting each lane's SOURCE chunk) into an NS-deep ring, one
// raw s_barrier per step and counted `s_waitcnt vmcnt` so NS-2 stages stay in flight across it;
// fragments of step i+1 are read while step i's MFMAs run. Out-of-range rows / chunks read through
// the buffer descriptor as zeros (no branches). 4 waves, 2 x 2 over a (32 TP) x (32 TQ) tile.
// Output: out[q * ldo + p] (p contiguous: a lane's 4 accumulator rows are one float4), with
// out = alpha * acc + (residual ? residual : accumulate ? out : 0) (+ bias[p]). Split-K slices store
// raw partials [split][N][M] and gemm_x6_reduce folds them in slice order: DETERMINISTIC (no atomics).
#include <cstdlib>

#include "ddl_common.h"

struct GemmX6Args {
  const bf16_t* a;      // A planes (h | m | l), plane stride a_ps elements, row pitch lda
  const bf16_t* b;      // B planes
  float* out;           // out[q * ldo + p]
  const float* res;     // optional: added instead of the old out (layout of out)
  const float* bias;    // optional: [M] along p
  float* partial;       // split-K slabs [split][N][M]
  long long a_ps, b_ps, partial_cap;
  int lda, ldb, ldo;
  int M, N, K;          // p extent (A rows), q extent (B rows), reduction
  int split_k, accumulate;
  float alpha;
  int probe;            // timing probes (wrong results): 1 skip MFMAs, 2 skip DMA, 4 skip fragment reads,
                        // 8 skip the epilogue, 16 return at entry
};

namespace {

constexpr int XBK = 32;  // fp32 reduction values per stage (two 16-deep MFMA steps)

typedef __attribute__((address_space(3))) s4v lds_s4v;
typedef __attribute__((address_space(3))) void lds_void;

// K-major image: per plane [rows][32 bf16] = 64-B rows of four 16-B chunks; chunk c of row r sits
// at c ^ ((r >> 2) & 3): the ds_read_b64 fragment reads (32-lane halves = 16 rows x 2 k-groups of
// one step) are conflict-free.
__device__ __forceinline__ int km_sw(int row) { return (row >> 2) & 3; }
// MN-major image: per plane [32 k][CW bf16]; chunk c of k-row k at c ^ mn_sw(k): the 8 k-rows of a
// transpose read's 32-lane half land on distinct 32-B bank segments.
template <int CW>
__device__ __forceinline__ int mn_sw(int k) {
  if constexpr (CW >= 128) return 2 * (k & 7);
  else return 2 * ((k >> 1) & 3);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// One LDS-DMA piece (16 B per lane to lds + 16 * lane; byte offset off + soff). Kept out of the
// kernel body: inline in a __global__ template (address-space cast, runtime scalar offset) the host
// pass silently drops the kernel's launch stub (conv_x6h.hip dma16).
__device__ __forceinline__ void dma16(const __amdgpu_buffer_rsrc_t& rs, char* lds, unsigned off, unsigned soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)lds, 16, off, soff, 0, 0);
}

// LDS byte address of a __shared__ object (kept out of the kernel templates: with the address-space
// cast inline in a __global__ template the host pass can drop the launch stub, conv_x6h.hip dma16)
__device__ __forceinline__ unsigned lds_base(const char* p) {
  return (unsigned)(size_t)(const __attribute__((address_space(3))) char*)p;
}
template <int OFF>
__device__ __forceinline__ i2v lds_rd64(unsigned addr) {
  i2v r;
  asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
  return r;
}
template <int OFF>
__device__ __forceinline__ i2v lds_rdtr(unsigned addr) {
  i2v r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
  return r;
}
// the asm reads' registers are valid only after this; the sched_barrier keeps the compiler from
// hoisting register-only MFMAs above the wait (cdna_hip_programming.md §5.4 rule 18)
__device__ __forceinline__ void lgkm_wait() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}



// Operand geometry (per stage): T 16-row tiles per wave, 2 waves along the operand's output index.
template <int T, bool MN>
struct Opnd {
  static constexpr int ROWS = 32 * T;                          // output rows of the block tile
  static constexpr int CW = MN ? (ROWS <= 64 ? 64 : 128) : 0;  // MN image row length (bf16, pow2)
  static constexpr int BYTES_RAW = MN ? 3 * XBK * CW * 2 : 3 * ROWS * XBK * 2;
  static constexpr int NI = (BYTES_RAW / 1024 + 3) / 4 * 4;   // DMA wave-instructions (multiple of 4)
  static constexpr int BYTES = NI * 1024;
  static constexpr int PW = NI / 4;                           // per wave
  static constexpr bool MN_ = MN;
  static constexpr int ROWS_ = ROWS, CW_ = CW;
};

template <int TP, int TQ, bool AMN, bool BMN, int NS>
struct X6Smem {
  using OA = Opnd<TP, AMN>;
  using OB = Opnd<TQ, BMN>;
  static constexpr int STAGE = OA::BYTES + OB::BYTES;
  static constexpr int OPITCH = 32 * TP + 4;  // epilogue staging row (floats): 16-B shifted per row
  static constexpr int EPI = 32 * TQ * OPITCH * 4;
  static constexpr int BYTES = NS * STAGE > EPI ? NS * STAGE : EPI;
};

template <int TP, int TQ, bool AMN, bool BMN, int NS>
__global__ __launch_bounds__(256, 1) void gemm_x6_kernel(GemmX6Args a) {
  using OA = Opnd<TP, AMN>;
  using OB = Opnd<TQ, BMN>;
  using SM = X6Smem<TP, TQ, AMN, BMN, NS>;
  constexpr int STAGE = SM::STAGE;
  constexpr int OPS = OA::PW + OB::PW;  // DMA instructions per wave per stage
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wp = wid >> 1, wq = wid & 1;
  const int wsc = __builtin_amdgcn_readfirstlane(wid);
  const int ntp = (a.M + OA::ROWS - 1) / OA::ROWS, ntq = (a.N + OB::ROWS - 1) / OB::ROWS;
  const int ntiles = ntp * ntq;
  const int nwg = gridDim.x;
  const int u = xcd_remap(blockIdx.x, nwg);
  const int tile = u % ntiles, split = u / ntiles, nsplit = a.split_k;
  const int p0 = (tile % ntp) * OA::ROWS, q0 = (tile / ntp) * OB::ROWS;
  if (a.probe & 16) return;  // launch / dispatch cost only

  const int nk_all = (a.K + XBK - 1) / XBK;
  const int per = (nk_all + nsplit - 1) / nsplit;
  const int kt0 = split * per, kt1 = min(nk_all, kt0 + per);
  const int nk = max(0, kt1 - kt0);

  constexpr unsigned OOB = 0xFFFFFFF0u;
  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)a.a, 0, (int)(a.a_ps * 3 * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)a.b, 0, (int)(a.b_ps * 3 * 2), 0x00020000);

  // Per-lane source element offset of each of this wave's DMA instructions at stage k0 = 0 (-1:
  // always out of range) and the lane's reduction coordinate (K-major: chunk column; MN: k-row).
  auto src_base = [&](auto op, int j, int r0, int rdim, int ld, long long ps, int& kcoord) -> long long {
    using O = decltype(op);
    kcoord = 0;
    if constexpr (!O::MN_) {
      const int gr = 16 * j + (lane >> 2);  // row over [plane][ROWS]
      const int plane = gr / O::ROWS_, row = gr - plane * O::ROWS_;
      const int lc = (lane & 3) ^ km_sw(row);
      kcoord = 8 * lc;
      if (plane >= 3 || r0 + row >= rdim) return -1;
      return plane * ps + (long long)(r0 + row) * ld + 8 * lc;
    } else {
      constexpr int CPR = O::CW_ / 8, RPI = 64 / CPR;
      const int gr = RPI * j + lane / CPR;  // k-row over [plane][32]
      const int plane = gr / XBK, k = gr - plane * XBK;
      const int lc = (lane % CPR) ^ mn_sw<O::CW_>(k);
      kcoord = k;
      const int col = r0 + 8 * lc;
      if (plane >= 3 || 8 * lc >= O::ROWS_ || col >= rdim) return -1;
      return plane * ps + (long long)k * ld + col;
    }
  };
  long long sa[OA::PW], sb[OB::PW];
  int ka[OA::PW], kb[OB::PW];
#pragma unroll
  for (int i = 0; i < OA::PW; ++i) sa[i] = src_base(OA{}, wsc + 4 * i, p0, a.M, a.lda, a.a_ps, ka[i]);
#pragma unroll
  for (int i = 0; i < OB::PW; ++i) sb[i] = src_base(OB{}, wsc + 4 * i, q0, a.N, a.ldb, a.b_ps, kb[i]);
  // 32-bit per-lane byte offsets at stage 0 (invalid rows / columns: OOBV) and the stage advance in
  // the SCALAR offset: a piece costs no VALU. The planes are zero-padded to whole 32-deep stages
  // along the reduction (ops/gemm_x6.py split), so a partial last stage needs no per-lane k test.
  // Stages past the slice take the scalar offset OOBS: every wave issues the same, constant number
  // of pieces per stage (constant vmcnt waits, no branch). Images are < 2^30 B (host-checked), so
  // OOBV + any advance and any valid offset + OOBS both stay in [2^30, 2^31): past the range.
  constexpr unsigned OOBV = 0x40000000u, OOBS = 0x40000000u;
  unsigned va[OA::PW], vb[OB::PW];
#pragma unroll
  for (int i = 0; i < OA::PW; ++i) va[i] = sa[i] >= 0 ? (unsigned)(sa[i] * 2) : OOBV;
#pragma unroll
  for (int i = 0; i < OB::PW; ++i) vb[i] = sb[i] >= 0 ? (unsigned)(sb[i] * 2) : OOBV;
  const unsigned a_adv = AMN ? (unsigned)(XBK * a.lda * 2) : (unsigned)(XBK * 2);  // bytes per stage
  const unsigned b_adv = BMN ? (unsigned)(XBK * a.ldb * 2) : (unsigned)(XBK * 2);

  // DMA piece d (0 .. OPS-1: this wave's A pieces, then its B pieces) of stage kt into `slot`
  auto dma_piece = [&](int d, int kt, int slot) {
    char* base = smem + slot * STAGE;
    const bool kin = kt < kt1;
    if (d < OA::PW) {
      dma16(rA, base + (wsc + 4 * d) * 1024, va[d], kin ? (unsigned)kt * a_adv : OOBS);
    } else {
      const int i = d - OA::PW;
      dma16(rB, base + OA::BYTES + (wsc + 4 * i) * 1024, vb[i], kin ? (unsigned)kt * b_adv : OOBS);
    }
  };

  // Fragment reads are inline-asm ds_reads: the compiler cannot see them as LDS reads, so it does
  // not drain every in-flight LDS-DMA (vmcnt(0)) before each one — it cannot tell the ring slots
  // apart. Ordering is explicit: the counted vmcnt + barrier before a stage's first read, and
  // lgkm_wait() before the MFMAs consume a read's registers.
  // Per-lane byte offsets (within a stage slot) of this lane's fragment of tile t, step s.
  constexpr int APL = AMN ? XBK * OA::CW * 2 : OA::ROWS * 64;  // plane stride in the image (bytes)
  constexpr int BPL = BMN ? XBK * OB::CW * 2 : OB::ROWS * 64;
  auto frag_off = [&](auto op, int rb, int s) -> unsigned {
    using O = decltype(op);
    if constexpr (!O::MN_) {
      const int row = rb + (lane & 15), g = lane >> 4;
      const int ch = 2 * s + (g >> 1);
      return (unsigned)(row * 64 + ((ch ^ km_sw(row)) << 4) + 8 * (g & 1));
    } else {
      const int g = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
      const int k = 16 * s + 4 * g + q4, col = rb + 4 * p4;
      return (unsigned)(k * O::CW_ * 2 + ((((col >> 3) ^ mn_sw<O::CW_>(k))) << 4) + 8 * ((col >> 2) & 1));
    }
  };
  const unsigned lds0 = lds_base(smem);
  unsigned fofA[2][TP], fofB[2][TQ];
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
    for (int t = 0; t < TP; ++t) fofA[s2][t] = lds0 + frag_off(OA{}, wp * 16 * TP + 16 * t, s2);
#pragma unroll
    for (int t = 0; t < TQ; ++t) fofB[s2][t] = lds0 + OA::BYTES + frag_off(OB{}, wq * 16 * TQ + 16 * t, s2);
  }
  // a fragment is the two MFMA operands (l | h) and (h | m), each read straight into its own 4-VGPR
  // tuple (h is read twice: the register coalescer then needs no copies; with three piece vectors
  // the compiler assembled the operands by v_perm / v_mov / v_bfi, ~500 VALU per 96 MFMAs)
  struct Frag { i4v lh, hm; };
  Frag fa0[TP], fb0[TQ], fa1[TP], fb1[TQ];
  auto pack = [](i2v l, i2v h1, i2v h2, i2v m) {
    Frag f;
    f.lh = (i4v){l.x, l.y, h1.x, h1.y};
    f.hm = (i4v){h2.x, h2.y, m.x, m.y};
    return f;
  };
  // fragment c (0 .. TP-1: A tiles, then B tiles) of step s2 of the stage in `slot`
  auto read_frag = [&](int c, int slot, int s2, Frag (&fa)[TP], Frag (&fb)[TQ]) {
    const unsigned sb = (unsigned)(slot * STAGE);
    if (c < TP) {
      const unsigned ad = fofA[s2][c] + sb;
      if constexpr (AMN) fa[c] = pack(lds_rdtr<2 * APL>(ad), lds_rdtr<0>(ad), lds_rdtr<0>(ad), lds_rdtr<APL>(ad));
      else fa[c] = pack(lds_rd64<2 * APL>(ad), lds_rd64<0>(ad), lds_rd64<0>(ad), lds_rd64<APL>(ad));
    } else {
      const int t = c - TP;
      const unsigned ad = fofB[s2][t] + sb;
      if constexpr (BMN) fb[t] = pack(lds_rdtr<2 * BPL>(ad), lds_rdtr<0>(ad), lds_rdtr<0>(ad), lds_rdtr<BPL>(ad));
      else fb[t] = pack(lds_rd64<2 * BPL>(ad), lds_rd64<0>(ad), lds_rd64<0>(ad), lds_rd64<BPL>(ad));
    }
  };

  f4v acc[TP][TQ], cc[TP][TQ];
#pragma unroll
  for (int i = 0; i < TP; ++i)
#pragma unroll
    for (int j = 0; j < TQ; ++j) acc[i][j] = (f4v){0.f, 0.f, 0.f, 0.f};

  // One 16-deep step: three piece-pair MFMAs per tile, smallest products first (`first`: the
  // chain starts from zero; `last`: ONE IEEE add of the chain into the running fp32 sum), with the
  // NEXT step's fragment reads and (dma) the ring's next DMA pieces interleaved into the MFMA
  // stream at even spacing, each group pinned by a sched_barrier: issued in a burst ahead of the
  // MFMAs, the DMA pieces stalled the wave's MFMA issue and load and compute serialised.
  constexpr int NM = 3 * TP * TQ, NC = TP + TQ;
  auto step = [&](const Frag (&fa)[TP], const Frag (&fb)[TQ], bool first, bool last, int rslot, int rs2,
                  Frag (&na)[TP], Frag (&nb)[TQ], bool dma, int dkt, int dslot) {
#pragma unroll
    for (int e = 0; e < NM; ++e) {
#pragma unroll
      for (int c = 0; c < NC; ++c)
        if (e == (c * NM) / NC) read_frag(c, rslot, rs2, na, nb);
      if (dma) {
#pragma unroll
        for (int d = 0; d < OPS; ++d)
          if (e == (d * NM) / OPS) dma_piece(d, dkt, dslot);
      }
      const int pass = e / (TP * TQ), i = (e % (TP * TQ)) / TQ, j = e % TQ;
      const s8v alh = __builtin_bit_cast(s8v, fa[i].lh), ahm = __builtin_bit_cast(s8v, fa[i].hm);
      const s8v blh = __builtin_bit_cast(s8v, fb[j].lh), bhm = __builtin_bit_cast(s8v, fb[j].hm);
      if (pass == 0)
        cc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(alh, bhm, first ? (f4v){0.f, 0.f, 0.f, 0.f} : cc[i][j],
                                                           0, 0, 0);
      else if (pass == 1)
        cc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahm, blh, cc[i][j], 0, 0, 0);
      else
        cc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahm, bhm, cc[i][j], 0, 0, 0);
      if ((e + 1) % (NM / NC) == 0) __builtin_amdgcn_sched_barrier(0);
    }
    if (last) {
#pragma unroll
      for (int i = 0; i < TP; ++i)
#pragma unroll
        for (int j = 0; j < TQ; ++j) {
#pragma unroll
          for (int v = 0; v < 4; ++v) acc[i][j][v] = acc[i][j][v] + cc[i][j][v];
          asm volatile("" : "+v"(acc[i][j]));  // the add belongs to this stage
        }
    }
    __builtin_amdgcn_sched_barrier(0);
  };

  if (nk > 0 && !(a.probe & 2)) {
    // Ring: stage j lives in slot j % NS. Prologue: stages 0 .. NS-1 issued, stage 0 landed, its
    // step-0 fragments requested. Iteration j: step 0 of stage j (reading step 1's fragments);
    // then stage j+1 must have landed (own DMA: NS-2 later stages may still fly) and be visible
    // (barrier), which also retires every wave's reads of stage j's slot; step 1 of stage j reads
    // stage j+1's step-0 fragments and DMAs stage j+NS into slot j % NS.
#pragma unroll
    for (int s2 = 0; s2 < NS; ++s2)
#pragma unroll
      for (int d = 0; d < OPS; ++d) dma_piece(d, kt0 + s2, s2);
    wait_vm<(NS - 1) * OPS>();
    raw_barrier();
#pragma unroll
    for (int c = 0; c < NC; ++c) read_frag(c, 0, 0, fa0, fb0);
    // one stage: its two 16-deep steps; the MFMA chain runs over TWO stages (four steps, 12 piece
    // products per tile) before its IEEE add
    auto iter = [&](int i, bool first, bool last) {
      const int slot = i % NS, nslot = (i + 1) % NS;
      lgkm_wait();  // step 0's fragments
      step(fa0, fb0, first, false, slot, 1, fa1, fb1, false, 0, 0);
      wait_vm<(NS - 2) * OPS>();
      lgkm_wait();  // step 1's fragments (before the barrier: the slot's last reads)
      raw_barrier();
      step(fa1, fb1, false, last, nslot, 0, fa0, fb0, true, kt0 + i + NS, slot);
    };
    int i = 0;
    for (; i + 1 < nk; i += 2) {
      iter(i, true, false);
      iter(i + 1, false, true);
    }
    if (i < nk) iter(i, true, true);
    wait_vm<0>();  // the ring's trailing (zero-fill) pieces land before the LDS is reused
  }

  // ---- epilogue: acc[i][j][v] = D[p = pb + 4 (lane >> 4) + v][q = qb + (lane & 15)], staged through
  // LDS as [q][p] rows so every global store is a whole-row 16-B-per-lane write
  const bool split_store = nsplit > 1;
  if (a.probe & 8) {
    float sink = 0.f;
#pragma unroll
    for (int i = 0; i < TP; ++i)
#pragma unroll
      for (int j = 0; j < TQ; ++j) sink += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    if (sink == 1.2345f) a.out[0] = sink;
    return;
  }
  __syncthreads();  // every wave is past its last fragment read: the ring is free
  float* stg = (float*)smem;
  constexpr int OP = SM::OPITCH;
#pragma unroll
  for (int i = 0; i < TP; ++i)
#pragma unroll
    for (int j = 0; j < TQ; ++j) {
      const int pl = wp * 16 * TP + 16 * i + 4 * (lane >> 4);
      const int ql = wq * 16 * TQ + 16 * j + (lane & 15);
      *(float4*)(stg + ql * OP + pl) = make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
    }
  __syncthreads();
  constexpr int RF4 = 8 * TP;  // float4 per staged row
  constexpr int NF4 = RF4 * 32 * TQ;
  const int pmax = a.M - p0, qmax = a.N - q0;
#pragma unroll 4
  for (int e = tid; e < NF4; e += 256) {
    const int ql = e / RF4, pl = 4 * (e - ql * RF4);
    if (ql >= qmax || pl >= pmax) continue;
    const float4 v = *(const float4*)(stg + ql * OP + pl);
    const int p = p0 + pl, q = q0 + ql;
    if (split_store) {
      *(float4*)(a.partial + ((long long)split * a.N + q) * a.M + p) = v;
      continue;
    }
    float* d = a.out + (long long)q * a.ldo + p;
    const float4 b = a.res ? *(const float4*)(a.res + (long long)q * a.ldo + p)
                           : (a.accumulate ? *(const float4*)d : make_float4(0.f, 0.f, 0.f, 0.f));
    const float4 bi = a.bias ? *(const float4*)(a.bias + p) : make_float4(0.f, 0.f, 0.f, 0.f);
    *(float4*)d = make_float4(a.alpha * v.x + b.x + bi.x, a.alpha * v.y + b.y + bi.y, a.alpha * v.z + b.z + bi.z,
                              a.alpha * v.w + b.w + bi.w);
  }
}

// split-K fold, slice order (bitwise the sequential sum), then the direct epilogue
__global__ __launch_bounds__(256) void gemm_x6_reduce(GemmX6Args a) {
  const long long nv = (long long)a.N * (a.M / 4);
  GSTRIDE_LOOP(t, nv) {
    const int q = (int)(t / (a.M / 4)), p = (int)(t - (long long)q * (a.M / 4)) * 4;
    const float* src = a.partial + (long long)q * a.M + p;
    const long long ss = (long long)a.N * a.M;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    int k = 0;
    for (; k + 4 <= a.split_k; k += 4) {
      float4 v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = *(const float4*)(src + (k + j) * ss);
#pragma unroll
      for (int j = 0; j < 4; ++j) { s.x += v[j].x; s.y += v[j].y; s.z += v[j].z; s.w += v[j].w; }
    }
    for (; k < a.split_k; ++k) {
      const float4 v = *(const float4*)(src + k * ss);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    float* d = a.out + (long long)q * a.ldo + p;
    const float4 b = a.res ? *(const float4*)(a.res + (long long)q * a.ldo + p)
                           : (a.accumulate ? *(const float4*)d : make_float4(0.f, 0.f, 0.f, 0.f));
    const float4 bi = a.bias ? *(const float4*)(a.bias + p) : make_float4(0.f, 0.f, 0.f, 0.f);
    *(float4*)d = make_float4(a.alpha * s.x + b.x + bi.x, a.alpha * s.y + b.y + bi.y, a.alpha * s.z + b.z + bi.z,
                              a.alpha * s.w + b.w + bi.w);
  }
}

// fp32 X[R][C] (row pitch ld) -> planes h | m | l [R][C] bf16 (row pitch ldp, plane stride ps):
// x = h + m + l exactly (truncation split: h the top 8 significand bits, m the next 8, l the rest).
// 8 consecutive columns per thread: two 16-B loads, one 16-B store per plane.
__device__ __forceinline__ void split1(float x, uint16_t& h, uint16_t& m, uint16_t& l) {
  const uint32_t u = __float_as_uint(x);
  const float r1 = x - __uint_as_float(u & 0xFFFF0000u);
  const uint32_t um = __float_as_uint(r1);
  const float r2 = r1 - __uint_as_float(um & 0xFFFF0000u);
  h = (uint16_t)(u >> 16);
  m = (uint16_t)(um >> 16);
  l = (uint16_t)(__float_as_uint(r2) >> 16);
}

__global__ __launch_bounds__(256) void x6_planes_kernel(const float* __restrict__ x, long long ld, bf16_t* out,
                                                        long long ldp, long long ps, int R, int C, int Rp, int Cp) {
  const int c8 = Cp / 8;
  GSTRIDE_LOOP(t, (long long)Rp * c8) {
    const long long r = t / c8;
    const int c = (int)(t - r * c8) * 8;
    const bool in = r < R && c < C;  // the zero padding (to whole 32-deep GEMM stages) is written too
    const float4 v0 = in ? *(const float4*)(x + r * ld + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 v1 = in ? *(const float4*)(x + r * ld + c + 4) : make_float4(0.f, 0.f, 0.f, 0.f);
    const float e[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
    uint16_t h[8], m[8], l[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) split1(e[i], h[i], m[i], l[i]);
    i4v vh, vm, vl;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      vh[i] = (int)((uint32_t)h[2 * i] | ((uint32_t)h[2 * i + 1] << 16));
      vm[i] = (int)((uint32_t)m[2 * i] | ((uint32_t)m[2 * i + 1] << 16));
      vl[i] = (int)((uint32_t)l[2 * i] | ((uint32_t)l[2 * i + 1] << 16));
    }
    bf16_t* d = out + r * ldp + c;
    *(i4v*)d = vh;
    *(i4v*)(d + ps) = vm;
    *(i4v*)(d + 2 * ps) = vl;
  }
}

template <int TP, int TQ, bool AMN, bool BMN, int NS>
int launch(const GemmX6Args& a, hipStream_t s) {
  using OA = Opnd<TP, AMN>;
  using OB = Opnd<TQ, BMN>;
  const size_t lds = (size_t)X6Smem<TP, TQ, AMN, BMN, NS>::BYTES;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_x6_kernel<TP, TQ, AMN, BMN, NS>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  const long long ntiles = (long long)((a.M + OA::ROWS - 1) / OA::ROWS) * ((a.N + OB::ROWS - 1) / OB::ROWS);
  hipLaunchKernelGGL((gemm_x6_kernel<TP, TQ, AMN, BMN, NS>), dim3((unsigned)(ntiles * a.split_k)), dim3(256), lds,
                     s, a);
  return (int)hipGetLastError();
}

template <int TP, int TQ, int NS>
int launch_orient(const GemmX6Args& a, int amn, int bmn, hipStream_t s) {
  if (!amn && !bmn) return launch<TP, TQ, false, false, NS>(a, s);
  if (amn && !bmn) return launch<TP, TQ, true, false, NS>(a, s);
  if (!amn && bmn) return launch<TP, TQ, false, true, NS>(a, s);
  return launch<TP, TQ, true, true, NS>(a, s);
}

}  // namespace

// cfg: TP | TQ << 4 | a_mn << 8 | b_mn << 9 | NS << 12   (TP, TQ in {2, 3, 4}; NS 3 for TQ 4, else 4)
DDL_API int ddl_gemm_x6(const GemmX6Args* ap, int cfg, hipStream_t s) {
  GemmX6Args a = *ap;
  const int TP = cfg & 15, TQ = (cfg >> 4) & 15, amn = (cfg >> 8) & 1, bmn = (cfg >> 9) & 1, NS = (cfg >> 12) & 15;
  if (a.M < 1 || a.N < 1 || a.K < 1) return (int)hipErrorInvalidValue;
  // chunk granularity: K-major operands need K % 8, MN-major ones their output extent % 8; float4 epilogue
  if (a.M % 8 || a.N % 8 || a.K % 8 || a.ldo % 4 || a.lda % 8 || a.ldb % 8 || a.a_ps % 8 || a.b_ps % 8)
    return (int)hipErrorInvalidValue;
  if (a.a_ps * 6 >= (1LL << 30) || a.b_ps * 6 >= (1LL << 30)) return (int)hipErrorInvalidValue;
  if (a.split_k < 1) a.split_k = 1;
  if (a.split_k > 1) {
    if (!a.partial || (long long)a.split_k * a.M * a.N > a.partial_cap) return (int)hipErrorInvalidValue;
  }
  int e;
#define X6_CASE(tp, tq, ns) \
  if (TP == tp && TQ == tq && NS == ns) e = launch_orient<tp, tq, ns>(a, amn, bmn, s); else
  X6_CASE(4, 4, 3) X6_CASE(3, 4, 3) X6_CASE(4, 2, 4) X6_CASE(3, 2, 4) X6_CASE(2, 4, 4) X6_CASE(2, 2, 4)
  return (int)hipErrorInvalidValue;
#undef X6_CASE
  if (e != (int)hipSuccess || a.split_k == 1) return e;
  hipLaunchKernelGGL(gemm_x6_reduce, dim3(grid_for((long long)a.N * (a.M / 4), 256)), dim3(256), 0, s, a);
  return (int)hipGetLastError();
}

// planes of x [R][C] (pitch ld) as [3][Rp][Cp] (pitch ldp >= Cp, plane stride ps), zero-padded
DDL_API int ddl_x6_planes(const float* x, long long ld, void* out, long long ldp, long long ps, int R, int C,
                          int Rp, int Cp, hipStream_t s) {
  if (R < 1 || C < 1 || C % 8 || Cp % 8 || Cp < C || Rp < R || ld % 4 || ldp % 8 || ldp < Cp || ps % 8)
    return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(x6_planes_kernel, dim3(grid_for((long long)Rp * (Cp / 8), 256)), dim3(256), 0, s, x, ld,
                     (bf16_t*)out, ldp, ps, R, C, Rp, Cp);
  return (int)hipGetLastError();
}

DDL_API int ddl_gemm_x6_args_size() { return (int)sizeof(GemmX6Args); }
