// One whole training EPOCH of a small fp32 MLP graph in ONE persistent workgroup: the split-NN of
// the vertical-FL lab (reference lab/tutorial_2b/vfl.py:11-102 — per-party bottom MLPs, concat,
// top MLP, soft-target CE, AdamW, one optimizer step per mini-batch, vfl.py:58-82) and any other
// Linear+act(+dropout) DAG of the same kind (ops/mlp_epoch.py builds the tables).
//
// Why one workgroup: the nets are ~44 K parameters on 64-row mini-batches. Unfused, a mini-batch
// is ~40 launches of 1-6 us kernels that each fill a few CUs, i.e. launch / tail bound. Here one
// workgroup of 16 waves walks every mini-batch of the epoch: forward levels, the CE, backward
// levels, the AdamW update, with a workgroup barrier between phases. Activations / gradients live
// in a few hundred KB of scratch that stays in the CU's L1 / the XCD's L2; nothing returns to the
// host until the epoch ends (loss / accuracy accumulate on the device).
//
// Math: every product is an exact-fp32 v_mfma_f32_16x16x4_f32 (the reference trains in fp32). A
// wave owns a 32x32 output tile (2x2 MFMA tiles sharing their A / B loads):
//   FWD   z[m][n]  = drop(act(sum_k in[m][k] W[n][k] + b[n]))      (A, B K-major)
//   DGRAD d[m][k]  = sum_n dp[m][n] W[n][k], times the INPUT buffer's act'(z) * mask * scale, so
//                    every gradient buffer holds the pre-activation gradient ("dp") directly
//   WGRAD g[n][k]  = sum_m dp[m][n] in[m][k]                        (A, B MN-major)
//   BIAS  g[b + n] = sum_m dp[m][n]                                  (row order: deterministic)
// Dropout masks are Philox(seed; element, step, buffer) (the step = the optimizer's device step
// counter), recomputed in backward, never stored. act' is read from the stored post-dropout
// value z: a kept element has sign(z) == sign(y), a dropped one has gradient 0 anyway.
// AdamW is the FlatAdam kernel's arithmetic (optim.hip adam_kernel, decoupled weight decay).
#include "ddl_common.h"

namespace {

#ifndef MLP_NT
#define MLP_NT 1024  // 16 waves, 4 per SIMD: more latency hiding than 8 despite ~40 VGPR spills outside the
                     // MFMA loops (120.7 vs 125 us per mini-batch; 512 threads need no spills)
#endif
#ifndef MLP_RING
#define MLP_RING 1  // chunks of a global operand in flight (scripts/mlp_epoch_variants.sh A/B)
#endif
#ifndef MLP_ADAM_OVERLAP
#define MLP_ADAM_OVERLAP 0  // 1: AdamW of level l + 1 inside level l's WGRAD phase; 0: one phase at the end
#endif
constexpr int NT = MLP_NT, NWAVE = NT / 64;
constexpr int MAXL = 12, MAXB = 12, MAXP = 4, MAXLEV = 8;
// profile slots: forward level l -> l, CE -> MAXLEV, backward level l -> MAXLEV + 1 + l, AdamW -> last
constexpr int NPROF = 2 * MAXLEV + 2;

struct MlpBuf {       // an activation buffer [round32(B)][ld] at float offset `off` of the LDS arena
  int off, ld, width, act;  // act: 0 none, 1 relu, 2 leaky relu
  float slope, drop;        // dropout probability applied after the activation (0: none)
};
struct MlpLayer {     // out[:, out_col : out_col + N] = drop(act(in[:, in_col : in_col + K] W^T + b))
  int in_buf;         // >= 0 buffer, < 0: party input -(p + 1) (rows of x[p], global memory)
  int in_col, out_buf, out_col, K, N, level, need_dx;
  long long w, b;     // offsets of W [N][K] (row-major) and b [N] in the flat parameter buffer
};
struct MlpEpochArgs {
  const float* x[MAXP]; int x_ld[MAXP];
  const float* y;                      // soft targets [n][ncls] (probabilities / float one-hot)
  float *p, *g, *m, *v;                // flat parameters / gradients / Adam moments
  unsigned long long* step_dev;        // optimizer step counter (FlatAdam.t_dev), advanced per step
  float* stats;                        // += {sum of mini-batch mean losses, correct predictions}
  unsigned long long* prof;            // optional [NPROF]: += wall-clock ticks (100 MHz) per phase
  long long nparam, lds_floats;        // flat length, LDS arena size (floats; host-checked)
  unsigned long long seed;
  float lr, beta1, beta2, eps, wd;
  int n, B, ncls, nlayers, nbufs, nlev, logits_buf, probe;  // timing bits: 1 no GEMM loads, 2 no MFMA, 4 no epilogue, 8 no tiles, 16 no AdamW, 32 no DGRAD, 64 no WGRAD, 128 DGRAD reads W as if transposed
  MlpBuf bufs[MAXB];
  MlpLayer layers[MAXL];
};

// Activations are branch-free with one per-buffer factor: relu 0, leaky relu `slope`, none 1.
__device__ __forceinline__ float act_neg(int act, float slope) {
  return act == 1 ? 0.f : (act == 2 ? slope : 1.f);
}
__device__ __forceinline__ float act_fwd(float v, float neg) {
  return v > 0.f ? v : neg * v + 0.f;  // + 0: relu of a negative is +0, as fmaxf(v, 0) gives
}
__device__ __forceinline__ float act_grad(float z, float neg) { return z > 0.f ? 1.f : neg; }
// Dropout: one Philox call yields the keep draws of 4 consecutive rows of a column: element
// (row p, column c) of buffer `buf` uses word p & 3 of Philox(key; (p >> 2) * ld + c, step,
// 0x7f4a7c15, buf) -- the 4 rows an MFMA lane holds share one call.
__device__ __forceinline__ uint4 drop4(uint2 key, uint32_t step, int buf, int p4, int ld, int col) {
  return philox4x32(make_uint4((uint32_t)(p4 * ld + col), step, 0x7f4a7c15u, (uint32_t)buf), key);
}
__device__ __forceinline__ uint32_t word(const uint4& r, int w) {
  return w == 0 ? r.x : (w == 1 ? r.y : (w == 2 ? r.z : r.w));
}

// Data pointers read from the tables are generic; global accesses go through these global-address-
// space views so the loads are global_load (vmcnt only), not flat_load (vmcnt + lgkmcnt).
typedef __attribute__((address_space(1))) float gfloat;
typedef __attribute__((address_space(1))) f4v gfloat4;  // native vector (HIP's float4 class has no addrspace copy)
__device__ __forceinline__ gfloat* gp(float* p) { return (gfloat*)p; }
__device__ __forceinline__ const gfloat* gp(const float* p) { return (const gfloat*)p; }

// Every activation buffer of the mini-batch lives in this LDS arena (host-sized, <= 159 KB): the
// phases hand activations / gradients to each other through LDS, so a phase boundary is an LDS
// barrier, not a global store-acknowledge round trip. Backward is in place: at each level the
// WGRAD (+ bias) phase consumes the layer input, then the DGRAD phase overwrites that input with
// its gradient (same element, same thread: act' / mask read, gradient written).
extern __shared__ float arena[];

// GEMM operands. Four kinds: in the LDS arena or in global memory, K-major (element (row, k) at
// row * ld + k) or MN-major (at row + k * ld).
//  * LDS operands are read WITHOUT bounds checks: the arena is zeroed at launch, rows are padded
//    to a multiple of 32 (rows >= M of every buffer are written as zeros), and whatever lies
//    past an operand's reduction extent meets a zero in the other operand (a global operand,
//    zeroed there) -- so the loads are bare ds_reads with 32-bit offsets.
//  * Global operands (weights, party inputs) clamp their row (a clamped row only feeds output
//    rows / columns the epilogue drops) and zero the reduction tail, the tail chunk only.
enum { O_LK = 0, O_LMN = 1, O_GK = 2, O_GMN = 3 };
struct Opnd {
  const gfloat* g;  // global base (O_G*)
  int l;            // arena offset (O_L*)
  int ld, R, vec;   // leading dimension, rows (global), 16-byte vector loads possible (K-major)
};
__device__ __forceinline__ Opnd gop(const float* base, int ld, int R) {
  Opnd o{gp(base), 0, ld, R, 0};
  o.vec = (ld & 3) == 0 && (((uintptr_t)base) & 15) == 0;
  return o;
}
__device__ __forceinline__ Opnd lop(int off, int ld) {
  Opnd o{nullptr, off, ld, 0, 0};
  o.vec = (ld & 3) == 0 && (off & 3) == 0;
  return o;
}
// v[j] = operand(row, k + j), j < 4 (global operands: clamped, see tail_zero)
template <int KIND>
__device__ __forceinline__ void load4(const Opnd& o, int row, int k, int Kr, float (&v)[4]) {
  if (KIND == O_LK) {
    const int e = o.l + row * o.ld + k;
    if (o.vec) {
      const f4v t = *reinterpret_cast<const f4v*>(arena + e);
      v[0] = t[0]; v[1] = t[1]; v[2] = t[2]; v[3] = t[3];
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = arena[e + j];
    }
  } else if (KIND == O_LMN) {
    const int e = o.l + row + k * o.ld;
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = arena[e + j * o.ld];
  } else {
    // clamped (always in bounds) and raw: the reduction tail is zeroed where the chunk is
    // consumed (tail_zero), so no select waits on the load here and the loads stay in flight
    const unsigned rr = (unsigned)min(row, o.R - 1);
    if (KIND == O_GK && o.vec && k + 3 < Kr) {
      const f4v t = *reinterpret_cast<const gfloat4*>(o.g + (rr * (unsigned)o.ld + (unsigned)k));
      v[0] = t[0]; v[1] = t[1]; v[2] = t[2]; v[3] = t[3];
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const unsigned kk = (unsigned)min(k + j, Kr - 1);
        v[j] = KIND == O_GK ? o.g[rr * (unsigned)o.ld + kk] : o.g[rr + kk * (unsigned)o.ld];
      }
    }
  }
}
// zero the elements of a global operand's chunk past the reduction extent (the tail chunk only)
__device__ __forceinline__ void tail_zero(float (&v)[2][4], int k, int Kr) {
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) v[i][j] = k + j < Kr ? v[i][j] : 0.f;
}

// acc[i][jj] (16x16 tile at rows p0 + 16 i, cols q0 + 16 jj) += sum_k A(p, k) B(q, k), for the
// ni x nj sub-tiles that hold any output (a 2-wide logits layer issues a quarter of the MFMAs).
// Lane group g = lane >> 4 feeds k = k0 + 4 g + j to MFMA j: the four MFMAs of a 16-deep chunk
// cover its 16 k's once (the order inside a chunk is MFMA-internal, as for any fp32 GEMM).
// The B operand in global memory (weights; a party's features) runs through a RING of D chunks in
// flight: a global round trip is ~1-2 us here against ~0.2 us of MFMAs per chunk, so the refill
// of a slot is issued D chunks ahead. LDS operands (A always, B in WGRAD) are read one chunk ahead.
template <int AK, int BK, int ni, int nj>
__device__ __forceinline__ void mma_tile_n(const Opnd& A, const Opnd& Bo, int p0, int q0, int Kr,
                                           f4v (&acc)[2][2], int probe) {
  constexpr bool BG = BK >= O_GK;
  constexpr int D = BG ? MLP_RING : 1;
  const int lane = threadIdx.x & 63, r = lane & 15, g = lane >> 4;
  const bool ld = !(probe & 1);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) acc[i][jj] = f4v{0.f, 0.f, 0.f, 0.f};
  const int nch = (Kr + 15) >> 4;
  auto fetchA = [&](int ch, float (&a)[2][4]) {
    const int k0 = ch * 16;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (ld && i < ni) load4<AK>(A, p0 + 16 * i + r, k0 + 4 * g, Kr, a[i]);
      else {
#pragma unroll
        for (int j = 0; j < 4; ++j) a[i][j] = 0.f;
      }
    }
  };
  auto fetchB = [&](int ch, float (&b)[2][4]) {
    const int k0 = ch * 16;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (ld && i < nj && ch < nch) load4<BK>(Bo, q0 + 16 * i + r, k0 + 4 * g, Kr, b[i]);
      else {
#pragma unroll
        for (int j = 0; j < 4; ++j) b[i][j] = 0.f;
      }
    }
  };
  constexpr bool AG = AK >= O_GK;
  auto mfmas = [&](int ch, float (&a)[2][4], float (&b)[2][4]) {
    if (ch * 16 + 16 > Kr) {  // the tail chunk: zero the global operands past Kr
      if (AG) tail_zero(a, ch * 16 + 4 * g, Kr);
      if (BG) tail_zero(b, ch * 16 + 4 * g, Kr);
    }
    if (!(probe & 2)) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int jj = 0; jj < 2; ++jj)
            if (i < ni && jj < nj)
              acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][j], b[jj][j], acc[i][jj], 0, 0, 0);
    } else {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) acc[i][jj][0] += a[i][0] * b[jj][1];
    }
  };
  if (BG) {
    float rb[D][2][4];
#pragma unroll
    for (int d = 0; d < D; ++d) fetchB(d, rb[d]);
    for (int c0 = 0; c0 < nch; c0 += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const int ch = c0 + d;
        if (ch < nch) {
          float a[2][4], b[2][4];
          fetchA(ch, a);
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) b[i][j] = rb[d][i][j];
          if (ch + D < nch) fetchB(ch + D, rb[d]);
          mfmas(ch, a, b);
        }
      }
    }
  } else {  // ping-pong: chunk ch + 1 loads while chunk ch's MFMAs issue, no register copies
    float a0[2][4], b0[2][4], a1[2][4], b1[2][4];
    fetchA(0, a0);
    fetchB(0, b0);
    for (int ch = 0; ch < nch; ch += 2) {
      if (ch + 1 < nch) { fetchA(ch + 1, a1); fetchB(ch + 1, b1); }
      mfmas(ch, a0, b0);
      if (ch + 1 >= nch) break;
      if (ch + 2 < nch) { fetchA(ch + 2, a0); fetchB(ch + 2, b0); }
      mfmas(ch + 1, a1, b1);
    }
  }
}

// ni x nj (1 or 2 each): the sub-tiles holding output, a compile-time shape so the MFMAs of a
// chunk form one straight-line block (runtime guards would put each MFMA behind a branch)
template <int AK, int BK>
__device__ __forceinline__ void mma_tile(const Opnd& A, const Opnd& Bo, int p0, int q0, int ni, int nj,
                                         int Kr, f4v (&acc)[2][2], int probe) {
  if (ni == 2) {
    if (nj == 2) mma_tile_n<AK, BK, 2, 2>(A, Bo, p0, q0, Kr, acc, probe);
    else mma_tile_n<AK, BK, 2, 1>(A, Bo, p0, q0, Kr, acc, probe);
  } else {
    if (nj == 2) mma_tile_n<AK, BK, 1, 2>(A, Bo, p0, q0, Kr, acc, probe);
    else mma_tile_n<AK, BK, 1, 1>(A, Bo, p0, q0, Kr, acc, probe);
  }
}

// Phase hand-off through LDS: wait for this wave's LDS traffic, then the workgroup barrier. Global
// stores (weight gradients) stay in flight: their consumer, AdamW, sits behind a full
// __syncthreads, as does the next mini-batch's read of the updated weights.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

struct Ctx {
  const MlpEpochArgs* a;
  uint2 key;
  uint32_t step;  // this mini-batch's optimizer step (1-based, = FlatAdam t)
  int r0, M;      // first row of the mini-batch, rows in it
  int yoff;       // the mini-batch's targets [M][ncls], staged in the arena at step start
  float astep, sbc2;  // AdamW: lr / (1 - beta1^t), sqrt(1 - beta2^t)
};

// Job kinds of a phase; a wave takes tiles t = wave, wave + NWAVE, ... across the phase's jobs.
enum { J_FWD = 0, J_DGRAD = 1, J_WGRAD = 2, J_BIAS = 3, J_ADAM = 4 };
constexpr int ADAM_TILE = 1024;  // floats of one AdamW job tile (a wave: 4 float4 per lane)
__device__ __forceinline__ int slot64(int n) { return (n + 63) & ~63; }  // FlatAdam's parameter slots

__device__ __forceinline__ int job_tiles(const Ctx& c, const MlpLayer& L, int kind) {
  switch (kind) {
    case J_FWD: return ((c.M + 31) >> 5) * ((L.N + 31) >> 5);
    case J_DGRAD: return (L.need_dx && !(c.a->probe & 32)) ? ((c.M + 31) >> 5) * ((L.K + 31) >> 5) : 0;
    case J_WGRAD: return (c.a->probe & 64) ? 0 : ((L.N + 31) >> 5) * ((L.K + 31) >> 5);
    case J_BIAS: return (L.N + 63) >> 6;
    default:  // AdamW over the layer's W and b slots
      return (c.a->probe & 16) ? 0 : (slot64(L.N * L.K) + ADAM_TILE - 1) / ADAM_TILE + (slot64(L.N) + ADAM_TILE - 1) / ADAM_TILE;
  }
}

__device__ __forceinline__ float adam1(float p, float g, float& m, float& v, float lr, float wd, float b1,
                                       float b2, float step, float sbc2, float eps) {
  p *= (1.f - lr * wd);
  m = b1 * m + (1.f - b1) * g;
  v = b2 * v + (1.f - b2) * g * g;
  return p - step * m / (sqrtf(v) / sbc2 + eps);
}

// AdamW (optim.hip adam_kernel arithmetic) on `len` floats from `base` (a multiple of 64, inside
// one FlatAdam slot: whole float4s); the wave issues all of its loads before the first update.
__device__ __forceinline__ void adam_tile(const Ctx& c, long long base, int len) {
  const MlpEpochArgs& a = *c.a;
  const int lane = threadIdx.x & 63;
  gfloat4* P = reinterpret_cast<gfloat4*>(gp(a.p) + base);
  const gfloat4* G = reinterpret_cast<const gfloat4*>(gp(a.g) + base);
  gfloat4* Mm = reinterpret_cast<gfloat4*>(gp(a.m) + base);
  gfloat4* V = reinterpret_cast<gfloat4*>(gp(a.v) + base);
  constexpr int U = ADAM_TILE / 256;
  const int n4 = len >> 2;
  f4v p[U], g[U], m[U], v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int e = u * 64 + lane;
    if (e < n4) { p[u] = P[e]; g[u] = G[e]; m[u] = Mm[e]; v[u] = V[e]; }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int e = u * 64 + lane;
    if (e >= n4) continue;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float mm = m[u][q], vv = v[u][q];
      p[u][q] = adam1(p[u][q], g[u][q], mm, vv, a.lr, a.wd, a.beta1, a.beta2, c.astep, c.sbc2, a.eps);
      m[u][q] = mm;
      v[u][q] = vv;
    }
    P[e] = p[u]; Mm[e] = m[u]; V[e] = v[u];
  }
}

// AdamW over the whole flat buffer by all NT threads (the end-of-step form): three float4 per
// array per thread in flight, consecutive threads on consecutive float4s.
__device__ __forceinline__ void adam_all(const Ctx& c) {
  const MlpEpochArgs& a = *c.a;
  const long long n4 = a.nparam >> 2;
  gfloat4* P = reinterpret_cast<gfloat4*>(gp(a.p));
  const gfloat4* G = reinterpret_cast<const gfloat4*>(gp(a.g));
  gfloat4* Mm = reinterpret_cast<gfloat4*>(gp(a.m));
  gfloat4* V = reinterpret_cast<gfloat4*>(gp(a.v));
  constexpr int U = 3;
  for (long long e0 = threadIdx.x; e0 < n4; e0 += (long long)NT * U) {
    f4v p[U], g[U], m[U], v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long e = e0 + (long long)u * NT;
      if (e < n4) { p[u] = P[e]; g[u] = G[e]; m[u] = Mm[e]; v[u] = V[e]; }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long e = e0 + (long long)u * NT;
      if (e >= n4) continue;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float mm = m[u][q], vv = v[u][q];
        p[u][q] = adam1(p[u][q], g[u][q], mm, vv, a.lr, a.wd, a.beta1, a.beta2, c.astep, c.sbc2, a.eps);
        m[u][q] = mm;
        v[u][q] = vv;
      }
      P[e] = p[u]; Mm[e] = m[u]; V[e] = v[u];
    }
  }
}

template <int kind>
__device__ __forceinline__ void run_tile(const Ctx& c, const MlpLayer& L, int t) {
  const MlpEpochArgs& a = *c.a;
  const int lane = threadIdx.x & 63;
  if (a.probe & 8) return;
  if (kind == J_ADAM) {  // AdamW on one 1024-float tile of the layer's W slot, then its b slot
    const int nw = (slot64(L.N * L.K) + ADAM_TILE - 1) / ADAM_TILE;
    const long long base = t < nw ? L.w + (long long)t * ADAM_TILE : L.b + (long long)(t - nw) * ADAM_TILE;
    const int len = t < nw ? min(ADAM_TILE, slot64(L.N * L.K) - t * ADAM_TILE)
                           : min(ADAM_TILE, slot64(L.N) - (t - nw) * ADAM_TILE);
    adam_tile(c, base, len);
    return;
  }
  const MlpBuf& ob = a.bufs[L.out_buf];
  const int dpo = ob.off + L.out_col;  // this layer's output gradient (dp) in the arena
  if (kind == J_BIAS) {  // db[n] = sum_m dp[m][n], one column per lane, rows in order
    const int n = t * 64 + lane;
    if (n < L.N) {
      const float* d = arena + dpo + n;
      float s = 0.f;
#pragma unroll 16
      for (int m = 0; m < c.M; ++m) s += d[m * ob.ld];
      gp(a.g)[L.b + n] = s;
    }
    return;
  }
  const float* W = a.p + L.w;
  int P, Q;  // output extent: rows p (acc row index), cols q (lane column)
  if (kind == J_FWD) { P = c.M; Q = L.N; }
  else if (kind == J_DGRAD) { P = c.M; Q = L.K; }
  else { P = L.N; Q = L.K; }
  const int tq = (Q + 31) >> 5;
  const int p0 = (t / tq) * 32, q0 = (t % tq) * 32;
  const int ni = P - p0 > 16 ? 2 : 1, nj = Q - q0 > 16 ? 2 : 1;
  // epilogue operand issued before the MFMA loop: the bias of this lane's two columns
  float bias[2] = {0.f, 0.f};
  if (kind == J_FWD) {
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) bias[jj] = gp(a.p)[L.b + min(q0 + 16 * jj + (lane & 15), Q - 1)];
  }
  f4v acc[2][2];
  const bool xin = L.in_buf < 0;  // the input is a party's features (global memory)
  const int xp = xin ? -L.in_buf - 1 : 0;
  const float* xb = xin ? a.x[xp] + (long long)c.r0 * a.x_ld[xp] + L.in_col : nullptr;
  const MlpBuf& ib = a.bufs[xin ? 0 : L.in_buf];
  if (kind == J_FWD) {        // z[m][n]: A = in (m, k), B = W (n, k)
    if (xin) mma_tile<O_GK, O_GK>(gop(xb, a.x_ld[xp], c.M), gop(W, L.K, Q), p0, q0, ni, nj, L.K, acc, a.probe);
    else mma_tile<O_LK, O_GK>(lop(ib.off + L.in_col, ib.ld), gop(W, L.K, Q), p0, q0, ni, nj, L.K, acc, a.probe);
  } else if (kind == J_DGRAD) {  // d[m][k]: A = dp (m, n), B = W^T (k, n)
    if (a.probe & 128)  // timing probe: W^T read with the float4 pattern of a transposed copy
      mma_tile<O_LK, O_GK>(lop(dpo, ob.ld), gop(W, L.N, Q), p0, q0, ni, nj, L.N, acc, a.probe);
    else
      mma_tile<O_LK, O_GMN>(lop(dpo, ob.ld), gop(W, L.K, Q), p0, q0, ni, nj, L.N, acc, a.probe);
  } else {                    // g[n][k]: A = dp^T (n, m), B = in^T (k, m)
    if (xin) mma_tile<O_LMN, O_GMN>(lop(dpo, ob.ld), gop(xb, a.x_ld[xp], Q), p0, q0, ni, nj, c.M, acc, a.probe);
    else mma_tile<O_LMN, O_LMN>(lop(dpo, ob.ld), lop(ib.off + L.in_col, ib.ld), p0, q0, ni, nj, c.M, acc, a.probe);
  }
  if (a.probe & 4) {  // timing probe: no epilogue (keep the accumulators alive)
    if (acc[0][0][0] == 12345.f && acc[1][1][3] == 54321.f) gp(a.g)[0] = acc[0][1][2] + acc[1][0][1];
    return;
  }
  // C/D layout: column q = q0 + 16 jj + (lane & 15), rows p = p0 + 16 i + 4 (lane >> 4) + e.
  // FWD / DGRAD write every row of the tile (all inside the 32-padded arena): rows >= M as zeros,
  // which keeps the next WGRAD's reduction over the batch rows exact without checks.
  const bool fwd = kind == J_FWD;
  const MlpBuf& eb = fwd ? ob : ib;  // the buffer the epilogue writes (FWD: output; DGRAD: input, in place)
  const int ebuf = fwd ? L.out_buf : L.in_buf, ecol = fwd ? L.out_col : L.in_col;
  const float neg = act_neg(eb.act, eb.slope), drop = eb.drop, dscale = 1.f / (1.f - drop);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int q = q0 + 16 * jj + (lane & 15);
      if (q >= Q) continue;
      if (kind == J_WGRAD) {
        const int p = p0 + 16 * i + 4 * (lane >> 4);
        gfloat* gw = gp(a.g) + L.w + (unsigned)(p * L.K + q);
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (p + e < P) gw[e * L.K] = acc[i][jj][e];
        continue;
      }
      const int pr = p0 + 16 * i + 4 * (lane >> 4);  // this lane's 4 rows pr .. pr + 3
      const int col = ecol + q;
      uint4 rnd = make_uint4(0u, 0u, 0u, 0u);
      if (drop > 0.f) rnd = drop4(c.key, c.step, ebuf, pr >> 2, eb.ld, col);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int p = pr + e;
        float* dst = arena + eb.off + p * eb.ld + col;
        float v = acc[i][jj][e];
        if (fwd) v = act_fwd(v + bias[jj], neg);
        else v *= act_grad(*dst, neg);  // DGRAD: in place over the consumed input activation
        if (drop > 0.f) v = u32_to_unit(word(rnd, e)) > drop ? v * dscale : 0.f;
        *dst = p < P ? v : 0.f;
      }
    }
}

// One job (a layer x a kind): this wave's tiles t = wave - base (mod NWAVE), + NWAVE, ...; `base`
// carries the round-robin position over the phase's jobs so the waves stay balanced.
template <int KIND>
__device__ __forceinline__ void run_job(const Ctx& c, const MlpLayer& L, int& base, int& total) {
  const int wave = threadIdx.x >> 6;
  const int nt = job_tiles(c, L, KIND);
  int t = wave - base;
  if (t < 0) t += NWAVE;
  for (; t < nt; t += NWAVE) run_tile<KIND>(c, L, t);
  base = (base + nt) % NWAVE;
  total += nt;
}

// Run every tile of the jobs (layers of `level`, kinds in KMASK -- compile-time, so a phase holds
// only its own code; AdamW of the layers of `adam_level`, -2 = all) over the NWAVE waves;
// returns whether the phase had any work.
template <int KMASK>
__device__ __forceinline__ bool run_phase(const Ctx& c, int level, int adam_level = -1) {
  const MlpEpochArgs& a = *c.a;
  int base = 0, total = 0;
  for (int l = 0; l < a.nlayers; ++l) {
    const MlpLayer& L = a.layers[l];
    if (L.level == level) {
      if (KMASK & (1 << J_FWD)) run_job<J_FWD>(c, L, base, total);
      if (KMASK & (1 << J_DGRAD)) run_job<J_DGRAD>(c, L, base, total);
      if (KMASK & (1 << J_WGRAD)) run_job<J_WGRAD>(c, L, base, total);
      if (KMASK & (1 << J_BIAS)) run_job<J_BIAS>(c, L, base, total);
    }
    if ((KMASK & (1 << J_ADAM)) && (adam_level == -2 || L.level == adam_level)) run_job<J_ADAM>(c, L, base, total);
  }
  return total > 0;
}

// Soft-target CE over the logits buffer (wave 0, rows in order): loss_m = sum_c t (lse - z_c);
// batch loss = mean; the logits gradient (p * sum t - t) / M times the buffer's act' * mask,
// written in place over the logits.
__device__ __forceinline__ void ce_phase(const Ctx& c, float& loss_acc, float& correct_acc) {
  const MlpEpochArgs& a = *c.a;
  if (threadIdx.x >= 64) return;
  const int lane = threadIdx.x;
  const MlpBuf& lb = a.bufs[a.logits_buf];
  const int C = a.ncls;
  float lsum = 0.f, corr = 0.f;
  for (int m0 = 0; m0 < c.M; m0 += 64) {
    const int m = m0 + lane;
    if (m < c.M) {
      float* z = arena + lb.off + m * lb.ld;
      const float* t = arena + c.yoff + m * C;
      float mx = -INFINITY, tmx = -INFINITY;
      int am = 0, at = 0;
      for (int k = 0; k < C; ++k) {
        if (z[k] > mx) { mx = z[k]; am = k; }
        if (t[k] > tmx) { tmx = t[k]; at = k; }
      }
      float se = 0.f, ts = 0.f, tz = 0.f;
      for (int k = 0; k < C; ++k) {
        se += __expf(z[k] - mx);
        ts += t[k];
        tz += t[k] * z[k];
      }
      const float lse = mx + __logf(se);
      lsum += ts * lse - tz;
      corr += am == at ? 1.f : 0.f;
      const float neg = act_neg(lb.act, lb.slope);
      for (int k = 0; k < C; ++k) {
        const float zk = z[k];
        float v = (__expf(zk - mx) / se * ts - t[k]) / (float)c.M;
        v *= act_grad(zk, neg);
        if (lb.drop > 0.f)
          v = u32_to_unit(word(drop4(c.key, c.step, a.logits_buf, m >> 2, lb.ld, k), m & 3)) > lb.drop
                  ? v * (1.f / (1.f - lb.drop)) : 0.f;
        z[k] = v;
      }
    }
  }
  lsum = wave_sum(lsum);
  corr = wave_sum(corr);
  loss_acc += lsum / (float)c.M;
  correct_acc += corr;
}

__global__ __launch_bounds__(NT) void mlp_epoch_kernel(const MlpEpochArgs* __restrict__ ap) {
  // the tables: uniform loads through a const __restrict__ pointer -> scalar loads into SGPRs
  const MlpEpochArgs& args = *ap;
  Ctx c;
  c.a = ap;
  c.key = make_uint2((uint32_t)args.seed, (uint32_t)(args.seed >> 32));
  const unsigned long long t0 = *args.step_dev;
  const int nsteps = (args.n + args.B - 1) / args.B;
  float loss_acc = 0.f, correct_acc = 0.f;
  // phase clock (thread 0, LDS accumulators): only when a profile buffer is given
  __shared__ unsigned long long pt[NPROF];
  const bool prof = args.prof != nullptr;
  unsigned long long tprev = 0;
  if (prof && threadIdx.x < NPROF) pt[threadIdx.x] = 0;
  if (prof) {
    __syncthreads();
    tprev = wall_clock64();
  }
  auto tick = [&](int slot) {
    if (prof && threadIdx.x == 0) {
      const unsigned long long now = wall_clock64();
      pt[slot] += now - tprev;
      tprev = now;
    }
  };
  c.yoff = (int)args.lds_floats - args.B * args.ncls;
  for (int e = threadIdx.x; e < (int)args.lds_floats; e += NT) arena[e] = 0.f;  // pad rows / columns stay 0
  __syncthreads();
  for (int s = 0; s < nsteps; ++s) {
    c.r0 = s * args.B;
    c.M = min(args.B, args.n - c.r0);
    c.step = (uint32_t)(t0 + s + 1);
    {
      const float tf = (float)c.step;
      c.astep = args.lr / (1.f - powf(args.beta1, tf));
      c.sbc2 = sqrtf(1.f - powf(args.beta2, tf));
    }
    if ((threadIdx.x >> 6) == NWAVE - 1) {  // the last wave (no tile in the first phases) stages the targets
      const gfloat* y = gp(args.y) + (long long)c.r0 * args.ncls;
      for (int e = threadIdx.x & 63; e < c.M * args.ncls; e += 64) arena[c.yoff + e] = y[e];
    }
    for (int lev = 0; lev < args.nlev; ++lev) {
      run_phase<1 << J_FWD>(c, lev);
      lds_barrier();
      tick(lev);
    }
    ce_phase(c, loss_acc, correct_acc);
    lds_barrier();
    tick(MAXLEV);
    // Backward, level by level. AdamW of level l + 1 rides in level l's WGRAD phase: its weights
    // were last read by its DGRAD phase, and its gradients landed at the full barrier after it.
    for (int lev = args.nlev - 1; lev >= 0; --lev) {
      // reads this level's input activation
      if (MLP_ADAM_OVERLAP)
        run_phase<(1 << J_WGRAD) | (1 << J_BIAS) | (1 << J_ADAM)>(c, lev, lev + 1 < args.nlev ? lev + 1 : -1);
      else
        run_phase<(1 << J_WGRAD) | (1 << J_BIAS)>(c, lev);
      lds_barrier();
      run_phase<1 << J_DGRAD>(c, lev);  // then overwrites it with its gradient
      if (MLP_ADAM_OVERLAP) __syncthreads();  // + this level's weight-gradient stores have landed
      else lds_barrier();
      tick(MAXLEV + 1 + lev);
    }
    if (!MLP_ADAM_OVERLAP) __syncthreads();  // every weight-gradient store has landed
    if (MLP_ADAM_OVERLAP) run_phase<1 << J_ADAM>(c, -1, 0);  // AdamW of level 0
    else if (!(args.probe & 16)) adam_all(c);                 // AdamW of every level
    __syncthreads();  // the updated weights are visible to the next mini-batch
    tick(NPROF - 1);
  }
  if (prof && threadIdx.x < NPROF) args.prof[threadIdx.x] += pt[threadIdx.x];
  if (threadIdx.x == 0) {
    *args.step_dev = t0 + nsteps;
    args.stats[0] += loss_acc;
    args.stats[1] += correct_acc;
  }
}

constexpr int LDS_MAX_BYTES = 160 * 1024 - 1024;  // the arena; the phase clock takes the rest

}  // namespace

// a: the tables on the host (validated here); dev: the same bytes in device memory (the kernel
// reads its tables from there: uploaded once per configuration by ops/mlp_epoch.py)
DDL_API int ddl_mlp_epoch(const MlpEpochArgs* a, const MlpEpochArgs* dev, hipStream_t s) {
  if (a->n <= 0 || a->B <= 0 || a->nlayers <= 0 || a->nlayers > MAXL || a->nbufs <= 0 || a->nbufs > MAXB ||
      a->nlev <= 0 || a->nlev > MAXLEV || a->logits_buf < 0 || a->logits_buf >= a->nbufs || a->ncls <= 0 ||
      a->ncls > a->bufs[a->logits_buf].width || a->lds_floats <= 0 || a->lds_floats * 4 > LDS_MAX_BYTES)
    return (int)hipErrorInvalidValue;
  if ((a->nparam & 3) || ((uintptr_t)a->p | (uintptr_t)a->g | (uintptr_t)a->m | (uintptr_t)a->v) & 15)
    return (int)hipErrorInvalidValue;  // AdamW runs on float4s
  const long long yoff = a->lds_floats - (long long)a->B * a->ncls;  // the staged targets end the arena
  const long long rows = (a->B + 31) / 32 * 32;  // buffers are padded to whole 32-row tiles
  for (int i = 0; i < a->nbufs; ++i) {  // every buffer [rows][ld] inside the arena, before the targets
    const MlpBuf& b = a->bufs[i];
    if (b.off < 0 || (b.off & 3) || (b.ld & 3) || b.width <= 0 || b.ld < b.width + 1 ||
        (long long)b.off + rows * b.ld > yoff)
      return (int)hipErrorInvalidValue;
  }
  for (int l = 0; l < a->nlayers; ++l) {
    const MlpLayer& L = a->layers[l];
    if (L.K <= 0 || L.N <= 0 || L.level < 0 || L.level >= a->nlev || L.out_buf < 0 || L.out_buf >= a->nbufs ||
        L.out_col < 0 || L.out_col + L.N > a->bufs[L.out_buf].width || L.w < 0 || L.b < 0 ||
        L.w + (long long)L.N * L.K > a->nparam || L.b + L.N > a->nparam)
      return (int)hipErrorInvalidValue;
    if (L.in_buf >= 0) {
      if (L.in_buf >= a->nbufs || L.in_col < 0 || L.in_col + L.K > a->bufs[L.in_buf].width)
        return (int)hipErrorInvalidValue;
    } else {
      const int p = -L.in_buf - 1;
      if (p >= MAXP || !a->x[p] || L.in_col < 0 || L.in_col + L.K > a->x_ld[p] || L.need_dx)
        return (int)hipErrorInvalidValue;
    }
  }
  if (!dev) return (int)hipErrorInvalidValue;
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute((const void*)mlp_epoch_kernel,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX_BYTES);
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  hipLaunchKernelGGL(mlp_epoch_kernel, dim3(1), dim3(NT), (size_t)a->lds_floats * 4, s, dev);
  return (int)hipGetLastError();
}

DDL_API int ddl_mlp_epoch_args_size() { return (int)sizeof(MlpEpochArgs); }
DDL_API int ddl_mlp_epoch_lds_max() { return LDS_MAX_BYTES; }
