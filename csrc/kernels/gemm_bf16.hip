// Wide-output bf16 GEMM  Y[T][V] = X[T][C] . W[V][C]^T  (bf16 in, fp32 accumulate, bf16 out) on
// the gfx950 double-rate MFMA (v_mfma_f32_16x16x32_bf16) — the LLaMA LM-head forward
// (8192 tokens x 288 -> 32000 vocab: 151 GFLOP, a 524 MB logits write; reference
// lab/tutorial_1b/primer/intro.py:17-30 via simplellm's LLama). The general MFMA conv-GEMM
// (conv_igemm.hip) runs this shape at 389 us against hipBLASLt's 264 us: with only 9 reduction
// steps its tile's output write is never overlapped. Here:
//   * 128 (vocab) x 128 (token) tiles, 4 waves in 2x2, each 64 x 64 = 4 x 4 MFMA tiles; 32-deep
//     steps (one x32 MFMA k-extent) through a 2-stage LDS ring, register-prefetched one step
//     ahead with 16-byte buffer loads (rows past T / V read as zeros, branch-free);
//   * LDS image [row][32 bf16] with 16-B chunk c at c ^ ((row >> 2) & 2): every fragment is one
//     conflict-free ds_read_b128 for the b128 lane groups;
//   * D is oriented vocab x token, so a lane's accumulator holds 4 consecutive vocab entries of
//     one token; the finished tile is staged through LDS as [token][vocab] and written as whole
//     256-B rows with 16-B stores (the write is the roofline of this shape: 65 us of 8 TB/s);
//   * small per-block LDS (34 KB) and ~100 VGPRs: 4 blocks per CU, so one block's store burst
//     overlaps its neighbours' MFMA loops;
//   * block order: consecutive blocks share a vocab tile across a group of 4 token tiles (the W
//     tile is reused 4x while resident) and the group's token tiles stay hot in L2 while the
//     vocab tiles advance; xcd_remap gives each XCD a contiguous range of that order.
#include "ddl_common.h"

namespace {
constexpr int GB = 128;       // tile edge (vocab and token)
constexpr int GK = 32;        // reduction step
constexpr int GROUP = 4;      // token tiles per W-tile reuse group
constexpr int STG = GB + 8;   // staging row stride (bf16) for the output tile

__device__ __forceinline__ int goff(int row, int ch) { return row * GK + ((ch ^ ((row >> 2) & 2)) << 3); }

__global__ __launch_bounds__(256, 4) void gemm_nt_bf16_kernel(const bf16_t* __restrict__ X,
                                                             const bf16_t* __restrict__ Wv,
                                                             bf16_t* __restrict__ Y, int T, int V,
                                                             int C, long long ldy) {
  constexpr int IMG = GB * GK;  // bf16 per operand image
  __shared__ __attribute__((aligned(16))) bf16_t smem[(2 * 2 * IMG > GB * STG) ? 2 * 2 * IMG : GB * STG];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wp = wid >> 1, wq = wid & 1;
  const int ntp = (V + GB - 1) / GB, ntq = (T + GB - 1) / GB;
  const int nwg = gridDim.x;
  const int u = xcd_remap(blockIdx.x, nwg);
  const int per_group = ntp * GROUP;
  const int tg = u / per_group, rem = u - tg * per_group;
  const int tp = rem / GROUP, tq = tg * GROUP + rem % GROUP;
  if (tq >= ntq) return;
  const int p0 = tp * GB, q0 = tq * GB;

  constexpr unsigned OOB = 0xFFFFFFF0u;
  const __amdgpu_buffer_rsrc_t rW = __builtin_amdgcn_make_buffer_rsrc((void*)Wv, 0, (int)((long long)V * C * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rX = __builtin_amdgcn_make_buffer_rsrc((void*)X, 0, (int)((long long)T * C * 2), 0x00020000);
  // two 16-B chunks per operand per thread and step: chunk id c = tid + 256 i -> row c >> 2, ch c & 3
  int rowc[2], chc[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = tid + 256 * i;
    rowc[i] = c >> 2;
    chc[i] = c & 3;
  }
  i4v rp[2], rq[2];
  auto load_step = [&](int kt) {
    const int k0 = kt * GK;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int p = p0 + rowc[i], q = q0 + rowc[i];
      const unsigned kb = (unsigned)(k0 + 8 * chc[i]) * 2u;
      rp[i] = __builtin_bit_cast(i4v, __builtin_amdgcn_raw_buffer_load_b128(
          rW, p < V ? (unsigned)p * (unsigned)C * 2u + kb : OOB, 0, 0));
      rq[i] = __builtin_bit_cast(i4v, __builtin_amdgcn_raw_buffer_load_b128(
          rX, q < T ? (unsigned)q * (unsigned)C * 2u + kb : OOB, 0, 0));
    }
  };
  auto store_step = [&](int buf) {
    bf16_t* Ps = smem + buf * 2 * IMG;
    bf16_t* Qs = Ps + IMG;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      *(i4v*)(Ps + goff(rowc[i], chc[i])) = rp[i];
      *(i4v*)(Qs + goff(rowc[i], chc[i])) = rq[i];
    }
  };

  f4v acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f4v){0.f, 0.f, 0.f, 0.f};

  const int nk = C / GK;
  load_step(0);
  store_step(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) load_step(kt + 1);
    const bf16_t* Ps = smem + cur * 2 * IMG;
    const bf16_t* Qs = Ps + IMG;
    s8v af[4], bfr[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      af[t] = *(const s8v*)(Ps + goff(wp * 64 + t * 16 + (lane & 15), lane >> 4));
      bfr[t] = *(const s8v*)(Qs + goff(wq * 64 + t * 16 + (lane & 15), lane >> 4));
    }
#pragma unroll
    for (int ti = 0; ti < 4; ++ti)
#pragma unroll
      for (int tj = 0; tj < 4; ++tj)
        acc[ti][tj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ti], bfr[tj], acc[ti][tj], 0, 0, 0);
    if (more) store_step(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue: stage [token][vocab] bf16 through LDS, then whole-row 16-B stores
  // acc[ti][tj][v] = D[p = wp*64 + ti*16 + 4*(lane>>4) + v][q = wq*64 + tj*16 + (lane&15)]
#pragma unroll
  for (int ti = 0; ti < 4; ++ti)
#pragma unroll
    for (int tj = 0; tj < 4; ++tj) {
      const int p = wp * 64 + ti * 16 + 4 * (lane >> 4);
      const int q = wq * 64 + tj * 16 + (lane & 15);
      i2v v;
      v[0] = (int)pack_bf2(acc[ti][tj][0], acc[ti][tj][1]);
      v[1] = (int)pack_bf2(acc[ti][tj][2], acc[ti][tj][3]);
      *(i2v*)(smem + q * STG + p) = v;
    }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < (GB * GB / 8) / 256; ++i) {
    const int c = tid + 256 * i;
    const int q = c >> 4, pc = (c & 15) * 8;
    const int gq = q0 + q, gp = p0 + pc;
    if (gq < T && gp < V) *(i4v*)(Y + (long long)gq * ldy + gp) = *(const i4v*)(smem + q * STG + pc);
  }
}
}  // namespace

// Y[T][V] (row stride ldy) = X[T][C] . W[V][C]^T, all bf16 row-major. C % 32 == 0, V % 8 == 0.
DDL_API int ddl_gemm_nt_bf16(const void* X, const void* W, void* Y, int T, int V, int C, long long ldy,
                             hipStream_t s) {
  if (T < 1 || V < 1 || C < GK || C % GK || V % 8 || ldy < V || ldy % 8) return (int)hipErrorInvalidValue;
  if ((long long)V * C * 2 >= (1LL << 31) || (long long)T * C * 2 >= (1LL << 31)) return (int)hipErrorInvalidValue;
  const long long ntp = (V + GB - 1) / GB, ntq = (T + GB - 1) / GB;
  const long long groups = (ntq + GROUP - 1) / GROUP;
  const long long blocks = groups * ntp * GROUP;
  if (blocks > 0x7fffffffLL) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(gemm_nt_bf16_kernel, dim3((unsigned)blocks), dim3(256), 0, s, (const bf16_t*)X,
                     (const bf16_t*)W, (bf16_t*)Y, T, V, C, ldy);
  return (int)hipGetLastError();
}
