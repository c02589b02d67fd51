// Common device helpers for the ddl25spring_amd HIP kernels (gfx950 / CDNA4 only).
//
// Conventions used by every kernel in csrc/kernels:
//   * activations are NHWC bf16 (or fp32 in the reference-precision mode: conv_f32.hip,
//     bn_f32.hip and the `_f32` twins of the memory-bound launchers) with a leading "group"
//     (= simulated FL client) dimension:
//     x[g][n][h][w][c]; every launch covers all groups through blockIdx.z (client-batched
//     execution, one launch for all clients resident on the GPU).
//   * master weights / grads / optimizer state are fp32 flat buffers [G][P]; the kernels
//     read a bf16 shadow of the weights with the same [G][P] layout.
//   * every exported launcher is `extern "C"` (loaded through ctypes) and returns a
//     hipError_t as int; 0 == success.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DDL_API extern "C" __attribute__((visibility("default")))

// Host helper: 1-D grid for a grid-stride loop over `work` items (capped: waves re-use blocks).
static inline int grid_for(long long work, int block, int cap = 8192) {
  long long b = (work + block - 1) / block;
  if (b > cap) b = cap;
  if (b < 1) b = 1;
  return (int)b;
}
#define GSTRIDE_LOOP(t, total) \
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < (total); \
       t += (long long)gridDim.x * blockDim.x)


typedef uint16_t bf16_t;
typedef short s8v __attribute__((ext_vector_type(8)));   // 8 x bf16 MFMA operand (4 VGPRs)
typedef short s4v __attribute__((ext_vector_type(4)));   // 4 x bf16
typedef float f4v __attribute__((ext_vector_type(4)));   // 16x16 MFMA accumulator
typedef int i4v __attribute__((ext_vector_type(4)));     // raw 16 bytes
typedef int i2v __attribute__((ext_vector_type(2)));     // raw 8 bytes

#define WAVE 64

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

// Plain cast: hipcc emits v_cvt_pk_bf16_f32 (RNE, NaN-preserving) on gfx950.
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}

__device__ __forceinline__ float lo_bf(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float hi_bf(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }
__device__ __forceinline__ uint32_t pack_bf2(float a, float b) {
  return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
}

// unpack 8 bf16 packed in an i4v into floats
__device__ __forceinline__ void unpack8(const i4v& v, float* f) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    uint32_t u = (uint32_t)v[i];
    f[2 * i] = lo_bf(u);
    f[2 * i + 1] = hi_bf(u);
  }
}
__device__ __forceinline__ i4v pack8(const float* f) {
  i4v v;
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = (int)pack_bf2(f[2 * i], f[2 * i + 1]);
  return v;
}

// 8 consecutive activations <-> 8 floats, for kernels templated on the activation type
// (bf16 storage: one 16-B access; fp32 storage — the reference-precision mode: two).
__device__ __forceinline__ void ld8(const bf16_t* p, float* v) { unpack8(*(const i4v*)p, v); }
__device__ __forceinline__ void ld8(const float* p, float* v) {
  const float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ void st8(bf16_t* p, const float* v) { *(i4v*)p = pack8(v); }
__device__ __forceinline__ void st8(float* p, const float* v) {
  *(float4*)p = make_float4(v[0], v[1], v[2], v[3]);
  *(float4*)(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}
__device__ __forceinline__ float ld1(const bf16_t* p) { return bf2f(*p); }
__device__ __forceinline__ float ld1(const float* p) { return *p; }
__device__ __forceinline__ void st1(bf16_t* p, float v) { *p = f2bf(v); }
__device__ __forceinline__ void st1(float* p, float v) { *p = v; }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Counter-based RNG (Philox-4x32-10): dropout / reparameterisation noise is a pure function
// of (seed, element index), so backward recomputes masks instead of storing them.
__device__ __forceinline__ uint4 philox4x32(uint4 ctr, uint2 key) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    uint32_t hi0 = __umulhi(0xD2511F53u, ctr.x), lo0 = 0xD2511F53u * ctr.x;
    uint32_t hi1 = __umulhi(0xCD9E8D57u, ctr.z), lo1 = 0xCD9E8D57u * ctr.z;
    ctr = make_uint4(hi1 ^ ctr.y ^ key.x, lo1, hi0 ^ ctr.w ^ key.y, lo0);
    key.x += 0x9E3779B9u;
    key.y += 0xBB67AE85u;
  }
  return ctr;
}
__device__ __forceinline__ float u32_to_unit(uint32_t x) {  // (0,1]
  return ((float)(x >> 8) + 1.0f) * (1.0f / 16777216.0f);
}

// Bijective XCD-aware remap of a 1-D block id (8 XCDs, round-robin dispatch): consecutive
// logical tiles land on the same XCD (shared L2) — see cdna_hip_programming.md T1.
// 3-D grid (tiles t fastest, then y, z) -> (t, y, z) such that every XCD gets the same MIX of t.
// Workgroups are dealt round-robin over the 8 XCDs in grid order, so with a small tile extent
// (causal attention: 4 query tiles at S = 256, work 1:2:3:4) XCD k would only ever receive tile
// k mod 4. Bijective when the grid divides into 8 x tiles; the identity otherwise.
__device__ __forceinline__ void xcd_spread_block(int& t, int& y, int& z) {
  const int nt = gridDim.x, ny = gridDim.y, nz = gridDim.z;
  const int lin = blockIdx.x + nt * (blockIdx.y + ny * blockIdx.z);
  if ((nt * ny * nz) % (8 * nt) == 0) {
    const int xcd = lin & 7, j = lin >> 3;
    // an XCD's 32 CUs take its workgroups in turn: rotating by the round (j / 32) also gives each
    // CU's co-resident workgroups different tiles (groups of nt consecutive j never straddle a
    // round when nt divides 32, so the map stays bijective)
    t = (32 % nt == 0) ? (j + (j >> 5)) % nt : j % nt;
    const int rest = (j / nt) * 8 + xcd;
    y = rest % ny;
    z = rest / ny;
  } else {
    t = blockIdx.x; y = blockIdx.y; z = blockIdx.z;
  }
}

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int nx = 8;
  if (nwg < nx * 2) return bid;
  int q = nwg / nx, r = nwg % nx;
  int xcd = bid % nx, idx = bid / nx;
  int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + idx;
}
