// Memory-bound NN building blocks (NHWC bf16, leading client-group dim), all vectorised to
// 16-byte accesses and grid-strided (cdna_hip_programming.md Guideline 11/13).
//
//   ddl_prep_images   : device-resident dataset gather (uint8 HWC) + normalise + optional stem
//                       im2col into a 32-channel NHWC bf16 tensor (fuses the first conv's im2col
//                       into the data loader so the stem runs as a K=32 GEMM on MFMA)
//   ddl_nchw_to_nhwc  : fp32 NCHW -> NHWC bf16 (channel-padded) for the torch-compatible API
//   ddl_maxpool2_*    : 2x2/2 max pool fwd + bwd (argmax recomputed, first-max like torch)
//   ddl_avgpool_*     : global average pool fwd + bwd
//   ddl_dropout       : Philox counter-based dropout, mask recomputed in backward
//   ddl_act_*         : relu / leaky-relu fwd + masked bwd
//   ddl_channel_sum   : per-channel sum (bias grads), fp32 atomics into the flat grad buffer
//   ddl_cast_*        : fp32 <-> bf16
//
// Reference parity: F.relu / F.max_pool2d / nn.Dropout / torch.flatten of MnistCnn
// (reference lab/tutorial_1a/hfl_complete.py:50-62) and transforms.Normalize (:19-24).
#include "ddl_common.h"

// ---------------------------------------------------------------------------------------------
// src: uint8 [num_samples][Hs][Ws][Cs]; idx: int32 [G*B] sample ids (row-major over g,b)
// im2col=0: out [G*B][Hs][Ws][Cout], channel c<Cs normalised, c>=Cs zero
// im2col=k>0: out [G*B][Ho][Wo][Cout] with Ho=(Hs+2pad-k)/stride+1, channel j=(r*k+s)*Cs+c
// (< k*k*Cs), rest 0 — the stem conv then runs as a 1x1 GEMM on MFMA.
// Also gathers the labels (labels_out[b] = labels[idx[b]], nullable) so a training step's whole
// batch materialisation is one launch.
template <typename T>
__global__ void prep_images_kernel(const uint8_t* __restrict__ src, const int* __restrict__ idx,
                                   const float* __restrict__ mean, const float* __restrict__ inv_std,
                                   T* __restrict__ out, int nimg, int Hs, int Ws, int Cs,
                                   int Ho, int Wo, int Cout, int im2col, int pad, int stride,
                                   const int* __restrict__ labels, int* __restrict__ labels_out) {
  const long long total = (long long)nimg * Ho * Wo * (Cout / 8);
  GSTRIDE_LOOP(t, total) {
    const int cchunk = (int)(t % (Cout / 8));
    long long pix = t / (Cout / 8);
    const int w = (int)(pix % Wo);
    pix /= Wo;
    const int h = (int)(pix % Ho);
    const int b = (int)(pix / Ho);
    const int id = idx[b];
    const long long sbase = (long long)id * Hs * Ws * Cs;
    if (labels && (cchunk | h | w) == 0) labels_out[b] = labels[id];
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int ch = cchunk * 8 + k;
      float val = 0.f;
      if (!im2col) {
        if (ch < Cs) val = ((float)src[sbase + ((long long)h * Ws + w) * Cs + ch] * (1.f / 255.f) - mean[ch]) * inv_std[ch];
      } else if (ch < im2col * im2col * Cs) {
        const int tap = ch / Cs, c = ch - tap * Cs;
        const int r = tap / im2col, s = tap - r * im2col;
        const int ih = h * stride - pad + r, iw = w * stride - pad + s;
        if ((unsigned)ih < (unsigned)Hs && (unsigned)iw < (unsigned)Ws)
          val = ((float)src[sbase + ((long long)ih * Ws + iw) * Cs + c] * (1.f / 255.f) - mean[c]) * inv_std[c];
        // zero padding happens in normalised space (matches conv zero-padding)
      }
      v[k] = val;
    }
    st8(out + t * 8, v);
  }
}

// Fast path of the 32-channel stem im2col (CIFAR 3x3x3 = 27, MNIST 3x3x1 = 9 of 32 channels): one
// thread per output pixel with 32-bit index math, the k x k x CS neighbourhood read once, and the
// pixel's 64 B written as four 16-B stores. The generic kernel above decodes 64-bit indices and
// re-gathers the neighbourhood per 8-channel chunk (ALU-bound: 57 us for the 8-client CIFAR
// batch, ~1 TB/s of output).
template <int K, int CS, typename T>
__global__ __launch_bounds__(256) void prep_stem32_kernel(
    const uint8_t* __restrict__ src, const int* __restrict__ idx, const float* __restrict__ mean,
    const float* __restrict__ inv_std, T* __restrict__ out, int nimg, int Hs, int Ws, int Ho,
    int Wo, int pad, int stride, const int* __restrict__ labels, int* __restrict__ labels_out) {
  static_assert(K * K * CS <= 32, "stem im2col fits 32 channels");
  const int hw = Ho * Wo;
  const int pix = blockIdx.x * 256 + threadIdx.x;
  if (pix >= nimg * hw) return;
  const int b = pix / hw, r = pix - b * hw;
  const int h = r / Wo, w = r - h * Wo;
  const int id = idx[b];
  if (labels && r == 0) labels_out[b] = labels[id];
  const uint8_t* img = src + (long long)id * Hs * Ws * CS;
  float m[CS], is[CS];
#pragma unroll
  for (int c = 0; c < CS; ++c) { m[c] = mean[c]; is[c] = inv_std[c]; }
  float v[32];
#pragma unroll
  for (int j = 0; j < 32; ++j) v[j] = 0.f;
#pragma unroll
  for (int tr = 0; tr < K; ++tr) {
    const int ih = h * stride - pad + tr;
#pragma unroll
    for (int ts = 0; ts < K; ++ts) {
      const int iw = w * stride - pad + ts;
      if ((unsigned)ih < (unsigned)Hs && (unsigned)iw < (unsigned)Ws) {
        const uint8_t* px = img + (ih * Ws + iw) * CS;
#pragma unroll
        for (int c = 0; c < CS; ++c)
          v[(tr * K + ts) * CS + c] = ((float)px[c] * (1.f / 255.f) - m[c]) * is[c];
      }
    }
  }
  T* o = out + (long long)pix * 32;
#pragma unroll
  for (int q = 0; q < 4; ++q) st8(o + 8 * q, v + 8 * q);
}

// Fast path of a wider stem im2col (ImageNet 7x7x3 / stride 2 -> 147 of 160 channels): one
// thread per (output pixel, 8-channel chunk) as the generic kernel, but 32-bit index math and
// compile-time tap decoding (the generic kernel's 64-bit divisions made the 1 GB ResNet-50 batch
// gather ALU-bound: 1.07 ms per step).
template <int K, int CS, typename T>
__global__ __launch_bounds__(256) void prep_im2col_kernel(
    const uint8_t* __restrict__ src, const int* __restrict__ idx, const float* __restrict__ mean,
    const float* __restrict__ inv_std, T* __restrict__ out, int nimg, int Hs, int Ws, int Ho,
    int Wo, int nch, int pad, int stride, const int* __restrict__ labels, int* __restrict__ labels_out) {
  const int hw = Ho * Wo;
  const unsigned total = (unsigned)nimg * hw * nch;
  const unsigned t = blockIdx.x * 256u + threadIdx.x;
  if (t >= total) return;
  const int chunk = (int)(t % (unsigned)nch);
  const int pix = (int)(t / (unsigned)nch);
  const int b = pix / hw, r = pix - b * hw;
  const int h = r / Wo, w = r - h * Wo;
  const int id = idx[b];
  if (labels && r == 0 && chunk == 0) labels_out[b] = labels[id];
  const uint8_t* img = src + (long long)id * Hs * Ws * CS;
  const int h0 = h * stride - pad, w0 = w * stride - pad;
  float v[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int j = chunk * 8 + k;
    const int tap = j / CS, c = j - tap * CS;
    const int tr = tap / K, ts = tap - tr * K;
    const int ih = h0 + tr, iw = w0 + ts;
    float val = 0.f;
    if (tap < K * K && (unsigned)ih < (unsigned)Hs && (unsigned)iw < (unsigned)Ws)
      val = ((float)img[(ih * Ws + iw) * CS + c] * (1.f / 255.f) - mean[c]) * inv_std[c];
    v[k] = val;
  }
  st8(out + (long long)t * 8, v);
}

// ImageNet stem im2col, one block per (image, output row): the K input rows the row's windows
// cover are staged in LDS once, normalised to fp32 with the zero padding materialised (coalesced
// 4-byte loads of the uint8 image), then every thread writes whole 16-byte chunks of consecutive
// pixels' im2col rows (the block's output is one contiguous Wo x Cout run). The per-chunk kernel
// above gathers its 8 bytes from 8 scattered taps of the uint8 image per thread: 667 us for a
// batch of 256 at 224x224 (1 GB written at 1.5 TB/s).
template <int K, int CS, typename T>
__global__ __launch_bounds__(256) void prep_im2col_row_kernel(
    const uint8_t* __restrict__ src, const int* __restrict__ idx, const float* __restrict__ mean,
    const float* __restrict__ inv_std, T* __restrict__ out, int Hs, int Ws, int Ho, int Wo,
    int nch, int pad, int stride, int Wl, const int* __restrict__ labels, int* __restrict__ labels_out) {
  extern __shared__ float rows[];  // [K][Wl][CS], column 0 = input column -pad
  const int b = blockIdx.y, h = blockIdx.x, tid = threadIdx.x;
  const int id = idx[b];
  if (labels && h == 0 && tid == 0) labels_out[b] = labels[id];
  const uint8_t* img = src + (long long)id * Hs * Ws * CS;
  const int h0 = h * stride - pad;
  float mu[CS], is[CS];
#pragma unroll
  for (int c = 0; c < CS; ++c) { mu[c] = mean[c]; is[c] = inv_std[c]; }
  const int per_row = Wl * CS;
  for (int t = tid; t < K * per_row; t += 256) {
    const int tr = t / per_row, rem = t - tr * per_row;
    const int col = rem / CS, c = rem - col * CS;
    const int ih = h0 + tr, iw = col - pad;
    float v = 0.f;
    if ((unsigned)ih < (unsigned)Hs && (unsigned)iw < (unsigned)Ws)
      v = ((float)img[((long long)ih * Ws + iw) * CS + c] * (1.f / 255.f) - mu[c]) * is[c];
    rows[t] = v;
  }
  __syncthreads();
  T* o = out + ((long long)b * Ho + h) * Wo * nch * 8;
  for (int q = tid; q < Wo * nch; q += 256) {
    const int px = q / nch, chunk = q - px * nch;
    const int wbase = px * stride;
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int j = chunk * 8 + k;
      const int tap = j / CS, c = j - tap * CS;
      const int tr = tap / K, ts = tap - tr * K;
      v[k] = tap < K * K ? rows[(tr * Wl + wbase + ts) * CS + c] : 0.f;
    }
    st8(o + (long long)q * 8, v);
  }
}

template <typename T>
static int prep_images_impl(const void* src, const int* idx, const float* mean, const float* inv_std,
                            void* out, int nimg, int Hs, int Ws, int Cs, int Cout, int im2col,
                            int pad, int stride, const int* labels, int* labels_out, hipStream_t s) {
  if (Cout % 8 || stride < 1) return (int)hipErrorInvalidValue;
  if (im2col && im2col * im2col * Cs > Cout) return (int)hipErrorInvalidValue;
  if ((labels == nullptr) != (labels_out == nullptr)) return (int)hipErrorInvalidValue;
  const int Ho = im2col ? (Hs + 2 * pad - im2col) / stride + 1 : Hs;
  const int Wo = im2col ? (Ws + 2 * pad - im2col) / stride + 1 : Ws;
  const long long pixels = (long long)nimg * Ho * Wo;
  if (Cout == 32 && im2col == 3 && (Cs == 3 || Cs == 1) && pixels < (1LL << 31) - 256) {
    const dim3 grid((unsigned)((pixels + 255) / 256));
    if (Cs == 3)
      hipLaunchKernelGGL((prep_stem32_kernel<3, 3, T>), grid, dim3(256), 0, s, (const uint8_t*)src, idx,
                         mean, inv_std, (T*)out, nimg, Hs, Ws, Ho, Wo, pad, stride, labels, labels_out);
    else
      hipLaunchKernelGGL((prep_stem32_kernel<3, 1, T>), grid, dim3(256), 0, s, (const uint8_t*)src, idx,
                         mean, inv_std, (T*)out, nimg, Hs, Ws, Ho, Wo, pad, stride, labels, labels_out);
    return (int)hipGetLastError();
  }
  const long long total = (long long)nimg * Ho * Wo * (Cout / 8);
  const int Wl = (Wo - 1) * stride + im2col;  // input columns the row's windows span
  if (im2col == 7 && Cs == 3 && 7 * Wl * 3 * 4 <= 64 * 1024 && Ho < 65536) {
    hipLaunchKernelGGL((prep_im2col_row_kernel<7, 3, T>), dim3(Ho, nimg), dim3(256), 7 * Wl * 3 * 4, s,
                       (const uint8_t*)src, idx, mean, inv_std, (T*)out, Hs, Ws, Ho, Wo, Cout / 8,
                       pad, stride, Wl, labels, labels_out);
    return (int)hipGetLastError();
  }
  if (im2col == 7 && Cs == 3 && total < (1LL << 31) - 256) {
    hipLaunchKernelGGL((prep_im2col_kernel<7, 3, T>), dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                       (const uint8_t*)src, idx, mean, inv_std, (T*)out, nimg, Hs, Ws, Ho, Wo,
                       Cout / 8, pad, stride, labels, labels_out);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(prep_images_kernel<T>, dim3(grid_for(total, 256)), dim3(256), 0, s,
                     (const uint8_t*)src, idx, mean, inv_std, (T*)out, nimg, Hs, Ws, Cs, Ho, Wo,
                     Cout, im2col, pad, stride, labels, labels_out);
  return (int)hipGetLastError();
}

// fp32 NCHW (already normalised) -> NHWC bf16, optionally im2col 3x3 (same rules as above)
template <typename T>
__global__ void nchw_to_nhwc_kernel(const float* __restrict__ x, T* __restrict__ out, int N,
                                    int Cs, int Hs, int Ws, int Ho, int Wo, int Cout, int im2col,
                                    int pad, int stride) {
  const long long total = (long long)N * Ho * Wo * (Cout / 8);
  GSTRIDE_LOOP(t, total) {
    const int cchunk = (int)(t % (Cout / 8));
    long long pix = t / (Cout / 8);
    const int w = (int)(pix % Wo);
    pix /= Wo;
    const int h = (int)(pix % Ho);
    const int n = (int)(pix / Ho);
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int ch = cchunk * 8 + k;
      float val = 0.f;
      if (!im2col) {
        if (ch < Cs) val = x[(((long long)n * Cs + ch) * Hs + h) * Ws + w];
      } else if (ch < im2col * im2col * Cs) {
        const int tap = ch / Cs, c = ch - tap * Cs;
        const int r = tap / im2col, s = tap - r * im2col;
        const int ih = h * stride - pad + r, iw = w * stride - pad + s;
        if ((unsigned)ih < (unsigned)Hs && (unsigned)iw < (unsigned)Ws)
          val = x[(((long long)n * Cs + c) * Hs + ih) * Ws + iw];
      }
      v[k] = val;
    }
    st8(out + t * 8, v);
  }
}

template <typename T>
static int nchw_to_nhwc_impl(const float* x, void* out, int N, int Cs, int Hs, int Ws, int Cout,
                             int im2col, int pad, int stride, hipStream_t s) {
  if (Cout % 8 || stride < 1) return (int)hipErrorInvalidValue;
  if (im2col && im2col * im2col * Cs > Cout) return (int)hipErrorInvalidValue;
  const int Ho = im2col ? (Hs + 2 * pad - im2col) / stride + 1 : Hs;
  const int Wo = im2col ? (Ws + 2 * pad - im2col) / stride + 1 : Ws;
  const long long total = (long long)N * Ho * Wo * (Cout / 8);
  hipLaunchKernelGGL(nchw_to_nhwc_kernel<T>, dim3(grid_for(total, 256)), dim3(256), 0, s, x,
                     (T*)out, N, Cs, Hs, Ws, Ho, Wo, Cout, im2col, pad, stride);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// 2x2 stride-2 max pool over NHWC (NB = G*N images)
template <typename T>
__global__ void maxpool2_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int NB,
                                    int H, int W, int C) {
  const int Ho = H / 2, Wo = W / 2, CC = C / 8;
  const long long total = (long long)NB * Ho * Wo * CC;
  GSTRIDE_LOOP(t, total) {
    const int cc = (int)(t % CC);
    long long p = t / CC;
    const int wo = (int)(p % Wo);
    p /= Wo;
    const int ho = (int)(p % Ho);
    const int n = (int)(p / Ho);
    const T* b = x + (((long long)n * H + 2 * ho) * W + 2 * wo) * C + cc * 8;
    float m[8], v[8];
    ld8(b, m);
    ld8(b + C, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) m[k] = (v[k] > m[k] || v[k] != v[k]) ? v[k] : m[k];
    ld8(b + (long long)W * C, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) m[k] = (v[k] > m[k] || v[k] != v[k]) ? v[k] : m[k];
    ld8(b + (long long)W * C + C, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) m[k] = (v[k] > m[k] || v[k] != v[k]) ? v[k] : m[k];
    st8(y + t * 8, m);
  }
}

template <typename T>
__global__ void maxpool2_bwd_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                    T* __restrict__ dx, int NB, int H, int W, int C) {
  const int Ho = H / 2, Wo = W / 2, CC = C / 8;
  const long long total = (long long)NB * Ho * Wo * CC;
  GSTRIDE_LOOP(t, total) {
    const int cc = (int)(t % CC);
    long long p = t / CC;
    const int wo = (int)(p % Wo);
    p /= Wo;
    const int ho = (int)(p % Ho);
    const int n = (int)(p / Ho);
    const long long o00 = (((long long)n * H + 2 * ho) * W + 2 * wo) * C + cc * 8;
    const long long offs[4] = {o00, o00 + C, o00 + (long long)W * C, o00 + (long long)W * C + C};
    float v[4][8], d[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) ld8(x + offs[j], v[j]);
    ld8(dy + t * 8, d);
    float out[4][8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      int am = 0;
      float m = v[0][k];
#pragma unroll
      for (int j = 1; j < 4; ++j)
        if (v[j][k] > m || v[j][k] != v[j][k]) { m = v[j][k]; am = j; }
#pragma unroll
      for (int j = 0; j < 4; ++j) out[j][k] = (j == am) ? d[k] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) st8(dx + offs[j], out[j]);
  }
}

template <typename T>
static int maxpool2_fwd_impl(const void* x, void* y, int NB, int H, int W, int C, hipStream_t s) {
  if (C % 8 || H % 2 || W % 2) return (int)hipErrorInvalidValue;
  const long long total = (long long)NB * (H / 2) * (W / 2) * (C / 8);
  hipLaunchKernelGGL(maxpool2_fwd_kernel<T>, dim3(grid_for(total, 256)), dim3(256), 0, s,
                     (const T*)x, (T*)y, NB, H, W, C);
  return (int)hipGetLastError();
}
template <typename T>
static int maxpool2_bwd_impl(const void* x, const void* dy, void* dx, int NB, int H, int W, int C,
                             hipStream_t s) {
  if (C % 8 || H % 2 || W % 2) return (int)hipErrorInvalidValue;
  const long long total = (long long)NB * (H / 2) * (W / 2) * (C / 8);
  hipLaunchKernelGGL(maxpool2_bwd_kernel<T>, dim3(grid_for(total, 256)), dim3(256), 0, s,
                     (const T*)x, (const T*)dy, (T*)dx, NB, H, W, C);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// global average pool: x [NB][HW][C] -> y [NB][C]; one thread per (image, 8-channel chunk)
template <typename T>
__global__ void avgpool_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int NB,
                                   int HW, int C) {
  const int CC = C / 8;
  const long long total = (long long)NB * CC;
  GSTRIDE_LOOP(t, total) {
    const int cc = (int)(t % CC);
    const long long n = t / CC;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int p = 0; p < HW; ++p) {
      float v[8];
      ld8(x + (n * HW + p) * C + cc * 8, v);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += v[k];
    }
    const float inv = 1.f / HW;
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] *= inv;
    st8(y + n * C + cc * 8, acc);
  }
}
template <typename T>
__global__ void avgpool_bwd_kernel(const T* __restrict__ dy, T* __restrict__ dx, int NB,
                                   int HW, int C) {
  const int CC = C / 8;
  const long long total = (long long)NB * HW * CC;
  const float inv = 1.f / HW;
  GSTRIDE_LOOP(t, total) {
    const int cc = (int)(t % CC);
    const long long n = t / CC / HW;
    float v[8];
    ld8(dy + n * C + cc * 8, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] *= inv;
    st8(dx + t * 8, v);
  }
}
// Global-average-pool backward fused with the backward reduce of the BatchNorm that produced the
// pooled input (a ResNet's last block: x = relu(bn(c) + shortcut)): dx = dy / HW masked by
// (x > 0), written once, and per channel s0 = sum dx, s1 = sum dx * (c - mean) * rstd added into
// stripe (blockIdx.x % 32) of part [G][32][2C] — the reduce pass of that BN's backward, which
// then runs fold + apply only (the block's bn_backward(part=...)). Layout as the BN passes: a
// 256-thread block covers RPI = 256 / (C/8) pixel rows, each thread one fixed 8-channel chunk.
__global__ __launch_bounds__(256) void avgpool_bwd_bn_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x, const bf16_t* __restrict__ c,
    const float* __restrict__ mean, const float* __restrict__ rstd, bf16_t* __restrict__ dx,
    float* __restrict__ part, int N, int HW, int C) {
  __shared__ float red[256 * 17];
  const int g = blockIdx.y;
  const int TPR = C / 8, RPI = 256 / TPR;
  const int tid = threadIdx.x, cc = tid % TPR, row = tid / TPR;
  const long long M = (long long)N * HW;
  float s0[8], s1[8], m8[8], r8[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) s0[k] = s1[k] = 0.f;
  const float* mg = mean + (long long)g * C + cc * 8;
  const float* rg = rstd + (long long)g * C + cc * 8;
#pragma unroll
  for (int k = 0; k < 8; ++k) { m8[k] = mg[k]; r8[k] = rg[k]; }
  const float inv = 1.f / HW;
  if (row < RPI) {
    constexpr int U = 4;  // 4 rows' loads in flight per thread
    const long long stride = (long long)gridDim.x * RPI;
    for (long long p0 = (long long)blockIdx.x * RPI + row; p0 < M; p0 += stride * U) {
      i4v rd[U], rx[U], rc[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long p = p0 + u * stride;
        if (p < M) {
          const long long e = ((long long)g * M + p) * C + cc * 8;
          rd[u] = *(const i4v*)(dy + ((long long)g * N + p / HW) * C + cc * 8);
          rx[u] = *(const i4v*)(x + e);
          rc[u] = *(const i4v*)(c + e);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long p = p0 + u * stride;
        if (p >= M) break;
        const long long e = ((long long)g * M + p) * C + cc * 8;
        float d[8], xv[8], cv[8];
        unpack8(rd[u], d);
        unpack8(rx[u], xv);
        unpack8(rc[u], cv);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          d[k] = xv[k] > 0.f ? d[k] * inv : 0.f;
          s0[k] += d[k];
          s1[k] += d[k] * (cv[k] - m8[k]) * r8[k];
        }
        st8(dx + e, d);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    red[tid * 17 + k] = s0[k];
    red[tid * 17 + 8 + k] = s1[k];
  }
  __syncthreads();
  int top = 1;
  while (top < RPI) top <<= 1;
  for (int half = top >> 1; half > 0; half >>= 1) {
    if (row < half && row + half < RPI) {
      const float* o = red + (tid + half * TPR) * 17;
      float* m = red + tid * 17;
#pragma unroll
      for (int k = 0; k < 16; ++k) m[k] += o[k];
    }
    __syncthreads();
  }
  if (row == 0) {
    float* pg = part + ((long long)g * 32 + blockIdx.x % 32) * 2 * C;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      atomicAdd(pg + cc * 8 + k, red[tid * 17 + k]);
      atomicAdd(pg + C + cc * 8 + k, red[tid * 17 + 8 + k]);
    }
  }
}

// dy [G][N][C], x / c / dx [G][N][HW][C] bf16, mean / rstd [G][C], part zeroed [G][32][2C]
DDL_API int ddl_avgpool_bwd_bn(const void* dy, const void* x, const void* c, const float* mean,
                               const float* rstd, void* dx, float* part, int G, int N, int HW, int C,
                               hipStream_t s) {
  if (C % 8 || C / 8 > 256) return (int)hipErrorInvalidValue;
  const int RPI = 256 / (C / 8);
  long long want = ((long long)N * HW + RPI * 4 - 1) / (RPI * 4);
  long long cap = (2048 + G - 1) / G;
  // each block ends with 2C atomics: keep ~512K per launch (batchnorm.hip reduce_blocks)
  long long acap = (512LL * 1024) / (2LL * C * G);
  if (cap > acap) cap = acap < 8 ? 8 : acap;
  if (want > cap) want = cap;
  hipLaunchKernelGGL(avgpool_bwd_bn_kernel, dim3((unsigned)(want < 1 ? 1 : want), G), dim3(256), 0, s,
                     (const bf16_t*)dy, (const bf16_t*)x, (const bf16_t*)c, mean, rstd, (bf16_t*)dx,
                     part, N, HW, C);
  return (int)hipGetLastError();
}

template <typename T>
static int avgpool_fwd_impl(const void* x, void* y, int NB, int HW, int C, hipStream_t s) {
  if (C % 8) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(avgpool_fwd_kernel<T>, dim3(grid_for((long long)NB * C / 8, 256)), dim3(256), 0,
                     s, (const T*)x, (T*)y, NB, HW, C);
  return (int)hipGetLastError();
}
template <typename T>
static int avgpool_bwd_impl(const void* dy, void* dx, int NB, int HW, int C, hipStream_t s) {
  if (C % 8) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(avgpool_bwd_kernel<T>, dim3(grid_for((long long)NB * HW * C / 8, 256)), dim3(256),
                     0, s, (const T*)dy, (T*)dx, NB, HW, C);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// dropout: keep iff philox(seed, element/4)[element%4] >= p ; scale 1/(1-p). Mask recomputed.
// The Philox counter base = offset + *offset_dev (if given): a device-resident per-layer counter
// advanced by ddl_u64_add after each backward, so a captured HIP graph draws a fresh mask on
// every replay while forward and backward of one step share it.
template <typename T>
__global__ void dropout_kernel(const T* __restrict__ x, T* __restrict__ y, long long n,
                               float p, unsigned long long seed, unsigned long long offset,
                               const unsigned long long* __restrict__ offset_dev) {
  if (offset_dev) offset += *offset_dev;
  const float scale = p < 1.f ? 1.f / (1.f - p) : 0.f;
  const uint2 key = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
  GSTRIDE_LOOP(t, n / 8) {
    float v[8];
    ld8(x + t * 8, v);
    const unsigned long long ctr0 = offset + (unsigned long long)t * 2;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const unsigned long long c = ctr0 + h;
      const uint4 r = philox4x32(make_uint4((uint32_t)c, (uint32_t)(c >> 32), 0x5bd1e995u, 0), key);
      const uint32_t rr[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) v[h * 4 + k] = (u32_to_unit(rr[k]) > p) ? v[h * 4 + k] * scale : 0.f;
    }
    st8(y + t * 8, v);
  }
}
template <typename T>
static int dropout_impl(const void* x, void* y, long long n, float p, unsigned long long seed,
                        unsigned long long offset, const unsigned long long* offset_dev,
                        hipStream_t s) {
  if (n % 8) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(dropout_kernel<T>, dim3(grid_for(n / 8, 256)), dim3(256), 0, s, (const T*)x,
                     (T*)y, n, p, seed, offset, offset_dev);
  return (int)hipGetLastError();
}

__global__ void u64_add_kernel(unsigned long long* p, unsigned long long inc) { *p += inc; }
DDL_API int ddl_u64_add(unsigned long long* p, unsigned long long inc, hipStream_t s) {
  hipLaunchKernelGGL(u64_add_kernel, dim3(1), dim3(1), 0, s, p, inc);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// act fwd: 1 relu, 2 leaky(slope), 3 tanh, 4 sigmoid; act bwd: dx = dy * act'(y) computed from the
// forward OUTPUT y (relu/leaky: sign preserved; tanh: 1-y^2; sigmoid: y(1-y))
template <typename T>
__global__ void act_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, long long n,
                               int act, float slope) {
  GSTRIDE_LOOP(t, n / 8) {
    float v[8];
    ld8(x + t * 8, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (act == 3) v[k] = tanhf(v[k]);
      else if (act == 4) v[k] = 1.f / (1.f + __expf(-v[k]));
      else v[k] = v[k] > 0.f ? v[k] : (act == 2 ? slope * v[k] : 0.f);
    }
    st8(y + t * 8, v);
  }
}
template <typename T>
__global__ void act_bwd_kernel(const T* __restrict__ y, const T* __restrict__ dy,
                               T* __restrict__ dx, long long n, int act, float slope) {
  GSTRIDE_LOOP(t, n / 8) {
    float v[8], d[8];
    ld8(y + t * 8, v);
    ld8(dy + t * 8, d);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (act == 3) d[k] *= 1.f - v[k] * v[k];
      else if (act == 4) d[k] *= v[k] * (1.f - v[k]);
      else d[k] = v[k] > 0.f ? d[k] : (act == 2 ? slope * d[k] : 0.f);
    }
    st8(dx + t * 8, d);
  }
}
template <typename T>
static int act_fwd_impl(const void* x, void* y, long long n, int act, float slope, hipStream_t s) {
  if (n % 8) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(act_fwd_kernel<T>, dim3(grid_for(n / 8, 256)), dim3(256), 0, s, (const T*)x,
                     (T*)y, n, act, slope);
  return (int)hipGetLastError();
}
template <typename T>
static int act_bwd_impl(const void* y, const void* dy, void* dx, long long n, int act, float slope,
                        hipStream_t s) {
  if (n % 8) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(act_bwd_kernel<T>, dim3(grid_for(n / 8, 256)), dim3(256), 0, s, (const T*)y,
                     (const T*)dy, (T*)dx, n, act, slope);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// per-channel sum of x [G][M][C] bf16 -> out [G] (+g*gs) fp32 accumulate
template <typename T>
__global__ __launch_bounds__(256) void channel_sum_kernel(const T* __restrict__ x,
                                                          float* __restrict__ out, long long gs,
                                                          long long M, int C) {
  __shared__ float red[256 * 9];
  const int g = blockIdx.y;
  const int TPR = C / 8, RPI = 256 / TPR;
  const int tid = threadIdx.x, cc = tid % TPR, row = tid / TPR;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (row < RPI) {
    for (long long p = (long long)blockIdx.x * RPI + row; p < M; p += (long long)gridDim.x * RPI) {
      float v[8];
      ld8(x + ((long long)g * M + p) * C + cc * 8, v);
#pragma unroll
      for (int k = 0; k < 8; ++k) s[k] += v[k];
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) red[tid * 9 + k] = s[k];
  __syncthreads();
  if (tid < TPR) {
    float t8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int r = 0; r < RPI; ++r)
#pragma unroll
      for (int k = 0; k < 8; ++k) t8[k] += red[(r * TPR + tid) * 9 + k];
#pragma unroll
    for (int k = 0; k < 8; ++k) atomicAdd(out + (long long)g * gs + tid * 8 + k, t8[k]);
  }
}
template <typename T>
static int channel_sum_impl(const void* x, float* out, long long gs, long long M, int C, int G,
                            hipStream_t s) {
  if (C % 8 || C / 8 > 256) return (int)hipErrorInvalidValue;
  const int RPI = 256 / (C / 8);
  long long blocks = (M + (long long)RPI * 16 - 1) / ((long long)RPI * 16);
  if (blocks > 512) blocks = 512;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(channel_sum_kernel<T>, dim3((unsigned)blocks, G), dim3(256), 0, s,
                     (const T*)x, out, gs, M, C);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
__global__ void cast_f32_bf16_kernel(const float* __restrict__ x, bf16_t* __restrict__ y, long long n) {
  GSTRIDE_LOOP(t, (n + 3) / 4) {
    const long long e = t * 4;
    if (e + 4 <= n) {
      const float4 v = *(const float4*)(x + e);
      i2v o;
      o[0] = (int)pack_bf2(v.x, v.y);
      o[1] = (int)pack_bf2(v.z, v.w);
      *(i2v*)(y + e) = o;
    } else {
      for (long long k = e; k < n; ++k) y[k] = f2bf(x[k]);
    }
  }
}
__global__ void cast_bf16_f32_kernel(const bf16_t* __restrict__ x, float* __restrict__ y, long long n) {
  GSTRIDE_LOOP(t, n) y[t] = bf2f(x[t]);
}
DDL_API int ddl_cast_f32_bf16(const float* x, void* y, long long n, hipStream_t s) {
  hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3(grid_for((n + 3) / 4, 256)), dim3(256), 0, s, x,
                     (bf16_t*)y, n);
  return (int)hipGetLastError();
}
DDL_API int ddl_cast_bf16_f32(const void* x, float* y, long long n, hipStream_t s) {
  hipLaunchKernelGGL(cast_bf16_f32_kernel, dim3(grid_for(n, 256)), dim3(256), 0, s, (const bf16_t*)x,
                     y, n);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// general k x k / stride / pad max pool (ImageNet stem 3x3/2 p1); -inf padding like torch
// am (optional): window-local argmax r*k+s per output element (uint8), consumed by the backward
// I: index type (int when every element offset fits in 31 bits: no 64-bit division per item)
template <typename I, typename T>
__global__ void maxpool_fwd_kernel(const T* __restrict__ x, T* __restrict__ y,
                                   unsigned char* __restrict__ am, int NB,
                                   int H, int W, int C, int k, int st, int pd, int Ho, int Wo) {
  const int CC = C / 8;
  const I total = (I)NB * Ho * Wo * CC;
  for (I t = blockIdx.x * (I)blockDim.x + threadIdx.x; t < total; t += (I)gridDim.x * blockDim.x) {
    const int cc = (int)(t % CC);
    I p = t / CC;
    const int wo = (int)(p % Wo);
    p /= Wo;
    const int ho = (int)(p % Ho);
    const int n = (int)(p / Ho);
    float m[8];
    int ai[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { m[e] = -INFINITY; ai[e] = 0; }
    for (int r = 0; r < k; ++r) {
      const int ih = ho * st - pd + r;
      if ((unsigned)ih >= (unsigned)H) continue;
      for (int s2 = 0; s2 < k; ++s2) {
        const int iw = wo * st - pd + s2;
        if ((unsigned)iw >= (unsigned)W) continue;
        float v[8];
        ld8(x + (((I)n * H + ih) * W + iw) * C + cc * 8, v);
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (v[e] > m[e] || (v[e] != v[e] && m[e] == m[e])) { m[e] = v[e]; ai[e] = r * k + s2; }
      }
    }
    st8(y + t * 8, m);
    if (am) {
      unsigned long long packed = 0;
#pragma unroll
      for (int e = 0; e < 8; ++e) packed |= (unsigned long long)(ai[e] & 0xff) << (8 * e);
      *(unsigned long long*)(am + t * 8) = packed;
    }
  }
}

// backward from the saved argmax: each input pixel gathers dy of the (<= ceil(k/st)^2) windows
// that contain it and chose it — one byte + one bf16 per window and channel, no recomputation
template <typename I, typename T>
__global__ void maxpool_bwd_am_kernel(const unsigned char* __restrict__ am,
                                      const T* __restrict__ dy, T* __restrict__ dx,
                                      int NB, int H, int W, int C, int k, int st, int pd, int Ho,
                                      int Wo) {
  const int CC = C / 8;
  const I total = (I)NB * H * W * CC;
  for (I t = blockIdx.x * (I)blockDim.x + threadIdx.x; t < total; t += (I)gridDim.x * blockDim.x) {
    const int cc = (int)(t % CC);
    I p = t / CC;
    const int iw0 = (int)(p % W);
    p /= W;
    const int ih0 = (int)(p % H);
    const int n = (int)(p / H);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const int ho_lo = max(0, (ih0 + pd - k + st) / st), ho_hi = min(Ho - 1, (ih0 + pd) / st);
    const int wo_lo = max(0, (iw0 + pd - k + st) / st), wo_hi = min(Wo - 1, (iw0 + pd) / st);
    for (int ho = ho_lo; ho <= ho_hi; ++ho)
      for (int wo = wo_lo; wo <= wo_hi; ++wo) {
        const int local = (ih0 - (ho * st - pd)) * k + (iw0 - (wo * st - pd));
        const I o = (((I)n * Ho + ho) * Wo + wo) * C + cc * 8;
        const unsigned long long a8 = *(const unsigned long long*)(am + o);
        float d[8];
        ld8(dy + o, d);
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if ((int)((a8 >> (8 * e)) & 0xff) == local) acc[e] += d[e];
      }
    st8(dx + t * 8, acc);
  }
}
// backward as a gather over the windows that contain each input pixel (no atomics): an input
// element receives dy of every window whose (first) argmax it is.
template <typename T>
__global__ void maxpool_bwd_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                   T* __restrict__ dx, int NB, int H, int W, int C, int k,
                                   int st, int pd, int Ho, int Wo) {
  const int CC = C / 8;
  const long long total = (long long)NB * H * W * CC;
  GSTRIDE_LOOP(t, total) {
    const int cc = (int)(t % CC);
    long long p = t / CC;
    const int iw0 = (int)(p % W);
    p /= W;
    const int ih0 = (int)(p % H);
    const int n = (int)(p / H);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const int ho_lo = max(0, (ih0 + pd - k + st) / st), ho_hi = min(Ho - 1, (ih0 + pd) / st);
    const int wo_lo = max(0, (iw0 + pd - k + st) / st), wo_hi = min(Wo - 1, (iw0 + pd) / st);
    for (int ho = ho_lo; ho <= ho_hi; ++ho)
      for (int wo = wo_lo; wo <= wo_hi; ++wo) {
        float m[8];
        int am[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) { m[e] = -INFINITY; am[e] = -1; }
        for (int r = 0; r < k; ++r) {
          const int ih = ho * st - pd + r;
          if ((unsigned)ih >= (unsigned)H) continue;
          for (int s2 = 0; s2 < k; ++s2) {
            const int iw = wo * st - pd + s2;
            if ((unsigned)iw >= (unsigned)W) continue;
            float v[8];
            ld8(x + (((long long)n * H + ih) * W + iw) * C + cc * 8, v);
#pragma unroll
            for (int e = 0; e < 8; ++e)
              if (v[e] > m[e] || (v[e] != v[e] && m[e] == m[e])) { m[e] = v[e]; am[e] = ih * W + iw; }
          }
        }
        float d[8];
        ld8(dy + (((long long)n * Ho + ho) * Wo + wo) * C + cc * 8, d);
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (am[e] == ih0 * W + iw0) acc[e] += d[e];
      }
    st8(dx + t * 8, acc);
  }
}
template <typename T>
static int maxpool_fwd_impl(const void* x, void* y, void* am, int NB, int H, int W, int C, int k,
                            int st, int pd, hipStream_t s) {
  if (C % 8) return (int)hipErrorInvalidValue;
  const int Ho = (H + 2 * pd - k) / st + 1, Wo = (W + 2 * pd - k) / st + 1;
  const long long total = (long long)NB * Ho * Wo * (C / 8);
  if (k > 15) return (int)hipErrorInvalidValue;  // argmax index must fit a byte
  if ((long long)NB * H * W * C < (1LL << 31) - 64)  // 32-bit offsets, one item per thread
    hipLaunchKernelGGL((maxpool_fwd_kernel<int, T>), dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                       (const T*)x, (T*)y, (unsigned char*)am, NB, H, W, C, k, st, pd, Ho, Wo);
  else
    hipLaunchKernelGGL((maxpool_fwd_kernel<long long, T>), dim3(grid_for(total, 256)), dim3(256), 0, s,
                       (const T*)x, (T*)y, (unsigned char*)am, NB, H, W, C, k, st, pd, Ho, Wo);
  return (int)hipGetLastError();
}
template <typename T>
static int maxpool_bwd_impl(const void* x, const void* dy, const void* am, void* dx, int NB, int H,
                            int W, int C, int k, int st, int pd, hipStream_t s) {
  if (C % 8) return (int)hipErrorInvalidValue;
  const int Ho = (H + 2 * pd - k) / st + 1, Wo = (W + 2 * pd - k) / st + 1;
  const long long total = (long long)NB * H * W * (C / 8);
  if (am) {
    if ((long long)NB * H * W * C < (1LL << 31) - 64)
      hipLaunchKernelGGL((maxpool_bwd_am_kernel<int, T>), dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                         (const unsigned char*)am, (const T*)dy, (T*)dx, NB, H, W, C, k, st,
                         pd, Ho, Wo);
    else
      hipLaunchKernelGGL((maxpool_bwd_am_kernel<long long, T>), dim3(grid_for(total, 256)), dim3(256), 0, s,
                         (const unsigned char*)am, (const T*)dy, (T*)dx, NB, H, W, C, k, st,
                         pd, Ho, Wo);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(maxpool_bwd_kernel<T>, dim3(grid_for(total, 256)), dim3(256), 0, s,
                     (const T*)x, (const T*)dy, (T*)dx, NB, H, W, C, k, st, pd, Ho, Wo);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// exports: bf16 activations (ddl_x) and fp32 activations (ddl_x_f32, the reference-precision mode)
#define NN_EXPORT(name, params, args)                                      \
  DDL_API int ddl_##name params { return name##_impl<bf16_t> args; }       \
  DDL_API int ddl_##name##_f32 params { return name##_impl<float> args; }
NN_EXPORT(prep_images, (const void* src, const int* idx, const float* mean, const float* inv_std, void* out,
                        int nimg, int Hs, int Ws, int Cs, int Cout, int im2col, int pad, int stride,
                        const int* labels, int* labels_out, hipStream_t s),
          (src, idx, mean, inv_std, out, nimg, Hs, Ws, Cs, Cout, im2col, pad, stride, labels, labels_out, s))
NN_EXPORT(nchw_to_nhwc, (const float* x, void* out, int N, int Cs, int Hs, int Ws, int Cout, int im2col, int pad,
                         int stride, hipStream_t s),
          (x, out, N, Cs, Hs, Ws, Cout, im2col, pad, stride, s))
NN_EXPORT(maxpool2_fwd, (const void* x, void* y, int NB, int H, int W, int C, hipStream_t s), (x, y, NB, H, W, C, s))
NN_EXPORT(maxpool2_bwd, (const void* x, const void* dy, void* dx, int NB, int H, int W, int C, hipStream_t s),
          (x, dy, dx, NB, H, W, C, s))
NN_EXPORT(avgpool_fwd, (const void* x, void* y, int NB, int HW, int C, hipStream_t s), (x, y, NB, HW, C, s))
NN_EXPORT(avgpool_bwd, (const void* dy, void* dx, int NB, int HW, int C, hipStream_t s), (dy, dx, NB, HW, C, s))
NN_EXPORT(dropout, (const void* x, void* y, long long n, float p, unsigned long long seed, unsigned long long offset,
                    const unsigned long long* offset_dev, hipStream_t s),
          (x, y, n, p, seed, offset, offset_dev, s))
NN_EXPORT(act_fwd, (const void* x, void* y, long long n, int act, float slope, hipStream_t s), (x, y, n, act, slope, s))
NN_EXPORT(act_bwd, (const void* y, const void* dy, void* dx, long long n, int act, float slope, hipStream_t s),
          (y, dy, dx, n, act, slope, s))
NN_EXPORT(channel_sum, (const void* x, float* out, long long gs, long long M, int C, int G, hipStream_t s),
          (x, out, gs, M, C, G, s))
NN_EXPORT(maxpool_fwd, (const void* x, void* y, void* am, int NB, int H, int W, int C, int k, int st, int pd,
                        hipStream_t s),
          (x, y, am, NB, H, W, C, k, st, pd, s))
NN_EXPORT(maxpool_bwd, (const void* x, const void* dy, const void* am, void* dx, int NB, int H, int W, int C, int k,
                        int st, int pd, hipStream_t s),
          (x, dy, am, dx, NB, H, W, C, k, st, pd, s))

// ---------------------------------------------------------------------------------------------
// Federated-DCGAN round inputs generated on the device (fl/gan.py): for slot g (a client of the
// round, desc[g] = {seed, n, off}) and local step i, the batch indices
//   idx[i][g*B + b] = off + floor(u32 * n / 2^32),  u32 = Philox(seed, i*B + b, tag A).x
// and the generator noise z[i][g][b][k] ~ N(0, 1) by Box-Muller on Philox(seed, (i*B+b)*nz + k, tag B).
// Both are pure functions of the client's (round, client) seed, so a client's batches and noise do
// not depend on its slot or on how many ranks share the clients; ops/reference.gan_inputs is the
// numpy twin (the CPU engines).
__global__ __launch_bounds__(256) void gan_inputs_kernel(const long long* __restrict__ desc, int G, int steps, int B,
                                                         int nz, long long* __restrict__ idx, float* __restrict__ z) {
  const long long ni = (long long)steps * G * B, nzt = ni * nz;
  for (long long t = blockIdx.x * 256LL + threadIdx.x; t < ni + nzt; t += (long long)gridDim.x * 256) {
    if (t < ni) {  // idx [steps][G*B]
      const int i = (int)(t / ((long long)G * B));
      const int gb = (int)(t - (long long)i * G * B), g = gb / B, b = gb - g * B;
      const unsigned long long seed = (unsigned long long)desc[3 * g];
      const unsigned long long e = (unsigned long long)i * B + b;
      const uint4 r = philox4x32(make_uint4((uint32_t)e, (uint32_t)(e >> 32), 0x1d872b41u, 0u),
                                 make_uint2((uint32_t)seed, (uint32_t)(seed >> 32)));
      idx[t] = desc[3 * g + 2] + (long long)(((unsigned long long)r.x * (unsigned long long)desc[3 * g + 1]) >> 32);
    } else {  // z [steps][G][B][nz]
      const long long u = t - ni;
      const long long row = u / nz;
      const int k = (int)(u - row * nz);
      const int i = (int)(row / ((long long)G * B));
      const int gb = (int)(row - (long long)i * G * B), g = gb / B, b = gb - g * B;
      const unsigned long long seed = (unsigned long long)desc[3 * g];
      const unsigned long long e = ((unsigned long long)i * B + b) * nz + k;
      const uint4 r = philox4x32(make_uint4((uint32_t)e, (uint32_t)(e >> 32), 0x6a09e667u, 0u),
                                 make_uint2((uint32_t)seed, (uint32_t)(seed >> 32)));
      const float u1 = fmaxf(u32_to_unit(r.x), 1e-12f), u2 = u32_to_unit(r.y);
      z[u] = sqrtf(-2.f * logf(u1)) * cosf(6.28318530717958648f * u2);
    }
  }
}

DDL_API int ddl_gan_inputs(const long long* desc, int G, int steps, int B, int nz, long long* idx, float* z,
                           hipStream_t s) {
  if (G < 1 || steps < 1 || B < 1 || nz < 1) return (int)hipErrorInvalidValue;
  const long long work = (long long)steps * G * B * (nz + 1);
  hipLaunchKernelGGL(gan_inputs_kernel, dim3(grid_for(work, 256)), dim3(256), 0, s, desc, G, steps, B, nz, idx, z);
  return (int)hipGetLastError();
}
