// Fused classification / reconstruction losses (forward value + gradient in one pass).
//
//   ddl_ce_fwd_bwd     : softmax cross-entropy with hard labels (== log_softmax + nll_loss of
//                        reference hfl_complete.py:62,78) or probability targets (the float
//                        one-hot CrossEntropyLoss of reference lab/tutorial_2b/vfl.py:51,79).
//                        One wave per row; loss accumulated per client group; optional correct-
//                        prediction counter (argmax == label) for accuracy (hfl_complete.py:180-181).
//   ddl_ce_vocab       : same op for wide rows (LM head, vocab ~32k): one 256-thread block per row,
//                        online max/sum-exp, bf16 logits in, bf16 grads out.
//   ddl_mse_kl         : MSE(sum) + KL(N(mu,sigma) || N(0,1)) with gradients (customLoss of
//                        reference lab/tutorial_2a/generative-modeling.py:121-130).
#include "ddl_common.h"

// logits [R][ld] bf16 with R = G*N rows; labels int32 [R] (hard) or targets fp32 [R][ncls] (soft)
// loss[g] += scale * sum_rows_of_g loss_row ; dlogits = scale * (softmax*sum(t) - t) (0 for pad cols)
template <typename T>
__global__ __launch_bounds__(256) void ce_kernel(const T* __restrict__ logits,
                                                 const int* __restrict__ labels,
                                                 const float* __restrict__ targets, int R, int N,
                                                 int ncls, int ld, float scale,
                                                 float* __restrict__ loss, T* __restrict__ dlogits,
                                                 int* __restrict__ correct) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;
  const T* z = logits + (long long)row * ld;
  float mx = -INFINITY;
  int amax = 0;
  for (int c = lane; c < ncls; c += 64) {
    const float v = ld1(z + c);
    if (v > mx) { mx = v; amax = c; }
  }
  // wave argmax (first max wins on ties, like torch.argmax)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(mx, o, 64);
    const int oa = __shfl_xor(amax, o, 64);
    if (om > mx || (om == mx && oa < amax)) { mx = om; amax = oa; }
  }
  float se = 0.f;
  for (int c = lane; c < ncls; c += 64) se += __expf(ld1(z + c) - mx);
  se = wave_sum(se);
  const float lse = mx + __logf(se);
  float lrow = 0.f, tsum = 1.f;
  if (targets) {
    const float* t = targets + (long long)row * ncls;
    float ts = 0.f, l = 0.f;
    for (int c = lane; c < ncls; c += 64) {
      ts += t[c];
      l += t[c] * (lse - ld1(z + c));
    }
    tsum = wave_sum(ts);
    lrow = wave_sum(l);
  } else {
    const int y = labels[row];
    lrow = lse - ld1(z + y);
  }
  if (dlogits) {
    T* dz = dlogits + (long long)row * ld;
    for (int c = lane; c < ld; c += 64) {
      float gv = 0.f;
      if (c < ncls) {
        const float p = __expf(ld1(z + c) - lse);
        const float tc = targets ? targets[(long long)row * ncls + c] : (c == labels[row] ? 1.f : 0.f);
        gv = scale * (p * tsum - tc);
      }
      st1(dz + c, gv);
    }
  }
  if (lane == 0) {
    const int g = row / N;
    if (loss) atomicAdd(loss + g, lrow * scale);
    if (correct) {
      int y;
      if (targets) {  // argmax of the target row
        const float* t = targets + (long long)row * ncls;
        y = 0;
        for (int c = 1; c < ncls; ++c) if (t[c] > t[y]) y = c;
      } else {
        y = labels[row];
      }
      if (amax == y) atomicAdd(correct + g, 1);
    }
  }
}

template <typename T>
static int ce_fwd_bwd_impl(const void* logits, const int* labels, const float* targets, int R, int N, int ncls,
                           int ld, float scale, float* loss, void* dlogits, int* correct, hipStream_t s) {
  if (ncls > ld || N <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(ce_kernel<T>, dim3((R + 3) / 4), dim3(256), 0, s, (const T*)logits, labels,
                     targets, R, N, ncls, ld, scale, loss, (T*)dlogits, correct);
  return (int)hipGetLastError();
}
DDL_API int ddl_ce_fwd_bwd(const void* logits, const int* labels, const float* targets, int R, int N,
                           int ncls, int ld, float scale, float* loss, void* dlogits, int* correct,
                           hipStream_t s) {
  return ce_fwd_bwd_impl<bf16_t>(logits, labels, targets, R, N, ncls, ld, scale, loss, dlogits, correct, s);
}
// fp32 logits / gradients (the reference-precision mode)
DDL_API int ddl_ce_fwd_bwd_f32(const void* logits, const int* labels, const float* targets, int R, int N,
                               int ncls, int ld, float scale, float* loss, void* dlogits, int* correct,
                               hipStream_t s) {
  return ce_fwd_bwd_impl<float>(logits, labels, targets, R, N, ncls, ld, scale, loss, dlogits, correct, s);
}

// ---------------------------------------------------------------------------------------------
// wide-row CE (LM head): block per row, vectorised 8-wide, online softmax
__global__ __launch_bounds__(256) void ce_vocab_kernel(const bf16_t* __restrict__ logits,
                                                       const int* __restrict__ labels, int V, int ld,
                                                       float scale, int ignore_index,
                                                       float* __restrict__ loss,
                                                       bf16_t* __restrict__ dlogits) {
  __shared__ float sm[2][4];
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const bf16_t* z = logits + (long long)row * ld;
  float m = -INFINITY, se = 0.f;
  for (int c = tid * 8; c < V; c += 256 * 8) {
    float v[8];
    unpack8(*(const i4v*)(z + c), v);
    float lm = v[0];
#pragma unroll
    for (int k = 1; k < 8; ++k) lm = fmaxf(lm, v[k]);
    const float nm = fmaxf(m, lm);
    se = se * __expf(m - nm);
#pragma unroll
    for (int k = 0; k < 8; ++k) se += __expf(v[k] - nm);
    m = nm;
  }
  // combine (m, se) across the block
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(m, o, 64), os = __shfl_xor(se, o, 64);
    const float nm = fmaxf(m, om);
    se = (m == -INFINITY ? 0.f : se * __expf(m - nm)) + (om == -INFINITY ? 0.f : os * __expf(om - nm));
    m = nm;
  }
  if (lane == 0) { sm[0][w] = m; sm[1][w] = se; }
  __syncthreads();
  float M = sm[0][0];
  for (int i = 1; i < 4; ++i) M = fmaxf(M, sm[0][i]);
  float SE = 0.f;
  for (int i = 0; i < 4; ++i) SE += sm[1][i] * __expf(sm[0][i] - M);
  const float lse = M + __logf(SE);
  const int y = labels[row];
  const bool ign = (y == ignore_index);
  if (tid == 0 && loss && !ign) atomicAdd(loss, (lse - bf2f(z[y])) * scale);
  if (dlogits) {
    bf16_t* dz = dlogits + (long long)row * ld;
    for (int c = tid * 8; c < V; c += 256 * 8) {
      float v[8];
      unpack8(*(const i4v*)(z + c), v);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float p = __expf(v[k] - lse);
        v[k] = ign ? 0.f : scale * (p - ((c + k) == y ? 1.f : 0.f));
      }
      *(i4v*)(dz + c) = pack8(v);
    }
  }
}

DDL_API int ddl_ce_vocab(const void* logits, const int* labels, int R, int V, int ld, float scale,
                         int ignore_index, float* loss, void* dlogits, hipStream_t s) {
  if (V % 8 || ld % 8) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(ce_vocab_kernel, dim3(R), dim3(256), 0, s, (const bf16_t*)logits, labels, V,
                     ld, scale, ignore_index, loss, (bf16_t*)dlogits);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// LM-head CE for autograd in ONE read of the logits: the forward writes the loss AND the
// gradient at unit upstream scale, d = (*inv) * (softmax(z) - onehot(y)) (0 for ignored rows);
// the backward only rescales it by the upstream gradient, in place, and only when that is not 1
// (ce_vocab_scale_kernel reads it on the device: no host sync). Against lse-in-forward +
// gradient-in-backward this reads the [rows, V] logits once instead of twice. The normaliser
// stays a device scalar (*inv).
// The row stays in registers between the two sweeps (16 chunks of 8 bf16 per thread: V <= 32768)
// so the logits are read from HBM once; a row is 64 KB at V = 32000 and the rows of the blocks in
// flight on an XCD overflow its L2, so a second load would go to HBM again.
constexpr int CE_RC = 16;
__global__ __launch_bounds__(256) void ce_vocab_fused_kernel(const bf16_t* __restrict__ logits,
                                                             const int* __restrict__ labels, int V,
                                                             int ld, const float* __restrict__ inv,
                                                             int ignore_index, float* __restrict__ loss,
                                                             bf16_t* __restrict__ dlogits) {
  __shared__ float sm[2][4];
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const bf16_t* z = logits + (long long)row * ld;
  const int y = labels[row];
  const float sc = *inv;
  i4v raw[CE_RC];
#pragma unroll
  for (int i = 0; i < CE_RC; ++i) {
    const int c = (i * 256 + tid) * 8;
    if (c < V) raw[i] = *(const i4v*)(z + c);
  }
  float m = -INFINITY, se = 0.f;
#pragma unroll
  for (int i = 0; i < CE_RC; ++i) {
    const int c = (i * 256 + tid) * 8;
    if (c < V) {
      float v[8];
      unpack8(raw[i], v);
      float lm = v[0];
#pragma unroll
      for (int k = 1; k < 8; ++k) lm = fmaxf(lm, v[k]);
      const float nm = fmaxf(m, lm);
      se = se * __expf(m - nm);
#pragma unroll
      for (int k = 0; k < 8; ++k) se += __expf(v[k] - nm);
      m = nm;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(m, o, 64), os = __shfl_xor(se, o, 64);
    const float nm = fmaxf(m, om);
    se = (m == -INFINITY ? 0.f : se * __expf(m - nm)) + (om == -INFINITY ? 0.f : os * __expf(om - nm));
    m = nm;
  }
  if (lane == 0) { sm[0][w] = m; sm[1][w] = se; }
  __syncthreads();
  float M = sm[0][0];
  for (int i = 1; i < 4; ++i) M = fmaxf(M, sm[0][i]);
  float SE = 0.f;
  for (int i = 0; i < 4; ++i) SE += sm[1][i] * __expf(sm[0][i] - M);
  const float lse = M + __logf(SE);
  const bool ign = (y == ignore_index);
  if (tid == 0 && !ign) atomicAdd(loss, (lse - bf2f(z[y])) * sc);
  bf16_t* dz = dlogits + (long long)row * ld;
#pragma unroll
  for (int i = 0; i < CE_RC; ++i) {
    const int c = (i * 256 + tid) * 8;
    if (c < V) {
      float v[8];
      unpack8(raw[i], v);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = ign ? 0.f : sc * (__expf(v[k] - lse) - ((c + k) == y ? 1.f : 0.f));
      *(i4v*)(dz + c) = pack8(v);
    }
  }
}

// x *= *g in place, unless *g == 1 (every block reads it first and returns: the common
// loss.backward() case costs one near-empty launch)
__global__ void ce_vocab_scale_kernel(bf16_t* __restrict__ x, long long n8, const float* __restrict__ g) {
  const float s = *g;
  if (s == 1.f) return;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n8;
       i += (long long)gridDim.x * blockDim.x) {
    float v[8];
    unpack8(*(const i4v*)(x + i * 8), v);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] *= s;
    *(i4v*)(x + i * 8) = pack8(v);
  }
}

DDL_API int ddl_ce_vocab_fused(const void* logits, const int* labels, int R, int V, int ld,
                               const float* inv, int ignore_index, float* loss, void* dlogits,
                               hipStream_t s) {
  if (V % 8 || ld % 8 || V > CE_RC * 256 * 8) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(ce_vocab_fused_kernel, dim3(R), dim3(256), 0, s, (const bf16_t*)logits, labels, V,
                     ld, inv, ignore_index, loss, (bf16_t*)dlogits);
  return (int)hipGetLastError();
}

DDL_API int ddl_ce_vocab_scale(void* x, long long n, const float* g, hipStream_t s) {
  if (n % 8) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(ce_vocab_scale_kernel, dim3(grid_for(n / 8, 256, 2048)), dim3(256), 0, s,
                     (bf16_t*)x, n / 8, g);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Split LM-head CE for autograd without host syncs or extra passes over the [rows, V] logits:
//   fwd : lse[row] and loss += (lse - z_y) * (*inv)          (inv = 1 / #non-ignored rows, device)
//   bwd : dz = (*g) * (*inv) * (softmax(z) - onehot(y))      (g = upstream grad, device scalar)
// so the mean normaliser and the upstream scale (e.g. 1/micro-batches) never leave the device, and
// the gradient is produced in backward, in one read of z and one write of dz.
__global__ __launch_bounds__(256) void ce_vocab_lse_kernel(const bf16_t* __restrict__ logits,
                                                           const int* __restrict__ labels, int V,
                                                           int ld, const float* __restrict__ inv,
                                                           int ignore_index, float* __restrict__ loss,
                                                           float* __restrict__ lse_out) {
  __shared__ float sm[2][4];
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const bf16_t* z = logits + (long long)row * ld;
  float m = -INFINITY, se = 0.f;
  for (int c = tid * 8; c < V; c += 256 * 8) {
    float v[8];
    unpack8(*(const i4v*)(z + c), v);
    float lm = v[0];
#pragma unroll
    for (int k = 1; k < 8; ++k) lm = fmaxf(lm, v[k]);
    const float nm = fmaxf(m, lm);
    se = se * __expf(m - nm);
#pragma unroll
    for (int k = 0; k < 8; ++k) se += __expf(v[k] - nm);
    m = nm;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(m, o, 64), os = __shfl_xor(se, o, 64);
    const float nm = fmaxf(m, om);
    se = (m == -INFINITY ? 0.f : se * __expf(m - nm)) + (om == -INFINITY ? 0.f : os * __expf(om - nm));
    m = nm;
  }
  if (lane == 0) { sm[0][w] = m; sm[1][w] = se; }
  __syncthreads();
  if (tid != 0) return;
  float M = sm[0][0];
  for (int i = 1; i < 4; ++i) M = fmaxf(M, sm[0][i]);
  float SE = 0.f;
  for (int i = 0; i < 4; ++i) SE += sm[1][i] * __expf(sm[0][i] - M);
  const float lse = M + __logf(SE);
  lse_out[row] = lse;
  const int y = labels[row];
  if (y != ignore_index) atomicAdd(loss, (lse - bf2f(z[y])) * (*inv));
}

__global__ __launch_bounds__(256) void ce_vocab_grad_kernel(const bf16_t* __restrict__ logits,
                                                            const int* __restrict__ labels, int V,
                                                            int ld, const float* __restrict__ lse,
                                                            const float* __restrict__ inv,
                                                            const float* __restrict__ g,
                                                            int ignore_index,
                                                            bf16_t* __restrict__ dlogits) {
  const int row = blockIdx.x;
  const int y = labels[row];
  const bool ign = y == ignore_index;
  const float sc = (*g) * (*inv), L = lse[row];
  const bf16_t* z = logits + (long long)row * ld;
  bf16_t* dz = dlogits + (long long)row * ld;
  for (int c = threadIdx.x * 8; c < V; c += 256 * 8) {
    float v[8];
    unpack8(*(const i4v*)(z + c), v);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = ign ? 0.f : sc * (__expf(v[k] - L) - ((c + k) == y ? 1.f : 0.f));
    *(i4v*)(dz + c) = pack8(v);
  }
}

DDL_API int ddl_ce_vocab_lse(const void* logits, const int* labels, int R, int V, int ld,
                             const float* inv, int ignore_index, float* loss, float* lse,
                             hipStream_t s) {
  if (V % 8 || ld % 8) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(ce_vocab_lse_kernel, dim3(R), dim3(256), 0, s, (const bf16_t*)logits, labels, V,
                     ld, inv, ignore_index, loss, lse);
  return (int)hipGetLastError();
}

DDL_API int ddl_ce_vocab_grad(const void* logits, const int* labels, int R, int V, int ld,
                              const float* lse, const float* inv, const float* g, int ignore_index,
                              void* dlogits, hipStream_t s) {
  if (V % 8 || ld % 8) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(ce_vocab_grad_kernel, dim3(R), dim3(256), 0, s, (const bf16_t*)logits, labels,
                     V, ld, lse, inv, g, ignore_index, (bf16_t*)dlogits);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// loss += sum (xr - x)^2 + kl_w * -0.5*sum(1 + lv - mu^2 - exp(lv));  fp32 tensors
// grads: dxr = 2(xr - x)*gs ; dmu = kl_w*mu*gs ; dlv = kl_w*0.5*(exp(lv) - 1)*gs
__global__ void mse_kl_kernel(const float* __restrict__ xr, const float* __restrict__ x, long long n,
                              const float* __restrict__ mu, const float* __restrict__ lv,
                              long long nz, float kl_w, float gs, float* __restrict__ loss,
                              float* __restrict__ dxr, float* __restrict__ dmu,
                              float* __restrict__ dlv) {
  float acc = 0.f;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n + nz;
       i += (long long)gridDim.x * blockDim.x) {
    if (i < n) {
      const float d = xr[i] - x[i];
      acc += d * d;
      if (dxr) dxr[i] = 2.f * d * gs;
    } else {
      const long long j = i - n;
      const float m = mu[j], l = lv[j], e = __expf(l);
      acc += kl_w * -0.5f * (1.f + l - m * m - e);
      if (dmu) dmu[j] = kl_w * m * gs;
      if (dlv) dlv[j] = kl_w * 0.5f * (e - 1.f) * gs;
    }
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) atomicAdd(loss, acc);
}

DDL_API int ddl_mse_kl(const float* xr, const float* x, long long n, const float* mu,
                       const float* lv, long long nz, float kl_w, float gs, float* loss,
                       float* dxr, float* dmu, float* dlv, hipStream_t s) {
  long long tot = n + nz;
  long long b = (tot + 255) / 256;
  if (b > 1024) b = 1024;
  if (b < 1) b = 1;
  hipLaunchKernelGGL(mse_kl_kernel, dim3((unsigned)b), dim3(256), 0, s, xr, x, n, mu, lv, nz, kl_w,
                     gs, loss, dxr, dmu, dlv);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Binary cross-entropy on logits (nn.BCEWithLogitsLoss / BCELoss∘sigmoid of the DCGAN
// discriminator). logits bf16 [R] with row stride ld (column 0 of a padded linear output);
// target = targets[r] if given else tval. loss += sum_r bce ; dlogits[r*ld] = (sigmoid(l)-t)*gs.
__global__ void bce_logits_kernel(const bf16_t* __restrict__ logits, int ld, const float* __restrict__ targets,
                                  float tval, int R, float gs, float* __restrict__ loss,
                                  bf16_t* __restrict__ dlogits) {
  float acc = 0.f;
  for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < R; r += gridDim.x * blockDim.x) {
    const float l = bf2f(logits[(long long)r * ld]);
    const float t = targets ? targets[r] : tval;
    acc += fmaxf(l, 0.f) - l * t + log1pf(__expf(-fabsf(l)));
    if (dlogits) dlogits[(long long)r * ld] = f2bf((1.f / (1.f + __expf(-l)) - t) * gs);
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) atomicAdd(loss, acc);
}

DDL_API int ddl_bce_logits(const void* logits, int ld, const float* targets, float tval, int R,
                           float gs, float* loss, void* dlogits, hipStream_t s) {
  int b = (R + 255) / 256;
  if (b > 256) b = 256;
  if (b < 1) b = 1;
  hipLaunchKernelGGL(bce_logits_kernel, dim3(b), dim3(256), 0, s, (const bf16_t*)logits, ld, targets,
                     tval, R, gs, loss, (bf16_t*)dlogits);
  return (int)hipGetLastError();
}

// fp32 logits (the reference-precision DCGAN): one workgroup, the per-thread partial sums meet in a
// fixed-order LDS tree, so the loss is bitwise reproducible (no float atomics); R = clients x batch
// rows is small. The loss is written, not accumulated.
__global__ __launch_bounds__(256) void bce_logits_f32_kernel(const float* __restrict__ logits, int ld,
                                                             const float* __restrict__ targets, float tval, int R,
                                                             float gs, float* __restrict__ loss,
                                                             float* __restrict__ dlogits) {
  __shared__ float red[256];
  float acc = 0.f;
  for (int r = threadIdx.x; r < R; r += 256) {
    const float l = logits[(long long)r * ld];
    const float t = targets ? targets[r] : tval;
    acc += fmaxf(l, 0.f) - l * t + log1pf(expf(-fabsf(l)));
    if (dlogits) {
      float* d = dlogits + (long long)r * ld;
      d[0] = (1.f / (1.f + expf(-l)) - t) * gs;
      for (int j = 1; j < ld; ++j) d[j] = 0.f;  // the padded columns: the caller needs no memset
    }
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) *loss = red[0];
}

DDL_API int ddl_bce_logits_f32(const float* logits, int ld, const float* targets, float tval, int R, float gs,
                               float* loss, float* dlogits, hipStream_t s) {
  if (R < 1 || ld < 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(bce_logits_f32_kernel, dim3(1), dim3(256), 0, s, logits, ld, targets, tval, R, gs, loss, dlogits);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Fused classifier head of a training step: global average pool -> Linear (+bias) -> softmax CE
// with hard labels -> the Linear's weight / bias gradients -> the pool's input gradient, masked by
// the pooled input's ReLU and reduced for the BatchNorm that produced it. The unfused chain is
// seven launches (avgpool, FC FWD, CE, bias sum, FC WGRAD, FC DGRAD, pool backward), four of them
// single-digit-workgroup grids whose dependent latency is most of their cost at one client per GPU
// (profiles/step_trace_r2_1client.txt: ~70 us per step). Here it is two:
//   head_train_kernel : a workgroup owns S samples of one client group; the class rows of W are
//                       staged in LDS once; logits, softmax and the pooled vectors stay fp32 in LDS;
//                       it writes the pooled means and d logits to scratch for
//   head_wgrad_kernel : dW = dlogits^T . pooled and db, one workgroup per (64 channels, <= 32
//                       samples, group), so each gradient element takes a handful of atomics —
//                       the single-launch form (every sample block adding its dW) put ~100 atomics
//                       on every address and took 68 us at one client.
struct HeadArgs {
  const bf16_t* x;     // [G][N][HW][C]: the pooled input
  const bf16_t* w;     // group g at g * w_gs: [Kp][C] bf16 (the Linear's shadow weight)
  const float* b;      // group g at g * b_gs: [Kp] fp32 (null: no bias)
  const int* labels;   // [G][N]
  float* loss;         // [G]  += scale * sum of the rows' CE
  int* correct;        // [G]  += (argmax == label) (null: off)
  float* dw;           // group g at g * dw_gs: [Kp][C] fp32, accumulated
  float* db;           // group g at g * db_gs: [Kp] fp32, accumulated (null: no bias)
  bf16_t* dx;          // [G][N][HW][C]
  const bf16_t* c;     // BN fusion (null: plain pool backward): the BN's input [G][N][HW][C]
  const float* mean;   // [G][C]
  const float* rstd;   // [G][C]
  float* part;         // [G][32][2][C] zeroed: (sum dx, sum dx * (c - mean) * rstd)
  float* pooled;       // scratch [G][N][C] fp32: pooled means
  float* dlog;         // scratch [G][N][64] fp32: d logits
  long long w_gs, b_gs, dw_gs, db_gs;
  int G, N, HW, C, ncls, S;
  float scale;
};

// One sample per workgroup; a thread owns one 8-channel chunk (cc) and every RP-th pixel (row).
// With CACHE, the thread's (<= 4) pixels of x and of the BN input are loaded once, at the start,
// together with everything else the block reads (W rows, bias, label, BN mean / rstd), so the
// block's dependent chain has one load round trip; without it (large HW) they are re-read.
template <bool CACHE>
__global__ __launch_bounds__(256) void head_train_kernel(HeadArgs a) {
  extern __shared__ float hsm[];
  const int C = a.C, CC = C / 8, RP = 256 / CC, HW = a.HW, g = blockIdx.y, n = blockIdx.x;
  float* pooled = hsm;         // [C] pooled mean
  float* dp = pooled + C;      // [C] d pooled / HW
  float* zl = dp + C;          // [64] logits, then d logits
  float* rb = zl + 64;         // [RP][C] row partials (RP * C = 2048)
  bf16_t* wl = (bf16_t*)(rb + 2048);  // [ncls][C] the class rows of W
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, cc = tid % CC, row = tid / CC;
  const float inv = 1.f / HW;
  const long long rowg = (long long)g * a.N + n;
  const bf16_t* wg = a.w + g * a.w_gs;
  const bool bn = a.c != nullptr;
  const long long base = rowg * HW * C + cc * 8;
  // all independent loads first
  for (int t = tid; t < a.ncls * CC; t += 256)
    *(i4v*)(wl + t * 8) = *(const i4v*)(wg + t * 8);
  i4v xr[CACHE ? 4 : 1], cr[CACHE ? 4 : 1];
  if constexpr (CACHE) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int p = row + i * RP;
      if (p < HW) {
        xr[i] = *(const i4v*)(a.x + base + (long long)p * C);
        if (bn) cr[i] = *(const i4v*)(a.c + base + (long long)p * C);
      }
    }
  }
  const int y = a.labels[rowg];
  const float bias = (a.b && lane < a.ncls) ? a.b[g * a.b_gs + lane] : 0.f;
  float m8[8], r8[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    m8[k] = bn ? a.mean[(long long)g * C + cc * 8 + k] : 0.f;
    r8[k] = bn ? a.rstd[(long long)g * C + cc * 8 + k] : 0.f;
  }
  // 1. pool: registers over the thread's pixels, then the RP row partials
  {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if constexpr (CACHE) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (row + i * RP < HW) {
          float v[8];
          unpack8(xr[i], v);
#pragma unroll
          for (int k = 0; k < 8; ++k) acc[k] += v[k];
        }
      }
    } else {
      for (int p = row; p < HW; p += RP) {
        float v[8];
        unpack8(*(const i4v*)(a.x + base + (long long)p * C), v);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += v[k];
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) rb[row * C + cc * 8 + k] = acc[k];
  }
  __syncthreads();
  for (int t = tid; t < C; t += 256) {
    float v = 0.f;
    for (int r = 0; r < RP; ++r) v += rb[r * C + t];
    pooled[t] = v * inv;
  }
  __syncthreads();
  // 2. logits: one wave per class, lanes over channels
  for (int k = wv; k < a.ncls; k += 4) {
    float acc = 0.f;
    for (int c8 = lane; c8 < CC; c8 += 64) {
      float w8[8];
      unpack8(*(const i4v*)(wl + k * C + c8 * 8), w8);
      const float* pp = pooled + c8 * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += pp[j] * w8[j];
    }
    acc = wave_sum(acc);
    if (lane == 0) zl[k] = acc;
  }
  __syncthreads();
  // 3. softmax CE on wave 0, one lane per class
  if (wv == 0) {
    const bool on = lane < a.ncls;
    const float z = on ? zl[lane] + bias : -INFINITY;
    float mx = z;
    int am = on ? lane : 0x7fffffff;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {  // argmax, first max wins (torch.argmax)
      const float om = __shfl_xor(mx, o, 64);
      const int oa = __shfl_xor(am, o, 64);
      if (om > mx || (om == mx && oa < am)) { mx = om; am = oa; }
    }
    const float e = on ? __expf(z - mx) : 0.f;
    const float lse = mx + __logf(wave_sum(e));
    const float zy = __shfl(z, y, 64);
    const float d = on ? a.scale * (__expf(z - lse) - (lane == y ? 1.f : 0.f)) : 0.f;
    zl[lane] = d;
    a.dlog[rowg * 64 + lane] = d;
    if (lane == 0) {
      atomicAdd(a.loss + g, (lse - zy) * a.scale);
      if (a.correct && am == y) atomicAdd(a.correct + g, 1);
    }
  }
  for (int t = tid; t < C; t += 256) a.pooled[rowg * C + t] = pooled[t];
  __syncthreads();
  // 4. d pooled = dl . W (/ HW for the pool backward)
  for (int c8 = tid; c8 < CC; c8 += 256) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < a.ncls; ++k) {
      const float d = zl[k];
      float w8[8];
      unpack8(*(const i4v*)(wl + k * C + c8 * 8), w8);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += d * w8[j];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) dp[c8 * 8 + j] = acc[j] * inv;
  }
  __syncthreads();
  // 5. pool backward (+ the BN's ReLU mask and backward reduce)
  float d0[8], s0[8], s1[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    d0[k] = dp[cc * 8 + k];
    s0[k] = s1[k] = 0.f;
  }
  auto one = [&](long long e, const i4v& xv4, const i4v& cv4) {
    float d[8];
    if (bn) {
      float xv[8], cv[8];
      unpack8(xv4, xv);
      unpack8(cv4, cv);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        d[k] = xv[k] > 0.f ? d0[k] : 0.f;
        const float dr = bf2f(f2bf(d[k]));  // the sums see the stored (bf16) gradient
        s0[k] += dr;
        s1[k] += dr * (cv[k] - m8[k]) * r8[k];
      }
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) d[k] = d0[k];
    }
    *(i4v*)(a.dx + e) = pack8(d);
  };
  if constexpr (CACHE) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int p = row + i * RP;
      if (p < HW) one(base + (long long)p * C, xr[i], cr[i]);
    }
  } else {
    for (int p = row; p < HW; p += RP) {
      const long long e = base + (long long)p * C;
      const i4v zero4 = {0, 0, 0, 0};
      one(e, bn ? *(const i4v*)(a.x + e) : zero4, bn ? *(const i4v*)(a.c + e) : zero4);
    }
  }
  if (!bn) return;
  float* pg = a.part + ((long long)g * 32 + n % 32) * 2 * C;
  for (int h = 0; h < 2; ++h) {  // fold the RP row partials of s0, then of s1
#pragma unroll
    for (int k = 0; k < 8; ++k) rb[row * C + cc * 8 + k] = h ? s1[k] : s0[k];
    __syncthreads();
    for (int t = tid; t < C; t += 256) {
      float v = 0.f;
      for (int r = 0; r < RP; ++r) v += rb[r * C + t];
      atomicAdd(pg + h * C + t, v);
    }
    __syncthreads();
  }
}

// dW[k][c] += sum_n dl[n][k] * pooled[n][c] ; db[k] += sum_n dl[n][k]: grid (C/64, N/32, G); a
// thread owns one channel and the classes k = kg, kg + 4, ... (kg = its wave); its <= 32 pooled
// values are loaded up front.
constexpr int HEAD_WG_ROWS = 32;
__global__ __launch_bounds__(256) void head_wgrad_kernel(HeadArgs a) {
  __shared__ float dls[HEAD_WG_ROWS * 64];
  const int g = blockIdx.z, tid = threadIdx.x, kg = tid >> 6;
  const int c = blockIdx.x * 64 + (tid & 63);
  const int n0 = blockIdx.y * HEAD_WG_ROWS;
  const int nr = a.N - n0 < HEAD_WG_ROWS ? a.N - n0 : HEAD_WG_ROWS;
  const long long row0 = (long long)g * a.N + n0;
  float pv[HEAD_WG_ROWS];
  const float* pc = a.pooled + row0 * a.C + (c < a.C ? c : 0);
#pragma unroll
  for (int i = 0; i < HEAD_WG_ROWS; ++i) pv[i] = i < nr ? pc[(long long)i * a.C] : 0.f;
  for (int t = tid; t < HEAD_WG_ROWS * 64; t += 256) dls[t] = t < nr * 64 ? a.dlog[row0 * 64 + t] : 0.f;
  __syncthreads();
  if (blockIdx.x == 0 && a.db && tid < a.ncls) {
    float s = 0.f;
    for (int i = 0; i < nr; ++i) s += dls[i * 64 + tid];
    atomicAdd(a.db + g * a.db_gs + tid, s);
  }
  if (c >= a.C) return;
  float* dwg = a.dw + g * a.dw_gs + c;
  for (int k = kg; k < a.ncls; k += 4) {
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < HEAD_WG_ROWS; ++i) acc += dls[i * 64 + k] * pv[i];
    atomicAdd(dwg + (long long)k * a.C, acc);
  }
}

static int head_lds_bytes(int C, int ncls) { return (2 * C + 64 + 2048) * 4 + ncls * C * 2; }

DDL_API int ddl_head_args_size() { return (int)sizeof(HeadArgs); }

DDL_API int ddl_head_train(const HeadArgs* ap, hipStream_t s) {
  HeadArgs a = *ap;
  if (a.C % 8 || 256 % (a.C / 8) || a.ncls < 1 || a.ncls > 64 || a.N < 1 || a.G < 1 || a.HW < 1 ||
      a.ncls * a.C * 2 > 32 * 1024 || !a.pooled || !a.dlog)
    return (int)hipErrorInvalidValue;
  a.S = 1;
  const int rp = 256 / (a.C / 8);
  if (a.HW <= 4 * rp)
    hipLaunchKernelGGL(head_train_kernel<true>, dim3(a.N, a.G), dim3(256), head_lds_bytes(a.C, a.ncls), s, a);
  else
    hipLaunchKernelGGL(head_train_kernel<false>, dim3(a.N, a.G), dim3(256), head_lds_bytes(a.C, a.ncls), s, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(head_wgrad_kernel, dim3((a.C + 63) / 64, (a.N + HEAD_WG_ROWS - 1) / HEAD_WG_ROWS, a.G),
                     dim3(256), 0, s, a);
  return (int)hipGetLastError();
}
