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
__global__ __launch_bounds__(256) void ce_kernel(const bf16_t* __restrict__ logits,
                                                 const int* __restrict__ labels,
                                                 const float* __restrict__ targets, int R, int N,
                                                 int ncls, int ld, float scale,
                                                 float* __restrict__ loss, bf16_t* __restrict__ dlogits,
                                                 int* __restrict__ correct) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;
  const bf16_t* z = logits + (long long)row * ld;
  float mx = -INFINITY;
  int amax = 0;
  for (int c = lane; c < ncls; c += 64) {
    const float v = bf2f(z[c]);
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
  for (int c = lane; c < ncls; c += 64) se += __expf(bf2f(z[c]) - mx);
  se = wave_sum(se);
  const float lse = mx + __logf(se);
  float lrow = 0.f, tsum = 1.f;
  if (targets) {
    const float* t = targets + (long long)row * ncls;
    float ts = 0.f, l = 0.f;
    for (int c = lane; c < ncls; c += 64) {
      ts += t[c];
      l += t[c] * (lse - bf2f(z[c]));
    }
    tsum = wave_sum(ts);
    lrow = wave_sum(l);
  } else {
    const int y = labels[row];
    lrow = lse - bf2f(z[y]);
  }
  if (dlogits) {
    bf16_t* dz = dlogits + (long long)row * ld;
    for (int c = lane; c < ld; c += 64) {
      float gv = 0.f;
      if (c < ncls) {
        const float p = __expf(bf2f(z[c]) - lse);
        const float tc = targets ? targets[(long long)row * ncls + c] : (c == labels[row] ? 1.f : 0.f);
        gv = scale * (p * tsum - tc);
      }
      dz[c] = f2bf(gv);
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

DDL_API int ddl_ce_fwd_bwd(const void* logits, const int* labels, const float* targets, int R, int N,
                           int ncls, int ld, float scale, float* loss, void* dlogits, int* correct,
                           hipStream_t s) {
  if (ncls > ld || N <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(ce_kernel, dim3((R + 3) / 4), dim3(256), 0, s, (const bf16_t*)logits, labels,
                     targets, R, N, ncls, ld, scale, loss, (bf16_t*)dlogits, correct);
  return (int)hipGetLastError();
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
