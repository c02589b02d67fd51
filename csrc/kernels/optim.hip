// Fused multi-tensor optimizers over flat fp32 parameter buffers ([G][P], all clients at once).
// Every update also refreshes the bf16 weight shadow that the MFMA kernels read, so there is no
// separate cast pass per step. Semantics follow torch.optim.SGD / Adam / AdamW exactly
// (momentum buffer initialised to the first gradient, bias-corrected Adam, decoupled AdamW decay)
// which is what the reference uses (hfl_complete.py:196,319 SGD; intro.py:22 Adam 8e-4;
// vfl.py:50 AdamW; generative-modeling.py:154 Adam).
#include "ddl_common.h"

struct SGDArgs {
  float* p; const float* g; float* mom; bf16_t* shadow;
  long long n;
  float lr, wd, momentum, dampening, grad_scale;
  int nesterov, first_step;
};

__global__ void sgd_kernel(SGDArgs a) {
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t * 4 < a.n;
       t += (long long)gridDim.x * blockDim.x) {
    const long long e = t * 4;
    const int cnt = (int)min(4LL, a.n - e);
    float p[4], g[4], m[4] = {0, 0, 0, 0};
    if (cnt == 4) {
      const float4 pv = *(const float4*)(a.p + e), gv = *(const float4*)(a.g + e);
      p[0] = pv.x; p[1] = pv.y; p[2] = pv.z; p[3] = pv.w;
      g[0] = gv.x; g[1] = gv.y; g[2] = gv.z; g[3] = gv.w;
      if (a.mom && !a.first_step) {
        const float4 mv = *(const float4*)(a.mom + e);
        m[0] = mv.x; m[1] = mv.y; m[2] = mv.z; m[3] = mv.w;
      }
    } else {
      for (int k = 0; k < cnt; ++k) {
        p[k] = a.p[e + k]; g[k] = a.g[e + k];
        if (a.mom && !a.first_step) m[k] = a.mom[e + k];
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float d = g[k] * a.grad_scale + a.wd * p[k];
      if (a.momentum != 0.f) {
        m[k] = a.first_step ? d : a.momentum * m[k] + (1.f - a.dampening) * d;
        d = a.nesterov ? d + a.momentum * m[k] : m[k];
      }
      p[k] -= a.lr * d;
    }
    if (cnt == 4) {
      *(float4*)(a.p + e) = make_float4(p[0], p[1], p[2], p[3]);
      if (a.mom && a.momentum != 0.f) *(float4*)(a.mom + e) = make_float4(m[0], m[1], m[2], m[3]);
      if (a.shadow) {
        i2v o;
        o[0] = (int)pack_bf2(p[0], p[1]);
        o[1] = (int)pack_bf2(p[2], p[3]);
        *(i2v*)(a.shadow + e) = o;
      }
    } else {
      for (int k = 0; k < cnt; ++k) {
        a.p[e + k] = p[k];
        if (a.mom && a.momentum != 0.f) a.mom[e + k] = m[k];
        if (a.shadow) a.shadow[e + k] = f2bf(p[k]);
      }
    }
  }
}

DDL_API int ddl_sgd(const SGDArgs* a, hipStream_t s) {
  hipLaunchKernelGGL(sgd_kernel, dim3(grid_for((a->n + 3) / 4, 256)), dim3(256), 0, s, *a);
  return (int)hipGetLastError();
}

struct AdamArgs {
  float* p; const float* g; float* m; float* v; bf16_t* shadow;
  long long n;
  float lr, beta1, beta2, eps, wd, grad_scale;
  float bc1, bc2;  // 1 - beta^t
  int decoupled, amsgrad_unused;
  // optional device step counter (advanced by ddl_u64_add before the launch): the bias corrections
  // are then computed on the device, so a captured HIP graph stays exact on every replay
  const unsigned long long* step_dev;
  // > 0: the buffers are rows of row_len elements (client slots of a client-batched model), each
  // with its OWN device step counter step_dev[row] (clients that joined different numbers of
  // rounds keep their own bias correction)
  long long row_len;
};

__global__ void adam_kernel(AdamArgs a) {
  float bc1 = a.bc1, bc2 = a.bc2;
  if (a.step_dev && a.row_len <= 0) {
    const float t = (float)*a.step_dev;
    bc1 = 1.f - powf(a.beta1, t);
    bc2 = 1.f - powf(a.beta2, t);
  }
  float sbc2 = sqrtf(bc2);
  float step = a.lr / bc1;
  long long row = -1;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < a.n;
       e += (long long)gridDim.x * blockDim.x) {
    if (a.row_len > 0 && e / a.row_len != row) {
      row = e / a.row_len;
      const float t = (float)a.step_dev[row];
      sbc2 = sqrtf(1.f - powf(a.beta2, t));
      step = a.lr / (1.f - powf(a.beta1, t));
    }
    float p = a.p[e];
    float g = a.g[e] * a.grad_scale;
    if (a.decoupled) p *= (1.f - a.lr * a.wd);
    else g += a.wd * p;
    const float m = a.beta1 * a.m[e] + (1.f - a.beta1) * g;
    const float v = a.beta2 * a.v[e] + (1.f - a.beta2) * g * g;
    a.m[e] = m;
    a.v[e] = v;
    p -= step * m / (sqrtf(v) / sbc2 + a.eps);
    a.p[e] = p;
    if (a.shadow) a.shadow[e] = f2bf(p);
  }
}

DDL_API int ddl_adam(const AdamArgs* a, hipStream_t s) {
  if (a->row_len > 0 && !a->step_dev) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(adam_kernel, dim3(grid_for(a->n, 256)), dim3(256), 0, s, *a);
  return (int)hipGetLastError();
}

// Plain SGD (no momentum / weight decay) over rows [rows][P] whose direct-eligible columns were
// already updated inside the backward (conv WGRAD atomics of -lr * dW straight into the master
// weights, ConvArgs::gscale): those columns only refresh the bf16 shadow (6 B/param instead of the
// 14 B of sgd_kernel, and no zero-fill of their gradients). dmap[col / 16] marks them (parameters
// start and pad to 16-element boundaries). The other columns (BatchNorm, classifier head, biases)
// take the ordinary step and have their gradient zeroed for the next step in the same pass.
struct SGDDirectArgs {
  float* p; float* g; bf16_t* shadow; const unsigned char* dmap;
  long long rows, P;
  float lr, grad_scale;
};

__global__ __launch_bounds__(256) void sgd_direct_kernel(SGDDirectArgs a) {
  const long long n4 = a.rows * a.P / 4;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < n4;
       t += (long long)gridDim.x * blockDim.x) {
    const long long e = t * 4;
    const long long col = e % a.P;
    const bool direct = a.dmap[col >> 4] != 0;
    if (direct && !a.shadow) continue;  // fp32 mode: the WGRAD already stepped them, no shadow
    float4 pv = *(const float4*)(a.p + e);
    if (!direct) {
      const float4 gv = *(const float4*)(a.g + e);
      const float s = a.lr * a.grad_scale;
      pv.x -= s * gv.x; pv.y -= s * gv.y; pv.z -= s * gv.z; pv.w -= s * gv.w;
      *(float4*)(a.p + e) = pv;
      *(float4*)(a.g + e) = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (!a.shadow) continue;
    i2v o;
    o[0] = (int)pack_bf2(pv.x, pv.y);
    o[1] = (int)pack_bf2(pv.z, pv.w);
    *(i2v*)(a.shadow + e) = o;
  }
}

DDL_API int ddl_sgd_direct(const SGDDirectArgs* a, hipStream_t s) {
  if (a->P % 16) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(sgd_direct_kernel, dim3(grid_for(a->rows * a->P / 4, 256)), dim3(256), 0, s, *a);
  return (int)hipGetLastError();
}

DDL_API int ddl_sgd_direct_args_size() { return (int)sizeof(SGDDirectArgs); }
DDL_API int ddl_sgd_args_size() { return (int)sizeof(SGDArgs); }
DDL_API int ddl_adam_args_size() { return (int)sizeof(AdamArgs); }
