// Characterise the rounding of gfx950 MFMA fp32 accumulation (why long MFMA accumulator chains bias
// fp32-exact sums): for random bf16 operands, compare v_mfma_f32_16x16x32_bf16 (and the fp32
// v_mfma_f32_16x16x4_f32) against a float64 host reference and report the mean SIGNED error in
// units of the result's ulp (0 = unbiased, like IEEE round-to-nearest; about -0.5 = truncation).
//   (a) C = 0: the 32 products' own summation
//   (b) C = big: the accumulator add (|C| >> the products' sum)
//   (c) a chain of 64 dependent MFMAs vs 64 zero-start MFMAs summed with IEEE fp32 adds
// Build + run:  hipcc --offload-arch=gfx950 -O2 scripts/mfma_rounding.hip -o /tmp/mfma_rounding && /tmp/mfma_rounding
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef short s8v __attribute__((ext_vector_type(8)));
typedef float f4v __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int NCH = 64;  // chain length

// A: [NCH][16 rows][32 k] bf16, B: [NCH][32 k][16 cols] bf16 (stored as [col][k]), C0: [16][16]
// out_chain[16][16] = C0 + sum_c A_c B_c as one dependent chain; out_sep[c][16][16] = 0-start per c
__global__ void mfma_bf16(const unsigned short* A, const unsigned short* B, const float* C0, float* out_chain,
                          float* out_sep) {
  const int lane = threadIdx.x;
  f4v acc;
  for (int v = 0; v < 4; ++v) acc[v] = C0[(4 * (lane >> 4) + v) * 16 + (lane & 15)];
  for (int c = 0; c < NCH; ++c) {
    s8v a, b;
    // 16x16x32: lane l holds row (l & 15), k = 8*(l >> 4) + j
    for (int j = 0; j < 8; ++j) {
      a[j] = (short)A[(c * 16 + (lane & 15)) * 32 + 8 * (lane >> 4) + j];
      b[j] = (short)B[(c * 16 + (lane & 15)) * 32 + 8 * (lane >> 4) + j];
    }
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
    f4v z = {0.f, 0.f, 0.f, 0.f};
    f4v s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, z, 0, 0, 0);
    for (int v = 0; v < 4; ++v) out_sep[(c * 16 + 4 * (lane >> 4) + v) * 16 + (lane & 15)] = s[v];
  }
  for (int v = 0; v < 4; ++v) out_chain[(4 * (lane >> 4) + v) * 16 + (lane & 15)] = acc[v];
}

// fp32 MFMA 16x16x4: lane l holds row (l & 15), k = l >> 4
__global__ void mfma_f32(const float* A, const float* B, const float* C0, float* out_chain, float* out_sep) {
  const int lane = threadIdx.x;
  f4v acc;
  for (int v = 0; v < 4; ++v) acc[v] = C0[(4 * (lane >> 4) + v) * 16 + (lane & 15)];
  for (int c = 0; c < NCH; ++c) {
    const float a = A[(c * 16 + (lane & 15)) * 4 + (lane >> 4)];
    const float b = B[(c * 16 + (lane & 15)) * 4 + (lane >> 4)];
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
    f4v z = {0.f, 0.f, 0.f, 0.f};
    f4v s = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, z, 0, 0, 0);
    for (int v = 0; v < 4; ++v) out_sep[(c * 16 + 4 * (lane >> 4) + v) * 16 + (lane & 15)] = s[v];
  }
  for (int v = 0; v < 4; ++v) out_chain[(4 * (lane >> 4) + v) * 16 + (lane & 15)] = acc[v];
}

static unsigned short to_bf16(float f) {  // round to nearest even
  unsigned u;
  memcpy(&u, &f, 4);
  u += 0x7fff + ((u >> 16) & 1);
  return (unsigned short)(u >> 16);
}
static float bf2f(unsigned short h) {
  unsigned u = (unsigned)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}
static double ulp_err(float got, double ref) {
  if (ref == 0.0) return 0.0;
  int e;
  frexp(ref, &e);
  const double ulp = ldexp(1.0, e - 24);
  return ((double)got - ref) / ulp;
}

int main() {
  srand(7);
  auto rnd = [] { return (float)rand() / RAND_MAX * 2.f - 1.f; };
  const int trials = 200;
  double bias_a = 0, bias_b = 0, bias_chain = 0, bias_sepsum = 0, fa = 0, fb = 0, fchain = 0, fsep = 0;
  long na = 0, nb = 0, nc = 0;
  std::vector<unsigned short> A(NCH * 16 * 32), B(NCH * 16 * 32);
  std::vector<float> Af(NCH * 16 * 4), Bf(NCH * 16 * 4), C0(256), chain(256), sep(NCH * 256);
  unsigned short *dA, *dB;
  float *dAf, *dBf, *dC, *dchain, *dsep;
  CK(hipMalloc(&dA, A.size() * 2)); CK(hipMalloc(&dB, B.size() * 2));
  CK(hipMalloc(&dAf, Af.size() * 4)); CK(hipMalloc(&dBf, Bf.size() * 4));
  CK(hipMalloc(&dC, 1024)); CK(hipMalloc(&dchain, 1024)); CK(hipMalloc(&dsep, sep.size() * 4));
  for (int t = 0; t < trials; ++t) {
    const bool bigC = (t & 1);
    for (auto& x : A) x = to_bf16(rnd());
    for (auto& x : B) x = to_bf16(rnd());
    for (auto& x : Af) x = rnd();
    for (auto& x : Bf) x = rnd();
    for (auto& x : C0) x = bigC ? rnd() * 4096.f : 0.f;
    CK(hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, B.data(), B.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dC, C0.data(), 1024, hipMemcpyHostToDevice));
    mfma_bf16<<<1, 64>>>(dA, dB, dC, dchain, dsep);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(chain.data(), dchain, 1024, hipMemcpyDeviceToHost));
    CK(hipMemcpy(sep.data(), dsep, sep.size() * 4, hipMemcpyDeviceToHost));
    for (int r = 0; r < 16; ++r)
      for (int q = 0; q < 16; ++q) {
        double tot = C0[r * 16 + q];
        float sepsum = C0[r * 16 + q];
        for (int c = 0; c < NCH; ++c) {
          double d = 0;
          for (int k = 0; k < 32; ++k)
            d += (double)bf2f(A[(c * 16 + r) * 32 + k]) * bf2f(B[(c * 16 + q) * 32 + k]);
          if (c == 0 && !bigC) { bias_a += ulp_err(sep[(c * 16 + r) * 16 + q], d); ++na; }
          if (c == 0 && bigC) {  // one MFMA with a big accumulator
          }
          tot += d;
          sepsum = sepsum + sep[(c * 16 + r) * 16 + q];
        }
        if (bigC) { bias_b += ulp_err(chain[r * 16 + q], tot); ++nb; }
        else {
          bias_chain += ulp_err(chain[r * 16 + q], tot);
          bias_sepsum += ulp_err(sepsum, tot);
          ++nc;
        }
      }
    // fp32 MFMA
    CK(hipMemcpy(dAf, Af.data(), Af.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dBf, Bf.data(), Bf.size() * 4, hipMemcpyHostToDevice));
    mfma_f32<<<1, 64>>>(dAf, dBf, dC, dchain, dsep);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(chain.data(), dchain, 1024, hipMemcpyDeviceToHost));
    CK(hipMemcpy(sep.data(), dsep, sep.size() * 4, hipMemcpyDeviceToHost));
    for (int r = 0; r < 16; ++r)
      for (int q = 0; q < 16; ++q) {
        double tot = C0[r * 16 + q];
        float sepsum = C0[r * 16 + q];
        for (int c = 0; c < NCH; ++c) {
          double d = 0;
          for (int k = 0; k < 4; ++k) d += (double)Af[(c * 16 + r) * 4 + k] * Bf[(c * 16 + q) * 4 + k];
          if (c == 0 && !bigC) fa += ulp_err(sep[(c * 16 + r) * 16 + q], d);
          tot += d;
          sepsum = sepsum + sep[(c * 16 + r) * 16 + q];
        }
        if (bigC) fb += ulp_err(chain[r * 16 + q], tot);
        else { fchain += ulp_err(chain[r * 16 + q], tot); fsep += ulp_err(sepsum, tot); }
      }
  }
  printf("bf16 16x16x32: mean signed error (ulp of result)\n");
  printf("  (a) one MFMA, C=0              : %+.3f\n", bias_a / na);
  printf("  (b) %d-chain, |C| >> products  : %+.3f\n", NCH, bias_b / nb);
  printf("  (c) %d-chain, C=0              : %+.3f\n", NCH, bias_chain / nc);
  printf("      %d zero-start + IEEE adds  : %+.3f\n", NCH, bias_sepsum / nc);
  printf("fp32 16x16x4:\n");
  printf("  (a) one MFMA, C=0              : %+.3f\n", fa / na);
  printf("  (b) %d-chain, |C| >> products  : %+.3f\n", NCH, fb / nb);
  printf("  (c) %d-chain, C=0              : %+.3f\n", NCH, fchain / nc);
  printf("      %d zero-start + IEEE adds  : %+.3f\n", NCH, fsep / nc);
  return 0;
}
