// Probe: do 16-byte LDS reads at 2-byte-misaligned addresses work on gfx950, and what do they cost
// against aligned ones? (A halo-staged WGRAD would read pixel windows shifted by one bf16 element.)
// Build + run: hipcc --offload-arch=gfx950 -O2 scripts/lds_unaligned.hip -o /tmp/lds_unaligned && /tmp/lds_unaligned
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef short s8v __attribute__((ext_vector_type(8)));
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <int MIS>
__global__ void probe(int* out, long long* cyc, int iters) {
  __shared__ __attribute__((aligned(16))) unsigned short lds[64 * 16 + 64];
  const int lane = threadIdx.x;
  for (int i = lane; i < 64 * 16 + 64; i += 64) lds[i] = (unsigned short)i;
  __syncthreads();
  // correctness: lane reads 8 elements starting at element 8 * lane + MIS
  const char* base = (const char*)lds + 2 * (8 * lane + MIS);
  s8v v = *(const s8v*)base;
  int ok = 1;
  for (int j = 0; j < 8; ++j) ok &= (unsigned short)v[j] == (unsigned short)(8 * lane + MIS + j);
  out[lane] = ok;
  // cost: dependent-address chain of reads
  int acc = 0;
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
    const char* p = (const char*)lds + 2 * ((8 * lane + MIS + (acc & 1)) % 1000);
    s8v w = *(const s8v*)p;
    acc += w[0] + w[7];
  }
  const long long t1 = clock64();
  if (lane == 0) cyc[0] = t1 - t0;
  out[64 + lane] = acc;
}

int main() {
  int* d;
  long long* c;
  CK(hipMalloc(&d, 128 * 4));
  CK(hipMalloc(&c, 8));
  int h[128];
  long long cyc;
  for (int mis = 0; mis < 2; ++mis) {
    if (mis == 0) probe<0><<<1, 64>>>(d, c, 4096);
    else probe<1><<<1, 64>>>(d, c, 4096);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h, d, 128 * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&cyc, c, 8, hipMemcpyDeviceToHost));
    int ok = 1;
    for (int i = 0; i < 64; ++i) ok &= h[i];
    printf("misaligned by %d bf16: values %s, %.1f cycles per dependent ds_read_b128\n", mis, ok ? "correct" : "WRONG",
           (double)cyc / 4096);
  }
  return 0;
}
