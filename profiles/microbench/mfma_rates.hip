// Micro-benchmark: issue cost of the matrix-core forms the backward blend can use for its per-candidate
// sums (v_mfma_f32_16x16x4_f32 now; v_mfma_f64_16x16x4_f64 for exact sums), on one MI355X.
// 4 independent accumulator chains per wave; cycles per MFMA per SIMD = elapsed cycles x SIMDs / MFMAs.
// Build: hipcc --offload-arch=gfx950 -O3 mfma_rates.hip -o mfma_rates ; run on the GPU box.
#include <hip/hip_runtime.h>
#include <stdio.h>

#define N 2048
typedef float f4 __attribute__((ext_vector_type(4)));
typedef double d4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(64) void k(float* out, float seed) {
  const float a = seed + threadIdx.x, b = seed * 0.5f + threadIdx.x;
  if (MODE == 0) {
    f4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    for (int it = 0; it < N; ++it) {
      c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c3, 0, 0, 0);
    }
    out[blockIdx.x * 64 + threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
  } else {
    const double ad = a, bd = b;
    d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    for (int it = 0; it < N; ++it) {
      c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(ad, bd, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(ad, bd, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(ad, bd, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(ad, bd, c3, 0, 0, 0);
    }
    out[blockIdx.x * 64 + threadIdx.x] = (float)(c0[0] + c1[1] + c2[2] + c3[3]);
  }
}

template <int MODE>
void run(const char* name, int blocks, float* d) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  k<MODE><<<blocks, 64>>>(d, 1.f);
  hipEventRecord(e0);
  k<MODE><<<blocks, 64>>>(d, 1.f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double mfma = (double)blocks * N * 4;
  const double simd_cycles = ms * 1e-3 * 2.4e9 * 1024;
  printf("%-26s blocks %6d  %.3f ms  %.2f SIMD-cycles per MFMA\n", name, blocks, ms, simd_cycles / mfma);
}

int main() {
  float* d;
  hipMalloc(&d, 64 * 65536 * sizeof(float));
  for (int blocks : {1024, 4096}) {
    run<0>("v_mfma_f32_16x16x4_f32", blocks, d);
    run<1>("v_mfma_f64_16x16x4_f64", blocks, d);
  }
  return 0;
}
