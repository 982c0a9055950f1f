// Micro-benchmark: issue throughput of the VALU forms the blend kernels use, on one MI355X.
// Each kernel runs N iterations of 10 independent chains (like the backward's 10 gradient terms);
// cycles per instruction per SIMD = elapsed cycles * SIMDs / (waves * instructions).
// Build: hipcc --offload-arch=gfx950 -O3 valu_rates.hip -o valu_rates ; run on the GPU box.
#include <hip/hip_runtime.h>
#include <stdio.h>

#define N 4096
template <int MODE>
__global__ __launch_bounds__(64) void k(float* out, float seed) {
  float v[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) v[i] = seed + threadIdx.x + i;
  for (int it = 0; it < N; ++it) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      if (MODE == 0) v[i] = v[i] + 1.0001f;  // v_add_f32
      if (MODE == 1)                           // v_add_f32_dpp row_shr:1
        v[i] += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v[i]), 0x111, 0xf, 0xf, true));
      if (MODE == 2) v[i] = __expf(v[i]) * 0.5f;  // v_exp_f32 + mul
      if (MODE == 3) v[i] = __builtin_amdgcn_rcpf(v[i]) + 1.0f;
      if (MODE == 4) v[i] = fmaf(v[i], 1.0001f, 0.5f);  // v_fma_f32
    }
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 10; ++i) s += v[i];
  out[blockIdx.x * 64 + threadIdx.x] = s;
}

template <int MODE>
void run(const char* name, int blocks, float* d) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  k<MODE><<<blocks, 64>>>(d, 1.f);
  hipEventRecord(a);
  k<MODE><<<blocks, 64>>>(d, 1.f);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  const double instr = (double)blocks * N * 10;  // wave-instructions of the measured form
  const double simd_cycles = ms * 1e-3 * 2.4e9 * 1024;
  printf("%-28s blocks %6d  %.3f ms  %.2f SIMD-cycles per wave-instruction\n", name, blocks, ms, simd_cycles / instr);
}

int main() {
  float* d;
  hipMalloc(&d, 64 * 65536 * sizeof(float));
  for (int blocks : {1024, 4096, 8192}) {
    run<0>("v_add_f32", blocks, d);
    run<4>("v_fma_f32", blocks, d);
    run<1>("v_add_f32 + dpp row_shr", blocks, d);
    run<2>("v_exp_f32 + v_mul", blocks, d);
    run<3>("v_rcp_f32 + v_add", blocks, d);
  }
  return 0;
}
