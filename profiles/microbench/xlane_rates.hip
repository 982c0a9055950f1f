// Micro-benchmark: cross-lane primitives used by reductions, on one MI355X.
// Cycles per wave-instruction per SIMD at 8 waves/SIMD (8192 blocks of 64).
#include <hip/hip_runtime.h>
#include <stdio.h>

#define N 2048
template <int MODE>
__global__ __launch_bounds__(64) void k(float* out, float seed) {
  float v[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) v[i] = seed + threadIdx.x + i;
  for (int it = 0; it < N; ++it) {
    if (MODE == 0) {  // permlane32_swap + add, 5 independent pairs
#pragma unroll
      for (int i = 0; i < 10; i += 2) {
        const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[i]), __float_as_uint(v[i + 1]), false, false);
        v[i] = __uint_as_float(r[0]) + 1.0001f;
        v[i + 1] = __uint_as_float(r[1]) + 1.0001f;
      }
    }
    if (MODE == 1) {  // permlane16_swap + add
#pragma unroll
      for (int i = 0; i < 10; i += 2) {
        const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[i]), __float_as_uint(v[i + 1]), false, false);
        v[i] = __uint_as_float(r[0]) + 1.0001f;
        v[i + 1] = __uint_as_float(r[1]) + 1.0001f;
      }
    }
    if (MODE == 2) {  // ds_swizzle-free: __shfl_xor (ds_bpermute) + add
#pragma unroll
      for (int i = 0; i < 10; ++i) v[i] += __shfl_xor(v[i], 16, 64);
    }
    if (MODE == 3) {  // DPP row_shr:1 add
#pragma unroll
      for (int i = 0; i < 10; ++i)
        v[i] += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v[i]), 0x111, 0xf, 0xf, true));
    }
    if (MODE == 4) {  // DPP row_ror:8 add (no bound_ctrl)
#pragma unroll
      for (int i = 0; i < 10; ++i)
        v[i] += __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v[i]), __float_as_int(v[i]), 0x128, 0xf, 0xf, false));
    }
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 10; ++i) s += v[i];
  out[blockIdx.x * 64 + threadIdx.x] = s;
}

template <int MODE>
void run(const char* name, int blocks, float* d, int instr_per_iter) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  k<MODE><<<blocks, 64>>>(d, 1.f);
  (void)hipEventRecord(a);
  k<MODE><<<blocks, 64>>>(d, 1.f);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  const double ops = (double)blocks * N * instr_per_iter;
  printf("%-36s blocks %6d  %.3f ms  %.2f SIMD-cycles per op\n", name, blocks, ms, ms * 1e-3 * 2.4e9 * 1024 / ops);
}

int main() {
  float* d;
  (void)hipMalloc(&d, 64 * 65536 * sizeof(float));
  for (int blocks : {2048, 8192}) {
    run<0>("permlane32_swap (+2 adds)", blocks, d, 5);
    run<1>("permlane16_swap (+2 adds)", blocks, d, 5);
    run<2>("shfl_xor 16 (bpermute) + add", blocks, d, 10);
    run<3>("dpp row_shr:1 + add", blocks, d, 10);
    run<4>("dpp row_ror:8 + add", blocks, d, 10);
  }
  return 0;
}
