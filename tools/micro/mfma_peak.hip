// Practical fp32 MFMA ceiling: every wave issues back-to-back v_mfma_f32_32x32x2_f32 on 4
// independent accumulators.  usage: ./mfma_peak  → TFLOP/s for 1..4 waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float floatx16 __attribute__((ext_vector_type(16)));

__global__ __launch_bounds__(256) void mfma_loop(float* out, int iters, float a0) {
  floatx16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  float a = a0 + threadIdx.x * 1e-7f, b = 1.0f - threadIdx.x * 1e-7f;
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(b, a, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, a, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_32x32x2f32(b, b, c3, 0, 0, 0);
  }
  float s = 0.f;
  for (int e = 0; e < 16; ++e) s += c0[e] + c1[e] + c2[e] + c3[e];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  float* out;
  (void)hipMalloc(&out, sizeof(float) * 256 * cus * 8);
  const int iters = 20000;
  for (int wps = 1; wps <= 4; ++wps) {  // waves per SIMD = workgroups of 4 waves per CU
    const int blocks = cus * wps;
    hipEvent_t s, e;
    (void)hipEventCreate(&s);
    (void)hipEventCreate(&e);
    mfma_loop<<<blocks, 256>>>(out, 100, 1.f);
    (void)hipEventRecord(s);
    mfma_loop<<<blocks, 256>>>(out, iters, 1.f);
    (void)hipEventRecord(e);
    (void)hipEventSynchronize(e);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, s, e);
    const double flops = (double)blocks * 4 /*waves*/ * iters * 4 /*mfma*/ * 32 * 32 * 2 * 2;
    printf("waves/SIMD %d: %.2f ms  %.1f TFLOP/s  (implied clock %.3f GHz at 256 FLOP/clk/CU)\n", wps,
           ms, flops / ms / 1e9, flops / (ms * 1e-3) / (256.0 * cus) / 1e9);
  }
  return 0;
}
