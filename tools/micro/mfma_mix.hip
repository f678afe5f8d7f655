// fp32 MFMA rate vs instruction mix: number of independent accumulators per wave, and
// independent VALU work (v_pk_fma_f32) between the MFMAs.  usage: ./mfma_mix
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx2 __attribute__((ext_vector_type(2)));

template <int NACC, int NVALU>
__global__ __launch_bounds__(256, 2) void mix(float* out, int iters, float a0) {
  floatx16 c[NACC];
  for (int k = 0; k < NACC; ++k) c[k] = floatx16{};
  floatx2 v[8];
  for (int k = 0; k < 8; ++k) v[k] = floatx2{a0 + k, a0 - k};
  const floatx2 m = {1.0001f, 0.9999f};
  float a = a0 + threadIdx.x * 1e-7f, b = 1.0f - threadIdx.x * 1e-7f;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int r = 0; r < 8 / NACC + (NACC > 8); ++r)
#pragma unroll
      for (int k = 0; k < NACC; ++k) {
        c[k] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c[k], 0, 0, 0);
#pragma unroll
        for (int q = 0; q < NVALU; ++q) v[q & 7] = v[q & 7] * m + v[(q + 3) & 7];
      }
  }
  float s = 0.f;
  for (int k = 0; k < NACC; ++k)
    for (int e = 0; e < 16; ++e) s += c[k][e];
  for (int k = 0; k < 8; ++k) s += v[k][0] + v[k][1];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NACC, int NVALU>
void run(float* out, int cus) {
  const int iters = 4000, blocks = cus * 2;
  hipEvent_t s, e;
  (void)hipEventCreate(&s);
  (void)hipEventCreate(&e);
  mix<NACC, NVALU><<<blocks, 256>>>(out, 10, 1.f);
  (void)hipEventRecord(s);
  mix<NACC, NVALU><<<blocks, 256>>>(out, iters, 1.f);
  (void)hipEventRecord(e);
  (void)hipEventSynchronize(e);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, s, e);
  const int per_iter = (8 / NACC + (NACC > 8)) * NACC;
  const double flops = (double)blocks * 4 * iters * per_iter * 32 * 32 * 2 * 2;
  printf("2 waves/SIMD, %d accumulators, %d pk_fma per MFMA: %.1f TFLOP/s\n", NACC, NVALU, flops / ms / 1e9);
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  float* out;
  (void)hipMalloc(&out, sizeof(float) * 256 * cus * 8);
  run<1, 0>(out, cus); run<2, 0>(out, cus); run<4, 0>(out, cus); run<8, 0>(out, cus);
  run<2, 1>(out, cus); run<2, 2>(out, cus); run<2, 4>(out, cus); run<2, 8>(out, cus);
  run<4, 2>(out, cus); run<4, 4>(out, cus); run<8, 2>(out, cus); run<8, 4>(out, cus);
  return 0;
}
