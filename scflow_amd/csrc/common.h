// Shared helpers for the gfx950 SCFlow kernels.  Wave64, CDNA4 only.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "../../include/scflow_hip.h"

#define SCFLOW_API extern "C" __attribute__((visibility("default")))

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

// Static unroll: StaticFor<I, N>::run(f) calls f(integral_constant<int, i>) for i = I .. N-1 as
// straight-line code (MFMA block loops: compile-time register-ring slots and exact wait counts,
// which a rolled loop over a runtime-indexed register ring does not get)
template <int I, int N>
struct StaticFor {
  template <class F>
  __device__ __forceinline__ static void run(F& f) {
    f(std::integral_constant<int, I>{});
    StaticFor<I + 1, N>::run(f);
  }
};
template <int N>
struct StaticFor<N, N> {
  template <class F>
  __device__ __forceinline__ static void run(F&) {}
};

static inline int scflow_launch_status() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? SCFLOW_OK : (int)e;
}

static inline bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

static inline int ceil_div(long long a, long long b) { return (int)((a + b - 1) / b); }

// compute units of the current device (256 on MI355X; also the fallback without a device)
static inline int device_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
  }
  return cus;
}

__device__ __forceinline__ float act_apply(float v, int act) {
  switch (act) {
    case SCFLOW_ACT_RELU: return v > 0.f ? v : 0.f;
    case SCFLOW_ACT_SIGMOID: return 1.f / (1.f + expf(-v));
    case SCFLOW_ACT_TANH: return tanhf(v);
    default: return v;
  }
}

__device__ __forceinline__ float sigmoidf_(float v) { return 1.f / (1.f + expf(-v)); }

// scale / shift of GroupNorm(groups) for channel c of image img from tpi partial statistics
// st [n][tpi][groups][2] (fp64 sum, sum of squares over hw pixels of the group's channels),
// summed in a fixed order (the pose head's fused-statistics convs, scflow_ph_conv_gn)
__device__ __forceinline__ void ph_gn_affine(const double* st, int tpi, int groups, int c, int cin,
                                             int img, int hw, const float* gamma, const float* beta,
                                             float eps, float& sc, float& sh) {
  const int cpg = cin / groups, g = c / cpg;
  double A = 0, B = 0;
  for (int t = 0; t < tpi; ++t) {
    const double* p = st + (((size_t)img * tpi + t) * groups + g) * 2;
    A += p[0];
    B += p[1];
  }
  const double cnt = (double)hw * cpg;
  const double mean = A / cnt;
  double var = B / cnt - mean * mean;
  if (var < 0) var = 0;
  const float rstd = (float)(1.0 / sqrt(var + (double)eps));
  sc = gamma[c] * rstd;
  sh = beta[c] - (float)mean * sc;
}
