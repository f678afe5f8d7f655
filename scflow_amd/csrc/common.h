// Shared helpers for the gfx950 SCFlow kernels.  Wave64, CDNA4 only.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <cstdlib>
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

// Environment switch for A/B runs of a launch-time choice: read on first use and cached (these
// sit on launch-bound paths — the decoder's recorded launches replay every iteration), re-read
// after scflow_debug_reload_switches() bumps the generation (in-process A/B).
extern std::atomic<int> g_switch_gen;
struct EnvSwitch {
  const char* name;
  int dflt;
  std::atomic<int> gen{-1};
  std::atomic<int> val{0};
  EnvSwitch(const char* n, int d) : name(n), dflt(d) {}
  int get() {
    const int g = g_switch_gen.load(std::memory_order_relaxed);
    if (gen.load(std::memory_order_acquire) != g) {
      const char* e = getenv(name);
      val.store(e ? atoi(e) : dflt, std::memory_order_relaxed);
      gen.store(g, std::memory_order_release);
    }
    return val.load(std::memory_order_relaxed);
  }
};

__device__ __forceinline__ float act_apply(float v, int act) {
  switch (act) {
    case SCFLOW_ACT_RELU: return v > 0.f ? v : 0.f;
    case SCFLOW_ACT_SIGMOID: return 1.f / (1.f + expf(-v));
    case SCFLOW_ACT_TANH: return tanhf(v);
    default: return v;
  }
}

// The GRU gates' nonlinearities (SepConvGRU z, r: sigmoid; q: tanh) on the hardware exp2 and
// reciprocal (v_exp_f32 of x·log2 e, v_rcp_f32; ≈ 1 ulp each) instead of libm's range-reduced expf
// and an IEEE division (≈ 20 VALU instructions per value: in a one-round grid the GRU epilogue
// is not overlapped by other workgroups).  Error ≤ 4e-7 absolute over the whole range (tanh: the
// 1 − 2/(1 + e^2x) form's cancellation near 0 is absolute, not relative); ±inf limits exact.
__device__ __forceinline__ float exp_hw(float v) { return __builtin_amdgcn_exp2f(v * 1.44269504089f); }
__device__ __forceinline__ float sigmoidf_(float v) { return __builtin_amdgcn_rcpf(1.f + exp_hw(-v)); }
__device__ __forceinline__ float tanhf_(float v) { return 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + exp_hw(2.f * v)); }
