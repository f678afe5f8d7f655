// STREAM-like HBM ceiling on MI355X (confirm the 8 TB/s spec by measurement)
// plus FETCH_SIZE calibration patterns for the counter corrections bench.py applies.
//
//   hipcc -O3 --offload-arch=gfx950 tools/micro/stream.hip -o tools/micro/stream
//   ./stream                 → GB/s per kernel (best of 20), buffers far past the 256 MiB IC
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace -- ./stream 1   → one launch per kernel: compare each
//                              kernel's FETCH_SIZE (KiB) with its known compulsory byte count
//
// Kernels (every byte read exactly once):
//   copy_f4   b[i] = a[i]            16 B/lane loads and stores (the guide's calibrated pattern)
//   read_f4   sum of a               16 B/lane loads, one store per wave
//   write_f4  b[i] = c               16 B/lane stores
//   read_b32  sum of a               4 B/lane coalesced loads
//   gather_b32  the pyramid lookup's pattern (csrc/lookup.hip): 16 lanes read one 64-B 4×4 tile
//               with 4-byte loads, tiles visited in a scattered (hashed) order, each tile once
//   gather2_b32 the same with 128-B pieces (two adjacent tiles per 32 lanes)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));       \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

__global__ __launch_bounds__(256) void copy_f4(const float4* __restrict__ a, float4* __restrict__ b,
                                               long long n) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
    b[i] = a[i];
}

__global__ __launch_bounds__(256) void read_f4(const float4* __restrict__ a, float* __restrict__ out,
                                               long long n) {
  float s = 0.f;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const float4 v = a[i];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 12345.678f) out[blockIdx.x] = s;  // keeps the loads; never true for the data used
}

__global__ __launch_bounds__(256) void write_f4(float4* __restrict__ b, long long n, float c) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
    b[i] = make_float4(c, c, c, c);
}

__global__ __launch_bounds__(256) void read_b32(const float* __restrict__ a, float* __restrict__ out,
                                                long long n) {
  float s = 0.f;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
    s += a[i];
  if (s == 12345.678f) out[blockIdx.x] = s;
}

// tiles of 16 floats (64 B); tile t is visited by the 16-lane group g = perm(t): a bijective
// scatter over a power-of-two tile count (odd multiplier mod 2^k)
__global__ __launch_bounds__(256) void gather_b32(const float* __restrict__ a, float* __restrict__ out,
                                                  long long tiles) {
  float s = 0.f;
  const long long groups = (long long)gridDim.x * 16;
  for (long long g = blockIdx.x * 16LL + (threadIdx.x >> 4); g < tiles; g += groups) {
    const long long t = (g * 2654435761LL) & (tiles - 1);
    s += a[t * 16 + (threadIdx.x & 15)];
  }
  if (s == 12345.678f) out[blockIdx.x] = s;
}

// as gather_b32 but with 128-B pieces: 32 lanes read two adjacent 64-B tiles (one 128-B line)
__global__ __launch_bounds__(256) void gather2_b32(const float* __restrict__ a, float* __restrict__ out,
                                                   long long lines) {
  float s = 0.f;
  const long long groups = (long long)gridDim.x * 8;
  for (long long g = blockIdx.x * 8LL + (threadIdx.x >> 5); g < lines; g += groups) {
    const long long t = (g * 2654435761LL) & (lines - 1);
    s += a[t * 32 + (threadIdx.x & 31)];
  }
  if (s == 12345.678f) out[blockIdx.x] = s;
}

int main(int argc, char** argv) {
  const bool once = argc > 1;  // profiling: one launch per kernel
  const long long bytes = 2LL << 30;  // 2 GiB per buffer: 8× the Infinity Cache
  const long long n4 = bytes / 16, n1 = bytes / 4, tiles = bytes / 64;
  float *a, *b, *out;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMalloc(&out, 1 << 20));
  CK(hipMemset(a, 0, bytes));
  CK(hipMemset(b, 0, bytes));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int grid = cus * 16;
  hipEvent_t s, e;
  CK(hipEventCreate(&s));
  CK(hipEventCreate(&e));
  struct K {
    const char* name;
    double moved;  // compulsory bytes per launch
    int which;
  } ks[] = {{"copy_f4", 2.0 * bytes, 0}, {"read_f4", 1.0 * bytes, 1}, {"write_f4", 1.0 * bytes, 2},
            {"read_b32", 1.0 * bytes, 3}, {"gather_b32", 1.0 * bytes, 4},
            {"gather2_b32", 1.0 * bytes, 5}};
  for (const K& k : ks) {
    float best = 1e30f;
    const int reps = once ? 1 : 20;
    for (int r = 0; r < reps + (once ? 0 : 2); ++r) {
      CK(hipEventRecord(s));
      switch (k.which) {
        case 0: copy_f4<<<grid, 256>>>((const float4*)a, (float4*)b, n4); break;
        case 1: read_f4<<<grid, 256>>>((const float4*)a, out, n4); break;
        case 2: write_f4<<<grid, 256>>>((float4*)b, n4, 1.f); break;
        case 3: read_b32<<<grid, 256>>>(a, out, n1); break;
        case 4: gather_b32<<<grid, 256>>>(a, out, tiles); break;
        case 5: gather2_b32<<<grid, 256>>>(a, out, tiles / 2); break;
      }
      CK(hipGetLastError());
      CK(hipEventRecord(e));
      CK(hipEventSynchronize(e));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, s, e));
      if (r >= (once ? 0 : 2) && ms < best) best = ms;
    }
    printf("%-10s %8.3f ms  %7.1f GB/s  (%.0f MB moved, %.0f KiB)\n", k.name, best,
           k.moved / (best * 1e-3) / 1e9, k.moved / 1e6, k.moved / 1024.0);
  }
  CK(hipFree(a));
  CK(hipFree(b));
  CK(hipFree(out));
  return 0;
}
