// 1×1 MFMA conv (channels-last GEMM C[M,N] = A[M,K]·W[K,N] + bias, ReLU) pipeline variants at
// corr_net.0's shape (M = 16·32·32, K = 324 padded to 336, N = 256), HIP-event timed and checked
// against a plain fp32 kernel.  Weights packed as the product's conv_mfma ([N/64][stage][64][16]).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/micro/conv1x1_variants tools/micro/conv1x1_variants.hip
//   ./tools/micro/conv1x1_variants [M] [K] [N]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

constexpr int PK = 16;   // packed stage depth
constexpr int PBN = 64;  // packed n block
constexpr int LDA = PK + 4;

struct Args {
  const float* a;  // [M][lda]
  int lda, K, nst; // K real channels, nst = padded/16 stages
  const float* w;  // packed [N/64][nst][64][16]
  const float* bias;
  float* out;      // [M][N]
  int M, N;
};

// TM × TN per workgroup, WGM × WGN waves, each wave (TM/WGM) × (TN/WGN) = RB × CB blocks of 32×32.
// SUB packed stages per pipeline step.  DB: LDS double buffer, one barrier per step; else the
// product's scheme (store, barrier, issue next loads, MFMAs, barrier).
template <int TM, int TN, int WGM, int WGN, int SUB, bool DB, int MINB>
__global__ __launch_bounds__(64 * WGM * WGN, MINB) void k1x1(Args P) {
  constexpr int NT = 64 * WGM * WGN;
  constexpr int RB = TM / WGM / 32, CB = TN / WGN / 32;
  constexpr int A4 = TM * PK / 4 * SUB, B4 = TN * PK / 4 * SUB;  // float4 per step
  constexpr int NA = (A4 + NT - 1) / NT, NB = (B4 + NT - 1) / NT;
  constexpr int ASZ = SUB * TM * LDA, BSZ = SUB * TN * LDA;
  extern __shared__ float smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % WGM, wn = wave / WGM, li = lane & 31, hh = lane >> 5;
  const int m0 = blockIdx.x * TM, nb0 = blockIdx.y * (TN / PBN);
  const int steps = (P.nst + SUB - 1) / SUB;

  floatx4 ra[NA], rb[NB];
  auto gload = [&](int t) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      const int idx = tid + NT * j;
      const int sub = idx / (TM * PK / 4), r = idx % (TM * PK / 4);
      const int row = r / (PK / 4), q = r % (PK / 4);
      const int c = (t * SUB + sub) * PK + 4 * q;
      floatx4 v = {0.f, 0.f, 0.f, 0.f};
      if ((A4 % NT == 0 || idx < A4) && c < P.K) v = *(const floatx4*)(P.a + (size_t)(m0 + row) * P.lda + c);
      ra[j] = v;
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int idx = tid + NT * j;
      const int sub = idx / (TN * PK / 4), r = idx % (TN * PK / 4);
      const int nrow = r / (PK / 4), q = r % (PK / 4);
      const int s = t * SUB + sub;
      floatx4 v = {0.f, 0.f, 0.f, 0.f};
      if ((B4 % NT == 0 || idx < B4) && s < P.nst)
        v = *(const floatx4*)(P.w + (((size_t)(nb0 + nrow / PBN) * P.nst + s) * PBN + nrow % PBN) * PK + 4 * q);
      rb[j] = v;
    }
  };
  auto lstore = [&](int buf) __attribute__((always_inline)) {
    float* As = smem + buf * (ASZ + BSZ);
    float* Bs = As + ASZ;
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      const int idx = tid + NT * j;
      if (A4 % NT == 0 || idx < A4) {
        const int sub = idx / (TM * PK / 4), r = idx % (TM * PK / 4);
        *(floatx4*)(As + (sub * TM + r / (PK / 4)) * LDA + 4 * (r % (PK / 4))) = ra[j];
      }
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int idx = tid + NT * j;
      if (B4 % NT == 0 || idx < B4) {
        const int sub = idx / (TN * PK / 4), r = idx % (TN * PK / 4);
        *(floatx4*)(Bs + (sub * TN + r / (PK / 4)) * LDA + 4 * (r % (PK / 4))) = rb[j];
      }
    }
  };
  floatx16 acc[RB][CB];
#pragma unroll
  for (int r = 0; r < RB; ++r)
#pragma unroll
    for (int c = 0; c < CB; ++c)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[r][c][e] = 0.f;
  auto compute = [&](int buf, int t) __attribute__((always_inline)) {
    const float* As = smem + buf * (ASZ + BSZ);
    const float* Bs = As + ASZ;
#pragma unroll
    for (int sub = 0; sub < SUB; ++sub) {
      if (SUB > 1 && t * SUB + sub >= P.nst) break;
#pragma unroll
      for (int kb = 0; kb < PK; kb += 8) {
        floatx4 av[RB], bv[CB];
#pragma unroll
        for (int r = 0; r < RB; ++r)
          av[r] = *(const floatx4*)(As + (sub * TM + wm * (TM / WGM) + r * 32 + li) * LDA + kb + 4 * hh);
#pragma unroll
        for (int c = 0; c < CB; ++c)
          bv[c] = *(const floatx4*)(Bs + (sub * TN + wn * (TN / WGN) + c * 32 + li) * LDA + kb + 4 * hh);
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int r = 0; r < RB; ++r)
#pragma unroll
            for (int c = 0; c < CB; ++c)
              acc[r][c] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[r][e], bv[c][e], acc[r][c], 0, 0, 0);
      }
    }
  };

  if constexpr (DB) {
    gload(0);
    lstore(0);
    __syncthreads();
    for (int t = 0; t < steps; ++t) {
      if (t + 1 < steps) gload(t + 1);
      compute(t & 1, t);
      if (t + 1 < steps) lstore((t + 1) & 1);
      __syncthreads();
    }
  } else {
    gload(0);
    for (int t = 0; t < steps; ++t) {
      __syncthreads();
      lstore(0);
      __syncthreads();
      if (t + 1 < steps) gload(t + 1);
      compute(0, t);
    }
  }
#pragma unroll
  for (int c = 0; c < CB; ++c) {
    const int col = blockIdx.y * TN + wn * (TN / WGN) + c * 32 + li;
    const float b = P.bias[col];
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = m0 + wm * (TM / WGM) + r * 32 + (e & 3) + 8 * (e >> 2) + 4 * hh;
        const float v = acc[r][c][e] + b;
        P.out[(size_t)row * P.N + col] = v > 0.f ? v : 0.f;
      }
  }
}

__global__ void ref_kernel(const float* a, int lda, int K, const float* wt /*[N][K]*/, const float* bias,
                           float* out, int M, int N) {
  const int col = blockIdx.y * 64 + threadIdx.x % 64;
  const int row = blockIdx.x * 4 + threadIdx.x / 64;
  if (row >= M || col >= N) return;
  float s = 0.f;
  for (int k = 0; k < K; ++k) s += a[(size_t)row * lda + k] * wt[(size_t)col * K + k];
  s += bias[col];
  out[(size_t)row * N + col] = s > 0.f ? s : 0.f;
}

template <int TM, int TN, int WGM, int WGN, int SUB, bool DB, int MINB>
void run(const char* name, Args P, const float* ref, int reps) {
  constexpr int ASZ = SUB * TM * LDA, BSZ = SUB * TN * LDA;
  const size_t lds = (size_t)(DB ? 2 : 1) * (ASZ + BSZ) * 4;
  auto kern = k1x1<TM, TN, WGM, WGN, SUB, DB, MINB>;
  if (lds > 64 * 1024) CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  dim3 grid(P.M / TM, P.N / TN);
  CK(hipMemset(P.out, 0, (size_t)P.M * P.N * 4));
  for (int i = 0; i < 3; ++i) kern<<<grid, 64 * WGM * WGN, lds>>>(P);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) kern<<<grid, 64 * WGM * WGN, lds>>>(P);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<float> h((size_t)P.M * P.N), r((size_t)P.M * P.N);
  CK(hipMemcpy(h.data(), P.out, h.size() * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(r.data(), ref, r.size() * 4, hipMemcpyDeviceToHost));
  double err = 0, mx = 0;
  for (size_t i = 0; i < h.size(); ++i) {
    err = fmax(err, fabs((double)h[i] - r[i]));
    mx = fmax(mx, fabs((double)r[i]));
  }
  const double us = ms * 1e3 / reps;
  const double fl = 2.0 * P.M * P.N * P.K;
  printf("%-34s grid %5d lds %6zu B  %7.2f us  %6.1f TF/s  max err %.2e (of %.2e)\n", name,
         grid.x * grid.y, lds, us, fl / us / 1e6, err, mx);
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 16384, K = argc > 2 ? atoi(argv[2]) : 324,
            N = argc > 3 ? atoi(argv[3]) : 256;
  const int nst = (K + PK - 1) / PK;
  std::vector<float> a((size_t)M * K), wt((size_t)N * K), bias(N), wp((size_t)N * nst * PK, 0.f);
  srand(7);
  for (auto& v : a) v = (float)rand() / RAND_MAX - 0.5f;
  for (auto& v : wt) v = ((float)rand() / RAND_MAX - 0.5f) * 0.1f;
  for (auto& v : bias) v = ((float)rand() / RAND_MAX - 0.5f);
  for (int n = 0; n < N; ++n)
    for (int k = 0; k < K; ++k) {
      const int s = k / PK, kk = k % PK;
      wp[(((size_t)(n / PBN) * nst + s) * PBN + n % PBN) * PK + kk] = wt[(size_t)n * K + k];
    }
  float *da, *dwt, *dwp, *db, *dout, *dref;
  CK(hipMalloc(&da, a.size() * 4));
  CK(hipMalloc(&dwt, wt.size() * 4));
  CK(hipMalloc(&dwp, wp.size() * 4));
  CK(hipMalloc(&db, N * 4));
  CK(hipMalloc(&dout, (size_t)M * N * 4));
  CK(hipMalloc(&dref, (size_t)M * N * 4));
  CK(hipMemcpy(da, a.data(), a.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dwt, wt.data(), wt.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dwp, wp.data(), wp.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(db, bias.data(), N * 4, hipMemcpyHostToDevice));
  ref_kernel<<<dim3(M / 4, N / 64), 256>>>(da, K, K, dwt, db, dref, M, N);
  CK(hipDeviceSynchronize());
  Args P{da, K, K, nst, dwp, db, dout, M, N};
  const int reps = 50;
  printf("M=%d K=%d N=%d\n", M, K, N);
  for (int rep = 0; rep < 2; ++rep) {
    run<128, 64, 2, 2, 1, false, 2>("base 128x64 4w sub1", P, dref, reps);
    run<128, 64, 2, 2, 1, true, 2>("db 128x64 4w sub1", P, dref, reps);
    run<128, 64, 2, 2, 2, true, 2>("db 128x64 4w sub2", P, dref, reps);
    run<128, 64, 2, 2, 4, true, 2>("db 128x64 4w sub4", P, dref, reps);
    run<64, 64, 2, 2, 2, true, 4>("db 64x64 4w sub2", P, dref, reps);
    run<64, 64, 1, 2, 2, true, 4>("db 64x64 2w sub2 (64x32/w)", P, dref, reps);
    run<128, 128, 2, 2, 2, true, 1>("db 128x128 4w sub2 (64x64/w)", P, dref, reps);
    run<128, 128, 4, 2, 2, true, 1>("db 128x128 8w sub2", P, dref, reps);
    run<256, 64, 4, 2, 2, true, 1>("db 256x64 8w sub2", P, dref, reps);
    run<128, 64, 4, 2, 2, true, 2>("db 128x64 8w sub2 (32x32/w)", P, dref, reps);
  }
  return 0;
}
