// Batched, strided fp32 GEMM on the matrix cores for the training step's plain contractions —
// the correlation volume's backward (dF1 = dC·F2ᵀ/√C, dF2 = dCᵀ·F1/√C; the adjoint of
// CorrelationPyramid, /root/reference/models/decoder/raft_decoder.py:35-58), the 7×7 convs'
// weight gradient dYᵀ·cols, and the pose head's fully connected layers (forward and both
// backward products; models/head/pose_head.py:201-211).  These used to go to the vendor GEMM
// (hipBLASLt through torch.matmul), whose kernels a hipGraph capture of the training step
// cannot instantiate on this stack; with this kernel every launch of the step is ours.
//
//   C[b][m][n] = alpha · Σ_k A[b][m][k]·B[b][k][n]  (+ beta · C[b][m][n])  (+ bias)
//
// Every operand is addressed through explicit (batch, row, column) element strides, so
// transposes are free.  v_mfma_f32_32x32x2_f32 (exact fp32 FMA chains).  The workgroup tile is
// T×T (T = 128: 4 waves of 64×64, or T = 64: 4 waves of 32×32 for thin problems), K staged GK
// deep through LDS with the next stage's global loads in flight during the MFMAs.  A stage costs
// about one global-load latency (≈1 µs) when its MFMAs are few, so the thin, latency-bound
// products (under two rounds of workgroups: the FC layers, the deep-K weight gradients) take
// 32-deep stages and splits of K that leave each workgroup a few of them; products with many
// workgroups keep 16-deep stages (more workgroups resident to hide the latency).  A tile is
// loaded as float4 along whichever of its dimensions has unit stride (template AV / BV: 0 =
// along M / N, 1 = along K), element-wise with bounds checks at the edges or when unaligned.
// Deep, narrow products (the 7×7 weight gradients: K = every output pixel, M·N one or two
// tiles; the pose head's FC layers: M = 16 rows) split K over the grid into a caller-provided
// workspace, summed in split order by a second launch (deterministic; no atomics).  The
// epilogue reads every C element it accumulates onto (beta ≠ 0) before writing any: the reads
// are independent of the stores, not a load→store chain per element.
#include "common.h"

#include <algorithm>

namespace {

struct GemmArgs {
  const float* A;
  const float* B;
  float* C;
  const float* bias;
  int M, N, K;
  long long sab, sam, sak, sbb, sbk, sbn, scb, scm, scn;
  float alpha, beta;
  int bias_mode;  // 0 none, 1 per column n, 2 per row m
  int vec_a, vec_b;  // float4 loads allowed (16-B aligned bases and batch/outer strides)
  int batch, kchunk;  // K split: blockIdx.z = split·batch + b covers k ∈ [split·kchunk, +kchunk)
  float* ws;          // split > 1: raw partial sums [split][batch][M][N]; the epilogue is the reduce's
};

constexpr int gemm_nj(int T, int GK) { return GK * T / 1024; }  // float4 per thread per operand stage

// one operand tile [GK][T] (k-major in LDS) from X[k][t] = X + t·st + k·sk; V = 0: float4 along t
// (st == 1), V = 1: float4 along k (sk == 1)
template <int T, int GK, int V>
__device__ __forceinline__ void gemm_gload(const float* X, long long st, long long sk, int t0, int k0,
                                           int T_lim, int K, bool vec, floatx4 (&r)[gemm_nj(T, GK)]) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int j = 0; j < gemm_nj(T, GK); ++j) {
    const int idx = tid + 256 * j;
    int t, k;
    if (V == 0) {
      k = idx / (T / 4);
      t = (idx % (T / 4)) * 4;
    } else {
      t = idx / (GK / 4);
      k = (idx % (GK / 4)) * 4;
    }
    const int gt = t0 + t, gk = k0 + k;
    if (V == 0 && vec && gk < K && gt + 3 < T_lim) {
      r[j] = *(const floatx4*)(X + (size_t)gk * sk + gt);
    } else if (V == 1 && vec && gt < T_lim && gk + 3 < K) {
      r[j] = *(const floatx4*)(X + (size_t)gt * st + gk);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int tt = V == 0 ? gt + e : gt, kk = V == 0 ? gk : gk + e;
        r[j][e] = (tt < T_lim && kk < K) ? X[(size_t)tt * st + (size_t)kk * sk] : 0.f;
      }
    }
  }
}

template <int T, int GK, int V>
__device__ __forceinline__ void gemm_lstore(float (*S)[T + 4], const floatx4 (&r)[gemm_nj(T, GK)]) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int j = 0; j < gemm_nj(T, GK); ++j) {
    const int idx = tid + 256 * j;
    if (V == 0) {
      *(floatx4*)&S[idx / (T / 4)][(idx % (T / 4)) * 4] = r[j];
    } else {
      const int t = idx / (GK / 4), k = (idx % (GK / 4)) * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e) S[k + e][t] = r[j][e];
    }
  }
}

template <int T, int GK, int AV, int BV>
__global__ __launch_bounds__(256, 2) void gemm_f32_kernel(GemmArgs g) {
  constexpr int WT = T / 2;       // wave tile (2×2 waves)
  constexpr int NB = WT / 32;     // 32×32 MFMA blocks per wave dimension
  __shared__ float As[GK][T + 4];
  __shared__ float Bs[GK][T + 4];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave & 1, wn = wave >> 1, li = lane & 31, hh = lane >> 5;
  const int b = blockIdx.z % g.batch, split = blockIdx.z / g.batch;
  const int m0 = blockIdx.y * T, n0 = blockIdx.x * T;
  const int kbeg = split * g.kchunk;
  const int K = min(g.K - kbeg, g.kchunk);  // this split's depth
  const float* A = g.A + (size_t)b * g.sab + (size_t)kbeg * g.sak;
  const float* B = g.B + (size_t)b * g.sbb + (size_t)kbeg * g.sbk;
  // A as [k][m]: element (m, k) at m·sam + k·sak;  B as [k][n]: (k, n) at n·sbn + k·sbk
  floatx4 ra[gemm_nj(T, GK)], rb[gemm_nj(T, GK)];
  floatx16 acc[NB][NB];
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  gemm_gload<T, GK, AV>(A, g.sam, g.sak, m0, 0, g.M, K, g.vec_a, ra);
  gemm_gload<T, GK, BV>(B, g.sbn, g.sbk, n0, 0, g.N, K, g.vec_b, rb);
  for (int k0 = 0; k0 < K; k0 += GK) {
    __syncthreads();
    gemm_lstore<T, GK, AV>(As, ra);
    gemm_lstore<T, GK, BV>(Bs, rb);
    __syncthreads();
    if (k0 + GK < K) {
      gemm_gload<T, GK, AV>(A, g.sam, g.sak, m0, k0 + GK, g.M, K, g.vec_a, ra);
      gemm_gload<T, GK, BV>(B, g.sbn, g.sbk, n0, k0 + GK, g.N, K, g.vec_b, rb);
    }
#pragma unroll
    for (int kk = 0; kk < GK; kk += 2) {
      float av[NB], bv[NB];
#pragma unroll
      for (int i = 0; i < NB; ++i) av[i] = As[kk + hh][wm * WT + i * 32 + li];
#pragma unroll
      for (int j = 0; j < NB; ++j) bv[j] = Bs[kk + hh][wn * WT + j * 32 + li];
#pragma unroll
      for (int i = 0; i < NB; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
  }

  // C/D layout of a 32×32 block: col = lane & 31 (→ n), row = (r & 3) + 8(r >> 2) + 4(lane >> 5)
  if (g.ws) {  // K split: raw partial sums, reduced (with alpha / beta / bias) by gemm_reduce_kernel
    float* W = g.ws + (size_t)blockIdx.z * g.M * g.N;
#pragma unroll
    for (int i = 0; i < NB; ++i)
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const int n = n0 + wn * WT + j * 32 + li;
        if (n >= g.N) continue;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + wm * WT + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
          if (m < g.M) W[(size_t)m * g.N + n] = acc[i][j][r];
        }
      }
    return;
  }
  float* C = g.C + (size_t)b * g.scb;
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int n = n0 + wn * WT + j * 32 + li;
      const bool nok = n < g.N;
      const float bn = g.bias_mode == 1 && nok ? g.bias[n] : 0.f;
      float old[16];
      if (g.beta != 0.f) {  // every read first (independent loads in flight together)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + wm * WT + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
          old[r] = nok && m < g.M ? C[(size_t)m * g.scm + (size_t)n * g.scn] : 0.f;
        }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * WT + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
        if (!nok || m >= g.M) continue;
        float v = g.alpha * acc[i][j][r] + bn;
        if (g.bias_mode == 2) v += g.bias[m];
        if (g.beta != 0.f) v += g.beta * old[r];
        C[(size_t)m * g.scm + (size_t)n * g.scn] = v;
      }
    }
}

// C = alpha·Σ_split ws + beta·C + bias.  Block = 64 outputs × 4 split lanes: lane group q sums
// the splits ≡ q (mod 4) in order (unrolled: independent loads in flight), then the four partial
// sums are added in a fixed order through LDS (deterministic).
__global__ __launch_bounds__(256) void gemm_reduce_kernel(GemmArgs g, int splits) {
  __shared__ float part[4][64];
  const long long total = (long long)g.batch * g.M * g.N;
  const int o = threadIdx.x & 63, q = threadIdx.x >> 6;
  const long long i = blockIdx.x * 64LL + o;
  float s = 0.f;
  if (i < total) {
#pragma unroll 8
    for (int k = q; k < splits; k += 4) s += g.ws[(size_t)k * total + i];
  }
  part[q][o] = s;
  __syncthreads();
  if (q != 0 || i >= total) return;
  s = (part[0][o] + part[1][o]) + (part[2][o] + part[3][o]);
  const int n = (int)(i % g.N);
  const int m = (int)((i / g.N) % g.M);
  const int b = (int)(i / ((long long)g.N * g.M));
  float v = g.alpha * s;
  if (g.bias_mode == 1) v += g.bias[n];
  if (g.bias_mode == 2) v += g.bias[m];
  float* c = g.C + (size_t)b * g.scb + (size_t)m * g.scm + (size_t)n * g.scn;
  if (g.beta != 0.f) v += g.beta * *c;
  *c = v;
}

template <int T, int GK, int AV, int BV>
int gemm_launch(const GemmArgs& g, int splits, hipStream_t st) {
  dim3 grid(ceil_div(g.N, T), ceil_div(g.M, T), g.batch * splits);
  gemm_f32_kernel<T, GK, AV, BV><<<grid, 256, 0, st>>>(g);
  int s = scflow_launch_status();
  if (s || splits == 1) return s;
  const long long total = (long long)g.batch * g.M * g.N;
  gemm_reduce_kernel<<<(unsigned)((total + 63) / 64), 256, 0, st>>>(g, splits);
  return scflow_launch_status();
}

template <int T, int GK>
int gemm_dispatch(const GemmArgs& g, int av, int bv, int splits, hipStream_t st) {
  if (av == 0 && bv == 0) return gemm_launch<T, GK, 0, 0>(g, splits, st);
  if (av == 0 && bv == 1) return gemm_launch<T, GK, 0, 1>(g, splits, st);
  if (av == 1 && bv == 0) return gemm_launch<T, GK, 1, 0>(g, splits, st);
  return gemm_launch<T, GK, 1, 1>(g, splits, st);
}

// workgroup tile: 128 when that still gives a full round of workgroups, else 64
int gemm_tile(int M, int N, int batch) {
  const long long t128 = (long long)ceil_div(M, 128) * ceil_div(N, 128) * batch;
  return (M >= 128 && N >= 128 && t128 >= device_cus()) ? 128 : 64;
}

// stage depth: 32 for the latency-bound thin products (under two rounds of workgroups before
// any K split), 16 otherwise
int gemm_gk(int M, int N, int batch) {
  const int T = gemm_tile(M, N, batch);
  const long long tiles = (long long)ceil_div(M, T) * ceil_div(N, T) * batch;
  return tiles < 2LL * device_cus() ? 32 : 16;
}

}  // namespace

SCFLOW_API int scflow_gemm_f32_splits(int batch, int M, int N, int K) {
  if (batch <= 0 || M <= 0 || N <= 0 || K <= 0) return SCFLOW_EINVAL;
  const int T = gemm_tile(M, N, batch);
  const long long tiles = (long long)ceil_div(M, T) * ceil_div(N, T) * batch;
  // split K up to four workgroups per CU while every split keeps ≥ 4 stages of 32 (each stage
  // is about one load latency: few deep splits were latency-bound); at most 256 splits
  long long s = 1;
  while (tiles * s * 2 <= 4LL * device_cus() && K / (s * 2) >= 4 * 32 && s < 256) s *= 2;
  return (int)s;
}

SCFLOW_API int scflow_gemm_f32(const float* A, const float* B, float* C, const float* bias, int batch,
                               int M, int N, int K, long long sab, long long sam, long long sak,
                               long long sbb, long long sbk, long long sbn, long long scb,
                               long long scm, long long scn, float alpha, float beta, int bias_mode,
                               int splits, float* workspace, void* stream) {
  if (!A || !B || !C || batch <= 0 || M <= 0 || N <= 0 || K <= 0 || bias_mode < 0 || bias_mode > 2 ||
      (bias_mode && !bias) || splits < 1 || (splits > 1 && !workspace) ||
      (long long)batch * splits > 65535 || ceil_div(M, 64) > 65535)
    return SCFLOW_EINVAL;
  const int gk = gemm_gk(M, N, batch);
  const int kchunk = ceil_div(ceil_div(K, splits), gk) * gk;
  splits = ceil_div(K, kchunk);  // no empty split
  GemmArgs g{A, B, C, bias, M, N, K, sab, sam, sak, sbb, sbk, sbn, scb, scm, scn, alpha, beta, bias_mode,
             0, 0, batch, kchunk, splits > 1 ? workspace : nullptr};
  // the float4 direction of each operand: its unit-stride dimension (M/N first)
  const int av = sam == 1 ? 0 : (sak == 1 ? 1 : 0);
  const int bv = sbn == 1 ? 0 : (sbk == 1 ? 1 : 0);
  const long long a_outer = av == 0 ? sak : sam, b_outer = bv == 0 ? sbk : sbn;
  const bool a_unit = av == 0 ? sam == 1 : sak == 1, b_unit = bv == 0 ? sbn == 1 : sbk == 1;
  g.vec_a = a_unit && aligned16(A) && a_outer % 4 == 0 && (batch == 1 || sab % 4 == 0);
  g.vec_b = b_unit && aligned16(B) && b_outer % 4 == 0 && (batch == 1 || sbb % 4 == 0);
  hipStream_t st = (hipStream_t)stream;
  if (gemm_tile(M, N, batch) == 128)
    return gk == 32 ? gemm_dispatch<128, 32>(g, av, bv, splits, st)
                    : gemm_dispatch<128, 16>(g, av, bv, splits, st);
  return gk == 32 ? gemm_dispatch<64, 32>(g, av, bv, splits, st)
                  : gemm_dispatch<64, 16>(g, av, bv, splits, st);
}
