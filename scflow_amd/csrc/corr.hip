// a1 — all-pairs correlation volume + average-pooled pyramid (CorrelationPyramid,
// /root/reference/models/decoder/raft_decoder.py:35-58).
//
// level0[n][p][q] = Σ_c f1[n][c][p]·f2[n][c][q] / sqrt(C): per pair a P×P×C GEMM whose operands
// are k-major as NCHW stores them (f1[c][p], f2[c][q]), so both tiles stream coalesced rows
// of P floats.  fp32 MFMA (v_mfma_f32_32x32x2_f32: exact fp32 FMA chains, the only matrix rate
// for f32 on gfx950); 128×128 output tile per 256-thread workgroup, each wave 64×64 (2×2 MFMA
// blocks), K staged 16 deep through LDS with the next stage's global loads in flight during the
// MFMAs.  The √C division is the epilogue.  Levels 1.. are AvgPool2d(2,2) of the previous level
// (sum in (0,0),(0,1),(1,0),(1,1) order, /4), one launch each.
#include "common.h"

namespace {

constexpr int TM = 128, TN = 128, TK = 16;

__global__ __launch_bounds__(256, 2) void corr_gemm_kernel(const float* __restrict__ f1,
                                                           const float* __restrict__ f2,
                                                           float* __restrict__ out, int C, int P,
                                                           int tiles_q, float sqrt_c) {
  __shared__ float As[TK][TM];
  __shared__ float Bs[TK][TN];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave & 1, wn = wave >> 1, li = lane & 31, hh = lane >> 5;
  const int n = blockIdx.y;
  const int tp = blockIdx.x / tiles_q, tq = blockIdx.x % tiles_q;
  const int p0 = tp * TM, q0 = tq * TN;
  const float* A = f1 + (size_t)n * C * P;
  const float* B = f2 + (size_t)n * C * P;

  // each thread stages 2 float4 of A and 2 of B per K-step: rows k = tid/32 (+8), cols 4·(tid%32)
  const int lr = tid >> 5, lc = (tid & 31) * 4;
  const bool vec = (P % 4) == 0;
  floatx4 ra[2], rb[2];
  auto gload = [&](int k0) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int k = k0 + lr + 8 * j;
      const int pa = p0 + lc, pb = q0 + lc;
      if (vec && k < C && pa + 3 < P) {
        ra[j] = *(const floatx4*)(A + (size_t)k * P + pa);
      } else {
        for (int e = 0; e < 4; ++e) ra[j][e] = (k < C && pa + e < P) ? A[(size_t)k * P + pa + e] : 0.f;
      }
      if (vec && k < C && pb + 3 < P) {
        rb[j] = *(const floatx4*)(B + (size_t)k * P + pb);
      } else {
        for (int e = 0; e < 4; ++e) rb[j][e] = (k < C && pb + e < P) ? B[(size_t)k * P + pb + e] : 0.f;
      }
    }
  };

  floatx16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  gload(0);
  for (int k0 = 0; k0 < C; k0 += TK) {
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      *(floatx4*)&As[lr + 8 * j][lc] = ra[j];
      *(floatx4*)&Bs[lr + 8 * j][lc] = rb[j];
    }
    __syncthreads();
    if (k0 + TK < C) gload(k0 + TK);
#pragma unroll
    for (int kk = 0; kk < TK; kk += 2) {
      float av[2], bv[2];
#pragma unroll
      for (int a = 0; a < 2; ++a) av[a] = As[kk + hh][wm * 64 + a * 32 + li];
#pragma unroll
      for (int b = 0; b < 2; ++b) bv[b] = Bs[kk + hh][wn * 64 + b * 32 + li];
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[a], bv[b], acc[a][b], 0, 0, 0);
    }
  }

  // epilogue: C/D layout of 32x32: col = lane&31, row = (r&3) + 8(r>>2) + 4(lane>>5)
  float* O = out + (size_t)n * P * P;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int q = q0 + wn * 64 + b * 32 + li;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int p = p0 + wm * 64 + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
        if (p < P && q < P) O[(size_t)p * P + q] = acc[a][b][r] / sqrt_c;
      }
    }
}

// ---------------------------------------------------------------------------------------------
// Tiled pyramid (scflow_corr_pyramid_tiled): every level's map of a query pixel stored in 4×4
// tiles of 16 floats (64 B, tiles row-major): element (y, x) of an hl×wl map at
// ((y>>2)·(wl>>2) + (x>>2))·16 + (y&3)·4 + (x&3).  A lookup window of (2r+2)² taps then touches
// ≈ 3.3² whole 64-B sectors instead of 2r+2 row segments that straddle them.
//
// The GEMM's N dimension runs over the target pixels q in 8×8-block order (block-major, then
// row-major inside the 8×8 block), so each wave's 64 accumulator columns are one 8×8 block of the
// map: the epilogue writes level 0 (each 32-lane half-row pair is one contiguous 128-B run: two
// adjacent tiles), then pools level 1 (the block's 4×4 = one tile), 2 (2×2) and 3 (1×1) from the
// registers with lane shuffles — the same sums in the same order as AvgPool2d's reference kernel
// (s00 + s01 + s10 + s11, then /4), so the levels are bit-identical to the row-major path's.
// Needs h, w multiples of 8 and each level ≥ 4 wide/tall (h, w multiples of 4·2^(L−1)).
__device__ __forceinline__ size_t tiled_off(int y, int x, int wl) {
  return (size_t)(((y >> 2) * (wl >> 2) + (x >> 2)) * 16 + (y & 3) * 4 + (x & 3));
}

__global__ __launch_bounds__(256, 2) void corr_gemm_pyr_kernel(const float* __restrict__ f1,
                                                               const float* __restrict__ f2,
                                                               float* __restrict__ pyr, int C, int H,
                                                               int W, int tiles_q, int L,
                                                               long long NP, float sqrt_c) {
  __shared__ float As[TK][TM];
  __shared__ float Bs[TK][TN];
  const int P = H * W;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave & 1, wn = wave >> 1, li = lane & 31, hh = lane >> 5;
  const int n = blockIdx.y;
  const int tp = blockIdx.x / tiles_q, tq = blockIdx.x % tiles_q;
  const int p0 = tp * TM, q0 = tq * TN;
  const float* A = f1 + (size_t)n * C * P;
  const float* B = f2 + (size_t)n * C * P;
  const int bw = W / 8;  // 8×8 blocks per map row
  const int lr = tid >> 5, lc = (tid & 31) * 4;
  // this thread's B columns: block-order index q' = q0 + lc (4 consecutive x of one block row)
  int qb;
  {
    const int qq = q0 + lc, blk = qq >> 6, in = qq & 63;
    qb = ((blk / bw) * 8 + (in >> 3)) * W + (blk % bw) * 8 + (in & 7);
  }
  floatx4 ra[2], rb[2];
  auto gload = [&](int k0) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int k = k0 + lr + 8 * j;
      const floatx4 z = {0.f, 0.f, 0.f, 0.f};
      ra[j] = (k < C && p0 + lc < P) ? *(const floatx4*)(A + (size_t)k * P + p0 + lc) : z;
      rb[j] = (k < C && q0 + lc < P) ? *(const floatx4*)(B + (size_t)k * P + qb) : z;
    }
  };
  floatx16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  gload(0);
  for (int k0 = 0; k0 < C; k0 += TK) {
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      *(floatx4*)&As[lr + 8 * j][lc] = ra[j];
      *(floatx4*)&Bs[lr + 8 * j][lc] = rb[j];
    }
    __syncthreads();
    if (k0 + TK < C) gload(k0 + TK);
#pragma unroll
    for (int kk = 0; kk < TK; kk += 2) {
      float av[2], bv[2];
#pragma unroll
      for (int a = 0; a < 2; ++a) av[a] = As[kk + hh][wm * 64 + a * 32 + li];
#pragma unroll
      for (int b = 0; b < 2; ++b) bv[b] = Bs[kk + hh][wn * 64 + b * 32 + li];
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[a], bv[b], acc[a][b], 0, 0, 0);
    }
  }
  // epilogue: this wave's columns are the 8×8 block blk of the map; lane li of accumulator
  // column block b holds (ly, lx) = (4b + li/8, li%8).  C/D rows: p = … + (r&3) + 8(r>>2) + 4hh
  const int blk = (q0 + wn * 64) >> 6;
  if (q0 + wn * 64 >= P) return;
  const int by0 = (blk / bw) * 8, bx0 = (blk % bw) * 8;
  const int lx = li & 7, lyq = li >> 3;  // ly = 4b + lyq
  size_t loff[4];  // level bases
  {
    size_t o = 0;
    int hl = H, wl = W;
    for (int l = 0; l < 4; ++l) {
      loff[l] = o;
      o += (size_t)NP * hl * wl;
      hl >>= 1;
      wl >>= 1;
    }
  }
#pragma unroll
  for (int a = 0; a < 2; ++a) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int p = p0 + wm * 64 + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
      const bool pv = p < P;
      const size_t m = (size_t)n * P + p;  // query pixel (map index)
      float v0[2], v1[2], v2[2];
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const float v = acc[a][b][r] / sqrt_c;
        v0[b] = v;
        const int y = by0 + 4 * b + lyq, x = bx0 + lx;
        if (pv) pyr[loff[0] + m * P + tiled_off(y, x, W)] = v;
      }
      if (L < 2) continue;
      // level 1: lanes with even (lx, ly) sum their 2×2 (x+1: lane+1, y+1: lane+8)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const float s01 = __shfl(v0[b], lane + 1), s10 = __shfl(v0[b], lane + 8),
                    s11 = __shfl(v0[b], lane + 9);
        float v = v0[b];
        v += s01;
        v += s10;
        v += s11;
        v1[b] = v / 4.f;
        const int y1 = (by0 + 4 * b + lyq) >> 1, x1 = (bx0 + lx) >> 1;
        if (pv && !(lx & 1) && !(lyq & 1)) pyr[loff[1] + m * (P / 4) + tiled_off(y1, x1, W / 2)] = v1[b];
      }
      if (L < 3) continue;
      // level 2: level-1 cells at lanes with lx%4 == 0, lyq even; x+1 → lane+2, y+1 → lane+16
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const float s01 = __shfl(v1[b], lane + 2), s10 = __shfl(v1[b], lane + 16),
                    s11 = __shfl(v1[b], lane + 18);
        float v = v1[b];
        v += s01;
        v += s10;
        v += s11;
        v2[b] = v / 4.f;
        const int y2 = (by0 + 4 * b) >> 2, x2 = (bx0 + lx) >> 2;
        if (pv && !(lx & 3) && lyq == 0) pyr[loff[2] + m * (P / 16) + tiled_off(y2, x2, W / 4)] = v2[b];
      }
      if (L < 4) continue;
      // level 3: level-2 cells (b, lx/4): x+1 → lane+4, y+1 → the b = 1 value of the same lane
      {
        const float s01 = __shfl(v2[0], lane + 4), s11 = __shfl(v2[1], lane + 4);
        float v = v2[0];
        v += s01;
        v += v2[1];
        v += s11;
        v = v / 4.f;
        if (pv && lx == 0 && lyq == 0)
          pyr[loff[3] + m * (P / 64) + tiled_off(by0 >> 3, bx0 >> 3, W / 8)] = v;
      }
    }
  }
}

// one pyramid level: out[m][y][x] = (in[2y][2x] + in[2y][2x+1] + in[2y+1][2x] + in[2y+1][2x+1])/4
__global__ void avgpool2_kernel(const float* __restrict__ in, float* __restrict__ out, long long M,
                                int Hi, int Wi, int Ho, int Wo) {
  const long long total = M * Ho * Wo;
  for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * blockDim.x) {
    const int x = (int)(idx % Wo);
    const long long t = idx / Wo;
    const int y = (int)(t % Ho);
    const long long m = t / Ho;
    const float* s = in + (size_t)m * Hi * Wi + (size_t)(2 * y) * Wi + 2 * x;
    float v = s[0];
    v += s[1];
    v += s[Wi];
    v += s[Wi + 1];
    out[idx] = v / 4.f;
  }
}

}  // namespace

SCFLOW_API long long scflow_corr_pyramid_size(int n, int h, int w, int num_levels) {
  if (n <= 0 || h <= 0 || w <= 0 || num_levels <= 0) return -1;
  long long P = (long long)h * w, tot = 0;
  for (int l = 0; l < num_levels; ++l) tot += (long long)(h >> l) * (w >> l);
  return (long long)n * P * tot;
}

SCFLOW_API int scflow_corr_pyramid(const float* f1, const float* f2, float* pyr, int n, int c,
                                   int h, int w, int num_levels, void* stream) {
  if (!f1 || !f2 || !pyr || n <= 0 || c <= 0 || h <= 0 || w <= 0 || num_levels < 1 ||
      num_levels > 8)
    return SCFLOW_EINVAL;
  if ((h >> (num_levels - 1)) < 1 || (w >> (num_levels - 1)) < 1) return SCFLOW_EUNSUPPORTED;
  hipStream_t st = (hipStream_t)stream;
  const int P = h * w;
  const int tp = ceil_div(P, TM), tq = ceil_div(P, TN);
  dim3 grid(tp * tq, n);
  corr_gemm_kernel<<<grid, 256, 0, st>>>(f1, f2, pyr, c, P, tq, sqrtf((float)c));
  int s = scflow_launch_status();
  if (s) return s;
  const float* prev = pyr;
  float* cur = pyr + (size_t)n * P * P;
  int Hi = h, Wi = w;
  for (int l = 1; l < num_levels; ++l) {
    const int Ho = Hi / 2, Wo = Wi / 2;
    const long long M = (long long)n * P;
    const long long total = M * Ho * Wo;
    const int blocks = (int)((total + 255) / 256 < 65535 * 8 ? (total + 255) / 256 : 65535 * 8);
    avgpool2_kernel<<<blocks, 256, 0, st>>>(prev, cur, M, Hi, Wi, Ho, Wo);
    s = scflow_launch_status();
    if (s) return s;
    prev = cur;
    cur += (size_t)M * Ho * Wo;
    Hi = Ho;
    Wi = Wo;
  }
  return SCFLOW_OK;
}

SCFLOW_API int scflow_corr_pyramid_tiled(const float* f1, const float* f2, float* pyr, int n, int c,
                                         int h, int w, int num_levels, void* stream) {
  if (!f1 || !f2 || !pyr || n <= 0 || c <= 0 || h <= 0 || w <= 0 || num_levels < 1 ||
      num_levels > 4)
    return SCFLOW_EINVAL;
  const int g = 4 << (num_levels - 1);  // every level's map a whole number of 4×4 tiles
  if (h % 8 || w % 8 || h % g || w % g) return SCFLOW_EUNSUPPORTED;
  if (((uintptr_t)f1 & 15) || ((uintptr_t)f2 & 15)) return SCFLOW_EALIGN;
  const int P = h * w;
  const int tp = ceil_div(P, TM), tq = ceil_div(P, TN);
  dim3 grid(tp * tq, n);
  corr_gemm_pyr_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(f1, f2, pyr, c, h, w, tq, num_levels,
                                                            (long long)n * P, sqrtf((float)c));
  return scflow_launch_status();
}
