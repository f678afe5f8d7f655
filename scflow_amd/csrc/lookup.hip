// a2 — multi-scale pyramid window lookup (CorrLookup, /root/reference/models/utils/corr_lookup.py:102-136).
//
// One WAVE per source pixel p (4 per workgroup):
//  1. 2·L·D lanes compute the sample coordinates of every level once — the reference's own
//     arithmetic: centroid (x+flow)/2^l, + window offset, normalise g·2/max(W−1,1)−1 and the
//     align_corners unnormalise ((g+1)/2)·(W−1), FP contraction off, so each sample's floor()
//     is grid_sample's;
//  2. the wave stages, per level, the (D+3)² window around floor(first sample) − 1 in LDS with
//     zero padding (one-tap margin each side: a rounded sample coordinate can move its floor by
//     at most one);
//  3. lanes produce the L·D² outputs (channel k = l·D² + a·D + b samples x+a−r, y+b−r) from LDS
//     with grid_sample's bilinear weights (nw, ne, sw, se) — contiguous channels-last stores.
// The pyramid (≈5.6 MB per pair at 256²) is read through L2 / Infinity Cache.
// A generic one-thread-per-(p, l, a) kernel remains for L > 4 or r > 6.
#include "common.h"

namespace {

__device__ __forceinline__ float unnorm_coord(float s, int size) {
#pragma clang fp contract(off)
  const float g = (s * 2.f) / (float)(size - 1 > 1 ? size - 1 : 1) - 1.f;
  return ((g + 1.f) / 2.f) * (float)(size - 1);
}

__device__ __forceinline__ float tap(const float* __restrict__ m, int x, int y, int Wl, int Hl) {
  return (x >= 0 && x < Wl && y >= 0 && y < Hl) ? m[y * Wl + x] : 0.f;
}

template <int R>
__global__ __launch_bounds__(256) void corr_lookup_kernel(
    const float* __restrict__ pyr, const float* __restrict__ flow, int flow_layout,
    float* __restrict__ out, int out_layout, int out_stride, int N, int H, int W, int L,
    long long total) {
#pragma clang fp contract(off)
  constexpr int r = R;
  constexpr int D = 2 * R + 1;
  const int P = H * W;
  const long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int a = (int)(idx % D);
  long long t = idx / D;
  const int lvl = (int)(t % L);
  t /= L;
  const int p = (int)(t % P);
  const int n = (int)(t / P);
  const int y = p / W, x = p % W;
  float fx, fy;
  if (flow_layout == SCFLOW_LAYOUT_NHWC) {
    fx = flow[((size_t)n * P + p) * 2 + 0];
    fy = flow[((size_t)n * P + p) * 2 + 1];
  } else {
    fx = flow[((size_t)n * 2 + 0) * P + p];
    fy = flow[((size_t)n * 2 + 1) * P + p];
  }
  // level base offset
  size_t off = 0;
  int Hl = H, Wl = W;
  for (int l = 0; l < lvl; ++l) {
    off += (size_t)N * P * Hl * Wl;
    Hl >>= 1;
    Wl >>= 1;
  }
  const float* m = pyr + off + ((size_t)n * P + p) * Hl * Wl;
  const float scale = (float)(1 << lvl);
  const float cx = ((float)x + fx) / scale;
  const float cy = ((float)y + fy) / scale;
  const float ix = unnorm_coord(cx + (float)(a - r), Wl);
  const float ix_w = floorf(ix);
  const float ix_e = ix_w + 1.f;
  const int xw = (int)ix_w, xe = xw + 1;
  float* o = out_layout == SCFLOW_LAYOUT_NHWC
                 ? out + ((size_t)n * P + p) * out_stride + lvl * D * D + a * D
                 : out + ((size_t)n * L * D * D + lvl * D * D + a * D) * P + p;
  const int ostep = out_layout == SCFLOW_LAYOUT_NHWC ? 1 : P;
#pragma unroll
  for (int b = 0; b < D; ++b) {
    const float iy = unnorm_coord(cy + (float)(b - r), Hl);
    const float iy_n = floorf(iy);
    const float iy_s = iy_n + 1.f;
    const int yn = (int)iy_n, ys = yn + 1;
    const float nw = (ix_e - ix) * (iy_s - iy);
    const float ne = (ix - ix_w) * (iy_s - iy);
    const float sw = (ix_e - ix) * (iy - iy_n);
    const float se = (ix - ix_w) * (iy - iy_n);
    float v = 0.f;
    v += tap(m, xw, yn, Wl, Hl) * nw;
    v += tap(m, xe, yn, Wl, Hl) * ne;
    v += tap(m, xw, ys, Wl, Hl) * sw;
    v += tap(m, xe, ys, Wl, Hl) * se;
    o[(size_t)b * ostep] = v;
  }
}

constexpr int LK_MAXL = 4;
constexpr int LK_PPW = 4;              // pixels per wave (16 lanes each)
constexpr int LK_GL = 64 / LK_PPW;     // lanes per pixel

template <int R>
__global__ __launch_bounds__(256) void corr_lookup_lds_kernel(
    const float* __restrict__ pyr, const float* __restrict__ flow, int flow_layout,
    float* __restrict__ out, int out_layout, int out_stride, int N, int H, int W, int L) {
#pragma clang fp contract(off)
  constexpr int D = 2 * R + 1;
  constexpr int WIN = D + 3;
  constexpr int SLOTS = 4 * LK_PPW;  // pixels per workgroup
  __shared__ float win[SLOTS][LK_MAXL][WIN][WIN];
  __shared__ float crd[SLOTS][LK_MAXL][2][D];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int slot = wave * LK_PPW + lane / LK_GL;  // this lane's pixel slot
  const int gl = lane % LK_GL;                     // lane within the pixel's group
  const int P = H * W;
  const long long gp = (long long)blockIdx.x * SLOTS + slot;  // global pixel n·P + p
  const bool active = gp < (long long)N * P;
  const int n = active ? (int)(gp / P) : 0;
  const int p = active ? (int)(gp % P) : 0;
  const int y = p / W, x = p % W;
  float fx = 0.f, fy = 0.f;
  if (active) {
    if (flow_layout == SCFLOW_LAYOUT_NHWC) {
      fx = flow[((size_t)n * P + p) * 2 + 0];
      fy = flow[((size_t)n * P + p) * 2 + 1];
    } else {
      fx = flow[((size_t)n * 2 + 0) * P + p];
      fy = flow[((size_t)n * 2 + 1) * P + p];
    }
  }
  // 1. sample coordinates, once per (level, axis, index)
  for (int t = gl; t < L * 2 * D; t += LK_GL) {
    const int l = t / (2 * D), axis = (t / D) % 2, i = t % D;
    const int size = axis == 0 ? (W >> l) : (H >> l);
    const float c = ((float)(axis == 0 ? x : y) + (axis == 0 ? fx : fy)) / (float)(1 << l);
    crd[slot][l][axis][i] = unnorm_coord(c + (float)(i - R), size);
  }
  __syncthreads();
  // 2. windows (zero padded), origin = floor(first sample) − 1 per level and axis; every load
  //    of the pixel's L windows is issued before the LDS writes (one memory latency)
  constexpr int NW1 = (WIN * WIN + LK_GL - 1) / LK_GL;  // loads per lane per level
  float vals[LK_MAXL][NW1];
  int oxl[LK_MAXL], oyl[LK_MAXL];
  bool finl[LK_MAXL];
  {
    size_t loff = 0;
    int Hl = H, Wl = W;
#pragma unroll
    for (int l = 0; l < LK_MAXL; ++l) {
      const bool use = l < L;
      const float* m = pyr + loff + ((size_t)n * P + p) * Hl * Wl;
      const float c0x = use ? crd[slot][l][0][0] : 0.f, c0y = use ? crd[slot][l][1][0] : 0.f;
      finl[l] = use && active && isfinite(c0x) && isfinite(c0y) && fabsf(c0x) < 1e8f &&
                fabsf(c0y) < 1e8f;
      oxl[l] = finl[l] ? (int)floorf(c0x) - 1 : 0;
      oyl[l] = finl[l] ? (int)floorf(c0y) - 1 : 0;
#pragma unroll
      for (int j = 0; j < NW1; ++j) {
        const int i = gl + LK_GL * j;
        const int gx = oxl[l] + i % WIN, gy = oyl[l] + i / WIN;
        float v = 0.f;
        if (i < WIN * WIN && finl[l] && gx >= 0 && gx < Wl && gy >= 0 && gy < Hl) v = m[gy * Wl + gx];
        vals[l][j] = v;
      }
      if (use) loff += (size_t)N * P * Hl * Wl;
      Hl >>= 1;
      Wl >>= 1;
    }
  }
#pragma unroll
  for (int l = 0; l < LK_MAXL; ++l)
#pragma unroll
    for (int j = 0; j < NW1; ++j) {
      const int i = gl + LK_GL * j;
      if (i < WIN * WIN) (&win[slot][l][0][0])[i] = vals[l][j];
    }
  __syncthreads();
  if (!active) return;
  // 3. samples: lane g takes (level, a) pairs g, g+16, …; per pair the x coordinate, x weights
  //    and window column are computed once for the D samples b of that column
  const int K = L * D * D;
  float* o = out_layout == SCFLOW_LAYOUT_NHWC ? out + ((size_t)n * P + p) * out_stride
                                              : out + (size_t)n * K * P + p;
  const int ostep = out_layout == SCFLOW_LAYOUT_NHWC ? 1 : P;
#pragma unroll
  for (int l = 0; l < LK_MAXL; ++l) {
    if (l >= L) break;
    for (int a = gl; a < D; a += LK_GL) {
      const float ix = crd[slot][l][0][a];
      const bool okx = finl[l] && isfinite(ix);
      const float ix_w = floorf(ix), ix_e = ix_w + 1.f;
      const float wxe = ix - ix_w, wxw = ix_e - ix;
      const int rx = okx ? (int)ix_w - oxl[l] : -1;
      const bool inx = rx >= 0 && rx + 1 < WIN;
      float* ol = o + (size_t)(l * D * D + a * D) * ostep;
#pragma unroll
      for (int b = 0; b < D; ++b) {
        const float iy = crd[slot][l][1][b];
        float v = 0.f;
        if (inx && isfinite(iy)) {
          const float iy_n = floorf(iy), iy_s = iy_n + 1.f;
          const int ry = (int)iy_n - oyl[l];
          if (ry >= 0 && ry + 1 < WIN) {
            const float* wr = &win[slot][l][ry][rx];
            v += wr[0] * (wxw * (iy_s - iy));
            v += wr[1] * (wxe * (iy_s - iy));
            v += wr[WIN] * (wxw * (iy - iy_n));
            v += wr[WIN + 1] * (wxe * (iy - iy_n));
          }
        }
        ol[(size_t)b * ostep] = v;
      }
    }
  }
}

}  // namespace

SCFLOW_API int scflow_corr_lookup(const float* pyr, const float* flow, int flow_layout, float* out,
                                  int out_layout, int out_stride, int n, int h, int w,
                                  int num_levels, int radius, void* stream) {
  if (!pyr || !flow || !out || n <= 0 || h <= 0 || w <= 0 || num_levels < 1 || num_levels > 8 ||
      radius < 0)
    return SCFLOW_EINVAL;
  if (radius > 6) return SCFLOW_EUNSUPPORTED;
  const int K = num_levels * (2 * radius + 1) * (2 * radius + 1);
  if (out_layout == SCFLOW_LAYOUT_NHWC && out_stride < K) return SCFLOW_EINVAL;
  if (out_layout != SCFLOW_LAYOUT_NHWC && out_layout != SCFLOW_LAYOUT_NCHW) return SCFLOW_EINVAL;
  if ((h >> (num_levels - 1)) < 1 || (w >> (num_levels - 1)) < 1) return SCFLOW_EUNSUPPORTED;
  hipStream_t st = (hipStream_t)stream;
  if (num_levels <= LK_MAXL && radius >= 1 && radius <= 4) {
    const unsigned blk = (unsigned)(((long long)n * h * w + 4 * LK_PPW - 1) / (4 * LK_PPW));
    switch (radius) {
      case 1: corr_lookup_lds_kernel<1><<<blk, 256, 0, st>>>(pyr, flow, flow_layout, out, out_layout, out_stride, n, h, w, num_levels); break;
      case 2: corr_lookup_lds_kernel<2><<<blk, 256, 0, st>>>(pyr, flow, flow_layout, out, out_layout, out_stride, n, h, w, num_levels); break;
      case 3: corr_lookup_lds_kernel<3><<<blk, 256, 0, st>>>(pyr, flow, flow_layout, out, out_layout, out_stride, n, h, w, num_levels); break;
      default: corr_lookup_lds_kernel<4><<<blk, 256, 0, st>>>(pyr, flow, flow_layout, out, out_layout, out_stride, n, h, w, num_levels); break;
    }
    return scflow_launch_status();
  }
  const long long total = (long long)n * h * w * num_levels * (2 * radius + 1);
  const int blocks = (int)((total + 255) / 256);
#define SCFLOW_LK(RR)                                                                            \
  case RR:                                                                                       \
    corr_lookup_kernel<RR><<<blocks, 256, 0, st>>>(pyr, flow, flow_layout, out, out_layout,      \
                                                   out_stride, n, h, w, num_levels, total);      \
    break;
  switch (radius) {
    SCFLOW_LK(0) SCFLOW_LK(1) SCFLOW_LK(2) SCFLOW_LK(3) SCFLOW_LK(4) SCFLOW_LK(5) SCFLOW_LK(6)
    default: return SCFLOW_EUNSUPPORTED;
  }
#undef SCFLOW_LK
  return scflow_launch_status();
}
