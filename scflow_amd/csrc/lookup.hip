// a2 — multi-scale pyramid window lookup (CorrLookup, /root/reference/models/utils/corr_lookup.py:102-136).
//
// One thread per (pixel p, level l, window column a): it produces the 2r+1 samples b = 0..2r of
// output channels l·D² + a·D + b (D = 2r+1), which are contiguous in the channels-last output,
// so 36 neighbouring threads write one pixel's 324 floats in one contiguous run.  Each sample
// keeps the reference's own coordinate arithmetic — centroid (x+flow)/2^l, + window offset,
// normalise g·2/max(W−1,1)−1, align_corners unnormalise ((g+1)/2)·(W−1) — with FP contraction off,
// so the floor() of every tap matches grid_sample's, then grid_sample's bilinear weights
// (nw, ne, sw, se) with zero padding.  The pyramid (≈5.6 MB per pair at 256²) is read through
// L2 / Infinity Cache; every thread of a pixel reads the same small region of one level map.
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
  const long long total = (long long)n * h * w * num_levels * (2 * radius + 1);
  const int blocks = (int)((total + 255) / 256);
  hipStream_t st = (hipStream_t)stream;
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
