// §8(f)-2 — training-step building blocks (backward passes of the hot path).
//
//  * im2col_kernel — the patch matrix of a channels-last conv input, so the weight gradient of
//    every conv (decoder, pose head, encoders; any kernel size / stride) is one plain GEMM
//    dW = dYᵀ·cols (run on hipBLASLt: the task's "plain library GEMM" case).  float4 per
//    thread along the channels when cin % 4 == 0.
//  * corr_lookup_bwd_kernel — the adjoint of CorrLookup (models/utils/corr_lookup.py:102-136):
//    every output sample scatters its gradient to the 4 bilinear taps of its pyramid level with
//    the same weights grid_sample used (same fp32 coordinate arithmetic as lookup.hip, FP
//    contraction off, so the taps and weights are bit-identical to the forward's).  fp32
//    atomics: the order of additions is not deterministic (training only).
#include "common.h"

namespace {

__global__ void im2col_kernel(const float* __restrict__ x, int sx, float* __restrict__ cols, int h,
                              int w, int cin, int kh, int kw, int stride, int ph, int pw, int oh,
                              int ow, long long total_vec, int vec) {
  const int K = kh * kw * cin;
  const int kv = K / vec;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total_vec; i += (long long)gridDim.x * 256) {
    const long long p = i / kv;
    const int k = (int)(i % kv) * vec;
    const int tap = k / cin, c = k % cin;
    const int ty = tap / kw, tx = tap % kw;
    const int ox = (int)(p % ow);
    const long long t = p / ow;
    const int oy = (int)(t % oh);
    const int img = (int)(t / oh);
    const int iy = oy * stride - ph + ty, ix = ox * stride - pw + tx;
    const bool ok = iy >= 0 && iy < h && ix >= 0 && ix < w;
    const float* src = x + ((size_t)(img * h + iy) * w + ix) * sx + c;
    float* dst = cols + p * K + k;
    if (vec == 4) {
      floatx4 v = {0.f, 0.f, 0.f, 0.f};
      if (ok) v = *(const floatx4*)src;
      *(floatx4*)dst = v;
    } else {
      *dst = ok ? *src : 0.f;
    }
  }
}

__device__ __forceinline__ float unnorm_coord_b(float s, int size) {
#pragma clang fp contract(off)
  const float g = (s * 2.f) / (float)(size - 1 > 1 ? size - 1 : 1) - 1.f;
  return ((g + 1.f) / 2.f) * (float)(size - 1);
}

__device__ __forceinline__ void tap_add(float* m, int x, int y, int Wl, int Hl, float v) {
  if (x >= 0 && x < Wl && y >= 0 && y < Hl) atomicAdd(m + y * Wl + x, v);
}

// thread = (pixel, level, a): the D samples b of column a (x + a − r), like the forward's
// generic kernel, accumulating into the level's map of that pixel
template <int R>
__global__ __launch_bounds__(256) void corr_lookup_bwd_kernel(
    const float* __restrict__ dout, int out_layout, int out_stride, const float* __restrict__ flow,
    int flow_layout, float* __restrict__ dpyr, int N, int H, int W, int L, long long total) {
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
  size_t off = 0;
  int Hl = H, Wl = W;
  for (int l = 0; l < lvl; ++l) {
    off += (size_t)N * P * Hl * Wl;
    Hl >>= 1;
    Wl >>= 1;
  }
  float* m = dpyr + off + ((size_t)n * P + p) * Hl * Wl;
  const float scale = (float)(1 << lvl);
  const float cx = ((float)x + fx) / scale;
  const float cy = ((float)y + fy) / scale;
  const float ix = unnorm_coord_b(cx + (float)(a - r), Wl);
  const float ix_w = floorf(ix);
  const float ix_e = ix_w + 1.f;
  const int xw = (int)ix_w, xe = xw + 1;
  const float* g = out_layout == SCFLOW_LAYOUT_NHWC
                       ? dout + ((size_t)n * P + p) * out_stride + lvl * D * D + a * D
                       : dout + ((size_t)n * L * D * D + lvl * D * D + a * D) * P + p;
  const int gstep = out_layout == SCFLOW_LAYOUT_NHWC ? 1 : P;
  for (int b = 0; b < D; ++b) {
    const float gv = g[(size_t)b * gstep];
    if (gv == 0.f) continue;
    const float iy = unnorm_coord_b(cy + (float)(b - r), Hl);
    const float iy_n = floorf(iy);
    const float iy_s = iy_n + 1.f;
    const int yn = (int)iy_n, ys = yn + 1;
    tap_add(m, xw, yn, Wl, Hl, gv * ((ix_e - ix) * (iy_s - iy)));
    tap_add(m, xe, yn, Wl, Hl, gv * ((ix - ix_w) * (iy_s - iy)));
    tap_add(m, xw, ys, Wl, Hl, gv * ((ix_e - ix) * (iy - iy_n)));
    tap_add(m, xe, ys, Wl, Hl, gv * ((ix - ix_w) * (iy - iy_n)));
  }
}

}  // namespace

SCFLOW_API int scflow_im2col(const float* x, int sx, float* cols, int n, int h, int w, int cin,
                             int kh, int kw, int stride, int ph, int pw, void* stream) {
  if (!x || !cols || n <= 0 || h <= 0 || w <= 0 || cin <= 0 || kh <= 0 || kw <= 0 || stride <= 0 ||
      ph < 0 || pw < 0 || sx < cin)
    return SCFLOW_EINVAL;
  const int oh = (h + 2 * ph - kh) / stride + 1, ow = (w + 2 * pw - kw) / stride + 1;
  if (oh <= 0 || ow <= 0) return SCFLOW_EINVAL;
  const int vec = (cin % 4 == 0 && sx % 4 == 0 && aligned16(x) && aligned16(cols)) ? 4 : 1;
  const long long total = (long long)n * oh * ow * kh * kw * cin / vec;
  const int blocks = (int)((total + 255) / 256 < 65536 ? (total + 255) / 256 : 65536);
  im2col_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(x, sx, cols, h, w, cin, kh, kw, stride, ph,
                                                         pw, oh, ow, total, vec);
  return scflow_launch_status();
}

SCFLOW_API int scflow_corr_lookup_backward(const float* dout, int out_layout, int out_stride,
                                           const float* flow, int flow_layout, float* dpyr, int n,
                                           int h, int w, int num_levels, int radius, void* stream) {
  if (!dout || !flow || !dpyr || n <= 0 || h <= 0 || w <= 0 || num_levels < 1 || num_levels > 8 ||
      radius < 0)
    return SCFLOW_EINVAL;
  const int D = 2 * radius + 1;
  if (out_layout == SCFLOW_LAYOUT_NHWC && out_stride < num_levels * D * D) return SCFLOW_EINVAL;
  if ((h >> (num_levels - 1)) < 1 || (w >> (num_levels - 1)) < 1) return SCFLOW_EINVAL;
  const long long total = (long long)n * h * w * num_levels * D;
  const unsigned blocks = (unsigned)((total + 255) / 256);
  hipStream_t st = (hipStream_t)stream;
  switch (radius) {
#define SCFLOW_LKB(RR)                                                                            \
  case RR:                                                                                        \
    corr_lookup_bwd_kernel<RR><<<blocks, 256, 0, st>>>(dout, out_layout, out_stride, flow,        \
                                                       flow_layout, dpyr, n, h, w, num_levels,    \
                                                       total);                                    \
    break;
    SCFLOW_LKB(1)
    SCFLOW_LKB(2)
    SCFLOW_LKB(3)
    SCFLOW_LKB(4)
    SCFLOW_LKB(5)
    SCFLOW_LKB(6)
#undef SCFLOW_LKB
    default:
      return SCFLOW_EUNSUPPORTED;
  }
  return scflow_launch_status();
}
