// XHead hidden conv + predictors in two launches (round 6) — included by conv.hip after
// conv_pair.h (in an anonymous namespace).  Reference: the update block's two XHeads,
// models/decoder/raft_decoder.py:256-294 (flow head: 3×3 128 → 256 + ReLU, 3×3 256 → 2; mask
// head: 3×3 128 → 256 + ReLU, 1×1 256 → 1 + sigmoid), called from scflow_decoder.py:211-218.
//
// The decoder ran the two hidden convs as one 512-wide F(4×4,3×3) conv (HEAD, 2 KiB per pixel
// written) and then the predictors (the 3×3 as a channel contraction, conv_thinz.h; the 1×1
// chunked) reading HEAD back.  Here the predictors' channel contraction moves into the F(4×4)
// GEMM's epilogue (w4_pred_round, conv_wino4.h): each 32-channel block contracts its relu(y) with
// the predictor weights into per-block partial sums — the 3×3 predictor's Z[q][tap·2 + o] (18 of
// W4PZ = 20 floats per pixel), the 1×1's one float — and xhead_pred_sum_kernel adds the blocks and
// the 3×3 taps: out[p][o] = b[o] + Σ_tap Σ_block Zf[block][p + off(tap)][tap·2 + o],
// mask[p] = σ(b + Σ_block Zm[block][p]).  HEAD is never written or read.  fp32 throughout; only the
// summation order differs from the separate convs.
//
// Partial-sum buffer (zp): Zf [nbf][M][W4PZ] then Zm [nbm][M], M = n·h·w pixels, nbf = flow hidden
// channels / 32, nbm = mask hidden channels / 32 (xhead_pred_ws_bytes).

#ifndef XH_R32
#define XH_R32 2  // output rows per sum workgroup at width 32
#endif

long long xhead_pred_ws_bytes(long long m, int nbf, int nbm) {
  return (m * nbf * W4PZ + m * nbm) * (long long)sizeof(float);
}

// Workgroup = R output rows of one image (W columns).  Phase 1 sums the flow blocks of the R + 2
// input rows the 3×3 taps reach into LDS (float4 loads, zero rows outside the image); phase 2 sums
// the taps per (pixel, output) and the mask blocks per pixel.
template <int W, int R>
__global__ __launch_bounds__(256) void xhead_pred_sum_kernel(const float* __restrict__ zp, int nbf,
                                                             int nbm, int h, long long M,
                                                             const float* __restrict__ fb,
                                                             const float* __restrict__ mb, int fact,
                                                             int mact, float* __restrict__ fo,
                                                             int fso, float* __restrict__ mo, int mso) {
  constexpr int SR = R + 2, SLD = 19, NQ = W4PZ / 4;
  __shared__ float S[SR * W * SLD];
  const int tiles = h / R;
  const int img = blockIdx.x / tiles, oy0 = (blockIdx.x - img * tiles) * R;
  const size_t bstride = (size_t)M * W4PZ;
  // the mask blocks' loads first (in flight under phase 1; ≤ 8 blocks in registers)
  const float* zm = zp + (size_t)nbf * bstride;
  const int mp = threadIdx.x;
  const size_t mpix = (size_t)(img * h + oy0) * W + mp;
  float mv[8];
#pragma unroll
  for (int b = 0; b < 8; ++b) mv[b] = (mp < R * W && b < nbm) ? zm[b * (size_t)M + mpix] : 0.f;
  for (int i = threadIdx.x; i < SR * W * NQ; i += 256) {
    const int qd = i % NQ, px = i / NQ;
    const int r = px / W, x = px - r * W;
    const int iy = oy0 - 1 + r;
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    if (iy >= 0 && iy < h) {
      const float* zq = zp + ((size_t)(img * h + iy) * W + x) * W4PZ + 4 * qd;
#pragma unroll 8
      for (int b = 0; b < nbf; ++b) acc += *(const floatx4*)(zq + b * bstride);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (4 * qd + e < 18) S[px * SLD + 4 * qd + e] = acc[e];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < R * W * 2; i += 256) {
    const int o = i & 1, p = i >> 1;
    const int py = p / W, x = p - py * W;
    float v = fb ? fb[o] : 0.f;
#pragma unroll
    for (int ty = 0; ty < 3; ++ty)
#pragma unroll
      for (int tx = 0; tx < 3; ++tx) {
        const int xx = x + tx - 1;
        if (xx >= 0 && xx < W) v += S[((py + ty) * W + xx) * SLD + (ty * 3 + tx) * 2 + o];
      }
    fo[((size_t)(img * h + oy0 + py) * W + x) * fso + o] = act_apply(v, fact);
  }
  if (mp < R * W) {
    float v = mb ? mb[0] : 0.f;
#pragma unroll
    for (int b = 0; b < 8; ++b) v += mv[b];
    for (int b = 8; b < nbm; ++b) v += zm[b * (size_t)M + mpix];
    mo[mpix * mso] = act_apply(v, mact);
  }
  static_assert(R * W <= 256, "one mask pixel per thread");
}

template <int D>
int launch_wino4_pred_gemm(const Wino4Params& p, dim3 grid, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)conv_wino4_kernel<SCFLOW_ACT_RELU, D, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  conv_wino4_kernel<SCFLOW_ACT_RELU, D, true><<<grid, 256, W4_PRED_LDS, st>>>(p);
  return scflow_launch_status();
}

// hidden: the two hidden convs as one F(4×4,3×3) conv (flow channels first, ReLU, plain
// epilogue, bias only; its `out` is not written); pw [hidden.cout][W4PZ] (host packing,
// scflow_xhead_pred in include/scflow_hip.h)
int launch_xhead_pred(const scflow_conv_args& a, int flow_ch, const float* pw, float* zp,
                      long long zp_bytes, const float* fb, const float* mb, int fact, int mact,
                      float* fo, int fso, float* mo, int mso, hipStream_t st) {
  if (a.bk != SCFLOW_CONV_WINO4 || a.act != SCFLOW_ACT_RELU || has_fused_norm(a) || a.bias_map ||
      a.epilogue != SCFLOW_EPI_PLAIN || flow_ch <= 0 || flow_ch % 32 || a.cout % 32 ||
      a.cout <= flow_ch || (a.w != 32 && a.w != 64) || a.h % 4)
    return SCFLOW_EUNSUPPORTED;
  const long long M = (long long)a.n * a.h * a.w;
  const int nbf = flow_ch / 32, nbm = (a.cout - flow_ch) / 32;
  if (!zp || zp_bytes < xhead_pred_ws_bytes(M, nbf, nbm) || !pw || !fo || !mo || fso < 2 || mso < 1)
    return SCFLOW_EINVAL;
  if (!aligned16(zp) || !aligned16(pw)) return SCFLOW_EALIGN;
  Wino4Params p;
  dim3 grid;
  int e = wino4_prepare(a, st, p, grid);
  if (e) return e;
  p.pw = pw;
  p.zp = zp;
  p.pnbf = nbf;
  e = wino4_depth2(p, grid) ? launch_wino4_pred_gemm<2>(p, grid, st) : launch_wino4_pred_gemm<1>(p, grid, st);
  if (e) return e;
  if (a.w == 32) {
    constexpr int R = XH_R32;
    const unsigned blocks32 = (unsigned)(a.n * (a.h / R));
    xhead_pred_sum_kernel<32, R><<<blocks32, 256, 0, st>>>(zp, nbf, nbm, a.h, M, fb, mb, fact, mact, fo, fso, mo, mso);
    return scflow_launch_status();
  }
  const unsigned blocks = (unsigned)(a.n * (a.h / 2));
  xhead_pred_sum_kernel<64, 2><<<blocks, 256, 0, st>>>(zp, nbf, nbm, a.h, M, fb, mb, fact, mact, fo, fso, mo, mso);
  return scflow_launch_status();
}
