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
//  * wgrad_kernel — the conv weight (and bias) gradient as an implicit GEMM on
//    v_mfma_f32_32x32x2_f32 with the PIXELS as the reduction dimension:
//        dW[co][ty][tx][ci] = Σ_p dY[p][co] · X[pix(p) + (ty, tx)][ci]
//    A workgroup owns a 64 (co) × 64 (ci) tile for ALL kh·kw taps (4 waves, each 32 co × 32 ci
//    × taps accumulators) and a contiguous run of pixel chunks (split-K over the grid's y).
//    Per chunk (TR×TC output pixels) it stages dY[chunk][64 co] and the input HALO of the chunk
//    ((TR−1)·s+kh rows × (TC−1)·s+kw cols × 64 ci) in LDS once; every tap then reads its
//    shifted window out of the same halo — no im2col matrix in HBM.  k = 2 pixels per MFMA
//    (lane half hh supplies pixel p0+hh): A = dY_lds[p][co] and B = halo[p+tap][ci] are both
//    32 consecutive floats per half-wave (ds_read_b32, conflict-free).  Partial sums go to a
//    per-split slab; wgrad_reduce_kernel sums the slabs in a fixed order (deterministic) and
//    writes dW in the torch [cout][cin][kh][kw] layout, plus db = Σ_p dY when asked.  Two input
//    sources = a channel concat without a copy (GRU cat[h, x]).
#include "common.h"

namespace {

// column order (ty, tx, c), or with cmajor (c, ty, tx) — a conv weight's own [cout][cin][kh][kw]
// order, so the weight-gradient GEMM writes (or accumulates into) dW in place.  Index maths in
// 32 bits when the matrix allows (I = unsigned): 64-bit division is a long software sequence.
template <typename I>
__global__ void im2col_kernel(const float* __restrict__ x, int sx, float* __restrict__ cols, int h,
                              int w, int cin, int kh, int kw, int stride, int ph, int pw, int oh,
                              int ow, long long total_vec, int vec, int cmajor) {
  const I K = (I)(kh * kw * cin);
  const I kv = K / (I)vec;
  const I taps = (I)(kh * kw);
  for (I i = (I)blockIdx.x * 256 + threadIdx.x; i < (I)total_vec; i += (I)gridDim.x * 256) {
    const I p = i / kv;
    const int k = (int)(i - p * kv) * vec;
    const int tap = cmajor ? (int)((I)k % taps) : k / cin, c = cmajor ? (int)((I)k / taps) : k % cin;
    const int ty = tap / kw, tx = tap - ty * kw;
    const I t = p / (I)ow;
    const int ox = (int)(p - t * (I)ow);
    const I img = t / (I)oh;
    const int oy = (int)(t - img * (I)oh);
    const int iy = oy * stride - ph + ty, ix = ox * stride - pw + tx;
    const bool ok = iy >= 0 && iy < h && ix >= 0 && ix < w;
    const float* src = x + ((size_t)((size_t)img * h + iy) * w + ix) * sx + c;
    float* dst = cols + (size_t)p * K + k;
    if (vec == 4) {
      floatx4 v = {0.f, 0.f, 0.f, 0.f};
      if (ok) v = *(const floatx4*)src;
      *(floatx4*)dst = v;
    } else {
      *dst = ok ? *src : 0.f;
    }
  }
}

// col2im: the adjoint of im2col — dx[n][iy][ix][c] = Σ over the taps (ty, tx) whose output pixel
// oy = (iy + ph − ty)/s, ox = (ix + pw − tx)/s is integral and inside the output grid of
// cols[(n, oy, ox)][(ty·kw + tx)·cin + c].  A gather (no atomics, fixed order): the strided
// conv's dX as cols = dY·Wmat (one GEMM with exactly the needed products) + this.
template <typename I>
__global__ void col2im_kernel(const float* __restrict__ cols, float* __restrict__ dx, int sdx,
                              int h, int w, int cin, int kh, int kw, int stride, int ph, int pw,
                              int oh, int ow, long long total_vec, int vec) {
  const int K = kh * kw * cin;
  const I cv = (I)(cin / vec);
  for (I i = (I)blockIdx.x * 256 + threadIdx.x; i < (I)total_vec; i += (I)gridDim.x * 256) {
    const I pix = i / cv;
    const int c = (int)(i - pix * cv) * vec;
    const I t = pix / (I)w;
    const int ix = (int)(pix - t * (I)w);
    const int img = (int)(t / (I)h);
    const int iy = (int)(t - (I)img * (I)h);
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int ty = 0; ty < kh; ++ty) {
      const int ny = iy + ph - ty;
      if (ny < 0 || ny % stride) continue;
      const int oy = ny / stride;
      if (oy >= oh) continue;
      for (int tx = 0; tx < kw; ++tx) {
        const int nx = ix + pw - tx;
        if (nx < 0 || nx % stride) continue;
        const int ox = nx / stride;
        if (ox >= ow) continue;
        const float* src = cols + ((size_t)(img * oh + oy) * ow + ox) * K + (ty * kw + tx) * cin + c;
        if (vec == 4) {
          const floatx4 v = *(const floatx4*)src;
          acc[0] += v[0]; acc[1] += v[1]; acc[2] += v[2]; acc[3] += v[3];
        } else {
          acc[0] += *src;
        }
      }
    }
    float* dst = dx + (size_t)pix * sdx + c;
    if (vec == 4)
      *(floatx4*)dst = acc;
    else
      *dst = acc[0];
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

// thread = (level, image, pixel): the whole D×D sample grid of one (pixel, level) map.  The grid
// is separable — x taps depend on a only, y taps on b only — and the taps of sample column a
// fall in window columns a..a+2 (rows likewise), so the (D+2)² window of the map accumulates in
// registers (static indices after unrolling) and is written back with plain read-modify-writes:
// this thread is the map's only writer.  No atomics, and a deterministic summation order.
template <int R>
__global__ __launch_bounds__(256) void corr_lookup_bwd_win_kernel(
    const float* __restrict__ dout, int out_layout, int out_stride, const float* __restrict__ flow,
    int flow_layout, float* __restrict__ dpyr, int N, int H, int W, int L, long long total) {
#pragma clang fp contract(off)
  constexpr int r = R;
  constexpr int D = 2 * R + 1;
  const int P = H * W;
  const long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  const int p = (int)(idx % P);
  long long t = idx / P;
  const int n = (int)(t % N);
  const int lvl = (int)(t / N);
  if (idx >= total) return;
  // (staging the block's gradient rows through LDS for coalesced loads measured slower: 98 vs
  // 74 µs at configs[3]'s training shapes — one block per CU then waits on the whole stage)
  const float* g = out_layout == SCFLOW_LAYOUT_NHWC
                       ? dout + ((size_t)n * P + p) * out_stride + lvl * D * D
                       : dout + ((size_t)n * L * D * D + lvl * D * D) * P + p;
  const int gstep = out_layout == SCFLOW_LAYOUT_NHWC ? 1 : P;
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
  if (!(fabsf(cx) < 1e6f && fabsf(cy) < 1e6f)) return;  // every tap outside the map
  // sample column a: west tap xw(a) = x0 + a + ox[a] with ox ∈ {0, 1}, east tap one further;
  // x0 = rint(cx − r) − 1 (and the same in y).  Checked exhaustively over integer, half- and
  // quarter-integer and random coordinates; a thread outside it takes the per-tap path.
  const int x0 = (int)rintf(cx + (float)(-r)) - 1;
  const int y0 = (int)rintf(cy + (float)(-r)) - 1;
  float wxw[D], wxe[D], wyn[D], wys[D];
  int ox[D], oy[D];
  bool regular = true;
#pragma unroll
  for (int k = 0; k < D; ++k) {
    const float ix = unnorm_coord_b(cx + (float)(k - r), Wl);
    const float ix_w = floorf(ix);
    wxw[k] = (ix_w + 1.f) - ix;
    wxe[k] = ix - ix_w;
    ox[k] = (int)ix_w - x0 - k;
    const float iy = unnorm_coord_b(cy + (float)(k - r), Hl);
    const float iy_n = floorf(iy);
    wyn[k] = (iy_n + 1.f) - iy;
    wys[k] = iy - iy_n;
    oy[k] = (int)iy_n - y0 - k;
    regular = regular && (unsigned)ox[k] <= 1u && (unsigned)oy[k] <= 1u;
  }
  if (!regular) {
    for (int a = 0; a < D; ++a) {
      const int xw = x0 + a + ox[a];
      for (int b = 0; b < D; ++b) {
        const float gv = g[(size_t)(a * D + b) * gstep];
        const int yn = y0 + b + oy[b];
        tap_add(m, xw, yn, Wl, Hl, gv * (wxw[a] * wyn[b]));
        tap_add(m, xw + 1, yn, Wl, Hl, gv * (wxe[a] * wyn[b]));
        tap_add(m, xw, yn + 1, Wl, Hl, gv * (wxw[a] * wys[b]));
        tap_add(m, xw + 1, yn + 1, Wl, Hl, gv * (wxe[a] * wys[b]));
      }
    }
    return;
  }
  // per column a the x weights over window columns a, a+1, a+2 (and y likewise)
  float ux0[D], ux1[D], ux2[D];
#pragma unroll
  for (int a = 0; a < D; ++a) {
    ux0[a] = ox[a] ? 0.f : wxw[a];
    ux1[a] = ox[a] ? wxw[a] : wxe[a];
    ux2[a] = ox[a] ? wxe[a] : 0.f;
  }
  constexpr int WN = D + 2;
  unsigned inb = 0;  // bit i: window column x0 + i inside the map
#pragma unroll
  for (int i = 0; i < WN; ++i) inb |= (x0 + i >= 0 && x0 + i < Wl) ? 1u << i : 0u;
  // the window starts from the map's current values (all loads before any store: with the row
  // pitch unknown to the compiler, interleaved read-modify-writes would serialise on aliasing)
  float win[WN][WN];
#pragma unroll
  for (int j = 0; j < WN; ++j) {
    const int yy = y0 + j;
    const bool rin = yy >= 0 && yy < Hl;
    const float* row = m + (ptrdiff_t)yy * Wl + x0;
#pragma unroll
    for (int i = 0; i < WN; ++i) win[j][i] = (rin && (inb >> i & 1u)) ? row[i] : 0.f;
  }
  // separable accumulation: row b of samples → a window-wide vector, spread over 3 window rows
#pragma unroll
  for (int b = 0; b < D; ++b) {
    float v[WN];
#pragma unroll
    for (int i = 0; i < WN; ++i) v[i] = 0.f;
#pragma unroll
    for (int a = 0; a < D; ++a) {
      const float gv = g[(size_t)(a * D + b) * gstep];
      v[a] += gv * ux0[a];
      v[a + 1] += gv * ux1[a];
      v[a + 2] += gv * ux2[a];
    }
    const float u0 = oy[b] ? 0.f : wyn[b];
    const float u1 = oy[b] ? wyn[b] : wys[b];
    const float u2 = oy[b] ? wys[b] : 0.f;
#pragma unroll
    for (int i = 0; i < WN; ++i) {
      win[b][i] += u0 * v[i];
      win[b + 1][i] += u1 * v[i];
      win[b + 2][i] += u2 * v[i];
    }
  }
#pragma unroll
  for (int j = 0; j < WN; ++j) {
    const int yy = y0 + j;
    if (yy < 0 || yy >= Hl) continue;
    float* row = m + (ptrdiff_t)yy * Wl + x0;
#pragma unroll
    for (int i = 0; i < WN; ++i)
      if (inb >> i & 1u) row[i] = win[j][i];
  }
}

// ------------------------------------------------------------------------------ wgrad
// equally shaped segments summed by one launch (scflow_conv_wgrad_batched): segment s holds
// images [s·nimg, (s+1)·nimg) of the walk, at its own dY / input bases (one segment: the args')
constexpr int WG_MAXSEG = 8;
struct WgSegs {
  int nimg;
  const float* dy[WG_MAXSEG];
  const float* src0[WG_MAXSEG];
  const float* src1[WG_MAXSEG];
};

// segment s's pointer, selected with uniform compares (no dynamic kernarg indexing)
__device__ __forceinline__ const float* wg_pick(const float* const (&arr)[WG_MAXSEG], int s) {
  const float* p = arr[0];
#pragma unroll
  for (int i = 1; i < WG_MAXSEG; ++i) p = s == i ? arr[i] : p;
  return p;
}

inline void wg_single_seg(const scflow_wgrad_args& a, WgSegs* s) {
  s->nimg = a.n;
  s->dy[0] = a.dy;
  s->src0[0] = a.src0;
  s->src1[0] = a.src1;
}

struct WgParams {
  scflow_wgrad_args a;
  int oh, ow, tr, tc, ltc, hr, hc, cp, nchunks, cps, co_tiles, copad, cinp, wco;
  WgSegs sg;
};

constexpr int WT = 64;  // ci tile of a workgroup (and the co tile of the 4-wave variant)

// float4 per thread needed to stage the largest halo a (KH, KW, S) launch can have (NT threads)
constexpr int wg_nx(int kh, int kw, int s, int nt) {
  const int cp = s == 1 ? 64 : 32;
  int best = 0;
  for (int tc = 2; tc <= 32; tc *= 2) {
    const int tr = cp / tc;
    const int hr = (tr - 1) * s + kh, hc = (tc - 1) * s + kw;
    const int v = (hr * hc * (WT / 4) + nt - 1) / nt;
    if (v > best) best = v;
  }
  return best;
}

// WCO = output channels per workgroup (64: 2 co × 2 ci waves of 32×32; 128: 4 co × 2 ci).
// KS = 2: a second set of waves takes every other pair of k-steps of each chunk (two waves per
// SIMD, so one wave's LDS reads and chunk barriers hide under the other's MFMAs); the two sets'
// accumulators are summed through LDS before the slab write.
template <int KH, int KW, int S, bool VEC, bool DB, int WCO = 64, int KS = 1>
__global__ __launch_bounds__(WCO * 4 * KS, (KH * KW >= 9 || WCO * KS > 64) ? 1 : 2) void wgrad_kernel(
    WgParams P, float* __restrict__ slab, float* __restrict__ bslab) {
  constexpr int NT = WCO * 4 * KS; // threads
  constexpr int CQ = WCO / 4;      // float4 per dY pixel row of the tile
  constexpr int NWCO = WCO / 32;   // waves along co
  constexpr int TAPS = KH * KW;
  constexpr int NX = VEC ? wg_nx(KH, KW, S, NT) : 1;
  constexpr int ND = VEC ? (S == 1 ? 64 : 32) * CQ / NT : 1;
  extern __shared__ float smem[];
  const scflow_wgrad_args& a = P.a;
  float* Ds = smem;                 // [cp][WCO] dY chunk, then [hr*hc][64] input halo; ×2 (float4)
  float* Xs = smem + P.cp * WCO;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 31, hh = lane >> 5, wq = wave % (2 * NWCO);
  const int wco = wq % NWCO, wci = wq / NWCO, ks = wave / (2 * NWCO);
  const int co_t = blockIdx.x % P.co_tiles, ci_t = blockIdx.x / P.co_tiles;
  const int co0 = co_t * WCO, ci0 = ci_t * WT;
  const int cin = a.cin0 + a.cin1;
  const int c_begin = blockIdx.y * P.cps;
  const int c_end = min(P.nchunks, c_begin + P.cps);
  const int tiles_c = P.ow / P.tc, tiles_r = P.oh / P.tr;
  const bool do_bias = bslab != nullptr && ci_t == 0;
  const int nh = P.hr * P.hc;

  floatx16 acc[TAPS];
#pragma unroll
  for (int t = 0; t < TAPS; ++t)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[t][e] = 0.f;
  float bsum = 0.f;

  // global → register prefetch of one chunk (float4 path)
  floatx4 rd[ND], rx[NX];
  auto chunk_origin = [&](int ch, int* img, int* oy0, int* ox0) {
    *img = ch / (tiles_r * tiles_c);
    const int rem = ch - *img * tiles_r * tiles_c;
    *oy0 = (rem / tiles_c) * P.tr;
    *ox0 = (rem % tiles_c) * P.tc;
  };
  auto gload = [&](int ch) {
    int img, oy0, ox0;
    chunk_origin(ch, &img, &oy0, &ox0);
    const int seg = img / P.sg.nimg;  // workgroup-uniform
    img -= seg * P.sg.nimg;
    const float* dyp = P.sg.dy[seg];
    const float* s0p = P.sg.src0[seg];
    const float* s1p = P.sg.src1[seg];
#pragma unroll
    for (int j = 0; j < ND; ++j) {
      const int idx = tid + NT * j;
      const int p = idx / CQ, co = co0 + 4 * (idx % CQ);
      floatx4 v = {0.f, 0.f, 0.f, 0.f};
      if (p < P.cp && co < a.cout) {
        const size_t m = ((size_t)img * P.oh + oy0 + (p >> P.ltc)) * P.ow + ox0 + (p & (P.tc - 1));
        v = *(const floatx4*)(dyp + m * a.sdy + co);
      }
      rd[j] = v;
    }
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      const int idx = tid + NT * j;
      const int hp = idx >> 4, c = ci0 + 4 * (idx & 15);
      floatx4 v = {0.f, 0.f, 0.f, 0.f};
      if (hp < nh && c < cin) {
        const int hy = hp / P.hc, hx = hp - hy * P.hc;
        const int iy = oy0 * S - a.ph + hy, ix = ox0 * S - a.pw + hx;
        if (iy >= 0 && iy < a.h && ix >= 0 && ix < a.w) {
          const size_t pix = ((size_t)img * a.h + iy) * a.w + ix;
          v = c < a.cin0 ? *(const floatx4*)(s0p + pix * a.s0 + c)
                         : *(const floatx4*)(s1p + pix * a.s1 + (c - a.cin0));
        }
      }
      rx[j] = v;
    }
  };
  auto lstore = [&](int buf = 0) {
    float* D = Ds + buf * (P.cp * WCO + nh * WT);
    float* X = D + P.cp * WCO;
#pragma unroll
    for (int j = 0; j < ND; ++j) {
      const int idx = tid + NT * j;
      if (idx < P.cp * CQ) *(floatx4*)(D + (idx / CQ) * WCO + 4 * (idx % CQ)) = rd[j];
    }
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      const int idx = tid + NT * j;
      if (idx < nh * (WT / 4)) *(floatx4*)(X + (idx >> 4) * WT + 4 * (idx & 15)) = rx[j];
    }
  };
  auto stage_scalar = [&](int ch) {  // cin or cout not a multiple of 4: element-wise staging
    int img, oy0, ox0;
    chunk_origin(ch, &img, &oy0, &ox0);
    const int seg = img / P.sg.nimg;
    img -= seg * P.sg.nimg;
    const float* dyp = P.sg.dy[seg];
    const float* s0p = P.sg.src0[seg];
    const float* s1p = P.sg.src1[seg];
    for (int idx = tid; idx < P.cp * WCO; idx += NT) {
      const int p = idx / WCO, co = co0 + (idx % WCO);
      const size_t m = ((size_t)img * P.oh + oy0 + (p >> P.ltc)) * P.ow + ox0 + (p & (P.tc - 1));
      Ds[idx] = co < a.cout ? dyp[m * a.sdy + co] : 0.f;
    }
    for (int idx = tid; idx < nh * WT; idx += NT) {
      const int hp = idx >> 6, c = ci0 + (idx & 63);
      const int hy = hp / P.hc, hx = hp - hy * P.hc;
      const int iy = oy0 * S - a.ph + hy, ix = ox0 * S - a.pw + hx;
      float v = 0.f;
      if (iy >= 0 && iy < a.h && ix >= 0 && ix < a.w && c < cin) {
        const size_t pix = ((size_t)img * a.h + iy) * a.w + ix;
        v = c < a.cin0 ? s0p[pix * a.s0 + c] : s1p[pix * a.s1 + (c - a.cin0)];
      }
      Xs[idx] = v;
    }
  };

  // float4 path, DB: LDS double buffer — chunk ch+1 is written into the other buffer from the
  // prefetch registers after this chunk's MFMAs have been issued; one barrier per chunk.
  // float4 path, !DB: one buffer; the next chunk's global loads are in flight (registers)
  // during this chunk's MFMAs.  Scalar path: one buffer, staged in place.
  const int bufsz = P.cp * WCO + nh * WT;
  if (VEC && c_begin < c_end) {
    gload(c_begin);
    if (DB) {
      lstore();
      __syncthreads();
      if (c_begin + 1 < c_end) gload(c_begin + 1);
    }
  }
  for (int ch = c_begin; ch < c_end; ++ch) {
    const int cur = (VEC && DB) ? ((ch - c_begin) & 1) : 0;
    float* Dc = Ds + cur * bufsz;
    float* Xc = Dc + P.cp * WCO;
    if (!VEC) {
      __syncthreads();
      stage_scalar(ch);
      __syncthreads();
    } else if (!DB) {
      __syncthreads();
      lstore();
      __syncthreads();
      if (ch + 1 < c_end) gload(ch + 1);
    }
    if (do_bias)  // every thread: one channel (tid % WCO), every (NT / WCO)-th pixel
      for (int p = tid / WCO; p < P.cp; p += NT / WCO) bsum += Dc[p * WCO + (tid % WCO)];
    const float* Da = Dc + wco * 32 + li;
    const float* Xb = Xc + wci * 32 + li;
    // software pipeline: the operands of k-step p0+2 are read from LDS before the MFMAs of
    // k-step p0 issue, so the LDS latency hides under TAPS matrix ops even at 1 wave / SIMD
    float av, bv[TAPS];
    auto ldk = [&](int p0, float& a_, float* b_) {
      const int pix = p0 + hh;
      const int r = pix >> P.ltc, c = pix & (P.tc - 1);
      a_ = Da[pix * WCO];
      const float* xb = Xb + (r * S * P.hc + c * S) * WT;
#pragma unroll
      for (int ty = 0; ty < KH; ++ty)
#pragma unroll
        for (int tx = 0; tx < KW; ++tx) b_[ty * KW + tx] = xb[(ty * P.hc + tx) * WT];
    };
    // two register sets, two k-steps per trip (cp % 4 == 0): set 1's reads are issued before
    // set 0's MFMAs and vice versa, with no copies between the sets
    float a1, b1[TAPS];
    ldk(4 * ks, av, bv);
    for (int p0 = 4 * ks; p0 < P.cp; p0 += 4 * KS) {
      ldk(p0 + 2, a1, b1);
#pragma unroll
      for (int t = 0; t < TAPS; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv[t], acc[t], 0, 0, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, TAPS + 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, TAPS, 0);
      ldk(p0 + 4 * KS < P.cp ? p0 + 4 * KS : p0, av, bv);
#pragma unroll
      for (int t = 0; t < TAPS; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1[t], acc[t], 0, 0, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, TAPS + 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, TAPS, 0);
    }
    if (VEC && DB && ch + 1 < c_end) {
      lstore(cur ^ 1);
      __syncthreads();
      if (ch + 2 < c_end) gload(ch + 2);
    }
  }
  if constexpr (KS == 2) {  // the second wave set's accumulators onto the first's, tap by tap
    constexpr int HALF = NT / 2;
#pragma unroll
    for (int t = 0; t < TAPS; ++t) {
      __syncthreads();
      if (ks == 1)
#pragma unroll
        for (int r = 0; r < 16; ++r) smem[r * HALF + (tid - HALF)] = acc[t][r];
      __syncthreads();
      if (ks == 0)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t][r] += smem[r * HALF + tid];
    }
  }
  // partial slab [split][copad][TAPS][cinp]; C/D layout: col = lane&31, row = (r&3)+8(r>>2)+4hh
  float* sl = slab + (size_t)blockIdx.y * P.copad * TAPS * P.cinp;
  const int ci = ci0 + wci * 32 + li;
  if (ks == 0)
#pragma unroll
    for (int t = 0; t < TAPS; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = co0 + wco * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
        sl[((size_t)co * TAPS + t) * P.cinp + ci] = acc[t][r];
      }
  if (do_bias) {
    constexpr int NG = NT / WCO;  // partial sums per channel
    __syncthreads();
    smem[tid] = bsum;
    __syncthreads();
    if (tid < WCO) {
      float b = 0.f;
#pragma unroll
      for (int g = 0; g < NG; ++g) b += smem[tid + g * WCO];
      bslab[(size_t)blockIdx.y * P.copad + co0 + tid] = b;
    }
  }
}

// Σ over the splits, fixed order.  Workgroup = 256/G consecutive slab entries (a run of one
// (co, tap) row's ci) × G lanes of partial sums (G = 2^lg ≤ 16 ≈ splits/4: lane k sums splits
// k, k+G, …, two loads in flight), then the G partials in order through LDS.  The bias slab
// rides along as the last, row-less workgroups.
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(
    const float* __restrict__ slab, const float* __restrict__ bslab, float* __restrict__ dw,
    float* __restrict__ db, int splits, int cout, int cin, int taps, int copad, int cinp,
    int accumulate, int lg) {
  __shared__ float part[256];
  const int G = 1 << lg, OPB = 256 >> lg;
  const int o = threadIdx.x & (OPB - 1), k = threadIdx.x >> (8 - lg);
  const long long wtot = (long long)cout * taps * cinp;
  const long long nw = (wtot + OPB - 1) / OPB;  // weight blocks; then bias blocks
  const bool wblk = blockIdx.x < nw;
  const size_t sstride = (size_t)copad * taps * cinp;
  long long i;
  const float* src;
  size_t step;
  bool valid;
  if (wblk) {
    i = (long long)blockIdx.x * OPB + o;  // = row·cinp + ci
    src = slab + i;
    step = sstride;
    valid = i < wtot && (int)(i % cinp) < cin;
  } else {
    i = (long long)(blockIdx.x - nw) * OPB + o;  // channel
    src = bslab + i;
    step = (size_t)copad;
    valid = i < cout;
  }
  float s0 = 0.f, s1 = 0.f;
  if (valid) {
    int b = k;
    for (; b + G < splits; b += 2 * G) {
      s0 += src[b * step];
      s1 += src[(b + G) * step];
    }
    if (b < splits) s0 += src[b * step];
  }
  part[threadIdx.x] = s0 + s1;
  __syncthreads();
  if (k == 0 && valid) {
    float s = 0.f;
    for (int j = 0; j < G; ++j) s += part[j * OPB + o];
    if (wblk) {
      const int row = (int)(i / cinp), ci = (int)(i % cinp);
      const int co = row / taps, t = row % taps;
      float* d = dw + ((size_t)co * cin + ci) * taps + t;
      *d = accumulate ? *d + s : s;
    } else {
      db[i] = accumulate ? db[i] + s : s;
    }
  }
}

#include "wgrad_wino.h"
#include "wgrad_wino5.h"
#include "wgrad_1x1.h"

bool wgrad_geometry(const scflow_wgrad_args& a, WgParams* P, int* splits) {
  if (a.stride != 1 && a.stride != 2) return false;
  const bool shape_ok = (a.kh == 1 && a.kw == 1) || (a.kh == 3 && a.kw == 3) ||
                        (a.stride == 1 && ((a.kh == 1 && a.kw == 5) || (a.kh == 5 && a.kw == 1)));
  if (!shape_ok) return false;
  P->a = a;
  P->oh = (a.h + 2 * a.ph - a.kh) / a.stride + 1;
  P->ow = (a.w + 2 * a.pw - a.kw) / a.stride + 1;
  if (P->oh <= 0 || P->ow <= 0) return false;
  const int tcmax = a.stride == 1 ? 32 : 16, cpmax = a.stride == 1 ? 64 : 32;
  P->tc = P->ow < tcmax ? P->ow : tcmax;
  if (P->tc & (P->tc - 1)) return false;  // power of two
  P->ltc = 0;
  while ((1 << P->ltc) < P->tc) ++P->ltc;
  P->tr = cpmax / P->tc < P->oh ? cpmax / P->tc : P->oh;
  if (P->ow % P->tc || P->oh % P->tr) return false;
  P->cp = P->tr * P->tc;
  if (P->cp & 3) return false;  // two k-steps (4 pixels) per trip of the MFMA loop
  P->hr = (P->tr - 1) * a.stride + a.kh;
  P->hc = (P->tc - 1) * a.stride + a.kw;
  P->nchunks = a.n * (P->oh / P->tr) * (P->ow / P->tc);
  P->co_tiles = (a.cout + WT - 1) / WT;
  const int cin = a.cin0 + a.cin1;
  const int ci_tiles = (cin + WT - 1) / WT;
  P->copad = P->co_tiles * WT;
  P->cinp = ci_tiles * WT;
  // split the pixel reduction until the grid fills the CUs once at the kernel's occupancy
  const int tiles = P->co_tiles * ci_tiles;
  const int occ = a.kh * a.kw >= 9 ? 1 : 2;  // the kernel's resident workgroups per CU
  int want = (occ * device_cus() + tiles - 1) / tiles;
  static const int forced = [] {  // SCFLOW_WGRAD_SPLITS=k forces k splits (tuning only)
    const char* e = getenv("SCFLOW_WGRAD_SPLITS");
    return e ? atoi(e) : 0;
  }();
  if (forced > 0) {
    want = forced < P->nchunks ? forced : P->nchunks;
    P->cps = (P->nchunks + want - 1) / want;
    *splits = (P->nchunks + P->cps - 1) / P->cps;
    return true;
  }
  // ≥ 8 chunks per split, unless that leaves CUs idle: then down to one chunk per split until
  // every CU has a workgroup, while the partial slabs (splits × the padded weight size, written
  // and read once more by the reduction) stay under 8 Mi floats
  long long maxs = P->nchunks / 8 > 0 ? P->nchunks / 8 : 1;
  if ((long long)tiles * maxs < device_cus()) {
    const long long per_split = (long long)P->copad * a.kh * a.kw * P->cinp;
    long long m = (device_cus() + tiles - 1) / tiles;
    if (m > P->nchunks) m = P->nchunks;
    if (m > (8ll << 20) / per_split) m = (8ll << 20) / per_split;
    if (m > maxs) maxs = m;
  }
  if (want > maxs) want = (int)maxs;
  if (want < 1) want = 1;
  P->cps = (P->nchunks + want - 1) / want;
  *splits = (P->nchunks + P->cps - 1) / P->cps;
  return true;
}

// ---------------------------------------------------------------------------------------------
// Thin weight gradients: one side of the conv at most 4 channels (the flow / mask predictors'
// 256→2 / 256→1, the mask encoder's 1→64 input; kernels up to 5×5).  On the 64×64 MFMA
// tile such a shape wastes ≥ 16/17 of every matrix op and its grid is a handful of workgroups;
// here it is a plain fp32 reduction over the pixels.  The WIDE side (C ≤ 256 channels, C % 4
// == 0) is spread over the lanes as float4 groups g; the lanes that share a group are pixel
// streams st.  A workgroup owns a run of ppb output pixels and one kernel row ty (grid.y), and
// keeps T (thin channels) × KW (taps of the row) × 4 (the float4) fp32 accumulators per lane:
//   THIN_CO (cout ≤ T): acc[co][tx][e] += dy[p][co]       · x[p + (ty, tx)][4g + e]
//   !THIN_CO (cin ≤ T): acc[ci][tx][e] += dy[p][4g + e]   · x[p + (ty, tx)][ci]
// The streams are summed through LDS in a fixed order and each workgroup writes its partial
// dw (torch layout) to a slab row; wthin_reduce_kernel sums the rows in a fixed order.
// Segments (scflow_conv_wgrad_batched): grid.z = segment, each with its own dY / input bases
// and nbp pixel runs of its nimg images; slab row = z·nbp + x.
struct WtParams {
  scflow_wgrad_args a;
  int oh, ow, cin, C, G, lg2, ppb, nbp, thin_co;
  int nseg, nimg;  // segments, images per segment
  WgSegs sg;
};

// nseg = 0: the workspace query (the whole walk as one segment, rows for any segment count)
bool wthin_geometry(const scflow_wgrad_args& a, WtParams* P, int nseg = 1) {
  static const bool off = [] {
    const char* e = getenv("SCFLOW_WGRAD_THIN");
    return e && e[0] == '0';
  }();
  if (off) return false;
  const int cin = a.cin0 + a.cin1;
  // 7×7 (the stem, the flow encoders' 2→128) stays on im2col + GEMM: measured faster there
  // (batched over the decoder's 8 uses too: 246 µs on this kernel, where the 14 scalar input
  // loads per pixel and tap row are latency-bound, vs one concatenated GEMM)
  if (a.kw != 1 && a.kw != 3 && a.kw != 5) return false;
  if (a.kh < 1 || a.kh > 5 || a.stride < 1 || a.stride > 2) return false;
  const bool thin_co = a.cout <= 4 && cin % 4 == 0 && a.cin0 % 4 == 0 && cin <= 256 &&
                       a.s0 % 4 == 0 && aligned16(a.src0) &&
                       (a.cin1 == 0 || (a.s1 % 4 == 0 && aligned16(a.src1)));
  const bool thin_ci = !thin_co && cin <= 4 && a.cin1 == 0 && a.cout % 4 == 0 && a.cout <= 256 &&
                       a.sdy % 4 == 0 && aligned16(a.dy);
  if (!thin_co && !thin_ci) return false;
  P->a = a;
  P->cin = cin;
  P->oh = (a.h + 2 * a.ph - a.kh) / a.stride + 1;
  P->ow = (a.w + 2 * a.pw - a.kw) / a.stride + 1;
  if (P->oh <= 0 || P->ow <= 0) return false;
  P->thin_co = thin_co;
  P->C = thin_co ? cin : a.cout;
  P->G = P->C / 4;
  P->lg2 = 0;
  while ((1 << P->lg2) < P->G) ++P->lg2;
  const long long pix = (long long)a.n * P->oh * P->ow;
  // ≥ 64 pixels per workgroup, at most 512 workgroups per kernel row (the slab rows) + one per
  // extra segment
  long long ppb = (pix + 511) / 512;
  if (ppb < 64) ppb = 64;
  P->ppb = (int)ppb;
  const int ns = nseg < 1 ? 1 : nseg;
  P->nseg = ns;
  P->nimg = a.n / ns;
  const long long spix = (long long)P->nimg * P->oh * P->ow;
  P->nbp = (int)((spix + ppb - 1) / ppb);
  if (nseg == 0) P->nbp += WG_MAXSEG;  // the query: ns·⌈spix/ppb⌉ ≤ ⌈pix/ppb⌉ + ns
  return true;
}

template <int T, int KW, bool THIN_CO>
__global__ __launch_bounds__(256) void wgrad_thin_kernel(WtParams P, float* __restrict__ slab,
                                                         float* __restrict__ bslab) {
  constexpr int NA = T * KW * 4 + 4;  // accumulators + 4 bias partials
  __shared__ float red[256][17];
  const scflow_wgrad_args& a = P.a;
  const int tid = threadIdx.x;
  const int G2 = 1 << P.lg2, S = 256 >> P.lg2;
  const int g = tid & (G2 - 1), st = tid >> P.lg2;
  const bool act = g < P.G;
  const int ty = blockIdx.y;
  const long long ohw = (long long)P.oh * P.ow;
  const long long pix = P.nimg * ohw;
  const long long pb0 = (long long)blockIdx.x * P.ppb;
  const long long pb1 = pb0 + P.ppb < pix ? pb0 + P.ppb : pix;
  const float* dyp = wg_pick(P.sg.dy, blockIdx.z);
  const float* s0p = wg_pick(P.sg.src0, blockIdx.z);
  const float* s1p = wg_pick(P.sg.src1, blockIdx.z);
  const int tn = THIN_CO ? a.cout : P.cin;  // thin channels actually present
  float acc[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) acc[i] = 0.f;
  const int c4 = 4 * g;
  if (act) {
#pragma unroll 2
    for (long long p = pb0 + st; p < pb1; p += S) {
      const int img = (int)(p / ohw);
      const int rem = (int)(p - img * ohw);
      const int oy = rem / P.ow, ox = rem - oy * P.ow;
      const int iy = oy * a.stride - a.ph + ty;
      const bool rok = iy >= 0 && iy < a.h;
      const size_t rowpix = ((size_t)img * a.h + iy) * a.w;
      if (THIN_CO) {
        float d[T];
#pragma unroll
        for (int t = 0; t < T; ++t) d[t] = t < tn ? dyp[p * a.sdy + t] : 0.f;
#pragma unroll
        for (int t = 0; t < T; ++t) acc[T * KW * 4 + t] += d[t];
#pragma unroll
        for (int tx = 0; tx < KW; ++tx) {
          const int ix = ox * a.stride - a.pw + tx;
          floatx4 v = {0.f, 0.f, 0.f, 0.f};
          if (rok && ix >= 0 && ix < a.w) {
            const size_t q = rowpix + ix;
            v = c4 < a.cin0 ? *(const floatx4*)(s0p + q * a.s0 + c4)
                            : *(const floatx4*)(s1p + q * a.s1 + (c4 - a.cin0));
          }
#pragma unroll
          for (int t = 0; t < T; ++t)
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[(t * KW + tx) * 4 + e] += d[t] * v[e];
        }
      } else {
        const floatx4 d = *(const floatx4*)(dyp + p * a.sdy + c4);
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[T * KW * 4 + e] += d[e];
#pragma unroll
        for (int tx = 0; tx < KW; ++tx) {
          const int ix = ox * a.stride - a.pw + tx;
          const bool ok = rok && ix >= 0 && ix < a.w;
          const size_t q = rowpix + ix;
#pragma unroll
          for (int t = 0; t < T; ++t) {
            const float xv = ok && t < tn ? s0p[q * a.s0 + t] : 0.f;
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[(t * KW + tx) * 4 + e] += d[e] * xv;
          }
        }
      }
    }
  }
  // Σ over the streams (fixed order), 16 accumulators per round; lanes st == 0 write the row
  const int taps = a.kh * a.kw;
  const size_t srow = (size_t)blockIdx.z * P.nbp + blockIdx.x;
  float* row = slab + srow * a.cout * P.cin * taps;
#pragma unroll
  for (int r0 = 0; r0 < NA; r0 += 16) {
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (r0 + j < NA) red[tid][j] = acc[r0 + j];
    __syncthreads();
    if (st == 0 && act) {
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int i = r0 + j;
        if (i >= NA) break;
        float s = 0.f;
        for (int k = 0; k < S; ++k) s += red[k * G2 + g][j];
        if (i < T * KW * 4) {
          const int e = i & 3, tx = (i >> 2) % KW, t = (i >> 2) / KW;
          if (t < tn) {
            const int co = THIN_CO ? t : c4 + e, ci = THIN_CO ? c4 + e : t;
            row[((size_t)co * P.cin + ci) * taps + ty * a.kw + tx] = s;
          }
        } else if (bslab && ty == 0) {
          const int e = i - T * KW * 4;
          if (THIN_CO) {
            if (g == 0 && e < tn) bslab[srow * a.cout + e] = s;
          } else {
            bslab[srow * a.cout + c4 + e] = s;
          }
        }
      }
    }
    __syncthreads();
  }
}

// dst[i] (+)= Σ_b slab[b][i], b in order: 16 outputs × 16 lanes of partial sums per workgroup
__global__ __launch_bounds__(256) void wthin_reduce_kernel(const float* __restrict__ slab, int nb,
                                                           long long total, float* __restrict__ dst,
                                                           int accumulate) {
  __shared__ float part[16][17];
  const int o = threadIdx.x & 15, k = threadIdx.x >> 4;
  const long long i = (long long)blockIdx.x * 16 + o;
  float s0 = 0.f, s1 = 0.f;
  if (i < total) {
    int b = k;
    for (; b + 16 < nb; b += 32) {
      s0 += slab[(size_t)b * total + i];
      s1 += slab[(size_t)(b + 16) * total + i];
    }
    if (b < nb) s0 += slab[(size_t)b * total + i];
  }
  part[k][o] = s0 + s1;
  __syncthreads();
  if (k == 0 && i < total) {
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) s += part[j][o];
    dst[i] = accumulate ? dst[i] + s : s;
  }
}

long long wthin_workspace(const WtParams& P) {
  const scflow_wgrad_args& a = P.a;
  const long long rows = (long long)P.nseg * P.nbp;
  return rows * a.cout * P.cin * a.kh * a.kw + rows * a.cout;
}

int wthin_launch(const WtParams& P, hipStream_t st) {
  const scflow_wgrad_args& a = P.a;
  if (a.workspace_floats < wthin_workspace(P)) return SCFLOW_EINVAL;
  const bool thin_co = P.thin_co != 0;
  const int tn = thin_co ? a.cout : P.cin;
  const int rows = P.nseg * P.nbp;
  float* slab = a.workspace;
  const long long total = (long long)a.cout * P.cin * a.kh * a.kw;
  float* bslab = a.db ? a.workspace + (size_t)rows * total : nullptr;
  const dim3 grid((unsigned)P.nbp, (unsigned)a.kh, (unsigned)P.nseg);
#define SCFLOW_WT(T_, KW_)                                                                   \
  if (a.kw == KW_ && tn <= T_) {                                                             \
    if (thin_co)                                                                             \
      wgrad_thin_kernel<T_, KW_, true><<<grid, 256, 0, st>>>(P, slab, bslab);                \
    else                                                                                     \
      wgrad_thin_kernel<T_, KW_, false><<<grid, 256, 0, st>>>(P, slab, bslab);               \
  } else
  SCFLOW_WT(1, 1) SCFLOW_WT(2, 1) SCFLOW_WT(4, 1)
  SCFLOW_WT(1, 3) SCFLOW_WT(2, 3) SCFLOW_WT(4, 3)
  SCFLOW_WT(1, 5) SCFLOW_WT(2, 5) SCFLOW_WT(4, 5)
  return SCFLOW_EUNSUPPORTED;
#undef SCFLOW_WT
  int rc = scflow_launch_status();
  if (rc != SCFLOW_OK) return rc;
  wthin_reduce_kernel<<<(unsigned)((total + 15) / 16), 256, 0, st>>>(slab, rows, total, a.dw,
                                                                     a.accumulate);
  if (a.db)
    wthin_reduce_kernel<<<(unsigned)((a.cout + 15) / 16), 256, 0, st>>>(bslab, rows, a.cout, a.db,
                                                                         a.accumulate);
  return scflow_launch_status();
}

// ---------------------------------------------------------------------------------------------
// InstanceNorm2d(affine=False) (+ ReLU) forward / backward for the training step's feature
// encoder (raft_encoder.py / resnet.py BasicBlock norms), channels-last x [n][hw][c], c % 4 == 0.
// Statistics: scflow_enc_stats + scflow_enc_norm_finalize (fp64 partials) → scale = rstd,
// shift = −mean·rstd, so x̂ = x·scale + shift.  Backward, with g = dy·[x̂ > 0 if relu]:
//   dx = rstd · (g − mean_hw(g) − x̂ · mean_hw(g·x̂))
// in three launches: fp64 partial sums of g and g·x̂ per (image, pixel chunk) in a fixed order,
// their finalisation per (image, channel), and the elementwise dx.

// y = act(x·scale + shift [+ res]) — res: the residual block's identity, added before the ReLU
// (raft_encoder.py BasicBlock: relu(norm2(conv2(·)) + x)), so the block's sum and ReLU cost no
// launches of their own
__global__ void in_apply_kernel(const float* __restrict__ x, const float* __restrict__ sc,
                                const float* __restrict__ sh, const float* __restrict__ res,
                                float* __restrict__ y, int hw, int c, int relu, long long total4) {
  const int c4 = c / 4;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total4; i += (long long)gridDim.x * 256) {
    const int cq = (int)(i % c4) * 4;
    const int img = (int)(i / c4 / hw);
    const size_t so = (size_t)img * c + cq;
    const floatx4 v = ((const floatx4*)x)[i];
    const floatx4 a = *(const floatx4*)(sc + so), b = *(const floatx4*)(sh + so);
    floatx4 rv = {0.f, 0.f, 0.f, 0.f};
    if (res) rv = ((const floatx4*)res)[i];
    floatx4 r;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      r[e] = v[e] * a[e] + b[e];
      if (res) r[e] += rv[e];
      if (relu) r[e] = fmaxf(r[e], 0.f);
    }
    ((floatx4*)y)[i] = r;
  }
}

__global__ __launch_bounds__(256) void in_bwd_stats_kernel(const float* __restrict__ dy,
                                                           const float* __restrict__ x,
                                                           const float* __restrict__ sc,
                                                           const float* __restrict__ sh,
                                                           const float* __restrict__ ym, int hw,
                                                           int c, int chunks, int relu,
                                                           double* __restrict__ partial,
                                                           const float* __restrict__ gm = nullptr,
                                                           const float* __restrict__ bt = nullptr) {
  __shared__ double red[2][256][4];
  const int img = blockIdx.y, ch = blockIdx.x;
  const int tpp = c / 4, ppp = 256 / tpp;
  const int q = threadIdx.x % tpp, ps = threadIdx.x / tpp;
  const int p_begin = (int)((long long)hw * ch / chunks), p_end = (int)((long long)hw * (ch + 1) / chunks);
  double s[4] = {0, 0, 0, 0}, s2[4] = {0, 0, 0, 0};
  if (ps < ppp) {
    const size_t so = (size_t)img * c + 4 * q;
    const floatx4 a = *(const floatx4*)(sc + so), b = *(const floatx4*)(sh + so);
    floatx4 ga = {1.f, 1.f, 1.f, 1.f}, be = {0.f, 0.f, 0.f, 0.f};  // BatchNorm affine (mask only)
    if (gm) {
      ga = *(const floatx4*)(gm + 4 * q);
      be = *(const floatx4*)(bt + 4 * q);
    }
    const size_t base = (size_t)img * hw * c + 4 * q;
    for (int p = p_begin + ps; p < p_end; p += ppp) {
      const floatx4 g = *(const floatx4*)(dy + base + (size_t)p * c);
      const floatx4 v = *(const floatx4*)(x + base + (size_t)p * c);
      floatx4 mk = {1.f, 1.f, 1.f, 1.f};
      if (ym) mk = *(const floatx4*)(ym + base + (size_t)p * c);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float xh = v[e] * a[e] + b[e];
        // ReLU mask: of the block output y (residual form), else of the pre-activation
        // γ·x̂ + β (x̂ itself for InstanceNorm)
        const float pre = gm ? ga[e] * xh + be[e] : xh;
        const float gg = ym ? (mk[e] > 0.f ? g[e] : 0.f) : (relu && !(pre > 0.f) ? 0.f : g[e]);
        s[e] += (double)gg;
        s2[e] += (double)gg * (double)xh;
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    red[0][threadIdx.x][e] = s[e];
    red[1][threadIdx.x][e] = s2[e];
  }
  __syncthreads();
  if (threadIdx.x < c) {
    const int qq = threadIdx.x / 4, e = threadIdx.x % 4;
    double a0 = 0, a1 = 0;
    for (int k = 0; k < ppp; ++k) {
      a0 += red[0][k * tpp + qq][e];
      a1 += red[1][k * tpp + qq][e];
    }
    double* o = partial + (((size_t)img * chunks + ch) * 2) * c;
    o[threadIdx.x] = a0;
    o[c + threadIdx.x] = a1;
  }
}

// m1 = mean(g), m2 = mean(g·x̂) per (image, channel), as floats into mm [n][2][c]
__global__ void in_bwd_finalize_kernel(const double* __restrict__ partial, int n, int chunks, int c,
                                       int hw, float* __restrict__ mm) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * c) return;
  const int img = i / c, ch = i % c;
  double s = 0, s2 = 0;
  // unrolled so the chunks' loads are in flight together (the fp64 sums keep their order)
#pragma unroll 16
  for (int k = 0; k < chunks; ++k) {
    const double* o = partial + (((size_t)img * chunks + k) * 2) * c;
    s += o[ch];
    s2 += o[c + ch];
  }
  mm[(size_t)img * 2 * c + ch] = (float)(s / hw);
  mm[(size_t)img * 2 * c + c + ch] = (float)(s2 / hw);
}

__global__ void in_bwd_apply_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                    const float* __restrict__ sc, const float* __restrict__ sh,
                                    const float* __restrict__ mm, const float* __restrict__ ym,
                                    float* __restrict__ dres, float* __restrict__ dx, int hw,
                                    int c, int relu, long long total4,
                                    const float* __restrict__ gm = nullptr,
                                    const float* __restrict__ bt = nullptr) {
  const int c4 = c / 4;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total4; i += (long long)gridDim.x * 256) {
    const int cq = (int)(i % c4) * 4;
    const int img = (int)(i / c4 / hw);
    const size_t so = (size_t)img * c + cq;
    const floatx4 g = ((const floatx4*)dy)[i], v = ((const floatx4*)x)[i];
    const floatx4 a = *(const floatx4*)(sc + so), b = *(const floatx4*)(sh + so);
    const floatx4 m1 = *(const floatx4*)(mm + (size_t)img * 2 * c + cq);
    const floatx4 m2 = *(const floatx4*)(mm + (size_t)img * 2 * c + c + cq);
    floatx4 mk = {1.f, 1.f, 1.f, 1.f};
    if (ym) mk = ((const floatx4*)ym)[i];
    floatx4 ga = {1.f, 1.f, 1.f, 1.f}, be = {0.f, 0.f, 0.f, 0.f};
    if (gm) {
      ga = *(const floatx4*)(gm + cq);
      be = *(const floatx4*)(bt + cq);
    }
    floatx4 r, gr;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float xh = v[e] * a[e] + b[e];
      const float pre = gm ? ga[e] * xh + be[e] : xh;
      const float gg = ym ? (mk[e] > 0.f ? g[e] : 0.f) : (relu && !(pre > 0.f) ? 0.f : g[e]);
      gr[e] = gg;
      r[e] = (gm ? ga[e] * a[e] : a[e]) * (gg - m1[e] - xh * m2[e]);
    }
    ((floatx4*)dx)[i] = r;
    if (dres) ((floatx4*)dres)[i] = gr;  // the identity branch's gradient (residual form)
  }
}

// BatchNorm2d in train mode (the context encoder's norms, resnet.py BasicBlock with BN): the
// InstanceNorm kernels over ONE image of all n·h·w pixels give the batch statistics per channel;
// these finalise them with the affine (γ, β) and the running-statistics update, and turn the
// backward's fp64 sums into mean(g), mean(g·x̂) plus dγ = Σ g·x̂, dβ = Σ g.
__global__ void bn_finalize_kernel(const double* __restrict__ partial, int chunks, int c,
                                   long long m, float eps, const float* __restrict__ gm,
                                   const float* __restrict__ bt, float momentum,
                                   float* __restrict__ rmean, float* __restrict__ rvar,
                                   float* __restrict__ sc, float* __restrict__ sh,
                                   float* __restrict__ rstd_out, float* __restrict__ shift_out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= c) return;
  double s = 0, s2 = 0;
#pragma unroll 16
  for (int k = 0; k < chunks; ++k) {
    const double* o = partial + (size_t)k * 2 * c;
    s += o[i];
    s2 += o[c + i];
  }
  const double mean = s / (double)m;
  double var = s2 / (double)m - mean * mean;
  if (var < 0) var = 0;
  const double rstd = 1.0 / sqrt(var + (double)eps);
  rstd_out[i] = (float)rstd;
  shift_out[i] = (float)(-mean * rstd);
  const double g = gm ? (double)gm[i] : 1.0, b = bt ? (double)bt[i] : 0.0;
  sc[i] = (float)(g * rstd);
  sh[i] = (float)(b - g * mean * rstd);
  if (rmean) {  // torch: running ← (1 − momentum)·running + momentum·batch (unbiased variance)
    const double ub = m > 1 ? var * (double)m / (double)(m - 1) : var;
    rmean[i] = (float)((1.0 - momentum) * (double)rmean[i] + momentum * mean);
    rvar[i] = (float)((1.0 - momentum) * (double)rvar[i] + momentum * ub);
  }
}

__global__ void bn_bwd_finalize_kernel(const double* __restrict__ partial, int chunks, int c,
                                       long long m, float* __restrict__ mm, float* __restrict__ dg,
                                       float* __restrict__ db, int accumulate) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= c) return;
  double s = 0, s2 = 0;
#pragma unroll 16
  for (int k = 0; k < chunks; ++k) {
    const double* o = partial + (size_t)k * 2 * c;
    s += o[i];
    s2 += o[c + i];
  }
  mm[i] = (float)(s / (double)m);
  mm[c + i] = (float)(s2 / (double)m);
  if (dg) dg[i] = accumulate ? dg[i] + (float)s2 : (float)s2;
  if (db) db[i] = accumulate ? db[i] + (float)s : (float)s;
}

// Column sums of a row-major [rows][ld] matrix (a conv's or linear layer's bias gradient,
// Σ_p dY[p][c]): fixed row chunks summed by one kernel into partials [chunk][cols], the chunks
// then summed in order per column (deterministic) — torch's column reduction of a tall, narrow
// matrix ran at ~0.45 TB/s
int colsum_chunks(int rows) { return rows <= 256 ? 1 : (rows / 128 < 256 ? rows / 128 : 256); }

__global__ __launch_bounds__(256) void colsum_partial_kernel(const float* __restrict__ x, int rows,
                                                             int cols, int ld, int chunk,
                                                             float* __restrict__ part) {
  const int c = blockIdx.y * 256 + threadIdx.x;
  if (c >= cols) return;
  const int r0 = blockIdx.x * chunk, r1 = min(rows, r0 + chunk);
  float s = 0.f;
#pragma unroll 8
  for (int r = r0; r < r1; ++r) s += x[(size_t)r * ld + c];
  part[(size_t)blockIdx.x * cols + c] = s;
}

__global__ __launch_bounds__(256) void colsum_final_kernel(const float* __restrict__ x, int rows,
                                                           int cols, int ld, float* __restrict__ out,
                                                           int accumulate) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= cols) return;
  float s = 0.f;
#pragma unroll 8
  for (int r = 0; r < rows; ++r) s += x[(size_t)r * ld + c];
  out[c] = accumulate ? out[c] + s : s;
}

// ---------------------------------------------------------------------------------------------
// SepConvGRU gate algebra of the training step (raft_decoder.py:235-253 with the reference's
// z = σ(convz), r = σ(convr), q = tanh(convq(r·h ⊕ x)), h' = (1 − z)·h + z·q), channels-last,
// zr = the z | r conv's sigmoid output [p][2c] (z = channels 0..c−1, r = c..2c−1), c % 4 == 0.
//   rh = r·h;   h' = h + z·(q − h)
// backward, given dh' and (through the q conv) d(rh):
//   dq_pre = dh'·z·(1 − q²)            dzr[:, :c] = dh'·(q − h)·z(1 − z)     dh_a = dh'·(1 − z)
//   dzr[:, c:] = d(rh)·h·r(1 − r)       dh = dh_a + d(rh)·r
// (the activations' derivatives fused: the convs' backward then runs on pre-activation grads).
__global__ void gru_fwd_kernel(const float* __restrict__ zr, const float* __restrict__ h,
                               const float* __restrict__ q, float* __restrict__ out, int c,
                               long long total4, int mode) {
  const int c4 = c / 4;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total4; i += (long long)gridDim.x * 256) {
    const long long p = i / c4;
    const int cq = (int)(i % c4) * 4;
    const floatx4 hv = *(const floatx4*)(h + p * c + cq);
    floatx4 r;
    if (mode == 0) {  // rh = r·h
      const floatx4 rv = *(const floatx4*)(zr + p * 2 * c + c + cq);
#pragma unroll
      for (int e = 0; e < 4; ++e) r[e] = rv[e] * hv[e];
    } else {          // h' = h + z·(q − h)
      const floatx4 zv = *(const floatx4*)(zr + p * 2 * c + cq);
      const floatx4 qv = *(const floatx4*)(q + p * c + cq);
#pragma unroll
      for (int e = 0; e < 4; ++e) r[e] = hv[e] + zv[e] * (qv[e] - hv[e]);
    }
    *(floatx4*)(out + p * c + cq) = r;
  }
}

__global__ void gru_bwd_q_kernel(const float* __restrict__ dh2, int sdh2, const float* __restrict__ zr,
                                 const float* __restrict__ h, const float* __restrict__ q,
                                 float* __restrict__ dq, float* __restrict__ dzr,
                                 float* __restrict__ dha, int c, long long total4) {
  const int c4 = c / 4;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total4; i += (long long)gridDim.x * 256) {
    const long long p = i / c4;
    const int cq = (int)(i % c4) * 4;
    const floatx4 g = *(const floatx4*)(dh2 + p * sdh2 + cq);
    const floatx4 zv = *(const floatx4*)(zr + p * 2 * c + cq);
    const floatx4 hv = *(const floatx4*)(h + p * c + cq);
    const floatx4 qv = *(const floatx4*)(q + p * c + cq);
    floatx4 a, b, d;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      a[e] = g[e] * zv[e] * (1.f - qv[e] * qv[e]);
      b[e] = g[e] * (qv[e] - hv[e]) * (zv[e] * (1.f - zv[e]));
      d[e] = g[e] * (1.f - zv[e]);
    }
    *(floatx4*)(dq + p * c + cq) = a;
    *(floatx4*)(dzr + p * 2 * c + cq) = b;
    *(floatx4*)(dha + p * c + cq) = d;
  }
}

// dh may alias drh (the dX buffer's h channels, overwritten in place): no __restrict__ on those two
__global__ void gru_bwd_r_kernel(const float* drh, int sdrh, const float* __restrict__ zr,
                                 const float* __restrict__ h, const float* __restrict__ dha,
                                 float* __restrict__ dzr, float* dh, int sdh, int c,
                                 long long total4) {
  const int c4 = c / 4;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total4; i += (long long)gridDim.x * 256) {
    const long long p = i / c4;
    const int cq = (int)(i % c4) * 4;
    const floatx4 g = *(const floatx4*)(drh + p * sdrh + cq);
    const floatx4 rv = *(const floatx4*)(zr + p * 2 * c + c + cq);
    const floatx4 hv = *(const floatx4*)(h + p * c + cq);
    const floatx4 av = *(const floatx4*)(dha + p * c + cq);
    floatx4 a, b;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      a[e] = g[e] * hv[e] * (rv[e] * (1.f - rv[e]));
      b[e] = av[e] + g[e] * rv[e];
    }
    *(floatx4*)(dzr + p * 2 * c + c + cq) = a;
    *(floatx4*)(dh + p * sdh + cq) = b;
  }
}

// Nearest predicted point of every GT point (pytorch3d knn_points K=1 in the symmetric-class
// point-matching loss, point_matching_loss.py:183-186): idx[b][i] = argmin_j Σ_d (g[b][i][d] −
// q[b][j][d])², the first minimum in index order (torch.argmin's tie rule), the squared
// distance summed d = 0, 1, 2 in order.  Workgroup = 256 GT points of one sample; the sample's
// predicted points staged in LDS in chunks of 1024.
__global__ __launch_bounds__(256) void knn1_kernel(const float* __restrict__ g,
                                                   const float* __restrict__ q,
                                                   long long* __restrict__ idx, int P, int Q) {
#pragma clang fp contract(off)
  __shared__ float qs[1024 * 3];
  const int b = blockIdx.y;
  const int i = blockIdx.x * 256 + threadIdx.x;
  float gx = 0.f, gy = 0.f, gz = 0.f;
  if (i < P) {
    const float* gp = g + ((size_t)b * P + i) * 3;
    gx = gp[0];
    gy = gp[1];
    gz = gp[2];
  }
  float best = 0.f;
  int bi = -1;
  for (int j0 = 0; j0 < Q; j0 += 1024) {
    const int nq = Q - j0 < 1024 ? Q - j0 : 1024;
    __syncthreads();
    for (int t = threadIdx.x; t < nq * 3; t += 256) qs[t] = q[((size_t)b * Q + j0) * 3 + t];
    __syncthreads();
    for (int j = 0; j < nq; ++j) {
      const float dx = gx - qs[3 * j], dy = gy - qs[3 * j + 1], dz = gz - qs[3 * j + 2];
      const float d = dx * dx + dy * dy + dz * dz;
      if (bi < 0 || d < best) {
        best = d;
        bi = j0 + j;
      }
    }
  }
  if (i < P) idx[(size_t)b * P + i] = bi;
}

// Training-step pose update for the ortho6d Δrotation (pose.py:124-169 — get_pose_from_delta_pose
// with get_rotation_matrix_from_ortho6d; what train/model.py:pose_update computes with ~30 tiny
// torch ops forward and ~60 backward), one thread per sample:
//   x = a/|a|, z = (x × b)/|x × b|, y = z × x (|·| clamped at 1e-12), Rn = [x y z]·R,
//   vz = t2·e^(−dt2) ('exp') or t2·(dt2 + 1), v_xy = vz'·(dt_xy/weight + t_xy/t2) (vz' = vz, its
//   gradient cut when detach_xy), tn = (vx, vy, vz).
// The backward recomputes the forward and applies the chain rule by hand (normalise:
// g_v = (g_u − u·(u·g_u))/|v|; cross c = p × q: g_p = q × g_c, g_q = g_c × p).
struct Vec3 { float x, y, z; };
__device__ __forceinline__ Vec3 v3(const float* p) { return {p[0], p[1], p[2]}; }
__device__ __forceinline__ Vec3 cross3(Vec3 a, Vec3 b) {
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
__device__ __forceinline__ float dot3(Vec3 a, Vec3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ float norm3(Vec3 a) { return sqrtf(a.x * a.x + a.y * a.y + a.z * a.z); }
__device__ __forceinline__ Vec3 scale3(Vec3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ Vec3 add3(Vec3 a, Vec3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ Vec3 div3(Vec3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
__device__ __forceinline__ float comp(Vec3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
// gradient of u = v / max(|v|, 1e-12) given g_u
__device__ __forceinline__ Vec3 norm_back(Vec3 u, float nv, Vec3 gu) {
  if (nv < 1e-12f) return div3(gu, 1e-12f);
  const float d = dot3(u, gu);
  return div3({gu.x - u.x * d, gu.y - u.y * d, gu.z - u.z * d}, nv);
}

__global__ void pose_update6_kernel(const float* __restrict__ drot, const float* __restrict__ dt,
                                    const float* __restrict__ R, const float* __restrict__ t,
                                    const float* __restrict__ gRn, const float* __restrict__ gtn,
                                    float* __restrict__ o0, float* __restrict__ o1,
                                    float* __restrict__ o2, float* __restrict__ o3, int n,
                                    float weight, int depth_exp, int detach_xy, int backward) {
#pragma clang fp contract(off)
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  const Vec3 a = v3(drot + s * 6), b = v3(drot + s * 6 + 3);
  const float na = norm3(a), nac = na < 1e-12f ? 1e-12f : na;
  const Vec3 x = div3(a, nac);
  const Vec3 c = cross3(x, b);
  const float nc = norm3(c), ncc = nc < 1e-12f ? 1e-12f : nc;
  const Vec3 z = div3(c, ncc);
  const Vec3 y = cross3(z, x);
  const float* Rs = R + s * 9;
  const float* ts = t + s * 3;
  const float* ds = dt + s * 3;
  const float e = depth_exp ? expf(ds[2]) : 0.f;
  const float vz = depth_exp ? ts[2] / e : ts[2] * (ds[2] + 1.f);
  const float fx = ds[0] / weight + ts[0] / ts[2], fy = ds[1] / weight + ts[1] / ts[2];
  if (!backward) {  // o0 = Rn [3][3], o1 = tn [3]
    for (int i = 0; i < 3; ++i) {
      const float m0 = comp(x, i), m1 = comp(y, i), m2 = comp(z, i);
      for (int k = 0; k < 3; ++k) o0[s * 9 + i * 3 + k] = (m0 * Rs[k] + m1 * Rs[3 + k]) + m2 * Rs[6 + k];
    }
    o1[s * 3 + 0] = vz * fx;
    o1[s * 3 + 1] = vz * fy;
    o1[s * 3 + 2] = vz;
    return;
  }
  // backward: o0 = g drot [6], o1 = g dt [3], o2 = g R [3][3], o3 = g t [3]
  const float* G = gRn + s * 9;
  Vec3 gx, gy, gz;  // g M[:, j] = Σ_k gRn[i][k]·R[j][k]
  float gm[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      gm[i][j] = (G[i * 3 + 0] * Rs[j * 3 + 0] + G[i * 3 + 1] * Rs[j * 3 + 1]) + G[i * 3 + 2] * Rs[j * 3 + 2];
  gx = {gm[0][0], gm[1][0], gm[2][0]};
  gy = {gm[0][1], gm[1][1], gm[2][1]};
  gz = {gm[0][2], gm[1][2], gm[2][2]};
  for (int j = 0; j < 3; ++j)  // g R[j][k] = Σ_i M[i][j]·gRn[i][k]
    for (int k = 0; k < 3; ++k) {
      const Vec3 col = j == 0 ? x : (j == 1 ? y : z);
      o2[s * 9 + j * 3 + k] = (col.x * G[0 * 3 + k] + col.y * G[1 * 3 + k]) + col.z * G[2 * 3 + k];
    }
  gz = add3(gz, cross3(x, gy));  // y = z × x
  gx = add3(gx, cross3(gy, z));
  const Vec3 gc = norm_back(z, nc, gz);  // z = c / |c|
  gx = add3(gx, cross3(b, gc));  // c = x × b
  const Vec3 gb = cross3(gc, x);
  const Vec3 ga = norm_back(x, na, gx);  // x = a / |a|
  float* gd = o0 + s * 6;
  gd[0] = ga.x; gd[1] = ga.y; gd[2] = ga.z; gd[3] = gb.x; gd[4] = gb.y; gd[5] = gb.z;
  const float gvx = gtn[s * 3 + 0], gvy = gtn[s * 3 + 1], gvz = gtn[s * 3 + 2];
  float gt0 = gvx * vz / ts[2], gt1 = gvy * vz / ts[2];
  float gt2 = gvx * vz * (-ts[0] / (ts[2] * ts[2])) + gvy * vz * (-ts[1] / (ts[2] * ts[2]));
  const float gvz_all = gvz + (detach_xy ? 0.f : gvx * fx + gvy * fy);
  const float dvz_ddt = depth_exp ? -vz : ts[2];
  const float dvz_dt2 = depth_exp ? 1.f / e : ds[2] + 1.f;
  o1[s * 3 + 0] = gvx * vz / weight;
  o1[s * 3 + 1] = gvy * vz / weight;
  o1[s * 3 + 2] = gvz_all * dvz_ddt;
  gt2 += gvz_all * dvz_dt2;
  o3[s * 3 + 0] = gt0;
  o3[s * 3 + 1] = gt1;
  o3[s * 3 + 2] = gt2;
}

// Disentangled point-matching loss of one refinement iteration (DisentanglePointMatchingLoss,
// point_matching_loss.py:159-218: l1, disentangle_z, reduction mean), fused:
//   pm_points: gt_rt[b][p] = R_gt·x + t_gt, pred_rot[b][p] = R_pred·x + t_gt (x = the sample's model
//              point; rotation by the torch matmul3 order Σ_j in j order);
//   pm_loss:   l_rot = mean_p Σ_d |pred_rot[m] − gt_rt[p]| (m = the nearest predicted point of p
//              for symmetric samples, else p), l_z = |t_pred,z − t_gt,z|, l_xy = Σ_{x,y} |…|,
//              loss = weight · Σ_b (l_rot + l_z + l_xy)/diam_b / B — one workgroup, fixed order;
//   pm_grad:   g R_pred[b] = c_b/P · Σ_p sgn(pred_rot[m] − gt_rt[p]) ⊗ x[m], g t_pred = c_b·sgn(Δt)
//              with c_b = g_loss · weight / (B · diam_b) (sgn 0 = 0, as torch's abs backward).
__global__ void pm_points_kernel(const float* __restrict__ pts, const float* __restrict__ gr,
                                 const float* __restrict__ gtt, const float* __restrict__ pr,
                                 float* __restrict__ gt_rt, float* __restrict__ pred_rot, int B,
                                 int P) {
#pragma clang fp contract(off)
  const long long i = blockIdx.x * 256LL + threadIdx.x;
  if (i >= (long long)B * P) return;
  const int b = (int)(i / P);
  const float* x = pts + i * 3;
  const float* G = gr + b * 9;
  const float* Q = pr + b * 9;
  const float* tg = gtt + b * 3;
  for (int k = 0; k < 3; ++k) {
    const float gk = (x[0] * G[k * 3 + 0] + x[1] * G[k * 3 + 1]) + x[2] * G[k * 3 + 2];
    const float pk = (x[0] * Q[k * 3 + 0] + x[1] * Q[k * 3 + 1]) + x[2] * Q[k * 3 + 2];
    gt_rt[i * 3 + k] = gk + tg[k];
    pred_rot[i * 3 + k] = pk + tg[k];
  }
}

__device__ __forceinline__ float sgnf(float v) { return v > 0.f ? 1.f : (v < 0.f ? -1.f : 0.f); }

__global__ __launch_bounds__(256) void pm_loss_kernel(
    const float* __restrict__ gt_rt, const float* __restrict__ pred_rot,
    const long long* __restrict__ idx, const float* __restrict__ sym, const float* __restrict__ pt,
    const float* __restrict__ gtt, const float* __restrict__ diam, float* __restrict__ loss, int B,
    int P, float weight) {
#pragma clang fp contract(off)
  __shared__ float red[256];
  float total = 0.f;
  for (int b = 0; b < B; ++b) {
    const bool s = sym && sym[b] != 0.f;
    float acc = 0.f;
    for (int p = threadIdx.x; p < P; p += 256) {
      const long long m = s ? idx[(size_t)b * P + p] : p;
      const float* a = pred_rot + ((size_t)b * P + m) * 3;
      const float* g = gt_rt + ((size_t)b * P + p) * 3;
      acc += (fabsf(a[0] - g[0]) + fabsf(a[1] - g[1])) + fabsf(a[2] - g[2]);
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
      if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      const float lrot = red[0] / (float)P;
      const float lz = fabsf(pt[b * 3 + 2] - gtt[b * 3 + 2]);
      const float lxy = fabsf(pt[b * 3 + 0] - gtt[b * 3 + 0]) + fabsf(pt[b * 3 + 1] - gtt[b * 3 + 1]);
      total += ((lrot + lz) + lxy) / diam[b];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) loss[0] = weight * total / (float)B;
}

__global__ __launch_bounds__(256) void pm_grad_kernel(
    const float* __restrict__ gloss, const float* __restrict__ pts, const float* __restrict__ gt_rt,
    const float* __restrict__ pred_rot, const long long* __restrict__ idx,
    const float* __restrict__ sym, const float* __restrict__ pt, const float* __restrict__ gtt,
    const float* __restrict__ diam, float* __restrict__ gR, float* __restrict__ gT, int B, int P,
    float weight) {
#pragma clang fp contract(off)
  __shared__ float red[9][256];
  const int b = blockIdx.x;
  const bool s = sym && sym[b] != 0.f;
  const float cb = gloss[0] * weight / ((float)B * diam[b]);
  float acc[9];
#pragma unroll
  for (int q = 0; q < 9; ++q) acc[q] = 0.f;
  for (int p = threadIdx.x; p < P; p += 256) {
    const long long m = s ? idx[(size_t)b * P + p] : p;
    const float* a = pred_rot + ((size_t)b * P + m) * 3;
    const float* g = gt_rt + ((size_t)b * P + p) * 3;
    const float* x = pts + ((size_t)b * P + m) * 3;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const float sg = sgnf(a[i] - g[i]);
#pragma unroll
      for (int j = 0; j < 3; ++j) acc[i * 3 + j] += sg * x[j];
    }
  }
#pragma unroll
  for (int q = 0; q < 9; ++q) red[q][threadIdx.x] = acc[q];
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w)
#pragma unroll
      for (int q = 0; q < 9; ++q) red[q][threadIdx.x] += red[q][threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x < 9) gR[b * 9 + threadIdx.x] = cb / (float)P * red[threadIdx.x][0];
  if (threadIdx.x < 3) gT[b * 3 + threadIdx.x] = cb * sgnf(pt[b * 3 + threadIdx.x] - gtt[b * 3 + threadIdx.x]);
}

// Full-resolution L1 losses of the sequence loss (RAFTLoss / L1Loss, sequence_loss.py:15-36)
// on the ×s upsampled prediction (F.interpolate bilinear, align_corners=True — ATen's source
// index scale·dst and its two-level weighting order), fused with the upsampling:
//   partial[block] = Σ_{pixels, c} v·|s_val·up(f)_c − target_c|,  sgn_out = v·sgn(s_val·up − t)
// (v = the valid mask or 1); up_l1_finish sums the partials in order: loss = weight·Σ/denom.
// f is channels-last [N][h][w][C] (the decoder's low-resolution flow / mask), target and sgn
// NCHW [N][C][H][W]; the backward is the GEMM adjoint of the upsampling applied to sgn_out.
__global__ __launch_bounds__(256) void up_l1_kernel(
    const float* __restrict__ f, int C, int h, int w, const float* __restrict__ tgt,
    const float* __restrict__ vmask, int N, int H, int W, float sval, float* __restrict__ sgn,
    float* __restrict__ partial) {
#pragma clang fp contract(off)
  __shared__ float red[256];
  const long long HW = (long long)H * W;
  const long long i = blockIdx.x * 256LL + threadIdx.x;
  float acc = 0.f;
  if (i < N * HW) {
    const int n = (int)(i / HW);
    const int rem = (int)(i - n * HW);
    const int Y = rem / W, X = rem - Y * W;
    const float sy = H > 1 ? (float)(h - 1) / (float)(H - 1) : 0.f;
    const float sx = W > 1 ? (float)(w - 1) / (float)(W - 1) : 0.f;
    const float ry = sy * (float)Y, rx = sx * (float)X;
    const int y0 = (int)ry, x0 = (int)rx;
    const int y1 = y0 + (y0 < h - 1 ? 1 : 0), x1 = x0 + (x0 < w - 1 ? 1 : 0);
    const float ly1 = ry - (float)y0, lx1 = rx - (float)x0;
    const float ly0 = 1.f - ly1, lx0 = 1.f - lx1;
    const float v = vmask ? vmask[i] : 1.f;
    const float* f00 = f + (((size_t)n * h + y0) * w + x0) * C;
    const float* f01 = f + (((size_t)n * h + y0) * w + x1) * C;
    const float* f10 = f + (((size_t)n * h + y1) * w + x0) * C;
    const float* f11 = f + (((size_t)n * h + y1) * w + x1) * C;
    for (int c = 0; c < C; ++c) {
      const float up = ly0 * (lx0 * f00[c] + lx1 * f01[c]) + ly1 * (lx0 * f10[c] + lx1 * f11[c]);
      const size_t o = ((size_t)n * C + c) * HW + rem;
      const float d = sval * up - tgt[o];
      acc += v * fabsf(d);
      sgn[o] = v * (d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f));
    }
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
}

__global__ __launch_bounds__(256) void up_l1_finish(const float* __restrict__ partial, int nb,
                                                    const float* __restrict__ denom, float cdenom,
                                                    float weight, float* __restrict__ loss) {
  __shared__ float red[256];
  float acc = 0.f;
  for (int b = threadIdx.x; b < nb; b += 256) acc += partial[b];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) loss[0] = weight * red[0] / (denom ? denom[0] : cdenom);
}

int gru_grid(long long total4) {
  const long long b = (total4 + 255) / 256;
  return (int)(b < 8192 ? b : 8192);
}


// ------------------------------------------------------------------------------ group norm
// GroupNorm (+ReLU) of the pose head (pose_head.py:160-170: conv → GN(32) → ReLU) on channels-last
// data with 4 channels per group: block = (image, group), a float4 per pixel.
template <int K>
__device__ __forceinline__ void gn_block_sum(float (&v)[K], float* red) {
#pragma unroll
  for (int k = 0; k < K; ++k)
    for (int o = 32; o > 0; o >>= 1) v[k] += __shfl_xor(v[k], o, 64);
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int k = 0; k < K; ++k) red[wv * K + k] = v[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = ((red[k] + red[K + k]) + red[2 * K + k]) + red[3 * K + k];
  __syncthreads();
}

__global__ __launch_bounds__(256) void gn_fwd_kernel(const float* __restrict__ x,
                                                     const float* __restrict__ gamma,
                                                     const float* __restrict__ beta,
                                                     float* __restrict__ y, float* __restrict__ stats,
                                                     int HW, int C, int G, float eps, int relu) {
#pragma clang fp contract(off)
  __shared__ float red[4];
  const int n = blockIdx.x / G, g = blockIdx.x % G;
  const size_t base = (size_t)n * HW * C + g * 4;
  float s[1] = {0.f};
  for (int p = threadIdx.x; p < HW; p += 256) {
    const floatx4 v = *(const floatx4*)(x + base + (size_t)p * C);
    s[0] += (v[0] + v[1]) + (v[2] + v[3]);
  }
  gn_block_sum<1>(s, red);
  const float M = (float)(4 * HW);
  const float mean = s[0] / M;
  float q[1] = {0.f};
  for (int p = threadIdx.x; p < HW; p += 256) {
    const floatx4 v = *(const floatx4*)(x + base + (size_t)p * C);
#pragma unroll
    for (int c = 0; c < 4; ++c) q[0] += (v[c] - mean) * (v[c] - mean);
  }
  gn_block_sum<1>(q, red);
  const float rstd = 1.f / sqrtf(q[0] / M + eps);
  const floatx4 ga = *(const floatx4*)(gamma + g * 4);
  const floatx4 be = *(const floatx4*)(beta + g * 4);
  for (int p = threadIdx.x; p < HW; p += 256) {
    const floatx4 v = *(const floatx4*)(x + base + (size_t)p * C);
    floatx4 o;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float z = ((v[c] - mean) * rstd) * ga[c] + be[c];
      o[c] = relu && !(z > 0.f) ? 0.f : z;
    }
    *(floatx4*)(y + base + (size_t)p * C) = o;
  }
  if (threadIdx.x == 0) {
    stats[blockIdx.x * 2 + 0] = mean;
    stats[blockIdx.x * 2 + 1] = rstd;
  }
}

// dx of one (image, group) and its per-channel Σdz·x̂ / Σdz partials (dz: dy through the ReLU,
// recomputed from x exactly as the forward formed its output)
__global__ __launch_bounds__(256) void gn_bwd_kernel(
    const float* __restrict__ dy, const float* __restrict__ x, const float* __restrict__ gamma,
    const float* __restrict__ beta, const float* __restrict__ stats, float* __restrict__ dx,
    float* __restrict__ part, int HW, int C, int G, int relu) {
#pragma clang fp contract(off)
  __shared__ float red[4 * 8];
  const int n = blockIdx.x / G, g = blockIdx.x % G;
  const size_t base = (size_t)n * HW * C + g * 4;
  const float mean = stats[blockIdx.x * 2 + 0], rstd = stats[blockIdx.x * 2 + 1];
  const floatx4 ga = *(const floatx4*)(gamma + g * 4);
  const floatx4 be = *(const floatx4*)(beta + g * 4);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // Σdz[c], Σdz·x̂[c]
  for (int p = threadIdx.x; p < HW; p += 256) {
    const floatx4 v = *(const floatx4*)(x + base + (size_t)p * C);
    const floatx4 d = *(const floatx4*)(dy + base + (size_t)p * C);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float xh = (v[c] - mean) * rstd;
      const float z = xh * ga[c] + be[c];
      const float dz = relu && !(z > 0.f) ? 0.f : d[c];
      acc[c] += dz;
      acc[4 + c] += dz * xh;
    }
  }
  gn_block_sum<8>(acc, red);
  const float M = (float)(4 * HW);
  float a = 0.f, b = 0.f;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    a += ga[c] * acc[c];
    b += ga[c] * acc[4 + c];
  }
  a /= M;
  b /= M;
  for (int p = threadIdx.x; p < HW; p += 256) {
    const floatx4 v = *(const floatx4*)(x + base + (size_t)p * C);
    const floatx4 d = *(const floatx4*)(dy + base + (size_t)p * C);
    floatx4 o;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float xh = (v[c] - mean) * rstd;
      const float z = xh * ga[c] + be[c];
      const float dz = relu && !(z > 0.f) ? 0.f : d[c];
      o[c] = rstd * ((dz * ga[c] - a) - xh * b);
    }
    *(floatx4*)(dx + base + (size_t)p * C) = o;
  }
  if (threadIdx.x < 4) {
    part[((size_t)n * C + g * 4 + threadIdx.x) * 2 + 0] = acc[4 + threadIdx.x];
    part[((size_t)n * C + g * 4 + threadIdx.x) * 2 + 1] = acc[threadIdx.x];
  }
}

// dγ, dβ: the per-image partials summed in image order (deterministic), set or accumulated
__global__ void gn_param_kernel(const float* __restrict__ part, float* __restrict__ dgamma,
                                float* __restrict__ dbeta, int N, int C, int accumulate) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float sg = 0.f, sb = 0.f;
  for (int n = 0; n < N; ++n) {
    sg += part[((size_t)n * C + c) * 2 + 0];
    sb += part[((size_t)n * C + c) * 2 + 1];
  }
  if (accumulate) {
    dgamma[c] += sg;
    dbeta[c] += sb;
  } else {
    dgamma[c] = sg;
    dbeta[c] = sb;
  }
}

}  // namespace

SCFLOW_API int scflow_pose_update6_train(const float* drot, const float* dt, const float* R,
                                         const float* t, const float* gRn, const float* gtn,
                                         float* o0, float* o1, float* o2, float* o3, int n,
                                         float weight, int depth_exp, int detach_xy, int backward,
                                         void* stream) {
  if (!drot || !dt || !R || !t || !o0 || !o1 || n <= 0 || weight == 0.f ||
      (backward && (!gRn || !gtn || !o2 || !o3)))
    return SCFLOW_EINVAL;
  pose_update6_kernel<<<(n + 63) / 64, 64, 0, (hipStream_t)stream>>>(
      drot, dt, R, t, gRn, gtn, o0, o1, o2, o3, n, weight, depth_exp, detach_xy, backward);
  return scflow_launch_status();
}

SCFLOW_API int scflow_pm_loss(const float* pts, const float* gt_r, const float* gt_t,
                              const float* pred_r, const float* pred_t, const float* sym,
                              const float* diam, float* gt_rt, float* pred_rot, long long* idx,
                              float* loss, int B, int P, float weight, void* stream) {
  if (!pts || !gt_r || !gt_t || !pred_r || !pred_t || !diam || !gt_rt || !pred_rot || !loss ||
      (sym && !idx) || B <= 0 || P <= 0)
    return SCFLOW_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  const long long n = (long long)B * P;
  pm_points_kernel<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(pts, gt_r, gt_t, pred_r, gt_rt,
                                                                pred_rot, B, P);
  if (sym) {
    const dim3 grid((unsigned)((P + 255) / 256), (unsigned)B);
    knn1_kernel<<<grid, 256, 0, st>>>(gt_rt, pred_rot, idx, P, P);
  }
  pm_loss_kernel<<<1, 256, 0, st>>>(gt_rt, pred_rot, idx, sym, pred_t, gt_t, diam, loss, B, P,
                                    weight);
  return scflow_launch_status();
}

SCFLOW_API int scflow_pm_loss_backward(const float* gloss, const float* pts, const float* gt_rt,
                                       const float* pred_rot, const long long* idx,
                                       const float* sym, const float* pred_t, const float* gt_t,
                                       const float* diam, float* g_pred_r, float* g_pred_t, int B,
                                       int P, float weight, void* stream) {
  if (!gloss || !pts || !gt_rt || !pred_rot || (sym && !idx) || !pred_t || !gt_t || !diam ||
      !g_pred_r || !g_pred_t || B <= 0 || P <= 0)
    return SCFLOW_EINVAL;
  pm_grad_kernel<<<B, 256, 0, (hipStream_t)stream>>>(gloss, pts, gt_rt, pred_rot, idx, sym, pred_t,
                                                     gt_t, diam, g_pred_r, g_pred_t, B, P, weight);
  return scflow_launch_status();
}

SCFLOW_API int scflow_up_l1_loss(const float* f, int C, int h, int w, const float* target,
                                 const float* vmask, int N, int H, int W, float sval,
                                 const float* denom, float cdenom, float weight, float* sgn,
                                 float* partial, float* loss, void* stream) {
  if (!f || !target || !sgn || !partial || !loss || C <= 0 || h <= 0 || w <= 0 || N <= 0 ||
      H <= 0 || W <= 0 || (!denom && cdenom == 0.f))
    return SCFLOW_EINVAL;
  const long long n = (long long)N * H * W;
  const int nb = (int)((n + 255) / 256);
  hipStream_t st = (hipStream_t)stream;
  up_l1_kernel<<<nb, 256, 0, st>>>(f, C, h, w, target, vmask, N, H, W, sval, sgn, partial);
  up_l1_finish<<<1, 256, 0, st>>>(partial, nb, denom, cdenom, weight, loss);
  return scflow_launch_status();
}

SCFLOW_API int scflow_knn1(const float* gt, const float* pred, long long* idx, int batch, int P,
                           int Q, void* stream) {
  if (!gt || !pred || !idx || batch <= 0 || P <= 0 || Q <= 0) return SCFLOW_EINVAL;
  const dim3 grid((unsigned)((P + 255) / 256), (unsigned)batch);
  knn1_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(gt, pred, idx, P, Q);
  return scflow_launch_status();
}

SCFLOW_API int scflow_gru_gate_forward(const float* zr, const float* h, const float* q, float* out,
                                       long long npix, int c, int mode, void* stream) {
  if (!zr || !h || !out || npix <= 0 || c <= 0 || (c & 3) || (mode != 0 && mode != 1) ||
      (mode == 1 && !q) || !aligned16(zr) || !aligned16(h) || !aligned16(out) ||
      (q && !aligned16(q)))
    return SCFLOW_EINVAL;
  const long long t4 = npix * c / 4;
  gru_fwd_kernel<<<gru_grid(t4), 256, 0, (hipStream_t)stream>>>(zr, h, q, out, c, t4, mode);
  return scflow_launch_status();
}

SCFLOW_API int scflow_gru_gate_backward_q(const float* dh2, int sdh2, const float* zr,
                                          const float* h, const float* q, float* dq, float* dzr,
                                          float* dha, long long npix, int c, void* stream) {
  if (!dh2 || !zr || !h || !q || !dq || !dzr || !dha || npix <= 0 || c <= 0 || (c & 3) ||
      sdh2 < c || (sdh2 & 3) ||
      !aligned16(dh2) || !aligned16(zr) || !aligned16(h) || !aligned16(q) || !aligned16(dq) ||
      !aligned16(dzr) || !aligned16(dha))
    return SCFLOW_EINVAL;
  const long long t4 = npix * c / 4;
  gru_bwd_q_kernel<<<gru_grid(t4), 256, 0, (hipStream_t)stream>>>(dh2, sdh2, zr, h, q, dq, dzr, dha,
                                                                  c, t4);
  return scflow_launch_status();
}

SCFLOW_API int scflow_gru_gate_backward_r(const float* drh, int sdrh, const float* zr,
                                          const float* h, const float* dha, float* dzr, float* dh,
                                          int sdh, long long npix, int c, void* stream) {
  if (!drh || !zr || !h || !dha || !dzr || !dh || npix <= 0 || c <= 0 || (c & 3) || sdrh < c ||
      (sdrh & 3) || sdh < c || (sdh & 3) || !aligned16(drh) || !aligned16(zr) || !aligned16(h) || !aligned16(dha) ||
      !aligned16(dzr) || !aligned16(dh))
    return SCFLOW_EINVAL;
  const long long t4 = npix * c / 4;
  gru_bwd_r_kernel<<<gru_grid(t4), 256, 0, (hipStream_t)stream>>>(drh, sdrh, zr, h, dha, dzr, dh,
                                                                  sdh, c, t4);
  return scflow_launch_status();
}

SCFLOW_API int scflow_conv_wgrad_workspace(const scflow_wgrad_args* args, long long* floats) {
  if (!args || !floats) return SCFLOW_EINVAL;
  WtParams Q;
  if (wthin_geometry(*args, &Q, 0)) {  // rows for a batched call of any segment count
    *floats = wthin_workspace(Q);
    return SCFLOW_OK;
  }
  WwParams R;
  if (wwino_geometry(*args, &R)) {
    *floats = wwino_workspace(R);
    return SCFLOW_OK;
  }
  W5wParams R5;
  if (wwino5_geometry(*args, &R5)) {
    *floats = wwino5_workspace(R5);
    return SCFLOW_OK;
  }
  W1Params R1;
  if (w1_geometry(*args, 1, &R1)) {
    *floats = w1_workspace(R1);
    return SCFLOW_OK;
  }
  WgParams P;
  int splits = 0;
  if (!wgrad_geometry(*args, &P, &splits)) return SCFLOW_EUNSUPPORTED;
  const int taps = args->kh * args->kw;
  *floats = (long long)splits * P.copad * taps * P.cinp + (long long)splits * P.copad;
  return SCFLOW_OK;
}

// the direct implicit-GEMM weight gradient (wgrad_kernel) over the segments sg: geometry, the
// variant's launch and the split reduction
static int wgrad_direct_launch(const scflow_wgrad_args& a, const WgSegs& sg, hipStream_t st) {
  WgParams P;
  int splits = 0;
  if (!wgrad_geometry(a, &P, &splits)) return SCFLOW_EUNSUPPORTED;
  P.sg = sg;
  const int taps = a.kh * a.kw;
  const long long need = (long long)splits * P.copad * taps * P.cinp + (long long)splits * P.copad;
  if (a.workspace_floats < need) return SCFLOW_EINVAL;
  float* slab = a.workspace;
  float* bslab = a.db ? a.workspace + (size_t)splits * P.copad * taps * P.cinp : nullptr;
  const bool vec = a.cout % 4 == 0 && a.sdy % 4 == 0 && aligned16(a.dy) && a.cin0 % 4 == 0 &&
                   a.s0 % 4 == 0 && aligned16(a.src0) &&
                   (a.cin1 == 0 || (a.cin1 % 4 == 0 && a.s1 % 4 == 0 && aligned16(a.src1)));
  // (3×3: one workgroup per CU; SCFLOW_WGRAD_KS=1 keeps one wave set, tuning only)
  static const int ks_env = [] {
    const char* e = getenv("SCFLOW_WGRAD_KS");
    return e ? atoi(e) : 2;
  }();
  // the GRU's 1×5 / 5×1: two wave sets when cout ≤ 128 (q: 90 → 81 µs for 5×1, 80 → 71 for 1×5
  // at configs[3]); one for the 256-wide z | r, which two sets slow (131 → 137, 146 → 155 µs).
  // SCFLOW_WGRAD_KS5=0 never, 2 always (tuning)
  static const int ks5_env = [] {
    const char* e = getenv("SCFLOW_WGRAD_KS5");
    return e ? atoi(e) : 1;
  }();
  const size_t lds1 = sizeof(float) * (size_t)(P.cp + P.hr * P.hc) * WT;
  const bool ks5 = taps == 5 && (ks5_env == 2 || (ks5_env == 1 && a.cout <= 128));
  const int occ = taps >= 9 || ks5 ? 1 : 2;
  const bool db2 = vec && 2 * lds1 * occ <= 160 * 1024;  // double-buffer if it keeps occupancy
  const size_t lds = lds1 * (db2 ? 2 : 1);
  if (lds > 160 * 1024) return SCFLOW_EUNSUPPORTED;
  const dim3 grid((unsigned)(P.co_tiles * (P.cinp / WT)), (unsigned)splits);
  // two wave sets splitting each chunk's k-steps
  const bool ks2 = vec && ((taps >= 9 && ks_env == 2) || ks5);
#define SCFLOW_WG(KH_, KW_, S_)                                                                  \
  if (a.kh == KH_ && a.kw == KW_ && a.stride == S_) {                                            \
    if (KH_ * KW_ >= 5 && ks2) {                                                                 \
      if (db2)                                                                                   \
        wgrad_kernel<KH_, KW_, S_, true, true, 64, 2><<<grid, 512, lds, st>>>(P, slab, bslab);   \
      else                                                                                       \
        wgrad_kernel<KH_, KW_, S_, true, false, 64, 2><<<grid, 512, lds, st>>>(P, slab, bslab);  \
    } else if (db2)                                                                              \
      wgrad_kernel<KH_, KW_, S_, true, true><<<grid, 256, lds, st>>>(P, slab, bslab);            \
    else if (vec)                                                                                \
      wgrad_kernel<KH_, KW_, S_, true, false><<<grid, 256, lds, st>>>(P, slab, bslab);           \
    else                                                                                         \
      wgrad_kernel<KH_, KW_, S_, false, false><<<grid, 256, lds, st>>>(P, slab, bslab);          \
  } else
  SCFLOW_WG(3, 3, 1)
  SCFLOW_WG(1, 1, 1)
  SCFLOW_WG(1, 5, 1)
  SCFLOW_WG(5, 1, 1)
  SCFLOW_WG(3, 3, 2)
  SCFLOW_WG(1, 1, 2)
  return SCFLOW_EUNSUPPORTED;
#undef SCFLOW_WG
  int rc = scflow_launch_status();
  if (rc != SCFLOW_OK) return rc;
  int lg = 0;  // 2^lg lanes of partial sums per output, ≈ splits / 4 of them, ≤ 16
  while (lg < 4 && (4 << lg) < splits) ++lg;
  const int opb = 256 >> lg;
  const unsigned rblocks = (unsigned)(((long long)a.cout * taps * P.cinp + opb - 1) / opb +
                                      (a.db ? (a.cout + opb - 1) / opb : 0));
  wgrad_reduce_kernel<<<rblocks, 256, 0, st>>>(slab, bslab, a.dw, a.db, splits, a.cout,
                                               a.cin0 + a.cin1, taps, P.copad, P.cinp, a.accumulate,
                                               lg);
  return scflow_launch_status();
}

SCFLOW_API int scflow_conv_wgrad_batched(const scflow_wgrad_args* args, int segs,
                                         const float* const* dys, const float* const* src0s,
                                         const float* const* src1s, void* stream) {
  if (!args || segs < 1 || segs > WG_MAXSEG || !dys || !src0s || (args->cin1 > 0 && !src1s) ||
      !args->dw || !args->workspace || args->n <= 0)
    return SCFLOW_EINVAL;
  for (int i = 0; i < segs; ++i)
    if (!dys[i] || !src0s[i] || !aligned16(dys[i]) || !aligned16(src0s[i]) ||
        (args->cin1 > 0 && (!src1s[i] || !aligned16(src1s[i]))))
      return SCFLOW_EINVAL;
  scflow_wgrad_args t = *args;  // the walk: all segments' images in a row
  t.n = args->n * segs;
  t.dy = dys[0];
  t.src0 = src0s[0];
  t.src1 = args->cin1 > 0 ? src1s[0] : nullptr;
  WgSegs sg;
  sg.nimg = args->n;
  for (int i = 0; i < WG_MAXSEG; ++i) {
    const int j = i < segs ? i : 0;
    sg.dy[i] = dys[j];
    sg.src0[i] = src0s[j];
    sg.src1[i] = args->cin1 > 0 ? src1s[j] : nullptr;
  }
  WwParams R;
  if (wwino_geometry(t, &R)) {
    if (t.workspace_floats < wwino_workspace(R)) return SCFLOW_EINVAL;
    R.sg = sg;
    return wwino_launch(R, (hipStream_t)stream);
  }
  W5wParams R5;
  if (wwino5_geometry(t, &R5)) {
    if (t.workspace_floats < wwino5_workspace(R5)) return SCFLOW_EINVAL;
    R5.sg = sg;
    return wwino5_launch(R5, (hipStream_t)stream);
  }
  WtParams Q;
  if (wthin_geometry(t, &Q, segs)) {
    Q.sg = sg;
    return wthin_launch(Q, (hipStream_t)stream);
  }
  W1Params R1;
  if (w1_geometry(t, segs, &R1)) {
    R1.sg = sg;
    return w1_launch(R1, (hipStream_t)stream);
  }
  return wgrad_direct_launch(t, sg, (hipStream_t)stream);
}

SCFLOW_API int scflow_conv_wgrad(const scflow_wgrad_args* args, void* stream) {
  if (!args) return SCFLOW_EINVAL;
  const scflow_wgrad_args& a = *args;
  if (!a.dy || !a.src0 || !a.dw || !a.workspace || a.n <= 0 || a.h <= 0 || a.w <= 0 ||
      a.cout <= 0 || a.cin0 <= 0 || a.cin1 < 0 || (a.cin1 > 0 && !a.src1) || a.sdy < a.cout ||
      a.s0 < a.cin0 || (a.cin1 > 0 && a.s1 < a.cin1) || a.ph < 0 || a.pw < 0)
    return SCFLOW_EINVAL;
  WtParams Q;
  if (wthin_geometry(a, &Q)) {
    wg_single_seg(a, &Q.sg);
    return wthin_launch(Q, (hipStream_t)stream);
  }
  WwParams R;
  if (wwino_geometry(a, &R)) {
    if (a.workspace_floats < wwino_workspace(R)) return SCFLOW_EINVAL;
    wg_single_seg(a, &R.sg);
    return wwino_launch(R, (hipStream_t)stream);
  }
  W5wParams R5;
  if (wwino5_geometry(a, &R5)) {
    if (a.workspace_floats < wwino5_workspace(R5)) return SCFLOW_EINVAL;
    wg_single_seg(a, &R5.sg);
    return wwino5_launch(R5, (hipStream_t)stream);
  }
  W1Params R1;
  if (w1_geometry(a, 1, &R1)) {
    wg_single_seg(a, &R1.sg);
    return w1_launch(R1, (hipStream_t)stream);
  }
  WgSegs sg;
  wg_single_seg(a, &sg);
  return wgrad_direct_launch(a, sg, (hipStream_t)stream);
}

SCFLOW_API int scflow_im2col_ex(const float* x, int sx, float* cols, int n, int h, int w, int cin,
                                int kh, int kw, int stride, int ph, int pw, int channel_major,
                                void* stream) {
  if (!x || !cols || n <= 0 || h <= 0 || w <= 0 || cin <= 0 || kh <= 0 || kw <= 0 || stride <= 0 ||
      ph < 0 || pw < 0 || sx < cin)
    return SCFLOW_EINVAL;
  const int oh = (h + 2 * ph - kh) / stride + 1, ow = (w + 2 * pw - kw) / stride + 1;
  if (oh <= 0 || ow <= 0) return SCFLOW_EINVAL;
  const int vec =
      (!channel_major && cin % 4 == 0 && sx % 4 == 0 && aligned16(x) && aligned16(cols)) ? 4 : 1;
  const long long total = (long long)n * oh * ow * kh * kw * cin / vec;
  const int blocks = (int)((total + 255) / 256 < 65536 ? (total + 255) / 256 : 65536);
  if (total * vec < (1LL << 31) - 256LL * 65536)
    im2col_kernel<unsigned><<<blocks, 256, 0, (hipStream_t)stream>>>(
        x, sx, cols, h, w, cin, kh, kw, stride, ph, pw, oh, ow, total, vec, channel_major ? 1 : 0);
  else
    im2col_kernel<unsigned long long><<<blocks, 256, 0, (hipStream_t)stream>>>(
        x, sx, cols, h, w, cin, kh, kw, stride, ph, pw, oh, ow, total, vec, channel_major ? 1 : 0);
  return scflow_launch_status();
}

SCFLOW_API int scflow_im2col(const float* x, int sx, float* cols, int n, int h, int w, int cin,
                             int kh, int kw, int stride, int ph, int pw, void* stream) {
  return scflow_im2col_ex(x, sx, cols, n, h, w, cin, kh, kw, stride, ph, pw, 0, stream);
}

SCFLOW_API int scflow_col2im(const float* cols, float* dx, int sdx, int n, int h, int w, int cin,
                             int kh, int kw, int stride, int ph, int pw, void* stream) {
  if (!cols || !dx || n <= 0 || h <= 0 || w <= 0 || cin <= 0 || kh <= 0 || kw <= 0 || stride <= 0 ||
      ph < 0 || pw < 0 || sdx < cin)
    return SCFLOW_EINVAL;
  const int oh = (h + 2 * ph - kh) / stride + 1, ow = (w + 2 * pw - kw) / stride + 1;
  if (oh <= 0 || ow <= 0) return SCFLOW_EINVAL;
  const int vec = (cin % 4 == 0 && sdx % 4 == 0 && aligned16(dx) && aligned16(cols)) ? 4 : 1;
  const long long total = (long long)n * h * w * cin / vec;
  const int blocks = (int)((total + 255) / 256 < 65536 ? (total + 255) / 256 : 65536);
  if (total * vec < (1LL << 31) - 256LL * 65536)
    col2im_kernel<unsigned><<<blocks, 256, 0, (hipStream_t)stream>>>(cols, dx, sdx, h, w, cin, kh, kw,
                                                                     stride, ph, pw, oh, ow, total, vec);
  else
    col2im_kernel<unsigned long long><<<blocks, 256, 0, (hipStream_t)stream>>>(
        cols, dx, sdx, h, w, cin, kh, kw, stride, ph, pw, oh, ow, total, vec);
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
  static const bool win_off = [] {
    const char* e = getenv("SCFLOW_LOOKUP_BWD_WIN");
    return e && e[0] == '0';
  }();
  if (radius >= 1 && radius <= 4 && !win_off) {
    const long long tw = (long long)n * h * w * num_levels;
    const unsigned bw = (unsigned)((tw + 255) / 256);
    switch (radius) {
#define SCFLOW_LKW(RR)                                                                             \
  case RR:                                                                                         \
    corr_lookup_bwd_win_kernel<RR><<<bw, 256, 0, st>>>(dout, out_layout, out_stride, flow,         \
                                                       flow_layout, dpyr, n, h, w, num_levels, tw); \
    break;
      SCFLOW_LKW(1)
      SCFLOW_LKW(2)
      SCFLOW_LKW(3)
      SCFLOW_LKW(4)
#undef SCFLOW_LKW
      default:
        return SCFLOW_EUNSUPPORTED;
    }
    return scflow_launch_status();
  }
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

SCFLOW_API int scflow_colsum(const float* x, int rows, int cols, int ld, float* out, int accumulate,
                             float* workspace, void* stream) {
  if (!x || !out || rows <= 0 || cols <= 0 || ld < cols || (rows > 256 && !workspace))
    return SCFLOW_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  if (rows <= 256) {  // one pass: thread per column over every row
    colsum_final_kernel<<<ceil_div(cols, 256), 256, 0, st>>>(x, rows, cols, ld, out, accumulate);
    return scflow_launch_status();
  }
  const int nch = colsum_chunks(rows);
  const int chunk = ceil_div(rows, nch);
  colsum_partial_kernel<<<dim3(nch, ceil_div(cols, 256)), 256, 0, st>>>(x, rows, cols, ld, chunk,
                                                                        workspace);
  colsum_final_kernel<<<ceil_div(cols, 256), 256, 0, st>>>(workspace, nch, cols, cols, out, accumulate);
  return scflow_launch_status();
}

SCFLOW_API int scflow_colsum_workspace(int rows, int cols) {
  return rows <= 256 ? 0 : colsum_chunks(rows) * cols;
}

SCFLOW_API int scflow_in_apply(const float* x, const float* scale, const float* shift, float* y,
                               int n, int hw, int c, int relu, void* stream) {
  if (!x || !scale || !shift || !y || n <= 0 || hw <= 0 || c <= 0) return SCFLOW_EINVAL;
  if (c % 4) return SCFLOW_EUNSUPPORTED;
  if (!aligned16(x) || !aligned16(y) || !aligned16(scale) || !aligned16(shift)) return SCFLOW_EALIGN;
  const long long total4 = (long long)n * hw * c / 4;
  const int blocks = (int)((total4 + 255) / 256 < 16384 ? (total4 + 255) / 256 : 16384);
  in_apply_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(x, scale, shift, nullptr, y, hw, c,
                                                            relu ? 1 : 0, total4);
  return scflow_launch_status();
}

SCFLOW_API int scflow_in_apply_residual(const float* x, const float* scale, const float* shift,
                                        const float* res, float* y, int n, int hw, int c,
                                        void* stream) {
  if (!x || !scale || !shift || !res || !y || n <= 0 || hw <= 0 || c <= 0) return SCFLOW_EINVAL;
  if (c % 4) return SCFLOW_EUNSUPPORTED;
  if (!aligned16(x) || !aligned16(y) || !aligned16(res) || !aligned16(scale) || !aligned16(shift))
    return SCFLOW_EALIGN;
  const long long total4 = (long long)n * hw * c / 4;
  const int blocks = (int)((total4 + 255) / 256 < 16384 ? (total4 + 255) / 256 : 16384);
  in_apply_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(x, scale, shift, res, y, hw, c, 1, total4);
  return scflow_launch_status();
}

SCFLOW_API int scflow_in_backward(const float* dy, const float* x, const float* scale,
                                  const float* shift, float* dx, double* partial, float* mm, int n,
                                  int hw, int c, int chunks, int relu, void* stream) {
  if (!dy || !x || !scale || !shift || !dx || !partial || !mm || n <= 0 || hw <= 0 || c <= 0 ||
      chunks <= 0)
    return SCFLOW_EINVAL;
  if (c % 4 || c > 256) return SCFLOW_EUNSUPPORTED;
  if (!aligned16(dy) || !aligned16(x) || !aligned16(dx) || !aligned16(scale) || !aligned16(shift) ||
      !aligned16(mm))
    return SCFLOW_EALIGN;
  hipStream_t st = (hipStream_t)stream;
  in_bwd_stats_kernel<<<dim3(chunks, n), 256, 0, st>>>(dy, x, scale, shift, nullptr, hw, c, chunks,
                                                       relu ? 1 : 0, partial);
  in_bwd_finalize_kernel<<<ceil_div((long long)n * c, 256), 256, 0, st>>>(partial, n, chunks, c, hw, mm);
  const long long total4 = (long long)n * hw * c / 4;
  const int blocks = (int)((total4 + 255) / 256 < 16384 ? (total4 + 255) / 256 : 16384);
  in_bwd_apply_kernel<<<blocks, 256, 0, st>>>(dy, x, scale, shift, mm, nullptr, nullptr, dx, hw, c,
                                              relu ? 1 : 0, total4);
  return scflow_launch_status();
}

SCFLOW_API int scflow_in_backward_residual(const float* dy, const float* x, const float* scale,
                                           const float* shift, const float* y, float* dx,
                                           float* dres, double* partial, float* mm, int n, int hw,
                                           int c, int chunks, void* stream) {
  if (!dy || !x || !scale || !shift || !y || !dx || !dres || !partial || !mm || n <= 0 ||
      hw <= 0 || c <= 0 || chunks <= 0)
    return SCFLOW_EINVAL;
  if (c % 4 || c > 256) return SCFLOW_EUNSUPPORTED;
  if (!aligned16(dy) || !aligned16(x) || !aligned16(y) || !aligned16(dx) || !aligned16(dres) ||
      !aligned16(scale) || !aligned16(shift) || !aligned16(mm))
    return SCFLOW_EALIGN;
  hipStream_t st = (hipStream_t)stream;
  in_bwd_stats_kernel<<<dim3(chunks, n), 256, 0, st>>>(dy, x, scale, shift, y, hw, c, chunks, 1,
                                                       partial);
  in_bwd_finalize_kernel<<<ceil_div((long long)n * c, 256), 256, 0, st>>>(partial, n, chunks, c, hw, mm);
  const long long total4 = (long long)n * hw * c / 4;
  const int blocks = (int)((total4 + 255) / 256 < 16384 ? (total4 + 255) / 256 : 16384);
  in_bwd_apply_kernel<<<blocks, 256, 0, st>>>(dy, x, scale, shift, mm, y, dres, dx, hw, c, 1, total4);
  return scflow_launch_status();
}

SCFLOW_API int scflow_bn_forward(const float* x, const float* gamma, const float* beta,
                                 const float* res, float* y, float* running_mean,
                                 float* running_var, float* rstd, float* shift, float* sc, float* sh,
                                 double* partial, long long m, int c, int chunks, float eps,
                                 float momentum, int relu, void* stream) {
  if (!x || !y || !rstd || !shift || !sc || !sh || !partial || m <= 0 || c <= 0 || chunks <= 0 ||
      (m / chunks) > INT32_MAX || m > INT32_MAX)
    return SCFLOW_EINVAL;
  if (c % 4 || c > 256 || (!gamma) != (!beta) || (!running_mean) != (!running_var))
    return SCFLOW_EUNSUPPORTED;
  if (!aligned16(x) || !aligned16(y) || (res && !aligned16(res)) || !aligned16(sc) || !aligned16(sh))
    return SCFLOW_EALIGN;
  hipStream_t st = (hipStream_t)stream;
  // the batch statistics: the InstanceNorm statistics kernel over one image of m pixels
  int rc = scflow_enc_stats(x, 1, (int)m, c, chunks, partial, stream);
  if (rc != SCFLOW_OK) return rc;
  bn_finalize_kernel<<<ceil_div(c, 256), 256, 0, st>>>(partial, chunks, c, m, eps, gamma, beta,
                                                        momentum, running_mean, running_var, sc, sh,
                                                        rstd, shift);
  const long long total4 = m * c / 4;
  const int blocks = (int)((total4 + 255) / 256 < 16384 ? (total4 + 255) / 256 : 16384);
  in_apply_kernel<<<blocks, 256, 0, st>>>(x, sc, sh, res, y, (int)m, c, (relu || res) ? 1 : 0, total4);
  return scflow_launch_status();
}

SCFLOW_API int scflow_bn_backward(const float* dy, const float* x, const float* rstd,
                                  const float* shift, const float* gamma, const float* beta,
                                  const float* y, float* dx, float* dres, float* dgamma,
                                  float* dbeta, double* partial, float* mm, long long m, int c,
                                  int chunks, int relu, int accumulate, void* stream) {
  if (!dy || !x || !rstd || !shift || !dx || !partial || !mm || m <= 0 || c <= 0 || chunks <= 0 ||
      m > INT32_MAX || (dres && !y))
    return SCFLOW_EINVAL;
  if (c % 4 || c > 256 || (!gamma) != (!beta)) return SCFLOW_EUNSUPPORTED;
  if (!aligned16(dy) || !aligned16(x) || !aligned16(dx) || !aligned16(rstd) || !aligned16(shift) ||
      !aligned16(mm) || (y && !aligned16(y)) || (dres && !aligned16(dres)) ||
      (gamma && (!aligned16(gamma) || !aligned16(beta))))
    return SCFLOW_EALIGN;
  hipStream_t st = (hipStream_t)stream;
  in_bwd_stats_kernel<<<dim3(chunks, 1), 256, 0, st>>>(dy, x, rstd, shift, y, (int)m, c, chunks,
                                                       relu ? 1 : 0, partial, gamma, beta);
  bn_bwd_finalize_kernel<<<ceil_div(c, 256), 256, 0, st>>>(partial, chunks, c, m, mm, dgamma, dbeta,
                                                            accumulate);
  const long long total4 = m * c / 4;
  const int blocks = (int)((total4 + 255) / 256 < 16384 ? (total4 + 255) / 256 : 16384);
  in_bwd_apply_kernel<<<blocks, 256, 0, st>>>(dy, x, rstd, shift, mm, y, dres, dx, (int)m, c,
                                              relu ? 1 : 0, total4, gamma, beta);
  return scflow_launch_status();
}

static int gn_check(const void* a, const void* b, const void* c, int n, int hw, int ch, int groups) {
  if (!a || !b || !c || n <= 0 || hw <= 0 || groups <= 0 || ch != 4 * groups) return SCFLOW_EINVAL;
  if (((uintptr_t)a | (uintptr_t)b | (uintptr_t)c) & 15) return SCFLOW_EINVAL;
  return 0;
}

SCFLOW_API int scflow_group_norm_forward(const float* x, const float* gamma, const float* beta,
                                         float* y, float* stats, int n, int hw, int c, int groups,
                                         float eps, int relu, void* stream) {
  if (int e = gn_check(x, y, gamma, n, hw, c, groups)) return e;
  if (!beta || !stats || ((uintptr_t)beta & 15)) return SCFLOW_EINVAL;
  gn_fwd_kernel<<<n * groups, 256, 0, (hipStream_t)stream>>>(x, gamma, beta, y, stats, hw, c, groups,
                                                             eps, relu ? 1 : 0);
  return scflow_launch_status();
}

SCFLOW_API int scflow_group_norm_backward(const float* dy, const float* x, const float* gamma,
                                          const float* beta, const float* stats, float* dx,
                                          float* part, float* dgamma, float* dbeta, int n, int hw,
                                          int c, int groups, int relu, int accumulate,
                                          void* stream) {
  if (int e = gn_check(dy, x, dx, n, hw, c, groups)) return e;
  if (!gamma || !beta || !stats || !part || !dgamma || !dbeta || ((uintptr_t)(gamma) & 15) ||
      ((uintptr_t)beta & 15))
    return SCFLOW_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  gn_bwd_kernel<<<n * groups, 256, 0, st>>>(dy, x, gamma, beta, stats, dx, part, hw, c, groups,
                                            relu ? 1 : 0);
  gn_param_kernel<<<(c + 127) / 128, 128, 0, st>>>(part, dgamma, dbeta, n, c, accumulate ? 1 : 0);
  return scflow_launch_status();
}
