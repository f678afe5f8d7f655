// Winograd F(4×4, 3×3) convolution on fp32 MFMA (round 5) — included by conv.hip (inside its
// anonymous namespace).  For the update block's wide 3×3 stride-1 pad-1 convs (the XHead hidden
// convs 128 → 2·256, corr_net.1 256 → 192, out_net 256 → 126; reference
// models/decoder/raft_decoder.py:75-85,256-294): 36 transform points per 4×4 output tile, so the
// channel contractions execute 2.25 multiplies per output pixel and tap set instead of F(2×2,3×3)'s
// 4 (1.78× fewer MFMAs) and the direct conv's 9.
//
// Interpolation points {0, 1, −1, 2, −½, ∞} (Toom–Cook), chosen over Lavin's {0, ±1, ±2, ∞} for
// accuracy: in an fp32 restatement with 256 input channels the max error against fp64 is 1.3e-5
// of outputs ≈ 4 (Lavin's points 3.8e-5; F(2×2,3×3) 2.8e-6, the direct fp32 conv 1.3e-6).
//   Bᵀ = [1 3/2 −2 −3/2 1 0; 0 −1 −5/2 −1/2 1 0; 0 1 1/2 −5/2 1 0; 0 −1/2 −1 1/2 1 0;
//         0 2 −1 −2 1 0; 0 1 3/2 −2 −3/2 1]
//   G  = [1 0 0; −1/3 −1/3 −1/3; 1/3 −1/3 1/3; 1/15 2/15 4/15; −16/15 8/15 −4/15; 0 0 1]
//   Aᵀ = [1 1 1 1 1 0; 0 1 −1 2 −1/2 0; 0 1 1 4 1/4 0; 0 1 −1 8 −1/8 1]
// Y = Aᵀ[(G g Gᵀ) ⊙ (Bᵀ d B)]A for the 6×6 input patch d of a 4×4 output tile.
//
// Two launches per conv:
//  1. wino4_vt_kernel — the input transform V = Bᵀ d B of every (tile, channel) once, written to
//     a workspace in the GEMM's lane order [tile block][8-channel sub-step][point][lane][4]
//     (2.25× the input's bytes; L2 / Infinity-Cache resident).  Computing V once per conv instead
//     of once per output-channel block (as the F(2×2,3×3) kernel does, from its LDS halo) keeps
//     the VALU work — 6× that of F(2×2,3×3) per MFMA — out of the MFMA loop.
//  2. conv_wino4_kernel — 36 independent GEMMs M_ξ[tile][co] = Σ_ci V_ξ[tile][ci]·U_ξ[ci][co]:
//     workgroup = 32 tiles × 32 output channels, 4 waves, wave w owns points ξ = 9w .. 9w+8 and
//     streams their V and U slices from L2 as lane-ordered 1 KiB buffer loads (each point's pair
//     reloaded for the next sub-step right after its 4 MFMAs issue): no LDS, no barrier and no
//     VALU in the main loop.  Epilogue: the points meet in LDS 8 tiles at a time (36 × 32 × 9
//     floats), one (tile, channel) per thread applies Aᵀ·A and the fused bias / affine / bias-map
//     / residual / activation, channel-contiguous stores.

constexpr int W4P = 36;   // transform points per tile
constexpr int W4KC = 8;   // input channels per sub-step (lanes 0-31: channels 0-3, 32-63: 4-7)
constexpr int W4TM = 32;  // tiles per block (MFMA rows)
constexpr int W4NPW = W4P / 4;  // points per wave
constexpr int W4CP = 32;  // epilogue LDS row: 32 output channels (16-B reads conflict-free)
constexpr int W4_LDS = W4P * 16 * W4CP * 4;  // epilogue bytes: [36 points][16 tiles][W4CP]

__device__ __forceinline__ bool w4_al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// four consecutive floats p[0..3] of which the first nv are valid (zeros after), as one 16-B
// load when vec
__device__ __forceinline__ floatx4 w4_ld4(const float* p, bool vec, int nv) {
  if (vec) return *(const floatx4*)p;
  floatx4 r = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int e = 0; e < 4; ++e)
    if (e < nv) r[e] = p[e];
  return r;
}

struct Wino4Params {
  scflow_conv_args a;
  const float* v;   // transformed input [ntb][nsub][36][64][4]
  int cp0;          // source-0 channels padded to W4KC (source 1 starts there)
  int nsub;         // sub-steps over both sources
  int th, tw;       // tiles per image column / row (h/4, w/4)
  int ntiles, ntb;  // tiles, tile blocks
  int xgt, xgc;     // XCD-blocked GEMM order (w4_block): xgt tile blocks × xgc channel blocks, 0 = off
  unsigned long long* stamps;  // profiling (scflow_debug_conv_stamps), or NULL
  // predictor contraction (conv_wino4_kernel<·, ·, true>, scflow_xhead_pred): weights
  // [cout][W4PZ], partial sums out (xhead_pred.h), channel blocks < pnbf feed the 3×3 two-output
  // predictor, the rest the 1×1 one-output predictor
  const float* pw = nullptr;
  float* zp = nullptr;
  int pnbf = 0;
};
constexpr int W4PZ = 20;  // predictor columns per hidden channel (3×3 taps × 2 outputs, padded)

// (tile block, output-channel block) of a GEMM workgroup.  Workgroups go round-robin over the 8
// XCDs in linear order (x fastest), each XCD with its own 4 MB L2.  In linear order the ≈ 64
// workgroups an XCD runs at a time are ≈ 32 tile blocks × 2 channel blocks, so every V slice is
// fetched from the memory side once per channel block (16× for the 512-wide heads conv at 64×64
// maps: 10× the conv's algorithmic bytes, round 5).  Blocked (xgt > 0): linear id L is logical
// index (L mod 8)·N/8 + L/8, so each XCD owns a contiguous range of the logical order, which
// walks xgt × xgc blocks (channel blocks fastest inside a block): an XCD's concurrent
// workgroups share xgt V slices and xgc U slices through its L2, the sub-step they all stream
// at once being ≈ 37 KB per slice.  The host picks xgt, xgc dividing the grid, N ≡ 0 mod 8.
__device__ __forceinline__ void w4_block(const Wino4Params& P, int& tb, int& cb) {
  tb = blockIdx.x;
  cb = blockIdx.y;
  if (P.xgt <= 0) return;
  const int R = gridDim.x, C = gridDim.y;
  const int L = blockIdx.y * R + blockIdx.x;
  const int per = (R * C) >> 3;
  const int id = (L & 7) * per + (L >> 3);
  const int bsz = P.xgt * P.xgc, cblocks = C / P.xgc;
  const int blk = id / bsz, r = id - blk * bsz;
  tb = (blk / cblocks) * P.xgt + r / P.xgc;
  cb = (blk % cblocks) * P.xgc + r % P.xgc;
}

// v = Bᵀ·d over one axis (6 float4)
__device__ __forceinline__ void w4_bt(const floatx4 (&d)[6], floatx4 (&v)[6]) {
  v[0] = d[0] + 1.5f * d[1] - 2.f * d[2] - 1.5f * d[3] + d[4];
  v[1] = d[4] - d[1] - 2.5f * d[2] - 0.5f * d[3];
  v[2] = d[1] + 0.5f * d[2] - 2.5f * d[3] + d[4];
  v[3] = d[4] - 0.5f * d[1] - d[2] + 0.5f * d[3];
  v[4] = 2.f * d[1] - d[2] - 2.f * d[3] + d[4];
  v[5] = d[1] + 1.5f * d[2] - 2.f * d[3] - 1.5f * d[4] + d[5];
}

// y = Aᵀ·m over one axis (6 → 4)
__device__ __forceinline__ void w4_at(const float (&m)[6], float (&y)[4]) {
  const float s12 = m[1] + m[2], d12 = m[1] - m[2];
  y[0] = m[0] + s12 + m[3] + m[4];
  y[1] = d12 + 2.f * m[3] - 0.5f * m[4];
  y[2] = s12 + 4.f * m[3] + 0.25f * m[4];
  y[3] = d12 + 8.f * m[3] - 0.125f * m[4] + m[5];
}

// 1. input transform: workgroup = (tile block blockIdx.x, sub-step blockIdx.y), 6 waves; lane =
//    (tile li, channel quad hh).  Wave x first transforms patch column x (6 loads in flight per
//    lane, t[i][x] = (Bᵀ d)[i] into LDS), then wave i transforms row i of t (V[i][·] = Bᵀ t[i]) and
//    stores its 6 points as 1 KiB lane-ordered pieces.
constexpr int W4VT_THREADS = 6 * 64;
__global__ __launch_bounds__(W4VT_THREADS) void wino4_vt_kernel(Wino4Params P) {
  __shared__ floatx4 tl4[6][6][64];  // [i][x][lane]
  const scflow_conv_args& a = P.a;
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // column x, then row i
  const int tb = blockIdx.x, k = blockIdx.y, li = lane & 31, hh = lane >> 5;
  const int T = tb * W4TM + li;
  const int c = k * W4KC + 4 * hh;  // padded channel of this lane's quad
  const bool s1 = c >= P.cp0;
  const float* src = s1 ? a.src1 : a.src0;
  const int cs = s1 ? a.c1 : a.c0;
  const int ss = s1 ? a.s1 : a.s0;
  const int cc = s1 ? c - P.cp0 : c;
  const bool ok_c = T < P.ntiles && cc < cs;
  int img = 0, ty = 0, tx = 0;
  if (T < P.ntiles) {
    const int per = P.th * P.tw;
    img = T / per;
    const int r = T - img * per;
    ty = r / P.tw;
    tx = r - ty * P.tw;
  }
  const long long npix = (long long)a.n * a.h * a.w;
  const __amdgpu_buffer_rsrc_t rs =
      wino_rsrc(src, (unsigned)(((npix - 1) * ss + (cs > 0 ? cs : 0)) * 4));
  const int ix = 4 * tx - 1 + wv;
  floatx4 d[6];
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    const int iy = 4 * ty - 1 + r;
    const bool ok = ok_c && iy >= 0 && iy < a.h && ix >= 0 && ix < a.w;
    const long long pix = ((long long)img * a.h + iy) * a.w + ix;
    d[r] = wino_bload(rs, ok ? (int)((pix * ss + cc) * 4) : WINO_OOB, 0);
  }
  if (a.in_scale != nullptr && !s1 && ok_c) {  // input InstanceNorm + ReLU (zero padding stays 0)
    const floatx4 isc = *(const floatx4*)(a.in_scale + (size_t)img * a.c0 + cc);
    const floatx4 ish = *(const floatx4*)(a.in_shift + (size_t)img * a.c0 + cc);
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      const int iy = 4 * ty - 1 + r;
      if (iy >= 0 && iy < a.h && ix >= 0 && ix < a.w) {
#pragma unroll
        for (int e = 0; e < 4; ++e) d[r][e] = fmaxf(d[r][e] * isc[e] + ish[e], 0.f);
      }
    }
  }
  floatx4 col[6];
  w4_bt(d, col);
#pragma unroll
  for (int i = 0; i < 6; ++i) tl4[i][wv][lane] = col[i];
  __syncthreads();
  floatx4 trow[6], v[6];
#pragma unroll
  for (int x = 0; x < 6; ++x) trow[x] = tl4[wv][x][lane];
  w4_bt(trow, v);
  floatx4* out = (floatx4*)(P.v + ((size_t)tb * P.nsub + k) * W4P * 256) + lane;
#pragma unroll
  for (int j = 0; j < 6; ++j) out[(6 * wv + j) * 64] = v[j];
}

// Predictor contraction of one epilogue round (the XHead fusion, scflow_xhead_pred): the round's
// 16 tiles × 16 pixels × 32 hidden channels, relu(y + bias), meet in LDS (the M region, after
// every thread's reads of it), then thread (tile tl2, pixel px) contracts its pixel's 32 channels
// with the predictor weights — 18 columns (tap·2 + o) for the 3×3 two-output predictor's blocks,
// 1 for the 1×1 one-output predictor's — and stores the block's partial sums: Zf[cb][pixel][W4PZ]
// or Zm[cb − pnbf][pixel] (xhead_pred_sum_kernel adds the blocks and the taps).  The block's
// weights sit in LDS behind the M region (W4_PRED_LDS), read with wave-uniform addresses
// (broadcast); scalar loads of them ran in SGPR-sized batches, each waited on.
// Y rows: 36 floats per pixel (16-B reads of 4 channels; rows 4 banks apart), plus 8 floats per
// tile so the 4 tiles a wave writes land on different banks.
constexpr int W4YP = 36;
constexpr int W4_PRED_LDS = W4_LDS + 32 * W4PZ * 4;  // + one channel block's predictor weights
typedef float w4f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void w4_pred_round(const Wino4Params& P, const w4f2 (&y)[4][4],
                                              w4f2 bias2, int T0, int tl, int cp, int cb) {
  extern __shared__ float w4s[];
  __syncthreads();  // every thread's M reads are done: Y overwrites them
#pragma unroll
  for (int ya = 0; ya < 4; ++ya)
#pragma unroll
    for (int xb = 0; xb < 4; ++xb) {
      w4f2 v;
#pragma unroll
      for (int e = 0; e < 2; ++e) v[e] = fmaxf(y[ya][xb][e] + bias2[e], 0.f);
      *(w4f2*)(w4s + (tl * 16 + 4 * ya + xb) * W4YP + tl * 8 + 2 * cp) = v;
    }
  __syncthreads();
  const int tid = threadIdx.x;
  const int tl2 = tid >> 4, px = tid & 15;
  const int T = T0 + tl2;
  if (T >= P.ntiles) return;
  const scflow_conv_args& a = P.a;
  const int per = P.th * P.tw;
  const int img = T / per, r = T - img * per;
  const int ty = r / P.tw, tx = r - ty * P.tw;
  const long long M = (long long)a.n * a.h * a.w;
  const long long pix = ((long long)img * a.h + 4 * ty + (px >> 2)) * a.w + 4 * tx + (px & 3);
  const floatx4* yr = (const floatx4*)(w4s + (tl2 * 16 + px) * W4YP + tl2 * 8);
  const float* wl = w4s + W4_LDS / 4;
  const int cbu = __builtin_amdgcn_readfirstlane(cb);
  if (cbu < P.pnbf) {
    float z[18];
#pragma unroll
    for (int t = 0; t < 18; ++t) z[t] = 0.f;
#pragma unroll 2
    for (int c4 = 0; c4 < 8; ++c4) {  // (fully unrolled, the weight reads are hoisted: spills)
      const floatx4 yv = yr[c4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float* wc = wl + (4 * c4 + e) * W4PZ;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const floatx4 w = *(const floatx4*)(wc + 4 * k);
#pragma unroll
          for (int i = 0; i < 4; ++i) z[4 * k + i] = fmaf(yv[e], w[i], z[4 * k + i]);
        }
        const w4f2 w2 = *(const w4f2*)(wc + 16);
        z[16] = fmaf(yv[e], w2[0], z[16]);
        z[17] = fmaf(yv[e], w2[1], z[17]);
      }
    }
    float* zo = P.zp + ((size_t)cbu * M + pix) * W4PZ;
#pragma unroll
    for (int k = 0; k < 4; ++k) *(floatx4*)(zo + 4 * k) = floatx4{z[4 * k], z[4 * k + 1], z[4 * k + 2], z[4 * k + 3]};
    *(w4f2*)(zo + 16) = w4f2{z[16], z[17]};
  } else {
    float z = 0.f;
#pragma unroll
    for (int c4 = 0; c4 < 8; ++c4) {
      const floatx4 yv = yr[c4];
#pragma unroll
      for (int e = 0; e < 4; ++e) z = fmaf(yv[e], wl[(4 * c4 + e) * W4PZ], z);
    }
    P.zp[(size_t)P.pnbf * M * W4PZ + (size_t)(cbu - P.pnbf) * M + pix] = z;
  }
}

// 2. the point GEMMs + output transform.  D = sub-steps of V / U in flight per wave: 1 (two
//    workgroups per CU, each point's pair reloaded 9 points ahead) or 2 (one workgroup per CU,
//    the register budget of two, each pair reloaded 18 points ahead) — the choice for grids of
//    ≤ one workgroup per CU, where no second wave per SIMD hides the L2 / MALL latency.
template <int ACT, int D, bool PRED = false>
__global__ __launch_bounds__(256, D == 2 ? 1 : 2) void conv_wino4_kernel(Wino4Params P) {
  extern __shared__ float w4s[];  // epilogue [36][32 co][W4EP]
  const scflow_conv_args& a = P.a;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 31, hh = lane >> 5;
  int tb, cb;
  w4_block(P, tb, cb);
  const int nsub = P.nsub;  // a multiple of D (launch_wino4)
  wino_stamp(P.stamps, 0);
  const unsigned blk = (unsigned)nsub * W4P * 1024;  // bytes of one block's V / U slice
  const __amdgpu_buffer_rsrc_t vsrc = wino_rsrc(P.v + (size_t)tb * nsub * W4P * 256, blk);
  const __amdgpu_buffer_rsrc_t usrc = wino_rsrc(a.weight + (size_t)cb * nsub * W4P * 256, blk);
  const int p0 = W4NPW * wv;  // this wave's first point
  floatx4 v[D][W4NPW], u[D][W4NPW];
  floatx16 acc[W4NPW];
#pragma unroll
  for (int j = 0; j < W4NPW; ++j)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;
  auto load = [&](int k, int b, int j) __attribute__((always_inline)) {
    const int off = (k * W4P + p0 + j) * 1024;  // wave-uniform (SGPR offset)
    v[b][j] = wino_bload(vsrc, lane * 16, off);
    u[b][j] = wino_bload(usrc, lane * 16, off);
  };
#pragma unroll
  for (int b = 0; b < D; ++b)
#pragma unroll
    for (int j = 0; j < W4NPW; ++j) load(b, b, j);
  wino_stamp(P.stamps, 1);
  for (int k = 0; k < nsub; k += D) {
    auto step = [&](auto bc) __attribute__((always_inline)) {
      constexpr int b = decltype(bc)::value;
      // sub-step k + b from buffer b; the buffer's next sub-step is k + b + D (the last ones
      // reload the final sub-step: no branches)
      const int kn = k + b + D < nsub ? k + b + D : nsub - 1;
      auto point = [&](auto jc) __attribute__((always_inline)) {
        constexpr int j = decltype(jc)::value;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(v[b][j][e], u[b][j][e], acc[j], 0, 0, 0);
        load(kn, b, j);  // D · eight points' MFMAs (≈ D · 2000 cycles) to arrive
        __builtin_amdgcn_sched_barrier(0);
      };
      StaticFor<0, W4NPW>::run(point);
    };
    StaticFor<0, D>::run(step);
  }

  if (P.stamps) {
    __builtin_amdgcn_s_waitcnt(0);
    wino_stamp(P.stamps, 2);
  }
  // epilogue, 16 tiles per round (2 rounds): round q holds accumulator rows 8q..8q+7 = tiles
  // 16q + 8s + 4hh + rr (s = 0, 1), staged as M[point][tile][channel]; thread = (tile, channel
  // pair) computes the tile's whole 4×4 output for its 2 channels — every point read once (Aᵀ
  // over the rows i per column x, accumulated over x with A), where per-output-row threads
  // re-read all 36 points 4 times over.  8-B reads and stores (a wave: 4 tiles × 32 channels).
  typedef float floatx2 __attribute__((ext_vector_type(2)));
  const int per = P.th * P.tw;
  const int tl = tid >> 4, cp = tid & 15;
  const int col = cb * 32 + 2 * cp;
  const int nv = a.cout - col < 2 ? a.cout - col : 2;  // valid channels of the pair (≤ 0: none)
  const bool vo = nv == 2 && (a.so & 1) == 0 && ((uintptr_t)a.out & 7) == 0;
  auto ld2 = [&](const float* q, bool ok2) -> floatx2 {
    floatx2 r = {0.f, 0.f};
    if (ok2) return *(const floatx2*)q;
    if (nv > 0) r[0] = q[0];
    if (nv > 1) r[1] = q[1];
    return r;
  };
  const bool vb = nv == 2 && (a.sbm & 1) == 0 && ((uintptr_t)a.bias_map & 7) == 0;
  const bool vr = nv == 2 && (a.sres & 1) == 0 && ((uintptr_t)a.res & 7) == 0;
  const floatx2 zero2 = {0.f, 0.f}, one2 = {1.f, 1.f};
  const floatx2 bias2 = (nv > 0 && a.bias) ? ld2(a.bias + col, false) : zero2;
  const floatx2 osc2 = (nv > 0 && a.out_scale) ? ld2(a.out_scale + col, false) : one2;
  const floatx2 osh2 = (nv > 0 && a.out_scale) ? ld2(a.out_shift + col, false) : zero2;
  const floatx2* M2 = (const floatx2*)w4s;
  if constexpr (PRED) {  // this channel block's predictor weights behind the M region
    if (tid < 32 * W4PZ / 4)
      ((floatx4*)(w4s + W4_LDS / 4))[tid] = ((const floatx4*)(P.pw + (size_t)cb * 32 * W4PZ))[tid];
  }
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    if (q) __syncthreads();  // the previous round's reads are done
#pragma unroll
    for (int j = 0; j < W4NPW; ++j)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr)
          w4s[((p0 + j) * 16 + 8 * s2 + 4 * hh + rr) * W4CP + li] = acc[j][8 * q + 4 * s2 + rr];
    __syncthreads();
    const int T = tb * W4TM + 16 * q + tl;
    if (!PRED && (T >= P.ntiles || nv <= 0)) continue;
    // Y[ya][xb] = Σ_x (Aᵀ M)[ya][x] · Aᵀ[xb][x]; Aᵀ = [1 1 1 1 1 0; 0 1 −1 2 −½ 0; 0 1 1 4 ¼ 0;
    // 0 1 −1 8 −⅛ 1] (coefficients exact in fp32; products by ±1 fold to adds)
    constexpr float AT[4][6] = {{1.f, 1.f, 1.f, 1.f, 1.f, 0.f},
                                {0.f, 1.f, -1.f, 2.f, -0.5f, 0.f},
                                {0.f, 1.f, 1.f, 4.f, 0.25f, 0.f},
                                {0.f, 1.f, -1.f, 8.f, -0.125f, 1.f}};
    floatx2 y[4][4];
#pragma unroll
    for (int x = 0; x < 6; ++x) {
      floatx2 m[6];
#pragma unroll
      for (int i = 0; i < 6; ++i) m[i] = M2[((6 * i + x) * 16 + tl) * (W4CP / 2) + cp];
      const floatx2 s12 = m[1] + m[2], d12 = m[1] - m[2];
      floatx2 t[4];
      t[0] = m[0] + s12 + m[3] + m[4];
      t[1] = d12 + 2.f * m[3] - 0.5f * m[4];
      t[2] = s12 + 4.f * m[3] + 0.25f * m[4];
      t[3] = d12 + 8.f * m[3] - 0.125f * m[4] + m[5];
#pragma unroll
      for (int ya = 0; ya < 4; ++ya)
#pragma unroll
        for (int xb = 0; xb < 4; ++xb) {
          if (x == 0) {
            y[ya][xb] = AT[xb][0] * t[ya];
          } else if (AT[xb][x] == 1.f) {
            y[ya][xb] += t[ya];
          } else if (AT[xb][x] == -1.f) {
            y[ya][xb] -= t[ya];
          } else if (AT[xb][x] != 0.f) {
            y[ya][xb] += AT[xb][x] * t[ya];
          }
        }
    }
    if constexpr (PRED) {
      w4_pred_round(P, y, bias2, tb * W4TM + 16 * q, tl, cp, cb);
      continue;
    }
    const int img = T / per;
    const int r = T - img * per;
    const int ty = r / P.tw, tx = r - ty * P.tw;
#pragma unroll
    for (int ya = 0; ya < 4; ++ya) {
      const size_t pix0 = ((size_t)img * a.h + 4 * ty + ya) * a.w + 4 * tx;
      floatx2 val[4];
#pragma unroll
      for (int xb = 0; xb < 4; ++xb) val[xb] = (y[ya][xb] + bias2) * osc2 + osh2;
      // every global read (bias map, residual) of the row before its stores
      if (a.bias_map) {
#pragma unroll
        for (int xb = 0; xb < 4; ++xb) val[xb] += ld2(a.bias_map + (pix0 + xb) * a.sbm + col, vb);
      }
      if (a.res) {
#pragma unroll
        for (int xb = 0; xb < 4; ++xb) val[xb] += ld2(a.res + (pix0 + xb) * a.sres + col, vr);
      }
#pragma unroll
      for (int xb = 0; xb < 4; ++xb) {
        floatx2 o;
#pragma unroll
        for (int e = 0; e < 2; ++e) o[e] = act_apply(val[xb][e], ACT);
        float* dst = a.out + (pix0 + xb) * a.so + col;
        if (vo) {
          *(floatx2*)dst = o;
        } else {
#pragma unroll
          for (int e = 0; e < 2; ++e)
            if (e < nv) dst[e] = o[e];
        }
      }
    }
  }
  if (P.stamps) {
    __builtin_amdgcn_s_waitcnt(0);
    wino_stamp(P.stamps, 3);
  }
}

// U = G g Gᵀ per (co, ci) in fp64, packed [cout block][sub-step][point][lane][4] with lane =
// li + 32·hh ↔ co = 32·block + li, padded input channel 8·sub-step + 4·hh + e (source 1 from cp0)
__global__ void wino4_pack_kernel(const float* __restrict__ w, float* __restrict__ out, int cout,
                                  int c0, int c1, int cp0, int nsub, long long total) {
  const double G[6][3] = {{1., 0., 0.},
                          {-1. / 3, -1. / 3, -1. / 3},
                          {1. / 3, -1. / 3, 1. / 3},
                          {1. / 15, 2. / 15, 4. / 15},
                          {-16. / 15, 8. / 15, -4. / 15},
                          {0., 0., 1.}};
  for (long long idx = blockIdx.x * 256LL + threadIdx.x; idx < total; idx += (long long)gridDim.x * 256) {
    const int e = (int)(idx & 3), lane = (int)((idx >> 2) & 63);
    const long long rest = idx >> 8;
    const int xi = (int)(rest % W4P);
    const long long rk = rest / W4P;
    const int k = (int)(rk % nsub), cbk = (int)(rk / nsub);
    const int co = cbk * 32 + (lane & 31);
    const int kc = k * W4KC + 4 * (lane >> 5) + e;
    const int ci = kc < cp0 ? (kc < c0 ? kc : -1) : (kc - cp0 < c1 ? c0 + kc - cp0 : -1);
    double val = 0.;
    if (co < cout && ci >= 0) {
      const float* g = w + ((size_t)co * (c0 + c1) + ci) * 9;
      const int i = xi / 6, j = xi % 6;
      for (int ky = 0; ky < 3; ++ky)
        for (int kx = 0; kx < 3; ++kx) val += G[i][ky] * (double)g[ky * 3 + kx] * G[j][kx];
    }
    out[idx] = (float)val;
  }
}

long long wino4_packed_size(int cout, int c0, int c1) {
  const int nsub = (round_up(c0, W4KC) + round_up(c1, W4KC)) / W4KC;
  return (long long)(round_up(cout, 32) / 32) * nsub * W4P * 256;
}

bool wino4_shape(const scflow_conv_args& a) {
  return a.kh == 3 && a.kw == 3 && a.stride == 1 && a.ph == 1 && a.pw == 1 && a.h % 4 == 0 &&
         a.w % 4 == 0 && a.c0 % 4 == 0 && a.c1 % 4 == 0 && a.epilogue == SCFLOW_EPI_PLAIN &&
         (a.c1 == 0 || a.in_scale == nullptr);
}

long long wino4_workspace_bytes(const scflow_conv_args& a) {
  const long long ntiles = (long long)a.n * (a.h / 4) * (a.w / 4);
  const long long ntb = (ntiles + W4TM - 1) / W4TM;
  const int nsub = (round_up(a.c0, W4KC) + round_up(a.c1, W4KC)) / W4KC;
  return ntb * nsub * W4P * 1024;
}

template <int ACT, int D>
void w4_set_lds() {
  (void)hipFuncSetAttribute((const void*)conv_wino4_kernel<ACT, D>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

template <int D>
int launch_wino4_gemm(const Wino4Params& p, dim3 grid, hipStream_t st) {
  static bool attr = false;
  if (!attr) {  // W4_LDS > 64 KiB: opt every instantiation in once
    w4_set_lds<SCFLOW_ACT_RELU, D>();
    w4_set_lds<SCFLOW_ACT_SIGMOID, D>();
    w4_set_lds<SCFLOW_ACT_TANH, D>();
    w4_set_lds<SCFLOW_ACT_NONE, D>();
    attr = true;
  }
  switch (p.a.act) {  // the activation as a template argument: one epilogue body per kernel
    case SCFLOW_ACT_RELU: conv_wino4_kernel<SCFLOW_ACT_RELU, D><<<grid, 256, W4_LDS, st>>>(p); break;
    case SCFLOW_ACT_SIGMOID: conv_wino4_kernel<SCFLOW_ACT_SIGMOID, D><<<grid, 256, W4_LDS, st>>>(p); break;
    case SCFLOW_ACT_TANH: conv_wino4_kernel<SCFLOW_ACT_TANH, D><<<grid, 256, W4_LDS, st>>>(p); break;
    default: conv_wino4_kernel<SCFLOW_ACT_NONE, D><<<grid, 256, W4_LDS, st>>>(p); break;
  }
  return scflow_launch_status();
}

// the input transform launch and the GEMM's parameters / grid (launch_wino4, launch_xhead_pred)
int wino4_prepare(const scflow_conv_args& a, hipStream_t st, Wino4Params& p, dim3& grid) {
  if (!wino4_shape(a)) return SCFLOW_EUNSUPPORTED;
  if (!a.ws || a.ws_bytes < wino4_workspace_bytes(a)) return SCFLOW_EINVAL;
  if (!aligned16(a.src0) || (a.s0 & 3) || (a.c1 > 0 && (!aligned16(a.src1) || (a.s1 & 3))) ||
      !aligned16(a.weight) || !aligned16(a.ws))
    return SCFLOW_EALIGN;
  p = Wino4Params{};
  p.a = a;
  p.v = a.ws;
  p.cp0 = round_up(a.c0, W4KC);
  p.nsub = (p.cp0 + round_up(a.c1, W4KC)) / W4KC;
  p.th = a.h / 4;
  p.tw = a.w / 4;
  const long long ntiles = (long long)a.n * p.th * p.tw;
  if (ntiles >= (1LL << 30) || (long long)p.nsub * W4P * 1024 >= (1LL << 31)) return SCFLOW_EUNSUPPORTED;
  p.ntiles = (int)ntiles;
  p.ntb = (int)((ntiles + W4TM - 1) / W4TM);
  p.stamps = g_wino_stamps;
  wino4_vt_kernel<<<dim3(p.ntb, p.nsub), W4VT_THREADS, 0, st>>>(p);
  const int e = scflow_launch_status();
  if (e) return e;
  grid = dim3(p.ntb, round_up(a.cout, 32) / 32);
  // XCD-blocked order (w4_block) for grids of more than one round of two workgroups per CU:
  // ≈ 64 workgroups (an XCD's 32 CUs × 2) per block, channel blocks up to 8, tile blocks a power
  // of two.  Measured (round 6, profiles/r06/g2): configs[4] memory-side traffic of the
  // transform + GEMM pair 10.0× → 5.6× its algorithmic bytes, corr_net.1 465 → 412 µs and the
  // heads conv 455 → 431 µs alone, decoder 8.69k → 8.91k iters/s; configs[1] (one round or
  // less) ±1 µs, so its grids keep the linear order.  SCFLOW_WINO4_XCD = 0 off, 2 every grid.
  static EnvSwitch xcd_sw("SCFLOW_WINO4_XCD", 1);
  const long long nwg = (long long)grid.x * grid.y;
  p.xgt = p.xgc = 0;
  if (xcd_sw.get() && nwg % 8 == 0 && (xcd_sw.get() == 2 || nwg > 2LL * device_cus())) {
    int gc = 1;
    for (int c = (int)grid.y < 8 ? (int)grid.y : 8; c >= 1; --c)
      if (grid.y % c == 0) { gc = c; break; }
    int gt = 1;
    while (gt * 2 * gc <= 64 && grid.x % (gt * 2) == 0) gt *= 2;
    const long long nblk = ((long long)grid.x / gt) * (grid.y / gc);
    if (gt * gc >= 16 && nblk >= 1) { p.xgt = gt; p.xgc = gc; }
  }
  return 0;
}

// two sub-steps in flight when the grid leaves CUs with a single workgroup
// (SCFLOW_WINO4_DEPTH = 1 / 2 forces one)
bool wino4_depth2(const Wino4Params& p, dim3 grid) {
  static EnvSwitch depth_sw("SCFLOW_WINO4_DEPTH", 0);
  const int depth_env = depth_sw.get();
  return p.nsub % 2 == 0 && (depth_env == 2 || (depth_env != 1 && (long long)grid.x * grid.y <= 256));
}

int launch_wino4(const scflow_conv_args& a, hipStream_t st) {
  Wino4Params p;
  dim3 grid;
  const int e = wino4_prepare(a, st, p, grid);
  if (e) return e;
  return wino4_depth2(p, grid) ? launch_wino4_gemm<2>(p, grid, st) : launch_wino4_gemm<1>(p, grid, st);
}
