// Channels-last fp32 convolutions of the SCFlow update block, with fused epilogues.
//
// Reference modules replaced (all mmcv ConvModule = conv + bias + act, /root/reference):
//   ConvGRU SeqConv (1×5 then 5×1, z/r/q gates)      models/decoder/raft_decoder.py:180-253
//   MotionEncoder corr_net / flow_net / out_net       models/decoder/raft_decoder.py:75-166
//   XHead flow / mask                                  models/decoder/raft_decoder.py:256-294
//   delta_flow_encoder / mask_encoder                  models/decoder/scflow_decoder.py:103-124
//
// Three kernel families, chosen by shape (select_variant, shared by packing and launching):
//
//  * conv_mfma — implicit GEMM on v_mfma_f32_32x32x2_f32 (exact fp32; gfx950's only f32 matrix
//    rate).  Workgroup tile = 128 output pixels (128/W whole image rows) × 64 output channels;
//    4 waves, each 64 px × 32 ch (two 32×32 accumulators).  K is walked in stages of 16 input
//    channels of one source; per stage the workgroup stages the input HALO of its rows once —
//    (rows+kh−1)×(W+kw−1) pixels — plus the stage's weights for every tap (packed contiguous per
//    stage, so that is one coalesced block), and all kh·kw taps then run out of LDS (pixel rows
//    padded to 20 floats: ds_read_b128 conflict-free).  Software pipeline: the next stage's
//    global loads are issued into registers before this stage's MFMAs and written to LDS after
//    them, so L2/HBM latency hides under ≥ 2.5k cycles of matrix work.  A second input source
//    is a channel concat without a copy (GRU cat[h,x] / cat[r·h,x], MotionEncoder cat[c,f]).
//    Epilogues: bias+act; GRU ZR writes z and r·h; GRU Q computes h ← (1−z)·h + z·tanh(q) in
//    place (the reference's three ConvModules + elementwise ops in two launches).
//  * conv_smallcin — cin ≤ 4 (7×7 2→128 flow encoders, 3×3 1→64 mask encoder): on MFMA with
//    K = taps·cin in k-pairs (conv_smallcin_mfma_kernel) for W ∈ {32, 64}; otherwise one LANE
//    per output channel with its kh·kw·cin weights in VGPRs, the input halo in LDS read as
//    wave-uniform broadcasts.
//  * conv_thin — cout ≤ 4 (flow head 3×3 256→2, mask head 1×1 256→1): one LANE per output
//    pixel, channels streamed through an LDS halo in chunks of 32, weights wave-uniform.
#include "common.h"

#include <stdlib.h>

namespace {

constexpr int BM = 128;  // output pixels per workgroup (mfma)
constexpr int BN = 64;   // output channels per workgroup (mfma)
constexpr int BK = 16;   // default input channels per K-stage (mfma); 8 on request (scflow_conv_args.bk)
constexpr int CPAD = 16; // each source's channels are padded to a multiple of 16 (either depth)
constexpr int THIN_CC = 32;        // channels per LDS chunk (thin)
constexpr int THIN_LD = THIN_CC + 4;

enum Variant { V_MFMA = 0, V_SMALLCIN = 1, V_THIN = 2, V_NONE = -1 };

struct Geometry {
  int variant;
  int oh, ow, tr, hr, hc, taps, cp0, cp1, nst, ktot, npad;
  size_t lds;
};

int round_up(int a, int b) { return (a + b - 1) / b * b; }

bool mfma_shape(int kh, int kw) {
  return (kh == 1 && kw == 1) || (kh == 3 && kw == 3) || (kh == 1 && kw == 5) || (kh == 5 && kw == 1);
}

Geometry select_variant(int cout, int c0, int c1, int kh, int kw, int stride, int h, int w, int ph,
                        int pw) {
  Geometry g{};
  g.variant = V_NONE;
  g.taps = kh * kw;
  g.oh = (h + 2 * ph - kh) / stride + 1;
  g.ow = (w + 2 * pw - kw) / stride + 1;
  if (stride != 1) return g;
  const int cin = c0 + c1;
  if (cin <= 4 && c1 == 0) {
    g.variant = V_SMALLCIN;
    g.ktot = g.taps * cin;
    g.npad = round_up(cout, 64);
    return g;
  }
  if (cout <= 4) {
    if (cin % 4 || c0 % 4) return g;
    g.variant = V_THIN;
    g.ktot = g.taps * cin;
    g.npad = cout;
    return g;
  }
  if (c0 % 4 || c1 % 4 || !mfma_shape(kh, kw)) return g;
  if (w != g.ow || h != g.oh || (g.ow != 32 && g.ow != 64)) return g;  // tile = whole rows
  g.tr = BM / g.ow;
  if (g.oh % g.tr) return g;
  g.hr = g.tr + kh - 1;
  g.hc = g.ow + kw - 1;
  g.cp0 = round_up(c0, CPAD);
  g.cp1 = round_up(c1, CPAD);
  g.nst = (g.cp0 + g.cp1) / BK;
  g.ktot = g.taps * (g.cp0 + g.cp1);
  g.npad = round_up(cout, BN);
  g.variant = V_MFMA;
  return g;
}

// ------------------------------------------------------------------------------------------
// MFMA implicit-GEMM conv
// packed weights: [npad/BN][nst][taps][BN][bk] — one contiguous block per (n-tile, stage),
// bk = the stage depth the weights are packed for (16 by default, 8 on request)
// ------------------------------------------------------------------------------------------
struct MfmaParams {
  scflow_conv_args a;
  int oh, ow, tr, hr, hc, cp0, nst;
};

// max float4 of the A halo per thread over the supported widths (32, 64)
constexpr int na_max(int bm, int kh, int kw, int bk) {
  const int a32 = (bm / 32 + kh - 1) * (32 + kw - 1) * (bk / 4);
  const int a64 = ((bm / 64 > 0 ? bm / 64 : 1) + kh - 1) * (64 + kw - 1) * (bk / 4);
  const int m = a32 > a64 ? a32 : a64;
  return (m + 255) / 256;
}

// TILE_M output pixels × BN channels per workgroup; 4 waves as 2 (M) × 2 (N); each wave owns
// TILE_M/2 pixels (RB = TILE_M/64 row blocks of 32) × 32 channels.
// BKS = stage depth: 16 (fewer barriers per MFMA) or 8 (half the LDS, so more workgroups are
// resident when the grid needs it; the weights must then be packed with bk = 8).
template <int EPI, int KH, int KW, int TILE_M, int BKS>
__global__ __launch_bounds__(256, 2) void conv_mfma_kernel(MfmaParams P) {
  constexpr int BK = BKS;
  constexpr int LDA = BK + 4;
  constexpr int TAPS = KH * KW;
  constexpr int RB = TILE_M / 64;
  constexpr int NA = na_max(TILE_M, KH, KW, BK);
  constexpr int NBT = TAPS * BN * (BK / 4);  // float4 of one stage's weights
  constexpr int NB = (NBT + 255) / 256;
  extern __shared__ float smem[];
  const scflow_conv_args& a = P.a;
  const int hc = P.hc, ow = P.ow;
  float* As = smem;                             // [hr*hc][LDA]
  float* Bs = smem + (size_t)P.hr * hc * LDA;   // [TAPS][BN][LDA]
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave & 1, wn = wave >> 1, li = lane & 31, hh = lane >> 5;
  const int tiles_per_img = P.oh / P.tr;
  const int img = blockIdx.x / tiles_per_img;
  const int oy0 = (blockIdx.x % tiles_per_img) * P.tr;
  const int n0 = blockIdx.y * BN;
  const int na = P.hr * hc * (BK / 4);
  const int nst0 = P.cp0 / BK;

  // stage-invariant halo addressing, computed once: input pixel index (or -1 = zero padding)
  int apix[NA], acq[NA];
#pragma unroll
  for (int j = 0; j < NA; ++j) {
    const int idx = tid + 256 * j;
    const int q = idx % (BK / 4), pix = idx / (BK / 4);
    const int hr = pix / hc, hcol = pix - hr * hc;
    const int iy = oy0 - a.ph + hr, ix = hcol - a.pw;
    const bool ok = idx < na && iy >= 0 && iy < a.h && ix >= 0 && ix < a.w;
    apix[j] = ok ? (img * a.h + iy) * a.w + ix : -1;
    acq[j] = 4 * q;
  }

  floatx4 ra[NA], rb[NB];
  auto gload = [&](int s) {
    const bool s1 = s >= nst0;
    const float* src = s1 ? a.src1 : a.src0;
    const int cs = s1 ? a.c1 : a.c0;
    const int ss = s1 ? a.s1 : a.s0;
    const int cc = (s1 ? s - nst0 : s) * BK;
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      floatx4 v = {0.f, 0.f, 0.f, 0.f};
      const int c = cc + acq[j];
      if (apix[j] >= 0 && c < cs) v = *(const floatx4*)(src + (size_t)apix[j] * ss + c);
      ra[j] = v;
    }
    const float* wb = a.weight + ((size_t)blockIdx.y * P.nst + s) * (TAPS * BN * BK);
#pragma unroll
    for (int j = 0; j < NB; ++j)
      if (NBT % 256 == 0 || tid + 256 * j < NBT) rb[j] = *(const floatx4*)(wb + (size_t)(tid + 256 * j) * 4);
  };
  auto lstore = [&]() {
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      const int idx = tid + 256 * j;
      if (idx < na) *(floatx4*)(As + (idx / (BK / 4)) * LDA + 4 * (idx % (BK / 4))) = ra[j];
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int idx = tid + 256 * j;
      if (NBT % 256 == 0 || idx < NBT) *(floatx4*)(Bs + (idx / (BK / 4)) * LDA + 4 * (idx % (BK / 4))) = rb[j];
    }
  };

  // this lane's RB A rows (output pixels) as halo offsets
  int abase[RB];
#pragma unroll
  for (int r = 0; r < RB; ++r) {
    const int m = wm * (TILE_M / 2) + r * 32 + li;
    abase[r] = ((m / ow) * hc + (m % ow)) * LDA + 4 * hh;
  }
  const int bbase = (wn * 32 + li) * LDA + 4 * hh;

  floatx16 acc[RB];
#pragma unroll
  for (int r = 0; r < RB; ++r)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[r][e] = 0.f;

  gload(0);
  for (int s = 0; s < P.nst; ++s) {
    __syncthreads();
    lstore();
    __syncthreads();
    if (s + 1 < P.nst) gload(s + 1);
#pragma unroll
    for (int ty = 0; ty < KH; ++ty) {
#pragma unroll
      for (int tx = 0; tx < KW; ++tx) {
        const int aoff = (ty * hc + tx) * LDA;
        const float* Bb = Bs + (ty * KW + tx) * BN * LDA + bbase;
#pragma unroll
        for (int kb = 0; kb < BK; kb += 8) {
          floatx4 av[RB];
#pragma unroll
          for (int r = 0; r < RB; ++r) av[r] = *(const floatx4*)(As + abase[r] + aoff + kb);
          const floatx4 b0 = *(const floatx4*)(Bb + kb);
#pragma unroll
          for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int r = 0; r < RB; ++r)
              acc[r] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[r][e], b0[e], acc[r], 0, 0, 0);
        }
      }
    }
  }

  // epilogue; C/D layout: col = lane&31, row = (r&3) + 8(r>>2) + 4(lane>>5).
  // All global reads (bias map, h, z) are issued before any store: the stores may alias them
  // as far as the compiler knows, so interleaving would serialise every read's latency.
  const int col = n0 + wn * 32 + li;
  if (col >= a.cout) return;
  const float bias = a.bias ? a.bias[col] : 0.f;
  size_t pixv[RB][16];
#pragma unroll
  for (int rr = 0; rr < RB; ++rr)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = wm * (TILE_M / 2) + rr * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
      pixv[rr][r] = ((size_t)img * P.oh + oy0 + m / ow) * ow + m % ow;
    }
  if (a.bias_map) {
#pragma unroll
    for (int rr = 0; rr < RB; ++rr)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[rr][r] += a.bias_map[pixv[rr][r] * a.sbm + col];
  }
  if constexpr (EPI == SCFLOW_EPI_PLAIN) {
#pragma unroll
    for (int rr = 0; rr < RB; ++rr)
#pragma unroll
      for (int r = 0; r < 16; ++r) a.out[pixv[rr][r] * a.so + col] = act_apply(acc[rr][r] + bias, a.act);
  } else if constexpr (EPI == SCFLOW_EPI_GRU_ZR) {
    const int hcn = a.cout >> 1;
    if (col < hcn) {
#pragma unroll
      for (int rr = 0; rr < RB; ++rr)
#pragma unroll
        for (int r = 0; r < 16; ++r) a.gate[pixv[rr][r] * a.sg + col] = sigmoidf_(acc[rr][r] + bias);
    } else {
      const int c = col - hcn;
      float hv[RB][16];
#pragma unroll
      for (int rr = 0; rr < RB; ++rr)
#pragma unroll
        for (int r = 0; r < 16; ++r) hv[rr][r] = a.hid[pixv[rr][r] * a.sh + c];
#pragma unroll
      for (int rr = 0; rr < RB; ++rr)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          a.rh[pixv[rr][r] * a.srh + c] = sigmoidf_(acc[rr][r] + bias) * hv[rr][r];
    }
  } else {  // GRU_Q
    float zv[RB][16], hv[RB][16];
#pragma unroll
    for (int rr = 0; rr < RB; ++rr)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        zv[rr][r] = a.gate[pixv[rr][r] * a.sg + col];
        hv[rr][r] = a.hid[pixv[rr][r] * a.sh + col];
      }
#pragma unroll
    for (int rr = 0; rr < RB; ++rr)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float q = tanhf_(acc[rr][r] + bias);
        a.hid[pixv[rr][r] * a.sh + col] = (1.f - zv[rr][r]) * hv[rr][r] + zv[rr][r] * q;
      }
  }
}

// ------------------------------------------------------------------------------------------
// 1×1 stride-1 conv (MotionEncoder corr_net.0 324 → 256, raft_decoder.py:75-85; the training
// step's 1×1 forward / dX convs): the GEMM over 128 consecutive pixel rows × 64 output channels,
// same packed weights and stage pipeline as conv_mfma_kernel<·,1,1,128,16> but without its halo
// machinery — rows are contiguous, so a stage's A tile is 128 rows × 16 channels of one source
// (two float4 per thread) and the epilogue addresses rows directly (32 vs 38 µs at corr_net.0's
// shape, tools/micro/conv1x1_variants.hip).  Plain epilogue: bias, bias map, activation.
__global__ __launch_bounds__(256, 2) void conv1x1_kernel(MfmaParams P) {
  constexpr int TM = 128, LDA = BK + 4;
  __shared__ float As[TM * LDA];
  __shared__ float Bs[BN * LDA];
  const scflow_conv_args& a = P.a;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave & 1, wn = wave >> 1, li = lane & 31, hh = lane >> 5;
  const int m0 = blockIdx.x * TM;
  const long long M = (long long)a.n * a.h * a.w;
  const int nst0 = P.cp0 / BK;
  floatx4 ra[2], rb;
  auto gload = [&](int s) __attribute__((always_inline)) {
    const bool s1 = s >= nst0;
    const float* src = s1 ? a.src1 : a.src0;
    const int cs = s1 ? a.c1 : a.c0;
    const int ss = s1 ? a.s1 : a.s0;
    const int cc = (s1 ? s - nst0 : s) * BK;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int idx = tid + 256 * j;
      const long long m = m0 + (idx >> 2);
      const int c = cc + 4 * (idx & 3);
      floatx4 v = {0.f, 0.f, 0.f, 0.f};
      if (m < M && c < cs) v = *(const floatx4*)(src + m * ss + c);
      ra[j] = v;
    }
    rb = *(const floatx4*)(a.weight + ((size_t)blockIdx.y * P.nst + s) * (BN * BK) + (size_t)tid * 4);
  };
  auto lstore = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int idx = tid + 256 * j;
      *(floatx4*)(As + (idx >> 2) * LDA + 4 * (idx & 3)) = ra[j];
    }
    *(floatx4*)(Bs + (tid >> 2) * LDA + 4 * (tid & 3)) = rb;
  };
  floatx16 acc[2];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[r][e] = 0.f;
  const int abase = (wm * 64 + li) * LDA + 4 * hh, bbase = (wn * 32 + li) * LDA + 4 * hh;
  gload(0);
  for (int s = 0; s < P.nst; ++s) {
    __syncthreads();
    lstore();
    __syncthreads();
    if (s + 1 < P.nst) gload(s + 1);
#pragma unroll
    for (int kb = 0; kb < BK; kb += 8) {
      const floatx4 a0 = *(const floatx4*)(As + abase + kb);
      const floatx4 a1 = *(const floatx4*)(As + abase + 32 * LDA + kb);
      const floatx4 b0 = *(const floatx4*)(Bs + bbase + kb);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[e], b0[e], acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[e], b0[e], acc[1], 0, 0, 0);
      }
    }
  }
  // epilogue; C/D layout: col = lane&31, row = (r&3) + 8(r>>2) + 4(lane>>5); all global reads
  // (bias map) before any store
  const int col = blockIdx.y * BN + wn * 32 + li;
  if (col >= a.cout) return;
  const float bias = a.bias ? a.bias[col] : 0.f;
  float v[2][16];
#pragma unroll
  for (int rr = 0; rr < 2; ++rr)
#pragma unroll
    for (int r = 0; r < 16; ++r) v[rr][r] = acc[rr][r] + bias;
  if (a.bias_map) {
#pragma unroll
    for (int rr = 0; rr < 2; ++rr)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const long long m = m0 + wm * 64 + rr * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
        if (m < M) v[rr][r] += a.bias_map[m * a.sbm + col];
      }
  }
#pragma unroll
  for (int rr = 0; rr < 2; ++rr)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const long long m = m0 + wm * 64 + rr * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
      if (m < M) a.out[m * a.so + col] = act_apply(v[rr][r], a.act);
    }
}

// ------------------------------------------------------------------------------------------
// small-cin conv: lane = output channel, weights in VGPRs, input halo in LDS (broadcast reads)
// packed weights: [taps*cin][npad]  (channel-contiguous)
// block: 256 threads; tile = 32 consecutive output pixels of one row; wave w handles channel
// group (w % G) (G = npad/64 ≤ 4) and a share of the 32 pixels.
// ------------------------------------------------------------------------------------------
template <int CIN, int KH, int KW>
__global__ __launch_bounds__(256) void conv_smallcin_kernel(scflow_conv_args a, int oh, int ow,
                                                            int npad) {
  constexpr int HCOLS = 32 + KW - 1;
  __shared__ float halo[KH][HCOLS][CIN];
  const int tiles_x = (ow + 31) / 32;
  const int t = blockIdx.x;
  const int tx0 = (t % tiles_x) * 32;
  const int oy = (t / tiles_x) % oh;
  const int img = t / (tiles_x * oh);
  for (int i = threadIdx.x; i < KH * HCOLS * CIN; i += 256) {
    const int c = i % CIN, col = (i / CIN) % HCOLS, row = i / (CIN * HCOLS);
    const int iy = oy - a.ph + row, ix = tx0 - a.pw + col;
    float v = 0.f;
    if (iy >= 0 && iy < a.h && ix >= 0 && ix < a.w) v = a.src0[((size_t)(img * a.h + iy) * a.w + ix) * a.s0 + c];
    halo[row][col][c] = v;
  }
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int G = npad / 64;               // channel groups (1, 2 or 4)
  const int grp = wave % G;
  const int pshare = 4 / G;              // waves per channel group
  const int pw_ = 32 / pshare;           // pixels per wave
  const int p0 = (wave / G) * pw_;
  const int co = grp * 64 + lane;
  float wr[KH * KW * CIN];
#pragma unroll
  for (int k = 0; k < KH * KW * CIN; ++k) wr[k] = a.weight[(size_t)k * npad + co];
  const float bias = (a.bias && co < a.cout) ? a.bias[co] : 0.f;
  __syncthreads();
  for (int p = p0; p < p0 + pw_; ++p) {
    const int ox = tx0 + p;
    if (ox >= ow) break;
    float acc = bias;
#pragma unroll
    for (int ty = 0; ty < KH; ++ty)
#pragma unroll
      for (int tx = 0; tx < KW; ++tx)
#pragma unroll
        for (int c = 0; c < CIN; ++c) acc += wr[(ty * KW + tx) * CIN + c] * halo[ty][p + tx][c];
    if (co < a.cout) a.out[((size_t)(img * oh + oy) * ow + ox) * a.so + co] = act_apply(acc, a.act);
  }
}

// profiling (scflow_debug_conv_stamps): 4 real-time-clock stamps per workgroup of the next
// instrumented launches (F(2×2,3×3), F(4,5), F(4×4,3×3), small-cin MFMA), or NULL
static unsigned long long* g_wino_stamps = nullptr;
__device__ __forceinline__ void sc_stamp(unsigned long long* st, int k) {
  if (st && threadIdx.x == 0)
    st[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 4 + k] = __builtin_amdgcn_s_memrealtime();
}
__device__ __forceinline__ void sc_stamp_id(unsigned long long* st, int sid, int k) {
  if (st && threadIdx.x == 0) st[(size_t)sid * 4 + k] = __builtin_amdgcn_s_memrealtime();
}

// small-cin conv on MFMA: K = taps·cin (≤ 98) walked in k-pairs — one v_mfma_f32_32x32x2_f32
// per pair (for cin = 2 a pair is the two channels of one tap, for cin = 1 two taps).  Tile =
// 64 output pixels (64/W whole rows) × npad (64 or 128) channels; 4 waves as 2 (M) × 2 (N), each
// 32 px × npad/2 channels.  The wave's B fragments (its columns' weights for every k) are loaded
// once into VGPRs from the small-cin packing [taps·cin][npad]; the tile's input halo
// (rows+kh−1)×(W+kw−1)×cin sits in LDS.
// Round 6: a workgroup walks tiles blockIdx.x, +gridDim.x, … (the grid is capped at a few
// workgroups per CU, SCFLOW_SMALLCIN_WGS): at 64×64 maps one tile per workgroup meant 2048
// short-lived workgroups (prologue, 98 MFMAs, epilogue ≈ 11 µs each) dispatched in 4 rounds of
// 512 — 57 µs alone, 214 µs in the decoder beside other kernels.  Walking tiles, the weights are
// loaded once per workgroup and the next tile's halo is in flight (registers, then the other LDS
// buffer) during this tile's MFMAs and stores: one barrier per tile.
// body: workgroup blk of nblk walking tiles, channel slice cby (grid.y of the split launch),
// stamps at slot sid (conv_pair.h launches two bodies in one grid)
template <int CIN, int KH, int KW, int NBW>
__device__ __forceinline__ void conv_smallcin_mfma_body(const scflow_conv_args& a, int oh, int ow,
                                                        int npad, int ntiles, int blk, int nblk,
                                                        int cby, unsigned long long* stamps,
                                                        int sid) {
  constexpr int K = KH * KW * CIN;
  constexpr int KP = (K + 1) / 2;  // MFMA k-steps
  extern __shared__ float halo[];  // 2 × [(tr+KH-1)][(ow+KW-1)][CIN]
  const int tr = 64 / ow;
  const int hc = ow + KW - 1, hr = tr + KH - 1;
  const int tiles_per_img = oh / tr;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave & 1, wn = wave >> 1, li = lane & 31, hh = lane >> 5;
  const int cb = cby * NBW * 64;  // channel slice of this workgroup (grid.y splits npad)
  sc_stamp_id(stamps, sid, 0);
  // the halo's global loads (at most SC_NH per thread: W 32 → (KH+1) × (31+KW) · CIN floats,
  // W 64 → KH × (63+KW) · CIN, the only widths dispatched here) as buffer loads: a padding or
  // tail element reads offset 0x7ffffff0, beyond the resource, as 0 — no branches, whose waits
  // would serialise the loads (the dispatch keeps offsets < 2^31)
  constexpr int SC_H32 = (KH + 1) * (31 + KW) * CIN, SC_H64 = KH * (63 + KW) * CIN;
  constexpr int SC_NH = ((SC_H32 > SC_H64 ? SC_H32 : SC_H64) + 255) / 256;
  const int nh = hr * hc * CIN;
  const __amdgpu_buffer_rsrc_t hsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(a.src0), (short)0,
      (int)((((long long)a.n * a.h * a.w - 1) * a.s0 + CIN) * 4), 0x00020000);
  float hv[SC_NH];
  auto hfetch = [&](int t) __attribute__((always_inline)) {
    const int img = t / tiles_per_img;
    const int oy0 = (t - img * tiles_per_img) * tr;
#pragma unroll
    for (int j = 0; j < SC_NH; ++j) {
      const int i = threadIdx.x + 256 * j;
      const int c = i % CIN, col = (i / CIN) % hc, row = i / (CIN * hc);
      const int iy = oy0 - a.ph + row, ix = col - a.pw;
      const bool ok = i < nh && iy >= 0 && iy < a.h && ix >= 0 && ix < a.w;
      const int off = ok ? (((img * a.h + iy) * a.w + ix) * a.s0 + c) * 4 : 0x7ffffff0;
      hv[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(hsrc, off, 0, 0));
    }
  };
  auto hput = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < SC_NH; ++j) {
      const int i = threadIdx.x + 256 * j;
      if (i < nh) halo[buf * nh + i] = hv[j];
    }
  };
  int t = blk;
  hfetch(t);
  // B fragments (k = 2·kp + hh, column = cb + wn·NBW·32 + nb·32 + li) and the bias, in flight
  // together with the first halo
  float bw[NBW][KP], bias_v[NBW];
#pragma unroll
  for (int nb = 0; nb < NBW; ++nb) {
    const int col = cb + (wn * NBW + nb) * 32 + li;
    bias_v[nb] = a.bias && col < a.cout ? a.bias[col] : 0.f;
#pragma unroll
    for (int kp = 0; kp < KP; ++kp) {
      const int k = 2 * kp + hh;
      bw[nb][kp] = k < K ? a.weight[(size_t)k * npad + cb + (wn * NBW + nb) * 32 + li] : 0.f;
    }
  }
  hput(0);
  __syncthreads();
  sc_stamp_id(stamps, sid, 1);
  const int m = wm * 32 + li;  // this lane's A row (output pixel of the tile)
  const int pbase = ((m / ow) * hc + (m % ow)) * CIN;
  // epilogue; C/D layout: col = lane&31, row = (r&3) + 8(r>>2) + 4(lane>>5).  The activation is
  // a template constant of the store loop (one branch-free body per activation)
  // A tile is 64 consecutive pixels of the flattened (image, row, column) order (64/W whole
  // rows), so the lane's output row r is pixel 64·t + wm·32 + 4·hh + (r&3) + 8(r>>2): one base
  // address per tile and wave-uniform offsets (nothing per element for the compiler to hoist
  // out of the tile loop into registers)
  auto store = [&](auto actc, const floatx16(&acc)[NBW], int t) __attribute__((always_inline)) {
    constexpr int ACT = decltype(actc)::value;
    float* ob = a.out + ((size_t)t * 64 + wm * 32 + 4 * hh) * a.so + cb + wn * NBW * 32 + li;
#pragma unroll
    for (int nb = 0; nb < NBW; ++nb) {
      if (cb + (wn * NBW + nb) * 32 + li < a.cout) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          ob[(size_t)((r & 3) + 8 * (r >> 2)) * a.so + nb * 32] = act_apply(acc[nb][r] + bias_v[nb], ACT);
      }
    }
  };
  // (the stride as a wave-uniform value: as a plain int argument the compiler kept the tile
  // loop's state in VGPRs — 256 registers and spills for the 7×7)
  const int stride = __builtin_amdgcn_readfirstlane(nblk);
  for (int it = 0; t < ntiles; ++it, t += stride) {
    const int buf = it & 1;
    const int tn = t + stride;
    const bool more = tn < ntiles;  // workgroup-uniform
    if (more) hfetch(tn);           // the next tile's halo in flight under this tile's MFMAs
    __builtin_amdgcn_sched_barrier(0);
    const float* hb = halo + buf * nh;
    floatx16 acc[NBW];
#pragma unroll
    for (int nb = 0; nb < NBW; ++nb)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[nb][e] = 0.f;
    // k-steps in groups of 7 behind scheduling barriers: the A reads of a group are issued
    // together, but not all 49 of a 7×7 at once (49 VGPRs of prefetch on top of the 98 B
    // fragments pushed the kernel to 256 VGPRs and spills)
    auto kstep = [&](auto kpc) __attribute__((always_inline)) {
      constexpr int kp = decltype(kpc)::value;
      const int k = 2 * kp + hh;
      const int tap = (k < K ? k : 0) / CIN, c = (k < K ? k : 0) % CIN;
      const float av = k < K ? hb[pbase + ((tap / KW) * hc + tap % KW) * CIN + c] : 0.f;
#pragma unroll
      for (int nb = 0; nb < NBW; ++nb)
        acc[nb] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bw[nb][kp], acc[nb], 0, 0, 0);
      if constexpr (kp % 7 == 6) __builtin_amdgcn_sched_barrier(0);
    };
    StaticFor<0, KP>::run(kstep);
    switch (a.act) {
      case SCFLOW_ACT_RELU: store(std::integral_constant<int, SCFLOW_ACT_RELU>{}, acc, t); break;
      case SCFLOW_ACT_SIGMOID: store(std::integral_constant<int, SCFLOW_ACT_SIGMOID>{}, acc, t); break;
      case SCFLOW_ACT_TANH: store(std::integral_constant<int, SCFLOW_ACT_TANH>{}, acc, t); break;
      default: store(std::integral_constant<int, SCFLOW_ACT_NONE>{}, acc, t); break;
    }
    if (more) hput(buf ^ 1);  // its readers finished with buf ^ 1 before the last barrier
    __syncthreads();
  }
  if (stamps) {
    sc_stamp_id(stamps, sid, 2);
    __builtin_amdgcn_s_waitcnt(0);
    sc_stamp_id(stamps, sid, 3);
  }
}

template <int CIN, int KH, int KW, int NBW>
__global__ __launch_bounds__(256, 2) void conv_smallcin_mfma_kernel(scflow_conv_args a, int oh, int ow,
                                                                 int npad, int ntiles,
                                                                 unsigned long long* stamps) {
  conv_smallcin_mfma_body<CIN, KH, KW, NBW>(a, oh, ow, npad, ntiles, blockIdx.x, gridDim.x,
                                            blockIdx.y, stamps,
                                            blockIdx.y * gridDim.x + blockIdx.x);
}

// generic small-cin fallback (any kernel size): thread = pixel, 16 channels per thread
template <int CIN>
__global__ __launch_bounds__(256) void conv_smallcin_generic(scflow_conv_args a, int oh, int ow,
                                                             int npad) {
  const long long M = (long long)a.n * oh * ow;
  const long long pix = blockIdx.x * 256LL + threadIdx.x;
  const int co0 = blockIdx.y * 16;
  if (pix >= M) return;
  const int ox = (int)(pix % ow);
  const long long t = pix / ow;
  const int oy = (int)(t % oh);
  const int img = (int)(t / oh);
  float acc[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) acc[j] = (a.bias && co0 + j < a.cout) ? a.bias[co0 + j] : 0.f;
  for (int ty = 0; ty < a.kh; ++ty) {
    const int iy = oy - a.ph + ty;
    for (int tx = 0; tx < a.kw; ++tx) {
      const int ix = ox - a.pw + tx;
      const bool ok = iy >= 0 && iy < a.h && ix >= 0 && ix < a.w;
      const float* sp = a.src0 + ((size_t)(img * a.h + iy) * a.w + ix) * a.s0;
#pragma unroll
      for (int c = 0; c < CIN; ++c) {
        const float v = ok ? sp[c] : 0.f;
        const float* wk = a.weight + (size_t)((ty * a.kw + tx) * CIN + c) * npad + co0;
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[j] += wk[j] * v;
      }
    }
  }
  float* op = a.out + (size_t)pix * a.so + co0;
#pragma unroll
  for (int j = 0; j < 16; ++j)
    if (co0 + j < a.cout) op[j] = act_apply(acc[j], a.act);
}

// ------------------------------------------------------------------------------------------
// thin conv (cout ≤ 4): lane = output pixel of a 64-pixel tile (64/W whole rows); the 4 waves
// split every 32-channel chunk 4 ways (8 channels each) and reduce through LDS at the end.
// The chunk's input halo is staged in LDS (coalesced 16-B loads), the next chunk's halo is
// prefetched into registers while this one is consumed; weights are wave-uniform (s_load).
// packed weights: [cout][taps][cin]
// ------------------------------------------------------------------------------------------
constexpr int thin_na(int kh, int kw) {  // float4 per thread of one chunk's halo, W ∈ {32, 64}
  const int a32 = (2 + kh - 1) * (32 + kw - 1) * (THIN_CC / 4);
  const int a64 = (1 + kh - 1) * (64 + kw - 1) * (THIN_CC / 4);
  const int m = a32 > a64 ? a32 : a64;
  return (m + 255) / 256;
}

template <int COUT, int KH, int KW>
__device__ __forceinline__ void conv_thin_body(const scflow_conv_args& a, int oh, int ow, int blk,
                                               int nblk) {
  constexpr int NA = thin_na(KH, KW);
  // [(tr+KH-1)*(ow+KW-1)][THIN_LD], reused for the reduction; float4-typed so the halo accesses
  // are ds_write_b128 / ds_read_b128 (a float array's unknown alignment split the 16-B stores
  // into ds_write2_b32 pairs, 4-way bank conflicts)
  extern __shared__ floatx4 thin_smem4[];
  float* halo = (float*)thin_smem4;
  const int tr = 64 / ow;
  const int hcols = ow + KW - 1;
  const int nh = (tr + KH - 1) * hcols * (THIN_CC / 4);
  const int tiles_per_img = oh / tr;
  // XCD-aware tile order (as conv_thin_full_kernel): each XCD covers a contiguous run of row
  // tiles, so the halo rows neighbouring tiles share come from that XCD's L2 — in dispatch order
  // the three tiles reading an input row sat on three XCDs, each fetching it from the MALL
  const int bid = nblk % 8 ? blk : (blk % 8) * (nblk / 8) + blk / 8;
  const int img = bid / tiles_per_img;
  const int oy0 = (bid % tiles_per_img) * tr;
  const int cin = a.c0 + a.c1;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int py = lane / ow, px = lane % ow;
  floatx4 ra[NA];
  auto gload = [&](int cc) {
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      const int idx = threadIdx.x + 256 * j;
      floatx4 v = {0.f, 0.f, 0.f, 0.f};
      if (idx < nh) {
        const int q = idx % (THIN_CC / 4), pix = idx / (THIN_CC / 4);
        const int hr = pix / hcols, hcol = pix % hcols;
        const int iy = oy0 - a.ph + hr, ix = hcol - a.pw;
        const int c = cc + 4 * q;
        if (iy >= 0 && iy < a.h && ix >= 0 && ix < a.w && c < cin) {
          const size_t ip = (size_t)(img * a.h + iy) * a.w + ix;
          v = c < a.c0 ? *(const floatx4*)(a.src0 + ip * a.s0 + c)
                       : *(const floatx4*)(a.src1 + ip * a.s1 + (c - a.c0));
        }
      }
      ra[j] = v;
    }
  };
  // all weights in LDS once, [tap][ci][o] (packed global layout is [o][tap][ci]): the compute
  // loop reads them as wave-wide broadcasts instead of per-lane global loads
  float* wl = halo + (size_t)(tr + KH - 1) * hcols * THIN_LD;
  {
    const int nw = KH * KW * cin * COUT;
    for (int i = threadIdx.x; i < nw; i += 256) {
      const int o = i % COUT, k = i / COUT;  // k = tap·cin + ci
      wl[i] = a.weight[(size_t)o * KH * KW * cin + k];
    }
  }
  float acc[COUT];
#pragma unroll
  for (int o = 0; o < COUT; ++o) acc[o] = 0.f;
  gload(0);
  for (int cc = 0; cc < cin; cc += THIN_CC) {
    __syncthreads();
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      const int idx = threadIdx.x + 256 * j;
      if (idx < nh) thin_smem4[(idx / (THIN_CC / 4)) * (THIN_LD / 4) + idx % (THIN_CC / 4)] = ra[j];
    }
    __syncthreads();
    if (cc + THIN_CC < cin) gload(cc + THIN_CC);
    const int c0 = wave * 8;  // this wave's 8 channels of the chunk
    if (cc + c0 < cin) {
#pragma unroll
      for (int ty = 0; ty < KH; ++ty)
#pragma unroll
        for (int tx = 0; tx < KW; ++tx) {
          const floatx4* hp = thin_smem4 + ((py + ty) * hcols + px + tx) * (THIN_LD / 4) + c0 / 4;
          const floatx4 v0 = hp[0];
          const floatx4 v1 = hp[1];
          float w[8 * COUT];  // [ci][o] for this tap's 8 channels
          const float* wp = wl + ((size_t)(ty * KW + tx) * cin + cc + c0) * COUT;
#pragma unroll
          for (int i = 0; i < 2 * COUT; ++i) {
            const floatx4 t = *(const floatx4*)(wp + 4 * i);
            w[4 * i] = t[0]; w[4 * i + 1] = t[1]; w[4 * i + 2] = t[2]; w[4 * i + 3] = t[3];
          }
#pragma unroll
          for (int o = 0; o < COUT; ++o)
            acc[o] += v0[0] * w[0 * COUT + o] + v0[1] * w[1 * COUT + o] + v0[2] * w[2 * COUT + o] +
                      v0[3] * w[3 * COUT + o] + v1[0] * w[4 * COUT + o] + v1[1] * w[5 * COUT + o] +
                      v1[2] * w[6 * COUT + o] + v1[3] * w[7 * COUT + o];
        }
    }
  }
  __syncthreads();
#pragma unroll
  for (int o = 0; o < COUT; ++o) halo[(wave * COUT + o) * 64 + lane] = acc[o];
  __syncthreads();
  if (wave == 0) {
    const size_t pix = ((size_t)img * oh + oy0 + py) * ow + px;
#pragma unroll
    for (int o = 0; o < COUT; ++o) {
      float v = halo[(0 * COUT + o) * 64 + lane];
      v += halo[(1 * COUT + o) * 64 + lane];
      v += halo[(2 * COUT + o) * 64 + lane];
      v += halo[(3 * COUT + o) * 64 + lane];
      const float b = a.bias ? a.bias[o] : 0.f;
      a.out[pix * a.so + o] = act_apply(v + b, a.act);
    }
  }
}

template <int COUT, int KH, int KW>
__global__ __launch_bounds__(256) void conv_thin_kernel(scflow_conv_args a, int oh, int ow) {
  conv_thin_body<COUT, KH, KW>(a, oh, ow, blockIdx.x, gridDim.x);
}

// thin conv, whole halo at once (the decoder's XHead predictors, 256 → 2 / 1, raft_decoder.py:
// 256-294): one workgroup of 1024 threads per 64-pixel tile stages the tile's input halo for ALL
// channels in LDS with a single round of coalesced 16-B loads (one memory latency, where the
// chunked kernel above pays one per 32 channels), then each of the 16 waves contracts a 1/16
// share of the channels for the 64 pixels (lane = pixel, weights as wave-uniform scalar loads)
// and the 16 partials are summed in wave order through LDS: deterministic.
constexpr int THINF_WAVES = 16;
__host__ __device__ constexpr int thinf_ld(int cin) { return cin + 4; }  // pixel stride (floats)

template <int COUT, int KH, int KW>
__global__ __launch_bounds__(THINF_WAVES * 64) void conv_thin_full_kernel(scflow_conv_args a,
                                                                          int oh, int ow,
                                                                          unsigned long long* stamps) {
  // [(tr+KH-1)·(ow+KW-1)][cin + 4], reused for the partials; float4-typed: ds_*_b128 halo
  // accesses (see conv_thin_kernel)
  extern __shared__ floatx4 thinf_smem4[];
  float* halo = (float*)thinf_smem4;
  const int tr = 64 / ow;
  const int hcols = ow + KW - 1;
  const int cin = a.c0;
  const int ld = thinf_ld(cin);
  const int q4 = cin / 4;
  const int nh = (tr + KH - 1) * hcols * q4;  // float4 of the halo
  const int tiles_per_img = oh / tr;
  // XCD-aware tile order: workgroups are dealt round-robin over the 8 XCDs, so block b takes tile
  // (b % 8)·(grid / 8) + b / 8 and each XCD covers a contiguous run of row tiles — the halo rows
  // two neighbouring tiles share are fetched once into that XCD's L2 (flow predictor at B = 16:
  // 15.0 -> 14.6 us in isolation, tools/sess_variant.sh)
  const int bid = gridDim.x % 8 ? (int)blockIdx.x
                                : (int)(blockIdx.x % 8) * (int)(gridDim.x / 8) + (int)(blockIdx.x / 8);
  const int img = bid / tiles_per_img;
  const int oy0 = (bid % tiles_per_img) * tr;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  sc_stamp(stamps, 0);
  // the packed weights [o][tap][ci] go to LDS behind the halo, loaded in the same round (the
  // contraction then reads them as wave-uniform ds_read_b128 broadcasts: as scalar loads inside
  // the channel loop each tap's pair of s_load waited out its own L2 round trip — 10 of the
  // launch's 17 µs at B = 16)
  const int nw4 = KH * KW * cin * COUT / 4;
  floatx4* wl4 = thinf_smem4 + (size_t)(tr + KH - 1) * hcols * (ld / 4);
  constexpr int NWL = 2;  // float4 of weights per thread (≤ 2048: 3×3 × 256 × 2 = 1152)
  floatx4 wv[NWL];
#pragma unroll
  for (int j = 0; j < NWL; ++j) {
    const int idx = tid + THINF_WAVES * 64 * j;
    if (idx < nw4) wv[j] = ((const floatx4*)a.weight)[idx];
  }
  // every load first, then every LDS store (at most 9 float4 per thread at 4 × 34 × 256)
  constexpr int NL = 12;
  floatx4 v[NL];
#pragma unroll
  for (int j = 0; j < NL; ++j) {
    const int idx = tid + THINF_WAVES * 64 * j;
    v[j] = floatx4{0.f, 0.f, 0.f, 0.f};
    if (idx < nh) {
      const int q = idx % q4, pix = idx / q4;
      const int hr = pix / hcols, hcol = pix % hcols;
      const int iy = oy0 - a.ph + hr, ix = hcol - a.pw;
      if (iy >= 0 && iy < a.h && ix >= 0 && ix < a.w)
        v[j] = *(const floatx4*)(a.src0 + ((size_t)(img * a.h + iy) * a.w + ix) * a.s0 + 4 * q);
    }
  }
#pragma unroll
  for (int j = 0; j < NL; ++j) {
    const int idx = tid + THINF_WAVES * 64 * j;
    if (idx < nh) thinf_smem4[(idx / q4) * (ld / 4) + idx % q4] = v[j];
  }
#pragma unroll
  for (int j = 0; j < NWL; ++j) {
    const int idx = tid + THINF_WAVES * 64 * j;
    if (idx < nw4) wl4[idx] = wv[j];
  }
  __syncthreads();
  sc_stamp(stamps, 1);
  const int py = lane / ow, px = lane % ow;
  const int cw = cin / THINF_WAVES;  // channels of this wave (a multiple of 4)
  const int c0 = wave * cw;
  float acc[COUT];
#pragma unroll
  for (int o = 0; o < COUT; ++o) acc[o] = 0.f;
  // weights [o][tap][ci] in LDS: wave-uniform addresses → broadcast reads
  const float* wls = (const float*)wl4;
  for (int ty = 0; ty < KH; ++ty)
    for (int tx = 0; tx < KW; ++tx) {
      const floatx4* hp = thinf_smem4 + ((py + ty) * hcols + px + tx) * (ld / 4) + c0 / 4;
      const float* wp = wls + (size_t)(ty * KW + tx) * cin + c0;
#ifdef THINF_UNROLL  // channel-chunk loop unroll of the contraction (tuning build flag)
#pragma unroll THINF_UNROLL
#endif
      for (int c = 0; c < cw; c += 4) {
        const floatx4 x = hp[c / 4];
#pragma unroll
        for (int o = 0; o < COUT; ++o) {
          const floatx4 w = *(const floatx4*)(wp + (size_t)o * KH * KW * cin + c);
          acc[o] += x[0] * w[0] + x[1] * w[1] + x[2] * w[2] + x[3] * w[3];
        }
      }
    }
  __syncthreads();
  sc_stamp(stamps, 2);
#pragma unroll
  for (int o = 0; o < COUT; ++o) halo[(wave * COUT + o) * 64 + lane] = acc[o];
  __syncthreads();
  if (wave == 0) {
    const size_t pix = ((size_t)img * oh + oy0 + py) * ow + px;
#pragma unroll
    for (int o = 0; o < COUT; ++o) {
      float r = 0.f;
      for (int w = 0; w < THINF_WAVES; ++w) r += halo[(w * COUT + o) * 64 + lane];
      const float b = a.bias ? a.bias[o] : 0.f;
      a.out[pix * a.so + o] = act_apply(r + b, a.act);
    }
  }
  if (stamps) {
    __builtin_amdgcn_s_waitcnt(0);
    sc_stamp(stamps, 3);
  }
}

#include "conv_thinz.h"

// generic thin fallback: one wave per output pixel, lanes split the channels
template <int COUT>
__global__ __launch_bounds__(256) void conv_thin_generic(scflow_conv_args a, int oh, int ow) {
  const int cin = a.c0 + a.c1;
  const int taps = a.kh * a.kw;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long long M = (long long)a.n * oh * ow;
  const long long pix = blockIdx.x * 4LL + wave;
  if (pix >= M) return;
  const int ox = (int)(pix % ow);
  const long long t = pix / ow;
  const int oy = (int)(t % oh);
  const int img = (int)(t / oh);
  float acc[COUT];
#pragma unroll
  for (int o = 0; o < COUT; ++o) acc[o] = 0.f;
  for (int ty = 0; ty < a.kh; ++ty) {
    const int iy = oy - a.ph + ty;
    if (iy < 0 || iy >= a.h) continue;
    for (int tx = 0; tx < a.kw; ++tx) {
      const int ix = ox - a.pw + tx;
      if (ix < 0 || ix >= a.w) continue;
      const size_t ip = (size_t)(img * a.h + iy) * a.w + ix;
      const int tap = ty * a.kw + tx;
      for (int c = lane * 4; c < cin; c += 256) {
        const floatx4 v = c < a.c0 ? *(const floatx4*)(a.src0 + ip * a.s0 + c)
                                   : *(const floatx4*)(a.src1 + ip * a.s1 + (c - a.c0));
#pragma unroll
        for (int o = 0; o < COUT; ++o) {
          const float* w = a.weight + ((size_t)o * taps + tap) * cin + c;
          acc[o] += v[0] * w[0] + v[1] * w[1] + v[2] * w[2] + v[3] * w[3];
        }
      }
    }
  }
#pragma unroll
  for (int o = 0; o < COUT; ++o) {
    float v = acc[o];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    acc[o] = v;
  }
  if (lane == 0) {
#pragma unroll
    for (int o = 0; o < COUT; ++o) {
      const float b = a.bias ? a.bias[o] : 0.f;
      a.out[(size_t)pix * a.so + o] = act_apply(acc[o] + b, a.act);
    }
  }
}

// packing: w_oihw [cout][cin][kh][kw] → variant layout
__global__ void pack_kernel(const float* __restrict__ w, float* __restrict__ out, int variant,
                            int cout, int c0, int c1, int kh, int kw, int cp0, int nst, int npad,
                            int bk, long long total) {
  const int cin = c0 + c1, taps = kh * kw;
  for (long long idx = blockIdx.x * 256LL + threadIdx.x; idx < total; idx += (long long)gridDim.x * 256) {
    float v = 0.f;
    if (variant == V_MFMA) {
      // [nt][s][tap][col][k]
      long long r = idx;
      const int k = (int)(r % bk); r /= bk;
      const int col = (int)(r % BN); r /= BN;
      const int tap = (int)(r % taps); r /= taps;
      const int s = (int)(r % nst);
      const int nt = (int)(r / nst);
      const int o = nt * BN + col;
      const int kc = s * bk + k;  // channel index in the padded concat space
      int ci = -1;
      if (kc < cp0) {
        if (kc < c0) ci = kc;
      } else if (kc - cp0 < c1) {
        ci = c0 + (kc - cp0);
      }
      if (o < cout && ci >= 0) v = w[((size_t)o * cin + ci) * taps + tap];
    } else if (variant == V_SMALLCIN) {  // [tap*cin + ci][npad]
      const int o = (int)(idx % npad);
      const int k = (int)(idx / npad);
      const int tap = k / cin, ci = k % cin;
      if (o < cout) v = w[((size_t)o * cin + ci) * taps + tap];
    } else {  // thin: [o][tap][ci]
      const int ktot = taps * cin;
      const int o = (int)(idx / ktot);
      const int k = (int)(idx % ktot);
      const int tap = k / cin, ci = k % cin;
      v = w[((size_t)o * cin + ci) * taps + tap];
    }
    out[idx] = v;
  }
}

#include "conv_wino.h"
#include "conv_wino5.h"
#include "conv1x1w.h"

// Winograd eligibility: F(2×2,3×3) (conv_wino.h) for 3×3, F(4,5) (conv_wino5.h) for 1×5 / 5×1;
// stride 1, "same" padding, whole-row tiles of 32 tiles
bool wino_shape(int kh, int kw, int stride, int w) {
  if (kh == 3 && kw == 3) return stride == 1 && (w == 32 || w == 64 || w == 128);
  const bool k = (kh == 1 && kw == 5) || (kh == 5 && kw == 1);
  return k && stride == 1 && (w == 32 || w == 64);
}
bool has_fused_norm(const scflow_conv_args& a) {
  return a.in_scale || a.in_shift || a.out_scale || a.out_shift || a.res;
}
bool wino_launchable(const scflow_conv_args& a) {
  if (!wino_shape(a.kh, a.kw, a.stride, a.w) || a.c0 % 4 || a.c1 % 4 || a.cout <= 4 ||
      (a.c0 + a.c1 <= 4 && a.c1 == 0))
    return false;
  if (a.kh == 3)
    return a.ph == 1 && a.pw == 1 && a.h % (a.w == 32 ? 4 : 2) == 0 &&
           a.epilogue == SCFLOW_EPI_PLAIN &&
           (!(a.in_scale || a.in_shift) || (a.in_scale && a.in_shift && a.c1 == 0)) &&
           (!a.out_scale) == (!a.out_shift);
  if (has_fused_norm(a)) return false;
  if (a.kh == 1) return a.ph == 0 && a.pw == 2 && a.h % (128 / a.w) == 0;
  return a.ph == 2 && a.pw == 0 && a.h % 4 == 0;
}
long long wino_packed_size(int cout, int c0, int c1, int kh) {
  if (kh == 3) {
    const int nsub = (round_up(c0, WSC) + round_up(c1, WSC)) / WKC;
    return (long long)(round_up(cout, 64) / 32) * nsub * 16 * 256;
  }
  const int nsub = (round_up(c0, W5SC) + round_up(c1, W5SC)) / W5KC;
  return (long long)(round_up(cout, 64) / 32) * nsub * 8 * 2 * 256;
}
// output rows per workgroup (the grid's x extent is n · h / rows · column blocks)
long long wino_blocks(const scflow_conv_args& a) {
  if (a.kh == 3) return (long long)a.n * (a.h / (a.w == 32 ? 4 : 2)) * (a.w == 128 ? 2 : 1);
  if (a.kh == 1) return (long long)a.n * (a.h / (128 / a.w));
  return (long long)a.n * (a.h / 4) * (a.w / 32);
}
// 64 output channels per workgroup when that still gives ≥ 1.5 workgroups per CU, else 32;
// SCFLOW_WINO_NBW=1|2 forces one, =4 disables the 96-channel choice (tuning only)
// (measured per decoder shape at B = 16, tools/conv_bench.py: 3×3 256→192 85 vs 95 µs at 384
// workgroups; 256→126, 128→64 and the GRU q convs at 256 or fewer prefer 32)
int wino_nbw(const scflow_conv_args& a, int cus) {
  static int forced = -1;
  if (forced < 0) {
    const char* e = getenv("SCFLOW_WINO_NBW");
    forced = e ? atoi(e) : 0;
  }
  if (forced == 1 || forced == 2) return forced;
  if (a.cout <= 32) return 1;
  // 96 channels when that is exactly one workgroup per CU where 64 would leave 1.5 (3×3, W = 32)
  if (forced != 4 && a.kh == 3 && a.w == 32 && a.cout % 96 == 0 &&
      wino_blocks(a) * (a.cout / 96) == cus && (2 * wino_blocks(a) * (a.cout / 64)) % (2LL * cus))
    return 3;
  return 2 * wino_blocks(a) * (round_up(a.cout, 64) / 64) >= 3LL * cus ? 2 : 1;
}
bool wino_enabled(int kh) {
  static int on3 = -1, on5 = -1;
  if (on3 < 0) {
    const char* e = getenv("SCFLOW_CONV_WINO");  // 0: off, 3: 3×3 only, 5: 1×5/5×1 only
    const int v = e ? atoi(e) : 1;
    on3 = v == 1 || v == 3;
    on5 = v == 1 || v == 5;
  }
  return kh == 3 ? on3 : on5;
}

// XCD-aware block order for a (R row blocks) × (C column blocks) Winograd grid: the number of
// column parts across the 8 XCDs (wino_block), 0 when the grid does not divide.
// SCFLOW_WINO_SWZ=c forces c column parts (tuning); default WINO_SWZ_DEFAULT.
#ifndef WINO_SWZ_DEFAULT
#define WINO_SWZ_DEFAULT 0
#endif
int wino_swz(int R, int C) {
  static int forced = -2;
  if (forced == -2) {
    const char* e = getenv("SCFLOW_WINO_SWZ");
    forced = e ? atoi(e) : -1;
  }
  int c = forced >= 0 ? forced : WINO_SWZ_DEFAULT;
  while (c > 1 && (C % c || 8 % c)) c >>= 1;  // largest usable power of two ≤ c
  if (c <= 0 || R % (8 / c)) return 0;
  return c;
}

// profiling: where the next F(2×2,3×3) Winograd launches write their per-workgroup stamps

#include "conv_wino4.h"

// F(4×4,3×3) (conv_wino4.h) for the 3×3 convs it covers with at least WINO4_MIN_COUT output
// channels; SCFLOW_CONV_WINO4 = 0 off, 1 default, 2 every covered shape (A/B).  Measured at
// configs[1] (B=16, 32×32; tools/sess_w4c.sh, round 5): XHead hidden 128→512 59 vs 91 µs,
// corr_net.1 256→192 57 vs 78 µs (F(2×2,3×3)), out_net 256→126 56 vs 50 µs — at 126 channels
// the grid is 128 workgroups on 256 CUs and the transform pass (≈ 12 µs at 256 input channels)
// is not paid back; decoder 4.98 vs 5.11 ms/forward with both wide convs on F(4×4).
#ifndef WINO4_MIN_COUT
#define WINO4_MIN_COUT 160
#endif
#ifndef WINO4_DEFAULT
#define WINO4_DEFAULT 1
#endif
// Round 6: with the GEMM's XCD-blocked order (conv_wino4.h) out_net (256 → 126) at configs[4]
// runs F(4×4,3×3) faster (337 → 310 µs alone, profiles/r06/g7_wino4_all_ab.txt), so convs of ≥ 120
// output channels whose GEMM grid exceeds one round of two workgroups per CU take it too; the
// 64-channel ones stay on F(2×2,3×3) there (flow_net.1 102 vs 110 µs, mask encoder 32 vs 50 µs;
// every eligible conv on F(4×4): decoder 8.36k vs 8.85k iters/s).
#ifndef WINO4_MIN_COUT_MULTI
#define WINO4_MIN_COUT_MULTI 120
#endif
bool wino4_pick(const scflow_conv_args& a) {
  static int mode = -1;
  if (mode < 0) {
    const char* e = getenv("SCFLOW_CONV_WINO4");
    mode = e ? atoi(e) : WINO4_DEFAULT;
  }
  if (!mode || !wino4_shape(a)) return false;
  if (mode == 2 || a.cout >= WINO4_MIN_COUT) return true;
  const long long tiles = (long long)a.n * (a.h / 4) * (a.w / 4);
  const long long wgs = (tiles + 31) / 32 * ((a.cout + 31) / 32);
  return a.cout >= WINO4_MIN_COUT_MULTI && wgs > 2LL * device_cus();
}


template <int W, int NBW>
int launch_wino_w(WinoParams p, hipStream_t st) {
  using G = WinoGeom<W>;
  const size_t lds = wino_lds_bytes<W, NBW>();
  static bool attr = false;
  if (lds > 64 * 1024 && !attr) {
    (void)hipFuncSetAttribute((const void*)conv_wino_kernel<W, NBW>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  dim3 grid(p.a.n * (p.a.h / G::OROWS) * G::XB, round_up(p.a.cout, 32 * NBW) / (32 * NBW));
  p.swz_c = wino_swz(grid.x, grid.y);
  p.stamps = g_wino_stamps;
  conv_wino_kernel<W, NBW><<<grid, 256, lds, st>>>(p);
  return scflow_launch_status();
}

template <int DIR, int W, int NBW, int EPI>
int launch_wino5_k(Wino5Params p, hipStream_t st) {
  using G = Wino5Geom<DIR, W>;
  const size_t lds = wino5_lds_bytes<DIR, W, NBW>();
  static bool attr = false;
  if (lds > 64 * 1024 && !attr) {
    (void)hipFuncSetAttribute((const void*)conv_wino5_kernel<DIR, W, NBW, EPI>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  dim3 grid(p.a.n * (p.a.h / G::OROWS) * (W / G::OCOLS), round_up(p.a.cout, 32 * NBW) / (32 * NBW));
  p.swz_c = wino_swz(grid.x, grid.y);
  p.stamps = g_wino_stamps;
  conv_wino5_kernel<DIR, W, NBW, EPI><<<grid, 256, lds, st>>>(p);
  return scflow_launch_status();
}

template <int EPI>
int launch_wino5_epi(const Wino5Params& p, int nbw, hipStream_t st) {
  const bool x = p.a.kh == 1;
  if (p.a.w == 32) {
    if (x) return nbw == 2 ? launch_wino5_k<0, 32, 2, EPI>(p, st) : launch_wino5_k<0, 32, 1, EPI>(p, st);
    return nbw == 2 ? launch_wino5_k<1, 32, 2, EPI>(p, st) : launch_wino5_k<1, 32, 1, EPI>(p, st);
  }
  if (x) return nbw == 2 ? launch_wino5_k<0, 64, 2, EPI>(p, st) : launch_wino5_k<0, 64, 1, EPI>(p, st);
  return nbw == 2 ? launch_wino5_k<1, 64, 2, EPI>(p, st) : launch_wino5_k<1, 64, 1, EPI>(p, st);
}

int launch_wino(const scflow_conv_args& a, hipStream_t st) {
  if (!wino_launchable(a)) return SCFLOW_EUNSUPPORTED;
  if (!aligned16(a.src0) || (a.s0 & 3) || (a.c1 > 0 && (!aligned16(a.src1) || (a.s1 & 3))) ||
      !aligned16(a.weight))
    return SCFLOW_EALIGN;
  if (a.kh != 3) {
    Wino5Params p;
    p.a = a;
    p.cp0 = round_up(a.c0, W5SC);
    p.nst = (p.cp0 + round_up(a.c1, W5SC)) / W5SC;
    const int nbw = wino_nbw(a, device_cus());
    switch (a.epilogue) {
      case SCFLOW_EPI_GRU_ZR: return launch_wino5_epi<SCFLOW_EPI_GRU_ZR>(p, nbw, st);
      case SCFLOW_EPI_GRU_Q: return launch_wino5_epi<SCFLOW_EPI_GRU_Q>(p, nbw, st);
      default: return launch_wino5_epi<SCFLOW_EPI_PLAIN>(p, nbw, st);
    }
  }
  WinoParams p;
  p.a = a;
  p.cp0 = round_up(a.c0, WSC);
  p.nst = (p.cp0 + round_up(a.c1, WSC)) / WSC;
  const int nbw = wino_nbw(a, device_cus());
  if (a.w == 32) {
    return nbw == 3 ? launch_wino_w<32, 3>(p, st)
                    : nbw == 2 ? launch_wino_w<32, 2>(p, st) : launch_wino_w<32, 1>(p, st);
  }
  if (a.w == 128) return nbw == 2 ? launch_wino_w<128, 2>(p, st) : launch_wino_w<128, 1>(p, st);
  return nbw == 2 ? launch_wino_w<64, 2>(p, st) : launch_wino_w<64, 1>(p, st);
}

// Workgroup-count heuristic (measured on MI355X, tools/conv_bench.py): 128-pixel tiles when
// that still gives ≥ 2 workgroups per CU (≥ 512), else 64-pixel tiles (GRU q: 103 vs 94 TF,
// N=64 convs: 85 vs 54 TF, N=192: 94 vs 91 TF; z|r and the 512-wide heads prefer 128).
// SCFLOW_CONV_TILE_M=64|128 forces one (tuning only).
int pick_tile_m(long long m, int ntiles) {
  static int forced = -1;
  if (forced < 0) {
    const char* e = getenv("SCFLOW_CONV_TILE_M");
    forced = e ? atoi(e) : 0;
  }
  if (forced == 64 || forced == 128) return forced;
  const long long wg = (m / 128) * ntiles;
  if (wg >= 512) return 128;
  return 64;
}

size_t mfma_lds(int hr, int hc, int taps, int bk) {
  return sizeof(float) * ((size_t)hr * hc + (size_t)taps * BN) * (bk + 4);
}

// Stage depth for a launch: 16 (fewer barriers per MFMA) unless the grid needs more resident
// workgroups than 16-deep stages' LDS allows and 8-deep ones would take fewer rounds
// (measured on the decoder's 3×3 256→192 conv at B=16: 768 workgroups, 2 per CU at 16 =
// 1.5 rounds; 85 → 101 TFLOP/s at 8).  Resident workgroups per CU are capped by VGPRs at
// 2 (128-pixel tiles) / 3 (64).  SCFLOW_CONV_BK=8|16 forces one (tuning only).
int pick_bk(int kh, int kw, int tm, int hr, int hc, long long wgs, int cus) {
  static int forced = -1;
  if (forced < 0) {
    const char* e = getenv("SCFLOW_CONV_BK");
    forced = e ? atoi(e) : 0;
  }
  if (forced == 8 || forced == 16) return forced;
  auto rounds = [&](int bk) {
    long long per_cu = (long long)(160 * 1024 / mfma_lds(hr, hc, kh * kw, bk));
    const long long cap = tm == 64 ? 3 : 2;
    if (per_cu > cap) per_cu = cap;
    if (per_cu < 1) per_cu = 1;
    return (wgs + per_cu * cus - 1) / (per_cu * cus);
  };
  return rounds(8) < rounds(16) ? 8 : 16;
}

// the 1×1 kernel (conv1x1_kernel) for stride-1 1×1 convs on 128-row tiles; SCFLOW_CONV1X1=0
// keeps them on conv_mfma_kernel (tuning only)
// SCFLOW_SMALLCIN_SPLIT=1: the 128-channel small-cin MFMA conv as two workgroups per 64-pixel tile
// (one per 64-channel half) instead of one (each wave 2 × 32 channels).  Measured: 13.1 -> 12.1 us
// in isolation (7x7 2->128, B=16), no gain inside the decoder (5.263 vs 5.233 ms/forward), so off.
bool smallcin_split() {  // cached (scflow_debug_reload_switches)
  static EnvSwitch sw("SCFLOW_SMALLCIN_SPLIT", 0);
  return sw.get() != 0;
}

bool conv1x1_enabled() {
  static int on = -1;
  if (on < 0) {
    const char* e = getenv("SCFLOW_CONV1X1");
    on = !(e && e[0] == '0');
  }
  return on != 0;
}

// tile rows / halo rows / tile size for a launch (shared by the launcher and scflow_conv_pick_bk)
int launch_tile(const scflow_conv_args& a, const Geometry& g, int* tr, int* hr) {
  const long long m = (long long)a.n * g.oh * g.ow;
  const int tm = (pick_tile_m(m, g.npad / BN) == 64 && g.ow <= 64) ? 64 : 128;
  *tr = tm / g.ow;
  *hr = *tr + a.kh - 1;
  return tm;
}

template <int EPI, int KH, int KW, int TM, int BKS>
int launch_mfma_bk(MfmaParams p, Geometry g, hipStream_t st) {
  p.nst = (g.cp0 + g.cp1) / BKS;
  const size_t lds = mfma_lds(g.hr, g.hc, g.taps, BKS);
  static bool attr = false;
  if (lds > 64 * 1024 && !attr) {
    (void)hipFuncSetAttribute((const void*)conv_mfma_kernel<EPI, KH, KW, TM, BKS>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  dim3 grid(p.a.n * (g.oh / g.tr), g.npad / BN);
  conv_mfma_kernel<EPI, KH, KW, TM, BKS><<<grid, 256, lds, st>>>(p);
  return scflow_launch_status();
}

template <int EPI, int KH, int KW, int TM>
int launch_mfma_tm(MfmaParams p, Geometry g, hipStream_t st) {
  g.tr = TM / g.ow;
  if (g.tr < 1 || g.oh % g.tr) return SCFLOW_EUNSUPPORTED;
  g.hr = g.tr + KH - 1;
  p.tr = g.tr;
  p.hr = g.hr;
  if (p.a.bk == 8) return launch_mfma_bk<EPI, KH, KW, TM, 8>(p, g, st);
  return launch_mfma_bk<EPI, KH, KW, TM, 16>(p, g, st);
}

template <int EPI, int KH, int KW>
int launch_mfma(const MfmaParams& p, const Geometry& g, hipStream_t st) {
  int tr, hr;
  if (launch_tile(p.a, g, &tr, &hr) == 64) return launch_mfma_tm<EPI, KH, KW, 64>(p, g, st);
  return launch_mfma_tm<EPI, KH, KW, 128>(p, g, st);
}

template <int EPI>
int dispatch_mfma(const MfmaParams& p, const Geometry& g, hipStream_t st) {
  const int kh = p.a.kh, kw = p.a.kw;
  if (kh == 1 && kw == 1) return launch_mfma<EPI, 1, 1>(p, g, st);
  if (kh == 3 && kw == 3) return launch_mfma<EPI, 3, 3>(p, g, st);
  if (kh == 1 && kw == 5) return launch_mfma<EPI, 1, 5>(p, g, st);
  if (kh == 5 && kw == 1) return launch_mfma<EPI, 5, 1>(p, g, st);
  return SCFLOW_EUNSUPPORTED;
}

}  // namespace

// ---- wide 1×1 (conv1x1w.h): which shapes, how packed, how launched
// SCFLOW_CONV1X1W=0 keeps the 1×1 convs on conv1x1_kernel (A/B)
bool conv1x1w_enabled() {
  static int on = -1;
  if (on < 0) {
    const char* e = getenv("SCFLOW_CONV1X1W");
    on = !(e && e[0] == '0');
  }
  return on != 0;
}
int conv1x1w_kb(int c0) { return (c0 + 7) / 8; }
bool conv1x1w_kb_ok(int kb) { return kb == 41 || kb == 32 || kb == 16; }
bool conv1x1w_shape(int cout, int c0, int c1, int kh, int kw, int stride) {
  return kh == 1 && kw == 1 && stride == 1 && c1 == 0 && c0 % 4 == 0 && cout > 4 && cout <= 256 &&
         conv1x1w_kb_ok(conv1x1w_kb(c0));
}
bool conv1x1w_launchable(const scflow_conv_args& a) {
  return conv1x1w_shape(a.cout, a.c0, a.c1, a.kh, a.kw, a.stride) && a.ph == 0 && a.pw == 0 &&
         a.epilogue == SCFLOW_EPI_PLAIN && !has_fused_norm(a);
}
long long conv1x1w_packed_size(int cout, int c0) {
  return (long long)(round_up(cout, 64) / 32) * conv1x1w_kb(c0) * 256;
}
template <int KB>
int launch_conv1x1w_kb(const scflow_conv_args& a, hipStream_t st) {
  const size_t lds = conv1x1w_lds_bytes<KB>();
  static bool attr = false;
  if (lds > 64 * 1024 && !attr) {
    (void)hipFuncSetAttribute((const void*)conv1x1w_kernel<KB>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  const long long M = (long long)a.n * a.h * a.w;
  conv1x1w_kernel<KB><<<(unsigned)((M + W1_PX - 1) / W1_PX), 256, lds, st>>>(a);
  return scflow_launch_status();
}
int launch_conv1x1w(const scflow_conv_args& a, hipStream_t st) {
  if (!conv1x1w_launchable(a)) return SCFLOW_EUNSUPPORTED;
  if (!aligned16(a.src0) || (a.s0 & 3) || !aligned16(a.weight)) return SCFLOW_EALIGN;
  switch (conv1x1w_kb(a.c0)) {
    case 41: return launch_conv1x1w_kb<41>(a, st);
    case 32: return launch_conv1x1w_kb<32>(a, st);
    case 16: return launch_conv1x1w_kb<16>(a, st);
    default: return SCFLOW_EUNSUPPORTED;
  }
}

SCFLOW_API long long scflow_conv_packed_size(int cout, int c0, int c1, int kh, int kw, int stride,
                                             int w) {
  // packing depends on the width (tile = whole rows) but not on the height or padding
  Geometry g = select_variant(cout, c0, c1, kh, kw, stride, w == 64 ? 64 : 32 * 4, w, (kh - 1) / 2,
                              (kw - 1) / 2);
  if (g.variant == V_NONE) return SCFLOW_EUNSUPPORTED;
  return (long long)g.npad * g.ktot;
}

SCFLOW_API long long scflow_conv_packed_size_bk(int cout, int c0, int c1, int kh, int kw,
                                                int stride, int w, int bk) {
  if (bk == SCFLOW_CONV_1X1W) {
    if (!conv1x1w_shape(cout, c0, c1, kh, kw, stride)) return SCFLOW_EUNSUPPORTED;
    return conv1x1w_packed_size(cout, c0);
  }
  if (bk == SCFLOW_CONV_WINO) {
    if (cout <= 4 || c0 <= 0 || c1 < 0 || c0 % 4 || c1 % 4 || !wino_shape(kh, kw, stride, w))
      return SCFLOW_EUNSUPPORTED;
    return wino_packed_size(cout, c0, c1, kh);
  }
  if (bk == SCFLOW_CONV_WINO4) {
    if (c0 <= 0 || c1 < 0 || c0 % 4 || c1 % 4 || kh != 3 || kw != 3 || stride != 1)
      return SCFLOW_EUNSUPPORTED;
    return wino4_packed_size(cout, c0, c1);
  }
  if (bk != 0 && bk != 8 && bk != 16) return SCFLOW_EINVAL;
  return scflow_conv_packed_size(cout, c0, c1, kh, kw, stride, w);
}

SCFLOW_API int scflow_conv_pack_weights(const float* w_oihw, float* packed, int cout, int c0,
                                        int c1, int kh, int kw, int stride, int w, int bk,
                                        void* stream) {
  if (!w_oihw || !packed || cout <= 0 || c0 <= 0 || c1 < 0 || kh <= 0 || kw <= 0) return SCFLOW_EINVAL;
  if (bk == SCFLOW_CONV_1X1W) {
    const long long total = scflow_conv_packed_size_bk(cout, c0, c1, kh, kw, stride, w, bk);
    if (total < 0) return (int)total;
    const int blocks = (int)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
    conv1x1w_pack_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(w_oihw, packed, cout, c0,
                                                                   conv1x1w_kb(c0), total);
    return scflow_launch_status();
  }
  if (bk == SCFLOW_CONV_WINO4) {
    const long long total = scflow_conv_packed_size_bk(cout, c0, c1, kh, kw, stride, w, bk);
    if (total < 0) return (int)total;
    const int cp0 = round_up(c0, W4KC);
    const int nsub = (cp0 + round_up(c1, W4KC)) / W4KC;
    const int blocks = (int)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
    wino4_pack_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(w_oihw, packed, cout, c0, c1, cp0,
                                                                nsub, total);
    return scflow_launch_status();
  }
  if (bk == SCFLOW_CONV_WINO) {
    const long long total = scflow_conv_packed_size_bk(cout, c0, c1, kh, kw, stride, w, bk);
    if (total < 0) return (int)total;
    // channels padded per source to the kernel's stage depth; packed per sub-step
    const int kc = kh == 3 ? WKC : W5KC, sc = kh == 3 ? WSC : W5SC;
    const int cp0 = round_up(c0, sc);
    const int nst = (cp0 + round_up(c1, sc)) / kc;
    const int blocks = (int)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
    if (kh == 3)
      wino_pack_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(w_oihw, packed, cout, c0, c1, cp0,
                                                                 nst, total);
    else
      wino5_pack_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(w_oihw, packed, cout, c0, c1, cp0,
                                                                  nst, total);
    return scflow_launch_status();
  }
  if (bk == 0) bk = BK;
  if (bk != 8 && bk != 16) return SCFLOW_EINVAL;
  Geometry g = select_variant(cout, c0, c1, kh, kw, stride, w == 64 ? 64 : 32 * 4, w, (kh - 1) / 2,
                              (kw - 1) / 2);
  if (g.variant == V_NONE) return SCFLOW_EUNSUPPORTED;
  const long long total = (long long)g.npad * g.ktot;
  const int blocks = (int)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
  pack_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(w_oihw, packed, g.variant, cout, c0, c1, kh,
                                                       kw, g.cp0, (g.cp0 + g.cp1) / bk, g.npad, bk,
                                                       total);
  return scflow_launch_status();
}

SCFLOW_API int scflow_conv_pick_bk(const scflow_conv_args* args) {
  if (!args) return SCFLOW_EINVAL;
  const scflow_conv_args& a = *args;
  if (a.n <= 0 || a.h <= 0 || a.w <= 0 || a.cout <= 0 || a.c0 <= 0 || a.c1 < 0) return SCFLOW_EINVAL;
  if (wino4_pick(a)) return SCFLOW_CONV_WINO4;
  if (wino_enabled(a.kh) && wino_launchable(a)) return SCFLOW_CONV_WINO;
  // the wide 1×1 kernel up to two workgroups per CU (configs[1]'s corr_net.0: 256, the same
  // 32.3 µs as conv1x1_kernel); larger grids keep conv1x1_kernel (configs[4], 2048 workgroups:
  // 236 vs 243 µs standalone, 48.7 vs 50.1 ms per decoder forward — session r4c / r4e)
  if (conv1x1w_enabled() && conv1x1w_launchable(a) &&
      (long long)a.n * a.h * a.w <= (long long)W1_PX * 2 * device_cus())
    return SCFLOW_CONV_1X1W;
  Geometry g = select_variant(a.cout, a.c0, a.c1, a.kh, a.kw, a.stride, a.h, a.w, a.ph, a.pw);
  if (g.variant != V_MFMA) return BK;  // other variants ignore the stage depth
  int tr, hr;
  const int tm = launch_tile(a, g, &tr, &hr);
  if (tr < 1 || g.oh % tr) return BK;
  const long long wgs = (long long)a.n * (g.oh / tr) * (g.npad / BN);
  return pick_bk(a.kh, a.kw, tm, hr, g.hc, wgs, device_cus());
}

SCFLOW_API long long scflow_conv_workspace_bytes(const scflow_conv_args* args) {
  if (!args) return SCFLOW_EINVAL;
  if (args->bk != SCFLOW_CONV_WINO4) return 0;
  if (!wino4_shape(*args) || args->n <= 0 || args->c0 <= 0) return SCFLOW_EUNSUPPORTED;
  return wino4_workspace_bytes(*args);
}

// the thin 3×3 contraction's preconditions (conv_thinz.h; shared with conv_pair.h)
bool thinz_ok(const scflow_conv_args& a, const Geometry& g, bool tiled) {
  static EnvSwitch thinz_sw("SCFLOW_THINZ", 1);
  return tiled && thinz_sw.get() && a.c1 == 0 && a.c0 == 256 && a.kh == 3 && a.kw == 3 &&
         a.ph == 1 && a.pw == 1 && a.stride == 1 && (a.cout == 1 || a.cout == 2) &&
         aligned16(a.weight) && ((long long)a.n * a.h * a.w * a.s0 + 256) * 4 < 0x7ffffff0LL &&
         g.oh % (g.ow == 64 ? 4 : 2) == 0;
}

// small-cin MFMA conv workgroups: at most SCFLOW_SMALLCIN_WGS per CU (default 2), each walking
// its tiles
long long smallcin_blocks(int ntiles) {
  static EnvSwitch wgs_sw("SCFLOW_SMALLCIN_WGS", 2);
  const int per_cu = wgs_sw.get() > 0 ? wgs_sw.get() : 2;
  const long long cap = (long long)per_cu * device_cus();
  return ntiles < cap ? ntiles : cap;
}

namespace {  // the grouped-launch and XHead kernels: internal linkage like the rest
#include "conv_pair.h"
#include "xhead_pred.h"
}  // namespace

bool conv_args_valid(const scflow_conv_args& a) {
  if (!a.src0 || !a.weight || a.n <= 0 || a.h <= 0 || a.w <= 0 || a.cout <= 0 || a.c0 <= 0 ||
      a.c1 < 0 || (a.c1 > 0 && !a.src1) || a.kh <= 0 || a.kw <= 0 || a.ph < 0 || a.pw < 0)
    return false;
  if (a.epilogue == SCFLOW_EPI_PLAIN) return a.out != nullptr;
  if (a.epilogue == SCFLOW_EPI_GRU_ZR) return a.gate && a.rh && a.hid && !(a.cout & 1);
  if (a.epilogue == SCFLOW_EPI_GRU_Q) return a.gate && a.hid;
  return false;
}

SCFLOW_API int scflow_conv2d(const scflow_conv_args* args, void* stream) {
  if (!args) return SCFLOW_EINVAL;
  const scflow_conv_args& a = *args;
  if (!conv_args_valid(a)) return SCFLOW_EINVAL;
  if (a.bk == SCFLOW_CONV_WINO) return launch_wino(a, (hipStream_t)stream);
  if (a.bk == SCFLOW_CONV_WINO4) return launch_wino4(a, (hipStream_t)stream);
  if (a.bk == SCFLOW_CONV_1X1W) return launch_conv1x1w(a, (hipStream_t)stream);
  if (has_fused_norm(a)) return SCFLOW_EUNSUPPORTED;  // Winograd 3×3 only
  if (a.bk != 0 && a.bk != 8 && a.bk != 16) return SCFLOW_EINVAL;
  Geometry g = select_variant(a.cout, a.c0, a.c1, a.kh, a.kw, a.stride, a.h, a.w, a.ph, a.pw);
  if (g.variant == V_NONE) return SCFLOW_EUNSUPPORTED;
  if (g.oh <= 0 || g.ow <= 0) return SCFLOW_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  if (g.variant == V_MFMA) {
    if (!aligned16(a.src0) || (a.s0 & 3) || (a.c1 > 0 && (!aligned16(a.src1) || (a.s1 & 3))) ||
        !aligned16(a.weight))
      return SCFLOW_EALIGN;
    MfmaParams p;
    p.a = a;
    p.oh = g.oh;
    p.ow = g.ow;
    p.tr = g.tr;
    p.hr = g.hr;
    p.hc = g.hc;
    p.cp0 = g.cp0;
    p.nst = g.nst;
    if (a.kh == 1 && a.kw == 1 && a.epilogue == SCFLOW_EPI_PLAIN && a.bk != 8 && conv1x1_enabled()) {
      int tr, hr;
      if (launch_tile(a, g, &tr, &hr) == 128) {
        const long long M = (long long)a.n * g.oh * g.ow;
        p.nst = (g.cp0 + g.cp1) / BK;
        conv1x1_kernel<<<dim3((unsigned)((M + 127) / 128), g.npad / BN), 256, 0, st>>>(p);
        return scflow_launch_status();
      }
    }
    switch (a.epilogue) {
      case SCFLOW_EPI_GRU_ZR: return dispatch_mfma<SCFLOW_EPI_GRU_ZR>(p, g, st);
      case SCFLOW_EPI_GRU_Q: return dispatch_mfma<SCFLOW_EPI_GRU_Q>(p, g, st);
      default: return dispatch_mfma<SCFLOW_EPI_PLAIN>(p, g, st);
    }
  }
  if (a.epilogue != SCFLOW_EPI_PLAIN || a.bias_map) return SCFLOW_EUNSUPPORTED;
  const long long M = (long long)a.n * g.oh * g.ow;
  if (g.variant == V_SMALLCIN) {
    const bool mfma_ok = (g.ow == 32 || g.ow == 64) && g.ow == a.w && g.oh == a.h &&
                         g.oh % (64 / g.ow) == 0 && (g.npad == 64 || g.npad == 128) &&
                         (long long)a.n * a.h * a.w * a.s0 * 4 < 0x7ffffff0LL;  // buffer offsets
    if (mfma_ok) {
      const int ntiles = a.n * (g.oh / (64 / g.ow));
      const unsigned blocks = (unsigned)smallcin_blocks(ntiles);
      const size_t lds = 2 * sizeof(float) * (size_t)(64 / g.ow + a.kh - 1) * (g.ow + a.kw - 1) * a.c0;
#define SCFLOW_SCM(CI, KH_, KW_)                                                                   \
  if (a.c0 == CI && a.kh == KH_ && a.kw == KW_) {                                                  \
    if (g.npad == 128 && smallcin_split())                                                         \
      conv_smallcin_mfma_kernel<CI, KH_, KW_, 1><<<dim3(blocks, 2), 256, lds, st>>>(a, g.oh, g.ow, g.npad, ntiles, g_wino_stamps); \
    else if (g.npad == 128)                                                                        \
      conv_smallcin_mfma_kernel<CI, KH_, KW_, 2><<<blocks, 256, lds, st>>>(a, g.oh, g.ow, g.npad, ntiles, g_wino_stamps); \
    else                                                                                           \
      conv_smallcin_mfma_kernel<CI, KH_, KW_, 1><<<blocks, 256, lds, st>>>(a, g.oh, g.ow, g.npad, ntiles, g_wino_stamps); \
    return scflow_launch_status();                                                                 \
  }
      SCFLOW_SCM(2, 7, 7)
      SCFLOW_SCM(1, 3, 3)
      SCFLOW_SCM(2, 3, 3)
#undef SCFLOW_SCM
    }
    const unsigned tiles = (unsigned)((long long)a.n * g.oh * ((g.ow + 31) / 32));
    if (g.npad == 64 || g.npad == 128 || g.npad == 256) {
      if (a.c0 == 2 && a.kh == 7 && a.kw == 7) {
        conv_smallcin_kernel<2, 7, 7><<<tiles, 256, 0, st>>>(a, g.oh, g.ow, g.npad);
        return scflow_launch_status();
      }
      if (a.c0 == 1 && a.kh == 3 && a.kw == 3) {
        conv_smallcin_kernel<1, 3, 3><<<tiles, 256, 0, st>>>(a, g.oh, g.ow, g.npad);
        return scflow_launch_status();
      }
      if (a.c0 == 2 && a.kh == 3 && a.kw == 3) {
        conv_smallcin_kernel<2, 3, 3><<<tiles, 256, 0, st>>>(a, g.oh, g.ow, g.npad);
        return scflow_launch_status();
      }
    }
    dim3 grid((unsigned)((M + 255) / 256), g.npad / 16);
    switch (a.c0) {
      case 1: conv_smallcin_generic<1><<<grid, 256, 0, st>>>(a, g.oh, g.ow, g.npad); break;
      case 2: conv_smallcin_generic<2><<<grid, 256, 0, st>>>(a, g.oh, g.ow, g.npad); break;
      case 3: conv_smallcin_generic<3><<<grid, 256, 0, st>>>(a, g.oh, g.ow, g.npad); break;
      case 4: conv_smallcin_generic<4><<<grid, 256, 0, st>>>(a, g.oh, g.ow, g.npad); break;
      default: return SCFLOW_EUNSUPPORTED;
    }
    return scflow_launch_status();
  }
  // thin
  if (!aligned16(a.src0) || (a.s0 & 3) || (a.c1 > 0 && (!aligned16(a.src1) || (a.s1 & 3))))
    return SCFLOW_EALIGN;
  const bool tiled = (g.ow == 32 || g.ow == 64) && (a.c0 % 8) == 0 && (a.c1 % 8) == 0 &&
                     g.oh % (64 / g.ow) == 0 && g.ow == a.w && g.oh == a.h;
  // channel contraction on MFMA (conv_thinz.h): 3×3 same-padded, one 256-channel source,
  // ≤ 2 outputs; SCFLOW_THINZ = 0 keeps the LDS kernels below (A/B)
  // Measured (profiles/r06/g9_thinz_ab.txt): flow predictor 3×3 256 → 2 at configs[4] 81 → 51 µs
  // alone (decoder 8.84k → 8.88k iters/s), at configs[1] 14.9 → 10.2 µs (decoder 27.49k → 27.72k).
  // The 1×1 256 → 1 mask predictor stays on the chunked kernel (20.8 vs 33.8 µs at configs[4]:
  // one Z column of 32 leaves the MFMAs 97 % idle; configs[1] equal, g10_thinz_mask1x1_ab.txt).
  if (thinz_ok(a, g, tiled)) {
    const int R = g.ow == 64 ? 4 : 2;
    const unsigned blocks = (unsigned)(a.n * (g.oh / R));
#define SCFLOW_THINZ(CO, W_, R_) conv_thinz_kernel<CO, 3, 3, W_, R_><<<blocks, 256, 0, st>>>(a)
    if (g.ow == 64) {
      if (a.cout == 2) SCFLOW_THINZ(2, 64, 4); else SCFLOW_THINZ(1, 64, 4);
    } else {
      if (a.cout == 2) SCFLOW_THINZ(2, 32, 2); else SCFLOW_THINZ(1, 32, 2);
    }
#undef SCFLOW_THINZ
    return scflow_launch_status();
  }
  // whole-halo variant: one source, channels a multiple of 64, the halo within 160 KB of LDS
  static const bool thin_full_off = [] {
    const char* e = getenv("SCFLOW_THIN_FULL");
    return e && e[0] == '0';
  }();
  if (tiled && !thin_full_off && a.c1 == 0 && a.c0 % (4 * THINF_WAVES) == 0) {
    const int tr = 64 / g.ow;
    const unsigned blocks = (unsigned)(a.n * (g.oh / tr));
#define SCFLOW_THINF(CO, KH_, KW_)                                                                if (a.cout == CO && a.kh == KH_ && a.kw == KW_) {                                                 const size_t nh4 = (size_t)(tr + KH_ - 1) * (g.ow + KW_ - 1) * (a.c0 / 4);                      size_t lds = sizeof(float) * (size_t)(tr + KH_ - 1) * (g.ow + KW_ - 1) * thinf_ld(a.c0);        if (lds < sizeof(float) * THINF_WAVES * CO * 64) lds = sizeof(float) * THINF_WAVES * CO * 64;     const size_t nw4 = (size_t)KH_ * KW_ * a.c0 * CO / 4;                                           lds += 16 * nw4; /* the weights behind the halo */                                             if (lds <= 160 * 1024 && nh4 <= (size_t)12 * THINF_WAVES * 64 && nw4 <= (size_t)2 * THINF_WAVES * 64 && aligned16(a.weight)) {                                  static bool attr = false;                                                                       if (!attr) {                                                                                      (void)hipFuncSetAttribute((const void*)conv_thin_full_kernel<CO, KH_, KW_>,                                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);              attr = true;                                                                                  }                                                                                               conv_thin_full_kernel<CO, KH_, KW_><<<blocks, THINF_WAVES * 64, lds, st>>>(a, g.oh, g.ow, g_wino_stamps);       return scflow_launch_status();                                                                }                                                                                             }
    // (1×1: the chunked kernel below is faster — its 32-channel chunks need no halo)
    SCFLOW_THINF(1, 3, 3)
    SCFLOW_THINF(2, 3, 3)
#undef SCFLOW_THINF
  }
  if (tiled) {
    const int tr = 64 / g.ow;
    const unsigned blocks = (unsigned)(a.n * (g.oh / tr));
#define SCFLOW_THIN(CO, KH_, KW_)                                                               \
  if (a.cout == CO && a.kh == KH_ && a.kw == KW_) {                                             \
    size_t lds = sizeof(float) * (size_t)(tr + KH_ - 1) * (g.ow + KW_ - 1) * THIN_LD;           \
    if (lds < sizeof(float) * 4 * CO * 64) lds = sizeof(float) * 4 * CO * 64;                    \
    lds += sizeof(float) * (size_t)KH_ * KW_ * (a.c0 + a.c1) * CO; /* weights */                \
    if (lds > 64 * 1024) (void)hipFuncSetAttribute((const void*)conv_thin_kernel<CO, KH_, KW_>,  \
                                                  hipFuncAttributeMaxDynamicSharedMemorySize,    \
                                                  160 * 1024);                                   \
    conv_thin_kernel<CO, KH_, KW_><<<blocks, 256, lds, st>>>(a, g.oh, g.ow);                    \
    return scflow_launch_status();                                                              \
  }
    SCFLOW_THIN(1, 1, 1)
    SCFLOW_THIN(2, 1, 1)
    SCFLOW_THIN(1, 3, 3)
    SCFLOW_THIN(2, 3, 3)
    SCFLOW_THIN(2, 7, 7)  // training: dX of the 2 → 128 7×7 flow encoders
#undef SCFLOW_THIN
  }
  const unsigned blocks = (unsigned)((M + 3) / 4);
  switch (a.cout) {
    case 1: conv_thin_generic<1><<<blocks, 256, 0, st>>>(a, g.oh, g.ow); break;
    case 2: conv_thin_generic<2><<<blocks, 256, 0, st>>>(a, g.oh, g.ow); break;
    case 3: conv_thin_generic<3><<<blocks, 256, 0, st>>>(a, g.oh, g.ow); break;
    case 4: conv_thin_generic<4><<<blocks, 256, 0, st>>>(a, g.oh, g.ow); break;
    default: return SCFLOW_EUNSUPPORTED;
  }
  return scflow_launch_status();
}

// Two independent convs (neither reads what the other writes) as one grouped launch when a paired
// kernel covers them (conv_pair.h), else as two scflow_conv2d launches in order.  Results equal
// the two separate launches bit for bit.  SCFLOW_CONV_PAIR=0 always launches separately (A/B).
SCFLOW_API int scflow_conv2d_pair(const scflow_conv_args* args_a, const scflow_conv_args* args_b,
                                  void* stream) {
  if (!args_a || !args_b || !conv_args_valid(*args_a) || !conv_args_valid(*args_b))
    return SCFLOW_EINVAL;
  static EnvSwitch pair_sw("SCFLOW_CONV_PAIR", 1);
  if (pair_sw.get()) {
    hipStream_t st = (hipStream_t)stream;
    int r = try_pair(*args_a, *args_b, st);
    if (r == 0) r = try_pair(*args_b, *args_a, st);
    if (r == 1) return SCFLOW_OK;
    if (r != 0) return r;
  }
  const int e = scflow_conv2d(args_a, stream);
  return e ? e : scflow_conv2d(args_b, stream);
}

// The XHeads' hidden conv with both predictors contracted in its epilogue, plus the block / tap
// sum (xhead_pred.h): hidden = the 512-wide F(4×4,3×3) conv args (flow channels first), pred_w
// [hidden.cout][20] packed predictor weights, workspace for the partial sums.
SCFLOW_API long long scflow_xhead_pred_workspace_bytes(int n, int h, int w, int flow_channels,
                                                       int hidden_channels) {
  if (n <= 0 || h <= 0 || w <= 0 || flow_channels <= 0 || flow_channels % 32 ||
      hidden_channels <= flow_channels || hidden_channels % 32)
    return SCFLOW_EINVAL;
  return xhead_pred_ws_bytes((long long)n * h * w, flow_channels / 32,
                             (hidden_channels - flow_channels) / 32);
}

SCFLOW_API int scflow_xhead_pred(const scflow_conv_args* hidden, int flow_channels,
                                 const float* pred_w, float* workspace, long long workspace_bytes,
                                 const float* flow_bias, const float* mask_bias, int flow_act,
                                 int mask_act, float* flow_out, int flow_stride, float* mask_out,
                                 int mask_stride, void* stream) {
  if (!hidden || !hidden->src0 || !hidden->weight || hidden->n <= 0 || hidden->h <= 0 ||
      hidden->w <= 0 || hidden->c0 <= 0 || hidden->c1 < 0 || (hidden->c1 > 0 && !hidden->src1))
    return SCFLOW_EINVAL;
  return launch_xhead_pred(*hidden, flow_channels, pred_w, workspace, workspace_bytes, flow_bias,
                           mask_bias, flow_act, mask_act, flow_out, flow_stride, mask_out,
                           mask_stride, (hipStream_t)stream);
}

// Profiling only: later Winograd launches (F(2×2,3×3) and F(4,5)) write 4 u64 real-time-clock stamps per
// workgroup (start, prologue done, main loop done, epilogue done) to `stamps`, or stop (NULL).
SCFLOW_API int scflow_debug_conv_stamps(void* stamps) {
  g_wino_stamps = (unsigned long long*)stamps;
  return SCFLOW_OK;
}

// the same stamp buffer for the other translation units' instrumented launches (enc_conv_kernel)
unsigned long long* scflow_debug_stamps_ptr() { return g_wino_stamps; }
