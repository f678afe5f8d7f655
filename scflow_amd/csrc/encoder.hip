// §8(f)-1 — RAFTEncoder ('Basic'): the feature encoder (InstanceNorm) and the context encoder
// (BatchNorm with eval statistics) of SCFlowRefiner.extract_feat.
//
// Reference (/root/reference): RAFTEncoder.forward models/encoder/raft_encoder.py:286-314 (stem
// conv1 7×7/2 → norm1 → ReLU, res_layer1..3, conv2 1×1), BasicBlock models/backbone/resnet.py:
// 65-92 (conv3×3 → norm → ReLU → conv3×3 → norm, + identity or downsample(1×1/2 conv → norm),
// ReLU), ResLayer resnet.py:676-771; the encoder is run on the real and the rendered image and
// the context encoder on the rendered one (models/refiner/scflow_refiner.py:96-106).
//
// Kernels:
//  * enc_conv_kernel — implicit GEMM on v_mfma_f32_32x32x2_f32 for every 1×1 / 3×3 conv of the
//    residual stages.  Workgroup tile = TILE_M output pixels (whole output rows, width 32/64/128)
//    × 64 output channels, 4 waves of 32×32 MFMA blocks.  K walks stages of 16 input channels;
//    per stage the input HALO of the tile's rows — ((tr−1)·s + kh) × ((ow−1)·s + kw) pixels —
//    is staged once in LDS (rows padded to 20 floats) together with the stage's weights for
//    every tap, and all taps run out of LDS, with the next stage prefetched into registers.
//    The previous InstanceNorm + ReLU is applied to the staged halo (per (image, channel) scale
//    and shift; padding stays zero) so normalised activations are never written to HBM;
//    the epilogue fuses bias, an eval-BatchNorm affine, the residual add and the activation
//    (or a split tanh | relu for the context output).
//  * enc_stem_mfma_kernel — the 3-channel 7×7 stem as an implicit GEMM on fp32 MFMA (64 output
//    channels); enc_stem_kernel — the VALU form for wider stems: lane = output channel with its
//    147 weights in VGPRs, the tile's input halo staged from the NCHW image in LDS.
//  * enc_stats_kernel / enc_norm_finalize_kernel — InstanceNorm statistics in fp64 (partial sums
//    over pixel chunks, deterministic order), → per (image, channel) scale/shift.
//  * enc_apply_kernel — relu(norm(x) + identity') where the block output must be materialised
//    (the next block's identity), float4-vectorised.
#include "common.h"

unsigned long long* scflow_debug_stamps_ptr();  // conv.hip (scflow_debug_conv_stamps)

namespace {

constexpr int EBN = 64;  // output channels per workgroup
constexpr int EBK = 16;  // input channels per K stage
constexpr int ELDA = EBK + 4;

// float4 of the A halo per thread, worst case over tile widths tc = 8..TILE_M (tr = TILE_M/tc
// output rows of tc pixels)
constexpr int enc_na(int tm, int kh, int kw, int s) {
  int m = 0;
  for (int tc = 8; tc <= tm; tc *= 2) {
    const int tr = tm / tc;
    const int v = ((tr - 1) * s + kh) * ((tc - 1) * s + kw) * (EBK / 4);
    if (v > m) m = v;
  }
  return (m + 255) / 256;
}

struct EncParams {
  scflow_enc_conv_args a;
  int oh, ow, tr, tc, hr, hc, nst;  // output size, tile rows × cols, halo rows × cols, K stages
  int nst0;                         // stages of the first source
  int arp4;                         // A halo row pitch (float4; enc_a4, enc_row_pitch)
  unsigned long long* stamps;       // profiling (scflow_debug_conv_stamps), or NULL
};

// thread 0's real-time-clock stamp k of this workgroup (0 start, 1 first stage staged, 2 main
// loop done, 3 epilogue done; grid.z slabs after grid.y)
__device__ __forceinline__ void enc_stamp(unsigned long long* st, int k) {
  if (st && threadIdx.x == 0)
    st[(((size_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * 4 + k] =
        __builtin_amdgcn_s_memrealtime();
}

// A halo layout (float4 units): pixel (hr, hcol) at hr·arp4 + 5·hcol (+ one float4 every 2
// columns for stride 2, so the taps of consecutive output pixels — 2 columns apart — step by an
// odd 11 slots), the row pitch chosen on the host by a bank model of ds_read_b128's lane groups
// (enc_row_pitch): conflict-free A reads where a lane group spans several output rows
template <int S>
__host__ __device__ constexpr int enc_a4(int hr, int hcol, int arp4) {
  return hr * arp4 + hcol * (ELDA / 4) + (S == 2 ? hcol >> 1 : 0);
}

template <int KH, int KW, int S, int TILE_M, bool NORM>
__global__ __launch_bounds__(256, 2) void enc_conv_kernel(EncParams P) {
  constexpr int TAPS = KH * KW;
  constexpr int RB = TILE_M / 64;
  constexpr int NA = enc_na(TILE_M, KH, KW, S);
  constexpr int NB = TAPS * EBN * (EBK / 4) / 256;
  extern __shared__ float smem[];
  const scflow_enc_conv_args& a = P.a;
  const int hc = P.hc, ow = P.ow, tc = P.tc;
  floatx4* As4 = (floatx4*)smem;                       // [hr][arp4] float4 (enc_a4)
  const float* As = smem;
  float* Bs = smem + (size_t)P.hr * P.arp4 * 4;  // [TAPS][EBN][ELDA]
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave & 1, wn = wave >> 1, li = lane & 31, hh = lane >> 5;
  const int tiles_x = ow / tc;
  const int tiles_per_img = (P.oh / P.tr) * tiles_x;
  const int img = blockIdx.x / tiles_per_img;
  const int tin = blockIdx.x % tiles_per_img;
  const int oy0 = (tin / tiles_x) * P.tr, ox0 = (tin % tiles_x) * tc;
  const int n0 = blockIdx.y * EBN;
  const int na = P.hr * hc * (EBK / 4);
  const int cq = 4 * (tid & 3);  // this thread's 4 channels within every stage (stage-invariant)

  int apix[NA], alds[NA];
#pragma unroll
  for (int j = 0; j < NA; ++j) {
    const int idx = tid + 256 * j;
    const int pix = idx >> 2;
    const int hr = pix / hc, hcol = pix - hr * hc;
    const int iy = oy0 * S - a.pad + hr, ix = ox0 * S - a.pad + hcol;
    const bool ok = idx < na && iy >= 0 && iy < a.h && ix >= 0 && ix < a.w;
    apix[j] = ok ? (img * a.h + iy) * a.w + ix : -1;
    alds[j] = enc_a4<S>(hr, hcol, P.arp4) + (cq >> 2);
  }

  // K split (grid.z): this workgroup's stage range
  const int z = blockIdx.z, nsplit = gridDim.z;
  const int s_begin = (int)((long long)P.nst * z / nsplit);
  const int s_end = (int)((long long)P.nst * (z + 1) / nsplit);
  const int ctot = a.cin + a.cin1;

  floatx4 ra[NA], rb[NB], rsc, rsh;
  auto gload = [&](int s) {
    const bool second = s >= P.nst0;
    const float* src = second ? a.src1 : a.src;
    const int sin = second ? a.s_in1 : a.s_in;
    const int c = (second ? s - P.nst0 : s) * EBK + cq;
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      floatx4 v = {0.f, 0.f, 0.f, 0.f};
      if (apix[j] >= 0) v = *(const floatx4*)(src + (size_t)apix[j] * sin + c);
      ra[j] = v;
    }
    if constexpr (NORM) {
      const int cn = s * EBK + cq;  // channel in the concatenation
      rsc = *(const floatx4*)(a.in_scale + (size_t)img * ctot + cn);
      rsh = *(const floatx4*)(a.in_shift + (size_t)img * ctot + cn);
    }
    const float* wb = a.weight + ((size_t)blockIdx.y * P.nst + s) * (TAPS * EBN * EBK);
#pragma unroll
    for (int j = 0; j < NB; ++j) rb[j] = *(const floatx4*)(wb + (size_t)(tid + 256 * j) * 4);
  };
  auto lstore = [&]() {
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      const int idx = tid + 256 * j;
      floatx4 v = ra[j];
      if constexpr (NORM) {
        if (apix[j] >= 0) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e] * rsc[e] + rsh[e], 0.f);
        }
      }
      if (idx < na) As4[alds[j]] = v;
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int idx = tid + 256 * j;
      *(floatx4*)(Bs + (idx >> 2) * ELDA + 4 * (idx & 3)) = rb[j];
    }
  };

  int abase[RB];
#pragma unroll
  for (int r = 0; r < RB; ++r) {
    const int m = wm * (TILE_M / 2) + r * 32 + li;
    abase[r] = enc_a4<S>((m / tc) * S, (m % tc) * S, P.arp4) * 4 + 4 * hh;
  }
  const int bbase = (wn * 32 + li) * ELDA + 4 * hh;

  floatx16 acc[RB];
#pragma unroll
  for (int r = 0; r < RB; ++r)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[r][e] = 0.f;

  enc_stamp(P.stamps, 0);
  gload(s_begin);
  for (int s = s_begin; s < s_end; ++s) {
    __syncthreads();
    lstore();
    __syncthreads();
    if (s == s_begin) enc_stamp(P.stamps, 1);
    if (s + 1 < s_end) gload(s + 1);
#pragma unroll
    for (int ty = 0; ty < KH; ++ty) {
#pragma unroll
      for (int tx = 0; tx < KW; ++tx) {
        const int aoff = enc_a4<S>(ty, tx, P.arp4) * 4;  // (tile columns start even for S = 2)
        const float* Bb = Bs + (ty * KW + tx) * EBN * ELDA + bbase;
#pragma unroll
        for (int kb = 0; kb < EBK; kb += 8) {
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

  enc_stamp(P.stamps, 2);
  // epilogue; C/D layout: col = lane&31, row = (r&3) + 8(r>>2) + 4(lane>>5)
  const int col = n0 + wn * 32 + li;
  if (col >= a.cout) return;
  const float bias = a.bias ? a.bias[col] : 0.f;
  const float osc = a.out_scale ? a.out_scale[col] : 1.f;
  const float osh = a.out_scale ? a.out_shift[col] : 0.f;
  const int act = col < a.act_split ? a.act : a.act2;
  float* outz = a.out + (size_t)z * ((size_t)a.n * P.oh * P.ow * a.s_out);
  // every residual read is issued before any store (the stores may alias them as far as the
  // compiler knows; interleaved, each read's latency would be serialised)
  int pixv[RB][16];
#pragma unroll
  for (int rr = 0; rr < RB; ++rr)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = wm * (TILE_M / 2) + rr * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
      const int oy = oy0 + m / tc, ox = ox0 + m % tc;
      pixv[rr][r] = (img * P.oh + oy) * ow + ox;
    }
  float resv[RB][16];
#pragma unroll
  for (int rr = 0; rr < RB; ++rr)
#pragma unroll
    for (int r = 0; r < 16; ++r) resv[rr][r] = a.res ? a.res[(size_t)pixv[rr][r] * a.s_res + col] : 0.f;
#pragma unroll
  for (int rr = 0; rr < RB; ++rr) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float v = acc[rr][r] + bias;
      if (a.out_scale) v = v * osc + osh;
      v += resv[rr][r];
      outz[(size_t)pixv[rr][r] * a.s_out + col] = act_apply(v, act);
    }
  }
  if (P.stamps) {
    __builtin_amdgcn_s_waitcnt(0);
    enc_stamp(P.stamps, 3);
  }
}

// packed weights: [npad/EBN][nst][taps][EBN][EBK]
__global__ void enc_pack_kernel(const float* __restrict__ w, float* __restrict__ out, int cout,
                                int cin, int taps, int nst, long long total) {
  for (long long idx = blockIdx.x * 256LL + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * 256) {
    long long r = idx;
    const int k = (int)(r % EBK); r /= EBK;
    const int col = (int)(r % EBN); r /= EBN;
    const int tap = (int)(r % taps); r /= taps;
    const int s = (int)(r % nst);
    const int nt = (int)(r / nst);
    const int o = nt * EBN + col, ci = s * EBK + k;
    out[idx] = (o < cout && ci < cin) ? w[((size_t)o * cin + ci) * taps + tap] : 0.f;
  }
}

// ------------------------------------------------------------------------------------------
// stem: NCHW image → channels-last; tile = 32 consecutive output pixels of one row; wave w
// takes channel group w % G (G = npad/64) and a share of the pixels.  packed [taps·cin][npad].
// ------------------------------------------------------------------------------------------
template <int CIN, int KH, int KW, int S>
__global__ __launch_bounds__(256) void enc_stem_kernel(const float* __restrict__ img_in,
                                                       const float* __restrict__ wpk,
                                                       const float* __restrict__ bias,
                                                       const float* __restrict__ osc_,
                                                       const float* __restrict__ osh_,
                                                       float* __restrict__ out, int h, int w,
                                                       int oh, int ow, int cout, int npad, int pad,
                                                       int act) {
  constexpr int HCOLS = 31 * S + KW;
  __shared__ float halo[KH][HCOLS][CIN];
  const int tiles_x = (ow + 31) / 32;
  const int t = blockIdx.x;
  const int tx0 = (t % tiles_x) * 32;
  const int oy = (t / tiles_x) % oh;
  const int img = t / (tiles_x * oh);
  for (int i = threadIdx.x; i < KH * HCOLS * CIN; i += 256) {
    const int col = i % HCOLS, row = (i / HCOLS) % KH, c = i / (HCOLS * KH);
    const int iy = oy * S - pad + row, ix = tx0 * S - pad + col;
    float v = 0.f;
    if (iy >= 0 && iy < h && ix >= 0 && ix < w) v = img_in[(((size_t)img * CIN + c) * h + iy) * w + ix];
    halo[row][col][c] = v;
  }
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int G = npad / 64;
  const int grp = wave % G;
  const int pw_ = 32 / (4 / G);
  const int p0 = (wave / G) * pw_;
  const int co = grp * 64 + lane;
  float wr[KH * KW * CIN];
#pragma unroll
  for (int k = 0; k < KH * KW * CIN; ++k) wr[k] = wpk[(size_t)k * npad + co];
  const bool okc = co < cout;
  const float b = (bias && okc) ? bias[co] : 0.f;
  const float osc = (osc_ && okc) ? osc_[co] : 1.f;
  const float osh = (osc_ && okc) ? osh_[co] : 0.f;
  __syncthreads();
  for (int p = p0; p < p0 + pw_; ++p) {
    const int ox = tx0 + p;
    if (ox >= ow) break;
    float acc = 0.f;
#pragma unroll
    for (int ty = 0; ty < KH; ++ty)
#pragma unroll
      for (int tx = 0; tx < KW; ++tx)
#pragma unroll
        for (int c = 0; c < CIN; ++c) acc += wr[(ty * KW + tx) * CIN + c] * halo[ty][p * S + tx][c];
    float v = acc + b;
    if (osc_) v = v * osc + osh;
    if (okc) out[((size_t)(img * oh + oy) * ow + ox) * cout + co] = act_apply(v, act);
  }
}

// ------------------------------------------------------------------------------------------
// stem on the matrix cores (npad = 64): implicit GEMM, M = 128 output pixels of one row (wave
// w: pixels 32w..32w+31), N = 64 channels (two 32-column blocks), K = KH·KW·CIN taps (147 → 74
// k-pairs of v_mfma_f32_32x32x2_f32).  A workgroup runs STEM_ROWS (8) consecutive output rows: the
// packed weights [K][64] are staged in LDS once, each row's input halo [CIN][KH][HC] is staged
// in LDS from registers that were loaded while the previous row's MFMAs ran.  A lane reads its A
// value (pixel li, tap k = 2kp + hh) and its two B values straight from LDS — the tap offsets
// fold to constants in the unrolled K loop.  Same epilogue as enc_stem_kernel.  (The VALU kernel
// paid one LDS broadcast per FMA: ~25 TFLOP/s.)
// ------------------------------------------------------------------------------------------
template <int CIN, int KH, int KW, int S, int STEM_ROWS>
__global__ __launch_bounds__(256, 2) void enc_stem_mfma_kernel(
    const float* __restrict__ img_in, const float* __restrict__ wpk, const float* __restrict__ bias,
    const float* __restrict__ osc_, const float* __restrict__ osh_, float* __restrict__ out, int h,
    int w, int oh, int ow, int cout, int pad, int act) {
  constexpr int K = KH * KW * CIN;
  constexpr int KP = (K + 1) / 2;
  constexpr int HC = 127 * S + KW;
  constexpr int NH = KH * HC * CIN;
  constexpr int NJ = (NH + 255) / 256;
  __shared__ float halo[NH];
  __shared__ float ws[2 * KP * 64];
  const int tiles_x = (ow + 127) / 128;
  const int row_blocks = (oh + STEM_ROWS - 1) / STEM_ROWS;
  const int t = blockIdx.x;
  const int tx0 = (t % tiles_x) * 128;
  const int oy0 = ((t / tiles_x) % row_blocks) * STEM_ROWS;
  const int img = t / (tiles_x * row_blocks);
  const int oy1 = oy0 + STEM_ROWS < oh ? oy0 + STEM_ROWS : oh;
  float pre[NJ];
  auto gload = [&](int oy) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int i = threadIdx.x + 256 * j;
      const int col = i % HC, row = (i / HC) % KH, c = i / (HC * KH);
      const int iy = oy * S - pad + row, ix = tx0 * S - pad + col;
      float v = 0.f;
      if (i < NH && iy >= 0 && iy < h && ix >= 0 && ix < w)
        v = img_in[(((size_t)img * CIN + c) * h + iy) * w + ix];
      pre[j] = v;
    }
  };
  auto lstore = [&]() {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int i = threadIdx.x + 256 * j;
      if (i < NH) halo[i] = pre[j];
    }
  };
  gload(oy0);
  for (int i = threadIdx.x; i < 2 * KP * 64; i += 256) ws[i] = i < K * 64 ? wpk[i] : 0.f;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, li = lane & 31, hh = lane >> 5;
  const float* hp = halo + (wave * 32 + li) * S;
  const float* wp = ws + hh * 64 + li;
  float bv[2], sc[2], sh[2];
#pragma unroll
  for (int nb = 0; nb < 2; ++nb) {
    const int co = nb * 32 + li;
    const bool ok = co < cout;
    bv[nb] = (bias && ok) ? bias[co] : 0.f;
    sc[nb] = (osc_ && ok) ? osc_[co] : 1.f;
    sh[nb] = (osc_ && ok) ? osh_[co] : 0.f;
  }
  for (int oy = oy0; oy < oy1; ++oy) {
    __syncthreads();  // the previous row's MFMAs are done with the halo
    lstore();
    __syncthreads();
    if (oy + 1 < oy1) gload(oy + 1);
    floatx16 acc0, acc1;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc0[e] = acc1[e] = 0.f;
#pragma unroll
    for (int kp = 0; kp < KP; ++kp) {
      // tap offsets of k = 2kp and 2kp + 1 in the halo (the padding tap k = K reads tap 0: its
      // weight row is zero)
      const int k0 = 2 * kp, k1 = 2 * kp + 1 < K ? 2 * kp + 1 : 0;
      const int o0 = ((k0 % CIN) * KH + (k0 / CIN) / KW) * HC + (k0 / CIN) % KW;
      const int o1 = ((k1 % CIN) * KH + (k1 / CIN) / KW) * HC + (k1 / CIN) % KW;
      const float a = hp[hh ? o1 : o0];
      const float b0 = wp[kp * 128], b1 = wp[kp * 128 + 32];
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b0, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b1, acc1, 0, 0, 0);
    }
    // C/D layout: col = lane&31, row = (r&3) + 8(r>>2) + 4(lane>>5)
    float* orow = out + (size_t)(img * oh + oy) * ow * cout;
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      const int co = nb * 32 + li;
      if (co >= cout) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ox = tx0 + wave * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
        if (ox >= ow) continue;
        float v = (nb ? acc1[r] : acc0[r]) + bv[nb];
        if (osc_) v = v * sc[nb] + sh[nb];
        orow[(size_t)ox * cout + co] = act_apply(v, act);
      }
    }
  }
}

__global__ void enc_stem_pack_kernel(const float* __restrict__ w, float* __restrict__ out, int cout,
                                     int cin, int taps, int npad, long long total) {
  for (long long idx = blockIdx.x * 256LL + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * 256) {
    const int o = (int)(idx % npad);
    const int k = (int)(idx / npad);
    const int tap = k / cin, ci = k % cin;
    out[idx] = o < cout ? w[((size_t)o * cin + ci) * taps + tap] : 0.f;
  }
}

// ------------------------------------------------------------------------------------------
// InstanceNorm statistics: grid (chunks, n); thread = 4 channels × a pixel lane; fp64 sums
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void enc_stats_kernel(const float* __restrict__ x, int hw, int c,
                                                        int chunks, double* __restrict__ partial) {
  __shared__ double red[2][256][4];
  const int img = blockIdx.y, ch = blockIdx.x;
  const int tpp = c / 4;          // threads per pixel
  const int ppp = 256 / tpp;      // pixels per pass
  const int q = threadIdx.x % tpp, ps = threadIdx.x / tpp;
  const int p_begin = (int)((long long)hw * ch / chunks), p_end = (int)((long long)hw * (ch + 1) / chunks);
  double s[4] = {0, 0, 0, 0}, s2[4] = {0, 0, 0, 0};
  if (ps < ppp) {
    const float* xb = x + (size_t)img * hw * c + 4 * q;
    for (int p = p_begin + ps; p < p_end; p += ppp) {
      const floatx4 v = *(const floatx4*)(xb + (size_t)p * c);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        s[e] += (double)v[e];
        s2[e] += (double)v[e] * (double)v[e];
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    red[0][threadIdx.x][e] = s[e];
    red[1][threadIdx.x][e] = s2[e];
  }
  __syncthreads();
  // thread t < c: channel t = 4q + e, summed over the pixel slots in a fixed order
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

__global__ void enc_norm_finalize_kernel(const double* __restrict__ partial, int n, int chunks,
                                         int c, int hw, float eps, float* __restrict__ scale,
                                         float* __restrict__ shift) {
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
  const double mean = s / hw;
  double var = s2 / hw - mean * mean;
  if (var < 0) var = 0;
  const float sc = (float)(1.0 / sqrt(var + (double)eps));
  scale[i] = sc;
  shift[i] = (float)(-mean) * sc;
}

__global__ __launch_bounds__(256) void enc_apply_kernel(
    const float* __restrict__ x, const float* __restrict__ sc, const float* __restrict__ sh,
    const float* __restrict__ id, const float* __restrict__ isc, const float* __restrict__ ish,
    float* __restrict__ out, int hw, int c, long long total4) {
  const int c4 = c / 4;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total4; i += (long long)gridDim.x * 256) {
    const int cq = (int)(i % c4) * 4;
    const long long pix = i / c4;
    const int img = (int)(pix / hw);
    const size_t so = (size_t)img * c + cq;
    const floatx4 v = ((const floatx4*)x)[i];
    const floatx4 a = *(const floatx4*)(sc + so), b = *(const floatx4*)(sh + so);
    floatx4 r;
#pragma unroll
    for (int e = 0; e < 4; ++e) r[e] = v[e] * a[e] + b[e];
    if (id) {
      floatx4 u = ((const floatx4*)id)[i];
      if (isc) {
        const floatx4 ua = *(const floatx4*)(isc + so), ub = *(const floatx4*)(ish + so);
#pragma unroll
        for (int e = 0; e < 4; ++e) u[e] = u[e] * ua[e] + ub[e];
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) r[e] += u[e];
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) r[e] = fmaxf(r[e], 0.f);
    ((floatx4*)out)[i] = r;
  }
}

int rup(int a, int b) { return (a + b - 1) / b * b; }

// A halo row pitch (float4): the smallest ≥ the row's extent whose A-fragment reads are
// conflict-free — ds_read_b128 serves a wave in 16-lane groups {0-3, 12-15, 20-27},
// {4-11, 16-19, 28-31} (and +32, the other channel quad), each reading one 256-B bank row: the
// group's 16 lanes must address 16 distinct 16-B slots (MI355X_MICROARCH.md §LDS).  Lane li of
// wave (wm, ·) reads output pixel m = wm·TM/2 + 32r + li; the least-conflicted pitch of 16
// candidates wins.
template <int S>
int enc_row_pitch(int tc, int tm, int hc) {
  static const int groups[2][16] = {{0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27},
                                    {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31}};
  const int base = enc_a4<S>(0, hc, 0);  // ≥ the row's last pixel + 1
  int best = base, best_cost = 1 << 30;
  for (int pad = 0; pad < 16; ++pad) {
    const int rp = base + pad;
    int cost = 0;
    for (int wm = 0; wm < 2; ++wm)
      for (int r = 0; r < tm / 64; ++r)
        for (int g = 0; g < 2; ++g) {
          int cnt[16] = {0}, worst = 0;
          for (int i = 0; i < 16; ++i) {
            const int m = wm * (tm / 2) + 32 * r + groups[g][i];
            const int sl = enc_a4<S>((m / tc) * S, (m % tc) * S, rp) & 15;
            worst = ++cnt[sl] > worst ? cnt[sl] : worst;
          }
          cost += worst;
        }
    if (cost < best_cost) {
      best_cost = cost;
      best = rp;
    }
  }
  return best;
}

template <int KH, int KW, int S, int TM, bool NORM>
int launch_enc(EncParams p, hipStream_t st) {
  p.tc = p.ow < TM ? p.ow : TM;
  if (p.tc < 8 || TM % p.tc || p.ow % p.tc) return SCFLOW_EUNSUPPORTED;
  p.tr = TM / p.tc;
  if (p.oh % p.tr) return SCFLOW_EUNSUPPORTED;
  p.hr = (p.tr - 1) * S + KH;
  p.hc = (p.tc - 1) * S + KW;
  p.arp4 = enc_row_pitch<S>(p.tc, TM, p.hc);
  const size_t lds = sizeof(float) * ((size_t)p.hr * p.arp4 * 4 + (size_t)KH * KW * EBN * ELDA);
  if ((size_t)p.hr * p.hc * (EBK / 4) > (size_t)256 * enc_na(TM, KH, KW, S)) return SCFLOW_EUNSUPPORTED;
  static bool attr = false;
  if (lds > 64 * 1024 && !attr) {
    (void)hipFuncSetAttribute((const void*)enc_conv_kernel<KH, KW, S, TM, NORM>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  dim3 grid(p.a.n * (p.oh / p.tr) * (p.ow / p.tc), rup(p.a.cout, EBN) / EBN,
            p.a.ksplit > 1 ? p.a.ksplit : 1);
  enc_conv_kernel<KH, KW, S, TM, NORM><<<grid, 256, lds, st>>>(p);
  return scflow_launch_status();
}

template <int KH, int KW, int S, int TM>
int launch_enc_norm(const EncParams& p, hipStream_t st) {
  return p.a.in_scale ? launch_enc<KH, KW, S, TM, true>(p, st) : launch_enc<KH, KW, S, TM, false>(p, st);
}

}  // namespace

SCFLOW_API long long scflow_enc_conv_packed_size(int cout, int cin, int kh, int kw) {
  // cin = all input channels (cin + cin1 of the conv args)
  if (cout <= 0 || cin <= 0 || kh <= 0 || kw <= 0) return SCFLOW_EINVAL;
  return (long long)rup(cout, EBN) * rup(cin, EBK) * kh * kw;
}

SCFLOW_API int scflow_enc_conv_pack(const float* w_oihw, float* packed, int cout, int cin, int kh,
                                    int kw, void* stream) {
  if (!w_oihw || !packed || cout <= 0 || cin <= 0 || kh <= 0 || kw <= 0) return SCFLOW_EINVAL;
  const long long total = scflow_enc_conv_packed_size(cout, cin, kh, kw);
  const int blocks = (int)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
  enc_pack_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(w_oihw, packed, cout, cin, kh * kw,
                                                           rup(cin, EBK) / EBK, total);
  return scflow_launch_status();
}

SCFLOW_API int scflow_enc_conv(const scflow_enc_conv_args* args, void* stream) {
  if (!args) return SCFLOW_EINVAL;
  const scflow_enc_conv_args& a = *args;
  if (!a.src || !a.weight || !a.out || a.n <= 0 || a.h <= 0 || a.w <= 0 || a.cout <= 0 ||
      a.cin <= 0 || a.pad < 0 || a.stride < 1 || a.s_in < a.cin || a.s_out < a.cout ||
      (a.res && a.s_res < a.cout) || (!a.in_scale) != (!a.in_shift) ||
      (!a.out_scale) != (!a.out_shift))
    return SCFLOW_EINVAL;
  if (a.cin1 < 0 || (a.cin1 > 0 && (!a.src1 || a.s_in1 < a.cin1)) || a.ksplit < 0) return SCFLOW_EINVAL;
  if (a.ksplit > 1 && (a.bias || a.out_scale || a.res || a.act || a.act2)) return SCFLOW_EINVAL;
  if (a.cin % EBK || a.cin1 % EBK) return SCFLOW_EUNSUPPORTED;
  if (!aligned16(a.src) || (a.s_in & 3) || !aligned16(a.weight) ||
      (a.cin1 > 0 && (!aligned16(a.src1) || (a.s_in1 & 3))) ||
      (a.in_scale && (!aligned16(a.in_scale) || !aligned16(a.in_shift))))
    return SCFLOW_EALIGN;
  EncParams p{};
  p.a = a;
  p.stamps = scflow_debug_stamps_ptr();
  p.oh = (a.h + 2 * a.pad - a.kh) / a.stride + 1;
  p.ow = (a.w + 2 * a.pad - a.kw) / a.stride + 1;
  p.nst0 = a.cin / EBK;
  p.nst = (a.cin + a.cin1) / EBK;
  if (a.ksplit > p.nst) return SCFLOW_EINVAL;
  if (p.oh <= 0 || p.ow <= 0) return SCFLOW_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  if (a.kh == 3 && a.kw == 3 && a.stride == 1) return launch_enc_norm<3, 3, 1, 128>(p, st);
  if (a.kh == 3 && a.kw == 3 && a.stride == 2) return launch_enc_norm<3, 3, 2, 64>(p, st);
  if (a.kh == 1 && a.kw == 1 && a.stride == 1) return launch_enc_norm<1, 1, 1, 128>(p, st);
  if (a.kh == 1 && a.kw == 1 && a.stride == 2) return launch_enc_norm<1, 1, 2, 64>(p, st);
  return SCFLOW_EUNSUPPORTED;
}

SCFLOW_API long long scflow_enc_stem_packed_size(int cout, int cin, int kh, int kw) {
  if (cout <= 0 || cin <= 0 || kh <= 0 || kw <= 0) return SCFLOW_EINVAL;
  return (long long)kh * kw * cin * rup(cout, 64);
}

SCFLOW_API int scflow_enc_stem_pack(const float* w_oihw, float* packed, int cout, int cin, int kh,
                                    int kw, void* stream) {
  if (!w_oihw || !packed || cout <= 0 || cin <= 0 || kh <= 0 || kw <= 0) return SCFLOW_EINVAL;
  const long long total = scflow_enc_stem_packed_size(cout, cin, kh, kw);
  const int blocks = (int)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
  enc_stem_pack_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(w_oihw, packed, cout, cin, kh * kw,
                                                                rup(cout, 64), total);
  return scflow_launch_status();
}

SCFLOW_API int scflow_enc_stem(const float* img, const float* packed, const float* bias,
                               const float* out_scale, const float* out_shift, float* out, int n,
                               int cin, int h, int w, int cout, int kh, int kw, int stride,
                               int pad, int act, void* stream) {
  if (!img || !packed || !out || n <= 0 || h <= 0 || w <= 0 || cout <= 0 || pad < 0 ||
      (!out_scale) != (!out_shift))
    return SCFLOW_EINVAL;
  const int npad = rup(cout, 64);
  if (npad > 256 || npad == 192) return SCFLOW_EUNSUPPORTED;
  const int oh = (h + 2 * pad - kh) / stride + 1, ow = (w + 2 * pad - kw) / stride + 1;
  if (oh <= 0 || ow <= 0) return SCFLOW_EINVAL;
  const unsigned tiles = (unsigned)((long long)n * oh * ((ow + 31) / 32));
  hipStream_t st = (hipStream_t)stream;
  static int mfma = -1;  // SCFLOW_STEM_MFMA=0 keeps the VALU kernel (A/B only)
  if (mfma < 0) {
    const char* e = getenv("SCFLOW_STEM_MFMA");
    mfma = e ? atoi(e) != 0 : 1;
  }
  if (mfma && npad == 64 && cin == 3 && kh == 7 && kw == 7 && (stride == 1 || stride == 2)) {
    static int srows = 0;  // output rows per workgroup (SCFLOW_STEM_ROWS=4|8|16, tuning)
    if (!srows) {
      const char* e = getenv("SCFLOW_STEM_ROWS");
      srows = e ? atoi(e) : 8;  // 4 / 8 / 16 rows: 226 / 208 / 230 us per e2e stem call
      if (srows != 4 && srows != 16) srows = 8;
    }
    const unsigned rows = (unsigned)((long long)n * ((oh + srows - 1) / srows) * ((ow + 127) / 128));
#define STEM_LAUNCH(S_, R_)                                                                   \
  enc_stem_mfma_kernel<3, 7, 7, S_, R_><<<rows, 256, 0, st>>>(img, packed, bias, out_scale, \
                                                              out_shift, out, h, w, oh, ow,  \
                                                              cout, pad, act)
    if (stride == 2) {
      if (srows == 16) STEM_LAUNCH(2, 16);
      else if (srows == 4) STEM_LAUNCH(2, 4);
      else STEM_LAUNCH(2, 8);
    } else {
      STEM_LAUNCH(1, 4);
    }
#undef STEM_LAUNCH
    return scflow_launch_status();
  }
  if (cin == 3 && kh == 7 && kw == 7 && stride == 2) {
    enc_stem_kernel<3, 7, 7, 2><<<tiles, 256, 0, st>>>(img, packed, bias, out_scale, out_shift, out,
                                                       h, w, oh, ow, cout, npad, pad, act);
    return scflow_launch_status();
  }
  if (cin == 3 && kh == 7 && kw == 7 && stride == 1) {
    enc_stem_kernel<3, 7, 7, 1><<<tiles, 256, 0, st>>>(img, packed, bias, out_scale, out_shift, out,
                                                       h, w, oh, ow, cout, npad, pad, act);
    return scflow_launch_status();
  }
  return SCFLOW_EUNSUPPORTED;
}

SCFLOW_API int scflow_enc_stats(const float* x, int n, int hw, int c, int chunks, double* partial,
                                void* stream) {
  if (!x || !partial || n <= 0 || hw <= 0 || c <= 0 || chunks <= 0) return SCFLOW_EINVAL;
  if (c % 4 || c > 256) return SCFLOW_EUNSUPPORTED;
  if (!aligned16(x)) return SCFLOW_EALIGN;
  dim3 grid(chunks, n);
  enc_stats_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(x, hw, c, chunks, partial);
  return scflow_launch_status();
}

SCFLOW_API int scflow_enc_norm_finalize(const double* partial, int n, int chunks, int c, int hw,
                                        float eps, float* scale, float* shift, void* stream) {
  if (!partial || !scale || !shift || n <= 0 || chunks <= 0 || c <= 0 || hw <= 0) return SCFLOW_EINVAL;
  enc_norm_finalize_kernel<<<ceil_div((long long)n * c, 256), 256, 0, (hipStream_t)stream>>>(
      partial, n, chunks, c, hw, eps, scale, shift);
  return scflow_launch_status();
}

SCFLOW_API int scflow_enc_apply(const float* x, const float* scale, const float* shift,
                                const float* id, const float* id_scale, const float* id_shift,
                                float* out, int n, int hw, int c, void* stream) {
  if (!x || !scale || !shift || !out || n <= 0 || hw <= 0 || c <= 0 ||
      (!id_scale) != (!id_shift) || (id_scale && !id))
    return SCFLOW_EINVAL;
  if (c % 4) return SCFLOW_EUNSUPPORTED;
  if (!aligned16(x) || !aligned16(out) || !aligned16(scale) || !aligned16(shift) ||
      (id && !aligned16(id)) || (id_scale && (!aligned16(id_scale) || !aligned16(id_shift))))
    return SCFLOW_EALIGN;
  const long long total4 = (long long)n * hw * c / 4;
  const int blocks = (int)((total4 + 255) / 256 < 16384 ? (total4 + 255) / 256 : 16384);
  enc_apply_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(x, scale, shift, id, id_scale, id_shift,
                                                            out, hw, c, total4);
  return scflow_launch_status();
}
