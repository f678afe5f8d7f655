// Channels-last fp32 convolutions of the SCFlow update block, with fused epilogues.
//
// Reference modules replaced (all mmcv ConvModule = conv + bias + act, /root/reference):
//   ConvGRU SeqConv (1×5 then 5×1, z/r/q gates)      models/decoder/raft_decoder.py:180-253
//   MotionEncoder corr_net / flow_net / out_net       models/decoder/raft_decoder.py:75-166
//   XHead flow / mask                                  models/decoder/raft_decoder.py:256-294
//   delta_flow_encoder / mask_encoder                  models/decoder/scflow_decoder.py:103-124
//
// Three kernels, chosen by shape (select_variant, shared by packing and launching):
//  * conv_mfma  — implicit GEMM on v_mfma_f32_32x32x2_f32 (exact fp32, the chip's f32 matrix
//    rate).  Workgroup tile = 128 output pixels (128/W whole image rows) × 64 output channels;
//    4 waves, each 64 px × 32 ch (two 32×32 MFMA accumulators).  Per K-stage (16 input channels
//    of one source) the workgroup stages the input HALO of its rows once — (rows+kh−1)×(W+kw−1)
//    pixels — plus the weights of every tap, so each input pixel is fetched once per stage
//    instead of kh·kw times; all taps then run out of LDS (pixel rows padded to 20 floats:
//    ds_read_b128 conflict-free).  Second input source = channel concat without a copy
//    (GRU's cat[h,x] / cat[r·h,x], MotionEncoder's cat[corr,flow]).  Epilogues: bias+act, or the
//    GRU gates: ZR writes z and r·h; Q computes h ← (1−z)·h + z·tanh(q) in place.
//  * conv_smallcin — VALU direct conv for cin ≤ 4 (the 7×7 2→128 flow encoders, 3×3 1→64 mask
//    encoder): one thread per pixel × 16 output channels, weights wave-uniform.
//  * conv_thin — cout ≤ 4 (flow head 3×3 256→2, mask head 1×1 256→1): one wave per pixel,
//    lanes split the channels (float4 each), wave reduction; weights staged in LDS.
#include "common.h"

namespace {

constexpr int BM = 128;  // output pixels per workgroup
constexpr int BN = 64;   // output channels per workgroup
constexpr int BK = 16;   // input channels per K-stage
constexpr int LDA = BK + 4;

enum Variant { V_MFMA = 0, V_SMALLCIN = 1, V_THIN = 2, V_NONE = -1 };

struct Geometry {
  int variant;
  int oh, ow, tr, hr, hc, taps, cp0, cp1, ktot, npad;
  size_t lds;
};

int round_up(int a, int b) { return (a + b - 1) / b * b; }

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
    g.npad = round_up(cout, 16);
    return g;
  }
  if (cout <= 4) {
    if (cin % 4 || cin > 1024 || (long long)cout * g.taps * cin * 4 > 64 * 1024) return g;
    g.variant = V_THIN;
    g.ktot = g.taps * cin;
    g.npad = cout;
    return g;
  }
  if (c0 % 4 || c1 % 4) return g;
  if (w != g.ow || (BM % g.ow) != 0 || (g.ow % 32) != 0) return g;  // tile = whole image rows
  g.tr = BM / g.ow;
  if (g.oh % g.tr) return g;
  g.hr = g.tr + kh - 1;
  g.hc = g.ow + kw - 1;
  g.cp0 = round_up(c0, BK);
  g.cp1 = round_up(c1, BK);
  g.ktot = g.taps * (g.cp0 + g.cp1);
  g.npad = round_up(cout, BN);
  g.lds = sizeof(float) * ((size_t)g.hr * g.hc * LDA + (size_t)g.taps * BN * LDA);
  if (g.lds > 160 * 1024) return g;
  g.variant = V_MFMA;
  return g;
}

// ------------------------------------------------------------------------------------------
// MFMA implicit-GEMM conv
// ------------------------------------------------------------------------------------------
struct MfmaParams {
  scflow_conv_args a;
  int oh, ow, tr, hr, hc, taps, cp0, cp1, ktot;
};

template <int EPI>
__global__ __launch_bounds__(256, 2) void conv_mfma_kernel(MfmaParams P) {
  extern __shared__ float smem[];
  const scflow_conv_args& a = P.a;
  float* As = smem;                                  // [hr*hc][LDA]
  float* Bs = smem + (size_t)P.hr * P.hc * LDA;      // [taps][BN][LDA]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1, li = lane & 31, hh = lane >> 5;
  const int tiles_per_img = P.oh / P.tr;
  const int img = blockIdx.x / tiles_per_img;
  const int oy0 = (blockIdx.x % tiles_per_img) * P.tr;
  const int n0 = blockIdx.y * BN;
  const int ow = P.ow, hc = P.hc;

  // this lane's two A rows (output pixels) as (row, col) inside the tile
  int pr[2], pc[2];
#pragma unroll
  for (int rb = 0; rb < 2; ++rb) {
    const int m = wm * 64 + rb * 32 + li;
    pr[rb] = m / ow;
    pc[rb] = m % ow;
  }

  floatx16 acc[2];
#pragma unroll
  for (int rb = 0; rb < 2; ++rb)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[rb][r] = 0.f;

  const int nsrc = a.c1 > 0 ? 2 : 1;
  for (int s = 0; s < nsrc; ++s) {
    const float* src = s ? a.src1 : a.src0;
    const int cs = s ? a.c1 : a.c0;
    const int ss = s ? a.s1 : a.s0;
    const int koff = s ? P.cp0 : 0;
    for (int cc = 0; cc < cs; cc += BK) {
      __syncthreads();
      // input halo: (hr × hc) pixels × BK channels
      const int na = P.hr * hc * (BK / 4);
      for (int idx = tid; idx < na; idx += 256) {
        const int q = idx & 3, pix = idx >> 2;
        const int hr = pix / hc, hcol = pix - hr * hc;
        const int iy = oy0 - a.ph + hr, ix = hcol - a.pw;
        const int c = cc + 4 * q;
        floatx4 v = {0.f, 0.f, 0.f, 0.f};
        if (iy >= 0 && iy < a.h && ix >= 0 && ix < a.w && c < cs)
          v = *(const floatx4*)(src + ((size_t)(img * a.h + iy) * a.w + ix) * ss + c);
        *(floatx4*)(As + pix * LDA + 4 * q) = v;
      }
      // weights of every tap for this K-stage
      const int nb = P.taps * BN * (BK / 4);
      const int cpt = P.cp0 + P.cp1;
      for (int idx = tid; idx < nb; idx += 256) {
        const int q = idx & 3, row = idx >> 2;
        const int tap = row / BN, col = row - tap * BN;
        *(floatx4*)(Bs + row * LDA + 4 * q) =
            *(const floatx4*)(a.weight + (size_t)(n0 + col) * P.ktot + tap * cpt + koff + cc + 4 * q);
      }
      __syncthreads();
      for (int tap = 0; tap < P.taps; ++tap) {
        const int ty = tap / a.kw, tx = tap - ty * a.kw;
        const float* Ab0 = As + ((pr[0] + ty) * hc + pc[0] + tx) * LDA + 4 * hh;
        const float* Ab1 = As + ((pr[1] + ty) * hc + pc[1] + tx) * LDA + 4 * hh;
        const float* Bb = Bs + (tap * BN + wn * 32 + li) * LDA + 4 * hh;
#pragma unroll
        for (int kb = 0; kb < BK; kb += 8) {
          const floatx4 a0 = *(const floatx4*)(Ab0 + kb);
          const floatx4 a1 = *(const floatx4*)(Ab1 + kb);
          const floatx4 b0 = *(const floatx4*)(Bb + kb);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[e], b0[e], acc[0], 0, 0, 0);
            acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[e], b0[e], acc[1], 0, 0, 0);
          }
        }
      }
    }
  }

  // epilogue; C/D layout: col = lane&31, row = (r&3) + 8(r>>2) + 4(lane>>5)
  const int col = n0 + wn * 32 + li;
  if (col >= a.cout) return;
  const float bias = a.bias ? a.bias[col] : 0.f;
#pragma unroll
  for (int rb = 0; rb < 2; ++rb) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = wm * 64 + rb * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
      const int oy = oy0 + m / ow, ox = m % ow;
      const size_t pix = ((size_t)img * P.oh + oy) * ow + ox;
      const float v = acc[rb][r] + bias;
      if constexpr (EPI == SCFLOW_EPI_PLAIN) {
        a.out[pix * a.so + col] = act_apply(v, a.act);
      } else if constexpr (EPI == SCFLOW_EPI_GRU_ZR) {
        const int hcn = a.cout >> 1;
        const float g = sigmoidf_(v);
        if (col < hcn) {
          a.gate[pix * a.sg + col] = g;
        } else {
          const int c = col - hcn;
          a.rh[pix * a.srh + c] = g * a.hid[pix * a.sh + c];
        }
      } else {  // GRU_Q
        const float q = tanhf(v);
        const float z = a.gate[pix * a.sg + col];
        const float h = a.hid[pix * a.sh + col];
        a.hid[pix * a.sh + col] = (1.f - z) * h + z * q;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// small-cin direct conv (VALU): thread = output pixel, 16 output channels per thread
// weights packed [npad][kh][kw][cin]
// ------------------------------------------------------------------------------------------
template <int CIN>
__global__ __launch_bounds__(256) void conv_smallcin_kernel(scflow_conv_args a, int oh, int ow) {
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
  const int taps = a.kh * a.kw;
  const float* wb = a.weight + (size_t)co0 * taps * CIN;
  for (int ty = 0; ty < a.kh; ++ty) {
    const int iy = oy - a.ph + ty;
    for (int tx = 0; tx < a.kw; ++tx) {
      const int ix = ox - a.pw + tx;
      float v[CIN];
      const bool ok = iy >= 0 && iy < a.h && ix >= 0 && ix < a.w;
      const float* sp = a.src0 + ((size_t)(img * a.h + iy) * a.w + ix) * a.s0;
#pragma unroll
      for (int c = 0; c < CIN; ++c) v[c] = ok ? sp[c] : 0.f;
      const float* wt = wb + (ty * a.kw + tx) * CIN;
#pragma unroll
      for (int j = 0; j < 16; ++j)
#pragma unroll
        for (int c = 0; c < CIN; ++c) acc[j] += wt[(size_t)j * taps * CIN + c] * v[c];
    }
  }
  float* op = a.out + (size_t)pix * a.so + co0;
#pragma unroll
  for (int j = 0; j < 16; ++j)
    if (co0 + j < a.cout) op[j] = act_apply(acc[j], a.act);
}

// ------------------------------------------------------------------------------------------
// thin conv (cout ≤ 4): one wave per output pixel, lanes split the input channels
// weights packed [cout][kh][kw][cin]
// ------------------------------------------------------------------------------------------
template <int COUT>
__global__ __launch_bounds__(256) void conv_thin_kernel(scflow_conv_args a, int oh, int ow,
                                                        int px_per_wave) {
  extern __shared__ float wsh[];
  const int cin = a.c0 + a.c1;
  const int taps = a.kh * a.kw;
  const int nw = COUT * taps * cin;
  for (int i = threadIdx.x * 4; i < nw; i += 256 * 4) *(floatx4*)(wsh + i) = *(const floatx4*)(a.weight + i);
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long long M = (long long)a.n * oh * ow;
  const long long pbase = ((long long)blockIdx.x * 4 + wave) * px_per_wave;
  for (int pp = 0; pp < px_per_wave; ++pp) {
    const long long pix = pbase + pp;
    if (pix >= M) break;
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
        const size_t ipix = (size_t)(img * a.h + iy) * a.w + ix;
        const int tap = ty * a.kw + tx;
        for (int c = lane * 4; c < cin; c += 256) {
          const floatx4 v = c < a.c0 ? *(const floatx4*)(a.src0 + ipix * a.s0 + c)
                                     : *(const floatx4*)(a.src1 + ipix * a.s1 + (c - a.c0));
#pragma unroll
          for (int o = 0; o < COUT; ++o) {
            const floatx4 wv = *(const floatx4*)(wsh + ((size_t)o * taps + tap) * cin + c);
            acc[o] += v[0] * wv[0] + v[1] * wv[1] + v[2] * wv[2] + v[3] * wv[3];
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
}

// packing: w_oihw [cout][cin][kh][kw] → variant layout
__global__ void pack_kernel(const float* __restrict__ w, float* __restrict__ out, int variant,
                            int cout, int c0, int c1, int kh, int kw, int cp0, int cp1, int ktot,
                            int npad) {
  const long long total = (long long)npad * ktot;
  const int cin = c0 + c1, taps = kh * kw;
  for (long long idx = blockIdx.x * 256LL + threadIdx.x; idx < total; idx += (long long)gridDim.x * 256) {
    const int o = (int)(idx / ktot);
    const int k = (int)(idx % ktot);
    float v = 0.f;
    if (variant == V_MFMA) {
      const int cpt = cp0 + cp1;
      const int tap = k / cpt, cc = k % cpt;
      int ci = -1;
      if (cc < cp0) {
        if (cc < c0) ci = cc;
      } else if (cc - cp0 < c1) {
        ci = c0 + (cc - cp0);
      }
      if (o < cout && ci >= 0) v = w[((size_t)o * cin + ci) * taps + tap];
    } else {  // [o][tap][ci]
      const int tap = k / cin, ci = k % cin;
      if (o < cout) v = w[((size_t)o * cin + ci) * taps + tap];
    }
    out[idx] = v;
  }
}

bool lds_attr_done[3] = {false, false, false};

template <int EPI>
int launch_mfma(const MfmaParams& p, const Geometry& g, hipStream_t st) {
  if (g.lds > 64 * 1024 && !lds_attr_done[EPI]) {
    hipFuncSetAttribute((const void*)conv_mfma_kernel<EPI>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    lds_attr_done[EPI] = true;
  }
  dim3 grid(p.a.n * (g.oh / g.tr), g.npad / BN);
  conv_mfma_kernel<EPI><<<grid, 256, g.lds, st>>>(p);
  return scflow_launch_status();
}

}  // namespace

SCFLOW_API long long scflow_conv_packed_size(int cout, int c0, int c1, int kh, int kw, int stride,
                                             int w) {
  // packing does not depend on padding or height; use a 'same' geometry for the selection
  Geometry g = select_variant(cout, c0, c1, kh, kw, stride, 4 * 128, w, (kh - 1) / 2, (kw - 1) / 2);
  if (g.variant == V_NONE) return SCFLOW_EUNSUPPORTED;
  return (long long)g.npad * g.ktot;
}

SCFLOW_API int scflow_conv_pack_weights(const float* w_oihw, float* packed, int cout, int c0,
                                        int c1, int kh, int kw, int stride, int w, void* stream) {
  if (!w_oihw || !packed || cout <= 0 || c0 <= 0 || c1 < 0 || kh <= 0 || kw <= 0) return SCFLOW_EINVAL;
  Geometry g = select_variant(cout, c0, c1, kh, kw, stride, 4 * 128, w, (kh - 1) / 2, (kw - 1) / 2);
  if (g.variant == V_NONE) return SCFLOW_EUNSUPPORTED;
  const long long total = (long long)g.npad * g.ktot;
  const int blocks = (int)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
  pack_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(w_oihw, packed, g.variant, cout, c0, c1, kh,
                                                       kw, g.cp0, g.cp1, g.ktot, g.npad);
  return scflow_launch_status();
}

SCFLOW_API int scflow_conv2d(const scflow_conv_args* args, void* stream) {
  if (!args) return SCFLOW_EINVAL;
  const scflow_conv_args& a = *args;
  if (!a.src0 || !a.weight || a.n <= 0 || a.h <= 0 || a.w <= 0 || a.cout <= 0 || a.c0 <= 0 ||
      a.c1 < 0 || (a.c1 > 0 && !a.src1) || a.kh <= 0 || a.kw <= 0 || a.ph < 0 || a.pw < 0)
    return SCFLOW_EINVAL;
  if (a.epilogue == SCFLOW_EPI_PLAIN) {
    if (!a.out) return SCFLOW_EINVAL;
  } else if (a.epilogue == SCFLOW_EPI_GRU_ZR) {
    if (!a.gate || !a.rh || !a.hid || (a.cout & 1)) return SCFLOW_EINVAL;
  } else if (a.epilogue == SCFLOW_EPI_GRU_Q) {
    if (!a.gate || !a.hid) return SCFLOW_EINVAL;
  } else {
    return SCFLOW_EINVAL;
  }
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
    p.taps = g.taps;
    p.cp0 = g.cp0;
    p.cp1 = g.cp1;
    p.ktot = g.ktot;
    switch (a.epilogue) {
      case SCFLOW_EPI_GRU_ZR: return launch_mfma<SCFLOW_EPI_GRU_ZR>(p, g, st);
      case SCFLOW_EPI_GRU_Q: return launch_mfma<SCFLOW_EPI_GRU_Q>(p, g, st);
      default: return launch_mfma<SCFLOW_EPI_PLAIN>(p, g, st);
    }
  }
  if (a.epilogue != SCFLOW_EPI_PLAIN) return SCFLOW_EUNSUPPORTED;
  const long long M = (long long)a.n * g.oh * g.ow;
  if (g.variant == V_SMALLCIN) {
    dim3 grid((unsigned)((M + 255) / 256), g.npad / 16);
    switch (a.c0) {
      case 1: conv_smallcin_kernel<1><<<grid, 256, 0, st>>>(a, g.oh, g.ow); break;
      case 2: conv_smallcin_kernel<2><<<grid, 256, 0, st>>>(a, g.oh, g.ow); break;
      case 3: conv_smallcin_kernel<3><<<grid, 256, 0, st>>>(a, g.oh, g.ow); break;
      case 4: conv_smallcin_kernel<4><<<grid, 256, 0, st>>>(a, g.oh, g.ow); break;
      default: return SCFLOW_EUNSUPPORTED;
    }
    return scflow_launch_status();
  }
  // thin
  if (!aligned16(a.src0) || (a.s0 & 3) || (a.c1 > 0 && (!aligned16(a.src1) || (a.s1 & 3))) ||
      !aligned16(a.weight) || (a.c0 & 3))
    return SCFLOW_EALIGN;
  const int ppw = 16;
  const int blocks = (int)((M + 4 * ppw - 1) / (4 * ppw));
  const size_t lds = sizeof(float) * (size_t)a.cout * g.taps * (a.c0 + a.c1);
  switch (a.cout) {
    case 1: conv_thin_kernel<1><<<blocks, 256, lds, st>>>(a, g.oh, g.ow, ppw); break;
    case 2: conv_thin_kernel<2><<<blocks, 256, lds, st>>>(a, g.oh, g.ow, ppw); break;
    case 3: conv_thin_kernel<3><<<blocks, 256, lds, st>>>(a, g.oh, g.ow, ppw); break;
    case 4: conv_thin_kernel<4><<<blocks, 256, lds, st>>>(a, g.oh, g.ow, ppw); break;
    default: return SCFLOW_EUNSUPPORTED;
  }
  return scflow_launch_status();
}
