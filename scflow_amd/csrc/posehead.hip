// a7 — MultiClassPoseHead (/root/reference/models/head/pose_head.py:110-211) on gfx950.
//
//   3 × [3×3 stride-2 conv (no bias) → GroupNorm(32) → ReLU] → flatten (NCHW order)
//   → FC 2048→1024 + ReLU → FC 1024→256 + ReLU → rotation / translation heads
//   → index_select(label)[:, 0]  (every sample uses label[0]'s class head — reference quirk)
//
// Stock PyTorch runs this as ~15 small launches per refinement iteration (MIOpen conv +
// layout transposes, GroupNorm's moments / fused-params / apply kernels, ReLU clamps, copies,
// hipBLASLt GEMMs, index_select).  Here: 9 launches, no torch ops, no concatenation:
//
//  * scflow_ph_conv — gather-A implicit GEMM on v_mfma_f32_32x32x2_f32 for the strided convs.
//    Workgroup tile = 32 output pixels × 32 output channels; the 4 waves split K (16-deep
//    chunks, round robin) and reduce their 32×32 partials through LDS.  A (im2col rows) is
//    gathered straight from L2 per lane, two input sources concatenated on channels
//    (cat[h, Δflow-feat, mask-feat] never materialises), and the PREVIOUS layer's GroupNorm +
//    ReLU is applied on load (per-(sample, channel) scale/shift) — so GN never rewrites memory.
//    conv1 at B=16: 512 workgroups.
//  * scflow_ph_gn_stats / scflow_ph_gn_reduce — group mean/var (fp64 accumulation) over a
//    (sample, 32-channel) grid → scale = γ·rstd, shift = β − mean·γ·rstd per channel; the reduce
//    form first sums conv1's K-split partial slabs (scflow_enc_conv with ksplit) and writes the
//    sum.
//  * scflow_ph_fc — weight-streaming FC for M ≤ 16 rows: a wave per output neuron pair,
//    lanes split K, inputs staged once per workgroup in LDS; optional GN+ReLU+NCHW-flatten
//    gather of the input (FC1 reads conv3's raw output).
//  * scflow_ph_heads — the label[0] class's 6 rotation and 3 translation rows only.
#include "common.h"
#include "pose_dev.h"  // pose_heads: the heads' arithmetic shared with scflow_pose_step_heads

#include <stdlib.h>

#include <algorithm>

namespace {

constexpr int PH_K = 16;  // K chunk per MFMA group
struct PhConvArgs {
  const float* src0; int c0; int s0;
  const float* src1; int c1; int s1;
  const float* scale;   // [n][c0+c1] GN scale of the input (NULL: raw input)
  const float* shift;   // [n][c0+c1]
  const float* weight;  // packed [cout][taps][cinp], cinp = roundup(c0+c1, 16)
  const float* bias;    // [cout] or NULL
  float* out;           // [n][oh][ow][cout], or [ksplit][n][oh][ow][cout] partial slabs
  int n, h, w, oh, ow, cout, kh, kw, stride, pad, cinp;
  int ksplit;           // K chunks split over grid.z (partial slab z = out + z·M·cout)
};

// input element quad (channels c..c+3 of pixel (iy, ix) of image img), the input GroupNorm +
// ReLU applied from the affine table sc/sh (row (img − img_base), ld floats per row; NULL: raw)
__device__ __forceinline__ floatx4 ph_load_a(const PhConvArgs& a, int img, int iy, int ix, int c,
                                             const float* sc_t, const float* sh_t, int img_base,
                                             int ld) {
  floatx4 v = {0.f, 0.f, 0.f, 0.f};
  if (iy < 0 || iy >= a.h || ix < 0 || ix >= a.w) return v;
  const size_t pix = (size_t)(img * a.h + iy) * a.w + ix;
  const int cin = a.c0 + a.c1;
  if (c >= cin) return v;
  v = c < a.c0 ? *(const floatx4*)(a.src0 + pix * a.s0 + c)
               : *(const floatx4*)(a.src1 + pix * a.s1 + (c - a.c0));
  if (sc_t) {
    const floatx4 sc = *(const floatx4*)(sc_t + (size_t)(img - img_base) * ld + c);
    const floatx4 sh = *(const floatx4*)(sh_t + (size_t)(img - img_base) * ld + c);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e] * sc[e] + sh[e], 0.f);
  }
  return v;
}

#ifndef SCFLOW_PH_WAVES
#define SCFLOW_PH_WAVES 16
#endif
#ifndef SCFLOW_PH_BATCH
#define SCFLOW_PH_BATCH 2  // tuned (tools/ph_bench.py): 4 → 2 is 2–3 µs faster per launch
#endif
constexpr int PH_WAVES = SCFLOW_PH_WAVES;  // waves per workgroup; they split K
constexpr int PH_BATCH = SCFLOW_PH_BATCH;  // K chunks whose loads a wave issues together

// one 32×32 output tile (bx, by) of K slice bz; NW waves (threads ≥ NW·64 must not call);
// red: (NW/2)·32·33 floats of LDS
template <int NW>
__device__ __forceinline__ void ph_conv_body(const PhConvArgs& a, int bx, int by, int bz,
                                             float* red, const float* sc_t, const float* sh_t,
                                             int img_base, int ld) {
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int li = lane & 31, hh = lane >> 5;
  const int M = a.n * a.oh * a.ow;
  const int m0 = bx * 32, n0 = by * 32;
  // this lane's A row (output pixel) and B column (output channel)
  const int m = m0 + li;
  const bool mvalid = m < M;
  const int ox = mvalid ? m % a.ow : 0;
  const int oy = mvalid ? (m / a.ow) % a.oh : 0;
  const int img = mvalid ? m / (a.ow * a.oh) : 0;
  const int col = n0 + li;
  const bool nvalid = col < a.cout;
  const int taps = a.kh * a.kw;
  const int cchunks = a.cinp / PH_K;
  const int nall = taps * cchunks;
  // this workgroup's K range (grid.z splits the chunks; partial slab z)
  const int klo = (int)((long long)nall * bz / a.ksplit);
  const int nchunks = (int)((long long)nall * (bz + 1) / a.ksplit);
  floatx16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  for (int base = klo + wave; base < nchunks; base += NW * PH_BATCH) {
    floatx4 A0[PH_BATCH], A1[PH_BATCH], B0[PH_BATCH], B1[PH_BATCH];
#pragma unroll
    for (int c = 0; c < PH_BATCH; ++c) {  // issue every load of the batch first
      const floatx4 z = {0.f, 0.f, 0.f, 0.f};
      A0[c] = A1[c] = B0[c] = B1[c] = z;
      const int kc = base + c * NW;
      if (kc < nchunks) {
        const int tap = kc / cchunks, c0 = (kc % cchunks) * PH_K;
        const int ty = tap / a.kw, tx = tap % a.kw;
        const int iy = oy * a.stride - a.pad + ty, ix = ox * a.stride - a.pad + tx;
        if (mvalid) {
          A0[c] = ph_load_a(a, img, iy, ix, c0 + 4 * hh, sc_t, sh_t, img_base, ld);
          A1[c] = ph_load_a(a, img, iy, ix, c0 + 8 + 4 * hh, sc_t, sh_t, img_base, ld);
        }
        if (nvalid) {
          const float* wp = a.weight + ((size_t)col * taps + tap) * a.cinp + c0 + 4 * hh;
          B0[c] = *(const floatx4*)wp;
          B1[c] = *(const floatx4*)(wp + 8);
        }
      }
    }
#pragma unroll
    for (int c = 0; c < PH_BATCH; ++c) {
#pragma unroll
      for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(A0[c][e], B0[c][e], acc, 0, 0, 0);
#pragma unroll
      for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(A1[c][e], B1[c][e], acc, 0, 0, 0);
    }
  }
  // deterministic tree reduction of the waves' partial tiles behind ONE barrier: every wave parks
  // its 16 accumulator values ([wave][value][lane]), then wave w folds value w of all NW waves in
  // the level-by-level tree's order — (v, v + NW/2), then (v, v + NW/4), … — and stores it (the
  // same sums as 2·log2(NW) barriers of halving, with the fold spread over the waves)
#pragma unroll
  for (int r = 0; r < 16; ++r) red[(wave * 16 + r) * 64 + lane] = acc[r];
  __syncthreads();
  for (int r = wave; r < 16; r += NW) {
    float t[NW];
#pragma unroll
    for (int v = 0; v < NW; ++v) t[v] = red[(v * 16 + r) * 64 + lane];
#pragma unroll
    for (int half = NW / 2; half >= 1; half >>= 1)
#pragma unroll
      for (int v = 0; v < half; ++v) t[v] = t[v] + t[v + half];
    const int mm = m0 + (r & 3) + 8 * (r >> 2) + 4 * hh;
    if (nvalid && mm < M)
      a.out[(size_t)bz * M * a.cout + (size_t)mm * a.cout + col] = t[0] + (a.bias ? a.bias[col] : 0.f);
  }
}

__global__ __launch_bounds__(PH_WAVES * 64) void ph_conv_kernel(PhConvArgs a) {
  __shared__ float red[PH_WAVES * 16 * 64];  // 64 KiB: every wave's 16 values per lane
  ph_conv_body<PH_WAVES>(a, blockIdx.x, blockIdx.y, blockIdx.z, red, a.scale, a.shift, 0,
                         a.c0 + a.c1);
}

// GroupNorm statistics of x [n][hw][c] → per-channel scale/shift for y = relu(x·scale + shift),
// optionally first summing nsplit K-split partial slabs (x + z·split_stride) and writing the sum
// to y.  Grid (n, c/CB): a workgroup takes one sample's CB-channel block; thread t holds channel
// quad t%(CB/4) of pixel slot t/(CB/4) (256·4/CB slots), float4 loads; per-channel sums in fp64
// reduced over the slots in a fixed order (CB = 16: first 16 parts of 4 slots each, all threads),
// then per group (c/groups channels) → mean, biased variance.
// NS > 0: compile-time slab count; the pixel loop is unrolled PU-fold with every load of a
// round issued before any add (this kernel is latency-bound: 64 workgroups at B = 16 with CB =
// 32, 128 with CB = 16; at the pose head's first conv every slot's pixels × 4 slabs are one round)
template <int NS, int CB>
__global__ __launch_bounds__(256) void ph_gn_reduce_kernel(const float* __restrict__ x, int nsplit,
                                                           long long split_stride, float* __restrict__ y,
                                                           int hw, int c, int groups,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta, float eps,
                                                           float* __restrict__ scale,
                                                           float* __restrict__ shift) {
  constexpr int NQ = CB / 4, SL = 256 / NQ;  // channel quads, pixel slots
  __shared__ double s1[SL][CB + 1], s2[SL][CB + 1];
  __shared__ double gmean[CB], grstd[CB];
  const int img = blockIdx.x, cb = blockIdx.y * CB;
  const int q = threadIdx.x % NQ, slot = threadIdx.x / NQ;
  double a[4] = {0, 0, 0, 0}, b[4] = {0, 0, 0, 0};
  auto acc = [&](floatx4 v, size_t off) {
    if (y) *(floatx4*)(y + off) = v;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      a[e] += (double)v[e];
      b[e] += (double)v[e] * (double)v[e];
    }
  };
  int p = slot;
  if constexpr (NS > 0) {
    constexpr int PU = NS <= 4 ? 8 * 32 / SL : 1;  // ≤ 32 float4 loads in flight
    for (; p + SL * (PU - 1) < hw; p += SL * PU) {
      floatx4 v[PU][NS];
#pragma unroll
      for (int u = 0; u < PU; ++u)
#pragma unroll
        for (int z = 0; z < NS; ++z)
          v[u][z] = *(const floatx4*)(x + (size_t)z * split_stride + ((size_t)img * hw + p + SL * u) * c +
                                      cb + 4 * q);
#pragma unroll
      for (int u = 0; u < PU; ++u) {
#pragma unroll
        for (int z = 1; z < NS; ++z) v[u][0] += v[u][z];
        acc(v[u][0], ((size_t)img * hw + p + SL * u) * c + cb + 4 * q);
      }
    }
  }
  for (; p < hw; p += SL) {
    const size_t off = ((size_t)img * hw + p) * c + cb + 4 * q;
    floatx4 v = *(const floatx4*)(x + off);
    if constexpr (NS > 0) {
      floatx4 u[NS > 1 ? NS : 1];
#pragma unroll
      for (int z = 1; z < NS; ++z) u[z] = *(const floatx4*)(x + (size_t)z * split_stride + off);
#pragma unroll
      for (int z = 1; z < NS; ++z) v += u[z];
    } else {
      for (int z = 1; z < nsplit; ++z) {
        const floatx4 u = *(const floatx4*)(x + (size_t)z * split_stride + off);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += u[e];
      }
    }
    acc(v, off);
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    s1[slot][4 * q + e] = a[e];
    s2[slot][4 * q + e] = b[e];
  }
  __syncthreads();
  const int cpg = c / groups;       // channels per group (divides CB)
  const int ng = CB / cpg;          // groups in this block
  int nsl = SL;                     // slot rows left to fold
  if constexpr (CB == 16) {
    // 16 parts × 16 channels: thread t folds slots 4·(t/16) .. +3 of channel t%16 into row t/16
    const int ch = threadIdx.x % CB, part = threadIdx.x / CB;
    double A = 0, B = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      A += s1[4 * part + k][ch];
      B += s2[4 * part + k][ch];
    }
    __syncthreads();
    s1[part][ch] = A;
    s2[part][ch] = B;
    __syncthreads();
    nsl = 16;
  }
  if (threadIdx.x < ng) {
    double A = 0, B = 0;
    for (int k = 0; k < cpg; ++k)
      for (int sl = 0; sl < nsl; ++sl) {
        A += s1[sl][threadIdx.x * cpg + k];
        B += s2[sl][threadIdx.x * cpg + k];
      }
    const double cnt = (double)hw * cpg;
    const double mean = A / cnt;
    double var = B / cnt - mean * mean;
    if (var < 0) var = 0;
    gmean[threadIdx.x] = mean;
    grstd[threadIdx.x] = 1.0 / sqrt(var + (double)eps);
  }
  __syncthreads();
  if (threadIdx.x < CB) {
    const int ch = cb + threadIdx.x, g = threadIdx.x / cpg;
    const float sc = gamma[ch] * (float)grstd[g];
    scale[(size_t)img * c + ch] = sc;
    shift[(size_t)img * c + ch] = beta[ch] - (float)gmean[g] * sc;
  }
}

// FC on v_mfma_f32_16x16x4_f32: D[neuron i][row j] = Σ_k W[i][k]·X[j][k] for a 16-neuron
// tile (grid.x) and up to FC_RT·16 batch rows; PH_WAVES waves split K in 16-wide groups and
// issue all their loads before the MFMAs, then reduce through LDS (fixed order).
// Lane l: A = W[i0 + (l&15)][k..k+3], B = X[l&15][k..k+3] with k = 16g + 4(l>>4) — MFMA e
// consumes element e of both (a permutation of K, identical on both operands).
// Modes: plain X [m][ldx]; GN (gn_c > 0): X = relu(Y·scale + shift), Y [m][k] channels-last
// with channel = k % gn_c (W's columns must be in that order: scflow_ph_fc_permute);
// heads (label != NULL): neuron i < rch → Wr row label[0]·rch + i, i < rch+3 → Wt row
// label[0]·3 + i − rch; outputs drot [m][rch], dt [m][3].

struct FcArgs {
  const float* x; int ldx; int m; int k;
  const float* W; const float* bias; float* y; int n; int relu;
  int gn_c; const float* scale; const float* shift;
  const float* Wt; const float* bt; const long long* label; int num_class; int rch; float* dt;
  int ksplit;                            // >1: grid.y splits K, y + z·m·n gets partial sums
  int xsplit; long long xstride;         // >0: X = relu(Σ_z x[z·xstride] + xbias) (split producer)
  const float* xbias;
};

// one 16-neuron tile bx of K slice by; NW waves; red: (NW/2)·FC_RT·64·5 floats of LDS
template <int NW, int FC_RT>  // row tiles of 16 per pass
__device__ __forceinline__ void ph_fc_body(const FcArgs& f, int bx, int by, float* red,
                                           const float* sc_t, const float* sh_t) {
  constexpr int FB = FC_RT == 1 ? PH_BATCH : 2;  // K groups whose loads are issued together
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int li = lane & 15, kq = lane >> 4;
  const int i0 = bx * 16;
  // weight row of this lane's neuron
  const int ni = i0 + li;
  const float* wrow = nullptr;
  if (f.label) {
    long long cls = f.label[0];
    if (cls < 0 || cls >= f.num_class) cls = 0;
    if (ni < f.rch) wrow = f.W + ((size_t)cls * f.rch + ni) * f.k;
    else if (ni < f.rch + 3) wrow = f.Wt + ((size_t)cls * 3 + (ni - f.rch)) * f.k;
  } else if (ni < f.n) {
    wrow = f.W + (size_t)ni * f.k;
  }
  const int gall = f.k / 16;
  const int glo = f.ksplit > 1 ? (int)((long long)gall * by / f.ksplit) : 0;
  const int groups = f.ksplit > 1 ? (int)((long long)gall * (by + 1) / f.ksplit) : gall;
  float* yout = f.y + (f.ksplit > 1 ? (size_t)by * f.m * f.n : 0);
  for (int r0 = 0; r0 < f.m; r0 += 16 * FC_RT) {
    floatx4 acc[FC_RT];
#pragma unroll
    for (int t = 0; t < FC_RT; ++t) acc[t] = {0.f, 0.f, 0.f, 0.f};
    for (int base = glo + wave; base < groups; base += NW * FB) {
      floatx4 wv[FB], xv[FB][FC_RT];
#pragma unroll
      for (int c = 0; c < FB; ++c) {
        const int g = base + c * NW;
        const int kk = g * 16 + 4 * kq;
        const floatx4 z = {0.f, 0.f, 0.f, 0.f};
        wv[c] = (g < groups && wrow) ? *(const floatx4*)(wrow + kk) : z;
#pragma unroll
        for (int t = 0; t < FC_RT; ++t) {
          const int row = r0 + t * 16 + li;
          floatx4 v = z;
          if (g < groups && row < f.m) {
            v = *(const floatx4*)(f.x + (size_t)row * f.ldx + kk);
            if (f.xsplit > 0) {
              for (int z = 1; z < f.xsplit; ++z) v += *(const floatx4*)(f.x + z * f.xstride + (size_t)row * f.ldx + kk);
              const floatx4 xb = *(const floatx4*)(f.xbias + kk);
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e] + xb[e], 0.f);
            }
            if (f.gn_c > 0) {
              const int ch = kk % f.gn_c;
              const floatx4 sc = *(const floatx4*)(sc_t + (size_t)row * f.gn_c + ch);
              const floatx4 sh = *(const floatx4*)(sh_t + (size_t)row * f.gn_c + ch);
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e] * sc[e] + sh[e], 0.f);
            }
          }
          xv[c][t] = v;
        }
      }
#pragma unroll
      for (int c = 0; c < FB; ++c)
#pragma unroll
        for (int t = 0; t < FC_RT; ++t)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv[c][e], xv[c][t][e], acc[t], 0, 0, 0);
    }
    // the waves' partials folded behind ONE barrier (as ph_conv_body): every wave parks its
    // FC_RT·4 values, wave i folds value i of all NW waves in the halving tree's order and
    // stores it
    constexpr int NV = FC_RT * 4;
#pragma unroll
    for (int t = 0; t < FC_RT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[(wave * NV + 4 * t + r) * 64 + lane] = acc[t][r];
    __syncthreads();
    for (int iv = wave; iv < NV; iv += NW) {
      float u[NW];
#pragma unroll
      for (int v = 0; v < NW; ++v) u[v] = red[(v * NV + iv) * 64 + lane];
#pragma unroll
      for (int half = NW / 2; half >= 1; half >>= 1)
#pragma unroll
        for (int v = 0; v < half; ++v) u[v] = u[v] + u[v + half];
      // C/D layout (16x16): col = lane&15 (batch row), row = 4(lane>>4) + r (neuron)
      const int t = iv >> 2, r = iv & 3;
      const int row = r0 + t * 16 + li;
      const int i = i0 + 4 * kq + r;
      float v = u[0];
      if (row < f.m) {
        if (f.label) {
          long long cls = f.label[0];
          if (cls < 0 || cls >= f.num_class) cls = 0;
          if (i < f.rch)
            f.y[(size_t)row * f.rch + i] = v + f.bias[cls * f.rch + i];
          else if (i < f.rch + 3)
            f.dt[(size_t)row * 3 + (i - f.rch)] = v + f.bt[cls * 3 + (i - f.rch)];
        } else if (i < f.n) {
          if (f.ksplit <= 1) {
            v += f.bias ? f.bias[i] : 0.f;
            if (f.relu) v = fmaxf(v, 0.f);
          }
          yout[(size_t)row * f.n + i] = v;
        }
      }
    }
    if (r0 + 16 * FC_RT < f.m) __syncthreads();  // the next row block re-parks
  }
}

// the label[0] class's rotation / translation heads of sample row blockIdx.x (scflow_ph_heads*)
__global__ __launch_bounds__(256) void ph_heads_kernel(PoseStepArgs a) {
  __shared__ float hs[16 + 16 * 4];
  const int n = blockIdx.x, tid = threadIdx.x;
  pose_heads(a, hs, n, tid, 256);
  if (tid < a.hrch)
    a.drot_out[(size_t)n * a.hrch + tid] = hs[tid];
  else if (tid < a.hrch + 3)
    a.dt_out[(size_t)n * 3 + tid - a.hrch] = hs[tid];
}

template <int FC_RT>
__global__ __launch_bounds__(PH_WAVES * 64) void ph_fc_kernel(FcArgs f) {
  __shared__ float red[PH_WAVES * FC_RT * 4 * 64];
  ph_fc_body<PH_WAVES, FC_RT>(f, blockIdx.x, blockIdx.y, red, f.scale, f.shift);
}

// W [n][c·hw] with columns in NCHW-flatten order (c·hw + p) → Wp [n][hw·c] channels-last order
__global__ void ph_fc_permute_kernel(const float* __restrict__ W, float* __restrict__ Wp, int n,
                                     int c, int hw) {
  const long long total = (long long)n * c * hw;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int kk = (int)(i % ((long long)c * hw));
    const long long row = i / ((long long)c * hw);
    const int p = kk / c, ch = kk % c;
    Wp[i] = W[row * c * hw + (size_t)ch * hw + p];
  }
}

__global__ void ph_pack_kernel(const float* __restrict__ w, float* __restrict__ out, int cout,
                               int cin, int taps, int cinp) {
  const long long total = (long long)cout * taps * cinp;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int c = (int)(i % cinp);
    const int tap = (int)((i / cinp) % taps);
    const int o = (int)(i / ((long long)cinp * taps));
    out[i] = c < cin ? w[((size_t)o * cin + c) * taps + tap] : 0.f;
  }
}


}  // namespace

SCFLOW_API long long scflow_ph_conv_packed_size(int cout, int cin, int kh, int kw) {
  if (cout <= 0 || cin <= 0 || kh <= 0 || kw <= 0) return SCFLOW_EINVAL;
  return (long long)cout * kh * kw * ((cin + PH_K - 1) / PH_K * PH_K);
}

SCFLOW_API int scflow_ph_conv_pack(const float* w_oihw, float* packed, int cout, int cin, int kh,
                                   int kw, void* stream) {
  if (!w_oihw || !packed || cout <= 0 || cin <= 0 || kh <= 0 || kw <= 0) return SCFLOW_EINVAL;
  const int cinp = (cin + PH_K - 1) / PH_K * PH_K;
  const long long total = (long long)cout * kh * kw * cinp;
  const int blocks = (int)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
  ph_pack_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(w_oihw, packed, cout, cin, kh * kw, cinp);
  return scflow_launch_status();
}

SCFLOW_API int scflow_ph_conv(const float* src0, int c0, int s0, const float* src1, int c1, int s1,
                              const float* scale, const float* shift, const float* packed,
                              const float* bias, float* out, int n, int h, int w, int cout, int kh,
                              int kw, int stride, int pad, void* stream) {
  return scflow_ph_conv_split(src0, c0, s0, src1, c1, s1, scale, shift, packed, bias, out, n, h, w,
                              cout, kh, kw, stride, pad, 1, stream);
}

SCFLOW_API int scflow_ph_conv_split(const float* src0, int c0, int s0, const float* src1, int c1,
                                    int s1, const float* scale, const float* shift,
                                    const float* packed, const float* bias, float* out, int n, int h,
                                    int w, int cout, int kh, int kw, int stride, int pad, int ksplit,
                                    void* stream) {
  if (!src0 || !packed || !out || n <= 0 || h <= 0 || w <= 0 || cout <= 0 || c0 <= 0 || c1 < 0 ||
      (c1 > 0 && !src1) || kh <= 0 || kw <= 0 || stride <= 0 || pad < 0 || (scale && !shift) ||
      ksplit <= 0 || (ksplit > 1 && bias))
    return SCFLOW_EINVAL;
  if ((c0 & 3) || (c1 & 3) || (s0 & 3) || (c1 && (s1 & 3)) || !aligned16(src0) ||
      (c1 && !aligned16(src1)) || !aligned16(packed))
    return SCFLOW_EALIGN;
  PhConvArgs a{};
  a.src0 = src0; a.c0 = c0; a.s0 = s0;
  a.src1 = src1; a.c1 = c1; a.s1 = s1;
  a.scale = scale; a.shift = shift;
  a.weight = packed; a.bias = bias; a.out = out;
  a.n = n; a.h = h; a.w = w;
  a.oh = (h + 2 * pad - kh) / stride + 1;
  a.ow = (w + 2 * pad - kw) / stride + 1;
  if (a.oh <= 0 || a.ow <= 0) return SCFLOW_EINVAL;
  a.cout = cout; a.kh = kh; a.kw = kw; a.stride = stride; a.pad = pad;
  a.cinp = (c0 + c1 + PH_K - 1) / PH_K * PH_K;
  a.ksplit = ksplit;
  const long long M = (long long)n * a.oh * a.ow;
  dim3 grid((unsigned)((M + 31) / 32), (unsigned)((cout + 31) / 32), (unsigned)ksplit);
  ph_conv_kernel<<<grid, PH_WAVES * 64, 0, (hipStream_t)stream>>>(a);
  return scflow_launch_status();
}

SCFLOW_API int scflow_ph_gn_stats(const float* x, int n, int hw, int c, int groups,
                                  const float* gamma, const float* beta, float eps, float* scale,
                                  float* shift, void* stream) {
  return scflow_ph_gn_reduce(x, 1, 0, nullptr, n, hw, c, groups, gamma, beta, eps, scale, shift,
                             stream);
}

SCFLOW_API int scflow_ph_gn_reduce(const float* parts, int nsplit, long long split_stride, float* y,
                                   int n, int hw, int c, int groups, const float* gamma,
                                   const float* beta, float eps, float* scale, float* shift,
                                   void* stream) {
  if (!parts || !gamma || !beta || !scale || !shift || n <= 0 || hw <= 0 || c <= 0 ||
      groups <= 0 || nsplit <= 0 || c % groups || (nsplit > 1 && (!y || split_stride <= 0)))
    return SCFLOW_EINVAL;
  const int cpg = c / groups;
  if (c % 32 || 32 % cpg) return SCFLOW_EUNSUPPORTED;
  if (!aligned16(parts) || (y && !aligned16(y)) || (split_stride & 3)) return SCFLOW_EALIGN;
  // 16-channel blocks (twice the workgroups) when the group size allows; SCFLOW_GNR_CB=32 forces
  // the 32-channel blocks (A/B)
  static EnvSwitch cb_sw("SCFLOW_GNR_CB", 16);  // cached (scflow_debug_reload_switches)
  const int cbe = cb_sw.get();
  const bool c16 = cbe == 16 && 16 % cpg == 0;
  dim3 grid(n, c / (c16 ? 16 : 32));
#define SCFLOW_GNR(NS_)                                                                                    \
  do {                                                                                                     \
    if (c16)                                                                                               \
      ph_gn_reduce_kernel<NS_, 16><<<grid, 256, 0, (hipStream_t)stream>>>(parts, nsplit, split_stride, y, hw, \
                                                                          c, groups, gamma, beta, eps,       \
                                                                          scale, shift);                     \
    else                                                                                                   \
      ph_gn_reduce_kernel<NS_, 32><<<grid, 256, 0, (hipStream_t)stream>>>(parts, nsplit, split_stride, y, hw, \
                                                                          c, groups, gamma, beta, eps,       \
                                                                          scale, shift);                     \
  } while (0)
  switch (nsplit) {
    case 1: SCFLOW_GNR(1); break;
    case 2: SCFLOW_GNR(2); break;
    case 3: SCFLOW_GNR(3); break;
    case 4: SCFLOW_GNR(4); break;
    case 8: SCFLOW_GNR(8); break;
    default: SCFLOW_GNR(0); break;
  }
#undef SCFLOW_GNR
  return scflow_launch_status();
}

SCFLOW_API int scflow_ph_fc_permute(const float* W, float* Wp, int n, int c, int hw, void* stream) {
  if (!W || !Wp || n <= 0 || c <= 0 || hw <= 0) return SCFLOW_EINVAL;
  const long long total = (long long)n * c * hw;
  const int blocks = (int)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
  ph_fc_permute_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(W, Wp, n, c, hw);
  return scflow_launch_status();
}

SCFLOW_API int scflow_ph_fc(const float* x, int ldx, int m, int k, const float* W, const float* bias,
                            float* y, int n, int relu, int gn_c, const float* scale,
                            const float* shift, void* stream) {
  if (!x || !W || !y || m <= 0 || k <= 0 || n <= 0 || (k & 15) || (ldx & 3) || !aligned16(W) ||
      !aligned16(x) || (gn_c > 0 && (!scale || !shift || (gn_c & 3))))
    return SCFLOW_EINVAL;
  FcArgs f{};
  f.x = x; f.ldx = ldx; f.m = m; f.k = k; f.W = W; f.bias = bias; f.y = y; f.n = n; f.relu = relu;
  f.gn_c = gn_c; f.scale = scale; f.shift = shift;
  if (m <= 16)
    ph_fc_kernel<1><<<(n + 15) / 16, PH_WAVES * 64, 0, (hipStream_t)stream>>>(f);
  else
    ph_fc_kernel<2><<<(n + 15) / 16, PH_WAVES * 64, 0, (hipStream_t)stream>>>(f);
  return scflow_launch_status();
}

SCFLOW_API int scflow_ph_fc_split(const float* x, int ldx, int m, int k, const float* W,
                                  float* parts, int n, int ksplit, int gn_c, const float* scale,
                                  const float* shift, int xsplit, const float* xbias,
                                  void* stream) {
  if (!x || !W || !parts || m <= 0 || m > 32 || k <= 0 || n <= 0 || (k & 15) || (ldx & 3) ||
      ksplit <= 0 || ksplit > k / 16 || !aligned16(W) || !aligned16(x) ||
      (gn_c > 0 && (!scale || !shift || (gn_c & 3))) || xsplit < 0 || (xsplit > 0 && !xbias) ||
      (xsplit > 0 && gn_c > 0))
    return SCFLOW_EINVAL;
  FcArgs f{};
  f.x = x; f.ldx = ldx; f.m = m; f.k = k; f.W = W; f.y = parts; f.n = n;
  f.gn_c = gn_c; f.scale = scale; f.shift = shift; f.ksplit = ksplit;
  f.xsplit = xsplit; f.xstride = (long long)m * ldx; f.xbias = xbias;
  dim3 grid((unsigned)((n + 15) / 16), (unsigned)ksplit);
  if (m <= 16)
    ph_fc_kernel<1><<<grid, PH_WAVES * 64, 0, (hipStream_t)stream>>>(f);
  else
    ph_fc_kernel<2><<<grid, PH_WAVES * 64, 0, (hipStream_t)stream>>>(f);
  return scflow_launch_status();
}

SCFLOW_API int scflow_ph_fc_sum(const float* parts, int nsplit, int m, int k, const float* xbias,
                                const float* W, const float* bias, float* y, int n, int relu,
                                void* stream) {
  if (!parts || !xbias || !W || !y || nsplit <= 0 || m <= 0 || k <= 0 || n <= 0 || (k & 15) ||
      !aligned16(W) || !aligned16(parts) || !aligned16(xbias))
    return SCFLOW_EINVAL;
  FcArgs f{};
  f.x = parts; f.ldx = k; f.m = m; f.k = k; f.W = W; f.bias = bias; f.y = y; f.n = n; f.relu = relu;
  f.xsplit = nsplit; f.xstride = (long long)m * k; f.xbias = xbias;
  if (m <= 16)
    ph_fc_kernel<1><<<(n + 15) / 16, PH_WAVES * 64, 0, (hipStream_t)stream>>>(f);
  else
    ph_fc_kernel<2><<<(n + 15) / 16, PH_WAVES * 64, 0, (hipStream_t)stream>>>(f);
  return scflow_launch_status();
}

SCFLOW_API int scflow_ph_heads(const float* x, int m, int k, const float* Wr, const float* br,
                               int rch, const float* Wt, const float* bt, const long long* label,
                               int num_class, float* drot, float* dt, void* stream) {
  return scflow_ph_heads_sum(x, 0, nullptr, m, k, Wr, br, rch, Wt, bt, label, num_class, drot, dt,
                             stream);
}

SCFLOW_API int scflow_ph_heads_sum(const float* x, int xsplit, const float* xbias, int m, int k,
                                   const float* Wr, const float* br, int rch, const float* Wt,
                                   const float* bt, const long long* label, int num_class,
                                   float* drot, float* dt, void* stream) {
  if (xsplit < 0 || (xsplit > 0 && (!xbias || !aligned16(xbias)))) return SCFLOW_EINVAL;
  if (!x || !Wr || !br || !Wt || !bt || !label || !drot || !dt || m <= 0 || k <= 0 || (k & 15) ||
      rch <= 0 || rch + 3 > 9 || num_class <= 0 || !aligned16(x) || !aligned16(Wr) || !aligned16(Wt))
    return SCFLOW_EINVAL;
  // one workgroup per sample row, the arithmetic of the pose step's fused heads (pose_heads)
  PoseStepArgs a{};
  a.hx = x; a.hxs = (long long)m * k; a.hk = k; a.hsplit = xsplit; a.hxb = xbias;
  a.Wr = Wr; a.br = br; a.Wt = Wt; a.bt = bt; a.hlabel = label; a.hrch = rch; a.hncls = num_class;
  a.drot_out = drot; a.dt_out = dt;
  ph_heads_kernel<<<m, 256, 0, (hipStream_t)stream>>>(a);
  return scflow_launch_status();
}
