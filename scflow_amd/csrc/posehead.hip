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
#include "pose_dev.h"

#include <stdlib.h>

#include <algorithm>

namespace {

constexpr int PH_K = 16;  // K chunk per MFMA group
constexpr int PH_GN_KSMAX = 4;  // scflow_ph_conv_gn's K split at most (last-arriver fixup)
// arrival counters one per 256 B: device-scope atomics on one line serialise at the memory side
constexpr int PH_CNT_STRIDE = 64;

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
  // scflow_ph_conv_gn: the input's GroupNorm (+ ReLU) from its producer's per-tile partial
  // statistics (in_stats [n][in_tpi][in_groups][2] fp64 sum / sum of squares over in_hw pixels),
  // made into a per-workgroup affine table in LDS; this conv's own per-tile statistics into
  // out_stats [n][ph_gn_tpi(oh·ow)][out_groups][2].  All zero / NULL otherwise.
  const double* in_stats; int in_tpi, in_groups; const float* in_gamma; const float* in_beta;
  float in_eps;
  double* out_stats; int out_groups;
  float* parts; int* counters;  // scflow_ph_conv_gn K split: slabs + per-tile arrival counters
};

// partial statistics per image of a conv output with P = oh·ow pixels per image and 32-pixel
// tiles: one per tile when P % 32 == 0, one per image when a tile holds 32 / P whole images
// (P ∈ {16, 32}: at most two images per tile); 0 = unsupported
__host__ __device__ __forceinline__ int ph_gn_tpi(int P) {
  return P % 32 == 0 ? P / 32 : (P == 16 ? 1 : 0);
}

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
  // deterministic tree reduction of the waves' partial tiles
  for (int half = NW / 2; half >= 1; half >>= 1) {
    if (wave >= half && wave < 2 * half) {
#pragma unroll
      for (int r = 0; r < 16; ++r) red[((wave - half) * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh) * 33 + li] = acc[r];
    }
    __syncthreads();
    if (wave < half) {
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] += red[(wave * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh) * 33 + li];
    }
    __syncthreads();
  }
  if (a.counters && a.ksplit > 1) {
    // K-split fixup (scflow_ph_conv_gn): slab bz, then the tile's last-arriving workgroup sums
    // the slabs in slab order (its own from registers) and carries on with the full tile
    __shared__ int s_last;
    if (wave == 0 && nvalid) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int mm = m0 + (r & 3) + 8 * (r >> 2) + 4 * hh;
        if (mm < M)  // agent-scope stores: written through to the memory side
          __hip_atomic_store(a.parts + ((size_t)bz * M + mm) * a.cout + col, acc[r], __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int tile = by * gridDim.x + bx;
    if (threadIdx.x == 0) {  // agent-scope slab stores drained: no release fence needed
      const int old = __hip_atomic_fetch_add(a.counters + tile * PH_CNT_STRIDE, 1, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
      s_last = old == a.ksplit - 1;
    }
    __syncthreads();
    if (!s_last) return;
    if (wave == 0) {
      // every slab value first (≤ 4 slabs × 16: one memory latency), then the sums in slab order
      float sv[PH_GN_KSMAX][16];
#pragma unroll
      for (int zz = 0; zz < PH_GN_KSMAX; ++zz)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int mm = m0 + (r & 3) + 8 * (r >> 2) + 4 * hh;
          sv[zz][r] = (zz < a.ksplit && zz != bz && mm < M && nvalid)
                          ? __hip_atomic_load(a.parts + ((size_t)zz * M + mm) * a.cout + col,
                                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                          : 0.f;
        }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float v = 0.f;
#pragma unroll
        for (int zz = 0; zz < PH_GN_KSMAX; ++zz)
          if (zz < a.ksplit) v += zz == bz ? acc[r] : sv[zz][r];
        acc[r] = v;
      }
      if (threadIdx.x == 0)
        __hip_atomic_store(a.counters + tile * PH_CNT_STRIDE, 0, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (wave == 0 && nvalid) {
    const float b = a.bias ? a.bias[col] : 0.f;
    float* out = a.out + (a.counters ? 0 : (size_t)bz * M * a.cout);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int mm = m0 + (r & 3) + 8 * (r >> 2) + 4 * hh;
      if (mm < M) out[(size_t)mm * a.cout + col] = acc[r] + b;
    }
  }
  if (a.out_stats && wave == 0) {
    // this tile's GroupNorm partials: per lane (channel col, half hh) fp64 sums over its 16 rows
    // by image slot (rows of a second image when a tile holds two), then over hh (lane ^ 32) and
    // the group's channels (cpg adjacent lanes, cpg | 32), fixed order
    const int P = a.oh * a.ow;
    const int img0 = m0 / P;
    double s[2] = {0, 0}, q[2] = {0, 0};
    const float b = (nvalid && a.bias) ? a.bias[col] : 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int mm = m0 + (r & 3) + 8 * (r >> 2) + 4 * hh;
      if (mm < M && nvalid) {
        const double v = (double)(acc[r] + b);
        if (mm / P == img0) { s[0] += v; q[0] += v * v; } else { s[1] += v; q[1] += v * v; }
      }
    }
    const int cpg = a.cout / a.out_groups;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      s[k] += __shfl_xor(s[k], 32);
      q[k] += __shfl_xor(q[k], 32);
      for (int d = 1; d < cpg; d <<= 1) {
        s[k] += __shfl_xor(s[k], d);
        q[k] += __shfl_xor(q[k], d);
      }
    }
    if (hh == 0 && nvalid && col % cpg == 0) {
      const int tpi = ph_gn_tpi(P), g = col / cpg;
      const int t = P >= 32 ? (m0 % P) / 32 : 0;
      const int nimg = P >= 32 ? 1 : 2;
      for (int k = 0; k < nimg; ++k) {
        const int im = img0 + k;
        if (im >= a.n) break;
        double* o = a.out_stats + (((size_t)im * tpi + t) * a.out_groups + g) * 2;
        o[0] = s[k];
        o[1] = q[k];
      }
    }
  }
}

__global__ __launch_bounds__(PH_WAVES * 64) void ph_conv_kernel(PhConvArgs a) {
  __shared__ float red[PH_WAVES / 2 * 32 * 33];
  ph_conv_body<PH_WAVES>(a, blockIdx.x, blockIdx.y, blockIdx.z, red, a.scale, a.shift, 0,
                         a.c0 + a.c1);
}

// scflow_ph_conv_gn: the input GroupNorm affine of the (at most two) images this workgroup's
// output tile reads, from the producer's partial statistics, in LDS; then ph_conv_body
constexpr int PH_GN_MAXC = 256;
__global__ __launch_bounds__(PH_WAVES * 64) void ph_conv_gn_kernel(PhConvArgs a) {
  __shared__ float red[PH_WAVES / 2 * 32 * 33];
  __shared__ float tsc[2 * PH_GN_MAXC], tsh[2 * PH_GN_MAXC];
  const int cin = a.c0 + a.c1;
  const int P = a.oh * a.ow;
  const int img_lo = (blockIdx.x * 32) / P;
  if (a.in_stats) {
    for (int i = threadIdx.x; i < 2 * cin; i += blockDim.x) {
      const int im = img_lo + i / cin, c = i % cin;
      float sc = 0.f, sh = 0.f;
      if (im < a.n)
        ph_gn_affine(a.in_stats, a.in_tpi, a.in_groups, c, cin, im, a.h * a.w, a.in_gamma,
                     a.in_beta, a.in_eps, sc, sh);
      tsc[i] = sc;
      tsh[i] = sh;
    }
    __syncthreads();
  }
  ph_conv_body<PH_WAVES>(a, blockIdx.x, blockIdx.y, blockIdx.z, red, a.in_stats ? tsc : nullptr,
                         a.in_stats ? tsh : nullptr, img_lo, cin);
}

// GroupNorm statistics of x [n][hw][c] → per-channel scale/shift for y = relu(x·scale + shift),
// optionally first summing nsplit K-split partial slabs (x + z·split_stride) and writing the sum
// to y.  Grid (n, c/32): a workgroup takes one sample's 32-channel block; thread t holds channel
// quad t%8 of pixel slot t/8 (32 slots), float4 loads; per-channel sums in fp64 reduced over the
// slots in a fixed order, then per group (c/groups channels) → mean, biased variance.
// NS > 0: compile-time slab count; the pixel loop is unrolled PU-fold with every load of a
// round issued before any add (this kernel is latency-bound: 64 workgroups at B = 16; at the
// pose head's first conv every slot's 8 pixels × 4 slabs are one round)
template <int NS>
__global__ __launch_bounds__(256) void ph_gn_reduce_kernel(const float* __restrict__ x, int nsplit,
                                                           long long split_stride, float* __restrict__ y,
                                                           int hw, int c, int groups,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta, float eps,
                                                           float* __restrict__ scale,
                                                           float* __restrict__ shift) {
  __shared__ double s1[32][33], s2[32][33];
  __shared__ double gmean[32], grstd[32];
  const int img = blockIdx.x, cb = blockIdx.y * 32;
  const int q = threadIdx.x & 7, slot = threadIdx.x >> 3;
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
    constexpr int PU = NS <= 4 ? 8 : 1;  // ≤ 32 float4 loads in flight
    for (; p + 32 * (PU - 1) < hw; p += 32 * PU) {
      floatx4 v[PU][NS];
#pragma unroll
      for (int u = 0; u < PU; ++u)
#pragma unroll
        for (int z = 0; z < NS; ++z)
          v[u][z] = *(const floatx4*)(x + (size_t)z * split_stride + ((size_t)img * hw + p + 32 * u) * c +
                                      cb + 4 * q);
#pragma unroll
      for (int u = 0; u < PU; ++u) {
#pragma unroll
        for (int z = 1; z < NS; ++z) v[u][0] += v[u][z];
        acc(v[u][0], ((size_t)img * hw + p + 32 * u) * c + cb + 4 * q);
      }
    }
  }
  for (; p < hw; p += 32) {
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
  const int cpg = c / groups;       // channels per group (divides 32)
  const int ng = 32 / cpg;          // groups in this block
  if (threadIdx.x < ng) {
    double A = 0, B = 0;
    for (int k = 0; k < cpg; ++k)
      for (int sl = 0; sl < 32; ++sl) {
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
  if (threadIdx.x < 32) {
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
  // GN mode from the producer's partial statistics (scflow_ph_fc_split_gn): the per-(row,
  // channel) affine is built in LDS from gst [m][gst_tpi][gst_groups][2] over gst_hw pixels
  const double* gst; int gst_tpi, gst_groups, gst_hw; const float* gamma; const float* beta;
  float eps;
  int coherent_out;  // ksplit outputs stored at agent scope (read by a last-arriving workgroup)
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
    for (int half = NW / 2; half >= 1; half >>= 1) {
      if (wave >= half && wave < 2 * half) {
#pragma unroll
        for (int t = 0; t < FC_RT; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) red[(((wave - half) * FC_RT + t) * 64 + lane) * 5 + r] = acc[t][r];
      }
      __syncthreads();
      if (wave < half) {
#pragma unroll
        for (int t = 0; t < FC_RT; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[t][r] += red[((wave * FC_RT + t) * 64 + lane) * 5 + r];
      }
      __syncthreads();
    }
    if (wave == 0) {
      // C/D layout (16x16): col = lane&15 (batch row), row = 4(lane>>4) + r (neuron)
#pragma unroll
      for (int t = 0; t < FC_RT; ++t) {
        const int row = r0 + t * 16 + li;
        if (row >= f.m) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = i0 + 4 * kq + r;
          float v = acc[t][r];
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
            if (f.coherent_out)  // a last-arriver reads these from another XCD (fc2 + heads)
              __hip_atomic_store(yout + (size_t)row * f.n + i, v, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
            else
              yout[(size_t)row * f.n + i] = v;
          }
        }
      }
    }
  }
}

template <int FC_RT>
__global__ __launch_bounds__(PH_WAVES * 64) void ph_fc_kernel(FcArgs f) {
  __shared__ float red[PH_WAVES / 2 * FC_RT * 64 * 5];
  ph_fc_body<PH_WAVES, FC_RT>(f, blockIdx.x, blockIdx.y, red, f.scale, f.shift);
}

// FC2 + heads in one launch (scflow_ph_fc2_heads): the K-split FC2 partials as ph_fc_kernel,
// then the last-arriving workgroup (arrival counter hc, left at zero) sums them in slab order
// with FC2's bias + ReLU into LDS and computes label[0]'s rotation / translation rows
struct HeadsArgs {
  int dbg;  // tuning (SCFLOW_FC2H_DBG): bit 0 skips the heads, bit 1 plain FC2 stores, bit 2 the
            // arrival protocol
  int* counter;
  const float* b2;                      // FC2 bias [n2]
  const float* Wr; const float* br; int rch;
  const float* Wt; const float* bt;
  const long long* label; int num_class;
  float* drot; float* dt;
};

template <int FC_RT>
__global__ __launch_bounds__(PH_WAVES * 64) void ph_fc2_heads_kernel(FcArgs f, HeadsArgs h) {
  __shared__ float red[PH_WAVES / 2 * FC_RT * 64 * 5];
  __shared__ float x2[32 * 256];
  __shared__ float wrows[16 * 256];
  __shared__ int s_last;
  ph_fc_body<PH_WAVES, FC_RT>(f, blockIdx.x, blockIdx.y, red, f.scale, f.shift);
  if (h.dbg & 4) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {  // agent-scope slab stores drained: no release fence needed
    // two levels (one counter per 256 B): the K slices of a neuron tile, then the tiles — short
    // chains of device-scope atomics instead of one chain through every workgroup
    int* ct = h.counter + (1 + blockIdx.x) * PH_CNT_STRIDE;
    int last = __hip_atomic_fetch_add(ct, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
               (int)gridDim.y - 1;
    if (last) {
      __hip_atomic_store(ct, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = __hip_atomic_fetch_add(h.counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
             (int)gridDim.x - 1;
    }
    s_last = last;
  }
  __syncthreads();
  if (!s_last || (h.dbg & 1)) return;
  const int m = f.m, n2 = f.n;
  long long cls = h.label[0];
  if (cls < 0 || cls >= h.num_class) cls = 0;
  const int nout = h.rch + 3;
  float* wl = wrows;  // the class's nout ≤ 16 weight rows
  // every load first (one memory latency): FC2's ≤ 8 slabs per float4 of x2, the weight rows
  {
    constexpr int KSMAX = 8;
    for (int i4 = threadIdx.x; i4 < m * n2 / 4; i4 += blockDim.x) {
      floatx4 v[KSMAX];
#pragma unroll
      for (int z = 0; z < KSMAX; ++z)
        if (z < f.ksplit)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            v[z][e] = __hip_atomic_load(f.y + (size_t)z * m * n2 + 4 * i4 + e, __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT);
      floatx4 sum = v[0];
#pragma unroll
      for (int z = 1; z < KSMAX; ++z)
        if (z < f.ksplit) sum += v[z];
      const floatx4 b = *(const floatx4*)(h.b2 + (4 * i4) % n2);
#pragma unroll
      for (int e = 0; e < 4; ++e) x2[4 * i4 + e] = fmaxf(sum[e] + b[e], 0.f);
    }
    for (int i = threadIdx.x; i < nout * n2; i += blockDim.x) {
      const int o = i / n2, k = i % n2;
      wl[i] = o < h.rch ? h.Wr[((size_t)cls * h.rch + o) * n2 + k]
                        : h.Wt[((size_t)cls * 3 + (o - h.rch)) * n2 + k];
    }
  }
  if (threadIdx.x == 0) __hip_atomic_store(h.counter, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  // one wave per (row, output) pair: the lanes take consecutive k (conflict-free LDS reads),
  // then a fixed-order shuffle reduction
  {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int pr = wv; pr < m * nout; pr += blockDim.x / 64) {
      const int row = pr / nout, o = pr % nout;
      float acc = 0.f;
      for (int k = lane; k < n2; k += 64) acc += wl[o * n2 + k] * x2[row * n2 + k];
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) acc += __shfl_xor(acc, d);
      if (lane == 0) {
        if (o < h.rch)
          h.drot[(size_t)row * h.rch + o] = acc + h.br[cls * h.rch + o];
        else
          h.dt[(size_t)row * 3 + (o - h.rch)] = acc + h.bt[cls * 3 + (o - h.rch)];
      }
    }
  }
}

// FC with the input GroupNorm built from partial statistics: the [m][gn_c] affine in LDS first
constexpr int PH_FCGN_MAX = 32 * 128;
template <int FC_RT>
__global__ __launch_bounds__(PH_WAVES * 64) void ph_fc_gn_kernel(FcArgs f) {
  __shared__ float red[PH_WAVES / 2 * FC_RT * 64 * 5];
  __shared__ float tsc[PH_FCGN_MAX], tsh[PH_FCGN_MAX];
  for (int i = threadIdx.x; i < f.m * f.gn_c; i += blockDim.x) {
    float sc, sh;
    ph_gn_affine(f.gst, f.gst_tpi, f.gst_groups, i % f.gn_c, f.gn_c, i / f.gn_c, f.gst_hw, f.gamma,
                 f.beta, f.eps, sc, sh);
    tsc[i] = sc;
    tsh[i] = sh;
  }
  __syncthreads();
  ph_fc_body<PH_WAVES, FC_RT>(f, blockIdx.x, blockIdx.y, red, tsc, tsh);
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


// ---------------------------------------------------------------------------------------------
// scflow_ph_tail: GN 1 → conv 2 → GN 2 → conv 3 → GN 3 → FC1 → FC2 → heads (→ pose step) as one
// persistent launch.  Work items are numbered phase by phase (off[]); a workgroup takes the next
// ticket from sync[0], waits (one lane: relaxed sc1 polls + s_sleep, then ONE agent acquire) until
// the items it reads from have signalled, runs the item with the unfused kernels' bodies, and
// signals (every storing wave drains its stores, the workgroup joins, one lane releases at agent
// scope — the L2s of the 8 XCDs are not coherent with each other — and adds to the counter).  An
// item only waits for smaller tickets, all held by running workgroups, so the launch drains
// whatever the residency; every wait is bounded by the real-time clock (PHT_WAIT_TICKS) and a
// give-up sets the error word and lets every later wait fall through, so a protocol fault ends the
// launch instead of hanging it.  The host zeroes the sync words before every launch.
//   sync (ints): [0] ticket  [2] error  [3] GN-3 items done  [4] FC1 done  [5] FC2 done
//     [6] heads done  [8..12] first give-up: 1 + phase, ticket, counter index, value seen, target
//     [16 + i] GN 1 of sample i, [16 + n + i] conv 2 items over sample i, [16 + 2n + i] GN 2,
//     [16 + 3n + i] conv 3;  [16 + 4n + b] the last ticket workgroup b started (diagnostics)

struct PhGn {
  const float* x; int nsplit; long long sstride; float* y;
  int hw, c, groups; const float* gamma; const float* beta; float eps; float* scale; float* shift;
};

struct PhTail {
  int n;
  PhGn gn[3];
  PhConvArgs conv[2];
  FcArgs fc1, fc2, heads;
  int fc1_split, fc2_split;
  PoseStepArgs ps;
  int pose;
  int* sync;
  int off[10];  // first ticket of phase p; off[9] = total
  int dbg;      // debugging (SCFLOW_PHT_DBG): bit 0 skips the item bodies, bit 1 the publishes
  unsigned long long* stamps;  // debugging: per ticket 4 real-time stamps (start, waited, body, out)
  int* error;                  // sticky give-up flag across launches (host-checked), or null
};

enum { PHT_GN0, PHT_CONV2, PHT_GN1, PHT_CONV3, PHT_GN2, PHT_FC1, PHT_FC2, PHT_HEADS, PHT_POSE };
constexpr int PHT_CTR = 16;                          // first per-sample counter
constexpr unsigned long long PHT_WAIT_TICKS = 5000000;  // 50 ms of the 100 MHz real-time clock

__device__ __forceinline__ int pht_poll(int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// thread 0: until S[idx] ≥ target, then one agent acquire.  false: gave up (error set)
__device__ bool pht_wait(int* S, int idx, int target, int ticket, int ph) {
  int v = pht_poll(S + idx);
  if (v < target) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
      __builtin_amdgcn_s_sleep(2);
      v = pht_poll(S + idx);
      if (v >= target) break;
      if (pht_poll(S + 2) || __builtin_amdgcn_s_memrealtime() - t0 > PHT_WAIT_TICKS) {
        if (__hip_atomic_fetch_add(S + 8, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
          __hip_atomic_store(S + 9, ticket, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(S + 10, idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(S + 11, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(S + 12, target, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(S + 13, 1 + ph, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __hip_atomic_fetch_or(S + 2, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return false;
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  return true;
}

// after a thread-0 wait: the acquire's invalidate completes before any wave loads
__device__ __forceinline__ void pht_join_after_wait() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}

// GroupNorm of one (sample img, 32-channel block cb) with NW·64 threads: sums the K-split
// partial slabs (writes y when nsplit > 1, same order as ph_gn_reduce_kernel), fp64 moments —
// per wave by shuffles, then over the waves in a fixed order — then scale/shift per channel.
// red: NW·64 + 128 doubles of LDS.
template <int NW>
__device__ void ph_gn_body(const PhGn& g, int img, int cb, double* red) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int q = tid & 7, slot = tid >> 3;
  constexpr int SL = NW * 8;
  double a[4] = {0, 0, 0, 0}, b[4] = {0, 0, 0, 0};
  for (int p = slot; p < g.hw; p += SL) {
    const size_t off = ((size_t)img * g.hw + p) * g.c + cb + 4 * q;
    floatx4 u[4];
    u[0] = *(const floatx4*)(g.x + off);
#pragma unroll
    for (int z = 1; z < 4; ++z)
      if (z < g.nsplit) u[z] = *(const floatx4*)(g.x + z * g.sstride + off);
    floatx4 v = u[0];
#pragma unroll
    for (int z = 1; z < 4; ++z)
      if (z < g.nsplit) v += u[z];
    for (int z = 4; z < g.nsplit; z += 4) {  // the next ≤ 4 slabs' loads issued together
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (z + k < g.nsplit) u[k] = *(const floatx4*)(g.x + (z + k) * g.sstride + off);
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (z + k < g.nsplit) v += u[k];
    }
    if (g.nsplit > 1) *(floatx4*)(g.y + off) = v;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      a[e] += (double)v[e];
      b[e] += (double)v[e] * (double)v[e];
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
#pragma unroll
    for (int m = 8; m < 64; m <<= 1) {
      a[e] += __shfl_xor(a[e], m);
      b[e] += __shfl_xor(b[e], m);
    }
  }
  if (lane < 8) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      red[(wave * 2 + 0) * 32 + 4 * lane + e] = a[e];
      red[(wave * 2 + 1) * 32 + 4 * lane + e] = b[e];
    }
  }
  __syncthreads();
  double* ch = red + NW * 64;  // [2][32] per-channel sums
  if (tid < 64) {
    const int k = tid >> 5, cc = tid & 31;
    double s = 0;
    for (int w = 0; w < NW; ++w) s += red[(w * 2 + k) * 32 + cc];
    ch[k * 32 + cc] = s;
  }
  __syncthreads();
  const int cpg = g.c / g.groups, ng = 32 / cpg;
  double* gs = ch + 64;  // [2][≤32] group mean, rstd
  if (tid < ng) {
    double A = 0, B = 0;
    for (int k = 0; k < cpg; ++k) {
      A += ch[tid * cpg + k];
      B += ch[32 + tid * cpg + k];
    }
    const double cnt = (double)g.hw * cpg;
    const double mean = A / cnt;
    double var = B / cnt - mean * mean;
    if (var < 0) var = 0;
    gs[tid] = mean;
    gs[32 + tid] = 1.0 / sqrt(var + (double)g.eps);
  }
  __syncthreads();
  if (tid < 32) {
    const int c = cb + tid, gi = tid / cpg;
    const float sc = g.gamma[c] * (float)gs[32 + gi];
    g.scale[(size_t)img * g.c + c] = sc;
    g.shift[(size_t)img * g.c + c] = g.beta[c] - (float)gs[gi] * sc;
  }
}

constexpr int PHT_WAVES = 16;
constexpr int PHT_SMEM = PHT_WAVES / 2 * 32 * 33;  // floats: the largest body's LDS (conv)
static_assert(PHT_SMEM * 4 >= (PHT_WAVES * 64 + 192) * 8, "GN body LDS");
static_assert(PHT_SMEM >= PHT_WAVES / 2 * 2 * 64 * 5, "FC body LDS");

// the counters item (ph, i) waits for: [wait0, wait0 + wait_count), each up to `target`; and
// the ones it adds 1 to when done: [sig0, sig0 + sig_count)
struct PhtDeps {
  int wait0, wait_count, target;
  int sig0, sig_count;
};

// The kernel's arguments are read from the kernarg segment through a pointer made opaque once per
// item (asm): the compiler cannot hoist the ~1.2 KB of argument fields out of the ticket loop into
// registers (that spilled hundreds of SGPRs), it reloads what an item needs (scalar loads) into
// item-local copies.
typedef const PhTail __attribute__((address_space(4)))* PhTailK;

// an item-local copy of an argument sub-struct (word by word: scalar loads from the kernarg
// segment; a struct copy cannot bind an address-space-4 reference)
template <class T>
__device__ __forceinline__ T pht_kcopy(const T __attribute__((address_space(4)))* p) {
  static_assert(sizeof(T) % 4 == 0, "word copy");
  T v;
  const int __attribute__((address_space(4)))* src = (const int __attribute__((address_space(4)))*)p;
  int* dst = (int*)&v;
#pragma unroll
  for (int k = 0; k < (int)(sizeof(T) / 4); ++k) dst[k] = src[k];
  return v;
}

__device__ __forceinline__ PhtDeps pht_deps_k(PhTailK K, int ph, int i) {
  const int n = K->n;
  PhtDeps d{0, 0, 0, 0, 0};
  if (ph == PHT_GN0 || ph == PHT_GN1 || ph == PHT_GN2) {
    const int L = ph == PHT_GN0 ? 0 : ph == PHT_GN1 ? 1 : 2;
    const int img = i / (K->gn[L].c / 32);
    if (L > 0) {  // every conv item over this sample
      const int oh = K->conv[L - 1].oh, ow = K->conv[L - 1].ow;
      const int nt = (K->conv[L - 1].cout + 31) / 32, ks = K->conv[L - 1].ksplit;
      const int P = oh * ow;
      const int tiles = ((img + 1) * P - 1) / 32 - img * P / 32 + 1;
      d.wait0 = PHT_CTR + (L == 1 ? n : 3 * n) + img;
      d.wait_count = 1;
      d.target = tiles * nt * ks;
    }
    d.sig0 = L == 0 ? PHT_CTR + img : L == 1 ? PHT_CTR + 2 * n + img : 3;
    d.sig_count = 1;
  } else if (ph == PHT_CONV2 || ph == PHT_CONV3) {
    const int j = ph == PHT_CONV2 ? 0 : 1;
    const int nt = (K->conv[j].cout + 31) / 32, ks = K->conv[j].ksplit;
    const int bx = i / (ks * nt);
    const int P = K->conv[j].oh * K->conv[j].ow, M = n * P;
    const int lo = bx * 32 / P, hi = min(bx * 32 + 31, M - 1) / P;
    d.wait0 = PHT_CTR + (j == 0 ? 0 : 2 * n) + lo;
    d.wait_count = hi - lo + 1;
    d.target = K->gn[j].c / 32;
    d.sig0 = PHT_CTR + (j == 0 ? n : 3 * n) + lo;
    d.sig_count = hi - lo + 1;
  } else if (ph == PHT_FC1) {
    d.wait0 = 3; d.wait_count = 1; d.target = n * (K->gn[2].c / 32);
    d.sig0 = 4; d.sig_count = 1;
  } else if (ph == PHT_FC2) {
    d.wait0 = 4; d.wait_count = 1; d.target = K->off[PHT_FC1 + 1] - K->off[PHT_FC1];
    d.sig0 = 5; d.sig_count = 1;
  } else if (ph == PHT_HEADS) {
    d.wait0 = 5; d.wait_count = 1; d.target = K->off[PHT_FC2 + 1] - K->off[PHT_FC2];
    d.sig0 = 6; d.sig_count = 1;
  } else {
    d.wait0 = 6; d.wait_count = 1; d.target = 1;
  }
  return d;
}

template <int RT>
__global__ __launch_bounds__(PHT_WAVES * 64) void ph_tail_kernel(PhTail A) {
  __shared__ __attribute__((aligned(16))) float smem[PHT_SMEM];
  __shared__ int s_item;
  const int tid = threadIdx.x;
  PhTailK K = (PhTailK)__builtin_amdgcn_kernarg_segment_ptr();
  for (;;) {
    asm volatile("" : "+s"(K));
    int* const S = K->sync;
    if (tid == 0) s_item = __hip_atomic_fetch_add(S, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int t = __builtin_amdgcn_readfirstlane(s_item);
    __syncthreads();
    if (t >= K->off[9]) break;
    int ph = 0;
    while (t >= K->off[ph + 1]) ++ph;
    const int i = t - K->off[ph];
    const PhtDeps d = pht_deps_k(K, ph, i);
    unsigned long long* const st = K->stamps;
    if (st && tid == 0) st[4 * t] = __builtin_amdgcn_s_memrealtime();
    if (d.wait_count > 0) {
      if (tid == 0)
        for (int k = 0; k < d.wait_count; ++k)
          if (!pht_wait(S, d.wait0 + k, d.target, t, ph) && K->error)
            __hip_atomic_fetch_or(K->error, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      pht_join_after_wait();
    }
    const int dbg = K->dbg;
    if (st && tid == 0) st[4 * t + 1] = __builtin_amdgcn_s_memrealtime();
    if (!(dbg & 1)) {
      if (ph == PHT_GN0 || ph == PHT_GN1 || ph == PHT_GN2) {
        const int L = ph == PHT_GN0 ? 0 : ph == PHT_GN1 ? 1 : 2;
        const PhGn g = pht_kcopy(&K->gn[L]);
        const int ncb = g.c / 32;
        ph_gn_body<PHT_WAVES>(g, i / ncb, (i % ncb) * 32, (double*)smem);
      } else if (ph == PHT_CONV2 || ph == PHT_CONV3) {
        const PhConvArgs cv = pht_kcopy(&K->conv[ph == PHT_CONV2 ? 0 : 1]);
        const int nt = (cv.cout + 31) / 32;
        ph_conv_body<PHT_WAVES>(cv, i / (cv.ksplit * nt), (i / cv.ksplit) % nt, i % cv.ksplit, smem,
                                cv.scale, cv.shift, 0, cv.c0 + cv.c1);
      } else if (ph == PHT_FC1 || ph == PHT_FC2 || ph == PHT_HEADS) {
        const FcArgs f = pht_kcopy(ph == PHT_FC1 ? &K->fc1 : ph == PHT_FC2 ? &K->fc2 : &K->heads);
        const int split = ph == PHT_FC1 ? K->fc1_split : ph == PHT_FC2 ? K->fc2_split : 1;
        ph_fc_body<PHT_WAVES, RT>(f, i / split, i % split, smem, f.scale, f.shift);
      } else {
        const PoseStepArgs ps = pht_kcopy(&K->ps);
        const int nb = ps.bf + ps.bl;
        pose_step_body(ps, smem, i % nb, i / nb, tid, PHT_WAVES * 64, true);
      }
    }
    if (st) {
      __syncthreads();
      if (tid == 0) st[4 * t + 2] = __builtin_amdgcn_s_memrealtime();
    }
    if (d.sig_count > 0 && !(dbg & 2)) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's stores drained
      __syncthreads();
      if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        for (int k = 0; k < d.sig_count; ++k)
          __hip_atomic_fetch_add(S + d.sig0 + k, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    if (st && tid == 0) st[4 * t + 3] = __builtin_amdgcn_s_memrealtime();
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

SCFLOW_API int scflow_ph_gn_tpi(int oh, int ow) {
  if (oh <= 0 || ow <= 0) return SCFLOW_EINVAL;
  const int t = ph_gn_tpi(oh * ow);
  return t > 0 ? t : SCFLOW_EUNSUPPORTED;
}

SCFLOW_API int scflow_ph_conv_gn_plan_for(const scflow_ph_conv_gn_args* p,
                                          scflow_ph_conv_gn_plan* plan) {
  if (!p || !plan || p->n <= 0 || p->h <= 0 || p->w <= 0 || p->cout <= 0 || p->c0 <= 0 ||
      p->c1 < 0 || p->kh <= 0 || p->kw <= 0 || p->stride <= 0 || p->pad < 0)
    return SCFLOW_EINVAL;
  const int oh = (p->h + 2 * p->pad - p->kh) / p->stride + 1;
  const int ow = (p->w + 2 * p->pad - p->kw) / p->stride + 1;
  if (oh <= 0 || ow <= 0) return SCFLOW_EINVAL;
  const long long M = (long long)p->n * oh * ow;
  const int cin = p->c0 + p->c1;
  *plan = scflow_ph_conv_gn_plan{};
  // path 1: the halo-staged MFMA conv (tiles of whole output rows of one image)
  const int tm = p->stride == 1 ? 128 : 64;
  const int tc = ow < tm ? ow : tm;
  if (p->kh == 3 && p->kw == 3 && p->pad == 1 && (p->stride == 1 || p->stride == 2) &&
      p->c0 % 16 == 0 && p->c1 % 16 == 0 && p->cout % 64 == 0 && tc >= 8 && tm % tc == 0 &&
      ow % tc == 0 && oh % (tm / tc) == 0 && cin <= PH_GN_MAXC) {
    const int tpi_tiles = (oh / (tm / tc)) * (ow / tc);
    const long long tiles = (long long)p->n * tpi_tiles * (p->cout / 64);
    const int nst = cin / 16;
    plan->path = 1;
    plan->ksplit = (int)std::max(1LL, std::min({(long long)nst, (512 + tiles - 1) / tiles,
                                                (long long)PH_GN_KSMAX}));
    plan->tpi = 2 * tpi_tiles;
    plan->counters = (int)tiles;
  } else {
    const int tpi = ph_gn_tpi(oh * ow);
    if (!tpi || oh * ow < 16) return SCFLOW_EUNSUPPORTED;
    const long long tiles = ((M + 31) / 32) * ((p->cout + 31) / 32);
    const int nall = p->kh * p->kw * ((cin + PH_K - 1) / PH_K);
    plan->path = 0;
    plan->ksplit = (int)std::max(1LL, std::min({(long long)(nall / 16), (256 + tiles - 1) / tiles,
                                                (long long)PH_GN_KSMAX}));
    plan->tpi = tpi;
    plan->counters = (int)tiles;
  }
  plan->parts_floats = plan->ksplit > 1 ? (long long)plan->ksplit * M * p->cout : 0;
  plan->counters = plan->ksplit > 1 ? plan->counters * PH_CNT_STRIDE : 0;
  return SCFLOW_OK;
}

int scflow_enc_conv_gn_launch(const scflow_ph_conv_gn_args* g, int tm, void* stream);

SCFLOW_API int scflow_ph_conv_gn(const scflow_ph_conv_gn_args* p, void* stream) {
  if (!p || !p->src0 || !p->weight || !p->out || p->n <= 0 || p->h <= 0 || p->w <= 0 ||
      p->cout <= 0 || p->c0 <= 0 || p->c1 < 0 || (p->c1 > 0 && !p->src1) || p->kh <= 0 ||
      p->kw <= 0 || p->stride <= 0 || p->pad < 0 || p->ksplit < 1 ||
      (p->ksplit > 1 && (!p->parts || !p->counters)))
    return SCFLOW_EINVAL;
  scflow_ph_conv_gn_plan plan;
  const int pr = scflow_ph_conv_gn_plan_for(p, &plan);
  if (pr != SCFLOW_OK) return pr;
  if (p->ksplit != plan.ksplit) return SCFLOW_EINVAL;  // buffers were sized for the plan
  if (p->in_stats && (!p->in_gamma || !p->in_beta || p->in_groups <= 0 ||
                      (p->c0 + p->c1) % p->in_groups || p->in_tpi <= 0 || p->c0 + p->c1 > PH_GN_MAXC))
    return SCFLOW_EINVAL;
  if (p->out_stats && (p->out_groups <= 0 || p->cout % p->out_groups ||
                       32 % (p->cout / p->out_groups) || p->cout % 32))
    return SCFLOW_EUNSUPPORTED;
  if (plan.path == 1) {
    if (!aligned16(p->src0) || (p->s0 & 3) || !aligned16(p->weight) ||
        (p->c1 > 0 && (!aligned16(p->src1) || (p->s1 & 3))))
      return SCFLOW_EALIGN;
    return scflow_enc_conv_gn_launch(p, p->stride == 1 ? 128 : 64, stream);
  }
  if ((p->c0 & 3) || (p->c1 & 3) || (p->s0 & 3) || (p->c1 && (p->s1 & 3)) || !aligned16(p->src0) ||
      (p->c1 && !aligned16(p->src1)) || !aligned16(p->weight))
    return SCFLOW_EALIGN;
  PhConvArgs a{};
  a.src0 = p->src0; a.c0 = p->c0; a.s0 = p->s0;
  a.src1 = p->src1; a.c1 = p->c1; a.s1 = p->s1;
  a.weight = p->weight; a.out = p->out;
  a.n = p->n; a.h = p->h; a.w = p->w;
  a.oh = (p->h + 2 * p->pad - p->kh) / p->stride + 1;
  a.ow = (p->w + 2 * p->pad - p->kw) / p->stride + 1;
  if (a.oh <= 0 || a.ow <= 0) return SCFLOW_EINVAL;
  a.cout = p->cout; a.kh = p->kh; a.kw = p->kw; a.stride = p->stride; a.pad = p->pad;
  a.cinp = (p->c0 + p->c1 + PH_K - 1) / PH_K * PH_K;
  a.ksplit = p->ksplit;
  if (p->ksplit > 1) {
    a.parts = p->parts;
    a.counters = p->counters;
  }
  if (p->in_stats) {
    a.in_stats = p->in_stats; a.in_tpi = p->in_tpi; a.in_groups = p->in_groups;
    a.in_gamma = p->in_gamma; a.in_beta = p->in_beta; a.in_eps = p->in_eps;
  }
  if (p->out_stats) {
    a.out_stats = p->out_stats; a.out_groups = p->out_groups;
  }
  const long long M = (long long)p->n * a.oh * a.ow;
  dim3 grid((unsigned)((M + 31) / 32), (unsigned)((p->cout + 31) / 32), (unsigned)p->ksplit);
  ph_conv_gn_kernel<<<grid, PH_WAVES * 64, 0, (hipStream_t)stream>>>(a);
  return scflow_launch_status();
}

SCFLOW_API int scflow_ph_fc_split_gn(const float* x, int m, int k, const float* W, float* parts,
                                     int n, int ksplit, int gn_c, const double* stats, int tpi,
                                     int groups, int hw, const float* gamma, const float* beta,
                                     float eps, void* stream) {
  if (!x || !W || !parts || !stats || !gamma || !beta || m <= 0 || m > 32 || k <= 0 || n <= 0 ||
      (k & 15) || ksplit <= 0 || ksplit > k / 16 || gn_c <= 0 || (gn_c & 3) || k % gn_c ||
      groups <= 0 || gn_c % groups || tpi <= 0 || hw <= 0 || m * gn_c > PH_FCGN_MAX ||
      !aligned16(W) || !aligned16(x))
    return SCFLOW_EINVAL;
  FcArgs f{};
  f.x = x; f.ldx = k; f.m = m; f.k = k; f.W = W; f.y = parts; f.n = n; f.gn_c = gn_c;
  f.ksplit = ksplit;
  f.gst = stats; f.gst_tpi = tpi; f.gst_groups = groups; f.gst_hw = hw; f.gamma = gamma;
  f.beta = beta; f.eps = eps;
  dim3 grid((unsigned)((n + 15) / 16), (unsigned)ksplit);
  if (m <= 16)
    ph_fc_gn_kernel<1><<<grid, PH_WAVES * 64, 0, (hipStream_t)stream>>>(f);
  else
    ph_fc_gn_kernel<2><<<grid, PH_WAVES * 64, 0, (hipStream_t)stream>>>(f);
  return scflow_launch_status();
}

SCFLOW_API int scflow_ph_fc2_heads(const float* parts1, int xsplit, const float* b1, int m, int k,
                                   const float* W2, const float* b2, float* parts2, int n2,
                                   int ksplit, const float* Wr, const float* br, int rch,
                                   const float* Wt, const float* bt, const long long* label,
                                   int num_class, float* drot, float* dt, int* counter,
                                   void* stream) {
  if (!parts1 || xsplit <= 0 || !b1 || !W2 || !b2 || !parts2 || !Wr || !br || !Wt || !bt ||
      !label || !drot || !dt || !counter || m <= 0 || m > 32 || k <= 0 || (k & 15) || n2 <= 0 ||
      n2 % 4 || m * n2 > 32 * 256 || (rch + 3) * n2 > 16 * 256 || ksplit <= 0 || ksplit > 8 ||
      ksplit > k / 16 || rch <= 0 || num_class <= 0 ||
      !aligned16(parts1) || !aligned16(W2) || !aligned16(b1))
    return SCFLOW_EINVAL;
  FcArgs f{};
  f.x = parts1; f.ldx = k; f.m = m; f.k = k; f.W = W2; f.y = parts2; f.n = n2; f.ksplit = ksplit;
  f.xsplit = xsplit; f.xstride = (long long)m * k; f.xbias = b1;
  static const int dbg = [] {
    const char* e = getenv("SCFLOW_FC2H_DBG");
    return e ? atoi(e) : 0;
  }();
  f.coherent_out = (dbg & 2) ? 0 : 1;
  HeadsArgs h{dbg, counter, b2, Wr, br, rch, Wt, bt, label, num_class, drot, dt};
  dim3 grid((unsigned)((n2 + 15) / 16), (unsigned)ksplit);
  if (m <= 16)
    ph_fc2_heads_kernel<1><<<grid, PH_WAVES * 64, 0, (hipStream_t)stream>>>(f, h);
  else
    ph_fc2_heads_kernel<2><<<grid, PH_WAVES * 64, 0, (hipStream_t)stream>>>(f, h);
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
  dim3 grid(n, c / 32);
#define SCFLOW_GNR(NS_)                                                                           \
  ph_gn_reduce_kernel<NS_><<<grid, 256, 0, (hipStream_t)stream>>>(parts, nsplit, split_stride, y, hw, \
                                                                  c, groups, gamma, beta, eps,       \
                                                                  scale, shift)
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
      rch <= 0 || rch + 3 > 16 || num_class <= 0 || !aligned16(x) || !aligned16(Wr) || !aligned16(Wt))
    return SCFLOW_EINVAL;
  FcArgs f{};
  f.x = x; f.ldx = k; f.m = m; f.k = k; f.W = Wr; f.bias = br; f.y = drot; f.n = rch + 3;
  f.Wt = Wt; f.bt = bt; f.label = label; f.num_class = num_class; f.rch = rch; f.dt = dt;
  f.xsplit = xsplit; f.xstride = (long long)m * k; f.xbias = xbias;
  if (m <= 16)
    ph_fc_kernel<1><<<1, PH_WAVES * 64, 0, (hipStream_t)stream>>>(f);
  else
    ph_fc_kernel<2><<<1, PH_WAVES * 64, 0, (hipStream_t)stream>>>(f);
  return scflow_launch_status();
}

SCFLOW_API int scflow_ph_tail_sync_ints(int n) {
  if (n <= 0 || n > 32) return SCFLOW_EINVAL;
  return (PHT_CTR + 4 * n + 512 + 3) / 4 * 4;  // counters + per-workgroup diagnostics, 16-B multiple
}

SCFLOW_API int scflow_ph_tail(const scflow_ph_tail_args* p, void* stream) {
  if (!p) return SCFLOW_EINVAL;
  const int n = p->n, c = p->c;
  if (n <= 0 || n > 32 || c <= 0 || c % 32 || p->groups <= 0 || c % p->groups ||
      32 % (c / p->groups) || !p->conv1_parts || p->conv1_split <= 0 || !p->sync || !p->label ||
      !p->drot || !p->dt || p->kh <= 0 || p->stride <= 0 || p->pad < 0 || p->rch <= 0 ||
      p->rch + 3 > 16 || p->num_class <= 0)
    return SCFLOW_EINVAL;
  for (int l = 0; l < 3; ++l) {
    if (p->h[l] <= 0 || p->w[l] <= 0 || !p->gamma[l] || !p->beta[l] || !p->scale[l] ||
        !p->shift[l] || !p->y[l])
      return SCFLOW_EINVAL;
    if (l > 0 && (p->h[l] != (p->h[l - 1] + 2 * p->pad - p->kh) / p->stride + 1 ||
                  p->w[l] != (p->w[l - 1] + 2 * p->pad - p->kh) / p->stride + 1))
      return SCFLOW_EINVAL;
  }
  const int cinp = (c + PH_K - 1) / PH_K * PH_K;
  const int nchunks = p->kh * p->kh * (cinp / PH_K);
  for (int j = 0; j < 2; ++j)
    if (!p->conv_w[j] || !p->conv_parts[j] || p->conv_split[j] <= 0 || p->conv_split[j] > nchunks)
      return SCFLOW_EINVAL;
  const int k1 = c * p->h[2] * p->w[2];
  if (!p->fc1_w || !p->fc1_b || !p->fc1_parts || !p->fc2_w || !p->fc2_b || !p->fc2_parts ||
      !p->rot_w || !p->rot_b || !p->trans_w || !p->trans_b || p->fc1_n <= 0 || p->fc2_n <= 0 ||
      (k1 & 15) || (p->fc1_n & 15) || (p->fc2_n & 15) || p->fc1_split <= 0 ||
      p->fc1_split > k1 / 16 || p->fc2_split <= 0 || p->fc2_split > p->fc1_n / 16)
    return SCFLOW_EINVAL;
  if (!aligned16(p->conv1_parts) || !aligned16(p->fc1_w) || !aligned16(p->fc2_w) ||
      !aligned16(p->rot_w) || !aligned16(p->trans_w) || !aligned16(p->fc1_parts) ||
      !aligned16(p->fc2_parts) || !aligned16(p->fc1_b) || !aligned16(p->fc2_b))
    return SCFLOW_EALIGN;
  for (int l = 0; l < 3; ++l)
    if (!aligned16(p->y[l]) || !aligned16(p->scale[l]) || !aligned16(p->shift[l])) return SCFLOW_EALIGN;
  for (int j = 0; j < 2; ++j)
    if (!aligned16(p->conv_w[j]) || !aligned16(p->conv_parts[j])) return SCFLOW_EALIGN;

  PhTail A{};
  A.n = n;
  A.sync = p->sync;
  const float* gx[3] = {p->conv1_parts, p->conv_parts[0], p->conv_parts[1]};
  const int gs[3] = {p->conv1_split, p->conv_split[0], p->conv_split[1]};
  const float* gout[3];  // what the next consumer reads: the summed output (or the only slab)
  for (int l = 0; l < 3; ++l) {
    PhGn& g = A.gn[l];
    g.x = gx[l]; g.nsplit = gs[l]; g.hw = p->h[l] * p->w[l];
    g.sstride = (long long)n * g.hw * c; g.y = p->y[l];
    g.c = c; g.groups = p->groups; g.gamma = p->gamma[l]; g.beta = p->beta[l]; g.eps = p->eps[l];
    g.scale = p->scale[l]; g.shift = p->shift[l];
    gout[l] = gs[l] > 1 ? p->y[l] : gx[l];
  }
  for (int j = 0; j < 2; ++j) {
    PhConvArgs& a = A.conv[j];
    a.src0 = gout[j]; a.c0 = c; a.s0 = c;
    a.src1 = nullptr; a.c1 = 0; a.s1 = 0;
    a.scale = p->scale[j]; a.shift = p->shift[j];
    a.weight = p->conv_w[j]; a.bias = nullptr; a.out = p->conv_parts[j];
    a.n = n; a.h = p->h[j]; a.w = p->w[j]; a.oh = p->h[j + 1]; a.ow = p->w[j + 1];
    a.cout = c; a.kh = p->kh; a.kw = p->kh; a.stride = p->stride; a.pad = p->pad;
    a.cinp = cinp; a.ksplit = p->conv_split[j];
  }
  FcArgs& f1 = A.fc1;
  f1.x = gout[2]; f1.ldx = k1; f1.m = n; f1.k = k1; f1.W = p->fc1_w; f1.y = p->fc1_parts;
  f1.n = p->fc1_n; f1.gn_c = c; f1.scale = p->scale[2]; f1.shift = p->shift[2];
  f1.ksplit = p->fc1_split;
  FcArgs& f2 = A.fc2;
  f2.x = p->fc1_parts; f2.ldx = p->fc1_n; f2.m = n; f2.k = p->fc1_n; f2.W = p->fc2_w;
  f2.y = p->fc2_parts; f2.n = p->fc2_n; f2.ksplit = p->fc2_split; f2.xsplit = p->fc1_split;
  f2.xstride = (long long)n * p->fc1_n; f2.xbias = p->fc1_b;
  FcArgs& hd = A.heads;
  hd.x = p->fc2_parts; hd.ldx = p->fc2_n; hd.m = n; hd.k = p->fc2_n; hd.W = p->rot_w;
  hd.bias = p->rot_b; hd.y = p->drot; hd.n = p->rch + 3; hd.Wt = p->trans_w; hd.bt = p->trans_b;
  hd.label = p->label; hd.num_class = p->num_class; hd.rch = p->rch; hd.dt = p->dt;
  hd.xsplit = p->fc2_split; hd.xstride = (long long)n * p->fc2_n; hd.xbias = p->fc2_b;
  hd.ksplit = 1;
  A.fc1_split = p->fc1_split;
  A.fc2_split = p->fc2_split;
  int pose_items = 0;
  if (p->pose) {
    const scflow_pose_step_args* s = p->pose;
    if (s->n != n || s->drot6 != p->drot || s->dt != p->dt) return SCFLOW_EINVAL;
    const int st = pose_step_args(&A.ps, s->drot6, s->dt, s->R_src, s->t_src, s->K, s->points,
                                  s->R_dst, s->t_dst, s->flow, s->n, s->H, s->W, s->weight,
                                  s->depth_transform, s->invalid_num, s->lr, s->delta, s->mask,
                                  s->flow_up, s->mask_up, s->lr_next, s->s_next, s->hx_next,
                                  s->s_hx, s->h, s->w, s->up_scale, s->down_scale, PHT_WAVES * 64);
    if (st != SCFLOW_OK) return st;
    A.pose = 1;
    pose_items = (A.ps.bf + A.ps.bl) * n;
  }
  const int ncb = c / 32;
  const int items[9] = {
      n * ncb,
      ceil_div((long long)n * p->h[1] * p->w[1], 32) * ncb * p->conv_split[0],
      n * ncb,
      ceil_div((long long)n * p->h[2] * p->w[2], 32) * ncb * p->conv_split[1],
      n * ncb,
      ceil_div(p->fc1_n, 16) * p->fc1_split,
      ceil_div(p->fc2_n, 16) * p->fc2_split,
      1,
      pose_items};
  A.off[0] = 0;
  for (int k = 0; k < 9; ++k) A.off[k + 1] = A.off[k] + items[k];
  if (const char* e = getenv("SCFLOW_PHT_DBG")) A.dbg = atoi(e);
  A.stamps = (unsigned long long*)p->stamps;
  A.error = p->error;
  if (const char* e = getenv("SCFLOW_PHT_PHASES")) {  // debugging: run only the first k phases
    const int k = atoi(e);
    if (k >= 0 && k < 9) A.off[9] = A.off[k];
  }
  static int resident[2] = {0, 0};  // ≤ 512 (the diagnostics words)
  const int ri = n <= 16 ? 0 : 1;
  if (!resident[ri]) {
    int per_cu = 0;
    hipError_t e = ri == 0 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, ph_tail_kernel<1>, PHT_WAVES * 64, 0)
                           : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, ph_tail_kernel<2>, PHT_WAVES * 64, 0);
    if (e != hipSuccess || per_cu <= 0) per_cu = 1;
    resident[ri] = per_cu * device_cus() < 512 ? per_cu * device_cus() : 512;
  }
  const int grid = A.off[9] < 1 ? 1 : A.off[9] < resident[ri] ? A.off[9] : resident[ri];
  hipError_t me = hipMemsetAsync(p->sync, 0, scflow_ph_tail_sync_ints(n) * sizeof(int), (hipStream_t)stream);
  if (me != hipSuccess) return (int)me;
  if (ri == 0)
    ph_tail_kernel<1><<<grid, PHT_WAVES * 64, 0, (hipStream_t)stream>>>(A);
  else
    ph_tail_kernel<2><<<grid, PHT_WAVES * 64, 0, (hipStream_t)stream>>>(A);
  return scflow_launch_status();
}
