// Thin conv (cout ≤ 4, KH·KW·cout ≤ 32) as a channel contraction on fp32 MFMA (round 6) —
// included by conv.hip (inside its anonymous namespace).  The XHead flow predictor 256 → 2 (3×3,
// raft_decoder.py:256-294 / scflow_decoder.py:211-214).
//
// out[p][o] = Σ_tap Σ_c X[p + off(tap)][c]·W[o][tap][c] is rewritten as
//   Z[q][tap·cout + o] = Σ_c X[q][c]·W[o][tap][c]    (one GEMM: every input pixel q read ONCE)
//   out[p][o] = bias[o] + Σ_tap Z[p + off(tap)][tap·cout + o]
// so the 256 input channels of a pixel are contracted once into KH·KW·cout (18) partial sums,
// and only those cross the tap halo.  The chunked LDS kernel (conv_thin_kernel) staged 3 input
// rows per output row in 32-channel chunks (8 barrier-separated round trips, 3× L2 reads): at 64 ×
// 64 maps 82 µs alone, 105 µs in the decoder's critical path, for 134 MB of input.
//
// Workgroup = R output rows of one image (W = 32 or 64 columns); it contracts the R + KH − 1 rows
// of input pixels (the KH − 1 halo rows recomputed: (R+2)/R of the input read from L2) in blocks
// of 32 pixels on v_mfma_f32_32x32x2_f32 — A = the pixels' channels (lanes 0-31: channels 0-3 of an
// 8-channel group, lanes 32-63: 4-7; MFMA e takes channel 8g + 4hh + e on both operands), B = the
// packed weights, held in VGPRs for all channels (C/2 per lane), columns = tap·cout + o (≤ 32) —
// then the Z rows meet in LDS and each thread sums one output pixel's taps.  fp32 throughout;
// only the summation order differs from the direct conv.
// body: workgroup blk of a grid of nblk (conv_pair.h launches two bodies in one grid)
template <int COUT, int KH, int KW, int W, int R>
__device__ __forceinline__ void conv_thinz_body(const scflow_conv_args& a, int blk, int nblk) {
  constexpr int C = 256;                       // input channels (the dispatch checks)
  constexpr int NT = KH * KW * COUT;           // Z columns used
  constexpr int ZR = R + KH - 1;               // Z rows (input rows) per workgroup
  constexpr int NB = ZR * W / 32;              // 32-pixel blocks
  constexpr int NBW = (NB + 3) / 4;            // blocks per wave
  constexpr int ZLD = NT + 1;                  // LDS row of one Z pixel (odd: conflict-free)
  constexpr int G = C / 8;                     // 8-channel groups
  constexpr int GB = 8;                        // groups per load batch (64 channels in flight)
  static_assert(NT <= 32, "thinz: at most 32 Z columns");
  __shared__ float zs[ZR * W * ZLD];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int li = lane & 31, hh = lane >> 5;
  const int tiles_per_img = a.h / R;
  // XCD-aware order: each XCD takes a contiguous run of row tiles (shared halo rows in its L2)
  const int bid = nblk % 8 ? blk : (blk % 8) * (nblk / 8) + blk / 8;
  const int img = bid / tiles_per_img;
  const int oy0 = (bid - img * tiles_per_img) * R;
  // B fragments: W[o][tap][c] packed [o][tap][c]; lane (li, hh) of MFMA (g, e) holds column
  // t = li = tap·cout + o, channel 8g + 4hh + e
  float bw[G][4];
  {
    const int t = li < NT ? li : 0;
    const int tap = t / COUT, o = t - tap * COUT;
    const float* wp = a.weight + ((size_t)o * KH * KW + tap) * C + 4 * hh;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const floatx4 v = li < NT ? *(const floatx4*)(wp + 8 * g) : floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int e = 0; e < 4; ++e) bw[g][e] = v[e];
    }
  }
  const __amdgpu_buffer_rsrc_t src = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(a.src0), (short)0,
      (int)((((long long)a.n * a.h * W - 1) * a.s0 + C) * 4), 0x00020000);
#pragma unroll
  for (int j = 0; j < NBW; ++j) {
    const int blk = wave + 4 * j;  // wave-uniform
    if (blk >= NB) break;
    const int zp = blk * 32 + li;  // Z pixel of this lane's A row
    const int zr = zp / W, zx = zp - zr * W;
    const int iy = oy0 - KH / 2 + zr;
    const bool rok = iy >= 0 && iy < a.h;  // a halo row outside the image: Z = 0
    const int base = rok ? ((img * a.h + iy) * W + zx) * a.s0 * 4 + 16 * hh : 0x7ffffff0;
    floatx16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
    floatx4 xa[GB], xb[GB];
    auto ld = [&](floatx4(&x)[GB], int g0) __attribute__((always_inline)) {
#pragma unroll
      for (int k = 0; k < GB; ++k)
        x[k] = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(
                                               src, rok ? base + 32 * (g0 + k) : 0x7ffffff0, 0, 0));
    };
    auto mm = [&](const floatx4(&x)[GB], int g0) __attribute__((always_inline)) {
#pragma unroll
      for (int k = 0; k < GB; ++k)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(x[k][e], bw[g0 + k][e], acc, 0, 0, 0);
    };
    ld(xa, 0);
#pragma unroll
    for (int g0 = 0; g0 < G; g0 += 2 * GB) {
      if (g0 + GB < G) ld(xb, g0 + GB);
      __builtin_amdgcn_sched_barrier(0);
      mm(xa, g0);
      if (g0 + 2 * GB < G) ld(xa, g0 + 2 * GB);
      __builtin_amdgcn_sched_barrier(0);
      if (g0 + GB < G) mm(xb, g0 + GB);
    }
    // C/D layout: column (Z column t) = lane & 31, row (pixel) = (r&3) + 8(r>>2) + 4hh
    if (li < NT) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        zs[(blk * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh) * ZLD + li] = acc[r];
    }
  }
  __syncthreads();
  // taps: out[p][o] = bias[o] + Σ_{ty,tx} Z[row(p)+ty][col(p)+tx−KW/2][(ty·KW+tx)·cout + o]
  for (int i = threadIdx.x; i < R * W * COUT; i += 256) {
    const int o = i % COUT, p = i / COUT;
    const int py = p / W, px = p - py * W;
    float v = a.bias ? a.bias[o] : 0.f;
#pragma unroll
    for (int ty = 0; ty < KH; ++ty)
#pragma unroll
      for (int tx = 0; tx < KW; ++tx) {
        const int x = px + tx - KW / 2;
        if (x >= 0 && x < W) v += zs[((py + ty) * W + x) * ZLD + (ty * KW + tx) * COUT + o];
      }
    a.out[((size_t)(img * a.h + oy0 + py) * W + px) * a.so + o] = act_apply(v, a.act);
  }
}

template <int COUT, int KH, int KW, int W, int R>
__global__ __launch_bounds__(256, 2) void conv_thinz_kernel(scflow_conv_args a) {
  conv_thinz_body<COUT, KH, KW, W, R>(a, blockIdx.x, gridDim.x);
}
