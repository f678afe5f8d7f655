// a2 + a3's first layer fused: the pyramid window lookup (CorrLookup, /root/reference/models/
// utils/corr_lookup.py:102-136) straight into MotionEncoder corr_net.0 (1×1 324 → 256 + ReLU,
// models/decoder/raft_decoder.py:75-85,152-166) — the L·(2r+1)² correlation features of a
// pixel never leave the CU (the separate path writes and re-reads them: 21 MB per iteration at
// B = 16, 256²; 166 MB at configs[4]).
//
// Workgroup = 64 pixels × every output channel, one per CU, 8 waves in two roles:
//  * 4 producer waves build the A tile (64 pixels × K = 324 channels, + zero padding to 8-channel
//    blocks) in LDS level by level: per level the pixels' 16×16 tile-aligned regions of the TILED pyramid
//    (b128 loads of whole 4-float tile rows, the layout of scflow_corr_pyramid_tiled) go to LDS,
//    and the (2r+1)² samples of every pixel are computed from them with the lookup's own
//    arithmetic (corr_lookup_lds_kernel<4, true, true>: grid_sample's normalise / unnormalise
//    round trip with FP contraction off, the same region origins, zero outside) into the pixel's
//    A row, channel l·81 + a·9 + b;
//  * 4 consumer waves run the GEMM as conv1x1w_kernel (conv1x1w.h) does: weights pre-packed in
//    MFMA-lane order and streamed from L2 into registers, 2 × 2 blocks of v_mfma_f32_32x32x2_f32
//    per wave;
//  * the roles overlap level by level: while the producers load and sample level l the consumers
//    multiply the 8-channel blocks levels < l completed — the lookup's latency chain and its
//    VALU / LDS work sit beside the MFMAs instead of between them; one barrier per level.
// The A values are bit-identical to the lookup kernel's outputs and the MFMA order is
// conv1x1w_kernel's, so the result equals scflow_corr_lookup_tiled + the wide 1×1 conv bit for
// bit (tests/test_gpu_ops.py).
#include "common.h"

namespace {

constexpr int LC_PX = 64;        // pixels per workgroup
constexpr int LC_R = 4;          // window radius
constexpr int LC_D = 2 * LC_R + 1;
constexpr int LC_L = 4;          // levels
constexpr int LC_K = LC_L * LC_D * LC_D;  // 324
constexpr int LC_KB = (LC_K + 7) / 8;     // 41 blocks of 8 channels
constexpr int LC_KP = 8 * LC_KB + 4;      // A row (floats): ≡ 4·odd mod 64 words
constexpr int LC_TRW = 16;                // region side (floats)
constexpr int LC_WP = LC_TRW * LC_TRW + 4;  // region stride per pixel (floats, ≡ 4 mod 64)
constexpr int LC_PD = 3;                  // weight blocks in flight ahead of the MFMAs
constexpr int LC_OOB = 0x7ffffff0;
// the 8-channel blocks complete once levels 0..l are sampled: [LC_KEND[l-1], LC_KEND[l])
constexpr int LC_KEND[LC_L] = {(1 * LC_D * LC_D) / 8, (2 * LC_D * LC_D) / 8, (3 * LC_D * LC_D) / 8,
                               LC_KB};
__host__ __device__ constexpr int lc_level(int kb) {
  return kb < LC_KEND[0] ? 0 : kb < LC_KEND[1] ? 1 : kb < LC_KEND[2] ? 2 : 3;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t lc_rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ floatx4 lc_bload4(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}

// bilinear_sample's normalisation + grid_sample's unnormalisation (corr_lookup.py:63-64), exactly
// as lookup.hip's unnorm_coord
__device__ __forceinline__ float lc_unnorm(float s, int size, int ac) {
#pragma clang fp contract(off)
  const float g = (s * 2.f) / (float)(size - 1 > 1 ? size - 1 : 1) - 1.f;
  return ac ? ((g + 1.f) / 2.f) * (float)(size - 1) : ((g + 1.f) * (float)size - 1.f) / 2.f;
}

struct LcArgs {
  const float* pyr;     // tiled pyramid (scflow_corr_pyramid_tiled)
  const float* flow;    // [n·h·w][2] (NHWC)
  const float* weight;  // 1×1 packing (SCFLOW_CONV_1X1W) of the [cout][324] conv weight
  const float* bias;    // [cout] or NULL
  float* out;           // [n·h·w][so]
  int so, n, h, w, cout, act, ac;
};

__global__ __launch_bounds__(512, 1) void corr_lookup_conv1x1_kernel(LcArgs a) {
#pragma clang fp contract(off)
  extern __shared__ floatx4 smem4[];
  float* As = (float*)smem4;               // [64][LC_KP]
  float* Wn = As + LC_PX * LC_KP;          // [64][LC_WP] one level's regions
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // waves 0-3 multiply (consumers), waves 4-7 look up (producers)
  const bool producer = wave >= 4;
  const int li = lane & 31, hh = lane >> 5;
  const int H = a.h, W = a.w, P = H * W;
  const long long M = (long long)a.n * P;
  const long long m0 = (long long)blockIdx.x * LC_PX;
  const int npad = (a.cout + 63) / 64 * 64;
  const bool wave_on = !producer && wave * 64 < npad;
  // a consumer lane's two output channels' bias, fetched now: every workgroup of the one-round
  // grid reaches the epilogue together, where these loads all waited on the same cache lines
  float bias_v[2] = {0.f, 0.f};
  if (wave_on && a.bias) {
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      const int col = 64 * wave + 32 * nb + li;
      if (col < a.cout) bias_v[nb] = a.bias[col];
    }
  }

  // a producer thread's pixel (4 threads of one wave per pixel) and its share of the columns a
  const int pt = producer ? tid - 256 : 0;
  const int ps = pt >> 2, sub = pt & 3;
  const long long gp = m0 + ps;
  const bool active = gp < M;
  const int p = active ? (int)(gp % P) : 0;
  const int y = p / W, x = p % W;
  float fx = 0.f, fy = 0.f;
  if (active) {
    fx = a.flow[gp * 2];
    fy = a.flow[gp * 2 + 1];
  }
  const long long left = M - m0;
  const int npx = left < LC_PX ? (int)left : LC_PX;

  // region origin of level l (map coordinates, one axis): corr_lookup_lds_kernel<4, true, true>
  auto origin = [&](int l, int axis, float c0x, float c0y) __attribute__((always_inline)) {
    const bool fin = isfinite(c0x) && isfinite(c0y) && fabsf(c0x) < 1e8f && fabsf(c0y) < 1e8f;
    int o = fin ? (int)floorf(axis == 0 ? c0x : c0y) - 1 : -(1 << 29);
    return ((axis == 0 ? W : H) >> l) <= 8 ? -4 : (o >> 2) << 2;
  };
  auto first = [&](int l, int axis) __attribute__((always_inline)) {  // the level's first sample coordinate on an axis
    const int size = axis == 0 ? (W >> l) : (H >> l);
    const float c = ((float)(axis == 0 ? x : y) + (axis == 0 ? fx : fy)) / (float)(1 << l);
    return lc_unnorm(c + (float)(0 - LC_R), size, a.ac);
  };

  auto last = [&](int l, int axis) __attribute__((always_inline)) {  // ... and its last
    const int size = axis == 0 ? (W >> l) : (H >> l);
    const float c = ((float)(axis == 0 ? x : y) + (axis == 0 ? fx : fy)) / (float)(1 << l);
    return lc_unnorm(c + (float)LC_R, size, a.ac);
  };

  // region loads of level l: the pixel's 64 tile rows, 16 per thread (k = sub + 4j) — only the
  // tile rows that hold a tap some sample reads (the taps' extent [floor(first sample),
  // floor(last sample) + 1] per axis: the samples increase along an axis), the others read as
  // zero without touching memory; the sampling phase is unchanged (those taps are never read)
  floatx4 wr[16];
  auto rload = [&](int l) __attribute__((always_inline)) {
    size_t loff = 0;
    for (int k = 0; k < l; ++k) loff += (size_t)M * ((H >> k) * (W >> k));
    const int Hl = H >> l, Wl = W >> l, hw = Hl * Wl;
    const __amdgpu_buffer_rsrc_t rs =
        lc_rsrc(a.pyr + loff + (size_t)m0 * hw, (unsigned)(npx * hw * 4));
    const float c0x = first(l, 0), c0y = first(l, 1);
    const int ox = origin(l, 0, c0x, c0y), oy = origin(l, 1, c0x, c0y);
    const float c1x = last(l, 0), c1y = last(l, 1);
    const bool fin = isfinite(c0x) && isfinite(c0y) && fabsf(c0x) < 1e8f && fabsf(c0y) < 1e8f &&
                     isfinite(c1x) && isfinite(c1y) && fabsf(c1x) < 1e8f && fabsf(c1y) < 1e8f;
    const int xlo = fin ? (int)floorf(c0x) : 1, xhi = fin ? (int)floorf(c1x) + 1 : 0;
    const int ylo = fin ? (int)floorf(c0y) : 1, yhi = fin ? (int)floorf(c1y) + 1 : 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int k = sub + 4 * j, kt = k >> 2;
      const int gx = ox + (kt & 3) * 4, gy = oy + (kt >> 2) * 4 + (k & 3);
      const bool ok = active && gx >= 0 && gx < Wl && gy >= 0 && gy < Hl && gy >= ylo &&
                      gy <= yhi && gx + 3 >= xlo && gx <= xhi;
      const int e = ((gy >> 2) * (Wl >> 2) + (gx >> 2)) * 16 + (gy & 3) * 4;
      wr[j] = lc_bload4(rs, ok ? (ps * hw + e) * 4 : LC_OOB, 0);
    }
  };
  auto rstore = [&]() __attribute__((always_inline)) {
    float* sw = Wn + ps * LC_WP;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int k = sub + 4 * j, kt = k >> 2;
      *(floatx4*)(sw + ((kt >> 2) * 4 + (k & 3)) * LC_TRW + (kt & 3) * 4) = wr[j];
    }
  };
  // samples of level l into the A row: this thread's columns a = sub, sub + 4, sub + 8
  auto sample = [&](int l) __attribute__((always_inline)) {
#pragma clang fp contract(off)
    const int Hl = H >> l, Wl = W >> l;
    const float scale = (float)(1 << l);
    const float cx = ((float)x + fx) / scale, cy = ((float)y + fy) / scale;
    const float c0x = lc_unnorm(cx + (float)(0 - LC_R), Wl, a.ac);
    const float c0y = lc_unnorm(cy + (float)(0 - LC_R), Hl, a.ac);
    const bool fin = isfinite(c0x) && isfinite(c0y) && fabsf(c0x) < 1e8f && fabsf(c0y) < 1e8f;
    const int ox = origin(l, 0, c0x, c0y), oy = origin(l, 1, c0x, c0y);
    float iy[LC_D];
    int ry[LC_D];
#pragma unroll
    for (int b = 0; b < LC_D; ++b) {
      iy[b] = lc_unnorm(cy + (float)(b - LC_R), Hl, a.ac);
      ry[b] = fin && isfinite(iy[b]) ? (int)floorf(iy[b]) - oy : -1;
    }
    const float* sw = Wn + ps * LC_WP;
    float* arow = As + ps * LC_KP + l * LC_D * LC_D;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int aa = sub + 4 * q;
      if (aa < LC_D) {
        const float ix = lc_unnorm(cx + (float)(aa - LC_R), Wl, a.ac);
        const int rx = fin && isfinite(ix) ? (int)floorf(ix) - ox : -1;
        const bool okx = active && rx >= 0 && rx + 1 < LC_TRW;
        float t00[LC_D], t01[LC_D], t10[LC_D], t11[LC_D];
        bool ok[LC_D];
#pragma unroll
        for (int b = 0; b < LC_D; ++b) {
          ok[b] = okx && ry[b] >= 0 && ry[b] + 1 < LC_TRW;
          const float* wp = sw + (ok[b] ? ry[b] * LC_TRW + rx : 0);
          t00[b] = wp[0];
          t01[b] = wp[1];
          t10[b] = wp[LC_TRW];
          t11[b] = wp[LC_TRW + 1];
        }
        const float ix_w = floorf(ix), ix_e = ix_w + 1.f;
        const float wxw = ix_e - ix, wxe = ix - ix_w;
#pragma unroll
        for (int b = 0; b < LC_D; ++b) {
          const float iy_n = floorf(iy[b]), iy_s = iy_n + 1.f;
          const float wyn = iy_s - iy[b], wys = iy[b] - iy_n;
          float v = 0.f;
          v += t00[b] * (wxw * wyn);
          v += t01[b] * (wxe * wyn);
          v += t10[b] * (wxw * wys);
          v += t11[b] * (wxe * wys);
          arow[aa * LC_D + b] = ok[b] ? v : 0.f;
        }
      }
    }
  };

  // weights: output channels 64·wave .. +63 (two 32-blocks), 1×1 packing [nb32][kb][lane][4]
  const __amdgpu_buffer_rsrc_t wsrc = lc_rsrc(a.weight + (size_t)(2 * wave) * LC_KB * 256,
                                              (unsigned)(wave_on ? 2 * LC_KB * 1024 : 0));
  auto bload = [&](floatx4(&bb)[2], int kb) {
    const int k = kb < LC_KB ? kb : LC_KB - 1;
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) bb[nb] = lc_bload4(wsrc, lane * 16, (nb * LC_KB + k) * 1024);
  };
  floatx16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  floatx4 bq[LC_PD][2];
  const float* ar0 = As + li * LC_KP + 4 * hh;
  const float* ar1 = As + (32 + li) * LC_KP + 4 * hh;
  // one block as straight-line code (conv1x1w_kernel's structure): the weights PD blocks and the
  // A fragments one block ahead are issued first, then the 16 MFMAs; a phase's first block reads
  // its A fragments itself (they are published by the barrier right before it)
  floatx4 an0, an1;
  auto body = [&](auto kbc) __attribute__((always_inline)) {
    constexpr int kb = decltype(kbc)::value, sl = kb % LC_PD;
    constexpr int l = lc_level(kb);
    constexpr bool opens = kb == (l == 0 ? 0 : LC_KEND[l == 0 ? 0 : l - 1]);
    constexpr bool last = kb + 1 == LC_KEND[l];
    if constexpr (opens) {
      an0 = *(const floatx4*)(ar0 + 8 * kb);
      an1 = *(const floatx4*)(ar1 + 8 * kb);
    }
    const floatx4 a0 = an0, a1 = an1;
    floatx4 b[2] = {bq[sl][0], bq[sl][1]};
    if constexpr (kb + LC_PD < LC_KB) bload(bq[sl], kb + LC_PD);
    if constexpr (!last) {
      an0 = *(const floatx4*)(ar0 + 8 * (kb + 1));
      an1 = *(const floatx4*)(ar1 + 8 * (kb + 1));
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[e], b[0][e], acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[e], b[1][e], acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[e], b[0][e], acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[e], b[1][e], acc[1][1], 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  // a producer's level-l region: written and read only by the pixel's own 4 lanes (one wave), so
  // a wave-level completion wait orders the stores before the samples' reads
  auto regions_to_lds = [&]() __attribute__((always_inline)) {
    rstore();
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS stores done
    __builtin_amdgcn_wave_barrier();
  };

  // Phase 0: the producers load level 0's regions into LDS and sample level 0; the consumers
  // prefetch their first weight blocks and zero the padding channels.
  // Phase l = 1..4: the producers load and sample level l while the consumers multiply the blocks
  // levels < l completed; one barrier ends each phase.
  if (producer) {
    rload(0);
    regions_to_lds();
    sample(0);
  } else {
#pragma unroll
    for (int d = 0; d < LC_PD; ++d) bload(bq[d], d);
    if (tid < LC_PX) {
#pragma unroll
      for (int c = LC_K; c < 8 * LC_KB; ++c) As[tid * LC_KP + c] = 0.f;
    }
  }
  __syncthreads();
  auto phase = [&](auto lc) __attribute__((always_inline)) {
    constexpr int l = decltype(lc)::value;  // 1..4
    if (producer) {
      if constexpr (l < LC_L) {  // (the region loads' latency hides under the consumers' phase)
        rload(l);
        regions_to_lds();
        sample(l);
      }
    } else {
      StaticFor<(l == 1 ? 0 : LC_KEND[l == 1 ? 0 : l - 2]), LC_KEND[l - 1]>::run(body);
    }
    if constexpr (l < LC_L) __syncthreads();
  };
  StaticFor<1, LC_L + 1>::run(phase);

  // epilogue (conv1x1w_kernel's): bias, activation; C/D col = lane&31, row = (r&3) + 8(r>>2) +
  // 4(lane>>5)
  if (!wave_on) return;  // (producers and idle consumer waves)
  auto store = [&](auto actc) __attribute__((always_inline)) {  // one body per activation
    constexpr int ACT = decltype(actc)::value;
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      const int col = 64 * wave + 32 * nb + li;
      if (col >= a.cout) continue;
#pragma unroll
      for (int mb = 0; mb < 2; ++mb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const long long m = m0 + 32 * mb + (r & 3) + 8 * (r >> 2) + 4 * hh;
          if (m < M) a.out[m * a.so + col] = act_apply(acc[mb][nb][r] + bias_v[nb], ACT);
        }
    }
  };
  switch (a.act) {
    case SCFLOW_ACT_RELU: store(std::integral_constant<int, SCFLOW_ACT_RELU>{}); break;
    case SCFLOW_ACT_SIGMOID: store(std::integral_constant<int, SCFLOW_ACT_SIGMOID>{}); break;
    case SCFLOW_ACT_TANH: store(std::integral_constant<int, SCFLOW_ACT_TANH>{}); break;
    default: store(std::integral_constant<int, SCFLOW_ACT_NONE>{}); break;
  }
}

}  // namespace

SCFLOW_API long long scflow_corr_lookup_conv1x1_lds_bytes(void) {
  return (long long)sizeof(float) * LC_PX * (LC_KP + LC_WP);
}

SCFLOW_API int scflow_corr_lookup_conv1x1(const float* pyr, const float* flow, const float* weight,
                                          const float* bias, float* out, int out_stride, int n,
                                          int h, int w, int num_levels, int radius, int cout,
                                          int act, int align_corners, void* stream) {
  if (!pyr || !flow || !weight || !out || n <= 0 || h <= 0 || w <= 0 || cout <= 0 ||
      out_stride < cout)
    return SCFLOW_EINVAL;
  if (num_levels != LC_L || radius != LC_R || cout > 256 || h % 32 || w % 32)
    return SCFLOW_EUNSUPPORTED;  // tiled maps down to level 3 (4×4 tiles), r = 4, L = 4
  if (!aligned16(pyr) || !aligned16(weight)) return SCFLOW_EALIGN;
  // the tile-region loads address one workgroup's 64 pixel maps of a level through a buffer
  // descriptor (offsets < 2^31 bytes)
  if ((long long)LC_PX * h * w * 4 >= LC_OOB) return SCFLOW_EUNSUPPORTED;
  LcArgs a;
  a.pyr = pyr;
  a.flow = flow;
  a.weight = weight;
  a.bias = bias;
  a.out = out;
  a.so = out_stride;
  a.n = n;
  a.h = h;
  a.w = w;
  a.cout = cout;
  a.act = act;
  a.ac = align_corners ? 1 : 0;
  const size_t lds = (size_t)scflow_corr_lookup_conv1x1_lds_bytes();
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)corr_lookup_conv1x1_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  const long long M = (long long)n * h * w;
  corr_lookup_conv1x1_kernel<<<(unsigned)((M + LC_PX - 1) / LC_PX), 512, lds, (hipStream_t)stream>>>(a);
  return scflow_launch_status();
}
