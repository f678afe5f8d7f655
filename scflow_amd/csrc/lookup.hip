// a2 — multi-scale pyramid window lookup (CorrLookup, /root/reference/models/utils/corr_lookup.py:102-136).
//
// 16 lanes per source pixel p, 16 pixels per workgroup:
//  1. the pixel's lanes compute the sample coordinates of every level once — the reference's own
//     arithmetic: centroid (x+flow)/2^l, + window offset, normalise g·2/max(W−1,1)−1 and the
//     align_corners unnormalise ((g+1)/2)·(W−1), FP contraction off, so each sample's floor()
//     is grid_sample's;
//  2. they stage, per level, a region in LDS with rows of D+3 floats: the whole map with a
//     zero border when it fits (levels ≥ 2 at SCFlow's 32×32: 10 and 6 rows), else the
//     (D+3)² window around floor(first sample) − 1 with zero padding (one-tap margin each
//     side: a rounded sample coordinate can move its floor by at most one) — 480 instead of
//     576 floats per pixel at r = 4, L = 4, so every pixel of a B=16 batch is resident at once.
//     The region-relative floor of every (level, axis, index) is computed once here (not
//     once per sample);
//  3. the lanes take the L·D (level, column) pairs in turn and produce the D samples of each
//     (channel k = l·D² + a·D + b samples x+a−r, y+b−r) from LDS with grid_sample's bilinear
//     weights (nw, ne, sw, se; taps outside the map are zero).
// The pyramid (≈5.6 MB per pair at 256²) is read through L2 / Infinity Cache.
// A generic one-thread-per-(p, l, a) kernel remains for L > 4 or r > 6.
// scflow_corr_lookup_tiled reads a pyramid whose maps are stored in 4×4 tiles of 16 floats
// (scflow_corr_pyramid_tiled): the same loads, addressed into the tiles, so a wave's window
// loads coalesce into ≈ 3.3² whole 64-B sectors per level instead of 12 row segments that
// straddle sector boundaries (the configs[4] over-fetch, profiles/traffic_b32_s512.json).
// Round 3: on maps of at most 32×32 (the headline configs[1]) the tiled kernel stages 16×16
// tile-aligned regions through b128 tile-row loads / LDS stores (TR below, 4 loads per lane per
// level instead of 9).
#include "common.h"

namespace {

// bilinear_sample's normalisation g = s·2/max(size−1, 1) − 1 (corr_lookup.py:63-64), then
// grid_sample's unnormalisation: align_corners ((g+1)/2)·(size−1), else ((g+1)·size − 1)/2
__device__ __forceinline__ float unnorm_coord(float s, int size, int ac) {
#pragma clang fp contract(off)
  const float g = (s * 2.f) / (float)(size - 1 > 1 ? size - 1 : 1) - 1.f;
  return ac ? ((g + 1.f) / 2.f) * (float)(size - 1) : ((g + 1.f) * (float)size - 1.f) / 2.f;
}

__device__ __forceinline__ float tap(const float* __restrict__ m, int x, int y, int Wl, int Hl) {
  return (x >= 0 && x < Wl && y >= 0 && y < Hl) ? m[y * Wl + x] : 0.f;
}

template <int R>
__global__ __launch_bounds__(256) void corr_lookup_kernel(
    const float* __restrict__ pyr, const float* __restrict__ flow, int flow_layout,
    float* __restrict__ out, int out_layout, int out_stride, int N, int H, int W, int L,
    long long total, int ac) {
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
  // level base offset
  size_t off = 0;
  int Hl = H, Wl = W;
  for (int l = 0; l < lvl; ++l) {
    off += (size_t)N * P * Hl * Wl;
    Hl >>= 1;
    Wl >>= 1;
  }
  const float* m = pyr + off + ((size_t)n * P + p) * Hl * Wl;
  const float scale = (float)(1 << lvl);
  const float cx = ((float)x + fx) / scale;
  const float cy = ((float)y + fy) / scale;
  const float ix = unnorm_coord(cx + (float)(a - r), Wl, ac);
  const float ix_w = floorf(ix);
  const float ix_e = ix_w + 1.f;
  const int xw = (int)ix_w, xe = xw + 1;
  float* o = out_layout == SCFLOW_LAYOUT_NHWC
                 ? out + ((size_t)n * P + p) * out_stride + lvl * D * D + a * D
                 : out + ((size_t)n * L * D * D + lvl * D * D + a * D) * P + p;
  const int ostep = out_layout == SCFLOW_LAYOUT_NHWC ? 1 : P;
#pragma unroll
  for (int b = 0; b < D; ++b) {
    const float iy = unnorm_coord(cy + (float)(b - r), Hl, ac);
    const float iy_n = floorf(iy);
    const float iy_s = iy_n + 1.f;
    const int yn = (int)iy_n, ys = yn + 1;
    const float nw = (ix_e - ix) * (iy_s - iy);
    const float ne = (ix - ix_w) * (iy_s - iy);
    const float sw = (ix_e - ix) * (iy - iy_n);
    const float se = (ix - ix_w) * (iy - iy_n);
    float v = 0.f;
    v += tap(m, xw, yn, Wl, Hl) * nw;
    v += tap(m, xe, yn, Wl, Hl) * ne;
    v += tap(m, xw, ys, Wl, Hl) * sw;
    v += tap(m, xe, ys, Wl, Hl) * se;
    o[(size_t)b * ostep] = v;
  }
}

constexpr int LK_MAXL = 4;
constexpr int LK_PPW = 4;              // pixels per wave (16 lanes each)
constexpr int LK_GL = 64 / LK_PPW;     // lanes per pixel
constexpr int LK_SLOTS = 4 * LK_PPW;   // pixels per workgroup

// LDS region of level l for a pixel, rows of WIN floats: the whole map with a zero border
// ((h>>l)+2 rows) when it fits in the (D+3)-wide window, else the (D+3)² window.  Returns the
// floats of one pixel slot (all levels), ≡ 4 mod 8: 16-B aligned slots whose 4 per wave start
// in different banks.
__host__ __device__ inline bool lk_whole(int hl, int wl, int win) { return hl + 2 <= win && wl + 2 <= win; }
// region row length: tile regions 16; tile-row regions (TB, origin at the lowest tap) 2r + 3;
// plain regions (origin one tap below the first sample's floor) 2r + 4
__host__ __device__ constexpr int lk_win(int r, bool tr, bool tb) { return tr ? 16 : (tb ? 2 * r + 3 : 2 * r + 4); }
__host__ __device__ inline int lk_rows(int hl, int wl, int win) { return lk_whole(hl, wl, win) ? hl + 2 : win; }
__host__ __device__ inline int lk_slot_floats(int h, int w, int L, int win) {
  int t = 0;
  for (int l = 0; l < L; ++l) t += lk_rows(h >> l, w >> l, win) * win;
  t = (t + 3) & ~3;
  return (t & 7) ? t : t + 4;
}

// TB: two levels' regions at a time (levels 0, 1 are stored, then sampled, then levels 2, 3), so
// a pixel slot holds two regions of the largest level size — half the LDS of all four — and the
// region loads still in registers while a pair is sampled are the other pair's only: 6
// workgroups per CU instead of 4 (round 5).  Region p of the slot starts at p·lk_tb_region().
// Round 6: at r = 4 the TB regions use a swizzled row layout.  The sampling phase reads 4-byte
// taps, and ds_read_b32 serves a wave in two 32-lane groups over 32 banks ((a/4) mod 32,
// MI355X_MICROARCH.md §LDS): a group = 2 pixels × 16 consecutive samples s = 9a + b, whose tap
// (b + dy, a + dx) sat at (b + dy)·11 + a + dx — 2–3-way conflicts inside a pixel and between
// the two (SQ_LDS_BANK_CONFLICT 1.29e7 of 3.51e7 LDS cycles at configs[4], 63 % of them the tap
// reads: profiles/r06/g3_lookup_conflicts.txt).  Row r now starts at LK_TB_ROW[r] ≡ 25·r
// (mod 32) — 25 = 9⁻¹ mod 32, so a tap's bank is 25·s + const: 32 consecutive samples hit 32
// distinct banks — packed without overlap into 136 floats; the slot (two regions, 272 floats)
// ≡ 16 mod 32 puts the group's second pixel on the other 16 banks.  The region stores (rows
// 4j..4j+3 × 4 tiles per 16 lanes) land on distinct banks by the same residues.
// row starts {0, 89, 114, 11, 100, 125, 22, 47, 72, 33, 58} = (25·r mod 32) + 32·k_r, the k_r
// packed 2 bits per row (arithmetic, not a table: no memory lookup per tap)
__host__ __device__ constexpr int lk_tb_row4(int r) {
  return ((25 * r) & 31) + 32 * ((1462072 >> (2 * r)) & 3);
}
static_assert(lk_tb_row4(0) == 0 && lk_tb_row4(1) == 89 && lk_tb_row4(2) == 114 && lk_tb_row4(3) == 11 &&
              lk_tb_row4(4) == 100 && lk_tb_row4(5) == 125 && lk_tb_row4(6) == 22 &&
              lk_tb_row4(7) == 47 && lk_tb_row4(8) == 72 && lk_tb_row4(9) == 33 && lk_tb_row4(10) == 58,
              "swizzled row starts");
constexpr int LK_TB4_REGION = 136;
#ifndef LK_TB_SWZ  // 0: the round-5 row-major regions (A/B build)
#define LK_TB_SWZ 1
#endif
__host__ __device__ inline int lk_tb_region(int h, int w, int L, int win) {
  if (LK_TB_SWZ && win == 11) return LK_TB4_REGION;  // r = 4: the swizzled layout (rows ≤ 11)
  int t = 0;
  for (int l = 0; l < L; ++l) {
    const int r = lk_rows(h >> l, w >> l, win) * win;
    t = r > t ? r : t;
  }
  return (t + 3) & ~3;
}
__host__ __device__ inline int lk_tb_slot_floats(int h, int w, int L, int win) {
  const int t = 2 * lk_tb_region(h, w, L, win);
  if (LK_TB_SWZ && win == 11) return t;  // 272 ≡ 16 mod 32
  return (t & 7) ? t : t + 4;
}
// coordinates of a pixel slot: [level][axis][index] padded to ≡ 16 mod 32 floats, so the two
// pixels of a 32-lane group read them on different banks
__host__ __device__ constexpr int lk_crd_stride(int d) {
  return LK_TB_SWZ ? LK_MAXL * 2 * d + ((16 - (LK_MAXL * 2 * d) % 32) % 32 + 32) % 32 : LK_MAXL * 2 * d;
}

#ifndef LK_DBG_STORE_LINEAR
#define LK_DBG_STORE_LINEAR 0
#endif
#ifndef LK_DBG_SAMPLE_LINEAR
#define LK_DBG_SAMPLE_LINEAR 0
#endif
constexpr int LK_OOB = 0x7ffffff0;  // buffer voffset of a zero tap (beyond any num_records)

// TR (tile regions, tiled maps only): every level's region is the 4×4 block of 4×4 tiles (16×16
// floats) whose first tile holds floor(first sample) − 1 (a map axis of ≤ 8: the whole axis from
// −4, a zero tile before it), loaded as whole tile rows (one b128 per
// lane, 4 lanes per 64-B tile) and stored as b128 into 16-float LDS rows.  The 12×12 window it
// contains is what the plain regions hold; the extra columns / rows cost LDS, not memory-side
// bytes: the 12-wide window already touches 3–4 tiles per axis, every one of them whole 64-B
// sectors.  Slot stride ≡ 16 mod 64 floats so a wave's 4 pixel slots start in different banks.
constexpr int LK_TRW = 16;
__host__ __device__ inline int lk_tr_slot_floats(int L) { return L * LK_TRW * LK_TRW + 16; }

// A pixel's coordinates, floors and regions are written and read only by its own 16 lanes (one
// wave): the tile-row kernel (TB) orders its phases with a wave-level LDS barrier, so the 4 waves
// of a workgroup run their phases independently instead of meeting at every block barrier.
template <bool WAVE>
__device__ __forceinline__ void lk_sync() {
  if constexpr (WAVE) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  } else {
    __syncthreads();
  }
}

__device__ __forceinline__ float lk_bload(__amdgpu_buffer_rsrc_t r, int voff) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, 0, 0));
}

// TB (tiled maps, plain regions; round 5): the regions are filled from whole tile rows — one
// b128 load per (region row, tile), 4 lanes per 64-B tile, the 3–4 tiles of a region row
// contiguous in memory — and only the tiles that hold a tap some sample reads (the exact extent
// [min floor, max floor + 1] of the 9 samples per axis, clipped to the map) are loaded: ≈ 10.6
// instead of 14 whole 64-B sectors per windowed level, issued as 16-B lane pieces of 192–256-B
// runs instead of 9 scattered b32 gathers per lane.  Every region float is still written (data,
// or zero for a tile outside the extent or the map), so the sampling phase is unchanged.
//
// TILED: the pyramid's maps are in 4×4 tiles of 16 floats (scflow_corr_pyramid_tiled)
template <int R, bool TILED, bool TR = false, bool TB = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(TB ? 6 : 3))) void corr_lookup_lds_kernel(
    const float* __restrict__ pyr, const float* __restrict__ flow, int flow_layout,
    float* __restrict__ out, int out_layout, int out_stride, int N, int H, int W, int L,
    int vec_out, int ac, unsigned long long* stamps) {
#pragma clang fp contract(off)
  constexpr int D = 2 * R + 1;
  constexpr int WIN = lk_win(R, TR, TB);  // LDS row length of a level's region
  static_assert(!TR || (TILED && D + 3 <= LK_TRW - 3), "tile regions: tiled maps, r <= 4");
  static_assert(!TB || (TILED && !TR && WIN <= 13),
                "tile-row regions: tiled maps, plain regions of at most 13 columns (r <= 5)");
  // profiling (scflow_debug_lookup_stamps): thread 0's real-time-clock stamps at the phase
  // boundaries, 6 per workgroup
  auto stamp = [&](int k) {
    if (stamps && threadIdx.x == 0) stamps[(size_t)blockIdx.x * 6 + k] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  constexpr int NPR = (LK_MAXL * D + LK_GL - 1) / LK_GL;  // (level, a) pairs per lane
  extern __shared__ float win[];  // [LK_SLOTS][slot floats]
  __shared__ float crd_s[LK_SLOTS][lk_crd_stride(D)];
  auto crd = [&](int sl, int l, int axis, int i) -> float& { return crd_s[sl][(l * 2 + axis) * D + i]; };
  __shared__ signed char sr[LK_SLOTS][LK_MAXL][2][D];  // region-relative floor of a sample, −1: none
  // TB, r = 4: per (level, y sample) the swizzled starts of the tap rows ry, ry + 1 packed as
  // r0 | r1 << 7, or −1 when a tap row is off the region (computed once, not per sample)
  constexpr bool ROWT = TB && R == 4 && LK_TB_SWZ;
  __shared__ short rowt[ROWT ? LK_SLOTS : 1][LK_MAXL][D];
  __shared__ int org[LK_SLOTS][LK_MAXL][2];    // region origin (map coordinates)
  __shared__ int ext[LK_SLOTS][LK_MAXL][2][2];  // TB: taps read, [lo, hi] (map coordinates)
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ks = lane / LK_GL;                    // pixel slot within the wave
  const int slot = wave * LK_PPW + ks;
  const int gl = lane % LK_GL;                    // lane within the pixel's group
  const int P = H * W;
  const long long NP = (long long)N * P;
  float* sw = win + slot * (TR ? lk_tr_slot_floats(L)
                                : (TB ? lk_tb_slot_floats(H, W, L, WIN) : lk_slot_floats(H, W, L, WIN)));
  const long long gp0 = (long long)blockIdx.x * LK_SLOTS + wave * LK_PPW;  // wave's first pixel
  const long long gp = gp0 + ks;                                          // n·P + p
  const bool active = gp < NP;
  const int n = active ? (int)(gp / P) : 0;
  const int p = active ? (int)(gp % P) : 0;
  const int y = p / W, x = p % W;
  float fx = 0.f, fy = 0.f;
  if (active) {
    if (flow_layout == SCFLOW_LAYOUT_NHWC) {
      fx = flow[((size_t)n * P + p) * 2 + 0];
      fy = flow[((size_t)n * P + p) * 2 + 1];
    } else {
      fx = flow[((size_t)n * 2 + 0) * P + p];
      fy = flow[((size_t)n * 2 + 1) * P + p];
    }
  }
  // 1. sample coordinates, once per (level, axis, index)
  for (int t = gl; t < L * 2 * D; t += LK_GL) {
    const int l = t / (2 * D), axis = (t / D) % 2, i = t % D;
    const int size = axis == 0 ? (W >> l) : (H >> l);
    const float c = ((float)(axis == 0 ? x : y) + (axis == 0 ? fx : fy)) / (float)(1 << l);
    crd(slot, l, axis, i) = unnorm_coord(c + (float)(i - R), size, ac);
  }
  lk_sync<TB>();
  stamp(1);
  // 1b. per (level, axis): the region origin — −1 for a whole map, else floor(first sample) − 1
  //     (one-tap margin: a rounded sample coordinate moves its floor by at most one), far out
  //     of the map when the level has no finite samples; per (level, axis, index): the sample's
  //     region-relative floor
  for (int t = gl; t < L * 2 * D; t += LK_GL) {
    const int l = t / (2 * D), axis = (t / D) % 2, i = t % D;
    const bool whole = !TR && lk_whole(H >> l, W >> l, WIN);
    const float c0x = crd(slot, l, 0, 0), c0y = crd(slot, l, 1, 0);
    const bool fin = isfinite(c0x) && isfinite(c0y) && fabsf(c0x) < 1e8f && fabsf(c0y) < 1e8f;
    const float s = crd(slot, l, axis, i);
    int o = whole ? -1 : (fin ? (int)floorf(axis == 0 ? c0x : c0y) - 1 : -(1 << 29));
    // TB: the taps the samples read on this axis, [lo, hi] = [min floor, max floor + 1] over the
    // finite samples; the region starts at lo (D + 2 columns hold them: 9 samples at most
    // size/(size−1) < (D+1)/D apart on a windowed axis span < D columns)
    int lo = 1 << 30, hi = -(1 << 30);
    if (TB && fin) {
      for (int j = 0; j < D; ++j) {
        const float sj = crd(slot, l, axis, j);
        if (isfinite(sj)) {
          const int f = (int)floorf(sj);
          lo = min(lo, f);
          hi = max(hi, f + 1);
        }
      }
      if (!whole) o = lo;
    }
    // tile regions: an axis of at most 8 is held whole with a one-tile zero border ([−4, 12)),
    // else from the tile holding floor(first sample) − 1 (arithmetic shift: floor for negatives);
    // 9 samples spaced size/(size−1) ≤ 12/11 apart then end at most 14 columns into the region
    if (TR) o = ((axis == 0 ? W : H) >> l) <= 8 ? -4 : (o >> 2) << 2;
    // region-relative floor; anything outside [−1, WIN) is a sample with a tap off the region
    // (zero: the map's padding) — kept as −1 so it fits a byte
    const int rel = fin && isfinite(s) ? (int)floorf(s) - o : -1;
    sr[slot][l][axis][i] = (signed char)(rel >= 0 && rel < WIN ? rel : -1);
    if constexpr (ROWT) {
      if (axis == 1) {
        const int rows = lk_rows(H >> l, W >> l, WIN);
        rowt[slot][l][i] = (short)(rel >= 0 && rel + 1 < rows && rel + 1 < WIN
                                       ? lk_tb_row4(rel) | (lk_tb_row4(rel + 1) << 7) : -1);
      }
    }
    if (i == 0) org[slot][l][axis] = o;
    if (TB && i == 0) {
      ext[slot][l][axis][0] = lo;
      ext[slot][l][axis][1] = hi;
    }
  }
  lk_sync<TB>();
  // 2. regions (zero padded) through buffer loads (out-of-map taps read as zero, no branches):
  //    every load of the pixel's L regions is issued before the LDS writes
  int rn[LK_MAXL], ox[LK_MAXL], oy[LK_MAXL];
  constexpr int NS = 3;        // TB: (region row, tile) slots per lane and level
  floatx4 tbv[LK_MAXL][NS];    // TB: every level's region loads, in flight together
#pragma unroll
  for (int l = 0; l < LK_MAXL; ++l) {
    ox[l] = l < L ? org[slot][l][0] : 0;
    oy[l] = l < L ? org[slot][l][1] : 0;
  }
  if constexpr (TR) {
    // 16 lanes × 4 b128 = the region's 64 tile rows (tile kt = k / 4 of the 4×4 block, row k % 4)
    floatx4 tv4[LK_MAXL][4];
    size_t loff = 0;
    int Hl = H, Wl = W;
    const long long left = NP - gp0;
    const int npx = left < LK_PPW ? (int)left : LK_PPW;
#pragma unroll
    for (int l = 0; l < LK_MAXL; ++l) {
      const bool use = l < L;
      const int hw = Hl * Wl;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<float*>(pyr + loff + (size_t)gp0 * hw), (short)0, use ? npx * hw * 4 : 0,
          0x00020000);
      rn[l] = use ? LK_TRW * LK_TRW : 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = gl + LK_GL * j, kt = k >> 2;
        const int gx = ox[l] + (kt & 3) * 4, gy = oy[l] + (kt >> 2) * 4 + (k & 3);
        const bool ok = use && active && gx >= 0 && gx < Wl && gy >= 0 && gy < Hl;
        const int e = ((gy >> 2) * (Wl >> 2) + (gx >> 2)) * 16 + (gy & 3) * 4;
        tv4[l][j] = __builtin_bit_cast(
            floatx4, __builtin_amdgcn_raw_buffer_load_b128(rs, ok ? (ks * hw + e) * 4 : LK_OOB, 0, 0));
      }
      if (use) loff += (size_t)NP * hw;
      Hl >>= 1;
      Wl >>= 1;
    }
    stamp(2);
#pragma unroll
    for (int l = 0; l < LK_MAXL; ++l) {
      if (l < L) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int k = gl + LK_GL * j, kt = k >> 2;
          *(floatx4*)(sw + l * LK_TRW * LK_TRW + ((kt >> 2) * 4 + (k & 3)) * LK_TRW + (kt & 3) * 4) =
              tv4[l][j];
        }
      }
    }
  } else if constexpr (TB) {
    // 48 (region row, tile) slots per level, 3 per lane: slot k = row k / 4, tile k % 4 of the
    // 4 tiles from the one holding region column 0 (covers the ≤ 12 region columns); stored to
    // LDS level by level in the sampling phase
    floatx4 (&tv4)[LK_MAXL][NS] = tbv;
    size_t loff = 0;
    int Hl = H, Wl = W;
    const long long left = NP - gp0;
    const int npx = left < LK_PPW ? (int)left : LK_PPW;
#pragma unroll
    for (int l = 0; l < LK_MAXL; ++l) {
      const bool use = l < L;
      const int hw = Hl * Wl;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<float*>(pyr + loff + (size_t)gp0 * hw), (short)0, use ? npx * hw * 4 : 0,
          0x00020000);
      rn[l] = use ? lk_rows(Hl, Wl, WIN) * WIN : 0;
      const bool whole = lk_whole(Hl, Wl, WIN);
      // rows / columns to load: the taps' extent (a whole map: all of it), clipped to the map
      const int xlo = max(whole ? 0 : (use ? ext[slot][l][0][0] : 0), 0);
      const int xhi = min(whole ? Wl - 1 : (use ? ext[slot][l][0][1] : -1), Wl - 1);
      const int ylo = max(whole ? 0 : (use ? ext[slot][l][1][0] : 0), 0);
      const int yhi = min(whole ? Hl - 1 : (use ? ext[slot][l][1][1] : -1), Hl - 1);
      const int tx0 = ox[l] >> 2;  // arithmetic shift: floor for negative origins
#pragma unroll
      for (int j = 0; j < NS; ++j) {
        const int k = gl + LK_GL * j;
        const int gy = oy[l] + (k >> 2), tx = tx0 + (k & 3);
        const bool ok = use && active && gy >= ylo && gy <= yhi && 4 * tx + 3 >= xlo && 4 * tx <= xhi;
        const int e = ((gy >> 2) * (Wl >> 2) + tx) * 16 + (gy & 3) * 4;
        tv4[l][j] = __builtin_bit_cast(
            floatx4, __builtin_amdgcn_raw_buffer_load_b128(rs, ok ? (ks * hw + e) * 4 : LK_OOB, 0, 0));
      }
      if (use) loff += (size_t)NP * hw;
      Hl >>= 1;
      Wl >>= 1;
    }
    stamp(2);
  } else {
  constexpr int NW1 = (WIN * WIN + LK_GL - 1) / LK_GL;  // loads per lane per level
  float vals[LK_MAXL][NW1];
  {
    size_t loff = 0;
    int Hl = H, Wl = W;
    const long long left = NP - gp0;
    const int npx = left < LK_PPW ? (int)left : LK_PPW;  // pixels of this wave
#pragma unroll
    for (int l = 0; l < LK_MAXL; ++l) {
      const bool use = l < L;
      const int hw = Hl * Wl;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<float*>(pyr + loff + (size_t)gp0 * hw), (short)0, use ? npx * hw * 4 : 0,
          0x00020000);
      rn[l] = use ? lk_rows(Hl, Wl, WIN) * WIN : 0;
#pragma unroll
      for (int j = 0; j < NW1; ++j) {
        const int i = gl + LK_GL * j;
        const int gx = ox[l] + i % WIN, gy = oy[l] + i / WIN;
        const bool ok = i < rn[l] && active && gx >= 0 && gx < Wl && gy >= 0 && gy < Hl;
        const int e = TILED ? ((gy >> 2) * (Wl >> 2) + (gx >> 2)) * 16 + (gy & 3) * 4 + (gx & 3)
                            : gy * Wl + gx;
        vals[l][j] = lk_bload(rs, ok ? (ks * hw + e) * 4 : LK_OOB);
      }
      if (use) loff += (size_t)NP * hw;
      Hl >>= 1;
      Wl >>= 1;
    }
  }
  stamp(2);
  {
    int off = 0;
#pragma unroll
    for (int l = 0; l < LK_MAXL; ++l) {
#pragma unroll
      for (int j = 0; j < NW1; ++j) {
        const int i = gl + LK_GL * j;
        if (i < rn[l]) sw[off + i] = vals[l][j];
      }
      off += rn[l];
    }
  }
  }
  lk_sync<TB>();
  stamp(3);
  // 3. samples: the pixel's 16 lanes take its L·D (level, a) pairs in turn and produce the D
  //    samples b of each (channel k = l·D² + a·D + b samples x+a−r, y+b−r); a sample whose
  //    2×2 taps leave the region is zero (off the map: grid_sample's zero padding).  Every LDS
  //    read of a pair is issued before its arithmetic (clamped addresses, selects, no branches)
  int offl[LK_MAXL];
  {
    int o = 0;
#pragma unroll
    for (int l = 0; l < LK_MAXL; ++l) {
      offl[l] = o;
      o += rn[l];
    }
  }
  if constexpr (TB) {
    // level by level, sample s = gl + 16j of the level's D² (a = s / D, b = s % D: channel
    // l·D² + s), so the pixel's 16 lanes produce 16 consecutive output channels per round and
    // store them straight to memory (64 contiguous bytes per pixel, channels-last); no result
    // registers, no staging pass.  Region origin = the lowest tap, so the floors are ≈ (b, a)
    // and the 4 tap reads of a round hit a fixed bank pattern.
    if (!active) return;
    float* o = out_layout == SCFLOW_LAYOUT_NHWC ? out + ((size_t)n * P + p) * out_stride
                                                : out + (size_t)n * L * D * D * P + p;
    const size_t ostep = out_layout == SCFLOW_LAYOUT_NHWC ? 1 : (size_t)P;
    constexpr int NJ = (D * D + LK_GL - 1) / LK_GL;
    const int rsz = lk_tb_region(H, W, L, WIN);
#pragma unroll
    for (int l = 0; l < LK_MAXL; ++l) {
      if (l >= L) break;
      const int off = (l & 1) * rsz, rows = rn[l] / WIN;
      if ((l & 1) == 0) {  // levels l, l + 1 into the slot's two regions (data, or zero outside
                           // the extent / the map)
        if (l) lk_sync<TB>();  // the wave's samples of levels l − 2, l − 1 have read the slot
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const int lp = l + p;
          if (lp < LK_MAXL && lp < L) {
            const int rws = rn[lp] / WIN;
            const int c0 = ((ox[lp] >> 2) << 2) - ox[lp];  // region column of the first tile's column 0
#pragma unroll
            for (int j = 0; j < NS; ++j) {
              const int k = gl + LK_GL * j, r = k >> 2;
              const int cb = c0 + 4 * (k & 3);
              if (r < rws) {
#pragma unroll
                for (int q = 0; q < 4; ++q)
                  if (cb + q >= 0 && cb + q < WIN) {
#if LK_DBG_STORE_LINEAR  // attribution build only (bank conflicts per phase): conflict-free addresses
                    win[((p * NS * 4 + j * 4 + q) & 3) * 256 + (int)threadIdx.x] = tbv[lp][j][q];
#else
                    sw[p * rsz + (R == 4 && LK_TB_SWZ ? lk_tb_row4(r) : r * WIN) + cb + q] = tbv[lp][j][q];
#endif
                  }
              }
            }
          }
        }
        lk_sync<TB>();
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int sidx = gl + LK_GL * j;
        if (D * D % LK_GL != 0 && sidx >= D * D) break;
        const int a = sidx / D, b = sidx - a * D;
        const int rx = sr[slot][l][0][a];
        // y: the tap rows' validity, and (ROWT) their swizzled row starts, one LDS read
        const int ry = ROWT ? (int)rowt[slot][l][b] : (int)sr[slot][l][1][b];
        const float ix = crd(slot, l, 0, a), iy = crd(slot, l, 1, b);
        const bool ok = rx >= 0 && rx + 1 < WIN && ry >= 0 && (ROWT || ry + 1 < rows);
#if LK_DBG_SAMPLE_LINEAR  // attribution build only: conflict-free tap addresses
        const float* wr = win + (int)threadIdx.x + 0 * (off + ry * WIN + rx);
        const float t00 = wr[0], t01 = wr[256], t10 = wr[512], t11 = wr[768];
#else
        int r0, r1;  // row starts of the tap rows ry, ry + 1
        if constexpr (ROWT) {  // swizzled (lk_tb_row4), packed r0 | r1 << 7
          const int rp = ok ? ry : 0;
          r0 = rp & 127;
          r1 = rp >> 7;
        } else {
          r0 = ok ? ry * WIN : 0;
          r1 = ok ? (ry + 1) * WIN : 0;
        }
        const float* wr = sw + off + (ok ? rx : 0);
        const float t00 = wr[r0], t01 = wr[r0 + 1], t10 = wr[r1], t11 = wr[r1 + 1];
#endif
        const float ix_w = floorf(ix), ix_e = ix_w + 1.f;
        const float wxw = ix_e - ix, wxe = ix - ix_w;
        const float iy_n = floorf(iy), iy_s = iy_n + 1.f;
        const float wyn = iy_s - iy, wys = iy - iy_n;
        float v = 0.f;
        v += t00 * (wxw * wyn);
        v += t01 * (wxe * wyn);
        v += t10 * (wxw * wys);
        v += t11 * (wxe * wys);
        o[(size_t)(l * D * D + sidx) * ostep] = ok ? v : 0.f;
      }
    }
    if (stamps) {
      __builtin_amdgcn_s_waitcnt(0);
      stamp(4);
      stamp(5);
    }
    return;
  }
  float res[NPR][D];
#pragma unroll
  for (int q = 0; q < NPR; ++q) {
    const int t = gl + LK_GL * q;
    const bool tv = active && t < L * D;
    const int l = tv ? t / D : 0, a = tv ? t % D : 0;
    int off = offl[0], rows = rn[0] / WIN;
#pragma unroll
    for (int k = 1; k < LK_MAXL; ++k)
      if (l == k) { off = offl[k]; rows = rn[k] / WIN; }
    const int rx = sr[slot][l][0][a];
    const float ix = crd(slot, l, 0, a);
    int ry[D];
    float iy[D];
#pragma unroll
    for (int b = 0; b < D; ++b) {
      ry[b] = sr[slot][l][1][b];
      iy[b] = crd(slot, l, 1, b);
    }
    const bool okx = tv && rx >= 0 && rx + 1 < WIN;
    float t00[D], t01[D], t10[D], t11[D];
    bool ok[D];
#pragma unroll
    for (int b = 0; b < D; ++b) {
      ok[b] = okx && ry[b] >= 0 && ry[b] + 1 < rows;
      const float* wr = sw + off + (ok[b] ? ry[b] * WIN + rx : 0);
      t00[b] = wr[0];
      t01[b] = wr[1];
      t10[b] = wr[WIN];
      t11[b] = wr[WIN + 1];
    }
    const float ix_w = floorf(ix), ix_e = ix_w + 1.f;
    const float wxw = ix_e - ix, wxe = ix - ix_w;
#pragma unroll
    for (int b = 0; b < D; ++b) {
      const float iy_n = floorf(iy[b]), iy_s = iy_n + 1.f;
      const float wyn = iy_s - iy[b], wys = iy[b] - iy_n;
      float v = 0.f;
      v += t00[b] * (wxw * wyn);
      v += t01[b] * (wxe * wyn);
      v += t10[b] * (wxw * wys);
      v += t11[b] * (wxe * wys);
      res[q][b] = ok[b] ? v : 0.f;
    }
  }
  if (vec_out) {
    // channels-last with a 16-B aligned pixel stride: the pixel's L·D² outputs go through its
    // own LDS region (only its 16 lanes, one wave, read it) and out as 16-B stores
    __syncthreads();
    stamp(4);
#pragma unroll
    for (int q = 0; q < NPR; ++q) {
      const int t = gl + LK_GL * q;
      if (t < L * D) {
#pragma unroll
        for (int b = 0; b < D; ++b) sw[t * D + b] = res[q][b];
      }
    }
    __syncthreads();
    if (active) {
      float* o = out + (size_t)gp * out_stride;
      const int K4 = L * D * D / 4;
      for (int c = gl; c < K4; c += LK_GL) *(floatx4*)(o + 4 * c) = *(const floatx4*)(sw + 4 * c);
      for (int c = 4 * K4 + gl; c < L * D * D; c += LK_GL) o[c] = sw[c];
    }
    if (stamps) {
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
      stamp(5);
    }
    return;
  }
  if (!active) return;
  float* o = out_layout == SCFLOW_LAYOUT_NHWC ? out + ((size_t)n * P + p) * out_stride
                                              : out + (size_t)n * L * D * D * P + p;
  const int ostep = out_layout == SCFLOW_LAYOUT_NHWC ? 1 : P;
#pragma unroll
  for (int q = 0; q < NPR; ++q) {
    const int t = gl + LK_GL * q;
    if (t < L * D) {
#pragma unroll
      for (int b = 0; b < D; ++b) o[(size_t)(t * D + b) * ostep] = res[q][b];
    }
  }
}

}  // namespace

// profiling: where the next LDS-kernel launches write their phase stamps (NULL: off)
static unsigned long long* g_lk_stamps = nullptr;

// Tile regions (corr_lookup_lds_kernel TR) for the tiled r = 4 lookup when the feature map has at
// most 32×32 pixels: measured (tools/lookup_bench.py, tools/sess_lk.sh) 25.0 -> 23.1 us standalone
// and 34 -> 28 us inside the decoder at configs[1] (B=16, 32x32), but 165.6 -> 176.6 us at
// configs[4] (B=32, 64x64), where their 4 KB per pixel of LDS leaves 2 workgroups per CU instead
// of 3.  SCFLOW_LK_TILEREG=0 / 1 forces them off / on.
static bool lk_tile_regions(int h, int w) {
  static int v = -2;
  if (v == -2) {
    const char* e = getenv("SCFLOW_LK_TILEREG");
    v = e ? atoi(e) : -1;
  }
  return v < 0 ? (long long)h * w <= 32 * 32 : v != 0;
}

// TB tile-row regions for the tiled lookup on maps where the tile regions are off (round 5;
// SCFLOW_LK_TB=0 gives the b32-gather regions)
static bool lk_tile_rows() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("SCFLOW_LK_TB");
    v = e ? (atoi(e) != 0) : 1;
  }
  return v != 0;
}

static int corr_lookup_launch(const float* pyr, const float* flow, int flow_layout, float* out,
                              int out_layout, int out_stride, int n, int h, int w, int num_levels,
                              int radius, int align_corners, bool tiled, void* stream) {
  const int ac = align_corners ? 1 : 0;
  if (!pyr || !flow || !out || n <= 0 || h <= 0 || w <= 0 || num_levels < 1 || num_levels > 8 ||
      radius < 0)
    return SCFLOW_EINVAL;
  if (radius > 6) return SCFLOW_EUNSUPPORTED;
  const int K = num_levels * (2 * radius + 1) * (2 * radius + 1);
  if (out_layout == SCFLOW_LAYOUT_NHWC && out_stride < K) return SCFLOW_EINVAL;
  if (out_layout != SCFLOW_LAYOUT_NHWC && out_layout != SCFLOW_LAYOUT_NCHW) return SCFLOW_EINVAL;
  if ((h >> (num_levels - 1)) < 1 || (w >> (num_levels - 1)) < 1) return SCFLOW_EUNSUPPORTED;
  hipStream_t st = (hipStream_t)stream;
  // the LDS kernel addresses one wave's 4 pixel maps of a level through a buffer descriptor
  // (offsets < 2^31 bytes)
  // LDS kernel: a level's window holds D + 3 columns; without align_corners the samples are
  // size/(size−1) apart, which fits when every windowed level is ≥ 2r+1 wide and tall
  bool lds_ok = num_levels <= LK_MAXL && radius >= 1 && radius <= 4 &&
                (long long)LK_PPW * h * w * 4 < LK_OOB;
  if (lds_ok && !ac) {
    for (int l = 0; l < num_levels; ++l) {
      const int hl = h >> l, wl = w >> l;
      if (!lk_whole(hl, wl, 2 * radius + 4) && (hl < 2 * radius + 1 || wl < 2 * radius + 1)) lds_ok = false;
    }
  }
  if (tiled && (!lds_ok || (h >> (num_levels - 1)) % 4 || (w >> (num_levels - 1)) % 4))
    return SCFLOW_EUNSUPPORTED;
  if (lds_ok) {
    const unsigned blk = (unsigned)(((long long)n * h * w + LK_SLOTS - 1) / LK_SLOTS);
    const int D = 2 * radius + 1;
    const int sf = lk_slot_floats(h, w, num_levels, D + 3);
    const size_t lds = sizeof(float) * LK_SLOTS * sf;
    const int vec = out_layout == SCFLOW_LAYOUT_NHWC && out_stride % 4 == 0 &&
                    ((uintptr_t)out & 15) == 0 && sf >= num_levels * D * D;
#define SCFLOW_LKL(RR, TT)                                                                          \
  corr_lookup_lds_kernel<RR, TT><<<blk, 256, lds, st>>>(pyr, flow, flow_layout, out, out_layout,      \
                                                        out_stride, n, h, w, num_levels, vec, ac,  \
                                                        g_lk_stamps)
    if (tiled && radius == 4 && lk_tile_regions(h, w)) {
      const size_t lds_tr = sizeof(float) * LK_SLOTS * lk_tr_slot_floats(num_levels);
      corr_lookup_lds_kernel<4, true, true><<<blk, 256, lds_tr, st>>>(
          pyr, flow, flow_layout, out, out_layout, out_stride, n, h, w, num_levels, vec, ac, g_lk_stamps);
      return scflow_launch_status();
    }
    if (tiled && lk_tile_rows()) {
      const int sf_tb = lk_tb_slot_floats(h, w, num_levels, lk_win(radius, false, true));
      const size_t lds_tb = sizeof(float) * LK_SLOTS * sf_tb;
      const int vec_tb = vec || (out_layout == SCFLOW_LAYOUT_NHWC && out_stride % 4 == 0 &&
                                 ((uintptr_t)out & 15) == 0 && sf_tb >= num_levels * D * D);
      const int vtb = vec_tb && sf_tb >= num_levels * D * D;
      switch (radius) {
        case 1: corr_lookup_lds_kernel<1, true, false, true><<<blk, 256, lds_tb, st>>>(pyr, flow, flow_layout, out, out_layout, out_stride, n, h, w, num_levels, vtb, ac, g_lk_stamps); break;
        case 2: corr_lookup_lds_kernel<2, true, false, true><<<blk, 256, lds_tb, st>>>(pyr, flow, flow_layout, out, out_layout, out_stride, n, h, w, num_levels, vtb, ac, g_lk_stamps); break;
        case 3: corr_lookup_lds_kernel<3, true, false, true><<<blk, 256, lds_tb, st>>>(pyr, flow, flow_layout, out, out_layout, out_stride, n, h, w, num_levels, vtb, ac, g_lk_stamps); break;
        default: corr_lookup_lds_kernel<4, true, false, true><<<blk, 256, lds_tb, st>>>(pyr, flow, flow_layout, out, out_layout, out_stride, n, h, w, num_levels, vtb, ac, g_lk_stamps); break;
      }
      return scflow_launch_status();
    }
    switch (radius * 2 + (tiled ? 1 : 0)) {
      case 2: SCFLOW_LKL(1, false); break;
      case 3: SCFLOW_LKL(1, true); break;
      case 4: SCFLOW_LKL(2, false); break;
      case 5: SCFLOW_LKL(2, true); break;
      case 6: SCFLOW_LKL(3, false); break;
      case 7: SCFLOW_LKL(3, true); break;
      case 9: SCFLOW_LKL(4, true); break;
      default: SCFLOW_LKL(4, false); break;
    }
#undef SCFLOW_LKL
    return scflow_launch_status();
  }
  const long long total = (long long)n * h * w * num_levels * (2 * radius + 1);
  const int blocks = (int)((total + 255) / 256);
#define SCFLOW_LK(RR)                                                                            \
  case RR:                                                                                       \
    corr_lookup_kernel<RR><<<blocks, 256, 0, st>>>(pyr, flow, flow_layout, out, out_layout,      \
                                                   out_stride, n, h, w, num_levels, total, ac); \
    break;
  switch (radius) {
    SCFLOW_LK(0) SCFLOW_LK(1) SCFLOW_LK(2) SCFLOW_LK(3) SCFLOW_LK(4) SCFLOW_LK(5) SCFLOW_LK(6)
    default: return SCFLOW_EUNSUPPORTED;
  }
#undef SCFLOW_LK
  return scflow_launch_status();
}

SCFLOW_API int scflow_corr_lookup_ex(const float* pyr, const float* flow, int flow_layout, float* out,
                                     int out_layout, int out_stride, int n, int h, int w,
                                     int num_levels, int radius, int align_corners, void* stream) {
  return corr_lookup_launch(pyr, flow, flow_layout, out, out_layout, out_stride, n, h, w, num_levels,
                            radius, align_corners, false, stream);
}

SCFLOW_API int scflow_corr_lookup_tiled(const float* pyr, const float* flow, int flow_layout,
                                        float* out, int out_layout, int out_stride, int n, int h,
                                        int w, int num_levels, int radius, int align_corners,
                                        void* stream) {
  return corr_lookup_launch(pyr, flow, flow_layout, out, out_layout, out_stride, n, h, w, num_levels,
                            radius, align_corners, true, stream);
}

SCFLOW_API int scflow_corr_lookup(const float* pyr, const float* flow, int flow_layout, float* out,
                                  int out_layout, int out_stride, int n, int h, int w,
                                  int num_levels, int radius, void* stream) {
  return scflow_corr_lookup_ex(pyr, flow, flow_layout, out, out_layout, out_stride, n, h, w,
                               num_levels, radius, 1, stream);
}

// Profiling only: later LDS-kernel lookups write, per workgroup, 6 real-time-clock stamps
// (100 MHz) to `stamps` — start, coordinates done, window loads returned, windows in LDS,
// samples done, outputs stored (the last two with vec_out) — or stop (NULL).
SCFLOW_API int scflow_debug_lookup_stamps(void* stamps) {
  g_lk_stamps = (unsigned long long*)stamps;
  return SCFLOW_OK;
}
