// Winograd F(2×2, 3×3) weight gradient of a stride-1, pad-1 3×3 conv — included by train.hip
// (inside its anonymous namespace).  Training step only (SCFlowRefiner.loss → backward,
// scflow_refiner.py:182-256): the decoder's and encoders' 3×3 convs' dW.
//
// With the forward's transforms (Lavin & Gray; conv_wino.h) Y = Aᵀ[(G g Gᵀ) ⊙ (Bᵀ d B)]A per
// 2×2 output tile, the gradient of the transformed filter U = G g Gᵀ is, per transform point
// ξ = (i, j),
//     dU_ξ[co][ci] = Σ_tiles Ŷ_ξ[tile][co] · V_ξ[tile][ci],   Ŷ = A dY Aᵀ,  V = Bᵀ d B,
// and dW = Gᵀ dU G.  The 16 contractions over the tiles are fp32 MFMA GEMMs (M = co, N = ci,
// K = tiles): 16 products per 4 output pixels per (co, ci) instead of the direct 36 (2.25×
// fewer matrix operations than wgrad_kernel).
//
// Workgroup = 32 co × 64 ci, 8 waves: wave w owns the points (i = w & 3, 0..3) — 4 × 2
// accumulators of 32×32 (128 AGPRs) — for every other pair of k-steps (ks = w >> 2; two waves per
// SIMD, the two sets' sums added through LDS at the end).  The pixels are walked in chunks of 32
// tiles (4 output rows × 32 columns):
// the chunk's dY [4 rows][32 co][cols] and input halo [6 rows][64 ci][cols] are staged in LDS
// COLUMN-contiguous (transposing stores), so a lane reads its tile's two dY columns and its
// patch row's four input columns as 8-byte LDS reads; the next chunk's global loads are in
// flight in registers during this chunk's MFMAs.  Each wave computes its own row of Ŷ (2 + 2
// adds per tile pair) and of V (8 per 32 ci) on the fly.  Signs: row 3 of A and column 3 of
// Aᵀ are taken positive (Ŷ_{3,·}, Ŷ_{·,3} negated) and the reduction flips them back.
// The pixel reduction is split over the grid (fixed-order sum of the partial slabs
// [split][ξ][co][ci] in wwino_reduce_kernel, which also applies Gᵀ·G and writes torch's
// [co][ci][3][3] layout; deterministic).

constexpr int WWCO = 32;          // co per workgroup
constexpr int WWCI = 64;          // ci per workgroup
constexpr int WWD = 34;           // LDS row of dY: 32 columns + 2 pad (b64 reads conflict-free)
constexpr int WWX = 34;           // LDS row of the halo: 34 columns (4·34 ≡ 8 mod 64 banks: the
                                  // transposing stores of 16 channel quads spread over 8 banks)
constexpr int WWD_FL = 4 * WWCO * WWD;   // floats of the dY chunk
constexpr int WWX_FL = 6 * WWCI * WWX;   // floats of the halo chunk
constexpr int WW_NT = 512;        // threads
constexpr int WW_ND = 4 * 32 * (WWCO / 4) / WW_NT;                // dY float4 per thread (2)
constexpr int WW_NX = (6 * 34 * (WWCI / 4) + WW_NT - 1) / WW_NT;  // halo float4 per thread (7)

// XCD-aware (tile, split) of this workgroup on a grid of (tiles, splits): workgroups are dispatched
// round-robin over the 8 XCDs by linear id, so the ids are re-assigned such that all tiles of a
// split (which read the same dY / input chunks) run on one XCD and share its L2 — instead of
// every XCD fetching every chunk from HBM / MALL.  Identity when splits is not a multiple of 8.
__device__ __forceinline__ void wgrad_xcd_map(int tiles, int splits, int* tile, int* split) {
  if (splits % 8 == 0) {
    const int L = blockIdx.x + gridDim.x * blockIdx.y;
    const int xcd = L & 7, k = L >> 3;
    *split = (k / tiles) * 8 + xcd;
    *tile = k % tiles;
  } else {
    *tile = blockIdx.x;
    *split = blockIdx.y;
  }
}

struct WwParams {
  scflow_wgrad_args a;
  int cg, rg, nchunks, cps, co_tiles, copad, cinp;
  WgSegs sg;
};

// position of a chunk in the (segment, image, row group, column group) walk; consecutive chunks
// advance it by compares and increments (the static loops keep one per chunk instead of the four
// scalar integer divisions of a fresh lookup)
struct WgWalk {
  int seg, img, ry, cx;
};
__device__ __forceinline__ WgWalk wg_walk_at(int ch, int rg, int cg, int nimg) {
  WgWalk w;
  const int gi = ch / (rg * cg), rem = ch - gi * rg * cg;
  w.seg = gi / nimg;
  w.img = gi - w.seg * nimg;
  w.ry = rem / cg;
  w.cx = rem - w.ry * cg;
  return w;
}
__device__ __forceinline__ WgWalk wg_walk_next(WgWalk w, int rg, int cg, int nimg) {
  if (++w.cx == cg) {
    w.cx = 0;
    if (++w.ry == rg) {
      w.ry = 0;
      if (++w.img == nimg) {
        w.img = 0;
        ++w.seg;
      }
    }
  }
  return w;
}

typedef float floatx2w __attribute__((ext_vector_type(2)));

// one k-step's LDS operands before the transforms: dY rows 0, 1 of the tile pair and the halo
// rows r1, r2 (two 8-byte reads each) for both 32-ci blocks
struct WwRaw {
  floatx2w y0, y1, a0[2], a1[2], b0[2], b1[2];
};


__device__ const floatx4 ww_zero4 = {0.f, 0.f, 0.f, 0.f};  // source of the zero-padding lanes
// a float4 in the global address space: global_load (vmcnt only), not a flat load, which also
// counts in lgkmcnt and would make every LDS wait wait for it
typedef __attribute__((address_space(1))) floatx4 WwGlobal4;

// halo float4 slot j of thread tid: (pixel p of the 6 × 34 halo, first channel cq).  A wave-load
// covers 8 consecutive pixels × 8 channel quads (one 32-channel half, 128 B per pixel), so the
// transposing scalar LDS stores of a wave — bank (8·quad + 34·e + column) mod 64 — land on 64
// distinct banks (16 quads × 4 pixels per wave put two lanes on every bank)
__device__ __forceinline__ void ww_halo_slot(int tid, int j, int* p, int* cq) {
  const int b = (tid >> 6) + 8 * j, l = tid & 63;  // wave-load block b (0..55): 8 px × 8 quads
  *p = (b >> 1) * 8 + (l >> 3);
  *cq = 4 * ((b & 1) * 8 + (l & 7));
}

__global__ __launch_bounds__(WW_NT, 1) void wgrad_wino_kernel(WwParams P, float* __restrict__ slab,
                                                            float* __restrict__ bslab) {
  extern __shared__ float smem[];
  // two LDS buffers of [4][32 co][WWD] dY + [6][64 ci][WWX] halo: chunk c + 1 is stored while
  // the other waves still compute on chunk c (one barrier per chunk)
  constexpr int WBUF = WWD_FL + WWX_FL;
  float* Dl = smem;            // current chunk's dY
  float* Xl = smem + WWD_FL;   // current chunk's halo
  const scflow_wgrad_args& a = P.a;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wave = wv & 3, ks = wv >> 2;  // Winograd row i, k-step set
  const int li = lane & 31, hh = lane >> 5;
  int tile, split;
  wgrad_xcd_map(gridDim.x, gridDim.y, &tile, &split);
  const int co_t = tile % P.co_tiles, ci_t = tile / P.co_tiles;
  const int co0 = co_t * WWCO, ci0 = ci_t * WWCI;
  const int cin = a.cin0 + a.cin1;
  const int c_begin = split * P.cps;
  const int c_end = min(P.nchunks, c_begin + P.cps);
  const bool do_bias = bslab != nullptr && ci_t == 0;

  floatx4 rd[WW_ND], rx[WW_NX];
  auto origin = [&](int ch, int* img, int* oy0, int* ox0) {
    *img = ch / (P.rg * P.cg);
    const int rem = ch - *img * P.rg * P.cg;
    *oy0 = (rem / P.cg) * 4;
    *ox0 = (rem % P.cg) * 32;
  };
  auto gload = [&](int ch) {
    int img, oy0, ox0;
    origin(ch, &img, &oy0, &ox0);
    const int seg = img / P.sg.nimg;  // workgroup-uniform
    img -= seg * P.sg.nimg;
    const float* dyp = P.sg.dy[seg];
    const float* s0p = P.sg.src0[seg];
    const float* s1p = P.sg.src1[seg];
#pragma unroll
    for (int j = 0; j < WW_ND; ++j) {  // dY: 128 pixels × 8 co quads
      const int idx = tid + WW_NT * j;
      const int p = idx >> 3, co = co0 + 4 * (idx & 7);
      floatx4 v = {0.f, 0.f, 0.f, 0.f};
      if (co < a.cout) {
        const size_t m = ((size_t)img * a.h + oy0 + (p >> 5)) * a.w + ox0 + (p & 31);
        v = *(const floatx4*)(dyp + m * a.sdy + co);
      }
      rd[j] = v;
    }
#pragma unroll
    for (int j = 0; j < WW_NX; ++j) {  // halo: 6 × 34 pixels × 16 ci quads (ww_halo_slot)
      int p, cq;
      ww_halo_slot(tid, j, &p, &cq);
      const int c = ci0 + cq;
      floatx4 v = {0.f, 0.f, 0.f, 0.f};
      if (p < 6 * 34 && c < cin) {
        const int hr = p / 34, hc = p - hr * 34;
        const int iy = oy0 - 1 + hr, ix = ox0 - 1 + hc;
        if (iy >= 0 && iy < a.h && ix >= 0 && ix < a.w) {
          const size_t pix = ((size_t)img * a.h + iy) * a.w + ix;
          v = c < a.cin0 ? *(const floatx4*)(s0p + pix * a.s0 + c)
                         : *(const floatx4*)(s1p + pix * a.s1 + (c - a.cin0));
        }
      }
      rx[j] = v;
    }
  };
  auto lstore = [&](int buf) {  // transposing stores: channel-major rows, columns contiguous
    float* Dw = smem + buf * WBUF;
    float* Xw = Dw + WWD_FL;
#pragma unroll
    for (int j = 0; j < WW_ND; ++j) {
      const int idx = tid + WW_NT * j;
      const int p = idx >> 3, cq = 4 * (idx & 7);
      float* d = Dw + ((p >> 5) * WWCO + cq) * WWD + (p & 31);
#pragma unroll
      for (int e = 0; e < 4; ++e) d[e * WWD] = rd[j][e];
    }
#pragma unroll
    for (int j = 0; j < WW_NX; ++j) {
      int p, cq;
      ww_halo_slot(tid, j, &p, &cq);
      if (p < 6 * 34) {
        const int hr = p / 34, hc = p - hr * 34;
        float* d = Xw + (hr * WWCI + cq) * WWX + hc;
#pragma unroll
        for (int e = 0; e < 4; ++e) d[e * WWX] = rx[j][e];
      }
    }
  };

  floatx16 acc[4][2];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[j][cb][e] = 0.f;
  float bsum = 0.f;

  // this wave's rows: Bᵀ row i = d[r1] + s·d[r2]; A row i (row 3 taken positive)
  const int r1 = wave == 0 ? 0 : (wave == 2 ? 2 : 1);
  const int r2 = wave == 0 ? 2 : (wave == 1 ? 2 : (wave == 2 ? 1 : 3));
  const float sb = wave == 1 ? 1.f : -1.f;
  const float ya = wave == 3 ? 0.f : 1.f;                       // weight of dY row 0
  const float yb = wave == 0 ? 0.f : (wave == 2 ? -1.f : 1.f);  // weight of dY row 1

  // a k-step's operands in two halves: the raw LDS reads, then the arithmetic
  // step st of this wave: tile row st >> 2, tile column 4·ks + hh + 8·((st >> 1) & 1) + 2·(st & 1)
  // — per-thread bases plus compile-time offsets once unrolled (ds_read offset fields)
  const int tc0 = 4 * ks + hh;
  auto rawload = [&](int st, WwRaw& r) __attribute__((always_inline)) {
    const int ttr = st >> 2, co2 = 2 * (8 * ((st >> 1) & 1) + 2 * (st & 1));
    const float* db = Dl + li * WWD + 2 * tc0 + co2;
    r.y0 = *(const floatx2w*)(db + (2 * ttr) * WWCO * WWD);
    r.y1 = *(const floatx2w*)(db + (2 * ttr + 1) * WWCO * WWD);
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      const float* xb = Xl + (cb * 32 + li) * WWX + 2 * tc0 + co2;
      r.a0[cb] = *(const floatx2w*)(xb + (2 * ttr + r1) * WWCI * WWX);
      r.a1[cb] = *(const floatx2w*)(xb + (2 * ttr + r1) * WWCI * WWX + 2);
      r.b0[cb] = *(const floatx2w*)(xb + (2 * ttr + r2) * WWCI * WWX);
      r.b1[cb] = *(const floatx2w*)(xb + (2 * ttr + r2) * WWCI * WWX + 2);
    }
  };
  auto xform = [&](const WwRaw& r, float (&yv)[4], float (&vv)[2][4]) __attribute__((always_inline)) {
    const float q0 = ya * r.y0[0] + yb * r.y1[0], q1 = ya * r.y0[1] + yb * r.y1[1];
    yv[0] = q0;
    yv[1] = q0 + q1;
    yv[2] = q0 - q1;
    yv[3] = q1;
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      const float t0 = r.a0[cb][0] + sb * r.b0[cb][0], t1 = r.a0[cb][1] + sb * r.b0[cb][1];
      const float t2 = r.a1[cb][0] + sb * r.b1[cb][0], t3 = r.a1[cb][1] + sb * r.b1[cb][1];
      vv[cb][0] = t0 - t2;
      vv[cb][1] = t1 + t2;
      vv[cb][2] = t2 - t1;
      vv[cb][3] = t1 - t3;
    }
  };
  (void)rawload;
  (void)xform;

  // the next chunk's global loads in three pieces issued inside steps 0..2 of this chunk (their
  // address arithmetic in the MFMA shadow): every lane loads unconditionally — from ww_zero4
  // where the old code branched around the load (padding, channels beyond cout / cin)
  struct Gsrc {
    const float *dy, *s0, *s1;
    int oy0, ox0;
  };
  auto gsetup = [&](const WgWalk& w) __attribute__((always_inline)) {
    const size_t ipx = (size_t)w.img * a.h * a.w;
    return Gsrc{wg_pick(P.sg.dy, w.seg) + ipx * a.sdy, wg_pick(P.sg.src0, w.seg) + ipx * a.s0,
                wg_pick(P.sg.src1, w.seg) + ipx * a.s1, 4 * w.ry, 32 * w.cx};
  };
  auto gpiece = [&](const Gsrc& g, int part) __attribute__((always_inline)) {
    if (part == 0) {
#pragma unroll
      for (int j = 0; j < WW_ND; ++j) {
        const int idx = tid + WW_NT * j;
        const int p = idx >> 3, co = co0 + 4 * (idx & 7);
        const float* src = g.dy + ((size_t)(g.oy0 + (p >> 5)) * a.w + g.ox0 + (p & 31)) * a.sdy + co;
        rd[j] = *(const WwGlobal4*)(co < a.cout ? src : (const float*)&ww_zero4);
      }
    }
    const int j0 = part == 0 ? 0 : (part == 1 ? 1 : 4), j1 = part == 0 ? 1 : (part == 1 ? 4 : WW_NX);
#pragma unroll
    for (int j = j0; j < j1; ++j) {
      int p, cq;
      ww_halo_slot(tid, j, &p, &cq);
      const int c = ci0 + cq;
      const int hr = p / 34, hc = p - hr * 34;
      const int iy = g.oy0 - 1 + hr, ix = g.ox0 - 1 + hc;
      const bool ok = p < 6 * 34 && c < cin && iy >= 0 && iy < a.h && ix >= 0 && ix < a.w;
      const size_t pix = (size_t)iy * a.w + ix;
      const float* src = c < a.cin0 ? g.s0 + pix * a.s0 + c : g.s1 + pix * a.s1 + (c - a.cin0);
      rx[j] = *(const WwGlobal4*)(ok ? src : (const float*)&ww_zero4);
    }
  };

  if (c_begin < c_end) {
    gload(c_begin);
    lstore(0);
    __syncthreads();
  }
  WgWalk wk = wg_walk_at(c_begin, P.rg, P.cg, P.sg.nimg);
  for (int ch = c_begin; ch < c_end; ++ch) {
    const int cur = (ch - c_begin) & 1;
    Dl = smem + cur * WBUF;
    Xl = Dl + WWD_FL;
    if (do_bias) {  // Σ dY per channel: thread (co = tid & 31) over every 16th pixel
      const int co = tid & 31;
      for (int p = tid >> 5; p < 128; p += WW_NT / 32) bsum += Dl[((p >> 5) * WWCO + co) * WWD + (p & 31)];
    }
    // the wave's 8 k-steps s (kk = 2·ks + 4·(s >> 1) + (s & 1)) as straight-line code: step s
    // issues step s + 1's LDS reads, then its own 8 MFMAs with step s + 1's operand arithmetic
    // interleaved from the fourth MFMA on (by then the reads have landed) — no LDS wait in front
    // of an MFMA, and no exposed read latency
    WwRaw raw;
    float yv[2][4], vv[2][2][4];
    rawload(0, raw);
    xform(raw, yv[0], vv[0]);
    if (ch + 1 < c_end) wk = wg_walk_next(wk, P.rg, P.cg, P.sg.nimg);  // (the last reloads itself)
    const Gsrc gn = gsetup(wk);
    auto step = [&](auto sc) __attribute__((always_inline)) {
      constexpr int st = decltype(sc)::value, cu = st & 1, nx = (st + 1) & 1;
      if constexpr (st < 3) gpiece(gn, st);
      if constexpr (st + 1 < 8) rawload(st + 1, raw);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
          acc[j][cb] = __builtin_amdgcn_mfma_f32_32x32x2f32(yv[cu][j], vv[cu][cb][j], acc[j][cb], 0, 0, 0);
      if constexpr (st + 1 < 8) {
        xform(raw, yv[nx], vv[nx]);
        __builtin_amdgcn_sched_group_barrier(0x100, 10, 0);  // the DS reads
        __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);   // three MFMAs
#pragma unroll
        for (int m = 0; m < 5; ++m) {
          __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);  // five VALU
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one MFMA
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    };
    StaticFor<0, 8>::run(step);
    if (ch + 1 < c_end) {
      lstore(cur ^ 1);
      __syncthreads();
    }
  }
  // the second k-step set's sums onto the first's
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      __syncthreads();
      if (ks == 1)
#pragma unroll
        for (int r = 0; r < 16; ++r) smem[r * 256 + (tid - 256)] = acc[j][cb][r];
      __syncthreads();
      if (ks == 0)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][cb][r] += smem[r * 256 + tid];
    }
  // partial slab [split][ξ = 4i + j][copad][cinp]; C/D layout: col = lane&31, row = (r&3)+8(r>>2)+4hh
  const size_t plane = (size_t)P.copad * P.cinp;
  float* sl = slab + (size_t)split * 16 * plane;
  if (ks == 0)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        float* sp = sl + (size_t)(4 * wave + j) * plane + ci0 + cb * 32 + li;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int co = co0 + (r & 3) + 8 * (r >> 2) + 4 * hh;
          sp[(size_t)co * P.cinp] = acc[j][cb][r];
        }
      }
  if (do_bias) {
    __syncthreads();
    smem[tid] = bsum;
    __syncthreads();
    if (tid < WWCO) {
      float b = 0.f;
#pragma unroll
      for (int g = 0; g < WW_NT / 32; ++g) b += smem[tid + 32 * g];
      bslab[(size_t)split * P.copad + co0 + tid] = b;
    }
  }
}

// Σ over the splits (fixed order: 4 lanes of partial sums per output, then in order through
// LDS), the sign flips of row / column 3, dW = Gᵀ dU G, torch layout [co][ci][3][3] (+= when
// accumulating).  Workgroup = 64 ci of one co × 4 split lanes; the bias rides in extra blocks.
__global__ __launch_bounds__(256) void wwino_reduce_kernel(
    const float* __restrict__ slab, const float* __restrict__ bslab, float* __restrict__ dw,
    float* __restrict__ db, int splits, int cout, int cin, int copad, int cinp, int accumulate) {
  __shared__ float part[4][16][65];
  const int cblocks = cinp / 64;
  const int nw = cout * cblocks;
  const int o = threadIdx.x & 63, k = threadIdx.x >> 6;
  if ((int)blockIdx.x >= nw) {  // bias: channels (blockIdx.x − nw)·256 + tid, summed in order
    const int c = (blockIdx.x - nw) * 256 + threadIdx.x;
    if (c < cout) {
      float s = 0.f;
      for (int sp = 0; sp < splits; ++sp) s += bslab[(size_t)sp * copad + c];
      db[c] = accumulate ? db[c] + s : s;
    }
    return;
  }
  const int co = blockIdx.x / cblocks, ci = (blockIdx.x % cblocks) * 64 + o;
  const size_t plane = (size_t)copad * cinp;
  float s[16];
#pragma unroll
  for (int x = 0; x < 16; ++x) s[x] = 0.f;
  for (int sp = k; sp < splits; sp += 4) {
    const float* src = slab + (size_t)sp * 16 * plane + (size_t)co * cinp + ci;
#pragma unroll
    for (int x = 0; x < 16; ++x) s[x] += src[x * plane];
  }
#pragma unroll
  for (int x = 0; x < 16; ++x) part[k][x][o] = s[x];
  __syncthreads();
  if (k != 0 || ci >= cin) return;
  float u[4][4];
#pragma unroll
  for (int x = 0; x < 16; ++x) {
    const float v = (part[0][x][o] + part[1][x][o]) + (part[2][x][o] + part[3][x][o]);
    const int i = x >> 2, j = x & 3;
    u[i][j] = ((i == 3) != (j == 3)) ? -v : v;
  }
  float t[4][3];
#pragma unroll
  for (int i = 0; i < 4; ++i) {  // T = dU·G
    t[i][0] = u[i][0] + 0.5f * (u[i][1] + u[i][2]);
    t[i][1] = 0.5f * (u[i][1] - u[i][2]);
    t[i][2] = 0.5f * (u[i][1] + u[i][2]) + u[i][3];
  }
  float* d = dw + ((size_t)co * cin + ci) * 9;
#pragma unroll
  for (int q = 0; q < 3; ++q) {  // dW = Gᵀ·T
    const float w0 = t[0][q] + 0.5f * (t[1][q] + t[2][q]);
    const float w1 = 0.5f * (t[1][q] - t[2][q]);
    const float w2 = 0.5f * (t[1][q] + t[2][q]) + t[3][q];
    d[0 * 3 + q] = accumulate ? d[0 * 3 + q] + w0 : w0;
    d[1 * 3 + q] = accumulate ? d[1 * 3 + q] + w1 : w1;
    d[2 * 3 + q] = accumulate ? d[2 * 3 + q] + w2 : w2;
  }
}

// shapes: 3×3, stride 1, pad 1, h % 4 == 0, w % 32 == 0, float4-aligned channel groups
bool wwino_geometry(const scflow_wgrad_args& a, WwParams* P) {
  static const int off = [] {
    const char* e = getenv("SCFLOW_WGRAD_WINO");
    return e && e[0] == '0';
  }();
  if (off) return false;
  const int cin = a.cin0 + a.cin1;
  if (a.kh != 3 || a.kw != 3 || a.stride != 1 || a.ph != 1 || a.pw != 1) return false;
  if (a.h % 4 || a.w % 32) return false;
  if (a.cout % 4 || a.sdy % 4 || !aligned16(a.dy) || a.cin0 % 4 || a.s0 % 4 || !aligned16(a.src0) ||
      (a.cin1 > 0 && (a.cin1 % 4 || a.s1 % 4 || !aligned16(a.src1))))
    return false;
  if (a.cout < 64 || cin < 16) return false;  // narrow shapes: wthin / wgrad_kernel (measured)
  P->a = a;
  P->cg = a.w / 32;
  P->rg = a.h / 4;
  P->nchunks = a.n * P->rg * P->cg;
  P->co_tiles = (a.cout + WWCO - 1) / WWCO;
  P->copad = P->co_tiles * WWCO;
  P->cinp = (cin + WWCI - 1) / WWCI * WWCI;
  const int tiles = P->co_tiles * (P->cinp / WWCI);
  // one workgroup per CU; the partial slabs (16 planes per split) stay under 32 Mi floats
  // (rounded down: a partial second round of workgroups costs a whole chunk loop)
  long long want = (long long)device_cus() / tiles;
  const long long cap = (32LL << 20) / (16LL * P->copad * P->cinp);
  if (want > cap) want = cap;
  if (want > P->nchunks) want = P->nchunks;
  if (want < 1) want = 1;
  P->cps = (int)((P->nchunks + want - 1) / want);
  return true;
}

int wwino_splits(const WwParams& P) { return (P.nchunks + P.cps - 1) / P.cps; }

long long wwino_workspace(const WwParams& P) {
  const long long s = wwino_splits(P);
  return s * 16 * P.copad * P.cinp + s * P.copad;
}

int wwino_launch(const WwParams& P, hipStream_t st) {
  const scflow_wgrad_args& a = P.a;
  const int splits = wwino_splits(P);
  float* slab = a.workspace;
  float* bslab = a.db ? a.workspace + (size_t)splits * 16 * P.copad * P.cinp : nullptr;
  const size_t lds = sizeof(float) * (size_t)(2 * (WWD_FL + WWX_FL));
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)wgrad_wino_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  const dim3 grid((unsigned)(P.co_tiles * (P.cinp / WWCI)), (unsigned)splits);
  wgrad_wino_kernel<<<grid, WW_NT, lds, st>>>(P, slab, bslab);
  int rc = scflow_launch_status();
  if (rc != SCFLOW_OK) return rc;
  const int cin = a.cin0 + a.cin1;
  const unsigned rblocks = (unsigned)(a.cout * (P.cinp / 64) + (a.db ? (a.cout + 255) / 256 : 0));
  wwino_reduce_kernel<<<rblocks, 256, 0, st>>>(slab, bslab, a.dw, a.db, splits, a.cout, cin,
                                               P.copad, P.cinp, a.accumulate);
  return scflow_launch_status();
}
