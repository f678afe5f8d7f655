// Winograd F(4, 5) weight gradient of the SeqConv GRU's 1×5 / 5×1 convs (stride 1, pad 2 along
// the conv axis) — included by train.hip (inside its anonymous namespace).  Training step only: the GRU's dW, 8 launches per
// step per conv (raft_decoder.py:235-253 under SCFlowRefiner.loss → backward,
// scflow_refiner.py:182-256), plus the hoisted context part once.
//
// With the forward's transforms (conv_wino5.h) y = Aᵀ[(G g) ⊙ (Bᵀ d)] per tile of 4 output
// pixels along the conv axis (8 inputs d), the gradient of the transformed filter U_ξ at each of
// the 8 points ξ is
//     dU_ξ[co][ci] = Σ_tiles Ŷ_ξ[tile][co] · V_ξ[tile][ci],   Ŷ = A dY (the tile's 4 dY),  V = Bᵀ d,
// and dW = Gᵀ dU: 8 matrix products per 4 output pixels per (co, ci) instead of the direct 20
// (2.5× less matrix work than wgrad_kernel<1,5> / <5,1>).
//
// Workgroup = 64 co × 64 ci, 8 waves.  Wave w & 3 owns the point pair of conv_wino5.h:
// (1,2), (3,4), (5,6) — whose Ŷ rows are e ± o (e = dy0 + s2·dy2, o = s1·dy1 + s3·dy3 from the
// columns of Aᵀ) and whose V rows are b ± a (the forward's odd / even tap sums) — and (0, 7);
// 2 points × 2 co blocks × 2 ci blocks = 8 accumulators of 32×32 (128 AGPRs).  w >> 2 picks
// every other pair of k-steps (two wave sets; their sums added through LDS at the end).  The
// pixels are walked in chunks of 4 output rows × 32 columns = 32 tiles, 8 per row, the conv axis
// along the columns — a 5×1 conv is walked as the 1×5 conv of the transposed image (swapped pixel
// strides; the loads are channel-contiguous either way).  The chunk's dY and input halo sit in
// LDS as rows of 36 floats per channel (conflict-free b128 for 16 consecutive channels), so a
// lane reads its tile's 4 dY as one b128 and its 8 inputs as two; they are written the same way,
// one b128 per lane of 4 pixels of its channel.  One LDS buffer; the next chunk's global loads
// are in flight in registers during this chunk's MFMAs.
// Partial sums per split land in [split][ξ][copad][cinp]; wwino5_reduce_kernel sums the splits
// in a fixed order and applies Gᵀ (deterministic).

#include <type_traits>

constexpr int W5W_CO = 64;    // co per workgroup
constexpr int W5W_CI = 64;    // ci per workgroup
constexpr int W5W_NT = 512;   // threads
constexpr int W5W_RW = 36;    // 1×5: LDS row (floats) of one channel: 32 dY columns + 4 pad / 36 halo columns

// the transform point held in slot x (0, 1) of wave w (the pairing of conv_wino5.h's w5_point)
__host__ __device__ constexpr int w5w_point(int w, int x) {
  return w == 3 ? (x == 0 ? 0 : 7) : 2 * w + 1 + x;
}

// LDS layout (the conv axis runs along the chunk's columns: a 5×1 conv is walked as the 1×5 conv
// of the transposed image, through the pixel strides)
constexpr int W5W_DFL = 4 * W5W_CO * W5W_RW;   // dY: [4 rows][64 co][36]
constexpr int W5W_XFL = 4 * W5W_CI * W5W_RW;   // halo: [4 rows][64 ci][36 columns]
constexpr int W5W_ND = 4;                      // 4-pixel dY groups per lane per chunk (32 / 8 waves)
constexpr int W5W_NX = 5;                      // halo groups (4 rows × 9) per lane (36 / 8 waves)
__device__ __forceinline__ int w5w_addr(int r, int c, int ch) { return (r * 64 + ch) * W5W_RW + c; }


struct W5wParams {
  scflow_wgrad_args a;
  int H, W;        // the walked image: 1×5 (h, w); 5×1 the transpose (w, h)
  long long sy, sx;  // pixel strides of its rows / columns: (w, 1) or (1, w)
  int cg, rg, nchunks, cps, co_tiles, copad, cinp;
  WgSegs sg;       // segments (wgrad_wino.h)
};

__global__ __launch_bounds__(W5W_NT, 1) void wgrad_wino5_kernel(W5wParams P, float* __restrict__ slab,
                                                              float* __restrict__ bslab) {
  extern __shared__ float smem[];
  float* Dl = smem;
  float* Xl = smem + W5W_DFL;
  const scflow_wgrad_args& a = P.a;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wave = wv & 3, ks = wv >> 2;  // point pair, k-step set
  const int li = lane & 31, hh = lane >> 5;
  int tile, split;
  wgrad_xcd_map(gridDim.x, gridDim.y, &tile, &split);  // the split's tiles share one XCD's L2
  const int co_t = tile % P.co_tiles, ci_t = tile / P.co_tiles;
  const int co0 = co_t * W5W_CO, ci0 = ci_t * W5W_CI;
  const int cin = a.cin0 + a.cin1;
  const int c_begin = split * P.cps;
  const int c_end = min(P.nchunks, c_begin + P.cps);
  const bool do_bias = bslab != nullptr && ci_t == 0;

  // Global → register → LDS staging, channel per lane: a lane holds 4 pixels along the conv axis
  // of one channel (4 coalesced 4-byte loads: the wave's 64 lanes read 64 consecutive channels of
  // one pixel) and stores them as one b128 — consecutive lanes write consecutive / 36-float-strided
  // float4, free of bank conflicts (float4 channel loads with transposing scalar stores were
  // 60-80 % bank-conflict cycles).
  const int cl = tid & 63;  // this lane's channel in the workgroup's co / ci block
  floatx4 rd[W5W_ND], rx[W5W_NX];
  auto pix = [&](int img, int y, int x) __attribute__((always_inline)) {
    return (size_t)img * P.H * P.W + (size_t)y * P.sy + (size_t)x * P.sx;
  };
  floatx16 acc[2][2][2];  // [point slot][co block][ci block]
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int ib = 0; ib < 2; ++ib)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[x][cb][ib][e] = 0.f;
  float bsum = 0.f;

  // this wave's rows: Ŷ = e ± o with e = dy0 + s2·dy2, o = s1·dy1 + s3·dy3 (waves 0-2), (dy0, dy3)
  // for wave 3; V = b ± a as in the forward (conv_wino5.h)
  const float s1 = wave == 0 ? 1.f : (wave == 1 ? 2.f : 0.5f);
  const float s2 = wave == 0 ? 1.f : (wave == 1 ? 4.f : 0.25f);
  const float s3 = wave == 0 ? 1.f : (wave == 1 ? 8.f : 0.125f);
  const float c1 = wave == 0 ? 1.f : (wave == 1 ? 0.5f : 2.f);
  const float c3 = wave == 0 ? -4.25f : -2.5f;
  const float c5 = wave == 0 ? 1.f : (wave == 1 ? 2.f : 0.5f);
  const float c2 = wave == 0 ? 1.f : (wave == 1 ? 0.25f : 4.f);
  const float c4 = wave == 0 ? -4.25f : (wave == 1 ? -1.25f : -5.f);
  const bool w3 = wave == 3;  // wave-uniform

  auto mfmas = [&](const float (&yv)[2][2], const float (&vv)[2][2]) __attribute__((always_inline)) {
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int ib = 0; ib < 2; ++ib)
          acc[x][cb][ib] = __builtin_amdgcn_mfma_f32_32x32x2f32(yv[x][cb], vv[x][ib], acc[x][cb][ib], 0, 0, 0);
  };

  // Static form: two LDS buffers (one barrier per chunk); the next chunk's loads go out in five
  // pieces inside steps 0..4 (branch-free: lanes outside the data load ww_zero4), the wave's 8
  // k-steps st (kk = 2·ks + 4·(st >> 1) + (st & 1): tile row st >> 1, first column
  // 4·(4ks + hh) + 8·(st & 1)) as straight-line code — step st issues step st + 1's LDS reads, then
  // its MFMAs with step st + 1's operand arithmetic interleaved
  struct Gsrc {
    const float *dy, *src;
    int ss, oy0, ox0, img;
  };
  auto gsetup = [&](const WgWalk& w) __attribute__((always_inline)) {
    const int c = ci0 + cl;
    const float* s0 = wg_pick(P.sg.src0, w.seg);
    const float* s1 = wg_pick(P.sg.src1, w.seg);
    return Gsrc{wg_pick(P.sg.dy, w.seg), c < a.cin0 ? s0 + c : s1 + (c - a.cin0),
                c < a.cin0 ? a.s0 : a.s1, 4 * w.ry, 32 * w.cx, w.img};
  };
  typedef __attribute__((address_space(1))) float G1;
  auto gpiece = [&](const Gsrc& g, int part) __attribute__((always_inline)) {
    const float* zero = (const float*)&ww_zero4;
    if (part < 2) {
      const int co = co0 + cl;
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {  // dY: row q >> 3, columns 4(q & 7) + k
        const int j = 2 * part + jj, q = wv + 8 * j;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float* p = g.dy + pix(g.img, g.oy0 + (q >> 3), g.ox0 + 4 * (q & 7) + k) * a.sdy + co;
          rd[j][k] = *(const G1*)(co < a.cout ? p : zero);
        }
      }
      return;
    }
    const bool cok = ci0 + cl < cin;
    const int j0 = part == 2 ? 0 : (part == 3 ? 2 : 4), j1 = part == 2 ? 2 : (part == 3 ? 4 : 5);
#pragma unroll
    for (int j = j0; j < j1; ++j) {  // halo: row q / 9, columns x = ox0 − 2 + 4(q % 9) + k
      const int q = wv + 8 * j;
      const int y = g.oy0 + q / 9;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int x = g.ox0 - 2 + 4 * (q % 9) + k;
        const bool ok = q < 36 && cok && x >= 0 && x < P.W;
        const float* p = g.src + pix(g.img, y, x) * g.ss;
        rx[j][k] = *(const G1*)(ok ? p : zero);
      }
    }
  };
  auto lstore2 = [&](float* D, float* X) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < W5W_ND; ++j) {
      const int q = wv + 8 * j;
      *(floatx4*)(D + w5w_addr(q >> 3, 4 * (q & 7), cl)) = rd[j];
    }
#pragma unroll
    for (int j = 0; j < W5W_NX; ++j) {
      const int q = wv + 8 * j;
      if (q < 36) *(floatx4*)(X + w5w_addr(q / 9, 4 * (q % 9), cl)) = rx[j];
    }
  };
  struct Raw5 {
    floatx4 d[2], x0[2], x1[2];
  };
  const int cc0 = 4 * (4 * ks + hh);
  auto rawload = [&](int st, Raw5& r) __attribute__((always_inline)) {
    const int rr = st >> 1, c = cc0 + 8 * (st & 1);
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) r.d[cb] = *(const floatx4*)(Dl + w5w_addr(rr, c, cb * 32 + li));
#pragma unroll
    for (int ib = 0; ib < 2; ++ib) {
      r.x0[ib] = *(const floatx4*)(Xl + w5w_addr(rr, c, ib * 32 + li));
      r.x1[ib] = *(const floatx4*)(Xl + w5w_addr(rr, c + 4, ib * 32 + li));
    }
  };
  auto xform = [&](const Raw5& r, float (&yv)[2][2], float (&vv)[2][2], auto W3)
                   __attribute__((always_inline)) {
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      const floatx4 d = r.d[cb];
      if constexpr (decltype(W3)::value) {
        yv[0][cb] = d[0];
        yv[1][cb] = d[3];
      } else {
        const float e = d[0] + s2 * d[2], o = s1 * d[1] + s3 * d[3];
        yv[0][cb] = e + o;
        yv[1][cb] = e - o;
      }
    }
#pragma unroll
    for (int ib = 0; ib < 2; ++ib) {
      const floatx4 x0 = r.x0[ib], x1 = r.x1[ib];
      if constexpr (decltype(W3)::value) {
        vv[0][ib] = (x1[2] - x0[0]) + 5.25f * (x0[2] - x1[0]);
        vv[1][ib] = (x1[3] - x0[1]) + 5.25f * (x0[3] - x1[1]);
      } else {
        const float av = c1 * x0[1] + c3 * x0[3] + c5 * x1[1];
        const float bv = c2 * x0[2] + c4 * x1[0] + x1[2];
        vv[0][ib] = bv + av;
        vv[1][ib] = bv - av;
      }
    }
  };
  auto mainloop = [&](auto W3) __attribute__((always_inline)) {
    constexpr int BUF = W5W_DFL + W5W_XFL;
    WgWalk wk = wg_walk_at(c_begin, P.rg, P.cg, P.sg.nimg);
    if (c_begin < c_end) {
      const Gsrc g0 = gsetup(wk);
#pragma unroll
      for (int part = 0; part < 5; ++part) gpiece(g0, part);
      lstore2(smem, smem + W5W_DFL);
      __syncthreads();
    }
    for (int ch = c_begin; ch < c_end; ++ch) {
      const int cur = (ch - c_begin) & 1;
      Dl = smem + cur * BUF;
      Xl = Dl + W5W_DFL;
      if (do_bias) {  // Σ dY per channel: thread (co = tid & 63) over every 8th pixel
        const int co = tid & 63;
        for (int p = tid >> 6; p < 128; p += W5W_NT / 64) bsum += Dl[w5w_addr(p >> 5, p & 31, co)];
      }
      if (ch + 1 < c_end) wk = wg_walk_next(wk, P.rg, P.cg, P.sg.nimg);  // (the last reloads itself)
      const Gsrc gn = gsetup(wk);
      Raw5 raw;
      float yv[2][2][2], vv[2][2][2];
      rawload(0, raw);
      xform(raw, yv[0], vv[0], W3);
      auto step = [&](auto sc) __attribute__((always_inline)) {
        constexpr int st = decltype(sc)::value, cu = st & 1, nx = (st + 1) & 1;
        if constexpr (st < 5) gpiece(gn, st);
        if constexpr (st + 1 < 8) rawload(st + 1, raw);
        mfmas(yv[cu], vv[cu]);
        if constexpr (st + 1 < 8) {
          xform(raw, yv[nx], vv[nx], W3);
          __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);  // the DS reads
          __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);  // three MFMAs
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
        lstore2(smem + (cur ^ 1) * BUF, smem + (cur ^ 1) * BUF + W5W_DFL);
        __syncthreads();
      }
    }
  };
  if (w3)
    mainloop(std::true_type{});
  else
    mainloop(std::false_type{});
  // the second k-step set's sums onto the first's
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int ib = 0; ib < 2; ++ib) {
        __syncthreads();
        if (ks == 1)
#pragma unroll
          for (int r = 0; r < 16; ++r) smem[r * 256 + (tid - 256)] = acc[x][cb][ib][r];
        __syncthreads();
        if (ks == 0)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[x][cb][ib][r] += smem[r * 256 + tid];
      }
  // partial slab [split][ξ][copad][cinp]; C/D layout: col = lane & 31 (ci), row (co) =
  // (r & 3) + 8(r >> 2) + 4hh
  const size_t plane = (size_t)P.copad * P.cinp;
  float* sl = slab + (size_t)split * 8 * plane;
  if (ks == 0)
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int ib = 0; ib < 2; ++ib) {
          float* sp = sl + (size_t)w5w_point(wave, x) * plane + ci0 + ib * 32 + li;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int co = co0 + cb * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
            sp[(size_t)co * P.cinp] = acc[x][cb][ib][r];
          }
        }
  if (do_bias) {
    __syncthreads();
    smem[tid] = bsum;
    __syncthreads();
    if (tid < W5W_CO) {
      float b = 0.f;
#pragma unroll
      for (int g = 0; g < W5W_NT / 64; ++g) b += smem[tid + 64 * g];
      bslab[(size_t)split * P.copad + co0 + tid] = b;
    }
  }
}

// Σ over the splits (fixed order: 4 lanes of partial sums per output, then in order through
// LDS), dW[co][ci][k] = Σ_ξ G[ξ][k] dU_ξ (the 8×5 G of conv_wino5.h), torch layout [co][ci][5]
// (+= when accumulating).  Workgroup = 64 ci of one co × 4 split lanes; the bias rides in extra
// blocks.
__global__ __launch_bounds__(256) void wwino5_reduce_kernel(
    const float* __restrict__ slab, const float* __restrict__ bslab, float* __restrict__ dw,
    float* __restrict__ db, int splits, int cout, int cin, int copad, int cinp, int accumulate) {
  constexpr float Gm[8][5] = {{-1.f, 0.f, 0.f, 0.f, 0.f},
                              {-2.f / 9, -2.f / 9, -2.f / 9, -2.f / 9, -2.f / 9},
                              {-2.f / 9, 2.f / 9, -2.f / 9, 2.f / 9, -2.f / 9},
                              {1.f / 90, 1.f / 45, 2.f / 45, 4.f / 45, 8.f / 45},
                              {1.f / 90, -1.f / 45, 2.f / 45, -4.f / 45, 8.f / 45},
                              {32.f / 45, 16.f / 45, 8.f / 45, 4.f / 45, 2.f / 45},
                              {32.f / 45, -16.f / 45, 8.f / 45, -4.f / 45, 2.f / 45},
                              {0.f, 0.f, 0.f, 0.f, 1.f}};
  __shared__ float part[4][8][65];
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
  float s[8];
#pragma unroll
  for (int x = 0; x < 8; ++x) s[x] = 0.f;
  for (int sp = k; sp < splits; sp += 4) {
    const float* src = slab + (size_t)sp * 8 * plane + (size_t)co * cinp + ci;
#pragma unroll
    for (int x = 0; x < 8; ++x) s[x] += src[x * plane];
  }
#pragma unroll
  for (int x = 0; x < 8; ++x) part[k][x][o] = s[x];
  __syncthreads();
  if (k != 0 || ci >= cin) return;
  float u[8];
#pragma unroll
  for (int x = 0; x < 8; ++x) u[x] = (part[0][x][o] + part[1][x][o]) + (part[2][x][o] + part[3][x][o]);
  float* d = dw + ((size_t)co * cin + ci) * 5;
#pragma unroll
  for (int t = 0; t < 5; ++t) {
    float v = 0.f;
#pragma unroll
    for (int x = 0; x < 8; ++x) v += Gm[x][t] * u[x];
    d[t] = accumulate ? d[t] + v : v;
  }
}

// shapes: 1×5 (pad 0, 2) or 5×1 (pad 2, 0), stride 1, h % 4 == 0, w % 32 == 0, float4-aligned
// channel groups, cout ≥ 64 (narrower outputs stay on wgrad_kernel / wthin)
bool wwino5_geometry(const scflow_wgrad_args& a, W5wParams* P) {
  static const int off = [] {
    const char* e = getenv("SCFLOW_WGRAD_WINO5");
    return e && e[0] == '0';
  }();
  if (off) return false;
  const int cin = a.cin0 + a.cin1;
  if (a.stride != 1) return false;
  if (a.kh == 1 && a.kw == 5 && a.ph == 0 && a.pw == 2) {
    P->H = a.h, P->W = a.w, P->sy = a.w, P->sx = 1;
  } else if (a.kh == 5 && a.kw == 1 && a.ph == 2 && a.pw == 0) {  // the transposed image's 1×5
    P->H = a.w, P->W = a.h, P->sy = 1, P->sx = a.w;
  } else {
    return false;
  }
  if (P->H % 4 || P->W % 32) return false;
  if (a.cout % 4 || a.sdy % 4 || !aligned16(a.dy) || a.cin0 % 4 || a.s0 % 4 || !aligned16(a.src0) ||
      (a.cin1 > 0 && (a.cin1 % 4 || a.s1 % 4 || !aligned16(a.src1))))
    return false;
  if (a.cout < 64 || cin < 16) return false;
  P->a = a;
  P->cg = P->W / 32;
  P->rg = P->H / 4;
  P->nchunks = a.n * P->rg * P->cg;
  P->co_tiles = (a.cout + W5W_CO - 1) / W5W_CO;
  P->copad = P->co_tiles * W5W_CO;
  P->cinp = (cin + W5W_CI - 1) / W5W_CI * W5W_CI;
  const int tiles = P->co_tiles * (P->cinp / W5W_CI);
  // one workgroup per CU; the partial slabs (8 planes per split) stay under 32 Mi floats
  long long want = (long long)device_cus() / tiles;
  const long long cap = (32LL << 20) / (8LL * P->copad * P->cinp);
  if (want > cap) want = cap;
  if (want > P->nchunks) want = P->nchunks;
  if (want < 1) want = 1;
  P->cps = (int)((P->nchunks + want - 1) / want);
  return true;
}

int wwino5_splits(const W5wParams& P) { return (P.nchunks + P.cps - 1) / P.cps; }

long long wwino5_workspace(const W5wParams& P) {
  const long long s = wwino5_splits(P);
  return s * 8 * P.copad * P.cinp + s * P.copad;
}

int wwino5_launch(const W5wParams& P, hipStream_t st) {
  const scflow_wgrad_args& a = P.a;
  const int splits = wwino5_splits(P);
  float* slab = a.workspace;
  float* bslab = a.db ? a.workspace + (size_t)splits * 8 * P.copad * P.cinp : nullptr;
  const size_t lds = sizeof(float) * (size_t)(W5W_DFL + W5W_XFL) * 2;  // double-buffered
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)wgrad_wino5_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  const dim3 grid((unsigned)(P.co_tiles * (P.cinp / W5W_CI)), (unsigned)splits);
  wgrad_wino5_kernel<<<grid, W5W_NT, lds, st>>>(P, slab, bslab);
  int rc = scflow_launch_status();
  if (rc != SCFLOW_OK) return rc;
  const int cin = a.cin0 + a.cin1;
  const unsigned rblocks = (unsigned)(a.cout * (P.cinp / 64) + (a.db ? (a.cout + 255) / 256 : 0));
  wwino5_reduce_kernel<<<rblocks, 256, 0, st>>>(slab, bslab, a.dw, a.db, splits, a.cout, cin,
                                                P.copad, P.cinp, a.accumulate);
  return scflow_launch_status();
}
