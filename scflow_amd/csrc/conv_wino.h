// Winograd F(2×2, 3×3) convolution on fp32 MFMA — included by conv.hip (inside its anonymous
// namespace).  Used for the stride-1, pad-1 3×3 convs of the update block (corr_net.1,
// out_net, flow_net.1, the XHead hidden convs, delta_flow/mask encoders; reference
// models/decoder/raft_decoder.py:75-85,256-294, scflow_decoder.py:103-124) and their dX convs in
// training.  Exact-fp32 arithmetic throughout (v_mfma_f32_32x32x2_f32, fp32 transforms whose
// coefficients are 0, ±1 and ½): the result differs from the direct conv only by summation
// order, while the matrix work drops from 9 to 4 multiplies per output pixel and tap set
// (2.25×).
//
// Transforms (Lavin & Gray): Y = Aᵀ[(G g Gᵀ) ⊙ (Bᵀ d B)]A with d the 4×4 input patch of a
// 2×2 output tile,
//   Bᵀ = [1 0 -1 0; 0 1 1 0; 0 -1 1 0; 0 1 0 -1],  G = [1 0 0; ½ ½ ½; ½ -½ ½; 0 0 1],
//   Aᵀ = [1 1 1 0; 0 1 -1 -1].
// For each of the 16 transform points ξ = (i, j) the channel contraction is a GEMM
//   M_ξ[tile][co] = Σ_ci V_ξ[tile][ci] · U_ξ[ci][co],
// which is where the MFMAs go.  Row i = 2 of Bᵀ is stored negated in both V and U (the product
// is unchanged), so every wave's row transform is one FMA, t = d[r1] + s·d[r2].
//
// Workgroup = 32 tiles (128 output pixels: 4 image rows at W = 32, 2 at W = 64) × 32·NBW output
// channels, 4 waves.  Wave i owns the four points ξ = (i, 0..3): its Bᵀ row picks two patch rows,
// so the input transform of a wave's A operand is 8 LDS float4 reads and 16 packed adds per lane
// per 8-channel sub-step, computed straight into registers (V never exists in memory).  The
// transformed weights U are pre-packed in MFMA-lane order, so each wave streams its own points'
// U slice from L2 as one coalesced 1 KiB buffer load per (ξ, 32 channels), each point's slice
// reloaded for the next sub-step as soon as its MFMAs are issued; nothing of U is shared between
// waves, so it bypasses LDS.  Only the raw input halo ((rows + 2) × (W + 2) pixels × 32 channels
// per stage, double-buffered) is staged in LDS, shared by the 4 waves: one barrier per 4
// sub-steps (128 MFMAs per wave), the next stage's halo loaded and stored in quarters between
// this stage's sub-steps, the next sub-step's input transform computed between this sub-step's
// MFMAs.  All global loads are buffer loads (zero padding by the hardware range check, offsets in
// SGPRs), because every VALU instruction in the loop is paid for in MFMA issue cycles (≈ 6 per
// v_pk_fma_f32 at 2 waves per SIMD, tools/micro/mfma_mix.hip).  The epilogue applies Aᵀ·A:
// each wave folds its row of M over j (A), the four rows meet in LDS, and Aᵀ over i gives the
// 2×2 outputs, written channel-contiguous.

typedef float floatx2 __attribute__((ext_vector_type(2)));

// raw buffer resource over [p, p + bytes): loads at offsets ≥ bytes return 0
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wino_rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ floatx4 wino_bload(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}
constexpr int WINO_OOB = 0x7ffffff0;  // voffset of a zero-padding lane (beyond any num_records)

#ifndef WX_SCALAR_VALU
// a + s·b on float4 as two packed FMAs
__device__ __forceinline__ floatx4 fma_s4(floatx4 b, float s, floatx4 a) {
  floatx2 lo = __builtin_elementwise_fma(floatx2{b[0], b[1]}, floatx2{s, s}, floatx2{a[0], a[1]});
  floatx2 hi = __builtin_elementwise_fma(floatx2{b[2], b[3]}, floatx2{s, s}, floatx2{a[2], a[3]});
  return floatx4{lo[0], lo[1], hi[0], hi[1]};
}

// float4 a ± b as two packed ops
__device__ __forceinline__ floatx4 add4(floatx4 a, floatx4 b) {
  const floatx2 lo = floatx2{a[0], a[1]} + floatx2{b[0], b[1]};
  const floatx2 hi = floatx2{a[2], a[3]} + floatx2{b[2], b[3]};
  return floatx4{lo[0], lo[1], hi[0], hi[1]};
}
__device__ __forceinline__ floatx4 sub4(floatx4 a, floatx4 b) {
  const floatx2 lo = floatx2{a[0], a[1]} - floatx2{b[0], b[1]};
  const floatx2 hi = floatx2{a[2], a[3]} - floatx2{b[2], b[3]};
  return floatx4{lo[0], lo[1], hi[0], hi[1]};
}
#else
// scalar forms (v_fma_f32 / v_add_f32 issue beside MFMAs without the packed-op penalty);
// build with -fno-slp-vectorize so they stay scalar
__device__ __forceinline__ floatx4 fma_s4(floatx4 b, float s, floatx4 a) {
  return floatx4{__builtin_fmaf(b[0], s, a[0]), __builtin_fmaf(b[1], s, a[1]),
                 __builtin_fmaf(b[2], s, a[2]), __builtin_fmaf(b[3], s, a[3])};
}
__device__ __forceinline__ floatx4 add4(floatx4 a, floatx4 b) {
  return floatx4{a[0] + b[0], a[1] + b[1], a[2] + b[2], a[3] + b[3]};
}
__device__ __forceinline__ floatx4 sub4(floatx4 a, floatx4 b) {
  return floatx4{a[0] - b[0], a[1] - b[1], a[2] - b[2], a[3] - b[3]};
}
#endif

// Progress-keyed wave priority (WINO_PRIO): a one-round grid puts two workgroups on a CU, and
// the SQ's oldest-first issue lets the first-dispatched one finish its main loop well before the
// second (workgroup stamps, round 5), which then runs alone at one wave per SIMD.  Each wave sets
// its issue priority from its own progress — 3 in the first quarter of the stages down to 0 in
// the last — so the workgroup that is behind wins the arbitration and the two finish together.
#ifndef WINO_PRIO
#define WINO_PRIO 1
#endif
__device__ __forceinline__ void wino_prio(int s, int nst) {
#if WINO_PRIO
  const int pr = 3 - (4 * s) / nst;  // wave-uniform
  if (pr >= 3)
    __builtin_amdgcn_s_setprio(3);
  else if (pr == 2)
    __builtin_amdgcn_s_setprio(2);
  else if (pr == 1)
    __builtin_amdgcn_s_setprio(1);
  else
    __builtin_amdgcn_s_setprio(0);
#endif
}

#ifndef WINO_SCHED_BARRIER
#define WINO_SCHED_BARRIER 1
#endif
#ifndef WINO_U_AHEAD
#define WINO_U_AHEAD 1
#endif

constexpr int WKC = 8;    // input channels per sub-step (one MFMA k-pass per lane)
constexpr int WSC = 32;   // input channels per stage (one LDS halo buffer)
constexpr int WNSUB = WSC / WKC;
constexpr int WTM = 32;   // tiles per workgroup

struct WinoParams {
  scflow_conv_args a;
  int cp0, nst;  // source 0's channels padded to WSC, stages (WSC channels each) over both
  int swz_c;     // XCD-aware block order (wino_block): column parts across the 8 XCDs, 0 = off
  unsigned long long* stamps;  // profiling (scflow_debug_conv_stamps): 4 per workgroup, or NULL
};

// profiling: thread 0's real-time-clock stamp k (0 start, 1 prologue done, 2 main loop done,
// 3 epilogue done) of this workgroup
__device__ __forceinline__ void wino_stamp(unsigned long long* st, int k) {
  if (st && threadIdx.x == 0)
    st[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 4 + k] = __builtin_amdgcn_s_memrealtime();
}

// (tile block, output-channel block) of this workgroup.  Workgroups are dispatched round-robin
// over the 8 XCDs (each with its own L2) in linear block order; with swz_c > 0 the grid is cut
// into an (8/swz_c) × swz_c arrangement of row × column parts, one per XCD, so an XCD's
// workgroups share their transformed-weight slices (column part) and input halos (row part) in
// its L2 instead of every XCD touching every column's weights.  Host guarantees divisibility.
__device__ __forceinline__ void wino_block_ex(int swz_c, int lbx, int lby, int R, int C, int& bx,
                                              int& by) {
  bx = lbx;
  by = lby;
  if (swz_c <= 0) return;
  const int id = lby * R + lbx;
  const int xcd = id & 7, slot = id >> 3;
  const int rows = R / (8 / swz_c), cols = C / swz_c;
  by = (xcd % swz_c) * cols + slot % cols;
  bx = (xcd / swz_c) * rows + slot / cols;
}
__device__ __forceinline__ void wino_block(int swz_c, int& bx, int& by) {
  wino_block_ex(swz_c, blockIdx.x, blockIdx.y, gridDim.x, gridDim.y, bx, by);
}
__device__ __forceinline__ void wino_stamp_id(unsigned long long* st, int sid, int k) {
  if (st && threadIdx.x == 0) st[(size_t)sid * 4 + k] = __builtin_amdgcn_s_memrealtime();
}

template <int W>
struct WinoGeom {
  static constexpr int OCOLS = W < 64 ? W : 64;  // output columns per workgroup
  static constexpr int XB = W / OCOLS;           // column blocks per image row (2 at W = 128)
  static constexpr int TW = OCOLS / 2;      // tiles per tile row of the block
  static constexpr int TRW = WTM / TW;      // tile rows per workgroup
  static constexpr int OROWS = 2 * TRW;     // output rows per workgroup
  static constexpr int HR = OROWS + 2;      // halo rows
  static constexpr int HC = OCOLS + 2;      // halo columns
  static constexpr int NH4 = HR * HC * (WSC / 4);  // float4 of one stage's halo
  static constexpr int NA = (NH4 + 1023) / 1024;   // float4 per thread per quarter stage
  // LDS halo layout (float4 units): 8 per pixel and one more every 2 pixels (tiles 2 pixels
  // apart), plus a row pad where a ds_read_b128 lane group ({0-3, 12-15, 20-27}, {4-11, 16-19,
  // 28-31}, MI355X_MICROARCH.md §LDS) spans two tile rows (OCOLS = 32): 7 float4, so that every
  // group reads 16 distinct 16-B slots of the 256-B bank row (tools/dbg/lds_banks.py)
  static constexpr int ROWP = HC * 8 + HC / 2 + (TW < 32 ? 7 : 0);
  static constexpr int BUF4 = HR * ROWP;
  __device__ static constexpr int addr(int r, int c) { return r * ROWP + c * 8 + (c >> 1); }
};

template <int W, int NBW>
constexpr size_t wino_lds_bytes() {
  const size_t halo = (size_t)2 * WinoGeom<W>::BUF4 * 4;  // double-buffered
  const size_t epi = (size_t)4 * 2 * (WTM + 4) * 32 * NBW;
  return sizeof(float) * (halo > epi ? halo : epi);
}

// NBW = 3 (96 output channels, one workgroup per CU: 192 accumulator registers per lane) balances
// grids whose 64-channel version would leave 1.5 workgroups per CU (corr_net.1 at B = 16).
// (A K split for the 32-channel grids — two wave sets over alternate sub-steps, sums through LDS —
// was built in round 4 and measured in round 5: ±2 % alone, the decoder 2 % slower; removed.)
// body: logical block (lbx, lby) of an lgx × lgy grid, stamps at slot sid (conv_pair.h
// launches two bodies in one grid)
template <int W, int NBW>
__device__ __forceinline__ void conv_wino_body(const WinoParams& P, int lbx, int lby, int lgx,
                                               int lgy, int sid) {
  using G = WinoGeom<W>;
  constexpr int NT = 256;                                   // threads
  constexpr int NA = (G::NH4 + 4 * NT - 1) / (4 * NT);     // float4 per thread per quarter stage
  constexpr int BNW = 32 * NBW;  // output channels per workgroup
  extern __shared__ floatx4 smem4[];  // float4-typed so halo accesses are ds_*_b128
  float* smem = (float*)smem4;
  const scflow_conv_args& a = P.a;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar operands
  const int wave = wv & 3;                 // Winograd row i of the wave's points
  const int li = lane & 31, hh = lane >> 5;
  int bx, by;
  wino_block_ex(P.swz_c, lbx, lby, lgx, lgy, bx, by);
  wino_stamp_id(P.stamps, sid, 0);
  // the epilogue's per-channel operands (32-channel blocks: a few VGPRs to spare), fetched now:
  // in a one-round grid every workgroup reaches its epilogue together, and loads there all wait
  // on the same few cache lines (the small-cin conv's epilogue: 6.3 → 3.4 µs)
  float pre_bias = 0.f, pre_osc = 1.f, pre_osh = 0.f;
  if constexpr (NBW == 1 && NT % BNW == 0) {
    const int pcol = by * BNW + threadIdx.x % BNW;
    if (pcol < a.cout) {
      if (a.bias) pre_bias = a.bias[pcol];
      if (a.out_scale) {
        pre_osc = a.out_scale[pcol];
        pre_osh = a.out_shift[pcol];
      }
    }
  }
  const int blocks_per_img = (a.h / G::OROWS) * G::XB;
  const int img = bx / blocks_per_img;
  const int brem = bx % blocks_per_img;
  const int oy0 = (brem / G::XB) * G::OROWS, ox0 = (brem % G::XB) * G::OCOLS;
  const int nst0 = P.cp0 / WSC;
  const int nst = P.nst;
  const int npix = a.n * a.h * W;

  // halo staging: four quarters of NA float4 per thread; slot (part, j) is the (pixel, channel
  // quad) pair (idx >> 3, idx & 7), idx = tid + 256·(4j + part).  Per slot: the input pixel
  // (-1 = zero padding) and the LDS float4 index, both stage-invariant.
  bool inloop = false;  // tuning experiments (WX_NO_*): prologue loads still happen
  int hpix[4][NA], hlds[4][NA];
#pragma unroll
  for (int part = 0; part < 4; ++part)
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      const int idx = tid + NT * (4 * j + part);
      const int pix = idx >> 3;
      const int hr = pix / G::HC, hcol = pix - hr * G::HC;
      const int iy = oy0 - 1 + hr, ix = ox0 - 1 + hcol;
      const bool ok = idx < G::NH4 && iy >= 0 && iy < a.h && ix >= 0 && ix < W;
      hpix[part][j] = ok ? (img * a.h + iy) * W + ix : -1;
      hlds[part][j] = idx < G::NH4 ? G::addr(hr, hcol) + (idx & 7) : -1;
    }
  const int hq4 = 4 * (tid & 7);  // channel of this thread's quad within the stage (idx & 7 = tid & 7)
  floatx4 ra[2][NA];  // quarter part in slot part & 1
  // stage s's source, as a buffer starting at its first channel
  __amdgpu_buffer_rsrc_t hsrc;
  int hss4 = 0, hlim = 0;  // pixel stride in bytes, channels of the stage present in the source
  floatx4 isc = {1.f, 1.f, 1.f, 1.f}, ish = {0.f, 0.f, 0.f, 0.f};  // input affine (encoder IN)
  const bool in_aff = a.in_scale != nullptr;
  auto hsource = [&](int s) {
    const bool s1 = s >= nst0;
    const float* src = s1 ? a.src1 : a.src0;
    const int cs = s1 ? a.c1 : a.c0;
    const int ss = s1 ? a.s1 : a.s0;
    const int cc = (s1 ? s - nst0 : s) * WSC;
    hsrc = wino_rsrc(src + cc, (unsigned)(((long long)(npix - 1) * ss + cs - cc) * 4));
    hss4 = ss * 4;
    hlim = cs - cc;
    if (in_aff && hq4 < hlim) {  // this thread's 4 channels of the stage, for its image
      isc = *(const floatx4*)(a.in_scale + (size_t)img * a.c0 + cc + hq4);
      ish = *(const floatx4*)(a.in_shift + (size_t)img * a.c0 + cc + hq4);
    }
  };
  auto hload = [&](int part) {
#ifdef WX_NO_HALO
    if (inloop) return;
#endif
    const bool chan_ok = hq4 < hlim;
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      const int p = hpix[part][j];
      const bool ok = p >= 0 && chan_ok;
      floatx4 v = wino_bload(hsrc, ok ? p * hss4 + hq4 * 4 : WINO_OOB, 0);
      if (in_aff && ok) {  // zero padding stays zero (it pads the normalised activation)
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e] * isc[e] + ish[e], 0.f);
      }
      ra[part & 1][j] = v;
    }
  };
  auto hstore = [&](int buf, int part) {
#ifdef WX_NO_HALO
    if (inloop) return;
#endif
#pragma unroll
    for (int j = 0; j < NA; ++j)
      if (G::NH4 % (4 * NT) == 0 || hlds[part][j] >= 0) smem4[buf * G::BUF4 + hlds[part][j]] = ra[part & 1][j];
  };

  // transformed weights [nb32][sub-step (8 channels)][ξ 16][lane 64][4]; this wave's points are
  // ξ = 4·wave + j
  const int nsub = nst * WNSUB;
  const __amdgpu_buffer_rsrc_t wsrc =
      wino_rsrc(a.weight + (size_t)by * NBW * nsub * 16 * 256, (unsigned)(NBW * nsub * 16 * 1024));
  auto uload1 = [&](floatx4(&u)[NBW], int t, int j) {  // point j of sub-step t (clamped)
#ifdef WX_NO_U
    if (inloop) return;
#endif
    const int tt = t < nsub ? t : nsub - 1;
#pragma unroll
    for (int nb = 0; nb < NBW; ++nb)
      u[nb] = wino_bload(wsrc, lane * 16, (((nb * nsub + tt) * 16 + 4 * wave + j) * 1024));
  };

  // this wave's Bᵀ row (row 2 negated): t = d[r1] + sgn·d[r2]; the lane's tile (MFMA row li)
  // reads the patch rows r1, r2 of its 4×4 input patch
  const int r1 = wave == 0 ? 0 : 1;
  const int r2 = wave == 0 ? 2 : (wave == 3 ? 3 : 2);
  const float sgn = wave == 1 ? 1.f : -1.f;
  const int ttr = li / G::TW, ttc = li % G::TW;
  const int o1 = G::addr(2 * ttr + r1, 2 * ttc) + hh, o2 = G::addr(2 * ttr + r2, 2 * ttc) + hh;
  // column b of the patch: +8b float4 plus the skew (patches start at even columns)
  auto vcompute = [&](int buf, int k, floatx4(&v)[4]) {
    const floatx4* hb = smem4 + buf * G::BUF4 + 2 * k;
    floatx4 t[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int cb = b * 8 + (b >> 1);
      t[b] = fma_s4(hb[o2 + cb], sgn, hb[o1 + cb]);
    }
    v[0] = sub4(t[0], t[2]);
    v[1] = add4(t[1], t[2]);
    v[2] = sub4(t[2], t[1]);
    v[3] = sub4(t[1], t[3]);
  };

  floatx16 acc[4][NBW];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int nb = 0; nb < NBW; ++nb)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[j][nb][e] = 0.f;

  // U of the next UAH sub-steps in registers (sub-step t in slot t % UAH): a point's reload is for
  // the sub-step UAH ahead, so it has UAH − 1 further sub-steps plus this one's remaining points to
  // arrive (WINO_U_AHEAD = 2: the 32-channel workgroups, one wave per SIMD at B = 16)
  constexpr int UAH = (NBW == 1 && WINO_U_AHEAD > 1) ? 2 : 1;
  floatx4 u[UAH][4][NBW];
  // the MFMAs of point j of the sub-step in slot par, then point j's weights for sub-step tload
  // (the one UAH further along the wave's sequence) into the same slot
  auto point = [&](const floatx4(&v)[4], int j, int tload, int par) {
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int nb = 0; nb < NBW; ++nb)
        acc[j][nb] = __builtin_amdgcn_mfma_f32_32x32x2f32(v[j][e], u[par][j][nb][e], acc[j][nb], 0, 0, 0);
    uload1(u[par][j], tload, j);
    // keep the reload here, three points ahead of its use: left alone the scheduler sinks all four
    // reloads to the end of the sub-step, one MFMA before the next sub-step waits on them (an L2
    // round trip exposed per point at one wave per SIMD).  32-channel workgroups only: the
    // 64 / 96-channel ones run at the 256-VGPR limit (pinning the loads spills there) and have a
    // second wave per SIMD to cover the latency.
    if constexpr (WINO_SCHED_BARRIER && (NBW == 1 || WINO_SCHED_BARRIER > 1))
      __builtin_amdgcn_sched_barrier(0);
  };
  auto substep = [&](const floatx4(&v)[4], int tload, int par) {
#pragma unroll
    for (int j = 0; j < 4; ++j) point(v, j, tload, par);
  };
  // a sub-step with the NEXT sub-step's input transform (from LDS buffer buf, channels 8k..)
  // woven between its point groups in program order — the compiler issues in order, so the LDS
  // latency and the VALU sit under this sub-step's MFMAs instead of in front of them
  auto substep_next = [&](const floatx4(&v)[4], int tload, int par, int buf, int k,
                          floatx4(&vn)[4]) {
#ifdef WX_NO_V
    substep(v, tload, par);
    for (int j = 0; j < 4; ++j) vn[j] = v[j];
    return;
#endif
    const floatx4* hb = smem4 + buf * G::BUF4 + 2 * k;
    constexpr int cb1 = 8, cb2 = 16 + 1, cb3 = 24 + 1;  // column b of the patch (+ skew)
    const floatx4 a0 = hb[o1], b0 = hb[o2], a2 = hb[o1 + cb2], b2 = hb[o2 + cb2];
    point(v, 0, tload, par);
    const floatx4 t0 = fma_s4(b0, sgn, a0), t2 = fma_s4(b2, sgn, a2);
    vn[0] = sub4(t0, t2);
    const floatx4 a1 = hb[o1 + cb1], b1 = hb[o2 + cb1], a3 = hb[o1 + cb3], b3 = hb[o2 + cb3];
    point(v, 1, tload, par);
    const floatx4 t1 = fma_s4(b1, sgn, a1), t3 = fma_s4(b3, sgn, a3);
    vn[1] = add4(t1, t2);
    vn[2] = sub4(t2, t1);
    vn[3] = sub4(t1, t3);
    point(v, 2, tload, par);
    point(v, 3, tload, par);
  };

  // prologue: stage 0's halo in LDS buffer 0, sub-step 0's (and 1's) weights and transform in
  // registers
#pragma unroll
  for (int d = 0; d < UAH; ++d)
#pragma unroll
    for (int j = 0; j < 4; ++j) uload1(u[d][j], d, j);
  hsource(0);
#pragma unroll
  for (int part = 0; part < 4; ++part) {
    hload(part);
    hstore(0, part);
  }
  // Drain the prologue loads: otherwise the compiler's wait-count analysis merges the
  // loop-entry state with the steady state and waits for ALL loads in front of the MFMAs.
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  wino_stamp_id(P.stamps, sid, 1);
  floatx4 vA[4], vB[4];
  vcompute(0, 0, vA);
  inloop = true;
  for (int s = 0; s < nst; ++s) {
    const int buf = s & 1;
    hsource(s + 1 < nst ? s + 1 : s);  // the last stage re-stages itself (no branches)
    // sub-step t = 4s + k − 1 in slot t % UAH reloads its points for t + UAH
    const int t0 = s * WNSUB;
    hload(0);
    substep_next(vA, t0 + UAH, 0, buf, 1, vB);
    hstore(buf ^ 1, 0);
    hload(1);
    substep_next(vB, t0 + 1 + UAH, 1 % UAH, buf, 2, vA);
    hstore(buf ^ 1, 1);
    hload(2);
    substep_next(vA, t0 + 2 + UAH, 2 % UAH, buf, 3, vB);
    hstore(buf ^ 1, 2);
    hload(3);
    substep(vB, t0 + 3 + UAH, 3 % UAH);
    hstore(buf ^ 1, 3);
#ifndef WX_NO_SYNC
    __syncthreads();
#endif
#ifndef WX_NO_V
    vcompute(buf ^ 1, 0, vA);
#endif
  }

#ifdef WX_NO_EPI
  {
    float t = 0.f;
    for (int j = 0; j < 4; ++j)
      for (int nb = 0; nb < NBW; ++nb)
        for (int e = 0; e < 16; ++e) t += acc[j][nb][e];
    if (t == 12345.678f) a.out[tid] = t;
    return;
  }
#endif
  // epilogue.  M row i (this wave) folded over j: s0 = M0+M1+M2, s1 = M1−M2−M3, into
  // S[i][b][co][tile] (tiles contiguous, WEP-float rows: a lane's 4 accumulator rows r..r+3 of
  // a 32×32 block are 4 consecutive tiles, so each goes out as one 16-B store); then every
  // thread owns one output position (a, b) of its channel co over a run of tiles and reads the
  // four rows i of 4 tiles at a time (16-B loads): out[a][b] = Σ_i Aᵀ[a][i]·S[i][b].
  // C/D layout: col = lane&31, row = (r&3) + 8(r>>2) + 4(lane>>5).  Row stride WEP = 36 floats
  // keeps both the b128 stores (8-lane groups) and the b128 loads (16-lane groups) conflict-free.
  constexpr int WEP = WTM + 4;
  __syncthreads();
  wino_stamp_id(P.stamps, sid, 2);
  float* S = smem;
#pragma unroll
  for (int nb = 0; nb < NBW; ++nb)
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) {
      const int co = nb * 32 + li;
      floatx4 s0v, s1v;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int r = 4 * q4 + rr;
        const float y0 = acc[0][nb][r], y1 = acc[1][nb][r], y2 = acc[2][nb][r], y3 = acc[3][nb][r];
        s0v[rr] = y0 + y1 + y2;
        s1v[rr] = y1 - y2 - y3;
      }
      const int m0 = 8 * q4 + 4 * hh;
      *(floatx4*)&S[((wave * 2 + 0) * BNW + co) * WEP + m0] = s0v;
      *(floatx4*)&S[((wave * 2 + 1) * BNW + co) * WEP + m0] = s1v;
    }
  __syncthreads();
  if constexpr (NT % BNW == 0) {
    const int co = tid % BNW;
    const int col = by * BNW + co;
    if (col >= a.cout) return;
    float bias = pre_bias, osc = pre_osc, osh = pre_osh;
    if constexpr (NBW != 1) {
      bias = a.bias ? a.bias[col] : 0.f;
      osc = a.out_scale ? a.out_scale[col] : 1.f;
      osh = a.out_scale ? a.out_shift[col] : 0.f;
    }
    constexpr int GROUPS = NT / BNW;             // 4 (BNW 64) or 8 (BNW 32)
    constexpr int NPX = WTM * 4 / GROUPS;        // output pixels per thread
    const int g = tid / BNW;
    const int ar = (g >> 1) & 1, bc = g & 1;      // this thread's output position in the 2×2 tile
    const int mbase = (g >> 2) * NPX;             // its run of NPX tiles
    size_t pix[NPX];
    float val[NPX];
  #pragma unroll
    for (int q4 = 0; q4 < NPX / 4; ++q4) {
      const int m0 = mbase + 4 * q4;
      const float* Sb = S + ((size_t)bc * BNW + co) * WEP + m0;
      const floatx4 s0 = *(const floatx4*)(Sb + 0 * 2 * BNW * WEP);
      const floatx4 s1 = *(const floatx4*)(Sb + 1 * 2 * BNW * WEP);
      const floatx4 s2 = *(const floatx4*)(Sb + 2 * 2 * BNW * WEP);
      const floatx4 s3 = *(const floatx4*)(Sb + 3 * 2 * BNW * WEP);
  #pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int q = 4 * q4 + e, m = m0 + e;
        const float v = ar == 0 ? s0[e] + s1[e] + s2[e] : s1[e] - s2[e] - s3[e];
        const int y = oy0 + 2 * (m / G::TW) + ar, x = ox0 + 2 * (m % G::TW) + bc;
        pix[q] = ((size_t)img * a.h + y) * W + x;
        val[q] = (v + bias) * osc + osh;
      }
    }
    // all global reads (bias map, residual) before any store
    if (a.bias_map) {
  #pragma unroll
      for (int q = 0; q < NPX; ++q) val[q] += a.bias_map[pix[q] * a.sbm + col];
    }
    if (a.res) {
  #pragma unroll
      for (int q = 0; q < NPX; ++q) val[q] += a.res[pix[q] * a.sres + col];
    }
    // the activation as a constant of the store loop (one branch-free body per activation)
    auto store = [&](auto actc) __attribute__((always_inline)) {
      constexpr int ACT = decltype(actc)::value;
  #pragma unroll
      for (int q = 0; q < NPX; ++q) a.out[pix[q] * a.so + col] = act_apply(val[q], ACT);
    };
    switch (a.act) {
      case SCFLOW_ACT_RELU: store(std::integral_constant<int, SCFLOW_ACT_RELU>{}); break;
      case SCFLOW_ACT_SIGMOID: store(std::integral_constant<int, SCFLOW_ACT_SIGMOID>{}); break;
      case SCFLOW_ACT_TANH: store(std::integral_constant<int, SCFLOW_ACT_TANH>{}); break;
      default: store(std::integral_constant<int, SCFLOW_ACT_NONE>{}); break;
    }

  } else {
    // BNW does not divide the 256 threads: (output position, channel) pairs dealt round robin,
    // each pair over all WTM tiles (same arithmetic as above)
    for (int pi = tid; pi < 4 * BNW; pi += NT) {
      const int co = pi % BNW, g = pi / BNW;
      const int col = by * BNW + co;
      if (col >= a.cout) continue;
      const float bias = a.bias ? a.bias[col] : 0.f;
      const float osc = a.out_scale ? a.out_scale[col] : 1.f;
      const float osh = a.out_scale ? a.out_shift[col] : 0.f;
      const int ar = (g >> 1) & 1, bc = g & 1;
#pragma unroll 2
      for (int q4 = 0; q4 < WTM / 4; ++q4) {
        const int m0 = 4 * q4;
        const float* Sb = S + ((size_t)bc * BNW + co) * WEP + m0;
        const floatx4 s0 = *(const floatx4*)(Sb + 0 * 2 * BNW * WEP);
        const floatx4 s1 = *(const floatx4*)(Sb + 1 * 2 * BNW * WEP);
        const floatx4 s2 = *(const floatx4*)(Sb + 2 * 2 * BNW * WEP);
        const floatx4 s3 = *(const floatx4*)(Sb + 3 * 2 * BNW * WEP);
        size_t pix[4];
        float val[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int m = m0 + e;
          const float v = ar == 0 ? s0[e] + s1[e] + s2[e] : s1[e] - s2[e] - s3[e];
          const int y = oy0 + 2 * (m / G::TW) + ar, x = ox0 + 2 * (m % G::TW) + bc;
          pix[e] = ((size_t)img * a.h + y) * W + x;
          val[e] = (v + bias) * osc + osh;
        }
        if (a.bias_map) {
#pragma unroll
          for (int e = 0; e < 4; ++e) val[e] += a.bias_map[pix[e] * a.sbm + col];
        }
        if (a.res) {
#pragma unroll
          for (int e = 0; e < 4; ++e) val[e] += a.res[pix[e] * a.sres + col];
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) a.out[pix[e] * a.so + col] = act_apply(val[e], a.act);
      }
    }
  }
  if (P.stamps) {
    __builtin_amdgcn_s_waitcnt(0);
    wino_stamp_id(P.stamps, sid, 3);
  }
}

template <int W, int NBW>
__global__ __launch_bounds__(256, NBW >= 3 ? 1 : 2) void conv_wino_kernel(WinoParams P) {
  conv_wino_body<W, NBW>(P, blockIdx.x, blockIdx.y, gridDim.x, gridDim.y,
                         blockIdx.y * gridDim.x + blockIdx.x);
}

// U = G g Gᵀ per (co, ci) (row i = 2 negated), packed [nb32][sub-step][ξ][lane][4] with
// lane = li + 32·hh ↔ co = 32·nb32 + li, padded channel kc = 8·sub-step + 4·hh + e (source 1
// starts at cp0).
__global__ void wino_pack_kernel(const float* __restrict__ w, float* __restrict__ out, int cout,
                                 int c0, int c1, int cp0, int nsub, long long total) {
  const int cin = c0 + c1;
  for (long long idx = blockIdx.x * 256LL + threadIdx.x; idx < total; idx += (long long)gridDim.x * 256) {
    long long r = idx;
    const int e = (int)(r & 3); r >>= 2;
    const int lane = (int)(r & 63); r >>= 6;
    const int xi = (int)(r & 15); r >>= 4;
    const int s = (int)(r % nsub);
    const int nb = (int)(r / nsub);
    const int o = nb * 32 + (lane & 31);
    const int kc = s * WKC + 4 * (lane >> 5) + e;
    int ci = -1;
    if (kc < cp0) {
      if (kc < c0) ci = kc;
    } else if (kc - cp0 < c1) {
      ci = c0 + (kc - cp0);
    }
    float v = 0.f;
    if (o < cout && ci >= 0) {
      const float* g = w + ((size_t)o * cin + ci) * 9;
      const double Gm[4][3] = {{1, 0, 0}, {0.5, 0.5, 0.5}, {0.5, -0.5, 0.5}, {0, 0, 1}};
      const int i = xi >> 2, j = xi & 3;
      double acc = 0.0;
      for (int p = 0; p < 3; ++p)
        for (int q = 0; q < 3; ++q) acc += Gm[i][p] * (double)g[p * 3 + q] * Gm[j][q];
      v = (float)(i == 2 ? -acc : acc);
    }
    out[idx] = v;
  }
}
