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
// which is where the MFMAs go.
//
// Workgroup = 32 tiles (128 output pixels: 4 image rows at W = 32, 2 at W = 64) × 32·NBW output
// channels, 4 waves.  Wave i owns the four points ξ = (i, 0..3): its Bᵀ row picks two patch rows,
// so the input transform of a wave's A operand is 8 LDS float4 reads and 32 adds per lane per
// 8-channel stage, computed straight into registers (V never exists in memory).  The transformed
// weights U are pre-packed in MFMA-lane order, so each wave streams its own points' U slice from
// L2 as one coalesced 1 KiB load per (ξ, 32 channels), prefetched a stage ahead; nothing of U is
// shared between waves, so it bypasses LDS.  Only the raw input halo of the stage
// ((rows + 2) × (W + 2) pixels × 8 channels) is staged in LDS, shared by the 4 waves.  The
// epilogue applies Aᵀ·A: each wave folds its row of M over j (A), the four rows meet in LDS,
// and Aᵀ over i gives the 2×2 outputs, written channel-contiguous.

constexpr int WKC = 8;    // input channels per stage
constexpr int WLDP = 12;  // LDS pitch of one halo pixel (8 channels + 4 pad, 16-B aligned)
constexpr int WTM = 32;   // tiles per workgroup

struct WinoParams {
  scflow_conv_args a;
  int cp0, nst;  // padded channels of source 0, stages (8 channels each) over both sources
};

template <int W>
struct WinoGeom {
  static constexpr int TW = W / 2;          // tiles per tile row
  static constexpr int TRW = WTM / TW;      // tile rows per workgroup
  static constexpr int OROWS = 2 * TRW;     // output rows per workgroup
  static constexpr int HR = OROWS + 2;      // halo rows
  static constexpr int HC = W + 2;          // halo columns
  static constexpr int NH4 = HR * HC * 2;   // float4 of one stage's halo (2 per pixel)
  static constexpr int NA = (NH4 + 255) / 256;
  // LDS halo layout (float4 units): 3 per pixel (8 channels + pad) and one more every 2 pixels,
  // so the b128 patch reads of 16 consecutive lanes (tiles 2 pixels apart) hit distinct banks
  static constexpr int ROWP = HC * 3 + HC / 2;
  static constexpr int BUF4 = HR * ROWP;
  __device__ static constexpr int addr(int r, int c) { return r * ROWP + c * 3 + (c >> 1); }
};

template <int W, int NBW>
constexpr size_t wino_lds_bytes() {
  const size_t halo = (size_t)2 * WinoGeom<W>::BUF4 * 4;  // double-buffered
  const size_t epi = (size_t)4 * 2 * WTM * 32 * NBW;
  return sizeof(float) * (halo > epi ? halo : epi);
}

template <int W, int NBW>
__global__ __launch_bounds__(256, 2) void conv_wino_kernel(WinoParams P) {
  using G = WinoGeom<W>;
  constexpr int BNW = 32 * NBW;  // output channels per workgroup
  extern __shared__ floatx4 smem4[];  // float4-typed so halo accesses are ds_*_b128
  float* smem = (float*)smem4;
  const scflow_conv_args& a = P.a;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 31, hh = lane >> 5;
  const int blocks_per_img = a.h / G::OROWS;
  const int img = blockIdx.x / blocks_per_img;
  const int oy0 = (blockIdx.x % blocks_per_img) * G::OROWS;
  const int nst0 = P.cp0 / WKC;
  const int nst = P.nst;

  // halo addressing (stage-invariant): input pixel or -1 for zero padding, LDS slot
  int apix[G::NA], acq[G::NA], aslot[G::NA];
#pragma unroll
  for (int j = 0; j < G::NA; ++j) {
    const int idx = tid + 256 * j;
    const int pix = idx >> 1;
    const int hr = pix / G::HC, hcol = pix - hr * G::HC;
    const int iy = oy0 - 1 + hr, ix = hcol - 1;
    const bool ok = idx < G::NH4 && iy >= 0 && iy < a.h && ix >= 0 && ix < W;
    apix[j] = ok ? (img * a.h + iy) * W + ix : -1;
    acq[j] = 4 * (idx & 1);
    aslot[j] = idx < G::NH4 ? G::addr(hr, hcol) + (idx & 1) : -1;
  }
  floatx4 ra[G::NA];
  auto hload = [&](int s) {
    const bool s1 = s >= nst0;
    const float* src = s1 ? a.src1 : a.src0;
    const int cs = s1 ? a.c1 : a.c0;
    const int ss = s1 ? a.s1 : a.s0;
    const int cc = (s1 ? s - nst0 : s) * WKC;
#pragma unroll
    for (int j = 0; j < G::NA; ++j) {
      floatx4 v = {0.f, 0.f, 0.f, 0.f};
      const int c = cc + acq[j];
      if (apix[j] >= 0 && c < cs) v = *(const floatx4*)(src + (size_t)apix[j] * ss + c);
      ra[j] = v;
    }
  };
  auto hstore = [&](int buf) {
#pragma unroll
    for (int j = 0; j < G::NA; ++j)
      if (G::NH4 % 256 == 0 || aslot[j] >= 0) smem4[buf * G::BUF4 + aslot[j]] = ra[j];
  };

  // transformed weights: [nb32][stage][ξ 16][lane 64][4]; this wave's points are ξ = 4·wave + j
  const int nb0 = blockIdx.y * NBW;
  floatx4 ub[4][NBW], un[4][NBW];
  auto uload = [&](floatx4(&u)[4][NBW], int s) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int nb = 0; nb < NBW; ++nb)
        u[j][nb] = *(const floatx4*)(a.weight +
                                     ((((size_t)(nb0 + nb) * nst + s) * 16 + 4 * wave + j) * 64 + lane) * 4);
  };

  // this wave's Bᵀ row: t = c1·d[r1] + c2·d[r2]; the lane's tile (MFMA row li) reads the
  // patch rows r1, r2 of its 4×4 input patch
  const int r1 = wave == 0 ? 0 : 1;
  const int r2 = wave == 0 ? 2 : (wave == 3 ? 3 : 2);
  const float c1 = wave == 2 ? -1.f : 1.f;
  const float c2 = (wave == 0 || wave == 3) ? -1.f : 1.f;
  const int ttr = li / G::TW, ttc = li % G::TW;
  int off1[4], off2[4];
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    off1[b] = G::addr(2 * ttr + r1, 2 * ttc + b) + hh;
    off2[b] = G::addr(2 * ttr + r2, 2 * ttc + b) + hh;
  }
  // V for this lane's tile, 4 channels (4hh..4hh+3 of the stage) at once
  auto vcompute = [&](int buf, floatx4(&v)[4]) {
    const floatx4* hb = smem4 + buf * G::BUF4;
    floatx4 t[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) t[b] = c1 * hb[off1[b]] + c2 * hb[off2[b]];
    v[0] = t[0] - t[2];
    v[1] = t[1] + t[2];
    v[2] = t[2] - t[1];
    v[3] = t[1] - t[3];
  };

  floatx16 acc[4][NBW];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int nb = 0; nb < NBW; ++nb)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[j][nb][e] = 0.f;

  // Software pipeline, one barrier per stage: at stage s the halo of s+1 goes to the other
  // LDS buffer, the halo of s+2 and the weights of s+1 are loaded into registers, and the
  // input transform of s+1 runs between the MFMAs of s.  Loads past the last stage re-read it
  // (no branches in the loop).
  hload(0);
  uload(ub, 0);
  // Drain the prologue loads here: otherwise the compiler's wait-count analysis merges the
  // loop-entry state (ub still in flight) with the steady state and waits for ALL loads — this
  // stage's prefetch included — in front of every stage's first MFMA.
  __builtin_amdgcn_s_waitcnt(0);
  hstore(0);
  hload(nst > 1 ? 1 : 0);
  __syncthreads();
  floatx4 vc[4], vn[4];
  vcompute(0, vc);
  for (int s = 0; s < nst; ++s) {
    const int nbuf = (s + 1) & 1;
    hstore(nbuf);
    __syncthreads();
    hload(s + 2 < nst ? s + 2 : nst - 1);
    uload(un, s + 1 < nst ? s + 1 : nst - 1);
    vcompute(nbuf, vn);
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int nb = 0; nb < NBW; ++nb)
          acc[j][nb] = __builtin_amdgcn_mfma_f32_32x32x2f32(vc[j][e], ub[j][nb][e], acc[j][nb], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      vc[j] = vn[j];
#pragma unroll
      for (int nb = 0; nb < NBW; ++nb) ub[j][nb] = un[j][nb];
    }
  }

  // epilogue.  M row i (this wave) folded over j: s0 = M0+M1+M2, s1 = M1−M2−M3, into
  // S[i][b][tile][co]; then out[a][b] = Σ_i Aᵀ[a][i]·S[i][b].
  // C/D layout: col = lane&31, row = (r&3) + 8(r>>2) + 4(lane>>5).
  __syncthreads();
  float* S = smem;
#pragma unroll
  for (int nb = 0; nb < NBW; ++nb)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = (r & 3) + 8 * (r >> 2) + 4 * hh;
      const int co = nb * 32 + li;
      const float y0 = acc[0][nb][r], y1 = acc[1][nb][r], y2 = acc[2][nb][r], y3 = acc[3][nb][r];
      S[((wave * 2 + 0) * WTM + m) * BNW + co] = y0 + y1 + y2;
      S[((wave * 2 + 1) * WTM + m) * BNW + co] = y1 - y2 - y3;
    }
  __syncthreads();
  const int co = tid % BNW;
  const int col = blockIdx.y * BNW + co;
  if (col >= a.cout) return;
  const float bias = a.bias ? a.bias[col] : 0.f;
  constexpr int GROUPS = 256 / BNW;
  constexpr int NPX = WTM * 4 / GROUPS;  // output pixels per thread
  size_t pix[NPX];
  float val[NPX];
#pragma unroll
  for (int q = 0; q < NPX; ++q) {
    const int p = tid / BNW + GROUPS * q;  // 0..127: tile m = p>>2, a = (p>>1)&1, b = p&1
    const int m = p >> 2, ar = (p >> 1) & 1, bc = p & 1;
    const float* Sb = S + (size_t)bc * WTM * BNW + m * BNW + co;
    const float s0 = Sb[0 * 2 * WTM * BNW], s1 = Sb[1 * 2 * WTM * BNW];
    const float s2 = Sb[2 * 2 * WTM * BNW], s3 = Sb[3 * 2 * WTM * BNW];
    val[q] = ar == 0 ? s0 + s1 + s2 : s1 - s2 - s3;
    const int y = oy0 + 2 * (m / G::TW) + ar, x = 2 * (m % G::TW) + bc;
    pix[q] = ((size_t)img * a.h + y) * W + x;
  }
  if (a.bias_map) {
#pragma unroll
    for (int q = 0; q < NPX; ++q) val[q] += a.bias_map[pix[q] * a.sbm + col];
  }
#pragma unroll
  for (int q = 0; q < NPX; ++q) a.out[pix[q] * a.so + col] = act_apply(val[q] + bias, a.act);
}

// U = G g Gᵀ per (co, ci), packed [nb32][stage][ξ][lane][4] with lane = li + 32·hh ↔
// co = 32·nb32 + li, padded channel kc = 8·stage + 4·hh + e (source 1 starts at cp0).
__global__ void wino_pack_kernel(const float* __restrict__ w, float* __restrict__ out, int cout,
                                 int c0, int c1, int cp0, int nst, long long total) {
  const int cin = c0 + c1;
  for (long long idx = blockIdx.x * 256LL + threadIdx.x; idx < total; idx += (long long)gridDim.x * 256) {
    long long r = idx;
    const int e = (int)(r & 3); r >>= 2;
    const int lane = (int)(r & 63); r >>= 6;
    const int xi = (int)(r & 15); r >>= 4;
    const int s = (int)(r % nst);
    const int nb = (int)(r / nst);
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
      v = (float)acc;
    }
    out[idx] = v;
  }
}
