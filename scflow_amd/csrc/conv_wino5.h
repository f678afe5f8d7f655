// 1-D Winograd F(4, 5) convolution on fp32 MFMA for the SeqConv GRU's 1×5 and 5×1 convs —
// included by conv.hip (inside its anonymous namespace).  Reference: ConvGRU SeqConv,
// models/decoder/raft_decoder.py:180-181 (kernel table), :235-253 (z, r, q gates).
//
// A tile is 4 consecutive output pixels along the conv axis; its 8 input pixels d give
//   y = Aᵀ[(G g) ⊙ (Bᵀ d)],   transform points {0, ±1, ±2, ±½, ∞},
// i.e. 8 multiplies per tile instead of 20 (2.5× less matrix work).  The coefficients are the
// exact rationals of the Toom-Cook construction; the fp32 error of the whole conv measured in a
// numpy restatement (384 channels) is 2.0× that of the direct fp32 conv — the same order, far
// inside the decoder's tolerances.  The weight transform is done in fp64 once per packing.
//
// Per transform point ξ the channel contraction is a GEMM M_ξ[tile][co] = Σ_ci V_ξ·U_ξ on
// v_mfma_f32_32x32x2_f32.  Workgroup = 32 tiles (128 output pixels: 128/W whole rows for 1×5,
// a 4-row × 32-column block for 5×1) × 32·NBW output channels, 4 waves; wave i owns the points
// ξ = 2i, 2i+1: it forms its two rows of Bᵀd straight into registers from the stage's input
// halo in LDS (16 float4 reads, 64 FMAs per lane per 16-channel stage) and streams its points'
// pre-transformed weights from L2 (lane-ordered, 1 KiB per load, prefetched a stage ahead).
// The epilogue gathers the 8 points of every (tile, channel) in LDS, applies Aᵀ and runs the
// same fused epilogues as the direct conv (bias map, bias + activation, GRU z | r·h, GRU
// h ← (1−z)h + z·tanh(q)).

constexpr int W5KC = 16;  // input channels per stage
constexpr int W5P4 = 5;   // LDS pitch of one halo pixel in float4 (16 channels + 4 pad floats)
constexpr int W5TM = 32;  // tiles per workgroup

__constant__ float kW5BT[8][8] = {
    {-1.0f, 0.0f, 5.25f, 0.0f, -5.25f, 0.0f, 1.0f, 0.0f},
    {0.0f, 1.0f, 1.0f, -4.25f, -4.25f, 1.0f, 1.0f, 0.0f},
    {0.0f, -1.0f, 1.0f, 4.25f, -4.25f, -1.0f, 1.0f, 0.0f},
    {0.0f, 0.5f, 0.25f, -2.5f, -1.25f, 2.0f, 1.0f, 0.0f},
    {0.0f, -0.5f, 0.25f, 2.5f, -1.25f, -2.0f, 1.0f, 0.0f},
    {0.0f, 2.0f, 4.0f, -2.5f, -5.0f, 0.5f, 1.0f, 0.0f},
    {0.0f, -2.0f, 4.0f, 2.5f, -5.0f, -0.5f, 1.0f, 0.0f},
    {0.0f, -1.0f, 0.0f, 5.25f, 0.0f, -5.25f, 0.0f, 1.0f}};
constexpr float kW5AT[4][8] = {{1.0f, 1.0f, 1.0f, 1.0f, 1.0f, 1.0f, 1.0f, 0.0f},
                               {0.0f, 1.0f, -1.0f, 2.0f, -2.0f, 0.5f, -0.5f, 0.0f},
                               {0.0f, 1.0f, 1.0f, 4.0f, 4.0f, 0.25f, 0.25f, 0.0f},
                               {0.0f, 1.0f, -1.0f, 8.0f, -8.0f, 0.125f, -0.125f, 1.0f}};

struct Wino5Params {
  scflow_conv_args a;
  int cp0, nst;  // padded channels of source 0, stages (16 channels each) over both sources
};

template <int DIR, int W>  // DIR 0: 1×5 (along x), 1: 5×1 (along y)
struct Wino5Geom {
  static constexpr int TPR = DIR == 0 ? W / 4 : 32;     // tiles per row of the block
  static constexpr int OROWS = DIR == 0 ? 128 / W : 4;  // output rows per workgroup
  static constexpr int OCOLS = DIR == 0 ? W : 32;       // output columns per workgroup
  static constexpr int HR = DIR == 0 ? OROWS : OROWS + 4;
  static constexpr int HC = DIR == 0 ? W + 4 : 32;
  static constexpr int NH4 = HR * HC * 4;  // float4 of one stage's halo (4 per pixel)
  static constexpr int NA = (NH4 + 255) / 256;
  // LDS halo layout (float4 units): 5 per pixel (16 channels + pad); for 1×5 (lanes 4 pixels
  // apart, 2 or 4 tile rows per 16 lanes) one more float4 every SK pixels plus a row pad, so
  // the b128 reads of 16 consecutive lanes hit distinct banks (5×1: lanes 1 pixel apart, already
  // conflict-free)
  static constexpr int SK = DIR == 1 ? 0 : (W == 32 ? 2 : 4);
  static constexpr int ROWP = HC * W5P4 + (SK ? HC / SK : 0) + (DIR == 0 && W == 32 ? 1 : 0);
  static constexpr int BUF4 = HR * ROWP;
  __device__ static constexpr int addr(int r, int c) {
    return r * ROWP + c * W5P4 + (SK ? c / SK : 0);
  }
};

template <int DIR, int W, int NBW>
constexpr size_t wino5_lds_bytes() {
  const size_t halo = (size_t)2 * Wino5Geom<DIR, W>::BUF4 * 4;  // double-buffered
  const size_t epi = (size_t)8 * W5TM * 32 * NBW;
  return sizeof(float) * (halo > epi ? halo : epi);
}

// the fused epilogues of one output element (shared with the direct conv's semantics)
template <int EPI>
__device__ __forceinline__ void conv_epilogue_store(const scflow_conv_args& a, size_t pix, int col,
                                                   float v) {
  if constexpr (EPI == SCFLOW_EPI_PLAIN) {
    a.out[pix * a.so + col] = act_apply(v, a.act);
  } else if constexpr (EPI == SCFLOW_EPI_GRU_ZR) {
    const int hcn = a.cout >> 1;
    if (col < hcn) {
      a.gate[pix * a.sg + col] = sigmoidf_(v);
    } else {
      const int c = col - hcn;
      a.rh[pix * a.srh + c] = sigmoidf_(v) * a.hid[pix * a.sh + c];
    }
  } else {  // GRU_Q
    const float z = a.gate[pix * a.sg + col];
    const float h = a.hid[pix * a.sh + col];
    a.hid[pix * a.sh + col] = (1.f - z) * h + z * tanhf(v);
  }
}

template <int DIR, int W, int NBW, int EPI>
__global__ __launch_bounds__(256, 2) void conv_wino5_kernel(Wino5Params P) {
  using G = Wino5Geom<DIR, W>;
  constexpr int BNW = 32 * NBW;
  extern __shared__ floatx4 smem4[];
  float* smem = (float*)smem4;
  const scflow_conv_args& a = P.a;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 31, hh = lane >> 5;
  constexpr int XB = W / G::OCOLS;  // column blocks per image (1, or 2 for 5×1 at W = 64)
  const int blocks_per_img = (a.h / G::OROWS) * XB;
  const int img = blockIdx.x / blocks_per_img;
  const int rem = blockIdx.x % blocks_per_img;
  const int oy0 = (rem / XB) * G::OROWS, ox0 = (rem % XB) * G::OCOLS;
  const int nst0 = P.cp0 / W5KC;
  const int nst = P.nst;
  // halo origin in image coordinates
  const int hy0 = DIR == 0 ? oy0 : oy0 - 2, hx0 = DIR == 0 ? -2 : ox0;

  int apix[G::NA], acq[G::NA], aslot[G::NA];
#pragma unroll
  for (int j = 0; j < G::NA; ++j) {
    const int idx = tid + 256 * j;
    const int pix = idx >> 2;
    const int hr = pix / G::HC, hcol = pix - hr * G::HC;
    const int iy = hy0 + hr, ix = hx0 + hcol;
    const bool ok = idx < G::NH4 && iy >= 0 && iy < a.h && ix >= 0 && ix < W;
    apix[j] = ok ? (img * a.h + iy) * W + ix : -1;
    acq[j] = 4 * (idx & 3);
    aslot[j] = idx < G::NH4 ? G::addr(hr, hcol) + (idx & 3) : -1;
  }
  floatx4 ra[G::NA];
  auto hload = [&](int s) {
    const bool s1 = s >= nst0;
    const float* src = s1 ? a.src1 : a.src0;
    const int cs = s1 ? a.c1 : a.c0;
    const int ss = s1 ? a.s1 : a.s0;
    const int cc = (s1 ? s - nst0 : s) * W5KC;
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

  // weights [nb32][stage][ξ 8][q 2][lane 64][4]; this wave's points ξ = 2·wave + x
  const int nb0 = blockIdx.y * NBW;
  floatx4 ub[2][2][NBW], un[2][2][NBW];  // [q][x][nb]
  auto uload = [&](floatx4(&u)[2][2][NBW], int s) {
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int nb = 0; nb < NBW; ++nb)
          u[q][x][nb] = *(const floatx4*)(a.weight +
                                          (((((size_t)(nb0 + nb) * nst + s) * 8 + 2 * wave + x) * 2 + q) * 64 +
                                           lane) * 4);
  };
  // this wave's two Bᵀ rows (wave-uniform)
  float bt[2][8];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int t = 0; t < 8; ++t) bt[x][t] = kW5BT[2 * wave + x][t];
  // this lane's tile: LDS offsets of its 8 inputs along the conv axis
  int toff[8];
#pragma unroll
  for (int t = 0; t < 8; ++t)
    toff[t] = (DIR == 0 ? G::addr(li / G::TPR, 4 * (li % G::TPR) + t) : G::addr(t, li)) + hh;
  auto vcompute = [&](int buf, floatx4(&v)[2][2]) {  // [q][x]
    const floatx4* hb = smem4 + buf * G::BUF4;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      v[q][0] = v[q][1] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const floatx4 d = hb[toff[t] + 2 * q];
        v[q][0] += bt[0][t] * d;
        v[q][1] += bt[1][t] * d;
      }
    }
  };

  floatx16 acc[2][NBW];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int nb = 0; nb < NBW; ++nb)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[x][nb][e] = 0.f;

  // software pipeline as in conv_wino.h: one barrier per stage, next stage's input transform
  // between this stage's MFMAs
  hload(0);
  uload(ub, 0);
  __builtin_amdgcn_s_waitcnt(0);  // see conv_wino.h: keeps the prefetch off the MFMAs' wait
  hstore(0);
  hload(nst > 1 ? 1 : 0);
  __syncthreads();
  floatx4 vc[2][2], vn[2][2];
  vcompute(0, vc);
  for (int s = 0; s < nst; ++s) {
    const int nbuf = (s + 1) & 1;
    hstore(nbuf);
    __syncthreads();
    hload(s + 2 < nst ? s + 2 : nst - 1);
    uload(un, s + 1 < nst ? s + 1 : nst - 1);
    vcompute(nbuf, vn);
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
          for (int nb = 0; nb < NBW; ++nb)
            acc[x][nb] = __builtin_amdgcn_mfma_f32_32x32x2f32(vc[q][x][e], ub[q][x][nb][e], acc[x][nb], 0, 0, 0);
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int x = 0; x < 2; ++x) {
        vc[q][x] = vn[q][x];
#pragma unroll
        for (int nb = 0; nb < NBW; ++nb) ub[q][x][nb] = un[q][x][nb];
      }
  }

  // epilogue: M[ξ][tile][co] in LDS, then y[o] = Σ_ξ Aᵀ[o][ξ]·M[ξ]
  __syncthreads();
  float* S = smem;
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int nb = 0; nb < NBW; ++nb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = (r & 3) + 8 * (r >> 2) + 4 * hh;
        S[((2 * wave + x) * W5TM + m) * BNW + nb * 32 + li] = acc[x][nb][r];
      }
  __syncthreads();
  const int co = tid % BNW;
  const int col = blockIdx.y * BNW + co;
  if (col >= a.cout) return;
  const float bias = a.bias ? a.bias[col] : 0.f;
  constexpr int GROUPS = 256 / BNW;
  constexpr int NT = W5TM / GROUPS;  // tiles per thread
#pragma unroll
  for (int k = 0; k < NT; ++k) {
    const int m = tid / BNW + GROUPS * k;
    float mv[8];
#pragma unroll
    for (int xi = 0; xi < 8; ++xi) mv[xi] = S[(xi * W5TM + m) * BNW + co];
    float y[4];
    size_t pix[4];
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      float v = 0.f;
#pragma unroll
      for (int xi = 0; xi < 8; ++xi)
        if (kW5AT[o][xi] != 0.f) v += kW5AT[o][xi] * mv[xi];
      y[o] = v + bias;
      const int oy = DIR == 0 ? oy0 + m / G::TPR : oy0 + o;
      const int ox = DIR == 0 ? 4 * (m % G::TPR) + o : ox0 + m;
      pix[o] = ((size_t)img * a.h + oy) * W + ox;
    }
    if (a.bias_map) {
#pragma unroll
      for (int o = 0; o < 4; ++o) y[o] += a.bias_map[pix[o] * a.sbm + col];
    }
#pragma unroll
    for (int o = 0; o < 4; ++o) conv_epilogue_store<EPI>(a, pix[o], col, y[o]);
  }
}

// U_ξ = Σ_j G[ξ][j]·g[j] (fp64) per (co, ci), packed [nb32][stage][ξ][q][lane][4] with
// lane = li + 32·hh ↔ co = 32·nb32 + li, padded channel kc = 16·stage + 8·q + 4·hh + e.
__global__ void wino5_pack_kernel(const float* __restrict__ w, float* __restrict__ out, int cout,
                                  int c0, int c1, int cp0, int nst, long long total) {
  const double Gm[8][5] = {{-1.0, 0.0, 0.0, 0.0, 0.0},
                           {-2.0 / 9, -2.0 / 9, -2.0 / 9, -2.0 / 9, -2.0 / 9},
                           {-2.0 / 9, 2.0 / 9, -2.0 / 9, 2.0 / 9, -2.0 / 9},
                           {1.0 / 90, 1.0 / 45, 2.0 / 45, 4.0 / 45, 8.0 / 45},
                           {1.0 / 90, -1.0 / 45, 2.0 / 45, -4.0 / 45, 8.0 / 45},
                           {32.0 / 45, 16.0 / 45, 8.0 / 45, 4.0 / 45, 2.0 / 45},
                           {32.0 / 45, -16.0 / 45, 8.0 / 45, -4.0 / 45, 2.0 / 45},
                           {0.0, 0.0, 0.0, 0.0, 1.0}};
  const int cin = c0 + c1;
  for (long long idx = blockIdx.x * 256LL + threadIdx.x; idx < total; idx += (long long)gridDim.x * 256) {
    long long r = idx;
    const int e = (int)(r & 3); r >>= 2;
    const int lane = (int)(r & 63); r >>= 6;
    const int q = (int)(r & 1); r >>= 1;
    const int xi = (int)(r & 7); r >>= 3;
    const int s = (int)(r % nst);
    const int nb = (int)(r / nst);
    const int o = nb * 32 + (lane & 31);
    const int kc = s * W5KC + 8 * q + 4 * (lane >> 5) + e;
    int ci = -1;
    if (kc < cp0) {
      if (kc < c0) ci = kc;
    } else if (kc - cp0 < c1) {
      ci = c0 + (kc - cp0);
    }
    float v = 0.f;
    if (o < cout && ci >= 0) {
      const float* g = w + ((size_t)o * cin + ci) * 5;
      double acc = 0.0;
      for (int j = 0; j < 5; ++j) acc += Gm[xi][j] * (double)g[j];
      v = (float)acc;
    }
    out[idx] = v;
  }
}
