// Grouped launches of two independent convolutions (round 6) — included by conv.hip (in an
// anonymous namespace).  The decoder's iteration tail runs two short branches side by side — the
// flow predictor → Δflow encoder (3×3 256→2, 7×7 2→128, 3×3 128→64) and the mask predictor → mask
// encoder (1×1 256→1, 3×3 1→64, 3×3 64→32) (scflow_decoder.py:211-218).  Each of those launches
// is a one-round grid of at most one workgroup per CU, and the branches ran on two HIP streams
// joined by events whose fork and join cost 5–10 µs of queue time each.  Pairing the branches'
// k-th launches into ONE grid — workgroups [0, n_a) run conv a's body, the rest conv b's — keeps
// both on one stream with no events and gives each CU a second workgroup.  Each half runs
// exactly the body scflow_conv2d launches for it (same plan), so results are bit-identical to
// two separate launches.

// thin: the flow predictor's 3×3 contraction (conv_thinz.h) beside the mask predictor's 1×1
// chunked kernel
template <int W, int R>
__global__ __launch_bounds__(256, 2) void thin_pair_kernel(scflow_conv_args f, scflow_conv_args m,
                                                           int oh, int ow, int nf) {
  if ((int)blockIdx.x < nf)
    conv_thinz_body<2, 3, 3, W, R>(f, blockIdx.x, nf);
  else
    conv_thin_body<1, 1, 1>(m, oh, ow, (int)blockIdx.x - nf, (int)gridDim.x - nf);
}

// small-cin: the Δflow encoder's 7×7 2→128 beside the mask encoder's 3×3 1→64
__global__ __launch_bounds__(256, 2) void smallcin_pair_kernel(scflow_conv_args a, scflow_conv_args b,
                                                               int oh, int ow, int na, int nta,
                                                               int ntb, unsigned long long* stamps) {
  if ((int)blockIdx.x < na)
    conv_smallcin_mfma_body<2, 7, 7, 2>(a, oh, ow, 128, nta, blockIdx.x, na, 0, stamps, blockIdx.x);
  else
    conv_smallcin_mfma_body<1, 3, 3, 1>(b, oh, ow, 64, ntb, (int)blockIdx.x - na,
                                        (int)gridDim.x - na, 0, stamps, blockIdx.x);
}

// F(2×2,3×3): two Winograd convs of one width (the encoders' second layers), logical grids
// gxa × gya and gxb × gyb flattened
template <int W, int NA, int NB>
__global__ __launch_bounds__(256, 2) void wino_pair_kernel(WinoParams pa, WinoParams pb, int gxa,
                                                           int gya, int gxb, int gyb) {
  const int L = blockIdx.x, na = gxa * gya;
  if (L < na)
    conv_wino_body<W, NA>(pa, L % gxa, L / gxa, gxa, gya, L);
  else
    conv_wino_body<W, NB>(pb, (L - na) % gxb, (L - na) / gxb, gxb, gyb, L);
}

// plans (the same conditions scflow_conv2d applies; a plan that does not hold leaves the pair
// to two ordinary launches)
struct SmallcinPlan {
  int ci = 0, k = 0, npad = 0, ntiles = 0;
  unsigned blocks = 0;
  size_t lds = 0;
};
bool smallcin_plan(const scflow_conv_args& a, SmallcinPlan& p) {
  if (a.bk == SCFLOW_CONV_WINO || a.bk == SCFLOW_CONV_WINO4 || a.bk == SCFLOW_CONV_1X1W ||
      a.epilogue != SCFLOW_EPI_PLAIN || a.bias_map || has_fused_norm(a) || a.c1 != 0)
    return false;
  const Geometry g = select_variant(a.cout, a.c0, a.c1, a.kh, a.kw, a.stride, a.h, a.w, a.ph, a.pw);
  if (g.variant != V_SMALLCIN) return false;
  const bool mfma_ok = (g.ow == 32 || g.ow == 64) && g.ow == a.w && g.oh == a.h &&
                       g.oh % (64 / g.ow) == 0 && (g.npad == 64 || g.npad == 128) &&
                       (long long)a.n * a.h * a.w * a.s0 * 4 < 0x7ffffff0LL;
  if (!mfma_ok || (g.npad == 128 && smallcin_split())) return false;
  p.ci = a.c0;
  p.k = a.kh == a.kw ? a.kh : 0;
  p.npad = g.npad;
  p.ntiles = a.n * (g.oh / (64 / g.ow));
  p.blocks = (unsigned)smallcin_blocks(p.ntiles);
  p.lds = 2 * sizeof(float) * (size_t)(64 / g.ow + a.kh - 1) * (g.ow + a.kw - 1) * a.c0;
  return true;
}

bool wino_plan(const scflow_conv_args& a, WinoParams& p, int& nbw, int& gx, int& gy) {
  if (a.bk != SCFLOW_CONV_WINO || a.kh != 3 || !wino_launchable(a)) return false;
  if (!aligned16(a.src0) || (a.s0 & 3) || (a.c1 > 0 && (!aligned16(a.src1) || (a.s1 & 3))) ||
      !aligned16(a.weight) || (a.w != 32 && a.w != 64))
    return false;
  nbw = wino_nbw(a, device_cus());
  if (nbw != 1 && nbw != 2) return false;
  p.a = a;
  p.cp0 = round_up(a.c0, WSC);
  p.nst = (p.cp0 + round_up(a.c1, WSC)) / WSC;
  p.swz_c = 0;  // block order only: the logical grid is not dealt to XCDs in linear order here
  p.stamps = g_wino_stamps;
  const int orows = a.w == 32 ? WinoGeom<32>::OROWS : WinoGeom<64>::OROWS;
  const int xb = a.w == 32 ? WinoGeom<32>::XB : WinoGeom<64>::XB;
  gx = a.n * (a.h / orows) * xb;
  gy = round_up(a.cout, 32 * nbw) / (32 * nbw);
  return true;
}

template <int W, int NA, int NB>
int launch_wino_pair(const WinoParams& pa, const WinoParams& pb, int gxa, int gya, int gxb, int gyb,
                     hipStream_t st) {
  const size_t la = wino_lds_bytes<W, NA>(), lb = wino_lds_bytes<W, NB>();
  const size_t lds = la > lb ? la : lb;
  static bool attr = false;
  if (lds > 64 * 1024 && !attr) {
    (void)hipFuncSetAttribute((const void*)wino_pair_kernel<W, NA, NB>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  wino_pair_kernel<W, NA, NB><<<gxa * gya + gxb * gyb, 256, lds, st>>>(pa, pb, gxa, gya, gxb, gyb);
  return scflow_launch_status();
}

// the grouped launch of (a, b) if one exists (returns 1 after launching, 0 if none applies, < 0
// or a hipError on failure)
int try_pair(const scflow_conv_args& a, const scflow_conv_args& b, hipStream_t st) {
  // thin: a = 3×3 → 2 contraction, b = 1×1 → 1 chunked
  {
    const Geometry ga = select_variant(a.cout, a.c0, a.c1, a.kh, a.kw, a.stride, a.h, a.w, a.ph, a.pw);
    const Geometry gb = select_variant(b.cout, b.c0, b.c1, b.kh, b.kw, b.stride, b.h, b.w, b.ph, b.pw);
    const auto tiled = [](const scflow_conv_args& c, const Geometry& g) {
      return (g.ow == 32 || g.ow == 64) && (c.c0 % 8) == 0 && (c.c1 % 8) == 0 &&
             g.oh % (64 / g.ow) == 0 && g.ow == c.w && g.oh == c.h;
    };
    if (ga.variant == V_THIN && gb.variant == V_THIN && a.bk != SCFLOW_CONV_WINO &&
        b.bk != SCFLOW_CONV_WINO && a.epilogue == SCFLOW_EPI_PLAIN && !a.bias_map &&
        b.epilogue == SCFLOW_EPI_PLAIN && !b.bias_map && a.cout == 2 && thinz_ok(a, ga, tiled(a, ga)) &&
        b.cout == 1 && b.kh == 1 && b.kw == 1 && b.c1 == 0 && b.stride == 1 && tiled(b, gb) &&
        aligned16(b.src0) && (b.s0 & 3) == 0 && a.n == b.n && a.h == b.h && a.w == b.w) {
      const int R = ga.ow == 64 ? 4 : 2;
      const int nf = a.n * (ga.oh / R);
      const int nm = b.n * (gb.oh / (64 / gb.ow));
      size_t lds = sizeof(float) * (size_t)(64 / gb.ow) * gb.ow * THIN_LD;
      if (lds < sizeof(float) * 4 * 64) lds = sizeof(float) * 4 * 64;
      lds += sizeof(float) * (size_t)b.c0;  // the 1×1's weights
      if (ga.ow == 64)
        thin_pair_kernel<64, 4><<<nf + nm, 256, lds, st>>>(a, b, gb.oh, gb.ow, nf);
      else
        thin_pair_kernel<32, 2><<<nf + nm, 256, lds, st>>>(a, b, gb.oh, gb.ow, nf);
      const int e = scflow_launch_status();
      return e ? e : 1;
    }
  }
  // small-cin: a = 7×7 2 → 128, b = 3×3 1 → 64
  {
    SmallcinPlan pa, pb;
    if (smallcin_plan(a, pa) && smallcin_plan(b, pb) && pa.ci == 2 && pa.k == 7 && pa.npad == 128 &&
        pb.ci == 1 && pb.k == 3 && pb.npad == 64 && a.h == b.h && a.w == b.w) {
      const size_t lds = pa.lds > pb.lds ? pa.lds : pb.lds;
      smallcin_pair_kernel<<<pa.blocks + pb.blocks, 256, lds, st>>>(
          a, b, a.h, a.w, (int)pa.blocks, pa.ntiles, pb.ntiles, g_wino_stamps);
      const int e = scflow_launch_status();
      return e ? e : 1;
    }
  }
  // F(2×2,3×3) of one width
  {
    WinoParams pa, pb;
    int na, nb, gxa, gya, gxb, gyb;
    if (wino_plan(a, pa, na, gxa, gya) && wino_plan(b, pb, nb, gxb, gyb) && a.w == b.w) {
      int e;
      if (a.w == 32) {
        e = na == 1 ? (nb == 1 ? launch_wino_pair<32, 1, 1>(pa, pb, gxa, gya, gxb, gyb, st)
                               : launch_wino_pair<32, 1, 2>(pa, pb, gxa, gya, gxb, gyb, st))
                    : (nb == 1 ? launch_wino_pair<32, 2, 1>(pa, pb, gxa, gya, gxb, gyb, st)
                               : launch_wino_pair<32, 2, 2>(pa, pb, gxa, gya, gxb, gyb, st));
      } else {
        e = na == 1 ? (nb == 1 ? launch_wino_pair<64, 1, 1>(pa, pb, gxa, gya, gxb, gyb, st)
                               : launch_wino_pair<64, 1, 2>(pa, pb, gxa, gya, gxb, gyb, st))
                    : (nb == 1 ? launch_wino_pair<64, 2, 1>(pa, pb, gxa, gya, gxb, gyb, st)
                               : launch_wino_pair<64, 2, 2>(pa, pb, gxa, gya, gxb, gyb, st));
      }
      return e ? e : 1;
    }
  }
  return 0;
}
