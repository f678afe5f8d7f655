// 1×1 weight gradient (stride 1 or 2, no padding) — included by train.hip (inside its anonymous
// namespace) after the direct implicit-GEMM kernel, whose split reduction it shares.  Training
// step: the MotionEncoder's corr_net.0 (324 → 256, one batched launch over the decoder's 8
// iterations, raft_decoder.py:75-85 under SCFlowRefiner.loss → backward) and the encoders' 1×1
// downsample convs.
//
//   dW[co][ci] = Σ_p dY[p][co] · X[in(p)][ci],   db[co] = Σ_p dY[p][co]
//
// a GEMM whose contraction runs over the pixels.  On the direct kernel a 1×1 shape gives each
// wave ONE 32×32 accumulator, so every MFMA waits on its own two LDS reads (36 TF at corr_net.0's
// shape).  Here a workgroup owns 128 co × 128 ci, 4 waves of 64 co × 64 ci = 2 × 2 accumulators:
// per k-step (2 pixels) a lane reads two dY and two X values (ds_read_b32 of its channel, the
// two 32-lane halves on consecutive pixels: conflict-free) and issues 4 independent MFMAs, with
// the next k-step's reads in flight.  Pixels are staged 16 at a time in channels-last rows (the
// global layout: one float4 of 4 channels per lane, coalesced), double-buffered, one barrier per
// stage, the next stage's global loads in registers during this stage's MFMAs.  The pixel walk
// is split into runs inside one segment each (the batched call's per-iteration pairs): partial
// sums [split][copad][cinp] (+ the bias [split][copad]) → wgrad_reduce_kernel, fixed order.

constexpr int W1_T = 128;  // co and ci per workgroup
constexpr int W1_P = 16;   // pixels per stage
constexpr int W1_L = 128;  // LDS row (floats): one pixel's 128 channels

struct W1Params {
  scflow_wgrad_args a;
  int oh, ow, cin, co_tiles, ci_tiles, copad, cinp;
  int nseg, spl;     // segments, splits per segment (grid.y = nseg · spl)
  long long seg_pix; // output pixels per segment
  long long pps;     // pixels per split (a multiple of W1_P)
  long long max_splits;  // the workspace bound (any segment count ≤ WG_MAXSEG)
  WgSegs sg;
};

template <int S>
__global__ __launch_bounds__(256, 2) void wgrad_1x1_kernel(W1Params P, float* __restrict__ slab,
                                                           float* __restrict__ bslab) {
  __shared__ float Ds[2][W1_P][W1_L];
  __shared__ float Xs[2][W1_P][W1_L];
  __shared__ float bred[256];
  const scflow_wgrad_args& a = P.a;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 31, hh = lane >> 5;
  const int wco = wave & 1, wci = wave >> 1;
  const int co_t = blockIdx.x % P.co_tiles, ci_t = blockIdx.x / P.co_tiles;
  const int co0 = co_t * W1_T, ci0 = ci_t * W1_T;
  const int seg = blockIdx.y / P.spl, sp = blockIdx.y - seg * P.spl;
  const long long p0 = sp * P.pps;
  const long long p1 = p0 + P.pps < P.seg_pix ? p0 + P.pps : P.seg_pix;
  const int nstage = p1 > p0 ? (int)((p1 - p0 + W1_P - 1) / W1_P) : 0;
  const float* dy = wg_pick(P.sg.dy, seg);
  const float* x0 = wg_pick(P.sg.src0, seg);
  const float* x1 = wg_pick(P.sg.src1, seg);
  const bool do_bias = bslab != nullptr && ci_t == 0;

  // staging: float4 j of this thread is (pixel tid/32 + 8j, channel quad tid%32) of the stage
  const int q4 = 4 * (tid & 31), pr = tid >> 5;
  const int co_l = co0 + q4, ci_l = ci0 + q4;
  const bool co_ok = co_l < a.cout, ci_ok = ci_l < P.cin;
  const float* xsrc = ci_l < a.cin0 ? x0 + ci_l : x1 + (ci_l - a.cin0);
  const int xs = ci_l < a.cin0 ? a.s0 : a.s1;
  floatx4 rd[2], rx[2];
  auto gload = [&](int st) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const long long p = p0 + (long long)st * W1_P + pr + 8 * j;
      const bool ok = p < p1;
      floatx4 d = {0.f, 0.f, 0.f, 0.f}, x = {0.f, 0.f, 0.f, 0.f};
      if (ok && co_ok) d = *(const floatx4*)(dy + p * a.sdy + co_l);
      if (ok && ci_ok) {
        long long ip = p;
        if (S != 1) {  // output pixel → its input pixel (stride S, no padding)
          const long long ohw = (long long)P.oh * P.ow;
          const long long img = p / ohw;
          const int rem = (int)(p - img * ohw);
          const int oy = rem / P.ow, ox = rem - oy * P.ow;
          ip = (img * a.h + (long long)oy * S) * a.w + (long long)ox * S;
        }
        x = *(const floatx4*)(xsrc + ip * xs);
      }
      rd[j] = d;
      rx[j] = x;
    }
  };
  auto lstore = [&](int b) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      *(floatx4*)&Ds[b][pr + 8 * j][q4] = rd[j];
      *(floatx4*)&Xs[b][pr + 8 * j][q4] = rx[j];
    }
  };

  floatx16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][k][e] = 0.f;
  float bsum = 0.f;

  const int ca = wco * 64 + li, cb = wci * 64 + li;
  if (nstage > 0) {
    gload(0);
    lstore(0);
    __syncthreads();
  }
  for (int st = 0; st < nstage; ++st) {
    const int b = st & 1;
    if (st + 1 < nstage) gload(st + 1);
    if (do_bias)  // thread: channel tid % 128, every other pixel of the stage
#pragma unroll
      for (int p = tid >> 7; p < W1_P; p += 2) bsum += Ds[b][p][tid & 127];
    // k-step k: pixels 2k (lanes 0–31) and 2k + 1 (lanes 32–63); operands one k-step ahead
    float a0 = Ds[b][hh][ca], a1 = Ds[b][hh][ca + 32];
    float b0 = Xs[b][hh][cb], b1 = Xs[b][hh][cb + 32];
#pragma unroll
    for (int k = 0; k < W1_P / 2; ++k) {
      float na0 = 0.f, na1 = 0.f, nb0 = 0.f, nb1 = 0.f;
      if (k + 1 < W1_P / 2) {
        const int pn = 2 * (k + 1) + hh;
        na0 = Ds[b][pn][ca];
        na1 = Ds[b][pn][ca + 32];
        nb0 = Xs[b][pn][cb];
        nb1 = Xs[b][pn][cb + 32];
      }
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
      a0 = na0;
      a1 = na1;
      b0 = nb0;
      b1 = nb1;
    }
    if (st + 1 < nstage) lstore(b ^ 1);
    __syncthreads();
  }

  // partial slab [split][copad][cinp]; C/D layout: col = lane&31 (ci), row = (r&3)+8(r>>2)+4hh (co)
  float* sl = slab + (size_t)blockIdx.y * P.copad * P.cinp;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int ci = ci0 + wci * 64 + k * 32 + li;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = co0 + wco * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
        sl[(size_t)co * P.cinp + ci] = acc[i][k][r];
      }
    }
  if (do_bias) {
    bred[tid] = bsum;
    __syncthreads();
    if (tid < W1_T) bslab[(size_t)blockIdx.y * P.copad + co0 + tid] = bred[tid] + bred[tid + 128];
  }
}

bool w1_geometry(const scflow_wgrad_args& a, int nseg, W1Params* P) {
  static const bool off = [] {
    const char* e = getenv("SCFLOW_WGRAD_1X1");
    return e && e[0] == '0';
  }();
  if (off) return false;
  if (a.kh != 1 || a.kw != 1 || a.ph != 0 || a.pw != 0 || (a.stride != 1 && a.stride != 2))
    return false;
  const int cin = a.cin0 + a.cin1;
  // float4 staging: channel counts, strides and bases 16-B aligned; the thin kernels take ≤ 4
  if (a.cout <= 4 || cin <= 4 || a.cout % 4 || a.sdy % 4 || !aligned16(a.dy) || a.cin0 % 4 ||
      a.s0 % 4 || !aligned16(a.src0) ||
      (a.cin1 > 0 && (a.cin1 % 4 || a.s1 % 4 || !aligned16(a.src1))))
    return false;
  P->a = a;
  P->cin = cin;
  P->oh = (a.h - 1) / a.stride + 1;
  P->ow = (a.w - 1) / a.stride + 1;
  P->co_tiles = (a.cout + W1_T - 1) / W1_T;
  P->ci_tiles = (cin + W1_T - 1) / W1_T;
  P->copad = P->co_tiles * W1_T;
  P->cinp = P->ci_tiles * W1_T;
  P->nseg = nseg;
  P->seg_pix = (long long)(a.n / nseg) * P->oh * P->ow;
  // two workgroups per CU, the partial slabs under 8 Mi floats, ≥ 4 stages per split
  const int tiles = P->co_tiles * P->ci_tiles;
  long long want = (2LL * device_cus() + tiles - 1) / tiles;
  const long long per_split = (long long)P->copad * P->cinp;
  if (want > (8LL << 20) / per_split) want = (8LL << 20) / per_split;
  if (want < 1) want = 1;
  // the workspace query sees the whole walk as one segment: size it for any segment count
  P->max_splits = want > WG_MAXSEG ? want : WG_MAXSEG;
  long long spl = want / nseg;
  const long long max_spl = (P->seg_pix + 4 * W1_P - 1) / (4 * W1_P);
  if (spl > max_spl) spl = max_spl;
  if (spl < 1) spl = 1;
  P->pps = (P->seg_pix + spl - 1) / spl;
  P->pps = (P->pps + W1_P - 1) / W1_P * W1_P;
  P->spl = (int)((P->seg_pix + P->pps - 1) / P->pps);
  return true;
}

// floats of partial sums for any segment count (scflow_conv_wgrad_workspace)
long long w1_workspace(const W1Params& P) {
  return P.max_splits * ((long long)P.copad * P.cinp + P.copad);
}

int w1_launch(const W1Params& P, hipStream_t st) {
  const scflow_wgrad_args& a = P.a;
  const int splits = P.nseg * P.spl;
  if (a.workspace_floats < (long long)splits * ((long long)P.copad * P.cinp + P.copad))
    return SCFLOW_EINVAL;
  float* slab = a.workspace;
  float* bslab = a.db ? a.workspace + (size_t)splits * P.copad * P.cinp : nullptr;
  const dim3 grid((unsigned)(P.co_tiles * P.ci_tiles), (unsigned)splits);
  if (a.stride == 1)
    wgrad_1x1_kernel<1><<<grid, 256, 0, st>>>(P, slab, bslab);
  else
    wgrad_1x1_kernel<2><<<grid, 256, 0, st>>>(P, slab, bslab);
  int rc = scflow_launch_status();
  if (rc != SCFLOW_OK) return rc;
  int lg = 0;  // as wgrad_direct_launch: 2^lg lanes of partial sums per output
  while (lg < 4 && (4 << lg) < splits) ++lg;
  const int opb = 256 >> lg;
  const unsigned rblocks = (unsigned)(((long long)a.cout * P.cinp + opb - 1) / opb +
                                      (a.db ? (a.cout + opb - 1) / opb : 0));
  wgrad_reduce_kernel<<<rblocks, 256, 0, st>>>(slab, bslab, a.dw, a.db, splits, a.cout, P.cin, 1,
                                               P.copad, P.cinp, a.accumulate, lg);
  return scflow_launch_status();
}
