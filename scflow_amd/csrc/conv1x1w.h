// Wide 1×1 convolution (MotionEncoder corr_net.0, 324 → 256 + ReLU; reference
// models/decoder/raft_decoder.py:75-85,152-166) — included by conv.hip (inside its anonymous
// namespace, after conv_wino.h, whose buffer-load helpers it uses).
//
// The GEMM out[m][co] = act(Σ_k A[m][k]·W[co][k] + b[co]) with a workgroup owning 64 pixels × ALL
// output channels (≤ 256): the A tile of every input channel (64 × K ≤ 512) sits in LDS for the
// whole launch — loaded once, in NC chunks whose loads overlap the previous chunk's MFMAs, with one
// barrier per chunk — and the weights stream from L2 straight into registers, pre-packed in
// MFMA-lane order (one 1 KiB b128 load per 32 output channels and 8 input channels), prefetched
// PD 8-channel blocks ahead.  Each of the 4 waves owns 64 output channels × the 64 pixels (2 × 2
// blocks of v_mfma_f32_32x32x2_f32, 16 MFMAs per 8 channels and nothing else in the loop but two
// LDS reads and two buffer loads).  One workgroup per CU (256 at B = 16, 32² features): the
// MFMA pipe of each SIMD runs one wave's independent accumulator chains back to back, instead of
// conv1x1_kernel's 128 × 64 tiles with two barriers per 16 channels (0.45 of the fp32 peak).
//
// LDS rows are K + 4 floats (≡ 4·odd mod 64 words): the b128 A reads of a 16-lane group (16
// different pixels, same channels) hit distinct banks.

constexpr int W1_PX = 64;  // pixels per workgroup
#ifndef W1_PD_DEF
#define W1_PD_DEF 4
#endif
constexpr int W1_PD = W1_PD_DEF;  // weight blocks (8 channels) in flight ahead of the MFMAs
constexpr int W1_NC = 3;   // A-tile chunks

// packed weights: [nb32 = npad/32][kb = K/8][lane 64][4]; lane (li, hh) ↔ output channel
// 32·nb32 + li, input channel 8·kb + 4·hh + e (zero beyond cin / cout)
__global__ void conv1x1w_pack_kernel(const float* __restrict__ w, float* __restrict__ out, int cout,
                                     int cin, int kb, long long total) {
  for (long long idx = blockIdx.x * 256LL + threadIdx.x; idx < total; idx += (long long)gridDim.x * 256) {
    long long r = idx;
    const int e = (int)(r & 3); r >>= 2;
    const int lane = (int)(r & 63); r >>= 6;
    const int k8 = (int)(r % kb);
    const int nb = (int)(r / kb);
    const int o = nb * 32 + (lane & 31);
    const int ci = k8 * 8 + 4 * (lane >> 5) + e;
    out[idx] = (o < cout && ci < cin) ? w[(size_t)o * cin + ci] : 0.f;
  }
}

// KB = 8-channel blocks of the padded K; NW = waves (= output channel blocks of 64)
template <int KB>
constexpr size_t conv1x1w_lds_bytes() {
  return sizeof(float) * (size_t)W1_PX * (8 * KB + 4);
}

template <int KB>
__global__ __launch_bounds__(256, 1) void conv1x1w_kernel(scflow_conv_args a) {
  constexpr int KP = 8 * KB + 4;        // LDS row (floats)
  constexpr int Q = 2 * KB;             // float4 per A row
  constexpr int CB = (KB + W1_NC - 1) / W1_NC;  // 8-channel blocks per chunk (last may be short)
  constexpr int NLD = (W1_PX * 2 * CB + 255) / 256;  // float4 per thread per chunk
  extern __shared__ floatx4 smem4[];
  float* As = (float*)smem4;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 31, hh = lane >> 5;
  const long long M = (long long)a.n * a.h * a.w;
  const long long m0 = (long long)blockIdx.x * W1_PX;
  const int npad = (a.cout + 63) / 64 * 64;
  const bool wave_on = wave * 64 < npad;  // waves beyond the padded channels only load A
  // the lane's two output channels' bias, fetched now (in the one-round grid every workgroup
  // reaches the epilogue together, where these loads waited on the same cache lines)
  float bias_v[2] = {0.f, 0.f};
  if (wave_on && a.bias) {
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      const int col = 64 * wave + 32 * nb + (lane & 31);
      if (col < a.cout) bias_v[nb] = a.bias[col];
    }
  }

  // A chunk c = 8-channel blocks [c·CB, min(KB, (c+1)·CB)): thread slot j is (pixel, quad) =
  // (idx / (2·nb), idx % (2·nb)), idx = tid + 256 j
  const __amdgpu_buffer_rsrc_t asrc =
      wino_rsrc(a.src0, (unsigned)(((M - 1) * a.s0 + a.c0) * 4));
  floatx4 ra[NLD];
  auto aload = [&](int c) {
    const int b0 = c * CB, nb = (KB - b0 < CB ? KB - b0 : CB);
#pragma unroll
    for (int j = 0; j < NLD; ++j) {
      const int idx = tid + 256 * j;
      const int px = idx / (2 * nb), q = 2 * b0 + idx % (2 * nb);
      const long long m = m0 + px;
      const bool ok = idx < W1_PX * 2 * nb && m < M && 4 * q < a.c0;
      ra[j] = wino_bload(asrc, ok ? (int)((m * a.s0 + 4 * q) * 4) : WINO_OOB, 0);
    }
  };
  auto astore = [&](int c) {
    const int b0 = c * CB, nb = (KB - b0 < CB ? KB - b0 : CB);
#pragma unroll
    for (int j = 0; j < NLD; ++j) {
      const int idx = tid + 256 * j;
      if (idx < W1_PX * 2 * nb) {
        const int px = idx / (2 * nb), q = 2 * b0 + idx % (2 * nb);
        *(floatx4*)(As + px * KP + 4 * q) = ra[j];
      }
    }
  };

  // this wave's weights: output channels 64·wave .. +63 (two 32-blocks)
  const __amdgpu_buffer_rsrc_t wsrc = wino_rsrc(a.weight + (size_t)(2 * wave) * KB * 256,
                                                (unsigned)(wave_on ? 2 * KB * 1024 : 0));
  auto bload = [&](floatx4(&b)[2], int kb) {
    const int k = kb < KB ? kb : KB - 1;
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) b[nb] = wino_bload(wsrc, lane * 16, (nb * KB + k) * 1024);
  };

  floatx16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  floatx4 bq[W1_PD][2];
#pragma unroll
  for (int d = 0; d < W1_PD; ++d) bload(bq[d], d);
  aload(0);
  astore(0);
  __syncthreads();
  const float* ar0 = As + li * KP + 4 * hh;
  const float* ar1 = As + (32 + li) * KP + 4 * hh;
  // every block as straight-line code (StaticFor): compile-time ring slots and chunk points.  A
  // block's A fragments are read one block ahead (during the previous block's MFMAs) unless it
  // opens a chunk, whose rows are published by the barrier right before it.
  floatx4 an0, an1;
  auto body = [&](auto kbc) {
    constexpr int kb = decltype(kbc)::value;
    constexpr int c = kb / CB, kc = kb % CB, sl = kb % W1_PD;
    constexpr bool opens = kb == 0 || (kc == 0);  // first block of a chunk: read here
    constexpr bool last_of_chunk = c + 1 < W1_NC && kc == CB - 1 && (c + 1) * CB < KB;
    // the next chunk's A loads go out two blocks into this chunk (the weight loads already in
    // flight cover their latency); they are stored and published at the chunk's last block
    if constexpr (c + 1 < W1_NC && kc == 2 && (c + 1) * CB < KB) aload(c + 1);
    if constexpr (opens) {
      an0 = *(const floatx4*)(ar0 + 8 * kb);
      an1 = *(const floatx4*)(ar1 + 8 * kb);
    }
    const floatx4 a0 = an0, a1 = an1;
    floatx4 b[2] = {bq[sl][0], bq[sl][1]};
    if constexpr (kb + W1_PD < KB) bload(bq[sl], kb + W1_PD);
    if constexpr (kb + 1 < KB && !last_of_chunk) {
      an0 = *(const floatx4*)(ar0 + 8 * (kb + 1));
      an1 = *(const floatx4*)(ar1 + 8 * (kb + 1));
    }
    __builtin_amdgcn_sched_barrier(0);  // the prefetches stay ahead of this block's MFMAs
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[e], b[0][e], acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[e], b[1][e], acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[e], b[0][e], acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[e], b[1][e], acc[1][1], 0, 0, 0);
    }
    if constexpr (last_of_chunk) {
      astore(c + 1);
      __syncthreads();
    }
    // keep each block's loads where they are issued: the scheduler otherwise sinks them towards
    // their uses W1_PD blocks later, which turns the prefetch into a wait per block
    __builtin_amdgcn_sched_barrier(0);
  };
  StaticFor<0, KB>::run(body);

  // epilogue; C/D layout: col = lane&31, row = (r&3) + 8(r>>2) + 4(lane>>5); all global reads
  // (bias map) before any store
  if (!wave_on) return;
#pragma unroll
  for (int nb = 0; nb < 2; ++nb) {
    const int col = 64 * wave + 32 * nb + li;
    if (col >= a.cout) continue;
    const float bias = bias_v[nb];
    float v[2][16];
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
#pragma unroll
      for (int r = 0; r < 16; ++r) v[mb][r] = acc[mb][nb][r] + bias;
    if (a.bias_map) {
#pragma unroll
      for (int mb = 0; mb < 2; ++mb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const long long m = m0 + 32 * mb + (r & 3) + 8 * (r >> 2) + 4 * hh;
          if (m < M) v[mb][r] += a.bias_map[m * a.sbm + col];
        }
    }
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const long long m = m0 + 32 * mb + (r & 3) + 8 * (r >> 2) + 4 * hh;
        if (m < M) a.out[m * a.so + col] = act_apply(v[mb][r], a.act);
      }
  }
}
