/*
 * scflow_hip.h — C ABI of the MI355X (gfx950) SCFlow refinement hot path.
 *
 * One shared library, libscflow_hip.so (scflow_amd/lib/), built with
 * `hipcc --offload-arch=gfx950`.  Every entry point:
 *   - takes plain device pointers (fp32 unless stated), sizes and a hipStream_t passed as void*;
 *   - enqueues work on that stream and returns immediately (no host sync, no allocation, so
 *     callers may capture the calls into a hipGraph);
 *   - returns 0 on success, a negative SCFLOW_E* code for an argument/shape error (nothing
 *     launched), or a positive hipError_t if the launch failed;
 *   - is stateless and re-entrant (one process per GPU is the intended deployment).
 * The caller owns every buffer.  Tensors are contiguous unless a stride argument says otherwise.
 *
 * Reference interfaces replaced (GiaKhangLuu/SCFlow, /root/reference):
 *   scflow_corr_pyramid      <- CorrelationPyramid.forward      models/decoder/raft_decoder.py:35-58
 *   scflow_corr_lookup       <- CorrLookup.forward              models/utils/corr_lookup.py:102-136
 *   scflow_conv2d (+ GRU epilogues) <- ConvGRU.forward          models/decoder/raft_decoder.py:235-253
 *                               and the ConvModule convs of MotionEncoder / XHead / the decoder's
 *                               delta-flow and mask encoders (raft_decoder.py:152-166, 256-294;
 *                               scflow_decoder.py:103-124)
 *   scflow_pose_update       <- get_pose_from_delta_pose (ortho6d, exp)  models/utils/pose.py:124-169
 *   scflow_lift_points       <- cal_3d_2d_corr / lift_2d_to_3d            models/utils/pose.py:26-64
 *   scflow_pose_flow         <- get_flow_from_delta_pose_and_points       models/utils/pose.py:66-88
 *   scflow_pose_update_flow  <- the two calls above fused, as used at     scflow_decoder.py:231-244
 *   scflow_flow_downsample   <- 1/8·F.interpolate(flow, 1/8, bilinear, align_corners=True)  scflow_decoder.py:197-198
 *   scflow_flow_upsample     <- 8·F.interpolate(flow+Δflow, ×8) and mask ×8 (same)          scflow_decoder.py:223-228
 *   scflow_pose_step         <- one iteration's tail fused: pose update + pose flow + the ×8
 *                               prediction + the next iteration's ↓8 flow   scflow_decoder.py:197-198, 223-244
 *   scflow_transpose         <- layout plumbing (NCHW <-> channels-last slices), no reference equivalent
 *   scflow_ph_*              <- MultiClassPoseHead.forward                models/head/pose_head.py:201-211
 *   scflow_enc_*             <- RAFTEncoder.forward (Basic; IN / BN)      models/encoder/raft_encoder.py:286-314
 *   scflow_gemm_f32          <- torch.matmul / F.linear in the training step's adjoints (raft_decoder.py:35-58,
 *                               pose_head.py:201-211)
 */
#ifndef SCFLOW_HIP_H
#define SCFLOW_HIP_H

#ifdef __cplusplus
extern "C" {
#endif

#define SCFLOW_OK 0
#define SCFLOW_EINVAL (-1)      /* null pointer / non-positive size / bad enum */
#define SCFLOW_EUNSUPPORTED (-2) /* valid call, but a shape this build has no kernel for */
#define SCFLOW_EALIGN (-3)      /* pointer or stride not 16-byte aligned where float4 access is used */

#define SCFLOW_ACT_NONE 0
#define SCFLOW_ACT_RELU 1
#define SCFLOW_ACT_SIGMOID 2
#define SCFLOW_ACT_TANH 3

#define SCFLOW_EPI_PLAIN 0  /* out = act(conv + bias) */
#define SCFLOW_EPI_GRU_ZR 1 /* cout = 2·hc: z = σ(.) -> gate[:, :hc];  r = σ(.), rh = r·h -> rh   */
#define SCFLOW_EPI_GRU_Q 2  /* cout = hc:   q = tanh(.);  hid <- (1-z)·hid + z·q  (z from gate)     */

/* pose-update mode word (the depth_transform argument of scflow_pose_update / _update_flow /
 * _step): bit 0 = depth transform (0 'exp', 1 linear); | SCFLOW_POSE_QUAT_XYZW = the delta
 * rotation is a quaternion (x, y, z, w) [n][4] (pose.py:132-133) instead of ortho6d [n][6]. */
#define SCFLOW_POSE_QUAT_XYZW 16

#define SCFLOW_LAYOUT_NCHW 0 /* [N][C][H][W] */
#define SCFLOW_LAYOUT_NHWC 1 /* [N][H][W][stride], channels contiguous */

int scflow_version(void);
const char* scflow_strerror(int code);

/* a1: all-pairs correlation volume and its average-pooled pyramid.
 * f1, f2: [n][c][h][w] (render, real).  pyr: one buffer holding the levels back to back;
 * level l is [n·h·w][h>>l][w>>l] (AvgPool2d(2,2) floors), starting at float offset
 * n·h·w·Σ_{j<l}(h>>j)(w>>j).  level0 = (f1ᵀ f2)/sqrt(c).  num_levels in [1, 8]. */
long long scflow_corr_pyramid_size(int n, int h, int w, int num_levels);
int scflow_corr_pyramid(const float* f1, const float* f2, float* pyr, int n, int c, int h, int w,
                        int num_levels, void* stream);

/* a2: multi-scale (2r+1)² bilinear window lookup, align_corners=True (SCFlow's config), zero padding.
 * flow: [n][2][h][w] (flow_layout NCHW) or [n·h·w][2] (NHWC).  out channel
 * k = lvl·(2r+1)² + a·(2r+1) + b samples x+Δx=a−r, y+Δy=b−r.  out: NCHW [n][L(2r+1)²][h][w]
 * or NHWC with pixel stride out_stride (>= L(2r+1)²). */
int scflow_corr_lookup(const float* pyr, const float* flow, int flow_layout, float* out,
                       int out_layout, int out_stride, int n, int h, int w, int num_levels,
                       int radius, void* stream);
/* The same with grid_sample's align_corners chosen: 1 = the call above; 0 = CorrLookup(align_corners=
 * False) (bilinear_sample's own default, corr_lookup.py:35): sample (g+1)·size/2 − 1/2 after the same
 * g = s·2/max(size−1,1) − 1 normalisation (corr_lookup.py:63-64). */
int scflow_corr_lookup_ex(const float* pyr, const float* flow, int flow_layout, float* out,
                          int out_layout, int out_stride, int n, int h, int w, int num_levels,
                          int radius, int align_corners, void* stream);

/* a1 + a2 with the pyramid in TILED layout: level l of query pixel m is an (h>>l)×(w>>l) map
 * stored in 4×4 tiles of 16 contiguous floats, tiles row-major — element (y, x) at
 * ((y>>2)·((w>>l)>>2) + (x>>2))·16 + (y&3)·4 + (x&3) from the map's start (same map sizes and
 * level offsets as scflow_corr_pyramid).  scflow_corr_pyramid_tiled computes level 0 and pools
 * levels 1..L−1 inside the GEMM epilogue (one launch; values bit-identical to
 * scflow_corr_pyramid's); needs L ≤ 4, h and w multiples of 8 and of 4·2^(L−1), f1/f2 16-B
 * aligned.  scflow_corr_lookup_tiled = scflow_corr_lookup_ex on such a pyramid (same outputs). */
int scflow_corr_pyramid_tiled(const float* f1, const float* f2, float* pyr, int n, int c, int h,
                              int w, int num_levels, void* stream);
int scflow_corr_lookup_tiled(const float* pyr, const float* flow, int flow_layout, float* out,
                             int out_layout, int out_stride, int n, int h, int w, int num_levels,
                             int radius, int align_corners, void* stream);
/* a2 + a3's corr_net.0 fused (inference): out[m][·] = act(W·lookup(pyr, flow)[m] + bias), the
 * lookup of scflow_corr_lookup_tiled (TILED pyramid, num_levels 4, radius 4, h and w multiples of
 * 32) and the 1×1 conv of SCFLOW_CONV_1X1W (weight packed by scflow_conv_pack_weights with bk =
 * SCFLOW_CONV_1X1W, c0 = 324, c1 = 0; cout ≤ 256) in one launch: the correlation features stay
 * in LDS (replaces CorrLookup.forward, corr_lookup.py:102-136, followed by MotionEncoder's first
 * corr_net layer, raft_decoder.py:75-85,152-166).  flow: [n·h·w][2] (NHWC); out: [n·h·w] rows of
 * out_stride floats.  Bit-identical to the two launches it replaces. */
int scflow_corr_lookup_conv1x1(const float* pyr, const float* flow, const float* weight,
                               const float* bias, float* out, int out_stride, int n, int h, int w,
                               int num_levels, int radius, int cout, int act, int align_corners,
                               void* stream);
long long scflow_corr_lookup_conv1x1_lds_bytes(void);
/* ABI markers: scflow_abi_version() returns SCFLOW_ABI_VERSION of the header the library was
 * built from (2: scflow_conv_args ends with the F(4×4,3×3) workspace fields ws / ws_bytes, and
 * scflow_conv_pick_bk may return SCFLOW_CONV_WINO4; 3: + scflow_xhead_pred and its workspace
 * query); scflow_conv_args_size() its
 * sizeof(scflow_conv_args).  A binding checks both before its first call (scflow_amd/_lib.py
 * does, at load). */
#define SCFLOW_ABI_VERSION 3
int scflow_abi_version(void);
long long scflow_conv_args_size(void);
/* Tuning only: launch-time environment switches (SCFLOW_WINO4_DEPTH, SCFLOW_WINO4_XCD,
 * SCFLOW_GNR_CB, SCFLOW_SMALLCIN_SPLIT, SCFLOW_SMALLCIN_WGS, SCFLOW_THINZ) are read once and
 * cached; this makes their next use re-read the environment (in-process A/B). */
int scflow_debug_reload_switches(void);
/* Profiling only: later LDS-kernel lookups (scflow_corr_lookup*) write 6 u64 real-time-clock
 * stamps per workgroup of 16 query pixels to `stamps` (phase boundaries; NULL turns it off). */
int scflow_debug_lookup_stamps(void* stamps);
/* Profiling only: later instrumented conv launches (the Winograd F(2×2,3×3), F(4,5) and F(4×4,3×3)
 * kernels, the small-cin MFMA conv, the whole-halo thin conv, scflow_enc_conv) write 4 u64
 * real-time-clock stamps per workgroup (start, prologue done, main loop done, epilogue done), NULL
 * turns it off. */
int scflow_debug_conv_stamps(void* stamps);

/* Channels-last convolution (cross-correlation, like nn.Conv2d) with fused bias/activation and
 * optional ConvGRU gate epilogues.  Input channels = c0 (src0) ++ c1 (src1, may be 0).
 * Weights must be packed by scflow_conv_pack_weights for the same shape. */
typedef struct scflow_conv_args {
  const float* src0; int c0; int s0;     /* first input, channels, pixel stride (floats)      */
  const float* src1; int c1; int s1;     /* optional second input concatenated on channels     */
  const float* weight;                   /* packed, see scflow_conv_pack_weights               */
  const float* bias;                     /* [cout] or NULL                                     */
  float* out; int so;                    /* output (channel 0 of this conv), pixel stride      */
  int n, h, w;                           /* input batch and spatial size                       */
  int cout, kh, kw, ph, pw, stride;      /* output channels, kernel, padding, stride           */
  int act;                               /* SCFLOW_ACT_*                                       */
  int epilogue;                          /* SCFLOW_EPI_*                                       */
  float* gate; int sg;                   /* GRU z buffer and its pixel stride                  */
  float* rh; int srh;                    /* GRU_ZR: r·h output                                 */
  float* hid; int sh;                    /* GRU: hidden state (read by ZR, updated by Q)       */
  const float* bias_map; int sbm;        /* optional per-pixel additive term [pix][sbm] (MFMA  */
                                         /* variant): pre-activation += bias_map[pix·sbm + o]; */
                                         /* the decoder passes the loop-invariant context      */
                                         /* contribution of the GRU convs here                 */
  int bk;                                /* packing format of the weights: K-stage depth 0 or 16 */
                                         /* (default) or 8, or SCFLOW_CONV_WINO — see           */
                                         /* scflow_conv_pick_bk                                 */
  /* Winograd 3×3 only (NULL elsewhere) — the RAFT encoder's fused normalisation:              */
  const float* in_scale;                 /* src0 ← relu(src0·in_scale[n][c0] + in_shift[n][c0]) */
  const float* in_shift;                 /* on load (InstanceNorm + ReLU of the producer; c1=0) */
  const float* out_scale;                /* v ← (conv + bias)·out_scale[o] + out_shift[o]       */
  const float* out_shift;                /* (eval BatchNorm)                                    */
  const float* res; int sres;            /* v += res[pix·sres + o] before the activation        */
  /* SCFLOW_CONV_WINO4 only (NULL / 0 elsewhere): the transformed-input workspace of at least   */
  /* scflow_conv_workspace_bytes(args) bytes, 16-B aligned, private to this launch until it ends */
  float* ws; long long ws_bytes;
} scflow_conv_args;

/* scflow_conv_args.bk = SCFLOW_CONV_WINO selects the Winograd kernels: F(2×2,3×3) for 3×3, stride
 * 1, pad 1, width 32, 64 or 128 (height a multiple of 4 at 32, of 2 otherwise), SCFLOW_EPI_PLAIN;
 * F(4,5) for 1×5 (pad 0,2) / 5×1 (pad 2,0), width 32 or 64, every epilogue.  Exact fp32
 * arithmetic, 2.25× / 2.5× fewer matrix multiplies than the direct conv; the weights must be
 * packed with the same bk. */
#define SCFLOW_CONV_WINO 2
/* scflow_conv_args.bk = SCFLOW_CONV_1X1W selects the wide 1×1 kernel (corr_net.0's 324 → 256):
 * stride 1, no padding, one source (c1 = 0) with c0 a multiple of 4 and 8·⌈c0/8⌉ one of the
 * instantiated depths (128, 256, 328), cout ≤ 256, SCFLOW_EPI_PLAIN (bias, bias map, activation);
 * 64 pixels × every output channel per workgroup, the pixels' whole input rows in LDS. */
#define SCFLOW_CONV_1X1W 3
/* scflow_conv_args.bk = SCFLOW_CONV_WINO4 selects Winograd F(4×4,3×3) (round 5): 3×3, stride 1,
 * pad 1, height and width multiples of 4, channels multiples of 4, SCFLOW_EPI_PLAIN (bias, bias
 * map, residual, eval-BN affine, input IN+ReLU on load with c1 = 0, activation); 2.25 multiplies
 * per output and tap set (F(2×2,3×3): 4).  Two launches: the input transform into args.ws, then
 * the 36 point GEMMs with the output transform in their epilogue.  fp32 throughout; error vs fp64
 * ≈ 10× a direct fp32 conv's (points {0, ±1, 2, −½, ∞}). */
#define SCFLOW_CONV_WINO4 4
/* Two independent convolutions (neither reads what the other writes, no overlapping outputs) in
 * ONE grouped launch when a paired kernel covers the pair — the decoder tail's flow-predictor /
 * mask-predictor branches: 3×3 256→2 with 1×1 256→1, 7×7 2→128 with 3×3 1→64, two F(2×2,3×3)
 * convs of one width — else as two scflow_conv2d launches in order; results equal the separate
 * launches bit for bit (round 6; replaces running the two branches on two streams joined by
 * events, scflow_decoder.py:211-218). */
int scflow_conv2d_pair(const scflow_conv_args* args_a, const scflow_conv_args* args_b, void* stream);
/* The XHeads (raft_decoder.py:256-294, called at scflow_decoder.py:211-218): the two hidden 3×3
 * convs as ONE F(4×4,3×3) conv `hidden` (SCFLOW_CONV_WINO4, flow head's channels first —
 * flow_channels of hidden->cout —, ReLU, bias only; hidden->out is not written) with both
 * predictors contracted in its epilogue, then one launch summing the 32-channel blocks' partial
 * sums and the 3×3 predictor's taps (round 6; replaces the hidden conv's 2 KiB-per-pixel output
 * and the predictor convs that read it back).  pred_w [hidden->cout][20]: row c < flow_channels
 * holds the 3×3 two-output predictor's weights W[o][c][ty][tx] at column (3·ty + tx)·2 + o (18
 * used), row c ≥ flow_channels the 1×1 one-output predictor's W[0][c − flow_channels] at column 0.
 * flow_out [pixel][flow_stride] (2 channels) = flow_act(flow_bias + conv), mask_out
 * [pixel][mask_stride] = mask_act(mask_bias + conv) (biases may be NULL).  workspace ≥
 * scflow_xhead_pred_workspace_bytes, 16-byte aligned.  Width 32 or 64, height a multiple of 4,
 * both heads' hidden channels multiples of 32; else SCFLOW_EUNSUPPORTED.  fp32; only the
 * summation order differs from the separate convs. */
long long scflow_xhead_pred_workspace_bytes(int n, int h, int w, int flow_channels, int hidden_channels);
int scflow_xhead_pred(const scflow_conv_args* hidden, int flow_channels, const float* pred_w,
                      float* workspace, long long workspace_bytes, const float* flow_bias,
                      const float* mask_bias, int flow_act, int mask_act, float* flow_out,
                      int flow_stride, float* mask_out, int mask_stride, void* stream);
/* Bytes of args.ws a launch needs (0 for packing formats without a workspace). */
long long scflow_conv_workspace_bytes(const scflow_conv_args* args);

/* Number of floats of the packed weight buffer for bk 8 and 16 (the same for both); w_oihw is
 * nn.Conv2d's [cout][c0+c1][kh][kw]. */
long long scflow_conv_packed_size(int cout, int c0, int c1, int kh, int kw, int stride, int w);
/* The same for any packing format bk (0, 8, 16, SCFLOW_CONV_WINO or SCFLOW_CONV_1X1W). */
long long scflow_conv_packed_size_bk(int cout, int c0, int c1, int kh, int kw, int stride, int w,
                                     int bk);
/* bk: packing format (0 → 16, 8, SCFLOW_CONV_WINO or SCFLOW_CONV_1X1W); pass the same value in
 * scflow_conv_args.bk. */
int scflow_conv_pack_weights(const float* w_oihw, float* packed, int cout, int c0, int c1, int kh,
                             int kw, int stride, int w, int bk, void* stream);
/* Preferred packing format for this launch shape (batch, sizes, channels, kernel): Winograd
 * (SCFLOW_CONV_WINO) for the 3×3 stride-1 convs it covers, the wide 1×1 kernel
 * (SCFLOW_CONV_1X1W) for the 1×1 convs it covers, else the direct conv's K-stage depth,
 * 8 when the grid needs more resident workgroups than 16-deep stages' LDS allows, else 16. */
int scflow_conv_pick_bk(const scflow_conv_args* args);
int scflow_conv2d(const scflow_conv_args* args, void* stream);

/* a8: R_dst = R(ortho6d Δ)·R_src; t_z' = t_z/exp(Δt_z) (depth_transform 0) or t_z·(Δt_z+1) (1);
 * t_xy' = t_z'·(Δt_xy/weight + t_xy/t_z).  drot6 [n][6], dt [n][3], R [n][3][3], t [n][3]. */
int scflow_pose_update(const float* drot6, const float* dt, const float* R_src, const float* t_src,
                       float* R_dst, float* t_dst, int n, float weight, int depth_transform,
                       void* stream);

/* a9: object-frame point of every pixel: points[n][y][x] = {R⁻¹(K⁻¹[x·d,y·d,d] − t), valid},
 * valid = (depth>0) ? 1 : 0, float4 per pixel. */
int scflow_lift_points(const float* depth, const float* K, const float* R, const float* t,
                       float* points, int n, int h, int w, void* stream);

/* a10: flow[n][2][h][w] = proj(K(R·P+t)) − (x,y) where valid, else invalid_num. */
int scflow_pose_flow(const float* R, const float* t, const float* K, const float* points,
                     float* flow, int n, int h, int w, float invalid_num, void* stream);

/* a8+a10 fused (one launch per refinement iteration). */
int scflow_pose_update_flow(const float* drot6, const float* dt, const float* R_src,
                            const float* t_src, const float* K, const float* points, float* R_dst,
                            float* t_dst, float* flow, int n, int h, int w, float weight,
                            int depth_transform, float invalid_num, void* stream);

/* a11 down: out = value_scale · bilinear(flow[n][2][H][W] -> h×w, align_corners=True) written
 * channels-last to out0 (pixel stride s0) and, if out1 != NULL, also to out1 (stride s1). */
int scflow_flow_downsample(const float* flow, float* out0, int s0, float* out1, int s1, int n,
                           int H, int W, int h, int w, float value_scale, void* stream);

/* a11 up: flow_out[n][2][H][W] = value_scale·bilinear(lr + delta) and mask_out[n][1][H][W] =
 * bilinear(mask); lr/delta are channels-last [n·h·w][2] (delta may be NULL), mask [n·h·w][1]
 * (may be NULL, then mask_out is not written). */
int scflow_flow_upsample(const float* lr, const float* delta, const float* mask, float* flow_out,
                         float* mask_out, int n, int h, int w, int H, int W, float value_scale,
                         void* stream);

/* One launch = scflow_pose_update_flow(drot6 .. invalid_num; flow is [n][2][H][W]) +
 * scflow_flow_upsample(lr, delta, mask, flow_up, mask_up, n, h, w, H, W, up_scale) when flow_up
 * != NULL + scflow_flow_downsample(flow, lr_next, s_next, hx_next, s_hx, n, H, W, h, w,
 * down_scale) when lr_next != NULL (the ↓8 flow is computed from the new pose directly, bit-
 * identical to downsampling `flow`).  lr_next must not alias lr. */
int scflow_pose_step(const float* drot6, const float* dt, const float* R_src, const float* t_src,
                     const float* K, const float* points, float* R_dst, float* t_dst, float* flow,
                     int n, int H, int W, float weight, int depth_transform, float invalid_num,
                     const float* lr, const float* delta, const float* mask, float* flow_up,
                     float* mask_up, float* lr_next, int s_next, float* hx_next, int s_hx, int h,
                     int w, float up_scale, float down_scale, void* stream);

/* Cross-stream ordering on one device (the decoder's side stream): events without timing and
 * with a device-scope release (hipEventDisableSystemFence) — a default event's system-scope
 * release writes back the GPU caches on every record.  No reference equivalent (plumbing). */
int scflow_sync_event_create(void** event);
int scflow_sync_event_destroy(void* event);
int scflow_sync_event_record(void* event, void* stream);
int scflow_stream_wait_event(void* stream, void* event);
/* Timing events (device-scope release; destroy with scflow_sync_event_destroy, record with
 * scflow_sync_event_record); *ms = end − start after waiting for end. */
int scflow_timing_event_create(void** event);
int scflow_event_elapsed_ms(void* start, void* end, float* ms);

/* out[n·ons + b·obs + a] = in[n·ins + a·ias + b] for a < A, b < B (batched 2-D transpose; e.g.
 * NCHW -> a channel slice of an NHWC buffer, or back). */
int scflow_transpose(const float* in, float* out, int n, int A, int B, long long ins, int ias,
                     long long ons, int obs, void* stream);

/* a7: MultiClassPoseHead (pose_head.py:110-211) as 9 launches.
 * scflow_ph_conv: x (two channel sources, channels-last, pixel strides s0/s1) → raw conv output
 *   out [n][oh][ow][cout] (channels-last, + bias if given).  If scale/shift are given, the input
 *   is first mapped x ← relu(x·scale[n][c] + shift[n][c]) (the previous GroupNorm + ReLU).
 *   Weights packed by scflow_ph_conv_pack ([cout][kh·kw][roundup(cin,16)]).
 * scflow_ph_gn_stats: GroupNorm(groups) statistics of x [n][hw][c] → scale/shift [n][c] with
 *   scale = γ/sqrt(var+eps), shift = β − mean·scale (biased variance, like F.group_norm).
 * scflow_ph_fc: y [m][n] = act(x [m][k] · Wᵀ + b), W = nn.Linear weight [n][k] (k % 16 == 0).
 *   gn_c > 0: x is a raw conv output [m][hw][gn_c] (channels-last) mapped through scale/shift +
 *   ReLU; W's columns must then be in channels-last order — scflow_ph_fc_permute turns the
 *   reference's NCHW-flatten columns (k = c·hw + p, nn.Flatten) into that order.
 * scflow_ph_heads: drot [m][rch] and dt [m][3] from x [m][k] using only class label[0]'s rows of
 *   the rotation [num_class·rch][k] and translation [num_class·3][k] heads (index_select quirk). */
long long scflow_ph_conv_packed_size(int cout, int cin, int kh, int kw);
int scflow_ph_conv_pack(const float* w_oihw, float* packed, int cout, int cin, int kh, int kw,
                        void* stream);
int scflow_ph_conv(const float* src0, int c0, int s0, const float* src1, int c1, int s1,
                   const float* scale, const float* shift, const float* packed, const float* bias,
                   float* out, int n, int h, int w, int cout, int kh, int kw, int stride, int pad,
                   void* stream);
/* scflow_ph_conv with the K chunks split over ksplit workgroup slices: out = ksplit partial slabs
 *   [ksplit][n·oh·ow][cout] (bias must be NULL), summed by scflow_ph_gn_reduce. */
int scflow_ph_conv_split(const float* src0, int c0, int s0, const float* src1, int c1, int s1,
                         const float* scale, const float* shift, const float* packed,
                         const float* bias, float* out, int n, int h, int w, int cout, int kh,
                         int kw, int stride, int pad, int ksplit, void* stream);
int scflow_ph_gn_stats(const float* x, int n, int hw, int c, int groups, const float* gamma,
                       const float* beta, float eps, float* scale, float* shift, void* stream);
/* scflow_ph_gn_reduce: y = Σ_z parts[z] (nsplit slabs, split_stride floats apart; y written when
 *   nsplit > 1) and its GroupNorm scale/shift like scflow_ph_gn_stats (c % 32 == 0). */
int scflow_ph_gn_reduce(const float* parts, int nsplit, long long split_stride, float* y, int n,
                        int hw, int c, int groups, const float* gamma, const float* beta, float eps,
                        float* scale, float* shift, void* stream);
int scflow_ph_fc_permute(const float* W, float* Wp, int n, int c, int hw, void* stream);
int scflow_ph_fc(const float* x, int ldx, int m, int k, const float* W, const float* bias, float* y,
                 int n, int relu, int gn_c, const float* scale, const float* shift, void* stream);
/* scflow_ph_fc with K split over ksplit workgroup slices (m ≤ 32): parts [ksplit][m][n] = partial
 *   x·Wᵀ sums (no bias / activation); gn_c/scale/shift as in scflow_ph_fc, or xsplit > 0: x is
 *   the previous layer's split partial sums [xsplit][m][ldx] read as relu(Σ + xbias).
 * scflow_ph_fc_sum: y [m][n] = act(x' · Wᵀ + b) with x' = relu(Σ_z parts[z] + xbias), the input
 *   being the previous layer's split partial sums [nsplit][m][k] (its bias xbias, then ReLU).
 * scflow_ph_heads_sum: scflow_ph_heads on such a split input (xsplit = 0: plain x). */
int scflow_ph_fc_split(const float* x, int ldx, int m, int k, const float* W, float* parts, int n,
                       int ksplit, int gn_c, const float* scale, const float* shift, int xsplit,
                       const float* xbias, void* stream);
int scflow_ph_fc_sum(const float* parts, int nsplit, int m, int k, const float* xbias,
                     const float* W, const float* bias, float* y, int n, int relu, void* stream);
int scflow_ph_heads_sum(const float* x, int xsplit, const float* xbias, int m, int k,
                        const float* Wr, const float* br, int rch, const float* Wt, const float* bt,
                        const long long* label, int num_class, float* drot, float* dt,
                        void* stream);
int scflow_ph_heads(const float* x, int m, int k, const float* Wr, const float* br, int rch,
                    const float* Wt, const float* bt, const long long* label, int num_class,
                    float* drot, float* dt, void* stream);

/* scflow_pose_step_part: scflow_pose_step restricted to parts (bit 0: the full-resolution outputs
 *   — pose flow, ×8 flow prediction and mask; bit 1: the next iteration's ↓8 flow, lr_next /
 *   hx_next).  Each part recomputes the pose update; the part with the lowest block writes
 *   R_dst / t_dst.  The decoder runs bit 1 on its critical path and bit 0 on a side stream.
 *   drot6 == NULL (parts = 1 only): R_src / t_src ARE the updated pose (the bit-1 launch's
 *   R_dst / t_dst) — no update, dt / R_dst / t_dst unused, same outputs. */
int scflow_pose_step_part(const float* drot6, const float* dt, const float* R_src,
                          const float* t_src, const float* K, const float* points, float* R_dst,
                          float* t_dst, float* flow, int n, int H, int W, float weight,
                          int depth_transform, float invalid_num, const float* lr,
                          const float* delta, const float* mask, float* flow_up, float* mask_up,
                          float* lr_next, int s_next, float* hx_next, int s_hx, int h, int w,
                          float up_scale, float down_scale, int parts, void* stream);

/* scflow_pose_step_heads: scflow_pose_step_part with the pose head's rotation / translation heads
 *   (MultiClassPoseHead, models/head/pose_head.py:203-211 — label[0]'s class for every sample)
 *   computed in the same launch instead of by scflow_ph_heads_sum: x = relu(Σ_z x_z + xbias),
 *   the last FC's xsplit K-split partial sums [xsplit][n][k]; rch = 6 (ortho6d) or 4
 *   (quaternion, depth_transform's SCFLOW_POSE_QUAT_XYZW).  drot [n][rch] / dt [n][3] are
 *   OUTPUTS here (the decoder's returned deltas).  Replaces the heads launch + the pose step's
 *   delta reads of the reference's get_pose_ (models/decoder/scflow_decoder.py:230-236). */
int scflow_pose_step_heads(const float* x, int xsplit, const float* xbias, int k, const float* Wr,
                           const float* br, int rch, const float* Wt, const float* bt,
                           const long long* label, int num_class, float* drot, float* dt,
                           const float* R_src, const float* t_src, const float* K,
                           const float* points, float* R_dst, float* t_dst, float* flow, int n,
                           int H, int W, float weight, int depth_transform, float invalid_num,
                           const float* lr, const float* delta, const float* mask, float* flow_up,
                           float* mask_up, float* lr_next, int s_next, float* hx_next, int s_hx,
                           int h, int w, float up_scale, float down_scale, int parts,
                           void* stream);

/* §8(f)-1: RAFTEncoder (Basic) — feature encoder (InstanceNorm) and context encoder (BatchNorm,
 * eval statistics), models/encoder/raft_encoder.py:286-314, BasicBlock models/backbone/resnet.py:
 * 12-92, ResLayer resnet.py:676-771, called from SCFlowRefiner.extract_feat
 * (models/refiner/scflow_refiner.py:84-106).  Activations are channels-last [n][h][w][c].
 *
 * scflow_enc_conv: implicit-GEMM conv (fp32 MFMA), 1×1 or 3×3, stride 1 or 2, cin % 16 == 0;
 *   output width 8, 16, 32, 64 or a multiple of the tile (128 for stride 1, 64 for stride 2), and
 *   output height a multiple of the tile's rows (tile / width when the width is smaller).  Per element of the output:
 *     v = conv(x') + bias;  v = v·out_scale[c] + out_shift[c] (if given: eval BatchNorm);
 *     v += res[pix][c] (if given);  out = act(v) for c < act_split, act2(v) otherwise,
 *   where x' = relu(x·in_scale[img][c] + in_shift[img][c]) if in_scale is given (the previous
 *   InstanceNorm + ReLU applied on load; zero padding stays zero), else x.
 *   Weights packed by scflow_enc_conv_pack (same shape).
 * scflow_enc_stem: 7×7 conv of an NCHW image batch [n][3][h][w], stride 1 or 2 (other shapes:
 *   SCFLOW_EUNSUPPORTED), written channels-last with the same bias / out_scale / act epilogue
 *   (the stem conv1); cout ≤ 64 runs as an implicit GEMM on fp32 MFMA, wider stems on VALU.
 *   Weights packed by scflow_enc_stem_pack ([kh·kw·cin][roundup(cout,64)]).
 *   With src1 the input is cat[src, src1] (both normalised on load when in_scale is given,
 *   in_scale then covering cin + cin1 channels).
 * scflow_enc_stats + scflow_enc_norm_finalize: InstanceNorm statistics of x [n][hw][c]
 *   (fp64 partial sums over `chunks` pixel chunks per image, then per (img, c))
 *   → scale = 1/sqrt(var+eps), shift = −mean·scale (biased variance, affine=False);
 *   partial must hold n·chunks·2·c doubles.
 * scflow_enc_apply: out[p][c] = relu(x·scale[img][c] + shift[img][c] + id'), with
 *   id' = 0 (id NULL), id (id_scale NULL) or id·id_scale[img][c] + id_shift[img][c]. */
typedef struct scflow_enc_conv_args {
  const float* src; int cin; int s_in;            /* input, channels, pixel stride           */
  const float* src1; int cin1; int s_in1;          /* optional 2nd input, concatenated on     */
                                                   /* channels (cin1 % 16 == 0; 0 = none)     */
  int ksplit;                                      /* ≥ 2: K (channel stages) split over      */
                                                   /* grid.z; split z writes a raw partial    */
                                                   /* to out + z·n·oh·ow·s_out (no bias /     */
                                                   /* affine / residual / act allowed)        */
  const float* in_scale; const float* in_shift;    /* [n][cin] or NULL                        */
  const float* weight; const float* bias;          /* packed; bias [cout] or NULL             */
  const float* out_scale; const float* out_shift;  /* [cout] or NULL                          */
  const float* res; int s_res;                     /* residual or NULL, pixel stride          */
  float* out; int s_out;                           /* output, pixel stride                    */
  int n, h, w, cout, kh, kw, stride, pad;
  int act, act2, act_split;                        /* SCFLOW_ACT_* and the channel split      */
} scflow_enc_conv_args;

long long scflow_enc_conv_packed_size(int cout, int cin, int kh, int kw);
int scflow_enc_conv_pack(const float* w_oihw, float* packed, int cout, int cin, int kh, int kw,
                         void* stream);
int scflow_enc_conv(const scflow_enc_conv_args* args, void* stream);
long long scflow_enc_stem_packed_size(int cout, int cin, int kh, int kw);
int scflow_enc_stem_pack(const float* w_oihw, float* packed, int cout, int cin, int kh, int kw,
                         void* stream);
int scflow_enc_stem(const float* img, const float* packed, const float* bias,
                    const float* out_scale, const float* out_shift, float* out, int n, int cin,
                    int h, int w, int cout, int kh, int kw, int stride, int pad, int act,
                    void* stream);
int scflow_enc_stats(const float* x, int n, int hw, int c, int chunks, double* partial,
                     void* stream);
int scflow_enc_norm_finalize(const double* partial, int n, int chunks, int c, int hw, float eps,
                             float* scale, float* shift, void* stream);
int scflow_enc_apply(const float* x, const float* scale, const float* shift, const float* id,
                     const float* id_scale, const float* id_shift, float* out, int n, int hw,
                     int c, void* stream);

/* Training (§8(f)-2) building blocks.
 * scflow_im2col: cols[p][(ty·kw + tx)·cin + c] = x[n][oy·s − ph + ty][ox·s − pw + tx][c] (0 outside),
 *   p = (n·oh + oy)·ow + ox; x channels-last with pixel stride sx.  The conv weight gradient is
 *   then dW[o][tap·cin + c] = Σ_p dY[p][o] · cols[p][tap·cin + c] (a plain GEMM).
 * scflow_corr_lookup_backward: scatter-add of the lookup's output gradient (same layout options
 *   as scflow_corr_lookup) into the pyramid gradient (same layout as the pyramid; must be
 *   zeroed by the caller), with grid_sample's bilinear weights — the flow input is detached in
 *   SCFlow (scflow_decoder.py:193-194), so no flow gradient. */
int scflow_im2col(const float* x, int sx, float* cols, int n, int h, int w, int cin, int kh, int kw,
                  int stride, int ph, int pw, void* stream);
/* scflow_im2col_ex: scflow_im2col, or with channel_major the column order (c·kh + ty)·kw + tx —
 * the conv weight's own [cout][cin][kh][kw] order, so dW (and its accumulation) is one GEMM
 * written in place. */
int scflow_im2col_ex(const float* x, int sx, float* cols, int n, int h, int w, int cin, int kh,
                     int kw, int stride, int ph, int pw, int channel_major, void* stream);
/* scflow_pose_update6_train: the training step's pose update for an ortho6d Δrotation
 * (pose.py:124-169), forward (backward = 0: o0 = Rn [n][3][3], o1 = tn [n][3]) or its gradient
 * (backward = 1, given gRn, gtn: o0 = g drot [n][6], o1 = g dt [n][3], o2 = g R, o3 = g t);
 * depth_exp: depth_transform 'exp' (else 'linear'); detach_xy: detach_depth_for_xy. */
int scflow_pose_update6_train(const float* drot, const float* dt, const float* R, const float* t,
                              const float* gRn, const float* gtn, float* o0, float* o1, float* o2,
                              float* o3, int n, float weight, int depth_exp, int detach_xy,
                              int backward, void* stream);
/* scflow_pm_loss / scflow_pm_loss_backward: one refinement iteration's disentangled L1
 * point-matching loss (point_matching_loss.py:159-218, disentangle_z, mean) fused — model points
 * pts [B][P][3] (each sample's class's set), rotations [B][3][3], translations [B][3], sym [B]
 * (1.0 = symmetric class: nearest-point matching as scflow_knn1; NULL = none), diam [B];
 * workspace gt_rt, pred_rot [B][P][3], idx [B][P]; loss = weight·Σ_b l_b/diam_b/B (one float).
 * The backward takes the loss gradient (one float, device) and the forward's workspace and
 * writes g_pred_r [B][3][3], g_pred_t [B][3]. */
int scflow_pm_loss(const float* pts, const float* gt_r, const float* gt_t, const float* pred_r,
                   const float* pred_t, const float* sym, const float* diam, float* gt_rt,
                   float* pred_rot, long long* idx, float* loss, int B, int P, float weight,
                   void* stream);
int scflow_pm_loss_backward(const float* gloss, const float* pts, const float* gt_rt,
                            const float* pred_rot, const long long* idx, const float* sym,
                            const float* pred_t, const float* gt_t, const float* diam,
                            float* g_pred_r, float* g_pred_t, int B, int P, float weight,
                            void* stream);
/* scflow_up_l1_loss: a full-resolution L1 loss of the sequence loss on the ×(H/h) bilinear
 * (align_corners) upsampling of the channels-last low-resolution prediction f [N][h][w][C]:
 * loss = weight·Σ v·|sval·up(f) − target| / denom (target NCHW [N][C][H][W], v = vmask [N][H][W]
 * or 1, denom = *denom (device) or cdenom), RAFTLoss / L1Loss of sequence_loss.py:15-36 after
 * scflow_decoder.py:223-228.  Writes sgn = v·sgn(sval·up − target) [N][C][H][W] for the backward
 * (the upsampling adjoint) and uses partial[ceil(N·H·W/256)] as workspace. */
int scflow_up_l1_loss(const float* f, int C, int h, int w, const float* target, const float* vmask,
                      int N, int H, int W, float sval, const float* denom, float cdenom,
                      float weight, float* sgn, float* partial, float* loss, void* stream);
/* scflow_knn1: idx[b][i] = argmin_j |gt[b][i] − pred[b][j]|² over [batch][P][3] / [batch][Q][3]
 * point sets (first minimum in index order) — pytorch3d knn_points(K=1) in the symmetric-class
 * point-matching loss (point_matching_loss.py:183-186; pytorch3d is absent, torch.argmin's rule). */
int scflow_knn1(const float* gt, const float* pred, long long* idx, int batch, int P, int Q,
                void* stream);
/* GroupNorm (+ReLU) of the pose head's conv stack (pose_head.py:160-170, mmcv ConvModule with
 * norm_cfg GN(32) and ReLU; torch.nn.GroupNorm semantics: biased variance, eps inside the root),
 * channels-last x [n][hw][c] with exactly 4 channels per group (c == 4·groups), 16-byte aligned.
 *   forward: y = act((x − μ_g)·rstd_g·γ_c + β_c); stats [n·groups][2] = (μ, rstd)
 *   backward: dx; dγ / dβ summed over the images in order (part: n·c·2 floats of workspace),
 *             written (accumulate 0) or added onto dgamma / dbeta (accumulate 1) */
int scflow_group_norm_forward(const float* x, const float* gamma, const float* beta, float* y,
                              float* stats, int n, int hw, int c, int groups, float eps, int relu,
                              void* stream);
int scflow_group_norm_backward(const float* dy, const float* x, const float* gamma,
                               const float* beta, const float* stats, float* dx, float* part,
                               float* dgamma, float* dbeta, int n, int hw, int c, int groups,
                               int relu, int accumulate, void* stream);
/* SepConvGRU gate algebra of the training step (raft_decoder.py:235-253), channels-last,
 * c % 4 == 0, zr = the z | r conv's sigmoid output [npix][2c]:
 *   scflow_gru_gate_forward mode 0: out = r·h;  mode 1: out = h + z·(q − h)
 *   scflow_gru_gate_backward_q: dq = dh2·z·(1 − q²); dzr[:, :c] = dh2·(q − h)·z(1 − z);
 *                               dha = dh2·(1 − z)   (dh2 pixel stride sdh2 ≥ c)
 *   scflow_gru_gate_backward_r: dzr[:, c:] = drh·h·r(1 − r); dh = dha + drh·r (drh / dh pixel
 *                               strides sdrh / sdh ≥ c; dh may alias drh: each element is read
 *                               before it is written, by the same thread) */
int scflow_gru_gate_forward(const float* zr, const float* h, const float* q, float* out,
                            long long npix, int c, int mode, void* stream);
int scflow_gru_gate_backward_q(const float* dh2, int sdh2, const float* zr, const float* h,
                               const float* q, float* dq, float* dzr, float* dha, long long npix,
                               int c, void* stream);
int scflow_gru_gate_backward_r(const float* drh, int sdrh, const float* zr, const float* h,
                               const float* dha, float* dzr, float* dh, int sdh, long long npix,
                               int c, void* stream);
/* scflow_col2im: the adjoint of scflow_im2col (same geometry; dx has pixel stride sdx ≥ cin):
 *   dx[n][iy][ix][c] = Σ_{ty,tx: (iy+ph−ty)/s, (ix+pw−tx)/s integral, inside} cols[(n,oy,ox)][(ty·kw+tx)·cin+c]
 * — a fixed-order gather, written (not accumulated).  With cols = dY·Wmat (Wmat[co][(ty·kw+tx)·cin+ci]
 * = w[co][ci][ty][tx]) it is a strided conv's input gradient without zero insertion (training:
 * the stride-2 convs of the encoders and the pose head, resnet.py / pose_head.py:201-211). */
int scflow_col2im(const float* cols, float* dx, int sdx, int n, int h, int w, int cin, int kh, int kw,
                  int stride, int ph, int pw, void* stream);

/* scflow_conv_wgrad: weight (and bias) gradient of a channels-last conv without an im2col
 * matrix — dw[co][ci][ty][tx] (+)= Σ_p dy[p][co] · x[n][oy·s − ph + ty][ox·s − pw + tx][ci],
 * db[co] (+)= Σ_p dy[p][co] (db may be NULL); x = the channel concat of src0 (cin0) and src1
 * (cin1, optional).  Replaces the weight-gradient half of the reference's autograd for every
 * nn.Conv2d on the training path (torch.nn.grad.conv2d_weight, called by
 * SCFlowRefiner.loss → backward, scflow_refiner.py:182-256).  Shapes: 1×1 and 3×3 (stride 1
 * or 2), 1×5 and 5×1 (stride 1); others return SCFLOW_EUNSUPPORTED.  `workspace` holds the
 * per-split partial sums: at least scflow_conv_wgrad_workspace() floats.  The split count
 * follows the device's CU count; the reduction order is fixed (deterministic). */
typedef struct {
  const float* dy;
  int sdy;
  const float* src0;
  int cin0, s0;
  const float* src1;
  int cin1, s1;
  float* dw;
  float* db;
  float* workspace;
  long long workspace_floats;
  int n, h, w, cout, kh, kw, stride, ph, pw;
  int accumulate;
} scflow_wgrad_args;
/* Training: InstanceNorm2d(affine=False) (+ ReLU) of channels-last x [n][hw][c] (c % 4 == 0,
 * c ≤ 256 for the backward), the feature encoder's norms (resnet.py BasicBlock).  Statistics from
 * scflow_enc_stats + scflow_enc_norm_finalize (scale = rstd, shift = −mean·rstd);
 * scflow_in_apply: y = act(x·scale + shift);  scflow_in_backward: dx = rstd·(g − mean(g) −
 * x̂·mean(g·x̂)), g = dy masked by x̂ > 0 when relu — workspace partial: n·chunks·2·c doubles,
 * mm: n·2·c floats. */
int scflow_in_apply(const float* x, const float* scale, const float* shift, float* y, int n, int hw,
                    int c, int relu, void* stream);
/* The residual block's tail in one pass each way (raft_encoder.py BasicBlock: y = relu(norm2(·) +
 * identity)): scflow_in_apply_residual: y = max(x·scale + shift + res, 0);
 * scflow_in_backward_residual: g = dy·(y > 0) → dres = g and dx = the InstanceNorm backward of g
 * (same workspace as scflow_in_backward). */
/* scflow_colsum: out[c] (+)= Σ_r x[r·ld + c] for a row-major [rows][ld] matrix — the bias
 * gradient Σ_p dY[p][c] of the 7×7 convs and the FC layers in training (deterministic: fixed
 * row chunks, then the chunks in order).  workspace: scflow_colsum_workspace(rows, cols) floats
 * (0 for rows ≤ 256: one pass). */
int scflow_colsum(const float* x, int rows, int cols, int ld, float* out, int accumulate,
                  float* workspace, void* stream);
int scflow_colsum_workspace(int rows, int cols);
int scflow_in_apply_residual(const float* x, const float* scale, const float* shift, const float* res,
                             float* y, int n, int hw, int c, void* stream);
int scflow_in_backward_residual(const float* dy, const float* x, const float* scale,
                                const float* shift, const float* y, float* dx, float* dres,
                                double* partial, float* mm, int n, int hw, int c, int chunks,
                                void* stream);
int scflow_in_backward(const float* dy, const float* x, const float* scale, const float* shift,
                       float* dx, double* partial, float* mm, int n, int hw, int c, int chunks,
                       int relu, void* stream);
/* Training: BatchNorm2d in train mode (+ ReLU, + a residual identity added before the ReLU) of
 * channels-last x [m pixels][c] (c % 4 == 0, c ≤ 256), the context encoder's norms (resnet.py
 * BasicBlock, norm_fn 'batch'; torch.nn.functional.batch_norm(training=True)).  The batch
 * statistics in fp64 (the InstanceNorm statistics over one image of m pixels, chunks ≤ m/256
 * pixel chunks), then per channel rstd = 1/√(var + eps), shift = −mean·rstd (x̂ = x·rstd + shift),
 * the folded affine sc = γ·rstd, sh = β − γ·mean·rstd, and — when running_mean / running_var are
 * given — running ← (1 − momentum)·running + momentum·(mean, unbiased var); y = act(x·sc + sh
 * [+ res]) (ReLU when relu or res).  gamma / beta NULL: no affine.  partial: chunks·2·c doubles.
 * scflow_bn_backward: g = dy masked by y > 0 (y given: the residual form, dres = g) or by
 * γ·x̂ + β > 0 (relu), dx = γ·rstd·(g − mean(g) − x̂·mean(g·x̂)), dγ (+)= Σ g·x̂, dβ (+)= Σ g
 * (accumulate); mm: 2·c floats. */
int scflow_bn_forward(const float* x, const float* gamma, const float* beta, const float* res,
                      float* y, float* running_mean, float* running_var, float* rstd, float* shift,
                      float* sc, float* sh, double* partial, long long m, int c, int chunks,
                      float eps, float momentum, int relu, void* stream);
int scflow_bn_backward(const float* dy, const float* x, const float* rstd, const float* shift,
                       const float* gamma, const float* beta, const float* y, float* dx,
                       float* dres, float* dgamma, float* dbeta, double* partial, float* mm,
                       long long m, int c, int chunks, int relu, int accumulate, void* stream);
/* scflow_gemm_f32: batched strided fp32 GEMM on the matrix cores (training-step contractions:
 * the correlation volume's backward, the 7x7 convs' dY^T.cols weight gradient, the pose head's
 * fully connected layers forward/backward; replaces torch.matmul / F.linear there,
 * raft_decoder.py:35-58 and pose_head.py:201-211 adjoints):
 *   C[b][m][n] = alpha * sum_k A[b][m][k] * B[b][k][n] (+ beta * C[b][m][n]) (+ bias)
 * with element strides: A (b, m, k) at b*sab + m*sam + k*sak, B (b, k, n) at b*sbb + k*sbk + n*sbn,
 * C (b, m, n) at b*scb + m*scm + n*scn.  bias_mode 0: none, 1: bias[n], 2: bias[m].  Any strides
 * work; float4 loads are used along a unit-stride dimension when the base and outer strides are
 * 16-byte aligned.  splits > 1 splits K over the grid: workspace holds splits*batch*M*N floats
 * and a second launch sums the splits in order (deterministic); scflow_gemm_f32_splits() gives
 * the split count this build picks for a shape (1 = no workspace needed). */
int scflow_gemm_f32_splits(int batch, int M, int N, int K);
int scflow_gemm_f32(const float* A, const float* B, float* C, const float* bias, int batch, int M,
                    int N, int K, long long sab, long long sam, long long sak, long long sbb,
                    long long sbk, long long sbn, long long scb, long long scm, long long scn,
                    float alpha, float beta, int bias_mode, int splits, float* workspace,
                    void* stream);
int scflow_conv_wgrad_workspace(const scflow_wgrad_args* args, long long* floats);
int scflow_conv_wgrad(const scflow_wgrad_args* args, void* stream);
/* scflow_conv_wgrad_batched: the weight (and bias) gradient summed over `segs` (1..8) equally
 * shaped segments in one launch and one split reduction — the decoder's per-iteration uses of
 * one conv (its 8 refinement iterations under SCFlowRefiner.loss → backward,
 * scflow_refiner.py:182-256).  `args` describes one segment (n images; its dy / src0 / src1 are
 * ignored), dys[i] / src0s[i] / src1s[i] are segment i's bases with args' strides.  Shapes:
 * scflow_conv_wgrad's (Winograd 3×3 / 1×5 / 5×1, 1×1 stride 1–2, the implicit-GEMM 3×3, the
 * thin kernels for ≤ 4 channels on one side); others return SCFLOW_EUNSUPPORTED.  `workspace`: scflow_conv_wgrad_workspace() of args with n·segs
 * images (it sizes the partial sums for any segment count). */
int scflow_conv_wgrad_batched(const scflow_wgrad_args* args, int segs, const float* const* dys,
                              const float* const* src0s, const float* const* src1s, void* stream);
int scflow_corr_lookup_backward(const float* dout, int out_layout, int out_stride, const float* flow,
                                int flow_layout, float* dpyr, int n, int h, int w, int num_levels,
                                int radius, void* stream);

/* §8(f)-3 mesh renderer (replaces pytorch3d's MeshRasterizer + HardPhongShader behind
 * models/utils/rendering.py:196-248, configured as scflow_ycbv_real.py:261-274).
 * A batch of n_img images of size×size; image i shows one mesh whose vertices / faces are the
 * i-th block of the packed arrays (pytorch3d's join_meshes_as_batch packing: faces hold packed
 * vertex indices; vert_img / face_img give each packed vertex / face its image).  Outputs
 * (each optional except that images needs normals, colors and the light/material colours):
 *   images [n][size][size][4] RGBA (background colour, alpha 0 where empty),
 *   zbuf [n][size][size] (view depth, −1 empty), pix_to_face (packed face, −1 empty),
 *   bary [n][size][size][3] (perspective-corrected barycentrics, −1 empty).
 * Light placement (Renderer.forward :209-230): SCFLOW_LIGHT_FIXED = light_location (object
 * frame; pytorch3d's default (0, 1, 0)); SCFLOW_LIGHT_PER_IMAGE = R_i·(0, 0, max(z_i − 400, 0)),
 * z_i the image's nearest vertex depth (seperate_lights); SCFLOW_LIGHT_BATCH_ZNEAR =
 * R_i·(0, 0, znear/4), znear = ⌊min depth over the batch / 100⌋·100.  Vertex depths must be
 * positive (objects in front of the camera).  workspace: ≥ scflow_render_workspace() bytes. */
#define SCFLOW_LIGHT_FIXED 0
#define SCFLOW_LIGHT_PER_IMAGE 1
#define SCFLOW_LIGHT_BATCH_ZNEAR 2
typedef struct {
  const float* verts;    /* [total_verts][3] object frame */
  const float* normals;  /* [total_verts][3] (pytorch3d verts_normals) */
  const float* colors;   /* [total_verts][3] vertex colours in [0, 1] */
  const int* faces;      /* [total_faces][3] packed vertex indices */
  const int* vert_img;   /* [total_verts] image of each packed vertex */
  const int* face_img;   /* [total_faces] image of each packed face, non-decreasing (faces packed
                            image by image: the rasteriser bins each image's contiguous range) */
  const float* R;        /* [n_img][3][3] OpenCV rotation (object → camera) */
  const float* t;        /* [n_img][3] */
  const float* K;        /* [n_img][3][3] intrinsics */
  int n_img, size, total_verts, total_faces;
  int light_mode;
  const float* light_location;                  /* [3], SCFLOW_LIGHT_FIXED only */
  const float* ambient;                         /* [3] light·material ambient */
  const float* diffuse;                         /* [3] */
  const float* specular;                        /* [3] */
  float shininess;
  const float* background;                      /* [3] */
  float* images;
  float* zbuf;
  int* pix_to_face;
  float* bary;
  void* workspace;
  long long workspace_bytes;
  float* light_out;      /* optional [n_img][3]: the light location each image was shaded with
                            (object frame) — the reference's PointLights location, :209-230 */
} scflow_render_args;
long long scflow_render_workspace(int n_img, int size, int total_verts);
int scflow_render(const scflow_render_args* args, void* stream);

/* Profiling helper (bench.py roofline timing; no reference equivalent): a one-thread kernel
 * that stores the GPU's constant-rate wall clock (s_memrealtime) into stamps[idx].  Enqueued on
 * the stream of the kernel being timed, before and after it; as an ordinary kernel it is also a
 * node of a captured hipGraph, so every replay re-stamps.  scflow_wallclock_khz: its rate. */
int scflow_timestamp(unsigned long long* stamps, int idx, void* stream);
long long scflow_wallclock_khz(void);

#ifdef __cplusplus
}
#endif
#endif /* SCFLOW_HIP_H */
