// Device helpers of the pose kernels (pose.hip) shared with the fused pose-head tail
// (phtail.hip): pose update (pose.py:124-169), reprojection (pose.py:66-88), bilinear
// align_corners=True resampling (scflow_decoder.py:197-198, 223-228).
#pragma once
#include "common.h"
#include <stdlib.h>

namespace {

// ---- small fixed-size linear algebra (row-major 3×3) ----
__device__ void inv3x3(const float* m, float* o) {
  // adjugate / determinant in double: the reference uses torch.inverse (LU, fp32); computing the
  // inverse exactly then rounding keeps us within an ulp of it.
  double a = m[0], b = m[1], c = m[2], d = m[3], e = m[4], f = m[5], g = m[6], h = m[7], i = m[8];
  double A = e * i - f * h, B = -(d * i - f * g), C = d * h - e * g;
  double det = a * A + b * B + c * C;
  double id = 1.0 / det;
  o[0] = (float)(A * id);
  o[1] = (float)(-(b * i - c * h) * id);
  o[2] = (float)((b * f - c * e) * id);
  o[3] = (float)(B * id);
  o[4] = (float)((a * i - c * g) * id);
  o[5] = (float)(-(a * f - c * d) * id);
  o[6] = (float)(C * id);
  o[7] = (float)(-(a * h - b * g) * id);
  o[8] = (float)((a * e - b * d) * id);
}

// Pose-update mode word (scflow_pose_update / _flow / _step): bit 0 the depth transform
// (0 exp, 1 linear), SCFLOW_POSE_QUAT_XYZW (16) a 4-value quaternion delta rotation instead of
// ortho6d.
__host__ __device__ inline int pose_rot_dim(int mode) { return (mode & SCFLOW_POSE_QUAT_XYZW) ? 4 : 6; }
__host__ inline bool pose_mode_ok(int mode) { return (mode & ~(SCFLOW_POSE_QUAT_XYZW | 1)) == 0; }

// ΔR from the head's rotation output:
//  ortho6d (pose.py:153-169): x = normalize(o[0:3]), z = normalize(x × o[3:6]), y = z × x,
//    columns (x, y, z);
//  quaternion (pose.py:132-133, kornia.geometry.conversions.quaternion_to_rotation_matrix with
//    the x, y, z, w coefficient order that the head's identity bias [0, 0, 0, 1] implies,
//    pose_head.py:192-194): q = q / max(‖q‖, 1e-12), then the standard unit-quaternion matrix.
__device__ void delta_rotation(const float* d, int quat, float* D) {
#pragma clang fp contract(off)
  if (quat) {
    float q[4] = {d[0], d[1], d[2], d[3]};
    float nq = sqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    nq = fmaxf(nq, 1e-12f);
    for (int k = 0; k < 4; ++k) q[k] = q[k] / nq;
    const float x = q[0], y = q[1], z = q[2], w = q[3];
    const float tx = 2.f * x, ty = 2.f * y, tz = 2.f * z;
    const float twx = tx * w, twy = ty * w, twz = tz * w;
    const float txx = tx * x, txy = ty * x, txz = tz * x;
    const float tyy = ty * y, tyz = tz * y, tzz = tz * z;
    D[0] = 1.f - (tyy + tzz); D[1] = txy - twz;         D[2] = txz + twy;
    D[3] = txy + twz;         D[4] = 1.f - (txx + tzz); D[5] = tyz - twx;
    D[6] = txz - twy;         D[7] = tyz + twx;         D[8] = 1.f - (txx + tyy);
    return;
  }
  float x[3] = {d[0], d[1], d[2]}, yr[3] = {d[3], d[4], d[5]};
  float nx = sqrtf(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]);
  nx = fmaxf(nx, 1e-12f);
  for (int k = 0; k < 3; ++k) x[k] = x[k] / nx;
  float z[3] = {x[1] * yr[2] - x[2] * yr[1], x[2] * yr[0] - x[0] * yr[2], x[0] * yr[1] - x[1] * yr[0]};
  float nz = sqrtf(z[0] * z[0] + z[1] * z[1] + z[2] * z[2]);
  nz = fmaxf(nz, 1e-12f);
  for (int k = 0; k < 3; ++k) z[k] = z[k] / nz;
  float y[3] = {z[1] * x[2] - z[2] * x[1], z[2] * x[0] - z[0] * x[2], z[0] * x[1] - z[1] * x[0]};
  D[0] = x[0]; D[1] = y[0]; D[2] = z[0];
  D[3] = x[1]; D[4] = y[1]; D[5] = z[1];
  D[6] = x[2]; D[7] = y[2]; D[8] = z[2];
}

// ΔR (ortho6d or quaternion), then R_dst = ΔR·R_src, and the translation update
// (get_pose_from_delta_pose, pose.py:124-149)
__device__ void pose_update_one(const float* d6, const float* dt, const float* Rs, const float* ts,
                                float* Rd, float* td, float weight, int mode) {
#pragma clang fp contract(off)
  const int depth_transform = mode & 1;
  float D[9];
  delta_rotation(d6, (mode & SCFLOW_POSE_QUAT_XYZW) != 0, D);
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) {
      float s = D[r * 3 + 0] * Rs[0 * 3 + c];
      s += D[r * 3 + 1] * Rs[1 * 3 + c];
      s += D[r * 3 + 2] * Rs[2 * 3 + c];
      Rd[r * 3 + c] = s;
    }
  float vz = depth_transform == 0 ? ts[2] / expf(dt[2]) : ts[2] * (dt[2] + 1.f);
  td[0] = vz * (dt[0] / weight + ts[0] / ts[2]);
  td[1] = vz * (dt[1] / weight + ts[1] / ts[2]);
  td[2] = vz;
}

// flow of one pixel p (point P = {X, Y, Z, valid}) under the pose in LDS (R[9] t[3] K[9])
__device__ __forceinline__ void proj_flow(const float* sh, const floatx4 P, int X, int Y,
                                          float invalid, float& fx, float& fy) {
#pragma clang fp contract(off)
  fx = invalid;
  fy = invalid;
  if (P[3] != 0.f) {
    float c[3], u[3];
    for (int r = 0; r < 3; ++r) {
      float s = sh[r * 3 + 0] * P[0];
      s += sh[r * 3 + 1] * P[1];
      s += sh[r * 3 + 2] * P[2];
      c[r] = s + sh[9 + r];
    }
    for (int r = 0; r < 3; ++r) {
      float s = sh[12 + r * 3 + 0] * c[0];
      s += sh[12 + r * 3 + 1] * c[1];
      s += sh[12 + r * 3 + 2] * c[2];
      u[r] = s;
    }
    fx = u[0] / u[2] - (float)X;
    fy = u[1] / u[2] - (float)Y;
  }
}

// the pose of image n into LDS (R[9] t[3] K[9]); `upd` != 0: (R,t) from the delta first, and
// `store` (one workgroup per image) writes it to Rout / tout
__device__ __forceinline__ void pose_prologue(float* sh, int n, const float* drot6, const float* dtv,
                                              const float* Rsrc, const float* tsrc, const float* K,
                                              float* Rout, float* tout, float weight,
                                              int depth_transform, int upd, bool store) {
  if (threadIdx.x == 0) {
    if (upd) {
      pose_update_one(drot6 + pose_rot_dim(depth_transform) * n, dtv + 3 * n, Rsrc + 9 * n,
                      tsrc + 3 * n, sh, sh + 9, weight, depth_transform);
      if (store) {
        for (int k = 0; k < 9; ++k) Rout[9 * n + k] = sh[k];
        for (int k = 0; k < 3; ++k) tout[3 * n + k] = sh[9 + k];
      }
    } else {
      for (int k = 0; k < 9; ++k) sh[k] = Rsrc[9 * n + k];
      for (int k = 0; k < 3; ++k) sh[9 + k] = tsrc[3 * n + k];
    }
    for (int k = 0; k < 9; ++k) sh[12 + k] = K[9 * n + k];
  }
  __syncthreads();
}

// align_corners=True source index and weights, as ATen's upsample_bilinear2d
struct Lin {
  int i0, i1;
  float l0, l1;
};
__device__ __forceinline__ Lin lin_src(int dst, int in_size, int out_size) {
#pragma clang fp contract(off)
  const float scale = out_size > 1 ? (float)(in_size - 1) / (float)(out_size - 1) : 0.f;
  const float real = scale * (float)dst;
  Lin r;
  r.i0 = (int)real;
  r.i1 = r.i0 + (r.i0 < in_size - 1 ? 1 : 0);
  r.l1 = real - (float)r.i0;
  r.l0 = 1.f - r.l1;
  return r;
}

__device__ __forceinline__ float bilerp(float v00, float v01, float v10, float v11, const Lin& ly,
                                        const Lin& lx) {
#pragma clang fp contract(off)
  return ly.l0 * (lx.l0 * v00 + lx.l1 * v01) + ly.l1 * (lx.l0 * v10 + lx.l1 * v11);
}

// One refinement iteration's tail (decoder a8 + a10 + a11): pose update → pose-induced flow
// (work blocks bx < bf, as pose_flow_kernel), the iteration's 8× upsampled flow/mask prediction of
// the same full-resolution pixels (as upsample_kernel, from the iteration's low-resolution flow
// `lr`), and — blocks bx ≥ bf — the NEXT iteration's ↓8 flow (as downsample_kernel) computed
// straight from the new pose: each low-resolution pixel reprojects the 4 full-resolution points
// its bilinear tap reads (the same arithmetic as the stored flow), so nothing waits for the
// full-resolution flow.  lr_next must not alias lr.  A block is `nt` threads (tid < nt) and covers
// `nt` pixels per pass; `nb` blocks of kind bf ("full") / bl ("low") per image.
struct PoseStepArgs {
  const float* drot6; const float* dtv; const float* Rsrc; const float* tsrc; const float* K;
  const floatx4* pts;
  float* Rout; float* tout; float* flow;
  int H, W; float weight; int depth_transform; float invalid;
  const float* lr; const float* delta; const float* mask; float* fo; float* mo;
  float* o0; int s0; float* o1; int s1; int h, w; float up_scale, down_scale;
  int bf, bl;
  int given;  // 1: Rsrc / tsrc are the updated pose already (no update, Rout / tout unused)
  // heads fused (hx != NULL; scflow_pose_step_heads): the pose delta of image n is computed in
  // the launch from the last FC's K-split partial sums — x = relu(Σ_z hx[z·hxs] + hxb), the
  // label[0] class's rch rotation rows of Wr and 3 translation rows of Wt (MultiClassPoseHead,
  // pose_head.py:203-211) — instead of read from drot6 / dtv; block 0 of image n writes it to
  // drot_out / dt_out (the decoder's returned delta lists)
  const float* hx; long long hxs; int hk, hsplit; const float* hxb;
  const float* Wr; const float* br; const float* Wt; const float* bt; const long long* hlabel;
  int hrch, hncls; float* drot_out; float* dt_out;
};

// the heads' 9 (rch + 3) dot products of image n over the block's nt threads (threads split K),
// wave sums by xor shuffles, then the waves' partials in order through LDS → hs[0 .. rch+3)
// (bias added).  hs: 16·(nt/64) + 16 floats of LDS.  Every thread calls this (barrier inside).
// The separate heads launch (scflow_ph_heads*, ph_heads_kernel) runs this same function, so the
// fused and the separate tail give bit-identical deltas.
__device__ __forceinline__ void pose_heads(const PoseStepArgs& a, float* hs, int n, int tid, int nt) {
#pragma clang fp contract(off)
  const int nr = a.hrch + 3;
  long long cls = a.hlabel[0];  // every sample uses label[0]'s class (reference quirk)
  if (cls < 0 || cls >= a.hncls) cls = 0;
  // the bias with the weights (one dependent load round after the label, not two)
  float bias_r = 0.f;
  if (tid < nr) bias_r = tid < a.hrch ? a.br[cls * a.hrch + tid] : a.bt[cls * 3 + (tid - a.hrch)];
  float acc[9];
#pragma unroll
  for (int r = 0; r < 9; ++r) acc[r] = 0.f;
  for (int k = tid; k < a.hk; k += nt) {
    float x = a.hx[(size_t)n * a.hk + k];
    if (a.hsplit > 0) {  // the previous FC's K-split partial sums: relu(Σ + bias)
      for (int z = 1; z < a.hsplit; ++z) x += a.hx[z * a.hxs + (size_t)n * a.hk + k];
      x = fmaxf(x + a.hxb[k], 0.f);
    }
#pragma unroll
    for (int r = 0; r < 9; ++r) {
      if (r < nr) {
        const float* wrow = r < a.hrch ? a.Wr + ((size_t)cls * a.hrch + r) * a.hk
                                       : a.Wt + ((size_t)cls * 3 + (r - a.hrch)) * a.hk;
        acc[r] += wrow[k] * x;
      }
    }
  }
  const int lane = tid & 63, wv = tid >> 6;
#pragma unroll
  for (int r = 0; r < 9; ++r) {
    float v = acc[r];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) hs[16 + wv * 16 + r] = v;
  }
  __syncthreads();
  if (tid < nr) {
    float v = 0.f;
    for (int w = 0; w < nt / 64; ++w) v += hs[16 + w * 16 + tid];
    hs[tid] = v + bias_r;
  }
  __syncthreads();
}

// sh: 21 floats of LDS; every thread of the block calls this (barrier inside)
// fresh: drot6/dtv were written earlier in the same launch by another workgroup — read them
// with agent-scope (sc1, vector) loads, never through the scalar cache
__device__ __forceinline__ void pose_step_body(const PoseStepArgs& a, float* sh, int bx, int n,
                                               int tid, int nt, bool fresh = false,
                                               float* hs = nullptr) {
#pragma clang fp contract(off)
  const int H = a.H, W = a.W, h = a.h, w = a.w;
  const int HW = H * W;
  // Loads that depend on nothing computed here are issued first, so that they share one memory
  // round with the heads' inputs instead of each costing its own after a barrier: the source
  // pose and intrinsics (into LDS behind the heads, fused path) and the 4 full-resolution points
  // of this thread's first ↓8 pixel (the ↓8 blocks).
  const bool fused = hs && a.hx && !a.given;
  float pre = 0.f;
  if (fused) {
    if (tid < 9)
      pre = a.Rsrc[9 * n + tid];
    else if (tid < 12)
      pre = a.tsrc[3 * n + tid - 9];
    else if (tid < 21)
      pre = a.K[9 * n + tid - 12];
  }
  const int q0 = (bx - a.bf) * nt + tid;
  const bool lowres = bx >= a.bf;
  floatx4 p0[4];
  if (lowres && q0 < h * w) {
    const Lin ly = lin_src(q0 / w, H, h), lx = lin_src(q0 % w, W, w);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int cy = (k >> 1) ? ly.i1 : ly.i0, cx = (k & 1) ? lx.i1 : lx.i0;
      p0[k] = a.pts[(size_t)n * HW + (size_t)cy * W + cx];
    }
  }
  if (fused) {
    pose_heads(a, hs, n, tid, nt);
    if (tid < 21) hs[80 + tid] = pre;  // R[9] t[3] K[9]
    __syncthreads();
  }
  if (a.given) {  // the pose of this iteration was updated by the ↓8 part: 21 plain loads
    if (tid < 9)
      sh[tid] = a.Rsrc[9 * n + tid];
    else if (tid < 12)
      sh[tid] = a.tsrc[3 * n + tid - 9];
    else if (tid < 21)
      sh[tid] = a.K[9 * n + tid - 12];
  } else if (tid == 0) {
    const int rd = pose_rot_dim(a.depth_transform);
    float d[6], dt[3];
    if (hs && a.hx) {  // heads fused: the delta from LDS; block 0 writes it out
      for (int k = 0; k < rd; ++k) d[k] = hs[k];
      for (int k = 0; k < 3; ++k) dt[k] = hs[rd + k];
      if (bx == 0) {
        for (int k = 0; k < rd; ++k) a.drot_out[rd * n + k] = d[k];
        for (int k = 0; k < 3; ++k) a.dt_out[3 * n + k] = dt[k];
      }
    } else {
      for (int k = 0; k < rd; ++k)
        d[k] = fresh ? __hip_atomic_load(a.drot6 + rd * n + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                     : a.drot6[rd * n + k];
      for (int k = 0; k < 3; ++k)
        dt[k] = fresh ? __hip_atomic_load(a.dtv + 3 * n + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                      : a.dtv[3 * n + k];
    }
    if (fused)
      pose_update_one(d, dt, hs + 80, hs + 89, sh, sh + 9, a.weight, a.depth_transform);
    else
      pose_update_one(d, dt, a.Rsrc + 9 * n, a.tsrc + 3 * n, sh, sh + 9, a.weight, a.depth_transform);
    if (bx == 0) {
      for (int k = 0; k < 9; ++k) a.Rout[9 * n + k] = sh[k];
      for (int k = 0; k < 3; ++k) a.tout[3 * n + k] = sh[9 + k];
    }
    for (int k = 0; k < 9; ++k) sh[12 + k] = fused ? hs[92 + k] : a.K[9 * n + k];
  }
  __syncthreads();
  if (!lowres) {
    for (int p = bx * nt + tid; p < HW; p += a.bf * nt) {
      const int X = p % W, Y = p / W;
      float fx, fy;
      proj_flow(sh, a.pts[(size_t)n * HW + p], X, Y, a.invalid, fx, fy);
      a.flow[((size_t)n * 2 + 0) * HW + p] = fx;
      a.flow[((size_t)n * 2 + 1) * HW + p] = fy;
      if (a.fo) {
        const Lin ly = lin_src(Y, h, H), lx = lin_src(X, w, W);
        const size_t b = (size_t)n * h * w;
        const size_t i00 = b + (size_t)ly.i0 * w + lx.i0, i01 = b + (size_t)ly.i0 * w + lx.i1;
        const size_t i10 = b + (size_t)ly.i1 * w + lx.i0, i11 = b + (size_t)ly.i1 * w + lx.i1;
        for (int c = 0; c < 2; ++c) {
          float v00 = a.lr[i00 * 2 + c], v01 = a.lr[i01 * 2 + c], v10 = a.lr[i10 * 2 + c],
                v11 = a.lr[i11 * 2 + c];
          if (a.delta) {
            v00 = v00 + a.delta[i00 * 2 + c];
            v01 = v01 + a.delta[i01 * 2 + c];
            v10 = v10 + a.delta[i10 * 2 + c];
            v11 = v11 + a.delta[i11 * 2 + c];
          }
          a.fo[((size_t)n * 2 + c) * HW + p] = a.up_scale * bilerp(v00, v01, v10, v11, ly, lx);
        }
        if (a.mask && a.mo)
          a.mo[(size_t)n * HW + p] =
              bilerp(a.mask[i00], a.mask[i01], a.mask[i10], a.mask[i11], ly, lx);
      }
    }
    return;
  }
  for (int q = q0; q < h * w; q += a.bl * nt) {
    const int x = q % w, y = q / w;
    const Lin ly = lin_src(y, H, h), lx = lin_src(x, W, w);
    float f[4][2];  // [dy·2 + dx][axis]
    for (int k = 0; k < 4; ++k) {
      const int cy = (k >> 1) ? ly.i1 : ly.i0, cx = (k & 1) ? lx.i1 : lx.i0;
      const floatx4 P = q == q0 ? p0[k] : a.pts[(size_t)n * HW + (size_t)cy * W + cx];
      proj_flow(sh, P, cx, cy, a.invalid, f[k][0], f[k][1]);
    }
    const size_t idx = (size_t)n * h * w + q;
    for (int c = 0; c < 2; ++c) {
      const float v = a.down_scale * bilerp(f[0][c], f[1][c], f[2][c], f[3][c], ly, lx);
      a.o0[idx * a.s0 + c] = v;
      if (a.o1) a.o1[idx * a.s1 + c] = v;
    }
  }
}

// scflow_pose_step's argument checks and block split (blocks of `nt` threads): 0 or an error
// workgroups per image of the full-resolution part from a given pose (the decoder's deferred,
// side-stream launch); SCFLOW_FULLRES_BLOCKS overrides the default 64 (tuning)
static inline int fullres_blocks() {
  static int v = 0;
  if (v == 0) {
    const char* e = getenv("SCFLOW_FULLRES_BLOCKS");
    v = e && atoi(e) > 0 ? atoi(e) : 64;
  }
  return v;
}

static inline int pose_step_args(PoseStepArgs* a, const float* drot6, const float* dt,
                                 const float* R_src, const float* t_src, const float* K,
                                 const float* points, float* R_dst, float* t_dst, float* flow, int n,
                                 int H, int W, float weight, int depth_transform, float invalid_num,
                                 const float* lr, const float* delta, const float* mask,
                                 float* flow_up, float* mask_up, float* lr_next, int s_next,
                                 float* hx_next, int s_hx, int h, int w, float up_scale,
                                 float down_scale, int nt) {
  const bool given = !drot6;  // the full-resolution part from an updated pose (R_src, t_src)
  if ((!given && (!dt || !R_dst || !t_dst)) || !R_src || !t_src || !K || !points || !flow ||
      n <= 0 || H <= 0 || W <= 0 || (depth_transform & ~(SCFLOW_POSE_QUAT_XYZW | 1)) != 0)
    return SCFLOW_EINVAL;
  if (given && lr_next) return SCFLOW_EINVAL;
  if ((flow_up || lr_next) && (h <= 0 || w <= 0)) return SCFLOW_EINVAL;
  if (flow_up && !lr) return SCFLOW_EINVAL;
  if (lr_next && (s_next < 2 || (hx_next && s_hx < 2) || lr_next == lr)) return SCFLOW_EINVAL;
  if (!aligned16(points)) return SCFLOW_EALIGN;
  a->drot6 = drot6; a->dtv = dt; a->Rsrc = R_src; a->tsrc = t_src; a->K = K;
  a->pts = (const floatx4*)points; a->Rout = R_dst; a->tout = t_dst; a->flow = flow;
  a->H = H; a->W = W; a->weight = weight; a->depth_transform = depth_transform;
  a->invalid = invalid_num; a->lr = lr; a->delta = delta; a->mask = mask; a->fo = flow_up;
  a->mo = mask_up; a->o0 = lr_next; a->s0 = s_next; a->o1 = hx_next; a->s1 = s_hx; a->h = h;
  a->w = w; a->up_scale = up_scale; a->down_scale = down_scale;
  a->given = given ? 1 : 0;
  a->hx = nullptr;
  const int bf = ceil_div((long long)H * W, nt);
  // from a given pose the part runs beside other work (the decoder's side stream): 4 pixels per
  // thread, a quarter of the workgroups to schedule
  const int bfmax = given ? fullres_blocks() : 256;
  a->bf = bf < bfmax ? bf : bfmax;
  const int bl = ceil_div((long long)h * w, nt);
  a->bl = lr_next ? (bl < 64 ? bl : 64) : 0;
  return SCFLOW_OK;
}

}  // namespace
