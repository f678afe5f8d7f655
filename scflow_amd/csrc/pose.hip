// a8–a11: pose update, 2D-3D lift, pose-induced flow, flow resampling, layout transposes.
//
//   get_pose_from_delta_pose (ortho6d, exp)     /root/reference/models/utils/pose.py:124-169
//   cal_3d_2d_corr / lift_2d_to_3d              /root/reference/models/utils/pose.py:26-64
//   get_flow_from_delta_pose_and_points         /root/reference/models/utils/pose.py:66-88
//   flow ↓8 / flow, mask ↑8 (F.interpolate bilinear, align_corners=True)
//                                               /root/reference/models/decoder/scflow_decoder.py:197-198, 223-228
//
// The reference enumerates foreground pixels with torch.nonzero (a host sync per sample) and
// scatters the reprojected flow back with index_put inside a Python loop over the batch.  Here
// the lift is dense and predicated (one float4 {X,Y,Z,valid} per pixel, once per forward), and
// every refinement iteration is ONE launch that recomputes the pose update in its prologue
// (a few hundred flops per workgroup, kept in LDS) and reprojects every pixel: HBM-bound,
// 16 B read + 8 B written per pixel.
#include "common.h"

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

__global__ void pose_update_kernel(const float* drot6, const float* dt, const float* Rs,
                                   const float* ts, float* Rd, float* td, int n, float weight,
                                   int depth_transform) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  pose_update_one(drot6 + pose_rot_dim(depth_transform) * i, dt + 3 * i, Rs + 9 * i, ts + 3 * i,
                  Rd + 9 * i, td + 3 * i, weight, depth_transform);
}

__global__ __launch_bounds__(256) void lift_kernel(const float* __restrict__ depth,
                                                   const float* __restrict__ K,
                                                   const float* __restrict__ R,
                                                   const float* __restrict__ t,
                                                   floatx4* __restrict__ pts, int H, int W) {
#pragma clang fp contract(off)
  __shared__ float sh[21];  // Kinv[9], Rinv[9], t[3]
  const int n = blockIdx.y;
  if (threadIdx.x == 0) {
    inv3x3(K + 9 * n, sh);
    inv3x3(R + 9 * n, sh + 9);
    sh[18] = t[3 * n];
    sh[19] = t[3 * n + 1];
    sh[20] = t[3 * n + 2];
  }
  __syncthreads();
  const int HW = H * W;
  for (int p = blockIdx.x * 256 + threadIdx.x; p < HW; p += gridDim.x * 256) {
    const float d = depth[(size_t)n * HW + p];
    floatx4 o = {0.f, 0.f, 0.f, 0.f};
    if (d > 0.f) {
      const float px = (float)(p % W) * d, py = (float)(p / W) * d, pz = 1.f * d;
      float c[3];
      for (int r = 0; r < 3; ++r) {
        float s = sh[r * 3 + 0] * px;
        s += sh[r * 3 + 1] * py;
        s += sh[r * 3 + 2] * pz;
        c[r] = s - sh[18 + r];
      }
      for (int r = 0; r < 3; ++r) {
        float s = sh[9 + r * 3 + 0] * c[0];
        s += sh[9 + r * 3 + 1] * c[1];
        s += sh[9 + r * 3 + 2] * c[2];
        o[r] = s;
      }
      o[3] = 1.f;
    }
    pts[(size_t)n * HW + p] = o;
  }
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
// workgroup x == 0 stores it
__device__ __forceinline__ void pose_prologue(float* sh, int n, const float* drot6, const float* dtv,
                                              const float* Rsrc, const float* tsrc, const float* K,
                                              float* Rout, float* tout, float weight,
                                              int depth_transform, int upd) {
  if (threadIdx.x == 0) {
    if (upd) {
      pose_update_one(drot6 + pose_rot_dim(depth_transform) * n, dtv + 3 * n, Rsrc + 9 * n,
                      tsrc + 3 * n, sh, sh + 9, weight, depth_transform);
      if (blockIdx.x == 0) {
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

// flow[n][0/1][p] from pose (R,t) in LDS; `upd` != 0: compute (R,t) from the delta first
__global__ __launch_bounds__(256) void pose_flow_kernel(
    const float* __restrict__ drot6, const float* __restrict__ dtv, const float* __restrict__ Rsrc,
    const float* __restrict__ tsrc, const float* __restrict__ K, const floatx4* __restrict__ pts,
    float* __restrict__ Rout, float* __restrict__ tout, float* __restrict__ flow, int H, int W,
    float weight, int depth_transform, float invalid, int upd) {
  __shared__ float sh[21];  // R[9] t[3] K[9]
  const int n = blockIdx.y;
  pose_prologue(sh, n, drot6, dtv, Rsrc, tsrc, K, Rout, tout, weight, depth_transform, upd);
  const int HW = H * W;
  for (int p = blockIdx.x * 256 + threadIdx.x; p < HW; p += gridDim.x * 256) {
    float fx, fy;
    proj_flow(sh, pts[(size_t)n * HW + p], p % W, p / W, invalid, fx, fy);
    flow[((size_t)n * 2 + 0) * HW + p] = fx;
    flow[((size_t)n * 2 + 1) * HW + p] = fy;
  }
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

__global__ __launch_bounds__(256) void downsample_kernel(const float* __restrict__ flow,
                                                         float* __restrict__ o0, int s0,
                                                         float* __restrict__ o1, int s1, int N,
                                                         int H, int W, int h, int w, float vs) {
#pragma clang fp contract(off)
  const long long total = (long long)N * h * w;
  const long long idx = blockIdx.x * 256LL + threadIdx.x;
  if (idx >= total) return;
  const int x = (int)(idx % w);
  const long long t = idx / w;
  const int y = (int)(t % h);
  const int n = (int)(t / h);
  const Lin ly = lin_src(y, H, h), lx = lin_src(x, W, w);
  float r[2];
  for (int c = 0; c < 2; ++c) {
    const float* f = flow + ((size_t)n * 2 + c) * H * W;
    const float v = bilerp(f[(size_t)ly.i0 * W + lx.i0], f[(size_t)ly.i0 * W + lx.i1],
                           f[(size_t)ly.i1 * W + lx.i0], f[(size_t)ly.i1 * W + lx.i1], ly, lx);
    r[c] = vs * v;
  }
  o0[idx * s0 + 0] = r[0];
  o0[idx * s0 + 1] = r[1];
  if (o1) {
    o1[idx * s1 + 0] = r[0];
    o1[idx * s1 + 1] = r[1];
  }
}

__global__ __launch_bounds__(256) void upsample_kernel(const float* __restrict__ lr,
                                                       const float* __restrict__ delta,
                                                       const float* __restrict__ mask,
                                                       float* __restrict__ fo,
                                                       float* __restrict__ mo, int N, int h, int w,
                                                       int H, int W, float vs) {
#pragma clang fp contract(off)
  const long long total = (long long)N * H * W;
  const long long idx = blockIdx.x * 256LL + threadIdx.x;
  if (idx >= total) return;
  const int X = (int)(idx % W);
  const long long t = idx / W;
  const int Y = (int)(t % H);
  const int n = (int)(t / H);
  const Lin ly = lin_src(Y, h, H), lx = lin_src(X, w, W);
  const size_t b = (size_t)n * h * w;
  const size_t i00 = b + (size_t)ly.i0 * w + lx.i0, i01 = b + (size_t)ly.i0 * w + lx.i1;
  const size_t i10 = b + (size_t)ly.i1 * w + lx.i0, i11 = b + (size_t)ly.i1 * w + lx.i1;
  for (int c = 0; c < 2; ++c) {
    float v00 = lr[i00 * 2 + c], v01 = lr[i01 * 2 + c], v10 = lr[i10 * 2 + c], v11 = lr[i11 * 2 + c];
    if (delta) {
      v00 = v00 + delta[i00 * 2 + c];
      v01 = v01 + delta[i01 * 2 + c];
      v10 = v10 + delta[i10 * 2 + c];
      v11 = v11 + delta[i11 * 2 + c];
    }
    fo[((size_t)n * 2 + c) * H * W + (size_t)Y * W + X] = vs * bilerp(v00, v01, v10, v11, ly, lx);
  }
  if (mask && mo)
    mo[(size_t)n * H * W + (size_t)Y * W + X] = bilerp(mask[i00], mask[i01], mask[i10], mask[i11], ly, lx);
}

// One refinement iteration's tail in one launch (decoder a8 + a10 + a11): pose update →
// pose-induced flow (workgroups x < bf, as pose_flow_kernel), the iteration's 8× upsampled
// flow/mask prediction of the same full-resolution pixels (as upsample_kernel, from the
// iteration's low-resolution flow `lr`), and — workgroups x ≥ bf — the NEXT iteration's ↓8 flow
// (as downsample_kernel) computed straight from the new pose: each low-resolution pixel
// reprojects the 4 full-resolution points its bilinear tap reads (the same arithmetic as the
// stored flow), so nothing waits for the full-resolution flow.  lr_next must not alias lr.
__global__ __launch_bounds__(256) void pose_step_kernel(
    const float* __restrict__ drot6, const float* __restrict__ dtv, const float* __restrict__ Rsrc,
    const float* __restrict__ tsrc, const float* __restrict__ K, const floatx4* __restrict__ pts,
    float* __restrict__ Rout, float* __restrict__ tout, float* __restrict__ flow, int H, int W,
    float weight, int depth_transform, float invalid, const float* __restrict__ lr,
    const float* __restrict__ delta, const float* __restrict__ mask, float* __restrict__ fo,
    float* __restrict__ mo, float* __restrict__ o0, int s0, float* __restrict__ o1, int s1, int h,
    int w, float up_scale, float down_scale, int bf) {
#pragma clang fp contract(off)
  __shared__ float sh[21];
  const int n = blockIdx.y;
  pose_prologue(sh, n, drot6, dtv, Rsrc, tsrc, K, Rout, tout, weight, depth_transform, 1);
  const int HW = H * W;
  if ((int)blockIdx.x < bf) {
    for (int p = blockIdx.x * 256 + threadIdx.x; p < HW; p += bf * 256) {
      const int X = p % W, Y = p / W;
      float fx, fy;
      proj_flow(sh, pts[(size_t)n * HW + p], X, Y, invalid, fx, fy);
      flow[((size_t)n * 2 + 0) * HW + p] = fx;
      flow[((size_t)n * 2 + 1) * HW + p] = fy;
      if (fo) {
        const Lin ly = lin_src(Y, h, H), lx = lin_src(X, w, W);
        const size_t b = (size_t)n * h * w;
        const size_t i00 = b + (size_t)ly.i0 * w + lx.i0, i01 = b + (size_t)ly.i0 * w + lx.i1;
        const size_t i10 = b + (size_t)ly.i1 * w + lx.i0, i11 = b + (size_t)ly.i1 * w + lx.i1;
        for (int c = 0; c < 2; ++c) {
          float v00 = lr[i00 * 2 + c], v01 = lr[i01 * 2 + c], v10 = lr[i10 * 2 + c],
                v11 = lr[i11 * 2 + c];
          if (delta) {
            v00 = v00 + delta[i00 * 2 + c];
            v01 = v01 + delta[i01 * 2 + c];
            v10 = v10 + delta[i10 * 2 + c];
            v11 = v11 + delta[i11 * 2 + c];
          }
          fo[((size_t)n * 2 + c) * HW + p] = up_scale * bilerp(v00, v01, v10, v11, ly, lx);
        }
        if (mask && mo)
          mo[(size_t)n * HW + p] = bilerp(mask[i00], mask[i01], mask[i10], mask[i11], ly, lx);
      }
    }
    return;
  }
  const int bl = gridDim.x - bf;
  for (int q = (blockIdx.x - bf) * 256 + threadIdx.x; q < h * w; q += bl * 256) {
    const int x = q % w, y = q / w;
    const Lin ly = lin_src(y, H, h), lx = lin_src(x, W, w);
    float f[4][2];  // [dy·2 + dx][axis]
    for (int k = 0; k < 4; ++k) {
      const int cy = (k >> 1) ? ly.i1 : ly.i0, cx = (k & 1) ? lx.i1 : lx.i0;
      proj_flow(sh, pts[(size_t)n * HW + (size_t)cy * W + cx], cx, cy, invalid, f[k][0], f[k][1]);
    }
    const size_t idx = (size_t)n * h * w + q;
    for (int a = 0; a < 2; ++a) {
      const float v = down_scale * bilerp(f[0][a], f[1][a], f[2][a], f[3][a], ly, lx);
      o0[idx * s0 + a] = v;
      if (o1) o1[idx * s1 + a] = v;
    }
  }
}

// batched 2-D transpose through a padded LDS tile
__global__ __launch_bounds__(256) void transpose_kernel(const float* __restrict__ in,
                                                        float* __restrict__ out, int A, int B,
                                                        long long ins, int ias, long long ons,
                                                        int obs) {
  __shared__ float tile[32][33];
  const int n = blockIdx.z;
  const int a0 = blockIdx.y * 32, b0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 × 8
  for (int k = ty; k < 32; k += 8) {
    const int a = a0 + k, b = b0 + tx;
    if (a < A && b < B) tile[k][tx] = in[n * ins + (long long)a * ias + b];
  }
  __syncthreads();
  for (int k = ty; k < 32; k += 8) {
    const int b = b0 + k, a = a0 + tx;
    if (a < A && b < B) out[n * ons + (long long)b * obs + a] = tile[tx][k];
  }
}

}  // namespace

SCFLOW_API int scflow_pose_update(const float* drot6, const float* dt, const float* R_src,
                                  const float* t_src, float* R_dst, float* t_dst, int n,
                                  float weight, int depth_transform, void* stream) {
  if (!drot6 || !dt || !R_src || !t_src || !R_dst || !t_dst || n <= 0 ||
      !pose_mode_ok(depth_transform))
    return SCFLOW_EINVAL;
  pose_update_kernel<<<(n + 63) / 64, 64, 0, (hipStream_t)stream>>>(drot6, dt, R_src, t_src, R_dst,
                                                                   t_dst, n, weight, depth_transform);
  return scflow_launch_status();
}

SCFLOW_API int scflow_lift_points(const float* depth, const float* K, const float* R,
                                  const float* t, float* points, int n, int h, int w,
                                  void* stream) {
  if (!depth || !K || !R || !t || !points || n <= 0 || h <= 0 || w <= 0) return SCFLOW_EINVAL;
  if (!aligned16(points)) return SCFLOW_EALIGN;
  const int bx = ceil_div((long long)h * w, 256) < 256 ? ceil_div((long long)h * w, 256) : 256;
  lift_kernel<<<dim3(bx, n), 256, 0, (hipStream_t)stream>>>(depth, K, R, t, (floatx4*)points, h, w);
  return scflow_launch_status();
}

SCFLOW_API int scflow_pose_flow(const float* R, const float* t, const float* K,
                                const float* points, float* flow, int n, int h, int w,
                                float invalid_num, void* stream) {
  if (!R || !t || !K || !points || !flow || n <= 0 || h <= 0 || w <= 0) return SCFLOW_EINVAL;
  if (!aligned16(points)) return SCFLOW_EALIGN;
  const int bx = ceil_div((long long)h * w, 256) < 256 ? ceil_div((long long)h * w, 256) : 256;
  pose_flow_kernel<<<dim3(bx, n), 256, 0, (hipStream_t)stream>>>(
      nullptr, nullptr, R, t, K, (const floatx4*)points, nullptr, nullptr, flow, h, w, 10.f, 0,
      invalid_num, 0);
  return scflow_launch_status();
}

SCFLOW_API int scflow_pose_update_flow(const float* drot6, const float* dt, const float* R_src,
                                       const float* t_src, const float* K, const float* points,
                                       float* R_dst, float* t_dst, float* flow, int n, int h,
                                       int w, float weight, int depth_transform,
                                       float invalid_num, void* stream) {
  if (!drot6 || !dt || !R_src || !t_src || !K || !points || !R_dst || !t_dst || !flow || n <= 0 ||
      h <= 0 || w <= 0 || !pose_mode_ok(depth_transform))
    return SCFLOW_EINVAL;
  if (!aligned16(points)) return SCFLOW_EALIGN;
  const int bx = ceil_div((long long)h * w, 256) < 256 ? ceil_div((long long)h * w, 256) : 256;
  pose_flow_kernel<<<dim3(bx, n), 256, 0, (hipStream_t)stream>>>(
      drot6, dt, R_src, t_src, K, (const floatx4*)points, R_dst, t_dst, flow, h, w, weight,
      depth_transform, invalid_num, 1);
  return scflow_launch_status();
}

SCFLOW_API int scflow_flow_downsample(const float* flow, float* out0, int s0, float* out1, int s1,
                                      int n, int H, int W, int h, int w, float value_scale,
                                      void* stream) {
  if (!flow || !out0 || s0 < 2 || (out1 && s1 < 2) || n <= 0 || H <= 0 || W <= 0 || h <= 0 || w <= 0)
    return SCFLOW_EINVAL;
  const long long total = (long long)n * h * w;
  downsample_kernel<<<(unsigned)((total + 255) / 256), 256, 0, (hipStream_t)stream>>>(
      flow, out0, s0, out1, s1, n, H, W, h, w, value_scale);
  return scflow_launch_status();
}

SCFLOW_API int scflow_flow_upsample(const float* lr, const float* delta, const float* mask,
                                    float* flow_out, float* mask_out, int n, int h, int w, int H,
                                    int W, float value_scale, void* stream) {
  if (!lr || !flow_out || n <= 0 || h <= 0 || w <= 0 || H <= 0 || W <= 0) return SCFLOW_EINVAL;
  const long long total = (long long)n * H * W;
  upsample_kernel<<<(unsigned)((total + 255) / 256), 256, 0, (hipStream_t)stream>>>(
      lr, delta, mask, flow_out, mask_out, n, h, w, H, W, value_scale);
  return scflow_launch_status();
}

SCFLOW_API int scflow_pose_step(const float* drot6, const float* dt, const float* R_src,
                                const float* t_src, const float* K, const float* points,
                                float* R_dst, float* t_dst, float* flow, int n, int H, int W,
                                float weight, int depth_transform, float invalid_num,
                                const float* lr, const float* delta, const float* mask,
                                float* flow_up, float* mask_up, float* lr_next, int s_next,
                                float* hx_next, int s_hx, int h, int w, float up_scale,
                                float down_scale, void* stream) {
  if (!drot6 || !dt || !R_src || !t_src || !K || !points || !R_dst || !t_dst || !flow || n <= 0 ||
      H <= 0 || W <= 0 || !pose_mode_ok(depth_transform))
    return SCFLOW_EINVAL;
  if ((flow_up || lr_next) && (h <= 0 || w <= 0)) return SCFLOW_EINVAL;
  if (flow_up && !lr) return SCFLOW_EINVAL;
  if (lr_next && (s_next < 2 || (hx_next && s_hx < 2) || lr_next == lr)) return SCFLOW_EINVAL;
  if (!aligned16(points)) return SCFLOW_EALIGN;
  const int bf = ceil_div((long long)H * W, 256) < 256 ? ceil_div((long long)H * W, 256) : 256;
  const int bl = lr_next ? (ceil_div((long long)h * w, 256) < 64 ? ceil_div((long long)h * w, 256) : 64) : 0;
  pose_step_kernel<<<dim3(bf + bl, n), 256, 0, (hipStream_t)stream>>>(
      drot6, dt, R_src, t_src, K, (const floatx4*)points, R_dst, t_dst, flow, H, W, weight,
      depth_transform, invalid_num, lr, delta, mask, flow_up, mask_up, lr_next, s_next, hx_next,
      s_hx, h, w, up_scale, down_scale, bf);
  return scflow_launch_status();
}

SCFLOW_API int scflow_transpose(const float* in, float* out, int n, int A, int B, long long ins,
                                int ias, long long ons, int obs, void* stream) {
  if (!in || !out || n <= 0 || A <= 0 || B <= 0 || ias < B || obs < A) return SCFLOW_EINVAL;
  dim3 grid(ceil_div(B, 32), ceil_div(A, 32), n);
  transpose_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(in, out, A, B, ins, ias, ons, obs);
  return scflow_launch_status();
}

SCFLOW_API int scflow_version(void) { return 1; }

SCFLOW_API const char* scflow_strerror(int code) {
  switch (code) {
    case SCFLOW_OK: return "ok";
    case SCFLOW_EINVAL: return "invalid argument";
    case SCFLOW_EUNSUPPORTED: return "unsupported shape for this build";
    case SCFLOW_EALIGN: return "pointer or stride not 16-byte aligned";
    default: return hipGetErrorString((hipError_t)code);
  }
}

// ------------------------------------------------------------------------------------------
// profiling helper: GPU wall-clock timestamps as graph-capturable kernel nodes
// ------------------------------------------------------------------------------------------
__global__ void timestamp_kernel(unsigned long long* stamps, int idx) {
  stamps[idx] = __builtin_amdgcn_s_memrealtime();
}

SCFLOW_API int scflow_timestamp(unsigned long long* stamps, int idx, void* stream) {
  if (!stamps || idx < 0) return SCFLOW_EINVAL;
  timestamp_kernel<<<1, 1, 0, (hipStream_t)stream>>>(stamps, idx);
  return scflow_launch_status();
}

SCFLOW_API long long scflow_wallclock_khz(void) {
  int dev = 0, khz = 0;
  if (hipGetDevice(&dev) != hipSuccess) return SCFLOW_EINVAL;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess) return SCFLOW_EINVAL;
  return khz;
}
