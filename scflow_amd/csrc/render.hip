// §8(f)-3 — mesh renderer: z-buffer rasterisation + hard Phong shading of a batch of posed
// meshes, the inputs of the refinement hot path (rendered image, rendered depth).
//
// Replaces the pytorch3d pipeline the reference builds in models/utils/rendering.py
// (Renderer.forward :196-248 → MeshRendererWithFragments(MeshRasterizer, HardPhongShader) with
// cameras_from_opencv_projection :17-60), as configured in configs/refine_models/
// scflow_ycbv_real.py:261-274 (faces_per_pixel 1, blur 0, hard blending).  Conventions (see
// oracle/render_oracle.py for the restatement):
//   * view point X = R·v + t; NDC x = −(u − c0)/s, y = −(v − c0)/s, (u, v) the OpenCV projection,
//     c0 = (S−1)/2 = s; z = view depth;
//   * pixel (r, c) samples NDC (1 − (2c+1)/W, 1 − (2r+1)/H);
//   * 2D barycentrics from edge functions (area + 1e-8, |area| ≤ 1e-8 skipped), perspective
//     corrected; inside ⇔ all three > 0 and pz ≥ 0; nearest pz wins, ties → lower face index.
//
// Three launches:
//   render_project_kernel — one thread per packed vertex: NDC + depth into the per-image vertex
//     slots, and the image's minimum vertex depth (a wave-level min per image, then one atomicMin
//     on the float bits per image and wave; depths > 0) for the light placement.
//   render_tile_kernel    — one workgroup per 16×16 screen tile of an image: the image's faces
//     whose screen bbox meets the tile are binned into LDS, and each pixel keeps the minimum of
//     (depth bits << 32 | face) over them (positive floats order like their bit patterns), so the
//     nearest face wins and equal depths resolve to the lower index, independent of order.
//   render_shade_kernel   — one thread per pixel: decodes the winner, recomputes its perspective-
//     correct barycentrics and depth, writes zbuf / pix_to_face / bary, interpolates position,
//     normal and vertex colour and applies pytorch3d's Phong model (ambient + diffuse·texel +
//     specular, shininess 64) with one point light; background colour, alpha 0 where empty.
#include "common.h"

namespace {

constexpr float K_EPS = 1e-8f;

__global__ void render_project_kernel(scflow_render_args a, const int* __restrict__ vert_img,
                                      float* __restrict__ vproj, unsigned* __restrict__ zmin_bits,
                                      int nverts) {
  const int vi = blockIdx.x * blockDim.x + threadIdx.x;
  const bool valid = vi < nverts;
  int n = -1;
  unsigned key = 0xFFFFFFFFu;  // this vertex's depth bits (positive floats order like their bits)
  if (valid) {
    n = vert_img[vi];
    const float* R = a.R + 9 * n;
    const float* t = a.t + 3 * n;
    const float* K = a.K + 9 * n;
    const float x = a.verts[3 * vi], y = a.verts[3 * vi + 1], z = a.verts[3 * vi + 2];
    const float X = R[0] * x + R[1] * y + R[2] * z + t[0];
    const float Y = R[3] * x + R[4] * y + R[5] * z + t[1];
    const float Z = R[6] * x + R[7] * y + R[8] * z + t[2];
    const float u = K[0] * X / Z + K[2];
    const float v = K[4] * Y / Z + K[5];
    const float c0 = 0.5f * (float)(a.size - 1);
    vproj[3 * vi] = -(u - c0) / c0;
    vproj[3 * vi + 1] = -(v - c0) / c0;
    vproj[3 * vi + 2] = Z;
    if (Z > 0.f) key = __float_as_uint(Z);
  }
  // per-image minimum: the wave's lanes of one image (vertices are packed image by image, so a
  // wave spans one or two) reduce their depths first, then one atomicMin per image and wave
  const int lane = threadIdx.x & 63;
  unsigned long long pending = __ballot(valid);
  while (pending) {
    const int leader = __ffsll((long long)pending) - 1;
    const int ln = __shfl(n, leader);
    const bool mine = valid && n == ln;
    unsigned m = mine ? key : 0xFFFFFFFFu;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = min(m, (unsigned)__shfl_xor((int)m, off));
    if (lane == leader && m != 0xFFFFFFFFu) atomicMin(zmin_bits + ln, m);
    pending &= ~__ballot(mine);
  }
}

struct Bary {
  float b0, b1, b2, pz;
  bool inside;
};

__device__ __forceinline__ Bary bary_at(float px, float py, const float* p0, const float* p1,
                                        const float* p2) {
#pragma clang fp contract(off)
  Bary r;
  const float area0 = (p2[0] - p0[0]) * (p1[1] - p0[1]) - (p2[1] - p0[1]) * (p1[0] - p0[0]);
  const float area = area0 + K_EPS;
  const float w0 = ((px - p1[0]) * (p2[1] - p1[1]) - (py - p1[1]) * (p2[0] - p1[0])) / area;
  const float w1 = ((px - p2[0]) * (p0[1] - p2[1]) - (py - p2[1]) * (p0[0] - p2[0])) / area;
  const float w2 = ((px - p0[0]) * (p1[1] - p0[1]) - (py - p0[1]) * (p1[0] - p0[0])) / area;
  const float t0 = w0 * p1[2] * p2[2], t1 = p0[2] * w1 * p2[2], t2 = p0[2] * p1[2] * w2;
  const float den = fmaxf(t0 + t1 + t2, K_EPS);
  r.b0 = t0 / den;
  r.b1 = t1 / den;
  r.b2 = t2 / den;
  r.pz = r.b0 * p0[2] + r.b1 * p1[2] + r.b2 * p2[2];
  r.inside = r.b0 > 0.f && r.b1 > 0.f && r.b2 > 0.f && r.pz >= 0.f && fabsf(area0) > K_EPS;
  return r;
}

// the pixel range (margined, clamped screen bbox) a face is tested on; false when culled
// (entirely behind the camera) or off-screen
__device__ __forceinline__ bool face_bbox(const float* p0, const float* p1, const float* p2, int S,
                                          int* c_lo, int* c_hi, int* r_lo, int* r_hi) {
  if (p0[2] <= 0.f && p1[2] <= 0.f && p2[2] <= 0.f) return false;  // entirely behind the camera
  const float xmin = fminf(p0[0], fminf(p1[0], p2[0])), xmax = fmaxf(p0[0], fmaxf(p1[0], p2[0]));
  const float ymin = fminf(p0[1], fminf(p1[1], p2[1])), ymax = fmaxf(p0[1], fmaxf(p1[1], p2[1]));
  // pixel c samples x = 1 − (2c+1)/S  ⇒  c = ((1 − x)·S − 1)/2 (one pixel of margin)
  *c_lo = max((int)floorf(((1.f - xmax) * S - 1.f) * 0.5f) - 1, 0);
  *c_hi = min((int)ceilf(((1.f - xmin) * S - 1.f) * 0.5f) + 1, S - 1);
  *r_lo = max((int)floorf(((1.f - ymax) * S - 1.f) * 0.5f) - 1, 0);
  *r_hi = min((int)ceilf(((1.f - ymin) * S - 1.f) * 0.5f) + 1, S - 1);
  return *c_lo <= *c_hi && *r_lo <= *r_hi;
}

// Screen-binned rasterisation: workgroup = one 16×16 pixel tile of one image, thread = pixel.
// The image's faces (a contiguous range of the non-decreasing face_img, found by binary search)
// are walked 256 at a time: each thread sets up one face (bbox), the faces whose bbox meets the
// tile are compacted into LDS (index, projected vertices, bbox), then every pixel tests those
// against its centre with the same bbox and barycentric rules as a per-face rasteriser and keeps
// the minimum (depth bits << 32 | face) key — nearest face, ties to the lower index, independent
// of order — written once per pixel: no global atomics and no z-buffer clear.
constexpr int RT = 16;

__device__ __forceinline__ int lower_bound_i(const int* __restrict__ v, int n, int key) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (v[mid] < key) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__global__ __launch_bounds__(256) void render_tile_kernel(scflow_render_args a,
                                                          const int* __restrict__ face_img,
                                                          const float* __restrict__ vproj,
                                                          unsigned long long* __restrict__ zf) {
  __shared__ int range[2];
  __shared__ int cnt;
  __shared__ int lf[256];
  __shared__ int lbox[256][4];
  __shared__ float lv[256][9];
  const int S = a.size;
  const int tiles_x = (S + RT - 1) / RT;
  const int n = blockIdx.y;
  const int tx0 = (blockIdx.x % tiles_x) * RT, ty0 = (blockIdx.x / tiles_x) * RT;
  if (threadIdx.x < 2) range[threadIdx.x] = lower_bound_i(face_img, a.total_faces, n + (int)threadIdx.x);
  const int r = ty0 + (int)threadIdx.x / RT, c = tx0 + (int)threadIdx.x % RT;
  const float px = 1.f - (float)(2 * c + 1) / (float)S;
  const float py = 1.f - (float)(2 * r + 1) / (float)S;
  unsigned long long best = ~0ull;
  __syncthreads();
  const int fb = range[0], fe = range[1];
  for (int f0 = fb; f0 < fe; f0 += 256) {
    if (threadIdx.x == 0) cnt = 0;
    __syncthreads();
    const int f = f0 + (int)threadIdx.x;
    if (f < fe) {
      const float* p0 = vproj + 3 * a.faces[3 * f];
      const float* p1 = vproj + 3 * a.faces[3 * f + 1];
      const float* p2 = vproj + 3 * a.faces[3 * f + 2];
      int cl, ch, rl, rh;
      if (face_bbox(p0, p1, p2, S, &cl, &ch, &rl, &rh) && ch >= tx0 && cl < tx0 + RT &&
          rh >= ty0 && rl < ty0 + RT) {
        const int k = atomicAdd(&cnt, 1);  // LDS counter: the order does not matter (min key)
        lf[k] = f;
        lbox[k][0] = cl, lbox[k][1] = ch, lbox[k][2] = rl, lbox[k][3] = rh;
#pragma unroll
        for (int e = 0; e < 3; ++e) {
          lv[k][e] = p0[e];
          lv[k][3 + e] = p1[e];
          lv[k][6 + e] = p2[e];
        }
      }
    }
    __syncthreads();
    const int m = cnt;
    for (int k = 0; k < m; ++k) {
      if (c < lbox[k][0] || c > lbox[k][1] || r < lbox[k][2] || r > lbox[k][3]) continue;
      const Bary b = bary_at(px, py, &lv[k][0], &lv[k][3], &lv[k][6]);
      if (!b.inside) continue;
      const unsigned long long key = ((unsigned long long)__float_as_uint(b.pz) << 32) | (unsigned)lf[k];
      best = key < best ? key : best;
    }
    __syncthreads();  // the list is rebuilt for the next 256 faces
  }
  if (r < S && c < S) zf[((size_t)n * S + r) * S + c] = best;
}

__device__ __forceinline__ void normalize3(float* v, float eps = 1e-6f) {
  const float n = fmaxf(sqrtf(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]), eps);
  v[0] /= n;
  v[1] /= n;
  v[2] /= n;
}

// light location (object frame) of image n, Renderer.forward :209-230
__device__ __forceinline__ void light_of(const scflow_render_args& a, int n,
                                         const unsigned* __restrict__ zmin_bits, int n_img,
                                         float (&L)[3]) {
  if (a.light_mode == SCFLOW_LIGHT_FIXED) {
    L[0] = a.light_location[0];
    L[1] = a.light_location[1];
    L[2] = a.light_location[2];
    return;
  }
  float lz;
  if (a.light_mode == SCFLOW_LIGHT_PER_IMAGE) {
    lz = fmaxf(__uint_as_float(zmin_bits[n]) - 400.f, 0.f);
  } else {  // SCFLOW_LIGHT_BATCH_ZNEAR: znear = (min over the batch // 100)·100, light at znear/4
    float zn = __uint_as_float(zmin_bits[0]);
    for (int k = 1; k < n_img; ++k) zn = fminf(zn, __uint_as_float(zmin_bits[k]));
    lz = floorf(zn / 100.f) * 100.f / 4.f;
  }
  const float* R = a.R + 9 * n;
  L[0] = R[2] * lz;
  L[1] = R[5] * lz;
  L[2] = R[8] * lz;
}

__global__ void render_shade_kernel(scflow_render_args a, const float* __restrict__ vproj,
                                    const unsigned long long* __restrict__ zf,
                                    const unsigned* __restrict__ zmin_bits, int n_img) {
  const int S = a.size;
  const long long pix = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (pix >= (long long)n_img * S * S) return;
  const int n = (int)(pix / ((long long)S * S));
  const int rc = (int)(pix % ((long long)S * S));
  const int r = rc / S, c = rc % S;
  const unsigned long long key = zf[pix];
  float* img = a.images ? a.images + pix * 4 : nullptr;
  if (a.light_out && rc == 0) {  // the image's light location, once per image
    float L[3];
    light_of(a, n, zmin_bits, n_img, L);
    for (int k = 0; k < 3; ++k) a.light_out[3 * n + k] = L[k];
  }
  if (key == ~0ull) {
    if (a.zbuf) a.zbuf[pix] = -1.f;
    if (a.pix_to_face) a.pix_to_face[pix] = -1;
    if (a.bary) a.bary[3 * pix] = a.bary[3 * pix + 1] = a.bary[3 * pix + 2] = -1.f;
    if (img) {
      img[0] = a.background[0];
      img[1] = a.background[1];
      img[2] = a.background[2];
      img[3] = 0.f;
    }
    return;
  }
  const int f = (int)(key & 0xffffffffull);
  const int i0 = a.faces[3 * f], i1 = a.faces[3 * f + 1], i2 = a.faces[3 * f + 2];
  const float px = 1.f - (float)(2 * c + 1) / (float)S;
  const float py = 1.f - (float)(2 * r + 1) / (float)S;
  const Bary b = bary_at(px, py, vproj + 3 * i0, vproj + 3 * i1, vproj + 3 * i2);
  if (a.zbuf) a.zbuf[pix] = b.pz;
  if (a.pix_to_face) a.pix_to_face[pix] = f;
  if (a.bary) {
    a.bary[3 * pix] = b.b0;
    a.bary[3 * pix + 1] = b.b1;
    a.bary[3 * pix + 2] = b.b2;
  }
  if (!img) return;
  float P[3], N[3], T[3];
  for (int k = 0; k < 3; ++k) {
    P[k] = b.b0 * a.verts[3 * i0 + k] + b.b1 * a.verts[3 * i1 + k] + b.b2 * a.verts[3 * i2 + k];
    N[k] = b.b0 * a.normals[3 * i0 + k] + b.b1 * a.normals[3 * i1 + k] + b.b2 * a.normals[3 * i2 + k];
    T[k] = b.b0 * a.colors[3 * i0 + k] + b.b1 * a.colors[3 * i1 + k] + b.b2 * a.colors[3 * i2 + k];
  }
  const float* R = a.R + 9 * n;
  const float* t = a.t + 3 * n;
  float L[3];
  light_of(a, n, zmin_bits, n_img, L);
  // camera centre −Rᵀt
  const float C[3] = {-(R[0] * t[0] + R[3] * t[1] + R[6] * t[2]), -(R[1] * t[0] + R[4] * t[1] + R[7] * t[2]),
                      -(R[2] * t[0] + R[5] * t[1] + R[8] * t[2])};
  float D[3] = {L[0] - P[0], L[1] - P[1], L[2] - P[2]};
  float V[3] = {C[0] - P[0], C[1] - P[1], C[2] - P[2]};
  normalize3(N);
  normalize3(D);
  normalize3(V);
  const float cosv = N[0] * D[0] + N[1] * D[1] + N[2] * D[2];
  const float dif = fmaxf(cosv, 0.f);
  float Rf[3];
  for (int k = 0; k < 3; ++k) Rf[k] = -D[k] + 2.f * (cosv * N[k]);
  const float sa = cosv > 0.f ? fmaxf(V[0] * Rf[0] + V[1] * Rf[1] + V[2] * Rf[2], 0.f) : 0.f;
  const float spec = powf(sa, a.shininess);
  for (int k = 0; k < 3; ++k)
    img[k] = (a.ambient[k] + a.diffuse[k] * dif) * T[k] + a.specular[k] * spec;
  img[3] = 1.f;
}

}  // namespace

SCFLOW_API long long scflow_render_workspace(int n_img, int size, int total_verts) {
  // z-buffer keys (8 B/pixel) + projected vertices + per-image min depth
  return (long long)n_img * size * size * 8 + (long long)total_verts * 12 + (long long)n_img * 4 + 64;
}

SCFLOW_API int scflow_render(const scflow_render_args* args, void* stream) {
  if (!args) return SCFLOW_EINVAL;
  const scflow_render_args& a = *args;
  if (!a.verts || !a.faces || !a.vert_img || !a.face_img || !a.R || !a.t || !a.K ||
      !a.workspace || a.n_img <= 0 || a.size <= 0 || a.total_verts <= 0 || a.total_faces < 0)
    return SCFLOW_EINVAL;
  if (a.images && (!a.normals || !a.colors || !a.background || !a.ambient || !a.diffuse ||
                   !a.specular))
    return SCFLOW_EINVAL;
  if (a.light_mode < 0 || a.light_mode > 2 || (a.light_mode == SCFLOW_LIGHT_FIXED && !a.light_location))
    return SCFLOW_EINVAL;
  if (a.workspace_bytes < scflow_render_workspace(a.n_img, a.size, a.total_verts)) return SCFLOW_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  const size_t npix = (size_t)a.n_img * a.size * a.size;
  unsigned long long* zf = (unsigned long long*)a.workspace;
  float* vproj = (float*)(zf + npix);
  unsigned* zmin = (unsigned*)(vproj + 3 * (size_t)a.total_verts);
  hipError_t e = hipMemsetAsync(zmin, 0x7f, (size_t)a.n_img * 4, st);  // +large float
  if (e != hipSuccess) return (int)e;
  render_project_kernel<<<(a.total_verts + 255) / 256, 256, 0, st>>>(a, a.vert_img, vproj, zmin,
                                                                      a.total_verts);
  const int tiles = ((a.size + RT - 1) / RT) * ((a.size + RT - 1) / RT);
  render_tile_kernel<<<dim3(tiles, a.n_img), 256, 0, st>>>(a, a.face_img, vproj, zf);
  render_shade_kernel<<<(unsigned)((npix + 255) / 256), 256, 0, st>>>(a, vproj, zf, zmin, a.n_img);
  return scflow_launch_status();
}
