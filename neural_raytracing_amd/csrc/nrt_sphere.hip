// The analytic Sphere shape (shapes/shapes.py:11-97): quad_solve's ray / sphere roots per ray,
// one thread per ray, the hit list appended wave by wave.  The pathtracer's only non-SDF shape
// with a hot path: utils.sphere_examples / sphere_render_bsdf (utils.py:389-431) render every
// BSDF basis on it (scripts/visualize.py, dtu_vis.py, nerv_vis.py).  Per-ray VALU work and 6
// floats in / ~8 floats out per ray: HBM-bound, ~70 B a ray.
#include "nrt_launch.h"

namespace nrt {

// shapes.py:47-69 in the reference's float32 op order: fs = o - c; a = sum(d d); b = 2 sum(d fs);
// c = sum(fs fs) - r^2 (each sum ((x + y) + z)); quad_solve: disc = b b - (4 a) c, valid = disc >
// 0, sqrt only where valid (the reference keeps disc itself elsewhere), roots (-b +- disc') / (2 a);
// hit = valid && either root >= EPS; roots < EPS -> inf; t = min (upper = max, intersect_limits);
// p = o + t d, n = normalize(p - c) (F.normalize, eps 1e-12), p += 1e-5 n.  Misses keep the
// reference's values (t from the unsquared disc, p / n from that t).
template <int = 0>
__global__ void k_sphere_intersect(float cx, float cy, float cz, float sqr_r,
                                   const float* __restrict__ rays, int64_t P,
                                   float* __restrict__ t_out, uint8_t* __restrict__ hit_out,
                                   float* __restrict__ p_out, float* __restrict__ n_out,
                                   float* __restrict__ upper, int32_t* __restrict__ hit_idx,
                                   int32_t* __restrict__ hit_count) {
  constexpr float EPS = 1e-8f;
  const int lane = lane_id();
  for (int64_t ray = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; ray - lane < P;
       ray += (int64_t)gridDim.x * blockDim.x) {
    const bool live = ray < P;
    bool hit = false;
    if (live) {
      const float* r = rays + ray * 6;
      const float ox = r[0], oy = r[1], oz = r[2], dx = r[3], dy = r[4], dz = r[5];
      const float fx = ox - cx, fy = oy - cy, fz = oz - cz;
      const float a = (dx * dx + dy * dy) + dz * dz;
      const float b = 2.f * ((dx * fx + dy * fy) + dz * fz);
      const float c = ((fx * fx + fy * fy) + fz * fz) - sqr_r;
      float disc = b * b - (4.f * a) * c;
      const bool valid = disc > 0.f;
      if (valid) disc = sqrtf(disc);
      const float a2 = 2.f * a;
      float t0 = (-b + disc) / a2, t1 = (-b + (-disc)) / a2;
      hit = valid && (t0 >= EPS || t1 >= EPS);
      if (t0 < EPS) t0 = __builtin_inff();
      if (t1 < EPS) t1 = __builtin_inff();
      // torch.min / max propagate NaN (a zero direction)
      const bool nan = t0 != t0 || t1 != t1;
      const float t = nan ? __builtin_nanf("") : fminf(t0, t1);
      if (upper) upper[ray] = nan ? __builtin_nanf("") : fmaxf(t0, t1);
      if (t_out) t_out[ray] = t;
      if (hit_out) hit_out[ray] = hit ? 1 : 0;
      if (p_out) {
        float px = ox + t * dx, py = oy + t * dy, pz = oz + t * dz;
        float nx = px - cx, ny = py - cy, nz = pz - cz;
        normalize3(nx, ny, nz, 1e-12f);
        p_out[ray * 3] = px + nx * 1e-5f;
        p_out[ray * 3 + 1] = py + ny * 1e-5f;
        p_out[ray * 3 + 2] = pz + nz * 1e-5f;
        if (n_out) { n_out[ray * 3] = nx; n_out[ray * 3 + 1] = ny; n_out[ray * 3 + 2] = nz; }
      }
    }
    if (hit_idx) {
      const uint64_t mk = __ballot(hit);
      const int cnt = __popcll(mk);
      int base = 0;
      if (lane == 0 && cnt) base = atomicAdd(hit_count, cnt);
      base = __shfl(base, 0);
      if (hit) hit_idx[base + __popcll(mk & ((1ull << lane) - 1ull))] = (int32_t)ray;
    }
  }
}

// SphereCloud (shapes.py:99-206): the nearest hit over N spheres, one thread per ray, the sphere
// table (cx, cy, cz, r) read through the scalar cache.  Per sphere the Sphere kernel's float32
// quad_solve (radius^2 as r * r in f32, :138), a root counts when it lies in [EPS, t_max), roots
// < EPS become inf and a sphere without a counting root gives inf; per chunk of split_n spheres
// (:122-123) torch.min's first minimum (the sphere index WITHIN the chunk, as the reference keeps
// it, :162-167), which replaces the best distance (t_max at start) when the chunk had a hit and is
// strictly nearer.  p = o + t d; n = normalize(p - centers[face]) on hits, 0 elsewhere; p += 1e-5 n.
// The reference's broadcasting is well-formed for N = 1 (oracle SphereCloudRef): there the
// results are the reference's bit for bit; N > 1 follows the same per-ray statements.
template <int = 0>
__global__ void k_sphere_cloud(const float4* __restrict__ spheres, int N, int split_n, float t_max,
                               const float* __restrict__ rays, int64_t P,
                               float* __restrict__ t_out, uint8_t* __restrict__ hit_out,
                               float* __restrict__ p_out, float* __restrict__ n_out,
                               int32_t* __restrict__ hit_idx, int32_t* __restrict__ hit_count) {
  constexpr float EPS = 1e-8f;
  const float inf = __builtin_inff();
  const int lane = lane_id();
  for (int64_t ray = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; ray - lane < P;
       ray += (int64_t)gridDim.x * blockDim.x) {
    const bool live = ray < P;
    bool active = false;
    if (live) {
      const float* r = rays + ray * 6;
      const float ox = r[0], oy = r[1], oz = r[2], dx = r[3], dy = r[4], dz = r[5];
      const float a = (dx * dx + dy * dy) + dz * dz;
      const float a2 = 2.f * a, a4 = 4.f * a;
      float best = t_max;
      int face = -1;
      for (int j0 = 0; j0 < N; j0 += split_n) {
        const int j1 = j0 + split_n < N ? j0 + split_n : N;
        float mt = inf;
        int mi = 0;
        bool any = false;
        for (int j = j0; j < j1; ++j) {
          const float4 sp = spheres[j];
          const float fx = ox - sp.x, fy = oy - sp.y, fz = oz - sp.z;
          const float b = 2.f * ((dx * fx + dy * fy) + dz * fz);
          const float c = ((fx * fx + fy * fy) + fz * fz) - sp.w * sp.w;
          float disc = b * b - a4 * c;
          const bool valid = disc > 0.f;
          if (valid) disc = sqrtf(disc);
          float t0 = (-b + disc) / a2, t1 = (-b + (-disc)) / a2;
          const bool mask = valid && ((t0 >= EPS && t0 < t_max) || (t1 >= EPS && t1 < t_max));
          if (t0 < EPS) t0 = inf;
          if (t1 < EPS) t1 = inf;
          const float tj = mask ? fminf(t0, t1) : inf;
          any = any || mask;
          if (tj < mt) { mt = tj; mi = j - j0; }
        }
        active = active || any;
        if (any && best > mt) { best = mt; face = mi; }
      }
      float px = ox + best * dx, py = oy + best * dy, pz = oz + best * dz;
      float nx = 0.f, ny = 0.f, nz = 0.f;
      if (active && face >= 0) {
        const float4 cf = spheres[face];
        nx = px - cf.x; ny = py - cf.y; nz = pz - cf.z;
        normalize3(nx, ny, nz, 1e-12f);
      }
      if (t_out) t_out[ray] = best;
      if (hit_out) hit_out[ray] = active ? 1 : 0;
      if (p_out) {
        p_out[ray * 3] = px + nx * 1e-5f;
        p_out[ray * 3 + 1] = py + ny * 1e-5f;
        p_out[ray * 3 + 2] = pz + nz * 1e-5f;
        if (n_out) { n_out[ray * 3] = nx; n_out[ray * 3 + 1] = ny; n_out[ray * 3 + 2] = nz; }
      }
    }
    if (hit_idx) {
      const uint64_t mk = __ballot(active);
      const int cnt = __popcll(mk);
      int base = 0;
      if (lane == 0 && cnt) base = atomicAdd(hit_count, cnt);
      base = __shfl(base, 0);
      if (active) hit_idx[base + __popcll(mk & ((1ull << lane) - 1ull))] = (int32_t)ray;
    }
  }
}

}  // namespace nrt

using namespace nrt;

extern "C" {

int nrt_sphere_intersect(const float* center, double radius, const float* rays, int64_t P,
                         float* t, uint8_t* hit, float* p, float* n, float* upper,
                         int32_t* hit_idx, int32_t* hit_count, void* stream) {
  if (!center || P < 0 || (P > 0 && !rays) || (n && !p) || (hit_idx && !hit_count) ||
      !std::isfinite(radius)) {
    set_error("nrt_sphere_intersect: bad argument");
    return NRT_EINVAL;
  }
  hipStream_t st = (hipStream_t)stream;
  if (hit_count) NRT_HIP(hipMemsetAsync(hit_count, 0, sizeof(int32_t), st));
  if (P == 0) return NRT_OK;
  // sqr_radius is the python float radius * radius (double); the tensor op rounds it to f32
  const float sqr_r = (float)(radius * radius);
  const int64_t blocks = std::min<int64_t>(ceil_div64(P, 256), 4096);
  ProfScope prof("k_sphere_intersect", st);
  k_sphere_intersect<><<<dim3((unsigned)blocks), dim3(256), 0, st>>>(
      center[0], center[1], center[2], sqr_r, rays, P, t, hit, p, n, upper, hit_idx, hit_count);
  return check_launch("k_sphere_intersect");
}

int nrt_sphere_cloud_intersect(const float* spheres, int64_t N, int64_t split_n, double t_max,
                               const float* rays, int64_t P, float* t, uint8_t* hit, float* p,
                               float* n, int32_t* hit_idx, int32_t* hit_count, void* stream) {
  if (N < 1 || !spheres || split_n < 1 || P < 0 || (P > 0 && !rays) || (n && !p) ||
      (hit_idx && !hit_count) || N > INT32_MAX || std::isnan(t_max)) {
    set_error("nrt_sphere_cloud_intersect: bad argument");
    return NRT_EINVAL;
  }
  hipStream_t st = (hipStream_t)stream;
  if (hit_count) NRT_HIP(hipMemsetAsync(hit_count, 0, sizeof(int32_t), st));
  if (P == 0) return NRT_OK;
  // t_max: the python float, compared with float32 tensors (and the best-distance fill) as f32
  const float tm = (float)t_max;
  const int64_t blocks = std::min<int64_t>(ceil_div64(P, 256), 4096);
  ProfScope prof("k_sphere_cloud", st);
  k_sphere_cloud<><<<dim3((unsigned)blocks), dim3(256), 0, st>>>(
      reinterpret_cast<const float4*>(spheres), (int)N, (int)std::min<int64_t>(split_n, INT32_MAX),
      tm, rays, P, t, hit, p, n, hit_idx, hit_count);
  return check_launch("k_sphere_cloud");
}

}  // extern "C"
