// Sphere tracing, coarse scan and shadow test for SDF callables the library cannot pack (a warp
// such as edit_dtu.py:86-97's `bend`, a displacement add-on, any user function of p): the
// callable is evaluated by the caller between steps, these kernels do everything else of
// sdfs.py:111-181 -- the march state (depth, remaining, hit), the scan's running min / argmin,
// the shadow march's visibility -- and write the next query points.  One elementwise launch per
// step, rays in ray order: HBM-bound, coalesced, 32-60 bytes per ray per step.
//
// Query points follow torch's elementwise rounding: r_o + r_d * depth (one multiply, one add,
// sdfs.py:121/158/170), scan point j: r_o + (float)(step * j) * r_d (python float product,
// sdfs.py:243-244), best_pos: r_o + ((float)idx * (float)step) * r_d (sdfs.py:248).
#include "nrt_launch.h"

namespace nrt {
namespace {

__device__ __forceinline__ void put_point(const float* __restrict__ ray, float s, float* __restrict__ q) {
  q[0] = __fadd_rn(ray[0], __fmul_rn(ray[3], s));
  q[1] = __fadd_rn(ray[1], __fmul_rn(ray[4], s));
  q[2] = __fadd_rn(ray[2], __fmul_rn(ray[5], s));
}

// sdfs.py:118-131, one loop iteration split at the SDF call: consume the distances of the step
// just evaluated (dists == nullptr: initialise), then (prep) the next step's remaining test and
// query points; without prep q gets the final p = r_o + depth r_d (sdfs.py:133)
__global__ void k_march_step(const float* __restrict__ rays, int64_t P, const float* __restrict__ dists,
                             float eps, float max_t, int prep, float* __restrict__ t,
                             uint8_t* __restrict__ remaining, uint8_t* __restrict__ hit,
                             float* __restrict__ q) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P) return;
  float depth = 0.f;
  bool rem = true, act = false;
  if (dists) {
    depth = t[i];
    rem = remaining[i] != 0;
    act = hit[i] != 0;
    const float d = dists[i];
    const bool h = rem && d <= eps;
    act = act || h;
    rem = rem && !h;
    if (rem) depth = depth + d;
  }
  if (prep) rem = rem && depth < max_t;
  t[i] = depth;
  remaining[i] = rem ? 1 : 0;
  hit[i] = act ? 1 : 0;
  put_point(rays + i * 6, depth, q + i * 3);
}

// SDF.throughput's loop (sdfs.py:238-247): sd = sdf(scan point j); j = 0 initialises
// (curr_min = sd(r_o), idx = 0), j >= 1 keeps the first strict minimum (where(sd < m, j, idx),
// torch.minimum propagating NaN).  prep = 1 writes scan point j + 1, prep = 2 best_pos.
__global__ void k_scan_step(const float* __restrict__ rays, int64_t P, const float* __restrict__ sd,
                            int j, double step, int prep, float* __restrict__ curr_min,
                            int32_t* __restrict__ idx, float* __restrict__ q) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P) return;
  const float v = sd[i];
  float m;
  int k;
  if (j == 0) {
    m = v;
    k = 0;
  } else {
    m = curr_min[i];
    k = idx[i];
    if (v < m) k = j;
    m = (isnan(v) || isnan(m)) ? __int_as_float(0x7fc00000) : fminf(m, v);
  }
  curr_min[i] = m;
  idx[i] = k;
  if (prep == 1) put_point(rays + i * 6, (float)(step * (double)(j + 1)), q + i * 3);
  else if (prep == 2) put_point(rays + i * 6, __fmul_rn((float)k, (float)step), q + i * 3);
}

// SDF.intersect_test (sdfs.py:162-181): depth starts at t0 = 1e2 * eps (the python product, rounded
// to f32 by the caller); every step adds the distance of a
// remaining ray (the hit step included) and a distance < eps retires it.  phase 0 initialises,
// 1 consumes a step, 2 consumes the last step and writes visible = depth >= max_t | remaining.
__global__ void k_occlusion_step(const float* __restrict__ rays, int64_t P, const float* __restrict__ dists,
                                 float eps, float t0, const float* __restrict__ max_t, int phase,
                                 float* __restrict__ depth, uint8_t* __restrict__ remaining,
                                 float* __restrict__ q, uint8_t* __restrict__ visible) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P) return;
  float t;
  bool rem;
  if (phase == 0) {
    t = t0;
    rem = true;
  } else {
    t = depth[i];
    rem = remaining[i] != 0;
    const float d = dists[i];
    const bool h = rem && d < eps;
    if (rem) t = t + d;
    rem = rem && !h;
  }
  depth[i] = t;
  remaining[i] = rem ? 1 : 0;
  if (phase == 2) visible[i] = (t >= max_t[i] || rem) ? 1 : 0;
  else put_point(rays + i * 6, t, q + i * 3);
}

}  // namespace
}  // namespace nrt

using namespace nrt;

extern "C" {

int nrt_march_callable_step(const float* rays, int64_t P, const float* dists, float eps,
                            float max_t, int prep, float* t, uint8_t* remaining, uint8_t* hit,
                            float* q, void* stream) {
  if (P < 0 || !rays || !t || !remaining || !hit || !q) {
    set_error("nrt_march_callable_step: bad argument");
    return NRT_EINVAL;
  }
  if (P == 0) return NRT_OK;
  ProfScope prof("k_march_step", (hipStream_t)stream);
  k_march_step<<<dim3(ceil_div64(P, 256)), dim3(256), 0, (hipStream_t)stream>>>(
      rays, P, dists, eps, max_t, prep, t, remaining, hit, q);
  return check_launch("k_march_step");
}

int nrt_scan_callable_step(const float* rays, int64_t P, const float* sd, int32_t j, double step,
                           int prep, float* curr_min, int32_t* idx, float* q, void* stream) {
  if (P < 0 || !rays || !sd || !curr_min || !idx || (prep && !q) || j < 0 || prep < 0 || prep > 2) {
    set_error("nrt_scan_callable_step: bad argument");
    return NRT_EINVAL;
  }
  if (P == 0) return NRT_OK;
  ProfScope prof("k_scan_step", (hipStream_t)stream);
  k_scan_step<<<dim3(ceil_div64(P, 256)), dim3(256), 0, (hipStream_t)stream>>>(
      rays, P, sd, j, step, prep, curr_min, idx, q);
  return check_launch("k_scan_step");
}

int nrt_occlusion_callable_step(const float* rays, int64_t P, const float* dists, float eps,
                                float t0, const float* max_t, int phase, float* depth, uint8_t* remaining,
                                float* q, uint8_t* visible, void* stream) {
  if (P < 0 || !rays || !depth || !remaining || phase < 0 || phase > 2 ||
      (phase > 0 && !dists) || (phase < 2 && !q) || (phase == 2 && (!max_t || !visible))) {
    set_error("nrt_occlusion_callable_step: bad argument");
    return NRT_EINVAL;
  }
  if (P == 0) return NRT_OK;
  ProfScope prof("k_occlusion_step", (hipStream_t)stream);
  k_occlusion_step<<<dim3(ceil_div64(P, 256)), dim3(256), 0, (hipStream_t)stream>>>(
      rays, P, dists, eps, t0, max_t, phase, depth, remaining, q, visible);
  return check_launch("k_occlusion_step");
}

}  // extern "C"
