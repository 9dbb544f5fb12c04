// SphereSDF's smooth-min part under autograd (training): the value
//   v(p) = -log(max(sum_i exp(-k sd_i), 1e-4)) / k,   sd_i = |q_i| - R_i,   q_i = (I + tfs_i) p - c_i
// (sdfs.py:37-43, utils.py:386-387, k = 32) and its gradient g(p) = dv/dp (the normal's sphere
// part, SDF.autograd_diff with create_graph=True, sdfs.py:184-197), and the backward of both with
// respect to the sphere parameters -- for g that is the double backward the eikonal / shading
// losses need.  The torch restatement (differentiable.sphere_part under autograd.grad) runs ~40
// tensor ops over [n, P, 3] per training step; this is three launches.
//
// With alpha_i = w_i / S (w_i = exp(-k sd_i), S unclamped), u_i = q_i / |q_i|, T_i = I + tfs_i:
//   g = sum_i alpha_i T_i^T u_i,  dv / dsd_i = alpha_i.
// For J = sum_points (dv v + dg . g):
//   beta_i = (T_i dg) . u_i,  gamma = sum_j alpha_j beta_j,  kappa_i = -k alpha_i (beta_i - gamma),
//   c_i = dv alpha_i + kappa_i,  m_i = T_i dg,  mp_i = (m_i - (u_i . m_i) u_i) / |q_i|,
//   e_i = c_i u_i + alpha_i mp_i:
//   dR_i = -c_i,  dc_i = -e_i,  dT_i = e_i p^T + alpha_i u_i dg^T   (dtfs_i = dT_i).
// A clamped point (S < 1e-4) has constant v and g = 0 and contributes nothing (torch's clamp
// passes no gradient below its bound).
#include "nrt_launch.h"

namespace nrt {
namespace {

constexpr int kSphF = 13;  // T (9, row-major), c (3), R
constexpr int kSmBlock = 256;
constexpr int kMaxSpheres = 64 * 1024 / (kSphF * 4);  // the LDS table's capacity (1,260)
constexpr int64_t kSliceMin = 4096;                    // points per backward slice at least
constexpr int kMaxSlices = 32;

// point slices of the sphere-parameter backward: the grid is spheres x slices, each block sums
// its slice, k_smoothmin_reduce adds the slices in order (deterministic)
int bwd_slices(int64_t P) {
  return (int)std::max<int64_t>(1, std::min<int64_t>(kMaxSlices, (P + kSliceMin - 1) / kSliceMin));
}

// sphere table into LDS: [n][13]
__device__ __forceinline__ void stage_spheres(float* ls, const float* __restrict__ centers,
                                              const float* __restrict__ radii,
                                              const float* __restrict__ tfs, int n) {
  for (int q = threadIdx.x; q < n * kSphF; q += blockDim.x) {
    const int i = q / kSphF, f = q % kSphF;
    float v;
    if (f < 9) v = tfs[i * 9 + f] + ((f == 0 || f == 4 || f == 8) ? 1.f : 0.f);
    else if (f < 12) v = centers[i * 3 + (f - 9)];
    else v = radii[i];
    ls[q] = v;
  }
  __syncthreads();
}

struct SphereTerm {
  float q[3], r, sd;
};
__device__ __forceinline__ SphereTerm sphere_term(const float* s, float x, float y, float z) {
  SphereTerm t;
  t.q[0] = fmaf(s[2], z, fmaf(s[1], y, s[0] * x)) - s[9];
  t.q[1] = fmaf(s[5], z, fmaf(s[4], y, s[3] * x)) - s[10];
  t.q[2] = fmaf(s[8], z, fmaf(s[7], y, s[6] * x)) - s[11];
  t.r = sqrtf(fmaf(t.q[2], t.q[2], fmaf(t.q[1], t.q[1], t.q[0] * t.q[0])));
  t.sd = t.r - s[12];
  return t;
}

// value [P] and gradient [P, 3] (either may be null)
__global__ void __launch_bounds__(kSmBlock) k_smoothmin_fwd(
    const float* __restrict__ p, int64_t P, const float* __restrict__ centers,
    const float* __restrict__ radii, const float* __restrict__ tfs, int n, float k,
    float* __restrict__ value, float* __restrict__ grad) {
  extern __shared__ float ls[];
  stage_spheres(ls, centers, radii, tfs, n);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < P;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float x = p[i * 3], y = p[i * 3 + 1], z = p[i * 3 + 2];
    float S = 0.f, g0 = 0.f, g1 = 0.f, g2 = 0.f;
    for (int j = 0; j < n; ++j) {
      const float* s = ls + j * kSphF;
      const SphereTerm t = sphere_term(s, x, y, z);
      const float w = expf(-k * t.sd);
      S += w;
      if (t.r > 0.f) {
        const float a = w / t.r;  // w u_i, then T^T
        g0 = fmaf(a, fmaf(s[6], t.q[2], fmaf(s[3], t.q[1], s[0] * t.q[0])), g0);
        g1 = fmaf(a, fmaf(s[7], t.q[2], fmaf(s[4], t.q[1], s[1] * t.q[0])), g1);
        g2 = fmaf(a, fmaf(s[8], t.q[2], fmaf(s[5], t.q[1], s[2] * t.q[0])), g2);
      }
    }
    const bool live = S >= 1e-4f;
    if (value) value[i] = -logf(live ? S : 1e-4f) / k;
    if (grad) {
      const float inv = live ? 1.f / S : 0.f;
      grad[i * 3] = g0 * inv;
      grad[i * 3 + 1] = g1 * inv;
      grad[i * 3 + 2] = g2 * inv;
    }
  }
}

// per point: (1/S or 0 when clamped, gamma = sum_j alpha_j beta_j)
__global__ void __launch_bounds__(kSmBlock) k_smoothmin_pre(
    const float* __restrict__ p, int64_t P, const float* __restrict__ centers,
    const float* __restrict__ radii, const float* __restrict__ tfs, int n, float k,
    const float* __restrict__ dgrad, float2* __restrict__ pre) {
  extern __shared__ float ls[];
  stage_spheres(ls, centers, radii, tfs, n);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < P;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float x = p[i * 3], y = p[i * 3 + 1], z = p[i * 3 + 2];
    const float v0 = dgrad ? dgrad[i * 3] : 0.f, v1 = dgrad ? dgrad[i * 3 + 1] : 0.f,
                v2 = dgrad ? dgrad[i * 3 + 2] : 0.f;
    float S = 0.f, wb = 0.f;
    for (int j = 0; j < n; ++j) {
      const float* s = ls + j * kSphF;
      const SphereTerm t = sphere_term(s, x, y, z);
      const float w = expf(-k * t.sd);
      S += w;
      if (dgrad && t.r > 0.f) {  // beta_j = (T_j v) . u_j
        const float m0 = fmaf(s[2], v2, fmaf(s[1], v1, s[0] * v0));
        const float m1 = fmaf(s[5], v2, fmaf(s[4], v1, s[3] * v0));
        const float m2 = fmaf(s[8], v2, fmaf(s[7], v1, s[6] * v0));
        wb = fmaf(w, fmaf(m2, t.q[2], fmaf(m1, t.q[1], m0 * t.q[0])) / t.r, wb);
      }
    }
    const bool live = S >= 1e-4f;
    pre[i] = make_float2(live ? 1.f / S : 0.f, live ? wb / S : 0.f);
  }
}

// block (sphere j, slice s): the 13 parameter gradients summed over the slice's points in a fixed
// order, into part[(j S + s) 13 + f]
__global__ void __launch_bounds__(kSmBlock) k_smoothmin_bwd(
    const float* __restrict__ p, int64_t P, const float* __restrict__ centers,
    const float* __restrict__ radii, const float* __restrict__ tfs, int n, float k,
    const float* __restrict__ dvalue, const float* __restrict__ dgrad,
    const float2* __restrict__ pre, float* __restrict__ part) {
  __shared__ float red[kSphF][kSmBlock];
  const int j = blockIdx.x;
  const int S = (int)gridDim.y;
  const int64_t per = (P + S - 1) / S;
  const int64_t i0 = (int64_t)blockIdx.y * per, i1 = std::min<int64_t>(P, i0 + per);
  float s[kSphF];
  for (int f = 0; f < 9; ++f) s[f] = tfs[j * 9 + f] + ((f == 0 || f == 4 || f == 8) ? 1.f : 0.f);
  for (int f = 0; f < 3; ++f) s[9 + f] = centers[j * 3 + f];
  s[12] = radii[j];
  float acc[kSphF];
#pragma unroll
  for (int f = 0; f < kSphF; ++f) acc[f] = 0.f;
  for (int64_t i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
    const float2 pr = pre[i];
    if (pr.x == 0.f) continue;  // clamped: v constant, g = 0
    const float x = p[i * 3], y = p[i * 3 + 1], z = p[i * 3 + 2];
    const SphereTerm t = sphere_term(s, x, y, z);
    const float alpha = expf(-k * t.sd) * pr.x;
    const float dv = dvalue ? dvalue[i] : 0.f;
    float u[3] = {0.f, 0.f, 0.f}, v[3] = {0.f, 0.f, 0.f}, mp[3] = {0.f, 0.f, 0.f};
    float beta = 0.f;
    if (t.r > 0.f) {
      const float ir = 1.f / t.r;
      u[0] = t.q[0] * ir; u[1] = t.q[1] * ir; u[2] = t.q[2] * ir;
      if (dgrad) {
        v[0] = dgrad[i * 3]; v[1] = dgrad[i * 3 + 1]; v[2] = dgrad[i * 3 + 2];
        const float m0 = fmaf(s[2], v[2], fmaf(s[1], v[1], s[0] * v[0]));
        const float m1 = fmaf(s[5], v[2], fmaf(s[4], v[1], s[3] * v[0]));
        const float m2 = fmaf(s[8], v[2], fmaf(s[7], v[1], s[6] * v[0]));
        beta = fmaf(m2, u[2], fmaf(m1, u[1], m0 * u[0]));
        mp[0] = (m0 - beta * u[0]) * ir;
        mp[1] = (m1 - beta * u[1]) * ir;
        mp[2] = (m2 - beta * u[2]) * ir;
      }
    }
    const float kappa = -k * alpha * (beta - pr.y);
    const float c = fmaf(dv, alpha, kappa);
    float e[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) e[a] = fmaf(c, u[a], alpha * mp[a]);
    const float pp[3] = {x, y, z};
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
      for (int b = 0; b < 3; ++b) acc[3 * a + b] += fmaf(e[a], pp[b], alpha * u[a] * v[b]);
#pragma unroll
    for (int a = 0; a < 3; ++a) acc[9 + a] -= e[a];
    acc[12] -= c;
  }
  // block reduction, fixed order (deterministic)
#pragma unroll
  for (int f = 0; f < kSphF; ++f) red[f][threadIdx.x] = acc[f];
  __syncthreads();
  for (int w = kSmBlock / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w)
#pragma unroll
      for (int f = 0; f < kSphF; ++f) red[f][threadIdx.x] += red[f][threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x < kSphF) part[((int64_t)j * S + blockIdx.y) * kSphF + threadIdx.x] = red[threadIdx.x][0];
}

// (sphere j, field f): the slices' partial sums in slice order
__global__ void k_smoothmin_reduce(const float* __restrict__ part, int n, int S,
                                   float* __restrict__ dcenters, float* __restrict__ dradii,
                                   float* __restrict__ dtfs) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n * kSphF) return;
  const int j = e / kSphF, f = e % kSphF;
  float r = 0.f;
  for (int s = 0; s < S; ++s) r += part[((int64_t)j * S + s) * kSphF + f];
  if (f < 9) { if (dtfs) dtfs[j * 9 + f] = r; }
  else if (f < 12) { if (dcenters) dcenters[j * 3 + (f - 9)] = r; }
  else if (dradii) dradii[j] = r;
}

int grid_for(int64_t P) {
  return (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div64(P, kSmBlock), 4096));
}

}  // namespace
}  // namespace nrt

using namespace nrt;

extern "C" {

size_t nrt_sphere_smoothmin_workspace_bytes(int64_t P) {
  const size_t pre = ((size_t)std::max<int64_t>(P, 1) * sizeof(float2) + 255) & ~(size_t)255;
  return pre + (size_t)kMaxSpheres * bwd_slices(P) * kSphF * sizeof(float);
}

int nrt_sphere_smoothmin_forward(const float* p, int64_t P, const float* centers,
                                 const float* radii, const float* tfs, int32_t n, float k,
                                 float* value, float* grad, void* stream) {
  if (P < 0 || n < 1 || !centers || !radii || !tfs || !(k > 0.f)) {
    set_error("nrt_sphere_smoothmin_forward: bad argument");
    return NRT_EINVAL;
  }
  if (P == 0 || (!value && !grad)) return NRT_OK;
  if (!p) { set_error("nrt_sphere_smoothmin_forward: null points"); return NRT_EINVAL; }
  const size_t lds = (size_t)n * kSphF * sizeof(float);
  if (lds > 64 * 1024) { set_error("nrt_sphere_smoothmin_forward: too many spheres"); return NRT_EINVAL; }
  k_smoothmin_fwd<<<dim3(grid_for(P)), dim3(kSmBlock), lds, (hipStream_t)stream>>>(
      p, P, centers, radii, tfs, n, k, value, grad);
  return check_launch("k_smoothmin_fwd");
}

int nrt_sphere_smoothmin_backward(const float* p, int64_t P, const float* centers,
                                  const float* radii, const float* tfs, int32_t n, float k,
                                  const float* dvalue, const float* dgrad, float* dcenters,
                                  float* dradii, float* dtfs, void* workspace, void* stream) {
  if (P < 0 || n < 1 || !centers || !radii || !tfs || !(k > 0.f)) {
    set_error("nrt_sphere_smoothmin_backward: bad argument");
    return NRT_EINVAL;
  }
  hipStream_t st = (hipStream_t)stream;
  if (P == 0 || (!dvalue && !dgrad)) {  // no gradient flows: zeros
    if (dcenters) NRT_HIP(hipMemsetAsync(dcenters, 0, (size_t)n * 12, st));
    if (dradii) NRT_HIP(hipMemsetAsync(dradii, 0, (size_t)n * 4, st));
    if (dtfs) NRT_HIP(hipMemsetAsync(dtfs, 0, (size_t)n * 36, st));
    return NRT_OK;
  }
  if (!p || !workspace) { set_error("nrt_sphere_smoothmin_backward: null points / workspace"); return NRT_EINVAL; }
  const size_t lds = (size_t)n * kSphF * sizeof(float);
  if (lds > 64 * 1024) { set_error("nrt_sphere_smoothmin_backward: too many spheres"); return NRT_EINVAL; }
  float2* pre = (float2*)workspace;
  float* part = (float*)((char*)workspace + (((size_t)P * sizeof(float2) + 255) & ~(size_t)255));
  const int S = bwd_slices(P);
  k_smoothmin_pre<<<dim3(grid_for(P)), dim3(kSmBlock), lds, st>>>(p, P, centers, radii, tfs, n,
                                                                  k, dgrad, pre);
  if (int rc = check_launch("k_smoothmin_pre")) return rc;
  k_smoothmin_bwd<<<dim3(n, S), dim3(kSmBlock), 0, st>>>(p, P, centers, radii, tfs, n, k, dvalue,
                                                        dgrad, pre, part);
  if (int rc = check_launch("k_smoothmin_bwd")) return rc;
  k_smoothmin_reduce<<<dim3((n * kSphF + 255) / 256), dim3(256), 0, st>>>(part, n, S, dcenters,
                                                                         dradii, dtfs);
  return check_launch("k_smoothmin_reduce");
}

}  // extern "C"
