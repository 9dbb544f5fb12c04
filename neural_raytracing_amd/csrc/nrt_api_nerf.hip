// nrt_api_nerf.hip -- NeRFLE (NeRF + point-light, shapes/nerf.py:153-214) volume rendering:
// sample points, first MLP (density + 64-d latent), second MLP (rgb from latent, direction and
// light position), and the reference's front-to-back compositing with its quirks.
#include "nrt_launch.h"

namespace nrt {

// pts[s * P + p] = r_o + ts[s] * r_d   (nerf.py:178-179, tensordot(ts, r_d, dims=0))
template <int = 0>
__global__ void k_nerf_points(const float* __restrict__ rays, int64_t P, const float* __restrict__ ts,
                              int S, float* __restrict__ pts) {
  const int64_t n = (int64_t)S * P;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = i / P, p = i - s * P;
    const float t = ts[s];
    const float* r = rays + p * 6;
#pragma unroll
    for (int k = 0; k < 3; ++k) pts[i * 3 + k] = __fadd_rn(r[k], __fmul_rn(t, r[3 + k]));
  }
}

// second MLP input [latent (64) | r_d (3) | light location (3)]   (nerf.py:197-203)
template <int = 0>
__global__ void k_nerf_second_in(const float* __restrict__ first_out, const float* __restrict__ rays,
                                 int64_t P, int S, const float* __restrict__ light,
                                 float* __restrict__ x2) {
  const int64_t n = (int64_t)S * P;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = i % P;
    const float* f = first_out + i * 65;
    float* o = x2 + i * 70;
    for (int k = 0; k < 64; ++k) o[k] = f[1 + k];
    o[64] = rays[p * 6 + 3]; o[65] = rays[p * 6 + 4]; o[66] = rays[p * 6 + 5];
    o[67] = light[0]; o[68] = light[1]; o[69] = light[2];
  }
}

// nerf.py:203-214: rgb = sigmoid(second), sigma = relu(alpha_raw), a_s = 1 - exp(-sigma t_s)
// (absolute depth t, not a spacing), cp = cumprod(clamp(1 - a, 1e-10)) rolled by one with the
// LAST entry set to 1: w_0 = a_0 cp_{S-1}, w_s = a_s cp_{s-1} (1 <= s <= S-2), w_{S-1} = a_{S-1}.
template <int = 0>
__global__ void k_nerf_composite(const float* __restrict__ first_out, const float* __restrict__ rgb_raw,
                                 const float* __restrict__ ts, int64_t P, int S,
                                 float* __restrict__ out) {
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < P;
       p += (int64_t)gridDim.x * blockDim.x) {
    // pass 1: cp_{S-1} (the product over every sample), needed by w_0
    float cp = 1.f;
    for (int s = 0; s < S; ++s) {
      const float sig = fmaxf(first_out[((int64_t)s * P + p) * 65], 0.f);
      const float a = 1.f - expf(-(sig * ts[s]));
      cp = cp * fmaxf(1.f - a, 1e-10f);
    }
    const float cp_last = cp;
    float acc[3] = {0.f, 0.f, 0.f};
    float prev = 1.f;  // cp_{s-1}
    for (int s = 0; s < S; ++s) {
      const int64_t i = (int64_t)s * P + p;
      const float sig = fmaxf(first_out[i * 65], 0.f);
      const float a = 1.f - expf(-(sig * ts[s]));
      const float w = s == S - 1 ? a * 1.f : (s == 0 ? a * cp_last : a * prev);
      prev = prev * fmaxf(1.f - a, 1e-10f);
#pragma unroll
      for (int k = 0; k < 3; ++k) acc[k] += w * (1.f / (1.f + expf(-rgb_raw[i * 3 + k])));
    }
    out[p * 3] = acc[0]; out[p * 3 + 1] = acc[1]; out[p * 3 + 2] = acc[2];
  }
}

static size_t a256(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace nrt

using namespace nrt;

extern "C" {

size_t nrt_nerfle_workspace_bytes(int64_t P, int32_t S) {
  const size_t n = (size_t)std::max<int64_t>(P, 1) * (size_t)std::max(S, 1);
  return a256(n * 3 * 4) + a256(n * 65 * 4) + a256(n * 70 * 4) + a256(n * 3 * 4);
}

int nrt_nerfle_forward(const nrt_mlp* first, const nrt_mlp* second, const float* rays, int64_t P,
                       const float* ts, int32_t S, const float* light, float* rgb, void* workspace,
                       int precision, void* stream) {
  if (!first || !second || P < 0 || S < 1) { set_error("nrt_nerfle_forward: bad argument"); return NRT_EINVAL; }
  if (P == 0) return NRT_OK;
  if (!rays || !ts || !light || !rgb || !workspace) { set_error("nrt_nerfle_forward: null argument"); return NRT_EINVAL; }
  if (first->desc.in_size != 3 || first->desc.out != 65 || second->desc.in_size != 70 ||
      second->desc.out != 3) {
    set_error("nrt_nerfle_forward: expects first 3 -> 65 and second 70 -> 3 (nerf.py:162-172)");
    return NRT_EINVAL;
  }
  hipStream_t st = (hipStream_t)stream;
  const size_t n = (size_t)P * S;
  char* ws = (char*)workspace;
  float* pts = (float*)ws;
  float* f1 = (float*)(ws + a256(n * 12));
  float* x2 = (float*)(ws + a256(n * 12) + a256(n * 260));
  float* c2 = (float*)(ws + a256(n * 12) + a256(n * 260) + a256(n * 280));
  const int blocks = (int)std::min<int64_t>(ceil_div64((int64_t)n, 256), 4096);
  ProfScope prof("k_nerfle", st);
  k_nerf_points<><<<dim3(blocks), dim3(256), 0, st>>>(rays, P, ts, S, pts);
  if (int rc = check_launch("k_nerf_points")) return rc;
  if (int rc = nrt_mlp_forward(first, pts, nullptr, (int64_t)n, f1, precision, stream)) return rc;
  k_nerf_second_in<><<<dim3(blocks), dim3(256), 0, st>>>(f1, rays, P, S, light, x2);
  if (int rc = check_launch("k_nerf_second_in")) return rc;
  if (int rc = nrt_mlp_forward(second, x2, nullptr, (int64_t)n, c2, precision, stream)) return rc;
  k_nerf_composite<><<<dim3(std::min<int64_t>(ceil_div64(P, 256), 4096)), dim3(256), 0, st>>>(
      f1, c2, ts, P, S, rgb);
  return check_launch("k_nerf_composite");
}

}  // extern "C"
