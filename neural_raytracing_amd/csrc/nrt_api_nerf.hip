// nrt_api_nerf.hip -- NeRFLE (NeRF + point-light, shapes/nerf.py:153-214) volume rendering:
// sample points, first MLP (density + 64-d latent), second MLP (rgb from latent, direction and
// light position), and the reference's front-to-back compositing with its quirks.
#include <array>

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

// second MLP input [latent (64) | r_d (3) | light encoding (LK)]   (nerf.py:182-203): the point
// light's location (LK = 3) or its envmap over bins^2 directions (LK = 3 bins^2)
template <int = 0>
__global__ void k_nerf_second_in(const float* __restrict__ first_out, const float* __restrict__ rays,
                                 int64_t P, int S, const float* __restrict__ light, int LK,
                                 float* __restrict__ x2) {
  const int64_t n = (int64_t)S * P;
  const int in2 = 67 + LK;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = i % P;
    const float* f = first_out + i * 65;
    float* o = x2 + i * in2;
    for (int k = 0; k < 64; ++k) o[k] = f[1 + k];
    o[64] = rays[p * 6 + 3]; o[65] = rays[p * 6 + 4]; o[66] = rays[p * 6 + 5];
    for (int k = 0; k < LK; ++k) o[67 + k] = light[k];
  }
}

// torch.linspace(start, end, steps)[k] (float32, symmetric two-sided formula)
__device__ __forceinline__ float linspace_at(float start, float end, int steps, int k) {
  if (steps == 1) return start;
  const float step = (end - start) / (float)(steps - 1);
  return k < steps / 2 ? start + step * (float)k : end - step * (float)(steps - k - 1);
}

// PointLights.envmap(elev_azim_to_dir(meshgrid(linspace(0, 180, bins), linspace(0, 45, bins))))
// (nerf.py:183-191, utils.py:478-486, lights.py:81-88); the degrees go in as radians, as there.
template <int = 0>
__global__ void k_light_envmap(const LightDev* __restrict__ lp, int bins, float* __restrict__ out) {
  const LightDev& lt = *lp;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= bins * bins) return;
  const float limit = 3.14159265358979f - 1e-7f;
  const float elev = fminf(fmaxf(linspace_at(0.f, 180.f, bins, i / bins), -limit), limit);
  const float azim = fminf(fmaxf(linspace_at(0.f, 45.f, bins, i % bins), -limit), limit);
  const float dx = sinf(azim) * cosf(elev), dy = cosf(azim) * cosf(elev), dz = sinf(elev);
  const float vx = dx - lt.loc[0], vy = dy - lt.loc[1], vz = dz - lt.loc[2];
  const float dist = sqrtf(vx * vx + vy * vy + vz * vz);
  const float fall = fmaxf((lt.c + lt.l * dist) + lt.q * (dist * dist), 1e-6f);
  for (int k = 0; k < 3; ++k) out[i * 3 + k] = lt.scaled_dir[k] / fall;
}

// nerf.py:203-214: rgb = sigmoid(second), sigma = relu(alpha_raw), a_s = 1 - exp(-sigma t_s)
// (absolute depth t, not a spacing), cp = cumprod(clamp(1 - a, 1e-10)) rolled by one with the
// LAST entry set to 1: w_0 = a_0 cp_{S-1}, w_s = a_s cp_{s-1} (1 <= s <= S-2), w_{S-1} = a_{S-1}.
// alpha_raw[i * astride] is the first MLP's output 0 of sample i, rgb_raw[i * 3 + k] the second's.
template <int = 0>
__global__ void k_nerf_composite(const float* __restrict__ first_out, int astride,
                                 const float* __restrict__ rgb_raw, const float* __restrict__ ts,
                                 int64_t P, int S, float* __restrict__ out) {
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < P;
       p += (int64_t)gridDim.x * blockDim.x) {
    // pass 1: cp_{S-1} (the product over every sample), needed by w_0
    float cp = 1.f;
    for (int s = 0; s < S; ++s) {
      const float sig = fmaxf(first_out[((int64_t)s * P + p) * astride], 0.f);
      const float a = 1.f - expf(-(sig * ts[s]));
      cp = cp * fmaxf(1.f - a, 1e-10f);
    }
    const float cp_last = cp;
    float acc[3] = {0.f, 0.f, 0.f};
    float prev = 1.f;  // cp_{s-1}
    for (int s = 0; s < S; ++s) {
      const int64_t i = (int64_t)s * P + p;
      const float sig = fmaxf(first_out[i * astride], 0.f);
      const float a = 1.f - expf(-(sig * ts[s]));
      const float w = s == S - 1 ? a * 1.f : (s == 0 ? a * cp_last : a * prev);
      prev = prev * fmaxf(1.f - a, 1e-10f);
#pragma unroll
      for (int k = 0; k < 3; ++k) acc[k] += w * (1.f / (1.f + expf(-rgb_raw[i * 3 + k])));
    }
    out[p * 3] = acc[0]; out[p * 3 + 1] = acc[1]; out[p * 3 + 2] = acc[2];
  }
}

// The same compositing for the fused path's ray-major samples (alpha_raw[p * S + s],
// rgb_raw[(p * S + s) * 3 + k]): one wave per ray, 64 depths per step, the cumulative product as
// a wave prefix product carried across steps (the sequential product reassociated: FP32
// rounding differences only).
template <int = 0>
__global__ void k_nerf_composite_rm(const float* __restrict__ alpha_raw,
                                    const float* __restrict__ rgb_raw,
                                    const float* __restrict__ ts, int64_t P, int S,
                                    float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t p = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; p < P; p += nw) {
    const float* al = alpha_raw + p * S;
    const float* rg = rgb_raw + p * S * 3;
    float carry = 1.f;  // cp_{c0 - 1}
    float acc[3] = {0.f, 0.f, 0.f};
    float a_first = 0.f, c_first[3] = {0.f, 0.f, 0.f};
    for (int c0 = 0; c0 < S; c0 += 64) {
      const int s = c0 + lane;
      const bool v = s < S;
      float a = 0.f, q = 1.f, col[3] = {0.f, 0.f, 0.f};
      if (v) {
        const float sig = fmaxf(al[s], 0.f);
        a = 1.f - expf(-(sig * ts[s]));
        q = fmaxf(1.f - a, 1e-10f);
#pragma unroll
        for (int k = 0; k < 3; ++k) col[k] = 1.f / (1.f + expf(-rg[s * 3 + k]));
      }
      float inc = q;  // inclusive prefix product of q over the step's lanes
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const float o = __shfl_up(inc, d);
        if (lane >= d) inc *= o;
      }
      const float up = __shfl_up(inc, 1);
      const float prev = carry * (lane == 0 ? 1.f : up);  // cp_{s-1}
      if (s == 0) {
        a_first = a;
#pragma unroll
        for (int k = 0; k < 3; ++k) c_first[k] = col[k];
      }
      const float w = !v ? 0.f : (s == S - 1 ? a : (s == 0 ? 0.f : a * prev));
#pragma unroll
      for (int k = 0; k < 3; ++k) acc[k] += w * col[k];
      carry = carry * __shfl(inc, 63);
    }
    // w_0 = a_0 cp_{S-1} (the roll), unless S == 1 where w_0 = a_0
    if (lane == 0 && S > 1)
#pragma unroll
      for (int k = 0; k < 3; ++k) acc[k] += (a_first * carry) * c_first[k];
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) acc[k] += __shfl_xor(acc[k], d);
    if (lane == 0) {
      out[p * 3] = acc[0]; out[p * 3 + 1] = acc[1]; out[p * 3 + 2] = acc[2];
    }
  }
}

static size_t a256(size_t x) { return (x + 255) & ~(size_t)255; }

// ------------------------------------------------------------------------------------------
// PlainNeRF (shapes/nerf.py:9-74): latent-conditioned density MLP + direction MLP, tanh colours
// ------------------------------------------------------------------------------------------
// first MLP input of sample i = s * P + p: pts (3) and the latent row of the ray's camera
// (self.latent[None, :, None, None, None, :], nerf.py:52; row = p / rays_per_latent)
template <int = 0>
__global__ void k_plain_first_in(const float* __restrict__ rays, int64_t P,
                                 const float* __restrict__ ts, int S,
                                 const float* __restrict__ latent, int L, int64_t rays_per_latent,
                                 float* __restrict__ pts, float* __restrict__ lat1) {
  const int64_t n = (int64_t)S * P;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = i / P, p = i - s * P;
    const float t = ts[s];
    const float* r = rays + p * 6;
#pragma unroll
    for (int k = 0; k < 3; ++k) pts[i * 3 + k] = __fadd_rn(r[k], __fmul_rn(t, r[3 + k]));
    const float* lr = latent + (p / rays_per_latent) * L;
    for (int k = 0; k < L; ++k) lat1[i * L + k] = lr[k];
  }
}

// second MLP input: x = dir_to_elev_azim(r_d) (utils.py:490-494), latent = [intermediate, latent]
// (nerf.py:60-64; first_out = [alpha | intermediate (I)])
template <int = 0>
__global__ void k_plain_second_in(const float* __restrict__ first_out, int I,
                                  const float* __restrict__ rays, int64_t P, int S,
                                  const float* __restrict__ latent, int L, int64_t rays_per_latent,
                                  float* __restrict__ x2, float* __restrict__ lat2) {
  const int64_t n = (int64_t)S * P;
  const int L2 = I + L;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = i % P;
    float elev, azim;
    dir_elev_azim(rays[p * 6 + 3], rays[p * 6 + 4], rays[p * 6 + 5], elev, azim);
    x2[i * 2] = elev;
    x2[i * 2 + 1] = azim;
    const float* f = first_out + i * (1 + I);
    float* o = lat2 + i * L2;
    for (int k = 0; k < I; ++k) o[k] = f[1 + k];
    const float* lr = latent + (p / rays_per_latent) * L;
    for (int k = 0; k < L; ++k) o[I + k] = lr[k];
  }
}

// nerf.py:64-74: rgb = tanh(second), sigma = relu(alpha + noise), the NeRFLE weights (absolute
// depth, rolled cumprod with the last entry 1), out = (sum_s w_s rgb_s + 1) / 2
template <int = 0>
__global__ void k_plain_composite(const float* __restrict__ first_out, int astride,
                                  const float* __restrict__ noise, const float* __restrict__ rgb_raw,
                                  const float* __restrict__ ts, int64_t P, int S,
                                  float* __restrict__ out) {
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < P;
       p += (int64_t)gridDim.x * blockDim.x) {
    auto alpha_at = [&](int s) {
      const int64_t i = (int64_t)s * P + p;
      float a = first_out[i * astride];
      if (noise) a = a + noise[i];
      const float sig = fmaxf(a, 0.f);
      return 1.f - expf(-(sig * ts[s]));
    };
    float cp = 1.f;
    for (int s = 0; s < S; ++s) cp = cp * fmaxf(1.f - alpha_at(s), 1e-10f);
    const float cp_last = cp;
    float acc[3] = {0.f, 0.f, 0.f};
    float prev = 1.f;
    for (int s = 0; s < S; ++s) {
      const int64_t i = (int64_t)s * P + p;
      const float a = alpha_at(s);
      const float w = s == S - 1 ? a * 1.f : (s == 0 ? a * cp_last : a * prev);
      prev = prev * fmaxf(1.f - a, 1e-10f);
#pragma unroll
      for (int k = 0; k < 3; ++k) acc[k] += w * tanhf(rgb_raw[i * 3 + k]);
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) out[p * 3 + k] = (acc[k] + 1.f) / 2.f;
  }
}

// ------------------------------------------------------------------------------------------
// Fused FP16 NeRFLE sample kernel on the k-outer program engine (ring::KEngine): per wave 32
// samples (columns, ray-major: sample g = p * S + s); both MLPs, the second MLP's Fourier
// projection and its input assembly stay in registers; only alpha_raw and rgb_raw (16 B per
// sample) reach HBM.
//
// Program chunk order (build_nerf_program, consumed in exactly this order per batch):
//   first MLP (hidden 128 = 4 row blocks, F = 16, 3 -> 65): init enc [3 k-steps];
//     per hidden layer: hidden [8] k-steps, + enc [3] on skip layers; out (3 row blocks) [8]
//   projection: A_hi (7 k-steps) then A_lo (7) of basis^T (16 x 70) in one chunk
//   second MLP (hidden 64 = 2 row blocks, 70 -> 3): init enc [9]; per hidden layer hidden
//     [4] or, on skip layers, hidden + enc [13]; out [4] (1 row block)
// (chunks of at most kNerfMaxF fragments; one barrier per chunk)
// Second-MLP encoding k-steps (9): e0, e1 = sin/cos of projections q = 8e + 4h + jj (the usual
// pair order); e2..e7 = the first MLP's output tiles in accumulator order (row 1 + k = latent k;
// row 0 and rows > 64 have zero weight); e8 = (r_d, light) in half 0.
// ------------------------------------------------------------------------------------------
#ifndef NRT_NERF_TILES
#define NRT_NERF_TILES 2
#endif
#ifndef NRT_NERF_WAVES
#if NRT_NERF_TILES == 1
#define NRT_NERF_WAVES 12  // 3 waves per SIMD (162 VGPRs with the DMA engine)
#else
#define NRT_NERF_WAVES 8
#endif
#endif
#ifndef NRT_NERF_MAXF
#define NRT_NERF_MAXF 32
#endif
#ifndef NRT_NERF_DMA
#define NRT_NERF_DMA 1
#endif
constexpr int kNerfWaves = NRT_NERF_WAVES;
constexpr int kNerfTiles = NRT_NERF_TILES;  // 32-sample tiles per wave (each A read feeds them all)
constexpr bool kNerfDma = NRT_NERF_DMA != 0;  // weight chunks by LDS-DMA (KEngine DMA mode)
constexpr int kNerfMaxF = NRT_NERF_MAXF;  // fragments per ring slot (3 slots: 96 KiB of LDS at 32)
constexpr int kNerfKC1 = kNerfMaxF / 4;   // k-steps per chunk of the first MLP (4 row blocks)
constexpr int kNerfKC2 = kNerfMaxF / 2;   // ... of the second MLP (2 row blocks)
constexpr int kNerfL1 = 5, kNerfL2 = 8, kNerfSkip = 3;  // nerf.py:162-172 (SkipConnMLP skip 3)

// leaky_relu on packed halves (ring::kact's pk_mul + pk_max): act(enc) from the encoding's own
// FP16 values instead of a second sin / cos pass
__device__ __forceinline__ h8 leaky_h8(const h8& v) {
  const ring::h2 k = {(_Float16)0.01f, (_Float16)0.01f};
  h8 f;
#pragma unroll
  for (int j = 0; j < 8; j += 2) {
    const ring::h2 x = {v[j], v[j + 1]};
    const ring::h2 r = __builtin_elementwise_max(x, x * k);
    f[j] = r[0];
    f[j + 1] = r[1];
  }
  return f;
}

// acc[q][ib] += W[ib] * [b1[q][0..KS1), act(b2[q][0..KS2))] over chunks of KC k-steps, for the
// TT 32-sample tiles q of the wave: each A fragment read from the ring feeds TT MFMAs.  ACT2:
// act = leaky_relu on the packed halves at each use (the skip layers' act(encoding) is not kept
// in registers), else the identity
template <int NB, int KS1, int KS2, int KC, int TT, bool ACT2 = false, class Eng, int N1, int N2>
__device__ __forceinline__ void nerf_layer(Eng& E, f16v (&acc)[TT][NB],
                                           const h8 (&b1)[TT][N1], const h8 (&b2)[TT][N2]) {
  static_assert(KS1 <= N1 && KS2 <= N2, "fragment arrays too short");
  static_assert(KC * NB <= Eng::MAXF, "chunk larger than a ring slot");
  constexpr int KS = KS1 + KS2;
  constexpr int NCH = (KS + KC - 1) / KC;
#ifndef NRT_NERF_W
#define NRT_NERF_W 4
#endif
  // A fragments in flight (LDS latency cover: each one feeds TT MFMAs)
  constexpr int W = (NRT_NERF_W + TT - 1) / TT;
#pragma unroll
  for (int cc = 0; cc < NCH; ++cc) {
    const h8* A = E.begin();
    const int nf = ((KS - cc * KC) < KC ? (KS - cc * KC) : KC) * NB;  // fragments of this chunk
    h8 a[W];
#pragma unroll
    for (int w = 0; w < W; ++w)
      if (w < nf) a[w] = A[w * 64];
#pragma unroll
    for (int m = 0; m < KC * NB; ++m) {
      if (m < nf) {
        const int s = cc * KC + m / NB, ib = m % NB;
#pragma unroll
        for (int q = 0; q < TT; ++q) {
          h8 b;
          if (s < KS1) b = b1[q][s < KS1 ? s : 0];
          else if (ACT2) b = leaky_h8(b2[q][s >= KS1 ? s - KS1 : 0]);
          else b = b2[q][s >= KS1 ? s - KS1 : 0];
          acc[q][ib] = mfma16(a[m % W], b, acc[q][ib]);
        }
        if (m + W < nf) a[m % W] = A[(m + W) * 64];
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    E.end();
  }
}

// the first MLP (nerf.py:162-163: 5 x 128, F = 16, 3 -> 65) with its 3 output row blocks, on
// the wave's TT tiles (the layer biases read once from LDS for all of them)
template <int L, int SKIP, int TT, class Eng>
__device__ __forceinline__ void nerf_first(Eng& E, const ProgMlp& pm, const float (&x0)[TT],
                                           const float (&x1)[TT], const float (&x2)[TT],
                                           f16v (&o)[TT][3]) {
  constexpr int NB = 4, NE = 3;
  const int h = E.lane >> 5;
  const float4* basis = E.lbasis + pm.basis_off;
  f16v acc[TT][NB];
  h8 hv[TT][2 * NB];
  h8 enc[TT][NE];
#pragma unroll
  for (int q = 0; q < TT; ++q)
#pragma unroll
    for (int s = 0; s < NE; ++s) enc[q][s] = ring::enc_frag_k<-1>(basis, s, NE - 1, h, x0[q], x1[q], x2[q]);
  auto biases = [&](int layer) {
#pragma unroll
    for (int ib = 0; ib < NB; ++ib) {
      acc[0][ib] = E.bias_at(pm, layer, ib, h);
#pragma unroll
      for (int q = 1; q < TT; ++q) acc[q][ib] = acc[0][ib];
    }
  };
  biases(0);
  nerf_layer<NB, NE, 0, kNerfKC1, TT>(E, acc, enc, enc);
#pragma unroll
  for (int q = 0; q < TT; ++q)
#pragma unroll
    for (int s = 0; s < NE; ++s) enc[q][s] = leaky_h8(enc[q][s]);  // act(enc) from the same halves
#pragma unroll
  for (int i = 0; i < L; ++i) {
#pragma unroll
    for (int q = 0; q < TT; ++q) ring::kact<NB, ACT_LEAKY>(acc[q], hv[q]);
    biases(1 + i);
    nerf_layer<NB, 2 * NB, 0, kNerfKC1, TT>(E, acc, hv, hv);
    if (i != L - 1 && (i % SKIP) == 0) nerf_layer<NB, NE, 0, kNerfKC1, TT>(E, acc, enc, enc);
  }
#pragma unroll
  for (int q = 0; q < TT; ++q) ring::kact<NB, ACT_LEAKY>(acc[q], hv[q]);
#pragma unroll
  for (int ob = 0; ob < 3; ++ob) {
    o[0][ob] = E.bias_at(pm, L + 1, ob, h);
#pragma unroll
    for (int q = 1; q < TT; ++q) o[q][ob] = o[0][ob];
  }
  nerf_layer<3, 2 * NB, 0, kNerfKC1, TT>(E, o, hv, hv);
}

__device__ __forceinline__ h8 h8_of(const float (&v)[8]) {
  h8 f;
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = (_Float16)v[j];
  return f;
}

// v (8 f32) -> FP16 halves hi = RNE(v) and residuals lo = RNE(v - hi) (ring3::split2: one
// v_fma_mix per residual instead of a convert back and a subtract)
__device__ __forceinline__ void split_h8(const float (&v)[8], h8& hi, h8& lo) {
  ring3::u4v h, l;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t a, b;
    ring3::split2(v[2 * q], v[2 * q + 1], a, b);
    h[q] = a; l[q] = b;
  }
  hi = __builtin_bit_cast(h8, h);
  lo = __builtin_bit_cast(h8, l);
}

template <int WV, int TT>
__global__ void __launch_bounds__(64 * WV, 1) k_nerfle16(
    const ProgDev prog, const float* __restrict__ rays, int64_t P, const float* __restrict__ ts,
    int S, const float* __restrict__ light, float* __restrict__ alpha_raw,
    float* __restrict__ rgb_raw) {
  extern __shared__ __attribute__((aligned(16))) char smem_c[];
  const int64_t n = (int64_t)S * P;
  const int64_t per_block = 32 * TT * WV;
  if ((int64_t)blockIdx.x * per_block >= n) return;
  ring::KEngine<WV, kNerfMaxF, kNerfDma> E;
  E.init(prog, smem_c);
  const int lane = lane_id(), h = lane >> 5;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const ProgMlp& m1 = prog.mlp[0];
  const ProgMlp& m2 = prog.mlp[1];
  const float lx = light[0], ly = light[1], lz = light[2];
  for (int64_t b0 = (int64_t)blockIdx.x * per_block; b0 < n; b0 += (int64_t)gridDim.x * per_block) {
    // tile q of this wave: samples b0 + 32 (TT wv + q) + [0, 32) (recomputed where needed: the
    // registers go to the MLPs)
    auto sample = [&](int q) -> int64_t { return b0 + 32 * (TT * wv + q) + (lane & 31); };
    auto ray_of = [&](int q) -> const float* {
      const int64_t g = sample(q);
      return rays + ((g < n ? g : n - 1) / S) * 6;  // ray-major: a tile's columns share a ray
    };
    float x0[TT], x1[TT], x2[TT];
#pragma unroll
    for (int q = 0; q < TT; ++q) {
      const int64_t g = sample(q);
      const int64_t gg = g < n ? g : n - 1;
      const float t = ts[gg - (gg / S) * S];
      const float* r = ray_of(q);
      // pts = r_o + t r_d (nerf.py:179, no FMA contraction)
      x0[q] = __fadd_rn(r[0], __fmul_rn(t, r[3]));
      x1[q] = __fadd_rn(r[1], __fmul_rn(t, r[4]));
      x2[q] = __fadd_rn(r[2], __fmul_rn(t, r[5]));
    }
    f16v o[TT][3];
    nerf_first<kNerfL1, kNerfSkip, TT>(E, m1, x0, x1, x2, o);
    // second-MLP input fragments e2..e8 (hi) and their FP16 residuals (lo) for the projection
    h8 e[TT][9], lo[TT][7];
#pragma unroll
    for (int q = 0; q < TT; ++q) {
#pragma unroll
      for (int tt = 0; tt < 6; ++tt) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = o[q][tt >> 1][8 * (tt & 1) + j];
        split_h8(v, e[q][2 + tt], lo[q][tt]);
      }
      float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (h == 0) {
        const float* r = ray_of(q);
        v[0] = r[3]; v[1] = r[4]; v[2] = r[5]; v[3] = lx; v[4] = ly; v[5] = lz;
      }
      split_h8(v, e[q][8], lo[q][6]);
    }
    // projections x @ B (utils.py:37-40) as hi*hi + lo(A)*hi + hi*lo(x): FP32-accurate
    f16v pq[TT];
#pragma unroll
    for (int q = 0; q < TT; ++q)
#pragma unroll
      for (int k = 0; k < 16; ++k) pq[q][k] = 0.f;
    {
      const h8* A = E.begin();
#pragma unroll
      for (int tt = 0; tt < 7; ++tt) {
        const h8 ah = A[tt * 64], al = A[(7 + tt) * 64];
#pragma unroll
        for (int q = 0; q < TT; ++q) {
          pq[q] = mfma16(ah, e[q][2 + tt], pq[q]);
          pq[q] = mfma16(al, e[q][2 + tt], pq[q]);
          pq[q] = mfma16(ah, lo[q][tt], pq[q]);
        }
      }
      E.end();
    }
    // rows q = (reg & 3) + 8 (reg >> 2) + 4h: regs 0..3 -> q = 4h + jj, regs 4..7 -> 8 + 4h + jj
#pragma unroll
    for (int q = 0; q < TT; ++q) {
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        float v[8];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          v[2 * jj] = __sinf(pq[q][4 * s2 + jj]);
          v[2 * jj + 1] = __cosf(pq[q][4 * s2 + jj]);
        }
        e[q][s2] = h8_of(v);
      }
    }
    // the second MLP (nerf.py:168-172: 8 x 64, 70 -> 3)
    constexpr int NB = 2;
    f16v acc[TT][NB];
    h8 hv[TT][2 * NB];
    auto biases = [&](int layer) {
#pragma unroll
      for (int ib = 0; ib < NB; ++ib) {
        acc[0][ib] = E.bias_at(m2, layer, ib, h);
#pragma unroll
        for (int q = 1; q < TT; ++q) acc[q][ib] = acc[0][ib];
      }
    };
    biases(0);
    nerf_layer<NB, 9, 0, kNerfKC2, TT>(E, acc, e, e);
#pragma unroll
    for (int i = 0; i < kNerfL2; ++i) {
#pragma unroll
      for (int q = 0; q < TT; ++q) ring::kact<NB, ACT_LEAKY>(acc[q], hv[q]);
      biases(1 + i);
      if (i != kNerfL2 - 1 && (i % kNerfSkip) == 0) nerf_layer<NB, 2 * NB, 9, kNerfKC2, TT, true>(E, acc, hv, e);
      else nerf_layer<NB, 2 * NB, 0, kNerfKC2, TT>(E, acc, hv, hv);
    }
#pragma unroll
    for (int q = 0; q < TT; ++q) ring::kact<NB, ACT_LEAKY>(acc[q], hv[q]);
    f16v out[TT][1];
    out[0][0] = E.bias_at(m2, kNerfL2 + 1, 0, h);
#pragma unroll
    for (int q = 1; q < TT; ++q) out[q][0] = out[0][0];
    nerf_layer<1, 2 * NB, 0, kNerfKC2, TT>(E, out, hv, hv);
#pragma unroll
    for (int q = 0; q < TT; ++q) {
      const int64_t g = sample(q);
      if (g < n && h == 0) {
        alpha_raw[g] = o[q][0][0];
        rgb_raw[g * 3] = out[q][0][0]; rgb_raw[g * 3 + 1] = out[q][0][1]; rgb_raw[g * 3 + 2] = out[q][0][2];
      }
    }
  }
  E.drain();
}

// first: 3 -> 65, hidden 128, F 16; second: 67 + LK -> 3, hidden 64, F 16 (LK = 3: the point
// light's location; LK = 3 bins^2: NeRF+LE's envmap, folded into one constant input column by
// build_nerf_program); both leaky_relu, no latent
static bool nerf_fusable(const nrt_mlp* f, const nrt_mlp* s) {
  const MlpDev& a = f->host_dev;
  const MlpDev& b = s->host_dev;
  if (f->refreshed || s->refreshed) return false;  // stale program streams: unfused path
  return a.in_size == 3 && a.nb == 4 && a.freqs == 16 && a.out == 65 && a.latent == 0 &&
         a.act == ACT_LEAKY && b.in_size >= 70 && b.nb == 2 && b.freqs == 16 && b.out == 3 &&
         b.latent == 0 && b.act == ACT_LEAKY && a.n_hidden == kNerfL1 && b.n_hidden == kNerfL2 &&
         a.skip == kNerfSkip && b.skip == kNerfSkip && (int)f->host_w.size() == a.n_hidden + 2 &&
         (int)s->host_w.size() == b.n_hidden + 2 && a.ke == 48;
}

// the program stream of k_nerfle16 (chunk order in the kernel's header comment).
// env (NeRF+LE, nerf.py:183-199): the light's envmap, LK = s->in_size - 67 values.  It is one
// constant per frame, so its share of the colour MLP's input is folded into the kernel's 70-input
// layout: input column 67 is a constant 1 (the kernel's light input is (1, 0, 0)), its weight in
// the init and skip layers is W[:, env] . env and its row of the Fourier basis is env . B[env, :]
// (both summed in double, rounded once to f32); columns 68-69 are zero.  x'.B' = x.B and
// W' x' = W x up to the order of the sums: the FP16 kernel's products are unchanged in kind.
static int build_nerf_program(const nrt_mlp* f, const nrt_mlp* s, nrt_prog& out,
                              const float* env = nullptr) {
  out.ok = false;
  const MlpDev& a = f->host_dev;
  const MlpDev& b = s->host_dev;
  typedef std::array<_Float16, 512> Frag;  // [lane][8]
  std::vector<Frag> frags;
  std::vector<int> coff;
  // first MLP: its own k-outer stream ([layer][k-step][row block]); one chunk per layer part
  frags.resize(a.nk_frags);
  NRT_HIP(hipMemcpy(frags.data(), a.streamk16, (size_t)a.nk_frags * 1024, hipMemcpyDeviceToHost));
  {
    int base = 0;
    coff.push_back(base);  // init: 3 encoding k-steps x 4 row blocks
    base += 3 * 4;
    static_assert(kNerfKC1 >= 3 && 8 % kNerfKC1 == 0, "first-MLP chunking");
    for (int i = 0; i < a.n_hidden; ++i) {
      const bool skip = i != a.n_hidden - 1 && (i % a.skip) == 0;
      for (int st = 0; st < 8; st += kNerfKC1) coff.push_back(base + st * 4);  // 8 hidden k-steps
      if (skip) coff.push_back(base + 8 * 4);  // + 3 encoding k-steps
      base += (8 + (skip ? 3 : 0)) * 4;
    }
    for (int st = 0; st < 8; st += kNerfKC1) coff.push_back(base + st * 3);  // out: 8 x 3 blocks
    base += 8 * 3;
    if (base != a.nk_frags) {
      set_error("build_nerf_program: unexpected first-MLP stream layout");
      return NRT_EUNSUPPORTED;
    }
  }
  // element (h, j) of second-MLP encoding k-step e -> kernel input column (-1: none)
  const int IN = 70, F = 16;
  const int INo = s->host_dev.in_size;  // the MLP's own input width (70, or 67 + 3 bins^2)
  const int LK = INo - 67;
  if (env == nullptr && INo != IN) {
    set_error("build_nerf_program: a NeRF+LE colour MLP needs its envmap");
    return NRT_EINVAL;
  }
  auto enc_col = [&](int e, int hf, int j) -> int {
    if (e < 2) {
      const int q = 8 * e + 4 * hf + (j >> 1);
      return (j & 1) ? IN + F + q : IN + q;
    }
    if (e < 8) {
      const int t = e - 2;
      const int r = 32 * (t >> 1) + 16 * (t & 1) + 8 * (j >> 2) + 4 * hf + (j & 3);
      return (r >= 1 && r <= 64) ? r - 1 : -1;
    }
    return (hf == 0 && j < 6) ? 64 + j : -1;
  };
  // the second MLP's basis at kernel input column col (< IN), with the envmap fold
  auto basis_at = [&](int col, int q) -> float {
    if (env == nullptr || col < 67) return s->host_basis[(size_t)col * F + q];
    if (col > 67) return 0.f;
    double acc = 0.0;
    for (int k = 0; k < LK; ++k) acc += (double)env[k] * s->host_basis[(size_t)(67 + k) * F + q];
    return (float)acc;
  };
  // weight of layer l at (row, kernel column col) of its [hidden? H | x (IN) | sin F | cos F]
  // layout; Co is the layer's own width ([hidden? H | x (INo) | sin F | cos F])
  auto weight_at = [&](const std::vector<float>& W, int row, int col, int base, int Co) -> float {
    if (col < base) return W[(size_t)row * Co + col];
    const int ic = col - base;
    if (ic < 67 || env == nullptr) {
      const int oc = ic < IN ? ic : INo + (ic - IN);
      return W[(size_t)row * Co + base + oc];
    }
    if (ic >= IN) return W[(size_t)row * Co + base + INo + (ic - IN)];
    if (ic > 67) return 0.f;
    double acc = 0.0;
    for (int k = 0; k < LK; ++k) acc += (double)W[(size_t)row * Co + base + 67 + k] * env[k];
    return (float)acc;
  };
  // projection chunk: A[q][k] = basis[x index of k][q] split into hi and lo halves
  coff.push_back((int)frags.size());
  for (int part = 0; part < 2; ++part)
    for (int tt = 0; tt < 7; ++tt) {
      Frag fr;
      for (int lane = 0; lane < 64; ++lane) {
        const int q = lane & 31, hf = lane >> 5;
        for (int j = 0; j < 8; ++j) {
          const int col = enc_col(2 + tt, hf, j);
          const float v = (q < F && col >= 0) ? basis_at(col, q) : 0.f;
          const _Float16 hi = (_Float16)v;
          fr[lane * 8 + j] = part == 0 ? hi : (_Float16)(v - (float)hi);
        }
      }
      frags.push_back(fr);
    }
  // second MLP: k-steps per layer (hidden, then the 9 encoding steps), chunks of 16 k-steps
  const int H = 64, NB = 2, L = b.n_hidden;
  for (int l = 0; l < L + 2; ++l) {
    const bool init = l == 0, outl = l == L + 1;
    const int i = l - 1;
    const bool skip = !init && !outl && i != L - 1 && (i % b.skip) == 0;
    const bool hid = !init;
    const bool enc = init || skip;
    const int R = outl ? 3 : H, C = (hid ? H : 0) + (enc ? IN + 2 * F : 0);
    const int Co = (hid ? H : 0) + (enc ? INo + 2 * F : 0);
    const std::vector<float>& W = s->host_w[l];
    const int nrb = outl ? 1 : NB;
    const int ks = (hid ? 2 * NB : 0) + (enc ? 9 : 0);
    const int base = (int)frags.size();
    for (int st = 0; st < ks; ++st)
      for (int ib = 0; ib < nrb; ++ib) {
        Frag fr;
        for (int lane = 0; lane < 64; ++lane) {
          const int row = 32 * ib + (lane & 31), hf = lane >> 5;
          for (int j = 0; j < 8; ++j) {
            int col;
            if (hid && st < 2 * NB)
              col = 32 * (st >> 1) + 16 * (st & 1) + 8 * (j >> 2) + 4 * hf + (j & 3);
            else {
              const int c = enc_col(st - (hid ? 2 * NB : 0), hf, j);
              col = c < 0 ? -1 : (hid ? H : 0) + c;
            }
            const float v = (row < R && col >= 0 && col < C)
                                ? weight_at(W, row, col, hid ? H : 0, Co) : 0.f;
            fr[lane * 8 + j] = (_Float16)v;
          }
        }
        frags.push_back(fr);
      }
    for (int st = 0; st < ks; st += kNerfKC2) coff.push_back(base + st * nrb);
  }
  const size_t nfr = frags.size();
  frags.resize(nfr + 64);
  for (size_t q = nfr; q < frags.size(); ++q) frags[q].fill((_Float16)0.f);
  // biases [first: L1 + 2 layers x 128][second: L2 + 2 layers x 64]; first basis as float4
  std::vector<float> bias(f->host_bias);
  const int boff2 = (int)bias.size();
  bias.insert(bias.end(), s->host_bias.begin(), s->host_bias.end());
  std::vector<float4> basis;
  for (int q = 0; q < a.freqs; ++q)
    basis.push_back(make_float4(f->host_basis[q], f->host_basis[a.freqs + q],
                                f->host_basis[2 * a.freqs + q], 0.f));
  ProgDev& d = out.d;
  std::memset(&d, 0, sizeof(d));
  d.n_mlp = 2;
  d.n_chunks = (int)coff.size();
  d.bias_floats = (int)bias.size();
  d.basis_q = (int)basis.size();
  ProgMlp& p1 = d.mlp[0];
  p1.nb = 4; p1.ne = 3; p1.ob = 3; p1.L = a.n_hidden; p1.skip = a.skip; p1.out = a.out;
  p1.act = a.act; p1.F = a.freqs; p1.bias_off = 0; p1.bstride = a.bias16_stride; p1.basis_off = 0;
  ProgMlp& p2 = d.mlp[1];
  p2.nb = 2; p2.ne = 9; p2.ob = 1; p2.L = b.n_hidden; p2.skip = b.skip; p2.out = b.out;
  p2.act = b.act; p2.F = b.freqs; p2.bias_off = boff2; p2.bstride = b.bias16_stride;
  p2.basis_off = 0;
  const size_t stream_bytes = frags.size() * 1024;
  const size_t o_coff = a256(stream_bytes);
  const size_t o_bias = a256(o_coff + coff.size() * 4);
  const size_t o_basis = a256(o_bias + bias.size() * 4);
  const size_t o_light = a256(o_basis + basis.size() * 16);
  const size_t total = a256(o_light + 16);
  char* buf = nullptr;
  NRT_HIP(hipMalloc((void**)&buf, total));
  out.buf = buf;
  const float unit[4] = {1.f, 0.f, 0.f, 0.f};
  NRT_HIP(hipMemcpy(buf + o_light, unit, sizeof(unit), hipMemcpyHostToDevice));
  out.unit_light = env != nullptr ? reinterpret_cast<const float*>(buf + o_light) : nullptr;
  NRT_HIP(hipMemcpy(buf, frags.data(), stream_bytes, hipMemcpyHostToDevice));
  NRT_HIP(hipMemcpy(buf + o_coff, coff.data(), coff.size() * 4, hipMemcpyHostToDevice));
  NRT_HIP(hipMemcpy(buf + o_bias, bias.data(), bias.size() * 4, hipMemcpyHostToDevice));
  NRT_HIP(hipMemcpy(buf + o_basis, basis.data(), basis.size() * 16, hipMemcpyHostToDevice));
  d.stream = reinterpret_cast<const h8*>(buf);
  d.coff = reinterpret_cast<const int*>(buf + o_coff);
  d.bias = reinterpret_cast<const float*>(buf + o_bias);
  d.basis = reinterpret_cast<const float4*>(buf + o_basis);
  out.ok = true;
  return NRT_OK;
}

}  // namespace nrt

using namespace nrt;

extern "C" {

size_t nrt_nerfle_workspace_bytes(int64_t P, int32_t S, int32_t light_dim) {
  const size_t n = (size_t)std::max<int64_t>(P, 1) * (size_t)std::max(S, 1);
  const size_t in2 = 67 + (size_t)std::max(light_dim, 3);
  return a256(n * 3 * 4) + a256(n * 65 * 4) + a256(n * in2 * 4) + a256(n * 3 * 4);
}

size_t nrt_nerfle_workspace_bytes_for(const nrt_mlp* first, const nrt_mlp* second, int64_t P,
                                       int32_t S, int32_t light_dim, int32_t precision) {
  if (first && second && precision == NRT_FP16 && option(OPT_NERF_FUSED) != 0 && light_dim >= 3 &&
      second->host_dev.in_size == 67 + light_dim && nerf_fusable(first, second)) {
    // fused k_nerfle16: alpha_raw [P S] + rgb_raw [P S, 3]
    const size_t n = (size_t)std::max<int64_t>(P, 1) * (size_t)std::max(S, 1);
    return a256(n * 4) + a256(n * 12);
  }
  return nrt_nerfle_workspace_bytes(P, S, light_dim);
}

int nrt_light_envmap(const nrt_light* l, int32_t bins, float* out, void* stream) {
  if (!l || bins < 1 || !out) { set_error("nrt_light_envmap: bad argument"); return NRT_EINVAL; }
  if (l->host_dev.kind != 1 || l->host_dev.falloff != 0) {
    set_error("nrt_light_envmap: envmap is defined for the pathtracer's PointLights only "
              "(lights.py:81-88; the renderer's PointLights has none)");
    return NRT_EUNSUPPORTED;
  }
  k_light_envmap<><<<dim3(ceil_div64(bins * bins, 64)), dim3(64), 0, (hipStream_t)stream>>>(l->dev, bins, out);
  return check_launch("k_light_envmap");
}

int nrt_nerfle_forward(const nrt_mlp* first, const nrt_mlp* second, const float* rays, int64_t P,
                       const float* ts, int32_t S, const float* light, int32_t light_dim,
                       float* rgb, void* workspace, int precision, void* stream) {
  if (!first || !second || P < 0 || S < 1) { set_error("nrt_nerfle_forward: bad argument"); return NRT_EINVAL; }
  if (P == 0) return NRT_OK;
  if (!rays || !ts || !light || !rgb || !workspace) { set_error("nrt_nerfle_forward: null argument"); return NRT_EINVAL; }
  if (first->desc.in_size != 3 || first->desc.out != 65 || light_dim < 3 ||
      second->desc.in_size != 67 + light_dim || second->desc.out != 3) {
    set_error("nrt_nerfle_forward: expects first 3 -> 65 and second (67 + light_dim) -> 3 "
              "(nerf.py:162-172)");
    return NRT_EINVAL;
  }
  hipStream_t st = (hipStream_t)stream;
  const size_t n = (size_t)P * S;
  char* ws = (char*)workspace;
  if (precision == NRT_FP16 && option(OPT_NERF_FUSED) != 0 &&
      nerf_fusable(first, second)) {
    // NeRF+LE: the envmap (one constant per frame) is folded into the program; the host copy of
    // it decides whether the cached program still holds (one small read-back per call)
    std::vector<float> env;
    if (light_dim != 3) {
      env.resize((size_t)light_dim);
      NRT_HIP(hipMemcpyAsync(env.data(), light, env.size() * 4, hipMemcpyDeviceToHost, st));
      NRT_HIP(hipStreamSynchronize(st));
    }
    if (!second->nerf_prog || second->nerf_first_serial != first->serial ||
        second->nerf_env != env) {
      std::unique_ptr<nrt_prog> pr(new nrt_prog());
      if (int rc = build_nerf_program(first, second, *pr, env.empty() ? nullptr : env.data()))
        return rc;
      second->nerf_prog = std::move(pr);
      second->nerf_first_serial = first->serial;
      second->nerf_env = env;
    }
    const ProgDev& pd = second->nerf_prog->d;
    if (!env.empty()) light = second->nerf_prog->unit_light;
    float* alpha = (float*)ws;
    float* rgb_raw = (float*)(ws + a256(n * 4));
    auto kern = k_nerfle16<kNerfWaves, kNerfTiles>;
    const size_t lds = ring::KEngine<kNerfWaves, kNerfMaxF, kNerfDma>::lds_bytes(pd);
    if (int rc = set_lds(kern, lds)) return rc;
    int dev = 0, cus = 0, per_cu = 0;
    NRT_HIP(hipGetDevice(&dev));
    NRT_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    NRT_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64 * kNerfWaves, lds));
    // persistent grid: every resident block slot (independent blocks on a CU run out of phase,
    // so one block's layer-boundary bubbles are filled by the other's MFMAs)
    const int64_t want = ceil_div64((int64_t)n, 32 * kNerfTiles * kNerfWaves);
    const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(want, (int64_t)std::max(per_cu, 1) * cus));
    ProfScope prof("k_nerfle", st);
    kern<<<dim3(blocks), dim3(64 * kNerfWaves), lds, st>>>(pd, rays, P, ts, S, light, alpha, rgb_raw);
    if (int rc = check_launch("k_nerfle16")) return rc;
    k_nerf_composite_rm<><<<dim3(std::min<int64_t>(ceil_div64(P, 4), 16384)), dim3(256), 0, st>>>(
        alpha, rgb_raw, ts, P, S, rgb);
    return check_launch("k_nerf_composite_rm");
  }
  float* pts = (float*)ws;
  float* f1 = (float*)(ws + a256(n * 12));
  float* x2 = (float*)(ws + a256(n * 12) + a256(n * 260));
  const size_t in2 = 67 + (size_t)light_dim;
  float* c2 = (float*)(ws + a256(n * 12) + a256(n * 260) + a256(n * in2 * 4));
  const int blocks = (int)std::min<int64_t>(ceil_div64((int64_t)n, 256), 4096);
  ProfScope prof("k_nerfle", st);
  k_nerf_points<><<<dim3(blocks), dim3(256), 0, st>>>(rays, P, ts, S, pts);
  if (int rc = check_launch("k_nerf_points")) return rc;
  if (int rc = nrt_mlp_forward(first, pts, nullptr, (int64_t)n, f1, precision, stream)) return rc;
  k_nerf_second_in<><<<dim3(blocks), dim3(256), 0, st>>>(f1, rays, P, S, light, light_dim, x2);
  if (int rc = check_launch("k_nerf_second_in")) return rc;
  if (int rc = nrt_mlp_forward(second, x2, nullptr, (int64_t)n, c2, precision, stream)) return rc;
  k_nerf_composite<><<<dim3(std::min<int64_t>(ceil_div64(P, 256), 4096)), dim3(256), 0, st>>>(
      f1, 65, c2, ts, P, S, rgb);
  return check_launch("k_nerf_composite");
}

size_t nrt_plain_nerf_workspace_bytes(const nrt_mlp* first, const nrt_mlp* second, int64_t P,
                                      int32_t S) {
  if (!first || !second) return 0;
  const size_t n = (size_t)std::max<int64_t>(P, 1) * (size_t)std::max(S, 1);
  const size_t L1 = (size_t)std::max(first->desc.latent, 0);
  const size_t L2 = (size_t)std::max(second->desc.latent, 0);
  const size_t O1 = (size_t)std::max(first->desc.out, 1);
  return a256(n * 3 * 4) + a256(n * L1 * 4) + a256(n * O1 * 4) + a256(n * 2 * 4) +
         a256(n * L2 * 4) + a256(n * 3 * 4);
}

int nrt_plain_nerf_forward(const nrt_mlp* first, const nrt_mlp* second, const float* rays,
                           int64_t P, const float* ts, int32_t S, const float* latent,
                           int64_t rays_per_latent, const float* noise, float* rgb,
                           void* workspace, int precision, void* stream) {
  if (!first || !second || P < 0 || S < 1 || rays_per_latent < 1) {
    set_error("nrt_plain_nerf_forward: bad argument");
    return NRT_EINVAL;
  }
  if (P == 0) return NRT_OK;
  if (!rays || !ts || !latent || !rgb || !workspace) {
    set_error("nrt_plain_nerf_forward: null argument");
    return NRT_EINVAL;
  }
  const int L = first->desc.latent, I = first->desc.out - 1;
  if (first->desc.in_size != 3 || L < 1 || I < 0 || second->desc.in_size != 2 ||
      second->desc.latent != I + L || second->desc.out != 3) {
    set_error("nrt_plain_nerf_forward: expects first 3 (+latent L) -> 1 + I and second 2 "
              "(+latent I + L) -> 3 (nerf.py:23-39)");
    return NRT_EINVAL;
  }
  hipStream_t st = (hipStream_t)stream;
  const size_t n = (size_t)P * S;
  char* ws = (char*)workspace;
  float* pts = (float*)ws;            ws += a256(n * 3 * 4);
  float* lat1 = (float*)ws;           ws += a256(n * L * 4);
  float* f1 = (float*)ws;             ws += a256(n * (1 + I) * 4);
  float* x2 = (float*)ws;             ws += a256(n * 2 * 4);
  float* lat2 = (float*)ws;           ws += a256(n * (I + L) * 4);
  float* c2 = (float*)ws;
  const int blocks = (int)std::min<int64_t>(ceil_div64((int64_t)n, 256), 4096);
  ProfScope prof("k_plain_nerf", st);
  k_plain_first_in<><<<dim3(blocks), dim3(256), 0, st>>>(rays, P, ts, S, latent, L,
                                                          rays_per_latent, pts, lat1);
  if (int rc = check_launch("k_plain_first_in")) return rc;
  if (int rc = nrt_mlp_forward(first, pts, lat1, (int64_t)n, f1, precision, stream)) return rc;
  k_plain_second_in<><<<dim3(blocks), dim3(256), 0, st>>>(f1, I, rays, P, S, latent, L,
                                                           rays_per_latent, x2, lat2);
  if (int rc = check_launch("k_plain_second_in")) return rc;
  if (int rc = nrt_mlp_forward(second, x2, lat2, (int64_t)n, c2, precision, stream)) return rc;
  k_plain_composite<><<<dim3(std::min<int64_t>(ceil_div64(P, 256), 4096)), dim3(256), 0, st>>>(
      f1, 1 + I, noise, c2, ts, P, S, rgb);
  return check_launch("k_plain_composite");
}

}  // extern "C"
