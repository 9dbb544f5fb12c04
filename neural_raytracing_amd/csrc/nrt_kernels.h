// nrt_kernels.h -- gfx950 kernels of the ray-march render path and their launchers.
//
//   k_mlp_forward   SkipConnMLP on a flat batch                 neural_blocks.py:75-86
//   k_sdf_eval      SDF callable on a flat batch                sdfs.py:13, 40-44
//   k_sdf_grad      autograd normal (f32 backward)              sdfs.py:184-197
//   k_intersect     sphere trace + 128-step coarse scan         sdfs.py:111-137, 232-249
//   k_normals       normals + 5*eps offset of the hit rays      sdfs.py:152-158
//   k_frame_wi      shading frame and wi = to_local(-d)         interaction.py:9-41, sdfs.py:158-159
//   k_occlusion     shadow-ray march                            sdfs.py:162-181
//   k_shade_direct  light sample + spatially varying BSDF       integrators.py:173-189, bsdfs.py:515-536
//   k_raygen        NeRF / DTU / FoV primary rays               cameras.py:23-54, 132-192
//   k_composite     NeRFIntegrator alpha + background + tile    integrators.py:249-257, main.py:85-90
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>

#include "nrt_internal.h"
#include "nrt_ring3.h"

namespace nrt {

constexpr int kLdsBytes = 160 * 1024;

// ------------------------------------------------------------------------------------------
// generic MLP evaluation with runtime hidden-size dispatch
// ------------------------------------------------------------------------------------------
template <bool F16, int NB>
__device__ __forceinline__ void mlp_eval(const MlpDev& m, const EncIn& e, float* X, int RS,
                                         float* Y, int ys, float* zs) {
  if (F16) mlp16_forward<NB>(m, e, Y, ys);
  else mlp32_forward<NB>(m, e, X, RS, Y, ys, zs);
  wave_lds_fence();
}

// runtime hidden-size dispatch (one inlined copy per supported width)
template <bool F16>
__device__ __forceinline__ void mlp_eval_any(const MlpDev& m, const EncIn& e, float* X, int RS,
                                          float* Y, int ys) {
  switch (m.nb) {
    case 1: mlp_eval<F16, 1>(m, e, X, RS, Y, ys, nullptr); break;
    case 2: mlp_eval<F16, 2>(m, e, X, RS, Y, ys, nullptr); break;
    case 3: mlp_eval<F16, 3>(m, e, X, RS, Y, ys, nullptr); break;
    case 4: mlp_eval<F16, 4>(m, e, X, RS, Y, ys, nullptr); break;
    default: mlp_eval<F16, 8>(m, e, X, RS, Y, ys, nullptr); break;
  }
}

// per-wave LDS carve: FP32 slab X[32][RS] followed by Y[32][ys]
struct WaveLds {
  float* X;
  float* Y;
};

__device__ __forceinline__ WaveLds wave_lds(float* smem, int per_wave_floats, int RS, bool f16) {
  const int w = threadIdx.x >> 6;
  float* base = smem + (size_t)w * per_wave_floats;
  WaveLds l;
  l.X = base;
  l.Y = f16 ? base : base + 32 * RS;
  return l;
}

__host__ __device__ inline int wave_lds_floats(int RS, int ys, bool f16) {
  return (f16 ? 0 : 32 * RS) + 32 * ys;
}

// ------------------------------------------------------------------------------------------
// SDF
// ------------------------------------------------------------------------------------------
typedef __attribute__((address_space(4))) float ConstF;

template <bool FAST>
__device__ __forceinline__ float spheres_value(const SdfDev& s, float x, float y, float z) {
  // smooth_min(|(I+T_i) p - c_i| - r_i, k)   (sdfs.py:37-43, utils.py:386-387)
  float acc = 0.f;
  // the sphere table is uniform across the wave and read-only: constant address space, so the
  // compiler reads it with scalar loads instead of 64-lane flat loads that drain lgkmcnt
  const ConstF* sp = (const ConstF*)s.spheres;
  for (int i = 0; i < s.n_spheres; ++i, sp += 16) {
    float qx = fmaf(sp[2], z, fmaf(sp[1], y, sp[0] * x)) - sp[9];
    float qy = fmaf(sp[5], z, fmaf(sp[4], y, sp[3] * x)) - sp[10];
    float qz = fmaf(sp[8], z, fmaf(sp[7], y, sp[6] * x)) - sp[11];
    float d = sqrtf(qx * qx + qy * qy + qz * qz) - sp[12];
    acc += FAST ? __expf(-s.k * d) : expf(-s.k * d);
  }
  return -logf(fmaxf(acc, 1e-4f)) / s.k;
}

__device__ __forceinline__ void spheres_grad(const SdfDev& s, float x, float y, float z, float g[3]) {
  float acc = 0.f, gx = 0.f, gy = 0.f, gz = 0.f;
  const ConstF* sp = (const ConstF*)s.spheres;
  for (int i = 0; i < s.n_spheres; ++i, sp += 16) {
    float qx = fmaf(sp[2], z, fmaf(sp[1], y, sp[0] * x)) - sp[9];
    float qy = fmaf(sp[5], z, fmaf(sp[4], y, sp[3] * x)) - sp[10];
    float qz = fmaf(sp[8], z, fmaf(sp[7], y, sp[6] * x)) - sp[11];
    float nq = sqrtf(qx * qx + qy * qy + qz * qz);
    float w = expf(-s.k * (nq - sp[12]));
    acc += w;
    float inv = nq > 0.f ? w / nq : 0.f;
    float ux = qx * inv, uy = qy * inv, uz = qz * inv;  // w * q/|q|
    gx += sp[0] * ux + sp[3] * uy + sp[6] * uz;       // (I+T)^T (w q/|q|)
    gy += sp[1] * ux + sp[4] * uy + sp[7] * uz;
    gz += sp[2] * ux + sp[5] * uy + sp[8] * uz;
  }
  // d/dp -log(max(S,1e-4))/k = (1/S) sum w_i dd_i/dp   (zero where the clamp is active)
  float sc = acc >= 1e-4f ? 1.f / acc : 0.f;
  g[0] = gx * sc; g[1] = gy * sc; g[2] = gz * sc;
}

// SDF value of this lane's point; every lane of the wave must call it (MFMA is wave-wide).
template <bool F16, int NB>
__device__ __forceinline__ float sdf_value(const SdfDev& s, float x, float y, float z,
                                           const WaveLds& l, int RS, float* zs) {
  if (s.kind == 0) return sqrtf(x * x + y * y + z * z) - 1.f;
  float v = 0.f;
  if (s.kind == 2) v = spheres_value<F16>(s, x, y, z);
  if (s.mlp) {
    EncIn e;
    e.x[0] = x; e.x[1] = y; e.x[2] = z; e.x[3] = 0.f;
    e.xg = nullptr; e.lat = nullptr;
    mlp_eval<F16, NB>(*s.mlp, e, l.X, RS, l.Y, 1, zs);
    float m = l.Y[lane_id() & 31];
    wave_lds_fence();
    v = (s.kind == 2) ? v + m : m;
  }
  return v;
}

// d sdf / dp (FP32 slab path), every lane of the wave must call it
template <int NB>
__device__ __forceinline__ void sdf_gradient(const SdfDev& s, float x, float y, float z,
                                             const WaveLds& l, int RS, float* zs, float g[3]) {
  g[0] = g[1] = g[2] = 0.f;
  if (s.kind == 0) {
    float n = sqrtf(x * x + y * y + z * z);
    if (n > 0.f) { g[0] = x / n; g[1] = y / n; g[2] = z / n; }
    return;
  }
  if (s.kind == 2) spheres_grad(s, x, y, z, g);
  if (s.mlp) {
    EncIn e;
    e.x[0] = x; e.x[1] = y; e.x[2] = z; e.x[3] = 0.f;
    e.xg = nullptr; e.lat = nullptr;
    float gm[3];
    mlp32_forward<NB>(*s.mlp, e, l.X, RS, l.Y, 1, zs);
    mlp32_backward_out0<NB>(*s.mlp, e, l.X, RS, zs, gm);
    g[0] += gm[0]; g[1] += gm[1]; g[2] += gm[2];
  }
}

// ------------------------------------------------------------------------------------------
// flat-batch kernels (one wave = 32 rows)
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ int64_t wave_global() {
  return (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
}

template <bool F16, int NB>
__global__ void __launch_bounds__(256, F16 ? 2 : 1) k_mlp_forward(const MlpDev* __restrict__ mp,
                                                      const float* __restrict__ x,
                                                      const float* __restrict__ lat, int64_t M,
                                                      float* __restrict__ y, int RS, int per_wave) {
  extern __shared__ float smem[];
  const MlpDev& m = *mp;
  WaveLds l = wave_lds(smem, per_wave, RS, F16);
  const int lane = lane_id(), r = lane & 31;
  const int64_t row0 = wave_global() * 32;
  if (row0 >= M) return;  // whole wave exits together
  const int64_t row = row0 + r;
  const bool valid = row < M;
  const int64_t rr = valid ? row : M - 1;
  EncIn e;
  const int in = m.in_size;
  if (in <= 4) {
    for (int i = 0; i < 4; ++i) e.x[i] = (i < in) ? x[rr * in + i] : 0.f;
    e.xg = nullptr;
  } else {
    e.x[0] = e.x[1] = e.x[2] = e.x[3] = 0.f;
    e.xg = x + rr * in;
  }
  e.lat = (lat && m.latent > 0) ? lat + rr * m.latent : nullptr;
  mlp_eval<F16, NB>(m, e, l.X, RS, l.Y, m.out, nullptr);
  if (valid)
    for (int o = (lane >> 5); o < m.out; o += 2) y[row * m.out + o] = l.Y[r * m.out + o];
}

template <bool F16, int NB>
__global__ void __launch_bounds__(256, F16 ? 2 : 1) k_sdf_eval(const SdfDev* __restrict__ sp,
                                                   const float* __restrict__ p, int64_t M,
                                                   float* __restrict__ out, int RS, int per_wave) {
  extern __shared__ float smem[];
  const SdfDev& s = *sp;
  WaveLds l = wave_lds(smem, per_wave, RS, F16);
  const int lane = lane_id(), r = lane & 31;
  const int64_t row0 = wave_global() * 32;
  if (row0 >= M) return;
  const int64_t row = row0 + r;
  const int64_t rr = row < M ? row : M - 1;
  float v = sdf_value<F16, NB>(s, p[rr * 3], p[rr * 3 + 1], p[rr * 3 + 2], l, RS, nullptr);
  if (row < M && lane < 32) out[row] = v;
}

// gradient over a flat batch (optionally through an index list with a device-side count);
// grid-stride over waves with a per-resident-wave pre-activation scratch
template <int NB>
__global__ void __launch_bounds__(256) k_sdf_grad(
    const SdfDev* __restrict__ sp, const float* __restrict__ p, const int32_t* __restrict__ index,
    const int32_t* __restrict__ count, int64_t M, float* __restrict__ grad,
    float* __restrict__ n_out, float* __restrict__ p_io, float offset_eps,
    float* __restrict__ zscr, int RS, int per_wave, int64_t zs_per_wave) {
  extern __shared__ float smem[];
  const SdfDev& s = *sp;
  WaveLds l = wave_lds(smem, per_wave, RS, false);
  const int lane = lane_id(), r = lane & 31;
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
  const int64_t gw = wave_global();
  float* zs = zscr ? zscr + gw * zs_per_wave : nullptr;
  const int64_t total = count ? (int64_t)(*count) : M;
  for (int64_t w = gw; w * 32 < total; w += nw) {
    const int64_t i = w * 32 + r;
    const bool valid = i < total;
    const int64_t ii = valid ? i : total - 1;
    const int64_t idx = index ? (int64_t)index[ii] : ii;
    const float* pp = p_io ? p_io : p;
    const float x = pp[idx * 3], y = pp[idx * 3 + 1], z = pp[idx * 3 + 2];
    float g[3];
    sdf_gradient<NB>(s, x, y, z, l, RS, zs, g);
    if (valid && lane < 32) {
      if (grad) { grad[idx * 3] = g[0]; grad[idx * 3 + 1] = g[1]; grad[idx * 3 + 2] = g[2]; }
      if (n_out) {
        // normals[hit] = normalize(raw, eps=1e-6); p[hit] += normals * eps * 5  (sdfs.py:156-157)
        float nx = g[0], ny = g[1], nz = g[2];
        normalize3(nx, ny, nz, 1e-6f);
        n_out[idx * 3] = nx; n_out[idx * 3 + 1] = ny; n_out[idx * 3 + 2] = nz;
        if (p_io) {
          p_io[idx * 3] = x + (nx * offset_eps) * 5.f;
          p_io[idx * 3 + 1] = y + (ny * offset_eps) * 5.f;
          p_io[idx * 3 + 2] = z + (nz * offset_eps) * 5.f;
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// sphere tracing + coarse scan: one fused loop with a single SDF call site
// ------------------------------------------------------------------------------------------
struct MarchArgs {
  int max_steps;
  float eps;
  float max_t;
  int primary;
  double step;  // scan step = scan_max_t / 128 (python float)
  int32_t* scan_idx;  // optional [P] coarse-scan argmin output
  unsigned long long* evals = nullptr;  // profiling: ray-evaluations executed (nrt_profile_evals)
  // batched tiles (nrt_march_params.scan_max_t_groups): ray r scans with scan_max_t of group
  // r / group_rays (one random.random() draw per tile, sdfs.py:236); nullptr = `step` for all
  const double* groups = nullptr;
  int64_t group_rays = 1;
  // FP16 ring march: byte offset of an LDS copy of the SphereSDF table (0 = read it from the
  // constant cache); set by ring_march when the table fits beside the weight ring
  int lds_spheres = 0;
  // ring marches: deal rays to waves by XCD lines (OwnedRays; option "xcd_lines")
  int xcd_lines = 0;
  // NRT_MIXED (the FP16 march refined where FP16 cannot decide, nrt_ring_mixed.hip):
  //  * FP16 march: a step whose value lies within refine_d * (1 + i/16) of eps, or whose t lies that
  //    close to max_t, marks the ray -- amb[ray] = (i << 32 | t bits), the first such step's state
  //    (the march goes on; amb stays all-ones for a ray FP16 decided clearly);
  //  * FP16 scan: keys2[ray] = the runner-up key beside keys[ray] (top two over the 129 samples,
  //    merged lock-free across segments), so sdf(best) can re-evaluate both when they lie within
  //    refine_s of each other;
  //  * refinement launches: job k's ray is list[k] for k < *count, and a march starts from the
  //    state in start[ray] instead of (t = 0, i = 0);
  //  * sdf(best) with keys2: both candidates' values merge into kbest[ray] (atomic min of the key)
  float refine_d = 0.f, refine_s = 0.f;
  int drift_model = 0;  // 1: the flag bound follows a per-ray drift estimate (option "mixed_drift")
  float zone = 0.f;     // > 0: flagged rays resume at the first step within `zone` of a surface
  unsigned long long* amb = nullptr;
  unsigned long long* keys2 = nullptr;
  unsigned long long* kbest = nullptr;
  const unsigned long long* start = nullptr;
  const int32_t* list = nullptr;
  const int32_t* count = nullptr;
  // shadow march (march_body mode 3): each ray's distance to the light; `count` (device) bounds
  // the compacted ray list
  const float* occ_max_t = nullptr;
  // ring marches: one launch-wide job queue instead of per-wave lists (option "march_queue"):
  // a zeroed device counter; waves take kQueueChunk jobs at a time from the launch's whole list
  // ([march of every ray][scan segment s of every ray, s = 0 .. 7]); nullptr = per-wave lists
  unsigned int* queue = nullptr;
  // launch-queue march (mode 0, packed t): byte offset in the block's LDS of the per-wave line
  // stages (LineStage, kStageBytes a wave); 0 = every finished ray stores its own words
  int stage = 0;
};
#ifndef NRT_QUEUE_CHUNK
#define NRT_QUEUE_CHUNK 16
#endif
#ifndef NRT_QUEUE_TAIL
#define NRT_QUEUE_TAIL 16
#endif
constexpr int kQueueChunk = NRT_QUEUE_CHUNK;  // 32 measured slower (round 5)
constexpr int kQueueTail = NRT_QUEUE_TAIL;    // rays per wave of the grid whose scans are segmented

// ------------------------------------------------------------------------------------------
// Line staging of the march's per-ray words (MarchArgs::stage).  Under the launch queue a wave
// takes 16 consecutive jobs at a time, so the packed t of 16 consecutive rays (one 64-byte line)
// and, for whole scans, their 64-bit keys (one 128-byte line) finish in one wave -- but at
// different times, each as a lane-scattered 4- or 8-byte store (PMC: 45 MB of writes a 800^2
// launch for ~8 MB of words).  Here a finished ray's word goes to a per-wave LDS slot of its line
// instead; a slot whose line is complete is written by 16 lanes in one coalesced store, and a
// slot that must make room (more than kStageSlots lines in flight) or is still open when the wave
// ends is written with the lanes of its finished rays only.  Every ray's word is written exactly
// once either way: the same bits as the per-ray stores.  The slot table (line, finished-ray mask)
// lives in lanes 0 .. kStageSlots-1 of two VGPRs; all control is wave-uniform.
constexpr int kStageSlots = 8;
constexpr int kStageBytes = kStageSlots * 16 * (4 + 8);  // t words, then key words
template <class W>
struct LineStage {
  W* data;          // [kStageSlots][16] in LDS
  W* out;           // global: word of ray r at out[r]
  int64_t limit;    // rays [0, limit) are staged here (a line past it completes early)
  int tag = -1;     // lane q < kStageSlots: line held by slot q (-1 free)
  uint32_t msk = 0; // lane q: finished rays of that line
  int lane;
  __device__ __forceinline__ void init(W* d, W* o, int64_t lim, int ln) {
    data = d; out = o; limit = lim; lane = ln;
  }
  __device__ __forceinline__ void flush(int q, int line, uint32_t m) {
    if (lane < 16 && ((m >> lane) & 1u)) out[(int64_t)line * 16 + lane] = data[q * 16 + lane];
    if (lane == q) { tag = -1; msk = 0u; }
  }
  // lanes in `fin` (wave-uniform mask) finished their ray `ray` with word `v`
  __device__ __forceinline__ void put(uint64_t fin, int64_t ray, W v) {
    while (fin) {
      const int l = __builtin_ctzll(fin);
      fin &= fin - 1;
      const int64_t r = ((int64_t)__builtin_amdgcn_readlane((int)(ray >> 32), l) << 32) |
                        (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)ray, l);
      const int line = (int)(r >> 4), off = (int)(r & 15);
      const uint64_t own = __ballot(lane < kStageSlots && tag == line);
      int q;
      if (own) {
        q = __builtin_ctzll(own);
      } else {
        const uint64_t fr = __ballot(lane < kStageSlots && tag < 0);
        if (fr) {
          q = __builtin_ctzll(fr);
        } else {  // evict slot 0's line (its finished rays only)
          q = 0;
          flush(0, __builtin_amdgcn_readlane(tag, 0), (uint32_t)__builtin_amdgcn_readlane((int)msk, 0));
        }
        if (lane == q) { tag = line; msk = 0u; }
      }
      asm volatile("" ::: "memory");
      if (lane == l) data[q * 16 + off] = v;
      if (lane == q) msk |= 1u << off;
      const uint32_t m = (uint32_t)__builtin_amdgcn_readlane((int)msk, q);
      const int64_t n = limit - (int64_t)line * 16;
      const uint32_t full = n >= 16 ? 0xffffu : ((1u << (int)n) - 1u);
      asm volatile("" ::: "memory");
      if (m == full) flush(q, line, m);
      asm volatile("" ::: "memory");
    }
  }
  __device__ __forceinline__ void drain() {
#pragma unroll
    for (int q = 0; q < kStageSlots; ++q) {
      const int line = __builtin_amdgcn_readlane(tag, q);
      if (line >= 0) flush(q, line, (uint32_t)__builtin_amdgcn_readlane((int)msk, q));
    }
  }
};

// the scan step of `ray`: max_t / 128 in double, as the reference's python float (sdfs.py:237)
__device__ __forceinline__ double scan_step_of(const MarchArgs& a, int64_t ray) {
  return a.groups ? a.groups[ray / a.group_rays] / 128.0 : a.step;
}

template <bool F16, int NB>
__global__ void __launch_bounds__(256, F16 ? 2 : 1) k_intersect(
    const SdfDev* __restrict__ sp, const float* __restrict__ rays, int64_t P, MarchArgs a,
    float* __restrict__ t_out, uint8_t* __restrict__ hit_out, float* __restrict__ p_out,
    float* __restrict__ n_out, float* __restrict__ rawn_out, float* __restrict__ thr_out,
    int32_t* __restrict__ hit_idx, int32_t* __restrict__ hit_count, int RS, int per_wave) {
  extern __shared__ float smem[];
  const SdfDev& s = *sp;
  WaveLds l = wave_lds(smem, per_wave, RS, F16);
  const int lane = lane_id(), r = lane & 31;
  const int64_t ray0 = wave_global() * 32;
  if (ray0 >= P) return;
  const int64_t ray = ray0 + r;
  const bool valid = ray < P;
  const int64_t rr = valid ? ray : P - 1;
  const float ox = rays[rr * 6], oy = rays[rr * 6 + 1], oz = rays[rr * 6 + 2];
  const float dx = rays[rr * 6 + 3], dy = rays[rr * 6 + 4], dz = rays[rr * 6 + 5];
  const double step = scan_step_of(a, rr);

  // Phase 1 (sdfs.py:119-131): sphere tracing.  The reference evaluates every ray at every step;
  // a ray that stopped marching never changes again, so the wave leaves the phase as soon as none
  // of its rays is marching (identical results, fewer evaluations).
  // Phase 2 (sdfs.py:238-249): sdf(o), 128 samples at fl32(step*(i+1)), then sdf(best_pos).
  float t = 0.f;
  bool live = valid, hit = false;
  int i = 0;            // march step
  int j = -2;           // scan sample: -1 = origin, 0..127 = samples, 128 = best point
  float best = 0.f, thr = 0.f;
  int idx = 0;
  for (;;) {
    if (j == -2) {
      if (i >= a.max_steps || !wave_any(live)) {
        if (!a.primary) break;
        j = -1;
      } else {
        live = live && (t < a.max_t);
      }
    }
    float px, py, pz;
    if (j == -2) {
      px = __fadd_rn(ox, __fmul_rn(dx, t));
      py = __fadd_rn(oy, __fmul_rn(dy, t));
      pz = __fadd_rn(oz, __fmul_rn(dz, t));
    } else if (j == -1) {
      px = ox; py = oy; pz = oz;
    } else {
      float ts = (j < 128) ? (float)(step * (double)(j + 1)) : __fmul_rn((float)idx, (float)step);
      px = __fadd_rn(ox, __fmul_rn(ts, dx));
      py = __fadd_rn(oy, __fmul_rn(ts, dy));
      pz = __fadd_rn(oz, __fmul_rn(ts, dz));
    }
    const float d = sdf_value<F16, NB>(s, px, py, pz, l, RS, nullptr);
    if (j == -2) {
      const bool now = live && (d <= a.eps);
      hit = hit || now;
      live = live && !now;
      if (live) t = t + d;
      ++i;
    } else if (j == -1) {
      best = d;
      ++j;
    } else if (j < 128) {
      if (d < best) idx = j + 1;
      best = fminf(best, d);
      ++j;
    } else {
      thr = -1000.f * d;
      break;
    }
  }
  if (valid && lane < 32) {
    t_out[ray] = t;
    hit_out[ray] = hit ? 1 : 0;
    p_out[ray * 3] = __fadd_rn(ox, __fmul_rn(t, dx));
    p_out[ray * 3 + 1] = __fadd_rn(oy, __fmul_rn(t, dy));
    p_out[ray * 3 + 2] = __fadd_rn(oz, __fmul_rn(t, dz));
    n_out[ray * 3] = 0.f; n_out[ray * 3 + 1] = 0.f; n_out[ray * 3 + 2] = 0.f;
    if (rawn_out) { rawn_out[ray * 3] = 0.f; rawn_out[ray * 3 + 1] = 0.f; rawn_out[ray * 3 + 2] = 0.f; }
    if (a.primary) thr_out[ray] = thr;
    if (a.primary && a.scan_idx) a.scan_idx[ray] = idx;
  }
  if (hit_idx) {
    // wave-aggregated append of the hit rays (order is irrelevant downstream)
    const uint64_t m = __ballot(valid && hit && lane < 32);
    const int cnt = __popcll(m);
    int base = 0;
    if (lane == 0 && cnt) base = atomicAdd(hit_count, cnt);
    base = __shfl(base, 0);
    if (valid && hit && lane < 32) {
      const int off = __popcll(m & ((1ull << lane) - 1ull));
      hit_idx[base + off] = (int32_t)ray;
    }
  }
}

// FP16 march + coarse scan on the ring engine, load-balanced per lane.
//
// The reference evaluates every ray at every one of max_steps march steps and at the 130 scan
// points (sdfs.py:119-131, 232-249); only the march is data-dependent (hit / t >= max_t end it
// early), the scan is a fixed walk that does not depend on the march.  A wave therefore works
// through a private job list instead of a fixed 32-ray tile: the grid is persistent (one block
// per resident slot), wave w owns a strided sample of the image in chunks of consecutive rays
// (OwnedRays: every wave gets a similar mix of short hit marches and long miss marches), and its
// list is
//     [march of each owned ray] [scan segment 0 of each ray] ... [scan segment NSEG-1 ...]
// A lane whose job has ended takes the next list entry (ballot + prefix count on a wave-uniform
// cursor, no atomics), so lanes never idle on a finished ray; the list ends with short
// fixed-length segments, so lanes run out of work within one segment of each other.
// A segment keeps the running (min, first index) exactly as the reference loop does and merges
// it into the ray's 64-bit key [ordered min | index] with an atomic min: the smallest key is the
// smallest value and, among equal values, the first sample -- the reference's strict-< update.
// A second launch (mode 1) evaluates sdf(best) for the throughput.  Lanes l and l + 32 carry the
// same ray (the MFMA K halves) and run identical state machines.
constexpr int kScanSegs = 8;  // sample j in [0, 128]: segment 0 = [0, 16], segment q = [16q+1, 16q+16]
#ifndef NRT_SCAN_SPLIT
#define NRT_SCAN_SPLIT 64
#endif
constexpr int kScanSplit = NRT_SCAN_SPLIT;  // rays per wave scanned in segments (-1: all)

__device__ __forceinline__ uint64_t scan_key(float v, int idx) {
  uint32_t b = __float_as_uint(v + 0.f);  // -0 -> +0: equal values tie, as under the reference's <
  b = (b & 0x80000000u) ? ~b : (b | 0x80000000u);
  return ((uint64_t)b << 32) | (uint32_t)idx;
}
// the value of a scan key (inverse of scan_key's order-preserving map; all-ones -> NaN)
__device__ __forceinline__ float scan_key_value(uint64_t k) {
  uint32_t b = (uint32_t)(k >> 32);
  b = (b & 0x80000000u) ? (b & 0x7fffffffu) : ~b;
  return __uint_as_float(b);
}

// Rays owned by wave w of nw (the strided deal, kRayChunk = 1: ray w, w + nw, ...): every wave
// owns the same number of rays to within one and a sample of the whole image, so its mix of
// short (hit) and long (miss) marches stays near the frame's.  With kRayChunk > 1, whole rounds
// of kRayChunk consecutive rays (measured 7 % slower: chunk-correlated march lengths unbalance
// the waves).
//
// XCD lines (MarchArgs::xcd_lines): the same deal within each XCD.  The image is cut into lines
// of kLineRays consecutive rays (128 B of t, a line of p / n / keys between them); line k belongs
// to XCD group k % X, and a group's rays are dealt one at a time to the waves of its blocks
// (workgroups are dispatched round-robin over the 8 XCDs: block b runs on XCD b % 8).  The 32
// lane-scattered stores of a line then come from waves of one XCD and could merge in its L2 instead
// of reaching HBM as partial lines from up to 8 L2s.  Measured (PMC, 800^2 FP32 frame): HBM writes
// 131 -> 158 MB per k_march32 launch -- worse, so off by default (the lines are written over the
// whole launch and leave the L2 between stores anyway); the fix that works is fewer scattered
// bytes (k_march_finish).
#ifndef NRT_RAY_CHUNK
#define NRT_RAY_CHUNK 1  // 32 measured 7 % slower (chunk-correlated march lengths unbalance the waves)
#endif
constexpr int64_t kRayChunk = NRT_RAY_CHUNK;
constexpr int64_t kLineRays = 32;
constexpr int kXcds = 8;  // MI355X: 8 XCDs, each with its own L2
struct OwnedRays {
  int64_t nw, w, full, R;  // full = rays of this wave in whole chunk rounds
  // XCD lines: group g of X, the group's rays Rg, its waves nwg, this wave's index v in it
  bool lines = false;
  int64_t X = 1, g = 0, Rg = 0, nwg = 1, v = 0;
  __device__ __forceinline__ OwnedRays(int64_t P, int64_t nw_, int64_t w_) : nw(nw_), w(w_) {
    const int64_t rounds = P / (nw * kRayChunk);
    full = rounds * kRayChunk;
    const int64_t rem = P - rounds * nw * kRayChunk;
    R = full + (w < rem ? (rem - 1 - w) / nw + 1 : 0);
  }
  // wv waves per block; blocks = nw / wv
  __device__ __forceinline__ OwnedRays(int64_t P, int64_t nw_, int64_t w_, int wv, bool xcd)
      : OwnedRays(P, nw_, w_) {
    if (!xcd) return;
    lines = true;
    const int64_t blocks = nw / wv, b = w / wv;
    X = blocks < kXcds ? blocks : kXcds;
    g = b % X;
    const int64_t gb = (blocks - g + X - 1) / X;  // blocks of the group
    nwg = gb * wv;
    v = (b / X) * wv + (w % wv);
    const int64_t NL = (P + kLineRays - 1) / kLineRays;  // lines
    const int64_t ng = NL > g ? (NL - g + X - 1) / X : 0;  // lines of the group
    Rg = ng * kLineRays;
    if (ng > 0 && (NL - 1) % X == g) Rg -= NL * kLineRays - P;  // the short last line
    R = v < Rg ? (Rg - 1 - v) / nwg + 1 : 0;
  }
  __device__ __forceinline__ int64_t ray(int64_t k) const {
    if (lines) {
      const int64_t q = v + k * nwg;  // the group's q-th ray
      return (g + X * (q / kLineRays)) * kLineRays + (q % kLineRays);
    }
    if (k < full) return ((k / kRayChunk) * nw + w) * kRayChunk + (k % kRayChunk);
    return (full * nw) + w + (k - full) * nw;
  }
};

// The SDF evaluator of a ring march: FP16 (32-ray tiles, ring::eval, fast sphere exp) or FP32
// (16-ray tiles, ring32::eval; softplus_exact -- a few ulp of torch's log1pf(expf), see nrt_device.h).  RPW rays per wave; lane l serves
// ray l & (RPW - 1) and the other lanes of that ray mirror its state.
template <int NB, int NE, int WV, bool FOLD>
struct RingPol16 {
  static constexpr int RPW = 32, WAVES = WV;
  using Eng = ring::Engine<NB, NE, WV>;
  __device__ __forceinline__ static void init(Eng& E, const SdfDev& s, const MlpDev& m, char* lds,
                                              const MarchArgs& a) {
    E.init(m, lds);
    E.lspheres = nullptr;
    if (s.kind == 2 && a.lds_spheres > 0) {
      float4* ls = reinterpret_cast<float4*>(lds + a.lds_spheres);
      ring::build_sphere_pairs(s, ls);  // the pair layout of spheres_value_pairs
      __syncthreads();
      E.lspheres = ls;
    }
  }
  __device__ __forceinline__ static float sdf(Eng& E, const SdfDev& s, const MlpDev& m, float x, float y, float z) {
    float d = 0.f;
    if (s.kind == 2)
      d = E.lspheres ? ring::spheres_value_pairs(s, E.lspheres, E.lane, x, y, z)
                     : spheres_value<true>(s, x, y, z);
    return d + ring::eval<NB, NE, WV, FOLD, 8, 3>(E, m, x, y, z);
  }
  __device__ __forceinline__ static void finish(Eng&) {}
  static constexpr bool kGuard = false;
  __device__ __forceinline__ static bool retry(Eng&, bool, float) { return false; }
};
template <int KH, int KE, int WV, int ACT>
struct RingPol32 {
  static constexpr int RPW = 16, WAVES = WV;
  using Eng = ring32::Engine<KH, KE, WV>;
  __device__ __forceinline__ static void init(Eng& E, const SdfDev& s, const MlpDev& m, char* lds,
                                              const MarchArgs&) {
    E.init(m, s, lds, ring32::kSub * Eng::QE);
  }
  __device__ __forceinline__ static float sdf(Eng& E, const SdfDev& s, const MlpDev& m, float x, float y, float z) {
    const float d = (s.kind == 2) ? ring32::spheres_value16_pairs(s, E.lspheres, E.lane, x, y, z) : 0.f;
    return d + ring32::eval<KH, KE, WV, ACT>(E, m, x, y, z);
  }
  // forward-mode column value (ring32::eval TAN): 4 rays x (value, d/dx, d/dy, d/dz)
  __device__ __forceinline__ static float tan(Eng& E, const MlpDev& m, float x, float y, float z) {
    return ring32::eval<KH, KE, WV, ACT, true>(E, m, x, y, z);
  }
  __device__ __forceinline__ static void finish(Eng& E) { E.drain(); }
  static constexpr bool kGuard = false;
  __device__ __forceinline__ static bool retry(Eng&, bool, float) { return false; }
};

// FP32-accurate evaluation on FP16 matrix cores (nrt_ring3.h, the "fp32-split" precision):
// 16-ray tiles like RingPol32 (softplus_exact: a few ulp of torch's), sphere blobs as in ring32
template <int KH, int KQ, int WV, int ACT>
struct RingPol3 {
  static constexpr int RPW = 16, WAVES = WV;
  using Eng = ring3::Engine<KH, KQ, WV>;
  __device__ __forceinline__ static void init(Eng& E, const SdfDev& s, const MlpDev& m, char* lds,
                                              const MarchArgs&) {
    E.init(m, s, lds, 4 * KQ, 4 * KQ);  // chunks 0 and 1: the init layer's
  }
  // the f16 range guard (nrt_ring3.h): the wave's guarded flag picks the variant (a scalar
  // branch: both variants pass the same block barriers)
  __device__ __forceinline__ static float sdf(Eng& E, const SdfDev& s, const MlpDev& m, float x, float y, float z) {
    const float d = (s.kind == 2) ? ring32::spheres_value16(s, E.lspheres, E.lane, x, y, z) : 0.f;
#ifndef NRT_NOGUARD_EXP  // timing experiment only (tools/exp_variants.py): results need the guard
    if (__builtin_amdgcn_readfirstlane((int)E.guarded))
      return d + ring3::eval<KH, KQ, WV, ACT, false, true>(E, m, x, y, z);
#endif
    return d + ring3::eval<KH, KQ, WV, ACT>(E, m, x, y, z);
  }
  __device__ __forceinline__ static float tan(Eng& E, const MlpDev& m, float x, float y, float z) {
    if (__builtin_amdgcn_readfirstlane((int)E.guarded))
      return ring3::eval<KH, KQ, WV, ACT, true, true>(E, m, x, y, z);
    return ring3::eval<KH, KQ, WV, ACT, true>(E, m, x, y, z);
  }
  __device__ __forceinline__ static void finish(Eng& E) { E.drain(); }
  static constexpr bool kGuard = true;
  __device__ __forceinline__ static bool retry(Eng& E, bool active, float v) {
    return ring3::retry(E, active, v);
  }
};

// MX: the NRT_MIXED variant (MarchArgs' refine fields live); the plain kernels compile without
// any of it
template <class Pol, int MODE, bool MX = false>
__device__ __forceinline__ void march_body(
    const SdfDev s, const MlpDev m, const float* __restrict__ rays, int64_t P, MarchArgs a,
    float* __restrict__ t_out, uint8_t* __restrict__ hit_out, float* __restrict__ p_out,
    float* __restrict__ n_out, float* __restrict__ rawn_out, float* __restrict__ thr_out,
    unsigned long long* __restrict__ keys) {
  extern __shared__ __attribute__((aligned(16))) char smem_c[];
  constexpr int mode = MODE;
  constexpr int RPW = Pol::RPW, WV = Pol::WAVES;
  constexpr uint32_t kRayMask = RPW == 32 ? 0xffffffffu : ((1u << RPW) - 1u);
  const int lane = lane_id(), r = lane & (RPW - 1);
  const int64_t nw = (int64_t)gridDim.x * WV;
  const int64_t w = (int64_t)blockIdx.x * WV + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // a refinement launch works through the first *count entries of a ray list
  const int64_t Pe =
      ((MX || MODE == 3) && a.count)
          ? (int64_t)__builtin_amdgcn_readfirstlane(*(const NRT_GLOBAL int32_t*)a.count)
          : P;
  const OwnedRays own(Pe, nw, w, WV, a.xcd_lines != 0);
  // launch-wide queue (MarchArgs::queue): the list is every ray's, job k's ray is k, and every
  // scan runs as segments; otherwise this wave's own rays
  const bool dyn = a.queue != nullptr;
  const int64_t R = dyn ? Pe : own.R;  // rays of this wave's list
  const bool scan = mode == 0 && a.primary;
  // scan jobs: the whole 129-point scan of each of the first R - T rays (one plain key store),
  // then kScanSegs segments of each of the last T rays (atomic min merge) to level the tail; the
  // launch-wide queue segments the last 16 rays per wave of the grid (every ray segmented took
  // HBM traffic per 800^2 launch from 178 to 325 MB: 8 key atomics per ray)
  const int64_t tq = kQueueTail * nw;
  const int64_t T = dyn ? (R < tq ? R : tq)
                        : (kScanSplit < 0 ? R : (R < kScanSplit ? R : (int64_t)kScanSplit));
  // sdf(best) with a runner-up key: a second job per ray re-evaluates the runner-up where the
  // FP16 scan could not order the two (skipped elsewhere)
  const bool alt = MX && mode == 1 && a.keys2 != nullptr;
  const int64_t J = mode == 0 ? (scan ? R + (R - T) + T * kScanSegs : R) : (alt ? 2 * R : R);
  const uint32_t lt = (1u << r) - 1u;
  typename Pol::Eng E;
  Pol::init(E, s, m, smem_c, a);
  // lane state: kind -1 = wants a job, -2 = list exhausted, 0 march, 1 scan segment, 2 sdf(best)
  int kind = -1;
  int64_t ray = 0;
  float ox = 0.f, oy = 0.f, oz = 0.f, dx = 0.f, dy = 0.f, dz = 0.f;
  float t = 0.f, best = 0.f, second = 0.f;
  double step = a.step;  // this lane's scan step (per tile group when batched)
  int i = 0, j = 0, jend = 0, idx = 0, idx2 = 0;
  bool ended = false, hit = false, whole = false;
  unsigned long long ambs = ~0ull;  // NRT_MIXED: the first undecidable step's (i, t), or none
  float drift = 0.f, dprev = 1.f;   // NRT_MIXED: t's drift bound (units of the FP16 error)
  float mt = 0.f;                   // mode 3: the ray's distance to the light
  unsigned long long cps = ~0ull;   // NRT_MIXED: the zone checkpoint (MarchArgs::zone)
  int64_t cursor = 0;  // wave-uniform
  int64_t cend = 0;    // queue: end of the wave's current chunk [cursor, cend)
  bool dry = false;    // queue: drained
  // line staging (MarchArgs::stage): only the launch queue's plain march (job k's ray is k)
#ifdef NRT_NOSTAGE_EXP  // timing experiment only (tools/exp_variants.py): the staging compiled out
  constexpr bool stg = false;
#else
  const bool stg = !MX && mode == 0 && dyn && a.stage != 0 && p_out == nullptr;
#endif
  LineStage<float> st_t;
  LineStage<unsigned long long> st_k;
  if (stg) {
    char* base = smem_c + a.stage + (int)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) * kStageBytes;
    st_t.init(reinterpret_cast<float*>(base), t_out, Pe, lane);
    // whole scans are the rays [0, R - T); the segmented tail merges by atomic min in place
    st_k.init(reinterpret_cast<unsigned long long*>(base + kStageSlots * 16 * 4), keys, R - T, lane);
  }
  for (;;) {
    // retire ended jobs and hand out list entries until every lane has an evaluation to do
    for (;;) {
      bool fin_t = false, fin_k = false;  // line staging: this lane's ray finished its word
      if (mode == 3 && kind == 0) {
        // intersect_test (sdfs.py:162-181): visible = t >= max_t | live after max_steps.  t only
        // grows, so a march past the light is decided (visible) and stops there
        if (ended || i >= a.max_steps || t >= mt) {
          if (lane < RPW) hit_out[ray] = (t >= mt || !hit) ? 1 : 0;
          kind = -1;
        }
      } else if (kind == 0) {
        // sdfs.py:119-131: a march ends on a hit, when t leaves [0, max_t) or after max_steps
        if (ended || !(t < a.max_t) || i >= a.max_steps) {
          if (MX && lane < RPW && a.amb && ambs != ~0ull) a.amb[ray] = ambs;
          if (lane < RPW) {
            if (p_out) {
              t_out[ray] = t;
              hit_out[ray] = hit ? 1 : 0;
              p_out[ray * 3] = __fadd_rn(ox, __fmul_rn(t, dx));
              p_out[ray * 3 + 1] = __fadd_rn(oy, __fmul_rn(t, dy));
              p_out[ray * 3 + 2] = __fadd_rn(oz, __fmul_rn(t, dz));
              n_out[ray * 3] = 0.f; n_out[ray * 3 + 1] = 0.f; n_out[ray * 3 + 2] = 0.f;
              if (rawn_out) { rawn_out[ray * 3] = 0.f; rawn_out[ray * 3 + 1] = 0.f; rawn_out[ray * 3 + 2] = 0.f; }
            } else {
              // packed: t >= 0 always (it only grows by d > eps) and a hit's t is finite (a NaN t
              // ends the march as a miss), so the hit flag rides in the sign bit; k_march_finish unpacks it and writes p / n / hit with coalesced stores
              // (this lane-scattered 4-byte store is the march's only per-ray output)
              if (stg) fin_t = true;
              else t_out[ray] = hit ? -t : t;
            }
          }
          kind = -1;
        }
      } else if (kind == 1) {
        if (j > jend) {
          // a whole scan stores its key; a segment merges into it (all segments of a ray are
          // in this wave's list; the key buffer starts at all-ones)
          if (lane < RPW) {
            const unsigned long long k1 = scan_key(best, idx);
            if (whole) {
              if (stg) fin_k = true;
              else keys[ray] = k1;
              if (MX && a.keys2) a.keys2[ray] = scan_key(second, idx2);
            } else {
              const unsigned long long old = atomicMin(keys + ray, k1);
              if (MX && a.keys2) {
                // top two over the union, lock-free: every key that is not the final minimum
                // is either a segment's runner-up or lost one atomic min (old vs k1)
                atomicMin(a.keys2 + ray, old > k1 ? old : k1);
                atomicMin(a.keys2 + ray, (unsigned long long)scan_key(second, idx2));
              }
            }
          }
          kind = -1;
        }
      } else if (kind == 2) {
        if (ended) kind = -1;
      }
      if (stg) {
        const uint64_t ft = __ballot(fin_t) & kRayMask;
        if (ft) st_t.put(ft, ray, hit ? -t : t);
        const uint64_t fk = __ballot(fin_k) & kRayMask;
        if (fk) st_k.put(fk, ray, scan_key(best, idx));
      }
      const uint32_t want = (uint32_t)__ballot(kind == -1) & kRayMask;
      if (want == 0u) break;
      int64_t avail = J - cursor;  // list entries this pass can hand out from `cursor` on
      if (dyn) {
        if (cursor >= cend && !dry) {  // the next chunk of the launch's list
          unsigned int b = 0u;
          if (lane == 0) b = atomicAdd(a.queue, (unsigned int)kQueueChunk);
          cursor = (int64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)b);
          cend = cursor + kQueueChunk < J ? cursor + kQueueChunk : J;
          dry = cursor >= J;
        }
        avail = dry ? 0 : cend - cursor;
      }
      if (avail <= 0) {
        if (kind == -1) kind = -2;
        break;
      }
      if (kind == -1) {
        const int64_t q = cursor + __popc(want & lt);
        // (a lane past a queue chunk's end stays -1 and takes from the next chunk)
        if (q - cursor < avail) {
          int64_t k = q;
          int seg = -1;  // -1 march, kScanSegs whole scan, else a segment
          if (mode == 0 && q >= R) {
            k = q - R;
            if (k < R - T) {
              seg = kScanSegs;
            } else {
              k -= R - T;
              seg = (int)(k / T);
              k = R - T + (k - (int64_t)seg * T);
            }
          }
          const bool second_job = alt && q >= R;  // sdf(best)'s runner-up job
          if (second_job) k = q - R;
          ray = dyn ? k : own.ray(k);
          if (MX && a.list) ray = a.list[ray];
          if (mode == 2) {  // point evaluation: `rays` holds [P, 3] points, sdf(p) -> thr_out
            const float* pp = rays + ray * 3;
            ox = pp[0]; oy = pp[1]; oz = pp[2];
          } else {
            const float* rp = rays + ray * 6;
            ox = rp[0]; oy = rp[1]; oz = rp[2]; dx = rp[3]; dy = rp[4]; dz = rp[5];
          }
          ended = false;
          step = scan_step_of(a, ray);
          if (mode == 2) {
            kind = 2;
            idx = 0;
          } else if (mode == 1) {
            kind = 2;
            const unsigned long long k1 = keys[ray];
            idx = (int)(uint32_t)k1;
            if (second_job) {
              // the runner-up only where the FP16 values of the two lie within refine_s
              const unsigned long long k2 = a.keys2[ray];
              idx = (int)(uint32_t)k2;
              if (!(scan_key_value(k2) - scan_key_value(k1) <= a.refine_s)) kind = -1;
            }
          } else if (seg < 0) {
            kind = 0; t = 0.f; i = 0; hit = false; ambs = ~0ull; drift = 0.f; cps = ~0ull;
            if (mode == 3) {  // shadow rays start 100 eps out (sdfs.py:170)
              t = 0.f + 1e2f * a.eps;
              mt = a.occ_max_t[ray];
            }
            if (MX && a.start) {
              const unsigned long long s0 = a.start[ray];
              t = __uint_as_float((uint32_t)s0);
              i = (int)(s0 >> 32);
            }
          } else {
            kind = 1;
            whole = seg == kScanSegs;
            j = (seg == 0 || whole) ? 0 : 16 * seg + 1;
            jend = whole ? 16 * kScanSegs : 16 * seg + 16;
            idx = -1;
          }
        } else if (!dyn) {
          kind = -2;
        }
      }
      cursor += __popc(want) < avail ? (int64_t)__popc(want) : avail;
    }
    if (__syncthreads_or(kind >= 0 ? 1 : 0) == 0) break;
    float px = 0.f, py = 0.f, pz = 0.f;
    if (kind == 0) {
      px = __fadd_rn(ox, __fmul_rn(dx, t));
      py = __fadd_rn(oy, __fmul_rn(dy, t));
      pz = __fadd_rn(oz, __fmul_rn(dz, t));
    } else if (kind == 1 || kind == 2) {
      // scan point j: o + (step * j) dir (sdfs.py:241-245); sdf(best): o + (idx * step) dir
      if (kind == 1 && j == 0) {
        px = ox; py = oy; pz = oz;
      } else if (mode == 2) {
        px = ox; py = oy; pz = oz;
      } else {
        const float ts = kind == 1 ? (float)(step * (double)j) : __fmul_rn((float)idx, (float)step);
        px = __fadd_rn(ox, __fmul_rn(ts, dx));
        py = __fadd_rn(oy, __fmul_rn(ts, dy));
        pz = __fadd_rn(oz, __fmul_rn(ts, dz));
      }
    }
    const float d = Pol::sdf(E, s, m, px, py, pz);
    if (a.evals) {  // profiling only: the SDF evaluations this wave-evaluation did for live jobs
      const uint32_t busy = (uint32_t)__ballot(kind >= 0) & kRayMask;
      if (lane == 0) atomicAdd(a.evals, (unsigned long long)__popc(busy));
    }
    // fp32-split range guard: an evaluation whose activations left f16's range runs again,
    // guarded, with every lane's job state unchanged (each wave still makes one evaluation per
    // iteration, so the block's ring barriers stay matched)
    if (Pol::retry(E, kind >= 0, d)) continue;
    if (kind == 0) {
      if (MX && a.amb && ambs == ~0ull) {
        // NRT_MIXED: FP16 cannot tell this step's hit test (or the next t's max_t test) from
        // the FP32 one.  The FP16 value is off by its own error e, and t has drifted from the
        // FP32 march's by the earlier steps' errors: delta_{k+1} = delta_k (1 + g_k) + e_k with
        // g_k = d(sdf)/dt along the ray, which the march observes as (d_k - d_{k-1}) / d_{k-1}.
        // drift = that bound in units of e (a.drift_model), or the step-count rule 1 + i/16.
        if (a.drift_model && i > 0) drift = drift * fabsf(d / dprev) + 1.f;
        const float bound = a.refine_d * (a.drift_model ? 1.f + drift : 1.f + 0.0625f * (float)i);
        const float tn = t + d;
        const unsigned long long here = ((unsigned long long)(uint32_t)i << 32) | __float_as_uint(t);
        // a.zone: the refinement resumes at the first step that came within `zone` of a surface
        // (the drift of the far-field steps before it kept), instead of at the flagged step
        if (a.zone > 0.f && cps == ~0ull && d < a.zone) cps = here;
        if (fabsf(d - a.eps) <= bound || (d > a.eps && fabsf(tn - a.max_t) <= bound))
          ambs = (a.zone > 0.f && cps != ~0ull) ? cps : here;
        dprev = d;
      }
      if (mode == 3) {  // sdfs.py:175-179: t advances on the hit step too, the test is strict
        const bool now = d < a.eps;
        t = t + d;
        if (now) { hit = true; ended = true; }
      } else if (d <= a.eps) {
        hit = true; ended = true;
      } else {
        t = t + d;
      }
      ++i;
    } else if (kind == 1) {
      // sdfs.py:246-248: idx = where(s < m, i + 1, idx); m = min(m, s)
      if (idx < 0) { best = d; idx = j; second = __builtin_inff(); idx2 = j; }  // first sample
      else if constexpr (MX) {  // (second, idx2): the runner-up, for NRT_MIXED's sdf(best)
        if (d < best) { second = best; idx2 = idx; idx = j; }
        else if (d < second) { second = d; idx2 = j; }
        best = fminf(best, d);
      } else {
        if (d < best) idx = j;
        best = fminf(best, d);
      }
      ++j;
    } else if (kind == 2) {
      if (lane < RPW) {
        if (MX && mode == 1 && a.kbest)  // both candidates of a ray merge; k_scan_pick writes thr
          atomicMin(a.kbest + ray, (unsigned long long)scan_key(d, idx));
        else
          thr_out[ray] = mode == 2 ? d : -1000.f * d;
      }
      ended = true;
    }
  }
  if (stg) {
    st_t.drain();
    st_k.drain();
  }
  Pol::finish(E);
}

// the two passes as separately named kernels (profiles time the march + scan launch alone)
#define NRT_MARCH_ARGS                                                                         \
  const SdfDev s, const MlpDev m, const float* __restrict__ rays, int64_t P, MarchArgs a,       \
      float* __restrict__ t_out, uint8_t* __restrict__ hit_out, float* __restrict__ p_out,     \
      float* __restrict__ n_out, float* __restrict__ rawn_out, float* __restrict__ thr_out,    \
      unsigned long long* __restrict__ keys
#define NRT_MARCH_PASS t_out, hit_out, p_out, n_out, rawn_out, thr_out, keys
template <int NB, int NE, int WV, bool FOLD, bool MX = false>
__global__ void __launch_bounds__(64 * WV, WV >= 16 ? 1 : 2) k_march16(NRT_MARCH_ARGS) {
  march_body<RingPol16<NB, NE, WV, FOLD>, 0, MX>(s, m, rays, P, a, NRT_MARCH_PASS);
}
template <int NB, int NE, int WV, bool FOLD>
__global__ void __launch_bounds__(64 * WV, WV >= 16 ? 1 : 2) k_scan_best16(NRT_MARCH_ARGS) {
  march_body<RingPol16<NB, NE, WV, FOLD>, 1>(s, m, rays, P, a, NRT_MARCH_PASS);
}
// shadow march (intersect_test) on each ring engine: visible -> hit_out
template <int NB, int NE, int WV, bool FOLD>
__global__ void __launch_bounds__(64 * WV, WV >= 16 ? 1 : 2) k_occl16(NRT_MARCH_ARGS) {
  march_body<RingPol16<NB, NE, WV, FOLD>, 3>(s, m, rays, P, a, NRT_MARCH_PASS);
}
template <int KH, int KE, int WV, int ACT>
__global__ void __launch_bounds__(64 * WV, 1) k_occl32(NRT_MARCH_ARGS) {
  march_body<RingPol32<KH, KE, WV, ACT>, 3>(s, m, rays, P, a, NRT_MARCH_PASS);
}
template <int KH, int KQ, int WV, int ACT>
__global__ void __launch_bounds__(64 * WV, 1) k_occl3(NRT_MARCH_ARGS) {
  march_body<RingPol3<KH, KQ, WV, ACT>, 3>(s, m, rays, P, a, NRT_MARCH_PASS);
}
// FP32 (reference precision): one block of WV waves per CU (the ring takes most of the LDS), two
// waves per SIMD
template <int KH, int KE, int WV, int ACT>
__global__ void __launch_bounds__(64 * WV, 1) k_march32(NRT_MARCH_ARGS) {
  march_body<RingPol32<KH, KE, WV, ACT>, 0>(s, m, rays, P, a, NRT_MARCH_PASS);
}
template <int KH, int KE, int WV, int ACT>
__global__ void __launch_bounds__(64 * WV, 1) k_scan_best32(NRT_MARCH_ARGS) {
  march_body<RingPol32<KH, KE, WV, ACT>, 1>(s, m, rays, P, a, NRT_MARCH_PASS);
}
// fp32-split (FP32-accurate on FP16 MFMA): one block of WV waves per CU, two waves per SIMD
template <int KH, int KQ, int WV, int ACT, bool MX = false>
__global__ void __launch_bounds__(64 * WV, 1) k_march3(NRT_MARCH_ARGS) {
  march_body<RingPol3<KH, KQ, WV, ACT>, 0, MX>(s, m, rays, P, a, NRT_MARCH_PASS);
}
template <int KH, int KQ, int WV, int ACT, bool MX = false>
__global__ void __launch_bounds__(64 * WV, 1) k_scan_best3(NRT_MARCH_ARGS) {
  march_body<RingPol3<KH, KQ, WV, ACT>, 1, MX>(s, m, rays, P, a, NRT_MARCH_PASS);
}
// sdf(p) of P points on the ring engines (nrt_sdf_eval: fp32-split and FP32 precision)
template <int KH, int KQ, int WV, int ACT>
__global__ void __launch_bounds__(64 * WV, 1) k_sdf_eval3(NRT_MARCH_ARGS) {
  march_body<RingPol3<KH, KQ, WV, ACT>, 2>(s, m, rays, P, a, NRT_MARCH_PASS);
}
template <int KH, int KE, int WV, int ACT>
__global__ void __launch_bounds__(64 * WV, 1) k_sdf_eval32r(NRT_MARCH_ARGS) {
  march_body<RingPol32<KH, KE, WV, ACT>, 2>(s, m, rays, P, a, NRT_MARCH_PASS);
}
#undef NRT_MARCH_PASS
#undef NRT_MARCH_ARGS

// FP32 / fp32-split SDF normals on the hit list (sdfs.py:152-158 with the autograd normal of
// sdfs.py:184-197) by forward mode on the ring32 / ring3 engines: a 16-column tile = 4 rays x
// (value, d/dx, d/dy, d/dz), so one wave-evaluation yields 4 gradients at the MFMA cost of 16
// value evaluations.  Same outputs as k_normal16 / k_sdf_grad: raw gradient (sphere blobs
// analytic + the shift MLP's), normalize(g, 1e-6), p += 5 eps n.  Blocks stride over the
// device-counted hit list; the loop bound is block-uniform.
template <class Pol>
__global__ void __launch_bounds__(64 * Pol::WAVES, 1) k_normal_r(
    const SdfDev s, const MlpDev m, const int32_t* __restrict__ index,
    const int32_t* __restrict__ count, int64_t M, float* __restrict__ grad,
    float* __restrict__ n_out, float* __restrict__ p_io, float offset_eps) {
  extern __shared__ __attribute__((aligned(16))) char smem_c[];
  constexpr int WV = Pol::WAVES;
  const int64_t total = count ? (int64_t)(*(const NRT_GLOBAL int32_t*)count) : M;
  const int64_t per_block = 4 * WV;
  if ((int64_t)blockIdx.x * per_block >= total) return;  // whole block, before the ring starts
  typename Pol::Eng E;
  Pol::init(E, s, m, smem_c, MarchArgs{});
  const int lane = E.lane, comp = lane & 3;
  for (int64_t b0 = (int64_t)blockIdx.x * per_block; b0 < total; b0 += (int64_t)gridDim.x * per_block) {
    const int64_t i = b0 + 4 * E.wv + ((lane & 15) >> 2);
    const bool valid = i < total;
    const int64_t ii = valid ? i : total - 1;
    const int64_t idx = index ? (int64_t)index[ii] : ii;
    const float x = p_io[idx * 3], y = p_io[idx * 3 + 1], z = p_io[idx * 3 + 2];
    float v = Pol::tan(E, m, x, y, z);
    if constexpr (Pol::kGuard) {  // range guard: the whole block repeats the tile (one barrier)
      while (__syncthreads_or(Pol::retry(E, true, v) ? 1 : 0)) v = Pol::tan(E, m, x, y, z);
    }
    const float gx = __shfl(v, lane + 1), gy = __shfl(v, lane + 2), gz = __shfl(v, lane + 3);
    if (valid && lane < 16 && comp == 0) {
      float g[3] = {0.f, 0.f, 0.f};
      if (s.kind == 2) spheres_grad(s, x, y, z, g);
      g[0] += gx; g[1] += gy; g[2] += gz;
      if (grad) { grad[idx * 3] = g[0]; grad[idx * 3 + 1] = g[1]; grad[idx * 3 + 2] = g[2]; }
      float nx = g[0], ny = g[1], nz = g[2];
      normalize3(nx, ny, nz, 1e-6f);
      n_out[idx * 3] = nx; n_out[idx * 3 + 1] = ny; n_out[idx * 3 + 2] = nz;
      p_io[idx * 3] = x + (nx * offset_eps) * 5.f;
      p_io[idx * 3 + 1] = y + (ny * offset_eps) * 5.f;
      p_io[idx * 3 + 2] = z + (nz * offset_eps) * 5.f;
    }
  }
  Pol::finish(E);
}

// coarse-scan argmin index of each ray from the ring march's 64-bit keys ([ordered min | idx])
template <int = 0>
__global__ void k_keys_index(const unsigned long long* __restrict__ keys, int64_t P,
                             int32_t* __restrict__ idx) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < P) idx[i] = (int32_t)(uint32_t)keys[i];
}

// NRT_MIXED: the rays whose FP16 march met an undecidable step (amb != all-ones), as a list for
// the refinement march (wave-aggregated appends; order is irrelevant)
template <int = 0>
__global__ void k_refine_list(const unsigned long long* __restrict__ amb, int64_t P,
                              int32_t* __restrict__ list, int32_t* __restrict__ cnt) {
  const int lane = lane_id();
  for (int64_t ray = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; ray - lane < P;
       ray += (int64_t)gridDim.x * blockDim.x) {
    const bool f = ray < P && amb[ray] != ~0ull;
    const uint64_t mk = __ballot(f);
    const int c = __popcll(mk);
    int base = 0;
    if (lane == 0 && c) base = atomicAdd(cnt, c);
    base = __shfl(base, 0);
    if (f) list[base + __popcll(mk & ((1ull << lane) - 1ull))] = (int32_t)ray;
  }
}

// NRT_MIXED sdf(best): kbest holds the smaller (value, index) key of the candidates evaluated at
// FP32 accuracy; thr = -1000 * value (sdfs.py:137) and the key's index replaces the FP16 argmin
template <int = 0>
__global__ void k_scan_pick(const unsigned long long* __restrict__ kbest, int64_t P,
                            unsigned long long* __restrict__ keys, float* __restrict__ thr) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < P) {
    const unsigned long long k = kbest[i];
    thr[i] = -1000.f * scan_key_value(k);
    keys[i] = k;
  }
}

// After a ring march that packed (hit, t) into t's sign bit (march_body with p_out == nullptr):
// per ray, t = |t|, hit, p = o + t d (the march's rounding), n = raw_n = 0, and the hit list --
// one coalesced pass instead of ~45 lane-scattered bytes per ray inside the march (the strided
// ray deal writes every line of t / p / n in 4-byte pieces from many waves).
template <int = 0>
__global__ void k_march_finish(const float* __restrict__ rays, int64_t P, float* __restrict__ t_io,
                               uint8_t* __restrict__ hit_out, float* __restrict__ p_out,
                               float* __restrict__ n_out, float* __restrict__ rawn_out,
                               int32_t* __restrict__ idx, int32_t* __restrict__ cnt) {
  const int lane = lane_id();
  for (int64_t ray = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; ray - lane < P;
       ray += (int64_t)gridDim.x * blockDim.x) {
    bool h = false;
    if (ray < P) {
      // a NaN t (an SDF value that went NaN mid-march) ended as a miss; its sign bit is noise
      const float te = t_io[ray];
      h = __builtin_signbit(te) != 0 && te == te;
      const float t = fabsf(te);
      const float* r = rays + ray * 6;
      t_io[ray] = t;
      hit_out[ray] = h ? 1 : 0;
      p_out[ray * 3] = __fadd_rn(r[0], __fmul_rn(t, r[3]));
      p_out[ray * 3 + 1] = __fadd_rn(r[1], __fmul_rn(t, r[4]));
      p_out[ray * 3 + 2] = __fadd_rn(r[2], __fmul_rn(t, r[5]));
      n_out[ray * 3] = 0.f; n_out[ray * 3 + 1] = 0.f; n_out[ray * 3 + 2] = 0.f;
      if (rawn_out) { rawn_out[ray * 3] = 0.f; rawn_out[ray * 3 + 1] = 0.f; rawn_out[ray * 3 + 2] = 0.f; }
    }
    if (idx) {
      const uint64_t mk = __ballot(h);
      const int c = __popcll(mk);
      int base = 0;
      if (lane == 0 && c) base = atomicAdd(cnt, c);
      base = __shfl(base, 0);
      if (h) idx[base + __popcll(mk & ((1ull << lane) - 1ull))] = (int32_t)ray;
    }
  }
}

// hit list of a finished march (order is irrelevant downstream): wave-aggregated appends
template <int = 0>
__global__ void k_hit_list(const uint8_t* __restrict__ hit, int64_t P, int32_t* __restrict__ idx,
                           int32_t* __restrict__ cnt) {
  const int lane = lane_id();
  for (int64_t ray = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; ray - lane < P;
       ray += (int64_t)gridDim.x * blockDim.x) {
    const bool h = ray < P && hit[ray] != 0;
    const uint64_t mk = __ballot(h);
    const int c = __popcll(mk);
    int base = 0;
    if (lane == 0 && c) base = atomicAdd(cnt, c);
    base = __shfl(base, 0);
    if (h) idx[base + __popcll(mk & ((1ull << lane) - 1ull))] = (int32_t)ray;
  }
}

// FP16 normals on the ring engine by forward-mode differentiation: a wave's 32 MFMA columns
// are 8 hit rays x (value, d/dx, d/dy, d/dz), so one evaluation yields the SDF gradient of 8
// rays with no saved pre-activations.  Same outputs as k_sdf_grad: raw gradient, unit normal
// normalize(g, 1e-6), p += 5 eps n (sdfs.py:156-157, autograd normal sdfs.py:184-197).
// Blocks stride over the (device-counted) hit list together; the loop bound is block-uniform.
template <int NB, int NE, int WV, bool FOLD>
__global__ void __launch_bounds__(64 * WV, WV >= 16 ? 1 : 2) k_normal16(
    const SdfDev s, const MlpDev m, const int32_t* __restrict__ index,
    const int32_t* __restrict__ count, int64_t M, float* __restrict__ grad,
    float* __restrict__ n_out, float* __restrict__ p_io, float offset_eps) {
  extern __shared__ __attribute__((aligned(16))) char smem_c[];
  const int64_t total = count ? (int64_t)(*(const NRT_GLOBAL int32_t*)count) : M;
  const int64_t per_block = 8 * WV;
  if ((int64_t)blockIdx.x * per_block >= total) return;  // whole block, before the ring starts
  ring::Engine<NB, NE, WV> E;
  E.init(m, smem_c);
  const int lane = lane_id(), comp = lane & 3;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (int64_t b0 = (int64_t)blockIdx.x * per_block; b0 < total; b0 += (int64_t)gridDim.x * per_block) {
    const int64_t i = b0 + 8 * wv + ((lane & 31) >> 2);
    const bool valid = i < total;
    const int64_t ii = valid ? i : total - 1;
    const int64_t idx = index ? (int64_t)index[ii] : ii;
    const float x = p_io[idx * 3], y = p_io[idx * 3 + 1], z = p_io[idx * 3 + 2];
    const float v = ring::eval<NB, NE, WV, FOLD, 8, 3, true>(E, m, x, y, z);
    const float gx = __shfl(v, lane + 1), gy = __shfl(v, lane + 2), gz = __shfl(v, lane + 3);
    if (valid && lane < 32 && comp == 0) {
      float g[3] = {0.f, 0.f, 0.f};
      if (s.kind == 2) spheres_grad(s, x, y, z, g);
      g[0] += gx; g[1] += gy; g[2] += gz;
      if (grad) { grad[idx * 3] = g[0]; grad[idx * 3 + 1] = g[1]; grad[idx * 3 + 2] = g[2]; }
      float nx = g[0], ny = g[1], nz = g[2];
      normalize3(nx, ny, nz, 1e-6f);
      n_out[idx * 3] = nx; n_out[idx * 3 + 1] = ny; n_out[idx * 3 + 2] = nz;
      p_io[idx * 3] = x + (nx * offset_eps) * 5.f;
      p_io[idx * 3 + 1] = y + (ny * offset_eps) * 5.f;
      p_io[idx * 3 + 2] = z + (nz * offset_eps) * 5.f;
    }
  }
}

// shading frame of n (0 on misses) and wi = to_local(frame, -d)
__device__ __forceinline__ void make_frame(float nx, float ny, float nz, float f[9]) {
  // coordinate_system, interaction.py:9-27; f = [s | t | n] as columns: f[3*row + col]
  normalize3(nx, ny, nz, 1e-7f);
  float sign = nz >= 0.f ? 1.f : -1.f;
  float sz = sign + nz;
  float a = -(1.f / (fabsf(sz) < 1e-6f ? 1e-6f : sz));
  float b = nx * ny * a;
  float sx = (nx * nx * a * sign) + 1.f, sy = b * sign, szz = nx * -sign;
  normalize3(sx, sy, szz, 1e-7f);
  float tx = sy * nz - szz * ny, ty = szz * nx - sx * nz, tz = sx * ny - sy * nx;  // s x n
  normalize3(tx, ty, tz, 1e-7f);
  float s2x = ny * tz - nz * ty, s2y = nz * tx - nx * tz, s2z = nx * ty - ny * tx;  // n x t
  normalize3(s2x, s2y, s2z, 1e-7f);
  f[0] = s2x; f[3] = s2y; f[6] = s2z;
  f[1] = tx;  f[4] = ty;  f[7] = tz;
  f[2] = nx;  f[5] = ny;  f[8] = nz;
}

// to_local (interaction.py:37-41): normalize(mean_j frame[j][c] * w[j])
__device__ __forceinline__ void to_local(const float f[9], float wx, float wy, float wz,
                                         float o[3]) {
  for (int c = 0; c < 3; ++c) o[c] = ((f[c] * wx + f[3 + c] * wy) + f[6 + c] * wz) / 3.f;
  normalize3(o[0], o[1], o[2], 1e-7f);
}

template <int = 0>
__global__ void k_frame_wi(const float* __restrict__ rays, const float* __restrict__ n, int64_t P,
                           float* __restrict__ frame, float* __restrict__ wi) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P) return;
  float f[9];
  make_frame(n[i * 3], n[i * 3 + 1], n[i * 3 + 2], f);
  if (frame)
    for (int q = 0; q < 9; ++q) frame[i * 9 + q] = f[q];
  if (wi) {
    float o[3];
    to_local(f, -rays[i * 6 + 3], -rays[i * 6 + 4], -rays[i * 6 + 5], o);
    wi[i * 3] = o[0]; wi[i * 3 + 1] = o[1]; wi[i * 3 + 2] = o[2];
  }
}

// shadow-ray march (intersect_test, sdfs.py:162-181)
template <bool F16, int NB>
__global__ void __launch_bounds__(256, F16 ? 2 : 1) k_occlusion(const SdfDev* __restrict__ sp,
                                                    const float* __restrict__ rays, int64_t P,
                                                    const int32_t* __restrict__ count,
                                                    const float* __restrict__ max_t, int max_steps,
                                                    float eps, uint8_t* __restrict__ visible,
                                                    int RS, int per_wave) {
  extern __shared__ float smem[];
  const SdfDev& s = *sp;
  WaveLds l = wave_lds(smem, per_wave, RS, F16);
  const int lane = lane_id(), r = lane & 31;
  if (count) P = min(P, (int64_t)*count);  // a compacted list (shadow rays of the hit list)
  const int64_t ray0 = wave_global() * 32;
  if (ray0 >= P) return;
  const int64_t ray = ray0 + r;
  const bool valid = ray < P;
  const int64_t rr = valid ? ray : P - 1;
  const float ox = rays[rr * 6], oy = rays[rr * 6 + 1], oz = rays[rr * 6 + 2];
  const float dx = rays[rr * 6 + 3], dy = rays[rr * 6 + 4], dz = rays[rr * 6 + 5];
  float t = 0.f + 1e2f * eps;
  bool live = valid;
  for (int i = 0; i < max_steps; ++i) {
    if (!wave_any(live)) break;
    const float px = __fadd_rn(ox, __fmul_rn(dx, t));
    const float py = __fadd_rn(oy, __fmul_rn(dy, t));
    const float pz = __fadd_rn(oz, __fmul_rn(dz, t));
    const float d = sdf_value<F16, NB>(s, px, py, pz, l, RS, nullptr);
    const bool now = live && (d < eps);
    if (live) t = t + d;
    live = live && !now;
  }
  if (valid && lane < 32) visible[ray] = ((t >= max_t[ray]) || live) ? 1 : 0;
}

// PointLights.sample_direction at p: the unit-ish direction to the light, Le and the distance.
// falloff 0, the pathtracer's light (lights.py:89-110): d = normalize(loc - p) (eps 1e-6),
// Le = scale normalize(I) / max(c + l dist + q dist^2, 1e-6).  falloff 1, the renderer's
// PointLights (renderer/lighting.py:283-304, utils.sphere_examples' light): d = (loc - p) inv,
// Le = ((scale I) inv) inv with inv = 1 / (1e-7 + dist).
__device__ __forceinline__ void point_light(const LightDev& lt, float px, float py, float pz,
                                            float& lx, float& ly, float& lz, float le[3],
                                            float& dist) {
  const float vx = lt.loc[0] - px, vy = lt.loc[1] - py, vz = lt.loc[2] - pz;
  dist = sqrtf(vx * vx + vy * vy + vz * vz);
  if (lt.falloff == 1) {
    const float inv = 1.f / (1e-7f + dist);
    lx = vx * inv; ly = vy * inv; lz = vz * inv;
    for (int k = 0; k < 3; ++k) le[k] = (lt.scaled_dir[k] * inv) * inv;
  } else {
    lx = vx; ly = vy; lz = vz;
    normalize3(lx, ly, lz, 1e-6f);
    const float fall = fmaxf((lt.c + lt.l * dist) + lt.q * (dist * dist), 1e-6f);
    for (int k = 0; k < 3; ++k) le[k] = lt.scaled_dir[k] / fall;
  }
}

// shadow rays toward a point light for each hit-list position i (sample_emitter_dir_w_isect,
// scene.py:290-298 with PointLights.sample_direction, lights.py:89-110): [p, normalize(loc - p)],
// max_t = |loc - p|
template <int = 0>
__global__ void k_point_shadow_rays(const LightDev* __restrict__ lp, const float* __restrict__ P_,
                                    const int32_t* __restrict__ hit_idx,
                                    const int32_t* __restrict__ hit_count,
                                    float* __restrict__ rays, float* __restrict__ max_t) {
  const int64_t total = *hit_count;
  const LightDev& lt = *lp;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t idx = hit_idx[i];
    const float px = P_[idx * 3], py = P_[idx * 3 + 1], pz = P_[idx * 3 + 2];
    float vx, vy, vz, le[3], dist;
    point_light(lt, px, py, pz, vx, vy, vz, le, dist);
    float* o = rays + i * 6;
    o[0] = px; o[1] = py; o[2] = pz; o[3] = vx; o[4] = vy; o[5] = vz;
    max_t[i] = dist;
  }
}

// dir_to_elev_azim (utils.py:490-494)
__device__ __forceinline__ void dir_elev_azim(float x, float y, float z, float& elev, float& azim) {
  normalize3(x, y, z, 1e-12f);
  const float lo = -1.f + 1e-7f, hi = 1.f - 1e-7f;
  x = fminf(fmaxf(x, lo), hi);
  z = fminf(fmaxf(z, lo), hi);
  elev = asinf(z);
  azim = atan2f(x, sqrtf(fmaxf((1.f - x * x) - z * z, 1e-10f)));
}

// occ_rays = [p, dir_to_elev_azim(ds.d)] per listed ray (scene.py:309-312); d from the shadow rays
template <int = 0>
__global__ void k_occ_inputs(const float* __restrict__ P_, const int32_t* __restrict__ hit_idx,
                             const int32_t* __restrict__ hit_count, const float* __restrict__ rays,
                             float* __restrict__ x) {
  const int64_t total = *hit_count;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t idx = hit_idx[i];
    float* o = x + i * 5;
    o[0] = P_[idx * 3]; o[1] = P_[idx * 3 + 1]; o[2] = P_[idx * 3 + 2];
    dir_elev_azim(rays[i * 6 + 3], rays[i * 6 + 4], rays[i * 6 + 5], o[3], o[4]);
  }
}

// per listed ray, the factor on Le: visible -> 1; occluded -> 0 (scene.py:297) or
// sigmoid(occ(occ_rays)) (scene.py:313-317; occ_out 1 broadcasts over RGB, 3 is per channel)
template <int = 0>
__global__ void k_light_scale(const int32_t* __restrict__ hit_count, const uint8_t* __restrict__ vis,
                              const float* __restrict__ occ, int occ_out, float* __restrict__ ls) {
  const int64_t total = *hit_count;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const bool v = vis[i] != 0;
    for (int q = 0; q < 3; ++q) {
      float s = 1.f;
      if (!v) s = occ ? 1.f / (1.f + expf(-occ[i * occ_out + (occ_out == 3 ? q : 0)])) : 0.f;
      ls[i * 3 + q] = s;
    }
  }
}

// ------------------------------------------------------------------------------------------
// shading
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ float nz_eps(float v) { return fabsf(v) < 1e-7f ? 1e-7f : v; }

// param_rusin2(wo, wi), utils.py:233-258 (wo, wi already local)
__device__ __forceinline__ void rusin2(float ax, float ay, float az, float bx, float by, float bz,
                                       float out[3]) {
  normalize3(ax, ay, az, 1e-12f);  // wo
  normalize3(bx, by, bz, 1e-12f);  // wi
  float hx = ax + bx, hy = ay + by, hz = az + bz;
  normalize3(hx, hy, hz, 1e-12f);
  float r = fmaxf(hypotf(nz_eps(hy), nz_eps(hx)), 1e-6f);
  float c = hx / r, s = -(hy / r);
  // rotate wi about z: v*c + z*(v.z)*(1-c) + (z x v)*s, z x v = (-vy, vx, 0)
  float tx = bx * c + 0.f * bz * (1.f - c) + (0.f * bz - 1.f * by) * s;
  float ty = by * c + 0.f * bz * (1.f - c) + (1.f * bx - 0.f * bz) * s;
  float tz = bz * c + 1.f * bz * (1.f - c) + (0.f * by - 0.f * bx) * s;
  normalize3(tx, ty, tz, 1e-12f);
  float c2 = hz, s2 = -sqrtf(fmaxf(1.f - hz, 1e-6f));
  // rotate tmp about y: y x v = (vz, 0, -vx)
  float dx = tx * c2 + 0.f * ty * (1.f - c2) + (1.f * tz - 0.f * ty) * s2;
  float dy = ty * c2 + 1.f * ty * (1.f - c2) + (0.f * tx - 0.f * tz) * s2;
  float dz = tz * c2 + 0.f * ty * (1.f - c2) + (0.f * ty - 1.f * tx) * s2;
  normalize3(dx, dy, dz, 1e-12f);
  out[0] = cosf(atan2f(nz_eps(dy), nz_eps(dx)));
  out[1] = hz;
  out[2] = dz;
}

__device__ __forceinline__ float fresnel_conductor(float cos_t, float eta_r) {
  // bsdfs.py:327-341 with eta_i = 0
  float ct2 = cos_t * cos_t;
  float st2 = fmaxf(1.f - ct2, 1e-10f);
  float st4 = st2 * st2;
  float tmp = (float)((double)eta_r * (double)eta_r) - st2;
  float a2pb2 = sqrtf(fmaxf(tmp * tmp + 0.f, 1e-10f));
  float a = sqrtf(fmaxf(0.5f * (a2pb2 + tmp), 1e-10f));
  float t1 = a2pb2 + ct2;
  float t2 = 2.f * cos_t * a;
  float rs = (t1 - t2) / (t1 + t2);
  float t3 = a2pb2 * ct2 + st4;
  float t4 = t2 * st2;
  float rp = rs * (t3 - t4) / (t3 + t4);
  return 0.5f * (rs + rp);
}

// One wave shades 32 hit rays.  The MLP evaluations of the light, the spatial weights and each
// NeuralBSDF run through ONE call site (a job loop) so every hidden width is inlined once.
template <bool F16>
__global__ void __launch_bounds__(256) k_shade_direct(
    const BsdfDev* __restrict__ bp, const LightDev* __restrict__ lp, const float* __restrict__ P_,
    const float* __restrict__ N_, const float* __restrict__ WI, const int32_t* __restrict__ hit_idx,
    const int32_t* __restrict__ hit_count, const float* __restrict__ lscale,
    float* __restrict__ rgb, float* __restrict__ wout, int RS, int per_wave) {
  extern __shared__ float smem[];
  const BsdfDev& bs = *bp;
  const LightDev& lt = *lp;
  WaveLds l = wave_lds(smem, per_wave, RS, F16);
  // per-wave scratch after Y: spatial weights K[32][kMaxComponents]
  float* Kw = l.Y + 32 * 32;
  const int lane = lane_id(), r = lane & 31;
  const int ys = 32;
  const int nc = bs.n;
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
  const int64_t total = *hit_count;
  for (int64_t w = wave_global(); w * 32 < total; w += nw) {
    const int64_t i = w * 32 + r;
    const bool valid = i < total;
    const int64_t idx = hit_idx[valid ? i : total - 1];
    const float px = P_[idx * 3], py = P_[idx * 3 + 1], pz = P_[idx * 3 + 2];
    float fr[9];
    make_frame(N_[idx * 3], N_[idx * 3 + 1], N_[idx * 3 + 2], fr);
    const float wix = WI[idx * 3], wiy = WI[idx * 3 + 1], wiz = WI[idx * 3 + 2];

    float ldx = 0.f, ldy = 0.f, ldz = 0.f, le[3] = {0.f, 0.f, 0.f}, wo[3] = {0.f, 0.f, 0.f};
    float feat[3] = {0.f, 0.f, 0.f};
    float f[3] = {0.f, 0.f, 0.f};
    if (lt.kind == 1) {
      // PointLights.sample_direction (lights.py:89-110 / renderer/lighting.py:283-304)
      float dist;
      point_light(lt, px, py, pz, ldx, ldy, ldz, le, dist);
      to_local(fr, ldx, ldy, ldz, wo);
      rusin2(wix, wiy, wiz, wo[0], wo[1], wo[2], feat);
    }
    if (!bs.spatial)
      for (int j = lane >> 5; j < nc; j += 2) Kw[r * kMaxComponents + j] = 1.f;
    // job list: -2 light field, -1 spatial weights, 0..nc-1 components
    for (int job = -2; job < nc; ++job) {
      const MlpDev* m = nullptr;
      if (job == -2) m = (lt.kind == 0) ? lt.mlp : nullptr;
      else if (job == -1) m = bs.spatial;
      else m = (bs.comp[job].kind == 0) ? bs.comp[job].mlp : nullptr;
      if (m) {
        EncIn e;
        e.xg = nullptr; e.lat = nullptr; e.x[3] = 0.f;
        if (job < 0) { e.x[0] = px; e.x[1] = py; e.x[2] = pz; }
        else { e.x[0] = feat[0]; e.x[1] = feat[1]; e.x[2] = feat[2]; }
        mlp_eval_any<F16>(*m, e, l.X, RS, l.Y, ys);
      }
      if (job == -2) {
        if (lt.kind == 0) {
          // LightField.sample_direction (lights.py:175-195)
          float vx = l.Y[r * ys], vy = l.Y[r * ys + 1], vz = l.Y[r * ys + 2];
          float mag = sqrtf(vx * vx + vy * vy + vz * vz);
          ldx = vx; ldy = vy; ldz = vz;
          normalize3(ldx, ldy, ldz, 1e-6f);
          ldx = fminf(fmaxf(ldx, 1e-6f), 1.f);
          ldy = fminf(fmaxf(ldy, 1e-6f), 1.f);
          ldz = fminf(fmaxf(ldz, 1e-6f), 1.f);
          le[0] = mag * lt.color_sig[0]; le[1] = mag * lt.color_sig[1]; le[2] = mag * lt.color_sig[2];
          to_local(fr, ldx, ldy, ldz, wo);
          rusin2(wix, wiy, wiz, wo[0], wo[1], wo[2], feat);
        }
      } else if (job == -1) {
        if (m)
          for (int j = lane >> 5; j < nc; j += 2) Kw[r * kMaxComponents + j] = sigmoidf_(l.Y[r * ys + j]);
      } else {
        const BsdfCompDev& c = bs.comp[job];
        float v[3];
        if (c.kind == 0) {
          for (int q = 0; q < 3; ++q) v[q] = act_fwd<false>(l.Y[r * ys + q], c.act);
        } else if (c.kind == 1) {
          // Diffuse.eval_and_pdf (bsdfs.py:108-118)
          for (int q = 0; q < 3; ++q) {
            float x = wo[2] * c.params[q];
            v[q] = (c.act == ACT_NONE) ? x / (float)M_PI : act_fwd<false>(x, c.act);
          }
        } else {
          // Conductor.eval_and_pdf (bsdfs.py:364-388)
          float rx = -wix, ry = -wiy, rz = wiz;
          bool th = ((rx * wo[0] + ry * wo[1]) + rz * wo[2]) > 0.94f;
          float fres = fresnel_conductor(wiz, c.params[3]);
          for (int q = 0; q < 3; ++q) v[q] = th ? fres * act_fwd<false>(c.params[q], c.act) : 0.f;
        }
        wave_lds_fence();
        const float kj = Kw[r * kMaxComponents + job];
        f[0] += v[0] * kj; f[1] += v[1] * kj; f[2] += v[2] * kj;
      }
      wave_lds_fence();
    }
    if (lscale) {  // shadow test (scene.py:297) or learned occlusion (scene.py:313-318)
      const float* sc = lscale + (valid ? i : total - 1) * 3;
      le[0] *= sc[0]; le[1] *= sc[1]; le[2] *= sc[2];
    }
    if (valid && lane < 32) {
      // integrators.py:186-189: mis(=1) * bsdf_val * emitter_val, / emitter_samples(=1)
      rgb[idx * 3] = (1.f * f[0]) * le[0];
      rgb[idx * 3 + 1] = (1.f * f[1]) * le[1];
      rgb[idx * 3 + 2] = (1.f * f[2]) * le[2];
      if (wout)
        for (int j = 0; j < nc; ++j) wout[idx * nc + j] = Kw[r * kMaxComponents + j];
    }
    wave_lds_fence();
  }
}

// ------------------------------------------------------------------------------------------
// FP16 shading on the program engine: k_light16 (emitter sample per hit) then k_bsdf16
// (spatial weights + components).  Same math as k_shade_direct; LS carries, per position i of
// the hit list, le (3) | feat = param_rusin2(wi, wo) (3) | wo (3) | pad (3).
// ------------------------------------------------------------------------------------------
constexpr int kLsStride = 12;

__device__ __forceinline__ void light_from_field(float vx, float vy, float vz, const LightDev& lt,
                                                 const float fr[9], float wix, float wiy,
                                                 float wiz, float le[3], float wo[3],
                                                 float feat[3]) {
  // LightField.sample_direction (lights.py:175-195)
  const float mag = sqrtf(vx * vx + vy * vy + vz * vz);
  float ldx = vx, ldy = vy, ldz = vz;
  normalize3(ldx, ldy, ldz, 1e-6f);
  ldx = fminf(fmaxf(ldx, 1e-6f), 1.f);
  ldy = fminf(fmaxf(ldy, 1e-6f), 1.f);
  ldz = fminf(fmaxf(ldz, 1e-6f), 1.f);
  le[0] = mag * lt.color_sig[0]; le[1] = mag * lt.color_sig[1]; le[2] = mag * lt.color_sig[2];
  to_local(fr, ldx, ldy, ldz, wo);
  rusin2(wix, wiy, wiz, wo[0], wo[1], wo[2], feat);
}

// FIELD: LightField MLP (8 x 32 hidden blocks, F = 16) on the ring; else a point light (VALU only)
template <int WV, bool FIELD>
__global__ void __launch_bounds__(64 * WV, 1) k_light16(
    const ProgDev prog, const LightDev* __restrict__ lp, const float* __restrict__ P_,
    const float* __restrict__ N_, const float* __restrict__ WI, const int32_t* __restrict__ hit_idx,
    const int32_t* __restrict__ hit_count, const float* __restrict__ lscale, float* __restrict__ LS) {
  extern __shared__ __attribute__((aligned(16))) char smem_c[];
  const LightDev& lt = *lp;
  const int64_t total = *(const NRT_GLOBAL int32_t*)hit_count;
  const int64_t per_block = 32 * WV;
  if ((int64_t)blockIdx.x * per_block >= total) return;
  ring::KEngine<WV> E;
  if (FIELD) E.init(prog, smem_c);
  const int lane = lane_id(), r = lane & 31;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (int64_t b0 = (int64_t)blockIdx.x * per_block; b0 < total; b0 += (int64_t)gridDim.x * per_block) {
    const int64_t i = b0 + 32 * wv + r;
    const bool valid = i < total;
    const int64_t idx = hit_idx[valid ? i : total - 1];
    const float px = P_[idx * 3], py = P_[idx * 3 + 1], pz = P_[idx * 3 + 2];
    float fr[9];
    make_frame(N_[idx * 3], N_[idx * 3 + 1], N_[idx * 3 + 2], fr);
    const float wix = WI[idx * 3], wiy = WI[idx * 3 + 1], wiz = WI[idx * 3 + 2];
    float le[3], wo[3], feat[3];
    if (FIELD) {
      const f16v o = ring::keval<8, 3, WV, ACT_LEAKY>(E, prog.mlp[0], px, py, pz);
      light_from_field(ring::tile_row(o, 0, lane), ring::tile_row(o, 1, lane),
                       ring::tile_row(o, 2, lane), lt, fr, wix, wiy, wiz, le, wo, feat);
    } else {
      // PointLights.sample_direction (lights.py:89-110 / renderer/lighting.py:283-304)
      float ldx, ldy, ldz, dist;
      point_light(lt, px, py, pz, ldx, ldy, ldz, le, dist);
      to_local(fr, ldx, ldy, ldz, wo);
      rusin2(wix, wiy, wiz, wo[0], wo[1], wo[2], feat);
    }
    if (lscale) {  // shadow test (scene.py:297) or learned occlusion (scene.py:313-318)
      const float* sc = lscale + (valid ? i : total - 1) * 3;
      le[0] *= sc[0]; le[1] *= sc[1]; le[2] *= sc[2];
    }
    if (valid && lane < 32) {
      float* o = LS + i * kLsStride;
      o[0] = le[0]; o[1] = le[1]; o[2] = le[2];
      o[3] = feat[0]; o[4] = feat[1]; o[5] = feat[2];
      o[6] = wo[0]; o[7] = wo[1]; o[8] = wo[2];
    }
  }
}

// Spatial weights (16 layers x 256, F = 128) and NeuralBSDF components (6 x 96, F = 64) on the
// ring; program order = [spatial] + neural components in component order.
template <int WV, bool SPATIAL>
__global__ void __launch_bounds__(64 * WV, 1) k_bsdf16(
    const ProgDev prog, const BsdfDev* __restrict__ bp, const float* __restrict__ P_,
    const float* __restrict__ WI, const int32_t* __restrict__ hit_idx,
    const int32_t* __restrict__ hit_count, const float* __restrict__ LS, float* __restrict__ rgb,
    float* __restrict__ wout) {
  extern __shared__ __attribute__((aligned(16))) char smem_c[];
  const BsdfDev& bs = *bp;
  const int nc = bs.n;
  const int64_t total = *(const NRT_GLOBAL int32_t*)hit_count;
  const int64_t per_block = 32 * WV;
  if ((int64_t)blockIdx.x * per_block >= total) return;
  ring::KEngine<WV> E;
  E.init(prog, smem_c);
  const int lane = lane_id(), r = lane & 31;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // per-wave spatial weights K[32 rays][kMaxComponents] after the program's LDS
  float* Kw = reinterpret_cast<float*>(smem_c + ring::KEngine<WV>::lds_bytes(prog)) +
              wv * 32 * kMaxComponents;
  for (int64_t b0 = (int64_t)blockIdx.x * per_block; b0 < total; b0 += (int64_t)gridDim.x * per_block) {
    const int64_t i = b0 + 32 * wv + r;
    const bool valid = i < total;
    const int64_t ii = valid ? i : total - 1;
    const int64_t idx = hit_idx[ii];
    const float* ls = LS + ii * kLsStride;
    const float le0 = ls[0], le1 = ls[1], le2 = ls[2];
    const float ft0 = ls[3], ft1 = ls[4], ft2 = ls[5];
    const float wo0 = ls[6], wo1 = ls[7], wo2 = ls[8];
    int k = 0;
    if (SPATIAL) {
      const float px = P_[idx * 3], py = P_[idx * 3 + 1], pz = P_[idx * 3 + 2];
      const f16v o = ring::keval<8, 17, WV, ACT_LEAKY>(E, prog.mlp[0], px, py, pz);
      k = 1;
#pragma unroll
      for (int j = 0; j < kMaxComponents; ++j) {
        const float v = ring::tile_row(o, j, lane);
        if (j < nc && lane < 32) Kw[r * kMaxComponents + j] = sigmoidf_(v);
      }
    } else {
      for (int j = lane >> 5; j < nc; j += 2) Kw[r * kMaxComponents + j] = 1.f;
    }
    wave_lds_fence();
    float f0 = 0.f, f1 = 0.f, f2 = 0.f;
    for (int j = 0; j < nc; ++j) {
      const BsdfCompDev& c = bs.comp[j];
      float v[3];
      if (c.kind == 0) {
        const f16v o = ring::keval<3, 9, WV, ACT_LEAKY>(E, prog.mlp[k], ft0, ft1, ft2);
        ++k;
#pragma unroll
        for (int q = 0; q < 3; ++q) v[q] = act_fwd<false>(ring::tile_row(o, q, lane), c.act);
      } else if (c.kind == 1) {
        // Diffuse.eval_and_pdf (bsdfs.py:108-118)
        for (int q = 0; q < 3; ++q) {
          float x = wo2 * c.params[q];
          v[q] = (c.act == ACT_NONE) ? x / (float)M_PI : act_fwd<false>(x, c.act);
        }
      } else {
        // Conductor.eval_and_pdf (bsdfs.py:364-388)
        const float wix = WI[idx * 3], wiy = WI[idx * 3 + 1], wiz = WI[idx * 3 + 2];
        float rx = -wix, ry = -wiy, rz = wiz;
        bool th = ((rx * wo0 + ry * wo1) + rz * wo2) > 0.94f;
        float fres = fresnel_conductor(wiz, c.params[3]);
        for (int q = 0; q < 3; ++q) v[q] = th ? fres * act_fwd<false>(c.params[q], c.act) : 0.f;
      }
      const float kj = Kw[r * kMaxComponents + j];
      f0 += v[0] * kj; f1 += v[1] * kj; f2 += v[2] * kj;
    }
    if (valid && lane < 32) {
      // integrators.py:186-189: mis(=1) * bsdf_val * emitter_val, / emitter_samples(=1)
      rgb[idx * 3] = (1.f * f0) * le0;
      rgb[idx * 3 + 1] = (1.f * f1) * le1;
      rgb[idx * 3 + 2] = (1.f * f2) * le2;
      if (wout)
        for (int j = 0; j < nc; ++j) wout[idx * nc + j] = Kw[r * kMaxComponents + j];
    }
    wave_lds_fence();
  }
}

// ------------------------------------------------------------------------------------------
// cameras + composite
// ------------------------------------------------------------------------------------------
template <int = 0>
__global__ void k_raygen(const nrt_camera* __restrict__ cams, int N, int x0, int y0, int W, int H,
                         float with_noise, const float* __restrict__ noise,
                         const float* __restrict__ positions, float* __restrict__ rays) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t total = (int64_t)N * W * H;
  if (i >= total) return;
  const int yy = (int)(i % H);
  const int xx = (int)((i / H) % W);
  const int n = (int)(i / ((int64_t)W * H));
  const nrt_camera& c = cams[n];
  // positions = stack([gy, gx]) -> u = column (y), v = row (x)   (main.py:66-71)
  const int64_t pix = (int64_t)xx * H + yy;
  float u = (float)(y0 + yy), v = (float)(x0 + xx);
  if (positions) { u = positions[pix * 2]; v = positions[pix * 2 + 1]; }
  float o[3], d[3];
  if (c.kind == NRT_CAM_NERF) {
    if (with_noise != 0.f && noise) {
      u = u + (noise[pix] - 0.5f) * with_noise;
      v = v + (noise[(int64_t)W * H + pix] - 0.5f) * with_noise;
    }
    const float half = (float)((double)c.size * 0.5);
    float a0 = (u - half) / c.focal, a1 = -((v - half) / c.focal), a2 = -1.f;
    const float* M = c.mat;  // [3][4]
    for (int j = 0; j < 3; ++j) d[j] = (a0 * M[4 * j] + a1 * M[4 * j + 1]) + a2 * M[4 * j + 2];
    normalize3(d[0], d[1], d[2], 1e-12f);
    o[0] = M[3]; o[1] = M[7]; o[2] = M[11];
  } else if (c.kind == NRT_CAM_DTU) {
    const float su = 1600.f / (float)c.size, sv = 1200.f / (float)c.size;
    float uu = u * su, vv = v * sv;
    const float* K = c.intrinsic;
    float fx = K[0], fy = K[5], cx = K[2], cy = K[6], sk = K[1];
    float xl = ((((uu - cx) + cy * sk / fy) - sk * vv / fy) / fx) * 1.f;
    float yl = ((vv - cy) / fy) * 1.f;
    float pt[4] = {xl, yl, 1.f, 1.f};
    const float* Pm = c.mat;  // pose [4][4]
    float wv[3];
    for (int j = 0; j < 3; ++j)
      wv[j] = ((Pm[4 * j] * pt[0] + Pm[4 * j + 1] * pt[1]) + Pm[4 * j + 2] * pt[2]) + Pm[4 * j + 3] * pt[3];
    o[0] = Pm[3]; o[1] = Pm[7]; o[2] = Pm[11];
    d[0] = wv[0] - o[0]; d[1] = wv[1] - o[1]; d[2] = wv[2] - o[2];
    normalize3(d[0], d[1], d[2], 1e-12f);
  } else {
    // FoV (renderer/cameras.py:539-575): jitter, NDC, inverse projection, normalize(point)
    if (with_noise != 0.f && noise) {
      u = u + (with_noise * noise[pix * 2] - with_noise / 2.f);
      v = v + (with_noise * noise[pix * 2 + 1] - with_noise / 2.f);
    }
    float px = -2.f * (u / (float)c.size) + 1.f;
    float py = -2.f * (v / (float)c.size) + 1.f;
    float pt[4] = {px, py, 1.f, 1.f};
    const float* Mi = c.mat;  // row-vector convention: out = pt @ Mi
    float q[4];
    for (int j = 0; j < 4; ++j)
      q[j] = ((pt[0] * Mi[j] + pt[1] * Mi[4 + j]) + pt[2] * Mi[8 + j]) + pt[3] * Mi[12 + j];
    d[0] = q[0] / q[3]; d[1] = q[1] / q[3]; d[2] = q[2] / q[3];
    normalize3(d[0], d[1], d[2], 1e-12f);
    o[0] = c.origin[0]; o[1] = c.origin[1]; o[2] = c.origin[2];
  }
  float* rr = rays + i * 6;
  rr[0] = o[0]; rr[1] = o[1]; rr[2] = o[2]; rr[3] = d[0]; rr[4] = d[1]; rr[5] = d[2];
}

template <int = 0>
__global__ void k_composite(const float* __restrict__ rgb, const float* __restrict__ thr,
                            const uint8_t* __restrict__ hit, int N, int W, int H, int alpha,
                            int fill, float bg, float* __restrict__ img, int IW, int IH, int C,
                            int X0, int Y0) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t total = (int64_t)N * W * H;
  if (i >= total) return;
  const int yy = (int)(i % H);
  const int xx = (int)((i / H) % W);
  const int n = (int)(i / ((int64_t)W * H));
  float* o = img + (((int64_t)n * IW + (X0 + xx)) * IH + (Y0 + yy)) * C;
  const bool miss = fill && hit && !hit[i];
  for (int c = 0; c < 3 && c < C; ++c) o[c] = miss ? bg : rgb[i * 3 + c];
  if (alpha && C > 3) o[3] = miss ? bg : 1.f / (1.f + expf(-thr[i]));
}

}  // namespace nrt
