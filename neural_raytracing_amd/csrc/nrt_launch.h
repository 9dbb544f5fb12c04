// nrt_launch.h -- host-side launch helpers shared by the nrt_api_*.hip translation units
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>

#include "nrt_internal.h"
#include "nrt_kernels.h"

namespace nrt {

// Named runtime options (nrt_set_option, include/nrt.h): process-wide, read at launch time.
enum Option {
  OPT_RING16 = 0,      // "ring16"
  OPT_RING32,          // "ring32"
  OPT_NORMALS16,       // "normals16"
  OPT_SCAN_BEST32,     // "scan_best32"
  OPT_MARCH_BLOCKS,    // "march_blocks"
  OPT_SHADE_PROGRAM,   // "shade_program"
  OPT_NERF_FUSED,      // "nerf_fused"
  OPT_MAX_WAVES,       // "max_waves"
  OPT_SHADE_RING,      // "shade_ring"
  OPT_NORMALS_RING,    // "normals_ring"
  OPT_XCD_LINES,       // "xcd_lines"
  OPT_MIXED_D,         // "mixed_refine_d" (1e-7 units)
  OPT_MIXED_S,         // "mixed_refine_s" (1e-7 units)
  OPT_MIXED_RESTART,   // "mixed_restart"
  OPT_MIXED_DRIFT,     // "mixed_drift"
  OPT_RING_OCCLUSION,  // "ring_occlusion"
  OPT_MIXED_ZONE,      // "mixed_zone" (1e-7 units)
  OPT_BWD_COLSPLIT,    // "bwd_colsplit"
  OPT_BWD_RING,        // "bwd_ring"
  OPT_MARCH_QUEUE,     // "march_queue"
  OPT_TRAIN_SAVE,      // "train_save"
  OPT_WGRAD_TILE,      // "wgrad_tile"
  OPT_MARCH_STAGE,     // "march_stage"
  OPT_COUNT
};
int64_t option(Option o);

// compile-time hidden-block count for a runtime MLP width (32, 64, 96, 128, 256)
#define NRT_NB_SWITCH(nbv, ...)                               \
  switch (nbv) {                                              \
    case 2: { constexpr int NB = 2; __VA_ARGS__; } break;     \
    case 3: { constexpr int NB = 3; __VA_ARGS__; } break;     \
    case 4: { constexpr int NB = 4; __VA_ARGS__; } break;     \
    case 8: { constexpr int NB = 8; __VA_ARGS__; } break;     \
    default: { constexpr int NB = 1; __VA_ARGS__; } break;    \
  }

static inline int ceil_div64(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

// LDS layout of one launch: per-wave floats and waves per 64-thread-multiple block
struct LdsPlan {
  int RS = 1;         // FP32 slab stride
  int ys = 1;         // Y stride
  int per_wave = 0;   // floats
  int waves = 4;      // waves per block
  size_t bytes = 0;
};

static inline int opt_max_waves() {
  const int64_t v = option(OPT_MAX_WAVES);
  return v >= 1 && v <= 4 ? (int)v : 4;
}

static inline LdsPlan plan_lds(int hidden, int ke, int ys, bool f16, bool with_grad, int max_waves = 4) {
  LdsPlan p;
  max_waves = std::min(max_waves, opt_max_waves());
  p.ys = std::max(ys, 1);
  p.RS = f16 ? 1 : slab_stride(std::max(hidden, 32), std::max(ke, 16), with_grad);
  p.per_wave = wave_lds_floats(p.RS, p.ys, f16);
  int per_wave_bytes = p.per_wave * 4;
  p.waves = std::max(1, std::min(max_waves, kLdsBytes / std::max(per_wave_bytes, 1)));
  p.bytes = (size_t)p.waves * per_wave_bytes;
  return p;
}

// Re-cut an LDS-bound plan into the block size that fits the most waves per CU (at most 2 per
// SIMD): waves are independent, so a 29 KB-a-wave FP32 slab (the 6x96 NeuralBSDF) runs as five
// one-wave blocks per CU instead of one four-wave block.
static inline void spread_waves(LdsPlan& p) {
  const int per_cu = std::min(8, kLdsBytes / std::max(p.per_wave * 4, 1));
  int b = std::min(p.waves, per_cu);
  while (b > 1 && (per_cu / b) * b < per_cu) --b;
  p.waves = std::max(1, b);
  p.bytes = (size_t)p.waves * p.per_wave * 4;
}

template <typename K>
static inline int set_lds(K kernel, size_t bytes) {
  if (bytes > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e != hipSuccess) return hip_fail(e, "hipFuncSetAttribute(MaxDynamicSharedMemorySize)");
  }
  return NRT_OK;
}

// MarchArgs::stage (option "march_stage"): the per-wave line stages (LineStage) after the rest
// of the block's LDS, when the launch queue is on and they fit in the CU's 160 KiB
static inline void stage_lds(MarchArgs& a, size_t& lds, int waves) {
  if (!a.queue || option(OPT_MARCH_STAGE) == 0) return;
  const size_t off = (lds + 15) & ~(size_t)15;
  const size_t need = off + (size_t)waves * kStageBytes;
  if (off == 0 || need > 160 * 1024) return;
  a.stage = (int)off;
  lds = need;
}

static inline int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return hip_fail(e, what);
  return NRT_OK;
}

static inline int sdf_dims(const nrt_sdf* s, int& hidden, int& ke) {
  hidden = 32; ke = 16;
  if (s->mlp) { hidden = s->mlp->desc.hidden; ke = s->mlp->host_dev.ke; }
  return NRT_OK;
}

// ---- FP16 ring engine (nrt_ring_march.hip / nrt_ring_normal.hip) ----
// Configurations with a compiled ring kernel: 8 hidden layers of 128/256, skip 3, F = 16/32
// (3 or 5 encoding k-steps), 3 inputs, no latent, <= 32 outputs.
inline bool ring_supported(const nrt_sdf* s) {
  // a refreshed handle's FP16 ring stream is re-rounded by nrt_mlp_refresh (nrt_refresh.hip)
  if (!s->mlp || (s->mlp->refreshed && !s->mlp->ring16_refreshed)) return false;
  const MlpDev& m = s->mlp->host_dev;
  const int ne = m.ke / 16;
  return (m.nb == 8 || m.nb == 4) && (ne == 3 || ne == 5) && s->mlp->desc.num_layers == 8 &&
         s->mlp->desc.skip == 3 && s->mlp->desc.out <= 32 && m.in_size == 3 && m.latent == 0 &&
         m.freqs == 8 * (ne - 1);
}

inline size_t ring_bias_bytes(const nrt_sdf* s) {
  return (size_t)(s->mlp->desc.num_layers + 2) * s->mlp->host_dev.bias16_stride * 4;
}

// kWV waves per block share one LDS weight ring
#ifndef NRT_RING_WAVES
#define NRT_RING_WAVES 8
#endif
constexpr int kRingWaves = NRT_RING_WAVES;

// call F.template operator()<NB, NE, FOLD>() for the SDF's ring configuration
template <class F>
int ring_dispatch(const nrt_sdf* s, F&& f) {
  const MlpDev& m = s->mlp->host_dev;
  const int ne = m.ke / 16;
  const bool fold = m.fold != 0;
#define NRT_RING_CASE(NBV, NEV)                                               \
  if (m.nb == NBV && ne == NEV)                                               \
    return fold ? f.template operator()<NBV, NEV, true>() : f.template operator()<NBV, NEV, false>();
  NRT_RING_CASE(8, 3)
  NRT_RING_CASE(8, 5)
  NRT_RING_CASE(4, 3)
  NRT_RING_CASE(4, 5)
#undef NRT_RING_CASE
  set_error("ring engine: unsupported SDF configuration");
  return NRT_EINVAL;
}

int ring_march(const nrt_sdf* s, const float* rays, int64_t P, const MarchArgs& ma, float* t,
               uint8_t* hit, float* p, float* n, float* raw_n, float* thr, int32_t* idx,
               int32_t* cnt, unsigned long long* keys, hipStream_t st);
// k_march16 alone (packed t, scan keys; the caller initialises keys): NRT_MIXED's first pass;
// with `visible`, the shadow march k_occl16 instead (MarchArgs::occ_max_t / count)
int ring_march16_launch(const nrt_sdf* s, const float* rays, int64_t P, const MarchArgs& ma,
                        float* t, float* thr, unsigned long long* keys, hipStream_t st,
                        bool best16, uint8_t* visible = nullptr);

// ---- FP32 ring engine (nrt_ring_march32.hip) ----
// SDF MLPs with a compiled FP32 ring kernel: hidden 128 / 256, F = 16 / 32 with 3 inputs and no
// latent (ke = 48 / 80), <= 16 outputs, softplus or leaky_relu; any layer count and skip period.
// Refreshed handles qualify (nrt_mlp_refresh re-gathers stream32).
constexpr int kRing32Waves = 8;
inline size_t ring32_bias_bytes(const nrt_sdf* s) {
  return (size_t)(s->mlp->desc.num_layers + 2) * s->mlp->host_dev.bias16_stride * 4;
}
inline size_t ring32_sphere_bytes(const nrt_sdf* s) {
  // the per-sphere table (ring3) or the FP32 ring's pair table (ring32::build_sphere_pairs32)
  if (s->host_dev.kind != 2) return 0;
  const size_t one = (size_t)s->host_dev.n_spheres * 64;
  const size_t pairs = (size_t)4 * ring32::sphere_pairs32(s->host_dev.n_spheres) * ring32::kPair32F4 * 16;
  return one > pairs ? one : pairs;
}
inline bool ring32_supported(const nrt_sdf* s) {
  if (!s->mlp) return false;
  const MlpDev& m = s->mlp->host_dev;
  const int act = s->mlp->desc.activation;
  if (!((m.hidden == 128 || m.hidden == 256) && (m.ke == 48 || m.ke == 80) && m.in_size == 3 &&
        m.latent == 0 && m.out <= 16 && (act == NRT_ACT_SOFTPLUS || act == NRT_ACT_LEAKY_RELU)))
    return false;
  return ring32_sphere_bytes(s) + ring32_bias_bytes(s) <= 48 * 1024;
}
int ring_march32(const nrt_sdf* s, const float* rays, int64_t P, const MarchArgs& ma, float* t,
                 uint8_t* hit, float* p, float* n, float* raw_n, float* thr, int32_t* idx,
                 int32_t* cnt, unsigned long long* keys, hipStream_t st);
// k_scan_best32 alone: thr = -1000 sdf(best) on the FP32 engine at the argmins in keys
int ring_scan_best32(const nrt_sdf* s, const float* rays, int64_t P, const MarchArgs& ma,
                     float* thr, unsigned long long* keys, hipStream_t st);
// ---- fp32-split ring engine (nrt_ring_march3.hip, nrt_ring3.h): the ring32 configurations,
// from a handle packed by nrt_mlp_create or refreshed by nrt_mlp_refresh (which re-splits it)
constexpr int kRing3Waves = 8;
inline bool ring3_supported(const nrt_sdf* s) {
  if (!s->mlp || (s->mlp->refreshed && !s->mlp->split_refreshed)) return false;
  const MlpDev& m = s->mlp->host_dev;
  return ring32_supported(s) && (m.ke3 == 64 || m.ke3 == 96);
}
int ring_eval3(const nrt_sdf* s, const float* pts, int64_t M, float* out, hipStream_t st);
int ring_march3(const nrt_sdf* s, const float* rays, int64_t P, const MarchArgs& ma, float* t,
                uint8_t* hit, float* p, float* n, float* raw_n, float* thr, int32_t* idx,
                int32_t* cnt, unsigned long long* keys, hipStream_t st);
// the split engine's launches alone: which = 0 k_march3 (+ k_scan_best3 when primary), 1
// k_scan_best3 (the caller initialises keys); 2 / 3 the same as NRT_MIXED's refinement passes;
// 4 the shadow march k_occl3 (visible -> hit)
int ring3_launch(const nrt_sdf* s, const float* rays, int64_t P, const MarchArgs& ma, float* t,
                 float* thr, unsigned long long* keys, hipStream_t st, int which,
                 uint8_t* hit = nullptr);
// the FP32 ring's shadow march k_occl32
int ring_occlusion32(const nrt_sdf* s, const float* rays, int64_t P, const MarchArgs& ma,
                     uint8_t* visible, hipStream_t st);
// NRT_MIXED intersect (nrt_ring_mixed.hip): FP16 march + scan, split refinement of the
// undecidable steps and scan orders, split sdf(best); same outputs as ring_march
// The FP16 SDF error of the headline scene (tools/fp16_decompose.py, 1M scan points and the
// FP32 march's 279k stop points): median 1.9e-5, 99.99 % 5.6e-5, max 7.3e-5.  The march bound
// is larger: a ray that converges slowly (grazing) turns t's drift into a one-step flip whose
// FP16 values still sit well away from eps.  Measured on the 800^2 frame (tools/mixed_sweep.py,
// restart on): d = 1.2e-4 -> 4 step flips, 5,557 pixels > 1e-4, 125.4 ms; 5e-4 -> 920 pixels,
// 130.0 ms; 2e-3 -> 4 pixels (fp32-split's own count), 133.4 ms
constexpr int64_t kMixedRefineD = 20000;  // 2e-3
constexpr int64_t kMixedRefineS = 2000;   // 2e-4: two values' errors (<= 7.3e-5 each), with margin
inline bool mixed_supported(const nrt_sdf* s) { return ring_supported(s) && ring3_supported(s); }
inline size_t mixed_ws_bytes(int64_t P) {
  // keys2 | amb (reused as kbest) | list | count
  return 2 * (((size_t)P * 8 + 255) & ~(size_t)255) + (((size_t)P * 4 + 255) & ~(size_t)255) + 256;
}
int ring_march_mixed(const nrt_sdf* s, const float* rays, int64_t P, const MarchArgs& ma, float* t,
                     uint8_t* hit, float* p, float* n, float* raw_n, float* thr, int32_t* idx,
                     int32_t* cnt, unsigned long long* keys, char* mixed_ws, hipStream_t st);
// workspace of ring_march: one 64-bit scan key per ray
// scan keys (P x u64) | the job-queue counter (MarchArgs::queue)
inline size_t ring_march_ws_bytes(int64_t P) { return (((size_t)P * 8 + 255) & ~(size_t)255) + 256; }
inline unsigned int* ring_march_queue(char* keys_base, int64_t P) {
  return reinterpret_cast<unsigned int*>(keys_base + (((size_t)P * 8 + 255) & ~(size_t)255));
}
int ring_normals32(const nrt_sdf* s, const int32_t* idx, const int32_t* cnt, int64_t M, float* grad,
                   float* n, float* p_io, float eps, bool split, hipStream_t st);
int ring_normals(const nrt_sdf* s, const int32_t* idx, const int32_t* cnt, int64_t M, float* grad,
                 float* n, float* p_io, float eps, hipStream_t st);

// shadow march (intersect_test) on the ring engine of `precision` (FP16 ring, FP32 ring, split
// ring for fp32-split / mixed), or the per-wave k_occlusion where no ring kernel is compiled
int launch_occlusion(const nrt_sdf* s, const float* rays, int64_t P, const int32_t* count,
                     const float* max_t, int32_t max_steps, float eps, uint8_t* visible,
                     int precision, hipStream_t st);

// ---- shading programs (nrt_prog.hip) ----
int build_program(const std::vector<const nrt_mlp*>& mlps, nrt_prog& out);
int build_light_program(nrt_light* l);
int build_bsdf_program(nrt_bsdf* b);
int shade_program(const nrt_bsdf* b, const nrt_light* l, const float* p, const float* n,
                  const float* wi, const int32_t* hit_idx, const int32_t* hit_count, int64_t P,
                  const float* lscale, float* rgb, float* weights_out, hipStream_t st);

// ---- FP32 / fp32-split shading on the row-program ring engines (nrt_shade_ring.hip) ----
int build_rprog(const std::vector<const nrt_mlp*>& mlps, bool split, nrt_rprog& out, int mode = 0);
int solo_forward(const nrt_mlp* m, const float* x, int64_t M, float* y, hipStream_t st);
constexpr int kMaxSoloForward = 16;  // MLPs of one solo_forward_multi launch (rprog::kMaxSoloJobs)
// save (nullable; else one buffer per MLP, saved_bytes each): the training forward, which also
// stores the activations the ring backward reads (ring_backward with Ms >= 0)
int solo_forward_multi(const nrt_mlp* const* mlps, int n, const float* x, int64_t M,
                       float* const* y, hipStream_t st, void* const* save = nullptr);
bool saved_forward_ok(const nrt_mlp* m);
// one MLP's saved activations: A [L+1][M][H] | Eraw [M][dp] | Eact [M][dp], 256-byte aligned
struct SavedActs {
  float *A, *Eraw, *Eact;
};
inline size_t saved_part(size_t b) { return (b + 255) & ~(size_t)255; }
inline size_t saved_bytes(const MlpDev& d, int64_t M) {
  return saved_part((size_t)(d.n_hidden + 1) * M * d.hidden * 4) + 2 * saved_part((size_t)M * d.dp * 4);
}
inline SavedActs saved_split(const MlpDev& d, int64_t M, const void* base) {
  char* p = (char*)base;
  SavedActs s;
  s.A = (float*)p;
  p += saved_part((size_t)(d.n_hidden + 1) * M * d.hidden * 4);
  s.Eraw = (float*)p;
  p += saved_part((size_t)M * d.dp * 4);
  s.Eact = (float*)p;
  return s;
}
bool solo_refresh_maps(const nrt_mlp* m, std::vector<int>& stream_map, std::vector<int>& bias_map,
                       void*& stream_dst, void*& bias_dst);
int shade_ring(const nrt_bsdf* b, const nrt_light* l, const float* p, const float* n,
               const float* wi, const int32_t* hit_idx, const int32_t* hit_count, int64_t P,
               const float* lscale, float* rgb, float* weights_out, int precision, hipStream_t st);
// ---- the MLP backward on the ring engine (nrt_train_ring.h, launched from nrt_shade_ring.hip) --
// the bytes of the device job table ring_backward needs for n MLPs
size_t ring_backward_table_bytes(int n);
// true when every MLP has a ring-backward shape (and, refreshed, a refreshed backward program)
bool ring_backward_ok(const nrt_mlp* const* mlps, int n);
// per MLP k: dy[k] [M][out], dx[k] [M][3] or null, A[k] / dZ[k] [L+1][M][H], Eraw[k] / Eact[k]
// [M][dp]; table: ring_backward_table_bytes(n) bytes of device memory.  Ms >= 0: A[k] holds the
// training forward's saved activations [L+1][Ms][H] and Sraw[k] / Sact[k] its encoding [Ms][dp]
// (row i of this backward = saved row rows[i], or i when rows is null); only the backward chain
// runs; with rows, the saved rows it reads are copied to Acopy[k] [L+1][M][H] and Eraw[k] /
// Eact[k] [M][dp] (the weight gradients' operands, row-aligned with dZ).
int ring_backward(const nrt_mlp* const* mlps, int n, const float* x, int64_t M,
                  const float* const* dy, float* const* dx, float* const* A, float* const* dZ,
                  float* const* Eraw, float* const* Eact, void* table, hipStream_t st,
                  const int32_t* rows = nullptr, int64_t Ms = -1, float* const* Acopy = nullptr,
                  const float* const* Sraw = nullptr, const float* const* Sact = nullptr);
bool bwd_refresh_maps(const nrt_mlp* m, std::vector<int>& stream_map, std::vector<int>& bias_map,
                      void*& stream_dst, void*& bias_dst);

}  // namespace nrt
