// nrt_internal.h -- host-side objects behind the opaque C handles of include/nrt.h
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "../../include/nrt.h"
#include "nrt_device.h"

struct nrt_prog;

// A row program (RProgDev) for the FP32 / fp32-split shading kernels (nrt_shade_ring.hip), built on
// first use from the host copies of the MLPs' weights.
struct nrt_rprog {
  nrt::RProgDev d{};
  void* buf = nullptr;
  bool built = false;    // build attempted
  bool ok = false;       // false: some MLP has a shape without a compiled kernel
  int fwd_chunks = 0;    // backward programs (build_rprog mode 1): chunks of the forward part
  ~nrt_rprog() { if (buf) (void)hipFree(buf); }
};

struct nrt_mlp {
  nrt_mlp_desc desc;
  nrt::MlpDev host_dev;          // host copy of the device descriptor
  nrt::MlpDev* dev = nullptr;    // device copy
  void* blob = nullptr;          // all packed arrays
  size_t blob_bytes = 0;
  // host copies used to assemble shading programs (nrt_prog.hip)
  std::vector<int> host_chunkk;  // k-outer chunk offsets
  std::vector<float> host_bias;  // unfolded biases [layer][bias16_stride]
  std::vector<float> host_basis; // [in][F]
  std::vector<std::vector<float>> host_w;  // original weights per linear (init, hidden..., out)
  // fused NeRFLE program built for (nerf_first, this) on first use (nrt_api_nerf.hip)
  mutable std::unique_ptr<nrt_prog> nerf_prog;
  mutable uint64_t nerf_first_serial = 0;
  // NeRF+LE: the envmap the program's folded light column was built for (empty: point light)
  mutable std::vector<float> nerf_env;
  uint64_t serial = 0;  // unique per created MLP (cache key; addresses can be reused)
  // nrt_mlp_refresh (nrt_refresh.hip): gather maps of the per-kernel fragment arrays, built on
  // the first refresh; after a refresh the FP16 ring / program streams and the host copies
  // above are stale and the handle only serves nrt_mlp_forward / _backward / _grad_backward
  int* gather_map = nullptr;     // [n_gather] source index into [W_0..W_L+1 | b_0..b_L+1] or -1
  float* gather_src = nullptr;   // staging copy of the caller's weights and biases
  int64_t n_src = 0;
  std::vector<void*> gather_dst;   // per section: destination array, element count, FP16?
  std::vector<int64_t> gather_n;
  std::vector<char> gather_f16;   // section kind (nrt_refresh.hip SecKind)
  bool refreshed = false;
  bool split_refreshed = false;  // the refresh also re-split stream3 (fp32-split march)
  bool ring16_refreshed = false;  // ... and re-rounded stream16 (FP16 / mixed march)
  // single-MLP FP32 row program (nrt_shade_ring.hip) for nrt_mlp_forward on the ring engine;
  // nrt_mlp_refresh gathers its stream and bias table too once it exists
  mutable nrt_rprog solo32;
  bool solo_in_refresh = false;  // the refresh maps cover solo32
  // [forward | transposed] FP32 row program of the ring backward (nrt_train_ring.h), built on
  // first use; nrt_mlp_refresh gathers it too once it is in the maps
  mutable nrt_rprog bwd32;
  bool bwd_in_refresh = false;
  ~nrt_mlp();
};

// A device program (ProgDev) and the buffer holding its stream, chunk table, biases and basis.
struct nrt_prog {
  nrt::ProgDev d{};
  void* buf = nullptr;
  const float* unit_light = nullptr;  // NeRF+LE fold: (1, 0, 0) in buf, the kernel's light input
  bool ok = false;       // false: some MLP has a shape without a compiled program kernel
  ~nrt_prog() { if (buf) (void)hipFree(buf); }
};

struct nrt_sdf {
  nrt::SdfDev host_dev;
  nrt::SdfDev* dev = nullptr;
  float* spheres = nullptr;
  const nrt_mlp* mlp = nullptr;
};

namespace nrt {

struct LightDev {
  int kind;                 // 0 field, 1 point
  const MlpDev* mlp;
  float color_sig[3];       // sigmoid(color)
  float loc[3];
  float scaled_dir[3];      // scale * normalize(intensity) (falloff 0), scale * intensity (1)
  float c, l, q;            // clamped falloff coefficients
  int falloff;              // point lights: 0 the pathtracer's (lights.py:89-110), 1 the
                            // renderer's inverse square (renderer/lighting.py:283-304)
};

constexpr int kMaxComponents = 32;

struct BsdfCompDev {
  int kind;
  const MlpDev* mlp;
  int act;
  float params[4];
};

struct BsdfDev {
  int n;
  const MlpDev* spatial;
  BsdfCompDev comp[kMaxComponents];
};

}  // namespace nrt

struct nrt_light {
  nrt::LightDev host_dev;
  nrt::LightDev* dev = nullptr;
  const nrt_mlp* mlp = nullptr;
  nrt_prog prog;          // [light field MLP]
  mutable nrt_rprog rprog[2];  // FP32, fp32-split: [light field MLP]
};

struct nrt_bsdf {
  nrt::BsdfDev host_dev;
  nrt::BsdfDev* dev = nullptr;
  std::vector<const nrt_mlp*> mlps;
  const nrt_mlp* spatial = nullptr;
  nrt_prog prog;          // [spatial] + neural components, in component order
  mutable nrt_rprog rprog[2];  // FP32, fp32-split: same order
};

namespace nrt {
// launch timing registry (nrt_profile_*); begin/end are no-ops unless enabled
struct ProfScope {
  const char* name;
  hipStream_t stream;
  hipEvent_t start = nullptr;
  double flop = 0.0;  // algorithmic FLOP of the bracketed launches (nrt_profile_flop)
  ProfScope(const char* n, hipStream_t s, double flop = 0.0);
  ~ProfScope();
};
void set_error(const std::string& msg);
int hip_fail(hipError_t e, const char* what);
int max_hidden(const nrt_mlp* m);
// device counter of executed ray-evaluations of the ring marches while profiling is enabled
// (nullptr otherwise); read and cleared by nrt_profile_evals / nrt_profile_reset
unsigned long long* profile_eval_counter();

// Element order of the FP32 ring stream (MlpDev::stream32, consumed by nrt_device.h ring32 with
// v_mfma_f32_16x16x4_f32 on 16-ray tiles).  Shared by the packer (values, nrt_pack.hip) and the
// refresh map (source indices, nrt_refresh.hip).  f(layer, row, pos) is called once per stream
// float, in order; pos is the layer input: hidden feature k in [0, H) or H + encoding slot; rows
// past the layer's R are padding.
//   chunk = 64 output rows (ring32::kSub = 4 sub-blocks of 16) of one layer; the out layer is one
//   chunk of one sub-block (rows 0..15).  A chunk is quads u = 0 .. qh + qe - 1 (qh = H / 16
//   hidden, qe = ke / 16 encoding quads; the eval takes a skip layer's encoding quads as a chunk of
//   their own), each quad [sub-block b][lane][t] = 1 KiB per sub-block: lane (g =
//   lane >> 4, i = lane & 15) holds A[row 16 b + i][k = g] of k-steps 4u + t.  Hidden k-step s
//   takes feature 16 (s >> 2) + 4 g + (s & 3) in lane group g -- register s & 3 of sub-block s >> 2
//   of the previous layer's 16x16 accumulator -- and encoding k-step e takes slot 4 e + g.
struct Ring32Layer {
  int R;
  bool hid, enc;
};
template <class F>
inline void ring32_walk(const std::vector<Ring32Layer>& ls, int H, int ke, F&& f) {
  constexpr int S = ring32::kSub;  // sub-blocks per chunk (64 output rows)
  for (size_t l = 0; l < ls.size(); ++l) {
    const bool out = l + 1 == ls.size();
    const int nsub = out ? 1 : S, nch = out ? 1 : (ls[l].R + 16 * S - 1) / (16 * S);
    const int qh = ls[l].hid ? H / 16 : 0, qe = ls[l].enc ? ke / 16 : 0;
    for (int c = 0; c < nch; ++c)
      for (int u = 0; u < qh + qe; ++u)
        for (int b = 0; b < nsub; ++b)
          for (int lane = 0; lane < 64; ++lane)
            for (int t = 0; t < 4; ++t) {
              const int s = 4 * u + t, g = lane >> 4;
              const int pos = u < qh ? 16 * (s >> 2) + 4 * g + (s & 3) : H + 4 * (s - 4 * qh) + g;
              f((int)l, 16 * S * c + 16 * b + (lane & 15), pos);
            }
  }
}

// Element order of the split stream (MlpDev::stream3, consumed by nrt_ring3.h with
// v_mfma_f32_16x16x32_f16 on 16-ray tiles).  f(layer, row, pos, part) is called once per stream
// half, in order (part 0 = hi, 1 = lo); pos as in ring32_walk (hidden feature k < H, or H +
// encoding slot; rows past the layer's R are padding).
//   chunk = 32 output rows (sub-blocks b = 0, 1 of 16) of one layer; the out layer is one chunk of
//   one sub-block.  A chunk is k-steps u = 0 .. kh + kq - 1 (kh = H / 32 hidden, kq = ke3 / 32
//   encoding k-steps), each [sub-block b][part][lane][e] = 1 KiB per (b, part): lane (g = lane >> 4,
//   i = lane & 15) holds A[row 16 b + i][k = 8 g + e] of k-step u.  Hidden k-step u takes feature
//   16 (2u + (e >> 2)) + 4 g + (e & 3) -- register e & 3 of sub-block 2u + (e >> 2) of the previous
//   layer's 16x16 accumulators, which is chunk u of that layer -- and encoding k-step v takes slot
//   32 v + 8 g + e.
template <class F>
inline void ring3_walk(const std::vector<Ring32Layer>& ls, int H, int ke3, F&& f) {
  for (size_t l = 0; l < ls.size(); ++l) {
    const bool out = l + 1 == ls.size();
    const int nsub = out ? 1 : 2, nch = out ? 1 : (ls[l].R + 31) / 32;
    const int kh = ls[l].hid ? H / 32 : 0, kq = ls[l].enc ? ke3 / 32 : 0;
    for (int c = 0; c < nch; ++c)
      for (int u = 0; u < kh + kq; ++u)
        for (int b = 0; b < nsub; ++b)
          for (int part = 0; part < 2; ++part)
            for (int lane = 0; lane < 64; ++lane)
              for (int e = 0; e < 8; ++e) {
                const int g = lane >> 4;
                const int pos = u < kh ? 16 * (2 * u + (e >> 2)) + 4 * g + (e & 3)
                                       : H + 32 * (u - kh) + 8 * g + e;
                f((int)l, 32 * c + 16 * b + (lane & 15), pos, part);
              }
  }
}
}  // namespace nrt

#define NRT_HIP(call)                                         \
  do {                                                        \
    hipError_t _e = (call);                                   \
    if (_e != hipSuccess) return nrt::hip_fail(_e, #call);    \
  } while (0)
