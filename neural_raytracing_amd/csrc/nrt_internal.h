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
  uint64_t serial = 0;  // unique per created MLP (cache key; addresses can be reused)
  // nrt_mlp_refresh (nrt_refresh.hip): gather maps of the per-kernel fragment arrays, built on
  // the first refresh; after a refresh the FP16 ring / program streams and the host copies
  // above are stale and the handle only serves nrt_mlp_forward / _backward / _grad_backward
  int* gather_map = nullptr;     // [n_gather] source index into [W_0..W_L+1 | b_0..b_L+1] or -1
  float* gather_src = nullptr;   // staging copy of the caller's weights and biases
  int64_t n_src = 0;
  std::vector<void*> gather_dst;   // per section: destination array, element count, FP16?
  std::vector<int64_t> gather_n;
  std::vector<char> gather_f16;
  bool refreshed = false;
  ~nrt_mlp();
};

// A device program (ProgDev) and the buffer holding its stream, chunk table, biases and basis.
struct nrt_prog {
  nrt::ProgDev d{};
  void* buf = nullptr;
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
  float scaled_dir[3];      // scale * normalize(intensity)
  float c, l, q;            // clamped falloff coefficients
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
};

struct nrt_bsdf {
  nrt::BsdfDev host_dev;
  nrt::BsdfDev* dev = nullptr;
  std::vector<const nrt_mlp*> mlps;
  const nrt_mlp* spatial = nullptr;
  nrt_prog prog;          // [spatial] + neural components, in component order
};

namespace nrt {
// launch timing registry (nrt_profile_*); begin/end are no-ops unless enabled
struct ProfScope {
  const char* name;
  hipStream_t stream;
  hipEvent_t start = nullptr;
  ProfScope(const char* n, hipStream_t s);
  ~ProfScope();
};
void set_error(const std::string& msg);
int hip_fail(hipError_t e, const char* what);
int max_hidden(const nrt_mlp* m);
}  // namespace nrt

#define NRT_HIP(call)                                         \
  do {                                                        \
    hipError_t _e = (call);                                   \
    if (_e != hipSuccess) return nrt::hip_fail(_e, #call);    \
  } while (0)
