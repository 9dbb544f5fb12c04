// FP32 / fp32-split forward-mode SDF normals on the ring32 / ring3 engines (k_normal32 /
// k_normal3 = k_normal_r, nrt_kernels.h): the normal pass of nrt_sdf_intersect after a ring32 /
// ring3 march, in place of the per-wave reverse-mode k_sdf_grad.
#include "nrt_launch.h"

namespace nrt {

int ring_normals32(const nrt_sdf* s, const int32_t* idx, const int32_t* cnt, int64_t M, float* grad,
                   float* n, float* p_io, float eps, bool split, hipStream_t st) {
  const MlpDev& md = s->mlp->host_dev;
  const size_t extra = (size_t)md.freqs * 16 + ring32_bias_bytes(s) + ring32_sphere_bytes(s);
  int dev = 0, cus = 0;
  NRT_HIP(hipGetDevice(&dev));
  NRT_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  auto launch = [&](auto kern, size_t ring_bytes, int WV, const char* name) -> int {
    const size_t lds = ring_bytes + extra;
    if (int rc = set_lds(kern, lds)) return rc;
    int per_cu = 0;
    NRT_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64 * WV, lds));
    const int64_t slots = (int64_t)std::max(per_cu, 1) * std::max(cus, 1);
    const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(slots, ceil_div64(M, 4 * WV)));
    ProfScope prof(name, st);
    kern<<<dim3(blocks), dim3(64 * WV), lds, st>>>(s->host_dev, md, idx, cnt, M, grad, n, p_io, eps);
    return check_launch(name);
  };
  const bool sp = s->mlp->desc.activation == NRT_ACT_SOFTPLUS;
  if (split) {
    auto run = [&]<int KH, int KQ, int ACT>() -> int {
      constexpr int WV = kRing3Waves;
      return launch(k_normal_r<RingPol3<KH, KQ, WV, ACT>>, ring3::Engine<KH, KQ, WV>::RING_BYTES, WV,
                    "k_normal3");
    };
#define NRT_R3(H, KQV)                                                                   \
  if (md.hidden == H && md.ke3 == 32 * KQV)                                              \
    return sp ? run.template operator()<H / 32, KQV, ACT_SOFTPLUS>()                     \
              : run.template operator()<H / 32, KQV, ACT_LEAKY>();
    NRT_R3(256, 2) NRT_R3(256, 3) NRT_R3(128, 2) NRT_R3(128, 3)
#undef NRT_R3
  } else {
    auto run = [&]<int KH, int KE, int ACT>() -> int {
      constexpr int WV = kRing32Waves;
      return launch(k_normal_r<RingPol32<KH, KE, WV, ACT>>, ring32::Engine<KH, KE, WV>::RING_BYTES,
                    WV, "k_normal32");
    };
#define NRT_R32(H, KEV)                                                                   \
  if (md.hidden == H && md.ke == 4 * KEV)                                                 \
    return sp ? run.template operator()<H / 4, KEV, ACT_SOFTPLUS>()                       \
              : run.template operator()<H / 4, KEV, ACT_LEAKY>();
    NRT_R32(256, 12) NRT_R32(256, 20) NRT_R32(128, 12) NRT_R32(128, 20)
#undef NRT_R32
  }
  set_error("ring normals: unsupported SDF configuration");
  return NRT_EINVAL;
}

}  // namespace nrt
