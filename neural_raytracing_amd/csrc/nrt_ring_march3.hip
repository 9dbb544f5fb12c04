// fp32-split march + coarse scan (k_march3 / k_scan_best3, nrt_ring3.h): the FP32 ring's job
// lists, persistent grid and 16-ray tiles, with every SDF MLP layer on FP16 MFMA at FP32 accuracy
// (hi/lo operand halves, three products per block).
#include "nrt_launch.h"

namespace nrt {

// sdf(p) of M points [M, 3] -> out [M] on the split engine (march_body mode 2)
int ring_eval3(const nrt_sdf* s, const float* pts, int64_t M, float* out, hipStream_t st) {
  const MlpDev& md = s->mlp->host_dev;
  const size_t extra = (size_t)md.freqs * 16 + ring32_bias_bytes(s) + ring32_sphere_bytes(s);
  int dev = 0, cus = 0;
  NRT_HIP(hipGetDevice(&dev));
  NRT_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  MarchArgs ma{};
  auto run = [&]<int KH, int KQ, int ACT>() -> int {
    constexpr int WV = kRing3Waves;
    auto kern = k_sdf_eval3<KH, KQ, WV, ACT>;
    const size_t lds = ring3::Engine<KH, KQ, WV>::RING_BYTES + extra;
    if (int rc = set_lds(kern, lds)) return rc;
    int per_cu = 0;
    NRT_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64 * WV, lds));
    const int64_t slots = (int64_t)std::max(per_cu, 1) * std::max(cus, 1);
    const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(slots, ceil_div64(M, 16 * WV)));
    ProfScope prof("k_sdf_eval3", st);
    kern<<<dim3(blocks), dim3(64 * WV), lds, st>>>(s->host_dev, md, pts, M, ma, nullptr, nullptr,
                                                   nullptr, nullptr, nullptr, out, nullptr);
    return check_launch("k_sdf_eval3");
  };
  const bool sp = s->mlp->desc.activation == NRT_ACT_SOFTPLUS;
#define NRT_R3(H, KQV)                                                                   \
  if (md.hidden == H && md.ke3 == 32 * KQV)                                              \
    return sp ? run.template operator()<H / 32, KQV, ACT_SOFTPLUS>()                     \
              : run.template operator()<H / 32, KQV, ACT_LEAKY>();
  NRT_R3(256, 2) NRT_R3(256, 3) NRT_R3(128, 2) NRT_R3(128, 3)
#undef NRT_R3
  set_error("fp32-split ring engine: unsupported SDF configuration");
  return NRT_EINVAL;
}

int ring3_launch(const nrt_sdf* s, const float* rays, int64_t P, const MarchArgs& ma, float* t,
                 float* thr, unsigned long long* keys, hipStream_t st, int which, uint8_t* hit) {
  const MlpDev& md = s->mlp->host_dev;
  const size_t extra = (size_t)md.freqs * 16 + ring32_bias_bytes(s) + ring32_sphere_bytes(s);
  int dev = 0, cus = 0;
  NRT_HIP(hipGetDevice(&dev));
  NRT_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const bool scan = ma.primary != 0;
  auto run = [&]<int KH, int KQ, int ACT>() -> int {
    constexpr int WV = kRing3Waves;
    auto launch = [&](auto kern, const char* name, bool plain = false) -> int {
      size_t lds = ring3::Engine<KH, KQ, WV>::RING_BYTES + extra;
      MarchArgs mb = ma;
      if (plain) stage_lds(mb, lds, WV);  // the plain march's line stages (one block a CU)
      if (int rc = set_lds(kern, lds)) return rc;
      int per_cu = 0;
      NRT_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64 * WV, lds));
      const int64_t slots = (int64_t)std::max(per_cu, 1) * std::max(cus, 1);
      int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(slots, ceil_div64(P, 16 * WV)));
      if (const int64_t f = option(OPT_MARCH_BLOCKS)) blocks = (int)std::min<int64_t>(f, 1 << 20);
      if (ma.queue) NRT_HIP(hipMemsetAsync(ma.queue, 0, sizeof(unsigned int), st));
      ProfScope prof(name, st);
      // p / n / raw_n: written by k_march_finish (the march packs hit into t's sign bit)
      kern<<<dim3(blocks), dim3(64 * WV), lds, st>>>(s->host_dev, md, rays, P, mb, t, hit,
                                                     nullptr, nullptr, nullptr, thr, keys);
      return check_launch(name);
    };
    // profile names: the NRT_MIXED refinement launches (which 2 / 3) apart from the plain ones
    if (which == 4) return launch(k_occl3<KH, KQ, WV, ACT>, "k_occl3");
    if (which == 2) return launch(k_march3<KH, KQ, WV, ACT, true>, "k_refine3");
    if (which == 3) return launch(k_scan_best3<KH, KQ, WV, ACT, true>, "k_best3");
    if (which == 0)
      if (int rc = launch(k_march3<KH, KQ, WV, ACT>, "k_march3", true)) return rc;
    if (scan) return launch(k_scan_best3<KH, KQ, WV, ACT>, "k_scan_best3");
    return NRT_OK;
  };
  const bool sp = s->mlp->desc.activation == NRT_ACT_SOFTPLUS;
  int rc = NRT_EINVAL;
#define NRT_R3(H, KQV)                                                                   \
  if (md.hidden == H && md.ke3 == 32 * KQV)                                              \
    rc = sp ? run.template operator()<H / 32, KQV, ACT_SOFTPLUS>()                       \
            : run.template operator()<H / 32, KQV, ACT_LEAKY>();                         \
  else
  NRT_R3(256, 2) NRT_R3(256, 3) NRT_R3(128, 2) NRT_R3(128, 3) {
    set_error("fp32-split ring engine: unsupported SDF configuration");
    return NRT_EINVAL;
  }
#undef NRT_R3
  return rc;
}

int ring_march3(const nrt_sdf* s, const float* rays, int64_t P, const MarchArgs& ma, float* t,
                uint8_t* hit, float* p, float* n, float* raw_n, float* thr, int32_t* idx,
                int32_t* cnt, unsigned long long* keys, hipStream_t st) {
  if (ma.primary) NRT_HIP(hipMemsetAsync(keys, 0xff, (size_t)P * sizeof(unsigned long long), st));
  if (int rc = ring3_launch(s, rays, P, ma, t, thr, keys, st, 0)) return rc;
  k_march_finish<><<<dim3(std::min<int64_t>(ceil_div64(P, 256), 2048)), dim3(256), 0, st>>>(
      rays, P, t, hit, p, n, raw_n, idx, cnt);
  return check_launch("k_march_finish");
}

}  // namespace nrt
