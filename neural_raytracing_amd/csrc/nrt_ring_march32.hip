// FP32 (reference-precision) march + coarse scan on the block-cooperative LDS weight ring
// (k_march32 / k_scan_best32, nrt_device.h ring32): same job lists and persistent grid as the
// FP16 ring march (nrt_ring_march.hip), 16-ray tiles; accurate sincosf / sqrtf / expf and
// softplus_exact (a few ulp of torch's log1pf(expf), nrt_device.h).
#include "nrt_launch.h"

// waves per block of the 128-wide SDFs' FP32 ring march (timing experiments: -DNRT_R32_SMALL_WV)
#ifndef NRT_R32_SMALL_WV
#define NRT_R32_SMALL_WV 8
#endif

namespace nrt {

// which = 0: march + scan (k_march32, then k_scan_best32 when primary); 1: k_scan_best32 alone
// at the argmins already in `keys` (an FP16 march's scan, option "scan_best32"); 2: the shadow
// march k_occl32 (visible -> hit)
static int ring32_launch(const nrt_sdf* s, const float* rays, int64_t P, const MarchArgs& ma,
                         float* t, uint8_t* hit, float* p, float* n, float* raw_n, float* thr,
                         unsigned long long* keys, hipStream_t st, int which) {
  const MlpDev& md = s->mlp->host_dev;
  const size_t extra = (size_t)md.freqs * 16 + ring32_bias_bytes(s) + ring32_sphere_bytes(s);
  int dev = 0, cus = 0;
  NRT_HIP(hipGetDevice(&dev));
  NRT_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const bool scan = ma.primary != 0;
  if (scan && which == 0) NRT_HIP(hipMemsetAsync(keys, 0xff, (size_t)P * sizeof(unsigned long long), st));
  auto run = [&]<int KH, int KE, int ACT>() -> int {
    constexpr int WV = KH <= 32 ? NRT_R32_SMALL_WV : kRing32Waves;
    auto launch = [&](auto kern, const char* name, bool plain = false) -> int {
      size_t lds = ring32::Engine<KH, KE, WV>::RING_BYTES + extra;
      MarchArgs mb = ma;
      if (plain) stage_lds(mb, lds, WV);  // the march's line stages (one block a CU)
      if (int rc = set_lds(kern, lds)) return rc;
      int per_cu = 0;
      NRT_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64 * WV, lds));
      const int64_t slots = (int64_t)std::max(per_cu, 1) * std::max(cus, 1);
      int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(slots, ceil_div64(P, 16 * WV)));
      if (const int64_t f = option(OPT_MARCH_BLOCKS)) blocks = (int)std::min<int64_t>(f, 1 << 20);
      if (ma.queue) NRT_HIP(hipMemsetAsync(ma.queue, 0, sizeof(unsigned int), st));
      ProfScope prof(name, st);
      // p / n / raw_n: written by k_march_finish (the march packs hit into t's sign bit)
      kern<<<dim3(blocks), dim3(64 * WV), lds, st>>>(s->host_dev, md, rays, P, mb, t, hit, nullptr,
                                                     nullptr, nullptr, thr, keys);
      return check_launch(name);
    };
    if (which == 2) return launch(k_occl32<KH, KE, WV, ACT>, "k_occl32");
    if (which == 0)
      if (int rc = launch(k_march32<KH, KE, WV, ACT>, "k_march32", true)) return rc;
    if (scan) return launch(k_scan_best32<KH, KE, WV, ACT>, "k_scan_best32");
    return NRT_OK;
  };
  const bool sp = s->mlp->desc.activation == NRT_ACT_SOFTPLUS;
  int rc = NRT_EINVAL;
#define NRT_R32(H, KEV)                                                                   \
  if (md.hidden == H && md.ke == 4 * KEV)                                                 \
    rc = sp ? run.template operator()<H / 4, KEV, ACT_SOFTPLUS>()                         \
            : run.template operator()<H / 4, KEV, ACT_LEAKY>();                           \
  else
  NRT_R32(256, 12) NRT_R32(256, 20) NRT_R32(128, 12) NRT_R32(128, 20) {
    set_error("FP32 ring engine: unsupported SDF configuration");
    return NRT_EINVAL;
  }
#undef NRT_R32
  return rc;
}

int ring_occlusion32(const nrt_sdf* s, const float* rays, int64_t P, const MarchArgs& ma,
                     uint8_t* visible, hipStream_t st) {
  return ring32_launch(s, rays, P, ma, nullptr, visible, nullptr, nullptr, nullptr, nullptr,
                       nullptr, st, 2);
}

int ring_scan_best32(const nrt_sdf* s, const float* rays, int64_t P, const MarchArgs& ma,
                     float* thr, unsigned long long* keys, hipStream_t st) {
  return ring32_launch(s, rays, P, ma, nullptr, nullptr, nullptr, nullptr, nullptr, thr, keys, st, 1);
}

int ring_march32(const nrt_sdf* s, const float* rays, int64_t P, const MarchArgs& ma, float* t,
                 uint8_t* hit, float* p, float* n, float* raw_n, float* thr, int32_t* idx,
                 int32_t* cnt, unsigned long long* keys, hipStream_t st) {
  if (int rc = ring32_launch(s, rays, P, ma, t, hit, p, n, raw_n, thr, keys, st, 0)) return rc;
  // the march packed (hit, t) into t: unpack, p / n / raw_n and the hit list, coalesced
  k_march_finish<><<<dim3(std::min<int64_t>(ceil_div64(P, 256), 2048)), dim3(256), 0, st>>>(
      rays, P, t, hit, p, n, raw_n, idx, cnt);
  return check_launch("k_march_finish");
}

}  // namespace nrt
