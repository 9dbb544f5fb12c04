// FP16 march + coarse scan on the block-cooperative LDS weight ring (k_march16).
#include "nrt_launch.h"

namespace nrt {

int ring_march(const nrt_sdf* s, const float* rays, int64_t P, const MarchArgs& ma, float* t,
               uint8_t* hit, float* p, float* n, float* raw_n, float* thr, int32_t* idx,
               int32_t* cnt, hipStream_t st) {
  const size_t bias_bytes = ring_bias_bytes(s);
  return ring_dispatch(s, [&]<int NB, int NE, bool FOLD>() -> int {
    auto kern = k_march16<NB, NE, kRingWaves, FOLD>;
    const size_t lds = ring::Cfg<NB, NE, kRingWaves>::lds_bytes(bias_bytes);
    if (int rc = set_lds(kern, lds)) return rc;
    kern<<<dim3(ceil_div64(P, 32 * kRingWaves)), dim3(64 * kRingWaves), lds, st>>>(
        s->host_dev, s->mlp->host_dev, rays, P, ma, t, hit, p, n, raw_n, thr, idx, cnt);
    return check_launch("k_march16");
  });
}

}  // namespace nrt
