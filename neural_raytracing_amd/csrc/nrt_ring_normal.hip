// FP16 forward-mode SDF normals on the block-cooperative LDS weight ring (k_normal16).
#include "nrt_launch.h"

namespace nrt {

int ring_normals(const nrt_sdf* s, const int32_t* idx, const int32_t* cnt, int64_t M, float* grad,
                 float* n, float* p_io, float eps, hipStream_t st) {
  const size_t bias_bytes = ring_bias_bytes(s);
  return ring_dispatch(s, [&]<int NB, int NE, bool FOLD>() -> int {
    auto kern = k_normal16<NB, NE, kRingWaves, FOLD>;
    const size_t lds = ring::Cfg<NB, NE, kRingWaves>::lds_bytes(bias_bytes);
    if (int rc = set_lds(kern, lds)) return rc;
    // 8 rays per wave; blocks stride over the device-side hit count
    const int64_t blocks = std::min<int64_t>(ceil_div64(M, 8 * kRingWaves), 2048);
    kern<<<dim3(blocks), dim3(64 * kRingWaves), lds, st>>>(s->host_dev, s->mlp->host_dev, idx, cnt,
                                                             M, grad, n, p_io, eps);
    return check_launch("k_normal16");
  });
}

}  // namespace nrt
