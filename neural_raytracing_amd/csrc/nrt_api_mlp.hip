// nrt_api_mlp.hip -- nrt_mlp_forward launcher
#include "nrt_launch.h"

using namespace nrt;

extern "C" {
int nrt_mlp_forward(const nrt_mlp* m, const float* x, const float* latent, int64_t M, float* y,
                    int precision, void* stream) {
  if (!m || M < 0) { set_error("nrt_mlp_forward: bad argument"); return NRT_EINVAL; }
  if (M == 0) return NRT_OK;
  if (!x || !y) { set_error("nrt_mlp_forward: null x / y"); return NRT_EINVAL; }
  if (m->desc.latent > 0 && !latent) { set_error("nrt_mlp_forward: latent required"); return NRT_EINVAL; }
  const bool f16 = precision == NRT_FP16;
  hipStream_t st = (hipStream_t)stream;
  // FP32: the shading MLP shapes on the ring engine (nrt_shade_ring.hip), same arithmetic class
  if (!f16 && !latent && option(OPT_SHADE_RING) != 0) {
    const int rc = solo_forward(m, x, M, y, st);
    if (rc != NRT_EUNSUPPORTED) return rc;
  }
  LdsPlan p = plan_lds(m->desc.hidden, m->host_dev.ke, m->desc.out, f16, false);
  if (!f16) spread_waves(p);
  const int waves = ceil_div64(M, 32);
  dim3 grid(ceil_div64(waves, p.waves)), block(64 * p.waves);
  int rc = NRT_OK;
  ProfScope prof("k_mlp_forward", st);
  NRT_NB_SWITCH(m->desc.hidden / 32, {
    if (f16) {
      if (!(rc = set_lds(k_mlp_forward<true, NB>, p.bytes)))
        k_mlp_forward<true, NB><<<grid, block, p.bytes, st>>>(m->dev, x, latent, M, y, p.RS, p.per_wave);
    } else {
      if (!(rc = set_lds(k_mlp_forward<false, NB>, p.bytes)))
        k_mlp_forward<false, NB><<<grid, block, p.bytes, st>>>(m->dev, x, latent, M, y, p.RS, p.per_wave);
    }
  });
  if (rc) return rc;
  return check_launch("k_mlp_forward");
}

}  // extern "C"
