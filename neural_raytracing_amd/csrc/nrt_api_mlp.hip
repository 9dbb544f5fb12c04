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

size_t nrt_mlp_save_bytes(const nrt_mlp* m, int64_t M) {
  if (!m || M < 0 || m->desc.latent > 0 || option(OPT_TRAIN_SAVE) == 0 || !saved_forward_ok(m)) return 0;
  return saved_bytes(m->host_dev, std::max<int64_t>(M, 1));
}

int nrt_mlp_forward_multi(const nrt_mlp* const* mlps, int n, const float* x, int64_t M,
                          float* const* y, void* const* save, int precision, void* stream) {
  if (!mlps || !y || n < 0 || M < 0) { set_error("nrt_mlp_forward_multi: bad argument"); return NRT_EINVAL; }
  for (int k = 0; k < n; ++k) {
    if (!mlps[k] || !y[k]) { set_error("nrt_mlp_forward_multi: null MLP / output"); return NRT_EINVAL; }
    if (mlps[k]->desc.latent > 0) { set_error("nrt_mlp_forward_multi: MLPs with a latent input are not supported"); return NRT_EINVAL; }
    if (save && (!save[k] || !saved_forward_ok(mlps[k]))) {
      set_error("nrt_mlp_forward_multi: a save buffer for every MLP, each with nrt_mlp_save_bytes > 0");
      return NRT_EINVAL;
    }
  }
  if (save && precision == NRT_FP16) { set_error("nrt_mlp_forward_multi: the training forward (save) is FP32"); return NRT_EINVAL; }
  if (M == 0 || n == 0) return NRT_OK;
  if (!x) { set_error("nrt_mlp_forward_multi: null x"); return NRT_EINVAL; }
  hipStream_t st = (hipStream_t)stream;
  for (int k0 = 0; k0 < n; k0 += kMaxSoloForward) {
    const int nk = std::min(n - k0, kMaxSoloForward);
    int rc = NRT_EUNSUPPORTED;
    if (precision != NRT_FP16 && option(OPT_SHADE_RING) != 0)
      rc = solo_forward_multi(mlps + k0, nk, x, M, y + k0, st, save ? save + k0 : nullptr);
    if (rc == NRT_EUNSUPPORTED && save) {
      set_error("nrt_mlp_forward_multi: these MLPs have no saving forward (check nrt_mlp_save_bytes)");
      return NRT_EUNSUPPORTED;
    }
    if (rc == NRT_EUNSUPPORTED) {
      for (int k = k0; k < k0 + nk; ++k)
        if ((rc = nrt_mlp_forward(mlps[k], x, nullptr, M, y[k], precision, stream))) return rc;
    } else if (rc) {
      return rc;
    }
  }
  return NRT_OK;
}

}  // extern "C"
