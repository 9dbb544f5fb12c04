// nrt_api_shade.hip -- light / BSDF handles and the fused direct-shading launcher
#include "nrt_launch.h"

using namespace nrt;

extern "C" {
static float sigm(float x) { return 1.f / (1.f + std::exp(-x)); }

int nrt_light_create_field(const nrt_mlp* mlp, const float* color3, nrt_light** out) {
  if (!mlp || !color3 || !out) { set_error("nrt_light_create_field: null"); return NRT_EINVAL; }
  if (mlp->desc.in_size != 3 || mlp->desc.out != 3) { set_error("nrt_light_create_field: MLP must map 3 -> 3"); return NRT_EINVAL; }
  std::unique_ptr<nrt_light> l(new nrt_light());
  std::memset(&l->host_dev, 0, sizeof(LightDev));
  l->host_dev.kind = 0;
  l->host_dev.mlp = mlp->dev;
  for (int i = 0; i < 3; ++i) l->host_dev.color_sig[i] = sigm(color3[i]);
  l->mlp = mlp;
  NRT_HIP(hipMalloc(&l->dev, sizeof(LightDev)));
  NRT_HIP(hipMemcpy(l->dev, &l->host_dev, sizeof(LightDev), hipMemcpyHostToDevice));
  if (int rc = build_light_program(l.get())) return rc;
  *out = l.release();
  return NRT_OK;
}

int nrt_light_create_point(const float* loc, const float* inten, float c, float lin, float q,
                           float scale, nrt_light** out) {
  if (!loc || !inten || !out) { set_error("nrt_light_create_point: null"); return NRT_EINVAL; }
  std::unique_ptr<nrt_light> l(new nrt_light());
  std::memset(&l->host_dev, 0, sizeof(LightDev));
  l->host_dev.kind = 1;
  float nrm = std::sqrt(inten[0] * inten[0] + inten[1] * inten[1] + inten[2] * inten[2]);
  nrm = std::max(nrm, 1e-12f);
  for (int i = 0; i < 3; ++i) {
    l->host_dev.loc[i] = loc[i];
    l->host_dev.scaled_dir[i] = scale * (inten[i] / nrm);
  }
  l->host_dev.c = std::max(c, 1e-6f);
  l->host_dev.l = std::max(lin, 1e-6f);
  l->host_dev.q = std::max(q, 1e-6f);
  NRT_HIP(hipMalloc(&l->dev, sizeof(LightDev)));
  NRT_HIP(hipMemcpy(l->dev, &l->host_dev, sizeof(LightDev), hipMemcpyHostToDevice));
  *out = l.release();
  return NRT_OK;
}

int nrt_light_create_renderer_point(const float* loc, const float* inten, float scale,
                                    nrt_light** out) {
  if (!loc || !inten || !out || !std::isfinite(scale)) {
    set_error("nrt_light_create_renderer_point: bad argument");
    return NRT_EINVAL;
  }
  std::unique_ptr<nrt_light> l(new nrt_light());
  std::memset(&l->host_dev, 0, sizeof(LightDev));
  l->host_dev.kind = 1;
  l->host_dev.falloff = 1;
  for (int i = 0; i < 3; ++i) {
    l->host_dev.loc[i] = loc[i];
    l->host_dev.scaled_dir[i] = scale * inten[i];  // self.scale * self.intensity, in f32
  }
  NRT_HIP(hipMalloc(&l->dev, sizeof(LightDev)));
  NRT_HIP(hipMemcpy(l->dev, &l->host_dev, sizeof(LightDev), hipMemcpyHostToDevice));
  *out = l.release();
  return NRT_OK;
}

int nrt_light_destroy(nrt_light* l) {
  if (!l) return NRT_OK;
  if (l->dev) (void)hipFree(l->dev);
  delete l;
  return NRT_OK;
}
int nrt_bsdf_create(int32_t n, const nrt_bsdf_component* comps, const nrt_mlp* spatial, nrt_bsdf** out) {
  if (n < 1 || n > kMaxComponents || !comps || !out) { set_error("nrt_bsdf_create: 1..32 components required"); return NRT_EINVAL; }
  if (spatial && (spatial->desc.in_size != 3 || spatial->desc.out < n)) {
    set_error("nrt_bsdf_create: spatial MLP must map 3 -> n_components");
    return NRT_EINVAL;
  }
  std::unique_ptr<nrt_bsdf> b(new nrt_bsdf());
  std::memset(&b->host_dev, 0, sizeof(BsdfDev));
  b->host_dev.n = n;
  b->host_dev.spatial = spatial ? spatial->dev : nullptr;
  b->spatial = spatial;
  for (int j = 0; j < n; ++j) {
    const nrt_bsdf_component& c = comps[j];
    BsdfCompDev& d = b->host_dev.comp[j];
    d.kind = c.kind;
    d.act = c.activation;
    std::memcpy(d.params, c.params, sizeof(d.params));
    if (c.kind == NRT_BSDF_NEURAL) {
      if (!c.mlp || c.mlp->desc.in_size != 3 || c.mlp->desc.out != 3) {
        set_error("nrt_bsdf_create: NeuralBSDF MLP must map 3 -> 3");
        return NRT_EINVAL;
      }
      d.mlp = c.mlp->dev;
      b->mlps.push_back(c.mlp);
    } else if (c.kind != NRT_BSDF_DIFFUSE && c.kind != NRT_BSDF_CONDUCTOR) {
      set_error("nrt_bsdf_create: unknown component kind");
      return NRT_EINVAL;
    }
  }
  NRT_HIP(hipMalloc(&b->dev, sizeof(BsdfDev)));
  NRT_HIP(hipMemcpy(b->dev, &b->host_dev, sizeof(BsdfDev), hipMemcpyHostToDevice));
  if (int rc = build_bsdf_program(b.get())) return rc;
  *out = b.release();
  return NRT_OK;
}

int nrt_bsdf_destroy(nrt_bsdf* b) {
  if (!b) return NRT_OK;
  if (b->dev) (void)hipFree(b->dev);
  delete b;
  return NRT_OK;
}

}  // extern "C"

namespace {
int shade_direct_impl(const nrt_bsdf* b, const nrt_light* l, const float* p, const float* n,
                      const float* wi, const int32_t* hit_idx, const int32_t* hit_count, int64_t P,
                      const float* lscale, float* rgb, float* weights_out, int precision,
                      hipStream_t st) {
  const bool f16 = precision == NRT_FP16;
  int hidden = 32, ke = 16;
  auto upd = [&](const nrt_mlp* m) {
    if (!m) return;
    hidden = std::max(hidden, m->desc.hidden);
    ke = std::max(ke, m->host_dev.ke);
  };
  upd(l->mlp);
  upd(b->spatial);
  for (auto* m : b->mlps) upd(m);
  // FP16: light field, spatial weights and NeuralBSDFs on the program engine when compiled for
  // their shapes (NRT_NO_PROGRAM keeps the per-wave register path)
  if (f16 && option(OPT_SHADE_PROGRAM) != 0) {
    const int rc = shade_program(b, l, p, n, wi, hit_idx, hit_count, P, lscale, rgb, weights_out, st);
    if (rc != NRT_EUNSUPPORTED) return rc;
  }
  // FP32 / fp32-split: the row-program ring kernels (nrt_shade_ring.hip) for the reference's
  // shading MLP shapes
  if (!f16 && option(OPT_SHADE_RING) != 0) {
    const int rc = shade_ring(b, l, p, n, wi, hit_idx, hit_count, P, lscale, rgb, weights_out,
                              precision, st);
    if (rc != NRT_EUNSUPPORTED) return rc;
  }
  LdsPlan lp = plan_lds(hidden, ke, 64, f16, false);
  int blocks = std::max(1, std::min(ceil_div64(ceil_div64(P, 32), lp.waves), 2048));
  ProfScope prof("k_shade_direct", st);
  if (f16) {
    if (int rc = set_lds(k_shade_direct<true>, lp.bytes)) return rc;
    k_shade_direct<true><<<dim3(blocks), dim3(64 * lp.waves), lp.bytes, st>>>(
        b->dev, l->dev, p, n, wi, hit_idx, hit_count, lscale, rgb, weights_out, lp.RS, lp.per_wave);
  } else {
    if (int rc = set_lds(k_shade_direct<false>, lp.bytes)) return rc;
    k_shade_direct<false><<<dim3(blocks), dim3(64 * lp.waves), lp.bytes, st>>>(
        b->dev, l->dev, p, n, wi, hit_idx, hit_count, lscale, rgb, weights_out, lp.RS, lp.per_wave);
  }
  return check_launch("k_shade_direct");
}

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }
}  // namespace

extern "C" {
int nrt_shade_direct(const nrt_bsdf* b, const nrt_light* l, const float* p, const float* n,
                     const float* wi, const int32_t* hit_idx, const int32_t* hit_count, int64_t P,
                     float* rgb, float* weights_out, int precision, void* stream) {
  if (!b || !l || !p || !n || !wi || !hit_idx || !hit_count || !rgb || P < 0) {
    set_error("nrt_shade_direct: bad argument");
    return NRT_EINVAL;
  }
  if (P == 0) return NRT_OK;
  return shade_direct_impl(b, l, p, n, wi, hit_idx, hit_count, P, nullptr, rgb, weights_out,
                           precision, (hipStream_t)stream);
}

// workspace: shadow rays [P,6] | max_t [P] | visible [P] | occ inputs [P,5] | occ out [P,3] |
// Le factors [P,3]
size_t nrt_shadow_workspace_bytes(int64_t P) {
  P = std::max<int64_t>(P, 1);
  return align256((size_t)P * 6 * 4) + align256((size_t)P * 4) + align256((size_t)P) +
         align256((size_t)P * 5 * 4) + 2 * align256((size_t)P * 3 * 4);
}
}  // extern "C"

namespace {
int shade_shadowed_impl(const char* who, const nrt_bsdf* b, const nrt_light* l, const nrt_sdf* s,
                        const nrt_mlp* occ, int32_t max_steps, float eps, const float* p,
                        const float* n, const float* wi, const int32_t* hit_idx,
                        const int32_t* hit_count, int64_t P, float* rgb, float* weights_out,
                        uint8_t* visible_out, void* workspace, int precision, void* stream) {
  if (!b || !l || !s || !p || !n || !wi || !hit_idx || !hit_count || !rgb || P < 0 || !workspace) {
    set_error(std::string(who) + ": bad argument");
    return NRT_EINVAL;
  }
  if (occ && (occ->desc.in_size != 5 || (occ->desc.out != 1 && occ->desc.out != 3))) {
    set_error(std::string(who) + ": occlusion MLP must map [p, elev, azim] (5) -> 1 or 3");
    return NRT_EINVAL;
  }
  if (l->host_dev.kind != 1) {
    // the reference's LightField samples carry no distance, so its shadow test cannot run
    set_error(std::string(who) + ": shadow rays need a point light (LightField samples "
              "have no distance, lights.py:175-195)");
    return NRT_EUNSUPPORTED;
  }
  if (P == 0) return NRT_OK;
  hipStream_t st = (hipStream_t)stream;
  char* ws = (char*)workspace;
  size_t off = 0;
  auto take = [&](size_t bytes) { char* q = ws + off; off += align256(bytes); return q; };
  float* rays = (float*)take((size_t)P * 24);
  float* max_t = (float*)take((size_t)P * 4);
  uint8_t* vis_ws = (uint8_t*)take((size_t)P);
  float* occ_in = (float*)take((size_t)P * 20);
  float* occ_out = (float*)take((size_t)P * 12);
  float* lscale = (float*)take((size_t)P * 12);
  uint8_t* vis = visible_out ? visible_out : vis_ws;
  const dim3 grid(std::min<int64_t>(ceil_div64(P, 256), 1024)), block(256);
  k_point_shadow_rays<><<<grid, block, 0, st>>>(l->dev, p, hit_idx, hit_count, rays, max_t);
  if (int rc = check_launch("k_point_shadow_rays")) return rc;
  if (int rc = launch_occlusion(s, rays, P, hit_count, max_t, max_steps, eps, vis, precision, st))
    return rc;
  if (occ) {
    // occ(occ_rays) over the P list slots (rows past *hit_count are never read back)
    k_occ_inputs<><<<grid, block, 0, st>>>(p, hit_idx, hit_count, rays, occ_in);
    if (int rc = check_launch("k_occ_inputs")) return rc;
    if (int rc = nrt_mlp_forward(occ, occ_in, nullptr, P, occ_out, precision, stream)) return rc;
  }
  k_light_scale<><<<grid, block, 0, st>>>(hit_count, vis, occ ? occ_out : nullptr,
                                          occ ? occ->desc.out : 1, lscale);
  if (int rc = check_launch("k_light_scale")) return rc;
  return shade_direct_impl(b, l, p, n, wi, hit_idx, hit_count, P, lscale, rgb, weights_out,
                           precision, st);
}
}  // namespace

extern "C" {
int nrt_shade_direct_shadowed(const nrt_bsdf* b, const nrt_light* l, const nrt_sdf* s,
                              int32_t max_steps, float eps, const float* p, const float* n,
                              const float* wi, const int32_t* hit_idx, const int32_t* hit_count,
                              int64_t P, float* rgb, float* weights_out, uint8_t* visible_out,
                              void* workspace, int precision, void* stream) {
  return shade_shadowed_impl("nrt_shade_direct_shadowed", b, l, s, nullptr, max_steps, eps, p, n,
                             wi, hit_idx, hit_count, P, rgb, weights_out, visible_out, workspace,
                             precision, stream);
}

int nrt_shade_direct_learned_occ(const nrt_bsdf* b, const nrt_light* l, const nrt_sdf* s,
                                 const nrt_mlp* occ, int32_t max_steps, float eps, const float* p,
                                 const float* n, const float* wi, const int32_t* hit_idx,
                                 const int32_t* hit_count, int64_t P, float* rgb,
                                 float* weights_out, uint8_t* visible_out, void* workspace,
                                 int precision, void* stream) {
  if (!occ) { set_error("nrt_shade_direct_learned_occ: null occlusion MLP"); return NRT_EINVAL; }
  return shade_shadowed_impl("nrt_shade_direct_learned_occ", b, l, s, occ, max_steps, eps, p, n,
                             wi, hit_idx, hit_count, P, rgb, weights_out, visible_out, workspace,
                             precision, stream);
}
}  // extern "C"
