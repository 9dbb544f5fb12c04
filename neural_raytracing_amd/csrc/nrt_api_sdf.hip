// nrt_api_sdf.hip -- SDF handles, evaluation, gradient, intersect and occlusion launchers
#include "nrt_launch.h"

using namespace nrt;

extern "C" {
static int sdf_finish(std::unique_ptr<nrt_sdf>& s, nrt_sdf** out) {
  NRT_HIP(hipMalloc(&s->dev, sizeof(SdfDev)));
  NRT_HIP(hipMemcpy(s->dev, &s->host_dev, sizeof(SdfDev), hipMemcpyHostToDevice));
  *out = s.release();
  return NRT_OK;
}

int nrt_sdf_create_unit_sphere(nrt_sdf** out) {
  if (!out) return NRT_EINVAL;
  std::unique_ptr<nrt_sdf> s(new nrt_sdf());
  std::memset(&s->host_dev, 0, sizeof(SdfDev));
  s->host_dev.kind = 0;
  return sdf_finish(s, out);
}

int nrt_sdf_create_mlp(const nrt_mlp* mlp, nrt_sdf** out) {
  if (!mlp || !out) { set_error("nrt_sdf_create_mlp: null"); return NRT_EINVAL; }
  if (mlp->desc.out < 1 || mlp->desc.in_size != 3) {
    set_error("nrt_sdf_create_mlp: SDF MLP must map 3 -> >=1 (output 0 is the distance)");
    return NRT_EINVAL;
  }
  std::unique_ptr<nrt_sdf> s(new nrt_sdf());
  std::memset(&s->host_dev, 0, sizeof(SdfDev));
  s->host_dev.kind = 1;
  s->host_dev.mlp = mlp->dev;
  s->host_dev.nb = mlp->desc.hidden / 32;
  s->mlp = mlp;
  return sdf_finish(s, out);
}

int nrt_sdf_create_sphere_blob(int32_t n, const float* centers, const float* radii,
                               const float* tfs, float k, const nrt_mlp* shift, nrt_sdf** out) {
  if (n < 1 || !centers || !radii || !tfs || !out) { set_error("nrt_sdf_create_sphere_blob: bad argument"); return NRT_EINVAL; }
  if (shift && (shift->desc.in_size != 3 || shift->desc.out < 1)) {
    set_error("nrt_sdf_create_sphere_blob: shift MLP must map 3 -> 1");
    return NRT_EINVAL;
  }
  std::unique_ptr<nrt_sdf> s(new nrt_sdf());
  std::memset(&s->host_dev, 0, sizeof(SdfDev));
  std::vector<float> packed((size_t)n * 16, 0.f);
  for (int i = 0; i < n; ++i) {
    float* d = &packed[(size_t)i * 16];
    // (tfs + I): sdfs.py:38
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) d[3 * a + b] = tfs[(size_t)i * 9 + 3 * a + b] + (a == b ? 1.f : 0.f);
    d[9] = centers[i * 3]; d[10] = centers[i * 3 + 1]; d[11] = centers[i * 3 + 2];
    d[12] = radii[i];
  }
  NRT_HIP(hipMalloc(&s->spheres, packed.size() * sizeof(float)));
  NRT_HIP(hipMemcpy(s->spheres, packed.data(), packed.size() * sizeof(float), hipMemcpyHostToDevice));
  s->host_dev.kind = 2;
  s->host_dev.n_spheres = n;
  s->host_dev.k = k;
  s->host_dev.spheres = s->spheres;
  s->host_dev.mlp = shift ? shift->dev : nullptr;
  s->host_dev.nb = shift ? shift->desc.hidden / 32 : 0;
  s->mlp = shift;
  return sdf_finish(s, out);
}

}  // extern "C"

namespace {
// the SphereSDF table of nrt_sdf_create_sphere_blob from device tensors: row i = (I + tfs_i)
// row-major (9), centre (3), radius (1), pad (3)
template <int = 0>
__global__ void k_pack_spheres(int n, const float* __restrict__ c, const float* __restrict__ r,
                               const float* __restrict__ t, float* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float* d = out + (size_t)i * 16;
  for (int a = 0; a < 3; ++a)
    for (int b = 0; b < 3; ++b) d[3 * a + b] = t[(size_t)i * 9 + 3 * a + b] + (a == b ? 1.f : 0.f);
  d[9] = c[i * 3]; d[10] = c[i * 3 + 1]; d[11] = c[i * 3 + 2];
  d[12] = r[i];
  d[13] = 0.f; d[14] = 0.f; d[15] = 0.f;
}
}  // namespace

extern "C" {
int nrt_sdf_refresh_spheres(nrt_sdf* s, const float* centers, const float* radii, const float* tfs,
                            void* stream) {
  if (!s || !centers || !radii || !tfs) { set_error("nrt_sdf_refresh_spheres: null argument"); return NRT_EINVAL; }
  if (s->host_dev.kind != 2 || !s->spheres) {
    set_error("nrt_sdf_refresh_spheres: not a sphere-blob SDF");
    return NRT_EINVAL;
  }
  const int n = s->host_dev.n_spheres;
  k_pack_spheres<><<<dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream>>>(n, centers, radii,
                                                                                tfs, s->spheres);
  return check_launch("k_pack_spheres");
}

int nrt_sdf_destroy(nrt_sdf* s) {
  if (!s) return NRT_OK;
  if (s->spheres) (void)hipFree(s->spheres);
  if (s->dev) (void)hipFree(s->dev);
  delete s;
  return NRT_OK;
}

int nrt_sdf_eval(const nrt_sdf* s, const float* p, int64_t M, float* out, int precision, void* stream) {
  if (!s || M < 0) { set_error("nrt_sdf_eval: bad argument"); return NRT_EINVAL; }
  if (M == 0) return NRT_OK;
  if (!p || !out) { set_error("nrt_sdf_eval: null p / out"); return NRT_EINVAL; }
  if ((precision == NRT_FP32_SPLIT || precision == NRT_MIXED) && ring3_supported(s) &&
      option(OPT_RING32) != 0)
    return ring_eval3(s, p, M, out, (hipStream_t)stream);
  const bool f16 = precision == NRT_FP16;
  int hidden, ke;
  sdf_dims(s, hidden, ke);
  LdsPlan lp = plan_lds(hidden, ke, 1, f16, false);
  dim3 grid(ceil_div64(ceil_div64(M, 32), lp.waves)), block(64 * lp.waves);
  hipStream_t st = (hipStream_t)stream;
  int rc = NRT_OK;
  NRT_NB_SWITCH(s->host_dev.nb, {
    if (f16) {
      if (!(rc = set_lds(k_sdf_eval<true, NB>, lp.bytes)))
        k_sdf_eval<true, NB><<<grid, block, lp.bytes, st>>>(s->dev, p, M, out, lp.RS, lp.per_wave);
    } else {
      if (!(rc = set_lds(k_sdf_eval<false, NB>, lp.bytes)))
        k_sdf_eval<false, NB><<<grid, block, lp.bytes, st>>>(s->dev, p, M, out, lp.RS, lp.per_wave);
    }
  });
  if (rc) return rc;
  return check_launch("k_sdf_eval");
}

// gradient launch shared by nrt_sdf_grad and the normal pass of nrt_sdf_intersect
static const int kGradBlocks = 512;

static size_t grad_scratch_floats_per_wave(const nrt_sdf* s) {
  if (!s->mlp) return 0;
  return (size_t)(s->mlp->desc.num_layers + 1) * 32 * s->mlp->desc.hidden;
}

static LdsPlan grad_plan(const nrt_sdf* s) {
  int hidden, ke;
  sdf_dims(s, hidden, ke);
  return plan_lds(hidden, ke, 1, false, true);
}

static size_t grad_workspace_bytes(const nrt_sdf* s) {
  LdsPlan lp = grad_plan(s);
  return (size_t)kGradBlocks * lp.waves * grad_scratch_floats_per_wave(s) * sizeof(float);
}

static int launch_grad(const nrt_sdf* s, const float* p, const int32_t* index, const int32_t* count,
                       int64_t M, float* grad, float* n_out, float* p_io, float eps, void* ws,
                       hipStream_t st) {
  LdsPlan lp = grad_plan(s);
  const int64_t waves_needed = ceil_div64(M, 32);
  int blocks = (int)std::min<int64_t>(kGradBlocks, ceil_div64(waves_needed, lp.waves));
  blocks = std::max(blocks, 1);
  int rc = NRT_OK;
  ProfScope prof("k_sdf_grad", st);
  NRT_NB_SWITCH(s->host_dev.nb, {
    if (!(rc = set_lds(k_sdf_grad<NB>, lp.bytes)))
      k_sdf_grad<NB><<<dim3(blocks), dim3(64 * lp.waves), lp.bytes, st>>>(
          s->dev, p, index, count, M, grad, n_out, p_io, eps, s->mlp ? (float*)ws : nullptr, lp.RS,
          lp.per_wave, (int64_t)grad_scratch_floats_per_wave(s));
  });
  if (rc) return rc;
  return check_launch("k_sdf_grad");
}

int nrt_sdf_grad(const nrt_sdf* s, const float* p, int64_t M, float* grad, void* stream) {
  if (!s || M < 0) { set_error("nrt_sdf_grad: bad argument"); return NRT_EINVAL; }
  if (M == 0) return NRT_OK;
  if (!p || !grad) { set_error("nrt_sdf_grad: null p / grad"); return NRT_EINVAL; }
  void* ws = nullptr;
  size_t bytes = grad_workspace_bytes(s);
  if (bytes) NRT_HIP(hipMallocAsync(&ws, bytes, (hipStream_t)stream));
  int rc = launch_grad(s, p, nullptr, nullptr, M, grad, nullptr, nullptr, 0.f, ws, (hipStream_t)stream);
  if (ws) (void)hipFreeAsync(ws, (hipStream_t)stream);
  return rc;
}

// [f32 normal-pass scratch | 256 B align | FP16 ring march scan keys (P x u64)]
static size_t grad_ws_aligned(const nrt_sdf* s) { return (grad_workspace_bytes(s) + 255) & ~(size_t)255; }

size_t nrt_intersect_workspace_bytes(const nrt_sdf* s, int64_t P) {
  if (!s) return 0;
  const bool keys = ring_supported(s) || ring32_supported(s);
  P = std::max<int64_t>(P, 0);
  // NRT_MIXED's runner-up keys, march flags and refinement list behind the keys
  return grad_ws_aligned(s) + (keys ? ring_march_ws_bytes(P) : 0) +
         (mixed_supported(s) ? mixed_ws_bytes(P) : 0) + 256;
}

int nrt_sdf_intersect(const nrt_sdf* s, const float* rays, int64_t P, const nrt_march_params* a,
                      float* t, uint8_t* hit, float* p, float* n, float* raw_n, float* wi,
                      float* throughput, int32_t* hit_idx, int32_t* hit_count, void* workspace,
                      void* stream) {
  if (!s || !a || P < 0) { set_error("nrt_sdf_intersect: bad argument"); return NRT_EINVAL; }
  if (P == 0) return NRT_OK;
  if (!rays || !t || !hit || !p || !n) { set_error("nrt_sdf_intersect: null output"); return NRT_EINVAL; }
  if (a->primary && !throughput) { set_error("nrt_sdf_intersect: throughput required when primary"); return NRT_EINVAL; }
  if ((hit_idx == nullptr) != (hit_count == nullptr)) { set_error("nrt_sdf_intersect: hit_idx and hit_count go together"); return NRT_EINVAL; }
  if (s->mlp && !workspace) { set_error("nrt_sdf_intersect: workspace required"); return NRT_EINVAL; }
  if (P == 0) return NRT_OK;
  hipStream_t st = (hipStream_t)stream;
  // NRT_MIXED: the FP16 march + scan with split refinement (nrt_ring_mixed.hip); its normals, and
  // the whole intersect of an SDF without both ring engines, at fp32-split
  const bool mixed = a->precision == NRT_MIXED && mixed_supported(s) && option(OPT_RING16) != 0 &&
                     option(OPT_RING32) != 0;
  const int prec = a->precision == NRT_MIXED ? NRT_FP32_SPLIT : a->precision;
  const bool f16 = prec == NRT_FP16;
  int hidden, ke;
  sdf_dims(s, hidden, ke);
  MarchArgs ma;
  ma.max_steps = a->max_steps;
  ma.eps = a->epsilon;
  ma.max_t = a->max_t;
  ma.primary = a->primary;
  ma.xcd_lines = (int)option(OPT_XCD_LINES);
  ma.step = a->scan_max_t / 128.0;
  ma.scan_idx = a->primary ? a->scan_index : nullptr;
  ma.evals = profile_eval_counter();
  if (a->primary && a->scan_max_t_groups) {
    if (a->group_rays < 1) { set_error("nrt_sdf_intersect: group_rays must be >= 1"); return NRT_EINVAL; }
    if (a->scan_index) { set_error("nrt_sdf_intersect: scan_index with scan_max_t_groups is not supported"); return NRT_EINVAL; }
    ma.groups = a->scan_max_t_groups;
    ma.group_rays = a->group_rays;
  }
  // the normal pass needs the list of hit rays; use the caller's or a workspace-backed one
  int32_t* idx = hit_idx;
  int32_t* cnt = hit_count;
  char* ws = (char*)workspace;
  std::unique_ptr<char, void (*)(char*)> own(nullptr, [](char* q) { if (q) (void)hipFree(q); });
  if (!idx) {
    char* tmp = nullptr;
    NRT_HIP(hipMallocAsync((void**)&tmp, (size_t)P * 4 + 256, st));
    own.reset(tmp);
    cnt = (int32_t*)tmp;
    idx = (int32_t*)(tmp + 256);
  }
  NRT_HIP(hipMemsetAsync(cnt, 0, sizeof(int32_t), st));
  LdsPlan lp = plan_lds(hidden, ke, 1, f16, false);
  dim3 grid(ceil_div64(ceil_div64(P, 32), lp.waves)), block(64 * lp.waves);
  int rc0 = NRT_OK;
  // FP16 SDF MLPs of width 128/256 with F = 16/32 run the block-cooperative ring kernel
  const bool ring16 = f16 && ring_supported(s) && option(OPT_RING16) != 0;
  // ... and FP32 SDF MLPs of those widths the FP32 ring kernel (refreshed training handles too)
  const bool ring32 = !f16 && ring32_supported(s) && option(OPT_RING32) != 0;
  // ... and the fp32-split precision the FP32-accurate FP16-MFMA engine (nrt_ring3.h)
  const bool ring3 = ring32 && prec == NRT_FP32_SPLIT && ring3_supported(s);
  if (ring16 || ring32) {
    ProfScope prof("k_intersect", st);
    auto* keys = reinterpret_cast<unsigned long long*>(ws + grad_ws_aligned(s));
    // the launch-wide job queue: always (1), or (2, default) for batches of at least 64 rays a
    // resident wave (measured: the 800^2 frame 964 -> 955 ms FP32, 97.5 -> 96.0 ms mixed; the
    // 38,400-ray training march 22.0 -> 22.3 ms FP32, 6.7 -> 7.1 mixed, so small batches keep
    // their per-wave lists)
    const int64_t mq = option(OPT_MARCH_QUEUE);
    if (mq == 1 || (mq == 2 && P >= 64 * 2048)) ma.queue = ring_march_queue(ws + grad_ws_aligned(s), P);
    rc0 = mixed  ? ring_march_mixed(s, rays, P, ma, t, hit, p, n, raw_n, throughput, idx, cnt, keys,
                                    ws + grad_ws_aligned(s) + ring_march_ws_bytes(P), st)
        : ring16 ? ring_march(s, rays, P, ma, t, hit, p, n, raw_n, throughput, idx, cnt, keys, st)
        : ring3  ? ring_march3(s, rays, P, ma, t, hit, p, n, raw_n, throughput, idx, cnt, keys, st)
                 : ring_march32(s, rays, P, ma, t, hit, p, n, raw_n, throughput, idx, cnt, keys, st);
    if (!rc0 && ma.scan_idx) {
      k_keys_index<><<<dim3(ceil_div64(P, 256)), dim3(256), 0, st>>>(keys, P, ma.scan_idx);
      rc0 = check_launch("k_keys_index");
    }
  } else {
    ProfScope prof("k_intersect", st);
    NRT_NB_SWITCH(s->host_dev.nb, {
      if (f16) {
        if (!(rc0 = set_lds(k_intersect<true, NB>, lp.bytes)))
          k_intersect<true, NB><<<grid, block, lp.bytes, st>>>(s->dev, rays, P, ma, t, hit, p, n, raw_n,
                                                               throughput, idx, cnt, lp.RS, lp.per_wave);
      } else {
        if (!(rc0 = set_lds(k_intersect<false, NB>, lp.bytes)))
          k_intersect<false, NB><<<grid, block, lp.bytes, st>>>(s->dev, rays, P, ma, t, hit, p, n, raw_n,
                                                                throughput, idx, cnt, lp.RS, lp.per_wave);
      }
    });
  }
  if (rc0) return rc0;
  if (int rc = check_launch("k_intersect")) return rc;
  // normals on hit rays: raw gradient, unit normal, p += 5 eps n.  FP16 ring SDFs use the
  // forward-mode kernel (8 rays per wave-evaluation), everything else the f32 backward.
  if (ring16 && option(OPT_NORMALS16) != 0) {
    ProfScope prof("k_normal16", st);
    if (int rc = ring_normals(s, idx, cnt, P, raw_n, n, p, a->epsilon, st)) return rc;
  } else if (ring32 && option(OPT_NORMALS_RING) != 0) {
    // forward mode on the FP32 / split ring engine of the march (k_normal32 / k_normal3)
    if (int rc = ring_normals32(s, idx, cnt, P, raw_n, n, p, a->epsilon, ring3, st)) return rc;
  } else if (int rc = launch_grad(s, p, idx, cnt, P, raw_n, n, p, a->epsilon, ws, st)) {
    return rc;
  }
  if (wi) {
    k_frame_wi<><<<dim3(ceil_div64(P, 256)), dim3(256), 0, st>>>(rays, n, P, nullptr, wi);
    if (int rc = check_launch("k_frame_wi")) return rc;
  }
  if (own) {
    // keep the temporary list alive until the stream has consumed it
    (void)hipFreeAsync(own.release(), st);
  }
  return NRT_OK;
}

}  // extern "C"

namespace nrt {
// shadow march over rays[0, P) (or [0, *count) when count is a device counter)
int launch_occlusion(const nrt_sdf* s, const float* rays, int64_t P, const int32_t* count,
                     const float* max_t, int32_t max_steps, float eps, uint8_t* visible,
                     int precision, hipStream_t st) {
  const bool f16 = precision == NRT_FP16;
  if (option(OPT_RING_OCCLUSION) != 0) {
    MarchArgs ma{};
    ma.max_steps = max_steps;
    ma.eps = eps;
    ma.max_t = 0.f;  // unused: each ray stops at its own distance to the light (occ_max_t)
    ma.primary = 0;
    ma.count = count;
    ma.occ_max_t = max_t;
    ma.evals = profile_eval_counter();
    if (f16 && ring_supported(s) && option(OPT_RING16) != 0) {
      ProfScope prof("k_occlusion", st);
      return ring_march16_launch(s, rays, P, ma, nullptr, nullptr, nullptr, st, false, visible);
    }
    if (!f16 && ring32_supported(s) && option(OPT_RING32) != 0) {
      ProfScope prof("k_occlusion", st);
      const bool split = (precision == NRT_FP32_SPLIT || precision == NRT_MIXED) && ring3_supported(s);
      return split ? ring3_launch(s, rays, P, ma, nullptr, nullptr, nullptr, st, 4, visible)
                   : ring_occlusion32(s, rays, P, ma, visible, st);
    }
  }
  int hidden, ke;
  sdf_dims(s, hidden, ke);
  LdsPlan lp = plan_lds(hidden, ke, 1, f16, false);
  dim3 grid(ceil_div64(ceil_div64(P, 32), lp.waves)), block(64 * lp.waves);
  int rc = NRT_OK;
  ProfScope prof("k_occlusion", st);
  NRT_NB_SWITCH(s->host_dev.nb, {
    if (f16) {
      if (!(rc = set_lds(k_occlusion<true, NB>, lp.bytes)))
        k_occlusion<true, NB><<<grid, block, lp.bytes, st>>>(s->dev, rays, P, count, max_t, max_steps, eps, visible, lp.RS, lp.per_wave);
    } else {
      if (!(rc = set_lds(k_occlusion<false, NB>, lp.bytes)))
        k_occlusion<false, NB><<<grid, block, lp.bytes, st>>>(s->dev, rays, P, count, max_t, max_steps, eps, visible, lp.RS, lp.per_wave);
    }
  });
  if (rc) return rc;
  return check_launch("k_occlusion");
}
}  // namespace nrt

extern "C" {
int nrt_sdf_occlusion(const nrt_sdf* s, const float* rays, int64_t P, const float* max_t,
                      int32_t max_steps, float eps, uint8_t* visible, int precision, void* stream) {
  if (!s || P < 0) { set_error("nrt_sdf_occlusion: bad argument"); return NRT_EINVAL; }
  if (P == 0) return NRT_OK;
  if (!rays || !max_t || !visible) { set_error("nrt_sdf_occlusion: null argument"); return NRT_EINVAL; }
  return launch_occlusion(s, rays, P, nullptr, max_t, max_steps, eps, visible, precision,
                          (hipStream_t)stream);
}

int nrt_frames(const float* rays, const float* n, int64_t P, float* frame, float* wi, void* stream) {
  if (!n || (wi && !rays) || P < 0) { set_error("nrt_frames: bad argument"); return NRT_EINVAL; }
  if (P == 0 || (!frame && !wi)) return NRT_OK;
  k_frame_wi<><<<dim3(ceil_div64(P, 256)), dim3(256), 0, (hipStream_t)stream>>>(rays, n, P, frame, wi);
  return check_launch("k_frame_wi");
}

}  // extern "C"
