// nrt_api_path.hip -- one bounce of the Path integrator (integrators.py:275-354): emitter term
// weighted by the path throughput, spatially varying BSDF sampling (ComposeSpatialVarying.sample,
// bsdfs.py:500-513) with injected uniforms, throughput / active update and the spawned rays.
#include "nrt_launch.h"

namespace nrt {

// warps.py:10-30 (output (r sin phi, r cos phi), as written there) and :44-49
__device__ __forceinline__ void cos_hemisphere(float u0, float u1, float wo[3]) {
  const float vx = 2.f * u0 - 1.f, vy = 2.f * u1 - 1.f;
  const bool zero = vx == 0.f && vy == 0.f;
  const bool q13 = fabsf(vx) < fabsf(vy);
  float r = q13 ? vy : vx;
  const float rp = q13 ? vx : vy;
  const float sg = r > 0.f ? 1.f : (r < 0.f ? -1.f : 0.f);
  r = sg * fmaxf(fabsf(r), 1e-12f);
  float phi = (0.25f * (float)M_PI) * rp / r;
  if (q13) phi = 0.5f * (float)M_PI - phi;
  if (zero) phi = 0.f;
  const float px = r * sinf(phi), py = r * cosf(phi);
  const float z = sqrtf(fmaxf(1.f - (px * px + py * py), 1e-7f));
  wo[0] = px; wo[1] = py; wo[2] = z;
  normalize3(wo[0], wo[1], wo[2], 1e-12f);
}

// from_local (interaction.py:44-51): normalize(s x + t y + n z), f = [s | t | n] columns
__device__ __forceinline__ void from_local(const float f[9], const float v[3], float o[3]) {
  for (int r = 0; r < 3; ++r) o[r] = (f[3 * r] * v[0] + f[3 * r + 1] * v[1]) + f[3 * r + 2] * v[2];
  normalize3(o[0], o[1], o[2], 1e-7f);
}

// default spawn for every ray (inactive rays are marched but their hits are ignored)
template <int = 0>
__global__ void k_path_default_rays(const float* __restrict__ P_, int64_t P, float* __restrict__ rays) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < P;
       i += (int64_t)gridDim.x * blockDim.x) {
    float* o = rays + i * 6;
    o[0] = P_[i * 3]; o[1] = P_[i * 3 + 1]; o[2] = P_[i * 3 + 2];
    o[3] = 0.f; o[4] = 0.f; o[5] = 1.f;
  }
}

// Over the active list: result += throughput * rgb (the emitter term of this bounce, rgb from the
// shading pass), then the BSDF sample: every component's cosine-hemisphere direction from its
// uniforms, NeuralBSDF spectra act(MLP(param_rusin2(wi, wo_c))), Diffuse spectra preproc(rho),
// spatial weights k = sigmoid(sp_var(p)), selection = inverse CDF of k / sum k at u_sel;
// throughput = clamp(spec_sel, 1e-10) * throughput; active &= any(throughput > 0);
// rays = [p, from_local(frame, wo_sel)].
template <bool F16>
__global__ void __launch_bounds__(256) k_path_sample(
    const BsdfDev* __restrict__ bp, const float* __restrict__ P_, const float* __restrict__ N_,
    const float* __restrict__ WI, const int32_t* __restrict__ list, const int32_t* __restrict__ count,
    const float* __restrict__ rgb, const float* __restrict__ u_comp, const float* __restrict__ u_sel,
    uint8_t* __restrict__ active, float* __restrict__ thr, float* __restrict__ result,
    float* __restrict__ rays, int RS, int per_wave) {
  extern __shared__ float smem[];
  const BsdfDev& bs = *bp;
  WaveLds l = wave_lds(smem, per_wave, RS, F16);
  float* Kw = l.Y + 32 * 32;  // [32][kMaxComponents] spatial weights
  const int lane = lane_id(), r = lane & 31;
  const int ys = 32;
  const int nc = bs.n;
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
  const int64_t total = *count;
  for (int64_t w = wave_global(); w * 32 < total; w += nw) {
    const int64_t i = w * 32 + r;
    const bool valid = i < total;
    const int64_t idx = list[valid ? i : total - 1];
    const float px = P_[idx * 3], py = P_[idx * 3 + 1], pz = P_[idx * 3 + 2];
    float fr[9];
    make_frame(N_[idx * 3], N_[idx * 3 + 1], N_[idx * 3 + 2], fr);
    const float wix = WI[idx * 3], wiy = WI[idx * 3 + 1], wiz = WI[idx * 3 + 2];
    if (!bs.spatial)
      for (int j = lane >> 5; j < nc; j += 2) Kw[r * kMaxComponents + j] = 1.f;
    // selection first needs k: job -1 = spatial weights, then components in order
    float sel_wo[3] = {0.f, 0.f, 1.f}, sel_f[3] = {0.f, 0.f, 0.f};
    int sel = -1;
    for (int job = -1; job < nc; ++job) {
      const MlpDev* m = job < 0 ? bs.spatial : (bs.comp[job].kind == 0 ? bs.comp[job].mlp : nullptr);
      float wo[3] = {0.f, 0.f, 1.f};
      if (job >= 0) {
        const float* u = u_comp + (idx * nc + job) * 2;
        cos_hemisphere(u[0], u[1], wo);
      }
      if (m) {
        EncIn e;
        e.xg = nullptr; e.lat = nullptr; e.x[3] = 0.f;
        if (job < 0) { e.x[0] = px; e.x[1] = py; e.x[2] = pz; }
        else {
          float feat[3];
          rusin2(wix, wiy, wiz, wo[0], wo[1], wo[2], feat);
          e.x[0] = feat[0]; e.x[1] = feat[1]; e.x[2] = feat[2];
        }
        mlp_eval_any<F16>(*m, e, l.X, RS, l.Y, ys);
      }
      if (job == -1) {
        if (m)
          for (int j = lane >> 5; j < nc; j += 2) Kw[r * kMaxComponents + j] = sigmoidf_(l.Y[r * ys + j]);
        wave_lds_fence();
        // inverse CDF of k / sum(k) at u_sel (stands in for torch.multinomial, bsdfs.py:506)
        float ksum = 0.f;
        for (int j = 0; j < nc; ++j) ksum += Kw[r * kMaxComponents + j];
        const float u = u_sel[idx];
        float cdf = 0.f;
        sel = nc - 1;
        for (int j = 0; j < nc; ++j) {
          cdf += Kw[r * kMaxComponents + j] / ksum;
          if (u < cdf) { sel = j; break; }
        }
      } else if (job == sel) {
        const BsdfCompDev& c = bs.comp[job];
        if (c.kind == 0) {
          for (int q = 0; q < 3; ++q) sel_f[q] = act_fwd<false>(l.Y[r * ys + q], c.act);
        } else {
          // Diffuse.sample: spectrum = preproc(reflectance) (bsdfs.py:104)
          for (int q = 0; q < 3; ++q)
            sel_f[q] = (c.act == ACT_NONE) ? c.params[q] / (float)M_PI : act_fwd<false>(c.params[q], c.act);
        }
        sel_wo[0] = wo[0]; sel_wo[1] = wo[1]; sel_wo[2] = wo[2];
      }
      wave_lds_fence();
    }
    if (valid && lane < 32) {
      float t[3];
      bool any = false;
      for (int q = 0; q < 3; ++q) {
        const float tq = thr[idx * 3 + q];
        // integrators.py:331-335: result += mis(=1) * throughput * bsdf_val * emitter_val
        result[idx * 3 + q] += tq * rgb[idx * 3 + q];
        t[q] = fmaxf(sel_f[q], 1e-10f) * tq;  // :338
        thr[idx * 3 + q] = t[q];
        any = any || (t[q] > 0.f);
      }
      if (!any) active[idx] = 0;  // :341
      float d[3];
      from_local(fr, sel_wo, d);
      float* o = rays + idx * 6;
      o[0] = px; o[1] = py; o[2] = pz; o[3] = d[0]; o[4] = d[1]; o[5] = d[2];
    }
    wave_lds_fence();
  }
}

static size_t a256(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace nrt

using namespace nrt;

extern "C" {

size_t nrt_path_workspace_bytes(int64_t P) {
  P = std::max<int64_t>(P, 1);
  return a256((size_t)P * 4) + 256 + a256((size_t)P * 12) + nrt_shadow_workspace_bytes(P);
}

int nrt_path_bounce(const nrt_bsdf* b, const nrt_light* l, const nrt_sdf* s, int32_t shadow,
                    const nrt_mlp* occ, int32_t max_steps, float eps, const float* p, const float* n, const float* wi,
                    int64_t P, uint8_t* active, float* throughput, float* result,
                    const float* u_comp, const float* u_sel, float* rays_out, void* workspace,
                    int precision, void* stream) {
  if (!b || !l || !p || !n || !wi || P < 0 || !active || !throughput || !result || !u_comp ||
      !u_sel || !rays_out || !workspace || (shadow && !s)) {
    set_error("nrt_path_bounce: bad argument");
    return NRT_EINVAL;
  }
  for (int j = 0; j < b->host_dev.n; ++j)
    if (b->host_dev.comp[j].kind == NRT_BSDF_CONDUCTOR) {
      set_error("nrt_path_bounce: Conductor.sample is not defined (it fails in the reference, "
                "bsdfs.py:391-401)");
      return NRT_EUNSUPPORTED;
    }
  if (P == 0) return NRT_OK;
  hipStream_t st = (hipStream_t)stream;
  const bool f16 = precision == NRT_FP16;
  char* ws = (char*)workspace;
  int32_t* list = (int32_t*)ws;
  int32_t* cnt = (int32_t*)(ws + a256((size_t)P * 4));
  float* rgb = (float*)(ws + a256((size_t)P * 4) + 256);
  void* shadow_ws = ws + a256((size_t)P * 4) + 256 + a256((size_t)P * 12);
  // active rays -> list (the hit-list compaction kernel)
  NRT_HIP(hipMemsetAsync(cnt, 0, sizeof(int32_t), st));
  k_hit_list<><<<dim3(std::min<int64_t>(ceil_div64(P, 256), 1024)), dim3(256), 0, st>>>(active, P, list, cnt);
  if (int rc = check_launch("k_hit_list")) return rc;
  k_path_default_rays<><<<dim3(std::min<int64_t>(ceil_div64(P, 256), 1024)), dim3(256), 0, st>>>(p, P, rays_out);
  if (int rc = check_launch("k_path_default_rays")) return rc;
  // emitter term of this bounce: rgb[i] = f(wi, wo_light) * Le for listed rays
  int rc = !shadow ? nrt_shade_direct(b, l, p, n, wi, list, cnt, P, rgb, nullptr, precision, stream)
           : occ ? nrt_shade_direct_learned_occ(b, l, s, occ, max_steps, eps, p, n, wi, list, cnt, P,
                                                rgb, nullptr, nullptr, shadow_ws, precision, stream)
                 : nrt_shade_direct_shadowed(b, l, s, max_steps, eps, p, n, wi, list, cnt, P, rgb,
                                             nullptr, nullptr, shadow_ws, precision, stream);
  if (rc) return rc;
  int hidden = 32, ke = 16;
  auto upd = [&](const nrt_mlp* m) {
    if (!m) return;
    hidden = std::max(hidden, m->desc.hidden);
    ke = std::max(ke, m->host_dev.ke);
  };
  upd(b->spatial);
  for (auto* m : b->mlps) upd(m);
  LdsPlan lp = plan_lds(hidden, ke, 64, f16, false);
  const int blocks = std::max(1, std::min(ceil_div64(ceil_div64(P, 32), lp.waves), 2048));
  ProfScope prof("k_path_sample", st);
  if (f16) {
    if ((rc = set_lds(k_path_sample<true>, lp.bytes))) return rc;
    k_path_sample<true><<<dim3(blocks), dim3(64 * lp.waves), lp.bytes, st>>>(
        b->dev, p, n, wi, list, cnt, rgb, u_comp, u_sel, active, throughput, result, rays_out,
        lp.RS, lp.per_wave);
  } else {
    if ((rc = set_lds(k_path_sample<false>, lp.bytes))) return rc;
    k_path_sample<false><<<dim3(blocks), dim3(64 * lp.waves), lp.bytes, st>>>(
        b->dev, p, n, wi, list, cnt, rgb, u_comp, u_sel, active, throughput, result, rays_out,
        lp.RS, lp.per_wave);
  }
  return check_launch("k_path_sample");
}

}  // extern "C"
