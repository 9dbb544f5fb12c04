// Shading programs and the FP16 program-engine shading path (k_light16 + k_bsdf16).
//
// A program concatenates the k-outer weight streams of the MLPs one kernel evaluates per ray
// batch (the light field; or the spatial-weight MLP and every NeuralBSDF), so the LDS ring
// streams across MLP boundaries without draining.  Shapes with a compiled kernel:
//   light field   8 x 32 hidden blocks, F = 16  (LightField: 10 x 256)
//   spatial       8 x 32 hidden blocks, F = 128 (ComposeSpatialVarying: 16 x 256)
//   NeuralBSDF    3 x 32 hidden blocks, F = 64  (6 x 96)
// all with leaky_relu hidden activations and <= 32 outputs; anything else keeps k_shade_direct.
#include "nrt_launch.h"

namespace nrt {

namespace {

bool mlp_shape(const nrt_mlp* m, int nb, int ne) {
  const MlpDev& d = m->host_dev;
  return d.nb == nb && d.ke / 16 == ne && d.in_size == 3 && d.latent == 0 &&
         d.freqs == 8 * (ne - 1) && d.out <= 32 && d.act == ACT_LEAKY;
}

size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

}  // namespace

int build_program(const std::vector<const nrt_mlp*>& mlps, nrt_prog& out) {
  out.ok = false;
  if (mlps.empty() || (int)mlps.size() > kMaxProgMlp) return NRT_OK;
  for (const nrt_mlp* m : mlps)
    if (m->refreshed) {  // nrt_mlp_refresh does not re-pack the program streams
      set_error("shading program: an MLP handle refreshed by nrt_mlp_refresh cannot build one");
      return NRT_EINVAL;
    }
  ProgDev& d = out.d;
  std::memset(&d, 0, sizeof(d));
  std::vector<int> coff;
  std::vector<float> bias;
  std::vector<float4> basis;
  size_t frags = 0;
  for (size_t k = 0; k < mlps.size(); ++k) {
    const nrt_mlp* m = mlps[k];
    const MlpDev& md = m->host_dev;
    ProgMlp& pm = d.mlp[k];
    pm.nb = md.nb; pm.ne = md.ke / 16; pm.ob = md.ob; pm.L = md.n_hidden; pm.skip = md.skip;
    pm.out = md.out; pm.act = md.act; pm.F = md.freqs;
    pm.bstride = md.bias16_stride;
    pm.bias_off = (int)bias.size();
    pm.basis_off = (int)basis.size();
    pm.chunk0 = (int)coff.size();
    for (int c : m->host_chunkk) coff.push_back(c + (int)frags);
    bias.insert(bias.end(), m->host_bias.begin(), m->host_bias.end());
    const int F = md.freqs;
    for (int q = 0; q < F; ++q)
      basis.push_back(make_float4(m->host_basis[q], m->host_basis[F + q], m->host_basis[2 * F + q], 0.f));
    frags += (size_t)md.nk_frags;
  }
  d.n_mlp = (int)mlps.size();
  d.n_chunks = (int)coff.size();
  d.bias_floats = (int)bias.size();
  d.basis_q = (int)basis.size();
  const size_t stream_bytes = (frags + 64) * 1024;  // + zero tail for the unguarded prefetch
  const size_t o_coff = align256(stream_bytes);
  const size_t o_bias = align256(o_coff + coff.size() * 4);
  const size_t o_basis = align256(o_bias + bias.size() * 4);
  const size_t total = align256(o_basis + basis.size() * 16);
  char* buf = nullptr;
  NRT_HIP(hipMalloc((void**)&buf, total));
  out.buf = buf;
  NRT_HIP(hipMemset(buf, 0, stream_bytes));
  size_t off = 0;
  for (const nrt_mlp* m : mlps) {
    const size_t bytes = (size_t)m->host_dev.nk_frags * 1024;
    NRT_HIP(hipMemcpy(buf + off, m->host_dev.streamk16, bytes, hipMemcpyDeviceToDevice));
    off += bytes;
  }
  NRT_HIP(hipMemcpy(buf + o_coff, coff.data(), coff.size() * 4, hipMemcpyHostToDevice));
  NRT_HIP(hipMemcpy(buf + o_bias, bias.data(), bias.size() * 4, hipMemcpyHostToDevice));
  NRT_HIP(hipMemcpy(buf + o_basis, basis.data(), basis.size() * 16, hipMemcpyHostToDevice));
  d.stream = reinterpret_cast<const h8*>(buf);
  d.coff = reinterpret_cast<const int*>(buf + o_coff);
  d.bias = reinterpret_cast<const float*>(buf + o_bias);
  d.basis = reinterpret_cast<const float4*>(buf + o_basis);
  out.ok = true;
  return NRT_OK;
}

int build_light_program(nrt_light* l) {
  if (l->host_dev.kind != 0 || !l->mlp || !mlp_shape(l->mlp, 8, 3)) return NRT_OK;
  return build_program({l->mlp}, l->prog);
}

int build_bsdf_program(nrt_bsdf* b) {
  std::vector<const nrt_mlp*> v;
  if (b->spatial) {
    if (!mlp_shape(b->spatial, 8, 17)) return NRT_OK;
    v.push_back(b->spatial);
  }
  for (const nrt_mlp* m : b->mlps)
    if (!mlp_shape(m, 3, 9)) return NRT_OK;
  v.insert(v.end(), b->mlps.begin(), b->mlps.end());
  if (v.empty()) return NRT_OK;
  return build_program(v, b->prog);
}

namespace {
constexpr int kShadeWaves = 8;

template <class K>
int persistent_blocks(K kern, int threads, size_t lds, int64_t want) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 256;
  }
  int per_cu = 1;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(kern),
                                                   threads, lds) != hipSuccess || per_cu < 1)
    per_cu = 1;
  return (int)std::max<int64_t>(1, std::min<int64_t>(want, (int64_t)cus * per_cu));
}
}  // namespace

// NRT_EUNSUPPORTED when the program path does not cover this light / BSDF pair
int shade_program(const nrt_bsdf* b, const nrt_light* l, const float* p, const float* n,
                  const float* wi, const int32_t* hit_idx, const int32_t* hit_count, int64_t P,
                  const float* lscale, float* rgb, float* weights_out, hipStream_t st) {
  const bool field = l->host_dev.kind == 0;
  if ((field && !l->prog.ok) || !b->prog.ok) return NRT_EUNSUPPORTED;
  constexpr int WV = kShadeWaves;
  float* ls = nullptr;
  NRT_HIP(hipMallocAsync((void**)&ls, (size_t)P * kLsStride * sizeof(float), st));
  const int64_t want = ceil_div64(P, 32 * WV);
  int rc = NRT_OK;
  {
    ProfScope prof("k_light16", st);
    if (field) {
      auto kern = k_light16<WV, true>;
      const size_t lds = ring::KEngine<WV>::lds_bytes(l->prog.d);
      if (!(rc = set_lds(kern, lds))) {
        kern<<<dim3(persistent_blocks(kern, 64 * WV, lds, want)), dim3(64 * WV), lds, st>>>(
            l->prog.d, l->dev, p, n, wi, hit_idx, hit_count, lscale, ls);
        rc = check_launch("k_light16");
      }
    } else {
      auto kern = k_light16<WV, false>;
      kern<<<dim3(persistent_blocks(kern, 64 * WV, 0, want)), dim3(64 * WV), 0, st>>>(
          l->prog.d, l->dev, p, n, wi, hit_idx, hit_count, lscale, ls);
      rc = check_launch("k_light16");
    }
  }
  if (!rc) {
    ProfScope prof("k_bsdf16", st);
    const size_t lds = ring::KEngine<WV>::lds_bytes(b->prog.d) + (size_t)WV * 32 * kMaxComponents * 4;
    auto launch = [&](auto kern) {
      if ((rc = set_lds(kern, lds))) return;
      kern<<<dim3(persistent_blocks(kern, 64 * WV, lds, want)), dim3(64 * WV), lds, st>>>(
          b->prog.d, b->dev, p, wi, hit_idx, hit_count, ls, rgb, weights_out);
      rc = check_launch("k_bsdf16");
    };
    if (b->spatial) launch(k_bsdf16<WV, true>);
    else launch(k_bsdf16<WV, false>);
  }
  (void)hipFreeAsync(ls, st);
  return rc;
}

}  // namespace nrt
