// FP32 / fp32-split shading on the row-program ring engines (nrt_shade_ring.h): program builder
// and launcher.  Direct.sample's emitter and BSDF evaluation (integrators.py:173-189) for the
// reference's shading MLPs at its precision:
//   LightField            10 x 256, F = 16   (lights.py:159-164)
//   ComposeSpatialVarying 16 x 256, F = 128  (bsdfs.py:487-494), <= 16 components
//   NeuralBSDF             6 x 96,  F = 64   (bsdfs.py:616-621)
// all leaky_relu (the SkipConnMLP default, neural_blocks.py:26), 3 inputs, no latent.  Anything
// else keeps the per-wave k_shade_direct.
#include "nrt_launch.h"
#include "nrt_shade_ring.h"
#include "nrt_train_ring.h"

namespace nrt {

namespace {

size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

struct ShapeSpec {
  int H, F;
};
constexpr ShapeSpec kLightSpec{256, 16}, kSpatialSpec{256, 128}, kBsdfSpec{96, 64};

bool shape_ok(const nrt_mlp* m, ShapeSpec s) {
  const nrt_mlp_desc& d = m->desc;
  return d.hidden == s.H && d.freqs == s.F && d.in_size == 3 && d.latent == 0 && d.out <= 16 &&
         d.activation == NRT_ACT_LEAKY_RELU && d.num_layers + 2 <= kMaxLin && !m->refreshed &&
         (int)m->host_w.size() == d.num_layers + 2;
}

// Emits one MLP's stream in the order its evaluation consumes it (nrt_shade_ring.h eval32 /
// eval3) and records each chunk's (KiB offset, KiB count).  Layer l's inputs: the init layer the
// encoding, hidden layer i (l = 1 + i) the H hidden features and, on skip layers, the encoding;
// the out layer the hidden features (neural_blocks.py:46-55, 80-86).  Encoding slot s: 2q / 2q + 1
// = sin / cos of projection q, then x0..x2 -- reference columns [x, sin, cos] (utils.py:37-40).
//   FP32 piece  [lane 64][4 k-steps] floats: lane (g, i) = A[row 16 b + i][input of k-step s for
//               lane group g]: hidden k-step s -> feature 16 (s >> 2) + 4 g + (s & 3), encoding
//               k-step s -> slot 4 s + g.
//   split piece [lane 64][8] f16 halves of W 2^s_l: lane (g, i) = A[row 16 b + i][k = 8 g + e]:
//               hidden k-step u -> feature 16 (2u + (e >> 2)) + 4 g + (e & 3), encoding k-step v
//               -> slot 32 v + 8 g + e.
//   encoding part of a layer (k-outer): chunks of EQ quads (FP32) / EK k-steps (split) x every
//   sub-block [quad or k-step][sub-block]([hi, lo]); hidden part (row-outer): one chunk per 32 rows
//   [quad][b] / [k-step][b][hi, lo]; out layer: one chunk [quad] / [k-step][hi, lo] of sub-block 0.
//   A skip layer's hidden chunks come before its encoding chunks.
struct Walker {
  bool split;
  std::vector<float>* s32;
  std::vector<_Float16>* s3;
  std::vector<int>* chunks;
  // map mode (nrt_mlp_refresh): the source index of every FP32 stream element into
  // [W_0 .. W_{L+1} | b_0 .. b_{L+1}] instead of its value (-1: padding)
  std::vector<int>* map = nullptr;
  size_t pieces() const {
    return map ? map->size() / 256 : split ? s3->size() / 512 : s32->size() / 256;
  }
  void chunk_begin() { chunks->push_back((int)pieces()); chunks->push_back(0); }
  void chunk_end() { chunks->back() = (int)pieces() - chunks->at(chunks->size() - 2); }
};

// with_out = false: the backward program's forward part (no out layer)
int walk_mlp(const nrt_mlp* m, Walker& w, std::vector<float>& lscale, bool with_out = true) {
  const nrt_mlp_desc& d = m->desc;
  const int H = d.hidden, L = d.num_layers, F = d.freqs, in = 3;
  const int dp = in + 2 * F;
  const int ke = (dp + 15) / 16 * 16, ke3 = (dp + 31) / 32 * 32;
  const int NSB = H / 16, NC = H / 32;
  // slot -> column of the encoding [x, sin, cos]
  auto slot_col = [&](int s) -> int {
    if (s < 2 * F) return (s & 1) ? in + F + (s >> 1) : in + (s >> 1);
    if (s < 2 * F + in) return s - 2 * F;
    return -1;
  };
  const int nl = L + 2;
  std::vector<int> R(nl), C(nl);
  std::vector<char> hid(nl), enc(nl);
  for (int l = 0; l < nl; ++l) {
    const bool skip = l >= 1 && l <= L && (l - 1) != L - 1 && ((l - 1) % d.skip) == 0;
    hid[l] = l >= 1;
    enc[l] = l == 0 || skip;
    R[l] = l == nl - 1 ? d.out : H;
    C[l] = (hid[l] ? H : 0) + (enc[l] ? dp : 0);
    if ((int64_t)m->host_w[l].size() != (int64_t)R[l] * C[l]) {
      set_error("shading program: weight shape mismatch");
      return NRT_EINVAL;
    }
  }
  lscale.assign(nl, 1.f);
  if (w.split)
    for (int l = 0; l < nl; ++l) {
      float mx = 0.f;
      for (float v : m->host_w[l]) mx = std::max(mx, std::fabs(v));
      int e = 0;
      if (mx > 0.f && std::isfinite(mx)) (void)std::frexp(mx, &e);
      lscale[l] = std::ldexp(1.f, std::max(-64, std::min(64, 1 - e)));  // max|W| scale in [1, 2)
    }
  std::vector<int64_t> woff(nl + 1, 0);
  for (int l = 0; l < nl; ++l) woff[l + 1] = woff[l] + (int64_t)R[l] * C[l];
  auto W = [&](int l, int row, int col) -> float {
    if (row >= R[l] || col < 0 || col >= C[l]) return 0.f;
    return m->host_w[l][(size_t)row * C[l] + col];
  };
  auto Widx = [&](int l, int row, int col) -> int {
    if (row >= R[l] || col < 0 || col >= C[l]) return -1;
    return (int)(woff[l] + (int64_t)row * C[l] + col);
  };
  auto enc_col = [&](int l, int slot) -> int {
    const int c = slot_col(slot);
    return c < 0 ? -1 : (hid[l] ? H + c : c);
  };
  // FP32 element (l, row, col): its value, or in map mode its source index
  auto put32 = [&](int l, int row, int col) {
    if (w.map) w.map->push_back(Widx(l, row, col));
    else w.s32->push_back(W(l, row, col));
  };
  auto put3 = [&](int l, float v, int part) {
    const float x = v * lscale[l];
    const _Float16 hi = (_Float16)x;
    w.s3->push_back(part == 0 ? hi : (_Float16)(x - (float)hi));
  };
  auto enc_part = [&](int l) {
    if (!w.split) {
      const int QE = ke / 16, EQ = NSB >= 16 ? 2 : 32 / NSB;
      for (int u0 = 0; u0 < QE; u0 += EQ) {
        w.chunk_begin();
        for (int u = u0; u < std::min(QE, u0 + EQ); ++u)
          for (int sb = 0; sb < NSB; ++sb)
            for (int lane = 0; lane < 64; ++lane)
              for (int t = 0; t < 4; ++t) {
                const int g = lane >> 4, s = 4 * u + t;
                put32(l, 16 * sb + (lane & 15), enc_col(l, 4 * s + g));
              }
        w.chunk_end();
      }
    } else {
      const int KQ = ke3 / 32, EK = NSB >= 16 ? 1 : 16 / NSB;
      for (int v0 = 0; v0 < KQ; v0 += EK) {
        w.chunk_begin();
        for (int v = v0; v < std::min(KQ, v0 + EK); ++v)
          for (int sb = 0; sb < NSB; ++sb)
            for (int part = 0; part < 2; ++part)
              for (int lane = 0; lane < 64; ++lane)
                for (int e = 0; e < 8; ++e) {
                  const int g = lane >> 4;
                  put3(l, W(l, 16 * sb + (lane & 15), enc_col(l, 32 * v + 8 * g + e)), part);
                }
        w.chunk_end();
      }
    }
  };
  // hidden part of layer l, rows 32 ib + 16 b (nb = 2 sub-blocks, or 1 for the out layer)
  auto hidden_chunk = [&](int l, int ib, int nb) {
    w.chunk_begin();
    if (!w.split) {
      for (int u = 0; u < H / 16; ++u)
        for (int b = 0; b < nb; ++b)
          for (int lane = 0; lane < 64; ++lane)
            for (int t = 0; t < 4; ++t) {
              const int g = lane >> 4, s = 4 * u + t;
              put32(l, 32 * ib + 16 * b + (lane & 15), 16 * (s >> 2) + 4 * g + (s & 3));
            }
    } else {
      for (int u = 0; u < H / 32; ++u)
        for (int b = 0; b < nb; ++b)
          for (int part = 0; part < 2; ++part)
            for (int lane = 0; lane < 64; ++lane)
              for (int e = 0; e < 8; ++e) {
                const int g = lane >> 4;
                put3(l, W(l, 32 * ib + 16 * b + (lane & 15), 16 * (2 * u + (e >> 2)) + 4 * g + (e & 3)),
                     part);
              }
    }
    w.chunk_end();
  };
  enc_part(0);
  for (int i = 0; i < L; ++i) {  // skip layers: hidden part first, then the encoding part
    for (int ib = 0; ib < NC; ++ib) hidden_chunk(1 + i, ib, 2);
    if (enc[1 + i]) enc_part(1 + i);
  }
  if (with_out) hidden_chunk(L + 1, 0, 1);
  return NRT_OK;
}

// The transposed layers of the ring backward (nrt_train_ring.h bwd32), FP32, in the order it
// consumes them: T-out (one chunk [sb][lane][t]: lane (g, i) = W_out[4 g + t][16 sb + i], the
// outputs padded to 16), then for l = L .. 1 the T-enc chunks of a skip layer and the T-hidden
// chunks of layer l, then the init layer's T-enc chunks.  A T chunk is 32 output rows (inputs j of
// layer l: hidden features, or encoding slots 32 c + 16 b + i) x the layer's H outputs in the
// ring32 k order: quad u, sub-block b, lane (g, i), t -> W_l[16 u + 4 g + t][j].
int walk_mlp_bwd(const nrt_mlp* m, Walker& w) {
  const nrt_mlp_desc& d = m->desc;
  const int H = d.hidden, L = d.num_layers, F = d.freqs, in = 3;
  const int dp = in + 2 * F, NSB = H / 16, NC = H / 32, QH = H / 16;
  const int CEN = (dp + 31) / 32;
  const int nl = L + 2;
  std::vector<int> R(nl), C(nl);
  std::vector<char> hid(nl), enc(nl);
  for (int l = 0; l < nl; ++l) {
    const bool skip = l >= 1 && l <= L && (l - 1) != L - 1 && ((l - 1) % d.skip) == 0;
    hid[l] = l >= 1;
    enc[l] = l == 0 || skip;
    R[l] = l == nl - 1 ? d.out : H;
    C[l] = (hid[l] ? H : 0) + (enc[l] ? dp : 0);
    if ((int64_t)m->host_w[l].size() != (int64_t)R[l] * C[l]) {
      set_error("backward program: weight shape mismatch");
      return NRT_EINVAL;
    }
  }
  std::vector<int64_t> woff(nl + 1, 0);
  for (int l = 0; l < nl; ++l) woff[l + 1] = woff[l] + (int64_t)R[l] * C[l];
  auto slot_col = [&](int s) -> int {
    if (s < 2 * F) return (s & 1) ? in + F + (s >> 1) : in + (s >> 1);
    if (s < 2 * F + in) return s - 2 * F;
    return -1;
  };
  auto put32 = [&](int l, int row, int col) {
    const bool ok = row < R[l] && col >= 0 && col < C[l];
    if (w.map) w.map->push_back(ok ? (int)(woff[l] + (int64_t)row * C[l] + col) : -1);
    else w.s32->push_back(ok ? m->host_w[l][(size_t)row * C[l] + col] : 0.f);
  };
  // T-out
  w.chunk_begin();
  for (int sb = 0; sb < NSB; ++sb)
    for (int lane = 0; lane < 64; ++lane)
      for (int t = 0; t < 4; ++t) put32(L + 1, 4 * (lane >> 4) + t, 16 * sb + (lane & 15));
  w.chunk_end();
  // one T chunk of layer l: output rows j = col(32 c + 16 b + i)
  auto t_chunk = [&](int l, int c, auto&& col) {
    w.chunk_begin();
    for (int u = 0; u < QH; ++u)
      for (int b = 0; b < 2; ++b)
        for (int lane = 0; lane < 64; ++lane)
          for (int t = 0; t < 4; ++t)
            put32(l, 16 * u + 4 * (lane >> 4) + t, col(32 * c + 16 * b + (lane & 15)));
    w.chunk_end();
  };
  auto t_enc = [&](int l) {
    for (int c = 0; c < CEN; ++c)
      t_chunk(l, c, [&](int s) { const int cc = slot_col(s); return cc < 0 ? -1 : (hid[l] ? H + cc : cc); });
  };
  for (int l = L; l >= 1; --l) {
    if (enc[l]) t_enc(l);
    for (int c = 0; c < NC; ++c) t_chunk(l, c, [](int j) { return j; });
  }
  t_enc(0);
  return NRT_OK;
}

}  // namespace

// mode 0: the MLPs' forward evaluation; mode 1 (one FP32 MLP): the ring backward's program,
// the forward without the out layer, then the transposed layers (walk_mlp_bwd)
int build_rprog(const std::vector<const nrt_mlp*>& mlps, bool split, nrt_rprog& out, int mode) {
  out.built = true;
  out.ok = false;
  if (mlps.empty() || (int)mlps.size() > kMaxProgMlp) return NRT_OK;
  if (mode == 1 && (split || mlps.size() != 1)) return NRT_OK;
  RProgDev& d = out.d;
  std::memset(&d, 0, sizeof(d));
  std::vector<float> s32;
  std::vector<_Float16> s3;
  std::vector<int> chunks;
  std::vector<float> bias, scales;
  std::vector<float4> basis;
  Walker w{split, &s32, &s3, &chunks};
  for (size_t k = 0; k < mlps.size(); ++k) {
    const nrt_mlp* m = mlps[k];
    const nrt_mlp_desc& md = m->desc;
    std::vector<float> lscale;
    if (int rc = walk_mlp(m, w, lscale, mode == 0)) return rc;
    if (mode == 1) {
      out.fwd_chunks = (int)chunks.size() / 2;
      if (int rc = walk_mlp_bwd(m, w)) return rc;
    }
    RProgMlp& pm = d.mlp[k];
    pm.L = md.num_layers; pm.skip = md.skip; pm.F = md.freqs; pm.out = md.out;
    pm.bstride = md.hidden;  // >= 16 rows of the out layer's sub-block
    pm.bias_off = (int)bias.size();
    const int hs = m->host_dev.bias16_stride;
    for (int l = 0; l < md.num_layers + 2; ++l) {
      const int rows = l == md.num_layers + 1 ? md.out : md.hidden;
      for (int r = 0; r < pm.bstride; ++r)
        bias.push_back(r < rows ? m->host_bias[(size_t)l * hs + r] * lscale[l] : 0.f);
    }
    pm.scale_off = -1;  // filled below (scales follow the biases)
    for (int l = 0; l < md.num_layers + 2; ++l) scales.push_back(1.f / lscale[l]);
    pm.basis_off = (int)basis.size();
    const int F = md.freqs;
    for (int q = 0; q < F; ++q)
      basis.push_back(make_float4(m->host_basis[q], m->host_basis[F + q], m->host_basis[2 * F + q], 0.f));
  }
  {
    int off = (int)bias.size();
    for (size_t k = 0; k < mlps.size(); ++k) {
      d.mlp[k].scale_off = off;
      off += mlps[k]->desc.num_layers + 2;
    }
  }
  std::vector<float> tables(bias);
  tables.insert(tables.end(), scales.begin(), scales.end());
  d.n_mlp = (int)mlps.size();
  d.n_chunks = (int)chunks.size() / 2;
  d.table_floats = (int)tables.size();
  d.basis_q = (int)basis.size();
  const size_t sbytes = split ? s3.size() * sizeof(_Float16) : s32.size() * sizeof(float);
  if (sbytes >= (size_t)1 << 30) return NRT_OK;
  const size_t o_chunks = align256(sbytes);
  const size_t o_tab = align256(o_chunks + chunks.size() * 4);
  const size_t o_basis = align256(o_tab + tables.size() * 4);
  const size_t total = align256(o_basis + std::max<size_t>(basis.size(), 1) * 16);
  char* buf = nullptr;
  NRT_HIP(hipMalloc((void**)&buf, total));
  out.buf = buf;
  NRT_HIP(hipMemcpy(buf, split ? (const void*)s3.data() : (const void*)s32.data(), sbytes,
                    hipMemcpyHostToDevice));
  NRT_HIP(hipMemcpy(buf + o_chunks, chunks.data(), chunks.size() * 4, hipMemcpyHostToDevice));
  NRT_HIP(hipMemcpy(buf + o_tab, tables.data(), tables.size() * 4, hipMemcpyHostToDevice));
  if (!basis.empty())
    NRT_HIP(hipMemcpy(buf + o_basis, basis.data(), basis.size() * 16, hipMemcpyHostToDevice));
  d.stream = buf;
  d.stream_bytes = (int)sbytes;
  d.chunks = reinterpret_cast<const int*>(buf + o_chunks);
  d.tables = reinterpret_cast<const float*>(buf + o_tab);
  d.basis = reinterpret_cast<const float4*>(buf + o_basis);
  out.ok = true;
  return NRT_OK;
}

namespace {
constexpr int kRWaves = 8;

template <class K>
int persistent_grid(K kern, int threads, size_t lds, int64_t want) {
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

// ring depth: 3 slots where they fit beside the tables in the CU's LDS, else 2
template <int PREC, int WV, class F>
int with_depth(const RProgDev& d, F&& f) {
  if (rprog::Engine<3, WV>::lds_bytes(d) <= (size_t)kLdsBytes) return f(std::integral_constant<int, 3>{});
  if (rprog::Engine<2, WV>::lds_bytes(d) <= (size_t)kLdsBytes) return f(std::integral_constant<int, 2>{});
  return NRT_EUNSUPPORTED;
}

int blocks_per_cu(const void* kern, int threads, size_t lds) {
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, threads, lds) != hipSuccess) return 1;
  return std::max(per_cu, 1);
}

// as with_depth, but 2 slots where that keeps more blocks resident on a CU (a kernel with few
// registers: the 3-slot ring's LDS would hold the CU to one block); kern_of(depth) names the
// kernel of each depth
template <int WV, class KF, class F>
int with_depth_occ(const RProgDev& d, KF&& kern_of, F&& f) {
  using D3 = std::integral_constant<int, 3>;
  using D2 = std::integral_constant<int, 2>;
  const size_t l3 = rprog::Engine<3, WV>::lds_bytes(d), l2 = rprog::Engine<2, WV>::lds_bytes(d);
  if (l3 <= (size_t)kLdsBytes) {
    if (l2 <= (size_t)kLdsBytes &&
        blocks_per_cu(reinterpret_cast<const void*>(kern_of(D2{})), 64 * WV, l2) >
            blocks_per_cu(reinterpret_cast<const void*>(kern_of(D3{})), 64 * WV, l3))
      return f(D2{});
    return f(D3{});
  }
  if (l2 <= (size_t)kLdsBytes) return f(D2{});
  return NRT_EUNSUPPORTED;
}
}  // namespace

// NRT_EUNSUPPORTED when the row-program kernels do not cover this light / BSDF pair
int shade_ring(const nrt_bsdf* b, const nrt_light* l, const float* p, const float* n,
               const float* wi, const int32_t* hit_idx, const int32_t* hit_count, int64_t P,
               const float* lscale, float* rgb, float* weights_out, int precision, hipStream_t st) {
  const bool split = precision == NRT_FP32_SPLIT || precision == NRT_MIXED;  // NRT_MIXED shades at fp32-split
  const int pi = split ? 1 : 0;
  const bool field = l->host_dev.kind == 0;
  if (b->host_dev.n > 16) return NRT_EUNSUPPORTED;
  // build on first use
  nrt_rprog& lp = l->rprog[pi];
  nrt_rprog& bp = b->rprog[pi];
  if (field && !lp.built) {
    if (l->mlp && shape_ok(l->mlp, kLightSpec) && l->mlp->desc.out == 3) {
      if (int rc = build_rprog({l->mlp}, split, lp)) return rc;
    } else {
      lp.built = true;
    }
  }
  if (!bp.built) {
    std::vector<const nrt_mlp*> v;
    bool ok = true;
    if (b->spatial) {
      ok = shape_ok(b->spatial, kSpatialSpec);
      v.push_back(b->spatial);
    }
    for (const nrt_mlp* m : b->mlps) ok = ok && shape_ok(m, kBsdfSpec) && m->desc.out == 3;
    v.insert(v.end(), b->mlps.begin(), b->mlps.end());
    if (ok && !v.empty()) {
      if (int rc = build_rprog(v, split, bp)) return rc;
    } else {
      bp.built = true;
    }
  }
  if ((field && !lp.ok) || !bp.ok) return NRT_EUNSUPPORTED;
  constexpr int WV = kRWaves;
  float* ls = nullptr;
  NRT_HIP(hipMallocAsync((void**)&ls, (size_t)std::max<int64_t>(P, 1) * kLsStride * sizeof(float), st));
  const int64_t want = ceil_div64(P, 16 * WV);
  int rc = NRT_OK;
  auto run = [&]<int PREC>() -> int {
    {
      ProfScope prof(PREC == 2 ? "k_light3" : "k_light32", st);
      if (field) {
        rc = with_depth<PREC, WV>(lp.d, [&](auto dd) -> int {
          constexpr int D = decltype(dd)::value;
          auto kern = rprog::k_light_r<PREC, D, WV>;
          const size_t lds = rprog::Engine<D, WV>::lds_bytes(lp.d);
          if (int r = set_lds(kern, lds)) return r;
          kern<<<dim3(persistent_grid(kern, 64 * WV, lds, want)), dim3(64 * WV), lds, st>>>(
              lp.d, l->dev, p, n, wi, hit_idx, hit_count, lscale, ls);
          return check_launch("k_light_r");
        });
      } else {
        auto kern = k_light16<WV, false>;  // point light: VALU only, FP32 math
        kern<<<dim3(persistent_grid(kern, 64 * WV, 0, ceil_div64(P, 32 * WV))), dim3(64 * WV), 0, st>>>(
            ProgDev{}, l->dev, p, n, wi, hit_idx, hit_count, lscale, ls);
        rc = check_launch("k_light16");
      }
    }
    if (rc) return rc;
    ProfScope prof(PREC == 2 ? "k_bsdf3" : "k_bsdf32", st);
    return with_depth<PREC, WV>(bp.d, [&](auto dd) -> int {
      constexpr int D = decltype(dd)::value;
      const size_t lds = rprog::Engine<D, WV>::lds_bytes(bp.d);
      auto launch = [&](auto kern) -> int {
        if (int r = set_lds(kern, lds)) return r;
        kern<<<dim3(persistent_grid(kern, 64 * WV, lds, want)), dim3(64 * WV), lds, st>>>(
            bp.d, b->dev, p, wi, hit_idx, hit_count, ls, rgb, weights_out);
        return check_launch("k_bsdf_r");
      };
      return b->spatial ? launch(rprog::k_bsdf_r<PREC, D, WV, true>)
                        : launch(rprog::k_bsdf_r<PREC, D, WV, false>);
    });
  };
  rc = split ? run.template operator()<2>() : run.template operator()<0>();
  (void)hipFreeAsync(ls, st);
  return rc;
}

// ---- nrt_mlp_forward on the ring engine (training forwards of the shading MLPs) -------------
namespace {
// the compiled shapes; 0 = none
int solo_shape(const nrt_mlp* m) {
  const nrt_mlp_desc& d = m->desc;
  if (d.in_size != 3 || d.latent != 0 || d.out > 16 || d.activation != NRT_ACT_LEAKY_RELU ||
      d.num_layers + 2 > kMaxLin || (int)m->host_w.size() != d.num_layers + 2)
    return 0;
  if (d.hidden == kLightSpec.H && d.freqs == kLightSpec.F) return 1;
  if (d.hidden == kSpatialSpec.H && d.freqs == kSpatialSpec.F) return 2;
  if (d.hidden == kBsdfSpec.H && d.freqs == kBsdfSpec.F) return 3;
  return 0;
}
}  // namespace

// the refresh's gather maps of the solo program: its FP32 stream and bias table as source
// indices into [W_0 .. W_{L+1} | b_0 .. b_{L+1}] (-1 padding); builds the program first
// (from the host copies, which the refresh then overwrites).  false: not eligible.
bool solo_refresh_maps(const nrt_mlp* m, std::vector<int>& stream_map, std::vector<int>& bias_map,
                       void*& stream_dst, void*& bias_dst) {
  if (!solo_shape(m)) return false;
  nrt_rprog& sp = m->solo32;
  if (!sp.built && build_rprog({m}, false, sp) != NRT_OK) return false;
  if (!sp.ok) return false;
  std::vector<int> chunks;
  std::vector<float> lscale;
  Walker w{false, nullptr, nullptr, &chunks, &stream_map};
  if (walk_mlp(m, w, lscale) != NRT_OK) return false;
  const nrt_mlp_desc& d = m->desc;
  int64_t wtot = 0;
  for (const auto& v : m->host_w) wtot += (int64_t)v.size();
  int64_t boff = wtot;
  const int bstride = d.hidden;
  for (int l = 0; l < d.num_layers + 2; ++l) {
    const int rows = l == d.num_layers + 1 ? d.out : d.hidden;
    for (int r = 0; r < bstride; ++r) bias_map.push_back(r < rows ? (int)(boff + r) : -1);
    boff += rows;
  }
  if ((int64_t)stream_map.size() * 4 != sp.d.stream_bytes) return false;
  stream_dst = const_cast<void*>(sp.d.stream);
  bias_dst = const_cast<float*>(sp.d.tables);  // biases first (scales follow, 1 in FP32)
  return true;
}

// the backward program's refresh maps (as solo_refresh_maps, for m->bwd32)
bool bwd_refresh_maps(const nrt_mlp* m, std::vector<int>& stream_map, std::vector<int>& bias_map,
                      void*& stream_dst, void*& bias_dst) {
  if (!solo_shape(m)) return false;
  nrt_rprog& bp = m->bwd32;
  if (!bp.built && build_rprog({m}, false, bp, 1) != NRT_OK) return false;
  if (!bp.ok) return false;
  std::vector<int> chunks;
  std::vector<float> lscale;
  Walker w{false, nullptr, nullptr, &chunks, &stream_map};
  if (walk_mlp(m, w, lscale, false) != NRT_OK || walk_mlp_bwd(m, w) != NRT_OK) return false;
  const nrt_mlp_desc& d = m->desc;
  int64_t wtot = 0;
  for (const auto& v : m->host_w) wtot += (int64_t)v.size();
  int64_t boff = wtot;
  for (int l = 0; l < d.num_layers + 2; ++l) {
    const int rows = l == d.num_layers + 1 ? d.out : d.hidden;
    for (int r = 0; r < d.hidden; ++r) bias_map.push_back(r < rows ? (int)(boff + r) : -1);
    boff += rows;
  }
  if ((int64_t)stream_map.size() * 4 != bp.d.stream_bytes) return false;
  stream_dst = const_cast<void*>(bp.d.stream);
  bias_dst = const_cast<float*>(bp.d.tables);
  return true;
}

size_t ring_backward_table_bytes(int n) { return (size_t)std::max(n, 1) * sizeof(rprog::BwdRingJob); }

bool ring_backward_ok(const nrt_mlp* const* mlps, int n) {
  if (option(OPT_BWD_RING) == 0 || n < 1) return false;
  const int shape = solo_shape(mlps[0]);
  if (!shape) return false;
  for (int k = 0; k < n; ++k) {
    const nrt_mlp* m = mlps[k];
    if (solo_shape(m) != shape) return false;
    if (m->refreshed && !m->bwd_in_refresh) return false;
    if (!m->bwd32.built && build_rprog({m}, false, m->bwd32, 1) != NRT_OK) return false;
    if (!m->bwd32.ok) return false;
  }
  return true;
}

int ring_backward(const nrt_mlp* const* mlps, int n, const float* x, int64_t M,
                  const float* const* dy, float* const* dx, float* const* A, float* const* dZ,
                  float* const* Eraw, float* const* Eact, void* table, hipStream_t st,
                  const int32_t* rows, int64_t Ms, float* const* Acopy, const float* const* Sraw,
                  const float* const* Sact) {
  if (!ring_backward_ok(mlps, n)) return NRT_EUNSUPPORTED;
  const bool saved = Ms >= 0;
  std::vector<rprog::BwdRingJob> jobs(n);
  for (int k = 0; k < n; ++k)
    jobs[k] = rprog::BwdRingJob{mlps[k]->bwd32.d, dy[k], dx ? dx[k] : nullptr, A[k], dZ[k],
                                Eraw ? Eraw[k] : nullptr, Eact ? Eact[k] : nullptr, rows,
                                saved ? Ms : M, mlps[k]->bwd32.fwd_chunks,
                                Acopy ? Acopy[k] : nullptr, Sraw ? Sraw[k] : nullptr,
                                Sact ? Sact[k] : nullptr};
  NRT_HIP(hipMemcpyAsync(table, jobs.data(), (size_t)n * sizeof(rprog::BwdRingJob),
                         hipMemcpyHostToDevice, st));
  const auto* tj = (const rprog::BwdRingJob*)table;
  constexpr int WV = kRWaves;
  const int64_t want = ceil_div64(M, 16 * WV);
  const RProgDev& d0 = mlps[0]->bwd32.d;  // the same shape: the same LDS plan for every MLP
  auto run = [&](auto sh) -> int {
    using S = decltype(sh);
    auto go = [&](auto sv) -> int {
      constexpr bool SV = decltype(sv)::value;
      return with_depth_occ<WV>(d0, [](auto dd) { return rprog::k_mlp_bwd_ring<decltype(dd)::value, WV, S, SV>; },
                                [&](auto dd) -> int {
        constexpr int D = decltype(dd)::value;
        auto kern = rprog::k_mlp_bwd_ring<D, WV, S, SV>;
        const size_t lds = rprog::Engine<D, WV>::lds_bytes(d0);
        if (int r = set_lds(kern, lds)) return r;
        kern<<<dim3(persistent_grid(kern, 64 * WV, lds, want), n), dim3(64 * WV), lds, st>>>(tj, x, M);
        return check_launch("k_mlp_bwd_ring");
      });
    };
    return saved ? go(std::true_type{}) : go(std::false_type{});
  };
  const int shape = solo_shape(mlps[0]);
  if (shape == 1) return run(rprog::LightShape{});
  if (shape == 2) return run(rprog::SpatialShape{});
  return run(rprog::BsdfShape{});
}

// NRT_EUNSUPPORTED when an MLP has no compiled ring shape, the MLPs' shapes differ, or a
// refreshed handle's solo program is not covered by its refresh
// the training forward can save activations for the ring backward (nrt_mlp_save_bytes > 0)
bool saved_forward_ok(const nrt_mlp* m) {
  if (option(OPT_SHADE_RING) == 0 || !solo_shape(m) || (m->refreshed && !m->solo_in_refresh)) return false;
  return ring_backward_ok(&m, 1);
}

static_assert(kMaxSoloForward == rprog::kMaxSoloJobs, "solo job table size");
int solo_forward_multi(const nrt_mlp* const* mlps, int n, const float* x, int64_t M,
                       float* const* y, hipStream_t st, void* const* save) {
  if (n < 1 || n > rprog::kMaxSoloJobs) return NRT_EUNSUPPORTED;
  const int shape = solo_shape(mlps[0]);
  if (!shape) return NRT_EUNSUPPORTED;
  if (save && !ring_backward_ok(mlps, n)) return NRT_EUNSUPPORTED;
  rprog::SoloJobs jobs{};
  for (int k = 0; k < n; ++k) {
    const nrt_mlp* m = mlps[k];
    if (solo_shape(m) != shape || m->desc.out != mlps[0]->desc.out) return NRT_EUNSUPPORTED;
    nrt_rprog& sp = m->solo32;
    if (m->refreshed && !m->solo_in_refresh) return NRT_EUNSUPPORTED;
    if (!sp.built)
      if (int rc = build_rprog({m}, false, sp)) return rc;
    if (!sp.ok) return NRT_EUNSUPPORTED;
    const RProgDev& d = sp.d;
    SavedActs sa{nullptr, nullptr, nullptr};
    if (save) sa = saved_split(m->host_dev, M, save[k]);
    jobs.j[k] = rprog::SoloJob{d.stream, d.chunks, d.tables, d.basis, y[k], sa.A, sa.Eraw, sa.Eact,
                               d.stream_bytes, d.n_chunks, d.table_floats, d.basis_q, m->desc.out,
                               d.mlp[0]};
  }
  constexpr int WV = kRWaves;
  const int64_t want = ceil_div64(M, 16 * WV);
  const RProgDev& d0 = mlps[0]->solo32.d;  // one shape: one LDS plan
  auto run = [&](auto sh) -> int {
    using S = decltype(sh);
    auto go = [&](auto sv) -> int {
      constexpr bool SV = decltype(sv)::value;
      return with_depth_occ<WV>(d0, [](auto dd) { return rprog::k_mlp_ring<decltype(dd)::value, WV, S, SV>; },
                                [&](auto dd) -> int {
        constexpr int D = decltype(dd)::value;
        auto kern = rprog::k_mlp_ring<D, WV, S, SV>;
        const size_t lds = rprog::Engine<D, WV>::lds_bytes(d0);
        if (int r = set_lds(kern, lds)) return r;
        ProfScope prof("k_mlp_ring32", st);
        kern<<<dim3(persistent_grid(kern, 64 * WV, lds, want), n), dim3(64 * WV), lds, st>>>(jobs, x, M);
        return check_launch("k_mlp_ring32");
      });
    };
    return save ? go(std::true_type{}) : go(std::false_type{});
  };
  if (shape == 1) return run(rprog::LightShape{});
  if (shape == 2) return run(rprog::SpatialShape{});
  return run(rprog::BsdfShape{});
}

int solo_forward(const nrt_mlp* m, const float* x, int64_t M, float* y, hipStream_t st) {
  return solo_forward_multi(&m, 1, x, M, &y, st);
}

}  // namespace nrt
