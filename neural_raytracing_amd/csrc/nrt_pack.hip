// nrt_pack.hip -- host packer: torch-layout SkipConnMLP weights -> per-lane MFMA A fragments.
//
// Layer l input positions (neural_blocks.py:46-55, 80-86):
//   l = 0 (init)          : encoding slots                       (reference columns: enc cols)
//   l = 1..L (layers[l-1]): hidden 0..H-1, then slots if skip    (columns: h, then H + enc col)
//   l = L+1 (out)         : hidden 0..H-1
// Fragment (kstep s, rowblock ib) holds, for lane (i = l&31, half hf = l>>5), the values of
// W[32 ib + i][column] that the MFMA consumes at that lane:
//   FP16 hidden k-steps use the accumulator-as-operand order (k = 16*(s&1) + 8*(j>>2) + 4hf + (j&3)
//   inside 32-row block s>>1); FP16 encoding k-steps use slot 16s + 8hf + j; FP32 k-steps use
//   position 2s + hf.  W^T fragments (FP32 backward) swap the roles of rows and positions.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <atomic>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "nrt_internal.h"

namespace {

struct Layer {
  const float* W;  // [R][C]
  const float* b;  // [R]
  int R, C;
  bool hidden_in;  // has the H hidden inputs
  bool enc_in;     // has the encoding slots
};

struct Blob {
  std::vector<char> bytes;
  size_t add(const void* p, size_t n) {
    size_t off = (bytes.size() + 255) & ~size_t(255);
    bytes.resize(off + n);
    std::memcpy(bytes.data() + off, p, n);
    return off;
  }
};

}  // namespace

extern "C" int nrt_mlp_create(const nrt_mlp_desc* d, const float* basis,
                              const float* const* weights, const float* const* biases,
                              nrt_mlp** out) {
  using namespace nrt;
  if (!d || (!basis && d->freqs > 0) || !weights || !biases || !out) {
    set_error("nrt_mlp_create: null argument");
    return NRT_EINVAL;
  }
  const int in = d->in_size, H = d->hidden, L = d->num_layers, O = d->out, F = d->freqs;
  const int lat = d->latent;
  if (in < 1 || H < 32 || H % 32 || H > 256 || L < 1 || L + 2 > kMaxLin || O < 1 || O > 96 ||
      F < 0 || d->skip < 1 || lat < 0) {
    set_error("nrt_mlp_create: unsupported shape (hidden must be 32..256 step 32, out <= 96, "
              "layers <= 18)");
    return NRT_EUNSUPPORTED;
  }
  const int NB = H / 32;
  if (NB != 1 && NB != 2 && NB != 3 && NB != 4 && NB != 8) {
    set_error("nrt_mlp_create: hidden must be one of 32, 64, 96, 128, 256");
    return NRT_EUNSUPPORTED;
  }
  const int dp = in + 2 * F + lat;
  const int ke = (dp + 15) / 16 * 16;
  const int OB = (O + 31) / 32;

  // encoding slot -> reference encoding column ([x, sin, cos, latent]); -1 = padding
  std::vector<int> slot_col(ke, -1);
  for (int s = 0; s < ke; ++s) {
    if (s < 2 * F) slot_col[s] = (s & 1) ? in + F + (s >> 1) : in + (s >> 1);
    else if (s < 2 * F + in) slot_col[s] = s - 2 * F;
    else if (s < 2 * F + in + lat) slot_col[s] = in + 2 * F + (s - 2 * F - in);
  }

  std::vector<Layer> layers;
  layers.push_back({weights[0], biases[0], H, dp, false, true});
  for (int i = 0; i < L; ++i) {
    bool skip = (i != L - 1) && (i % d->skip == 0);
    layers.push_back({weights[1 + i], biases[1 + i], H, skip ? H + dp : H, true, skip});
  }
  layers.push_back({weights[L + 1], biases[L + 1], O, H, true, false});

  auto col_of_hidden = [](int k) { return k; };
  auto col_of_slot = [&](const Layer& ly, int slot) {
    int c = slot_col[slot];
    if (c < 0) return -1;
    return ly.hidden_in ? H + c : c;
  };
  auto wval = [](const Layer& ly, int row, int col) -> float {
    if (row < 0 || row >= ly.R || col < 0 || col >= ly.C) return 0.f;
    return ly.W[(size_t)row * ly.C + col];
  };

  Blob blob;
  MlpDev md;
  std::memset(&md, 0, sizeof(md));
  md.in_size = in; md.hidden = H; md.n_hidden = L; md.out = O; md.freqs = F;
  md.skip = d->skip; md.latent = lat; md.act = d->activation;
  md.dp = dp; md.ke = ke; md.nb = NB; md.ob = OB;

  // [in, F] basis; at F = 0 the caller's basis is empty (it may be null) and a zero row stands in
  // (found by the host ASan run, tools/asan: the copy read `in` floats past an empty basis)
  std::vector<float> basis_h((size_t)in * (F > 0 ? F : 1), 0.f);
  if (F > 0) std::memcpy(basis_h.data(), basis, sizeof(float) * (size_t)in * F);
  size_t off_basis = blob.add(basis_h.data(), sizeof(float) * basis_h.size());
  std::vector<size_t> off16(layers.size()), off32(layers.size()), offt(layers.size()),
      offb(layers.size());

  for (size_t l = 0; l < layers.size(); ++l) {
    const Layer& ly = layers[l];
    const int nrb = (ly.R + 31) / 32;
    // ---- FP16 fragments
    {
      std::vector<_Float16> f;
      const int ks_h = ly.hidden_in ? 2 * NB : 0;
      const int ks_e = ly.enc_in ? ke / 16 : 0;
      f.resize((size_t)(ks_h + ks_e) * nrb * 64 * 8);
      for (int s = 0; s < ks_h + ks_e; ++s)
        for (int ib = 0; ib < nrb; ++ib)
          for (int lane = 0; lane < 64; ++lane) {
            int i = lane & 31, hf = lane >> 5;
            for (int j = 0; j < 8; ++j) {
              int col;
              if (s < ks_h) {
                int k = 32 * (s >> 1) + 16 * (s & 1) + 8 * (j >> 2) + 4 * hf + (j & 3);
                col = col_of_hidden(k);
              } else {
                col = col_of_slot(ly, 16 * (s - ks_h) + 8 * hf + j);
              }
              f[(((size_t)s * nrb + ib) * 64 + lane) * 8 + j] = (_Float16)wval(ly, 32 * ib + i, col);
            }
          }
      off16[l] = blob.add(f.data(), f.size() * sizeof(_Float16));
    }
    // ---- FP32 fragments (natural k order over the slab: hidden then slots)
    {
      const int ks_h = ly.hidden_in ? H / 2 : 0;
      const int ks_e = ly.enc_in ? ke / 2 : 0;
      std::vector<float> f((size_t)(ks_h + ks_e) * nrb * 64);
      for (int s = 0; s < ks_h + ks_e; ++s)
        for (int ib = 0; ib < nrb; ++ib)
          for (int lane = 0; lane < 64; ++lane) {
            int i = lane & 31, hf = lane >> 5;
            int col = (s < ks_h) ? col_of_hidden(2 * s + hf) : col_of_slot(ly, 2 * (s - ks_h) + hf);
            f[((size_t)s * nrb + ib) * 64 + lane] = wval(ly, 32 * ib + i, col);
          }
      off32[l] = blob.add(f.data(), f.size() * sizeof(float));
    }
    // ---- FP32 W^T fragments (backward) for init and hidden layers
    if (l + 1 < layers.size()) {
      const int npos = (ly.hidden_in ? H : 0) + (ly.enc_in ? ke : 0);
      const int nrbt = (npos + 31) / 32;
      md.nbt[l] = nrbt;
      const int ks = H / 2;  // k over the layer's H output rows
      std::vector<float> f((size_t)ks * nrbt * 64);
      for (int s = 0; s < ks; ++s)
        for (int ib = 0; ib < nrbt; ++ib)
          for (int lane = 0; lane < 64; ++lane) {
            int i = lane & 31, hf = lane >> 5;
            int pos = 32 * ib + i;
            int col = -1;
            if (pos < npos) {
              if (ly.hidden_in && pos < H) col = col_of_hidden(pos);
              else col = col_of_slot(ly, pos - (ly.hidden_in ? H : 0));
            }
            f[((size_t)s * nrbt + ib) * 64 + lane] = wval(ly, 2 * s + hf, col);
          }
      offt[l] = blob.add(f.data(), f.size() * sizeof(float));
    }
    // ---- bias padded to row blocks
    {
      std::vector<float> b((size_t)nrb * 32, 0.f);
      for (int r = 0; r < ly.R; ++r) b[r] = ly.b[r];
      offb[l] = blob.add(b.data(), b.size() * sizeof(float));
    }
  }
  size_t off_w0 = blob.add(layers.back().W, sizeof(float) * H);  // out.weight[0, :]

  // ---- FP16 row-block-major weight stream (LDS-ring engine)
  const bool fold = d->activation == NRT_ACT_SOFTPLUS;
  const float kLog2e = 1.4426950408889634f, kLn2 = 0.6931471805599453f;
  std::vector<_Float16> stream;
  std::vector<int> chunk_off;
  const int bstride = std::max(NB, OB) * 32;
  std::vector<float> bias16(layers.size() * (size_t)bstride, 0.f);
  for (size_t l = 0; l < layers.size(); ++l) {
    const Layer& ly = layers[l];
    const bool is_init = (l == 0), is_out = (l + 1 == layers.size());
    const float wscale = fold ? (is_init ? kLog2e : (is_out ? kLn2 : 1.f)) : 1.f;
    const float bscale = fold && !is_out ? kLog2e : 1.f;
    const int nrb = (ly.R + 31) / 32;
    const int ks_h = ly.hidden_in ? 2 * NB : 0;
    const int ks_e = ly.enc_in ? ke / 16 : 0;
    auto frag = [&](int s2, int ib) {
      for (int lane = 0; lane < 64; ++lane) {
        int i = lane & 31, hf = lane >> 5;
        for (int j = 0; j < 8; ++j) {
          int col;
          if (s2 < ks_h) col = col_of_hidden(32 * (s2 >> 1) + 16 * (s2 & 1) + 8 * (j >> 2) + 4 * hf + (j & 3));
          else col = col_of_slot(ly, 16 * (s2 - ks_h) + 8 * hf + j);
          stream.push_back((_Float16)(wscale * wval(ly, 32 * ib + i, col)));
        }
      }
    };
    if (is_init || is_out || NB % kRingRB != 0) {
      // init: one chunk [row block][k-step]; out: one chunk of row block 0
      for (int ib = 0; ib < nrb; ++ib) {
        chunk_off.push_back((int)(stream.size() / (64 * 8)));
        for (int s2 = 0; s2 < ks_h + ks_e; ++s2) frag(s2, ib);
      }
    } else {
      // hidden layers: chunks of kRingRB row blocks, fragments [k-step][row block of the chunk]
      for (int c = 0; c < nrb / kRingRB; ++c) {
        chunk_off.push_back((int)(stream.size() / (64 * 8)));
        for (int s2 = 0; s2 < ks_h + ks_e; ++s2)
          for (int b = 0; b < kRingRB; ++b) frag(s2, kRingRB * c + b);
      }
    }
    for (int r = 0; r < ly.R; ++r) bias16[l * bstride + r] = bscale * ly.b[r];
  }
  const int n_chunks = (int)chunk_off.size();
  stream.resize(stream.size() + (size_t)64 * 64 * 8, (_Float16)0.f);  // tail for unguarded prefetch

  // ---- FP16 k-outer stream (program engine): per layer the w16 fragments [kstep][rowblock] in
  // chunks of kc k-steps (hidden and encoding parts chunked separately; the out layer is one
  // chunk of all its k-steps)
  const int kc = std::max(1, 16 / NB);
  std::vector<_Float16> streamk;
  std::vector<int> chunkk_off;
  for (size_t l = 0; l < layers.size(); ++l) {
    const Layer& ly = layers[l];
    const bool is_out = (l + 1 == layers.size());
    const int nrb = (ly.R + 31) / 32;
    const int ks_h = ly.hidden_in ? 2 * NB : 0;
    const int ks_e = ly.enc_in ? ke / 16 : 0;
    const int base = (int)(streamk.size() / (64 * 8));
    auto frag = [&](int s, int ib, int lane, int j) {
      int i = lane & 31, hf = lane >> 5;
      int col = (s < ks_h) ? col_of_hidden(32 * (s >> 1) + 16 * (s & 1) + 8 * (j >> 2) + 4 * hf + (j & 3))
                           : col_of_slot(ly, 16 * (s - ks_h) + 8 * hf + j);
      return (_Float16)wval(ly, 32 * ib + i, col);
    };
    for (int s = 0; s < ks_h + ks_e; ++s)
      for (int ib = 0; ib < nrb; ++ib)
        for (int lane = 0; lane < 64; ++lane)
          for (int j = 0; j < 8; ++j) streamk.push_back(frag(s, ib, lane, j));
    if (is_out) {
      chunkk_off.push_back(base);
    } else {
      for (int s = 0; s < ks_h; s += kc) chunkk_off.push_back(base + s * nrb);
      for (int s = 0; s < ks_e; s += kc) chunkk_off.push_back(base + (ks_h + s) * nrb);
    }
  }
  const int nk_frags = (int)(streamk.size() / (64 * 8));
  streamk.resize(streamk.size() + (size_t)64 * 64 * 8, (_Float16)0.f);

  // ---- FP32 ring stream (nrt_device.h ring32, v_mfma_f32_16x16x4_f32 on 16-ray tiles)
  std::vector<float> stream32;
  {
    std::vector<Ring32Layer> rl;
    for (const Layer& ly : layers) rl.push_back({ly.R, ly.hidden_in, ly.enc_in});
    ring32_walk(rl, H, ke, [&](int l, int row, int pos) {
      const Layer& ly = layers[l];
      const int col = pos < H ? col_of_hidden(pos) : col_of_slot(ly, pos - H);
      stream32.push_back(wval(ly, row, col));
    });
  }
  std::vector<float> bias32(layers.size() * (size_t)bstride, 0.f);
  for (size_t l = 0; l < layers.size(); ++l)
    for (int r = 0; r < layers[l].R; ++r) bias32[l * bstride + r] = layers[l].b[r];
  // ---- split stream (nrt_ring3.h): softplus MLPs folded into the log2 domain like stream16
  // (init W and init / hidden biases x log2 e, out W x ln 2), then per layer a power-of-two
  // scale 2^s with max|W| 2^s in [1, 2), then W 2^s = hi + lo in two RNE f16 halves
  const int ke3 = (dp + 31) / 32 * 32;
  auto wfold = [&](size_t l) {
    return fold ? (l == 0 ? kLog2e : (l + 1 == layers.size() ? kLn2 : 1.f)) : 1.f;
  };
  auto bfold = [&](size_t l) { return fold && l + 1 < layers.size() ? kLog2e : 1.f; };
  std::vector<float> lscale(layers.size(), 1.f);
  for (size_t l = 0; l < layers.size(); ++l) {
    float mx = 0.f;
    const Layer& ly = layers[l];
    for (size_t i = 0; i < (size_t)ly.R * ly.C; ++i) mx = std::max(mx, std::fabs(ly.W[i] * wfold(l)));
    int e = 0;
    if (mx > 0.f && std::isfinite(mx)) (void)std::frexp(mx, &e);  // mx = f 2^e, f in [0.5, 1)
    lscale[l] = std::ldexp(1.f, std::max(-64, std::min(64, 1 - e)));  // mx * scale in [1, 2)
  }
  std::vector<_Float16> stream3;
  {
    std::vector<Ring32Layer> rl;
    for (const Layer& ly : layers) rl.push_back({ly.R, ly.hidden_in, ly.enc_in});
    ring3_walk(rl, H, ke3, [&](int l, int row, int pos, int part) {
      const Layer& ly = layers[l];
      int col = -1;
      if (pos < H) col = col_of_hidden(pos);
      else if (pos - H < ke) col = col_of_slot(ly, pos - H);
      const float w = (wval(ly, row, col) * wfold(l)) * lscale[l];
      const _Float16 hi = (_Float16)w;
      stream3.push_back(part == 0 ? hi : (_Float16)(w - (float)hi));
    });
  }
  std::vector<float> bias3(layers.size() * (size_t)bstride, 0.f);
  for (size_t l = 0; l < layers.size(); ++l)
    for (int r = 0; r < layers[l].R; ++r) bias3[l * bstride + r] = (layers[l].b[r] * bfold(l)) * lscale[l];
  size_t off_stream3 = blob.add(stream3.data(), stream3.size() * sizeof(_Float16));
  size_t off_b3 = blob.add(bias3.data(), bias3.size() * sizeof(float));
  size_t off_stream32 = blob.add(stream32.data(), stream32.size() * sizeof(float));
  size_t off_b32 = blob.add(bias32.data(), bias32.size() * sizeof(float));
  size_t off_streamk = blob.add(streamk.data(), streamk.size() * sizeof(_Float16));
  size_t off_coffk = blob.add(chunkk_off.data(), chunkk_off.size() * sizeof(int));
  size_t off_stream = blob.add(stream.data(), stream.size() * sizeof(_Float16));
  size_t off_coff = blob.add(chunk_off.data(), chunk_off.size() * sizeof(int));
  size_t off_b16 = blob.add(bias16.data(), bias16.size() * sizeof(float));

  std::unique_ptr<nrt_mlp> m(new nrt_mlp());
  m->desc = *d;
  static std::atomic<uint64_t> next_serial{1};
  m->serial = next_serial.fetch_add(1);
  m->blob_bytes = blob.bytes.size();
  m->host_chunkk = chunkk_off;
  m->host_bias.assign(layers.size() * (size_t)bstride, 0.f);
  for (size_t l = 0; l < layers.size(); ++l)
    for (int r = 0; r < layers[l].R; ++r) m->host_bias[l * bstride + r] = layers[l].b[r];
  m->host_basis.assign(basis, basis + (size_t)in * F);
  for (const Layer& ly : layers) m->host_w.emplace_back(ly.W, ly.W + (size_t)ly.R * ly.C);
  NRT_HIP(hipMalloc(&m->blob, m->blob_bytes));
  NRT_HIP(hipMemcpy(m->blob, blob.bytes.data(), m->blob_bytes, hipMemcpyHostToDevice));
  char* base = static_cast<char*>(m->blob);
  md.basis = reinterpret_cast<const float*>(base + off_basis);
  for (size_t l = 0; l < layers.size(); ++l) {
    md.w16[l] = reinterpret_cast<const h8*>(base + off16[l]);
    md.w32[l] = reinterpret_cast<const float*>(base + off32[l]);
    md.wt32[l] = (l + 1 < layers.size()) ? reinterpret_cast<const float*>(base + offt[l]) : nullptr;
    md.bias[l] = reinterpret_cast<const float*>(base + offb[l]);
  }
  md.wout_row0 = reinterpret_cast<const float*>(base + off_w0);
  md.stream16 = reinterpret_cast<const h8*>(base + off_stream);
  md.stream16_bytes = (int)(stream.size() * sizeof(_Float16));
  md.chunk_off = reinterpret_cast<const int*>(base + off_coff);
  md.n_chunks = n_chunks;
  md.bias16 = reinterpret_cast<const float*>(base + off_b16);
  md.bias16_stride = bstride;
  md.fold = fold ? 1 : 0;
  md.streamk16 = reinterpret_cast<const h8*>(base + off_streamk);
  md.chunkk_off = reinterpret_cast<const int*>(base + off_coffk);
  md.nk_chunks = (int)chunkk_off.size();
  md.kc = kc;
  md.nk_frags = nk_frags;
  md.stream32 = reinterpret_cast<const float4*>(base + off_stream32);
  md.stream32_bytes = (int)(stream32.size() * sizeof(float));
  md.bias32 = reinterpret_cast<const float*>(base + off_b32);
  md.stream3 = reinterpret_cast<const float4*>(base + off_stream3);
  md.stream3_bytes = (int)(stream3.size() * sizeof(_Float16));
  md.bias3 = reinterpret_cast<const float*>(base + off_b3);
  for (size_t l = 0; l < layers.size(); ++l) md.scale3[l] = 1.f / lscale[l];
  md.ke3 = ke3;
  m->host_dev = md;
  NRT_HIP(hipMalloc(&m->dev, sizeof(MlpDev)));
  NRT_HIP(hipMemcpy(m->dev, &md, sizeof(MlpDev), hipMemcpyHostToDevice));
  *out = m.release();
  return NRT_OK;
}

nrt_mlp::~nrt_mlp() = default;  // nrt_prog is complete here

extern "C" int nrt_mlp_destroy(nrt_mlp* m) {
  if (!m) return NRT_OK;
  if (m->blob) (void)hipFree(m->blob);
  if (m->dev) (void)hipFree(m->dev);
  if (m->gather_map) (void)hipFree(m->gather_map);
  if (m->gather_src) (void)hipFree(m->gather_src);
  delete m;
  return NRT_OK;
}
