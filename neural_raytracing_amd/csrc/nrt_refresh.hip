// nrt_refresh.hip -- device-side re-pack of an MLP handle after an optimiser step (training,
// SURVEY §8f rank 1).  nrt_mlp_create packs on the host (a D2H copy of the weights, five fragment
// layouts, an H2D upload): ~8 ms per MLP per step, which a training loop pays for every MLP after
// every optimiser step.  nrt_mlp_refresh instead gathers the caller's device weights into the
// fragment arrays the training kernels read -- FP16 / FP32 A fragments, FP32 W^T fragments,
// padded biases, out.weight row 0 -- through a per-element index map built once on the host by
// the same loops as nrt_pack.hip.  The FP32 ring stream is refreshed too (the FP32 march of a
// training loop runs on it), and so is the fp32-split stream (folded, scaled and split into f16
// halves on the device, k_gather_split); the FP16 ring / program streams are not, and a refreshed
// handle refuses those paths (ring_supported, build_program).
#include <hip/hip_runtime.h>

#include <vector>

#include "nrt_launch.h"

namespace nrt {
namespace {

template <typename T>
__global__ void k_gather(T* __restrict__ dst, const int* __restrict__ map, int64_t n,
                         const float* __restrict__ src) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int k = map[i];
  dst[i] = (T)(k < 0 ? 0.f : src[k]);
}

// per-layer factors of the split stream (nrt_pack.hip): value = (x * fold[l]) * scale[l]
struct SplitCoef {
  float fold_w[kMaxLin], fold_b[kMaxLin], scale[kMaxLin];
};
// map entries of the split sections: source index | layer << 25 | part << 30 (-1 = padding)
constexpr int kSplitIdxBits = 25;

// split stream halves (part 0: hi = RNE_f16(v), part 1: lo = RNE_f16(v - hi)) or, BIAS, the
// scaled f32 biases -- the packer's arithmetic, on the device
template <bool BIAS>
__global__ void k_gather_split(void* __restrict__ dst, const int* __restrict__ map, int64_t n,
                               const float* __restrict__ src, SplitCoef c) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int v = map[i];
  if (v < 0) {
    if (BIAS) reinterpret_cast<float*>(dst)[i] = 0.f;
    else reinterpret_cast<_Float16*>(dst)[i] = (_Float16)0.f;
    return;
  }
  const int k = v & ((1 << kSplitIdxBits) - 1), l = (v >> kSplitIdxBits) & 31, part = (v >> 30) & 1;
  if (BIAS) {
    reinterpret_cast<float*>(dst)[i] = (src[k] * c.fold_b[l]) * c.scale[l];
    return;
  }
  const float w = (src[k] * c.fold_w[l]) * c.scale[l];
  const _Float16 hi = (_Float16)w;
  reinterpret_cast<_Float16*>(dst)[i] = part ? (_Float16)(w - (float)hi) : hi;
}

enum SecKind { SEC_F32 = 0, SEC_F16 = 1, SEC_SPLIT = 2, SEC_SPLIT_BIAS = 3 };
struct Section {
  void* dst;
  int64_t n;
  int kind;
};

// The fragment layouts of nrt_pack.hip, as source indices into [W_0 .. W_{L+1} | b_0 .. b_{L+1}]
// (row-major nn.Linear weights), -1 for padding.
void build_maps(const nrt_mlp* m, std::vector<int>& map, std::vector<Section>& secs,
                int64_t& n_src) {
  const nrt_mlp_desc& d = m->desc;
  const MlpDev& md = m->host_dev;
  const int in = d.in_size, H = d.hidden, L = d.num_layers, O = d.out, F = d.freqs;
  const int lat = d.latent, NB = H / 32;
  const int dp = in + 2 * F + lat, ke = md.ke;
  std::vector<int> slot_col(ke, -1);
  for (int s = 0; s < ke; ++s) {
    if (s < 2 * F) slot_col[s] = (s & 1) ? in + F + (s >> 1) : in + (s >> 1);
    else if (s < 2 * F + in) slot_col[s] = s - 2 * F;
    else if (s < 2 * F + in + lat) slot_col[s] = in + 2 * F + (s - 2 * F - in);
  }
  struct Ly { int R, C; bool hid, enc; int64_t woff, boff; };
  std::vector<Ly> ls;
  ls.push_back({H, dp, false, true, 0, 0});
  for (int i = 0; i < L; ++i) {
    const bool skip = (i != L - 1) && (i % d.skip == 0);
    ls.push_back({H, skip ? H + dp : H, true, skip, 0, 0});
  }
  ls.push_back({O, H, true, false, 0, 0});
  int64_t off = 0;
  for (Ly& l : ls) { l.woff = off; off += (int64_t)l.R * l.C; }
  for (Ly& l : ls) { l.boff = off; off += l.R; }
  n_src = off;
  auto idx = [](const Ly& l, int row, int col) -> int {
    if (row < 0 || row >= l.R || col < 0 || col >= l.C) return -1;
    return (int)(l.woff + (int64_t)row * l.C + col);
  };
  auto col_slot = [&](const Ly& l, int slot) {
    const int c = slot_col[slot];
    return c < 0 ? -1 : (l.hid ? H + c : c);
  };
  auto begin = [&](void* dst, int kind) { secs.push_back({dst, (int64_t)map.size(), kind}); };
  auto end = [&]() { secs.back().n = (int64_t)map.size() - secs.back().n; };
  for (size_t li = 0; li < ls.size(); ++li) {
    const Ly& l = ls[li];
    const int nrb = (l.R + 31) / 32;
    {  // FP16 A fragments
      const int ks_h = l.hid ? 2 * NB : 0, ks_e = l.enc ? ke / 16 : 0;
      begin((void*)md.w16[li], SEC_F16);
      for (int s = 0; s < ks_h + ks_e; ++s)
        for (int ib = 0; ib < nrb; ++ib)
          for (int lane = 0; lane < 64; ++lane) {
            const int i = lane & 31, hf = lane >> 5;
            for (int j = 0; j < 8; ++j) {
              const int col = s < ks_h ? 32 * (s >> 1) + 16 * (s & 1) + 8 * (j >> 2) + 4 * hf + (j & 3)
                                       : col_slot(l, 16 * (s - ks_h) + 8 * hf + j);
              map.push_back(idx(l, 32 * ib + i, col));
            }
          }
      end();
    }
    {  // FP32 A fragments
      const int ks_h = l.hid ? H / 2 : 0, ks_e = l.enc ? ke / 2 : 0;
      begin((void*)md.w32[li], SEC_F32);
      for (int s = 0; s < ks_h + ks_e; ++s)
        for (int ib = 0; ib < nrb; ++ib)
          for (int lane = 0; lane < 64; ++lane) {
            const int i = lane & 31, hf = lane >> 5;
            const int col = s < ks_h ? 2 * s + hf : col_slot(l, 2 * (s - ks_h) + hf);
            map.push_back(idx(l, 32 * ib + i, col));
          }
      end();
    }
    if (li + 1 < ls.size()) {  // FP32 W^T fragments
      const int npos = (l.hid ? H : 0) + (l.enc ? ke : 0);
      const int nrbt = (npos + 31) / 32;
      begin((void*)md.wt32[li], SEC_F32);
      for (int s = 0; s < H / 2; ++s)
        for (int ib = 0; ib < nrbt; ++ib)
          for (int lane = 0; lane < 64; ++lane) {
            const int i = lane & 31, hf = lane >> 5;
            const int pos = 32 * ib + i;
            int col = -1;
            if (pos < npos) col = (l.hid && pos < H) ? pos : col_slot(l, pos - (l.hid ? H : 0));
            map.push_back(idx(l, 2 * s + hf, col));
          }
      end();
    }
    begin((void*)md.bias[li], SEC_F32);  // biases padded to row blocks
    for (int r = 0; r < nrb * 32; ++r) map.push_back(r < l.R ? (int)(l.boff + r) : -1);
    end();
  }
  begin((void*)md.wout_row0, SEC_F32);  // out.weight[0, :]
  for (int k = 0; k < H; ++k) map.push_back(idx(ls.back(), 0, k));
  end();
  {  // FP32 ring stream (same walk as the packer)
    std::vector<Ring32Layer> rl;
    for (const Ly& l : ls) rl.push_back({l.R, l.hid, l.enc});
    begin((void*)md.stream32, SEC_F32);
    ring32_walk(rl, H, ke, [&](int li, int row, int pos) {
      const Ly& l = ls[li];
      map.push_back(idx(l, row, pos < H ? pos : col_slot(l, pos - H)));
    });
    end();
  }
  begin((void*)md.bias32, SEC_F32);  // [layer][bias16_stride]
  for (size_t li = 0; li < ls.size(); ++li)
    for (int r = 0; r < md.bias16_stride; ++r)
      map.push_back(r < ls[li].R ? (int)(ls[li].boff + r) : -1);
  end();
  // the split stream and its scaled biases (the fp32-split march of a training loop): the
  // packer's walk, each entry tagged with its layer and half; the pack-time scales stay (they
  // only keep the lo halves normal, and hi covers |W 2^s| up to 65504)
  if (n_src < (1 << kSplitIdxBits)) {
    std::vector<Ring32Layer> rl;
    for (const Ly& l : ls) rl.push_back({l.R, l.hid, l.enc});
    begin((void*)md.stream3, SEC_SPLIT);
    ring3_walk(rl, H, md.ke3, [&](int li, int row, int pos, int part) {
      const Ly& l = ls[li];
      int col = -1;
      if (pos < H) col = pos;
      else if (pos - H < ke) col = col_slot(l, pos - H);
      const int k = idx(l, row, col);
      map.push_back(k < 0 ? -1 : (k | (li << kSplitIdxBits) | (part << 30)));
    });
    end();
    begin((void*)md.bias3, SEC_SPLIT_BIAS);
    for (size_t li = 0; li < ls.size(); ++li)
      for (int r = 0; r < md.bias16_stride; ++r)
        map.push_back(r < ls[li].R ? (int)((ls[li].boff + r) | ((int64_t)li << kSplitIdxBits)) : -1);
    end();
  }
}

}  // namespace
}  // namespace nrt

using namespace nrt;

extern "C" int nrt_mlp_refresh(nrt_mlp* m, const float* const* weights, const float* const* biases,
                               void* stream) {
  if (!m || !weights || !biases) { set_error("nrt_mlp_refresh: null argument"); return NRT_EINVAL; }
  hipStream_t st = (hipStream_t)stream;
  if (!m->gather_map) {
    std::vector<int> map;
    std::vector<Section> secs;
    build_maps(m, map, secs, m->n_src);
    if (map.size() > (size_t)INT32_MAX) { set_error("nrt_mlp_refresh: MLP too large"); return NRT_EINVAL; }
    NRT_HIP(hipMalloc(&m->gather_map, map.size() * sizeof(int)));
    NRT_HIP(hipMemcpy(m->gather_map, map.data(), map.size() * sizeof(int), hipMemcpyHostToDevice));
    NRT_HIP(hipMalloc(&m->gather_src, (size_t)m->n_src * sizeof(float)));
    for (const Section& q : secs) {
      m->gather_dst.push_back(q.dst);
      m->gather_n.push_back(q.n);
      m->gather_f16.push_back((char)q.kind);
    }
  }
  // stage [W_0 .. W_{L+1} | b_0 .. b_{L+1}] from the caller's device tensors
  const int n_lin = m->desc.num_layers + 2;
  size_t off = 0;
  for (int l = 0; l < n_lin; ++l) {
    const size_t n = m->host_w[l].size();
    if (!weights[l]) { set_error("nrt_mlp_refresh: null weight"); return NRT_EINVAL; }
    NRT_HIP(hipMemcpyAsync(m->gather_src + off, weights[l], n * 4, hipMemcpyDeviceToDevice, st));
    off += n;
  }
  for (int l = 0; l < n_lin; ++l) {
    const size_t n = (size_t)(l == n_lin - 1 ? m->desc.out : m->desc.hidden);
    if (!biases[l]) { set_error("nrt_mlp_refresh: null bias"); return NRT_EINVAL; }
    NRT_HIP(hipMemcpyAsync(m->gather_src + off, biases[l], n * 4, hipMemcpyDeviceToDevice, st));
    off += n;
  }
  if ((int64_t)off != m->n_src) { set_error("nrt_mlp_refresh: layer sizes changed"); return NRT_EINVAL; }
  const MlpDev& md = m->host_dev;
  const bool fold = m->desc.activation == NRT_ACT_SOFTPLUS;
  const float kLog2e = 1.4426950408889634f, kLn2 = 0.6931471805599453f;
  SplitCoef coef{};
  for (int l = 0; l < n_lin && l < kMaxLin; ++l) {
    coef.fold_w[l] = fold ? (l == 0 ? kLog2e : (l == n_lin - 1 ? kLn2 : 1.f)) : 1.f;
    coef.fold_b[l] = fold && l < n_lin - 1 ? kLog2e : 1.f;
    coef.scale[l] = 1.f / md.scale3[l];  // a power of two: exact
  }
  int64_t moff = 0;
  for (size_t q = 0; q < m->gather_dst.size(); ++q) {
    const int64_t n = m->gather_n[q];
    const dim3 grid((unsigned)((n + 255) / 256)), block(256);
    if (n > 0) {
      const int kind = m->gather_f16[q];
      const int* mp = m->gather_map + moff;
      if (kind == SEC_F16)
        k_gather<_Float16><<<grid, block, 0, st>>>((_Float16*)m->gather_dst[q], mp, n, m->gather_src);
      else if (kind == SEC_F32)
        k_gather<float><<<grid, block, 0, st>>>((float*)m->gather_dst[q], mp, n, m->gather_src);
      else if (kind == SEC_SPLIT)
        k_gather_split<false><<<grid, block, 0, st>>>(m->gather_dst[q], mp, n, m->gather_src, coef);
      else
        k_gather_split<true><<<grid, block, 0, st>>>(m->gather_dst[q], mp, n, m->gather_src, coef);
    }
    moff += n;
  }
  if (int rc = check_launch("k_gather")) return rc;
  m->refreshed = true;
  m->split_refreshed = m->n_src < (1 << kSplitIdxBits);
  return NRT_OK;
}
