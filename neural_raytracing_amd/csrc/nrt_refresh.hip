// nrt_refresh.hip -- device-side re-pack of an MLP handle after an optimiser step (training,
// SURVEY §8f rank 1).  nrt_mlp_create packs on the host (a D2H copy of the weights, five fragment
// layouts, an H2D upload): ~8 ms per MLP per step, which a training loop pays for every MLP after
// every optimiser step.  nrt_mlp_refresh instead gathers the caller's device weights into the
// fragment arrays the training kernels read -- FP16 / FP32 A fragments, FP32 W^T fragments,
// padded biases, out.weight row 0 -- through a per-element index map built once on the host by
// the same loops as nrt_pack.hip.  The FP32 ring stream is refreshed too (the FP32 march of a
// training loop runs on it), and so are the fp32-split stream (folded, scaled and split into f16
// halves on the device, k_refresh_all) and the FP16 ring stream (folded, rounded to f16: the FP16
// / mixed march of a training loop); the FP16 program streams of the shading kernels are not, and
// a refreshed handle refuses those paths (build_program).
#include <hip/hip_runtime.h>

#include <vector>

#include "nrt_launch.h"

namespace nrt {
namespace {

// per-layer factors of the split stream (nrt_pack.hip): value = (x * fold[l]) * scale[l]
struct SplitCoef {
  float fold_w[kMaxLin], fold_b[kMaxLin], scale[kMaxLin];
};
// map entries of the split sections: source index | layer << 25 | part << 30 (-1 = padding)
constexpr int kSplitIdxBits = 25;

enum SecKind { SEC_F32 = 0, SEC_F16 = 1, SEC_SPLIT = 2, SEC_SPLIT_BIAS = 3, SEC_R16 = 4,
               SEC_R16_BIAS = 5 };

// Split sections: part 0 hi = RNE_f16(v), part 1 lo = RNE_f16(v - hi), or the scaled f32 biases
// -- the packer's arithmetic, on the device.
// One launch for the staging copy of every weight / bias tensor and one for every section's
// gather (round 2 issued a hipMemcpyAsync per tensor and a k_gather per section: ~60 launches per
// MLP, ~600 per training step).  Tables ride in the kernel arguments.
constexpr int kMaxStage = 2 * kMaxLin;
struct StageTable {
  const float* src[kMaxStage];
  int64_t off[kMaxStage + 1];  // prefix offsets into gather_src
  int n;
};
constexpr int kMaxSections = 96;  // 4 per layer + the streams (the 16-layer spatial MLP: 78)
struct SectionTable {
  void* dst[kMaxSections];
  int64_t off[kMaxSections + 1];  // prefix offsets into the concatenated map
  int kind[kMaxSections];
  int n;
};

__global__ void k_stage(StageTable t, float* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= t.off[t.n]) return;
  int lo = 0, hi = t.n - 1;  // the last tensor whose offset is <= i (binary search)
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (t.off[mid] <= i) lo = mid; else hi = mid - 1;
  }
  const int q = lo;
  dst[i] = t.src[q][i - t.off[q]];
}

__global__ void k_refresh_all(SectionTable t, const int* __restrict__ map,
                              const float* __restrict__ src, SplitCoef c) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= t.off[t.n]) return;
  int lo = 0, hi = t.n - 1;  // the last section whose offset is <= i (empty sections: skipped)
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (t.off[mid] <= i) lo = mid; else hi = mid - 1;
  }
  const int q = lo;
  const int64_t j = i - t.off[q];
  const int v = map[i];
  switch (t.kind[q]) {
    case SEC_F32: reinterpret_cast<float*>(t.dst[q])[j] = v < 0 ? 0.f : src[v]; break;
    case SEC_F16: reinterpret_cast<_Float16*>(t.dst[q])[j] = (_Float16)(v < 0 ? 0.f : src[v]); break;
    // the FP16 ring stream: (_Float16)(fold_w[l] * W) and fold_b[l] * b, as nrt_pack.hip
    case SEC_R16: {
      const int k = v & ((1 << kSplitIdxBits) - 1), l = (v >> kSplitIdxBits) & 31;
      reinterpret_cast<_Float16*>(t.dst[q])[j] = (_Float16)(v < 0 ? 0.f : src[k] * c.fold_w[l]);
      break;
    }
    case SEC_R16_BIAS: {
      const int k = v & ((1 << kSplitIdxBits) - 1), l = (v >> kSplitIdxBits) & 31;
      reinterpret_cast<float*>(t.dst[q])[j] = v < 0 ? 0.f : src[k] * c.fold_b[l];
      break;
    }
    default: {
      const bool bias = t.kind[q] == SEC_SPLIT_BIAS;
      if (v < 0) {
        if (bias) reinterpret_cast<float*>(t.dst[q])[j] = 0.f;
        else reinterpret_cast<_Float16*>(t.dst[q])[j] = (_Float16)0.f;
        break;
      }
      const int k = v & ((1 << kSplitIdxBits) - 1), l = (v >> kSplitIdxBits) & 31, part = (v >> 30) & 1;
      if (bias) {
        reinterpret_cast<float*>(t.dst[q])[j] = (src[k] * c.fold_b[l]) * c.scale[l];
      } else {
        const float w = (src[k] * c.fold_w[l]) * c.scale[l];
        const _Float16 hi = (_Float16)w;
        reinterpret_cast<_Float16*>(t.dst[q])[j] = part ? (_Float16)(w - (float)hi) : hi;
      }
    }
  }
}
struct Section {
  void* dst;
  int64_t n;
  int kind;
};

// The fragment layouts of nrt_pack.hip, as source indices into [W_0 .. W_{L+1} | b_0 .. b_{L+1}]
// (row-major nn.Linear weights), -1 for padding.
void build_maps(const nrt_mlp* m, std::vector<int>& map, std::vector<Section>& secs,
                int64_t& n_src, bool& solo, bool& bwd) {
  solo = false;
  bwd = false;
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
  // the FP16 ring stream and its biases (the FP16 / mixed march of a training loop): the packer's
  // chunk walk, each entry tagged with its layer for the softplus fold
  if (n_src < (1 << kSplitIdxBits)) {
    begin((void*)md.stream16, SEC_R16);
    for (size_t li = 0; li < ls.size(); ++li) {
      const Ly& l = ls[li];
      const bool is_init = li == 0, is_out = li + 1 == ls.size();
      const int nrb = (l.R + 31) / 32;
      const int ks_h = l.hid ? 2 * NB : 0, ks_e = l.enc ? ke / 16 : 0;
      auto frag = [&](int s2, int ib) {
        for (int lane = 0; lane < 64; ++lane) {
          const int i = lane & 31, hf = lane >> 5;
          for (int j = 0; j < 8; ++j) {
            const int col = s2 < ks_h ? 32 * (s2 >> 1) + 16 * (s2 & 1) + 8 * (j >> 2) + 4 * hf + (j & 3)
                                      : col_slot(l, 16 * (s2 - ks_h) + 8 * hf + j);
            const int k = idx(l, 32 * ib + i, col);
            map.push_back(k < 0 ? -1 : (k | ((int)li << kSplitIdxBits)));
          }
        }
      };
      if (is_init || is_out || NB % kRingRB != 0) {
        for (int ib = 0; ib < nrb; ++ib)
          for (int s2 = 0; s2 < ks_h + ks_e; ++s2) frag(s2, ib);
      } else {
        for (int c = 0; c < nrb / kRingRB; ++c)
          for (int s2 = 0; s2 < ks_h + ks_e; ++s2)
            for (int b = 0; b < kRingRB; ++b) frag(s2, kRingRB * c + b);
      }
    }
    end();
    begin((void*)md.bias16, SEC_R16_BIAS);
    for (size_t li = 0; li < ls.size(); ++li)
      for (int r = 0; r < md.bias16_stride; ++r)
        map.push_back(r < ls[li].R ? (int)((ls[li].boff + r) | ((int64_t)li << kSplitIdxBits)) : -1);
    end();
  }
  // the single-MLP FP32 row program of nrt_mlp_forward on the ring engine (nrt_shade_ring.hip)
  {
    std::vector<int> smap, bmap;
    void *sdst = nullptr, *bdst = nullptr;
    if (solo_refresh_maps(m, smap, bmap, sdst, bdst)) {
      begin(sdst, SEC_F32);
      map.insert(map.end(), smap.begin(), smap.end());
      end();
      begin(bdst, SEC_F32);
      map.insert(map.end(), bmap.begin(), bmap.end());
      end();
      solo = true;
    }
  }
  // the ring backward's program (nrt_train_ring.h): the forward part and the transposed layers
  {
    std::vector<int> smap, bmap;
    void *sdst = nullptr, *bdst = nullptr;
    if (bwd_refresh_maps(m, smap, bmap, sdst, bdst)) {
      begin(sdst, SEC_F32);
      map.insert(map.end(), smap.begin(), smap.end());
      end();
      begin(bdst, SEC_F32);
      map.insert(map.end(), bmap.begin(), bmap.end());
      end();
      bwd = true;
    }
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
    bool solo = false, bwd = false;
    build_maps(m, map, secs, m->n_src, solo, bwd);
    m->solo_in_refresh = solo;
    m->bwd_in_refresh = bwd;
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
  // stage [W_0 .. W_{L+1} | b_0 .. b_{L+1}] from the caller's device tensors (one launch)
  const int n_lin = m->desc.num_layers + 2;
  if (2 * n_lin > kMaxStage || m->gather_dst.size() > (size_t)kMaxSections) {
    set_error("nrt_mlp_refresh: too many layers");
    return NRT_EINVAL;
  }
  StageTable stg{};
  int64_t off = 0;
  for (int l = 0; l < 2 * n_lin; ++l) {
    const bool w = l < n_lin;
    const int ll = w ? l : l - n_lin;
    const float* p = w ? weights[ll] : biases[ll];
    if (!p) { set_error(w ? "nrt_mlp_refresh: null weight" : "nrt_mlp_refresh: null bias"); return NRT_EINVAL; }
    stg.src[l] = p;
    stg.off[l] = off;
    off += w ? (int64_t)m->host_w[ll].size() : (int64_t)(ll == n_lin - 1 ? m->desc.out : m->desc.hidden);
  }
  stg.off[2 * n_lin] = off;
  stg.n = 2 * n_lin;
  if (off != m->n_src) { set_error("nrt_mlp_refresh: layer sizes changed"); return NRT_EINVAL; }
  k_stage<<<dim3((unsigned)((off + 255) / 256)), dim3(256), 0, st>>>(stg, m->gather_src);
  if (int rc = check_launch("k_stage")) return rc;
  const MlpDev& md = m->host_dev;
  const bool fold = m->desc.activation == NRT_ACT_SOFTPLUS;
  const float kLog2e = 1.4426950408889634f, kLn2 = 0.6931471805599453f;
  SplitCoef coef{};
  for (int l = 0; l < n_lin && l < kMaxLin; ++l) {
    coef.fold_w[l] = fold ? (l == 0 ? kLog2e : (l == n_lin - 1 ? kLn2 : 1.f)) : 1.f;
    coef.fold_b[l] = fold && l < n_lin - 1 ? kLog2e : 1.f;
    coef.scale[l] = 1.f / md.scale3[l];  // a power of two: exact
  }
  // every section's gather (one launch)
  SectionTable sec{};
  int64_t moff = 0;
  for (size_t q = 0; q < m->gather_dst.size(); ++q) {
    sec.dst[q] = m->gather_dst[q];
    sec.kind[q] = m->gather_f16[q];
    sec.off[q] = moff;
    moff += m->gather_n[q];
  }
  sec.n = (int)m->gather_dst.size();
  sec.off[sec.n] = moff;
  if (moff > 0) {
    k_refresh_all<<<dim3((unsigned)((moff + 255) / 256)), dim3(256), 0, st>>>(sec, m->gather_map,
                                                                             m->gather_src, coef);
    if (int rc = check_launch("k_refresh_all")) return rc;
  }
  m->refreshed = true;
  m->split_refreshed = m->n_src < (1 << kSplitIdxBits);
  m->ring16_refreshed = m->split_refreshed;  // the same condition gates both tagged walks
  return NRT_OK;
}
