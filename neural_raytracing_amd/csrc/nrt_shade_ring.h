// nrt_shade_ring.h -- the shading MLPs (LightField, the spatial-weight MLP, NeuralBSDFs) at the
// reference's precision on the LDS-ring engines: FP32 on v_mfma_f32_16x16x4_f32 (exact f32, the
// ring32 tile) and "fp32-split" on v_mfma_f32_16x16x32_f16 with f16 hi/lo operand halves (the
// ring3 tile, nrt_ring3.h).  Reference: SkipConnMLP.forward (neural_blocks.py:75-86) inside
// Direct.sample's emitter / BSDF evaluation (integrators.py:173-189, lights.py:175-195,
// bsdfs.py:515-536, 613-637).
//
// A wave owns 16 hit rays (lane g = lane >> 4, j = lane & 15 serves ray j); a layer's 16x16
// accumulators are the next layer's B operand, so activations stay in registers (as ring32 /
// ring3).  What differs from the SDF engines:
//  * several MLPs per kernel ("row program"): their weight streams are concatenated and a chunk
//    table (KiB offset, KiB count per chunk, in evaluation order) drives the LDS-DMA, so the ring
//    prefetches across MLP boundaries and the evaluation code never names the next chunk;
//  * wide encodings (F = 128: 259 inputs) never sit in registers: the encoding part of a layer
//    (the init layer and every skip layer) is k-outer -- one k-step group of the encoding against
//    every output sub-block of the layer, each encoding value computed once per layer -- and the
//    hidden part stays row-outer (32 output rows per chunk, the previous chunk's activations
//    spread over the chunk's MFMAs; on skip layers it runs first and keeps its raw accumulators,
//    which the encoding part then completes);
//  * every output row (<= 16, one sub-block) is returned: row 4 g + r of ray j sits in register r
//    of lane 16 g + j.
// Stream layout per MLP and precision: nrt_shade_ring.hip (shade_walk).
#pragma once
#include "nrt_kernels.h"

namespace nrt {
namespace rprog {

typedef float f4v __attribute__((ext_vector_type(4)));
using ring3::u4v;

constexpr int kSlotKiB = 32;  // largest chunk of every supported shape (H = 256: 2 x 16 sub-blocks)

// Per-shape constants.  FP32 tile: k-step = 4 inputs (lane group g holds input g), quads of 4
// k-steps per 1-KiB piece.  Split tile: k-step = 32 inputs (lane group g holds 8 g .. 8 g + 7),
// one piece per (sub-block, half).
template <int H_, int KE_, int KQ_>
struct Shape {
  static constexpr int H = H_;
  static constexpr int NSB = H / 16;  // 16-row sub-blocks of a hidden layer
  static constexpr int NC = H / 32;   // row chunks of a hidden layer
  // FP32
  static constexpr int KE = KE_;      // encoding k-steps (ke / 4, ke = slots padded to 16)
  static constexpr int QE = KE / 4;   // encoding quads
  static constexpr int QH = H / 16;   // hidden quads
  static constexpr int EQ = NSB >= 16 ? 2 : 32 / NSB;  // encoding quads per chunk
  static constexpr int CE32 = (QE + EQ - 1) / EQ;
  // split
  static constexpr int KQ = KQ_;      // encoding k-steps (ke3 / 32)
  static constexpr int KH = H / 32;   // hidden k-steps
  static constexpr int EK = NSB >= 16 ? 1 : 16 / NSB;  // encoding k-steps per chunk
  static constexpr int CE3 = (KQ + EK - 1) / EK;
};
// LightField 10 x 256 F = 16, ComposeSpatialVarying 16 x 256 F = 128, NeuralBSDF 6 x 96 F = 64
using LightShape = Shape<256, 12, 2>;
using SpatialShape = Shape<256, 68, 9>;
using BsdfShape = Shape<96, 36, 5>;

template <int D, int WV>
struct Engine {
  static constexpr int SLOTQ = kSlotKiB;
  static constexpr int MAXL = (SLOTQ + WV - 1) / WV;  // DMA pieces per wave per chunk
  static constexpr int RING_BYTES = D * SLOTQ * 1024;
  static constexpr int kOutOfRange = 0x40000000;
  __host__ __device__ static size_t lds_bytes(const RProgDev& p) {
    return RING_BYTES + (size_t)p.basis_q * 16 + (size_t)p.table_floats * 4 +
           (size_t)p.n_mlp * kMaxLin * 4;
  }
  const float4* ring;
  uint32_t ring_lds;
  const float* ltab;      // LDS: biases | split scales
  const float4* lbasis;   // LDS: (B0q, B1q, B2q, 0) per frequency, all MLPs
  const void* sbase;
  int sbytes;
  const NRT_CONST int* chunks;  // [2 n]: (KiB offset, KiB count)
  int nch, ahead, slot, lane, wv;
  // fp32-split range guard (nrt_ring3.h), per block: lexp[mlp][l] = e_l of that MLP's linear
  // layer l (LDS, zero at start); `guarded` (block-uniform) selects eval3<..., GUARD>;
  // `changed` = this wave's last guarded evaluation raised an exponent
  int* lexp;
  bool guarded, changed;

  __device__ __forceinline__ void issue(int qoff, int nq, int s) {
    const int w = __builtin_amdgcn_readfirstlane(wv);
    const uint64_t sp = (uint64_t)(uintptr_t)sbase;
    const uint64_t spu = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(sp >> 32)) << 32) |
                         (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)sp);
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(uintptr_t)spu, 0, __builtin_amdgcn_readfirstlane(sbytes), 0x00020000);
    const int q0 = __builtin_amdgcn_readfirstlane(qoff) + w;
    const uint32_t dst0 = __builtin_amdgcn_readfirstlane(ring_lds + (uint32_t)(s * SLOTQ * 1024)) +
                          (uint32_t)w * 1024u;
    const int n = __builtin_amdgcn_readfirstlane(nq);
#pragma unroll
    for (int q = 0; q < MAXL; ++q) {
      const bool own = w + WV * q < n;  // fixed count per wave: pieces past the chunk load nothing
      ring::lds_dma16(r, own ? lane * 16 : kOutOfRange + lane * 16, (q0 + WV * q) * 1024,
                      dst0 + (uint32_t)(WV * q * 1024));
    }
  }
  // the chunk `ahead` of the table into ring slot s (the table wraps: after the last chunk of a
  // tile's evaluations comes the next tile's first)
  __device__ __forceinline__ void issue_next(int s) {
    issue(chunks[2 * ahead], chunks[2 * ahead + 1], s);
    ahead = ahead + 1 == nch ? 0 : ahead + 1;
  }
  // block-wide; afterwards chunks 0 .. D - 2 are in flight.  chunk0: the program starts at that
  // chunk of its table (the ring backward on saved activations skips the forward part)
  __device__ __forceinline__ void init(const RProgDev& p, char* lds, int chunk0 = 0) {
    ring = reinterpret_cast<const float4*>(lds);
    ring_lds = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)lds;
    float4* lq = reinterpret_cast<float4*>(lds + RING_BYTES);
    for (int q = threadIdx.x; q < p.basis_q; q += blockDim.x) lq[q] = p.basis[q];
    lbasis = lq;
    float* lt = reinterpret_cast<float*>(lds + RING_BYTES + (size_t)p.basis_q * 16);
    for (int i = threadIdx.x; i < p.table_floats; i += blockDim.x) lt[i] = p.tables[i];
    ltab = lt;
    lexp = reinterpret_cast<int*>(lt + p.table_floats);
    for (int i = threadIdx.x; i < p.n_mlp * kMaxLin; i += blockDim.x) lexp[i] = 0;
    guarded = false;
    changed = false;
    sbase = p.stream;
    sbytes = p.stream_bytes;
    chunks = (const NRT_CONST int*)p.chunks + 2 * chunk0;
    nch = p.n_chunks - chunk0;
    lane = threadIdx.x & 63;
    wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    slot = 0;
    ahead = 0;
#pragma unroll
    for (int d = 0; d < D - 1; ++d) issue_next(d);
    __syncthreads();
  }
  // start of the current chunk: wait for this wave's pieces of it (with 3 slots the next chunk's
  // MAXL pieces may stay in flight), the barrier makes every wave's pieces visible and retires
  // everyone's reads of the previous chunk, whose slot then receives chunk c + D - 1
  __device__ __forceinline__ const float4* begin() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(ring::waitcnt_vm_lgkm0(D == 3 ? MAXL : 0));
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    issue_next(slot == 0 ? D - 1 : slot - 1);
    __builtin_amdgcn_sched_barrier(0);
    return ring + slot * SLOTQ * 64 + lane;
  }
  __device__ __forceinline__ void end() { slot = slot + 1 == D ? 0 : slot + 1; }
  // the DMA issued by the last begin() must land before the block's LDS is released
  __device__ __forceinline__ void drain() { __builtin_amdgcn_s_waitcnt(ring::waitcnt_vm_lgkm0(0)); }
  // After a tile's split evaluations (ok = this lane's outputs are finite): true if the whole
  // block runs them again -- the first non-finite output switches the block to the guarded
  // variant, a guarded pass repeats while some wave raised an exponent.  Block-uniform (one
  // barrier per tile).
  __device__ __forceinline__ bool retry(bool ok) {
    int want;
    if (!guarded) {
      want = wave_any(!ok) ? 1 : 0;
    } else {
      want = changed ? 1 : 0;
      changed = false;
    }
    if (!__syncthreads_or(want)) return false;
    guarded = true;
    return true;
  }
  // acc[reg] = bias[layer][16 sb + 4 g + reg] of MLP m
  __device__ __forceinline__ f4v bias_at(const RProgMlp& m, int layer, int sb) const {
    const float4 q = *reinterpret_cast<const float4*>(ltab + m.bias_off + layer * m.bstride + 16 * sb +
                                                      4 * (lane >> 4));
    return f4v{q.x, q.y, q.z, q.w};
  }
};

// encoding slot value (utils.py:37-40 in the slot order of nrt_device.h: slot 2q / 2q + 1 = sin /
// cos of projection q, then x0, x1, x2, zeros); the projection in the FP32 path's fma order
__device__ __forceinline__ void enc_pair(const float4* basis, int F, int q, float x0, float x1,
                                         float x2, float& sn, float& cs) {
  if (q < F) {
    const float4 b = basis[q];
    float pr = x0 * b.x;
    pr = fmaf(x1, b.y, pr);
    pr = fmaf(x2, b.z, pr);
    sincosf(pr, &sn, &cs);
  } else {
    const int s = 2 * (q - F);  // slots 2F + s, 2F + s + 1
    sn = s == 0 ? x0 : s == 2 ? x2 : 0.f;
    cs = s == 0 ? x1 : 0.f;
  }
}
__device__ __forceinline__ float enc_slot(const float4* basis, int F, int slot, float x0, float x1,
                                          float x2) {
  if (slot < 2 * F) {
    const float4 b = basis[slot >> 1];
    float pr = x0 * b.x;
    pr = fmaf(x1, b.y, pr);
    pr = fmaf(x2, b.z, pr);
    float sn, cs;
    sincosf(pr, &sn, &cs);
    return (slot & 1) ? cs : sn;
  }
  return slot == 2 * F ? x0 : slot == 2 * F + 1 ? x1 : slot == 2 * F + 2 ? x2 : 0.f;
}

// ---------------------------------------------------------------------------------------------
// FP32 (exact f32 MFMA)
// ---------------------------------------------------------------------------------------------
// k-outer encoding part of one layer: acc[sb] += W_enc[sub-block sb] . act?(enc), pieces
// [quad][sub-block] (hidden layers: act(enc), neural_blocks.py:82-84; init: the raw encoding)
template <class S, int ACT, class En>
__device__ __forceinline__ void enc_part32(En& E, const RProgMlp& m, const float4* basis, bool actv,
                                           float x0, float x1, float x2, f4v (&acc)[S::NSB]) {
  const int g = E.lane >> 4;
#pragma unroll 1
  for (int cc = 0; cc < S::CE32; ++cc) {
    const float4* A = E.begin();
#pragma unroll
    for (int uu = 0; uu < S::EQ; ++uu) {
      const int u = cc * S::EQ + uu;
      if (u < S::QE) {
        float v[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const float e = enc_slot(basis, m.F, 4 * (4 * u + t) + g, x0, x1, x2);
          v[t] = actv ? ring32::act<ACT>(e) : e;
        }
#pragma unroll
        for (int sb = 0; sb < S::NSB; sb += 2) {
          const float4 w0 = A[(uu * S::NSB + sb) * 64], w1 = A[(uu * S::NSB + sb + 1) * 64];
          acc[sb] = ring32::mfma4(w0.x, v[0], acc[sb]); acc[sb + 1] = ring32::mfma4(w1.x, v[0], acc[sb + 1]);
          acc[sb] = ring32::mfma4(w0.y, v[1], acc[sb]); acc[sb + 1] = ring32::mfma4(w1.y, v[1], acc[sb + 1]);
          acc[sb] = ring32::mfma4(w0.z, v[2], acc[sb]); acc[sb + 1] = ring32::mfma4(w1.z, v[2], acc[sb + 1]);
          acc[sb] = ring32::mfma4(w0.w, v[3], acc[sb]); acc[sb + 1] = ring32::mfma4(w1.w, v[3], acc[sb + 1]);
        }
      }
    }
    E.end();
  }
}

// out layer (neural_blocks.py:86) on the last hidden activations dst (k-step order): one
// sub-block, two chains over even / odd quads
template <class S, class En>
__device__ __forceinline__ f4v out32(En& E, const RProgMlp& m, const float (&dst)[S::H / 4]) {
  constexpr int QH = S::QH;
  const float4* A = E.begin();
  f4v o0 = E.bias_at(m, m.L + 1, 0), o1 = f4v{0.f, 0.f, 0.f, 0.f};
  {
    float4 w0 = A[0], w1 = A[64];
#pragma unroll
    for (int u = 0; u < QH; u += 2) {
      float4 n0 = w0, n1 = w1;
      if (u + 2 < QH) { n0 = A[(u + 2) * 64]; n1 = A[(u + 3) * 64]; }
      o0 = ring32::mfma4(w0.x, dst[4 * u], o0); o1 = ring32::mfma4(w1.x, dst[4 * u + 4], o1);
      o0 = ring32::mfma4(w0.y, dst[4 * u + 1], o0); o1 = ring32::mfma4(w1.y, dst[4 * u + 5], o1);
      o0 = ring32::mfma4(w0.z, dst[4 * u + 2], o0); o1 = ring32::mfma4(w1.z, dst[4 * u + 6], o1);
      o0 = ring32::mfma4(w0.w, dst[4 * u + 3], o0); o1 = ring32::mfma4(w1.w, dst[4 * u + 7], o1);
      w0 = n0; w1 = n1;
    }
  }
  E.end();
  return o0 + o1;
}

// One SkipConnMLP evaluation for the wave's 16 rays; returns the out layer's 16x16 accumulator
// (row 4 g + r of ray j in register r of lane 16 g + j).  Every wave of the block runs it.
// Skip layers run their hidden part first (row-outer, raw accumulators kept), then the encoding
// part (k-outer) adds into them, then the activation: b + W_h h + W_e act(enc).
template <class S, int ACT, class En>
__device__ __forceinline__ f4v eval32(En& E, const RProgMlp& m, float x0, float x1, float x2) {
  constexpr int NSB = S::NSB, NC = S::NC, QH = S::QH, KH = S::H / 4;
  const float4* basis = E.lbasis + m.basis_off;
  const int L = m.L, SK = m.skip;
  float src[KH], dst[KH];
  f4v acc[NSB];
  auto act_all = [&]() {
#pragma unroll
    for (int sb = 0; sb < NSB; ++sb)
#pragma unroll
      for (int r = 0; r < 4; ++r) dst[4 * sb + r] = ring32::act<ACT>(acc[sb][r]);
  };
  // init layer (neural_blocks.py:80): the raw encoding, k-outer
#pragma unroll
  for (int sb = 0; sb < NSB; ++sb) acc[sb] = E.bias_at(m, 0, sb);
  enc_part32<S, ACT>(E, m, basis, false, x0, x1, x2, acc);
  act_all();
  f4v pend0, pend1;
  auto retire1 = [&](int ib, int k) {  // element k (< 8) of chunk ib
    float& d = dst[8 * ib + k];
    d = ring32::act<ACT>(k < 4 ? pend0[k & 3] : pend1[k & 3]);
    asm volatile("" : "+v"(d));
  };
  // hidden part of layer i; RAW keeps each chunk's accumulators for the encoding part, otherwise
  // the previous chunk's 8 activations are spread over the chunk's QH quads
  auto hidden = [&](int i, auto raw_c) {
    constexpr bool RAW = decltype(raw_c)::value;
#pragma unroll
    for (int ib = 0; ib < NC; ++ib) {
      const float4* A = E.begin();
      f4v a0 = E.bias_at(m, 1 + i, 2 * ib), a1 = E.bias_at(m, 1 + i, 2 * ib + 1);
      ring32::seg2<QH, 0, 0>(A, src, a0, a1, [&](int u) {
        if (!RAW && ib > 0)
#pragma unroll
          for (int k = (u * 8) / QH; k < ((u + 1) * 8) / QH; ++k) retire1(ib - 1, k);
      });
      if (RAW) { acc[2 * ib] = a0; acc[2 * ib + 1] = a1; }
      else { pend0 = a0; pend1 = a1; }
      E.end();
    }
    if (!RAW)
#pragma unroll
      for (int k = 0; k < 8; ++k) retire1(NC - 1, k);
  };
  // hidden layers: x = layer(act(cat[x, enc] if skip else x)) (neural_blocks.py:81-84)
  for (int i = 0; i < L; ++i) {
#pragma unroll
    for (int k = 0; k < KH; ++k) src[k] = dst[k];
    if (i != L - 1 && i % SK == 0) {
      hidden(i, std::true_type{});
      enc_part32<S, ACT>(E, m, basis, true, x0, x1, x2, acc);
      act_all();
    } else {
      hidden(i, std::false_type{});
    }
  }
  return out32<S>(E, m, dst);
}

// ---------------------------------------------------------------------------------------------
// fp32-split (f16 hi/lo halves, three f16 MFMA products, f32 accumulation)
// ---------------------------------------------------------------------------------------------
// k-outer encoding part: pieces [k-step][sub-block][hi, lo]
// (GUARD: every input times d, its magnitude noted for the range check)
template <class S, int ACT, bool GUARD = false, class En, class Note>
__device__ __forceinline__ void enc_part3(En& E, const RProgMlp& m, const float4* basis, bool actv,
                                          float x0, float x1, float x2, f4v (&acc)[S::NSB],
                                          float d, Note&& note) {
  const int g = E.lane >> 4;
#pragma unroll 1
  for (int cc = 0; cc < S::CE3; ++cc) {
    const float4* A = E.begin();
#pragma unroll
    for (int vv = 0; vv < S::EK; ++vv) {
      const int v = cc * S::EK + vv;
      if (v < S::KQ) {
        // element e of lane group g: slot 32 v + 8 g + e; pairs (e, e + 1) = (sin, cos) of
        // projection 16 v + 4 g + e / 2 (or x / zeros past 2F)
        u4v bh, bl;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float sn, cs;
          enc_pair(basis, m.F, 16 * v + 4 * g + q, x0, x1, x2, sn, cs);
          if (actv) { sn = ring3::act<ACT>(sn); cs = ring3::act<ACT>(cs); }
          if (GUARD) {
            sn *= d; cs *= d;
            note(sn); note(cs);
          }
          uint32_t hi, lo;
          ring3::split2(sn, cs, hi, lo);
          bh[q] = hi; bl[q] = lo;
        }
#pragma unroll
        for (int sb = 0; sb < S::NSB; sb += 2) {
          const int p = (vv * S::NSB + sb) * 2;
          const u4v h0 = __builtin_bit_cast(u4v, A[p * 64]), l0 = __builtin_bit_cast(u4v, A[(p + 1) * 64]);
          const u4v h1 = __builtin_bit_cast(u4v, A[(p + 2) * 64]), l1 = __builtin_bit_cast(u4v, A[(p + 3) * 64]);
          acc[sb] = ring3::mfma(h0, bh, acc[sb]); acc[sb + 1] = ring3::mfma(h1, bh, acc[sb + 1]);
          acc[sb] = ring3::mfma(h0, bl, acc[sb]); acc[sb + 1] = ring3::mfma(h1, bl, acc[sb + 1]);
          acc[sb] = ring3::mfma(l0, bh, acc[sb]); acc[sb + 1] = ring3::mfma(l1, bh, acc[sb + 1]);
        }
      }
    }
    E.end();
  }
}

// GUARD: the range-guarded variant (nrt_ring3.h header), exponents lexp[mi][l] of this MLP
template <class S, int ACT, bool GUARD = false, class En>
__device__ __forceinline__ f4v eval3(En& E, const RProgMlp& m, int mi, float x0, float x1, float x2) {
  constexpr int NSB = S::NSB, NC = S::NC, KH = S::KH;
  const float4* basis = E.lbasis + m.basis_off;
  const float* scl = E.ltab + m.scale_off;  // 2^-s per layer
  const int L = m.L, SK = m.skip;
  u4v sh[KH], sl[KH], dh[KH], dl[KH];
  f4v acc[NSB];
  f4v pend0, pend1;
  // range guard: inputs of linear layer l scaled by dn(l) = 2^-e_l, its accumulator by up(l)
  const int* lx = E.lexp + mi * kMaxLin;
  auto ex = [&](int l) -> int { return GUARD ? __builtin_amdgcn_readfirstlane(lx[l]) : 0; };
  auto dn = [&](int l) -> float { return GUARD ? __int_as_float((127 - ex(l)) << 23) : 1.f; };
  auto up = [&](int l) -> float { return GUARD ? __int_as_float((127 + ex(l)) << 23) : 1.f; };
  float gm = 0.f;
  bool fail = false;
  auto note = [&](float a) { if (GUARD) gm = fmaxf(gm, fabsf(a)); };
  auto guard = [&](int l) {  // as ring3::eval's, the exponent raised in LDS for the block
    if constexpr (GUARD) {
      const bool over = wave_any(gm >= 65504.f) && !fail;
      const int e = ex(l);
      if (over && e < 100) {
        if (E.lane == 0) atomicMax(E.lexp + mi * kMaxLin + l, e + 12);
        E.changed = true;
      }
      fail = fail || over;
      gm = 0.f;
    }
  };
  // activation pair q (< 4) of a chunk's accumulators into k-step ib of dst (B element pair 2q,
  // 2q + 1 = registers 2q, 2q + 1 of sub-block 2 ib for q < 2, of sub-block 2 ib + 1 after);
  // sc = the layer's scale (x up under GUARD), d = the next layer's input scale
  auto retire2 = [&](float sc, float d, int ib, int q) {
    const float z0 = (q < 2 ? pend0[2 * (q & 1)] : pend1[2 * (q & 1)]) * sc;
    const float z1 = (q < 2 ? pend0[2 * (q & 1) + 1] : pend1[2 * (q & 1) + 1]) * sc;
    float a0 = ring3::act<ACT>(z0), a1 = ring3::act<ACT>(z1);
    if (GUARD) {
      a0 *= d; a1 *= d;
      note(a0); note(a1);
    }
    uint32_t hi, lo;
    ring3::split2(a0, a1, hi, lo);
    asm volatile("" : "+v"(hi), "+v"(lo));
    dh[ib][q] = hi; dl[ib][q] = lo;
  };
  auto act_all = [&](float sc, float d) {
#pragma unroll
    for (int ib = 0; ib < NC; ++ib) {
      pend0 = acc[2 * ib]; pend1 = acc[2 * ib + 1];
#pragma unroll
      for (int q = 0; q < 4; ++q) retire2(sc, d, ib, q);
    }
  };
  auto bias = [&](int layer, int sb) {
    f4v b = E.bias_at(m, layer, sb);
    if (GUARD) b *= dn(layer);
    return b;
  };
  // init layer: the raw encoding, k-outer
#pragma unroll
  for (int sb = 0; sb < NSB; ++sb) acc[sb] = bias(0, sb);
  enc_part3<S, ACT, GUARD>(E, m, basis, false, x0, x1, x2, acc, dn(0), note);
  guard(0);
  act_all(GUARD ? scl[0] * up(0) : scl[0], dn(1));
  // hidden part of layer i (as eval32: RAW keeps the accumulators for the encoding part)
  auto hidden = [&](int i, float sc, float d, auto raw_c) {
    constexpr bool RAW = decltype(raw_c)::value;
#pragma unroll
    for (int ib = 0; ib < NC; ++ib) {
      const float4* A = E.begin();
      f4v a0 = bias(1 + i, 2 * ib), a1 = bias(1 + i, 2 * ib + 1);
      auto side = [&](int u) {
        if (!RAW && ib > 0)
#pragma unroll
          for (int q = (u * 4) / KH; q < ((u + 1) * 4) / KH; ++q) retire2(sc, d, ib - 1, q);
      };
      ring3::seg<KH, 0, KH, decltype(side)&, !GUARD>(A, sh, sl, a0, a1, side);
      if (RAW) { acc[2 * ib] = a0; acc[2 * ib + 1] = a1; }
      else { pend0 = a0; pend1 = a1; }
      E.end();
    }
    if (!RAW)
#pragma unroll
      for (int q = 0; q < 4; ++q) retire2(sc, d, NC - 1, q);
  };
  for (int i = 0; i < L; ++i) {
#pragma unroll
    for (int k = 0; k < KH; ++k) { sh[k] = dh[k]; sl[k] = dl[k]; }
    const float sc = GUARD ? scl[1 + i] * up(1 + i) : scl[1 + i];
    const float d = dn(2 + i);
    if (i != L - 1 && i % SK == 0) {
      hidden(i, sc, d, std::true_type{});
      enc_part3<S, ACT, GUARD>(E, m, basis, true, x0, x1, x2, acc, dn(1 + i), note);
      guard(1 + i);
      act_all(sc, d);
    } else {
      guard(1 + i);
      hidden(i, sc, d, std::false_type{});
    }
  }
  guard(L + 1);
  // out layer: pieces [k-step][hi, lo] of one sub-block; three chains (hi.hi, hi.lo, lo.hi)
  const float4* A = E.begin();
  f4v o0 = bias(L + 1, 0), o1 = f4v{0.f, 0.f, 0.f, 0.f}, o2 = o1;
  {
    float4 w0 = A[0], w1 = A[64];
#pragma unroll
    for (int u = 0; u < KH; ++u) {
      float4 n0 = w0, n1 = w1;
      if (u + 1 < KH) { n0 = A[(2 * u + 2) * 64]; n1 = A[(2 * u + 3) * 64]; }
      const u4v h = __builtin_bit_cast(u4v, w0), l = __builtin_bit_cast(u4v, w1);
      o0 = ring3::mfma(h, dh[u], o0);
      o1 = ring3::mfma(h, dl[u], o1);
      o2 = ring3::mfma(l, dh[u], o2);
      w0 = n0; w1 = n1;
    }
  }
  E.end();
  return (o0 + (o1 + o2)) * (GUARD ? scl[L + 1] * up(L + 1) : scl[L + 1]);
}

// MLP mi of the program; the split path takes the block's guarded variant once it is on
template <int PREC, class S, int ACT, class En>
__device__ __forceinline__ f4v eval(En& E, const RProgMlp& m, int mi, float x0, float x1, float x2) {
  if constexpr (PREC == 2) {
    if (__builtin_amdgcn_readfirstlane((int)E.guarded)) return eval3<S, ACT, true>(E, m, mi, x0, x1, x2);
    return eval3<S, ACT>(E, m, mi, x0, x1, x2);
  } else {
    return eval32<S, ACT>(E, m, x0, x1, x2);
  }
}

__device__ __forceinline__ bool finite4(const f4v& o) {
  return __builtin_isfinite(o[0]) && __builtin_isfinite(o[1]) && __builtin_isfinite(o[2]) &&
         __builtin_isfinite(o[3]);
}

// row q (< 16) of ray lane & 15 from an eval tile
__device__ __forceinline__ float out_row(const f4v& o, int q, int lane) {
  return __shfl(o[q & 3], 16 * (q >> 2) + (lane & 15));
}

// ---------------------------------------------------------------------------------------------
// kernels: k_light_r (LightField sample per hit) then k_bsdf_r (spatial weights + components);
// the same math and LS layout as k_light16 / k_bsdf16 (nrt_kernels.h)
// ---------------------------------------------------------------------------------------------
template <int PREC, int D, int WV>
__global__ void __launch_bounds__(64 * WV, 1) k_light_r(
    const RProgDev prog, const LightDev* __restrict__ lp, const float* __restrict__ P_,
    const float* __restrict__ N_, const float* __restrict__ WI, const int32_t* __restrict__ hit_idx,
    const int32_t* __restrict__ hit_count, const float* __restrict__ lscale, float* __restrict__ LS) {
  extern __shared__ __attribute__((aligned(16))) char smem_c[];
  const LightDev& lt = *lp;
  const int64_t total = *(const NRT_GLOBAL int32_t*)hit_count;
  const int64_t per_block = 16 * WV;
  if ((int64_t)blockIdx.x * per_block >= total) return;
  Engine<D, WV> E;
  E.init(prog, smem_c);
  const int lane = E.lane, j = lane & 15;
  for (int64_t b0 = (int64_t)blockIdx.x * per_block; b0 < total; b0 += (int64_t)gridDim.x * per_block) {
    const int64_t i = b0 + 16 * E.wv + j;
    const bool valid = i < total;
    const int64_t idx = hit_idx[valid ? i : total - 1];
    const float px = P_[idx * 3], py = P_[idx * 3 + 1], pz = P_[idx * 3 + 2];
    f4v o = eval<PREC, LightShape, ACT_LEAKY>(E, prog.mlp[0], 0, px, py, pz);
    if constexpr (PREC == 2) {  // range guard (nrt_ring3.h)
      while (E.retry(finite4(o))) o = eval<PREC, LightShape, ACT_LEAKY>(E, prog.mlp[0], 0, px, py, pz);
    }
    float fr[9];
    make_frame(N_[idx * 3], N_[idx * 3 + 1], N_[idx * 3 + 2], fr);
    const float wix = WI[idx * 3], wiy = WI[idx * 3 + 1], wiz = WI[idx * 3 + 2];
    float le[3], wo[3], feat[3];
    light_from_field(out_row(o, 0, lane), out_row(o, 1, lane), out_row(o, 2, lane), lt, fr, wix, wiy,
                     wiz, le, wo, feat);
    if (lscale) {  // shadow test (scene.py:297) or learned occlusion (scene.py:313-318)
      const float* sc = lscale + (valid ? i : total - 1) * 3;
      le[0] *= sc[0]; le[1] *= sc[1]; le[2] *= sc[2];
    }
    if (valid && lane < 16) {
      float* q = LS + i * kLsStride;
      q[0] = le[0]; q[1] = le[1]; q[2] = le[2];
      q[3] = feat[0]; q[4] = feat[1]; q[5] = feat[2];
      q[6] = wo[0]; q[7] = wo[1]; q[8] = wo[2];
    }
  }
  E.drain();
}

template <int PREC, int D, int WV, bool SPATIAL>
__global__ void __launch_bounds__(64 * WV, 1) k_bsdf_r(
    const RProgDev prog, const BsdfDev* __restrict__ bp, const float* __restrict__ P_,
    const float* __restrict__ WI, const int32_t* __restrict__ hit_idx,
    const int32_t* __restrict__ hit_count, const float* __restrict__ LS, float* __restrict__ rgb,
    float* __restrict__ wout) {
  extern __shared__ __attribute__((aligned(16))) char smem_c[];
  const BsdfDev& bs = *bp;
  const int nc = bs.n;
  const int64_t total = *(const NRT_GLOBAL int32_t*)hit_count;
  const int64_t per_block = 16 * WV;
  if ((int64_t)blockIdx.x * per_block >= total) return;
  Engine<D, WV> E;
  E.init(prog, smem_c);
  const int lane = E.lane, j = lane & 15;
  for (int64_t b0 = (int64_t)blockIdx.x * per_block; b0 < total; b0 += (int64_t)gridDim.x * per_block) {
    const int64_t i = b0 + 16 * E.wv + j;
    const bool valid = i < total;
    const int64_t ii = valid ? i : total - 1;
    const int64_t idx = hit_idx[ii];
    const float* ls = LS + ii * kLsStride;
    const float le0 = ls[0], le1 = ls[1], le2 = ls[2];
    const float ft0 = ls[3], ft1 = ls[4], ft2 = ls[5];
    const float wo0 = ls[6], wo1 = ls[7], wo2 = ls[8];
    float K[16];
    float f0, f1, f2;
    // the tile's evaluations; the split path repeats them while the range guard asks
    for (;;) {
    bool ok = true;
    int k = 0;
    if (SPATIAL) {
      const float px = P_[idx * 3], py = P_[idx * 3 + 1], pz = P_[idx * 3 + 2];
      const f4v o = eval<PREC, SpatialShape, ACT_LEAKY>(E, prog.mlp[0], 0, px, py, pz);
      ok = ok && finite4(o);
      k = 1;
#pragma unroll
      for (int q = 0; q < 16; ++q) K[q] = sigmoidf_(out_row(o, q, lane));
    } else {
#pragma unroll
      for (int q = 0; q < 16; ++q) K[q] = 1.f;
    }
    f0 = 0.f; f1 = 0.f; f2 = 0.f;
    for (int c = 0; c < nc; ++c) {
      const BsdfCompDev& cp = bs.comp[c];
      float v[3];
      if (cp.kind == 0) {
        const f4v o = eval<PREC, BsdfShape, ACT_LEAKY>(E, prog.mlp[k], k, ft0, ft1, ft2);
        ok = ok && finite4(o);
        ++k;
#pragma unroll
        for (int q = 0; q < 3; ++q) v[q] = act_fwd<false>(out_row(o, q, lane), cp.act);
      } else if (cp.kind == 1) {
        // Diffuse.eval_and_pdf (bsdfs.py:108-118)
        for (int q = 0; q < 3; ++q) {
          float x = wo2 * cp.params[q];
          v[q] = (cp.act == ACT_NONE) ? x / (float)M_PI : act_fwd<false>(x, cp.act);
        }
      } else {
        // Conductor.eval_and_pdf (bsdfs.py:364-388)
        const float wix = WI[idx * 3], wiy = WI[idx * 3 + 1], wiz = WI[idx * 3 + 2];
        float rx = -wix, ry = -wiy, rz = wiz;
        bool th = ((rx * wo0 + ry * wo1) + rz * wo2) > 0.94f;
        float fres = fresnel_conductor(wiz, cp.params[3]);
        for (int q = 0; q < 3; ++q) v[q] = th ? fres * act_fwd<false>(cp.params[q], cp.act) : 0.f;
      }
      float kj = K[0];
#pragma unroll
      for (int q = 1; q < 16; ++q) kj = c == q ? K[q] : kj;
      f0 += v[0] * kj; f1 += v[1] * kj; f2 += v[2] * kj;
    }
    if (PREC != 2 || !E.retry(ok)) break;
    }
    if (valid && lane < 16) {
      // integrators.py:186-189: mis(=1) * bsdf_val * emitter_val, / emitter_samples(=1)
      rgb[idx * 3] = (1.f * f0) * le0;
      rgb[idx * 3 + 1] = (1.f * f1) * le1;
      rgb[idx * 3 + 2] = (1.f * f2) * le2;
      if (wout)
#pragma unroll
        for (int q = 0; q < 16; ++q)
          if (q < nc) wout[idx * nc + q] = K[q];
    }
  }
  E.drain();
}

// One MLP's single-MLP ("solo") row program and its output, a job of the forward kernel below.
// The jobs travel as kernel arguments (no job-table copy): 16 x 88 B.
struct SoloJob {
  const void* stream;
  const int* chunks;
  const float* tables;
  const float4* basis;
  float* y;  // [M, out] row-major
  // training forward (k_mlp_ring SAVE): the activations the ring backward reads (nrt_train_ring.h
  // BwdRingJob): A [L+1][M][H], the encoding raw / activated [M][dp]
  float *A, *Eraw, *Eact;
  int stream_bytes, n_chunks, table_floats, basis_q, out;
  RProgMlp mlp;
};
constexpr int kMaxSoloJobs = 16;
struct SoloJobs {
  SoloJob j[kMaxSoloJobs];
};

// (the forward kernel on SoloJobs, k_mlp_ring, is in nrt_train_ring.h beside its SAVE variant)

}  // namespace rprog
}  // namespace nrt
