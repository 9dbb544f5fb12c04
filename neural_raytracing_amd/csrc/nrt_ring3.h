// nrt_ring3.h -- the SDF MLP at FP32 accuracy on the FP16 matrix cores ("fp32-split" precision).
//
// gfx950 has no TF32/xf32 MFMA; its exact-f32 MFMA (v_mfma_f32_16x16x4_f32) runs at 1/16 of the
// FP16 rate.  This engine evaluates the same GEMMs as the FP32 ring (nrt_device.h ring32) with
// every operand split into two FP16 halves and three FP16 MFMAs per product block:
//     W 2^s = Wh + Wl,  a = ah + al   (Wh = RNE_f16(W 2^s), Wl = RNE_f16(W 2^s - Wh); likewise a)
//     acc  += Wh ah + Wh al + Wl ah     (v_mfma_f32_16x16x32_f16, f32 accumulation)
//     z     = acc 2^-s                 (s per layer: max|W| 2^s in [1, 2), so Wl is a normal f16)
// The halves carry 22 significant bits of each operand; the dropped Wl al term is 2^-22 of a
// product and the split residuals 2^-23, while the accumulation rounds once per MFMA (24 times
// per 256-input row instead of 256 fma roundings): the result is as close to the float64 value
// as the FP32 fma chain's (tests/test_gpu_split.py measures both against float64).  Throughput:
// 3 x 16 cycles per 16x16x32 block against 8 x 32 cycles for the same block on f32 MFMA.
//
// Layout is ring32's with K steps of 32: a wave owns 16 rays (lane (g = lane >> 4, j = lane & 15)
// serves ray j, lane group g holds k = 8 g .. 8 g + 7 of each k-step); the 16x16 accumulator of
// output sub-block b holds rows 16 b + 4 g + r of ray j in register r, so sub-blocks 2u, 2u + 1 of
// a layer are k-step u of the next layer's B operand (the packer permutes W's columns to match,
// nrt_internal.h ring3_walk) and activations never leave registers: per lane H / 16 f16 words for
// the hi halves and as many for the lo halves (32 + 32 VGPRs at H = 256).  The weight stream
// moves through a 2-slot LDS ring by LDS-DMA exactly as in ring32 (chunk = 32 output rows =
// one k-step of the next layer: 2 sub-blocks x 2 halves x 1 KiB per k-step).
//
// Range guard.  An f16 half holds |a| < 65520; the weights are scaled per layer by the packer
// (scale3), activations are data-dependent.  An activation past f16's range makes its hi half
// +-inf and its lo half the opposite infinity, so the next layer's Wh ah + Wh al is inf - inf =
// NaN in every row (0 x inf is NaN too) and the evaluation's output is NaN: a non-finite output
// is the overflow signal, at no cost per element.  The caller (RingPol3::retry, the normal and
// shading kernels) then re-runs the evaluation in the guarded variant (GUARD): the inputs of
// linear layer l are scaled by 2^-e_l before the split (and its bias with them), its accumulator
// by 2^e_l after -- powers of two, exact -- and each layer's largest scaled input is checked;
// the first layer whose inputs still leave the range gets e_l raised by 12, and the evaluation
// runs again, until no layer overflows (a few retries per layer at most).
// The exponents stay with the wave (or block) for its later evaluations.  Small inputs of a
// scaled layer keep an absolute resolution of 2^(e_l - 25), i.e. ~2^-35 of the layer's largest.
#pragma once
#include "nrt_device.h"

namespace nrt {
namespace ring3 {

typedef float f4v __attribute__((ext_vector_type(4)));
typedef uint32_t u4v __attribute__((ext_vector_type(4)));
typedef _Float16 hv2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f4v mfma(const u4v& a, const u4v& b, f4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, a), __builtin_bit_cast(h8, b),
                                                c, 0, 0, 0);
}

// (a, b) -> packed hi = RNE_f16(a, b) and lo = RNE_f16(a - hi.x, b - hi.y).  The remainders are
// exact in f32 (hi holds a's top 11 bits); v_fma_mix_f32 reads hi's f16 half directly (one
// instruction instead of a convert and a subtract).
__device__ __forceinline__ void split2(float a, float b, uint32_t& hi, uint32_t& lo) {
  const hv2 h = {(_Float16)a, (_Float16)b};
  const uint32_t hw = __builtin_bit_cast(uint32_t, h);
  float ra, rb;
  asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(ra) : "v"(hw), "v"(a));
  asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(rb) : "v"(hw), "v"(b));
  const hv2 l = {(_Float16)ra, (_Float16)rb};
  hi = hw;
  lo = __builtin_bit_cast(uint32_t, l);
}

// The activation on the split path.  Softplus MLPs are folded into the log2 domain by the packer
// (init W and every init / hidden bias x log2 e, out W x ln 2, as the FP16 ring stream), so the
// device computes softplus(x) / ln 2 = log2(1 + 2^z) at z = x log2 e: v_exp + v_add + v_log, with
// z itself above 64 (log2(1 + 2^z) == z in f32 there; 2^z would overflow at 128).  Against torch's
// F.softplus (threshold 20, log1p(exp(x))) the difference is the rounding of 1 + 2^z and the
// ~1-ulp v_exp / v_log: ~1e-7 absolute, the size of FP32 accumulation noise (the accuracy test
// against float64, tests/test_gpu_split.py, holds the path to the FP32 fma chain's error).
template <int ACT>
__device__ __forceinline__ float act(float z) {
  if (ACT == ACT_SOFTPLUS) {
    const float l = __builtin_amdgcn_logf(1.f + __builtin_amdgcn_exp2f(z));
    return z > 64.f ? z : l;
  }
  return act_fwd<false>(z, ACT);
}
// the encoding's activation (skip-layer inputs): act(enc) in the fold's units
template <int ACT>
__device__ __forceinline__ float act_enc(float v) {
  return ACT == ACT_SOFTPLUS ? act<ACT>(v * 1.4426950408889634f) : act<ACT>(v);
}

// KH = H / 32 hidden k-steps, KQ = ke3 / 32 encoding k-steps.  Ring depth: 3 slots (the DMA runs
// two chunks ahead) where they fit beside the basis / bias / sphere tables in 160 KiB, else 2.
template <int KH, int KQ, int WV>
struct Engine {
  static constexpr int MAXQ = 4 * (KH + KQ);            // largest chunk (a skip layer's), KiB
  static constexpr int MAXL = (MAXQ + WV - 1) / WV;     // DMA pieces per wave per chunk
  static constexpr int SLOTQ = MAXL * WV;
  static constexpr int D = 3 * SLOTQ * 1024 <= 128 * 1024 ? 3 : 2;
  static constexpr int RING_BYTES = D * SLOTQ * 1024;
  static constexpr int kOutOfRange = 0x40000000;
  // LDS of one block: ring | basis (float4 per frequency) | biases | sphere table
  static size_t lds_bytes(int F, size_t bias_bytes, size_t sphere_bytes) {
    return RING_BYTES + (size_t)F * 16 + bias_bytes + sphere_bytes;
  }
  const float4* ring;
  uint32_t ring_lds;
  const float* lbias;
  const float4* lbasis;
  const float4* lspheres;   // [n][4] float4 (SdfDev layout), read by ring32::spheres_value16
  const void* sbase;
  int sbytes, bstride;
  int slot;
  int lane, wv;
  // range guard (see the header): lane l holds e_l, the exponent of linear layer l's inputs;
  // `guarded` selects eval<..., GUARD>; `changed` = the last guarded evaluation raised an e_l
  int gexp = 0;
  bool guarded = false, changed = false;

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

  // block-wide; afterwards chunk 0 (the init layer's, nq0 pieces) is in flight to slot 0 and,
  // with a 3-slot ring, chunk 1 (nq1 pieces) to slot 1
  __device__ __forceinline__ void init(const MlpDev& m, const SdfDev& s, char* lds, int nq0,
                                       int nq1) {
    ring = reinterpret_cast<const float4*>(lds);
    ring_lds = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)lds;
    char* p = lds + RING_BYTES;
    const int F = m.freqs;
    float4* lq = reinterpret_cast<float4*>(p);
    for (int q = threadIdx.x; q < F; q += blockDim.x)
      lq[q] = make_float4(m.basis[q], m.basis[F + q], m.basis[2 * F + q], 0.f);
    lbasis = lq;
    p += (size_t)F * 16;
    float* lb = reinterpret_cast<float*>(p);
    const int nb = (m.n_hidden + 2) * m.bias16_stride;
    for (int i = threadIdx.x; i < nb; i += blockDim.x) lb[i] = m.bias3[i];
    lbias = lb;
    p += (size_t)nb * 4;
    float4* ls = reinterpret_cast<float4*>(p);
    if (s.kind == 2)
      for (int i = threadIdx.x; i < s.n_spheres * 4; i += blockDim.x)
        ls[i] = reinterpret_cast<const float4*>(s.spheres)[i];
    lspheres = ls;
    bstride = m.bias16_stride;
    sbase = m.stream3;
    sbytes = m.stream3_bytes;
    lane = threadIdx.x & 63;
    wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    slot = 0;
    // pieces of one whole evaluation (chunk offsets wrap at it): init NC x 4 KQ, hidden layers
    // NC x 4 (KH + KQ on skip layers), out 2 KH
    {
      const int L = m.n_hidden, SK = m.skip;
      int nskip = 0;
      for (int i = 0; i < L; ++i) nskip += (i != L - 1 && i % SK == 0) ? 1 : 0;
      tot = KH * 4 * KQ + 2 * KH + L * KH * 4 * KH + KH * 4 * KQ * nskip;
    }
    issue(0, nq0, 0);
    if (D == 3) {
      issue(nq0, nq1, 1);
      dma_off = nq0 + nq1;  // stream offset of the chunk after the two in flight
    } else {
      dma_off = nq0;
    }
    __syncthreads();
  }
  int dma_off;  // stream offset of the next chunk to DMA (wave-uniform)
  int tot;      // pieces per evaluation
  // Start of the current chunk: wait for it, then DMA a chunk ahead -- with 2 slots the next one,
  // with 3 the one after (chunk c + 2 lands in the slot chunk c - 1 used, which every wave has
  // left once it passes this barrier); nq_ahead pieces, the offset wrapping to the next
  // evaluation's first chunk.  The pieces of one wave complete in issue order, so the wait for
  // the current chunk leaves the younger chunk's MAXL pieces in flight (vmcnt(MAXL)).
  __device__ __forceinline__ const float4* begin(int nq_ahead) {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(ring::waitcnt_vm_lgkm0(D == 3 ? MAXL : 0));
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int o = dma_off >= tot ? dma_off - tot : dma_off;
    issue(o, nq_ahead, slot == 0 ? D - 1 : slot - 1);
    dma_off = o + nq_ahead;
    __builtin_amdgcn_sched_barrier(0);
    return ring + slot * SLOTQ * 64 + lane;
  }
  __device__ __forceinline__ void end() { slot = slot + 1 == D ? 0 : slot + 1; }
  __device__ __forceinline__ void drain() { __builtin_amdgcn_s_waitcnt(ring::waitcnt_vm_lgkm0(0)); }
  // acc[reg] = bias3[layer][16 sb + 4 g + reg]
  __device__ __forceinline__ f4v bias_at(int layer, int sb) const {
    const float4 q = *reinterpret_cast<const float4*>(lbias + layer * bstride + 16 * sb + 4 * (lane >> 4));
    return f4v{q.x, q.y, q.z, q.w};
  }
};

// One segment of a two-sub-block chunk: NU k-steps at ring pieces P0 + 4u + {hi b0, lo b0, hi b1,
// lo b1}; chains a0 / a1 alternate so consecutive MFMAs are independent.  Each k-step's four LDS
// reads are issued one k-step ahead.  side(u) runs before k-step u + 1's reads in program order.
struct NoSide {
  __device__ __forceinline__ void operator()(int) const {}
};
// PF = false (the guarded variant): each k-step's pieces are read in place, not a k-step ahead
// (fewer live registers on the rare path, so the fast path keeps its allocation).
template <int NU, int P0, int NBV, class Side, bool PF = true>
__device__ __forceinline__ void seg(const float4* A, const u4v (&Bh)[NBV], const u4v (&Bl)[NBV],
                                    f4v& a0, f4v& a1, Side&& side) {
  if constexpr (!PF) {
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      side(u);
      const u4v h0 = __builtin_bit_cast(u4v, A[(P0 + 4 * u) * 64]);
      const u4v l0 = __builtin_bit_cast(u4v, A[(P0 + 4 * u + 1) * 64]);
      const u4v h1 = __builtin_bit_cast(u4v, A[(P0 + 4 * u + 2) * 64]);
      const u4v l1 = __builtin_bit_cast(u4v, A[(P0 + 4 * u + 3) * 64]);
      a0 = mfma(h0, Bh[u], a0); a1 = mfma(h1, Bh[u], a1);
      a0 = mfma(h0, Bl[u], a0); a1 = mfma(h1, Bl[u], a1);
      a0 = mfma(l0, Bh[u], a0); a1 = mfma(l1, Bh[u], a1);
    }
    return;
  }
  float4 w0 = A[P0 * 64], w1 = A[(P0 + 1) * 64], w2 = A[(P0 + 2) * 64], w3 = A[(P0 + 3) * 64];
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    side(u);
    float4 n0 = w0, n1 = w1, n2 = w2, n3 = w3;
    if (u + 1 < NU) {
      n0 = A[(P0 + 4 * u + 4) * 64]; n1 = A[(P0 + 4 * u + 5) * 64];
      n2 = A[(P0 + 4 * u + 6) * 64]; n3 = A[(P0 + 4 * u + 7) * 64];
    }
    const u4v h0 = __builtin_bit_cast(u4v, w0), l0 = __builtin_bit_cast(u4v, w1);
    const u4v h1 = __builtin_bit_cast(u4v, w2), l1 = __builtin_bit_cast(u4v, w3);
    a0 = mfma(h0, Bh[u], a0); a1 = mfma(h1, Bh[u], a1);
    a0 = mfma(h0, Bl[u], a0); a1 = mfma(h1, Bl[u], a1);
    a0 = mfma(l0, Bh[u], a0); a1 = mfma(l1, Bh[u], a1);
    w0 = n0; w1 = n1; w2 = n2; w3 = n3;
  }
}

// forward-mode activation (TAN, columns 4 ray + comp as ring32::eval): act(z) on the value column,
// act'(z) dz on the tangent columns, z from the quad leader.  Softplus in the log2 fold:
// d log2(1 + 2^z) / dz = 1 / (1 + 2^-z), and the fold's units carry through the tangent unchanged.
template <int ACT>
__device__ __forceinline__ float act_tan(float z, bool value) {
  const float zv = ring::quad_leader(z);
  if (ACT == ACT_SOFTPLUS) {
    const float e = __builtin_amdgcn_exp2f(-fabsf(zv));
    const float sig = (zv >= 0.f ? 1.f : e) * __builtin_amdgcn_rcpf(1.f + e);
    return value ? act<ACT>(zv) : sig * z;
  }
  return value ? act<ACT>(zv) : act_bwd(zv, ACT) * z;
}
// tangent of the encoding's activation (skip-layer inputs) at raw value v, raw tangent t
template <int ACT>
__device__ __forceinline__ float act_enc_tan(float v, float t) {
  if (ACT == ACT_SOFTPLUS) {
    // d log2(1 + 2^(v log2e)) / dv = log2e sigmoid(v)
    return 1.4426950408889634f * t * __builtin_amdgcn_rcpf(1.f + __expf(-v));
  }
  return act_bwd(v, ACT) * t;
}

// One SkipConnMLP evaluation (output row 0) for the wave's 16 columns; every lane of a column gets
// the value.  Columns are rays, or (TAN) 4 rays x (value, d/dx, d/dy, d/dz) as ring32::eval.
// Every wave of the block must call it the same number of times.
template <int KH, int KQ, int WV, int ACT, bool TAN = false, bool GUARD = false>
__device__ __forceinline__ float eval(Engine<KH, KQ, WV>& E, const MlpDev& m, float x0, float x1,
                                      float x2) {
  constexpr int NC = KH;  // 32-row chunks per hidden layer (= k-steps of the next layer)
  static_assert(KH == 4 || KH == 8, "hidden 128 or 256");
  const int g = E.lane >> 4;
  const int comp = TAN ? (E.lane & 3) : 0;
  const bool value = comp == 0;
  const int F = m.freqs, L = m.n_hidden, SK = m.skip;
  // range guard: 2^-e_l scales linear layer l's inputs (dn), 2^e_l its accumulator (up); gm =
  // this lane's largest scaled input of the layer being checked; fail = a layer overflowed in
  // this pass (later layers are NaN: only the first one is rescaled per pass)
  auto ex = [&](int l) -> int { return GUARD ? __builtin_amdgcn_readlane(E.gexp, l) : 0; };
  // 2^-e / 2^e from the exponent bits (scalar ALU: e is wave-uniform, |e| <= 100)
  auto dn = [&](int l) -> float { return GUARD ? __int_as_float((127 - ex(l)) << 23) : 1.f; };
  auto up = [&](int l) -> float { return GUARD ? __int_as_float((127 + ex(l)) << 23) : 1.f; };
  float gm = 0.f;
  bool fail = false;
  auto note = [&](float a) { if (GUARD) gm = fmaxf(gm, fabsf(a)); };
  auto guard = [&](int l) {
    if constexpr (GUARD) {
      // first overflowing layer of the pass: its inputs' scale 2^-e_l drops by 2^-12 (a wave
      // max reduction here costs the fast variant registers); inputs up to 2^27 then fit, a
      // larger range takes another pass.  e_l stops at 100 (an f32 overflow, +-inf activations,
      // is the reference's too: nothing to rescale), so every retry loop ends.
      // branch-free (selects on wave-uniform conditions)
      const bool over = wave_any(gm >= 65504.f) && !fail;
      const bool raise = over && __builtin_amdgcn_readlane(E.gexp, l) < 100;
      E.gexp += (raise && E.lane == l) ? 12 : 0;
      E.changed = E.changed || raise;
      fail = fail || over;
      gm = 0.f;
    }
  };
  // values r (and, TAN, tangents tr) of the encoding pair q of k-step v of this lane
  auto enc_vals = [&](int v, int q, float (&r)[2], float (&tr)[2]) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int slot = 32 * v + 8 * g + 2 * q + t;
      float val = 0.f, tv = 0.f;
      if (slot < 2 * F) {
        const float4 b = E.lbasis[slot >> 1];
        float pr = x0 * b.x;
        pr = fmaf(x1, b.y, pr);
        pr = fmaf(x2, b.z, pr);
        float sn, cs;
        sincosf(pr, &sn, &cs);
        val = t ? cs : sn;
        if (TAN) {
          const float bk = comp == 1 ? b.x : comp == 2 ? b.y : b.z;
          tv = t ? -sn * bk : cs * bk;
        }
      } else if (slot == 2 * F) {
        val = x0;
        tv = comp == 1 ? 1.f : 0.f;
      } else if (slot == 2 * F + 1) {
        val = x1;
        tv = comp == 2 ? 1.f : 0.f;
      } else if (slot == 2 * F + 2) {
        val = x2;
        tv = comp == 3 ? 1.f : 0.f;
      }
      r[t] = val;
      tr[t] = tv;
    }
  };
  // act(enc) (skip-layer inputs) of pair q of k-step v, times d: value columns act_enc(r),
  // tangent columns its tangent
  auto enc_act = [&](int v, int q, float d, uint32_t& hi, uint32_t& lo) {
    float r[2], tr[2];
    enc_vals(v, q, r, tr);
    float a0, a1;
    if (TAN && !value) {
      a0 = act_enc_tan<ACT>(r[0], tr[0]); a1 = act_enc_tan<ACT>(r[1], tr[1]);
    } else {
      a0 = act_enc<ACT>(r[0]); a1 = act_enc<ACT>(r[1]);
    }
    if (GUARD) {
      a0 *= d; a1 *= d;
      note(a0); note(a1);
    }
    split2(a0, a1, hi, lo);
  };
  // the raw encoding (init-layer inputs) and, unguarded, act(enc) for the skip layers (the
  // guarded variant recomputes act(enc) per skip layer at that layer's scale instead of holding
  // it: fewer live registers on the rare path)
  u4v erh[KQ], erl[KQ], eah[GUARD ? 1 : KQ], eal[GUARD ? 1 : KQ];
#pragma unroll
  for (int v = 0; v < KQ; ++v) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float r[2], tr[2];
      enc_vals(v, q, r, tr);
      float e0 = (TAN && !value) ? tr[0] : r[0], e1 = (TAN && !value) ? tr[1] : r[1];
      if (GUARD) {
        const float d0 = dn(0);
        e0 *= d0; e1 *= d0;
        note(e0); note(e1);
      }
      uint32_t hi, lo;
      split2(e0, e1, hi, lo);
      erh[v][q] = hi; erl[v][q] = lo;
      if constexpr (!GUARD) {
        enc_act(v, q, 1.f, hi, lo);
        eah[v][q] = hi; eal[v][q] = lo;
      }
    }
  }
  auto chunk_q = [&](int i) {  // pieces of hidden layer i's chunks (i == L: the out layer)
    if (i >= L) return 2 * KH;
    return 4 * (KH + ((i != L - 1 && i % SK == 0) ? KQ : 0));
  };
  // pieces of chunk c of the evaluation's chunk sequence (init NC, hidden L x NC, out 1; c past
  // the end is the next evaluation's): the ring DMAs chunk c + D - 1 at the start of chunk c
  const int NCH = NC + L * NC + 1;
  auto size_at = [&](int c) {
    if (c >= NCH) c -= NCH;
    if (c < NC) return 4 * KQ;
    if (c < NCH - 1) return chunk_q((c - NC) / NC);
    return 2 * KH;
  };
  constexpr int AH = Engine<KH, KQ, WV>::D - 1;  // chunks the DMA runs ahead
  u4v sh[KH], sl[KH], dh[KH], dl[KH];
  f4v pend0, pend1;
  // activation of chunk ib's accumulators (layer `layer`) into k-step ib of dst, one pair of
  // elements at a time: pair q = elements 2q, 2q + 1 of the B fragment (registers 2q, 2q + 1 of
  // sub-block 2 ib for q < 2, of sub-block 2 ib + 1 after).  The empty asm pins each result inside
  // the chunk that computes it (dst is read only by the next layer).
  auto retire2 = [&](int layer, int ib, int q) {
    const float sc = GUARD ? m.scale3[layer] * up(layer) : m.scale3[layer];
    const float z0 = (q < 2 ? pend0[2 * q] : pend1[2 * q - 4]) * sc;
    const float z1 = (q < 2 ? pend0[2 * q + 1] : pend1[2 * q - 3]) * sc;
    uint32_t hi, lo;
    float a0 = TAN ? act_tan<ACT>(z0, value) : act<ACT>(z0);
    float a1 = TAN ? act_tan<ACT>(z1, value) : act<ACT>(z1);
    if (GUARD) {
      const float d = dn(layer + 1);
      a0 *= d; a1 *= d;
      note(a0); note(a1);
    }
    split2(a0, a1, hi, lo);
    asm volatile("" : "+v"(hi), "+v"(lo));
    dh[ib][q] = hi; dl[ib][q] = lo;
  };
  const float bmask = value ? 1.f : 0.f;
  auto bias = [&](int layer, int sb) {
    f4v b = E.bias_at(layer, sb);
    if (TAN) b *= bmask;
    if (GUARD) b *= dn(layer);
    return b;
  };
  auto retire = [&](int layer, int ib) {
#pragma unroll
    for (int q = 0; q < 4; ++q) retire2(layer, ib, q);
  };
  guard(0);
  // init layer (neural_blocks.py:80): raw encoding in
#pragma unroll
  for (int ib = 0; ib < NC; ++ib) {
    const float4* A = E.begin(size_at(ib + AH));
    f4v a0 = bias(0, 2 * ib), a1 = bias(0, 2 * ib + 1);
    if (ib > 0) retire(0, ib - 1);
    seg<KQ, 0, KQ, NoSide, !GUARD>(A, erh, erl, a0, a1, NoSide{});
    pend0 = a0; pend1 = a1;
    E.end();
  }
  retire(0, NC - 1);
  // hidden layers: x = layer(act(cat[x, enc] if skip else x)) (neural_blocks.py:81-84)
  for (int i = 0; i < L; ++i) {
#pragma unroll
    for (int k = 0; k < KH; ++k) { sh[k] = dh[k]; sl[k] = dl[k]; }
    const bool skip = i != L - 1 && i % SK == 0;
    u4v gah[GUARD ? KQ : 1], gal[GUARD ? KQ : 1];
    if constexpr (GUARD) {
      if (skip) {
        const float d = dn(1 + i);
#pragma unroll
        for (int v = 0; v < KQ; ++v)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            uint32_t hi, lo;
            enc_act(v, q, d, hi, lo);
            gah[v][q] = hi; gal[v][q] = lo;
          }
      }
    }
    guard(1 + i);
#pragma unroll
    for (int ib = 0; ib < NC; ++ib) {
      const float4* A = E.begin(size_at(NC + i * NC + ib + AH));
      f4v a0 = bias(1 + i, 2 * ib), a1 = bias(1 + i, 2 * ib + 1);
      // the previous chunk's four activation pairs, spread over the chunk's k-steps
      auto side = [&](int u) {
        if (ib > 0 && (KH == 4 || (u & 1) == 0)) retire2(1 + i, ib - 1, KH == 4 ? u : u >> 1);
      };
      seg<KH, 0, KH, decltype(side)&, !GUARD>(A, sh, sl, a0, a1, side);
      if (skip) {
        if constexpr (GUARD) seg<KQ, 4 * KH, KQ, NoSide, false>(A, gah, gal, a0, a1, NoSide{});
        else seg<KQ, 4 * KH>(A, eah, eal, a0, a1, NoSide{});
      }
      pend0 = a0; pend1 = a1;
      E.end();
    }
    retire(1 + i, NC - 1);
  }
  guard(L + 1);
  // out layer (neural_blocks.py:86): one 16-row sub-block, pieces [k-step][hi, lo]; two chains
  // (even / odd k-steps); row 0 of ray j sits in register 0 of lane j
  const float4* A = E.begin(size_at(NCH - 1 + AH));
  f4v o0 = bias(L + 1, 0), o1 = f4v{0.f, 0.f, 0.f, 0.f};
  {
    float4 w0 = A[0], w1 = A[64], w2 = A[2 * 64], w3 = A[3 * 64];
#pragma unroll
    for (int u = 0; u < KH; u += 2) {
      float4 n0 = w0, n1 = w1, n2 = w2, n3 = w3;
      if (u + 2 < KH) {
        n0 = A[(2 * u + 4) * 64]; n1 = A[(2 * u + 5) * 64];
        n2 = A[(2 * u + 6) * 64]; n3 = A[(2 * u + 7) * 64];
      }
      const u4v h0 = __builtin_bit_cast(u4v, w0), l0 = __builtin_bit_cast(u4v, w1);
      const u4v h1 = __builtin_bit_cast(u4v, w2), l1 = __builtin_bit_cast(u4v, w3);
      o0 = mfma(h0, dh[u], o0); o1 = mfma(h1, dh[u + 1], o1);
      o0 = mfma(h0, dl[u], o0); o1 = mfma(h1, dl[u + 1], o1);
      o0 = mfma(l0, dh[u], o0); o1 = mfma(l1, dh[u + 1], o1);
      w0 = n0; w1 = n1; w2 = n2; w3 = n3;
    }
  }
  E.end();
  const float o = (o0[0] + o1[0]) * (GUARD ? m.scale3[L + 1] * up(L + 1) : m.scale3[L + 1]);
  return __shfl(o, E.lane & 15);
}

// After an evaluation of the wave (output v of this lane, `active` = the lane's result is used):
// true if it must run again -- an unguarded evaluation whose output is not finite somewhere
// switches the wave to the guarded variant; a guarded one repeats while it raised an exponent.
// The result is wave-uniform.
template <class Eng>
__device__ __forceinline__ bool retry(Eng& E, bool active, float v) {
  if (!__builtin_amdgcn_readfirstlane((int)E.guarded)) {
    if (!wave_any(active && !__builtin_isfinite(v))) return false;
    E.guarded = true;
    E.gexp = 0;
    E.changed = false;
    return true;
  }
  const bool ch = __builtin_amdgcn_readfirstlane((int)E.changed) != 0;
  E.changed = false;
  return ch;
}

}  // namespace ring3
}  // namespace nrt
