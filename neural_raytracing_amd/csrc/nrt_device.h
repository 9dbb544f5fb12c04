// nrt_device.h -- device-side building blocks of the gfx950 ray-march path.
//
// Work unit: one wavefront owns 32 rays.  Lane l serves ray r = l & 31 and lane-half h = l >> 5;
// both halves carry the same ray state, and the MFMA fragment layout splits the K dimension
// between them.  Every MLP layer is one GEMM  Z^T[N_out, 32 rays] = W[N_out, K] . U^T[K, 32 rays]
// computed with 32x32 MFMA tiles: W is the A operand (pre-packed per lane on the host, read from
// L2), the layer input U^T is the B operand.
//
//  * FP16 path ("register path"): v_mfma_f32_32x32x16_f16.  A layer's f32 accumulator tile has
//    the ray on the lane and the output feature in the 16 registers, which is exactly the B
//    fragment layout of the next layer; activations never leave registers (the k order inside
//    a fragment is permuted, and the host packer permutes W's columns to match).
//  * FP32 path ("LDS path"): v_mfma_f32_32x32x2_f32 (exact f32 fma chain).  Two 16-register
//    tiles per input do not fit, so each wave keeps its 32 rays' activations in an LDS slab
//    X[32][RS] and the B operand is one ds_read_b32 per k-step.
//
// Reference semantics restated here: SkipConnMLP.forward (neural_blocks.py:75-86) with the
// fourier2 encoding (utils.py:37-40).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

namespace nrt {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));

// address-space qualifiers: uniform tables through the scalar cache, streams as global loads
#define NRT_GLOBAL __attribute__((address_space(1)))
#define NRT_CONST __attribute__((address_space(4)))

constexpr int kMaxLin = 20;  // init + up to 18 hidden + out

// Row blocks (of 32 output rows) per hidden-layer chunk of the FP16 ring stream (MlpDev::stream16):
// two independent MFMA chains per chunk, half the block barriers of one-row-block chunks.
#ifndef NRT_RING_RB
#define NRT_RING_RB 2
#endif
constexpr int kRingRB = NRT_RING_RB;

enum { ACT_LEAKY = 0, ACT_SOFTPLUS = 1, ACT_NONE = 2, ACT_SIGMOID = 3, ACT_RELU = 4 };

// Device descriptor of a packed SkipConnMLP (built by nrt_mlp_create, lives in device memory).
//
// Encoding slot order (both paths): slot 2q / 2q+1 = sin / cos of projection q (q < F), then the
// raw inputs x_0..x_{in-1}, then the latent, then zero padding up to `ke` (multiple of 16).
// The packer maps slots back to the reference's column order [x, sin(xB), cos(xB), latent].
struct MlpDev {
  int in_size, hidden, n_hidden, out, freqs, skip, latent, act;
  int dp;   // in + 2F + latent (reference encoding width)
  int ke;   // encoding slots, padded to 16
  int nb;   // hidden / 32
  int ob;   // ceil(out / 32)
  const float* basis;              // [in][F]
  const h8* w16[kMaxLin];          // FP16 A fragments  [kstep][rowblock][64 lanes]
  const float* w32[kMaxLin];       // FP32 A fragments  [kstep][rowblock][64 lanes]
  const float* wt32[kMaxLin];      // FP32 A fragments of W^T (backward)
  const float* bias[kMaxLin];      // [rowblocks*32]
  const float* wout_row0;          // out.weight[0, :]  (gradient seed of an SDF head)
  int nbt[kMaxLin];                // row blocks of W^T (input positions / 32, rounded up)
  // FP16 weight stream for the block-cooperative LDS-ring engine (row-block-major chunks):
  // chunk (layer l, row block ib) = the nks(l) A fragments of that row block, contiguous.
  // Softplus MLPs are folded into the log2 domain: z' = log2e * z, a' = log2(1 + 2^z'), so the
  // init layer's W and every init/hidden bias carry a log2e factor and out.weight carries ln2.
  const h8* stream16;              // [frags (+ zero tail)][64 lanes]
  int stream16_bytes;              // buffer range of stream16 (loads past it return zeros)
  const int* chunk_off;            // first fragment of each chunk
  int n_chunks;
  const float* bias16;             // [layer][bias16_stride] (folded like stream16)
  int bias16_stride;               // max(nb, ob) * 32
  int fold;                        // 1 when softplus was folded
  // FP16 k-outer stream for the program engine (shading MLPs): layer by layer, chunks of kc
  // consecutive k-steps x all row blocks ([kstep][rowblock][64 lanes], kc = 16 / nb), same
  // fragments as w16 (never folded).
  const h8* streamk16;
  const int* chunkk_off;           // per chunk, fragment offset within streamk16
  int nk_chunks;
  int kc;
  int nk_frags;                    // fragments in streamk16 (without tail)
  // FP32 weight stream of the FP32 ring engine (ring32, v_mfma_f32_16x16x4_f32 on 16-ray
  // tiles): chunks of 32 output rows in consumption order, unfolded weights (exact FP32
  // arithmetic); element order in nrt_internal.h ring32_walk.
  const float4* stream32;
  int stream32_bytes;
  const float* bias32;             // [layer][bias16_stride], unfolded
  // FP32-accurate split stream of the ring3 engine (nrt_ring3.h): every weight of layer l (folded
  // into the log2 domain for softplus MLPs, as stream16) as
  // W 2^s_l = hi + lo, two f16 (hi = RNE(W 2^s_l), lo = RNE(W 2^s_l - hi)), fragments of
  // v_mfma_f32_16x16x32_f16 on 16-ray tiles in consumption order (nrt_internal.h ring3_walk);
  // s_l puts the layer's largest |W| in [1, 2) so lo stays a normal f16 for all but the smallest
  // weights.  bias3 = bias 2^s_l (the accumulator's initial value), scale3[l] = 2^-s_l.
  const float4* stream3;
  int stream3_bytes;
  const float* bias3;              // [layer][bias16_stride]
  float scale3[kMaxLin];
  int ke3;                         // encoding slots padded to 32 (one f16 k-step)
};

// A shading "program": the MLPs one kernel evaluates per ray batch, concatenated into one
// k-outer weight stream so the LDS ring prefetches across MLP boundaries.
constexpr int kMaxProgMlp = 40;
struct ProgMlp {
  int nb, ne, ob, L, skip, out, act, F;
  int bias_off;      // floats into ProgDev::bias (layer stride bstride)
  int bstride;
  int basis_off;     // float4 index into ProgDev::basis
  int chunk0;        // first chunk of this MLP in the program
};
struct ProgDev {
  const h8* stream;        // [frags + tail][64 lanes]
  const int* coff;         // per chunk, fragment offset
  int n_chunks;
  const float* bias;       // all MLPs' biases [mlp][layer][bstride]
  int bias_floats;
  const float4* basis;     // all MLPs' (B0q, B1q, B2q, 0)
  int basis_q;
  int n_mlp;
  ProgMlp mlp[kMaxProgMlp];
};

// A "row program" (nrt_shade_ring.h): shading MLPs evaluated one after another per 16-ray tile by
// the FP32 / fp32-split ring engines; concatenated weight streams, a chunk table driving the
// LDS-DMA, and biases / split scales / bases copied to LDS.
struct RProgMlp {
  int L, skip, F, out;
  int bias_off;      // floats into RProgDev::tables (layer stride bstride)
  int bstride;
  int basis_off;     // float4 index into RProgDev::basis
  int scale_off;     // floats into RProgDev::tables: 2^-s per layer (split; 1 for FP32)
};
struct RProgDev {
  const void* stream;      // all MLPs' streams, in evaluation order
  int stream_bytes;
  const int* chunks;       // [n_chunks][2]: KiB offset, KiB count, in evaluation order
  int n_chunks;
  const float* tables;     // biases | scales
  int table_floats;
  const float4* basis;
  int basis_q;
  int n_mlp;
  RProgMlp mlp[kMaxProgMlp];
};

struct SdfDev {
  int kind;         // 0 unit sphere, 1 MLP, 2 sphere blob (+ optional shift MLP)
  int n_spheres;
  float k;          // smooth-min sharpness (32)
  const float* spheres;  // [n][16]: (I+tfs) row-major (9), centre (3), radius (1), pad (3)
  const MlpDev* mlp;     // MLP or shift MLP (nullptr if none)
  int nb;
};

// ------------------------------------------------------------------------------------------
// small helpers
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

__device__ __forceinline__ bool wave_any(bool p) { return __ballot(p) != 0ull; }

// compiler-only fence: keeps LDS writes and the following cross-lane reads of one wave in
// program order (a wave's DS instructions execute in order in hardware)
__device__ __forceinline__ void wave_lds_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// F.softplus (beta 1, threshold 20) in FP32 on the hardware transcendentals: max(x, 0) +
// log1p(e), e = exp(-|x|) in (0, 1], with log1p(e) = log(u) e / (u - 1), u = fl(1 + e) -- the
// classic compensation of the rounding of 1 + e (Goldberg), accurate to a few ulp with the ~1-ulp
// v_exp / v_log / v_rcp.  ~12 VALU against ~100 for ocml's log1pf(expf(x)) (double-float
// arithmetic), which left the FP32 march VALU-bound (one chunk's activations cost as much issue
// time as its 128 MFMAs) and most of the SDF shift backward's issue time.  Every FP32 softplus of
// the library uses it (act_fwd<false>: the generic k_mlp_forward / backward too), so the FP32
// paths are not bit-equal to torch's log1pf(expf(x)) but within a few ulp per activation; the
// parity suite holds them at the 1e-4 bar against the oracle (measured: max 4.5e-8 on the smoke
// crop, 0 hit / step flips on the ring32 march configurations, tests/test_gpu_ring32.py).
//
// Round 6: the compensation is additive, log1p(e) = log(u) + c / u with c = e - (u - 1) the exact
// rounding error of u, and 1/u taken as 1.5 - u/2 (exact at u = 1 and 2, within 12 % between:
// c <= 2^-24 u, so that error stays far below an ulp of the result; e < 2^-24 gives u = 1, c = e).
// One transcendental (v_rcp) and two compare / selects fewer than Goldberg's ratio form, the same
// accuracy (float32 emulation over x in [-30, 20] and 1e6 N(0, 5) samples against float64
// log1p(exp(x)): max 4.8e-7 absolute, mean 2.1 ulp, both forms).  Measured (timing-only variant,
// softplus -> max(x, 0)): the FP32 ring march spends 12 % (8x256) / 17 % (8x128) of its time in
// the softplus VALU -- on gfx950 the f32 MFMA and the VALU of the two waves of a SIMD do not
// overlap fully, so VALU cuts show up as time.
// torch's threshold (x > 20 -> x) needs no select: there e < 2.1e-9, below half an ulp of x, so
// max(x, 0) + log1p(e) rounds to x exactly (and +-inf / NaN come out as torch's).
__device__ __forceinline__ float softplus_exact(float x) {
  const float kLog2e = 1.4426950408889634f, kLn2 = 0.6931471805599453f;
  const float e = __builtin_amdgcn_exp2f(fabsf(x) * -kLog2e);
  const float u = 1.f + e;
  const float c = e - (u - 1.f);
  const float l1p = fmaf(__builtin_amdgcn_logf(u), kLn2, c * fmaf(-0.5f, u, 1.5f));
  return fmaxf(x, 0.f) + l1p;
}

typedef float f2v __attribute__((ext_vector_type(2)));
// softplus_exact on two elements: the same IEEE operations, the non-transcendental ones as packed
// f32 (v_pk_mul / v_pk_add / v_pk_fma_f32, two elements an instruction): the same bits
__device__ __forceinline__ f2v softplus_exact2(f2v x) {
  const float kLog2e = 1.4426950408889634f, kLn2 = 0.6931471805599453f;
  const f2v one = {1.f, 1.f};
  const f2v ax = {fabsf(x[0]), fabsf(x[1])};
  const f2v t = ax * f2v{-kLog2e, -kLog2e};
  const f2v e = {__builtin_amdgcn_exp2f(t[0]), __builtin_amdgcn_exp2f(t[1])};
  const f2v u = one + e;
  const f2v c = e - (u - one);
  const f2v r = __builtin_elementwise_fma(f2v{-0.5f, -0.5f}, u, f2v{1.5f, 1.5f});
  const f2v lg = {__builtin_amdgcn_logf(u[0]), __builtin_amdgcn_logf(u[1])};
  const f2v l1p = __builtin_elementwise_fma(lg, f2v{kLn2, kLn2}, c * r);
  const f2v m = {fmaxf(x[0], 0.f), fmaxf(x[1], 0.f)};
  return m + l1p;
}

// torch semantics: F.leaky_relu (slope 0.01), F.softplus (beta 1, threshold 20), sigmoid, relu
template <bool FAST>
__device__ __forceinline__ float act_fwd(float x, int act) {
  switch (act) {
    case ACT_LEAKY: return x > 0.f ? x : x * 0.01f;
    case ACT_SOFTPLUS:
      if (FAST) return x > 20.f ? x : __logf(1.f + __expf(x));
      return softplus_exact(x);
    case ACT_SIGMOID:
      return FAST ? 1.f / (1.f + __expf(-x)) : 1.f / (1.f + expf(-x));
    case ACT_RELU: return x > 0.f ? x : 0.f;
    default: return x;
  }
}

// derivative of act at pre-activation x (torch backward formulas)
__device__ __forceinline__ float act_bwd(float x, int act) {
  switch (act) {
    case ACT_LEAKY: return x > 0.f ? 1.f : 0.01f;
    case ACT_SOFTPLUS: {
      if (x > 20.f) return 1.f;
      float z = expf(x);
      return z / (z + 1.f);
    }
    case ACT_SIGMOID: {
      float s = 1.f / (1.f + expf(-x));
      return s * (1.f - s);
    }
    case ACT_RELU: return x > 0.f ? 1.f : 0.f;
    default: return 1.f;
  }
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + expf(-x)); }

// F.normalize(v, eps): v / max(|v|, eps)
__device__ __forceinline__ void normalize3(float& x, float& y, float& z, float eps) {
  float n = sqrtf(x * x + y * y + z * z);
  n = fmaxf(n, eps);
  x = x / n; y = y / n; z = z / n;
}

// ------------------------------------------------------------------------------------------
// Encoding
// ------------------------------------------------------------------------------------------
// Input of one MLP evaluation for this lane's ray: up to 4 inputs in registers, or a pointer to
// a row in global memory (inputs wider than 4, e.g. NeRFLE's second MLP).
struct EncIn {
  float x[4];
  const float* xg;   // row pointer when in_size > 4, else nullptr
  const float* lat;  // latent row or nullptr
};

template <bool FAST>
__device__ __forceinline__ float proj(const MlpDev& m, const EncIn& e, int q) {
  const float* B = m.basis;
  const int F = m.freqs;
  float s = 0.f;
  if (e.xg == nullptr) {
    // x @ B for in_size <= 4 (utils.py:39); same k order as a BLAS dot of length in
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (i < m.in_size) s = (i == 0) ? e.x[0] * B[q] : fmaf(e.x[i], B[i * F + q], s);
  } else {
    for (int i = 0; i < m.in_size; ++i) s = (i == 0) ? e.xg[0] * B[q] : fmaf(e.xg[i], B[i * F + q], s);
  }
  return s;
}

template <bool FAST>
__device__ __forceinline__ void sincos_(float a, float& s, float& c) {
  if (FAST) { s = __sinf(a); c = __cosf(a); }
  else sincosf(a, &s, &c);
}

// value of the raw (non-sin/cos) encoding slot: inputs, latent, zero padding
__device__ __forceinline__ float enc_plain(const MlpDev& m, const EncIn& e, int slot) {
  int i = slot - 2 * m.freqs;
  if (i < m.in_size) {
    if (e.xg) return e.xg[i];
    float v = e.x[0];
    v = (i == 1) ? e.x[1] : v;
    v = (i == 2) ? e.x[2] : v;
    v = (i == 3) ? e.x[3] : v;
    return v;
  }
  i -= m.in_size;
  if (i < m.latent && e.lat) return e.lat[i];
  return 0.f;
}

// two adjacent slots (2q, 2q+1) starting at an even slot
template <bool FAST>
__device__ __forceinline__ void enc_pair(const MlpDev& m, const EncIn& e, int slot, float& a,
                                         float& b) {
  if (slot < 2 * m.freqs) {
    sincos_<FAST>(proj<FAST>(m, e, slot >> 1), a, b);
  } else {
    a = enc_plain(m, e, slot);
    b = enc_plain(m, e, slot + 1);
  }
}

// ------------------------------------------------------------------------------------------
// FP16 register path
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ f16v mfma16(h8 a, h8 b, f16v c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

// acc[reg] = bias[32*blk + (reg&3) + 8*(reg>>2) + 4*h]
__device__ __forceinline__ f16v bias_tile(const float* __restrict__ bias, int blk, int h) {
  f16v v;
  const float* b = bias + 32 * blk + 4 * h;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    float4 q = *reinterpret_cast<const float4*>(b + 8 * g);
    v[4 * g + 0] = q.x; v[4 * g + 1] = q.y; v[4 * g + 2] = q.z; v[4 * g + 3] = q.w;
  }
  return v;
}

// B fragment of encoding k-step s (slots 16s + 8h + j), optionally through the activation
template <bool FAST>
__device__ __forceinline__ h8 enc_frag16(const MlpDev& m, const EncIn& e, int s, int h, int act) {
  h8 f;
  const int base = 16 * s + 8 * h;
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) {
    float a, b;
    enc_pair<FAST>(m, e, base + 2 * jj, a, b);
    if (act >= 0) { a = act_fwd<FAST>(a, act); b = act_fwd<FAST>(b, act); }
    f[2 * jj] = (_Float16)a;
    f[2 * jj + 1] = (_Float16)b;
  }
  return f;
}

template <int NB>
__device__ __forceinline__ void act_to_frags(const f16v (&acc)[NB], h8 (&hb)[2 * NB], int act) {
#pragma unroll
  for (int ib = 0; ib < NB; ++ib)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      h8 f;
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = (_Float16)act_fwd<true>(acc[ib][8 * s2 + j], act);
      hb[2 * ib + s2] = f;
    }
}

// Full SkipConnMLP forward for the wave's 32 rays.  Output rows < m.out are written to
// y[r * ystride + row] (LDS or global, f32).
template <int NB>
__device__ __forceinline__ void mlp16_forward(const MlpDev& m, const EncIn& e, float* __restrict__ y, int ystride) {
  const int lane = lane_id();
  const int r = lane & 31, h = lane >> 5;
  const int neb = m.ke >> 4;
  f16v acc[NB];
  h8 hb[2 * NB];

  // init layer: raw encoding in, no activation (neural_blocks.py:80)
#pragma unroll
  for (int ib = 0; ib < NB; ++ib) acc[ib] = bias_tile(m.bias[0], ib, h);
  {
    const h8* __restrict__ A = m.w16[0] + lane;
    for (int s = 0; s < neb; ++s) {
      h8 b = enc_frag16<true>(m, e, s, h, -1);
#pragma unroll
      for (int ib = 0; ib < NB; ++ib) acc[ib] = mfma16(A[(s * NB + ib) * 64], b, acc[ib]);
    }
  }
  // hidden layers: x = layer(act(cat[x, enc] if skip else x))   (neural_blocks.py:81-84)
  for (int i = 0; i < m.n_hidden; ++i) {
    act_to_frags<NB>(acc, hb, m.act);
#pragma unroll
    for (int ib = 0; ib < NB; ++ib) acc[ib] = bias_tile(m.bias[1 + i], ib, h);
    const h8* __restrict__ A = m.w16[1 + i] + lane;
#pragma unroll
    for (int s = 0; s < 2 * NB; ++s)
#pragma unroll
      for (int ib = 0; ib < NB; ++ib) acc[ib] = mfma16(A[(s * NB + ib) * 64], hb[s], acc[ib]);
    if (i != m.n_hidden - 1 && (i % m.skip) == 0) {
      A += 2 * NB * NB * 64;
      for (int s = 0; s < neb; ++s) {
        h8 b = enc_frag16<true>(m, e, s, h, m.act);
#pragma unroll
        for (int ib = 0; ib < NB; ++ib) acc[ib] = mfma16(A[(s * NB + ib) * 64], b, acc[ib]);
      }
    }
  }
  act_to_frags<NB>(acc, hb, m.act);
  // out layer (neural_blocks.py:86)
  const float* __restrict__ bo = m.bias[m.n_hidden + 1];
  const h8* __restrict__ A = m.w16[m.n_hidden + 1] + lane;
  for (int ob = 0; ob < m.ob; ++ob) {
    f16v o = bias_tile(bo, ob, h);
#pragma unroll
    for (int s = 0; s < 2 * NB; ++s) o = mfma16(A[(s * m.ob + ob) * 64], hb[s], o);
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      int row = 32 * ob + (reg & 3) + 8 * (reg >> 2) + 4 * h;
      if (row < m.out) y[r * ystride + row] = o[reg];
    }
  }
}

// ------------------------------------------------------------------------------------------
// FP32 LDS path
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ f16v mfma32(float a, float b, f16v c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// LDS row stride (floats) of the per-wave activation slab: hidden | enc | [enc grad]
__host__ __device__ inline int slab_stride(int hidden, int ke, bool with_grad) {
  int rs = hidden + ke + (with_grad ? ke : 0);
  return rs | 1;  // odd stride: 32 lanes of a ds_read_b32 hit 32 different banks
}

template <bool FAST>
__device__ __forceinline__ void write_enc_slab(const MlpDev& m, const EncIn& e, float* X, int RS) {
  const int lane = lane_id();
  const int r = lane & 31, h = lane >> 5;
  float* row = X + r * RS + m.hidden;
  // the two lane halves share the pairs: half h takes pairs 2h, 2h+4, ...  (slots multiple of 4)
  for (int slot = 2 * h; slot < m.ke; slot += 4) {
    float a, b;
    enc_pair<FAST>(m, e, slot, a, b);
    row[slot] = a;
    row[slot + 1] = b;
  }
}

// One FP32 GEMM over `nks` k-steps of the slab starting at column kcol; accumulates into acc.
// act_in >= 0 applies the activation to B on the fly (skip-concat of the encoding).
// The A fragments are read through a global-address-space pointer (generic "flat" loads also
// count in lgkmcnt, so the slab's ds_read waits drained them) and prefetched PF - 1 k-steps
// ahead through PF rotating buffers: a k-step's wait covers only loads issued PF - 1 steps
// earlier.  PF = 2 is the ping-pong of the occupancy-rich kernels; the training kernels run one
// wave per SIMD and hide the L2 latency with PF = 4.
template <int NB, int PF = 2>
__device__ __forceinline__ void gemm32(f16v (&acc)[NB], const float* __restrict__ A, int nrb,
                                       int rb0, int nks, const float* X, int RS, int kcol,
                                       int act_in) {
  using gptr = const __attribute__((address_space(1))) float*;
  if (nks <= 0) return;
  const int lane = lane_id();
  const int r = lane & 31, h = lane >> 5;
  const float* xr = X + r * RS + kcol + h;
  const gptr Ag = (gptr)(A + (size_t)rb0 * 64 + lane);
  const int stride = nrb * 64;
  // loads are unconditional (clamped row block / k-step) so the compiler counts them exactly
  int off[NB];
#pragma unroll
  for (int ib = 0; ib < NB; ++ib) off[ib] = (rb0 + ib < nrb ? ib : nrb - 1 - rb0) * 64;
  // rotating fragment buffers (no register copies, which would wait for the prefetch)
  float a[PF][NB];
#pragma unroll
  for (int p = 0; p < PF; ++p)
#pragma unroll
    for (int ib = 0; ib < NB; ++ib) a[p][ib] = Ag[(size_t)(p < nks ? p : nks - 1) * stride + off[ib]];
  auto step = [&](const float (&av)[NB], int s) {
    float b = xr[2 * s];
    if (act_in >= 0) b = act_fwd<false>(b, act_in);
#pragma unroll
    for (int ib = 0; ib < NB; ++ib)
      if (rb0 + ib < nrb) acc[ib] = mfma32(av[ib], b, acc[ib]);
  };
  int s = 0;
  for (; s + PF <= nks; s += PF) {
#pragma unroll
    for (int p = 0; p < PF; ++p) {
      step(a[p], s + p);
      const int sn = s + p + PF < nks ? s + p + PF : nks - 1;
#pragma unroll
      for (int ib = 0; ib < NB; ++ib) a[p][ib] = Ag[(size_t)sn * stride + off[ib]];
    }
  }
#pragma unroll
  for (int p = 0; p < PF; ++p)
    if (s + p < nks) step(a[p], s + p);
}

// gemm32 with B from a per-wave global tile T[slot][32 rows] (coalesced: a k-step reads two
// 128-byte rows) instead of the LDS slab; B is prefetched with the A fragments.
// Used by k_mlp_backward32 to keep the encoding out of LDS.
template <int NB, int PF = 2>
__device__ __forceinline__ void gemm32_tile(f16v (&acc)[NB], const float* __restrict__ A, int nrb,
                                            int rb0, int nks, const float* T, int act_in) {
  using gptr = const __attribute__((address_space(1))) float*;
  if (nks <= 0) return;
  const int lane = lane_id();
  const int r = lane & 31, h = lane >> 5;
  const gptr Bg = (gptr)(T + h * 32 + r);
  const gptr Ag = (gptr)(A + (size_t)rb0 * 64 + lane);
  const int stride = nrb * 64;
  int off[NB];
#pragma unroll
  for (int ib = 0; ib < NB; ++ib) off[ib] = (rb0 + ib < nrb ? ib : nrb - 1 - rb0) * 64;
  float a[PF][NB], bb[PF];
#pragma unroll
  for (int p = 0; p < PF; ++p) {
    const int sp = p < nks ? p : nks - 1;
#pragma unroll
    for (int ib = 0; ib < NB; ++ib) a[p][ib] = Ag[(size_t)sp * stride + off[ib]];
    bb[p] = Bg[sp * 64];
  }
  auto step = [&](const float (&av)[NB], float b) {
    if (act_in >= 0) b = act_fwd<false>(b, act_in);
#pragma unroll
    for (int ib = 0; ib < NB; ++ib)
      if (rb0 + ib < nrb) acc[ib] = mfma32(av[ib], b, acc[ib]);
  };
  int s = 0;
  for (; s + PF <= nks; s += PF) {
#pragma unroll
    for (int p = 0; p < PF; ++p) {
      step(a[p], bb[p]);
      const int sn = s + p + PF < nks ? s + p + PF : nks - 1;
#pragma unroll
      for (int ib = 0; ib < NB; ++ib) a[p][ib] = Ag[(size_t)sn * stride + off[ib]];
      bb[p] = Bg[sn * 64];
    }
  }
#pragma unroll
  for (int p = 0; p < PF; ++p)
    if (s + p < nks) step(a[p], bb[p]);
}

template <int NB>
__device__ __forceinline__ void bias32(f16v (&acc)[NB], const float* bias, int rb0, int nrb, int h) {
#pragma unroll
  for (int ib = 0; ib < NB; ++ib)
    if (rb0 + ib < nrb) acc[ib] = bias_tile(bias, rb0 + ib, h);
}

// Forward through the FP32 slab.  If zs != nullptr the pre-activations of the init layer and
// of every hidden layer are stored to zs[(layer*32 + r)*hidden + row] for the backward pass.
template <int NB>
__device__ __forceinline__ void mlp32_forward(const MlpDev& m, const EncIn& e, float* X, int RS,
                              float* __restrict__ y, int ystride, float* __restrict__ zs) {
  const int lane = lane_id();
  const int r = lane & 31, h = lane >> 5;
  const int H = m.hidden;
  write_enc_slab<false>(m, e, X, RS);
  wave_lds_fence();
  f16v acc[NB];
  for (int l = 0; l <= m.n_hidden; ++l) {
    bias32<NB>(acc, m.bias[l], 0, NB, h);
    if (l == 0) {
      gemm32<NB>(acc, m.w32[0], NB, 0, m.ke >> 1, X, RS, H, -1);
    } else {
      const int i = l - 1;
      gemm32<NB>(acc, m.w32[l], NB, 0, H >> 1, X, RS, 0, -1);
      if (i != m.n_hidden - 1 && (i % m.skip) == 0)
        gemm32<NB>(acc, m.w32[l] + (H >> 1) * NB * 64, NB, 0, m.ke >> 1, X, RS, H, m.act);
    }
    wave_lds_fence();
#pragma unroll
    for (int ib = 0; ib < NB; ++ib)
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        int row = 32 * ib + (reg & 3) + 8 * (reg >> 2) + 4 * h;
        float z = acc[ib][reg];
        if (zs) zs[(l * 32 + r) * H + row] = z;
        X[r * RS + row] = act_fwd<false>(z, m.act);
      }
    wave_lds_fence();
  }
  // out layer
  const float* Ao = m.w32[m.n_hidden + 1];
  for (int ob = 0; ob < m.ob; ++ob) {
    f16v o[1];
    o[0] = bias_tile(m.bias[m.n_hidden + 1], ob, h);
    // k-steps over hidden; A is [s][ob][64] (row block ob of m.ob), prefetched like the hidden layers
    gemm32<1>(o, Ao, m.ob, ob, H >> 1, X, RS, 0, -1);
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      int row = 32 * ob + (reg & 3) + 8 * (reg >> 2) + 4 * h;
      if (row < m.out) y[r * ystride + row] = o[0][reg];
    }
  }
  wave_lds_fence();
}

// d out[0] / d x for the wave's rays, after mlp32_forward(..., zs) on the same slab.
// Returns the gradient with respect to the first min(in_size, 3) inputs in g[0..2].
template <int NB>
__device__ __forceinline__ void mlp32_backward_out0(const MlpDev& m, const EncIn& e, float* X, int RS,
                                    const float* __restrict__ zs, float g[3]) {
  const int lane = lane_id();
  const int r = lane & 31, h = lane >> 5;
  const int H = m.hidden;
  const int ke = m.ke;
  float* row = X + r * RS;
  float* egrad = row + H + ke;
  for (int s = h; s < ke; s += 2) egrad[s] = 0.f;
  // seed: dy/dh_last = W_out[0,:] * act'(z_last)
  const float* zl = zs + (m.n_hidden * 32 + r) * H;
  for (int k = h; k < H; k += 2) row[k] = m.wout_row0[k] * act_bwd(zl[k], m.act);
  wave_lds_fence();
  f16v acc[NB];
  for (int l = m.n_hidden; l >= 0; --l) {
    const float* At = m.wt32[l];
    const int nrb = m.nbt[l];
    const bool has_hidden_in = (l != 0);
    const bool has_enc_in = (l == 0) || ((l - 1) != m.n_hidden - 1 && ((l - 1) % m.skip) == 0);
    const int hid_rb = has_hidden_in ? NB : 0;
    // encoding positions first (they only accumulate), hidden block group last (in place)
    if (has_enc_in) {
      const int enc_pos0 = has_hidden_in ? H : 0;
      for (int rb0 = hid_rb; rb0 < nrb; rb0 += NB) {
#pragma unroll
        for (int ib = 0; ib < NB; ++ib) acc[ib] = f16v{};
        gemm32<NB>(acc, At, nrb, rb0, H >> 1, X, RS, 0, -1);
#pragma unroll
        for (int ib = 0; ib < NB; ++ib) {
          if (rb0 + ib >= nrb) continue;
#pragma unroll
          for (int reg = 0; reg < 16; ++reg) {
            int pos = 32 * (rb0 + ib) + (reg & 3) + 8 * (reg >> 2) + 4 * h;
            int slot = pos - enc_pos0;
            if (slot >= 0 && slot < ke) {
              float v = acc[ib][reg];
              // skip inputs are act(enc) (neural_blocks.py:84); the init input is raw enc
              if (l != 0) v *= act_bwd(row[H + slot], m.act);
              egrad[slot] += v;
            }
          }
        }
      }
      wave_lds_fence();
    }
    if (has_hidden_in) {
#pragma unroll
      for (int ib = 0; ib < NB; ++ib) acc[ib] = f16v{};
      gemm32<NB>(acc, At, nrb, 0, H >> 1, X, RS, 0, -1);
      wave_lds_fence();
      const float* zp = zs + ((l - 1) * 32 + r) * H;
#pragma unroll
      for (int ib = 0; ib < NB; ++ib)
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
          int pos = 32 * ib + (reg & 3) + 8 * (reg >> 2) + 4 * h;
          row[pos] = acc[ib][reg] * act_bwd(zp[pos], m.act);
        }
      wave_lds_fence();
    }
  }
  // encoding -> input:  d sin(xB_q) = cos(xB_q) B_q,  d cos(xB_q) = -sin(xB_q) B_q,  d x_i = e_i
  float gx[3] = {0.f, 0.f, 0.f};
  const int F = m.freqs;
  for (int q = h; q < F; q += 2) {
    float s, c;
    sincosf(proj<false>(m, e, q), &s, &c);
    float w = egrad[2 * q] * c - egrad[2 * q + 1] * s;
#pragma unroll
    for (int i = 0; i < 3; ++i)
      if (i < m.in_size) gx[i] = fmaf(w, m.basis[i * F + q], gx[i]);
  }
  if (h == 0) {
#pragma unroll
    for (int i = 0; i < 3; ++i)
      if (i < m.in_size) gx[i] += egrad[2 * F + i];
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) g[i] = gx[i] + __shfl_xor(gx[i], 32);
  wave_lds_fence();
}

}  // namespace nrt

// ------------------------------------------------------------------------------------------
// FP16 block-cooperative engine: LDS weight ring shared by the WV waves of a block
// ------------------------------------------------------------------------------------------
// Every wave of the block evaluates the same MLP at the same time for its own 32 rays.  The
// weight stream (MlpDev::stream16) is consumed chunk by chunk, one chunk = one 32-row output
// block of one layer (row-block-outer order: only one accumulator tile is live, and the
// activation of tile ib overlaps the MFMAs of tile ib+1).  Chunks are staged through a 3-slot
// LDS ring: at chunk c a wave writes the fragments it loaded during chunk c-1 (chunk c+1) to
// LDS, issues its global loads for chunk c+2 into registers, then runs chunk c's MFMAs with A
// read by ds_read_b128 from LDS; one barrier per chunk.  Loads and stores are unconditional
// (fixed count per wave; slots are padded) so hipcc never drains vmcnt inside the loop.
namespace nrt {
namespace ring {

__device__ __forceinline__ float sp2(float x) {
  // softplus in the log2 domain, log2(1 + 2^x), as exp + add + log (20 issue cycles, 3 VALU per
  // element: one MFMA gap holds one element's activation).  Against max(x,0) + log2(1 + 2^-|x|)
  // the only loss is below the f16 the result is rounded to: 1 + 2^x rounds to 1 for x < -24
  // (true value < 9e-8) and 2^x overflows for x >= 128 (a natural pre-activation above 88),
  // which the FP16 path does not support; the FP32 path keeps torch's exact form.
  return __builtin_amdgcn_logf(1.f + __builtin_amdgcn_exp2f(x));
}

// Sphere blob part of a SphereSDF (sdfs.py:37-43, utils.py:386-387) for a 32-ray tile: the two
// lanes of a ray (l, l + 32) sum exp(-k d_i) over the even / odd spheres from the LDS table and
// add the halves (commutative: both lanes get the same bits) -- half the VALU of every lane
// walking the whole table.  FP16-path math: fast exp, as spheres_value<true>.
// The FP16 march's SphereSDF table in LDS as sphere PAIRS for packed-f32 VALU (v_pk_fma_f32 /
// v_pk_mul_f32 handle two spheres per instruction): record 2 j + h holds spheres h + 4 j and
// h + 4 j + 2 (the two lanes of a ray, h = lane >> 5, split the spheres by parity), as 13 float2
// (m00 m01 m02 m10 m11 m12 m20 m21 m22 cx cy cz, c) + pad = 7 float4, where c = k log2(e) r puts
// the radius into the exponent: exp(-k (|q| - r)) = exp2(-k log2(e) |q| + c).  A missing second
// sphere has c = -inf (exp2 -> 0).
constexpr int kSpherePairF4 = 7;
__host__ __device__ inline int sphere_pair_records(int n) {
  const int pairs = ((n + 1) / 2 + 1) / 2;  // pairs of the half with more spheres (h = 0)
  return 2 * pairs;
}
__device__ __forceinline__ void build_sphere_pairs(const SdfDev& s, float4* out) {
  const int n = s.n_spheres, R = sphere_pair_records(n);
  const float kl = s.k * 1.4426950408889634f;
  const float4* src = reinterpret_cast<const float4*>(s.spheres);
  for (int rec = threadIdx.x; rec < R; rec += blockDim.x) {
    const int h = rec & 1, j = rec >> 1;
    float v[2][13];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = h + 4 * j + 2 * u;
      if (i < n) {
        const float4 r0 = src[4 * i], r1 = src[4 * i + 1], r2 = src[4 * i + 2], r3 = src[4 * i + 3];
        const float m[13] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w, r2.x, r2.y, r2.z, r2.w,
                             kl * r3.x};
        for (int k = 0; k < 13; ++k) v[u][k] = m[k];
      } else {
        for (int k = 0; k < 12; ++k) v[u][k] = 0.f;
        v[u][12] = -__builtin_inff();
      }
    }
    float* o = reinterpret_cast<float*>(out + rec * kSpherePairF4);
    for (int k = 0; k < 13; ++k) { o[2 * k] = v[0][k]; o[2 * k + 1] = v[1][k]; }
    o[26] = 0.f; o[27] = 0.f;
  }
}

// FP16-path sphere smooth-min over the pair table (the FP16 march's SDF precision: fast v_sqrt,
// fused arithmetic, pairwise sums -- ~10 VALU per sphere instead of ~30); the two lanes of a
// ray sum their spheres and combine with one cross-half add
__device__ __forceinline__ float spheres_value_pairs(const SdfDev& s, const float4* sp, int lane,
                                                     float x, float y, float z) {
  const int h = lane >> 5, R = sphere_pair_records(s.n_spheres);
  const f2v xx = {x, x}, yy = {y, y}, zz = {z, z};
  const float nkl = -s.k * 1.4426950408889634f;
  const f2v nk2 = {nkl, nkl};
  f2v acc = {0.f, 0.f};
  for (int rec = h; rec < R; rec += 2) {
    const float4* q = sp + rec * kSpherePairF4;
    const float4 a = q[0], b = q[1], c = q[2], d = q[3], e = q[4], f = q[5], g = q[6];
    const f2v m00 = {a.x, a.y}, m01 = {a.z, a.w}, m02 = {b.x, b.y}, m10 = {b.z, b.w};
    const f2v m11 = {c.x, c.y}, m12 = {c.z, c.w}, m20 = {d.x, d.y}, m21 = {d.z, d.w};
    const f2v m22 = {e.x, e.y}, cx = {e.z, e.w}, cy = {f.x, f.y}, cz = {f.z, f.w};
    const f2v cr = {g.x, g.y};
    const f2v qx = __builtin_elementwise_fma(m02, zz, __builtin_elementwise_fma(m01, yy, __builtin_elementwise_fma(m00, xx, -cx)));
    const f2v qy = __builtin_elementwise_fma(m12, zz, __builtin_elementwise_fma(m11, yy, __builtin_elementwise_fma(m10, xx, -cy)));
    const f2v qz = __builtin_elementwise_fma(m22, zz, __builtin_elementwise_fma(m21, yy, __builtin_elementwise_fma(m20, xx, -cz)));
    const f2v q2 = __builtin_elementwise_fma(qx, qx, __builtin_elementwise_fma(qy, qy, qz * qz));
    const f2v len = {__builtin_amdgcn_sqrtf(q2.x), __builtin_amdgcn_sqrtf(q2.y)};
    const f2v ex = __builtin_elementwise_fma(nk2, len, cr);
    const f2v w = {__builtin_amdgcn_exp2f(ex.x), __builtin_amdgcn_exp2f(ex.y)};
    acc += w;
  }
  float t = acc.x + acc.y;
  t += __shfl_xor(t, 32);
  return -logf(fmaxf(t, 1e-4f)) / s.k;
}

// Chunk schedule of one 8-layer (L hidden, skip period SK) evaluation, fixed at compile time:
// chunk 0 = the whole init layer (NB row blocks x NE encoding k-steps), chunk 1 + NB i + ib =
// row block ib of hidden layer i (2NB hidden k-steps, + NE encoding k-steps on skip layers),
// chunk NCH-1 = the out layer's row block.  The stream16 layout is exactly this order, so a
// chunk's first fragment is a prefix sum; every index below folds to a constant once eval()
// is unrolled, and each wave loads and stores only the fragments a chunk has.
template <int NB, int NE, int L, int SK>
struct Sched {
  static constexpr int RB = NB % kRingRB == 0 ? kRingRB : 1;  // row blocks per hidden chunk
  static constexpr int G = NB / RB;                             // hidden chunks per layer
  static constexpr int NCH = 2 + L * G;
  static constexpr bool skip(int i) { return i != L - 1 && i % SK == 0; }
  static constexpr int size(int c) {
    return c == 0 ? NB * NE : (c == NCH - 1 ? 2 * NB : RB * (2 * NB + (skip((c - 1) / G) ? NE : 0)));
  }
  // skip layers among hidden layers 0..i-1 (i <= L - 1, so layer L - 1 is never counted)
  static constexpr int skips_before(int i) { return (i + SK - 1) / SK; }
  // closed form (no loops: it must fold to a constant inside the unrolled evaluation)
  static constexpr int offset(int c) {
    if (c == 0) return 0;
    const int i = (c - 1) / G, j = (c - 1) % G;
    return NB * NE + i * 2 * NB * NB + NE * NB * skips_before(i) +
           (i < L ? j * RB * (2 * NB + (skip(i) ? NE : 0)) : 0);
  }
  static constexpr int max_size() {
    return NB * NE > RB * (2 * NB + NE) ? NB * NE : RB * (2 * NB + NE);
  }
};

#ifndef NRT_RING_DEPTH
#define NRT_RING_DEPTH (kRingRB > 1 ? 3 : 4)  // ring slots = chunks in flight + 1 (the one read)
#endif

template <int NB, int NE, int WV>
struct Cfg {
  using S = Sched<NB, NE, 8, 3>;
  static constexpr int D = NRT_RING_DEPTH;
  static constexpr int MAXF = S::max_size();              // fragments in the largest chunk
  static constexpr int MAXL = (MAXF + WV - 1) / WV;       // loads per wave per chunk
  static constexpr int SLOTF = MAXL * WV;                 // fragments per ring slot
  static constexpr int RING_BYTES = D * SLOTF * 1024;
  // ring SDFs have 3 inputs, no latent and F = 8 (NE - 1) frequencies (2F + 3 slots -> NE k-steps)
  static constexpr int F = 8 * (NE - 1);
  static constexpr int BASIS_BYTES = F * 16;  // float4 (B[0][q], B[1][q], B[2][q], 0) per q
  // LDS of one block: ring | basis | bias16
  static size_t lds_bytes(size_t bias_bytes) { return RING_BYTES + BASIS_BYTES + bias_bytes; }
  // LDS-DMA instructions one wave issues for chunk c
  static constexpr int loads(int c) { return (S::size(c % S::NCH) + WV - 1) / WV; }
};

// s_waitcnt vmcnt(n) lgkmcnt(0) (gfx9 encoding: vmcnt [3:0] + [15:14], expcnt [6:4] left at 7,
// lgkmcnt [11:8])
__device__ __forceinline__ constexpr int waitcnt_vm_lgkm0(int n) {
  return (n & 15) | (7 << 4) | (0 << 8) | ((n >> 4) << 14);
}
// f(integral_constant<int, 0>) ... f(integral_constant<int, N-1>): chunk indices that are
// C++ constants (waitcnt immediates, LDS offsets) in a straight-line evaluation
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  [&]<int... I>(std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
  }(std::make_integer_sequence<int, N>{});
}

// One 1-KiB LDS-DMA piece: lane l's 16 bytes at stream + soff + voff land at LDS m0 + 16 l.
// Written as asm so hipcc neither drains it with vmcnt(0) before every ring read (it cannot
// tell the DMA target from the slot being read) nor counts it: the engine waits for it itself.
// M0 is compiler-reserved, so it is saved and restored inside the statement.
__device__ __forceinline__ void lds_dma16(__amdgpu_buffer_rsrc_t srd, int voff, int soff,
                                          uint32_t lds_addr) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, %4 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(srd), "s"(lds_addr), "s"(soff));
}

template <int NB, int NE, int WV>
struct Engine {
  using C = Cfg<NB, NE, WV>;
  using S = typename C::S;
  static constexpr int D = C::D;
  h8* ring;                 // LDS [D][SLOTF][64]
  uint32_t ring_lds;        // LDS byte address of the ring
  const float* lbias;       // LDS copy of bias16
  const float4* lbasis;     // LDS copy of the Fourier basis, one float4 per frequency
  const float4* lspheres;   // LDS copy of the SphereSDF table (k_march16) or nullptr
  const void* sbase;        // FP16 weight stream (buffer base and range)
  int sbytes;
  int slot;                 // ring slot of the current chunk
  int lane, wv;

  // Wave wv moves fragments wv + WV q (q < loads) of a chunk by LDS-DMA.  Slots hold SLOTF =
  // MAXL * WV fragments, so in a chunk of n < SLOTF fragments the waves past the end load out
  // of the buffer's range (the lane offset is pushed past num_records = the stream's size: no
  // memory access) into the slot's unused tail: the count per wave is compile-time.
  static constexpr int kOutOfRange = 0x40000000;
  // piece q of chunk c into slot s (see issue())
  __device__ __forceinline__ void piece(int c, int s, int q) {
    const int w = __builtin_amdgcn_readfirstlane(wv);
    int base = w * 1024;
    asm volatile("" : "+s"(base));
    const int n = S::size(c % S::NCH);
    const int off = S::offset(c % S::NCH) * 1024 + base;
    const uint32_t dst = __builtin_amdgcn_readfirstlane(ring_lds + (uint32_t)(s * C::SLOTF * 1024)) + base;
    const uint64_t sp = (uint64_t)(uintptr_t)sbase;
    const uint64_t spu = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(sp >> 32)) << 32) |
                         (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)sp);
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(uintptr_t)spu, 0, __builtin_amdgcn_readfirstlane(sbytes), 0x00020000);
    const bool own = WV * (q + 1) <= n || w < n - WV * q;
    lds_dma16(r, own ? lane * 16 : kOutOfRange + lane * 16, off + WV * q * 1024, dst + WV * q * 1024);
  }
  // Spread the refill of chunk CH's predecessor slot over chunk CH's MFMA chain: call at every
  // MFMA index k < nm of the chunk; piece q goes out at k = (2q + 1) nm / (2 pieces).  Issuing
  // all pieces right after the barrier makes every wave of the block queue on the texture unit at
  // once, stalling their MFMA issue.
  template <int CH>
  __device__ __forceinline__ void dma_at(int k, int nm) {
    constexpr int c = CH + D - 1;
    const int pieces = C::loads(c);
#pragma unroll
    for (int q = 0; q < C::MAXL; ++q)
      if (q < pieces && k == (2 * q + 1) * nm / (2 * pieces)) piece(c, slot == 0 ? D - 1 : slot - 1, q);
  }
  __device__ __forceinline__ void issue(int c, int s) {
    // the asm wants SGPR operands: re-assert uniformity (inside the static_for lambdas hipcc
    // can lose track of it and would otherwise fail with "illegal VGPR to SGPR copy")
    const int w = __builtin_amdgcn_readfirstlane(wv);
    int base = w * 1024;
    asm volatile("" : "+s"(base));  // per-chunk s_add in place, not ~130 hoisted constants
    const int n = S::size(c % S::NCH);
    const int off = S::offset(c % S::NCH) * 1024 + base;
    const uint32_t dst = __builtin_amdgcn_readfirstlane(ring_lds + (uint32_t)(s * C::SLOTF * 1024)) + base;
    const uint64_t sp = (uint64_t)(uintptr_t)sbase;
    const uint64_t spu = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(sp >> 32)) << 32) |
                         (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)sp);
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(uintptr_t)spu, 0, __builtin_amdgcn_readfirstlane(sbytes), 0x00020000);
#pragma unroll
    for (int q = 0; q < C::MAXL; ++q)
      if (WV * q < n) {
        const bool own = WV * (q + 1) <= n || w < n - WV * q;
        lds_dma16(r, own ? lane * 16 : kOutOfRange + lane * 16, off + WV * q * 1024,
                  dst + WV * q * 1024);
      }
  }

  // block-wide; afterwards chunks 0 .. D-2 are in flight into slots 0 .. D-2
  __device__ __forceinline__ void init(const MlpDev& m, char* lds) {
    ring = reinterpret_cast<h8*>(lds);
    ring_lds = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)lds;
    float4* lq = reinterpret_cast<float4*>(lds + C::RING_BYTES);
    for (int q = threadIdx.x; q < C::F; q += blockDim.x)
      lq[q] = make_float4(m.basis[q], m.basis[C::F + q], m.basis[2 * C::F + q], 0.f);
    lbasis = lq;
    float* lb = reinterpret_cast<float*>(lds + C::RING_BYTES + C::BASIS_BYTES);
    const int nb16 = (m.n_hidden + 2) * m.bias16_stride;
    const NRT_GLOBAL float* gb = (const NRT_GLOBAL float*)m.bias16;
    for (int i = threadIdx.x; i < nb16; i += blockDim.x) lb[i] = gb[i];
    lbias = lb;
    bstride_ = m.bias16_stride;
    sbase = m.stream16;
    sbytes = m.stream16_bytes;
    lane = threadIdx.x & 63;
    wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    slot = 0;
#pragma unroll
    for (int k = 0; k < D - 1; ++k) issue(k, k);
    __syncthreads();  // bias / basis copies
  }
  // start of chunk c (schedule index 0..NCH-1): wait until chunk c has landed in every wave's
  // share of the slot, then refill the slot read in chunk c-1 with chunk c + D - 1 (the next
  // evaluation's first chunks near the end); returns this lane's A base.
  static constexpr int after(int c) {  // this wave's DMAs issued after chunk c's: c+1 .. c+D-2
    int a = 0;
    for (int k = 1; k <= D - 2; ++k) a += C::loads(c + k);
    return a;
  }
  template <int CH>
  __device__ __forceinline__ const h8* begin() {
    constexpr int c = CH;
    // own DMAs of chunk c landed; own LDS reads (of slot c-1, about to be refilled) retired --
    // hipcc may leave the last A reads of chunk c-1 in flight past the barrier otherwise
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(waitcnt_vm_lgkm0(after(c)));
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    return ring + slot * C::SLOTF * 64 + lane;
  }
  __device__ __forceinline__ void end() { slot = slot == D - 1 ? 0 : slot + 1; }
  __device__ __forceinline__ f16v bias_at(int layer, int ib, int h) const {
    f16v v;
    const float* b = lbias + layer * bstride_ + 32 * ib + 4 * h;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      float4 q = *reinterpret_cast<const float4*>(b + 8 * g);
      v[4 * g + 0] = q.x; v[4 * g + 1] = q.y; v[4 * g + 2] = q.z; v[4 * g + 3] = q.w;
    }
    return v;
  }
  int bstride_;
};

// schedule of one chunk's dependent MFMA chain: keep two A reads in flight ahead of the MFMAs
// (hipcc otherwise hoists all of a chunk's ds_reads and runs out of registers)
template <int K>
__device__ __forceinline__ void chain_schedule() {
  __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
#pragma unroll
  for (int s = 0; s < K - 2; ++s) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
  }
  __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
}

template <bool FOLD>
__device__ __forceinline__ void act_pack1(const f16v& acc, h8& lo, h8& hi, int act) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float a = acc[j], b = acc[8 + j];
    if (FOLD) { a = sp2(a); b = sp2(b); }
    else { a = act_fwd<true>(a, act); b = act_fwd<true>(b, act); }
    lo[j] = (_Float16)a;
    hi[j] = (_Float16)b;
  }
}

// Forward-mode tangent columns (TAN): column c = 4 * ray + comp; comp 0 carries the value
// pre-activation z, comps 1..3 the tangent dz/dx_{comp-1}.  Every lane takes its ray's z from
// the quad leader (DPP quad broadcast) and returns act(z) (comp 0) or act'(z) * dz (comps 1..3).
__device__ __forceinline__ float quad_leader(float x) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x00, 0xf, 0xf, false));
}

template <bool FOLD>
__device__ __forceinline__ float act_tan(float z, bool value, int act) {
  const float zv = quad_leader(z);
  if (FOLD) {
    // log2 domain: a = log2(1 + 2^z), da/dz = 1 / (1 + 2^-z)
    const float e = __builtin_amdgcn_exp2f(-fabsf(zv));
    const float den = 1.f + e;
    const float pos = __int_as_float(max(__float_as_int(zv), 0));
    const float val = pos + __builtin_amdgcn_logf(den);
    const float sig = (zv >= 0.f ? 1.f : e) * __builtin_amdgcn_rcpf(den);
    return value ? val : sig * z;
  }
  return value ? act_fwd<true>(zv, act) : act_bwd(zv, act) * z;
}

template <bool FOLD, bool TAN>
__device__ __forceinline__ void act_pack(const f16v& acc, h8& lo, h8& hi, int act, bool value) {
  if (!TAN) { act_pack1<FOLD>(acc, lo, hi, act); return; }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    lo[j] = (_Float16)act_tan<FOLD>(acc[j], value, act);
    hi[j] = (_Float16)act_tan<FOLD>(acc[8 + j], value, act);
  }
}

// One SkipConnMLP evaluation (output row 0) for the wave's 32 columns through the ring; L
// hidden layers and skip period SK are compile-time so the whole evaluation is straight-line
// code.  Every wave of the block must call it the same number of times.  Columns are rays
// (TAN = false) or 8 rays x (value, d/dx, d/dy, d/dz) (TAN = true, forward-mode gradient:
// tangent columns get no bias, and their inputs are the encoding's derivatives).
template <int NB, int NE, int WV, bool FOLD, int L, int SK, bool TAN = false>
__device__ __forceinline__ float eval(Engine<NB, NE, WV>& E, const MlpDev& m, float x0, float x1,
                                      float x2) {
  const int h = E.lane >> 5;
  const int comp = TAN ? (E.lane & 3) : 0;
  const bool value = comp == 0;
  const float kLog2e = 1.4426950408889634f;
  // encoding fragments, raw (init) and activated (skip inputs).  Slot 16s + 8h + 2jj: k-steps
  // s < NE-1 hold the sin/cos pairs of projection q = 8s + 4h + jj (utils.py:37-40, same fma
  // order as proj()), the last k-step holds x0, x1, x2 in the h = 0 half and zeros.
  constexpr int F = Engine<NB, NE, WV>::C::F;
  h8 eraw[NE], eact[NE];
#pragma unroll
  for (int s = 0; s < NE; ++s) {
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      float a, b;
      float4 bq;
      if (s < NE - 1) {
        bq = E.lbasis[8 * s + 4 * h + jj];
        float pr = __fmul_rn(x0, bq.x);
        pr = fmaf(x1, bq.y, pr);
        pr = fmaf(x2, bq.z, pr);
        a = __sinf(pr);
        b = __cosf(pr);
      } else {
        a = (h == 0 && jj == 0) ? x0 : (h == 0 && jj == 1) ? x2 : 0.f;
        b = (h == 0 && jj == 0) ? x1 : 0.f;
      }
      float ra = a, rb = b, xa, xb;
      if (FOLD) { xa = sp2(a * kLog2e); xb = sp2(b * kLog2e); }
      else { xa = act_fwd<true>(a, m.act); xb = act_fwd<true>(b, m.act); }
      if (TAN && !value) {
        // d enc / d x_k:  sin/cos pair -> (cos, -sin) * B[k][q];  raw input slot i -> [i == k]
        const int k = comp - 1;
        float ta, tb;
        if (s < NE - 1) {
          const float bk = k == 0 ? bq.x : (k == 1 ? bq.y : bq.z);
          ta = b * bk;
          tb = -a * bk;
        } else {
          const int i = 8 * h + 2 * jj;
          ta = (i == k) ? 1.f : 0.f;
          tb = (i + 1 == k) ? 1.f : 0.f;
        }
        ra = ta; rb = tb;
        if (FOLD) {
          // d sp2(log2e * a) / da = log2e * sigmoid(a)
          xa = kLog2e * ta * __builtin_amdgcn_rcpf(1.f + __expf(-a));
          xb = kLog2e * tb * __builtin_amdgcn_rcpf(1.f + __expf(-b));
        } else {
          xa = act_bwd(a, m.act) * ta;
          xb = act_bwd(b, m.act) * tb;
        }
      }
      eraw[s][2 * jj] = (_Float16)ra;
      eraw[s][2 * jj + 1] = (_Float16)rb;
      eact[s][2 * jj] = (_Float16)xa;
      eact[s][2 * jj + 1] = (_Float16)xb;
    }
  }
  const float bmask = value ? 1.f : 0.f;
  auto bias = [&](int layer, int ib) {
    f16v b = E.bias_at(layer, ib, h);
    if (TAN) b *= bmask;
    return b;
  };
  h8 hv[2][2 * NB];
  // Software pipeline: the region of chunk k (between two barriers) holds chunk k's MFMA chains
  // (RB row blocks, one independent chain each) and the activation of chunk k-1's accumulators
  // (`pend`), so the scheduler can put that VALU work into the MFMA gaps.  A pending tile that
  // the current chains consume (last row blocks of the previous layer) is ordered by the
  // register dependency.
  using S = typename Engine<NB, NE, WV>::S;
  constexpr int RB = S::RB, G = S::G;
  f16v pend[RB];
  // init layer: one chunk of NB row blocks x NE k-steps over the raw encoding, RB at a time
  {
    const h8* A = E.template begin<0>();
#pragma unroll
    for (int ib0 = 0; ib0 < NB; ib0 += RB) {
      f16v acc[RB];
#pragma unroll
      for (int b = 0; b < RB; ++b) acc[b] = bias(0, ib0 + b);
#pragma unroll
      for (int s = 0; s < NE; ++s)
#pragma unroll
        for (int b = 0; b < RB; ++b) {
          acc[b] = mfma16(A[((ib0 + b) * NE + s) * 64], eraw[s], acc[b]);
          E.template dma_at<0>((ib0 + b) * NE + s, NB * NE);
        }
      if (ib0 > 0)
#pragma unroll
        for (int b = 0; b < RB; ++b)
          act_pack<FOLD, TAN>(pend[b], hv[0][2 * (ib0 - RB + b)], hv[0][2 * (ib0 - RB + b) + 1], m.act, value);
#pragma unroll
      for (int b = 0; b < RB; ++b) pend[b] = acc[b];
    }
    E.end();
  }
  static_for<L>([&](auto I) {
    constexpr int i = I;
    constexpr int src = i & 1, dst = src ^ 1;
    constexpr bool skip = (i != L - 1) && (i % SK) == 0;
    static_for<G>([&](auto J) {
      constexpr int j = J;
      const h8* A = E.template begin<1 + i * G + j>();
      f16v acc[RB];
#pragma unroll
      for (int b = 0; b < RB; ++b) acc[b] = bias(1 + i, RB * j + b);
      if constexpr (j == 0)
#pragma unroll
        for (int b = 0; b < RB; ++b)
          act_pack<FOLD, TAN>(pend[b], hv[src][2 * (NB - RB + b)], hv[src][2 * (NB - RB + b) + 1], m.act, value);
      constexpr int nm = RB * (2 * NB + (skip ? NE : 0));
#pragma unroll
      for (int s = 0; s < 2 * NB; ++s)
#pragma unroll
        for (int b = 0; b < RB; ++b) {
          acc[b] = mfma16(A[(s * RB + b) * 64], hv[src][s], acc[b]);
          E.template dma_at<1 + i * G + j>(s * RB + b, nm);
        }
      if (skip) {
#pragma unroll
        for (int s = 0; s < NE; ++s)
#pragma unroll
          for (int b = 0; b < RB; ++b) {
            acc[b] = mfma16(A[((2 * NB + s) * RB + b) * 64], eact[s], acc[b]);
            E.template dma_at<1 + i * G + j>((2 * NB + s) * RB + b, nm);
          }
      }
      if constexpr (j > 0)
#pragma unroll
        for (int b = 0; b < RB; ++b)
          act_pack<FOLD, TAN>(pend[b], hv[dst][2 * (RB * (j - 1) + b)], hv[dst][2 * (RB * (j - 1) + b) + 1], m.act, value);
#pragma unroll
      for (int b = 0; b < RB; ++b) pend[b] = acc[b];
      // keep each A read about two MFMAs ahead of its MFMA (left alone, hipcc hoists a chunk's
      // reads and runs out of registers)
      if (RB > 1) {
        __builtin_amdgcn_sched_group_barrier(0x100, 4 * RB + 2, 0);
#pragma unroll
        for (int k = 0; k < nm - 2; ++k) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      }
      E.end();
    });
  });
  // out layer (one 32-row block; output row 0 sits in register 0 of the h == 0 lanes)
  const h8* A = E.template begin<1 + L * G>();
  f16v acc = bias(L + 1, 0);
#pragma unroll
  for (int b = 0; b < RB; ++b)
    act_pack<FOLD, TAN>(pend[b], hv[L & 1][2 * (NB - RB + b)], hv[L & 1][2 * (NB - RB + b) + 1], m.act, value);
#pragma unroll
  for (int s = 0; s < 2 * NB; ++s) {
    acc = mfma16(A[s * 64], hv[L & 1][s], acc);
    E.template dma_at<1 + L * G>(s, 2 * NB);
  }
  E.end();
  return __shfl(acc[0], E.lane & 31);
}


// ------------------------------------------------------------------------------------------
// k-outer program engine (shading MLPs): chunk = KC k-steps x all NB row blocks, so the NB
// accumulators are independent MFMA chains; the encoding k-steps are computed on the fly (once
// per layer), which keeps wide encodings (F = 64 / 128) out of the register file.  The layer
// count and skip period are runtime values.
// ------------------------------------------------------------------------------------------
// DMA = true: the chunks go global -> LDS by LDS-DMA (buffer_load ... lds, as ring::Engine):
// no staging registers and no ds_write per piece; a wave waits for its own pieces of the next
// chunk with a counted vmcnt before the chunk barrier.
template <int WV, int MAXF_ = 16, bool DMA = false>
struct KEngine {
  static constexpr int MAXF = MAXF_;  // fragments per chunk: KC * NB <= MAXF (out layer: KC)
  static constexpr int MAXL = (MAXF + WV - 1) / WV;
  static constexpr int SLOTF = MAXL * WV;
  static constexpr int RING_BYTES = 3 * SLOTF * 1024;
  static constexpr int NSTG = DMA ? 1 : MAXL;
  h8* ring;
  uint32_t ring_lds;
  const float* lbias;
  const float4* lbasis;
  __amdgpu_buffer_rsrc_t srd;
  const NRT_CONST int* coff;
  int nch, c, slot, lane, wv;
  h8 stg[NSTG];

  __host__ __device__ static size_t lds_bytes(const ProgDev& p) {
    return RING_BYTES + (size_t)p.basis_q * 16 + (size_t)p.bias_floats * 4;
  }
  __device__ __forceinline__ void load(int chunk) {
    const int off = coff[chunk] + wv;
#pragma unroll
    for (int q = 0; q < MAXL; ++q) {
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(srd, lane * 16, (off + WV * q) * 1024, 0);
      stg[q] = __builtin_bit_cast(h8, v);
    }
  }
  __device__ __forceinline__ void store(int sl) {
    h8* D = ring + sl * SLOTF * 64 + lane;
#pragma unroll
    for (int q = 0; q < MAXL; ++q) D[(wv + WV * q) * 64] = stg[q];
  }
  // DMA: this wave's MAXL pieces of `chunk` into slot sl (pieces past the chunk's end read the
  // stream's zero padding / next chunk: harmless, and the count stays compile-time)
  __device__ __forceinline__ void dma(int chunk, int sl) {
    const int w = __builtin_amdgcn_readfirstlane(wv);
    const int off = __builtin_amdgcn_readfirstlane((coff[chunk] + w) * 1024);
    const uint32_t dst = __builtin_amdgcn_readfirstlane(ring_lds + (uint32_t)((sl * SLOTF + w) * 1024));
#pragma unroll
    for (int q = 0; q < MAXL; ++q) lds_dma16(srd, lane * 16, off + WV * q * 1024, dst + WV * q * 1024);
  }
  __device__ __forceinline__ int nxt(int x) const { return x + 1 == nch ? 0 : x + 1; }
  // block-wide: LDS = ring | basis | bias; afterwards slot 0 = chunk 0 and chunk 1 is on its way
  // (DMA: in flight into slot 1; otherwise staged in stg)
  __device__ __forceinline__ void init(const ProgDev& p, char* lds) {
    ring = reinterpret_cast<h8*>(lds);
    ring_lds = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)lds;
    float4* lq = reinterpret_cast<float4*>(lds + RING_BYTES);
    for (int q = threadIdx.x; q < p.basis_q; q += blockDim.x) lq[q] = p.basis[q];
    lbasis = lq;
    float* lb = reinterpret_cast<float*>(lds + RING_BYTES + (size_t)p.basis_q * 16);
    for (int i = threadIdx.x; i < p.bias_floats; i += blockDim.x) lb[i] = p.bias[i];
    lbias = lb;
    srd = __builtin_amdgcn_make_buffer_rsrc((void*)p.stream, 0, 0x7ffffff0, 0x00020000);
    coff = (const NRT_CONST int*)p.coff;
    nch = p.n_chunks;
    lane = threadIdx.x & 63;
    wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    c = 0;
    slot = 0;
    if (DMA) {
      dma(0, 0);
      dma(nxt(0), 1);
      __builtin_amdgcn_s_waitcnt(ring::waitcnt_vm_lgkm0(MAXL));  // chunk 0 landed
    } else {
      load(0);
      store(0);
      load(nxt(0));
    }
    __syncthreads();
  }
  __device__ __forceinline__ const h8* begin() {
    const int s1 = slot == 2 ? 0 : slot + 1;
    if (DMA) {
      dma(nxt(nxt(c)), s1 == 2 ? 0 : s1 + 1);  // into the slot chunk c-1 was read from
    } else {
      store(s1);
      load(nxt(nxt(c)));
    }
    __builtin_amdgcn_sched_barrier(0);
    return ring + slot * SLOTF * 64 + lane;
  }
  __device__ __forceinline__ void end() {
    if (DMA) {
      // own pieces of chunk c+1 landed (those of c+2 may fly on); own reads of this slot retired
      asm volatile("" ::: "memory");
      __builtin_amdgcn_s_waitcnt(ring::waitcnt_vm_lgkm0(MAXL));
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    } else {
      __syncthreads();
    }
    c = nxt(c);
    slot = slot == 2 ? 0 : slot + 1;
  }
  // DMA: no LDS write may still be in flight when the block's waves exit
  __device__ __forceinline__ void drain() {
    if (DMA) __builtin_amdgcn_s_waitcnt(ring::waitcnt_vm_lgkm0(0));
  }
  // acc[reg] = bias[layer][32 ib + (reg&3) + 8 (reg>>2) + 4h]
  __device__ __forceinline__ f16v bias_at(const ProgMlp& pm, int layer, int ib, int h) const {
    f16v v;
    const float* b = lbias + pm.bias_off + layer * pm.bstride + 32 * ib + 4 * h;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      float4 q = *reinterpret_cast<const float4*>(b + 8 * g);
      v[4 * g + 0] = q.x; v[4 * g + 1] = q.y; v[4 * g + 2] = q.z; v[4 * g + 3] = q.w;
    }
    return v;
  }
};

// B fragment of encoding k-step s for 3-input, latent-free MLPs with F = 8 (NE - 1):
// s < NE-1 -> sin/cos of projections q = 8s + 4h + jj, s = NE-1 -> (x0, x1, x2, 0...) in half 0.
template <int ACTIN>
__device__ __forceinline__ h8 enc_frag_k(const float4* basis, int s, int last, int h, float x0,
                                         float x1, float x2) {
  h8 f;
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) {
    float a, b;
    if (s < last) {
      const float4 bq = basis[8 * s + 4 * h + jj];
      float pr = __fmul_rn(x0, bq.x);
      pr = fmaf(x1, bq.y, pr);
      pr = fmaf(x2, bq.z, pr);
      a = __sinf(pr);
      b = __cosf(pr);
    } else {
      a = (h == 0 && jj == 0) ? x0 : (h == 0 && jj == 1) ? x2 : 0.f;
      b = (h == 0 && jj == 0) ? x1 : 0.f;
    }
    if (ACTIN >= 0) { a = act_fwd<true>(a, ACTIN); b = act_fwd<true>(b, ACTIN); }
    f[2 * jj] = (_Float16)a;
    f[2 * jj + 1] = (_Float16)b;
  }
  return f;
}

typedef _Float16 h2 __attribute__((ext_vector_type(2)));

template <int NB, int ACT>
__device__ __forceinline__ void kact(const f16v (&acc)[NB], h8 (&hv)[2 * NB]) {
#pragma unroll
  for (int ib = 0; ib < NB; ++ib)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      h8 f;
      if (ACT == ACT_LEAKY) {
        // leaky_relu(x) = max(x, 0.01 x) on packed halves: cvt_pk + pk_mul + pk_max per pair
        // (1.5 VALU per element instead of cmp + mul + cndmask + cvt)
        const h2 k = {(_Float16)0.01f, (_Float16)0.01f};
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
          const h2 v = {(_Float16)acc[ib][8 * s2 + j], (_Float16)acc[ib][8 * s2 + j + 1]};
          const h2 r = __builtin_elementwise_max(v, v * k);
          f[j] = r[0];
          f[j + 1] = r[1];
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = (_Float16)act_fwd<true>(acc[ib][8 * s2 + j], ACT);
      }
      hv[2 * ib + s2] = f;
    }
}

// One evaluation of program MLP `pm` (compile-time NB, NE, activation) for the wave's 32 rays;
// returns the first output row block (rows (reg&3) + 8(reg>>2) + 4h of column lane&31).
// Every wave of the block must run the same sequence of evaluations (the ring is shared).
template <int NB, int NE, int WV, int ACT>
__device__ __forceinline__ f16v keval(KEngine<WV>& E, const ProgMlp& pm, float x0, float x1,
                                      float x2) {
  constexpr int KC = 16 / NB;
  constexpr int CE = (NE + KC - 1) / KC;   // chunks of the encoding part
  constexpr int CH = (2 * NB + KC - 1) / KC;  // chunks of the hidden part
  const int h = E.lane >> 5;
  const float4* basis = E.lbasis + pm.basis_off;
  f16v acc[NB];
  h8 hv[2 * NB];
#pragma unroll
  for (int ib = 0; ib < NB; ++ib) acc[ib] = E.bias_at(pm, 0, ib, h);
  // init layer: raw encoding (neural_blocks.py:80)
#pragma unroll
  for (int cc = 0; cc < CE; ++cc) {
    const h8* A = E.begin();
#pragma unroll
    for (int j = 0; j < KC; ++j) {
      const int s = cc * KC + j;
      if (s < NE) {
        const h8 b = enc_frag_k<-1>(basis, s, NE - 1, h, x0, x1, x2);
#pragma unroll
        for (int ib = 0; ib < NB; ++ib) acc[ib] = mfma16(A[(j * NB + ib) * 64], b, acc[ib]);
      }
    }
    E.end();
  }
  // hidden layers: x = layer(act(cat[x, enc] if skip else x)) (neural_blocks.py:81-84)
  for (int i = 0; i < pm.L; ++i) {
    kact<NB, ACT>(acc, hv);
#pragma unroll
    for (int ib = 0; ib < NB; ++ib) acc[ib] = E.bias_at(pm, 1 + i, ib, h);
#pragma unroll
    for (int cc = 0; cc < CH; ++cc) {
      const h8* A = E.begin();
#pragma unroll
      for (int j = 0; j < KC; ++j) {
        const int s = cc * KC + j;
        if (s < 2 * NB) {
#pragma unroll
          for (int ib = 0; ib < NB; ++ib) acc[ib] = mfma16(A[(j * NB + ib) * 64], hv[s], acc[ib]);
        }
      }
      E.end();
    }
    if (i != pm.L - 1 && (i % pm.skip) == 0) {
#pragma unroll
      for (int cc = 0; cc < CE; ++cc) {
        const h8* A = E.begin();
#pragma unroll
        for (int j = 0; j < KC; ++j) {
          const int s = cc * KC + j;
          if (s < NE) {
            const h8 b = enc_frag_k<ACT>(basis, s, NE - 1, h, x0, x1, x2);
#pragma unroll
            for (int ib = 0; ib < NB; ++ib) acc[ib] = mfma16(A[(j * NB + ib) * 64], b, acc[ib]);
          }
        }
        E.end();
      }
    }
  }
  kact<NB, ACT>(acc, hv);
  // out layer (one row block, all 2NB k-steps in one chunk)
  f16v o = E.bias_at(pm, pm.L + 1, 0, h);
  {
    const h8* A = E.begin();
#pragma unroll
    for (int s = 0; s < 2 * NB; ++s) o = mfma16(A[s * 64], hv[s], o);
    E.end();
  }
  return o;
}

// output row j (< 32) of a keval tile for this lane's column
__device__ __forceinline__ float tile_row(const f16v& o, int j, int lane) {
  const int reg = (j & 3) + 4 * (j >> 3), hh = (j >> 2) & 1;
  return __shfl(o[reg], (lane & 31) + 32 * hh);
}

}  // namespace ring

// ------------------------------------------------------------------------------------------
// FP32 block-cooperative engine (ring32): the reference-precision SDF MLP on the LDS ring.
// ------------------------------------------------------------------------------------------
// v_mfma_f32_16x16x4_f32 (exact f32: each MFMA adds 4 fma products per output, same as a VALU
// fma chain) on 16-ray tiles: lane (g = lane >> 4, j = lane & 15) serves ray j, and the four lane
// groups split the K dimension.  The 16x16 accumulator of a 16-row sub-block holds row 4 g + reg
// of ray j in register reg -- exactly the B operand of four k-steps of the next layer, so a whole
// layer's activations stay in registers: H / 4 floats per lane (64 for H = 256), in the k order
// the packer permutes W's columns to (nrt_internal.h ring32_walk).  32x32x2 tiles would need H / 2
// per lane and twice that with the next layer's outputs, which is more than a wave can hold.
// The weights stream through a 2-slot LDS ring shared by the WV waves of the block: chunk = 32
// output rows of one layer (two sub-blocks = two independent MFMA chains); at the start of chunk
// c every wave waits for its own LDS-DMA pieces of chunk c, the block barrier makes all of them
// visible and retires everyone's reads of chunk c - 1, and the waves then DMA chunk c + 1 into
// the slot chunk c - 1 used.  The activation (torch's exact softplus / leaky_relu) of chunk c - 1's
// accumulators runs in the MFMA gaps of chunk c.  Layer count and skip period are runtime values.
namespace ring32 {

typedef float f4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4v mfma4(float a, float b, f4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// 16-row sub-blocks per chunk: 64 output rows (four independent MFMA chains) between barriers.
// Round 4 ran 32-row chunks; the headline march's PMC showed 28 % of wave time parked at the
// per-chunk barrier (MFMA busy 0.76), so a chunk now carries twice the MFMAs per barrier.  A skip
// layer's encoding part is a chunk of its own (64 rows x the encoding quads), which keeps the
// largest chunk (and the 2-slot ring) at 64 KiB for H = 256.
constexpr int kSub = 4;

// The FP32 ring's SphereSDF table in LDS as sphere PAIRS for packed-f32 VALU: lane group g
// (lane >> 4) owns spheres g, g + 4, g + 8, ... and record 4 j + g holds its spheres g + 8 j and
// g + 8 j + 4 as 13 float2 (m00 m01 m02 m10 m11 m12 m20 m21 m22 cx cy cz r) + pad = 7 float4; a
// missing sphere has r = -inf (its term exp2(+inf * -k log2 e) is 0).  nrt_launch.h
// ring32_sphere_bytes sizes it.
constexpr int kPair32F4 = 7;
__host__ __device__ inline int sphere_pairs32(int n) { return ((n + 3) / 4 + 1) / 2; }  // per group
__device__ __forceinline__ void build_sphere_pairs32(const SdfDev& s, float4* out) {
  const int n = s.n_spheres, R = 4 * sphere_pairs32(n);
  const float4* src = reinterpret_cast<const float4*>(s.spheres);
  for (int rec = threadIdx.x; rec < R; rec += blockDim.x) {
    const int g = rec & 3, j = rec >> 2;
    float* o = reinterpret_cast<float*>(out + rec * kPair32F4);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = g + 8 * j + 4 * u;
      if (i < n) {
        const float4 r0 = src[4 * i], r1 = src[4 * i + 1], r2 = src[4 * i + 2], r3 = src[4 * i + 3];
        const float m[13] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w, r2.x, r2.y, r2.z, r2.w,
                             r3.x};
        for (int k = 0; k < 13; ++k) o[2 * k + u] = m[k];
      } else {
        for (int k = 0; k < 12; ++k) o[2 * k + u] = 0.f;
        o[24 + u] = -__builtin_inff();
      }
    }
    o[26] = 0.f; o[27] = 0.f;
  }
}

// KH = H / 4 hidden k-steps, KE = ke / 4 encoding k-steps (ke = encoding slots padded to 16)
template <int KH, int KE, int WV>
struct Engine {
  static constexpr int QH = KH / 4, QE = KE / 4;        // quads per sub-block
  static constexpr int MAXQ = kSub * (QH > QE ? QH : QE);  // largest chunk, KiB
  static constexpr int MAXL = (MAXQ + WV - 1) / WV;     // DMA pieces per wave per chunk
  static constexpr int SLOTQ = MAXL * WV;
  static constexpr int RING_BYTES = 2 * SLOTQ * 1024;
  static constexpr int kOutOfRange = 0x40000000;
  // LDS of one block: ring | basis (float4 per frequency) | biases | sphere table
  static size_t lds_bytes(int F, size_t bias_bytes, size_t sphere_bytes) {
    return RING_BYTES + (size_t)F * 16 + bias_bytes + sphere_bytes;
  }
  const float4* ring;
  uint32_t ring_lds;
  const float* lbias;
  const float4* lbasis;
  const float4* lspheres;   // [n][4] float4: (I+T) rows, centre, radius (SdfDev layout)
  const void* sbase;
  int sbytes, bstride;
  int off, next_off;        // quad offset of the current / next chunk in stream32 (wave-uniform)
  int slot;
  int lane, wv;

  // DMA chunk (quad offset qoff, nq quads) into ring slot s: wave wv moves quads wv + WV q
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

  // block-wide; afterwards chunk 0 (the init layer's first, nq0 quads) is in flight to slot 0
  __device__ __forceinline__ void init(const MlpDev& m, const SdfDev& s, char* lds, int nq0) {
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
    for (int i = threadIdx.x; i < nb; i += blockDim.x) lb[i] = m.bias32[i];
    lbias = lb;
    p += (size_t)nb * 4;
    float4* ls = reinterpret_cast<float4*>(p);
    if (s.kind == 2) build_sphere_pairs32(s, ls);
    lspheres = ls;
    bstride = m.bias16_stride;
    sbase = m.stream32;
    sbytes = m.stream32_bytes;
    lane = threadIdx.x & 63;
    wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    off = 0;
    slot = 0;
    issue(0, nq0, 0);
    __syncthreads();
  }
  // start of the current chunk (nq quads): wait for it, then DMA the next one (nq_next quads; at
  // offset 0 when `wrap`, i.e. the next evaluation's first chunk); returns this lane's A base
  __device__ __forceinline__ const float4* begin(int nq, int nq_next, bool wrap) {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(ring::waitcnt_vm_lgkm0(0));
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    next_off = wrap ? 0 : off + nq;
    issue(next_off, nq_next, slot ^ 1);
    __builtin_amdgcn_sched_barrier(0);
    return ring + slot * SLOTQ * 64 + lane;
  }
  __device__ __forceinline__ void end() {
    off = next_off;
    slot ^= 1;
  }
  // the DMA issued by the last begin() must land before the block's LDS is released
  __device__ __forceinline__ void drain() { __builtin_amdgcn_s_waitcnt(ring::waitcnt_vm_lgkm0(0)); }
  // acc[reg] = bias[layer][16 sb + 4 g + reg]
  __device__ __forceinline__ f4v bias_at(int layer, int sb) const {
    const float4 q = *reinterpret_cast<const float4*>(lbias + layer * bstride + 16 * sb + 4 * (lane >> 4));
    return f4v{q.x, q.y, q.z, q.w};
  }
};

// the FP32 ring engine's softplus (softplus_exact, above)
__device__ __forceinline__ float softplus_f32(float x) { return softplus_exact(x); }

// the MLP activation with the code a template argument (torch semantics, FP32)
template <int ACT>
__device__ __forceinline__ float act(float x) {
  if (ACT == ACT_SOFTPLUS) return softplus_f32(x);
  return act_fwd<false>(x, ACT);
}

// One segment of a two-sub-block chunk: NQ quads at ring positions P0 + 2u + b (sub-block b),
// k-step 4u + t takes B[4u + t]; chains a0 / a1 alternate, so consecutive MFMAs are independent.
// Each quad's two LDS reads are issued one quad ahead of its MFMAs.  side(u) runs before quad
// u + 1's reads in program order: the previous chunk's activations, one element per quad, each
// pinned by an empty volatile asm (which LDS reads cannot cross), so they spread over the chunk
// instead of running as one block at its start while the MFMA pipe idles.
template <int NQ, int P0, int BO, int NBV, class Side>
__device__ __forceinline__ void seg2(const float4* A, const float (&B)[NBV], f4v& a0, f4v& a1,
                                     Side&& side) {
  float4 w0 = A[P0 * 64], w1 = A[(P0 + 1) * 64];
#pragma unroll
  for (int u = 0; u < NQ; ++u) {
    side(u);  // side work of quad u (program order pins it between the LDS reads)
    float4 n0 = w0, n1 = w1;
    if (u + 1 < NQ) { n0 = A[(P0 + 2 * u + 2) * 64]; n1 = A[(P0 + 2 * u + 3) * 64]; }
    a0 = mfma4(w0.x, B[BO + 4 * u], a0); a1 = mfma4(w1.x, B[BO + 4 * u], a1);
    a0 = mfma4(w0.y, B[BO + 4 * u + 1], a0); a1 = mfma4(w1.y, B[BO + 4 * u + 1], a1);
    a0 = mfma4(w0.z, B[BO + 4 * u + 2], a0); a1 = mfma4(w1.z, B[BO + 4 * u + 2], a1);
    a0 = mfma4(w0.w, B[BO + 4 * u + 3], a0); a1 = mfma4(w1.w, B[BO + 4 * u + 3], a1);
    w0 = n0; w1 = n1;
  }
}
template <int NQ, int P0, int BO, int NBV>
__device__ __forceinline__ void seg2(const float4* A, const float (&B)[NBV], f4v& a0, f4v& a1) {
  seg2<NQ, P0, BO>(A, B, a0, a1, [](int) {});
}

// seg2 for a four-sub-block chunk: NQ quads at ring positions P0 + 4u + b, four chains a[b];
// each quad's four LDS reads issued one quad ahead of its MFMAs, side(u) before them
template <int NQ, int P0, int BO, int NBV, class Side>
__device__ __forceinline__ void seg4(const float4* A, const float (&B)[NBV], f4v (&a)[kSub],
                                     Side&& side) {
  float4 w[kSub];
#pragma unroll
  for (int b = 0; b < kSub; ++b) w[b] = A[(P0 + b) * 64];
#pragma unroll
  for (int u = 0; u < NQ; ++u) {
    side(u);
    float4 n[kSub];
#pragma unroll
    for (int b = 0; b < kSub; ++b) n[b] = (u + 1 < NQ) ? A[(P0 + kSub * (u + 1) + b) * 64] : w[b];
#pragma unroll
    for (int b = 0; b < kSub; ++b) a[b] = mfma4(w[b].x, B[BO + 4 * u], a[b]);
#pragma unroll
    for (int b = 0; b < kSub; ++b) a[b] = mfma4(w[b].y, B[BO + 4 * u + 1], a[b]);
#pragma unroll
    for (int b = 0; b < kSub; ++b) a[b] = mfma4(w[b].z, B[BO + 4 * u + 2], a[b]);
#pragma unroll
    for (int b = 0; b < kSub; ++b) a[b] = mfma4(w[b].w, B[BO + 4 * u + 3], a[b]);
#pragma unroll
    for (int b = 0; b < kSub; ++b) w[b] = n[b];
  }
}

// forward-mode activation (TAN): the lane's column is 4 ray + comp, comp 0 the value
// pre-activation z, comps 1..3 the tangent dz/dx_{comp-1}; every lane takes its ray's z from the
// quad leader and returns act(z) (comp 0) or act'(z) dz (torch's backward formulas, act_bwd)
template <int ACT>
__device__ __forceinline__ float act_tan32(float z, bool value) {
  const float zv = ring::quad_leader(z);
  return value ? act<ACT>(zv) : act_bwd(zv, ACT) * z;
}

// One SkipConnMLP evaluation (output row 0) for the wave's 16 columns, every lane of a column
// gets its value.  Columns are rays, or (TAN) 4 rays x (value, d/dx, d/dy, d/dz): forward-mode
// gradient, tangent columns take the encoding's derivatives as input and no bias (as ring::eval).
// Every wave of the block must call it the same number of times.
template <int KH, int KE, int WV, int ACT, bool TAN = false>
__device__ __forceinline__ float eval(Engine<KH, KE, WV>& E, const MlpDev& m, float x0, float x1,
                                      float x2) {
  using En = Engine<KH, KE, WV>;
  constexpr int QH = En::QH, QE = En::QE;
  constexpr int NC = KH / (4 * kSub);  // 64-row chunks per layer
  static_assert(QH >= 8 && KH % (4 * kSub) == 0, "hidden chunks must spread the pending activations");
  const int g = E.lane >> 4;
  const int comp = TAN ? (E.lane & 3) : 0;
  const bool value = comp == 0;
  const int F = m.freqs, L = m.n_hidden, SK = m.skip;
  // encoding: k-step e of lane group g is slot 4 e + g: sin / cos of projection (4e + g) / 2
  // (utils.py:37-40, same fma order and accurate sincosf as the FP32 slab path), then x, zeros
  float eraw[KE], eact[KE];
#pragma unroll
  for (int e = 0; e < KE; ++e) {
    const int slot = 4 * e + g;
    float v = 0.f, tv = 0.f;  // value and (TAN) d/dx_{comp-1}
    if (slot < 2 * F) {
      const float4 b = E.lbasis[slot >> 1];
      float pr = x0 * b.x;
      pr = fmaf(x1, b.y, pr);
      pr = fmaf(x2, b.z, pr);
      float sn, cs;
      sincosf(pr, &sn, &cs);
      v = (slot & 1) ? cs : sn;
      if (TAN) {
        const float bk = comp == 1 ? b.x : comp == 2 ? b.y : b.z;
        tv = (slot & 1) ? -sn * bk : cs * bk;
      }
    } else if (slot == 2 * F) {
      v = x0;
      tv = comp == 1 ? 1.f : 0.f;
    } else if (slot == 2 * F + 1) {
      v = x1;
      tv = comp == 2 ? 1.f : 0.f;
    } else if (slot == 2 * F + 2) {
      v = x2;
      tv = comp == 3 ? 1.f : 0.f;
    }
    if (TAN && !value) {
      eraw[e] = tv;
      eact[e] = act_bwd(v, ACT) * tv;
    } else {
      eraw[e] = v;
      eact[e] = act<ACT>(v);
    }
  }
  const float bmask = value ? 1.f : 0.f;
  auto bias = [&](int layer, int sb) {
    f4v b = E.bias_at(layer, sb);
    if (TAN) b *= bmask;
    return b;
  };
  constexpr int CH = kSub * QH, CE = kSub * QE;  // KiB of a hidden-part / encoding-part chunk
  // the first chunk of hidden layer i (i == L: the out layer)
  auto first_q = [&](int i) { return i >= L ? QH : CH; };
  float src[KH], dst[KH];
  f4v pend[kSub];
  // activation of chunk ib's accumulators into dst.  The empty asm pins each result inside the
  // chunk that computes it: dst is read only by the next layer, so the compiler would otherwise
  // sink every chunk's activations to the end of the layer, out of the MFMA gaps.
  auto retire1 = [&](int ib, int k) {  // element k (< 4 kSub) of chunk ib
    const int r = k & 3;
    float& d = dst[4 * kSub * ib + k];
    if (TAN) d = act_tan32<ACT>(pend[k >> 2][r], value);
    else d = act<ACT>(pend[k >> 2][r]);
    asm volatile("" : "+v"(d));
  };
  // elements 2q, 2q + 1 of chunk ib: softplus on packed f32 (softplus_exact2, the same bits)
  constexpr bool PK = !TAN && ACT == ACT_SOFTPLUS;
  auto retire2 = [&](int ib, int q) {
    if constexpr (PK) {
      const int k = 2 * q, r = k & 3;
      const f2v v = softplus_exact2(f2v{pend[k >> 2][r], pend[k >> 2][r + 1]});
      float& d0 = dst[4 * kSub * ib + k];
      float& d1 = dst[4 * kSub * ib + k + 1];
      d0 = v[0];
      d1 = v[1];
      asm volatile("" : "+v"(d0), "+v"(d1));
    } else {
      retire1(ib, 2 * q);
      retire1(ib, 2 * q + 1);
    }
  };
  auto retire = [&](int ib) {
#pragma unroll
    for (int q = 0; q < 2 * kSub; ++q) retire2(ib, q);
  };
  // init layer (neural_blocks.py:80): raw encoding in
#pragma unroll
  for (int ib = 0; ib < NC; ++ib) {
    const float4* A = E.begin(CE, ib + 1 < NC ? CE : first_q(0), false);
    f4v a[kSub];
#pragma unroll
    for (int b = 0; b < kSub; ++b) a[b] = bias(0, kSub * ib + b);
    if (ib > 0) retire(ib - 1);
    seg4<QE, 0, 0>(A, eraw, a, [](int) {});
#pragma unroll
    for (int b = 0; b < kSub; ++b) pend[b] = a[b];
    E.end();
  }
  retire(NC - 1);
  // hidden layers: x = layer(act(cat[x, enc] if skip else x)) (neural_blocks.py:81-84)
  for (int i = 0; i < L; ++i) {
#pragma unroll
    for (int k = 0; k < KH; ++k) src[k] = dst[k];
    const bool skip = i != L - 1 && i % SK == 0;
#pragma unroll
    for (int ib = 0; ib < NC; ++ib) {
      const int after = ib + 1 < NC ? CH : first_q(i + 1);  // the chunk after this row block
      const float4* A = E.begin(CH, skip ? CE : after, false);
      f4v a[kSub];
#pragma unroll
      for (int b = 0; b < kSub; ++b) a[b] = bias(1 + i, kSub * ib + b);
      // the previous chunk's 4 kSub activations spread over this chunk's QH quads, in pairs
      seg4<QH, 0, 0>(A, src, a, [&](int u) {
        if (ib > 0)
#pragma unroll
          for (int q = (u * 2 * kSub) / QH; q < ((u + 1) * 2 * kSub) / QH; ++q) retire2(ib - 1, q);
      });
      E.end();
      if (skip) {  // the encoding part: a chunk of its own
        const float4* B = E.begin(CE, after, false);
        seg4<QE, 0, 0>(B, eact, a, [](int) {});
        E.end();
      }
#pragma unroll
      for (int b = 0; b < kSub; ++b) pend[b] = a[b];
    }
    retire(NC - 1);
  }
  // out layer (neural_blocks.py:86): one 16-row sub-block, two half chains (k-steps of even /
  // odd quads) so consecutive MFMAs are independent; row 0 of ray j sits in register 0 of lane j
  const float4* A = E.begin(QH, CE, true);
  f4v o0 = bias(L + 1, 0), o1 = f4v{0.f, 0.f, 0.f, 0.f};
  {
    float4 w0 = A[0], w1 = A[64];
#pragma unroll
    for (int u = 0; u < QH; u += 2) {
      float4 n0 = w0, n1 = w1;
      if (u + 2 < QH) { n0 = A[(u + 2) * 64]; n1 = A[(u + 3) * 64]; }
      o0 = mfma4(w0.x, dst[4 * u], o0); o1 = mfma4(w1.x, dst[4 * u + 4], o1);
      o0 = mfma4(w0.y, dst[4 * u + 1], o0); o1 = mfma4(w1.y, dst[4 * u + 5], o1);
      o0 = mfma4(w0.z, dst[4 * u + 2], o0); o1 = mfma4(w1.z, dst[4 * u + 6], o1);
      o0 = mfma4(w0.w, dst[4 * u + 3], o0); o1 = mfma4(w1.w, dst[4 * u + 7], o1);
      w0 = n0; w1 = n1;
    }
  }
  E.end();
  const float o = o0[0] + o1[0];
  return __shfl(o, E.lane & 15);
}

// sphere blob part of a SphereSDF (sdfs.py:37-43, utils.py:386-387) for a 16-ray tile: lane group
// g sums exp(-k d_i) over spheres i = g, g + 4, ... from the LDS table, the four partial sums are
// combined with two butterfly adds (commutative, so every lane gets the same bits)
__device__ __forceinline__ float spheres_value16(const SdfDev& s, const float4* sp, int lane,
                                                 float x, float y, float z) {
  const float nk2 = -s.k * 1.4426950408889634f;
  float acc = 0.f;
  for (int i = lane >> 4; i < s.n_spheres; i += 4) {
    const float4 r0 = sp[4 * i], r1 = sp[4 * i + 1], r2 = sp[4 * i + 2], r3 = sp[4 * i + 3];
    // row-major (I+T): r0 = (m00 m01 m02 m10), r1 = (m11 m12 m20 m21), r2 = (m22 cx cy cz), r3 = (r ...)
    const float qx = fmaf(r0.z, z, fmaf(r0.y, y, r0.x * x)) - r2.y;
    const float qy = fmaf(r1.y, z, fmaf(r1.x, y, r0.w * x)) - r2.z;
    const float qz = fmaf(r2.x, z, fmaf(r1.w, y, r1.z * x)) - r2.w;
    // v_sqrt_f32 (1 ulp) and exp(-k d) as v_exp_f32 of -k log2(e) d (a few ulp; a term that
    // leaves the normal range is 0, below the 1e-4 floor of the sum): round 6, ~15 VALU a
    // sphere fewer than the correctly rounded sqrtf / expf, 3e-9 on the SDF value
    const float d = __builtin_amdgcn_sqrtf(qx * qx + qy * qy + qz * qz) - r3.x;
    acc += __builtin_amdgcn_exp2f(d * nk2);
  }
  acc += __shfl_xor(acc, 16);
  acc += __shfl_xor(acc, 32);
  return -logf(fmaxf(acc, 1e-4f)) / s.k;
}

// spheres_value16 over the pair table (build_sphere_pairs32): the same per-sphere operations in
// the same order on packed f32 (v_pk_mul / v_pk_fma / v_pk_add: two spheres an instruction, half
// the VALU), the two halves of a lane's sum added at the end (a different summation order than
// spheres_value16's single running sum: an ulp of the sum)
__device__ __forceinline__ float spheres_value16_pairs(const SdfDev& s, const float4* sp, int lane,
                                                       float x, float y, float z) {
  const int g = lane >> 4, NP = sphere_pairs32(s.n_spheres);
  const float nk = -s.k * 1.4426950408889634f;
  const f2v xx = {x, x}, yy = {y, y}, zz = {z, z}, nk2 = {nk, nk};
  f2v acc = {0.f, 0.f};
  for (int j = 0; j < NP; ++j) {
    const float4* q = sp + (4 * j + g) * kPair32F4;
    const float4 a = q[0], b = q[1], c = q[2], d = q[3], e = q[4], f = q[5], h = q[6];
    const f2v m00 = {a.x, a.y}, m01 = {a.z, a.w}, m02 = {b.x, b.y}, m10 = {b.z, b.w};
    const f2v m11 = {c.x, c.y}, m12 = {c.z, c.w}, m20 = {d.x, d.y}, m21 = {d.z, d.w};
    const f2v m22 = {e.x, e.y}, cx = {e.z, e.w}, cy = {f.x, f.y}, cz = {f.z, f.w};
    const f2v r = {h.x, h.y};
    const f2v qx = __builtin_elementwise_fma(m02, zz, __builtin_elementwise_fma(m01, yy, m00 * xx)) - cx;
    const f2v qy = __builtin_elementwise_fma(m12, zz, __builtin_elementwise_fma(m11, yy, m10 * xx)) - cy;
    const f2v qz = __builtin_elementwise_fma(m22, zz, __builtin_elementwise_fma(m21, yy, m20 * xx)) - cz;
    const f2v n2 = (qx * qx + qy * qy) + qz * qz;
    const f2v dd = f2v{__builtin_amdgcn_sqrtf(n2.x), __builtin_amdgcn_sqrtf(n2.y)} - r;
    const f2v t = dd * nk2;
    acc += f2v{__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)};
  }
  float v = acc.x + acc.y;
  v += __shfl_xor(v, 16);
  v += __shfl_xor(v, 32);
  return -logf(fmaxf(v, 1e-4f)) / s.k;
}

}  // namespace ring32
}  // namespace nrt
