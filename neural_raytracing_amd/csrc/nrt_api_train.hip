// nrt_api_train.hip -- SkipConnMLP backward (first slice): the gradients
// torch autograd produces for `y = mlp(x, latent)` (neural_blocks.py:75-86) given dL/dy.
//
//   k_mlp_backward32  per wave 32 rows, FP32 MFMA (v_mfma_f32_32x32x2_f32) on the LDS slab:
//                     forward with saved pre-activations Z_l and activations A_l = act(Z_l),
//                     the encoding (raw and activated) in the reference's column order, then the
//                     row-local backward chain dZ_l = (dZ_{l+1} W_{l+1}) * act'(Z_l) with the W^T
//                     fragments, the encoding gradient, and dL/dx, dL/dlatent.  TILE moves the
//                     encoding and its gradient out of the slab into per-wave global tiles.
//   weight gradients  dW_l = dZ_l^T In_l over the batch (K = M) and bias gradients (In = ones):
//                     every layer of one backward call in one k_wgrad_batch launch (split-K
//                     exact-f32 MFMA on the saved activations) + k_split_reduce_batch (slices
//                     summed in order: deterministic).

#include "nrt_launch.h"

namespace nrt {

// A-fragment prefetch depth of the training kernels' slab GEMMs (gemm32): they run one wave per
// SIMD from 4 row blocks up (accumulators + slab), where 8 buffers fit; at 3 row blocks and
// below 4, which keeps two waves per SIMD
constexpr int train_pf(int nb) { return nb >= 4 ? 8 : 4; }

// reference encoding column of slot s ([x, sin(xB), cos(xB), latent], utils.py:37-40); -1 = pad
__device__ __forceinline__ int enc_col(const MlpDev& m, int s) {
  const int F = m.freqs, in = m.in_size;
  if (s < 2 * F) return (s & 1) ? in + F + (s >> 1) : in + (s >> 1);
  if (s < 2 * F + in) return s - 2 * F;
  if (s < 2 * F + in + m.latent) return in + 2 * F + (s - 2 * F - in);
  return -1;
}

// TILE: the encoding and its gradient live in per-wave global tiles [ke][32 rows] (L2-resident)
// and the LDS slab row is the H hidden columns only -- for MLPs whose H + ke slab row caps the CU
// at two waves (the 16x256 F=128 spatial-weights MLP: 68 KB a wave -> 33 KB).  Otherwise the slab
// row is [hidden | encoding], and the encoding slots take the encoding gradient in the backward.
template <int NB, bool TILE>
__device__ __forceinline__ void mlp_backward32(
    const MlpDev* __restrict__ mp, const float* __restrict__ x, const float* __restrict__ lat,
    int64_t M, const float* __restrict__ dY, float* __restrict__ dX, float* __restrict__ dLat,
    float* __restrict__ Zg, float* __restrict__ Ag, float* __restrict__ Eraw,
    float* __restrict__ Eact, float* __restrict__ dZg, float* __restrict__ Et,
    float* __restrict__ Gt, int RS, int per_wave) {
  extern __shared__ float smem[];
  const MlpDev& m = *mp;
  float* X = smem + (size_t)(threadIdx.x >> 6) * per_wave;
  const int lane = lane_id(), r = lane & 31, h = lane >> 5;
  const int64_t wg = wave_global();
  const int64_t row0 = wg * 32;
  if (row0 >= M) return;  // whole wave exits together
  const int64_t row = row0 + r;
  const bool valid = row < M;
  const int64_t rr = valid ? row : M - 1;
  const int H = m.hidden, L = m.n_hidden, ke = m.ke, dp = m.dp, in = m.in_size;
  EncIn e;
  if (in <= 4) {
    for (int i = 0; i < 4; ++i) e.x[i] = (i < in) ? x[rr * in + i] : 0.f;
    e.xg = nullptr;
  } else {
    e.x[0] = e.x[1] = e.x[2] = e.x[3] = 0.f;
    e.xg = x + rr * in;
  }
  e.lat = (lat && m.latent > 0) ? lat + rr * m.latent : nullptr;
  float* rowp = X + r * RS;
  // slot s of this lane's row: encoding in the forward, its gradient in the backward
  float* const et = TILE ? Et + wg * ke * 32 + r : rowp + H;
  float* const gt = TILE ? Gt + wg * ke * 32 + r : rowp + H;
  constexpr int es = TILE ? 32 : 1;
  // ---- forward (mlp32_forward's order of operations), saving Z_l, A_l and the encoding
  for (int slot = 2 * h; slot < ke; slot += 4) {
    float a, b;
    enc_pair<false>(m, e, slot, a, b);
    et[slot * es] = a;
    et[(slot + 1) * es] = b;
  }
  wave_lds_fence();
  if (TILE) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
  if (valid)
    for (int s = h; s < ke; s += 2) {
      const int c = enc_col(m, s);
      if (c < 0) continue;
      const float v = et[s * es];
      Eraw[row * dp + c] = v;
      Eact[row * dp + c] = act_fwd<false>(v, m.act);
    }
  f16v acc[NB];
  for (int l = 0; l <= L; ++l) {
    bias32<NB>(acc, m.bias[l], 0, NB, h);
    if (l == 0) {
      if (TILE) gemm32_tile<NB, train_pf(NB)>(acc, m.w32[0], NB, 0, ke >> 1, et - r, -1);
      else gemm32<NB, train_pf(NB)>(acc, m.w32[0], NB, 0, ke >> 1, X, RS, H, -1);
    } else {
      const int i = l - 1;
      gemm32<NB, train_pf(NB)>(acc, m.w32[l], NB, 0, H >> 1, X, RS, 0, -1);
      if (i != L - 1 && (i % m.skip) == 0) {
        const float* Ws = m.w32[l] + (H >> 1) * NB * 64;
        if (TILE) gemm32_tile<NB, train_pf(NB)>(acc, Ws, NB, 0, ke >> 1, et - r, m.act);
        else gemm32<NB, train_pf(NB)>(acc, Ws, NB, 0, ke >> 1, X, RS, H, m.act);
      }
    }
    wave_lds_fence();
    // registers 4g..4g+3 of a row block are 4 consecutive columns of the lane's row: one 16-byte
    // store each for Z and A (H is a multiple of 32, the arrays 256-byte aligned)
#pragma unroll
    for (int ib = 0; ib < NB; ++ib)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int k0 = 32 * ib + 8 * g + 4 * h;
        float4 zv, av;
        float* zp = &zv.x;
        float* ap = &av.x;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          zp[j] = acc[ib][4 * g + j];
          ap[j] = act_fwd<false>(zp[j], m.act);
          rowp[k0 + j] = ap[j];
        }
        if (valid) {
          *reinterpret_cast<float4*>(Zg + ((int64_t)l * M + row) * H + k0) = zv;
          *reinterpret_cast<float4*>(Ag + ((int64_t)l * M + row) * H + k0) = av;
        }
      }
    wave_lds_fence();
  }
  // ---- backward seed: dZ_L = (dY W_out) * act'(Z_L)
  // The encoding gradient accumulates in gt: slot s of row r belongs to lane (r, (s >> 2) & 1)
  // in every accumulation pass (the MFMA output layout), so a lane only re-reads its own stores
  // until the fence before dL/dx.  The skip layers' act'(enc) reads the raw encoding back from
  // Eraw, which this wave wrote above (row rr is always one of this wave's own rows) -- other
  // lanes' stores, so the fence orders them in both variants (the TILE variant's earlier fence
  // precedes the Eraw stores and does not cover them).
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  const float* eraw_row = Eraw + rr * dp;
  for (int s = 4 * h; s < ke; s += 8)
#pragma unroll
    for (int j = 0; j < 4; ++j) gt[(s + j) * es] = 0.f;
  const float* Ao = m.w32[L + 1];
  const int out = m.out;
  for (int k = h; k < H; k += 2) {
    float g = 0.f;
    for (int o = 0; o < out; ++o)
      g = fmaf(dY[rr * out + o], Ao[((k >> 1) * m.ob + (o >> 5)) * 64 + (k & 1) * 32 + (o & 31)], g);
    rowp[k] = g * act_bwd(Zg[((int64_t)L * M + rr) * H + k], m.act);
  }
  wave_lds_fence();
  for (int l = L; l >= 0; --l) {
    if (valid)
      for (int k = 4 * h; k < H; k += 8)
        *reinterpret_cast<float4*>(dZg + ((int64_t)l * M + row) * H + k) =
            make_float4(rowp[k], rowp[k + 1], rowp[k + 2], rowp[k + 3]);
    const float* At = m.wt32[l];
    const int nrb = m.nbt[l];
    const bool has_hidden_in = (l != 0);
    const bool has_enc_in = (l == 0) || ((l - 1) != L - 1 && ((l - 1) % m.skip) == 0);
    const int hid_rb = has_hidden_in ? NB : 0;
    if (has_enc_in) {
      const int enc_pos0 = has_hidden_in ? H : 0;
      for (int rb0 = hid_rb; rb0 < nrb; rb0 += NB) {
#pragma unroll
        for (int ib = 0; ib < NB; ++ib) acc[ib] = f16v{};
        gemm32<NB, train_pf(NB)>(acc, At, nrb, rb0, H >> 1, X, RS, 0, -1);
        // per row block: every load first (clamped addresses, unconditional), then the
        // activation's branches -- a load inside the act switch would wait on its own.  From
        // four row blocks up (one wave per SIMD already); below, the registers keep two waves.
#pragma unroll
        for (int ib = 0; ib < NB; ++ib) {
          if (rb0 + ib >= nrb) continue;
          if constexpr (NB < 4) {
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
              const int pos = 32 * (rb0 + ib) + (reg & 3) + 8 * (reg >> 2) + 4 * h;
              const int slot = pos - enc_pos0;
              if (slot >= 0 && slot < ke) {
                float v = acc[ib][reg];
                if (l != 0) {  // skip inputs are act(enc)
                  const int c = enc_col(m, slot);
                  v = c < 0 ? 0.f : v * act_bwd(eraw_row[c], m.act);
                }
                gt[slot * es] += v;
              }
            }
            continue;
          }
          float ev[16], gv[16];
#pragma unroll
          for (int reg = 0; reg < 16; ++reg) {
            const int pos = 32 * (rb0 + ib) + (reg & 3) + 8 * (reg >> 2) + 4 * h;
            const int slot = min(max(pos - enc_pos0, 0), ke - 1);
            const int c = l != 0 ? enc_col(m, slot) : -1;
            ev[reg] = eraw_row[c < 0 ? 0 : c];
            gv[reg] = gt[slot * es];
          }
#pragma unroll
          for (int reg = 0; reg < 16; ++reg) {
            const int pos = 32 * (rb0 + ib) + (reg & 3) + 8 * (reg >> 2) + 4 * h;
            const int slot = pos - enc_pos0;
            if (slot >= 0 && slot < ke) {
              float v = acc[ib][reg];
              if (l != 0) {  // skip inputs are act(enc)
                const int c = enc_col(m, slot);
                v = c < 0 ? 0.f : v * act_bwd(ev[reg], m.act);
              }
              gt[slot * es] = gv[reg] + v;
            }
          }
        }
      }
      wave_lds_fence();
    }
    if (has_hidden_in) {
#pragma unroll
      for (int ib = 0; ib < NB; ++ib) acc[ib] = f16v{};
      gemm32<NB, train_pf(NB)>(acc, At, nrb, 0, H >> 1, X, RS, 0, -1);
      wave_lds_fence();
      // the row block's four Z loads issue together, ahead of the activation's branches (from
      // four row blocks up, as above)
#pragma unroll
      for (int ib = 0; ib < NB; ++ib) {
        constexpr int Q = NB < 4 ? 1 : 4;
#pragma unroll
        for (int g0 = 0; g0 < 4; g0 += Q) {
          float4 zq[Q];
#pragma unroll
          for (int q = 0; q < Q; ++q)
            zq[q] = *reinterpret_cast<const float4*>(Zg + ((int64_t)(l - 1) * M + rr) * H + 32 * ib + 8 * (g0 + q) + 4 * h);
#pragma unroll
          for (int q = 0; q < Q; ++q) {
            const int k0 = 32 * ib + 8 * (g0 + q) + 4 * h;
            const float* zp = &zq[q].x;
#pragma unroll
            for (int j = 0; j < 4; ++j) rowp[k0 + j] = acc[ib][4 * (g0 + q) + j] * act_bwd(zp[j], m.act);
          }
        }
      }
      wave_lds_fence();
    }
  }
  // ---- encoding -> inputs: d sin(p_q) = cos(p_q) B_iq, d cos(p_q) = -sin(p_q) B_iq, x_i direct
  wave_lds_fence();
  if (TILE) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
  const float* egrad = gt;  // egrad[es * s] = slot s of this lane's row
  const int F = m.freqs;
  for (int i = 0; i < in; ++i) {
    float g = 0.f;
    for (int q = h; q < F; q += 2) {
      float s, c;
      sincosf(proj<false>(m, e, q), &s, &c);
      g = fmaf(egrad[es * (2 * q)] * c - egrad[es * (2 * q + 1)] * s, m.basis[i * F + q], g);
    }
    if (h == 0) g += egrad[es * (2 * F + i)];
    g += __shfl_xor(g, 32);
    if (dX && valid && h == 0) dX[row * in + i] = g;
  }
  if (dLat && valid)
    for (int j = h; j < m.latent; j += 2) dLat[row * m.latent + j] = egrad[es * (2 * F + in + j)];
}

// ---- column-split backward: one block of CW waves per 32 rows -------------------------------
// The per-wave variant above gives a training batch one wave per 32 rows: a ~19k-row backward is
// ~600 waves on 1,024 SIMDs, each running every layer's full 256-column GEMM alone at one wave
// per SIMD (round-3 PMC: MFMA busy 0.09-0.17, 0.4-1.1 resident waves per SIMD).  Here the CW
// waves of a block share one slab (the same 32 rows) and wave w computes output row blocks
// [w NBW, (w + 1) NBW) of every layer -- its slice of the weight fragments, the whole slab as B --
// so the batch runs CW times the waves at NBW accumulators each (two or more waves per SIMD), and
// every layer boundary is a block barrier (all waves have read the slab before any overwrites it).
// Same operations per output element in the same order: results bit-equal to the per-wave kernel.
// gemm32 with the slab's B operand prefetched PF - 1 k-steps ahead too (rotating registers, as
// the A fragments): the column-split kernels run one row block per wave, one MFMA per k-step,
// where gemm32's in-step ds_read left the LDS latency exposed at ~1 wave per SIMD.  Same MFMAs
// on the same values in the same order.
template <int NB, int PF>
__device__ __forceinline__ void gemm32_pb(f16v (&acc)[NB], const float* __restrict__ A, int nrb,
                                          int rb0, int nks, const float* X, int RS, int kcol,
                                          int act_in) {
  using gptr = const __attribute__((address_space(1))) float*;
  if (nks <= 0) return;
  const int lane = lane_id();
  const int r = lane & 31, h = lane >> 5;
  const float* xr = X + r * RS + kcol + h;
  const gptr Ag = (gptr)(A + (size_t)rb0 * 64 + lane);
  const int stride = nrb * 64;
  int off[NB];
#pragma unroll
  for (int ib = 0; ib < NB; ++ib) off[ib] = (rb0 + ib < nrb ? ib : nrb - 1 - rb0) * 64;
  float a[PF][NB], bq[PF];
#pragma unroll
  for (int p = 0; p < PF; ++p) {
    const int sp = p < nks ? p : nks - 1;
#pragma unroll
    for (int ib = 0; ib < NB; ++ib) a[p][ib] = Ag[(size_t)sp * stride + off[ib]];
    bq[p] = xr[2 * sp];
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
      step(a[p], bq[p]);
      const int sn = s + p + PF < nks ? s + p + PF : nks - 1;
#pragma unroll
      for (int ib = 0; ib < NB; ++ib) a[p][ib] = Ag[(size_t)sn * stride + off[ib]];
      bq[p] = xr[2 * sn];
    }
  }
#pragma unroll
  for (int p = 0; p < PF; ++p)
    if (s + p < nks) step(a[p], bq[p]);
}

template <int NB>
struct ColSplit {
  // row blocks per wave: one (two put the 256-column kernels at the 256-VGPR cap with spills,
  // measured slower than the per-wave kernel)
  static constexpr int NBW = 1;
  static constexpr int CW = NB / NBW;                            // waves per block
};

template <int NB, bool TILE>
__device__ __forceinline__ void mlp_backward_cs(
    const MlpDev* __restrict__ mp, const float* __restrict__ x, const float* __restrict__ lat,
    int64_t M, const float* __restrict__ dY, float* __restrict__ dX, float* __restrict__ dLat,
    float* __restrict__ Zg, float* __restrict__ Ag, float* __restrict__ Eraw,
    float* __restrict__ Eact, float* __restrict__ dZg, float* __restrict__ Et,
    float* __restrict__ Gt, int RS) {
  constexpr int NBW = ColSplit<NB>::NBW, CW = ColSplit<NB>::CW;
  constexpr int PF = 8;
  extern __shared__ float smem[];
  const MlpDev& m = *mp;
  float* X = smem;
  const int lane = lane_id(), r = lane & 31, h = lane >> 5;
  const int w = (int)(threadIdx.x >> 6);
  const int rbw = w * NBW;  // this wave's first output row block
  const int64_t grp = blockIdx.x;
  const int64_t row0 = grp * 32;
  if (row0 >= M) return;  // whole block exits together
  const int64_t row = row0 + r;
  const bool valid = row < M;
  const int64_t rr = valid ? row : M - 1;
  const int H = m.hidden, L = m.n_hidden, ke = m.ke, dp = m.dp, in = m.in_size;
  EncIn e;
  if (in <= 4) {
    for (int i = 0; i < 4; ++i) e.x[i] = (i < in) ? x[rr * in + i] : 0.f;
    e.xg = nullptr;
  } else {
    e.x[0] = e.x[1] = e.x[2] = e.x[3] = 0.f;
    e.xg = x + rr * in;
  }
  e.lat = (lat && m.latent > 0) ? lat + rr * m.latent : nullptr;
  float* rowp = X + r * RS;
  float* const et = TILE ? Et + grp * ke * 32 + r : rowp + H;
  float* const gt = TILE ? Gt + grp * ke * 32 + r : rowp + H;
  constexpr int es = TILE ? 32 : 1;
  // ---- forward, saving Z_l, A_l and the encoding (the waves share the encoding's slot pairs)
  for (int slot = 2 * h + 4 * w; slot < ke; slot += 4 * CW) {
    float a, b;
    enc_pair<false>(m, e, slot, a, b);
    et[slot * es] = a;
    et[(slot + 1) * es] = b;
  }
  __syncthreads();
  if (valid)
    for (int s = h + 2 * w; s < ke; s += 2 * CW) {
      const int c = enc_col(m, s);
      if (c < 0) continue;
      const float v = et[s * es];
      Eraw[row * dp + c] = v;
      Eact[row * dp + c] = act_fwd<false>(v, m.act);
    }
  f16v acc[NBW];
  for (int l = 0; l <= L; ++l) {
    bias32<NBW>(acc, m.bias[l], rbw, NB, h);
    if (l == 0) {
      if (TILE) gemm32_tile<NBW, PF>(acc, m.w32[0], NB, rbw, ke >> 1, et - r, -1);
      else gemm32_pb<NBW, PF>(acc, m.w32[0], NB, rbw, ke >> 1, X, RS, H, -1);
    } else {
      const int i = l - 1;
      gemm32_pb<NBW, PF>(acc, m.w32[l], NB, rbw, H >> 1, X, RS, 0, -1);
      if (i != L - 1 && (i % m.skip) == 0) {
        const float* Ws = m.w32[l] + (H >> 1) * NB * 64;
        if (TILE) gemm32_tile<NBW, PF>(acc, Ws, NB, rbw, ke >> 1, et - r, m.act);
        else gemm32_pb<NBW, PF>(acc, Ws, NB, rbw, ke >> 1, X, RS, H, m.act);
      }
    }
    __syncthreads();  // every wave has read the layer's inputs from the slab
#pragma unroll
    for (int ib = 0; ib < NBW; ++ib)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int k0 = 32 * (rbw + ib) + 8 * g + 4 * h;
        float4 zv, av;
        float* zp = &zv.x;
        float* ap = &av.x;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          zp[j] = acc[ib][4 * g + j];
          ap[j] = act_fwd<false>(zp[j], m.act);
          rowp[k0 + j] = ap[j];
        }
        if (valid) {
          *reinterpret_cast<float4*>(Zg + ((int64_t)l * M + row) * H + k0) = zv;
          *reinterpret_cast<float4*>(Ag + ((int64_t)l * M + row) * H + k0) = av;
        }
      }
    __syncthreads();  // the layer's activations are in the slab
  }
  // ---- backward seed: dZ_L = (dY W_out) * act'(Z_L); the encoding gradient starts at zero.
  // Slot s is accumulated by one wave and lane in every pass (its row block's owner, at the MFMA
  // output position), so only the barrier before dL/dx orders it across waves.
  const float* eraw_row = Eraw + rr * dp;
  for (int s = 4 * h + 8 * w; s < ke; s += 8 * CW)
#pragma unroll
    for (int j = 0; j < 4; ++j) gt[(s + j) * es] = 0.f;
  const float* Ao = m.w32[L + 1];
  const int out = m.out;
  for (int k = h + 2 * w; k < H; k += 2 * CW) {
    float g = 0.f;
    for (int o = 0; o < out; ++o)
      g = fmaf(dY[rr * out + o], Ao[((k >> 1) * m.ob + (o >> 5)) * 64 + (k & 1) * 32 + (o & 31)], g);
    rowp[k] = g * act_bwd(Zg[((int64_t)L * M + rr) * H + k], m.act);
  }
  __syncthreads();
  for (int l = L; l >= 0; --l) {
    if (valid)
      for (int k = 4 * h + 8 * w; k < H; k += 8 * CW)
        *reinterpret_cast<float4*>(dZg + ((int64_t)l * M + row) * H + k) =
            make_float4(rowp[k], rowp[k + 1], rowp[k + 2], rowp[k + 3]);
    const float* At = m.wt32[l];
    const int nrb = m.nbt[l];
    const bool has_hidden_in = (l != 0);
    const bool has_enc_in = (l == 0) || ((l - 1) != L - 1 && ((l - 1) % m.skip) == 0);
    const int hid_rb = has_hidden_in ? NB : 0;
    if (has_enc_in) {
      const int enc_pos0 = has_hidden_in ? H : 0;
      for (int rb0 = hid_rb + rbw; rb0 < nrb; rb0 += NB) {
#pragma unroll
        for (int ib = 0; ib < NBW; ++ib) acc[ib] = f16v{};
        gemm32_pb<NBW, PF>(acc, At, nrb, rb0, H >> 1, X, RS, 0, -1);
        // per row block: every load first (clamped addresses, unconditional), then the
        // activation's branches
#pragma unroll
        for (int ib = 0; ib < NBW; ++ib) {
          if (rb0 + ib >= nrb) continue;
          float ev[16], gv[16];
#pragma unroll
          for (int reg = 0; reg < 16; ++reg) {
            const int pos = 32 * (rb0 + ib) + (reg & 3) + 8 * (reg >> 2) + 4 * h;
            const int slot = min(max(pos - enc_pos0, 0), ke - 1);
            const int c = l != 0 ? enc_col(m, slot) : -1;
            ev[reg] = eraw_row[c < 0 ? 0 : c];
            gv[reg] = gt[slot * es];
          }
#pragma unroll
          for (int reg = 0; reg < 16; ++reg) {
            const int pos = 32 * (rb0 + ib) + (reg & 3) + 8 * (reg >> 2) + 4 * h;
            const int slot = pos - enc_pos0;
            if (slot >= 0 && slot < ke) {
              float v = acc[ib][reg];
              if (l != 0) {  // skip inputs are act(enc)
                const int c = enc_col(m, slot);
                v = c < 0 ? 0.f : v * act_bwd(ev[reg], m.act);
              }
              gt[slot * es] = gv[reg] + v;
            }
          }
        }
      }
    }
    if (has_hidden_in) {
#pragma unroll
      for (int ib = 0; ib < NBW; ++ib) acc[ib] = f16v{};
      gemm32_pb<NBW, PF>(acc, At, nrb, rbw, H >> 1, X, RS, 0, -1);
    }
    __syncthreads();  // every wave has read dZ_l from the slab
    if (has_hidden_in) {
#pragma unroll
      for (int ib = 0; ib < NBW; ++ib) {
        float4 zq[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          zq[q] = *reinterpret_cast<const float4*>(Zg + ((int64_t)(l - 1) * M + rr) * H + 32 * (rbw + ib) + 8 * q + 4 * h);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int k0 = 32 * (rbw + ib) + 8 * q + 4 * h;
          const float* zp = &zq[q].x;
#pragma unroll
          for (int j = 0; j < 4; ++j) rowp[k0 + j] = acc[ib][4 * q + j] * act_bwd(zp[j], m.act);
        }
      }
      __syncthreads();
    }
  }
  // ---- encoding -> inputs (every wave's slots of the encoding gradient: the barrier above)
  const float* egrad = gt;
  const int F = m.freqs;
  for (int i = w; i < in; i += CW) {
    float g = 0.f;
    for (int q = h; q < F; q += 2) {
      float s, c;
      sincosf(proj<false>(m, e, q), &s, &c);
      g = fmaf(egrad[es * (2 * q)] * c - egrad[es * (2 * q + 1)] * s, m.basis[i * F + q], g);
    }
    if (h == 0) g += egrad[es * (2 * F + i)];
    g += __shfl_xor(g, 32);
    if (dX && valid && h == 0) dX[row * in + i] = g;
  }
  if (dLat && valid)
    for (int j = h + 2 * w; j < m.latent; j += 2 * CW) dLat[row * m.latent + j] = egrad[es * (2 * F + in + j)];
}

template <int NB, bool TILE>
__global__ void __launch_bounds__(64 * ColSplit<NB>::CW, 2) k_mlp_backward32_cs(
    const MlpDev* __restrict__ mp, const float* __restrict__ x, const float* __restrict__ lat,
    int64_t M, const float* __restrict__ dY, float* __restrict__ dX, float* __restrict__ dLat,
    float* __restrict__ Zg, float* __restrict__ Ag, float* __restrict__ Eraw,
    float* __restrict__ Eact, float* __restrict__ dZg, float* __restrict__ Et,
    float* __restrict__ Gt, int RS) {
  mlp_backward_cs<NB, TILE>(mp, x, lat, M, dY, dX, dLat, Zg, Ag, Eraw, Eact, dZg, Et, Gt, RS);
}

struct BwdJob;
template <int NB, bool TILE>
__global__ void __launch_bounds__(64 * ColSplit<NB>::CW, 2) k_mlp_backward32_multi_cs(
    const BwdJob* __restrict__ jobs, const float* __restrict__ x, int64_t M, int RS);

// below four row blocks two waves per SIMD fit (registers and slab): ask the compiler for that
template <int NB, bool TILE>
__global__ void __launch_bounds__(256, NB <= 4 ? 2 : 1) k_mlp_backward32(
    const MlpDev* __restrict__ mp, const float* __restrict__ x, const float* __restrict__ lat,
    int64_t M, const float* __restrict__ dY, float* __restrict__ dX, float* __restrict__ dLat,
    float* __restrict__ Zg, float* __restrict__ Ag, float* __restrict__ Eraw,
    float* __restrict__ Eact, float* __restrict__ dZg, float* __restrict__ Et,
    float* __restrict__ Gt, int RS, int per_wave) {
  mlp_backward32<NB, TILE>(mp, x, lat, M, dY, dX, dLat, Zg, Ag, Eraw, Eact, dZg, Et, Gt, RS, per_wave);
}

// n same-shape MLPs on one input (the NeuralBSDFs of a spatially varying mixture all read the
// same Rusinkiewicz features): one launch, blockIdx.y = MLP.  Each MLP alone is 1,200 32-row waves
// on 1,024 SIMDs for a 38,400-ray training batch; together they fill the machine.
struct BwdJob {
  const MlpDev* mp;
  const float* dY;
  float *dX, *Z, *A, *Eraw, *Eact, *dZ, *Et, *Gt;
};

template <int NB, bool TILE>
__global__ void __launch_bounds__(256, NB <= 4 ? 2 : 1) k_mlp_backward32_multi(
    const BwdJob* __restrict__ jobs, const float* __restrict__ x, int64_t M, int RS, int per_wave) {
  const BwdJob j = jobs[blockIdx.y];
  mlp_backward32<NB, TILE>(j.mp, x, nullptr, M, j.dY, j.dX, nullptr, j.Z, j.A, j.Eraw, j.Eact,
                           j.dZ, j.Et, j.Gt, RS, per_wave);
}

template <int NB, bool TILE>
__global__ void __launch_bounds__(64 * ColSplit<NB>::CW, 2) k_mlp_backward32_multi_cs(
    const BwdJob* __restrict__ jobs, const float* __restrict__ x, int64_t M, int RS) {
  const BwdJob j = jobs[blockIdx.y];
  mlp_backward_cs<NB, TILE>(j.mp, x, nullptr, M, j.dY, j.dX, nullptr, j.Z, j.A, j.Eraw, j.Eact,
                            j.dZ, j.Et, j.Gt, RS);
}

// second derivative of act at pre-activation x (torch double-backward formulas:
// softplus_double_backward = s(1-s) where x < threshold, sigmoid: s(1-s)(1-2s), piecewise-linear: 0)
__device__ __forceinline__ float act_bwd2(float x, int act) {
  switch (act) {
    case ACT_SOFTPLUS: {
      if (!(x < 20.f)) return 0.f;
      const float s = 1.f / (1.f + expf(-x));
      return s * (1.f - s);
    }
    case ACT_SIGMOID: {
      const float s = 1.f / (1.f + expf(-x));
      return s * (1.f - s) * (1.f - 2.f * s);
    }
    default: return 0.f;
  }
}

// Double backward of the input gradient g(x) = d(sum_o y_o)/dx (SDF.autograd_diff with
// create_graph=True, sdfs.py:184-197): the parameter gradients of J = sum_rows v . g(x) for a
// given v = dL/dg.  J is the forward-mode derivative of sum_o y_o along v, so one pass runs the
// MLP forward with a tangent (z_l, zt_l = W_l tangent-inputs), then the reverse of both chains:
//   zt_bar = at_bar act'(z),   z_bar = a_bar act'(z) + at_bar act''(z) zt,
//   a_bar(l-1) = W_l^T z_bar,   at_bar(l-1) = W_l^T zt_bar     (hidden inputs; at_bar_L = W_out^T 1)
// and dW_l = z_bar^T In_l + zt_bar^T InT_l, db_l = sum z_bar, done afterwards as one GEMM over the
// stacked [primal; tangent] rows.  Slab row: [a | enc | enc tangent | a tangent].
template <int NB>
__global__ void __launch_bounds__(256, NB <= 4 ? 2 : 1) k_mlp_grad_backward32(
    const MlpDev* __restrict__ mp, const float* __restrict__ x, const float* __restrict__ lat,
    const float* __restrict__ v, int64_t M, float* __restrict__ Zg, float* __restrict__ Tg,
    float* __restrict__ Ag, float* __restrict__ E0, float* __restrict__ E1,
    float* __restrict__ dZg, int RS, int per_wave) {
  extern __shared__ float smem[];
  const MlpDev& m = *mp;
  float* X = smem + (size_t)(threadIdx.x >> 6) * per_wave;
  const int lane = lane_id(), r = lane & 31, h = lane >> 5;
  const int64_t row0 = wave_global() * 32;
  if (row0 >= M) return;  // whole wave exits together
  const int64_t row = row0 + r;
  const bool valid = row < M;
  const int64_t rr = valid ? row : M - 1;
  const int H = m.hidden, L = m.n_hidden, ke = m.ke, dp = m.dp, in = m.in_size, F = m.freqs;
  const int EE = H, ET = H + ke, PT = H + 2 * ke;
  const int64_t M2 = 2 * M;
  EncIn e;
  if (in <= 4) {
    for (int i = 0; i < 4; ++i) e.x[i] = (i < in) ? x[rr * in + i] : 0.f;
    e.xg = nullptr;
  } else {
    e.x[0] = e.x[1] = e.x[2] = e.x[3] = 0.f;
    e.xg = x + rr * in;
  }
  e.lat = (lat && m.latent > 0) ? lat + rr * m.latent : nullptr;
  float* rowp = X + r * RS;
  const float* vr = v + rr * in;
  // ---- encoding and its tangent along v: d sin(xB_q) = cos(xB_q) (vB)_q, d cos = -sin (vB)_q
  write_enc_slab<false>(m, e, X, RS);
  for (int s = h; s < ke; s += 2) {
    float tv = 0.f;
    if (s < 2 * F) {
      const int q = s >> 1;
      float vb = vr[0] * m.basis[q];
      for (int i = 1; i < in; ++i) vb = fmaf(vr[i], m.basis[i * F + q], vb);
      float sn, cs;
      sincosf(proj<false>(m, e, q), &sn, &cs);
      tv = (s & 1) ? -sn * vb : cs * vb;
    } else if (s < 2 * F + in) {
      tv = vr[s - 2 * F];
    }
    rowp[ET + s] = tv;
  }
  wave_lds_fence();
  if (valid)
    for (int s = h; s < ke; s += 2) {
      const int c = enc_col(m, s);
      if (c < 0) continue;
      const float ev = rowp[EE + s], tv = rowp[ET + s];
      E0[row * dp + c] = ev;
      E0[(M + row) * dp + c] = tv;
      E1[row * dp + c] = act_fwd<false>(ev, m.act);
      E1[(M + row) * dp + c] = act_bwd(ev, m.act) * tv;
    }
  // ---- forward: primal then tangent per layer
  f16v acc[NB];
  for (int l = 0; l <= L; ++l) {
    const bool skip = l > 0 && (l - 1) != L - 1 && ((l - 1) % m.skip) == 0;
    bias32<NB>(acc, m.bias[l], 0, NB, h);
    if (l == 0) {
      gemm32<NB, train_pf(NB)>(acc, m.w32[0], NB, 0, ke >> 1, X, RS, EE, -1);
    } else {
      gemm32<NB, train_pf(NB)>(acc, m.w32[l], NB, 0, H >> 1, X, RS, 0, -1);
      if (skip) gemm32<NB, train_pf(NB)>(acc, m.w32[l] + (H >> 1) * NB * 64, NB, 0, ke >> 1, X, RS, EE, m.act);
    }
    wave_lds_fence();
#pragma unroll
    for (int ib = 0; ib < NB; ++ib)
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int k = 32 * ib + (reg & 3) + 8 * (reg >> 2) + 4 * h;
        const float z = acc[ib][reg];
        const float a = act_fwd<false>(z, m.act);
        if (valid) {
          Zg[((int64_t)l * M + row) * H + k] = z;
          Ag[((int64_t)l * M2 + row) * H + k] = a;
        }
        rowp[k] = a;
      }
    wave_lds_fence();
#pragma unroll
    for (int ib = 0; ib < NB; ++ib) acc[ib] = f16v{};
    if (l == 0) {
      gemm32<NB, train_pf(NB)>(acc, m.w32[0], NB, 0, ke >> 1, X, RS, ET, -1);
    } else {
      gemm32<NB, train_pf(NB)>(acc, m.w32[l], NB, 0, H >> 1, X, RS, PT, -1);
      if (skip) gemm32<NB, train_pf(NB)>(acc, m.w32[l] + (H >> 1) * NB * 64, NB, 0, ke >> 1, X, RS, ET, -1);
    }
    wave_lds_fence();
#pragma unroll
    for (int ib = 0; ib < NB; ++ib)
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int k = 32 * ib + (reg & 3) + 8 * (reg >> 2) + 4 * h;
        const float zt = acc[ib][reg];
        const float z = valid ? Zg[((int64_t)l * M + row) * H + k] : 0.f;
        const float at = act_bwd(z, m.act) * zt;
        if (valid) {
          Tg[((int64_t)l * M + row) * H + k] = zt;
          Ag[((int64_t)l * M2 + M + row) * H + k] = at;
        }
        rowp[PT + k] = at;
      }
    if (l == 0)  // skip layers consume act(enc): tangent act'(enc) * enc tangent
      for (int s = h; s < ke; s += 2) rowp[ET + s] = act_bwd(rowp[EE + s], m.act) * rowp[ET + s];
    wave_lds_fence();
  }
  // ---- reverse: seed a_bar_L = 0, at_bar_L = W_out^T 1
  const float* Ao = m.w32[L + 1];
  for (int k = h; k < H; k += 2) {
    float g = 0.f;
    for (int o = 0; o < m.out; ++o) g += Ao[((k >> 1) * m.ob + (o >> 5)) * 64 + (k & 1) * 32 + (o & 31)];
    rowp[k] = 0.f;
    rowp[PT + k] = g;
  }
  wave_lds_fence();
  for (int l = L; l >= 0; --l) {
    for (int k = h; k < H; k += 2) {
      const float z = valid ? Zg[((int64_t)l * M + row) * H + k] : 0.f;
      const float zt = valid ? Tg[((int64_t)l * M + row) * H + k] : 0.f;
      const float d1 = act_bwd(z, m.act);
      const float ab = rowp[k], atb = rowp[PT + k];
      const float zb = ab * d1 + atb * act_bwd2(z, m.act) * zt;
      const float ztb = atb * d1;
      rowp[k] = zb;
      rowp[PT + k] = ztb;
      if (valid) {
        dZg[((int64_t)l * M2 + row) * H + k] = zb;
        dZg[((int64_t)l * M2 + M + row) * H + k] = ztb;
      }
    }
    wave_lds_fence();
    if (l == 0) break;
    const float* At = m.wt32[l];
    const int nrb = m.nbt[l];
    for (int pass = 0; pass < 2; ++pass) {
      const int col = pass ? PT : 0;
#pragma unroll
      for (int ib = 0; ib < NB; ++ib) acc[ib] = f16v{};
      gemm32<NB, train_pf(NB)>(acc, At, nrb, 0, H >> 1, X, RS, col, -1);
      wave_lds_fence();
#pragma unroll
      for (int ib = 0; ib < NB; ++ib)
#pragma unroll
        for (int reg = 0; reg < 16; ++reg)
          rowp[col + 32 * ib + (reg & 3) + 8 * (reg >> 2) + 4 * h] = acc[ib][reg];
      wave_lds_fence();
    }
  }
}

// Column-split variant of k_mlp_grad_backward32 (as mlp_backward_cs): one block of NB waves per
// 32 rows sharing one slab, wave w computing output row block w of every layer's primal and
// tangent GEMMs (both before one barrier, then both writes).  The [a | enc | enc tangent | a
// tangent] slab row (~53 KB a wave for the 8x128 SDF shift) held the per-wave kernel at three
// waves per CU; here three blocks of four waves fit.  Same operations per element: bit-equal.
template <int NB>
__global__ void __launch_bounds__(64 * NB, 2) k_mlp_grad_backward32_cs(
    const MlpDev* __restrict__ mp, const float* __restrict__ x, const float* __restrict__ lat,
    const float* __restrict__ v, int64_t M, float* __restrict__ Zg, float* __restrict__ Tg,
    float* __restrict__ Ag, float* __restrict__ E0, float* __restrict__ E1,
    float* __restrict__ dZg, int RS) {
  constexpr int CW = NB, PF = 8;
  extern __shared__ float smem[];
  const MlpDev& m = *mp;
  float* X = smem;
  const int lane = lane_id(), r = lane & 31, h = lane >> 5;
  const int w = (int)(threadIdx.x >> 6);
  const int64_t row0 = (int64_t)blockIdx.x * 32;
  if (row0 >= M) return;  // whole block exits together
  const int64_t row = row0 + r;
  const bool valid = row < M;
  const int64_t rr = valid ? row : M - 1;
  const int H = m.hidden, L = m.n_hidden, ke = m.ke, dp = m.dp, in = m.in_size, F = m.freqs;
  const int EE = H, ET = H + ke, PT = H + 2 * ke;
  const int64_t M2 = 2 * M;
  EncIn e;
  if (in <= 4) {
    for (int i = 0; i < 4; ++i) e.x[i] = (i < in) ? x[rr * in + i] : 0.f;
    e.xg = nullptr;
  } else {
    e.x[0] = e.x[1] = e.x[2] = e.x[3] = 0.f;
    e.xg = x + rr * in;
  }
  e.lat = (lat && m.latent > 0) ? lat + rr * m.latent : nullptr;
  float* rowp = X + r * RS;
  const float* vr = v + rr * in;
  // ---- encoding (write_enc_slab's pairs, shared by the waves) and its tangent along v
  for (int slot = 2 * h + 4 * w; slot < ke; slot += 4 * CW) {
    float a, b;
    enc_pair<false>(m, e, slot, a, b);
    rowp[EE + slot] = a;
    rowp[EE + slot + 1] = b;
  }
  for (int s = h + 2 * w; s < ke; s += 2 * CW) {
    float tv = 0.f;
    if (s < 2 * F) {
      const int q = s >> 1;
      float vb = vr[0] * m.basis[q];
      for (int i = 1; i < in; ++i) vb = fmaf(vr[i], m.basis[i * F + q], vb);
      float sn, cs;
      sincosf(proj<false>(m, e, q), &sn, &cs);
      tv = (s & 1) ? -sn * vb : cs * vb;
    } else if (s < 2 * F + in) {
      tv = vr[s - 2 * F];
    }
    rowp[ET + s] = tv;
  }
  __syncthreads();
  if (valid)
    for (int s = h + 2 * w; s < ke; s += 2 * CW) {
      const int c = enc_col(m, s);
      if (c < 0) continue;
      const float ev = rowp[EE + s], tv = rowp[ET + s];
      E0[row * dp + c] = ev;
      E0[(M + row) * dp + c] = tv;
      E1[row * dp + c] = act_fwd<false>(ev, m.act);
      E1[(M + row) * dp + c] = act_bwd(ev, m.act) * tv;
    }
  // ---- forward: primal and tangent GEMMs of a layer, one barrier, then both writes
  f16v acc[1], act_[1];
  for (int l = 0; l <= L; ++l) {
    const bool skip = l > 0 && (l - 1) != L - 1 && ((l - 1) % m.skip) == 0;
    bias32<1>(acc, m.bias[l], w, NB, h);
    act_[0] = f16v{};
    if (l == 0) {
      gemm32_pb<1, PF>(acc, m.w32[0], NB, w, ke >> 1, X, RS, EE, -1);
      gemm32_pb<1, PF>(act_, m.w32[0], NB, w, ke >> 1, X, RS, ET, -1);
    } else {
      gemm32_pb<1, PF>(acc, m.w32[l], NB, w, H >> 1, X, RS, 0, -1);
      if (skip) gemm32_pb<1, PF>(acc, m.w32[l] + (H >> 1) * NB * 64, NB, w, ke >> 1, X, RS, EE, m.act);
      gemm32_pb<1, PF>(act_, m.w32[l], NB, w, H >> 1, X, RS, PT, -1);
      if (skip) gemm32_pb<1, PF>(act_, m.w32[l] + (H >> 1) * NB * 64, NB, w, ke >> 1, X, RS, ET, -1);
    }
    __syncthreads();  // every wave has read the layer's inputs
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int k = 32 * w + (reg & 3) + 8 * (reg >> 2) + 4 * h;
      const float z = acc[0][reg], zt = act_[0][reg];
      const float a = act_fwd<false>(z, m.act);
      const float at = act_bwd(valid ? z : 0.f, m.act) * zt;
      if (valid) {
        Zg[((int64_t)l * M + row) * H + k] = z;
        Ag[((int64_t)l * M2 + row) * H + k] = a;
        Tg[((int64_t)l * M + row) * H + k] = zt;
        Ag[((int64_t)l * M2 + M + row) * H + k] = at;
      }
      rowp[k] = a;
      rowp[PT + k] = at;
    }
    if (l == 0)  // skip layers consume act(enc): tangent act'(enc) * enc tangent
      for (int s = h + 2 * w; s < ke; s += 2 * CW) rowp[ET + s] = act_bwd(rowp[EE + s], m.act) * rowp[ET + s];
    __syncthreads();
  }
  // ---- reverse: seed a_bar_L = 0, at_bar_L = W_out^T 1
  const float* Ao = m.w32[L + 1];
  for (int k = h + 2 * w; k < H; k += 2 * CW) {
    float g = 0.f;
    for (int o = 0; o < m.out; ++o) g += Ao[((k >> 1) * m.ob + (o >> 5)) * 64 + (k & 1) * 32 + (o & 31)];
    rowp[k] = 0.f;
    rowp[PT + k] = g;
  }
  __syncthreads();
  for (int l = L; l >= 0; --l) {
    for (int k = h + 2 * w; k < H; k += 2 * CW) {
      const float z = valid ? Zg[((int64_t)l * M + row) * H + k] : 0.f;
      const float zt = valid ? Tg[((int64_t)l * M + row) * H + k] : 0.f;
      const float d1 = act_bwd(z, m.act);
      const float ab = rowp[k], atb = rowp[PT + k];
      const float zb = ab * d1 + atb * act_bwd2(z, m.act) * zt;
      const float ztb = atb * d1;
      rowp[k] = zb;
      rowp[PT + k] = ztb;
      if (valid) {
        dZg[((int64_t)l * M2 + row) * H + k] = zb;
        dZg[((int64_t)l * M2 + M + row) * H + k] = ztb;
      }
    }
    __syncthreads();
    if (l == 0) break;
    const float* At = m.wt32[l];
    const int nrb = m.nbt[l];
    acc[0] = f16v{};
    act_[0] = f16v{};
    gemm32_pb<1, PF>(acc, At, nrb, w, H >> 1, X, RS, 0, -1);
    gemm32_pb<1, PF>(act_, At, nrb, w, H >> 1, X, RS, PT, -1);
    __syncthreads();
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int k = 32 * w + (reg & 3) + 8 * (reg >> 2) + 4 * h;
      rowp[k] = acc[0][reg];
      rowp[PT + k] = act_[0][reg];
    }
    __syncthreads();
  }
}

template <int = 0>
__global__ void k_fill(float* __restrict__ p, int64_t n, float v) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] = v;
}

namespace {
size_t a256(size_t v) { return (v + 255) & ~(size_t)255; }

// Algorithmic FLOP per row (2 per multiply-add, real widths) for nrt_profile_flop: a forward
// through the layers below the out layer (init, hidden, skip parts); the backward kernel is that
// recompute plus the input gradient of every one of those layers and the out layer's seed; the
// double backward runs the primal and tangent forwards and the two hidden reverse chains.
double fwd_row_flop(const MlpDev& d) {
  const int L = d.n_hidden, H = d.hidden;
  double f = 2.0 * d.dp * H;
  for (int i = 0; i < L; ++i) {
    const bool skip = i != L - 1 && (i % d.skip) == 0;
    f += 2.0 * H * (H + (skip ? d.dp : 0));
  }
  return f;
}
double bwd_row_flop(const MlpDev& d) { return 2.0 * fwd_row_flop(d) + 2.0 * d.out * d.hidden; }
double grad_bwd_row_flop(const MlpDev& d) {
  return 2.0 * fwd_row_flop(d) + 4.0 * d.hidden * d.hidden * d.n_hidden;
}

constexpr size_t kWgradTableBytes = 16384;  // device copy of a WgradBatch's job table

struct TrainWs {
  float *Z, *A, *dZ, *Eraw, *Eact, *Et, *Gt, *table, *part;
};

// per-wave encoding / encoding-gradient tiles of k_mlp_backward32: [waves][ke][32] floats
static inline size_t enc_tile_bytes(const MlpDev& d, int64_t M) {
  return (size_t)((M + 31) / 32) * 32 * (size_t)d.ke * 4;
}

TrainWs carve(const nrt_mlp* m, int64_t M, void* base) {
  const MlpDev& d = m->host_dev;
  const size_t lay = (size_t)(d.n_hidden + 1) * (size_t)M * d.hidden * 4;
  const size_t enc = (size_t)M * d.dp * 4;
  char* p = (char*)base;
  TrainWs w;
  w.Z = (float*)p; p += a256(lay);
  w.A = (float*)p; p += a256(lay);
  w.dZ = (float*)p; p += a256(lay);
  w.Eraw = (float*)p; p += a256(enc);
  w.Eact = (float*)p; p += a256(enc);
  w.Et = (float*)p; p += a256(enc_tile_bytes(d, M));
  w.Gt = (float*)p; p += a256(enc_tile_bytes(d, M));
  w.table = (float*)p; p += a256(kWgradTableBytes);  // weight-gradient job table
  w.part = (float*)p;  // batched partial products
  return w;
}

}  // namespace
// (outside the anonymous namespace: the HIP runtime could not find k_wgrad's device symbol under
// internal linkage -- "Cannot find Symbol with name: _ZN3nrt12_GLOBAL__N_17k_wgrad...")

// Split-K weight gradients.  dW = dZ^T In has a small output (R x C <= 256 x 550) and a long K
// (the batch, ~10^4-10^5): the batch is cut into S slices, one block computes one 64 x 64 output
// tile of one slice on exact-f32 MFMA (v_mfma_f32_32x32x2_f32, an fma chain) with a 2 x 2 grid of
// 32x32 accumulators -- wave w of kWgradWaves takes the slice's groups of 16 rows w, w +
// kWgradWaves, ...; lane (i = l & 31, h = l >> 5) loads dZ[m + h][r0 + 32a + i] (the A operand,
// dZ^T) and In[m + h][c0 + 32b + i] (B), 128-byte row segments per half-wave -- then the waves'
// accumulators are summed in wave order through LDS and the slice partials in slice order
// (deterministic).  S is chosen from the shapes alone (same inputs, same bits).
constexpr int kSplitMax = 64;
#ifndef NRT_WG_SLICE_ROWS
#define NRT_WG_SLICE_ROWS 256
#endif
#ifndef NRT_WG_U
#define NRT_WG_U 8
#endif
#ifndef NRT_WG_WPE
#define NRT_WG_WPE 3
#endif
constexpr int64_t kSliceRows = NRT_WG_SLICE_ROWS;  // batch rows per slice at least
constexpr int kWgradWaves = 4;        // waves per block

// ---- every weight and bias gradient of one backward call in two launches --------------------
// A job is dW[r][c0 + c] (ldw) = sum_m dZ[m][r] In[m][c] (row-major dZ [M][R], In [M][ldi]), or
// (bias) db[r] = sum_m dZ[m][r] -- the same product with In a column of ones.  All jobs share the
// slice count S (from the shapes alone: same inputs, same bits); blocks are (job, 64 x 64 tile,
// slice), the partials of slice s of job j sit at part + part_off + s R C, and k_split_reduce_batch
// sums them in slice order.  Per training step this replaces ~500 launches (round 2: a k_wgrad +
// k_split_reduce pair per layer part, two column-sum launches per bias) by two per MLP backward.
struct WgradJob {
  const float* dZ;
  const float* In;   // nullptr: bias job (a column of ones)
  float* dW;
  int64_t M, slice_rows, part_off, out0;
  int R, C, ldi, ldw, c0, tiles_c, n_tiles, block0;
  int bias;  // 1: db = the column sums of dZ (In unused)
  // k_wgrad_tile: this weight job's c0 = 0 tiles also sum dZ's rows below bias_M into the partials
  // at bias_off (a bias job's, which then has no blocks of its own); -1: none
  int64_t bias_off, bias_M;
};

template <int = 0>
__global__ void __launch_bounds__(64 * kWgradWaves) __attribute__((amdgpu_waves_per_eu(NRT_WG_WPE))) k_wgrad_batch(
    const WgradJob* __restrict__ jobs, int n_jobs, int S, float* __restrict__ part) {
  typedef float f16v_ __attribute__((ext_vector_type(16)));
  __shared__ float red[kWgradWaves - 1][16][64];
  int j = 0;
  while (j + 1 < n_jobs && (int)blockIdx.x >= jobs[j + 1].block0) ++j;
  const WgradJob& jb = jobs[j];
  const int b = (int)blockIdx.x - jb.block0;
  const int tile = b % jb.n_tiles, slice = b / jb.n_tiles;
  const float* __restrict__ dZ = jb.dZ;
  const float* __restrict__ In = jb.In;
  const int R = jb.R, C = jb.C, ldi = jb.ldi;
  const int w = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63, i = lane & 31, h = lane >> 5;
  const int r0 = (tile / jb.tiles_c) * 64, c0 = (tile % jb.tiles_c) * 64;
  const int64_t m0 = (int64_t)slice * jb.slice_rows;
  const int64_t m1 = std::min<int64_t>(jb.M, m0 + jb.slice_rows);
  f16v_ acc[4] = {};
  constexpr int U = NRT_WG_U;  // k-steps (2 rows each) per group
  // clamped indices as in k_wgrad: loads are unconditional, rows past the slice are zeroed in
  // the A operand, clamped columns / rows feed only outputs that are never stored
  const int ia = std::min(r0 + i, R - 1), ib = std::min(r0 + 32 + i, R - 1);
  const int ja = std::min(c0 + i, C - 1), jbb = std::min(c0 + 32 + i, C - 1);
  // software-pipelined over groups of U k-steps: group g + 1's loads are in flight while group
  // g's MFMAs run (two register sets, the loop unrolled by two)
  struct Grp { float a0[U], a1[U], b0[U], b1[U]; int ok; };
  auto load = [&](Grp& q, int64_t m) {
    q.ok = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t row = m + 2 * u + h;
      q.ok |= row < m1 ? (1 << u) : 0;
      const int64_t rc = row < m1 ? row : m1 - 1;
      const float* zr = dZ + rc * R;
      q.a0[u] = zr[ia]; q.a1[u] = zr[ib];
      if (In) {
        const float* ir = In + rc * ldi;
        q.b0[u] = ir[ja]; q.b1[u] = ir[jbb];
      } else {
        q.b0[u] = 1.f; q.b1[u] = 1.f;
      }
    }
  };
  auto mma = [&](const Grp& q) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool o = (q.ok >> u) & 1;
      const float x0 = o ? q.a0[u] : 0.f, x1 = o ? q.a1[u] : 0.f;
      acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(x0, q.b0[u], acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(x0, q.b1[u], acc[1], 0, 0, 0);
      acc[2] = __builtin_amdgcn_mfma_f32_32x32x2f32(x1, q.b0[u], acc[2], 0, 0, 0);
      acc[3] = __builtin_amdgcn_mfma_f32_32x32x2f32(x1, q.b1[u], acc[3], 0, 0, 0);
    }
  };
  const int64_t gstep = (int64_t)kWgradWaves * 2 * U;
  int64_t m = m0 + (int64_t)w * 2 * U;
  Grp g0, g1;
  if (m < m1) load(g0, m);
  while (m < m1) {
    const int64_t mn = m + gstep;
    if (mn < m1) load(g1, mn);
    mma(g0);
    m = mn;
    if (m >= m1) break;
    const int64_t mn2 = m + gstep;
    if (mn2 < m1) load(g0, mn2);
    mma(g1);
    m = mn2;
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    if (w > 0) {
#pragma unroll
      for (int q = 0; q < 16; ++q) red[w - 1][q][lane] = acc[t][q];
    }
    __syncthreads();
    if (w == 0) {
#pragma unroll
      for (int v = 0; v < kWgradWaves - 1; ++v)
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[t][q] += red[v][q][lane];
    }
    __syncthreads();
  }
  if (w != 0) return;
  float* out = part + jb.part_off + (size_t)slice * R * C;
  const bool cok[2] = {c0 + i < C, c0 + 32 + i < C};
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int rr = r0 + 32 * (t >> 1) + (q & 3) + 8 * (q >> 2) + 4 * h;
      if (rr < R && cok[t & 1]) out[(size_t)rr * C + c0 + 32 * (t & 1) + i] = acc[t][q];
    }
}

// ---- LDS-staged weight gradients (option "wgrad_tile"; measured 10 % slower than k_wgrad_batch
// on the training step: MFMA busy 0.36 vs 0.51, 32 % of wave time parked at the stage barriers,
// 1.85 waves per SIMD; profiles/r05/probe/pmc_wgrad_stall.txt) ----------------------------------
// k_wgrad_batch feeds each MFMA from 4-byte global loads in the MFMA's lane order and, with 64 x 64
// tiles, reads a 256-wide layer's dZ and In slices four times each (16 FLOP per byte fetched;
// round-4 PMC: 65-75 % of wave time waiting at ~0.5 MFMA busy).  Here a block of four waves
// computes a 128 x 128 output tile over its slice of the batch -- operands read twice per layer,
// 32 FLOP per byte -- with the rows streaming through three LDS stages of 16 rows ([16][128 + 1]
// floats of dZ and of In: coalesced 512-byte row segments, loaded two stages ahead into registers
// so ~4k cycles of MFMA cover each load).  Wave (wr, wc) takes rows 64 wr .., columns 64 wc .. of
// the tile as 2 x 2 v_mfma_f32_32x32x2_f32 accumulators with operands read from LDS.  Exact f32,
// each output's products in row order within the slice (deterministic).  The bias gradient of a
// layer (dZ's column sums) rides on the layer's first weight tiles (c0 = 0): the staged dZ rows are
// summed from LDS (bias_off / bias_M); a bias job with no such weight job (the double backward's
// biases over the primal half of the stacked rows) is a column sum of its own (wave-parallel).
// A round-5 256 x 256 / 8-wave version of this kernel ran at one wave per SIMD on these batches and
// with the biases as per-thread load chains: 2x slower than k_wgrad_batch.
constexpr int kWgT = 128;   // tile side
constexpr int kWgKS = 16;   // rows per LDS stage
constexpr int kWgNS = 3;    // stages
constexpr int kWgLd = kWgT + 1;
constexpr int kWgThreads = 256;  // four waves, 2 x 2 of 64 x 64

template <int = 0>
__global__ void __launch_bounds__(kWgThreads, 3) k_wgrad_tile(const WgradJob* __restrict__ jobs, int n_jobs,
                                                              int S, float* __restrict__ part) {
  typedef float f16v_ __attribute__((ext_vector_type(16)));
  extern __shared__ float wsm[];  // [kWgNS][2][kWgKS][kWgLd]
  int j = 0;
  while (j + 1 < n_jobs && (int)blockIdx.x >= jobs[j + 1].block0) ++j;
  const WgradJob& jb = jobs[j];
  const int b = (int)blockIdx.x - jb.block0;
  const int tile = b % jb.n_tiles, slice = b / jb.n_tiles;
  const float* __restrict__ dZ = jb.dZ;
  const float* __restrict__ In = jb.In;
  const int R = jb.R, C = jb.C, ldi = jb.ldi;
  const int64_t m0 = (int64_t)slice * jb.slice_rows;
  const int64_t m1 = std::min<int64_t>(jb.M, m0 + jb.slice_rows);
  const int t = threadIdx.x;
  const int w = t >> 6, lane = t & 63, i = lane & 31, h = lane >> 5;
  float* out = part + jb.part_off + (size_t)slice * R * C;
  if (jb.bias) {  // a bias job of its own: column sums over the slice, wave w takes rows w, w + 4 ..
    constexpr int NW = kWgThreads / 64;
    __shared__ float red[NW - 1][256];
    for (int cb = 0; cb < R; cb += 256) {  // columns cb + lane + 64 q
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
      for (int64_t m = m0 + w; m < m1; m += NW) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (cb + lane + 64 * q < R) acc[q] += dZ[m * R + cb + lane + 64 * q];
      }
      if (w > 0)
#pragma unroll
        for (int q = 0; q < 4; ++q) red[w - 1][lane + 64 * q] = acc[q];
      __syncthreads();
      if (w == 0)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float v = acc[q];
#pragma unroll
          for (int k = 0; k < NW - 1; ++k) v += red[k][lane + 64 * q];
          if (cb + lane + 64 * q < R) out[cb + lane + 64 * q] = v;
        }
      __syncthreads();
    }
    return;
  }
  const int r0 = (tile / jb.tiles_c) * kWgT, c0 = (tile % jb.tiles_c) * kWgT;
  const int wr = w >> 1, wc = w & 1;
  // this wave's rows / columns hold any output (the rest of its tile is padding)
  const bool live = r0 + 64 * wr < R && c0 + 64 * wc < C;
  // the layer's bias rides on its c0 = 0 tiles: threads t < kWgT sum column r0 + t of the staged dZ
  const bool bias_here = jb.bias_off >= 0 && c0 == 0;
  float bsum = 0.f;
  // staging: thread t loads column (t & 127) of rows (t >> 7) + 2 k, k < 8, of both operands
  const int lc = t & (kWgT - 1), lr = t >> 7;
  const bool rok = r0 + lc < R, cok = c0 + lc < C;
  // through global-address-space pointers: flat loads would also count in lgkmcnt, so every LDS
  // read's wait would drain the staging loads in flight
  using gptr = const __attribute__((address_space(1))) float*;
  const gptr zcol = (gptr)(dZ + (rok ? r0 + lc : 0));
  const gptr icol = (gptr)(In + (cok ? c0 + lc : 0));
  auto sA = [&](int st, int row, int col) -> float& { return wsm[((st * 2) * kWgKS + row) * kWgLd + col]; };
  auto sB = [&](int st, int row, int col) -> float& { return wsm[((st * 2 + 1) * kWgKS + row) * kWgLd + col]; };
  float za[2][kWgKS / 2], ia[2][kWgKS / 2];
  // raw loads (clamped rows); the masking waits for the stash, so no load is consumed early
  auto load = [&](int q, int64_t ms) {
#pragma unroll
    for (int k = 0; k < kWgKS / 2; ++k) {
      const int64_t m = ms + lr + 2 * k;
      const int64_t mm = m < m1 ? m : m0;
      za[q][k] = zcol[mm * R];
      ia[q][k] = icol[mm * ldi];
    }
  };
  auto stash = [&](int q, int st, int64_t ms) {
#pragma unroll
    for (int k = 0; k < kWgKS / 2; ++k) {
      const bool ok = ms + lr + 2 * k < m1;
      sA(st, lr + 2 * k, lc) = ok && rok ? za[q][k] : 0.f;
      sB(st, lr + 2 * k, lc) = ok && cok ? ia[q][k] : 0.f;
    }
  };
  f16v_ acc[2][2] = {};
  const int64_t nst = (m1 - m0 + kWgKS - 1) / kWgKS;  // stages of the slice
  // prologue: stage 0 into LDS, stage 1 into registers
  if (nst > 0) { load(0, m0); stash(0, 0, m0); }
  if (nst > 1) load(1, m0 + kWgKS);
  __syncthreads();
  // stage s: LDS slot s % kWgNS; register set Q = s & 1 (compile-time in each half of the loop
  // body: a runtime index would put the sets in scratch memory)
  auto body = [&](int64_t s, auto qc) {
    constexpr int Q = decltype(qc)::value;
    const int st = (int)(s % kWgNS);
    // stage s + 2 into set Q (unconditional: rows past the slice load clamped and stash as zeros;
    // a load under a branch makes the compiler's wait-count analysis drain every load early)
    load(Q, m0 + (s + 2) * kWgKS);
    if (live) {
#pragma unroll
      for (int ks = 0; ks < kWgKS / 2; ++ks) {
        const int row = 2 * ks + h;
        float a[2], bv[2];
#pragma unroll
        for (int x = 0; x < 2; ++x) a[x] = sA(st, row, 64 * wr + 32 * x + i);
#pragma unroll
        for (int y = 0; y < 2; ++y) bv[y] = sB(st, row, 64 * wc + 32 * y + i);
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
          for (int y = 0; y < 2; ++y)
            acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[x], bv[y], acc[x][y], 0, 0, 0);
      }
    }
    if (bias_here && t < kWgT) {  // the stage's dZ rows below bias_M, in row order
      const int64_t ms = m0 + s * kWgKS;
#pragma unroll
      for (int row = 0; row < kWgKS; ++row)
        if (ms + row < jb.bias_M) bsum += sA(st, row, t);
    }
    // stage s + 1 (registers) into its slot: the slot of stage s - 2, read two barriers ago
    stash(Q ^ 1, (int)((s + 1) % kWgNS), m0 + (s + 1) * kWgKS);
    __syncthreads();
  };
  for (int64_t s = 0; s < nst; s += 2) {
    body(s, std::integral_constant<int, 0>{});
    if (s + 1 < nst) body(s + 1, std::integral_constant<int, 1>{});
  }
  if (bias_here && t < kWgT && r0 + t < R) part[jb.bias_off + (size_t)slice * R + r0 + t] = bsum;
  if (!live) return;
  // accumulator (x, y) register q: row 64 wr + 32 x + (q & 3) + 8 (q >> 2) + 4 h, column
  // 64 wc + 32 y + i of the tile
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) {
      const int cc = c0 + 64 * wc + 32 * y + i;
      if (cc >= C) continue;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int rr = r0 + 64 * wr + 32 * x + (q & 3) + 8 * (q >> 2) + 4 * h;
        if (rr < R) out[(size_t)rr * C + cc] = acc[x][y][q];
      }
    }
}
constexpr size_t kWgLdsBytes = (size_t)kWgNS * 2 * kWgKS * kWgLd * sizeof(float);

// element e of the concatenated outputs (job j owns [out0, out0 + R C)): the sum over slices in
// slice order
template <int = 0>
__global__ void k_split_reduce_batch(const WgradJob* __restrict__ jobs, int n_jobs, int S,
                                     int64_t total, const float* __restrict__ part) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  int j = 0;
  while (j + 1 < n_jobs && e >= jobs[j + 1].out0) ++j;
  const WgradJob& jb = jobs[j];
  const int64_t n = (int64_t)jb.R * jb.C, i = e - jb.out0;
  const float* p = part + jb.part_off + i;
  float acc = 0.f;
  for (int k = 0; k < S; ++k) acc += p[(int64_t)k * n];
  const int r = (int)(i / jb.C), c = (int)(i % jb.C);
  jb.dW[(int64_t)r * jb.ldw + jb.c0 + c] = acc;
}

namespace {
constexpr int kMaxWgradJobs = 3 * kMaxLin;
static_assert(kMaxWgradJobs * sizeof(WgradJob) <= kWgradTableBytes, "job table");

// the slice count of a batch: about 3 blocks (12 waves, the kernel's occupancy) per CU over all
// the batch's tiles, at least kSliceRows rows per slice
int batch_slices(int64_t total_tiles, int64_t M) {
  int64_t S = std::max<int64_t>(1, (256 * 3 + total_tiles - 1) / total_tiles);
  S = std::min<int64_t>(S, kSplitMax);
  S = std::max<int64_t>(1, std::min<int64_t>(S, (M + kSliceRows - 1) / kSliceRows));
  return (int)S;
}

struct WgradBatch {
  std::vector<WgradJob> jobs;
  int max_jobs = kMaxWgradJobs;  // the device table's capacity
  // the slice count the workspace was sized with (the full job plan's); 0 = plan it.  A batch
  // with some gradients not requested has fewer tiles, so planning it anew would choose more
  // slices than the partial-product region holds.
  int slices = 0;
  void weight(const float* dZ, int R, const float* In, int C, int64_t M, float* dW, int ldw, int c0) {
    WgradJob j{};
    j.dZ = dZ; j.In = In; j.dW = dW; j.M = M; j.R = R; j.C = C; j.ldi = C; j.ldw = ldw; j.c0 = c0;
    jobs.push_back(j);
  }
  void bias(const float* dZ, int R, int64_t M, float* db) {
    WgradJob j{};
    j.dZ = dZ; j.In = nullptr; j.dW = db; j.M = M; j.R = R; j.C = 1; j.ldi = 1; j.ldw = 1; j.c0 = 0;
    j.bias = 1;
    jobs.push_back(j);
  }
  // which kernel: k_wgrad_batch (the default) or k_wgrad_tile (option "wgrad_tile" nonzero)
  bool tile = option(OPT_WGRAD_TILE) != 0;
  // lay out tiles, slices and partial offsets; returns the partial floats needed
  size_t plan(int& S) {
    int64_t tiles = 0, Mmax = 1;
    std::vector<int> link(jobs.size(), -1);  // bias job -> the weight job that sums it
    for (size_t b = 0; tile && b < jobs.size(); ++b) {
      if (!jobs[b].bias) continue;
      for (size_t w = 0; w < jobs.size(); ++w) {
        const WgradJob& q = jobs[w];
        if (!q.bias && q.dZ == jobs[b].dZ && q.R == jobs[b].R && q.M >= jobs[b].M) { link[b] = (int)w; break; }
      }
    }
    for (size_t k = 0; k < jobs.size(); ++k) {
      WgradJob& j = jobs[k];
      j.bias_off = -1;
      j.bias_M = 0;
      if (!tile) {
        j.tiles_c = (j.C + 63) / 64;
        j.n_tiles = ((j.R + 63) / 64) * j.tiles_c;
      } else if (j.bias) {
        // summed by its weight job's tiles, or one column-sum block per slice
        j.tiles_c = 1;
        j.n_tiles = link[k] >= 0 ? 0 : 1;
      } else {
        j.tiles_c = (j.C + kWgT - 1) / kWgT;
        j.n_tiles = ((j.R + kWgT - 1) / kWgT) * j.tiles_c;
      }
      tiles += j.n_tiles;
      Mmax = std::max(Mmax, j.M);
    }
    S = slices > 0 ? slices : batch_slices(std::max<int64_t>(tiles, 1), Mmax);
    int64_t block = 0, out = 0;
    size_t off = 0;
    for (auto& j : jobs) {
      j.slice_rows = ((j.M + S - 1) / S + 15) / 16 * 16;
      j.block0 = (int)block;
      block += (int64_t)j.n_tiles * S;
      j.part_off = (int64_t)off;
      off += (size_t)S * j.R * j.C;
      j.out0 = out;
      out += (int64_t)j.R * j.C;
    }
    for (size_t b = 0; b < jobs.size(); ++b)
      if (link[b] >= 0) {
        // the weight job's slices (its slice_rows) carry the sums; rows past the bias job's M
        // (the stacked tangent half of the double backward) are not summed
        jobs[link[b]].bias_off = jobs[b].part_off;
        jobs[link[b]].bias_M = jobs[b].M;
      }
    return off;
  }
  // table: kMaxWgradJobs * sizeof(WgradJob) bytes of device memory; part: the plan's floats
  // part_cap: the floats the workspace's partial-product region holds
  int run(void* table, float* part, size_t part_cap, hipStream_t st) {
    if (jobs.empty()) return NRT_OK;
    if ((int)jobs.size() > max_jobs) { set_error("weight gradients: too many jobs"); return NRT_EINVAL; }
    int S = 1;
    if (plan(S) > part_cap) { set_error("weight gradients: partial products exceed the workspace"); return NRT_EINVAL; }
    int64_t blocks = 0, total = 0;
    for (auto& j : jobs) { blocks += (int64_t)j.n_tiles * S; total += (int64_t)j.R * j.C; }
    NRT_HIP(hipMemcpyAsync(table, jobs.data(), jobs.size() * sizeof(WgradJob), hipMemcpyHostToDevice, st));
    const WgradJob* tj = (const WgradJob*)table;
    double flop = 0.0;
    for (auto& j : jobs) flop += 2.0 * j.R * j.C * (double)j.M;
    {
      ProfScope prof("k_wgrad", st, flop);
      if (!tile) {
        k_wgrad_batch<><<<dim3((unsigned)blocks), dim3(64 * kWgradWaves), 0, st>>>(tj, (int)jobs.size(), S, part);
        if (int rc = check_launch("k_wgrad_batch")) return rc;
      } else if (blocks > 0) {
        if (int rc = set_lds(k_wgrad_tile<>, kWgLdsBytes)) return rc;
        k_wgrad_tile<><<<dim3((unsigned)blocks), dim3(kWgThreads), kWgLdsBytes, st>>>(tj, (int)jobs.size(), S, part);
        if (int rc = check_launch("k_wgrad_tile")) return rc;
      }
    }
    k_split_reduce_batch<><<<dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st>>>(
        tj, (int)jobs.size(), S, total, part);
    return check_launch("k_split_reduce_batch");
  }
};

// the jobs of one nrt_mlp_backward (rows M) or nrt_mlp_grad_backward (weights over the stacked
// 2M rows, biases over the M primal rows): shared by the workspace size and the launch
template <class F>
void backward_jobs(const MlpDev& d, bool grad_bwd, F&& f) {
  const int L = d.n_hidden, H = d.hidden;
  for (int l = 0; l <= L + 1; ++l) {
    const bool outl = l == L + 1;
    const int R = outl ? d.out : H;
    if (l == 0) {
      f(l, R, 0, d.dp, d.dp, 0);
    } else {
      const int i = l - 1;
      const bool skip = !outl && i != L - 1 && (i % d.skip) == 0;
      const int C = H + (skip ? d.dp : 0);
      f(l, R, 1, H, C, 0);
      if (skip) f(l, R, 2, d.dp, C, H);
    }
    if (!(grad_bwd && outl)) f(l, R, 3, 1, 1, 0);  // bias
  }
}

// the partial floats and slice count of every job of one MLP's backward (the workspace's plan)
size_t batch_part_floats(const MlpDev& d, int64_t M, bool grad_bwd, int* slices = nullptr) {
  WgradBatch b;
  backward_jobs(d, grad_bwd, [&](int, int R, int kind, int C, int ldw, int c0) {
    if (kind == 3) b.bias(nullptr, R, M, nullptr);
    else b.weight(nullptr, R, nullptr, C, grad_bwd ? 2 * M : M, nullptr, ldw, c0);
  });
  int S = 1;
  const size_t floats = b.plan(S);
  if (slices) *slices = S;
  return floats;
}
// k_mlp_backward32's LDS plan: slab row [hidden | encoding] (H + ke floats), or [hidden] with the
// encoding in global tiles when that at least doubles the waves per CU (TILE)
LdsPlan backward_plan(const MlpDev& d, bool& tile) {
  auto plan = [&](bool t) {
    LdsPlan p;
    p.RS = (std::max(d.hidden, 32) + (t ? 0 : d.ke)) | 1;
    p.per_wave = wave_lds_floats(p.RS, 1, false);
    p.waves = std::max(1, std::min(4, kLdsBytes / (p.per_wave * 4)));
    p.bytes = (size_t)p.waves * p.per_wave * 4;
    spread_waves(p);
    return p;
  };
  const LdsPlan slab = plan(false), tiled = plan(true);
  const auto per_cu = [](const LdsPlan& p) { return std::min(8, kLdsBytes / (p.per_wave * 4)); };
  tile = per_cu(tiled) >= 2 * per_cu(slab);
  return tile ? tiled : slab;
}
// the column-split kernels' plan: one slab per block of ColSplit<nb>::CW waves (same TILE rule,
// counted in blocks per CU)
LdsPlan backward_plan_cs(const MlpDev& d, bool& tile) {
  auto plan = [&](bool t) {
    LdsPlan p;
    p.RS = (std::max(d.hidden, 32) + (t ? 0 : d.ke)) | 1;
    p.per_wave = 32 * p.RS;
    p.waves = 1;
    p.bytes = (size_t)p.per_wave * 4;
    return p;
  };
  const LdsPlan slab = plan(false), tiled = plan(true);
  const auto per_cu = [](const LdsPlan& p) { return std::min(8, kLdsBytes / (p.per_wave * 4)); };
  // the per-wave kernels' rule (TILE where it doubles the blocks per CU: the 16x256 F = 128
  // MLP, 4 blocks of 8 waves per CU instead of 2; measured 0.5 ms a training step faster);
  // option bwd_colsplit 2: the slab unless fewer than two blocks fit
  tile = (option(OPT_BWD_COLSPLIT) != 2 || per_cu(slab) < 2) && per_cu(tiled) >= 2 * per_cu(slab);
  return tile ? tiled : slab;
}
#define NRT_CW(NBv) (ColSplit<NBv>::CW)

// one MLP's activations / gradients region of the multi-MLP workspace (carve's first seven arrays)
size_t region_bytes(const MlpDev& d, int64_t M) {
  const size_t lay = (size_t)(d.n_hidden + 1) * (size_t)M * d.hidden * 4;
  const size_t enc = (size_t)M * d.dp * 4;
  return 3 * a256(lay) + 2 * a256(enc) + 2 * a256(enc_tile_bytes(d, M));
}

bool same_shape(const nrt_mlp* a, const nrt_mlp* b) {
  const MlpDev &x = a->host_dev, &y = b->host_dev;
  return x.hidden == y.hidden && x.n_hidden == y.n_hidden && x.ke == y.ke && x.dp == y.dp &&
         x.in_size == y.in_size && x.out == y.out && x.skip == y.skip && x.freqs == y.freqs &&
         x.latent == y.latent && x.nb == y.nb && a->desc.activation == b->desc.activation;
}

// the combined weight-gradient batch of n same-shape MLPs (pointers filled by the caller's f)
template <class F>
void multi_jobs(const MlpDev& d, int n, int64_t M, WgradBatch& b, F&& f) {
  b.max_jobs = n * kMaxWgradJobs;
  for (int i = 0; i < n; ++i)
    backward_jobs(d, false, [&](int l, int R, int kind, int C, int ldw, int c0) { f(i, l, R, kind, C, ldw, c0); });
  (void)M;
}

// the partial floats and slice count of every job of n same-shape MLPs' backward
size_t multi_part_floats(const MlpDev& d, int n, int64_t M, int* slices = nullptr) {
  WgradBatch b;
  multi_jobs(d, n, M, b, [&](int, int, int R, int kind, int C, int, int) {
    if (kind == 3) b.bias(nullptr, R, M, nullptr);
    else b.weight(nullptr, R, nullptr, C, M, nullptr, 0, 0);
  });
  int S = 1;
  const size_t floats = b.plan(S);
  if (slices) *slices = S;
  return floats;
}
}  // namespace


}  // namespace nrt

using namespace nrt;

extern "C" {

size_t nrt_mlp_backward_workspace_bytes(const nrt_mlp* m, int64_t M) {
  if (!m) return 0;
  M = std::max<int64_t>(M, 1);
  const MlpDev& d = m->host_dev;
  const size_t lay = (size_t)(d.n_hidden + 1) * (size_t)M * d.hidden * 4;
  const size_t enc = (size_t)M * d.dp * 4;
  return 3 * a256(lay) + 2 * a256(enc) + 2 * a256(enc_tile_bytes(d, M)) +
         a256(kWgradTableBytes) + a256(batch_part_floats(d, M, false) * 4);
}

int nrt_mlp_backward(const nrt_mlp* m, const float* x, const float* latent, int64_t M,
                     const float* dy, float* dx, float* dlatent, float* const* dweights,
                     float* const* dbiases, void* workspace, void* stream) {
  if (!m || M < 0 || (M > 0 && (!x || !dy || !workspace))) {
    set_error("nrt_mlp_backward: bad argument");
    return NRT_EINVAL;
  }
  const MlpDev& d = m->host_dev;
  if (d.latent > 0 && !latent) { set_error("nrt_mlp_backward: latent required"); return NRT_EINVAL; }
  if (M > INT32_MAX) { set_error("nrt_mlp_backward: at most 2^31-1 rows per call"); return NRT_EINVAL; }
  hipStream_t st = (hipStream_t)stream;
  const int L = d.n_hidden, H = d.hidden;
  if (M == 0) {  // zero gradients
    for (int l = 0; l < L + 2; ++l) {
      const int R = l == L + 1 ? d.out : H;
      const int C = m->host_w[l].size() / (size_t)R;
      if (dweights && dweights[l]) NRT_HIP(hipMemsetAsync(dweights[l], 0, (size_t)R * C * 4, st));
      if (dbiases && dbiases[l]) NRT_HIP(hipMemsetAsync(dbiases[l], 0, (size_t)R * 4, st));
    }
    return NRT_OK;
  }
  TrainWs w = carve(m, M, workspace);
  bool tile = false;
  const bool cs = option(OPT_BWD_COLSPLIT) != 0;
  const LdsPlan lp = cs ? backward_plan_cs(d, tile) : backward_plan(d, tile);
  const int waves = ceil_div64(M, 32);
  dim3 grid(ceil_div64(waves, lp.waves)), block(64 * lp.waves);
  int rc = NRT_OK;
  // the shading MLPs' shapes: the ring backward (nrt_train_ring.h), its job table in the
  // workspace's weight-gradient table region (the weight gradients copy theirs after it ran)
  if (!latent && ring_backward_ok(&m, 1) && ring_backward_table_bytes(1) <= kWgradTableBytes) {
    ProfScope prof("k_mlp_backward32", st, bwd_row_flop(d) * (double)M);
    if ((rc = ring_backward(&m, 1, x, M, &dy, &dx, &w.A, &w.dZ, &w.Eraw, &w.Eact, w.table, st)))
      return rc;
  } else {
    ProfScope prof("k_mlp_backward32", st, bwd_row_flop(d) * (double)M);
    NRT_NB_SWITCH(d.nb, {
      if (cs) {
        const dim3 gcs(waves), bcs(64 * NRT_CW(NB));
        if (tile) {
          if (!(rc = set_lds(k_mlp_backward32_cs<NB, true>, lp.bytes)))
            k_mlp_backward32_cs<NB, true><<<gcs, bcs, lp.bytes, st>>>(
                m->dev, x, latent, M, dy, dx, dlatent, w.Z, w.A, w.Eraw, w.Eact, w.dZ, w.Et, w.Gt, lp.RS);
        } else {
          if (!(rc = set_lds(k_mlp_backward32_cs<NB, false>, lp.bytes)))
            k_mlp_backward32_cs<NB, false><<<gcs, bcs, lp.bytes, st>>>(
                m->dev, x, latent, M, dy, dx, dlatent, w.Z, w.A, w.Eraw, w.Eact, w.dZ, w.Et, w.Gt, lp.RS);
        }
      } else if (tile) {
        if (!(rc = set_lds(k_mlp_backward32<NB, true>, lp.bytes)))
          k_mlp_backward32<NB, true><<<grid, block, lp.bytes, st>>>(
              m->dev, x, latent, M, dy, dx, dlatent, w.Z, w.A, w.Eraw, w.Eact, w.dZ, w.Et, w.Gt,
              lp.RS, lp.per_wave);
      } else {
        if (!(rc = set_lds(k_mlp_backward32<NB, false>, lp.bytes)))
          k_mlp_backward32<NB, false><<<grid, block, lp.bytes, st>>>(
              m->dev, x, latent, M, dy, dx, dlatent, w.Z, w.A, w.Eraw, w.Eact, w.dZ, w.Et, w.Gt,
              lp.RS, lp.per_wave);
      }
    });
    if (rc) return rc;
    if ((rc = check_launch("k_mlp_backward32"))) return rc;
  }
  if (!dweights && !dbiases) return NRT_OK;
  // every weight and bias gradient in one batched split-K launch (+ its slice reduction)
  const size_t lay = (size_t)M * H;
  WgradBatch batch;
  const size_t cap = batch_part_floats(d, M, false, &batch.slices);
  backward_jobs(d, false, [&](int l, int R, int kind, int C, int ldw, int c0) {
    const float* dZ = l == L + 1 ? dy : w.dZ + (size_t)l * lay;
    if (kind == 3) {
      if (dbiases && dbiases[l]) batch.bias(dZ, R, M, dbiases[l]);
      return;
    }
    if (!dweights || !dweights[l]) return;
    const float* In = kind == 0 ? w.Eraw : kind == 1 ? w.A + (size_t)(l - 1) * lay : w.Eact;
    batch.weight(dZ, R, In, C, M, dweights[l], ldw, c0);
  });
  return batch.run(w.table, w.part, cap, st);
}

size_t nrt_mlp_backward_multi_workspace_bytes(const nrt_mlp* const* mlps, int n, int64_t M) {
  if (!mlps || n <= 0 || !mlps[0]) return 0;
  M = std::max<int64_t>(M, 1);
  const MlpDev& d = mlps[0]->host_dev;
  const size_t part = multi_part_floats(d, n, M);
  return (size_t)n * region_bytes(d, M) + a256((size_t)n * sizeof(BwdJob)) +
         a256((size_t)n * kWgradTableBytes) + a256(part * 4);
}

int nrt_mlp_backward_multi(const nrt_mlp* const* mlps, int n, const float* x, int64_t M,
                           const float* const* dy, float* const* dx, float* const* dweights,
                           float* const* dbiases, void* workspace, void* stream) {
  if (!mlps || n <= 0 || M < 0 || !dy || (M > 0 && (!x || !workspace))) {
    set_error("nrt_mlp_backward_multi: bad argument");
    return NRT_EINVAL;
  }
  for (int i = 0; i < n; ++i) {
    if (!mlps[i] || !same_shape(mlps[0], mlps[i])) {
      set_error("nrt_mlp_backward_multi: the MLPs must share one shape");
      return NRT_EINVAL;
    }
  }
  const MlpDev& d = mlps[0]->host_dev;
  if (d.latent > 0) { set_error("nrt_mlp_backward_multi: latent MLPs are not supported"); return NRT_EINVAL; }
  if (M > INT32_MAX) { set_error("nrt_mlp_backward_multi: at most 2^31-1 rows per call"); return NRT_EINVAL; }
  const int L = d.n_hidden, H = d.hidden, NL = L + 2;
  if (M == 0) {
    for (int i = 0; i < n; ++i)
      if (int rc = nrt_mlp_backward(mlps[i], x, nullptr, 0, dy[i], nullptr, nullptr,
                                    dweights ? dweights + (size_t)i * NL : nullptr,
                                    dbiases ? dbiases + (size_t)i * NL : nullptr, workspace, stream))
        return rc;
    return NRT_OK;
  }
  hipStream_t st = (hipStream_t)stream;
  char* p = (char*)workspace;
  std::vector<TrainWs> ws(n);
  std::vector<BwdJob> jobs(n);
  for (int i = 0; i < n; ++i) {
    ws[i] = carve(mlps[i], M, p);  // its first seven arrays; table / part are not used
    p += region_bytes(d, M);
    jobs[i] = BwdJob{mlps[i]->dev, dy[i], dx ? dx[i] : nullptr, ws[i].Z, ws[i].A, ws[i].Eraw,
                     ws[i].Eact, ws[i].dZ, ws[i].Et, ws[i].Gt};
  }
  BwdJob* tj = (BwdJob*)p;
  p += a256((size_t)n * sizeof(BwdJob));
  void* table = p;
  p += a256((size_t)n * kWgradTableBytes);
  float* part = (float*)p;
  NRT_HIP(hipMemcpyAsync(tj, jobs.data(), (size_t)n * sizeof(BwdJob), hipMemcpyHostToDevice, st));
  bool tile = false;
  const bool cs = option(OPT_BWD_COLSPLIT) != 0;
  const LdsPlan lp = cs ? backward_plan_cs(d, tile) : backward_plan(d, tile);
  const int waves = ceil_div64(M, 32);
  dim3 grid(ceil_div64(waves, lp.waves), n), block(64 * lp.waves);
  int rc = NRT_OK;
  if (ring_backward_ok(mlps, n) && ring_backward_table_bytes(n) <= (size_t)n * kWgradTableBytes) {
    // the ring backward (nrt_train_ring.h), blockIdx.y = MLP; its job table in the weight-gradient
    // table region
    std::vector<float*> A(n), dZ(n), Er(n), Ea(n);
    for (int i = 0; i < n; ++i) { A[i] = ws[i].A; dZ[i] = ws[i].dZ; Er[i] = ws[i].Eraw; Ea[i] = ws[i].Eact; }
    ProfScope prof("k_mlp_backward32", st, bwd_row_flop(d) * (double)M * n);
    if ((rc = ring_backward(mlps, n, x, M, dy, dx, A.data(), dZ.data(), Er.data(), Ea.data(), table, st)))
      return rc;
  } else {
    ProfScope prof("k_mlp_backward32", st, bwd_row_flop(d) * (double)M * n);
    NRT_NB_SWITCH(d.nb, {
      if (cs) {
        const dim3 gcs(waves, n), bcs(64 * NRT_CW(NB));
        if (tile) {
          if (!(rc = set_lds(k_mlp_backward32_multi_cs<NB, true>, lp.bytes)))
            k_mlp_backward32_multi_cs<NB, true><<<gcs, bcs, lp.bytes, st>>>(tj, x, M, lp.RS);
        } else {
          if (!(rc = set_lds(k_mlp_backward32_multi_cs<NB, false>, lp.bytes)))
            k_mlp_backward32_multi_cs<NB, false><<<gcs, bcs, lp.bytes, st>>>(tj, x, M, lp.RS);
        }
      } else if (tile) {
        if (!(rc = set_lds(k_mlp_backward32_multi<NB, true>, lp.bytes)))
          k_mlp_backward32_multi<NB, true><<<grid, block, lp.bytes, st>>>(tj, x, M, lp.RS, lp.per_wave);
      } else {
        if (!(rc = set_lds(k_mlp_backward32_multi<NB, false>, lp.bytes)))
          k_mlp_backward32_multi<NB, false><<<grid, block, lp.bytes, st>>>(tj, x, M, lp.RS, lp.per_wave);
      }
    });
    if (rc) return rc;
    if ((rc = check_launch("k_mlp_backward32_multi"))) return rc;
  }
  if (!dweights && !dbiases) return NRT_OK;
  const size_t lay = (size_t)M * H;
  WgradBatch batch;
  const size_t cap = multi_part_floats(d, n, M, &batch.slices);
  multi_jobs(d, n, M, batch, [&](int i, int l, int R, int kind, int C, int ldw, int c0) {
    const TrainWs& w = ws[i];
    const float* dZ = l == L + 1 ? dy[i] : w.dZ + (size_t)l * lay;
    if (kind == 3) {
      if (dbiases && dbiases[(size_t)i * NL + l]) batch.bias(dZ, R, M, dbiases[(size_t)i * NL + l]);
      return;
    }
    if (!dweights || !dweights[(size_t)i * NL + l]) return;
    const float* In = kind == 0 ? w.Eraw : kind == 1 ? w.A + (size_t)(l - 1) * lay : w.Eact;
    batch.weight(dZ, R, In, C, M, dweights[(size_t)i * NL + l], ldw, c0);
  });
  return batch.run(table, part, cap, st);
}

int nrt_mlp_backward_saved(const nrt_mlp* const* mlps, int n, const float* x, int64_t M,
                           const int32_t* rows, const void* const* saved, int64_t Ms,
                           const float* const* dy, float* const* dx, float* const* dweights,
                           float* const* dbiases, void* workspace, void* stream) {
  if (!mlps || n <= 0 || M < 0 || !dy || !saved || Ms < 0 || (!rows && M != Ms) ||
      (M > 0 && (!x || !workspace))) {
    set_error("nrt_mlp_backward_saved: bad argument");
    return NRT_EINVAL;
  }
  for (int i = 0; i < n; ++i) {
    if (!mlps[i] || !saved[i] || !same_shape(mlps[0], mlps[i])) {
      set_error("nrt_mlp_backward_saved: the MLPs must share one shape, each with its saved activations");
      return NRT_EINVAL;
    }
  }
  const MlpDev& d = mlps[0]->host_dev;
  if (M > INT32_MAX || Ms > INT32_MAX) { set_error("nrt_mlp_backward_saved: at most 2^31-1 rows per call"); return NRT_EINVAL; }
  if (!ring_backward_ok(mlps, n)) {
    set_error("nrt_mlp_backward_saved: no ring backward for these MLPs (nrt_mlp_save_bytes is 0)");
    return NRT_EUNSUPPORTED;
  }
  const int L = d.n_hidden, H = d.hidden, NL = L + 2;
  if (M == 0)
    return nrt_mlp_backward_multi(mlps, n, x, 0, dy, dx, dweights, dbiases, workspace, stream);
  hipStream_t st = (hipStream_t)stream;
  char* p = (char*)workspace;  // nrt_mlp_backward_multi_workspace_bytes(mlps, n, M)
  std::vector<TrainWs> ws(n);
  std::vector<SavedActs> sa(n);
  std::vector<float*> A(n), dZ(n), Ac(n), Er(n), Ea(n);
  std::vector<const float*> Sr(n), Sa(n);
  for (int i = 0; i < n; ++i) {
    ws[i] = carve(mlps[i], M, p);
    p += region_bytes(d, M);
    sa[i] = saved_split(d, Ms, saved[i]);
    A[i] = sa[i].A;
    dZ[i] = ws[i].dZ;
    // compacted rows: the backward copies the saved rows it reads into the workspace (the
    // weight gradients' operands, row-aligned with dZ)
    Ac[i] = ws[i].A; Er[i] = ws[i].Eraw; Ea[i] = ws[i].Eact;
    Sr[i] = sa[i].Eraw; Sa[i] = sa[i].Eact;
    if (!rows) { Ac[i] = nullptr; Er[i] = nullptr; Ea[i] = nullptr; }
  }
  p += a256((size_t)n * sizeof(BwdJob));
  void* table = p;
  p += a256((size_t)n * kWgradTableBytes);
  float* part = (float*)p;
  int rc = NRT_OK;
  {
    ProfScope prof("k_mlp_backward32", st, bwd_row_flop(d) * (double)M * n * 0.5);
    if ((rc = ring_backward(mlps, n, x, M, dy, dx, A.data(), dZ.data(), Er.data(), Ea.data(), table, st,
                            rows, Ms, Ac.data(), Sr.data(), Sa.data())))
      return rc;
  }
  if (!dweights && !dbiases) return NRT_OK;
  const size_t lay = (size_t)M * H;
  WgradBatch batch;
  const size_t cap = multi_part_floats(d, n, M, &batch.slices);
  multi_jobs(d, n, M, batch, [&](int i, int l, int R, int kind, int C, int ldw, int c0) {
    const float* dZl = l == L + 1 ? dy[i] : ws[i].dZ + (size_t)l * lay;
    if (kind == 3) {
      if (dbiases && dbiases[(size_t)i * NL + l]) batch.bias(dZl, R, M, dbiases[(size_t)i * NL + l]);
      return;
    }
    if (!dweights || !dweights[(size_t)i * NL + l]) return;
    // without compaction the saved activations themselves (Ms == M), else their compacted copy
    const float* Ar = rows ? ws[i].A : sa[i].A;
    const float* In = kind == 0 ? (rows ? ws[i].Eraw : sa[i].Eraw)
                    : kind == 1 ? Ar + (size_t)(l - 1) * lay
                                : (rows ? ws[i].Eact : sa[i].Eact);
    batch.weight(dZl, R, In, C, M, dweights[(size_t)i * NL + l], ldw, c0);
  });
  return batch.run(table, part, cap, st);
}

static size_t gb_sizes(const MlpDev& d, int64_t M, size_t sz[9]) {
  const size_t lay = (size_t)(d.n_hidden + 1) * (size_t)M * d.hidden * 4;
  sz[0] = lay;          // Z
  sz[1] = lay;          // Z tangent
  sz[2] = 2 * lay;      // A stacked
  sz[3] = 2 * lay;      // dZ stacked
  sz[4] = (size_t)2 * M * d.dp * 4;   // E0
  sz[5] = sz[4];                      // E1
  sz[6] = (size_t)2 * M * d.out * 4;  // output seed
  sz[7] = kWgradTableBytes;                          // weight-gradient job table
  sz[8] = batch_part_floats(d, M, true) * 4;        // batched split-K partial products
  size_t tot = 0;
  for (int i = 0; i < 9; ++i) tot += a256(sz[i]);
  return tot;
}

size_t nrt_mlp_grad_backward_workspace_bytes(const nrt_mlp* m, int64_t M) {
  if (!m) return 0;
  size_t sz[9];
  return gb_sizes(m->host_dev, std::max<int64_t>(M, 1), sz);
}

int nrt_mlp_grad_backward(const nrt_mlp* m, const float* x, const float* latent, int64_t M,
                          const float* v, float* const* dweights, float* const* dbiases,
                          void* workspace, void* stream) {
  if (!m || M < 0 || (M > 0 && (!x || !v || !workspace))) {
    set_error("nrt_mlp_grad_backward: bad argument");
    return NRT_EINVAL;
  }
  const MlpDev& d = m->host_dev;
  if (d.latent > 0 && !latent) { set_error("nrt_mlp_grad_backward: latent required"); return NRT_EINVAL; }
  if (M > INT32_MAX / 2) { set_error("nrt_mlp_grad_backward: at most 2^30-1 rows per call"); return NRT_EINVAL; }
  hipStream_t st = (hipStream_t)stream;
  const int L = d.n_hidden, H = d.hidden;
  auto zero_all = [&]() -> int {
    for (int l = 0; l < L + 2; ++l) {
      const int R = l == L + 1 ? d.out : H;
      const int C = m->host_w[l].size() / (size_t)R;
      if (dweights && dweights[l]) NRT_HIP(hipMemsetAsync(dweights[l], 0, (size_t)R * C * 4, st));
      if (dbiases && dbiases[l]) NRT_HIP(hipMemsetAsync(dbiases[l], 0, (size_t)R * 4, st));
    }
    return NRT_OK;
  };
  if (M == 0) return zero_all();
  if (!dweights && !dbiases) return NRT_OK;
  size_t sz[9];
  gb_sizes(d, M, sz);
  float* buf[9];
  char* p = (char*)workspace;
  for (int i = 0; i < 9; ++i) { buf[i] = (float*)p; p += a256(sz[i]); }
  // slab row: primal activations | encoding | encoding tangent | tangent activations
  const int RS = (2 * std::max(H, 32) + 2 * std::max(d.ke, 16)) | 1;
  const int per_wave = 32 * RS;
  const int waves = std::max(1, std::min(4, kLdsBytes / (per_wave * 4)));
  const size_t bytes = (size_t)waves * per_wave * 4;
  if (bytes > (size_t)kLdsBytes) { set_error("nrt_mlp_grad_backward: MLP too wide for LDS"); return NRT_EINVAL; }
  const int nwaves = ceil_div64(M, 32);
  dim3 grid(ceil_div64(nwaves, waves)), block(64 * waves);
  const bool cs = option(OPT_BWD_COLSPLIT) != 0;
  int rc = NRT_OK;
  {
    ProfScope prof("k_mlp_grad_backward32", st, grad_bwd_row_flop(d) * (double)M);
    NRT_NB_SWITCH(d.nb, {
      if (cs) {
        const size_t bcs = (size_t)per_wave * 4;
        if (!(rc = set_lds(k_mlp_grad_backward32_cs<NB>, bcs)))
          k_mlp_grad_backward32_cs<NB><<<dim3(nwaves), dim3(64 * NB), bcs, st>>>(
              m->dev, x, latent, v, M, buf[0], buf[1], buf[2], buf[4], buf[5], buf[3], RS);
      } else if (!(rc = set_lds(k_mlp_grad_backward32<NB>, bytes)))
        k_mlp_grad_backward32<NB><<<grid, block, bytes, st>>>(m->dev, x, latent, v, M, buf[0], buf[1],
                                                             buf[2], buf[4], buf[5], buf[3], RS,
                                                             per_wave);
    });
    if (rc) return rc;
    if ((rc = check_launch("k_mlp_grad_backward32"))) return rc;
  }
  const int64_t M2 = 2 * M;
  float* seed = buf[6];
  float* part = buf[7];
  NRT_HIP(hipMemsetAsync(seed, 0, (size_t)M * d.out * 4, st));
  k_fill<><<<dim3(std::min<int64_t>(ceil_div64(M * d.out, 256), 1024)), dim3(256), 0, st>>>(
      seed + (size_t)M * d.out, M * d.out, 1.f);
  if ((rc = check_launch("k_fill"))) return rc;
  const size_t lay2 = (size_t)M2 * H;
  // the out layer's bias takes no gradient from J (its tangent rows carry no bias)
  if (dbiases && dbiases[L + 1]) NRT_HIP(hipMemsetAsync(dbiases[L + 1], 0, (size_t)d.out * 4, st));
  WgradBatch batch;
  const size_t cap = batch_part_floats(d, M, true, &batch.slices);
  backward_jobs(d, true, [&](int l, int R, int kind, int C, int ldw, int c0) {
    const float* dZ = l == L + 1 ? seed : buf[3] + (size_t)l * lay2;
    if (kind == 3) {  // bias: the primal rows only
      if (dbiases && dbiases[l]) batch.bias(dZ, R, M, dbiases[l]);
      return;
    }
    if (!dweights || !dweights[l]) return;
    const float* In = kind == 0 ? buf[4] : kind == 1 ? buf[2] + (size_t)(l - 1) * lay2 : buf[5];
    batch.weight(dZ, R, In, C, M2, dweights[l], ldw, c0);
  });
  return batch.run(part, buf[8], cap, st);
}

}  // extern "C"
