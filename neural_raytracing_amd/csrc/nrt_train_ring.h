// nrt_train_ring.h -- the SkipConnMLP backward (training) of the shading MLPs
// on the FP32 row-program ring engine (nrt_shade_ring.h): LightField 10 x 256 F = 16, the
// spatial-weights MLP 16 x 256 F = 128, NeuralBSDF 6 x 96 F = 64 (leaky_relu, 3 inputs, no
// latent).  Reference: torch autograd of SkipConnMLP.forward (neural_blocks.py:75-86) given dL/dy.
//
// A wave owns 16 rows (lane g = lane >> 4, j = lane & 15 serves row j) on v_mfma_f32_16x16x4_f32
// (exact f32), and a block's waves share one LDS ring of weight chunks moved by LDS-DMA, as the
// forward row programs do.  The program of one MLP (build_rprog mode 1) is its forward stream
// without the out layer, then the transposed ("T") layers in reverse order:
//   T-out      dA_L = W_out^T dY: H output rows, k = the outputs padded to 16 (one quad per
//              sub-block, all sub-blocks in one chunk, [sb][lane][t]);
//   T-hidden l dA_{l-1} = W_l[:, :H]^T dZ_l: chunks of 32 output rows (the layer's input
//              features), k = H in the ring32 k order ([u][b][lane][t], as a forward hidden chunk);
//   T-enc l    (skip layers and the init layer) W_l[:, enc]^T dZ_l: the encoding slots as output
//              rows, 32 a chunk, k = H.
// The accumulator of a 16x16 sub-block is the next T-layer's B operand (row 4 g + r of row j in
// register r of lane 16 g + j = k-step 4 sb + r), so dZ never leaves registers: dZ_{l-1} =
// dA_{l-1} * leaky'(A_{l-1}), with leaky'(z) read off the saved activation's sign (a > 0 iff
// z > 0, torch's leaky_relu_backward).  The forward pass of the tile (the same ring evaluation as
// nrt_mlp_forward) runs first and stores every hidden layer's activations A_l [L+1][M][H] and the
// encoding (raw and activated, reference column order [M][dp]) for the weight gradients; the
// backward stores dZ_l [L+1][M][H].  The encoding rows of the T-enc layers fold straight into
// dL/dx (three running sums per lane): d sin(p_q)/dx_i = cos(p_q) B_iq, d cos(p_q)/dx_i =
// -sin(p_q) B_iq, d x_i / dx_i = 1, times leaky'(enc) on skip layers (their input is act(enc)).
//
// Saved activations (round 5): the training forward k_mlp_ring<..., SAVE> (below; nrt_mlp_forward_
// multi with save buffers) runs fwd32_save + out32 on the solo program and stores A_l and the
// encoding, and k_mlp_bwd_ring<..., SAVED> starts the backward program after its forward chunks
// (BwdRingJob::fwd_chunks) and reads A through the caller's live-row index, copying the rows it
// reads compactly for the weight gradients.  Same bits as the recomputing variant.
#pragma once
#include "nrt_shade_ring.h"

namespace nrt {
namespace rprog {

// leaky_relu'(z) from a = leaky_relu(z) (negative slope 0.01): a > 0 iff z > 0
__device__ __forceinline__ float dleaky(float a) { return a > 0.f ? 1.f : 0.01f; }

// The forward pass of one tile with its activations saved: eval32 (nrt_shade_ring.h) without the
// out layer (dst: the last hidden layer's activations, out32's input); save_a(layer, sb, f4v)
// receives every hidden layer's activations per sub-block, save_e(slot, raw, act) every encoding
// slot this lane computes (once per tile).  Same arithmetic as eval32.
template <class S, class En, class SaveA, class SaveE>
__device__ __forceinline__ void fwd32_save(En& E, const RProgMlp& m, float x0, float x1, float x2,
                                           float (&dst)[S::H / 4], SaveA&& save_a, SaveE&& save_e) {
  constexpr int NSB = S::NSB, NC = S::NC, QH = S::QH, KH = S::H / 4;
  const float4* basis = E.lbasis + m.basis_off;
  const int L = m.L, SK = m.skip;
  const int g = E.lane >> 4;
  float src[KH];
  f4v acc[NSB];
  // k-outer encoding part (enc_part32 with the encoding stored on the first pass)
  auto enc_part = [&](bool actv, bool store) {
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
            const int slot = 4 * (4 * u + t) + g;
            const float e = enc_slot(basis, m.F, slot, x0, x1, x2);
            const float a = ring32::act<ACT_LEAKY>(e);
            if (store) save_e(slot, e, a);
            v[t] = actv ? a : e;
          }
#pragma unroll
          for (int sb = 0; sb < NSB; sb += 2) {
            const float4 w0 = A[(uu * NSB + sb) * 64], w1 = A[(uu * NSB + sb + 1) * 64];
            acc[sb] = ring32::mfma4(w0.x, v[0], acc[sb]); acc[sb + 1] = ring32::mfma4(w1.x, v[0], acc[sb + 1]);
            acc[sb] = ring32::mfma4(w0.y, v[1], acc[sb]); acc[sb + 1] = ring32::mfma4(w1.y, v[1], acc[sb + 1]);
            acc[sb] = ring32::mfma4(w0.z, v[2], acc[sb]); acc[sb + 1] = ring32::mfma4(w1.z, v[2], acc[sb + 1]);
            acc[sb] = ring32::mfma4(w0.w, v[3], acc[sb]); acc[sb + 1] = ring32::mfma4(w1.w, v[3], acc[sb + 1]);
          }
        }
      }
      E.end();
    }
  };
  auto act_all = [&](int layer) {
#pragma unroll
    for (int sb = 0; sb < NSB; ++sb) {
      f4v a;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        a[r] = ring32::act<ACT_LEAKY>(acc[sb][r]);
        dst[4 * sb + r] = a[r];
      }
      save_a(layer, sb, a);
    }
  };
  // init layer (neural_blocks.py:80): the raw encoding, k-outer
#pragma unroll
  for (int sb = 0; sb < NSB; ++sb) acc[sb] = E.bias_at(m, 0, sb);
  enc_part(false, true);
  act_all(0);
  f4v pend0, pend1;
  auto retire1 = [&](int ib, int k) {
    float& d = dst[8 * ib + k];
    d = ring32::act<ACT_LEAKY>(k < 4 ? pend0[k & 3] : pend1[k & 3]);
    asm volatile("" : "+v"(d));
  };
  auto save_chunk = [&](int layer, int ib) {
#pragma unroll
    for (int b = 0; b < 2; ++b)
      save_a(layer, 2 * ib + b, f4v{dst[8 * ib + 4 * b], dst[8 * ib + 4 * b + 1],
                                    dst[8 * ib + 4 * b + 2], dst[8 * ib + 4 * b + 3]});
  };
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
      if (!RAW && ib > 0) save_chunk(1 + i, ib - 1);
      if (RAW) { acc[2 * ib] = a0; acc[2 * ib + 1] = a1; }
      else { pend0 = a0; pend1 = a1; }
      E.end();
    }
    if (!RAW) {
#pragma unroll
      for (int k = 0; k < 8; ++k) retire1(NC - 1, k);
      save_chunk(1 + i, NC - 1);
    }
  };
  for (int i = 0; i < L; ++i) {
#pragma unroll
    for (int k = 0; k < KH; ++k) src[k] = dst[k];
    if (i != L - 1 && i % SK == 0) {
      hidden(i, std::true_type{});
      enc_part(true, false);
      act_all(1 + i);
    } else {
      hidden(i, std::false_type{});
    }
  }
}

// The backward chain of one tile after fwd32_save (the ring is at the T-out chunk).  dy(s) = dL/dy
// of output 4 g + s of this lane's row (0 past the outputs); load_a(layer, sb) -> the saved
// activations (f4v, this lane's registers of sub-block sb); save_dz(layer, sb, f4v).  Returns the
// lane's partial dL/dx (summed over its encoding slots; the caller reduces over lane groups).
template <class S, class En, class LoadA, class SaveDz>
__device__ __forceinline__ void bwd32(En& E, const RProgMlp& m, float x0, float x1, float x2,
                                      const float (&dy)[4], LoadA&& load_a, SaveDz&& save_dz,
                                      float (&dx)[3]) {
  constexpr int NSB = S::NSB, NC = S::NC, QH = S::QH, KH = S::H / 4;
  const float4* basis = E.lbasis + m.basis_off;
  const int L = m.L, SK = m.skip, F = m.F;
  const int g = E.lane >> 4;
  // encoding rows of the T-enc layers: ke padded to 32 (two sub-blocks a chunk)
  constexpr int CEN = (S::KE * 4 + 31) / 32;
  float src[KH], dst[KH];
  dx[0] = dx[1] = dx[2] = 0.f;
  // ---- T-out: dA_L = W_out^T dY, dZ_L = dA_L * leaky'(A_L)
  {
    const float4* A = E.begin();
    f4v acc[NSB];
#pragma unroll
    for (int sb = 0; sb < NSB; ++sb) {
      const float4 w = A[sb * 64];
      f4v a = f4v{0.f, 0.f, 0.f, 0.f};
      a = ring32::mfma4(w.x, dy[0], a);
      a = ring32::mfma4(w.y, dy[1], a);
      a = ring32::mfma4(w.z, dy[2], a);
      a = ring32::mfma4(w.w, dy[3], a);
      acc[sb] = a;
    }
    E.end();
#pragma unroll
    for (int sb = 0; sb < NSB; ++sb) {
      const f4v av = load_a(L, sb);
      f4v z;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        z[r] = acc[sb][r] * dleaky(av[r]);
        src[4 * sb + r] = z[r];
      }
      save_dz(L, sb, z);
    }
  }
  // ---- T-enc of layer l: the encoding gradient W_l[:, enc]^T dZ_l (src), folded into dx
  f4v pe0, pe1;
  auto fold = [&](int c, bool skip_act) {
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const f4v& pv = b == 0 ? pe0 : pe1;
#pragma unroll
      for (int h = 0; h < 2; ++h) {  // slots s, s + 1 = (sin, cos) of projection q
        const int s = 32 * c + 16 * b + 4 * g + 2 * h;
        float gs = pv[2 * h], gc = pv[2 * h + 1];
        if (s < 2 * F) {
          const int q = s >> 1;
          const float4 bq = basis[q];
          float pr = x0 * bq.x;
          pr = fmaf(x1, bq.y, pr);
          pr = fmaf(x2, bq.z, pr);
          float sn, cs;
          sincosf(pr, &sn, &cs);
          if (skip_act) { gs *= dleaky(sn); gc *= dleaky(cs); }
          const float t = gs * cs - gc * sn;  // d/dp_q of gs sin + gc cos
          dx[0] = fmaf(t, bq.x, dx[0]);
          dx[1] = fmaf(t, bq.y, dx[1]);
          dx[2] = fmaf(t, bq.z, dx[2]);
        } else {
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const int xi = s + e - 2 * F;  // slots 2F .. 2F + 2: x0 .. x2, zeros past them
            float gv = e == 0 ? gs : gc;
            const float xv = xi == 0 ? x0 : xi == 1 ? x1 : x2;
            if (skip_act) gv *= dleaky(xv);
            if (xi == 0) dx[0] += gv;
            else if (xi == 1) dx[1] += gv;
            else if (xi == 2) dx[2] += gv;
          }
        }
      }
    }
  };
  auto t_enc = [&](bool skip_act) {
#pragma unroll 1
    for (int c = 0; c < CEN; ++c) {
      const float4* A = E.begin();
      f4v a0 = f4v{0.f, 0.f, 0.f, 0.f}, a1 = a0;
      ring32::seg2<QH, 0, 0>(A, src, a0, a1);
      E.end();
      pe0 = a0; pe1 = a1;
      fold(c, skip_act);
    }
  };
  // ---- T-hidden of layer l: dA_{l-1} = W_l[:, :H]^T dZ_l, dZ_{l-1} = dA_{l-1} leaky'(A_{l-1})
  f4v pend0, pend1;
  f4v acur0, acur1, anext0, anext1;  // saved activations of the chunk being retired / computed
  auto retire1 = [&](int ib, int k) {
    float& d = dst[8 * ib + k];
    const float a = k < 4 ? acur0[k & 3] : acur1[k & 3];
    d = (k < 4 ? pend0[k & 3] : pend1[k & 3]) * dleaky(a);
    asm volatile("" : "+v"(d));
  };
  for (int l = L; l >= 1; --l) {
    const int i = l - 1;
    if (i != L - 1 && i % SK == 0) t_enc(true);
#pragma unroll
    for (int ib = 0; ib < NC; ++ib) {
      anext0 = load_a(l - 1, 2 * ib);
      anext1 = load_a(l - 1, 2 * ib + 1);
      const float4* A = E.begin();
      f4v a0 = f4v{0.f, 0.f, 0.f, 0.f}, a1 = a0;
      ring32::seg2<QH, 0, 0>(A, src, a0, a1, [&](int u) {
        if (ib > 0)
#pragma unroll
          for (int k = (u * 8) / QH; k < ((u + 1) * 8) / QH; ++k) retire1(ib - 1, k);
      });
      if (ib > 0) {
        save_dz(l - 1, 2 * ib - 2, f4v{dst[8 * ib - 8], dst[8 * ib - 7], dst[8 * ib - 6], dst[8 * ib - 5]});
        save_dz(l - 1, 2 * ib - 1, f4v{dst[8 * ib - 4], dst[8 * ib - 3], dst[8 * ib - 2], dst[8 * ib - 1]});
      }
      pend0 = a0; pend1 = a1;
      acur0 = anext0; acur1 = anext1;
      E.end();
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) retire1(NC - 1, k);
    save_dz(l - 1, 2 * NC - 2, f4v{dst[8 * NC - 8], dst[8 * NC - 7], dst[8 * NC - 6], dst[8 * NC - 5]});
    save_dz(l - 1, 2 * NC - 1, f4v{dst[8 * NC - 4], dst[8 * NC - 3], dst[8 * NC - 2], dst[8 * NC - 1]});
#pragma unroll
    for (int k = 0; k < KH; ++k) src[k] = dst[k];
  }
  // ---- T-enc of the init layer (raw encoding in)
  t_enc(false);
}

// one MLP of a backward launch: its [forward | backward] row program and the tensors it touches
struct BwdRingJob {
  RProgDev prog;
  const float* dY;   // [M][out]
  float* dX;         // [M][3] or null
  float* A;          // [L+1][M][H] activations of the hidden layers (SAVED: [L+1][Ms][H], read)
  float* dZ;         // [L+1][M][H] their gradients
  float* Eraw;       // [M][dp] the encoding, reference columns [x, sin, cos]
  float* Eact;       // [M][dp] leaky_relu of it (the skip layers' input)
  // SAVED (the training forward stored A and the encoding, nrt_mlp_forward_multi with save
  // buffers): row i of this backward is saved row rows[i] (nullptr: i) of Ms; the program starts
  // after its forward part.  With rows, the saved rows read are copied compactly: A -> Acopy,
  // Sraw / Sact (the saved encoding) -> Eraw / Eact (nothing written without rows).
  const int32_t* rows;
  int64_t Ms;
  int fwd_chunks;
  float* Acopy;
  const float* Sraw;
  const float* Sact;
};

// slot (the ring's encoding order: sin / cos pairs, then x) -> reference column (utils.py:37-40)
__device__ __forceinline__ int slot_column(int s, int F) {
  if (s < 2 * F) return (s & 1) ? 3 + F + (s >> 1) : 3 + (s >> 1);
  if (s < 2 * F + 3) return s - 2 * F;
  return -1;
}

// nrt_mlp_forward(_multi) at FP32: block (x, y) evaluates row tiles of MLP y on its solo program
// (same-shape MLPs on one input -- the NeuralBSDF components of a spatial mixture, bsdfs.py:
// 634-637 -- in one launch: n times the blocks, so a 38,400-row batch fills the CUs).  SAVE: the
// training forward, which also stores what the ring backward reads (SoloJob A / Eraw / Eact), so
// the backward does not evaluate the forward again.
template <int D, int WV, class S, bool SAVE>
__global__ void __launch_bounds__(64 * WV, 1) k_mlp_ring(const SoloJobs jobs, const float* __restrict__ x,
                                                        int64_t M) {
  extern __shared__ __attribute__((aligned(16))) char smem_c[];
  const int64_t per_block = 16 * WV;
  if ((int64_t)blockIdx.x * per_block >= M) return;
  const SoloJob& jb = jobs.j[blockIdx.y];
  RProgDev pd;
  pd.stream = jb.stream;
  pd.stream_bytes = jb.stream_bytes;
  pd.chunks = jb.chunks;
  pd.n_chunks = jb.n_chunks;
  pd.tables = jb.tables;
  pd.table_floats = jb.table_floats;
  pd.basis = jb.basis;
  pd.basis_q = jb.basis_q;
  pd.n_mlp = 1;
  Engine<D, WV> E;
  E.init(pd, smem_c);
  const RProgMlp m = jb.mlp;
  const int out = jb.out, F = m.F, dp = 3 + 2 * F;
  float* __restrict__ y = jb.y;
  const int lane = E.lane, j = lane & 15, g = lane >> 4;
  constexpr int H = S::H;
  for (int64_t b0 = (int64_t)blockIdx.x * per_block; b0 < M; b0 += (int64_t)gridDim.x * per_block) {
    const int64_t i = b0 + 16 * E.wv + j;
    const bool valid = i < M;
    const int64_t ii = valid ? i : M - 1;
    const float x0 = x[ii * 3], x1 = x[ii * 3 + 1], x2 = x[ii * 3 + 2];
    f4v o;
    if constexpr (SAVE) {
      float last[H / 4];
      const size_t lay = (size_t)M * H;
      fwd32_save<S>(E, m, x0, x1, x2, last,
                    [&](int layer, int sb, const f4v& a) {
                      if (valid)
                        *reinterpret_cast<float4*>(jb.A + (size_t)layer * lay + (size_t)ii * H + 16 * sb + 4 * g) =
                            make_float4(a[0], a[1], a[2], a[3]);
                    },
                    [&](int slot, float raw, float act) {
                      const int c = slot_column(slot, F);
                      if (valid && c >= 0) {
                        jb.Eraw[ii * dp + c] = raw;
                        jb.Eact[ii * dp + c] = act;
                      }
                    });
      o = out32<S>(E, m, last);
    } else {
      o = eval<0, S, ACT_LEAKY>(E, m, 0, x0, x1, x2);
    }
    if (valid)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (4 * g + r < out) y[i * out + 4 * g + r] = o[r];
  }
  E.drain();
}

// blockIdx.y = MLP (the mixture's NeuralBSDFs share x); a persistent grid over 16-row tiles.
// SAVED: the activations come from the training forward (BwdRingJob rows / Ms) and the tile runs
// the backward chain only.
template <int D, int WV, class S, bool SAVED>
__global__ void __launch_bounds__(64 * WV, 1) k_mlp_bwd_ring(const BwdRingJob* __restrict__ jobs,
                                                            const float* __restrict__ x, int64_t M) {
  extern __shared__ __attribute__((aligned(16))) char smem_c[];
  const BwdRingJob& jb = jobs[blockIdx.y];
  const int64_t per_block = 16 * WV;
  if ((int64_t)blockIdx.x * per_block >= M) return;
  Engine<D, WV> E;
  E.init(jb.prog, smem_c, SAVED ? jb.fwd_chunks : 0);
  const RProgMlp& m = jb.prog.mlp[0];
  const int lane = E.lane, j = lane & 15, g = lane >> 4;
  const int out = m.out, F = m.F, dp = 3 + 2 * F;
  constexpr int H = S::H;
  float* const Ag = jb.A;
  float* const dZg = jb.dZ;
  const size_t lay = (size_t)M * H;
  const size_t alay = SAVED ? (size_t)jb.Ms * H : lay;  // A's layer stride
  for (int64_t b0 = (int64_t)blockIdx.x * per_block; b0 < M; b0 += (int64_t)gridDim.x * per_block) {
    const int64_t i = b0 + 16 * E.wv + j;
    const bool valid = i < M;
    const int64_t ii = valid ? i : M - 1;
    const float x0 = x[ii * 3], x1 = x[ii * 3 + 1], x2 = x[ii * 3 + 2];
    const int64_t ia = SAVED && jb.rows ? (int64_t)jb.rows[ii] : ii;  // A's row
    const bool copy = SAVED && jb.rows != nullptr && valid;
    if (copy) {  // the saved encoding row -> its compact row (4 lanes a row)
      for (int c = g; c < dp; c += 4) {
        jb.Eraw[ii * dp + c] = jb.Sraw[ia * dp + c];
        jb.Eact[ii * dp + c] = jb.Sact[ia * dp + c];
      }
    }
    auto at = [&](float* base, int layer, int sb) -> float* {
      return base + (size_t)layer * lay + (size_t)ii * H + 16 * sb + 4 * g;
    };
    auto at_a = [&](int layer, int sb) -> float* {
      return Ag + (size_t)layer * alay + (size_t)ia * H + 16 * sb + 4 * g;
    };
    if constexpr (!SAVED) {
      float last[H / 4];
      fwd32_save<S>(E, m, x0, x1, x2, last,
                    [&](int layer, int sb, const f4v& a) {
                      if (valid) *reinterpret_cast<float4*>(at_a(layer, sb)) = make_float4(a[0], a[1], a[2], a[3]);
                    },
                    [&](int slot, float raw, float act) {
                      const int c = slot_column(slot, F);
                      if (valid && c >= 0) {
                        jb.Eraw[ii * dp + c] = raw;
                        jb.Eact[ii * dp + c] = act;
                      }
                    });
    }
    float dy[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) dy[s] = 4 * g + s < out ? jb.dY[ii * out + 4 * g + s] : 0.f;
    float dx[3];
    bwd32<S>(E, m, x0, x1, x2, dy,
             [&](int layer, int sb) -> f4v {
               const float4 v = *reinterpret_cast<const float4*>(at_a(layer, sb));
               // every (layer, sub-block) of the tile is read exactly once: its compact copy
               if (copy) *reinterpret_cast<float4*>(at(jb.Acopy, layer, sb)) = v;
               return f4v{v.x, v.y, v.z, v.w};
             },
             [&](int layer, int sb, const f4v& z) {
               if (valid) *reinterpret_cast<float4*>(at(dZg, layer, sb)) = make_float4(z[0], z[1], z[2], z[3]);
             },
             dx);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      dx[k] += __shfl_xor(dx[k], 16);
      dx[k] += __shfl_xor(dx[k], 32);
    }
    if (jb.dX && valid && g == 0) {
      jb.dX[ii * 3] = dx[0];
      jb.dX[ii * 3 + 1] = dx[1];
      jb.dX[ii * 3 + 2] = dx[2];
    }
  }
  E.drain();
}

}  // namespace rprog
}  // namespace nrt
