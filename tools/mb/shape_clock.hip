// Microbenchmark: does the FP16 ring march's inner loop run faster with 16x16x32 MFMAs than with
// 32x32x16 at the same FLOPs, LDS bytes and VALU per FLOP?  (MI355X_MICROARCH.md 'DVFS give-back'
// item 7: the chip can hold a higher clock on one shape.)  Models one hidden-layer chunk of
// k_march16 on random data, 4 waves per SIMD, every CU busy:
//   S32: 16 x v_mfma_f32_32x32x16_f16 (A from LDS by ds_read_b128, B = 16 register fragments),
//        then the previous chunk's 16 activations per lane: exp2, add, log2, cvt_pk.
//   S16: 16 ds_read_b128, each feeding two v_mfma_f32_16x16x32_f16 (two 16-ray tiles), two
//        chains per tile; the same 16 activations per lane.
// Prints wall time per chunk-iteration and the in-kernel clock (s_memtime / s_memrealtime).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef float f4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float sp2(float x) {
  return __builtin_amdgcn_logf(1.f + __builtin_amdgcn_exp2f(x));
}

template <int SHAPE>
__global__ void __launch_bounds__(256, SHAPE == 64 ? 2 : 4) k_chunk(const h8* __restrict__ seed, float* out,
                                                  long long* stamps, int iters) {
  __shared__ h8 lds[16 * 64 * 2];
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 16 * 64 * 2; i += blockDim.x) lds[i] = seed[(blockIdx.x * 7 + i) % 4096];
  __syncthreads();
  h8 hv[16], hv2[16];
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    hv[s] = seed[(lane * 16 + s + blockIdx.x) % 4096];
    hv2[s] = seed[(lane * 16 + s + blockIdx.x + 77) % 4096];
  }
  f16v acc32 = {}, pend32 = {}, acc64 = {};
  f4v acc[4] = {}, pend[4] = {};
  const long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
    const h8* A = lds + (it & 1) * 16 * 64 + lane;
    if (SHAPE == 64) {
      // two 32-ray tiles per wave: each A read feeds two independent 32x32x16 MFMAs
      f16v a = pend32, b = pend32;
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const h8 w = A[s * 64];
        a = __builtin_amdgcn_mfma_f32_32x32x16_f16(w, hv[s], a, 0, 0, 0);
        b = __builtin_amdgcn_mfma_f32_32x32x16_f16(w, hv2[s], b, 0, 0, 0);
      }
      h8 lo, hi, lo2, hi2;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        lo[j] = (_Float16)sp2(acc32[j]);
        hi[j] = (_Float16)sp2(acc32[8 + j]);
        lo2[j] = (_Float16)sp2(acc64[j]);
        hi2[j] = (_Float16)sp2(acc64[8 + j]);
      }
      hv[0] = lo; hv[1] = hi; hv2[0] = lo2; hv2[1] = hi2;
      acc32 = a; acc64 = b;
    } else if (SHAPE == 32) {
      f16v a = pend32;
#pragma unroll
      for (int s = 0; s < 16; ++s) a = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[s * 64], hv[s], a, 0, 0, 0);
      // activations of the previous chunk into two of the next chunk's operand fragments
      h8 lo, hi;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        lo[j] = (_Float16)sp2(acc32[j]);
        hi[j] = (_Float16)sp2(acc32[8 + j]);
      }
      hv[0] = lo;
      hv[1] = hi;
      acc32 = a;
    } else {
      f4v a[4] = {pend[0], pend[1], pend[2], pend[3]};
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const h8 w = A[s * 64];
        // two 16-ray tiles (B = hv[s] / hv[s ^ 8]), two chains per tile (alternate k-steps)
        a[(s & 1)] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w, hv[s], a[s & 1], 0, 0, 0);
        a[2 + (s & 1)] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w, hv[s ^ 8], a[2 + (s & 1)], 0, 0, 0);
      }
      h8 lo, hi;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        lo[r] = (_Float16)sp2(acc[0][r]);
        lo[4 + r] = (_Float16)sp2(acc[1][r]);
        hi[r] = (_Float16)sp2(acc[2][r]);
        hi[4 + r] = (_Float16)sp2(acc[3][r]);
      }
      hv[0] = lo;
      hv[8] = hi;
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t] = a[t];
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
  for (int r = 0; r < 16; ++r) s += acc32[r] + acc64[r];
  for (int k = 0; k < 16; ++k) for (int j = 0; j < 8; ++j) s += (float)hv2[k][j];
  for (int t = 0; t < 4; ++t) for (int r = 0; r < 4; ++r) s += acc[t][r];
  for (int k = 0; k < 16; ++k) for (int j = 0; j < 8; ++j) s += (float)hv[k][j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) { stamps[2 * blockIdx.x] = t1 - t0; stamps[2 * blockIdx.x + 1] = r1 - r0; }
}

template <int SHAPE>
void run(const char* name, const h8* seed, float* out, long long* st, int blocks, int iters) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int w = 0; w < 3; ++w) k_chunk<SHAPE><<<blocks, 256>>>(seed, out, st, iters);
  (void)hipEventRecord(a);
  const int reps = 5;
  for (int w = 0; w < reps; ++w) k_chunk<SHAPE><<<blocks, 256>>>(seed, out, st, iters);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, a, b);
  std::vector<long long> h(2 * blocks);
  (void)hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost);
  std::vector<double> clk;
  for (int i = 0; i < blocks; ++i) clk.push_back(h[2 * i] / (double)h[2 * i + 1] * 100.0);
  std::sort(clk.begin(), clk.end());
  const double flop = (double)blocks * 4 * iters * 16 * 32768.0 * reps * (SHAPE == 64 ? 2 : 1);
  printf("%-44s %8.3f ms/launch  %7.1f TF/s  clock %6.0f MHz\n", name, ms / reps,
         flop / (ms * 1e-3) / 1e12, clk[clk.size() / 2]);
}

int main() {
  const int blocks = 256 * 4, iters = 20000;  // 2 blocks of 4 waves per CU... x2 rounds
  std::vector<_Float16> hs(4096 * 8);
  unsigned x = 12345;
  for (auto& v : hs) { x = x * 1664525u + 1013904223u; v = (_Float16)(((x >> 9) & 0xffff) / 65536.0f - 0.5f); }
  h8* seed;
  float* out;
  long long* st;
  (void)hipMalloc(&seed, hs.size() * 2);
  (void)hipMemcpy(seed, hs.data(), hs.size() * 2, hipMemcpyHostToDevice);
  (void)hipMalloc(&out, blocks * 256 * 4);
  (void)hipMalloc(&st, blocks * 16);
  run<32>("S32: 16 x 32x32x16, 16 activations/lane", seed, out, st, blocks, iters);
  run<16>("S16: 32 x 16x16x32 (2 tiles), 16 act/lane", seed, out, st, blocks, iters);
  run<64>("S64: 2 tiles x 32x32x16 share A, 2 w/SIMD", seed, out, st, blocks / 2, iters);
  run<32>("S32 again", seed, out, st, blocks, iters);
  run<16>("S16 again", seed, out, st, blocks, iters);
  return 0;
}
