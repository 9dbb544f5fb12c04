// Microbenchmark: cycles per v_mfma_f32_32x32x16_f16 with K filler instructions of one kind in
// each MFMA gap (one wave per SIMD, 256 CUs).  Measures what the softplus of the FP16 ring engine
// (k_march16) costs beside its MFMAs: v_exp/v_log in f32 and f16, v_add, v_cvt_pk, SALU moves.
// Output: one line per variant, median over waves of (s_memtime delta) / iterations.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));

#define F4(x) x x x x
template <int V>
__global__ void __launch_bounds__(256) k_issue(float* out, long long* cyc, int iters) {
  f16v acc = {}, acc1 = {}, acc2 = {}, acc3 = {};
  h8 a, b;
  for (int j = 0; j < 8; ++j) { a[j] = (_Float16)(threadIdx.x * 1e-3f); b[j] = (_Float16)(j * 1e-2f); }
  float x = threadIdx.x * 1e-3f, y = x + 1.f, z = x + 2.f, w = x + 3.f;
  int s0 = 0, s1 = 1;
  long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 2
  for (int i = 0; i < iters; ++i) {
    if (i & 1) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
    else acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc1, 0, 0, 0);
    if (V == 1) asm volatile(F4("v_exp_f32 %0, %0\n") : "+v"(x));
    if (V == 2) asm volatile(F4("v_log_f32 %0, %0\n") : "+v"(x));
    if (V == 3) asm volatile(F4("v_exp_f16 %0, %0\n") : "+v"(x));
    if (V == 4) asm volatile(F4("v_log_f16 %0, %0\n") : "+v"(x));
    if (V == 5) asm volatile(F4("v_add_f32 %0, %0, %0\n") : "+v"(x));
    if (V == 6) asm volatile(F4("v_cvt_pk_f16_f32 %0, %0, %0\n") : "+v"(x));
    if (V == 7) asm volatile(F4("s_mov_b32 %0, %1\n") : "+s"(s0) : "s"(s1));
    if (V == 8) asm volatile(F4("v_pk_fma_f16 %0, %0, %0, %0\n") : "+v"(x));
    // the current softplus per element, twice: exp, add, log, (half a cvt_pk)
    if (V == 9) asm volatile("v_exp_f32 %0, %0\nv_add_f32 %0, 1.0, %0\nv_log_f32 %0, %0\n"
                             "v_exp_f32 %1, %1\nv_add_f32 %1, 1.0, %1\nv_log_f32 %1, %1\n"
                             "v_cvt_pk_f16_f32 %2, %0, %1\n" : "+v"(x), "+v"(y), "+v"(z));
    // independent chains (latency hidden): 4 exp_f32 on 4 registers
    if (V == 10) asm volatile("v_exp_f32 %0, %0\nv_exp_f32 %1, %1\nv_exp_f32 %2, %2\nv_exp_f32 %3, %3\n"
                              : "+v"(x), "+v"(y), "+v"(z), "+v"(w));
    if (V == 11) asm volatile("v_exp_f16 %0, %0\nv_exp_f16 %1, %1\nv_exp_f16 %2, %2\nv_exp_f16 %3, %3\n"
                              : "+v"(x), "+v"(y), "+v"(z), "+v"(w));
    if (V == 12) asm volatile("v_log_f16 %0, %0\nv_log_f16 %1, %1\nv_log_f16 %2, %2\nv_log_f16 %3, %3\n"
                              : "+v"(x), "+v"(y), "+v"(z), "+v"(w));
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  float s = x + y + z + w + (float)s0;
  for (int r = 0; r < 16; ++r) s += acc[r] + acc1[r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

template <int V>
void run(const char* name, float* out, long long* cyc, int blocks, int iters) {
  k_issue<V><<<blocks, 256>>>(out, cyc, iters);
  (void)hipDeviceSynchronize();
  k_issue<V><<<blocks, 256>>>(out, cyc, iters);
  (void)hipDeviceSynchronize();
  std::vector<long long> h(blocks * 4);
  (void)hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.end());
  printf("%-28s %8.2f cyc/MFMA (median over %d waves)\n", name, (double)h[h.size() / 2] / iters,
         (int)h.size());
}

int main() {
  const int blocks = 256, iters = 4096;
  float* out;
  long long* cyc;
  (void)hipMalloc(&out, blocks * 256 * 4);
  (void)hipMalloc(&cyc, blocks * 4 * 8);
  run<0>("mfma only", out, cyc, blocks, iters);
  run<1>("+4 v_exp_f32 (dep)", out, cyc, blocks, iters);
  run<2>("+4 v_log_f32 (dep)", out, cyc, blocks, iters);
  run<3>("+4 v_exp_f16 (dep)", out, cyc, blocks, iters);
  run<4>("+4 v_log_f16 (dep)", out, cyc, blocks, iters);
  run<5>("+4 v_add_f32 (dep)", out, cyc, blocks, iters);
  run<6>("+4 v_cvt_pk_f16_f32 (dep)", out, cyc, blocks, iters);
  run<7>("+4 s_mov_b32", out, cyc, blocks, iters);
  run<8>("+4 v_pk_fma_f16 (dep)", out, cyc, blocks, iters);
  run<9>("+2 softplus (exp,add,log)+cvt", out, cyc, blocks, iters);
  run<10>("+4 v_exp_f32 (indep)", out, cyc, blocks, iters);
  run<11>("+4 v_exp_f16 (indep)", out, cyc, blocks, iters);
  run<12>("+4 v_log_f16 (indep)", out, cyc, blocks, iters);
  return 0;
}
