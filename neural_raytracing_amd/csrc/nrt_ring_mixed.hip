// NRT_MIXED intersect: the FP16 march + coarse scan (k_march16, the 2.5 PF path) with the few
// decisions FP16 cannot make taken again at FP32 accuracy on the split engine (nrt_ring3.h).
//
// The march's hit test `sdf <= eps` and its `t < max_t` test (sdfs.py:119-131), and the scan's
// argmin (sdfs.py:243-246), are the only places where an SDF error changes the result
// discontinuously; everywhere else FP16's error moves t, p and the throughput by about the error
// itself.  So:
//   1. k_march16 marches every ray and scans every primary ray at FP16 as usual, and flags a ray
//      at its first step whose value lies within refine_d * (1 + i/16) of eps (or whose next t lies
//      that close to max_t) -- amb[ray] = that step's (i, t); the scan also keeps the runner-up
//      key (keys2) beside the minimum;
//   2. k_refine_list gathers the flagged rays, and k_march3 (the split engine, FP32 accuracy)
//      marches each of them again from t = 0 (option "mixed_restart"; resuming at the flagged
//      step's (i, t) instead keeps t's FP16 drift, and a slowly converging ray then still stops
//      one step off the FP32 march: measured 1,464 step flips vs 4 on the 800^2 frame);
//   3. sdf(best) runs on the split engine for every ray, and for a ray whose FP16 minimum and
//      runner-up lie within refine_s of each other at the runner-up too; the smaller value (the
//      first index on a tie, the reference's strict-<) gives the throughput and the argmin;
//   4. k_march_finish unpacks t / hit into p, n and the hit list as for every ring march.
// The normals and the shading of an NRT_MIXED frame run at fp32-split (nrt_sdf_intersect and the
// shading entries map NRT_MIXED to NRT_FP32_SPLIT).
#include "nrt_launch.h"

namespace nrt {

__global__ void k_add_count(const int32_t* __restrict__ count, unsigned long long* __restrict__ acc) {
  if (threadIdx.x == 0) atomicAdd(acc, (unsigned long long)*count);
}

int ring_march_mixed(const nrt_sdf* s, const float* rays, int64_t P, const MarchArgs& ma, float* t,
                     uint8_t* hit, float* p, float* n, float* raw_n, float* thr, int32_t* idx,
                     int32_t* cnt, unsigned long long* keys, char* ws, hipStream_t st) {
  const bool scan = ma.primary != 0;
  const size_t k8 = ((size_t)P * 8 + 255) & ~(size_t)255;
  auto* keys2 = reinterpret_cast<unsigned long long*>(ws);
  auto* amb = reinterpret_cast<unsigned long long*>(ws + k8);
  auto* list = reinterpret_cast<int32_t*>(ws + 2 * k8);
  auto* lcount = reinterpret_cast<int32_t*>(ws + 2 * k8 + (((size_t)P * 4 + 255) & ~(size_t)255));
  const float rd = 1e-7f * (float)option(OPT_MIXED_D), rs = 1e-7f * (float)option(OPT_MIXED_S);
  if (scan) {
    NRT_HIP(hipMemsetAsync(keys, 0xff, (size_t)P * 8, st));
    NRT_HIP(hipMemsetAsync(keys2, 0xff, (size_t)P * 8, st));
  }
  NRT_HIP(hipMemsetAsync(amb, 0xff, (size_t)P * 8, st));
  NRT_HIP(hipMemsetAsync(lcount, 0, sizeof(int32_t), st));
  // 1. FP16 march + scan, flagging
  MarchArgs m16 = ma;
  m16.refine_d = rd;
  m16.drift_model = (int)option(OPT_MIXED_DRIFT);
  const int64_t restart = option(OPT_MIXED_RESTART);
  // restart 2: resume at the zone checkpoint (option "mixed_zone")
  m16.zone = restart == 2 ? 1e-7f * (float)option(OPT_MIXED_ZONE) : 0.f;
  m16.amb = amb;
  m16.keys2 = scan ? keys2 : nullptr;
  if (int rc = ring_march16_launch(s, rays, P, m16, t, thr, keys, st, false)) return rc;
  // 2. the flagged rays, resumed on the split engine
  k_refine_list<><<<dim3(std::min<int64_t>(ceil_div64(P, 256), 2048)), dim3(256), 0, st>>>(
      amb, P, list, lcount);
  if (int rc = check_launch("k_refine_list")) return rc;
  if (ma.evals)  // profiling only: the flagged-ray count (nrt_profile_refined)
    k_add_count<<<dim3(1), dim3(64), 0, st>>>(lcount, ma.evals + 1);
  MarchArgs mr = ma;
  mr.primary = 0;
  mr.scan_idx = nullptr;
  mr.list = list;
  mr.count = lcount;
  // option "mixed_restart" (default): a flagged ray marches again from t = 0 -- resumed at the
  // flagged step instead, it would carry the FP16 march's drift of t into the decision
  mr.start = restart == 1 ? nullptr : amb;
  if (int rc = ring3_launch(s, rays, P, mr, t, nullptr, nullptr, st, 2)) return rc;
  // 3. sdf(best) at FP32 accuracy, over both candidates where FP16 could not order them
  if (scan) {
    auto* kbest = amb;  // the march flags are spent
    NRT_HIP(hipMemsetAsync(kbest, 0xff, (size_t)P * 8, st));
    MarchArgs mb = ma;
    mb.keys2 = keys2;
    mb.kbest = kbest;
    mb.refine_s = rs;
    if (int rc = ring3_launch(s, rays, P, mb, nullptr, thr, keys, st, 3)) return rc;
    k_scan_pick<><<<dim3(ceil_div64(P, 256)), dim3(256), 0, st>>>(kbest, P, keys, thr);
    if (int rc = check_launch("k_scan_pick")) return rc;
  }
  // 4. unpack
  k_march_finish<><<<dim3(std::min<int64_t>(ceil_div64(P, 256), 2048)), dim3(256), 0, st>>>(
      rays, P, t, hit, p, n, raw_n, idx, cnt);
  return check_launch("k_march_finish");
}

}  // namespace nrt
