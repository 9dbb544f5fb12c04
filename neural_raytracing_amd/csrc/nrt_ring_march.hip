// FP16 march + coarse scan on the block-cooperative LDS weight ring (k_march16), load-balanced
// job lists on a persistent grid; then sdf(best) (mode 1) and the hit list.
#include "nrt_launch.h"

namespace nrt {

int ring_march16_launch(const nrt_sdf* s, const float* rays, int64_t P, const MarchArgs& ma,
                        float* t, float* thr, unsigned long long* keys, hipStream_t st,
                        bool best16, uint8_t* visible) {
  const size_t bias_bytes = ring_bias_bytes(s);
  int dev = 0, cus = 0;
  NRT_HIP(hipGetDevice(&dev));
  NRT_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const bool scan = ma.primary != 0;
  return ring_dispatch(s, [&]<int NB, int NE, bool FOLD>() -> int {
    // the SphereSDF table goes into LDS behind the ring when it fits and costs no resident block
    // (spheres_value_halves: the two lanes of a ray split the spheres; colocate's 64 spheres:
    // k_march16 51.3 -> 43.8 ms); a table of a few spheres stays on scalar loads
    constexpr int kLdsSpheresMin = 8;
    const size_t base = ring::Cfg<NB, NE, kRingWaves>::lds_bytes(bias_bytes);
    const size_t ring_lds = (base + 15) & ~size_t(15);
    const size_t sph = s->host_dev.kind == 2
                           ? (size_t)ring::sphere_pair_records(s->host_dev.n_spheres) * ring::kSpherePairF4 * 16
                           : 0;  // the pair table (ring::build_sphere_pairs)
    MarchArgs a = ma;
    a.lds_spheres = (sph > 0 && s->host_dev.n_spheres >= kLdsSpheresMin && ring_lds + sph <= (size_t)kLdsBytes &&
                     kLdsBytes / (ring_lds + sph) == kLdsBytes / base) ? (int)ring_lds : 0;
    const size_t lds0 = a.lds_spheres ? ring_lds + sph : base;
    auto launch = [&](auto kern, const char* name, bool plain = false) -> int {
      // the plain march stages its lines (MarchArgs::stage) when that keeps the blocks per CU
      MarchArgs b = a;
      size_t lds = lds0;
      if (plain) {
        stage_lds(b, lds, kRingWaves);
        if (b.stage && kLdsBytes / lds != kLdsBytes / lds0) { b.stage = 0; lds = lds0; }
      }
      if (int rc = set_lds(kern, lds)) return rc;
      int per_cu = 0;
      NRT_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64 * kRingWaves, lds));
      // persistent grid: every resident block slot, but no more waves than 32-ray tiles
      const int64_t slots = (int64_t)std::max(per_cu, 1) * std::max(cus, 1);
      // every resident slot unless the rays are fewer than 16 a wave: a small batch (a training
      // step's 38,400 rays) spreads over every CU, the job lists giving idle lanes scan segments
      // (measured: the mixed training step 33.5 -> 31.6 ms against 32 rays a wave)
      int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(slots, ceil_div64(P, 16 * kRingWaves)));
      // option "march_blocks": force the grid (tests check that results do not depend on the schedule)
      if (const int64_t f = option(OPT_MARCH_BLOCKS)) blocks = (int)std::min<int64_t>(f, 1 << 20);
      if (a.queue) NRT_HIP(hipMemsetAsync(a.queue, 0, sizeof(unsigned int), st));
      ProfScope prof(name, st);
      kern<<<dim3(blocks), dim3(64 * kRingWaves), lds, st>>>(
          s->host_dev, s->mlp->host_dev, rays, P, b, t, visible, nullptr, nullptr, nullptr, thr, keys);
      return check_launch(name);
    };
    // the shadow march (visible != nullptr) and NRT_MIXED's flagging march are their own
    // instantiations (the plain march carries none of them)
    if (visible) return launch(k_occl16<NB, NE, kRingWaves, FOLD>, "k_occl16");
    if (ma.amb) return launch(k_march16<NB, NE, kRingWaves, FOLD, true>, "k_march16");
    if (int rc = launch(k_march16<NB, NE, kRingWaves, FOLD>, "k_march16", true)) return rc;
    if (scan && best16) return launch(k_scan_best16<NB, NE, kRingWaves, FOLD>, "k_scan_best16");
    return NRT_OK;
  });
}

int ring_march(const nrt_sdf* s, const float* rays, int64_t P, const MarchArgs& ma, float* t,
               uint8_t* hit, float* p, float* n, float* raw_n, float* thr, int32_t* idx,
               int32_t* cnt, unsigned long long* keys, hipStream_t st) {
  const bool scan = ma.primary != 0;
  // option "scan_best32": sdf(best) on the FP32 engine -- the throughput -1000 sdf(best)
  // (sdfs.py:137) multiplies the FP16 SDF error by 1000 in the alpha logit
  const bool best32 = scan && option(OPT_SCAN_BEST32) != 0 && ring32_supported(s);
  if (scan) NRT_HIP(hipMemsetAsync(keys, 0xff, (size_t)P * sizeof(unsigned long long), st));
  if (int rc = ring_march16_launch(s, rays, P, ma, t, thr, keys, st, !best32)) return rc;
  if (best32)
    if (int rc2 = ring_scan_best32(s, rays, P, ma, thr, keys, st)) return rc2;
  // the march packed (hit, t) into t: unpack, p / n / raw_n and the hit list, coalesced
  k_march_finish<><<<dim3(std::min<int64_t>(ceil_div64(P, 256), 2048)), dim3(256), 0, st>>>(
      rays, P, t, hit, p, n, raw_n, idx, cnt);
  return check_launch("k_march_finish");
}

}  // namespace nrt
