// nrt_render_tile -- one fused pathtrace tile (main.py:63-90) for Direct / NeRFIntegrator(Direct)
// in one C-ABI call: raygen -> march + coarse scan + normals -> Direct shading -> composite.  The
// same launches render.py chains from Python (nrt_raygen, nrt_sdf_intersect, nrt_shade_direct,
// nrt_composite), stream-ordered, with every intermediate in one caller-owned workspace, so a
// binding (ctypes / cgo / JNI) renders a tile with one call and no allocation.
#include "nrt_launch.h"

namespace nrt {
namespace {

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// workspace carve: rays [P,6] | t [P] | hit u8[P] | p, n, raw_n, wi [P,3] | throughput [P] |
// rgb [P,3] | hit_idx i32[P] | hit_count i32 | the intersect workspace
struct TileWs {
  float *rays, *t, *p, *n, *raw, *wi, *thr, *rgb;
  uint8_t* hit;
  int32_t *idx, *cnt;
  void* iws;
};

size_t tile_bytes(const nrt_sdf* sdf, int64_t P, TileWs* w, char* base) {
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* q = base ? base + off : nullptr;
    off += align256(bytes);
    return q;
  };
  TileWs x{};
  x.rays = (float*)take((size_t)P * 24);
  x.t = (float*)take((size_t)P * 4);
  x.hit = (uint8_t*)take((size_t)P);
  x.p = (float*)take((size_t)P * 12);
  x.n = (float*)take((size_t)P * 12);
  x.raw = (float*)take((size_t)P * 12);
  x.wi = (float*)take((size_t)P * 12);
  x.thr = (float*)take((size_t)P * 4);
  x.rgb = (float*)take((size_t)P * 12);
  x.idx = (int32_t*)take((size_t)std::max<int64_t>(P, 1) * 4);
  x.cnt = (int32_t*)take(4);
  x.iws = take(nrt_intersect_workspace_bytes(sdf, P));
  if (w) *w = x;
  return off;
}

}  // namespace
}  // namespace nrt

using namespace nrt;

extern "C" {

size_t nrt_render_tile_workspace_bytes(const nrt_sdf* sdf, int32_t N, int32_t W, int32_t H) {
  if (!sdf || N < 1 || W < 0 || H < 0) return 0;
  return tile_bytes(sdf, (int64_t)N * W * H, nullptr, nullptr);
}

int nrt_render_tile(const nrt_camera* host_cams, int32_t N, int32_t x0, int32_t y0, int32_t W,
                    int32_t H, float with_noise, const float* noise, const nrt_sdf* sdf,
                    const nrt_march_params* params, const nrt_bsdf* bsdf, const nrt_light* light,
                    int32_t with_alpha, float background, float* image, int32_t img_w,
                    int32_t img_h, int32_t channels, int32_t X0, int32_t Y0, void* workspace,
                    void* stream) {
  if (!host_cams || N < 1 || W < 0 || H < 0 || !sdf || !params || !bsdf || !light || !image ||
      !workspace) {
    set_error("nrt_render_tile: bad argument");
    return NRT_EINVAL;
  }
  if (channels != (with_alpha ? 4 : 3)) {
    set_error("nrt_render_tile: channels must be 4 with alpha (NeRFIntegrator), 3 without");
    return NRT_EINVAL;
  }
  const int64_t P = (int64_t)N * W * H;
  if (P == 0) return NRT_OK;
  TileWs w;
  tile_bytes(sdf, P, &w, (char*)workspace);
  hipStream_t st = (hipStream_t)stream;
  if (int rc = nrt_raygen(host_cams, N, x0, y0, W, H, with_noise, noise, nullptr, w.rays, stream))
    return rc;
  const bool primary = params->primary != 0;
  if (int rc = nrt_sdf_intersect(sdf, w.rays, P, params, w.t, w.hit, w.p, w.n, w.raw, w.wi,
                                 primary ? w.thr : nullptr, w.idx, w.cnt, w.iws, stream))
    return rc;
  // Direct.sample leaves misses black (integrators.py:156-206); without the scan the throughput
  // (alpha logit) is 0 as in the reference's non-primary interaction
  NRT_HIP(hipMemsetAsync(w.rgb, 0, (size_t)P * 12, st));
  if (!primary) NRT_HIP(hipMemsetAsync(w.thr, 0, (size_t)P * 4, st));
  if (int rc = nrt_shade_direct(bsdf, light, w.p, w.n, w.wi, w.idx, w.cnt, P, w.rgb, nullptr,
                                params->precision, stream))
    return rc;
  return nrt_composite(w.rgb, w.thr, w.hit, N, W, H, with_alpha ? 1 : 0, with_alpha ? 0 : 1,
                       background, image, img_w, img_h, channels, X0, Y0, stream);
}

}  // extern "C"
