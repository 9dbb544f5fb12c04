// nrt_api_cam.hip -- ray generation, frames and composite launchers
#include "nrt_launch.h"

using namespace nrt;

extern "C" {
int nrt_raygen(const nrt_camera* cams, int32_t N, int32_t x0, int32_t y0, int32_t W, int32_t H,
               float with_noise, const float* noise, const float* positions, float* rays,
               void* stream) {
  if (!cams || N < 1 || W < 0 || H < 0 || !rays) { set_error("nrt_raygen: bad argument"); return NRT_EINVAL; }
  const int64_t total = (int64_t)N * W * H;
  if (total == 0) return NRT_OK;
  hipStream_t st = (hipStream_t)stream;
  nrt_camera* dcam = nullptr;
  NRT_HIP(hipMallocAsync((void**)&dcam, sizeof(nrt_camera) * N, st));
  NRT_HIP(hipMemcpyAsync(dcam, cams, sizeof(nrt_camera) * N, hipMemcpyHostToDevice, st));
  k_raygen<><<<dim3(ceil_div64(total, 256)), dim3(256), 0, st>>>(dcam, N, x0, y0, W, H, with_noise, noise, positions, rays);
  int rc = check_launch("k_raygen");
  (void)hipFreeAsync(dcam, st);
  return rc;
}

int nrt_composite(const float* rgb, const float* thr, const uint8_t* hit, int32_t N, int32_t W,
                  int32_t H, int32_t alpha, int32_t fill, float bg, float* img, int32_t IW,
                  int32_t IH, int32_t C, int32_t X0, int32_t Y0, void* stream) {
  if (!rgb || !img || (alpha && !thr) || (fill && !hit)) { set_error("nrt_composite: bad argument"); return NRT_EINVAL; }
  const int64_t total = (int64_t)N * W * H;
  if (total == 0) return NRT_OK;
  if (X0 < 0 || Y0 < 0 || X0 + W > IW || Y0 + H > IH) { set_error("nrt_composite: tile outside image"); return NRT_EINVAL; }
  k_composite<><<<dim3(ceil_div64(total, 256)), dim3(256), 0, (hipStream_t)stream>>>(
      rgb, thr, hit, N, W, H, alpha, fill, bg, img, IW, IH, C, X0, Y0);
  return check_launch("k_composite");
}


}  // extern "C"
