// Host-side AddressSanitizer run of the MLP packer (SURVEY §5 debug aids): nrt_mlp_create builds
// every fragment layout and index map on the host before its first device allocation, so on a
// machine without a GPU it runs all of that code and then fails at hipMalloc.  Built host-only
// with -fsanitize=address by tools/asan/run.sh; any out-of-range access in the packing loops
// aborts with an ASan report.  Shapes: every MLP the path packs (tests/test_gpu_train.py SHAPES)
// plus ragged out / latent / skip corners.
#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>

#include "nrt.h"

static int pack(int in, int hidden, int layers, int out, int freqs, int skip, int latent) {
  nrt_mlp_desc d{in, hidden, layers, out, freqs, skip, latent, NRT_ACT_LEAKY_RELU};
  const int dp = in + 2 * freqs + latent;
  std::mt19937 rng(hidden * 131 + layers);
  std::uniform_real_distribution<float> u(-1.f, 1.f);
  std::vector<std::vector<float>> W, B;
  auto add = [&](int R, int C) {
    W.emplace_back(R * C);
    B.emplace_back(R);
    for (float& v : W.back()) v = u(rng);
    for (float& v : B.back()) v = u(rng);
  };
  add(hidden, dp);
  for (int i = 0; i < layers; ++i)
    add(hidden, hidden + ((i != layers - 1 && i % skip == 0) ? dp : 0));
  add(out, hidden);
  std::vector<float> basis(std::max(1, in * freqs));  // never a null pointer at F = 0
  for (float& v : basis) v = u(rng);
  std::vector<const float*> wp, bp;
  for (size_t l = 0; l < W.size(); ++l) {
    wp.push_back(W[l].data());
    bp.push_back(B[l].data());
  }
  nrt_mlp* m = nullptr;
  const int rc = nrt_mlp_create(&d, basis.data(), wp.data(), bp.data(), &m);
  if (m) nrt_mlp_destroy(m);
  std::printf("pack %dx%d in=%d out=%d F=%d skip=%d latent=%d -> rc %d (%s)\n", layers, hidden, in,
              out, freqs, skip, latent, rc, rc ? nrt_last_error() : "ok");
  // no device here: the packing ran and the upload failed (NRT_EHIP); anything else is a bug
  return rc == NRT_OK || rc == NRT_EHIP ? 0 : 1;
}

int main() {
  int bad = 0;
  bad += pack(3, 64, 8, 3, 16, 3, 0);
  bad += pack(3, 128, 8, 1, 32, 3, 0);
  bad += pack(70, 64, 8, 3, 16, 3, 0);
  bad += pack(3, 32, 4, 4, 8, 3, 8);
  bad += pack(3, 96, 6, 3, 64, 3, 0);
  bad += pack(3, 256, 16, 8, 128, 3, 0);
  bad += pack(3, 256, 10, 3, 16, 3, 0);
  bad += pack(3, 256, 8, 1, 16, 3, 0);
  bad += pack(3, 128, 5, 65, 16, 3, 0);
  bad += pack(70, 64, 8, 3, 16, 3, 0);
  bad += pack(5, 32, 1, 96, 0, 1, 3);
  bad += pack(3, 64, 7, 33, 5, 2, 1);
  std::printf("%s\n", bad ? "FAIL" : "asan pack driver: all shapes packed cleanly");
  return bad ? 1 : 0;
}
