// nrt_common.hip -- error state and library identity
#include "nrt_launch.h"

#include <atomic>
#include <vector>

namespace nrt {

static thread_local std::string g_err;

void set_error(const std::string& msg) { g_err = msg; }

int hip_fail(hipError_t e, const char* what) {
  g_err = std::string(what) + ": " + hipGetErrorString(e);
  return NRT_EHIP;
}

int max_hidden(const nrt_mlp* m) { return m ? m->desc.hidden : 0; }

// nrt_set_option table: name, default
struct OptionDef {
  const char* name;
  int64_t def;
};
static const OptionDef kOptions[OPT_COUNT] = {
    {"ring16", 1}, {"ring32", 1}, {"normals16", 1}, {"scan_best32", 1},
    {"march_blocks", 0}, {"shade_program", 1}, {"nerf_fused", 1}, {"max_waves", 0},
    {"shade_ring", 1}, {"normals_ring", 1}, {"xcd_lines", 0},
    {"mixed_refine_d", kMixedRefineD}, {"mixed_refine_s", kMixedRefineS}, {"mixed_restart", 1},
    {"mixed_drift", 0}, {"ring_occlusion", 1}, {"mixed_zone", 500000},
    {"bwd_colsplit", 1}, {"bwd_ring", 1}, {"march_queue", 2}, {"train_save", 1}, {"wgrad_tile", 0},
    {"march_stage", 1},
};
static std::atomic<int64_t> g_opts[OPT_COUNT] = {1, 1, 1, 1, 0, 1, 1, 0, 1, 1, 0,
                                                 kMixedRefineD, kMixedRefineS, 1, 0, 1, 500000, 1, 1, 2, 1, 0,
                                                 1};

int64_t option(Option o) { return g_opts[o].load(std::memory_order_relaxed); }

static int option_index(const char* name) {
  if (!name) return -1;
  for (int i = 0; i < OPT_COUNT; ++i)
    if (std::strcmp(kOptions[i].name, name) == 0) return i;
  return -1;
}

struct ProfRec {
  std::string name;
  hipEvent_t a, b;
  double flop;
};
static bool g_prof = false;        // NRT_PROF_TIMING: hipEvents around the profiled launches
static bool g_prof_evals = false;  // NRT_PROF_EVALS: the ring marches' evaluation counter
static std::vector<ProfRec> g_recs;

ProfScope::ProfScope(const char* n, hipStream_t s, double f) : name(n), stream(s), flop(f) {
  if (!g_prof) return;
  if (hipEventCreate(&start) != hipSuccess) { start = nullptr; return; }
  (void)hipEventRecord(start, stream);
}

ProfScope::~ProfScope() {
  if (!start) return;
  hipEvent_t stop;
  if (hipEventCreate(&stop) != hipSuccess) return;
  (void)hipEventRecord(stop, stream);
  g_recs.push_back({name, start, stop, flop});
}

static unsigned long long* g_evals[64] = {};

unsigned long long* profile_eval_counter() {
  if (!g_prof_evals) return nullptr;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  if (!g_evals[dev]) {
    // [0] SDF evaluations, [1] NRT_MIXED rays re-marched by the refinement
    if (hipMalloc(&g_evals[dev], 2 * sizeof(unsigned long long)) != hipSuccess) { g_evals[dev] = nullptr; return nullptr; }
    if (hipMemset(g_evals[dev], 0, 2 * sizeof(unsigned long long)) != hipSuccess) return nullptr;
  }
  return g_evals[dev];
}

}  // namespace nrt

using namespace nrt;

extern "C" {

void nrt_profile_enable(int flags) {
  nrt::g_prof = (flags & NRT_PROF_TIMING) != 0;
  nrt::g_prof_evals = (flags & NRT_PROF_EVALS) != 0;
  if (nrt::g_prof_evals) (void)nrt::profile_eval_counter();  // allocate outside any timed region
}

void nrt_profile_reset(void) {
  for (auto& r : nrt::g_recs) { (void)hipEventDestroy(r.a); (void)hipEventDestroy(r.b); }
  nrt::g_recs.clear();
  int dev = 0;
  if (hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < 64 && nrt::g_evals[dev])
    (void)hipMemset(nrt::g_evals[dev], 0, 2 * sizeof(unsigned long long));
}

int nrt_profile_evals(uint64_t* evals) {
  if (!evals) { set_error("nrt_profile_evals: null argument"); return NRT_EINVAL; }
  *evals = 0;
  int dev = 0;
  NRT_HIP(hipGetDevice(&dev));
  if (dev < 0 || dev >= 64 || !nrt::g_evals[dev]) return NRT_OK;
  unsigned long long v = 0;
  NRT_HIP(hipMemcpy(&v, nrt::g_evals[dev], sizeof(v), hipMemcpyDeviceToHost));
  *evals = v;
  return NRT_OK;
}

int nrt_profile_refined(uint64_t* rays) {
  if (!rays) { set_error("nrt_profile_refined: null argument"); return NRT_EINVAL; }
  *rays = 0;
  int dev = 0;
  NRT_HIP(hipGetDevice(&dev));
  if (dev < 0 || dev >= 64 || !nrt::g_evals[dev]) return NRT_OK;
  unsigned long long v = 0;
  NRT_HIP(hipMemcpy(&v, nrt::g_evals[dev] + 1, sizeof(v), hipMemcpyDeviceToHost));
  *rays = v;
  return NRT_OK;
}

int nrt_profile_read(const char* name, double* total_ms, int64_t* launches) {
  double tot = 0.0;
  int64_t n = 0;
  for (auto& r : nrt::g_recs) {
    if (name && r.name != name) continue;
    if (hipEventSynchronize(r.b) != hipSuccess) { set_error("nrt_profile_read: event sync failed"); return NRT_EHIP; }
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, r.a, r.b) != hipSuccess) { set_error("nrt_profile_read: elapsed failed"); return NRT_EHIP; }
    tot += ms;
    ++n;
  }
  if (total_ms) *total_ms = tot;
  if (launches) *launches = n;
  return NRT_OK;
}

int nrt_profile_flop(const char* name, double* flop) {
  if (!flop) { set_error("nrt_profile_flop: null argument"); return NRT_EINVAL; }
  double tot = 0.0;
  for (auto& r : nrt::g_recs)
    if (!name || r.name == name) tot += r.flop;
  *flop = tot;
  return NRT_OK;
}

int nrt_set_option(const char* name, int64_t value) {
  const int i = nrt::option_index(name);
  if (i < 0) { set_error(std::string("nrt_set_option: unknown option ") + (name ? name : "(null)")); return NRT_EINVAL; }
  if (value < 0) { set_error("nrt_set_option: negative value"); return NRT_EINVAL; }
  nrt::g_opts[i].store(value, std::memory_order_relaxed);
  return NRT_OK;
}

int nrt_get_option(const char* name, int64_t* value) {
  const int i = nrt::option_index(name);
  if (i < 0 || !value) { set_error("nrt_get_option: unknown option or null value"); return NRT_EINVAL; }
  *value = nrt::g_opts[i].load(std::memory_order_relaxed);
  return NRT_OK;
}

int nrt_reset_options(void) {
  for (int i = 0; i < OPT_COUNT; ++i) nrt::g_opts[i].store(nrt::kOptions[i].def, std::memory_order_relaxed);
  return NRT_OK;
}

const char* nrt_last_error(void) { return nrt::g_err.c_str(); }
int nrt_version(void) { return 1; }

int nrt_device_ok(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n < 1) return 0;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, 0) != hipSuccess) return 0;
  return std::strncmp(prop.gcnArchName, "gfx950", 6) == 0 ? 1 : 0;
}

}  // extern "C"
