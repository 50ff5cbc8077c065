// Runtime plumbing: thread-local error string, device buffers, hipEvent timing hook.
#include <algorithm>
#include <cmath>
#include <cstdio>

#include "../../include/mec.h"
#include "models.h"

namespace mec {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }
const char* last_error() { return g_last_error.c_str(); }

// Options / tune cache of the handle the calling thread is serving (OptScope), else the
// process defaults (handle-less kernel entry points such as mec_gemm_f16).
Options& default_options() {
  static Options o;
  return o;
}
TuneCache& default_tune_cache() {
  static TuneCache c;
  return c;
}
static thread_local const Options* t_opts = nullptr;
static thread_local TuneCache* t_tune = nullptr;
static thread_local unsigned* t_flag = nullptr;
const Options& opt() { return t_opts ? *t_opts : default_options(); }
TuneCache& tune_cache() { return t_tune ? *t_tune : default_tune_cache(); }
unsigned* range_flag() { return t_flag; }
OptScope::OptScope(const Options* o, TuneCache* t, unsigned* flag) : po(t_opts), pt(t_tune), pf(t_flag) {
  t_opts = o;
  t_tune = t;
  t_flag = flag;
}
OptScope::~OptScope() {
  t_opts = po;
  t_tune = pt;
  t_flag = pf;
}

int DevBuf::ensure(size_t n) {
  if (n <= bytes) return 0;
  release();
  MEC_HIP(hipMalloc(&p, n));
  bytes = n;
  return 0;
}

void DevBuf::release() {
  if (p) (void)hipFree(p);
  p = nullptr;
  bytes = 0;
}

int upload(DevBuf& b, const void* host, size_t bytes) {
  MEC_TRY(b.ensure(bytes));
  MEC_HIP(hipMemcpy(b.p, host, bytes, hipMemcpyHostToDevice));
  return 0;
}

int Prof::begin(int t, hipStream_t s) {
  if (t != tag || tag == TAG_NONE) return 0;
  while (ev.size() < used + 2) {
    hipEvent_t e;
    MEC_HIP(hipEventCreate(&e));
    ev.push_back(e);
  }
  MEC_HIP(hipEventRecord(ev[used], s));
  return 0;
}

int Prof::end(int t, hipStream_t s) {
  if (t != tag || tag == TAG_NONE) return 0;
  MEC_HIP(hipEventRecord(ev[used + 1], s));
  used += 2;
  return 0;
}

int Prof::read(double* total_ms, int* count) {
  double tot = 0.0;
  for (size_t i = 0; i + 1 < used; i += 2) {
    MEC_HIP(hipEventSynchronize(ev[i + 1]));
    float ms = 0.f;
    MEC_HIP(hipEventElapsedTime(&ms, ev[i], ev[i + 1]));
    tot += ms;
  }
  *total_ms = tot;
  *count = (int)(used / 2);
  return 0;
}

Prof::~Prof() {
  for (auto e : ev) (void)hipEventDestroy(e);
}

int Model::alloc_range_flag() {
  if (range_host) return 0;
  MEC_HIP(hipHostMalloc(reinterpret_cast<void**>(&range_host), sizeof(unsigned), hipHostMallocMapped));
  *range_host = 0;
  MEC_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&range_dev), range_host, 0));
  return 0;
}

Model::~Model() {
  if (range_host) (void)hipHostFree(range_host);
}

int Model::check() {
  if (!range_host || !*reinterpret_cast<volatile unsigned*>(range_host)) return 0;
  *range_host = 0;
  set_error("fp32x3: an activation left the f16 hi / lo range (|x| >= 65520, or NaN / inf) in a forward since "
            "the last check; its outputs are invalid (re-run the batch on an MEC_PREC_FP32 handle, and create "
            "the fp32x3 handle again with more x3_headroom: mec_create_opt; mec_model_x3_report lists the "
            "exponents)");
  return MEC_ERR_X3_RANGE;
}

void Model::x3_note(const std::string& name, int s, double bound) {
  char buf[160];
  snprintf(buf, sizeof buf, "%s s=%d bound=%.6g\n", name.c_str(), s, bound);
  x3_report += buf;
}

float split_planes(const float* w, size_t n, f16* hi, f16* lo) {
  float mx = 0.f;
  for (size_t i = 0; i < n; ++i) mx = std::max(mx, std::fabs(w[i]));
  int e = 0;
  if (mx > 0.f && std::isfinite(mx)) {
    e = (int)std::floor(std::log2(16384.0 / (double)mx));
    while (std::ldexp((double)mx, e) > 16384.0) --e;  // guard the log2 rounding
  }
  for (size_t i = 0; i < n; ++i) {
    const float x = std::ldexp(w[i], e);  // exact (power of two), unless it leaves the f32 range
    const f16 h = (f16)x;
    hi[i] = h;
    lo[i] = (f16)(x - (float)h);  // x - hi is exact in f32
  }
  return std::ldexp(1.0f, -e);
}

int activation_exp(double bound, double target) {
  if (!(bound > 0.0) || !std::isfinite(bound)) return 0;
  int e = (int)std::floor(std::log2(target / bound));
  while (std::ldexp(bound, e) > target) --e;  // guard the log2 rounding
  return std::max(-40, std::min(40, e));
}

}  // namespace mec
