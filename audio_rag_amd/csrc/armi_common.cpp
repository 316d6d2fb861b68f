// Error plumbing of the C ABI (thread-local last error).
#include <cstdio>
#include <map>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "armi_common.h"

namespace armi {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const std::string& msg) {
  set_error(msg);
  return code;
}

int hip_fail(hipError_t e, const char* what) {
  std::string m = std::string(what) + ": " + hipGetErrorName(e) + " (" + hipGetErrorString(e) + ")";
  set_error(m);
  return ARMI_ERR_HIP;
}

int allow_lds_raw(const void* kernel, size_t bytes) {
  if (bytes <= 65536) return ARMI_OK;
  static std::mutex mu;
  static std::map<std::pair<int, const void*>, size_t> raised;
  int dev = 0;
  ARMI_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> g(mu);
  size_t& have = raised[{dev, kernel}];
  if (have >= bytes) return ARMI_OK;
  ARMI_HIP(hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
  have = bytes;
  return ARMI_OK;
}

struct Timing {
  bool enabled = false;
  int period = 1;                        // time every period-th launch of a slot
  int64_t seen[ARMI_TIMING_SLOTS] = {};  // launches of the slot since timing was enabled
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pending[ARMI_TIMING_SLOTS];
  std::vector<std::pair<hipEvent_t, hipEvent_t>> spare;
  std::mutex mu;
};
static Timing& timing() {
  static Timing t;
  return t;
}

int TimedLaunch::begin(int s, hipStream_t st) {
  Timing& t = timing();
  std::lock_guard<std::mutex> g(t.mu);
  if (!t.enabled || s < 0 || s >= ARMI_TIMING_SLOTS) return 0;
  if (t.seen[s]++ % t.period != 0) return 0;
  if (t.spare.empty()) {
    hipEvent_t a, b;
    ARMI_HIP(hipEventCreate(&a));
    ARMI_HIP(hipEventCreate(&b));
    t.spare.emplace_back(a, b);
  }
  ev[0] = t.spare.back().first;
  ev[1] = t.spare.back().second;
  t.spare.pop_back();
  slot = s;
  stream = st;
  ARMI_HIP(hipEventRecord(ev[0], stream));
  return 1;
}

int TimedKernel::begin(int s, hipStream_t stream) {
  Timing& t = timing();
  std::lock_guard<std::mutex> g(t.mu);
  if (!t.enabled || s < 0 || s >= ARMI_TIMING_SLOTS) return 0;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  ARMI_HIP(hipStreamIsCapturing(stream, &cs));
  if (cs != hipStreamCaptureStatusNone) return 0;
  if (t.seen[s]++ % t.period != 0) return 0;
  if (t.spare.empty()) {
    hipEvent_t a, b;
    ARMI_HIP(hipEventCreate(&a));
    ARMI_HIP(hipEventCreate(&b));
    t.spare.emplace_back(a, b);
  }
  ev[0] = t.spare.back().first;
  ev[1] = t.spare.back().second;
  t.spare.pop_back();
  slot = s;
  return 1;
}

int TimedKernel::commit() {
  if (slot < 0) return ARMI_OK;
  Timing& t = timing();
  std::lock_guard<std::mutex> g(t.mu);
  t.pending[slot].emplace_back(ev[0], ev[1]);
  slot = -1;
  return ARMI_OK;
}

int TimedLaunch::end() {
  if (slot < 0) return ARMI_OK;
  Timing& t = timing();
  std::lock_guard<std::mutex> g(t.mu);
  ARMI_HIP(hipEventRecord(ev[1], stream));
  t.pending[slot].emplace_back(ev[0], ev[1]);
  slot = -1;
  return ARMI_OK;
}

}  // namespace armi

extern "C" {

const char* armi_last_error(void) { return armi::g_last_error.c_str(); }

int armi_abi_version(void) { return ARMI_ABI_VERSION; }

#ifndef ARMI_SOURCE_DIGEST
#define ARMI_SOURCE_DIGEST "unknown"
#endif
const char* armi_source_digest(void) { return ARMI_SOURCE_DIGEST; }

int armi_scan_timing_enable(int enable) {
  armi::Timing& t = armi::timing();
  std::lock_guard<std::mutex> g(t.mu);
  t.enabled = enable > 0;
  t.period = enable > 1 ? enable : 1;
  for (auto& c : t.seen) c = 0;
  return ARMI_OK;
}

int armi_kernel_timing_read(int slot, double* total_ms, int64_t* launches) {
  ARMI_REQUIRE(total_ms && launches, "armi_kernel_timing_read: null pointer argument");
  ARMI_REQUIRE(slot >= 0 && slot < ARMI_TIMING_SLOTS, "armi_kernel_timing_read: bad slot");
  armi::Timing& t = armi::timing();
  std::lock_guard<std::mutex> g(t.mu);
  double sum = 0.0;
  for (auto& ev : t.pending[slot]) {
    ARMI_HIP(hipEventSynchronize(ev.second));
    float ms = 0.f;
    ARMI_HIP(hipEventElapsedTime(&ms, ev.first, ev.second));
    sum += ms;
    t.spare.push_back(ev);
  }
  *total_ms = sum;
  *launches = (int64_t)t.pending[slot].size();
  t.pending[slot].clear();
  return ARMI_OK;
}

int armi_scan_timing_read(double* total_ms, int64_t* launches) {
  return armi_kernel_timing_read(ARMI_TIMING_DENSE_SCAN, total_ms, launches);
}

}  // extern "C"
