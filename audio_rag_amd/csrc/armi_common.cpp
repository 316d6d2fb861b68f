// Error plumbing of the C ABI (thread-local last error).
#include <cstdio>
#include <string>

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

}  // namespace armi

extern "C" {

const char* armi_last_error(void) { return armi::g_last_error.c_str(); }

int armi_abi_version(void) { return ARMI_ABI_VERSION; }

}  // extern "C"
