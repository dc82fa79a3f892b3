// C-ABI plumbing: thread-local error messages and version.
#include "common.h"

namespace samq {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

int check_hip(hipError_t e, const char* what) {
  if (e == hipSuccess) return SAMQ_OK;
  g_last_error = std::string(what) + ": " + hipGetErrorString(e);
  return SAMQ_ERR_HIP;
}

}  // namespace samq

extern "C" const char* samq_last_error(void) { return samq::g_last_error.c_str(); }

extern "C" int samq_version(void) { return 100; }

