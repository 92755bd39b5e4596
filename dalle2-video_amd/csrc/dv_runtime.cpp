// Error plumbing for the C-ABI (no exceptions cross the boundary).
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/dv_hip.h"

namespace dv {
static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g_last_error = std::string(what) + ": " + hipGetErrorString(e);
    return DV_ERR_LAUNCH;
  }
  return DV_OK;
}
}  // namespace dv

extern "C" const char* dv_last_error(void) { return dv::g_last_error.c_str(); }
extern "C" int dv_abi_version(void) { return 1; }
