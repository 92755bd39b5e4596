// Error plumbing for the C-ABI (no exceptions cross the boundary).
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/dv_hip.h"

namespace dv {
static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

__global__ void zero_f32_kernel(float* p, long long n) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    p[i] = 0.f;
}

void zero_f32(float* p, long long n, hipStream_t st) {
  if (n <= 0) return;
  long long blocks = (n + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  zero_f32_kernel<<<(unsigned)blocks, 256, 0, st>>>(p, n);
}

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
extern "C" int dv_abi_version(void) { return 4; }

extern "C" int dv_zero_f32(float* p, long long n, void* stream) {
  if (!p) {
    dv::set_error("dv_zero_f32: null pointer");
    return DV_ERR_INVALID;
  }
  dv::zero_f32(p, n, (hipStream_t)stream);
  return dv::check_launch("zero_f32");
}
