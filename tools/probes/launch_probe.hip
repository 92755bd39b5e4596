// Kernel-boundary cost on MI355X: how long does one graph-replayed launch of
// a near-empty kernel take, and what does a grid-wide barrier inside one
// kernel cost instead?  Decides whether fusing a GroupNorm reduce + apply
// pair into one launch (with a grid barrier) can pay.
//   hipcc -O3 --offload-arch=gfx950 tools/probes/launch_probe.hip -o /tmp/launch_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__global__ void touch_kernel(float* p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] += 1.f;
}

// ticket barrier: the counter only grows (no reset between launches / replays);
// a bounded spin so the grid always drains (a failed barrier sets *err)
__device__ __forceinline__ void grid_barrier(unsigned long long* cnt, int* err) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long n = gridDim.x;
    const unsigned long long old = __hip_atomic_fetch_add(cnt, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long target = (old / n + 1) * n;
    int spins = 0;
    while (__hip_atomic_load(cnt, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1 << 14)) {
        atomicAdd(err, 1);
        break;
      }
    }
  }
  __syncthreads();
}

__global__ void barrier_kernel(float* p, int n, unsigned long long* cnt, int* err, int nbar) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] += 1.f;
  for (int b = 0; b < nbar; ++b) grid_barrier(cnt, err);
  if (i < n) p[i] += 1.f;
}

template <class F>
static float graph_time(hipStream_t st, int reps, F launch_once) {
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
  for (int r = 0; r < reps; ++r) launch_once();
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ge, st));
  CK(hipStreamSynchronize(st));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a, st));
  const int it = 10;
  for (int w = 0; w < it; ++w) CK(hipGraphLaunch(ge, st));
  CK(hipEventRecord(b, st));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  return ms * 1e3f / it / reps;  // us per launch
}

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const int n = 1 << 24;
  float* p;
  unsigned long long* cnt;
  int* err;
  CK(hipMalloc(&p, n * sizeof(float)));
  CK(hipMalloc(&cnt, 8));
  CK(hipMalloc(&err, 4));
  CK(hipMemset(p, 0, n * sizeof(float)));
  CK(hipMemset(cnt, 0, 8));
  CK(hipMemset(err, 0, 4));
  int occ = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, barrier_kernel, 256, 0));
  printf("CUs %d, barrier_kernel resident blocks/CU at 256 threads: %d\n", cus, occ);
  const int reps = 200;
  for (int blocks : {1, 256, 1024, 4096}) {
    const int m = blocks * 256;
    float us = graph_time(st, reps, [&] { touch_kernel<<<blocks, 256, 0, st>>>(p, m); });
    printf("touch  %5d blocks (%8.2f MB rw): %7.2f us/launch\n", blocks, m * 8.0 / 1e6, us);
  }
  for (int blocks : {256, 512, 1024}) {
    if (blocks > occ * cus) continue;
    const int m = blocks * 256;
    for (int nbar : {0, 1, 4}) {
      float us = graph_time(st, 10, [&] { barrier_kernel<<<blocks, 256, 0, st>>>(p, m, cnt, err, nbar); });
      int herr = 0;
      CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
      printf("barrier %4d blocks, %d grid barriers: %7.2f us/launch (timeouts so far %d)\n", blocks, nbar, us, herr);
    }
  }
  int herr = 0;
  CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
  printf("barrier timeouts: %d\n", herr);
  return herr ? 2 : 0;
}
