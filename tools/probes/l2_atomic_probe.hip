// Split-K partial hand-off options for the stripe wgrad (256 workgroups, each
// holding one 64 x 576 f32 tile of the same weight gradient):
//   store  : each workgroup stores its tile as a bf16 partial (today's scheme)
//   xcd    : f32 no-return atomic adds into its XCD's own accumulator (8 per
//            launch, selected by HW_REG_XCC_ID; workgroup scope = the L2 the
//            XCD owns), the later sum reads 8 tiles instead of 256
//   agent  : f32 atomic adds into one accumulator at agent scope
// Checks the xcd / agent sums against the known total and times each form.
//   hipcc -O3 --offload-arch=gfx950 tools/probes/l2_atomic_probe.hip -o tools/probes/l2_atomic_probe
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

constexpr int TILE = 64 * 576;  // floats per workgroup tile
constexpr int NT = 512;
constexpr int PER = TILE / NT;  // 72 per thread

__device__ __forceinline__ int xcc_id() {
  int v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 7;
}

__device__ __forceinline__ float val(int blk, int i) { return (float)((blk * 7 + i) % 13) * 0.25f; }

__global__ __launch_bounds__(NT) void store_kernel(__hip_bfloat16* part) {
  __hip_bfloat16* dst = part + (long long)blockIdx.x * TILE;
#pragma unroll 8
  for (int j = 0; j < PER; ++j) {
    const int i = j * NT + threadIdx.x;
    dst[i] = __float2bfloat16(val(blockIdx.x, i));
  }
}

__global__ __launch_bounds__(NT) void xcd_kernel(float* acc, int* xcd_of) {
  const int x = xcc_id();
  if (threadIdx.x == 0) xcd_of[blockIdx.x] = x;
  float* dst = acc + (long long)x * TILE;
#pragma unroll 8
  for (int j = 0; j < PER; ++j) {
    const int i = j * NT + threadIdx.x;
    __hip_atomic_fetch_add(dst + i, val(blockIdx.x, i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
}

__global__ __launch_bounds__(NT) void agent_kernel(float* acc) {
#pragma unroll 8
  for (int j = 0; j < PER; ++j) {
    const int i = j * NT + threadIdx.x;
    __hip_atomic_fetch_add(acc + i, val(blockIdx.x, i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <class F>
static float time_us(hipStream_t st, F f) {
  for (int w = 0; w < 3; ++w) f();
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a, st));
  const int it = 20;
  for (int w = 0; w < it; ++w) f();
  CK(hipEventRecord(b, st));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1e3f / it;
}

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  for (int nblk : {256, 512}) {
    __hip_bfloat16* part;
    float* acc;
    int* xcd_of;
    CK(hipMalloc(&part, (size_t)nblk * TILE * 2));
    CK(hipMalloc(&acc, (size_t)8 * TILE * 4));
    CK(hipMalloc(&xcd_of, nblk * 4));
    const float ts = time_us(st, [&] { store_kernel<<<nblk, NT, 0, st>>>(part); });
    const float tx = time_us(st, [&] { xcd_kernel<<<nblk, NT, 0, st>>>(acc, xcd_of); });
    const float ta = time_us(st, [&] { agent_kernel<<<nblk, NT, 0, st>>>(acc); });
    // correctness of one xcd launch and one agent launch
    CK(hipMemsetAsync(acc, 0, (size_t)8 * TILE * 4, st));
    xcd_kernel<<<nblk, NT, 0, st>>>(acc, xcd_of);
    CK(hipStreamSynchronize(st));
    std::vector<float> h((size_t)8 * TILE);
    std::vector<int> xo(nblk);
    CK(hipMemcpy(h.data(), acc, h.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(xo.data(), xcd_of, nblk * 4, hipMemcpyDeviceToHost));
    double maxerr = 0;
    int per[8] = {0};
    for (int b = 0; b < nblk; ++b) per[xo[b]]++;
    for (int i = 0; i < TILE; i += 37) {
      double want = 0, got = 0;
      for (int b = 0; b < nblk; ++b) want += (double)((b * 7 + i) % 13) * 0.25;
      for (int x = 0; x < 8; ++x) got += h[(size_t)x * TILE + i];
      maxerr = fmax(maxerr, fabs(got - want));
    }
    CK(hipMemsetAsync(acc, 0, (size_t)TILE * 4, st));
    agent_kernel<<<nblk, NT, 0, st>>>(acc);
    CK(hipStreamSynchronize(st));
    CK(hipMemcpy(h.data(), acc, (size_t)TILE * 4, hipMemcpyDeviceToHost));
    double maxerr_a = 0;
    for (int i = 0; i < TILE; i += 37) {
      double want = 0;
      for (int b = 0; b < nblk; ++b) want += (double)((b * 7 + i) % 13) * 0.25;
      maxerr_a = fmax(maxerr_a, fabs(h[i] - want));
    }
    printf("%d workgroups x %d-float tile: store bf16 %.2f us (%.1f MB)  xcd atomics %.2f us  agent atomics %.2f us\n",
           nblk, TILE, ts, nblk * TILE * 2 / 1e6, tx, ta);
    printf("   xcd sum max err %.3g (blocks per XCD %d %d %d %d %d %d %d %d), agent sum max err %.3g\n", maxerr,
           per[0], per[1], per[2], per[3], per[4], per[5], per[6], per[7], maxerr_a);
    CK(hipFree(part));
    CK(hipFree(acc));
    CK(hipFree(xcd_of));
  }
  return 0;
}
