// Probe of the gfx950 block-scaled MFMA v_mfma_scale_f32_32x32x64_f8f6f4 with
// e4m3 operands, and of v_cvt_pk_fp8_f32.  Exact small-integer data.
//  E1: unscaled product (all scales 2^0) under "lane l = row/col l&31, byte j of
//      lane half h = k 32h + j" for BOTH operands: passes iff A and B use the
//      same k order per (half, byte) (what a kernel needs).
//  E2: which bytes each lane's scale multiplies: A (B) all ones, scale 2^1 on
//      lane 0 and 2^2 on lane 32 (row / column 0), one byte of lane 0 / 32 set
//      to 2: the growth of D[0][0] names the scale that byte is under.
// hipcc --offload-arch=gfx950 -O2 mx8_probe.hip -o mx8_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

__global__ void mma(const unsigned char* A, const unsigned char* B, const int* sa, const int* sb,
                    float* D) {
  const int l = threadIdx.x;
  v8i a, b;
  memcpy(&a, A + 32 * l, 32);
  memcpy(&b, B + 32 * l, 32);
  v16f acc = {};
  acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, acc, 0, 0, 0, sa[l], 0, sb[l]);
  for (int e = 0; e < 16; ++e) D[l * 16 + e] = acc[e];
}

__global__ void cvt(const float* x, unsigned* y, int n) {
  const int i = threadIdx.x;
  if (2 * i + 1 < n) y[i] = __builtin_amdgcn_cvt_pk_fp8_f32(x[2 * i], x[2 * i + 1], 0, false);
}

static float e4m3_to_f(unsigned char v) {
  const int s = v >> 7, e = (v >> 3) & 15, m = v & 7;
  float r;
  if (e == 15 && m == 7) return NAN;
  if (e == 0) r = std::ldexp((float)m, -9);
  else r = std::ldexp(1.0f + m / 8.0f, e - 7);
  return s ? -r : r;
}
static unsigned char f_to_e4m3(float f) {  // exact small values only
  for (int v = 0; v < 256; ++v)
    if (e4m3_to_f((unsigned char)v) == f) return (unsigned char)v;
  return 0x7f;
}

struct Dev {
  unsigned char *A, *B;
  int *sa, *sb;
  float* D;
  Dev() {
    (void)hipMalloc(&A, 2048); (void)hipMalloc(&B, 2048); (void)hipMalloc(&sa, 256);
    (void)hipMalloc(&sb, 256); (void)hipMalloc(&D, 4096);
  }
  std::vector<float> run(const std::vector<unsigned char>& a, const std::vector<unsigned char>& b,
                         const std::vector<int>& s1, const std::vector<int>& s2) {
    (void)hipMemcpy(A, a.data(), 2048, hipMemcpyHostToDevice);
    (void)hipMemcpy(B, b.data(), 2048, hipMemcpyHostToDevice);
    (void)hipMemcpy(sa, s1.data(), 256, hipMemcpyHostToDevice);
    (void)hipMemcpy(sb, s2.data(), 256, hipMemcpyHostToDevice);
    mma<<<1, 64>>>(A, B, sa, sb, D);
    std::vector<float> d(1024);
    (void)hipMemcpy(d.data(), D, 4096, hipMemcpyDeviceToHost);
    return d;
  }
};
// D element (row, col) in the standard 32x32 C/D layout
static float at(const std::vector<float>& d, int row, int col) {
  const int h = (row >> 2) & 1, e = (row & 3) + 4 * (row >> 3);
  return d[(col + 32 * h) * 16 + e];
}

int main() {
  Dev dev;
  // E1
  std::vector<float> Af(32 * 64), Bf(64 * 32);
  for (int r = 0; r < 32; ++r)
    for (int k = 0; k < 64; ++k) Af[r * 64 + k] = (float)(((r * 7 + k * 3) % 9) - 4);
  for (int k = 0; k < 64; ++k)
    for (int c = 0; c < 32; ++c) Bf[k * 32 + c] = (float)(((k * 5 + c * 11 + k * c) % 7) - 3);
  std::vector<unsigned char> A(2048), B(2048);
  std::vector<int> one(64, 127);
  for (int l = 0; l < 64; ++l) {
    const int rc = l & 31, h = l >> 5;
    for (int j = 0; j < 32; ++j) {
      A[32 * l + j] = f_to_e4m3(Af[rc * 64 + 32 * h + j]);
      B[32 * l + j] = f_to_e4m3(Bf[(32 * h + j) * 32 + rc]);
    }
  }
  auto d = dev.run(A, B, one, one);
  int bad = 0;
  for (int r = 0; r < 32; ++r)
    for (int c = 0; c < 32; ++c) {
      double want = 0;
      for (int k = 0; k < 64; ++k) want += (double)Af[r * 64 + k] * Bf[k * 32 + c];
      if (at(d, r, c) != (float)want) {
        if (bad < 4) printf("  E1 D[%d][%d] = %g want %g\n", r, c, at(d, r, c), want);
        ++bad;
      }
    }
  printf("E1 unscaled, same (half, byte) -> k map for A and B: %s (%d bad)\n", bad ? "FAIL" : "PASS", bad);

  // E2
  const unsigned char o = f_to_e4m3(1.0f), t = f_to_e4m3(2.0f);
  for (int which = 0; which < 2; ++which) {  // 0: A operand, 1: B operand
    std::vector<unsigned char> a1(2048, o), b1(2048, o);
    std::vector<int> s1(64, 127), s2(64, 127);
    std::vector<int>& sx = which ? s2 : s1;
    sx[0] = 128;
    sx[32] = 129;
    const float base = at(dev.run(a1, b1, s1, s2), 0, 0);
    printf("E2 %s: base D[0][0] = %g; scale seen by byte j of lane 0 | lane 32:\n   ", which ? "B" : "A", base);
    for (int ln = 0; ln < 64; ln += 32) {
      for (int j = 0; j < 32; ++j) {
        std::vector<unsigned char> a2 = a1, b2 = b1;
        (which ? b2 : a2)[32 * ln + j] = t;
        const float g = at(dev.run(a2, b2, s1, s2), 0, 0) - base;
        printf("%g", g);
      }
      printf(ln == 0 ? " | " : "\n");
    }
  }

  // conversion: exact values, rounding, saturation
  float xs[8] = {1.0f, -2.5f, 448.0f, 500.0f, 1e6f, 0.001953125f, 3.3f, -1000.0f};
  float* dx;
  unsigned* dy;
  (void)hipMalloc(&dx, 32);
  (void)hipMalloc(&dy, 16);
  (void)hipMemcpy(dx, xs, 32, hipMemcpyHostToDevice);
  cvt<<<1, 4>>>(dx, dy, 8);
  unsigned ys[4];
  (void)hipMemcpy(ys, dy, 16, hipMemcpyDeviceToHost);
  for (int i = 0; i < 8; ++i) {
    const unsigned char b = (ys[i / 2] >> (8 * (i % 2))) & 0xff;
    printf("  cvt %g -> 0x%02x = %g\n", xs[i], b, e4m3_to_f(b));
  }
  return 0;
}
