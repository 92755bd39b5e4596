// CLIP-style cross attention of ResnetBlock3D (dalle2_video.py:159-162, 192-201;
// dalle2-pytorch CrossAttention: 8 heads x 64, a learned null k/v prepended to
// the 2 time tokens -> 3 keys per head, logit factor 64^-0.5, gain-only
// LayerNorms before (g1) and after (g2) the block, residual add).
//
// MI355X design.  With only 3 keys per head, the q/out projections fold per
// batch b into two C x 24 matrices (computed once per call, f32):
//   A~[c][hj] = s * sum_d Wq[h*64+d][c] K[b,h,j,d]     scores = LN(x) . A~
//   V~[c][hj] =     sum_d Wo[c][h*64+d] V[b,h,j,d]     o      = V~ p
// Heads are padded to 4 rows (k' = 4h + j, j = 3 dummy) so that in a 32x32
// MFMA accumulator every lane owns whole heads (softmax is lane-local).
// Per wave = 32 tokens of one batch:
//   S^T = Kt . X^T      Kt[k'][c] = g1[c] A~[c][hj]; raw x is the MFMA
//                       operand, LN_in (mean/rstd from the same pass) is
//                       applied algebraically: s = rs*(S^T - mu*colsum(Kt))
//   O^T = Vt . P^T      P^T accumulator reused as the MFMA B operand
//   out = LN_g2(o) + x  (o recomputed per 32-channel tile; 2 passes)
// Backward: dP^T = Vt^T dO^T, dXhat^T = KtT dS^T on MFMA; the LN_in sums are
// analytic (sum dxhat = ds.colsum, sum dxhat*xhat = ds.log p); the token
// reductions dKt, dV~ and dg2 are batched TN GEMMs (dv_gemm_tn_batched).
#include "dv_common.h"

#include <algorithm>
#include <cstdlib>

using namespace dv;

// Diagnostic build only (make stamp): per-workgroup s_memrealtime stamps of
// the cross-attention kernels' phases (tools/xattn_stamp.py)
#ifdef DV_STAMP
constexpr int XA_NSTAMP = 8;
__device__ unsigned long long g_xa_stamp[16384 * XA_NSTAMP];
#define XA_STAMP_AT(i)                                                                         \
  do {                                                                                         \
    if (threadIdx.x == 0 && blockIdx.x < 16384)                                                \
      g_xa_stamp[blockIdx.x * XA_NSTAMP + (i)] = __builtin_amdgcn_s_memrealtime();             \
  } while (0)
extern "C" int dv_debug_stamps_xattn(unsigned long long* host, long long n) {
  if (n > 16384 * XA_NSTAMP) n = 16384 * XA_NSTAMP;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_xa_stamp), n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#else
#define XA_STAMP_AT(i) \
  do {                 \
  } while (0)
#endif

namespace {

constexpr int NH = 8, DH = 64, NK = 3, HK = NH * NK;  // 24 folded columns
constexpr int KP = 32;                                  // padded k' rows

__device__ __forceinline__ int kprime(int hj) { return 4 * (hj / 3) + hj % 3; }
__device__ __forceinline__ int hj_of(int kp) { return (kp & 3) < 3 ? (kp >> 2) * 3 + (kp & 3) : -1; }
__device__ __forceinline__ int acc_row(int e, int h) { return (e & 3) + 8 * (e >> 2) + 4 * h; }

int grid_for(long long work, int per_block = 256, int cap = 16384) {
  long long b = (work + per_block - 1) / per_block;
  if (b > cap) b = cap;
  if (b < 1) b = 1;
  return (int)b;
}

template <typename T> struct Mma;
template <> struct Mma<bf16> {
  __device__ static inline f32x16 run(u32x4 a, u32x4 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                   __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
  }
};
template <> struct Mma<float> {
  __device__ static inline f32x16 run(u32x4 a, u32x4 b, f32x16 c) {
    const f32x4 af = __builtin_bit_cast(f32x4, a), bf = __builtin_bit_cast(f32x4, b);
#pragma unroll
    for (int j = 0; j < 4; ++j) c = __builtin_amdgcn_mfma_f32_32x32x2f32(af[j], bf[j], c, 0, 0, 0);
    return c;
  }
};

// acc(32x32) += A(32 x 32) . X, X an f32 accumulator tile (sum over its rows);
// A row-major in global memory, element (i, k) at A[i*lda + k].
template <typename T> __device__ f32x16 mm_acc_g(const T* A, int lda, const f32x16& X, f32x16 acc, int r, int h);
template <>
__device__ f32x16 mm_acc_g<bf16>(const bf16* A, int lda, const f32x16& X, f32x16 acc, int r, int h) {
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    bf16x8 bx;
#pragma unroll
    for (int j = 0; j < 8; ++j) bx[j] = (bf16)X[8 * s + j];
    const u32x2 lo = *(const u32x2*)(A + (long long)r * lda + 16 * s + 4 * h);
    const u32x2 hi = *(const u32x2*)(A + (long long)r * lda + 16 * s + 8 + 4 * h);
    const u32x4 a = u32x4{lo[0], lo[1], hi[0], hi[1]};
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), bx, acc, 0, 0, 0);
  }
  return acc;
}
// mm_acc_g<bf16> split into its A-fragment loads and the MFMAs, so a kernel
// can issue the loads early and reuse the fragments
__device__ __forceinline__ void ld_afrag(const bf16* A, int lda, int r, int h, u32x4 (&a)[2]) {
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const u32x2 lo = *(const u32x2*)(A + (long long)r * lda + 16 * s + 4 * h);
    const u32x2 hi = *(const u32x2*)(A + (long long)r * lda + 16 * s + 8 + 4 * h);
    a[s] = u32x4{lo[0], lo[1], hi[0], hi[1]};
  }
}
// ld_afrag from an LDS image (row stride lda bf16)
__device__ __forceinline__ void ld_afrag_lds(const bf16* A, int lda, int r, int h, u32x4 (&a)[2]) {
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const u32x2 lo = *(const u32x2*)(A + r * lda + 16 * s + 4 * h);
    const u32x2 hi = *(const u32x2*)(A + r * lda + 16 * s + 8 + 4 * h);
    a[s] = u32x4{lo[0], lo[1], hi[0], hi[1]};
  }
}
__device__ __forceinline__ f32x16 mm_acc_f(const u32x4 (&a)[2], const f32x16& X, f32x16 acc) {
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    bf16x8 bx;
#pragma unroll
    for (int j = 0; j < 8; ++j) bx[j] = (bf16)X[8 * s + j];
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a[s]), bx, acc, 0, 0, 0);
  }
  return acc;
}

template <>
__device__ f32x16 mm_acc_g<float>(const float* A, int lda, const f32x16& X, f32x16 acc, int r, int h) {
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const f32x4 a4 = *(const f32x4*)(A + (long long)r * lda + 8 * m + 4 * h);
#pragma unroll
    for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4[e], X[4 * m + e], acc, 0, 0, 0);
  }
  return acc;
}

template <typename T> __device__ __forceinline__ void ld4(const T* p, float* v);
template <> __device__ __forceinline__ void ld4<float>(const float* p, float* v) {
  const f32x4 t = *(const f32x4*)p;
  v[0] = t[0]; v[1] = t[1]; v[2] = t[2]; v[3] = t[3];
}
template <> __device__ __forceinline__ void ld4<bf16>(const bf16* p, float* v) {
  const bf16x4 t = *(const bf16x4*)p;
  v[0] = (float)t[0]; v[1] = (float)t[1]; v[2] = (float)t[2]; v[3] = (float)t[3];
}
template <typename T> __device__ __forceinline__ void st4(T* p, const float* v);
template <> __device__ __forceinline__ void st4<float>(float* p, const float* v) {
  *(f32x4*)p = f32x4{v[0], v[1], v[2], v[3]};
}
template <> __device__ __forceinline__ void st4<bf16>(bf16* p, const float* v) {
  *(bf16x4*)p = bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
}

// K/V of head h, key j (j = 0: null kv) for batch b
__device__ __forceinline__ float kf(const float* kv, const float* null_kv, int b, int h, int j, int d,
                                    int v) {
  if (j == 0) return null_kv[v * DH + d];
  return kv[((long long)b * 2 + (j - 1)) * (2 * NH * DH) + v * NH * DH + h * DH + d];
}

// ---------------------------------------------------------------------------
// fold: A~, V~ (f32 [nb][C][24]) and the MFMA operand images
// ---------------------------------------------------------------------------
// one workgroup per (head, clip, 64-channel block): the head's 3 keys / values
// (null + 2 time tokens) are staged in LDS; thread (c, dq) sums a quarter of
// the 64 head dims for channel c (Wq columns read coalesced across threads,
// its Wo row segment as 16-B vectors) and the quarters meet in LDS
__device__ __forceinline__ void fold_fwd_body(const float* wq, const float* wo, const float* kv,
                                              const float* null_kv, float* at, float* vt, int C,
                                              float scale, int h, int b, int cz) {
  __shared__ float sk[NK][DH], sv[NK][DH];
  __shared__ float part[4][6][64];
  for (int i = threadIdx.x; i < NK * DH; i += 256) {
    const int j = i / DH, d = i % DH;
    sk[j][d] = kf(kv, null_kv, b, h, j, d, 0);
    sv[j][d] = kf(kv, null_kv, b, h, j, d, 1);
  }
  __syncthreads();
  const int cl = threadIdx.x & 63, dq = threadIdx.x >> 6;
  const int c = cz * 64 + cl;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, v0 = 0.f, v1 = 0.f, v2 = 0.f;
  if (c < C) {
    const float* wor = wo + (long long)c * (NH * DH) + h * DH;
#pragma unroll
    for (int d = 16 * dq; d < 16 * dq + 16; d += 4) {
      const f32x4 w4 = *(const f32x4*)(wor + d);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float q = wq[(long long)(h * DH + d + e) * C + c];
        a0 += q * sk[0][d + e]; a1 += q * sk[1][d + e]; a2 += q * sk[2][d + e];
        v0 += w4[e] * sv[0][d + e]; v1 += w4[e] * sv[1][d + e]; v2 += w4[e] * sv[2][d + e];
      }
    }
  }
  part[dq][0][cl] = a0; part[dq][1][cl] = a1; part[dq][2][cl] = a2;
  part[dq][3][cl] = v0; part[dq][4][cl] = v1; part[dq][5][cl] = v2;
  __syncthreads();
  if (dq == 0 && c < C) {
    float t[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) t[k] = part[0][k][cl] + part[1][k][cl] + part[2][k][cl] + part[3][k][cl];
    const long long o = ((long long)b * C + c) * HK + h * NK;
    at[o] = t[0] * scale; at[o + 1] = t[1] * scale; at[o + 2] = t[2] * scale;
    vt[o] = t[3]; vt[o + 1] = t[4]; vt[o + 2] = t[5];
  }
}

__global__ __launch_bounds__(256) void fold_fwd_kernel(const float* wq, const float* wo,
                                                       const float* kv, const float* null_kv,
                                                       float* at, float* vt, int nb, int C,
                                                       float scale) {
  fold_fwd_body(wq, wo, kv, null_kv, at, vt, C, scale, blockIdx.x, blockIdx.y, blockIdx.z);
}

// Kt[b][k'][c], KtT[b][c][k'], Vt[b][c][k'], VtT[b][k'][c] (T); dummies zero
// images are padded to Cp = roundup(C, 32) channels with zeros
template <typename T>
__device__ __forceinline__ void fold_pack_body(const float* at, const float* vt, const float* g1,
                                               T* Kt, T* KtT, T* Vt, T* VtT, int nb, int C,
                                               int Cp) {
  const long long n = (long long)nb * KP * Cp;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % Cp);
    const long long bk = i / Cp;
    const int kp = (int)(bk % KP), b = (int)(bk / KP);
    const int hj = c < C ? hj_of(kp) : -1;
    const float a = hj >= 0 ? g1[c] * at[((long long)b * C + c) * HK + hj] : 0.f;
    const float v = hj >= 0 ? vt[((long long)b * C + c) * HK + hj] : 0.f;
    Kt[i] = (T)a;
    VtT[i] = (T)v;
    KtT[((long long)b * Cp + c) * KP + kp] = (T)a;
    Vt[((long long)b * Cp + c) * KP + kp] = (T)v;
  }
}

template <typename T>
__global__ void fold_pack_kernel(const float* at, const float* vt, const float* g1, T* Kt, T* KtT,
                                 T* Vt, T* VtT, int nb, int C, int Cp) {
  fold_pack_body<T>(at, vt, g1, Kt, KtT, Vt, VtT, nb, C, Cp);
}

// colsum[b][k'] = sum_c Kt[b][k'][c] (of the values the MFMA sees)
template <typename T>
__global__ void fold_colsum_kernel(const T* Kt, float* colsum, int nb, int Cp) {
  const int row = blockIdx.x;  // b*KP + k'
  float s = 0.f;
  for (int c = threadIdx.x; c < Cp; c += 64) s += (float)Kt[(long long)row * Cp + c];
  s = wave_sum(s);
  if (threadIdx.x == 0) colsum[row] = s;
}

// Every cross-attention block's fold in three launches (the folds depend on
// weights and the context only, so Unet3D runs them all up front): the job
// table rides in the kernel arguments (graph-safe, no host-to-device copy).
struct FoldBatch {
  DvFoldJob j[DV_FOLD_MAX];
  int n;
  float scale;
};

__global__ __launch_bounds__(256) void fold_fwd_batched_kernel(FoldBatch t) {
  const DvFoldJob& J = t.j[blockIdx.z / 8];
  const int cz = blockIdx.z % 8;
  if ((int)blockIdx.y >= J.nb || cz * 64 >= J.C) return;
  fold_fwd_body(J.wq, J.wo, J.kv, J.null_kv, J.at, J.vt, J.C, t.scale, blockIdx.x, blockIdx.y, cz);
}

template <typename T>
__global__ void fold_pack_batched_kernel(FoldBatch t) {
  const DvFoldJob& J = t.j[blockIdx.y];
  fold_pack_body<T>(J.at, J.vt, J.g1, (T*)J.Kt, (T*)J.KtT, (T*)J.Vt, (T*)J.VtT, J.nb, J.C,
                    (J.C + 31) / 32 * 32);
}

template <typename T>
__global__ void fold_colsum_batched_kernel(FoldBatch t) {
  const DvFoldJob& J = t.j[blockIdx.y];
  const int row = blockIdx.x, Cp = (J.C + 31) / 32 * 32;
  if (row >= J.nb * KP) return;
  const T* Kt = (const T*)J.Kt;
  float s = 0.f;
  for (int c = threadIdx.x; c < Cp; c += 64) s += (float)Kt[(long long)row * Cp + c];
  s = wave_sum(s);
  if (threadIdx.x == 0) J.colsum[row] = s;
}

// ---------------------------------------------------------------------------
// forward: one wave = 32 tokens (of one batch element)
// ---------------------------------------------------------------------------

// Channel-split mode (CS = 4): the 4 waves of a workgroup share ONE 32-token
// tile and take every 4th 32-channel tile each, meeting in LDS for the
// per-token reductions (scores / dP accumulators, LayerNorm sums).  Used when
// the token count is too small to give every CU a tile of its own (the 8x8
// and 16x16 stages): 4x the workgroups, 1/4 of each wave's serial chain.
constexpr int XRS = 18;  // reduction slots per lane
template <int CS>
__device__ __forceinline__ void xwave_sum(float* v, int n, float* sh, int cw, int lane) {
  if (CS == 1) return;
  __syncthreads();  // the previous use of sh is complete
  for (int i = 0; i < n; ++i) sh[(cw * XRS + i) * 64 + lane] = v[i];
  __syncthreads();
  for (int i = 0; i < n; ++i) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < CS; ++w) t += sh[(w * XRS + i) * 64 + lane];
    v[i] = t;
  }
}

template <typename T, int CS, int NCT>
__global__ __launch_bounds__(CS == 8 ? 512 : 256) void xattn_fwd_kernel(const T* x, int ldx, T* out, int ldo,
                                                        long long ntok, long long P, int C,
                                                        const T* Kt, const T* Vt,
                                                        const float* colsum, const float* g2,
                                                        float eps, float* stats, T* pbuf) {
  constexpr int VEC = 16 / sizeof(T);
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  // waves tile each batch element's P tokens; lanes past P mirror token P-1
  // (their MFMA columns are independent) and store nothing
  __shared__ float xred[CS == 1 ? 1 : CS * XRS * 64];
  // LN_out gain staged in LDS: a global load between the output stores would
  // wait for every earlier store (vmcnt retires in order); LDS reads do not
  __shared__ float g2s[256 * CS];  // C <= 32 * 8 * CS (host-checked)
  for (int i = threadIdx.x; i < C; i += 64 * (CS == 8 ? 8 : 4)) g2s[i] = g2[i];
  __syncthreads();
  const int cw = CS == 1 ? 0 : (threadIdx.x >> 6);  // channel group of this wave
  const long long wpb = (P + 31) / 32;
  const long long wv = CS == 1 ? (long long)blockIdx.x * 4 + (threadIdx.x >> 6) : (long long)blockIdx.x;
  if (wv >= (ntok / P) * wpb) return;  // uniform per workgroup when CS > 1
  const int b = (int)(wv / wpb);
  const long long tin = (wv % wpb) * 32 + r;
  const bool valid = tin < P;
  const bool lead = cw == 0;  // stores the per-token outputs shared by the channel groups
  const long long tok = (long long)b * P + (valid ? tin : P - 1);
  XA_STAMP_AT(0);
  // the colsum terms of the softmax, loaded with the first batch (before any store)
  float csr[4][3];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int j = 0; j < 3; ++j) csr[m][j] = colsum[b * KP + 8 * m + 4 * h + j];
  const T* xr = x + tok * ldx;
  const int Cp = (C + 31) / 32 * 32;
  const T* Ktb = Kt + (long long)b * KP * Cp;
  const T* Vtb = Vt + (long long)b * Cp * KP;
  // exact-trip bf16 path: the residual's x values (pass-3 layout) are loaded
  // up front with the pass-1 reads of the same lines (no second round trip)
  constexpr bool CACHE = NCT > 0 && NCT <= 4 && sizeof(T) == 2;
  u32x2 xres[CACHE ? NCT : 1][4];
  u32x4 vfr[CACHE ? NCT : 1][2];  // V~ fragments of passes 2 and 3
  if constexpr (CACHE) {
#pragma unroll
    for (int it = 0; it < NCT; ++it) {
#pragma unroll
      for (int g = 0; g < 4; ++g) xres[it][g] = *(const u32x2*)(xr + 32 * cw + it * 32 * CS + 8 * g + 4 * h);
      ld_afrag((const bf16*)(Vtb + (long long)(32 * cw + it * 32 * CS) * KP), KP, r, h, vfr[it]);
    }
  }
  // ---- scores: S^T = Kt . X^T over raw x, LN stats in the same pass ----
  f32x16 acc;
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] = 0.f;
  float sx = 0.f, sxx = 0.f;
  // channel loops: NCT > 0 = exactly NCT 32-channel tiles per wave and
  // C % 32 == 0 (checked on the host): straight-line unrolled code, so every
  // tile's loads can issue up front; NCT == 0: bounded loop with exits
  constexpr int NIT = NCT > 0 ? NCT : 8;
#pragma unroll
  for (int it = 0; it < NIT * 32 / (2 * VEC); ++it) {
    const int c0 = 2 * VEC * cw + it * 2 * VEC * CS;
    if (NCT == 0 && c0 >= Cp) break;
    const int c = c0 + h * VEC;
    const u32x4 xv = (NCT > 0 || c < C) ? *(const u32x4*)(xr + c) : u32x4{0u, 0u, 0u, 0u};
    const u32x4 kv = *(const u32x4*)(Ktb + (long long)r * Cp + c);
    float f[VEC];
    Vec<T>::to_f(xv, f);
#pragma unroll
    for (int e = 0; e < VEC; ++e) { sx += f[e]; sxx += f[e] * f[e]; }
    acc = Mma<T>::run(kv, xv, acc);
  }
  XA_STAMP_AT(1);
  if (CS > 1) {
    float v[XRS];
#pragma unroll
    for (int e = 0; e < 16; ++e) v[e] = acc[e];
    v[16] = sx;
    v[17] = sxx;
    xwave_sum<CS>(v, XRS, xred, cw, lane);
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = v[e];
    sx = v[16];
    sxx = v[17];
  }
  XA_STAMP_AT(2);
  sx += __shfl_xor(sx, 32, 64);
  sxx += __shfl_xor(sxx, 32, 64);
  const float mu = sx / C;
  const float rs = rsqrtf(fmaxf(sxx / C - mu * mu, 0.f) + eps);
  // ---- lane-local softmax over each head's 3 keys ----
  f32x16 p;
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    float s3[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      s3[j] = rs * (acc[4 * m + j] - mu * csr[m][j]);
    }
    const float mx = fmaxf(s3[0], fmaxf(s3[1], s3[2]));
    const float e0 = __expf(s3[0] - mx), e1 = __expf(s3[1] - mx), e2 = __expf(s3[2] - mx);
    const float inv = 1.f / (e0 + e1 + e2);
    float pv[4] = {e0 * inv, e1 * inv, e2 * inv, 0.f};
    // P as stored (T-rounded) is what both O and the backward use
    T pt[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) { pt[j] = (T)pv[j]; p[4 * m + j] = (float)pt[j]; }
    float pw[4] = {(float)pt[0], (float)pt[1], (float)pt[2], (float)pt[3]};
    if (valid && lead) st4<T>(pbuf + tok * KP + 8 * m + 4 * h, pw);
  }
  XA_STAMP_AT(3);
  // ---- o statistics (pass 1), then the normalised output + residual (pass 2) ----
  float so = 0.f, soo = 0.f;
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int ct = 32 * cw + it * 32 * CS;
    if (NCT == 0 && ct >= Cp) break;
    f32x16 o;
#pragma unroll
    for (int e = 0; e < 16; ++e) o[e] = 0.f;
    if constexpr (CACHE) o = mm_acc_f(vfr[it], p, o);
    else o = mm_acc_g<T>(Vtb + (long long)ct * KP, KP, p, o, r, h);
#pragma unroll
    for (int e = 0; e < 16; ++e) { so += o[e]; soo += o[e] * o[e]; }
  }
  if (CS > 1) {
    float v[2] = {so, soo};
    xwave_sum<CS>(v, 2, xred, cw, lane);
    so = v[0];
    soo = v[1];
  }
  XA_STAMP_AT(4);
  so += __shfl_xor(so, 32, 64);
  soo += __shfl_xor(soo, 32, 64);
  const float mu2 = so / C;
  const float rs2 = rsqrtf(fmaxf(soo / C - mu2 * mu2, 0.f) + eps);
  T* orow = out + tok * ldo;
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int ct = 32 * cw + it * 32 * CS;
    if (NCT == 0 && ct >= Cp) break;
    f32x16 o;
#pragma unroll
    for (int e = 0; e < 16; ++e) o[e] = 0.f;
    if constexpr (CACHE) o = mm_acc_f(vfr[it], p, o);
    else o = mm_acc_g<T>(Vtb + (long long)ct * KP, KP, p, o, r, h);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int c = ct + 8 * g + 4 * h;
      if (NCT == 0 && c >= C) continue;
      float xv[4], y[4];
      if constexpr (CACHE) {
        const bf16x4 t = __builtin_bit_cast(bf16x4, xres[it][g]);
        xv[0] = (float)t[0]; xv[1] = (float)t[1]; xv[2] = (float)t[2]; xv[3] = (float)t[3];
      } else {
        ld4<T>(xr + c, xv);
      }
      const f32x4 gg = *(const f32x4*)(g2s + c);
#pragma unroll
      for (int e = 0; e < 4; ++e) y[e] = (o[4 * g + e] - mu2) * rs2 * gg[e] + xv[e];
      if (valid) st4<T>(orow + c, y);
    }
  }
  if (h == 0 && valid && lead) *(f32x4*)(stats + tok * 4) = f32x4{mu, rs, mu2, rs2};
  XA_STAMP_AT(5);
#ifdef DV_STAMP
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  XA_STAMP_AT(6);
#endif
}

// ---------------------------------------------------------------------------
// backward: one wave = 32 tokens
//   writes dx (incl. residual), dO (tokens x C), dS' = rs*dS and
//   P' = rs2*P (k'=3 -> mu2*rs2) (tokens x 32) for the batched GEMMs, and
//   (the LN mean correction sum_t mu_t*rs_t*dS_tk' is NOT accumulated here:
//    it equals (1/C) sum_c R[b][k'][c], the row sums of the R = dS'^T X GEMM)
// ---------------------------------------------------------------------------
template <typename T, int CS, int NCT>
__global__ __launch_bounds__(CS == 8 ? 512 : 256, CS == 8 ? 1 : 2) void xattn_bwd_kernel(const T* dy, int lddy, const T* x, int ldx,
                                                        T* dx, int lddx, long long ntok,
                                                        long long P, int C, const T* KtT,
                                                        const T* Vt, const T* VtT,
                                                        const float* colsum, const float* g2,
                                                        const float* stats, const T* pbuf,
                                                        T* dobuf, T* dsbuf, T* p2buf) {
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  // waves tile each batch element's P tokens; lanes past P mirror token P-1
  // (their MFMA columns are independent) and store nothing
  __shared__ float xred[CS == 1 ? 1 : CS * XRS * 64];
  __shared__ float g2s[256 * CS];  // LN_out gain in LDS (see the forward)
  constexpr int NTH = 64 * (CS == 8 ? 8 : 4);
  for (int i = threadIdx.x; i < C; i += NTH) g2s[i] = g2[i];
  const long long wpb = (P + 31) / 32;
  // workgroups never straddle two clips: CS = 1 takes 4 consecutive tiles of
  // one clip (bpc workgroups per clip), CS > 1 one tile
  const long long bpc = CS == 1 ? (wpb + 3) / 4 : wpb;
  const int b = (int)(blockIdx.x / bpc);
  const long long tic = CS == 1 ? (blockIdx.x % bpc) * 4 + (threadIdx.x >> 6) : blockIdx.x % bpc;
  const bool clip_ok = b < ntok / P;
  // exact-trip bf16: the clip's Vt^T (KP x Cp) and Kt^T (Cp x KP) operand
  // images and its colsum staged in LDS once per workgroup (rows padded
  // against bank conflicts)
  constexpr bool STAGE = NCT > 0 && NCT <= 4 && sizeof(T) == 2;  // the CACHE path below
  constexpr int CPS = 32 * (NCT > 0 ? NCT : 1) * CS;  // Cp of the exact path
  constexpr int SV_LD = CPS + 8, SK_LD = KP + 8;      // bf16 row strides
  __shared__ __attribute__((aligned(16))) bf16 sfr[STAGE ? KP * SV_LD + CPS * SK_LD : 8];
  __shared__ float scs[KP];
  bf16* const sVtT = sfr;
  bf16* const sKtT = sfr + KP * SV_LD;
  if (clip_ok) {
    if (threadIdx.x < KP) scs[threadIdx.x] = colsum[b * KP + threadIdx.x];
    if constexpr (STAGE) {
      const bf16* gv = (const bf16*)VtT + (long long)b * KP * CPS;
      const bf16* gk = (const bf16*)KtT + (long long)b * CPS * KP;
      for (int i = threadIdx.x; i < KP * CPS / 8; i += NTH) {  // 16-B pieces
        const int row = i / (CPS / 8), col = (i % (CPS / 8)) * 8;
        *(u32x4*)(sVtT + row * SV_LD + col) = *(const u32x4*)(gv + (long long)row * CPS + col);
      }
      for (int i = threadIdx.x; i < CPS * KP / 8; i += NTH) {
        const int row = i / (KP / 8), col = (i % (KP / 8)) * 8;
        *(u32x4*)(sKtT + row * SK_LD + col) = *(const u32x4*)(gk + (long long)row * KP + col);
      }
    }
  }
  __syncthreads();
  const int cw = CS == 1 ? 0 : (threadIdx.x >> 6);  // channel group of this wave
  if (!clip_ok || tic >= wpb) return;  // uniform per wave (per workgroup when CS > 1)
  const long long tin = tic * 32 + r;
  const bool valid = tin < P;
  const bool lead = cw == 0;
  const long long tok = (long long)b * P + (valid ? tin : P - 1);
  XA_STAMP_AT(0);
  const T* xr = x + tok * ldx;
  const T* dyr = dy + tok * lddy;
  const int Cp = (C + 31) / 32 * 32;
  const T* Vtb = Vt + (long long)b * Cp * KP;
  const T* VtTb = VtT + (long long)b * KP * Cp;
  const T* KtTb = KtT + (long long)b * Cp * KP;
  constexpr int NIT = NCT > 0 ? NCT : 8;
  // exact-trip bf16 path: this lane's dy and x channels (16 per tile) are
  // loaded once, up front, and serve all three passes (one global round trip
  // instead of one per pass)
  constexpr bool CACHE = NCT > 0 && NCT <= 4 && sizeof(T) == 2;
  u32x2 dyc[CACHE ? NCT : 1][4], xcc[CACHE ? NCT : 1][4];
  u32x4 vfr[CACHE ? NCT : 1][2];  // V~ fragments of passes A and B
  if constexpr (CACHE) {
#pragma unroll
    for (int it = 0; it < NCT; ++it) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c = 32 * cw + it * 32 * CS + 8 * g + 4 * h;
        dyc[it][g] = *(const u32x2*)(dyr + c);
        xcc[it][g] = *(const u32x2*)(xr + c);
      }
      ld_afrag((const bf16*)(Vtb + (long long)(32 * cw + it * 32 * CS) * KP), KP, r, h, vfr[it]);
    }
  }
  auto unpack4 = [](u32x2 q, float* v) {
    const bf16x4 t = __builtin_bit_cast(bf16x4, q);
    v[0] = (float)t[0]; v[1] = (float)t[1]; v[2] = (float)t[2]; v[3] = (float)t[3];
  };
  auto ld_dy = [&](int it, int g, int c, float* v) {
    if constexpr (CACHE) unpack4(dyc[it][g], v);
    else ld4<T>(dyr + c, v);
  };
  auto ld_x = [&](int it, int g, int c, float* v) {
    if constexpr (CACHE) unpack4(xcc[it][g], v);
    else ld4<T>(xr + c, v);
  };
  const f32x4 st = *(const f32x4*)(stats + tok * 4);
  const float mu = st[0], rs = st[1], mu2 = st[2], rs2 = st[3];
  f32x16 p;
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    float v[4];
    ld4<T>(pbuf + tok * KP + 8 * m + 4 * h, v);
#pragma unroll
    for (int j = 0; j < 4; ++j) p[4 * m + j] = v[j];
  }
  // ---- pass A: LN_out backward statistics ----
  float m1 = 0.f, m2 = 0.f;
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int ct = 32 * cw + it * 32 * CS;
    if (NCT == 0 && ct >= Cp) break;
    f32x16 o;
#pragma unroll
    for (int e = 0; e < 16; ++e) o[e] = 0.f;
    if constexpr (CACHE) o = mm_acc_f(vfr[it], p, o);
    else o = mm_acc_g<T>(Vtb + (long long)ct * KP, KP, p, o, r, h);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int c = ct + 8 * g + 4 * h;
      if (NCT == 0 && c >= C) continue;
      float dv[4];
      ld_dy(it, g, c, dv);
      const f32x4 gg = *(const f32x4*)(g2s + c);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float doh = dv[e] * gg[e];
        m1 += doh;
        m2 += doh * (o[4 * g + e] - mu2) * rs2;
      }
    }
  }
  if (CS > 1) {
    float v[2] = {m1, m2};
    xwave_sum<CS>(v, 2, xred, cw, lane);
    m1 = v[0];
    m2 = v[1];
  }
  m1 = (m1 + __shfl_xor(m1, 32, 64)) / C;
  m2 = (m2 + __shfl_xor(m2, 32, 64)) / C;
  XA_STAMP_AT(1);
  // ---- pass B: dO (stored) and dP^T = Vt^T . dO^T ----
  // (staged: the Vt^T fragments come from LDS -- a global load behind the dO
  // stores would wait for them, vmcnt retiring in order)
  f32x16 dp;
#pragma unroll
  for (int e = 0; e < 16; ++e) dp[e] = 0.f;
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int ct = 32 * cw + it * 32 * CS;
    if (NCT == 0 && ct >= Cp) break;
    f32x16 o;
#pragma unroll
    for (int e = 0; e < 16; ++e) o[e] = 0.f;
    if constexpr (CACHE) o = mm_acc_f(vfr[it], p, o);
    else o = mm_acc_g<T>(Vtb + (long long)ct * KP, KP, p, o, r, h);
    f32x16 dO;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int c = ct + 8 * g + 4 * h;
      if (NCT == 0 && c >= C) {
#pragma unroll
        for (int e = 0; e < 4; ++e) dO[4 * g + e] = 0.f;
        continue;
      }
      float dv[4], w[4];
      ld_dy(it, g, c, dv);
      const f32x4 gg = *(const f32x4*)(g2s + c);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float oh = (o[4 * g + e] - mu2) * rs2;
        const T q = (T)(rs2 * (dv[e] * gg[e] - m1 - oh * m2));
        w[e] = (float)q;
        dO[4 * g + e] = w[e];
      }
      if (valid) st4<T>(dobuf + tok * C + c, w);
    }
    if constexpr (STAGE) {
      u32x4 a[2];
      ld_afrag_lds(sVtT + ct, SV_LD, r, h, a);
      dp = mm_acc_f(a, dO, dp);
    } else {
      dp = mm_acc_g<T>(VtTb + ct, Cp, dO, dp, r, h);
    }
  }
  if (CS > 1) {
    float v[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) v[e] = dp[e];
    xwave_sum<CS>(v, 16, xred, cw, lane);
#pragma unroll
    for (int e = 0; e < 16; ++e) dp[e] = v[e];
  }
  XA_STAMP_AT(2);
  // ---- softmax backward (lane-local heads) ----
  f32x16 ds;
  float a1 = 0.f, a2 = 0.f;
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const float sd = p[4 * m] * dp[4 * m] + p[4 * m + 1] * dp[4 * m + 1] + p[4 * m + 2] * dp[4 * m + 2];
    float w[4], q[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int kp = 8 * m + 4 * h + j;
      const float d = j < 3 ? p[4 * m + j] * (dp[4 * m + j] - sd) : 0.f;
      ds[4 * m + j] = d;
      a1 += d * scs[kp];  // d = 0 at j = 3
      if (j < 3 && p[4 * m + j] > 0.f) a2 += d * __logf(p[4 * m + j]);
      w[j] = rs * d;
      q[j] = j < 3 ? rs2 * p[4 * m + j] : (kp == 3 ? mu2 * rs2 : 0.f);
    }
    if (valid && lead) st4<T>(dsbuf + tok * KP + 8 * m + 4 * h, w);
    if (valid && lead) st4<T>(p2buf + tok * KP + 8 * m + 4 * h, q);
  }
  a1 = (a1 + __shfl_xor(a1, 32, 64)) / C;  // mean_c dxhat
  a2 = (a2 + __shfl_xor(a2, 32, 64)) / C;  // mean_c dxhat*xhat
  XA_STAMP_AT(3);
  // ---- pass C: dXhat^T = KtT . dS^T, LN_in backward + residual ----
  T* dxr = dx + tok * lddx;
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int ct = 32 * cw + it * 32 * CS;
    if (NCT == 0 && ct >= Cp) break;
    f32x16 dxh;
#pragma unroll
    for (int e = 0; e < 16; ++e) dxh[e] = 0.f;
    if constexpr (STAGE) {
      u32x4 a[2];
      ld_afrag_lds(sKtT + ct * SK_LD, SK_LD, r, h, a);
      dxh = mm_acc_f(a, ds, dxh);
    } else {
      dxh = mm_acc_g<T>(KtTb + (long long)ct * KP, KP, ds, dxh, r, h);
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int c = ct + 8 * g + 4 * h;
      if (NCT == 0 && c >= C) continue;
      float xv[4], dv[4], w[4];
      ld_x(it, g, c, xv);
      ld_dy(it, g, c, dv);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float xh = (xv[e] - mu) * rs;
        w[e] = rs * (dxh[4 * g + e] - a1 - xh * a2) + dv[e];
      }
      if (valid) st4<T>(dxr + c, w);
    }
  }
  XA_STAMP_AT(4);
#ifdef DV_STAMP
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  XA_STAMP_AT(5);
#endif
}

// mcorr[b][k'] = (1/C) sum_c R[b][k'][c]  (= sum_t mu_t * dS'_tk', mu_t the
// channel mean of token t); one block per (b, k'), R rows read coalesced
__global__ __launch_bounds__(256) void fold_mcorr_kernel(const float* wsR, float* mcorr, int C) {
  __shared__ float red[4];
  const int row = blockIdx.x;  // b*KP + k'
  float s = 0.f;
  for (int c = threadIdx.x; c < C; c += 256) s += wsR[(long long)row * C + c];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) mcorr[row] = (red[0] + red[1] + red[2] + red[3]) / C;
}

// dat/dvt [nb][C][24] from the GEMM results (ws_* [nb][32][C]) and the LN gain
// grads.  grid (ceil(C/64), nb), 256 threads = 64 channels x 4 groups of 6
// folded columns; dg1/dg2 (pre-zeroed unless accumulating) take one atomic
// per (b, c).
__device__ __forceinline__ void fold_grad_finish_body(
    float* wsR, float* wsV, float* wsQ, const float* mcorr, const float* at,
    const float* vt, const float* g1, float* dat, float* dvt, float* dg1, float* dg2, int C,
    int bx, int b) {
  __shared__ float red[2][4][64];
  const int cl = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int c = bx * 64 + cl;
  float s1 = 0.f, s2 = 0.f;
  if (c < C) {
    const float g = g1[c];
#pragma unroll
    for (int q = 0; q < HK / 4; ++q) {
      const int hj = grp * (HK / 4) + q;
      const int kp = kprime(hj);
      const long long wi = ((long long)b * KP + kp) * C + c;
      const long long fi = ((long long)b * C + c) * HK + hj;
      const float dk = wsR[wi] - mcorr[b * KP + kp];
      dat[fi] = g * dk;
      s1 += at[fi] * dk;
      dvt[fi] = wsV[wi];
      s2 += vt[fi] * wsQ[wi];
    }
    if (grp == 0) s2 -= wsQ[((long long)b * KP + 3) * C + c];
  }
  red[0][grp][cl] = s1;
  red[1][grp][cl] = s2;
  __syncthreads();
  if (c < C) {  // consumed: leave the GEMM accumulators zeroed for the next call
    float *wr = wsR, *wv = wsV, *wq2 = wsQ;
#pragma unroll
    for (int q = 0; q < KP / 4; ++q) {
      const long long wi = ((long long)b * KP + grp * (KP / 4) + q) * C + c;
      wr[wi] = 0.f;
      wv[wi] = 0.f;
      wq2[wi] = 0.f;
    }
  }
  if (grp == 0 && c < C) {
    const float t1 = red[0][0][cl] + red[0][1][cl] + red[0][2][cl] + red[0][3][cl];
    const float t2 = red[1][0][cl] + red[1][1][cl] + red[1][2][cl] + red[1][3][cl];
    if (dg1) atomicAdd(dg1 + c, t1);
    if (dg2) atomicAdd(dg2 + c, t2);
  }
}

__global__ __launch_bounds__(256) void fold_grad_finish_kernel(
    float* wsR, float* wsV, float* wsQ, const float* mcorr, const float* at,
    const float* vt, const float* g1, float* dat, float* dvt, float* dg1, float* dg2, int nb,
    int C) {
  fold_grad_finish_body(wsR, wsV, wsQ, mcorr, at, vt, g1, dat, dvt, dg1, dg2, C, blockIdx.x,
                        blockIdx.y);
}

// parameter grads of the fold: dWq, dWo
__device__ __forceinline__ void fold_bwd_w_body(const float* dat, const float* dvt, const float* kv,
                                               const float* null_kv, float* dwq, float* dwo, int nb,
                                               int C, float scale, int accumulate) {
  const long long n = (long long)NH * DH * C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    {  // dWq[hd][c]   (i = hd*C + c)
      const int c = (int)(i % C), hd = (int)(i / C);
      const int h = hd / DH, d = hd % DH;
      float s = 0.f;
      for (int b = 0; b < nb; ++b)
        for (int j = 0; j < NK; ++j)
          s += dat[((long long)b * C + c) * HK + h * NK + j] * kf(kv, null_kv, b, h, j, d, 0);
      dwq[i] = accumulate ? dwq[i] + s * scale : s * scale;
    }
    {  // dWo[c][hd]   (i = c*512 + hd)
      const int hd = (int)(i % (NH * DH)), c = (int)(i / (NH * DH));
      const int h = hd / DH, d = hd % DH;
      float s = 0.f;
      for (int b = 0; b < nb; ++b)
        for (int j = 0; j < NK; ++j)
          s += dvt[((long long)b * C + c) * HK + h * NK + j] * kf(kv, null_kv, b, h, j, d, 1);
      dwo[i] = accumulate ? dwo[i] + s : s;
    }
  }
}

__global__ void fold_bwd_w_kernel(const float* dat, const float* dvt, const float* kv,
                                  const float* null_kv, float* dwq, float* dwo, int nb, int C,
                                  float scale, int accumulate) {
  fold_bwd_w_body(dat, dvt, kv, null_kv, dwq, dwo, nb, C, scale, accumulate);
}

// dK/dV of (b, h, all 3 keys) -> d(kv) (j >= 1) or dnull (j == 0).
// grid (NH, nb, 2): z = 0 computes dK = scale * dat[:, hj]^T Wq_h^T (wave w owns
// 16 head dims, lanes sweep c, wave reductions); z = 1 computes
// dV = dvt[:, hj]^T Wo_h (lane = head dim, coalesced Wo rows, waves split c).
__device__ __forceinline__ void fold_bwd_kv_body(const float* dat, const float* dvt,
                                                 const float* wq, const float* wo, float* dkv,
                                                 float* dnull, int C, float scale, int h, int b,
                                                 int part) {
  __shared__ float red[4][NK][DH];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float* datb = dat + (long long)b * C * HK + h * NK;
  const float* dvtb = dvt + (long long)b * C * HK + h * NK;
  auto emit = [&](int j, int d, float v) {
    if (j == 0) atomicAdd(dnull + part * DH + d, v);
    else dkv[((long long)b * 2 + (j - 1)) * (2 * NH * DH) + part * NH * DH + h * DH + d] = v;
  };
  if (part == 0) {
    // stage dat[b][:, h*3 .. h*3+2] once (C x 3 floats); thread (j, d) owns one
    // output and sweeps its Wq row as 16-B vectors (no cross-lane reductions)
    extern __shared__ float dsh[];  // 3*C floats
    for (int c = threadIdx.x; c < C; c += 256) {
      const float* dr = datb + (long long)c * HK;
      dsh[3 * c] = dr[0];
      dsh[3 * c + 1] = dr[1];
      dsh[3 * c + 2] = dr[2];
    }
    __syncthreads();
    const int d = lane, j = w;
    if (j < NK) {
      const float* wr = wq + (long long)(h * DH + d) * C;
      float s0 = 0.f, s1 = 0.f;
      int c = 0;
      for (; c + 8 <= C; c += 8) {
        const f32x4 u = *(const f32x4*)(wr + c), v = *(const f32x4*)(wr + c + 4);
        s0 += u[0] * dsh[3 * c + j] + u[1] * dsh[3 * (c + 1) + j] + u[2] * dsh[3 * (c + 2) + j] +
              u[3] * dsh[3 * (c + 3) + j];
        s1 += v[0] * dsh[3 * (c + 4) + j] + v[1] * dsh[3 * (c + 5) + j] + v[2] * dsh[3 * (c + 6) + j] +
              v[3] * dsh[3 * (c + 7) + j];
      }
      for (; c < C; ++c) s0 += wr[c] * dsh[3 * c + j];
      emit(j, d, (s0 + s1) * scale);
    }
  } else {
    float s0 = 0.f, s1 = 0.f, s2 = 0.f;
#pragma unroll 4
    for (int c = w; c < C; c += 4) {
      const float wv = wo[(long long)c * (NH * DH) + h * DH + lane];
      const float* dr = dvtb + (long long)c * HK;
      s0 += dr[0] * wv;
      s1 += dr[1] * wv;
      s2 += dr[2] * wv;
    }
    red[w][0][lane] = s0;
    red[w][1][lane] = s1;
    red[w][2][lane] = s2;
    __syncthreads();
    if (w < NK) emit(w, lane, red[0][w][lane] + red[1][w][lane] + red[2][w][lane] + red[3][w][lane]);
  }
}

__global__ __launch_bounds__(256) void fold_bwd_kv_kernel(const float* dat, const float* dvt,
                                                          const float* wq, const float* wo,
                                                          float* dkv, float* dnull, int C,
                                                          float scale) {
  fold_bwd_kv_body(dat, dvt, wq, wo, dkv, dnull, C, scale, blockIdx.x, blockIdx.y, blockIdx.z);
}

template <typename T>
int fold_t(const float* wq, const float* wo, const float* kv, const float* null_kv,
           const float* g1, float* at, float* vt, void* Kt, void* KtT, void* Vt, void* VtT,
           float* colsum, int nb, int C, float scale, hipStream_t st) {
  const long long n = (long long)nb * C * HK;
  fold_fwd_kernel<<<dim3(NH, nb, (C + 63) / 64), 256, 0, st>>>(wq, wo, kv, null_kv, at, vt, nb, C, scale);
  const int Cp = (C + 31) / 32 * 32;
  fold_pack_kernel<T><<<grid_for((long long)nb * KP * Cp), 256, 0, st>>>(at, vt, g1, (T*)Kt, (T*)KtT, (T*)Vt, (T*)VtT, nb, C, Cp);
  fold_colsum_kernel<T><<<nb * KP, 64, 0, st>>>((const T*)Kt, colsum, nb, Cp);
  return check_launch("xattn_fold");
}

}  // namespace

// ---- batched fold backward: every block's fold gradients in four launches,
// run once all blocks' token reductions are done (the kv gradients feed the
// grouped to_kv backward, the rest are parameter gradients) ----
struct FoldBwdBatch {
  DvFoldBwdJob j[DV_FOLD_BWD_MAX];
  int n;
  float scale;
};

__global__ __launch_bounds__(256) void fold_mcorr_batched_kernel(FoldBwdBatch t) {
  const DvFoldBwdJob& J = t.j[blockIdx.y];
  const int row = blockIdx.x;
  if (row >= J.nb * KP) return;
  if (row == 0) {  // zero what the later launches accumulate into
    if (!J.acc_g) {
      for (int c = threadIdx.x; c < J.C; c += 256) {
        if (J.dg1) J.dg1[c] = 0.f;
        if (J.dg2) J.dg2[c] = 0.f;
      }
    }
    if (!J.acc_w && threadIdx.x < 2 * DH) J.dnull[threadIdx.x] = 0.f;
  }
  __shared__ float red[4];
  float s = 0.f;
  for (int c = threadIdx.x; c < J.C; c += 256) s += J.wsR[(long long)row * J.C + c];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) J.mcorr[row] = (red[0] + red[1] + red[2] + red[3]) / J.C;
}

__global__ __launch_bounds__(256) void fold_grad_finish_batched_kernel(FoldBwdBatch t) {
  const DvFoldBwdJob& J = t.j[blockIdx.z];
  if ((int)blockIdx.x * 64 >= J.C || (int)blockIdx.y >= J.nb) return;
  fold_grad_finish_body(J.wsR, J.wsV, J.wsQ, J.mcorr, J.at, J.vt, J.g1, J.dat, J.dvt, J.dg1, J.dg2,
                        J.C, blockIdx.x, blockIdx.y);
}

__global__ void fold_bwd_w_batched_kernel(FoldBwdBatch t) {
  const DvFoldBwdJob& J = t.j[blockIdx.y];
  fold_bwd_w_body(J.dat, J.dvt, J.kv, J.null_kv, J.dwq, J.dwo, J.nb, J.C, t.scale, J.acc_w);
}

__global__ __launch_bounds__(256) void fold_bwd_kv_batched_kernel(FoldBwdBatch t) {
  const DvFoldBwdJob& J = t.j[blockIdx.z >> 1];
  if ((int)blockIdx.y >= J.nb) return;
  fold_bwd_kv_body(J.dat, J.dvt, J.wq, J.wo, J.dkv, J.dnull, J.C, t.scale, blockIdx.x, blockIdx.y,
                   blockIdx.z & 1);
}

extern "C" int dv_xattn_fold_bwd_batched(const DvFoldBwdJob* jobs, int n, float scale,
                                         void* stream) {
  DV_REQUIRE(jobs && n >= 0 && n <= DV_FOLD_BWD_MAX, "bad job table");
  if (n == 0) return DV_OK;
  FoldBwdBatch t;
  t.n = n;
  t.scale = scale;
  int nbmax = 0, cmax = 0;
  for (int i = 0; i < n; ++i) {
    const DvFoldBwdJob& J = jobs[i];
    DV_REQUIRE(J.wsR && J.wsV && J.wsQ && J.mcorr && J.at && J.vt && J.g1 && J.wq && J.wo && J.kv &&
                   J.null_kv && J.dat && J.dvt && J.dwq && J.dwo && J.dkv && J.dnull, "null pointer");
    DV_REQUIRE(J.nb > 0 && J.C > 0 && J.C <= 512, "bad job shape");
    t.j[i] = J;
    nbmax = std::max(nbmax, J.nb);
    cmax = std::max(cmax, J.C);
  }
  hipStream_t st = (hipStream_t)stream;
  fold_mcorr_batched_kernel<<<dim3(nbmax * KP, n), 256, 0, st>>>(t);
  fold_grad_finish_batched_kernel<<<dim3((cmax + 63) / 64, nbmax, n), 256, 0, st>>>(t);
  fold_bwd_w_batched_kernel<<<dim3(grid_for((long long)NH * DH * cmax), n), 256, 0, st>>>(t);
  fold_bwd_kv_batched_kernel<<<dim3(NH, nbmax, 2 * n), 256, sizeof(float) * 3 * cmax, st>>>(t);
  return check_launch("xattn_fold_bwd_batched");
}

extern "C" int dv_xattn_fold_batched(int dtype, const DvFoldJob* jobs, int n, float scale,
                                     void* stream) {
  DV_REQUIRE(jobs && n >= 0 && n <= DV_FOLD_MAX, "bad job table");
  if (n == 0) return DV_OK;
  FoldBatch t;
  t.n = n;
  t.scale = scale;
  int nbmax = 0, rowsmax = 0;
  long long packmax = 0;
  for (int i = 0; i < n; ++i) {
    const DvFoldJob& J = jobs[i];
    DV_REQUIRE(J.wq && J.wo && J.kv && J.null_kv && J.g1 && J.at && J.vt && J.Kt && J.KtT && J.Vt &&
                   J.VtT && J.colsum, "null pointer");
    DV_REQUIRE(J.nb > 0 && J.C > 0 && J.C <= 512, "bad job shape");
    t.j[i] = J;
    nbmax = std::max(nbmax, J.nb);
    rowsmax = std::max(rowsmax, J.nb * KP);
    packmax = std::max(packmax, (long long)J.nb * KP * ((J.C + 31) / 32 * 32));
  }
  hipStream_t st = (hipStream_t)stream;
  fold_fwd_batched_kernel<<<dim3(NH, nbmax, n * 8), 256, 0, st>>>(t);
  const dim3 pg((unsigned)std::min<long long>((packmax + 255) / 256, 1024), n);
  if (dtype == DV_BF16) {
    fold_pack_batched_kernel<bf16><<<pg, 256, 0, st>>>(t);
    fold_colsum_batched_kernel<bf16><<<dim3(rowsmax, n), 64, 0, st>>>(t);
  } else {
    fold_pack_batched_kernel<float><<<pg, 256, 0, st>>>(t);
    fold_colsum_batched_kernel<float><<<dim3(rowsmax, n), 64, 0, st>>>(t);
  }
  return check_launch("xattn_fold_batched");
}

extern "C" int dv_xattn_fold(int dtype, const float* wq, const float* wo, const float* kv,
                             const float* null_kv, const float* g1, float* at, float* vt,
                             void* Kt, void* KtT, void* Vt, void* VtT, float* colsum, int nb,
                             int C, float scale, void* stream) {
  DV_REQUIRE(wq && wo && kv && null_kv && g1 && at && vt && Kt && KtT && Vt && VtT && colsum,
             "null pointer");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == DV_BF16) return fold_t<bf16>(wq, wo, kv, null_kv, g1, at, vt, Kt, KtT, Vt, VtT, colsum, nb, C, scale, st);
  return fold_t<float>(wq, wo, kv, null_kv, g1, at, vt, Kt, KtT, Vt, VtT, colsum, nb, C, scale, st);
}

// channel-split threshold: token tiles below it run 4 waves per tile
static long long xa_split_tiles() { return 1024; }
// 8 waves per tile (512-thread workgroups) for the grids of <= 256 tiles whose
// channels split 8 ways (the 8x8 stage at 256 / 512 channels: each wave's serial
// channel chain halves)
static int xa_cs(long long tiles, int C, bool split) {
  if (!split) return 1;
  return tiles <= 256 && C % 256 == 0 ? 8 : 4;
}

// unrolled channel-loop trips: 32-channel tiles per wave (0 if above 8)
static int xa_nct(int C, int cs) {
  const int cp = (C + 31) / 32 * 32;
  const int n = (cp / 32 + cs - 1) / cs;
  return n <= 8 ? n : 0;
}
// the exact-trip instantiation serves C % 32 == 0 with every wave taking the
// same number of tiles, a power of two; anything else runs NCT = 0
static int xa_exact(int C, int cs) {
  const int n = xa_nct(C, cs);
  const bool ok = C % 32 == 0 && (C / 32) % cs == 0 && (n == 1 || n == 2 || n == 4 || n == 8);
  return ok ? n : 0;
}

extern "C" int dv_xattn_fwd(int dtype, const void* x, int ldx, void* out, int ldo, long long ntok,
                            long long P, int C, const void* Kt, const void* Vt,
                            const float* colsum, const float* g2, float eps, float* stats,
                            void* pbuf, void* stream) {
  DV_REQUIRE(x && out && Kt && Vt && colsum && g2 && stats && pbuf, "null pointer");
  DV_REQUIRE(P > 0 && ntok % P == 0, "ntok must be a multiple of P");
  const int VEC = dtype == DV_BF16 ? 8 : 4;
  DV_REQUIRE(C % VEC == 0 && ldx % VEC == 0 && ldo % 4 == 0, "C / strides must be multiples of 16 bytes");
  hipStream_t st = (hipStream_t)stream;
  const long long tiles = (ntok / P) * ((P + 31) / 32);
  const bool split = tiles < xa_split_tiles() && C >= 128;  // fewer than 256 four-wave workgroups otherwise
  const int cs = xa_cs(tiles, C, split);
  const int blocks = (int)(split ? tiles : (tiles + 3) / 4);
  const int nct = xa_nct(C, cs), ex = xa_exact(C, cs);
  DV_REQUIRE(nct > 0, "C too large for the channel loop (Cp / (32 * CS) <= 8)");
#define XF_LAUNCH(T, CS, N)                                                                         \
  xattn_fwd_kernel<T, CS, N><<<blocks, CS == 8 ? 512 : 256, 0, st>>>(                              \
      (const T*)x, ldx, (T*)out, ldo, ntok, P, C, (const T*)Kt, (const T*)Vt, colsum, g2, eps,      \
      stats, (T*)pbuf)
#define XF_DISPATCH(T)                                                                 \
  switch ((cs == 8 ? 32 : split ? 16 : 0) + ex) {                                      \
    case 1: XF_LAUNCH(T, 1, 1); break;  case 2: XF_LAUNCH(T, 1, 2); break;             \
    case 4: XF_LAUNCH(T, 1, 4); break;  case 8: XF_LAUNCH(T, 1, 8); break;             \
    case 17: XF_LAUNCH(T, 4, 1); break; case 18: XF_LAUNCH(T, 4, 2); break;            \
    case 20: XF_LAUNCH(T, 4, 4); break; case 24: XF_LAUNCH(T, 4, 8); break;            \
    case 33: XF_LAUNCH(T, 8, 1); break; case 34: XF_LAUNCH(T, 8, 2); break;            \
    default: if (cs == 8) XF_LAUNCH(T, 8, 0); else if (split) XF_LAUNCH(T, 4, 0); else XF_LAUNCH(T, 1, 0); break; \
  }
  if (dtype == DV_BF16) {
    XF_DISPATCH(bf16);
  } else {
    XF_DISPATCH(float);
  }
#undef XF_LAUNCH
#undef XF_DISPATCH
  return check_launch("xattn_fwd");
}

extern "C" int dv_xattn_bwd_tokens(int dtype, const void* dy, int lddy, const void* x, int ldx,
                                   void* dx, int lddx, long long ntok, long long P, int C,
                                   const void* KtT, const void* Vt, const void* VtT,
                                   const float* colsum, const float* g2, const float* stats,
                                   const void* pbuf, void* dobuf, void* dsbuf, void* p2buf,
                                   void* stream) {
  DV_REQUIRE(dy && x && dx && KtT && Vt && VtT && colsum && g2 && stats && pbuf && dobuf && dsbuf &&
             p2buf, "null pointer");
  DV_REQUIRE(P > 0 && ntok % P == 0 && C % 8 == 0, "bad shape");
  hipStream_t st = (hipStream_t)stream;
  const long long tiles = (ntok / P) * ((P + 31) / 32);
  const bool split = tiles < xa_split_tiles() && C >= 128;
  const int cs = xa_cs(tiles, C, split);
  // one clip per workgroup (the kernel stages the clip's operand images)
  const int blocks = (int)(split ? tiles : (ntok / P) * (((P + 31) / 32 + 3) / 4));
#define XB_ARGS(T) (const T*)dy, lddy, (const T*)x, ldx, (T*)dx, lddx, ntok, P, C, (const T*)KtT, \
    (const T*)Vt, (const T*)VtT, colsum, g2, stats, (const T*)pbuf, (T*)dobuf, (T*)dsbuf, (T*)p2buf
  const int nct = xa_nct(C, cs), ex = xa_exact(C, cs);
  DV_REQUIRE(nct > 0, "C too large for the channel loop (Cp / (32 * CS) <= 8)");
#define XB_LAUNCH(T, CS, N) xattn_bwd_kernel<T, CS, N><<<blocks, CS == 8 ? 512 : 256, 0, st>>>(XB_ARGS(T))
#define XB_DISPATCH(T)                                                                 \
  switch ((cs == 8 ? 32 : split ? 16 : 0) + ex) {                                      \
    case 1: XB_LAUNCH(T, 1, 1); break;  case 2: XB_LAUNCH(T, 1, 2); break;             \
    case 4: XB_LAUNCH(T, 1, 4); break;  case 8: XB_LAUNCH(T, 1, 8); break;             \
    case 17: XB_LAUNCH(T, 4, 1); break; case 18: XB_LAUNCH(T, 4, 2); break;            \
    case 20: XB_LAUNCH(T, 4, 4); break; case 24: XB_LAUNCH(T, 4, 8); break;            \
    case 33: XB_LAUNCH(T, 8, 1); break; case 34: XB_LAUNCH(T, 8, 2); break;            \
    default: if (cs == 8) XB_LAUNCH(T, 8, 0); else if (split) XB_LAUNCH(T, 4, 0); else XB_LAUNCH(T, 1, 0); break; \
  }
  if (dtype == DV_BF16) {
    XB_DISPATCH(bf16);
  } else {
    XB_DISPATCH(float);
  }
#undef XB_LAUNCH
#undef XB_DISPATCH
#undef XB_ARGS
  return check_launch("xattn_bwd_tokens");
}

extern "C" int dv_xattn_fold_bwd(float* wsR, float* wsV, float* wsQ,
                                 float* mcorr, const float* at, const float* vt,
                                 const float* g1, const float* wq, const float* wo,
                                 const float* kv, const float* null_kv, float* dat, float* dvt,
                                 float* dg1, float* dg2, float* dwq, float* dwo, float* dkv,
                                 float* dnull, int nb, int C, float scale, int acc_g, int acc_w,
                                 void* stream) {
  DV_REQUIRE(wsR && wsV && wsQ && mcorr && at && vt && g1 && wq && wo && kv && null_kv && dat &&
             dvt && dwq && dwo && dkv && dnull, "null pointer");
  hipStream_t st = (hipStream_t)stream;
  if (!acc_g) {
    if (dg1) zero_f32(dg1, C, st);
    if (dg2) zero_f32(dg2, C, st);
  }
  fold_mcorr_kernel<<<nb * KP, 256, 0, st>>>(wsR, mcorr, C);
  fold_grad_finish_kernel<<<dim3((C + 63) / 64, nb), 256, 0, st>>>(wsR, wsV, wsQ, mcorr, at, vt, g1, dat, dvt, dg1, dg2, nb, C);
  fold_bwd_w_kernel<<<grid_for((long long)NH * DH * C), 256, 0, st>>>(dat, dvt, kv, null_kv, dwq, dwo, nb, C, scale, acc_w);
  if (!acc_w) zero_f32(dnull, 2 * DH, st);
  fold_bwd_kv_kernel<<<dim3(NH, nb, 2), 256, sizeof(float) * 3 * C, st>>>(dat, dvt, wq, wo, dkv, dnull,
                                                     C, scale);
  return check_launch("xattn_fold_bwd");
}
