// Mid-block self attention of Unet3D (mid_attn = RearrangeToSequence(Residual(
// Attention(512, heads=16, dim_head=32))), dalle2_video.py:424-432, 551,
// 921-922): multi-query attention — 16 query heads share ONE key/value head,
// a learned null key/value is key 0, logit factor dim_head^-1 (dalle2-pytorch
// scales q by d^-0.5 and q,k by d^-0.25 each).  Flash-style on MFMA: S is
// never materialised; the forward keeps O^T and the softmax state in
// registers, the backward recomputes P from the saved log-sum-exp.
//
// Tile = 32 queries x 32 keys per wave; 4 waves per block.  Products:
//   S^T = K Q^T        (A = K rows, B = Q rows; natural k = d)
//   O^T += V^T P^T     (P^T accumulator reused as the B operand)
//   dkdv: S = Q K^T, dP = dO V^T, dV^T += dO^T P, dK^T += Q^T dS
//   dq:   S^T, dP^T = V dO^T, dQ^T += K^T dS^T
#include <cstdlib>

#include "dv_common.h"

using namespace dv;

// Diagnostic build only (make stamp): per-workgroup s_memrealtime stamps of
// the mid-attention kernels' phases (tools/mqa_stamp.py): kernel k (0 fwd,
// 1 dq, 2 dk/dv), stamps 0 entry, 1 operands staged (loop start), 2 loop
// done, 3 results stored.  The product build compiles none of it.
#ifdef DV_STAMP
constexpr int MQ_NBLK = 4096, MQ_NSTAMP = 4;
__device__ unsigned long long g_mq_stamp[3 * MQ_NBLK * MQ_NSTAMP];
#define MQ_STAMP_AT(k, i)                                                                                  \
  do {                                                                                                     \
    if (threadIdx.x == 0) {                                                                                \
      const long long blin = blockIdx.x + (long long)gridDim.x * (blockIdx.y + (long long)gridDim.y * blockIdx.z); \
      if (blin < MQ_NBLK) g_mq_stamp[((k) * MQ_NBLK + blin) * MQ_NSTAMP + (i)] = __builtin_amdgcn_s_memrealtime(); \
    }                                                                                                      \
  } while (0)
extern "C" int dv_debug_stamps_mqa(unsigned long long* host, long long n) {
  if (n > 3 * MQ_NBLK * MQ_NSTAMP) n = 3 * MQ_NBLK * MQ_NSTAMP;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_mq_stamp), n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#else
#define MQ_STAMP_AT(k, i) \
  do {                    \
  } while (0)
#endif

namespace {

constexpr int DH = 32;  // head dim

template <typename T> struct Mma;
template <> struct Mma<bf16> {
  static constexpr int NS = 2;  // natural k-steps over d = 32
  __device__ static inline f32x16 run(u32x4 a, u32x4 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                   __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
  }
};
template <> struct Mma<float> {
  static constexpr int NS = 4;
  __device__ static inline f32x16 run(u32x4 a, u32x4 b, f32x16 c) {
    const f32x4 af = __builtin_bit_cast(f32x4, a), bf = __builtin_bit_cast(f32x4, b);
#pragma unroll
    for (int j = 0; j < 4; ++j) c = __builtin_amdgcn_mfma_f32_32x32x2f32(af[j], bf[j], c, 0, 0, 0);
    return c;
  }
};

// LDS row strides (bytes): natural tiles read as 16-B chunks, transposed
// tiles read as 8-B (bf16) / 16-B (f32) pieces; padded to avoid conflicts.
template <typename T> constexpr int NAT() { return DH * (int)sizeof(T) + 16; }
template <typename T> constexpr int TRB() { return DH * (int)sizeof(T) + (sizeof(T) == 2 ? 8 : 16); }

// acc(32 x 32) += A(32 x 32) . X where X is an f32 accumulator tile (sum over
// X's row index) and A^T is stored in LDS as AT[i][k] (row stride RB bytes).
template <typename T> __device__ f32x16 mm_acc(const char* AT, f32x16 X, f32x16 acc, int r, int h);
template <>
__device__ f32x16 mm_acc<bf16>(const char* AT, f32x16 X, f32x16 acc, int r, int h) {
  constexpr int RB = TRB<bf16>();
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    bf16x8 bx;
#pragma unroll
    for (int j = 0; j < 8; ++j) bx[j] = (bf16)X[8 * s + j];
    const u32x2 lo = *(const u32x2*)(AT + r * RB + (16 * s + 4 * h) * 2);
    const u32x2 hi = *(const u32x2*)(AT + r * RB + (16 * s + 8 + 4 * h) * 2);
    const u32x4 a = u32x4{lo[0], lo[1], hi[0], hi[1]};
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), bx, acc, 0, 0, 0);
  }
  return acc;
}
template <>
__device__ f32x16 mm_acc<float>(const char* AT, f32x16 X, f32x16 acc, int r, int h) {
  constexpr int RB = TRB<float>();
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const f32x4 a4 = *(const f32x4*)(AT + r * RB + (8 * m + 4 * h) * 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4[e], X[4 * m + e], acc, 0, 0, 0);
  }
  return acc;
}

// cooperative staging of a 32 x 32 tile (rows `src + row*ld`) into a natural
// LDS image and/or a transposed one, by `nthr` threads starting at `t0`.
template <typename T>
__device__ __forceinline__ void stage_tile(const T* src, long long ld, int nvalid, char* nat,
                                           char* tr, int t, int nthr) {
  constexpr int VEC = 16 / sizeof(T);
  constexpr int CPR = DH / VEC;  // chunks per row
  for (int v = t; v < 32 * CPR; v += nthr) {
    const int row = v / CPR, ch = v % CPR;
    u32x4 val = {0u, 0u, 0u, 0u};
    if (row < nvalid) val = *(const u32x4*)(src + row * ld + ch * VEC);
    if (nat) *(u32x4*)(nat + row * NAT<T>() + ch * 16) = val;
    if (tr) {
      const T* e = (const T*)&val;
#pragma unroll
      for (int i = 0; i < VEC; ++i) *(T*)(tr + (ch * VEC + i) * TRB<T>() + row * (int)sizeof(T)) = e[i];
    }
  }
}

template <typename T>
__device__ __forceinline__ void load_nat_regs(const T* row, u32x4* f, int h) {
  constexpr int VEC = 16 / sizeof(T);
#pragma unroll
  for (int s = 0; s < Mma<T>::NS; ++s) f[s] = *(const u32x4*)(row + (2 * s + h) * VEC);
}

template <typename T>
__device__ __forceinline__ f32x16 mm_nat_lds(const char* nat, const u32x4* bf, f32x16 acc, int r, int h) {
#pragma unroll
  for (int s = 0; s < Mma<T>::NS; ++s)
    acc = Mma<T>::run(*(const u32x4*)(nat + r * NAT<T>() + (2 * s + h) * 16), bf[s], acc);
  return acc;
}

__device__ __forceinline__ int acc_row(int e, int h) { return (e & 3) + 8 * (e >> 2) + 4 * h; }

// --------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void mqa_fwd_kernel(const T* q, int ldq, const T* kp, const T* vp,
                                                      T* o, int ldo, float* lse, int N, int NKP,
                                                      int nkeys, int H, float scale) {
  __shared__ __attribute__((aligned(16))) char sK[32 * NAT<T>()];
  __shared__ __attribute__((aligned(16))) char sVt[32 * TRB<T>()];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int b = blockIdx.z, head = blockIdx.y * 4 + wave, q0 = blockIdx.x * 32;
  const bool qok = q0 + r < N;
  u32x4 qf[Mma<T>::NS];
  {
    const long long qrow = (long long)b * N + (qok ? q0 + r : 0);
    load_nat_regs<T>(q + qrow * ldq + head * DH, qf, h);
  }
  f32x16 oacc;
#pragma unroll
  for (int e = 0; e < 16; ++e) oacc[e] = 0.f;
  float m = -INFINITY, l = 0.f;
  const int nkt = NKP / 32;
  for (int kt = 0; kt < nkt; ++kt) {
    __syncthreads();
    stage_tile<T>(kp + ((long long)b * NKP + kt * 32) * DH, DH, 32, sK, nullptr, tid, 256);
    stage_tile<T>(vp + ((long long)b * NKP + kt * 32) * DH, DH, 32, nullptr, sVt, tid, 256);
    __syncthreads();
    f32x16 s;
#pragma unroll
    for (int e = 0; e < 16; ++e) s[e] = 0.f;
    s = mm_nat_lds<T>(sK, qf, s, r, h);
    float mx = -INFINITY;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int key = kt * 32 + acc_row(e, h);
      const float v = key < nkeys ? s[e] * scale : -INFINITY;
      s[e] = v;
      mx = fmaxf(mx, v);
    }
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mnew = fmaxf(m, mx);
    const float alpha = __expf(m - mnew);
    float ps = 0.f;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const float p = __expf(s[e] - mnew);
      s[e] = p;
      ps += p;
    }
    ps += __shfl_xor(ps, 32, 64);
    l = l * alpha + ps;
    m = mnew;
#pragma unroll
    for (int e = 0; e < 16; ++e) oacc[e] *= alpha;
    oacc = mm_acc<T>(sVt, s, oacc, r, h);
  }
  if (qok) {
    const float inv = 1.f / l;
    T* orow = o + ((long long)b * N + q0 + r) * ldo + head * DH;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
#pragma unroll
      for (int e = 0; e < 4; ++e) orow[8 * g + 4 * h + e] = (T)(oacc[4 * g + e] * inv);
    }
    if (h == 0) lse[((long long)b * H + head) * N + q0 + r] = m + __logf(l);
  }
}

// D[b][head][q] = sum_d dO * O
template <typename T>
__global__ void mqa_bwd_d_kernel(const T* o, int ldo, const T* dout, int lddo, float* D, int B,
                                 int N, int H) {
  const long long n = (long long)B * N * H;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int head = (int)(i % H);
    const long long tok = i / H;
    const int b = (int)(tok / N), qq = (int)(tok % N);
    float s = 0.f;
    for (int d = 0; d < DH; ++d)
      s += (float)o[tok * ldo + head * DH + d] * (float)dout[tok * lddo + head * DH + d];
    D[((long long)b * H + head) * N + qq] = s;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void mqa_dq_kernel(const T* q, int ldq, const T* dout, int lddo,
                                                     const float* lse, const float* D, const T* kp,
                                                     const T* vp, T* dq, int lddq, int N, int NKP,
                                                     int nkeys, int H, float scale) {
  __shared__ __attribute__((aligned(16))) char sK[32 * NAT<T>()];
  __shared__ __attribute__((aligned(16))) char sV[32 * NAT<T>()];
  __shared__ __attribute__((aligned(16))) char sKt[32 * TRB<T>()];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int b = blockIdx.z, head = blockIdx.y * 4 + wave, q0 = blockIdx.x * 32;
  const bool qok = q0 + r < N;
  const long long qrow = (long long)b * N + (qok ? q0 + r : 0);
  u32x4 qf[Mma<T>::NS], df[Mma<T>::NS];
  load_nat_regs<T>(q + qrow * ldq + head * DH, qf, h);
  load_nat_regs<T>(dout + qrow * lddo + head * DH, df, h);
  const float Lq = lse[((long long)b * H + head) * N + (qok ? q0 + r : 0)];
  const float Dq = D[((long long)b * H + head) * N + (qok ? q0 + r : 0)];
  f32x16 dqt;
#pragma unroll
  for (int e = 0; e < 16; ++e) dqt[e] = 0.f;
  for (int kt = 0; kt < NKP / 32; ++kt) {
    __syncthreads();
    stage_tile<T>(kp + ((long long)b * NKP + kt * 32) * DH, DH, 32, sK, sKt, tid, 256);
    stage_tile<T>(vp + ((long long)b * NKP + kt * 32) * DH, DH, 32, sV, nullptr, tid, 256);
    __syncthreads();
    f32x16 s, dp;
#pragma unroll
    for (int e = 0; e < 16; ++e) s[e] = dp[e] = 0.f;
    s = mm_nat_lds<T>(sK, qf, s, r, h);
    dp = mm_nat_lds<T>(sV, df, dp, r, h);
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int key = kt * 32 + acc_row(e, h);
      const float p = key < nkeys ? __expf(s[e] * scale - Lq) : 0.f;
      s[e] = p * (dp[e] - Dq);
    }
    dqt = mm_acc<T>(sKt, s, dqt, r, h);
  }
  if (qok) {
    T* row = dq + ((long long)b * N + q0 + r) * lddq + head * DH;
#pragma unroll
    for (int e = 0; e < 16; ++e) row[acc_row(e, h)] = (T)(dqt[e] * scale);
  }
}

// grid (NKP/32, head groups, B); each wave loops over heads w, w+4, ... of its group
template <typename T>
__global__ __launch_bounds__(256) void mqa_dkdv_kernel(const T* q, int ldq, const T* dout, int lddo,
                                                       const float* lse, const float* D,
                                                       const T* kp, const T* vp, float* dkp,
                                                       float* dvp, int N, int NKP, int nkeys,
                                                       int H, int heads_per_group, float scale) {
  constexpr int WS = 2 * 32 * NAT<T>() + 2 * 32 * TRB<T>() + 2 * 32 * 4;  // per-wave LDS
  __shared__ __attribute__((aligned(16))) char smem[4 * WS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int b = blockIdx.z, kt = blockIdx.x;
  char* sQ = smem + wave * WS;
  char* sdO = sQ + 32 * NAT<T>();
  char* sQt = sdO + 32 * NAT<T>();
  char* sdOt = sQt + 32 * TRB<T>();
  float* sL = (float*)(sdOt + 32 * TRB<T>());
  float* sD = sL + 32;
  u32x4 kf[Mma<T>::NS], vf[Mma<T>::NS];
  {
    const long long krow = (long long)b * NKP + kt * 32 + r;
    load_nat_regs<T>(kp + krow * DH, kf, h);
    load_nat_regs<T>(vp + krow * DH, vf, h);
  }
  const bool kok = kt * 32 + r < nkeys;
  f32x16 dkt, dvt;
#pragma unroll
  for (int e = 0; e < 16; ++e) dkt[e] = dvt[e] = 0.f;
  const int nqt = (N + 31) / 32;
  const int iters = (heads_per_group / 4) * nqt;
  for (int it = 0; it < iters; ++it) {
    const int head = blockIdx.y * heads_per_group + wave + 4 * (it / nqt);
    const int qt = it % nqt;
    const int nval = N - qt * 32 < 32 ? N - qt * 32 : 32;
    __syncthreads();
    const long long qrow0 = (long long)b * N + qt * 32;
    stage_tile<T>(q + qrow0 * ldq + head * DH, ldq, nval, sQ, sQt, lane, 64);
    stage_tile<T>(dout + qrow0 * lddo + head * DH, lddo, nval, sdO, sdOt, lane, 64);
    if (lane < 32) {
      const bool ok = lane < nval;
      sL[lane] = ok ? lse[((long long)b * H + head) * N + qt * 32 + lane] : 0.f;
      sD[lane] = ok ? D[((long long)b * H + head) * N + qt * 32 + lane] : 0.f;
    }
    __syncthreads();
    f32x16 s, dp;
#pragma unroll
    for (int e = 0; e < 16; ++e) s[e] = dp[e] = 0.f;
    s = mm_nat_lds<T>(sQ, kf, s, r, h);    // S[q][key]: column key = r
    dp = mm_nat_lds<T>(sdO, vf, dp, r, h); // dP[q][key]
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int qi = acc_row(e, h);
      const float p = (kok && qi < nval) ? __expf(s[e] * scale - sL[qi]) : 0.f;
      s[e] = p;
      dp[e] = p * (dp[e] - sD[qi]);
    }
    dvt = mm_acc<T>(sdOt, s, dvt, r, h);   // dV^T[d][key] += dO^T P
    dkt = mm_acc<T>(sQt, dp, dkt, r, h);   // dK^T[d][key] += Q^T dS
  }
  if (kok) {
    const long long krow = (long long)b * NKP + kt * 32 + r;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      atomicAdd(dkp + krow * DH + acc_row(e, h), dkt[e] * scale);
      atomicAdd(dvp + krow * DH + acc_row(e, h), dvt[e]);
    }
  }
}

// K/V with the null key/value at index 0, zero-padded to NKP keys; keys
// multiplied by kscale (1, or the bf16 path's scale * log2 e: scores then come
// out of the MFMA in log2 units)
template <typename T>
__global__ void mqa_prep_kernel(const T* kv, int ldkv, const float* null_kv, T* kp, T* vp, int B,
                                int N, int NKP, float kscale) {
  const long long n = (long long)B * NKP * DH;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int d = (int)(i % DH);
    const long long bk = i / DH;
    const int key = (int)(bk % NKP), b = (int)(bk / NKP);
    float kv_k = 0.f, kv_v = 0.f;
    if (key == 0) {
      kv_k = null_kv[d];
      kv_v = null_kv[DH + d];
    } else if (key <= N) {
      const long long tok = (long long)b * N + key - 1;
      kv_k = (float)kv[tok * ldkv + d];
      kv_v = (float)kv[tok * ldkv + DH + d];
    }
    kp[i] = (T)(kv_k * kscale);
    vp[i] = (T)kv_v;
  }
}

// bf16 prep, grid (ceil(NKP / 64), B): 64 key rows per block, 4 threads per
// row (8 dims of k and of v each, 16-B loads when the kv rows allow them):
// the rows of mqa_prep_kernel plus each block's largest key norm |k'| (log2
// units) in kmax[b * gridDim.x + block] -- the forward bounds every score by
// |q| max|k'|
constexpr int PREP_KEYS = 64;
__global__ __launch_bounds__(256) void mqa_prep_rows_kernel(const bf16* kv, int ldkv, const float* null_kv,
                                                            bf16* kp, bf16* vp, int N, int NKP, float kscale,
                                                            float* kmax) {
  __shared__ float red[4];
  const int b = blockIdx.y, key = blockIdx.x * PREP_KEYS + (threadIdx.x >> 2), d0 = (threadIdx.x & 3) * 8;
  float n2 = 0.f;
  if (key < NKP) {
    float kf[8], vf[8];
    if (key == 0) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { kf[j] = null_kv[d0 + j]; vf[j] = null_kv[DH + d0 + j]; }
    } else if (key <= N) {
      const bf16* row = kv + ((long long)b * N + key - 1) * ldkv;
      if ((reinterpret_cast<unsigned long long>(row + d0) & 15) == 0) {  // 16-B aligned rows
        const bf16x8 k8 = *(const bf16x8*)(row + d0), v8 = *(const bf16x8*)(row + DH + d0);
#pragma unroll
        for (int j = 0; j < 8; ++j) { kf[j] = (float)k8[j]; vf[j] = (float)v8[j]; }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) { kf[j] = (float)row[d0 + j]; vf[j] = (float)row[DH + d0 + j]; }
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) kf[j] = vf[j] = 0.f;
    }
    bf16x8 ko, vo;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      ko[j] = (bf16)(kf[j] * kscale);
      vo[j] = (bf16)vf[j];
      n2 += (float)ko[j] * (float)ko[j];
    }
    const long long o = ((long long)b * NKP + key) * DH + d0;
    *(bf16x8*)(kp + o) = ko;
    *(bf16x8*)(vp + o) = vo;
  }
  n2 += __shfl_xor(n2, 1, 64);  // the row's 4 threads
  n2 += __shfl_xor(n2, 2, 64);
#pragma unroll
  for (int o = 4; o <= 32; o <<= 1) n2 = fmaxf(n2, __shfl_xor(n2, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = n2;
  __syncthreads();
  if (threadIdx.x == 0)
    kmax[(long long)b * gridDim.x + blockIdx.x] = sqrtf(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
}

template <typename T>
__global__ void mqa_finish_kernel(const float* dkp, const float* dvp, T* dkv, int lddkv,
                                  float* dnull, int B, int N, int NKP, int accumulate) {
  const long long n = (long long)B * N * DH;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int d = (int)(i % DH);
    const long long tok = i / DH;
    const int b = (int)(tok / N), key = (int)(tok % N) + 1;
    dkv[tok * lddkv + d] = (T)dkp[((long long)b * NKP + key) * DH + d];
    dkv[tok * lddkv + DH + d] = (T)dvp[((long long)b * NKP + key) * DH + d];
  }
  if (blockIdx.x == 0 && threadIdx.x < 2 * DH) {
    const int v = threadIdx.x / DH, d = threadIdx.x % DH;
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += (v ? dvp : dkp)[(long long)b * NKP * DH + d];
    dnull[threadIdx.x] = accumulate ? dnull[threadIdx.x] + s : s;
  }
}

// ==========================================================================
// bf16 fast path (gfx950).  Multi-query attention is single-head attention
// of R = N*H query rows per clip (row j = n*H + head, 64 B each when
// ldq == H*32) against NKP keys, so:
//   * forward and dq are query-major: a 512-thread workgroup holds the whole
//     clip's K and V (NKP x 64 B each, <= 160 KiB) in LDS, staged once, and
//     each wave streams all key tiles for its 32 query rows with no further
//     barrier;
//   * dk/dv is key-major: each wave keeps K/V rows of 32 keys in registers
//     and streams 32-row Q / dO tiles (double-buffered, one barrier per two
//     tiles) over a slice of the rows; slices write f32 partials that the
//     finish kernel sums (no atomics).
// LDS images use 64-B rows with the 16-B chunk swizzle c ^ ((r >> 2) & 3),
// which makes both the ds_read_b128 row reads and the ds_read_b64_tr_b16
// transposed reads conflict-free.  Softmax runs in log2 units (c = scale *
// log2 e), lse/D are [B][R]; the running max is only raised when a tile's
// max exceeds it by more than 8 (p <= 256), which skips almost every O
// rescale.
namespace fa {
constexpr int ROW = 64;
constexpr int NW = 16;  // waves per workgroup (4 per SIMD)
constexpr int RG = 8;   // 32-row groups per forward / dq workgroup (256 rows)
typedef __attribute__((ext_vector_type(8))) short s16x8;

__device__ __forceinline__ int img(int r, int c) { return r * ROW + 16 * (c ^ ((r >> 2) & 3)); }

__device__ __forceinline__ s16x4 tr_read(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
}
__device__ __forceinline__ bf16x8 cat8(s16x4 a, s16x4 b) {
  const s16x8 v = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}
// per-lane byte offsets of the row / transposed fragments inside a 32-row
// tile; a tile at row k0 (k0 % 16 == 0) adds k0 * ROW (the swizzle only
// depends on the row within 16)
struct FragOff {
  int row[2];
  int tr[2][2];
};
__device__ __forceinline__ FragOff frag_off(int lane) {
  const int r = lane & 31, h = lane >> 5, q = (lane >> 2) & 3;
  const int c = 2 * ((lane >> 4) & 1) + ((lane & 3) >> 1), bo = 8 * (lane & 1);
  FragOff f;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    f.row[s] = img(r, 2 * s + h);
#pragma unroll
    for (int t = 0; t < 2; ++t) f.tr[s][t] = img(16 * s + 8 * t + 4 * h + q, c) + bo;
  }
  return f;
}
// fragments of a 32-row tile at `base` with addresses computed in place
__device__ __forceinline__ bf16x8 tr_frag(const char* base, int s, int lane) {
  const int h = lane >> 5, q = (lane >> 2) & 3;
  const int c = 2 * ((lane >> 4) & 1) + ((lane & 3) >> 1), bo = 8 * (lane & 1);
  const int r0 = 16 * s + 4 * h + q;
  return cat8(tr_read(base + img(r0, c) + bo), tr_read(base + img(r0 + 8, c) + bo));
}
__device__ __forceinline__ bf16x8 row_frag(const char* base, int s, int r, int h) {
  return *(const bf16x8*)(base + img(r, 2 * s + h));
}
__device__ __forceinline__ bf16x8 row_at(const char* tile, const FragOff& f, int s) {
  return *(const bf16x8*)(tile + f.row[s]);
}
__device__ __forceinline__ bf16x8 tr_at(const char* tile, const FragOff& f, int s) {
  return cat8(tr_read(tile + f.tr[s][0]), tr_read(tile + f.tr[s][1]));
}

// V^T fragments (both k-steps) of a 32-key tile by ds_read_b64_tr_b16 from
// inline asm, waiting for its own reads only: the builtin carries no memory
// operand, so hipcc drains vmcnt before it — i.e. waits for the NEXT chunk's
// LDS-DMA in the streamed kernel on every tile.
__device__ __forceinline__ unsigned lds_off(const char* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
// The reads and their wait are ONE asm statement: the compiler takes an asm
// output as written when the statement ends, so a split issue / wait lets the
// register allocator copy a fragment before its data has landed (measured:
// nondeterministic NaN rows).  tr_issue returns with the data in registers.
struct TrFrag {
  s16x4 x[4];
};
__device__ __forceinline__ TrFrag tr_issue(const char* tile, const FragOff& f) {
  TrFrag t;
  const unsigned b = lds_off(tile);
  asm volatile(
      "ds_read_b64_tr_b16 %0, %4\n\t"
      "ds_read_b64_tr_b16 %1, %5\n\t"
      "ds_read_b64_tr_b16 %2, %6\n\t"
      "ds_read_b64_tr_b16 %3, %7\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(t.x[0]), "=&v"(t.x[1]), "=&v"(t.x[2]), "=&v"(t.x[3])
      : "v"(b + f.tr[0][0]), "v"(b + f.tr[0][1]), "v"(b + f.tr[1][0]), "v"(b + f.tr[1][1])
      : "memory");
  return t;
}
__device__ __forceinline__ void tr_wait(const TrFrag& t, bf16x8& a0, bf16x8& a1) {
  a0 = cat8(t.x[0], t.x[1]);
  a1 = cat8(t.x[2], t.x[3]);
}
// the V^T fragments of two adjacent 32-key tiles (tile1 = tile0 + 32 rows):
// the eight reads differ from two lane bases by immediates (tr[1][t] =
// tr[0][t] + 16 rows, tile1 = +32 rows), so two address adds instead of eight
__device__ __forceinline__ void tr_issue_pair(const char* tile0, const FragOff& f, TrFrag& t0, TrFrag& t1) {
  const unsigned b = lds_off(tile0);
  const unsigned a0 = b + f.tr[0][0], a1 = b + f.tr[0][1];
  static_assert(16 * ROW == 1024 && 32 * ROW == 2048, "immediates below");
  asm volatile(
      "ds_read_b64_tr_b16 %0, %8\n\t"
      "ds_read_b64_tr_b16 %1, %9\n\t"
      "ds_read_b64_tr_b16 %2, %8 offset:1024\n\t"
      "ds_read_b64_tr_b16 %3, %9 offset:1024\n\t"
      "ds_read_b64_tr_b16 %4, %8 offset:2048\n\t"
      "ds_read_b64_tr_b16 %5, %9 offset:2048\n\t"
      "ds_read_b64_tr_b16 %6, %8 offset:3072\n\t"
      "ds_read_b64_tr_b16 %7, %9 offset:3072\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(t0.x[0]), "=&v"(t0.x[1]), "=&v"(t0.x[2]), "=&v"(t0.x[3]), "=&v"(t1.x[0]), "=&v"(t1.x[1]),
        "=&v"(t1.x[2]), "=&v"(t1.x[3])
      : "v"(a0), "v"(a1)
      : "memory");
}

// f32 pair -> packed bf16 (hipcc emits v_cvt_pk_bf16_f32).  Compiler-visible on
// purpose: an inline-asm VALU op that reads a v_exp result or an MFMA result
// gets no hazard wait states from hipcc (it reads the register stale).
__device__ __forceinline__ unsigned cvt_pk(float lo, float hi) {
  typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
  const bf16x2_t v = {(__bf16)lo, (__bf16)hi};
  return __builtin_bit_cast(unsigned, v);
}
// the same as one inline-asm op with its own trans-result wait state (s_nop 0:
// hipcc adds none in front of an asm consumer of v_exp): the dk/dv loop keeps
// its register allocation (no spill at 128 VGPRs) with it
__device__ __forceinline__ unsigned cvt_pk_asm(float lo, float hi) {
  unsigned r;
  asm("s_nop 0\n\tv_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(lo), "v"(hi));
  return r;
}
__device__ __forceinline__ bf16x8 pack8a(const f32x16& x, int s) {
  const u32x4 v = {cvt_pk_asm(x[8 * s], x[8 * s + 1]), cvt_pk_asm(x[8 * s + 2], x[8 * s + 3]),
                   cvt_pk_asm(x[8 * s + 4], x[8 * s + 5]), cvt_pk_asm(x[8 * s + 6], x[8 * s + 7])};
  return __builtin_bit_cast(bf16x8, v);
}
__device__ __forceinline__ bf16x8 pack8(const f32x16& x, int s) {
  const u32x4 v = {cvt_pk(x[8 * s], x[8 * s + 1]), cvt_pk(x[8 * s + 2], x[8 * s + 3]),
                   cvt_pk(x[8 * s + 4], x[8 * s + 5]), cvt_pk(x[8 * s + 6], x[8 * s + 7])};
  return __builtin_bit_cast(bf16x8, v);
}
__device__ __forceinline__ f32x16 mma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float ex2(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ float dot8(bf16x8 a, bf16x8 b) {
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += (float)a[j] * (float)b[j];
  return s;
}
// max of three (hipcc folds chains of fmaxf into v_max3_f32 and inserts the
// MFMA-result wait states an inline-asm form does not get)
__device__ __forceinline__ float max3(float a, float b, float c) {
  return __builtin_fmaxf(__builtin_fmaxf(a, b), c);
}
__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int e = 0; e < 16; ++e) z[e] = 0.f;
  return z;
}

// whole-clip K and V images (NKP rows each) into LDS by LDS-DMA: one 1-KiB
// piece (16 rows) per wave-instruction, source chunks permuted so the
// lane-linear write lands in the swizzled image.  Caller waits vmcnt(0) and
// barriers before reading.
__device__ __forceinline__ void dma_kv(const bf16* kb, const bf16* vb, char* sK, char* sV, int NKP,
                                       int wave, int lane) {
  const __amdgpu_buffer_rsrc_t rk = dma_rsrc(kb, (unsigned)NKP * ROW);
  const __amdgpu_buffer_rsrc_t rv = dma_rsrc(vb, (unsigned)NKP * ROW);
  const int np = NKP / 16;
  const int rr = lane >> 2, slot = lane & 3;
  for (int i = wave; i < 2 * np; i += NW) {
    const bool isv = i >= np;
    const int pc = isv ? i - np : i;
    const int row = pc * 16 + rr;
    const unsigned voff = row * ROW + 16 * (slot ^ ((row >> 2) & 3));
    if (isv)
      dma16(rv, sV + pc * 1024, voff);
    else
      dma16(rk, sK + pc * 1024, voff);
  }
}

__device__ __forceinline__ bf16x8 load_row8(const bf16* p, bool ok) {
  if (!ok) return bf16x8{};
  return *(const bf16x8*)p;
}

// ---- forward --------------------------------------------------------------
// Keys are stored pre-multiplied by c = scale * log2 e (dv_mqa_prep), so S^T =
// K Q^T is the logit in log2 units, and the running max enters as the MFMA's
// C operand (negm = 16 copies of -m per lane: every element a lane holds
// belongs to its one query row): the tile leaves the MFMA as c s - m and
// p = exp2 of it, one VALU op per score.  The next tile's scores are issued
// before this tile's softmax, so its MFMAs run under the exp / sum VALU.
struct Soft {
  f32x16 acc, negm;
  float m, l;
};

__device__ __forceinline__ f32x16 bcast16(float v) {
  f32x16 z;
#pragma unroll
  for (int e = 0; e < 16; ++e) z[e] = v;
  return z;
}
__device__ __forceinline__ f32x16 score(const char* tK, const FragOff& fo, bf16x8 q0, bf16x8 q1, f32x16 c) {
  c = mma(row_at(tK, fo, 0), q0, c);
  return mma(row_at(tK, fo, 1), q1, c);
}
// keys >= nkeys of the tile at global key kg -> -inf (the last tile only).
// The tail test is a scalar branch; the per-element selects sit inside it
// (written as per-element ifs, hipcc evaluated all 16 lane compares and an
// s_or chain on EVERY tile to form the branch mask: ~45 VALU per key pair).
__device__ __forceinline__ void mask_keys(f32x16& s, int kg, int nkeys, int h) {
  const int lim = __builtin_amdgcn_readfirstlane(nkeys - kg);  // keys of this tile still valid
  if (lim < 32) {
    asm volatile("" ::: "memory");  // a side effect: keeps the branch (no if-conversion into selects)
    const int lh = lim - 4 * h;  // acc_row(e, h) = 4 h + an immediate per e
#pragma unroll
    for (int e = 0; e < 16; ++e) s[e] = ((e & 3) + 8 * (e >> 2)) >= lh ? -INFINITY : s[e];
  }
}
// max over the 32 keys of a lane's query column (both half-waves)
__device__ __forceinline__ float half_max(const f32x16& s) {
  float mx = max3(s[0], s[1], s[2]);
#pragma unroll
  for (int e = 3; e < 15; e += 2) mx = max3(mx, s[e], s[e + 1]);
  return __builtin_fmaxf(mx, s[15]);
}
__device__ __forceinline__ float cross_half(float mx) {
  const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
  return max3(mx, __uint_as_float(sw[0]), __uint_as_float(sw[1]));
}
__device__ __forceinline__ float col_max(const f32x16& s) { return cross_half(half_max(s)); }
// first tile of a key range: m = its max
__device__ __forceinline__ void soft_init(Soft& st, f32x16& s) {
  st.m = col_max(s);
#pragma unroll
  for (int e = 0; e < 16; ++e) s[e] -= st.m;
  st.negm = bcast16(-st.m);
  st.acc = zero16();
  st.l = 0.f;
}
// softmax + PV of the tile in s (= c s - m); sn (the next tile's, same m) is
// shifted with it when the max is raised (lazily: only past m + 8)
__device__ __forceinline__ void soft_tile(Soft& st, f32x16& s, f32x16& sn, const char* tV, const FragOff& fo) {
  TrFrag vt = tr_issue(tV, fo);  // V^T of this tile: in flight under the max / exp
  const float mx = col_max(s);
  const bool upd = mx > 8.f;
  if (__builtin_amdgcn_ballot_w64(upd)) {
    const float d = upd ? mx : 0.f;
    const float a = ex2(-d);
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      s[e] -= d;
      sn[e] -= d;
      st.acc[e] *= a;
    }
    st.l *= a;
    st.m += d;
    st.negm = bcast16(-st.m);
  }
#pragma unroll
  for (int e = 0; e < 16; ++e) s[e] = ex2(s[e]);
  float t[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) t[j] = s[2 * j] + s[2 * j + 1];
  st.l += ((t[0] + t[1]) + (t[2] + t[3])) + ((t[4] + t[5]) + (t[6] + t[7]));
  bf16x8 v0, v1;
  tr_wait(vt, v0, v1);
  st.acc = mma(v0, pack8(s, 0), st.acc);
  st.acc = mma(v1, pack8(s, 1), st.acc);
}
// Two key tiles per step (64 keys): one max chain, 32 independent exps and
// 4 PV MFMAs per dependency round — the per-wave chain max -> exp -> PV is
// the bound at 4 waves / SIMD, so a step carries twice the keys.
__device__ __forceinline__ float col_max2(const f32x16& a, const f32x16& b) {
  return cross_half(__builtin_fmaxf(half_max(a), half_max(b)));
}
__device__ __forceinline__ float sum16(const f32x16& s) {
  float t[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) t[j] = s[2 * j] + s[2 * j + 1];
  return ((t[0] + t[1]) + (t[2] + t[3])) + ((t[4] + t[5]) + (t[6] + t[7]));
}
// one step over the key tiles in s0 / s1 (raw log2-unit scores, masked):
// max, lazy rescale, p = exp2(s - m), row sums, then the NEXT pair is scored
// into the dead s0 / s1 registers (its MFMAs overlap this step's PV MFMAs and
// the tail VALU) before this pair's PV.  No C-operand max here: 16 fewer
// VGPRs (the pair step needs them) for one v_sub per score.
__device__ __forceinline__ void soft_step2(Soft& st, f32x16& s0, f32x16& s1, const char* tV0, const char* tV1,
                                           const char* tKn0, const char* tKn1, const FragOff& fo, bf16x8 q0,
                                           bf16x8 q1) {
  TrFrag vt0, vt1;  // tV1 == tV0 + 32 rows
  tr_issue_pair(tV0, fo, vt0, vt1);
  const float mx = col_max2(s0, s1);
  const bool upd = mx > st.m + 8.f;
  if (__builtin_amdgcn_ballot_w64(upd)) {
    const float mn = upd ? mx : st.m;
    const float a = ex2(st.m - mn);
#pragma unroll
    for (int e = 0; e < 16; ++e) st.acc[e] *= a;
    st.l *= a;
    st.m = mn;
  }
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    s0[e] = ex2(s0[e] - st.m);
    s1[e] = ex2(s1[e] - st.m);
  }
  st.l += sum16(s0) + sum16(s1);
  const bf16x8 p00 = pack8(s0, 0), p01 = pack8(s0, 1), p10 = pack8(s1, 0), p11 = pack8(s1, 1);
  s0 = score(tKn0, fo, q0, q1, zero16());
  s1 = score(tKn1, fo, q0, q1, zero16());
  bf16x8 a0, a1, b0, b1;
  tr_wait(vt0, a0, a1);
  tr_wait(vt1, b0, b1);
  st.acc = mma(a0, p00, st.acc);
  st.acc = mma(a1, p01, st.acc);
  st.acc = mma(b0, p10, st.acc);
  st.acc = mma(b1, p11, st.acc);
}
// soft_range with two tiles per step; the state's m is a plain running max
// here (negm unused; the caller starts it at -inf, l = 0, acc = 0); an odd
// range starts with one single-tile step
__device__ __forceinline__ void soft_range2(Soft& st, bool first, const char* sK, const char* sV, int kbeg, int kend,
                                            int kg0, int nkeys, const FragOff& fo, bf16x8 q0, bf16x8 q1, int h) {
  if (kbeg >= kend) return;
  int kt = kbeg;
  if ((kend - kbeg) & 1) {  // single tile: raw scores through the pair step's rules
    f32x16 s = score(sK + kt * 32 * ROW, fo, q0, q1, zero16());
    mask_keys(s, kg0 + kt * 32, nkeys, h);
    TrFrag vt = tr_issue(sV + kt * 32 * ROW, fo);
    const float mx = col_max(s);
    const bool upd = mx > st.m + 8.f;
    if (__builtin_amdgcn_ballot_w64(upd)) {
      const float mn = upd ? mx : st.m;
      const float a = st.m == -INFINITY ? 0.f : ex2(st.m - mn);
#pragma unroll
      for (int e = 0; e < 16; ++e) st.acc[e] *= a;
      st.l *= a;
      st.m = mn;
    }
#pragma unroll
    for (int e = 0; e < 16; ++e) s[e] = ex2(s[e] - st.m);
    st.l += sum16(s);
    bf16x8 a0, a1;
    tr_wait(vt, a0, a1);
    st.acc = mma(a0, pack8(s, 0), st.acc);
    st.acc = mma(a1, pack8(s, 1), st.acc);
    ++kt;
  }
  if (kt >= kend) return;
  f32x16 s0 = score(sK + kt * 32 * ROW, fo, q0, q1, zero16());
  f32x16 s1 = score(sK + (kt + 1) * 32 * ROW, fo, q0, q1, zero16());
  mask_keys(s0, kg0 + kt * 32, nkeys, h);
  mask_keys(s1, kg0 + (kt + 1) * 32, nkeys, h);
  if (st.m == -INFINITY) st.m = col_max2(s0, s1);  // the first step: m = the pair's max
  for (; kt < kend; kt += 2) {
    const int kn0 = kt + 2 < kend ? kt + 2 : kt, kn1 = kn0 + 1;  // the last step re-scores its own pair
    soft_step2(st, s0, s1, sV + kt * 32 * ROW, sV + (kt + 1) * 32 * ROW, sK + kn0 * 32 * ROW,
               sK + kn1 * 32 * ROW, fo, q0, q1);
    mask_keys(s0, kg0 + kn0 * 32, nkeys, h);
    mask_keys(s1, kg0 + kn1 * 32, nkeys, h);
  }
}
// Bounded scores (round 4): when every score of a wave's rows satisfies
// |s| <= |q| max|k'| <= FIX_BOUND (log2 units), p = exp2(s) itself is a
// normal f32 / bf16 number (2^-64 .. 2^64) and the row sums stay far below
// f32's range, so the softmax needs no running max at all: m = 0, no max
// chain, no rescale, one exp2 per score -- the same softmax, exactly.
constexpr float FIX_BOUND = 64.f;
// (Row sums on the MFMA pipe, an all-ones A operand, measured slower in
// round 4 -- profiles/r04l_mqa_msum_ab.txt -- and were removed in round 5.)
__device__ __forceinline__ void soft_step2_fixed(Soft& st, f32x16& s0, f32x16& s1, const char* tV0,
                                                 const char* tV1, const char* tKn0, const char* tKn1,
                                                 const FragOff& fo, bf16x8 q0, bf16x8 q1) {
  TrFrag vt0, vt1;  // tV1 == tV0 + 32 rows
  tr_issue_pair(tV0, fo, vt0, vt1);
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    s0[e] = ex2(s0[e]);
    s1[e] = ex2(s1[e]);
  }
  st.l += sum16(s0) + sum16(s1);
  const bf16x8 p00 = pack8(s0, 0), p01 = pack8(s0, 1), p10 = pack8(s1, 0), p11 = pack8(s1, 1);
  s0 = score(tKn0, fo, q0, q1, zero16());
  s1 = score(tKn1, fo, q0, q1, zero16());
  bf16x8 a0, a1, b0, b1;
  tr_wait(vt0, a0, a1);
  tr_wait(vt1, b0, b1);
  st.acc = mma(a0, p00, st.acc);
  st.acc = mma(a1, p01, st.acc);
  st.acc = mma(b0, p10, st.acc);
  st.acc = mma(b1, p11, st.acc);
}
// soft_range2 for a bounded wave (st.m stays 0)
__device__ __forceinline__ void soft_range2_fixed(Soft& st, const char* sK, const char* sV, int kbeg,
                                                  int kend, int kg0, int nkeys, const FragOff& fo, bf16x8 q0,
                                                  bf16x8 q1, int h) {
  st.m = 0.f;
  if (kbeg >= kend) return;
  int kt = kbeg;
  if ((kend - kbeg) & 1) {
    f32x16 s = score(sK + kt * 32 * ROW, fo, q0, q1, zero16());
    mask_keys(s, kg0 + kt * 32, nkeys, h);
    TrFrag vt = tr_issue(sV + kt * 32 * ROW, fo);
#pragma unroll
    for (int e = 0; e < 16; ++e) s[e] = ex2(s[e]);
    st.l += sum16(s);
    bf16x8 a0, a1;
    tr_wait(vt, a0, a1);
    const bf16x8 ps0 = pack8(s, 0), ps1 = pack8(s, 1);
    st.acc = mma(a0, ps0, st.acc);
    st.acc = mma(a1, ps1, st.acc);
    ++kt;
  }
  if (kt >= kend) return;
  f32x16 s0 = score(sK + kt * 32 * ROW, fo, q0, q1, zero16());
  f32x16 s1 = score(sK + (kt + 1) * 32 * ROW, fo, q0, q1, zero16());
  mask_keys(s0, kg0 + kt * 32, nkeys, h);
  mask_keys(s1, kg0 + (kt + 1) * 32, nkeys, h);
  for (; kt < kend; kt += 2) {
    const int kn0 = kt + 2 < kend ? kt + 2 : kt, kn1 = kn0 + 1;
    soft_step2_fixed(st, s0, s1, sV + kt * 32 * ROW, sV + (kt + 1) * 32 * ROW, sK + kn0 * 32 * ROW,
                     sK + kn1 * 32 * ROW, fo, q0, q1);
    mask_keys(s0, kg0 + kn0 * 32, nkeys, h);
    mask_keys(s1, kg0 + kn1 * 32, nkeys, h);
  }
}
// wave-uniform: every score of this wave's rows within FIX_BOUND?  (kmax:
// the prep's per-block key norms of clip b; NULL = unknown -> online max)
__device__ __forceinline__ bool scores_bounded(const float* kmax, int nkb, int b, int lane, bf16x8 q0, bf16x8 q1) {
  if (kmax == nullptr) return false;
  float km = 0.f;
  for (int i = lane; i < nkb; i += 64) km = fmaxf(km, kmax[(long long)b * nkb + i]);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) km = fmaxf(km, __shfl_xor(km, o, 64));
  float q2 = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) q2 += (float)q0[j] * (float)q0[j] + (float)q1[j] * (float)q1[j];
  q2 += __shfl_xor(q2, 32, 64);
  const bool over = sqrtf(q2) * km > FIX_BOUND;
  return __builtin_amdgcn_readfirstlane((int)(__builtin_amdgcn_ballot_w64(over) == 0)) != 0;
}

// merge the two key halves (half 1 parks its state in LDS at `red`) and store
// O (bf16) and lse (log2 units); returns with only half 0 alive
__device__ __forceinline__ void soft_finish(Soft& st, float* red, int kh, int lane, int h, bool rok,
                                            bf16* orow, float* lsep) {
  __syncthreads();
  if (kh) {
#pragma unroll
    for (int e = 0; e < 16; ++e) red[e * 64 + lane] = st.acc[e];
    red[16 * 64 + lane] = st.l;
    red[17 * 64 + lane] = st.m;
  }
  __syncthreads();
  if (kh) return;
  const float m1 = red[17 * 64 + lane], mn = fmaxf(st.m, m1);
  const float a0 = ex2(st.m - mn), a1 = ex2(m1 - mn);
#pragma unroll
  for (int e = 0; e < 16; ++e) st.acc[e] = st.acc[e] * a0 + red[e * 64 + lane] * a1;
  float l = st.l * a0 + red[16 * 64 + lane] * a1;
  l += __shfl_xor(l, 32, 64);
  if (rok) {
    const float inv = 1.f / l;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const u32x2 v = {cvt_pk(st.acc[4 * g] * inv, st.acc[4 * g + 1] * inv),
                       cvt_pk(st.acc[4 * g + 2] * inv, st.acc[4 * g + 3] * inv)};
      *(u32x2*)(orow + 8 * g + 4 * h) = v;
    }
    if (h == 0) *lsep = mn + __log2f(l);
  }
}

// grid (ceil(R / 256), B), 1024 threads, dynamic LDS 2 * NKP * 64 B.
// Wave w: 32 query rows (group w & 7) against key half w >> 3 of the whole
// clip's K / V, staged once by LDS-DMA; the halves merge through LDS.
__global__ __launch_bounds__(NW * 64) void mqa_fwd_fa_kernel(const bf16* __restrict__ q,
                                                             const bf16* __restrict__ kp,
                                                             const bf16* __restrict__ vp,
                                                             bf16* __restrict__ o, float* lse,
                                                             int R, int NKP, int nkeys, const float* kmax,
                                                             int nkb) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* sK = smem;
  char* sV = smem + NKP * ROW;
  MQ_STAMP_AT(0, 0);
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar loop control
  const int rg = wave & (RG - 1), kh = wave / RG;
  const int b = blockIdx.y;
  const int nkt = NKP / 32, kmid = (nkt + 1) / 2;
  const bf16* kb = kp + (long long)b * NKP * 32;
  const bf16* vb = vp + (long long)b * NKP * 32;
  dma_kv(kb, vb, sK, sV, NKP, wave, lane);
  const int row = blockIdx.x * RG * 32 + rg * 32 + r;
  const bool rok = row < R;
  const bf16* qrow = q + ((long long)b * R + (rok ? row : 0)) * 32;
  const bf16x8 qf0 = load_row8(qrow + 8 * h, rok), qf1 = load_row8(qrow + 16 + 8 * h, rok);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  MQ_STAMP_AT(0, 1);
  const FragOff fo = frag_off(lane);
  const int k0 = kh ? kmid : 0, k1 = kh ? nkt : kmid;
  Soft st{zero16(), zero16(), -INFINITY, 0.f};
  if (scores_bounded(kmax, nkb, b, lane, qf0, qf1))
    soft_range2_fixed(st, sK, sV, k0, k1, 0, nkeys, fo, qf0, qf1, h);
  else
    soft_range2(st, true, sK, sV, k0, k1, 0, nkeys, fo, qf0, qf1, h);
  MQ_STAMP_AT(0, 2);
  soft_finish(st, (float*)smem + rg * 18 * 64, kh, lane, h, rok, o + ((long long)b * R + row) * 32,
              lse + (long long)b * R + row);
#ifdef DV_STAMP
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  MQ_STAMP_AT(0, 3);
}

// Long sequences (config 5: 32 x 16 x 16 = 8,192 tokens, K / V = 1 MiB per
// clip): the same forward with K / V streamed through LDS in chunks of SCK
// keys, double-buffered by LDS-DMA (chunk c + 1 lands while chunk c is
// multiplied); the two key halves of the workgroup take the two halves of
// every chunk.  LDS: 2 buffers x (K + V) x SCK x 64 B = 128 KiB.
constexpr int SCK = 512;
__device__ __forceinline__ void dma_kv_chunk(const __amdgpu_buffer_rsrc_t& rk,
                                             const __amdgpu_buffer_rsrc_t& rv, char* sK, char* sV,
                                             int row0, int nrows, int wave, int lane) {
  const int np = nrows / 16;
  const int rr = lane >> 2, slot = lane & 3;
  for (int i = wave; i < 2 * np; i += NW) {
    const bool isv = i >= np;
    const int pc = isv ? i - np : i;
    const int row = row0 + pc * 16 + rr;
    const unsigned voff = row * ROW + 16 * (slot ^ ((row >> 2) & 3));
    if (isv)
      dma16(rv, sV + pc * 1024, voff);
    else
      dma16(rk, sK + pc * 1024, voff);
  }
}

__global__ __launch_bounds__(NW * 64) void mqa_fwd_fa_stream_kernel(const bf16* __restrict__ q,
                                                                    const bf16* __restrict__ kp,
                                                                    const bf16* __restrict__ vp,
                                                                    bf16* __restrict__ o, float* lse,
                                                                    int R, int NKP, int nkeys, const float* kmax,
                                                                    int nkb) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar loop control
  const int rg = wave & (RG - 1), kh = wave / RG;
  const int b = blockIdx.y;
  const __amdgpu_buffer_rsrc_t rk = dma_rsrc(kp + (long long)b * NKP * 32, (unsigned)NKP * ROW);
  const __amdgpu_buffer_rsrc_t rv = dma_rsrc(vp + (long long)b * NKP * 32, (unsigned)NKP * ROW);
  auto buf_k = [&](int i) { return smem + i * 2 * SCK * ROW; };
  auto buf_v = [&](int i) { return smem + i * 2 * SCK * ROW + SCK * ROW; };
  const int nch = (NKP + SCK - 1) / SCK;
  dma_kv_chunk(rk, rv, buf_k(0), buf_v(0), 0, min(SCK, NKP), wave, lane);
  const int row = blockIdx.x * RG * 32 + rg * 32 + r;
  const bool rok = row < R;
  const bf16* qrow = q + ((long long)b * R + (rok ? row : 0)) * 32;
  const bf16x8 qf0 = load_row8(qrow + 8 * h, rok), qf1 = load_row8(qrow + 16 + 8 * h, rok);
  const FragOff fo = frag_off(lane);
  Soft st{zero16(), zero16(), -INFINITY, 0.f};
  const bool fixed = scores_bounded(kmax, nkb, b, lane, qf0, qf1);
  // chunk ch landed (the only DMA in flight); every wave is done with the
  // buffer chunk ch + 1 goes to (it held chunk ch - 1)
  auto next_chunk = [&](int ch) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int row0 = ch * SCK;
    if (ch + 1 < nch)
      dma_kv_chunk(rk, rv, buf_k((ch + 1) & 1), buf_v((ch + 1) & 1), row0 + SCK,
                   min(SCK, NKP - row0 - SCK), wave, lane);
  };
  // two chunk loops (bounded / online): one loop holding both range bodies
  // spilled at the 128-VGPR cap
  if (fixed) {
    for (int ch = 0; ch < nch; ++ch) {
      next_chunk(ch);
      const int row0 = ch * SCK, nkt = min(SCK, NKP - row0) / 32, kmid = (nkt + 1) / 2;
      soft_range2_fixed(st, buf_k(ch & 1), buf_v(ch & 1), kh ? kmid : 0, kh ? nkt : kmid, row0, nkeys, fo, qf0,
                        qf1, h);
    }
  } else {
    for (int ch = 0; ch < nch; ++ch) {
      next_chunk(ch);
      const int row0 = ch * SCK, nkt = min(SCK, NKP - row0) / 32, kmid = (nkt + 1) / 2;
      soft_range2(st, ch == 0, buf_k(ch & 1), buf_v(ch & 1), kh ? kmid : 0, kh ? nkt : kmid, row0, nkeys, fo, qf0,
                  qf1, h);
    }
  }
  soft_finish(st, (float*)smem + rg * 18 * 64, kh, lane, h, rok, o + ((long long)b * R + row) * 32,
              lse + (long long)b * R + row);
}

// ---- MX-fp8 PV (BASELINE config 5 sampling) --------------------------------
// The streamed forward with O^T += V^T P^T on the block-scaled
// v_mfma_scale_f32_32x32x64_f8f6f4: one MFMA per two 32-key tiles instead of
// four bf16 32x32x16.  The K index k of a 32-key K-block is key
// sigma(k) = 4 (k >> 4) + 8 ((k >> 2) & 3) + (k & 3) of its tile -- the order
// in which lane (q, h) already holds the tile's probabilities in the S^T
// accumulator (element 4g + e = key 4h + 8g + e) -- so P^T is the B operand
// straight from registers (tile t -> bytes 0-15, tile t + 1 -> 16-31; the
// instruction's lane layout, dv_mx8.hip).  V^T comes from an fp8 image
// (mqa_v8_kernel): per 32-key tile 32 rows d of 32 e4m3 bytes in that K order
// (the two 16-B halves swapped on rows with d & 8: conflict-free ds_read_b128)
// and one e8m0 scale per (tile, d), the image of a chunk staged by LDS-DMA
// beside its bf16 K.  P's scale is per key pair and query:
// 2^(floor(max s - m) - 7) puts the pair's largest probability in [128, 256)
// (e4m3 max 448; v_cvt_pk_fp8_f32 does not saturate); the row sums l stay f32
// over the unquantised probabilities.  Online max only (the bounded-score path
// computes no per-tile max to scale by).  QK^T stays bf16: at d = 32 the
// 64-deep fp8 MFMA would be half zeros.
constexpr int V8_TILE = 32 * 32;  // one tile's image: 32 rows d x 32 B
typedef int v8i __attribute__((ext_vector_type(8)));

__device__ __forceinline__ int v8_key(int k) { return 4 * (k >> 4) + 8 * ((k >> 2) & 3) + (k & 3); }
// lane (d, h)'s 16-B half h of row d in a tile image
__device__ __forceinline__ int v8_off(int d, int h) { return d * 32 + 16 * (h ^ ((d >> 3) & 1)); }
__device__ __forceinline__ v8i cat_v8(u32x4 a, u32x4 b) {
  typedef __attribute__((ext_vector_type(8))) unsigned u32x8;
  return __builtin_bit_cast(v8i, (u32x8)__builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
}
// 16 floats (already scaled, |v| < 448) -> 16 e4m3 bytes, element i at byte i
__device__ __forceinline__ u32x4 f8pack16(const float* v) {
  u32x4 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    // high half first over an unspecified word (no zeroing / copy move), then the low half
    const unsigned w =
        __builtin_amdgcn_cvt_pk_fp8_f32(v[4 * i + 2], v[4 * i + 3], __builtin_nondeterministic_value(0u), true);
    r[i] = __builtin_amdgcn_cvt_pk_fp8_f32(v[4 * i], v[4 * i + 1], w, false);
  }
  return r;
}
__device__ __forceinline__ u32x4 f8pack16(const f32x16& s) {
  float v[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) v[e] = s[e];
  return f8pack16(v);
}
__device__ __forceinline__ f32x16 mma8(v8i a, v8i b, f32x16 c, int sa, int sb) {
  return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 0, 0, 0, sa, 0, sb);
}
// scale exponent of a probability block whose largest log2-unit score is mx
// (running max m): p / 2^e then peaks in [128, 256)
__device__ __forceinline__ int p8_exp(float mx, float m) { return (int)floorf(fmaxf(mx - m, -120.f)) - 7; }

// one step over the tiles in s0 / s1 (raw scores, masked), as soft_step2
__device__ __forceinline__ void soft_step2_f8(Soft& st, f32x16& s0, f32x16& s1, const char* tV, const uint8_t* tS,
                                              const char* tKn0, const char* tKn1, const FragOff& fo, int aoff,
                                              int d, int h, bf16x8 q0, bf16x8 q1) {
  const u32x4 va0 = *(const u32x4*)(tV + aoff), va1 = *(const u32x4*)(tV + V8_TILE + aoff);
  const int sa = tS[32 * h + d];  // lane half h: the scale of tile t + h, row d
  const float mx = col_max2(s0, s1);
  const bool upd = mx > st.m + 8.f;
  if (__builtin_amdgcn_ballot_w64(upd)) {
    const float mn = upd ? mx : st.m;
    const float a = ex2(st.m - mn);
#pragma unroll
    for (int e = 0; e < 16; ++e) st.acc[e] *= a;
    st.l *= a;
    st.m = mn;
  }
  const int ex = p8_exp(mx, st.m);
  const float mo = st.m + (float)ex;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    s0[e] = ex2(s0[e] - mo);
    s1[e] = ex2(s1[e] - mo);
  }
  st.l += ldexpf(sum16(s0) + sum16(s1), ex);
  v8i pb = cat_v8(f8pack16(s0), f8pack16(s1));
  // the next pair's scores go into s0 / s1 only after P is packed: the K
  // fragment offsets pass through one asm statement with P, so the loads (and
  // MFMAs) cannot move above the exps.  Unordered, hipcc sank the exps below
  // the next scores: 32 more live VGPRs, spills and 16 copies per step.
  FragOff fk = fo;
  asm volatile("" : "+v"(pb), "+v"(fk.row[0]), "+v"(fk.row[1]));
  s0 = score(tKn0, fk, q0, q1, zero16());
  s1 = score(tKn1, fk, q0, q1, zero16());
  st.acc = mma8(cat_v8(va0, va1), pb, st.acc, sa, ex + 127);
}
__device__ __forceinline__ void soft_range2_f8(Soft& st, const char* sK, const char* sV, const uint8_t* sS, int kbeg,
                                               int kend, int kg0, int nkeys, const FragOff& fo, int aoff, int d,
                                               int h, bf16x8 q0, bf16x8 q1) {
  if (kbeg >= kend) return;
  int kt = kbeg;
  if ((kend - kbeg) & 1) {  // one tile: K-block 1 of both operands is zero
    f32x16 s = score(sK + kt * 32 * ROW, fo, q0, q1, zero16());
    mask_keys(s, kg0 + kt * 32, nkeys, h);
    const u32x4 va = *(const u32x4*)(sV + kt * V8_TILE + aoff), z = {0u, 0u, 0u, 0u};
    const int sa = h ? 127 : sS[kt * 32 + d];  // (tile kt + 1 may lie past the chunk)
    const float mx = col_max(s);
    const bool upd = mx > st.m + 8.f;
    if (__builtin_amdgcn_ballot_w64(upd)) {
      const float mn = upd ? mx : st.m;
      const float a = st.m == -INFINITY ? 0.f : ex2(st.m - mn);
#pragma unroll
      for (int e = 0; e < 16; ++e) st.acc[e] *= a;
      st.l *= a;
      st.m = mn;
    }
    const int ex = p8_exp(mx, st.m);
    const float mo = st.m + (float)ex;
#pragma unroll
    for (int e = 0; e < 16; ++e) s[e] = ex2(s[e] - mo);
    st.l += ldexpf(sum16(s), ex);
    st.acc = mma8(cat_v8(va, z), cat_v8(f8pack16(s), z), st.acc, sa, ex + 127);
    ++kt;
  }
  if (kt >= kend) return;
  f32x16 s0 = score(sK + kt * 32 * ROW, fo, q0, q1, zero16());
  f32x16 s1 = score(sK + (kt + 1) * 32 * ROW, fo, q0, q1, zero16());
  mask_keys(s0, kg0 + kt * 32, nkeys, h);
  mask_keys(s1, kg0 + (kt + 1) * 32, nkeys, h);
  if (st.m == -INFINITY) st.m = col_max2(s0, s1);
  for (; kt < kend; kt += 2) {
    const int kn0 = kt + 2 < kend ? kt + 2 : kt, kn1 = kn0 + 1;
    soft_step2_f8(st, s0, s1, sV + kt * V8_TILE, sS + kt * 32, sK + kn0 * 32 * ROW, sK + kn1 * 32 * ROW, fo, aoff,
                  d, h, q0, q1);
    mask_keys(s0, kg0 + kn0 * 32, nkeys, h);
    mask_keys(s1, kg0 + kn1 * 32, nkeys, h);
  }
}

// the fp8 V^T image of clip b: [NKP / 32 tiles][32 d][32 B] then the scales
// [NKP / 32][32 d] (NKP * 33 bytes per clip).  grid (ceil(NKP / 256), B),
// thread (tile blockIdx.x * 8 + tid / 32, d = tid % 32); vp: dv_mqa_prep's
// bf16 image (null value at key 0, zero padding)
__global__ __launch_bounds__(256) void mqa_v8_kernel(const bf16* __restrict__ vp, uint8_t* __restrict__ v8,
                                                     int NKP) {
  const int b = blockIdx.y, t = blockIdx.x * 8 + (threadIdx.x >> 5), d = threadIdx.x & 31;
  if (t * 32 >= NKP) return;
  const bf16* src = vp + ((long long)b * NKP + t * 32) * DH + d;
  float v[32], amax = 0.f;
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    v[k] = (float)src[v8_key(k) * DH];
    amax = fmaxf(amax, fabsf(v[k]));
  }
  // e8m0 scale 2^(sb - 127) with amax / scale in [128, 256)
  const int eb = (int)((__float_as_uint(amax) >> 23) & 255u);
  const int sb = amax > 0.f ? max(eb - 7, 0) : 127;
  const float inv = __uint_as_float((unsigned)(254 - sb) << 23);
#pragma unroll
  for (int k = 0; k < 32; ++k) v[k] *= inv;
  uint8_t* img = v8 + (long long)b * NKP * 33;
  char* row = (char*)img + (long long)t * V8_TILE + d * 32;
  const int sw = (d >> 3) & 1;
  *(u32x4*)(row + 16 * sw) = f8pack16(v);
  *(u32x4*)(row + 16 * (1 - sw)) = f8pack16(v + 16);
  img[(long long)NKP * 32 + t * 32 + d] = (uint8_t)sb;
}

// chunk pieces: bf16 K rows (16 per piece, swizzled as dma_kv), the chunk's
// fp8 V^T tiles (one per piece) and one piece of scales (32 tiles' worth)
__device__ __forceinline__ void dma_kv8_chunk(const __amdgpu_buffer_rsrc_t& rk, const __amdgpu_buffer_rsrc_t& rv,
                                              char* sK, char* sV, char* sS, int row0, int nrows, int NKP, int wave,
                                              int lane) {
  const int np = nrows / 16, nv = nrows / 32;
  const int rr = lane >> 2, slot = lane & 3;
  for (int i = wave; i < np + nv + 1; i += NW) {
    if (i < np) {
      const int row = row0 + i * 16 + rr;
      dma16(rk, sK + i * 1024, row * ROW + 16 * (slot ^ ((row >> 2) & 3)));
    } else if (i < np + nv) {
      const int t = i - np;
      dma16(rv, sV + t * V8_TILE, (unsigned)((row0 / 32 + t) * V8_TILE + lane * 16));
    } else {
      dma16(rv, sS, (unsigned)(NKP * 32 + row0 + lane * 16));  // scales of tiles row0 / 32 ..
    }
  }
}

// grid (ceil(R / 256), B), 1024 threads, dynamic LDS 2 * (SCK * (64 + 32) + 1024) B
constexpr int S8_BUF = SCK * ROW + SCK * 32 + 1024;
__global__ __launch_bounds__(NW * 64) void mqa_fwd_fa_stream8_kernel(const bf16* __restrict__ q,
                                                                     const bf16* __restrict__ kp,
                                                                     const uint8_t* __restrict__ v8,
                                                                     bf16* __restrict__ o, float* lse, int R,
                                                                     int NKP, int nkeys) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int rg = wave & (RG - 1), kh = wave / RG;
  const int b = blockIdx.y;
  const __amdgpu_buffer_rsrc_t rk = dma_rsrc(kp + (long long)b * NKP * 32, (unsigned)NKP * ROW);
  const __amdgpu_buffer_rsrc_t rv = dma_rsrc(v8 + (long long)b * NKP * 33, (unsigned)NKP * 33);
  auto buf_k = [&](int i) { return smem + i * S8_BUF; };
  auto buf_v = [&](int i) { return smem + i * S8_BUF + SCK * ROW; };
  auto buf_s = [&](int i) { return smem + i * S8_BUF + SCK * ROW + SCK * 32; };
  const int nch = (NKP + SCK - 1) / SCK;
  dma_kv8_chunk(rk, rv, buf_k(0), buf_v(0), buf_s(0), 0, min(SCK, NKP), NKP, wave, lane);
  const int row = blockIdx.x * RG * 32 + rg * 32 + r;
  const bool rok = row < R;
  const bf16* qrow = q + ((long long)b * R + (rok ? row : 0)) * 32;
  const bf16x8 qf0 = load_row8(qrow + 8 * h, rok), qf1 = load_row8(qrow + 16 + 8 * h, rok);
  const FragOff fo = frag_off(lane);
  const int aoff = v8_off(r, h);
  Soft st{zero16(), zero16(), -INFINITY, 0.f};
  for (int ch = 0; ch < nch; ++ch) {
    // chunk ch landed (the only DMA in flight); every wave is done with the
    // buffer chunk ch + 1 goes to (it held chunk ch - 1)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int row0 = ch * SCK;
    if (ch + 1 < nch)
      dma_kv8_chunk(rk, rv, buf_k((ch + 1) & 1), buf_v((ch + 1) & 1), buf_s((ch + 1) & 1), row0 + SCK,
                    min(SCK, NKP - row0 - SCK), NKP, wave, lane);
    const int nkt = min(SCK, NKP - row0) / 32, kmid = (nkt + 1) / 2;
    soft_range2_f8(st, buf_k(ch & 1), buf_v(ch & 1), (const uint8_t*)buf_s(ch & 1), kh ? kmid : 0,
                   kh ? nkt : kmid, row0, nkeys, fo, aoff, r, h, qf0, qf1);
  }
  soft_finish(st, (float*)smem + rg * 18 * 64, kh, lane, h, rok, o + ((long long)b * R + row) * 32,
              lse + (long long)b * R + row);
}

// (A ping-pong forward -- two 8-wave groups per SIMD a half iteration apart
// -- measured slower in round 4, profiles/r04b_pp_ab.txt; removed in round 5.)

// dq (query-major, as the forward: key halves summed through LDS) and
// D = rowsum(dO * O) for the dk/dv pass.  Both per-row constants enter as C
// operands: S^T arrives as c s - L (keys pre-scaled by c), dP^T as dP - D, so
// dS = exp2(.) * (.) is two VALU ops per score.  dq = (K^T dS^T) / log2 e
// (the keys carry c = scale * log2 e; dq needs scale).
__global__ __launch_bounds__(NW * 64) void mqa_dq_fa_kernel(
    const bf16* __restrict__ q, const bf16* __restrict__ o, const bf16* __restrict__ dout,
    const float* __restrict__ lse, const bf16* __restrict__ kp, const bf16* __restrict__ vp,
    bf16* __restrict__ dq, float* __restrict__ D, int R, int NKP, int nkeys) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* sK = smem;
  char* sV = smem + NKP * ROW;
  MQ_STAMP_AT(1, 0);
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar loop control
  const int rg = wave & (RG - 1), kh = wave / RG;
  const int b = blockIdx.y;
  const int nkt = NKP / 32, kmid = (nkt + 1) / 2;
  const bf16* kb = kp + (long long)b * NKP * 32;
  const bf16* vb = vp + (long long)b * NKP * 32;
  dma_kv(kb, vb, sK, sV, NKP, wave, lane);
  const int row = blockIdx.x * RG * 32 + rg * 32 + r;
  const bool rok = row < R;
  const long long ro = ((long long)b * R + (rok ? row : 0)) * 32;
  const bf16x8 qf0 = load_row8(q + ro + 8 * h, rok), qf1 = load_row8(q + ro + 16 + 8 * h, rok);
  const bf16x8 df0 = load_row8(dout + ro + 8 * h, rok), df1 = load_row8(dout + ro + 16 + 8 * h, rok);
  float dd = dot8(df0, load_row8(o + ro + 8 * h, rok)) + dot8(df1, load_row8(o + ro + 16 + 8 * h, rok));
  dd += __shfl_xor(dd, 32, 64);
  const float L2 = rok ? lse[(long long)b * R + row] : 0.f;
  if (rok && h == 0 && kh == 0) D[(long long)b * R + row] = dd;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  MQ_STAMP_AT(1, 1);
  const FragOff fo = frag_off(lane);
  const f32x16 negL = bcast16(-L2), negD = bcast16(-dd);
  f32x16 acc = zero16();
  const int kbeg = kh ? kmid : 0, kend = kh ? nkt : kmid;
  auto tile = [&](int kt) {
    const int k0 = kt * 32;
    const char* tK = sK + k0 * ROW;
    const char* tV = sV + k0 * ROW;
    f32x16 s = score(tK, fo, qf0, qf1, negL);
    f32x16 dp = mma(row_at(tV, fo, 0), df0, negD);
    dp = mma(row_at(tV, fo, 1), df1, dp);
#pragma unroll
    for (int e = 0; e < 16; ++e) s[e] = ex2(s[e]) * dp[e];
    const int lim = __builtin_amdgcn_readfirstlane(nkeys - k0);  // valid keys of this tile
    if (lim < 32) {  // the last tile only: a scalar branch (see mask_keys)
      asm volatile("" ::: "memory");
      const int lh = lim - 4 * h;
#pragma unroll
      for (int e = 0; e < 16; ++e) s[e] = ((e & 3) + 8 * (e >> 2)) >= lh ? 0.f : s[e];
    }
    acc = mma(tr_at(tK, fo, 0), pack8(s, 0), acc);
    acc = mma(tr_at(tK, fo, 1), pack8(s, 1), acc);
  };
  for (int kt = kbeg; kt < kend; ++kt) tile(kt);
  MQ_STAMP_AT(1, 2);
  __syncthreads();
  float* red = (float*)smem + rg * 16 * 64;
  if (kh) {
#pragma unroll
    for (int e = 0; e < 16; ++e) red[e * 64 + lane] = acc[e];
  }
  __syncthreads();
  if (kh) return;
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] += red[e * 64 + lane];
  if (rok) {
    constexpr float INV_LOG2E = 0.6931471805599453f;
    bf16* qrow = dq + ((long long)b * R + row) * 32;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const u32x2 v = {cvt_pk(acc[4 * g] * INV_LOG2E, acc[4 * g + 1] * INV_LOG2E),
                       cvt_pk(acc[4 * g + 2] * INV_LOG2E, acc[4 * g + 3] * INV_LOG2E)};
      *(u32x2*)(qrow + 8 * g + 4 * h) = v;
    }
  }
#ifdef DV_STAMP
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  MQ_STAMP_AT(1, 3);
}

// dk/dv, key-major.  grid (ceil(nkt / 4), S, B); wave w: key tile
// blockIdx.x * 4 + (w & 3), query-tile parity w >> 2 (four tiles per step).
// Partials ws[split][b][NKP][64] = (scale * dK | dV) over the split's rows.
// Rows past the slice load a clamped row with -L = -inf (p = 0), so every
// step issues the same loads (exact vmcnt accounting, no exec branches).
constexpr int TB = 2 * 32 * ROW + 2 * 32 * 4;  // one tile: Q, dO images, L, -D
constexpr int QP = NW / 4;                      // query-tile parities
constexpr int RED = 2 * 4 * 2 * 16 * 64 * 4;    // parity combine (two parities at a time)
// (Two query tiles per wave between barriers measured slower in round 4,
// profiles/r04o_mqa_ph_tps_ab.txt: one tile per step.)
__global__ __launch_bounds__(NW * 64) void mqa_dkdv_fa_kernel(
    const bf16* __restrict__ q, const bf16* __restrict__ dout, const float* __restrict__ lse,
    const float* __restrict__ D, const bf16* __restrict__ kp, const bf16* __restrict__ vp,
    float* __restrict__ ws, int R, int NKP, int nkeys, int rows_per_split, float scale) {
  constexpr int TPS = 1;
  __shared__ __attribute__((aligned(16))) char smem[2 * QP * TPS * TB > RED ? 2 * QP * TPS * TB : RED];
  MQ_STAMP_AT(2, 0);
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar loop control
  const int b = blockIdx.z, split = blockIdx.y;
  const int kt = blockIdx.x * 4 + (wave & 3), qp = wave >> 2;
  const bool kvalid = kt < NKP / 32;
  const long long krow = (long long)b * NKP + (kvalid ? kt * 32 + r : 0);
  bf16x8 kf0 = *(const bf16x8*)(kp + krow * 32 + 8 * h), kf1 = *(const bf16x8*)(kp + krow * 32 + 16 + 8 * h);
  bf16x8 vf0 = *(const bf16x8*)(vp + krow * 32 + 8 * h), vf1 = *(const bf16x8*)(vp + krow * 32 + 16 + 8 * h);
  const int r0 = split * rows_per_split;
  const int r1 = min(R, r0 + rows_per_split);
  const int nsteps = r1 > r0 ? (r1 - r0 + 32 * QP * TPS - 1) / (32 * QP * TPS) : 0;
  // staging role: thread t -> tile parity t >> 8; u < 128 Q chunk, else dO chunk; u < 32 also L, -D
  const int sp = tid >> 8, u = tid & 255, cu = u & 127, crow = cu >> 2, cch = cu & 3;
  const bf16* src = (u < 128 ? q : dout) + (long long)b * R * 32;
  const float* lsrc = lse + (long long)b * R;
  const float* dsrc = D + (long long)b * R;
  u32x4 cv[TPS];
  float lv[TPS], dv[TPS];
  int lrow[TPS];
  auto load = [&](int st) {
#pragma unroll
    for (int j = 0; j < TPS; ++j) {
      const int tq = QP * (TPS * st + j) + sp;  // query tile of the split
      const int rr = r0 + tq * 32 + crow;
      cv[j] = *(const u32x4*)(src + (long long)min(rr, r1 - 1) * 32 + cch * 8);
      lrow[j] = r0 + tq * 32 + (u & 31);
      lv[j] = lsrc[min(lrow[j], r1 - 1)];
      dv[j] = dsrc[min(lrow[j], r1 - 1)];
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int j = 0; j < TPS; ++j) {
      char* t = smem + (QP * (TPS * buf + j) + sp) * TB;
      *(u32x4*)(t + (u < 128 ? 0 : 32 * ROW) + img(crow, cch)) = cv[j];
      if (u < 32) {
        ((float*)(t + 2 * 32 * ROW))[u] = lrow[j] < r1 ? -lv[j] : -INFINITY;
        ((float*)(t + 2 * 32 * ROW))[32 + u] = -dv[j];
      }
    }
  };
  // retire the K/V fragment loads here so the loop carries no vmcnt for them
  asm volatile("" : "+v"(kf0), "+v"(kf1), "+v"(vf0), "+v"(vf1));
  f32x16 dk = zero16(), dvv = zero16();
  if (nsteps > 0) {
    load(0);
    store(0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // step st+1's tile was loaded during step st-1 and is stored at the top of
  // step st (its buffer was read in step st-1, before the last barrier), then
  // step st+2's loads go out: a whole step of latency cover instead of one
  // step's compute (33.0-33.6 -> 31.6-31.7 us, profiles/r04o_mqa_early_ab.txt)
  if (nsteps > 1) load(1);
  __syncthreads();
  MQ_STAMP_AT(2, 1);
  for (int st = 0; st < nsteps; ++st) {
    const bool more = st + 1 < nsteps;
    if (more) store((st + 1) & 1);
    if (st + 2 < nsteps) load(st + 2);
#pragma unroll
    for (int j = 0; j < TPS; ++j) {
    const char* t = smem + (QP * (TPS * (st & 1) + j) + qp) * TB;
    if (kvalid) {
      const char* sQ = t;
      const char* sdO = t + 32 * ROW;
      const float* sL = (const float*)(t + 2 * 32 * ROW);
      const float* sD = sL + 32;
      // dP arrives as dP - D (C operand -D); S in log2 units (keys pre-scaled)
      f32x16 s = zero16(), dp;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 d4 = *(const f32x4*)(sD + 8 * g + 4 * h);
#pragma unroll
        for (int e = 0; e < 4; ++e) dp[4 * g + e] = d4[e];
      }
      s = mma(row_frag(sQ, 0, r, h), kf0, s);
      dp = mma(row_frag(sdO, 0, r, h), vf0, dp);
      s = mma(row_frag(sQ, 1, r, h), kf1, s);
      dp = mma(row_frag(sdO, 1, r, h), vf1, dp);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 l4 = *(const f32x4*)(sL + 8 * g + 4 * h);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float p = ex2(s[4 * g + e] + l4[e]);  // the staged value is -L
          s[4 * g + e] = p;
          dp[4 * g + e] *= p;
        }
      }
      dvv = mma(tr_frag(sdO, 0, lane), pack8a(s, 0), dvv);
      dk = mma(tr_frag(sQ, 0, lane), pack8a(dp, 0), dk);
      dvv = mma(tr_frag(sdO, 1, lane), pack8a(s, 1), dvv);
      dk = mma(tr_frag(sQ, 1, lane), pack8a(dp, 1), dk);
    }
    }
    __syncthreads();
  }
  MQ_STAMP_AT(2, 2);
  // combine the parities through LDS (3,2 -> 1,0, then 1 -> 0), one partial per split
  float* red = (float*)smem;
  auto park = [&](int slot) {
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      red[((slot * 4 + (wave & 3)) * 32 + e) * 64 + lane] = dk[e];
      red[((slot * 4 + (wave & 3)) * 32 + 16 + e) * 64 + lane] = dvv[e];
    }
  };
  auto take = [&](int slot) {
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      dk[e] += red[((slot * 4 + (wave & 3)) * 32 + e) * 64 + lane];
      dvv[e] += red[((slot * 4 + (wave & 3)) * 32 + 16 + e) * 64 + lane];
    }
  };
  if (qp >= 2) park(qp - 2);
  __syncthreads();
  if (qp < 2) take(qp);
  __syncthreads();
  if (qp == 1) park(0);
  __syncthreads();
  if (qp == 0 && kvalid) {
    take(0);
    float* w = ws + (((long long)split * gridDim.z + b) * NKP + kt * 32 + r) * 64;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      f32x4 a, v;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        a[e] = dk[4 * g + e] * scale;
        v[e] = dvv[4 * g + e];
      }
      *(f32x4*)(w + 8 * g + 4 * h) = a;
      *(f32x4*)(w + 32 + 8 * g + 4 * h) = v;
    }
  }
#ifdef DV_STAMP
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  MQ_STAMP_AT(2, 3);
}

// dkv[b*N + n] = sum over splits of ws[.][b][n + 1]; dnull (+)= sum over b, splits of key 0
template <int S>
__global__ void mqa_finish_fa_kernel(const float* __restrict__ ws, int B, int N, int NKP,
                                     bf16* __restrict__ dkv, int lddkv, float* dnull, int accumulate) {
  const long long n = (long long)B * N * 16;  // float4 groups
  const long long sstride = (long long)B * NKP * 64;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int g = (int)(i & 15);
    const long long tok = i >> 4;
    const int b = (int)(tok / N), key = (int)(tok % N) + 1;
    const float* p = ws + ((long long)b * NKP + key) * 64 + 4 * g;
    f32x4 v[S];
#pragma unroll
    for (int s = 0; s < S; ++s) v[s] = *(const f32x4*)(p + s * sstride);
#pragma unroll
    for (int s = 1; s < S; ++s) v[0] += v[s];
    const u32x2 o = {cvt_pk(v[0][0], v[0][1]), cvt_pk(v[0][2], v[0][3])};
    *(u32x2*)(dkv + tok * lddkv + 4 * g) = o;
  }
  if (blockIdx.x == 0 && threadIdx.x < 64) {
    float s = 0.f;
    for (int b = 0; b < B; ++b)
      for (int sp = 0; sp < S; ++sp) s += ws[sp * sstride + (long long)b * NKP * 64 + threadIdx.x];
    dnull[threadIdx.x] = accumulate ? dnull[threadIdx.x] + s : s;
  }
}

constexpr float LOG2E = 1.4426950408889634f;

// the forward and the backward must take the same path (lse layout/units)
bool eligible(int dtype, int ldq, int ldo, int H, int NKP) {
  return dtype == DV_BF16 && ldq == H * DH && ldo == H * DH &&
         (long long)NKP * 2 * ROW <= 160 * 1024;
}
// the streamed forward: bf16, packed rows, K / V larger than one LDS image
bool eligible_stream(int dtype, int ldq, int ldo, int H, int NKP) {
  return dtype == DV_BF16 && ldq == H * DH && ldo == H * DH && !eligible(dtype, ldq, ldo, H, NKP) &&
         (long long)NKP * ROW < (1ll << 31);
}

int splits(int NKP, int B) {
  const int nkg = (NKP / 32 + 3) / 4;
  int s = 256 / (nkg * B);
  return s < 1 ? 1 : (s > 16 ? 16 : s);
}

template <int S>
void launch_finish(int s, int grid, hipStream_t st, const float* ws, int B, int N, int NKP, bf16* dkv,
                   int lddkv, float* dnull, int accumulate) {
  if constexpr (S >= 1) {
    if (s == S)
      mqa_finish_fa_kernel<S><<<grid, 256, 0, st>>>(ws, B, N, NKP, dkv, lddkv, dnull, accumulate);
    else
      launch_finish<S - 1>(s, grid, st, ws, B, N, NKP, dkv, lddkv, dnull, accumulate);
  }
}

void set_lds(const void* fn, int bytes) {
  (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}
}  // namespace fa

int grid_for(long long work) {
  long long b = (work + 255) / 256;
  if (b > 16384) b = 16384;
  return (int)(b < 1 ? 1 : b);
}

}  // namespace

extern "C" int dv_mqa_prep(int dtype, const void* kv, int ldkv, const float* null_kv, void* kp,
                           void* vp, int B, int N, int NKP, float scale, float* kmax, void* stream) {
  DV_REQUIRE(kv && null_kv && kp && vp && NKP >= N + 1 && NKP % 32 == 0, "bad arguments");
  hipStream_t st = (hipStream_t)stream;
  const long long n = (long long)B * NKP * DH;
  if (dtype == DV_BF16 && kmax)  // keys in log2 units of the logit + the key-norm bound
    mqa_prep_rows_kernel<<<dim3((NKP + PREP_KEYS - 1) / PREP_KEYS, B), 256, 0, st>>>((const bf16*)kv, ldkv, null_kv, (bf16*)kp,
                                                                    (bf16*)vp, N, NKP, scale * fa::LOG2E, kmax);
  else if (dtype == DV_BF16)  // keys in log2 units of the logit (the fa kernels' contract)
    mqa_prep_kernel<bf16><<<grid_for(n), 256, 0, st>>>((const bf16*)kv, ldkv, null_kv, (bf16*)kp, (bf16*)vp, B, N, NKP,
                                                      scale * fa::LOG2E);
  else
    mqa_prep_kernel<float><<<grid_for(n), 256, 0, st>>>((const float*)kv, ldkv, null_kv, (float*)kp, (float*)vp, B, N,
                                                       NKP, 1.f);
  return check_launch("mqa_prep");
}

extern "C" int dv_mqa_fwd(int dtype, const void* q, int ldq, const void* kp, const void* vp,
                          void* o, int ldo, float* lse, int B, int N, int NKP, int H, float scale,
                          const float* kmax, void* stream) {
  // kmax: dv_mqa_prep's key-norm bound (NULL: online max everywhere)
  const int nkb = (NKP + PREP_KEYS - 1) / PREP_KEYS;
  DV_REQUIRE(q && kp && vp && o && lse && H % 4 == 0 && NKP % 32 == 0, "bad arguments");
  DV_REQUIRE(ldq % 8 == 0 && ldo >= H * DH, "bad strides");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == DV_BF16) {
    // bf16 keys come from dv_mqa_prep pre-scaled: only the fa kernels read them
    DV_REQUIRE(ldq == H * DH && ldo == H * DH, "bf16 path needs dense q / o rows");
    const int R = N * H;
    const dim3 grid((R + 255) / 256, B);
    if (fa::eligible(dtype, ldq, ldo, H, NKP)) {
      const int lds = max(NKP * 2 * fa::ROW, fa::RG * 18 * 64 * 4);
      fa::set_lds((const void*)fa::mqa_fwd_fa_kernel, lds);
      fa::mqa_fwd_fa_kernel<<<grid, fa::NW * 64, lds, st>>>((const bf16*)q, (const bf16*)kp, (const bf16*)vp,
                                                            (bf16*)o, lse, R, NKP, N + 1, kmax, nkb);
    } else {
      // the whole clip's K / V do not fit LDS: stream them in 512-key chunks
      DV_REQUIRE((long long)NKP * fa::ROW < (1ll << 31), "sequence too long");
      const int lds = 4 * fa::SCK * fa::ROW;
      fa::set_lds((const void*)fa::mqa_fwd_fa_stream_kernel, lds);
      fa::mqa_fwd_fa_stream_kernel<<<grid, fa::NW * 64, lds, st>>>(
          (const bf16*)q, (const bf16*)kp, (const bf16*)vp, (bf16*)o, lse, R, NKP, N + 1, kmax, nkb);
    }
  } else {
    dim3 grid((N + 31) / 32, H / 4, B);
    mqa_fwd_kernel<float><<<grid, 256, 0, st>>>((const float*)q, ldq, (const float*)kp, (const float*)vp, (float*)o,
                                                ldo, lse, N, NKP, N + 1, H, scale);
  }
  return check_launch("mqa_fwd");
}

extern "C" int dv_mqa_fwd_fp8_ws(int B, int NKP, long long* bytes) {
  DV_REQUIRE(bytes && B > 0 && NKP > 0 && NKP % 32 == 0, "bad arguments");
  *bytes = (long long)B * NKP * 33;
  return DV_OK;
}

extern "C" int dv_mqa_fwd_fp8(const void* q, int ldq, const void* kp, const void* vp, void* v8, long long v8_bytes,
                              void* o, int ldo, float* lse, int B, int N, int NKP, int H, void* stream) {
  DV_REQUIRE(q && kp && vp && v8 && o && lse && B > 0 && N > 0, "bad arguments");
  DV_REQUIRE(NKP % 32 == 0 && NKP >= N + 1 && ldq == H * DH && ldo == H * DH && H > 0, "bad shape / strides");
  DV_REQUIRE(v8_bytes >= (long long)B * NKP * 33 && (long long)NKP * fa::ROW < (1ll << 31),
             "workspace too small (see dv_mqa_fwd_fp8_ws) or sequence too long");
  hipStream_t st = (hipStream_t)stream;
  fa::mqa_v8_kernel<<<dim3((NKP / 32 + 7) / 8, B), 256, 0, st>>>((const bf16*)vp, (uint8_t*)v8, NKP);
  const int R = N * H;
  const int lds = 2 * fa::S8_BUF;
  fa::set_lds((const void*)fa::mqa_fwd_fa_stream8_kernel, lds);
  fa::mqa_fwd_fa_stream8_kernel<<<dim3((R + 255) / 256, B), fa::NW * 64, lds, st>>>(
      (const bf16*)q, (const bf16*)kp, (const uint8_t*)v8, (bf16*)o, lse, R, NKP, N + 1);
  return check_launch("mqa_fwd_fp8");
}

extern "C" int dv_mqa_bwd_ws(int dtype, int ldq, int ldo, int B, int N, int NKP, int H,
                             long long* floats) {
  DV_REQUIRE(floats && B > 0 && N > 0 && NKP % 32 == 0, "bad arguments");
  if (fa::eligible(dtype, ldq, ldo, H, NKP))
    *floats = (long long)fa::splits(NKP, B) * B * NKP * 64;
  else
    *floats = (long long)B * NKP * DH * 2;
  return DV_OK;
}

extern "C" int dv_mqa_bwd(int dtype, const void* q, int ldq, const void* o, int ldo,
                          const void* dout, int lddo, const float* lse, const void* kp,
                          const void* vp, void* dq, int lddq, float* D, float* ws,
                          long long ws_floats, void* dkv, int lddkv, float* dnull, int B, int N,
                          int NKP, int H, float scale, int accumulate, void* stream) {
  DV_REQUIRE(q && o && dout && lse && kp && vp && dq && D && ws && dkv && dnull, "null pointer");
  DV_REQUIRE(H % 8 == 0 && NKP % 32 == 0, "bad shape");
  long long need = 0;
  dv_mqa_bwd_ws(dtype, ldq, ldo, B, N, NKP, H, &need);
  DV_REQUIRE(ws_floats >= need, "workspace too small (see dv_mqa_bwd_ws)");
  hipStream_t st = (hipStream_t)stream;
  if (fa::eligible(dtype, ldq, ldo, H, NKP)) {
    DV_REQUIRE(lddo == H * DH && lddq == H * DH, "bf16 path needs dense dout/dq rows");
    const int R = N * H, lds = max(NKP * 2 * fa::ROW, fa::RG * 16 * 64 * 4), S = fa::splits(NKP, B);
    const int rps = ((R + S - 1) / S + 63) / 64 * 64;
    fa::set_lds((const void*)fa::mqa_dq_fa_kernel, lds);
    fa::mqa_dq_fa_kernel<<<dim3((R + 255) / 256, B), fa::NW * 64, lds, st>>>(
        (const bf16*)q, (const bf16*)o, (const bf16*)dout, lse, (const bf16*)kp, (const bf16*)vp, (bf16*)dq, D, R,
        NKP, N + 1);
    const dim3 gkv((NKP / 32 + 3) / 4, S, B);
    fa::mqa_dkdv_fa_kernel<<<gkv, fa::NW * 64, 0, st>>>((const bf16*)q, (const bf16*)dout, lse, D, (const bf16*)kp,
                                                        (const bf16*)vp, ws, R, NKP, N + 1, rps, scale);
    DV_REQUIRE(S >= 1 && S <= 16, "split count out of range");
    fa::launch_finish<16>(S, grid_for((long long)B * N * 16), st, ws, B, N, NKP, (bf16*)dkv, lddkv,
                          dnull, accumulate);

    return check_launch("mqa_bwd");
  }
  DV_REQUIRE(dtype == DV_F32, "bf16 backward needs the whole clip's K / V in LDS (NKP <= 1280)");
  float* dkp = ws;
  float* dvp = ws + (long long)B * NKP * DH;
  zero_f32(dkp, (long long)B * NKP * DH, st);
  zero_f32(dvp, (long long)B * NKP * DH, st);
  const int hg = 2, hpg = H / hg;
  mqa_bwd_d_kernel<float><<<grid_for((long long)B * N * H), 256, 0, st>>>((const float*)o, ldo, (const float*)dout, lddo, D, B, N, H);
  mqa_dq_kernel<float><<<dim3((N + 31) / 32, H / 4, B), 256, 0, st>>>((const float*)q, ldq, (const float*)dout, lddo, lse, D, (const float*)kp, (const float*)vp, (float*)dq, lddq, N, NKP, N + 1, H, scale);
  mqa_dkdv_kernel<float><<<dim3(NKP / 32, hg, B), 256, 0, st>>>((const float*)q, ldq, (const float*)dout, lddo, lse, D, (const float*)kp, (const float*)vp, dkp, dvp, N, NKP, N + 1, H, hpg, scale);
  mqa_finish_kernel<float><<<grid_for((long long)B * N * DH), 256, 0, st>>>(dkp, dvp, (float*)dkv, lddkv, dnull, B, N, NKP, accumulate);
  return check_launch("mqa_bwd");
}
