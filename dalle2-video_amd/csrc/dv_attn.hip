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
#include "dv_common.h"

using namespace dv;

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

// K/V with the null key/value at index 0, zero-padded to NKP keys
template <typename T>
__global__ void mqa_prep_kernel(const T* kv, int ldkv, const float* null_kv, T* kp, T* vp, int B,
                                int N, int NKP) {
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
    kp[i] = (T)kv_k;
    vp[i] = (T)kv_v;
  }
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

int grid_for(long long work) {
  long long b = (work + 255) / 256;
  if (b > 16384) b = 16384;
  return (int)(b < 1 ? 1 : b);
}

}  // namespace

extern "C" int dv_mqa_prep(int dtype, const void* kv, int ldkv, const float* null_kv, void* kp,
                           void* vp, int B, int N, int NKP, void* stream) {
  DV_REQUIRE(kv && null_kv && kp && vp && NKP >= N + 1 && NKP % 32 == 0, "bad arguments");
  hipStream_t st = (hipStream_t)stream;
  const long long n = (long long)B * NKP * DH;
  if (dtype == DV_BF16)
    mqa_prep_kernel<bf16><<<grid_for(n), 256, 0, st>>>((const bf16*)kv, ldkv, null_kv, (bf16*)kp, (bf16*)vp, B, N, NKP);
  else
    mqa_prep_kernel<float><<<grid_for(n), 256, 0, st>>>((const float*)kv, ldkv, null_kv, (float*)kp, (float*)vp, B, N, NKP);
  return check_launch("mqa_prep");
}

extern "C" int dv_mqa_fwd(int dtype, const void* q, int ldq, const void* kp, const void* vp,
                          void* o, int ldo, float* lse, int B, int N, int NKP, int H, float scale,
                          void* stream) {
  DV_REQUIRE(q && kp && vp && o && lse && H % 4 == 0 && NKP % 32 == 0, "bad arguments");
  DV_REQUIRE(ldq % 8 == 0 && ldo >= H * DH, "bad strides");
  dim3 grid((N + 31) / 32, H / 4, B);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == DV_BF16)
    mqa_fwd_kernel<bf16><<<grid, 256, 0, st>>>((const bf16*)q, ldq, (const bf16*)kp, (const bf16*)vp, (bf16*)o, ldo, lse, N, NKP, N + 1, H, scale);
  else
    mqa_fwd_kernel<float><<<grid, 256, 0, st>>>((const float*)q, ldq, (const float*)kp, (const float*)vp, (float*)o, ldo, lse, N, NKP, N + 1, H, scale);
  return check_launch("mqa_fwd");
}

extern "C" int dv_mqa_bwd(int dtype, const void* q, int ldq, const void* o, int ldo,
                          const void* dout, int lddo, const float* lse, const void* kp,
                          const void* vp, void* dq, int lddq, float* D, float* dkp, float* dvp,
                          void* dkv, int lddkv, float* dnull, int B, int N, int NKP, int H,
                          float scale, int accumulate, void* stream) {
  DV_REQUIRE(q && o && dout && lse && kp && vp && dq && D && dkp && dvp && dkv && dnull, "null pointer");
  DV_REQUIRE(H % 8 == 0 && NKP % 32 == 0, "bad shape");
  hipStream_t st = (hipStream_t)stream;
  zero_f32(dkp, (long long)B * NKP * DH, st);
  zero_f32(dvp, (long long)B * NKP * DH, st);
  const int hg = 2, hpg = H / hg;
  if (dtype == DV_BF16) {
    mqa_bwd_d_kernel<bf16><<<grid_for((long long)B * N * H), 256, 0, st>>>((const bf16*)o, ldo, (const bf16*)dout, lddo, D, B, N, H);
    mqa_dq_kernel<bf16><<<dim3((N + 31) / 32, H / 4, B), 256, 0, st>>>((const bf16*)q, ldq, (const bf16*)dout, lddo, lse, D, (const bf16*)kp, (const bf16*)vp, (bf16*)dq, lddq, N, NKP, N + 1, H, scale);
    mqa_dkdv_kernel<bf16><<<dim3(NKP / 32, hg, B), 256, 0, st>>>((const bf16*)q, ldq, (const bf16*)dout, lddo, lse, D, (const bf16*)kp, (const bf16*)vp, dkp, dvp, N, NKP, N + 1, H, hpg, scale);
    mqa_finish_kernel<bf16><<<grid_for((long long)B * N * DH), 256, 0, st>>>(dkp, dvp, (bf16*)dkv, lddkv, dnull, B, N, NKP, accumulate);
  } else {
    mqa_bwd_d_kernel<float><<<grid_for((long long)B * N * H), 256, 0, st>>>((const float*)o, ldo, (const float*)dout, lddo, D, B, N, H);
    mqa_dq_kernel<float><<<dim3((N + 31) / 32, H / 4, B), 256, 0, st>>>((const float*)q, ldq, (const float*)dout, lddo, lse, D, (const float*)kp, (const float*)vp, (float*)dq, lddq, N, NKP, N + 1, H, scale);
    mqa_dkdv_kernel<float><<<dim3(NKP / 32, hg, B), 256, 0, st>>>((const float*)q, ldq, (const float*)dout, lddo, lse, D, (const float*)kp, (const float*)vp, dkp, dvp, N, NKP, N + 1, H, hpg, scale);
    mqa_finish_kernel<float><<<grid_for((long long)B * N * DH), 256, 0, st>>>(dkp, dvp, (float*)dkv, lddkv, dnull, B, N, NKP, accumulate);
  }
  return check_launch("mqa_bwd");
}
