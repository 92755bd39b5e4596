// Convolutions (1,k,k) / token linears for the Unet3D path as implicit GEMMs
// on gfx950 MFMA.  Serves nn.Conv3d at dalle2_video.py:107,170,25,537,48,
// 224-232,637 and the bias-free attention projections.
//
// Forward / dgrad: C^T[n][m] = sum_k Wp[n][k] * X_im2col[m][k]
//   A operand = packed weight rows (n), B operand = im2col pixel rows (m);
//   each lane of the 32x32 accumulator then owns one pixel and 4 consecutive
//   channels per register quad -> vector epilogue stores.
//   Tile BM(pixels) x BN(channels) x 64 B of K, 4 waves (2x2), LDS double
//   buffer with a 16-B chunk XOR swizzle (conflict-free ds_read_b128).
//   bf16: v_mfma_f32_32x32x16_bf16; f32 (parity): v_mfma_f32_32x32x2_f32.
// Wgrad: dW[co][n'] = sum_p dY[p][co] * X_im2col[p][n'], split-K over pixels,
//   operands staged pixel-major and read transposed (ds_read_b64_tr_b16),
//   f32 atomics into a packed [co][tap][ci] workspace (coalesced rows).
#include "dv_common.h"

#include <type_traits>

#include <algorithm>
#include <cstdlib>

using namespace dv;

// Diagnostic build only (make stamp): per-workgroup s_memrealtime stamps of
// a kernel's phases into a device array read back by dv_debug_stamps
// (tools/wgrad_stamp.py).  The product build compiles none of it.
#ifdef DV_STAMP
constexpr int DV_NSTAMP = 8;
__device__ unsigned long long g_dv_stamp[16384 * DV_NSTAMP];
#define DV_STAMP_AT(i)                                                                  \
  do {                                                                                  \
    if (threadIdx.x == 0) {                                                             \
      const long long blin = blockIdx.x + (long long)gridDim.x * (blockIdx.y + (long long)gridDim.y * blockIdx.z); \
      if (blin < 16384) g_dv_stamp[blin * DV_NSTAMP + (i)] = __builtin_amdgcn_s_memrealtime(); \
    }                                                                                   \
  } while (0)
extern "C" int dv_debug_stamps(unsigned long long* host, long long n) {
  if (n > 16384 * DV_NSTAMP) n = 16384 * DV_NSTAMP;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_dv_stamp), n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#else
#define DV_STAMP_AT(i) \
  do {                 \
  } while (0)
#endif
// the stripe kernel's stamps 4..7: stage 1's phases, or (DV_STAMP_PRO) the
// prologue's (7 stage 0 DMA issued, 4 all DMA issued, 5 stage 0 + weights landed,
// 6 weights in registers; tools/gn_fold_probe.py with DV_STAMP_PRO=1)
#ifdef DV_STAMP_PRO
#define DV_SP(i) DV_STAMP_AT(i)
#define DV_S1(i) do { } while (0)
#else
#define DV_SP(i) do { } while (0)
#define DV_S1(i) DV_STAMP_AT(i)
#endif

namespace {

__device__ __forceinline__ int sw_off(int row, int chunk) {
  return row * 64 + ((chunk ^ ((row >> 2) & 3)) << 4);
}

template <typename T> struct Mma;
template <> struct Mma<bf16> {
  __device__ static inline f32x16 run(u32x4 a, u32x4 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                   __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
  }
};
template <> struct Mma<float> {
  // 4 k-steps of 2: the k-slot h of step j is element 4*chunk + j on BOTH
  // operands, so the permuted k order is consistent.
  // NB (hipcc 7.2): bit-casting single elements of a u32x4 (`bit_cast<float>(a[j])`)
  // inside this unrolled loop miscompiles to element 0 for every j; cast the
  // whole vector first.
  __device__ static inline f32x16 run(u32x4 a, u32x4 b, f32x16 c) {
    const f32x4 af = __builtin_bit_cast(f32x4, a), bf = __builtin_bit_cast(f32x4, b);
#pragma unroll
    for (int j = 0; j < 4; ++j) c = __builtin_amdgcn_mfma_f32_32x32x2f32(af[j], bf[j], c, 0, 0, 0);
    return c;
  }
};

template <typename T>
struct ConvFwdArgs {
  const T* x0;
  const T* x1;
  int ld0, ld1, c0;
  const T* w;
  const float* bias;
  const T* res;
  int ldres;
  // a second residual (the unet skip gradient a dgrad adds besides the shared
  // input-gradient buffer, ops.SkipGrad); null: none.  Launchers move a lone
  // res2 into res, so res2 != null implies res != null.
  const T* res2 = nullptr;
  int ldres2 = 0;
  T* y;
  int ldy;
  int H, W, cin, cout, ks, act;
  long long M;
  int K;
  // GroupNorm statistics epilogue (Block3D: conv -> GroupNorm, dalle2_video.py:
  // 107-109): per-(clip, channel) sum / sum of squares of the STORED output
  // added into gn_sums[replica][clip][cout][2] (zero on entry; replica =
  // workgroup % gn_R, stride gn_rstride), clip = pixel / gn_P.  Null: off.
  float* gn_sums;
  long long gn_P;
  int gn_R;
  long long gn_rstride;
  // window kernel: output-channel groups the 8 XCDs split into (the other
  // factor of 8 splits the pixel tiles); 0: one channel block per XCD
  int xcd_c;
  // stripe kernel: the weight image holds wcin channels per tap (0: 64) and
  // this pass reads channels [wc0, wc0 + 64) of each tap -- one source of a
  // dual-source conv run as two passes (conv_fwd_t)
  int wcin = 0, wc0 = 0;
  // stripe kernel, W = 64: a GroupNorm (+ FiLM) + SiLU folded into the input
  // (dv_conv_fwd_gn_in).  x0 holds the GroupNorm's input z; each staged window
  // row becomes silu(A z + B) in LDS before the MFMAs read it, A / B per
  // (clip, channel) from z's statistics (gi_sums: gi_R replicas, stride
  // gi_rstride, [clip][64][2]) and gamma / beta / FiLM.  Null gi_sums: off.
  const float* gi_sums = nullptr;
  long long gi_rstride = 0, gi_P = 1;
  int gi_R = 1;
  float gi_eps = 0.f;
  const float *gi_gamma = nullptr, *gi_beta = nullptr, *gi_ss = nullptr;
  float *gi_mean = nullptr, *gi_rstd = nullptr;  // the GroupNorm's saved statistics
  T* gi_y = nullptr;                              // silu(A z + B), stored for the wgrad
  int gi_ldy = 0;
  float* gi_zero = nullptr;                       // zeroed (the next GroupNorm's sums)
  long long gi_zero_n = 0;
};

// GroupNorm statistics of a wave's tile, register-light: every lane holds
// NV = 2 * NC values v[0..NC) = its pixels' sums of channels chan(k) and
// v[NC..2NC) = their sums of squares (the same channels on all 32 lanes of a
// half-wave h = lane >> 5).  Recursive halving over the 32 lanes (offsets
// 16 .. 1, 31 shuffles for NV = 32) leaves lane r with the half-wave totals
// of value indices r * (NV / 32) + t, which it adds for clip b: NV / 32
// atomic instructions per wave, no arrays kept live across the tile loops.
template <int NV, int O>
__device__ __forceinline__ void rs_step(float (&v)[NV], int r) {
  // current segment: v[0 .. 32 * NV / (32 * O) ... ) -- see gn_rs_reduce
  constexpr int HALF = NV * O / 32;  // values kept after this step
  const bool up = (r & O) != 0;
#pragma unroll
  for (int k = 0; k < HALF; ++k) {
    const float send = up ? v[k] : v[k + HALF];
    const float keep = up ? v[k + HALF] : v[k];
    v[k] = keep + __shfl_xor(send, O, 64);
  }
}
template <int NV>
__device__ __forceinline__ void gn_rs_reduce(float (&v)[NV], int r) {
  static_assert(NV % 32 == 0, "NV must be a multiple of 32");
  rs_step<NV, 16>(v, r);  // 2 * NV / 32 * 16 = NV / 2 kept
  rs_step<NV, 8>(v, r);
  rs_step<NV, 4>(v, r);
  rs_step<NV, 2>(v, r);
  rs_step<NV, 1>(v, r);   // NV / 32 kept: value indices r * (NV / 32) + t
}
template <typename T, int NV, typename Chan>
__device__ __forceinline__ void gn_rs_add(const ConvFwdArgs<T>& p, const float (&v)[NV],
                                          long long b, Chan chan) {
  constexpr int NC = NV / 2, S = NV / 32;
  const int r = threadIdx.x & 31;
  const int blk = blockIdx.x + gridDim.x * blockIdx.y;
  float* base = p.gn_sums + (long long)(blk % p.gn_R) * p.gn_rstride + b * p.cout * 2;
#pragma unroll
  for (int t = 0; t < S; ++t) {
    const int j = r * S + t, stat = j / NC, k = j % NC;
    const int n = chan(k);
    if (n < p.cout) atomicAdd(base + 2 * n + stat, v[t]);
  }
}

// Block-level version (every wave of the workgroup calls it): the waves'
// reduce-scattered totals are combined in LDS (ds_add_f32 into red[2 * nblk],
// LDS that no wave still reads) and the workgroup adds ONE value per (channel,
// statistic) of its nblk channels [n0, n0 + nblk): device-scope float
// atomics are the expensive part (measured: 4-8x fewer of them per tile).
template <typename T, int NV, typename Chan>
__device__ __forceinline__ void gn_block_add(const ConvFwdArgs<T>& p, const float (&v)[NV],
                                             long long b, Chan chan, float* red, int n0, int nblk) {
  constexpr int NC = NV / 2, S = NV / 32;
  __syncthreads();  // red may alias LDS the main loop read
  for (int i = threadIdx.x; i < 2 * nblk; i += blockDim.x) red[i] = 0.f;
  __syncthreads();
  const int r = threadIdx.x & 31;
#pragma unroll
  for (int t = 0; t < S; ++t) {
    const int j = r * S + t, stat = j / NC, k = j % NC;
    const int n = chan(k);
    if (n < p.cout) atomicAdd(red + 2 * (n - n0) + stat, v[t]);
  }
  __syncthreads();
  const int blk = blockIdx.x + gridDim.x * blockIdx.y;
  float* base = p.gn_sums + (long long)(blk % p.gn_R) * p.gn_rstride + (b * p.cout + n0) * 2;
  for (int i = threadIdx.x; i < 2 * nblk; i += blockDim.x)
    if (n0 + i / 2 < p.cout) atomicAdd(base + i, red[i]);
}

// value as stored (the GroupNorm reads the rounded tensor)
template <typename T>
__device__ __forceinline__ float stored(float v) { return (float)(T)v; }

template <typename T>
__device__ __forceinline__ void store4(T* dst, const float* v);
template <>
__device__ __forceinline__ void store4<float>(float* dst, const float* v) {
  *(f32x4*)dst = f32x4{v[0], v[1], v[2], v[3]};
}
template <>
__device__ __forceinline__ void store4<bf16>(bf16* dst, const float* v) {
  *(bf16x4*)dst = bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
}
template <typename T>
__device__ __forceinline__ void load4(const T* src, float* v);
template <>
__device__ __forceinline__ void load4<float>(const float* src, float* v) {
  f32x4 t = *(const f32x4*)src;
  v[0] = t[0]; v[1] = t[1]; v[2] = t[2]; v[3] = t[3];
}
template <>
__device__ __forceinline__ void load4<bf16>(const bf16* src, float* v) {
  bf16x4 t = *(const bf16x4*)src;
  v[0] = (float)t[0]; v[1] = (float)t[1]; v[2] = (float)t[2]; v[3] = (float)t[3];
}

// epilogue: lane owns pixel column r of each 32-pixel tile; channels
// 8g + 4h + e of each 32-channel tile.  y = act(acc + bias) + res.
// STATS: also the GroupNorm statistics of the stored y (gn_rs_reduce) — a
// separate instantiation, so the plain epilogue keeps its register budget.
template <typename T, int TI, int TJ, bool STATS = false>
__device__ __forceinline__ void conv_epilogue(const ConvFwdArgs<T>& p, const f32x16 (&acc)[TJ][TI],
                                              long long mb, int nb, int r, int h,
                                              long long blk_m0 = 0, int blk_bm = 0, int blk_n0 = 0,
                                              int blk_bn = 0, float* red = nullptr) {
  const bool vec_ok = ((p.ldy & 3) == 0) && (p.res == nullptr || (p.ldres & 3) == 0) &&
                      (p.res2 == nullptr || (p.ldres2 & 3) == 0);
  constexpr int NC = 16 * TJ, NV = STATS ? 2 * NC : 1;
  float sv[NV];
  long long clip = 0;
  bool one_clip = true;
  if constexpr (STATS) {
#pragma unroll
    for (int k = 0; k < NV; ++k) sv[k] = 0.f;
    // the workgroup's pixel rows lie in one clip unless its tile straddles
    // clips (small shapes only: one atomic pair per element then); decided
    // per workgroup, so the block-level add below is block-uniform
    const long long last = (blk_m0 + blk_bm < p.M ? blk_m0 + blk_bm : p.M) - 1;
    clip = blk_m0 / p.gn_P;
    one_clip = last / p.gn_P == clip;
  }
  // Bias and residual of the whole tile are loaded BEFORE the first store:
  // vmcnt counts loads and stores in order, so a load issued behind a store
  // waits for that store's write (one write round trip per 4-channel group,
  // TI*TJ*4 of them per tile, when loads and stores interleaved).  Indices are
  // clamped (unconditional loads); lanes past M / cout skip the store.
  f32x4 bv[TJ][4];
  using RV = typename std::conditional<sizeof(T) == 2, u32x2, f32x4>::type;
  RV rv[TI][TJ][4], rv2[TI][TJ][4];
  if (vec_ok && p.cout >= 4) {
    if (p.bias) {
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int n = min(nb + 32 * j + 8 * g + 4 * h, p.cout - 4);
          bv[j][g] = *(const f32x4*)(p.bias + n);
        }
    }
    if (p.res) {
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const long long m = min(mb + 32 * i + r, p.M - 1);
#pragma unroll
        for (int j = 0; j < TJ; ++j)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int n = min(nb + 32 * j + 8 * g + 4 * h, p.cout - 4);
            rv[i][j][g] = *(const RV*)(p.res + m * p.ldres + n);
            if (p.res2) rv2[i][j][g] = *(const RV*)(p.res2 + m * p.ldres2 + n);
          }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < TI; ++i) {
    const long long m = mb + 32 * i + r;
    if (m >= p.M) continue;
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int n = nb + 32 * j + 8 * g + 4 * h;
        if (n >= p.cout) continue;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = acc[j][i][4 * g + e];
        if (vec_ok && n + 3 < p.cout) {
          if (p.bias) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += bv[j][g][e];
          }
          if (p.act == DV_ACT_SILU) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = silu_f(v[e]);
          }
          if (p.res) {
            float rr[4];
            if constexpr (sizeof(T) == 2) {
              const bf16x4 t4 = __builtin_bit_cast(bf16x4, rv[i][j][g]);
#pragma unroll
              for (int e = 0; e < 4; ++e) rr[e] = (float)t4[e];
            } else {
#pragma unroll
              for (int e = 0; e < 4; ++e) rr[e] = rv[i][j][g][e];
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += rr[e];
            if (p.res2) {
              if constexpr (sizeof(T) == 2) {
                const bf16x4 t4 = __builtin_bit_cast(bf16x4, rv2[i][j][g]);
#pragma unroll
                for (int e = 0; e < 4; ++e) rr[e] = (float)t4[e];
              } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) rr[e] = rv2[i][j][g][e];
              }
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] += rr[e];
            }
          }
          store4<T>(p.y + m * p.ldy + n, v);
          if constexpr (STATS) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float q = stored<T>(v[e]);
              if (one_clip) {
                sv[16 * j + 4 * g + e] += q;
                sv[NC + 16 * j + 4 * g + e] += q * q;
              } else {
                float* sb = p.gn_sums + ((m / p.gn_P) * p.cout + n + e) * 2;
                atomicAdd(sb, q);
                atomicAdd(sb + 1, q * q);
              }
            }
          }
        } else {
          for (int e = 0; e < 4 && n + e < p.cout; ++e) {
            float t = v[e] + (p.bias ? p.bias[n + e] : 0.f);
            if (p.act == DV_ACT_SILU) t = silu_f(t);
            if (p.res) t += (float)p.res[m * p.ldres + n + e];
            if (p.res2) t += (float)p.res2[m * p.ldres2 + n + e];
            p.y[m * p.ldy + n + e] = (T)t;
            if constexpr (STATS) {
              const float q = stored<T>(t);
              float* sb = p.gn_sums + ((m / p.gn_P) * p.cout + n + e) * 2;
              atomicAdd(sb, q);
              atomicAdd(sb + 1, q * q);
            }
          }
        }
      }
    }
  }
  if constexpr (STATS) {
    if (one_clip) {  // block-uniform
      gn_rs_reduce<NV>(sv, r);
      gn_block_add<T, NV>(p, sv, clip, [&](int k) {
        return nb + 32 * (k / 16) + 8 * ((k % 16) / 4) + 4 * h + (k % 4);
      }, red, blk_n0, blk_bn);
    }
  }
}

template <typename T, int BM, int BN, bool STATS = false>
__global__ __launch_bounds__(256) void conv_fwd_kernel(ConvFwdArgs<T> p) {
  constexpr int VEC = 16 / sizeof(T);
  constexpr int BK = 4 * VEC;  // K elements per 64-byte LDS row
  constexpr int TI = BM / 64;  // 32-pixel MFMA tiles per wave
  constexpr int TJ = BN / 64;  // 32-channel MFMA tiles per wave
  constexpr int LA = BM / 64;  // pixel-row vectors loaded per thread
  constexpr int LB = BN / 64;  // weight-row vectors loaded per thread
  __shared__ __attribute__((aligned(16))) char smem[2 * (BM + BN) * 64];
  char* sX = smem;
  char* sW = smem + 2 * BM * 64;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const long long m0 = (long long)blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int HW = p.H * p.W, pad = p.ks >> 1, K = p.K;
  const int chunk = tid & 3;

  int a_f[LA], a_y[LA], a_x[LA];
  bool a_ok[LA];
#pragma unroll
  for (int i = 0; i < LA; ++i) {
    long long m = m0 + (tid >> 2) + 64 * i;
    a_ok[i] = m < p.M;
    long long mm = a_ok[i] ? m : 0;
    int f = (int)(mm / HW);
    int rem = (int)(mm - (long long)f * HW);
    a_f[i] = f;
    a_y[i] = rem / p.W;
    a_x[i] = rem - a_y[i] * p.W;
  }
  // K position of this thread's vector: k = kc*BK + chunk*VEC -> (tap, ci)
  int k_tap = 0, k_ci = chunk * VEC;
  while (k_ci >= p.cin) { k_ci -= p.cin; ++k_tap; }

  u32x4 ra[LA], rb[LB];
  auto gload = [&](int kc) {
    const int k = kc * BK + chunk * VEC;
    const bool kin = k < K;
    const int dy = k_tap / p.ks - pad, dx = k_tap % p.ks - pad;
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int yy = a_y[i] + dy, xx = a_x[i] + dx;
      u32x4 v = {0u, 0u, 0u, 0u};
      if (kin && a_ok[i] && yy >= 0 && yy < p.H && xx >= 0 && xx < p.W) {
        long long pix = ((long long)a_f[i] * p.H + yy) * p.W + xx;
        const T* src = k_ci < p.c0 ? p.x0 + pix * p.ld0 + k_ci : p.x1 + pix * p.ld1 + (k_ci - p.c0);
        v = *(const u32x4*)src;
      }
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int n = n0 + (tid >> 2) + 64 * i;
      u32x4 v = {0u, 0u, 0u, 0u};
      if (kin && n < p.cout) v = *(const u32x4*)(p.w + (long long)n * K + k);
      rb[i] = v;
    }
    // advance (tap, ci) by BK for the next chunk
    k_ci += BK;
    while (k_ci >= p.cin) { k_ci -= p.cin; ++k_tap; }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < LA; ++i)
      *(u32x4*)(sX + buf * BM * 64 + sw_off((tid >> 2) + 64 * i, chunk)) = ra[i];
#pragma unroll
    for (int i = 0; i < LB; ++i)
      *(u32x4*)(sW + buf * BN * 64 + sw_off((tid >> 2) + 64 * i, chunk)) = rb[i];
  };

  f32x16 acc[TJ][TI];
#pragma unroll
  for (int j = 0; j < TJ; ++j)
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[j][i][e] = 0.f;

  const int nk = (K + BK - 1) / BK;
  const int r = lane & 31, h = lane >> 5;
  gload(0);
  lstore(0);
  __syncthreads();
  for (int kc = 0; kc < nk; ++kc) {
    const int buf = kc & 1;
    if (kc + 1 < nk) gload(kc + 1);
    const char* bx = sX + buf * BM * 64;
    const char* bw = sW + buf * BN * 64;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int c = 2 * s + h;
      u32x4 wa[TJ], xb[TI];
#pragma unroll
      for (int j = 0; j < TJ; ++j) wa[j] = *(const u32x4*)(bw + sw_off(wn * 32 * TJ + 32 * j + r, c));
#pragma unroll
      for (int i = 0; i < TI; ++i) xb[i] = *(const u32x4*)(bx + sw_off(wm * 32 * TI + 32 * i + r, c));
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int i = 0; i < TI; ++i) acc[j][i] = Mma<T>::run(wa[j], xb[i], acc[j][i]);
    }
    if (kc + 1 < nk) lstore(buf ^ 1);
    __syncthreads();
  }

  conv_epilogue<T, TI, TJ, STATS>(p, acc, m0 + wm * 32 * TI, n0 + wn * 32 * TJ, r, h, m0, BM, n0, BN,
                                  (float*)smem);
}


// ---------------------------------------------------------------------------
// bf16 forward, cin % 64 == 0: LDS-DMA (global_load_lds_dwordx4) staging,
// BK = 64 (one 128-B row per pixel / per output channel and K-tile; a K-tile
// is 64 input channels of ONE tap), two LDS buffers, one K-tile in flight
// across the raw barrier (counted vmcnt).  LDS images are lane-linear (the
// DMA writes base + lane*16); the 16-B chunk XOR swizzle is applied to the
// SOURCE address and undone on the ds_read_b128 (both sides, same involution).
// Out-of-image taps and tail pixels / channels read a zeroed 16-B line.
// Block ids are remapped so each XCD owns a contiguous pixel range (its
// im2col halos and all cout tiles of a pixel tile share that XCD's L2).
// ---------------------------------------------------------------------------
__device__ __attribute__((aligned(64))) unsigned int g_zero_line[16];
// 16 KB of zeros: DMA lanes that must load zeros from a real address (two
// sources per wave, no single raw buffer) spread over 1,024 16-B lines, i.e.
// over every L2 channel, instead of all hitting one line
__device__ __attribute__((aligned(64))) unsigned int g_zero_buf[4096];
__device__ __forceinline__ const bf16* zero_src(unsigned salt) {
  return (const bf16*)(g_zero_buf + (salt & 1023u) * 4);
}

__device__ __forceinline__ int swz8(int row) { return (row >> 1) & 7; }

template <int BM, int BN, int NBUF, bool STATS = false>
__global__ __launch_bounds__(256) void conv_fwd_glds_kernel(ConvFwdArgs<bf16> p, int tiles_n) {
  constexpr int TI = BM / 64, TJ = BN / 64;
  constexpr int GB = BM / 32, GA = BN / 32;  // DMA instructions per thread per K-tile
  constexpr int BUF = (BM + BN) * 128;
  constexpr int DPK = GA + GB;               // DMAs per thread per K-tile
  __shared__ __attribute__((aligned(1024))) char smem[NBUF * BUF];

  // XCD-aware bijective remap of the 1-D block id
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int q = nwg >> 3, rr8 = nwg & 7, xcd = orig & 7;
  const int wg = (xcd < rr8 ? xcd * (q + 1) : rr8 * (q + 1) + (xcd - rr8) * q) + (orig >> 3);
  const int tn = wg % tiles_n;
  const long long m0 = (long long)(wg / tiles_n) * BM;
  const int n0 = tn * BN;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int HW = p.H * p.W, pad = p.ks >> 1;
  const int cblocks = p.cin >> 6;
  const int chunk = lane & 7;

  // pixel rows this thread DMAs: row = 32*i + (tid >> 3).  Offsets are 32-bit
  // (the dispatcher guarantees M*ld < 2^31); invalid rows get y = -2^20 so
  // every tap of them selects the zero line.
  int b_y[GB], b_x[GB], b_pix[GB];
#pragma unroll
  for (int i = 0; i < GB; ++i) {
    const int row = 32 * i + (tid >> 3);
    const long long m = m0 + row;
    const bool ok = m < p.M;
    const int mi = ok ? (int)m : 0;
    const int f = mi / HW;
    const int rem = mi - f * HW;
    const int y = rem / p.W;
    b_y[i] = ok ? y : -(1 << 20);
    b_x[i] = rem - y * p.W;
    b_pix[i] = mi;
  }
  const int a_rowoff = (tid >> 3);
  // per-workgroup raw buffers over the pixels any tap of this tile can read
  // and over this tile's weight rows: out-of-image taps, tail pixels and rows
  // past cout load out of range (zeros without a memory access) instead of
  // all hitting one shared zero line (a hot L2 channel)
  const int reach = pad * p.W + pad;
  const long long plo = m0 - reach > 0 ? m0 - reach : 0;
  const long long phi = m0 + BM + reach < p.M ? m0 + BM + reach : p.M;
  const __amdgpu_buffer_rsrc_t xr0 = dma_rsrc(p.x0 + plo * p.ld0, (unsigned)((phi - plo) * p.ld0 * 2));
  const __amdgpu_buffer_rsrc_t xr1 = dma_rsrc(p.x1 + plo * p.ld1, (unsigned)((phi - plo) * p.ld1 * 2));
  const int nrows = p.cout - n0 < BN ? p.cout - n0 : BN;
  const __amdgpu_buffer_rsrc_t wr = dma_rsrc(p.w + (long long)n0 * p.K, (unsigned)(nrows * p.K * 2));
  const int poff = (int)(-plo);

  // per-row DMA state, computed once: the row pixel's byte offset in each
  // source (relative to the raw buffer base plo, with the row's swizzled
  // chunk) and the mask of the taps whose input pixel is inside the frame;
  // per K-tile each DMA then adds one uniform tap offset (no multiply and no
  // exec-masked block per DMA: 10+ VALU per DMA before), and the weight DMAs
  // take the K-tile offset in the instruction's soffset (no VALU at all)
  unsigned rb0[GB], rb1[GB], tmask[GB], ab[GA];
#pragma unroll
  for (int i = 0; i < GB; ++i) {
    const int row = 32 * i + (tid >> 3);
    const int cs = chunk ^ swz8(row);
    rb0[i] = (unsigned)(((b_pix[i] + poff) * p.ld0 + cs * 8) * 2);
    rb1[i] = (unsigned)(((b_pix[i] + poff) * p.ld1 + cs * 8) * 2);
    // ks is 1 or 3 (host-checked); tap t = 3 (dy + 1) + dx + 1
    const int y = b_y[i], x = b_x[i];
    const unsigned H = (unsigned)p.H, Wd = (unsigned)p.W;
    if (p.ks == 1) {
      tmask[i] = (unsigned)y < H ? 1u : 0u;
    } else {
      const unsigned ym = ((unsigned)(y - 1) < H ? 1u : 0u) | ((unsigned)y < H ? 2u : 0u) |
                          ((unsigned)(y + 1) < H ? 4u : 0u);
      const unsigned xm = ((unsigned)(x - 1) < Wd ? 1u : 0u) | 2u | ((unsigned)(x + 1) < Wd ? 4u : 0u);
      tmask[i] = ((ym & 1u) ? xm : 0u) | ((ym & 2u) ? xm << 3 : 0u) | ((ym & 4u) ? xm << 6 : 0u);
    }
  }
#pragma unroll
  for (int i = 0; i < GA; ++i) {
    const int row = 32 * i + a_rowoff;
    ab[i] = (unsigned)((row * p.K + (chunk ^ swz8(row)) * 8) * 2);
  }

  auto issue = [&](int kt, int buf) {
    const int tap = kt / cblocks;
    const int ci = ((kt - tap * cblocks) << 6);
    const int dy = tap / p.ks - pad, dx = tap % p.ks - pad;
    const bool first = ci < p.c0;  // wave-uniform: the 64-channel block never straddles c0
    const int cof = first ? ci : ci - p.c0;
    const int ld = first ? p.ld0 : p.ld1;
    const unsigned toff = (unsigned)(((dy * p.W + dx) * ld + cof) * 2);  // mod 2^32 (dy, dx < 0)
    char* sB = smem + buf * BUF;
    char* sA = sB + BM * 128;
#pragma unroll
    for (int i = 0; i < GB; ++i) {
      const bool in = (tmask[i] >> tap) & 1u;
      const unsigned voff = in ? (first ? rb0[i] : rb1[i]) + toff : DMA_OOB;
      dma16(first ? xr0 : xr1, sB + (32 * i + 8 * wave) * 128, voff);
    }
#pragma unroll
    for (int i = 0; i < GA; ++i) dma16s(wr, sA + (32 * i + 8 * wave) * 128, ab[i], (unsigned)kt * 128);
  };

  f32x16 acc[TJ][TI];
#pragma unroll
  for (int j = 0; j < TJ; ++j)
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[j][i][e] = 0.f;

  const int r = lane & 31, h = lane >> 5;
  const int nk = (p.K >> 6);
  // NBUF-deep ring, NBUF - 1 K-tiles in flight (deep rings when few
  // workgroups share a CU: the load latency is then hidden by prefetch
  // distance instead of by other workgroups)
#pragma unroll
  for (int i = 0; i < NBUF - 1; ++i)
    if (i < nk) issue(i, i);
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt % NBUF;
    const int ahead = nk - 1 - kt;  // K-tiles issued after this one (before the new issue)
    if (ahead >= NBUF - 1) {
      issue(kt + NBUF - 1, (kt + NBUF - 1) % NBUF);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DPK * (NBUF - 1)) : "memory");
    } else if (NBUF >= 5 && ahead >= 4) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DPK * 4) : "memory");
    } else if (NBUF >= 4 && ahead >= 3) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DPK * 3) : "memory");
    } else if (NBUF >= 3 && ahead >= 2) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DPK * 2) : "memory");
    } else if (ahead >= 1) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DPK) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    const char* sB = smem + buf * BUF;
    const char* sA = sB + BM * 128;
    // fragments of k-step s + 1 are read before the MFMAs of k-step s (with
    // the reads issued just ahead of their own MFMAs every k-step exposed the
    // LDS latency)
    u32x4 wa[2][TJ], xb[2][TI];
    auto rd = [&](int s, int sl) {
      const int c = 2 * s + h;
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int row = wn * 32 * TJ + 32 * j + r;
        wa[sl][j] = *(const u32x4*)(sA + row * 128 + ((c ^ swz8(row)) << 4));
      }
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const int row = wm * 32 * TI + 32 * i + r;
        xb[sl][i] = *(const u32x4*)(sB + row * 128 + ((c ^ swz8(row)) << 4));
      }
    };
    rd(0, 0);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      if (s + 1 < 4) rd(s + 1, (s + 1) & 1);
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int i = 0; i < TI; ++i) acc[j][i] = Mma<bf16>::run(wa[s & 1][j], xb[s & 1][i], acc[j][i]);
      __builtin_amdgcn_sched_barrier(0);
    }
    // every wave's reads of `buf` are done before the next iteration re-fills it
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  conv_epilogue<bf16, TI, TJ, STATS>(p, acc, m0 + wm * 32 * TI, n0 + wn * 32 * TJ, r, h, m0, BM, n0, BN,
                                     (float*)smem);
}

// ---------------------------------------------------------------------------
// bf16 1x1 convolution with K = 64 * KT <= 128 input channels and cout = BN
// (64 or 128): the res_conv / skip 1x1s of the 64x64 stage and their dgrads
// (accumulated into the shared dX).  HBM-bound (≈ 85-170 flop/B), so the
// shape of the glds kernel — one tile per workgroup, load / compute / store
// in sequence — leaves the memory idle between phases.  Here a persistent
// workgroup keeps the weights LDS-resident, streams 128-pixel tiles through
// an NB-deep LDS-DMA ring (NB - 1 tiles in flight) and prefetches the next
// tile's residual into registers while this tile computes; one counted
// vmcnt per tile, every DMA issued unconditionally (tiles past the end read
// the zero line) so the count is a constant.
// 8 waves = 4 pixel groups of 32 x 2 channel halves of BN / 2.
// The residual loads are inline asm: hipcc cannot count them against the
// LDS-DMA queue and drained it (vmcnt(0)) at every tile, twice, when they were
// compiler-visible.  Two register sets alternate (the loop is unrolled by two)
// so a prefetched residual is never copied before it lands, and the
// top-of-tile wait is tied to the set it releases.
// ---------------------------------------------------------------------------
__device__ __forceinline__ u32x2 gload_b64_asm(const void* ptr) {
  u32x2 v;
  asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(v) : "v"(ptr) : "memory");
  return v;
}
template <int N, int R>
__device__ __forceinline__ void vm_wait_tied(u32x2 (&v)[R]) {
  static_assert(R == 1 || R == 4 || R == 8, "residual sets of 1 / 4 / 8");
  if constexpr (R == 8)
    asm volatile("s_waitcnt vmcnt(%8)"
                 : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7])
                 : "n"(N) : "memory");
  else if constexpr (R == 4)
    asm volatile("s_waitcnt vmcnt(%4)" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]) : "n"(N) : "memory");
  else
    asm volatile("s_waitcnt vmcnt(%1)" : "+v"(v[0]) : "n"(N) : "memory");
}
// RLDS (where the ring still fits the LDS): the residual tile rides in the
// ring beside the X tile, by the same LDS-DMA (1-KB coalesced pieces, 16-B
// chunks swizzled by row), and the epilogue reads it from LDS -- instead of
// per-lane 8-B register loads (32 rows x 16 B per instruction).
template <int BN, int KT, int NB, bool RES>
__global__ __launch_bounds__(512) void conv1x1_stream_kernel(ConvFwdArgs<bf16> p, int ntiles) {
  constexpr int BM = 128;
  constexpr int XT = BM * 128 * KT;  // one pixel tile: KT 64-channel blocks of 128-B rows
  constexpr int WBYTES = BN * 128 * KT;
  constexpr int RT = BM * BN * 2;    // one residual tile: 128 rows of BN bf16
  constexpr bool RLDS = RES && WBYTES + NB * (XT + RT) <= 160 * 1024;
  constexpr int TJ = BN / 64;        // 32-channel MFMA tiles per wave
  constexpr int XD = 2 * KT;         // X-tile DMA instructions per thread (64 rows per round)
  constexpr int WD = BN * KT / 64;   // weight DMA instructions per thread
  constexpr int RD = RLDS ? RT / (512 * 16) : 0;        // residual DMA instructions per thread
  constexpr int RL = RES && !RLDS ? 4 * TJ : 0;         // residual register loads per thread per tile
  constexpr int SLOT = XT + (RLDS ? RT : 0);            // one ring slot: X tile (+ residual tile)
  constexpr int CPR = BN / 8;                           // 16-B chunks per residual row
  __shared__ __attribute__((aligned(1024))) char smem[WBYTES + NB * SLOT];
  char* sW = smem;
  char* sX = smem + WBYTES;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int r = lane & 31, h = lane >> 5;
  const int chunk = lane & 7, rrow = tid >> 3;  // DMA slot: row rrow (0..63) of a round, 16-B chunk

  auto issue_x = [&](int t, int buf) {  // tile t (>= ntiles: zeros) into ring slot buf
    const long long m0 = (long long)t * BM;
#pragma unroll
    for (int i = 0; i < XD; ++i) {
      const int kb = i / 2, row = 64 * (i % 2) + rrow;
      const int cs = chunk ^ swz8(row);
      const long long m = m0 + row;
      const bool first = kb * 64 < p.c0;
      const bf16* src = (t < ntiles && m < p.M)
                            ? (first ? p.x0 + m * p.ld0 + kb * 64 : p.x1 + m * p.ld1 + (kb * 64 - p.c0)) + cs * 8
                            : zero_src(tid + 97u * blockIdx.x + 31u * i);
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(sX + buf * SLOT + kb * (BM * 128) +
                                                                               (64 * (i % 2) + 8 * wave) * 128),
                                       16, 0, 0);
    }
    if constexpr (RLDS) {  // the residual tile: slot q = i * 512 + tid -> row q / CPR, chunk q % CPR
#pragma unroll
      for (int i = 0; i < RD; ++i) {
        const int q = i * 512 + tid, row = q / CPR, cs = (q % CPR) ^ (row % CPR);
        const long long m = m0 + row;
        const bf16* src = (t < ntiles && m < p.M) ? p.res + m * p.ldres + cs * 8
                                                  : zero_src(tid + 89u * blockIdx.x + 37u * i);
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                         (__attribute__((address_space(3))) void*)(sX + buf * SLOT + XT +
                                                                                 (i * 512 + 64 * wave) * 16),
                                         16, 0, 0);
      }
    }
  };
  // residual of this lane's outputs (pixel row r of group wm, channels n0 + 8g + 4h .. +3)
  constexpr int NR = RES && !RLDS ? 4 * TJ : 1;
  u32x2 resA[NR], resB[NR];
  auto load_res = [&](int t, u32x2 (&dst)[NR]) {
    if constexpr (RES && !RLDS) {
      long long m = (long long)t * BM + wm * 32 + r;
      if (t >= ntiles || m >= p.M) m = 0;  // a valid address; the value is not stored
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int n = wn * (BN / 2) + 32 * j + 8 * g + 4 * h;
          dst[4 * j + g] = gload_b64_asm(p.res + m * p.ldres + n);
        }
    }
  };

  // ---- prologue: weights, NB - 1 tiles, the first residual ----
#pragma unroll
  for (int i = 0; i < WD; ++i) {
    const int q = i * 512 + tid;  // 16-B chunk index over [kb][co][8]
    const int kb = q / (BN * 8), rem = q - kb * BN * 8;
    const int co = rem >> 3, c = rem & 7;
    const bf16* src = p.w + (long long)co * p.K + kb * 64 + ((c ^ swz8(co)) << 3);
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)(sW + (long long)(i * 512 + 64 * wave) * 16),
                                     16, 0, 0);
  }
  // issue order (vmcnt is in order): prologue W, X(0 .. NB-3), res(0), X(NB-2);
  // iteration k: res(k+1), X(k+NB-1).  After res(k) come exactly X(k+NB-2),
  // res(k+1), X(k+NB-1), so vmcnt(2 XD + RL) means res(k) — and X(k), issued
  // before it (NB >= 3) — landed, with two X tiles still in flight.  (RLDS:
  // X(k) carries its residual tile, RD more pieces per tile: 2 (XD + RD).)
  static_assert(NB >= 3, "the ring needs two tiles in flight");
  int t = blockIdx.x;
#pragma unroll
  for (int i = 0; i < NB - 2; ++i) issue_x(t + i * (int)gridDim.x, i);
  load_res(t, resA);
  issue_x(t + (NB - 2) * (int)gridDim.x, NB - 2);

  float bias[TJ][4][4];
#pragma unroll
  for (int j = 0; j < TJ; ++j)
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int n = wn * (BN / 2) + 32 * j + 8 * g + 4 * h + e;
        bias[j][g][e] = p.bias ? p.bias[n] : 0.f;
      }

  // one tile: its residual in `rcur` (prefetched a tile ago), the next tile's into `rnxt`
  auto tile = [&](int it, u32x2 (&rcur)[NR], u32x2 (&rnxt)[NR]) {
    const int buf = it % NB;
    load_res(t + (int)gridDim.x, rnxt);
    issue_x(t + (NB - 1) * (int)gridDim.x, (it + NB - 1) % NB);
    if constexpr (RES && !RLDS) vm_wait_tied<2 * XD + RL>(rcur);
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (XD + RD) + RL) : "memory");
    __builtin_amdgcn_s_barrier();
    f32x16 acc[TJ];
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;
    const char* xs = sX + buf * SLOT;
#pragma unroll
    for (int kb = 0; kb < KT; ++kb)
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int c = 2 * s + h;
        const int xrow = wm * 32 + r;
        const u32x4 xb = *(const u32x4*)(xs + kb * (BM * 128) + xrow * 128 + ((c ^ swz8(xrow)) << 4));
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          const int wrow = wn * (BN / 2) + 32 * j + r;
          const u32x4 wa = *(const u32x4*)(sW + kb * (BN * 128) + wrow * 128 + ((c ^ swz8(wrow)) << 4));
          acc[j] = Mma<bf16>::run(wa, xb, acc[j]);
        }
      }
    // epilogue: D[co][px] — lane: pixel r, channels 8g + 4h + e of each 32-channel tile
    const long long m = (long long)t * BM + wm * 32 + r;
    if (m < p.M) {
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int n = wn * (BN / 2) + 32 * j + 8 * g + 4 * h;
          float v[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] = acc[j][4 * g + e] + bias[j][g][e];
            if (p.act == DV_ACT_SILU) v[e] = silu_f(v[e]);
          }
          if constexpr (RLDS) {
            const int row = wm * 32 + r, c16 = n >> 3;
            const bf16x4 rv = *(const bf16x4*)(xs + XT + row * (BN * 2) + ((c16 ^ (row % CPR)) << 4) + (n & 7) * 2);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += (float)rv[e];
          } else if constexpr (RES) {
            const bf16x4 rv = __builtin_bit_cast(bf16x4, rcur[4 * j + g]);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += (float)rv[e];
          }
          store4<bf16>(p.y + m * p.ldy + n, v);
        }
    }
    // every wave's reads of `buf` are done before the next iteration re-fills it
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };
  for (int it = 0; t < ntiles;) {
    tile(it, resA, resB);
    ++it;
    t += gridDim.x;
    if (t >= ntiles) break;
    tile(it, resB, resA);
    ++it;
    t += gridDim.x;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the ring's trailing DMAs and residual loads drain
}

// ---------------------------------------------------------------------------
// wgrad
// ---------------------------------------------------------------------------
template <typename T>
struct WgradArgs {
  const T* dy;
  int lddy;
  const T* x0;
  const T* x1;
  int ld0, ld1, c0;
  float* ws;  // packed [cout][K]
  float* db;  // optional: db[co] += sum_p dY[p][co] (blocks with blockIdx.y == 0)
  int H, W, cin, cout, ks, K;
  long long M;
  int pix_per_split;
  // batched mode (1x1 only): pixels form nbatch groups of batch_pix; each
  // group reduces into its own ws + g*ws_bstride (splits never straddle groups)
  long long batch_pix, ws_bstride;
  int splits_per_batch;
};

// transposed 4x16 bf16 block read (gfx950 ds_read_b64_tr_b16)
__device__ __forceinline__ s16x4 tr_read(const char* lds_addr) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(lds_addr));
}
// LDS byte address (32-bit) of a shared-memory pointer, and a transposed read
// at base + a compile-time offset (the ds_read's immediate field)
typedef __attribute__((address_space(3))) char lds_char;
__device__ __forceinline__ unsigned lds_u32(const char* p) {
  return (unsigned)(size_t)(const lds_char*)p;
}
__device__ __forceinline__ s16x4 tr_read_at(unsigned base, int off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)((lds_char*)(size_t)base + off));
}

// ds_read_b64_tr_b16 at base + OFF outside hipcc's waitcnt tracking; the
// caller waits with a counted lgkmcnt tied to the result.  Why: hipcc drains
// vmcnt(0) before every ds_read_b64_tr_b16 it can see while an LDS-DMA is in
// flight (it cannot tell ring buffers apart; a plain ds_read_b128 does not get
// the drain), which serialises a DMA ring with the MFMAs that read it.
template <int OFF>
__device__ __forceinline__ u32x2 tr_read_asm(unsigned base) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset is 16 bits");
  u32x2 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(base), "n"(OFF));
  return r;
}

template <typename T, int BMC, int BNK>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(WgradArgs<T> p) {
  constexpr int VEC = 16 / sizeof(T);
  constexpr int BP = 32;                              // pixels per K chunk
  constexpr int SA = BMC * (int)sizeof(T) + 64;       // padded LDS row strides
  constexpr int SB = BNK * (int)sizeof(T) + 64;
  constexpr int TJ = BMC / 64, TI = BNK / 64;         // 2x2 waves
  constexpr int VA = BMC / VEC, VB = BNK / VEC;       // vectors per LDS row
  constexpr int LA = BP * VA / 256, LB = BP * VB / 256;
  static_assert(LA >= 1 && LB >= 1, "tile too small");
  __shared__ __attribute__((aligned(16))) char smem[BP * (SA + SB)];
  char* sA = smem;
  char* sB = smem + BP * SA;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int co0 = blockIdx.x * BMC, nk0 = blockIdx.y * BNK;
  long long pbeg, pend;
  float* wsb = p.ws;
  if (p.batch_pix > 0) {
    const int bi = blockIdx.z / p.splits_per_batch, lz = blockIdx.z % p.splits_per_batch;
    pbeg = bi * p.batch_pix + (long long)lz * p.pix_per_split;
    pend = pbeg + p.pix_per_split;
    if (pend > (bi + 1) * p.batch_pix) pend = (bi + 1) * p.batch_pix;
    wsb = p.ws + bi * p.ws_bstride;
  } else {
    pbeg = (long long)blockIdx.z * p.pix_per_split;
    pend = pbeg + p.pix_per_split;
    if (pend > p.M) pend = p.M;
  }
  const int HW = p.H * p.W, pad = p.ks >> 1;

  // fixed column per thread for A (co) and B (tap, ci)
  const int a_col = (tid % VA) * VEC;
  const int b_col = (tid % VB) * VEC;
  const int b_n = nk0 + b_col;
  const bool b_nok = b_n < p.K;
  const int b_tap = b_nok ? b_n / p.cin : 0;
  const int b_ci = b_n - b_tap * p.cin;
  const int b_dy = b_tap / p.ks - pad, b_dx = b_tap % p.ks - pad;
  const bool a_cok = co0 + a_col < p.cout;

  f32x16 acc[TJ][TI];
#pragma unroll
  for (int j = 0; j < TJ; ++j)
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[j][i][e] = 0.f;

  const int r = lane & 31, h = lane >> 5;
  const bool do_bias = p.db != nullptr && blockIdx.y == 0;
  float bsum[VEC];
#pragma unroll
  for (int e = 0; e < VEC; ++e) bsum[e] = 0.f;
  u32x4 ra[LA], rb[LB];
  auto gload = [&](long long pb) {
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int row = tid / VA + (256 / VA) * i;
      const long long m = pb + row;
      u32x4 v = {0u, 0u, 0u, 0u};
      if (m < pend && a_cok) v = *(const u32x4*)(p.dy + m * p.lddy + co0 + a_col);
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int row = tid / VB + (256 / VB) * i;
      const long long m = pb + row;
      u32x4 v = {0u, 0u, 0u, 0u};
      if (m < pend && b_nok) {
        const int f = (int)(m / HW);
        const int rem = (int)(m - (long long)f * HW);
        const int y = rem / p.W, x = rem - (rem / p.W) * p.W;
        const int yy = y + b_dy, xx = x + b_dx;
        if (yy >= 0 && yy < p.H && xx >= 0 && xx < p.W) {
          const long long pix = ((long long)f * p.H + yy) * p.W + xx;
          const T* src = b_ci < p.c0 ? p.x0 + pix * p.ld0 + b_ci : p.x1 + pix * p.ld1 + (b_ci - p.c0);
          v = *(const u32x4*)src;
        }
      }
      rb[i] = v;
    }
  };
  auto lstore = [&]() {
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int row = tid / VA + (256 / VA) * i;
      *(u32x4*)(sA + row * SA + a_col * (int)sizeof(T)) = ra[i];
      if (do_bias) {
        float t[VEC];
        Vec<T>::to_f(ra[i], t);
#pragma unroll
        for (int e = 0; e < VEC; ++e) bsum[e] += t[e];
      }
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int row = tid / VB + (256 / VB) * i;
      *(u32x4*)(sB + row * SB + b_col * (int)sizeof(T)) = rb[i];
    }
  };

  if (pbeg < pend) gload(pbeg);
  for (long long pb = pbeg; pb < pend; pb += BP) {
    __syncthreads();  // previous chunk's LDS reads done
    lstore();
    __syncthreads();
    if (pb + BP < pend) gload(pb + BP);  // next chunk in flight under the MFMAs
    if constexpr (sizeof(T) == 2) {
      const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int R0 = 16 * s + 8 * (g >> 1);
        u32x4 fa[TJ], fb[TI];
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          const int C0 = wm * 32 * TJ + 32 * j + 16 * (g & 1);
          s16x4 lo = tr_read(sA + (R0 + q) * SA + (C0 + 4 * pp) * 2);
          s16x4 hi = tr_read(sA + (R0 + 4 + q) * SA + (C0 + 4 * pp) * 2);
          u32x2 l2 = __builtin_bit_cast(u32x2, lo), h2 = __builtin_bit_cast(u32x2, hi);
          fa[j] = u32x4{l2[0], l2[1], h2[0], h2[1]};
        }
#pragma unroll
        for (int i = 0; i < TI; ++i) {
          const int C0 = wn * 32 * TI + 32 * i + 16 * (g & 1);
          s16x4 lo = tr_read(sB + (R0 + q) * SB + (C0 + 4 * pp) * 2);
          s16x4 hi = tr_read(sB + (R0 + 4 + q) * SB + (C0 + 4 * pp) * 2);
          u32x2 l2 = __builtin_bit_cast(u32x2, lo), h2 = __builtin_bit_cast(u32x2, hi);
          fb[i] = u32x4{l2[0], l2[1], h2[0], h2[1]};
        }
#pragma unroll
        for (int j = 0; j < TJ; ++j)
#pragma unroll
          for (int i = 0; i < TI; ++i) acc[j][i] = Mma<bf16>::run(fa[j], fb[i], acc[j][i]);
      }
    } else {
#pragma unroll 4
      for (int s = 0; s < BP / 2; ++s) {
        const int row = 2 * s + h;
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          const float a = *(const float*)(sA + row * SA + (wm * 32 * TJ + 32 * j + r) * 4);
#pragma unroll
          for (int i = 0; i < TI; ++i) {
            const float b = *(const float*)(sB + row * SB + (wn * 32 * TI + 32 * i + r) * 4);
            acc[j][i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[j][i], 0, 0, 0);
          }
        }
      }
    }
  }

  if (do_bias) {  // reduce the column sums of the threads sharing a_col
    float* red = (float*)smem;
    __syncthreads();
#pragma unroll
    for (int e = 0; e < VEC; ++e) red[tid * VEC + e] = bsum[e];
    __syncthreads();
    if (tid < VA && a_cok) {
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        float t = 0.f;
        for (int k = 0; k < 256 / VA; ++k) t += red[(tid + k * VA) * VEC + e];
        if (co0 + a_col + e < p.cout) atomicAdd(p.db + co0 + a_col + e, t);
      }
    }
  }
  // acc[j][i]: row co = (reg&3) + 8*(reg>>2) + 4h, column n' = r
#pragma unroll
  for (int j = 0; j < TJ; ++j)
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      const int n = nk0 + wn * 32 * TI + 32 * i + r;
      if (n >= p.K) continue;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int co = co0 + wm * 32 * TJ + 32 * j + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (co < p.cout) atomicAdd(wsb + (long long)co * p.K + n, acc[j][i][e]);
      }
    }
}

// ---------------------------------------------------------------------------
// bf16 wgrad on LDS-DMA staging.  Stage = 64 pixels; the A image (dY rows,
// BMC channels) and the B image (im2col rows, BNK columns of (tap, ci)) are
// pixel-major and read transposed (ds_read_b64_tr_b16) as MFMA operands.
// Each lane DMAs a FIXED 16-B chunk column of every row it stages (the chunk
// XOR of a row depends only on row & 3 or (row >> 1) & 1), so its (tap, ci)
// and source pointer are loop-invariant; per-row im2col coordinates come from
// magic-number division.  The bias gradient rides on the MFMA: waves of the
// blockIdx.y == 0 column multiply the dY fragments by a ones fragment.
// ---------------------------------------------------------------------------
struct FastDiv {
  unsigned m;
  int s1, s2;
  unsigned d;
};
inline FastDiv make_fastdiv(unsigned d) {
  FastDiv f;
  int l = 0;
  while ((1ull << l) < d) ++l;
  f.m = (unsigned)(((1ull << 32) * ((1ull << l) - d)) / d + 1);
  f.s1 = l < 1 ? l : 1;
  f.s2 = l > 1 ? l - 1 : 0;
  f.d = d;
  return f;
}
__device__ __forceinline__ unsigned fdiv(unsigned n, const FastDiv& f) {
  const unsigned t = __umulhi(n, f.m);
  return (t + ((n - t) >> f.s1)) >> f.s2;
}

struct WgradGArgs {
  const bf16* dy;
  int lddy;
  const bf16* x0;
  const bf16* x1;
  int ld0, ld1, c0;
  float* ws;
  float* db;
  int H, W, cin, cout, ks, K;
  int M;  // pixels (< 2^31, checked)
  int pix_per_split;
  int batch_pix, splits_per_batch;
  long long ws_bstride;
  FastDiv fd_hw, fd_w, fd_cin, fd_ks;
  // ngemm > 1: grid z holds ngemm same-shape 1x1 problems of zper blocks each,
  // problem g reading mdy[g] / mx[g] and adding into mws[g]
  int ngemm, zper;
  const bf16* mdy[3];
  const bf16* mx[3];
  int mlddy[3], mld[3];
  float* mws[3];
};

// byte offset of 16-B chunk `ch` of `row` in an image with RB-byte rows
template <int RB>
__device__ __forceinline__ int img_off(int row, int ch) {
  const int x = RB == 128 ? (((row >> 1) & 1) << 2) : ((row & 3) << 2);
  return row * RB + ((ch ^ x) << 4);
}

// K1: 1x1 (ks == 1: the 1x1 wgrads and the batched token GEMMs) -- a B row is
// the pixel itself, so the per-DMA (frame, row, column) divisions and the
// window bounds test drop out of the stage loop (PMC: 31-36 VALU per MFMA)
template <int BMC, int BNK, bool K1>
__global__ __launch_bounds__(256) void conv_wgrad_glds_kernel(WgradGArgs p) {
  constexpr int BP = 64;
  constexpr int RA = BMC * 2, RB = BNK * 2;  // row bytes
  constexpr int RPI_A = 1024 / RA, RPI_B = 1024 / RB;  // rows per wave-instruction
  constexpr int GA = BP / (4 * RPI_A), GB = BP / (4 * RPI_B);  // DMAs per thread per stage
  constexpr int BUF = BP * (RA + RB);
  constexpr int WM = BMC / 64, WN = 4 / WM;  // wave grid
  constexpr int TJ = 2, TI = BNK / (32 * WN);  // 32x32 tiles per wave
  static_assert(TI >= 1, "tile");
  __shared__ __attribute__((aligned(1024))) char smem[2 * BUF];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int co0 = blockIdx.x * BMC, nk0 = blockIdx.y * BNK;
  int pbeg, pend, bz = blockIdx.z;
  float* wsb = p.ws;
  const bf16 *pdy = p.dy, *px0 = p.x0, *px1 = p.x1;
  int lddy = p.lddy, ld0 = p.ld0, ld1 = p.ld1;
  if (p.ngemm > 1) {
    const int gi = bz / p.zper;
    bz -= gi * p.zper;
    pdy = p.mdy[gi]; px0 = px1 = p.mx[gi]; wsb = p.mws[gi];
    lddy = p.mlddy[gi]; ld0 = ld1 = p.mld[gi];
  }
  if (p.batch_pix > 0) {
    const int bi = bz / p.splits_per_batch, lz = bz % p.splits_per_batch;
    pbeg = bi * p.batch_pix + lz * p.pix_per_split;
    pend = min(pbeg + p.pix_per_split, (bi + 1) * p.batch_pix);
    wsb += bi * p.ws_bstride;
  } else {
    pbeg = bz * p.pix_per_split;
    pend = min(pbeg + p.pix_per_split, p.M);
  }
  const int pad = p.ks >> 1;

  // A: this lane's fixed chunk column (channels co0 + 8*cha .. +7)
  const int a_lrow = lane / (RA / 16), a_slot = lane % (RA / 16);
  // rows this lane stages are a_row0 + 4*RPI_A*i: same XOR for all of them
  const int a_row0 = wave * RPI_A + a_lrow;
  const int a_x = RA == 128 ? (((a_row0 >> 1) & 1) << 2) : ((a_row0 & 3) << 2);
  const int cha = a_slot ^ a_x;
  const bool a_ok = co0 + 8 * cha < p.cout;
  const bf16* a_src = pdy + co0 + 8 * cha;
  // B: fixed chunk column -> (tap, ci)
  const int b_lrow = lane / (RB / 16), b_slot = lane % (RB / 16);
  const int b_row0 = wave * RPI_B + b_lrow;
  const int b_x = RB == 128 ? (((b_row0 >> 1) & 1) << 2) : ((b_row0 & 3) << 2);
  const int chb = b_slot ^ b_x;
  const int n = nk0 + 8 * chb;
  const bool b_ok = n < p.K;
  const int tap = K1 ? 0 : (b_ok ? (int)fdiv((unsigned)n, p.fd_cin) : 0);
  const int ci = n - tap * p.cin;
  const int ty = K1 ? 0 : (b_ok ? (int)fdiv((unsigned)tap, p.fd_ks) : 0);
  const int dy = K1 ? 0 : ty - pad, dx = K1 ? 0 : tap - ty * p.ks - pad;
  const bool first = ci < p.c0;
  const bf16* b_src = first ? px0 + ci : px1 + (ci - p.c0);
  const int b_ld = first ? ld0 : ld1;
  const int doff = dy * p.W + dx;

  auto issue = [&](int pb, int buf) {
    char* sA = smem + buf * BUF;
    char* sB = sA + BP * RA;
#pragma unroll
    for (int i = 0; i < GA; ++i) {
      const int row = (4 * i + wave) * RPI_A + a_lrow;
      const int m = pb + row;
      const bf16* src = (a_ok && m < pend) ? a_src + m * lddy : zero_src(tid + 97u * blockIdx.x + 31u * i);
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(sA + (4 * i + wave) * 1024),
                                       16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < GB; ++i) {
      const int row = (4 * i + wave) * RPI_B + b_lrow;
      const int m = pb + row;
      bool in = b_ok && m < pend;
      if (!K1) {
        const int f = (int)fdiv((unsigned)m, p.fd_hw);
        const int rem = m - f * p.H * p.W;
        const int y = (int)fdiv((unsigned)rem, p.fd_w);
        const int xx = rem - y * p.W + dx, yy = y + dy;
        in = in && (unsigned)yy < (unsigned)p.H && (unsigned)xx < (unsigned)p.W;
      }
      const bf16* src = in ? b_src + (m + doff) * b_ld : zero_src(tid + 97u * blockIdx.x + 31u * i + 512u);
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(sB + (4 * i + wave) * 1024),
                                       16, 0, 0);
    }
  };

  f32x16 acc[TJ][TI], accb[TJ];
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[j][i][e] = 0.f;
#pragma unroll
    for (int e = 0; e < 16; ++e) accb[j][e] = 0.f;
  }
  const bool do_bias = p.db != nullptr && blockIdx.y == 0 && wn == 0;  // wave-uniform
  const u32x4 ones = {0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u};  // bf16 1.0 x8

  const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  const int nst = (pend - pbeg + BP - 1) / BP;
  if (nst > 0) issue(pbeg, 0);
  for (int st = 0; st < nst; ++st) {
    const int buf = st & 1;
    if (st + 1 < nst) {
      issue(pbeg + (st + 1) * BP, buf ^ 1);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GA + GB) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    const char* sA = smem + buf * BUF;
    const char* sB = sA + BP * RA;
    // operand bases of k-step 0 (row R0 = 8 (g >> 1) + q; the swizzle of rows
    // R0 + 16 s and + 4 equals row R0's, so k-step s and the high half are
    // immediate offsets 16 s RA (RB) and 4 RA (RB)); asm reads, counted waits
    unsigned abase[TJ], bbase[TI];
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int C0 = wm * 64 + 32 * j + 16 * (g & 1) + 4 * pp;  // element column
      abase[j] = lds_u32(sA) + img_off<RA>(8 * (g >> 1) + q, C0 >> 3) + (C0 & 7) * 2;
    }
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      const int C0 = wn * 32 * TI + 32 * i + 16 * (g & 1) + 4 * pp;
      bbase[i] = lds_u32(sB) + img_off<RB>(8 * (g >> 1) + q, C0 >> 3) + (C0 & 7) * 2;
    }
    constexpr int NS = BP / 16, NRD = 2 * (TJ + TI);  // k-steps, reads per k-step
    u32x2 ra[2][TJ][2], rb[2][TI][2];
    auto rd = [&](auto S) {
      constexpr int s = decltype(S)::value;
      static_for<0, TJ>([&](auto J) {
        ra[s & 1][J][0] = tr_read_asm<16 * s * RA>(abase[J]);
        ra[s & 1][J][1] = tr_read_asm<16 * s * RA + 4 * RA>(abase[J]);
      });
      static_for<0, TI>([&](auto I) {
        rb[s & 1][I][0] = tr_read_asm<16 * s * RB>(bbase[I]);
        rb[s & 1][I][1] = tr_read_asm<16 * s * RB + 4 * RB>(bbase[I]);
      });
    };
    rd(std::integral_constant<int, 0>{});
    static_for<0, NS>([&](auto S) {
      constexpr int s = decltype(S)::value;
      if constexpr (s + 1 < NS) rd(std::integral_constant<int, s + 1>{});
      u32x4 fa[TJ], fb[TI];
      static_for<0, TJ>([&](auto J) {
        asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(ra[s & 1][J][0]), "+v"(ra[s & 1][J][1])
                     : "n"(s + 1 < NS ? NRD : 0));
        fa[J] = u32x4{ra[s & 1][J][0][0], ra[s & 1][J][0][1], ra[s & 1][J][1][0], ra[s & 1][J][1][1]};
      });
      static_for<0, TI>([&](auto I) {
        asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(rb[s & 1][I][0]), "+v"(rb[s & 1][I][1])
                     : "n"(s + 1 < NS ? NRD : 0));
        fb[I] = u32x4{rb[s & 1][I][0][0], rb[s & 1][I][0][1], rb[s & 1][I][1][0], rb[s & 1][I][1][1]};
      });
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int i = 0; i < TI; ++i) acc[j][i] = Mma<bf16>::run(fa[j], fb[i], acc[j][i]);
      if (do_bias) {
#pragma unroll
        for (int j = 0; j < TJ; ++j) accb[j] = Mma<bf16>::run(fa[j], ones, accb[j]);
      }
    });
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }

  const int r = lane & 31, h = lane >> 5;
  if (do_bias && r == 0) {  // every column of accb holds the row sums
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int co = co0 + wm * 64 + 32 * j + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (co < p.cout) atomicAdd(p.db + co, accb[j][e]);
      }
  }
#pragma unroll
  for (int j = 0; j < TJ; ++j)
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      const int nn = nk0 + wn * 32 * TI + 32 * i + r;
      if (nn >= p.K) continue;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int co = co0 + wm * 64 + 32 * j + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (co < p.cout) atomicAdd(wsb + (long long)co * p.K + nn, acc[j][i][e]);
      }
    }
}

template <int BMC, int BNK>
int launch_wgrad_glds(WgradGArgs a, hipStream_t st) {
  const int mt = (a.cout + BMC - 1) / BMC, nt = (a.K + BNK - 1) / BNK;
  constexpr long long target = 512;
  // many K tiles (the 15x15 init conv: K = 1800) make the im2col gather the
  // cost: 4x the workgroups there (measured 244 -> 179 us); a one- or two-tile
  // output keeps 512 (more splits only add same-address atomics: 43 -> 65 us)
  const long long tiles = (long long)mt * nt;
  long long want = (tiles >= 8 ? 4 * target : target) / tiles;
  if (want < 1) want = 1;
  long long per = ((long long)a.M + want - 1) / want;
  per = ((per + 255) / 256) * 256;
  if (per < 256) per = 256;
  // batched GEMMs have tiny outputs: cap the blocks adding into one element
  // (same-address atomic contention); measured at 16 / 32 / 64 / 128 for the
  // cross-attention token reductions (4 x 16384 rows, 32 x 64): 19.9 / 11.6 /
  // 8.5 / 8.7 us -- below 64 the per-block row loop dominates.  Wider outputs
  // (32 x K) add K / 64 times the atomics per block: the cap falls with K
  // (the chip's L2 atomics run ~270 G adds/s, profiles/r04d_l2_atomic_probe.txt)
  const int cap = a.K <= 64 ? 64 : std::max(16, 64 * 64 / a.K);
  if (a.batch_pix > 0 && (a.batch_pix + per - 1) / per > cap)
    per = ((a.batch_pix + cap - 1) / cap + 63) / 64 * 64;
  unsigned splits;
  if (a.batch_pix > 0) {
    const long long nbatch = a.M / a.batch_pix;
    long long spb = (a.batch_pix + per - 1) / per;
    per = (a.batch_pix + spb - 1) / spb;
    a.splits_per_batch = (int)spb;
    splits = (unsigned)(nbatch * spb);
  } else {
    splits = (unsigned)((a.M + per - 1) / per);
  }
  a.pix_per_split = (int)per;
  a.zper = (int)splits;
  if (a.ngemm > 1) splits *= (unsigned)a.ngemm;
  if (a.ks == 1) conv_wgrad_glds_kernel<BMC, BNK, true><<<dim3(mt, nt, splits), 256, 0, st>>>(a);
  else conv_wgrad_glds_kernel<BMC, BNK, false><<<dim3(mt, nt, splits), 256, 0, st>>>(a);
  return check_launch("conv_wgrad_glds");
}

static int launch_wgrad_glds_any(WgradGArgs& a, hipStream_t st) {
  if (a.cout <= 64) {
    if (a.K >= 2048 || a.K % 256 == 0) return launch_wgrad_glds<64, 256>(a, st);
    return launch_wgrad_glds<64, 128>(a, st);
  }
  return launch_wgrad_glds<128, 128>(a, st);
}

int conv_wgrad_glds(const void* dy, int lddy, const void* x0, int ld0, int c0, const void* x1,
                    int ld1, float* ws, float* db, int nf, int h, int w, int cin, int cout, int ks,
                    hipStream_t st, long long batch_pix) {
  WgradGArgs a;
  a.dy = (const bf16*)dy; a.lddy = lddy; a.x0 = (const bf16*)x0;
  a.x1 = (const bf16*)(x1 ? x1 : x0); a.ld0 = ld0; a.ld1 = x1 ? ld1 : ld0; a.c0 = x1 ? c0 : cin;
  a.ws = ws; a.db = db; a.H = h; a.W = w; a.cin = cin; a.cout = cout; a.ks = ks;
  a.K = ks * ks * cin; a.M = nf * h * w;
  a.batch_pix = (int)batch_pix; a.splits_per_batch = 1; a.pix_per_split = 0;
  a.ws_bstride = (long long)cout * a.K;
  a.fd_hw = make_fastdiv((unsigned)(h * w)); a.fd_w = make_fastdiv((unsigned)w);
  a.fd_cin = make_fastdiv((unsigned)cin); a.fd_ks = make_fastdiv((unsigned)ks);
  a.ngemm = 1; a.zper = 0;
  if (a.M == 0) return DV_OK;
  return launch_wgrad_glds_any(a, st);
}

// ngemm same-shape batched TN GEMMs out_g[b][i][j] += sum_r A_g[r][i] B_g[r][j]
// in ONE launch (the three cross-attention token reductions of a block share
// rows, m and n: one launch fills the chip three times as wide as each alone)
static int gemm_tn_multi_glds(int ngemm, const void* const* a, const int* lda, const void* const* b,
                              const int* ldb, float* const* out, long long batch_rows, int nbatch,
                              int m, int n, hipStream_t st) {
  WgradGArgs g;
  g.dy = (const bf16*)a[0]; g.lddy = lda[0]; g.x0 = g.x1 = (const bf16*)b[0];
  g.ld0 = g.ld1 = ldb[0]; g.c0 = n; g.ws = out[0]; g.db = nullptr;
  g.H = 1; g.W = 1; g.cin = n; g.cout = m; g.ks = 1; g.K = n;
  g.M = (int)(batch_rows * nbatch);
  g.batch_pix = (int)batch_rows; g.splits_per_batch = 1; g.pix_per_split = 0;
  g.ws_bstride = (long long)m * n;
  g.fd_hw = make_fastdiv(1u); g.fd_w = make_fastdiv(1u);
  g.fd_cin = make_fastdiv((unsigned)n); g.fd_ks = make_fastdiv(1u);
  g.ngemm = ngemm; g.zper = 0;
  for (int i = 0; i < 3; ++i) {
    const int j = i < ngemm ? i : 0;
    g.mdy[i] = (const bf16*)a[j]; g.mx[i] = (const bf16*)b[j];
    g.mlddy[i] = lda[j]; g.mld[i] = ldb[j]; g.mws[i] = out[j];
  }
  if (g.M == 0) return DV_OK;
  return launch_wgrad_glds_any(g, st);
}

// Weight packing, LDS-staged so both the torch-layout reads and the packed
// writes are coalesced:
//   mode 0 (forward):  out[co][tap][ci_p]  <- w[co][ci][tap]   (tile = 1 co row)
//   mode 1 (dgrad):    out[ci][tap'][co_p] <- w[co][ci][taps-1-tap']
//                      (tile = CT input channels: every co's contiguous
//                      w[co][ci0:ci0+CT][:] segment is read, then transposed)
//   modes 2 / 3: modes 0 / 1 with each row 16-channel-chunk-major,
//                      out[row][c_p / 16][tap][16] (pad % 16 == 0): the 8x8
//                      frame conv reads one chunk of a row as one contiguous run
__device__ __forceinline__ void pack_col(int j, int taps, int pad, bool chunked, int& tap, int& c) {
  if (chunked) {
    const int ch = j / (taps * 16), rem = j - ch * taps * 16;
    tap = rem >> 4;
    c = ch * 16 + (rem & 15);
  } else {
    tap = j / pad;
    c = j - tap * pad;
  }
}
constexpr int PACK_LDS = 8192;   // floats: the largest row / column group accepted
constexpr int PACK_TILE = 8192;  // floats staged per tile (several rows when they are small)
constexpr int PACK_CB = 64;      // dgrad tiles: output columns (co) per tile

// n contiguous floats -> LDS: 16-B loads (when the source is 16-B aligned),
// 4 in flight per lane
__device__ __forceinline__ void pack_stage(const float* src, float* sm, int n) {
  if ((reinterpret_cast<uintptr_t>(src) & 15) == 0) {
    const int n4 = n >> 2;
    for (int i0 = threadIdx.x; i0 < n4; i0 += 1024) {
      // unconditional loads (index clamped): a load under a lane branch makes
      // the compiler wait for every outstanding load at the join
      f32x4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = ((const f32x4*)src)[min(i0 + 256 * u, n4 - 1)];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (i0 + 256 * u < n4) ((f32x4*)sm)[i0 + 256 * u] = v[u];
    }
    for (int i = 4 * n4 + threadIdx.x; i < n; i += 256) sm[i] = src[i];
  } else {  // unaligned (a weight after an odd-sized one in the flat buffer): 8 loads in flight
    for (int i0 = threadIdx.x; i0 < n; i0 += 2048) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = src[min(i0 + 256 * u, n - 1)];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (i0 + 256 * u < n) sm[i0 + 256 * u] = v[u];
    }
  }
}

__device__ __forceinline__ void pack_tile(const DvPackEntry& e, int tile, float* sm) {  // inlined: sm stays an LDS pointer (ds_ ops, not flat)
  const int taps = e.taps, cin = e.cin, cout = e.cout, pad = e.pad_to;
  const bool fwd = (e.mode & 1) == 0, chunked = (e.mode & 2) != 0;
  if ((long long)(fwd ? cin : cout) * taps > PACK_LDS) return;  // rejected on the host
  const bool bf = e.dtype == DV_BF16;
  if (fwd) {
    const int row = cin * taps;
    int rt = PACK_TILE / row;
    if (rt < 1) rt = 1;
    const int co0 = tile * rt, rn = min(rt, cout - co0);
    const float* src = e.w + (long long)co0 * row;  // rn consecutive rows: contiguous
    pack_stage(src, sm, rn * row);
    __syncthreads();
    const int orow = taps * pad;
    const long long ob = (long long)co0 * orow;
    if (bf && pad % 8 == 0) {  // 8 consecutive outputs share (row, tap): one 16-B store
      for (int i = threadIdx.x * 8; i < rn * orow; i += 256 * 8) {
        const int rl = i / orow, j = i - rl * orow;
        int tap, ci;
        pack_col(j, taps, pad, chunked, tap, ci);
        const float* r = sm + rl * row + tap;
        float v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {  // clamped index: unconditional reads, then select
          const float t = r[min(ci + q, cin - 1) * taps];
          v[q] = ci + q < cin ? t : 0.f;
        }
        *(bf16x8*)((bf16*)e.out + ob + i) =
            bf16x8{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3], (bf16)v[4], (bf16)v[5], (bf16)v[6], (bf16)v[7]};
      }
    } else {
      for (int i = threadIdx.x; i < rn * orow; i += 256) {
        const int rl = i / orow, j = i - rl * orow;
        int tap, ci;
        pack_col(j, taps, pad, chunked, tap, ci);
        const float v = ci < cin ? sm[rl * row + ci * taps + tap] : 0.f;
        if (bf) ((bf16*)e.out)[ob + i] = (bf16)v;
        else ((float*)e.out)[ob + i] = v;
      }
    }
  } else {
    // 2-D tile: PACK_CB output columns (co) x ci_t input channels, so every
    // co row contributes one contiguous ci_t * taps run (>= 256 B for 3x3)
    // instead of a taps-long 36-B segment per (co, ci)
    const int ci_t = max(1, PACK_TILE / (PACK_CB * taps));
    const int nci = (cin + ci_t - 1) / ci_t;
    const int co0 = (tile / nci) * PACK_CB, ci0 = (tile % nci) * ci_t;
    const int cn = min(ci_t, cin - ci0);
    const int con = max(0, min(PACK_CB, cout - co0));  // real co rows (0 in the pad-only tail)
    const int seg = cn * taps;
    // 4 loads in flight per lane (the rows' segments are not 16-B aligned)
    for (int i0 = threadIdx.x; i0 < con * seg; i0 += 1024) {
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = min(i0 + 256 * u, con * seg - 1);  // clamped: unconditional loads
        const int r = i / seg, j = i - r * seg;
        v[u] = e.w[((long long)(co0 + r) * cin + ci0) * taps + j];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (i0 + 256 * u < con * seg) sm[i0 + 256 * u] = v[u];
    }
    __syncthreads();
    const int cw = min(PACK_CB, pad - co0);  // columns of this tile
    const int per_ci = taps * cw;
    const long long orow = (long long)taps * pad;
    auto ocol = [&](int tapd, int co) {
      return chunked ? (co >> 4) * taps * 16 + tapd * 16 + (co & 15) : tapd * pad + co;
    };
    if (bf && pad % 8 == 0) {  // 8 consecutive co share (ci, tap): one 16-B store
      for (int i = threadIdx.x * 8; i < cn * per_ci; i += 256 * 8) {
        const int cl = i / per_ci, rem = i - cl * per_ci;
        const int tapd = rem / cw, cc = rem - tapd * cw;
        const float* r = sm + cl * taps + (taps - 1 - tapd);
        float v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {  // clamped index: unconditional reads, then select
          const float t = r[max(0, min(cc + q, con - 1)) * seg];
          v[q] = cc + q < con ? t : 0.f;
        }
        *(bf16x8*)((bf16*)e.out + (ci0 + cl) * orow + ocol(tapd, co0 + cc)) =
            bf16x8{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3], (bf16)v[4], (bf16)v[5], (bf16)v[6], (bf16)v[7]};
      }
    } else {
      for (int i = threadIdx.x; i < cn * per_ci; i += 256) {
        const int cl = i / per_ci, rem = i - cl * per_ci;
        const int tapd = rem / cw, cc = rem - tapd * cw;
        const float v = cc < con ? sm[cc * seg + cl * taps + (taps - 1 - tapd)] : 0.f;
        const long long o = (ci0 + cl) * orow + ocol(tapd, co0 + cc);
        if (bf) ((bf16*)e.out)[o] = (bf16)v;
        else ((float*)e.out)[o] = v;
      }
    }
  }
  __syncthreads();  // sm is reused by the next tile
}

__device__ __forceinline__ int pack_tiles(const DvPackEntry& e) {
  if ((e.mode & 1) == 0) {
    const int per = max(1, PACK_TILE / (e.cin * e.taps));
    return (e.cout + per - 1) / per;
  }
  const int ci_t = max(1, PACK_TILE / (PACK_CB * e.taps));
  return ((e.pad_to + PACK_CB - 1) / PACK_CB) * ((e.cin + ci_t - 1) / ci_t);
}

__global__ __launch_bounds__(256) void pack_weight_kernel(DvPackEntry e) {
  __shared__ __attribute__((aligned(16))) float sm[PACK_LDS];  // one row may need up to PACK_LDS floats
  for (int t = blockIdx.x; t < pack_tiles(e); t += gridDim.x) pack_tile(e, t, sm);
}

// many weights in one launch: blockIdx.y selects the table entry
__global__ __launch_bounds__(256) void pack_weight_batched_kernel(const DvPackEntry* table) {
  __shared__ __attribute__((aligned(16))) float sm[PACK_LDS];
  const DvPackEntry e = table[blockIdx.y];
  for (int t = blockIdx.x; t < pack_tiles(e); t += gridDim.x) pack_tile(e, t, sm);
}

// Both images of a bf16 3x3 weight from one staged (64 co) x (16 ci) x 9 tile:
// the forward rows co0..co0+63 (16 input channels each) and the dgrad rows
// ci0..ci0+15 (64 output channels each) -- the f32 weight is read once, not
// once per image, and a tile is 36 KB (the per-image forward tile of a
// 512-channel weight held one 18 KB row)
constexpr int PP_CO = 64, PP_CI = 16, PP_T = 9, PP_SROW = PP_CI * PP_T + 1;
__global__ __launch_bounds__(256) void pack_pair_kernel(const DvPackPair* table, const int* tile_entry) {
  __shared__ float sm[PP_CO * PP_SROW];
  const int tid = threadIdx.x;
  const int ei = tile_entry[blockIdx.x];
  const DvPackPair e = table[ei];
  const int t = (int)(blockIdx.x - e.tile0);
  const int nci = e.cin / PP_CI;
  const int co0 = (t / nci) * PP_CO, ci0 = (t - (t / nci) * nci) * PP_CI;
  constexpr int SEG = PP_CI * PP_T;  // 144 contiguous floats per co row
  const float* src = e.w + ((long long)co0 * e.cin + ci0) * PP_T;
  const long long rstride = (long long)e.cin * PP_T;
  // 64 x 144 floats, 9 loads in flight per lane (index clamped: unconditional loads)
  constexpr int N = PP_CO * SEG, U = 9;
  for (int i0 = tid; i0 < N; i0 += 256 * U) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = min(i0 + 256 * u, N - 1);
      const int r = i / SEG, j = i - r * SEG;
      v[u] = src[r * rstride + j];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + 256 * u;
      if (i < N) {
        const int r = i / SEG, j = i - r * SEG;
        sm[r * PP_SROW + j] = v[u];
      }
    }
  }
  __syncthreads();
  const int mf = e.modes & 255, md = e.modes >> 8;
  // forward image: row co, tap, 8 input channels per 16-B store
  {
    bf16* out = (bf16*)e.out_fwd;
    const long long orow = (long long)PP_T * e.cin;
    for (int idx = tid; idx < PP_CO * PP_T * 2; idx += 256) {
      const int co = idx / (PP_T * 2), rem = idx - co * (PP_T * 2);
      const int tap = rem >> 1, h8 = (rem & 1) * 8;
      const float* r = sm + co * PP_SROW + h8 * PP_T + tap;
      const long long o = (long long)(co0 + co) * orow +
                          (mf == 2 ? (ci0 / 16) * (PP_T * 16) + tap * 16 + h8 : (long long)tap * e.cin + ci0 + h8);
      *(bf16x8*)(out + o) = bf16x8{(bf16)r[0], (bf16)r[PP_T], (bf16)r[2 * PP_T], (bf16)r[3 * PP_T],
                                   (bf16)r[4 * PP_T], (bf16)r[5 * PP_T], (bf16)r[6 * PP_T], (bf16)r[7 * PP_T]};
    }
  }
  // dgrad image: row ci, flipped tap, 8 output channels per 16-B store
  {
    bf16* out = (bf16*)e.out_dgrad;
    const long long orow = (long long)PP_T * e.cout;
    for (int idx = tid; idx < PP_CI * PP_T * (PP_CO / 8); idx += 256) {
      const int ci = idx / (PP_T * 8), rem = idx - ci * (PP_T * 8);
      const int tpd = rem >> 3, g8 = rem & 7;
      const float* r = sm + (g8 * 8) * PP_SROW + ci * PP_T + (PP_T - 1 - tpd);
      const int co = co0 + g8 * 8;
      const long long o = (long long)(ci0 + ci) * orow +
                          (md == 3 ? (co >> 4) * (PP_T * 16) + tpd * 16 + (co & 15) : (long long)tpd * e.cout + co);
      *(bf16x8*)(out + o) = bf16x8{(bf16)r[0], (bf16)r[PP_SROW], (bf16)r[2 * PP_SROW], (bf16)r[3 * PP_SROW],
                                   (bf16)r[4 * PP_SROW], (bf16)r[5 * PP_SROW], (bf16)r[6 * PP_SROW],
                                   (bf16)r[7 * PP_SROW]};
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void bias_grad_kernel(const T* dy, int lddy, float* db,
                                                        long long npix, int c, long long rows_per) {
  __shared__ float sh[4][64];
  const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int ch = blockIdx.x * 64 + cl;
  long long beg = blockIdx.y * rows_per, end = beg + rows_per;
  if (end > npix) end = npix;
  float s = 0.f;
  if (ch < c)
    for (long long m = beg + rg; m < end; m += 4) s += (float)dy[m * lddy + ch];
  sh[rg][cl] = s;
  __syncthreads();
  if (rg == 0 && ch < c) atomicAdd(db + ch, sh[0][cl] + sh[1][cl] + sh[2][cl] + sh[3][cl]);
}

template <typename T, int BM, int BN>
int launch_fwd(const ConvFwdArgs<T>& a, hipStream_t st) {
  dim3 grid((unsigned)((a.M + BM - 1) / BM), (unsigned)((a.cout + BN - 1) / BN));
  if (a.gn_sums) conv_fwd_kernel<T, BM, BN, true><<<grid, 256, 0, st>>>(a);
  else conv_fwd_kernel<T, BM, BN, false><<<grid, 256, 0, st>>>(a);
  return check_launch("conv_fwd");
}

// the 1x1 streaming kernel's shapes (see conv1x1_stream_kernel)
bool conv1x1_ok(const ConvFwdArgs<bf16>& a, bool split) {
  return a.ks == 1 && (a.cin == 64 || a.cin == 128) && (!split || a.c0 == 64) &&
         (a.cout == 64 || a.cout == 128) && a.gn_sums == nullptr && (a.ldy & 3) == 0 &&
         (a.res == nullptr || (a.ldres & 3) == 0) && (a.ld0 & 7) == 0 && (!split || (a.ld1 & 7) == 0) &&
         a.M * std::max(a.ld0, split ? a.ld1 : 0) < (1ll << 31) &&
         a.M * std::max(a.ldy, a.res ? a.ldres : 0) < (1ll << 31);
}

template <int BN, int KT>
int launch_conv1x1(const ConvFwdArgs<bf16>& a, hipStream_t st) {
  constexpr int NB = 3;
  constexpr int LDS = BN * 128 * KT + NB * 128 * 128 * KT;
  // (the residual variant keeps its residual tiles in the ring when they fit:
  // mirror of conv1x1_stream_kernel's RLDS)
  constexpr int LDS_RES = LDS + NB * 128 * BN * 2 <= 160 * 1024 ? LDS + NB * 128 * BN * 2 : LDS;
  const int ntiles = (int)((a.M + 127) / 128);
  const int grid = std::min(ntiles, 256 * ((160 * 1024) / (a.res ? LDS_RES : LDS)));
  if (a.res) conv1x1_stream_kernel<BN, KT, NB, true><<<grid, 512, 0, st>>>(a, ntiles);
  else conv1x1_stream_kernel<BN, KT, NB, false><<<grid, 512, 0, st>>>(a, ntiles);
  return check_launch("conv1x1_stream");
}

template <int BM, int BN>
int launch_fwd_glds(const ConvFwdArgs<bf16>& a, hipStream_t st) {
  const int tn = (a.cout + BN - 1) / BN;
  const long long nb = ((a.M + BM - 1) / BM) * tn;
  // ring depth by residency: one workgroup per CU -> as deep as LDS allows
  constexpr int BUF = (BM + BN) * 128;
  constexpr int DEEP = (160 * 1024) / BUF > 6 ? 6 : (160 * 1024) / BUF;
  constexpr int MID = (80 * 1024) / BUF > 3 ? 3 : (80 * 1024) / BUF;
  const bool stats = a.gn_sums != nullptr;
#define DV_GL(NB) (stats ? conv_fwd_glds_kernel<BM, BN, NB, true><<<(unsigned)nb, 256, 0, st>>>(a, tn) \
                         : conv_fwd_glds_kernel<BM, BN, NB, false><<<(unsigned)nb, 256, 0, st>>>(a, tn))
  if (nb <= 256) DV_GL(DEEP);
  else if (nb <= 512 && MID >= 3) DV_GL(MID);
  else DV_GL(2);
#undef DV_GL
  return check_launch("conv_fwd_glds");
}


// ---------------------------------------------------------------------------
// bf16 3x3 forward / dgrad, stripe form (cin == 64 single source, cout % 64
// == 0, W in {32, 64, 128}): one workgroup = 64 output channels over a contiguous
// range of 128-pixel stages.  8 waves: 4 pixel tiles x 2 channel halves, one
// 32 x 32 accumulator each (initialised to the bias).  Each wave keeps the A
// fragments of its 32 output channels for all 36 k-steps in REGISTERS (144
// VGPRs), so the MFMA loop reads only the X window from LDS: one
// ds_read_b128 per MFMA, issued 8 k-steps ahead (inline asm, hand-counted
// lgkmcnt).  Per stage the window (128 / W + 2 image rows of W + 2 pixels,
// halo zero) is staged ONCE for all nine taps, which read it at row offsets
// dy*(W+2) + dx; pixel rows padded to 144 B (16 consecutive rows start
// 9 x 16 B apart mod 256 B: conflict-free ds_read_b128, every tap / k-step
// offset an immediate).  Windows and the one-time weight image arrive by
// LDS-DMA through a raw buffer resource (halo and pad slots out of range:
// zeros without traffic) into a 4-buffer ring, three stages ahead, counted
// vmcnt + one raw barrier per stage.  All LDS in ONE __shared__ array (a
// second object can make hipcc drain vmcnt before the first ds_read).
// Measured 64->64 @ 64x64 x 64 frames: 37.5 -> ~25 us (prologue ~4 us of it).
// ---------------------------------------------------------------------------
constexpr int FS_XP = 144;   // window pixel pitch (64 bf16 + 16 B)

constexpr int FS_WROW = 1168;    // LDS weight row pitch: 576 bf16 + 16 B
constexpr int FS_WPIECES = 73;   // 64 rows x 73 16-B slots = 73 DMA pieces of 1 KB

// Row ring (round 5).  A stage's window is SEG + 2 image rows, of which the
// first two are the previous stage's last two: only SEG new rows are staged
// per stage (half the LDS-DMA bytes at W = 64, where the per-CU DMA intake
// bound the loop: phase stamps, profiles/r05n_conv_stamps.txt).  Rows live in
// a ring of R = 4 SEG + 2 row slots (three stages ahead + the stage being
// read); a row slot is PPR whole 1-KB DMA pieces (WP pixels x 9 16-B slots,
// padded), so no piece straddles two rows and rows need not be adjacent: each
// tap row dy has its own base address.  A workgroup's stages lie in one frame
// (the launcher picks stages_per_block | stages per frame), so the reused rows
// are always the right ones.
template <int W>
struct FsGeom {
  static constexpr int WP = W + 2, SEG = 128 / W;
  static constexpr int PPR = (WP * 9 + 63) / 64;     // 1-KB pieces per row slot
  static constexpr int ROWB = PPR * 1024;            // row slot bytes
  static constexpr int R = 4 * SEG + 2;              // row slots in the ring
  static constexpr int NP = SEG * PPR;               // pieces of a stage's new rows
  static constexpr int NPW = (NP + 7) / 8;           // per wave (spare ones repeat the last)
  static constexpr int NP0 = (SEG + 2) * PPR;        // stage 0 stages its whole window
  static constexpr int NPW0 = (NP0 + 7) / 8;
  // weight image: beyond the rows of stages 0..2; where that does not fit
  // (W = 128: 19-KB rows) beyond stages 0..1, and stage 2's rows go out only
  // after the weights are in registers (LATE)
  static constexpr bool LATE = (3 * SEG + 2) * ROWB + 64 * FS_WROW > 160 * 1024;
  static constexpr int WOFF = (LATE ? 2 * SEG + 2 : 3 * SEG + 2) * ROWB;
  static constexpr int LDS = R * ROWB > WOFF + 64 * FS_WROW ? R * ROWB : WOFF + 64 * FS_WROW;
  static_assert(LDS <= 160 * 1024, "stripe ring exceeds the LDS");
  // the stage loop issues a wave's pieces of stage st+3 at k-steps k % 7 == 3
  // (k < 36: at most 5 of them), and the hand-counted waits assume exactly NPW
  // pieces per stage; the largest vmcnt immediate (two residuals: 2*8 + 12 +
  // 2*NPW) must fit the 6-bit field
  static_assert(NPW <= 5, "stripe stage pieces exceed the k-step issue slots");
  static_assert(2 * 8 + 12 + 2 * NPW <= 63, "stripe vmcnt immediate out of range");
};
// immediate offset of k-step k (tap k / 4 = 3 dy + dx, 16 channels at
// (k % 4) * 16) from the lane's tap row dy base
constexpr int fs_koff(int k) { return ((k >> 2) % 3) * FS_XP + (k & 3) * 32; }

typedef float __attribute__((ext_vector_type(2))) gf2;
#ifndef FS_TSTEP
#define FS_TSTEP 4
#endif

template <int W, int NRES, bool STATS, bool GNIN = false>
__global__ __launch_bounds__(512) void conv_fwd_stripe_kernel(ConvFwdArgs<bf16> p, int nstages,
                                                              int stages_per_block) {
  using G = FsGeom<W>;
  constexpr int WP = G::WP, SEG = G::SEG, PPR = G::PPR, ROWB = G::ROWB, R = G::R;
  constexpr int NP = G::NP, NPW = G::NPW, NP0 = G::NP0, NPW0 = G::NPW0;
  static_assert(!GNIN || (W == 64 && NRES == 0), "the folded GroupNorm input is built for W = 64, no residual");
  // GNIN: the coefficient scratch (128 sums, 4 x 64 parameters, the A / B table, 64 biases) past the ring
  __shared__ __attribute__((aligned(1024))) char smem[G::LDS + (GNIN ? 2304 : 0)];
  DV_STAMP_AT(0);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int pt = wave & 3, ch = wave >> 2;
  const int co0 = blockIdx.y * 64;
  const int sbeg = blockIdx.x * stages_per_block;
  const int nst = min(sbeg + stages_per_block, nstages) - sbeg;
  const int HW = p.H * W;
  // the workgroup's frame and first output row; window row q is image row yq0 + q
  const int m00 = sbeg * 128;
  const int fbase = (m00 / HW) * HW;                 // first pixel of the frame
  const int yq0 = (m00 - fbase) / W - 1;

  // GNIN: this thread's window slot of every staged row (W = 64: a row's 64
  // pixels x 8 16-B channel slots are the 512 threads): pixel gx, channels
  // 8 gc .. 8 gc + 7 = GroupNorm group gc (64 channels, 8 groups).  The
  // per-channel A / B are computed here, before any DMA is issued (plain loads
  // + two barriers, ~1 round trip: no compiler-counted vector load among the
  // hand-counted DMA waits below), into an LDS table [group][A 0..7, B 0..7]
  // that fold_rows reads (registers would spill beside the statistics epilogue).
  const int gx = tid >> 3, gc = tid & 7;
  float* gi_tab = (float*)(smem + G::LDS) + 384;
  float* gi_bias = gi_tab + 128;  // the workgroup's 64 output channels' bias
  if constexpr (GNIN) {
    // the next GroupNorm's sums buffer, zeroed across the grid (stores older
    // than every DMA: the prologue's waits cover them)
    if (p.gi_zero) {
      const long long nblk = (long long)gridDim.x * gridDim.y;
      const long long per = ((p.gi_zero_n + nblk - 1) / nblk + 3) / 4 * 4;
      const long long i0 = ((long long)blockIdx.y * gridDim.x + blockIdx.x) * per;
      for (long long i = i0 + tid * 4; i < i0 + per && i < p.gi_zero_n; i += 2048) {
        if (i + 4 <= p.gi_zero_n) *(f32x4*)(p.gi_zero + i) = f32x4{0.f, 0.f, 0.f, 0.f};
        else for (long long j = i; j < p.gi_zero_n; ++j) p.gi_zero[j] = 0.f;
      }
    }
    float* cs = (float*)(smem + G::LDS);  // [64][2] clip totals, then gamma, beta, 1 + scale, shift
    float* prm = cs + 128;
    const long long b = m00 / p.gi_P;     // the workgroup's clip (stages never straddle one)
    if (tid < 128) {  // all replicas in flight at once (a runtime-bound loop waited per load)
      float v[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) v[r] = p.gi_sums[min(r, p.gi_R - 1) * p.gi_rstride + b * 128 + tid];
      float s = 0.f;
#pragma unroll
      for (int r = 0; r < 8; ++r) s += r < p.gi_R ? v[r] : 0.f;
      for (int r = 8; r < p.gi_R; ++r) s += p.gi_sums[r * p.gi_rstride + b * 128 + tid];
      cs[tid] = s;
    } else if (tid >= 256 && tid < 320) {
      gi_bias[tid - 256] = p.bias ? p.bias[co0 + tid - 256] : 0.f;
    } else if (tid >= 128 && tid < 192) {
      const int c = tid - 128;
      prm[c] = p.gi_gamma[c];
      prm[64 + c] = p.gi_beta[c];
      prm[128 + c] = p.gi_ss ? 1.f + p.gi_ss[b * 128 + c] : 1.f;
      prm[192 + c] = p.gi_ss ? p.gi_ss[b * 128 + 64 + c] : 0.f;
    }
    __syncthreads();
    if (tid < 64) {  // channel tid of group tid / 8
      const int g = tid >> 3;
      double d1 = 0.0, d2 = 0.0;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        d1 += cs[2 * (8 * g + e)];
        d2 += cs[2 * (8 * g + e) + 1];
      }
      const double n = (double)p.gi_P * 8;
      const double m = d1 / n;
      double var = d2 / n - m * m;
      if (var < 0) var = 0;
      const float mu = (float)m, rs = (float)(1.0 / sqrt(var + (double)p.gi_eps));
      const float gm = prm[tid], bt = prm[64 + tid], sc = prm[128 + tid], sh = prm[192 + tid];
      gi_tab[16 * g + (tid & 7)] = rs * gm * sc;
      gi_tab[16 * g + 8 + (tid & 7)] = (bt - mu * rs * gm) * sc + sh;
      // the clip's first workgroup of channel tile 0 saves the statistics
      if (blockIdx.y == 0 && m00 % p.gi_P == 0 && (tid & 7) == 0) {
        p.gi_mean[b * 8 + g] = mu;
        p.gi_rstd[b * 8 + g] = rs;
      }
    }
    __syncthreads();
  }
  const __amdgpu_buffer_rsrc_t yr =
      dma_rsrc(GNIN ? (const void*)p.gi_y : nullptr, GNIN && p.gi_y ? (unsigned)(p.M * p.gi_ldy * 2) : 0u);
  // GNIN: rows q0 .. q0 + NQ - 1 of the window ring -> silu(A z + B) in place
  // (image rows outside the frame stay zero), each also stored to gi_y when
  // the workgroup owns it (window rows 1 .. nst SEG: its output rows).  Every
  // thread issues exactly NQ stores (a dropped one goes out of range), so the
  // stage loop's hand-counted vmcnt waits can count them.
  auto fold_rows = [&](auto nq, int q0) {
    constexpr int NQ = decltype(nq)::value;
    u32x4 v[NQ], kt[4];
    unsigned la[NQ];
    const unsigned ta = lds_addr(gi_tab + 16 * gc);
    kt[0] = ds_read_b128_off<0>(ta);
    kt[1] = ds_read_b128_off<16>(ta);
    kt[2] = ds_read_b128_off<32>(ta);
    kt[3] = ds_read_b128_off<48>(ta);
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
      la[i] = lds_addr(smem + ((q0 + i) % R) * ROWB + (gx + 1) * FS_XP + gc * 16);
      v[i] = ds_read_b128_off<0>(la[i]);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) lgkm_wait_tied<0>(kt[i]);
#pragma unroll
    for (int i = 0; i < NQ; ++i) lgkm_wait_tied<0>(v[i]);
    gf2 gi_A[4], gi_B[4];
    {
      const f32x4 a0 = __builtin_bit_cast(f32x4, kt[0]), a1 = __builtin_bit_cast(f32x4, kt[1]);
      const f32x4 b0 = __builtin_bit_cast(f32x4, kt[2]), b1 = __builtin_bit_cast(f32x4, kt[3]);
      gi_A[0] = gf2{a0[0], a0[1]}; gi_A[1] = gf2{a0[2], a0[3]};
      gi_A[2] = gf2{a1[0], a1[1]}; gi_A[3] = gf2{a1[2], a1[3]};
      gi_B[0] = gf2{b0[0], b0[1]}; gi_B[1] = gf2{b0[2], b0[3]};
      gi_B[2] = gf2{b1[0], b1[1]}; gi_B[3] = gf2{b1[2], b1[3]};
    }
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
      const int q = q0 + i, y = yq0 + q;
      const bool in = (unsigned)y < (unsigned)p.H;
      float z[8];
      Vec<bf16>::to_f(v[i], z);
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        gf2 t = gf2{z[2 * j], z[2 * j + 1]} * gi_A[j] + gi_B[j];
        const gf2 mm = t * -1.4426950408889634f;  // silu as the GroupNorm apply computes it
        const gf2 d = 1.f + gf2{__builtin_amdgcn_exp2f(mm.x), __builtin_amdgcn_exp2f(mm.y)};
        t *= gf2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
        o[2 * j] = (bf16)t.x;
        o[2 * j + 1] = (bf16)t.y;
      }
      const u32x4 ov = in ? __builtin_bit_cast(u32x4, o) : u32x4{0u, 0u, 0u, 0u};
      asm volatile("ds_write_b128 %0, %1" ::"v"(la[i]), "v"(ov) : "memory");
      const bool own = in && q >= 1 && q <= nst * SEG;
      __builtin_amdgcn_raw_buffer_store_b128(
          ov, yr, own ? (unsigned)(((fbase + y * W + gx) * p.gi_ldy + gc * 8) * 2) : DMA_OOB, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };

  // this lane's 16-B slot of each of the wave's pieces: a column byte offset
  // within an image row (or -1: halo / pad slot) and the row within the
  // pieces' rows (stage 0: the window's SEG + 2 rows; later: the SEG new ones)
  auto slot_of = [&](int piece, int& rr, int& coff) {
    rr = piece / PPR;
    const int slot = (piece - rr * PPR) * 64 + lane, px = slot / 9, c = slot - px * 9;
    const bool ok = slot < WP * 9 && c < 8 && px >= 1 && px <= W;
    coff = ok ? ((px - 1) * p.ld0 + c * 8) * 2 : -1;
  };
  int s_rr[NPW], s_co[NPW];
#pragma unroll
  for (int i = 0; i < NPW; ++i) slot_of(min(wave + 8 * i, NP - 1), s_rr[i], s_co[i]);
  // x0 as a raw buffer: halo and pad slots load out of range (zeros, no traffic)
  const __amdgpu_buffer_rsrc_t xr = dma_rsrc(p.x0, (unsigned)(p.M * p.ld0 * 2));
  // one piece of window row q (its ring slot q % R, piece part of the row)
  auto dma_row = [&](int q, int piece, int coff) {
    const int y = yq0 + q;
    const bool in = coff >= 0 && (unsigned)y < (unsigned)p.H;
    dma16(xr, smem + (q % R) * ROWB + (piece % PPR) * 1024,
          in ? (unsigned)((fbase + y * W) * p.ld0 * 2 + coff) : DMA_OOB);
  };
  // piece i of stage st >= 1: its new rows q = st SEG + 2 .. st SEG + SEG + 1
  auto issue1 = [&](int st, int i) {
    if constexpr (GNIN) {  // recomputed from an opaque lane id: no VGPRs held across the stage loop
      int ln = lane, rr;
      asm volatile("" : "+v"(ln));
      const int piece = min(wave + 8 * i, NP - 1);
      rr = piece / PPR;
      const int slot = (piece - rr * PPR) * 64 + ln, px = slot / 9, c = slot - px * 9;
      const bool ok = slot < WP * 9 && c < 8 && px >= 1 && px <= W;
      dma_row(st * SEG + 2 + rr, piece, ok ? ((px - 1) * p.ld0 + c * 8) * 2 : -1);
    } else {
      dma_row(st * SEG + 2 + s_rr[i], min(wave + 8 * i, NP - 1), s_co[i]);
    }
  };
  auto issue = [&](int st) {
#pragma unroll
    for (int i = 0; i < NPW; ++i) issue1(st, i);
  };

  // prologue: stage 0's whole window, the weight image (beyond the rows of
  // stages 0..2), the bias, then stages 1 and 2: only the weights and stage 0
  // are waited for before the fragments are read into registers.
  // (Direct per-wave global loads of the weight fragments touch 32 lines per
  // instruction for 8 KB of use: ~20k cycles of prologue.)
  if (nst > 0) {
#pragma unroll
    for (int i = 0; i < NPW0; ++i) {
      const int piece = min(wave + 8 * i, NP0 - 1);
      int rr, coff;
      slot_of(piece, rr, coff);
      dma_row(rr, piece, coff);
    }
  }
  DV_SP(7);
  {
    char* sW = smem + G::WOFF;
    const int wci = p.wcin ? p.wcin : 64;  // image channels per tap (row pitch 9 wci)
    const __amdgpu_buffer_rsrc_t wr = dma_rsrc(p.w + (long long)co0 * 9 * wci, 64 * 9 * wci * 2);
#pragma unroll
    for (int i = 0; i < FS_WPIECES / 8 + 1; ++i) {
      const int piece = min(wave + 8 * i, FS_WPIECES - 1);
      const int slot = piece * 64 + lane, row = slot / 73, c = slot - row * 73;
      // 16-B slot c of the row's 9 x 64 channels: tap c / 8, channels wc0 + 8 (c % 8)
      dma16(wr, sW + piece * 1024,
            c < 72 ? (unsigned)((row * 9 * wci + (c >> 3) * wci + p.wc0 + (c & 7) * 8) * 2) : DMA_OOB);
    }
  }
  // bias of the lane's 16 accumulator channels (8g + 4h + e of the wave's 32),
  // by SCALAR loads of the wave's 32 (lgkmcnt): a vector load here was the
  // last vmcnt op hipcc knew of before the stage loop, so it put a vmcnt(0)
  // at the loop entry -- which also drained the DMA of stages 1 and 2
  // (GNIN: the bias is added in the epilogue from LDS instead -- 16 VGPRs the
  // in-loop transform needs beside the statistics accumulators)
  f32x16 bias_acc;
  if constexpr (!GNIN) {
    float bw[32];
    const float* bp = p.bias ? p.bias + co0 + ch * 32 : nullptr;
#pragma unroll
    for (int j = 0; j < 32; ++j) bw[j] = bp ? __builtin_nontemporal_load(bp + j) : 0.f;
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int e = 0; e < 4; ++e) bias_acc[4 * g + e] = (lane >> 5) ? bw[8 * g + 4 + e] : bw[8 * g + e];
  }
  if (nst > 1) issue(1);
  if (!G::LATE && nst > 2) issue(2);
  DV_SP(4);
  // stage 0, weights and bias landed; stages 1 and 2 (when issued) younger.
  // GNIN: stage 1's rows too (stage 0 transforms them among its MFMAs).
  // (The weight image loaded through VGPRs -- coalesced 16-B loads, then
  // ds_write -- instead of LDS-DMA measured slower: 33.9 vs 30.9 us per 64^2
  // call, profiles/r06o_stripe_prologue.txt.)
  if constexpr (GNIN) {
    if (nst > 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NPW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    if (!G::LATE && nst > 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NPW) : "memory");
    else if (nst > 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NPW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  // raw barriers (asm, memory-clobbering): __syncthreads()'s fence made hipcc
  // wait for EVERY outstanding vector-memory op (vmcnt(0)) -- the DMA of
  // stages 1 and 2 as well -- before the weights could be read
  asm volatile("s_barrier" ::: "memory");
  DV_SP(5);
  u32x4 wA[36];
  {
    // inline-asm reads (a compiler-visible LDS read beside the pending DMA
    // got a vmcnt(0) in front in some instantiations: stages 1 and 2 drained)
    const unsigned aw = lds_addr(smem + G::WOFF + (ch * 32 + (lane & 31)) * FS_WROW + (lane >> 5) * 16);
    static_for<0, 36>([&](auto kk) {
      constexpr int k = decltype(kk)::value;
      wA[k] = ds_read_b128_off<32 * k>(aw);
    });
    static_for<0, 36>([&](auto kk) { lgkm_wait_tied<0>(wA[decltype(kk)::value]); });
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  asm volatile("s_barrier" ::: "memory");  // the weight image is dead: stage 3's rows may land over it
  DV_SP(6);
  // LATE: stage 2's rows now (over the dead weight image).  They are still
  // issued after D1 and before stage 0's residual loads: the per-stage vmcnt
  // counts below hold unchanged.
  if (G::LATE && nst > 2) issue(2);
  asm volatile("" ::: "memory");  // (stage 0's residual loads stay younger than D2)
  // GNIN: stage 0's whole window (SEG + 2 rows, landed) transformed here (Y0
  // stores per thread); stage s >= 1's SEG new rows during stage s - 1
  constexpr int Y0 = SEG + 2;
  if constexpr (GNIN) {
    if (nst > 0) {  // (two rows at a time: four spill beside the statistics accumulators)
      fold_rows(std::integral_constant<int, 2>{}, 0);
      fold_rows(std::integral_constant<int, SEG>{}, 2);
    }
    asm volatile("s_barrier" ::: "memory");
  }
  DV_STAMP_AT(1);

  const int r = lane & 31, h = lane >> 5;
  const int px = pt * 32 + r;           // lane's pixel in the stage
  const int orow = px / W;              // its output row in the stage (wave-uniform)
  const int loff = (px % W) * FS_XP + h * 16;
  // GroupNorm statistics (STATS, compile-time like NRES): per stage only the
  // first step of the half-wave reduce-scatter (lanes r, r ^ 16: 16 shuffles
  // instead of the 31 of gn_rs_reduce) and a lane accumulates the 16 values
  // it keeps over the stages (16 VGPRs); the remaining four steps run once,
  // when the stage range crosses into the next clip (128-pixel stages never
  // straddle one: the host requires gn_P % 128 == 0) and at the end.  (Round 5
  // reduced every stage fully: ~6 us per 64^2 launch over the plain kernel.)
  float sacc[32];  // [0, 16) live across stages
#pragma unroll
  for (int i = 0; i < 16; ++i) sacc[i] = 0.f;
  auto rs_tail = [&]() {  // gn_rs_reduce's steps after the first
    rs_step<32, 8>(sacc, r);
    rs_step<32, 4>(sacc, r);
    rs_step<32, 2>(sacc, r);
    rs_step<32, 1>(sacc, r);
  };
  constexpr bool stats = STATS;
  auto chan = [&](int k) { return co0 + ch * 32 + 8 * (k / 4) + 4 * h + (k % 4); };

  for (int st = 0; st < nst; ++st) {
    if constexpr (stats) if (st > 0) {
      const long long c_prev = (long long)(sbeg + st - 1) * 128 / p.gn_P;
      if ((long long)(sbeg + st) * 128 / p.gn_P != c_prev) {
        rs_tail();
        gn_rs_add<bf16, 32>(p, sacc, c_prev, chan);
#pragma unroll
        for (int i = 0; i < 16; ++i) sacc[i] = 0.f;
      }
    }
    // GNIN: the next stage's SEG new rows (landed at the last barrier; no wave
    // reads them in this stage) are transformed among this stage's MFMAs: the
    // thread's slot of each row and its group's A / B read here, ahead of the
    // window fragments (the first fragment wait covers them), one channel
    // pair per k-step 1 .. 4 SEG, written back / stored after the loop.
    const bool tr = GNIN && st + 1 < nst;  // wave-uniform
    u32x4 tk[4], tv[SEG];
    if constexpr (GNIN) if (tr) {
      // (slot coordinates from an opaque thread id: recomputed per stage, not
      // held in VGPRs across the loop beside the statistics accumulators)
      int ot = tid;
      asm volatile("" : "+v"(ot));
      const int gx = ot >> 3, gc = ot & 7;
      const unsigned ta = lds_addr(gi_tab + 16 * gc);
      tk[0] = ds_read_b128_off<0>(ta);
      tk[1] = ds_read_b128_off<16>(ta);
      tk[2] = ds_read_b128_off<32>(ta);
      tk[3] = ds_read_b128_off<48>(ta);
#pragma unroll
      for (int i = 0; i < SEG; ++i)
        tv[i] = ds_read_b128_off<0>(lds_addr(smem + (((st + 1) * SEG + 2 + i) % R) * ROWB + (gx + 1) * FS_XP + gc * 16));
    }
    // the lane's three tap rows dy = 0..2: window rows st SEG + orow + dy
    const int q0 = st * SEG + orow;
    const unsigned xa0 = lds_addr(smem + (q0 % R) * ROWB + loff);
    const unsigned xa1 = lds_addr(smem + ((q0 + 1) % R) * ROWB + loff);
    const unsigned xa2 = lds_addr(smem + ((q0 + 2) % R) * ROWB + loff);
    auto xrow = [&](int k) { return (k >> 2) / 3 == 0 ? xa0 : ((k >> 2) / 3 == 1 ? xa1 : xa2); };
    // window fragments read FSD k-steps ahead of their MFMA (k-step k = tap
    // k / 4, 16 channels at (k % 4) * 16).  The reads are inline asm with
    // hand-counted lgkmcnt: beside the LDS-DMA hipcc's waitcnt pass treats
    // the LGKM queue as out of order and drains it to 0 every few reads.
    // (fewer VGPRs of read-ahead beside two residuals, a folded input, a
    // residual with the statistics epilogue: no spill)
    constexpr int FSD = (GNIN || NRES > 0 || W == 128) && STATS ? 4 : (NRES > 1 || GNIN) ? 6 : 8;
    u32x4 bq[FSD];
    static_for<0, FSD>([&](auto kk) {
      constexpr int k = decltype(kk)::value;
      bq[k] = ds_read_b128_off<fs_koff(k)>(xrow(k));
    });
    bf16x4 rv[4], rv2[4];
    const long long m = (long long)(sbeg + st) * 128 + px;
    if (NRES > 0) {  // (a compile-time branch: a runtime one becomes a per-stage vmcnt(0))
#pragma unroll
      for (int g = 0; g < 4; ++g)
        rv[g] = *(const bf16x4*)(p.res + m * p.ldres + co0 + ch * 32 + 8 * g + 4 * h);
    }
    if (NRES > 1) {
#pragma unroll
      for (int g = 0; g < 4; ++g)
        rv2[g] = *(const bf16x4*)(p.res2 + m * p.ldres2 + co0 + ch * 32 + 8 * g + 4 * h);
    }
    f32x16 acc;  // the accumulator starts at the bias (GNIN: at zero)
    if constexpr (GNIN) acc = f32x16{};
    else acc = bias_acc;
    // stage st+3's new rows go out among this stage's MFMAs (one piece per 7):
    // their ring slots were last read in stage st-1, before the barrier that
    // ended it
    const bool pre = st + 3 < nst;  // wave-uniform
    static_for<0, 36>([&](auto kk) {
      constexpr int k = decltype(kk)::value;
      constexpr int younger = (FSD - 1 < 35 - k) ? FSD - 1 : 35 - k;
      lgkm_wait_tied<younger>(bq[k % FSD]);
      acc = Mma<bf16>::run(wA[k], bq[k % FSD], acc);
      if constexpr (k + FSD < 36) bq[k % FSD] = ds_read_b128_off<fs_koff(k + FSD)>(xrow(k + FSD));
      if constexpr (k % 7 == 3 && k / 7 < NPW) {
        if (pre) issue1(st + 3, k / 7);
      }
      // (one channel pair every FS_TSTEP k-steps: the transform's VALU spread thin between MFMAs)
      if constexpr (GNIN && k >= 1 && (k - 1) % FS_TSTEP == 0 && (k - 1) / FS_TSTEP < 4 * SEG) {
        if (tr) {  // channel pair j of row slot i: silu(A z + B) as the GroupNorm apply computes it
          constexpr int i = ((k - 1) / FS_TSTEP) >> 2, j = ((k - 1) / FS_TSTEP) & 3;
          const unsigned wd = tv[i][j];
          const f32x4 a4 = __builtin_bit_cast(f32x4, tk[j >> 1]), b4 = __builtin_bit_cast(f32x4, tk[2 + (j >> 1)]);
          gf2 t = gf2{__uint_as_float(wd << 16), __uint_as_float(wd & 0xffff0000u)} *
                      gf2{a4[(2 * j) & 3], a4[(2 * j + 1) & 3]} + gf2{b4[(2 * j) & 3], b4[(2 * j + 1) & 3]};
          const gf2 mm = t * -1.4426950408889634f;
          const gf2 d = 1.f + gf2{__builtin_amdgcn_exp2f(mm.x), __builtin_amdgcn_exp2f(mm.y)};
          t *= gf2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
          const bf16 lo = (bf16)t.x, hi = (bf16)t.y;
          tv[i][j] = (unsigned)__builtin_bit_cast(unsigned short, lo) | ((unsigned)__builtin_bit_cast(unsigned short, hi) << 16);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    });
    if constexpr (GNIN) if (tr) {  // the transformed rows back into the ring (Y(st): SEG stores)
      int ot = tid;
      asm volatile("" : "+v"(ot));
      const int gx = ot >> 3, gc = ot & 7;
#pragma unroll
      for (int i = 0; i < SEG; ++i) {
        const int q = (st + 1) * SEG + 2 + i, y = yq0 + q;
        const bool in = (unsigned)y < (unsigned)p.H;
        const u32x4 ov = in ? tv[i] : u32x4{0u, 0u, 0u, 0u};
        asm volatile("ds_write_b128 %0, %1" ::"v"(lds_addr(smem + (q % R) * ROWB + (gx + 1) * FS_XP + gc * 16)),
                     "v"(ov) : "memory");
        const bool own = in && q <= nst * SEG;
        __builtin_amdgcn_raw_buffer_store_b128(
            ov, yr, own ? (unsigned)(((fbase + y * W + gx) * p.gi_ldy + gc * 8) * 2) : DMA_OOB, 0, 0);
      }
    }
#ifdef DV_STAMP
    if (st == 1) {
      asm volatile("s_nop 0" : "+v"(acc));
      DV_S1(4);
    }
#endif
    // epilogue: lane owns pixel m, channels 8g + 4h + e of the wave's 32
    const bool silu = p.act == DV_ACT_SILU;
    float sv[stats ? 32 : 1];
    const unsigned gba = lds_addr(gi_bias + ch * 32 + 4 * h);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int n = ch * 32 + 8 * g + 4 * h;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = acc[4 * g + e];
      if constexpr (GNIN) {
        u32x4 gb = ds_read_b128_off<0>(gba + 32 * g);
        lgkm_wait_tied<0>(gb);
        const f32x4 bb = __builtin_bit_cast(f32x4, gb);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += bb[e];
      }
      if (silu) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = silu_f(v[e]);
      }
      if (NRES > 0) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += (float)rv[g][e];
      }
      if (NRES > 1) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += (float)rv2[g][e];
      }
      store4<bf16>(p.y + m * p.ldy + co0 + n, v);
      if constexpr (stats) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float q = stored<bf16>(v[e]);
          sv[4 * g + e] = q;
          sv[16 + 4 * g + e] = q * q;
        }
      }
    }
    if constexpr (stats) {
      rs_step<32, 16>(sv, r);
#pragma unroll
      for (int i = 0; i < 16; ++i) sacc[i] += sv[i];
    }
    if (st == 1) DV_S1(5);
    // stage st+1's rows landed.  vmcnt(N) = all but the wave's N youngest
    // vector-memory ops done (loads, stores, DMA in issue order).  Per stage s
    // a wave issues: its residual loads R (NR), the NPW pieces of D(s+3) (if
    // s+3 < nst) among the MFMAs, its 4 stores.  D(1), D(2) come from the
    // prologue; D(s+1), s >= 2, from stage s-2.  Younger than D(st+1):
    //   st = 0: D2, R0, D3, S0;   st = 1: R0, D3, S0, R1, D4, S1;
    //   st >= 2: S(st-2), R(st-1), D(st+2), S(st-1), R(st), D(st+3), S(st).
    // (A statistics epilogue's clip-boundary atomics only add younger ops:
    // the wait then covers more, never less.)  Every window read of this
    // stage was waited for by the last MFMA: no lgkmcnt drain.
    // GNIN waits one stage further ahead, for D(st+2) (transformed during
    // stage st+1), and a stage's transformed rows add SEG stores Y(s) before
    // its output stores.  Younger than D(st+2):
    //   st = 0: Y0, D3, Y(0), S0;   st >= 1: Y(st-1), S(st-1), D(st+3), Y(st), S(st).
    if constexpr (GNIN) {
      if (st + 2 < nst) {
        constexpr int B0 = Y0 + SEG + 4, B1 = 2 * SEG + 8;
        static_assert(B0 + NPW <= 63 && B1 + NPW <= 63, "stripe vmcnt immediate out of range");
        const bool d3 = st + 3 < nst;
        if (st == 0) {
          if (d3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(B0 + NPW) : "memory");
          else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(B0) : "memory");
        } else {
          if (d3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(B1 + NPW) : "memory");
          else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(B1) : "memory");
        }
      }
      if (tr) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the ring writes, before the barrier
    } else if (st + 1 < nst) {
      constexpr int NR = 4 * NRES;
      constexpr int A0 = NR + 4, A1 = 2 * NR + 8, A2 = 2 * NR + 12;
      static_assert(A1 + 2 * NPW <= 63 && A2 + 2 * NPW <= 63, "stripe vmcnt immediate out of range");
      const int nd = (st + 2 < nst) + (st + 3 < nst);  // DMA stages issued after D(st+1)
      if (st == 0) {
        if (nd == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(A0 + 2 * NPW) : "memory");
        else if (nd == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(A0 + NPW) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(A0) : "memory");
      } else if (st == 1) {
        if (nd == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(A1 + 2 * NPW) : "memory");
        else if (nd == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(A1 + NPW) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(A1) : "memory");
      } else {
        if (nd == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(A2 + 2 * NPW) : "memory");
        else if (nd == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(A2 + NPW) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(A2) : "memory");
      }
    }
    if (st == 1) DV_S1(6);
    __builtin_amdgcn_s_barrier();
    if (st == 0) DV_STAMP_AT(2);
    if (st == 1) DV_S1(7);
  }
  DV_STAMP_AT(3);
  if constexpr (stats) {
    // the clip of the block's last stage (block-uniform); earlier clips were
    // added per wave at the crossing (rare: stage ranges align with clips)
    __shared__ float red[2 * 64];
    rs_tail();
    if (nst > 0) gn_block_add<bf16, 32>(p, sacc, (long long)(sbeg + nst - 1) * 128 / p.gn_P, chan, red, co0, 64);
  }
}

bool fwd_stripe_ok(long long M, int h, int w, int cin, bool split, int cout, int ks, int ld0) {
  return ks == 3 && cin == 64 && !split && cout % 64 == 0 && (w == 32 || w == 64 || w == 128) &&
         h % (128 / w) == 0 && M % 128 == 0 && ld0 % 8 == 0 && M * ld0 * 2 < (long long)DMA_OOB;
}

int launch_fwd_stripe(const ConvFwdArgs<bf16>& a, hipStream_t st) {
  const int nstages = (int)(a.M / 128);
  const int ct = a.cout / 64;
  int bx = 256 / ct;
  if (bx < 1) bx = 1;
  if (bx > nstages) bx = nstages;
  // the row ring reuses rows across a workgroup's stages: its stage range
  // must lie in one frame, so stages_per_block divides the stages per frame
  const int spf = a.H / (128 / a.W);
  int sps = (nstages + bx - 1) / bx;
  if (sps >= spf) sps = spf;
  else while (spf % sps) ++sps;
  bx = (nstages + sps - 1) / sps;
  dim3 grid(bx, ct);
  const int nres = a.res2 ? 2 : a.res ? 1 : 0;
  const bool stats = a.gn_sums != nullptr;
  if (a.gi_sums) {  // (conv_fwd_gn_in checked W = 64, no residual)
    if (stats) conv_fwd_stripe_kernel<64, 0, true, true><<<grid, 512, 0, st>>>(a, nstages, sps);
    else conv_fwd_stripe_kernel<64, 0, false, true><<<grid, 512, 0, st>>>(a, nstages, sps);
    return check_launch("conv_fwd_stripe_gn_in");
  }
#define DV_FS(WW, RR) (stats ? conv_fwd_stripe_kernel<WW, RR, true><<<grid, 512, 0, st>>>(a, nstages, sps) \
                             : conv_fwd_stripe_kernel<WW, RR, false><<<grid, 512, 0, st>>>(a, nstages, sps))
  // (residuals come from dgrads only: no statistics epilogue beside them,
  // whose registers would spill; conv_fwd_t routes that pair elsewhere)
#define DV_FSR(WW) (nres == 2 ? (void)conv_fwd_stripe_kernel<WW, 2, false><<<grid, 512, 0, st>>>(a, nstages, sps) \
                    : nres == 1 ? (void)conv_fwd_stripe_kernel<WW, 1, false><<<grid, 512, 0, st>>>(a, nstages, sps) \
                                : DV_FS(WW, 0))
  // W = 64 also has the residual + statistics pairing: the second pass of a
  // dual-source conv whose GroupNorm reads its output (conv_fwd_t)
  if (a.W == 64 && nres == 1 && stats) conv_fwd_stripe_kernel<64, 1, true><<<grid, 512, 0, st>>>(a, nstages, sps);
  else if (a.W == 64) DV_FSR(64);
  else if (a.W == 128) DV_FSR(128);
  else DV_FSR(32);
#undef DV_FSR
#undef DV_FS
  return check_launch("conv_fwd_stripe");
}


// ---------------------------------------------------------------------------
// bf16 3x3 forward / dgrad, streamed-weight stripe form (cin % 32 == 0,
// cout % 64 == 0, W in {8, 16, 32, 64}; the 8x8 / 16x16 / 32x32 stage convs
// with cin >= 128 and their dgrads): one workgroup = 64 output channels x ONE
// 128-pixel stage.  The K loop runs over 32-channel half-chunks; per
// half-chunk the workgroup stages (a) its 64 channels' weights for all nine
// taps (64 x 288 bf16) and (b) the X window of the stage for those 32
// channels (one window serves all nine taps, as in the resident form).  Per
// CU that is ~52 KB of L2 traffic per 1152 MFMA cycles, against ~94 B/clk for
// the 64x128 implicit-GEMM tile it replaces.  Rows padded to 592 B (weights)
// / 80 B (window): ds_read_b128 conflict-free, immediate tap offsets.
// Register-staged, double-buffered.  8 waves: 4 pixel tiles x 2 channel
// halves, one 32x32 accumulator each.
// ---------------------------------------------------------------------------
bool stripe_geom(int h, int w, int& seg, int& nseg);

constexpr int F2_WP = 592;  // weight row pitch: 9 taps x 32 ci bf16 + 16 B
constexpr int F2_XP = 80;   // window pixel pitch: 32 ci bf16 + 16 B

template <int W, bool STATS = false>
__global__ __launch_bounds__(512) void conv_fwd_stripe2_kernel(ConvFwdArgs<bf16> p, int seg, int nseg) {
  constexpr int WP = W + 2;
  constexpr int NWIN = W == 8 ? 200 : (128 / W + 2) * WP;   // window pixels (max over H)
  constexpr int WB = 64 * F2_WP, XB = NWIN * F2_XP;
  constexpr int BUF = WB + XB;
  constexpr int NLW = (64 * 36 + 511) / 512;                // weight 16-B chunks per thread
  constexpr int NLX = (NWIN * 4 + 511) / 512;               // window 16-B chunks per thread
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int pt = wave & 3, ch = wave >> 2;
  const int co0 = blockIdx.y * 64;
  const long long m0 = (long long)blockIdx.x * 128;
  const int HW = p.H * W, segrows = (seg + 2) * WP;
  const int y0 = nseg > 1 ? 0 : (int)((m0 % HW) / W);

  // static load slots: weights (row, 16-B chunk of 36), window (pixel, chunk of 4)
  int w_src[NLW], w_dst[NLW];
#pragma unroll
  for (int i = 0; i < NLW; ++i) {
    const int idx = tid + 512 * i;
    const int row = idx / 36, c = idx - row * 36;  // c: tap = c / 4, 8-ci group = c % 4
    const bool ok = row < 64;
    w_src[i] = ok ? (co0 + row) * p.K + (c >> 2) * p.cin + (c & 3) * 8 : -1;
    w_dst[i] = row * F2_WP + c * 16;
  }
  int x_off[NLX], x_ry[NLX], x_dst[NLX], x_c[NLX];
#pragma unroll
  for (int i = 0; i < NLX; ++i) {
    const int idx = tid + 512 * i;
    const int px = idx >> 2, c = idx & 3;
    const int sg = px / segrows, rem = px - sg * segrows;
    const int ry = rem / WP, rx = rem - ry * WP;
    const bool ok = px < NWIN && sg < nseg && rx >= 1 && rx <= W;
    x_ry[i] = ok ? ry - 1 : -(1 << 20);
    x_off[i] = sg * seg * W + (ry - 1) * W + (rx - 1);
    x_dst[i] = px < NWIN ? px * F2_XP + c * 16 : -1;
    x_c[i] = c * 8;
  }
  u32x4 rw[NLW], rx_[NLX];
  auto load = [&](int hc) {
    const int ci = hc * 32;
    const bool first = ci < p.c0;
    const bf16* xb = first ? p.x0 + ci : p.x1 + (ci - p.c0);
    const int ld = first ? p.ld0 : p.ld1;
#pragma unroll
    for (int i = 0; i < NLW; ++i)
      if (w_src[i] >= 0) rw[i] = *(const u32x4*)(p.w + w_src[i] + ci);
#pragma unroll
    for (int i = 0; i < NLX; ++i) {
      const bool in = (unsigned)(y0 + x_ry[i]) < (unsigned)p.H;
      rx_[i] = in ? *(const u32x4*)(xb + (m0 + x_off[i]) * ld + x_c[i]) : u32x4{0u, 0u, 0u, 0u};
    }
  };
  auto store = [&](int buf) {
    char* b = smem + buf * BUF;
#pragma unroll
    for (int i = 0; i < NLW; ++i)
      if (w_src[i] >= 0) *(u32x4*)(b + w_dst[i]) = rw[i];
#pragma unroll
    for (int i = 0; i < NLX; ++i)
      if (x_dst[i] >= 0) *(u32x4*)(b + WB + x_dst[i]) = rx_[i];
  };

  const int r = lane & 31, h = lane >> 5;
  const int px = pt * 32 + r;
  const int sl = px / (seg * W), rl = px - sl * seg * W;
  const int wrow = sl * segrows + (rl / W) * WP + rl % W;
  const int aofs = (ch * 32 + r) * F2_WP + h * 16;
  const int bofs = WB + wrow * F2_XP + h * 16;

  f32x16 acc[1][1];
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[0][0][e] = 0.f;
  const int nhc = p.cin / 32;
  load(0);
  store(0);
  __syncthreads();
  for (int hc = 0; hc < nhc; ++hc) {
    if (hc + 1 < nhc) load(hc + 1);
    const char* b = smem + (hc & 1) * BUF;
#pragma unroll
    for (int d = 0; d < 9; ++d) {
      const int toff = ((d / 3) * WP + (d % 3)) * F2_XP;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const u32x4 av = *(const u32x4*)(b + aofs + (d * 32 + ks * 16) * 2);
        const u32x4 bv = *(const u32x4*)(b + bofs + toff + ks * 32);
        acc[0][0] = Mma<bf16>::run(av, bv, acc[0][0]);
      }
    }
    if (hc + 1 < nhc) store((hc + 1) & 1);
    __syncthreads();
  }
  conv_epilogue<bf16, 1, 1, STATS>(p, acc, m0 + pt * 32, co0 + ch * 32, r, h, m0, 128, co0, 64,
                                   (float*)smem);
}

bool fwd_stripe2_ok(long long M, int h, int w, int cin, int c0, bool split, int cout, int ks, int& seg,
                    int& nseg) {
  if (ks != 3 || cin % 32 || (split && c0 % 32) || cout % 64 || M % 128 || !stripe_geom(h, w, seg, nseg))
    return false;
  // measured against the glds implicit GEMM (tools/ab_fwd.sh): the streamed
  // stripe wins on the whole-frame windows of the 8x8 stage and on the
  // smaller 16x16 convs; at W >= 32 the deep-ring glds tiles win
  return w == 8 || (w == 16 && (long long)cin * cout <= 256 * 256);
}

int launch_fwd_stripe2(const ConvFwdArgs<bf16>& a, int seg, int nseg, hipStream_t st) {
  dim3 grid((unsigned)(a.M / 128), a.cout / 64);
  switch (a.W) {
#define DV_S2(WW) (a.gn_sums ? conv_fwd_stripe2_kernel<WW, true><<<grid, 512, 0, st>>>(a, seg, nseg) \
                          : conv_fwd_stripe2_kernel<WW, false><<<grid, 512, 0, st>>>(a, seg, nseg))
    case 64: DV_S2(64); break;
    case 32: DV_S2(32); break;
    case 16: DV_S2(16); break;
    default: DV_S2(8); break;
#undef DV_S2
  }
  return check_launch("conv_fwd_stripe2");
}

// ---------------------------------------------------------------------------
// bf16 3x3 forward / dgrad, "window" form, for frame widths W = 8 (H = 8),
// 16, 32, 64 (H*W % 128 == 0): the Unet3D 8x8 / 16x16 / 32x32 / 64x64
// stage convs with cin % 16 == 0 and cout % 64 == 0, and their dgrads.
// Weights are packed 16-channel-chunk-major (dv_pack_conv_weight modes 2 /
// 3), so a chunk of a weight row is one contiguous 288-B run (with [tap][ci]
// rows every 16-channel piece was a separate 32-B request and L2 moved twice
// the bytes).  One workgroup = 128 pixels (two 8x8 frames, or 128 / W rows
// of one frame) x 64 output channels, 4 waves; each wave owns 32 pixels x
// 64 channels (two 32x32 accumulators sharing one window fragment: 1.5 LDS
// reads per MFMA, against 2 for one accumulator per wave).  K runs over
// 16-channel chunks: per chunk the block's 64 weight rows (9 taps x 16 ci)
// and the pixel window (zero halo) arrive by LDS-DMA into a 4-5 deep ring;
// counted vmcnt + one raw barrier per chunk; the chunk offset rides in the
// DMA's SGPR soffset; no VGPR staging.
// Window image: rows of WQ pixel slots, 3 16-B slots per pixel (2 data +
// pad).  Lanes map to pixels (fw_pix) so that each ds_read_b128 16-lane
// group takes one pixel of every residue of the window index mod 16 (for
// W = 8 the row pitch 12 makes every residue occur exactly twice among a
// wave's 32 pixels): with the odd slot pitch every window read is
// conflict-free for all nine taps.  Weight rows: 19 slots (odd): conflict-
// free.  Blocks are ordered so that one XCD works on one output-channel
// block at a time (its 64 weight rows stay in that XCD's L2).
// Measured (512->512 at 8x8, 64 frames): 44 us (stripe2) -> 28 us.
// ---------------------------------------------------------------------------
// Window geometry per frame width (a 128-pixel tile: two 8x8 frames, or
// 128 / W rows of one frame when H*W % 128 == 0): window rows NWR of WQ pixel
// slots (W + 2 used; W = 8 pads to 12 so the residues work out, see above),
// three 16-B slots per pixel.
constexpr int F8_WROW = 19;                                // 16-B slots per weight row
// CO output channels per tile: 64 (two 32x32 accumulators per wave), or 32
// for the grids that would leave CUs idle (M = 4,096 at 256 channels: 128
// tiles of 64 channels for 256 CUs)
template <int W, int CO = 64, int NWV = 4, int NB = 0>
struct FwGeom {
  static constexpr int CG = CO * (NWV / 4);                  // channels per workgroup
  static constexpr int NF = W == 8 ? 2 : 1;                  // frames per tile
  static constexpr int NWR = W == 8 ? 10 : 128 / W + 2;      // window rows per frame
  static constexpr int WQ = W == 8 ? 12 : W + 2;             // pixel slots per window row
  static constexpr int FPIX = NWR * WQ;                      // window pixels per frame
  static constexpr int WPIX = NF * FPIX;
  static constexpr int XPIECES = (WPIX * 3 + 63) / 64;
  static constexpr int WPC = (CG * F8_WROW + 63) / 64;       // CG weight rows x 19 slots
  static constexpr int PIECES = WPC + XPIECES;
  static constexpr int NPW = (PIECES + NWV - 1) / NWV;
  static constexpr int BUF = PIECES * 1024;
  static constexpr int NBUF = NB ? NB : ((160 * 1024 - 1024) / BUF >= 5 ? 5 : (160 * 1024 - 1024) / BUF);
};

// lane r -> pixel (row * W + col) of the wave's 32-pixel tile so that the
// ds_read_b128 16-lane group {0-3, 12-15, 20-27} and its complement each take
// one pixel of every residue of the window index mod 16:
//   W = 8 (4 rows x 8): group A rows 0 and 2, the rest rows 1 and 3
//   W = 16 (2 rows x 16): group A row 0, the rest row 1
//   W >= 32 (32 columns of one row): group A columns 0-15, the rest 16-31
template <int W>
__device__ __forceinline__ int fw_pix(int r) {
  const bool ga = r < 4 || (r >= 12 && r < 16) || (r >= 20 && r < 28);
  const int a = ga ? (r < 4 ? r : (r < 16 ? r - 8 : r - 12))
                   : (r < 12 ? r - 4 : (r < 20 ? r - 8 : r - 16));
  if constexpr (W == 8) return (2 * (a >> 3) + (ga ? 0 : 1)) * 8 + (a & 7);
  else if constexpr (W == 16) return (ga ? 0 : 16) + a;
  else return (ga ? 0 : 16) + a;
}

// NWV = 8: a 128-pixel x 2*CO-channel tile per workgroup, waves 4-7 on the
// second channel half (the pixel window is staged once for both halves): for
// the grids whose CO-channel tiles would run in two rounds on the 256 CUs.
// TS (tap split, round 5; NWV = 8): the same 128 x CO tile as 4 waves, but 8
// waves, waves 4-7 taking taps 5-8 of every chunk and waves 0-3 taps 0-4:
// two waves per SIMD on the M = 4,096 grids whose tile count already equals
// the CU count (one tile per CU leaves one wave per SIMD to hide every LDS /
// DMA latency with its own MFMAs).  Same ring, same LDS reads and DMA pieces
// per MFMA; the halves' partial sums meet in LDS and each half stores 32 of
// the CO channels.
// (Measured and removed in round 5, see DESIGN.md: a K split over two
// workgroups per tile, register staging, one barrier per two chunks.)
template <int W, bool STATS = false, int PF = 2, int DEFER = 0, int CO = 64, bool SPLIT = true, int NWV = 4,
          bool TS = false>
__global__ __launch_bounds__(NWV * 64) void conv_fwd_frame_kernel(ConvFwdArgs<bf16> p) {
  using G = FwGeom<W, CO, TS ? 4 : NWV>;
  constexpr int PIECES = G::PIECES, BUF = G::BUF, NBUF = G::NBUF, WQ = G::WQ;
  constexpr int NPW = (PIECES + NWV - 1) / NWV;  // DMA pieces per wave per chunk
  constexpr int WPC = G::WPC, NJ = TS ? 1 : CO / 32, CG = G::CG;
  static_assert(NWV == 4 || (NWV == 8 && (TS || !STATS)), "the 8-wave 2*CO tile has no statistics epilogue");
  static_assert(!TS || (NWV == 8 && CO == 64), "the tap split runs 8 waves on a 64-channel tile");
  static_assert(NPW <= 9, "one DMA piece per tap");
  __shared__ __attribute__((aligned(1024))) char smem[NBUF * BUF];
  DV_STAMP_AT(0);
  const int tid = threadIdx.x, lane = tid & 63;
  // masked: the DMA piece type folds per (wave, i) at compile time
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6) & (NWV - 1);
  const int wq = wave & 3;                    // pixel sub-tile
  const int chh = TS ? 0 : wave >> 2;         // channel half (NWV = 8 without TS)
  const int half = TS ? wave >> 2 : 0;        // tap half (TS)
  const int npx = (int)(p.M / 128), nblk = npx * (p.cout / CG);
  int L = blockIdx.x;
  int co0;
  long long m0;
  if (p.xcd_c > 0) {
    // XCD x = block % 8 takes channel group x / xp and pixel group x % xp: its
    // L2 holds 1/xc of the weights and 1/xp of the input (host-checked splits)
    const int xc = p.xcd_c, xp = 8 / xc, x = L % 8, j = L / 8;
    const int tpc = (p.cout / CG) / xc, ppg = npx / xp;
    co0 = ((x / xp) * tpc + j / ppg) * CG;
    m0 = (long long)((x % xp) * ppg + j % ppg) * 128;
  } else {
    if (nblk % 8 == 0) L = (L % 8) * (nblk / 8) + L / 8;  // consecutive blocks share an XCD
    co0 = (L / npx) * CG;
    m0 = (long long)(L % npx) * 128;
  }
  const int cbeg = 0, cend = p.cin / 16;
  const int nch = cend - cbeg;  // 16-channel chunks
  const int HW = p.H * W;
  const int y0 = W == 8 ? 0 : (int)((m0 % HW) / W);        // tile's first image row
  const long long fb = W == 8 ? m0 : m0 - (m0 % HW) + (long long)y0 * W;  // pixel of (y0, 0)

  // this lane's slot of each of the wave's DMA pieces: a fixed byte offset
  // (or DMA_OOB); the chunk's offset rides in the instruction's soffset
  unsigned voff0[NPW], voff1[NPW];
#pragma unroll
  for (int i = 0; i < NPW; ++i) {
    const int k = min(wave + NWV * i, PIECES - 1);
    voff0[i] = voff1[i] = DMA_OOB;
    if (k < WPC) {
      // chunk-major packed row (mode 2/3): [cin / 16][9 taps][16]; slot c = 2 tap + half
      const int slot = k * 64 + lane, row = slot / F8_WROW, c = slot - row * F8_WROW;
      if (c < 18 && row < CG) voff0[i] = (unsigned)((((long long)co0 + row) * p.K + c * 8) * 2);
    } else {
      const int slot = (k - WPC) * 64 + lane, px = slot / 3, s = slot - px * 3;
      const int f = px / G::FPIX, rem = px - f * G::FPIX, wy = rem / WQ, wx = rem - wy * WQ;
      const int y = y0 + wy - 1;  // image row (W = 8: within frame f of the tile)
      if (px < G::WPIX && s < 2 && wx >= 1 && wx <= W && y >= 0 && y < p.H &&
          (W == 8 || wy <= 128 / W + 1)) {
        const long long pix = fb + (long long)f * 64 + (long long)(wy - 1) * W + (wx - 1);
        voff0[i] = (unsigned)(pix * p.ld0 * 2 + s * 16);
        voff1[i] = (unsigned)(pix * p.ld1 * 2 + s * 16);
      }
    }
  }
  const __amdgpu_buffer_rsrc_t wr = dma_rsrc(p.w, (unsigned)((long long)p.cout * p.K * 2));
  const __amdgpu_buffer_rsrc_t xr0 = dma_rsrc(p.x0, (unsigned)(p.M * p.ld0 * 2));
  const __amdgpu_buffer_rsrc_t xr1 = dma_rsrc(p.x1, (unsigned)(p.M * p.ld1 * 2));
  // piece i of chunk c (i < NPW)
  auto issue1 = [&](int c, int i) {
    const int ci0 = c * 16;
    const bool first = ci0 < p.c0;
    char* b = smem + (c % NBUF) * BUF;
    const int k = min(wave + NWV * i, PIECES - 1);
    if (k < WPC) dma16s(wr, b + k * 1024, voff0[i], (unsigned)ci0 * 18);
    else if (!SPLIT || first) dma16s(xr0, b + k * 1024, voff0[i], (unsigned)ci0 * 2);
    else dma16s(xr1, b + k * 1024, voff1[i], (unsigned)(ci0 - p.c0) * 2);
  };
  auto issue = [&](int c) {
#pragma unroll
    for (int i = 0; i < NPW; ++i) issue1(c, i);
  };
  constexpr int AHEAD = NBUF - 1;  // chunks in flight beyond the one being read
  // prologue: chunks cbeg .. cbeg+AHEAD-1 in flight, wait for chunk cbeg
#pragma unroll
  for (int c = 0; c < AHEAD; ++c)
    if (c < nch) issue(cbeg + c);
  {
    const int pro = min(AHEAD, nch) - 1;  // younger chunks than chunk 0
    if (pro >= 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * NPW) : "memory");
    else if (pro == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NPW) : "memory");
    else if (pro == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NPW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  DV_STAMP_AT(1);
#ifdef DV_STAMP
  // diagnostic: one wave's (FRAME_STAMP_WAVE, default 0) shader-clock totals
  // over the chunk loop of its time at the DMA wait and at the barrier
  // (stamps 5, 6) and of the whole loop (7)
  unsigned long long st_wait = 0, st_bar = 0;
  const unsigned long long st_l0 = __builtin_amdgcn_s_memtime();
#endif

  const int r = lane & 31, h = lane >> 5;
  const int pix = fw_pix<W>(r);                    // within the wave's 32 pixels
  const int tpx = wq * 32 + pix;                   // within the 128-pixel tile
  const int wb = W == 8 ? (tpx >> 6) * G::FPIX + ((tpx & 63) >> 3) * WQ + (tpx & 7)
                        : (tpx / W) * WQ + tpx % W;  // window pixel of tap (0, 0)
  const int bofs = WPC * 1024 + (wb * 3 + h) * 16;
  const int aofs = (chh * CO + r) * (F8_WROW * 16) + h * 16;
  // two accumulator chains per channel half (even / odd taps): four
  // independent MFMA chains, summed in the epilogue
  f32x16 acc0, acc1, acc2, acc3;
#pragma unroll
  for (int e = 0; e < 16; ++e) acc0[e] = acc1[e] = acc2[e] = acc3[e] = 0.f;
  // DEFER: the last tap's MFMAs of chunk c run after the chunk's barrier, while
  // chunk c+1's first fragment reads are in flight (its operands are in
  // registers before the barrier, so the buffer may be refilled under them)
  // DEFER = 2: taps 7 and 8 (slot 0: tap 7, odd -> chains 2 / 3; slot 1: tap 8)
  static_assert(DEFER <= 2, "at most the last two taps are deferred");
  u32x4 lb[2], la0[2], la1[2];
  auto run_deferred = [&](auto HALF) {
    constexpr int D1 = TS && decltype(HALF)::value == 0 ? 5 : 9;  // the half's last tap + 1
#pragma unroll
    for (int t = 0; t < DEFER; ++t) {
      const int tap = D1 - DEFER + t;
      if (tap & 1) {
        acc2 = Mma<bf16>::run(la0[t], lb[t], acc2);
        if (CO == 64) acc3 = Mma<bf16>::run(la1[t], lb[t], acc3);
      } else {
        acc0 = Mma<bf16>::run(la0[t], lb[t], acc0);
        if (CO == 64) acc1 = Mma<bf16>::run(la1[t], lb[t], acc1);
      }
    }
  };
  // the deferred fragments are in registers before the barrier (their
  // buffer may be refilled behind it)
  auto defer_wait = [&]() {
    if (DEFER == 2 && CO == 64)
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(lb[0]), "+v"(la0[0]), "+v"(la1[0]), "+v"(lb[1]), "+v"(la0[1]),
                   "+v"(la1[1])::"memory");
    else if (DEFER == 2)
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(lb[0]), "+v"(la0[0]), "+v"(lb[1]), "+v"(la0[1])::"memory");
    else if (DEFER && CO == 64)
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(lb[0]), "+v"(la0[0]), "+v"(la1[0])::"memory");
    else if (DEFER)
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(lb[0]), "+v"(la0[0])::"memory");
    else
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };
  // one chunk; PRE (compile-time): chunk c + AHEAD exists and is issued here.
  // The loop is split into the chunks that issue and the AHEAD tail, so the
  // main loop carries no per-piece branch and a constant vmcnt
  auto chunk = [&](int c, auto PRE, auto HALF) {
    const char* b = smem + (c % NBUF) * BUF;
    // this wave's taps [D0, D1): all nine, or one half of them (TS)
    constexpr int D0 = TS && decltype(HALF)::value == 1 ? 5 : 0;
    constexpr int D1 = TS && decltype(HALF)::value == 0 ? 5 : 9;
    // fragments of tap d + PF are read while tap d multiplies (one wave per
    // SIMD: the LDS latency is hidden by this wave's own MFMAs only)
    constexpr int NS = PF + 1;
    u32x4 bq[NS], aq0[NS], aq1[NS];
    auto rd = [&](int d, int s) {
      const int T = ((d / 3) * WQ + (d % 3)) * 48;
      bq[s] = *(const u32x4*)(b + bofs + T);
      aq0[s] = *(const u32x4*)(b + aofs + d * 32);
      if (CO == 64) aq1[s] = *(const u32x4*)(b + aofs + 32 * F8_WROW * 16 + d * 32);
    };
#pragma unroll
    for (int d = D0; d < D0 + PF; ++d) rd(d, d % NS);
    if (DEFER && c > cbeg) run_deferred(HALF);  // the last taps of chunk c-1
    // chunk c+AHEAD's pieces go out one per tap, in the MFMA shadow: its
    // buffer was last read in chunk c-1, before the last barrier
#pragma unroll
    for (int d = D0; d < D1; ++d) {
      if (d + PF < D1) rd(d + PF, (d + PF) % NS);
      if (DEFER && d >= D1 - DEFER) {
        const int t = d - (D1 - DEFER);
        lb[t] = bq[d % NS];
        la0[t] = aq0[d % NS];
        if (CO == 64) la1[t] = aq1[d % NS];
      } else if (d & 1) {
        acc2 = Mma<bf16>::run(aq0[d % NS], bq[d % NS], acc2);
        if (CO == 64) acc3 = Mma<bf16>::run(aq1[d % NS], bq[d % NS], acc3);
      } else {
        acc0 = Mma<bf16>::run(aq0[d % NS], bq[d % NS], acc0);
        if (CO == 64) acc1 = Mma<bf16>::run(aq1[d % NS], bq[d % NS], acc1);
      }
      if constexpr (decltype(PRE)::value) {
        if (d - D0 < NPW) issue1(c + AHEAD, d - D0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // chunk c+1 landed: younger are the pieces of chunks c+2 .. c+AHEAD
#ifdef DV_STAMP
    const unsigned long long tw0 = __builtin_amdgcn_s_memtime();
#endif
    if constexpr (decltype(PRE)::value) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((AHEAD - 1) * NPW) : "memory");
    } else {
      const int young = min(c + AHEAD, cend - 1) - (c + 1);
      if (young >= 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * NPW) : "memory");
      else if (young == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NPW) : "memory");
      else if (young == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NPW) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (DEFER) defer_wait();
#ifdef DV_STAMP
    const unsigned long long tw1 = __builtin_amdgcn_s_memtime();
#endif
    __builtin_amdgcn_s_barrier();
#ifdef DV_STAMP
    const unsigned long long tw2 = __builtin_amdgcn_s_memtime();
    st_wait += tw1 - tw0;
    st_bar += tw2 - tw1;
#endif
  };
  using H0 = std::integral_constant<int, 0>;
  using H1 = std::integral_constant<int, 1>;
  int c = cbeg;
  if (half == 0) {  // wave-uniform
    for (; c + AHEAD < cend; ++c) chunk(c, std::true_type{}, H0{});
    for (; c < cend; ++c) chunk(c, std::false_type{}, H0{});
    if (DEFER && nch > 0) run_deferred(H0{});
  } else {
    for (; c + AHEAD < cend; ++c) chunk(c, std::true_type{}, H1{});
    for (; c < cend; ++c) chunk(c, std::false_type{}, H1{});
    if (DEFER && nch > 0) run_deferred(H1{});
  }
  DV_STAMP_AT(2);
#ifdef DV_STAMP
#ifndef FRAME_STAMP_WAVE
#define FRAME_STAMP_WAVE 0
#endif
  if (threadIdx.x == 64 * (FRAME_STAMP_WAVE < NWV ? FRAME_STAMP_WAVE : NWV - 1)) {
    const long long blin = blockIdx.x + (long long)gridDim.x * (blockIdx.y + (long long)gridDim.y * blockIdx.z);
    if (blin < 16384) {
      g_dv_stamp[blin * DV_NSTAMP + 5] = st_wait;
      g_dv_stamp[blin * DV_NSTAMP + 6] = st_bar;
      g_dv_stamp[blin * DV_NSTAMP + 7] = __builtin_amdgcn_s_memtime() - st_l0;
    }
  }
#endif
  // per output-channel group j of this wave: the accumulated sum (two tap
  // chains).  TS: each half holds partial sums of all CO channels; half 0
  // keeps channels [0, 32) and half 1 [32, 64), the other half's part of
  // them arriving through LDS (the ring is dead: every wave passed the last
  // chunk's barrier)
  f32x16 fin[NJ];
  if constexpr (TS) {
    f32x16 keep, give;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const float s0 = acc0[e] + acc2[e], s1 = acc1[e] + acc3[e];
      keep[e] = half ? s1 : s0;
      give[e] = half ? s0 : s1;
    }
    f32x4* xb = (f32x4*)smem;  // [2 halves][4 pixel groups][4][64 lanes]
#pragma unroll
    for (int g = 0; g < 4; ++g)
      xb[((half * 4 + wq) * 4 + g) * 64 + lane] = f32x4{give[4 * g], give[4 * g + 1], give[4 * g + 2], give[4 * g + 3]};
    __syncthreads();
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 o = xb[(((1 - half) * 4 + wq) * 4 + g) * 64 + lane];
#pragma unroll
      for (int e = 0; e < 4; ++e) keep[4 * g + e] += o[e];
    }
    fin[0] = keep;
  } else {
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) fin[j][e] = j ? acc1[e] + acc3[e] : acc0[e] + acc2[e];
  }
  // epilogue: lane owns pixel m, channels co0 + 32j + 8g + 4h + e.  Bias and
  // residual are loaded for all 8 channel groups BEFORE the first store (vmcnt
  // retires loads and stores in order: a load behind a store waits for the
  // write, one round trip per group when they interleaved)
  const long long m = m0 + tpx;
  const int cw = co0 + chh * CO + half * 32;  // this wave's first output channel
  constexpr int NSV = 32 * NJ;                // STATS: [0, 16 NJ) sums, then squares, of the lane's channels
  float sv[STATS ? NSV : 1];
  f32x4 bb[NJ][4];
  u32x2 rq[NJ][4], rq2[NJ][4];
  if (p.bias) {
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) bb[j][g] = *(const f32x4*)(p.bias + cw + 32 * j + 8 * g + 4 * h);
  }
  if (p.res) {
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) rq[j][g] = *(const u32x2*)(p.res + m * p.ldres + cw + 32 * j + 8 * g + 4 * h);
  }
  if (p.res2) {
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) rq2[j][g] = *(const u32x2*)(p.res2 + m * p.ldres2 + cw + 32 * j + 8 * g + 4 * h);
  }
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int n = cw + 32 * j + 8 * g + 4 * h;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = fin[j][4 * g + e];
      if (p.bias) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += bb[j][g][e];
      }
      if (p.act == DV_ACT_SILU) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = silu_f(v[e]);
      }
      if (p.res) {
        const bf16x4 t4 = __builtin_bit_cast(bf16x4, rq[j][g]);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += (float)t4[e];
      }
      if (p.res2) {
        const bf16x4 t4 = __builtin_bit_cast(bf16x4, rq2[j][g]);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += (float)t4[e];
      }
      store4<bf16>(p.y + m * p.ldy + n, v);
      if constexpr (STATS) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float q = stored<bf16>(v[e]);
          sv[16 * j + 4 * g + e] = q;
          sv[NSV / 2 + 16 * j + 4 * g + e] = q * q;
        }
      }
    }
  }
  if constexpr (STATS) {  // the host requires gn_P % 128 == 0: the tile is in one clip
    gn_rs_reduce<NSV>(sv, r);
    gn_block_add<bf16, NSV>(p, sv, m0 / p.gn_P, [&](int k) {
      return cw + 32 * (k / 16) + 8 * ((k % 16) / 4) + 4 * h + (k % 4);
    }, (float*)smem, co0, CG);
  }
#ifdef DV_STAMP
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  DV_STAMP_AT(4);
}

bool fwd_frame_ok(const ConvFwdArgs<bf16>& a, int h, int w) {
  const long long maxb = (long long)DMA_OOB;
  const bool geom = (h == 8 && w == 8) || ((w == 16 || w == 32 || w == 64) && (h * w) % 128 == 0);
  return a.ks == 3 && geom && a.cin % 16 == 0 && a.c0 % 16 == 0 && a.cout % 64 == 0 &&
         a.M % 128 == 0 && a.ld0 % 8 == 0 && a.ld1 % 8 == 0 && (a.ldy & 3) == 0 &&
         (a.res == nullptr || (a.ldres & 3) == 0) && (a.res2 == nullptr || (a.ldres2 & 3) == 0) &&
         a.M * a.ld0 * 2 < maxb &&
         a.M * a.ld1 * 2 < maxb && (long long)a.cout * a.K * 2 < maxb &&
         ((uintptr_t)a.x0 & 15) == 0 && ((uintptr_t)a.x1 & 15) == 0 && ((uintptr_t)a.w & 15) == 0;
}

// channel x pixel split of the window conv's tiles over the 8 XCDs that
// minimises the L2 fill traffic xp * |w| + xc * |x| (each XCD's L2 reads its
// 1/xc of the weights and 1/xp of the input once)
int frame_xcd_split(const ConvFwdArgs<bf16>& a, int co) {
  const int ntco = a.cout / co, npx = (int)(a.M / 128);
  auto ok = [&](int xc) { return ntco % xc == 0 && npx % (8 / xc) == 0; };
  const double wb = (double)a.cout * a.K, xb = (double)a.M * a.cin;
  int best = 0;
  double bc = 0;
  for (int xc = 1; xc <= 8; xc *= 2) {
    if (!ok(xc)) continue;
    const double c = (8 / xc) * wb + xc * xb;
    if (!best || c < bc) { best = xc; bc = c; }
  }
  return best;
}

int launch_fwd_frame(const ConvFwdArgs<bf16>& a0, hipStream_t st) {
  ConvFwdArgs<bf16> a = a0;
  const int tiles64 = (int)(a.M / 128) * (a.cout / 64);
  // grids of <= 128 64-channel tiles (half the CUs): 32-channel tiles
  const int co = tiles64 <= 128 ? 32 : 64;
  // 8 waves on 128 channels for the 16-wide frames whose 64-channel tiles
  // would take two rounds of the 256 CUs
  const bool w8 = a.W == 16 && co == 64 && !a.gn_sums && a.cout % 128 == 0 && (a.M / 128) * (a.cout / 64) > 256;
  a.xcd_c = frame_xcd_split(a, w8 ? 128 : co);
  const int nblk = (int)(a.M / 128) * (a.cout / (w8 ? 128 : co));
  if (w8) {
    if (a.c0 < a.cin) conv_fwd_frame_kernel<16, false, 3, 1, 64, true, 8><<<nblk, 512, 0, st>>>(a);
    else conv_fwd_frame_kernel<16, false, 3, 1, 64, false, 8><<<nblk, 512, 0, st>>>(a);
    return check_launch("conv_fwd_frame");
  }
  // fragment prefetch distance PF = 3 taps and DEFER (the last tap's MFMAs
  // after the chunk barrier): same-box per-launch A/B (tools/frame_ab.py,
  // profiles/r03_frame_ab.txt) put PF 3 + DEFER 1 1-3 % ahead of PF 2 without
  // the deferral
  // 8x8 frames with 64-channel tiles: the tap split (two waves per SIMD)
  if (a.W == 8 && co == 64) {
#define DV_FTS(SP) (a.gn_sums ? conv_fwd_frame_kernel<8, true, 3, 1, 64, SP, 8, true><<<nblk, 512, 0, st>>>(a) \
                              : conv_fwd_frame_kernel<8, false, 3, 1, 64, SP, 8, true><<<nblk, 512, 0, st>>>(a))
    if (a.c0 < a.cin) DV_FTS(true);
    else DV_FTS(false);
#undef DV_FTS
    return check_launch("conv_fwd_frame");
  }
  switch (a.W) {
#define DV_FW5(WW, C, SP) (a.gn_sums ? conv_fwd_frame_kernel<WW, true, 3, 1, C, SP><<<nblk, 256, 0, st>>>(a) \
                                 : conv_fwd_frame_kernel<WW, false, 3, 1, C, SP><<<nblk, 256, 0, st>>>(a))
  // SPLIT: the input is a channel concat of two sources (the up-path skips)
#define DV_FW4(WW, C) (a.c0 < a.cin ? DV_FW5(WW, C, true) : DV_FW5(WW, C, false))
#define DV_FW(WW) (co == 32 ? DV_FW4(WW, 32) : DV_FW4(WW, 64))
    case 8: DV_FW(8); break;
    case 16: DV_FW(16); break;
    case 32: DV_FW(32); break;
    default: DV_FW(64); break;
#undef DV_FW
#undef DV_FW4
#undef DV_FW5
  }
  return check_launch("conv_fwd_frame");
}

// tile choice for the glds path (mirrored by ops.conv_tile for kernel naming)
inline void glds_tile(long long M, int cout, int K, int& bm, int& bn) {
  // (64-channel tiles where 128-channel ones leave a half-empty column, cout =
  // 192, measured slower: profiles/r04k_ragged_tiles_ab.txt)
  bn = cout <= 64 ? 64 : 128;
  bm = bn == 64 ? 256 : 128;
  if (((M + bm - 1) / bm) * ((cout + bn - 1) / bn) < 512) bm = 128;
  // fewer 128-pixel tiles than CUs (8x8 stage, mid block): halve the pixel tile
  if (bn == 128 && ((M + 127) / 128) * ((cout + 127) / 128) < 256) bm = 64;
  // (K <= 128, the memory-bound 1x1 convs: smaller tiles / more resident
  // workgroups measured no faster, tools/k1x1.py: 4.2 TB/s either way)
  (void)K;
}

// the statistics epilogue's fields (off when gn_sums is null)
template <typename T>
void set_gn(ConvFwdArgs<T>& a, float* gn_sums, long long gn_P, int gn_R) {
  a.gn_sums = gn_sums;
  a.gn_P = gn_sums ? gn_P : 1;
  a.gn_R = gn_R > 0 ? gn_R : 1;
  a.gn_rstride = gn_sums ? (a.M / a.gn_P) * a.cout * 2 : 0;
}

template <typename T>
int conv_fwd_t(const void* x0, int ld0, int c0, const void* x1, int ld1, const void* w,
               const float* bias, const void* res, int ldres, const void* res2, int ldres2, void* y,
               int ldy, int nf, int h, int wd, int cin, int cout, int ks, int act, float* gn_sums,
               long long gn_P, int gn_R, hipStream_t st) {
  if (!res && res2) {  // a lone second residual is the first
    res = res2; ldres = ldres2; res2 = nullptr; ldres2 = 0;
  }
  ConvFwdArgs<T> a;
  a.x0 = (const T*)x0; a.x1 = (const T*)(x1 ? x1 : x0); a.ld0 = ld0; a.ld1 = x1 ? ld1 : ld0;
  a.c0 = x1 ? c0 : cin; a.w = (const T*)w; a.bias = bias; a.res = (const T*)res;
  a.ldres = ldres; a.res2 = (const T*)res2; a.ldres2 = ldres2;
  a.y = (T*)y; a.ldy = ldy; a.H = h; a.W = wd; a.cin = cin; a.cout = cout;
  a.ks = ks; a.act = act; a.M = (long long)nf * h * wd; a.K = ks * ks * cin;
  set_gn(a, gn_sums, gn_P, gn_R);
  if (a.M == 0 || cout == 0) return DV_OK;
  if constexpr (sizeof(T) == 2) {
    // a 3x3 conv over a 64 + 64 channel concat (the 64^2 up-path block1 convs,
    // dalle2_video.py:926-945): two resident-weight stripe passes, one per
    // source -- pass 2 adds onto pass 1's output in its residual epilogue
    // (in place: each lane reads its pixel's y before it stores it).  Measured
    // against the glds implicit GEMM it replaces: DESIGN.md §3.
    if (x1 && c0 == 64 && cin == 128 && act == DV_ACT_NONE && (!gn_sums || (wd == 64 && gn_P % 128 == 0)) &&
        !res2 && ld1 % 8 == 0 &&
        fwd_stripe_ok(a.M, h, wd, 64, false, cout, ks, ld0) && a.M * ld1 * 2 < (long long)DMA_OOB &&
        (ldy & 3) == 0 && (res == nullptr || (ldres & 3) == 0)) {
      ConvFwdArgs<T> p1 = a;
      p1.cin = 64; p1.c0 = 64; p1.x1 = p1.x0; p1.ld1 = p1.ld0; p1.K = ks * ks * 64;
      p1.wcin = 128; p1.wc0 = 0;
      set_gn(p1, nullptr, 0, 0);  // statistics of the final sum: pass 2's epilogue
      const int rc = launch_fwd_stripe(p1, st);
      if (rc != DV_OK) return rc;
      ConvFwdArgs<T> p2 = p1;
      p2.x0 = a.x1; p2.ld0 = a.ld1; p2.x1 = a.x1; p2.ld1 = a.ld1; p2.wc0 = 64;
      p2.bias = nullptr; p2.res = a.y; p2.ldres = ldy;
      set_gn(p2, gn_sums, gn_P, gn_R);
      return launch_fwd_stripe(p2, st);
    }
    // the stripe kernel flushes statistics per 128-pixel stage: clips must
    // be whole stages
    if (fwd_stripe_ok(a.M, h, wd, cin, x1 != nullptr, cout, ks, ld0) && (ldy & 3) == 0 &&
        (res == nullptr || ((ldres & 3) == 0 && !gn_sums)) && (res2 == nullptr || (ldres2 & 3) == 0) &&
        (!gn_sums || gn_P % 128 == 0))
      return launch_fwd_stripe(a, st);
    int seg, nseg;
    if (fwd_stripe2_ok(a.M, h, wd, cin, a.c0, x1 != nullptr, cout, ks, seg, nseg) &&
        a.M * std::max(ld0, x1 ? ld1 : 0) < (1ll << 31))
      return launch_fwd_stripe2(a, seg, nseg, st);
    if (conv1x1_ok(a, x1 != nullptr) && !res2) {  // (the streamed 1x1 takes one residual)
      if (cout == 64) return cin == 64 ? launch_conv1x1<64, 1>(a, st) : launch_conv1x1<64, 2>(a, st);
      return cin == 64 ? launch_conv1x1<128, 1>(a, st) : launch_conv1x1<128, 2>(a, st);
    }
    const long long maxld = ld0 > (x1 ? ld1 : 0) ? ld0 : ld1;
    if (cin % 64 == 0 && a.c0 % 64 == 0 && a.M * maxld < (1ll << 31) && (ks == 1 || ks == 3)) {  // the kernel's tap mask
      int bm, bn;
      glds_tile(a.M, cout, a.K, bm, bn);
      if (bm == 256) return launch_fwd_glds<256, 64>(a, st);
      if (bn == 64) return launch_fwd_glds<128, 64>(a, st);
      if (bm == 64) return launch_fwd_glds<64, 128>(a, st);
      return launch_fwd_glds<128, 128>(a, st);
    }
  }
  const long long mt128 = (a.M + 127) / 128;
  int bn = cout <= 64 ? 64 : 128;
  int bm = 128;
  if (mt128 * ((cout + bn - 1) / bn) < 512) bm = 64;
  if (bm == 64 && bn == 128 && ((a.M + 63) / 64) * ((cout + 127) / 128) < 512) bn = 64;
  if (bm == 128 && bn == 128) return launch_fwd<T, 128, 128>(a, st);
  if (bm == 128 && bn == 64) return launch_fwd<T, 128, 64>(a, st);
  if (bm == 64 && bn == 128) return launch_fwd<T, 64, 128>(a, st);
  return launch_fwd<T, 64, 64>(a, st);
}

template <typename T, int BMC, int BNK>
int launch_wgrad(WgradArgs<T> a, hipStream_t st) {
  const int mt = (a.cout + BMC - 1) / BMC, nt = (a.K + BNK - 1) / BNK;
  // aim for ~4 blocks per CU over the whole grid, at least 256 pixels/split
  long long want = 1024 / ((long long)mt * nt);
  if (want < 1) want = 1;
  long long per = (a.M + want - 1) / want;
  per = ((per + 255) / 256) * 256;
  if (per < 256) per = 256;
  unsigned splits;
  if (a.batch_pix > 0) {
    const long long nbatch = a.M / a.batch_pix;
    long long spb = (a.batch_pix + per - 1) / per;
    per = (a.batch_pix + spb - 1) / spb;
    a.splits_per_batch = (int)spb;
    splits = (unsigned)(nbatch * spb);
  } else {
    splits = (unsigned)((a.M + per - 1) / per);
  }
  a.pix_per_split = (int)per;
  dim3 grid(mt, nt, splits);
  conv_wgrad_kernel<T, BMC, BNK><<<grid, 256, 0, st>>>(a);
  return check_launch("conv_wgrad");
}

template <typename T>
int conv_wgrad_t(const void* dy, int lddy, const void* x0, int ld0, int c0, const void* x1,
                 int ld1, float* ws, float* db, int nf, int h, int w, int cin, int cout, int ks,
                 hipStream_t st, long long batch_pix = 0) {
  WgradArgs<T> a;
  a.db = db;
  a.dy = (const T*)dy; a.lddy = lddy; a.x0 = (const T*)x0; a.x1 = (const T*)(x1 ? x1 : x0);
  a.ld0 = ld0; a.ld1 = x1 ? ld1 : ld0; a.c0 = x1 ? c0 : cin; a.ws = ws; a.H = h; a.W = w;
  a.cin = cin; a.cout = cout; a.ks = ks; a.K = ks * ks * cin; a.M = (long long)nf * h * w;
  a.pix_per_split = 0;
  a.batch_pix = batch_pix;
  a.ws_bstride = (long long)cout * a.K;
  a.splits_per_batch = 1;
  if (a.M == 0) return DV_OK;
  if constexpr (sizeof(T) == 2) {
    const long long maxld = std::max<long long>(std::max(lddy, ld0), x1 ? ld1 : 0);
    if (a.M * maxld < (1ll << 31) && (long long)cout * a.K < (1ll << 31))
      return conv_wgrad_glds(dy, lddy, x0, ld0, c0, x1, ld1, ws, db, nf, h, w, cin, cout, ks, st,
                             batch_pix);
  }
  const bool small_co = cout <= 64;
  const bool small_k = a.K <= 64;
  if (small_co && small_k) return launch_wgrad<T, 64, 64>(a, st);
  if (small_co) return launch_wgrad<T, 64, 128>(a, st);
  if (small_k) return launch_wgrad<T, 128, 64>(a, st);
  return launch_wgrad<T, 128, 128>(a, st);
}

// ---------------------------------------------------------------------------
// bf16 3x3 wgrad, stripe form (cin, cout % 64 == 0; W in {8, 16, 32, 64}):
// dW[co][tap][ci] = sum_p dY[p][co] X[p + tap][ci] for ALL nine taps of a
// 64(co) x 64(ci) tile in one workgroup, over a contiguous range of 128-pixel
// stages (grid z = pixel split).  A stage stages its 128 dY rows and the
// WINDOW of X pixels they see — NSEG segments of (seg + 2) image rows of
// W + 2 pixels (halo from a zeroed line), 128 B per pixel — so X is staged
// once per stage (not once per tap: the nine taps read the same window at
// row offsets dy*(W+2) + dx), and each CU does all nine taps' MFMAs per byte
// staged.  8 waves: waves 4-7 take the second 64-pixel half of every stage;
// each wave owns a 32(co) x 32(ci) tile of every tap (9 accumulators).  The
// two halves are summed through LDS and written with plain stores to
// part[z][co][tap][ci] (no atomics); wgrad_reduce_kernel sums the splits.
// ---------------------------------------------------------------------------
struct WgradSArgs {
  const bf16* dy;
  int lddy;
  const bf16* x0;
  const bf16* x1;
  int ld0, ld1, c0;
  float* part;    // [S][cout][cin][9] partials (S > 1): f32, or bf16 when part_bf16
  float* dbpart;  // [S][cout] or null (f32)
  float* dw;      // (cout, cin, 1, 3, 3) gradient (S == 1)
  float* db;      // [cout] or null
  int acc_w, acc_b, part_bf16;
  int H, cin, cout, K;
  int nstages, stages_per_split;
};

// the row-window wgrad tile epilogue (both wgrad kernels): the two pixel
// halves summed through LDS, then the 64 x 64 x NT tile written in the torch
// layout -- bf16 split partials, f32 split partials or the gradient itself
template <int NT>
__device__ __forceinline__ void wgrad_tile_store(const WgradSArgs& a, f32x16 (&acc)[NT], float accb, char* smem,
                                                 int half, int wq, int wm, int wn, int lane, int co0, int ci0,
                                                 bool do_bias, int bz) {

  // ---- sum the two pixel halves through LDS in one pass (16-B rows per lane) ----
  float* red = (float*)smem;
  constexpr int PERW = (NT * 16 + 1) * 64;  // floats per wave
  if (half == 1) {
#pragma unroll
    for (int d = 0; d < NT; ++d)
#pragma unroll
      for (int e4 = 0; e4 < 4; ++e4)
        *(f32x4*)(red + wq * PERW + (d * 4 + e4) * 256 + lane * 4) =
            f32x4{acc[d][4 * e4], acc[d][4 * e4 + 1], acc[d][4 * e4 + 2], acc[d][4 * e4 + 3]};
    red[wq * PERW + NT * 16 * 64 + lane] = accb;
  }
  __syncthreads();
  if (half == 0) {
#pragma unroll
    for (int d = 0; d < NT; ++d)
#pragma unroll
      for (int e4 = 0; e4 < 4; ++e4) {
        const f32x4 v = *(const f32x4*)(red + wq * PERW + (d * 4 + e4) * 256 + lane * 4);
#pragma unroll
        for (int k = 0; k < 4; ++k) acc[d][4 * e4 + k] += v[k];
        __builtin_amdgcn_sched_barrier(0);  // bounded reads in flight (else they all hoist: spills)
      }
    accb += red[wq * PERW + NT * 16 * 64 + lane];
  }
  __syncthreads();
  DV_STAMP_AT(3);
  if (gridDim.z > 1 && a.part_bf16) {
    // ---- bf16 split partials: the four half-0 waves round their 32 x 32 x 9
    // tiles to bf16 and transpose them into the torch layout in LDS together
    // (one round), and all 8 waves write the block's 64 x 576 partial as 16-B
    // stores ----
    constexpr int TP = 32 * NT;  // bf16 per output channel of a wave tile
    bf16* tiles = (bf16*)smem;
    const int r = lane & 31, h = lane >> 5;
    if (half == 0) {
      bf16* tb = tiles + wq * 32 * TP;
#pragma unroll
      for (int d = 0; d < NT; ++d)
#pragma unroll
        for (int e = 0; e < 16; ++e) tb[((e & 3) + 8 * (e >> 2) + 4 * h) * TP + r * NT + d] = (bf16)acc[d][e];
    }
    __syncthreads();
    bf16* dstb = (bf16*)a.part + (long long)bz * a.cout * a.K;
    constexpr int CPR = TP / 8;  // 16-B chunks per output-channel row of a tile
    for (int idx = threadIdx.x; idx < 4 * 32 * CPR; idx += 512) {
      const int t4 = idx / (32 * CPR), rem = idx - t4 * (32 * CPR);
      const int col = rem / CPR, j = rem - col * CPR;
      const u32x4 v = *(const u32x4*)(tiles + (t4 * 32 + col) * TP + 8 * j);
      const long long oi = (long long)(co0 + (t4 >> 1) * 32 + col) * a.K + (ci0 + (t4 & 1) * 32) * NT + 8 * j;
      *(u32x4*)(dstb + oi) = v;
    }
#ifdef DV_STAMP
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    DV_STAMP_AT(4);
    if (do_bias && half == 0 && lane < 32) a.dbpart[(long long)bz * a.cout + co0 + wm * 32 + lane] = accb;
    return;
  }

  // ---- torch-layout output [co][ci][tap]: each wave's 32 x 32 x 9 tile is
  // transposed through LDS (two tiles per round, 36 KB each) so every output
  // channel's 32 ci x 9 taps go out as 1152 contiguous bytes (float4 stores).
  // One split writes the gradient itself (accumulate honoured); several
  // splits write partials that wgrad_reduce4_kernel sums. ----
  const bool direct = gridDim.z == 1;
  const bool pbf = !direct && a.part_bf16;  // bf16 partials: half the split-K bytes
  float* dst = direct ? a.dw : a.part + (pbf ? 0 : (long long)bz * a.cout * a.K);
  bf16* dstb = (bf16*)a.part + (long long)bz * a.cout * a.K;
  const int acc_o = direct && a.acc_w;
  const int r = lane & 31, h = lane >> 5;
  constexpr int TP = 32 * NT;  // floats per output channel in a tile
#pragma unroll
  for (int rnd = 0; rnd < 2; ++rnd) {
    float* tile = red + wn * (32 * TP);
    if (half == 0 && wm == rnd) {
#pragma unroll
      for (int d = 0; d < NT; ++d)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int col = (e & 3) + 8 * (e >> 2) + 4 * h;  // local co
          tile[col * TP + r * NT + d] = acc[d][e];
        }
    }
    __syncthreads();
    // all 8 waves store the round's two tiles (the store phase is
    // issue-bound: two storing waves left it at ~40 % of a small wgrad's time)
    for (int idx = threadIdx.x; idx < 2 * 32 * (TP / 4); idx += 512) {
      const int t2 = idx / (32 * (TP / 4)), rem = idx - t2 * (32 * (TP / 4));
      const int col = rem / (TP / 4), j = rem - col * (TP / 4);
      f32x4 v = *(const f32x4*)(red + t2 * (32 * TP) + col * TP + 4 * j);
      const long long rowbase = (long long)(co0 + rnd * 32) * a.K + (ci0 + t2 * 32) * NT;
      const long long oi = rowbase + (long long)col * a.K + 4 * j;
      if (pbf) {
        const float t4[4] = {v[0], v[1], v[2], v[3]};
        store4<bf16>(dstb + oi, t4);
        continue;
      }
      f32x4* o = (f32x4*)(dst + oi);
      if (acc_o) v += *o;
      *o = v;
    }
    __syncthreads();
  }
#ifdef DV_STAMP
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the partial stores written
#endif
  DV_STAMP_AT(4);
  if (do_bias && half == 0 && lane < 32) {
    const int co = co0 + wm * 32 + lane;
    if (direct) a.db[co] = a.acc_b ? a.db[co] + accb : accb;
    else a.dbpart[(long long)bz * a.cout + co] = accb;
  }
}

// ---------------------------------------------------------------------------
// bf16 1x1 wgrad (res_conv / Downsample3D / PixelShuffle / stage-3 1x1 convs,
// cin, cout % 64 == 0): dW[co][ci] = sum_p dY[p][co] X[p][ci].  A workgroup
// owns a 64 co x 64 ci tile over a contiguous range of 128-pixel stages, 8
// waves (waves 4-7 on the second 64-pixel half, one 32 x 32 quadrant per
// wave), the halves summed by wgrad_tile_store.  A stage is 128 dY rows and
// 128 X rows by LDS-DMA into a 2-deep ring of 64-B half-row images (conflict-
// free transposed reads, every k-step an immediate offset); 64 KB of LDS and
// 4 waves per SIMD: two workgroups share a CU (a stage holds 4 MFMAs per wave,
// too little to cover the next stage's DMA inside one workgroup).
// ---------------------------------------------------------------------------
template <int NBUF = 2>
__global__ __launch_bounds__(512, 4) void conv_wgrad_1x1_kernel(WgradSArgs a) {
  constexpr int AIMG = 2 * 128 * 64, BHALF = 128 * 64, STG = AIMG + 2 * BHALF;
  constexpr int DPS = 4;                      // DMAs per thread per stage
  constexpr int RED1 = 4 * (16 + 1) * 64 * 4;  // wgrad_tile_store's halves sum
  constexpr int RING = NBUF * STG;
  __shared__ __attribute__((aligned(1024))) char smem[RING > RED1 ? RING : RED1];

  DV_STAMP_AT(0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int half = wave >> 2, wq = wave & 3, wm = wq >> 1, wn = wq & 1;
  const int co0 = blockIdx.x * 64, ci0 = blockIdx.y * 64;
  const int sbeg = blockIdx.z * a.stages_per_split;
  const int send = min(sbeg + a.stages_per_split, a.nstages);
  const int nst = send - sbeg;

  // this lane's DMA slot: row 16 * wave + (lane >> 2), 16-B chunk (lane & 3)
  // of a 64-B half row
  const int l4 = lane >> 2, c4 = lane & 3, drow = 16 * wave;
  const bool first = ci0 < a.c0;
  const int xld = first ? a.ld0 : a.ld1;
  const __amdgpu_buffer_rsrc_t yrs = dma_rsrc(a.dy, (unsigned)((long long)a.nstages * 128 * a.lddy * 2));
  const __amdgpu_buffer_rsrc_t xrs =
      dma_rsrc(first ? a.x0 : a.x1, (unsigned)((long long)a.nstages * 128 * xld * 2));
  const unsigned yoff = (unsigned)(((drow + l4) * a.lddy + co0 + 8 * c4) * 2);
  const unsigned xoff = (unsigned)(((drow + l4) * xld + (first ? ci0 : ci0 - a.c0) + 8 * c4) * 2);
  auto issue = [&](int st, int buf) {
    const unsigned m0 = (unsigned)(sbeg + st) * 128;
    char* sA = smem + buf * STG;
    char* sB = sA + AIMG;
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      dma16s(yrs, sA + hh * (AIMG / 2) + drow * 64, yoff + 64 * hh, m0 * a.lddy * 2);
      dma16s(xrs, sB + hh * BHALF + drow * 64, xoff + 64 * hh, m0 * xld * 2);
    }
  };

  f32x16 acc[1];
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[0][e] = 0.f;
  float accb = 0.f;
  const bool do_bias = a.db != nullptr && blockIdx.y == 0 && wn == 0;  // wave-uniform
  const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  const int colb = 32 * (g & 1) + 8 * pp;
  const int r0 = (half * 64 + 8 * (g >> 1) + q) * 64 + colb;  // k-step 0's row of this lane

#pragma unroll
  for (int i = 0; i < NBUF - 1; ++i)
    if (i < nst) issue(i, i);
  for (int st = 0; st < nst; ++st) {
    const int buf = st % NBUF;
    if (st + NBUF - 1 < nst) {
      issue(st + NBUF - 1, (st + NBUF - 1) % NBUF);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DPS * (NBUF - 1)) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    if (st == 0) DV_STAMP_AT(1);
    // A and B of k-step s at + 1024 s (+ 256 for the high half): asm reads in
    // the order (A0, B0, A1, B1, ...), counted waits (tr_read_asm)
    const unsigned ab = lds_u32(smem + buf * STG + wm * (AIMG / 2)) + r0;
    const unsigned bb = lds_u32(smem + buf * STG + AIMG + wn * BHALF) + r0;
    u32x2 r[4][4];
    static_for<0, 4>([&](auto S) {
      constexpr int k = decltype(S)::value;
      r[k][0] = tr_read_asm<1024 * k>(ab);
      r[k][1] = tr_read_asm<1024 * k + 256>(ab);
      r[k][2] = tr_read_asm<1024 * k>(bb);
      r[k][3] = tr_read_asm<1024 * k + 256>(bb);
    });
    static_for<0, 4>([&](auto S) {
      constexpr int k = decltype(S)::value;
      asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(r[k][0]), "+v"(r[k][1]), "+v"(r[k][2]), "+v"(r[k][3])
                   : "n"(4 * (3 - k)));
      const u32x4 fa = u32x4{r[k][0][0], r[k][0][1], r[k][1][0], r[k][1][1]};
      const u32x4 fb = u32x4{r[k][2][0], r[k][2][1], r[k][3][0], r[k][3][1]};
      acc[0] = Mma<bf16>::run(fa, fb, acc[0]);
      if (do_bias) {  // a lane's A fragment holds 8 pixels of ONE output channel
        float t[8];
        Vec<bf16>::to_f(fa, t);
        accb += ((t[0] + t[1]) + (t[2] + t[3])) + ((t[4] + t[5]) + (t[6] + t[7]));
      }
    });
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  DV_STAMP_AT(2);
  accb += __shfl_xor(accb, 32, 64);  // both k-halves of the channel
  wgrad_tile_store<1>(a, acc, accb, smem, half, wq, wm, wn, lane, co0, ci0, do_bias, (int)blockIdx.z);
}

// ---------------------------------------------------------------------------
// bf16 3x3 wgrad, window form (round 5; cin, cout % 64 == 0):
//   dW[co][dy][dx][ci] = sum_p dY[p][co] X[p + (dy - 1, dx - 1)][ci]
// Same workgroup shape as the stripe kernel (a 64 co x 64 ci x 9 tap tile over
// a contiguous range of 128-pixel stages, 8 waves, waves 4-7 on the second
// 64-pixel half, the halves summed through LDS by wgrad_tile_store), but the
// four 16-pixel k-steps of a half are VERTICAL TRANSLATES of one another:
// k-step s covers image row r0 + s (W >= 16: 16 columns; W = 8: rows s and
// s + 4 of one 8 x 8 frame).  The window fragment of tap (dy, dx) at k-step s
// is then the fragment of row shift t = s + dy, so each wave reads only
// (4 + 2) x 3 = 18 window fragments per stage for its 36 MFMAs (the stripe
// kernel read 36): half the ds_read_b64_tr_b16 traffic, which had the LDS
// return FIFO full (profiles/r04w_conv_families_pmc.txt).  A stage is a
// 4-row x 32-column block (W >= 32), an 8 x 16 block (W = 16) or two 8 x 8
// frames (W = 8); its window is (rows + 2) x (columns + 2) pixels: 204 / 180
// / 200 (the W = 64 stripe window was 264), so every width runs a 3-deep
// ring.  Operand addresses: one VGPR per wave, every (t, dx) an immediate.
// ---------------------------------------------------------------------------
template <int W> struct WinGeom {
  static constexpr int NFR = W == 8 ? 2 : 1;                      // frames per stage
  static constexpr int SC = W >= 32 ? 32 : W;                     // stage columns
  static constexpr int SR = W == 8 ? 8 : 128 / SC;                // stage rows (per frame)
  static constexpr int WQ = SC + 2;                               // window pixels per row
  static constexpr int FPIX = (SR + 2) * WQ;                      // window pixels per frame
  static constexpr int WR = NFR * FPIX;                           // 200 / 180 / 204
  static constexpr int NRH = (WR + 127) / 128;                    // 128-row DMA rounds per ci half
  static constexpr int AIMG = 2 * 128 * 64;                       // dY image: 2 co halves x 128 rows x 64 B
  static constexpr int BHALF = NRH * 128 * 64;                    // window image of one ci half
  static constexpr int STG = AIMG + 2 * BHALF;
  static constexpr int NBUF = 3;
  static_assert(NBUF * STG <= 160 * 1024, "ring exceeds LDS");
};

bool wgrad_win_geom_ok(int h, int w) {
  if (w == 8) return h == 8;
  if (w == 16) return h % 8 == 0;
  return (w == 32 || w == 64) && h % 4 == 0;
}

// One barrier per stage; every wave issues its own six DMA pieces of stage
// st + 2 among the MFMAs of row shifts 0-2 (same box, r05e: 387 vs 407 us
// over the Cfg2 shapes for waves 4-7 issuing all of them before the barrier).
template <int W>
__global__ __launch_bounds__(512, 1) void conv_wgrad_win_kernel(WgradSArgs a) {
  using G = WinGeom<W>;
  constexpr int WQ = G::WQ, NRH = G::NRH, STG = G::STG, NBUF = G::NBUF, AIMG = G::AIMG, BHALF = G::BHALF;
  constexpr int NT = 9;
  constexpr int DPS = 2 + 2 * NRH;  // DMAs per thread per stage
  constexpr int RED1 = 4 * (NT * 16 + 1) * 64 * 4;
  constexpr int RING = NBUF * STG;
  __shared__ __attribute__((aligned(1024))) char smem[RING > RED1 ? RING : RED1];

  DV_STAMP_AT(0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int half = wave >> 2, wq = wave & 3, wm = wq >> 1, wn = wq & 1;
  // (dealing the tiles to XCDs in contiguous chunks cut the L2 fill traffic
  // 1.2-3x and measured slower: 424-430 vs 409-411 us over the Cfg2 shapes, r05b)
  const int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  const int co0 = bx * 64, ci0 = by * 64;
  const int sbeg = bz * a.stages_per_split;
  const int send = min(sbeg + a.stages_per_split, a.nstages);
  const int nst = send - sbeg;
  const int H = a.H, HW = H * W;
  constexpr int CB = W >= 32 ? W / 32 : 1;  // column blocks per row block
  const int spf = W == 8 ? 1 : (H / G::SR) * CB;  // stages per frame
  // first pixel (frame-linear) and image row / column of stage st
  auto stage_base = [&](int st, int& y0, int& x0) -> int {
    if constexpr (W == 8) {
      y0 = 0;
      x0 = 0;
      return st * 128;
    } else {
      const int f = st / spf, r = st - f * spf;
      const int rb = r / CB, cb = r - rb * CB;
      y0 = rb * G::SR;
      x0 = cb * G::SC;
      return f * HW + y0 * W + x0;
    }
  };
  // stage-local pixel j = 64 half + 16 s + k -> offset from the stage's first pixel
  auto rel = [&](int j) -> int {
    const int h = j >> 6, s = (j >> 4) & 3, k = j & 15;
    if constexpr (W >= 32) return s * W + 16 * h + k;
    else if constexpr (W == 16) return j;
    else return h * 64 + (s + 4 * (k >> 3)) * 8 + (k & 7);
  };

  // ---- static per-lane DMA slots: row 16 * vw + (lane >> 2) of each 128-row
  // round, 16-B chunk (lane & 3) of a 64-B half row; waves 4-7 issue for the
  // virtual waves (w & 3) and w ----
  const int l4 = lane >> 2, c4 = lane & 3;
  // dY through a raw buffer resource as well (a global_load_lds DMA made hipcc
  // drain vmcnt before every LDS read: the ring then ran one stage deep)
  const __amdgpu_buffer_rsrc_t yrs = dma_rsrc(a.dy, (unsigned)((long long)a.nstages * 128 * a.lddy * 2));
  const int a_c = co0 + 8 * c4;
  const bool first = ci0 < a.c0;
  const int xld = first ? a.ld0 : a.ld1;
  const int b_c = (first ? ci0 : ci0 - a.c0) + 8 * c4;
  const __amdgpu_buffer_rsrc_t xrs =
      dma_rsrc(first ? a.x0 : a.x1, (unsigned)((long long)a.nstages * 128 * xld * 2));
  int a_rel[1], b_off[1][NRH], b_ry[1][NRH], b_rx[1][NRH];
#pragma unroll
  for (int k = 0; k < 1; ++k) {
    const int vw = wave;
    a_rel[k] = rel(16 * vw + l4);
#pragma unroll
    for (int i = 0; i < NRH; ++i) {
      const int wpx = 128 * i + 16 * vw + l4;
      const int fr = wpx / G::FPIX, rem = wpx - fr * G::FPIX;
      const int wy = rem / WQ, wx = rem - wy * WQ;
      const bool ok = wpx < G::WR;
      b_ry[k][i] = ok ? wy - 1 : -(1 << 20);
      b_rx[k][i] = wx - 1;
      b_off[k][i] = fr * HW + (wy - 1) * W + (wx - 1);
    }
  }
  // piece p of virtual wave slot k: p = 0 the dY rows (2 DMAs), p = 1 + i
  // window round i (2 DMAs)
  auto issue_piece = [&](int base, int y0, int x0, int buf, int k, int p) {
    const int vw = wave;
    char* sA = smem + buf * STG;
    char* sB = sA + AIMG;
    if (p == 0) {
      const unsigned yoff = (unsigned)(((base + a_rel[k]) * a.lddy + a_c) * 2);
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) dma16(yrs, sA + hh * (AIMG / 2) + 16 * vw * 64, yoff + 64 * hh);
    } else {
      const int i = p - 1;
      // halo / pad rows load out of the raw buffer's range: zeros, no access
      const bool in = (unsigned)(y0 + b_ry[k][i]) < (unsigned)H && (unsigned)(x0 + b_rx[k][i]) < (unsigned)W;
      const unsigned voff = in ? (unsigned)(((base + b_off[k][i]) * xld + b_c) * 2) : DMA_OOB;
      const int drow = 128 * i + 16 * vw;  // wave-uniform
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) dma16(xrs, sB + hh * BHALF + drow * 64, in ? voff + 64 * hh : DMA_OOB);
    }
  };
  constexpr int NP = 1 + NRH;  // pieces per virtual wave
  auto issue = [&](int st, int buf) {
    int y0, x0;
    const int base = stage_base(sbeg + st, y0, x0);
#pragma unroll
    for (int p = 0; p < NP; ++p) issue_piece(base, y0, x0, buf, 0, p);
  };

  f32x16 acc[NT];
#pragma unroll
  for (int d = 0; d < NT; ++d)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[d][e] = 0.f;
  float accb = 0.f;
  const bool do_bias = a.db != nullptr && by == 0 && wn == 0;  // wave-uniform

  const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  const int colb = 32 * (g & 1) + 8 * pp;  // byte column of this lane in a 64-B half row
  const int k0 = 8 * (g >> 1) + q;         // this lane's first k (pixel) of a k-step
  // window pixel of (t, dx) = (0, 0) for this lane's k-step-0 pixel
  const int bpix = W >= 32 ? 16 * half + k0
                 : W == 16 ? 4 * half * WQ + k0
                           : half * G::FPIX + 4 * (g >> 1) * WQ + q;
  const int blane = bpix * 64 + colb;
  const int a0 = (half * 64 + 8 * (g >> 1) + q) * 64 + colb;

#pragma unroll
  for (int i = 0; i < NBUF - 1; ++i)
    if (i < nst) issue(i, i);
  for (int st = 0; st < nst; ++st) {
    const int buf = st % NBUF;
    // stage st + 2 goes into the buffer of stage st - 1, which every wave
    // finished reading before this barrier; stage st + 1 may still land
    const bool pre = st + NBUF - 1 < nst;
    int nbase = 0, ny0 = 0, nx0 = 0;
    if (st + 1 < nst) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DPS) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (pre) nbase = stage_base(sbeg + st + NBUF - 1, ny0, nx0);
    __builtin_amdgcn_s_barrier();
    const int nbuf = (st + NBUF - 1) % NBUF;
    if (st == 0) DV_STAMP_AT(1);
    const char* sA = smem + buf * STG + wm * (AIMG / 2);
    // one operand base per stage, made opaque so that each (t, dx) offset
    // stays the ds_read immediate (otherwise hoisted as loop invariants)
    unsigned bb = lds_u32(smem + buf * STG + AIMG + wn * BHALF) + blane;
    asm volatile("" : "+v"(bb));
    // The operand reads are inline asm with hand-counted lgkmcnt waits: hipcc
    // drains vmcnt(0) before a ds_read_b64_tr_b16 it can see while any LDS-DMA
    // is in flight (it cannot tell the ring buffers apart), which collapsed
    // the three-stage ring to one stage and parked the waves ~half of the time
    // (SQ_WAIT_ANY 0.46-0.50, r05b).  Nothing else in the stage loop touches
    // LDS or the scalar cache, so the counts below are exact: fa (8 reads),
    // then 6 per row shift.
    const unsigned ab = lds_u32(sA) + a0;
    u32x2 fa2[4][2], fb2[3][3][2];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      fa2[s][0] = tr_read_asm<0>(ab + s * 1024);
      fa2[s][1] = tr_read_asm<256>(ab + s * 1024);
    }
    auto rdT = [&](auto T) {
      constexpr int t = decltype(T)::value;
      static_for<0, 3>([&](auto DX) {
        constexpr int dx = decltype(DX)::value, off = (t * WQ + dx) * 64;
        fb2[t % 3][dx][0] = tr_read_asm<off>(bb);
        fb2[t % 3][dx][1] = tr_read_asm<off + 256>(bb);
      });
    };
    rdT(std::integral_constant<int, 0>{});
    rdT(std::integral_constant<int, 1>{});
    u32x4 fa[4];
    static_for<0, 6>([&](auto T) {
      constexpr int t = decltype(T)::value;
      if constexpr (t + 2 < 6) rdT(std::integral_constant<int, t + 2>{});
      // reads issued after row shift t's: those of t + 1 and t + 2
      constexpr int younger = 6 * ((t + 2 < 6 ? 2 : (t + 1 < 6 ? 1 : 0)));
      u32x2(&f)[3][2] = fb2[t % 3];
      asm volatile("s_waitcnt lgkmcnt(%6)"
                   : "+v"(f[0][0]), "+v"(f[0][1]), "+v"(f[1][0]), "+v"(f[1][1]), "+v"(f[2][0]), "+v"(f[2][1])
                   : "n"(younger));
      if constexpr (t == 0) {
        asm volatile("" : "+v"(fa2[0][0]), "+v"(fa2[0][1]), "+v"(fa2[1][0]), "+v"(fa2[1][1]));
        asm volatile("" : "+v"(fa2[2][0]), "+v"(fa2[2][1]), "+v"(fa2[3][0]), "+v"(fa2[3][1]));
#pragma unroll
        for (int s = 0; s < 4; ++s) fa[s] = u32x4{fa2[s][0][0], fa2[s][0][1], fa2[s][1][0], fa2[s][1][1]};
      }
      u32x4 fb[3];
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) fb[dx] = u32x4{f[dx][0][0], f[dx][0][1], f[dx][1][0], f[dx][1][1]};
      constexpr int slo = t > 2 ? t - 2 : 0, shi = t < 3 ? t : 3;
#pragma unroll
      for (int dx = 0; dx < 3; ++dx)
#pragma unroll
        for (int s = slo; s <= shi; ++s) acc[(t - s) * 3 + dx] = Mma<bf16>::run(fa[s], fb[dx], acc[(t - s) * 3 + dx]);
      // the next stage's pieces among the MFMAs: piece t after row shift t
      if constexpr (t < NP) {
        if (pre) issue_piece(nbase, ny0, nx0, nbuf, 0, t);
      }
      if constexpr (t < 4) {
        if (do_bias) {
          float f8[8];
          Vec<bf16>::to_f(fa[t], f8);
          accb += ((f8[0] + f8[1]) + (f8[2] + f8[3])) + ((f8[4] + f8[5]) + (f8[6] + f8[7]));
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    });
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  // the halves sum below reuses the ring: no wave may write it while another
  // still reads the last stage's operands (the loop has no end-of-stage
  // barrier; without this one a wave ahead by part of a stage clobbered them
  // -- an occasional wrong split partial, found as a rare non-finite
  // gradient, tools/nan_stress.py)
  __syncthreads();
  DV_STAMP_AT(2);
  accb += __shfl_xor(accb, 32, 64);  // both k-halves of the channel
  wgrad_tile_store<NT>(a, acc, accb, smem, half, wq, wm, wn, lane, co0, ci0, do_bias, bz);
}

// dw (+)= sum_s part[s] over float4s (partials already in torch layout).
// A workgroup = (256 / G) float4 columns x G split groups (G <= 8, a power
// of two <= S): every lane keeps 8 loads in flight and the groups meet in
// LDS, so even a 256-split sum of a small gradient spreads over hundreds of
// workgroups.  The bias partials ([S][cout], cout % 4 == 0) are reduced the
// same way by the workgroups after the weight ones.
// One lane handles 8 consecutive elements: a 16-B load of bf16 partials (or
// two 16-B loads of f32 ones) per split, so the loads in flight per lane carry
// twice the bytes of a float4 column and a workgroup covers 2,048 / G elements
// (the big gradients have S = 4: one float4 per lane left the blocks mostly
// overhead).
struct F8 {
  f32x4 lo, hi;
};

__device__ __forceinline__ F8 part8(const void* p, bool pbf, long long i) {
  if (!pbf) return F8{((const f32x4*)p)[2 * i], ((const f32x4*)p)[2 * i + 1]};
  const u32x4 t = ((const u32x4*)p)[i];
  F8 r;
  r.lo = f32x4{__builtin_bit_cast(float, t[0] << 16), __builtin_bit_cast(float, t[0] & 0xffff0000u),
               __builtin_bit_cast(float, t[1] << 16), __builtin_bit_cast(float, t[1] & 0xffff0000u)};
  r.hi = f32x4{__builtin_bit_cast(float, t[2] << 16), __builtin_bit_cast(float, t[2] & 0xffff0000u),
               __builtin_bit_cast(float, t[3] << 16), __builtin_bit_cast(float, t[3] & 0xffff0000u)};
  return r;
}

__device__ __forceinline__ void reduce8_block(F8* sh, long long blk, const float* part, int S,
                                              int G, long long n8, float* dw, int acc_w,
                                              const float* dbpart, float* db, int cout, int acc_b,
                                              int part_bf16) {
  const int cols = 256 / G;
  const long long wblocks = (n8 + cols - 1) / cols;
  const bool bias = blk >= wblocks;
  const long long n = bias ? cout / 8 : n8;
  const void* src = bias ? (const void*)dbpart : (const void*)part;
  const bool pbf = part_bf16 && !bias;  // the bias partials stay f32
  float* dst = bias ? db : dw;
  const int acc = bias ? acc_b : acc_w;
  const int c = threadIdx.x % cols, grp = threadIdx.x / cols;
  const long long i = (bias ? blk - wblocks : blk) * (long long)cols + c;
  const long long ic = i < n ? i : n - 1;  // clamped: every load unconditional
  F8 v = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  int s = grp;
  for (; s + 3 * G < S; s += 4 * G) {
    F8 t[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) t[u] = part8(src, pbf, (long long)(s + u * G) * n + ic);
    v.lo += (t[0].lo + t[1].lo) + (t[2].lo + t[3].lo);
    v.hi += (t[0].hi + t[1].hi) + (t[2].hi + t[3].hi);
  }
  for (; s < S; s += G) {
    const F8 t = part8(src, pbf, (long long)s * n + ic);
    v.lo += t.lo;
    v.hi += t.hi;
  }
  if (G > 1) {
    sh[threadIdx.x] = v;
    __syncthreads();
    if (grp != 0) return;
    for (int gg = 1; gg < G; ++gg) {
      v.lo += sh[gg * cols + c].lo;
      v.hi += sh[gg * cols + c].hi;
    }
  }
  if (i >= n) return;
  f32x4* o = (f32x4*)dst + 2 * i;
  if (acc) {
    v.lo += o[0];
    v.hi += o[1];
  }
  o[0] = v.lo;
  o[1] = v.hi;
}

// n4 = gradient elements / 4 (the table's unit); every stripe-wgrad gradient
// and bias has a multiple of 8 elements (cin, cout % 64 == 0)
inline long long reduce4_blocks(long long n4, int G, int cout, bool bias) {
  const int cols = 256 / G;
  return (n4 / 2 + cols - 1) / cols + (bias ? (cout / 8 + cols - 1) / cols : 0);
}

__global__ __launch_bounds__(256) void wgrad_reduce4_kernel(const float* part, int S, int G,
                                                            long long n4, float* dw, int acc_w,
                                                            const float* dbpart, float* db,
                                                            int cout, int acc_b, int part_bf16) {
  __shared__ F8 sh[256];
  reduce8_block(sh, blockIdx.x, part, S, G, n4 / 2, dw, acc_w, dbpart, db, cout, acc_b, part_bf16);
}

// every pending split-K sum of a backward pass in one launch: block b belongs
// to the last entry whose blk0 <= b (binary search over the small table)
__global__ __launch_bounds__(256) void wgrad_reduce_batched_kernel(const DvWgradReduceEntry* table,
                                                                   int n) {
  __shared__ F8 sh[256];
  const long long b = blockIdx.x;
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (table[mid].blk0 <= b) lo = mid;
    else hi = mid - 1;
  }
  const DvWgradReduceEntry e = table[lo];
  reduce8_block(sh, b - e.blk0, e.part, e.S, e.G, e.n4 / 2, e.dw, e.acc_w, e.dbpart, e.db, e.cout,
                e.acc_b, e.part_bf16);
}

// split groups per workgroup: each lane keeps >= 4 splits (4 loads in flight)
inline int reduce4_groups(int S) {
  constexpr int gmax = 8;
  int G = 1;
  while (G * 2 <= gmax && G * 8 <= S) G *= 2;
  return G;
}

// dw[co][ci][tap] (torch layout, real sizes) (+)= sum_s part[s][co][tap][ci]
// and db[co] (+)= sum_s dbpart[s][co].  A workgroup sums 64 consecutive
// packed elements; its 4 waves take every 4th split (coalesced 256-B rows,
// 4 loads in flight per lane) and meet in LDS.  The last ceil(cout/64)
// workgroups reduce the bias partials the same way.
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* part, int S, int cout,
                                                           int cin, int taps, float* dw,
                                                           int cout_real, int cin_real, int acc_w,
                                                           const float* dbpart, float* db,
                                                           int acc_b) {
  __shared__ float sh[4][64];
  const long long total = (long long)cout * cin * taps;
  const long long wblocks = (total + 63) / 64;
  const int ol = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const bool bias = blockIdx.x >= wblocks;
  const long long o = (bias ? blockIdx.x - wblocks : blockIdx.x) * 64 + ol;
  const long long n = bias ? cout : total;
  const float* src = bias ? dbpart : part;
  float v = 0.f;
  if (o < n) {
    int s = grp;
    for (; s + 12 < S; s += 16) {
      const float p0 = src[(long long)s * n + o], p1 = src[(long long)(s + 4) * n + o];
      const float p2 = src[(long long)(s + 8) * n + o], p3 = src[(long long)(s + 12) * n + o];
      v += (p0 + p1) + (p2 + p3);
    }
    for (; s < S; s += 4) v += src[(long long)s * n + o];
  }
  sh[grp][ol] = v;
  __syncthreads();
  if (grp != 0 || o >= n) return;
  v = sh[0][ol] + sh[1][ol] + sh[2][ol] + sh[3][ol];
  if (bias) {
    if (o < cout_real) db[o] = acc_b ? db[o] + v : v;
    return;
  }
  const int ci = (int)(o % cin);
  const long long t = o / cin;
  const int tap = (int)(t % taps), co = (int)(t / taps);
  if (co >= cout_real || ci >= cin_real) return;
  float* out = dw + ((long long)co * cin_real + ci) * taps + tap;
  *out = acc_w ? *out + v : v;
}

void launch_wgrad_reduce(const float* part, int S, int cout, int cin, int taps, float* dw,
                         int cout_real, int cin_real, int acc_w, const float* dbpart, float* db,
                         int acc_b, hipStream_t st) {
  const long long total = (long long)cout * cin * taps;
  const long long blocks = (total + 63) / 64 + (db ? (cout + 63) / 64 : 0);
  wgrad_reduce_kernel<<<(unsigned)blocks, 256, 0, st>>>(part, S, cout, cin, taps, dw, cout_real,
                                                          cin_real, acc_w, dbpart, db, acc_b);
}

// stage geometry for the stripe wgrad (0 = shape not supported)
bool stripe_geom(int h, int w, int& seg, int& nseg) {
  if (!(w == 8 || w == 16 || w == 32 || w == 64)) return false;
  const int hw = h * w;
  if (hw >= 128) {
    seg = 128 / w;
    nseg = 1;
    return h % seg == 0 && (w != 8 || seg + 2 <= 20);
  }
  if (128 % hw) return false;
  seg = h;
  nseg = 128 / hw;
  return nseg * (h + 2) * (w + 2) <= (w == 8 ? 200 : (128 / w + 2) * (w + 2));
}

bool wgrad_stripe_ok(int nf, int h, int w, int cin, int c0, bool split, int cout, int ks,
                     long long maxld = 0) {
  if ((ks != 3 && ks != 1) || cin % 64 || cout % 64 || (split && c0 % 64)) return false;
  const long long M = (long long)nf * h * w;
  if (M % 128 || M >= (1ll << 31)) return false;
  if (M * std::max<long long>(maxld, cout) * 2 >= (long long)DMA_OOB) return false;  // raw-buffer resources
  return ks == 1 || wgrad_win_geom_ok(h, w);
}

// split count: ~256 workgroups (one per CU: the 3x3 stage ring takes 144 KB
// of LDS; the 1x1 kernel's 64 KB ring runs two per CU: ~512).  Capping the splits by stages or by partial bytes was measured
// slower on every Cfg2 shape (tools/ab_fwd.sh): occupancy wins.
inline void stripe_split(int nstages, int grid_xy, long long grad_floats, int ks, int& sps, int& S) {
  (void)grad_floats;
  // 1x1 with the 2-deep ring: two workgroups per CU
  long long want = (ks == 1 ? 512 : 256) / grid_xy;
  if (want > nstages) want = nstages;
  if (want < 1) want = 1;
  sps = (int)((nstages + want - 1) / want);
  S = (nstages + sps - 1) / sps;
}

// split-K partials in bf16 (halves their write and the sum's read; the sum
// and the gradient stay f32)
inline bool stripe_part_bf16() { return true; }

long long wgrad_stripe_ws(int nf, int h, int w, int cin, int cout, int ks) {
  const int nstages = (int)((long long)nf * h * w / 128);
  int sps, S;
  stripe_split(nstages, (cout / 64) * (cin / 64), (long long)cout * ks * ks * cin, ks, sps, S);
  const long long wpart = (long long)S * cout * ks * ks * cin;  // cout % 64 == 0: even
  return (stripe_part_bf16() ? wpart / 2 : wpart) + (long long)S * cout;
}

int conv_wgrad_stripe(const void* dy, int lddy, const void* x0, int ld0, int c0, const void* x1,
                      int ld1, float* ws, float* dw, int acc_w, float* db, int acc_b, int nf, int h,
                      int w, int cin, int cout, int ks, hipStream_t st,
                      DvWgradReduceEntry* defer = nullptr) {
  WgradSArgs a;
  a.dy = (const bf16*)dy; a.lddy = lddy; a.x0 = (const bf16*)x0;
  a.x1 = (const bf16*)(x1 ? x1 : x0); a.ld0 = ld0; a.ld1 = x1 ? ld1 : ld0; a.c0 = x1 ? c0 : cin;
  a.H = h; a.cin = cin; a.cout = cout; a.K = ks * ks * cin;
  a.nstages = (int)((long long)nf * h * w / 128);
  int S;
  stripe_split(a.nstages, (cout / 64) * (cin / 64), (long long)cout * a.K, ks, a.stages_per_split, S);
  a.part = ws;
  a.part_bf16 = S > 1 && stripe_part_bf16();
  a.dbpart = db ? ws + (long long)S * cout * a.K / (a.part_bf16 ? 2 : 1) : nullptr;
  a.dw = dw; a.db = db; a.acc_w = acc_w; a.acc_b = acc_b;
  dim3 grid(cout / 64, cin / 64, S);
  if (ks == 1) {
    conv_wgrad_1x1_kernel<><<<grid, 512, 0, st>>>(a);
  } else {
    switch (w) {
      case 64: conv_wgrad_win_kernel<64><<<grid, 512, 0, st>>>(a); break;
      case 32: conv_wgrad_win_kernel<32><<<grid, 512, 0, st>>>(a); break;
      case 16: conv_wgrad_win_kernel<16><<<grid, 512, 0, st>>>(a); break;
      default: conv_wgrad_win_kernel<8><<<grid, 512, 0, st>>>(a); break;
    }
  }
  if (S > 1) {
    const long long n4 = (long long)cout * a.K / 4;
    const int G = reduce4_groups(S);
    if (defer) {  // the caller sums the partials later (dv_wgrad_reduce_batched)
      *defer = DvWgradReduceEntry{ws, a.dbpart, dw, db, n4, 0, S, G, cout, acc_w, acc_b, a.part_bf16};
    } else {
      wgrad_reduce4_kernel<<<(unsigned)reduce4_blocks(n4, G, cout, db != nullptr), 256, 0, st>>>(
          ws, S, G, n4, dw, acc_w, a.dbpart, db, cout, acc_b, a.part_bf16);
    }
  }
  return check_launch("conv_wgrad_stripe");
}

}  // namespace

extern "C" int dv_conv_fwd(int dtype, const void* x0, int ld0, int c0, const void* x1, int ld1,
                           const void* wpack, const float* bias, const void* res, int ldres,
                           const void* res2, int ldres2, void* y, int ldy, int nf, int h, int w,
                           int cin, int cout, int ksize, int act, float* gn_sums, long long gn_P,
                           int gn_R, void* stream) {
  DV_REQUIRE(x0 && wpack && y, "null pointer");
  DV_REQUIRE(cin > 0 && cin % 8 == 0, "cin must be a positive multiple of 8");
  DV_REQUIRE(!gn_sums || (gn_P > 0 && ((long long)nf * h * w) % gn_P == 0 && gn_R >= 1),
             "GroupNorm statistics: the pixels must be whole clips of gn_P");
  DV_REQUIRE(ld0 % 8 == 0 && (!x1 || (ld1 % 8 == 0 && c0 % 8 == 0 && c0 > 0 && c0 < cin)),
             "input strides / split must be multiples of 8");
  DV_REQUIRE(ksize >= 1 && (ksize & 1), "ksize must be odd");
  DV_REQUIRE(ldy >= cout && (!res || ldres >= cout) && (!res2 || ldres2 >= cout), "bad output stride");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == DV_F32)
    return conv_fwd_t<float>(x0, ld0, c0, x1, ld1, wpack, bias, res, ldres, res2, ldres2, y, ldy, nf,
                             h, w, cin, cout, ksize, act, gn_sums, gn_P, gn_R, st);
  if (dtype == DV_BF16)
    return conv_fwd_t<bf16>(x0, ld0, c0, x1, ld1, wpack, bias, res, ldres, res2, ldres2, y, ldy, nf,
                            h, w, cin, cout, ksize, act, gn_sums, gn_P, gn_R, st);
  DV_REQUIRE(false, "unknown dtype");
}

extern "C" int dv_conv_fwd_gn_in(const DvGnIn* g, const void* z, int ldz, const void* wpack,
                                 const float* bias, void* y, int ldy, int nf, int h, int w, int cin,
                                 int cout, float* gn_sums, long long gn_P, int gn_R, void* stream) {
  DV_REQUIRE(g && z && wpack && y && g->sums && g->gamma && g->beta && g->mean && g->rstd, "null pointer");
  DV_REQUIRE(g->R >= 1 && g->P > 0 && ((long long)nf * h * w) % g->P == 0, "GroupNorm: whole clips of P pixels");
  DV_REQUIRE(!gn_sums || (gn_P > 0 && ((long long)nf * h * w) % gn_P == 0 && gn_R >= 1),
             "GroupNorm statistics: the pixels must be whole clips of gn_P");
  DV_REQUIRE(ldy >= cout && ldz >= cin && (!g->y || g->ldy >= cin) && g->zero_n >= 0, "bad stride");
  const long long M = (long long)nf * h * w;
  // the one shape the folded stripe kernel is built for: 64 -> 64k channels at
  // W = 64, 8 groups of 8 channels, clips of whole 128-pixel stages
  if (!(cin == 64 && g->groups == 8 && w == 64 && fwd_stripe_ok(M, h, w, 64, false, cout, 3, ldz) &&
        (ldy & 3) == 0 && g->P % 128 == 0 && (!gn_sums || gn_P % 128 == 0) &&
        (!g->y || (g->ldy % 8 == 0 && M * g->ldy * 2 < (long long)DMA_OOB))))
    return DV_ERR_UNSUPPORTED;
  ConvFwdArgs<bf16> a;
  a.x0 = a.x1 = (const bf16*)z; a.ld0 = a.ld1 = ldz; a.c0 = cin; a.w = (const bf16*)wpack; a.bias = bias;
  a.res = nullptr; a.ldres = 0; a.y = (bf16*)y; a.ldy = ldy; a.H = h; a.W = w; a.cin = cin; a.cout = cout;
  a.ks = 3; a.act = DV_ACT_NONE; a.M = M; a.K = 9 * cin;
  set_gn(a, gn_sums, gn_P, gn_R);
  a.gi_sums = g->sums; a.gi_rstride = g->rstride; a.gi_P = g->P; a.gi_R = g->R; a.gi_eps = g->eps;
  a.gi_gamma = g->gamma; a.gi_beta = g->beta; a.gi_ss = g->ss; a.gi_mean = g->mean; a.gi_rstd = g->rstd;
  a.gi_y = (bf16*)g->y; a.gi_ldy = g->y ? g->ldy : 0; a.gi_zero = g->zero; a.gi_zero_n = g->zero ? g->zero_n : 0;
  return launch_fwd_stripe(a, (hipStream_t)stream);
}

extern "C" int dv_conv_fwd8(int dtype, const void* x0, int ld0, int c0, const void* x1, int ld1,
                            const void* wpack, const float* bias, const void* res, int ldres,
                            const void* res2, int ldres2, void* y, int ldy, int nf, int h, int w,
                            int cin, int cout, int act, float* gn_sums, long long gn_P, int gn_R,
                            void* stream) {
  DV_REQUIRE(dtype == DV_BF16, "the window conv is bf16 only");
  DV_REQUIRE(!gn_sums || (gn_P > 0 && gn_P % 128 == 0 && ((long long)nf * h * w) % gn_P == 0 &&
                          gn_R >= 1),
             "GroupNorm statistics in the window conv: clips of gn_P % 128 == 0 pixels");
  DV_REQUIRE(x0 && wpack && y, "null pointer");
  DV_REQUIRE(cin > 0 && (!x1 || (c0 > 0 && c0 < cin)), "bad channel split");
  DV_REQUIRE(ldy >= cout && (!res || ldres >= cout) && (!res2 || ldres2 >= cout), "bad output stride");
  if (!res && res2) {  // a lone second residual is the first
    res = res2; ldres = ldres2; res2 = nullptr; ldres2 = 0;
  }
  ConvFwdArgs<bf16> a;
  a.x0 = (const bf16*)x0; a.x1 = (const bf16*)(x1 ? x1 : x0); a.ld0 = ld0; a.ld1 = x1 ? ld1 : ld0;
  a.c0 = x1 ? c0 : cin; a.w = (const bf16*)wpack; a.bias = bias; a.res = (const bf16*)res;
  a.ldres = ldres; a.res2 = (const bf16*)res2; a.ldres2 = ldres2; a.y = (bf16*)y; a.ldy = ldy; a.H = h; a.W = w; a.cin = cin; a.cout = cout;
  a.ks = 3; a.act = act; a.M = (long long)nf * h * w; a.K = 9 * cin;
  set_gn(a, gn_sums, gn_P, gn_R);
  DV_REQUIRE(fwd_frame_ok(a, h, w), "shape/stride outside the window conv (see dv_hip.h)");
  if (a.M == 0) return DV_OK;
  return launch_fwd_frame(a, (hipStream_t)stream);
}

extern "C" int dv_conv_wgrad_ws(int dtype, int nf, int h, int w, int cin, int c0, int split,
                                int cout, int ksize, long long* floats) {
  DV_REQUIRE(floats, "null pointer");
  DV_REQUIRE(cin > 0 && cout > 0 && ksize >= 1, "bad sizes");
  const long long K = (long long)ksize * ksize * cin;
  if (dtype == DV_BF16 && wgrad_stripe_ok(nf, h, w, cin, c0, split != 0, cout, ksize))
    *floats = wgrad_stripe_ws(nf, h, w, cin, cout, ksize);
  else
    *floats = (long long)cout * (K + 1);
  return DV_OK;
}

static int conv_wgrad_impl(int dtype, const void* dy, int lddy, const void* x0, int ld0, int c0,
                           const void* x1, int ld1, float* dw, int accumulate_w, float* db,
                           int accumulate_b, float* ws, long long ws_floats, int nf, int h, int w,
                           int cin, int cout, int cout_real, int cin_real, int ksize,
                           DvWgradReduceEntry* defer, void* stream) {
  if (defer) defer->S = 0;
  DV_REQUIRE(dy && x0 && dw && ws, "null pointer");
  DV_REQUIRE(cin % 8 == 0 && cout % 8 == 0, "cin/cout must be multiples of 8");
  DV_REQUIRE(cout_real <= cout && cin_real <= cin && cout_real > 0 && cin_real > 0,
             "real sizes exceed the padded ones");
  DV_REQUIRE(lddy % 8 == 0 && ld0 % 8 == 0 && (!x1 || (ld1 % 8 == 0 && c0 % 8 == 0)),
             "strides must be multiples of 8");
  DV_REQUIRE(dtype == DV_F32 || dtype == DV_BF16, "unknown dtype");
  long long need = 0;
  dv_conv_wgrad_ws(dtype, nf, h, w, cin, c0, x1 != nullptr, cout, ksize, &need);
  DV_REQUIRE(ws_floats >= need, "workspace too small (see dv_conv_wgrad_ws)");
  hipStream_t st = (hipStream_t)stream;
  if ((long long)nf * h * w == 0) return DV_OK;
  if (dtype == DV_BF16 && cout_real == cout && cin_real == cin &&
      wgrad_stripe_ok(nf, h, w, cin, c0, x1 != nullptr, cout, ksize, std::max(std::max(ld0, x1 ? ld1 : 0), lddy)))
    return conv_wgrad_stripe(dy, lddy, x0, ld0, c0, x1, ld1, ws, dw, accumulate_w, db, accumulate_b,
                             nf, h, w, cin, cout, ksize, st, defer);
  // general path: f32 atomics into the zeroed packed workspace, then one reduce
  const long long K = (long long)ksize * ksize * cin;
  float* dbp = db ? ws + cout * K : nullptr;
  zero_f32(ws, cout * (K + 1), st);
  int rc = dtype == DV_F32
               ? conv_wgrad_t<float>(dy, lddy, x0, ld0, c0, x1, ld1, ws, dbp, nf, h, w, cin, cout, ksize, st)
               : conv_wgrad_t<bf16>(dy, lddy, x0, ld0, c0, x1, ld1, ws, dbp, nf, h, w, cin, cout, ksize, st);
  if (rc != DV_OK) return rc;
  launch_wgrad_reduce(ws, 1, cout, cin, ksize * ksize, dw, cout_real, cin_real, accumulate_w, dbp,
                      db, accumulate_b, st);
  return check_launch("conv_wgrad");
}

extern "C" int dv_conv_wgrad(int dtype, const void* dy, int lddy, const void* x0, int ld0,
                             int c0, const void* x1, int ld1, float* dw, int accumulate_w,
                             float* db, int accumulate_b, float* ws, long long ws_floats, int nf,
                             int h, int w, int cin, int cout, int cout_real, int cin_real,
                             int ksize, void* stream) {
  DV_REQUIRE(dy && x0 && dw && ws, "null pointer");
  return conv_wgrad_impl(dtype, dy, lddy, x0, ld0, c0, x1, ld1, dw, accumulate_w, db, accumulate_b,
                         ws, ws_floats, nf, h, w, cin, cout, cout_real, cin_real, ksize, nullptr,
                         stream);
}

extern "C" int dv_conv_wgrad_deferred(int dtype, const void* dy, int lddy, const void* x0,
                                      int ld0, int c0, const void* x1, int ld1, float* dw,
                                      int accumulate_w, float* db, int accumulate_b, float* ws,
                                      long long ws_floats, int nf, int h, int w, int cin, int cout,
                                      int cout_real, int cin_real, int ksize,
                                      DvWgradReduceEntry* entry, void* stream) {
  DV_REQUIRE(entry && dy && x0 && dw && ws, "null pointer");
  return conv_wgrad_impl(dtype, dy, lddy, x0, ld0, c0, x1, ld1, dw, accumulate_w, db, accumulate_b,
                         ws, ws_floats, nf, h, w, cin, cout, cout_real, cin_real, ksize, entry,
                         stream);
}

extern "C" int dv_wgrad_reduce_plan(DvWgradReduceEntry* t, int n, long long* blocks) {
  DV_REQUIRE(t && blocks && n > 0, "bad table");
  long long blk = 0;
  for (int i = 0; i < n; ++i) {
    DV_REQUIRE(t[i].S >= 1 && t[i].n4 > 0 && t[i].n4 % 2 == 0 && t[i].cout % 8 == 0 && t[i].part && t[i].dw &&
                   (!t[i].db || t[i].dbpart),
               "bad entry");
    t[i].G = reduce4_groups(t[i].S);
    t[i].blk0 = blk;
    blk += reduce4_blocks(t[i].n4, t[i].G, t[i].cout, t[i].db != nullptr);
  }
  *blocks = blk;
  return DV_OK;
}

extern "C" int dv_wgrad_reduce_batched(const DvWgradReduceEntry* table, int n, long long blocks,
                                       void* stream) {
  DV_REQUIRE(table && n >= 0 && blocks >= 0 && blocks < (1ll << 31), "bad table");
  if (n == 0 || blocks == 0) return DV_OK;
  wgrad_reduce_batched_kernel<<<(unsigned)blocks, 256, 0, (hipStream_t)stream>>>(table, n);
  return check_launch("wgrad_reduce_batched");
}

extern "C" int dv_wgrad_reduce_one(const DvWgradReduceEntry* e, void* stream) {
  DV_REQUIRE(e && e->S >= 1 && e->n4 > 0 && e->n4 % 2 == 0 && e->cout % 8 == 0 && e->part && e->dw && (!e->db || e->dbpart),
             "bad entry");
  const int G = reduce4_groups(e->S);
  wgrad_reduce4_kernel<<<(unsigned)reduce4_blocks(e->n4, G, e->cout, e->db != nullptr), 256, 0,
                         (hipStream_t)stream>>>(e->part, e->S, G, e->n4, e->dw, e->acc_w, e->dbpart, e->db,
                                                e->cout, e->acc_b, e->part_bf16);
  return check_launch("wgrad_reduce_one");
}

extern "C" int dv_pack_conv_weights_batched(const DvPackEntry* table, int n, long long max_elems,
                                            void* stream) {
  DV_REQUIRE(table && n >= 0 && n <= 65535, "bad table");
  if (n == 0 || max_elems <= 0) return DV_OK;
  long long bx = (max_elems + 4095) / 4096;
  if (bx > 128) bx = 128;
  pack_weight_batched_kernel<<<dim3((unsigned)bx, (unsigned)n), 256, 0, (hipStream_t)stream>>>(table);
  return check_launch("pack_conv_weights_batched");
}

extern "C" int dv_pack_conv_weight_pairs(const DvPackPair* table, const int* tile_entry, long long total_tiles,
                                         void* stream) {
  DV_REQUIRE(table && tile_entry && total_tiles >= 0 && total_tiles < (1ll << 31), "bad table");
  if (total_tiles == 0) return DV_OK;
  pack_pair_kernel<<<(unsigned)total_tiles, 256, 0, (hipStream_t)stream>>>(table, tile_entry);
  return check_launch("pack_conv_weight_pairs");
}

extern "C" int dv_bias_grad(int dtype, const void* dy, int lddy, float* db, long long npix, int c,
                            void* stream) {
  DV_REQUIRE(dy && db, "null pointer");
  if (npix == 0) return DV_OK;
  long long rows_per = 2048;
  dim3 grid((c + 63) / 64, (unsigned)((npix + rows_per - 1) / rows_per));
  hipStream_t st = (hipStream_t)stream;
  if (dtype == DV_F32)
    bias_grad_kernel<float><<<grid, 256, 0, st>>>((const float*)dy, lddy, db, npix, c, rows_per);
  else
    bias_grad_kernel<bf16><<<grid, 256, 0, st>>>((const bf16*)dy, lddy, db, npix, c, rows_per);
  return check_launch("bias_grad");
}

extern "C" int dv_pack_conv_weight(int dtype, const float* w, void* out, int cout, int cin,
                                   int ksize, int pad_to, int mode, void* stream) {
  DV_REQUIRE(w && out, "null pointer");
  DV_REQUIRE(mode >= 0 && mode <= 3 && (mode < 2 || pad_to % 16 == 0), "bad mode / pad_to");
  const bool fwd = (mode & 1) == 0;
  DV_REQUIRE(fwd ? pad_to >= cin : pad_to >= cout, "pad_to too small");
  DV_REQUIRE(!fwd || (long long)cin * ksize * ksize <= PACK_LDS, "cin * k * k too large");
  DV_REQUIRE(fwd || (long long)cout * ksize * ksize <= PACK_LDS, "cout * k * k too large");
  DvPackEntry e;
  e.w = w; e.out = out; e.dtype = dtype; e.cout = cout; e.cin = cin; e.taps = ksize * ksize;
  e.pad_to = pad_to; e.mode = mode;
  const int rows = fwd ? cout : cin;
  int blocks = rows < 256 ? rows : 256;
  if (blocks < 1) return DV_OK;
  pack_weight_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(e);
  return check_launch("pack_conv_weight");
}

extern "C" int dv_gemm_tn_batched(int dtype, const void* a, int lda, const void* b, int ldb,
                                  float* out, long long batch_rows, int nbatch, int m, int n,
                                  void* stream) {
  // out[g][i][j] += sum_{r in group g} A[r][i] * B[r][j]  (A: rows x m, B: rows x n)
  DV_REQUIRE(a && b && out && m % 8 == 0 && n % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0,
             "m, n and strides must be multiples of 8");
  if (nbatch <= 0 || batch_rows <= 0) return DV_OK;
  hipStream_t st = (hipStream_t)stream;
  const int W = (int)(batch_rows * nbatch);
  if (dtype == DV_F32)
    return conv_wgrad_t<float>(a, lda, b, ldb, n, nullptr, 0, out, nullptr, 1, 1, W, n, m, 1, st, batch_rows);
  if (dtype == DV_BF16)
    return conv_wgrad_t<bf16>(a, lda, b, ldb, n, nullptr, 0, out, nullptr, 1, 1, W, n, m, 1, st, batch_rows);
  DV_REQUIRE(false, "unknown dtype");
}

extern "C" int dv_gemm_tn_batched_multi(int dtype, int ngemm, const void* const* a, const int* lda,
                                        const void* const* b, const int* ldb, float* const* out,
                                        long long batch_rows, int nbatch, int m, int n, void* stream) {
  // ngemm (1..3) dv_gemm_tn_batched problems of one shape, one launch when bf16
  DV_REQUIRE(a && lda && b && ldb && out && ngemm >= 1 && ngemm <= 3, "bad ngemm / null arrays");
  long long maxld = 0;
  for (int i = 0; i < ngemm; ++i) {
    DV_REQUIRE(a[i] && b[i] && out[i] && lda[i] % 8 == 0 && ldb[i] % 8 == 0,
               "null operand or stride not a multiple of 8");
    maxld = std::max<long long>(maxld, std::max(lda[i], ldb[i]));
  }
  DV_REQUIRE(m % 8 == 0 && n % 8 == 0, "m, n and strides must be multiples of 8");
  if (nbatch <= 0 || batch_rows <= 0) return DV_OK;
  const long long rows = batch_rows * nbatch;
  if (dtype == DV_BF16 && rows * maxld < (1ll << 31))
    return gemm_tn_multi_glds(ngemm, a, lda, b, ldb, out, batch_rows, nbatch, m, n, (hipStream_t)stream);
  for (int i = 0; i < ngemm; ++i) {
    const int rc = dv_gemm_tn_batched(dtype, a[i], lda[i], b[i], ldb[i], out[i], batch_rows, nbatch,
                                      m, n, stream);
    if (rc != DV_OK) return rc;
  }
  return DV_OK;
}
