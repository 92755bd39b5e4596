// GroupNorm (Block3D.norm + scale/shift + SiLU, dalle2_video.py:109-131) and
// row LayerNorm (dalle2-pytorch LayerNorm, used by Attention at :430 and
// nn.LayerNorm norm_cond/norm_mid_cond at :374-375).  HBM-bound: each pass
// reads/writes the activation once with 16-byte vectors; statistics are f32.
#include "dv_common.h"

#include <algorithm>
#include <cstdlib>

using namespace dv;

// Diagnostic build only (make stamp): per-workgroup s_memrealtime stamps of the
// single-launch GroupNorm's phases (tools/gn_coop_probe.py reads them with
// dv_debug_stamps_gn).  The product build compiles none of it.
#ifdef DV_STAMP
constexpr int GN_NSTAMP = 8;
__device__ unsigned long long g_gn_stamp[4096 * GN_NSTAMP];
#define GN_STAMP_AT(i)                                                                   \
  do {                                                                                   \
    if (threadIdx.x == 0 && blockIdx.x < 4096)                                           \
      g_gn_stamp[blockIdx.x * GN_NSTAMP + (i)] = __builtin_amdgcn_s_memrealtime();       \
  } while (0)
extern "C" int dv_debug_stamps_gn(unsigned long long* host, long long n) {
  if (n > 4096 * GN_NSTAMP) n = 4096 * GN_NSTAMP;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_gn_stamp), n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#else
#define GN_STAMP_AT(i) \
  do {                 \
  } while (0)
#endif

namespace {

template <typename T>
__device__ __forceinline__ void ld_vec(const T* p, float* o) {
  Vec<T>::to_f(*(const u32x4*)p, o);
}
template <typename T>
__device__ __forceinline__ void st_vec(T* p, const float* v);
template <>
__device__ __forceinline__ void st_vec<float>(float* p, const float* v) {
  *(f32x4*)p = f32x4{v[0], v[1], v[2], v[3]};
}
template <>
__device__ __forceinline__ void st_vec<bf16>(bf16* p, const float* v) {
  *(bf16x8*)p = bf16x8{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3],
                       (bf16)v[4], (bf16)v[5], (bf16)v[6], (bf16)v[7]};
}

// --------------------------------------------------------------------------
// GroupNorm in two launches per direction, no finalize launch:
//   reduce: per-(batch, channel) partial sums into `sums` [nb][C][2] (f32
//           atomics; zero on entry):
//             MODE 0 (stats): f = z, g = z^2
//             MODE 1 (bwd):   f = dv, g = dv*zhat   (dv = dy * act'(v))
//   apply:  every workgroup derives its sample's per-group terms from the
//           2C sums in its prologue (mean/rstd, or m1/m2), then streams.
// The sums are not re-zeroed by the call that used them (its apply
// workgroups are still reading them); instead every apply zeroes `next`, the
// buffer the NEXT GroupNorm call accumulates into (the caller alternates two
// buffers), so no counter, fence or serial tail is needed.
// --------------------------------------------------------------------------
struct GnArgs {
  const void* z; int ldz;
  const void* dy; int lddy;
  void* out; int ldo;
  const void* res; int ldres;
  int nb; long long P; int C, G;
  float* mean; float* rstd;   // fwd: written by the apply; bwd: read
  const float* gamma; const float* beta;
  const float* ss;  // (nb, 2C): scale | shift, or null
  int act;
  float* sums;      // nb * C * 2, zero on entry
  float* next;      // zeroed by the apply (next call's sums), or null
  long long next_n;
  int R;            // replicas of the sums the reduce spreads its atomics over
  long long rstride;
  float eps;
  float *dgamma, *dbeta, *dss;
  int accumulate;
  long long rows_per_block;
  uint8_t* q;       // fwd, bf16: the output also as MX-fp8 (see QNT), or null
  unsigned* qs;
  int exp;  // timing experiments only (DV_GN_EXP): 1 no prologue math, 2 no `next` zeroing, 4 no block-0 section
};

// Per-thread fixed channel vector [cv, cv+VEC) of batch b = blockIdx.y; the
// per-channel affine coefficients are hoisted out of the pixel loop:
//   v = z*A + B,  zhat = z*rs + zb   (A = rs*g*(1+s), B = (beta - mu*rs*g)(1+s) + sh)
struct ChanCoef {
  float A, B, rs, zb, K1;
};
// The per-channel parameters of sample b -- gamma, beta, 1 + FiLM scale,
// FiLM shift -- staged in LDS as prm[0..C), [C..2C), [2C..3C), [3C..4C) by one
// coalesced round of loads (not 4 x VEC dependent per-lane global loads in
// every workgroup's prologue).
constexpr int GN_CMAX = 1024;
__device__ __forceinline__ void stage_params(const GnArgs& a, int b, float* prm) {
  const float* ssb = a.ss ? a.ss + (long long)b * 2 * a.C : nullptr;
  for (int c = threadIdx.x; c < a.C; c += 256) {
    const float g = a.gamma[c], bt = a.beta[c];
    const float sc = ssb ? 1.f + ssb[c] : 1.f, sh = ssb ? ssb[a.C + c] : 0.f;
    prm[c] = g;
    prm[a.C + c] = bt;
    prm[2 * a.C + c] = sc;
    prm[3 * a.C + c] = sh;
  }
}

template <int VEC>
__device__ __forceinline__ void load_coef(const GnArgs& a, int cv, const float* mean,
                                          const float* rstd, const float* prm, ChanCoef* k) {
#pragma unroll
  for (int e = 0; e < VEC; ++e) {
    const int c = cv + e, g = c / (a.C / a.G);
    const float mu = mean[g], rs = rstd[g];
    const float gm = prm[c], bt = prm[a.C + c], sc = prm[2 * a.C + c], sh = prm[3 * a.C + c];
    k[e].A = rs * gm * sc;
    k[e].B = (bt - mu * rs * gm) * sc + sh;
    k[e].rs = rs;
    k[e].zb = -mu * rs;
    k[e].K1 = rs * sc * gm;
  }
}

// Pairs of channels on packed-f32 VALU (v_pk_fma/mul/add_f32); exp / rcp
// stay per lane.  The element loops below are VALU-bound at their occupancy.
typedef float __attribute__((ext_vector_type(2))) f2;
__device__ __forceinline__ f2 sigmoid2(f2 v) {
  const f2 m = v * -1.4426950408889634f;
  const f2 d = 1.f + f2{__builtin_amdgcn_exp2f(m.x), __builtin_amdgcn_exp2f(m.y)};
  return f2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
}
// d silu(v) / dv = s * (1 + v * (1 - s))
__device__ __forceinline__ f2 silu_grad2(f2 v) {
  const f2 sg = sigmoid2(v);
  return sg * (v * (1.f - sg) + 1.f);
}
// per-channel coefficients regrouped as channel pairs
template <int VEC>
struct Coef2 {
  f2 A[VEC / 2], B[VEC / 2], rs[VEC / 2], zb[VEC / 2], K1[VEC / 2];
  __device__ __forceinline__ void set(const ChanCoef* k) {
#pragma unroll
    for (int j = 0; j < VEC / 2; ++j) {
      A[j] = f2{k[2 * j].A, k[2 * j + 1].A};
      B[j] = f2{k[2 * j].B, k[2 * j + 1].B};
      rs[j] = f2{k[2 * j].rs, k[2 * j + 1].rs};
      zb[j] = f2{k[2 * j].zb, k[2 * j + 1].zb};
      K1[j] = f2{k[2 * j].K1, k[2 * j + 1].K1};
    }
  }
};

__device__ __forceinline__ float silu_grad(float v) {
  const float sg = sigmoid_f(v);
  return sg * (1.f + v * (1.f - sg));
}

// U pixel rows per thread are loaded before any is used (U x 16 B, or 2U x 16 B
// in the backward, in flight per lane) so the streaming passes are not
// latency-bound; the reduce keeps ~768 workgroups so its per-(b, c) atomics
// stay lightly contended.
constexpr int GN_U = 4;

template <typename T, int MODE, int U, bool SILU, bool DIR>  // DIR: MODE 1 register prologue
__global__ __launch_bounds__(256) void gn_reduce_kernel(GnArgs a) {
  constexpr int VEC = 16 / sizeof(T);
  constexpr int NL = MODE == 1 ? 2 : 1;  // tensors streamed (z, dy)
  __shared__ float sh[2][256 * VEC];
  __shared__ float smu[64], srs[64];
  __shared__ float prm[MODE == 1 ? 4 * GN_CMAX : 1];
  const int tpr = a.C / VEC;                 // threads per pixel row
  const int rpp = 256 / tpr;                 // rows per pass
  const int tid = threadIdx.x;
  const int rr = tid / tpr, cv = (tid % tpr) * VEC;
  const int b = blockIdx.y;
  const long long beg = blockIdx.x * a.rows_per_block;
  long long end = beg + a.rows_per_block;
  if (end > a.P) end = a.P;
  const long long step = (long long)rpp * U;
  const T* zb = (const T*)a.z + (long long)b * a.P * a.ldz + cv;
  const T* dyb = (const T*)a.dy + (long long)b * a.P * a.lddy + cv;
  const bool act_rows = rr < rpp;
  // batch loads (rows p0 + u*rpp), issued one batch ahead of their use.
  // Unconditional, with the row clamped to the last one: a load under a
  // per-lane branch makes the compiler wait for ALL outstanding loads
  // (vmcnt(0)) at the branch join, which serialised the U rows in flight.
  // Clamped lanes read the same line (coalesced, ~free) and are not summed.
  u32x4 cur[NL][U], nxt[NL][U];
  auto load = [&](long long p0, u32x4 (&buf)[NL][U]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      long long p = p0 + (long long)u * rpp;
      p = p < end ? p : end - 1;
      buf[0][u] = *(const u32x4*)(zb + p * a.ldz);
      if (MODE == 1) buf[NL - 1][u] = *(const u32x4*)(dyb + p * a.lddy);
    }
  };
  long long p0 = beg + rr;
  // MODE 1: the parameter / statistics loads go out BEFORE the data batch
  // (global loads return in order: issued after it they would wait for it)
  ChanCoef kd[VEC];  // DIR: this thread's coefficients, straight from registers
  if constexpr (MODE == 1 && DIR) {
    // the VEC channels [cv, cv+VEC) lie in one group (cg % VEC == 0): the
    // thread loads its own parameters and its group's statistics -- no LDS
    // staging, no barrier
    const bool has_ss = a.ss != nullptr;
    const float* scp = has_ss ? a.ss + (long long)b * 2 * a.C + cv : a.gamma + cv;
    const float* shp = has_ss ? scp + a.C : a.gamma + cv;
    f32x4 gm[VEC / 4], bt[VEC / 4], sc[VEC / 4], sh[VEC / 4];
#pragma unroll
    for (int v = 0; v < VEC / 4; ++v) {
      gm[v] = *(const f32x4*)(a.gamma + cv + 4 * v);
      bt[v] = *(const f32x4*)(a.beta + cv + 4 * v);
      sc[v] = *(const f32x4*)(scp + 4 * v);
      sh[v] = *(const f32x4*)(shp + 4 * v);
    }
    const int g = cv / (a.C / a.G);
    const float mu = a.mean[b * a.G + g], rs = a.rstd[b * a.G + g];
    __builtin_amdgcn_sched_barrier(0);
    load(p0, cur);  // in flight across the prologue
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
      const float gme = gm[e / 4][e % 4], bte = bt[e / 4][e % 4];
      const float sce = has_ss ? 1.f + sc[e / 4][e % 4] : 1.f, she = has_ss ? sh[e / 4][e % 4] : 0.f;
      kd[e].A = rs * gme * sce;
      kd[e].B = (bte - mu * rs * gme) * sce + she;
      kd[e].rs = rs;
      kd[e].zb = -mu * rs;
      kd[e].K1 = 0.f;
    }
    if (!a.accumulate && blockIdx.x == 0 && b == 0) {  // the apply atomically adds
      for (int c = tid; c < a.C; c += 256) {
        if (a.dgamma) a.dgamma[c] = 0.f;
        if (a.dbeta) a.dbeta[c] = 0.f;
      }
    }
  } else {
  const bool pre = MODE == 1 && a.C <= 512;
  float pg[2] = {0.f, 0.f}, pbt[2] = {0.f, 0.f}, psc[2] = {1.f, 1.f}, psh[2] = {0.f, 0.f};
  float mu_r = 0.f, rs_r = 0.f;
  if (pre) {  // unconditional loads from clamped indices (see load() below)
    const bool has_ss = a.ss != nullptr;
    const float* scp = has_ss ? a.ss + (long long)b * 2 * a.C : a.gamma;
    const float* shp = has_ss ? scp + a.C : a.gamma;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      int c = tid + 256 * k;
      c = c < a.C ? c : a.C - 1;
      pg[k] = a.gamma[c];
      pbt[k] = a.beta[c];
      psc[k] = scp[c];  // raw (selected after the data batch is issued)
      psh[k] = shp[c];
    }
    const int g = tid < a.G ? tid : a.G - 1;
    mu_r = a.mean[b * a.G + g];
    rs_r = a.rstd[b * a.G + g];
  }
  load(p0, cur);  // in flight across the prologue
  if (MODE == 1 && !a.accumulate && blockIdx.x == 0 && b == 0) {  // the apply atomically adds
    for (int c = tid; c < a.C; c += 256) {
      if (a.dgamma) a.dgamma[c] = 0.f;
      if (a.dbeta) a.dbeta[c] = 0.f;
    }
  }
  if (MODE == 1) {
    if (pre) {
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int c = tid + 256 * k;
        if (c < a.C) {
          prm[c] = pg[k];
          prm[a.C + c] = pbt[k];
          prm[2 * a.C + c] = a.ss ? 1.f + psc[k] : 1.f;
          prm[3 * a.C + c] = a.ss ? psh[k] : 0.f;
        }
      }
      if (tid < a.G) { smu[tid] = mu_r; srs[tid] = rs_r; }
    } else {
      stage_params(a, b, prm);
      for (int g = tid; g < a.G; g += 256) { smu[g] = a.mean[b * a.G + g]; srs[g] = a.rstd[b * a.G + g]; }
    }
    __syncthreads();
  }
  }
  f2 s1[VEC / 2], s2[VEC / 2];
#pragma unroll
  for (int j = 0; j < VEC / 2; ++j) s1[j] = s2[j] = f2{0.f, 0.f};
  if (act_rows) {
    Coef2<VEC> k2;
    if constexpr (MODE == 1 && DIR) {
      k2.set(kd);
    } else if (MODE == 1) {
      ChanCoef k[VEC];
      load_coef<VEC>(a, cv, smu, srs, prm, k);
      k2.set(k);
    }
    for (; p0 < end; p0 += step) {
      load(p0 + step, nxt);  // past the end: clamped re-reads of the last row
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (p0 + (long long)u * rpp >= end) break;
        float z[VEC];
        Vec<T>::to_f(cur[0][u], z);
        if (MODE == 0) {
#pragma unroll
          for (int j = 0; j < VEC / 2; ++j) {
            const f2 zz{z[2 * j], z[2 * j + 1]};
            s1[j] += zz;
            s2[j] += zz * zz;
          }
        } else {
          float dy[VEC];
          Vec<T>::to_f(cur[NL - 1][u], dy);
#pragma unroll
          for (int j = 0; j < VEC / 2; ++j) {
            const f2 zz{z[2 * j], z[2 * j + 1]}, dd{dy[2 * j], dy[2 * j + 1]};
            f2 dv = dd;
            if (SILU) dv *= silu_grad2(zz * k2.A[j] + k2.B[j]);
            s1[j] += dv;
            s2[j] += dv * (zz * k2.rs[j] + k2.zb[j]);
          }
        }
      }
#pragma unroll
      for (int l = 0; l < NL; ++l)
#pragma unroll
        for (int u = 0; u < U; ++u) cur[l][u] = nxt[l][u];
    }
  }
  // block reduce over the row slots, then one atomic per channel.  Very narrow
  // rows (tpr a power of two <= 4: C <= 32 bf16, where the LDS sum below is a
  // serial 64..256-row loop per channel) first fold the wave's rows with lane
  // shuffles (lanes tpr apart hold the same channels), leaving 4 wave partials
  // per channel.  Wider rows keep the [rpp][C] LDS sum (measured ~5 % faster
  // than shuffles at C = 64 .. 256).
  const int lane = tid & 63, wv = tid >> 6;
  const bool shfl = tpr <= 4 && (tpr & (tpr - 1)) == 0;
  int nrow = rpp;
  if (shfl) {
#pragma unroll
    for (int j = 0; j < VEC / 2; ++j) {
      for (int o = tpr; o < 64; o <<= 1) {
        s1[j].x += __shfl_xor(s1[j].x, o, 64);
        s1[j].y += __shfl_xor(s1[j].y, o, 64);
        s2[j].x += __shfl_xor(s2[j].x, o, 64);
        s2[j].y += __shfl_xor(s2[j].y, o, 64);
      }
    }
    if (lane < tpr) {
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        sh[0][wv * a.C + cv + e] = s1[e / 2][e % 2];
        sh[1][wv * a.C + cv + e] = s2[e / 2][e % 2];
      }
    }
    nrow = 4;
  } else {
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
      sh[0][tid * VEC + e] = (rr < rpp) ? s1[e / 2][e % 2] : 0.f;
      sh[1][tid * VEC + e] = (rr < rpp) ? s2[e / 2][e % 2] : 0.f;
    }
  }
  __syncthreads();
  for (int c = tid; c < a.C; c += 256) {
    float t1 = 0.f, t2 = 0.f;
    for (int r = 0; r < nrow; ++r) {
      t1 += sh[0][r * a.C + c];
      t2 += sh[1][r * a.C + c];
    }
    float* rs = a.sums + (blockIdx.x % a.R) * a.rstride;  // 1/R of the same-address contention
    atomicAdd(rs + ((long long)b * a.C + c) * 2, t1);
    atomicAdd(rs + ((long long)b * a.C + c) * 2 + 1, t2);
  }
}


// apply prologue: this sample's per-channel totals (summed over the R
// replicas; one parallel round of loads) staged in LDS as cs[0..C) / cs[C..2C),
// then one wave per group (channel sums combined in double for the variance).
//   MODE 0: t1 = mean, t2 = rstd      MODE 1: t1 = m1, t2 = m2
template <int MODE>
__device__ void gn_group_math(const GnArgs& a, const float* cs, const float* prm, float* t1, float* t2);

template <int MODE>
__device__ void gn_group_terms(const GnArgs& a, int b, float* cs, float* prm, float* t1, float* t2) {
  const long long sb = (long long)b * a.C * 2;
  for (int c = threadIdx.x; c < a.C; c += 256) {
    float v1 = 0.f, v2 = 0.f;
    for (int r0 = 0; r0 < a.R; r0 += 8) {  // 8 replicas in flight at once (R <= 64)
      float __attribute__((ext_vector_type(2))) v[8];
#pragma unroll
      for (int r = 0; r < 8; ++r)
        if (r0 + r < a.R) v[r] = *(const float __attribute__((ext_vector_type(2)))*)(a.sums + (r0 + r) * a.rstride + sb + 2 * c);
#pragma unroll
      for (int r = 0; r < 8; ++r)
        if (r0 + r < a.R) { v1 += v[r][0]; v2 += v[r][1]; }
    }
    cs[c] = v1;
    cs[a.C + c] = v2;
  }
  stage_params(a, b, prm);
  __syncthreads();
  gn_group_math<MODE>(a, cs, prm, t1, t2);
}

// The same prologue in two halves (C <= 512, R <= 8): gn_terms_issue puts the
// sums / parameter loads in flight BEFORE the caller issues its first data
// batch, gn_terms_finish consumes them.  Global loads return in order, so
// issued after the data batch they would wait for it (~2.5 us per apply
// launch measured with the prologue stubbed out).
struct GnTermRegs {
  f2 s[2][8];
  float gm[2], bt[2], sc[2], sh[2];
};
__device__ __forceinline__ bool gn_terms_split_ok(const GnArgs& a) { return a.C <= 512 && a.R <= 8; }

// Every load is unconditional (channel and replica indices clamped, the FiLM
// pointer swapped for a dummy when absent): a load under a lane branch makes
// the compiler wait for all outstanding loads at the join, which held the
// data batch's issue behind these loads' full latency.
__device__ __forceinline__ void gn_terms_issue(const GnArgs& a, int b, GnTermRegs& r) {
  const long long sb = (long long)b * a.C * 2;
  const bool has_ss = a.ss != nullptr;
  const float* scp = has_ss ? a.ss + (long long)b * 2 * a.C : a.gamma;
  const float* shp = has_ss ? scp + a.C : a.gamma;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    int c = threadIdx.x + 256 * k;
    c = c < a.C ? c : a.C - 1;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int qq = q < a.R ? q : a.R - 1;
      r.s[k][q] = *(const f2*)(a.sums + qq * a.rstride + sb + 2 * c);
    }
    r.gm[k] = a.gamma[c];
    r.bt[k] = a.beta[c];
    r.sc[k] = scp[c];  // raw: any arithmetic here would wait for the load before
    r.sh[k] = shp[c];  // the caller's data batch is issued (gn_terms_finish selects)
  }
}

template <int MODE>
__device__ __forceinline__ void gn_terms_finish(const GnArgs& a, const GnTermRegs& r, float* cs, float* prm,
                                                float* t1, float* t2) {
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int c = threadIdx.x + 256 * k;
    if (c < a.C) {
      float v1 = 0.f, v2 = 0.f;
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (q < a.R) { v1 += r.s[k][q][0]; v2 += r.s[k][q][1]; }
      cs[c] = v1;
      cs[a.C + c] = v2;
      prm[c] = r.gm[k];
      prm[a.C + c] = r.bt[k];
      prm[2 * a.C + c] = a.ss ? 1.f + r.sc[k] : 1.f;
      prm[3 * a.C + c] = a.ss ? r.sh[k] : 0.f;
    }
  }
  __syncthreads();
  gn_group_math<MODE>(a, cs, prm, t1, t2);
}

template <int MODE>
__device__ void gn_group_math(const GnArgs& a, const float* cs, const float* prm, float* t1, float* t2) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, cg = a.C / a.G;
  for (int g = wave; g < a.G; g += 4) {
    if (MODE == 0) {
      double s1 = 0.0, s2 = 0.0;
      for (int c = g * cg + lane; c < (g + 1) * cg; c += 64) {
        s1 += cs[c];
        s2 += cs[a.C + c];
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) { s1 += __shfl_xor(s1, o, 64); s2 += __shfl_xor(s2, o, 64); }
      if (lane == 0) {
        const double n = (double)a.P * cg;
        const double mu = s1 / n;
        double var = s2 / n - mu * mu;
        if (var < 0) var = 0;
        t1[g] = (float)mu;
        t2[g] = (float)(1.0 / sqrt(var + (double)a.eps));
      }
    } else {
      float m1 = 0.f, m2 = 0.f;
      for (int c = g * cg + lane; c < (g + 1) * cg; c += 64) {
        const float k = prm[c] * prm[2 * a.C + c];
        m1 += k * cs[c];
        m2 += k * cs[a.C + c];
      }
      m1 = wave_sum(m1);
      m2 = wave_sum(m2);
      if (lane == 0) {
        const float n = (float)((double)a.P * cg);
        t1[g] = m1 / n;
        t2[g] = m2 / n;
      }
    }
  }
}

// --------------------------------------------------------------------------
// Register-only apply prologue (DIRECT): no LDS, no workgroup barrier.
// A thread owns the VEC channels [cv, cv+VEC) of one group.  The lanes of a
// wave that hold the same channel vector (row slots, tpr lanes apart) split
// the R sums replicas between them; xor shuffles then fold the replicas
// (offsets tpr .. 32) and the group's tpc = cg/VEC channel vectors (offsets
// 1 .. tpc/2).  Valid when tpr = C/VEC is a power of two <= 64, cg % VEC == 0
// and R <= GN_DQ * (64 / tpr).  Every load is issued by gn_direct_issue
// before the caller's first data batch (loads return in order).
// --------------------------------------------------------------------------
constexpr int GN_DQ = 4;  // sums replicas loaded per thread (at most)
template <int VEC, int DQ>
struct GnDirRegs {
  f32x4 s[DQ][VEC / 2];     // (sum1, sum2) of VEC channels, DQ replicas
  f32x4 gm[VEC / 4], bt[VEC / 4], sc[VEC / 4], sh[VEC / 4];
  float mu, rs;             // MODE 1: the forward's group statistics
};

__host__ __device__ inline bool gn_direct_ok(const GnArgs& a, int vec) {
  const int tpr = a.C / vec, cg = a.C / a.G;
  return tpr <= 64 && (tpr & (tpr - 1)) == 0 && cg % vec == 0 && a.R <= GN_DQ * (64 / tpr);
}

// replicas each thread loads: ceil(R / (64 / tpr)), as 1, 2 or 4
__host__ __device__ inline int gn_direct_dq(const GnArgs& a, int vec) {
  const int rw = 64 / (a.C / vec), nq = (a.R + rw - 1) / rw;
  return nq <= 1 ? 1 : nq <= 2 ? 2 : 4;
}

template <int VEC, int MODE, int DQ>
__device__ __forceinline__ void gn_direct_issue(const GnArgs& a, int b, int cv, GnDirRegs<VEC, DQ>& r) {
  const int lane = threadIdx.x & 63, tpr = a.C / VEC, rw = 64 / tpr, qi = lane / tpr;
  const float* sb = a.sums + ((long long)b * a.C + cv) * 2;
#pragma unroll
  for (int i = 0; i < DQ; ++i) {
    int q = qi + rw * i;
    q = q < a.R ? q : a.R - 1;  // clamped (weighted 0 in finish): unconditional loads
#pragma unroll
    for (int v = 0; v < VEC / 2; ++v) r.s[i][v] = *(const f32x4*)(sb + q * a.rstride + 4 * v);
  }
  const bool has_ss = a.ss != nullptr;
  const float* scp = has_ss ? a.ss + (long long)b * 2 * a.C + cv : a.gamma + cv;
  const float* shp = has_ss ? scp + a.C : a.gamma + cv;
#pragma unroll
  for (int v = 0; v < VEC / 4; ++v) {
    r.gm[v] = *(const f32x4*)(a.gamma + cv + 4 * v);
    r.bt[v] = *(const f32x4*)(a.beta + cv + 4 * v);
    r.sc[v] = *(const f32x4*)(scp + 4 * v);
    r.sh[v] = *(const f32x4*)(shp + 4 * v);
  }
  if (MODE == 1) {
    const int g = cv / (a.C / a.G);
    r.mu = a.mean[b * a.G + g];
    r.rs = a.rstd[b * a.G + g];
  }
}

// xor-fold over lanes `lo, 2lo, .. < hi`
template <typename V>
__device__ __forceinline__ V lane_fold(V v, int lo, int hi) {
  for (int o = lo; o < hi; o <<= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Per-channel coefficients of the thread's VEC channels (and, MODE 1, the
// negated m1/m2 terms); block 0 of each clip also writes the saved statistics
// (MODE 0) or this clip's FiLM gradients and its dgamma/dbeta share (MODE 1).
template <int VEC, int MODE, int DQ>
__device__ __forceinline__ void gn_direct_finish(const GnArgs& a, int b, int cv, int rr,
                                                 const GnDirRegs<VEC, DQ>& r, ChanCoef* k, f2* m1, f2* m2) {
  const int lane = threadIdx.x & 63, tpr = a.C / VEC, rw = 64 / tpr, qi = lane / tpr;
  const int cg = a.C / a.G, tpc = cg / VEC, g = cv / cg;
  // this lane's replica slice, per channel
  float s1[VEC], s2[VEC];
#pragma unroll
  for (int e = 0; e < VEC; ++e) s1[e] = s2[e] = 0.f;
#pragma unroll
  for (int i = 0; i < DQ; ++i) {
    const float w = qi + rw * i < a.R ? 1.f : 0.f;
#pragma unroll
    for (int v = 0; v < VEC / 2; ++v) {
      s1[2 * v] += w * r.s[i][v][0];
      s2[2 * v] += w * r.s[i][v][1];
      s1[2 * v + 1] += w * r.s[i][v][2];
      s2[2 * v + 1] += w * r.s[i][v][3];
    }
  }
  float gm[VEC], bt[VEC], sc[VEC], sh[VEC];
#pragma unroll
  for (int e = 0; e < VEC; ++e) {
    gm[e] = r.gm[e / 4][e % 4];
    bt[e] = r.bt[e / 4][e % 4];
    sc[e] = a.ss ? 1.f + r.sc[e / 4][e % 4] : 1.f;
    sh[e] = a.ss ? r.sh[e / 4][e % 4] : 0.f;
  }
  const double n = (double)a.P * cg;
  float mu, rs;
  if (MODE == 0) {
    double d1 = 0.0, d2 = 0.0;
#pragma unroll
    for (int e = 0; e < VEC; ++e) { d1 += s1[e]; d2 += s2[e]; }
    d1 = lane_fold(lane_fold(d1, tpr, 64), 1, tpc);
    d2 = lane_fold(lane_fold(d2, tpr, 64), 1, tpc);
    const double m = d1 / n;
    double var = d2 / n - m * m;
    if (var < 0) var = 0;
    mu = (float)m;
    rs = (float)(1.0 / sqrt(var + (double)a.eps));
    if (blockIdx.x == 0 && !(a.exp & 4) && rr == 0 && (lane % tpr) % tpc == 0) {
      a.mean[b * a.G + g] = mu;
      a.rstd[b * a.G + g] = rs;
    }
  } else {
    mu = r.mu;
    rs = r.rs;
    float t1 = 0.f, t2 = 0.f;
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
      const float kk = gm[e] * sc[e];
      t1 += kk * s1[e];
      t2 += kk * s2[e];
    }
    t1 = lane_fold(lane_fold(t1, tpr, 64), 1, tpc) / (float)n;
    t2 = lane_fold(lane_fold(t2, tpr, 64), 1, tpc) / (float)n;
#pragma unroll
    for (int j = 0; j < VEC / 2; ++j) {
      m1[j] = f2{-rs * t1, -rs * t1};
      m2[j] = f2{-rs * t2, -rs * t2};
    }
    if (blockIdx.x == 0 && !(a.exp & 4)) {  // wave-uniform: every lane joins the folds
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        s1[e] = lane_fold(s1[e], tpr, 64);
        s2[e] = lane_fold(s2[e], tpr, 64);
      }
      if (rr == 0) {  // one lane per channel vector of the clip
#pragma unroll
        for (int e = 0; e < VEC; ++e) {
          const int c = cv + e;
          if (a.dss) {
            a.dss[(long long)b * 2 * a.C + c] = gm[e] * s2[e] + bt[e] * s1[e];  // d scale
            a.dss[(long long)b * 2 * a.C + a.C + c] = s1[e];                    // d shift
          }
          if (a.dgamma) atomicAdd(a.dgamma + c, sc[e] * s2[e]);
          if (a.dbeta) atomicAdd(a.dbeta + c, sc[e] * s1[e]);
        }
      }
    }
  }
#pragma unroll
  for (int e = 0; e < VEC; ++e) {
    k[e].A = rs * gm[e] * sc[e];
    k[e].B = (bt[e] - mu * rs * gm[e]) * sc[e] + sh[e];
    k[e].rs = rs;
    k[e].zb = -mu * rs;
    k[e].K1 = rs * sc[e] * gm[e];
  }
}

// the next GroupNorm call's sums start at zero (spread over the grid)
__device__ __forceinline__ void gn_zero_next(const GnArgs& a) {
  const long long nblk = (long long)gridDim.x * gridDim.y;
  const long long per = ((a.next_n + nblk - 1) / nblk + 3) / 4 * 4;
  const long long i0 = ((long long)blockIdx.y * gridDim.x + blockIdx.x) * per;
  for (long long i = i0 + threadIdx.x * 4; i < i0 + per && i < a.next_n; i += 1024) {
    if (i + 4 <= a.next_n) *(f32x4*)(a.next + i) = f32x4{0.f, 0.f, 0.f, 0.f};
    else for (long long j = i; j < a.next_n; ++j) a.next[j] = 0.f;
  }
}

// MODE 0: forward apply  out = act(v) (+ res)
// MODE 1: backward apply out = dz = rs*(dv*(1+s)*g - m1 - zhat*m2)
// QNT (MODE 0, bf16, C % 64 == 0): the stored output is also written as the
// MX-fp8 operand of the 3x3 conv that reads it (dv_mx8_quant's layout and
// rounding, bit for bit: q [M][C] e4m3, qs [C/64][M] scale pairs): the 4
// lanes holding one 32-channel block fold their amax with two lane xors
template <typename T, int MODE, int U, bool SILU, bool RES, int DQ, bool QNT = false>  // DQ 0: LDS prologue
__global__ __launch_bounds__(256) void gn_apply_kernel(GnArgs a) {
  constexpr int VEC = 16 / sizeof(T);
  __shared__ float t1[64], t2[64], smu[64], srs[64];
  __shared__ float cs[2 * GN_CMAX];  // this sample's per-channel totals
  __shared__ float prm[4 * GN_CMAX];
  const int tid = threadIdx.x;
  const int tpr = a.C / VEC, rpp = 256 / tpr;
  const int rr = tid / tpr, cv = (tid % tpr) * VEC;
  const int b = blockIdx.y, cg = a.C / a.G;
  const long long beg = blockIdx.x * a.rows_per_block;
  long long end = beg + a.rows_per_block;
  if (end > a.P) end = a.P;
  const long long pb = (long long)b * a.P;
  const long long step = (long long)rpp * U;
  const bool act_rows = rr < rpp;
  constexpr bool has_x = MODE == 1 || RES;  // second stream: dy (bwd) or res (fwd)
  const T* xsrc = MODE == 1 ? (const T*)a.dy : (const T*)a.res;
  const int ldx = MODE == 1 ? a.lddy : a.ldres;
  u32x4 zc[U], xc[U], zn[U], xn[U];
  // unconditional loads, row clamped to the last one (see gn_reduce_kernel):
  // no lane branch around a load, so the U rows really are in flight at once
  auto load = [&](long long p0, u32x4 (&zb)[U], u32x4 (&xb)[U]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      long long p = p0 + (long long)u * rpp;
      p = p < end ? p : end - 1;
      zb[u] = *(const u32x4*)((const T*)a.z + (pb + p) * a.ldz + cv);
      if (has_x) xb[u] = *(const u32x4*)(xsrc + (pb + p) * ldx + cv);
    }
  };
  long long p0 = beg + rr;
  Coef2<VEC> k2;
  f2 m1[VEC / 2], m2[VEC / 2];
  if constexpr (DQ > 0) {
    GnDirRegs<VEC, DQ> dr;
    gn_direct_issue<VEC, MODE, DQ>(a, b, cv, dr);
    __builtin_amdgcn_sched_barrier(0);  // prologue loads ahead of the data batch
    load(p0, zc, xc);
    ChanCoef k[VEC];
    if (!(a.exp & 1)) gn_direct_finish<VEC, MODE, DQ>(a, b, cv, rr, dr, k, m1, m2);
    k2.set(k);
    if (a.next && !(a.exp & 2)) gn_zero_next(a);
    if (!act_rows) return;
  } else {
  const bool split = gn_terms_split_ok(a);
  GnTermRegs tr;
  float mu_r = 0.f, rs_r = 0.f;
  // older than the data batch: returns first.  Issued unconditionally (indices
  // clamped; unused when !split): under a branch, its join waited for them.
  gn_terms_issue(a, b, tr);
  if (MODE == 1) {
    const int g = tid < a.G ? tid : a.G - 1;
    mu_r = a.mean[b * a.G + g];
    rs_r = a.rstd[b * a.G + g];
  }
  // keep the prologue loads ahead of the data batch in the machine schedule
  // (they return in order), and consume them on every path so the IR cannot
  // sink them into the `split` branch below the batch either
  __builtin_amdgcn_sched_barrier(0);
  load(p0, zc, xc);  // the first batch is in flight across the prologue
  if (!(a.exp & 1)) gn_terms_finish<MODE>(a, tr, cs, prm, t1, t2);
  if (!split) {  // C > 512 or R > 8: redo from all replicas (not on the Cfg2 path)
    __syncthreads();
    gn_group_terms<MODE>(a, b, cs, prm, t1, t2);
  }
  if (MODE == 1 && tid < a.G) { smu[tid] = mu_r; srs[tid] = rs_r; }
  __syncthreads();
  if (blockIdx.x == 0 && !(a.exp & 4)) {
    if (MODE == 0) {  // saved for the backward
      for (int g = tid; g < a.G; g += 256) { a.mean[b * a.G + g] = t1[g]; a.rstd[b * a.G + g] = t2[g]; }
    } else {  // this sample's FiLM gradients; its share of dgamma / dbeta (zeroed by the reduce)
      for (int c = tid; c < a.C; c += 256) {
        const float r1 = cs[c], r2 = cs[a.C + c];
        const float sc = a.ss ? 1.f + a.ss[(long long)b * 2 * a.C + c] : 1.f;
        const float gm = a.gamma[c], bt = a.beta[c];
        if (a.dss) {
          a.dss[(long long)b * 2 * a.C + c] = gm * r2 + bt * r1;  // d scale
          a.dss[(long long)b * 2 * a.C + a.C + c] = r1;           // d shift
        }
        if (a.dgamma) atomicAdd(a.dgamma + c, sc * r2);
        if (a.dbeta) atomicAdd(a.dbeta + c, sc * r1);
      }
    }
  }
  if (a.next && !(a.exp & 2)) gn_zero_next(a);
  if (!act_rows) return;
  {
    ChanCoef k[VEC];
    float n1[VEC], n2[VEC];
    if (MODE == 0) {
      load_coef<VEC>(a, cv, t1, t2, prm, k);
    } else {
      load_coef<VEC>(a, cv, smu, srs, prm, k);
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        const int g = (cv + e) / cg;
        n1[e] = -k[e].rs * t1[g];
        n2[e] = -k[e].rs * t2[g];
      }
#pragma unroll
      for (int j = 0; j < VEC / 2; ++j) {
        m1[j] = f2{n1[2 * j], n1[2 * j + 1]};
        m2[j] = f2{n2[2 * j], n2[2 * j + 1]};
      }
    }
    k2.set(k);
  }
  }  // DQ == 0
  for (; p0 < end; p0 += step) {
    load(p0 + step, zn, xn);  // past the end: clamped re-reads of the last row
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long p = p0 + (long long)u * rpp;
      if (p >= end) break;
      float z[VEC], o[VEC];
      Vec<T>::to_f(zc[u], z);
      if (MODE == 0) {
        float r[VEC];
        if (has_x) Vec<T>::to_f(xc[u], r);
#pragma unroll
        for (int j = 0; j < VEC / 2; ++j) {
          const f2 zz{z[2 * j], z[2 * j + 1]};
          f2 v = zz * k2.A[j] + k2.B[j];
          if (SILU) v *= sigmoid2(v);
          if (has_x) v += f2{r[2 * j], r[2 * j + 1]};
          o[2 * j] = v.x;
          o[2 * j + 1] = v.y;
        }
        if constexpr (QNT) {
          float ob[VEC], am = 0.f;
#pragma unroll
          for (int e = 0; e < VEC; ++e) {
            ob[e] = (float)(T)o[e];  // the value stored below
            am = fmaxf(am, fabsf(ob[e]));
          }
          am = fmaxf(am, __shfl_xor(am, 1, 64));
          am = fmaxf(am, __shfl_xor(am, 2, 64));
          const int E = mx_exp(am);
          const float inv = mx_inv(E);
          u32x2 w;
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            unsigned t = __builtin_amdgcn_cvt_pk_fp8_f32(ob[4 * i] * inv, ob[4 * i + 1] * inv, 0, false);
            w[i] = __builtin_amdgcn_cvt_pk_fp8_f32(ob[4 * i + 2] * inv, ob[4 * i + 3] * inv, t, true);
          }
          const long long m = pb + p;
          *(u32x2*)(a.q + m * a.C + cv) = w;
          const int E1 = __shfl_xor(E, 4, 64);  // the chunk's second 32-channel block
          if ((cv & 63) == 0)
            a.qs[(long long)(cv >> 6) * ((long long)a.nb * a.P) + m] =
                (unsigned)(E + 127) | ((unsigned)(E1 + 127) << 8);
        }
      } else {
        float dy[VEC];
        Vec<T>::to_f(xc[u], dy);
#pragma unroll
        for (int j = 0; j < VEC / 2; ++j) {
          const f2 zz{z[2 * j], z[2 * j + 1]}, dd{dy[2 * j], dy[2 * j + 1]};
          f2 dv = dd;
          if (SILU) dv *= silu_grad2(zz * k2.A[j] + k2.B[j]);
          const f2 zhat = zz * k2.rs[j] + k2.zb[j];
          const f2 v = dv * k2.K1[j] + m1[j] + zhat * m2[j];
          o[2 * j] = v.x;
          o[2 * j + 1] = v.y;
        }
      }
      st_vec<T>((T*)a.out + (pb + p) * a.ldo + cv, o);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) { zc[u] = zn[u]; xc[u] = xn[u]; }
  }
}

int grid_for(long long work, int per_block = 256) {
  long long b = (work + per_block - 1) / per_block;
  if (b > 16384) b = 16384;
  if (b < 1) b = 1;
  return (int)b;
}

// rows per workgroup: a multiple of one unrolled pass (rpp * U), sized for
// about `target` workgroups over the whole call
// (A floor on the bytes each workgroup streams measured slower on the whole
// step, 74.3-78.9 vs 79.2 steps/s: the small 8x8 / 16x16 calls want the
// parallelism more than fewer prologues.)
long long gn_rows(const GnArgs& a, int vec, int u, long long target) {
  const long long pass = (long long)(256 / (a.C / vec)) * u;
  long long r = (a.P * a.nb + target - 1) / target;
  r = (r + pass - 1) / pass * pass;
  return r < pass ? pass : r;
}

// replicas of the sums: enough that ~16 reduce workgroups share one address
// (a clip's reduce blocks all add into its C sums), no more -- every apply
// workgroup reads all R replicas in its prologue
int gn_replicas(const GnArgs& a, int blocks_per_clip) {
  int r = (blocks_per_clip + 15) / 16;
  r = std::min(r, 8);
  if (a.R < r) r = a.R;  // the caller's buffer holds a.R replicas
  return std::max(r, 1);
}

// Launch shape (measured, tools/gn_*_sweep.sh): unroll depth U (pixel rows
// in flight per lane) and the workgroup-count target of each pass.
struct GnTune {
  int ur0, ua0, ur1, ua1;   // U: fwd reduce / fwd apply / bwd reduce / bwd apply
  long long tr0, ta0, tr1, ta1;
};
const GnTune& gn_tune() {
  // ta0: 1024 before the register prologue
  static const GnTune t{2 * GN_U, GN_U, GN_U, 2, 768, 512, 768, 768};
  return t;
}

template <typename T, int MODE>
void gn_reduce_launch(GnArgs& a, int u, long long target, hipStream_t st) {
  const int VEC = 16 / sizeof(T);
  a.rows_per_block = gn_rows(a, VEC, u, target);
  dim3 g((unsigned)((a.P + a.rows_per_block - 1) / a.rows_per_block), a.nb);
  a.R = gn_replicas(a, (int)g.x);
  const bool silu = a.act == DV_ACT_SILU;
  // the backward reduce's register prologue
  const bool dir = MODE == 1 && (a.C / a.G) % VEC == 0;
#define DV_GN_RED2(UU, D) (silu ? gn_reduce_kernel<T, MODE, UU, true, D><<<g, 256, 0, st>>>(a) \
                                : gn_reduce_kernel<T, MODE, UU, false, D><<<g, 256, 0, st>>>(a))
#define DV_GN_RED(UU) (dir ? DV_GN_RED2(UU, true) : DV_GN_RED2(UU, false))
  switch (u) {
    case 2: DV_GN_RED(2); break;
    case 4: DV_GN_RED(4); break;
    default: DV_GN_RED(8); break;
  }
#undef DV_GN_RED
#undef DV_GN_RED2
}

template <typename T, int MODE, int U, bool SILU, bool RES, int DQ>
void gn_apply_go(const GnArgs& a, dim3 g, hipStream_t st) {
  if constexpr (MODE == 0 && sizeof(T) == 2) {
    if (a.q) {
      gn_apply_kernel<T, MODE, U, SILU, RES, DQ, true><<<g, 256, 0, st>>>(a);
      return;
    }
  }
  gn_apply_kernel<T, MODE, U, SILU, RES, DQ><<<g, 256, 0, st>>>(a);
}

template <typename T, int MODE>
void gn_apply_launch(GnArgs& a, int u, long long target, hipStream_t st) {
  const int VEC = 16 / sizeof(T);
  a.exp = 0;
  a.rows_per_block = gn_rows(a, VEC, u, target);
  dim3 g((unsigned)((a.P + a.rows_per_block - 1) / a.rows_per_block), a.nb);
  const bool silu = a.act == DV_ACT_SILU;
  const bool res = MODE == 0 && a.res != nullptr;
  // the forward apply's register prologue (the backward apply's measured equal: LDS)
  const int dq = sizeof(T) == 2 && MODE == 0 && gn_direct_ok(a, VEC) ? gn_direct_dq(a, VEC) : 0;
#define DV_GN_APP2(UU, D)                                                 \
  (silu ? (res ? gn_apply_go<T, MODE, UU, true, true, D>(a, g, st)         \
               : gn_apply_go<T, MODE, UU, true, false, D>(a, g, st))       \
        : (res ? gn_apply_go<T, MODE, UU, false, true, D>(a, g, st)        \
               : gn_apply_go<T, MODE, UU, false, false, D>(a, g, st)))
#define DV_GN_APP(UU) \
  (dq == 1 ? DV_GN_APP2(UU, 1) : dq == 2 ? DV_GN_APP2(UU, 2) : dq == 4 ? DV_GN_APP2(UU, 4) : DV_GN_APP2(UU, 0))
  switch (u) {
    case 2: DV_GN_APP(2); break;
    case 8: DV_GN_APP(8); break;
    default: DV_GN_APP(4); break;
  }
#undef DV_GN_APP
#undef DV_GN_APP2
}

// --------------------------------------------------------------------------
// Single-launch GroupNorm (bf16, round 6): reduce and apply in ONE kernel with
// the workgroup's rows held in registers between the two phases.
//   grid = nb * k workgroups of GN_CT threads, nb * k <= 256 (one per CU: every
//   workgroup of the grid is resident at once); workgroup (b, j) owns rows
//   [j * rpw, (j + 1) * rpw) of clip b, all C channels.
//   phase 1  load the rows (z; and dy in the backward) into registers, sum the
//            per-channel statistics (MODE 0: z, z^2; MODE 1: dv, dv * zhat),
//            add them into replica j % R of `sums` (agent-scope atomics), then
//            count the workgroup in its clip's arrival counter (release).
//   wait     one lane polls the counter (acquire) until the clip's k workgroups
//            have arrived.  Bounded: after GN_SPIN polls the workgroup sums the
//            whole clip from memory itself (correct, only slower), so a
//            workgroup that is not resident can never hang the grid.
//   phase 2  group terms from the clip totals, applied to the rows still in
//            registers.  Workgroup j == 0 also writes the clip's mean / rstd
//            (fwd) or FiLM gradients and its dgamma / dbeta share (bwd).
// HBM traffic per element: fwd read z (+ res) and write y, bwd read z, dy and
// write dz -- each once (the two-launch form re-reads z, and dy, in its apply),
// and one launch instead of two.
// --------------------------------------------------------------------------
constexpr int GN_CT = 512;      // threads per workgroup
#ifndef GN_COOP_RMAX
#define GN_COOP_RMAX 4
#endif
constexpr int GN_SPIN = 20000;  // counter polls (s_sleep 2 each, ~1 ms) before the fallback

struct GnCoop {
  GnArgs a;
  int k;               // workgroups per clip
  long long rpw;       // rows per workgroup (NV passes of rpp rows)
  int* cnt;            // [nb] arrival counters, zero on entry (the tail of `sums`)
  int force_fallback;  // test hook: skip the wait and recompute the clip's sums
};

template <int MODE, bool SILU>
__device__ __forceinline__ void coop_accum(const float* z, const float* dy, const Coef2<8>& k2, f2* s1, f2* s2) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const f2 zz{z[2 * j], z[2 * j + 1]};
    if (MODE == 0) {
      s1[j] += zz;
      s2[j] += zz * zz;
    } else {
      f2 dv = f2{dy[2 * j], dy[2 * j + 1]};
      if (SILU) dv *= silu_grad2(zz * k2.A[j] + k2.B[j]);
      s1[j] += dv;
      s2[j] += dv * (zz * k2.rs[j] + k2.zb[j]);
    }
  }
}

// per-channel totals of this workgroup's threads: fold the lanes holding the
// same channel vector, then the waves' partials in LDS; thread c < C gets
// channel c's (sum1, sum2)
__device__ __forceinline__ void coop_block_sum(f2* s1, f2* s2, int C, int tpr, float* red, float& t1, float& t2) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, cv = (tid % tpr) * 8;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    for (int o = tpr; o < 64; o <<= 1) {
      s1[j].x += __shfl_xor(s1[j].x, o, 64);
      s1[j].y += __shfl_xor(s1[j].y, o, 64);
      s2[j].x += __shfl_xor(s2[j].x, o, 64);
      s2[j].y += __shfl_xor(s2[j].y, o, 64);
    }
  }
  __syncthreads();  // red may still be read by a previous use
  if (lane < tpr) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[(wv * C + cv + e) * 2] = s1[e / 2][e % 2];
      red[(wv * C + cv + e) * 2 + 1] = s2[e / 2][e % 2];
    }
  }
  __syncthreads();
  t1 = t2 = 0.f;
  if (tid < C) {
#pragma unroll
    for (int w = 0; w < GN_CT / 64; ++w) {  // every wave wrote a partial of every channel
      t1 += red[(w * C + tid) * 2];
      t2 += red[(w * C + tid) * 2 + 1];
    }
  }
}

// KEEPX: the second stream (dy, or res) stays in registers too; otherwise
// phase 2 reads it again (an L2 / MALL hit: the largest slabs, whose two
// streams do not fit the register budget at 16 passes)
template <int MODE, int NV, bool SILU, bool RES, bool KEEPX>
__global__ __launch_bounds__(GN_CT) void gn_coop_kernel(GnCoop q) {
  const GnArgs& a = q.a;
  GN_STAMP_AT(0);
  __shared__ float red[(GN_CT / 64) * 512 * 2];  // wave partials [wave][C][2]
  __shared__ float cs[2 * 512];                   // the clip's per-channel totals
  __shared__ float gt1[64], gt2[64];              // group terms
  __shared__ int ok_sh;
  const int tid = threadIdx.x;
  const int C = a.C, tpr = C / 8, rpp = GN_CT / tpr;
  const int r0 = tid / tpr, cv = (tid % tpr) * 8;
  const int b = blockIdx.x % a.nb, j = blockIdx.x / a.nb;
  const long long beg = (long long)j * q.rpw;
  const long long end = beg + q.rpw < a.P ? beg + q.rpw : a.P;
  constexpr bool has_x = MODE == 1 || RES;
  const int ldx = MODE == 1 ? a.lddy : a.ldres;
  // rows through raw buffer resources: one 32-bit lane offset per tensor, the
  // pass stride in the instruction's scalar offset, rows past the workgroup's
  // end out of range (loads return zeros, stores are dropped)
  const long long row0 = (long long)b * a.P + beg + r0;
  const unsigned nvalid = beg + r0 < end ? (unsigned)((end - beg - r0 + rpp - 1) / rpp) : 0u;
  const __amdgpu_buffer_rsrc_t zrs = dma_rsrc(a.z, (unsigned)((long long)a.nb * a.P * a.ldz * 2));
  const __amdgpu_buffer_rsrc_t xrs = dma_rsrc(MODE == 1 ? a.dy : (RES ? a.res : a.z),
                                              (unsigned)((long long)a.nb * a.P * (has_x ? ldx : a.ldz) * 2));
  const __amdgpu_buffer_rsrc_t ors = dma_rsrc(a.out, (unsigned)((long long)a.nb * a.P * a.ldo * 2));
  const unsigned zoff = (unsigned)((row0 * a.ldz + cv) * 2), zstr = (unsigned)(rpp * a.ldz * 2);
  const unsigned xoff = has_x ? (unsigned)((row0 * ldx + cv) * 2) : 0u, xstr = has_x ? (unsigned)(rpp * ldx * 2) : 0u;
  const unsigned ooff = (unsigned)((row0 * a.ldo + cv) * 2), ostr = (unsigned)(rpp * a.ldo * 2);
  auto vo = [&](unsigned off, int i) { return (unsigned)i < nvalid ? off : DMA_OOB; };

  // parameters of the thread's 8 channels (and, bwd, its group's forward
  // statistics): issued before the data rows (loads return in order)
  const bool has_ss = a.ss != nullptr;
  const float* scp = has_ss ? a.ss + (long long)b * 2 * C + cv : a.gamma + cv;
  const float* shp = has_ss ? scp + C : a.gamma + cv;
  const int grp = cv / (C / a.G);
  Coef2<8> k2;
  auto coef = [&](float mu, float rs) {
    f32x4 gm[2], bt[2], sc[2], sh[2];
#pragma unroll
    for (int v = 0; v < 2; ++v) {
      gm[v] = *(const f32x4*)(a.gamma + cv + 4 * v);
      bt[v] = *(const f32x4*)(a.beta + cv + 4 * v);
      sc[v] = *(const f32x4*)(scp + 4 * v);
      sh[v] = *(const f32x4*)(shp + 4 * v);
    }
    ChanCoef k[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float g = gm[e / 4][e % 4], bb = bt[e / 4][e % 4];
      const float c = has_ss ? 1.f + sc[e / 4][e % 4] : 1.f, h = has_ss ? sh[e / 4][e % 4] : 0.f;
      k[e].A = rs * g * c;
      k[e].B = (bb - mu * rs * g) * c + h;
      k[e].rs = rs;
      k[e].zb = -mu * rs;
      k[e].K1 = rs * c * g;
    }
    k2.set(k);
  };
  float mu_f = 0.f, rs_f = 0.f;
  if (MODE == 1) {
    mu_f = a.mean[b * a.G + grp];
    rs_f = a.rstd[b * a.G + grp];
    coef(mu_f, rs_f);
  }
  __builtin_amdgcn_sched_barrier(0);
  u32x4 zr[NV], xr[KEEPX ? NV : 1];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    zr[i] = __builtin_amdgcn_raw_buffer_load_b128(zrs, vo(zoff, i), i * zstr, 0);
    if (MODE == 1 && KEEPX) xr[i] = __builtin_amdgcn_raw_buffer_load_b128(xrs, vo(xoff, i), i * xstr, 0);
  }
  // the next GroupNorm call's sums and counters start at zero
  if (a.next) gn_zero_next(a);

  // ---- phase 1: this workgroup's statistics (rows out of range read zeros:
  // they add nothing in the forward; the backward masks them)
  f2 s1[4], s2[4];
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) s1[jj] = s2[jj] = f2{0.f, 0.f};
  // without KEEPX the second stream is read in groups of XG rows, each group
  // fenced off so the scheduler cannot hoist every load (and its registers)
  constexpr int XG = 4;
  u32x4 xt[XG];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    float z[8], dy[8];
    Vec<bf16>::to_f(zr[i], z);
    if (MODE == 1) {
      if constexpr (!KEEPX) {
        if (i % XG == 0) {
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int u = 0; u < XG; ++u)
            xt[u] = __builtin_amdgcn_raw_buffer_load_b128(xrs, vo(xoff, i + u), (i + u) * xstr, 0);
        }
      }
      Vec<bf16>::to_f(KEEPX ? xr[KEEPX ? i : 0] : xt[i % XG], dy);  // zero past the end: dv = 0
    }
    coop_accum<MODE, SILU>(z, dy, k2, s1, s2);
  }
  float t1, t2;
  GN_STAMP_AT(1);
  coop_block_sum(s1, s2, C, tpr, red, t1, t2);
  if (tid < C) {
    float* rp = a.sums + (long long)(j % a.R) * a.rstride + ((long long)b * C + tid) * 2;
    atomicAdd(rp, t1);
    atomicAdd(rp + 1, t2);
  }
  // every wave's atomics performed (acknowledged by the coherent point), then
  // the workgroup counts itself in.  Deliberately no release / acquire fences:
  // on gfx950 those write back / invalidate the whole XCD L2 (measured: ~15 us
  // per launch).  Nothing but atomics crosses workgroups here -- the sums and
  // the counter are agent-scope atomic RMWs and are read back with agent-scope
  // atomic loads (sc1), issued only after the counter load returned k.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  GN_STAMP_AT(2);
  if (tid == 0) {
    __hip_atomic_fetch_add(q.cnt + b, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int ok = !q.force_fallback;
    for (int n = 0; ok && __hip_atomic_load(q.cnt + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < q.k; ++n) {
      if (n >= GN_SPIN) ok = 0;
      else __builtin_amdgcn_s_sleep(2);
    }
    ok_sh = ok;
  }
  __syncthreads();
  GN_STAMP_AT(3);
  if (ok_sh) {
    if (tid < C) {  // every replica's pair in flight at once (a runtime loop waited per load)
      float v[2 * GN_COOP_RMAX];
#pragma unroll
      for (int r = 0; r < GN_COOP_RMAX; ++r) {
        float* rp = a.sums + (long long)min(r, a.R - 1) * a.rstride + ((long long)b * C + tid) * 2;
        v[2 * r] = __hip_atomic_load(rp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        v[2 * r + 1] = __hip_atomic_load(rp + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      float v1 = 0.f, v2 = 0.f;
#pragma unroll
      for (int r = 0; r < GN_COOP_RMAX; ++r)
        if (r < a.R) { v1 += v[2 * r]; v2 += v[2 * r + 1]; }
      cs[tid] = v1;
      cs[C + tid] = v2;
    }
  } else {
    // fallback: the whole clip from memory, by this workgroup alone
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) s1[jj] = s2[jj] = f2{0.f, 0.f};
    const unsigned zc0 = (unsigned)((((long long)b * a.P + r0) * a.ldz + cv) * 2);
    const unsigned xc0 = has_x ? (unsigned)((((long long)b * a.P + r0) * ldx + cv) * 2) : 0u;
    for (long long p = r0, i = 0; p < a.P; p += rpp, ++i) {
      float z[8], dy[8];
      Vec<bf16>::to_f(__builtin_amdgcn_raw_buffer_load_b128(zrs, zc0, (unsigned)(i * zstr), 0), z);
      if (MODE == 1) Vec<bf16>::to_f(__builtin_amdgcn_raw_buffer_load_b128(xrs, xc0, (unsigned)(i * xstr), 0), dy);
      coop_accum<MODE, SILU>(z, dy, k2, s1, s2);
    }
    float u1, u2;
    coop_block_sum(s1, s2, C, tpr, red, u1, u2);
    if (tid < C) {
      cs[tid] = u1;
      cs[C + tid] = u2;
    }
  }
  __syncthreads();

  // ---- group terms (MODE 0: mean, rstd; MODE 1: m1, m2)
  {
    const int lane = tid & 63, wave = tid >> 6, cg = C / a.G;
    for (int g = wave; g < a.G; g += GN_CT / 64) {
      if (MODE == 0) {
        double d1 = 0.0, d2 = 0.0;
        for (int c = g * cg + lane; c < (g + 1) * cg; c += 64) { d1 += cs[c]; d2 += cs[C + c]; }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) { d1 += __shfl_xor(d1, o, 64); d2 += __shfl_xor(d2, o, 64); }
        if (lane == 0) {
          const double n = (double)a.P * cg;
          const double m = d1 / n;
          double var = d2 / n - m * m;
          if (var < 0) var = 0;
          gt1[g] = (float)m;
          gt2[g] = (float)(1.0 / sqrt(var + (double)a.eps));
        }
      } else {
        const float* ssb = has_ss ? a.ss + (long long)b * 2 * C : nullptr;
        float m1 = 0.f, m2 = 0.f;
        for (int c = g * cg + lane; c < (g + 1) * cg; c += 64) {
          const float kk = a.gamma[c] * (ssb ? 1.f + ssb[c] : 1.f);
          m1 += kk * cs[c];
          m2 += kk * cs[C + c];
        }
        m1 = wave_sum(m1);
        m2 = wave_sum(m2);
        if (lane == 0) {
          const float n = (float)((double)a.P * cg);
          gt1[g] = m1 / n;
          gt2[g] = m2 / n;
        }
      }
    }
  }
  __syncthreads();
  if (j == 0) {
    if (MODE == 0) {
      if (tid < a.G) { a.mean[b * a.G + tid] = gt1[tid]; a.rstd[b * a.G + tid] = gt2[tid]; }
    } else if (tid < C) {
      const float r1 = cs[tid], r2 = cs[C + tid];
      const float scc = has_ss ? 1.f + a.ss[(long long)b * 2 * C + tid] : 1.f;
      const float gmc = a.gamma[tid], btc = a.beta[tid];
      if (a.dss) {
        a.dss[(long long)b * 2 * C + tid] = gmc * r2 + btc * r1;  // d scale
        a.dss[(long long)b * 2 * C + C + tid] = r1;               // d shift
      }
      if (a.dgamma) atomicAdd(a.dgamma + tid, scc * r2);  // fresh buffers were zeroed by the host
      if (a.dbeta) atomicAdd(a.dbeta + tid, scc * r1);
    }
  }

  // ---- phase 2: apply to the rows held in registers
  GN_STAMP_AT(4);
  f2 m1v = f2{0.f, 0.f}, m2v = f2{0.f, 0.f};
  if (MODE == 0) {
    coef(gt1[grp], gt2[grp]);
  } else {
    m1v = f2{-rs_f * gt1[grp], -rs_f * gt1[grp]};
    m2v = f2{-rs_f * gt2[grp], -rs_f * gt2[grp]};
  }
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    float z[8], o[8];
    // opaque: hipcc would otherwise keep phase 1's unpacked floats of every
    // row alive across the wait (8 VGPRs per row instead of 4)
    asm volatile("" : "+v"(zr[i]));
    if constexpr (KEEPX && MODE == 1) asm volatile("" : "+v"(xr[KEEPX ? i : 0]));
    Vec<bf16>::to_f(zr[i], z);
    if constexpr (has_x && !(KEEPX && MODE == 1)) {
      if (i % XG == 0) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < XG && u < NV; ++u)
          xt[u] = __builtin_amdgcn_raw_buffer_load_b128(xrs, vo(xoff, i + u), (i + u) * xstr, 0);
      }
    }
    float x[8];
    Vec<bf16>::to_f(KEEPX && MODE == 1 ? xr[KEEPX ? i : 0] : xt[i % XG], x);
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const f2 zz{z[2 * jj], z[2 * jj + 1]};
      if (MODE == 0) {
        f2 v = zz * k2.A[jj] + k2.B[jj];
        if (SILU) v *= sigmoid2(v);
        if (RES) v += f2{x[2 * jj], x[2 * jj + 1]};
        o[2 * jj] = v.x;
        o[2 * jj + 1] = v.y;
      } else {
        f2 dv = f2{x[2 * jj], x[2 * jj + 1]};
        if (SILU) dv *= silu_grad2(zz * k2.A[jj] + k2.B[jj]);
        const f2 zhat = zz * k2.rs[jj] + k2.zb[jj];
        const f2 v = dv * k2.K1[jj] + m1v + zhat * m2v;
        o[2 * jj] = v.x;
        o[2 * jj + 1] = v.y;
      }
    }
    const bf16x8 ob = bf16x8{(bf16)o[0], (bf16)o[1], (bf16)o[2], (bf16)o[3],
                             (bf16)o[4], (bf16)o[5], (bf16)o[6], (bf16)o[7]};
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, ob), ors, vo(ooff, i), i * ostr, 0);
  }
#ifdef DV_STAMP
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  GN_STAMP_AT(5);
#endif
}

// 0: automatic, 1: always the two-launch form, 2: single launch wherever it
// applies, with the wait skipped (every workgroup recomputes its clip's sums:
// the fallback's test), 3: single launch wherever it applies.
// Automatic = single launch only for the backward at 16 register passes (the
// 64^2 Cfg2 slabs): there it saves the second read of z and dy (33.0 vs 34.3
// us); everywhere else the two launches are faster.  The cross-workgroup sum
// costs ~8-10 us on MI355X -- agent-scope atomics and sc1 loads each take
// ~2 us to the coherent point and back (phase stamps, tools/gn_coop_probe.py,
// profiles/r06d_gn_single_launch_ab.txt) -- more than the kernel boundary it
// removes.
int g_gn_path = 0;

// The single-launch plan: bf16, C a power of two in [8, 512], nb <= 256, the
// rows of a workgroup in NV <= 16 register passes, and a `next` buffer large
// enough for R replicas of the sums plus nb counters.
bool gn_coop_plan(const GnArgs& a, GnCoop& q, int& nv, bool bwd) {
  if (g_gn_path == 1) return false;
  const int C = a.C;
  // a thread's 8 channels lie in one group (cg % 8 == 0)
  if (C < 8 || C > 512 || (C & (C - 1)) || a.G > 64 || (C / a.G) % 8 || a.nb < 1 || a.nb > 256 || !a.next)
    return false;
  if (a.ldz % 8 || a.ldo % 8 || (a.dy && a.lddy % 8) || (a.res && a.ldres % 8)) return false;
  const long long rows = (long long)a.nb * a.P;  // raw-buffer ranges stay below DMA_OOB
  const int ldmax = std::max({a.ldz, a.ldo, a.dy ? a.lddy : 0, a.res ? a.ldres : 0});
  if (rows * ldmax * 2 >= (long long)DMA_OOB) return false;
  const int tpr = C / 8, rpp = GN_CT / tpr;
  const long long kmax = 256 / a.nb;
  const long long nvmin = (a.P + kmax * rpp - 1) / (kmax * rpp);
  if (nvmin > 16) return false;
  nv = nvmin <= 1 ? 1 : nvmin <= 2 ? 2 : nvmin <= 4 ? 4 : nvmin <= 8 ? 8 : 16;
  if (g_gn_path == 0 && !(bwd && nv == 16)) return false;  // measured: two launches win
  q.rpw = (long long)nv * rpp;
  q.k = (int)((a.P + q.rpw - 1) / q.rpw);
  const long long rs = (long long)a.nb * C * 2;
  long long R = (a.next_n - a.nb) / rs;
  if (R < 1) return false;
  q.a = a;
  q.a.R = (int)(R < GN_COOP_RMAX ? R : GN_COOP_RMAX);  // 64 workgroups per clip: 64 / R adds per address
  q.a.rstride = rs;
  q.cnt = (int*)(a.sums + a.next_n - a.nb);
  q.force_fallback = g_gn_path == 2;
  return true;
}

// backward: dy stays in registers up to this many passes (both streams fit)
constexpr int GN_KEEPX_NV = 16;

template <int MODE>
void gn_coop_launch(const GnCoop& q, int nv, hipStream_t st) {
  const bool silu = q.a.act == DV_ACT_SILU, res = MODE == 0 && q.a.res != nullptr;
  dim3 g((unsigned)(q.a.nb * q.k));
#define DV_GNC3(NVV, S, R) gn_coop_kernel<MODE, NVV, S, R, (MODE == 1 && NVV <= GN_KEEPX_NV)><<<g, GN_CT, 0, st>>>(q)
#define DV_GNC2(NVV) (silu ? (res ? DV_GNC3(NVV, true, true) : DV_GNC3(NVV, true, false)) \
                           : (res ? DV_GNC3(NVV, false, true) : DV_GNC3(NVV, false, false)))
  switch (nv) {
    case 1: DV_GNC2(1); break;
    case 2: DV_GNC2(2); break;
    case 4: DV_GNC2(4); break;
    case 8: DV_GNC2(8); break;
    default: DV_GNC2(16); break;
  }
#undef DV_GNC2
#undef DV_GNC3
}

template <typename T>
int gn_fwd_t(GnArgs a, int sums_replicas, hipStream_t st) {
  const GnTune& t = gn_tune();
  if constexpr (sizeof(T) == 2) {
    GnCoop q{};
    int nv = 0;
    if (sums_replicas == 0 && !a.q && gn_coop_plan(a, q, nv, false)) {  // one launch: reduce + apply
      gn_coop_launch<0>(q, nv, st);
      return check_launch("gn_fwd");
    }
  }
  if (sums_replicas > 0) a.R = sums_replicas;  // statistics from the conv epilogue
  else gn_reduce_launch<T, 0>(a, t.ur0, t.tr0, st);
  gn_apply_launch<T, 0>(a, t.ua0, t.ta0, st);
  return check_launch("gn_fwd");
}

template <typename T>
int gn_bwd_t(GnArgs a, hipStream_t st) {
  const GnTune& t = gn_tune();
  if constexpr (sizeof(T) == 2) {
    GnCoop q{};
    int nv = 0;
    if (gn_coop_plan(a, q, nv, true)) {  // one launch: reduce + apply, data in registers
      if (!a.accumulate) {  // the kernel adds every clip's share
        if (a.dgamma) zero_f32(a.dgamma, a.C, st);
        if (a.dbeta) zero_f32(a.dbeta, a.C, st);
      }
      gn_coop_launch<1>(q, nv, st);
      return check_launch("gn_bwd");
    }
  }
  gn_reduce_launch<T, 1>(a, t.ur1, t.tr1, st);
  gn_apply_launch<T, 1>(a, t.ua1, t.ta1, st);  // U=2 (123 VGPRs, 4 waves/SIMD) measured ahead of U=4
  return check_launch("gn_bwd");
}

// --------------------------------------------------------------------------
// row LayerNorm: y = (x - mean) * rstd * g (+ b) (+ res); one wave per row,
// NV 16-byte vectors per lane (C <= 64 * VEC * NV).  Every load is
// unconditional (vector index clamped, out-of-row lanes masked to zero): a
// load under a lane branch made the compiler wait for all outstanding loads
// at the join, so x, res and dy of a row went out one after another.
// The backward writes per-block column partials of dg / db (plain stores) and
// ln_colsum_kernel sums them: 1,024 blocks adding 2C floats each into the
// same few lines with atomics serialised (33 us for 4,096 x 512 rows).
// --------------------------------------------------------------------------
template <typename T, int MODE, int NV>  // MODE 0 fwd, 1 bwd
__global__ __launch_bounds__(256) void ln_kernel(const T* x, int ldx, const T* dy, int lddy, T* out,
                                                 int ldo, const T* res, int ldres, long long rows,
                                                 int C, const float* g, const float* bias,
                                                 float eps, float* mean, float* rstd, float* part,
                                                 float* dg, float* db) {
  constexpr int VEC = 16 / sizeof(T);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int c0[NV];
  bool live[NV];
  float gv[NV][VEC];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = (k * 64 + lane) * VEC;
    live[k] = c < C;
    c0[k] = live[k] ? c : C - VEC;  // clamped: a valid address, masked below
#pragma unroll
    for (int e = 0; e < VEC; ++e) gv[k][e] = g[c0[k] + e];
  }
  float pg[NV][VEC], pb[NV][VEC];
#pragma unroll
  for (int k = 0; k < NV; ++k)
#pragma unroll
    for (int e = 0; e < VEC; ++e) pg[k][e] = pb[k][e] = 0.f;
  for (long long row = (long long)blockIdx.x * 4 + wave; row < rows; row += (long long)gridDim.x * 4) {
    u32x4 xr[NV], yr[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      xr[k] = *(const u32x4*)(x + row * ldx + c0[k]);
      if (MODE == 1) yr[k] = *(const u32x4*)(dy + row * lddy + c0[k]);
      else if (res) yr[k] = *(const u32x4*)(res + row * ldres + c0[k]);
    }
    float xv[NV][VEC];
    float s = 0.f, q = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      Vec<T>::to_f(xr[k], xv[k]);
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        if (!live[k]) xv[k][e] = 0.f;
        s += xv[k][e];
      }
    }
    const float mu = wave_sum(s) / C;
#pragma unroll
    for (int k = 0; k < NV; ++k)
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        const float d = live[k] ? xv[k][e] - mu : 0.f;
        q += d * d;
      }
    const float rs = rsqrtf(wave_sum(q) / C + eps);
    if (MODE == 0) {
      if (lane == 0 && mean) { mean[row] = mu; rstd[row] = rs; }
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        float o[VEC], r[VEC];
        if (res) Vec<T>::to_f(yr[k], r);
#pragma unroll
        for (int e = 0; e < VEC; ++e) {
          o[e] = (xv[k][e] - mu) * rs * gv[k][e] + (bias ? bias[c0[k] + e] : 0.f);
          if (res) o[e] += r[e];
        }
        if (live[k]) st_vec<T>(out + row * ldo + c0[k], o);
      }
    } else {
      // dxhat = dy*g; dx = rs*(dxhat - mean(dxhat) - xhat*mean(dxhat*xhat))
      float dyv[NV][VEC];
      float m1 = 0.f, m2 = 0.f;
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        Vec<T>::to_f(yr[k], dyv[k]);
#pragma unroll
        for (int e = 0; e < VEC; ++e) {
          if (!live[k]) dyv[k][e] = 0.f;
          const float xh = (xv[k][e] - mu) * rs;
          const float dxh = dyv[k][e] * gv[k][e];
          m1 += dxh;
          m2 += dxh * xh;
          pg[k][e] += dyv[k][e] * xh;
          pb[k][e] += dyv[k][e];
        }
      }
      m1 = wave_sum(m1) / C;
      m2 = wave_sum(m2) / C;
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        float o[VEC];
#pragma unroll
        for (int e = 0; e < VEC; ++e) {
          const float xh = (xv[k][e] - mu) * rs;
          o[e] = rs * (dyv[k][e] * gv[k][e] - m1 - xh * m2);
        }
        if (live[k]) st_vec<T>(out + row * ldo + c0[k], o);
      }
    }
  }
  if (MODE == 1) {  // this block's column partials: part[blk][0..C) dg, [C..2C) db
    __shared__ float red[2][4][64 * VEC * NV];
#pragma unroll
    for (int k = 0; k < NV; ++k)
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        red[0][wave][(k * 64 + lane) * VEC + e] = pg[k][e];
        red[1][wave][(k * 64 + lane) * VEC + e] = pb[k][e];
      }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += 256) {
      const float tg = red[0][0][c] + red[0][1][c] + red[0][2][c] + red[0][3][c];
      const float tb = red[1][0][c] + red[1][1][c] + red[1][2][c] + red[1][3][c];
      if (part) {  // many blocks: partials, summed by ln_colsum_kernel
        part[(long long)blockIdx.x * 2 * C + c] = tg;
        part[(long long)blockIdx.x * 2 * C + C + c] = tb;
      } else {     // a few blocks: atomics are uncontended, no second launch
        if (dg) atomicAdd(dg + c, tg);
        if (db) atomicAdd(db + c, tb);
      }
    }
  }
}

// dg[c] (+)= sum_b part[b][c], db[c] (+)= sum_b part[b][C + c]: block
// (x, y) owns 64 columns and every gridDim.y-th block row; its 4 waves take
// every 4th of those (8 loads in flight per lane), meet in LDS, and add their
// total with one atomic per column (gridDim.y adds per address)
__global__ __launch_bounds__(256) void ln_colsum_kernel(const float* part, int nblk, int C, float* dg,
                                                        float* db) {
  __shared__ float sh[4][64];
  const int col = blockIdx.x * 64 + (threadIdx.x & 63), grp = threadIdx.x >> 6;
  const int n2 = 2 * C, rs = 4 * gridDim.y;
  float v = 0.f;
  if (col < n2) {
    int r = blockIdx.y * 4 + grp;
    for (; r + 7 * rs < nblk; r += 8 * rs) {
      float t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) t[u] = part[(long long)(r + u * rs) * n2 + col];
      v += ((t[0] + t[1]) + (t[2] + t[3])) + ((t[4] + t[5]) + (t[6] + t[7]));
    }
    for (; r < nblk; r += rs) v += part[(long long)r * n2 + col];
  }
  sh[grp][threadIdx.x & 63] = v;
  __syncthreads();
  if (grp != 0 || col >= n2) return;
  v = sh[0][threadIdx.x] + sh[1][threadIdx.x] + sh[2][threadIdx.x] + sh[3][threadIdx.x];
  float* o = col < C ? (dg ? dg + col : nullptr) : (db ? db + col - C : nullptr);
  if (o) atomicAdd(o, v);  // dg / db accumulate (the caller zeroes fresh buffers)
}

template <typename T, int MODE>
void ln_launch(int nv, int blocks, const T* x, int ldx, const T* dy, int lddy, T* out, int ldo,
               const T* res, int ldres, long long rows, int C, const float* g, const float* bias,
               float eps, float* mean, float* rstd, float* part, float* dg, float* db, hipStream_t st) {
#define DV_LN(NVV) ln_kernel<T, MODE, NVV><<<blocks, 256, 0, st>>>(x, ldx, dy, lddy, out, ldo, res, ldres, \
                                                                  rows, C, g, bias, eps, mean, rstd, part, dg, db)
  switch (nv) {
    case 1: DV_LN(1); break;
    case 2: DV_LN(2); break;
    default: DV_LN(4); break;
  }
#undef DV_LN
}

}  // namespace

// DV_REQUIRE reporting the C entry point's name
#define DV_REQUIRE_AS(fn, cond, msg)                         \
  do {                                                       \
    if (!(cond)) {                                           \
      ::dv::set_error(std::string(fn) + ": " + (msg));       \
      return DV_ERR_INVALID;                                 \
    }                                                        \
  } while (0)

static int gn_fwd_impl(int dtype, const void* z, int ldz, void* y, int ldy, const void* res,
                       int ldres, int nb, long long P, int C, int G, float eps,
                       const float* gamma, const float* beta, const float* ss, int act,
                       float* mean, float* rstd, float* sums, float* next, long long next_n,
                       int sums_replicas, void* q, void* qs, void* stream, const char* fn) {
  DV_REQUIRE_AS(fn, z && y && gamma && beta && mean && rstd && sums, "null pointer");
  DV_REQUIRE_AS(fn, !q || (qs && dtype == DV_BF16 && C % 64 == 0 && ((uintptr_t)q & 7) == 0),
             "the MX-fp8 copy needs bf16, C % 64 == 0 and 8-B aligned q (with qs)");
  DV_REQUIRE_AS(fn, sums_replicas >= 0 && sums_replicas <= 64 &&
             (sums_replicas == 0 || !next || (long long)sums_replicas * nb * C * 2 <= next_n),
             "sums_replicas must fit the sums buffer (<= 64)");
  DV_REQUIRE_AS(fn, C % G == 0, "C % G != 0");
  const int VEC = dtype == DV_BF16 ? 8 : 4;
  DV_REQUIRE_AS(fn, C % VEC == 0 && ldz % VEC == 0 && ldy % VEC == 0 && (!res || ldres % VEC == 0),
             "channel counts / strides must be multiples of 16 bytes");
  DV_REQUIRE_AS(fn, C <= GN_CMAX && G <= 64, "C > 1024 or G > 64");
  DV_REQUIRE_AS(fn, next != sums || !next, "next must not alias sums");
  GnArgs a{};
  a.z = z; a.ldz = ldz; a.out = y; a.ldo = ldy; a.res = res; a.ldres = ldres; a.nb = nb;
  a.P = P; a.C = C; a.G = G; a.mean = mean; a.rstd = rstd; a.gamma = gamma; a.beta = beta;
  a.ss = ss; a.act = act; a.sums = sums; a.next = next; a.next_n = next ? next_n : 0; a.eps = eps;
  a.rstride = (long long)nb * C * 2;
  a.R = next && a.rstride > 0 ? (int)std::min<long long>(8, std::max<long long>(1, next_n / a.rstride)) : 1;
  a.q = (uint8_t*)q; a.qs = (unsigned*)qs;
  if (nb == 0 || P == 0) return DV_OK;
  hipStream_t st = (hipStream_t)stream;
  return dtype == DV_BF16 ? gn_fwd_t<bf16>(a, sums_replicas, st) : gn_fwd_t<float>(a, sums_replicas, st);
}

extern "C" int dv_gn_fwd(int dtype, const void* z, int ldz, void* y, int ldy, const void* res,
                         int ldres, int nb, long long P, int C, int G, float eps,
                         const float* gamma, const float* beta, const float* ss, int act,
                         float* mean, float* rstd, float* sums, float* next, long long next_n,
                         int sums_replicas, void* stream) {
  return gn_fwd_impl(dtype, z, ldz, y, ldy, res, ldres, nb, P, C, G, eps, gamma, beta, ss, act, mean,
                     rstd, sums, next, next_n, sums_replicas, nullptr, nullptr, stream, __func__);
}

extern "C" int dv_gn_fwd_mx8(const void* z, int ldz, void* y, int ldy, const void* res, int ldres,
                             int nb, long long P, int C, int G, float eps, const float* gamma,
                             const float* beta, const float* ss, int act, float* mean, float* rstd,
                             float* sums, float* next, long long next_n, int sums_replicas, void* q,
                             void* qs, void* stream) {
  DV_REQUIRE(q && qs, "null pointer");
  return gn_fwd_impl(DV_BF16, z, ldz, y, ldy, res, ldres, nb, P, C, G, eps, gamma, beta, ss, act, mean,
                     rstd, sums, next, next_n, sums_replicas, q, qs, stream, __func__);
}

extern "C" int dv_gn_bwd(int dtype, const void* dy, int lddy, const void* z, int ldz, void* dz,
                         int lddz, int nb, long long P, int C, int G, const float* gamma,
                         const float* beta, const float* ss, int act, const float* mean,
                         const float* rstd, float* dgamma, float* dbeta, float* dss, float* sums,
                         float* next, long long next_n, int accumulate, void* stream) {
  DV_REQUIRE(dy && z && dz && gamma && beta && mean && rstd && sums, "null pointer");
  const int VEC = dtype == DV_BF16 ? 8 : 4;
  DV_REQUIRE(C % VEC == 0 && ldz % VEC == 0 && lddy % VEC == 0 && lddz % VEC == 0,
             "channel counts / strides must be multiples of 16 bytes");
  DV_REQUIRE(C <= GN_CMAX && G <= 64 && C % G == 0, "bad C / G");
  DV_REQUIRE(next != sums || !next, "next must not alias sums");
  GnArgs a{};
  a.z = z; a.ldz = ldz; a.dy = dy; a.lddy = lddy; a.out = dz; a.ldo = lddz; a.nb = nb; a.P = P;
  a.C = C; a.G = G; a.mean = (float*)mean; a.rstd = (float*)rstd; a.gamma = gamma; a.beta = beta;
  a.ss = ss; a.act = act; a.sums = sums; a.next = next; a.next_n = next ? next_n : 0;
  a.rstride = (long long)nb * C * 2;
  a.R = next && a.rstride > 0 ? (int)std::min<long long>(8, std::max<long long>(1, next_n / a.rstride)) : 1;
  a.dgamma = dgamma; a.dbeta = dbeta; a.dss = dss; a.accumulate = accumulate;
  if (nb == 0 || P == 0) return DV_OK;
  hipStream_t st = (hipStream_t)stream;
  return dtype == DV_BF16 ? gn_bwd_t<bf16>(a, st) : gn_bwd_t<float>(a, st);
}

extern "C" int dv_gn_path(int mode) {
  DV_REQUIRE(mode >= 0 && mode <= 3,
             "mode must be 0 (auto), 1 (two launches), 2 (single launch, fallback) or 3 (single launch)");
  g_gn_path = mode;
  return DV_OK;
}

// 16-byte vectors per lane of one row (1, 2 or 4)
static int ln_nv(int C, int vec) {
  const int n = (C + 64 * vec - 1) / (64 * vec);
  return n <= 1 ? 1 : n <= 2 ? 2 : 4;
}

extern "C" int dv_ln_fwd(int dtype, const void* x, int ldx, void* y, int ldy, const void* res,
                         int ldres, long long rows, int C, const float* g, const float* b,
                         float eps, float* mean, float* rstd, void* stream) {
  DV_REQUIRE(x && y && g, "null pointer");
  const int VEC = dtype == DV_BF16 ? 8 : 4;
  DV_REQUIRE(C <= 64 * VEC * 4 && C % VEC == 0, "C must be a multiple of 16 bytes, <= 256 vectors");
  DV_REQUIRE(ldx % VEC == 0 && ldy % VEC == 0 && (!res || ldres % VEC == 0),
             "strides must be multiples of 16 bytes");
  if (rows == 0) return DV_OK;
  const int blocks = grid_for(rows, 4);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == DV_BF16)
    ln_launch<bf16, 0>(ln_nv(C, VEC), blocks, (const bf16*)x, ldx, nullptr, 0, (bf16*)y, ldy,
                       (const bf16*)res, ldres, rows, C, g, b, eps, mean, rstd, nullptr, nullptr, nullptr, st);
  else
    ln_launch<float, 0>(ln_nv(C, VEC), blocks, (const float*)x, ldx, nullptr, 0, (float*)y, ldy,
                        (const float*)res, ldres, rows, C, g, b, eps, mean, rstd, nullptr, nullptr, nullptr, st);
  return check_launch("ln_fwd");
}

extern "C" int dv_ln_bwd_ws(long long rows, int C, long long* need) {
  DV_REQUIRE(need && rows >= 0 && C > 0, "bad arguments");
  *need = (long long)std::max(1, std::min(grid_for(rows, 4), 1024)) * 2 * C;
  return DV_OK;
}

extern "C" int dv_ln_bwd(int dtype, const void* dy, int lddy, const void* x, int ldx, void* dx,
                         int lddx, long long rows, int C, const float* g, float eps, float* dg,
                         float* db, float* ws, long long ws_n, void* stream) {
  DV_REQUIRE(dy && x && dx && g && ws, "null pointer");
  const int VEC = dtype == DV_BF16 ? 8 : 4;
  DV_REQUIRE(C <= 64 * VEC * 4 && C % VEC == 0, "C must be a multiple of 16 bytes, <= 256 vectors");
  DV_REQUIRE(ldx % VEC == 0 && lddy % VEC == 0 && lddx % VEC == 0, "strides must be multiples of 16 bytes");
  if (rows == 0) return DV_OK;
  const int blocks = std::min(grid_for(rows, 4), 1024);
  DV_REQUIRE(ws_n >= (long long)blocks * 2 * C, "workspace smaller than dv_ln_bwd_ws");
  hipStream_t st = (hipStream_t)stream;
  float* part = blocks > 8 ? ws : nullptr;  // <= 8 blocks: direct atomics
  if (dtype == DV_BF16)
    ln_launch<bf16, 1>(ln_nv(C, VEC), blocks, (const bf16*)x, ldx, (const bf16*)dy, lddy, (bf16*)dx, lddx,
                       nullptr, 0, rows, C, g, nullptr, eps, nullptr, nullptr, part, dg, db, st);
  else
    ln_launch<float, 1>(ln_nv(C, VEC), blocks, (const float*)x, ldx, (const float*)dy, lddy, (float*)dx,
                        lddx, nullptr, 0, rows, C, g, nullptr, eps, nullptr, nullptr, part, dg, db, st);
  if (part && (dg || db)) {
    const unsigned ys = (unsigned)std::max(1, std::min(16, blocks / 32));  // >= 32 rows per block
    ln_colsum_kernel<<<dim3((2 * C + 63) / 64, ys), 256, 0, st>>>(ws, blocks, C, dg, db);
  }
  return check_launch("ln_bwd");
}
