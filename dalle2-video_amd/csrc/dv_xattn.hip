// CLIP-style cross attention of ResnetBlock3D (dalle2_video.py:159-162,
// 192-201; dalle2-pytorch CrossAttention, 8 heads x 64, null k/v prepended,
// logit factor 64^-0.5).  Each head attends over only 3 keys (null + 2 time
// tokens), so the projections fold per batch b:
//   A~[b][c][h*3+j] = s * sum_d Wq[h*64+d][c] K[b][h][j][d]      (scores = hn . A~)
//   V~[b][c][h*3+j] =     sum_d Wo[c][h*64+d] V[b][h][j][d]      (o = V~ p)
// A token then costs 2*24*C MACs instead of 2*512*C: the whole block
//   out = LN_g2(V~ softmax(LN_g1(x) A~)) + x
// is one HBM pass (read x, write out) in `xattn_fwd_kernel`.
#include "dv_common.h"

using namespace dv;

namespace {

constexpr int NH = 8, DH = 64, NK = 3, HK = NH * NK;  // 24 folded columns
constexpr int PPAD = 32;                                // padded P / dS row

int grid_for(long long work, int per_block = 256, int cap = 16384) {
  long long b = (work + per_block - 1) / per_block;
  if (b > cap) b = cap;
  if (b < 1) b = 1;
  return (int)b;
}

// K/V of head h, key j (j = 0: null kv) for batch b
__device__ __forceinline__ float kf(const float* kv, const float* null_kv, int b, int h, int j, int d,
                                    int v) {
  if (j == 0) return null_kv[v * DH + d];
  return kv[((long long)b * 2 + (j - 1)) * (2 * NH * DH) + v * NH * DH + h * DH + d];
}

// A~ and V~ as [nb][C][24]
__global__ void fold_fwd_kernel(const float* wq, const float* wo, const float* kv,
                                const float* null_kv, float* at, float* vt, int nb, int C,
                                float scale) {
  const long long n = (long long)nb * C * HK;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int k = (int)(i % HK);
    const long long bc = i / HK;
    const int c = (int)(bc % C), b = (int)(bc / C);
    const int h = k / NK, j = k % NK;
    float sa = 0.f, sv = 0.f;
    for (int d = 0; d < DH; ++d) {
      sa += wq[(long long)(h * DH + d) * C + c] * kf(kv, null_kv, b, h, j, d, 0);
      sv += wo[(long long)c * (NH * DH) + h * DH + d] * kf(kv, null_kv, b, h, j, d, 1);
    }
    at[i] = sa * scale;
    vt[i] = sv;
  }
}

template <typename T>
__device__ __forceinline__ float ldc(const T* p) { return (float)*p; }

// thread per token.  Saves per-token LN stats and P (T dtype, 32-wide rows).
template <typename T>
__global__ __launch_bounds__(256) void xattn_fwd_kernel(const T* x, int ldx, T* out, int ldo,
                                                        long long ntok, long long P, int C,
                                                        const float* g1, const float* g2,
                                                        const float* at, const float* vt,
                                                        float eps, float* stats, T* pbuf) {
  const long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (t >= ntok) return;
  const int b = (int)(t / P);
  const T* xr = x + t * ldx;
  const float* A = at + (long long)b * C * HK;
  const float* V = vt + (long long)b * C * HK;
  float mu = 0.f;
  for (int c = 0; c < C; ++c) mu += ldc(xr + c);
  mu /= C;
  float var = 0.f;
  for (int c = 0; c < C; ++c) { const float d = ldc(xr + c) - mu; var += d * d; }
  const float rs = rsqrtf(var / C + eps);
  float s[HK];
#pragma unroll
  for (int k = 0; k < HK; ++k) s[k] = 0.f;
  for (int c = 0; c < C; ++c) {
    const float hn = (ldc(xr + c) - mu) * rs * g1[c];
    const f32x4* a4 = (const f32x4*)(A + (long long)c * HK);
#pragma unroll
    for (int q = 0; q < HK / 4; ++q) {
      const f32x4 av = a4[q];
      s[4 * q] += hn * av[0]; s[4 * q + 1] += hn * av[1];
      s[4 * q + 2] += hn * av[2]; s[4 * q + 3] += hn * av[3];
    }
  }
#pragma unroll
  for (int h = 0; h < NH; ++h) {
    const float m = fmaxf(s[3 * h], fmaxf(s[3 * h + 1], s[3 * h + 2]));
    const float e0 = __expf(s[3 * h] - m), e1 = __expf(s[3 * h + 1] - m), e2 = __expf(s[3 * h + 2] - m);
    const float inv = 1.f / (e0 + e1 + e2);
    s[3 * h] = e0 * inv; s[3 * h + 1] = e1 * inv; s[3 * h + 2] = e2 * inv;
  }
  // the P row as stored (T-rounded) is what the backward recomputes with
  T* pr = pbuf + t * PPAD;
#pragma unroll
  for (int k = 0; k < PPAD; ++k) {
    const T v = (T)(k < HK ? s[k] : 0.f);
    pr[k] = v;
    if (k < HK) s[k] = (float)v;
  }
  auto o_at = [&](int c) {
    const f32x4* v4 = (const f32x4*)(V + (long long)c * HK);
    float o = 0.f;
#pragma unroll
    for (int q = 0; q < HK / 4; ++q) {
      const f32x4 vv = v4[q];
      o += s[4 * q] * vv[0] + s[4 * q + 1] * vv[1] + s[4 * q + 2] * vv[2] + s[4 * q + 3] * vv[3];
    }
    return o;
  };
  float mu2 = 0.f;
  for (int c = 0; c < C; ++c) mu2 += o_at(c);
  mu2 /= C;
  float var2 = 0.f;
  for (int c = 0; c < C; ++c) { const float d = o_at(c) - mu2; var2 += d * d; }
  const float rs2 = rsqrtf(var2 / C + eps);
  T* orow = out + t * ldo;
  for (int c = 0; c < C; ++c) orow[c] = (T)((o_at(c) - mu2) * rs2 * g2[c] + ldc(xr + c));
  float* st = stats + t * 4;
  st[0] = mu; st[1] = rs; st[2] = mu2; st[3] = rs2;
}

// Backward per token.  Writes dx (incl. the residual), dO (for dV~), dS' = rs1*dS
// (for dA~) and accumulates dg1, dg2 and the per-batch correction m[b][k] =
// sum_t mu1_t * dS'_tk.
template <typename T>
__global__ __launch_bounds__(256) void xattn_bwd_kernel(const T* dy, int lddy, const T* x, int ldx,
                                                        T* dx, int lddx, long long ntok,
                                                        long long P, int C, const float* g1,
                                                        const float* g2, const float* at,
                                                        const float* vt, const float* stats,
                                                        const T* pbuf, T* dobuf, T* dsbuf,
                                                        float* dg1, float* dg2, float* mcorr) {
  __shared__ float sg1[1024], sg2[1024];
  for (int c = threadIdx.x; c < C; c += blockDim.x) { sg1[c] = 0.f; sg2[c] = 0.f; }
  __syncthreads();
  const long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  const bool live = t < ntok;
  const long long tt = live ? t : 0;
  const int b = (int)(tt / P);
  const int lane = threadIdx.x & 63;
  const T* xr = x + tt * ldx;
  const T* dyr = dy + tt * lddy;
  const float* A = at + (long long)b * C * HK;
  const float* V = vt + (long long)b * C * HK;
  const float mu = stats[tt * 4], rs = stats[tt * 4 + 1], mu2 = stats[tt * 4 + 2], rs2 = stats[tt * 4 + 3];
  float p[HK];
#pragma unroll
  for (int k = 0; k < HK; ++k) p[k] = (float)pbuf[tt * PPAD + k];
  auto o_at = [&](int c) {
    const f32x4* v4 = (const f32x4*)(V + (long long)c * HK);
    float o = 0.f;
#pragma unroll
    for (int q = 0; q < HK / 4; ++q) {
      const f32x4 vv = v4[q];
      o += p[4 * q] * vv[0] + p[4 * q + 1] * vv[1] + p[4 * q + 2] * vv[2] + p[4 * q + 3] * vv[3];
    }
    return o;
  };
  // LN_out backward statistics
  float m1 = 0.f, m2 = 0.f;
  for (int c = 0; c < C; ++c) {
    const float oh = (o_at(c) - mu2) * rs2;
    const float dyc = live ? ldc(dyr + c) : 0.f;
    const float doh = dyc * g2[c];
    m1 += doh;
    m2 += doh * oh;
    float part = wave_sum(dyc * oh);
    if (lane == 0) atomicAdd(&sg2[c], part);
  }
  m1 /= C;
  m2 /= C;
  // do_c, dp
  float dp[HK];
#pragma unroll
  for (int k = 0; k < HK; ++k) dp[k] = 0.f;
  for (int c = 0; c < C; ++c) {
    const float oh = (o_at(c) - mu2) * rs2;
    const float dyc = live ? ldc(dyr + c) : 0.f;
    const float dO = rs2 * (dyc * g2[c] - m1 - oh * m2);
    if (live) dobuf[tt * C + c] = (T)dO;
    const f32x4* v4 = (const f32x4*)(V + (long long)c * HK);
#pragma unroll
    for (int q = 0; q < HK / 4; ++q) {
      const f32x4 vv = v4[q];
      dp[4 * q] += dO * vv[0]; dp[4 * q + 1] += dO * vv[1];
      dp[4 * q + 2] += dO * vv[2]; dp[4 * q + 3] += dO * vv[3];
    }
  }
  // softmax backward per head
  float ds[HK];
#pragma unroll
  for (int h = 0; h < NH; ++h) {
    const float sdot = p[3 * h] * dp[3 * h] + p[3 * h + 1] * dp[3 * h + 1] + p[3 * h + 2] * dp[3 * h + 2];
#pragma unroll
    for (int j = 0; j < NK; ++j) ds[3 * h + j] = p[3 * h + j] * (dp[3 * h + j] - sdot);
  }
  if (live) {
#pragma unroll
    for (int k = 0; k < PPAD; ++k) dsbuf[tt * PPAD + k] = (T)(k < HK ? rs * ds[k] : 0.f);
  }
  // per-batch correction m[b][k] = sum_t mu1_t * rs1_t * ds_tk
  const int b0 = __builtin_amdgcn_readfirstlane(b);
  const bool uniform = __all(b == b0);
#pragma unroll
  for (int k = 0; k < HK; ++k) {
    const float v = live ? mu * rs * ds[k] : 0.f;
    if (uniform) {
      const float w = wave_sum(v);
      if (lane == 0) atomicAdd(mcorr + (long long)b0 * HK + k, w);
    } else if (live) {
      atomicAdd(mcorr + (long long)b * HK + k, v);
    }
  }
  // LN_in backward: dhn_c = sum_k ds_k A[c][k]
  auto dhn_at = [&](int c) {
    const f32x4* a4 = (const f32x4*)(A + (long long)c * HK);
    float r = 0.f;
#pragma unroll
    for (int q = 0; q < HK / 4; ++q) {
      const f32x4 av = a4[q];
      r += ds[4 * q] * av[0] + ds[4 * q + 1] * av[1] + ds[4 * q + 2] * av[2] + ds[4 * q + 3] * av[3];
    }
    return r;
  };
  float n1 = 0.f, n2 = 0.f;
  for (int c = 0; c < C; ++c) {
    const float xh = (ldc(xr + c) - mu) * rs;
    const float dhn = dhn_at(c);
    const float dxh = dhn * g1[c];
    n1 += dxh;
    n2 += dxh * xh;
    float part = wave_sum(live ? dhn * xh : 0.f);
    if (lane == 0) atomicAdd(&sg1[c], part);
  }
  n1 /= C;
  n2 /= C;
  if (live) {
    T* dxr = dx + tt * lddx;
    for (int c = 0; c < C; ++c) {
      const float xh = (ldc(xr + c) - mu) * rs;
      const float dxh = dhn_at(c) * g1[c];
      dxr[c] = (T)(rs * (dxh - n1 - xh * n2) + ldc(dyr + c));
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    atomicAdd(dg1 + c, sg1[c]);
    atomicAdd(dg2 + c, sg2[c]);
  }
}

// dA~ = g1 * (raw - m), raw = ws_a[b][k][c] (from the wgrad GEMM), in place into
// [nb][C][24] layout; dV~ from ws_v[b][k][c] likewise (no correction).
__global__ void fold_grad_finish_kernel(const float* ws_a, const float* ws_v, const float* g1,
                                        const float* mcorr, float* dat, float* dvt, int nb, int C) {
  const long long n = (long long)nb * C * HK;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int k = (int)(i % HK);
    const long long bc = i / HK;
    const int c = (int)(bc % C), b = (int)(bc / C);
    const long long wi = ((long long)b * PPAD + k) * C + c;
    dat[i] = g1[c] * (ws_a[wi] - mcorr[b * HK + k]);
    dvt[i] = ws_v[wi];
  }
}

// parameter grads of the fold: dWq, dWo and dK/dV -> d(kv) and d(null_kv)
__global__ void fold_bwd_w_kernel(const float* dat, const float* dvt, const float* kv,
                                  const float* null_kv, float* dwq, float* dwo, int nb, int C,
                                  float scale, int accumulate) {
  const long long n = (long long)NH * DH * C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    // dWq[hd][c]   (i = hd*C + c)
    {
      const int c = (int)(i % C), hd = (int)(i / C);
      const int h = hd / DH, d = hd % DH;
      float s = 0.f;
      for (int b = 0; b < nb; ++b)
        for (int j = 0; j < NK; ++j)
          s += dat[((long long)b * C + c) * HK + h * NK + j] * kf(kv, null_kv, b, h, j, d, 0);
      dwq[i] = accumulate ? dwq[i] + s * scale : s * scale;
    }
    // dWo[c][hd]   (i = c*512 + hd)
    {
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

// dKf/dVf[b][h][j][d] -> dkv[b][n][...] (j>=1) and dnull_kv (j==0, summed)
__global__ void fold_bwd_kv_kernel(const float* dat, const float* dvt, const float* wq,
                                   const float* wo, float* dkv, float* dnull, int nb, int C,
                                   float scale) {
  const int n = nb * NH * NK * DH;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int d = i % DH;
  const int j = (i / DH) % NK;
  const int h = (i / (DH * NK)) % NH;
  const int b = i / (DH * NK * NH);
  float sk = 0.f, sv = 0.f;
  for (int c = 0; c < C; ++c) {
    sk += dat[((long long)b * C + c) * HK + h * NK + j] * wq[(long long)(h * DH + d) * C + c];
    sv += dvt[((long long)b * C + c) * HK + h * NK + j] * wo[(long long)c * (NH * DH) + h * DH + d];
  }
  sk *= scale;
  if (j == 0) {
    atomicAdd(dnull + d, sk);
    atomicAdd(dnull + DH + d, sv);
  } else {
    dkv[((long long)b * 2 + (j - 1)) * (2 * NH * DH) + h * DH + d] = sk;
    dkv[((long long)b * 2 + (j - 1)) * (2 * NH * DH) + NH * DH + h * DH + d] = sv;
  }
}

}  // namespace

extern "C" int dv_xattn_fold(const float* wq, const float* wo, const float* kv,
                             const float* null_kv, float* at, float* vt, int nb, int C,
                             float scale, void* stream) {
  DV_REQUIRE(wq && wo && kv && null_kv && at && vt, "null pointer");
  const long long n = (long long)nb * C * HK;
  fold_fwd_kernel<<<grid_for(n), 256, 0, (hipStream_t)stream>>>(wq, wo, kv, null_kv, at, vt, nb, C, scale);
  return check_launch("xattn_fold");
}

extern "C" int dv_xattn_fwd(int dtype, const void* x, int ldx, void* out, int ldo, long long ntok,
                            long long P, int C, const float* g1, const float* g2, const float* at,
                            const float* vt, float eps, float* stats, void* pbuf, void* stream) {
  DV_REQUIRE(x && out && g1 && g2 && at && vt && stats && pbuf, "null pointer");
  DV_REQUIRE(C <= 1024, "C too large");
  hipStream_t st = (hipStream_t)stream;
  const int g = grid_for(ntok);
  if (dtype == DV_BF16)
    xattn_fwd_kernel<bf16><<<g, 256, 0, st>>>((const bf16*)x, ldx, (bf16*)out, ldo, ntok, P, C, g1, g2, at, vt, eps, stats, (bf16*)pbuf);
  else
    xattn_fwd_kernel<float><<<g, 256, 0, st>>>((const float*)x, ldx, (float*)out, ldo, ntok, P, C, g1, g2, at, vt, eps, stats, (float*)pbuf);
  return check_launch("xattn_fwd");
}

extern "C" int dv_xattn_bwd_tokens(int dtype, const void* dy, int lddy, const void* x, int ldx,
                                   void* dx, int lddx, long long ntok, long long P, int C,
                                   const float* g1, const float* g2, const float* at,
                                   const float* vt, const float* stats, const void* pbuf,
                                   void* dobuf, void* dsbuf, float* dg1, float* dg2, float* mcorr,
                                   void* stream) {
  DV_REQUIRE(dy && x && dx && stats && pbuf && dobuf && dsbuf && dg1 && dg2 && mcorr, "null pointer");
  DV_REQUIRE(C <= 1024, "C too large");
  hipStream_t st = (hipStream_t)stream;
  const int g = (int)((ntok + 255) / 256);
  if (dtype == DV_BF16)
    xattn_bwd_kernel<bf16><<<g, 256, 0, st>>>((const bf16*)dy, lddy, (const bf16*)x, ldx, (bf16*)dx, lddx, ntok, P, C, g1, g2, at, vt, stats, (const bf16*)pbuf, (bf16*)dobuf, (bf16*)dsbuf, dg1, dg2, mcorr);
  else
    xattn_bwd_kernel<float><<<g, 256, 0, st>>>((const float*)dy, lddy, (const float*)x, ldx, (float*)dx, lddx, ntok, P, C, g1, g2, at, vt, stats, (const float*)pbuf, (float*)dobuf, (float*)dsbuf, dg1, dg2, mcorr);
  return check_launch("xattn_bwd_tokens");
}

extern "C" int dv_xattn_fold_bwd(const float* ws_a, const float* ws_v, const float* g1,
                                 const float* mcorr, const float* wq, const float* wo,
                                 const float* kv, const float* null_kv, float* dat, float* dvt,
                                 float* dwq, float* dwo, float* dkv, float* dnull, int nb, int C,
                                 float scale, int accumulate, void* stream) {
  DV_REQUIRE(ws_a && ws_v && g1 && mcorr && wq && wo && kv && null_kv && dat && dvt && dwq && dwo && dkv && dnull,
             "null pointer");
  hipStream_t st = (hipStream_t)stream;
  const long long n = (long long)nb * C * HK;
  fold_grad_finish_kernel<<<grid_for(n), 256, 0, st>>>(ws_a, ws_v, g1, mcorr, dat, dvt, nb, C);
  fold_bwd_w_kernel<<<grid_for((long long)NH * DH * C), 256, 0, st>>>(dat, dvt, kv, null_kv, dwq, dwo, nb, C, scale, accumulate);
  if (!accumulate) (void)hipMemsetAsync(dnull, 0, sizeof(float) * 2 * DH, st);
  fold_bwd_kv_kernel<<<(nb * NH * NK * DH + 255) / 256, 256, 0, st>>>(dat, dvt, wq, wo, dkv, dnull, nb, C, scale);
  return check_launch("xattn_fold_bwd");
}
