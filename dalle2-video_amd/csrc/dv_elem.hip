// Byte-moving and small kernels of the Unet3D path (all HBM- or launch-bound):
//   layout conversion at the NCTHW module boundary, space-to-depth
//   (Downsample3D, dalle2_video.py:22-25), SiLU+PixelShuffle
//   (PixelShuffleUpsample3D, :64-78), q_sample + l2 loss (p_losses :1956,
//   :1997-2002), the p_sample posterior update (:1551-1664), the time MLPs
//   (:348-357, :755-761, ResnetBlock3D.time_mlp :150-155), AdamW and the
//   gradient norm (trainer.py:247-274).
#include "dv_common.h"

using namespace dv;

namespace {

int grid_for(long long work, int per_block = 256, int cap = 16384) {
  long long b = (work + per_block - 1) / per_block;
  if (b > cap) b = cap;
  if (b < 1) b = 1;
  return (int)b;
}

#define GRID_STRIDE(i, n) \
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < (n); i += (long long)gridDim.x * blockDim.x)

template <typename T>
__global__ void ncthw_to_cl_kernel(const float* x, T* y, int B, int C, int T_, int HW, int cpad) {
  const long long npix = (long long)B * T_ * HW;
  GRID_STRIDE(p, npix) {
    const int hw = (int)(p % HW);
    const long long ft = p / HW;
    const int t = (int)(ft % T_), b = (int)(ft / T_);
    for (int c = 0; c < cpad; ++c) {
      float v = c < C ? x[(((long long)b * C + c) * T_ + t) * HW + hw] : 0.f;
      y[p * cpad + c] = (T)v;
    }
  }
}

template <typename T>
__global__ void cl_to_ncthw_kernel(const T* y, int ld, float* x, int B, int C, int T_, int HW) {
  const long long npix = (long long)B * T_ * HW;
  GRID_STRIDE(p, npix) {
    const int hw = (int)(p % HW);
    const long long ft = p / HW;
    const int t = (int)(ft % T_), b = (int)(ft / T_);
    for (int c = 0; c < C; ++c) x[(((long long)b * C + c) * T_ + t) * HW + hw] = (float)y[p * ld + c];
  }
}

// unit = (frame, low-res y, x, group of VEC high-res channels); grid y walks the
// low-res rows (f, y), grid x a row's (x, channel group) units: one 32-bit
// division per unit (a flat 64-bit index took four 64-bit divisions, each a
// ~150-instruction sequence, and left the pass VALU-bound)
// MODE 1 adds r0 / r1 (high-res, strides ldr0 / ldr1; null: none) to the output
// Rows past the grid's 65,535 go two per trip, both rows' loads ahead of
// either row's stores.
template <typename T>
struct ShufIn {
  u32x4 a[4];  // MODE 1: the low-res span; MODE 0: the four high-res pixels
  u32x4 b[4];  // MODE 1: r0 at the four high-res pixels; MODE 0: z (the low-res span)
  u32x4 c[4];  // MODE 1: r1 at the four high-res pixels
};
// NX: the extra sources (MODE 1: r0, r1; MODE 0: z), a template count so no
// load sits under a run-time branch (hipcc drained vmcnt at each such join)
template <typename T, int MODE, int NX>
__global__ __launch_bounds__(256, 2) void shuffle_kernel(const T* src, int lds, T* dst, int ldd, const T* z, int ldz,
                               const T* r0, int ldr0, const T* r1, int ldr1, int nf, int H, int W,
                               int C, int act) {
  constexpr int VEC = 16 / sizeof(T);
  const int cg = C / VEC;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= W * cg) return;
  const int x = t / cg, g = t - x * cg;
  const int c0 = g * VEC;
  const int rows = nf * H;
  auto hp_of = [&](int row, int i, int j) {
    const long long f = row / H;
    const int y = row - (int)f * H;
    return (f * 2 * H + 2 * y + i) * 2 * W + 2 * x + j;
  };
  auto load = [&](int row, ShufIn<T>& in) {
    const long long lp = (long long)row * W + x;  // low-res pixel
    if (MODE == 1) {
#pragma unroll
      for (int q = 0; q < 4; ++q) in.a[q] = *(const u32x4*)(src + lp * lds + c0 * 4 + q * VEC);
      if constexpr (NX >= 1) {
#pragma unroll
        for (int q = 0; q < 4; ++q) in.b[q] = *(const u32x4*)(r0 + hp_of(row, q >> 1, q & 1) * ldr0 + c0);
      }
      if constexpr (NX >= 2) {
#pragma unroll
        for (int q = 0; q < 4; ++q) in.c[q] = *(const u32x4*)(r1 + hp_of(row, q >> 1, q & 1) * ldr1 + c0);
      }
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) in.a[q] = *(const u32x4*)(src + hp_of(row, q >> 1, q & 1) * lds + c0);
      if constexpr (NX >= 1) {
#pragma unroll
        for (int q = 0; q < 4; ++q) in.b[q] = *(const u32x4*)(z + lp * ldz + c0 * 4 + q * VEC);
      }
    }
  };
  auto finish = [&](int row, const ShufIn<T>& in) {
    const long long lp = (long long)row * W + x;
    float lo[4 * VEC];  // low-res span, element (c - c0)*4 + i*2 + j
    if (MODE == 1) {
#pragma unroll
      for (int q = 0; q < 4; ++q) Vec<T>::to_f(in.a[q], lo + q * VEC);
#pragma unroll
      for (int e = 0; e < 4 * VEC; ++e) lo[e] = act == DV_ACT_SILU ? silu_f(lo[e]) : lo[e];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float hv[VEC];
#pragma unroll
        for (int e = 0; e < VEC; ++e) hv[e] = lo[e * 4 + q];
        if constexpr (NX >= 1) {
          float rv[VEC];
          Vec<T>::to_f(in.b[q], rv);
#pragma unroll
          for (int e = 0; e < VEC; ++e) hv[e] += rv[e];
        }
        if constexpr (NX >= 2) {
          float rv[VEC];
          Vec<T>::to_f(in.c[q], rv);
#pragma unroll
          for (int e = 0; e < VEC; ++e) hv[e] += rv[e];
        }
        T o[VEC];
#pragma unroll
        for (int e = 0; e < VEC; ++e) o[e] = (T)hv[e];
        *(u32x4*)(dst + hp_of(row, q >> 1, q & 1) * ldd + c0) = *(const u32x4*)o;
      }
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float hv[VEC];
        Vec<T>::to_f(in.a[q], hv);
#pragma unroll
        for (int e = 0; e < VEC; ++e) lo[e * 4 + q] = hv[e];
      }
      if constexpr (NX >= 1) {  // backward of SiLU+shuffle: multiply by silu'(z)
        float zz[4 * VEC];
#pragma unroll
        for (int q = 0; q < 4; ++q) Vec<T>::to_f(in.b[q], zz + q * VEC);
#pragma unroll
        for (int e = 0; e < 4 * VEC; ++e) {
          const float sg = sigmoid_f(zz[e]);
          lo[e] *= sg * (1.f + zz[e] * (1.f - sg));
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        T o[VEC];
#pragma unroll
        for (int e = 0; e < VEC; ++e) o[e] = (T)lo[q * VEC + e];
        *(u32x4*)(dst + lp * ldd + c0 * 4 + q * VEC) = *(const u32x4*)o;
      }
    }
  };
  const int gy = gridDim.y;
  int row = blockIdx.y;
  for (; row + gy < rows; row += 2 * gy) {
    ShufIn<T> in0, in1;
    load(row, in0);
    load(row + gy, in1);
    __builtin_amdgcn_sched_barrier(0);  // every load of both rows ahead of the math
    finish(row, in0);
    finish(row + gy, in1);
  }
  if (row < rows) {
    ShufIn<T> in0;
    load(row, in0);
    finish(row, in0);
  }
}

template <typename T>
__global__ void q_sample_kernel(const float* x0, const float* noise, const long long* t,
                                const float* sa, const float* s1m, T* y, int B, int C, int T_,
                                int HW, int cpad, int normalize, int nt) {
  const long long npix = (long long)B * T_ * HW;
  GRID_STRIDE(p, npix) {
    const int hw = (int)(p % HW);
    const long long ft = p / HW;
    const int tt = (int)(ft % T_), b = (int)(ft / T_);
    const long long ti = t[b];
    // a timestep outside the schedule poisons the output (NaN) instead of
    // reading past the table (the reference's gather raises)
    const bool ok = ti >= 0 && ti < nt;
    const float a = ok ? sa[ti] : __builtin_nanf(""), s = ok ? s1m[ti] : __builtin_nanf("");
    for (int c = 0; c < cpad; ++c) {
      float v = 0.f;
      if (c < C) {
        const long long i = (((long long)b * C + c) * T_ + tt) * HW + hw;
        const float xs = normalize ? x0[i] * 2.f - 1.f : x0[i];
        v = a * xs + s * noise[i];
      }
      y[p * cpad + c] = (T)v;
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void mse_kernel(const T* pred, int ld, const float* target, int B,
                                                  int C, int T_, int HW, const float* w,
                                                  float* loss, float scale) {
  __shared__ float sh[4];
  const long long npix = (long long)B * T_ * HW;
  const long long stride = (long long)gridDim.x * blockDim.x;
  float acc = 0.f;
  // 4 pixels per trip, their loads independent of each other (few blocks: every
  // block ends in ONE atomic on the loss word, and same-word atomics serialise)
  for (long long p0 = (long long)blockIdx.x * blockDim.x + threadIdx.x; p0 < npix; p0 += 4 * stride) {
    long long pp[4];
    long long tb[4];
    float wb[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long long p = p0 + u * stride;
      const bool live = p < npix;
      pp[u] = live ? p : p0;
      const int hw = (int)(pp[u] % HW);
      const long long ft = pp[u] / HW;
      const int tt = (int)(ft % T_), b = (int)(ft / T_);
      tb[u] = ((long long)b * C * T_ + tt) * HW + hw;  // channel 0 of this pixel in the NCTHW target
      wb[u] = live ? (w ? w[b] : 1.f) : 0.f;
    }
    for (int c = 0; c < C; ++c) {
      float d[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        d[u] = (float)pred[pp[u] * ld + c] - target[tb[u] + (long long)c * T_ * HW];
#pragma unroll
      for (int u = 0; u < 4; ++u) acc += wb[u] * d[u] * d[u];
    }
  }
  acc = block_sum<256>(acc, sh);
  if (threadIdx.x == 0) atomicAdd(loss, acc * scale);
}

template <typename T>
__global__ void mse_bwd_kernel(const T* pred, int ld, const float* target, int B, int C, int T_,
                               int HW, const float* w, const float* dloss, float scale, T* dp,
                               int lddp) {
  const long long npix = (long long)B * T_ * HW;
  const float g = dloss[0] * scale;
  GRID_STRIDE(p, npix) {
    const int hw = (int)(p % HW);
    const long long ft = p / HW;
    const int tt = (int)(ft % T_), b = (int)(ft / T_);
    const float wb = w ? w[b] : 1.f;
    for (int c = 0; c < C; ++c) {
      const float d = (float)pred[p * ld + c] - target[(((long long)b * C + c) * T_ + tt) * HW + hw];
      dp[p * lddp + c] = (T)(2.f * g * wb * d);
    }
  }
}

// freqs[k] = exp(-k*ln(1e4)/(half-1)) is a constant table built once on the host
// exactly as SinusoidalPosEmb builds it; t is cast to f32 (time.type_as(x)).
__global__ void sinusoidal_kernel(const long long* t, const float* freqs, float* out, int B, int dim) {
  const int half = dim / 2;
  GRID_STRIDE(i, (long long)B * dim) {
    const int b = (int)(i / dim), k = (int)(i % dim);
    const float a = (float)t[b] * freqs[k < half ? k : k - half];
    out[i] = k < half ? sinf(a) : cosf(a);
  }
}

__device__ __forceinline__ float act_in_f(float x, int act) { return act == 1 ? silu_f(x) : x; }
__device__ __forceinline__ float act_in_d(float x, int act) {
  if (act != 1) return 1.f;
  const float s = sigmoid_f(x);
  return s * (1.f + x * (1.f - s));
}
__device__ __forceinline__ float gelu_f(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_d(float x) {
  return 0.5f * (1.f + erff(x * 0.70710678118654752f)) + x * 0.39894228040143268f * expf(-0.5f * x * x);
}

// y[b][n] = act_out(sum_k act_in(x[b][k]) W[n][k] + bias[n]); one wave per n
__global__ __launch_bounds__(256) void linear_small_kernel(const float* x, int ldx, const float* W,
                                                           const float* bias, float* y, int ldy,
                                                           float* z, int B, int K, int N,
                                                           int act_in, int act_out) {
  const int lane = threadIdx.x & 63;
  const int n = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (n >= N) return;
  for (int b = 0; b < B; ++b) {
    float s = 0.f;
    for (int k = lane; k < K; k += 64) s += act_in_f(x[(long long)b * ldx + k], act_in) * W[(long long)n * K + k];
    s = wave_sum(s);
    if (lane == 0) {
      s += bias ? bias[n] : 0.f;
      if (z) z[(long long)b * N + n] = s;
      y[(long long)b * ldy + n] = act_out == 2 ? gelu_f(s) : s;
    }
  }
}

__device__ __forceinline__ float lin_g(const float* dy, int lddy, const float* z, int b, int n, int N,
                                       int act_out) {
  const float d = dy[(long long)b * lddy + n];
  return act_out == 2 ? d * gelu_d(z[(long long)b * N + n]) : d;
}

__global__ void linear_small_dw_kernel(const float* dy, int lddy, const float* x, int ldx,
                                       const float* z, float* dW, float* db, int B, int K, int N,
                                       int act_in, int act_out, int accumulate) {
  GRID_STRIDE(i, (long long)N * K) {
    const int n = (int)(i / K), k = (int)(i % K);
    float s = 0.f, sb = 0.f;
    for (int b = 0; b < B; ++b) {
      const float g = lin_g(dy, lddy, z, b, n, N, act_out);
      s += g * act_in_f(x[(long long)b * ldx + k], act_in);
      sb += g;
    }
    dW[i] = accumulate ? dW[i] + s : s;
    if (db && k == 0) db[n] = accumulate ? db[n] + sb : sb;
  }
}

// dx[b][k] (+)= act_in'(x) * sum_n g[b][n] W[n][k].  Block = 256 k-columns x
// one 32-row slice of n (grid.y); g for the slice is staged in LDS once, W
// rows are streamed coalesced with 8 loads in flight; slices meet in f32
// atomics (dx pre-zeroed or accumulated into).  B <= 16.
__global__ __launch_bounds__(256) void linear_small_dx_kernel(const float* dy, int lddy,
                                                              const float* x, int ldx,
                                                              const float* W, const float* z,
                                                              float* dx, int lddx, int B, int K,
                                                              int N, int act_in, int act_out) {
  constexpr int MAXB = 16, NS = 32;
  __shared__ float gs[MAXB][NS];
  const int n0 = blockIdx.y * NS;
  const int nend = min(NS, N - n0);
  for (int i = threadIdx.x; i < MAXB * NS; i += 256) {
    const int b = i / NS, nn = i % NS;
    gs[b][nn] = (b < B && nn < nend) ? lin_g(dy, lddy, z, b, n0 + nn, N, act_out) : 0.f;
  }
  __syncthreads();
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k >= K) return;
  float acc[MAXB];
#pragma unroll
  for (int b = 0; b < MAXB; ++b) acc[b] = 0.f;
  const float* wp = W + (long long)n0 * K + k;
#pragma unroll 8
  for (int nn = 0; nn < nend; ++nn) {
    const float w = wp[(long long)nn * K];
#pragma unroll
    for (int b = 0; b < MAXB; ++b) acc[b] += gs[b][nn] * w;  // rows b >= B are zero
  }
  for (int b = 0; b < B; ++b)
    atomicAdd(dx + (long long)b * lddx + k, acc[b] * act_in_d(x[(long long)b * ldx + k], act_in));
}


// ---------------------------------------------------------------------------
// grouped small linears (dv_linear_group_*): every entry's rows are cut into
// 64-row workgroup tiles; the entry table rides in the kernel arguments (no
// device table, graph-capture safe).  Forward: 4 lanes per output row stream
// its W row in 16-B pieces against act_in(x) staged in LDS, then a 2-step
// lane reduction.  Backward: the same row mapping writes dW / db; for dx each
// thread owns a k column and streams the tile's W rows coalesced, and the
// tiles meet in f32 atomics in `ws`; the workgroup arriving last applies
// act_in'(x), writes dx and re-zeroes ws.
// ---------------------------------------------------------------------------
constexpr int LG_MAX = 48, LG_ROWS = 64, LG_MAXB = 8, LG_MAXK = 512;
struct LinGroupArgs {
  const float* x;
  float* dx;
  float* ws;
  int B, K, act_in, n, acc_dx, finalize;
  int blk0[LG_MAX + 1];
  DvLinEntry e[LG_MAX];
};

__device__ __forceinline__ int lg_entry(const LinGroupArgs& a, int blk) {
  int e = 0;
  while (e + 1 < a.n && blk >= a.blk0[e + 1]) ++e;
  return e;
}

// act_in(x) into LDS: every thread's (at most 16) loads issued together from
// clamped indices (a run-time trip count left one load in flight per thread)
__device__ __forceinline__ void lg_stage_x(const LinGroupArgs& a, float* xs) {
  const int nx = a.B * a.K, tid = threadIdx.x;
  float v[LG_MAXB * LG_MAXK / 256];
#pragma unroll
  for (int u = 0; u < LG_MAXB * LG_MAXK / 256; ++u) v[u] = a.x[min(tid + 256 * u, nx - 1)];
#pragma unroll
  for (int u = 0; u < LG_MAXB * LG_MAXK / 256; ++u)
    if (tid + 256 * u < nx) xs[tid + 256 * u] = act_in_f(v[u], a.act_in);
}

__global__ __launch_bounds__(256) void linear_group_fwd_kernel(LinGroupArgs a) {
  __shared__ __attribute__((aligned(16))) float xs[LG_MAXB * LG_MAXK];
  const int tid = threadIdx.x;
  const int e = lg_entry(a, blockIdx.x);
  const DvLinEntry E = a.e[e];
  const int lane = tid & 63, q = lane & 3;
  const int n = (blockIdx.x - a.blk0[e]) * LG_ROWS + (tid >> 6) * 16 + (lane >> 2);
  // the lane's W pieces (k = 4q + 16u), 8 at a time in flight; rows past the
  // entry and k past K read clamped addresses and are masked (the loop waited
  // for each load before the next with one load per trip under a branch)
  const float* wr = E.w + (long long)min(n, E.n - 1) * a.K;
  constexpr int U = 8;
  f32x4 w[U];
#pragma unroll
  for (int u = 0; u < U; ++u) w[u] = *(const f32x4*)(wr + min(q * 4 + 16 * u, a.K - 4));
  lg_stage_x(a, xs);
  __syncthreads();
  float acc[LG_MAXB];
#pragma unroll
  for (int b = 0; b < LG_MAXB; ++b) acc[b] = 0.f;
  for (int k0 = 0; k0 < a.K; k0 += 16 * U) {
    f32x4 wn[U];
    if (k0 + 16 * U < a.K) {
#pragma unroll
      for (int u = 0; u < U; ++u) wn[u] = *(const f32x4*)(wr + min(k0 + 16 * U + q * 4 + 16 * u, a.K - 4));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = k0 + q * 4 + 16 * u;
      if (k < a.K) {
#pragma unroll
        for (int b = 0; b < LG_MAXB; ++b) {
          if (b < a.B) {
            const f32x4 xv = *(const f32x4*)(xs + b * a.K + k);
            acc[b] += w[u][0] * xv[0] + w[u][1] * xv[1] + w[u][2] * xv[2] + w[u][3] * xv[3];
          }
        }
      }
    }
    if (k0 + 16 * U < a.K) {
#pragma unroll
      for (int u = 0; u < U; ++u) w[u] = wn[u];
    }
  }
#pragma unroll
  for (int b = 0; b < LG_MAXB; ++b) {
    acc[b] += __shfl_xor(acc[b], 1, 64);
    acc[b] += __shfl_xor(acc[b], 2, 64);
  }
  if (n < E.n && q == 0) {
    const float bias = E.bias ? E.bias[n] : 0.f;
#pragma unroll
    for (int b = 0; b < LG_MAXB; ++b)
      if (b < a.B) E.y[(long long)b * E.n + n] = acc[b] + bias;
  }
}

__global__ __launch_bounds__(256) void linear_group_bwd_kernel(LinGroupArgs a) {
  __shared__ __attribute__((aligned(16))) float xs[LG_MAXB * LG_MAXK];
  __shared__ float gs[LG_MAXB][LG_ROWS];
  __shared__ int last;
  const int tid = threadIdx.x;
  lg_stage_x(a, xs);
  const int e = lg_entry(a, blockIdx.x);
  const DvLinEntry E = a.e[e];
  const int row0 = (blockIdx.x - a.blk0[e]) * LG_ROWS;
  const int rows = min(LG_ROWS, E.n - row0);
  {
    float g[LG_MAXB * LG_ROWS / 256];
#pragma unroll
    for (int u = 0; u < LG_MAXB * LG_ROWS / 256; ++u) {
      const int i = tid + 256 * u, b = i / LG_ROWS, r = i % LG_ROWS;
      g[u] = E.y[(long long)min(b, a.B - 1) * E.n + row0 + min(r, rows - 1)];
    }
#pragma unroll
    for (int u = 0; u < LG_MAXB * LG_ROWS / 256; ++u) {
      const int i = tid + 256 * u, b = i / LG_ROWS, r = i % LG_ROWS;
      gs[b][r] = (b < a.B && r < rows) ? g[u] : 0.f;
    }
  }
  __syncthreads();
  // dW / db rows: 4 lanes per row
  if (E.dw) {
    const int lane = tid & 63, q = lane & 3, r = (tid >> 6) * 16 + (lane >> 2);
    if (r < rows) {
      const int n = row0 + r;
      float* dwr = E.dw + (long long)n * a.K;
      constexpr int U = 8;  // pieces k = k0 + 4q + 16u; the accumulated dW read U at a time
      for (int k0 = 0; k0 < a.K; k0 += 16 * U) {
        f32x4 prev[U];
        if (E.accumulate_w) {
#pragma unroll
          for (int u = 0; u < U; ++u) prev[u] = *(const f32x4*)(dwr + min(k0 + q * 4 + 16 * u, a.K - 4));
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int k = k0 + q * 4 + 16 * u;
          if (k < a.K) {
            f32x4 s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int b = 0; b < LG_MAXB; ++b) {
              if (b < a.B) {
                const f32x4 xv = *(const f32x4*)(xs + b * a.K + k);
                s += gs[b][r] * xv;
              }
            }
            if (E.accumulate_w) s += prev[u];
            *(f32x4*)(dwr + k) = s;
          }
        }
      }
      if (E.db && q == 0) {
        float sb = 0.f;
        for (int b = 0; b < a.B; ++b) sb += gs[b][r];
        E.db[n] = E.accumulate_w ? E.db[n] + sb : sb;
      }
    }
  }
  // dx partial over this tile's rows: one thread per k column
  if (a.dx) {
    for (int k = tid; k < a.K; k += 256) {
      float acc[LG_MAXB];
#pragma unroll
      for (int b = 0; b < LG_MAXB; ++b) acc[b] = 0.f;
      const float* wp = E.w + (long long)row0 * a.K + k;
      // 8 rows per trip, their loads together (clamped rows: gs is zero past `rows`)
      for (int r0 = 0; r0 < rows; r0 += 8) {
        float w[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) w[j] = wp[(long long)min(r0 + j, rows - 1) * a.K];
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
          for (int b = 0; b < LG_MAXB; ++b) acc[b] += gs[b][r0 + j] * w[j];  // rows b >= B are zero
      }
      for (int b = 0; b < a.B; ++b) atomicAdd(a.ws + b * a.K + k, acc[b]);
    }
    if (!a.finalize) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's atomics are performed
    __syncthreads();
    if (tid == 0) last = atomicAdd((unsigned*)(a.ws + a.B * a.K), 1u) == gridDim.x - 1;
    __syncthreads();
    if (!last) return;
    // the last workgroup's pass is the launch's tail: every load of it in one batch
    constexpr int UF = LG_MAXB * LG_MAXK / 256;
    const int nx = a.B * a.K;
    float v[UF], xv[UF], dv[UF];
#pragma unroll
    for (int u = 0; u < UF; ++u) {
      const int i = min(tid + 256 * u, nx - 1);
      v[u] = __hip_atomic_load(a.ws + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      xv[u] = a.x[i];
      dv[u] = a.acc_dx ? a.dx[i] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < UF; ++u) {
      const int i = tid + 256 * u;
      if (i < nx) {
        a.ws[i] = 0.f;
        a.dx[i] = dv[u] + v[u] * act_in_d(xv[u], a.act_in);
      }
    }
    if (tid == 0) *(unsigned*)(a.ws + a.B * a.K) = 0u;
  }
}

__device__ __forceinline__ void adamw_elem(float& pi, float gi, float& mi, float& vi, bool decay, float lr,
                                           float b1, float b2, float eps, float wd, float step,
                                           float bc2_sqrt) {
  if (decay) pi *= 1.f - lr * wd;
  mi = mi + (1.f - b1) * (gi - mi);
  vi = vi * b2 + (1.f - b2) * gi * gi;
  const float denom = sqrtf(vi) / bc2_sqrt + eps;
  pi = pi - step * (mi / denom);
}

// scalar form (any alignment)
__global__ void adamw_kernel(float* p, const float* g, float* m, float* v, long long n,
                             long long n_wd, float lr, float b1, float b2, float eps, float wd,
                             float bc1, float bc2_sqrt, const float* clip) {
  const float cc = clip ? clip[0] : 1.f;
  const float step = lr / bc1;
  GRID_STRIDE(i, n) {
    float pi = p[i], mi = m[i], vi = v[i];
    adamw_elem(pi, g[i] * cc, mi, vi, i < n_wd, lr, b1, b2, eps, wd, step, bc2_sqrt);
    m[i] = mi;
    v[i] = vi;
    p[i] = pi;
  }
}

// 16-B vectors, two per thread per trip: all eight loads of a trip are issued
// before its six stores (vmcnt retires loads and stores in order, so a load
// issued behind a store would also wait for that store's write)
__global__ void adamw_vec_kernel(float* p, const float* g, float* m, float* v, long long n,
                             long long n_wd, float lr, float b1, float b2, float eps, float wd,
                             float bc1, float bc2_sqrt, const float* clip) {
  const float cc = clip ? clip[0] : 1.f;
  const float step = lr / bc1;
  const long long n4 = n / 4;
  const long long stride = (long long)gridDim.x * blockDim.x;
  f32x4* P4 = (f32x4*)p;
  const f32x4* G4 = (const f32x4*)g;
  f32x4* M4 = (f32x4*)m;
  f32x4* V4 = (f32x4*)v;
  for (long long i0 = (long long)blockIdx.x * blockDim.x + threadIdx.x; i0 < n4; i0 += 2 * stride) {
    long long ix[2] = {i0, i0 + stride};
    const bool live1 = ix[1] < n4;
    if (!live1) ix[1] = i0;  // clamped: unconditional loads, store skipped
    f32x4 pv[2], gv[2], mv[2], vv[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      gv[k] = G4[ix[k]];
      pv[k] = P4[ix[k]];
      mv[k] = M4[ix[k]];
      vv[k] = V4[ix[k]];
    }
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float pi = pv[k][e], mi = mv[k][e], vi = vv[k][e];
        adamw_elem(pi, gv[k][e] * cc, mi, vi, 4 * ix[k] + e < n_wd, lr, b1, b2, eps, wd, step, bc2_sqrt);
        pv[k][e] = pi;
        mv[k][e] = mi;
        vv[k][e] = vi;
      }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      if (k == 1 && !live1) break;
      M4[ix[k]] = mv[k];
      V4[ix[k]] = vv[k];
      P4[ix[k]] = pv[k];
    }
  }
  // the n % 4 tail
  const long long t = 4 * n4 + (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) {
    float pi = p[t], mi = m[t], vi = v[t];
    adamw_elem(pi, g[t] * cc, mi, vi, t < n_wd, lr, b1, b2, eps, wd, step, bc2_sqrt);
    m[t] = mi;
    v[t] = vi;
    p[t] = pi;
  }
}

// sum of squares of the flat gradient: 16-B loads, 8 independent loads in
// flight per lane (the scalar grid-stride loop was latency-bound at ~2.7 TB/s).
// Each block writes its partial to part[blockIdx.x]; clip_coef_kernel sums
// the partials in a fixed order, so the norm — and the clipped update — is
// bit-identical run to run and on every data-parallel rank (an atomic sum
// made the ranks' weights drift apart by an ulp per step)
__global__ __launch_bounds__(256) void sumsq_kernel(const float* x, long long n, float* part) {
  __shared__ float sh[4];
  const long long stride = (long long)gridDim.x * blockDim.x;
  const long long t0 = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  f32x4 a = {0.f, 0.f, 0.f, 0.f}, b = a;
  long long n4 = 0;
  if (((uintptr_t)x & 15) == 0) {
    n4 = n / 4;
    const f32x4* x4 = (const f32x4*)x;
    long long i = t0;
    for (; i + 7 * stride < n4; i += 8 * stride) {  // 8 x 16 B in flight per lane
      f32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = x4[i + u * stride];
      a += (v[0] * v[0] + v[1] * v[1]) + (v[2] * v[2] + v[3] * v[3]);
      b += (v[4] * v[4] + v[5] * v[5]) + (v[6] * v[6] + v[7] * v[7]);
    }
    for (; i < n4; i += stride) a += x4[i] * x4[i];
  }
  a += b;
  float acc = (a[0] + a[1]) + (a[2] + a[3]);
  for (long long i = n4 * 4 + t0; i < n; i += stride) acc += x[i] * x[i];
  acc = block_sum<256>(acc, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = acc;
}

// coef = prescale * min(max_norm / (||prescale * g|| + 1e-6), 1)  (prescale = 1/world
// folds the DDP average into the update; torch.nn.utils.clip_grad_norm_ semantics).
// One block: thread t sums partials t, t + 256, ... then a fixed-shape block sum.
__global__ __launch_bounds__(256) void clip_coef_kernel(const float* part, int nparts, float max_norm,
                                                        float prescale, float* coef) {
  __shared__ float sh[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < nparts; i += 256) s += part[i];
  s = block_sum<256>(s, sh);
  if (threadIdx.x != 0) return;
  const float norm = prescale * sqrtf(s);
  float c = max_norm > 0.f ? max_norm / (norm + 1e-6f) : 1.f;
  coef[0] = prescale * (c < 1.f ? c : 1.f);
  coef[1] = norm;
}

template <typename T>
__global__ void p_sample_kernel(const float* x, const T* eps, int ld, const float* noise,
                                const long long* t, const float* sra, const float* srm1,
                                const float* c1, const float* c2, const float* logvar, float* out,
                                float* x0_out, int B, int C, int T_, int HW, int clip, int nt) {
  const long long n = (long long)B * C * T_ * HW;
  GRID_STRIDE(i, n) {
    const int hw = (int)(i % HW);
    long long r = i / HW;
    const int tt = (int)(r % T_);
    r /= T_;
    const int c = (int)(r % C), b = (int)(r / C);
    const long long ti0 = t[b];
    const bool ok = ti0 >= 0 && ti0 < nt;  // out-of-schedule t: NaN, no OOB read
    const long long ti = ok ? ti0 : 0;
    const long long p = ((long long)b * T_ + tt) * HW + hw;
    const float e = ld > 0 ? (float)eps[p * ld + c] : ((const float*)eps)[i];
    float x0 = sra[ti] * x[i] - srm1[ti] * e;
    if (clip) x0 = fminf(fmaxf(x0, -1.f), 1.f);
    const float mean = c1[ti] * x0 + c2[ti] * x[i];
    const float nz = ti == 0 ? 0.f : 1.f;
    out[i] = ok ? mean + nz * expf(0.5f * logvar[ti]) * noise[i] : __builtin_nanf("");
    if (x0_out) x0_out[i] = ok ? x0 : __builtin_nanf("");
  }
}


// per-frame nearest resize of NCTHW f32 planes (F.interpolate(mode="nearest"),
// resize_image_to at dalle2_video.py:2257, 1129-1146); optional clamp
__device__ __forceinline__ int nearest_src(int o, int in, int out) {
  if (out == in) return o;
  if (out == 2 * in) return o >> 1;
  const float scale = (float)in / (float)out;
  const int s = (int)floorf((float)o * scale);
  return s < in - 1 ? s : in - 1;
}
__global__ void resize_nearest_kernel(const float* x, float* y, long long planes, int hin, int win,
                                      int hout, int wout, int do_clamp, float lo, float hi) {
  const long long n = planes * hout * wout;
  GRID_STRIDE(i, n) {
    const int ox = (int)(i % wout);
    const long long r = i / wout;
    const int oy = (int)(r % hout);
    const long long pl = r / hout;
    float v = x[(pl * hin + nearest_src(oy, hin, hout)) * win + nearest_src(ox, win, wout)];
    if (do_clamp) v = fminf(fmaxf(v, lo), hi);
    y[i] = v;
  }
}

// kornia gaussian_blur2d per frame: separable normalized gaussian, 'reflect' border
__device__ __forceinline__ int reflect_idx(int i, int n) {
  if (i < 0) i = -i;
  if (i >= n) i = 2 * n - 2 - i;
  return i;
}
__global__ void blur_kernel(const float* x, float* y, long long planes, int H, int W, int ks,
                            const float* w1) {
  const long long n = planes * H * W;
  const int r = ks / 2;
  GRID_STRIDE(i, n) {
    const int ox = (int)(i % W);
    const long long rr = i / W;
    const int oy = (int)(rr % H);
    const long long pl = rr / H;
    float acc = 0.f;
    for (int dy = -r; dy <= r; ++dy) {
      const int yy = reflect_idx(oy + dy, H);
      float row = 0.f;
      for (int dx = -r; dx <= r; ++dx) row += w1[dx + r] * x[(pl * H + yy) * W + reflect_idx(ox + dx, W)];
      acc += w1[dy + r] * row;
    }
    y[i] = acc;
  }
}

}  // namespace

#define DISPATCH(dtype, KERNEL_CALL_F32, KERNEL_CALL_BF16) \
  do {                                                      \
    if ((dtype) == DV_F32) { KERNEL_CALL_F32; }             \
    else if ((dtype) == DV_BF16) { KERNEL_CALL_BF16; }      \
    else DV_REQUIRE(false, "unknown dtype");                \
  } while (0)

extern "C" int dv_ncthw_to_cl(int dtype, const float* x, void* y, int B, int C, int T, int H,
                              int W, int cpad, void* stream) {
  DV_REQUIRE(x && y && cpad >= C, "bad arguments");
  const long long npix = (long long)B * T * H * W;
  hipStream_t st = (hipStream_t)stream;
  DISPATCH(dtype,
           (ncthw_to_cl_kernel<float><<<grid_for(npix), 256, 0, st>>>(x, (float*)y, B, C, T, H * W, cpad)),
           (ncthw_to_cl_kernel<bf16><<<grid_for(npix), 256, 0, st>>>(x, (bf16*)y, B, C, T, H * W, cpad)));
  return check_launch("ncthw_to_cl");
}

extern "C" int dv_cl_to_ncthw(int dtype, const void* y, int ld, float* x, int B, int C, int T, int H,
                              int W, void* stream) {
  DV_REQUIRE(x && y && ld >= C, "bad arguments");
  const long long npix = (long long)B * T * H * W;
  hipStream_t st = (hipStream_t)stream;
  DISPATCH(dtype,
           (cl_to_ncthw_kernel<float><<<grid_for(npix), 256, 0, st>>>((const float*)y, ld, x, B, C, T, H * W)),
           (cl_to_ncthw_kernel<bf16><<<grid_for(npix), 256, 0, st>>>((const bf16*)y, ld, x, B, C, T, H * W)));
  return check_launch("cl_to_ncthw");
}

extern "C" int dv_shuffle(int dtype, int mode, const void* src, int lds, void* dst, int ldd,
                          const void* z, int ldz, const void* r0, int ldr0, const void* r1,
                          int ldr1, int nf, int H, int W, int C, int act, void* stream) {
  DV_REQUIRE(src && dst && (mode == 0 || mode == 1), "bad arguments");
  DV_REQUIRE(mode == 1 || (!r0 && !r1), "residuals are added by mode 1 only");
  if (!r0 && r1) {
    r0 = r1; ldr0 = ldr1; r1 = nullptr;
  }
  const int VEC = dtype == DV_BF16 ? 8 : 4;
  DV_REQUIRE(C % VEC == 0 && lds % VEC == 0 && ldd % VEC == 0 && (!z || ldz % VEC == 0) &&
                 (!r0 || (ldr0 % VEC == 0 && ldr0 >= C)) && (!r1 || (ldr1 % VEC == 0 && ldr1 >= C)),
             "channels / strides must be multiples of 16 bytes");
  if ((long long)nf * H * W * C == 0) return DV_OK;
  DV_REQUIRE((long long)W * (C / VEC) < (1ll << 31) && (long long)nf * H < (1ll << 31), "shape too large");
  // (a grid of fewer rows -- several row pairs per workgroup -- measured equal:
  // profiles/r05ag_shuffle_ab.txt)
  const dim3 grid((unsigned)((W * (C / VEC) + 255) / 256), (unsigned)std::min(nf * H, 65535));
  hipStream_t st = (hipStream_t)stream;
  const int nx = mode == 0 ? (z ? 1 : 0) : (r1 ? 2 : r0 ? 1 : 0);
#define DV_SH(TT, M, NX) shuffle_kernel<TT, M, NX><<<grid, 256, 0, st>>>((const TT*)src, lds, (TT*)dst, ldd, \
    (const TT*)z, ldz, (const TT*)r0, ldr0, (const TT*)r1, ldr1, nf, H, W, C, act)
#define DV_SH_T(TT)                          \
  if (mode == 0) {                           \
    if (nx) DV_SH(TT, 0, 1);                 \
    else DV_SH(TT, 0, 0);                    \
  } else {                                   \
    if (nx == 2) DV_SH(TT, 1, 2);            \
    else if (nx == 1) DV_SH(TT, 1, 1);       \
    else DV_SH(TT, 1, 0);                    \
  }
  if (dtype == DV_F32) {
    DV_SH_T(float)
  } else {
    DV_SH_T(bf16)
  }
#undef DV_SH_T
#undef DV_SH
  return check_launch("shuffle");
}

extern "C" int dv_q_sample(int dtype, const float* x0, const float* noise, const long long* t,
                           const float* sqrt_ac, const float* sqrt_1m_ac, void* y, int B, int C,
                           int T, int H, int W, int cpad, int normalize, int num_timesteps,
                           void* stream) {
  DV_REQUIRE(x0 && noise && t && sqrt_ac && sqrt_1m_ac && y && cpad >= C && num_timesteps > 0,
             "bad arguments");
  const long long npix = (long long)B * T * H * W;
  hipStream_t st = (hipStream_t)stream;
  DISPATCH(dtype,
           (q_sample_kernel<float><<<grid_for(npix), 256, 0, st>>>(x0, noise, t, sqrt_ac, sqrt_1m_ac, (float*)y, B, C, T, H * W, cpad, normalize, num_timesteps)),
           (q_sample_kernel<bf16><<<grid_for(npix), 256, 0, st>>>(x0, noise, t, sqrt_ac, sqrt_1m_ac, (bf16*)y, B, C, T, H * W, cpad, normalize, num_timesteps)));
  return check_launch("q_sample");
}

extern "C" int dv_mse_loss(int dtype, const void* pred, int ld, const float* target, int B, int C,
                           int T, int H, int W, const float* sample_w, float* loss, void* stream) {
  DV_REQUIRE(pred && target && loss, "bad arguments");
  const long long npix = (long long)B * T * H * W;
  const float scale = 1.f / (float)((double)B * C * T * H * W);
  hipStream_t st = (hipStream_t)stream;
  zero_f32(loss, 1, st);
  const int g = grid_for((npix + 3) / 4, 256, 256);
  DISPATCH(dtype,
           (mse_kernel<float><<<g, 256, 0, st>>>((const float*)pred, ld, target, B, C, T, H * W, sample_w, loss, scale)),
           (mse_kernel<bf16><<<g, 256, 0, st>>>((const bf16*)pred, ld, target, B, C, T, H * W, sample_w, loss, scale)));
  return check_launch("mse_loss");
}

extern "C" int dv_mse_loss_bwd(int dtype, const void* pred, int ld, const float* target, int B,
                               int C, int T, int H, int W, const float* sample_w,
                               const float* dloss, void* dpred, int lddp, void* stream) {
  DV_REQUIRE(pred && target && dloss && dpred, "bad arguments");
  const long long npix = (long long)B * T * H * W;
  const float scale = 1.f / (float)((double)B * C * T * H * W);
  hipStream_t st = (hipStream_t)stream;
  DISPATCH(dtype,
           (mse_bwd_kernel<float><<<grid_for(npix), 256, 0, st>>>((const float*)pred, ld, target, B, C, T, H * W, sample_w, dloss, scale, (float*)dpred, lddp)),
           (mse_bwd_kernel<bf16><<<grid_for(npix), 256, 0, st>>>((const bf16*)pred, ld, target, B, C, T, H * W, sample_w, dloss, scale, (bf16*)dpred, lddp)));
  return check_launch("mse_loss_bwd");
}

extern "C" int dv_sinusoidal(const long long* t, const float* freqs, float* out, int B, int dim,
                             void* stream) {
  DV_REQUIRE(t && freqs && out && dim >= 4 && dim % 2 == 0, "bad arguments");
  sinusoidal_kernel<<<grid_for((long long)B * dim), 256, 0, (hipStream_t)stream>>>(t, freqs, out, B, dim);
  return check_launch("sinusoidal");
}

extern "C" int dv_linear_small_fwd(const float* x, int ldx, const float* W, const float* bias,
                                   float* y, int ldy, float* z, int B, int K, int N, int act_in,
                                   int act_out, void* stream) {
  DV_REQUIRE(x && W && y && (act_out != 2 || z), "bad arguments");
  linear_small_kernel<<<(N + 3) / 4, 256, 0, (hipStream_t)stream>>>(x, ldx, W, bias, y, ldy, z, B,
                                                                     K, N, act_in, act_out);
  return check_launch("linear_small_fwd");
}

extern "C" int dv_linear_small_bwd(const float* dy, int lddy, const float* x, int ldx,
                                   const float* W, const float* z, float* dx, int lddx, float* dW,
                                   float* db, int B, int K, int N, int act_in, int act_out,
                                   int accumulate_dx, int accumulate_w, void* stream) {
  DV_REQUIRE(dy && x && W && (act_out != 2 || z), "bad arguments");
  hipStream_t st = (hipStream_t)stream;
  DV_REQUIRE(B <= 16, "linear_small supports B <= 16 rows");
  if (dW) linear_small_dw_kernel<<<grid_for((long long)N * K), 256, 0, st>>>(dy, lddy, x, ldx, z, dW, db, B, K, N, act_in, act_out, accumulate_w);
  if (dx) {
    if (!accumulate_dx) zero_f32(dx, (long long)(B - 1) * lddx + K, st);
    dim3 grid((K + 255) / 256, (N + 31) / 32);
    linear_small_dx_kernel<<<grid, 256, 0, st>>>(dy, lddy, x, ldx, W, z, dx, lddx, B, K, N, act_in, act_out);
  }
  return check_launch("linear_small_bwd");
}

extern "C" int dv_adamw(float* p, const float* g, float* m, float* v, long long n, long long n_wd,
                        float lr, float beta1, float beta2, float eps, float wd, float bc1,
                        float bc2_sqrt, const float* clip_coef, void* stream) {
  DV_REQUIRE(p && g && m && v, "null pointer");
  const bool al16 = ((reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(g) |
                      reinterpret_cast<uintptr_t>(m) | reinterpret_cast<uintptr_t>(v)) & 15) == 0;
  if (al16)
    adamw_vec_kernel<<<grid_for((n + 7) / 8, 256, 8192), 256, 0, (hipStream_t)stream>>>(
        p, g, m, v, n, n_wd, lr, beta1, beta2, eps, wd, bc1, bc2_sqrt, clip_coef);
  else
    adamw_kernel<<<grid_for(n, 256, 8192), 256, 0, (hipStream_t)stream>>>(p, g, m, v, n, n_wd, lr, beta1, beta2, eps, wd, bc1, bc2_sqrt, clip_coef);
  return check_launch("adamw");
}

extern "C" int dv_grad_clip_coef(const float* g, long long n, float max_norm, float prescale,
                                 float* ws, void* stream) {
  // ws[1] = update coefficient, ws[2] = gradient norm, ws[4 ..] = per-block
  // partial sums (DV_CLIP_WS_FLOATS in all)
  DV_REQUIRE(g && ws, "null pointer");
  hipStream_t st = (hipStream_t)stream;
  const unsigned nb = grid_for(n, 256, DV_CLIP_WS_FLOATS - 4);
  sumsq_kernel<<<nb, 256, 0, st>>>(g, n, ws + 4);
  clip_coef_kernel<<<1, 256, 0, st>>>(ws + 4, (int)nb, max_norm, prescale, ws + 1);
  return check_launch("grad_clip_coef");
}

extern "C" int dv_p_sample(int dtype, const float* x, const void* eps, int ld, const float* noise,
                           const long long* t, const float* sqrt_recip_ac,
                           const float* sqrt_recipm1_ac, const float* coef1, const float* coef2,
                           const float* logvar, float* out, float* x0_out, int B, int C, int T,
                           int H, int W, int clip, int num_timesteps, void* stream) {
  DV_REQUIRE(x && eps && noise && t && out && num_timesteps > 0, "bad arguments");
  const long long n = (long long)B * C * T * H * W;
  hipStream_t st = (hipStream_t)stream;
  DISPATCH(dtype,
           (p_sample_kernel<float><<<grid_for(n), 256, 0, st>>>(x, (const float*)eps, ld, noise, t, sqrt_recip_ac, sqrt_recipm1_ac, coef1, coef2, logvar, out, x0_out, B, C, T, H * W, clip, num_timesteps)),
           (p_sample_kernel<bf16><<<grid_for(n), 256, 0, st>>>(x, (const bf16*)eps, ld, noise, t, sqrt_recip_ac, sqrt_recipm1_ac, coef1, coef2, logvar, out, x0_out, B, C, T, H * W, clip, num_timesteps)));
  return check_launch("p_sample");
}

extern "C" int dv_resize_nearest(const float* x, float* y, long long planes, int hin, int win,
                                 int hout, int wout, int do_clamp, float lo, float hi,
                                 void* stream) {
  DV_REQUIRE(x && y && hin > 0 && win > 0 && hout > 0 && wout > 0, "bad arguments");
  resize_nearest_kernel<<<grid_for(planes * hout * wout), 256, 0, (hipStream_t)stream>>>(
      x, y, planes, hin, win, hout, wout, do_clamp, lo, hi);
  return check_launch("resize_nearest");
}

extern "C" int dv_gaussian_blur(const float* x, float* y, long long planes, int H, int W, int ks,
                                const float* w1, void* stream) {
  DV_REQUIRE(x && y && w1 && (ks & 1) && ks / 2 < H && ks / 2 < W, "bad arguments");
  blur_kernel<<<grid_for(planes * H * W), 256, 0, (hipStream_t)stream>>>(x, y, planes, H, W, ks, w1);
  return check_launch("gaussian_blur");
}

static int linear_group(bool bwd, const float* x, int B, int K, int act_in, const DvLinEntry* entries,
                        int n_entries, float* dx, int accumulate_dx, float* ws, hipStream_t st) {
  bool any = false;
  for (int s0 = 0; s0 < n_entries; s0 += LG_MAX) {
    LinGroupArgs a;
    a.x = x; a.dx = dx; a.ws = ws; a.B = B; a.K = K; a.act_in = act_in; a.acc_dx = accumulate_dx;
    a.n = n_entries - s0 < LG_MAX ? n_entries - s0 : LG_MAX;
    a.finalize = s0 + LG_MAX >= n_entries;
    int blk = 0;
    for (int i = 0; i < a.n; ++i) {
      a.e[i] = entries[s0 + i];
      a.blk0[i] = blk;
      blk += (entries[s0 + i].n + LG_ROWS - 1) / LG_ROWS;
    }
    a.blk0[a.n] = blk;
    if (blk == 0) continue;
    any = true;
    if (bwd) linear_group_bwd_kernel<<<blk, 256, 0, st>>>(a);
    else linear_group_fwd_kernel<<<blk, 256, 0, st>>>(a);
  }
  if (bwd && dx && !any) {  // no rows at all: dx gets nothing (still honour accumulate)
    if (!accumulate_dx) zero_f32(dx, (long long)B * K, st);
  }
  return check_launch(bwd ? "linear_group_bwd" : "linear_group_fwd");
}

static const char* lg_validate(const float* x, int B, int K, const DvLinEntry* entries,
                               int n_entries) {
  if (!x || !entries || n_entries < 0) return "null pointer";
  if (B < 1 || B > LG_MAXB || K < 4 || K > LG_MAXK || K % 4 != 0)
    return "need 1 <= B <= 8, K % 4 == 0, K <= 512";
  for (int i = 0; i < n_entries; ++i)
    if (!entries[i].w || !entries[i].y || entries[i].n < 0) return "bad entry";
  return nullptr;
}

extern "C" int dv_linear_group_fwd(const float* x, int B, int K, int act_in, const DvLinEntry* entries,
                                   int n_entries, void* stream) {
  const char* bad = lg_validate(x, B, K, entries, n_entries);
  DV_REQUIRE(!bad, bad ? bad : "");
  return linear_group(false, x, B, K, act_in, entries, n_entries, nullptr, 0, nullptr,
                      (hipStream_t)stream);
}

extern "C" int dv_linear_group_bwd(const float* x, int B, int K, int act_in, const DvLinEntry* entries,
                                   int n_entries, float* dx, int accumulate_dx, float* ws,
                                   void* stream) {
  const char* bad = lg_validate(x, B, K, entries, n_entries);
  DV_REQUIRE(!bad, bad ? bad : "");
  DV_REQUIRE(!dx || ws, "backward dx needs ws");
  return linear_group(true, x, B, K, act_in, entries, n_entries, dx, accumulate_dx, ws,
                      (hipStream_t)stream);
}
