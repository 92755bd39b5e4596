// CrossEmbedLayer3D (reference dalle2_video.py:208-244): the Unet3D input
// layer, parallel (1,k,k) convolutions of the 3-channel (6 with the lowres
// conditioning) input for k = 3, 7, 15 whose outputs are concatenated along
// channels (dim/2, dim/4, rest).  Direct kernels on MFMA for that shape —
// small cin, large windows — instead of one padded 15x15 implicit GEMM:
//
//  * K is ordered (dy, dx, c) with the pixel's channels padded to CP = 4 (or
//    8) only, so one image row of the LDS input window, flattened as
//    [column][CP], IS the im2col row of a pixel for one dy: operand reads are
//    plain 8-element runs at (pixel + dx0) * CP + j.
//  * Output channels go in tiles of 16 (v_mfma_f32_16x16x32_bf16); a tile
//    runs only its own window (the largest kernel among its channels), so the
//    3x3 channels do 3 dy rows of one 32-wide K step and the 15x15 ones 15
//    rows of two.  Executed / algorithmic MACs: 1.46 (CP 4) for 3/7/15.
//  * Weight gradient: M = 16 channels, N = 16 (dx, c) columns, K = 32 pixels
//    of one image row; both operands come from LDS by transposed reads
//    (ds_read_b64_tr_b16) — the im2col "rows" of consecutive pixels overlap
//    in the window image.  Each workgroup sums a band of image rows into its
//    own partial (plain stores); one finishing launch sums the bands and
//    scatters them into the torch-layout gradients of every branch.
#include "dv_common.h"

#include <algorithm>
#include <cstdlib>

using namespace dv;

namespace {

constexpr int XE_MAXT = 8;  // 16-channel tiles (total cout <= 128)

struct XeGeom {
  int ntiles, cout, cin, cp, kmax, nbranch;
  int cpad;           // 16 * ntiles: cout padded to whole tiles (zero weights / bias)
  int k[XE_MAXT];     // window of tile t (largest branch kernel among its channels)
  int jw[XE_MAXT];    // forward K per dy: k*cp rounded up to 32
  int jwp[XE_MAXT];   // LDS / image row pitch (elements) = jw + 8
  int woff[XE_MAXT];  // element offset of tile t's [16][k][jwp] weight image
  int boff;           // element offset of the f32 bias [cout] (16-B aligned)
  int image_elems;    // bf16 elements incl. the bias (multiple of 8)
  int nb16[XE_MAXT];  // wgrad 16-column blocks per dy: ceil(k*cp / 16)
  int poff[XE_MAXT];  // float offset of tile t's partial [16][k][nb16*16]
  int pfloats;        // floats per partial incl. the bias sums
  int items;          // sum over tiles of k * nb16 (16x16 wgrad accumulators)
  int bk[4], bco0[4], bcout[4];  // branches: kernel, first channel, channels
};

// fwd_only: also cin 9..16 (CP = 16; the weight-gradient kernel stages CP <= 8)
bool xe_geom(const DvCrossEmbed& ce, XeGeom& g, bool fwd_only = false) {
  if (ce.nbranch < 1 || ce.nbranch > 4 || ce.cin < 1 || ce.cin > (fwd_only ? 16 : 8)) return false;
  g = XeGeom{};
  g.nbranch = ce.nbranch;
  g.cin = ce.cin;
  g.cp = ce.cin <= 4 ? 4 : ce.cin <= 8 ? 8 : 16;
  int co = 0, kmax = 0;
  for (int b = 0; b < ce.nbranch; ++b) {
    if (ce.k[b] < 1 || ce.k[b] % 2 == 0 || ce.k[b] > 15 || ce.cout[b] < 1) return false;
    if (b && ce.k[b] < ce.k[b - 1]) return false;
    g.bk[b] = ce.k[b];
    g.bco0[b] = co;
    g.bcout[b] = ce.cout[b];
    co += ce.cout[b];
    kmax = std::max(kmax, ce.k[b]);
  }
  if (co % 8 || co > 16 * XE_MAXT) return false;
  g.cout = co;
  g.kmax = kmax;
  g.ntiles = (co + 15) / 16;
  g.cpad = 16 * g.ntiles;
  int woff = 0, poff = 0;
  for (int t = 0; t < g.ntiles; ++t) {
    int k = 0;
    for (int b = 0; b < ce.nbranch; ++b)
      if (g.bco0[b] < 16 * t + 16 && g.bco0[b] + g.bcout[b] > 16 * t) k = std::max(k, g.bk[b]);
    g.k[t] = k;
    g.jw[t] = (k * g.cp + 31) / 32 * 32;
    g.jwp[t] = g.jw[t] + 8;
    g.woff[t] = woff;
    woff += 16 * k * g.jwp[t];
    g.nb16[t] = (k * g.cp + 15) / 16;
    g.poff[t] = poff;
    poff += 16 * k * g.nb16[t] * 16;
    g.items += k * g.nb16[t];
  }
  g.boff = (woff + 7) / 8 * 8;
  g.image_elems = g.boff + 2 * g.cpad;  // f32 bias [cpad]: stays a multiple of 8
  g.pfloats = poff + g.cpad;
  return true;
}

__device__ __forceinline__ f32x4 mma16(u32x4 a, u32x4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

__device__ __forceinline__ s16x4 tr_read(const char* lds_addr) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(lds_addr));
}

__device__ __forceinline__ u32x4 tr_pair(const char* lo, const char* hi) {
  const u32x2 l2 = __builtin_bit_cast(u32x2, tr_read(lo)), h2 = __builtin_bit_cast(u32x2, tr_read(hi));
  return u32x4{l2[0], l2[1], h2[0], h2[1]};
}

// 8 consecutive bf16 at an 8-B aligned LDS address (two b64 reads)
__device__ __forceinline__ u32x4 lds8(const bf16* p) {
  const u32x2 a = *(const u32x2*)p, b = *(const u32x2*)(p + 4);
  return u32x4{a[0], a[1], b[0], b[1]};
}

__device__ __forceinline__ int branch_of(const XeGeom& g, int co) {
  int b = 0;
  while (b + 1 < g.nbranch && co >= g.bco0[b + 1]) ++b;
  return b;
}

// ---------------------------------------------------------------------------
// weight image: tile t: [16 co][k_t dy][jwp_t] bf16 with j = dx * cp + c,
// every tap outside the channel's own (centred) window, c >= cin and
// j >= k_t * cp zero; then the concatenated f32 bias.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void xe_pack_kernel(DvCrossEmbed ce, XeGeom g, bf16* img) {
  for (int i = blockIdx.x * 256 + threadIdx.x; i < g.boff + g.cpad; i += gridDim.x * 256) {
    if (i >= g.boff) {
      const int co = i - g.boff, b = branch_of(g, co);
      ((float*)(img + g.boff))[co] = co < g.cout && ce.b[b] ? ce.b[b][co - g.bco0[b]] : 0.f;
      continue;
    }
    int t = 0;
    while (t + 1 < g.ntiles && i >= g.woff[t + 1]) ++t;
    const int k = g.k[t], jwp = g.jwp[t];
    const int local = i - g.woff[t];
    float v = 0.f;
    if (local < 16 * k * jwp) {
      const int col = local / (k * jwp), rem = local - col * k * jwp;
      const int dy = rem / jwp, j = rem - dy * jwp;
      const int co = 16 * t + col, b = branch_of(g, co);
      const int kb = g.bk[b], o = (k - kb) / 2;
      const int dx = j / g.cp, c = j - dx * g.cp;
      const int ky = dy - o, kx = dx - o;
      if (co < g.cout && j < k * g.cp && c < g.cin && (unsigned)ky < (unsigned)kb &&
          (unsigned)kx < (unsigned)kb)
        v = ce.w[b][(((long long)(co - g.bco0[b]) * g.cin + c) * kb + ky) * kb + kx];
    }
    img[i] = (bf16)v;
  }
}

// ---------------------------------------------------------------------------
// forward: a workgroup = R output rows x WB columns of one frame, all output
// channels.  LDS: the weight image + the (R + kmax - 1) x (WB + kmax + 7)
// input window [col][CP].  A wave job = 32 pixels of one row (two 16-pixel
// MFMA columns sharing each weight fragment), every tile in turn.
// D[co][px]: lane holds pixel (l & 15), channels 4 (l >> 4) .. +3 -> one
// 8-byte store per lane per tile and pixel block.
// ---------------------------------------------------------------------------
// rows per forward workgroup (the tile knobs measured flat within +-5 %,
// profiles/r02_u_unet2_knob_sweep.txt)
int xe_r() { return 8; }

template <int CP>
__global__ __launch_bounds__(512) void xe_fwd_kernel(XeGeom g, const bf16* img, const bf16* x,
                                                     int ldx, const bf16* x1, int ld1, int c0,
                                                     const bf16* res, int ldres, bf16* y, int ldy,
                                                     int H, int W, int WB, int XE_R) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cgs = W / WB, rgs = (H + XE_R - 1) / XE_R;
  int bid = blockIdx.x;
  const int cg = bid % cgs;
  bid /= cgs;
  const int rg = bid % rgs, f = bid / rgs;
  const int y0 = rg * XE_R, x0 = cg * WB, half = g.kmax / 2;
  const int XR = XE_R + g.kmax - 1, XC = WB + g.kmax + 7;
  bf16* sW = (bf16*)smem;
  bf16* sX = sW + g.image_elems;

  // window staging: XS pixels per thread, every global load issued before any
  // LDS store (one memory round trip per workgroup, not one per pixel slot)
  constexpr int XS = 4, NJ = CP == 4 ? 1 : CP / 8;
  const int npx = XR * XC;
  u32x4 wreg = {};
  const bool wld = tid < g.image_elems / 8;
  if (wld) wreg = ((const u32x4*)img)[tid];
  u32x4 xv[XS][NJ];
#pragma unroll
  for (int s = 0; s < XS; ++s) {
    const int i = tid + 512 * s;
    const int rr = i / XC, cc = i - rr * XC;
    const int yy = y0 + rr - half, xx = x0 + cc - half;
    const bool in = i < npx && (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W &&
                    cc < WB + g.kmax - 1;
    const long long pix = (long long)(f * H + yy) * W + xx;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      xv[s][j] = u32x4{0u, 0u, 0u, 0u};
      if (CP == 4) {
        if (in) {
          const u32x2 q = *(const u32x2*)(x + pix * ldx);
          xv[s][j] = u32x4{q[0], q[1], 0u, 0u};
        }
      } else if (in && 8 * j < g.cin) {
        // 8-channel chunks: channels [0, c0) of x, [c0, cin) of x1 (c0 % 8 == 0)
        const bf16* src = 8 * j < c0 ? x + pix * ldx + 8 * j : x1 + pix * ld1 + (8 * j - c0);
        xv[s][j] = *(const u32x4*)src;
      }
    }
  }
  if (wld) ((u32x4*)sW)[tid] = wreg;
  for (int i = tid + 512; i < g.image_elems / 8; i += 512) ((u32x4*)sW)[i] = ((const u32x4*)img)[i];
#pragma unroll
  for (int s = 0; s < XS; ++s) {
    const int i = tid + 512 * s;
    if (i >= npx) break;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      bf16x8 e = __builtin_bit_cast(bf16x8, xv[s][j]);
      const int cl = CP == 4 ? 4 : 8;
#pragma unroll
      for (int c = 0; c < 8; ++c)
        if (c >= cl || 8 * j + c >= g.cin) e[c] = (bf16)0.f;
      if (CP == 4) {
        *(bf16x4*)(sX + (long long)i * 4) = bf16x4{e[0], e[1], e[2], e[3]};
      } else {
        *(bf16x8*)(sX + (long long)i * CP + 8 * j) = e;
      }
    }
  }
  for (int i = tid + 512 * XS; i < npx; i += 512) {  // windows beyond XS slots (wide kmax)
    const int rr = i / XC, cc = i - rr * XC;
    const int yy = y0 + rr - half, xx = x0 + cc - half;
    const bool in = (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W && cc < WB + g.kmax - 1;
    const long long pix = (long long)(f * H + yy) * W + xx;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      bf16x8 e = {};
      if (CP == 4) {
        if (in) {
          const bf16x4 q = __builtin_bit_cast(bf16x4, *(const u32x2*)(x + pix * ldx));
#pragma unroll
          for (int c = 0; c < 4; ++c) e[c] = c < g.cin ? q[c] : (bf16)0.f;
        }
        *(bf16x4*)(sX + (long long)i * 4) = bf16x4{e[0], e[1], e[2], e[3]};
      } else {
        if (in && 8 * j < g.cin) {
          const bf16* src = 8 * j < c0 ? x + pix * ldx + 8 * j : x1 + pix * ld1 + (8 * j - c0);
          e = __builtin_bit_cast(bf16x8, *(const u32x4*)src);
#pragma unroll
          for (int c = 0; c < 8; ++c)
            if (8 * j + c >= g.cin) e[c] = (bf16)0.f;
        }
        *(bf16x8*)(sX + (long long)i * CP + 8 * j) = e;
      }
    }
  }
  __syncthreads();

  const float* sb = (const float*)(sW + g.boff);
  const int jobs_per_row = WB / 32;
  const int px = lane & 15, kg = lane >> 4;
  for (int job = wave; job < XE_R * jobs_per_row; job += 8) {
    const int r = job / jobs_per_row, xb = (job - r * jobs_per_row) * 32;
    if (y0 + r >= H) break;
    const long long p = (long long)(f * H + y0 + r) * W + x0 + xb + px;
    for (int t = 0; t < g.ntiles; ++t) {
      const int k = g.k[t], jw = g.jw[t], jwp = g.jwp[t];
      const int cofs = half - k / 2;  // the tile's window inside the kmax halo
      const bf16* wt = sW + g.woff[t] + px * k * jwp + 8 * kg;
      f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
      for (int dy = 0; dy < k; ++dy) {
        const bf16* xr = sX + ((long long)(r + cofs + dy) * XC + xb + px + cofs) * CP + 8 * kg;
        const bf16* wr = wt + dy * jwp;
        for (int ks = 0; ks < jw; ks += 32) {
          const u32x4 wf = *(const u32x4*)(wr + ks);
          a0 = mma16(wf, lds8(xr + ks), a0);
          a1 = mma16(wf, lds8(xr + 16 * CP + ks), a1);
        }
      }
      const int co = 16 * t + 4 * kg;
      if (co >= g.cout) continue;  // padded channels of the last tile
      float r0[4] = {0.f, 0.f, 0.f, 0.f}, r1[4] = {0.f, 0.f, 0.f, 0.f};
      if (res) {
        const bf16x4 q0 = *(const bf16x4*)(res + p * ldres + co);
        const bf16x4 q1 = *(const bf16x4*)(res + (p + 16) * ldres + co);
#pragma unroll
        for (int e = 0; e < 4; ++e) { r0[e] = (float)q0[e]; r1[e] = (float)q1[e]; }
      }
      bf16x4 o0, o1;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        o0[e] = (bf16)(a0[e] + sb[co + e] + r0[e]);
        o1[e] = (bf16)(a1[e] + sb[co + e] + r1[e]);
      }
      *(bf16x4*)(y + p * ldy + co) = o0;
      *(bf16x4*)(y + (p + 16) * ldy + co) = o1;
    }
  }
}

// ---------------------------------------------------------------------------
// weight gradient.  Workgroup = a band of `rows` image rows of one frame,
// walked RB rows per step: LDS dY rows [RB][W][cout + 8] and the kmax + RB - 1
// input rows around them [kmax + RB - 1][W + kmax + 7][CP] (double-buffered:
// the next step's global loads are in registers while this step's MFMAs run).
// Wave w owns accumulator items [w * per, w * per + per) of the flat (tile,
// dy, 16-column block) list.  (Round 6: one row per step left each step's
// global loads exposed -- ~640 MFMA cycles per SIMD against a load round trip
// -- and re-read the kmax window rows for every output row: 65 us for the
// Cfg2 cross-embed, 0.06 of HBM.  RB = 4 rows per step amortises the latency
// and reads (kmax + 3) / 4 window rows per output row instead of kmax.)
// ---------------------------------------------------------------------------
template <int CP, int MAXI, int RB>
__global__ __launch_bounds__(512) void xe_wgrad_kernel(XeGeom g, const bf16* dy, int lddy,
                                                       const bf16* x, int ldx, float* part, int H,
                                                       int W, int rows, int per) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int bands = (H + rows - 1) / rows;
  const int f = blockIdx.x / bands, yb = (blockIdx.x % bands) * rows;
  const int yend = min(yb + rows, H);
  const int half = g.kmax / 2, XC = W + g.kmax + 7, XR = g.kmax + RB - 1;
  const int DS = g.cpad + 8;                      // dY row pitch (elements)
  const int DYB = RB * W * DS, XB = XR * XC * CP;  // buffer sizes (elements)
  bf16* sD = (bf16*)smem;                         // [2][RB][W][DS]
  bf16* sX = sD + 2 * DYB;                        // [2][XR][XC][CP]

  // ---- this wave's items: tile, LDS offsets ----
  int it_t[MAXI], it_boff[MAXI];
  const int i0 = wave * per;
#pragma unroll
  for (int i = 0; i < MAXI; ++i) {
    int idx = i0 + i, t = 0;
    it_t[i] = -1;
    it_boff[i] = 0;
    if (i >= per || idx >= g.items) continue;
    while (idx >= g.k[t] * g.nb16[t]) {
      idx -= g.k[t] * g.nb16[t];
      ++t;
    }
    const int d = idx / g.nb16[t], nb = idx - d * g.nb16[t];
    const int cofs = half - g.k[t] / 2;
    it_t[i] = t;
    it_boff[i] = ((d + cofs) * XC + cofs) * CP + 16 * nb;  // element offset (pixel 0, step row 0)
  }

  int t_lo = XE_MAXT, t_hi = -1;
#pragma unroll
  for (int i = 0; i < MAXI; ++i)
    if (it_t[i] >= 0) {
      t_lo = min(t_lo, it_t[i]);
      t_hi = max(t_hi, it_t[i]);
    }

  f32x4 acc[MAXI];
#pragma unroll
  for (int i = 0; i < MAXI; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float accb = 0.f;  // bias: waves < ntiles own tile `wave`

  // ---- staging: global -> registers (next step) -> LDS ----
  const int cch = g.cout / 8;                 // 16-B dY chunks per pixel
  const int dchunks = RB * W * cch;           // per step
  const int xelems = XR * XC;                 // window pixels per step
  constexpr int DPT = 4, XPT = 9;             // per-thread register slots (checked by the host)
  // a window pixel is CP bf16 = one 8- or 16-B vector: loaded, channel-masked
  // (c >= cin zero) and written to LDS whole (round 5 moved it element by
  // element: 8 ds_write_b16 per pixel)
  typedef typename std::conditional<CP == 8, u32x4, u32x2>::type XV;
  constexpr int XW = CP / 2;  // dwords per pixel
  u32x4 dreg[DPT];
  XV xreg[XPT];
  XV cmask;
#pragma unroll
  for (int j = 0; j < XW; ++j)
    cmask[j] = (2 * j < g.cin ? 0x0000ffffu : 0u) | (2 * j + 1 < g.cin ? 0xffff0000u : 0u);
  auto load_step = [&](int y0) {
#pragma unroll
    for (int s = 0; s < DPT; ++s) {
      const int i = tid + 512 * s;
      dreg[s] = u32x4{0u, 0u, 0u, 0u};
      if (i < dchunks) {
        const int rp = i / cch, c8 = i - rp * cch, r = rp / W, p = rp - r * W;
        if (y0 + r < yend)  // rows of the next band stay zero: they add nothing
          dreg[s] = *(const u32x4*)(dy + ((long long)(f * H + y0 + r) * W + p) * lddy + 8 * c8);
      }
    }
#pragma unroll
    for (int s = 0; s < XPT; ++s) {
      const int i = tid + 512 * s;
#pragma unroll
      for (int j = 0; j < XW; ++j) xreg[s][j] = 0u;
      if (i < xelems) {
        const int rr = i / XC, cc = i - rr * XC;
        const int sy = y0 + rr - half, sx = cc - half;
        if ((unsigned)sy < (unsigned)H && (unsigned)sx < (unsigned)W)
          xreg[s] = *(const XV*)(x + ((long long)(f * H + sy) * W + sx) * ldx) & cmask;
      }
    }
  };
  auto store_step = [&](int buf) {
    bf16* d = sD + buf * DYB;
#pragma unroll
    for (int s = 0; s < DPT; ++s) {
      const int i = tid + 512 * s;
      if (i < dchunks) {
        const int rp = i / cch, c8 = i - rp * cch;
        *(u32x4*)(d + rp * DS + 8 * c8) = dreg[s];
      }
    }
    bf16* xs = sX + buf * XB;
#pragma unroll
    for (int s = 0; s < XPT; ++s) {
      const int i = tid + 512 * s;
      if (i < xelems) *(XV*)(xs + i * CP) = xreg[s];
    }
  };

  // lane parts of the transposed reads: 16-lane group kg reads pixel rows
  // 8 kg + q (lo) and 8 kg + 4 + q (hi), 8-B chunk pp of a 32-B row
  const int kg = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  const int plo = 8 * kg + q;

  if (g.cpad != g.cout) {  // channels [cout, cpad) of both dY buffers stay zero
    for (int i = tid; i < 2 * RB * W; i += 512)
      for (int c = g.cout; c < g.cpad; c += 8) *(u32x4*)(sD + i * DS + c) = u32x4{0u, 0u, 0u, 0u};
    __syncthreads();
  }
  if (yb < yend) {
    load_step(yb);
    store_step(0);
  }
  __syncthreads();
  for (int y0 = yb; y0 < yend; y0 += RB) {
    const int buf = ((y0 - yb) / RB) & 1;
    const bool more = y0 + RB < yend;
    if (more) load_step(y0 + RB);
    const int nr = min(RB, yend - y0);
    for (int r = 0; r < nr; ++r) {
      const char* d = (const char*)(sD + buf * DYB + r * W * DS);
      const char* xs = (const char*)(sX + buf * XB + r * XC * CP);
      for (int p0 = 0; p0 < W; p0 += 32) {
        const char* arow = d + ((p0 + plo) * DS + 4 * pp) * 2;
        if (wave < g.ntiles) {  // bias: the dY^T fragment of tile `wave` summed on the VALU
          const char* a = arow + 32 * wave;
          const bf16x8 e = __builtin_bit_cast(bf16x8, tr_pair(a, a + 4 * DS * 2));
#pragma unroll
          for (int j = 0; j < 8; ++j) accb += (float)e[j];
        }
        const int lanex = ((p0 + plo) * CP + 4 * pp) * 2;
        // items are ordered by tile: one dY^T fragment per tile this wave touches
        for (int t = t_lo; t <= t_hi; ++t) {
          const char* a = arow + 32 * t;
          const u32x4 fa = tr_pair(a, a + 4 * DS * 2);
#pragma unroll
          for (int i = 0; i < MAXI; ++i) {
            if (it_t[i] != t) continue;
            const char* b = xs + it_boff[i] * 2 + lanex;
            acc[i] = mma16(fa, tr_pair(b, b + 4 * CP * 2), acc[i]);
          }
        }
      }
    }
    if (more) {
      store_step(buf ^ 1);
    }
    __syncthreads();
  }

  // ---- partial of this band: D[co][n]: lane n = l & 15, co = 4 kg + e ----
  float* pp_ = part + (long long)blockIdx.x * g.pfloats;
#pragma unroll
  for (int i = 0; i < MAXI; ++i) {
    if (it_t[i] < 0) continue;
    int idx = i0 + i, t = 0;
    while (idx >= g.k[t] * g.nb16[t]) {
      idx -= g.k[t] * g.nb16[t];
      ++t;
    }
    const int d = idx / g.nb16[t], nb = idx - d * g.nb16[t];
    const int row = g.nb16[t] * 16;
#pragma unroll
    for (int e = 0; e < 4; ++e)
      pp_[g.poff[t] + ((4 * kg + e) * g.k[t] + d) * row + 16 * nb + (lane & 15)] = acc[i][e];
  }
  if (wave < g.ntiles) {
    accb += __shfl_xor(accb, 16, 64);
    accb += __shfl_xor(accb, 32, 64);
    if (lane < 16) pp_[g.pfloats - g.cpad + 16 * wave + lane] = accb;
  }
}

// sum the bands and scatter into every branch's torch-layout gradient:
// 32 outputs x 8 split groups per workgroup, 8 loads in flight per lane
__global__ __launch_bounds__(256) void xe_wgrad_finish_kernel(DvCrossEmbed ce, XeGeom g,
                                                              const float* part, int S,
                                                              long long total) {
  __shared__ float sh[8][32];
  const int ol = threadIdx.x & 31, grp = threadIdx.x >> 5;
  const long long o = (long long)blockIdx.x * 32 + ol;
  int src = -1, b = 0;
  long long local = o;
  float* dst = nullptr;
  int acc = 0;
  if (o < total) {
    for (b = 0; b < g.nbranch; ++b) {
      const long long nw = (long long)g.bcout[b] * g.cin * g.bk[b] * g.bk[b];
      if (local < nw) {
        const int kb = g.bk[b];
        const int kx = (int)(local % kb), ky = (int)(local / kb % kb);
        const int c = (int)(local / (kb * kb) % g.cin), col = (int)(local / ((long long)kb * kb * g.cin));
        const int co = g.bco0[b] + col, t = co / 16, k = g.k[t], o2 = (k - kb) / 2;
        src = g.poff[t] + ((co % 16) * k + ky + o2) * g.nb16[t] * 16 + (kx + o2) * g.cp + c;
        dst = ce.dw[b] + local;
        acc = ce.accumulate_w;
        break;
      }
      local -= nw;
      if (local < g.bcout[b]) {
        src = g.pfloats - g.cpad + g.bco0[b] + (int)local;
        dst = ce.db[b] ? ce.db[b] + local : nullptr;
        acc = ce.accumulate_b;
        break;
      }
      local -= g.bcout[b];
    }
  }
  float v = 0.f;
  if (src >= 0) {
    const float* p = part + src;
    const long long st = g.pfloats;
    int s = grp;
    for (; s + 56 < S; s += 64) {
      float t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) t[u] = p[(long long)(s + 8 * u) * st];
      v += ((t[0] + t[1]) + (t[2] + t[3])) + ((t[4] + t[5]) + (t[6] + t[7]));
    }
    for (; s < S; s += 8) v += p[(long long)s * st];
  }
  sh[grp][ol] = v;
  __syncthreads();
  if (grp != 0 || !dst) return;
  v = ((sh[0][ol] + sh[1][ol]) + (sh[2][ol] + sh[3][ol])) + ((sh[4][ol] + sh[5][ol]) + (sh[6][ol] + sh[7][ol]));
  *dst = acc ? *dst + v : v;
}

long long xe_total_grads(const XeGeom& g) {
  long long n = 0;
  for (int b = 0; b < g.nbranch; ++b) n += (long long)g.bcout[b] * (g.cin * g.bk[b] * g.bk[b] + 1);
  return n;
}

int xe_fwd_wb(int w) {
  return w % 64 == 0 ? 64 : 32;
}

size_t xe_fwd_lds(const XeGeom& g, int w) {
  const int WB = xe_fwd_wb(w);
  return (size_t)g.image_elems * 2 + (size_t)(xe_r() + g.kmax - 1) * (WB + g.kmax + 7) * g.cp * 2;
}

constexpr int XE_RB = 4;  // wgrad: image rows per staging step (8 where they fit, 1 where 4 do not)

size_t xe_wgrad_lds(const XeGeom& g, int w, int rb) {
  return (size_t)2 * rb * w * (g.cpad + 8) * 2 + (size_t)2 * (g.kmax + rb - 1) * (w + g.kmax + 7) * g.cp * 2;
}

// the register staging slots (DPT = 4 dY chunks, XPT = 9 window pixels per
// thread) and the LDS hold rb rows per step
bool xe_wgrad_fits(const XeGeom& g, int w, int rb) {
  return (long long)rb * w * (g.cout / 8) <= 4 * 512 && (long long)(g.kmax + rb - 1) * (w + g.kmax + 7) <= 9 * 512 &&
         xe_wgrad_lds(g, w, rb) <= 160 * 1024;
}

int xe_rows(int nf, int h) {
  // ~256 bands (one 512-thread workgroup per CU)
  long long want = (long long)nf * h / 256;
  int rows = (int)std::max(1ll, want);
  return std::min(rows, h);
}

bool xe_shape_ok(const XeGeom& g, int nf, int h, int w, int ldx) {
  if (nf < 1 || h < 1 || w < 32 || w % 32 || ldx % std::min(g.cp, 8) || ldx < std::min(g.cin, 8))
    return false;
  if ((long long)nf * h * w * std::max(ldx, g.cout) >= (1ll << 31)) return false;
  return true;
}

template <typename F>
void xe_allow_lds(F* fn) {
  (void)hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

}  // namespace

extern "C" int dv_cross_embed_image_elems(const DvCrossEmbed* ce, long long* elems) {
  DV_REQUIRE(ce && elems, "null pointer");
  XeGeom g;
  DV_REQUIRE(xe_geom(*ce, g), "unsupported branch set (1..4 odd k <= 15 ascending, cin <= 8, "
                              "sum(cout) % 16 == 0, <= 128)");
  *elems = g.image_elems;
  return DV_OK;
}

extern "C" int dv_cross_embed_pack(const DvCrossEmbed* ce, void* image, void* stream) {
  DV_REQUIRE(ce && image, "null pointer");
  XeGeom g;
  DV_REQUIRE(xe_geom(*ce, g), "unsupported branch set");
  for (int b = 0; b < g.nbranch; ++b) DV_REQUIRE(ce->w[b], "null weight");
  const int blocks = std::min(1024, (g.boff + g.cout + 255) / 256);
  xe_pack_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(*ce, g, (bf16*)image);
  return check_launch("cross_embed_pack");
}

namespace {
int xe_fwd_launch(const XeGeom& g, const void* image, const void* x, int ldx, const void* x1, int ld1,
                  int c0, const void* res, int ldres, void* y, int ldy, int nf, int h, int w,
                  hipStream_t st) {
  const size_t lds = xe_fwd_lds(g, w);
  DV_REQUIRE(lds <= 160 * 1024, "LDS footprint too large");
  const int WB = xe_fwd_wb(w);
  const int R = xe_r();
  const long long blocks = (long long)nf * ((h + R - 1) / R) * (w / WB);
  static bool once = (xe_allow_lds(xe_fwd_kernel<4>), xe_allow_lds(xe_fwd_kernel<8>),
                      xe_allow_lds(xe_fwd_kernel<16>), true);
  (void)once;
#define XE_FW(CP)                                                                                \
  xe_fwd_kernel<CP><<<(unsigned)blocks, 512, lds, st>>>(g, (const bf16*)image, (const bf16*)x, ldx, \
                                                        (const bf16*)x1, ld1, c0, (const bf16*)res, \
                                                        ldres, (bf16*)y, ldy, h, w, WB, R)
  if (g.cp == 4) XE_FW(4);
  else if (g.cp == 8) XE_FW(8);
  else XE_FW(16);
#undef XE_FW
  return DV_OK;
}

DvCrossEmbed small_desc(const float* wt, const float* b, int cin, int cout, int ksize) {
  DvCrossEmbed ce{};
  ce.nbranch = 1;
  ce.cin = cin;
  ce.k[0] = ksize;
  ce.cout[0] = cout;
  ce.w[0] = wt;
  ce.b[0] = b;
  return ce;
}
}  // namespace

extern "C" int dv_cross_embed_fwd(const DvCrossEmbed* ce, const void* image, const void* x,
                                  int ldx, void* y, int ldy, int nf, int h, int w, void* stream) {
  DV_REQUIRE(ce && image && x && y, "null pointer");
  XeGeom g;
  DV_REQUIRE(xe_geom(*ce, g), "unsupported branch set");
  DV_REQUIRE(xe_shape_ok(g, nf, h, w, ldx) && ldx >= g.cin && ldy % 4 == 0 && ldy >= g.cout,
             "needs w % 32 == 0, ldx % (4 or 8) == 0, ldy % 4 == 0");
  const int rc = xe_fwd_launch(g, image, x, ldx, nullptr, 0, g.cin, nullptr, 0, y, ldy, nf, h, w,
                               (hipStream_t)stream);
  if (rc != DV_OK) return rc;
  return check_launch("cross_embed_fwd");
}

extern "C" int dv_conv_small_image_elems(int cin, int cout, int ksize, long long* elems) {
  DV_REQUIRE(elems, "null pointer");
  XeGeom g;
  DV_REQUIRE(xe_geom(small_desc(nullptr, nullptr, cin, cout, ksize), g, true),
             "unsupported shape (cin <= 16, cout % 8 == 0 <= 128, odd k <= 15)");
  *elems = g.image_elems;
  return DV_OK;
}

extern "C" int dv_conv_small_pack(const float* wt, const float* bias, int cin, int cout, int ksize,
                                  void* image, void* stream) {
  DV_REQUIRE(wt && image, "null pointer");
  const DvCrossEmbed ce = small_desc(wt, bias, cin, cout, ksize);
  XeGeom g;
  DV_REQUIRE(xe_geom(ce, g, true), "unsupported shape");
  const int blocks = std::min(1024, (g.boff + g.cpad + 255) / 256);
  xe_pack_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(ce, g, (bf16*)image);
  return check_launch("conv_small_pack");
}

namespace {
struct XeSmallPack {
  DvCrossEmbed ce;
  XeGeom g;
  bf16* img;
  int mode, wcin;  // DvSmallPackEntry
};
// entry blockIdx.y: the xe_pack_kernel loop over that entry's image
__global__ __launch_bounds__(256) void xe_pack_batched_kernel(const XeSmallPack* t) {
  const XeSmallPack& e = t[blockIdx.y];
  const DvCrossEmbed& ce = e.ce;
  const XeGeom& g = e.g;
  bf16* img = e.img;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < g.boff + g.cpad; i += gridDim.x * 256) {
    if (i >= g.boff) {
      const int co = i - g.boff;
      ((float*)(img + g.boff))[co] = co < g.cout && ce.b[0] ? ce.b[0][co] : 0.f;
      continue;
    }
    int tt = 0;
    while (tt + 1 < g.ntiles && i >= g.woff[tt + 1]) ++tt;
    const int k = g.k[tt], jwp = g.jwp[tt];
    const int local = i - g.woff[tt];
    float v = 0.f;
    if (local < 16 * k * jwp) {
      const int col = local / (k * jwp), rem = local - col * k * jwp;
      const int dy = rem / jwp, j = rem - dy * jwp;
      const int co = 16 * tt + col;
      const int dx = j / g.cp, c = j - dx * g.cp;
      if (co < g.cout && j < k * g.cp && c < g.cin && dx < k) {
        if (e.mode == 0) v = ce.w[0][(((long long)co * g.cin + c) * k + dy) * k + dx];
        else if (co < e.wcin)  // dgrad image: w[c][co][k-1-dy][k-1-dx] of the (cin_img, wcin) weight
          v = ce.w[0][(((long long)c * e.wcin + co) * k + (k - 1 - dy)) * k + (k - 1 - dx)];
      }
    }
    img[i] = (bf16)v;
  }
}
}  // namespace

extern "C" int dv_conv_small_pack_plan(const DvSmallPackEntry* entries, int n, void* table, long long* bytes,
                                       long long* max_elems) {
  DV_REQUIRE(entries && bytes && max_elems && n > 0, "null pointer / empty");
  *bytes = (long long)n * sizeof(XeSmallPack);
  long long mx = 0;
  for (int i = 0; i < n; ++i) {
    const DvSmallPackEntry& e = entries[i];
    DV_REQUIRE(e.w && e.image, "null weight / image");
    XeSmallPack t{};
    t.ce = small_desc(e.w, e.bias, e.cin, e.cout, e.ksize);
    DV_REQUIRE(xe_geom(t.ce, t.g, true), "unsupported shape");
    t.img = (bf16*)e.image;
    DV_REQUIRE(e.mode == 0 || (e.mode == 1 && e.wcin > 0 && e.wcin <= e.cout && !e.bias),
               "mode 1 (dgrad image) needs 0 < wcin <= cout and no bias");
    t.mode = e.mode;
    t.wcin = e.wcin;
    mx = std::max(mx, (long long)(t.g.boff + t.g.cpad));
    if (table) ((XeSmallPack*)table)[i] = t;
  }
  *max_elems = mx;
  return DV_OK;
}

extern "C" int dv_conv_small_pack_batched(const void* table, int n, long long max_elems, void* stream) {
  DV_REQUIRE(table && n > 0 && n <= 65535 && max_elems > 0, "bad table");
  const int blocks = (int)std::min<long long>(64, (max_elems + 255) / 256);
  xe_pack_batched_kernel<<<dim3(blocks, n), 256, 0, (hipStream_t)stream>>>((const XeSmallPack*)table);
  return check_launch("conv_small_pack_batched");
}

extern "C" int dv_conv_small_fwd(const void* x0, int ld0, int c0, const void* x1, int ld1,
                                 const void* image, const void* res, int ldres, void* y, int ldy,
                                 int nf, int h, int w, int cin, int cout, int ksize, void* stream) {
  DV_REQUIRE(x0 && image && y, "null pointer");
  XeGeom g;
  DV_REQUIRE(xe_geom(small_desc(nullptr, nullptr, cin, cout, ksize), g, true),
             "unsupported shape (cin <= 16, cout % 8 == 0 <= 128, odd k <= 15)");
  const bool two = x1 != nullptr;
  DV_REQUIRE(!two || (g.cp >= 8 && c0 % 8 == 0 && c0 > 0 && c0 < cin && ld1 % 8 == 0 && ld1 >= cin - c0),
             "second input needs c0 % 8 == 0 and ld1 % 8 == 0");
  const int cx0 = two ? c0 : cin;
  DV_REQUIRE(xe_shape_ok(g, nf, h, w, ld0) && ld0 >= cx0 && (g.cp == 4 || ld0 % 8 == 0),
             "needs w % 32 == 0 and 16-B aligned pixel rows");
  DV_REQUIRE(ldy % 4 == 0 && ldy >= cout && (!res || (ldres % 4 == 0 && ldres >= cout)),
             "ldy / ldres must be multiples of 4");
  DV_REQUIRE((long long)nf * h * w * std::max({ld0, ld1, ldy, ldres}) < (1ll << 31), "tensor too large");
  const int rc = xe_fwd_launch(g, image, x0, ld0, x1, ld1, cx0, res, ldres, y, ldy, nf, h, w,
                               (hipStream_t)stream);
  if (rc != DV_OK) return rc;
  return check_launch("conv_small_fwd");
}

extern "C" int dv_cross_embed_wgrad_ws(const DvCrossEmbed* ce, int nf, int h, int w,
                                       long long* floats) {
  DV_REQUIRE(ce && floats, "null pointer");
  XeGeom g;
  DV_REQUIRE(xe_geom(*ce, g), "unsupported branch set");
  DV_REQUIRE(nf > 0 && h > 0, "bad sizes");
  const int rows = xe_rows(nf, h);
  *floats = (long long)nf * ((h + rows - 1) / rows) * g.pfloats;
  return DV_OK;
}

extern "C" int dv_cross_embed_wgrad(const DvCrossEmbed* ce, const void* dy, int lddy,
                                    const void* x, int ldx, float* ws, long long ws_floats, int nf,
                                    int h, int w, void* stream) {
  DV_REQUIRE(ce && dy && x && ws, "null pointer");
  XeGeom g;
  DV_REQUIRE(xe_geom(*ce, g), "unsupported branch set");
  for (int b = 0; b < g.nbranch; ++b) DV_REQUIRE(ce->dw[b], "null weight gradient");
  DV_REQUIRE(xe_shape_ok(g, nf, h, w, ldx) && ldx >= g.cin && lddy % 8 == 0 && lddy >= g.cout,
             "needs w % 32 == 0, ldx % (4 or 8) == 0, lddy % 8 == 0");
  long long need = 0;
  dv_cross_embed_wgrad_ws(ce, nf, h, w, &need);
  DV_REQUIRE(ws_floats >= need, "workspace too small (see dv_cross_embed_wgrad_ws)");
  const int rb = xe_wgrad_fits(g, w, 2 * XE_RB) ? 2 * XE_RB : xe_wgrad_fits(g, w, XE_RB) ? XE_RB : 1;
  DV_REQUIRE(xe_wgrad_fits(g, w, rb), "image row too wide for the staging slots / LDS");
  const size_t lds = xe_wgrad_lds(g, w, rb);
  const int per = (g.items + 7) / 8;
  DV_REQUIRE(per <= 24, "too many accumulator tiles");
  const int rows = xe_rows(nf, h);
  const int S = nf * ((h + rows - 1) / rows);
  hipStream_t st = (hipStream_t)stream;
  static bool once = (xe_allow_lds(xe_wgrad_kernel<4, 12, XE_RB>), xe_allow_lds(xe_wgrad_kernel<4, 24, XE_RB>),
                      xe_allow_lds(xe_wgrad_kernel<8, 12, XE_RB>), xe_allow_lds(xe_wgrad_kernel<8, 24, XE_RB>),
                      xe_allow_lds(xe_wgrad_kernel<4, 12, 1>), xe_allow_lds(xe_wgrad_kernel<4, 24, 1>),
                      xe_allow_lds(xe_wgrad_kernel<8, 12, 1>), xe_allow_lds(xe_wgrad_kernel<8, 24, 1>),
                      xe_allow_lds(xe_wgrad_kernel<4, 12, 2 * XE_RB>), xe_allow_lds(xe_wgrad_kernel<4, 24, 2 * XE_RB>),
                      xe_allow_lds(xe_wgrad_kernel<8, 12, 2 * XE_RB>), xe_allow_lds(xe_wgrad_kernel<8, 24, 2 * XE_RB>),
                      true);
  (void)once;
  const bf16* d = (const bf16*)dy;
  const bf16* xx = (const bf16*)x;
#define XE_WG2(CP, MI, RB) \
  xe_wgrad_kernel<CP, MI, RB><<<(unsigned)S, 512, lds, st>>>(g, d, lddy, xx, ldx, ws, h, w, rows, per)
#define XE_WG(CP, MI) \
  (rb == 2 * XE_RB ? XE_WG2(CP, MI, 2 * XE_RB) : rb == XE_RB ? XE_WG2(CP, MI, XE_RB) : XE_WG2(CP, MI, 1))
  if (g.cp == 4) {
    if (per <= 12) XE_WG(4, 12);
    else XE_WG(4, 24);
  } else {
    if (per <= 12) XE_WG(8, 12);
    else XE_WG(8, 24);
  }
#undef XE_WG
#undef XE_WG2
  const long long total = xe_total_grads(g);
  xe_wgrad_finish_kernel<<<(unsigned)((total + 31) / 32), 256, 0, st>>>(*ce, g, ws, S, total);
  return check_launch("cross_embed_wgrad");
}
