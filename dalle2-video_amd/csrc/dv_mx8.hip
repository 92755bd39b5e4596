// MX-fp8 forward convolution for the sampling path (BASELINE config 5: unet1
// sampling on 32-frame 128x128 clips): the Block3D 3x3 convs
// (dalle2_video.py:107) with both operands in OCP MX-fp8 — e4m3 elements with
// one e8m0 power-of-two scale per 32 consecutive input channels — on the
// block-scaled v_mfma_scale_f32_32x32x64_f8f6f4, which runs at twice the bf16
// MFMA rate per clock (MI355X_MICROARCH.md, FP8 row), f32 accumulation, bf16
// output (bias + residual epilogue).
//
// Operand layout, measured on gfx950 (tools/probes/mx8_probe.hip): lane l of
// the 32x32x64 instruction holds row / column l & 31; its 32 bytes are
// K-block 0 elements 16h .. 16h + 15 (bytes 0-15) and K-block 1 elements
// 16h .. 16h + 15 (bytes 16-31), h = l >> 5; lane half h supplies the scale of
// K-block h.  So with a 64-channel chunk per MFMA, lane (r, h) reads the
// 16-B channel slots h and 2 + h of its row and the scale of channels
// [32h, 32h + 32).  v_cvt_pk_fp8_f32 rounds to nearest even and does NOT
// saturate (> 448 -> NaN): the scale exponent keeps every scaled value <= 448.
//
// Activations: dv_mx8_quant turns a bf16 channels-last tensor into q [M][C]
// e4m3 bytes + s [C/64][M] u32 scale pairs (byte h = block h of the chunk);
// weights: dv_mx8_pack_conv_weight builds the kernel's LDS image per
// (64-output-channel block, 64-channel chunk), XOR-swizzled so the fragment
// reads are conflict-free.
#include "dv_common.h"

#include <cstdint>

using namespace dv;

namespace {

typedef int v8i __attribute__((ext_vector_type(8)));
// 4 waves per workgroup (one per SIMD: the kernel needs ~360 registers per lane)
constexpr int MX_NW = 4;

constexpr int MX_WROW = 9 * 64;                      // e4m3 bytes of one packed weight row per chunk
constexpr int MX_WDATA = 64 * MX_WROW;               // 36,864
constexpr int MX_WIMG = MX_WDATA + 64 * 32;          // + per-row scales [h][16]: 38,912 B
constexpr int MX_WPIECES = MX_WIMG / 1024;           // 38 DMA pieces of 64 lanes x 16 B

// mx_exp / mx_inv (the block scale exponent): dv_common.h

// 16 floats (already scaled) -> 16 e4m3 bytes, element i at byte i
__device__ __forceinline__ u32x4 mx_cvt16(const float* v, float inv) {
  u32x4 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    unsigned w = __builtin_amdgcn_cvt_pk_fp8_f32(v[4 * i] * inv, v[4 * i + 1] * inv, 0, false);
    w = __builtin_amdgcn_cvt_pk_fp8_f32(v[4 * i + 2] * inv, v[4 * i + 3] * inv, w, true);
    r[i] = w;
  }
  return r;
}

// two 16-B fragments -> the 32-byte MFMA operand
__device__ __forceinline__ v8i cat8(u32x4 a, u32x4 b) {
  typedef __attribute__((ext_vector_type(8))) unsigned u32x8;
  return __builtin_bit_cast(v8i, (u32x8)__builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
}

__device__ __forceinline__ float amax16(const float* v) {
  float a = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) a = fmaxf(a, fabsf(v[i]));
  return a;
}

// ---------------------------------------------------------------------------
// activations: one thread per (64-channel chunk c, pixel m), c-major so the
// scale stores are contiguous; 128 B read, 64 + 4 B written
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void mx8_quant_kernel(const bf16* __restrict__ x, int ld, int C,
                                                        long long M, uint8_t* __restrict__ q,
                                                        unsigned* __restrict__ s) {
  const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
  const int nch = C / 64;
  if (t >= M * nch) return;
  const int c = (int)(t / M);
  const long long m = t - (long long)c * M;
  const u32x4* src = (const u32x4*)(x + m * ld + c * 64);
  u32x4 raw[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) raw[i] = src[i];
  float v[64];
#pragma unroll
  for (int i = 0; i < 8; ++i) Vec<bf16>::to_f(raw[i], v + 8 * i);
  const int E0 = mx_exp(fmaxf(amax16(v), amax16(v + 16)));
  const int E1 = mx_exp(fmaxf(amax16(v + 32), amax16(v + 48)));
  const float i0 = mx_inv(E0), i1 = mx_inv(E1);
  u32x4* dst = (u32x4*)(q + m * C + c * 64);
  dst[0] = mx_cvt16(v, i0);
  dst[1] = mx_cvt16(v + 16, i0);
  dst[2] = mx_cvt16(v + 32, i1);
  dst[3] = mx_cvt16(v + 48, i1);
  s[(long long)c * M + m] = (unsigned)(E0 + 127) | ((unsigned)(E1 + 127) << 8);
}

// ---------------------------------------------------------------------------
// weights (cout, cin, 1, 3, 3) f32 -> image [cout / 64][cin / 64][MX_WIMG]:
// row r (output channel co0 + r), tap d, 16-B slot t (channels 16t .. 16t+15 of
// the chunk) at r * 576 + (4d + (t ^ ((r >> 2) & 3))) * 16; the row's scales at
// MX_WDATA + r * 32 + 16h + d.  One thread per (output channel, chunk, tap).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void mx8_pack_weight_kernel(const float* __restrict__ w, int cout,
                                                              int cin, uint8_t* __restrict__ img) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  const int nch = cin / 64;
  if (t >= cout * nch * 9) return;
  const int d = t % 9, c = (t / 9) % nch, co = t / (9 * nch);
  const int cb = co / 64, r = co % 64;
  float v[64];
#pragma unroll 8
  for (int i = 0; i < 64; ++i) v[i] = w[((long long)co * cin + c * 64 + i) * 9 + d];
  const int E0 = mx_exp(fmaxf(amax16(v), amax16(v + 16)));
  const int E1 = mx_exp(fmaxf(amax16(v + 32), amax16(v + 48)));
  uint8_t* base = img + ((long long)cb * nch + c) * MX_WIMG;
  const int x = (r >> 2) & 3;
#pragma unroll
  for (int tt = 0; tt < 4; ++tt)
    *(u32x4*)(base + r * MX_WROW + (4 * d + (tt ^ x)) * 16) = mx_cvt16(v + 16 * tt, tt < 2 ? mx_inv(E0) : mx_inv(E1));
  base[MX_WDATA + r * 32 + d] = (uint8_t)(E0 + 127);
  base[MX_WDATA + r * 32 + 16 + d] = (uint8_t)(E1 + 127);
}

// ---------------------------------------------------------------------------
// the conv: window form (as conv_fwd_frame_kernel, dv_conv.hip) over TP =
// 32 * NW pixels x 64 output channels per workgroup, K in 64-channel chunks.
// Per chunk the block's weight image and the pixel window (zero halo) of
// e4m3 bytes + scales arrive by LDS-DMA into a 2-deep ring; every tap reads
// the same window at a fixed offset.  Window image: 64 B per window pixel p,
// its 16-B slots XOR-swizzled by (p >> 2) & 3 (conflict-free ds_read_b128 for
// any 16 lanes whose window indices are distinct mod 16 — fw_pix below); the
// pixel's scale pair in a separate u32 image.
// ---------------------------------------------------------------------------
struct Mx8Args {
  const uint8_t* q0;
  const unsigned* s0;
  const uint8_t* q1;
  const unsigned* s1;
  int c0, c1;  // channels in each source (c1 = 0: one source)
  const uint8_t* w;
  const float* bias;
  const bf16* res;
  int ldres;
  bf16* y;
  int ldy;
  int H, cin, cout;
  long long M;
};

template <int W, int TP>
struct MxGeom {
  static constexpr int NF = W == 8 ? TP / 64 : 1;          // frames per tile (8x8 frames)
  static constexpr int NWR = W == 8 ? 10 : TP / W + 2;     // window rows per frame
  static constexpr int WQ = W == 8 ? 12 : W + 2;           // window pixel slots per row
  static constexpr int FPIX = NWR * WQ;
  static constexpr int WPIX = NF * FPIX;
  static constexpr int NDP = (WPIX * 64 + 1023) / 1024;    // window data pieces (16-B DMA)
  static constexpr int NSP = (WPIX * 4 + 255) / 256;       // window scale pieces (4-B DMA)
  static constexpr int XOFF = MX_WIMG;                     // window data
  static constexpr int SOFF = XOFF + NDP * 1024;           // window scales
  static constexpr int BUF = SOFF + NSP * 256;
};

// lane r -> pixel of the wave's 32-pixel group: the ds_read_b128 16-lane
// groups {0-3, 12-15, 20-27} and their complement each take one pixel of
// every residue of the window index mod 16 (as dv_conv.hip's fw_pix)
template <int W>
__device__ __forceinline__ int mx_pix(int r) {
  const bool ga = r < 4 || (r >= 12 && r < 16) || (r >= 20 && r < 28);
  const int a = ga ? (r < 4 ? r : (r < 16 ? r - 8 : r - 12)) : (r < 12 ? r - 4 : (r < 20 ? r - 8 : r - 16));
  if constexpr (W == 8) return (2 * (a >> 3) + (ga ? 0 : 1)) * 8 + (a & 7);
  else return (ga ? 0 : 16) + a;
}

__device__ __forceinline__ void dma4s(__amdgpu_buffer_rsrc_t r, void* lds, unsigned voff, unsigned soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 4, (int)voff, (int)soff, 0, 0);
}

template <int W, int NW, bool SPLIT = true>
__global__ __launch_bounds__(NW * 64) void conv_fwd_mx8_kernel(Mx8Args p) {
  constexpr int TP = 32 * NW;
  using G = MxGeom<W, TP>;
  constexpr int BUF = G::BUF, WQ = G::WQ;
  __shared__ __attribute__((aligned(1024))) char smem[2 * BUF];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6) & (NW - 1);  // masked: piece types fold
  const int npx = (int)(p.M / TP), ncb = p.cout / 64;
  // consecutive blocks (one XCD each, round robin) take the pixel tiles of one
  // output-channel block: an XCD's L2 keeps that block's weights
  int L = blockIdx.x;
  const int nblk = npx * ncb;
  if (nblk % 8 == 0) L = (L % 8) * (nblk / 8) + L / 8;
  const int cb = L / npx;
  const long long m0 = (long long)(L % npx) * TP;
  const int co0 = cb * 64;
  const int nch0 = p.c0 / 64, nch = p.cin / 64;
  const int HW = p.H * W;
  const int y0 = W == 8 ? 0 : (int)((m0 % HW) / W);
  const long long fb = W == 8 ? m0 : m0 - (m0 % HW) + (long long)y0 * W;

  // DMA pieces per chunk, each type spread over the waves: weight pieces
  // (1 KB), window data pieces (1 KB), window scale pieces (256 B).  Piece i of
  // a type goes to wave i % NW; a wave's per-lane window offsets (or DMA_OOB)
  // are fixed for the launch, the chunk offset rides in soffset.
  constexpr int NWP = (MX_WPIECES + NW - 1) / NW, NXP = (G::NDP + NW - 1) / NW, NSPW = (G::NSP + NW - 1) / NW;
  unsigned xo0[NXP], xo1[NXP], so[NSPW];
  auto src_pix = [&](int wp, long long& pix) {
    const int f = wp / G::FPIX, rem = wp - f * G::FPIX, wy = rem / WQ, wx = rem - wy * WQ;
    const int yy = y0 + wy - 1;
    pix = fb + (long long)f * 64 + (long long)(wy - 1) * W + (wx - 1);
    return wp < G::WPIX && wx >= 1 && wx <= W && yy >= 0 && yy < p.H && (W == 8 || wy <= TP / W + 1);
  };
#pragma unroll
  for (int i = 0; i < NXP; ++i) {
    const int slot = min(wave + NW * i, G::NDP - 1) * 64 + lane, wp = slot >> 2;
    const int t = (slot & 3) ^ ((wp >> 2) & 3);  // the source 16-B chunk this LDS slot holds
    long long pix;
    const bool ok = src_pix(wp, pix);
    xo0[i] = ok ? (unsigned)(pix * p.c0 + t * 16) : DMA_OOB;
    xo1[i] = ok ? (unsigned)(pix * p.c1 + t * 16) : DMA_OOB;
  }
#pragma unroll
  for (int i = 0; i < NSPW; ++i) {
    long long pix;
    const bool ok = src_pix(min(wave + NW * i, G::NSP - 1) * 64 + lane, pix);
    so[i] = ok ? (unsigned)(pix * 4) : DMA_OOB;
  }
  const __amdgpu_buffer_rsrc_t wr = dma_rsrc(p.w + (long long)cb * nch * MX_WIMG, (unsigned)(nch * MX_WIMG));
  const __amdgpu_buffer_rsrc_t qr0 = dma_rsrc(p.q0, (unsigned)(p.M * p.c0));
  const __amdgpu_buffer_rsrc_t sr0 = dma_rsrc(p.s0, (unsigned)(p.M * 4 * nch0));
  const __amdgpu_buffer_rsrc_t qr1 = dma_rsrc(p.q1, (unsigned)(p.M * p.c1));
  const __amdgpu_buffer_rsrc_t sr1 = dma_rsrc(p.s1, (unsigned)(p.M * 4 * (nch - nch0)));
  constexpr int NPW = NWP + NXP + NSPW;  // pieces per wave per chunk

  // this wave's piece i of chunk c (i < NPW; the type is known at compile time
  // once the tap loop is unrolled)
  auto issue1 = [&](int c, int i) {
    char* b = smem + (c & 1) * BUF;
    const bool first = c < nch0;
    const int cc = first ? c : c - nch0;
    if (i < NWP) {
      const int k = min(wave + NW * i, MX_WPIECES - 1);
      dma16s(wr, b + k * 1024, (unsigned)(k * 1024 + lane * 16), (unsigned)(c * MX_WIMG));
    } else if (i < NWP + NXP) {
      const int j = i - NWP, k = min(wave + NW * j, G::NDP - 1);
      char* dst = b + G::XOFF + k * 1024;
      if (!SPLIT || first) dma16s(qr0, dst, xo0[j], (unsigned)(cc * 64));
      else dma16s(qr1, dst, xo1[j], (unsigned)(cc * 64));
    } else {
      const int j = i - NWP - NXP, k = min(wave + NW * j, G::NSP - 1);
      char* dst = b + G::SOFF + k * 256;
      const unsigned sof = (unsigned)(cc * (int)p.M * 4);  // < 2^31: host-checked
      if (!SPLIT || first) dma4s(sr0, dst, so[j], sof);
      else dma4s(sr1, dst, so[j], sof);
    }
  };

  // prologue: chunk 0
#pragma unroll
  for (int i = 0; i < NPW; ++i) issue1(0, i);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  const int r = lane & 31, h = lane >> 5;
  const int tpx = wave * 32 + mx_pix<W>(r);  // this lane's pixel within the tile
  const int wb = W == 8 ? (tpx >> 6) * G::FPIX + ((tpx & 63) >> 3) * WQ + (tpx & 7)
                        : (tpx / W) * WQ + tpx % W;  // window pixel of tap (0, 0)
  const int xr = (r >> 2) & 3;
  const int aoff0 = r * MX_WROW + ((h ^ xr) << 4), aoff1 = r * MX_WROW + (((2 + h) ^ xr) << 4);
  f32x16 acc[2][2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[j][0][e] = acc[j][1][e] = 0.f;

  // one chunk; PRE (compile-time): chunk c + 1 exists and is issued here (the
  // loop is split into the chunks that issue and the last one: no per-piece
  // branch between the MFMAs)
  auto chunk = [&](int c, auto PRE) {
    const char* b = smem + (c & 1) * BUF;
    // the lane's A scales of both 32-row halves: 9 tap bytes of K-block h
    unsigned as[2][3];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const unsigned* sp = (const unsigned*)(b + MX_WDATA + (32 * j + r) * 32 + 16 * h);
      as[j][0] = sp[0];
      as[j][1] = sp[1];
      as[j][2] = sp[2];
    }
    u32x4 bq[3][2], aq[3][2][2];
    unsigned bs[3];
    auto rd = [&](int d, int s) {
      const int pw = wb + (d / 3) * WQ + (d % 3);  // window pixel of tap d
      const int xp = (pw >> 2) & 3;
      const char* pb = b + G::XOFF + pw * 64;
      bq[s][0] = *(const u32x4*)(pb + ((h ^ xp) << 4));
      bq[s][1] = *(const u32x4*)(pb + (((2 + h) ^ xp) << 4));
      bs[s] = *(const uint8_t*)(b + G::SOFF + pw * 4 + h);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        aq[s][j][0] = *(const u32x4*)(b + 32 * j * MX_WROW + aoff0 + d * 64);
        aq[s][j][1] = *(const u32x4*)(b + 32 * j * MX_WROW + aoff1 + d * 64);
      }
    };
    rd(0, 0);
    rd(1, 1);
#pragma unroll
    for (int d = 0; d < 9; ++d) {
      if (d + 2 < 9) rd(d + 2, (d + 2) % 3);
      const int s = d % 3;
      const v8i bf = cat8(bq[s][0], bq[s][1]);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const v8i af = cat8(aq[s][j][0], aq[s][j][1]);
        const int sa = (int)((as[j][d / 4] >> (8 * (d % 4))) & 255u);
        acc[j][d & 1] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(af, bf, acc[j][d & 1], 0, 0, 0, sa, 0,
                                                                       (int)bs[s]);
      }
      // chunk c + 1's pieces go out in the MFMA shadow (its buffer was last
      // read in chunk c - 1, before the last barrier)
      if constexpr (decltype(PRE)::value) {
#pragma unroll
        for (int i = d; i < NPW; i += 9) issue1(c + 1, i);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };
  for (int c = 0; c + 1 < nch; ++c) chunk(c, std::true_type{});
  if (nch > 0) chunk(nch - 1, std::false_type{});

  // epilogue: lane owns pixel m, channels co0 + 32j + 8g + 4h + e; bias and
  // residual loaded for the whole tile before the first store
  const long long m = m0 + tpx;
  f32x4 bb[2][4];
  u32x2 rq[2][4];
  if (p.bias) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) bb[j][g] = *(const f32x4*)(p.bias + co0 + 32 * j + 8 * g + 4 * h);
  }
  if (p.res) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) rq[j][g] = *(const u32x2*)(p.res + m * p.ldres + co0 + 32 * j + 8 * g + 4 * h);
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = acc[j][0][4 * g + e] + acc[j][1][4 * g + e];
      if (p.bias) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += bb[j][g][e];
      }
      if (p.res) {
        const bf16x4 t4 = __builtin_bit_cast(bf16x4, rq[j][g]);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += (float)t4[e];
      }
      *(bf16x4*)(p.y + m * p.ldy + co0 + 32 * j + 8 * g + 4 * h) =
          bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
    }
  }
}

// ---------------------------------------------------------------------------
// Persistent form for the wide frames (W = 64 / 128) with one or two input
// chunks (cin <= 128: the 64² / 128² stage convs of config 5), where the
// per-tile kernel above re-fetched the whole weight image for one chunk of
// work and exposed the operand DMA latency of every tile.  The block's
// weight image (NCH chunks) stays resident in LDS for the workgroup's life;
// the workgroup walks a contiguous range of 128-pixel tiles of ONE
// output-channel block (consecutive tiles share two of their three window
// rows in this XCD's L2) as a sequence of (tile, chunk) steps whose pixel
// windows stream through a 3-deep LDS ring: the window of step s + 2 is in
// flight while step s multiplies, and the finished tile's stores go out at
// the start of the next tile.  No residual (the Block3D convs take none).
// ---------------------------------------------------------------------------
template <int W>
struct MxPGeom {
  using G = MxGeom<W, 128>;
  static constexpr int WBUF = G::NDP * 1024 + G::NSP * 256;  // one step's window (data + scales)
  static constexpr int NWB = 3;
};

template <int W, int NCH>
constexpr int mxp_lds() { return NCH * MX_WIMG + MxPGeom<W>::NWB * MxPGeom<W>::WBUF; }

template <int W, int NCH, bool SPLIT = true>
__global__ __launch_bounds__(256) void conv_fwd_mx8p_kernel(Mx8Args p, int tiles_per_wg, int wg_per_cb) {
  constexpr int NW = 4, TP = 128;
  using G = MxGeom<W, TP>;
  using PG = MxPGeom<W>;
  constexpr int WQ = G::WQ, WBUF = PG::WBUF, NWB = PG::NWB, RES = NCH * MX_WIMG;
  static_assert(W >= 16 && TP % W == 0, "whole-row tiles");
  __shared__ __attribute__((aligned(1024))) char smem[mxp_lds<W, NCH>()];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cb = blockIdx.x / wg_per_cb, g = blockIdx.x % wg_per_cb;
  const int co0 = cb * 64;
  const int npx = (int)(p.M / TP);
  const int t0 = g * tiles_per_wg, t1 = min(npx, t0 + tiles_per_wg);
  if (t0 >= t1) return;  // (uniform per workgroup)
  const int nsteps = (t1 - t0) * NCH;
  const int nch0 = p.c0 / 64;
  const int HW = p.H * W;

  // resident weights: the block's NCH chunk images, one DMA pass
  const __amdgpu_buffer_rsrc_t wr = dma_rsrc(p.w + (long long)cb * NCH * MX_WIMG, (unsigned)(NCH * MX_WIMG));
#pragma unroll
  for (int k = wave; k < NCH * MX_WPIECES; k += NW) dma16s(wr, smem + k * 1024, (unsigned)(k * 1024 + lane * 16), 0u);

  // per-lane window geometry (tile-relative): data pieces, then scale pieces
  constexpr int NXP = (G::NDP + NW - 1) / NW, NSPW = (G::NSP + NW - 1) / NW;
  int xoff[NXP], xwy[NXP], xt[NXP], soff[NSPW], swy[NSPW];
#pragma unroll
  for (int i = 0; i < NXP; ++i) {
    const int slot = min(wave + NW * i, G::NDP - 1) * 64 + lane, wp = slot >> 2;
    const int wy = wp / WQ, wx = wp - wy * WQ;
    const bool ok = wp < G::WPIX && wx >= 1 && wx <= W;
    xt[i] = ((slot & 3) ^ ((wp >> 2) & 3)) * 16;
    xoff[i] = (wy - 1) * W + (wx - 1);
    xwy[i] = ok ? wy : -(1 << 20);
  }
#pragma unroll
  for (int i = 0; i < NSPW; ++i) {
    const int wp = min(wave + NW * i, G::NSP - 1) * 64 + lane;
    const int wy = wp / WQ, wx = wp - wy * WQ;
    const bool ok = wp < G::WPIX && wx >= 1 && wx <= W;
    soff[i] = (wy - 1) * W + (wx - 1);
    swy[i] = ok ? wy : -(1 << 20);
  }
  const __amdgpu_buffer_rsrc_t qr0 = dma_rsrc(p.q0, (unsigned)(p.M * p.c0));
  const __amdgpu_buffer_rsrc_t sr0 = dma_rsrc(p.s0, (unsigned)(p.M * 4 * nch0));
  const __amdgpu_buffer_rsrc_t qr1 = dma_rsrc(p.q1, (unsigned)(p.M * p.c1));
  const __amdgpu_buffer_rsrc_t sr1 = dma_rsrc(p.s1, (unsigned)(p.M * 4 * (NCH - nch0)));
  // the window of step s into ring slot s % NWB (piece j of this wave).  The
  // step's tile row, source and chunk are worked out once per step in 32-bit
  // arithmetic (M * C < 2^31, host-checked): a 64-bit modulo per DMA piece
  // was a ~150-instruction scalar division in front of every DMA.
  struct StepDma {
    int m0, y0, cc, buf;
    bool first;
  };
  auto step_dma = [&](int st) {
    StepDma sd;
    const int tile = t0 + st / NCH, c = st % NCH;
    sd.m0 = tile * TP;
    sd.y0 = (sd.m0 % HW) / W;
    sd.first = c < nch0;
    sd.cc = sd.first ? c : c - nch0;
    sd.buf = st % NWB;
    return sd;
  };
  auto issue1 = [&](const StepDma& sd, int j) {
    char* b = smem + RES + sd.buf * WBUF;
    if (j < NXP) {
      const int k = min(wave + NW * j, G::NDP - 1);
      const int yy = sd.y0 + xwy[j] - 1;
      const bool ok = (unsigned)yy < (unsigned)p.H;
      const int pix = sd.m0 + xoff[j];
      const unsigned vo = ok ? (unsigned)(pix * ((!SPLIT || sd.first) ? p.c0 : p.c1) + xt[j]) : DMA_OOB;
      if (!SPLIT || sd.first) dma16s(qr0, b + k * 1024, vo, (unsigned)(sd.cc * 64));
      else dma16s(qr1, b + k * 1024, vo, (unsigned)(sd.cc * 64));
    } else {
      const int jj = j - NXP, k = min(wave + NW * jj, G::NSP - 1);
      const int yy = sd.y0 + swy[jj] - 1;
      const bool ok = (unsigned)yy < (unsigned)p.H;
      const unsigned vo = ok ? (unsigned)((sd.m0 + soff[jj]) * 4) : DMA_OOB;
      const unsigned so = (unsigned)(sd.cc * (int)p.M * 4);
      char* dst = b + G::NDP * 1024 + k * 256;
      if (!SPLIT || sd.first) dma4s(sr0, dst, vo, so);
      else dma4s(sr1, dst, vo, so);
    }
  };
  constexpr int NPWX = NXP + NSPW;
  // prologue: steps 0 and 1 in flight with the weights; wait for everything
#pragma unroll
  for (int st = 0; st < NWB - 1; ++st)
    if (st < nsteps) {
      const StepDma sd = step_dma(st);
#pragma unroll
      for (int j = 0; j < NPWX; ++j) issue1(sd, j);
    }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  const int r = lane & 31, h = lane >> 5;
  const int tpx = wave * 32 + mx_pix<W>(r);
  const int wb = (tpx / W) * WQ + tpx % W;
  const int xr = (r >> 2) & 3;
  const int aoff0 = r * MX_WROW + ((h ^ xr) << 4), aoff1 = r * MX_WROW + (((2 + h) ^ xr) << 4);
  unsigned as[NCH][2][3];
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const unsigned* sp = (const unsigned*)(smem + c * MX_WIMG + MX_WDATA + (32 * j + r) * 32 + 16 * h);
      as[c][j][0] = sp[0];
      as[c][j][1] = sp[1];
      as[c][j][2] = sp[2];
    }
  f32x4 bb[2][4];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int gg = 0; gg < 4; ++gg)
      bb[j][gg] = p.bias ? *(const f32x4*)(p.bias + co0 + 32 * j + 8 * gg + 4 * h) : f32x4{0.f, 0.f, 0.f, 0.f};
  f32x16 acc[2][2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[j][0][e] = acc[j][1][e] = 0.f;
  auto epilogue = [&](int tile) {
    const long long m = (long long)tile * TP + tpx;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = acc[j][0][4 * gg + e] + acc[j][1][4 * gg + e] + bb[j][gg][e];
        *(bf16x4*)(p.y + m * p.ldy + co0 + 32 * j + 8 * gg + 4 * h) =
            bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
      }
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[j][0][e] = acc[j][1][e] = 0.f;
  };

  // one step; PRE (compile-time): step st + NWB - 1 exists and is issued here
  auto step = [&](int st, auto PRE) {
    const int c = st % NCH;
    const bool tile_start = c == 0 && st > 0;
    if (tile_start) epilogue(t0 + st / NCH - 1);  // 8 stores, before this step's DMA
    const char* wimg = smem + c * MX_WIMG;
    const char* win = smem + RES + (st % NWB) * WBUF;
    u32x4 bq[3][2], aq[3][2][2];
    unsigned bs[3];
    auto rd = [&](int d, int sl) {
      const int pw = wb + (d / 3) * WQ + (d % 3);
      const int xp = (pw >> 2) & 3;
      const char* pb = win + pw * 64;
      bq[sl][0] = *(const u32x4*)(pb + ((h ^ xp) << 4));
      bq[sl][1] = *(const u32x4*)(pb + (((2 + h) ^ xp) << 4));
      bs[sl] = *(const uint8_t*)(win + G::NDP * 1024 + pw * 4 + h);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        aq[sl][j][0] = *(const u32x4*)(wimg + 32 * j * MX_WROW + aoff0 + d * 64);
        aq[sl][j][1] = *(const u32x4*)(wimg + 32 * j * MX_WROW + aoff1 + d * 64);
      }
    };
    rd(0, 0);
    rd(1, 1);
    constexpr bool pre = decltype(PRE)::value;
    StepDma sdn;
    if constexpr (pre) sdn = step_dma(st + NWB - 1);
#pragma unroll
    for (int d = 0; d < 9; ++d) {
      if (d + 2 < 9) rd(d + 2, (d + 2) % 3);
      const int sl = d % 3;
      const v8i bf = cat8(bq[sl][0], bq[sl][1]);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const v8i af = cat8(aq[sl][j][0], aq[sl][j][1]);
        const int sa = (int)((as[c][j][d / 4] >> (8 * (d % 4))) & 255u);
        acc[j][d & 1] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(af, bf, acc[j][d & 1], 0, 0, 0, sa, 0,
                                                                       (int)bs[sl]);
      }
      if constexpr (pre) {
#pragma unroll
        for (int j = d; j < NPWX; j += 9) issue1(sdn, j);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // step st + 1's window landed: younger than its DMA are this step's
    // stores (8 when it began a tile) and this step's DMA for st + 2
    if (tile_start) {
      if constexpr (pre) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(8 + NPWX) : "memory");
      else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      if constexpr (pre) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NPWX) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };
  int st = 0;
  for (; st + NWB - 1 < nsteps; ++st) step(st, std::true_type{});
  for (; st < nsteps; ++st) step(st, std::false_type{});
  epilogue(t1 - 1);
}

template <int W, int NCH>
int launch_mx8p(const Mx8Args& a, hipStream_t st) {
  const int ncb = a.cout / 64, npx = (int)(a.M / 128);
  int g = 256 / ncb;  // one workgroup per CU (the LDS holds one)
  if (g < 1) g = 1;
  if (g > npx) g = npx;
  const int per = (npx + g - 1) / g;
  g = (npx + per - 1) / per;
  if (a.c1 > 0) conv_fwd_mx8p_kernel<W, NCH, true><<<ncb * g, 256, 0, st>>>(a, per, g);
  else conv_fwd_mx8p_kernel<W, NCH, false><<<ncb * g, 256, 0, st>>>(a, per, g);
  return check_launch("conv_fwd_mx8p");
}

template <int W>
int launch_mx8(const Mx8Args& a, hipStream_t st) {
  constexpr int NW = MX_NW;
  const int nblk = (int)(a.M / (32 * NW)) * (a.cout / 64);
  if (a.c1 > 0) conv_fwd_mx8_kernel<W, NW, true><<<nblk, NW * 64, 0, st>>>(a);
  else conv_fwd_mx8_kernel<W, NW, false><<<nblk, NW * 64, 0, st>>>(a);
  return check_launch("conv_fwd_mx8");
}

}  // namespace

extern "C" int dv_mx8_quant(const void* x, int ld, int C, long long M, void* q, void* s, void* stream) {
  DV_REQUIRE(x && q && s, "null pointer");
  DV_REQUIRE(C > 0 && C % 64 == 0 && ld >= C && ld % 8 == 0, "C must be a multiple of 64, ld >= C, ld % 8 == 0");
  DV_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)q & 15) == 0 && ((uintptr_t)s & 3) == 0, "misaligned");
  if (M == 0) return DV_OK;
  const long long n = M * (C / 64);
  mx8_quant_kernel<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>((const bf16*)x, ld, C, M,
                                                                                (uint8_t*)q, (unsigned*)s);
  return check_launch("mx8_quant");
}

extern "C" int dv_mx8_image_bytes(int cout, int cin, long long* bytes) {
  DV_REQUIRE(bytes, "null pointer");
  DV_REQUIRE(cout > 0 && cout % 64 == 0 && cin > 0 && cin % 64 == 0, "cout and cin must be multiples of 64");
  *bytes = (long long)(cout / 64) * (cin / 64) * MX_WIMG;
  return DV_OK;
}

extern "C" int dv_mx8_pack_conv_weight(const float* w, int cout, int cin, void* img, void* stream) {
  DV_REQUIRE(w && img, "null pointer");
  DV_REQUIRE(cout > 0 && cout % 64 == 0 && cin > 0 && cin % 64 == 0, "cout and cin must be multiples of 64");
  const int n = cout * (cin / 64) * 9;
  mx8_pack_weight_kernel<<<(n + 255) / 256, 256, 0, (hipStream_t)stream>>>(w, cout, cin, (uint8_t*)img);
  return check_launch("mx8_pack_weight");
}

extern "C" int dv_conv_fwd_mx8(const void* q0, const void* s0, int c0, const void* q1, const void* s1, int c1,
                               const void* wimg, const float* bias, const void* res, int ldres, void* y, int ldy,
                               int nf, int h, int w, int cout, void* stream) {
  DV_REQUIRE(q0 && s0 && wimg && y, "null pointer");
  DV_REQUIRE(c0 > 0 && c0 % 64 == 0 && c1 >= 0 && c1 % 64 == 0 && (c1 == 0 || (q1 && s1)),
             "source channels must be multiples of 64");
  DV_REQUIRE(cout > 0 && cout % 64 == 0 && ldy >= cout && ldy % 4 == 0 && (!res || (ldres >= cout && ldres % 4 == 0)),
             "bad output channels / strides");
  constexpr int TP = 32 * MX_NW;
  const bool geom = (w == 8 && h == 8) || ((w == 16 || w == 32 || w == 64 || w == 128) && h % (TP / w) == 0);
  DV_REQUIRE(geom, "frame geometry outside the MX-fp8 window conv (W in {16,32,64,128} with H % (128/W) == 0, or 8x8)");
  const long long M = (long long)nf * h * w;
  DV_REQUIRE(M % TP == 0, "pixel count must be a multiple of 128");
  const int cin = c0 + c1;
  DV_REQUIRE(M * c0 < (long long)DMA_OOB && M * c1 < (long long)DMA_OOB && M * 4 * (cin / 64) < (long long)DMA_OOB &&
                 (long long)(cin / 64) * MX_WIMG < (long long)DMA_OOB,
             "tensor too large for the 32-bit DMA offsets");
  DV_REQUIRE(((uintptr_t)q0 & 15) == 0 && (!q1 || ((uintptr_t)q1 & 15) == 0) && ((uintptr_t)wimg & 15) == 0,
             "operands must be 16-B aligned");
  if (M == 0) return DV_OK;
  Mx8Args a;
  a.q0 = (const uint8_t*)q0; a.s0 = (const unsigned*)s0;
  a.q1 = (const uint8_t*)(c1 ? q1 : q0); a.s1 = (const unsigned*)(c1 ? s1 : s0);
  a.c0 = c0; a.c1 = c1; a.w = (const uint8_t*)wimg; a.bias = bias; a.res = (const bf16*)res; a.ldres = ldres;
  a.y = (bf16*)y; a.ldy = ldy; a.H = h; a.cin = cin; a.cout = cout; a.M = M;
  hipStream_t st = (hipStream_t)stream;
  // the persistent resident-weight form for the wide frames with <= 2 chunks
  if (!res && (w == 64 || w == 128) && cin <= 128) {
    if (w == 128) return cin == 64 ? launch_mx8p<128, 1>(a, st) : launch_mx8p<128, 2>(a, st);
    return cin == 64 ? launch_mx8p<64, 1>(a, st) : launch_mx8p<64, 2>(a, st);
  }
  switch (w) {
    case 8: return launch_mx8<8>(a, st);
    case 16: return launch_mx8<16>(a, st);
    case 32: return launch_mx8<32>(a, st);
    case 64: return launch_mx8<64>(a, st);
    default: return launch_mx8<128>(a, st);
  }
}
