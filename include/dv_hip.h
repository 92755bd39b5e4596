/* libdv_hip — C-ABI of the MI355X (gfx950) Unet3D denoising path.
 *
 * The reference (SeanNobel/DALLE2-video) is pure Python: its "FFI" for this
 * path is the set of PyTorch modules in dalle2_video/dalle2_video.py whose
 * arithmetic PyTorch dispatches to vendor kernels.  Each entry point below
 * replaces the device work behind one of those modules; the cited file:line
 * is the reference call site it serves (paths relative to the reference
 * root).  The Python mirror (dalle2-video_amd/dalle2_video/_lib.py) binds
 * these with ctypes — see INTEGRATION.md.
 *
 * Conventions
 *   - Activations are channels-last frames: element (frame f, y, x, channel c)
 *     of a [nf][h][w][*] tensor lives at ptr[((f*h + y)*w + x)*ld + c]; `ld`
 *     (channel stride per pixel) lets a caller pass a channel slice of a
 *     wider buffer (the skip concatenations, dalle2_video.py:926-945, are
 *     never materialised).  nf = batch * frames.
 *   - `dtype` is DV_F32 (parity mode, exact f32 MFMA/VALU) or DV_BF16 (bf16
 *     storage, f32 accumulation).  Parameters, statistics and gradients of
 *     parameters are always f32.
 *   - All pointers are caller-owned device buffers; nothing here allocates.
 *     Calls are asynchronous on `stream` (a hipStream_t, may be NULL).
 *   - Return 0 on success, a negative DV_ERR_* code otherwise; the message is
 *     in dv_last_error() (thread-local).  No C++ exception crosses the ABI.
 */
#ifndef DV_HIP_H
#define DV_HIP_H
#ifdef __cplusplus
extern "C" {
#endif

enum { DV_F32 = 0, DV_BF16 = 1 };
enum { DV_OK = 0, DV_ERR_INVALID = -1, DV_ERR_LAUNCH = -2, DV_ERR_UNSUPPORTED = -3 };
enum { DV_ACT_NONE = 0, DV_ACT_SILU = 1, DV_ACT_GELU = 2 };

const char* dv_last_error(void);
int dv_abi_version(void);
/* Zero n floats on the stream with a kernel (graph-capture safe: a kernel
 * node, not a memset node).  Used to reset cached workspaces.               */
int dv_zero_f32(float* p, long long n, void* stream);

/* ---- convolutions (1,k,k), stride 1, padding k//2 -------------------------
 * Replaces nn.Conv3d in Block3D.project (dalle2_video.py:107), res_conv
 * (:170), Downsample3D (:25), the stage-3 projection (:537),
 * PixelShuffleUpsample3D.conv (:48), CrossEmbedLayer3D (:224-232) and to_out
 * (:637); also every bias-free nn.Linear over tokens (k=1).
 * Implicit GEMM on MFMA: M = nf*h*w pixels, N = cout, K = k*k*cin.
 * Input channels [0,c0) come from x0 (stride ld0), [c0,cin) from x1 (ld1);
 * c0 must be a multiple of 8 (pass c0=cin, x1=NULL for one source).
 * wpack: packed weight [cout][k*k][cin] of `dtype` (dv_pack_conv_weight).
 * Epilogue: y = act(acc + bias) + res + res2 (res / res2 may be NULL; each
 * with its own pixel stride; res2 carries the unet skip gradient a dgrad
 * adds besides the shared input-gradient buffer, ops.SkipGrad, the hiddens
 * of dalle2_video.py:926-936).  cin % 8 == 0 required.
 * GroupNorm statistics epilogue (Block3D conv -> GroupNorm, :107-109): when
 * gn_sums != NULL the stored y's per-(clip, channel) sum and sum of squares
 * are added into gn_sums[replica][nf*h*w / gn_P][cout][2] (zero on entry;
 * gn_R replicas, clip = pixel / gn_P; nf*h*w % gn_P == 0), the `sums` a
 * following dv_gn_fwd(..., sums_replicas = gn_R) consumes without its
 * reduce pass.  NULL: no statistics (gn_P / gn_R ignored).                */
int dv_conv_fwd(int dtype, const void* x0, int ld0, int c0, const void* x1, int ld1,
                const void* wpack, const float* bias, const void* res, int ldres,
                const void* res2, int ldres2, void* y, int ldy, int nf, int h, int w, int cin,
                int cout, int ksize, int act, float* gn_sums, long long gn_P, int gn_R,
                void* stream);

/* 3x3 conv of a GroupNorm + FiLM + SiLU output that is never produced by its
 * own pass (Block3D -> the next Block3D's project, dalle2_video.py:107-133):
 * z is the GroupNorm's INPUT; the conv stages y = silu(A z + B) into LDS,
 * A = rstd*gamma*(1+scale), B = (beta - mean*rstd*gamma)*(1+scale) + shift,
 * mean / rstd per (clip, group) from z's statistics `sums` (R replicas,
 * stride rstride, [clip][C][2], as dv_conv_fwd's statistics epilogue leaves
 * them).  Writes mean / rstd ([clip][groups], the GroupNorm's saved
 * statistics), y itself when y != NULL (for the conv's weight gradient), and
 * zeroes zero[0, zero_n) (the GroupNorm call's duty towards the next call's
 * sums, dv_gn_fwd's `next`).  Output / statistics as dv_conv_fwd (bf16, no
 * residual, act none).  Built for cin = 64, 8 groups, w = 64, cout % 64 == 0,
 * clips of whole 128-pixel stages; DV_ERR_UNSUPPORTED otherwise (run
 * dv_gn_fwd + dv_conv_fwd instead).                                        */
typedef struct {
  const float* sums;
  long long rstride;
  int R;
  long long P;        /* pixels per clip */
  int groups;
  float eps;
  const float* gamma; /* [C] */
  const float* beta;  /* [C] */
  const float* ss;    /* [clips][2C] (scale, shift) or NULL */
  float* mean;        /* [clips][groups], written */
  float* rstd;
  void* y;            /* [M][ldy] bf16, written, or NULL */
  int ldy;
  float* zero;        /* zeroed, or NULL */
  long long zero_n;
} DvGnIn;
int dv_conv_fwd_gn_in(const DvGnIn* g, const void* z, int ldz, const void* wpack,
                      const float* bias, void* y, int ldy, int nf, int h, int w, int cin,
                      int cout, float* gn_sums, long long gn_P, int gn_R, void* stream);

/* Weight (and fused bias) gradient of dv_conv_fwd, written in torch layout:
 * dw (cout_real, cin_real, 1, k, k) (+)= sum_p dY[p][co] X[p + tap][ci]
 * (accumulate_w), db[cout_real] (+)= sum_p dY[p][co] (accumulate_b; db may
 * be NULL).  cout / cin are the padded sizes of dy's channels / x's channels.
 * ws: caller-owned f32 scratch of at least dv_conv_wgrad_ws() floats (no
 * zeroing required).  bf16 3x3 / 1x1 convolutions with cin, cout % 64 == 0
 * run the row-window kernel (split over pixels, plain-store partials summed
 * by a second launch); other shapes run f32-atomic split-K over pixels.     */
int dv_conv_wgrad_ws(int dtype, int nf, int h, int w, int cin, int c0, int split, int cout,
                     int ksize, long long* floats);
int dv_conv_wgrad(int dtype, const void* dy, int lddy, const void* x0, int ld0, int c0,
                  const void* x1, int ld1, float* dw, int accumulate_w, float* db,
                  int accumulate_b, float* ws, long long ws_floats, int nf, int h, int w,
                  int cin, int cout, int cout_real, int cin_real, int ksize, void* stream);

/* Deferred split-K sum.  dv_conv_wgrad_deferred is dv_conv_wgrad, except that
 * when the row-window kernel runs with several pixel splits it only writes
 * the partials into `ws` (which must then stay untouched until the sum has
 * run) and describes the pending sum in *entry (host memory; entry->S > 0).
 * Otherwise the gradient is complete on return and entry->S = 0.
 * dv_wgrad_reduce_plan fills blk0 / G of a host table of n pending sums and
 * the launch's block count (*blocks); dv_wgrad_reduce_batched (table copied to
 * the DEVICE) then performs all n sums in one launch.  Entries must not share
 * a dw or db target.  The trainer defers every conv of one backward pass and
 * sums them once at its end (replaces a reduce launch per conv).          */
typedef struct {
  const float* part;    /* [S][cout * K] partials (f32, or bf16 below) */
  const float* dbpart;  /* [S][cout] bias partials or NULL             */
  float* dw;            /* (cout, cin, 1, k, k) target                 */
  float* db;            /* [cout] target or NULL                       */
  long long n4;         /* cout * K / 4                                */
  long long blk0;       /* first block of this entry (plan)            */
  int S, G, cout, acc_w, acc_b;
  int part_bf16;        /* 1: part holds bf16 values (bias partials f32) */
} DvWgradReduceEntry;
int dv_conv_wgrad_deferred(int dtype, const void* dy, int lddy, const void* x0, int ld0, int c0,
                           const void* x1, int ld1, float* dw, int accumulate_w, float* db,
                           int accumulate_b, float* ws, long long ws_floats, int nf, int h,
                           int w, int cin, int cout, int cout_real, int cin_real, int ksize,
                           DvWgradReduceEntry* entry, void* stream);
int dv_wgrad_reduce_plan(DvWgradReduceEntry* host_table, int n, long long* blocks);
int dv_wgrad_reduce_batched(const DvWgradReduceEntry* table, int n, long long blocks,
                            void* stream);
/* One pending entry (a HOST pointer: the fields ride in the kernel arguments,
 * no device table), e.g. on a side stream right after its wgrad.          */
int dv_wgrad_reduce_one(const DvWgradReduceEntry* entry, void* stream);

/* ---- CrossEmbedLayer3D (dalle2_video.py:208-244, Unet3D.init_conv) ------
 * nbranch parallel (1,k_b,k_b) 'same' convolutions of one small-channel
 * input (cin <= 8: the video, + the lowres conditioning for upsampler unets),
 * outputs concatenated along channels in branch order (dim/2, dim/4, rest).
 * Direct MFMA kernels: each 16-channel output tile runs only its own window.
 * w[b] / b[b]: torch Conv3d weight (cout_b, cin, 1, k_b, k_b) and bias
 * (f32, b may be NULL).  dw / db (wgrad only): gradients of the same shapes,
 * written or added to (accumulate_w / accumulate_b; db[b] may be NULL).
 * Requirements: k_b odd <= 15 ascending, sum(cout_b) % 8 == 0 and <= 128
 * (the last 16-channel tile is zero-padded);
 * bf16 activations, w % 32 == 0, ldx % 4 == 0 (cin <= 4) or % 8 == 0,
 * ldy % 4 == 0, lddy % 8 == 0.
 *   dv_cross_embed_pack: weights + biases -> `image` (device, bf16 elements
 *     from dv_cross_embed_image_elems; repack whenever the weights change);
 *   dv_cross_embed_fwd: y[p][0..sum cout) = concat_b conv_b(x)[p] + bias;
 *   dv_cross_embed_wgrad: weight / bias gradients from dy; ws = f32 scratch
 *     of dv_cross_embed_wgrad_ws floats.                                    */
typedef struct {
  int nbranch, cin;
  int k[4], cout[4];
  const float* w[4];
  const float* b[4];
  float* dw[4];
  float* db[4];
  int accumulate_w, accumulate_b;
} DvCrossEmbed;
int dv_cross_embed_image_elems(const DvCrossEmbed* ce, long long* elems);
int dv_cross_embed_pack(const DvCrossEmbed* ce, void* image, void* stream);
int dv_cross_embed_fwd(const DvCrossEmbed* ce, const void* image, const void* x, int ldx,
                       void* y, int ldy, int nf, int h, int w, void* stream);
int dv_cross_embed_wgrad_ws(const DvCrossEmbed* ce, int nf, int h, int w, long long* floats);
int dv_cross_embed_wgrad(const DvCrossEmbed* ce, const void* dy, int lddy, const void* x,
                         int ldx, float* ws, long long ws_floats, int nf, int h, int w,
                         void* stream);

/* Small-channel (1,k,k) convolution forward on the same direct kernel (the
 * cascade's 256x256 unet, dim 8: Block3D.project / res_conv with cin <= 16,
 * cout <= 128, dalle2_video.py:107, 170 — an implicit GEMM with N = 8 runs
 * its MFMA tiles 1/8 full).  y = conv(cat(x0[:, :c0], x1)) + bias (+ res);
 * x1 may be NULL (then c0 is ignored), else c0 % 8 == 0.  bf16, w % 32 == 0,
 * ld0 / ld1 % 8 == 0 (ld0 % 4 with cin <= 4), ldy / ldres % 4 == 0, cout % 8.
 *   dv_conv_small_pack: torch weight (cout, cin, 1, k, k) f32 + bias (NULL:
 *     zero) -> image of dv_conv_small_image_elems bf16 elements.           */
int dv_conv_small_image_elems(int cin, int cout, int ksize, long long* elems);
int dv_conv_small_pack(const float* w, const float* bias, int cin, int cout, int ksize,
                       void* image, void* stream);
int dv_conv_small_fwd(const void* x0, int ld0, int c0, const void* x1, int ld1, const void* image,
                      const void* res, int ldres, void* y, int ldy, int nf, int h, int w, int cin,
                      int cout, int ksize, void* stream);
/* Many dv_conv_small_pack calls in ONE launch (the trainer repacks every
 * small-channel conv image once per optimizer step).  dv_conv_small_pack_plan
 * expands n host entries into the launch table: with `table` NULL it only
 * reports its size in *bytes; the caller copies the table to the device and
 * passes it to dv_conv_small_pack_batched (tables depend on the entries'
 * pointers and shapes only, so one upload serves every step).              */
typedef struct {
  const float* w;     /* f32 torch weight (cout_w, cin_w, 1, k, k) */
  const float* bias;  /* f32 [cout] or NULL (mode 0 only) */
  void* image;        /* dv_conv_small_image_elems(cin, cout, ksize) bf16 elements */
  int cin, cout, ksize;
  /* 0: the conv's own image (cin = cin_w, cout = cout_w).  1: the image of its
   * input gradient (dgrad as a conv of dY): input channels cin = cout_w, output
   * channels cout >= wcin (rows >= wcin zero), taps flipped,
   * image[ci][co][dy][dx] = w[co][ci][k-1-dy][k-1-dx]                        */
  int mode, wcin;
} DvSmallPackEntry;
int dv_conv_small_pack_plan(const DvSmallPackEntry* entries, int n, void* table, long long* bytes,
                            long long* max_elems);
int dv_conv_small_pack_batched(const void* table, int n, long long max_elems, void* stream);

/* 3x3 forward / dgrad, window form (dalle2_video.py:107 Block3D.project at
 * the 8x8 .. 64x64 stages, and the dgrads of those convs): same contract as
 * dv_conv_fwd with ksize = 3, but `wpack` is the 16-channel-chunk-major
 * image of dv_pack_conv_weight mode 2 (forward) or 3 (dgrad).  bf16 only;
 * needs (h, w) = (8, 8) with nf even, or w in {16, 32, 64} with
 * h * w % 128 == 0; cin % 16 == 0, c0 % 16 == 0 (split), cout % 64 == 0,
 * ld0 / ld1 % 8 == 0, ldy / ldres / ldres2 % 4 == 0, 16-B aligned x0 / x1 / wpack,
 * nf * h * w * ld * 2 < 2^31; returns DV_ERR_INVALID otherwise.
 * gn_sums / gn_P / gn_R as dv_conv_fwd, with gn_P % 128 == 0.             */
int dv_conv_fwd8(int dtype, const void* x0, int ld0, int c0, const void* x1, int ld1,
                 const void* wpack, const float* bias, const void* res, int ldres,
                 const void* res2, int ldres2, void* y, int ldy, int nf, int h, int w, int cin,
                 int cout, int act, float* gn_sums, long long gn_P, int gn_R, void* stream);

/* ---- MX-fp8 3x3 forward (sampling; BASELINE config 5 — Block3D.project,
 * dalle2_video.py:107, no autograd).  OCP MX-fp8: e4m3 elements, one e8m0
 * power-of-two scale per 32 consecutive channels, on the block-scaled
 * v_mfma_scale_f32_32x32x64_f8f6f4 (f32 accumulation).
 *   dv_mx8_quant: bf16 channels-last x[M][ld] (C channels) -> q[M][C] e4m3
 *     bytes + s[C/64][M] u32 (byte h = scale of channels [64c + 32h, +32)).
 *     Scale 2^E with E the smallest power keeping the block max <= 448 in its
 *     top binade; round to nearest even.  C % 64 == 0, ld % 8 == 0.
 *   dv_mx8_image_bytes / dv_mx8_pack_conv_weight: f32 weight (cout, cin, 1,
 *     3, 3) -> the kernel's swizzled image of e4m3 rows + scales,
 *     [cout/64][cin/64][38,912 B].  cout, cin % 64 == 0.
 *   dv_conv_fwd_mx8: y = conv3x3(cat(x0, x1)) + bias (+ res), y bf16.  x0 =
 *     (q0, s0) with c0 channels, x1 = (q1, s1) with c1 (0: none), both % 64;
 *     (h, w) = (8, 8), or w in {16, 32, 64, 128} with h % (128 / w) == 0;
 *     nf * h * w % 128 == 0; cout % 64 == 0; ldy, ldres % 4 == 0; 16-B
 *     aligned q / wimg.                                                     */
int dv_mx8_quant(const void* x, int ld, int C, long long M, void* q, void* s, void* stream);
int dv_mx8_image_bytes(int cout, int cin, long long* bytes);
int dv_mx8_pack_conv_weight(const float* w, int cout, int cin, void* img, void* stream);
int dv_conv_fwd_mx8(const void* q0, const void* s0, int c0, const void* q1, const void* s1, int c1,
                    const void* wimg, const float* bias, const void* res, int ldres, void* y,
                    int ldy, int nf, int h, int w, int cout, void* stream);

/* db[c] += sum_p dy[p][c]  (f32 atomics) */
int dv_bias_grad(int dtype, const void* dy, int lddy, float* db, long long npix, int c,
                 void* stream);

/* f32 torch weight (cout, cin, 1, k, k) -> packed `dtype`
 *   mode 0 (forward):  out[co][tap][ci_pad]          (ci >= cin zero)
 *   mode 1 (dgrad):    out[ci][tap'][co_pad] = w[co][ci][k*k-1-tap']
 *   modes 2 / 3:       modes 0 / 1 with each row chunk-major,
 *                      [pad / 16][k*k][16] (pad_to % 16 == 0; dv_conv_fwd8) 
 * LDS-staged (coalesced both ways); needs cin*k*k (mode 0) or cout*k*k
 * (mode 1) <= 8192.                                                        */
int dv_pack_conv_weight(int dtype, const float* w, void* out, int cout, int cin, int ksize,
                        int pad_to, int mode, void* stream);

/* Repack many weights in one launch (the trainer calls it once per optimizer
 * step for every cached conv / token-linear weight).  `table` is a DEVICE
 * array of n entries; max_elems = the largest entry's element count.       */
typedef struct {
  const float* w;  /* f32 torch weight (cout, cin, 1, k, k) */
  void* out;       /* packed image, layout as dv_pack_conv_weight(mode) */
  int dtype, cout, cin, taps, pad_to, mode;
} DvPackEntry;
int dv_pack_conv_weights_batched(const DvPackEntry* table, int n, long long max_elems,
                                 void* stream);

/* Both images of each bf16 3x3 weight from ONE read of it: the forward image
 * (mode 0 or 2, pad = cin) and the dgrad image (mode 1 or 3, pad = cout),
 * cout % 64 == 0, cin % 16 == 0.  Tile t of entry e is (64 co) x (16 ci);
 * entries own consecutive tile ranges starting at tile0, and `tile_entry`
 * (DEVICE, total_tiles ints) maps every tile to its entry.                 */
typedef struct {
  const float* w;   /* f32 torch weight (cout, cin, 1, 3, 3) */
  void* out_fwd;    /* bf16 image, mode = modes & 255 (0 or 2) */
  void* out_dgrad;  /* bf16 image, mode = modes >> 8 (1 or 3) */
  int cout, cin, taps, modes;
  long long tile0;
} DvPackPair;
int dv_pack_conv_weight_pairs(const DvPackPair* table, const int* tile_entry, long long total_tiles,
                              void* stream);

/* ---- grouped small linears ------------------------------------------------
 * Many nn.Linear layers over the SAME f32 input rows x [B][K] in ONE launch:
 * y_e [B][n_e] = act_in(x) W_e^T (+ bias_e) for every entry e.  Serves the
 * time_mlp of every ResnetBlock3D (SiLU -> Linear(time_cond_dim, 2*dim_out),
 * dalle2_video.py:143-146, applied at :182-185 — all 27 blocks of unet1 take
 * the same time embedding t) and the to_kv projections of CrossAttention over
 * the shared context c / mid_c (dalle2-pytorch CrossAttention, called at
 * :195-201).  B <= 8, K <= 512, K % 4 == 0, act_in: DV_ACT_*; W_e f32
 * [n_e][K] row-major; more than 48 entries are split into several launches. */
typedef struct DvLinEntry {
  const float* w;     /* [n][K] */
  const float* bias;  /* [n] or NULL */
  float* y;           /* forward: output [B][n]; backward: dy [B][n] */
  float* dw;          /* backward: [n][K] (+)= gradient, or NULL */
  float* db;          /* backward: [n] (+)= gradient, or NULL */
  int n;
  int accumulate_w;   /* backward: 1 adds into dw/db, 0 overwrites */
} DvLinEntry;
int dv_linear_group_fwd(const float* x, int B, int K, int act_in, const DvLinEntry* entries,
                        int n_entries, void* stream);
/* dx [B][K] (+)= act_in'(x) * sum_e dy_e W_e (accumulate_dx), dw/db per entry.
 * ws: B*K + 1 floats, ZERO on entry and left zeroed.                          */
int dv_linear_group_bwd(const float* x, int B, int K, int act_in, const DvLinEntry* entries,
                        int n_entries, float* dx, int accumulate_dx, float* ws, void* stream);

/* Batched TN GEMM on the wgrad engine: out[g][i][j] += sum_{r in group g}
 * A[r][i]*B[r][j]; A rows x m (lda), B rows x n (ldb), nbatch groups of
 * batch_rows consecutive rows; out f32 [nbatch][m][n] (atomics, pre-zeroed).
 * Used for the token reductions of the cross-attention backward.           */
int dv_gemm_tn_batched(int dtype, const void* a, int lda, const void* b, int ldb, float* out,
                       long long batch_rows, int nbatch, int m, int n, void* stream);
/* ngemm (1..3) dv_gemm_tn_batched problems sharing batch_rows, nbatch, m, n
 * (host arrays of operand pointers / strides / outputs): one launch in bf16.  */
int dv_gemm_tn_batched_multi(int dtype, int ngemm, const void* const* a, const int* lda,
                             const void* const* b, const int* ldb, float* const* out,
                             long long batch_rows, int nbatch, int m, int n, void* stream);

/* ---- GroupNorm (+ FiLM scale/shift, SiLU, residual) -----------------------
 * Block3D.norm/act with ResnetBlock3D's scale_shift (dalle2_video.py:109-133,
 * 183-189): y = act(GN(z)*gamma + beta) (optionally *(ss_scale+1)+ss_shift,
 * ss = [nb][2C] f32 with scale first), + res.  nb batch elements of P pixels
 * (all frames of one clip form one GroupNorm sample), C channels, G groups.
 * mean/rstd [nb][G] f32 are written for the backward.  Two launches per
 * call (reduce, apply).  sums: next_n floats (>= nb*C*2) that must be ZERO on
 * entry — the reduce spreads its atomics over up to 8 replicas of the
 * nb*C*2 sums that fit; the call does NOT re-zero them (its apply still
 * reads them) but zeroes `next` (next_n floats; NULL means one replica and
 * no zeroing): the buffer the caller's NEXT GroupNorm call (forward or
 * backward) will pass as `sums`.  Alternating two buffers keeps both zero on
 * entry without any memset launch.
 * C % (16 B) == 0, C <= 256 vectors, G <= 64.  act: DV_ACT_*.
 * sums_replicas > 0: `sums` already holds z's statistics in that many
 * replicas, <= 64 (the producing dv_conv_fwd / dv_conv_fwd8 epilogue): the reduce
 * launch is skipped and the call is one apply launch.                      */
int dv_gn_fwd(int dtype, const void* z, int ldz, void* y, int ldy, const void* res, int ldres,
              int nb, long long P, int C, int G, float eps, const float* gamma,
              const float* beta, const float* ss, int act, float* mean, float* rstd, float* sums,
              float* next, long long next_n, int sums_replicas, void* stream);
/* dv_gn_fwd (bf16) that also writes y as the MX-fp8 operand of the 3x3 conv
 * reading it (sampling in fp8, BASELINE config 5): q [nb*P][C] e4m3 and qs
 * [C/64][nb*P] scale pairs, bit-identical to dv_mx8_quant(y); C % 64 == 0. */
int dv_gn_fwd_mx8(const void* z, int ldz, void* y, int ldy, const void* res, int ldres, int nb,
                  long long P, int C, int G, float eps, const float* gamma, const float* beta,
                  const float* ss, int act, float* mean, float* rstd, float* sums, float* next,
                  long long next_n, int sums_replicas, void* q, void* qs, void* stream);
/* dz from dy (z is the pre-norm input); dgamma/dbeta [C] and dss [nb][2C]
 * (+)= their gradients (accumulate != 0 adds).  sums/next as dv_gn_fwd.      */
int dv_gn_bwd(int dtype, const void* dy, int lddy, const void* z, int ldz, void* dz, int lddz,
              int nb, long long P, int C, int G, const float* gamma, const float* beta,
              const float* ss, int act, const float* mean, const float* rstd, float* dgamma,
              float* dbeta, float* dss, float* sums, float* next, long long next_n,
              int accumulate, void* stream);

/* GroupNorm path selection (A/B and test hook; process-wide).  The single-
 * launch form runs reduce and apply as ONE kernel (bf16, C a power of two in
 * [8, 512] with C/G % 8 == 0, nb <= 256, a workgroup's rows in <= 16 register
 * passes; per-clip arrival counters in the last nb words of `sums`, which
 * must then hold next_n floats as `next` does).  0: automatic -- the single
 * launch only for backward calls at 16 passes (measured faster there only),
 * two launches otherwise.  1: always two launches.  2: single launch wherever
 * it applies, with the cross-workgroup wait skipped (each workgroup
 * recomputes its clip's sums: the bounded-wait fallback, for tests).
 * 3: single launch wherever it applies.                                     */
int dv_gn_path(int mode);

/* ---- row LayerNorm over channels (dalle2-pytorch LayerNorm, gain only, eps
 * 1e-5 fp32; the mid-attention pre/post norms, dalle2_video.py:431, 551,
 * 921-922).  y = (x-mu)*rstd*g (+b) (+res).  One wave per row; C a
 * multiple of 16 bytes, at most 256 such vectors.                           */
int dv_ln_fwd(int dtype, const void* x, int ldx, void* y, int ldy, const void* res, int ldres,
              long long rows, int C, const float* g, const float* b, float eps, float* mean,
              float* rstd, void* stream);
/* dg / db (+)= column sums (accumulated: zero fresh buffers).  ws: caller-owned
 * f32 scratch of *need (dv_ln_bwd_ws) floats for the per-block partials. */
int dv_ln_bwd_ws(long long rows, int C, long long* need);
int dv_ln_bwd(int dtype, const void* dy, int lddy, const void* x, int ldx, void* dx, int lddx,
              long long rows, int C, const float* g, float eps, float* dg, float* db, float* ws,
              long long ws_n, void* stream);

/* ---- layout, space-to-depth / pixel shuffle --------------------------------
 * NCTHW f32 <-> channels-last frames (cpad: padded channel stride, zeros).  */
int dv_ncthw_to_cl(int dtype, const float* x, void* y, int B, int C, int T, int H, int W, int cpad,
                   void* stream);
int dv_cl_to_ncthw(int dtype, const void* y, int ld, float* x, int B, int C, int T, int H, int W,
                   void* stream);
/* mode 0: space-to-depth 2x2 (Downsample3D's "(h 2) (w 2) -> (c 4)",
 * dalle2_video.py:18-30), src [nf][H][W][C] -> dst [nf][H/2][W/2][4C];
 * mode 1: PixelShuffle(2) after SiLU (PixelShuffleUpsample3D,
 * dalle2_video.py:64-79), src [nf][H][W][4C] -> dst [nf][2H][2W][C];
 * backward passes use the inverse mode, with z (the pre-SiLU conv output)
 * for SiLU' when act = DV_ACT_SILU.  Mode 1 adds r0 / r1 ([nf][2H][2W][C],
 * strides ldr0 / ldr1; NULL: none) to its output: the space-to-depth
 * backward sums the unet skip gradients of its input there (ops.SkipGrad). */
int dv_shuffle(int dtype, int mode, const void* src, int lds, void* dst, int ldd, const void* z,
               int ldz, const void* r0, int ldr0, const void* r1, int ldr1, int nf, int H, int W,
               int C, int act, void* stream);

/* ---- diffusion step pieces (VideoDecoder.p_losses, dalle2_video.py:1908-2010)
 * x_noisy = sqrt_ac[t]*x0 + sqrt_1m_ac[t]*noise, written channels-last into
 * y (cpad stride); normalize != 0 maps x0 from [0,1] to [-1,1] first
 * (normalize_neg_one_to_one, :1277, 1947-1956).                             */
int dv_q_sample(int dtype, const float* x0, const float* noise, const long long* t,
                const float* sqrt_ac, const float* sqrt_1m_ac, void* y, int B, int C, int T,
                int H, int W, int cpad, int normalize, int num_timesteps, void* stream);
/* loss = mean_b( w[b] * mean_(c,t,h,w) (pred - target)^2 )   (:1997-2000;
 * sample_w = p2 loss weights, NULL = 1).  loss: one f32, overwritten.        */
int dv_mse_loss(int dtype, const void* pred, int ld, const float* target, int B, int C, int T,
                int H, int W, const float* sample_w, float* loss, void* stream);
int dv_mse_loss_bwd(int dtype, const void* pred, int ld, const float* target, int B, int C, int T,
                    int H, int W, const float* sample_w, const float* dloss, void* dpred, int lddp,
                    void* stream);
/* one ancestral DDPM step (VideoDecoder.p_sample, :1621-1665, with
 * NoiseScheduler.q_posterior and predict_start_from_noise): eps is the unet
 * output (channels-last, stride ld; ld == 0: NCTHW f32).  clip != 0 clamps
 * x0 to [-1,1].  out and (optional) x0_out are NCTHW f32.                    */
int dv_p_sample(int dtype, const float* x, const void* eps, int ld, const float* noise,
                const long long* t, const float* sqrt_recip_ac, const float* sqrt_recipm1_ac,
                const float* coef1, const float* coef2, const float* logvar, float* out,
                float* x0_out, int B, int C, int T, int H, int W, int clip, int num_timesteps,
                void* stream);

/* ---- time conditioning MLPs (Unet3D.to_time_hiddens / to_time_tokens /
 * to_time_cond, dalle2_video.py:348-357; ResnetBlock3D.time_mlp, :152-155)
 * SinusoidalPosEmb (:349): out[b] = [sin(t*f), cos(t*f)], freqs = dim/2
 * host-built f32 frequencies (bit-identical to the torch expression).       */
int dv_sinusoidal(const long long* t, const float* freqs, float* out, int B, int dim, void* stream);
/* y = act_out(act_in(x) W^T + bias), B rows (the batch; <= 16 for the
 * backward), f32;
 * act_in: DV_ACT_SILU or none; act_out: none / SiLU / 2 = GELU (erf).
 * z (optional) keeps the pre-activation for the backward.                   */
int dv_linear_small_fwd(const float* x, int ldx, const float* W, const float* bias, float* y,
                        int ldy, float* z, int B, int K, int N, int act_in, int act_out,
                        void* stream);
int dv_linear_small_bwd(const float* dy, int lddy, const float* x, int ldx, const float* W,
                        const float* z, float* dx, int lddx, float* dW, float* db, int B, int K,
                        int N, int act_in, int act_out, int accumulate_dx, int accumulate_w,
                        void* stream);

/* ---- optimizer (trainer.py:65 get_optimizer -> torch AdamW; :254-257
 * clip_grad_norm_).  Flat f32 buffers; elements [0, n_wd) get weight decay
 * (ndim >= 2 parameters).  clip_coef: device scalar multiplying g (NULL: 1). */
int dv_adamw(float* p, const float* g, float* m, float* v, long long n, long long n_wd, float lr,
             float beta1, float beta2, float eps, float wd, float bc1, float bc2_sqrt,
             const float* clip_coef, void* stream);
/* ws[1] = prescale * min(max_norm / (||prescale*g|| + 1e-6), 1), ws[2] = the
 * norm (torch clip_grad_norm_ semantics; prescale = 1/world after the RCCL
 * sum).  ws: DV_CLIP_WS_FLOATS floats (per-block partials summed in a fixed
 * order: the result is bit-identical on every rank and run).  max_norm <= 0:
 * no clipping.                                                              */
#define DV_CLIP_WS_FLOATS 516
int dv_grad_clip_coef(const float* g, long long n, float max_norm, float prescale, float* ws,
                      void* stream);

/* ---- low-resolution conditioning (LowresVideoConditioner,
 * dalle2_video.py:1044-1112): resize_video_to (nearest, PyTorch index rule,
 * optional clamp) and the per-frame gaussian_blur2d (reflect padding, odd
 * ks, w1 = normalised 1-D kernel).  planes = B*C*T images, f32.             */
int dv_resize_nearest(const float* x, float* y, long long planes, int hin, int win, int hout,
                      int wout, int do_clamp, float lo, float hi, void* stream);
int dv_gaussian_blur(const float* x, float* y, long long planes, int H, int W, int ks,
                     const float* w1, void* stream);

/* All cross-attention folds of a Unet3D forward in three launches: one job
 * per block, the same arguments as dv_xattn_fold (host-memory table of at
 * most DV_FOLD_MAX jobs, copied into the kernel arguments; graph-safe). */
#define DV_FOLD_MAX 24
typedef struct DvFoldJob {
  const float* wq;
  const float* wo;
  const float* kv;
  const float* null_kv;
  const float* g1;
  float* at;
  float* vt;
  void* Kt;
  void* KtT;
  void* Vt;
  void* VtT;
  float* colsum;
  int nb, C;
} DvFoldJob;
int dv_xattn_fold_batched(int dtype, const DvFoldJob* jobs, int n, float scale, void* stream);

/* Fold gradients of many blocks in four launches: the same pointers and
 * flags as dv_xattn_fold_bwd per job (host table, <= DV_FOLD_BWD_MAX).
 * Run after every job's token reductions (ws_*) are complete.            */
#define DV_FOLD_BWD_MAX 20
typedef struct DvFoldBwdJob {
  float* wsR;
  float* wsV;
  float* wsQ;
  float* mcorr;
  const float* at;
  const float* vt;
  const float* g1;
  const float* wq;
  const float* wo;
  const float* kv;
  const float* null_kv;
  float* dat;
  float* dvt;
  float* dg1;
  float* dg2;
  float* dwq;
  float* dwo;
  float* dkv;
  float* dnull;
  int nb, C, acc_g, acc_w;
} DvFoldBwdJob;
int dv_xattn_fold_bwd_batched(const DvFoldBwdJob* jobs, int n, float scale, void* stream);

/* ---- ResnetBlock3D cross attention (dalle2_video.py:159-162, 192-201;
 * dalle2-pytorch CrossAttention, 8 heads x 64, null kv + 2 time tokens, LN
 * before/after, residual).  Projections fold per clip b into C x 24
 * matrices: dv_xattn_fold computes at/vt [nb][C][24]
 * f32 and the MFMA operand images Kt,VtT [nb][32][Cp], KtT,Vt [nb][Cp][32]
 * (Cp = roundup(C,32)) and colsum [nb][32]; kv [nb][2][1024] f32 is the
 * to_kv projection of the context tokens.                                    */
int dv_xattn_fold(int dtype, const float* wq, const float* wo, const float* kv,
                  const float* null_kv, const float* g1, float* at, float* vt, void* Kt, void* KtT,
                  void* Vt, void* VtT, float* colsum, int nb, int C, float scale, void* stream);
/* out = LN_g2(attn(LN_g1(x))) + x over ntok = nb*P tokens (P per clip, any
 * P; C % 8 == 0).  stats [ntok][4] f32 and pbuf [ntok][32] are saved.       */
int dv_xattn_fwd(int dtype, const void* x, int ldx, void* out, int ldo, long long ntok,
                 long long P, int C, const void* Kt, const void* Vt, const float* colsum,
                 const float* g2, float eps, float* stats, void* pbuf, void* stream);
/* token part of the backward: dx (incl. residual); dobuf [ntok][C], dsbuf
 * and p2buf [ntok][32] feed three dv_gemm_tn_batched reductions.           */
int dv_xattn_bwd_tokens(int dtype, const void* dy, int lddy, const void* x, int ldx, void* dx,
                        int lddx, long long ntok, long long P, int C, const void* KtT,
                        const void* Vt, const void* VtT, const float* colsum, const float* g2,
                        const float* stats, const void* pbuf, void* dobuf, void* dsbuf,
                        void* p2buf, void* stream);
/* parameter part: from the GEMM results wsR/wsV/wsQ [nb][32][C] to
 * dg1, dg2 (acc_g), dwq [512][C], dwo [C][512], dnull [2][64] (acc_w) and
 * dkv [nb][2][1024] (overwritten).  wsR/wsV/wsQ are consumed and left
 * ZEROED, so cached accumulators need no memset before the next call; mcorr
 * [nb][32] is scratch (the LN mean correction, from the row sums of wsR).  */
int dv_xattn_fold_bwd(float* wsR, float* wsV, float* wsQ, float* mcorr,
                      const float* at, const float* vt, const float* g1, const float* wq,
                      const float* wo, const float* kv, const float* null_kv, float* dat,
                      float* dvt, float* dg1, float* dg2, float* dwq, float* dwo, float* dkv,
                      float* dnull, int nb, int C, float scale, int acc_g, int acc_w,
                      void* stream);

/* ---- mid self-attention (Unet3D.mid_attn = Residual(Attention(mid_dim)),
 * dalle2_video.py:431, 551, 921-922; dalle2-pytorch Attention: 16 heads x 32,
 * ONE shared k/v head (multi-query), learned null k/v at key 0, q scaled
 * twice by 32^-0.5 with cosine-sim off -> logit factor 1/32).
 * prep: kv [B][N][*] (k at 0, v at 32, stride ldkv) -> kp/vp [B][NKP][32]
 * (row 0 null, rows > N zero; NKP = roundup(N+1, 32)).  `scale` is the
 * logit factor later passed to dv_mqa_fwd / dv_mqa_bwd: on the bf16 path kp
 * holds k * scale * log2(e) (the MFMA then yields the logit in log2 units);
 * f32 kp holds k.  kmax (bf16 path, may be NULL): B * ceil(NKP / 64) floats,
 * receives the largest |k * scale * log2(e)| of every 64-key block, the
 * bound dv_mqa_fwd uses to drop the running max when |q| max|k| <= 64.     */
int dv_mqa_prep(int dtype, const void* kv, int ldkv, const float* null_kv, void* kp, void* vp,
                int B, int N, int NKP, float scale, float* kmax, void* stream);
/* o[b][n][h*32+d] = softmax_j(scale * q.k_j) v_j; lse f32 saved (opaque to the
 * caller, B*H*N floats: [B][N*H] log2 units on the bf16 path, [B][H][N]
 * natural-log otherwise).  bf16 needs dense rows (ldq == ldo == H*32): NKP
 * <= 1280 runs the whole-clip-K/V-in-LDS kernel, longer clips the K/V-
 * streamed one.  kmax: dv_mqa_prep's key-norm blocks (NULL: every wave
 * keeps the online running max).                                           */
int dv_mqa_fwd(int dtype, const void* q, int ldq, const void* kp, const void* vp, void* o, int ldo,
               float* lse, int B, int N, int NKP, int H, float scale, const float* kmax, void* stream);
/* MX-fp8 PV forward (BASELINE config 5 sampling; forward only): the
 * K/V-streamed forward with O^T += V^T P^T on the block-scaled
 * v_mfma_scale_f32_32x32x64_f8f6f4 (e4m3 P and V, an e8m0 scale per 32 keys;
 * QK^T stays bf16).  kp / vp: dv_mqa_prep's bf16 images; v8 (>=
 * dv_mqa_fwd_fp8_ws bytes) receives V's fp8 image; o / lse as dv_mqa_fwd's
 * streamed bf16 path (dense rows, lse [B][N*H] log2 units).                 */
int dv_mqa_fwd_fp8_ws(int B, int NKP, long long* bytes);
int dv_mqa_fwd_fp8(const void* q, int ldq, const void* kp, const void* vp, void* v8, long long v8_bytes,
                   void* o, int ldo, float* lse, int B, int N, int NKP, int H, void* stream);
/* f32 scratch dv_mqa_bwd needs (floats); same path choice as dv_mqa_fwd.     */
int dv_mqa_bwd_ws(int dtype, int ldq, int ldo, int B, int N, int NKP, int H, long long* floats);
/* dq, dkv (k at 0, v at 32, stride lddkv) and dnull (+)= (accumulate);
 * D (B*H*N floats) and ws (>= dv_mqa_bwd_ws floats, no zeroing needed) are
 * scratch.  bf16 path (NKP <= 1280): dq (query-major) writes D, dk/dv
 * (key-major) writes per-slice partials to ws, a finish launch sums them.   */
int dv_mqa_bwd(int dtype, const void* q, int ldq, const void* o, int ldo, const void* dout,
               int lddo, const float* lse, const void* kp, const void* vp, void* dq, int lddq,
               float* D, float* ws, long long ws_floats, void* dkv, int lddkv, float* dnull, int B,
               int N, int NKP, int H, float scale, int accumulate, void* stream);

/* ---- gradient exchange over RCCL (xGMI) -----------------------------------
 * Replaces the bucket all-reduces DDP issues from its gradient hooks inside
 * accelerator.backward (reference trainer.py:360; accelerate wraps the
 * decoder in DistributedDataParallel at trainer.py:117-124).  One process per
 * GPU; the communicator belongs to this library, so a collective enqueued
 * inside a HIP-graph capture has no host-side work object that another thread
 * could poll.  RCCL is resolved at run time (the instance torch loaded, else
 * /opt/rocm/lib); without it these return DV_ERR_UNSUPPORTED.
 * unique_id: 128 opaque bytes made on one rank and handed to every rank
 * (the trainer uses the torch.distributed store).  init: blocking, every rank
 * at once, on `device`.  allreduce: in place on `stream`, `average` != 0 ->
 * mean over ranks (idempotent on data every rank already holds, as DDP's
 * averaged buckets are), else sum.  async_error: DV_OK while the
 * communicator is healthy (pollable from any thread: the trainer's
 * watchdog).  destroy: after the last collective completed; abort: frees it
 * without waiting for outstanding work (a dead peer).                        */
int dv_comm_unique_id(void* id_out);
int dv_comm_init(const void* id, int nranks, int rank, int device, void** comm_out);
int dv_comm_allreduce(void* comm, void* buf, long long count, int dtype, int average, void* stream);
int dv_comm_async_error(void* comm);
int dv_comm_destroy(void* comm);
int dv_comm_abort(void* comm);

#ifdef __cplusplus
}
#endif
#endif /* DV_HIP_H */
