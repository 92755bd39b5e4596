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
enum { DV_ACT_NONE = 0, DV_ACT_SILU = 1 };

const char* dv_last_error(void);
int dv_abi_version(void);

/* ---- convolutions (1,k,k), stride 1, padding k//2 -------------------------
 * Replaces nn.Conv3d in Block3D.project (dalle2_video.py:107), res_conv
 * (:170), Downsample3D (:25), the stage-3 projection (:537),
 * PixelShuffleUpsample3D.conv (:48), CrossEmbedLayer3D (:224-232) and to_out
 * (:637); also every bias-free nn.Linear over tokens (k=1).
 * Implicit GEMM on MFMA: M = nf*h*w pixels, N = cout, K = k*k*cin.
 * Input channels [0,c0) come from x0 (stride ld0), [c0,cin) from x1 (ld1);
 * c0 must be a multiple of 8 (pass c0=cin, x1=NULL for one source).
 * wpack: packed weight [cout][k*k][cin] of `dtype` (dv_pack_conv_weight).
 * Epilogue: y = act(acc + bias) + res.  cin % 8 == 0 required.            */
int dv_conv_fwd(int dtype, const void* x0, int ld0, int c0, const void* x1, int ld1,
                const void* wpack, const float* bias, const void* res, int ldres,
                void* y, int ldy, int nf, int h, int w, int cin, int cout, int ksize,
                int act, void* stream);

/* ws[co][tap][ci] += sum_pixels dY[p][co] * X[p + tap][ci]: f32 atomics into a
 * zeroed packed workspace (cout*k*k*cin floats; for k=1 this IS the torch
 * layout, so ws may be the parameter's gradient); split-K over pixels.
 * db (optional): db[co] += sum_p dY[p][co] — the conv bias gradient, fused.
 * cin, cout multiples of 8 (pad and mask with dv_unpack_wgrad).            */
int dv_conv_wgrad(int dtype, const void* dy, int lddy, const void* x0, int ld0, int c0,
                  const void* x1, int ld1, float* ws, float* db, int nf, int h, int w, int cin,
                  int cout, int ksize, void* stream);

/* dw (torch layout (cout_real, cin_real, 1, k, k)) (+)= ws[co][tap][ci]; zeroes
 * ws behind itself so a cached workspace needs no memset before reuse.       */
int dv_unpack_wgrad(float* ws, float* dw, int cout, int cin, int ksize, int cout_real,
                    int cin_real, int accumulate, void* stream);

/* db[c] += sum_p dy[p][c]  (f32 atomics) */
int dv_bias_grad(int dtype, const void* dy, int lddy, float* db, long long npix, int c,
                 void* stream);

/* f32 torch weight (cout, cin, 1, k, k) -> packed `dtype`
 *   mode 0 (forward):  out[co][tap][ci_pad]          (ci >= cin zero)
 *   mode 1 (dgrad):    out[ci][tap'][co_pad] = w[co][ci][k*k-1-tap']      */
int dv_pack_conv_weight(int dtype, const float* w, void* out, int cout, int cin, int ksize,
                        int pad_to, int mode, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* DV_HIP_H */
