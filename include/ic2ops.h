/*
 * ic2ops.h -- C ABI of libic2ops.so, the MI355X (gfx950) kernels behind the encode -> quantize ->
 * synthesize path of yubster4525/image_compression_2 (reference snapshot mounted at /root/reference).
 *
 * Conventions (every entry point):
 *   - all tensor pointers are DEVICE pointers owned by the caller (PyTorch's caching allocator);
 *     nothing is allocated, freed or synchronised inside -> every call is hipGraph-capturable;
 *   - work is enqueued on `stream` (a hipStream_t passed as void*; NULL = the legacy default stream);
 *   - return IC2_OK (0) or an IC2_E_* code; ic2_last_error() returns the thread-local message;
 *   - dtype codes: IC2_F32 = 0, IC2_BF16 = 1, IC2_F16 = 2 (f16 only where an entry point says so).  Activations on the synthesis path are NHWC with a
 *     channel stride padded to a multiple of 32 ("c_p"); padded channels hold zeros.
 *   - IC2_BF16X3 = 3 (split bf16, only where an entry point says so): an f32 value v stored as hi = bf16(v),
 *     lo = bf16(v - hi).  An NHWC activation of logical stride c_p is laid out as 2 * c_p bf16 channels per pixel,
 *     [hi | lo] (round 3: [hi | hi | lo]); a packed weight as [cout_p][kh][kw][3 * cin_p] = [hi | lo | hi].  The
 *     conv entry points take such an input with dtype IC2_BF16X3 and cin_p' = 3 * cin_p: the GEMM's K runs over
 *     [hi | hi | lo] (the hi block read twice) and accumulates x_hi*w_hi + x_hi*w_lo + x_lo*w_hi in f32: the product
 *     to ~2^-16 relative (the dropped x_lo*w_lo term is ~2^-18) at three bf16 MFMAs -- the encoder's parity mode that
 *     keeps the 8-bit latent indices of the fp32 reference.
 *   - IC2_F16X2 = 4 (split weights, f16 input, only where an entry point says so): the activation is plain f16 NHWC
 *     (stride c_p), a packed weight [cout_p][kh][kw][2 * cin_p] f16 = [hi | lo] (lo = f16(w - hi)).  Conv entry
 *     points take it with cin_p' = 2 * cin_p: K runs over [x | x] and accumulates x*w_hi + x*w_lo in f32 (two f16
 *     MFMAs; the activation to 2^-11, the weight to ~2^-22).  The split encoder's first blocks.
 *
 * The reference has no native code and no C ABI: each entry point names the Python
 * function of the reference (or of the un-vendored NVlabs/stylegan3 ops it calls) that it replaces.
 */
#ifndef IC2OPS_H_
#define IC2OPS_H_

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { IC2_OK = 0, IC2_E_INVALID = 1, IC2_E_UNSUPPORTED = 2, IC2_E_LAUNCH = 3 };
enum { IC2_F32 = 0, IC2_BF16 = 1, IC2_F16 = 2, IC2_BF16X3 = 3, IC2_F16X2 = 4,
       /* an out_dtype of ic2_conv_igemm / ic2_conv_igemm_ws / ic2_conv_wino only: f16 output converted IEEE (an
        * overflow stores +-inf instead of saturating at +-65504) -- the gradient convs of the f16 training path, so a
        * loss-scaled gradient that overflows reaches the GradScaler as inf (the reference's fp16 autocast behaviour,
        * stylegan3_hvae_full.py:693-696) */
       IC2_F16_IEEE = 5 };
enum { IC2_ACT_LINEAR = 0, IC2_ACT_LRELU = 1 };
/* NHWC16: channel-blocked NHWC, [n][c_p / 16][h][w][16] (the synthesis conv -> fused filtered lrelu hand-off) */
enum { IC2_LAYOUT_NHWC = 0, IC2_LAYOUT_NCHW = 1, IC2_LAYOUT_NHWC16 = 2 };

const char* ic2_last_error(void);
int ic2_abi_version(void);

/* ---------------------------------------------------------------- quantizers (HBM-bound) ---- */

/* StyleGAN3Compressor.compress quantizer, stylegan3_hvae_full.py:313-316:
 *   q = round(((w + 1) * 0.5) * S) / S * 2 - 1,  S = 2^bits - 1, fp32 in the written op order,
 *   round half-to-even, no clamp.  idx_out (nullable) = the integer numerator round(((w+1)*0.5)*S). */
int ic2_quantize_uniform(const float* w, int64_t n, int bits, float* q_out, int32_t* idx_out, void* stream);

/* GumbelSoftmaxDiscretization.forward index path, gumbel_softmax_compression.py:93-118:
 *   idx = argmin_k |z - codebook[k]| (exact fp32 distances, first index on ties).
 *   zq_out (nullable) = codebook[idx] (the hard code, :258); hist_out (nullable, k counters, zeroed
 *   by the caller) = code usage histogram (:121-123, feeds the perplexity :126-127). */
int ic2_quantize_codebook_argmin(const float* z, int64_t n, const float* codebook, int k, int64_t* idx_out,
                                 float* zq_out, uint32_t* hist_out, void* stream);

/* GumbelSoftmaxCompressor.decompress lookup, gumbel_softmax_compression.py:255-259:
 *   w = codebook[codes].  Out-of-range codes set *oob_flag (device int, zeroed by caller) and write 0. */
int ic2_codebook_lookup(const int64_t* codes, int64_t n, const float* codebook, int k, float* w_out,
                        int32_t* oob_flag, void* stream);

/* GumbelSoftmaxDiscretization.forward, gumbel_softmax_compression.py:73-129, fused per latent:
 *   y = (-|z - codebook| + gumbel) / tau;  soft = softmax(y);  ret = hard ? onehot(argmax) - soft + soft : soft;
 *   disc_out = ret @ codebook;  idx_out (nullable) = exact argmin |z - c| (first index);
 *   prob_sum_out (nullable, k floats, zeroed by caller) += column sums of ret (-> perplexity).
 * tau = exp(*log_tau) when log_tau (device) is non-NULL, else `tau`.  Noise: gumbel_noise (device
 * [n][k], nullable) or an in-kernel Philox4x32-10 stream keyed by (seed, offset + i*k + j). k <= 1024. */
int ic2_gumbel_softmax_quantize(const float* z, int64_t n, const float* codebook, int k, const float* log_tau,
                                float tau, int hard, uint64_t seed, uint64_t offset, const float* gumbel_noise,
                                float* disc_out, int64_t* idx_out, float* prob_sum_out, void* stream);
/* The same with the Philox seed read from device memory (*seed_dev, e.g. a torch.randint drawn on the device
 * generator as F.gumbel_softmax draws its noise on the tensor's device, gumbel_softmax_compression.py:103-108): no
 * host sync, and the CPU generator -- which the reference's fine projector re-creates fc1 from on every call,
 * stylegan3_hvae_full.py:225-230 -- is left untouched. */
int ic2_gumbel_softmax_quantize_dseed(const float* z, int64_t n, const float* codebook, int k, const float* log_tau,
                                      float tau, int hard, const int64_t* seed_dev, uint64_t offset,
                                      const float* gumbel_noise, float* disc_out, int64_t* idx_out,
                                      float* prob_sum_out, void* stream);

/* Per-batch code record (SURVEY.md 8e metric record; usage / perplexity over the batch,
 * gumbel_softmax_compression.py:121-127): kind 0 = f32 latents from ic2_quantize_uniform at `bits` (code =
 * round((q + 1) * 0.5 * (2^bits - 1)), k = 2^bits), kind 1 = int64 codebook indices (k codes).  counts uint32 [k + 2],
 * zeroed by the caller: += hist[0 .. k), codes outside [0, k) in counts[k], elements differing from golden (nullable,
 * same kind; bitwise for kind 0) in counts[k + 1]. */
int ic2_code_record(const void* codes, int kind, int k, int bits, const void* golden, int64_t n, uint32_t* counts,
                    void* stream);

/* ------------------------------------------- StyleGAN3 ops (torch_utils/ops, NVlabs/stylegan3) ---- */

/* bias_act.bias_act(x, b, dim, act, alpha, gain, clamp) [SG3-public]; x viewed as [outer, c, inner],
 * bias along c.  act: IC2_ACT_LINEAR / IC2_ACT_LRELU.  clamp < 0 = none. */
int ic2_bias_act(const void* x, const float* b, void* y, int dtype, int64_t outer, int64_t c, int64_t inner,
                 int act, float alpha, float gain, float clamp, void* stream);

/* upfirdn2d.upfirdn2d(x, f, up, down, padding, flip_filter, gain) [SG3-public] on NCHW (nc planes).
 * f (DEVICE pointer, f32): f_ndim = 1: separable f[f_w] (each pass scaled by sqrt(gain));
 * f_ndim = 2: f[f_h][f_w] (scaled by gain).
 * f == NULL: identity 1x1 filter.  Output size must be
 *   out = (in*up + pad0 + pad1 - (taps-1)) / down  (ceil of the strided slice, as the ref computes). */
int ic2_upfirdn2d(const void* x, void* y, int dtype, int64_t nc, int in_h, int in_w, int out_h, int out_w,
                  const float* f, int f_ndim, int f_h, int f_w, int up_x, int up_y, int down_x, int down_y,
                  int px0, int px1, int py0, int py1, int flip, float gain, void* stream);

/* filtered_lrelu.filtered_lrelu(x, fu, fd, b, up, down, padding, gain, slope, clamp, flip_filter)
 * [SG3-public] on NCHW, one fused launch: bias -> zero-insert up -> FIR fu (gain up^2) -> lrelu*gain ->
 * clamp -> FIR fd -> keep every down-th.  fu/fd are 1-D separable taps in HOST memory (layer constants,
 * passed by value in the kernel arguments; NULL = identity), b is a device pointer.
 * Returns IC2_E_UNSUPPORTED for (up, down, taps) combinations without a fused instance; the caller
 * then composes ic2_bias_act + ic2_upfirdn2d. */
int ic2_filtered_lrelu(const void* x, void* y, int dtype, int64_t n, int64_t c, int in_h, int in_w, int out_h,
                       int out_w, const float* fu, int fu_taps, const float* fd, int fd_taps, const float* b,
                       int up, int down, int px0, int px1, int py0, int py1, float gain, float slope,
                       float clamp, int flip, void* stream);

/* The synthesis-path variant of the same fused op: NHWC in/out with padded channel stride c_p,
 * bias already folded into the producer (b may be NULL), and an optional per-(sample, channel)
 * post_scale [n][c_p] (the NEXT layer's modulation, see ic2_modconv_prep) applied to the output.
 * bf16 -> bf16 and the SG3-T configurations (up 2/4 with 6*up taps, down 2 with 12) run on MFMA with f16
 * operands; dtype_in may then also be IC2_F16 (the conv epilogue's f16 output). */
int ic2_flrelu_nhwc(const void* x, void* y, int dtype_in, int dtype_out, int n, int c_p, int in_h, int in_w,
                    int out_h, int out_w, const float* fu, int fu_taps, const float* fd, int fd_taps, const float* b,
                    int up, int down, int px0, int px1, int py0, int py1, float gain, float slope, float clamp,
                    int flip, const float* post_scale, void* stream);

/* ic2_flrelu_nhwc with the input in the channel-blocked layout IC2_LAYOUT_NHWC16 ([n][c_p/16][in_h][in_w][16],
 * f16 or bf16: what ic2_conv_igemm writes with out_layout 2), output plain NHWC bf16.  Each 16-channel tile of the
 * fused kernel then reads contiguous rows instead of 32 B out of every c_p*2-byte pixel.  Same semantics as
 * ic2_flrelu_nhwc (SynthesisLayer's filtered_lrelu, SG3-public; called at stylegan3_hvae_full.py:274,329);
 * configurations without an MFMA instance return IC2_E_UNSUPPORTED. */
int ic2_flrelu_nhwc16(const void* x, void* y, int dtype_in, int dtype_out, int n, int c_p, int in_h, int in_w,
                      int out_h, int out_w, const float* fu, int fu_taps, const float* fd, int fd_taps, const float* b,
                      int up, int down, int px0, int px1, int py0, int py1, float gain, float slope, float clamp,
                      int flip, const float* post_scale, void* stream);

/* ----------------------------------------------------------------- modulated conv (MFMA) ---- */

/* FullyConnectedLayer.forward [SG3-public] and nn.Linear (stylegan3_hvae_full.py:206-234):
 *   y[n][o] = act((sum_i x[n*ldx + i] * w[o][i]) * w_gain + b[o] * b_gain) * act_gain   (fp32). */
int ic2_fc(const float* x, int64_t ldx, const float* w, const float* b, float* y, int n, int in_f, int out_f,
           float w_gain, float b_gain, int act, float alpha, float act_gain, void* stream);

/* Weight packing for the implicit GEMM: w[cout][cin][kh][kw] f32 -> w_out[cout_p][kh][kw][cin_p]
 * (dtype) times `scale`, zero padded; dtype IC2_BF16X3 -> w_out[cout_p][kh][kw][3 * cin_p] bf16 = [hi | lo | hi],
 * IC2_F16X2 -> w_out[cout_p][kh][kw][2 * cin_p] f16 = [hi | lo].
 * prenorm != 0 applies modulated_conv2d's w * rsqrt(mean(w^2,[1,2,3]))
 * and writes wsq_out[cout][cin] = sum_k w_norm^2 (nullable).  Called once per weight version. */
int ic2_pack_weight(const float* w, int cout, int cin, int kh, int kw, int cout_p, int cin_p, int prenorm,
                    float scale, void* w_out, int dtype, float* wsq_out, void* stream);

/* The dgrad pack of the same weight (training; replaces ic2_pack_weight on w.transpose(0, 1).flip(2, 3)):
 * w[cout][cin][kh][kw] f32 -> w_out[cin_p][kh][kw][cout_p] (IC2_F32 / IC2_BF16 / IC2_F16), w_out[ci][ky][kx][co] =
 * w[co][ci][kh-1-ky][kw-1-kx], zero padded.  The forward conv (ic2_conv_igemm) on it with padding k - 1 - pad is the
 * adjoint of nn.Conv2d's. */
int ic2_pack_weight_adjoint(const float* w, int cout, int cin, int kh, int kw, int cin_p, int cout_p, void* w_out,
                            int dtype, void* stream);

/* modulated_conv2d's modulation/demodulation coefficients [SG3-public], as the equivalent
 * activation-scaling form y[n,o] = oscale[n,o] * sum_{i,k} w_norm[o,i,k] * (xscale[n,i] * x[n,i]):
 *   demod:  s' = s * rsqrt(mean(s^2)) (batch-global), xscale = s',
 *           oscale = input_gain * rsqrt(sum_i s'^2 * wsq[o][i] + 1e-8);
 *   !demod: xscale = s * style_gain, oscale = input_gain.
 * styles [n][cin] f32; xscale_out [n][cin_p]; oscale_out [n][cout_p]; scratch: unused (may be NULL). */
int ic2_modconv_prep(const float* styles, const float* wsq, int n, int cin, int cout, int cin_p, int cout_p,
                     int demod, float style_gain, float input_gain, float* xscale_out, float* oscale_out,
                     float* scratch, void* stream);

/* Every synthesis layer's affine FC + ic2_modconv_prep in three launches (bit-identical to ic2_fc followed by
 * ic2_modconv_prep per layer).  ws [n][ldx] f32 (the broadcast ws rows); layers: nl <= 20 records of 16 int64:
 *   {aw, ab, wsq, styles, xscale_out, oscale_out, ws_off, cin, cin_p, cout, cout_p, demod,
 *    w_gain, b_gain, style_gain, input_gain}
 * pointers as integers (device memory; styles [n][cin] is scratch), the four gains as the float's bit pattern.
 * Layer l's FC reads ws[row][ws_off .. ws_off + w_dim).  Replaces the per-layer affine + modulation of
 * SynthesisLayer.forward [SG3-public] at the call site SynthesisNetwork.forward (stylegan3_hvae_full.py:274,329). */
int ic2_modconv_prep_batched(const float* ws, int64_t ldx, int n, int w_dim, int nl, const int64_t* layers,
                             void* stream);

/* The kernel instance(s) ic2_conv_igemm_ws launches for a geometry (its launch plan; host-only, no GPU needed),
 * e.g. "igemm8_og2", "hg4_o128_w32_p2", "hconv_64_64", "torgb", "igemm_128x128_splitk".  Static storage. */
const char* ic2_conv_plan(int dtype, int out_dtype, int out_layout, int n, int h, int w, int cin_p, int cout_p,
                          int cout_valid, int kh, int kw, int pad);

/* Non-zero when IC2_DEV=1: the development knobs (forced kernel instances, A/B switches; IC2_HG4, IC2_IGEMM_TILE,
 * ...) are read from the environment only then -- otherwise the launch plan never depends on it. */
int ic2_dev_mode(void);

/* NHWC implicit-GEMM convolution on MFMA (bf16: v_mfma_f32_16x16x32_bf16, f32: v_mfma_f32_16x16x4_f32):
 *   acc[n,p,o] = sum_{ky,kx,i} w[o][ky][kx][i] * x[n, p + (ky,kx) - pad, i]   (zero outside the image)
 *   v = acc * (oscale ? oscale[n][o] : 1) + (bias ? bias[o] : 0);  if act: v = clamp(lrelu(v)*act_gain)
 *   y = v * out_mul  -> NHWC [n][ho][wo][cout_p] (layout 0), NCHW f32 [n][cout_valid][ho][wo] (layout 1) or
 *   channel-blocked NHWC16 [n][cout_p/16][ho][wo][16] (layout 2, any out dtype).
 * Replaces the grouped conv2d of modulated_conv2d [SG3-public] and nn.Conv2d of VGGBlock
 * (stylegan3_hvae_full.py:175-176) / from_rgb (:62).  cin_p, cout_p multiples of 32.  dtype IC2_BF16X3: the
 * split-bf16 input stored [hi | lo] (2/3 * cin_p channels per pixel), cin_p = the tripled K channel count (a multiple
 * of 96), weights from ic2_pack_weight(IC2_BF16X3), NHWC output.  dtype IC2_F16X2: the f16 input (cin_p / 2 channels
 * per pixel), cin_p = the doubled K channel count (a multiple of 64), weights from ic2_pack_weight(IC2_F16X2), NHWC
 * output. */
int ic2_conv_igemm(const void* x, const void* w, void* y, int dtype, int out_dtype, int n, int h, int w_,
                   int cin_p, int cout_p, int cout_valid, int kh, int kw, int pad, int ho, int wo,
                   const float* oscale, const float* bias, int act, float slope, float act_gain, float clamp,
                   float out_mul, int out_layout, void* stream);

/* ic2_conv_igemm with a caller-owned f32 workspace for split-K.  Launches that would not fill the
 * chip (the encoder's 16^2 .. 2^2 blocks) split the K reduction over up to 32 slices; each slice
 * writes f32 partial sums to the workspace and a second kernel adds them in slice order
 * (deterministic) and applies the epilogue.  ws_bytes below the size ic2_conv_igemm_ws_bytes
 * returns for the same geometry (0 = no split) runs unsplit.  Same contract otherwise. */
int64_t ic2_conv_igemm_ws_bytes(int dtype, int n, int h, int w_, int cin_p, int cout_p, int kh, int kw, int pad);
int ic2_conv_igemm_ws(const void* x, const void* w, void* y, int dtype, int out_dtype, int n, int h, int w_,
                      int cin_p, int cout_p, int cout_valid, int kh, int kw, int pad, int ho, int wo,
                      const float* oscale, const float* bias, int act, float slope, float act_gain, float clamp,
                      float out_mul, int out_layout, void* workspace, int64_t ws_bytes, void* stream);

/* Winograd F(2,3)-along-x weights for ic2_conv_wino: w[cout][cin][3][3] f32 -> u_out[cout_p][3][4][cin_p] (f16),
 * U[o][ky][nu][c] = (G w[o][c][ky][:])[nu] * scale (times rsqrt(mean(w^2,[1,2,3])) when prenorm, as
 * ic2_pack_weight), G = [1 0 0; .5 .5 .5; .5 -.5 .5; 0 0 1], zero padded.  Once per weight version. */
int ic2_pack_weight_wino(const float* w, int cout, int cin, int cout_p, int cin_p, int prenorm, float scale,
                         void* u_out, int dtype, void* stream);

/* The 3x3 convolution of ic2_conv_igemm (same output / epilogue contract, kh = kw = 3, f16 operands) as a fused
 * Winograd F(2,3) along x on MFMA: 2/3 of the direct conv's MFMA work; x NHWC f16 [n][h][w][cin_p], u from
 * ic2_pack_weight_wino.  Replaces the grouped conv2d of modulated_conv2d [SG3-public] on the f16 synthesis path
 * (stylegan3_hvae_full.py:274,329).  f16 rounding of the transformed input: tools/wino_emu.py. */
int ic2_conv_wino(const void* x, const void* u, void* y, int dtype, int out_dtype, int n, int h, int w_, int cin_p,
                  int cout_p, int cout_valid, int pad, int ho, int wo, const float* oscale, const float* bias, int act,
                  float slope, float act_gain, float clamp, float out_mul, int out_layout, void* stream);

/* 1 when the library's launch plan runs this 3x3 conv as ic2_conv_wino (f16 operands, a geometry where it beats the
 * direct implicit GEMM), else 0.  Host only. */
int ic2_conv_wino_preferred(int dtype, int n, int h, int w_, int cin_p, int cout_p, int kh, int kw, int pad);

/* Diagnostic builds only (IC2_WX_STAMP, tools/build_abl.sh winostamp): a device buffer for ic2_conv_wino's per-wave
 * section timestamps (u64 [blocks][8 waves][8]); IC2_E_INVALID in the product build. */
int ic2_conv_wino_stamps(void* buf, int64_t bytes);

/* ic2_conv_wino's launch plan for a geometry, e.g. "wino_fx_o128_p15x8_f16" (tile: 15 pairs x 8 rows).  Host only. */
const char* ic2_conv_wino_plan(int n, int h, int w_, int cin_p, int cout_p, int pad);

/* SynthesisInput.forward Fourier features [SG3-public]: t [n][4] = affine(w); per sample the
 * rotation/translation of freqs/phases, the amplitude damping and sin(2*pi*(grid.f + phi)) * amp on a
 * size x size grid -> x_out NHWC [n][size][size][c_p].  (The trailing @ W/sqrt(C) is an ic2_conv_igemm.) */
int ic2_synth_input_features(const float* t, const float* freqs, const float* phases, const float* transform,
                             int n, int c, int c_p, int size, float sampling_rate, float bandwidth, void* x_out,
                             int dtype, void* stream);

/* ------------------------------------------------------------------ encoder (HVAE_VGG) ---- */

/* NCHW f32 -> NHWC (dtype) with channel stride c_p (zero padded), optionally times scale[n][c_p]
 * (nullable; a modulated layer's input scaling); the encoder's input packing.  dtype IC2_BF16X3: 2 * c_p channels. */
/* HVAE_VGG_Encoder.from_rgb (nn.Conv2d(cin, cout, 3, padding=1), stylegan3_hvae_full.py:62,175) read straight
 * from the NCHW f32 image: x [n][cin][h][w] f32 (cin <= 4, rounded to bf16 as ic2_nchw_to_nhwc does), w packed
 * bf16 [cout_p][3][3][cin_p] (ic2_pack_weight), bias [cout_p] f32 -> y bf16 NHWC [n][h][w][cout_p], cout_p in
 * {32, 64}.  Equals ic2_nchw_to_nhwc + ic2_conv_igemm (bf16) up to f32 summation order. */
int ic2_from_rgb_conv(const float* x, int cin, const void* w, int cin_p, const float* bias, void* y, int n, int h,
                      int w_, int cout_p, void* stream);

/* The same from_rgb in the encoder's split-bf16 mode: x f32 NCHW (not rounded), w the nn.Conv2d weight as is
 * (f32 [cout][cin][3][3]), bias [cout_p] f32; exact f32 FMAs (tap order) -> y IC2_BF16X3 NHWC [n][h][w][2 * cout_p]
 * ([hi | lo], the input layout of the next split-bf16 conv).  cin <= 4, cout <= cout_p, cout_p in {32, 64, 128}. */
int ic2_from_rgb_conv_x3(const float* x, int cin, const float* w, int cout, const float* bias, void* y, int n, int h,
                         int w_, int cout_p, void* stream);
/* The same exact-f32 from_rgb with the result rounded once to f16 -> y NHWC f16 [n][h][w][cout_p]: the input of an
 * IC2_F16X2 conv (the split encoder's first block).  cout_p in {32, 64, 128}. */
int ic2_from_rgb_conv_f16(const float* x, int cin, const float* w, int cout, const float* bias, void* y, int n, int h,
                          int w_, int cout_p, void* stream);

int ic2_nchw_to_nhwc(const float* x, void* y, int dtype, int n, int c, int h, int w, int c_p, const float* scale,
                     void* stream);

/* NHWC (dtype, channel stride c_p) -> NCHW f32 with c channels (layer-level API outputs). */
int ic2_nhwc_to_nchw(const void* x, int dtype, float* y, int n, int c, int h, int w, int c_p, void* stream);

/* nn.GroupNorm statistics (stylegan3_hvae_full.py:179-180; eps 1e-5): per (n, group) mean and
 * rstd = 1/sqrt(var + eps) over (channels of the group) x H x W of the NHWC tensor y.
 * stats_out [n][groups][2] f32, followed by scratch: ic2_group_norm_stats_floats() floats in total.
 * Two-level deterministic reduction (no atomics). */
int64_t ic2_group_norm_stats_floats(int n, int hw, int groups);
int ic2_group_norm_stats(const void* y, int dtype, int n, int hw, int c_p, int c, int groups, float eps,
                         float* stats_out, void* stream);

/* GroupNorm apply + F.leaky_relu(0.2) (+ AvgPool2d(2,2) when pool != 0), VGGBlock.forward :183-191:
 *   out = pool(lrelu((y - mean) * rstd * gamma[c] + beta[c]))  NHWC -> NHWC (floor pooling).  dtype_out may be
 *   IC2_BF16X3 (f32 arithmetic, then split: out [n][oh][ow][2 * c_p]), also from dtype_in IC2_F16 (an IC2_F16X2
 *   conv's output); dtype_out IC2_F16 is the input of an IC2_F16X2 conv. */
int ic2_gn_lrelu_pool(const void* y, void* out, int dtype_in, int dtype_out, int n, int h, int w, int c_p, int c,
                      int groups, const float* stats, const float* gamma, const float* beta, float slope,
                      int pool, void* stream);

/* AdaptiveAvgPool2d(1) of HierarchyProjector (:218): out [n][c] f32 = mean over H x W (NHWC input; dtype
 * IC2_BF16X3 sums hi + lo); `out` is followed by scratch: ic2_global_avg_pool_floats() floats in total. */
int64_t ic2_global_avg_pool_floats(int n, int hw, int c_p, int c);
int ic2_global_avg_pool(const void* x, int dtype, int n, int hw, int c_p, int c, float* out, void* stream);

/* HierarchyProjector tail (:237-245): params [n][num_ws][2*w_dim] -> mean, logvar (chunk), and
 * w = mean + eps * exp(0.5*logvar) (eps nullable -> w = mean).  Outputs written at slot offset
 * ws_off of [n][ws_total][w_dim] tensors (the torch.cat of :163-165 done in place). */
int ic2_reparameterize(const float* params, const float* eps, int n, int num_ws, int w_dim, int ws_total,
                       int ws_off, float* w_out, float* mean_out, float* logvar_out, void* stream);

/* ------------------------------------------------------------------------------ metrics ---- */

/* PSNR support (hvae_training.py:368-388 uint8 conversion): per image sum of squared differences of
 * trunc(clamp(v*0.5+0.5,0,1)*255) between two NCHW f32 batches -> sse_out [n_img] (f64).
 * scratch: ic2_uint8_sse_scratch_doubles(n_img) doubles (per-chunk partials; deterministic). */
int64_t ic2_uint8_sse_scratch_doubles(int64_t n_img);
int ic2_uint8_sse(const float* a, const float* b, int64_t n_img, int64_t per_img, double* sse_out, double* scratch,
                  void* stream);

/* F.interpolate(mode='bilinear', align_corners=False, no antialias) of StyleGAN3Compressor.forward
 * (stylegan3_hvae_full.py:277-279), NCHW f32. */
int ic2_resize_bilinear(const float* x, float* y, int64_t nc, int h, int w, int oh, int ow, void* stream);

/* ---- entropy coding of the codebook indices (HOST pointers; no GPU) ----------------------------------------
 * Replaces the reference's CABAC stage (cabac_compression.py:60-406: ContextModel, ArithmeticCoder,
 * cabac_encode / cabac_decode; non-functional there) with a context-adaptive binary range coder:
 * bit-tree binarisation, contexts = (previous symbol in the w vector, same position in the previous w vector).
 * codes: int32 [n_streams][num_ws][w_dim], each in [0, n_symbols); one independent byte stream per image,
 * concatenated into out; stream_bytes[n_streams] receives the sizes.  n_threads <= 0: hardware concurrency
 * (capped at 16).  ic2_rc_bound gives a sufficient out_cap. */
int64_t ic2_rc_bound(int64_t n_streams, int64_t per_stream);
int ic2_rc_encode(const int32_t* codes, int64_t n_streams, int num_ws, int w_dim, int n_symbols, uint8_t* out,
                  int64_t out_cap, int64_t* stream_bytes, int n_threads);
int ic2_rc_decode(const uint8_t* in, const int64_t* stream_bytes, int64_t n_streams, int num_ws, int w_dim,
                  int n_symbols, int32_t* codes_out, int n_threads);

/* ---- training path (BASELINE C5; the reference's train_hvae_encoder backward, stylegan3_hvae_full.py:693-696:
 * torch autograd through HVAE_VGG_Encoder).  The conv input gradient is ic2_conv_igemm on flipped / transposed
 * weights; these are the remaining encoder backward ops. ---- */

/* nn.Conv2d weight gradient (VGGBlock.conv1/conv2, from_rgb: :62, :175-176): dw [cout_p][kh][kw][cin_p] f32 =
 * sum over output pixels of dy[p][o] * x[p shifted by the tap][i]; x NHWC [n][h][w][cin_p], dy NHWC
 * [n][ho][wo][cout_p] (dtype f32 / bf16, channel strides multiples of 32), stride 1, zero padding `pad`.
 * Workspace: ic2_conv_wgrad_ws_floats() floats (per-slice partial sums, reduced in slice order). */
int64_t ic2_conv_wgrad_ws_floats(int n, int h, int w, int cin_p, int cout_p, int kh, int kw, int pad);
int ic2_conv_wgrad(const void* x, const void* dy, float* dw, int dtype, int n, int h, int w, int cin_p, int cout_p,
                   int kh, int kw, int pad, float* workspace, int64_t ws_floats, void* stream);
/* The same gradient written in nn.Conv2d's weight layout dw [cout][cin][kh][kw] f32 (the parameter's .grad shape,
 * valid channels only) instead of the packed [cout_p][kh][kw][cin_p]. */
int ic2_conv_wgrad_oihw(const void* x, const void* dy, float* dw, int dtype, int n, int h, int w, int cin_p,
                        int cout_p, int cout, int cin, int kh, int kw, int pad, float* workspace, int64_t ws_floats,
                        void* stream);

/* Backward of ic2_gn_lrelu_pool (VGGBlock :183-191: GroupNorm -> leaky_relu(0.2) -> AvgPool2d(2) when `pool`):
 * y = the GroupNorm input (NHWC [n][h][w][c_p]), stats = ic2_group_norm_stats' output, dout = gradient of the
 * block output (pooled resolution when `pool`) -> dy (NHWC, same shape as y), dgamma, dbeta [c] (nullable).
 * dtypes f32 / bf16 each.  Workspace: ic2_gn_lrelu_pool_bwd_floats() floats.  Deterministic. */
int64_t ic2_gn_lrelu_pool_bwd_floats(int n, int h, int w, int c_p, int groups);
int ic2_gn_lrelu_pool_bwd(const void* y, const void* dout, void* dy, int dtype_y, int dtype_dout, int dtype_dy, int n,
                          int h, int w, int c_p, int c, int groups, const float* stats, const float* gamma,
                          const float* beta, float slope, int pool, float* dgamma, float* dbeta, float* workspace,
                          int64_t ws_floats, void* stream);
/* The same, plus dsum[c] = sum over (n, p) of dy (nullable): the bias gradient of the conv whose output y is
 * (VGGBlock :183-191, conv -> GroupNorm), from the pass-1 channel sums (sum dz, sum dz * xhat, sum xhat) in f64
 * instead of a reduction over the stored dy. */
int ic2_gn_lrelu_pool_bwd_db(const void* y, const void* dout, void* dy, int dtype_y, int dtype_dout, int dtype_dy,
                             int n, int h, int w, int c_p, int c, int groups, const float* stats, const float* gamma,
                             const float* beta, float slope, int pool, float* dgamma, float* dbeta, float* dsum,
                             float* workspace, int64_t ws_floats, void* stream);

/* Backward of ic2_global_avg_pool (AdaptiveAvgPool2d(1), :218): dx [n][hw][c_p] = dpooled [n][c] / hw. */
int ic2_gap_bwd(const float* dpooled, void* dx, int dtype, int n, int hw, int c_p, int c, void* stream);

/* VGGBlock conv + GroupNorm statistics (SURVEY 8b `ic2_conv3x3_gn_fwd`; stylegan3_hvae_full.py:175-191, the
 * conv1/conv2 -> norm1/norm2 pairs): y = conv(x, w) + bias (NHWC, dtype = the activation dtype) and the GroupNorm
 * (mean, rstd) per (sample, group) of y's first cout_valid channels in stats[0 .. 2*n*groups).  When the halo conv
 * kernel runs the layer (bf16, cin_p <= 96, cout_p <= 64) the per-tile sums come out of its epilogue, computed on the
 * stored (rounded) values, so y is not read a second time; otherwise the two-stage statistics pass of
 * ic2_group_norm_stats runs after the conv.  stats: ic2_conv3x3_gn_stats_floats() floats (statistics + partial
 * sums); conv_ws / conv_ws_bytes: the conv's split-K workspace as for ic2_conv_igemm_ws.  fuse: 1 = fused statistics
 * where the halo conv runs, 0 = always the separate pass, -1 = default (separate; env IC2_CONV_GN=1 fuses -- measured
 * at parity on MI355X).  Deterministic.  dtype IC2_BF16X3: the split-bf16 encoder -- x stored
 * [hi | lo] with cin_p = the tripled (GEMM K) channel count, w from ic2_pack_weight(IC2_BF16X3), y f32 NHWC; the
 * statistics come out of the 4-wave halo GEMM's epilogue (on the f32 values as stored) when it runs a 64- / 128-wide
 * layer with 32 groups (fuse != 0), else the separate pass.  dtype IC2_F16X2: the same with the f16 input and
 * [hi | lo] f16 weights (cin_p = the doubled K), the f16 instances of those kernels, y f16 NHWC (the statistics of
 * the stored f16 values). */
int64_t ic2_conv3x3_gn_stats_floats(int dtype, int n, int h, int w, int cin_p, int cout_p, int kh, int kw, int pad,
                                    int groups);
int ic2_conv3x3_gn_fwd(const void* x, const void* w, void* y, int dtype, int n, int h, int w_, int cin_p, int cout_p,
                       int cout_valid, int kh, int kw, int pad, const float* bias, int groups, float eps, float* stats,
                       int64_t stats_floats, void* conv_ws, int64_t conv_ws_bytes, int fuse, void* stream);
/* The same for IC2_F16X2 with the weights packed times a power of two 2^s (ic2_pack_weight's `scale`, so that the
 * f16 low halves stay normal) and bias [cout_p] times 2^s: y = (conv(x, w) + bias) * out_mul with out_mul = 2^-s,
 * exact; the statistics are of y. */
int ic2_conv3x3_gn_fwd_scaled(const void* x, const void* w, void* y, int dtype, int n, int h, int w_, int cin_p,
                              int cout_p, int cout_valid, int kh, int kw, int pad, const float* bias, float out_mul,
                              int groups, float eps, float* stats, int64_t stats_floats, void* conv_ws,
                              int64_t conv_ws_bytes, int fuse, void* stream);
/* 1 when ic2_conv3x3_gn_fwd with these arguments takes the statistics from the conv's epilogue (a host query). */
int ic2_conv3x3_gn_fuses(int dtype, int n, int h, int w, int cin_p, int cout_p, int cout_valid, int kh, int kw, int pad,
                         int groups, int fuse);

/* VGGBlock's second conv with the first GroupNorm + lrelu applied to its INPUT as the halo conv stages it
 * (stylegan3_hvae_full.py:183-191: conv2(lrelu(norm1(conv1(x))))): the normalised activation is never written to
 * HBM.  x = conv1's raw output (bf16 NHWC, cin_p 64); in_gn = ic2_gn_affine_table() of norm1 [n][cin_p][4] f32;
 * in_slope = the lrelu slope; zero padding stays zero (the reference pads the normalised activation).  Otherwise as
 * ic2_conv3x3_gn_fwd.  Bit-identical to ic2_gn_lrelu_pool (no pool) followed by ic2_conv3x3_gn_fwd.  Returns
 * IC2_E_UNSUPPORTED unless ic2_conv3x3_gnin_supported() (the halo conv runs the shape). */
int ic2_conv3x3_gnin_supported(int dtype, int n, int h, int w, int cin_p, int cout_p, int kh, int kw, int pad);
int ic2_gn_affine_table(const float* stats, const float* gamma, const float* beta, int n, int c, int c_p, int groups,
                        float* table, void* stream);
int ic2_conv3x3_gnin_gn_fwd(const void* x, const float* in_gn, float in_slope, const void* w, void* y, int dtype, int n,
                            int h, int w_, int cin_p, int cout_p, int cout_valid, int kh, int kw, int pad,
                            const float* bias, int groups, float eps, float* stats, int64_t stats_floats, void* conv_ws,
                            int64_t conv_ws_bytes, int fuse, void* stream);

/* Backward of ic2_flrelu_nhwc w.r.t. its input (SynthesisLayer's filtered_lrelu, SG3-public; the encoder's loss
 * reaches W+ through it, :669-696): x = the forward's input (NHWC [n][in_h][in_w][c_p], f32 or f16), gout = the
 * gradient of its output (NHWC [n][out_h][out_w][c_p], f32 or bf16) -> gx (NHWC, f32).  Recomputes the upsampled
 * pre-activation, masks the adjoint down-FIR by lrelu' * gain (zero where clamped) and applies the adjoint up-FIR.
 * fu / fd: HOST taps.  StyleGAN3-T geometries (up 2 / 4 with 6*up taps, down 2 with 12 taps, px0 == py0); other
 * configurations return IC2_E_UNSUPPORTED (the caller composes ic2_upfirdn2d then). */
int ic2_flrelu_bwd_nhwc(const void* x, int x_dtype, const void* gout, int g_dtype, float* gx, int n, int c_p, int in_h,
                        int in_w, int out_h, int out_w, const float* fu, int fu_taps, const float* fd, int fd_taps,
                        int up, int down, int px0, int px1, int py0, int py1, float gain, float slope, float clamp,
                        int flip, void* stream);

/* ic2_flrelu_bwd_nhwc with the modulated conv's backward fused into its store (x = conv * oscale + bias, the
 * synthesis conv epilogue): gx = (dL/dx) * oscale[n][c] (the gradient w.r.t. the raw conv output, f32 or bf16 for
 * the dgrad GEMM), and ydot[n][tile][c] = per-tile sums of (dL/dx) * (x - bias[c]) -> dL/doscale = sum / oscale.
 * oscale / bias / ydot nullable.  ydot: ic2_flrelu_bwd_ydot_floats() floats. */
int64_t ic2_flrelu_bwd_ydot_floats(int n, int c_p, int in_h, int in_w, int up);
int ic2_flrelu_bwd_nhwc_ex(const void* x, int x_dtype, const void* gout, int g_dtype, void* gx, int gx_dtype, int n,
                           int c_p, int in_h, int in_w, int out_h, int out_w, const float* fu, int fu_taps,
                           const float* fd, int fd_taps, int up, int down, int px0, int px1, int py0, int py1,
                           float gain, float slope, float clamp, int flip, const float* oscale, const float* bias,
                           float* ydot, int64_t ydot_floats, void* stream);

/* Backward of the synthesis input modulation a = x * xscale[n][c] (SG3 modulated_conv2d's style multiply in the
 * activation-scaling form): dx = da * xscale (NHWC, f32 / bf16) and part[n][chunk][c] = per-chunk sums of da * x
 * (dL/dxscale = sum over chunks).  part: ic2_scale_bwd_part_floats() floats.  dx may be NULL (the partial sums only:
 * the training path folds xscale into the FLR backward's per-channel multiplier instead).  Deterministic. */
int64_t ic2_scale_bwd_part_floats(int n, int hw, int c_p);
int ic2_scale_bwd_nhwc(const void* da, const void* x, const float* xscale, void* dx, int dtype, int n, int hw, int c_p,
                       float* part, int64_t part_floats, void* stream);

/* The per-(sample, channel) finish of those partial sums: out[n][c] = (sum over r of part[n][r][c]) / den[n][c], and 0
 * where den[n][c] == 0 (den = NULL: the plain sum).  part [n][rows][c] f32 (ic2_scale_bwd_nhwc's part, or
 * ic2_flrelu_bwd_nhwc_ex's ydot), out [n][c] f32.  dL/dxscale = sum / xscale_next on the modulation-folded path and
 * dL/doscale = sum / oscale: the torch `where(den != 0, sum / den, 0)` chain of SG3's modulated_conv2d backward
 * (stylegan3_hvae_full.py:274) in one launch.  Deterministic (rows summed in order). */
int ic2_colsum_div(const float* part, int n, int rows, int c, const float* den, float* out, void* stream);

/* Its forward on the training path (SynthLayerNHWC; inference folds xscale into the producer's epilogue):
 * a[n][p][c] = x[n][p][c] * xscale[n][c], NHWC f32 / bf16, c_p % 8 == 0.  Replaces the reference's
 * `x * styles` broadcast inside modulated_conv2d (SG3-public, called at stylegan3_hvae_full.py:274). */
int ic2_scale_nhwc(const void* x, const float* xscale, void* a, int dtype, int n, int hw, int c_p, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* IC2OPS_H_ */
