// Shared between the fused filtered-lrelu kernels (flrelu.hip: VALU, every dtype/layout;
// flrelu_mfma.hip: the bf16 NHWC synthesis path on MFMA).
#pragma once
#include "common.h"

namespace ic2 {

struct FlrArgs {
  const void* x;
  void* y;
  const float* bias;
  const float* post_scale;  // [n][c_p] or null
  int64_t xsn, xsy, xsx, xsc;  // input strides (elements)
  int64_t xcb;                 // MFMA kernels: offset of the next 16-channel block (16 NHWC, 16*h*w blocked)
  int64_t ysn, ysy, ysx, ysc;  // output strides
  int c, c_p;                   // valid channels, post_scale row stride
  int in_h, in_w, out_h, out_w;
  int py0, px0;                 // leading padding
  int tiles_x, tiles_y, cblocks, nimg;
  int order;  // wide MFMA kernel: tile order, 0 = channel block fastest, 1 = x, y fastest (one plane per XCD run)
  int out_f16;  // MFMA kernels: output f16 (saturated) instead of bf16 (the synthesis's f16 mode)
  float slope, lim;  // lrelu slope (<= 1) and clamp bound / gain (+inf = no clamp)
  float gdg[12];     // down taps * gain (horizontal pass, right after the activation)
  float gu[24];  // flipped (unless flip_filter) and scaled by `up` (sqrt of the up^2 gain per pass)
  float gd[12];  // flipped (unless flip_filter)
  // MFMA clamp-split kernels (finite lim): the horizontal passes' taps with the clamp scaling folded in on the host
  // before the joint f16 rounding (f16_round_taps), so each polyphase group keeps its DC gain
  float guh[24];  // gu / lim
  float gdgl[12];  // gdg * lim
};

// taps -> f16-representable values, rounded jointly per group t mod stride_groups (minimal group sum error):
// the MFMA kernels' f16 FIR taps (flrelu.hip; shared with the MFMA backward, flrelu_bwd.hip)
void f16_round_taps(const float* exact, float* out, int n, int stride_groups);

// NHWC or channel-blocked NHWC16 (strides in a), f16 (in_f16) or bf16 input, bf16 or f16 (a.out_f16) output, up in {2, 4} with 6*up taps, down 2 with 12 taps, no
// bias (folded into the producer).  Sets tiles/cblocks itself.  Returns IC2_E_UNSUPPORTED when the
// configuration has no MFMA instance.
int flrelu_mfma_launch(FlrArgs a, int in_f16, int up, int down, int tu, int td, int delta, int n, hipStream_t s);

}  // namespace ic2
