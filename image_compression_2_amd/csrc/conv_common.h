// Conv helpers shared by the implicit-GEMM (igemm.hip) and Winograd (wino.hip) kernels: MFMA operand types, the
// launch argument record, the fused epilogue store and the XCD-aware block remap.
#pragma once
#include "common.h"

namespace ic2 {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

// The 2-byte operand MFMA: bf16 (v_mfma_f32_16x16x32_bf16) or f16 (v_mfma_f32_16x16x32_f16, the same rate on gfx950).
// Fragments travel as raw 16-B bf16x8 registers either way (LDS-DMA / ds_read move bits), reinterpreted here.
template <bool F16>
__device__ __forceinline__ f32x4 mfma32(bf16x8 a, bf16x8 b, f32x4 c) {
  if constexpr (F16)
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
// 2-byte activation / weight dtypes (bf16 or f16): the same kernels, a different MFMA
__host__ __device__ inline bool is16(int dtype) { return dtype == IC2_BF16 || dtype == IC2_F16; }

struct IgemmArgs {
  const void* x;
  const void* w;
  void* y;
  const float* oscale;
  const float* bias;
  float* ws;    // split-K partial sums [gridDim.y][M][cout_p] f32 (gridDim.y > 1 only)
  int n, h, w_, cin_p, cout_p, cout_valid, kh, kw, pad, ho, wo;
  int M;        // n * ho * wo
  int K;        // kh * kw * cin_p
  int nq;       // K-chunks: K / 32 (K / 64 for the 8-phase kernels)
  int tiles_o;  // ceil(cout_p / BO)
  int nblocks;  // tiles_o * tiles_p
  int group;    // p-tiles per o-sweep (tile_coords)
  int korder;   // 8-phase kernels: 0 = tap-major K, 1 = channel-major K (taps innermost)
  int o_base;   // 8-phase kernels: first output channel of this launch (a cout_p split over two tile shapes)
  int tile_base;  // 8-phase kernels: first logical tile of this launch (the split tail of a grid, see ig_plan)
  int act;
  float slope, act_gain, clamp, out_mul;
  int out_layout, out_dtype;
  // fused GroupNorm statistics (hconv only; ic2_conv3x3_gn_fwd): per (image, group, tile) f64 (sum, sumsq) of
  // the stored (rounded) outputs of channels < gn_c; null = off
  double* gn_part;
  int gn_groups, gn_c;
  // GroupNorm + lrelu of the INPUT applied while the halo conv stages it (hconv, cin_p 32 / 64 only): per
  // (sample, input channel) (mean, rstd * gamma, beta, 0) f32 [n][cin_p][4]; null = the input is used as is
  const float* in_gn;
  float in_slope;
  // input storage: x_pix = elements per input pixel (cin_p, or 2/3 of it for the split-bf16 input, stored [hi | lo]
  // while the GEMM's K runs over [hi | hi | lo] against [hi | lo | hi] weights); x_hb32 = 32-channel blocks of the hi
  // part (0: plain storage).  K block b of 32 channels reads stored block ig_xb32(a, b): b, or b - x_hb32 past hi
  int x_pix, x_hb32;
  // Winograd F(2,3)-along-x kernel (wino.hip) only: output tile = wx_th rows x wx_twp pixel pairs, each row
  // served by wx_ns 16-lane pair blocks; halo line pitch wx_hp (64-B LDS rows per (halo row, column parity) line),
  // wx_nh halo rows used, wx_tx x wx_ty tiles per image
  int wx_twp, wx_th, wx_ns, wx_hp, wx_nh, wx_tx, wx_ty;
  // f16 output converted IEEE (out_dtype IC2_F16_IEEE at the entry point: the training path's gradient convs) instead
  // of saturated to the f16 range (activations)
  int out_ieee;
};
__device__ __forceinline__ int ig_xb32(const IgemmArgs& a, int b) { return b >= a.x_hb32 ? b - a.x_hb32 : b; }

// Per-channel epilogue operands.  The epilogues load them for all their channel blocks BEFORE the first store: a
// load placed after a store to y may alias it, so loading inside the store loop serialised one load round trip per
// 16 x 16 block (33 `s_waitcnt vmcnt(0)` per wave in the 8-phase and halo kernels' epilogues).
__device__ __forceinline__ float4 ig_load_oscale(const IgemmArgs& a, int nn, int ob) {
  return a.oscale && ob < a.cout_p ? *reinterpret_cast<const float4*>(a.oscale + (int64_t)nn * a.cout_p + ob)
                                   : make_float4(1.f, 1.f, 1.f, 1.f);
}
__device__ __forceinline__ float4 ig_load_bias(const IgemmArgs& a, int ob) {
  return a.bias && ob < a.cout_p ? *reinterpret_cast<const float4*>(a.bias + ob) : make_float4(0.f, 0.f, 0.f, 0.f);
}
// Retire the preloads with a real s_waitcnt vmcnt(0) (gfx9 encoding: expcnt / lgkmcnt left at their maxima), so the
// waitcnt pass sees them complete; otherwise it re-waits vmcnt(0) -- behind the previous block's stores -- at
// every join of the branchy store code below.
__device__ __forceinline__ void ig_preloads_done() { __builtin_amdgcn_s_waitcnt(0x0F70); }

// y = act(acc * oscale[n][o] + bias[o]) * out_mul for the channels ob .. ob+3 of output pixel p = (nn, pix),
// stored NHWC / NHWC16 (bf16 / f16 / f32) or NCHW (f32, channels < cout_valid only); sc / bi = the preloaded
// oscale[nn][ob..ob+3] / bias[ob..ob+3].
__device__ __forceinline__ void ig_store4v(const IgemmArgs& a, int p, int nn, int pix, int ob, const float (&acc)[4],
                                           float4 sc, float4 bi, float (*vout)[4] = nullptr) {
  const float scv[4] = {sc.x, sc.y, sc.z, sc.w}, biv[4] = {bi.x, bi.y, bi.z, bi.w};
  float v[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float t = acc[r] * scv[r] + biv[r];
    if (a.act) t = lrelu_gain_clamp(t, a.slope, a.act_gain, a.clamp);
    v[r] = t * a.out_mul;
  }
  if (vout != nullptr) {  // the f32 values this call stores (the fused GroupNorm statistics read them)
#pragma unroll
    for (int r = 0; r < 4; ++r) (*vout)[r] = v[r];
  }
  if (a.out_layout != IC2_LAYOUT_NCHW) {
    // NHWC, or channel-blocked NHWC16 [n][cout_p / 16][ho][wo][16] (the fused filtered lrelu's input: its
    // 16-channel tiles read contiguous rows)
    const int64_t e = a.out_layout == IC2_LAYOUT_NHWC
                          ? (int64_t)p * a.cout_p + ob
                          : (((int64_t)nn * (a.cout_p >> 4) + (ob >> 4)) * ((int64_t)a.ho * a.wo) + pix) * 16 + (ob & 15);
    if (a.out_dtype == IC2_BF16) {
      uint2 pk;
      pk.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
      pk.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
      *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(a.y) + e) = pk;
    } else if (a.out_dtype == IC2_F16) {
      typedef _Float16 h2 __attribute__((ext_vector_type(2)));
      float s_[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) s_[r] = a.out_ieee ? v[r] : __builtin_amdgcn_fmed3f(v[r], -65504.f, 65504.f);
      const h2 q0 = h2{(_Float16)s_[0], (_Float16)s_[1]}, q1 = h2{(_Float16)s_[2], (_Float16)s_[3]};
      if (vout != nullptr) {  // the statistics of what is stored (the f16 values), as the separate pass sees them
        (*vout)[0] = (float)q0.x; (*vout)[1] = (float)q0.y; (*vout)[2] = (float)q1.x; (*vout)[3] = (float)q1.y;
      }
      uint2 pk;
      pk.x = __builtin_bit_cast(uint32_t, q0);
      pk.y = __builtin_bit_cast(uint32_t, q1);
      *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(a.y) + e) = pk;
    } else {
      *reinterpret_cast<float4*>(reinterpret_cast<float*>(a.y) + e) = make_float4(v[0], v[1], v[2], v[3]);
    }
  } else {
    float* yo = reinterpret_cast<float*>(a.y);
    const int hw = a.ho * a.wo;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (ob + r < a.cout_valid) yo[((int64_t)nn * a.cout_valid + ob + r) * hw + pix] = v[r];
  }
}
__device__ __forceinline__ void ig_store4(const IgemmArgs& a, int p, int nn, int pix, int ob, const float (&acc)[4]) {
  ig_store4v(a, p, nn, pix, ob, acc, ig_load_oscale(a, nn, ob), ig_load_bias(a, ob));
}

// XCD-aware, bijective block remap: blocks b and b+8 share an XCD -> give each XCD a contiguous run
// of logical tiles (tiles adjacent in p share input rows; same-p tiles share the X panel).
__device__ __forceinline__ int xcd_remap(int b, int nblocks) {
  const int xcd = b & 7, loc = b >> 3;
  const int q8 = nblocks >> 3, r8 = nblocks & 7;
  return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
}

constexpr uint32_t kOob = 0x7ffffff0u;            // num_records of a live descriptor = the zero-answer offset
constexpr int kRsrcWord3 = 0x00020000;            // raw buffer descriptor word 3 (gfx9 family)

}  // namespace ic2
