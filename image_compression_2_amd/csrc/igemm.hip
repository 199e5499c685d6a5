// NHWC implicit-GEMM convolution on CDNA4 MFMA.
//
// Replaces (a) the grouped conv2d inside StyleGAN3's modulated_conv2d [SG3-public; call sites
// /root/reference/stylegan3_hvae_full.py:274,329] in its activation-scaling form, (b) the VGGBlock
// and from_rgb nn.Conv2d of HVAE_VGG_Encoder (stylegan3_hvae_full.py:62,175-176) and (c) the
// 1x1 "x @ W^T" of SynthesisInput.
//
// GEMM view (per launch):  C^T[o][p] = sum_k W[o][k] * X[p][k]
//   o = output channel (MFMA A rows, weights stored [cout_p][kh][kw][cin_p], K-contiguous)
//   p = output pixel over the whole batch (MFMA B cols; NHWC input gives 8 consecutive k per lane)
//   k = (ky, kx, ci) with ci innermost; one K-chunk = 32 channels of one tap.
// Tile 128(o) x 128(p) x 32(k), 256 threads = 4 waves in 2x2, each wave 64x64 = 4x4 MFMA tiles.
//   bf16: v_mfma_f32_16x16x32_bf16 (one MFMA per 16x16 tile per chunk)
//   f32 : v_mfma_f32_16x16x4_f32   (exact fp32 FMA chain; 8 MFMAs per tile per chunk)
// LDS: double-buffered W and X tiles, rows XOR-swizzled per 16-B chunk (bank-conflict-free reads
// for bf16, 2-way for f32); register-staged global loads of the next chunk overlap the MFMAs.
#include "common.h"

namespace ic2 {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

struct IgemmArgs {
  const void* x;
  const void* w;
  void* y;
  const float* oscale;
  const float* bias;
  int n, h, w_, cin_p, cout_p, cout_valid, kh, kw, pad, ho, wo;
  int M;        // n * ho * wo
  int K;        // kh * kw * cin_p
  int nq;       // K / 32
  int tiles_o;  // ceil(cout_p / 128)
  int act;
  float slope, act_gain, clamp, out_mul;
  int out_layout, out_dtype;
};

template <bool BF16>
struct IgTraits {
  static constexpr int ESZ = BF16 ? 2 : 4;       // element bytes
  static constexpr int EPC = 16 / ESZ;           // elements per 16-B chunk
  static constexpr int CPR = 32 / EPC;           // chunks per 32-element row (4 / 8)
  static constexpr int ROWB = 32 * ESZ;          // row bytes (64 / 128)
  static constexpr int NLD = 128 * CPR / 256;    // chunks per thread per operand (2 / 4)
  static constexpr int TILEB = 128 * ROWB;       // bytes per operand tile
  static constexpr int RSTEP = 256 / CPR;        // row step between a thread's chunks
  __device__ static __forceinline__ int swz(int row) { return BF16 ? ((row >> 1) & 3) : ((row >> 1) & 7); }
  __device__ static __forceinline__ int off(int row, int ch) { return row * ROWB + ((ch ^ swz(row)) << 4); }
};

template <bool BF16>
__global__ void __launch_bounds__(256, 2) igemm_kernel(IgemmArgs a) {
  using TR = IgTraits<BF16>;
  constexpr int CPR = TR::CPR, NLD = TR::NLD, EPC = TR::EPC, ESZ = TR::ESZ;
  __shared__ __attribute__((aligned(16))) char lds[2 * 2 * TR::TILEB];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wo_ = wid >> 1, wp_ = wid & 1;

  const int bid = blockIdx.x;
  const int o_tile = bid % a.tiles_o;
  const int p_tile = bid / a.tiles_o;
  const int o0 = o_tile * 128;
  const int m0 = p_tile * 128;

  const char* __restrict__ xg = reinterpret_cast<const char*>(a.x);
  const char* __restrict__ wg = reinterpret_cast<const char*>(a.w);

  // ---- per-thread load slots: rows r_j = tid / CPR + j * RSTEP, chunk ch = tid % CPR
  const int ch = tid % CPR;
  int x_nb[NLD], x_oy[NLD], x_ox[NLD];
  bool x_ok[NLD];
  bool w_ok[NLD];
  int64_t w_base[NLD];
#pragma unroll
  for (int j = 0; j < NLD; ++j) {
    const int row = tid / CPR + j * TR::RSTEP;
    const int m = m0 + row;
    x_ok[j] = m < a.M;
    const int mm = x_ok[j] ? m : 0;
    const int hw = a.ho * a.wo;
    const int nn = mm / hw;
    const int rem = mm - nn * hw;
    const int oy = rem / a.wo;
    x_nb[j] = nn * a.h;
    x_oy[j] = oy - a.pad;
    x_ox[j] = rem - oy * a.wo - a.pad;
    const int o = o0 + row;
    w_ok[j] = o < a.cout_p;
    w_base[j] = (int64_t)(w_ok[j] ? o : 0) * a.K * ESZ + ch * 16;
  }

  const int CB = a.cin_p >> 5;
  int q_cb = 0, q_kx = 0, q_ky = 0;  // decomposition of the chunk being loaded

  uint4 xr[NLD], wr[NLD];
  auto load_chunk = [&](int q) {
#pragma unroll
    for (int j = 0; j < NLD; ++j) {
      const int iy = x_oy[j] + q_ky;
      const int ix = x_ox[j] + q_kx;
      const bool ok = x_ok[j] && (unsigned)iy < (unsigned)a.h && (unsigned)ix < (unsigned)a.w_;
      if (ok) {
        const int64_t e = ((int64_t)(x_nb[j] + iy) * a.w_ + ix) * a.cin_p + q_cb * 32 + ch * EPC;
        xr[j] = *reinterpret_cast<const uint4*>(xg + e * ESZ);
      } else {
        xr[j] = make_uint4(0, 0, 0, 0);
      }
      if (w_ok[j]) {
        wr[j] = *reinterpret_cast<const uint4*>(wg + w_base[j] + (int64_t)q * 32 * ESZ);
      } else {
        wr[j] = make_uint4(0, 0, 0, 0);
      }
    }
    (void)q;
    if (++q_cb == CB) {
      q_cb = 0;
      if (++q_kx == a.kw) {
        q_kx = 0;
        ++q_ky;
      }
    }
  };
  auto store_chunk = [&](int buf) {
    char* wl = lds + buf * 2 * TR::TILEB;
    char* xl = wl + TR::TILEB;
#pragma unroll
    for (int j = 0; j < NLD; ++j) {
      const int row = tid / CPR + j * TR::RSTEP;
      *reinterpret_cast<uint4*>(wl + TR::off(row, ch)) = wr[j];
      *reinterpret_cast<uint4*>(xl + TR::off(row, ch)) = xr[j];
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  load_chunk(0);
  store_chunk(0);
  __syncthreads();

  const int fr = lane & 15;
  const int fh = lane >> 4;

  for (int q = 0; q < a.nq; ++q) {
    const int cur = q & 1;
    const bool more = q + 1 < a.nq;
    if (more) load_chunk(q + 1);
    const char* wl = lds + cur * 2 * TR::TILEB;
    const char* xl = wl + TR::TILEB;
    if constexpr (BF16) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = wo_ * 64 + i * 16 + fr;
        af[i] = *reinterpret_cast<const bf16x8*>(wl + TR::off(row, fh));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = wp_ * 64 + j * 16 + fr;
        bfr[j] = *reinterpret_cast<const bf16x8*>(xl + TR::off(row, fh));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    } else {
      // lane group fh uses k = 8*fh + s for step s: chunks 2fh (s<4) and 2fh+1 (s>=4)
      f32x4 af[4][2], bfr[4][2];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = wo_ * 64 + i * 16 + fr;
        af[i][0] = *reinterpret_cast<const f32x4*>(wl + TR::off(row, 2 * fh));
        af[i][1] = *reinterpret_cast<const f32x4*>(wl + TR::off(row, 2 * fh + 1));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = wp_ * 64 + j * 16 + fr;
        bfr[j][0] = *reinterpret_cast<const f32x4*>(xl + TR::off(row, 2 * fh));
        bfr[j][1] = *reinterpret_cast<const f32x4*>(xl + TR::off(row, 2 * fh + 1));
      }
#pragma unroll
      for (int s = 0; s < 8; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i][s >> 2][s & 3], bfr[j][s >> 2][s & 3], acc[i][j], 0, 0, 0);
    }
    if (more) store_chunk(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue: lane holds C[o = base + 4*fh + r][p = base + fr]
  const int hw = a.ho * a.wo;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int p = m0 + wp_ * 64 + j * 16 + fr;
    if (p >= a.M) continue;
    const int nn = p / hw;
    const int pix = p - nn * hw;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ob = o0 + wo_ * 64 + i * 16 + 4 * fh;
      if (ob >= a.cout_p) continue;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float t = acc[i][j][r];
        if (a.oscale) t *= a.oscale[(int64_t)nn * a.cout_p + ob + r];
        if (a.bias) t += a.bias[ob + r];
        if (a.act) t = lrelu_gain_clamp(t, a.slope, a.act_gain, a.clamp);
        v[r] = t * a.out_mul;
      }
      if (a.out_layout == IC2_LAYOUT_NHWC) {
        const int64_t e = (int64_t)p * a.cout_p + ob;
        if (a.out_dtype == IC2_BF16) {
          uint2 pk;
          pk.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
          pk.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
          *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(a.y) + e) = pk;
        } else {
          *reinterpret_cast<float4*>(reinterpret_cast<float*>(a.y) + e) = make_float4(v[0], v[1], v[2], v[3]);
        }
      } else {
        float* yo = reinterpret_cast<float*>(a.y);
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (ob + r < a.cout_valid) yo[((int64_t)nn * a.cout_valid + ob + r) * hw + pix] = v[r];
      }
    }
  }
}

}  // namespace ic2

using namespace ic2;

extern "C" int ic2_conv_igemm(const void* x, const void* w, void* y, int dtype, int out_dtype, int n, int h, int w_,
                              int cin_p, int cout_p, int cout_valid, int kh, int kw, int pad, int ho, int wo,
                              const float* oscale, const float* bias, int act, float slope, float act_gain,
                              float clamp, float out_mul, int out_layout, void* stream) {
  IC2_CHECK_ARG(x && w && y, "conv_igemm: null pointer");
  IC2_CHECK_ARG(dtype == IC2_F32 || dtype == IC2_BF16, "conv_igemm: bad dtype %d", dtype);
  IC2_CHECK_ARG(out_dtype == IC2_F32 || out_dtype == IC2_BF16, "conv_igemm: bad out dtype %d", out_dtype);
  IC2_CHECK_ARG(cin_p > 0 && cin_p % 32 == 0 && cout_p > 0 && cout_p % 32 == 0,
                "conv_igemm: channel strides must be positive multiples of 32 (cin_p=%d cout_p=%d)", cin_p, cout_p);
  IC2_CHECK_ARG(n > 0 && h > 0 && w_ > 0 && kh > 0 && kw > 0 && pad >= 0, "conv_igemm: bad geometry");
  IC2_CHECK_ARG(ho == h + 2 * pad - kh + 1 && wo == w_ + 2 * pad - kw + 1,
                "conv_igemm: output size %dx%d does not match input %dx%d, k=%dx%d, pad=%d", ho, wo, h, w_, kh, kw, pad);
  IC2_CHECK_ARG(out_layout == IC2_LAYOUT_NHWC || (out_layout == IC2_LAYOUT_NCHW && out_dtype == IC2_F32 &&
                                                  cout_valid > 0 && cout_valid <= cout_p),
                "conv_igemm: NCHW output needs f32 and 0 < cout_valid <= cout_p");
  const int64_t M = (int64_t)n * ho * wo;
  IC2_CHECK_ARG(M < (1LL << 31), "conv_igemm: too many output pixels");
  IgemmArgs a;
  a.x = x; a.w = w; a.y = y; a.oscale = oscale; a.bias = bias;
  a.n = n; a.h = h; a.w_ = w_; a.cin_p = cin_p; a.cout_p = cout_p; a.cout_valid = cout_valid;
  a.kh = kh; a.kw = kw; a.pad = pad; a.ho = ho; a.wo = wo;
  a.M = (int)M; a.K = kh * kw * cin_p; a.nq = a.K / 32; a.tiles_o = (cout_p + 127) / 128;
  a.act = act; a.slope = slope; a.act_gain = act_gain; a.clamp = clamp; a.out_mul = out_mul;
  a.out_layout = out_layout; a.out_dtype = out_dtype;
  const int64_t tiles = ceil_div(M, 128) * a.tiles_o;
  IC2_CHECK_ARG(tiles < (1LL << 31), "conv_igemm: grid too large");
  if (dtype == IC2_BF16)
    hipLaunchKernelGGL(igemm_kernel<true>, dim3((unsigned)tiles), dim3(256), 0, as_stream(stream), a);
  else
    hipLaunchKernelGGL(igemm_kernel<false>, dim3((unsigned)tiles), dim3(256), 0, as_stream(stream), a);
  IC2_CHECK_LAUNCH("conv_igemm");
  return IC2_OK;
}
