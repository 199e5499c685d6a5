// NHWC implicit-GEMM convolution on CDNA4 MFMA.
//
// Replaces (a) the grouped conv2d inside StyleGAN3's modulated_conv2d [SG3-public; call sites
// /root/reference/stylegan3_hvae_full.py:274,329] in its activation-scaling form, (b) the VGGBlock
// and from_rgb nn.Conv2d of HVAE_VGG_Encoder (stylegan3_hvae_full.py:62,175-176) and (c) the
// 1x1 "x @ W^T" of SynthesisInput.
//
// GEMM view (per launch):  C^T[o][p] = sum_k W[o][k] * X[p][k]
//   o = output channel (MFMA A rows; weights stored [cout_p][kh][kw][cin_p], K-contiguous)
//   p = output pixel over the whole batch (MFMA B cols; NHWC input gives 8 consecutive k per lane)
//   k = (ky, kx, ci) with ci innermost; one K-chunk = 32 channels of one tap.
// Tile BO(o) x BP(p) x 32(k); WGO x WGP waves, each owning (BO/WGO) x (BP/WGP) = I x J MFMA tiles.
//   bf16: v_mfma_f32_16x16x32_bf16 (one MFMA per 16x16 tile per chunk)
//   f32 : v_mfma_f32_16x16x4_f32   (exact fp32 FMA chain; 8 MFMAs per tile per chunk)
// Global -> LDS by LDS-DMA (global_load_lds_dwordx4) into an NSTAGE-deep ring with counted vmcnt
// and raw s_barrier (chunks q+1 .. q+NSTAGE-2 stay in flight across the barrier).  LDS rows are
// XOR-swizzled per 16-B chunk through the SOURCE address (DMA writes lane-linear), the fragment
// reads apply the same XOR (conflict-free for bf16, 2-way for f32).  Out-of-image taps and padded
// output channels read a zero line instead of branching.  Blocks are remapped so consecutive
// logical tiles (which share input rows / weight panels) land on the same XCD's L2.
#include "common.h"

#include <cstdlib>

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
  int tiles_o;  // ceil(cout_p / BO)
  int nblocks;
  int act;
  float slope, act_gain, clamp, out_mul;
  int out_layout, out_dtype;
};

template <bool BF16, int BO, int BP, int WGO, int WGP, int NSTAGE>
struct IgCfg {
  static constexpr int NW = WGO * WGP;
  static constexpr int ESZ = BF16 ? 2 : 4;       // element bytes
  static constexpr int EPC = 16 / ESZ;           // elements per 16-B chunk
  static constexpr int ROWB = 32 * ESZ;          // LDS row bytes (one K-chunk of one row)
  static constexpr int WB = BO * ROWB, XB = BP * ROWB;  // bytes per stage per operand
  static constexpr int NIW_T = WB / 1024, NIX_T = XB / 1024;            // DMA instructions per stage
  static constexpr int NIW = (NIW_T + NW - 1) / NW, NIX = (NIX_T + NW - 1) / NW;  // per wave
  static constexpr int PER = NIW + NIX;          // DMA instructions per wave per chunk
  static constexpr int TO = BO / WGO, TP = BP / WGP;
  static constexpr int I = TO / 16, J = TP / 16;
  static constexpr int STAGEB = WB + XB;
  __device__ static __forceinline__ int swz(int row) { return BF16 ? ((row >> 1) & 3) : ((row >> 1) & 7); }
  __device__ static __forceinline__ int off(int row, int ch) { return row * ROWB + ((ch ^ swz(row)) << 4); }
};

template <bool BF16, int BO, int BP, int WGO, int WGP, int NSTAGE>
__global__ void __launch_bounds__(64 * WGO * WGP, 1) igemm_kernel(IgemmArgs a) {
  using C = IgCfg<BF16, BO, BP, WGO, WGP, NSTAGE>;
  constexpr int EPC = C::EPC, ESZ = C::ESZ, I = C::I, J = C::J, NIW = C::NIW, NIX = C::NIX;
  static_assert(C::I >= 1 && C::J >= 1, "wave tile smaller than one MFMA tile");
  static_assert(C::NIW_T >= 1 && C::NIX_T >= 1, "tile smaller than one DMA instruction");
  __shared__ __attribute__((aligned(16))) char lds[NSTAGE * C::STAGEB];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wid_u = __builtin_amdgcn_readfirstlane(wid);
  const int wo_ = wid / WGP, wp_ = wid % WGP;

  // XCD-aware, bijective block remap: blocks b and b+8 share an XCD -> give each XCD a contiguous
  // run of logical tiles (tiles adjacent in p share input rows; same-p tiles share the X panel).
  int logical;
  {
    const int b = blockIdx.x;
    const int xcd = b & 7, loc = b >> 3;
    const int q8 = a.nblocks >> 3, r8 = a.nblocks & 7;
    logical = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
  }
  const int o_tile = logical % a.tiles_o;
  const int p_tile = logical / a.tiles_o;
  const int o0 = o_tile * BO;
  const int m0 = p_tile * BP;

  const char* __restrict__ xg = reinterpret_cast<const char*>(a.x);
  const char* __restrict__ wg = reinterpret_cast<const char*>(a.w);

  // ---- per-lane DMA slots.  Instruction g of an operand fills LDS bytes [g KiB, g+1 KiB): lane l
  // lands on row g*(1024/ROWB) + l/(ROWB/16), physical slot l%(ROWB/16) = logical chunk slot^swz(row).
  // Waves beyond an operand's instruction count repeat its last instruction (identical bytes).
  int x_nb[NIX], x_oy[NIX], x_ox[NIX], x_ch[NIX], x_seg[NIX];
  bool x_ok[NIX];
  int64_t w_off[NIW];
  bool w_ok[NIW];
  int w_seg[NIW];
  const int hw = a.ho * a.wo;
#pragma unroll
  for (int k = 0; k < NIX; ++k) {
    const int g = min(wid_u + C::NW * k, C::NIX_T - 1);
    x_seg[k] = g * 1024;
    const int off = g * 1024 + lane * 16;
    const int row = off / C::ROWB;
    x_ch[k] = ((off % C::ROWB) >> 4) ^ C::swz(row);
    const int m = m0 + row;
    x_ok[k] = m < a.M;
    const int mm = x_ok[k] ? m : 0;
    const int nn = mm / hw;
    const int rem = mm - nn * hw;
    const int oy = rem / a.wo;
    x_nb[k] = nn * a.h;
    x_oy[k] = oy - a.pad;
    x_ox[k] = rem - oy * a.wo - a.pad;
  }
#pragma unroll
  for (int k = 0; k < NIW; ++k) {
    const int g = min(wid_u + C::NW * k, C::NIW_T - 1);
    w_seg[k] = g * 1024;
    const int off = g * 1024 + lane * 16;
    const int row = off / C::ROWB;
    const int chl = ((off % C::ROWB) >> 4) ^ C::swz(row);
    const int o = o0 + row;
    w_ok[k] = o < a.cout_p;
    w_off[k] = (int64_t)(w_ok[k] ? o : 0) * a.K * ESZ + chl * 16;
  }
  const int CB = a.cin_p >> 5;

#define IC2_IG_ISSUE(q_, buf_)                                                                                \
  {                                                                                                          \
    const int q__ = (q_);                                                                                    \
    const int tap = q__ / CB;                                                                                \
    const int cbk = q__ - tap * CB;                                                                          \
    const int ky = tap / a.kw;                                                                               \
    const int kx = tap - ky * a.kw;                                                                          \
    char* wl_ = lds + (buf_) * C::STAGEB;                                                                    \
    char* xl_ = wl_ + C::WB;                                                                                 \
    _Pragma("unroll") for (int k = 0; k < NIW; ++k) {                                                        \
      const void* ws = w_ok[k] ? (const void*)(wg + w_off[k] + (int64_t)q__ * 32 * ESZ) : zero_line();       \
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)ws,                     \
                                       (__attribute__((address_space(3))) void*)(wl_ + w_seg[k]), 16, 0, 0); \
    }                                                                                                        \
    _Pragma("unroll") for (int k = 0; k < NIX; ++k) {                                                        \
      const int iy = x_oy[k] + ky;                                                                           \
      const int ix = x_ox[k] + kx;                                                                           \
      const bool ok = x_ok[k] && (unsigned)iy < (unsigned)a.h && (unsigned)ix < (unsigned)a.w_;              \
      const int64_t e = ((int64_t)(x_nb[k] + iy) * a.w_ + ix) * a.cin_p + cbk * 32 + x_ch[k] * EPC;          \
      const void* xs = ok ? (const void*)(xg + e * ESZ) : zero_line();                                       \
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)xs,                     \
                                       (__attribute__((address_space(3))) void*)(xl_ + x_seg[k]), 16, 0, 0); \
    }                                                                                                        \
  }

  f32x4 acc[I][J];
#pragma unroll
  for (int i = 0; i < I; ++i)
#pragma unroll
    for (int j = 0; j < J; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s_ = 0; s_ < NSTAGE - 1; ++s_) IC2_IG_ISSUE(s_ < a.nq ? s_ : a.nq - 1, s_);

  const int fr = lane & 15;
  const int fh = lane >> 4;

  for (int q = 0; q < a.nq; ++q) {
    const int cur = q % NSTAGE;
    if constexpr (NSTAGE == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NSTAGE - 2) * C::PER) : "memory");
    __builtin_amdgcn_s_barrier();  // chunk q landed for every wave; chunk q-1 fully read
    __builtin_amdgcn_sched_barrier(0);
    {
      const int qn = q + NSTAGE - 1;
      IC2_IG_ISSUE(qn < a.nq ? qn : a.nq - 1, qn % NSTAGE);  // refill the slot chunk q-1 used
    }
    __builtin_amdgcn_sched_barrier(0);
    const char* wl = lds + cur * C::STAGEB;
    const char* xl = wl + C::WB;
    if constexpr (BF16) {
      bf16x8 bfr[J];
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const int row = wp_ * C::TP + j * 16 + fr;
        bfr[j] = *reinterpret_cast<const bf16x8*>(xl + C::off(row, fh));
      }
#pragma unroll
      for (int i = 0; i < I; ++i) {
        const int row = wo_ * C::TO + i * 16 + fr;
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(wl + C::off(row, fh));
#pragma unroll
        for (int j = 0; j < J; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[j], acc[i][j], 0, 0, 0);
      }
    } else {
      // lane group fh uses k = 8*fh + s for step s: chunks 2fh (s<4) and 2fh+1 (s>=4)
      f32x4 af[I][2], bfr[J][2];
#pragma unroll
      for (int i = 0; i < I; ++i) {
        const int row = wo_ * C::TO + i * 16 + fr;
        af[i][0] = *reinterpret_cast<const f32x4*>(wl + C::off(row, 2 * fh));
        af[i][1] = *reinterpret_cast<const f32x4*>(wl + C::off(row, 2 * fh + 1));
      }
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const int row = wp_ * C::TP + j * 16 + fr;
        bfr[j][0] = *reinterpret_cast<const f32x4*>(xl + C::off(row, 2 * fh));
        bfr[j][1] = *reinterpret_cast<const f32x4*>(xl + C::off(row, 2 * fh + 1));
      }
#pragma unroll
      for (int s = 0; s < 8; ++s)
#pragma unroll
        for (int i = 0; i < I; ++i)
#pragma unroll
          for (int j = 0; j < J; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i][s >> 2][s & 3], bfr[j][s >> 2][s & 3], acc[i][j], 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);  // every MFMA of this chunk before the next wait
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the redundant tail DMAs before exit
#undef IC2_IG_ISSUE

  // ---- epilogue: lane holds C[o = base + 4*fh + r][p = base + fr]
  const bool has_os = a.oscale != nullptr, has_b = a.bias != nullptr;
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int p = m0 + wp_ * C::TP + j * 16 + fr;
    if (p >= a.M) continue;
    const int nn = p / hw;
    const int pix = p - nn * hw;
#pragma unroll
    for (int i = 0; i < I; ++i) {
      const int ob = o0 + wo_ * C::TO + i * 16 + 4 * fh;
      if (ob >= a.cout_p) continue;
      float4 sc = make_float4(1.f, 1.f, 1.f, 1.f), bi = make_float4(0.f, 0.f, 0.f, 0.f);
      if (has_os) sc = *reinterpret_cast<const float4*>(a.oscale + (int64_t)nn * a.cout_p + ob);
      if (has_b) bi = *reinterpret_cast<const float4*>(a.bias + ob);
      float v[4];
      const float scv[4] = {sc.x, sc.y, sc.z, sc.w}, biv[4] = {bi.x, bi.y, bi.z, bi.w};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float t = acc[i][j][r] * scv[r] + biv[r];
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

template <bool BF16, int BO, int BP, int WGO, int WGP, int NSTAGE>
static void launch_igemm(IgemmArgs a, hipStream_t s) {
  a.tiles_o = (a.cout_p + BO - 1) / BO;
  a.nblocks = (int)(ceil_div(a.M, BP) * a.tiles_o);
  hipLaunchKernelGGL((igemm_kernel<BF16, BO, BP, WGO, WGP, NSTAGE>), dim3(a.nblocks), dim3(64 * WGO * WGP), 0, s, a);
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
  IC2_CHECK_ARG(((uintptr_t)oscale | (uintptr_t)bias) % 16 == 0, "conv_igemm: oscale/bias must be 16-byte aligned");
  const int64_t M = (int64_t)n * ho * wo;
  IC2_CHECK_ARG(M < (1LL << 30), "conv_igemm: too many output pixels");
  IgemmArgs a;
  a.x = x; a.w = w; a.y = y; a.oscale = oscale; a.bias = bias;
  a.n = n; a.h = h; a.w_ = w_; a.cin_p = cin_p; a.cout_p = cout_p; a.cout_valid = cout_valid;
  a.kh = kh; a.kw = kw; a.pad = pad; a.ho = ho; a.wo = wo;
  a.M = (int)M; a.K = kh * kw * cin_p; a.nq = a.K / 32;
  a.act = act; a.slope = slope; a.act_gain = act_gain; a.clamp = clamp; a.out_mul = out_mul;
  a.out_layout = out_layout; a.out_dtype = out_dtype;
  hipStream_t s = as_stream(stream);
  if (dtype == IC2_BF16) {
    // the widest o-tile the layer fills; 256-pixel tiles while the grid keeps >= 2 workgroups per CU
    // IC2_IGEMM_TILE=1..4 forces a tile (tests exercise every instance on small problems)
    static const int forced = [] {
      const char* e = getenv("IC2_IGEMM_TILE");
      return e ? atoi(e) : 0;
    }();
    // o-tile: the widest of {256, 128, 64, 32} that divides cout_p (no padded MFMA rows), 256-pixel
    // tiles while the grid keeps >= 2 workgroups per CU, else the 128 x 128 tile
    const bool big_m = ceil_div(M, 256) * ((cout_p + 255) / 256) >= 512;
    int tile;
    if (!big_m) tile = cout_p <= 32 ? 2 : 4;
    else if (cout_p % 256 == 0) tile = 1;
    else if (cout_p % 128 == 0) tile = 3;
    else if (cout_p % 64 == 0) tile = 5;
    else tile = 2;
    if (forced >= 1 && forced <= 5) tile = forced;
    switch (tile) {
      case 1: launch_igemm<true, 256, 256, 2, 4, 4>(a, s); break;
      case 2: launch_igemm<true, 32, 256, 1, 4, 4>(a, s); break;
      case 3: launch_igemm<true, 128, 256, 2, 4, 4>(a, s); break;
      case 5: launch_igemm<true, 64, 256, 1, 4, 4>(a, s); break;
      default: launch_igemm<true, 128, 128, 2, 2, 4>(a, s); break;
    }
  } else {
    launch_igemm<false, 128, 128, 2, 2, 2>(a, s);
  }
  IC2_CHECK_LAUNCH("conv_igemm");
  return IC2_OK;
}
