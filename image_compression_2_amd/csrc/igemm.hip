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
// LDS: double-buffered W and X tiles filled by LDS-DMA (global_load_lds_dwordx4) one chunk ahead of
// the MFMAs; rows XOR-swizzled per 16-B chunk via the source address (conflict-free fragment reads
// for bf16, 2-way for f32).
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
  static constexpr int NSTAGE = BF16 ? 4 : 2;    // LDS ring depth (chunks in flight = NSTAGE - 1)
  __device__ static __forceinline__ int swz(int row) { return BF16 ? ((row >> 1) & 3) : ((row >> 1) & 7); }
  __device__ static __forceinline__ int off(int row, int ch) { return row * ROWB + ((ch ^ swz(row)) << 4); }
};

template <bool BF16>
__global__ void __launch_bounds__(256, 2) igemm_kernel(IgemmArgs a) {
  using TR = IgTraits<BF16>;
  constexpr int CPR = TR::CPR, NLD = TR::NLD, EPC = TR::EPC, ESZ = TR::ESZ;
  constexpr int NSTAGE = TR::NSTAGE;
  __shared__ __attribute__((aligned(16))) char lds[NSTAGE * 2 * TR::TILEB];

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

  // ---- global -> LDS by LDS-DMA (global_load_lds_dwordx4): no register staging, so nothing can
  // serialise the loads behind a wait.  Wave w, instruction k fills LDS bytes
  // [(w*NI + k) * 1 KiB, +1 KiB) of an operand tile, lane l writing base + 16*l (lane-linear).  The
  // bank swizzle therefore moves to the SOURCE: the lane that lands on physical 16-B slot p of row r
  // fetches logical chunk p ^ swz(r); the fragment reads apply the same XOR.  Out-of-image pixels
  // and padded output channels read the code object's zero line.
  constexpr int NI = TR::TILEB / 1024 / 4;  // DMA instructions per wave per operand (2 / 4)
  const int wid_u = __builtin_amdgcn_readfirstlane(wid);
  int x_nb[NI], x_oy[NI], x_ox[NI], x_ch[NI];
  bool x_ok[NI];
  int64_t w_off[NI];
  bool w_ok[NI];
#pragma unroll
  for (int k = 0; k < NI; ++k) {
    const int off = (wid * NI + k) * 1024 + lane * 16;
    const int row = off / TR::ROWB;
    const int chl = ((off % TR::ROWB) >> 4) ^ TR::swz(row);
    x_ch[k] = chl;
    const int m = m0 + row;
    x_ok[k] = m < a.M;
    const int mm = x_ok[k] ? m : 0;
    const int hw = a.ho * a.wo;
    const int nn = mm / hw;
    const int rem = mm - nn * hw;
    const int oy = rem / a.wo;
    x_nb[k] = nn * a.h;
    x_oy[k] = oy - a.pad;
    x_ox[k] = rem - oy * a.wo - a.pad;
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
    char* wl_ = lds + (buf_) * 2 * TR::TILEB;                                                                \
    char* xl_ = wl_ + TR::TILEB;                                                                             \
    _Pragma("unroll") for (int k = 0; k < NI; ++k) {                                                         \
      const int iy = x_oy[k] + ky;                                                                           \
      const int ix = x_ox[k] + kx;                                                                           \
      const bool ok = x_ok[k] && (unsigned)iy < (unsigned)a.h && (unsigned)ix < (unsigned)a.w_;              \
      const int64_t e = ((int64_t)(x_nb[k] + iy) * a.w_ + ix) * a.cin_p + cbk * 32 + x_ch[k] * EPC;          \
      const void* xs = ok ? (const void*)(xg + e * ESZ) : zero_line();                                       \
      const void* ws = w_ok[k] ? (const void*)(wg + w_off[k] + (int64_t)q__ * 32 * ESZ) : zero_line();       \
      const int seg = (wid_u * NI + k) * 1024;                                                               \
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)xs,                     \
                                       (__attribute__((address_space(3))) void*)(xl_ + seg), 16, 0, 0);      \
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)ws,                     \
                                       (__attribute__((address_space(3))) void*)(wl_ + seg), 16, 0, 0);      \
    }                                                                                                        \
  }

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ring pipeline: chunks q+1 .. q+NSTAGE-2 stay in flight across the barrier (counted vmcnt, raw
  // s_barrier -- __syncthreads() would drain every DMA with vmcnt(0))
  constexpr int PER = 2 * NI;  // DMA instructions per wave per chunk
#pragma unroll
  for (int s_ = 0; s_ < NSTAGE - 1; ++s_) IC2_IG_ISSUE(s_ < a.nq ? s_ : a.nq - 1, s_);

  const int fr = lane & 15;
  const int fh = lane >> 4;

  for (int q = 0; q < a.nq; ++q) {
    const int cur = q % NSTAGE;
    if constexpr (NSTAGE == 4) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NSTAGE - 2) * PER) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // chunk q landed for every wave; chunk q-1 fully read
    __builtin_amdgcn_sched_barrier(0);
    {
      const int qn = q + NSTAGE - 1;
      IC2_IG_ISSUE(qn < a.nq ? qn : a.nq - 1, qn % NSTAGE);  // refill the slot chunk q-1 used
    }
    __builtin_amdgcn_sched_barrier(0);
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
    __builtin_amdgcn_sched_barrier(0);  // every MFMA of this chunk before the next wait
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the redundant tail DMAs before exit

#undef IC2_IG_ISSUE
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
