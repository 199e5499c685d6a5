// Backward of the fused filtered leaky-ReLU on NHWC activations: the synthesis layers' gradient w.r.t. their
// conv output when the reference trains its encoder through the frozen generator
// (/root/reference/stylegan3_hvae_full.py:669-696; SG3-public filtered_lrelu, whose backward is the adjoint of
// upfirdn2d(fu, up) -> lrelu*gain, clamp -> upfirdn2d(fd, down)).
//
// Per axis, with g_u[t] = fu[tu-1-t] * up (flipped, the per-axis share of the up^2 gain) and g_d[t] = fd[td-1-t]:
//   forward   U[k]  = sum_t g_u[t] * xp[k + t]        xp = x zero-inserted by `up`, shifted by p0
//             out[o] = sum_t g_d[t] * V[o*down + t]    V = clamp(gain * lrelu(U), +-clamp)
//   backward  gV[k] = sum_{o : 0 <= k - o*down < td} g_d[k - o*down] * gout[o]
//             gU[k] = gV[k] * gain * (U > 0 ? 1 : slope) * (|V| < clamp)        (U recomputed from x)
//             gx[i] = sum_{k : 0 <= i*up + p0 - k < tu} g_u[i*up + p0 - k] * gU[k]
// One workgroup = one (sample, TIY x TIX tile of gx, NP channel pairs).  With the tile's first lrelu-grid row
// k0 = i0*up + p0 - tu + 1 every polyphase tap index is a compile-time function of the local row/column
// (x rows start at i0 - tu/up + 1; gout rows at (k0 - td + 1 + ph) / down with the phase folded into R), so the
// FIR loops unroll completely and zero-inserted samples are never touched:
//   stage A  vertical passes: x columns -> up-FIR rows of U (LDS a_v); gout columns -> up-by-down FIR rows of gV
//            (LDS b_v)
//   stage B  per grid row: horizontal up-FIR (U), horizontal up-by-down FIR (gV), gU = gV * act'(U), horizontal
//            down-by-up FIR -> written back over the thread's own a_v row
//   stage C  per column: vertical down-by-up FIR -> gx (f32) -> global
// f32 arithmetic throughout (the gradient is returned in f32 whatever the forward's storage dtype).
#include "common.h"
#include "flrelu.h"

#include <cstdlib>

namespace ic2 {

int flrelu_bwd_mfma_launch(const void* x, const void* gout, void* gx, const float* oscale, const float* bias,
                           float* ydot, int64_t ydot_floats, int n, int c_p, int in_h, int in_w, int out_h, int out_w,
                           const float* gu, const float* gd, int up, int p0, float gain, float slope, float lim,
                           bool grad_f16, hipStream_t s);

typedef float bf2v __attribute__((ext_vector_type(2)));
typedef _Float16 hh2v __attribute__((ext_vector_type(2)));

struct FlrBwdArgs {
  const void* x;     // conv output that fed the forward (NHWC [n][in_h][in_w][c_p], f32 or f16)
  const void* gout;  // gradient of the layer output (NHWC [n][out_h][out_w][c_p], f32 or bf16)
  void* gx;          // gradient of x (NHWC, f32; or bf16 when out_bf16), times oscale[n][c] when oscale is set
  const float* oscale;  // [n][c_p] or null
  const float* bias;    // [c_p] or null: x = conv * oscale + bias (for the ydot partials)
  float* ydot;          // [n][tiles][c_p] per-tile sum of gx * (x - bias), or null
  int out_bf16;
  int c_p;
  int in_h, in_w, out_h, out_w;
  int p0;            // leading padding (px0 == py0)
  int tiles_x, tiles_y, cblocks;
  float slope, gain, lim;  // lim = clamp / gain (+inf: no clamp)
  float gu[24];
  float gd[12];
};

template <typename T> __device__ __forceinline__ bf2v ldp(const T* p, bool ok);
template <> __device__ __forceinline__ bf2v ldp<float>(const float* p, bool ok) {
  const float2 v = *reinterpret_cast<const float2*>(ok ? (const void*)p : zero_line());
  return bf2v{v.x, v.y};
}
template <> __device__ __forceinline__ bf2v ldp<_Float16>(const _Float16* p, bool ok) {
  const uint32_t u = *reinterpret_cast<const uint32_t*>(ok ? (const void*)p : zero_line());
  const hh2v h = __builtin_bit_cast(hh2v, u);
  return bf2v{(float)h.x, (float)h.y};
}
template <> __device__ __forceinline__ bf2v ldp<bf16_t>(const bf16_t* p, bool ok) {
  const uint32_t u = *reinterpret_cast<const uint32_t*>(ok ? (const void*)p : zero_line());
  return bf2v{__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u)};
}

__device__ __forceinline__ float dact(float u, float slope, float gain, float lim) {
  const float l = u > 0.f ? u : u * slope;
  return fabsf(l) < lim ? (u > 0.f ? gain : gain * slope) : 0.f;
}

template <int UP, int DN, int TU, int TD, int TIY, int TIX>
struct FbGeom {
  static constexpr int KY = (TIY - 1) * UP + TU;   // lrelu-grid rows feeding the tile
  static constexpr int KX = (TIX - 1) * UP + TU;
  static constexpr int NJY = TIY + 2 * (TU / UP) - 2;  // x rows / columns feeding them
  static constexpr int NJX = TIX + 2 * (TU / UP) - 2;
};

template <typename TI, typename TG, int UP, int DN, int TU, int TD, int R, int TIY, int TIX, int NP, int NT>
__global__ void __launch_bounds__(NT) flrelu_bwd_kernel(FlrBwdArgs a) {
  static_assert(TU % UP == 0 && TD % DN == 0 && UP % DN == 0, "polyphase loops assume whole phases");
  using G = FbGeom<UP, DN, TU, TD, TIY, TIX>;
  constexpr int KY = G::KY, KX = G::KX, NJY = G::NJY, NJX = G::NJX;
  constexpr int NOY = (R + KY - 1) / DN + 1;  // gout rows / columns feeding the grid rows
  constexpr int NOX = (R + KX - 1) / DN + 1;
  constexpr int PA = NJX | 1, PB = NOX | 1;   // odd row pitches
  __shared__ __attribute__((aligned(16))) bf2v a_v[KY * PA * NP];
  __shared__ __attribute__((aligned(16))) bf2v b_v[KY * PB * NP];

  int bid = blockIdx.x;
  const int cb = bid % a.cblocks;
  bid /= a.cblocks;
  const int tx = bid % a.tiles_x;
  bid /= a.tiles_x;
  const int ty = bid % a.tiles_y;
  const int n = bid / a.tiles_y;
  const int i0y = ty * TIY, i0x = tx * TIX;
  const int j0y = i0y - TU / UP + 1, j0x = i0x - TU / UP + 1;
  // first gout row / column: (k0 - td + 1 + ph) / down, exact (R = td - 1 - ph)
  const int o0y = (i0y * UP + a.p0 - TU + 1 - R) / DN;
  const int o0x = (i0x * UP + a.p0 - TU + 1 - R) / DN;
  const int c0 = cb * 2 * NP;
  const TI* __restrict__ xin = reinterpret_cast<const TI*>(a.x) + (int64_t)n * a.in_h * a.in_w * a.c_p;
  const TG* __restrict__ gin = reinterpret_cast<const TG*>(a.gout) + (int64_t)n * a.out_h * a.out_w * a.c_p;

  // ---------------- stage A: vertical passes
  for (int item = threadIdx.x; item < (NJX + NOX) * NP; item += NT) {
    const int col = item / NP;
    const int p = item - col * NP;
    const int c = c0 + 2 * p;
    if (col < NJX) {
      const int ix = j0x + col;
      const bool cok = (unsigned)ix < (unsigned)a.in_w;
      const TI* pc = xin + (int64_t)ix * a.c_p + c;
      bf2v in[NJY];
#pragma unroll
      for (int j = 0; j < NJY; ++j) {
        const int iy = j0y + j;
        const bool ok = cok && (unsigned)iy < (unsigned)a.in_h;
        const bf2v v = ldp<TI>(pc + (int64_t)iy * a.in_w * a.c_p, ok);
        in[j] = ok ? v : bf2v{0.f, 0.f};
      }
#pragma unroll
      for (int k = 0; k < KY; ++k) {
        bf2v acc = bf2v{0.f, 0.f};
#pragma unroll
        for (int m = 0; m < TU / UP; ++m) {
          const int j = k / UP + m;
          const int t = (j + 1) * UP - 1 - k;
          if (j < NJY && t >= 0 && t < TU) acc += a.gu[t] * in[j];
        }
        a_v[(k * PA + col) * NP + p] = acc;
      }
    } else {
      const int oc = col - NJX;
      const int ox = o0x + oc;
      const bool cok = (unsigned)ox < (unsigned)a.out_w;
      const TG* pc = gin + (int64_t)ox * a.c_p + c;
      bf2v in[NOY];
#pragma unroll
      for (int o = 0; o < NOY; ++o) {
        const int oy = o0y + o;
        const bool ok = cok && (unsigned)oy < (unsigned)a.out_h;
        const bf2v v = ldp<TG>(pc + (int64_t)oy * a.out_w * a.c_p, ok);
        in[o] = ok ? v : bf2v{0.f, 0.f};
      }
#pragma unroll
      for (int k = 0; k < KY; ++k) {
        bf2v acc = bf2v{0.f, 0.f};
#pragma unroll
        for (int m = 0; m < TD / DN; ++m) {
          const int o = (R + k) / DN - m;
          const int t = R + k - o * DN;
          if (o >= 0 && o < NOY && t < TD) acc += a.gd[t] * in[o];
        }
        b_v[(k * PB + oc) * NP + p] = acc;
      }
    }
  }
  __syncthreads();

  // ---------------- stage B: horizontal passes per grid row
  for (int item = threadIdx.x; item < KY * NP; item += NT) {
    const int k = item / NP;
    const int p = item - k * NP;
    bf2v ua[NJX], gb[NOX], ch[TIX];
#pragma unroll
    for (int j = 0; j < NJX; ++j) ua[j] = a_v[(k * PA + j) * NP + p];
#pragma unroll
    for (int o = 0; o < NOX; ++o) gb[o] = b_v[(k * PB + o) * NP + p];
#pragma unroll
    for (int i = 0; i < TIX; ++i) ch[i] = bf2v{0.f, 0.f};
#pragma unroll
    for (int kx = 0; kx < KX; ++kx) {
      bf2v u = bf2v{0.f, 0.f}, g = bf2v{0.f, 0.f};
#pragma unroll
      for (int m = 0; m < TU / UP; ++m) {
        const int j = kx / UP + m;
        const int t = (j + 1) * UP - 1 - kx;
        if (j < NJX && t >= 0 && t < TU) u += a.gu[t] * ua[j];
      }
#pragma unroll
      for (int m = 0; m < TD / DN; ++m) {
        const int o = (R + kx) / DN - m;
        const int t = R + kx - o * DN;
        if (o >= 0 && o < NOX && t < TD) g += a.gd[t] * gb[o];
      }
      g.x *= dact(u.x, a.slope, a.gain, a.lim);
      g.y *= dact(u.y, a.slope, a.gain, a.lim);
#pragma unroll
      for (int m = 0; m < TU / UP; ++m) {  // outputs i with 0 <= i*UP + TU - 1 - kx < TU
        const int i = (kx - TU + UP + UP * TU) / UP - TU + m;  // ceil((kx - TU + 1) / UP) + m, kept >= 0 inside
        const int t = i * UP + TU - 1 - kx;
        if (i >= 0 && i < TIX && t >= 0 && t < TU) ch[i] += a.gu[t] * g;
      }
    }
#pragma unroll
    for (int i = 0; i < TIX; ++i) a_v[(k * PA + i) * NP + p] = ch[i];
  }
  __syncthreads();

  // ---------------- stage C: vertical down-by-up pass per column, store
  // Optional epilogue (the modulated conv's backward, x = conv * oscale + bias): gx * oscale is stored (bf16 for
  // the dgrad GEMM), and sum gx * (x - bias) over the tile goes to ydot -> d oscale = sum / oscale on the host.
  constexpr int S3 = (TIY % 2 == 0 && TIX * NP * 2 <= NT) ? 2 : 1;
  constexpr int RG = TIY / S3;
  constexpr int RGK = (RG - 1) * UP + TU;
  constexpr int NITEM = TIX * NP * S3;
  static_assert(NITEM <= NT, "stage C: one item per thread");
  bf2v ydp = bf2v{0.f, 0.f};
  const int item = threadIdx.x;
  const int p = item % NP;
  const int c = c0 + 2 * p;
  if (item < NITEM) {
    const int ix = (item / NP) % TIX;
    const int rg = item / (NP * TIX);
    const int gxx = i0x + ix;
    if (gxx < a.in_w) {
      bf2v o[RG];
#pragma unroll
      for (int r = 0; r < RG; ++r) o[r] = bf2v{0.f, 0.f};
      const int kb = rg * RG * UP;
#pragma unroll
      for (int kk = 0; kk < RGK; ++kk) {
        const bf2v v = a_v[((kb + kk) * PA + ix) * NP + p];
#pragma unroll
        for (int m = 0; m < TU / UP; ++m) {
          const int r = (kk - TU + UP + UP * TU) / UP - TU + m;
          const int t = r * UP + TU - 1 - kk;
          if (r >= 0 && r < RG && t >= 0 && t < TU) o[r] += a.gu[t] * v;
        }
      }
      bf2v os = bf2v{1.f, 1.f}, bi = bf2v{0.f, 0.f};
      if (a.oscale) os = bf2v{a.oscale[(int64_t)n * a.c_p + c], a.oscale[(int64_t)n * a.c_p + c + 1]};
      if (a.bias) bi = bf2v{a.bias[c], a.bias[c + 1]};
      // the ydot operand x of every row BEFORE the first gx store: a load placed after a store to gx may alias
      // it, which serialised one round trip per row (vmcnt(0) per row in the up-4 instances)
      if (a.ydot) {
        bf2v xv[RG];
#pragma unroll
        for (int r = 0; r < RG; ++r) {
          const int gyy = i0y + rg * RG + r;
          xv[r] = ldp<TI>(xin + ((int64_t)gyy * a.in_w + gxx) * a.c_p + c, gyy < a.in_h);
        }
#pragma unroll
        for (int r = 0; r < RG; ++r)
          if (i0y + rg * RG + r < a.in_h) ydp += o[r] * (xv[r] - bi);
      }
#pragma unroll
      for (int r = 0; r < RG; ++r) {
        const int gyy = i0y + rg * RG + r;
        if (gyy >= a.in_h) continue;
        const int64_t e = ((int64_t)gyy * a.in_w + gxx) * a.c_p + c;
        const bf2v v = o[r] * os;
        if (a.out_bf16) {
          bf16_t* po = reinterpret_cast<bf16_t*>(a.gx) + (int64_t)n * a.in_h * a.in_w * a.c_p + e;
          *reinterpret_cast<uint32_t*>(po) = (uint32_t)f2bf(v.x) | ((uint32_t)f2bf(v.y) << 16);
        } else {
          float* po = reinterpret_cast<float*>(a.gx) + (int64_t)n * a.in_h * a.in_w * a.c_p + e;
          *reinterpret_cast<float2*>(po) = make_float2(v.x, v.y);
        }
      }
    }
  }
  if (a.ydot) {  // fixed-order reduction of the tile's items per channel pair (LDS reused after a barrier)
    __syncthreads();
    if (item < NITEM) a_v[item] = ydp;
    __syncthreads();
    if (item < NP) {
      bf2v t = bf2v{0.f, 0.f};
      for (int k = item; k < NITEM; k += NP) t += a_v[k];
      const int tile = ty * a.tiles_x + tx;
      float* py = a.ydot + ((int64_t)n * a.tiles_y * a.tiles_x + tile) * a.c_p + c;
      py[0] = t.x;
      py[1] = t.y;
    }
  }
}

template <int UP, int DN, int TU, int TD, int R, int TIY, int TIX, int NP, int NT>
static void fb_launch(const FlrBwdArgs& a, int ti, int tg, int grid, hipStream_t s) {
#define IC2_FB(TI_, TG_) \
  hipLaunchKernelGGL((flrelu_bwd_kernel<TI_, TG_, UP, DN, TU, TD, R, TIY, TIX, NP, NT>), dim3(grid), dim3(NT), 0, s, a)
  if (ti == IC2_F32 && tg == IC2_F32) IC2_FB(float, float);
  else if (ti == IC2_F32) IC2_FB(float, bf16_t);
  else if (tg == IC2_F32) IC2_FB(_Float16, float);
  else IC2_FB(_Float16, bf16_t);
#undef IC2_FB
}

}  // namespace ic2

using namespace ic2;

extern "C" int64_t ic2_flrelu_bwd_ydot_floats(int n, int c_p, int in_h, int in_w, int up) {
  const int tiy = 16, tix = 16;  // the default tile variant
  (void)up;
  return (int64_t)n * ceil_div(in_h, tiy) * ceil_div(in_w, tix) * c_p;
}

extern "C" int ic2_flrelu_bwd_nhwc_ex(const void* x, int x_dtype, const void* gout, int g_dtype, void* gx,
                                      int gx_dtype, int n, int c_p, int in_h, int in_w, int out_h, int out_w,
                                      const float* fu, int fu_taps, const float* fd, int fd_taps, int up, int down,
                                      int px0, int px1, int py0, int py1, float gain, float slope, float clamp,
                                      int flip, const float* oscale, const float* bias, float* ydot,
                                      int64_t ydot_floats, void* stream) {
  IC2_CHECK_ARG(x && gout && gx && fu && fd, "flrelu_bwd_nhwc: null pointer");
  IC2_CHECK_ARG(n > 0 && c_p > 0 && in_h > 0 && in_w > 0, "flrelu_bwd_nhwc: bad geometry");
  IC2_CHECK_ARG(x_dtype == IC2_F32 || x_dtype == IC2_F16, "flrelu_bwd_nhwc: x must be f32 or f16");
  IC2_CHECK_ARG(g_dtype == IC2_F32 || g_dtype == IC2_BF16 || g_dtype == IC2_F16,
                "flrelu_bwd_nhwc: gout must be f32, bf16 or f16");
  const int ew = (in_w * up + (px0 + px1) - (fu_taps - 1) - (fd_taps - 1) + (down - 1)) / down;
  const int eh = (in_h * up + (py0 + py1) - (fu_taps - 1) - (fd_taps - 1) + (down - 1)) / down;
  IC2_CHECK_ARG(out_h == eh && out_w == ew && out_h > 0, "flrelu_bwd_nhwc: output %dx%d, expected %dx%d", out_h, out_w,
                eh, ew);
  IC2_CHECK_ARG(px0 == py0, "flrelu_bwd_nhwc: needs px0 == py0");
  IC2_CHECK_ARG(slope >= 0.f && slope <= 1.f && gain > 0.f, "flrelu_bwd_nhwc: needs 0 <= slope <= 1, gain > 0");
  const bool cfg2 = up == 2 && down == 2 && fu_taps == 12 && fd_taps == 12;
  const bool cfg4 = up == 4 && down == 2 && fu_taps == 24 && fd_taps == 12;
  if (!cfg2 && !cfg4) {
    set_error("flrelu_bwd_nhwc: no instance for up=%d down=%d taps=%d/%d (StyleGAN3-T: up 2/4, down 2, 6*up / 12 taps)",
              up, down, fu_taps, fd_taps);
    return IC2_E_UNSUPPORTED;
  }
  IC2_CHECK_ARG(gx_dtype == IC2_F32 || gx_dtype == IC2_BF16 || gx_dtype == IC2_F16,
                "flrelu_bwd_nhwc: gx must be f32, bf16 or f16");
  // f16 gradients (the f16 training path, loss-scaled): the MFMA kernel's f16-operand instance only
  IC2_CHECK_ARG((g_dtype == IC2_F16) == (gx_dtype == IC2_F16) && (g_dtype != IC2_F16 || x_dtype == IC2_F16),
                "flrelu_bwd_nhwc: f16 gradients need f16 x, f16 gout and f16 gx");
  FlrBwdArgs a;
  a.x = x; a.gout = gout; a.gx = gx;
  a.oscale = oscale; a.bias = bias; a.ydot = ydot; a.out_bf16 = gx_dtype == IC2_BF16;
  a.c_p = c_p; a.in_h = in_h; a.in_w = in_w; a.out_h = out_h; a.out_w = out_w; a.p0 = px0;
  a.slope = slope; a.gain = gain; a.lim = clamp >= 0.f ? clamp / gain : INFINITY;
  for (int t = 0; t < 24; ++t) a.gu[t] = 0.f;
  for (int t = 0; t < 12; ++t) a.gd[t] = 0.f;
  for (int t = 0; t < fu_taps; ++t) a.gu[t] = (flip ? fu[t] : fu[fu_taps - 1 - t]) * (float)up;
  for (int t = 0; t < fd_taps; ++t) a.gd[t] = flip ? fd[t] : fd[fd_taps - 1 - t];
  // the bf16 training path (f16 x, bf16 gout and gx): the MFMA kernel (flrelu_bwd_mfma.hip) unless knob
  // IC2_FLRB_MFMA=0; ydot from the stored gx there
  static const bool mfma = knob("IC2_FLRB_MFMA", 1) != 0;
  const bool gf16 = g_dtype == IC2_F16;
  if ((mfma || gf16) && x_dtype == IC2_F16 && ((g_dtype == IC2_BF16 && gx_dtype == IC2_BF16) || gf16)) {
    const int64_t need = (int64_t)n * ceil_div(in_h, 16) * ceil_div(in_w, 16) * c_p;
    IC2_CHECK_ARG(ydot == nullptr || ydot_floats >= need, "flrelu_bwd_nhwc: ydot needs %lld floats", (long long)need);
    // U is recomputed with f16 taps rounded as the forward rounds its vertical taps (joint per-phase rounding, ADVICE
    // r3), so the lrelu side is decided on the forward's operands.  With a finite clamp the forward's horizontal up pass
    // runs on separately rounded taps gu / lim (its clamp-split activation, flrelu_mfma.hip) and compares with 1, so an
    // element within an f16 rounding of the clamp boundary can take the other clamp decision here than in the forward
    // (its gradient is then 0 instead of gain, or the reverse) -- ADVICE r4; elsewhere the decisions agree.
    float gur[24] = {}, gdr[12] = {};
    f16_round_taps(a.gu, gur, fu_taps, up);
    f16_round_taps(a.gd, gdr, fd_taps, 1);
    const int rc = flrelu_bwd_mfma_launch(x, gout, gx, oscale, bias, ydot, need, n, c_p, in_h, in_w, out_h, out_w, gur,
                                          gdr, up, px0, gain, slope, a.lim, gf16, as_stream(stream));
    if (rc == IC2_OK) {
      IC2_CHECK_LAUNCH("flrelu_bwd_nhwc (mfma)");
      return IC2_OK;
    }
    if (rc != IC2_E_UNSUPPORTED || gf16) return rc;
  }
  // gout phase: R = td - 1 - ph with ph = (-(p0 - tu + 1 - td + 1)) mod down (up % down == 0: same for every tile)
  const int q = px0 - fu_taps + 1 - fd_taps + 1;
  const int ph = ((-q) % down + down) % down;
  const int R = fd_taps - 1 - ph;
  // tile variants (TIY, TIX, channel pairs, threads); knob IC2_FLRB_VARIANT=k picks one (tuning, tools/bench_flr_bwd.py)
  static const int variant = knob("IC2_FLRB_VARIANT", -1);
  const int v = variant >= 0 ? variant : 1;   // 16x16 tiles: fastest on every SG3-T-256 layer (profiles/r2_flr_bwd_variants.txt)
  int tiy, tix, np;
  if (v == 1) { tiy = 16; tix = 16; np = cfg2 ? 2 : 1; }
  else if (v == 2) { tiy = 8; tix = 16; np = cfg2 ? 2 : 1; }
  else { tiy = cfg2 ? 8 : 4; tix = cfg2 ? 16 : 8; np = 4; }
  a.tiles_x = (int)ceil_div(in_w, tix);
  a.tiles_y = (int)ceil_div(in_h, tiy);
  IC2_CHECK_ARG(c_p % (2 * np) == 0, "flrelu_bwd_nhwc: c_p must be a multiple of %d", 2 * np);
  a.cblocks = c_p / (2 * np);
  const int64_t grid = (int64_t)n * a.tiles_y * a.tiles_x * a.cblocks;
  IC2_CHECK_ARG(grid < (1LL << 31), "flrelu_bwd_nhwc: grid too large");
  IC2_CHECK_ARG(ydot == nullptr || (v == 1 && ydot_floats >= (int64_t)n * a.tiles_y * a.tiles_x * c_p),
                "flrelu_bwd_nhwc: ydot needs the default tiles and %lld floats",
                (long long)((int64_t)n * a.tiles_y * a.tiles_x * c_p));
  hipStream_t s = as_stream(stream);
#define IC2_FB_R(U_, TU_, TIY_, TIX_, NP_, NT_)                                                     \
  do {                                                                                              \
    if (R == 11) fb_launch<U_, 2, TU_, 12, 11, TIY_, TIX_, NP_, NT_>(a, x_dtype, g_dtype, (int)grid, s); \
    else fb_launch<U_, 2, TU_, 12, 10, TIY_, TIX_, NP_, NT_>(a, x_dtype, g_dtype, (int)grid, s);         \
  } while (0)
  if (cfg2) {
    if (v == 1) IC2_FB_R(2, 12, 16, 16, 2, 128);
    else if (v == 2) IC2_FB_R(2, 12, 8, 16, 2, 64);
    else IC2_FB_R(2, 12, 8, 16, 4, 128);
  } else {
    if (v == 1) IC2_FB_R(4, 24, 16, 16, 1, 128);
    else if (v == 2) IC2_FB_R(4, 24, 8, 16, 1, 64);
    else IC2_FB_R(4, 24, 4, 8, 4, 128);
  }
#undef IC2_FB_R
  IC2_CHECK_LAUNCH("flrelu_bwd_nhwc");
  return IC2_OK;
}


extern "C" int ic2_flrelu_bwd_nhwc(const void* x, int x_dtype, const void* gout, int g_dtype, float* gx, int n, int c_p,
                                   int in_h, int in_w, int out_h, int out_w, const float* fu, int fu_taps,
                                   const float* fd, int fd_taps, int up, int down, int px0, int px1, int py0, int py1,
                                   float gain, float slope, float clamp, int flip, void* stream) {
  return ic2_flrelu_bwd_nhwc_ex(x, x_dtype, gout, g_dtype, gx, IC2_F32, n, c_p, in_h, in_w, out_h, out_w, fu, fu_taps, fd,
                                fd_taps, up, down, px0, px1, py0, py1, gain, slope, clamp, flip, nullptr, nullptr,
                                nullptr, 0, stream);
}
