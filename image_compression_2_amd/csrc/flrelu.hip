// Fused filtered leaky-ReLU [SG3-public: torch_utils/ops/filtered_lrelu.py, whose reference path is
//   bias_act(b) -> upfirdn2d(fu, up, padding, gain=up^2) -> bias_act(lrelu, slope, gain, clamp)
//   -> upfirdn2d(fd, down)]; called by SynthesisLayer.forward for every layer of
// G.synthesis (/root/reference/stylegan3_hvae_full.py:274,329).
//
// One workgroup = one (sample, 16x16 output tile (NHWC bf16; 24x8 otherwise), 16-channel block).  Lanes own channel PAIRS
// (packed fp32 math, bf16x2 loads), the spatial FIR runs from registers with every tap index
// resolved at compile time (polyphase: zero-inserted samples are never multiplied), and the
// up-sampled grid lives only in LDS:
//   stage 1  vertical up-FIR   : input column (registers)        -> LDS  a_v[RAY][NINX]
//   stage 2  horizontal up-FIR : LDS row -> lrelu*gain, clamp -> horizontal down-FIR (registers)
//                                -> written back over the thread's own LDS row (no barrier)
//   stage 3  vertical down-FIR : LDS column -> * post_scale -> global
// Filters are separable 1-D taps (the StyleGAN3-T configuration).  Zero padding / negative
// padding (crop) is exact: input samples outside [0, L) are zero, as in the reference.
#include "flrelu.h"

#include <cmath>

#include <cstdlib>
#include <type_traits>

namespace ic2 {

typedef float f2v __attribute__((ext_vector_type(2)));

template <int U, int D, int TU, int TD, int TOY, int TOX>
struct FlrGeom {
  static constexpr int RAY = (TOY - 1) * D + TD;       // lrelu-grid rows of one tile
  static constexpr int RAX = (TOX - 1) * D + TD;
  static constexpr int NINY = (RAY + TU - 2) / U + 1;  // input rows feeding them
  static constexpr int NINX = (RAX + TU - 2) / U + 1;
  static constexpr int NINXP = NINX | 1;               // odd row pitch: conflict-free ds_read_b64
};

// Branch-free pair access: an out-of-range sample reads the code object's zero line and is then
// masked, so no load sits behind a branch (hipcc would otherwise wait vmcnt(0) per element).
template <typename T, bool CHLAST>
__device__ __forceinline__ f2v load2(const T* p, int64_t sc, bool ok, bool ok2);
template <> __device__ __forceinline__ f2v load2<float, true>(const float* p, int64_t, bool ok, bool) {
  const float2 v = *reinterpret_cast<const float2*>(ok ? (const void*)p : zero_line());
  return f2v{v.x, v.y};
}
template <> __device__ __forceinline__ f2v load2<bf16_t, true>(const bf16_t* p, int64_t, bool ok, bool) {
  const uint32_t v = *reinterpret_cast<const uint32_t*>(ok ? (const void*)p : zero_line());
  return f2v{__uint_as_float(v << 16), __uint_as_float(v & 0xffff0000u)};
}
template <> __device__ __forceinline__ f2v load2<float, false>(const float* p, int64_t sc, bool ok, bool ok2) {
  const float a = *reinterpret_cast<const float*>(ok ? (const void*)p : zero_line());
  const float b = *reinterpret_cast<const float*>(ok && ok2 ? (const void*)(p + sc) : zero_line());
  return f2v{a, b};
}
template <> __device__ __forceinline__ f2v load2<bf16_t, false>(const bf16_t* p, int64_t sc, bool ok, bool ok2) {
  const bf16_t a = *reinterpret_cast<const bf16_t*>(ok ? (const void*)p : zero_line());
  const bf16_t b = *reinterpret_cast<const bf16_t*>(ok && ok2 ? (const void*)(p + sc) : zero_line());
  return f2v{bf2f(a), bf2f(b)};
}
template <typename T, bool CHLAST> __device__ __forceinline__ void store2(T* p, int64_t sc, bool ok2, f2v v);
template <> __device__ __forceinline__ void store2<float, true>(float* p, int64_t, bool, f2v v) {
  *reinterpret_cast<float2*>(p) = make_float2(v.x, v.y);
}
template <> __device__ __forceinline__ void store2<bf16_t, true>(bf16_t* p, int64_t, bool, f2v v) {
  *reinterpret_cast<uint32_t*>(p) = (uint32_t)f2bf(v.x) | ((uint32_t)f2bf(v.y) << 16);
}
template <> __device__ __forceinline__ void store2<float, false>(float* p, int64_t sc, bool ok2, f2v v) {
  p[0] = v.x;
  if (ok2) p[sc] = v.y;
}
template <> __device__ __forceinline__ void store2<bf16_t, false>(bf16_t* p, int64_t sc, bool ok2, f2v v) {
  p[0] = f2bf(v.x);
  if (ok2) p[sc] = f2bf(v.y);
}

// LDS storage of the up-sampled grid: fp32 pairs (parity path) or packed bf16 pairs (bf16 path:
// halves the LDS footprint -> twice the resident workgroups; one extra rounding of the vertically
// up-sampled input, below the bf16 rounding of the output itself).
template <typename LT> struct LdsPair;
template <> struct LdsPair<f2v> {
  __device__ static __forceinline__ f2v pack(f2v v) { return v; }
  __device__ static __forceinline__ f2v unpack(f2v v) { return v; }
};
template <> struct LdsPair<uint32_t> {
  __device__ static __forceinline__ uint32_t pack(f2v v) { return (uint32_t)f2bf(v.x) | ((uint32_t)f2bf(v.y) << 16); }
  __device__ static __forceinline__ f2v unpack(uint32_t v) {
    return f2v{__uint_as_float(v << 16), __uint_as_float(v & 0xffff0000u)};
  }
};

// lrelu + clamp on a channel pair in 5 instructions: one packed multiply, two max (slope <= 1 makes
// lrelu(v) = max(v, slope*v)) and two med3 clamps.  The gain is folded into the horizontal down taps
// and the clamp bound divided by it: clamp(gain*lrelu(v), +-c) = gain * clamp(lrelu(v), +-c/gain).
__device__ __forceinline__ f2v act2(f2v v, float slope, float lim) {
  const f2v sv = v * slope;
  f2v r;
  r.x = __builtin_amdgcn_fmed3f(fmaxf(v.x, sv.x), -lim, lim);
  r.y = __builtin_amdgcn_fmed3f(fmaxf(v.y, sv.y), -lim, lim);
  return r;
}

constexpr int FLR_S3 = 4;                // stage-3 row split (items = columns x pairs x FLR_S3)

// First input sample j whose up-FIR tap t = U*j + DELTA - i lies in [0, TU): j = ceil((i - DELTA) / U),
// clamped at 0.  The TU/U samples j, j+1, ... are exactly the polyphase taps of grid position i.
template <int U, int DELTA>
__host__ __device__ constexpr int up_first(int i) {
  return i < DELTA ? 0 : (i - DELTA + U - 1) / U;
}

template <typename TI, typename TO, bool CHLAST, int U, int D, int TU, int TD, int DELTA, int TOY, int TOX, int FLR_CPB,
          int FLR_THREADS>
__global__ void __launch_bounds__(FLR_THREADS) __attribute__((amdgpu_waves_per_eu(4))) flrelu_kernel(FlrArgs a) {
  constexpr int FLR_NCG = FLR_CPB / 2;  // channel pairs per workgroup
  static_assert(TU % U == 0 && TD % D == 0, "polyphase loops assume whole phases");
  using G = FlrGeom<U, D, TU, TD, TOY, TOX>;
  using LT = typename std::conditional<std::is_same<TI, bf16_t>::value, uint32_t, f2v>::type;
  using LP = LdsPair<LT>;
  constexpr int RAY = G::RAY, RAX = G::RAX, NINY = G::NINY, NINX = G::NINX, NINXP = G::NINXP;
  constexpr int NCG = FLR_NCG;
  __shared__ __attribute__((aligned(16))) LT buf[RAY * NINXP * NCG];

  int bid = blockIdx.x;
  const int cb = bid % a.cblocks;
  bid /= a.cblocks;
  const int tx = bid % a.tiles_x;
  bid /= a.tiles_x;
  const int ty = bid % a.tiles_y;
  const int n = bid / a.tiles_y;

  const int oy0 = ty * TOY, ox0 = tx * TOX;
  // first input sample feeding the tile: s_lo = (ka - p0 + DELTA) / U with ka = o0 * D
  const int sy0 = (oy0 * D - a.py0 + DELTA) / U;
  const int sx0 = (ox0 * D - a.px0 + DELTA) / U;
  const int c0 = cb * FLR_CPB;

  const TI* __restrict__ xin = reinterpret_cast<const TI*>(a.x) + (int64_t)n * a.xsn;
  TO* __restrict__ yout = reinterpret_cast<TO*>(a.y) + (int64_t)n * a.ysn;

  // ---------------- stage 1: vertical up-FIR of NINX input columns
  for (int item = threadIdx.x; item < NINX * NCG; item += FLR_THREADS) {
    const int xs = item / NCG;
    const int cg = item - xs * NCG;
    const int c = c0 + 2 * cg;
    const int ix = sx0 + xs;
    const bool col_ok = (unsigned)ix < (unsigned)a.in_w && c < a.c;
    const bool ok2 = c + 1 < a.c;
    f2v bsum = f2v{0.f, 0.f};
    if (a.bias) {
      const int cc = col_ok ? c : 0;
      bsum = f2v{a.bias[cc], ok2 ? a.bias[cc + 1] : 0.f};
    }
    const TI* pcol = xin + (int64_t)ix * a.xsx + (int64_t)c * a.xsc;
    f2v in[NINY];
#pragma unroll
    for (int j = 0; j < NINY; ++j) {
      const int iy = sy0 + j;
      const bool ok = col_ok && (unsigned)iy < (unsigned)a.in_h;
      const f2v v = load2<TI, CHLAST>(pcol + (int64_t)iy * a.xsy, a.xsc, ok, ok2) + bsum;
      in[j] = ok ? v : f2v{0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < RAY; ++i) {
      f2v acc = f2v{0.f, 0.f};
#pragma unroll
      for (int m = 0; m < TU / U; ++m) {  // the TU/U polyphase taps landing on grid row i
        const int j = up_first<U, DELTA>(i) + m;
        if (j < NINY) acc += a.gu[U * j + DELTA - i] * in[j];
      }
      buf[(i * NINXP + xs) * NCG + cg] = LP::pack(acc);
    }
  }
  __syncthreads();

  // ---------------- stage 2: horizontal up-FIR, activation, horizontal down-FIR per grid row
  for (int item = threadIdx.x; item < RAY * NCG; item += FLR_THREADS) {
    const int i = item / NCG;
    const int cg = item - i * NCG;
    f2v in[NINX];
#pragma unroll
    for (int j = 0; j < NINX; ++j) in[j] = LP::unpack(buf[(i * NINXP + j) * NCG + cg]);
    f2v d[TOX];
#pragma unroll
    for (int o = 0; o < TOX; ++o) d[o] = f2v{0.f, 0.f};
#pragma unroll
    for (int k = 0; k < RAX; ++k) {
      f2v v = f2v{0.f, 0.f};
#pragma unroll
      for (int m = 0; m < TU / U; ++m) {
        const int j = up_first<U, DELTA>(k) + m;
        if (j < NINX) v += a.gu[U * j + DELTA - k] * in[j];
      }
      v = act2(v, a.slope, a.lim);
#pragma unroll
      for (int m = 0; m < TD / D; ++m) {  // outputs o with 0 <= k - o*D < TD
        const int o = k / D - m;
        if (o >= 0 && o < TOX) d[o] += a.gdg[k - o * D] * v;
      }
    }
#pragma unroll
    for (int o = 0; o < TOX; ++o) buf[(i * NINXP + o) * NCG + cg] = LP::pack(d[o]);
  }
  __syncthreads();

  // ---------------- stage 3: vertical down-FIR per output column (FLR_S3 row groups), store
  static_assert(TOY % FLR_S3 == 0, "TOY must split into FLR_S3 row groups");
  constexpr int RG = TOY / FLR_S3;            // output rows per item
  constexpr int RGI = (RG - 1) * D + TD;      // grid rows feeding them
  for (int item = threadIdx.x; item < TOX * NCG * FLR_S3; item += FLR_THREADS) {
    const int cg = item % NCG;
    const int ox = (item / NCG) % TOX;
    const int rg = item / (NCG * TOX);
    const int c = c0 + 2 * cg;
    const int gx = ox0 + ox;
    if (gx >= a.out_w || c >= a.c) continue;
    const bool ok2 = c + 1 < a.c;
    f2v o[RG];
#pragma unroll
    for (int r = 0; r < RG; ++r) o[r] = f2v{0.f, 0.f};
    const int i0 = rg * RG * D;
#pragma unroll
    for (int ii = 0; ii < RGI; ++ii) {
      const f2v v = LP::unpack(buf[((i0 + ii) * NINXP + ox) * NCG + cg]);
#pragma unroll
      for (int m = 0; m < TD / D; ++m) {
        const int r = ii / D - m;
        if (r >= 0 && r < RG) o[r] += a.gd[ii - r * D] * v;
      }
    }
    f2v ps = f2v{1.f, 1.f};
    if (a.post_scale) ps = f2v{a.post_scale[(int64_t)n * a.c_p + c], ok2 ? a.post_scale[(int64_t)n * a.c_p + c + 1] : 0.f};
    TO* pout = yout + (int64_t)gx * a.ysx + (int64_t)c * a.ysc;
#pragma unroll
    for (int r = 0; r < RG; ++r) {
      const int gy = oy0 + rg * RG + r;
      if (gy < a.out_h) store2<TO, CHLAST>(pout + (int64_t)gy * a.ysy, a.ysc, ok2, o[r] * ps);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// dispatch
// ------------------------------------------------------------------------------------------------
// Tile geometries (TOY, TOX, channels per workgroup, threads).  The bf16 NHWC instances (the synthesis
// throughput path) are tuned per up-factor; every other dtype/layout uses geometry 0 only.
// IC2_FLR_VARIANT=k forces geometry k on the bf16 NHWC path (tuning, tools/bench_kernels.py).
struct FlrGeomSel {
  int toy, tox, cpb, nt;
};
static const FlrGeomSel kFlrGeoms[] = {
    {24, 8, 16, 256}, {16, 8, 16, 256}, {16, 16, 16, 256}, {8, 16, 16, 256}, {12, 16, 16, 256}, {16, 16, 8, 128}};
constexpr int kNumFlrGeoms = sizeof(kFlrGeoms) / sizeof(kFlrGeoms[0]);
static int flr_variant() {
  static const int v = [] {
    const int x = knob("IC2_FLR_VARIANT", -1);
    return (x >= 0 && x < kNumFlrGeoms) ? x : -1;
  }();
  return v;
}
static int flr_pick(bool tuned, int up) {
  if (!tuned) return 0;
  if (flr_variant() >= 0) return flr_variant();
  (void)up;
  return 2;  // 16x16 tiles: fastest on every SG3-T-256 layer but the 36^2 ones (profiles/r1_flr_variants.txt)
}

template <typename TI, typename TO, bool CHLAST, int U, int D, int TU, int TD, int DL>
static int launch_geom(const FlrArgs& a, int geom, int grid, hipStream_t s) {
#define IC2_FLR_LAUNCH(TY, TX, CPB, NT)                                                                            \
  hipLaunchKernelGGL((flrelu_kernel<TI, TO, CHLAST, U, D, TU, TD, DL, TY, TX, CPB, NT>), dim3(grid), dim3(NT), 0, s, a)
  constexpr bool tuned = CHLAST && std::is_same<TI, bf16_t>::value;
  if constexpr (tuned) {
    switch (geom) {
      case 1: IC2_FLR_LAUNCH(16, 8, 16, 256); return IC2_OK;
      case 2: IC2_FLR_LAUNCH(16, 16, 16, 256); return IC2_OK;
      case 3: IC2_FLR_LAUNCH(8, 16, 16, 256); return IC2_OK;
      case 4: IC2_FLR_LAUNCH(12, 16, 16, 256); return IC2_OK;
      case 5: IC2_FLR_LAUNCH(16, 16, 8, 128); return IC2_OK;
      default: break;
    }
  }
  if (geom != 0) return IC2_E_UNSUPPORTED;
  IC2_FLR_LAUNCH(24, 8, 16, 256);
  return IC2_OK;
#undef IC2_FLR_LAUNCH
}

template <typename TI, typename TO, bool CHLAST, int U, int D, int TU, int TD>
static int launch_delta(const FlrArgs& a, int delta, int geom, int grid, hipStream_t s) {
  switch (delta) {
    case 0: return launch_geom<TI, TO, CHLAST, U, D, TU, TD, 0>(a, geom, grid, s);
    case 1: return launch_geom<TI, TO, CHLAST, U, D, TU, TD, 1>(a, geom, grid, s);
    case 2: if constexpr (U > 2) return launch_geom<TI, TO, CHLAST, U, D, TU, TD, 2>(a, geom, grid, s); break;
    case 3: if constexpr (U > 3) return launch_geom<TI, TO, CHLAST, U, D, TU, TD, 3>(a, geom, grid, s); break;
  }
  return IC2_E_UNSUPPORTED;
}

template <typename TI, typename TO, bool CHLAST>
static int launch_cfg(const FlrArgs& a, int up, int down, int tu, int td, int delta, int geom, int grid,
                      hipStream_t s) {
  if (up == 2 && down == 2 && tu == 12 && td == 12)
    return launch_delta<TI, TO, CHLAST, 2, 2, 12, 12>(a, delta, geom, grid, s);
  if (up == 4 && down == 2 && tu == 24 && td == 12)
    return launch_delta<TI, TO, CHLAST, 4, 2, 24, 12>(a, delta, geom, grid, s);
  return IC2_E_UNSUPPORTED;
}

// The MFMA kernels run their FIRs with f16 taps.  Rounding each tap to the nearest f16 leaves every polyphase
// component's DC gain off by up to n/2 ulp, a fixed filter error that 14 layers compound (CPU emulation of the
// SG3-T-256 f16 synthesis: 52.9 dB SNR with nearest taps, 59.4 dB with these, 60.0 dB with exact taps).  So each
// group of taps that forms one output (one polyphase phase of the up filter, the whole down filter) is rounded
// jointly: every tap to one of its two f16 neighbours, chosen so the group's sum error is minimal.
static float f16_nearest(float v) { return (float)(_Float16)v; }
static float f16_step(float r, bool up) {  // the next f16 value above / below r
  uint16_t b = __builtin_bit_cast(uint16_t, (_Float16)r);
  const bool neg = b & 0x8000u;
  if ((b & 0x7fffu) == 0) return up ? 5.96046448e-8f : -5.96046448e-8f;
  b = (up != neg) ? b + 1 : b - 1;
  return (float)__builtin_bit_cast(_Float16, b);
}
void f16_round_taps(const float* exact, float* out, int n, int stride_groups) {
  // out[t] = f16-representable, per group (t mod stride_groups) sum error minimal
  for (int t = 0; t < n; ++t) out[t] = f16_nearest(exact[t]);
  for (int g = 0; g < stride_groups; ++g) {
    for (int it = 0; it < n; ++it) {
      double e = 0.0;
      for (int t = g; t < n; t += stride_groups) e += (double)out[t] - (double)exact[t];
      double best = std::fabs(e);
      int bi = -1;
      float bc = 0.f;
      for (int t = g; t < n; t += stride_groups) {
        if (exact[t] == 0.f) continue;
        for (int dir = 0; dir < 2; ++dir) {
          const float c = f16_step(out[t], dir == 0);
          if (((double)c - exact[t]) * ((double)out[t] - exact[t]) > 0.0) continue;  // not the other neighbour
          const double e2 = std::fabs(e - (double)out[t] + (double)c);
          if (e2 < best) { best = e2; bi = t; bc = c; }
        }
      }
      if (bi < 0) break;
      out[bi] = bc;
    }
  }
}

static int flrelu_common(const void* x, void* y, int dtype_in, int dtype_out, bool chlast, int n, int c, int c_p,
                         int in_h, int in_w, int out_h, int out_w, const float* fu, int fu_taps, const float* fd,
                         int fd_taps, const float* b, int up, int down, int px0, int px1, int py0, int py1,
                         float gain, float slope, float clamp, int flip, const float* post_scale, void* stream,
                         const char* name, bool in_blocked = false) {
  IC2_CHECK_ARG(x && y, "%s: null pointer", name);
  IC2_CHECK_ARG(n > 0 && c > 0 && in_h > 0 && in_w > 0 && up >= 1 && down >= 1, "%s: bad geometry", name);
  IC2_CHECK_ARG(fu_taps >= 1 && fd_taps >= 1 && fu_taps <= 24 && fd_taps <= 12, "%s: unsupported taps", name);
  const int ew = (in_w * up + (px0 + px1) - (fu_taps - 1) - (fd_taps - 1) + (down - 1)) / down;
  const int eh = (in_h * up + (py0 + py1) - (fu_taps - 1) - (fd_taps - 1) + (down - 1)) / down;
  IC2_CHECK_ARG(out_h == eh && out_w == ew, "%s: output %dx%d, expected %dx%d", name, out_h, out_w, eh, ew);
  IC2_CHECK_ARG(out_h > 0 && out_w > 0, "%s: empty output", name);
  // one polyphase offset serves both axes -> needs px0 == py0 (mod up); the fused instances exist for
  // the StyleGAN3-T configurations only
  const int dx = ((px0 % up) + up) % up, dy = ((py0 % up) + up) % up;
  if (dx != dy) {
    set_error("%s: px0 and py0 differ mod up", name);
    return IC2_E_UNSUPPORTED;
  }
  if (!(slope >= 0.f && slope <= 1.f && gain > 0.f)) {  // the fused activation uses max(v, slope*v)
    set_error("%s: fused path needs 0 <= slope <= 1 and gain > 0", name);
    return IC2_E_UNSUPPORTED;
  }
  FlrArgs a;
  a.x = x; a.y = y; a.bias = b; a.post_scale = post_scale;
  a.xcb = 16;
  if (in_blocked) {  // channel-blocked NHWC16 input: [n][c_p / 16][in_h][in_w][16]
    a.xsc = 1; a.xsx = 16; a.xsy = (int64_t)in_w * 16; a.xsn = (int64_t)in_h * in_w * c_p;
    a.xcb = (int64_t)in_h * in_w * 16;
    a.ysc = 1; a.ysx = c_p; a.ysy = (int64_t)out_w * c_p; a.ysn = (int64_t)out_h * out_w * c_p;
  } else if (chlast) {
    a.xsc = 1; a.xsx = c_p; a.xsy = (int64_t)in_w * c_p; a.xsn = (int64_t)in_h * in_w * c_p;
    a.ysc = 1; a.ysx = c_p; a.ysy = (int64_t)out_w * c_p; a.ysn = (int64_t)out_h * out_w * c_p;
  } else {
    a.xsx = 1; a.xsy = in_w; a.xsc = (int64_t)in_h * in_w; a.xsn = (int64_t)c * in_h * in_w;
    a.ysx = 1; a.ysy = out_w; a.ysc = (int64_t)out_h * out_w; a.ysn = (int64_t)c * out_h * out_w;
  }
  a.c = chlast ? c_p : c;  // NHWC: padded channels are processed too (they are zero) and stay zero
  a.c_p = c_p;
  a.in_h = in_h; a.in_w = in_w; a.out_h = out_h; a.out_w = out_w;
  a.py0 = py0; a.px0 = px0;
  hipStream_t s = as_stream(stream);
  // bf16 NHWC (the synthesis throughput path): the MFMA formulation (flrelu_mfma.hip) unless
  // knob IC2_FLR_MFMA=0 asks for the VALU kernel below
  static const bool use_mfma = knob("IC2_FLR_MFMA", 1) != 0;
  // f16 input (the synthesis conv epilogue's output) exists only for the MFMA formulation
  // (one polyphase phase for both axes: the instances take a single delta)
  const bool mfma_ok = chlast && (dtype_in == IC2_BF16 || dtype_in == IC2_F16) &&
                       (dtype_out == IC2_BF16 || dtype_out == IC2_F16) && b == nullptr && dx == dy;
  a.out_f16 = dtype_out == IC2_F16;
  if ((use_mfma || dtype_in == IC2_F16) && mfma_ok) {
    float gu[24] = {}, gd[12] = {}, gdg[12] = {};
    for (int t = 0; t < fu_taps; ++t) gu[t] = (fu ? (flip ? fu[t] : fu[fu_taps - 1 - t]) : 1.f) * (float)up;
    for (int t = 0; t < fd_taps; ++t) gd[t] = fd ? (flip ? fd[t] : fd[fd_taps - 1 - t]) : 1.f;
    for (int t = 0; t < fd_taps; ++t) gdg[t] = gd[t] * gain;
    for (int t = 0; t < 24; ++t) a.gu[t] = 0.f;
    for (int t = 0; t < 12; ++t) a.gd[t] = a.gdg[t] = 0.f;
    f16_round_taps(gu, a.gu, fu_taps, up);  // one group per polyphase phase (fu_taps = 6 * up)
    f16_round_taps(gd, a.gd, fd_taps, 1);
    f16_round_taps(gdg, a.gdg, fd_taps, 1);
    a.slope = slope;
    a.lim = clamp >= 0.f ? clamp / gain : INFINITY;
    for (int t = 0; t < 24; ++t) a.guh[t] = 0.f;
    for (int t = 0; t < 12; ++t) a.gdgl[t] = 0.f;
    if (clamp >= 0.f) {  // the clamp-split kernels' horizontal passes: u / lim and the gain * lim down taps
      float guh[24] = {}, gdgl[12] = {};
      for (int t = 0; t < fu_taps; ++t) guh[t] = gu[t] / a.lim;
      for (int t = 0; t < fd_taps; ++t) gdgl[t] = gdg[t] * a.lim;
      f16_round_taps(guh, a.guh, fu_taps, up);
      f16_round_taps(gdgl, a.gdgl, fd_taps, 1);
    }
    if (flrelu_mfma_launch(a, dtype_in == IC2_F16, up, down, fu_taps, fd_taps, dx, n, s) == IC2_OK) {
      IC2_CHECK_LAUNCH(name);
      return IC2_OK;
    }
  }
  if (in_blocked) {
    set_error("%s: channel-blocked input needs the MFMA instance (f16/bf16 in, bf16/f16 out, no bias, up 2/4 with 6*up "
              "taps, down 2 / 12 taps)", name);
    return IC2_E_UNSUPPORTED;
  }
  if (dtype_in == IC2_F16) {
    set_error("%s: f16 input needs the MFMA instance (NHWC, bf16/f16 out, no bias, up 2/4 with 6*up taps, down 2 / 12 taps)",
              name);
    return IC2_E_UNSUPPORTED;
  }
  const int geom = flr_pick(chlast && dtype_in == IC2_BF16 && dtype_out == IC2_BF16, up);
  const FlrGeomSel fv = kFlrGeoms[geom];
  a.tiles_x = (int)ceil_div(out_w, fv.tox);
  a.tiles_y = (int)ceil_div(out_h, fv.toy);
  a.cblocks = (int)ceil_div(a.c, fv.cpb);
  a.nimg = n;
  a.slope = slope;
  a.lim = clamp >= 0.f ? clamp / gain : INFINITY;
  for (int t = 0; t < 24; ++t) a.gu[t] = 0.f;
  for (int t = 0; t < 12; ++t) a.gd[t] = 0.f;
  // NOTE: fu / fd are HOST pointers here (filters are layer constants; they travel in the kernarg)
  for (int t = 0; t < fu_taps; ++t) a.gu[t] = (fu ? (flip ? fu[t] : fu[fu_taps - 1 - t]) : 1.f) * (float)up;
  for (int t = 0; t < fd_taps; ++t) a.gd[t] = fd ? (flip ? fd[t] : fd[fd_taps - 1 - t]) : 1.f;
  for (int t = 0; t < 12; ++t) a.gdg[t] = a.gd[t] * gain;
  const int64_t grid = (int64_t)n * a.tiles_y * a.tiles_x * a.cblocks;
  IC2_CHECK_ARG(grid < (1LL << 31), "%s: grid too large", name);
  int rc;
  if (dtype_in == IC2_BF16 && dtype_out == IC2_BF16)
    rc = chlast ? launch_cfg<bf16_t, bf16_t, true>(a, up, down, fu_taps, fd_taps, dx, geom, (int)grid, s)
                : launch_cfg<bf16_t, bf16_t, false>(a, up, down, fu_taps, fd_taps, dx, geom, (int)grid, s);
  else if (dtype_in == IC2_F32 && dtype_out == IC2_F32)
    rc = chlast ? launch_cfg<float, float, true>(a, up, down, fu_taps, fd_taps, dx, geom, (int)grid, s)
                : launch_cfg<float, float, false>(a, up, down, fu_taps, fd_taps, dx, geom, (int)grid, s);
  else {
    set_error("%s: unsupported dtype pair %d -> %d", name, dtype_in, dtype_out);
    return IC2_E_INVALID;
  }
  if (rc != IC2_OK) {
    set_error("%s: no fused instance for up=%d down=%d taps=%d/%d", name, up, down, fu_taps, fd_taps);
    return rc;
  }
  IC2_CHECK_LAUNCH(name);
  return IC2_OK;
}

}  // namespace ic2

using namespace ic2;

extern "C" int ic2_filtered_lrelu(const void* x, void* y, int dtype, int64_t n, int64_t c, int in_h, int in_w,
                                  int out_h, int out_w, const float* fu, int fu_taps, const float* fd, int fd_taps,
                                  const float* b, int up, int down, int px0, int px1, int py0, int py1, float gain,
                                  float slope, float clamp, int flip, void* stream) {
  IC2_CHECK_ARG(n < (1 << 30) && c < (1 << 30), "filtered_lrelu: sizes too large");
  return flrelu_common(x, y, dtype, dtype, false, (int)n, (int)c, (int)c, in_h, in_w, out_h, out_w, fu, fu_taps, fd,
                       fd_taps, b, up, down, px0, px1, py0, py1, gain, slope, clamp, flip, nullptr, stream,
                       "filtered_lrelu");
}

extern "C" int ic2_flrelu_nhwc(const void* x, void* y, int dtype_in, int dtype_out, int n, int c_p, int in_h,
                               int in_w, int out_h, int out_w, const float* fu, int fu_taps, const float* fd,
                               int fd_taps, const float* b, int up, int down, int px0, int px1, int py0, int py1,
                               float gain, float slope, float clamp, int flip, const float* post_scale,
                               void* stream) {
  IC2_CHECK_ARG(c_p % 16 == 0, "flrelu_nhwc: c_p must be a multiple of 16");
  return flrelu_common(x, y, dtype_in, dtype_out, true, n, c_p, c_p, in_h, in_w, out_h, out_w, fu, fu_taps, fd,
                       fd_taps, b, up, down, px0, px1, py0, py1, gain, slope, clamp, flip, post_scale, stream,
                       "flrelu_nhwc");
}

extern "C" int ic2_flrelu_nhwc16(const void* x, void* y, int dtype_in, int dtype_out, int n, int c_p, int in_h,
                                 int in_w, int out_h, int out_w, const float* fu, int fu_taps, const float* fd,
                                 int fd_taps, const float* b, int up, int down, int px0, int px1, int py0, int py1,
                                 float gain, float slope, float clamp, int flip, const float* post_scale,
                                 void* stream) {
  IC2_CHECK_ARG(c_p % 16 == 0, "flrelu_nhwc16: c_p must be a multiple of 16");
  IC2_CHECK_ARG(dtype_in == IC2_F16 || dtype_in == IC2_BF16, "flrelu_nhwc16: f16 or bf16 input");
  return flrelu_common(x, y, dtype_in, dtype_out, true, n, c_p, c_p, in_h, in_w, out_h, out_w, fu, fu_taps, fd,
                       fd_taps, b, up, down, px0, px1, py0, py1, gain, slope, clamp, flip, post_scale, stream,
                       "flrelu_nhwc16", true);
}
