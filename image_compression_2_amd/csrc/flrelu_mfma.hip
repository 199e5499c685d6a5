// Fused filtered leaky-ReLU on the matrix cores: the bf16 NHWC synthesis path of
// SynthesisLayer.forward [SG3-public filtered_lrelu: bias_act -> upfirdn2d(fu, up) -> lrelu*gain, clamp
// -> upfirdn2d(fd, down)], called for every layer of G.synthesis (/root/reference/stylegan3_hvae_full.py:274,329).
//
// Every separable FIR pass is a small banded matrix applied along one axis, and the FIR never mixes
// channels, so each pass is an MFMA with 16 channels on one side and 16 positions along the filtered
// axis on the other:
//   vertical up     V^T[c][ky] = X^T[c][jy] . Gu^T[jy][ky]      (A from LDS by transposed read)
//   horizontal up   U[kx][c]   = Gu[kx][jx] . V[jx][c]          (B from LDS by transposed read)
//   activation      lrelu(U) * gain, clamp  (f32, on the accumulator)
//   horizontal down D^T[c][ox] = act(U)^T[c][kx] . GdT[kx][ox]  (the accumulator IS the A operand)
//   vertical down   O^T[c][oy] = D^T[c][ky] . GdT[ky][oy]       (A from LDS by transposed read)
// The filter matrices are built once per workgroup into registers (bf16 taps); 16x16x16 MFMAs for the
// up passes (a 16-output band spans <= 14 inputs), 16x16x32 where K can be filled (horizontal down).
// A tile = one sample x one 16x16 output tile x 16 channels; 4 waves split columns / rows / output
// columns of each 16-row grid block; the up-sampled grid exists only 16 rows at a time in LDS.  Persistent
// workgroups loop over tiles and prefetch the next tile's input (LDS-DMA) while finishing the current one.
#include "flrelu_mfma.h"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

namespace ic2 {

template <int U>
struct FmGeom {
  static constexpr int TU = 6 * U, TD = 12;
  static constexpr int TO = 16;                        // output tile side
  static constexpr int RA = (TO - 1) * 2 + TD;         // 42 lrelu-grid rows / columns per tile
  static constexpr int NIN = (RA + TU - 2) / U + 1;    // 27 (up 2) / 17 (up 4) input rows / columns
  static constexpr int NB = (RA + 15) / 16;            // 3 grid blocks of 16
  // LDS images (dwords); pitches chosen for conflict-free transposed reads / b64 writes
  static constexpr int IN_PITCH = NIN * 8;             // [jy][x][16 ch]: NIN odd -> 8 rows hit 8 bank groups
  // allocated in whole 1-KB LDS-DMA instructions: the last one's tail lanes (zeros) must not spill into V
  static constexpr int IN_DW = (NIN * NIN * 2 + 63) / 64 * 256;
  static constexpr int V_PITCH = NIN * 8 + 2;          // [ky][x][16 ch]: 16 rows of b64 writes hit 16 bank pairs
  static constexpr int V_DW = 16 * V_PITCH;
  static constexpr int D_XP = 10;                      // [ky][ox][16 ch], ox pitch 10 dwords
  static constexpr int D_PITCH = 16 * D_XP + 8;        // 168 = 40 mod 64: 8 rows hit 8 bank groups
  static constexpr int D_DW = 16 * D_PITCH;
  static constexpr int LDS_DW = IN_DW + V_DW + D_DW + FM_TAPS;
  // V and D sharing one region (two more barriers per grid block): 38.6 KB for up 2, i.e. 4 workgroups per CU
  static constexpr int VD_DW = V_DW > D_DW ? V_DW : D_DW;
  static constexpr int LDS_DW_ALIAS = IN_DW + VD_DW + FM_TAPS;
  static_assert(NIN % 2 == 1 && NIN >= 16, "input image width must be odd and cover a 16-wide window");
};

// first input sample feeding grid position i (polyphase), then clipped so a 16-wide window stays
// inside the NIN-sample image (taps outside the band are zero, so a window shifted back is exact)
template <int U, int DELTA, int NIN>
__device__ constexpr int fm_win(int i) {
  const int j = i < DELTA ? 0 : (i - DELTA + U - 1) / U;
  return j < NIN - 16 ? j : NIN - 16;
}

#ifdef IC2_FM_NOPS
#define FM_SETTLE(v) asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" : "+a"(v))
#else
#define FM_SETTLE(v) (void)0
#endif

// bf16 pair -> f16 pair, saturated to the f16 range (a pre-activation beyond +-65504 ends up clamped
// by the activation anyway)
__device__ __forceinline__ uint32_t fm_bf2_to_h2(uint32_t v) {
  const float lo = __builtin_amdgcn_fmed3f(__uint_as_float(v << 16), -65504.f, 65504.f);
  const float hi = __builtin_amdgcn_fmed3f(__uint_as_float(v & 0xffff0000u), -65504.f, 65504.f);
  return fm_h2u(lo, hi);
}

// the output quad (bf16, or f16 saturated in the synthesis's f16 mode)
__device__ __forceinline__ uint2 fm_out4(bool f16, float a, float b, float c, float d) {
  if (f16) {
    const float lo = -65504.f, hi = 65504.f;
    return fm_pack4(__builtin_amdgcn_fmed3f(a, lo, hi), __builtin_amdgcn_fmed3f(b, lo, hi),
                    __builtin_amdgcn_fmed3f(c, lo, hi), __builtin_amdgcn_fmed3f(d, lo, hi));
  }
  return make_uint2((uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16), (uint32_t)f2bf(c) | ((uint32_t)f2bf(d) << 16));
}

// lrelu + clamp on a pair in 5 instructions (gain folded into the horizontal down taps):
// for 0 <= slope <= 1, med3(v, slope*v, lim) is lrelu(v) clamped from above wherever |slope*v| <= lim, and
// the outer med3 finishes the clamp for the rest (no fmaxf: it would cost a canonicalizing max per value)
__device__ __forceinline__ fm_f2 fm_act2(fm_f2 v, float slope, float lim) {
  const fm_f2 sv = v * slope;
  fm_f2 r;
  r.x = __builtin_amdgcn_fmed3f(__builtin_amdgcn_fmed3f(v.x, sv.x, lim), -lim, lim);
  r.y = __builtin_amdgcn_fmed3f(__builtin_amdgcn_fmed3f(v.y, sv.y, lim), -lim, lim);
  return r;
}

// the same on an f16 pair, after the conversion the next MFMA needs anyway: 3 packed instructions per pair
// (slope*v, maximum3(v, slope*v, -lim) = lrelu clamped from below, min(., lim)).  f16 rounding happens
// before the activation instead of after it: for v >= 0 identical, for v < 0 slope*f16(v) vs f16(slope*v)
// differ by <= 1 ulp of f16 (the operand is f16 either way).
// Two pairs per asm block, interleaved (one block keeps the compiler from padding dependent inline-asm
// instructions with s_nop; plain VALU RAW dependences interlock in hardware).
__device__ __forceinline__ uint2 fm_act_h4(uint32_t h0, uint32_t h1, uint32_t slope2, uint32_t nlim2, uint32_t lim2) {
  uint32_t t0, t1;
  asm("v_pk_mul_f16 %2, %0, %4\n\t"
      "v_pk_mul_f16 %3, %1, %4\n\t"
      "v_pk_maximum3_f16 %0, %0, %2, %5\n\t"
      "v_pk_maximum3_f16 %1, %1, %3, %5\n\t"
      "v_pk_min_f16 %0, %0, %6\n\t"
      "v_pk_min_f16 %1, %1, %6"
      : "+v"(h0), "+v"(h1), "=&v"(t0), "=&v"(t1)
      : "v"(slope2), "v"(nlim2), "v"(lim2));
  return make_uint2(h0, h1);
}

// clamp-split activation for a finite clamp (CL kernels): the up pass produces u' = u / lim, and
//   lrelu(u) clamped to [-lim, lim] = lim * (clamp01(u') - clamp01(-slope * u'))
// (u >= 0: min(u, lim); u < 0: max(slope * u, -lim)), so after the f16 conversion each pair costs two packed
// instructions with the hardware [0, 1] clamp; the factor lim and the subtraction go into the down-pass
// matrices, whose K doubles (positive and negative parts), on the otherwise idle matrix pipe.
__device__ __forceinline__ void fm_act_split(uint32_t h0, uint32_t h1, uint32_t nslope2, uint2& pos, uint2& neg) {
  uint32_t p0, p1, n0, n1;
  asm("v_pk_max_f16 %0, %4, 0 clamp\n\t"
      "v_pk_max_f16 %1, %5, 0 clamp\n\t"
      "v_pk_mul_f16 %2, %4, %6 clamp\n\t"
      "v_pk_mul_f16 %3, %5, %6 clamp"
      : "=&v"(p0), "=&v"(p1), "=&v"(n0), "=&v"(n1)
      : "v"(h0), "v"(h1), "v"(nslope2));
  pos = make_uint2(p0, p1);
  neg = make_uint2(n0, n1);
}


#ifdef IC2_FM_DEBUG
// diagnostic build only: workgroup 0 dumps its LDS images (input, V and D of grid block 0)
__device__ uint32_t g_fm_dbg[3][8192];
extern "C" int ic2_fm_debug_fetch(uint32_t* host, int which) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_fm_dbg), 8192 * 4, (size_t)which * 8192 * 4, hipMemcpyDeviceToHost);
}
#define FM_DUMP(which, ptr, ndw) \
  if (blockIdx.x == 0) for (int i_ = tid; i_ < (ndw); i_ += (int)blockDim.x) g_fm_dbg[which][i_] = (ptr)[i_];
#else
#define FM_DUMP(which, ptr, ndw) (void)0
#endif

template <int U, int DELTA, bool IN_F16, bool ALIAS, int NW>
__global__ void __launch_bounds__(64 * NW) flrelu_mfma_kernel(FlrArgs a, int ntiles) {
  static_assert(NW == 4 || NW == 8, "4 or 8 waves");
  constexpr int NT = 64 * NW, RR = 16 / NW;  // threads; grid rows (and output columns) per wave per block
  using G = FmGeom<U>;
  constexpr int NIN = G::NIN, NCH = NIN * NIN * 2;  // input pixels x 16-B halves
  __shared__ __attribute__((aligned(16))) uint32_t lds[ALIAS ? G::LDS_DW_ALIAS : G::LDS_DW];
  uint32_t* const in_img = lds;
  uint32_t* const v_img = lds + G::IN_DW;
  uint32_t* const d_img = ALIAS ? v_img : v_img + G::V_DW;
  // FM_TAPS floats, layout below
  float* const taps = reinterpret_cast<float*>(v_img + (ALIAS ? G::VD_DW : G::V_DW + G::D_DW));

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, li = lane & 15;
  const int tq = li >> 2, tp = li & 3;  // this lane's (row, 4-column group) in a transposed read

  // tap tables with zero guard bands, so every per-lane filter-matrix entry below is a branch-free read
  // (tap ranges: up [-43, 63], down [-30, 47]): gu at [48, 72) of [0, 116), gd at [148, 160) of [116, 196),
  // gdg (gain folded) at [228, 240) of [196, 276)
  for (int i = tid; i < FM_TAPS; i += NT) {
    float v = 0.f;
    if (i >= 48 && i < 72) v = a.gu[i - 48];
    else if (i >= 148 && i < 160) v = a.gd[i - 148];
    else if (i >= 228 && i < 240) v = a.gdg[i - 228];
    taps[i] = v;
  }

  // persistent: this workgroup runs tiles slot, slot + gridDim.x, ...  Logical tiles run channel block
  // fastest and consecutive slots share an XCD, so the channel blocks of one tile (16 channels = 32 B of
  // each 128-B line of the input) are fetched once into that XCD's L2.
  const int slot = fm_xcd_remap(blockIdx.x, gridDim.x);
  const uint16_t* xin = reinterpret_cast<const uint16_t*>(a.x);
  auto tile_geom = [&](int t, int& n, int& oy0, int& ox0, int& c0) {
    const int cb = t % a.cblocks;
    t /= a.cblocks;
    const int tx = t % a.tiles_x;
    t /= a.tiles_x;
    const int ty = t % a.tiles_y;
    n = t / a.tiles_y;
    oy0 = ty * 16;
    ox0 = tx * 16;
    c0 = cb * 16;
  };
  // input tile -> in_img[jy][x][16 ch] (zeros outside the image).  The image is dense (pixel p at 32 B * p),
  // i.e. lane-linear in (pixel, 16-B half): f16 input goes to LDS by LDS-DMA, asynchronously.  Which (row,
  // column, half) a lane moves in its i-th DMA instruction does not depend on the tile: precomputed once
  // (jy | x << 16, -1 past the image), so a tile's DMA costs a few 32-bit ops per instruction: a raw buffer
  // load whose descriptor base is the tile's sample + channel block and whose per-lane offset is the pixel's,
  // or FM_OOB (answered with zeros) outside the input image.
  constexpr int NDMA = (NCH + 63) / 64;            // 1-KiB DMA instructions per tile
  constexpr int NDW = (NDMA + NW - 1) / NW;        // per wave, at most
  int dma_yx[NDW];
#pragma unroll
  for (int i = 0; i < NDW; ++i) {
    const int k = wave + NW * i;
    const int e = k * 64 + lane;
    const int pix = e >> 1;
    const int jy = pix / NIN, x = pix - (pix / NIN) * NIN;
    dma_yx[i] = (k < NDMA && e < NCH) ? (jy | (x << 16)) : -1;
  }
  const int half8 = (lane & 1) * 8;
  const int xsy = (int)a.xsy, xsx = (int)a.xsx;  // < 2^31: checked by the launcher (per-sample image < 2 GiB)
  auto chunk_src = [&](int e, int n, int sy0, int sx0, int c0) -> const void* {
    const int pix = e >> 1, half = e & 1;
    const int jy = pix / NIN, x = pix - jy * NIN;
    const int iy = sy0 + jy, ix = sx0 + x;
    const bool ok = e < NCH && (unsigned)iy < (unsigned)a.in_h && (unsigned)ix < (unsigned)a.in_w;
    const uint16_t* src = xin + n * a.xsn + (c0 >> 4) * a.xcb + iy * a.xsy + ix * a.xsx + half * 8;
    return ok ? (const void*)src : zero_line();
  };
  auto load_tile = [&](int t) {
    int n, oy0, ox0, c0;
    tile_geom(t, n, oy0, ox0, c0);
    const int sy0 = (oy0 * 2 - a.py0 + DELTA) / U, sx0 = (ox0 * 2 - a.px0 + DELTA) / U;
    if constexpr (IN_F16) {
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(xin + n * a.xsn + (c0 >> 4) * a.xcb), 0, FM_OOB, 0x00020000);
#pragma unroll
      for (int i = 0; i < NDW; ++i) {
        const int k = wave + NW * i;
        if (k < NDMA) {
          const int yx = dma_yx[i];
          const int iy = sy0 + (yx & 0xffff), ix = sx0 + (yx >> 16);
          const bool ok = yx >= 0 && (unsigned)iy < (unsigned)a.in_h && (unsigned)ix < (unsigned)a.in_w;
          const uint32_t off = ok ? (uint32_t)((iy * xsy + ix * xsx + half8) * 2) : FM_OOB;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(in_img + k * 256), 16,
                                                   off, 0, 0, 0);
        }
      }
    } else {
      constexpr int PER = (NCH + NT - 1) / NT;
      uint4 v[PER];
#pragma unroll
      for (int r = 0; r < PER; ++r)  // every load in flight before the first conversion
        v[r] = *reinterpret_cast<const uint4*>(chunk_src(tid + NT * r, n, sy0, sx0, c0));
#pragma unroll
      for (int r = 0; r < PER; ++r) {
        const int e = tid + NT * r;
        if (e < NCH)
          *reinterpret_cast<uint4*>(in_img + e * 4) =
              make_uint4(fm_bf2_to_h2(v[r].x), fm_bf2_to_h2(v[r].y), fm_bf2_to_h2(v[r].z), fm_bf2_to_h2(v[r].w));
      }
    }
  };
  if (IN_F16 && slot < ntiles) load_tile(slot);
  __syncthreads();  // taps

  // ---- filter matrices (f16: 11-bit taps; bf16 taps cost 5e-3 mean relative error on the critically
  // sampled layers) in registers, once per workgroup
  // gmat[t]: Gu[16t + li][win(16t) + 4g + j]  (B of the vertical pass, A of the horizontal pass)
  fm_h4 gmat[G::NB];
#pragma unroll
  for (int t = 0; t < G::NB; ++t) {
    const int w0 = fm_win<U, DELTA, NIN>(16 * t);
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int tap = U * (w0 + 4 * g + j) + DELTA - (16 * t + li);
      v[j] = taps[48 + tap];
    }
    gmat[t] = fm_h4_of(fm_pack4(v[0], v[1], v[2], v[3]));
  }
  // horizontal down (gain folded): GdT[kx][ox = li]; x32 operands over kx blocks (0,1) and (2, zero)
  fm_h8 gdh01, gdh2;
  {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int kx = (j < 4 ? 4 * g + j : 16 + 4 * g + (j - 4));
      v[j] = taps[228 + kx - 2 * li];
    }
    gdh01 = fm_h8_of(fm_pack4(v[0], v[1], v[2], v[3]), fm_pack4(v[4], v[5], v[6], v[7]));
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = taps[228 + 32 + 4 * g + j - 2 * li];
    gdh2 = fm_h8_of(fm_pack4(v[0], v[1], v[2], v[3]), make_uint2(0u, 0u));
  }
  // vertical down: GdT[ky = 16b + 4g + j][oy = li]
  fm_h4 gdv[G::NB];
#pragma unroll
  for (int b = 0; b < G::NB; ++b) {
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = taps[148 + 16 * b + 4 * g + j - 2 * li];
    gdv[b] = fm_h4_of(fm_pack4(v[0], v[1], v[2], v[3]));
  }
  const float slope = a.slope, lim = a.lim;
  const uint32_t slope2 = fm_h2u(slope, slope), lim2 = fm_h2u(lim, lim), nlim2 = fm_h2u(-lim, -lim);
  bf16_t* yout = reinterpret_cast<bf16_t*>(a.y);

  for (int t = slot; t < ntiles; t += gridDim.x) {
    int n, oy0, ox0, c0;
    tile_geom(t, n, oy0, ox0, c0);
    if constexpr (!IN_F16) load_tile(t);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's LDS-DMA (and last tile's stores)
    __syncthreads();                                   // everyone's; and the previous tile fully consumed
    FM_DUMP(0, in_img, G::IN_DW);

    fm_f4 acc[RR];
#pragma unroll
    for (int i = 0; i < RR; ++i) acc[i] = fm_f4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
    for (int b = 0; b < G::NB; ++b) {
      // ---- vertical up: V^T[c][ky] for the 16 grid rows of block b, every input column.  Fixed trip
      // count; the tail columns past NIN repeat column NIN-1 (identical bytes to the same place).  Issued
      // as groups (every column's LDS read, then every MFMA, then every store) with scheduling barriers
      // between them, so the columns' LDS and MFMA latencies overlap instead of forming one serial chain
      {
        constexpr int NC = (NIN + NW - 1) / NW;
        const int w0 = fm_win<U, DELTA, NIN>(16 * b);
        fm_s4 xa[NC];
        fm_f4 vt[NC];
#pragma unroll
        for (int i = 0; i < NC; ++i) {
          const int x = min(wave + NW * i, NIN - 1);
          xa[i] = fm_tr_read(in_img + (w0 + 4 * g + tq) * G::IN_PITCH + x * 8 + 2 * tp);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < NC; ++i)
          vt[i] = __builtin_amdgcn_mfma_f32_16x16x16f16(__builtin_bit_cast(fm_h4, xa[i]), gmat[b],
                                                        fm_f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        // V overwrites D: every wave's vertical-down reads of the previous block are done (block 0: the
        // tile-top barrier already separates them)
        if constexpr (ALIAS) {
          if (b > 0) __syncthreads();
        }
#pragma unroll
        for (int i = 0; i < NC; ++i) {
          const int x = min(wave + NW * i, NIN - 1);
          FM_SETTLE(vt[i]);
          *reinterpret_cast<uint2*>(v_img + li * G::V_PITCH + x * 8 + 2 * g) =
              fm_pack4(vt[i][0], vt[i][1], vt[i][2], vt[i][3]);
        }
      }
      __syncthreads();
      if (b == 0) FM_DUMP(1, v_img, G::V_DW);
      // the input image is dead after the last vertical pass: prefetch the next tile behind the rest
      if (IN_F16 && b == G::NB - 1 && t + (int)gridDim.x < ntiles) load_tile(t + gridDim.x);
      // ---- horizontal: up, activation, down, for this wave's 4 grid rows of the block (the rows past RA in
      // the last block too: finite, and weighted by zero in the vertical down; no branch, so the rows'
      // MFMA chains interleave)
      // grouped like the vertical pass: all 12 LDS reads, all 12 up MFMAs, the activations, the 8 down
      // MFMAs, the stores
      fm_s4 vb[RR][G::NB];
#pragma unroll
      for (int rr = 0; rr < RR; ++rr)
#pragma unroll
        for (int tt = 0; tt < G::NB; ++tt) {
          const int w0 = fm_win<U, DELTA, NIN>(16 * tt);
          vb[rr][tt] = fm_tr_read(v_img + (wave + NW * rr) * G::V_PITCH + (w0 + 4 * g + tq) * 8 + 2 * tp);
        }
      __builtin_amdgcn_sched_barrier(0);
      fm_f4 u[RR][G::NB];
#pragma unroll
      for (int rr = 0; rr < RR; ++rr)
#pragma unroll
        for (int tt = 0; tt < G::NB; ++tt)
          u[rr][tt] = __builtin_amdgcn_mfma_f32_16x16x16f16(gmat[tt], __builtin_bit_cast(fm_h4, vb[rr][tt]),
                                                            fm_f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      fm_h4 au[RR][G::NB];
#pragma unroll
      for (int rr = 0; rr < RR; ++rr)
#pragma unroll
        for (int tt = 0; tt < G::NB; ++tt) {
          FM_SETTLE(u[rr][tt]);
#ifdef IC2_FM_F32_ACT
          const fm_f2 p0 = fm_act2(fm_f2{u[rr][tt][0], u[rr][tt][1]}, slope, lim);
          const fm_f2 p1 = fm_act2(fm_f2{u[rr][tt][2], u[rr][tt][3]}, slope, lim);
          au[rr][tt] = fm_h4_of(fm_pack4(p0.x, p0.y, p1.x, p1.y));
#else
          au[rr][tt] = fm_h4_of(fm_act_h4(fm_h2u(u[rr][tt][0], u[rr][tt][1]), fm_h2u(u[rr][tt][2], u[rr][tt][3]),
                                          slope2, nlim2, lim2));
#endif
        }
      __builtin_amdgcn_sched_barrier(0);
      fm_f4 d[RR];
#pragma unroll
      for (int rr = 0; rr < RR; ++rr) {
        const uint2 a0 = __builtin_bit_cast(uint2, au[rr][0]), a1 = __builtin_bit_cast(uint2, au[rr][1]);
        d[rr] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fm_h8_of(a0, a1), gdh01, fm_f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      }
      // block 2 as a second 16x16x32 with a zero upper half: a 16x16x16 accumulating onto the 16x16x32's
      // result one instruction later reads stale rows 0-1 of the accumulator (mixed-shape srcC hazard)
#pragma unroll
      for (int rr = 0; rr < RR; ++rr) {
        const uint2 a2 = __builtin_bit_cast(uint2, au[rr][2]);
        d[rr] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fm_h8_of(a2, make_uint2(0u, 0u)), gdh2, d[rr], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (ALIAS) __syncthreads();  // D overwrites V: every wave's horizontal reads are done
#pragma unroll
      for (int rr = 0; rr < RR; ++rr) {
        FM_SETTLE(d[rr]);
        *reinterpret_cast<uint2*>(d_img + (wave + NW * rr) * G::D_PITCH + li * G::D_XP + 2 * g) =
            fm_pack4(d[rr][0], d[rr][1], d[rr][2], d[rr][3]);
      }
      __syncthreads();
      if (b == 0) FM_DUMP(2, d_img, G::D_DW);
      // ---- vertical down: accumulate block b's 16 grid rows into this wave's 4 output columns
      fm_s4 da[RR];
#pragma unroll
      for (int i = 0; i < RR; ++i)
        da[i] = fm_tr_read(d_img + (4 * g + tq) * G::D_PITCH + (wave + NW * i) * G::D_XP + 2 * tp);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < RR; ++i)
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x16f16(__builtin_bit_cast(fm_h4, da[i]), gdv[b], acc[i], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }

    // ---- store: lane (g, oy = li) holds channels c0 + 4g .. +3 of output pixel (oy, ox)
    float ps[4] = {1.f, 1.f, 1.f, 1.f};
    if (a.post_scale) {
      const float4 p = *reinterpret_cast<const float4*>(a.post_scale + (int64_t)n * a.c_p + c0 + 4 * g);
      ps[0] = p.x; ps[1] = p.y; ps[2] = p.z; ps[3] = p.w;
    }
    const int gy = oy0 + li;
#pragma unroll
    for (int i = 0; i < RR; ++i) {
      const int gx = ox0 + wave + NW * i;
      if (gy < a.out_h && gx < a.out_w) {
        const uint2 v = fm_out4(a.out_f16, acc[i][0] * ps[0], acc[i][1] * ps[1], acc[i][2] * ps[2], acc[i][3] * ps[3]);
        *reinterpret_cast<uint2*>(yout + (((int64_t)n * a.out_h + gy) * a.out_w + gx) * a.c_p + c0 + 4 * g) = v;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Wide-tile variant (f16 input, the synthesis path): one tile = one sample x 16 output rows x TOX (32)
// output columns x 16 channels, NW (8) waves.  Per output it computes 48 x 80 / (16 x 32) = 7.5 lrelu-grid
// points instead of 48 x 48 / 256 = 9 (the 12-tap down filter needs 2 * 31 + 12 = 74 grid columns for 32
// outputs: 5 blocks of 16), amortises each phase's barrier over twice the outputs, and its 79 KB of LDS (the
// tap table aliases the D image: it is only read before the first tile) keeps 2 workgroups = 16 waves per CU.
// Same passes and per-pass matrices as flrelu_mfma_kernel; the horizontal down pass of output block ob reads
// grid blocks 2 ob .. 2 ob + 2 with the block-0 matrices (the band is translation invariant).
template <int U, int TOX>
struct FmGeom2 {
  static constexpr int TU = 6 * U, TD = 12;
  static constexpr int RAY = 15 * 2 + TD, RAX = (TOX - 1) * 2 + TD;  // 42 x 74 grid rows x columns
  static constexpr int NINY = (RAY + TU - 2) / U + 1, NINX = (RAX + TU - 2) / U + 1;  // up 2: 27 x 43
  static constexpr int NBY = (RAY + 15) / 16, NBX = (RAX + 15) / 16;                   // 3 x 5 grid blocks
  static constexpr int NOB = TOX / 16;                                                  // output column blocks
  static constexpr int IN_PITCH = NINX * 8;  // [jy][x][16 ch] (dwords); NINX odd
  static constexpr int NCH = NINY * NINX * 2;
  static constexpr int IN_DW = (NCH + 63) / 64 * 256;
  static constexpr int V_PITCH = NINX * 8 + 2;
  static constexpr int V_DW = 16 * V_PITCH;
  static constexpr int D_XP = 10;
  static constexpr int D_PITCH = TOX * D_XP + 8;
  static constexpr int D_DW = 16 * D_PITCH;
  static constexpr int DT_DW = D_DW > FM_TAPS_CL ? D_DW : FM_TAPS_CL;  // D image, aliased by the tap table
  static constexpr int LDS_DW = IN_DW + V_DW + DT_DW + 16;       // + the tile's 16 post-scale floats
  static_assert(NINX % 2 == 1 && NINY % 2 == 1 && NINY >= 16, "input image sides must be odd and cover a window");
  static_assert(NBX == 2 * NOB + 1, "horizontal down: output block ob reads grid blocks 2ob .. 2ob+2");
};

template <int U, int DELTA, int TOX, int NW, bool CL, int ABL>
__global__ void __launch_bounds__(64 * NW, 32 / NW) flrelu_mfma2_kernel(FlrArgs a, int ntiles) {  // 2 WGs / CU
  constexpr int NT = 64 * NW, RR = 16 / NW, OCW = TOX / NW;  // grid rows per wave per block; output columns per wave
  using G = FmGeom2<U, TOX>;
  constexpr int NINY = G::NINY, NINX = G::NINX, NBX = G::NBX, NOB = G::NOB, NCH = G::NCH;
  __shared__ __attribute__((aligned(16))) uint32_t lds[G::LDS_DW];
  uint32_t* const in_img = lds;
  uint32_t* const v_img = lds + G::IN_DW;
  uint32_t* const d_img = v_img + G::V_DW;
  float* const taps = reinterpret_cast<float*>(d_img);  // read only before the first tile
  uint32_t* const ps_lds = d_img + G::DT_DW;             // the tile's post-scale row (DMA'd with its input)

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, li = lane & 15;
  const int tq = li >> 2, tp = li & 3;

  for (int i = tid; i < FM_TAPS_CL; i += NT) {
    float v = 0.f;
    if (i >= 48 && i < 72) v = a.gu[i - 48];
    else if (i >= 148 && i < 160) v = a.gd[i - 148];
    else if (i >= 228 && i < 240) v = a.gdg[i - 228];
    else if (i >= 328 && i < 352) v = a.guh[i - 328];
    else if (i >= 428 && i < 440) v = a.gdgl[i - 428];
    taps[i] = v;
  }

  // persistent tile walk.  order 0 / 1: slot, slot + G, ... over the XCD-remapped grid (consecutive slots on one
  // XCD).  order 2: XCD x walks its own contiguous eighth of the tiles in raster order (one or a few samples),
  // so vertically adjacent tiles, whose input halos overlap, share that XCD's L2
  int slot = fm_xcd_remap(blockIdx.x, gridDim.x), tstep = gridDim.x, tend = ntiles;
  if (a.order == 2) {
    const int xcd = blockIdx.x & 7, nx = ((int)gridDim.x - xcd + 7) >> 3, chunk = (ntiles + 7) >> 3;
    slot = xcd * chunk + (blockIdx.x >> 3);
    tstep = nx;
    tend = min(ntiles, (xcd + 1) * chunk);
  }
  const uint16_t* xin = reinterpret_cast<const uint16_t*>(a.x);
  auto tile_geom = [&](int t, int& n, int& oy0, int& ox0, int& c0) {
    int cb, tx, ty;
    if (a.order != 1) {
      cb = t % a.cblocks;
      t /= a.cblocks;
      tx = t % a.tiles_x;
      t /= a.tiles_x;
      ty = t % a.tiles_y;
      n = t / a.tiles_y;
    } else {
      tx = t % a.tiles_x;
      t /= a.tiles_x;
      ty = t % a.tiles_y;
      t /= a.tiles_y;
      cb = t % a.cblocks;
      n = t / a.cblocks;
    }
    oy0 = ty * 16;
    ox0 = tx * TOX;
    c0 = cb * 16;
  };
  // per-lane DMA pattern (tile independent): jy | x << 16, -1 past the image
  constexpr int NDMA = (NCH + 63) / 64;
  constexpr int NDW = (NDMA + NW - 1) / NW;
  int dma_yx[NDW];
#pragma unroll
  for (int i = 0; i < NDW; ++i) {
    const int k = wave + NW * i;
    const int e = k * 64 + lane;
    const int pix = e >> 1;
    const int jy = pix / NINX, x = pix - (pix / NINX) * NINX;
    dma_yx[i] = (k < NDMA && e < NCH) ? (jy | (x << 16)) : -1;
  }
  const int half8 = (lane & 1) * 8;
  const int xsy = (int)a.xsy, xsx = (int)a.xsx;  // < 2^31: checked by the launcher (per-sample image < 2 GiB)
  auto load_tile = [&](int t) {
    int n, oy0, ox0, c0;
    tile_geom(t, n, oy0, ox0, c0);
    const int sy0 = (oy0 * 2 - a.py0 + DELTA) / U, sx0 = (ox0 * 2 - a.px0 + DELTA) / U;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(xin + n * a.xsn + (c0 >> 4) * a.xcb), 0, FM_OOB, 0x00020000);
#pragma unroll
    for (int i = 0; i < NDW; ++i) {
      const int k = wave + NW * i;
      if (k < NDMA) {
        const int yx = dma_yx[i];
        const int iy = sy0 + (yx & 0xffff), ix = sx0 + (yx >> 16);
        const bool ok = yx >= 0 && (unsigned)iy < (unsigned)a.in_h && (unsigned)ix < (unsigned)a.in_w;
        const uint32_t off = ok ? (uint32_t)((iy * xsy + ix * xsx + half8) * 2) : FM_OOB;
        fm_dma16(rs, off, in_img + k * 256);
      }
    }
    if (a.post_scale != nullptr && wave == NW - 1 && lane < 4) {  // 64 B: post_scale[n][c0 .. c0 + 16)
      const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(a.post_scale + (int64_t)n * a.c_p + c0), 0, 64, 0x00020000);
      fm_dma16(prs, lane * 16, ps_lds);
    }
  };
  if (slot < tend) load_tile(slot);
  __syncthreads();  // taps

  // filter matrices (f16) in registers; y and x windows differ only through NINY / NINX clipping
  fm_h4 gmy[3], gmx[NBX];
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    const int w0 = fm_win<U, DELTA, NINY>(16 * t);
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = taps[48 + U * (w0 + 4 * g + j) + DELTA - (16 * t + li)];
    gmy[t] = fm_h4_of(fm_pack4(v[0], v[1], v[2], v[3]));
  }
  // CL: the horizontal up pass yields u / lim (host-scaled taps guh), the down taps carry lim (gdgl)
#pragma unroll
  for (int t = 0; t < NBX; ++t) {
    const int w0 = fm_win<U, DELTA, NINX>(16 * t);
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = taps[(CL ? 328 : 48) + U * (w0 + 4 * g + j) + DELTA - (16 * t + li)];
    gmx[t] = fm_h4_of(fm_pack4(v[0], v[1], v[2], v[3]));
  }
  // horizontal down matrices over kx blocks (K = 32 per MFMA).  Plain: [b0; b1], [b2; 0] against (u0, u1),
  // (u2, 0).  CL: taps * lim, [bi; -bi] against the quad (pos_i, neg_i) of grid block i: each block's quad is
  // one register tuple, shared as-is by the two output blocks that read it (no operand copies)
  fm_h8 gdh01, gdh2, gdq[3];
  {
    auto tap = [&](int blk, int j) { return taps[(CL ? 428 : 228) + 16 * blk + 4 * g + j - 2 * li]; };
    float v[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[j] = tap(0, j);
      v[4 + j] = tap(1, j);
    }
    gdh01 = fm_h8_of(fm_pack4(v[0], v[1], v[2], v[3]), fm_pack4(v[4], v[5], v[6], v[7]));
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[j] = tap(2, j);
      v[4 + j] = 0.f;
    }
    gdh2 = fm_h8_of(fm_pack4(v[0], v[1], v[2], v[3]), fm_pack4(v[4], v[5], v[6], v[7]));
#pragma unroll
    for (int bi = 0; bi < 3; ++bi) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[j] = tap(bi, j);
        v[4 + j] = -tap(bi, j);
      }
      gdq[bi] = fm_h8_of(fm_pack4(v[0], v[1], v[2], v[3]), fm_pack4(v[4], v[5], v[6], v[7]));
    }
  }
  fm_h4 gdv[3];
#pragma unroll
  for (int b = 0; b < 3; ++b) {
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = taps[148 + 16 * b + 4 * g + j - 2 * li];
    gdv[b] = fm_h4_of(fm_pack4(v[0], v[1], v[2], v[3]));
  }
  const float slope = a.slope, lim = CL ? 1.f : a.lim;
  const uint32_t slope2 = fm_h2u(slope, slope), lim2 = fm_h2u(lim, lim), nlim2 = fm_h2u(-lim, -lim);
  const uint32_t nslope2 = fm_h2u(-slope, -slope);
  bf16_t* yout = reinterpret_cast<bf16_t*>(a.y);
  __syncthreads();  // every wave's tap reads are done before the first D store overwrites the table

  for (int t = slot; t < tend; t += tstep) {
    int n, oy0, ox0, c0;
    tile_geom(t, n, oy0, ox0, c0);
    // this wave's LDS-DMA of the tile; the previous tile's OCW output stores (issued after that DMA, always
    // exactly OCW: out-of-range ones are dropped by the buffer bounds, not branched around) stay in flight
    if (t == slot) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(OCW) : "memory");
    __syncthreads();  // everyone's DMA; and the previous tile fully consumed
    // the post-scale row came with the DMA; into registers before the next tile's DMA overwrites it
    float4 psv = make_float4(1.f, 1.f, 1.f, 1.f);
    if (a.post_scale) psv = *reinterpret_cast<const float4*>(ps_lds + 4 * g);

    fm_f4 acc[OCW];
#pragma unroll
    for (int i = 0; i < OCW; ++i) acc[i] = fm_f4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
    for (int b = 0; b < 3; ++b) {
      // ---- vertical up: V^T[c][ky] of block b for every input column (tail columns repeat the last one)
      {
        constexpr int NC = (NINX + NW - 1) / NW;
        const int w0 = fm_win<U, DELTA, NINY>(16 * b);
        fm_s4 xa[NC];
        fm_f4 vt[NC];
#pragma unroll
        for (int i = 0; i < NC; ++i) {
          const int x = min(wave + NW * i, NINX - 1);
          xa[i] = fm_tr_read(in_img + (w0 + 4 * g + tq) * G::IN_PITCH + x * 8 + 2 * tp);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < NC; ++i)
          vt[i] = __builtin_amdgcn_mfma_f32_16x16x16f16(__builtin_bit_cast(fm_h4, xa[i]), gmy[b],
                                                        fm_f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < NC; ++i) {
          const int x = min(wave + NW * i, NINX - 1);
          *reinterpret_cast<uint2*>(v_img + li * G::V_PITCH + x * 8 + 2 * g) = fm_pack4(vt[i][0], vt[i][1], vt[i][2], vt[i][3]);
        }
      }
      if constexpr (!(ABL & 1)) __syncthreads();
      if (!(ABL & 4) && b == 2 && t + tstep < tend) load_tile(t + tstep);  // input image dead: prefetch
      // ---- horizontal: up (NBX column blocks), activation, down (NOB output blocks), one grid row of this
      // wave at a time (bounded register pressure: 2 workgroups per CU need <= 128 VGPRs)
      if constexpr (!(ABL & 16))
#pragma unroll
      for (int rr = 0; rr < RR; ++rr) {
        const int row = wave + NW * rr;
        fm_s4 vb[NBX];
#pragma unroll
        for (int tt = 0; tt < NBX; ++tt) {
          const int w0 = fm_win<U, DELTA, NINX>(16 * tt);
          vb[tt] = fm_tr_read(v_img + row * G::V_PITCH + (w0 + 4 * g + tq) * 8 + 2 * tp);
        }
        __builtin_amdgcn_sched_barrier(0);
        fm_f4 u[NBX];
#pragma unroll
        for (int tt = 0; tt < NBX; ++tt)
          u[tt] = __builtin_amdgcn_mfma_f32_16x16x16f16(gmx[tt], __builtin_bit_cast(fm_h4, vb[tt]),
                                                        fm_f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        fm_f4 d[NOB];
        if constexpr (CL) {
          fm_h8 q[NBX];  // (pos, neg) of grid block tt as one tuple
#pragma unroll
          for (int tt = 0; tt < NBX; ++tt) {
            uint2 p, m;
            if constexpr (ABL & 2) { p = make_uint2(fm_h2u(u[tt][0], u[tt][1]), fm_h2u(u[tt][2], u[tt][3])); m = p; }
            else fm_act_split(fm_h2u(u[tt][0], u[tt][1]), fm_h2u(u[tt][2], u[tt][3]), nslope2, p, m);
            q[tt] = fm_h8_of(p, m);
          }
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int bi = 0; bi < 3; ++bi)
#pragma unroll
            for (int ob = 0; ob < NOB; ++ob)
              d[ob] = __builtin_amdgcn_mfma_f32_16x16x32_f16(q[2 * ob + bi], gdq[bi],
                                                             bi == 0 ? fm_f4{0.f, 0.f, 0.f, 0.f} : d[ob], 0, 0, 0);
        } else {
          uint2 au[NBX];
#pragma unroll
          for (int tt = 0; tt < NBX; ++tt)
            au[tt] = fm_act_h4(fm_h2u(u[tt][0], u[tt][1]), fm_h2u(u[tt][2], u[tt][3]), slope2, nlim2, lim2);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int ob = 0; ob < NOB; ++ob)
            d[ob] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fm_h8_of(au[2 * ob], au[2 * ob + 1]), gdh01,
                                                           fm_f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
#pragma unroll
          for (int ob = 0; ob < NOB; ++ob)
            d[ob] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fm_h8_of(au[2 * ob + 2], make_uint2(0u, 0u)), gdh2, d[ob],
                                                           0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int ob = 0; ob < NOB; ++ob)
          *reinterpret_cast<uint2*>(d_img + row * G::D_PITCH + (16 * ob + li) * G::D_XP + 2 * g) =
              fm_pack4(d[ob][0], d[ob][1], d[ob][2], d[ob][3]);
      }
      if constexpr (!(ABL & 1)) __syncthreads();
      // ---- vertical down: accumulate block b's 16 grid rows into this wave's output columns
      if constexpr (!(ABL & 32)) {
        fm_s4 da[OCW];
#pragma unroll
        for (int i = 0; i < OCW; ++i)
          da[i] = fm_tr_read(d_img + (4 * g + tq) * G::D_PITCH + (wave + NW * i) * G::D_XP + 2 * tp);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < OCW; ++i)
          acc[i] = __builtin_amdgcn_mfma_f32_16x16x16f16(__builtin_bit_cast(fm_h4, da[i]), gdv[b], acc[i], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    }

    // ---- store: lane (g, oy = li) holds channels c0 + 4g .. +3 of output pixel (oy, ox); buffer stores with
    // the per-sample image as the resource, out-of-range pixels at the dropped offset FM_OOB
    const float ps[4] = {psv.x, psv.y, psv.z, psv.w};
    const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(yout + (int64_t)n * a.out_h * a.out_w * a.c_p + c0), 0, FM_OOB, 0x00020000);
    const int gy = oy0 + li;
#pragma unroll
    for (int i = 0; i < OCW; ++i) {
      const int gx = ox0 + wave + NW * i;
      uint32_t off = (gy < a.out_h && gx < a.out_w) ? (uint32_t)(((gy * a.out_w + gx) * a.c_p + 4 * g) * 2) : FM_OOB;
      if constexpr ((ABL & 64) != 0)  // diagnostic: channel-blocked output addressing (wrong layout for consumers)
        off = (gy < a.out_h && gx < a.out_w)
                  ? (uint32_t)((((c0 >> 4) * a.out_h + gy) * a.out_w + gx) * 32 + 8 * g) - (uint32_t)(c0 * 2)
                  : FM_OOB;
      const uint2 v = fm_out4(a.out_f16, acc[i][0] * ps[0], acc[i][1] * ps[1], acc[i][2] * ps[2], acc[i][3] * ps[3]);
      if constexpr (!(ABL & 8))
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u32_t, v), ors, off, 0, 0);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Strip-streaming variant (round 3).  A work item is a strip: one sample x 32 output columns x 16 channels x a
// run of consecutive 16-row tiles, walked top to bottom.  Tile t needs lrelu-grid rows 32t .. 32t+41, i.e. grid
// blocks 2t, 2t+1, 2t+2 of 16 rows, and block 2t+2 is block 0 of tile t+1: the strip computes every grid block
// once (2 per tile instead of 3) and carries that shared block's vertical-down contribution to the next tile in
// registers (acc_b).  Its input rows live in an LDS ring of U+1 groups of 16/U rows: block k reads rows
// 16k/U .. 16k/U+15 (strip-relative; with DELTA = py0 mod U this window covers every tap of the block's rows for
// every k, so one vertical-up matrix serves all blocks), and after block k's vertical up the group it no longer
// needs is refilled with the rows block k+2 will need: 16/U new input rows per block (16 / 8 per 16 output rows,
// up 2 / 4) instead of the tile kernel's 27 / 17.  The horizontal passes are flrelu_mfma2_kernel's.
template <int U>
struct FmGeom3 {
  using G2 = FmGeom2<U, 32>;
  static constexpr int NINX = G2::NINX;        // 43 (up 2) / 25 (up 4) input columns
  static constexpr int S = 16 / U;             // input rows per grid block (8 / 4)
  static constexpr int NG = U + 1;             // ring groups of S rows
  static constexpr int IN_PITCH = NINX * 8;    // dwords per input row [x][16 ch]; NINX odd
  static constexpr int GCH = S * NINX * 2;     // 16-B chunks per group
  static constexpr int NGI = (GCH + 63) / 64;  // 1-KiB DMA instructions per group
  static constexpr int GRP_DW = NGI * 256;
  static constexpr int RING_DW = NG * GRP_DW;
  static constexpr int LDS_DW = RING_DW + G2::V_DW + G2::DT_DW + 16;
  static_assert(U * S == 16 && NINX % 2 == 1, "geometry");
  // the surplus columns' reads (x < NW * ceil(NINX / NW)) of the last row of the last group stay in the ring
  static_assert((NG - 1) * GRP_DW + (S - 1) * IN_PITCH + 8 * 8 * ((NINX + 7) / 8) <= RING_DW, "ring bounds");
};

// diagnostic builds only (tools/build_abl.sh, wrong results): IC2_FM3_ABL bit 0 skips the ring waits, bit 1 the ring
// DMAs, bit 2 the horizontal pass, bit 3 the vertical up, bit 4 the vertical down, bit 5 the two in-block barriers,
// bit 6 the output stores (issued to the dropped offset: same instructions, no bytes)
#ifndef IC2_FM3_ABL
#define IC2_FM3_ABL 0
#endif
// ring DMA of block k+2 issued right after block k's vertical-up barrier (1) or after its horizontal pass (0)
#ifndef FM3_EARLY
#define FM3_EARLY 1
#endif
// a finished tile's stores deferred into the next block, behind its ring DMA (1), or at the end of the block (0,
// default: the deferral measured 4 % slower over the C2 layers, profiles/r4s_flr_defer_ab.txt)
#ifndef FM3_DEFER_ST
#define FM3_DEFER_ST 0
#endif
template <int U, int DELTA, int NW, bool CL>
__global__ void __launch_bounds__(64 * NW, 32 / NW) flrelu_mfma3_kernel(FlrArgs a, int nitems, int nseg, int seg_len) {
  constexpr int TOX = 32, NT = 64 * NW, RR = 16 / NW, OCW = TOX / NW;
  using G2 = FmGeom2<U, TOX>;
  using G = FmGeom3<U>;
  constexpr int NINX = G::NINX, NBX = G2::NBX, NOB = G2::NOB, S = G::S, NG = G::NG;
  __shared__ __attribute__((aligned(16))) uint32_t lds[G::LDS_DW];
  uint32_t* const ring = lds;
  uint32_t* const v_img = lds + G::RING_DW;
  uint32_t* const d_img = v_img + G2::V_DW;
  float* const taps = reinterpret_cast<float*>(d_img);  // read only before the first strip
  uint32_t* const ps_lds = d_img + G2::DT_DW;            // the strip's post-scale row (DMA'd with its first rows)

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, li = lane & 15;
  const int tq = li >> 2, tp = li & 3;
  // this lane's row in a vertical-up window, as (ring group offset, row in group)
  const int qoff = (4 * g + tq) / S, roff = (4 * g + tq) % S;

  for (int i = tid; i < FM_TAPS_CL; i += NT) {
    float v = 0.f;
    if (i >= 48 && i < 72) v = a.gu[i - 48];
    else if (i >= 148 && i < 160) v = a.gd[i - 148];
    else if (i >= 228 && i < 240) v = a.gdg[i - 228];
    else if (i >= 328 && i < 352) v = a.guh[i - 328];
    else if (i >= 428 && i < 440) v = a.gdgl[i - 428];
    taps[i] = v;
  }

  // work item w = ((n * tiles_x + tx) * nseg + seg) * cblocks + cb: the channel blocks of one strip run on
  // consecutive slots of one XCD, so they walk down together and their output stores (32 B of each pixel's
  // row each) meet in its L2
  const int slot = fm_xcd_remap(blockIdx.x, gridDim.x);
  const uint16_t* xin = reinterpret_cast<const uint16_t*>(a.x);
  auto item_geom = [&](int w, int& n, int& ox0, int& c0, int& t0, int& nt) {
    const int cb = w % a.cblocks;
    w /= a.cblocks;
    const int seg = w % nseg;
    w /= nseg;
    const int tx = w % a.tiles_x;
    n = w / a.tiles_x;
    ox0 = tx * TOX;
    c0 = cb * 16;
    t0 = seg * seg_len;
    nt = min(seg_len, a.tiles_y - t0);
  };
  const int xsy = (int)a.xsy, xsx = (int)a.xsx;  // < 2^31: checked by the launcher (per-sample image < 2 GiB)
  // group q (strip-relative input rows qS .. qS+S-1 of the item's first tile) -> ring slot q mod NG.  Which
  // (row, column, half) a lane moves is recomputed per DMA from an opaque copy of the lane id: hoisted out of the
  // item loop as loop invariants, these per-lane values pushed the kernel past 128 VGPRs into scratch
  // this wave's DMA instructions per ring group (wave-uniform; at most 2: the wait counts above)
  const int my_dma = wave < G::NGI ? (G::NGI - 1 - wave) / NW + 1 : 0;
  static_assert((G::NGI + NW - 1) / NW <= 2, "ring group DMA per wave");
  auto load_group = [&](int n, int iy0, int sx0, int c0, int q) __attribute__((always_inline)) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(xin + n * a.xsn + (c0 >> 4) * a.xcb), 0, FM_OOB, 0x00020000);
    uint32_t* const dst = ring + (q % NG) * G::GRP_DW;
    int ln = lane;
    asm volatile("" : "+v"(ln));
#pragma unroll
    for (int i = 0; i < (G::NGI + NW - 1) / NW; ++i) {
      const int k = wave + NW * i;
      if (k < G::NGI) {
        const int e = k * 64 + ln;
        const int pix = e >> 1;
        const int row = pix / NINX, x = pix - row * NINX;
        const int iy = iy0 + q * S + row, ix = sx0 + x;
        const bool ok = e < G::GCH && (unsigned)iy < (unsigned)a.in_h && (unsigned)ix < (unsigned)a.in_w;
        const uint32_t off = ok ? (uint32_t)((iy * xsy + ix * xsx + (e & 1) * 8) * 2) : FM_OOB;
        fm_dma16(rs, off, dst + k * 256);
      }
    }
  };
  // an item's first U+1 groups and its post-scale row (every slot of the ring: issued only once the previous
  // item's last vertical up is done)
  auto load_item = [&](int w) __attribute__((always_inline)) {
    int n, ox0, c0, t0, nt;
    item_geom(w, n, ox0, c0, t0, nt);
    const int iy0 = (32 * t0 + DELTA - a.py0) / U, sx0 = (ox0 * 2 - a.px0 + DELTA) / U;
#pragma unroll
    for (int q = 0; q < NG; ++q) load_group(n, iy0, sx0, c0, q);
    if (a.post_scale != nullptr && wave == NW - 1 && lane < 4) {  // 64 B: post_scale[n][c0 .. c0 + 16)
      const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(a.post_scale + (int64_t)n * a.c_p + c0), 0, 64, 0x00020000);
      fm_dma16(prs, lane * 16, ps_lds);
    }
  };
  if (slot < nitems) load_item(slot);
  __syncthreads();  // taps

  // filter matrices.  Vertical up: grid row 16k + li of block k from input row kS + 4g + j, tap U(4g + j) +
  // DELTA - li (the same for every block)
  fm_h4 gmy, gmx[NBX];
  {
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = taps[48 + U * (4 * g + j) + DELTA - li];
    gmy = fm_h4_of(fm_pack4(v[0], v[1], v[2], v[3]));
  }
#pragma unroll
  for (int t = 0; t < NBX; ++t) {
    const int w0 = fm_win<U, DELTA, NINX>(16 * t);
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = taps[(CL ? 328 : 48) + U * (w0 + 4 * g + j) + DELTA - (16 * t + li)];
    gmx[t] = fm_h4_of(fm_pack4(v[0], v[1], v[2], v[3]));
  }
  fm_h8 gdh01, gdh2, gdq[3];
  {
    auto tap = [&](int blk, int j) { return taps[(CL ? 428 : 228) + 16 * blk + 4 * g + j - 2 * li]; };
    float v[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[j] = tap(0, j);
      v[4 + j] = tap(1, j);
    }
    gdh01 = fm_h8_of(fm_pack4(v[0], v[1], v[2], v[3]), fm_pack4(v[4], v[5], v[6], v[7]));
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[j] = tap(2, j);
      v[4 + j] = 0.f;
    }
    gdh2 = fm_h8_of(fm_pack4(v[0], v[1], v[2], v[3]), fm_pack4(v[4], v[5], v[6], v[7]));
#pragma unroll
    for (int bi = 0; bi < 3; ++bi) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[j] = tap(bi, j);
        v[4 + j] = -tap(bi, j);
      }
      gdq[bi] = fm_h8_of(fm_pack4(v[0], v[1], v[2], v[3]), fm_pack4(v[4], v[5], v[6], v[7]));
    }
  }
  fm_h4 gdv[3];
#pragma unroll
  for (int b = 0; b < 3; ++b) {
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = taps[148 + 16 * b + 4 * g + j - 2 * li];
    gdv[b] = fm_h4_of(fm_pack4(v[0], v[1], v[2], v[3]));
  }
  const float slope = a.slope, lim = CL ? 1.f : a.lim;
  const uint32_t slope2 = fm_h2u(slope, slope), lim2 = fm_h2u(lim, lim), nlim2 = fm_h2u(-lim, -lim);
  const uint32_t nslope2 = fm_h2u(-slope, -slope);
  bf16_t* yout = reinterpret_cast<bf16_t*>(a.y);
  __syncthreads();  // every wave's tap reads are done before the first D store overwrites the table

  bool first = true;
  for (int w = slot; w < nitems; w += gridDim.x) {
    int n, ox0, c0, t0, nt;
    item_geom(w, n, ox0, c0, t0, nt);
    const int iy0 = (32 * t0 + DELTA - a.py0) / U, sx0 = (ox0 * 2 - a.px0 + DELTA) / U;
    const bool has_next = w + (int)gridDim.x < nitems;
    // this wave's DMA of the item's first rows; the previous item's last OCW output stores (issued after that
    // DMA, always exactly OCW) stay in flight
    if (first) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(OCW) : "memory");
    first = false;
    __syncthreads();
    float4 psv = make_float4(1.f, 1.f, 1.f, 1.f);
    if (a.post_scale) psv = *reinterpret_cast<const float4*>(ps_lds + 4 * g);
    const float ps[4] = {psv.x, psv.y, psv.z, psv.w};
    const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(yout + (int64_t)n * a.out_h * a.out_w * a.c_p + c0), 0, FM_OOB, 0x00020000);
    const int kend = 2 * nt;  // blocks 0 .. kend

    fm_f4 acc_a[OCW], acc_b[OCW];
    // store tile t0 + tt from acc_a: lane (g, oy = li) holds channels c0 + 4g .. +3 of output pixel (oy, ox); exactly
    // OCW buffer stores per wave (out-of-range pixels at the dropped offset FM_OOB)
    auto store_tile = [&](int tt) __attribute__((always_inline)) {
      const int gy = 16 * (t0 + tt) + li;
#pragma unroll
      for (int i = 0; i < OCW; ++i) {
        const int gx = ox0 + wave + NW * i;
        const uint32_t off =
            (gy < a.out_h && gx < a.out_w) ? (uint32_t)(((gy * a.out_w + gx) * a.c_p + 4 * g) * 2) : FM_OOB;
        const uint2 v = fm_out4(a.out_f16, acc_a[i][0] * ps[0], acc_a[i][1] * ps[1], acc_a[i][2] * ps[2], acc_a[i][3] * ps[3]);
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u32_t, v), ors, (IC2_FM3_ABL & 64) ? FM_OOB : off, 0, 0);
      }
    };
    // grid block k of the item: vertical up (ring -> V), horizontal up / activation / down (V -> D), vertical down
    // (D -> acc).  MODE 0: block 0, starts acc_b; 1: odd block, acc_a = acc_b + its share; 2: even block >= 2,
    // finishes acc_a and starts acc_b for the next tile.  A tile finished at block k < kend is stored in block k+1,
    // right after that block's ring DMA (acc_a is untouched until its vertical down): the stores are then younger
    // than every DMA waited for in the next two blocks, so those waits do not wait for the stores to be written
    // (vmcnt retires in issue order; FM3_DEFER_ST=0 stores at the end of block k)
    auto block = [&](int k, auto mode_c) __attribute__((always_inline)) {
      constexpr int MODE = decltype(mode_c)::value;
      if constexpr (!(IC2_FM3_ABL & 8)) {
        constexpr int NC = (NINX + NW - 1) / NW;
        // column x = wave + NW i: one per-lane base per block and immediate offsets.  Columns past NINX - 1 (the
        // last round's surplus waves) read in-bounds bytes of the ring and are not stored
        const int q = k + qoff;
        const uint32_t* rowp = ring + (q % NG) * G::GRP_DW + roff * G::IN_PITCH + 2 * tp + wave * 8;
        fm_s4 xa[NC];
        fm_f4 vt[NC];
#pragma unroll
        for (int i = 0; i < NC; ++i) xa[i] = fm_tr_read(rowp + i * NW * 8);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < NC; ++i)
          vt[i] = __builtin_amdgcn_mfma_f32_16x16x16f16(__builtin_bit_cast(fm_h4, xa[i]), gmy,
                                                        fm_f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        uint32_t* const vp = v_img + li * G2::V_PITCH + 2 * g + wave * 8;
#pragma unroll
        for (int i = 0; i < NC; ++i)
          if (i < NC - 1 || wave + NW * i < NINX)
            *reinterpret_cast<uint2*>(vp + i * NW * 8) = fm_pack4(vt[i][0], vt[i][1], vt[i][2], vt[i][3]);
      }
      if constexpr (!(IC2_FM3_ABL & 32)) __syncthreads();  // V complete; the ring group k is dead; v-down k-1 done
      // the item's last block: every ring group is dead -> the next item's first rows
      if (k == kend && has_next) load_item(w + gridDim.x);
      // the rows block k+2 needs go out now, into the slot of group k (every wave's vertical up of block k is done):
      // they land behind this block's horizontal pass and vertical down and the next block's vertical up
      const bool dma = !(IC2_FM3_ABL & 2) && k + 2 <= kend;
      if (FM3_EARLY && dma) load_group(n, iy0, sx0, c0, k + U + 1);
      if constexpr (FM3_DEFER_ST && MODE == 1) {
        if (k >= 3) store_tile((k - 3) >> 1);  // the tile block k-1 finished
      }
#pragma unroll
      for (int rr = 0; rr < ((IC2_FM3_ABL & 4) ? 0 : RR); ++rr) {
        const int row = wave + NW * rr;
        fm_s4 vb[NBX];
#pragma unroll
        for (int tt = 0; tt < NBX; ++tt) {
          const int w0 = fm_win<U, DELTA, NINX>(16 * tt);
          vb[tt] = fm_tr_read(v_img + row * G2::V_PITCH + (w0 + 4 * g + tq) * 8 + 2 * tp);
        }
        __builtin_amdgcn_sched_barrier(0);
        fm_f4 u[NBX];
#pragma unroll
        for (int tt = 0; tt < NBX; ++tt)
          u[tt] = __builtin_amdgcn_mfma_f32_16x16x16f16(gmx[tt], __builtin_bit_cast(fm_h4, vb[tt]),
                                                        fm_f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        fm_f4 d[NOB];
        if constexpr (CL) {
          fm_h8 qv[NBX];
#pragma unroll
          for (int tt = 0; tt < NBX; ++tt) {
            uint2 p, m;
            fm_act_split(fm_h2u(u[tt][0], u[tt][1]), fm_h2u(u[tt][2], u[tt][3]), nslope2, p, m);
            qv[tt] = fm_h8_of(p, m);
          }
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int bi = 0; bi < 3; ++bi)
#pragma unroll
            for (int ob = 0; ob < NOB; ++ob)
              d[ob] = __builtin_amdgcn_mfma_f32_16x16x32_f16(qv[2 * ob + bi], gdq[bi],
                                                             bi == 0 ? fm_f4{0.f, 0.f, 0.f, 0.f} : d[ob], 0, 0, 0);
        } else {
          uint2 au[NBX];
#pragma unroll
          for (int tt = 0; tt < NBX; ++tt)
            au[tt] = fm_act_h4(fm_h2u(u[tt][0], u[tt][1]), fm_h2u(u[tt][2], u[tt][3]), slope2, nlim2, lim2);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int ob = 0; ob < NOB; ++ob)
            d[ob] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fm_h8_of(au[2 * ob], au[2 * ob + 1]), gdh01,
                                                           fm_f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
#pragma unroll
          for (int ob = 0; ob < NOB; ++ob)
            d[ob] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fm_h8_of(au[2 * ob + 2], make_uint2(0u, 0u)), gdh2, d[ob],
                                                           0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int ob = 0; ob < NOB; ++ob)
          *reinterpret_cast<uint2*>(d_img + row * G2::D_PITCH + (16 * ob + li) * G2::D_XP + 2 * g) =
              fm_pack4(d[ob][0], d[ob][1], d[ob][2], d[ob][3]);
      }
      // the ring group this block's DMA (issued at block k-1's barrier below) filled must have landed before
      // block k+1's vertical up: wait for it behind the stores of the tile finished at block k-1 (odd k >= 3)
      if (!(IC2_FM3_ABL & 1) && k >= 1 && k < kend) {
        // block k-1's ring DMA must have landed (block k+1 reads it); younger: the stores of a tile (exactly OCW) --
        // deferred: issued in this block (odd k >= 3) or in block k-1 after its DMA (even k >= 4); else issued at the
        // end of block k-1 (odd k >= 3) -- and, issued early, this block's own DMA (this wave's share, uniform)
        const bool st = (MODE == 1 && k >= 3) || (FM3_DEFER_ST && MODE == 2 && k >= 4);
        const int nd = FM3_EARLY && dma ? my_dma : 0;
        if (nd == 0) {
          if (st) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(OCW) : "memory");
          else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else if (nd == 1) {
          if (st) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(OCW + 1) : "memory");
          else asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
        } else {
          if (st) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(OCW + 2) : "memory");
          else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        }
      }
      if constexpr (!(IC2_FM3_ABL & 32)) __syncthreads();  // D complete; every wave's horizontal reads of V are done
      if (!FM3_EARLY && dma) load_group(n, iy0, sx0, c0, k + U + 1);  // rows of block k+2
      if constexpr (!(IC2_FM3_ABL & 16)) {
        fm_s4 da[OCW];
#pragma unroll
        for (int i = 0; i < OCW; ++i)
          da[i] = fm_tr_read(d_img + (4 * g + tq) * G2::D_PITCH + (wave + NW * i) * G2::D_XP + 2 * tp);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (MODE == 0) {
#pragma unroll
          for (int i = 0; i < OCW; ++i)
            acc_b[i] = __builtin_amdgcn_mfma_f32_16x16x16f16(__builtin_bit_cast(fm_h4, da[i]), gdv[0],
                                                             fm_f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        } else if constexpr (MODE == 1) {
#pragma unroll
          for (int i = 0; i < OCW; ++i)
            acc_a[i] = __builtin_amdgcn_mfma_f32_16x16x16f16(__builtin_bit_cast(fm_h4, da[i]), gdv[1], acc_b[i], 0, 0, 0);
        } else {
#pragma unroll
          for (int i = 0; i < OCW; ++i)
            acc_a[i] = __builtin_amdgcn_mfma_f32_16x16x16f16(__builtin_bit_cast(fm_h4, da[i]), gdv[2], acc_a[i], 0, 0, 0);
          if (k < kend) {
#pragma unroll
            for (int i = 0; i < OCW; ++i)
              acc_b[i] = __builtin_amdgcn_mfma_f32_16x16x16f16(__builtin_bit_cast(fm_h4, da[i]), gdv[0],
                                                               fm_f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    };

    block(0, std::integral_constant<int, 0>{});
    for (int t = 0; t < nt; ++t) {
      block(2 * t + 1, std::integral_constant<int, 1>{});
      block(2 * t + 2, std::integral_constant<int, 2>{});
      if (!FM3_DEFER_ST || t == nt - 1) store_tile(t);  // the item's last tile: stored at once (see block)
    }
  }
}

template <int U, int DELTA, bool CL>
static void fm3_launch_cl(FlrArgs a, int n, hipStream_t s) {
  constexpr int TOX = 32, NW = 8;
  a.tiles_x = (int)ceil_div(a.out_w, TOX);
  a.tiles_y = (int)ceil_div(a.out_h, 16);
  a.cblocks = a.c_p / 16;
  static int resident = 0;
  if (resident == 0) {
    int dev = 0, cus = 0, per_cu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, flrelu_mfma3_kernel<U, DELTA, NW, CL>, 64 * NW, 0);
    resident = (cus > 0 ? cus : 256) * (per_cu > 0 ? per_cu : 1);
  }
  // strip segmentation: fm_strip_segments (flrelu_mfma.h); knob IC2_FLR_SEGS=0 keeps the round-3 rule
  static const int segs_mode = knob("IC2_FLR_SEGS", 1);
  const int64_t nstrips = (int64_t)n * a.tiles_x * a.cblocks;
  int nseg = fm_strip_segments(nstrips, a.tiles_y, resident, segs_mode == 1);
  const int seg_len = (int)ceil_div(a.tiles_y, nseg);
  nseg = (int)ceil_div(a.tiles_y, seg_len);
  const int nitems = (int)(nstrips * nseg);
  const int grid = nitems < resident ? nitems : resident;
  hipLaunchKernelGGL((flrelu_mfma3_kernel<U, DELTA, NW, CL>), dim3((unsigned)grid), dim3(64 * NW), 0, s, a, nitems,
                     nseg, seg_len);
}

template <int U, int DELTA, bool CL, int ABL>
static void fm2_launch_cl(FlrArgs a, int n, hipStream_t s) {
  constexpr int TOX = 32, NW = 8;
  a.tiles_x = (int)ceil_div(a.out_w, TOX);
  a.tiles_y = (int)ceil_div(a.out_h, 16);
  a.cblocks = a.c_p / 16;
  // knob IC2_FLR_ORDER=1: spatial tiles fastest, so the tiles one XCD runs together share their input halos in its L2
  static const int order = knob("IC2_FLR_ORDER", 0);
  a.order = order;
  const int ntiles = n * a.tiles_y * a.tiles_x * a.cblocks;
  static int resident = 0;
  if (resident == 0) {
    int dev = 0, cus = 0, per_cu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, flrelu_mfma2_kernel<U, DELTA, TOX, NW, CL, ABL>, 64 * NW, 0);
    resident = (cus > 0 ? cus : 256) * (per_cu > 0 ? per_cu : 1);
  }
  const int grid = ntiles < resident ? ntiles : resident;
  hipLaunchKernelGGL((flrelu_mfma2_kernel<U, DELTA, TOX, NW, CL, ABL>), dim3((unsigned)grid), dim3(64 * NW), 0, s, a, ntiles);
}

// the clamp-split activation needs a finite clamp whose reciprocal scaling keeps the f16 operands normal
// (lim in [2^-4, 2^12]: SG3's conv_clamp 256 / sqrt(2)); knob IC2_FLR_CLSPLIT=0 keeps the 3-instruction activation.
// (The kernel's ABL template parameter held the round-2 ablation builds; only ABL = 0 is instantiated.)
template <int U, int DELTA>
static void fm2_launch(FlrArgs a, int n, hipStream_t s) {
  static const bool split = knob("IC2_FLR_CLSPLIT", 1) != 0;
  // knob IC2_FLR_STRIP=0: the round-2 tile kernel instead of the strip-streaming one
  static const bool strip = knob("IC2_FLR_STRIP", 1) != 0;
  const bool cl = split && a.lim >= 0.0625f && a.lim <= 4096.f;
  if (strip) {
    if (cl) fm3_launch_cl<U, DELTA, true>(a, n, s);
    else fm3_launch_cl<U, DELTA, false>(a, n, s);
  } else if (cl) {
    fm2_launch_cl<U, DELTA, true, 0>(a, n, s);
  } else {
    fm2_launch_cl<U, DELTA, false, 0>(a, n, s);
  }
}

template <int U, int DELTA, bool IN_F16, bool ALIAS, int NW>
static void fm_launch_alias(const FlrArgs& a, int ntiles, hipStream_t s) {
  // persistent grid: every CU filled to the kernel's occupancy, capped by the tile count
  static int resident = 0;
  if (resident == 0) {
    int dev = 0, cus = 0, per_cu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, flrelu_mfma_kernel<U, DELTA, IN_F16, ALIAS, NW>, 64 * NW,
                                                       0);
    resident = (cus > 0 ? cus : 256) * (per_cu > 0 ? per_cu : 1);
  }
  const int grid = ntiles < resident ? ntiles : resident;
  hipLaunchKernelGGL((flrelu_mfma_kernel<U, DELTA, IN_F16, ALIAS, NW>), dim3((unsigned)grid), dim3(64 * NW), 0, s, a,
                     ntiles);
}

// The separate-V/D LDS layout on 4 waves.  Measured and not kept (round 2): the aliased layout (4 workgroups per
// CU instead of 3; 1180 vs 1185 img/s -- the extra barriers cancel the occupancy gain) and the same tile on 8 waves
// (FLR 9.0 vs 8.1 ms per C2 step: the kernel wants independent MFMA chains per wave more than it wants waves).
template <int U, int DELTA, bool IN_F16>
static void fm_launch_one(const FlrArgs& a, int ntiles, hipStream_t s) {
  fm_launch_alias<U, DELTA, IN_F16, false, 4>(a, ntiles, s);
}

template <bool IN_F16>
static void fm_launch(const FlrArgs& a, int up, int delta, int ntiles, hipStream_t s) {
  if (up == 2) {
    if (delta == 0) fm_launch_one<2, 0, IN_F16>(a, ntiles, s);
    else fm_launch_one<2, 1, IN_F16>(a, ntiles, s);
  } else {
    switch (delta) {
      case 0: fm_launch_one<4, 0, IN_F16>(a, ntiles, s); break;
      case 1: fm_launch_one<4, 1, IN_F16>(a, ntiles, s); break;
      case 2: fm_launch_one<4, 2, IN_F16>(a, ntiles, s); break;
      default: fm_launch_one<4, 3, IN_F16>(a, ntiles, s); break;
    }
  }
}

int flrelu_mfma_launch(FlrArgs a, int in_f16, int up, int down, int tu, int td, int delta, int n, hipStream_t s) {
  if (down != 2 || td != 12 || tu != 6 * up || (up != 2 && up != 4) || a.bias != nullptr || a.c_p % 16 != 0)
    return IC2_E_UNSUPPORTED;
  if ((int64_t)a.in_h * a.in_w * a.c_p * 2 >= (int64_t)FM_OOB) return IC2_E_UNSUPPORTED;  // 32-bit buffer offsets
  if (a.xsc != 1 || a.xsx % 8 != 0) return IC2_E_UNSUPPORTED;  // 16-B chunks of 8 channels
  if ((int64_t)a.out_h * a.out_w * a.c_p * 2 >= (int64_t)FM_OOB) return IC2_E_UNSUPPORTED;  // output offsets too
  // the wide (16 x 32) tile for the f16-input synthesis path unless knob IC2_FLR_WIDE=0
  static const bool wide = knob("IC2_FLR_WIDE", 1) != 0;
  // everywhere, including the 36-wide SG3 layers whose 32-column strips pad the output to 64 columns (r4: 70-74 us
  // against the 16-column tile kernel's 77 us per C2 layer, profiles/r4j_flr_wide_all.txt); knob IC2_FLR_WIDE_ALL=0
  // keeps the tile kernel where 32-column strips would pad wider than 16-column tiles
  static const bool wide_all = knob("IC2_FLR_WIDE_ALL", 1) != 0;
  if (in_f16 && wide && (wide_all || ceil_div(a.out_w, 32) * 32 <= ceil_div(a.out_w, 16) * 16) &&
      (int64_t)n * ceil_div(a.out_h, 16) * ceil_div(a.out_w, 32) * (a.c_p / 16) < (1LL << 31)) {
    if (up == 2) {
      if (delta == 0) fm2_launch<2, 0>(a, n, s);
      else fm2_launch<2, 1>(a, n, s);
    } else {
      switch (delta) {
        case 0: fm2_launch<4, 0>(a, n, s); break;
        case 1: fm2_launch<4, 1>(a, n, s); break;
        case 2: fm2_launch<4, 2>(a, n, s); break;
        default: fm2_launch<4, 3>(a, n, s); break;
      }
    }
    return IC2_OK;
  }
  a.tiles_x = (int)ceil_div(a.out_w, 16);
  a.tiles_y = (int)ceil_div(a.out_h, 16);
  a.cblocks = a.c_p / 16;
  const int64_t grid = (int64_t)n * a.tiles_y * a.tiles_x * a.cblocks;
  if (grid >= (1LL << 31)) return IC2_E_UNSUPPORTED;
  if (in_f16) fm_launch<true>(a, up, delta, (int)grid, s);
  else fm_launch<false>(a, up, delta, (int)grid, s);
  return IC2_OK;
}

}  // namespace ic2
