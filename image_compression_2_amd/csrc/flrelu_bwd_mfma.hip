// Backward of the fused filtered leaky-ReLU on the matrix cores: the bf16 training path's gradient w.r.t. a synthesis
// layer's conv output (/root/reference/stylegan3_hvae_full.py:669-696 trains the encoder through the frozen G;
// SG3-public filtered_lrelu's backward is the adjoint of upfirdn2d(fu, up) -> lrelu*gain, clamp -> upfirdn2d(fd, 2)).
//
// Per axis, in global coordinates (J: conv-output sample, K: lrelu-grid sample, O: layer-output sample, p0 the
// leading padding, gu = flipped fu * up, gd = flipped fd):
//   forward   U[K] = sum_J gu[U J + p0 - K] x[J]            out[O] = sum_K gd[K - 2 O] act(U[K])
//   backward  GA[K] = sum_O gd[K - 2 O] gout[O]     GU[K] = GA[K] * act'(U[K])     gx[J] = sum_K gu[U J + p0 - K] GU[K]
// Every pass is a banded matrix along one axis, so (as in the forward, flrelu_mfma.hip) each is an MFMA with 16
// channels on one side and 16 samples along the filtered axis on the other:
//   vertical:    V^T[c][ky]  = X^T[c][jy] . Gu^T          GAv^T[c][ky] = GO^T[c][oy] . Gd      (per column, from LDS)
//   horizontal:  U[kx][c]    = Gu . V[jx][c]              GA[kx][c]    = Gd^T . GAv[ox][c]    (per grid row)
//                GU = GA * act'(U) on the accumulators;   P^T[c][jx]   = GU^T[c][kx] . Gu      (GU is the A operand)
//   vertical:    GX^T[c][jy] += P^T[c][ky] . Gu           (per gx column, P from LDS)
// U is recomputed exactly as the forward computes it (f16 operands, f16 taps, V rounded to f16), so the lrelu / clamp
// decisions are the forward's; the gradient passes run on the gradient dtype's operands with f32 accumulation: bf16
// (the bf16 training path: the range of f16 does not hold an unscaled dL/dout) or f16 (GF16: the f16 training path,
// whose loss is scaled as the reference's GradScaler does, stylegan3_hvae_full.py:487,693-696; stores overflow to
// inf, never saturate, so the scaler sees an overflow).
//
// A work item is a strip: one sample x TJX gx columns x 16 channels x a run of 16-row tiles, walked top to bottom
// like the forward's strip kernel.  Tile t needs grid rows 16 U t - 6 U + 1 + p0 ... (21 U of them): NBT blocks of 16
// of which U are new per tile; the blocks shared with the next tile add their v-up^T share to its accumulator too.
// x rows stream through an LDS ring of U+1 groups of 16/U rows, gout rows through a ring of 3 groups of 8 rows
// (8 new per grid block at down 2).  P reuses each grid row's V row.
#include "flrelu_mfma.h"

#include <algorithm>
#include <cmath>
#include <type_traits>

namespace ic2 {

typedef short fb_s4 __attribute__((ext_vector_type(4)));

struct FlrBwdMArgs {
  const void* x;        // conv output that fed the forward, f16 NHWC [n][in_h][in_w][c_p]
  const void* gout;     // gradient of the layer output, bf16 NHWC [n][out_h][out_w][c_p]
  void* gx;             // gradient of x times oscale, bf16 NHWC
  const float* oscale;  // [n][c_p] or null
  int c_p, in_h, in_w, out_h, out_w, p0;
  int tiles_x, tiles_y, cblocks;
  float slope, gain, lim;  // lim = clamp / gain (+inf: no clamp)
  float gu[24], gd[12];
};

template <int U, int TJX>
struct FbmGeom {
  static constexpr int NW = 8;
  static constexpr int S = 16 / U;                         // x rows per grid block (one ring group)
  static constexpr int NGX = U + 1;                        // x ring groups
  static constexpr int NBT = (21 * U + 15) / 16;           // grid blocks per 16-row tile (3 / 6)
  static constexpr int NBX = (U * (TJX - 1) + 6 * U + 15) / 16;  // grid-column blocks of a strip (3 / 4)
  static constexpr int NG = NBT > NBX ? NBT : NBX;         // v-up^T / h-up^T tap matrices
  static constexpr int NINX = (16 * (NBX - 1) / U + 6 + 15 / U) | 1;  // x columns (29 / 21), odd
  static constexpr int NOX = (8 * (NBX - 1) + 14) | 1;     // gout columns (31 / 39), odd
  static constexpr int OCW = TJX / NW;                     // gx columns per wave
  // LDS (dwords).  Ring groups in whole 1-KiB DMA instructions; rows [x][16 ch] at 8 dwords per sample (odd sample
  // counts: 8 rows of a transposed read hit 8 bank groups)
  static constexpr int XP = NINX * 8, GP = NOX * 8;
  static constexpr int XGI = (S * NINX * 2 + 63) / 64, GGI = (8 * NOX * 2 + 63) / 64;  // DMA instructions per group
  static constexpr int XG_DW = XGI * 256, GG_DW = GGI * 256;
  static constexpr int XR_DW = NGX * XG_DW, GR_DW = 3 * GG_DW;
  static constexpr int VP = NINX * 8 + 2, AP = NOX * 8 + 2;  // V / GAv rows: 16 rows of b64 writes hit 16 bank pairs
  static constexpr int V_DW = 16 * VP, A_DW = 16 * AP;
  static constexpr int P_XP = 10;                          // P (in V's rows): [ky][jx][16 ch] at 10 dwords per jx
  static constexpr int TAPS = 220;                         // gu at [80, 80 + 6U), gd at [188, 200), zero guards
  static constexpr int LDS_DW = XR_DW + GR_DW + V_DW + A_DW;
  static_assert(16 * P_XP <= VP, "a P row fits in its V row");
  static_assert(A_DW >= TAPS, "the tap table aliases GAv");
  static_assert(LDS_DW * 4 <= 80 * 1024, "two workgroups per CU");
  static_assert(TJX % NW == 0 && TJX <= 16, "gx columns");
  // the surplus columns' transposed reads (up to NW * ceil(N / NW) columns) of the last ring row stay in the ring
  static_assert((NGX - 1) * XG_DW + (S - 1) * XP + 8 * NW * ((NINX + NW - 1) / NW) <= XR_DW, "x ring bounds");
  static_assert(2 * GG_DW + 7 * GP + 8 * NW * ((NOX + NW - 1) / NW) <= GR_DW, "gout ring bounds");
};

// gradient-dtype helpers: GF16 = f16 operands (IEEE conversion: overflow -> inf), else bf16
template <bool GF16>
__device__ __forceinline__ uint32_t fb_g2(float a, float b) {
  if constexpr (GF16) return fm_h2u(a, b);
  else return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
}
template <bool GF16>
__device__ __forceinline__ fb_s4 fb_g4(float a, float b, float c, float d) {
  return __builtin_bit_cast(fb_s4, make_uint2(fb_g2<GF16>(a, b), fb_g2<GF16>(c, d)));
}
template <bool GF16>
__device__ __forceinline__ fm_f4 fb_mfma_g(fb_s4 a, fb_s4 b, fm_f4 c) {
  if constexpr (GF16)
    return __builtin_amdgcn_mfma_f32_16x16x16f16(__builtin_bit_cast(fm_h4, a), __builtin_bit_cast(fm_h4, b), c, 0, 0, 0);
  else return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ fm_f4 fb_mfma_f16(fm_h4 a, fm_h4 b, fm_f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x16f16(a, b, c, 0, 0, 0);
}
// act'(u) * ga: the forward's lrelu * gain clamped to +-clamp, differentiated (0 where the clamp is active)
__device__ __forceinline__ float fb_dact(float u, float ga, float slope, float gain, float lim) {
  const float gs = u > 0.f ? gain : gain * slope;
  const float l = u > 0.f ? u : -u * slope;
  return l < lim ? ga * gs : 0.f;
}

// the item's oscale row: 1 (default) = DMA'd into a 64-B LDS slot by four lanes of the last wave with the ring groups,
// as the forward strip kernel DMAs its post-scale row (flrelu_mfma.hip flrelu_mfma3_kernel ps_lds), retired by the
// item-top vmcnt + barrier; 0 = a plain global load per lane and a vmcnt(0) at the item top.  (Round 3 fell back to 0
// after wrong rows; the cause was fm_dma16's missing wait states, flrelu_mfma.h; 2 = the diagnostic build that found it)
#ifndef FBM_OS_DMA
#define FBM_OS_DMA 1
#endif
#if FBM_OS_DMA == 2
// diagnostic (FBM_OS_DMA=2): the DMA'd row is checked against a plain load of the same row; mismatches are counted
// per (first item / later item), per wave, and the first one is described (item, wave, lane, got, want, and whether the
// value read is the previous item's row)
// g_fbm_dbg[63] is the mode: bit 0 = at the DMA's issue (block kend of the previous item) wave NW-1 waits for it and
// checks the slot itself ([5] good, [6] bad there); [42..57] the slot's 16 dwords at the first bad read, [58..61] the
// first LDS dword indices (of this workgroup's allocation) holding the expected value's bits, [62] the item the slot's
// last DMA was issued for (recorded in LDS by the issuing lane)
__device__ unsigned int g_fbm_dbg[64];
extern "C" int ic2_fbm_debug_fetch(unsigned int* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_fbm_dbg), sizeof(g_fbm_dbg), 0, hipMemcpyDeviceToHost);
}
extern "C" int ic2_fbm_debug_reset(unsigned int mode) {
  unsigned int z[64] = {};
  z[63] = mode;
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_fbm_dbg), z, sizeof(z), 0, hipMemcpyHostToDevice);
}
#endif

template <int U, int TJX, bool GF16>
__global__ void __launch_bounds__(512, 4) flrelu_bwd_mfma_kernel(FlrBwdMArgs a, int nitems, int nseg, int seg_len) {
  using G = FbmGeom<U, TJX>;
  constexpr int NW = G::NW, NT = 64 * NW, NBT = G::NBT, NBX = G::NBX, NINX = G::NINX, NOX = G::NOX, S = G::S;
  constexpr int OCW = G::OCW, NGX = G::NGX;
  __shared__ __attribute__((aligned(16))) uint32_t lds[G::LDS_DW + (FBM_OS_DMA ? (FBM_OS_DMA == 2 ? 32 : 16) : 0)];
  uint32_t* const xring = lds;
  uint32_t* const os_lds = lds + G::LDS_DW;  // FBM_OS_DMA: the item's oscale row (its own slot)
  uint32_t* const gring = lds + G::XR_DW;
  uint32_t* const v_img = gring + G::GR_DW;  // V (f16), then P (bf16) row by row
  uint32_t* const a_img = v_img + G::V_DW;   // GAv (bf16)
  float* const taps = reinterpret_cast<float*>(a_img);  // read only before the first item

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, li = lane & 15;
  const int tq = li >> 2, tp = li & 3;

  for (int i = tid; i < G::TAPS; i += NT) {
    float v = 0.f;
    if (i >= 80 && i < 80 + 6 * U) v = a.gu[i - 80];
    else if (i >= 188 && i < 200) v = a.gd[i - 188];
    taps[i] = v;
  }
  auto gu_t = [&](int t) { return taps[80 + t]; };   // t in [-72, 84)
  auto gd_t = [&](int t) { return taps[188 + t]; };  // t in [-20, 32)

  const int slot = fm_xcd_remap(blockIdx.x, gridDim.x);
  const uint16_t* xin = reinterpret_cast<const uint16_t*>(a.x);
  const uint16_t* gin = reinterpret_cast<const uint16_t*>(a.gout);
  auto item_geom = [&](int w, int& n, int& jx0, int& c0, int& t0, int& nt) {
    const int cb = w % a.cblocks;
    w /= a.cblocks;
    const int seg = w % nseg;
    w /= nseg;
    const int tx = w % a.tiles_x;
    n = w / a.tiles_x;
    jx0 = tx * TJX;
    c0 = cb * 16;
    t0 = seg * seg_len;
    nt = min(seg_len, a.tiles_y - t0);
  };
  // first gout row / column of a strip whose first grid row / column is k0: ceil((k0 - 11) / 2)
  auto o_first = [](int k0) { return (k0 - 10) >> 1; };
  const int xsy = a.in_w * a.c_p, osy = a.out_w * a.c_p;  // < 2^31 elements per sample: checked by the launcher

  // ring group q of an item: x rows 16 t0 - 5 + qS .., gout rows oy0 + 8q .., into slot q mod (groups); the lane's
  // (row, column, half) is recomputed per DMA from an opaque lane id (loop-invariant hoisting spills)
  auto load_xgroup = [&](int n, int iy0, int ix0, int c0, int q) __attribute__((always_inline)) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(xin + (int64_t)n * a.in_h * xsy + c0), 0, FM_OOB, 0x00020000);
    uint32_t* const dst = xring + (q % NGX) * G::XG_DW;
    int ln = lane;
    asm volatile("" : "+v"(ln));
#pragma unroll
    for (int i = 0; i < (G::XGI + NW - 1) / NW; ++i) {
      const int k = wave + NW * i;
      if (k < G::XGI) {
        const int e = k * 64 + ln;
        const int pix = e >> 1;
        const int row = pix / NINX, col = pix - row * NINX;
        const int iy = iy0 + q * S + row, ix = ix0 + col;
        const bool ok = e < S * NINX * 2 && (unsigned)iy < (unsigned)a.in_h && (unsigned)ix < (unsigned)a.in_w;
        const uint32_t off = ok ? (uint32_t)((iy * xsy + ix * a.c_p + (e & 1) * 8) * 2) : FM_OOB;
        fm_dma16(rs, off, dst + k * 256);
      }
    }
  };
  auto load_ggroup = [&](int n, int oy0, int ox0, int c0, int q) __attribute__((always_inline)) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(gin + (int64_t)n * a.out_h * osy + c0), 0, FM_OOB, 0x00020000);
    uint32_t* const dst = gring + (q % 3) * G::GG_DW;
    int ln = lane;
    asm volatile("" : "+v"(ln));
#pragma unroll
    for (int i = 0; i < (G::GGI + NW - 1) / NW; ++i) {
      const int k = wave + NW * i;
      if (k < G::GGI) {
        const int e = k * 64 + ln;
        const int pix = e >> 1;
        const int row = pix / NOX, col = pix - row * NOX;
        const int oy = oy0 + q * 8 + row, ox = ox0 + col;
        const bool ok = e < 8 * NOX * 2 && (unsigned)oy < (unsigned)a.out_h && (unsigned)ox < (unsigned)a.out_w;
        const uint32_t off = ok ? (uint32_t)((oy * osy + ox * a.c_p + (e & 1) * 8) * 2) : FM_OOB;
        fm_dma16(rs, off, dst + k * 256);
      }
    }
  };
  // geometry of an item: x origin (row of ring row 0, column of tile column 0), gout origin
  struct Org { int iy0, ix0, oy0, ox0; };
  auto origin = [&](int jx0, int t0) {
    Org o;
    o.iy0 = 16 * t0 - 5;
    o.ix0 = jx0 - 5;
    o.oy0 = o_first(16 * U * t0 + a.p0 - 6 * U + 1);
    o.ox0 = o_first(U * jx0 + a.p0 - 6 * U + 1);
    return o;
  };
  auto load_item = [&](int w) __attribute__((always_inline)) {
    int n, jx0, c0, t0, nt;
    item_geom(w, n, jx0, c0, t0, nt);
    const Org o = origin(jx0, t0);
#pragma unroll
    for (int q = 0; q < NGX; ++q) load_xgroup(n, o.iy0, o.ix0, c0, q);
#pragma unroll
    for (int q = 0; q < 3; ++q) load_ggroup(n, o.oy0, o.ox0, c0, q);
    if (FBM_OS_DMA && a.oscale != nullptr && wave == NW - 1 && lane < 4) {  // 64 B: oscale[n][c0 .. c0 + 16)
      const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(a.oscale + (int64_t)n * a.c_p + c0), 0, 64, 0x00020000);
      fm_dma16(prs, lane * 16, os_lds);
#if FBM_OS_DMA == 2
      if (lane == 0) os_lds[16] = (uint32_t)w;
      if (g_fbm_dbg[63] & 1u) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const float want = a.oscale[(int64_t)n * a.c_p + c0 + 4 * lane];
        const uint32_t got = os_lds[4 * lane];
        atomicAdd(&g_fbm_dbg[got == __float_as_uint(want) ? 5 : 6], 1u);
      }
#endif
    }
  };
  if (slot < nitems) load_item(slot);
  __syncthreads();  // taps

  // ---- tap matrices (see the header for the passes).  r0 = K0 - 2 O0 of every strip (10 or 11: the parity of
  // p0 + 1, the same on both axes)
  const int r0 = (a.p0 - 6 * U + 1) - 2 * o_first(a.p0 - 6 * U + 1);
  fm_h4 gmy, gmx[NBX];  // f16: vertical up B [jj][kk]; horizontal up A [kk][jj] over the clipped V window of block tt
  fb_s4 gdy, gdx[NBX];  // gradient dtype: vertical GA B [oo][kk]; horizontal GA A [kk][oo] over the clipped GAv window
  fb_s4 gT[G::NG];      // gradient dtype: h-up^T / v-up^T B [k][j] of grid block b: gu[U j + 6U - 1 - 16 b - k]
  {
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = gu_t(U * (4 * g + j) + U - 1 - li);
    gmy = fm_h4_of(fm_pack4(v[0], v[1], v[2], v[3]));
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = gd_t(r0 + li - 2 * (4 * g + j));
    gdy = fb_g4<GF16>(v[0], v[1], v[2], v[3]);
#pragma unroll
    for (int tt = 0; tt < NBX; ++tt) {
      const int wv = min(16 * tt / U, NINX - 16), wo = min(8 * tt, NOX - 16);
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = gu_t(U * (wv + 4 * g + j) + U - 1 - 16 * tt - li);
      gmx[tt] = fm_h4_of(fm_pack4(v[0], v[1], v[2], v[3]));
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = gd_t(r0 + 16 * tt + li - 2 * (wo + 4 * g + j));
      gdx[tt] = fb_g4<GF16>(v[0], v[1], v[2], v[3]);
    }
#pragma unroll
    for (int b = 0; b < G::NG; ++b) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = gu_t(U * li + 6 * U - 1 - 16 * b - (4 * g + j));
      gT[b] = fb_g4<GF16>(v[0], v[1], v[2], v[3]);
    }
  }
  const float slope = a.slope, gain = a.gain, lim = a.lim;
  uint16_t* gxo = reinterpret_cast<uint16_t*>(a.gx);
  __syncthreads();  // every wave's tap reads are done before the first GAv store overwrites the table

  bool first = true;
#if FBM_OS_DMA == 2
  int prev_w = -1;
#endif
  for (int w = slot; w < nitems; w += gridDim.x) {
    int n, jx0, c0, t0, nt;
    item_geom(w, n, jx0, c0, t0, nt);
    const Org o = origin(jx0, t0);
    const bool has_next = w + (int)gridDim.x < nitems;
#if FBM_OS_DMA == 2
    const bool first_item = first;
#endif
    if (first) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(OCW) : "memory");  // the previous item's last stores stay in flight
    first = false;
    __syncthreads();
    // the item's oscale[n][c0 + 4g .. +3], retired here with a waitcnt the compiler accounts for (its own wait would
    // land at the first tile's epilogue, behind the ring DMAs issued by then)
    float4 osv = make_float4(1.f, 1.f, 1.f, 1.f);
    if (a.oscale) {
      if (FBM_OS_DMA) {
        osv = *reinterpret_cast<const float4*>(os_lds + 4 * g);  // landed: the wait + barrier above
#if FBM_OS_DMA == 2
        const float4 ref = *reinterpret_cast<const float4*>(a.oscale + (int64_t)n * a.c_p + c0 + 4 * g);
        const float* rp = &ref.x;
        const float* gp = &osv.x;
        bool bad = false;
        for (int j = 0; j < 4; ++j) bad |= __float_as_uint(rp[j]) != __float_as_uint(gp[j]);
        if (bad) {
          atomicAdd(&g_fbm_dbg[0], 1u);
          atomicAdd(&g_fbm_dbg[first_item ? 1 : 2], 1u);
          atomicAdd(&g_fbm_dbg[8 + wave], 1u);
          atomicAdd(&g_fbm_dbg[16 + g], 1u);
          if (prev_w >= 0) {  // is it the previous item's row?
            int pn, pj, pc, pt, pnt;
            item_geom(prev_w, pn, pj, pc, pt, pnt);
            const float4 pv = *reinterpret_cast<const float4*>(a.oscale + (int64_t)pn * a.c_p + pc + 4 * g);
            if (__float_as_uint(pv.x) == __float_as_uint(osv.x)) atomicAdd(&g_fbm_dbg[3], 1u);
          }
          if (atomicCAS(&g_fbm_dbg[32], 0u, 1u) == 0u) {
            g_fbm_dbg[33] = (unsigned)w; g_fbm_dbg[34] = (unsigned)wave; g_fbm_dbg[35] = (unsigned)lane;
            g_fbm_dbg[36] = __float_as_uint(osv.x); g_fbm_dbg[37] = __float_as_uint(ref.x);
            g_fbm_dbg[38] = (unsigned)prev_w; g_fbm_dbg[39] = (unsigned)blockIdx.x;
            g_fbm_dbg[40] = (unsigned)nitems; g_fbm_dbg[41] = (unsigned)gridDim.x;
            for (int j = 0; j < 16; ++j) g_fbm_dbg[42 + j] = os_lds[j];
            int hits = 0;
            for (int j = 0; j < G::LDS_DW + 16 && hits < 4; ++j)
              if (lds[j] == __float_as_uint(ref.x)) g_fbm_dbg[58 + hits++] = (unsigned)j;
            g_fbm_dbg[62] = os_lds[16];
          }
        }
        atomicAdd(&g_fbm_dbg[4], 1u);  // rows read
#endif
      } else {
        osv = *reinterpret_cast<const float4*>(a.oscale + (int64_t)n * a.c_p + c0 + 4 * g);
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
      }
    }
    const float osc[4] = {osv.x, osv.y, osv.z, osv.w};
    const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(gxo + (int64_t)n * a.in_h * xsy + c0), 0, FM_OOB, 0x00020000);
    const int kend = U * (nt - 1) + NBT - 1;  // blocks 0 .. kend

    fm_f4 accA[OCW], accB[OCW];  // accA: the older of the two tiles a block can feed, accB: the newer
#pragma unroll
    for (int i = 0; i < OCW; ++i) accA[i] = accB[i] = fm_f4{0.f, 0.f, 0.f, 0.f};

    // grid block k = U t1 + BB (BB compile-time): feeds tile t1 as its block BB and tile t1 - 1 as its block BB + U
    auto block = [&](int k, int t1, auto bb_c) __attribute__((always_inline)) {
      constexpr int BB = decltype(bb_c)::value;
      // ---- A: vertical up (x ring -> V) and vertical GA (gout ring -> GAv), one column per MFMA
      {
        constexpr int NC = (NINX + NW - 1) / NW;
        const int q = k + (4 * g + tq) / S;
        const uint32_t* rowp = xring + (q % NGX) * G::XG_DW + ((4 * g + tq) % S) * G::XP + 2 * tp + wave * 8;
        fm_s4 xa[NC];
#pragma unroll
        for (int i = 0; i < NC; ++i) xa[i] = fm_tr_read(rowp + i * NW * 8);  // surplus columns read in-bounds bytes
        constexpr int NCO = (NOX + NW - 1) / NW;
        const int qo = k + (4 * g + tq) / 8;
        const uint32_t* orow = gring + (qo % 3) * G::GG_DW + ((4 * g + tq) % 8) * G::GP + 2 * tp + wave * 8;
        fm_s4 ga_[NCO];
#pragma unroll
        for (int i = 0; i < NCO; ++i) ga_[i] = fm_tr_read(orow + i * NW * 8);
        __builtin_amdgcn_sched_barrier(0);
        fm_f4 vt[NC], at[NCO];
#pragma unroll
        for (int i = 0; i < NC; ++i) vt[i] = fb_mfma_f16(__builtin_bit_cast(fm_h4, xa[i]), gmy, fm_f4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
        for (int i = 0; i < NCO; ++i) at[i] = fb_mfma_g<GF16>(ga_[i], gdy, fm_f4{0.f, 0.f, 0.f, 0.f});
        __builtin_amdgcn_sched_barrier(0);
        // V overwrites P: every wave's v-up^T reads of block k-1 are done (block 0: the item-top barrier)
        if (k > 0) __syncthreads();
        uint32_t* const vp = v_img + li * G::VP + 2 * g + wave * 8;
#pragma unroll
        for (int i = 0; i < NC; ++i)
          if (i < NC - 1 || wave + NW * i < NINX)
            *reinterpret_cast<uint2*>(vp + i * NW * 8) = fm_pack4(vt[i][0], vt[i][1], vt[i][2], vt[i][3]);
        uint32_t* const ap = a_img + li * G::AP + 2 * g + wave * 8;
#pragma unroll
        for (int i = 0; i < NCO; ++i)
          if (i < NCO - 1 || wave + NW * i < NOX)
            *reinterpret_cast<uint2*>(ap + i * NW * 8) = make_uint2(fb_g2<GF16>(at[i][0], at[i][1]), fb_g2<GF16>(at[i][2], at[i][3]));
      }
      __syncthreads();  // B1: V and GAv complete; the ring groups k are dead; every wave's v-up^T of block k-1 done
      if (k == kend && has_next) load_item(w + gridDim.x);  // every ring slot is dead: the next item's first rows
      // ---- B: per grid row of this wave: U and GA over the strip's grid columns, GU = GA act'(U), P^T = GU^T Gu
#pragma unroll
      for (int rr = 0; rr < 16 / NW; ++rr) {
        const int row = wave + NW * rr;
        fm_s4 vb[NBX], gb[NBX];
#pragma unroll
        for (int tt = 0; tt < NBX; ++tt) {
          const int wv = min(16 * tt / U, NINX - 16), wo = min(8 * tt, NOX - 16);
          vb[tt] = fm_tr_read(v_img + row * G::VP + (wv + 4 * g + tq) * 8 + 2 * tp);
          gb[tt] = fm_tr_read(a_img + row * G::AP + (wo + 4 * g + tq) * 8 + 2 * tp);
        }
        __builtin_amdgcn_sched_barrier(0);
        fm_f4 u[NBX], ga[NBX];
#pragma unroll
        for (int tt = 0; tt < NBX; ++tt) {
          u[tt] = fb_mfma_f16(gmx[tt], __builtin_bit_cast(fm_h4, vb[tt]), fm_f4{0.f, 0.f, 0.f, 0.f});
          ga[tt] = fb_mfma_g<GF16>(gdx[tt], gb[tt], fm_f4{0.f, 0.f, 0.f, 0.f});
        }
        __builtin_amdgcn_sched_barrier(0);
        fm_f4 pt = fm_f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int tt = 0; tt < NBX; ++tt) {
          // U as the forward stores it (f16) decides the lrelu side and the clamp
          float uu[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) uu[r] = (float)(_Float16)u[tt][r];
          const fb_s4 gu4 = fb_g4<GF16>(fb_dact(uu[0], ga[tt][0], slope, gain, lim), fb_dact(uu[1], ga[tt][1], slope, gain, lim),
                                   fb_dact(uu[2], ga[tt][2], slope, gain, lim), fb_dact(uu[3], ga[tt][3], slope, gain, lim));
          pt = fb_mfma_g<GF16>(gu4, gT[tt], pt);
        }
        __builtin_amdgcn_sched_barrier(0);
        // P row `row` over this wave's own V row (its reads of it above are done: LDS ops of a wave run in order)
        *reinterpret_cast<uint2*>(v_img + row * G::VP + li * G::P_XP + 2 * g) =
            make_uint2(fb_g2<GF16>(pt[0], pt[1]), fb_g2<GF16>(pt[2], pt[3]));
      }
      // B2: the ring groups loaded at block k-1 (for block k+1) must have landed; the stores of a tile finished at
      // block k-1 (issued after that DMA, exactly OCW) may stay in flight
      constexpr int BBP = (BB + U - 1) % U;  // block k-1's position
      constexpr bool STORED_PREV = ((NBT - 1) % U) == BBP;
      if (k >= 1 && k < kend) {
        if (STORED_PREV && k - 1 >= NBT - 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(OCW) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __syncthreads();  // P complete; every wave's h-pass reads of V / GAv are done
      if (k + 2 <= kend) {  // groups of block k+2 (x group k and gout group k are dead)
        load_xgroup(n, o.iy0, o.ix0, c0, k + U + 1);
        load_ggroup(n, o.oy0, o.ox0, c0, k + 3);
      }
      // ---- C: vertical up^T into the gx tiles this block feeds
      {
        fm_s4 pa[OCW];
#pragma unroll
        for (int i = 0; i < OCW; ++i)
          pa[i] = fm_tr_read(v_img + (4 * g + tq) * G::VP + (wave + NW * i) * G::P_XP + 2 * tp);
        __builtin_amdgcn_sched_barrier(0);
        if (t1 < nt) {
#pragma unroll
          for (int i = 0; i < OCW; ++i) accB[i] = fb_mfma_g<GF16>(pa[i], gT[BB], accB[i]);
        }
        if constexpr (BB + U < NBT) {
          if (t1 >= 1) {
#pragma unroll
            for (int i = 0; i < OCW; ++i) accA[i] = fb_mfma_g<GF16>(pa[i], gT[BB + U], accA[i]);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      // tile t1 - 1 complete: store gx * oscale (exactly OCW buffer stores per wave; out of range -> FM_OOB)
      if constexpr (BB + U == NBT - 1) {
        if (t1 >= 1) {
          const int gy = 16 * (t0 + t1 - 1) + li;
#pragma unroll
          for (int i = 0; i < OCW; ++i) {
            const int gxc = jx0 + wave + NW * i;
            const uint32_t off = (gy < a.in_h && gxc < a.in_w) ? (uint32_t)((gy * xsy + gxc * a.c_p + 4 * g) * 2) : FM_OOB;
            const uint2 v = make_uint2(fb_g2<GF16>(accA[i][0] * osc[0], accA[i][1] * osc[1]),
                                       fb_g2<GF16>(accA[i][2] * osc[2], accA[i][3] * osc[3]));
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u32_t, v), ors, off, 0, 0);
          }
        }
      }
    };

    // blocks in order; at the first block of each tile t1 the accumulators shift (accA <- tile t1 - 1)
    for (int t1 = 0; U * t1 <= kend; ++t1) {
      if (t1 >= 1) {
#pragma unroll
        for (int i = 0; i < OCW; ++i) {
          accA[i] = accB[i];
          accB[i] = fm_f4{0.f, 0.f, 0.f, 0.f};
        }
      }
      block(U * t1, t1, std::integral_constant<int, 0>{});
      if (U * t1 + 1 <= kend) block(U * t1 + 1, t1, std::integral_constant<int, 1>{});
      if constexpr (U == 4) {
        if (U * t1 + 2 <= kend) block(U * t1 + 2, t1, std::integral_constant<int, 2>{});
        if (U * t1 + 3 <= kend) block(U * t1 + 3, t1, std::integral_constant<int, 3>{});
      }
    }
#if FBM_OS_DMA == 2
    prev_w = w;
#endif
  }
}

template <int U, int TJX, bool GF16>
static void fbm_launch(FlrBwdMArgs a, int n, hipStream_t s) {
  a.tiles_x = (int)ceil_div(a.in_w, TJX);
  a.tiles_y = (int)ceil_div(a.in_h, 16);
  a.cblocks = a.c_p / 16;
  static int resident = 0;
  if (resident == 0) {
    int dev = 0, cus = 0, per_cu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, flrelu_bwd_mfma_kernel<U, TJX, GF16>, 512, 0);
    resident = (cus > 0 ? cus : 256) * (per_cu > 0 ? per_cu : 1);
  }
  // strip segmentation as the forward's (fm_strip_segments); knob IC2_FLRB_SEGS=0 keeps the round-3 rule
  static const int segs_mode = knob("IC2_FLRB_SEGS", 1);
  const int64_t nstrips = (int64_t)n * a.tiles_x * a.cblocks;
  int nseg = fm_strip_segments(nstrips, a.tiles_y, resident, segs_mode == 1);
  const int seg_len = (int)ceil_div(a.tiles_y, nseg);
  nseg = (int)ceil_div(a.tiles_y, seg_len);
  const int nitems = (int)(nstrips * nseg);
  const int grid = nitems < resident ? nitems : resident;
  hipLaunchKernelGGL((flrelu_bwd_mfma_kernel<U, TJX, GF16>), dim3((unsigned)grid), dim3(512), 0, s, a, nitems, nseg, seg_len);
}

// per (sample, pixel chunk, channel) sums of gx * (x - bias) = dc * (x - bias) / oscale: the modulated conv's
// d oscale numerator (as the f32 kernel's ydot) from the stored dc = gx * oscale; chunk c covers pixels
// [c * per, (c + 1) * per)
template <bool GF16>
__global__ void __launch_bounds__(256) fb_ydot_kernel(const uint16_t* __restrict__ dc, const uint16_t* __restrict__ x,
                                                      const float* __restrict__ oscale, const float* __restrict__ bias,
                                                      float* __restrict__ part, int hw, int c_p, int nchunks, int per) {
  // thread t: channel octet (t mod octs) of pixels p0 + t / octs, stepping by 256 / octs (16-B loads); two pixels in
  // flight per thread; fixed-order reduction over the pixel lanes in LDS
  __shared__ float red[256 * 9];
  const int n = blockIdx.y, chunk = blockIdx.x;
  const int p0 = chunk * per, p1 = min(hw, p0 + per);
  const int C8 = c_p >> 3;
  for (int cbase = 0; cbase < C8; cbase += 256) {
    const int octs = min(256, C8 - cbase);
    const int lanes = 256 / octs;
    const int t = threadIdx.x;
    const int o8 = t % octs, pl = t / octs;
    const int c = 8 * (cbase + o8);
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    if (pl < lanes) {
      float b[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) b[j] = bias ? bias[c + j] : 0.f;
      const int64_t base = (int64_t)n * hw * c_p + c;
#pragma unroll 2
      for (int p = p0 + pl; p < p1; p += lanes) {
        const uint4 dv = *reinterpret_cast<const uint4*>(dc + base + (int64_t)p * c_p);
        const uint4 xv = *reinterpret_cast<const uint4*>(x + base + (int64_t)p * c_p);
        const uint32_t dw[4] = {dv.x, dv.y, dv.z, dv.w}, xw[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const fm_h2 xh = __builtin_bit_cast(fm_h2, xw[k]);
          float d0, d1;
          if constexpr (GF16) {
            const fm_h2 dh = __builtin_bit_cast(fm_h2, dw[k]);
            d0 = (float)dh.x;
            d1 = (float)dh.y;
          } else {
            d0 = __uint_as_float(dw[k] << 16);
            d1 = __uint_as_float(dw[k] & 0xffff0000u);
          }
          acc[2 * k] += d0 * ((float)xh.x - b[2 * k]);
          acc[2 * k + 1] += d1 * ((float)xh.y - b[2 * k + 1]);
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 8; ++j) red[t * 9 + j] = acc[j];
    __syncthreads();
    if (t < octs) {
      float* pp = part + ((int64_t)n * nchunks + chunk) * c_p + c;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float sum = 0.f;
        for (int l = 0; l < lanes; ++l) sum += red[(l * octs + t) * 9 + j];
        if (oscale) {
          const float o = oscale[(int64_t)n * c_p + c + j];
          sum = o != 0.f ? sum / o : 0.f;
        }
        pp[j] = sum;
      }
    }
  }
}

// The training path's FLR backward on MFMA (called by ic2_flrelu_bwd_nhwc_ex for f16 x and bf16 gout / gx, or f16
// gout / gx with grad_f16; returns IC2_E_UNSUPPORTED for the geometries it has no instance for).  ydot (optional): n x nchunks x c_p partial
// sums of dc * (x - bias), nchunks = ydot_floats / (n c_p).
int flrelu_bwd_mfma_launch(const void* x, const void* gout, void* gx, const float* oscale, const float* bias,
                           float* ydot, int64_t ydot_floats, int n, int c_p, int in_h, int in_w, int out_h, int out_w,
                           const float* gu, const float* gd, int up, int p0, float gain, float slope, float lim,
                           bool grad_f16, hipStream_t s) {
  if (c_p % 16 != 0 || (up != 2 && up != 4)) return IC2_E_UNSUPPORTED;
  if ((int64_t)in_h * in_w * c_p * 2 >= (int64_t)FM_OOB || (int64_t)out_h * out_w * c_p * 2 >= (int64_t)FM_OOB)
    return IC2_E_UNSUPPORTED;
  if ((int64_t)n * ceil_div(in_h, 16) * ceil_div(in_w, 8) * (c_p / 16) >= (1LL << 31)) return IC2_E_UNSUPPORTED;
  FlrBwdMArgs a;
  a.x = x; a.gout = gout; a.gx = gx; a.oscale = oscale;
  a.c_p = c_p; a.in_h = in_h; a.in_w = in_w; a.out_h = out_h; a.out_w = out_w; a.p0 = p0;
  a.slope = slope; a.gain = gain; a.lim = lim;
  for (int t = 0; t < 24; ++t) a.gu[t] = gu[t];
  for (int t = 0; t < 12; ++t) a.gd[t] = gd[t];
  if (grad_f16) {
    if (up == 2) fbm_launch<2, 16, true>(a, n, s);
    else fbm_launch<4, 8, true>(a, n, s);
  } else {
    if (up == 2) fbm_launch<2, 16, false>(a, n, s);
    else fbm_launch<4, 8, false>(a, n, s);
  }
  if (ydot) {
    const int nchunks = (int)(ydot_floats / ((int64_t)n * c_p));
    if (nchunks < 1) return IC2_E_INVALID;
    const int hw = in_h * in_w, per = (int)ceil_div(hw, nchunks);
    if (grad_f16)
      hipLaunchKernelGGL(fb_ydot_kernel<true>, dim3((unsigned)nchunks, (unsigned)n), dim3(256), 0, s,
                         reinterpret_cast<const uint16_t*>(gx), reinterpret_cast<const uint16_t*>(x), oscale, bias, ydot,
                         hw, c_p, nchunks, per);
    else
      hipLaunchKernelGGL(fb_ydot_kernel<false>, dim3((unsigned)nchunks, (unsigned)n), dim3(256), 0, s,
                         reinterpret_cast<const uint16_t*>(gx), reinterpret_cast<const uint16_t*>(x), oscale, bias, ydot,
                         hw, c_p, nchunks, per);
  }
  return IC2_OK;
}

}  // namespace ic2
