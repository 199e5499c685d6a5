// Fused Winograd F(2,3)-along-x 3x3 convolution on CDNA4 MFMA (f16 operands, f32 accumulation).
//
// Replaces the grouped conv2d inside StyleGAN3's modulated_conv2d [SG3-public; call sites
// /root/reference/stylegan3_hvae_full.py:274,329] in its activation-scaling form (ic2_conv_igemm's contract for
// kh = kw = 3), for the f16 synthesis path.
//
// Along x every pair of outputs (2t, 2t+1) of a 3-tap row is the minimal filtering algorithm F(2,3):
//   V = B^T d  (d = the 4 input pixels 2t .. 2t+3 of the row), U = G g (the 3 taps), m = U . V (4 products),
//   y = A^T m,   B^T = [1 0 -1 0; 0 1 1 0; 0 -1 1 0; 0 1 0 -1], G = [1 0 0; .5 .5 .5; .5 -.5 .5; 0 0 1],
//   A^T = [1 1 1 0; 0 1 -1 -1],
// and along y the three kernel rows stay a direct sum.  Summed over channels, each of the 4 positions nu is a GEMM
// with K = (ky, channel): acc_nu[o][pair] = sum_{ky,c} U[o][ky][nu][c] * V_nu[c][row + ky][pair]; the output
// transform y0 = acc_0 + acc_1 + acc_2, y1 = acc_1 - acc_2 - acc_3 is lane-local in the epilogue.  12 products per
// output pair instead of 18: 2/3 of the direct conv's MFMA work.  (The 2-D F(2x2,3x3) would cut 4/9 of it but needs
// 4 accumulators per output pixel: at the register file's ~64 K accumulators per CU its tiles hold 64 outputs x 256
// pixels, and the 16 U slabs per K-step then cost 1.5x this kernel's L2 -> LDS bytes per useful FLOP.)
//
// Workgroup: 8 waves (2 per SIMD), 128 output channels x 128 output pairs (wx_th rows x wx_twp pairs of one image);
// wave (og, pg) owns 64 channels x 32 pairs x the 4 positions (128 accumulator registers).
// K-step = (32-channel block cb, kernel row ky); per step and wave: 16 A fragments (4 nu x 4 channel blocks of 16)
// from the U slab, 8 input fragments (4 pixels x 2 pair blocks) from the halo, 4 packed-f16 adds per V fragment,
// 32 v_mfma_f32_16x16x32_f16.
//   U slab of a step: rows (nu, o) x 32 channels = 32 KiB, a 3-slab ring (slab s+2 issued at step s).
//   Halo of a block: the (wx_th + 2) input rows x (2 wx_twp + 2) pixels x 32 channels, stored de-interleaved
//   ([row][x parity][x / 2], wx_hp = wx_twp + 1 64-B LDS rows per line), double-buffered, issued as one burst at the
//   block's first kernel row.  A 16-lane pair block is 16 consecutive pairs of ONE output row (a tile row is served
//   by wx_ns blocks), so a fragment read covers 16 consecutive LDS rows of one line.
//   LDS rows of 64 B.  U slab: 16-B chunk c stored at c ^ (((row >> 2) & 1) << 1) (hg4's conflict-free swizzle for 16
//   consecutive rows).  Halo: the same swizzle on the index WITHIN the line, so any line pitch and any kernel-row
//   shift keeps a read conflict-free (brute-forced over the ds_read_b128 lane groups; the round-5 first version,
//   swizzled on the absolute row with lanes wrapping across output rows, spent 25 % of its LDS cycles on conflicts).
// V is formed in f16 (packed adds, one rounding per add; the CPU emulation tools/wino_emu.py prices the rounding).
#include "conv_common.h"

namespace ic2 {

constexpr int WX_BO = 128, WX_NW = 8, WX_NS = 3;
constexpr int WX_SLAB = 4 * WX_BO * 64;                   // 32 KiB: one K-step's U (a 6 half-slab ring = 3 slabs)
constexpr int WX_HROWS = 384, WX_HALO = WX_HROWS * 64;    // 24 KiB
constexpr int WX_HPW = WX_HROWS / 16 / WX_NW;             // 3 halo DMAs per wave per block
constexpr int WX_SLACK = 8 * 1024;                        // idle lanes read past the last halo line (unused values)
constexpr int WX_LDS = WX_NS * WX_SLAB + 2 * WX_HALO + WX_SLACK;  // 155,648 B: one workgroup per CU
static_assert(WX_LDS <= 160 * 1024, "LDS");

// packed f16 add / subtract of 16-B fragments: 4 v_pk_add_f16 each (neg modifiers for the subtraction).  Written
// out because the compiler splits an 8-wide f16 vector subtraction into scalar v_sub_f16 + v_pack (3x the VALU).
typedef __attribute__((ext_vector_type(4))) uint32_t wx_u4;
__device__ __forceinline__ f16x8 wx_sub(f16x8 a, f16x8 b) {
  const wx_u4 x = __builtin_bit_cast(wx_u4, a), y = __builtin_bit_cast(wx_u4, b);
  wx_u4 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) asm("v_pk_add_f16 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r[i]) : "v"(x[i]), "v"(y[i]));
  return __builtin_bit_cast(f16x8, r);
}
__device__ __forceinline__ f16x8 wx_add(f16x8 a, f16x8 b) {
  const wx_u4 x = __builtin_bit_cast(wx_u4, a), y = __builtin_bit_cast(wx_u4, b);
  wx_u4 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) asm("v_pk_add_f16 %0, %1, %2" : "=v"(r[i]) : "v"(x[i]), "v"(y[i]));
  return __builtin_bit_cast(f16x8, r);
}

__device__ __forceinline__ int wx_off(int row, int chunk) { return row * 64 + ((chunk ^ (((row >> 2) & 1) << 1)) << 4); }
__device__ __forceinline__ int wx_hoff(int line, int hp, int idx, int chunk) {
  return (line * hp + idx) * 64 + ((chunk ^ (((idx >> 2) & 1) << 1)) << 4);
}

// diagnostic builds only (wrong results; tools/build_abl.sh wino): IC2_WX_ABL bit 0 skips the U DMAs after the first
// channel block, bit 1 the section barriers, bit 2 the input-fragment reads, bit 3 the MFMAs, bit 4 the DMA waits
#ifndef IC2_WX_ABL
#define IC2_WX_ABL 0
#endif
// diagnostic build IC2_WX_STAMP=1 (tools/build_abl.sh winostamp): s_memtime stamps around the sections, summed per
// wave over the K loop and stored to a.ws[(block * 8 + wave) * 8 + k] as u64 (the launch passes a buffer there):
// 0 R reads + V, 1 R DMA issue, 2 vmcnt wait, 3 barrier after R + lgkmcnt, 4 M issue, 5 barrier after M, 6 loop
#ifndef IC2_WX_STAMP
#define IC2_WX_STAMP 0
#endif
// schedule variants (A/B): 0 = reads, V, then DMAs in R; 1 = DMAs first in R; 2 = DMAs first, and the next step's
// input fragments read inside the second M section of the step (halo DMAs one section later to keep the WAR distance).
// (Round 6 also tried the next section's A fragments read inside this section's M section, right behind the MFMAs that
// consumed their registers, with and without the input fragments: level / 2-3 % slower, profiles/r6_schedule_ab.txt.)
#ifndef IC2_WX_SCHED
#define IC2_WX_SCHED 0
#endif
// wave priority A/B (diagnostic builds, tools/build_abl.sh winoprio): 0 = s_setprio 1 over the M section's MFMAs
// (default), 1 = no s_setprio, 2 = s_setprio 1 over the R section (reads, V adds, DMA issue) instead
#ifndef IC2_WX_PRIO
#define IC2_WX_PRIO 0
#endif

__global__ void __launch_bounds__(512, 1) wino_fx_f16_kernel(IgemmArgs a) {
  __shared__ __attribute__((aligned(16))) char lds[WX_LDS];
  char* const wsl = lds;
  char* const hal = lds + WX_NS * WX_SLAB;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int half = wid >> 2;  // positions 2 half, 2 half + 1; waves 4-7 also run one barrier behind (ping-pong)
  const int pg = wid & 3;     // pairs 32 pg .. 32 pg + 31
  const int fr = lane & 15, fh = lane >> 4;

  // logical tile -> (o-tile, pixel tile): the o-tiles run in groups of a.group (fastest within a group), each group
  // over all pixel tiles; the XCD remap hands every XCD a contiguous range, so its L2 holds the U slabs of one group
  const int logical = xcd_remap(blockIdx.x, a.nblocks);
  const int per_group = a.group * (a.nblocks / a.tiles_o);
  const int gi = logical / per_group, grem = logical - gi * per_group;
  const int o_tile = gi * a.group + grem % a.group;
  int pt = grem / a.group;
  const int tx = pt % a.wx_tx;
  pt /= a.wx_tx;
  const int ty = pt % a.wx_ty;
  const int nn = pt / a.wx_ty;
  const int o0 = o_tile * WX_BO;
  const int twp = a.wx_twp, hp = a.wx_hp;
  const int oy0 = ty * a.wx_th, px0 = tx * twp;  // first output row, first output pair of the tile

  const char* __restrict__ xg = reinterpret_cast<const char*>(a.x);
  const char* __restrict__ ug = reinterpret_cast<const char*>(a.w);
  const int lrow = lane >> 2, pch = lane & 3;  // DMA: 16 rows x 4 chunks of 16 B per instruction

  // U half-slab (step (cb, ky), channel half h): rows (nu, o0 + 64 h + r), r < 64: U[o][ky][nu][c] at
  // ((o * 3 + ky) * 4 + nu) * cin_p + c; the (cb, ky) part is the descriptor base.  2 DMAs per wave per half-slab.
  uint32_t w_off[2][2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int row = (wid + WX_NW * k) * 16 + lrow;
      const int nu = row >> 6, ol = h * 64 + (row & 63), o = o0 + ol;
      w_off[h][k] =
          o < a.cout_p ? (uint32_t)(((ol * 12 + nu) * a.cin_p) * 2 + ((pch ^ (((row >> 2) & 1) << 1)) << 4)) : kOob;
    }
  const char* const ug0 = ug + (int64_t)o0 * 12 * a.cin_p * 2;
  // halo rows l = (hr * 2 + parity) * hp + idx  <-  input pixel (oy0 - pad + hr, 2 px0 - pad + 2 idx + parity)
  uint32_t h_off[WX_HPW];
#pragma unroll
  for (int k = 0; k < WX_HPW; ++k) {
    const int l = (wid + WX_NW * k) * 16 + lrow;
    const int line = l / hp, idx = l - line * hp;
    const int iy = oy0 - a.pad + (line >> 1), ix = 2 * px0 - a.pad + 2 * idx + (line & 1);
    const bool ok = l < a.wx_nh && (unsigned)iy < (unsigned)a.h && (unsigned)ix < (unsigned)a.w_;
    h_off[k] = ok ? (uint32_t)((((nn * a.h + iy) * a.w_ + ix) * a.cin_p + ((pch ^ (((idx >> 2) & 1) << 1)) << 3)) * 2)
                  : kOob;
  }
  // input-fragment offsets at ky = 0: pair block b = 2 pg + jb is 16 pairs of tile row b / ns; this half's 3 of the
  // pair's 4 pixels (half + m, m < 3: positions 0, 1 use pixels 0..2, positions 2, 3 pixels 1..3).  Lanes past the
  // tile's pairs read past their line (conflict-free, unused); blocks past the tile's rows repeat its last row.
  int boff[2][3];
  const int ns = a.wx_ns;
#pragma unroll
  for (int jb = 0; jb < 2; ++jb) {
    const int b = pg * 2 + jb;
    const int rr = min(b / ns, a.wx_th - 1), t = (b % ns) * 16 + fr;
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      const int j = half + m;
      boff[jb][m] = wx_hoff(rr * 2 + (j & 1), hp, t + (j >> 1), fh);
    }
  }
  const int ky_step = 2 * hp * 64;  // bytes per kernel row in the halo
  const int aoff = wx_off(fr, fh) + half * 2 * 64 * 64;
  const int CB = a.cin_p >> 5;

  // half-slab j (0..5) of block cb: kernel row j >> 1, channel half j & 1 -> ring slot j (size 0 past the end)
  auto issue_hs = [&](int cb, int j) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(ug0 + ((int64_t)(4 * (j >> 1)) * a.cin_p + cb * 32) * 2), 0, cb < CB ? kOob : 0, kRsrcWord3);
    char* dst = wsl + j * (WX_SLAB / 2);
#pragma unroll
    for (int k = 0; k < 2; ++k)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs, (__attribute__((address_space(3))) void*)(dst + (wid + WX_NW * k) * 1024), 16, w_off[j & 1][k], 0, 0, 0);
  };
  auto issue_hp = [&](int cb, int k) {  // DMA k of this wave for the halo of block cb -> halo cb & 1
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(xg + (int64_t)cb * 64), 0, cb < CB ? kOob : 0, kRsrcWord3);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        rs, (__attribute__((address_space(3))) void*)(hal + (cb & 1) * WX_HALO + (wid + WX_NW * k) * 1024), 16,
        h_off[k], 0, 0, 0);
  };

  f32x4 acc[2][8][2];  // [position - 2 half][16-channel block][pair block]
#pragma unroll
  for (int nl = 0; nl < 2; ++nl)
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int jb = 0; jb < 2; ++jb) acc[nl][i][jb] = f32x4{0.f, 0.f, 0.f, 0.f};

  // this half's 3 input fragments of a step -> its 2 V fragments (B^T d), packed f16 adds:
  //   positions 0, 1 (pixels 0..2): V0 = d0 - d2, V1 = d1 + d2;  positions 2, 3 (pixels 1..3): V2 = d2 - d1, V3 = d1 - d3
  f16x8 d[2][3];
  f16x8 v[2][2];
  auto read_d = [&](const char* hl) {
#pragma unroll
    for (int jb = 0; jb < 2; ++jb)
#pragma unroll
      for (int m = 0; m < 3; ++m) d[jb][m] = *reinterpret_cast<const f16x8*>(hl + boff[jb][m]);
  };
  auto make_v = [&]() {
    if (half == 0) {
#pragma unroll
      for (int jb = 0; jb < 2; ++jb) {
        v[0][jb] = wx_sub(d[jb][0], d[jb][2]);
        v[1][jb] = wx_add(d[jb][1], d[jb][2]);
      }
    } else {
#pragma unroll
      for (int jb = 0; jb < 2; ++jb) {
        v[0][jb] = wx_sub(d[jb][1], d[jb][0]);
        v[1][jb] = wx_sub(d[jb][0], d[jb][2]);
      }
    }
  };

  // Schedule (the 8-phase kernel's ping-pong, igemm.hip): every K-step (cb, ky) is two R/M section pairs, one per
  // 64-channel half of the U slab; R = that half-slab's 8 A fragments, V / input work, this wave's DMAs, counted
  // vmcnt, barrier; M = 16 MFMAs, barrier.  Waves 4-7 run one barrier behind, so on every SIMD one wave's MFMAs
  // overlap the other's R.   R_0(s): V_s from d(s), A(o 0..63);  R_1(s): A(o 64..127), d(s+1) read.
  // Half-slab ring of 6 (one block's 6): R section r issues half-slab r + 5 (slot (r+5) % 6, last read at section
  // r-1 by both halves: WAR clear after the barrier that ends r-1 for waves 4-7).  Halo DMAs, one per wave per
  // section: block cb+2's pieces 0, 1 at block section 4, 5 and block cb+1's piece 2 at section 0 (buffer cb & 1 is
  // last read by the d(3cb+2) prefetch at section 3).  A wave's DMAs of section r are complete by the end of its
  // section r+3; a half-slab / halo DMA is first read >= 5 sections after it is issued.  vmcnt at the end of block
  // section j = this wave's DMAs of sections j-2 .. j: 9 8 7 6 7 8.
  issue_hp(0, 0);
  issue_hp(0, 1);
  issue_hp(0, 2);
#pragma unroll
  for (int j = 0; j < 5; ++j) issue_hs(0, j);
  issue_hp(1, 0);
  if constexpr (IC2_WX_SCHED == 2) {
    asm volatile("s_waitcnt vmcnt(5)" ::: "memory");  // halo 0, half-slabs 0-2 landed (3, 4, halo 1 p0 in flight)
  } else {
    issue_hp(1, 1);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");  // halo 0, half-slabs 0-2 landed (3, 4, halo 1 p0-1 in flight)
  }
  __builtin_amdgcn_s_barrier();
  read_d(hal);
  bf16x8 af[2][4];
  auto read_a = [&](const char* wl, int nl) {
#pragma unroll
    for (int i = 0; i < 4; ++i) af[nl][i] = *reinterpret_cast<const bf16x8*>(wl + (nl * 64 + i * 16) * 64);
  };
  if (half == 1) __builtin_amdgcn_s_barrier();  // waves 4-7 run one barrier behind
  __builtin_amdgcn_sched_barrier(0);

  uint64_t st[7] = {0, 0, 0, 0, 0, 0, 0};
  uint64_t t_prev = 0, t_loop = 0;
  auto stamp = [&](int k) {
    if constexpr (IC2_WX_STAMP) {
      const uint64_t t = __builtin_amdgcn_s_memtime();
      st[k] += t - t_prev;
      t_prev = t;
    }
  };
  if constexpr (IC2_WX_STAMP) t_loop = t_prev = __builtin_amdgcn_s_memtime();
  for (int cb = 0; cb < CB; ++cb) {
    const char* hb_cur = hal + (cb & 1) * WX_HALO;
    const char* hb_nxt = hal + ((cb + 1) & 1) * WX_HALO;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const int ky = j >> 1, hx = j & 1;
      const char* wl = wsl + j * (WX_SLAB / 2) + aoff;
      // ---- R section
      auto r_dma = [&]() {
        if (!(IC2_WX_ABL & 1) || cb == 0) issue_hs(cb + (j + 5) / 6, (j + 5) % 6);
        if constexpr (IC2_WX_SCHED == 2) {
          if (j == 0) issue_hp(cb + 1, 1);
          if (j == 1) issue_hp(cb + 1, 2);
          if (j == 5) issue_hp(cb + 2, 0);
        } else {
          if (j == 0) issue_hp(cb + 1, 2);
          if (j >= 4) issue_hp(cb + 2, j - 4);
        }
      };
      if constexpr (IC2_WX_PRIO == 2) __builtin_amdgcn_s_setprio(1);
      if constexpr (IC2_WX_SCHED >= 1) r_dma();
      if (hx == 0) make_v();
      read_a(wl, 0);
      read_a(wl, 1);
      if (hx == 1 && IC2_WX_SCHED < 2) {
        if constexpr (!(IC2_WX_ABL & 4)) read_d(ky < 2 ? hb_cur + (ky + 1) * ky_step : hb_nxt);
      }
      if constexpr (IC2_WX_STAMP) {
        __builtin_amdgcn_sched_barrier(0);
        stamp(0);
      }
      if constexpr (IC2_WX_SCHED == 0) r_dma();
      __builtin_amdgcn_sched_barrier(0);
      stamp(1);
      if constexpr (!(IC2_WX_ABL & 16)) {
        if constexpr (IC2_WX_SCHED == 2) {  // halo DMAs at sections 5, 0, 1: 8 9 8 7 6 7
          if (j == 1) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
          if (j == 0 || j == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
          if (j == 3 || j == 5) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
          if (j == 4) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        } else {
          if (j == 0) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
          if (j == 1 || j == 5) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
          if (j == 2 || j == 4) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
          if (j == 3) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        }
      }
      stamp(2);
      if constexpr (!(IC2_WX_ABL & 2)) __builtin_amdgcn_s_barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      stamp(3);
      // ---- M section
      if constexpr (IC2_WX_PRIO == 0) __builtin_amdgcn_s_setprio(1);
      if constexpr (IC2_WX_PRIO == 2) __builtin_amdgcn_s_setprio(0);
#pragma unroll
      for (int nl = 0; nl < 2; ++nl) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int jb = 0; jb < 2; ++jb) {
            if constexpr (IC2_WX_ABL & 8) asm volatile("" ::"v"(af[nl][i]), "v"(v[nl][jb]));
            else
              acc[nl][4 * hx + i][jb] =
                  mfma32<true>(af[nl][i], __builtin_bit_cast(bf16x8, v[nl][jb]), acc[nl][4 * hx + i][jb]);
          }
        if (IC2_WX_SCHED == 2 && hx == 1 && nl == 0) {  // the next step's input fragments behind the MFMAs
          __builtin_amdgcn_sched_barrier(0);
          if constexpr (!(IC2_WX_ABL & 4)) read_d(ky < 2 ? hb_cur + (ky + 1) * ky_step : hb_nxt);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      if constexpr (IC2_WX_PRIO == 0) __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (IC2_WX_STAMP) {  // the MFMAs issued (the last one still in the pipe)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
      stamp(4);
      if constexpr (!(IC2_WX_ABL & 2)) __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      stamp(5);
    }
  }
  if constexpr (IC2_WX_STAMP) {
    st[6] = __builtin_amdgcn_s_memtime() - t_loop;
    if (lane == 0) {
      uint64_t* o = reinterpret_cast<uint64_t*>(a.ws) + ((int64_t)blockIdx.x * 8 + wid) * 8;
#pragma unroll
      for (int k = 0; k < 7; ++k) o[k] = st[k];
    }
  }
  if (half == 0) __builtin_amdgcn_s_barrier();  // balance the waves 4-7 offset barrier
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the tail (zero-size) DMAs
  __syncthreads();  // every wave is past its last LDS read: the exchange below reuses the ring

  // output transform y(2t) = m0 + m1 + m2, y(2t+1) = m1 - m2 - m3 across the halves, through LDS: waves 0-3 keep
  // channel blocks 0..3 and hand over (m0 + m1, m1) of blocks 4..7; waves 4-7 keep 4..7 and hand over (m2, m2 + m3)
  // of 0..3.  [pg][giver half][block][pair block][element] float2 per lane (128 KiB).
  float2* ex = reinterpret_cast<float2*>(lds);
  auto exi = [&](int giver, int i, int jb, int e) { return ((((pg * 2 + giver) * 4 + i) * 2 + jb) * 4 + e) * 64 + lane; };
  // (compile-time register indices on both sides of the wave-uniform branch: a half-dependent index would demote acc
  // to scratch)
  if (half == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int jb = 0; jb < 2; ++jb)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float p0 = acc[0][4 + i][jb][e], p1 = acc[1][4 + i][jb][e];
          ex[exi(0, i, jb, e)] = make_float2(p0 + p1, p1);
        }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int jb = 0; jb < 2; ++jb)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float p0 = acc[0][i][jb][e], p1 = acc[1][i][jb][e];
          ex[exi(1, i, jb, e)] = make_float2(p0, p0 + p1);
        }
  }
  __syncthreads();
  const int hw = a.ho * a.wo;
  float4 sc[4], bi[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int ob = o0 + (4 * half + i) * 16 + 4 * fh;
    sc[i] = ig_load_oscale(a, nn, ob);
    bi[i] = ig_load_bias(a, ob);
  }
  ig_preloads_done();
#pragma unroll
  for (int jb = 0; jb < 2; ++jb) {
    const int b = pg * 2 + jb;
    const int r = b / ns, t = (b % ns) * 16 + fr;
    if (r >= a.wx_th || t >= twp) continue;
    const int oy = oy0 + r, ox = 2 * (px0 + t);
    if (oy >= a.ho || ox >= a.wo) continue;
    const int pix = oy * a.wo + ox;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ob = o0 + (4 * half + i) * 16 + 4 * fh;
      if (ob >= a.cout_p) continue;
      float y0[4], y1[4];
      if (half == 0) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float2 q = ex[exi(1, i, jb, e)];
          const float p0 = acc[0][i][jb][e], p1 = acc[1][i][jb][e];
          y0[e] = p0 + p1 + q.x;
          y1[e] = p1 - q.y;
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float2 q = ex[exi(0, i, jb, e)];
          const float p0 = acc[0][4 + i][jb][e], p1 = acc[1][4 + i][jb][e];
          y0[e] = q.x + p0;
          y1[e] = q.y - (p0 + p1);
        }
      }
      ig_store4v(a, nn * hw + pix, nn, pix, ob, y0, sc[i], bi[i]);
      if (ox + 1 < a.wo) ig_store4v(a, nn * hw + pix + 1, nn, pix + 1, ob, y1, sc[i], bi[i]);
    }
  }
}

// U[o][ky][nu][c] = (G g)[nu] for the kernel row g = w[o][c][ky][0..2] (times modulated_conv2d's rsqrt(mean w^2)
// when prenorm), rounded once from f32; zero for padded o / c
__global__ void __launch_bounds__(256) pack_wino_kernel(const float* __restrict__ w, int cout, int cin, int cout_p,
                                                        int cin_p, int prenorm, float gscale,
                                                        _Float16* __restrict__ out) {
  const int o = blockIdx.x;
  __shared__ float red[256];
  float scale = gscale;
  if (o < cout && prenorm) {
    float s = 0.f;
    for (int i = threadIdx.x; i < cin * 9; i += 256) {
      const float v = w[(int64_t)o * cin * 9 + i];
      s += v * v;
    }
    red[threadIdx.x] = s;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
      if (threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
      __syncthreads();
    }
    scale *= rsqrtf(red[0] / (float)(cin * 9));
  }
  for (int e = threadIdx.x; e < 3 * cin_p; e += 256) {
    const int ky = e / cin_p, c = e - ky * cin_p;
    float g0 = 0.f, g1 = 0.f, g2 = 0.f;
    if (o < cout && c < cin) {
      const float* p = w + ((int64_t)o * cin + c) * 9 + ky * 3;
      g0 = p[0] * scale;
      g1 = p[1] * scale;
      g2 = p[2] * scale;
    }
    const float u[4] = {g0, 0.5f * (g0 + g1 + g2), 0.5f * (g0 - g1 + g2), g2};
    _Float16* row = out + ((int64_t)o * 3 + ky) * 4 * cin_p + c;
#pragma unroll
    for (int nu = 0; nu < 4; ++nu) row[nu * cin_p] = (_Float16)__builtin_amdgcn_fmed3f(u[nu], -65504.f, 65504.f);
  }
}

// The tile of one launch: th rows x twp pairs, each row served by ns 16-lane pair blocks (th * ns <= 8 blocks,
// twp <= 16 ns), halo (th + 2) * 2 * (twp + 1) <= WX_HROWS rows; fewest rounds of one workgroup per CU over the chip's
// 256 CUs, then fewest workgroups, then full pair blocks.
struct WxTile {
  int twp, th, ns, hp, nh, tx, ty, to;
  int64_t blocks;
};
static WxTile wx_tile(int n, int ho, int wo, int cout_p) {
  static const int force_twp = knob("IC2_WINO_TWP", 0), force_th = knob("IC2_WINO_TH", 0);
  const int pairs = (wo + 1) / 2;
  WxTile best{};
  int64_t best_rounds = -1;
  for (int ns = 1; ns <= 8; ns *= 2)
    for (int th = 1; th * ns <= 8; ++th) {
      if (force_th && th != force_th) continue;
      for (int twp = 1; twp <= 16 * ns; ++twp) {
        if (force_twp && twp != force_twp) continue;
        const int hp = twp + 1, nh = (th + 2) * 2 * hp;
        if (nh > WX_HROWS) break;
        WxTile t;
        t.twp = twp; t.th = th; t.ns = ns; t.hp = hp; t.nh = nh;
        t.tx = (int)ceil_div(pairs, twp);
        t.ty = (int)ceil_div(ho, th);
        t.to = (int)ceil_div(cout_p, WX_BO);
        t.blocks = (int64_t)n * t.tx * t.ty * t.to;
        const int64_t rounds = ceil_div(t.blocks, 256);
        // ties: the fewest workgroups, then full 16-pair blocks (16 x 8 beat 15 x 8 at equal counts by 0.4-1.3 % on
        // the SG3-T-256 148-px layers, profiles/r5_wino_tile_sweep.txt)
        const bool full = twp % 16 == 0, best_full = best.twp % 16 == 0;
        if (best_rounds < 0 || rounds < best_rounds ||
            (rounds == best_rounds && (t.blocks < best.blocks || (t.blocks == best.blocks && full && !best_full)))) {
          best = t;
          best_rounds = rounds;
        }
      }
    }
  return best;
}

static int wx_chunk_n(int n, int h, int w_, int cin_p) {
  const int64_t per_img = (int64_t)h * w_ * cin_p * 2;
  if ((int64_t)n * per_img < (int64_t)kOob || per_img >= (int64_t)kOob) return n;
  const int64_t c = ((int64_t)kOob - 1) / per_img;
  return (int)ceil_div(n, ceil_div(n, c));
}

static void* g_wx_stamp = nullptr;  // diagnostic stamp buffer (IC2_WX_STAMP builds)
static int64_t g_wx_stamp_bytes = 0;

}  // namespace ic2

using namespace ic2;

extern "C" int ic2_conv_wino_stamps(void* buf, int64_t bytes) {
  IC2_CHECK_ARG(IC2_WX_STAMP, "conv_wino_stamps: not a stamp build (IC2_WX_STAMP)");
  g_wx_stamp = buf;
  g_wx_stamp_bytes = bytes;
  return IC2_OK;
}

extern "C" int ic2_pack_weight_wino(const float* w, int cout, int cin, int cout_p, int cin_p, int prenorm,
                                    float scale, void* u_out, int dtype, void* stream) {
  IC2_CHECK_ARG(w && u_out && cout > 0 && cin > 0 && cout_p >= cout && cin_p >= cin, "pack_weight_wino: bad arguments");
  IC2_CHECK_ARG(dtype == IC2_F16, "pack_weight_wino: only f16 U (dtype %d)", dtype);
  hipLaunchKernelGGL(pack_wino_kernel, dim3(cout_p), dim3(256), 0, as_stream(stream), w, cout, cin, cout_p, cin_p,
                     prenorm, scale, (_Float16*)u_out);
  IC2_CHECK_LAUNCH("pack_weight_wino");
  return IC2_OK;
}

// Where the Winograd kernel beats the direct implicit GEMM (tools/bench_wino.py, f16 at batch 32): the >= 256-wide
// convs on >= 50-pixel outputs (SG3-T-256 L4-L10: 1.10-1.18x); the 38-pixel L0-L3 (tiles pad the 19-pair rows) and
// the <= 192-wide L11-L13 (hg4) stay direct.  IC2_WINO=0 / 2 (dev knob): never / wherever legal.
extern "C" int ic2_conv_wino_preferred(int dtype, int n, int h, int w_, int cin_p, int cout_p, int kh, int kw,
                                       int pad) {
  static const int mode = knob("IC2_WINO", 1);
  const int ho = h + 2 * pad - kh + 1, wo = w_ + 2 * pad - kw + 1;
  const bool legal = dtype == IC2_F16 && kh == 3 && kw == 3 && n > 0 && ho > 0 && wo > 0 && cin_p % 32 == 0 &&
                     cout_p % 32 == 0 && (int64_t)cout_p * 12 * cin_p * 2 < (int64_t)kOob;
  if (!legal || mode == 0) return 0;
  if (mode == 2) return 1;
  return cin_p >= 256 && cout_p >= 256 && ho >= 50 && wo >= 50;
}

extern "C" const char* ic2_conv_wino_plan(int n, int h, int w_, int cin_p, int cout_p, int pad) {
  const int ho = h + 2 * pad - 2, wo = w_ + 2 * pad - 2;
  if (n <= 0 || ho <= 0 || wo <= 0 || cin_p <= 0 || cin_p % 32 || cout_p <= 0 || cout_p % 32) return "invalid";
  const WxTile t = wx_tile(wx_chunk_n(n, h, w_, cin_p), ho, wo, cout_p);
  static thread_local char buf[64];
  snprintf(buf, sizeof(buf), "wino_fx_o128_p%dx%d_f16", t.twp, t.th);
  return buf;
}

extern "C" int ic2_conv_wino(const void* x, const void* u, void* y, int dtype, int out_dtype, int n, int h, int w_,
                             int cin_p, int cout_p, int cout_valid, int pad, int ho, int wo, const float* oscale,
                             const float* bias, int act, float slope, float act_gain, float clamp, float out_mul,
                             int out_layout, void* stream) {
  IC2_CHECK_ARG(x && u && y, "conv_wino: null pointer");
  IC2_CHECK_ARG(dtype == IC2_F16, "conv_wino: f16 operands only (dtype %d)", dtype);
  IC2_CHECK_ARG(out_dtype == IC2_F32 || out_dtype == IC2_BF16 ||
                    ((out_dtype == IC2_F16 || out_dtype == IC2_F16_IEEE) && out_layout != IC2_LAYOUT_NCHW),
                "conv_wino: bad out dtype %d", out_dtype);
  IC2_CHECK_ARG(cin_p > 0 && cin_p % 32 == 0 && cout_p > 0 && cout_p % 32 == 0,
                "conv_wino: channel strides must be positive multiples of 32 (cin_p=%d cout_p=%d)", cin_p, cout_p);
  IC2_CHECK_ARG(n > 0 && h > 0 && w_ > 0 && pad >= 0, "conv_wino: bad geometry");
  IC2_CHECK_ARG(ho == h + 2 * pad - 2 && wo == w_ + 2 * pad - 2 && ho > 0 && wo > 0,
                "conv_wino: output size %dx%d does not match input %dx%d, k=3x3, pad=%d", ho, wo, h, w_, pad);
  IC2_CHECK_ARG(out_layout == IC2_LAYOUT_NHWC || out_layout == IC2_LAYOUT_NHWC16 ||
                    (out_layout == IC2_LAYOUT_NCHW && out_dtype == IC2_F32 && cout_valid > 0 && cout_valid <= cout_p),
                "conv_wino: NCHW output needs f32 and 0 < cout_valid <= cout_p (layout %d)", out_layout);
  IC2_CHECK_ARG(((uintptr_t)oscale | (uintptr_t)bias) % 16 == 0, "conv_wino: oscale/bias must be 16-byte aligned");
  IC2_CHECK_ARG((int64_t)cout_p * 12 * cin_p * 2 < (int64_t)kOob, "conv_wino: weights too large");
  const int nc = wx_chunk_n(n, h, w_, cin_p);
  if (nc < n) {
    const int64_t x_img = (int64_t)h * w_ * cin_p * 2;
    const int64_t y_img = out_layout == IC2_LAYOUT_NCHW ? (int64_t)cout_valid * ho * wo * 4
                                                        : (int64_t)ho * wo * cout_p * (out_dtype == IC2_F32 ? 4 : 2);
    for (int n0 = 0; n0 < n; n0 += nc) {
      const int nn = n - n0 < nc ? n - n0 : nc;
      const int rc = ic2_conv_wino(reinterpret_cast<const char*>(x) + n0 * x_img, u,
                                   reinterpret_cast<char*>(y) + n0 * y_img, dtype, out_dtype, nn, h, w_, cin_p, cout_p,
                                   cout_valid, pad, ho, wo, oscale ? oscale + (int64_t)n0 * cout_p : nullptr, bias, act,
                                   slope, act_gain, clamp, out_mul, out_layout, stream);
      if (rc != IC2_OK) return rc;
    }
    return IC2_OK;
  }
  const WxTile t = wx_tile(n, ho, wo, cout_p);
  IC2_CHECK_ARG(t.blocks > 0 && t.blocks < (1LL << 31), "conv_wino: bad tile plan");
  const int out_ieee = out_dtype == IC2_F16_IEEE;
  if (out_ieee) out_dtype = IC2_F16;
  IgemmArgs a{};
  a.x = x; a.w = u; a.y = y; a.oscale = oscale; a.bias = bias;
  a.ws = IC2_WX_STAMP && (int64_t)t.blocks * 8 * 8 * 8 <= g_wx_stamp_bytes ? reinterpret_cast<float*>(g_wx_stamp)
                                                                          : nullptr;
  IC2_CHECK_ARG(!IC2_WX_STAMP || a.ws, "conv_wino: stamp build without a large enough ic2_conv_wino_stamps buffer");
  a.n = n; a.h = h; a.w_ = w_; a.cin_p = cin_p; a.cout_p = cout_p; a.cout_valid = cout_valid;
  a.kh = 3; a.kw = 3; a.pad = pad; a.ho = ho; a.wo = wo;
  a.M = n * ho * wo; a.K = 9 * cin_p; a.nq = 3 * (cin_p / 32);
  // o-tiles per L2 group (1: each XCD streams one o-tile's U, 1.5 MiB at 512 channels; the input halos are read by
  // tiles_o XCDs instead of one)
  static const int og_knob = knob("IC2_WINO_OGROUP", 1);
  int og = og_knob < 1 ? 1 : og_knob > t.to ? t.to : og_knob;
  while (t.to % og) --og;
  a.tiles_o = t.to; a.nblocks = (int)t.blocks; a.group = og; a.korder = 1; a.o_base = 0;
  a.act = act; a.slope = slope; a.act_gain = act_gain; a.clamp = clamp; a.out_mul = out_mul;
  a.out_layout = out_layout; a.out_dtype = out_dtype; a.out_ieee = out_ieee;
  a.gn_part = nullptr; a.gn_groups = 0; a.gn_c = 0; a.in_gn = nullptr; a.in_slope = 0.f;
  a.x_pix = cin_p; a.x_hb32 = 0;
  a.wx_twp = t.twp; a.wx_th = t.th; a.wx_ns = t.ns; a.wx_hp = t.hp; a.wx_nh = t.nh; a.wx_tx = t.tx; a.wx_ty = t.ty;
  hipLaunchKernelGGL(wino_fx_f16_kernel, dim3((unsigned)t.blocks), dim3(64 * WX_NW), 0, as_stream(stream), a);
  IC2_CHECK_LAUNCH("conv_wino");
  return IC2_OK;
}
