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
// Launches that would not fill the chip (the encoder's 16^2 .. 2^2 blocks) split K over gridDim.y:
// each slice stores f32 partial sums in a caller-owned workspace and igemm_splitk_reduce_kernel
// combines them in slice order (deterministic) through the same epilogue.
#include "conv_common.h"

#include <cstdlib>

namespace ic2 {

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

// Epilogue shared by the kernels: lane holds C[o = obase + 16i + 4*fh + r][p = pbase + 16j + fr].
// A split-K slice (gridDim.y > 1) stores its raw partial sums instead.
template <int I, int J>
__device__ __forceinline__ void ig_epilogue(const IgemmArgs& a, const f32x4 (&acc)[I][J], int obase, int pbase, int fr,
                                            int fh) {
  const int hw = a.ho * a.wo;
  if (gridDim.y > 1) {  // split-K slice: raw partial sums
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int p = pbase + j * 16 + fr;
      if (p >= a.M) continue;
#pragma unroll
      for (int i = 0; i < I; ++i) {
        const int ob = obase + i * 16 + 4 * fh;
        if (ob < a.cout_p) *reinterpret_cast<f32x4*>(a.ws + ((int64_t)blockIdx.y * a.M + p) * a.cout_p + ob) = acc[i][j];
      }
    }
    return;
  }
  // bias for every channel block, then per 16-pixel column the oscale rows of its samples (a wave's pixels may
  // span two samples), loaded before that column's stores
  float4 bi[I];
#pragma unroll
  for (int i = 0; i < I; ++i) bi[i] = ig_load_bias(a, obase + i * 16 + 4 * fh);
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int p = pbase + j * 16 + fr;
    const int pc = p < a.M ? p : a.M - 1;
    const int nn = pc / hw;
    const int pix = pc - nn * hw;
    float4 sc[I];
#pragma unroll
    for (int i = 0; i < I; ++i) sc[i] = ig_load_oscale(a, nn, obase + i * 16 + 4 * fh);
    ig_preloads_done();
    if (p >= a.M) continue;
#pragma unroll
    for (int i = 0; i < I; ++i) {
      const int ob = obase + i * 16 + 4 * fh;
      if (ob >= a.cout_p) continue;
      const float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      ig_store4v(a, p, nn, pix, ob, v, sc[i], bi[i]);
    }
  }
}

// logical tile -> (o_tile, p_tile), bijective: runs of `group` consecutive p-tiles sweep one o-tile at a
// time, so the blocks resident on one XCD at once share a single weight panel in its L2 (all o-tiles of
// a p-tile side by side would keep tiles_o panels live).  The last run may be shorter.
__device__ __forceinline__ void tile_coords(int logical, int tiles_o, int tiles_p, int group, int& o_tile,
                                            int& p_tile) {
  const int per = group * tiles_o;
  const int gi = logical / per;
  const int rem = logical - gi * per;
  const int gsz = min(group, tiles_p - gi * group);
  o_tile = rem / gsz;
  p_tile = gi * group + (rem - o_tile * gsz);
}

template <bool BF16, int BO, int BP, int WGO, int WGP, int NSTAGE, bool F16 = false>
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

  const int logical = xcd_remap(blockIdx.x, a.nblocks);
  int o_tile, p_tile;
  tile_coords(logical, a.tiles_o, a.nblocks / a.tiles_o, a.group, o_tile, p_tile);
  const int o0 = o_tile * BO;
  const int m0 = p_tile * BP;

  const char* __restrict__ xg = reinterpret_cast<const char*>(a.x);
  const char* __restrict__ wg = reinterpret_cast<const char*>(a.w);

  // ---- per-lane DMA slots.  Instruction g of an operand fills LDS bytes [g KiB, g+1 KiB): lane l
  // lands on row g*(1024/ROWB) + l/(ROWB/16), physical slot l%(ROWB/16) = logical chunk slot^swz(row).
  // Waves beyond an operand's instruction count repeat its last instruction (identical bytes).
  // X: per-lane base pointer at tap (0,0) of the lane's pixel; a chunk adds a uniform byte offset.
  const char* x_base[NIX];
  int x_oy[NIX], x_ox[NIX], x_seg[NIX];
  const char* w_base[NIW];
  int w_seg[NIW];
  const int hw = a.ho * a.wo;
#pragma unroll
  for (int k = 0; k < NIX; ++k) {
    const int g = min(wid_u + C::NW * k, C::NIX_T - 1);
    x_seg[k] = g * 1024;
    const int off = g * 1024 + lane * 16;
    const int row = off / C::ROWB;
    const int ch = ((off % C::ROWB) >> 4) ^ C::swz(row);
    const int m = m0 + row;
    const bool ok = m < a.M;
    const int mm = ok ? m : 0;
    const int nn = mm / hw;
    const int rem = mm - nn * hw;
    const int oy = rem / a.wo;
    const int ox = rem - oy * a.wo;
    // rows past M get an out-of-range y so every tap reads the zero line
    x_oy[k] = ok ? oy - a.pad : -(1 << 20);
    x_ox[k] = ox - a.pad;
    const int64_t e = ((int64_t)(nn * a.h + x_oy[k]) * a.w_ + x_ox[k]) * a.x_pix + ch * EPC;
    x_base[k] = xg + (ok ? e : 0) * ESZ;
  }
#pragma unroll
  for (int k = 0; k < NIW; ++k) {
    const int g = min(wid_u + C::NW * k, C::NIW_T - 1);
    w_seg[k] = g * 1024;
    const int off = g * 1024 + lane * 16;
    const int row = off / C::ROWB;
    const int chl = ((off % C::ROWB) >> 4) ^ C::swz(row);
    const int o = o0 + row;
    w_base[k] = o < a.cout_p ? wg + (int64_t)o * a.K * ESZ + chl * 16 : nullptr;
  }
  const int CB = a.cin_p >> 5;
  // split-K: slice blockIdx.y of gridDim.y covers the K-chunks [q0, q1)
  const int q0 = (int)((int64_t)a.nq * blockIdx.y / gridDim.y);
  const int q1 = (int)((int64_t)a.nq * (blockIdx.y + 1) / gridDim.y);
  // chunk cursor of the next DMA (uniform): chunk index, its tap (ky, kx) and 32-channel block
  int iq = q0, icb = q0 % CB, ikx = (q0 / CB) % a.kw, iky = (q0 / CB) / a.kw;
  const int64_t xrow = (int64_t)a.w_ * a.x_pix * ESZ;

#define IC2_IG_ISSUE(buf_)                                                                                    \
  {                                                                                                          \
    char* wl_ = lds + (buf_) * C::STAGEB;                                                                    \
    char* xl_ = wl_ + C::WB;                                                                                 \
    const int64_t wq = (int64_t)iq * 32 * ESZ;                                                               \
    const int64_t xq = iky * xrow + ((int64_t)ikx * a.x_pix + ig_xb32(a, icb) * 32) * ESZ;                    \
    _Pragma("unroll") for (int k = 0; k < NIW; ++k) {                                                        \
      const void* ws = w_base[k] ? (const void*)(w_base[k] + wq) : zero_line();                              \
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)ws,                     \
                                       (__attribute__((address_space(3))) void*)(wl_ + w_seg[k]), 16, 0, 0); \
    }                                                                                                        \
    _Pragma("unroll") for (int k = 0; k < NIX; ++k) {                                                        \
      const bool ok = (unsigned)(x_oy[k] + iky) < (unsigned)a.h && (unsigned)(x_ox[k] + ikx) < (unsigned)a.w_; \
      const void* xs = ok ? (const void*)(x_base[k] + xq) : zero_line();                                     \
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)xs,                     \
                                       (__attribute__((address_space(3))) void*)(xl_ + x_seg[k]), 16, 0, 0); \
    }                                                                                                        \
    { /* advance (branch-free); past the slice end the last chunk is re-issued (never consumed) */         \
      const int adv = iq + 1 < q1;                                                                           \
      iq += adv;                                                                                             \
      icb += adv;                                                                                            \
      const int wrap = icb == CB;                                                                            \
      icb = wrap ? 0 : icb;                                                                                  \
      ikx += wrap;                                                                                           \
      const int wrap2 = ikx == a.kw;                                                                         \
      ikx = wrap2 ? 0 : ikx;                                                                                 \
      iky += wrap2;                                                                                          \
    }                                                                                                        \
  }

  f32x4 acc[I][J];
#pragma unroll
  for (int i = 0; i < I; ++i)
#pragma unroll
    for (int j = 0; j < J; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s_ = 0; s_ < NSTAGE - 1; ++s_) IC2_IG_ISSUE(s_);

  const int fr = lane & 15;
  const int fh = lane >> 4;

  for (int q = 0; q < q1 - q0; ++q) {
    const int cur = q % NSTAGE;
    if constexpr (NSTAGE == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NSTAGE - 2) * C::PER) : "memory");
    __builtin_amdgcn_s_barrier();  // chunk q landed for every wave; chunk q-1 fully read
    __builtin_amdgcn_sched_barrier(0);
    const char* wl = lds + cur * C::STAGEB;
    const char* xl = wl + C::WB;
    if constexpr (BF16) {
      // all fragment reads first (B, then A in use order), then the refill of the slot chunk q-1 used
      // (its address math runs under the read latency), then the MFMAs: group i waits only for its
      // own A fragment (counted lgkmcnt), the later reads stay in flight
      bf16x8 bfr[J], af[I];
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const int row = wp_ * C::TP + j * 16 + fr;
        bfr[j] = *reinterpret_cast<const bf16x8*>(xl + C::off(row, fh));
      }
#pragma unroll
      for (int i = 0; i < I; ++i) af[i] = *reinterpret_cast<const bf16x8*>(wl + C::off(wo_ * C::TO + i * 16 + fr, fh));
      __builtin_amdgcn_sched_barrier(0);
      IC2_IG_ISSUE((q + NSTAGE - 1) % NSTAGE);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < I; ++i)
#pragma unroll
        for (int j = 0; j < J; ++j)
          acc[i][j] = mfma32<F16>(af[i], bfr[j], acc[i][j]);
    } else {
      IC2_IG_ISSUE((q + NSTAGE - 1) % NSTAGE);
      __builtin_amdgcn_sched_barrier(0);
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

  ig_epilogue<I, J>(a, acc, o0 + wo_ * C::TO, m0 + wp_ * C::TP, fr, fh);
}

// split-K combine: sum the slices in slice order (deterministic), then the epilogue; one thread per
// (pixel, 4 channels)
__global__ void __launch_bounds__(256) igemm_splitk_reduce_kernel(IgemmArgs a, int splits, int p_lo) {
  const int c4 = a.cout_p >> 2;
  const int total = (a.M - p_lo) * c4;  // < 2^31 (checked by the launcher); pixels [p_lo, M) (the split tail)
  const int hw = a.ho * a.wo;
  const int64_t slice = (int64_t)a.M * a.cout_p;
  for (int e = blockIdx.x * 256 + threadIdx.x; e < total; e += gridDim.x * 256) {
    const int q = e / c4;
    const int p = p_lo + q;
    const int ob = (e - q * c4) * 4;
    const float* src = a.ws + (int64_t)p * a.cout_p + ob;
    f32x4 s = *reinterpret_cast<const f32x4*>(src);
    for (int k = 1; k < splits; ++k) s += *reinterpret_cast<const f32x4*>(src + k * slice);
    const int nn = p / hw;
    const float v[4] = {s[0], s[1], s[2], s[3]};
    ig_store4(a, p, nn, p - nn * hw, ob, v);
  }
}

// ------------------------------------------------------------------------------------------------
// 8-phase kernels, 64-deep K-tiles (64 channels of one tap), 8 waves each owning 128 x 64 outputs:
//   OG = 2: 256 x 256 tile, 2 o-groups x 4 p-groups;
//   OG = 1: 128 x 512 tile (the cout_p <= 128 layers), 1 o-group x 8 p-groups.
// Eight phases per iteration (two K-tiles, LDS double buffer): phase = (ds_read the quadrant's
// fragments, DMA one half-tile, [counted vmcnt], s_barrier, 16 MFMAs at raised priority, s_barrier).
// Waves 4-7 run one barrier behind waves 0-3, so on every SIMD (one wave of each half) one wave's
// MFMAs overlap the other's LDS reads and DMA issue.
//   quadrant per phase&3 : (qm,qn) = (0,0) (0,1) (1,1) (1,0); reads A(qm)+B(qn), B(1), A(1), B(0)
//   half-tile restaged   : ph0 buf1.A1<-t+1  ph1 buf1.B0<-t+1  ph2..5 buf0.{A0,B1,A1,B0}<-t+2
//                          ph6 buf1.A0<-t+3  ph7 buf1.B1<-t+3      (t = 2*iteration)
// Every half is restaged >= 2 phases after its last read (WAR) and read >= 1 phase after the
// vmcnt + barrier that retires it (RAW: the waits in phases 3 and 7 leave only the two newest halves,
// NA + NB DMA instructions, in flight).  Half-tile qm of A = the rows {128*og + 64*qm + [0, 64)};
// half-tile qn of B = the rows {64*pg + 32*qn + [0, 32)}: NA = OG and NB = 4 / OG 1-KiB DMA
// instructions per wave.  LDS rows are 128 B, 16-B chunk c stored at c ^ ((row >> 1) & 7)
// (conflict-free ds_read_b128 for the fragment lane groups).  64-row quadrants lying wholly in the
// o-padding (cout_p 64 / 192 / 384) skip their MFMAs: their accumulators stay 0, which is what those
// rows hold, and the SIMD's partner wave gets the matrix pipe to itself.
template <int OG>
struct G8 {
  static constexpr int BO = 128 * OG, BP = 512 / OG;
  static constexpr int NA = OG, NB = 4 / OG;                    // DMA instructions per wave per half-tile
  static constexpr int BOFF = BO * 128, BUF = (BO + BP) * 128;  // bytes: B offset in a buffer, one buffer
};
__device__ __forceinline__ int g8_off(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }
__device__ __forceinline__ int g8_arow(int qm, int g, int l) { return (g >> 3) * 128 + qm * 64 + (g & 7) * 8 + l; }
__device__ __forceinline__ int g8_brow(int qn, int g, int l) { return (g >> 2) * 64 + qn * 32 + (g & 3) * 8 + l; }

template <int OG, bool F16 = false>
__device__ __forceinline__ void igemm8_body(const IgemmArgs& a) {
  using G = G8<OG>;
  constexpr int NA = G::NA, NB = G::NB;
  __shared__ __attribute__((aligned(16))) char lds[2 * G::BUF];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid_u = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int half = wid_u >> 2;                     // waves 4-7 run one barrier behind waves 0-3
  const int grp = OG == 2 ? half : 0;              // o-group
  const int wp_ = OG == 2 ? (wid_u & 3) : wid_u;   // p-group (64 pixels)
  // a launch may cover logical tiles [tile_base, tile_base + gridDim.x) of the a.nblocks-tile grid (the split tail)
  const int logical = a.tile_base + xcd_remap(blockIdx.x, gridDim.x);
  int o_tile, p_tile;
  tile_coords(logical, a.tiles_o, a.nblocks / a.tiles_o, a.group, o_tile, p_tile);
  const int o0 = a.o_base + o_tile * G::BO;  // o_base: a launch covering output channels [o_base, ...) only
  const int m0 = p_tile * G::BP;
  const char* __restrict__ xg = reinterpret_cast<const char*>(a.x);
  const char* __restrict__ wg = reinterpret_cast<const char*>(a.w);

  // per-lane DMA sources: [half][instruction]; instruction k of wave w moves row block g = w + 8k.
  // Buffer loads (raw, stride 0): the per-K-tile part of the address is a scalar descriptor base, the
  // per-lane part a constant 32-bit offset; a tap outside the image / a row past M or cout_p gets the
  // offset kOob (>= num_records), which the hardware answers with zeros.  No per-lane 64-bit math.
  uint32_t w_off[2][NA], x_off[2][NB], x_tap[2][NB];
  const int hw = a.ho * a.wo;
  const int lrow = lane >> 3;                    // row within the 8-row block
  const int pch = lane & 7;                      // physical 16-B chunk written by this lane
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int k = 0; k < NA; ++k) {
      const int ar = g8_arow(h, wid_u + 8 * k, lrow);
      const int o = o0 + ar;
      w_off[h][k] = o < a.cout_p ? (uint32_t)(o * a.K * 2 + ((pch ^ ((ar >> 1) & 7)) << 4)) : kOob;
    }
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      const int br = g8_brow(h, wid_u + 8 * k, lrow);
      const int m = m0 + br;
      const bool ok = m < a.M;
      const int mm = ok ? m : 0;
      const int nn = mm / hw;
      const int rem = mm - nn * hw;
      const int oy = rem / a.wo;
      const int ox = rem - oy * a.wo;
      // offset of the output pixel's own (oy, ox) position; the descriptor base carries the tap shift
      x_off[h][k] = (uint32_t)((((nn * a.h + oy) * a.w_ + ox) * a.x_pix + ((pch ^ ((br >> 1) & 7)) << 3)) * 2);
      uint32_t mask = 0;
      for (int ky = 0; ky < a.kh; ++ky)
        for (int kx = 0; kx < a.kw; ++kx) {
          const bool in = ok && (unsigned)(oy - a.pad + ky) < (unsigned)a.h && (unsigned)(ox - a.pad + kx) < (unsigned)a.w_;
          mask |= (uint32_t)in << (ky * a.kw + kx);
        }
      x_tap[h][k] = mask;
    }
  }
  const int CB = a.cin_p >> 6;

  // K-tile cursor (uniform): tile index, tap (ky, kx), 64-channel block
  struct Cur {
    int t, ky, kx, cb;
  };
  // K order.  tap-major (cb innermost: K-tile t is the contiguous weight column t) streams a WG's whole
  // 256-pixel x cin_p panel once per tap, so the 9 shifted re-reads of a pixel are cin_p / 64 K-tiles apart and
  // the ~32 resident WGs of an XCD cycle ~8 MB through its 4 MB L2 between them (PMC: 5.4x the compulsory HBM
  // bytes on s148).  channel-major (taps innermost, the halo kernels' order) re-reads each 64-channel panel at the
  // 9 taps back to back.  IC2_IGEMM_KORDER=0 / 1 selects tap- / channel-major.
  const bool cmaj = a.korder != 0;
  auto advance = [&](Cur c) {
    c.t += 1;
    if (cmaj) {
      c.kx += 1;
      const int wrap = c.kx == a.kw;
      c.kx = wrap ? 0 : c.kx;
      c.ky += wrap;
      const int wrap2 = c.ky == a.kh;
      c.ky = wrap2 ? 0 : c.ky;
      c.cb += wrap2;
    } else {
      c.cb += 1;
      const int wrap = c.cb == CB;
      c.cb = wrap ? 0 : c.cb;
      c.kx += wrap;
      const int wrap2 = c.kx == a.kw;
      c.kx = wrap2 ? 0 : c.kx;
      c.ky += wrap2;
    }
    // the selects above come out as v_cndmask: without this the compiler treats the cursor as divergent and wraps
    // every DMA whose descriptor derives from it in a readfirstlane waterfall loop
    c.t = __builtin_amdgcn_readfirstlane(c.t);
    c.ky = __builtin_amdgcn_readfirstlane(c.ky);
    c.kx = __builtin_amdgcn_readfirstlane(c.kx);
    c.cb = __builtin_amdgcn_readfirstlane(c.cb);
    return c;
  };

#define IC2_G8_ISSUE_A(h_, buf_, c_)                                                                          \
  {                                                                                                          \
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(                                     \
        (void*)(wg + (int64_t)(((c_).ky * a.kw + (c_).kx) * CB + (c_).cb) * 128), 0, (c_).t < t_end ? kOob : 0, \
        kRsrcWord3);                                                                                         \
    _Pragma("unroll") for (int k = 0; k < NA; ++k)                                                           \
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(lds + (buf_) * G::BUF + \
                                                                                       g8_arow(h_, wid_u + 8 * k, 0) * 128), \
                                               16, w_off[h_][k], 0, 0, 0);                                   \
  }
#define IC2_G8_ISSUE_B(h_, buf_, c_)                                                                          \
  {                                                                                                          \
    const int tap = (c_).ky * a.kw + (c_).kx;                                                                \
    const int64_t sh = ((int64_t)((c_).ky - a.pad) * a.w_ + ((c_).kx - a.pad)) * a.x_pix * 2 +                \
                       ig_xb32(a, 2 * (c_).cb) * 64;                                                          \
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)(xg + sh), 0,                  \
                                                                        (c_).t < t_end ? kOob : 0, kRsrcWord3); \
    _Pragma("unroll") for (int k = 0; k < NB; ++k) {                                                         \
      const uint32_t vo = ((x_tap[h_][k] >> tap) & 1u) ? x_off[h_][k] : kOob;                                \
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(lds + (buf_) * G::BUF + \
                                                                                       G::BOFF + g8_brow(h_, wid_u + 8 * k, 0) * 128), \
                                               16, vo, 0, 0, 0);                                             \
    }                                                                                                        \
  }

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15;
  const int fh = lane >> 4;
  bf16x8 af[4][2], bfr[2][2];
  const int orow = o0 + grp * 128;
  const bool live0 = orow < a.cout_p, live1 = orow + 64 < a.cout_p;

  // split-K (gridDim.y slices, small grids): this workgroup's K-tiles [t_begin, t_end); tiles past t_end come in
  // as zeros (descriptor size 0), so the phase loop needs no tail case
  const int per = (a.nq + (int)gridDim.y - 1) / (int)gridDim.y;
  const int t_begin = __builtin_amdgcn_readfirstlane(min(a.nq, (int)blockIdx.y * per));
  const int t_end = __builtin_amdgcn_readfirstlane(min(a.nq, t_begin + per));
  const int ntap = a.kh * a.kw;
  Cur c0;
  c0.t = t_begin;
  {
    const int tap = cmaj ? t_begin % ntap : t_begin / CB;
    c0.cb = __builtin_amdgcn_readfirstlane(cmaj ? t_begin / ntap : t_begin % CB);
    c0.ky = __builtin_amdgcn_readfirstlane(tap / a.kw);
    c0.kx = __builtin_amdgcn_readfirstlane(tap - (tap / a.kw) * a.kw);
  }

  // prologue: tile 0 -> buf0 (all four halves), tile 1 -> buf1.A0 / buf1.B1 (what phases 6-7 would issue)
  Cur c1 = advance(c0);
  IC2_G8_ISSUE_A(0, 0, c0);
  IC2_G8_ISSUE_B(0, 0, c0);
  IC2_G8_ISSUE_A(1, 0, c0);
  IC2_G8_ISSUE_B(1, 0, c0);
  IC2_G8_ISSUE_A(0, 1, c1);
  IC2_G8_ISSUE_B(1, 1, c1);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NA + NB) : "memory");
  __builtin_amdgcn_s_barrier();
  if (half == 1) __builtin_amdgcn_s_barrier();  // waves 4-7 run one barrier behind
  __builtin_amdgcn_sched_barrier(0);

#define IC2_G8_READ_A(buf_, qm_)                                                                              \
  _Pragma("unroll") for (int i = 0; i < 4; ++i) _Pragma("unroll") for (int s = 0; s < 2; ++s) af[i][s] =    \
      *reinterpret_cast<const bf16x8*>(lds + (buf_) * G::BUF + g8_off(grp * 128 + (qm_) * 64 + i * 16 + fr, 4 * s + fh));
#define IC2_G8_READ_B(buf_, qn_)                                                                              \
  _Pragma("unroll") for (int j = 0; j < 2; ++j) _Pragma("unroll") for (int s = 0; s < 2; ++s) bfr[j][s] =   \
      *reinterpret_cast<const bf16x8*>(lds + (buf_) * G::BUF + G::BOFF +                                      \
                                       g8_off(wp_ * 64 + (qn_) * 32 + j * 16 + fr, 4 * s + fh));
#define IC2_G8_COMPUTE(qm_, qn_, WAIT_)                                                                       \
  __builtin_amdgcn_sched_barrier(0);                                                                         \
  WAIT_;                                                                                                     \
  __builtin_amdgcn_s_barrier();                                                                              \
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                                         \
  __builtin_amdgcn_sched_barrier(0);                                                                         \
  __builtin_amdgcn_s_setprio(1);                                                                             \
  if ((qm_) == 0 ? live0 : live1) {                                                                          \
    _Pragma("unroll") for (int i = 0; i < 4; ++i) _Pragma("unroll") for (int j = 0; j < 2; ++j)             \
        _Pragma("unroll") for (int s = 0; s < 2; ++s) acc[(qm_) * 4 + i][(qn_) * 2 + j] =                    \
            mfma32<F16>(af[i][s], bfr[j][s], acc[(qm_) * 4 + i][(qn_) * 2 + j]);                                   \
  }                                                                                                          \
  __builtin_amdgcn_s_setprio(0);                                                                             \
  __builtin_amdgcn_sched_barrier(0);                                                                         \
  __builtin_amdgcn_s_barrier();                                                                              \
  __builtin_amdgcn_sched_barrier(0);
#define IC2_G8_NOWAIT (void)0
#define IC2_G8_WAIT asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NA + NB) : "memory")

  const int niter = (t_end - t_begin + 1) >> 1;
  Cur cn = c1;  // tile 2i+1
  for (int it = 0; it < niter; ++it) {
    const Cur cA = cn;               // 2i+1
    const Cur cB = advance(cA);      // 2i+2
    const Cur cC = advance(cB);      // 2i+3
    // phase 0: buf0 quadrant (0,0); restage buf1.A1 <- 2i+1
    IC2_G8_READ_B(0, 0);
    IC2_G8_READ_A(0, 0);
    IC2_G8_ISSUE_A(1, 1, cA);
    IC2_G8_COMPUTE(0, 0, IC2_G8_NOWAIT);
    // phase 1: (0,1); buf1.B0 <- 2i+1
    IC2_G8_READ_B(0, 1);
    IC2_G8_ISSUE_B(0, 1, cA);
    IC2_G8_COMPUTE(0, 1, IC2_G8_NOWAIT);
    // phase 2: (1,1); buf0.A0 <- 2i+2
    IC2_G8_READ_A(0, 1);
    IC2_G8_ISSUE_A(0, 0, cB);
    IC2_G8_COMPUTE(1, 1, IC2_G8_NOWAIT);
    // phase 3: (1,0); buf0.B1 <- 2i+2; retire tile 2i+1 (buf1) for phases 4-7
    IC2_G8_READ_B(0, 0);
    IC2_G8_ISSUE_B(1, 0, cB);
    IC2_G8_COMPUTE(1, 0, IC2_G8_WAIT);
    // phase 4: buf1 quadrant (0,0); buf0.A1 <- 2i+2
    IC2_G8_READ_B(1, 0);
    IC2_G8_READ_A(1, 0);
    IC2_G8_ISSUE_A(1, 0, cB);
    IC2_G8_COMPUTE(0, 0, IC2_G8_NOWAIT);
    // phase 5: (0,1); buf0.B0 <- 2i+2
    IC2_G8_READ_B(1, 1);
    IC2_G8_ISSUE_B(0, 0, cB);
    IC2_G8_COMPUTE(0, 1, IC2_G8_NOWAIT);
    // phase 6: (1,1); buf1.A0 <- 2i+3
    IC2_G8_READ_A(1, 1);
    IC2_G8_ISSUE_A(0, 1, cC);
    IC2_G8_COMPUTE(1, 1, IC2_G8_NOWAIT);
    // phase 7: (1,0); buf1.B1 <- 2i+3; retire tile 2i+2 (buf0) for the next iteration
    IC2_G8_READ_B(1, 0);
    IC2_G8_ISSUE_B(1, 1, cC);
    IC2_G8_COMPUTE(1, 0, IC2_G8_WAIT);
    cn = cC;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the tail DMAs (zero tiles) before exit
  if (half == 0) __builtin_amdgcn_s_barrier();      // balance the waves 4-7 offset barrier
#undef IC2_G8_ISSUE_A
#undef IC2_G8_ISSUE_B
#undef IC2_G8_READ_A
#undef IC2_G8_READ_B
#undef IC2_G8_COMPUTE
#undef IC2_G8_NOWAIT
#undef IC2_G8_WAIT
  ig_epilogue<8, 4>(a, acc, orow, m0 + wp_ * 64, fr, fh);
}

// one non-template kernel per instance (a __global__ template's host stub is not emitted here)
__global__ void __launch_bounds__(512, 1) igemm8_og2_kernel(IgemmArgs a) { igemm8_body<2>(a); }
__global__ void __launch_bounds__(512, 1) igemm8_og1_kernel(IgemmArgs a) { igemm8_body<1>(a); }
__global__ void __launch_bounds__(512, 1) igemm8_og2_f16_kernel(IgemmArgs a) { igemm8_body<2, true>(a); }
__global__ void __launch_bounds__(512, 1) igemm8_og1_f16_kernel(IgemmArgs a) { igemm8_body<1, true>(a); }

template <bool BF16, int BO, int BP, int WGO, int WGP, int NSTAGE, bool F16 = false>
static void launch_igemm(IgemmArgs a, int splits, hipStream_t s) {
  a.tiles_o = (a.cout_p + BO - 1) / BO;
  a.nblocks = (int)(ceil_div(a.M, BP) * a.tiles_o);
  hipLaunchKernelGGL((igemm_kernel<BF16, BO, BP, WGO, WGP, NSTAGE, F16>), dim3(a.nblocks, splits),
                     dim3(64 * WGO * WGP), 0, s, a);
}

// tiles [tile_base, tile_base + ntiles) of the grid (ntiles < 0: all of it from tile_base)
template <int OG, bool F16 = false>
static void launch_g8(IgemmArgs a, hipStream_t s, int o_base = 0, int o_end = -1, int splits = 1, int tile_base = 0,
                      int ntiles = -1) {
  a.o_base = o_base;
  a.tiles_o = ((o_end < 0 ? a.cout_p : o_end) - o_base + G8<OG>::BO - 1) / G8<OG>::BO;
  a.nq = a.K / 64;
  a.nblocks = (int)(ceil_div(a.M, G8<OG>::BP) * a.tiles_o);
  a.tile_base = tile_base;
  const unsigned grid = (unsigned)(ntiles < 0 ? a.nblocks - tile_base : ntiles);
  if constexpr (OG == 2)
    hipLaunchKernelGGL(F16 ? igemm8_og2_f16_kernel : igemm8_og2_kernel, dim3(grid, splits), dim3(512), 0, s, a);
  else
    hipLaunchKernelGGL(F16 ? igemm8_og1_f16_kernel : igemm8_og1_kernel, dim3(grid, splits), dim3(512), 0, s, a);
}

// ------------------------------------------------------------------------------------------------
// Halo implicit GEMM, 4-wave form (`hg4`).  The implicit GEMM above stages a shifted pixel panel per tap, so every
// input pixel crosses L2 -> LDS nine times per channel block; here the output tile is a 2-D block of pixels of one
// sample whose (TH+2) x (TW+2) input halo is staged ONCE per 32-channel block and read at nine shifted offsets.
// An 8-wave form of the same idea (one workgroup per CU, all waves meeting at each K-step barrier: MFMA busy
// 0.30-0.38, round 2) was removed; here a workgroup is 4 waves (one per SIMD) and needs <= 74 KB of LDS, so two
// independent workgroups share each CU and one's barrier / fragment-read phase overlaps the other's MFMAs.
//   K-step = one tap x 32 channels (64-B LDS rows); wave tile (16 I) o x (16 J) px, 2 fragments per MFMA pair
//   read per step: I + J ds_read_b128 for I*J MFMAs (8 + 4 for 32 at the 128 x 256 tile: 12 KB per wave and
//   step).
//   Weights stream through a 3-slab ring (the slab for step t+2 is issued at step t, so a DMA has a whole step
//   plus the barrier to land); the next 32-channel block's halo is spread over the first taps of the current
//   block, one 1-KiB DMA per wave per step, so every step waits for the same small count (vmcnt(NWI [+1])).
//   LDS rows of 64 B, 16-B chunk c stored at c ^ (((row >> 2) & 1) << 1): conflict-free ds_read_b128 for 16
//   consecutive rows starting at ANY row (the halo fragments start at tap-shifted rows), checked by brute force
//   over the four ds_read_b128 lane groups.
template <int I, int J, int WGO, int WGP, int TW, int NS, bool HB = false>
struct H4 {
  static constexpr int BO = 16 * I * WGO, BP = 16 * J * WGP, TH = BP / TW;
  static constexpr int HW = TW + 2, HH = TH + 2, NH = HH * HW;  // halo pixels
  static constexpr int NHI = (NH + 15) / 16;                    // 1-KiB DMA instructions per halo (16 px)
  static constexpr int HPW = (NHI + 3) / 4;                     // per wave, at most
  static constexpr int HALO_B = NHI * 1024;
  static constexpr int WS_B = BO * 64;                          // one weight slab: BO rows x 32 channels
  static constexpr int NWI = (BO / 16 + 3) / 4;                 // weight DMA instructions per wave
  static constexpr int LDS_B = NS * WS_B + 2 * HALO_B + (HB ? 1024 : 0);  // NS-slab weight ring (+ HB dummy slot)
  static_assert(BP % TW == 0 && TW % 16 == 0, "pixel tile");
  // weight slab rows split over the 4 waves: evenly, or (BO = 96) waves 2-3 issue one DMA fewer, which only the
  // one-step lookahead of the multi-tap loop (L = 1: its waits do not count weight DMAs) allows
  static_assert((BO / 16) % 4 == 0 || BO == 96, "weight slab rows over the 4 waves");
  static_assert(HB || HPW <= 8, "halo DMA spread over the first 8 taps");
  static_assert(LDS_B <= 80 * 1024, "two workgroups per CU");
};
__device__ __forceinline__ int h4_off(int row, int chunk) { return row * 64 + ((chunk ^ (((row >> 2) & 1) << 1)) << 4); }

// diagnostic builds only (tools/build_abl.sh hg4, wrong results): IC2_HG4_ABL bit 0 skips the multi-tap loop's
// per-step DMA waits, bit 1 its barrier, bit 2 its fragment reads after the first step, bit 3 its MFMAs, bit 4 its
// weight DMAs after the first step
#ifndef IC2_HG4_ABL
#define IC2_HG4_ABL 0
#endif
// IC2_HG4_PAIR=0 (diagnostic builds): the split-weight f16 statistics-epilogue kernels in the plain K order
#ifndef IC2_HG4_PAIR
#define IC2_HG4_PAIR 1
#endif

// HB: the next block's halo is issued as one burst at the block's first tap, every wave exactly HPW DMAs (the ones
// past the halo into a 1-KiB dummy slot), so no per-tap selection of a halo-offset register (a uniform branch
// chain, ~60 SALU per step) and a wait count that depends only on the tap
// PAIR (split-weight f16 input, IC2_F16X2, TPB = 2): K blocks cb and cb + CB/2 (x * w_hi, x * w_lo) read the same
// stored channel block, so the steps run tap-major over the pair -- (tap, hi), (tap, lo) share one barrier step and one
// set of halo fragments, and each stored block's halo is loaded once for its 18 steps instead of twice for 9 each
template <int I, int J, int WGO, int WGP, int TW, int NS, bool HB = false, bool F16 = false, int TPB = 1,
          bool GN = false, bool PAIR = false>
__device__ __forceinline__ void hg4_body(const IgemmArgs& a, int tiles_x, int tiles_y) {
  using G = H4<I, J, WGO, WGP, TW, NS, HB>;
  static_assert(!PAIR || (TPB == 2 && HB), "PAIR: two taps per barrier step with the halo burst");
  static_assert((G::BO / 16) % 4 == 0 || (TPB == 2 && NS == 4), "uneven weight DMAs need the L = 1 multi-tap loop");
  constexpr int LA = NS - 1;  // weight slabs in flight ahead of the step being computed
  constexpr int NWI = G::NWI, HPW = G::HPW;
  __shared__ __attribute__((aligned(16))) char lds[G::LDS_B];
  char* const wsl = lds;                    // NS weight slabs
  char* const hal = lds + NS * G::WS_B;     // 2 halos
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int og = wid / WGP, pg = wid % WGP;
  const int fr = lane & 15, fh = lane >> 4;

  const int logical = xcd_remap(blockIdx.x, a.nblocks);
  const int o_tile = logical % a.tiles_o;
  int pt = logical / a.tiles_o;
  const int tx = pt % tiles_x;
  pt /= tiles_x;
  const int ty = pt % tiles_y;
  const int nn = pt / tiles_y;
  const int o0 = o_tile * G::BO;
  const int oy0 = ty * G::TH, ox0 = tx * TW;

  const char* __restrict__ xg = reinterpret_cast<const char*>(a.x);
  const char* __restrict__ wg = reinterpret_cast<const char*>(a.w);
  const int lrow = lane >> 2, pch = lane & 3;  // DMA: 16 rows x 4 chunks of 16 B per instruction

  uint32_t w_off[NWI];
#pragma unroll
  for (int k = 0; k < NWI; ++k) {
    const int row = (wid + 4 * k) * 16 + lrow;
    const int o = o0 + row;
    w_off[k] = (row < G::BO && o < a.cout_p) ? (uint32_t)(o * a.K * 2 + ((pch ^ (((row >> 2) & 1) << 1)) << 4)) : kOob;
  }
  uint32_t h_off[HPW];
#pragma unroll
  for (int k = 0; k < HPW; ++k) {
    const int g = wid + 4 * k;
    const int hp = g * 16 + lrow;
    const int hy = hp / G::HW, hx = hp - (hp / G::HW) * G::HW;
    const int iy = oy0 - a.pad + hy, ix = ox0 - a.pad + hx;
    const bool ok = g < G::NHI && hp < G::NH && (unsigned)iy < (unsigned)a.h && (unsigned)ix < (unsigned)a.w_;
    h_off[k] = ok ? (uint32_t)((((nn * a.h + iy) * a.w_ + ix) * a.x_pix + ((pch ^ (((hp >> 2) & 1) << 1)) << 3)) * 2)
                  : kOob;
  }
  int brow[J];
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int pb = pg * J + j;
    brow[j] = (pb * 16 / TW) * G::HW + (pb * 16) % TW + fr;
  }
  const int obase = og * 16 * I;
  const bool live = o0 + obase < a.cout_p;
  const int CB = a.cin_p >> 5;
  const int nq = CB * 9;
  constexpr int SPB = PAIR ? 18 : 9;    // K-steps per halo block
  const int HBK = PAIR ? CB >> 1 : CB;  // halo blocks
  // K-step t -> (halo block, K block, tap)
  auto step_of = [&](int t, int& hbk, int& cb, int& tap) {
    if constexpr (PAIR) {
      hbk = t / 18;
      const int r = t - hbk * 18;
      tap = r >> 1;
      cb = hbk + (r & 1) * (CB >> 1);
    } else {
      cb = t / 9;
      tap = t - cb * 9;
      hbk = cb;
    }
  };

  auto issue_w = [&](int t) {  // weight slab of K-step t -> slab t % NS
    int hbk_, cb, tap;
    step_of(t, hbk_, cb, tap);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(wg + ((int64_t)tap * a.cin_p + cb * 32) * 2), 0, t < nq ? kOob : 0, kRsrcWord3);
    char* dst = wsl + (t % NS) * G::WS_B;
#pragma unroll
    for (int k = 0; k < NWI; ++k)
      if ((G::BO / 16) % 4 == 0 || wid + 4 * k < G::BO / 16)  // uneven split (BO 96): wave-uniform skip
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rs, (__attribute__((address_space(3))) void*)(dst + (wid + 4 * k) * 1024), 16, w_off[k], 0, 0, 0);
  };
  auto issue_hb = [&](int cb) {  // HB: all HPW DMAs of this wave for the halo of block cb -> halo cb & 1 (or dummy)
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(xg + (int64_t)ig_xb32(a, cb) * 64), 0, kOob, kRsrcWord3);
#pragma unroll
    for (int k = 0; k < HPW; ++k) {
      char* dst = wid + 4 * k < G::NHI ? hal + (cb & 1) * G::HALO_B + (wid + 4 * k) * 1024 : hal + 2 * G::HALO_B;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)dst, 16, h_off[k], 0, 0, 0);
    }
  };
  auto issue_h1 = [&](int cb, int k) {  // DMA k of this wave for the halo of block cb -> halo cb & 1
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(xg + (int64_t)ig_xb32(a, cb) * 64), 0, kOob, kRsrcWord3);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        rs, (__attribute__((address_space(3))) void*)(hal + (cb & 1) * G::HALO_B + (wid + 4 * k) * 1024), 16, h_off[k],
        0, 0, 0);
  };

  f32x4 acc[I][J];
#pragma unroll
  for (int i = 0; i < I; ++i)
#pragma unroll
    for (int j = 0; j < J; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int k = 0; k < HPW; ++k)
    if (wid + 4 * k < G::NHI) issue_h1(0, k);
  if constexpr (TPB > 1) {
    // TPB taps per barrier: step s computes taps TPB*s .. TPB*s+TPB-1 (with TPB = 2 a pair may straddle two channel
    // blocks; both halos are resident).  Slabs of step s+L are issued at step s into the ring positions step s-1
    // read, so the ring holds L+1 steps; the DMA lookahead in MFMA cycles is TPB*L taps (the one-tap ring: LA-1).
    static_assert(HB && NS % TPB == 0 && NS >= 2 * TPB && (TPB == 2 || TPB == 3), "TPB: halo burst, ring of steps");
    constexpr int L = NS / TPB - 1;
    const int nst = (nq + TPB - 1) / TPB;
    auto burst_at = [&](int st) {  // block cb0+1's halo: first step with no tap of block cb0-1
      const int t0 = TPB * st, cb0 = t0 / SPB;
      return t0 - cb0 * SPB < TPB && cb0 + 1 < HBK;
    };
#pragma unroll
    for (int t = 0; t < TPB * L; ++t) issue_w(t);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((L - 1) * TPB * NWI) : "memory");  // halo 0 and step 0's slabs landed
    bf16x8 af[TPB][I], bfr[TPB][J];
    for (int s = 0; s < nst; ++s) {
      if constexpr (!(IC2_HG4_ABL & 2)) __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      const int t0 = TPB * s;
      if (!(IC2_HG4_ABL & 16) || s == 0) {
#pragma unroll
        for (int u = 0; u < TPB; ++u) issue_w(t0 + u + TPB * L);
      }
      const bool burst = burst_at(s);  // first read >= 3 steps later
      if (burst) issue_hb(t0 / SPB + 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < TPB; ++u) {
        if ((IC2_HG4_ABL & 4) && s > 0) break;
        const int t = t0 + u;
        int hbk, cb, tap;
        step_of(t, hbk, cb, tap);
        // the swizzle depends on the absolute halo row: the tap shift goes into the row, not the base pointer
        const int sh = (tap / 3) * G::HW + tap % 3;
        const char* hb = hal + (hbk & 1) * G::HALO_B;
        const char* wl = wsl + (t % NS) * G::WS_B;
        if (!PAIR || u == 0) {  // PAIR: the step's second K block reads the same halo fragments
#pragma unroll
          for (int j = 0; j < J; ++j) bfr[u][j] = *reinterpret_cast<const bf16x8*>(hb + h4_off(brow[j] + sh, fh));
        }
#pragma unroll
        for (int i = 0; i < I; ++i) af[u][i] = *reinterpret_cast<const bf16x8*>(wl + h4_off(obase + i * 16 + fr, fh));
      }
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
      if (live) {
#pragma unroll
        for (int u = 0; u < TPB; ++u) {
          if (u == 0 || t0 + u < nq) {  // the tail step of an odd tap count has one tap
#pragma unroll
            for (int i = 0; i < I; ++i)
#pragma unroll
              for (int j = 0; j < J; ++j) {
                if constexpr (IC2_HG4_ABL & 8) asm volatile("" ::"v"(af[u][i]), "v"(bfr[PAIR ? 0 : u][j]));
                else acc[i][j] = mfma32<F16>(af[u][i], bfr[PAIR ? 0 : u][j], acc[i][j]);
              }
          }
        }
      }
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      // step s+1's slabs landed (issued at step s+1-L); a burst of the last L steps may stay in flight (issued after
      // its step's slabs; bursts are >= 3 steps apart)
      const bool recent = burst || (L > 1 && s > 0 && burst_at(s - 1));
      if constexpr (!(IC2_HG4_ABL & 1)) {
        if (recent) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((L - 1) * TPB * NWI + HPW) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"((L - 1) * TPB * NWI) : "memory");
      }
    }
  } else {
#pragma unroll
  for (int t = 0; t < LA; ++t) issue_w(t);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"((LA - 1) * NWI) : "memory");  // halo 0 and slab 0 landed
  for (int t = 0; t < nq; ++t) {
    __builtin_amdgcn_s_barrier();  // slab t and block t/9's halo landed for every wave; step t-1's reads done
    __builtin_amdgcn_sched_barrier(0);
    const int cb = t / 9, tap = t - (t / 9) * 9;
    const int ky = tap / 3, kx = tap - (tap / 3) * 3;
    issue_w(t + LA);  // slab (t+LA) % NS was last read by step t-1
    // the next block's halo (halo (cb+1) & 1 was last read by block cb-1): HB one burst at tap 0, else one DMA
    // per step over the block's first taps; wave-uniform conditions
    const bool hdma = !HB && tap < HPW && cb + 1 < CB && wid + 4 * tap < G::NHI;
    if constexpr (HB) {
      if (tap == 0 && cb + 1 < CB) issue_hb(cb + 1);
    } else if (hdma) {
#pragma unroll
      for (int k = 0; k < HPW; ++k)
        if (k == tap) issue_h1(cb + 1, k);
    }
    __builtin_amdgcn_sched_barrier(0);
    const char* wl = wsl + (t % NS) * G::WS_B;
    const char* hl = hal + (cb & 1) * G::HALO_B;
    bf16x8 af[I], bfr[J];
#pragma unroll
    for (int j = 0; j < J; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(hl + h4_off(brow[j] + ky * G::HW + kx, fh));
#pragma unroll
    for (int i = 0; i < I; ++i) af[i] = *reinterpret_cast<const bf16x8*>(wl + h4_off(obase + i * 16 + fr, fh));
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    if (live) {
#pragma unroll
      for (int i = 0; i < I; ++i)
#pragma unroll
        for (int j = 0; j < J; ++j) acc[i][j] = mfma32<F16>(af[i], bfr[j], acc[i][j]);
    }
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    // slab t+1 (issued at step t+1-LA) landed; the DMAs of the last LA-1 steps may stay in flight (each step
    // issues NWI weight DMAs and, on the block's first taps, one halo DMA; counting the halo DMAs of earlier
    // steps as landed is conservative: vmcnt retires in issue order)
    if constexpr (HB) {  // a burst issued within the last LA-1 steps (tap < LA-1 of a block that issued one)
      if (tap < LA - 1 && cb + 1 < CB) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((LA - 1) * NWI + HPW) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"((LA - 1) * NWI) : "memory");
    } else {
      if (hdma) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((LA - 1) * NWI + 1) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"((LA - 1) * NWI) : "memory");
    }
  }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the tail (zero-size) DMAs before the epilogue

  const int hw = a.ho * a.wo;
  float4 sc[I], bi[I];  // one sample per tile: every channel block's operands before the first store
#pragma unroll
  for (int i = 0; i < I; ++i) {
    sc[i] = ig_load_oscale(a, nn, o0 + obase + i * 16 + 4 * fh);
    bi[i] = ig_load_bias(a, o0 + obase + i * 16 + 4 * fh);
  }
  ig_preloads_done();
  // GN: 32 groups over cout_p = BO channels; a lane's 4 channels of block i are GL whole groups of CPG
  constexpr int CPG = G::BO / 32, GL = 4 / CPG;
  float gs[GN ? I : 1][GL], gq[GN ? I : 1][GL];  // per-group sums of the stored values over this lane's pixels
  if constexpr (GN) {
#pragma unroll
    for (int i = 0; i < I; ++i)
#pragma unroll
      for (int r = 0; r < GL; ++r) gs[i][r] = gq[i][r] = 0.f;
  }
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int pb = pg * J + j;
    const int oy = oy0 + pb * 16 / TW, ox = ox0 + (pb * 16) % TW + fr;
    if (oy >= a.ho || ox >= a.wo) continue;
    const int pix = oy * a.wo + ox;
    const int p = nn * hw + pix;
#pragma unroll
    for (int i = 0; i < I; ++i) {
      const int ob = o0 + obase + i * 16 + 4 * fh;
      if (ob >= a.cout_p) continue;
      const float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if constexpr (GN) {
        float st[4];
        ig_store4v(a, p, nn, pix, ob, v, sc[i], bi[i], &st);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          gs[i][r / CPG] += st[r];
          gq[i][r / CPG] += st[r] * st[r];
        }
      } else {
        ig_store4v(a, p, nn, pix, ob, v, sc[i], bi[i]);
      }
    }
  }
  if constexpr (GN) {
    // GroupNorm partial sums of this tile: the 16 pixel lanes by an xor tree, the WGP pixel waves of a channel
    // block through LDS, then one thread per group adds the waves in a fixed order in f64 -> gn_part[(nn, g, tile)]
    static_assert(G::BO == 64 || G::BO == 128, "GN epilogue: 2 or 4 channels per group");
#pragma unroll
    for (int i = 0; i < I; ++i)
#pragma unroll
      for (int r = 0; r < GL; ++r)
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) {
          gs[i][r] += __shfl_xor(gs[i][r], off, 64);
          gq[i][r] += __shfl_xor(gq[i][r], off, 64);
        }
    __syncthreads();  // every wave is past its last LDS fragment read
    float* red = reinterpret_cast<float*>(lds);  // [2][WGP][32 groups]
    if (fr == 0) {
#pragma unroll
      for (int i = 0; i < I; ++i)
#pragma unroll
        for (int r = 0; r < GL; ++r) {
          const int g = (obase + i * 16 + 4 * fh) / CPG + r;
          red[pg * 32 + g] = gs[i][r];
          red[(WGP + pg) * 32 + g] = gq[i][r];
        }
    }
    __syncthreads();
    if (tid < 32) {
      double sg = 0.0, qg = 0.0;
#pragma unroll
      for (int w = 0; w < WGP; ++w) {
        sg += (double)red[w * 32 + tid];
        qg += (double)red[(WGP + w) * 32 + tid];
      }
      double* o = a.gn_part + (((int64_t)nn * 32 + tid) * (tiles_x * tiles_y) + (ty * tiles_x + tx)) * 2;
      o[0] = sg;
      o[1] = qg;
    }
  }
}

#define IC2_HG4_KERNEL(name, I, J, WGO, WGP, TW, NS)                                                             \
  __global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) name(IgemmArgs a, int tx,  \
                                                                                          int ty) {            \
    hg4_body<I, J, WGO, WGP, TW, NS>(a, tx, ty);                                                                 \
  }                                                                                                              \
  __global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) name##_f16(IgemmArgs a,     \
                                                                                                int tx, int ty) { \
    hg4_body<I, J, WGO, WGP, TW, NS, false, true>(a, tx, ty);                                                    \
  }
// the launch plan's instances: 4-slab one-tap rings for 16-wide pixel tiles, multi-tap halo-burst kernels (below)
// for 32-wide ones
IC2_HG4_KERNEL(hg4_o128_w16_s4_kernel, 8, 4, 1, 4, 16, 4)  // 128 o x (16 x 16) px
IC2_HG4_KERNEL(hg4_o192_w16_s4_kernel, 6, 4, 2, 2, 16, 4)  // 192 o x (8 x 16) px
IC2_HG4_KERNEL(hg4_o64_w16_s4_kernel, 4, 4, 1, 4, 16, 4)   // 64 o x (16 x 16) px
#define IC2_HG4_KERNEL_P(name, I, J, WGO, WGP, TW, NS, TPB)                                                     \
  __global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) name(IgemmArgs a, int tx,  \
                                                                                          int ty) {            \
    hg4_body<I, J, WGO, WGP, TW, NS, true, false, TPB>(a, tx, ty);                                               \
  }                                                                                                              \
  __global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) name##_f16(IgemmArgs a,     \
                                                                                                int tx, int ty) { \
    hg4_body<I, J, WGO, WGP, TW, NS, true, true, TPB>(a, tx, ty);                                                \
  }
// 32-wide tiles: halo burst + several taps per barrier (two for o128 / o192, whose 4-slab ring and double halo
// fill the 80 KB; three for o64 with a 6-slab ring, one barrier per kernel row), profiles/r3_hg4_taps_ab.txt
IC2_HG4_KERNEL_P(hg4_o128_w32_p2_kernel, 8, 4, 1, 4, 32, 4, 2)  // 128 o x (8 x 32) px
IC2_HG4_KERNEL_P(hg4_o192_w32_p2_kernel, 6, 4, 2, 2, 32, 4, 2)  // 192 o x (4 x 32) px
IC2_HG4_KERNEL_P(hg4_o64_w32_p3_kernel, 4, 4, 1, 4, 32, 6, 3)   // 64 o x (8 x 32) px
IC2_HG4_KERNEL_P(hg4_o96_w32_p2_kernel, 6, 4, 1, 4, 32, 4, 2)   // 96 o x (8 x 32) px
// the split-bf16 encoder's 64- / 128-wide convs with the GroupNorm statistics of their f32 output in the epilogue
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2)))
hg4_o64_w32_p3_gn_kernel(IgemmArgs a, int tx, int ty) {
  hg4_body<4, 4, 1, 4, 32, 6, true, false, 3, true>(a, tx, ty);
}
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2)))
hg4_o128_w32_p2_gn_kernel(IgemmArgs a, int tx, int ty) {
  hg4_body<8, 4, 1, 4, 32, 4, true, false, 2, true>(a, tx, ty);
}
// 64-wide outputs on 12 x 32-pixel tiles (wave tile 64 x 96: a weight slab feeds 384 pixels, 1.5x the 8-row tile's)
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2)))
hg4_o64_w32_t12_gn_kernel(IgemmArgs a, int tx, int ty) {
  hg4_body<4, 6, 1, 4, 32, 4, true, false, 2, true>(a, tx, ty);
}
// the same three with f16 operands: the split encoder's first blocks (IC2_F16X2: f16 input, [hi | lo] f16 weights),
// the two-tap-per-step ones walking each tap's hi / lo K blocks as one step (PAIR)
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2)))
hg4_o64_w32_p3_gn_kernel_f16(IgemmArgs a, int tx, int ty) {
  hg4_body<4, 4, 1, 4, 32, 6, true, true, 3, true>(a, tx, ty);
}
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2)))
hg4_o128_w32_p2_gn_kernel_f16(IgemmArgs a, int tx, int ty) {
  hg4_body<8, 4, 1, 4, 32, 4, true, true, 2, true, IC2_HG4_PAIR>(a, tx, ty);
}
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2)))
hg4_o64_w32_t12_gn_kernel_f16(IgemmArgs a, int tx, int ty) {
  hg4_body<4, 6, 1, 4, 32, 4, true, true, 2, true, IC2_HG4_PAIR>(a, tx, ty);
}
#undef IC2_HG4_KERNEL
#undef IC2_HG4_KERNEL_P


// instance: o-tile 96 when cout_p % 192 == 0 (two 96-wide o-tiles on 8 x 32-pixel tiles: a weight slab feeds 256
// pixels instead of the 192-wide tile's 128, so 2.1 instead of 3.4 LDS-DMA pieces per 24 MFMAs; SG3-T-256 L11
// 2.27 -> 2.15 ms, profiles/r4x_hg4_o96.txt), 128 when cout_p % 128 == 0, else 64; IC2_HG4_BO = 192 / 128 / 96 / 64
// forces one where it divides.  Pixel tile 32 or 16 wide, whichever pads the output less (a 96-wide o-tile whose
// output pads less on 16-wide tiles runs as the 192-wide 16-wide-tile instance).
struct H4Plan {
  int bo;
  bool tw32;
  int64_t blocks;
};
static H4Plan h4_plan(int n, int ho, int wo, int cout_p) {
  static const int force_bo = knob("IC2_HG4_BO", 0);
  H4Plan p;
  p.bo = cout_p % 192 == 0 ? 96 : cout_p % 128 == 0 ? 128 : 64;
  if ((force_bo == 192 || force_bo == 128 || force_bo == 96 || force_bo == 64) && cout_p % force_bo == 0)
    p.bo = force_bo;
  const int bp32 = p.bo <= 128 ? 256 : 128, bp16 = p.bo <= 128 && p.bo != 96 ? 256 : 128;
  const int th32 = bp32 / 32, th16 = bp16 / 16;
  const int64_t a32 = ceil_div(ho, th32) * th32 * ceil_div(wo, 32) * 32;
  const int64_t a16 = ceil_div(ho, th16) * th16 * ceil_div(wo, 16) * 16;
  p.tw32 = a32 <= a16;
  if (p.bo == 96 && !p.tw32) p.bo = 192;
  const int64_t tiles = p.tw32 ? ceil_div(ho, th32) * ceil_div(wo, 32) : ceil_div(ho, th16) * ceil_div(wo, 16);
  p.blocks = n * tiles * ceil_div(cout_p, p.bo);
  return p;
}

template <int I, int J, int WGO, int WGP, int TW>
static void launch_hg4(IgemmArgs a, hipStream_t s, void (*kern)(IgemmArgs, int, int)) {
  constexpr int BO = 16 * I * WGO, TH = 16 * J * WGP / TW;
  const int tiles_x = (int)ceil_div(a.wo, TW), tiles_y = (int)ceil_div(a.ho, TH);
  a.tiles_o = (a.cout_p + BO - 1) / BO;
  a.nblocks = a.n * tiles_x * tiles_y * a.tiles_o;
  hipLaunchKernelGGL(kern, dim3(a.nblocks), dim3(256), 0, s, a, tiles_x, tiles_y);
}

// the halo burst on 32-wide tiles (s276a +2.6 %, s276b +3 %, SG3-T-1024 L11 +7 % over spreading the halo DMAs over
// the first taps, profiles/r2f_hg4_hb.txt); a 4-slab weight ring (+0.5-1 % over 3, profiles/r2e_hg4_sweep.txt)
static void hg4_dispatch(const IgemmArgs& a, hipStream_t s, bool f16) {
  const H4Plan p = h4_plan(a.n, a.ho, a.wo, a.cout_p);
  if (p.tw32) {
    if (p.bo == 192) launch_hg4<6, 4, 2, 2, 32>(a, s, f16 ? hg4_o192_w32_p2_kernel_f16 : hg4_o192_w32_p2_kernel);
    else if (p.bo == 128) launch_hg4<8, 4, 1, 4, 32>(a, s, f16 ? hg4_o128_w32_p2_kernel_f16 : hg4_o128_w32_p2_kernel);
    else if (p.bo == 96) launch_hg4<6, 4, 1, 4, 32>(a, s, f16 ? hg4_o96_w32_p2_kernel_f16 : hg4_o96_w32_p2_kernel);
    else launch_hg4<4, 4, 1, 4, 32>(a, s, f16 ? hg4_o64_w32_p3_kernel_f16 : hg4_o64_w32_p3_kernel);
  } else {
    if (p.bo == 192) launch_hg4<6, 4, 2, 2, 16>(a, s, f16 ? hg4_o192_w16_s4_kernel_f16 : hg4_o192_w16_s4_kernel);
    else if (p.bo == 128) launch_hg4<8, 4, 1, 4, 16>(a, s, f16 ? hg4_o128_w16_s4_kernel_f16 : hg4_o128_w16_s4_kernel);
    else launch_hg4<4, 4, 1, 4, 16>(a, s, f16 ? hg4_o64_w16_s4_kernel_f16 : hg4_o64_w16_s4_kernel);
  }
}

// bf16 3x3 with 32-deep channel blocks.  Default: on a grid of >= 2 workgroups per CU, <= 512 channels in, <= 192
// out, >= 93 % pixel-tile utilisation (tools/sweep_igemm.py, profiles/r2e_hg4_sweep.txt).  Knob IC2_HG4 (IC2_DEV=1):
// 0 disables it, 2 forces it wherever legal (the tests' forced-instance runs).
static bool hg4_legal(int dtype, int cin_p, int cout_p, int kh, int kw, int64_t x_elems) {
  return is16(dtype) && kh == 3 && kw == 3 && cin_p % 32 == 0 && cout_p % 64 == 0 &&
         x_elems * 2 < (int64_t)kOob && (int64_t)cout_p * 9 * cin_p * 2 < (int64_t)kOob;
}
static bool hg4_eligible(int dtype, int cin_p, int cout_p, int kh, int kw, int64_t x_elems, int n, int ho, int wo) {
  static const int mode = knob("IC2_HG4", 1);
  if (!mode || !hg4_legal(dtype, cin_p, cout_p, kh, kw, x_elems)) return false;
  if (mode == 2) return true;
  const H4Plan p = h4_plan(n, ho, wo, cout_p);
  if (p.blocks < 512) return false;
  const int th = (p.bo <= 128 ? 256 : 128) / (p.tw32 ? 32 : 16);
  const double util = (double)ho * wo / ((double)ceil_div(ho, th) * th * ceil_div(wo, p.tw32 ? 32 : 16) * (p.tw32 ? 32 : 16));
  // inputs up to 512 channels (the split encoder's 384-wide block-1 conv2: og1 -> hg4 + fused statistics, C4
  // +1.1 %, profiles/r3_hg4_maxc_ab.txt); knob IC2_HG4_MAXC for the A/B
  static const int maxc = knob("IC2_HG4_MAXC", 512);
  return cin_p <= maxc && cout_p <= 192 && util >= 0.93;
}

// ------------------------------------------------------------------------------------------------
// launch plan: tile instance and K split.  Tile ids: 0 = f32 128x128 (2-stage); bf16: 1 = 256x256,
// 2 = 32x256, 3 = 128x256, 4 = 128x128, 5 = 64x256 (4-stage ring), 6 = 8-phase 256x256, 7 = 8-phase 128x512.
// Knobs (IC2_DEV=1 only): IC2_IGEMM_TILE=1..7 forces a bf16 tile (the tests exercise every instance on small
// problems), IC2_IGEMM_G8N=0 keeps the cout_p <= 128 layers off the 8-phase kernel, IC2_IGEMM_SPLITK=0 disables
// split-K.
struct IgPlan {
  int tile, bo, bp, splits;
  int tail = 0;  // tile 6, one full-K launch of whole rounds + the remaining tiles split over K in two (see ig_plan)
};

static IgPlan ig_plan(int dtype, int64_t M, int cout_p, int cin_p, int kh, int kw, int64_t x_elems, bool x8 = true) {
  static const int BOs[8] = {128, 256, 32, 128, 128, 64, 256, 128};
  static const int BPs[8] = {128, 256, 256, 256, 128, 256, 256, 512};
  static const int forced = knob("IC2_IGEMM_TILE", 0);
  static const bool g8n = knob("IC2_IGEMM_G8N", 1) != 0;
  static const bool splitk = knob("IC2_IGEMM_SPLITK", 1) != 0;
  const int64_t K = (int64_t)kh * kw * cin_p;
  int tile = 0;
  if (is16(dtype)) {
    // o-tile: the widest of {256, 128, 64, 32} that divides cout_p (no padded MFMA rows), 256-pixel
    // tiles while the grid keeps >= 2 workgroups per CU, else the 128 x 128 tile
    const bool big_m = ceil_div(M, 256) * ((cout_p + 255) / 256) >= 512;
    if (!big_m) tile = cout_p <= 32 ? 2 : 4;
    else if (cout_p % 256 == 0) tile = 1;
    else if (cout_p % 128 == 0) tile = 3;
    else if (cout_p % 64 == 0) tile = 5;
    else tile = 2;
    // the 8-phase kernels wherever K-tiles are 64 deep (their buffer descriptors address < 2 GiB per
    // operand and their tap masks hold <= 32 taps) and the grid keeps ~1 workgroup per CU (measured on the
    // bench shapes, tools/sweep_igemm.py): 256 x 256 for cout_p > 128 (padded 64-row quadrants skip their
    // MFMAs) unless cout_p is an odd multiple of 128 (384: the 128 x 512 tile pads nothing), 128 x 512 for
    // 64 < cout_p <= 128; cout_p = 64 keeps the 64 x 256 tile
    const bool fits8 = x8 && cin_p % 64 == 0 && kh * kw <= 32 && x_elems * 2 < (int64_t)kOob &&
                       (int64_t)cout_p * K * 2 < (int64_t)kOob;
    const bool odd128 = cout_p % 256 == 128 && cout_p > 128;
    // small grids (the encoder's 512-wide blocks at <= 32^2): the same 8-phase tiles with K split over
    // gridDim.y so the launch reaches ~1 workgroup per CU, instead of the 4-stage 128 x 128 split-K tile
    static const bool g8_splitk = knob("IC2_G8_SPLITK", 1) != 0;
    const int64_t g6 = ceil_div(M, 256) * ((cout_p + 255) / 256), g7 = ceil_div(M, 512) * ((cout_p + 127) / 128);
    const bool k_deep = K / 64 >= 32;
    int g8_split = 1;
    // knob IC2_G8_TARGET: workgroups the split aims at (default 240, ~1 per CU of the 1-workgroup-per-CU kernel)
    static const int g8_target = knob("IC2_G8_TARGET", 240);
    // (a full-K grid of 1-2 rounds is not split for wave balance: SG3-T-256 L0-L3's 362 workgroups as 724 half-K ones
    // measured 10 % slower, the f32 partials and the combine costing more than the idle tail, r6_schedule_ab.txt)
    if (fits8 && cout_p > 128 && !odd128 && g6 >= 240) tile = 6;
    else if (g8n && fits8 && (odd128 || (cout_p > 64 && cout_p <= 128)) && g7 >= 240) tile = 7;
    else if (g8_splitk && splitk && fits8 && k_deep && cout_p > 128 && !odd128)
      tile = 6, g8_split = (int)ceil_div(g8_target, g6);
    if (g8_split > 1) {
      int64_t sp = g8_split;
      if (sp > K / 64 / 8) sp = K / 64 / 8;  // >= 8 K-tiles of 64 per slice
      if (sp > 32) sp = 32;
      g8_split = M * cout_p < (1LL << 31) ? (int)sp : 1;
    }
    if (forced >= 1 && forced <= 7) tile = forced, g8_split = 1;
    if ((tile == 6 || tile == 7) && !fits8) tile = 1, g8_split = 1;
    if (g8_split > 1) return IgPlan{tile, BOs[tile], BPs[tile], g8_split};
  }
  IgPlan pl{tile, BOs[tile], BPs[tile], 1};
  // Wave balance of a full-K 256 x 256 grid (one workgroup per CU on 256 CUs): a last round of r <= 128 tiles runs as
  // 2r half-K workgroups -- one round of half the time -- behind a launch of the whole rounds; the tail's f32 partials
  // are combined over its pixels only (SG3-T-256 L0-L2 at batch 32: 362 tiles = 256 + 106, 2 rounds -> 1.5).  Round 6
  // split every tile of such a grid instead (724 half-K workgroups: 10 % slower, every tile paying the partials).
  static const bool g8_tail = knob("IC2_G8_TAIL", 1) != 0;
  if (tile == 6 && g8_tail && splitk && K / 64 >= 16 && M * cout_p < (1LL << 31)) {
    const int64_t tiles_o = (cout_p + 255) / 256, tiles = ceil_div(M, 256) * tiles_o, rem = tiles % 256;
    if (tiles > 256 && rem > 0 && rem <= 128 && (tiles - rem) % tiles_o == 0) pl.tail = 1;
  }
  if (tile < 6 && splitk) {
    // fewer workgroups than ~1.25 per CU: split K so the launch reaches ~512 workgroups, each slice
    // keeping >= 8 chunks of 32
    const int64_t blocks = ceil_div(M, pl.bp) * ceil_div(cout_p, pl.bo);
    const int64_t nq32 = K / 32;
    if (blocks < 320 && M * cout_p < (1LL << 31)) {
      int64_t sp = ceil_div(512, blocks);
      if (sp > nq32 / 8) sp = nq32 / 8;
      if (sp > 32) sp = 32;
      pl.splits = sp < 1 ? 1 : (int)sp;
    }
  }
  return pl;
}

// ------------------------------------------------------------------------------------------------
// Halo direct conv for narrow 3x3 layers (cin_p <= 96, cout_p <= 64; bf16): the encoder's block 0 and from_rgb
// and the SG3-T-1024 tail (L11_1044_51, L12_1044_32, L13_1024_32) at >= 256^2.  There the implicit GEMM above re-fetches
// every input pixel once per tap (9 shifted 256-pixel panels per 32 channels) for only 32-64 MACs per
// fetched element, and its per-chunk barrier guards 8-16 MFMAs.  Here a persistent workgroup keeps the
// whole packed weight [cout_p][9][cin_p] in LDS, stages one (TH+2) x (32+2) x cin_p input halo per
// TH x 32-pixel output tile (TH = 8, or 4 at 96 channels; fetched once: 1.6x instead of 9x), and runs all 9 * cin_p/32 K-steps without
// a barrier.  The next tile's halo is loaded into registers while the current tile computes.
// Wave w of 8 owns pixel blocks {w, w+8, ...} (16 pixels of one row) x every 16-channel o-block:
// A = weights (lane: o = 16i + fr, k = 8 fh .. +7), B = halo pixels (lane: pixel fr, k = 8 fh .. +7).
// Epilogue = ig_store4 (same oscale / bias / activation / output layouts as the implicit GEMM).
// lrelu((v - mean) * scale + shift) on 8 bf16 values, rounded back to bf16: the arithmetic of
// gn_apply_oct_kernel (encoder_ops.hip) on the same operands, so a fused input equals the materialised one bit for bit
__device__ __forceinline__ uint4 gn_lrelu_bf16x8(uint4 u, const float4 (&p)[8], float slope) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
  uint32_t o[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float lo = __uint_as_float(w[k] << 16), hi = __uint_as_float(w[k] & 0xffff0000u);
    lo = __builtin_fmaf(lo - p[2 * k].x, p[2 * k].y, p[2 * k].z);
    hi = __builtin_fmaf(hi - p[2 * k + 1].x, p[2 * k + 1].y, p[2 * k + 1].z);
    lo = lo < 0.f ? lo * slope : lo;
    hi = hi < 0.f ? hi * slope : hi;
    o[k] = (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
  }
  return make_uint4(o[0], o[1], o[2], o[3]);
}

template <int CINP, int COUTP, int TH>
struct HcCfg {
  static constexpr int TW = 32, HR = TH + 2, HC = TW + 2;
  static constexpr int PPB = CINP * 2 + 16;          // halo pixel pitch (bytes): 16 lanes hit distinct banks
  static constexpr int WPB = 9 * CINP * 2 + 16;      // weight row pitch (bytes)
  static constexpr int HALO_B = HR * HC * PPB, W_B = COUTP * WPB;
  static constexpr int CB = CINP / 32, OB = COUTP / 16, JB = TH * 2 / 8;
  static constexpr int NPIECE = HR * HC * (CINP / 8);  // 16-B pieces per halo
  static constexpr int PER_T = (NPIECE + 511) / 512;
};

template <int CINP, int COUTP, int TH, bool GN, bool F16 = false>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(CINP == 32 ? 4 : 1)))
hconv_kernel(IgemmArgs a, int tiles_x, int tiles_y, int ntiles) {
  static_assert(!(F16 && GN), "the fused GroupNorm statistics are an encoder (bf16) feature");
  using C = HcCfg<CINP, COUTP, TH>;
  __shared__ __attribute__((aligned(16))) char lds[C::HALO_B + C::W_B];
  char* const halo = lds;
  char* const wts = lds + C::HALO_B;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fh = lane >> 4;

  // packed weight -> LDS, once per workgroup
  const char* wg = reinterpret_cast<const char*>(a.w);
  constexpr int WPIECE = 9 * CINP / 8;
  for (int e = tid; e < COUTP * WPIECE; e += 512) {
    const int o = e / WPIECE, r = e - o * WPIECE;
    *reinterpret_cast<uint4*>(wts + o * C::WPB + r * 16) =
        *reinterpret_cast<const uint4*>(wg + ((int64_t)o * 9 * CINP + r * 8) * 2);
  }

  const char* xg = reinterpret_cast<const char*>(a.x);
  uint4 pre[C::PER_T];
  // input GroupNorm + lrelu (a.in_gn; the 64-channel instances only -- the 32-channel ones run at 4 waves per SIMD
  // and would spill the 32 extra VGPRs): 512 % 8 == 0, so a thread's pieces all hold channels (tid % 8) * 8 .. +7,
  // whose (mean, scale, shift) are loaded once per tile
  constexpr bool kGnIn = CINP == 64;
  float4 gnp[8];
  uint32_t inimg = 0;
  auto fetch = [&](int t) {
    const int tx = t % tiles_x;
    const int t2 = t / tiles_x;
    const int ty = t2 % tiles_y;
    const int nn = t2 / tiles_y;
    const int y0 = ty * TH - a.pad, x0 = tx * C::TW - a.pad;
    inimg = 0;
#pragma unroll
    for (int k = 0; k < C::PER_T; ++k) {
      const int e = tid + 512 * k;
      const int pi = e / (CINP / 8), part = e - pi * (CINP / 8);
      const int hr = pi / C::HC, hc = pi - hr * C::HC;
      const int iy = y0 + hr, ix = x0 + hc;
      const bool ok = e < C::NPIECE && (unsigned)iy < (unsigned)a.h && (unsigned)ix < (unsigned)a.w_;
      inimg |= (uint32_t)ok << k;
      pre[k] = ok ? *reinterpret_cast<const uint4*>(xg + ((((int64_t)nn * a.h + iy) * a.w_ + ix) * CINP + part * 8) * 2)
                  : make_uint4(0u, 0u, 0u, 0u);
    }
    if constexpr (kGnIn) {
      if (a.in_gn) {
        const float4* tb = reinterpret_cast<const float4*>(a.in_gn) + ((int64_t)nn * CINP + (tid % (CINP / 8)) * 8);
#pragma unroll
        for (int c = 0; c < 8; ++c) gnp[c] = tb[c];
      }
    }
  };
  if (blockIdx.x < ntiles) fetch(blockIdx.x);

  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    __syncthreads();  // the previous tile's halo reads (and the weight stores) are done
#pragma unroll
    for (int k = 0; k < C::PER_T; ++k) {
      const int e = tid + 512 * k;
      if (e < C::NPIECE) {
        const int pi = e / (CINP / 8), part = e - pi * (CINP / 8);
        uint4 v = pre[k];
        if constexpr (kGnIn) {  // zero padding stays zero: only in-image pieces are normalised
          if (a.in_gn && ((inimg >> k) & 1u)) v = gn_lrelu_bf16x8(v, gnp, a.in_slope);
        }
        *reinterpret_cast<uint4*>(halo + pi * C::PPB + part * 16) = v;
      }
    }
    __syncthreads();
    if (t + (int)gridDim.x < ntiles) fetch(t + gridDim.x);  // in flight during this tile's MFMAs

    f32x4 acc[C::OB][C::JB];
#pragma unroll
    for (int i = 0; i < C::OB; ++i)
#pragma unroll
      for (int j = 0; j < C::JB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int ky = tap / 3, kx = tap - 3 * (tap / 3);
#pragma unroll
      for (int cb = 0; cb < C::CB; ++cb) {
        bf16x8 bfr[C::JB], af[C::OB];
#pragma unroll
        for (int j = 0; j < C::JB; ++j) {
          const int pb = wave + 8 * j;
          const int r = pb >> 1, c0 = (pb & 1) * 16;
          bfr[j] = *reinterpret_cast<const bf16x8*>(halo + ((r + ky) * C::HC + c0 + kx + fr) * C::PPB + cb * 64 +
                                                    fh * 16);
        }
#pragma unroll
        for (int i = 0; i < C::OB; ++i)
          af[i] = *reinterpret_cast<const bf16x8*>(wts + (16 * i + fr) * C::WPB + (tap * CINP + cb * 32) * 2 + fh * 16);
#pragma unroll
        for (int i = 0; i < C::OB; ++i)
#pragma unroll
          for (int j = 0; j < C::JB; ++j)
            acc[i][j] = mfma32<F16>(af[i], bfr[j], acc[i][j]);
      }
    }

    const int tx = t % tiles_x;
    const int t2 = t / tiles_x;
    const int ty = t2 % tiles_y;
    const int nn = t2 / tiles_y;
    // GN (fused statistics, groups = 32 over all COUTP channels): CPG = COUTP / 32 channels per group, so a
    // lane's 4 channels 16i + 4fh .. +3 fall in 4 / CPG groups
    constexpr int CPG = COUTP / 32, GL = 4 / CPG;
    float gs[C::OB][GL], gq[C::OB][GL];
    if constexpr (GN) {
#pragma unroll
      for (int i = 0; i < C::OB; ++i)
#pragma unroll
        for (int r = 0; r < GL; ++r) gs[i][r] = gq[i][r] = 0.f;
    }
    // every channel block's operands before the first store (see ig_load_oscale); not in the 32 -> 64 instance,
    // whose 4-waves-per-SIMD register budget (128) would spill them (measured 142 -> 179 us on e0a) and whose
    // occupancy hides the per-block loads instead
    constexpr bool kPre = !(CINP == 32 && COUTP == 64);
    float4 sc[C::OB], bi[C::OB];
    if constexpr (kPre) {
#pragma unroll
      for (int i = 0; i < C::OB; ++i) {
        sc[i] = ig_load_oscale(a, nn, 16 * i + 4 * fh);
        bi[i] = ig_load_bias(a, 16 * i + 4 * fh);
      }
      ig_preloads_done();
    }
#pragma unroll
    for (int j = 0; j < C::JB; ++j) {
      const int pb = wave + 8 * j;
      const int oy = ty * TH + (pb >> 1), ox = tx * C::TW + (pb & 1) * 16 + fr;
      if (oy >= a.ho || ox >= a.wo) continue;
      const int pix = oy * a.wo + ox;
      const int p = nn * a.ho * a.wo + pix;
#pragma unroll
      for (int i = 0; i < C::OB; ++i) {
        const float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        if constexpr (!kPre) {
          sc[i] = ig_load_oscale(a, nn, 16 * i + 4 * fh);
          bi[i] = ig_load_bias(a, 16 * i + 4 * fh);
        }
        ig_store4v(a, p, nn, pix, 16 * i + 4 * fh, v, sc[i], bi[i]);
        if constexpr (GN) {  // statistics of the value as stored: bias added, rounded to bf16
          const float bv[4] = {bi[i].x, bi[i].y, bi[i].z, bi[i].w};
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float st = bf2f(f2bf(v[r] + bv[r]));
            gs[i][r / CPG] += st;
            gq[i][r / CPG] += st * st;
          }
        }
      }
    }
    if constexpr (GN) {
      // wave: sum over the 16 pixel lanes; workgroup: 8 waves through LDS (the halo region, after a barrier);
      // then one thread per group sums the waves in a fixed order -> part[(nn, g, tile)]
#pragma unroll
      for (int i = 0; i < C::OB; ++i)
#pragma unroll
        for (int r = 0; r < GL; ++r)
#pragma unroll
          for (int off = 1; off < 16; off <<= 1) {
            gs[i][r] += __shfl_xor(gs[i][r], off, 64);
            gq[i][r] += __shfl_xor(gq[i][r], off, 64);
          }
      __syncthreads();  // every wave is past its halo reads
      float* red = reinterpret_cast<float*>(halo);  // [2][8 waves][32 groups]
      if (fr == 0) {
#pragma unroll
        for (int i = 0; i < C::OB; ++i)
#pragma unroll
          for (int r = 0; r < GL; ++r) {
            const int g = (16 * i + 4 * fh) / CPG + r;
            red[wave * 32 + g] = gs[i][r];
            red[(8 + wave) * 32 + g] = gq[i][r];
          }
      }
      __syncthreads();
      if (tid < 32) {
        double sg = 0.0, qg = 0.0;
#pragma unroll
        for (int w8 = 0; w8 < 8; ++w8) {
          sg += (double)red[w8 * 32 + tid];
          qg += (double)red[(8 + w8) * 32 + tid];
        }
        double* o = a.gn_part + (((int64_t)nn * 32 + tid) * (tiles_x * tiles_y) + (ty * tiles_x + tx)) * 2;
        o[0] = sg;
        o[1] = qg;
      }
      // the next tile's first barrier orders these LDS reads before its halo stores
    }
  }
}

template <int CINP, int COUTP, bool GN = false, bool F16 = false>
static void launch_hconv(const IgemmArgs& a, hipStream_t s) {
  constexpr int TH = CINP > 64 ? 4 : 8;  // 96 channels: 4-row tiles keep halo + weight within 160 KB of LDS
  const int tiles_x = (int)ceil_div(a.wo, 32), tiles_y = (int)ceil_div(a.ho, TH);
  const int ntiles = a.n * tiles_x * tiles_y;
  static int resident = 0;
  if (resident == 0) {
    int dev = 0, cus = 0, per_cu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, hconv_kernel<CINP, COUTP, TH, GN, F16>, 512, 0);
    resident = (cus > 0 ? cus : 256) * (per_cu > 0 ? per_cu : 1);
  }
  const int grid = ntiles < resident ? ntiles : resident;
  hipLaunchKernelGGL((hconv_kernel<CINP, COUTP, TH, GN, F16>), dim3((unsigned)grid), dim3(512), 0, s, a, tiles_x,
                     tiles_y, ntiles);
}

// the halo kernel for bf16 3x3 convs with cin_p in {32, 64, 96}, cout_p in {32, 64} and >= 64K output
// pixels; knob IC2_HCONV=0 keeps them on the implicit GEMM
static bool hconv_eligible(int dtype, int64_t M, int cin_p, int cout_p, int kh, int kw) {
  static const bool on = knob("IC2_HCONV", 1) != 0;
  return on && is16(dtype) && kh == 3 && kw == 3 && (cin_p == 32 || cin_p == 64 || cin_p == 96) &&
         (cout_p == 32 || cout_p == 64) && M >= 65536;
}

// ------------------------------------------------------------------------------------------------
// ToRGB (1x1 conv to <= 4 channels, NCHW f32 output; SG3 SynthesisLayer L14, is_torgb): HBM-bound, so a
// VALU dot product instead of a 32-row MFMA tile that is 29/32 padding.  L = cin_p/16 lanes per pixel,
// 16 channels (2 x 16 B) each, a fixed xor-shuffle tree over the L lanes, then the igemm epilogue math
// (oscale, bias, activation / clamp, out_mul) on the group's first lane.
// 2-byte element -> f32 (bf16: the high half; f16: a conversion)
template <bool F16>
__device__ __forceinline__ float h2f(uint32_t bits16) {
  if constexpr (F16) return (float)__builtin_bit_cast(_Float16, (uint16_t)bits16);
  else return __uint_as_float(bits16 << 16);
}

template <int L, int CV, bool F16 = false>
__global__ void __launch_bounds__(256) torgb_kernel(IgemmArgs a) {
  const int tid = blockIdx.x * 256 + threadIdx.x;
  const int sub = threadIdx.x & (L - 1);
  const int hw = a.ho * a.wo;
  float wv[CV][16];
  const uint16_t* wg = reinterpret_cast<const uint16_t*>(a.w);
#pragma unroll
  for (int o = 0; o < CV; ++o)
#pragma unroll
    for (int k = 0; k < 16; ++k) wv[o][k] = h2f<F16>(wg[(int64_t)o * a.cin_p + sub * 16 + k]);
  float bi[CV];
#pragma unroll
  for (int o = 0; o < CV; ++o) bi[o] = a.bias ? a.bias[o] : 0.f;
  const uint16_t* xg = reinterpret_cast<const uint16_t*>(a.x);
  float* yo = reinterpret_cast<float*>(a.y);
  const int stride = gridDim.x * (256 / L);
  for (int p = tid / L; p < a.M; p += stride) {
    const uint4* src = reinterpret_cast<const uint4*>(xg + (int64_t)p * a.cin_p + sub * 16);
    const uint4 u0 = src[0], u1 = src[1];
    const uint32_t w32[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
    float acc[CV];
#pragma unroll
    for (int o = 0; o < CV; ++o) acc[o] = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float lo = h2f<F16>(w32[k] & 0xffffu), hi = h2f<F16>(w32[k] >> 16);
#pragma unroll
      for (int o = 0; o < CV; ++o) acc[o] = fmaf(wv[o][2 * k + 1], hi, fmaf(wv[o][2 * k], lo, acc[o]));
    }
#pragma unroll
    for (int m = 1; m < L; m <<= 1)
#pragma unroll
      for (int o = 0; o < CV; ++o) acc[o] += __shfl_xor(acc[o], m, 64);
    if (sub == 0) {
      const int nn = p / hw, pix = p - nn * hw;
#pragma unroll
      for (int o = 0; o < CV; ++o) {
        if (o >= a.cout_valid) break;
        float t = acc[o] * (a.oscale ? a.oscale[(int64_t)nn * a.cout_p + o] : 1.f) + bi[o];
        if (a.act) t = lrelu_gain_clamp(t, a.slope, a.act_gain, a.clamp);
        yo[((int64_t)nn * a.cout_valid + o) * hw + pix] = t * a.out_mul;
      }
    }
  }
}

// (the kernel maps output pixel p to input pixel p: 1x1, no padding)
static bool torgb_eligible(int dtype, int cin_p, int cout_valid, int kh, int kw, int pad, int out_layout,
                           int out_dtype) {
  static const bool on = knob("IC2_TORGB", 1) != 0;
  return on && is16(dtype) && kh == 1 && kw == 1 && pad == 0 && cout_valid <= 4 && out_layout == IC2_LAYOUT_NCHW &&
         out_dtype == IC2_F32 && (cin_p == 32 || cin_p == 64 || cin_p == 128);
}

template <bool F16>
static void launch_torgb(const IgemmArgs& a, hipStream_t s) {
  const int L = a.cin_p / 16;
  const int64_t need = ceil_div((int64_t)a.M * L, 256);
  const unsigned grid = (unsigned)(need < 8192 ? need : 8192);
  if (L == 2) hipLaunchKernelGGL((torgb_kernel<2, 4, F16>), dim3(grid), dim3(256), 0, s, a);
  else if (L == 4) hipLaunchKernelGGL((torgb_kernel<4, 4, F16>), dim3(grid), dim3(256), 0, s, a);
  else hipLaunchKernelGGL((torgb_kernel<8, 4, F16>), dim3(grid), dim3(256), 0, s, a);
}

// the 2-byte (bf16 / f16) implicit-GEMM tiles and the halo conv configurations, by operand type
// first tile of the split tail of a 256 x 256 8-phase grid (IgPlan::tail): the whole rounds before it
static int g8_tail_first(int64_t M, int cout_p) {
  const int64_t g6 = ceil_div(M, 256) * ((cout_p + 255) / 256);
  return (int)(g6 - g6 % 256);
}
template <bool F16>
static void launch_igemm16(const IgemmArgs& a, hipStream_t s, const IgPlan& pl, bool split384, int cout_p) {
  switch (pl.tile) {
    case 6:
      if (pl.tail) {  // whole rounds at full K, then the tail tiles split over K in two (ig_plan)
        const int full = g8_tail_first(a.M, a.cout_p);
        launch_g8<2, F16>(a, s, 0, -1, 1, 0, full);
        launch_g8<2, F16>(a, s, 0, -1, 2, full, -1);
      } else {
        launch_g8<2, F16>(a, s, 0, -1, pl.splits);
      }
      break;
    case 7:
      if (split384) {
        launch_g8<2, F16>(a, s, 0, cout_p - 128, pl.splits);
        launch_g8<1, F16>(a, s, cout_p - 128, cout_p, pl.splits);
      } else {
        launch_g8<1, F16>(a, s, 0, -1, pl.splits);
      }
      break;
    case 1: launch_igemm<true, 256, 256, 2, 4, 4, F16>(a, pl.splits, s); break;
    case 2: launch_igemm<true, 32, 256, 1, 4, 4, F16>(a, pl.splits, s); break;
    case 3: launch_igemm<true, 128, 256, 2, 4, 4, F16>(a, pl.splits, s); break;
    case 5: launch_igemm<true, 64, 256, 1, 4, 4, F16>(a, pl.splits, s); break;
    default: launch_igemm<true, 128, 128, 2, 2, 4, F16>(a, pl.splits, s); break;
  }
}
template <bool F16>
static void launch_hconv_cfg(const IgemmArgs& a, hipStream_t s, int cin_p, int cout_p) {
  if (cin_p == 32 && cout_p == 32) launch_hconv<32, 32, false, F16>(a, s);
  else if (cin_p == 32) launch_hconv<32, 64, false, F16>(a, s);
  else if (cin_p == 64 && cout_p == 32) launch_hconv<64, 32, false, F16>(a, s);
  else if (cin_p == 64) launch_hconv<64, 64, false, F16>(a, s);
  else if (cout_p == 32) launch_hconv<96, 32, false, F16>(a, s);
  else launch_hconv<96, 64, false, F16>(a, s);
}

// ------------------------------------------------------------------------------------------------
// The launch plan of ic2_conv_igemm_ws, in one place: the dispatcher, the workspace query and the plan-name query
// (tests / bench) all read it, so what is tested and timed is what runs.
// stored elements per input pixel: the split-bf16 input (IC2_BF16X3, cin_p = the GEMM's tripled K channels) is
// stored [hi | lo], 2/3 of them; the f16 input of the split-weight mode (IC2_F16X2, cin_p = the doubled K) half
static int x_pix_of(int dtype, int cin_p) {
  return dtype == IC2_BF16X3 ? cin_p / 3 * 2 : dtype == IC2_F16X2 ? cin_p / 2 : cin_p;
}
// 32-channel blocks of the stored input the split K runs over twice (hi, hi) / once more (x, x) (0: plain input)
static int x_hb32_of(int dtype, int cin_p) { return dtype == IC2_BF16X3 ? cin_p / 96 : dtype == IC2_F16X2 ? cin_p / 64 : 0; }

enum ConvKind { CK_TORGB, CK_HG4, CK_HCONV, CK_IGEMM };
struct ConvChoice {
  ConvKind kind;
  IgPlan pl;
  bool split384;  // tile 7 on an odd multiple of 128 above 128: two 8-phase launches (og2 + og1)
};

static ConvChoice conv_choice(int dtype, int out_layout, int out_dtype, int n, int h, int w_, int cin_p, int cout_p,
                              int cout_valid, int kh, int kw, int pad) {
  const int ho = h + 2 * pad - kh + 1, wo = w_ + 2 * pad - kw + 1;
  const int64_t M = (int64_t)n * ho * wo;
  const int64_t x_elems = (int64_t)n * h * w_ * x_pix_of(dtype, cin_p);  // stored elements (buffer-offset limits)
  ConvChoice c;
  // the split inputs (IC2_BF16X3 [hi | lo] storage, IC2_F16X2 plain f16) run on the kernels whose input addressing
  // maps the tripled / doubled K onto them (implicit GEMM, 8-phase, hg4), planned as the 16-bit GEMM over that K.
  // The 8-phase kernels address 64-channel K blocks: the doubled K needs an even number of stored 32-channel blocks
  const bool x3 = dtype == IC2_BF16X3 || dtype == IC2_F16X2;
  const bool x8 = dtype != IC2_F16X2 || (cin_p / 2) % 64 == 0;
  if (x3) dtype = dtype == IC2_F16X2 ? IC2_F16 : IC2_BF16;
  c.pl = ig_plan(dtype, M, cout_p, cin_p, kh, kw, x_elems, x8);
  c.split384 = false;
  if (!x3 && torgb_eligible(dtype, cin_p, cout_valid, kh, kw, pad, out_layout, out_dtype)) {
    c.kind = CK_TORGB;
    c.pl.splits = 1;
    return c;
  }
  // hg4 ahead of the halo direct conv for >= 96 input channels (SG3-T-1024 L11: 1532 -> 1363 us at batch 8); the
  // 32 / 64-channel encoder layers stay on hconv (faster there).  Knob IC2_HG4_HCONV = 0 / 1: never / always.
  static const int hg4_over_hconv = knob("IC2_HG4_HCONV", -1);
  const bool hg4_ok = hg4_eligible(dtype, cin_p, cout_p, kh, kw, x_elems, n, ho, wo);
  const bool hg4_pref = hg4_over_hconv == 1 || (hg4_over_hconv < 0 && cin_p >= 96);
  if (hg4_ok && hg4_pref) c.kind = CK_HG4;
  else if (!x3 && hconv_eligible(dtype, M, cin_p, cout_p, kh, kw)) c.kind = CK_HCONV;
  else if (hg4_ok) c.kind = CK_HG4;
  else c.kind = CK_IGEMM;
  if (c.kind != CK_IGEMM) {
    c.pl.splits = 1;
    return c;
  }
  // an odd multiple of 128 above 128 (384: SG3-T-256 L9, SG3-T-1024 L7): the 256-wide tile on all but the last
  // 128 channels, the 128 x 512 tile on those (both read the same input panel); knob IC2_IGEMM_SPLIT=0 keeps one
  // 128 x 512 launch
  static const bool split = knob("IC2_IGEMM_SPLIT", 1) != 0;
  c.split384 = is16(dtype) && c.pl.tile == 7 && split && cout_p % 256 == 128 && cout_p > 128 &&
               ceil_div(M, 256) >= 240;
  return c;
}

static const char* conv_choice_name(const ConvChoice& c, int dtype, int n, int ho, int wo, int cin_p, int cout_p) {
  static thread_local char buf[64];
  switch (c.kind) {
    case CK_TORGB: return "torgb";
    case CK_HCONV:
      snprintf(buf, sizeof(buf), "hconv_%d_%d", cin_p, cout_p);
      return buf;
    case CK_HG4: {
      const H4Plan p = h4_plan(n, ho, wo, cout_p);
      snprintf(buf, sizeof(buf), "hg4_o%d_w%s", p.bo, !p.tw32 ? "16_s4" : p.bo == 64 ? "32_p3" : "32_p2");
      return buf;
    }
    default: break;
  }
  if (dtype == IC2_F32) {
    snprintf(buf, sizeof(buf), "igemm_f32_128x128%s", c.pl.splits > 1 ? "_splitk" : "");
    return buf;
  }
  if (c.pl.tile == 6) return c.pl.splits > 1 ? "igemm8_og2_splitk" : c.pl.tail ? "igemm8_og2_tail" : "igemm8_og2";
  if (c.pl.tile == 7) return c.split384 ? "igemm8_og2+og1" : "igemm8_og1";
  snprintf(buf, sizeof(buf), "igemm_%dx%d%s", c.pl.bo, c.pl.bp, c.pl.splits > 1 ? "_splitk" : "");
  return buf;
}

// Images per launch: the buffer-descriptor kernels (8-phase, hg4) address < 2^31 bytes per operand, so a batch whose
// input exceeds that runs in chunks of whole images (each chunk with its own launch plan) instead of falling back to
// the generic tile (SG3-T-1024 / the 1024^2 encoder at batch 8: 1024^2 x 192 x 2 B = 403 MB per image).
static int conv_chunk_n(int dtype, int n, int h, int w_, int cin_p) {
  const int64_t per_img = (int64_t)h * w_ * x_pix_of(dtype, cin_p) * (dtype == IC2_F32 ? 4 : 2);
  if ((int64_t)n * per_img < (int64_t)kOob || per_img >= (int64_t)kOob) return n;
  const int64_t c = ((int64_t)kOob - 1) / per_img;
  const int64_t chunks = ceil_div(n, c);
  return (int)ceil_div(n, chunks);  // balanced chunks
}

}  // namespace ic2

using namespace ic2;

extern "C" const char* ic2_conv_plan(int dtype, int out_dtype, int out_layout, int n, int h, int w_, int cin_p,
                                     int cout_p, int cout_valid, int kh, int kw, int pad) {
  const int ho = h + 2 * pad - kh + 1, wo = w_ + 2 * pad - kw + 1;
  if (n <= 0 || ho <= 0 || wo <= 0 || cin_p <= 0 || cout_p <= 0) return "invalid";
  const int nc = conv_chunk_n(dtype, n, h, w_, cin_p);
  const ConvChoice c = conv_choice(dtype, out_layout, out_dtype, nc, h, w_, cin_p, cout_p, cout_valid, kh, kw, pad);
  const char* name = conv_choice_name(c, dtype, nc, ho, wo, cin_p, cout_p);
  if (dtype != IC2_F16 && dtype != IC2_F16X2) return name;
  static thread_local char f16_name[80];  // the f16-operand instance of the same kernel
  snprintf(f16_name, sizeof(f16_name), "%s_f16", name);
  return f16_name;
}

extern "C" int64_t ic2_conv_igemm_ws_bytes(int dtype, int n, int h, int w_, int cin_p, int cout_p, int kh, int kw,
                                           int pad) {
  const int ho = h + 2 * pad - kh + 1, wo = w_ + 2 * pad - kw + 1;
  if (n <= 0 || h <= 0 || w_ <= 0 || ho <= 0 || wo <= 0 || cin_p <= 0 || cout_p <= 0 || kh <= 0 || kw <= 0) return 0;
  const int nc = conv_chunk_n(dtype, n, h, w_, cin_p);
  const ConvChoice c = conv_choice(dtype, IC2_LAYOUT_NHWC, dtype, nc, h, w_, cin_p, cout_p, cout_p, kh, kw, pad);
  if (c.kind != CK_IGEMM || (c.pl.splits == 1 && !c.pl.tail)) return 0;
  return (int64_t)(c.pl.tail ? 2 : c.pl.splits) * nc * ho * wo * cout_p * 4;
}

extern "C" int ic2_conv_igemm_ws(const void* x, const void* w, void* y, int dtype, int out_dtype, int n, int h, int w_,
                                 int cin_p, int cout_p, int cout_valid, int kh, int kw, int pad, int ho, int wo,
                                 const float* oscale, const float* bias, int act, float slope, float act_gain,
                                 float clamp, float out_mul, int out_layout, void* workspace, int64_t ws_bytes,
                                 void* stream) {
  IC2_CHECK_ARG(x && w && y, "conv_igemm: null pointer");
  IC2_CHECK_ARG(dtype == IC2_F32 || dtype == IC2_BF16 || dtype == IC2_F16 || dtype == IC2_BF16X3 || dtype == IC2_F16X2,
                "conv_igemm: bad dtype %d", dtype);
  IC2_CHECK_ARG(dtype != IC2_BF16X3 || (cin_p % 96 == 0 && out_layout == IC2_LAYOUT_NHWC),
                "conv_igemm: split-bf16 input needs cin_p = 3 x a multiple of 32 and NHWC output (cin_p=%d)", cin_p);
  IC2_CHECK_ARG(dtype != IC2_F16X2 || (cin_p % 64 == 0 && out_layout == IC2_LAYOUT_NHWC),
                "conv_igemm: split-weight f16 input needs cin_p = 2 x a multiple of 32 and NHWC output (cin_p=%d)", cin_p);
  IC2_CHECK_ARG(out_dtype == IC2_F32 || out_dtype == IC2_BF16 ||
                    ((out_dtype == IC2_F16 || out_dtype == IC2_F16_IEEE) && out_layout != IC2_LAYOUT_NCHW),
                "conv_igemm: bad out dtype %d", out_dtype);
  IC2_CHECK_ARG(cin_p > 0 && cin_p % 32 == 0 && cout_p > 0 && cout_p % 32 == 0,
                "conv_igemm: channel strides must be positive multiples of 32 (cin_p=%d cout_p=%d)", cin_p, cout_p);
  IC2_CHECK_ARG(n > 0 && h > 0 && w_ > 0 && kh > 0 && kw > 0 && pad >= 0, "conv_igemm: bad geometry");
  IC2_CHECK_ARG(ho == h + 2 * pad - kh + 1 && wo == w_ + 2 * pad - kw + 1,
                "conv_igemm: output size %dx%d does not match input %dx%d, k=%dx%d, pad=%d", ho, wo, h, w_, kh, kw, pad);
  IC2_CHECK_ARG(out_layout == IC2_LAYOUT_NHWC || out_layout == IC2_LAYOUT_NHWC16 ||
                    (out_layout == IC2_LAYOUT_NCHW && out_dtype == IC2_F32 && cout_valid > 0 && cout_valid <= cout_p),
                "conv_igemm: NCHW output needs f32 and 0 < cout_valid <= cout_p (layout %d)", out_layout);
  IC2_CHECK_ARG(((uintptr_t)oscale | (uintptr_t)bias | (uintptr_t)workspace) % 16 == 0,
                "conv_igemm: oscale/bias/workspace must be 16-byte aligned");
  const int nc = conv_chunk_n(dtype, n, h, w_, cin_p);
  if (nc < n) {
    const int64_t x_img = (int64_t)h * w_ * x_pix_of(dtype, cin_p) * (dtype == IC2_F32 ? 4 : 2);
    const int64_t y_img = out_layout == IC2_LAYOUT_NCHW ? (int64_t)cout_valid * ho * wo * 4
                                                        : (int64_t)ho * wo * cout_p * (out_dtype == IC2_F32 ? 4 : 2);
    for (int n0 = 0; n0 < n; n0 += nc) {
      const int nn = n - n0 < nc ? n - n0 : nc;
      const int rc = ic2_conv_igemm_ws(reinterpret_cast<const char*>(x) + n0 * x_img, w,
                                       reinterpret_cast<char*>(y) + n0 * y_img, dtype, out_dtype, nn, h, w_, cin_p,
                                       cout_p, cout_valid, kh, kw, pad, ho, wo,
                                       oscale ? oscale + (int64_t)n0 * cout_p : nullptr, bias, act, slope, act_gain,
                                       clamp, out_mul, out_layout, workspace, ws_bytes, stream);
      if (rc != IC2_OK) return rc;
    }
    return IC2_OK;
  }
  const int64_t M = (int64_t)n * ho * wo;
  IC2_CHECK_ARG(M < (1LL << 30), "conv_igemm: too many output pixels");
  const int out_ieee = out_dtype == IC2_F16_IEEE;
  if (out_ieee) out_dtype = IC2_F16;
  IgemmArgs a;
  a.x = x; a.w = w; a.y = y; a.oscale = oscale; a.bias = bias; a.ws = reinterpret_cast<float*>(workspace);
  a.n = n; a.h = h; a.w_ = w_; a.cin_p = cin_p; a.cout_p = cout_p; a.cout_valid = cout_valid;
  a.kh = kh; a.kw = kw; a.pad = pad; a.ho = ho; a.wo = wo;
  a.M = (int)M; a.K = kh * kw * cin_p; a.nq = a.K / 32;
  a.act = act; a.slope = slope; a.act_gain = act_gain; a.clamp = clamp; a.out_mul = out_mul;
  a.out_layout = out_layout; a.out_dtype = out_dtype; a.out_ieee = out_ieee;
  a.gn_part = nullptr; a.gn_groups = 0; a.gn_c = 0;
  a.in_gn = nullptr; a.in_slope = 0.f;
  a.x_pix = x_pix_of(dtype, cin_p);
  a.x_hb32 = x_hb32_of(dtype, cin_p);
  const int kdt = dtype == IC2_BF16X3 ? IC2_BF16 : dtype == IC2_F16X2 ? IC2_F16 : dtype;  // the kernels' operand type
  static const int group = [] {
    const int g = knob("IC2_IGEMM_GROUP", 1);  // 1 = o-tiles of a p-tile side by side (measured best)
    return g >= 1 ? g : 1;
  }();
  a.group = group;
  // channel-major K order: s148 +3 %, s148b +5 %, s148c +7 %, C2 +2.6 % (profiles/r2f_korder.txt)
  static const int korder = knob("IC2_IGEMM_KORDER", 1);
  a.korder = korder;
  a.o_base = 0;
  hipStream_t s = as_stream(stream);
  ConvChoice c = conv_choice(dtype, out_layout, out_dtype, n, h, w_, cin_p, cout_p, cout_valid, kh, kw, pad);
  dtype = kdt;
  IgPlan& pl = c.pl;
  if (pl.splits > 1 && (workspace == nullptr || ws_bytes < (int64_t)pl.splits * M * cout_p * 4)) pl.splits = 1;
  if (pl.tail && (workspace == nullptr || ws_bytes < 2 * M * cout_p * 4 || a.group != 1)) pl.tail = 0;
  switch (c.kind) {
    case CK_TORGB:
      if (dtype == IC2_F16) launch_torgb<true>(a, s);
      else launch_torgb<false>(a, s);
      break;
    case CK_HG4: hg4_dispatch(a, s, dtype == IC2_F16); break;
    case CK_HCONV:
      if (dtype == IC2_F16) launch_hconv_cfg<true>(a, s, cin_p, cout_p);
      else launch_hconv_cfg<false>(a, s, cin_p, cout_p);
      break;
    case CK_IGEMM:
      if (dtype == IC2_F32) launch_igemm<false, 128, 128, 2, 2, 2>(a, pl.splits, s);
      else if (dtype == IC2_F16) launch_igemm16<true>(a, s, pl, c.split384, cout_p);
      else launch_igemm16<false>(a, s, pl, c.split384, cout_p);
      if (pl.splits > 1 || pl.tail) {
        // the tail's pixels: its first tile's p-tile (tiles are p-tile major at group 1) times 256
        const int p_lo = pl.tail ? g8_tail_first(M, cout_p) / ((cout_p + 255) / 256) * 256 : 0;
        const int64_t total = (M - p_lo) * (cout_p / 4);
        const int grid = (int)(ceil_div(total, 256) < 4096 ? ceil_div(total, 256) : 4096);
        hipLaunchKernelGGL(igemm_splitk_reduce_kernel, dim3(grid), dim3(256), 0, s, a, pl.tail ? 2 : pl.splits, p_lo);
      }
      break;
  }
  IC2_CHECK_LAUNCH("conv_igemm");
  return IC2_OK;
}

namespace ic2 {
// conv (bias only, NHWC bf16 out) with the GroupNorm partial sums fused into the halo conv's epilogue when that
// kernel is the one the dispatcher picks.  Returns the number of per-image chunks written to `part`
// ([n][groups][chunks][2] f64), 0 when the conv ran unfused (the caller then computes the statistics itself),
// or -1 on an argument error (message set).
bool conv_gn_in_supported(int dtype, int n, int h, int w_, int cin_p, int cout_p, int kh, int kw, int pad) {
  const int ho = h + 2 * pad - kh + 1, wo = w_ + 2 * pad - kw + 1;
  if (dtype != IC2_BF16 || cin_p != 64 || ho <= 0 || wo <= 0) return false;
  return hconv_eligible(dtype, (int64_t)n * ho * wo, cin_p, cout_p, kh, kw);
}

static int conv_chunk_n(int dtype, int n, int h, int w_, int cin_p);

// split-bf16 (IC2_BF16X3) / split-weight f16 (IC2_F16X2) conv with f32 output: the hg4 instance the plan picks (per chunk of images, as
// ic2_conv_igemm_ws launches it) carries the statistics in its epilogue when it is a 32-wide-tile o64 / o128 kernel
// over exactly 32 groups of 2 / 4 channels
static bool x3_gn_hg4(int dtype, int n, int h, int w_, int cin_p, int cout_p, int cout_valid, int kh, int kw, int pad,
                      int groups, H4Plan* plan) {
  const int ho = h + 2 * pad - kh + 1, wo = w_ + 2 * pad - kw + 1;
  if (ho <= 0 || wo <= 0 || groups != 32 || cout_valid != cout_p || (cout_p != 64 && cout_p != 128)) return false;
  const int nc = conv_chunk_n(dtype, n, h, w_, cin_p);
  const ConvChoice c = conv_choice(dtype, IC2_LAYOUT_NHWC, IC2_F32, nc, h, w_, cin_p, cout_p, cout_valid, kh, kw, pad);
  if (c.kind != CK_HG4) return false;
  const H4Plan p = h4_plan(nc, ho, wo, cout_p);
  if (!p.tw32 || p.bo != cout_p) return false;
  if (plan) *plan = p;
  return true;
}

// rows of the statistics-epilogue kernel's pixel tile: 12 for the 64-wide outputs (knob IC2_X3_GN_T12=0: 8), else 8
static int x3_gn_th(int cout_p) {
  static const bool t12 = knob("IC2_X3_GN_T12", 1) != 0;
  return cout_p == 64 && t12 ? 12 : 8;
}
static int64_t x3_gn_part_doubles(int dtype, int n, int h, int w_, int cin_p, int cout_p, int cout_valid, int kh, int kw,
                                  int pad, int groups) {
  if (!x3_gn_hg4(dtype, n, h, w_, cin_p, cout_p, cout_valid, kh, kw, pad, groups, nullptr)) return 0;
  const int ho = h + 2 * pad - kh + 1, wo = w_ + 2 * pad - kw + 1;
  return (int64_t)n * groups * ceil_div(wo, 32) * ceil_div(ho, x3_gn_th(cout_p)) * 2;  // the kernel's 32-wide tiles
}

bool conv_gn_fuses(int dtype, int n, int h, int w_, int cin_p, int cout_p, int cout_valid, int kh, int kw, int pad,
                   int groups, int fuse_mode) {
  static const bool x3_env = knob("IC2_X3_GN", 1) == 1;  // A/B: 0 = the separate statistics pass by default
  if (dtype == IC2_BF16X3 || dtype == IC2_F16X2)
    return (fuse_mode > 0 || (fuse_mode < 0 && x3_env)) &&
           x3_gn_hg4(dtype, n, h, w_, cin_p, cout_p, cout_valid, kh, kw, pad, groups, nullptr);
  const int ho = h + 2 * pad - kh + 1, wo = w_ + 2 * pad - kw + 1;
  if (ho <= 0 || wo <= 0) return false;
  static const bool fuse_env = knob("IC2_CONV_GN", 0) == 1;
  const bool fuse_req = fuse_mode < 0 ? fuse_env : fuse_mode > 0;
  // the statistics epilogue exists for the bf16 halo conv only (hconv_eligible also admits f16 operands)
  return fuse_req && dtype == IC2_BF16 && hconv_eligible(dtype, (int64_t)n * ho * wo, cin_p, cout_p, kh, kw) &&
         groups == 32 && cout_valid == cout_p;
}

int conv_gn_fused(const void* x, const void* w, void* y, int dtype, int n, int h, int w_, int cin_p, int cout_p,
                  int cout_valid, int kh, int kw, int pad, const float* bias, int groups, double* part,
                  int64_t part_doubles, void* workspace, int64_t ws_bytes, int fuse_mode, hipStream_t s,
                  const float* in_gn, float in_slope, float out_mul) {
  const int ho = h + 2 * pad - kh + 1, wo = w_ + 2 * pad - kw + 1;
  const int64_t M = (int64_t)n * ho * wo;
  if (dtype == IC2_BF16X3 || dtype == IC2_F16X2) {
    // default on: the statistics epilogue of the non-persistent hg4 costs less than the separate f32 pass saves.
    // Output f32 (split bf16) / f16 (split-weight f16: its consumer's operand is f16 anyway)
    const int ydt = dtype == IC2_F16X2 ? IC2_F16 : IC2_F32;
    H4Plan p;
    const bool fuse = conv_gn_fuses(dtype, n, h, w_, cin_p, cout_p, cout_valid, kh, kw, pad, groups, fuse_mode) &&
                      in_gn == nullptr && bias != nullptr && part != nullptr &&
                      x3_gn_hg4(dtype, n, h, w_, cin_p, cout_p, cout_valid, kh, kw, pad, groups, &p) &&
                      part_doubles >= x3_gn_part_doubles(dtype, n, h, w_, cin_p, cout_p, cout_valid, kh, kw, pad, groups);
    if (in_gn != nullptr) {
      set_error("conv3x3_gnin_gn_fwd: no input GroupNorm fusion in the split modes");
      return -2;
    }
    if (!fuse) {
      const int rc = ic2_conv_igemm_ws(x, w, y, dtype, ydt, n, h, w_, cin_p, cout_p, cout_valid, kh, kw, pad, ho, wo,
                                       nullptr, bias, 0, 0.f, 1.f, -1.f, out_mul, IC2_LAYOUT_NHWC, workspace,
                                       ws_bytes, s);
      return rc == IC2_OK ? 0 : -1;
    }
    IgemmArgs a;
    a.x = x; a.w = w; a.y = y; a.oscale = nullptr; a.bias = bias; a.ws = nullptr;
    a.n = n; a.h = h; a.w_ = w_; a.cin_p = cin_p; a.cout_p = cout_p; a.cout_valid = cout_valid;
    a.kh = kh; a.kw = kw; a.pad = pad; a.ho = ho; a.wo = wo;
    a.M = (int)M; a.K = kh * kw * cin_p; a.nq = a.K / 32;
    a.act = 0; a.slope = 0.f; a.act_gain = 1.f; a.clamp = -1.f; a.out_mul = out_mul;
    a.out_layout = IC2_LAYOUT_NHWC; a.out_dtype = ydt; a.out_ieee = 0;
    a.gn_part = part; a.gn_groups = groups; a.gn_c = cout_valid;
    a.group = 1; a.korder = 0; a.o_base = 0;
    a.in_gn = nullptr; a.in_slope = 0.f;
    a.x_pix = x_pix_of(dtype, cin_p);
    a.x_hb32 = x_hb32_of(dtype, cin_p);
    const bool f16 = dtype == IC2_F16X2;
    const int nc = conv_chunk_n(dtype, n, h, w_, cin_p);
    const int64_t ntile = ceil_div(wo, 32) * ceil_div(ho, x3_gn_th(cout_p));
    for (int i0 = 0; i0 < n; i0 += nc) {  // chunks of whole images (< 2^31 input bytes per launch)
      const int cnt = n - i0 < nc ? n - i0 : nc;
      a.x = reinterpret_cast<const char*>(x) + (int64_t)i0 * h * w_ * a.x_pix * 2;
      a.y = reinterpret_cast<char*>(y) + (int64_t)i0 * ho * wo * cout_p * (ydt == IC2_F16 ? 2 : 4);
      a.gn_part = part + (int64_t)i0 * groups * ntile * 2;
      a.n = cnt;
      a.M = (int)((int64_t)cnt * ho * wo);
      if (p.bo == 64 && x3_gn_th(64) == 12)
        launch_hg4<4, 6, 1, 4, 32>(a, s, f16 ? hg4_o64_w32_t12_gn_kernel_f16 : hg4_o64_w32_t12_gn_kernel);
      else if (p.bo == 64) launch_hg4<4, 4, 1, 4, 32>(a, s, f16 ? hg4_o64_w32_p3_gn_kernel_f16 : hg4_o64_w32_p3_gn_kernel);
      else launch_hg4<8, 4, 1, 4, 32>(a, s, f16 ? hg4_o128_w32_p2_gn_kernel_f16 : hg4_o128_w32_p2_gn_kernel);
    }
    return (int)ntile;
  }
  const bool hconv = hconv_eligible(dtype, M, cin_p, cout_p, kh, kw);
  const int th = cin_p > 64 ? 4 : 8;
  const int64_t nch = ceil_div(wo, 32) * ceil_div(ho, th);
  // fused instances: 32 groups over all cout_p channels (VGGBlock: GroupNorm(min(32, c), c) with c = 32 / 64).
  // Off by default: measured on MI355X the epilogue reduction (two extra barriers per tile in the persistent
  // kernel) costs what the saved read of y gains -- C4 357.1 -> 356.7 img/s, C2 1277 -> 1256 (profiles/
  // r2b_conv_gn_ab.txt); knob IC2_CONV_GN=1 enables it.
  static const bool fuse_env = knob("IC2_CONV_GN", 0) == 1;
  const bool fuse_req = fuse_mode < 0 ? fuse_env : fuse_mode > 0;
  const bool fuse = fuse_req && hconv && dtype == IC2_BF16 && part != nullptr && part_doubles >= (int64_t)n * groups * nch * 2 &&
                    groups == 32 && cout_valid == cout_p && bias != nullptr;
  if (in_gn != nullptr && !conv_gn_in_supported(dtype, n, h, w_, cin_p, cout_p, kh, kw, pad)) {
    set_error("conv3x3_gn_fwd: input GroupNorm fusion needs the halo conv (bf16, cin_p 64)");
    return -2;
  }
  if (!fuse && in_gn == nullptr) {
    const int rc = ic2_conv_igemm_ws(x, w, y, dtype, dtype, n, h, w_, cin_p, cout_p, cout_valid, kh, kw, pad, ho, wo,
                                     nullptr, bias, 0, 0.f, 1.f, -1.f, 1.f, IC2_LAYOUT_NHWC, workspace, ws_bytes, s);
    return rc == IC2_OK ? 0 : -1;
  }
  IgemmArgs a;
  a.x = x; a.w = w; a.y = y; a.oscale = nullptr; a.bias = bias; a.ws = nullptr;
  a.n = n; a.h = h; a.w_ = w_; a.cin_p = cin_p; a.cout_p = cout_p; a.cout_valid = cout_valid;
  a.kh = kh; a.kw = kw; a.pad = pad; a.ho = ho; a.wo = wo;
  a.M = (int)M; a.K = kh * kw * cin_p; a.nq = a.K / 32;
  a.act = 0; a.slope = 0.f; a.act_gain = 1.f; a.clamp = -1.f; a.out_mul = 1.f;
  a.out_layout = IC2_LAYOUT_NHWC; a.out_dtype = dtype; a.out_ieee = 0;
  a.gn_part = fuse ? part : nullptr; a.gn_groups = groups; a.gn_c = cout_valid;
  a.group = 1;
  a.korder = 0;
  a.o_base = 0;
  a.in_gn = in_gn; a.in_slope = in_slope;
  a.x_pix = cin_p; a.x_hb32 = 0;
  if (fuse) {
    if (cin_p == 32 && cout_p == 32) launch_hconv<32, 32, true>(a, s);
    else if (cin_p == 32) launch_hconv<32, 64, true>(a, s);
    else if (cin_p == 64 && cout_p == 32) launch_hconv<64, 32, true>(a, s);
    else if (cin_p == 64) launch_hconv<64, 64, true>(a, s);
    else if (cout_p == 32) launch_hconv<96, 32, true>(a, s);
    else launch_hconv<96, 64, true>(a, s);
    return (int)nch;
  }
  if (cin_p == 32 && cout_p == 32) launch_hconv<32, 32>(a, s);
  else if (cin_p == 32) launch_hconv<32, 64>(a, s);
  else if (cin_p == 64 && cout_p == 32) launch_hconv<64, 32>(a, s);
  else launch_hconv<64, 64>(a, s);
  return 0;
}

int64_t conv_gn_fused_part_doubles(int dtype, int n, int h, int w_, int cin_p, int cout_p, int kh, int kw, int pad,
                                   int groups) {
  if (dtype == IC2_BF16X3 || dtype == IC2_F16X2)
    return x3_gn_part_doubles(dtype, n, h, w_, cin_p, cout_p, cout_p, kh, kw, pad, groups);
  const int ho = h + 2 * pad - kh + 1, wo = w_ + 2 * pad - kw + 1;
  if (dtype != IC2_BF16 || !hconv_eligible(dtype, (int64_t)n * ho * wo, cin_p, cout_p, kh, kw)) return 0;
  const int th = cin_p > 64 ? 4 : 8;
  return (int64_t)n * groups * ceil_div(wo, 32) * ceil_div(ho, th) * 2;
}
}  // namespace ic2

extern "C" int ic2_conv_igemm(const void* x, const void* w, void* y, int dtype, int out_dtype, int n, int h, int w_,
                              int cin_p, int cout_p, int cout_valid, int kh, int kw, int pad, int ho, int wo,
                              const float* oscale, const float* bias, int act, float slope, float act_gain,
                              float clamp, float out_mul, int out_layout, void* stream) {
  return ic2_conv_igemm_ws(x, w, y, dtype, out_dtype, n, h, w_, cin_p, cout_p, cout_valid, kh, kw, pad, ho, wo, oscale,
                           bias, act, slope, act_gain, clamp, out_mul, out_layout, nullptr, 0, stream);
}
