// Backward kernels of the training path (BASELINE config C5): the reference trains
// HVAE_VGG_Encoder through torch autograd (stylegan3_hvae_full.py:655-707: recon / KL losses, backward at
// :693-696).  The encoder's hot ops get hand-written backward kernels here; the 3x3 conv's input gradient
// is the forward implicit GEMM on flipped / transposed weights (ic2_conv_igemm), so only the weight
// gradient and the GroupNorm + lrelu + avg-pool backward are new.
//
//   ic2_conv_wgrad : dW[o][ky][kx][i] = sum_p dy[p][o] * x[p shifted by (ky, kx)][i]  (MFMA; K = pixels)
//   ic2_gn_lrelu_pool_bwd : d(AvgPool2(lrelu(GroupNorm(y)))) / dy, dgamma, dbeta
//   ic2_gap_bwd : d(mean over H x W) / dx  (the HierarchyProjector's AdaptiveAvgPool2d(1))
#include "common.h"

#include <type_traits>

namespace ic2 {

typedef __attribute__((ext_vector_type(8))) __bf16 wg_bf16x8;
typedef __attribute__((ext_vector_type(8))) _Float16 wg_f16x8;
typedef _Float16 bw_h2 __attribute__((ext_vector_type(2)));
typedef __attribute__((ext_vector_type(4))) float wg_f32x4;
typedef short wg_s4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------------------------------------
// weight gradient as a GEMM over pixels: C[o][j] (j = one tap's 64 input channels) = sum_p A[o][p] B[p][j],
// A = dy^T, B = the tap-shifted input.  Both operands are pixel-major in HBM (NHWC), so a 32-pixel chunk of
// each is staged row-per-pixel in LDS and the MFMA fragments (8 consecutive pixels of one column) are read
// with the transposing ds_read_b64_tr_b16 (two per fragment).  Tile 64 (o) x 64 (j) x 32 (p), 4 waves of
// 32 x 32; the pixels are split over gridDim.y into f32 partial slabs summed in slice order by
// wgrad_reduce_kernel (deterministic).  f32 operands: 16x16x4 f32 MFMAs on plain LDS reads.
constexpr int WG_BO = 64, WG_BJ = 64, WG_KP = 32;
constexpr int WG_PITCH = WG_BO + 8;  // LDS row pitch (elements)

struct WgradArgs {
  const void* x;
  const void* dy;
  float* part;  // [splits][cout_p][kh*kw][cin_p]
  int n, h, w, cin_p, cout_p, kh, kw, pad, ho, wo;
  int P;        // n * ho * wo
  int chunks;   // ceil(P / 32)
  int j_tiles;  // kh * kw * cin_p / 64
};

__device__ __forceinline__ wg_s4 wg_tr_read(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) wg_s4*)p);
}

template <typename T>
__global__ void __launch_bounds__(256) wgrad_kernel(WgradArgs a) {
  __shared__ __attribute__((aligned(16))) T sdy[WG_KP * WG_PITCH];
  __shared__ __attribute__((aligned(16))) T sx[WG_KP * WG_PITCH];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int o_tiles = (a.cout_p + WG_BO - 1) / WG_BO;  // channel strides are multiples of 32: a 32-wide tail
  const int o0 = (blockIdx.x % o_tiles) * WG_BO;       // tile reads zeros and stores nothing past the stride
  const int jt = blockIdx.x / o_tiles;                 // j tile: tap = jt / ceil(cin_p/64), ci block
  const int cib = (a.cin_p + WG_BJ - 1) / WG_BJ;
  const int tap = jt / cib, ci0 = (jt - tap * cib) * WG_BJ;
  const int ky = tap / a.kw, kx = tap - (tap / a.kw) * a.kw;
  const int c0 = (int)((int64_t)a.chunks * blockIdx.y / gridDim.y);
  const int c1 = (int)((int64_t)a.chunks * (blockIdx.y + 1) / gridDim.y);
  const int wo_ = wave >> 1, wj_ = wave & 1;           // this wave's 32 x 32 sub-tile
  const T* dyg = reinterpret_cast<const T*>(a.dy);
  const T* xg = reinterpret_cast<const T*>(a.x);
  // staging: thread -> (pixel row r = tid / 8, 8-element segment s = tid % 8) of each operand
  const int r = tid >> 3, seg = tid & 7;
  const int hwo = a.ho * a.wo;

  wg_f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = wg_f32x4{0.f, 0.f, 0.f, 0.f};

  // the next chunk's rows are loaded into registers while this chunk's MFMAs run (the loop was one exposed global
  // load round trip per 32 pixels)
  constexpr int NV = sizeof(T) / 2;  // 16-B registers per 8-element row segment
  uint4 vd[NV], vx[NV];
  auto load_chunk = [&](int ch) {
    const int p = ch * WG_KP + r;
    const bool okp = p < a.P;
    const int pp = okp ? p : 0;
    const int nn = pp / hwo;
    const int rem = pp - nn * hwo;
    const int oy = rem / a.wo, ox = rem - (rem / a.wo) * a.wo;
    const int iy = oy - a.pad + ky, ix = ox - a.pad + kx;
    const bool okx = okp && (unsigned)iy < (unsigned)a.h && (unsigned)ix < (unsigned)a.w;
    const bool oko = okp && o0 + seg * 8 < a.cout_p, oki = okx && ci0 + seg * 8 < a.cin_p;
    const uint4* sd = reinterpret_cast<const uint4*>(dyg + (int64_t)pp * a.cout_p + (oko ? o0 + seg * 8 : 0));
    const uint4* sxp = reinterpret_cast<const uint4*>(
        xg + (((int64_t)nn * a.h + (okx ? iy : 0)) * a.w + (okx ? ix : 0)) * a.cin_p + (oki ? ci0 + seg * 8 : 0));
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      vd[v] = oko ? sd[v] : make_uint4(0u, 0u, 0u, 0u);
      vx[v] = oki ? sxp[v] : make_uint4(0u, 0u, 0u, 0u);
    }
  };
  if (c0 < c1) load_chunk(c0);
  for (int ch = c0; ch < c1; ++ch) {
    __syncthreads();  // previous chunk's fragment reads done
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      reinterpret_cast<uint4*>(sdy + r * WG_PITCH + seg * 8)[v] = vd[v];
      reinterpret_cast<uint4*>(sx + r * WG_PITCH + seg * 8)[v] = vx[v];
    }
    __syncthreads();
    if (ch + 1 < c1) load_chunk(ch + 1);
    if constexpr (sizeof(T) == 2) {
      // A[m = o][k = p]: lane (g, li) = pixels 8g .. 8g+7 of column o; two transposed reads of 4 rows each.
      // Within a 16-lane group, lane (tq = li / 4, tp = li % 4) reads row base + tq, elements 4 tp .. 4 tp + 3.
      const int tq = li >> 2, tp = li & 3;
      wg_bf16x8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int col = wo_ * 32 + i * 16 + 4 * tp;
        const wg_s4 lo = wg_tr_read(reinterpret_cast<const bf16_t*>(sdy) + (8 * g + tq) * WG_PITCH + col);
        const wg_s4 hi = wg_tr_read(reinterpret_cast<const bf16_t*>(sdy) + (8 * g + 4 + tq) * WG_PITCH + col);
        af[i] = __builtin_bit_cast(wg_bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = wj_ * 32 + j * 16 + 4 * tp;
        const wg_s4 lo = wg_tr_read(reinterpret_cast<const bf16_t*>(sx) + (8 * g + tq) * WG_PITCH + col);
        const wg_s4 hi = wg_tr_read(reinterpret_cast<const bf16_t*>(sx) + (8 * g + 4 + tq) * WG_PITCH + col);
        bfr[j] = __builtin_bit_cast(wg_bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          if constexpr (std::is_same<T, _Float16>::value)   // the f16 training path: f16 operands, same fragments
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(wg_f16x8, af[i]),
                                                               __builtin_bit_cast(wg_f16x8, bfr[j]), acc[i][j], 0, 0, 0);
          else
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        }
    } else {
      // f32: 16x16x4 MFMA, lane (g, li) holds A[m = li][k = g] / B[k = g][n = li] per 4-pixel step (exact fp32)
      const float* fdy = reinterpret_cast<const float*>(sdy);
      const float* fx = reinterpret_cast<const float*>(sx);
#pragma unroll
      for (int s = 0; s < WG_KP / 4; ++s) {
        float av[2], bv[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) av[i] = fdy[(4 * s + g) * WG_PITCH + wo_ * 32 + i * 16 + li];
#pragma unroll
        for (int j = 0; j < 2; ++j) bv[j] = fx[(4 * s + g) * WG_PITCH + wj_ * 32 + j * 16 + li];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bv[j], acc[i][j], 0, 0, 0);
      }
    }
  }
  // C[o = o0 + 32 wo + 16 i + 4 g + rr][j = ci0 + 32 wj + 16 jj + li] -> part[split][o][tap][ci]
  const int K = a.kh * a.kw * a.cin_p;
  float* dst = a.part + (int64_t)blockIdx.y * a.cout_p * K;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int o = o0 + wo_ * 32 + i * 16 + 4 * g + rr;
        const int ci = ci0 + wj_ * 32 + j * 16 + li;
        if (o < a.cout_p && ci < a.cin_p) dst[(int64_t)o * K + tap * a.cin_p + ci] = acc[i][j][rr];
      }
}

__global__ void __launch_bounds__(256) wgrad_reduce_kernel(const float* __restrict__ part, float* __restrict__ dw,
                                                           int64_t total, int splits) {
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    float s = part[e];
    for (int k = 1; k < splits; ++k) s += part[(int64_t)k * total + e];
    dw[e] = s;
  }
}
// the same sums written in nn.Conv2d's weight layout [cout][cin][kh][kw] (valid channels only): the parameter's
// gradient without a slice + permute copy
__global__ void __launch_bounds__(256) wgrad_reduce_oihw_kernel(const float* __restrict__ part, float* __restrict__ dw,
                                                                int64_t total, int splits, int cin_p, int taps,
                                                                int cout, int cin) {
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int i = (int)(e % cin_p);
    const int64_t ot = e / cin_p;
    const int t = (int)(ot % taps), o = (int)(ot / taps);
    if (o >= cout || i >= cin) continue;
    float s = part[e];
    for (int k = 1; k < splits; ++k) s += part[(int64_t)k * total + e];
    dw[((int64_t)o * cin + i) * taps + t] = s;
  }
}

// ------------------------------------------------------------------------------------------------
// Weight gradient, 16-bit operands (round 4): the same GEMM over pixels with KP-pixel stages, double-buffered LDS
// (one barrier per stage instead of two per 32 pixels) and the j axis flattened over (tap, input channel), so a
// j tile of a 32-channel input covers several taps instead of reading a zero half.  Tile BT (o) x BT (j), 4 waves of
// BT/2 x BT/2 (BT 64: 4 MFMAs 16x16x32 per 8 transposed fragment reads per k-step; BT 128: 16 per 16, for the
// >= 128-channel layers); the next stage's rows are loaded into registers while the current one is computed.
template <typename T, int KP, int BT>
__global__ void __launch_bounds__(256) wgrad2_kernel(WgradArgs a) {
  static_assert(sizeof(T) == 2, "16-bit operands");
  constexpr int PITCH = BT + 8;          // LDS row pitch (elements)
  constexpr int STAGE = KP * PITCH;      // elements per operand and stage
  constexpr int SEGS = BT / 8;           // 16-B segments per staged row
  constexpr int RPP = 256 / SEGS;        // rows per staging pass
  constexpr int NQ = KP / RPP;           // staged rows per thread and operand
  constexpr int FI = BT / 32;            // 16-wide fragments per wave and operand
  static_assert(KP % RPP == 0 && KP % 32 == 0, "stage geometry");
  __shared__ __attribute__((aligned(16))) T lds[2][2][STAGE];  // [stage buffer][dy | x]
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int tq = li >> 2, tp = li & 3;
  const int o_tiles = (a.cout_p + BT - 1) / BT;
  const int o0 = (blockIdx.x % o_tiles) * BT;
  const int j0 = (blockIdx.x / o_tiles) * BT;  // flattened j = tap * cin_p + ci
  const int K = a.kh * a.kw * a.cin_p;
  const int c0 = (int)((int64_t)a.chunks * blockIdx.y / gridDim.y);
  const int c1 = (int)((int64_t)a.chunks * (blockIdx.y + 1) / gridDim.y);
  const int wo_ = wave >> 1, wj_ = wave & 1;
  const T* dyg = reinterpret_cast<const T*>(a.dy);
  const T* xg = reinterpret_cast<const T*>(a.x);
  const int hwo = a.ho * a.wo;
  // staging: thread -> 8-element segment seg of rows r0 + RPP q (q < NQ); the segment's j (tap, channel) is fixed
  const int r0 = tid / SEGS, seg = tid % SEGS;
  const int jseg = j0 + seg * 8;
  const bool jok = jseg < K;
  const int tap = jok ? jseg / a.cin_p : 0;
  const int ci = jseg - tap * a.cin_p;
  const int ky = tap / a.kw, kx = tap - (tap / a.kw) * a.kw;
  const bool ook = o0 + seg * 8 < a.cout_p;

  wg_f32x4 acc[FI][FI];
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FI; ++j) acc[i][j] = wg_f32x4{0.f, 0.f, 0.f, 0.f};

  uint4 vd[NQ], vx[NQ];
  auto load_stage = [&](int ch) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int p = ch * KP + r0 + RPP * q;
      const bool okp = p < a.P;
      const int pp = okp ? p : 0;
      const int nn = pp / hwo;
      const int rem = pp - nn * hwo;
      const int oy = rem / a.wo, ox = rem - (rem / a.wo) * a.wo;
      const int iy = oy - a.pad + ky, ix = ox - a.pad + kx;
      const bool okx = okp && jok && (unsigned)iy < (unsigned)a.h && (unsigned)ix < (unsigned)a.w;
      vd[q] = (okp && ook) ? *reinterpret_cast<const uint4*>(dyg + (int64_t)pp * a.cout_p + o0 + seg * 8)
                           : make_uint4(0u, 0u, 0u, 0u);
      vx[q] = okx ? *reinterpret_cast<const uint4*>(xg + (((int64_t)nn * a.h + iy) * a.w + ix) * a.cin_p + ci)
                  : make_uint4(0u, 0u, 0u, 0u);
    }
  };
  auto store_stage = [&](int buf) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      *reinterpret_cast<uint4*>(&lds[buf][0][(r0 + RPP * q) * PITCH + seg * 8]) = vd[q];
      *reinterpret_cast<uint4*>(&lds[buf][1][(r0 + RPP * q) * PITCH + seg * 8]) = vx[q];
    }
  };
  if (c0 < c1) {
    load_stage(c0);
    store_stage(0);
    __syncthreads();
    if (c0 + 1 < c1) load_stage(c0 + 1);
  }
  for (int ch = c0; ch < c1; ++ch) {
    const int buf = (ch - c0) & 1;
    const bf16_t* sdy = reinterpret_cast<const bf16_t*>(lds[buf][0]);
    const bf16_t* sx = reinterpret_cast<const bf16_t*>(lds[buf][1]);
#pragma unroll
    for (int ks = 0; ks < KP / 32; ++ks) {
      wg_bf16x8 af[FI], bfr[FI];
#pragma unroll
      for (int i = 0; i < FI; ++i) {
        const int col = wo_ * (BT / 2) + i * 16 + 4 * tp;
        const wg_s4 lo = wg_tr_read(sdy + (32 * ks + 8 * g + tq) * PITCH + col);
        const wg_s4 hi = wg_tr_read(sdy + (32 * ks + 8 * g + 4 + tq) * PITCH + col);
        af[i] = __builtin_bit_cast(wg_bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int j = 0; j < FI; ++j) {
        const int col = wj_ * (BT / 2) + j * 16 + 4 * tp;
        const wg_s4 lo = wg_tr_read(sx + (32 * ks + 8 * g + tq) * PITCH + col);
        const wg_s4 hi = wg_tr_read(sx + (32 * ks + 8 * g + 4 + tq) * PITCH + col);
        bfr[j] = __builtin_bit_cast(wg_bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < FI; ++j) {
          if constexpr (std::is_same<T, _Float16>::value)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(wg_f16x8, af[i]),
                                                               __builtin_bit_cast(wg_f16x8, bfr[j]), acc[i][j], 0, 0, 0);
          else
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        }
    }
    // the other buffer's last readers (stage ch-1) passed the barrier ending that stage
    if (ch + 1 < c1) store_stage(buf ^ 1);
    __syncthreads();
    if (ch + 2 < c1) load_stage(ch + 2);
  }
  float* dst = a.part + (int64_t)blockIdx.y * a.cout_p * K;
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FI; ++j)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int o = o0 + wo_ * (BT / 2) + i * 16 + 4 * g + rr;
        const int jj = j0 + wj_ * (BT / 2) + j * 16 + li;
        if (o < a.cout_p && jj < K) dst[(int64_t)o * K + jj] = acc[i][j][rr];
      }
}

static int wgrad_splits(const WgradArgs& a) {
  const int64_t tiles = ceil_div(a.cout_p, WG_BO) * a.j_tiles;
  int64_t sp = ceil_div(4096, tiles);  // ~16 workgroups per CU: the shallow layers have only 9-18 tiles
  if (sp > a.chunks) sp = a.chunks;
  if (sp > 256) sp = 256;
  return (int)(sp < 1 ? 1 : sp);
}

// wgrad2_kernel's plan: bt x bt tiles, j over the flattened (tap, channel) axis, kp-pixel stages, `target`
// workgroups with at least 4 stages each.  The 128-wide tile where both the output and the j extent fill it.
// (128 only under knob IC2_WGRAD2=3: over the encoder's layers it measured 2.4 % slower than 64 everywhere,
// profiles/r4p_wgrad_layers.txt)
static int wgrad2_tile(int cout_p, int K) { return cout_p >= 128 && K >= 128 ? 128 : 64; }
static int wgrad2_splits(const WgradArgs& a, int kp = 64, int target = 4096, int bt = 64) {
  const int64_t tiles = ceil_div(a.cout_p, bt) * ceil_div((int64_t)a.kh * a.kw * a.cin_p, bt);
  const int64_t chunks = ceil_div(a.P, kp);
  int64_t sp = ceil_div(target, tiles);
  if (sp > chunks / 4) sp = chunks / 4;
  if (sp > 256) sp = 256;
  return (int)(sp < 1 ? 1 : sp);
}

// ------------------------------------------------------------------------------------------------
// GroupNorm + lrelu (+ 2x2 avg-pool) backward.  Forward (ic2_group_norm_stats + ic2_gn_lrelu_pool):
//   xhat = (y - mean[n,g]) rstd[n,g],  z = gamma xhat + beta,  a = lrelu(z),  out = pool ? avgpool2(a) : a.
// Given dout: da = pool ? dout[h/2, w/2] / 4 (0 on a floor-dropped odd row / column) : dout;
//   dz = da (z > 0 ? 1 : slope);  A[n,c] = sum_hw dz,  B[n,c] = sum_hw dz xhat;
//   dbeta = sum_n A,  dgamma = sum_n B,  S1[n,g] = sum_{c in g} gamma A,  S2 = sum_{c in g} gamma B,
//   dy = rstd (gamma dz - S1 / Ng - xhat S2 / Ng),  Ng = H W C / groups.
// Pass 1: per (n, pixel chunk) per-channel partial sums; pass 2: per (n, c) ordered sum over chunks (f64)
// -> A, B; pass 3: per (n, g) S1, S2 and per c dbeta, dgamma; pass 4: elementwise dy.  Deterministic.
constexpr int GNB_CHUNK = 256;  // pixels per pass-1 workgroup

template <typename T> __device__ __forceinline__ float gld(const T* p, int64_t i) { return ld(p + i); }

__device__ __forceinline__ float gnb_dz(float yv, float da, float mean, float rstd, float gam, float bet, float slope,
                                        float& xhat) {
  xhat = (yv - mean) * rstd;
  const float z = gam * xhat + bet;
  return z > 0.f ? da : da * slope;
}


// 8 consecutive channels per thread (16-B bf16 / 32-B f32 accesses; c_p % 8 == 0: padded to 32 channels)
__device__ __forceinline__ void ld8(const float* p, float (&v)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ void ld8(const bf16_t* p, float (&v)[8]) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[2 * k] = __uint_as_float(w[k] << 16);
    v[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
  }
}
__device__ __forceinline__ void ld8(const _Float16* p, float (&v)[8]) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const bw_h2 h = __builtin_bit_cast(bw_h2, w[k]);
    v[2 * k] = (float)h.x;
    v[2 * k + 1] = (float)h.y;
  }
}
__device__ __forceinline__ void st8(float* p, const float (&v)[8]) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}
__device__ __forceinline__ void st8(bf16_t* p, const float (&v)[8]) {
  uint32_t w[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) w[k] = (uint32_t)f2bf(v[2 * k]) | ((uint32_t)f2bf(v[2 * k + 1]) << 16);
  *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
}
// f16 (the f16 training path): IEEE conversion, so a loss-scaled gradient that overflows reaches the scaler as inf
__device__ __forceinline__ void st8(_Float16* p, const float (&v)[8]) {
  uint32_t w[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) w[k] = __builtin_bit_cast(uint32_t, bw_h2{(_Float16)v[2 * k], (_Float16)v[2 * k + 1]});
  *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
}
// dL/da of output pixel p (channels cc0 .. cc0 + 7): dout, or a quarter of the pooled gradient (0 on a floor-dropped
// odd row / column)
template <typename TD>
__device__ __forceinline__ void gnb_da8(const TD* dout, int nn, int p, int h, int w, int c_p, int cc0, int pool,
                                        float (&dv)[8]) {
  if (!pool) {
    ld8(dout + ((int64_t)nn * h * w + p) * c_p + cc0, dv);
    return;
  }
  const int yy = p / w, xx = p - (p / w) * w;
  const int oh = h / 2, ow = w / 2;
  if (yy >= 2 * oh || xx >= 2 * ow) {
#pragma unroll
    for (int j = 0; j < 8; ++j) dv[j] = 0.f;
    return;
  }
  ld8(dout + (((int64_t)nn * oh + yy / 2) * ow + xx / 2) * c_p + cc0, dv);
#pragma unroll
  for (int j = 0; j < 8; ++j) dv[j] *= 0.25f;
}

// Pass 1: thread = 8 channels (fixed) x pixel lane; per-channel coefficients in registers; two pixels in flight
template <typename TY, typename TD>
__global__ void __launch_bounds__(256) gnb_partial_kernel(const TY* __restrict__ y, const TD* __restrict__ dout, int n,
                                                          int h, int w, int c_p, int c, int groups,
                                                          const float* __restrict__ stats,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, float slope, int pool,
                                                          int nchunks, float* __restrict__ part) {
  __shared__ float sAB[256 * 25];  // [thread][8 A, 8 B, 8 X] (+1: odd row pitch)
  const int hw = h * w;
  const int chunk = blockIdx.x % nchunks, nn = blockIdx.x / nchunks;
  const int p0 = chunk * GNB_CHUNK, p1 = min(hw, p0 + GNB_CHUNK);
  const int C8 = c_p >> 3;
  const int CT = C8 < 256 ? C8 : 256, PS = 256 / CT;
  const int cpg = c / groups;
  const int cl = threadIdx.x % CT, ph = threadIdx.x / CT;
  for (int cb = 0; cb < C8; cb += CT) {
    const int c8 = cb + cl, cc0 = 8 * c8;
    float sa[8], sb[8], sx[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) sa[j] = sb[j] = sx[j] = 0.f;
    if (ph < PS && c8 < C8 && cc0 < c) {
      float mean[8], rstd[8], gam[8], bet[8], valid[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int cc = cc0 + j;
        const bool ok = cc < c;
        const int gi = ok ? cc / cpg : 0;
        mean[j] = stats[(nn * groups + gi) * 2];
        rstd[j] = stats[(nn * groups + gi) * 2 + 1];
        gam[j] = ok ? gamma[cc] : 0.f;
        bet[j] = ok ? beta[cc] : 0.f;
        valid[j] = ok ? 1.f : 0.f;
      }
#pragma unroll 2
      for (int p = p0 + ph; p < p1; p += PS) {
        float yv[8], dv[8];
        ld8(y + ((int64_t)nn * hw + p) * c_p + cc0, yv);
        gnb_da8(dout, nn, p, h, w, c_p, cc0, pool, dv);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float xhat;
          const float dz = gnb_dz(yv[j], dv[j] * valid[j], mean[j], rstd[j], gam[j], bet[j], slope, xhat);
          sa[j] += dz;
          sb[j] += dz * xhat;
          sx[j] += xhat;
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sAB[threadIdx.x * 25 + j] = sa[j];
      sAB[threadIdx.x * 25 + 8 + j] = sb[j];
      sAB[threadIdx.x * 25 + 16 + j] = sx[j];
    }
    __syncthreads();
    if (ph == 0 && c8 < C8) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float a = 0.f, b = 0.f, x = 0.f;
        for (int k = 0; k < PS; ++k) {
          a += sAB[(k * CT + cl) * 25 + j];
          b += sAB[(k * CT + cl) * 25 + 8 + j];
          x += sAB[(k * CT + cl) * 25 + 16 + j];
        }
        float* o = part + (((int64_t)nn * c_p + cc0 + j) * nchunks + chunk) * 3;
        o[0] = a;
        o[1] = b;
        o[2] = x;
      }
    }
  }
}

// per (n, c): ordered f64 sum over the chunks -> AB[n][c][3] (sum dz, sum dz * xhat, sum xhat)
__global__ void __launch_bounds__(256) gnb_chunks_kernel(const float* __restrict__ part, int nc, int nchunks,
                                                         double* __restrict__ ab) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= nc) return;
  double a = 0.0, b = 0.0, x = 0.0;
  for (int k = 0; k < nchunks; ++k) {
    a += part[((int64_t)i * nchunks + k) * 3];
    b += part[((int64_t)i * nchunks + k) * 3 + 1];
    x += part[((int64_t)i * nchunks + k) * 3 + 2];
  }
  ab[3 * i] = a;
  ab[3 * i + 1] = b;
  ab[3 * i + 2] = x;
}

// one thread per (n, g): S1, S2 (f32 out, divided by Ng); then one thread per channel: dbeta, dgamma (sum over n)
__global__ void __launch_bounds__(256) gnb_group_kernel(const double* __restrict__ ab, int n, int c_p, int c,
                                                        int groups, double ng, const float* __restrict__ gamma,
                                                        float* __restrict__ s12, float* __restrict__ dgamma,
                                                        float* __restrict__ dbeta) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int cpg = c / groups;
  if (i < n * groups) {
    const int nn = i / groups, gi = i - (i / groups) * groups;
    double s1 = 0.0, s2 = 0.0;
    for (int k = 0; k < cpg; ++k) {
      const int cc = gi * cpg + k;
      s1 += (double)gamma[cc] * ab[((int64_t)nn * c_p + cc) * 3];
      s2 += (double)gamma[cc] * ab[((int64_t)nn * c_p + cc) * 3 + 1];
    }
    s12[2 * i] = (float)(s1 / ng);
    s12[2 * i + 1] = (float)(s2 / ng);
  }
  if (i < c) {
    double db = 0.0, dg = 0.0;
    for (int nn = 0; nn < n; ++nn) {
      db += ab[((int64_t)nn * c_p + i) * 3];
      dg += ab[((int64_t)nn * c_p + i) * 3 + 1];
    }
    if (dbeta) dbeta[i] = (float)db;
    if (dgamma) dgamma[i] = (float)dg;
  }
}

// one thread per channel: the sum of dy over (n, p) -- the bias gradient of the conv that produced y -- from the
// pass-1 channel sums and the same f32 S1 / Ng, S2 / Ng the apply pass uses:
//   sum_p dy[n][p][c] = rstd * (gamma * sum_p dz - HW * s1 - s2 * sum_p xhat)
__global__ void __launch_bounds__(256) gnb_dsum_kernel(const double* __restrict__ ab, int n, int c_p, int c, int groups,
                                                       const float* __restrict__ gamma,
                                                       const float* __restrict__ stats,
                                                       const float* __restrict__ s12, double hw,
                                                       float* __restrict__ dsum) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= c) return;
  const int gi = i / (c / groups);
  double ds = 0.0;
  for (int nn = 0; nn < n; ++nn) {
    const int sidx = nn * groups + gi;
    const double* a = ab + ((int64_t)nn * c_p + i) * 3;
    ds += (double)stats[2 * sidx + 1] *
          ((double)gamma[i] * a[0] - hw * (double)s12[2 * sidx] - (double)s12[2 * sidx + 1] * a[2]);
  }
  dsum[i] = (float)ds;
}

// Pass 4: grid (pixel blocks, n); thread = 8 channels (fixed, coefficients in registers) x pixel lane
template <typename TY, typename TD, typename TO>
__global__ void __launch_bounds__(256) gnb_apply_kernel(const TY* __restrict__ y, const TD* __restrict__ dout,
                                                        TO* __restrict__ dy, int n, int h, int w, int c_p, int c,
                                                        int groups, const float* __restrict__ stats,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, float slope, int pool,
                                                        const float* __restrict__ s12) {
  const int hw = h * w, nn = blockIdx.y;
  const int C8 = c_p >> 3;
  const int CT = C8 < 256 ? C8 : 256, PS = 256 / CT;
  const int cpg = c / groups;
  const int cl = threadIdx.x % CT, ph = threadIdx.x / CT;
  if (ph >= PS) return;
  for (int cb = 0; cb < C8; cb += CT) {
    const int c8 = cb + cl, cc0 = 8 * c8;
    if (c8 >= C8) continue;
    float mean[8], rstd[8], gam[8], bet[8], s1[8], s2[8], valid[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int cc = cc0 + j;
      const bool ok = cc < c;
      const int sidx = nn * groups + (ok ? cc / cpg : 0);
      mean[j] = stats[2 * sidx];
      rstd[j] = stats[2 * sidx + 1];
      gam[j] = ok ? gamma[cc] : 0.f;
      bet[j] = ok ? beta[cc] : 0.f;
      s1[j] = s12[2 * sidx];
      s2[j] = s12[2 * sidx + 1];
      valid[j] = ok ? 1.f : 0.f;
    }
#pragma unroll 2
    for (int p = blockIdx.x * PS + ph; p < hw; p += gridDim.x * PS) {
      const int64_t e = ((int64_t)nn * hw + p) * c_p + cc0;
      float yv[8], dv[8], v[8];
      ld8(y + e, yv);
      gnb_da8(dout, nn, p, h, w, c_p, cc0, pool, dv);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float xhat;
        const float dz = gnb_dz(yv[j], dv[j], mean[j], rstd[j], gam[j], bet[j], slope, xhat);
        v[j] = valid[j] * rstd[j] * (gam[j] * dz - s1[j] - xhat * s2[j]);
      }
      st8(dy + e, v);
    }
  }
}

// d mean_{hw}(x) / dx: dx[n][p][c] = dpooled[n][c] / hw (padded channels 0)
template <typename TO>
__global__ void __launch_bounds__(256) gap_bwd_kernel(const float* __restrict__ dp, TO* __restrict__ dx, int n, int hw,
                                                      int c_p, int c) {
  const int64_t total = (int64_t)n * hw * c_p;
  const float inv = 1.f / (float)hw;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int cc = (int)(e % c_p);
    const int nn = (int)(e / ((int64_t)hw * c_p));
    const float v = cc < c ? dp[(int64_t)nn * c + cc] * inv : 0.f;
    if constexpr (std::is_same<TO, _Float16>::value) dx[e] = (_Float16)v;   // IEEE (the scaler sees an overflow)
    else st(dx + e, v);
  }
}

static unsigned grid_for(int64_t total) {
  int64_t g = ceil_div(total, 256);
  return (unsigned)(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}

// ------------------------------------------------------------------------------------------------
// Backward of the synthesis layers' input modulation a = x * xscale[n][c] (SG3 modulated_conv2d's style
// multiply in activation-scaling form): dx = da * xscale, and d xscale[n][c] = sum_p da * x as per-chunk partial
// sums (fixed order; the host sums the chunks).  Block = (sample, pixel chunk); threads own channel pairs.
// ------------------------------------------------------------------------------------------------
__host__ __device__ inline int sb_chunk_pix(int n, int hw) {
  const int64_t want = ceil_div((int64_t)n * hw, 2048);
  return (int)(want < 16 ? 16 : (want > 1024 ? 1024 : want));
}

template <typename T> __device__ __forceinline__ float2 sb_ld2(const T* p);
template <> __device__ __forceinline__ float2 sb_ld2<float>(const float* p) { return *reinterpret_cast<const float2*>(p); }
template <> __device__ __forceinline__ float2 sb_ld2<bf16_t>(const bf16_t* p) {
  const uint32_t v = *reinterpret_cast<const uint32_t*>(p);
  return make_float2(__uint_as_float(v << 16), __uint_as_float(v & 0xffff0000u));
}
template <typename T> __device__ __forceinline__ void sb_st2(T* p, float2 v);
template <> __device__ __forceinline__ void sb_st2<float>(float* p, float2 v) { *reinterpret_cast<float2*>(p) = v; }
template <> __device__ __forceinline__ void sb_st2<bf16_t>(bf16_t* p, float2 v) {
  *reinterpret_cast<uint32_t*>(p) = (uint32_t)f2bf(v.x) | ((uint32_t)f2bf(v.y) << 16);
}
template <> __device__ __forceinline__ float2 sb_ld2<_Float16>(const _Float16* p) {
  const bw_h2 h = *reinterpret_cast<const bw_h2*>(p);
  return make_float2((float)h.x, (float)h.y);
}
template <> __device__ __forceinline__ void sb_st2<_Float16>(_Float16* p, float2 v) {
  *reinterpret_cast<bw_h2*>(p) = bw_h2{(_Float16)v.x, (_Float16)v.y};
}

template <typename T>
__global__ void __launch_bounds__(256) scale_bwd_kernel(const T* __restrict__ da, const T* __restrict__ x,
                                                        const float* __restrict__ xs, T* __restrict__ dx,
                                                        float* __restrict__ part, int hw, int c_p, int nchunks,
                                                        int chunk_pix) {
  extern __shared__ __attribute__((aligned(16))) float sbred[];  // [PS][c_p]
  const int chunk = blockIdx.x % nchunks;
  const int nn = blockIdx.x / nchunks;
  const int npair = c_p >> 1;
  const int CT = npair < 256 ? npair : 256;
  const int PS = 256 / CT;
  const int cq0 = threadIdx.x % CT, pp = threadIdx.x / CT;
  const int p0 = chunk * chunk_pix, p1 = min(hw, p0 + chunk_pix);
  const int64_t base = (int64_t)nn * hw * c_p;
  if (pp < PS) {
    for (int cq = cq0; cq < npair; cq += CT) {
      const float2 sc = *reinterpret_cast<const float2*>(xs + (int64_t)nn * c_p + 2 * cq);
      float s0 = 0.f, s1 = 0.f;
      for (int p = p0 + pp; p < p1; p += PS) {
        const int64_t e = base + (int64_t)p * c_p + 2 * cq;
        const float2 g = sb_ld2(da + e), v = sb_ld2(x + e);
        s0 += g.x * v.x;
        s1 += g.y * v.y;
        if (dx != nullptr) sb_st2(dx + e, make_float2(g.x * sc.x, g.y * sc.y));
      }
      sbred[pp * c_p + 2 * cq] = s0;
      sbred[pp * c_p + 2 * cq + 1] = s1;
    }
  }
  __syncthreads();
  for (int ch = threadIdx.x; ch < c_p; ch += 256) {
    float t = 0.f;
    for (int k = 0; k < PS; ++k) t += sbred[k * c_p + ch];
    part[((int64_t)nn * nchunks + chunk) * c_p + ch] = t;
  }
}

}  // namespace ic2

using namespace ic2;

extern "C" int64_t ic2_scale_bwd_part_floats(int n, int hw, int c_p) {
  if (n <= 0 || hw <= 0 || c_p <= 0) return 0;
  return (int64_t)n * ceil_div(hw, sb_chunk_pix(n, hw)) * c_p;
}

// a = x * xscale[n][c]: grid (pixel blocks, n), thread = 8 channels (scale in registers) x pixel lane
template <typename T>
__global__ void __launch_bounds__(256) scale_fwd_kernel(const T* __restrict__ x, const float* __restrict__ xs,
                                                        T* __restrict__ a, int hw, int c_p) {
  const int nn = blockIdx.y, C8 = c_p >> 3;
  const int CT = C8 < 256 ? C8 : 256, PS = 256 / CT;
  const int cl = threadIdx.x % CT, ph = threadIdx.x / CT;
  if (ph >= PS) return;
  for (int c8 = cl; c8 < C8; c8 += CT) {
    float sc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) sc[j] = xs[(int64_t)nn * c_p + 8 * c8 + j];
#pragma unroll 2
    for (int p = blockIdx.x * PS + ph; p < hw; p += gridDim.x * PS) {
      const int64_t e = ((int64_t)nn * hw + p) * c_p + 8 * c8;
      float v[8];
      ld8(x + e, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] *= sc[j];
      st8(a + e, v);
    }
  }
}

extern "C" int ic2_scale_nhwc(const void* x, const float* xscale, void* a, int dtype, int n, int hw, int c_p,
                              void* stream) {
  IC2_CHECK_ARG(x && xscale && a && n > 0 && n <= 65535 && hw > 0 && c_p > 0 && c_p % 8 == 0, "scale_nhwc: bad arguments");
  const int ps = 256 / (c_p / 8 < 256 ? c_p / 8 : 256);
  const int64_t pb = ceil_div(ceil_div((int64_t)hw, ps), 4);
  const dim3 grid((unsigned)(pb < 1 ? 1 : (pb > 65535 ? 65535 : pb)), (unsigned)n);
  hipStream_t s = as_stream(stream);
  if (dtype == IC2_F32)
    hipLaunchKernelGGL(scale_fwd_kernel<float>, grid, dim3(256), 0, s, (const float*)x, xscale, (float*)a, hw, c_p);
  else if (dtype == IC2_BF16)
    hipLaunchKernelGGL(scale_fwd_kernel<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)x, xscale, (bf16_t*)a, hw, c_p);
  else if (dtype == IC2_F16)
    hipLaunchKernelGGL(scale_fwd_kernel<_Float16>, grid, dim3(256), 0, s, (const _Float16*)x, xscale, (_Float16*)a, hw,
                       c_p);
  else
    IC2_CHECK_ARG(false, "scale_nhwc: bad dtype %d", dtype);
  IC2_CHECK_LAUNCH("scale_nhwc");
  return IC2_OK;
}

extern "C" int ic2_scale_bwd_nhwc(const void* da, const void* x, const float* xscale, void* dx, int dtype, int n, int hw,
                                  int c_p, float* part, int64_t part_floats, void* stream) {
  IC2_CHECK_ARG(da && x && xscale && part && n > 0 && hw > 0 && c_p > 0 && c_p % 2 == 0 && c_p <= 512,
                "scale_bwd_nhwc: bad arguments");  // dx may be null: the partial sums only
  IC2_CHECK_ARG(part_floats >= ic2_scale_bwd_part_floats(n, hw, c_p), "scale_bwd_nhwc: partial buffer too small");
  const int chunk_pix = sb_chunk_pix(n, hw);
  const int nchunks = (int)ceil_div(hw, chunk_pix);
  const int npair = c_p / 2, CT = npair < 256 ? npair : 256, PS = 256 / CT;
  const size_t lds = (size_t)PS * c_p * sizeof(float);
  hipStream_t s = as_stream(stream);
  if (dtype == IC2_F32)
    hipLaunchKernelGGL(scale_bwd_kernel<float>, dim3(n * nchunks), dim3(256), lds, s, (const float*)da, (const float*)x,
                       xscale, (float*)dx, part, hw, c_p, nchunks, chunk_pix);
  else if (dtype == IC2_BF16)
    hipLaunchKernelGGL(scale_bwd_kernel<bf16_t>, dim3(n * nchunks), dim3(256), lds, s, (const bf16_t*)da,
                       (const bf16_t*)x, xscale, (bf16_t*)dx, part, hw, c_p, nchunks, chunk_pix);
  else if (dtype == IC2_F16)
    hipLaunchKernelGGL(scale_bwd_kernel<_Float16>, dim3(n * nchunks), dim3(256), lds, s, (const _Float16*)da,
                       (const _Float16*)x, xscale, (_Float16*)dx, part, hw, c_p, nchunks, chunk_pix);
  else
    IC2_CHECK_ARG(false, "scale_bwd_nhwc: bad dtype %d", dtype);
  IC2_CHECK_LAUNCH("scale_bwd_nhwc");
  return IC2_OK;
}

// out[n][c] = (sum over r of part[n][r][c]) / den[n][c], 0 where den[n][c] == 0 (no den: the plain sum).  Block =
// (64 channels, sample): lane group k sums rows k, k+4, ... (coalesced 256-B rows, 4 loads in flight), the 4 group
// sums combine in a fixed order through LDS: deterministic.
__global__ void __launch_bounds__(256) colsum_div_kernel(const float* __restrict__ part, int rows, int c,
                                                         const float* __restrict__ den, float* __restrict__ out) {
  __shared__ float red[4][64];
  const int nn = blockIdx.y, cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int ch = blockIdx.x * 64 + cl;
  float t = 0.f;
  if (ch < c) {
    const float* p = part + (int64_t)nn * rows * c + ch;
    int r = rg;
    for (; r + 12 < rows; r += 16) {
      const float a0 = p[(int64_t)r * c], a1 = p[(int64_t)(r + 4) * c], a2 = p[(int64_t)(r + 8) * c],
                  a3 = p[(int64_t)(r + 12) * c];
      t += a0;
      t += a1;
      t += a2;
      t += a3;
    }
    for (; r < rows; r += 4) t += p[(int64_t)r * c];
  }
  red[rg][cl] = t;
  __syncthreads();
  if (rg == 0 && ch < c) {
    float s = red[0][cl] + red[1][cl];
    s += red[2][cl];
    s += red[3][cl];
    const int64_t i = (int64_t)nn * c + ch;
    if (den != nullptr) {
      const float d = den[i];
      s = d != 0.f ? s / d : 0.f;
    }
    out[i] = s;
  }
}

extern "C" int ic2_colsum_div(const float* part, int n, int rows, int c, const float* den, float* out, void* stream) {
  IC2_CHECK_ARG(part && out && n > 0 && n <= 65535 && rows > 0 && c > 0, "colsum_div: bad arguments");
  hipLaunchKernelGGL(colsum_div_kernel, dim3((unsigned)ceil_div(c, 64), (unsigned)n), dim3(256), 0, as_stream(stream),
                     part, rows, c, den, out);
  IC2_CHECK_LAUNCH("colsum_div");
  return IC2_OK;
}

extern "C" int64_t ic2_conv_wgrad_ws_floats(int n, int h, int w, int cin_p, int cout_p, int kh, int kw, int pad) {
  WgradArgs a{};
  a.ho = h + 2 * pad - kh + 1;
  a.wo = w + 2 * pad - kw + 1;
  if (n <= 0 || a.ho <= 0 || a.wo <= 0 || cin_p % 32 || cout_p % 32) return 0;
  a.P = n * a.ho * a.wo;
  a.chunks = (int)ceil_div(a.P, WG_KP);
  a.cout_p = cout_p;
  a.cin_p = cin_p; a.kh = kh; a.kw = kw;
  a.j_tiles = kh * kw * (int)ceil_div(cin_p, WG_BJ);
  // enough for either kernel (the 16-bit one plans its own splits)
  const int sp = std::max(wgrad_splits(a), std::max(wgrad2_splits(a, 64, 4096, 64), wgrad2_splits(a, 64, 2048, 128)));
  return (int64_t)sp * cout_p * kh * kw * cin_p;
}

static int conv_wgrad_impl(const void* x, const void* dy, float* dw, int dtype, int n, int h, int w, int cin_p,
                           int cout_p, int kh, int kw, int pad, float* workspace, int64_t ws_floats, void* stream,
                           int oihw_cout, int oihw_cin);

extern "C" int ic2_conv_wgrad(const void* x, const void* dy, float* dw, int dtype, int n, int h, int w, int cin_p,
                              int cout_p, int kh, int kw, int pad, float* workspace, int64_t ws_floats, void* stream) {
  return conv_wgrad_impl(x, dy, dw, dtype, n, h, w, cin_p, cout_p, kh, kw, pad, workspace, ws_floats, stream, 0, 0);
}

extern "C" int ic2_conv_wgrad_oihw(const void* x, const void* dy, float* dw, int dtype, int n, int h, int w,
                                   int cin_p, int cout_p, int cout, int cin, int kh, int kw, int pad, float* workspace,
                                   int64_t ws_floats, void* stream) {
  IC2_CHECK_ARG(cout > 0 && cout <= cout_p && cin > 0 && cin <= cin_p, "conv_wgrad_oihw: bad channel counts");
  return conv_wgrad_impl(x, dy, dw, dtype, n, h, w, cin_p, cout_p, kh, kw, pad, workspace, ws_floats, stream, cout,
                         cin);
}

static int conv_wgrad_impl(const void* x, const void* dy, float* dw, int dtype, int n, int h, int w, int cin_p,
                           int cout_p, int kh, int kw, int pad, float* workspace, int64_t ws_floats, void* stream,
                           int oihw_cout, int oihw_cin) {
  IC2_CHECK_ARG(x && dy && dw && workspace, "conv_wgrad: null pointer");
  IC2_CHECK_ARG(dtype == IC2_F32 || dtype == IC2_BF16 || dtype == IC2_F16, "conv_wgrad: bad dtype %d", dtype);
  IC2_CHECK_ARG(cin_p > 0 && cin_p % 32 == 0 && cout_p > 0 && cout_p % 32 == 0,
                "conv_wgrad: channel strides must be positive multiples of 32 (cin_p=%d cout_p=%d)", cin_p, cout_p);
  IC2_CHECK_ARG(n > 0 && h > 0 && w > 0 && kh > 0 && kw > 0 && pad >= 0, "conv_wgrad: bad geometry");
  WgradArgs a{};
  a.x = x; a.dy = dy; a.part = workspace;
  a.n = n; a.h = h; a.w = w; a.cin_p = cin_p; a.cout_p = cout_p; a.kh = kh; a.kw = kw; a.pad = pad;
  a.ho = h + 2 * pad - kh + 1;
  a.wo = w + 2 * pad - kw + 1;
  IC2_CHECK_ARG(a.ho > 0 && a.wo > 0, "conv_wgrad: empty output");
  IC2_CHECK_ARG((int64_t)n * a.ho * a.wo < (1LL << 30), "conv_wgrad: too many pixels");
  a.P = n * a.ho * a.wo;
  a.chunks = (int)ceil_div(a.P, WG_KP);
  a.j_tiles = kh * kw * (int)ceil_div(cin_p, WG_BJ);
  // knob IC2_WGRAD2: 1 = the staged kernel, 64-wide tiles (default), 3 = 128-wide tiles where they fill, 0 = the
  // round-3 kernel for 16-bit operands too
  static const int v2 = knob("IC2_WGRAD2", 1);
  const bool wide = v2 != 0 && dtype != IC2_F32;
  const int bt = v2 == 3 ? wgrad2_tile(cout_p, kh * kw * cin_p) : 64;
  // knob IC2_WGRAD_TARGET: workgroups per launch the K split aims at (64-wide tiles; the split-K partials it writes
  // are re-read by wgrad_reduce_kernel)
  static const int target = std::max(64, std::min(knob("IC2_WGRAD_TARGET", 4096), 4096));  // <= the workspace plan's
  const int splits = wide ? wgrad2_splits(a, 64, bt == 128 ? target / 2 : target, bt) : wgrad_splits(a);
  const int64_t total = (int64_t)cout_p * kh * kw * cin_p;
  IC2_CHECK_ARG(ws_floats >= splits * total, "conv_wgrad: workspace too small (%lld < %lld floats)",
                (long long)ws_floats, (long long)(splits * total));
  hipStream_t s = as_stream(stream);
  if (wide) {
    a.chunks = (int)ceil_div(a.P, 64);
    const dim3 grid((unsigned)(ceil_div(cout_p, bt) * ceil_div((int64_t)kh * kw * cin_p, bt)), (unsigned)splits);
    if (bt == 128) {
      if (dtype == IC2_BF16) hipLaunchKernelGGL((wgrad2_kernel<bf16_t, 64, 128>), grid, dim3(256), 0, s, a);
      else hipLaunchKernelGGL((wgrad2_kernel<_Float16, 64, 128>), grid, dim3(256), 0, s, a);
    } else {
      if (dtype == IC2_BF16) hipLaunchKernelGGL((wgrad2_kernel<bf16_t, 64, 64>), grid, dim3(256), 0, s, a);
      else hipLaunchKernelGGL((wgrad2_kernel<_Float16, 64, 64>), grid, dim3(256), 0, s, a);
    }
  } else {
    const dim3 grid((unsigned)(ceil_div(cout_p, WG_BO) * a.j_tiles), (unsigned)splits);
    if (dtype == IC2_BF16) hipLaunchKernelGGL(wgrad_kernel<bf16_t>, grid, dim3(256), 0, s, a);
    else if (dtype == IC2_F16) hipLaunchKernelGGL(wgrad_kernel<_Float16>, grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL(wgrad_kernel<float>, grid, dim3(256), 0, s, a);
  }
  if (oihw_cout > 0)
    hipLaunchKernelGGL(wgrad_reduce_oihw_kernel, dim3(grid_for(total)), dim3(256), 0, s, workspace, dw, total, splits,
                       cin_p, kh * kw, oihw_cout, oihw_cin);
  else
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(grid_for(total)), dim3(256), 0, s, workspace, dw, total, splits);
  IC2_CHECK_LAUNCH("conv_wgrad");
  return IC2_OK;
}

extern "C" int64_t ic2_gn_lrelu_pool_bwd_floats(int n, int h, int w, int c_p, int groups) {
  const int64_t nchunks = ceil_div((int64_t)h * w, GNB_CHUNK);
  // part [n][c_p][nchunks][3] f32 | ab [n][c_p][3] f64 | s12 [n][groups][2] f32
  return (int64_t)n * c_p * nchunks * 3 + (int64_t)n * c_p * 3 * 2 + (int64_t)n * groups * 2 + 4;
}

extern "C" int ic2_gn_lrelu_pool_bwd_db(const void* y, const void* dout, void* dy, int dtype_y, int dtype_dout,
                                        int dtype_dy, int n, int h, int w, int c_p, int c, int groups,
                                        const float* stats, const float* gamma, const float* beta, float slope,
                                        int pool, float* dgamma, float* dbeta, float* dsum, float* workspace,
                                        int64_t ws_floats, void* stream);

extern "C" int ic2_gn_lrelu_pool_bwd(const void* y, const void* dout, void* dy, int dtype_y, int dtype_dout,
                                     int dtype_dy, int n, int h, int w, int c_p, int c, int groups, const float* stats,
                                     const float* gamma, const float* beta, float slope, int pool, float* dgamma,
                                     float* dbeta, float* workspace, int64_t ws_floats, void* stream) {
  return ic2_gn_lrelu_pool_bwd_db(y, dout, dy, dtype_y, dtype_dout, dtype_dy, n, h, w, c_p, c, groups, stats, gamma,
                                  beta, slope, pool, dgamma, dbeta, nullptr, workspace, ws_floats, stream);
}

extern "C" int ic2_gn_lrelu_pool_bwd_db(const void* y, const void* dout, void* dy, int dtype_y, int dtype_dout,
                                        int dtype_dy, int n, int h, int w, int c_p, int c, int groups,
                                        const float* stats, const float* gamma, const float* beta, float slope,
                                        int pool, float* dgamma, float* dbeta, float* dsum, float* workspace,
                                        int64_t ws_floats, void* stream) {
  IC2_CHECK_ARG(y && dout && dy && stats && gamma && beta && workspace && n > 0 && h > 0 && w > 0 && c > 0 &&
                    c <= c_p && groups > 0 && c % groups == 0,
                "gn_lrelu_pool_bwd: bad arguments");
  IC2_CHECK_ARG(!pool || (h >= 2 && w >= 2), "gn_lrelu_pool_bwd: pooling needs H, W >= 2");
  IC2_CHECK_ARG(c_p % 8 == 0 && n <= 65535, "gn_lrelu_pool_bwd: c_p must be a multiple of 8 (n <= 65535)");
  IC2_CHECK_ARG(ws_floats >= ic2_gn_lrelu_pool_bwd_floats(n, h, w, c_p, groups), "gn_lrelu_pool_bwd: workspace too small");
  const bool f16 = dtype_y == IC2_F16 || dtype_dout == IC2_F16 || dtype_dy == IC2_F16;
  IC2_CHECK_ARG(f16 ? (dtype_y == IC2_F16 && dtype_dout == IC2_F16 && dtype_dy == IC2_F16)
                    : ((dtype_y == IC2_F32 || dtype_y == IC2_BF16) && (dtype_dout == IC2_F32 || dtype_dout == IC2_BF16) &&
                       (dtype_dy == IC2_F32 || dtype_dy == IC2_BF16)),
                "gn_lrelu_pool_bwd: bad dtypes (f16 only as f16 y, dout and dy)");
  const int nchunks = (int)ceil_div((int64_t)h * w, GNB_CHUNK);
  float* part = workspace;
  double* ab = reinterpret_cast<double*>(workspace + (((int64_t)n * c_p * nchunks * 3 + 1) / 2) * 2);
  float* s12 = reinterpret_cast<float*>(ab + (int64_t)n * c_p * 3);
  hipStream_t s = as_stream(stream);
  const double ng = (double)h * w * (c / groups);
  // pass 4: (pixel blocks, n); a block covers 256 / min(c_p / 8, 256) pixels per step, ~4 steps per thread
  const int ps4 = 256 / (c_p / 8 < 256 ? c_p / 8 : 256);
  const int64_t pblocks = ceil_div(ceil_div((int64_t)h * w, ps4), 4);
  const dim3 apply_grid((unsigned)(pblocks < 1 ? 1 : (pblocks > 65535 ? 65535 : pblocks)), (unsigned)n);
#define IC2_GNB(TY, TD) IC2_GNB_O(TY, TD, bf16_t)
#define IC2_GNB_O(TY, TD, TOB)                                                                                   \
  do {                                                                                                           \
    hipLaunchKernelGGL((gnb_partial_kernel<TY, TD>), dim3((unsigned)(n * nchunks)), dim3(256), 0, s, (const TY*)y, \
                       (const TD*)dout, n, h, w, c_p, c, groups, stats, gamma, beta, slope, pool, nchunks, part);   \
    hipLaunchKernelGGL(gnb_chunks_kernel, dim3(grid_for((int64_t)n * c_p)), dim3(256), 0, s, part, n * c_p,        \
                       nchunks, ab);                                                                             \
    const int ng_th = n * groups > c ? n * groups : c;                                                           \
    hipLaunchKernelGGL(gnb_group_kernel, dim3((unsigned)ceil_div(ng_th, 256)), dim3(256), 0, s, ab, n, c_p, c,     \
                       groups, ng, gamma, s12, dgamma, dbeta);                                                   \
    if (dsum)                                                                                                    \
      hipLaunchKernelGGL(gnb_dsum_kernel, dim3((unsigned)ceil_div(c, 256)), dim3(256), 0, s, ab, n, c_p, c, groups, \
                         gamma, stats, s12, (double)h * w, dsum);                                                \
    if (dtype_dy == IC2_F32)                                                                                     \
      hipLaunchKernelGGL((gnb_apply_kernel<TY, TD, float>), apply_grid, dim3(256), 0, s, (const TY*)y,             \
                         (const TD*)dout, (float*)dy, n, h, w, c_p, c, groups, stats, gamma, beta, slope, pool,    \
                         s12);                                                                                   \
    else                                                                                                         \
      hipLaunchKernelGGL((gnb_apply_kernel<TY, TD, TOB>), apply_grid, dim3(256), 0, s, (const TY*)y,               \
                         (const TD*)dout, (TOB*)dy, n, h, w, c_p, c, groups, stats, gamma, beta, slope, pool,      \
                         s12);                                                                                   \
  } while (0)
  if (f16) IC2_GNB_O(_Float16, _Float16, _Float16);
  else if (dtype_y == IC2_F32 && dtype_dout == IC2_F32) IC2_GNB(float, float);
  else if (dtype_y == IC2_F32) IC2_GNB(float, bf16_t);
  else if (dtype_dout == IC2_F32) IC2_GNB(bf16_t, float);
  else IC2_GNB(bf16_t, bf16_t);
#undef IC2_GNB
#undef IC2_GNB_O
  IC2_CHECK_LAUNCH("gn_lrelu_pool_bwd");
  return IC2_OK;
}

extern "C" int ic2_gap_bwd(const float* dpooled, void* dx, int dtype, int n, int hw, int c_p, int c, void* stream) {
  IC2_CHECK_ARG(dpooled && dx && n > 0 && hw > 0 && c > 0 && c <= c_p, "gap_bwd: bad arguments");
  const int64_t total = (int64_t)n * hw * c_p;
  hipStream_t s = as_stream(stream);
  if (dtype == IC2_F32) hipLaunchKernelGGL(gap_bwd_kernel<float>, dim3(grid_for(total)), dim3(256), 0, s, dpooled,
                                           (float*)dx, n, hw, c_p, c);
  else if (dtype == IC2_BF16) hipLaunchKernelGGL(gap_bwd_kernel<bf16_t>, dim3(grid_for(total)), dim3(256), 0, s,
                                                 dpooled, (bf16_t*)dx, n, hw, c_p, c);
  else if (dtype == IC2_F16) hipLaunchKernelGGL(gap_bwd_kernel<_Float16>, dim3(grid_for(total)), dim3(256), 0, s,
                                                dpooled, (_Float16*)dx, n, hw, c_p, c);
  else IC2_CHECK_ARG(false, "gap_bwd: bad dtype");
  IC2_CHECK_LAUNCH("gap_bwd");
  return IC2_OK;
}
