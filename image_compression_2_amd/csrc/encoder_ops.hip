// HVAE_VGG_Encoder support kernels (/root/reference/stylegan3_hvae_full.py:105-247) and the metric /
// resize helpers of the compressor API.  All HBM-bound; NHWC with padded channel stride c_p.
#include "common.h"

#include <algorithm>
#include <type_traits>

namespace ic2 {

static int grid_1d(int64_t total, int per = 1) {
  int64_t g = ceil_div(ceil_div(total, per), 256);
  if (g < 1) g = 1;
  if (g > 8192) g = 8192;
  return (int)g;
}

// Split-bf16 activations (ic2ops.h IC2_BF16X3): logical channel stride c_p stored as 2 * c_p bf16 channels
// [hi | lo] per pixel, hi = bf16(v), lo = bf16(v - hi) (v - hi is exact in f32).  (Round 3 stored [hi | hi | lo];
// the convs now read the hi block twice through their K mapping, igemm.hip ig_xb32.)
struct bf16x3_t {
  bf16_t v;
};
__device__ __forceinline__ void split_bf16(float v, bf16_t& hi, bf16_t& lo) {
  hi = f2bf(v);
  lo = f2bf(v - bf2f(hi));
}
// ------------------------------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(256) nchw_to_nhwc_kernel(const float* __restrict__ x, T* __restrict__ y, int n,
                                                           int c, int hw, int c_p, const float* __restrict__ scale) {
  const int64_t total = (int64_t)n * hw * c_p;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int ch = (int)(e % c_p);
    const int64_t pix = e / c_p;
    const int p = (int)(pix % hw);
    const int64_t nn = pix / hw;
    float v = ch < c ? x[(nn * c + ch) * hw + p] : 0.f;
    if (scale) v *= scale[nn * c_p + ch];
    st(y + e, v);
  }
}

__global__ void __launch_bounds__(256) nchw_to_nhwc_x3_kernel(const float* __restrict__ x, bf16_t* __restrict__ y, int n,
                                                              int c, int hw, int c_p, const float* __restrict__ scale) {
  const int64_t total = (int64_t)n * hw * c_p;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int ch = (int)(e % c_p);
    const int64_t pix = e / c_p;
    const int p = (int)(pix % hw);
    const int64_t nn = pix / hw;
    float v = ch < c ? x[(nn * c + ch) * hw + p] : 0.f;
    if (scale) v *= scale[nn * c_p + ch];
    bf16_t hi, lo;
    split_bf16(v, hi, lo);
    bf16_t* o = y + pix * 2 * c_p + ch;
    o[0] = hi;
    o[c_p] = lo;
  }
}

template <typename T>
__global__ void __launch_bounds__(256) nhwc_to_nchw_kernel(const T* __restrict__ x, float* __restrict__ y, int n, int c,
                                                           int hw, int c_p) {
  const int64_t total = (int64_t)n * c * hw;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int p = (int)(e % hw);
    const int64_t r = e / hw;
    const int ch = (int)(r % c);
    const int64_t nn = r / c;
    y[e] = ld(x + (nn * hw + p) * c_p + ch);
  }
}

// ------------------------------------------------------------------------------------------------
// GroupNorm statistics: stage 1 = per (n, pixel chunk) per-group partial sums (f64) written to
// `part`; stage 2 = per (n, group) ordered sum over chunks -> mean, rstd.  Deterministic.
// The chunk length adapts to the layer so that every layer launches >= ~2048 workgroups
// (the 8x8 / 4x4 encoder blocks otherwise run 32 latency-bound workgroups).
// ------------------------------------------------------------------------------------------------
__host__ __device__ inline int gn_chunk_pix(int n, int hw) {
  const int64_t want = ceil_div((int64_t)n * hw, 2048);
  return (int)(want < 8 ? 8 : (want > 256 ? 256 : want));
}

// two channels per thread (bf16x2 / float2 loads)
template <typename T> __device__ __forceinline__ float2 ld2(const T* p);
template <> __device__ __forceinline__ float2 ld2<float>(const float* p) { return *reinterpret_cast<const float2*>(p); }
template <> __device__ __forceinline__ float2 ld2<bf16_t>(const bf16_t* p) {
  const uint32_t v = *reinterpret_cast<const uint32_t*>(p);
  return make_float2(__uint_as_float(v << 16), __uint_as_float(v & 0xffff0000u));
}
// f16 activations: the encoder's f16 training precision (the reference's fp16 autocast, BASELINE config 5)
typedef _Float16 ic2_h2 __attribute__((ext_vector_type(2)));
template <> __device__ __forceinline__ float2 ld2<_Float16>(const _Float16* p) {
  const ic2_h2 v = *reinterpret_cast<const ic2_h2*>(p);
  return make_float2((float)v.x, (float)v.y);
}

template <typename T>
__global__ void __launch_bounds__(256) gn_partial_kernel(const T* __restrict__ y, int hw, int c_p, int c, int groups,
                                                         int nchunks, int chunk_pix, double* __restrict__ part) {
  // thread t -> channel pair t % CT (+ k*CT*... when c_p > 512), pixel phase t / CT; per-thread fp32
  // sums over <= chunk_pix / PS pixels, then a fixed-order f64 group reduction
  extern __shared__ __attribute__((aligned(16))) double sred[];  // [2][max(512, c_p)]
  const int chunk = blockIdx.x % nchunks;
  const int nn = blockIdx.x / nchunks;
  const int cpg = c / groups;
  const int p0 = chunk * chunk_pix;
  const int p1 = min(hw, p0 + chunk_pix);
  const T* yb = y + (int64_t)nn * hw * c_p;
  const int npair = c_p >> 1;
  const int CT = npair < 256 ? npair : 256;  // channel pairs covered per pass
  const int PS = 256 / CT;                   // pixel phases
  const int cp0 = threadIdx.x % CT;
  const int pp = threadIdx.x / CT;
  const int nslots = c_p < 512 ? 512 : c_p;
  double* ssum = sred;
  double* ssq = sred + nslots;
  if (pp < PS) {
    for (int cq = cp0; cq < npair; cq += 256) {
      float s0 = 0.f, q0 = 0.f, s1 = 0.f, q1 = 0.f;
#pragma unroll 8
      for (int p = p0 + pp; p < p1; p += PS) {
        const float2 v = ld2(yb + (int64_t)p * c_p + 2 * cq);
        s0 += v.x;
        q0 += v.x * v.x;
        s1 += v.y;
        q1 += v.y * v.y;
      }
      // slot = (phase, channel) for c_p < 512, else channel
      const int slot = c_p < 512 ? pp * c_p + 2 * cq : 2 * cq;
      ssum[slot] = s0;
      ssq[slot] = q0;
      ssum[slot + 1] = s1;
      ssq[slot + 1] = q1;
    }
  }
  __syncthreads();
  for (int g = threadIdx.x; g < groups; g += 256) {
    double s = 0.0, q = 0.0;
    for (int k = 0; k < cpg; ++k) {
      const int cc = g * cpg + k;
      if (c_p < 512) {
        for (int ph = 0; ph < PS; ++ph) {
          s += ssum[ph * c_p + cc];
          q += ssq[ph * c_p + cc];
        }
      } else {
        s += ssum[cc];
        q += ssq[cc];
      }
    }
    double* o = part + (((int64_t)nn * groups + g) * nchunks + chunk) * 2;
    o[0] = s;
    o[1] = q;
  }
}

// one wave per (sample, group): lanes sum the chunk partials in a fixed strided order, then a fixed xor tree
// (deterministic; the chunk partials of one group are contiguous, so the wave's loads coalesce)
__global__ void __launch_bounds__(64) gn_finalize_kernel(const double* __restrict__ part, int ngroups_total,
                                                         int nchunks, double count, float eps,
                                                         float* __restrict__ stats) {
  const int i = blockIdx.x;
  const int lane = threadIdx.x;
  double s = 0.0, q = 0.0;
  const double* pg = part + (int64_t)i * nchunks * 2;
  for (int k = lane; k < nchunks; k += 64) {
    s += pg[2 * k];
    q += pg[2 * k + 1];
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    s += __shfl_xor(s, off, 64);
    q += __shfl_xor(q, off, 64);
  }
  if (lane != 0) return;
  const double mean = s / count;
  double var = q / count - mean * mean;
  if (var < 0) var = 0;
  stats[i * 2 + 0] = (float)mean;
  stats[i * 2 + 1] = (float)(1.0 / sqrt(var + (double)eps));
}

// ------------------------------------------------------------------------------------------------
// GroupNorm apply + lrelu (+ 2x2 average pool); 8 channels (one 16-B bf16 / 2x16-B f32 vector) per thread
// ------------------------------------------------------------------------------------------------
template <typename T> __device__ __forceinline__ void ld8(const T* p, float (&v)[8]);
template <> __device__ __forceinline__ void ld8<float>(const float* p, float (&v)[8]) {
  const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
template <> __device__ __forceinline__ void ld8<bf16_t>(const bf16_t* p, float (&v)[8]) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[2 * k] = __uint_as_float(w[k] << 16);
    v[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
  }
}
template <> __device__ __forceinline__ void ld8<_Float16>(const _Float16* p, float (&v)[8]) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const ic2_h2 h = __builtin_bit_cast(ic2_h2, w[k]);
    v[2 * k] = (float)h.x;
    v[2 * k + 1] = (float)h.y;
  }
}
template <typename T> __device__ __forceinline__ void st8(T* p, const float (&v)[8]);
template <> __device__ __forceinline__ void st8<float>(float* p, const float (&v)[8]) {
  reinterpret_cast<float4*>(p)[0] = make_float4(v[0], v[1], v[2], v[3]);
  reinterpret_cast<float4*>(p)[1] = make_float4(v[4], v[5], v[6], v[7]);
}
template <> __device__ __forceinline__ void st8<bf16_t>(bf16_t* p, const float (&v)[8]) {
  uint4 u;
  u.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
  u.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
  u.z = (uint32_t)f2bf(v[4]) | ((uint32_t)f2bf(v[5]) << 16);
  u.w = (uint32_t)f2bf(v[6]) | ((uint32_t)f2bf(v[7]) << 16);
  *reinterpret_cast<uint4*>(p) = u;
}
template <> __device__ __forceinline__ void st8<_Float16>(_Float16* p, const float (&v)[8]) {
  uint32_t w[4];
#pragma unroll
  for (int k = 0; k < 4; ++k)  // activations saturate at the f16 range (Elem<_Float16>, the synthesis's f16 mode)
    w[k] = __builtin_bit_cast(uint32_t, ic2_h2{(_Float16)__builtin_amdgcn_fmed3f(v[2 * k], -65504.f, 65504.f),
                                               (_Float16)__builtin_amdgcn_fmed3f(v[2 * k + 1], -65504.f, 65504.f)});
  *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
}

// eight consecutive channels ch0 .. ch0+7 of pixel `pix` (tensor-global pixel index) with logical stride c_p
template <typename T>
__device__ __forceinline__ void st8p(T* out, int64_t pix, int c_p, int ch0, const float (&v)[8]) {
  st8(out + pix * c_p + ch0, v);
}
template <>
__device__ __forceinline__ void st8p<bf16x3_t>(bf16x3_t* out, int64_t pix, int c_p, int ch0, const float (&v)[8]) {
  bf16_t* b = reinterpret_cast<bf16_t*>(out) + pix * 2 * c_p + ch0;
  uint32_t h[4], l[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    bf16_t h0, l0, h1, l1;
    split_bf16(v[2 * k], h0, l0);
    split_bf16(v[2 * k + 1], h1, l1);
    h[k] = (uint32_t)h0 | ((uint32_t)h1 << 16);
    l[k] = (uint32_t)l0 | ((uint32_t)l1 << 16);
  }
  *reinterpret_cast<uint4*>(b) = make_uint4(h[0], h[1], h[2], h[3]);
  *reinterpret_cast<uint4*>(b + c_p) = make_uint4(l[0], l[1], l[2], l[3]);
}

template <typename TI, typename TO>
__global__ void __launch_bounds__(256) gn_apply_kernel(const TI* __restrict__ y, TO* __restrict__ out, int n, int h,
                                                       int w, int c_p, int c, int groups,
                                                       const float* __restrict__ stats,
                                                       const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, float slope, int pool) {
  const int oh = pool ? h / 2 : h, ow = pool ? w / 2 : w;
  const int c8 = c_p / 8;
  const int64_t total = (int64_t)n * oh * ow * c8;
  const int cpg = c / groups;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int ch0 = (int)(e % c8) * 8;
    const int64_t pix = e / c8;
    const int ox = (int)(pix % ow);
    const int oy = (int)((pix / ow) % oh);
    const int nn = (int)(pix / ((int64_t)ow * oh));
    float mu[8], sc[8], sh[8];  // t = (v - mean) * (rstd * gamma) + beta
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int ch = ch0 + k;
      if (ch < c) {
        const int g = ch / cpg;
        const float mean = stats[((int64_t)nn * groups + g) * 2 + 0];
        const float rstd = stats[((int64_t)nn * groups + g) * 2 + 1];
        mu[k] = mean;
        sc[k] = rstd * gamma[ch];
        sh[k] = beta[ch];
      } else {
        mu[k] = 0.f;
        sc[k] = 0.f;
        sh[k] = 0.f;
      }
    }
    float res[8];
    auto f = [&](int yy, int xx, float (&r)[8], bool accum) {
      float v[8];
      ld8(y + (((int64_t)nn * h + yy) * w + xx) * c_p + ch0, v);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float t = (v[k] - mu[k]) * sc[k] + sh[k];
        t = t < 0.f ? t * slope : t;
        r[k] = accum ? r[k] + t : t;
      }
    };
    if (pool) {
      f(2 * oy, 2 * ox, res, false);
      f(2 * oy, 2 * ox + 1, res, true);
      f(2 * oy + 1, 2 * ox, res, true);
      f(2 * oy + 1, 2 * ox + 1, res, true);
#pragma unroll
      for (int k = 0; k < 8; ++k) res[k] = res[k] / 4.f;
    } else {
      f(oy, ox, res, false);
    }
    st8p(out, pix, c_p, ch0, res);
  }
}

// Sample-major variant for power-of-two channel-octet counts: blockIdx.y = sample, each thread keeps one
// channel octet (its GN mean / scale / shift loaded once) and strides over pixels with 32-bit index math
// (the generic kernel above pays 64-bit div/mod and 24 parameter loads per 8 outputs)
template <typename TI, typename TO, bool POOL>
__global__ void __launch_bounds__(256) gn_apply_oct_kernel(const TI* __restrict__ y, TO* __restrict__ out, int h,
                                                           int w, int c_p, int c, int groups,
                                                           const float* __restrict__ stats,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta, float slope) {
  const int nn = blockIdx.y;
  const int c8 = c_p >> 3;
  const int oct = threadIdx.x & (c8 - 1);
  const int ppi = 256 / c8;
  const int prow = threadIdx.x / c8;
  const int oh = POOL ? h / 2 : h, ow = POOL ? w / 2 : w;
  const int ohw = oh * ow;
  const int ch0 = oct * 8;
  const int cpg = c / groups;
  float mu[8], sc[8], sh[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int ch = ch0 + k;
    if (ch < c) {
      const int g = ch / cpg;
      mu[k] = stats[((int64_t)nn * groups + g) * 2 + 0];
      sc[k] = stats[((int64_t)nn * groups + g) * 2 + 1] * gamma[ch];
      sh[k] = beta[ch];
    } else {
      mu[k] = 0.f;
      sc[k] = 0.f;
      sh[k] = 0.f;
    }
  }
  const TI* yb = y + (int64_t)nn * h * w * c_p + ch0;
  for (int pix = blockIdx.x * ppi + prow; pix < ohw; pix += gridDim.x * ppi) {
    float res[8];
    auto f = [&](int idx, bool accum) {
      float v[8];
      ld8(yb + (int64_t)idx * c_p, v);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float t = __builtin_fmaf(v[k] - mu[k], sc[k], sh[k]);  // as gn_lrelu_bf16x8 (igemm.hip), bit for bit
        t = t < 0.f ? t * slope : t;
        res[k] = accum ? res[k] + t : t;
      }
    };
    if constexpr (POOL) {
      const int oy = pix / ow, ox = pix - oy * ow;
      const int i0 = (2 * oy) * w + 2 * ox;
      f(i0, false);
      f(i0 + 1, true);
      f(i0 + w, true);
      f(i0 + w + 1, true);
#pragma unroll
      for (int k = 0; k < 8; ++k) res[k] = res[k] / 4.f;
    } else {
      f(pix, false);
    }
    st8p(out, (int64_t)nn * ohw + pix, c_p, ch0, res);
  }
}

// ------------------------------------------------------------------------------------------------
// global average pool: stage 1 per (n, chunk) channel partials, stage 2 ordered chunk sum
// ------------------------------------------------------------------------------------------------
constexpr int GAP_CHUNK = 64;

template <typename T>
__global__ void __launch_bounds__(256) gap_partial_kernel(const T* __restrict__ x, int hw, int c_p, int nchunks,
                                                          float* __restrict__ part) {
  const int chunk = blockIdx.y;
  const int nn = blockIdx.z;
  const int ch = blockIdx.x * 256 + threadIdx.x;
  if (ch >= c_p) return;
  const int p0 = chunk * GAP_CHUNK, p1 = min(hw, p0 + GAP_CHUNK);
  float s = 0.f;
  if constexpr (std::is_same<T, bf16x3_t>::value) {
    const bf16_t* xb = reinterpret_cast<const bf16_t*>(x);
    for (int p = p0; p < p1; ++p) {
      const bf16_t* px = xb + ((int64_t)nn * hw + p) * 2 * c_p + ch;
      s += bf2f(px[0]) + bf2f(px[c_p]);
    }
  } else {
    for (int p = p0; p < p1; ++p) s += ld(x + ((int64_t)nn * hw + p) * c_p + ch);
  }
  part[((int64_t)nn * nchunks + chunk) * c_p + ch] = s;
}

// grid (ceil(c / 16), n): 16 channels x 16 chunk lanes per block (the 1024^2 encoder's fine projector has 256+
// chunks per image: one thread per (n, c) summing them in sequence was a serial chain of loads); each lane sums
// chunks lane, lane + 16, ... and the lanes combine in a fixed order (deterministic)
__global__ void __launch_bounds__(256) gap_finalize_kernel(const float* __restrict__ part, int n, int c_p, int c,
                                                           int nchunks, int hw, float* __restrict__ out) {
  __shared__ float red[16][17];
  const int nn = blockIdx.y, cl = threadIdx.x & 15, lane = threadIdx.x >> 4;
  const int ch = blockIdx.x * 16 + cl;
  float s = 0.f;
  if (ch < c)
    for (int k = lane; k < nchunks; k += 16) s += part[((int64_t)nn * nchunks + k) * c_p + ch];
  red[lane][cl] = s;
  __syncthreads();
  if (lane == 0 && ch < c) {
    float t = 0.f;
#pragma unroll
    for (int l = 0; l < 16; ++l) t += red[l][cl];
    out[(int64_t)nn * c + ch] = t / (float)hw;
  }
}

// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) reparam_kernel(const float* __restrict__ params, const float* __restrict__ eps,
                                                      int n, int num_ws, int w_dim, int ws_total, int ws_off,
                                                      float* __restrict__ w_out, float* __restrict__ mean_out,
                                                      float* __restrict__ logvar_out) {
#pragma clang fp contract(off)  // mean + eps * std as two roundings, like the reference's torch ops (:243-245)
  const int64_t total = (int64_t)n * num_ws * w_dim;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int d = (int)(e % w_dim);
    const int64_t r = e / w_dim;
    const int s = (int)(r % num_ws);
    const int64_t nn = r / num_ws;
    const float m = params[r * 2 * w_dim + d];
    const float lv = params[r * 2 * w_dim + w_dim + d];
    const int64_t o = (nn * ws_total + ws_off + s) * w_dim + d;
    if (mean_out) mean_out[o] = m;
    if (logvar_out) logvar_out[o] = lv;
    if (w_out) {
      const float sd = expf(0.5f * lv);
      w_out[o] = eps ? m + eps[e] * sd : m;
    }
  }
}

// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ int to_u8(float v) {
#pragma clang fp contract(off)  // (x * 0.5 + 0.5) as two roundings (hvae_training.py:368-388)
  float t = v * 0.5f + 0.5f;
  t = fminf(fmaxf(t, 0.f), 1.f);
  return (int)(t * 255.f);  // truncation, as numpy astype(np.uint8) on [0, 255]
}

// stage 1: per (image, chunk) partial sums (each thread: float4 loads, exact integer squares summed in
// f64); stage 2: per image ordered sum over the chunks.  Deterministic, no atomics.
constexpr int SSE_CHUNKS = 64;

__global__ void __launch_bounds__(256) uint8_sse_partial_kernel(const float* __restrict__ a,
                                                                const float* __restrict__ b, int64_t per_img,
                                                                int vec, double* __restrict__ part) {
  __shared__ double red[4];
  const int chunk = blockIdx.x, img = blockIdx.y;
  const int64_t len = ceil_div(ceil_div(per_img, SSE_CHUNKS), 4) * 4;
  const int64_t i0 = (int64_t)chunk * len, i1 = min(per_img, i0 + len);
  const float* pa = a + (int64_t)img * per_img;
  const float* pb = b + (int64_t)img * per_img;
  double acc = 0.0;
  if (vec) {
    for (int64_t i = i0 + 4 * threadIdx.x; i < i1; i += 1024) {
      const float4 u = *reinterpret_cast<const float4*>(pa + i), v = *reinterpret_cast<const float4*>(pb + i);
      const int d0 = to_u8(u.x) - to_u8(v.x), d1 = to_u8(u.y) - to_u8(v.y);
      const int d2 = to_u8(u.z) - to_u8(v.z), d3 = to_u8(u.w) - to_u8(v.w);
      acc += (double)(d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3);
    }
  } else {
    for (int64_t i = i0 + threadIdx.x; i < i1; i += 256) {
      const int d = to_u8(pa[i]) - to_u8(pb[i]);
      acc += (double)(d * d);
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[(int64_t)img * SSE_CHUNKS + chunk] = ((red[0] + red[1]) + red[2]) + red[3];
}

__global__ void __launch_bounds__(256) uint8_sse_finalize_kernel(const double* __restrict__ part, int64_t n_img,
                                                                 double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n_img) return;
  double s = 0.0;
  for (int k = 0; k < SSE_CHUNKS; ++k) s += part[i * SSE_CHUNKS + k];
  out[i] = s;
}

// F.interpolate(bilinear, align_corners=False): src = max(0, (dst + 0.5) * in/out - 0.5)
__global__ void __launch_bounds__(256) resize_bilinear_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                              int64_t nc, int h, int w, int oh, int ow) {
  const int64_t total = nc * oh * ow;
  const float sh = (float)h / (float)oh, sw = (float)w / (float)ow;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int ox = (int)(e % ow);
    const int oy = (int)((e / ow) % oh);
    const int64_t pl = e / ((int64_t)ow * oh);
    float sy = fmaxf(sh * (oy + 0.5f) - 0.5f, 0.f);
    float sx = fmaxf(sw * (ox + 0.5f) - 0.5f, 0.f);
    const int y0 = (int)sy, x0 = (int)sx;
    const int y1 = y0 + (y0 < h - 1 ? 1 : 0), x1 = x0 + (x0 < w - 1 ? 1 : 0);
    const float ly = sy - y0, lx = sx - x0;
    const float* p = x + pl * h * w;
    const float v = (1.f - ly) * ((1.f - lx) * p[y0 * w + x0] + lx * p[y0 * w + x1]) +
                    ly * ((1.f - lx) * p[y1 * w + x0] + lx * p[y1 * w + x1]);
    y[e] = v;
  }
}

// igemm.hip: the conv with the GroupNorm partial sums fused into the halo conv's epilogue
int conv_gn_fused(const void* x, const void* w, void* y, int dtype, int n, int h, int w_, int cin_p, int cout_p,
                  int cout_valid, int kh, int kw, int pad, const float* bias, int groups, double* part,
                  int64_t part_doubles, void* workspace, int64_t ws_bytes, int fuse_mode, hipStream_t s,
                  const float* in_gn, float in_slope, float out_mul = 1.f);
bool conv_gn_in_supported(int dtype, int n, int h, int w_, int cin_p, int cout_p, int kh, int kw, int pad);
bool conv_gn_fuses(int dtype, int n, int h, int w_, int cin_p, int cout_p, int cout_valid, int kh, int kw, int pad,
                   int groups, int fuse_mode);
int64_t conv_gn_fused_part_doubles(int dtype, int n, int h, int w_, int cin_p, int cout_p, int kh, int kw, int pad,
                                   int groups);

}  // namespace ic2

using namespace ic2;

extern "C" int ic2_nchw_to_nhwc(const float* x, void* y, int dtype, int n, int c, int h, int w, int c_p,
                                const float* scale, void* stream) {
  IC2_CHECK_ARG(x && y && n > 0 && c > 0 && h > 0 && w > 0 && c_p >= c, "nchw_to_nhwc: bad arguments");
  const int64_t total = (int64_t)n * h * w * c_p;
  hipStream_t s = as_stream(stream);
  if (dtype == IC2_F32)
    hipLaunchKernelGGL(nchw_to_nhwc_kernel<float>, dim3(grid_1d(total)), dim3(256), 0, s, x, (float*)y, n, c, h * w, c_p,
                       scale);
  else if (dtype == IC2_BF16)
    hipLaunchKernelGGL(nchw_to_nhwc_kernel<bf16_t>, dim3(grid_1d(total)), dim3(256), 0, s, x, (bf16_t*)y, n, c, h * w,
                       c_p, scale);
  else if (dtype == IC2_F16)
    hipLaunchKernelGGL(nchw_to_nhwc_kernel<_Float16>, dim3(grid_1d(total)), dim3(256), 0, s, x, (_Float16*)y, n, c,
                       h * w, c_p, scale);
  else if (dtype == IC2_BF16X3)
    hipLaunchKernelGGL(nchw_to_nhwc_x3_kernel, dim3(grid_1d(total)), dim3(256), 0, s, x, (bf16_t*)y, n, c, h * w, c_p,
                       scale);
  else
    IC2_CHECK_ARG(false, "nchw_to_nhwc: bad dtype");
  IC2_CHECK_LAUNCH("nchw_to_nhwc");
  return IC2_OK;
}

// ------------------------------------------------------------------------------------------------
// from_rgb straight from the NCHW f32 image (HVAE_VGG_Encoder.from_rgb, stylegan3_hvae_full.py:62,175):
// 3x3, pad 1, cin <= 4, bias, bf16 NHWC [n][h][w][COUT] out.  The MFMA path first packs the image to a
// 32-channel bf16 NHWC tensor (10x the bytes of the 3-channel image) and then reads it back; here a workgroup
// stages its (8+2) x (32+2) x cin input tile in LDS (rounded to bf16 exactly as that packing does) and each
// thread computes one pixel's COUT outputs with packed FMAs against the bf16 weights held in LDS (broadcast
// reads).  Arithmetic: bf16 operands, f32 sums (tap order), + bias, one bf16 rounding -- as the MFMA conv.
// ------------------------------------------------------------------------------------------------
// X3 (the encoder's split-bf16 mode, ic2_from_rgb_conv_x3): wp is the nn.Conv2d weight itself (f32 [cout][cin][3][3],
// `cin_p` = cout there), the image is not rounded, and the f32 result is stored split ([hi | lo], 2 * COUT); H16
// (with X3: ic2_from_rgb_conv_f16) stores that f32 result rounded to f16 instead (COUT channels).
template <int COUT, bool X3 = false, bool H16 = false>
__global__ void __launch_bounds__(256) from_rgb_kernel(const float* __restrict__ x, int cin, const void* __restrict__ wp,
                                                       int cin_p, const float* __restrict__ bias, bf16_t* __restrict__ y,
                                                       int h, int w, int tiles_x, int tiles_y) {
  static_assert(X3 || !H16, "the f16 output is the f32-weight (X3) kernel's");
  constexpr int TH = 8, TW = 32, HH = TH + 2, HW = TW + 2;
  __shared__ float xin[4][HH][HW + 1];
  __shared__ __attribute__((aligned(16))) float wl[36][COUT];  // [tap * cin + c][o]
  const int t = threadIdx.x;
  int b = blockIdx.x;
  const int tx = b % tiles_x;
  b /= tiles_x;
  const int ty = b % tiles_y;
  const int nn = b / tiles_y;
  const int oy0 = ty * TH, ox0 = tx * TW;
  const int nk = 9 * cin;
  for (int e = t; e < nk * COUT; e += 256) {
    const int o = e % COUT, k = e / COUT;
    const int tap = k / cin, c = k - (k / cin) * cin;
    if constexpr (X3)
      wl[k][o] = o < cin_p ? reinterpret_cast<const float*>(wp)[((int64_t)o * cin + c) * 9 + tap] : 0.f;
    else
      wl[k][o] = bf2f(reinterpret_cast<const bf16_t*>(wp)[((int64_t)o * 9 + tap) * cin_p + c]);
  }
  for (int e = t; e < cin * HH * HW; e += 256) {
    const int c = e / (HH * HW), r = e - c * (HH * HW);
    const int yy = r / HW, xx = r - (r / HW) * HW;
    const int iy = oy0 - 1 + yy, ix = ox0 - 1 + xx;
    float v = 0.f;
    if ((unsigned)iy < (unsigned)h && (unsigned)ix < (unsigned)w) {
      v = x[(((int64_t)nn * cin + c) * h + iy) * w + ix];
      if constexpr (!X3) v = bf2f(f2bf(v));
    }
    xin[c][yy][xx] = v;
  }
  __syncthreads();
  const int py = t >> 5, px = t & 31;
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 acc[COUT / 2];
#pragma unroll
  for (int o = 0; o < COUT / 2; ++o) acc[o] = f2{0.f, 0.f};
  for (int tap = 0; tap < 9; ++tap) {
    const int ky = tap / 3, kx = tap - (tap / 3) * 3;
    for (int c = 0; c < cin; ++c) {
      const float xv = xin[c][py + ky][px + kx];
      const f2 xx = f2{xv, xv};
      const float4* wr = reinterpret_cast<const float4*>(&wl[tap * cin + c][0]);
#pragma unroll
      for (int q = 0; q < COUT / 4; ++q) {
        const float4 wv = wr[q];
        acc[2 * q] = __builtin_elementwise_fma(xx, f2{wv.x, wv.y}, acc[2 * q]);
        acc[2 * q + 1] = __builtin_elementwise_fma(xx, f2{wv.z, wv.w}, acc[2 * q + 1]);
      }
    }
  }
  const int oy = oy0 + py, ox = ox0 + px;
  if (oy >= h || ox >= w) return;
  if constexpr (H16) {
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    uint16_t* yo = reinterpret_cast<uint16_t*>(y) + (((int64_t)nn * h + oy) * w + ox) * COUT;
#pragma unroll
    for (int q = 0; q < COUT / 8; ++q) {
      uint32_t u[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int o = 8 * q + 2 * k;
        u[k] = __builtin_bit_cast(uint32_t, h2{(_Float16)(acc[o / 2].x + bias[o]), (_Float16)(acc[o / 2].y + bias[o + 1])});
      }
      reinterpret_cast<uint4*>(yo)[q] = make_uint4(u[0], u[1], u[2], u[3]);
    }
    return;
  } else if constexpr (X3) {
    bf16_t* yo = y + (((int64_t)nn * h + oy) * w + ox) * 2 * COUT;
#pragma unroll
    for (int q = 0; q < COUT / 8; ++q) {
      uint32_t hw_[4], lw_[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int o = 8 * q + 2 * k;
        bf16_t h0, l0, h1, l1;
        split_bf16(acc[o / 2].x + bias[o], h0, l0);
        split_bf16(acc[o / 2].y + bias[o + 1], h1, l1);
        hw_[k] = (uint32_t)h0 | ((uint32_t)h1 << 16);
        lw_[k] = (uint32_t)l0 | ((uint32_t)l1 << 16);
      }
      reinterpret_cast<uint4*>(yo)[q] = make_uint4(hw_[0], hw_[1], hw_[2], hw_[3]);
      reinterpret_cast<uint4*>(yo + COUT)[q] = make_uint4(lw_[0], lw_[1], lw_[2], lw_[3]);
    }
    return;
  }
  bf16_t* yo = y + (((int64_t)nn * h + oy) * w + ox) * COUT;
#pragma unroll
  for (int q = 0; q < COUT / 8; ++q) {
    uint4 pk;
    uint32_t u[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int o = 8 * q + 2 * k;
      u[k] = (uint32_t)f2bf(acc[o / 2].x + bias[o]) | ((uint32_t)f2bf(acc[o / 2].y + bias[o + 1]) << 16);
    }
    pk.x = u[0]; pk.y = u[1]; pk.z = u[2]; pk.w = u[3];
    reinterpret_cast<uint4*>(yo)[q] = pk;
  }
}

extern "C" int ic2_from_rgb_conv(const float* x, int cin, const void* w, int cin_p, const float* bias, void* y, int n,
                                 int h, int w_, int cout_p, void* stream) {
  IC2_CHECK_ARG(x && w && bias && y && n > 0 && h > 0 && w_ > 0, "from_rgb_conv: null pointer / bad geometry");
  IC2_CHECK_ARG(cin >= 1 && cin <= 4 && cin_p >= cin && (cout_p == 32 || cout_p == 64),
                "from_rgb_conv: needs 1 <= cin <= 4 and cout_p in {32, 64} (cin=%d cout_p=%d)", cin, cout_p);
  IC2_CHECK_ARG((uintptr_t)y % 16 == 0, "from_rgb_conv: output must be 16-byte aligned");
  const int tiles_x = (w_ + 31) / 32, tiles_y = (h + 7) / 8;
  const int64_t blocks = (int64_t)n * tiles_x * tiles_y;
  IC2_CHECK_ARG(blocks < (1LL << 31), "from_rgb_conv: too many tiles");
  hipStream_t s = as_stream(stream);
  if (cout_p == 32)
    hipLaunchKernelGGL(from_rgb_kernel<32>, dim3((unsigned)blocks), dim3(256), 0, s, x, cin, w, cin_p, bias,
                       (bf16_t*)y, h, w_, tiles_x, tiles_y);
  else
    hipLaunchKernelGGL(from_rgb_kernel<64>, dim3((unsigned)blocks), dim3(256), 0, s, x, cin, w, cin_p, bias,
                       (bf16_t*)y, h, w_, tiles_x, tiles_y);
  IC2_CHECK_LAUNCH("from_rgb_conv");
  return IC2_OK;
}

extern "C" int ic2_from_rgb_conv_x3(const float* x, int cin, const float* w, int cout, const float* bias, void* y, int n,
                                    int h, int w_, int cout_p, void* stream) {
  IC2_CHECK_ARG(x && w && bias && y && n > 0 && h > 0 && w_ > 0, "from_rgb_conv_x3: null pointer / bad geometry");
  IC2_CHECK_ARG(cin >= 1 && cin <= 4 && cout >= 1 && cout <= cout_p && (cout_p == 32 || cout_p == 64 || cout_p == 128),
                "from_rgb_conv_x3: needs 1 <= cin <= 4, cout <= cout_p, cout_p in {32, 64, 128} (cin=%d cout=%d cout_p=%d)",
                cin, cout, cout_p);
  IC2_CHECK_ARG((uintptr_t)y % 16 == 0, "from_rgb_conv_x3: output must be 16-byte aligned");
  const int tiles_x = (w_ + 31) / 32, tiles_y = (h + 7) / 8;
  const int64_t blocks = (int64_t)n * tiles_x * tiles_y;
  IC2_CHECK_ARG(blocks < (1LL << 31), "from_rgb_conv_x3: too many tiles");
  hipStream_t s = as_stream(stream);
  if (cout_p == 32)
    hipLaunchKernelGGL((from_rgb_kernel<32, true>), dim3((unsigned)blocks), dim3(256), 0, s, x, cin, w, cout, bias,
                       (bf16_t*)y, h, w_, tiles_x, tiles_y);
  else if (cout_p == 64)
    hipLaunchKernelGGL((from_rgb_kernel<64, true>), dim3((unsigned)blocks), dim3(256), 0, s, x, cin, w, cout, bias,
                       (bf16_t*)y, h, w_, tiles_x, tiles_y);
  else
    hipLaunchKernelGGL((from_rgb_kernel<128, true>), dim3((unsigned)blocks), dim3(256), 0, s, x, cin, w, cout, bias,
                       (bf16_t*)y, h, w_, tiles_x, tiles_y);
  IC2_CHECK_LAUNCH("from_rgb_conv_x3");
  return IC2_OK;
}

extern "C" int ic2_from_rgb_conv_f16(const float* x, int cin, const float* w, int cout, const float* bias, void* y, int n,
                                     int h, int w_, int cout_p, void* stream) {
  IC2_CHECK_ARG(x && w && bias && y && n > 0 && h > 0 && w_ > 0, "from_rgb_conv_f16: null pointer / bad geometry");
  IC2_CHECK_ARG(cin >= 1 && cin <= 4 && cout >= 1 && cout <= cout_p && (cout_p == 32 || cout_p == 64 || cout_p == 128),
                "from_rgb_conv_f16: needs 1 <= cin <= 4, cout <= cout_p, cout_p in {32, 64, 128} (cin=%d cout=%d cout_p=%d)",
                cin, cout, cout_p);
  IC2_CHECK_ARG((uintptr_t)y % 16 == 0, "from_rgb_conv_f16: output must be 16-byte aligned");
  const int tiles_x = (w_ + 31) / 32, tiles_y = (h + 7) / 8;
  const int64_t blocks = (int64_t)n * tiles_x * tiles_y;
  IC2_CHECK_ARG(blocks < (1LL << 31), "from_rgb_conv_f16: too many tiles");
  hipStream_t s = as_stream(stream);
  if (cout_p == 32)
    hipLaunchKernelGGL((from_rgb_kernel<32, true, true>), dim3((unsigned)blocks), dim3(256), 0, s, x, cin, w, cout, bias,
                       (bf16_t*)y, h, w_, tiles_x, tiles_y);
  else if (cout_p == 64)
    hipLaunchKernelGGL((from_rgb_kernel<64, true, true>), dim3((unsigned)blocks), dim3(256), 0, s, x, cin, w, cout, bias,
                       (bf16_t*)y, h, w_, tiles_x, tiles_y);
  else
    hipLaunchKernelGGL((from_rgb_kernel<128, true, true>), dim3((unsigned)blocks), dim3(256), 0, s, x, cin, w, cout,
                       bias, (bf16_t*)y, h, w_, tiles_x, tiles_y);
  IC2_CHECK_LAUNCH("from_rgb_conv_f16");
  return IC2_OK;
}

extern "C" int ic2_nhwc_to_nchw(const void* x, int dtype, float* y, int n, int c, int h, int w, int c_p, void* stream) {
  IC2_CHECK_ARG(x && y && n > 0 && c > 0 && h > 0 && w > 0 && c_p >= c, "nhwc_to_nchw: bad arguments");
  const int64_t total = (int64_t)n * h * w * c;
  hipStream_t s = as_stream(stream);
  if (dtype == IC2_F32)
    hipLaunchKernelGGL(nhwc_to_nchw_kernel<float>, dim3(grid_1d(total)), dim3(256), 0, s, (const float*)x, y, n, c, h * w,
                       c_p);
  else if (dtype == IC2_BF16)
    hipLaunchKernelGGL(nhwc_to_nchw_kernel<bf16_t>, dim3(grid_1d(total)), dim3(256), 0, s, (const bf16_t*)x, y, n, c,
                       h * w, c_p);
  else if (dtype == IC2_F16)
    hipLaunchKernelGGL(nhwc_to_nchw_kernel<_Float16>, dim3(grid_1d(total)), dim3(256), 0, s, (const _Float16*)x, y, n,
                       c, h * w, c_p);
  else
    IC2_CHECK_ARG(false, "nhwc_to_nchw: bad dtype");
  IC2_CHECK_LAUNCH("nhwc_to_nchw");
  return IC2_OK;
}

extern "C" int64_t ic2_group_norm_stats_floats(int n, int hw, int groups) {
  const int64_t stats_floats = ((int64_t)n * groups * 2 + 1) / 2 * 2;
  return stats_floats + (int64_t)n * groups * ceil_div(hw, gn_chunk_pix(n, hw)) * 2 * 2;
}

extern "C" int ic2_group_norm_stats(const void* y, int dtype, int n, int hw, int c_p, int c, int groups, float eps,
                                    float* stats_out, void* stream) {
  IC2_CHECK_ARG(y && stats_out && n > 0 && hw > 0 && c > 0 && groups > 0 && c % groups == 0 && c_p >= c,
                "group_norm_stats: bad arguments");
  IC2_CHECK_ARG(c_p % 2 == 0, "group_norm_stats: c_p must be even");
  const int chunk_pix = gn_chunk_pix(n, hw);
  const int nchunks = (int)ceil_div(hw, chunk_pix);
  // partials live right after the stats (8-byte aligned)
  const int64_t stats_floats = ((int64_t)n * groups * 2 + 1) / 2 * 2;
  double* part = reinterpret_cast<double*>(stats_out + stats_floats);
  hipStream_t s = as_stream(stream);
  const size_t lds = 2 * (size_t)(c_p < 512 ? 512 : c_p) * sizeof(double);
  if (dtype == IC2_F32)
    hipLaunchKernelGGL(gn_partial_kernel<float>, dim3(n * nchunks), dim3(256), lds, s, (const float*)y, hw, c_p, c,
                       groups, nchunks, chunk_pix, part);
  else if (dtype == IC2_BF16)
    hipLaunchKernelGGL(gn_partial_kernel<bf16_t>, dim3(n * nchunks), dim3(256), lds, s, (const bf16_t*)y, hw, c_p, c,
                       groups, nchunks, chunk_pix, part);
  else if (dtype == IC2_F16)
    hipLaunchKernelGGL(gn_partial_kernel<_Float16>, dim3(n * nchunks), dim3(256), lds, s, (const _Float16*)y, hw, c_p,
                       c, groups, nchunks, chunk_pix, part);
  else
    IC2_CHECK_ARG(false, "group_norm_stats: bad dtype");
  hipLaunchKernelGGL(gn_finalize_kernel, dim3((unsigned)(n * groups)), dim3(64), 0, s, part, n * groups,
                     nchunks, (double)hw * (c / groups), eps, stats_out);
  IC2_CHECK_LAUNCH("group_norm_stats");
  return IC2_OK;
}

extern "C" int64_t ic2_conv3x3_gn_stats_floats(int dtype, int n, int h, int w_, int cin_p, int cout_p, int kh, int kw,
                                               int pad, int groups) {
  const int ho = h + 2 * pad - kh + 1, wo = w_ + 2 * pad - kw + 1;
  if (n <= 0 || ho <= 0 || wo <= 0 || groups <= 0) return 0;
  const int64_t sep = ic2_group_norm_stats_floats(n, ho * wo, groups);
  const int64_t stats_floats = ((int64_t)n * groups * 2 + 1) / 2 * 2;
  const int64_t fused = stats_floats + 2 * conv_gn_fused_part_doubles(dtype, n, h, w_, cin_p, cout_p, kh, kw, pad, groups);
  return sep > fused ? sep : fused;
}

// VGGBlock conv (+ bias) and the GroupNorm statistics of its output.  When the halo
// conv runs the layer, the per-tile (sum, sumsq) come out of its epilogue (no second read of y); otherwise the
// separate two-stage statistics pass runs.  stats: ic2_conv3x3_gn_stats_floats() floats; the first n*groups*2 are
// (mean, rstd) per (sample, group), as ic2_group_norm_stats writes them.
static int conv3x3_gn_fwd_impl(const void* x, const void* w, void* y, int dtype, int n, int h, int w_, int cin_p,
                               int cout_p, int cout_valid, int kh, int kw, int pad, const float* bias, int groups,
                               float eps, float* stats, int64_t stats_floats, void* conv_ws, int64_t conv_ws_bytes,
                               int fuse, void* stream, const float* in_gn, float in_slope, float out_mul = 1.f) {
  IC2_CHECK_ARG(x && w && y && stats && groups > 0 && cout_valid > 0 && cout_valid % groups == 0,
                "conv3x3_gn_fwd: bad arguments");
  // the encoder's precisions only: the fused statistics epilogue and the input-GroupNorm staging are bf16 halo-conv
  // code, and an f16 operand must never reach the bf16 MFMA
  IC2_CHECK_ARG(dtype == IC2_F32 || dtype == IC2_BF16 || dtype == IC2_BF16X3 || dtype == IC2_F16X2,
                "conv3x3_gn_fwd: dtype must be IC2_F32, IC2_BF16, IC2_BF16X3 or IC2_F16X2");
  const int ho = h + 2 * pad - kh + 1, wo = w_ + 2 * pad - kw + 1;
  IC2_CHECK_ARG(stats_floats >= ic2_conv3x3_gn_stats_floats(dtype, n, h, w_, cin_p, cout_p, kh, kw, pad, groups),
                "conv3x3_gn_fwd: stats buffer too small");
  hipStream_t s = as_stream(stream);
  const int64_t sf = ((int64_t)n * groups * 2 + 1) / 2 * 2;
  double* part = reinterpret_cast<double*>(stats + sf);
  const int nch = conv_gn_fused(x, w, y, dtype, n, h, w_, cin_p, cout_p, cout_valid, kh, kw, pad, bias, groups, part,
                                (stats_floats - sf) / 2, conv_ws, conv_ws_bytes, fuse, s, in_gn, in_slope, out_mul);
  if (nch == -2) return IC2_E_UNSUPPORTED;
  if (nch < 0) return IC2_E_INVALID;
  if (nch == 0)  // split inputs: the conv wrote f32 (split bf16) / f16 (split-weight f16)
    return ic2_group_norm_stats(y, dtype == IC2_BF16X3 ? IC2_F32 : dtype == IC2_F16X2 ? IC2_F16 : dtype, n, ho * wo, cout_p, cout_valid, groups, eps,
                                stats, stream);
  hipLaunchKernelGGL(gn_finalize_kernel, dim3((unsigned)(n * groups)), dim3(64), 0, s, part, n * groups, nch,
                     (double)ho * wo * (cout_valid / groups), eps, stats);
  IC2_CHECK_LAUNCH("conv3x3_gn_fwd");
  return IC2_OK;
}

extern "C" int ic2_conv3x3_gn_fuses(int dtype, int n, int h, int w_, int cin_p, int cout_p, int cout_valid, int kh,
                                    int kw, int pad, int groups, int fuse) {
  return conv_gn_fuses(dtype, n, h, w_, cin_p, cout_p, cout_valid, kh, kw, pad, groups, fuse) ? 1 : 0;
}

extern "C" int ic2_conv3x3_gn_fwd(const void* x, const void* w, void* y, int dtype, int n, int h, int w_, int cin_p,
                                  int cout_p, int cout_valid, int kh, int kw, int pad, const float* bias, int groups,
                                  float eps, float* stats, int64_t stats_floats, void* conv_ws, int64_t conv_ws_bytes,
                                  int fuse, void* stream) {
  return conv3x3_gn_fwd_impl(x, w, y, dtype, n, h, w_, cin_p, cout_p, cout_valid, kh, kw, pad, bias, groups, eps, stats,
                             stats_floats, conv_ws, conv_ws_bytes, fuse, stream, nullptr, 0.f);
}

extern "C" int ic2_conv3x3_gn_fwd_scaled(const void* x, const void* w, void* y, int dtype, int n, int h, int w_,
                                         int cin_p, int cout_p, int cout_valid, int kh, int kw, int pad,
                                         const float* bias, float out_mul, int groups, float eps, float* stats,
                                         int64_t stats_floats, void* conv_ws, int64_t conv_ws_bytes, int fuse,
                                         void* stream) {
  IC2_CHECK_ARG(dtype == IC2_F16X2 && out_mul > 0.f, "conv3x3_gn_fwd_scaled: IC2_F16X2 with out_mul > 0 only");
  return conv3x3_gn_fwd_impl(x, w, y, dtype, n, h, w_, cin_p, cout_p, cout_valid, kh, kw, pad, bias, groups, eps, stats,
                             stats_floats, conv_ws, conv_ws_bytes, fuse, stream, nullptr, 0.f, out_mul);
}

// (mean, rstd * gamma, beta, 0) per (sample, channel) from GroupNorm stats [n][groups][2] (mean, rstd): the operands
// of gn_apply_oct_kernel, for a consumer that applies GroupNorm + lrelu while it loads (padded channels: 0)
__global__ void __launch_bounds__(256) gn_affine_table_kernel(const float* __restrict__ stats,
                                                              const float* __restrict__ gamma,
                                                              const float* __restrict__ beta, int n, int c, int c_p,
                                                              int groups, float4* __restrict__ table) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= n * c_p) return;
  const int ch = e % c_p, nn = e / c_p;
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  if (ch < c) {
    const int g = ch / (c / groups);
    v.x = stats[((int64_t)nn * groups + g) * 2 + 0];
    v.y = stats[((int64_t)nn * groups + g) * 2 + 1] * gamma[ch];
    v.z = beta[ch];
  }
  table[e] = v;
}

extern "C" int ic2_gn_affine_table(const float* stats, const float* gamma, const float* beta, int n, int c, int c_p,
                                   int groups, float* table, void* stream) {
  IC2_CHECK_ARG(stats && gamma && beta && table && n > 0 && c > 0 && c <= c_p && groups > 0 && c % groups == 0,
                "gn_affine_table: bad arguments");
  IC2_CHECK_ARG((uintptr_t)table % 16 == 0, "gn_affine_table: table must be 16-byte aligned");
  hipLaunchKernelGGL(gn_affine_table_kernel, dim3((unsigned)ceil_div((int64_t)n * c_p, 256)), dim3(256), 0,
                     as_stream(stream), stats, gamma, beta, n, c, c_p, groups, reinterpret_cast<float4*>(table));
  IC2_CHECK_LAUNCH("gn_affine_table");
  return IC2_OK;
}

extern "C" int ic2_conv3x3_gnin_supported(int dtype, int n, int h, int w_, int cin_p, int cout_p, int kh, int kw,
                                          int pad) {
  return conv_gn_in_supported(dtype, n, h, w_, cin_p, cout_p, kh, kw, pad) ? 1 : 0;
}

extern "C" int ic2_conv3x3_gnin_gn_fwd(const void* x, const float* in_gn, float in_slope, const void* w, void* y,
                                       int dtype, int n, int h, int w_, int cin_p, int cout_p, int cout_valid, int kh,
                                       int kw, int pad, const float* bias, int groups, float eps, float* stats,
                                       int64_t stats_floats, void* conv_ws, int64_t conv_ws_bytes, int fuse,
                                       void* stream) {
  IC2_CHECK_ARG(in_gn != nullptr && (uintptr_t)in_gn % 16 == 0, "conv3x3_gnin_gn_fwd: in_gn must be a 16-byte aligned table");
  return conv3x3_gn_fwd_impl(x, w, y, dtype, n, h, w_, cin_p, cout_p, cout_valid, kh, kw, pad, bias, groups, eps, stats,
                             stats_floats, conv_ws, conv_ws_bytes, fuse, stream, in_gn, in_slope);
}

extern "C" int ic2_gn_lrelu_pool(const void* y, void* out, int dtype_in, int dtype_out, int n, int h, int w, int c_p,
                                 int c, int groups, const float* stats, const float* gamma, const float* beta,
                                 float slope, int pool, void* stream) {
  IC2_CHECK_ARG(y && out && stats && gamma && beta && n > 0 && h > 0 && w > 0 && c_p % 8 == 0 && c <= c_p,
                "gn_lrelu_pool: bad arguments");
  IC2_CHECK_ARG(!pool || (h >= 2 && w >= 2), "gn_lrelu_pool: pooling needs H, W >= 2");
  const int oh = pool ? h / 2 : h, ow = pool ? w / 2 : w;
  const int64_t total = (int64_t)n * oh * ow * (c_p / 8);
  hipStream_t s = as_stream(stream);
  const int c8 = c_p / 8;
  const bool oct = c8 <= 256 && (c8 & (c8 - 1)) == 0 && (int64_t)h * w < (1LL << 31) / c_p;
  const int ohw = oh * ow;
  const unsigned gx = (unsigned)std::max<int64_t>(1, std::min<int64_t>(ceil_div(ohw, 256 / std::max(c8, 1)),
                                                                        ceil_div(4096, n)));
#define IC2_GN_LAUNCH(TI, TO)                                                                                     \
  do {                                                                                                          \
  if (oct && pool)                                                                                              \
    hipLaunchKernelGGL((gn_apply_oct_kernel<TI, TO, true>), dim3(gx, (unsigned)n), dim3(256), 0, s, (const TI*)y,  \
                       (TO*)out, h, w, c_p, c, groups, stats, gamma, beta, slope);                              \
  else if (oct)                                                                                                 \
    hipLaunchKernelGGL((gn_apply_oct_kernel<TI, TO, false>), dim3(gx, (unsigned)n), dim3(256), 0, s, (const TI*)y, \
                       (TO*)out, h, w, c_p, c, groups, stats, gamma, beta, slope);                              \
  else                                                                                                          \
    hipLaunchKernelGGL((gn_apply_kernel<TI, TO>), dim3(grid_1d(total)), dim3(256), 0, s, (const TI*)y, (TO*)out, n, \
                       h, w, c_p, c, groups, stats, gamma, beta, slope, pool);                          \
  } while (0)
  if (dtype_in == IC2_F32 && dtype_out == IC2_F32) IC2_GN_LAUNCH(float, float);
  else if (dtype_in == IC2_BF16 && dtype_out == IC2_BF16) IC2_GN_LAUNCH(bf16_t, bf16_t);
  else if (dtype_in == IC2_BF16 && dtype_out == IC2_F32) IC2_GN_LAUNCH(bf16_t, float);
  else if (dtype_in == IC2_F32 && dtype_out == IC2_BF16) IC2_GN_LAUNCH(float, bf16_t);
  else if (dtype_in == IC2_F32 && dtype_out == IC2_BF16X3) IC2_GN_LAUNCH(float, bf16x3_t);
  else if (dtype_in == IC2_F32 && dtype_out == IC2_F16) IC2_GN_LAUNCH(float, _Float16);
  else if (dtype_in == IC2_F16 && dtype_out == IC2_F16) IC2_GN_LAUNCH(_Float16, _Float16);
  else if (dtype_in == IC2_F16 && dtype_out == IC2_BF16X3) IC2_GN_LAUNCH(_Float16, bf16x3_t);
  else IC2_CHECK_ARG(false, "gn_lrelu_pool: bad dtypes");
#undef IC2_GN_LAUNCH
  IC2_CHECK_LAUNCH("gn_lrelu_pool");
  return IC2_OK;
}

extern "C" int64_t ic2_global_avg_pool_floats(int n, int hw, int c_p, int c) {
  return (int64_t)n * c + (int64_t)n * ceil_div(hw, GAP_CHUNK) * c_p;
}

extern "C" int ic2_global_avg_pool(const void* x, int dtype, int n, int hw, int c_p, int c, float* out, void* stream) {
  IC2_CHECK_ARG(x && out && n > 0 && hw > 0 && c > 0 && c_p >= c, "global_avg_pool: bad arguments");
  const int nchunks = (int)ceil_div(hw, GAP_CHUNK);
  float* part = out + (int64_t)n * c;
  hipStream_t s = as_stream(stream);
  dim3 grid((unsigned)ceil_div(c_p, 256), nchunks, n);
  if (dtype == IC2_F32)
    hipLaunchKernelGGL(gap_partial_kernel<float>, grid, dim3(256), 0, s, (const float*)x, hw, c_p, nchunks, part);
  else if (dtype == IC2_BF16)
    hipLaunchKernelGGL(gap_partial_kernel<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)x, hw, c_p, nchunks, part);
  else if (dtype == IC2_BF16X3)
    hipLaunchKernelGGL(gap_partial_kernel<bf16x3_t>, grid, dim3(256), 0, s, (const bf16x3_t*)x, hw, c_p, nchunks, part);
  else if (dtype == IC2_F16)
    hipLaunchKernelGGL(gap_partial_kernel<_Float16>, grid, dim3(256), 0, s, (const _Float16*)x, hw, c_p, nchunks, part);
  else
    IC2_CHECK_ARG(false, "global_avg_pool: bad dtype");
  hipLaunchKernelGGL(gap_finalize_kernel, dim3((unsigned)ceil_div(c, 16), (unsigned)n), dim3(256), 0, s, part, n, c_p,
                     c, nchunks, hw, out);
  IC2_CHECK_LAUNCH("global_avg_pool");
  return IC2_OK;
}

extern "C" int ic2_reparameterize(const float* params, const float* eps, int n, int num_ws, int w_dim, int ws_total,
                                  int ws_off, float* w_out, float* mean_out, float* logvar_out, void* stream) {
  IC2_CHECK_ARG(params && n > 0 && num_ws > 0 && w_dim > 0 && ws_off >= 0 && ws_off + num_ws <= ws_total,
                "reparameterize: bad arguments");
  const int64_t total = (int64_t)n * num_ws * w_dim;
  hipLaunchKernelGGL(reparam_kernel, dim3(grid_1d(total)), dim3(256), 0, as_stream(stream), params, eps, n, num_ws,
                     w_dim, ws_total, ws_off, w_out, mean_out, logvar_out);
  IC2_CHECK_LAUNCH("reparameterize");
  return IC2_OK;
}

extern "C" int64_t ic2_uint8_sse_scratch_doubles(int64_t n_img) { return n_img * SSE_CHUNKS; }

extern "C" int ic2_uint8_sse(const float* a, const float* b, int64_t n_img, int64_t per_img, double* sse_out,
                             double* scratch, void* stream) {
  IC2_CHECK_ARG(a && b && sse_out && scratch && n_img > 0 && per_img > 0 && n_img < 65536,
                "uint8_sse: bad arguments");
  hipStream_t s = as_stream(stream);
  const int vec = per_img % 4 == 0 && ((uintptr_t)a | (uintptr_t)b) % 16 == 0;
  hipLaunchKernelGGL(uint8_sse_partial_kernel, dim3(SSE_CHUNKS, (unsigned)n_img), dim3(256), 0, s, a, b, per_img, vec,
                     scratch);
  hipLaunchKernelGGL(uint8_sse_finalize_kernel, dim3((unsigned)ceil_div(n_img, 256)), dim3(256), 0, s, scratch, n_img,
                     sse_out);
  IC2_CHECK_LAUNCH("uint8_sse");
  return IC2_OK;
}

extern "C" int ic2_resize_bilinear(const float* x, float* y, int64_t nc, int h, int w, int oh, int ow, void* stream) {
  IC2_CHECK_ARG(x && y && nc > 0 && h > 0 && w > 0 && oh > 0 && ow > 0, "resize_bilinear: bad arguments");
  hipLaunchKernelGGL(resize_bilinear_kernel, dim3(grid_1d(nc * oh * ow)), dim3(256), 0, as_stream(stream), x, y, nc, h,
                     w, oh, ow);
  IC2_CHECK_LAUNCH("resize_bilinear");
  return IC2_OK;
}
