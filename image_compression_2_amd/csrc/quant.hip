// Latent quantizers (HBM-bound, elementwise).
//  - uniform n-bit:   StyleGAN3Compressor.compress, /root/reference/stylegan3_hvae_full.py:313-316
//  - codebook argmin: GumbelSoftmaxDiscretization.forward, gumbel_softmax_compression.py:93-118
//  - codebook lookup: GumbelSoftmaxCompressor.decompress, gumbel_softmax_compression.py:255-259
// Bit-exactness: every expression is evaluated in fp32 in the reference's op order with FP
// contraction disabled (no FMA fusion), rintf = torch.round (half-to-even), IEEE division.
#include "common.h"

namespace ic2 {

#pragma clang fp contract(off)

__device__ __forceinline__ void quant_one(float w, float S, float& q, int32_t& idx) {
  const float ws = (w + 1.0f) * 0.5f;
  const float r = rintf(ws * S);
  q = (r / S) * 2.0f - 1.0f;
  idx = (int32_t)r;
}

__global__ void __launch_bounds__(256) quantize_uniform_kernel(const float* __restrict__ w, int64_t n, float S,
                                                               float* __restrict__ q, int32_t* __restrict__ idx) {
  const int64_t nv = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += stride) {
    const float4 v = reinterpret_cast<const float4*>(w)[i];
    float4 o;
    int4 k;
    quant_one(v.x, S, o.x, k.x);
    quant_one(v.y, S, o.y, k.y);
    quant_one(v.z, S, o.z, k.z);
    quant_one(v.w, S, o.w, k.w);
    reinterpret_cast<float4*>(q)[i] = o;
    if (idx) reinterpret_cast<int4*>(idx)[i] = k;
  }
  // tail
  const int64_t t = (nv << 2) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n && blockIdx.x * blockDim.x + threadIdx.x < 4) {
    float o;
    int32_t k;
    quant_one(w[t], S, o, k);
    q[t] = o;
    if (idx) idx[t] = k;
  }
}

// One thread per latent; the k-entry codebook sits in LDS (broadcast reads).  Exact fp32 |z - c|,
// strict '<' keeps the FIRST minimum exactly like torch.argmin.
__global__ void __launch_bounds__(256) codebook_argmin_kernel(const float* __restrict__ z, int64_t n,
                                                              const float* __restrict__ cb, int k,
                                                              int64_t* __restrict__ idx, float* __restrict__ zq,
                                                              uint32_t* __restrict__ hist) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* scb = smem;
  uint32_t* shist = reinterpret_cast<uint32_t*>(smem + k);
  for (int i = threadIdx.x; i < k; i += blockDim.x) {
    scb[i] = cb[i];
    shist[i] = 0;
  }
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float v = z[i];
    float best = fabsf(v - scb[0]);
    int bi = 0;
    for (int j = 1; j < k; ++j) {
      const float d = fabsf(v - scb[j]);
      if (d < best) {
        best = d;
        bi = j;
      }
    }
    // NaN input: every compare is false -> index 0, matching torch.argmin's NaN-first rule only
    // when z itself is NaN (all distances NaN -> argmin returns 0).
    idx[i] = bi;
    if (zq) zq[i] = scb[bi];
    if (hist) atomicAdd(&shist[bi], 1u);
  }
  if (hist) {
    __syncthreads();
    for (int i = threadIdx.x; i < k; i += blockDim.x)
      if (shist[i]) atomicAdd(&hist[i], shist[i]);
  }
}

__global__ void __launch_bounds__(256) codebook_lookup_kernel(const int64_t* __restrict__ codes, int64_t n,
                                                              const float* __restrict__ cb, int k,
                                                              float* __restrict__ w, int32_t* __restrict__ oob) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t c = codes[i];
    if (c < 0 || c >= k) {
      w[i] = 0.f;
      if (oob) atomicOr(oob, 1);
    } else {
      w[i] = cb[c];
    }
  }
}

static int grid_for(int64_t n, int per_thread) {
  int64_t g = ceil_div(ceil_div(n, per_thread), 256);
  if (g < 1) g = 1;
  if (g > 2048) g = 2048;
  return (int)g;
}

}  // namespace ic2

using namespace ic2;

extern "C" int ic2_quantize_uniform(const float* w, int64_t n, int bits, float* q_out, int32_t* idx_out,
                                    void* stream) {
  IC2_CHECK_ARG(n >= 0, "quantize_uniform: n < 0");
  IC2_CHECK_ARG(bits >= 1 && bits <= 24, "quantize_uniform: bits must be in [1, 24], got %d", bits);
  IC2_CHECK_ARG(n == 0 || (w && q_out), "quantize_uniform: null pointer");
  IC2_CHECK_ARG(((uintptr_t)w | (uintptr_t)q_out | (uintptr_t)idx_out) % 16 == 0,
                "quantize_uniform: pointers must be 16-byte aligned");
  if (n == 0) return IC2_OK;
  const float S = (float)((1 << bits) - 1);
  hipLaunchKernelGGL(quantize_uniform_kernel, dim3(grid_for(n, 4)), dim3(256), 0, as_stream(stream), w, n, S, q_out,
                     idx_out);
  IC2_CHECK_LAUNCH("quantize_uniform");
  return IC2_OK;
}

extern "C" int ic2_quantize_codebook_argmin(const float* z, int64_t n, const float* codebook, int k,
                                            int64_t* idx_out, float* zq_out, uint32_t* hist_out, void* stream) {
  IC2_CHECK_ARG(n >= 0 && k >= 1 && k <= 8192, "codebook_argmin: bad sizes n=%lld k=%d", (long long)n, k);
  IC2_CHECK_ARG(n == 0 || (z && codebook && idx_out), "codebook_argmin: null pointer");
  if (n == 0) return IC2_OK;
  const size_t lds = (size_t)k * 8;
  hipLaunchKernelGGL(codebook_argmin_kernel, dim3(grid_for(n, 1)), dim3(256), lds, as_stream(stream), z, n,
                     codebook, k, idx_out, zq_out, hist_out);
  IC2_CHECK_LAUNCH("codebook_argmin");
  return IC2_OK;
}

extern "C" int ic2_codebook_lookup(const int64_t* codes, int64_t n, const float* codebook, int k, float* w_out,
                                   int32_t* oob_flag, void* stream) {
  IC2_CHECK_ARG(n >= 0 && k >= 1, "codebook_lookup: bad sizes");
  IC2_CHECK_ARG(n == 0 || (codes && codebook && w_out), "codebook_lookup: null pointer");
  if (n == 0) return IC2_OK;
  hipLaunchKernelGGL(codebook_lookup_kernel, dim3(grid_for(n, 1)), dim3(256), 0, as_stream(stream), codes, n,
                     codebook, k, w_out, oob_flag);
  IC2_CHECK_LAUNCH("codebook_lookup");
  return IC2_OK;
}

// ================================================================================================
// Gumbel-softmax quantizer forward (GumbelSoftmaxDiscretization.forward,
// gumbel_softmax_compression.py:73-129) fused per latent: logits = -|z - c|, + Gumbel noise,
// / tau, softmax, optional straight-through hard one-hot, disc = ret @ codebook, exact argmin index,
// and the column sums of ret for the perplexity (avg_probs = ret.mean(0), :126-127).
// One wave per latent, K/64 codebook entries per lane; the reference materialises >= six
// [N*8192, K] fp32 tensors for this -- here nothing but the outputs touches HBM.
// Noise: F.gumbel_softmax draws -log(Exponential(1)) from torch's generator; this kernel draws the
// same distribution from a counter-based Philox4x32-10 stream (seed, offset) -- distribution-equal,
// not stream-equal.  `gumbel_noise` (nullable, [n][k]) replaces the generator for exact testing.
// ================================================================================================
namespace ic2 {

__device__ __forceinline__ uint4 philox4x32_10(uint4 ctr, uint2 key) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * ctr.x;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * ctr.z;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    ctr = make_uint4(hi1 ^ ctr.y ^ key.x, lo1, hi0 ^ ctr.w ^ key.y, lo0);
    key.x += 0x9E3779B9u;
    key.y += 0xBB67AE85u;
  }
  return ctr;
}

__device__ __forceinline__ float gumbel_from_bits(uint32_t r) {
  const float u = ((float)(r >> 8) + 0.5f) * (1.0f / 16777216.0f);  // (0, 1)
  return -logf(-logf(u));
}

template <int KPL>
__global__ void __launch_bounds__(256) gumbel_softmax_kernel(const float* __restrict__ z, int64_t n,
                                                             const float* __restrict__ cb, int k,
                                                             const float* __restrict__ log_tau, float tau_const,
                                                             int hard, uint64_t seed,
                                                             const uint64_t* __restrict__ seed_dev, uint64_t offset,
                                                             const float* __restrict__ noise,
                                                             float* __restrict__ disc, int64_t* __restrict__ idx,
                                                             float* __restrict__ prob_sum) {
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  const float tau = log_tau ? expf(log_tau[0]) : tau_const;
  const float inv_tau = 1.f / tau;
  float c[KPL];
#pragma unroll
  for (int j = 0; j < KPL; ++j) {
    const int kk = lane + 64 * j;
    c[j] = kk < k ? cb[kk] : 0.f;
  }
  float psum[KPL];
#pragma unroll
  for (int j = 0; j < KPL; ++j) psum[j] = 0.f;
  // seed_dev: the seed drawn on the device generator by the caller (no host sync, and torch's CPU stream -- which the
  // reference's fine projector re-creates fc1 from -- is not consumed)
  const uint64_t sd = seed_dev ? seed_dev[0] : seed;
  const uint2 key = make_uint2((uint32_t)sd, (uint32_t)(sd >> 32));
  for (int64_t i = (int64_t)blockIdx.x * 4 + wv; i < n; i += nwaves) {
    const float v = z[i];
    float y[KPL];
    float dmin = INFINITY;
    int imin = 0x7fffffff;
    float ymax = -INFINITY;
    int iymax = 0x7fffffff;
#pragma unroll
    for (int j = 0; j < KPL; ++j) {
      const int kk = lane + 64 * j;
      if (kk < k) {
        const float d = fabsf(v - c[j]);
        if (d < dmin) {  // per-lane entries ascend in kk: strict < keeps the first
          dmin = d;
          imin = kk;
        }
        float g;
        if (noise) {
          g = noise[i * k + kk];
        } else {
          const uint64_t ctr = offset + (uint64_t)i * (uint64_t)k + (uint64_t)kk;
          const uint4 r = philox4x32_10(make_uint4((uint32_t)ctr, (uint32_t)(ctr >> 32), 0u, 0u), key);
          g = gumbel_from_bits(r.x);
        }
        y[j] = (-d + g) * inv_tau;
        if (y[j] > ymax) {
          ymax = y[j];
          iymax = kk;
        }
      } else {
        y[j] = -INFINITY;
      }
    }
    // wave reductions: argmin (first index on ties), max y (first index on ties)
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const float od = __shfl_xor(dmin, off, 64);
      const int oi = __shfl_xor(imin, off, 64);
      if (od < dmin || (od == dmin && oi < imin)) {
        dmin = od;
        imin = oi;
      }
      const float oy = __shfl_xor(ymax, off, 64);
      const int oyi = __shfl_xor(iymax, off, 64);
      if (oy > ymax || (oy == ymax && oyi < iymax)) {
        ymax = oy;
        iymax = oyi;
      }
    }
    float e[KPL];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < KPL; ++j) {
      e[j] = (lane + 64 * j < k) ? expf(y[j] - ymax) : 0.f;
      s += e[j];
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    const float inv_s = 1.f / s;
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < KPL; ++j) {
      const int kk = lane + 64 * j;
      float soft = e[j] * inv_s;
      float ret = soft;
      if (hard) ret = ((kk == iymax ? 1.f : 0.f) - soft) + soft;  // y_hard - y_soft.detach() + y_soft
      if (kk < k) {
        acc += ret * c[j];
        psum[j] += ret;
      }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if (lane == 0) {
      disc[i] = acc;
      if (idx) idx[i] = imin;
    }
  }
  if (prob_sum) {
    __shared__ float sp[4][KPL * 64];
#pragma unroll
    for (int j = 0; j < KPL; ++j) sp[wv][lane + 64 * j] = psum[j];
    __syncthreads();
    for (int kk = threadIdx.x; kk < k; kk += 256) {
      const float t = sp[0][kk] + sp[1][kk] + sp[2][kk] + sp[3][kk];
      if (t != 0.f) atomicAdd(&prob_sum[kk], t);
    }
  }
}

}  // namespace ic2

static int gumbel_softmax_quantize(const float* z, int64_t n, const float* codebook, int k, const float* log_tau,
                                   float tau, int hard, uint64_t seed, const uint64_t* seed_dev, uint64_t offset,
                                   const float* gumbel_noise, float* disc_out, int64_t* idx_out, float* prob_sum_out,
                                   void* stream) {
  IC2_CHECK_ARG(n >= 0 && k >= 1 && k <= 1024, "gumbel_softmax_quantize: need 1 <= k <= 1024 (k=%d)", k);
  IC2_CHECK_ARG(n == 0 || (z && codebook && disc_out), "gumbel_softmax_quantize: null pointer");
  IC2_CHECK_ARG(log_tau || tau > 0.f, "gumbel_softmax_quantize: temperature must be positive");
  if (n == 0) return IC2_OK;
  int64_t g = ic2::ceil_div(n, 4);
  if (g > 4096) g = 4096;
  hipStream_t s = ic2::as_stream(stream);
#define IC2_GS(KPL)                                                                                                   \
  hipLaunchKernelGGL(ic2::gumbel_softmax_kernel<KPL>, dim3((unsigned)g), dim3(256), 0, s, z, n, codebook, k, log_tau, \
                     tau, hard, seed, seed_dev, offset, gumbel_noise, disc_out, idx_out, prob_sum_out)
  if (k <= 64) IC2_GS(1);
  else if (k <= 128) IC2_GS(2);
  else if (k <= 256) IC2_GS(4);
  else if (k <= 512) IC2_GS(8);
  else IC2_GS(16);
#undef IC2_GS
  IC2_CHECK_LAUNCH("gumbel_softmax_quantize");
  return IC2_OK;
}

extern "C" int ic2_gumbel_softmax_quantize(const float* z, int64_t n, const float* codebook, int k,
                                           const float* log_tau, float tau, int hard, uint64_t seed,
                                           uint64_t offset, const float* gumbel_noise, float* disc_out,
                                           int64_t* idx_out, float* prob_sum_out, void* stream) {
  return gumbel_softmax_quantize(z, n, codebook, k, log_tau, tau, hard, seed, nullptr, offset, gumbel_noise, disc_out,
                                 idx_out, prob_sum_out, stream);
}

extern "C" int ic2_gumbel_softmax_quantize_dseed(const float* z, int64_t n, const float* codebook, int k,
                                                 const float* log_tau, float tau, int hard, const int64_t* seed_dev,
                                                 uint64_t offset, const float* gumbel_noise, float* disc_out,
                                                 int64_t* idx_out, float* prob_sum_out, void* stream) {
  IC2_CHECK_ARG(seed_dev != nullptr || gumbel_noise != nullptr || n == 0,
                "gumbel_softmax_quantize_dseed: seed_dev is null");
  return gumbel_softmax_quantize(z, n, codebook, k, log_tau, tau, hard, 0, reinterpret_cast<const uint64_t*>(seed_dev),
                                 offset, gumbel_noise, disc_out, idx_out, prob_sum_out, stream);
}

// ------------------------------------------------------------------------------------------------
// Per-batch code record for the metric all_reduce ([.., n_index_mismatch, hist[256]]; the
// reference's usage / perplexity are over the whole batch, gumbel_softmax_compression.py:121-127).
// kind 0: f32 uniform-quantized latents q (ic2_quantize_uniform's output) -> code round((q + 1) * 0.5 * S), exact for
// q on the grid; kind 1: int64 codebook indices.  counts [k + 2] uint32 (zeroed by the caller) accumulate
// hist[0 .. k), the codes outside [0, k) in counts[k], and the elements differing from `golden` (nullable, same
// kind) in counts[k + 1].  LDS histogram per workgroup, one global (vector) atomic add per bin.
namespace ic2 {
template <int KIND>
__global__ void __launch_bounds__(256) code_record_kernel(const void* __restrict__ codes, const void* __restrict__ golden,
                                                          int64_t n, int k, float S, uint32_t* __restrict__ counts) {
  extern __shared__ uint32_t sh[];
  for (int i = threadIdx.x; i < k + 2; i += 256) sh[i] = 0;
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    int64_t c;
    bool diff = false;
    if constexpr (KIND == 0) {
      const float q = reinterpret_cast<const float*>(codes)[i];
      c = (int64_t)rintf(((q + 1.0f) * 0.5f) * S);
      if (golden) diff = __float_as_uint(q) != __float_as_uint(reinterpret_cast<const float*>(golden)[i]);
    } else {
      c = reinterpret_cast<const int64_t*>(codes)[i];
      if (golden) diff = c != reinterpret_cast<const int64_t*>(golden)[i];
    }
    atomicAdd(&sh[(c >= 0 && c < k) ? (int)c : k], 1u);
    if (diff) atomicAdd(&sh[k + 1], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < k + 2; i += 256)
    if (sh[i]) atomicAdd(&counts[i], sh[i]);
}
}  // namespace ic2

extern "C" int ic2_code_record(const void* codes, int kind, int k, int bits, const void* golden, int64_t n,
                               uint32_t* counts, void* stream) {
  IC2_CHECK_ARG(codes && counts && n >= 0 && k > 0 && k <= 8192 && (kind == 0 || kind == 1),
                "code_record: bad arguments");
  IC2_CHECK_ARG(kind == 1 || (bits >= 1 && bits <= 16 && k == (1 << bits)), "code_record: uniform codes need k = 2^bits");
  if (n == 0) return IC2_OK;
  const int64_t g = ceil_div(n, 256 * 8);
  const unsigned grid = (unsigned)(g < 1024 ? (g < 1 ? 1 : g) : 1024);
  const size_t lds = (size_t)(k + 2) * sizeof(uint32_t);
  const float S = (float)((1 << (kind == 0 ? bits : 1)) - 1);
  if (kind == 0)
    hipLaunchKernelGGL(code_record_kernel<0>, dim3(grid), dim3(256), lds, as_stream(stream), codes, golden, n, k, S,
                       counts);
  else
    hipLaunchKernelGGL(code_record_kernel<1>, dim3(grid), dim3(256), lds, as_stream(stream), codes, golden, n, k, S,
                       counts);
  IC2_CHECK_LAUNCH("code_record");
  return IC2_OK;
}
