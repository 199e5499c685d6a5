// StyleGAN3 synthesis support kernels [SG3-public; call sites /root/reference/stylegan3_hvae_full.py:274,329]:
//   bias_act (generic), upfirdn2d (generic NCHW), FullyConnectedLayer / nn.Linear, weight packing for the
//   MFMA implicit GEMM, modulated_conv2d's (de)modulation coefficients, SynthesisInput Fourier features.
#include "common.h"

namespace ic2 {

// ------------------------------------------------------------------------------------------------
// bias_act: x viewed as [outer, c, inner]
// ------------------------------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(256) bias_act_kernel(const T* __restrict__ x, const float* __restrict__ b,
                                                       T* __restrict__ y, int64_t total, int64_t c, int64_t inner,
                                                       int act, float alpha, float gain, float clamp) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    float v = ld(x + i);
    if (b) v += b[(i / inner) % c];
    if (act == IC2_ACT_LRELU) v = v < 0.f ? v * alpha : v;
    if (gain != 1.f) v *= gain;
    if (clamp >= 0.f) v = fminf(fmaxf(v, -clamp), clamp);
    st(y + i, v);
  }
}

// ------------------------------------------------------------------------------------------------
// upfirdn2d, direct form: out[oy][ox] = sum_{ty,tx} v[oy*dy+ty][ox*dx+tx] * g[ty][tx]
//   v = pad(zero-insert(x)), g = flip(f) * gain (unless flip_filter); only taps that land on a
//   non-inserted sample are visited (stride up).  One thread per output pixel.
// ------------------------------------------------------------------------------------------------
struct UfdArgs {
  int64_t nc;
  int in_h, in_w, out_h, out_w;
  int f_ndim, f_h, f_w;
  int upx, upy, downx, downy, px0, py0;
  int flip;
  float gain_x, gain_y;  // per-axis gains (separable) or gain_x = gain, gain_y = 1 (2-D)
};

template <typename T>
__global__ void __launch_bounds__(256) upfirdn2d_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                        const float* __restrict__ f, UfdArgs a) {
  const int64_t total = a.nc * a.out_h * a.out_w;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int fh = a.f_ndim == 1 ? a.f_w : a.f_h;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int ox = (int)(i % a.out_w);
    const int oy = (int)((i / a.out_w) % a.out_h);
    const int64_t pl = i / ((int64_t)a.out_w * a.out_h);
    const T* xp = x + pl * a.in_h * a.in_w;
    float acc = 0.f;
    for (int ty = 0; ty < fh; ++ty) {
      const int vy = oy * a.downy + ty - a.py0;  // position on the zero-inserted grid
      if (vy < 0 || vy % a.upy) continue;
      const int iy = vy / a.upy;
      if (iy >= a.in_h) continue;
      const int fy = a.flip ? ty : fh - 1 - ty;
      for (int tx = 0; tx < a.f_w; ++tx) {
        const int vx = ox * a.downx + tx - a.px0;
        if (vx < 0 || vx % a.upx) continue;
        const int ix = vx / a.upx;
        if (ix >= a.in_w) continue;
        const int fx = a.flip ? tx : a.f_w - 1 - tx;
        float g;
        if (f == nullptr) g = 1.f;
        else if (a.f_ndim == 1) g = (f[fy] * a.gain_y) * (f[fx] * a.gain_x);
        else g = f[fy * a.f_w + fx] * a.gain_x;
        acc += ld(xp + (int64_t)iy * a.in_w + ix) * g;
      }
    }
    st(y + i, acc);
  }
}

// ------------------------------------------------------------------------------------------------
// fully connected: a workgroup = FC_OPB output features x 32 sample rows; each row's dot products are
// split over 8 lanes (contiguous K slices, float4 loads issued before the FMAs) and closed by
// three xor-shuffles.  Latency-bound sizes (32 x 512 x 512) -> 256 workgroups, one load round trip.
// ------------------------------------------------------------------------------------------------
constexpr int FC_OPB = 2;

__device__ __forceinline__ void fc_body(const float* __restrict__ x, int64_t ldx, const float* __restrict__ w,
                                        const float* __restrict__ b, float* __restrict__ y, int n, int in_f, int out_f,
                                        float w_gain, float b_gain, int act, float alpha, float act_gain, int vec) {
  const int t = threadIdx.x;
  const int r = t >> 3, sl = t & 7;
  const int nn = blockIdx.y * 32 + r;
  const int o0 = blockIdx.x * FC_OPB;
  const int len = (in_f + 7) >> 3;
  const int i0 = sl * len, i1 = min(in_f, i0 + len);
  const float* xr = x + (int64_t)(nn < n ? nn : 0) * ldx;
  const float* wr[FC_OPB];
#pragma unroll
  for (int o = 0; o < FC_OPB; ++o) wr[o] = w + (int64_t)min(o0 + o, out_f - 1) * in_f;
  float acc[FC_OPB];
#pragma unroll
  for (int o = 0; o < FC_OPB; ++o) acc[o] = 0.f;
  if (vec) {  // in_f % 32 == 0 and ldx % 4 == 0: every slice is whole float4s
#pragma unroll 8
    for (int i = i0; i < i1; i += 4) {
      const float4 xv = *reinterpret_cast<const float4*>(xr + i);
#pragma unroll
      for (int o = 0; o < FC_OPB; ++o) {
        const float4 wv = *reinterpret_cast<const float4*>(wr[o] + i);
        acc[o] += xv.x * wv.x + xv.y * wv.y + xv.z * wv.z + xv.w * wv.w;
      }
    }
  } else {
#pragma unroll 4
    for (int i = i0; i < i1; ++i) {
      const float xv = xr[i];
#pragma unroll
      for (int o = 0; o < FC_OPB; ++o) acc[o] += xv * wr[o][i];
    }
  }
#pragma unroll
  for (int o = 0; o < FC_OPB; ++o) {
    float v = acc[o];
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    v += __shfl_xor(v, 4, 64);
    acc[o] = v;
  }
  if (sl == 0 && nn < n) {
#pragma unroll
    for (int o = 0; o < FC_OPB; ++o) {
      if (o0 + o >= out_f) break;
      float v = acc[o] * w_gain + (b ? b[o0 + o] * b_gain : 0.f);
      if (act == IC2_ACT_LRELU) v = (v < 0.f ? v * alpha : v) * act_gain;
      y[(int64_t)nn * out_f + o0 + o] = v;
    }
  }
}

__global__ void __launch_bounds__(256) fc_kernel(const float* __restrict__ x, int64_t ldx, const float* __restrict__ w,
                                                 const float* __restrict__ b, float* __restrict__ y, int n, int in_f,
                                                 int out_f, float w_gain, float b_gain, int act, float alpha,
                                                 float act_gain, int vec) {
  fc_body(x, ldx, w, b, y, n, in_f, out_f, w_gain, b_gain, act, alpha, act_gain, vec);
}

// ------------------------------------------------------------------------------------------------
// weight packing [cout][cin][kh][kw] f32 -> [cout_p][kh][kw][cin_p] (dtype); optional pre-normalisation
// ------------------------------------------------------------------------------------------------
template <typename T, bool X3 = false, bool H2 = false>
__global__ void __launch_bounds__(256) pack_weight_kernel(const float* __restrict__ w, int cout, int cin, int kh,
                                                          int kw, int cout_p, int cin_p, int prenorm, float gscale,
                                                          T* __restrict__ out, float* __restrict__ wsq) {
  const int o = blockIdx.x;
  const int kk = kh * kw;
  const int per = cin * kk;
  __shared__ float red[256];
  float scale = 1.f;
  if (o < cout && prenorm) {
    float s = 0.f;
    for (int i = threadIdx.x; i < per; i += 256) {
      const float v = w[(int64_t)o * per + i];
      s += v * v;
    }
    red[threadIdx.x] = s;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
      if (threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
      __syncthreads();
    }
    scale = rsqrtf(red[0] / (float)per);
  }
  const int total = kk * cin_p;
  for (int e = threadIdx.x; e < total; e += 256) {
    const int i = e % cin_p;
    const int k = e / cin_p;
    float v = 0.f;
    if (o < cout && i < cin) v = w[((int64_t)o * cin + i) * kk + k] * scale * gscale;
    if constexpr (H2) {
      // split-weight f16: [hi | lo] along the doubled channel axis of tap k (ic2ops.h IC2_F16X2)
      _Float16* row = reinterpret_cast<_Float16*>(out) + ((int64_t)o * kk + k) * 2 * cin_p + i;
      const _Float16 hi = (_Float16)v;
      row[0] = hi;
      row[cin_p] = (_Float16)(v - (float)hi);
    } else if constexpr (X3) {
      // split bf16: [hi | lo | hi] along the tripled channel axis of tap k (ic2ops.h IC2_BF16X3)
      bf16_t* row = reinterpret_cast<bf16_t*>(out) + ((int64_t)o * kk + k) * 3 * cin_p + i;
      const bf16_t hi = f2bf(v);
      const bf16_t lo = f2bf(v - bf2f(hi));
      row[0] = hi;
      row[cin_p] = lo;
      row[2 * cin_p] = hi;
    } else {
      st(out + (int64_t)o * total + e, v);
    }
  }
  if (wsq && o < cout) {
    for (int i = threadIdx.x; i < cin; i += 256) {
      float s = 0.f;
      for (int k = 0; k < kk; ++k) {
        const float v = w[((int64_t)o * cin + i) * kk + k] * scale;
        s += v * v;
      }
      wsq[(int64_t)o * cin + i] = s;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// modulation / demodulation coefficients
// ------------------------------------------------------------------------------------------------
// xscale = s * g with g = rsqrt(mean(s^2)) over the whole batch (demod) or style_gain: one workgroup,
// f64 sum of squares (fixed order: per-thread strided sums, wave xor-tree, then 16 wave totals in order)
__device__ __forceinline__ void style_xscale_body(const float* __restrict__ s, int n, int cin, int cin_p, int demod,
                                                  float style_gain, float* __restrict__ xs) {
  __shared__ double red[16];
  __shared__ float gsh;
  const int64_t total = (int64_t)n * cin;
  float g = style_gain;
  if (demod) {
    double acc = 0.0;
    for (int64_t i = threadIdx.x; i < total; i += 1024) acc += (double)s[i] * (double)s[i];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
      double t = 0.0;
      for (int k = 0; k < 16; ++k) t += red[k];
      gsh = rsqrtf((float)(t / (double)total));
    }
    __syncthreads();
    g = gsh;
  }
  const int64_t tot_p = (int64_t)n * cin_p;
  for (int64_t e = threadIdx.x; e < tot_p; e += 1024) {
    const int i = (int)(e % cin_p);
    const int64_t nn = e / cin_p;
    xs[e] = i < cin ? s[nn * cin + i] * g : 0.f;
  }
}

__global__ void __launch_bounds__(1024) style_xscale_kernel(const float* __restrict__ s, int n, int cin, int cin_p,
                                                            int demod, float style_gain, float* __restrict__ xs) {
  style_xscale_body(s, n, cin, cin_p, demod, style_gain, xs);
}

// one wave per (n, o): lanes over cin
__device__ __forceinline__ void oscale_body(const float* __restrict__ xs, const float* __restrict__ wsq, int n, int cin,
                                            int cin_p, int cout, int cout_p, int demod, float input_gain,
                                            float* __restrict__ os) {
  const int lane = threadIdx.x & 63;
  const int64_t item = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (item >= (int64_t)n * cout_p) return;
  const int o = (int)(item % cout_p);
  const int64_t nn = item / cout_p;
  if (o >= cout) {
    if (lane == 0) os[item] = 0.f;
    return;
  }
  if (!demod) {
    if (lane == 0) os[item] = input_gain;
    return;
  }
  float acc = 0.f;
  for (int i = lane; i < cin; i += 64) {
    const float v = xs[nn * cin_p + i];
    acc += v * v * wsq[(int64_t)o * cin + i];
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  if (lane == 0) os[item] = input_gain * rsqrtf(acc + 1e-8f);
}

__global__ void __launch_bounds__(256) oscale_kernel(const float* __restrict__ xs, const float* __restrict__ wsq,
                                                     int n, int cin, int cin_p, int cout, int cout_p, int demod,
                                                     float input_gain, float* __restrict__ os) {
  oscale_body(xs, wsq, n, cin, cin_p, cout, cout_p, demod, input_gain, os);
}

// ------------------------------------------------------------------------------------------------
// All synthesis layers' modulation coefficients in three launches (the per-layer form above costs three
// small launches per layer, ~0.5 ms per C2 step for 15 layers): blockIdx.z / blockIdx.x = layer, each
// layer's arithmetic exactly the per-layer kernels' (same bodies), so the results are bit-identical.
// ------------------------------------------------------------------------------------------------
constexpr int kModMaxLayers = 20;
struct ModLayer {
  const float* aw;   // affine weight [cin][w_dim]
  const float* ab;   // affine bias [cin]
  const float* wsq;  // [cout][cin] (demodulated layers)
  float* styles;     // [n][cin] scratch
  float* xs;         // [n][cin_p]
  float* os;         // [n][cout_p]
  int64_t ws_off;    // element offset of this layer's w row in ws
  int cin, cin_p, cout, cout_p, demod, vec;
  float w_gain, b_gain, style_gain, input_gain;
};
struct ModBatch {
  int nl, n, w_dim;
  int64_t ldx;
  const float* ws;
  ModLayer L[kModMaxLayers];
};

// Both per-layer products of the modulation are small GEMMs over <= 512-long rows:
//   styles[n][o] = (sum_i ws[n][off + i] * aw[o][i]) * w_gain + ab[o] * b_gain      (affine FC)
//   oscale[n][o] = input_gain * rsqrt(sum_i xs[n][i]^2 * wsq[o][i] + 1e-8)           (demodulation)
// A workgroup owns 16 output features of one layer: their weight rows are staged in LDS once (row pitch K+1:
// the 16 rows land in distinct banks), then 16-sample chunks of the left operand; thread (o = t & 15,
// n = t >> 4) sums its dot product sequentially over i (fixed order, deterministic).  Replaces one wave per
// (n, o) reading the [cout][cin] weight again for every sample (86 us per C2 step for 15 layers).
constexpr int kSmK = 512;  // longest row (w_dim, cin)
template <bool OSCALE>
__device__ __forceinline__ void small_mm_body(const float* __restrict__ a, int64_t lda, const float* __restrict__ w,
                                              int n, int K, int nout, int out_p, float* __restrict__ out,
                                              const ModLayer& L) {
  // rows zero-padded to K4 (a multiple of 4) at a pitch of kSmK + 4 floats: 16-B aligned ds_read_b128 of 16
  // different rows land in 16 distinct 16-B bank slots (pitch = 16 mod 256 B)
  constexpr int P = kSmK + 4;
  __shared__ __attribute__((aligned(16))) float wl[16][P];
  __shared__ __attribute__((aligned(16))) float al[16][P];
  const int t = threadIdx.x;
  const int o0 = blockIdx.x * 16;
  const int K4 = (K + 3) & ~3;
  for (int e = t; e < 16 * K4; e += 256) {
    const int r = e / K4, i = e - (e / K4) * K4;
    wl[r][i] = o0 + r < nout && i < K ? w[(int64_t)(o0 + r) * K + i] : 0.f;
  }
  const int ol = t & 15, nl = t >> 4;
  const int o = o0 + ol;
  for (int n0 = 0; n0 < n; n0 += 16) {
    __syncthreads();  // weights staged / previous chunk consumed
    for (int e = t; e < 16 * K4; e += 256) {
      const int r = e / K4, i = e - (e / K4) * K4;
      float v = n0 + r < n && i < K ? a[(int64_t)(n0 + r) * lda + i] : 0.f;
      if (OSCALE) v = v * v;
      al[r][i] = v;
    }
    __syncthreads();
    float acc = 0.f;  // sequential over i (fixed order)
    for (int i = 0; i < K4; i += 4) {
      const float4 av = *reinterpret_cast<const float4*>(&al[nl][i]);
      const float4 wv = *reinterpret_cast<const float4*>(&wl[ol][i]);
      acc = fmaf(av.x, wv.x, acc);
      acc = fmaf(av.y, wv.y, acc);
      acc = fmaf(av.z, wv.z, acc);
      acc = fmaf(av.w, wv.w, acc);
    }
    const int nn = n0 + nl;
    if (nn < n && o < out_p) {
      float v;
      if (OSCALE) v = o < nout ? (L.demod ? L.input_gain * rsqrtf(acc + 1e-8f) : L.input_gain) : 0.f;
      else v = acc * L.w_gain + (L.ab ? L.ab[o] * L.b_gain : 0.f);
      if (OSCALE || o < nout) out[(int64_t)nn * out_p + o] = v;
    }
  }
}

__global__ void __launch_bounds__(256) fc_multi_kernel(ModBatch mb) {
  const ModLayer& L = mb.L[blockIdx.y];
  if ((int)blockIdx.x * 16 >= L.cin) return;
  small_mm_body<false>(mb.ws + L.ws_off, mb.ldx, L.aw, mb.n, mb.w_dim, L.cin, L.cin, L.styles, L);
}
__global__ void __launch_bounds__(1024) style_xscale_multi_kernel(ModBatch mb) {
  const ModLayer& L = mb.L[blockIdx.x];
  style_xscale_body(L.styles, mb.n, L.cin, L.cin_p, L.demod, L.style_gain, L.xs);
}
__global__ void __launch_bounds__(256) oscale_multi_kernel(ModBatch mb) {
  const ModLayer& L = mb.L[blockIdx.y];
  if ((int)blockIdx.x * 16 >= L.cout_p) return;
  if (!L.demod) {  // oscale = input_gain on the valid channels
    const int o0 = blockIdx.x * 16;
    for (int e = threadIdx.x; e < mb.n * 16; e += 256) {
      const int nn = e >> 4, o = o0 + (e & 15);
      if (o < L.cout_p) L.os[(int64_t)nn * L.cout_p + o] = o < L.cout ? L.input_gain : 0.f;
    }
    return;
  }
  small_mm_body<true>(L.xs, L.cin_p, L.wsq, mb.n, L.cin, L.cout, L.cout_p, L.os, L);
}

// ------------------------------------------------------------------------------------------------
// SynthesisInput Fourier features (NHWC)
// ------------------------------------------------------------------------------------------------
// one workgroup per (sample, row): each thread owns channels tid, tid + 256, ... and derives their rotated
// frequency, phase and amplitude once, then walks the row (stores coalesced along channels)
template <typename T>
__global__ void __launch_bounds__(256) synth_input_kernel(const float* __restrict__ t, const float* __restrict__ freqs,
                                                          const float* __restrict__ phases,
                                                          const float* __restrict__ tr, int n, int c, int c_p,
                                                          int size, float sr, float bw, T* __restrict__ out) {
  const int nn = blockIdx.x / size, yy = blockIdx.x - (blockIdx.x / size) * size;
  const float theta = 0.5f * (float)size / sr;
  const float two_pi = 6.283185307179586f;
  // t' = t / |t[:2]|
  const float* tn = t + nn * 4;
  const float nrm = sqrtf(tn[0] * tn[0] + tn[1] * tn[1]);
  const float rc = tn[0] / nrm, rs = tn[1] / nrm, tx = tn[2] / nrm, ty = tn[3] / nrm;
  // m_r @ m_t, then @ user transform tr (3x3)
  const float A[3][3] = {{rc, -rs, -rc * tx + rs * ty}, {rs, rc, -rs * tx - rc * ty}, {0.f, 0.f, 1.f}};
  float M[3][3];
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int q = 0; q < 3; ++q) M[r][q] = A[r][0] * tr[0 * 3 + q] + A[r][1] * tr[1 * 3 + q] + A[r][2] * tr[2 * 3 + q];
  // affine_grid(align_corners=False): base coordinate (2j+1)/size - 1, scaled by theta
  const float gy = ((2.f * yy + 1.f) / (float)size - 1.f) * theta;
  T* orow = out + ((int64_t)nn * size + yy) * size * c_p;
  for (int ch = threadIdx.x; ch < c_p; ch += 256) {
    if (ch >= c) {
      for (int xx = 0; xx < size; ++xx) st(orow + (int64_t)xx * c_p + ch, 0.f);
      continue;
    }
    const float f0 = freqs[ch * 2 + 0], f1 = freqs[ch * 2 + 1];
    const float ph = phases[ch] + (f0 * M[0][2] + f1 * M[1][2]);
    const float g0 = f0 * M[0][0] + f1 * M[1][0];
    const float g1 = f0 * M[0][1] + f1 * M[1][1];
    const float amp = fminf(fmaxf(1.f - (sqrtf(g0 * g0 + g1 * g1) - bw) / (sr * 0.5f - bw), 0.f), 1.f);
    const float rowc = gy * g1;
    for (int xx = 0; xx < size; ++xx) {
      const float gx = ((2.f * xx + 1.f) / (float)size - 1.f) * theta;
      const float arg = (gx * g0 + rowc) + ph;
      st(orow + (int64_t)xx * c_p + ch, sinf(arg * two_pi) * amp);
    }
  }
}

static int grid_1d(int64_t total) {
  int64_t g = ceil_div(total, 256);
  if (g < 1) g = 1;
  if (g > 4096) g = 4096;
  return (int)g;
}

}  // namespace ic2

using namespace ic2;

extern "C" int ic2_bias_act(const void* x, const float* b, void* y, int dtype, int64_t outer, int64_t c, int64_t inner,
                            int act, float alpha, float gain, float clamp, void* stream) {
  IC2_CHECK_ARG(x && y && outer >= 0 && c >= 1 && inner >= 1, "bias_act: bad arguments");
  IC2_CHECK_ARG(act == IC2_ACT_LINEAR || act == IC2_ACT_LRELU, "bias_act: unknown act %d", act);
  const int64_t total = outer * c * inner;
  if (total == 0) return IC2_OK;
  hipStream_t s = as_stream(stream);
  if (dtype == IC2_F32)
    hipLaunchKernelGGL(bias_act_kernel<float>, dim3(grid_1d(total)), dim3(256), 0, s, (const float*)x, b, (float*)y,
                       total, c, inner, act, alpha, gain, clamp);
  else if (dtype == IC2_BF16)
    hipLaunchKernelGGL(bias_act_kernel<bf16_t>, dim3(grid_1d(total)), dim3(256), 0, s, (const bf16_t*)x, b,
                       (bf16_t*)y, total, c, inner, act, alpha, gain, clamp);
  else
    IC2_CHECK_ARG(false, "bias_act: bad dtype %d", dtype);
  IC2_CHECK_LAUNCH("bias_act");
  return IC2_OK;
}

extern "C" int ic2_upfirdn2d(const void* x, void* y, int dtype, int64_t nc, int in_h, int in_w, int out_h, int out_w,
                             const float* f, int f_ndim, int f_h, int f_w, int up_x, int up_y, int down_x, int down_y,
                             int px0, int px1, int py0, int py1, int flip, float gain, void* stream) {
  IC2_CHECK_ARG(x && y && nc >= 0 && in_h > 0 && in_w > 0, "upfirdn2d: bad arguments");
  IC2_CHECK_ARG(up_x >= 1 && up_y >= 1 && down_x >= 1 && down_y >= 1, "upfirdn2d: bad scaling");
  if (f == nullptr) {
    f_ndim = 2;
    f_h = f_w = 1;
  }
  IC2_CHECK_ARG((f_ndim == 1 && f_w >= 1) || (f_ndim == 2 && f_h >= 1 && f_w >= 1), "upfirdn2d: bad filter shape");
  const int fh = f_ndim == 1 ? f_w : f_h;
  const int ew = (in_w * up_x + px0 + px1 - f_w + down_x) / down_x;
  const int eh = (in_h * up_y + py0 + py1 - fh + down_y) / down_y;
  IC2_CHECK_ARG(out_w == ew && out_h == eh, "upfirdn2d: output %dx%d, expected %dx%d", out_h, out_w, eh, ew);
  IC2_CHECK_ARG(out_w > 0 && out_h > 0, "upfirdn2d: empty output");
  UfdArgs a;
  a.nc = nc; a.in_h = in_h; a.in_w = in_w; a.out_h = out_h; a.out_w = out_w;
  a.f_ndim = f_ndim; a.f_h = fh; a.f_w = f_w;
  a.upx = up_x; a.upy = up_y; a.downx = down_x; a.downy = down_y; a.px0 = px0; a.py0 = py0; a.flip = flip;
  if (f_ndim == 1) {
    a.gain_x = sqrtf(gain);
    a.gain_y = sqrtf(gain);
  } else {
    a.gain_x = gain;
    a.gain_y = 1.f;
  }
  const int64_t total = nc * out_h * out_w;
  if (total == 0) return IC2_OK;
  hipStream_t s = as_stream(stream);
  if (dtype == IC2_F32)
    hipLaunchKernelGGL(upfirdn2d_kernel<float>, dim3(grid_1d(total)), dim3(256), 0, s, (const float*)x, (float*)y, f, a);
  else if (dtype == IC2_BF16)
    hipLaunchKernelGGL(upfirdn2d_kernel<bf16_t>, dim3(grid_1d(total)), dim3(256), 0, s, (const bf16_t*)x, (bf16_t*)y,
                       f, a);
  else
    IC2_CHECK_ARG(false, "upfirdn2d: bad dtype %d", dtype);
  IC2_CHECK_LAUNCH("upfirdn2d");
  return IC2_OK;
}

extern "C" int ic2_fc(const float* x, int64_t ldx, const float* w, const float* b, float* y, int n, int in_f,
                      int out_f, float w_gain, float b_gain, int act, float alpha, float act_gain, void* stream) {
  IC2_CHECK_ARG(x && w && y && n > 0 && in_f > 0 && out_f > 0 && ldx >= in_f, "fc: bad arguments");
  const int vec = in_f % 32 == 0 && ldx % 4 == 0 && ((uintptr_t)x | (uintptr_t)w) % 16 == 0;
  dim3 grid((unsigned)ceil_div(out_f, FC_OPB), (unsigned)ceil_div(n, 32));
  hipLaunchKernelGGL(fc_kernel, grid, dim3(256), 0, as_stream(stream), x, ldx, w, b, y, n, in_f, out_f, w_gain, b_gain,
                     act, alpha, act_gain, vec);
  IC2_CHECK_LAUNCH("fc");
  return IC2_OK;
}

// the adjoint (dgrad) pack of w[cout][cin][kh][kw]: out[ci][ky][kx][co] = w[co][ci][kh-1-ky][kw-1-kx], zero padded to
// [cin_p][kh][kw][cout_p] -- W flipped in space and transposed in channels, gathered straight from the parameter (the
// torch transpose / flip / contiguous it replaces cost two extra launches per conv and training step)
template <typename T>
__global__ void __launch_bounds__(256) pack_adjoint_kernel(const float* __restrict__ w, int cout, int cin, int kh,
                                                           int kw, int cin_p, int cout_p, T* __restrict__ out) {
  const int ci = blockIdx.x;  // the adjoint conv's output channel
  const int kk = kh * kw;
  const int total = kk * cout_p;
  for (int e = threadIdx.x; e < total; e += 256) {
    const int co = e % cout_p, k = e / cout_p;
    float v = 0.f;
    if (ci < cin && co < cout) v = w[((int64_t)co * cin + ci) * kk + (kk - 1 - k)];
    st(out + (int64_t)ci * total + e, v);
  }
}

extern "C" int ic2_pack_weight_adjoint(const float* w, int cout, int cin, int kh, int kw, int cin_p, int cout_p,
                                       void* w_out, int dtype, void* stream) {
  IC2_CHECK_ARG(w && w_out && cout > 0 && cin > 0 && kh > 0 && kw > 0 && cout_p >= cout && cin_p >= cin,
                "pack_weight_adjoint: bad arguments");
  hipStream_t s = as_stream(stream);
  if (dtype == IC2_F32)
    hipLaunchKernelGGL(pack_adjoint_kernel<float>, dim3(cin_p), dim3(256), 0, s, w, cout, cin, kh, kw, cin_p, cout_p,
                       (float*)w_out);
  else if (dtype == IC2_BF16)
    hipLaunchKernelGGL(pack_adjoint_kernel<bf16_t>, dim3(cin_p), dim3(256), 0, s, w, cout, cin, kh, kw, cin_p, cout_p,
                       (bf16_t*)w_out);
  else if (dtype == IC2_F16)
    hipLaunchKernelGGL(pack_adjoint_kernel<_Float16>, dim3(cin_p), dim3(256), 0, s, w, cout, cin, kh, kw, cin_p, cout_p,
                       (_Float16*)w_out);
  else
    IC2_CHECK_ARG(false, "pack_weight_adjoint: bad dtype %d", dtype);
  IC2_CHECK_LAUNCH("pack_weight_adjoint");
  return IC2_OK;
}

extern "C" int ic2_pack_weight(const float* w, int cout, int cin, int kh, int kw, int cout_p, int cin_p, int prenorm,
                               float scale, void* w_out, int dtype, float* wsq_out, void* stream) {
  IC2_CHECK_ARG(w && w_out && cout > 0 && cin > 0 && kh > 0 && kw > 0 && cout_p >= cout && cin_p >= cin,
                "pack_weight: bad arguments");
  hipStream_t s = as_stream(stream);
  if (dtype == IC2_F32)
    hipLaunchKernelGGL(pack_weight_kernel<float>, dim3(cout_p), dim3(256), 0, s, w, cout, cin, kh, kw, cout_p, cin_p,
                       prenorm, scale, (float*)w_out, wsq_out);
  else if (dtype == IC2_BF16)
    hipLaunchKernelGGL(pack_weight_kernel<bf16_t>, dim3(cout_p), dim3(256), 0, s, w, cout, cin, kh, kw, cout_p, cin_p,
                       prenorm, scale, (bf16_t*)w_out, wsq_out);
  else if (dtype == IC2_F16)
    hipLaunchKernelGGL(pack_weight_kernel<_Float16>, dim3(cout_p), dim3(256), 0, s, w, cout, cin, kh, kw, cout_p, cin_p,
                       prenorm, scale, (_Float16*)w_out, wsq_out);
  else if (dtype == IC2_BF16X3)
    hipLaunchKernelGGL((pack_weight_kernel<bf16_t, true>), dim3(cout_p), dim3(256), 0, s, w, cout, cin, kh, kw, cout_p,
                       cin_p, prenorm, scale, (bf16_t*)w_out, wsq_out);
  else if (dtype == IC2_F16X2)
    hipLaunchKernelGGL((pack_weight_kernel<_Float16, false, true>), dim3(cout_p), dim3(256), 0, s, w, cout, cin, kh, kw,
                       cout_p, cin_p, prenorm, scale, (_Float16*)w_out, wsq_out);
  else
    IC2_CHECK_ARG(false, "pack_weight: bad dtype %d", dtype);
  IC2_CHECK_LAUNCH("pack_weight");
  return IC2_OK;
}

extern "C" int ic2_modconv_prep(const float* styles, const float* wsq, int n, int cin, int cout, int cin_p, int cout_p,
                                int demod, float style_gain, float input_gain, float* xscale_out, float* oscale_out,
                                float* scratch, void* stream) {
  IC2_CHECK_ARG(styles && xscale_out && oscale_out && n > 0 && cin > 0 && cout > 0, "modconv_prep: bad arguments");
  IC2_CHECK_ARG(!demod || wsq, "modconv_prep: demodulation needs wsq");
  hipStream_t s = as_stream(stream);
  (void)scratch;
  hipLaunchKernelGGL(style_xscale_kernel, dim3(1), dim3(1024), 0, s, styles, n, cin, cin_p, demod, style_gain,
                     xscale_out);
  hipLaunchKernelGGL(oscale_kernel, dim3((unsigned)ceil_div((int64_t)n * cout_p, 4)), dim3(256), 0, s, xscale_out, wsq,
                     n, cin, cin_p, cout, cout_p, demod, input_gain, oscale_out);
  IC2_CHECK_LAUNCH("modconv_prep");
  return IC2_OK;
}

// layers: nl records of 16 int64 slots each (host array): {aw, ab, wsq, styles, xs, os, ws_off, cin, cin_p, cout,
// cout_p, demod, w_gain, b_gain, style_gain, input_gain} (pointers as integers, gains as float bit patterns in
// the low 32 bits) -- see include/ic2ops.h.
extern "C" int ic2_modconv_prep_batched(const float* ws, int64_t ldx, int n, int w_dim, int nl, const int64_t* layers,
                                        void* stream) {
  IC2_CHECK_ARG(ws && layers && n > 0 && w_dim > 0 && ldx >= w_dim && nl > 0 && nl <= kModMaxLayers,
                "modconv_prep_batched: bad arguments (nl=%d, max %d)", nl, kModMaxLayers);
  ModBatch mb;
  mb.nl = nl; mb.n = n; mb.w_dim = w_dim; mb.ldx = ldx; mb.ws = ws;
  int max_cin = 0, max_cout_p = 0;
  auto f32 = [](int64_t v) { return __builtin_bit_cast(float, (uint32_t)v); };
  for (int l = 0; l < nl; ++l) {
    const int64_t* r = layers + 16 * l;
    ModLayer& L = mb.L[l];
    L.aw = reinterpret_cast<const float*>(r[0]); L.ab = reinterpret_cast<const float*>(r[1]);
    L.wsq = reinterpret_cast<const float*>(r[2]); L.styles = reinterpret_cast<float*>(r[3]);
    L.xs = reinterpret_cast<float*>(r[4]); L.os = reinterpret_cast<float*>(r[5]);
    L.ws_off = r[6]; L.cin = (int)r[7]; L.cin_p = (int)r[8]; L.cout = (int)r[9]; L.cout_p = (int)r[10];
    L.demod = (int)r[11]; L.w_gain = f32(r[12]); L.b_gain = f32(r[13]); L.style_gain = f32(r[14]);
    L.input_gain = f32(r[15]);
    IC2_CHECK_ARG(L.aw && L.styles && L.xs && L.os && L.cin > 0 && L.cin_p >= L.cin && L.cout > 0 &&
                      L.cout_p >= L.cout && (!L.demod || L.wsq) && L.ws_off >= 0 && L.ws_off + w_dim <= ldx,
                  "modconv_prep_batched: bad layer record %d", l);
    L.vec = w_dim % 32 == 0 && ldx % 4 == 0 && L.ws_off % 4 == 0 && ((uintptr_t)ws | (uintptr_t)L.aw) % 16 == 0;
    IC2_CHECK_ARG(L.cin <= kSmK && w_dim <= kSmK, "modconv_prep_batched: rows longer than %d (layer %d)", kSmK, l);
    max_cin = max_cin > L.cin ? max_cin : L.cin;
    max_cout_p = max_cout_p > L.cout_p ? max_cout_p : L.cout_p;
  }
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(fc_multi_kernel, dim3((unsigned)ceil_div(max_cin, 16), nl), dim3(256), 0, s, mb);
  hipLaunchKernelGGL(style_xscale_multi_kernel, dim3(nl), dim3(1024), 0, s, mb);
  hipLaunchKernelGGL(oscale_multi_kernel, dim3((unsigned)ceil_div(max_cout_p, 16), nl), dim3(256), 0, s, mb);
  IC2_CHECK_LAUNCH("modconv_prep_batched");
  return IC2_OK;
}

extern "C" int ic2_synth_input_features(const float* t, const float* freqs, const float* phases, const float* transform,
                                        int n, int c, int c_p, int size, float sampling_rate, float bandwidth,
                                        void* x_out, int dtype, void* stream) {
  IC2_CHECK_ARG(t && freqs && phases && transform && x_out && n > 0 && c > 0 && c_p >= c && size > 0,
                "synth_input_features: bad arguments");
  hipStream_t s = as_stream(stream);
  if (dtype == IC2_F32)
    hipLaunchKernelGGL(synth_input_kernel<float>, dim3((unsigned)(n * size)), dim3(256), 0, s, t, freqs, phases, transform,
                       n, c, c_p, size, sampling_rate, bandwidth, (float*)x_out);
  else if (dtype == IC2_BF16)
    hipLaunchKernelGGL(synth_input_kernel<bf16_t>, dim3((unsigned)(n * size)), dim3(256), 0, s, t, freqs, phases, transform,
                       n, c, c_p, size, sampling_rate, bandwidth, (bf16_t*)x_out);
  else if (dtype == IC2_F16)
    hipLaunchKernelGGL(synth_input_kernel<_Float16>, dim3((unsigned)(n * size)), dim3(256), 0, s, t, freqs, phases,
                       transform, n, c, c_p, size, sampling_rate, bandwidth, (_Float16*)x_out);
  else
    IC2_CHECK_ARG(false, "synth_input_features: bad dtype %d", dtype);
  IC2_CHECK_LAUNCH("synth_input_features");
  return IC2_OK;
}
