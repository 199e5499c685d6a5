// Probe (diagnostic, not product): 16x16x16 vs 16x16x32 bf16 MFMA issue rate, the 16x16x16 operand
// maps and the ds_read_b64_tr_b16 lane mapping, checked with exact small-integer data.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef short s4 __attribute__((ext_vector_type(4)));
typedef __bf16 b4 __attribute__((ext_vector_type(4)));
typedef __bf16 b8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void rate16(float* out, int iters, long long* cyc) {
  b4 a, b;
  for (int j = 0; j < 4; ++j) { a[j] = (__bf16)(float)(threadIdx.x + j); b[j] = (__bf16)(float)(j + 1); }
  f4 c[4] = {};
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 4; ++u) c[u] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c[u], 0, 0, 0);
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
  out[blockIdx.x * 64 + threadIdx.x] = c[0][0] + c[1][1] + c[2][2] + c[3][3];
}
__global__ void rate32(float* out, int iters, long long* cyc) {
  b8 a, b;
  for (int j = 0; j < 8; ++j) { a[j] = (__bf16)(float)(threadIdx.x + j); b[j] = (__bf16)(float)(j + 1); }
  f4 c[4] = {};
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 4; ++u) c[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c[u], 0, 0, 0);
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
  out[blockIdx.x * 64 + threadIdx.x] = c[0][0] + c[1][1] + c[2][2] + c[3][3];
}
// C = A*B with A[m][k] = m + 16k (exact in bf16 for small ints? m+16k <= 255: exact), B[k][n] = (k == n) + k
__global__ void layout16(float* out) {
  const int l = threadIdx.x, g = l >> 4, r = l & 15;
  b4 a, b;
  for (int j = 0; j < 4; ++j) {
    const int k = 4 * g + j;
    a[j] = (__bf16)(float)(r + 16 * k);         // A[row r][k]
    b[j] = (__bf16)(float)((k == r ? 1 : 0) + 2 * k);  // B[k][col r]
  }
  f4 c = {};
  c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
  for (int q = 0; q < 4; ++q) out[l * 4 + q] = c[q];
}
// tr_b16: LDS holds v[row][col] = row*16 + col (16-bit), 16 rows x 16 cols; group g reads rows 4g..4g+3
__global__ void trread(float* out) {
  __shared__ __attribute__((aligned(16))) short lds[256];
  for (int i = threadIdx.x; i < 256; i += 64) lds[i] = (short)i;
  __syncthreads();
  const int l = threadIdx.x, g = l >> 4, i = l & 15, q = i >> 2, p = i & 3;
  const short* src = lds + (4 * g + q) * 16 + 4 * p;
  s4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)src);
  for (int e = 0; e < 4; ++e) out[l * 4 + e] = (float)v[e];
}
int main() {
  float* d; long long* cy;
  hipMalloc(&d, 1 << 22); hipMalloc(&cy, 8192 * 8);
  std::vector<float> h(1 << 20); std::vector<long long> hc(1024);
  // layout check
  hipLaunchKernelGGL(layout16, 1, 64, 0, 0, d); hipMemcpy(h.data(), d, 64 * 4 * 4, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int l = 0; l < 64; ++l) for (int q = 0; q < 4; ++q) {
    const int row = 4 * (l >> 4) + q, col = l & 15;
    double ref = 0; for (int k = 0; k < 16; ++k) ref += (double)(row + 16 * k) * ((k == col ? 1 : 0) + 2 * k);
    if (h[l * 4 + q] != (float)ref) ++bad;
  }
  printf("layout16 C[row=4(l>>4)+q][col=l&15] mismatches: %d\n", bad);
  hipLaunchKernelGGL(trread, 1, 64, 0, 0, d); hipMemcpy(h.data(), d, 64 * 4 * 4, hipMemcpyDeviceToHost);
  bad = 0;
  for (int l = 0; l < 64; ++l) for (int e = 0; e < 4; ++e) {
    const int g = l >> 4, i = l & 15;
    if (h[l * 4 + e] != (float)((4 * g + e) * 16 + i)) ++bad;  // lane i gets column i of rows 4g+e
  }
  printf("tr_b16 lane i <- column i, element e <- row 4g+e mismatches: %d\n", bad);
  for (int w = 0; w < 2; ++w) {
    const int blocks = 1024, it = 4096;
    for (int rep = 0; rep < 2; ++rep) {
      if (w == 0) hipLaunchKernelGGL(rate16, blocks, 256, 0, 0, d, it, cy);
      else hipLaunchKernelGGL(rate32, blocks, 256, 0, 0, d, it, cy);
      hipDeviceSynchronize();
    }
    hipMemcpy(hc.data(), cy, blocks * 8, hipMemcpyDeviceToHost);
    double s = 0; for (int b = 0; b < blocks; ++b) s += hc[b];
    // s_memtime ticks per MFMA per wave (4 waves/block share 4 SIMDs)
    printf("%s: %.2f ticks per MFMA (per wave, 4 independent accumulators)\n", w ? "16x16x32" : "16x16x16",
           s / blocks / (it * 4.0));
  }
  return 0;
}
