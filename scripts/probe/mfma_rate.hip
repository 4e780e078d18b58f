// Issue rate of independent MFMAs on one SIMD (one wave), in shader cycles.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef __bf16 b8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));
template <int KIND>
__global__ void rate(float *out, long long *cyc, int iters) {
  h8 a, b; b8 ab, bb;
  for (int j = 0; j < 8; ++j) { a[j] = (_Float16)(threadIdx.x * 0.001f + j); b[j] = (_Float16)0.5f;
                                ab[j] = (__bf16)(threadIdx.x * 0.001f + j); bb[j] = (__bf16)0.5f; }
  f4 c[8]; f16v d[4];
  for (int i = 0; i < 8; ++i) c[i] = f4{0, 0, 0, 0};
  for (int i = 0; i < 4; ++i) for (int r = 0; r < 16; ++r) d[i][r] = 0;
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (KIND == 0) c[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c[i], 0, 0, 0);
      if (KIND == 1) c[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, bb, c[i], 0, 0, 0);
      if (KIND == 2) d[i & 3] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, d[i & 3], 0, 0, 0);
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0;
  for (int i = 0; i < 8; ++i) s += c[i][0] + c[i][3];
  for (int i = 0; i < 4; ++i) s += d[i][0];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
int main() {
  float *o; long long *cy; hipMalloc(&o, 1 << 20); hipMalloc(&cy, 8192);
  const int iters = 4000;
  const char *names[3] = {"16x16x32 f16", "16x16x32 bf16", "32x32x16 f16"};
  for (int kind = 0; kind < 3; ++kind) {
    for (int wpb = 1; wpb <= 8; wpb *= 2) {   // waves per block: 1 -> 1 wave/SIMD ... 8 -> 2 waves/SIMD
      long long h[1];
      if (kind == 0) rate<0><<<1, 64 * wpb>>>(o, cy, iters);
      if (kind == 1) rate<1><<<1, 64 * wpb>>>(o, cy, iters);
      if (kind == 2) rate<2><<<1, 64 * wpb>>>(o, cy, iters);
      hipDeviceSynchronize();
      hipMemcpy(h, cy, 8, hipMemcpyDeviceToHost);
      printf("%s waves/block %d: %.1f cycles per MFMA per wave\n", names[kind], wpb,
             (double)h[0] / (iters * 8.0));
    }
  }
  return 0;
}
