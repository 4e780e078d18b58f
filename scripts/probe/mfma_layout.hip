// Probe the lane layout of v_mfma_f32_16x16x32_f16 (gfx950).
// A operand (arg0): lane l supplies 8 halves; we set them to encode (l, j).
// Experiment 1: arg0 lane l = [row-code (l&15) at k-slot j==0 of lanes 0..15 only]
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
__global__ void probe(float *out, int mode) {
  const int l = threadIdx.x;
  h8 a, b;
  for (int j = 0; j < 8; ++j) { a[j] = 0; b[j] = 0; }
  // lanes 0..15 hold k = 0..7 (for l>>4 == 0); put value at j == 0 -> k = 0
  if ((l >> 4) == 0) {
    if (mode == 0) { a[0] = (_Float16)(l + 1); b[0] = (_Float16)1; }          // arg0 = row code
    else           { a[0] = (_Float16)1;       b[0] = (_Float16)(l + 1); }    // arg1 = code
  }
  f4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) out[(mode * 64 + l) * 4 + r] = c[r];
}
int main() {
  float *d; hipMalloc(&d, 2 * 64 * 4 * sizeof(float));
  probe<<<1, 64>>>(d, 0); probe<<<1, 64>>>(d, 1);
  float h[512]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int mode = 0; mode < 2; ++mode) {
    printf("mode %d (%s carries the code): lane:reg -> value\n", mode, mode ? "arg1" : "arg0");
    for (int l = 0; l < 64; l += 5) {
      printf("  l=%2d:", l);
      for (int r = 0; r < 4; ++r) printf(" %4.0f", h[(mode * 64 + l) * 4 + r]);
      printf("\n");
    }
  }
  return 0;
}
