// Library reference point for the verify-step GEMMs (measurement only, never
// linked into libffmi.so): rocBLAS fp16 GEMM with fp32 accumulation, Y[T][N]
// = X[T][K] . W[N][K]^T, the LLaMA-7B verify / width-4 / prefill shapes, cold
// weights (rotating copies over > 256 MB).  Prints one JSON line per shape.
//   hipcc --offload-arch=gfx950 -O3 -o blas_ref blas_ref.hip -lrocblas
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#define CK(x)                                                          \
  do {                                                                 \
    auto e_ = (x);                                                     \
    if ((int)e_ != 0) {                                                \
      fprintf(stderr, "%s:%d error %d\n", __FILE__, __LINE__, (int)e_); \
      exit(1);                                                         \
    }                                                                  \
  } while (0)

__global__ void fill(uint16_t *p, size_t n, uint32_t seed) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15;
    h *= 2246822519u;
    h ^= h >> 13;
    _Float16 v = (_Float16)(((float)(h & 0xffff) / 65536.0f - 0.5f) * 0.1f);
    p[i] = *reinterpret_cast<uint16_t *>(&v);
  }
}

int main() {
  struct Shape {
    const char *name;
    int N, K;
  } shapes[] = {{"qkv", 12288, 4096}, {"o", 4096, 4096}, {"gate_up", 22016, 4096},
                {"down", 4096, 11008}, {"lm_head", 32000, 4096}};
  const int Ts[] = {168, 216, 1024};
  rocblas_handle h;
  CK(rocblas_create_handle(&h));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (const Shape &s : shapes) {
    const size_t wn = (size_t)s.N * s.K;
    const int copies = (int)(768.0 * (1 << 20) / (wn * 2.0)) + 1;
    std::vector<uint16_t *> W(copies);
    for (auto &w : W) {
      CK(hipMalloc(&w, wn * 2));
      hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, w, wn, 7u);
    }
    for (int T : Ts) {
      uint16_t *X, *Y;
      CK(hipMalloc(&X, (size_t)T * s.K * 2));
      CK(hipMalloc(&Y, (size_t)T * s.N * 2));
      hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, X, (size_t)T * s.K, 11u);
      const float alpha = 1.f, beta = 0.f;
      // column-major view: Y^T[N][T] = W[N][K] (op T of the col-major K x N) . X^T[K][T]
      auto run = [&](const uint16_t *w) {
        return rocblas_gemm_ex(h, rocblas_operation_transpose, rocblas_operation_none, s.N, T, s.K,
                               &alpha, w, rocblas_datatype_f16_r, s.K, X, rocblas_datatype_f16_r,
                               s.K, &beta, Y, rocblas_datatype_f16_r, s.N, Y,
                               rocblas_datatype_f16_r, s.N, rocblas_datatype_f32_r,
                               rocblas_gemm_algo_standard, 0, 0);
      };
      for (int i = 0; i < copies; ++i) CK(run(W[i]));
      const int iters = 30;
      CK(hipEventRecord(a));
      for (int i = 0; i < iters; ++i) CK(run(W[i % copies]));
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      const double us = ms * 1e3 / iters;
      const double bytes = 2.0 * ((double)wn + (double)T * s.K + (double)T * s.N);
      printf("{\"lib\": \"rocblas_gemm_ex f16/f32acc\", \"op\": \"%s\", \"T\": %d, \"N\": %d, \"K\": %d, "
             "\"us\": %.2f, \"GBps\": %.1f, \"TFLOPs\": %.1f}\n",
             s.name, T, s.N, s.K, us, bytes / (us * 1e-6) / 1e9,
             2.0 * T * (double)s.N * s.K / (us * 1e-6) / 1e12);
      fflush(stdout);
      CK(hipFree(X));
      CK(hipFree(Y));
    }
    for (auto &w : W) CK(hipFree(w));
  }
  rocblas_destroy_handle(h);
  return 0;
}
