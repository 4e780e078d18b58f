// gemm.hip -- skinny weight-streaming GEMM on MFMA for decode/verify shapes.
//
// Replaces the cublasGemmEx dense layer (linear_kernels.cu:450-582):
//   Y[T][N] = X[T][K] . W[N][K]^T, fp16 in/out, fp32 accumulate.
// (The reference runs cuBLAS with compute_type = fp16, linear_kernels.cu:509;
// accumulating in fp32 is a deliberate, documented precision upgrade.)
//
// Design (MI355X): at T <= ~200 the layer is HBM-bound on the weight stream
// (arithmetic intensity ~T flop/byte < the ~312 flop/byte ridge), so every
// weight byte must be read exactly once per step and at full bandwidth:
//  * weights are pre-packed in MFMA B-fragment order (weights.hip): a wave
//    streams contiguous 1 KiB per k-step, 16 B per lane, no LDS round trip
//    (guide: "GEMV / M <= 16: load straight to VGPRs, deep unroll");
//  * one workgroup owns NT 16-column tiles and splits K over its KW waves,
//    so small-N layers (o_proj, down_proj: 256 tiles) still put 8 waves on
//    every CU; U k-steps of loads are issued before their MFMAs;
//  * all M-tiles (<= MT*16 rows) of X share each weight fragment: weights
//    are read once regardless of T (X comes from L2);
//  * the per-element reduction order is fixed by (N-tile, K) only, so a
//    row's result does not depend on T or on which other rows are batched.
// Epilogue FFMI_EPI_SILU_MUL fuses SigmoidSiluMulti (sigmoid_silu_multi.cu:
// 37-47) on interleaved [gate|up] tiles.
#include "../ffmi_internal.h"

namespace ffmi {

// MULTI = 1 marks the multi-pass (T > 192, prefill) instantiation so that
// profiles separate it from the single-pass decode/verify launches.
template <int MT, int NT, int KW, int U, int EPI, int MULTI>
__global__ __launch_bounds__(KW * 64) void gemm_skinny_kernel(
    const uint16_t *__restrict__ X, const uint16_t *__restrict__ Wp,
    uint16_t *__restrict__ Y, int T, int N, int K, int KT, int NTILES) {
  extern __shared__ __attribute__((aligned(16))) float red[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int tile0 = blockIdx.x * NT;
  const int m0 = blockIdx.y * (MT * 16);
  const int per = (KT + KW - 1) / KW;
  const int kb = min(KT, wave * per);
  const int ke = min(KT, kb + per);

  f4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  const uint16_t *xrow[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    int r = min(m0 + i * 16 + (lane & 15), T - 1);
    xrow[i] = X + (size_t)r * K + 8 * (lane >> 4);
  }
  const uint16_t *wrow[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    int t = min(tile0 + j, NTILES - 1);
    wrow[j] = Wp + (size_t)t * KT * 512 + lane * 8;
  }

  int kt = kb;
  for (; kt + U <= ke; kt += U) {
    h8 b[U][NT];
    h8 a[U][MT];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < NT; ++j)
        b[u][j] = *reinterpret_cast<const h8 *>(wrow[j] + (size_t)(kt + u) * 512);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int i = 0; i < MT; ++i)
        a[u][i] = *reinterpret_cast<const h8 *>(xrow[i] + (kt + u) * 32);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[u][i], b[u][j], acc[i][j],
                                                            0, 0, 0);
  }
  for (; kt < ke; ++kt) {
    h8 b[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j)
      b[j] = *reinterpret_cast<const h8 *>(wrow[j] + (size_t)kt * 512);
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      h8 a = *reinterpret_cast<const h8 *>(xrow[i] + kt * 32);
#pragma unroll
      for (int j = 0; j < NT; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b[j], acc[i][j], 0, 0, 0);
    }
  }

  // Cross-wave K reduction in a fixed order (wave 0 + 1 + ... + KW-1).
  if (KW > 1) {
    constexpr int REGS = MT * NT * 4;
    if (wave > 0) {
      float *dst = red + (size_t)(wave - 1) * REGS * 64;
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) dst[((i * NT + j) * 4 + r) * 64 + lane] = acc[i][j][r];
    }
    __syncthreads();
    if (wave != 0) return;
    for (int w = 1; w < KW; ++w) {
      const float *src = red + (size_t)(w - 1) * REGS * 64;
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[i][j][r] += src[((i * NT + j) * 4 + r) * 64 + lane];
    }
  }

  // Epilogue: C/D layout col = lane&15, row = (lane>>4)*4 + r.
  if (EPI == 0) {
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      int n = (tile0 + j) * 16 + (lane & 15);
      if (tile0 + j >= NTILES || n >= N) continue;
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          int m = m0 + i * 16 + (lane >> 4) * 4 + r;
          if (m < T) Y[(size_t)m * N + n] = __half_as_ushort(__float2half_rn(acc[i][j][r]));
        }
    }
  } else {
    // tiles (2p, 2p+1) = (gate, up) of output columns [16p, 16p+16)
    int n = blockIdx.x * 16 + (lane & 15);
    if (n < N) {
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          int m = m0 + i * 16 + (lane >> 4) * 4 + r;
          if (m >= T) continue;
          float g = __half2float(__float2half_rn(acc[i][0][r]));
          float u = __half2float(__float2half_rn(acc[i][1][r]));
          float sg = __fdiv_rn(1.0f, __fadd_rn(1.0f, expf(-g)));
          float sh = __half2float(__float2half_rn(sg));
          float t = __half2float(__float2half_rn(__fmul_rn(g, sh)));
          Y[(size_t)m * N + n] = __half_as_ushort(__float2half_rn(__fmul_rn(t, u)));
        }
    }
  }
}

template <int MT, int NT, int KW, int U, int EPI, int MULTI>
static hipError_t run(const uint16_t *X, const uint16_t *Wp, uint16_t *Y, int T, int N,
                      int K, int KT, int NTILES, int mpasses, hipStream_t s) {
  dim3 grid((NTILES + NT - 1) / NT, mpasses);
  size_t lds = KW > 1 ? (size_t)(KW - 1) * MT * NT * 4 * 64 * sizeof(float) : 0;
  hipLaunchKernelGGL((gemm_skinny_kernel<MT, NT, KW, U, EPI, MULTI>), grid, dim3(KW * 64), lds,
                     s, X, Wp, Y, T, N, K, KT, NTILES);
  return hipGetLastError();
}

template <int MT, int U, int MULTI>
static hipError_t dispatch_nt(const uint16_t *X, const uint16_t *Wp, uint16_t *Y, int T,
                              int N, int K, int KT, int epi, int mpasses, hipStream_t s) {
  int ntiles = (N + 15) / 16;
  if (epi == FFMI_EPI_SILU_MUL)
    return run<MT, 2, 4, U, 1, MULTI>(X, Wp, Y, T, N, K, KT, 2 * ntiles, mpasses, s);
  if (MT >= 4 && ntiles >= 512)
    return run<MT, 2, 4, U, 0, MULTI>(X, Wp, Y, T, N, K, KT, ntiles, mpasses, s);
  // 8-wave groups only where the accumulators fit 2 waves/SIMD (no spills)
  if (ntiles >= 512 || MT >= 8)
    return run<MT, 1, 4, U, 0, MULTI>(X, Wp, Y, T, N, K, KT, ntiles, mpasses, s);
  return run<MT, 1, (MT >= 8 ? 4 : 8), U, 0, MULTI>(X, Wp, Y, T, N, K, KT, ntiles, mpasses, s);
}

hipError_t launch_gemm(const uint16_t *X, const uint16_t *Wp, uint16_t *Y, int T, int N,
                       int K, int epilogue, hipStream_t s) {
  if (T <= 0) return hipSuccess;
  const int KT = K / 32;
  const int mtiles = (T + 15) / 16;
  if (mtiles <= 1) return dispatch_nt<1, 8, 0>(X, Wp, Y, T, N, K, KT, epilogue, 1, s);
  if (mtiles <= 2) return dispatch_nt<2, 8, 0>(X, Wp, Y, T, N, K, KT, epilogue, 1, s);
  if (mtiles <= 4) return dispatch_nt<4, 4, 0>(X, Wp, Y, T, N, K, KT, epilogue, 1, s);
  if (mtiles <= 8) return dispatch_nt<8, 2, 0>(X, Wp, Y, T, N, K, KT, epilogue, 1, s);
  if (mtiles <= 12) return dispatch_nt<12, 2, 0>(X, Wp, Y, T, N, K, KT, epilogue, 1, s);
  return dispatch_nt<12, 2, 1>(X, Wp, Y, T, N, K, KT, epilogue, (mtiles + 11) / 12, s);
}

}  // namespace ffmi
