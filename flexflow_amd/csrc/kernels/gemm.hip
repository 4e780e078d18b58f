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
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <type_traits>

#include "../ffmi_internal.h"

namespace ffmi {

// compile-time loop: f(std::integral_constant<int, 0>) ... f(<N-1>)
template <int I, int N, class F>
__device__ __forceinline__ void static_for_impl(F &&f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for_impl<I + 1, N>(f);
  }
}
template <int N, class F>
__device__ __forceinline__ void static_for(F &&f) {
  static_for_impl<0, N>(f);
}

// SigmoidSiluMultiKernel numerics (sigmoid_silu_multi.cu:41-46): gate and up
// are fp16 values, out = half(half(g * half(sigmoid(g))) * u)
__device__ __forceinline__ uint16_t silu_mul_h(float gacc, float uacc) {
  const float g = __half2float(__float2half_rn(gacc));
  const float u = __half2float(__float2half_rn(uacc));
  const float sg = __half2float(__float2half_rn(1.0f / (1.0f + expf(-g))));
  const float t = __half2float(__float2half_rn(g * sg));
  return __half_as_ushort(__float2half_rn(t * u));
}

// Split-K over workgroups (grid.y = S > 1, small-N layers only): each
// workgroup reduces its K slice over its waves and writes an fp32 partial
// slab [S][T][NTILES*16] that the consumer combines in slice order
// (Partials, the M-split kernel's slab layout).
// v of the lane n places further up the same 16-lane DPP row (row_ror:n)
template <int NR>
__device__ __forceinline__ float row_ror_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v),
                                                               0x120 + NR, 0xf, 0xf, false));
}

// v of lane l (wave-uniform result), bit-exact
__device__ __forceinline__ float lane_f(float v, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}

// FZ (FuseArgs, ffmi_internal.h): 1 = residual-add producer epilogue (EPI 0,
// unsplit), 2 = RMSNorm consumer prologue on row-major X.  Y is restrict-
// qualified except in the producer, where it aliases fz.res_in (the residual
// is updated in place).
template <int FZ>
using SkinnyY = std::conditional_t<FZ == 1, uint16_t *, uint16_t *__restrict__>;
template <int MT, int NT, int KW, int U, int EPI, bool PIPE = false, bool NTL = false, int FZ = 0>
__global__ __launch_bounds__(KW * 64) void gemm_skinny_kernel(
    const uint16_t *__restrict__ X, const uint16_t *__restrict__ Wp,
    SkinnyY<FZ> Y, float *__restrict__ Ypart, int T, int N, int K, int KT,
    int NTILES, int xp, int yp, size_t wts, size_t wks, FuseArgs fz) {
  extern __shared__ __attribute__((aligned(16))) float red[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  // FZ == 1: the residual this wave-0 epilogue adds, loaded up front
  _Float16 rpre[FZ == 1 ? MT : 1][FZ == 1 ? NT : 1][4];
  if constexpr (FZ == 1) {
    if (wave == 0) {
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int n = min((int)(blockIdx.x * NT + j) * 16 + (lane & 15), N - 1);
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int m = min(i * 16 + (lane >> 4) * 4 + r, T - 1);
            rpre[i][j][r] = reinterpret_cast<const _Float16 *>(fz.res_in)[(size_t)m * N + n];
          }
      }
    }
  }
  // FZ == 2: rms of every row (the norm kernel's arithmetic on the
  // producer's per-tile sums of squares, summed in a fixed order), then the
  // rms of this lane's rows as an fp16 multiplier of its X fragments
  h8 rms8[FZ == 2 ? MT : 1];
  // wave w owns rows w, w + KW, ... (<= RPW of them); lane l sums partials
  // l, l + 64, ... (<= 4: nss <= 256) of each.  The loads go out first; the
  // sums, the LDS exchange and its barrier (rms_finish) run once the wave's
  // first batch of weight / X loads is in flight too (loads retire in order,
  // so waiting for these does not wait for those): the two round trips
  // overlap instead of adding up.  Every wave calls rms_finish exactly once.
  constexpr int RPW = (MT * 16 + KW - 1) / KW;
  __shared__ float sRms[FZ == 2 ? MT * 16 : 1];
  float pv[FZ == 2 ? RPW : 1][4];
  bool rdone = FZ != 2;
  if constexpr (FZ == 2) {
#pragma unroll
    for (int rr = 0; rr < RPW; ++rr) {
      const int m = min(wave + rr * KW, T - 1);
#pragma unroll
      for (int c = 0; c < 4; ++c)
        pv[rr][c] = fz.ss_in[(size_t)m * fz.nss + min(lane + 64 * c, fz.nss - 1)];
    }
  }
  // rms_finish contains the workgroup's only __syncthreads before the
  // cross-wave reduction.  It is called at several points (after the first
  // batch of loads of the pipelined loop, the batched loop or the tail, and
  // unconditionally after the k-loop) and runs once per wave (rdone): a wave
  // whose k-range is empty, or shorter than a batch, reaches it at the
  // post-loop call, so waves may arrive at s_barrier from different
  // program points.  That is well defined on CDNA (s_barrier counts waves,
  // not PCs); the builtin is convergent, so the compiler neither duplicates
  // nor moves it across the rdone branch.  Pinned by
  // test_gpu_kernels.py::test_fused_norm_consumer_empty_wave_ranges (KW 4 /
  // 8 with waves that own no k-step, T 1..32).
  auto rms_finish = [&]() {
    if constexpr (FZ == 2) {
      if (rdone) return;
      rdone = true;
#pragma unroll
      for (int rr = 0; rr < RPW; ++rr) {
        const int m = wave + rr * KW;
        float v = 0.f;
#pragma unroll
        for (int c = 0; c < 4; ++c)
          if (lane + 64 * c < fz.nss) v += pv[rr][c];
        // 16-lane DPP rows, then the four row sums in row order
        v += row_ror_f<1>(v);
        v += row_ror_f<2>(v);
        v += row_ror_f<4>(v);
        v += row_ror_f<8>(v);
        v = ((lane_f(v, 0) + lane_f(v, 16)) + lane_f(v, 32)) + lane_f(v, 48);
        if (lane == 0 && m < T) {
          const float rf = __fdiv_rn(1.0f, sqrtf(__fadd_rn(__fdiv_rn(v, (float)K), fz.eps)));
          sRms[m] = __half2float(__float2half_rn(rf));
        }
      }
      __syncthreads();
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const _Float16 r = (_Float16)sRms[min(i * 16 + (lane & 15), T - 1)];
        rms8[i] = h8{r, r, r, r, r, r, r, r};
      }
    }
  };
  // norm weight fragment of k-step k (this lane's 8 columns)
  auto ldwn = [&](int k) -> h8 {
    return *reinterpret_cast<const h8 *>(fz.wnorm + (size_t)k * 32 + 8 * (lane >> 4));
  };
  // y = half(half(x * rms) * w): two fp16 multiplies, as the norm kernel
  auto nrm = [&](h8 &a, int i, const h8 &w) {
    if constexpr (FZ == 2) a = (a * rms8[i]) * w;
  };
  const int cb = blockIdx.x, ks = blockIdx.y, S = gridDim.y;
  const int tile0 = cb * NT;
  const int m0 = 0;
  const int per_wg = (KT + S - 1) / S;
  const int kb_wg = min(KT, ks * per_wg), ke_wg = min(KT, kb_wg + per_wg);
  const int per = (ke_wg - kb_wg + KW - 1) / KW;
  const int kb = min(ke_wg, kb_wg + wave * per);
  const int ke = min(ke_wg, kb + per);

  f4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  // X row-major, or packed activation tiles (xp): 1 KiB per fragment load
  const int XS = xp ? 512 : 32;
  const uint16_t *xrow[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    if (xp) {
      const int mt = min((m0 + i * 16) >> 4, (T - 1) >> 4);
      xrow[i] = X + ((size_t)mt * KT * 64 + lane) * 8;
    } else {
      const int r = min(m0 + i * 16 + (lane & 15), T - 1);
      xrow[i] = X + (size_t)r * K + 8 * (lane >> 4);
    }
  }
  const uint16_t *wrow[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    int t = min(tile0 + j, NTILES - 1);
    wrow[j] = Wp + (size_t)t * wts + lane * 8;
  }

  int kt = kb;
  if constexpr (PIPE) {
    // software pipeline over batches of UP = U/2 k-steps, two register sets:
    // the next batch's loads are issued before this batch's MFMAs, so each
    // wave keeps UP..2*UP k-steps in flight
    constexpr int UP = U / 2;
    const int nb = (ke - kt) / UP;
    if (nb > 0) {
      h8 bA[UP][NT], aA[UP][MT], bB[UP][NT], aB[UP][MT];
      h8 wA[FZ == 2 ? UP : 1], wB[FZ == 2 ? UP : 1];
      auto ld = [&](h8(&bb)[UP][NT], h8(&aa)[UP][MT], h8(&ww)[FZ == 2 ? UP : 1], int k0) {
#pragma unroll
        for (int u = 0; u < UP; ++u)
#pragma unroll
          for (int j = 0; j < NT; ++j)
            bb[u][j] = ld_weight<NTL>(wrow[j] + (size_t)(k0 + u) * wks);
#pragma unroll
        for (int u = 0; u < UP; ++u) {
#pragma unroll
          for (int i = 0; i < MT; ++i)
            aa[u][i] = *reinterpret_cast<const h8 *>(xrow[i] + (size_t)(k0 + u) * XS);
          if constexpr (FZ == 2) ww[u] = ldwn(k0 + u);
        }
      };
      auto mm = [&](h8(&bb)[UP][NT], h8(&aa)[UP][MT], h8(&ww)[FZ == 2 ? UP : 1]) {
#pragma unroll
        for (int u = 0; u < UP; ++u)
#pragma unroll
          for (int i = 0; i < MT; ++i) nrm(aa[u][i], i, ww[FZ == 2 ? u : 0]);
#pragma unroll
        for (int u = 0; u < UP; ++u)
#pragma unroll
          for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int j = 0; j < NT; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(aa[u][i], bb[u][j], acc[i][j],
                                                                0, 0, 0);
      };
      ld(bA, aA, wA, kt);
      rms_finish();
      int q = 0;
      for (; q + 2 < nb; q += 2) {
        ld(bB, aB, wB, kt + UP);
        __builtin_amdgcn_sched_barrier(0);
        mm(bA, aA, wA);
        __builtin_amdgcn_sched_barrier(0);
        ld(bA, aA, wA, kt + 2 * UP);
        __builtin_amdgcn_sched_barrier(0);
        mm(bB, aB, wB);
        __builtin_amdgcn_sched_barrier(0);
        kt += 2 * UP;
      }
      if (q + 1 < nb) {  // two batches left
        ld(bB, aB, wB, kt + UP);
        __builtin_amdgcn_sched_barrier(0);
        mm(bA, aA, wA);
        __builtin_amdgcn_sched_barrier(0);
        mm(bB, aB, wB);
        kt += 2 * UP;
      } else {  // one batch left
        __builtin_amdgcn_sched_barrier(0);
        mm(bA, aA, wA);
        kt += UP;
      }
    }
  }
  for (; kt + U <= ke; kt += U) {
    h8 b[U][NT];
    h8 a[U][MT];
    h8 wn[FZ == 2 ? U : 1];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < NT; ++j)
        b[u][j] = ld_weight<NTL>(wrow[j] + (size_t)(kt + u) * wks);
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int i = 0; i < MT; ++i)
        a[u][i] = *reinterpret_cast<const h8 *>(xrow[i] + (size_t)(kt + u) * XS);
      if constexpr (FZ == 2) wn[u] = ldwn(kt + u);
    }
    rms_finish();
    // keep the whole batch of loads ahead of the MFMAs: left alone the
    // scheduler interleaves them and reuses registers, leaving ~7 loads in
    // flight per wave with a vmcnt wait before almost every MFMA
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int i = 0; i < MT; ++i) nrm(a[u][i], i, wn[FZ == 2 ? u : 0]);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[u][i], b[u][j], acc[i][j],
                                                            0, 0, 0);
  }
  // tail (< U k-steps; with a small K -- the SSM, K = 768 over 4-8 waves --
  // the whole loop): every load of the batch is issued before the first MFMA
  // (one memory round trip, not one per k-step).  Steps past ke re-load the
  // last step (valid addresses, no branch) and add a zero weight fragment.
  if (kt < ke) {
    const int rem = ke - kt;
    h8 b[U - 1][NT];
    h8 a[U - 1][MT];
    h8 wn[FZ == 2 ? U - 1 : 1];
#pragma unroll
    for (int u = 0; u < U - 1; ++u) {
      const int kk = min(kt + u, ke - 1);
#pragma unroll
      for (int j = 0; j < NT; ++j)
        b[u][j] = ld_weight<NTL>(wrow[j] + (size_t)kk * wks);
#pragma unroll
      for (int i = 0; i < MT; ++i)
        a[u][i] = *reinterpret_cast<const h8 *>(xrow[i] + (size_t)kk * XS);
      if constexpr (FZ == 2) wn[u] = ldwn(kk);
    }
    rms_finish();
    __builtin_amdgcn_sched_barrier(0);
    const h8 zero = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < U - 1; ++u)
#pragma unroll
      for (int i = 0; i < MT; ++i) nrm(a[u][i], i, wn[FZ == 2 ? u : 0]);
#pragma unroll
    for (int u = 0; u < U - 1; ++u) {
      if (u >= rem)
#pragma unroll
        for (int j = 0; j < NT; ++j) b[u][j] = zero;
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[u][i], b[u][j], acc[i][j], 0, 0, 0);
    }
  }

  rms_finish();  // (a wave with an empty k-range still meets the barrier)
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
  if (S > 1) {  // EPI == 0 only (host-checked)
    const int NP = NTILES * 16;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int n = (tile0 + j) * 16 + (lane & 15);
      if (tile0 + j >= NTILES) continue;
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + i * 16 + (lane >> 4) * 4 + r;
          if (m < T) Ypart[((size_t)ks * T + m) * NP + n] = acc[i][j][r];
        }
    }
    return;
  }
  if constexpr (FZ == 1) {
    // residual add (the norm kernel's correctly rounded fp16 add of the
    // rounded GEMM output), then per (row, tile) the sum of squares of the
    // 16 new values: a fixed butterfly over the 16 lanes of the row
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int n = (tile0 + j) * 16 + (lane & 15);
      const bool nok = tile0 + j < NTILES && n < N;
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + i * 16 + (lane >> 4) * 4 + r;
          const _Float16 rh = rpre[i][j][r] + (_Float16)acc[i][j][r];
          float sq = 0.f;
          if (nok && m < T) {
            reinterpret_cast<_Float16 *>(Y)[(size_t)m * N + n] = rh;
            const float f = (float)rh;
            sq = f * f;
          }
          // the 16 columns of the row are the 16 lanes of one DPP row:
          // rotate-and-add within the row (VALU, no LDS crossbar)
          sq += row_ror_f<1>(sq);
          sq += row_ror_f<2>(sq);
          sq += row_ror_f<4>(sq);
          sq += row_ror_f<8>(sq);
          if ((lane & 15) == 0 && m < T && tile0 + j < NTILES)
            fz.ss_out[(size_t)m * NTILES + tile0 + j] = sq;
        }
    }
    return;
  }
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
          if (m < T)
            Y[yp ? act_packed_off(m, n, N) : (size_t)m * N + n] =
                __half_as_ushort(__float2half_rn(acc[i][j][r]));
        }
    }
  } else {
    // tiles (2p, 2p+1) = (gate, up) of output columns [16p, 16p+16)
    int n = cb * 16 + (lane & 15);
    if (n < N) {
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          int m = m0 + i * 16 + (lane >> 4) * 4 + r;
          if (m >= T) continue;
          Y[yp ? act_packed_off(m, n, N) : (size_t)m * N + n] =
              silu_mul_h(acc[i][0][r], acc[i][1][r]);
        }
    }
  }
}

template <int MT, int NT, int KW, int U, int EPI, int FZ = 0>
static hipError_t run(const uint16_t *X, const uint16_t *Wp, uint16_t *Y, float *ws, int T,
                      int N, int K, int KT, int NTILES, int S, hipStream_t s, int xp, int yp,
                      bool nt, int wpitch, const FuseArgs &fz = FuseArgs()) {
  const size_t wts = w_tile_stride(KT), wks = w_k_stride(wpitch);
  const int ncb = (NTILES + NT - 1) / NT;
  dim3 grid(ncb, S);
  size_t lds = KW > 1 ? (size_t)(KW - 1) * MT * NT * 4 * 64 * sizeof(float) : 0;
  // software-pipelined k-loop once every wave has >= 2 full batches (LLaMA-7B
  // decode at T = 8, cold: qkv 21.2 -> 19.5 us, gate/up 39.1 -> 36.8, lm_head
  // 49.5 -> 46.1); short loops (the SSM, K = 768) keep the batched form, which
  // the pipeline slowed (SSM lm_head warm 9.3 -> 12.1 us).
  // FFMI_SKINNY_PIPE=0/1 forces it off/on (A/B runs).
  static const int force = getenv("FFMI_SKINNY_PIPE") ? atoi(getenv("FFMI_SKINNY_PIPE")) : -1;
  const int per_wave = ((KT + S - 1) / S + KW - 1) / KW;
  const bool pipe = force >= 0 ? force != 0 : per_wave >= 2 * U;
#define FFMI_SKINNY_LAUNCH(PP, NL)                                                             \
  hipLaunchKernelGGL((gemm_skinny_kernel<MT, NT, KW, U, EPI, PP, NL, FZ>), grid, dim3(KW * 64), \
                     lds, s, X, Wp, Y, ws, T, N, K, KT, NTILES, xp, yp, wts, wks, fz)
  if (pipe) {
    if (nt) FFMI_SKINNY_LAUNCH(true, true);
    else FFMI_SKINNY_LAUNCH(true, false);
  } else {
    if (nt) FFMI_SKINNY_LAUNCH(false, true);
    else FFMI_SKINNY_LAUNCH(false, false);
  }
#undef FFMI_SKINNY_LAUNCH
  return hipGetLastError();
}

// Wide, short-K layers (the 68M SSM's lm_head: 2000 tiles, K = 768): one
// WAVE per group of NT tiles over the whole K (a single MFMA chain per tile,
// no cross-wave reduction, no LDS), four independent waves per workgroup.
// The K-split form launches 1000 short 4-wave workgroups whose loads never
// fill the CU (13 us for 49 MB from the Infinity Cache); here each wave keeps
// two batches of UB k-steps in flight (double-buffered registers).
template <int MT, int NT, int UB, bool NTL, int WPG = 4>
__global__ __launch_bounds__(WPG * 64) void gemm_wave_kernel(const uint16_t *__restrict__ X,
                                                             const uint16_t *__restrict__ Wp,
                                                             uint16_t *__restrict__ Y, int T, int N,
                                                             int KT, int NTILES, int xp, int yp,
                                                             size_t wts, size_t wks) {
  const int lane = threadIdx.x & 63;
  const int g = blockIdx.x * WPG + (threadIdx.x >> 6);
  if (g * NT >= NTILES) return;
  const int XS = xp ? 512 : 32;
  const uint16_t *xrow[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    if (xp) {
      xrow[i] = X + ((size_t)min(i, (T - 1) >> 4) * KT * 64 + lane) * 8;
    } else {
      const int r = min(i * 16 + (lane & 15), T - 1);
      xrow[i] = X + (size_t)r * (KT * 32) + 8 * (lane >> 4);
    }
  }
  const uint16_t *wrow[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) wrow[j] = Wp + (size_t)min(g * NT + j, NTILES - 1) * wts + lane * 8;
  f4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  h8 bA[UB][NT], xA[UB][MT], bB[UB][NT], xB[UB][MT];
  auto ld = [&](h8(&bb)[UB][NT], h8(&xx)[UB][MT], int k0) {
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int kk = min(k0 + u, KT - 1);
#pragma unroll
      for (int j = 0; j < NT; ++j) bb[u][j] = ld_weight<NTL>(wrow[j] + (size_t)kk * wks);
#pragma unroll
      for (int i = 0; i < MT; ++i) xx[u][i] = *reinterpret_cast<const h8 *>(xrow[i] + (size_t)kk * XS);
    }
  };
  const h8 zero = {0, 0, 0, 0, 0, 0, 0, 0};
  auto mm = [&](h8(&bb)[UB][NT], h8(&xx)[UB][MT], int k0) {
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      if (k0 + u >= KT) {  // past K: re-loaded fragments times a zero weight
#pragma unroll
        for (int j = 0; j < NT; ++j) bb[u][j] = zero;
      }
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xx[u][i], bb[u][j], acc[i][j], 0, 0, 0);
    }
  };
  ld(bA, xA, 0);
  for (int k0 = 0; k0 < KT; k0 += 2 * UB) {
    if (k0 + UB < KT) ld(bB, xB, k0 + UB);
    __builtin_amdgcn_sched_barrier(0);
    mm(bA, xA, k0);
    __builtin_amdgcn_sched_barrier(0);
    if (k0 + 2 * UB < KT) ld(bA, xA, k0 + 2 * UB);
    __builtin_amdgcn_sched_barrier(0);
    if (k0 + UB < KT) mm(bB, xB, k0 + UB);
    __builtin_amdgcn_sched_barrier(0);
  }
  // C layout: column lane & 15, rows (lane >> 4) * 4 + r
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int n = (g * NT + j) * 16 + (lane & 15);
    if (g * NT + j >= NTILES || n >= N) continue;
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = i * 16 + (lane >> 4) * 4 + r;
        if (m < T)
          Y[yp ? act_packed_off(m, n, N) : (size_t)m * N + n] = __half_as_ushort(__float2half_rn(acc[i][j][r]));
      }
  }
}

// Split-K factor of the skinny path: only narrow layers (few column groups,
// e.g. the 68M SSM's o/down with 48 tiles) and only when the consumer takes
// the partial slabs (no reduce pass); keeps >= 4 k-steps per wave.
static int skinny_split(int T, int N, int K, int epi, bool deferrable) {
  // FFMI_SKINNY_SPLIT=0 keeps every skinny launch unsplit (A/B runs)
  static const bool off = getenv("FFMI_SKINNY_SPLIT") && atoi(getenv("FFMI_SKINNY_SPLIT")) == 0;
  if (off || !deferrable || epi || T > 64) return 1;
  const int ntiles = (N + 15) / 16;
  if (ntiles >= 128) return 1;
  const int KT = K / 32;
  int S = 256 / ntiles;
  S = std::min(S, std::max(1, KT / 8));  // >= 1 k-step per wave of an 8-wave slice
  return std::max(1, std::min(S, 8));
}

// The fused residual/norm forms (FuseArgs; S == 1, T <= 32): the unfused
// path's tile and wave choices, one instantiation set per role.
template <int MT, int U, int FZ>
static hipError_t dispatch_fused(const uint16_t *X, const uint16_t *Wp, uint16_t *Y, int T, int N,
                                 int K, int KT, int epi, hipStream_t s, int xp, int yp, bool nt,
                                 int wpitch, const FuseArgs &fz) {
  const int ntiles = (N + 15) / 16;
  // FFMI_FZ_KW8 (A/B): 8 K-split waves instead of 4 for the one-row-tile
  // consumer launches -- 1: qkv, 2: qkv and gate/up
  static const int kw8 = getenv("FFMI_FZ_KW8") ? atoi(getenv("FFMI_FZ_KW8")) : 0;
  if (epi == FFMI_EPI_SILU_MUL) {
    if constexpr (FZ == 2) {
      if (kw8 >= 2 && MT == 1)
        return run<MT, 2, 8, U, 1, 2>(X, Wp, Y, nullptr, T, N, K, KT, 2 * ntiles, 1, s, xp, yp, nt,
                                      wpitch, fz);
      return run<MT, 2, 4, U, 1, 2>(X, Wp, Y, nullptr, T, N, K, KT, 2 * ntiles, 1, s, xp, yp, nt,
                                    wpitch, fz);
    }
    return hipErrorInvalidValue;
  }
  if constexpr (FZ == 2)
    if (kw8 >= 1 && MT == 1 && ntiles >= 512)
      return run<MT, 1, 8, U, 0, FZ>(X, Wp, Y, nullptr, T, N, K, KT, ntiles, 1, s, xp, yp, nt, wpitch, fz);
  // FFMI_FZ_NT2=1: two tiles per workgroup at one row tile too (A/B)
  static const bool nt2 = getenv("FFMI_FZ_NT2") && atoi(getenv("FFMI_FZ_NT2")) != 0;
  if ((MT >= 2 || nt2) && ntiles >= 512)
    return run<MT, 2, 4, U, 0, FZ>(X, Wp, Y, nullptr, T, N, K, KT, ntiles, 1, s, xp, yp, nt, wpitch, fz);
  if (ntiles < 512 && KT >= 64 && !nt)
    return run<MT, 1, 8, U, 0, FZ>(X, Wp, Y, nullptr, T, N, K, KT, ntiles, 1, s, xp, yp, nt, wpitch, fz);
  return run<MT, 1, 4, U, 0, FZ>(X, Wp, Y, nullptr, T, N, K, KT, ntiles, 1, s, xp, yp, nt, wpitch, fz);
}

template <int MT, int U>
static hipError_t dispatch_nt(const uint16_t *X, const uint16_t *Wp, uint16_t *Y, float *ws,
                              int T, int N, int K, int KT, int epi, int S, hipStream_t s,
                              int xp, int yp, bool nt, int wpitch) {
  int ntiles = (N + 15) / 16;
  if (!wpitch) wpitch = epi == FFMI_EPI_SILU_MUL ? 2 * ntiles : ntiles;
  if (epi == FFMI_EPI_SILU_MUL)
    return run<MT, 2, 4, U, 1>(X, Wp, Y, ws, T, N, K, KT, 2 * ntiles, 1, s, xp, yp, nt, wpitch);
  // diagnostics: FFMI_SKINNY="NT,KW" forces the tile count and K-split waves
  // of every unsplit skinny launch (A/B runs, scripts/gemm_bench.py)
  static int fnt = -1, fkw = 0;
  if (fnt < 0) {
    fnt = 0;
    if (const char *e = getenv("FFMI_SKINNY")) (void)sscanf(e, "%d,%d", &fnt, &fkw);
  }
  if (fnt > 0 && S == 1 && MT <= 2) {
    if (fnt == 1 && fkw == 4) return run<MT, 1, 4, U, 0>(X, Wp, Y, ws, T, N, K, KT, ntiles, 1, s, xp, yp, nt, wpitch);
    if (fnt == 1 && fkw == 8) return run<MT, 1, 8, U, 0>(X, Wp, Y, ws, T, N, K, KT, ntiles, 1, s, xp, yp, nt, wpitch);
    if (fnt == 2 && fkw == 4) return run<MT, 2, 4, U, 0>(X, Wp, Y, ws, T, N, K, KT, ntiles, 1, s, xp, yp, nt, wpitch);
    if (fnt == 2 && fkw == 8) return run<MT, 2, 8, U, 0>(X, Wp, Y, ws, T, N, K, KT, ntiles, 1, s, xp, yp, nt, wpitch);
    if (fnt == 4 && fkw == 4) return run<MT, 4, 4, U, 0>(X, Wp, Y, ws, T, N, K, KT, ntiles, 1, s, xp, yp, nt, wpitch);
    if (fnt == 4 && fkw == 2) return run<MT, 4, 2, U, 0>(X, Wp, Y, ws, T, N, K, KT, ntiles, 1, s, xp, yp, nt, wpitch);
    if (fnt == 2 && fkw == 2) return run<MT, 2, 2, U, 0>(X, Wp, Y, ws, T, N, K, KT, ntiles, 1, s, xp, yp, nt, wpitch);
  }
  // wide, short-K layers (the SSM lm_head): one wave per 2 tiles over the
  // whole K (gemm_wave_kernel; FFMI_WAVE_GEMM=0 keeps the K-split form)
  static const bool wave_ok = !getenv("FFMI_WAVE_GEMM") || atoi(getenv("FFMI_WAVE_GEMM")) != 0;
  if (wave_ok && ntiles >= 1024 && KT <= 32 && S == 1) {
    const size_t wts = w_tile_stride(KT), wks = w_k_stride(wpitch);
    // two tiles per wave: SSM lm_head (32000 x 768) at T = 24 11.1 us (13.3
    // in the K-split form, 13.3 with one tile per wave and twice the waves),
    // T = 8 9.4 us (12.5)
    // (FFMI_WAVE_FORM=NT,WPG: tiles per wave and waves per workgroup, A/B)
    static int wnt = 2, wpg = 4;
    static bool wread = false;
    if (!wread) {
      wread = true;
      if (const char *e = getenv("FFMI_WAVE_FORM")) (void)sscanf(e, "%d,%d", &wnt, &wpg);
    }
#define FFMI_WAVE(NTV, WPGV, NL)                                                               \
  hipLaunchKernelGGL((gemm_wave_kernel<MT, NTV, 4, NL, WPGV>),                                 \
                     dim3(((ntiles + NTV - 1) / NTV + WPGV - 1) / WPGV), dim3(WPGV * 64), 0, s, X, \
                     Wp, Y, T, N, KT, ntiles, xp, yp, wts, wks)
    if (wnt == 4 && wpg == 2) {
      if (nt) FFMI_WAVE(4, 2, true);
      else FFMI_WAVE(4, 2, false);
    } else if (wnt == 4 && wpg == 4) {
      if (nt) FFMI_WAVE(4, 4, true);
      else FFMI_WAVE(4, 4, false);
    } else if (wnt == 3 && wpg == 2) {
      if (nt) FFMI_WAVE(3, 2, true);
      else FFMI_WAVE(3, 2, false);
    } else if (wnt == 2 && wpg == 2) {
      if (nt) FFMI_WAVE(2, 2, true);
      else FFMI_WAVE(2, 2, false);
    } else {
      if (nt) FFMI_WAVE(2, 4, true);
      else FFMI_WAVE(2, 4, false);
    }
#undef FFMI_WAVE
    return hipGetLastError();
  }
  // wide layers (lm_head): two tiles per workgroup once there are >= 2 row
  // tiles (SSM lm_head at T = 24: 16.1 -> 12.3 us warm; at one row tile a
  // single tile stays faster: LLaMA-7B lm_head T = 8 cold 47.8 vs 55.8 us)
  if (MT >= 2 && ntiles >= 512)
    return run<MT, 2, 4, U, 0>(X, Wp, Y, ws, T, N, K, KT, ntiles, S, s, xp, yp, nt, wpitch);
  // 8-wave groups only where the accumulators fit 2 waves/SIMD (no spills)
  if (ntiles >= 512 || MT >= 8)
    return run<MT, 1, 4, U, 0>(X, Wp, Y, ws, T, N, K, KT, ntiles, S, s, xp, yp, nt, wpitch);
  // ... and where each wave still gets a full batch of U k-steps (K = 768 of
  // the SSM: 4 waves x 6 k-steps beat 8 x 3, qkv T = 24: 5.7 -> 4.2 us).
  // Non-temporal weight loads (FFMI_W_STREAM) keep 4 waves at every row-tile
  // count (LLaMA-7B decode, cold, T = 1-16: o 7.6-8.8 -> 7.2-8.6 us, down
  // 17.0-24.8 -> 16.4-21.9 us over two runs of gemm_bench.py --wstream; T = 32
  // within noise), so a row's reduction order still depends on (N-tile, K,
  // policy) only, not on T: the threshold is a fixed 64 k-steps per slice
  // (8 waves x the largest batch U = 8), never U itself, which depends on T.
  if ((KT + S - 1) / S >= 64 && !nt)
    return run<MT, 1, 8, U, 0>(X, Wp, Y, ws, T, N, K, KT, ntiles, S, s, xp, yp, nt, wpitch);
  return run<MT, 1, 4, U, 0>(X, Wp, Y, ws, T, N, K, KT, ntiles, S, s, xp, yp, nt, wpitch);
}

// ---------------------------------------------------------------------------
// M-split GEMM for 64 < T (verify batches, SSM init, prefill blocks).
//
// The skinny kernel above re-reads the whole activation block from L2 in
// every wave (K split over waves) and runs at 1 wave/SIMD at T ~ 168, which
// made it latency-bound (~0.7 TB/s).  Here the 4 waves of a workgroup split
// the ROWS (MTW m-tiles each, 64*MTW rows per block) and share one weight
// tile of NTW 16-column tiles per 32-deep k-step, staged through LDS with a
// register double buffer (load k+1 while the MFMAs of k run, one barrier per
// k-step).  Each wave loads only its own rows of X.  Small-N layers are
// split over K across workgroups (S slices, fp32 partials reduced in slice
// order by gemm_reduce_kernel), so every layer puts >= ~256 workgroups on
// the 256 CUs.  Reduction order per output element: MFMA chain over the
// slice's k-steps, then slices 0..S-1 -- fixed by (N, K, S), not by T.
// ---------------------------------------------------------------------------
// Epilogue of the M-split kernel.  Its MFMAs compute D = W_tile . X_tile^T,
// so a lane's accumulator holds FOUR CONSECUTIVE OUTPUT COLUMNS
// n = tile*16 + (lane>>4)*4 + r of one row m = m0 + i*16 + (lane&15): the
// fp16 output goes out as one 8-byte store and an fp32 partial as one 16-byte
// store per (i, j) (scalar 2-/4-byte stores in the C layout were the
// kernel's single largest cost).
template <int MTW, int NTW, int EPI>
__device__ __forceinline__ void mid_store(const f4 (&acc)[MTW][NTW], uint16_t *__restrict__ Y,
                                          float *__restrict__ Ypart, int T, int N, int NTILES,
                                          int S, int ks, int tile0, int m0, int lane, int yp) {
  const int mr = lane & 15, nq = (lane >> 4) * 4;
  if (S > 1) {
    const int NP = NTILES * 16;
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      const int tile = tile0 + j;
      if (tile >= NTILES) continue;
#pragma unroll
      for (int i = 0; i < MTW; ++i) {
        const int m = m0 + i * 16 + mr;
        if (m < T)
          // (non-temporal stores here measured slower end to end: the
          // consumer then reads the slabs from memory instead of L2)
          *reinterpret_cast<f4 *>(Ypart + ((size_t)ks * T + m) * NP + tile * 16 + nq) = acc[i][j];
      }
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < NTW; j += (EPI ? 2 : 1)) {
    const int tile = tile0 + j;
    if (tile >= NTILES) continue;
    const int n = (EPI ? (tile >> 1) : tile) * 16 + nq;
    if (n >= N) continue;
#pragma unroll
    for (int i = 0; i < MTW; ++i) {
      const int m = m0 + i * 16 + mr;
      if (m >= T) continue;
      uint16_t o[4];
#pragma unroll
      for (int r = 0; r < 4; ++r)
        o[r] = EPI ? silu_mul_h(acc[i][j][r], acc[i][j + 1][r])
                   : __half_as_ushort(__float2half_rn(acc[i][j][r]));
      uint16_t *dst = yp ? Y + act_packed_off(m, n, N) : Y + (size_t)m * N + n;
      if (n + 4 <= N && (((uintptr_t)dst & 7) == 0)) {
        *reinterpret_cast<uint2 *>(dst) =
            make_uint2(o[0] | ((uint32_t)o[1] << 16), o[2] | ((uint32_t)o[3] << 16));
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (n + r < N) dst[r] = o[r];
      }
    }
  }
}

// Diagnostic stamps (FFMI_GEMM_STAMP=1 builds only): per wave
// {realtime start, after prologue, after k-loop, end, HW_ID, XCC_ID, core-clock
// counter (s_memtime) after prologue, after k-loop}; realtime is 100 MHz, so
// the k-loop's clock = d(memtime) / d(realtime) x 100 MHz.
__device__ long long *g_gemm_stamps;
__device__ __forceinline__ long long rt_now() { return __builtin_amdgcn_s_memrealtime(); }

template <int MTW, int NTW, int PF, int EPI, bool STAMP = false, bool XP = false, bool ULD = false,
          bool NTL = false>
// (two workgroups per CU = 256 registers per wave: up to 24 accumulator tiles,
// MTW x NTW; 4 x 8 takes the whole register file, one workgroup per CU)
__global__ __launch_bounds__(256, NTW <= 8 && MTW * NTW <= 24 ? 2 : 1) void gemm_mid_kernel(
    const uint16_t *__restrict__ X, const uint16_t *__restrict__ Wp,
    uint16_t *__restrict__ Y, float *__restrict__ Ypart, int T, int N, int K, int KT,
    int NTILES, int S, int yp, size_t wts, size_t wks) {
  long long st0 = 0, st1 = 0, st2 = 0, ck1 = 0, ck2 = 0;
  if (STAMP) st0 = rt_now();
  static_assert(NTW % 2 == 0, "gate/up tiles come in pairs");
  static_assert(PF >= 2, "ring depth");
  // weight tiles j = wave + 4p are loaded by wave (j % 4); with NTW % 4 != 0
  // the last round is loaded by the first NTW % 4 waves only
  constexpr int PPT = (NTW + 3) / 4;
  __shared__ __attribute__((aligned(16))) h8 sB[2][NTW][64];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int tile0 = blockIdx.x * NTW;
  const int ks = blockIdx.y;
  const int m0 = blockIdx.z * (4 * MTW * 16) + wave * MTW * 16;
  const int per = (KT + S - 1) / S;
  const int kb = min(KT, ks * per);
  const int ke = min(KT, kb + per);

  const uint16_t *bsrc[PPT];
  int bj[PPT];
#pragma unroll
  for (int p = 0; p < PPT; ++p) {
    bj[p] = wave + 4 * p;
    // ULD: waves past the last tile re-load the block's last tile (an L2 hit
    // beside the wave that owns it) so that EVERY wave issues PPT weight loads
    // per k-step: loads behind a wave-dependent branch are invisible to the
    // compiler's vmcnt counting, which then waits for ~2 ring slots, not PF-1
    const int t = min(tile0 + (ULD ? min(bj[p], NTW - 1) : bj[p]), NTILES - 1);
    bsrc[p] = Wp + (size_t)t * wts + lane * 8;
  }
  // X row-major [T][K] (16 rows x 64 B per fragment load), or XP: packed
  // activation tiles [T/16][KT][64 lanes][8] (one contiguous 1 KiB per load)
  constexpr int XS = XP ? 512 : 32;  // halves per k-step
  const uint16_t *xrow[MTW];
#pragma unroll
  for (int i = 0; i < MTW; ++i) {
    if (XP) {
      const int mt = min((m0 + i * 16) >> 4, (T - 1) >> 4);
      xrow[i] = X + ((size_t)mt * KT * 64 + lane) * 8;
    } else {
      const int r = min(m0 + i * 16 + (lane & 15), T - 1);
      xrow[i] = X + (size_t)r * K + 8 * (lane >> 4);
    }
  }
  f4 acc[MTW][NTW];
#pragma unroll
  for (int i = 0; i < MTW; ++i)
#pragma unroll
    for (int j = 0; j < NTW; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  // Software pipeline, one barrier per 32-deep k-step.  A PF-deep register
  // ring holds BOTH operands of k-steps k..k+PF-1: slot q = (X(k), B(k)).
  // Loads retire in issue order (vmcnt), so X must be issued as early as the
  // weights: X(k) is consumed PF steps after issue, B(k+1) goes to the LDS
  // tile PF-1 steps after issue, and no consumer waits on a young load.
  auto kloop = [&](auto NVc) {
    constexpr int NV = decltype(NVc)::value;
    h8 bq[PF][PPT];
    h8 xq[PF][MTW];
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      const int kq = min(kb + q, ke - 1);
#pragma unroll
      for (int i = 0; i < NV; ++i) xq[q][i] = *reinterpret_cast<const h8 *>(xrow[i] + (size_t)kq * XS);
#pragma unroll
      for (int p = 0; p < PPT; ++p)
        if (ULD || NTW % 4 == 0 || bj[p] < NTW) bq[q][p] = ld_weight<NTL>(bsrc[p] + (size_t)kq * wks);
    }
#pragma unroll
    for (int p = 0; p < PPT; ++p)
      if (NTW % 4 == 0 || bj[p] < NTW) sB[0][bj[p]][lane] = bq[0][p];
    __syncthreads();
    if (STAMP) st1 = rt_now(), ck1 = __builtin_amdgcn_s_memtime();
    // one k-step on ring slot Q; MFMAs read the slot in place, then it is
    // refilled (a copy would rotate the ring through fresh registers and
    // force vmcnt drains at the loop back-edge)
    int cur = 0;
    auto step = [&](auto Qc, int kt) {
      constexpr int Q = decltype(Qc)::value;
      h8 b[NTW];
#pragma unroll
      for (int j = 0; j < NTW; ++j) b[j] = sB[cur][j][lane];
#pragma unroll
      for (int i = 0; i < NV; ++i)
#pragma unroll
        for (int j = 0; j < NTW; ++j)  // D = W . X^T (see mid_store)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(b[j], xq[Q][i], acc[i][j], 0, 0, 0);
      const int kw = min(kt + PF, ke - 1);
#pragma unroll
      for (int i = 0; i < NV; ++i) xq[Q][i] = *reinterpret_cast<const h8 *>(xrow[i] + (size_t)kw * XS);
#pragma unroll
      for (int p = 0; p < PPT; ++p)
        if (ULD || NTW % 4 == 0 || bj[p] < NTW) bq[Q][p] = ld_weight<NTL>(bsrc[p] + (size_t)kw * wks);
      // B(kt+1) lives in ring slot (Q+1) % PF
#pragma unroll
      for (int p = 0; p < PPT; ++p)
        if (NTW % 4 == 0 || bj[p] < NTW) sB[cur ^ 1][bj[p]][lane] = bq[(Q + 1) % PF][p];
      __syncthreads();
      cur ^= 1;
    };
    int kt0 = kb;
    for (; kt0 + PF <= ke; kt0 += PF)  // steady state: whole ring turns
      static_for<PF>([&](auto Qc) { step(Qc, kt0 + decltype(Qc)::value); });
    static_for<PF - 1>([&](auto Qc) {  // tail: < PF steps, slots 0..
      if (kt0 + decltype(Qc)::value < ke) step(Qc, kt0 + decltype(Qc)::value);
    });
  };
  if (kb < ke) kloop(std::integral_constant<int, MTW>{});
  if (STAMP) st2 = rt_now(), ck2 = __builtin_amdgcn_s_memtime();

  mid_store<MTW, NTW, EPI>(acc, Y, Ypart, T, N, NTILES, S, ks, tile0, m0, lane, yp);
  if (STAMP) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const long long st3 = rt_now();
    unsigned hwid, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    if (lane == 0 && g_gemm_stamps) {
      const long b = blockIdx.x + (long)gridDim.x * (blockIdx.y + (long)gridDim.y * blockIdx.z);
      long long *d = g_gemm_stamps + (b * 4 + wave) * 8;
      d[0] = st0; d[1] = st1; d[2] = st2; d[3] = st3; d[4] = hwid; d[5] = xcc;
      d[6] = ck1; d[7] = ck2;
    }
  }
}

// Compute-bound form for prefill blocks (T >= 497, packed activations): one
// 512-thread workgroup per 256 x 256 output tile, the 8 waves as 2 (rows) x
// 4 (weight tiles), each wave 128 rows x 4 weight tiles (8 x 4 MFMA
// accumulators).  Both operands are already in MFMA fragment order (1 KiB per
// 16 x 32 fragment, weights.hip / pack_act_kernel), so every fragment lands in
// LDS with ONE global_load_lds_dwordx4 wave-instruction (lane-linear: no
// swizzle, conflict-free ds_read_b128 reads).  A ring of NB one-k-step stages
// (32 fragments = 32 KiB each, 4 per wave) with NB - 1 stages in flight across
// the barriers: a counted s_waitcnt vmcnt (never 0 in the steady state) and a
// raw s_barrier, never __syncthreads (its fence would drain the DMAs; cdna
// guide, "Pipelining across barriers").  The k order of every accumulator is
// the M-split kernel's (k-steps in sequence, one MFMA each), so outputs are
// bit-identical to gemm_mid_kernel at S = 1.  Blocks are remapped so the row
// blocks of a weight tile share an XCD (bijective remap): its weights come
// from HBM once per XCD L2.
template <int EPI, int NB>
__global__ __launch_bounds__(512, 1) void gemm_tile_kernel(
    const uint16_t *__restrict__ X, const uint16_t *__restrict__ Wp, uint16_t *__restrict__ Y,
    int T, int N, int KT, int NTILES, int MT, int nbm, int yp, size_t wts, size_t wks) {
  __shared__ __attribute__((aligned(1024))) h8 lds[NB][32][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nwg = gridDim.x, b = blockIdx.x;
  const int xcd = b & 7, q = nwg >> 3, r = nwg & 7;
  const int L = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
  const int bn = L / nbm, bm = L % nbm;
  // this wave's 4 DMA fragments f = wave + 8p of a stage: X m-tile f (< 16)
  // or weight tile f - 16
  const uint16_t *src[4];
  size_t step[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int f = wave + 8 * p;
    if (f < 16) {
      src[p] = X + (size_t)min(bm * 16 + f, MT - 1) * KT * 512 + lane * 8;
      step[p] = 512;
    } else {
      src[p] = Wp + (size_t)min(bn * 16 + f - 16, NTILES - 1) * wts + lane * 8;
      step[p] = wks;
    }
  }
  auto issue_one = [&](int kt, int p) {
    __builtin_amdgcn_global_load_lds(
        (const __attribute__((address_space(1))) void *)(src[p] + (size_t)kt * step[p]),
        (__attribute__((address_space(3))) void *)(&lds[kt % NB][wave + 8 * p][0]), 16, 0, 0);
  };
  auto issue = [&](int kt) {
#pragma unroll
    for (int p = 0; p < 4; ++p) issue_one(kt, p);
  };
  const int wm = wave >> 2, wn = wave & 3;
  f4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kt = 0; kt < NB - 1; ++kt)
    if (kt < KT) issue(kt);
  for (int kt = 0; kt < KT; ++kt) {
    // this wave's DMAs of step kt are done once at most the younger steps'
    // (up to NB - 2 of them, 4 ops each) remain; then the barrier makes every
    // wave's DMAs of step kt visible and retires every wave's reads of the
    // buffer step kt + NB - 1 overwrites (step kt - 1's)
    const int ahead = min(KT - 1 - kt, NB - 2);
    if (ahead >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const bool more = kt + NB - 1 < KT;
    const int buf = kt % NB;
    // the stage's fragment reads, then its 32 MFMAs with the next stage's 4
    // DMAs issued between them (an LDS-DMA issue costs ~60-185 cycles of the
    // wave's issue slots: issued in a block they serialise with the MFMAs,
    // spread they hide under the matrix pipe, cdna guide cycle table)
    h8 xf[8], wf[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) wf[j] = lds[buf][16 + wn * 4 + j][lane];
#pragma unroll
    for (int i = 0; i < 8; ++i) xf[i] = lds[buf][wm * 8 + i][lane];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j)  // D = W . X^T (see mid_store)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[j], xf[i], acc[i][j], 0, 0, 0);
      if ((i & 1) == 0 && more) issue_one(kt + NB - 1, i >> 1);
    }
  }
  mid_store<8, 4, EPI>(acc, Y, nullptr, T, N, NTILES, 1, 0, bn * 16 + wn * 4,
                       (bm * 16 + wm * 8) * 16, lane, yp);
}

static long long *stamp_buf() {
  static long long *buf = nullptr;
  if (!buf) {
    if (hipMalloc(&buf, (size_t)8 << 20) != hipSuccess) return nullptr;
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_gemm_stamps), &buf, sizeof(buf));
  }
  return buf;
}
static long g_stamp_entries = 0;


// Sum the S fp32 partial slabs in slice order, then the epilogue; one thread
// per 4 consecutive output columns (16-B slab loads, 8-B fp16 store).
template <int EPI, int MAXS>
__global__ void gemm_reduce_kernel(const float *__restrict__ Ypart, uint16_t *__restrict__ Y,
                                   int T, int N, int NTILES, int S, int yp) {
  const int NP = NTILES * 16;
  const int nq = (N + 3) / 4;
  const long idx = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (idx >= (long)T * nq) return;
  const int m = (int)(idx / nq), n = (int)(idx % nq) * 4;
  const size_t slab = (size_t)T * NP;
  f4 acc, up;
  // all MAXS >= S slab loads go out before the first add (one memory round
  // trip, not S); indices past S re-read the last slab and are not added
  f4 pa[MAXS], pu[MAXS];
  const float *src = EPI == 0 ? Ypart + (size_t)m * NP + n
                              : Ypart + (size_t)m * NP + (n >> 4) * 32 + (n & 15);
#pragma unroll
  for (int s = 0; s < MAXS; ++s) {
    const float *q = src + (size_t)min(s, S - 1) * slab;
    pa[s] = *reinterpret_cast<const f4 *>(q);
    if (EPI) pu[s] = *reinterpret_cast<const f4 *>(q + 16);
  }
  acc = pa[0];
  if (EPI) up = pu[0];
#pragma unroll
  for (int s = 1; s < MAXS; ++s)
    if (s < S) {
      acc += pa[s];
      if (EPI) up += pu[s];
    }
  uint16_t o[4];
#pragma unroll
  for (int r = 0; r < 4; ++r)
    o[r] = EPI ? silu_mul_h(acc[r], up[r]) : __half_as_ushort(__float2half_rn(acc[r]));
  uint16_t *dst = yp ? Y + act_packed_off(m, n, N) : Y + (size_t)m * N + n;
  if (n + 4 <= N && (((uintptr_t)dst & 7) == 0)) {
    *reinterpret_cast<uint2 *>(dst) =
        make_uint2(o[0] | ((uint32_t)o[1] << 16), o[2] | ((uint32_t)o[3] << 16));
  } else {
    for (int r = 0; r < 4; ++r)
      if (n + r < N) dst[r] = o[r];
  }
}

// Launch plan of the M-split kernel: weight tiles per workgroup (NTW) and
// split-K factor (S).  Each workgroup is bound by its CU's load path (per-wave
// timeline, scripts/diag_stamps.py: a k-step moves NTW KiB of weights + 4*MTW
// KiB of activations at ~50 GB/s per CU; two workgroups on one CU each run at
// half speed), so the plan keeps the grid within one wave of 256 workgroups,
// prefers wide tiles (fewer activation bytes per weight byte) and charges the
// split-K reduce pass.  Times in us; only the ranking matters.
struct MidPlan {
  int MTW, NTW, S, mblocks, nblk;
};
// FFMI_MID_MTW4=0: no 4-row-tile waves (A/B)
static const int mid_mtw4 = getenv("FFMI_MID_MTW4") && atoi(getenv("FFMI_MID_MTW4")) == 0 ? 3 : 4;
static MidPlan mid_plan(int T, int N, int K, int epi, bool deferred = false) {
  MidPlan p;
  const int mtiles = (T + 15) / 16;
  // row tiles per wave: 4 waves x MTW tiles cover one row block; 4 for 13-16
  // tiles (T 193-256: the width-4 verify step, T = 216, in ONE row block
  // instead of two that each re-read every weight tile) and for prefill
  // blocks (fewer row blocks re-reading the weights)
  p.MTW = mtiles <= 8 ? 2 : mtiles <= 12 ? 3 : mtiles <= 16 || mtiles > 24 ? mid_mtw4 : 3;
  p.mblocks = (mtiles + 4 * p.MTW - 1) / (4 * p.MTW);
  const int KT = K / 32;
  const int ntiles = (N + 15) / 16 * (epi ? 2 : 1);
  double best = 1e30;
  p.NTW = 8, p.S = 1;
  // measured k-step times (us) at MTW = 3, packed activations (diag_stamps.py)
  // (2 and 4: narrow per-rank shards of tensor parallelism, e.g. LLaMA-7B
  // o_proj at TP = 8 is 256 tiles x K = 512 -- 43 workgroups at NTW = 6)
  static const int ntw_opts[6] = {2, 4, 6, 8, 12, 16};
  static const double base[6] = {0.27, 0.30, 0.36, 0.40, 0.65, 0.90};
  static const int nopt = getenv("FFMI_MID_NARROW") && atoi(getenv("FFMI_MID_NARROW")) == 0 ? 4 : 6;
  for (int o = 6 - nopt; o < 6; ++o) {
    const int ntw = ntw_opts[o];
    if (p.MTW == 4 && ntw > 8) continue;  // (register budget, see launch_gemm)
    const int nblk = (ntiles + ntw - 1) / ntw;
    for (int S = 1; S <= 8 && S <= KT; ++S) {
      const long wgs = (long)nblk * S * p.mblocks;
      const double rounds = (double)((wgs + 255) / 256);
      const double steps = (double)((KT + S - 1) / S);
      const double tstep = base[o] * (ntw + 4.0 * p.MTW) / (ntw + 12.0);
      double t = rounds * (steps * tstep + 4.0);
      const double slab_mb = (double)S * T * ntiles * 16 * 4 / 1e6;
      // slabs cost their write here and their read in the consumer; a
      // deferred read (norm / attention prologue) is no cheaper than the
      // reduce pass's: /6 had picked 8 slabs for LLaMA-7B o_proj at T = 168,
      // 4 tiles x 4 slabs ran 0.6 % faster end to end (3 of 3 A/B pairs)
      // (the SiLU reduce pass re-reads the gate AND up slabs: at the verify
      // size, 9-12 row tiles in one block, a forced-plan sweep of the TP = 8
      // gate/up shard put 4 tiles x 4-5 slabs at 18.4-18.9 us against 21.7
      // for the 6 x 8 the /3 charge picked, profiles/r06_tp8_gateup_plans.log;
      // the TP 1 / 2 / 4 and 65B TP 8 picks are unchanged by /2)
      const double slab_rate = epi && p.MTW == 3 && p.mblocks == 1 ? 2.0 : 3.0;
      if (S > 1) t += deferred ? slab_mb / 3.0 : 3.0 + slab_mb / slab_rate;
      if (t < best - 1e-9) best = t, p.NTW = ntw, p.S = S;
    }
  }
  // prefill blocks (>= 4 row blocks: T > 576 at MTW = 3): the k-step model
  // above is calibrated at T = 168; forced-plan sweeps at T = 1024
  // (scripts/gpu_prefill_plans.sh, LLaMA-7B shapes) put 8 tiles unsplit
  // first on qkv / o / gate-up / lm_head and 8 tiles x 2 slices on the
  // K = 11008 down projection (gate/up 337 -> 270 us, qkv 149 -> 139,
  // down 148 -> 135, lm_head 428 -> 409); FFMI_PREFILL_PLAN=0 keeps the model
  static const bool prefill_plan = !getenv("FFMI_PREFILL_PLAN") || atoi(getenv("FFMI_PREFILL_PLAN")) != 0;
  if (prefill_plan && p.mblocks >= 4) {
    p.NTW = 8;
    p.S = K >= 8192 && KT >= 2 ? 2 : 1;
    // 4-row-tile waves run one workgroup per CU: only where the grid still
    // covers the CUs (T = 1024: o_proj 128 workgroups -> 3-tile waves, 56 vs
    // 70 us; gate/up, down (2 slices), qkv, lm_head keep 4: 267 vs 280 us,
    // 131 vs 142 us, equal)
    if (p.MTW == 4 && (long)((ntiles + 7) / 8) * p.S * p.mblocks < 256) {
      p.MTW = 3;
      p.mblocks = (mtiles + 11) / 12;
    }
  }
  // diagnostics: FFMI_GEMM_PLAN="NTW,S" forces the tile width and split of
  // every M-split launch; "N:K:NTW,S;..." only of the listed shapes
  static const char *force = getenv("FFMI_GEMM_PLAN");
  if (force) {
    const char *q = force;
    while (q && *q) {
      int a = 0, b = 0, c = 0, d = 0, ntw = 0, S = 0;
      const int n = sscanf(q, "%d:%d:%d,%d", &a, &b, &c, &d);
      if (n == 4 && a == N && b == K) ntw = c, S = d;
      else if (n != 4 && sscanf(q, "%d,%d", &a, &b) == 2) ntw = a, S = b;
      if ((ntw == 2 || ntw == 4 || ntw == 6 || ntw == 8 || ntw == 12 || ntw == 16) && S >= 1 &&
          S <= std::min(KT, 8)) {
        p.NTW = ntw, p.S = S;
        break;
      }
      q = strchr(q, ';');
      if (q) ++q;
    }
  }
  if (p.MTW == 4 && p.NTW > 8) p.NTW = 8;
  p.nblk = (ntiles + p.NTW - 1) / p.NTW;
  return p;
}

size_t gemm_workspace_bytes(int T, int N, int K, int epilogue) {
  epilogue &= ~(FFMI_X_PACKED | FFMI_Y_PACKED | FFMI_W_STREAM);
  const int mtiles = (T + 15) / 16;
  if (mtiles <= 4) {
    const int S = skinny_split(T, N, K, epilogue, true);
    return S > 1 ? (size_t)S * T * ((N + 15) / 16) * 16 * sizeof(float) : 0;
  }
  const int ntiles = (N + 15) / 16 * (epilogue ? 2 : 1);
  const int S = std::max(mid_plan(T, N, K, epilogue, false).S,
                         epilogue ? 1 : mid_plan(T, N, K, epilogue, true).S);
  return S > 1 ? (size_t)S * T * ntiles * 16 * sizeof(float) : 0;
}

template <int MTW, int NTW, int PF>
static hipError_t run_mid(const uint16_t *X, const uint16_t *Wp, uint16_t *Y, float *ws,
                          size_t ws_bytes, int T, int N, int K, int epi, hipStream_t s,
                          bool xpacked, int yp, int S, Partials *defer, bool nt, int wpitch) {
  const int KT = K / 32;
  const int ntiles = (N + 15) / 16 * (epi ? 2 : 1);
  const size_t wts = w_tile_stride(KT), wks = w_k_stride(wpitch ? wpitch : ntiles);
  const int mtiles = (T + 15) / 16;
  const int mblocks = (mtiles + 4 * MTW - 1) / (4 * MTW);
  const int nblk = (ntiles + NTW - 1) / NTW;
  const size_t need = (size_t)S * T * ntiles * 16 * sizeof(float);
  if (S > 1 && (!ws || ws_bytes < need)) S = 1;  // no workspace: un-split (slower)
  dim3 grid(nblk, S, mblocks);
  static const bool stamp = getenv("FFMI_GEMM_STAMP") != nullptr;
  // unconditional weight loads (ULD) whenever NTW % 4 != 0 (gate/up T = 168:
  // 55.9 -> 51.2 us, qkv 37.2 -> 34.6 us in scripts/gemm_bench.py);
  // FFMI_MID_ULD=0 turns them off (A/B runs)
  static const bool uld = !getenv("FFMI_MID_ULD") || atoi(getenv("FFMI_MID_ULD")) != 0;
  // non-temporal weight loads only where each weight tile has ONE reader
  // (mblocks == 1); prefill blocks re-read every tile from L2 / the MALL
  const bool ntl = nt && mblocks == 1;
#define FFMI_MID2(E, ST, XPK, U, NL)                                                               \
  hipLaunchKernelGGL((gemm_mid_kernel<MTW, NTW, PF, E, ST, XPK, U, NL>), grid, dim3(256), 0, s, X, \
                     Wp, Y, ws, T, N, K, KT, ntiles, S, yp, wts, wks)
#define FFMI_MID(E, ST, XPK)                                  \
  do {                                                        \
    const bool u_ = uld && NTW % 4;                           \
    if (ST) FFMI_MID2(E, ST, XPK, false, false);              \
    else if (u_ && ntl) FFMI_MID2(E, false, XPK, true, true); \
    else if (u_) FFMI_MID2(E, false, XPK, true, false);       \
    else if (ntl) FFMI_MID2(E, false, XPK, false, true);      \
    else FFMI_MID2(E, false, XPK, false, false);              \
  } while (0)
  if (stamp && !epi && stamp_buf()) {
    g_stamp_entries = (long)nblk * S * mblocks * 4;
    if (xpacked) FFMI_MID(0, true, true);
    else FFMI_MID(0, true, false);
  } else if (xpacked) {
    if (epi) FFMI_MID(1, false, true);
    else FFMI_MID(0, false, true);
  } else {
    if (epi) FFMI_MID(1, false, false);
    else FFMI_MID(0, false, false);
  }
#undef FFMI_MID
#undef FFMI_MID2
  if (defer) {
    defer->S = 0;
    if (S > 1 && !epi) {  // the consumer combines the slabs
      defer->p = ws, defer->S = S, defer->NP = ntiles * 16;
      return hipGetLastError();
    }
  }
  if (S > 1) {
    const long total = (long)T * ((N + 3) / 4);
    const unsigned blocks = (unsigned)((total + 255) / 256);
#define FFMI_RED(E, MS)                                                                    \
  hipLaunchKernelGGL((gemm_reduce_kernel<E, MS>), dim3(blocks), dim3(256), 0, s, ws, Y, T, N, \
                     ntiles, S, yp)
    if (epi) {
      if (S <= 2) FFMI_RED(1, 2);
      else if (S <= 4) FFMI_RED(1, 4);
      else FFMI_RED(1, 8);
    } else {
      if (S <= 2) FFMI_RED(0, 2);
      else if (S <= 4) FFMI_RED(0, 4);
      else FFMI_RED(0, 8);
    }
#undef FFMI_RED
  }
  return hipGetLastError();
}

hipError_t launch_partials_reduce(const Partials &p, uint16_t *Y, int T, int N, hipStream_t s) {
  if (T <= 0 || p.S <= 0) return hipSuccess;
  // (> 8: the per-head o-projection slabs of a small model, OprojArgs)
  if (p.S > 16 || p.NP % 16 || N > p.NP) return hipErrorInvalidValue;
  const long total = (long)T * ((N + 3) / 4);
  const unsigned blocks = (unsigned)((total + 255) / 256);
#define FFMI_PRED(MS)                                                                          \
  hipLaunchKernelGGL((gemm_reduce_kernel<0, MS>), dim3(blocks), dim3(256), 0, s, p.p, Y, T, N, \
                     p.NP / 16, p.S, 0)
  if (p.S <= 2) FFMI_PRED(2);
  else if (p.S <= 4) FFMI_PRED(4);
  else if (p.S <= 8) FFMI_PRED(8);
  else FFMI_PRED(16);
#undef FFMI_PRED
  return hipGetLastError();
}

hipError_t launch_gemm(const uint16_t *X, const uint16_t *Wp, uint16_t *Y, float *ws,
                       size_t ws_bytes, int T, int N, int K, int epilogue, hipStream_t s,
                       Partials *defer, int wpitch, const FuseArgs *fuse) {
  if (defer) defer->S = 0;
  if (T <= 0) return hipSuccess;
  const int KT = K / 32;
  const int mtiles = (T + 15) / 16;
  const bool xp = (epilogue & FFMI_X_PACKED) != 0;
  const int yp = (epilogue & FFMI_Y_PACKED) ? 1 : 0;
  const bool nt = (epilogue & FFMI_W_STREAM) != 0;
  epilogue &= ~(FFMI_X_PACKED | FFMI_Y_PACKED | FFMI_W_STREAM);
  if ((xp && K % 32) || (yp && N % 32)) return hipErrorInvalidValue;
  if (fuse && fuse->kind) {
    // producer: row-major residual out, plain epilogue; consumer: row-major X
    // (the residual), K = the norm width; both unsplit, T <= 32
    if (mtiles > 2 || N % 16 || K % 32) return hipErrorInvalidValue;
    if (fuse->kind == 1 && (epilogue || yp || !fuse->res_in || !fuse->ss_out))
      return hipErrorInvalidValue;
    if (fuse->kind == 2 && (xp || !fuse->ss_in || !fuse->wnorm || fuse->nss <= 0 || fuse->nss > 256))
      return hipErrorInvalidValue;
    const int wp = wpitch ? wpitch : (epilogue == FFMI_EPI_SILU_MUL ? 2 : 1) * ((N + 15) / 16);
#define FFMI_FZ(MTV, FZV) \
  return dispatch_fused<MTV, 8, FZV>(X, Wp, Y, T, N, K, KT, epilogue, s, xp, yp, nt, wp, *fuse)
    if (mtiles <= 1) {
      if (fuse->kind == 1) FFMI_FZ(1, 1);
      FFMI_FZ(1, 2);
    }
    if (fuse->kind == 1) FFMI_FZ(2, 1);
    FFMI_FZ(2, 2);
#undef FFMI_FZ
  }
  // prefill blocks: the compute-bound 256 x 256 tile form where its grid
  // covers the CUs (FFMI_TILE_GEMM: 0 never, 2 whenever the shape allows --
  // A/B runs and tests; read per call)
  if (mtiles >= 32 && xp && (!fuse || !fuse->kind)) {
    const char *e = getenv("FFMI_TILE_GEMM");
    const int mode = e ? atoi(e) : 1;
    const int ntiles = (N + 15) / 16 * (epilogue ? 2 : 1);
    const int nbn = (ntiles + 15) / 16, nbm = (mtiles + 15) / 16;
    // one 256 x 256 tile per CU and round: worth it where the rounds are
    // well filled (T = 1024: qkv 192 tiles 168 -> 140 us, lm_head 500 tiles
    // 396 -> 314, gate/up 344 tiles 274 -> 268; T = 577: gate/up's 258 tiles
    // = one round + 2, 188 -> 221, stays M-split)
    const int nwg = nbn * nbm, rounds = (nwg + 255) / 256;
    if (mode == 2 || (mode == 1 && nwg >= 160 && nwg * 10 >= rounds * 256 * 6)) {
      if (defer) defer->S = 0;
      const size_t wts = w_tile_stride(KT), wks = w_k_stride(wpitch ? wpitch : ntiles);
      if (epilogue)
        hipLaunchKernelGGL((gemm_tile_kernel<1, 4>), dim3(nbn * nbm), dim3(512), 0, s, X, Wp, Y, T,
                           N, KT, ntiles, mtiles, nbm, yp, wts, wks);
      else
        hipLaunchKernelGGL((gemm_tile_kernel<0, 4>), dim3(nbn * nbm), dim3(512), 0, s, X, Wp, Y, T,
                           N, KT, ntiles, mtiles, nbm, yp, wts, wks);
      return hipGetLastError();
    }
  }
  if (mtiles > 4) {
    const MidPlan p = mid_plan(T, N, K, epilogue, defer != nullptr && !epilogue);
#define FFMI_RUN(M, NW) \
  return run_mid<M, NW, 4>(X, Wp, Y, ws, ws_bytes, T, N, K, epilogue, s, xp, yp, p.S, defer, nt, \
                           wpitch)
    if (p.MTW == 4) {
      if (p.NTW == 2) FFMI_RUN(4, 2);
      if (p.NTW == 4) FFMI_RUN(4, 4);
      if (p.NTW == 6) FFMI_RUN(4, 6);
      FFMI_RUN(4, 8);  // (12 / 16 tiles: 4 x 16 accumulators exceed the register budget)
    }
    if (p.MTW == 3) {
      if (p.NTW == 2) FFMI_RUN(3, 2);
      if (p.NTW == 4) FFMI_RUN(3, 4);
      if (p.NTW == 16) FFMI_RUN(3, 16);
      if (p.NTW == 12) FFMI_RUN(3, 12);
      if (p.NTW == 6) FFMI_RUN(3, 6);
      FFMI_RUN(3, 8);
    }
    if (p.NTW == 2) FFMI_RUN(2, 2);
    if (p.NTW == 4) FFMI_RUN(2, 4);
    if (p.NTW == 16) FFMI_RUN(2, 16);
    if (p.NTW == 12) FFMI_RUN(2, 12);
    if (p.NTW == 6) FFMI_RUN(2, 6);
    FFMI_RUN(2, 8);
#undef FFMI_RUN
  }
  const int xi = xp ? 1 : 0;
  int S = skinny_split(T, N, K, epilogue, defer != nullptr);
  const size_t need = (size_t)S * T * ((N + 15) / 16) * 16 * sizeof(float);
  if (S > 1 && (!ws || ws_bytes < need)) S = 1;
  hipError_t e;
  if (mtiles <= 1) e = dispatch_nt<1, 8>(X, Wp, Y, ws, T, N, K, KT, epilogue, S, s, xi, yp, nt, wpitch);
  else if (mtiles <= 2) e = dispatch_nt<2, 8>(X, Wp, Y, ws, T, N, K, KT, epilogue, S, s, xi, yp, nt, wpitch);
  else e = dispatch_nt<4, 4>(X, Wp, Y, ws, T, N, K, KT, epilogue, S, s, xi, yp, nt, wpitch);
  if (S > 1 && e == hipSuccess) defer->p = ws, defer->S = S, defer->NP = (N + 15) / 16 * 16;
  return e;
}

// Packed activation tiles: Xp[mt][kt][lane][8] = X[mt*16 + (lane&15)][kt*32 + 8(lane>>4) + e]
// (rows >= T zero) -- the MFMA operand fragment order of the weights (weights.hip),
// so a GEMM reads each activation fragment as one contiguous 1 KiB.
__global__ void pack_act_kernel(const uint16_t *__restrict__ X, uint16_t *__restrict__ Xp, int T,
                                int K, int KT) {
  const int mt = blockIdx.y, kt = blockIdx.x, l = threadIdx.x;
  const int r = mt * 16 + (l & 15);
  uint4 v = make_uint4(0, 0, 0, 0);
  if (r < T) v = *reinterpret_cast<const uint4 *>(X + (size_t)r * K + kt * 32 + 8 * (l >> 4));
  *reinterpret_cast<uint4 *>(Xp + (((size_t)mt * KT + kt) * 64 + l) * 8) = v;
}

size_t packed_act_bytes(int T, int K) { return (size_t)((T + 15) / 16) * 16 * K * 2; }

hipError_t launch_pack_act(const uint16_t *X, uint16_t *Xp, int T, int K, hipStream_t s) {
  if (T <= 0) return hipSuccess;
  hipLaunchKernelGGL(pack_act_kernel, dim3(K / 32, (T + 15) / 16), dim3(64), 0, s, X, Xp, T, K,
                     K / 32);
  return hipGetLastError();
}

// diagnostics: stamps of the last FFMI_GEMM_STAMP launch (8 int64 per wave)
long gemm_debug_stamps(long long *dst, long max_waves) {
  long long *buf = stamp_buf();
  const long n = g_stamp_entries < max_waves ? g_stamp_entries : max_waves;
  if (!buf || n <= 0) return 0;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpy(dst, buf, (size_t)n * 8 * sizeof(long long), hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  return n;
}

}  // namespace ffmi
