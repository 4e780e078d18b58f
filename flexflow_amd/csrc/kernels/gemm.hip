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
#include <stdlib.h>
#include <string.h>

#include <algorithm>

#include "../ffmi_internal.h"

namespace ffmi {

// SigmoidSiluMultiKernel numerics (sigmoid_silu_multi.cu:41-46): gate and up
// are fp16 values, out = half(half(g * half(sigmoid(g))) * u)
__device__ __forceinline__ uint16_t silu_mul_h(float gacc, float uacc) {
  const float g = __half2float(__float2half_rn(gacc));
  const float u = __half2float(__float2half_rn(uacc));
  const float sg = __half2float(__float2half_rn(1.0f / (1.0f + expf(-g))));
  const float t = __half2float(__float2half_rn(g * sg));
  return __half_as_ushort(__float2half_rn(t * u));
}

// MULTI = 1: multi-pass over row blocks of MT*16 rows.  The grid is 1-D and
// XCD-grouped: the row blocks of one column block get linear ids 8 apart
// (ids are dealt round-robin over the 8 XCDs), so they run together on ONE
// XCD and the weight tile crosses HBM once and is re-read from that XCD's
// L2 by the sibling row blocks (MI355X_MICROARCH.md ring-vs-splitk: "tiles
// with the rows split").
template <int MT, int NT, int KW, int U, int EPI, int MULTI>
__global__ __launch_bounds__(KW * 64) void gemm_skinny_kernel(
    const uint16_t *__restrict__ X, const uint16_t *__restrict__ Wp,
    uint16_t *__restrict__ Y, int T, int N, int K, int KT, int NTILES, int mpasses) {
  extern __shared__ __attribute__((aligned(16))) float red[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  int cb = blockIdx.x, mb = 0;
  if (MULTI) {
    const int grp = 8 * mpasses;
    const int r = blockIdx.x % grp;
    cb = (blockIdx.x / grp) * 8 + (r & 7);
    mb = r >> 3;
    if (cb * NT >= NTILES) return;
  }
  const int tile0 = cb * NT;
  const int m0 = mb * (MT * 16);
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
    int n = cb * 16 + (lane & 15);
    if (n < N) {
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          int m = m0 + i * 16 + (lane >> 4) * 4 + r;
          if (m >= T) continue;
          Y[(size_t)m * N + n] = silu_mul_h(acc[i][0][r], acc[i][1][r]);
        }
    }
  }
}

template <int MT, int NT, int KW, int U, int EPI, int MULTI>
static hipError_t run(const uint16_t *X, const uint16_t *Wp, uint16_t *Y, int T, int N,
                      int K, int KT, int NTILES, int mpasses, hipStream_t s) {
  const int ncb = (NTILES + NT - 1) / NT;
  dim3 grid(MULTI ? (ncb + 7) / 8 * 8 * mpasses : ncb);
  size_t lds = KW > 1 ? (size_t)(KW - 1) * MT * NT * 4 * 64 * sizeof(float) : 0;
  hipLaunchKernelGGL((gemm_skinny_kernel<MT, NT, KW, U, EPI, MULTI>), grid, dim3(KW * 64), lds,
                     s, X, Wp, Y, T, N, K, KT, NTILES, MULTI ? mpasses : 1);
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
template <int MTW, int NTW, int EPI>
__global__ __launch_bounds__(256) void gemm_mid_kernel(
    const uint16_t *__restrict__ X, const uint16_t *__restrict__ Wp,
    uint16_t *__restrict__ Y, float *__restrict__ Ypart, int T, int N, int K, int KT,
    int NTILES, int S) {
  static_assert(NTW % 4 == 0, "NTW pieces are spread over 4 waves");
  constexpr int PPT = NTW / 4;
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
    const int t = min(tile0 + bj[p], NTILES - 1);
    bsrc[p] = Wp + (size_t)t * KT * 512 + lane * 8;
  }
  const uint16_t *xrow[MTW];
#pragma unroll
  for (int i = 0; i < MTW; ++i) {
    const int r = min(m0 + i * 16 + (lane & 15), T - 1);
    xrow[i] = X + (size_t)r * K + 8 * (lane >> 4);
  }
  f4 acc[MTW][NTW];
#pragma unroll
  for (int i = 0; i < MTW; ++i)
#pragma unroll
    for (int j = 0; j < NTW; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  // Software pipeline (per k-step: one barrier, weight tile double-buffered
  // in LDS).  Weight loads run PF=3 k-steps ahead in a register ring, X
  // fragments one step ahead; X(k+1) is issued BEFORE B(k+3) so that the
  // in-order vmcnt wait for X(k+1) never forces the younger weight loads.
  if (kb < ke) {
    constexpr int PF = 3;
    h8 bq[PF][PPT];
    h8 a[MTW], an[MTW];
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      const int kq = min(kb + q, ke - 1);
#pragma unroll
      for (int p = 0; p < PPT; ++p)
        bq[q][p] = *reinterpret_cast<const h8 *>(bsrc[p] + (size_t)kq * 512);
    }
#pragma unroll
    for (int i = 0; i < MTW; ++i) a[i] = *reinterpret_cast<const h8 *>(xrow[i] + kb * 32);
#pragma unroll
    for (int p = 0; p < PPT; ++p) sB[0][bj[p]][lane] = bq[0][p];
    __syncthreads();
    int cur = 0;
    for (int kt0 = kb; kt0 < ke; kt0 += PF) {
#pragma unroll
      for (int q = 0; q < PF; ++q) {
        const int kt = kt0 + q;
        if (kt >= ke) break;
        const int kx = min(kt + 1, ke - 1);
#pragma unroll
        for (int i = 0; i < MTW; ++i) an[i] = *reinterpret_cast<const h8 *>(xrow[i] + kx * 32);
        // slot q held B(kt); it is free once B(kt) went to LDS (previous step)
        const int kw = min(kt + PF, ke - 1);
        h8 b[NTW];
#pragma unroll
        for (int j = 0; j < NTW; ++j) b[j] = sB[cur][j][lane];
#pragma unroll
        for (int p = 0; p < PPT; ++p)
          bq[q][p] = *reinterpret_cast<const h8 *>(bsrc[p] + (size_t)kw * 512);
#pragma unroll
        for (int i = 0; i < MTW; ++i)
#pragma unroll
          for (int j = 0; j < NTW; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[i], b[j], acc[i][j], 0, 0, 0);
        // B(kt+1) lives in ring slot (q+1) % PF
#pragma unroll
        for (int p = 0; p < PPT; ++p) sB[cur ^ 1][bj[p]][lane] = bq[(q + 1) % PF][p];
        __syncthreads();
#pragma unroll
        for (int i = 0; i < MTW; ++i) a[i] = an[i];
        cur ^= 1;
      }
    }
  }

  // C/D layout: col = lane&15, row = (lane>>4)*4 + r
  if (S > 1) {
    const int NP = NTILES * 16;
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      const int tile = tile0 + j;
      if (tile >= NTILES) continue;
#pragma unroll
      for (int i = 0; i < MTW; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + i * 16 + (lane >> 4) * 4 + r;
          if (m < T) Ypart[((size_t)ks * T + m) * NP + tile * 16 + (lane & 15)] = acc[i][j][r];
        }
    }
    return;
  }
  if (EPI == 0) {
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      const int n = (tile0 + j) * 16 + (lane & 15);
      if (tile0 + j >= NTILES || n >= N) continue;
#pragma unroll
      for (int i = 0; i < MTW; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + i * 16 + (lane >> 4) * 4 + r;
          if (m < T) Y[(size_t)m * N + n] = __half_as_ushort(__float2half_rn(acc[i][j][r]));
        }
    }
  } else {
#pragma unroll
    for (int j = 0; j < NTW; j += 2) {
      const int n = ((tile0 + j) >> 1) * 16 + (lane & 15);
      if (tile0 + j >= NTILES || n >= N) continue;
#pragma unroll
      for (int i = 0; i < MTW; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + i * 16 + (lane >> 4) * 4 + r;
          if (m < T) Y[(size_t)m * N + n] = silu_mul_h(acc[i][j][r], acc[i][j + 1][r]);
        }
    }
  }
}

// ---------------------------------------------------------------------------
// LDS-DMA variant of the M-split kernel (the verify/prefill-chunk regime).
// Both operands travel HBM/L2 -> LDS by global_load_lds_dwordx4 (no VGPR
// staging), through an NST-deep ring of stages.  One stage = one 32-deep
// k-step: the 4 waves' own A fragments (4*MTW x 1 KiB, each wave loads its
// MTW) + the NTW shared weight fragments (NTW/4 per wave).  The packed
// weight fragment is already lane-linear (weights.hip), and an X fragment
// is lane-linear by construction (lane l: row l&15, k 8(l>>4)..+7), so the
// LDS image is read back with conflict-free ds_read_b128.  Waits are counted
// (vmcnt = loads of the stages still allowed in flight) and the barrier is a
// raw s_barrier, so NST-2 stages stay in flight across every barrier
// (cdna_hip_programming.md §5 "Pipelining across barriers").
// Same per-element reduction order as gemm_mid_kernel: MFMA chain over the
// slice's k-steps, then slices in order.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void glds16(const void *gsrc, uint32_t lds_dst) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_dst)
      : "memory");
}
template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}
// wait until at most G*ahead of this wave's DMA loads are outstanding
template <int G, int A>
__device__ __forceinline__ void vm_wait_stages(int ahead) {
  if constexpr (A == 0) {
    vm_wait<0>();
  } else {
    if (ahead >= A) vm_wait<G * A>();
    else vm_wait_stages<G, A - 1>(ahead);
  }
}

template <int MTW, int NTW, int EPI>
__device__ __forceinline__ void mid_store(const f4 (&acc)[MTW][NTW], uint16_t *__restrict__ Y,
                                          float *__restrict__ Ypart, int T, int N, int NTILES,
                                          int S, int ks, int tile0, int m0, int lane) {
  // C/D layout: col = lane&15, row = (lane>>4)*4 + r
  if (S > 1) {
    const int NP = NTILES * 16;
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      const int tile = tile0 + j;
      if (tile >= NTILES) continue;
#pragma unroll
      for (int i = 0; i < MTW; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + i * 16 + (lane >> 4) * 4 + r;
          if (m < T) Ypart[((size_t)ks * T + m) * NP + tile * 16 + (lane & 15)] = acc[i][j][r];
        }
    }
    return;
  }
  if (EPI == 0) {
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      const int n = (tile0 + j) * 16 + (lane & 15);
      if (tile0 + j >= NTILES || n >= N) continue;
#pragma unroll
      for (int i = 0; i < MTW; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + i * 16 + (lane >> 4) * 4 + r;
          if (m < T) Y[(size_t)m * N + n] = __half_as_ushort(__float2half_rn(acc[i][j][r]));
        }
    }
  } else {
#pragma unroll
    for (int j = 0; j < NTW; j += 2) {
      const int n = ((tile0 + j) >> 1) * 16 + (lane & 15);
      if (tile0 + j >= NTILES || n >= N) continue;
#pragma unroll
      for (int i = 0; i < MTW; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + i * 16 + (lane >> 4) * 4 + r;
          if (m < T) Y[(size_t)m * N + n] = silu_mul_h(acc[i][j][r], acc[i][j + 1][r]);
        }
    }
  }
}

template <int MTW, int NTW, int NST, int EPI>
__global__ __launch_bounds__(256, 1) void gemm_glds_kernel(
    const uint16_t *__restrict__ X, const uint16_t *__restrict__ Wp,
    uint16_t *__restrict__ Y, float *__restrict__ Ypart, int T, int N, int K, int KT,
    int NTILES, int S) {
  static_assert(NTW % 4 == 0, "NTW pieces are spread over 4 waves");
  constexpr int PPT = NTW / 4;
  constexpr int G = MTW + PPT;                   // DMA loads per wave per stage
  constexpr int STAGE = (4 * MTW + NTW) * 1024;  // bytes per stage
  static_assert(G * (NST - 2) <= 63, "vmcnt range");
  __shared__ __attribute__((aligned(1024))) char lds[NST * STAGE];
  const uint32_t lbase = (uint32_t)(uintptr_t)lds;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tile0 = blockIdx.x * NTW;
  const int ks = blockIdx.y;
  const int m0 = blockIdx.z * (4 * MTW * 16) + wave * MTW * 16;
  const int per = (KT + S - 1) / S;
  const int kb = min(KT, ks * per);
  const int ke = min(KT, kb + per);
  const int nk = ke - kb;

  const uint16_t *bsrc[PPT];
#pragma unroll
  for (int p = 0; p < PPT; ++p) {
    const int t = min(tile0 + wave + 4 * p, NTILES - 1);
    bsrc[p] = Wp + ((size_t)t * KT + kb) * 512 + lane * 8;
  }
  const uint16_t *xsrc[MTW];
#pragma unroll
  for (int i = 0; i < MTW; ++i) {
    const int r = min(m0 + i * 16 + (lane & 15), T - 1);
    xsrc[i] = X + (size_t)r * K + kb * 32 + 8 * (lane >> 4);
  }
  // LDS addresses: stage s at s*STAGE; A of wave w at (w*MTW+i) KiB, B tile j at (4*MTW+j) KiB
  const uint32_t a_dst = lbase + (uint32_t)(wave * MTW) * 1024u;
  const uint32_t b_dst = lbase + (uint32_t)(4 * MTW + wave) * 1024u;
  auto issue = [&](int st) {  // stage index st (relative to kb) -> ring slot st % NST
    const uint32_t so = (uint32_t)(st % NST) * STAGE;
#pragma unroll
    for (int i = 0; i < MTW; ++i) glds16(xsrc[i] + st * 32, a_dst + so + i * 1024u);
#pragma unroll
    for (int p = 0; p < PPT; ++p) glds16(bsrc[p] + (size_t)st * 512, b_dst + so + p * 4096u);
  };

  f4 acc[MTW][NTW];
#pragma unroll
  for (int i = 0; i < MTW; ++i)
#pragma unroll
    for (int j = 0; j < NTW; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int st = 0; st < NST - 1; ++st)
    if (st < nk) issue(st);
  // (waves whose rows are all past T still run the MFMAs on clamped rows: a
  // skip would put the accumulators through a phi and off the AGPRs)
  for (int k = 0; k < nk; ++k) {
    // stage k must have landed (this wave), then everyone's (barrier); the
    // barrier also retires every wave's reads of stage k-1, whose slot the
    // next issue overwrites
    vm_wait_stages<G, NST - 2>(min(NST - 2, nk - 1 - k));
    asm volatile("s_barrier" ::: "memory");
    if (k + NST - 1 < nk) issue(k + NST - 1);
    const char *sp = lds + (size_t)(k % NST) * STAGE;
    h8 a[MTW], b[NTW];
#pragma unroll
    for (int i = 0; i < MTW; ++i)
      a[i] = *reinterpret_cast<const h8 *>(sp + (wave * MTW + i) * 1024 + lane * 16);
#pragma unroll
    for (int j = 0; j < NTW; ++j)
      b[j] = *reinterpret_cast<const h8 *>(sp + (4 * MTW + j) * 1024 + lane * 16);
#pragma unroll
    for (int i = 0; i < MTW; ++i)
#pragma unroll
      for (int j = 0; j < NTW; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[i], b[j], acc[i][j], 0, 0, 0);
  }
  mid_store<MTW, NTW, EPI>(acc, Y, Ypart, T, N, NTILES, S, ks, tile0, m0, lane);
}

// Sum the S fp32 partial slabs in slice order, then the epilogue.
template <int EPI>
__global__ void gemm_reduce_kernel(const float *__restrict__ Ypart, uint16_t *__restrict__ Y,
                                   int T, int N, int NTILES, int S) {
  const int NP = NTILES * 16;
  const long idx = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (idx >= (long)T * N) return;
  const int m = (int)(idx / N), n = (int)(idx % N);
  if (EPI == 0) {
    float acc = Ypart[(size_t)m * NP + n];
    for (int s = 1; s < S; ++s) acc += Ypart[((size_t)s * T + m) * NP + n];
    Y[idx] = __half_as_ushort(__float2half_rn(acc));
  } else {
    const int gcol = (n >> 4) * 32 + (n & 15);
    float g = Ypart[(size_t)m * NP + gcol], u = Ypart[(size_t)m * NP + gcol + 16];
    for (int s = 1; s < S; ++s) {
      g += Ypart[((size_t)s * T + m) * NP + gcol];
      u += Ypart[((size_t)s * T + m) * NP + gcol + 16];
    }
    Y[idx] = silu_mul_h(g, u);
  }
}

static int mid_split(int KT, int blocks) {
  int S = (256 + blocks - 1) / blocks;
  S = S < 1 ? 1 : (S > 8 ? 8 : S);
  return S > KT ? KT : S;
}

static int glds_split(int KT, int blocks);

size_t gemm_workspace_bytes(int T, int N, int K, int epilogue) {
  const int mtiles = (T + 15) / 16;
  if (mtiles <= 4) return 0;
  const int ntiles = (N + 15) / 16 * (epilogue ? 2 : 1);
  const int MTW = mtiles <= 8 ? 2 : 3;
  const int mblocks = (mtiles + 4 * MTW - 1) / (4 * MTW);
  const int nblk = (ntiles + 7) / 8;
  const int S = std::max(mid_split(K / 32, nblk * mblocks), glds_split(K / 32, nblk * mblocks));
  return S > 1 ? (size_t)S * T * ntiles * 16 * sizeof(float) : 0;
}

// k-split for the one-workgroup-per-CU DMA kernel: whole waves of 256
// workgroups, ~8 k-steps of pipeline fill per workgroup.
static int glds_split(int KT, int blocks) {
  static const int force = getenv("FFMI_GEMM_S") ? atoi(getenv("FFMI_GEMM_S")) : 0;
  if (force > 0) return force > KT ? KT : force;
  int best = 1;
  long bestc = -1;
  for (int S = 1; S <= 8 && S <= KT; ++S) {
    const long rounds = (blocks * (long)S + 255) / 256;
    const long c = rounds * ((KT + S - 1) / S + 8) + (S > 1 ? 4 : 0);
    if (bestc < 0 || c < bestc) best = S, bestc = c;
  }
  return best;
}

static bool use_glds() {
  static const bool v = getenv("FFMI_GEMM_IMPL") && !strcmp(getenv("FFMI_GEMM_IMPL"), "glds");
  return v;
}

template <int MTW, int NST>
static hipError_t run_glds(const uint16_t *X, const uint16_t *Wp, uint16_t *Y, float *ws,
                           size_t ws_bytes, int T, int N, int K, int epi, hipStream_t s) {
  constexpr int NTW = 8;
  const int KT = K / 32;
  const int ntiles = (N + 15) / 16 * (epi ? 2 : 1);
  const int mtiles = (T + 15) / 16;
  const int mblocks = (mtiles + 4 * MTW - 1) / (4 * MTW);
  const int nblk = (ntiles + NTW - 1) / NTW;
  int S = glds_split(KT, nblk * mblocks);
  const size_t need = (size_t)S * T * ntiles * 16 * sizeof(float);
  if (S > 1 && (!ws || ws_bytes < need)) S = 1;
  dim3 grid(nblk, S, mblocks);
  if (epi)
    hipLaunchKernelGGL((gemm_glds_kernel<MTW, NTW, NST, 1>), grid, dim3(256), 0, s, X, Wp, Y, ws,
                       T, N, K, KT, ntiles, S);
  else
    hipLaunchKernelGGL((gemm_glds_kernel<MTW, NTW, NST, 0>), grid, dim3(256), 0, s, X, Wp, Y, ws,
                       T, N, K, KT, ntiles, S);
  if (S > 1) {
    const long total = (long)T * N;
    const unsigned blocks = (unsigned)((total + 255) / 256);
    if (epi)
      hipLaunchKernelGGL(gemm_reduce_kernel<1>, dim3(blocks), dim3(256), 0, s, ws, Y, T, N,
                         ntiles, S);
    else
      hipLaunchKernelGGL(gemm_reduce_kernel<0>, dim3(blocks), dim3(256), 0, s, ws, Y, T, N,
                         ntiles, S);
  }
  return hipGetLastError();
}

template <int MTW>
static hipError_t run_mid(const uint16_t *X, const uint16_t *Wp, uint16_t *Y, float *ws,
                          size_t ws_bytes, int T, int N, int K, int epi, hipStream_t s) {
  constexpr int NTW = 8;
  const int KT = K / 32;
  const int ntiles = (N + 15) / 16 * (epi ? 2 : 1);
  const int mtiles = (T + 15) / 16;
  const int mblocks = (mtiles + 4 * MTW - 1) / (4 * MTW);
  const int nblk = (ntiles + NTW - 1) / NTW;
  int S = mid_split(KT, nblk * mblocks);
  const size_t need = (size_t)S * T * ntiles * 16 * sizeof(float);
  if (S > 1 && (!ws || ws_bytes < need)) S = 1;  // no workspace: un-split (slower)
  dim3 grid(nblk, S, mblocks);
  if (epi)
    hipLaunchKernelGGL((gemm_mid_kernel<MTW, NTW, 1>), grid, dim3(256), 0, s, X, Wp, Y, ws, T, N,
                       K, KT, ntiles, S);
  else
    hipLaunchKernelGGL((gemm_mid_kernel<MTW, NTW, 0>), grid, dim3(256), 0, s, X, Wp, Y, ws, T, N,
                       K, KT, ntiles, S);
  if (S > 1) {
    const long total = (long)T * N;
    const unsigned blocks = (unsigned)((total + 255) / 256);
    if (epi)
      hipLaunchKernelGGL(gemm_reduce_kernel<1>, dim3(blocks), dim3(256), 0, s, ws, Y, T, N,
                         ntiles, S);
    else
      hipLaunchKernelGGL(gemm_reduce_kernel<0>, dim3(blocks), dim3(256), 0, s, ws, Y, T, N,
                         ntiles, S);
  }
  return hipGetLastError();
}

hipError_t launch_gemm(const uint16_t *X, const uint16_t *Wp, uint16_t *Y, float *ws,
                       size_t ws_bytes, int T, int N, int K, int epilogue, hipStream_t s) {
  if (T <= 0) return hipSuccess;
  const int KT = K / 32;
  const int mtiles = (T + 15) / 16;
  static const int mid_impl = [] {
    const char *e = getenv("FFMI_GEMM_IMPL");
    if (!e) return 0;
    if (!strcmp(e, "skinny4")) return 4;
    if (!strcmp(e, "skinny8")) return 8;
    if (!strcmp(e, "skinny2")) return 2;
    return 0;
  }();
  if (mtiles > 4 && mid_impl == 4)
    return dispatch_nt<4, 4, 1>(X, Wp, Y, T, N, K, KT, epilogue, (mtiles + 3) / 4, s);
  if (mtiles > 4 && mid_impl == 8)
    return dispatch_nt<8, 2, 1>(X, Wp, Y, T, N, K, KT, epilogue, (mtiles + 7) / 8, s);
  if (mtiles > 2 && mid_impl == 2)
    return dispatch_nt<2, 8, 1>(X, Wp, Y, T, N, K, KT, epilogue, (mtiles + 1) / 2, s);
  if (mtiles > 4 && use_glds()) {
    if (mtiles > 8) return run_glds<3, 6>(X, Wp, Y, ws, ws_bytes, T, N, K, epilogue, s);
    return run_glds<2, 7>(X, Wp, Y, ws, ws_bytes, T, N, K, epilogue, s);
  }
  if (mtiles > 8) return run_mid<3>(X, Wp, Y, ws, ws_bytes, T, N, K, epilogue, s);
  if (mtiles > 4) return run_mid<2>(X, Wp, Y, ws, ws_bytes, T, N, K, epilogue, s);
  if (mtiles <= 1) return dispatch_nt<1, 8, 0>(X, Wp, Y, T, N, K, KT, epilogue, 1, s);
  if (mtiles <= 2) return dispatch_nt<2, 8, 0>(X, Wp, Y, T, N, K, KT, epilogue, 1, s);
  if (mtiles <= 4) return dispatch_nt<4, 4, 0>(X, Wp, Y, T, N, K, KT, epilogue, 1, s);
  if (mtiles <= 8) return dispatch_nt<8, 2, 0>(X, Wp, Y, T, N, K, KT, epilogue, 1, s);
  if (mtiles <= 12) return dispatch_nt<12, 2, 0>(X, Wp, Y, T, N, K, KT, epilogue, 1, s);
  return dispatch_nt<12, 2, 1>(X, Wp, Y, T, N, K, KT, epilogue, (mtiles + 11) / 12, s);
}

}  // namespace ffmi
