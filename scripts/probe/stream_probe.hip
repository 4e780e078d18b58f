// Where does the M-split GEMM's k-step time go?  The gemm_mid_kernel loop
// with its parts switched on one by one (MODE bits: 1 = activation loads,
// 2 = weight tile staged through LDS + barrier, 4 = MFMAs), on the gate_up
// shape (K 4096, 1380 weight tiles, 168 rows), weights rotated over copies
// larger than the Infinity Cache.  KG = 2 puts a second group of 4 waves on
// the other half of K inside the workgroup (8 waves, LDS reduction).
//   hipcc --offload-arch=gfx950 -O3 -o stream_probe stream_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <type_traits>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

template <int I, int N, class F>
__device__ __forceinline__ void sfor_impl(F &&f) {
  if constexpr (I < N) { f(std::integral_constant<int, I>{}); sfor_impl<I + 1, N>(f); }
}
template <int N, class F>
__device__ __forceinline__ void sfor(F &&f) { sfor_impl<0, N>(f); }

template <int MTW, int NTW, int PF, int MODE, int KG>
__global__ __launch_bounds__(256 * KG, 1) void probe(const uint16_t *__restrict__ X,
                                                     const uint16_t *__restrict__ Wp,
                                                     float *__restrict__ out, int T, int KT,
                                                     int NTILES) {
  constexpr int PPT = (NTW + 3) / 4;
  __shared__ __attribute__((aligned(16))) h8 sB[KG][2][NTW][64];
  const int lane = threadIdx.x & 63;
  const int wave = (threadIdx.x >> 6) & 3;
  const int kg = threadIdx.x >> 8;
  const int tile0 = blockIdx.x * NTW;
  const int m0 = wave * MTW * 16;
  const int per = KT / KG;
  const int kb = kg * per, ke = kb + per;
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
    const int mt = min((m0 + i * 16) >> 4, (T - 1) >> 4);
    xrow[i] = X + ((size_t)mt * KT * 64 + lane) * 8;
  }
  f4 acc[MTW][NTW];
#pragma unroll
  for (int i = 0; i < MTW; ++i)
#pragma unroll
    for (int j = 0; j < NTW; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  h8 bq[PF][PPT];
  h8 xq[PF][MTW];
#pragma unroll
  for (int q = 0; q < PF; ++q) {
    const int kq = kb + q;
    if (MODE & 1)
#pragma unroll
      for (int i = 0; i < MTW; ++i) xq[q][i] = *reinterpret_cast<const h8 *>(xrow[i] + (size_t)kq * 512);
#pragma unroll
    for (int p = 0; p < PPT; ++p)
      if ((NTW % 4 == 0 || bj[p] < NTW) && !(MODE & 8)) bq[q][p] = *reinterpret_cast<const h8 *>(bsrc[p] + (size_t)kq * 512);
      else bq[q][p] = h8{};
  }
  if (!(MODE & 1))
#pragma unroll
    for (int q = 0; q < PF; ++q)
#pragma unroll
      for (int i = 0; i < MTW; ++i) xq[q][i] = bq[q][0];
  if (MODE & 2) {
#pragma unroll
    for (int p = 0; p < PPT; ++p)
      if (NTW % 4 == 0 || bj[p] < NTW) sB[kg][0][bj[p]][lane] = bq[0][p];
    __syncthreads();
  }
  int cur = 0;
  auto step = [&](auto Qc, int kt) {
    constexpr int Q = decltype(Qc)::value;
    h8 b[NTW];
    if (MODE & 2) {
#pragma unroll
      for (int j = 0; j < NTW; ++j) b[j] = sB[kg][cur][j][lane];
    } else {
#pragma unroll
      for (int j = 0; j < NTW; ++j) b[j] = bq[Q][j % PPT];
    }
    if (MODE & 4) {
#pragma unroll
      for (int i = 0; i < MTW; ++i)
#pragma unroll
        for (int j = 0; j < NTW; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(b[j], xq[Q][i], acc[i][j], 0, 0, 0);
    } else {
#pragma unroll
      for (int i = 0; i < MTW; ++i)
#pragma unroll
        for (int j = 0; j < NTW; ++j) acc[i][j][0] += (float)b[j][0] * (float)xq[Q][i][1];
    }
    const int kw = min(kt + PF, ke - 1);
    if (MODE & 1)
#pragma unroll
      for (int i = 0; i < MTW; ++i) xq[Q][i] = *reinterpret_cast<const h8 *>(xrow[i] + (size_t)kw * 512);
#pragma unroll
    for (int p = 0; p < PPT; ++p)
      if ((NTW % 4 == 0 || bj[p] < NTW) && !(MODE & 8)) bq[Q][p] = *reinterpret_cast<const h8 *>(bsrc[p] + (size_t)kw * 512);
    if (!(MODE & 1))
#pragma unroll
      for (int i = 0; i < MTW; ++i) xq[Q][i] = bq[Q][0];
    if (MODE & 2) {
#pragma unroll
      for (int p = 0; p < PPT; ++p)
        if (NTW % 4 == 0 || bj[p] < NTW) sB[kg][cur ^ 1][bj[p]][lane] = bq[(Q + 1) % PF][p];
      __syncthreads();
      cur ^= 1;
    }
  };
  int kt0 = kb;
  for (; kt0 + PF <= ke; kt0 += PF) sfor<PF>([&](auto Qc) { step(Qc, kt0 + decltype(Qc)::value); });
  float s = 0;
#pragma unroll
  for (int i = 0; i < MTW; ++i)
#pragma unroll
    for (int j = 0; j < NTW; ++j) s += acc[i][j][0] + acc[i][j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int MTW, int NTW, int PF, int MODE, int KG>
static void run(const char *tag, const uint16_t *X, uint16_t *W, size_t copy_halves, int copies,
                float *out, int T, int KT) {
  const int ntiles = 1380 / NTW * NTW;
  const int wgs = ntiles / NTW;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < copies; ++i)
    probe<MTW, NTW, PF, MODE, KG><<<wgs, 256 * KG>>>(X, W + i * copy_halves, out, T, KT, ntiles);
  const int iters = 3 * copies;
  hipEventRecord(a);
  for (int i = 0; i < iters; ++i)
    probe<MTW, NTW, PF, MODE, KG><<<wgs, 256 * KG>>>(X, W + (i % copies) * copy_halves, out, T, KT,
                                                     ntiles);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  const double us = ms * 1000.0 / iters;
  const double wbytes = (MODE & 8) ? 0.0 : (double)ntiles * KT * 1024;
  const double xbytes = (MODE & 1) ? (double)wgs * KG * 4 * MTW * (KT / KG) * 1024 : 0.0;
  printf("MTW %d NTW %2d PF %d KG %d mode %2d: %7.2f us  %6.0f GB/s weights  %5.1f GB/s/CU in (W+X)  (%d WGs)\n",
         MTW, NTW, PF, KG, MODE, us, wbytes / us / 1e3, (wbytes + xbytes) / us / 1e3 / wgs, wgs);
}


// Role split: waves 0-3 compute (own rows of X straight from L2 into
// registers, weight tiles from LDS, MFMA); waves 4-7 only stream the weight
// tiles (HBM -> registers -> LDS slot).  Separate waves keep the short-latency
// activation loads out of the weight stream's in-order vmcnt queue.
template <int MTW, int NTW, int PF, int XPF>
__global__ __launch_bounds__(512, 1) void probe_split(const uint16_t *__restrict__ X,
                                                      const uint16_t *__restrict__ Wp,
                                                      float *__restrict__ out, int T, int KT,
                                                      int NTILES) {
  constexpr int PPT = (NTW + 3) / 4;
  __shared__ __attribute__((aligned(16))) h8 sB[2][NTW][64];
  const int lane = threadIdx.x & 63;
  const int wave = (threadIdx.x >> 6) & 3;
  const bool loader = threadIdx.x >= 256;
  const int tile0 = blockIdx.x * NTW;
  const int kb = 0, ke = KT;
  f4 acc[MTW][NTW];
#pragma unroll
  for (int i = 0; i < MTW; ++i)
#pragma unroll
    for (int j = 0; j < NTW; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  if (loader) {
    const uint16_t *bsrc[PPT];
    int bj[PPT];
#pragma unroll
    for (int p = 0; p < PPT; ++p) {
      bj[p] = wave + 4 * p;
      const int t = min(tile0 + bj[p], NTILES - 1);
      bsrc[p] = Wp + (size_t)t * KT * 512 + lane * 8;
    }
    h8 bq[PF][PPT];
#pragma unroll
    for (int q = 0; q < PF; ++q)
#pragma unroll
      for (int p = 0; p < PPT; ++p)
        if (NTW % 4 == 0 || bj[p] < NTW) bq[q][p] = *reinterpret_cast<const h8 *>(bsrc[p] + (size_t)(kb + q) * 512);
#pragma unroll
    for (int p = 0; p < PPT; ++p)
      if (NTW % 4 == 0 || bj[p] < NTW) sB[0][bj[p]][lane] = bq[0][p];
    __syncthreads();
    int cur = 0;
    auto step = [&](auto Qc, int kt) {
      constexpr int Q = decltype(Qc)::value;
      const int kw = min(kt + PF, ke - 1);
#pragma unroll
      for (int p = 0; p < PPT; ++p)
        if (NTW % 4 == 0 || bj[p] < NTW) bq[Q][p] = *reinterpret_cast<const h8 *>(bsrc[p] + (size_t)kw * 512);
#pragma unroll
      for (int p = 0; p < PPT; ++p)
        if (NTW % 4 == 0 || bj[p] < NTW) sB[cur ^ 1][bj[p]][lane] = bq[(Q + 1) % PF][p];
      __syncthreads();
      cur ^= 1;
    };
    int kt0 = kb;
    for (; kt0 + PF <= ke; kt0 += PF) sfor<PF>([&](auto Qc) { step(Qc, kt0 + decltype(Qc)::value); });
    return;
  }
  const int m0 = wave * MTW * 16;
  const uint16_t *xrow[MTW];
#pragma unroll
  for (int i = 0; i < MTW; ++i) {
    const int mt = min((m0 + i * 16) >> 4, (T - 1) >> 4);
    xrow[i] = X + ((size_t)mt * KT * 64 + lane) * 8;
  }
  h8 xq[XPF][MTW];
#pragma unroll
  for (int q = 0; q < XPF; ++q)
#pragma unroll
    for (int i = 0; i < MTW; ++i) xq[q][i] = *reinterpret_cast<const h8 *>(xrow[i] + (size_t)(kb + q) * 512);
  __syncthreads();
  int cur = 0;
  auto cstep = [&](auto Qc, int kt) {
    constexpr int Q = decltype(Qc)::value;
    h8 b[NTW];
#pragma unroll
    for (int j = 0; j < NTW; ++j) b[j] = sB[cur][j][lane];
#pragma unroll
    for (int i = 0; i < MTW; ++i)
#pragma unroll
      for (int j = 0; j < NTW; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(b[j], xq[Q][i], acc[i][j], 0, 0, 0);
    const int kw = min(kt + XPF, ke - 1);
#pragma unroll
    for (int i = 0; i < MTW; ++i) xq[Q][i] = *reinterpret_cast<const h8 *>(xrow[i] + (size_t)kw * 512);
    __syncthreads();
    cur ^= 1;
  };
  static_assert(PF % XPF == 0, "same trip count");
  int kt0 = kb;
  for (; kt0 + XPF <= ke; kt0 += XPF) sfor<XPF>([&](auto Qc) { cstep(Qc, kt0 + decltype(Qc)::value); });
  float s = 0;
#pragma unroll
  for (int i = 0; i < MTW; ++i)
#pragma unroll
    for (int j = 0; j < NTW; ++j) s += acc[i][j][0] + acc[i][j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int MTW, int NTW, int PF, int XPF>
static void run_split(const uint16_t *X, uint16_t *W, size_t copy_halves, int copies, float *out,
                      int T, int KT) {
  const int ntiles = 1380 / NTW * NTW;
  const int wgs = ntiles / NTW;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < copies; ++i)
    probe_split<MTW, NTW, PF, XPF><<<wgs, 512>>>(X, W + i * copy_halves, out, T, KT, ntiles);
  const int iters = 3 * copies;
  hipEventRecord(a);
  for (int i = 0; i < iters; ++i)
    probe_split<MTW, NTW, PF, XPF><<<wgs, 512>>>(X, W + (i % copies) * copy_halves, out, T, KT, ntiles);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  const double us = ms * 1000.0 / iters;
  const double wbytes = (double)ntiles * KT * 1024;
  const double xbytes = (double)wgs * 4 * MTW * KT * 1024;
  printf("split MTW %d NTW %2d PF %d XPF %d      : %7.2f us  %6.0f GB/s weights  %5.1f GB/s/CU in (W+X)  (%d WGs)\n",
         MTW, NTW, PF, XPF, us, wbytes / us / 1e3, (wbytes + xbytes) / us / 1e3 / wgs, wgs);
}

int main() {
  const int T = 168, KT = 128;
  const size_t copy_halves = (size_t)1380 * KT * 512;  // 180 MB
  const int copies = 5;
  uint16_t *W, *X;
  float *out;
  hipMalloc(&W, copy_halves * copies * 2);
  hipMemset(W, 0, copy_halves * copies * 2);
  hipMalloc(&X, (size_t)12 * KT * 1024);
  hipMemset(X, 0, (size_t)12 * KT * 1024);
  hipMalloc(&out, 64 << 20);
#define R(MTW, NTW, PF, MODE, KG) run<MTW, NTW, PF, MODE, KG>(#MODE, X, W, copy_halves, copies, out, T, KT)
#define R1(MTW, NTW, PF, MODE, KG) run<MTW, NTW, PF, MODE, KG>(#MODE, X, W, copy_halves, 1, out, T, KT)
  printf("cold (5 rotating 180 MB copies)\n");
  R(3, 6, 4, 0, 1);
  R(3, 6, 4, 7, 1);
  R(3, 12, 4, 7, 1);
  printf("one copy, re-read (Infinity Cache resident as far as it fits)\n");
  R1(3, 6, 4, 0, 1);
  R1(3, 6, 4, 7, 1);
  R1(3, 6, 8, 7, 1);
  R1(3, 12, 4, 7, 1);
  R1(3, 4, 4, 7, 1);
  return 0;
}
