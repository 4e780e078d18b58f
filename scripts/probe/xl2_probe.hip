// Is the M-split GEMM's activation intake limited by L2 channel hot spots?
// Every workgroup of the T = 168 gate/up launch reads the same activation
// k-step at about the same time; in the packed [mt][kt] layout the 12 m-tile
// fragments of one k-step sit 128 KiB apart.  This probe runs the
// gemm_mid_kernel loop (MODE bits as stream_probe.hip: 1 = activations,
// 2 = weights through LDS, 4 = MFMA, 8 = no weight loads) with
//   ROT = 1: each workgroup starts its k loop at a different k-step (wraps),
//   LAY = 1: activations stored [kt][mt] (one k-step = 12 KiB contiguous).
//   hipcc --offload-arch=gfx950 -O3 -o xl2_probe xl2_probe.hip
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

template <int MTW, int NTW, int PF, int MODE, int ROT, int LAY, int WL = 0, int NTL = 0, int LB = 1, int WMOD = 0, int NOULD = 0>
__global__ __launch_bounds__(256, LB) void probe(const uint16_t *__restrict__ X,
                                                const uint16_t *__restrict__ Wp,
                                                float *__restrict__ out, int T, int KT,
                                                int NTILES) {
  constexpr int PPT = (NTW + 3) / 4;
  __shared__ __attribute__((aligned(16))) h8 sB[2][NTW][64];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int tile0 = blockIdx.x * NTW;
  const int m0 = wave * MTW * 16;
  const int MT = (T + 15) / 16;
  const int rot = ROT ? (int)((blockIdx.x * 37u) % (unsigned)KT) : 0;
  const uint16_t *bsrc[PPT];
#pragma unroll
  for (int p = 0; p < PPT; ++p) {
    int t = min(tile0 + min(wave + 4 * p, NTW - 1), NTILES - 1);
    if (WMOD) t %= WMOD;
    bsrc[p] = WL ? Wp + (size_t)t * 512 + lane * 8 : Wp + (size_t)t * KT * 512 + lane * 8;
  }
  const size_t wks = WL ? (size_t)(WMOD ? WMOD : NTILES) * 512 : 512;
  const uint16_t *xrow[MTW];
  size_t xs;
#pragma unroll
  for (int i = 0; i < MTW; ++i) {
    const int mt = min((m0 + i * 16) >> 4, MT - 1);
    xrow[i] = LAY ? X + ((size_t)mt * 64 + lane) * 8 : X + ((size_t)mt * KT * 64 + lane) * 8;
  }
  xs = LAY ? (size_t)MT * 512 : 512;
  f4 acc[MTW][NTW];
#pragma unroll
  for (int i = 0; i < MTW; ++i)
#pragma unroll
    for (int j = 0; j < NTW; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  auto kmap = [&](int k) { return ROT ? ((k + rot) & (KT - 1)) : k; };
  h8 bq[PF][PPT];
  h8 xq[PF][MTW];
#pragma unroll
  for (int q = 0; q < PF; ++q) {
    const int kq = kmap(q);
    if (MODE & 1)
#pragma unroll
      for (int i = 0; i < MTW; ++i) xq[q][i] = *reinterpret_cast<const h8 *>(xrow[i] + (size_t)kq * xs);
#pragma unroll
    for (int p = 0; p < PPT; ++p)
      if (!(MODE & 8) && (!NOULD || NTW % 4 == 0 || wave + 4 * p < NTW)) bq[q][p] = NTL ? __builtin_nontemporal_load(reinterpret_cast<const h8 *>(bsrc[p] + (size_t)kq * wks)) : *reinterpret_cast<const h8 *>(bsrc[p] + (size_t)kq * wks);
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
      if (NTW % 4 == 0 || wave + 4 * p < NTW) sB[0][wave + 4 * p][lane] = bq[0][p];
    __syncthreads();
  }
  int cur = 0;
  auto step = [&](auto Qc, int kt) {
    constexpr int Q = decltype(Qc)::value;
    h8 b[NTW];
    if (MODE & 2) {
#pragma unroll
      for (int j = 0; j < NTW; ++j) b[j] = sB[cur][j][lane];
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
    const int kw = kmap(min(kt + PF, KT - 1));
    if (MODE & 1)
#pragma unroll
      for (int i = 0; i < MTW; ++i) xq[Q][i] = *reinterpret_cast<const h8 *>(xrow[i] + (size_t)kw * xs);
#pragma unroll
    for (int p = 0; p < PPT; ++p)
      if (!(MODE & 8) && (!NOULD || NTW % 4 == 0 || wave + 4 * p < NTW)) bq[Q][p] = NTL ? __builtin_nontemporal_load(reinterpret_cast<const h8 *>(bsrc[p] + (size_t)kw * wks)) : *reinterpret_cast<const h8 *>(bsrc[p] + (size_t)kw * wks);
    if (!(MODE & 1))
#pragma unroll
      for (int i = 0; i < MTW; ++i) xq[Q][i] = bq[Q][0];
    if (MODE & 2) {
#pragma unroll
      for (int p = 0; p < PPT; ++p)
        if (NTW % 4 == 0 || wave + 4 * p < NTW) sB[cur ^ 1][wave + 4 * p][lane] = bq[(Q + 1) % PF][p];
      __syncthreads();
      cur ^= 1;
    }
  };
  int kt0 = 0;
  for (; kt0 + PF <= KT; kt0 += PF) sfor<PF>([&](auto Qc) { step(Qc, kt0 + decltype(Qc)::value); });
  float s = 0;
#pragma unroll
  for (int i = 0; i < MTW; ++i)
#pragma unroll
    for (int j = 0; j < NTW; ++j) s += acc[i][j][0] + acc[i][j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int MTW, int NTW, int PF, int MODE, int ROT, int LAY, int WL = 0, int NTL = 0, int LB = 1, int WMOD = 0, int NOULD = 0>
static void run(const uint16_t *X, uint16_t *W, size_t copy_halves, int copies, float *out, int T,
                int KT) {
  const int ntiles = 1380 / NTW * NTW;
  const int wgs = ntiles / NTW;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < copies; ++i)
    probe<MTW, NTW, PF, MODE, ROT, LAY, WL, NTL, LB, WMOD, NOULD><<<wgs, 256>>>(X, W + i * copy_halves, out, T, KT, ntiles);
  const int iters = 3 * copies;
  hipEventRecord(a);
  for (int i = 0; i < iters; ++i)
    probe<MTW, NTW, PF, MODE, ROT, LAY, WL, NTL, LB, WMOD, NOULD><<<wgs, 256>>>(X, W + (i % copies) * copy_halves, out, T,
                                                      KT, ntiles);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  const double us = ms * 1000.0 / iters;
  const double wbytes = (MODE & 8) ? 0.0 : (double)ntiles * KT * 1024;
  const double xbytes = (MODE & 1) ? (double)wgs * 4 * MTW * KT * 1024 : 0.0;
  printf("NOULD %d WMOD %d LB %d NTL %d NTW %2d PF %d mode %2d rot %d lay %d wl %d: %7.2f us  %5.1f GB/s/CU in (W+X)\n", NOULD, WMOD, LB, NTL, NTW, PF, MODE,
         ROT, LAY, WL, us, (wbytes + xbytes) / us / 1e3 / wgs);
}

__global__ void fillr(uint16_t *p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)(i * 2654435761u) ^ (uint32_t)(i >> 7);
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    _Float16 v = (_Float16)(((float)(h & 0xffff) / 65536.0f - 0.5f) * 0.1f);
    p[i] = *reinterpret_cast<uint16_t *>(&v);
  }
}

int main(int argc, char **argv) {
  const bool rnd = argc > 1;
  const int T = 168, KT = 128;
  const size_t copy_halves = (size_t)1380 * KT * 512;  // 180 MB
  const int copies = 5;
  uint16_t *W, *X;
  float *out;
  hipMalloc(&W, copy_halves * copies * 2);
  hipMemset(W, 0, copy_halves * copies * 2);
  hipMalloc(&X, (size_t)12 * KT * 1024);
  hipMemset(X, 0, (size_t)12 * KT * 1024);
  if (rnd) {
    fillr<<<4096, 256>>>(W, copy_halves * copies);
    fillr<<<1024, 256>>>(X, (size_t)12 * KT * 512);
    hipDeviceSynchronize();
    printf("random data\n");
  }
  hipMalloc(&out, 64 << 20);
#define R(NTW, PF, MODE, ROT, LAY) run<3, NTW, PF, MODE, ROT, LAY>(X, W, copy_halves, copies, out, T, KT)
#define RW(NTW, PF, MODE, ROT, WL) run<3, NTW, PF, MODE, ROT, 0, WL>(X, W, copy_halves, copies, out, T, KT)
#define RU(MODE, NU) run<3, 6, 4, MODE, 0, 0, 1, 1, 2, 0, NU>(X, W, copy_halves, copies, out, T, KT)
  RU(7, 0);
  RU(7, 1);
  RU(7, 0);
  RU(7, 1);
  RU(1, 0);
  RU(1, 1);
  return 0;
}
