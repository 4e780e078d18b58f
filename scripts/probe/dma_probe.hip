// Can an 8-wave, LDS-DMA-fed GEMM loop take in more bytes per CU than the
// register-staged gemm_mid_kernel (~45-50 GB/s per CU)?  The k-loop of the
// T = 168 gate/up GEMM (K 4096, 1380 weight tiles, 12 activation m-tiles,
// packed fragments, k-major weights) with:
//   - NTW weight tiles x all 12 m-tiles per workgroup, split-K S;
//   - every k-step's fragments (12 X + NTW W, 1 KiB each) land in an LDS ring
//     slot through global_load_lds_dwordx4 (lane-linear 1 KiB per wave op),
//     issued PF-1 steps ahead by all 8 waves, retired with a counted vmcnt and
//     one raw s_barrier per k-step;
//   - waves = 4 row groups (3 m-tiles) x 2 column halves (NTW/2 tiles), MFMA
//     16x16x32 f16 from LDS fragments.
// MODE 1: no MFMA (loads + barrier + LDS reads only).
//   hipcc --offload-arch=gfx950 -O3 -o dma_probe dma_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

template <int NTW, int PF, int MODE>
__global__ __launch_bounds__(512, 1) void dma_probe(const uint16_t *__restrict__ X,
                                                    const uint16_t *__restrict__ W,
                                                    float *__restrict__ out, int KT, int NTILES,
                                                    int S) {
  constexpr int MT = 12, NF = MT + NTW, PER = (NF + 7) / 8, NH = NTW / 2;
  extern __shared__ __attribute__((aligned(16))) h8 ring[];  // [PF][NF][64]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int rg = wave & 3, ch = wave >> 2;
  const int tile0 = blockIdx.x * NTW, ks = blockIdx.y;
  const int per = KT / S, kb = ks * per;
  // this wave's DMA fragments f = wave + 8p: f < MT -> X m-tile f, else W tile f - MT
  const uint16_t *src[PER];
#pragma unroll
  for (int p = 0; p < PER; ++p) {
    const int f = min(wave + 8 * p, NF - 1);
    src[p] = f < MT ? X + ((size_t)f * KT * 64 + lane) * 8
                    : W + ((size_t)min(tile0 + f - MT, NTILES - 1) * 64 + lane) * 8;
  }
  auto issue = [&](int kt, int slot) {
#pragma unroll
    for (int p = 0; p < PER; ++p) {
      const int f = wave + 8 * p;
      if (PER * 8 == NF || f < NF) {
        const size_t step = f < MT ? (size_t)512 : (size_t)NTILES * 512;
        __builtin_amdgcn_global_load_lds(
            (const __attribute__((address_space(1))) void *)(src[p] + (size_t)kt * step),
            (__attribute__((address_space(3))) void *)(&ring[(slot * NF + f) * 64]), 16, 0, 0);
      }
    }
  };
  f4 acc[3][NH];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < NH; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int q = 0; q < PF - 1; ++q) issue(kb + q, q);
  for (int k = 0; k < per; ++k) {
    const int slot = k % PF;
    // this wave's DMAs of step k are done once at most (PF-2) steps' remain
    if (PF == 4) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER) : "memory");
    __builtin_amdgcn_s_barrier();
    if (k + PF - 1 < per) issue(kb + k + PF - 1, (k + PF - 1) % PF);
    else if (PF == 4) {  // keep the vmcnt arithmetic: re-issue into the spare slot
      issue(kb + per - 1, (k + PF - 1) % PF);
    }
    h8 xf[3], wf[NH];
#pragma unroll
    for (int i = 0; i < 3; ++i) xf[i] = ring[(slot * NF + rg * 3 + i) * 64 + lane];
#pragma unroll
    for (int j = 0; j < NH; ++j) wf[j] = ring[(slot * NF + MT + ch * NH + j) * 64 + lane];
    if (MODE == 0) {
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < NH; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[j], xf[i], acc[i][j], 0, 0, 0);
    } else {
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < NH; ++j) acc[i][j][0] += (float)wf[j][0] * (float)xf[i][1];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  float s = 0;
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < NH; ++j) s += acc[i][j][0] + acc[i][j][3];
  out[(blockIdx.y * gridDim.x + blockIdx.x) * blockDim.x + threadIdx.x] = s;
}

__global__ void fillr(uint16_t *p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)(i * 2654435761u) ^ (uint32_t)(i >> 7);
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    _Float16 v = (_Float16)(((float)(h & 0xffff) / 65536.0f - 0.5f) * 0.1f);
    p[i] = *reinterpret_cast<uint16_t *>(&v);
  }
}

template <int NTW, int PF, int MODE>
static void run(const uint16_t *X, uint16_t *W, size_t copy_halves, int copies, float *out, int KT,
                int S) {
  const int ntiles = 1380 / NTW * NTW;
  const int wgs = ntiles / NTW;
  const size_t lds = (size_t)PF * (12 + NTW) * 1024;
  (void)hipFuncSetAttribute((const void *)dma_probe<NTW, PF, MODE>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int i = 0; i < copies; ++i)
    dma_probe<NTW, PF, MODE><<<dim3(wgs, S), 512, lds>>>(X, W + i * copy_halves, out, KT, ntiles, S);
  const int iters = 3 * copies;
  (void)hipEventRecord(a);
  for (int i = 0; i < iters; ++i)
    dma_probe<NTW, PF, MODE><<<dim3(wgs, S), 512, lds>>>(X, W + (i % copies) * copy_halves, out, KT,
                                                          ntiles, S);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  const double us = ms * 1000.0 / iters;
  const double wbytes = (double)ntiles * KT * 1024, xbytes = (double)wgs * S * 12 * (KT / S) * 1024;
  printf("NTW %2d S %d PF %d mode %d: %7.2f us  %5.1f GB/s/CU in (W+X), %d WGs\n", NTW, S, PF, MODE,
         us, (wbytes + xbytes) / us / 1e3 / (wgs * S), wgs * S);
}

int main() {
  const int KT = 128;
  const size_t copy_halves = (size_t)1380 * KT * 512;
  const int copies = 5;
  uint16_t *W, *X;
  float *out;
  (void)hipMalloc(&W, copy_halves * copies * 2);
  (void)hipMalloc(&X, (size_t)12 * KT * 1024);
  (void)hipMalloc(&out, 64 << 20);
  fillr<<<4096, 256>>>(W, copy_halves * copies);
  fillr<<<1024, 256>>>(X, (size_t)12 * KT * 512);
  (void)hipDeviceSynchronize();
  run<12, 4, 0>(X, W, copy_halves, copies, out, KT, 2);
  run<12, 4, 1>(X, W, copy_halves, copies, out, KT, 2);
  run<12, 3, 0>(X, W, copy_halves, copies, out, KT, 2);

  run<12, 4, 0>(X, W, copy_halves, copies, out, KT, 1);
  run<12, 4, 0>(X, W, copy_halves, copies, out, KT, 2);
  return 0;
}
