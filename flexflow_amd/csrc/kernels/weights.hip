// weights.hip -- seeded synthetic weights and MFMA-fragment weight packing.
//
// Weight values follow the counter-based splitmix64 spec of
// oracle/oracle.h:orc_gen_weight bit for bit (no FMA contraction: explicit
// _rn intrinsics), so the GPU model and the CPU oracle hold identical fp16
// weights without shipping checkpoints (none exist offline).
//
// Packed layout ("MFMA B-fragment order") for Y = X . W^T with
// v_mfma_f32_16x16x32_f16: the [N][K] matrix is cut into 16x32 blocks, 1 KiB
// each; lane l of a wave owns halves [l*8, l*8+8) = W[nt*16 + (l&15)][kt*32 +
// 8*(l>>4) + 0..7], exactly the B operand the MFMA wants, so a wave streaming
// one N-tile reads contiguous 1 KiB per k-step (fully coalesced, 16 B/lane).
// Blocks are stored K-MAJOR: block (nt, kt) at (kt * P + nt) * 512 halves,
// P = the allocation's tiles per k-row (w_tile_stride / w_k_stride).  All
// workgroups of a GEMM walk k in step, so at any moment the chip reads one
// contiguous band of k-row kt instead of ~230 streams 128 KiB apart: the
// T = 168 gate/up loop went 57 -> 44 us in scripts/probe/xl2_probe.hip (the
// old tile-major order, FFMI_W_TILE_MAJOR=1, stays for A/B runs).
#include "../ffmi_internal.h"

namespace ffmi {

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// value i: element src(i) of the stream, src = i, or for a row-permuted
// [rows][cols] tensor (cols > 0) element (perm(r), c), perm(r) = (r * pa + pb)
// mod rows (the token-chain init's tied lm_head, oracle.h orc_gen_weight_rows)
// (OUT = float: the full-precision model's fp32 weights, the same values
// before the fp16 rounding -- the oracle's fp32 mode)
template <class OUT>
__global__ void fill_weight_kernel(OUT *dst, size_t n, uint64_t key, float center, float amp,
                                   int cols, uint64_t pa, uint64_t pb) {
  const uint64_t rows = cols > 0 ? n / cols : 1;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    uint64_t src = i;
    if (cols > 0) src = ((i / cols) * pa + pb) % rows * cols + i % cols;
    uint64_t x = splitmix64(key + (src + 1) * 0x9E3779B97F4A7C15ull);
    float u = (float)(x >> 40) * (1.0f / 16777216.0f);
    float t = __fsub_rn(__fmul_rn(2.0f, u), 1.0f);
    float w = __fadd_rn(center, __fmul_rn(t, amp));
    if constexpr (sizeof(OUT) == 4) dst[i] = w;
    else dst[i] = __half_as_ushort(__float2half_rn(w));
  }
}

// amplitude of a weight kind (oracle.h orc_weight_amp: the same host float
// operations, so both generators hold identical values)
float weight_amp(int kind) {
  if (kind == 1) return 0.1f;
  if (kind & FFMI_WKIND_DEPTH) return 0.034641016f / sqrtf((float)(2 * (kind & 0xffff)));
  return 0.034641016f;
}

hipError_t launch_fill_weight(uint16_t *dst, size_t n, uint64_t key, int kind, hipStream_t s,
                              int cols, uint64_t pa, uint64_t pb, float scale) {
  if (n == 0) return hipSuccess;
  size_t blocks = (n + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(fill_weight_kernel<uint16_t>, dim3((unsigned)blocks), dim3(256), 0, s, dst, n,
                     key, kind == 1 ? 1.0f : 0.0f, weight_amp(kind) * scale, cols, pa, pb);
  return hipGetLastError();
}

hipError_t launch_fill_weight_f32(float *dst, size_t n, uint64_t key, int kind, hipStream_t s,
                                  int cols, uint64_t pa, uint64_t pb, float scale) {
  if (n == 0) return hipSuccess;
  size_t blocks = (n + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(fill_weight_kernel<float>, dim3((unsigned)blocks), dim3(256), 0, s, dst, n,
                     key, kind == 1 ? 1.0f : 0.0f, weight_amp(kind) * scale, cols, pa, pb);
  return hipGetLastError();
}

uint64_t weight_key(const char *name, uint64_t seed) {
  uint64_t h = 1469598103934665603ull;
  for (const char *p = name; *p; ++p) {
    h ^= (uint8_t)*p;
    h *= 1099511628211ull;
  }
  return seed ^ h;
}

// One thread per (block, lane): gathers 8 halves of W[row][k..k+7].
__global__ void pack_weight_kernel(const uint16_t *__restrict__ src, int ld, int row0,
                                   int col0, int N, int K, int NT, int KT,
                                   uint16_t *__restrict__ dst, int tile_step,
                                   int tile_offset, size_t ts, size_t ks) {
  long gid = blockIdx.x * (long)blockDim.x + threadIdx.x;
  long total = (long)NT * KT * 64;
  if (gid >= total) return;
  int lane = (int)(gid & 63);
  long blk = gid >> 6;
  int kt = (int)(blk % KT);
  int nt = (int)(blk / KT);
  int n = nt * 16 + (lane & 15);
  int k = kt * 32 + 8 * (lane >> 4);
  uint16_t v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j)
    v[j] = (n < N && k + j < K) ? src[(size_t)(row0 + n) * ld + col0 + k + j] : 0;
  const long dtile = (long)tile_step * nt + tile_offset;
  uint4 pk;
  pk.x = v[0] | ((uint32_t)v[1] << 16);
  pk.y = v[2] | ((uint32_t)v[3] << 16);
  pk.z = v[4] | ((uint32_t)v[5] << 16);
  pk.w = v[6] | ((uint32_t)v[7] << 16);
  *reinterpret_cast<uint4 *>(dst + dtile * ts + kt * ks + lane * 8) = pk;
}

bool weights_kmajor() {
  static const bool km = !(getenv("FFMI_W_TILE_MAJOR") && atoi(getenv("FFMI_W_TILE_MAJOR")) != 0);
  return km;
}

hipError_t launch_pack_weight(const uint16_t *src, int ld, int row0, int col0, int N,
                              int K, uint16_t *dst, int tile_step, int tile_offset, int pitch,
                              hipStream_t s) {
  int NT = (N + 15) / 16, KT = (K + 31) / 32;
  const size_t ts = w_tile_stride(KT), ks = w_k_stride(pitch);
  long total = (long)NT * KT * 64;
  unsigned blocks = (unsigned)((total + 255) / 256);
  hipLaunchKernelGGL(pack_weight_kernel, dim3(blocks), dim3(256), 0, s, src, ld, row0,
                     col0, N, K, NT, KT, dst, tile_step, tile_offset, ts, ks);
  return hipGetLastError();
}

}  // namespace ffmi
