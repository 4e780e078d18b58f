// norm.hip -- RMSNorm / ResidualRMSNorm, embedding, SiLU-mul, softmax+argmax/topk.
//
// HBM-bound row kernels: one 256-thread workgroup per row, 16-B vector
// loads/stores (8 halves per lane), the row kept in registers between the
// reduction and the scale pass (one read + one write per element).  Unlike
// the reference (which launches every buffer row, rms_norm_kernels.cu:133-134)
// only the T active rows are processed.
#include <algorithm>

#include "../ffmi_internal.h"

namespace ffmi {

__device__ __forceinline__ float h2f_(uint16_t v) { return __half2float(__ushort_as_half(v)); }
__device__ __forceinline__ uint16_t f2h_(float v) { return __half_as_ushort(__float2half_rn(v)); }

// exp(x) for the softmax / top-k terms and probabilities, bit-identical to the
// host libm expf the oracle calls (glibc's double-evaluated algorithm: x /
// ln2 * 32 rounded to k, 2^(k/32) from a 32-entry table, a cubic in the
// remainder, one rounding to float; checked against glibc 2.35 expf on every
// float in [-104, 0], scripts/diag/expf_ref_check.c: 1 difference in 1.1e9,
// at x = -63.1, whose fp16 probability is 0 either way).  The device
// library's expf differs from it by one float ulp on ~1e-4 of inputs, mostly
// near 0 -- where a flat row's terms all lie -- which moved fp16 p values
// across a rounding boundary and reordered tied top-k ids (the fresh-seed
// random-shape sweep of test_softmax_topk_random_shapes_exact).
__constant__ unsigned long long kExp2Tab[32] = {
    0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,
    0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,
    0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,
    0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,
    0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,
    0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,
    0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,
    0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull};
__device__ __forceinline__ float expf_ref_core(float x) {
  const double N = 32.0;
  const double InvLn2N = 0x1.71547652b82fep+0 * N, SHIFT = 0x1.8p+52;
  const double C0 = 0x1.c6af84b912394p-5 / N / N / N, C1 = 0x1.ebfce50fac4f3p-3 / N / N,
               C2 = 0x1.62e42ff0c52d6p-1 / N;
  const double z = __dmul_rn(InvLn2N, (double)x);
  double kd = __dadd_rn(z, SHIFT);
  const unsigned long long ki = (unsigned long long)__double_as_longlong(kd);
  kd = __dsub_rn(kd, SHIFT);
  const double r = __dsub_rn(z, kd);
  const double s = __longlong_as_double((long long)(kExp2Tab[ki & 31] + (ki << 47)));
  const double p = __fma_rn(C0, r, C1);
  const double r2 = __dmul_rn(r, r);
  double y = __fma_rn(C2, r, 1.0);
  y = __fma_rn(p, r2, y);
  return (float)__dmul_rn(y, s);
}
// Branch-free (every caller passes x = logit - row max <= 0): the formula runs
// on max(x, -104) and the result is selected, so an unrolled loop of terms
// issues all its table loads ahead of the arithmetic instead of one
// load-and-wait per term behind per-element branches.
__device__ __forceinline__ float expf_ref(float x) {
  const bool in = x > -104.0f;
  const float xr = in ? x : -104.0f;  // (NaN and -inf too: selected away below)
  const float y = expf_ref_core(xr);
  return in ? y : (x == x ? 0.0f : x);  // (underflow to 0; NaN stays NaN)
}

template <int NW, typename T>
__device__ __forceinline__ T block_sum(T v, T *scratch) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) scratch[wave] = v;
  __syncthreads();
  T r = scratch[0];
#pragma unroll
  for (int q = 1; q < NW; ++q) r += scratch[q];
  return r;
}

// rms_norm_kernels.cu:97-124 / residual_rms_norm_kernels.cu:98-131:
//   r = x1 (+ x2, rounded to half); rms = half(rsqrt(mean(r^2) + eps));
//   y = half(r * rms); out = half(y * w)
// One workgroup of NT threads per row, MAXC 8-element chunks per thread; every
// load of the row (x1, x2 or its split-K slabs, and w) is issued before the
// reduction, so a row costs one memory round trip.
// SRC (compile time, so that the loads are straight-line code: behind
// runtime branches the compiler reused a loaded register as the slab address
// and waited for the x1 load before issuing the slabs -- two round trips):
//   0: x1 only   1: x1 + x2 (fp16)   2: x1 + split-K slabs   3: gather (x1 =
//   embedding table, rows picked by the step's token ids)
//   4 / 5: 1 / 2 with the FFMI_FAULT_RESID_ROUND negative control (tests
//   only): the sum of squares takes the UNROUNDED fp32 residual sum, where
//   residual_rms_norm_kernels.cu:112-114 squares the half-rounded one
template <int NT, int MAXC, int MAXS, int SRC>
__global__ __launch_bounds__(NT) void rmsnorm_kernel(
    const uint16_t *__restrict__ x1, const uint16_t *__restrict__ x2,
    const uint16_t *__restrict__ w, uint16_t *__restrict__ res_out,
    uint16_t *__restrict__ out, int H, float eps, int out_packed,
    const float *__restrict__ x2p, int pS, int pNP, const char *__restrict__ gather,
    uint4 *__restrict__ blob_dst, int blob_n16, const int32_t *__restrict__ gprev) {
  __shared__ double scratch[NT / 64];
  const int row = blockIdx.x;
  const int T = gridDim.x;
  const int nchunk = H >> 3;
  // gather: x1 is the embedding table and row t reads its token's row (the
  // embedding lookup fused into the first layer's norm; res_out gets the copy)
  constexpr bool FAULT = SRC >= 4;
  constexpr int S = FAULT ? SRC - 3 : SRC;  // the data source of the variant
  // (a chained SSM beam step: token id -1 - i is entry i of the previous
  // step's top-k ids, gprev, which the host could not know when it staged
  // this step; ffmi_model beam_launch_chained)
  int gid = 0;
  if (S == 3) {
    gid = batch_view(gather).tokens[row].token_id;
    if (gid < 0) gid = gprev[-1 - gid];
  }
  const uint16_t *a = S == 3 ? x1 + (size_t)gid * H : x1 + (size_t)row * H;
  // blob fetch: gather is the step's staging blob in mapped host memory; the
  // grid copies it into device memory for the step's later kernels (replaces
  // the H2D copy node and the system-scope boundary after it), its loads in
  // flight together with the token-id read
  if (S == 3 && blob_dst) {
    const uint4 *src = reinterpret_cast<const uint4 *>(gather);
    for (int i = row * NT + threadIdx.x; i < blob_n16; i += T * NT) blob_dst[i] = src[i];
  }
  uint4 v[MAXC], wv[MAXC];
  // every load of the row first (slabs, x2, x1, w), then the arithmetic;
  // x2 = the deferred split-K slabs of the producing GEMM summed in order,
  // folded per chunk when a thread holds several chunks (register budget)
  uint4 xb[MAXC];
  f4 slo[MAXS], shi[MAXS];
  auto fold = [&]() {
    f4 lo = slo[0], hi = shi[0];
#pragma unroll
    for (int sl = 1; sl < MAXS; ++sl)
      if (sl < pS) lo += slo[sl], hi += shi[sl];
    uint16_t hb[8];
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) {
      hb[q4] = f2h_(lo[q4]);
      hb[q4 + 4] = f2h_(hi[q4]);
    }
    return *reinterpret_cast<uint4 *>(hb);
  };
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = min((int)threadIdx.x + c * NT, nchunk - 1);  // clamped: no branch
    if (S == 2) {
      const float *q = x2p + (size_t)row * pNP + ch * 8;
#pragma unroll
      for (int sl = 0; sl < MAXS; ++sl) {
        const float *qs = q + (size_t)min(sl, pS - 1) * T * pNP;
        slo[sl] = *reinterpret_cast<const f4 *>(qs);
        shi[sl] = *reinterpret_cast<const f4 *>(qs + 4);
      }
    }
    if (S == 1) xb[c] = *reinterpret_cast<const uint4 *>(x2 + (size_t)row * H + ch * 8);
    v[c] = *reinterpret_cast<const uint4 *>(a + ch * 8);
    wv[c] = *reinterpret_cast<const uint4 *>(w + ch * 8);
    if (S == 2 && MAXC > 1) xb[c] = fold();
  }
  if (S == 2 && MAXC == 1) xb[0] = fold();
  // the sum of squares in fp64, as the oracle's (exact products, then one
  // rounding to float): an fp32 sum in another order than the oracle's moved
  // rms across a half rounding boundary in ~1 row in 10^3 at H = 16160
  // (test_rmsnorm_random_shapes sweep), where every output of the row shifts
  double ss = 0.0;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = threadIdx.x + c * NT;
    if (ch < nchunk) {
      uint4 xa = v[c];
      if (S == 1 || S == 2) {
        const uint4 xbb = xb[c];
        const __half2 *pa = reinterpret_cast<const __half2 *>(&xa);
        const __half2 *pb = reinterpret_cast<const __half2 *>(&xbb);
        if (FAULT) {  // negative control: square the unrounded sum
          const uint16_t *ea = reinterpret_cast<const uint16_t *>(&xa);
          const uint16_t *eb = reinterpret_cast<const uint16_t *>(&xbb);
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const float f = h2f_(ea[q]) + h2f_(eb[q]);
            ss += (double)f * (double)f;
          }
        }
        __half2 r[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) r[q] = __hadd2(pa[q], pb[q]);  // correctly rounded
        xa = *reinterpret_cast<uint4 *>(r);
        *reinterpret_cast<uint4 *>(res_out + (size_t)row * H + ch * 8) = xa;
      } else if (S == 3) {
        *reinterpret_cast<uint4 *>(res_out + (size_t)row * H + ch * 8) = xa;
      }
      v[c] = xa;
      const uint16_t *e = reinterpret_cast<const uint16_t *>(&xa);
      if (!FAULT) {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const float f = h2f_(e[q]);
          ss += (double)f * (double)f;
        }
      }
    }
  }
  const float sum = (float)block_sum<NT / 64>(ss, scratch);
  // sqrtf: the correctly rounded square root (HIP's __fsqrt_rn is the native
  // v_sqrt_f32, ~1 ulp, unless OCML_BASIC_ROUNDED_OPERATIONS is defined)
  const float rms_f = __fdiv_rn(1.0f, sqrtf(__fadd_rn(__fdiv_rn(sum, (float)H), eps)));
  const float rms = h2f_(f2h_(rms_f));
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = threadIdx.x + c * NT;
    if (ch < nchunk) {
      const uint16_t *e = reinterpret_cast<const uint16_t *>(&v[c]);
      const uint16_t *we = reinterpret_cast<const uint16_t *>(&wv[c]);
      uint16_t o8[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        float y = h2f_(f2h_(__fmul_rn(h2f_(e[q]), rms)));
        o8[q] = f2h_(__fmul_rn(y, h2f_(we[q])));
      }
      uint16_t *dst = out_packed ? out + act_packed_off(row, ch * 8, H) : out + (size_t)row * H + ch * 8;
      *reinterpret_cast<uint4 *>(dst) = *reinterpret_cast<uint4 *>(o8);
    }
  }
}

// FFMI_FAULT_RESID_ROUND (tests only, process-wide): residual norms take the
// faulted variants (SRC 4 / 5)
static bool g_norm_fault = false;
void set_norm_fault(bool on) { g_norm_fault = on; }

hipError_t launch_rmsnorm(const uint16_t *x1, const uint16_t *x2, const uint16_t *w,
                          uint16_t *res_out, uint16_t *out, int T, int H, float eps,
                          hipStream_t s, bool out_packed, Partials x2p, const char *gather,
                          char *blob_dst, size_t blob_bytes, const int32_t *gather_prev) {
  if (gather && (x2 || x2p.S > 0 || !res_out)) return hipErrorInvalidValue;
  if (blob_dst && (!gather || blob_bytes > (size_t)1 << 30 || (uintptr_t)gather % 16 ||
                   (uintptr_t)blob_dst % 16))
    return hipErrorInvalidValue;
  // whole 16-byte chunks: the staging and device blobs are 16-aligned and
  // padded (ffmi_batch_create), so the rounded-up tail stays inside both
  const int blob_n16 = blob_dst ? (int)((blob_bytes + 15) / 16) : 0;
  if (T <= 0) return hipSuccess;
  if (out_packed && H % 32) return hipErrorInvalidValue;
  const int op = out_packed ? 1 : 0;
  const int nchunk = H / 8;
  if (nchunk > 4096) return hipErrorInvalidValue;
  const float *pp = x2p.S > 0 ? x2p.p : nullptr;
  // > 8 slabs: the per-head o-projection slabs of a small model (OprojArgs,
  // <= 16 heads, H <= 1024)
  if (pp && (x2p.S > 16 || (x2p.S > 8 && nchunk > 128))) return hipErrorInvalidValue;
  if ((x2 || pp) && !res_out) return hipErrorInvalidValue;
  // split-K slabs: one 8-column chunk per thread (H <= 8192); the model does
  // not defer its o/down partials beyond that
  if (pp && nchunk > 1024) return hipErrorInvalidValue;
  const int src = gather ? 3 : pp ? 2 : x2 ? 1 : 0;
  const int ms = !pp || x2p.S <= 1 ? 1 : x2p.S <= 2 ? 2 : x2p.S <= 4 ? 4 : x2p.S <= 8 ? 8
               : x2p.S <= 12 ? 12 : 16;
#define FFMI_RMS3(NT, MC, MS, SR)                                                              \
  hipLaunchKernelGGL((rmsnorm_kernel<NT, MC, MS, SR>), dim3(T), dim3(NT), 0, s, x1, x2, w,    \
                     res_out, out, H, eps, op, pp, x2p.S, x2p.NP, gather,               \
                     reinterpret_cast<uint4 *>(blob_dst), blob_n16, gather_prev)
#define FFMI_RMS(NT, MC)                                   \
  do {                                                     \
    if (src == 0) FFMI_RMS3(NT, MC, 1, 0);                 \
    else if (src == 1) FFMI_RMS3(NT, MC, 1, 1);            \
    else if (src == 3) FFMI_RMS3(NT, MC, 1, 3);            \
    else if (ms == 1) FFMI_RMS3(NT, MC, 1, 2);             \
    else if (ms == 2) FFMI_RMS3(NT, MC, 2, 2);             \
    else if (ms == 4) FFMI_RMS3(NT, MC, 4, 2);             \
    else FFMI_RMS3(NT, MC, 8, 2);                          \
  } while (0)
#define FFMI_RMS_NOSLAB(NT, MC)                            \
  do {                                                     \
    if (src == 0) FFMI_RMS3(NT, MC, 1, 0);                 \
    else if (src == 1) FFMI_RMS3(NT, MC, 1, 1);            \
    else FFMI_RMS3(NT, MC, 1, 3);                          \
  } while (0)
  if (g_norm_fault && (src == 1 || src == 2)) {  // negative control (tests only)
#define FFMI_RMSF(NT)                                      \
  do {                                                     \
    if (src == 1) FFMI_RMS3(NT, 1, 1, 4);                  \
    else if (ms == 1) FFMI_RMS3(NT, 1, 1, 5);              \
    else if (ms == 2) FFMI_RMS3(NT, 1, 2, 5);              \
    else if (ms == 4) FFMI_RMS3(NT, 1, 4, 5);              \
    else if (ms == 8) FFMI_RMS3(NT, 1, 8, 5);              \
    else return hipErrorInvalidValue;                      \
  } while (0)
    if (nchunk <= 128) FFMI_RMSF(128);
    else if (nchunk <= 256) FFMI_RMSF(256);
    else if (nchunk <= 512) FFMI_RMSF(512);
    else if (nchunk <= 1024) FFMI_RMSF(1024);
    else return hipErrorInvalidValue;
#undef FFMI_RMSF
    return hipGetLastError();
  }
  if (nchunk <= 128 && ms == 12) FFMI_RMS3(128, 1, 12, 2);
  else if (nchunk <= 128 && ms == 16) FFMI_RMS3(128, 1, 16, 2);
  else if (nchunk <= 128) FFMI_RMS(128, 1);
  else if (nchunk <= 256) FFMI_RMS(256, 1);
  else if (nchunk <= 512) FFMI_RMS(512, 1);
  else if (nchunk <= 1024) FFMI_RMS(1024, 1);
  else if (nchunk <= 2048) FFMI_RMS_NOSLAB(1024, 2);
  else FFMI_RMS_NOSLAB(1024, 4);
#undef FFMI_RMS_NOSLAB
#undef FFMI_RMS
#undef FFMI_RMS3
  return hipGetLastError();
}

// embed_forward_no_aggr (embedding_kernels.cu:233-244)
__global__ void embedding_kernel(const char *__restrict__ blob,
                                 const uint16_t *__restrict__ table,
                                 uint16_t *__restrict__ out, int H) {
  const BatchView bv = batch_view(blob);
  const int t = blockIdx.x;
  const int tok = bv.tokens[t].token_id;
  const uint4 *src = reinterpret_cast<const uint4 *>(table + (size_t)tok * H);
  uint4 *dst = reinterpret_cast<uint4 *>(out + (size_t)t * H);
  for (int c = threadIdx.x; c < H / 8; c += blockDim.x) dst[c] = src[c];
}

hipError_t launch_embedding(const char *blob, int T, const uint16_t *table, uint16_t *out,
                            int H, hipStream_t s) {
  if (T <= 0) return hipSuccess;
  if (H % 8 != 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(embedding_kernel, dim3(T), dim3(256), 0, s, blob, table, out, H);
  return hipGetLastError();
}

// SigmoidSiluMultiKernel (sigmoid_silu_multi.cu:37-47)
__global__ void silu_mul_kernel(const uint16_t *__restrict__ a, const uint16_t *__restrict__ b,
                                uint16_t *__restrict__ out, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    const float g = h2f_(a[i]);
    const float sg = __fdiv_rn(1.0f, __fadd_rn(1.0f, expf(-g)));
    const float t = h2f_(f2h_(__fmul_rn(g, h2f_(f2h_(sg)))));
    out[i] = f2h_(__fmul_rn(t, h2f_(b[i])));
  }
}

hipError_t launch_silu_mul(const uint16_t *a, const uint16_t *b, uint16_t *out, size_t n,
                           hipStream_t s) {
  if (n == 0) return hipSuccess;
  size_t blocks = (n + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(silu_mul_kernel, dim3((unsigned)blocks), dim3(256), 0, s, a, b, out, n);
  return hipGetLastError();
}

// Wave-wide reductions on DPP / permlane (device library), not LDS
// bpermute shuffles: the result is uniform across the wave.
extern "C" __device__ float __ockl_wfred_max_f32(float);
extern "C" __device__ double __ockl_wfred_add_f64(double);
extern "C" __device__ unsigned long long __ockl_wfred_max_u64(unsigned long long);

// softmax (fp16 output, softmax.cu:262-288) + ArgMax (argmax.cu:62-100) /
// ArgTopK (arg_topk.cu:339-448), register-resident: one TPB-thread workgroup
// per row reads the row ONCE as 16-B vectors (NV per thread) and keeps it in
// registers.  p_i = half(exp(x_i - max) / S); the pick is the lowest index of
// the largest p_i (ties created by the fp16 rounding resolve exactly as cub
// ArgMax / the top-k heap do).
//  * S = float(sum of exp(x_i - M) accumulated in double): the oracle's
//    float(double sum), whatever the summation order.
//  * p_i is computed only for CANDIDATES: p is non-decreasing in x, and the
//    k-th largest of the per-wave maxima, L, is <= the row's k-th largest
//    logit, so every member of the top-k (ties included) has fp16 p >= p(L),
//    i.e. an unrounded p_i above the lower rounding boundary of p(L): x_i >=
//    M + log(boundary * S).  That threshold (lowered by a margin that covers
//    the float error of exp/div/log) excludes all but a handful of logits, and
//    the 32000 exp + correctly rounded divisions of a full p pass go away.
//  * The candidates' (p desc, idx asc) keys go to an LDS list; one wave picks
//    the k best (k wave reductions, no workgroup barrier).  More than kCand
//    candidates (flat rows, planted ties) fall back to k rounds of a
//    workgroup-wide selection over the registers.
//  * G > 1 (few rows: the SSM's beam steps, decode): G workgroups per row
//    (grid G x T), each loading the whole row (max and wave maxima identical
//    in all of them) but summing the exp terms of only 1/G of every thread's
//    elements: the double-precision expf_ref terms are the kernel's cost, and
//    T = 24 rows kept them on 24 CUs.  Each workgroup publishes its partial
//    sum (one lane: agent-scope store, drained, then an agent-scope add on
//    the row's counter); the workgroup whose add comes last reads the G
//    partials by atomic reads, sums them in chunk order, resets the counter
//    and finishes the row from its registers.  No workgroup waits for
//    another.  The double sum is split differently than at G = 1 (and than
//    the oracle's serial loop): S = float(double sum) in any order, as above.
//    `part` = [T][G] doubles, `cnt` = [T] counters, zero before the first
//    launch and left zero.
template <int TPB, int NV, int G>
__global__ __launch_bounds__(TPB) void softmax_topk_reg_kernel(
    const uint16_t *__restrict__ logits, int V, int k, int32_t *__restrict__ ids,
    float *__restrict__ probs, double *__restrict__ part, unsigned *__restrict__ cnt,
    int32_t *__restrict__ ids2) {
  constexpr int NW = TPB / 64;
  constexpr int kCand = 128;
  static_assert(G == 1 || ((NV * 8) % G == 0 && NV * 8 / G >= 2),
                "split: whole dwords of a thread's elements per workgroup");
  constexpr int E = NV * 8 / G;  // elements of each thread's row part this workgroup sums
  // wave maxima / sums / selection keys, and the candidate list
  __shared__ double sh[NW + 2];
  __shared__ unsigned long long cand[kCand];
  __shared__ unsigned ncand;
  __shared__ int last_arrival;
  float *fsh = reinterpret_cast<float *>(sh);
  unsigned long long *ksh = reinterpret_cast<unsigned long long *>(sh);
  const int row = G == 1 ? blockIdx.x : blockIdx.y, chunk = G == 1 ? 0 : blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int nvec = V >> 3;
  const uint4 *x = reinterpret_cast<const uint4 *>(logits + (size_t)row * V);
  // split form: workgroup `chunk` loads the row's vectors rotated so that the
  // elements it sums are always its first E (compile-time register indices):
  // local vector v holds row vector gv(v); E < 8: a runtime half / quarter of
  // local vector 0, at element eo
  constexpr int EPV = E < 8 ? 8 / E : 1;  // workgroups sharing one vector
  const int vrot = G == 1 ? 0 : (E >= 8 ? chunk * (E / 8) : chunk / EPV);
  const int eo = E >= 8 ? 0 : (chunk % EPV) * E;
  auto gv = [&](int v) -> int { return (G == 1 ? v : (v + vrot) % NV) * TPB + tid; };
  uint4 r[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int i = gv(v);
    r[v] = i < nvec ? x[i] : make_uint4(0xfc00fc00u, 0xfc00fc00u, 0xfc00fc00u, 0xfc00fc00u);
  }
  if (tid == 0) ncand = 0;
  auto elem = [&](int v, int e) -> float {
    const uint32_t w = (&r[v].x)[e >> 1];
    return h2f_((uint16_t)((e & 1) ? (w >> 16) : (w & 0xffffu)));
  };
  float mx = -INFINITY;
#pragma unroll
  for (int v = 0; v < NV; ++v)
#pragma unroll
    for (int e = 0; e < 8; ++e) mx = fmaxf(mx, elem(v, e));
  mx = __ockl_wfred_max_f32(mx);
  if (lane == 0) fsh[wv] = mx;
  __syncthreads();
  float wmax[NW];
#pragma unroll
  for (int q = 0; q < NW; ++q) wmax[q] = fsh[q];
  __syncthreads();
  float M = wmax[0];
#pragma unroll
  for (int q = 1; q < NW; ++q) M = fmaxf(M, wmax[q]);
  // L = k-th largest wave maximum (k <= 4 <= NW): a lower bound of the k-th
  // largest logit
  float L = -INFINITY;
  {
    float top[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
    for (int q = 0; q < NW; ++q) {
      float v = wmax[q];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float hi = fmaxf(top[j], v), lo = fminf(top[j], v);
        top[j] = hi, v = lo;
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (j == k - 1) L = top[j];
  }
  // the sum's terms use the oracle's expf (expf_ref), as the p values do:
  // with the hardware exp2 (__expf, a few ulp) a peaked row, whose S a few
  // terms dominate, took their errors straight into S's float rounding, and
  // 1 p in ~10^4 came out one fp16 ulp off (the random-shape sweep of
  // test_softmax_topk_random_shapes_exact)
  double se = 0.0;
  if constexpr (E >= 8) {
#pragma unroll
    for (int v = 0; v < E / 8; ++v)
      if (gv(v) < nvec)
#pragma unroll
        for (int e = 0; e < 8; ++e) se += (double)expf_ref(elem(v, e) - M);
  } else {
    // dwords eo/2 .. eo/2 + E/2 - 1 of local vector 0 (selects, no indexing)
    const int d0 = eo >> 1;
    auto dw = [&](int d) -> uint32_t {  // selects (a runtime array index would go to scratch)
      const uint32_t lo = (d & 1) ? r[0].y : r[0].x, hi = (d & 1) ? r[0].w : r[0].z;
      return (d & 2) ? hi : lo;
    };
    if (gv(0) < nvec)
#pragma unroll
      for (int q = 0; q < E / 2; ++q) {
        const uint32_t w = dw(d0 + q);
        se += (double)expf_ref(h2f_((uint16_t)(w & 0xffffu)) - M);
        se += (double)expf_ref(h2f_((uint16_t)(w >> 16)) - M);
      }
  }
  se = __ockl_wfred_add_f64(se);
  if (lane == 0) sh[wv] = se;
  __syncthreads();
  double sd = 0.0;
#pragma unroll
  for (int q = 0; q < NW; ++q) sd += sh[q];
  if constexpr (G > 1) {
    // (the guide's single-counter hand-off: agent-scope store of the bytes,
    // drained, then the add; the last adder reads them with agent-scope
    // loads after its add returned -- one load per lane, all in flight)
    if (wv == 0) {
      unsigned before = 0;
      if (lane == 0) {
        __hip_atomic_store(&part[(size_t)row * G + chunk], sd, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        before = __hip_atomic_fetch_add(&cnt[row], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      const int last = __shfl(before, 0) == (unsigned)(G - 1);
      if (last) {
        double pq = 0.0;
        if (lane < G)
          pq = __hip_atomic_load(&part[(size_t)row * G + lane], __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
        double tot = 0.0;
#pragma unroll
        for (int q = 0; q < G; ++q) tot += __shfl(pq, q);  // chunk order
        if (lane == 0) {
          __hip_atomic_store(&cnt[row], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          sh[NW] = tot;
        }
      }
      if (lane == 0) last_arrival = last;
    }
    __syncthreads();
    if (!last_arrival) return;
    sd = sh[NW];
  }
  const float S = (float)sd;
  // candidate threshold from p(L): its lower fp16 rounding boundary, minus a
  // margin of 2^-10 in x (>> the float error of exp, the division and log)
  // (finite: logits set to -inf -- taken ones -- are never candidates)
  float thr = -3.402823466e38f;
  {
    const uint16_t pL = f2h_(__fdiv_rn(expf_ref(L - M), S));
    if (pL > 1) {
      const float lo = 0.5f * (h2f_(pL) + h2f_((uint16_t)(pL - 1)));
      thr = M + logf(lo * S) - 0.0009765625f * fmaxf(1.0f, fabsf(M));
    }
  }
  // keys: (p + 1) << 32 | ~idx, 0 = not a candidate / taken
  auto key_of = [&](float xv, unsigned i) -> unsigned long long {
    const uint16_t p = f2h_(__fdiv_rn(expf_ref(xv - M), S));
    return ((unsigned long long)(p + 1u) << 32) | (unsigned long long)(0xffffffffu - i);
  };
  auto emit = [&](int rd, unsigned long long b) {
    ids[(size_t)row * k + rd] = (int)(0xffffffffu - (unsigned)(b & 0xffffffffu));
    if (ids2) ids2[(size_t)row * k + rd] = (int)(0xffffffffu - (unsigned)(b & 0xffffffffu));
    if (probs) probs[(size_t)row * k + rd] = h2f_((uint16_t)((b >> 32) - 1u));
  };
#pragma unroll
  for (int v = 0; v < NV; ++v)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float xv = elem(v, e);
      const unsigned i = (unsigned)(gv(v) * 8 + e);
      if (xv >= thr && (int)i < V) {
        const unsigned slot = atomicAdd(&ncand, 1u);
        if (slot < (unsigned)kCand) cand[slot] = key_of(xv, i);
      }
    }
  __syncthreads();
  const unsigned n = ncand;
  if (n <= (unsigned)kCand) {
    if (wv == 0) {  // keys are distinct (they hold the index)
      unsigned long long a = (unsigned)lane < n ? cand[lane] : 0ull;
      unsigned long long b = (unsigned)(lane + 64) < n ? cand[lane + 64] : 0ull;
      for (int rd = 0; rd < k; ++rd) {
        const unsigned long long best = __ockl_wfred_max_u64(a > b ? a : b);
        if (lane == 0) emit(rd, best);
        if (a == best) a = 0ull;
        if (b == best) b = 0ull;
      }
    }
    return;
  }
  // many candidates: k rounds of a workgroup-wide selection
  for (int rd = 0; rd < k; ++rd) {
    unsigned long long best = 0;
#pragma unroll
    for (int v = 0; v < NV; ++v)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float xv = elem(v, e);
        const unsigned i = (unsigned)(gv(v) * 8 + e);
        if (xv >= thr && (int)i < V) {
          const unsigned long long key = key_of(xv, i);
          best = key > best ? key : best;
        }
      }
    best = __ockl_wfred_max_u64(best);
    if (lane == 0) ksh[wv] = best;
    __syncthreads();
    unsigned long long b = ksh[0];
#pragma unroll
    for (int q = 1; q < NW; ++q) b = ksh[q] > b ? ksh[q] : b;
    __syncthreads();
    const unsigned idx = 0xffffffffu - (unsigned)(b & 0xffffffffu);
    if (tid == 0) emit(rd, b);
    if (rd + 1 < k && (idx >> 3) % TPB == (unsigned)tid) {  // owner marks it taken (-inf)
#pragma unroll
      for (int v = 0; v < NV; ++v)
        if ((unsigned)gv(v) == (idx >> 3)) {
          // (compile-time register indices only: a runtime-indexed store
          // into the row's registers would put it in scratch)
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            uint32_t &w = (&r[v].x)[e >> 1];
            const uint32_t m = (e & 1) ? 0xffff0000u : 0x0000ffffu;
            if ((unsigned)e == (idx & 7)) w = (w & ~m) | (0xfc00fc00u & m);
          }
        }
    }
  }
}

// softmax (fp16 output, softmax.cu:262-288) + ArgMax (argmax.cu:62-100) /
// ArgTopK (arg_topk.cu:339-448) for rows the register kernel does not take
// (a vocabulary not a multiple of 8, unaligned rows, V > 32768 such as
// LLaMA-3's 128256): the same rule -- p_i = half(exp(x_i - max) / S), S =
// float(double sum), (p desc, index asc) -- in three strided passes over the
// row (max and wave maxima, sum, candidates; the second and third hit L2),
// the candidate threshold and LDS list of softmax_topk_reg_kernel below, and
// k workgroup-wide rounds over the row only when more than kCand logits are
// candidates.
template <int TPB>
__global__ __launch_bounds__(TPB) void softmax_topk_kernel(
    const uint16_t *__restrict__ logits, int V, int k, int32_t *__restrict__ ids,
    float *__restrict__ probs, int32_t *__restrict__ ids2) {
  constexpr int NW = TPB / 64;
  constexpr int kCand = 128;
  __shared__ double sh[NW + 2];
  __shared__ unsigned long long cand[kCand];
  __shared__ unsigned ncand;
  float *fsh = reinterpret_cast<float *>(sh);
  unsigned long long *ksh = reinterpret_cast<unsigned long long *>(sh);
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint16_t *x = logits + (size_t)row * V;
  if (tid == 0) ncand = 0;
  float mx = -INFINITY;
  for (int i = tid; i < V; i += TPB) mx = fmaxf(mx, h2f_(x[i]));
  mx = __ockl_wfred_max_f32(mx);
  if (lane == 0) fsh[wv] = mx;
  __syncthreads();
  float wmax[NW];
#pragma unroll
  for (int q = 0; q < NW; ++q) wmax[q] = fsh[q];
  __syncthreads();
  float M = wmax[0];
#pragma unroll
  for (int q = 1; q < NW; ++q) M = fmaxf(M, wmax[q]);
  // L = k-th largest wave maximum: the waves' index sets are disjoint, so it
  // is a lower bound of the row's k-th largest logit
  float L = -INFINITY;
  {
    float top[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
    for (int q = 0; q < NW; ++q) {
      float v = wmax[q];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float hi = fmaxf(top[j], v), lo = fminf(top[j], v);
        top[j] = hi, v = lo;
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (j == k - 1) L = top[j];
  }
  double se = 0.0;
  for (int i = tid; i < V; i += TPB) se += (double)expf_ref(h2f_(x[i]) - M);
  se = __ockl_wfred_add_f64(se);
  if (lane == 0) sh[wv] = se;
  __syncthreads();
  double sd = 0.0;
#pragma unroll
  for (int q = 0; q < NW; ++q) sd += sh[q];
  const float S = (float)sd;
  float thr = -3.402823466e38f;
  {
    const uint16_t pL = f2h_(__fdiv_rn(expf_ref(L - M), S));
    if (pL > 1) {
      const float lo = 0.5f * (h2f_(pL) + h2f_((uint16_t)(pL - 1)));
      thr = M + logf(lo * S) - 0.0009765625f * fmaxf(1.0f, fabsf(M));
    }
  }
  auto key_of = [&](float xv, unsigned i) -> unsigned long long {
    const uint16_t p = f2h_(__fdiv_rn(expf_ref(xv - M), S));
    return ((unsigned long long)(p + 1u) << 32) | (unsigned long long)(0xffffffffu - i);
  };
  auto emit = [&](int rd, unsigned long long b) {
    ids[(size_t)row * k + rd] = (int)(0xffffffffu - (unsigned)(b & 0xffffffffu));
    if (ids2) ids2[(size_t)row * k + rd] = (int)(0xffffffffu - (unsigned)(b & 0xffffffffu));
    if (probs) probs[(size_t)row * k + rd] = h2f_((uint16_t)((b >> 32) - 1u));
  };
  for (int i = tid; i < V; i += TPB) {
    const float xv = h2f_(x[i]);
    if (xv >= thr) {
      const unsigned slot = atomicAdd(&ncand, 1u);
      if (slot < (unsigned)kCand) cand[slot] = key_of(xv, (unsigned)i);
    }
  }
  __syncthreads();
  const unsigned n = ncand;
  if (n <= (unsigned)kCand) {
    if (wv == 0) {
      unsigned long long a = (unsigned)lane < n ? cand[lane] : 0ull;
      unsigned long long b = (unsigned)(lane + 64) < n ? cand[lane + 64] : 0ull;
      for (int rd = 0; rd < k; ++rd) {
        const unsigned long long best = __ockl_wfred_max_u64(a > b ? a : b);
        if (lane == 0) emit(rd, best);
        if (a == best) a = 0ull;
        if (b == best) b = 0ull;
      }
    }
    return;
  }
  int chosen[4] = {-1, -1, -1, -1};
  for (int rd = 0; rd < k; ++rd) {
    unsigned long long best = 0;
    for (int i = tid; i < V; i += TPB) {
      const float xv = h2f_(x[i]);
      if (xv < thr) continue;
      bool taken = false;
#pragma unroll
      for (int q = 0; q < 4; ++q) taken |= (q < rd && chosen[q] == i);
      if (taken) continue;
      const unsigned long long key = key_of(xv, (unsigned)i);
      best = key > best ? key : best;
    }
    best = __ockl_wfred_max_u64(best);
    if (lane == 0) ksh[wv] = best;
    __syncthreads();
    unsigned long long b = ksh[0];
#pragma unroll
    for (int q = 1; q < NW; ++q) b = ksh[q] > b ? ksh[q] : b;
    __syncthreads();
    chosen[rd] = (int)(0xffffffffu - (unsigned)(b & 0xffffffffu));
    if (tid == 0) emit(rd, b);
  }
}

// split-row workspace: [kSplitRows] row counters at a FIXED offset (one
// workspace serves steps of every T: a counter must never share bytes with
// another T's partials), then [T][G <= 16] partial sums
constexpr int kSplitRows = 256;
constexpr size_t kSplitPartOff = kSplitRows * 4;
size_t argmax_workspace_bytes(int T) {
  return T <= 0 ? 0 : kSplitPartOff + (size_t)std::min(T, kSplitRows) * 16 * 8;
}

hipError_t launch_argmax(const uint16_t *logits, int T, int V, int k, int32_t *ids,
                         float *probs, hipStream_t s, void *ws, size_t ws_bytes, int32_t *ids2) {
  if (T <= 0) return hipSuccess;
  if (k < 1 || k > 4) return hipErrorInvalidValue;
  // workgroups per row (the split form needs the caller's zeroed workspace):
  // T x G <= 256, one workgroup per CU; FFMI_TOPK_SPLIT = 0 (off) / G (forced)
  static const int split_env = getenv("FFMI_TOPK_SPLIT") ? atoi(getenv("FFMI_TOPK_SPLIT")) : -1;
  // (T 129-256, the verify step's argmax, two workgroups per row with
  // FFMI_TOPK_SPLIT2=1: measured slower, 20.0 vs 13.1 us at T = 168 after the
  // lm_head GEMM -- 336 workgroups put two on many CUs -- and the verify step
  // 5.30 vs 5.28 ms; off)
  static const bool split2 = getenv("FFMI_TOPK_SPLIT2") && atoi(getenv("FFMI_TOPK_SPLIT2"));
  // (T <= 16 took 16 before: 8 measured 0.5 us faster at T = 8, k 1 and 3,
  // profiles/r06_topk_g.log)
  int G = T <= 32 ? 8 : T <= 64 ? 4 : T <= 128 ? 2 : (T <= kSplitRows && split2) ? 2 : 1;
  if (split_env >= 0) G = split_env;
  if (!ws || ws_bytes < argmax_workspace_bytes(T) || T > kSplitRows) G = 1;
  unsigned *cnt = reinterpret_cast<unsigned *>(ws);
  double *part = ws ? reinterpret_cast<double *>(static_cast<char *>(ws) + kSplitPartOff) : nullptr;
  // workgroup width (A/B: FFMI_TOPK_TPB = 256 / 512 / 1024)
  static const int tpb = [] {
    const char *e = getenv("FFMI_TOPK_TPB");
    const int v = e ? atoi(e) : 1024;
    return v == 256 || v == 512 ? v : 1024;
  }();
  const int nv = (V / 8 + tpb - 1) / tpb;
  // (NV = 8 at 1024 threads would spill: larger vocabularies take the loop kernel)
  if (V % 8 == 0 && ((uintptr_t)logits & 15) == 0 && nv * tpb <= 4096) {
#define FFMI_SMR(TPB, NV)                                                                  \
  hipLaunchKernelGGL((softmax_topk_reg_kernel<TPB, NV, 1>), dim3(T), dim3(TPB), 0, s, logits, V, \
                     k, ids, probs, nullptr, nullptr, ids2)
#define FFMI_SMG(NV, GG)                                                                     \
  hipLaunchKernelGGL((softmax_topk_reg_kernel<1024, NV, GG>), dim3(GG, T), dim3(1024), 0, s, \
                     logits, V, k, ids, probs, part, cnt, ids2)
    const int gmax = 4 * std::max(1, nv);  // >= 2 of a thread's 8 NV elements per workgroup
    while (G > 1 && (G > gmax || (G & (G - 1)))) G >>= 1;
    if (tpb == 1024 && G > 1) {
      if (nv <= 1) {
        if (G >= 4) FFMI_SMG(1, 4);
        else FFMI_SMG(1, 2);
      } else if (nv <= 2) {
        if (G >= 8) FFMI_SMG(2, 8);
        else if (G == 4) FFMI_SMG(2, 4);
        else FFMI_SMG(2, 2);
      } else {
        if (G >= 16) FFMI_SMG(4, 16);
        else if (G == 8) FFMI_SMG(4, 8);
        else if (G == 4) FFMI_SMG(4, 4);
        else FFMI_SMG(4, 2);
      }
    } else if (tpb == 256) {
      if (nv <= 4) FFMI_SMR(256, 4);
      else if (nv <= 8) FFMI_SMR(256, 8);
      else FFMI_SMR(256, 16);
    } else if (tpb == 512) {
      if (nv <= 2) FFMI_SMR(512, 2);
      else if (nv <= 4) FFMI_SMR(512, 4);
      else FFMI_SMR(512, 8);
    } else {
      if (nv <= 1) FFMI_SMR(1024, 1);
      else if (nv <= 2) FFMI_SMR(1024, 2);
      else FFMI_SMR(1024, 4);
    }
#undef FFMI_SMR
#undef FFMI_SMG
  } else {
    hipLaunchKernelGGL(softmax_topk_kernel<1024>, dim3(T), dim3(1024), 0, s, logits, V, k, ids, probs,
                       ids2);
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Vocab-sharded greedy / speculative tail (model.cc:3392-3419 shards lm_head
// over the vocabulary and Combines; here every rank keeps its [T][V/P] logit
// shard and three small exchanges of per-row records make the pick global):
//   phase 0: local max m_r                     -> exchange -> M = max_r m_r
//   phase 1: local sum of exp(x - M) (double)  -> exchange -> S = float(sum)
//   phase 2: local top-k of p = half(exp(x-M)/S) (p desc, lowest global id)
//            -> exchange -> merge: the k best of the P*k candidates.
// M and S are the unsharded kernel's values (a max is exact; S is the float
// rounding of the same double sum, accumulated per shard then over ranks in
// rank order), and p is computed with the same expressions, so the pick and
// its tie rule (lowest index of the largest fp16 p, cub ArgMax / the top-k
// heap) are those of the one-GPU kernel.  Exchange records are [P][T][W]
// floats: a rank writes its own slot and zeroes the others, and the sum
// all-reduce then acts as an all-gather (x + 0 = x).
// ---------------------------------------------------------------------------
template <int TPB>
__global__ __launch_bounds__(TPB) void vshard_kernel(const uint16_t *__restrict__ logits, int T,
                                                      int Vl, int P, int rank, int k, int phase,
                                                      float *__restrict__ xch, int W,
                                                      int32_t *__restrict__ ids,
                                                      float *__restrict__ probs) {
  constexpr int NW = TPB / 64;
  constexpr int kCand = 128;
  __shared__ double dsh[NW];
  __shared__ float fsh[NW];
  __shared__ unsigned long long ksh[NW];
  __shared__ unsigned long long cand[kCand];
  __shared__ unsigned ncand;
  const int t = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint16_t *x = logits + (size_t)t * Vl;
  auto slot = [&](int r) { return xch + ((size_t)r * T + t) * W; };
  if (phase == 3) {  // merge the P*k candidates of the last exchange
    if (tid == 0) {
      int taken[4] = {-1, -1, -1, -1};
      for (int rd = 0; rd < k; ++rd) {
        unsigned long long best = 0;
        int bq = -1;
        for (int r = 0; r < P; ++r)
          for (int j = 0; j < k; ++j) {
            const float pv = slot(r)[2 * j], iv = slot(r)[2 * j + 1];
            if (iv < 0.f) continue;  // (empty candidate)
            const int q = r * k + j;
            bool used = false;
            for (int z = 0; z < rd; ++z) used |= taken[z] == q;
            if (used) continue;
            const unsigned long long key =
                ((unsigned long long)(f2h_(pv) + 1u) << 32) |
                (unsigned long long)(0xffffffffu - (unsigned)iv);
            if (key > best) best = key, bq = q;
          }
        taken[rd] = bq;
        ids[(size_t)t * k + rd] = (int)(0xffffffffu - (unsigned)(best & 0xffffffffu));
        if (probs) probs[(size_t)t * k + rd] = h2f_((uint16_t)((best >> 32) - 1u));
      }
    }
    return;
  }
  float *own = slot(rank);
  if (phase == 0) {
    float m = -INFINITY;
    for (int i = tid; i < Vl; i += TPB) m = fmaxf(m, h2f_(x[i]));
    m = __ockl_wfred_max_f32(m);
    if (lane == 0) fsh[wv] = m;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < NW; ++q) m = fmaxf(m, fsh[q]);
    if (tid < P * W) {
      const int r = tid / W, w = tid % W;
      slot(r)[w] = (r == rank && w == 0) ? m : 0.f;
    }
    return;
  }
  float M = -INFINITY;
  for (int r = 0; r < P; ++r) M = fmaxf(M, xch[((size_t)r * T + t) * W]);  // phase-0 records
  if (phase == 1) {
    // (exchange buffer: [P][T][W] of phase 0 is read above and rewritten
    //  below only after the whole block has read it)
    double se = 0.0;
    for (int i = tid; i < Vl; i += TPB) se += (double)expf_ref(h2f_(x[i]) - M);
    se = __ockl_wfred_add_f64(se);
    if (lane == 0) dsh[wv] = se;
    __syncthreads();
    se = 0.0;
#pragma unroll
    for (int q = 0; q < NW; ++q) se += dsh[q];
    if (tid < P * W) {
      const int r = tid / W, w = tid % W;
      const float hi = (float)se, lo = (float)(se - (double)hi);
      slot(r)[w] = r != rank ? 0.f : (w == 0 ? M : w == 1 ? hi : w == 2 ? lo : 0.f);
    }
    return;
  }
  // phase 2: global S from the phase-1 records, local top-k candidates --
  // only logits whose fp16 p can reach the k-th largest local wave maximum's
  // p are evaluated (the threshold of softmax_topk_reg_kernel), through an
  // LDS list picked by one wave; k workgroup-wide rounds if it overflows
  double sd = 0.0;
  for (int r = 0; r < P; ++r) {
    const float *q = xch + ((size_t)r * T + t) * W;
    sd += (double)q[1] + (double)q[2];
  }
  const float S = (float)sd;
  if (tid == 0) ncand = 0;
  float wm = -INFINITY;
  for (int i = tid; i < Vl; i += TPB) wm = fmaxf(wm, h2f_(x[i]));
  wm = __ockl_wfred_max_f32(wm);
  if (lane == 0) fsh[wv] = wm;
  __syncthreads();  // (also: every thread has read the phase-1 records)
  float L = -INFINITY;
  {
    float top[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
    for (int q = 0; q < NW; ++q) {
      float v = fsh[q];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float hi = fmaxf(top[j], v), lo = fminf(top[j], v);
        top[j] = hi, v = lo;
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (j == k - 1) L = top[j];
  }
  float thr = -3.402823466e38f;
  {
    const uint16_t pL = f2h_(__fdiv_rn(expf_ref(L - M), S));
    if (pL > 1) {
      const float lo = 0.5f * (h2f_(pL) + h2f_((uint16_t)(pL - 1)));
      thr = M + logf(lo * S) - 0.0009765625f * fmaxf(1.0f, fabsf(M));
    }
  }
  auto key_of = [&](float xv, int i) -> unsigned long long {
    const uint16_t p = f2h_(__fdiv_rn(expf_ref(xv - M), S));
    const unsigned gi = (unsigned)(rank * Vl + i);
    return ((unsigned long long)(p + 1u) << 32) | (unsigned long long)(0xffffffffu - gi);
  };
  auto emit = [&](int rd, unsigned long long b) {
    own[2 * rd] = b ? h2f_((uint16_t)((b >> 32) - 1u)) : 0.f;
    own[2 * rd + 1] = b ? (float)(0xffffffffu - (unsigned)(b & 0xffffffffu)) : -1.f;
  };
  for (int i = tid; i < Vl; i += TPB) {
    const float xv = h2f_(x[i]);
    if (xv >= thr) {
      const unsigned sl = atomicAdd(&ncand, 1u);
      if (sl < (unsigned)kCand) cand[sl] = key_of(xv, i);
    }
  }
  __syncthreads();
  const unsigned n = ncand;
  if (n <= (unsigned)kCand) {
    if (wv == 0) {  // keys are distinct (they hold the index)
      unsigned long long a = (unsigned)lane < n ? cand[lane] : 0ull;
      unsigned long long b = (unsigned)(lane + 64) < n ? cand[lane + 64] : 0ull;
      for (int rd = 0; rd < k; ++rd) {
        const unsigned long long best = __ockl_wfred_max_u64(a > b ? a : b);
        if (lane == 0) emit(rd, best);
        if (best) {
          if (a == best) a = 0ull;
          if (b == best) b = 0ull;
        }
      }
    }
  } else {
    int chosen[4] = {-1, -1, -1, -1};
    for (int rd = 0; rd < k; ++rd) {
      unsigned long long best = 0;
      for (int i = tid; i < Vl; i += TPB) {
        const float xv = h2f_(x[i]);
        if (xv < thr) continue;
        bool used = false;
#pragma unroll
        for (int z = 0; z < 4; ++z) used |= (z < rd && chosen[z] == i);
        if (used) continue;
        const unsigned long long key = key_of(xv, i);
        best = key > best ? key : best;
      }
      best = __ockl_wfred_max_u64(best);
      if (lane == 0) ksh[wv] = best;
      __syncthreads();
      unsigned long long b = ksh[0];
#pragma unroll
      for (int q = 1; q < NW; ++q) b = ksh[q] > b ? ksh[q] : b;
      __syncthreads();
      chosen[rd] = b ? (int)(0xffffffffu - (unsigned)(b & 0xffffffffu)) - rank * Vl : -1;
      if (tid == 0) emit(rd, b);
    }
  }
  if (tid < P * W) {  // zero the other ranks' slots and this slot's unused tail
    const int r = tid / W, w = tid % W;
    if (r != rank) slot(r)[w] = 0.f;
    else if (w >= 2 * k) own[w] = 0.f;
  }
}

hipError_t launch_vshard(const uint16_t *logits, int T, int Vl, int P, int rank, int k,
                         int phase, float *xch, int W, int32_t *ids, float *probs,
                         hipStream_t s) {
  if (T <= 0) return hipSuccess;
  if (k < 1 || k > 4 || P * W > 256 || W < 2 * k || W < 4) return hipErrorInvalidValue;
  hipLaunchKernelGGL((vshard_kernel<1024>), dim3(T), dim3(1024), 0, s, logits, T, Vl, P, rank, k,
                     phase, xch, W, ids, probs);
  return hipGetLastError();
}

// Sum of the ranks' buffers of an in-process shard group (ffmi_comm_create_
// local): out = sum over r in rank order, fp16 accumulated in fp32 then
// rounded once (RCCL's ring sums in fp16 in ring order; both are within an
// fp16 ulp of the exact sum).
struct GroupBufs {
  const void *p[8];
};
__global__ void group_sum_kernel(GroupBufs b, int n, void *__restrict__ out, size_t count,
                                 int dtype) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < count;
       i += (size_t)gridDim.x * blockDim.x) {
    if (dtype == FFMI_F16) {
      float a = 0.f;
      for (int r = 0; r < n; ++r) a += h2f_(reinterpret_cast<const uint16_t *>(b.p[r])[i]);
      reinterpret_cast<uint16_t *>(out)[i] = f2h_(a);
    } else if (dtype == FFMI_F32) {
      float a = 0.f;
      for (int r = 0; r < n; ++r) a += reinterpret_cast<const float *>(b.p[r])[i];
      reinterpret_cast<float *>(out)[i] = a;
    } else {
      int a = 0;
      for (int r = 0; r < n; ++r) a += reinterpret_cast<const int *>(b.p[r])[i];
      reinterpret_cast<int *>(out)[i] = a;
    }
  }
}

hipError_t launch_group_sum(const void *const *bufs, int n, void *out, size_t count, int dtype,
                            hipStream_t s) {
  if (n < 1 || n > 8) return hipErrorInvalidValue;
  if (count == 0) return hipSuccess;
  GroupBufs b;
  for (int r = 0; r < 8; ++r) b.p[r] = bufs[r < n ? r : 0];
  size_t blocks = (count + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(group_sum_kernel, dim3((unsigned)blocks), dim3(256), 0, s, b, n, out, count,
                     dtype);
  return hipGetLastError();
}

}  // namespace ffmi
