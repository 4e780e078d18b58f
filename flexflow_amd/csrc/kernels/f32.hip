// f32.hip -- the full-precision path: the reference's --use-full-precision
// (inference/spec_infer/spec_infer.cc:102, incr_decoding.cc:77), i.e. every
// operator of the LLaMA graph on DT_FLOAT -- weights, activations, KV cache,
// softmax.  The same operators as the half path (gemm.hip, attention.hip,
// norm.hip), restated for fp32 operands:
//  * Linear on v_mfma_f32_16x16x4_f32 -- exact fp32: the result is a k-ordered
//    fmaf chain per (wave, k range), no reduced-precision inputs (gfx950 has
//    no xf32), k ranges of a workgroup summed in a fixed order;
//  * RMSNorm / ResidualRMSNorm with the sum of squares in fp64 (as the oracle,
//    then rounded once to fp32), fp32 residual adds;
//  * attention: one workgroup per (token, head) over the token's visible keys
//    (its prefix + its tree bits, the packed rule of attention.hip), fp32
//    scores, __expf-free softmax (expf), fp64 sum, 1/(sum + 1e-6)
//    (inc_multihead_self_attention.cu:532-547 on DT_FLOAT);
//  * softmax + argmax / arg-top-k on fp32 probabilities (softmax.cu:262-288,
//    argmax.cu:62-100, arg_topk.cu:339-448): lowest index among equal maxima.
// KV cache fp32, K[req][head][slot][d] and V[req][head][slot][d].
#include <stdlib.h>

#include <algorithm>

#include "../ffmi_internal.h"

namespace ffmi {

// ---------------------------------------------------------------------------
// Linear: Y[T][N] = X[T][K] . W[N][K]^T (linear_kernels.cu:450-582, DT_FLOAT)
// ---------------------------------------------------------------------------
// Workgroup = 4 waves arranged WM x WN x KS (KS: the k-blocks of 32 split
// over waves, summed through LDS in wave order).  A wave owns MT x NT output
// tiles of 16 x 16.  Operand map of v_mfma_f32_16x16x4_f32: lane l supplies
// A[row l&15][k l>>4] and B[k l>>4][col l&15]; each lane loads 16 B of X / W
// at k0 + 4*(l>>4) (+16), so MFMA j of a 16-k half takes element j: the four
// lane groups cover k0 + 4g + j, g = 0..3 -- all 16 k of the half.
template <int MT, int NT, int WM, int WN, int KS>
__global__ __launch_bounds__(256) void f32_gemm_kernel(const float *__restrict__ X,
                                                      const float *__restrict__ W,
                                                      float *__restrict__ Y, int T, int N, int K) {
  static_assert(WM * WN * KS == 4, "four waves");
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ks = wave % KS, wn = (wave / KS) % WN, wm = wave / (KS * WN);
  const int row0 = blockIdx.y * (WM * MT * 16) + wm * MT * 16;
  const int col0 = blockIdx.x * (WN * NT * 16) + wn * NT * 16;
  const int r = lane & 15, g = lane >> 4;
  const int nb = K >> 5;  // k-blocks of 32 (host-checked K % 32 == 0)
  const int kb0 = ks * nb / KS, kb1 = (ks + 1) * nb / KS;
  const float *xp[MT], *wp[NT];
#pragma unroll
  for (int m = 0; m < MT; ++m) xp[m] = X + (size_t)min(row0 + m * 16 + r, T - 1) * K + 4 * g;
#pragma unroll
  for (int n = 0; n < NT; ++n) wp[n] = W + (size_t)min(col0 + n * 16 + r, N - 1) * K + 4 * g;
  f4 acc[MT][NT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[m][n] = f4{0.f, 0.f, 0.f, 0.f};
  f4 a[2][MT][2], b[2][NT][2];  // double-buffered k-block operands
  auto load = [&](int buf, int kb) {
    const int k = kb * 32;
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      a[buf][m][0] = *reinterpret_cast<const f4 *>(xp[m] + k);
      a[buf][m][1] = *reinterpret_cast<const f4 *>(xp[m] + k + 16);
    }
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      b[buf][n][0] = *reinterpret_cast<const f4 *>(wp[n] + k);
      b[buf][n][1] = *reinterpret_cast<const f4 *>(wp[n] + k + 16);
    }
  };
  auto mma = [&](int buf) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
          for (int n = 0; n < NT; ++n)
            acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[buf][m][h][j], b[buf][n][h][j],
                                                             acc[m][n], 0, 0, 0);
  };
  if (kb0 < kb1) {
    load(0, kb0);
    int kb = kb0;
    for (; kb + 2 <= kb1; kb += 2) {  // next block in flight while this one multiplies
      load(1, kb + 1);
      mma(0);
      if (kb + 2 < kb1) load(0, kb + 2);
      mma(1);
    }
    if (kb < kb1) mma(0);
  }
  if constexpr (KS > 1) {
    // k ranges summed in wave order: ks 0 + 1 + 2 + 3 (fixed, deterministic)
    __shared__ f4 red[KS - 1][WM * WN][MT * NT][64];
    const int grp = wm * WN + wn;
    if (ks > 0)
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < NT; ++n) red[ks - 1][grp][m * NT + n][lane] = acc[m][n];
    __syncthreads();
    if (ks > 0) return;
#pragma unroll
    for (int s = 0; s < KS - 1; ++s)
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[m][n] += red[s][grp][m * NT + n][lane];
  }
  // C/D map: col = lane & 15, row = 4 * (lane >> 4) + i
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      const int col = col0 + n * 16 + r;
      if (col >= N) continue;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = row0 + m * 16 + 4 * g + i;
        if (row < T) Y[(size_t)row * N + col] = acc[m][n][i];
      }
    }
}

hipError_t launch_gemm_f32(const float *X, const float *W, float *Y, int T, int N, int K,
                           hipStream_t s) {
  if (T <= 0 || N <= 0) return hipSuccess;
  if (K <= 0 || K % 32) return hipErrorInvalidValue;
  if (T <= 16) {
    hipLaunchKernelGGL((f32_gemm_kernel<1, 1, 1, 1, 4>), dim3((N + 15) / 16, 1), dim3(256), 0, s, X, W,
                       Y, T, N, K);
  } else if (T <= 32) {
    hipLaunchKernelGGL((f32_gemm_kernel<2, 1, 1, 1, 4>), dim3((N + 15) / 16, 1), dim3(256), 0, s, X, W,
                       Y, T, N, K);
  } else if (T <= 64) {
    hipLaunchKernelGGL((f32_gemm_kernel<4, 1, 1, 1, 4>), dim3((N + 15) / 16, 1), dim3(256), 0, s, X, W,
                       Y, T, N, K);
  } else {
    // 64 x 64 output tile per wave, K split over the workgroup's 4 waves: per
    // MFMA half the operand bytes of 32 x 32 wave tiles at the same grid
    // (FFMI_F32_GEMM_TILE=1: the 2 x 2-wave, 32 x 32-per-wave form, A/B)
    static const bool tile = getenv("FFMI_F32_GEMM_TILE") && atoi(getenv("FFMI_F32_GEMM_TILE"));
    if (tile)
      hipLaunchKernelGGL((f32_gemm_kernel<2, 2, 2, 2, 1>), dim3((N + 63) / 64, (T + 63) / 64),
                         dim3(256), 0, s, X, W, Y, T, N, K);
    else
      hipLaunchKernelGGL((f32_gemm_kernel<4, 4, 1, 1, 4>), dim3((N + 63) / 64, (T + 63) / 64),
                         dim3(256), 0, s, X, W, Y, T, N, K);
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// block reductions (256 threads)
// ---------------------------------------------------------------------------
template <class V, class Op>
__device__ __forceinline__ V block_reduce256(V v, V *sh, Op op) {
  // fixed order: lanes pairwise by xor within the wave, then waves 0..3
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = op(v, __shfl_xor(v, off));
  const int w = threadIdx.x >> 6;
  __syncthreads();  // sh may still be read from the previous reduction
  if ((threadIdx.x & 63) == 0) sh[w] = v;
  __syncthreads();
  V t = sh[0];
  for (int i = 1; i < (int)(blockDim.x >> 6); ++i) t = op(t, sh[i]);
  return t;
}

// ---------------------------------------------------------------------------
// RMSNorm / ResidualRMSNorm (rms_norm_kernels.cu:97-124,
// residual_rms_norm_kernels.cu:98-131) on fp32: r = x1 (+ x2); rms =
// 1/sqrt(sum(r^2)/H + eps) (sum in fp64, rounded once); out = (r * rms) * w.
// gather (layer 0): x1 is the embedding table, row t = the token's row
// (embedding_kernels.cu:233-244), res_out gets the looked-up row.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void f32_rmsnorm_kernel(
    const float *x1, const float *__restrict__ x2, const float *__restrict__ w, float *res_out,
    float *__restrict__ out, int H, float eps, const char *__restrict__ gather) {
  __shared__ double sh[4];
  const int row = blockIdx.x;
  const float *a = gather ? x1 + (size_t)batch_view(gather).tokens[row].token_id * H
                          : x1 + (size_t)row * H;
  const float *b = x2 ? x2 + (size_t)row * H : nullptr;
  double ss = 0.0;
  for (int j = threadIdx.x; j < H; j += blockDim.x) {
    const float v = b ? __fadd_rn(a[j], b[j]) : a[j];
    if (res_out) res_out[(size_t)row * H + j] = v;
    ss += (double)v * (double)v;
  }
  ss = block_reduce256(ss, sh, [](double p, double q) { return p + q; });
  const float sum = (float)ss;
  // sqrtf: the correctly rounded square root (HIP's __fsqrt_rn is the native
  // v_sqrt_f32, ~1 ulp, unless OCML_BASIC_ROUNDED_OPERATIONS is defined)
  const float rms = __fdiv_rn(1.0f, sqrtf(__fadd_rn(__fdiv_rn(sum, (float)H), eps)));
  // (res_out may alias x1: read back this thread's own sums, never x1 + x2 again)
  for (int j = threadIdx.x; j < H; j += blockDim.x) {
    const float v = res_out ? res_out[(size_t)row * H + j] : (b ? __fadd_rn(a[j], b[j]) : a[j]);
    out[(size_t)row * H + j] = __fmul_rn(__fmul_rn(v, rms), w[j]);
  }
}

hipError_t launch_rmsnorm_f32(const float *x1, const float *x2, const float *w, float *res_out,
                              float *out, int T, int H, float eps, hipStream_t s,
                              const char *gather) {
  if (T <= 0) return hipSuccess;
  hipLaunchKernelGGL(f32_rmsnorm_kernel, dim3(T), dim3(256), 0, s, x1, x2, w, res_out, out, H,
                     eps, gather);
  return hipGetLastError();
}

// SigmoidSiluMulti (sigmoid_silu_multi.cu:37-47) on fp32: out[t][f] =
// (a * sigmoid(a)) * b with a = A[t*lda + f], b = B[t*ldb + f] (the model's
// [T][2F] gate|up product: B = A + F, lda = ldb = 2F)
__global__ void f32_silu_mul_kernel(const float *__restrict__ A, const float *__restrict__ B,
                                    float *__restrict__ out, int T, int F, size_t lda,
                                    size_t ldb) {
  const size_t n = (size_t)T * F;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    const size_t t = i / F, f = i % F;
    const float a = A[t * lda + f], b = B[t * ldb + f];
    const float sg = __fdiv_rn(1.0f, __fadd_rn(1.0f, expf(-a)));
    out[i] = __fmul_rn(__fmul_rn(a, sg), b);
  }
}

hipError_t launch_silu_mul_f32(const float *A, const float *B, float *out, int T, int F,
                               size_t lda, size_t ldb, hipStream_t s) {
  if (T <= 0 || F <= 0) return hipSuccess;
  const size_t n = (size_t)T * F;
  const unsigned blocks = (unsigned)std::min<size_t>((n + 255) / 256, 65536);
  hipLaunchKernelGGL(f32_silu_mul_kernel, dim3(blocks), dim3(256), 0, s, A, B, out, T, F, lda,
                     ldb);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// KV update: RoPE (apply_rotary_embedding_hf, inc...cu:664-738: pair
// (i, i + d/2), products rounded then summed) on q and k, K/V stored at the
// token's cache slot, and -- TREE -- the rotated k / v staged in row t for the
// next step's commits (tree_inc...cu:335-396 reads them).  Grid (T, heads),
// d/2 threads.
// ---------------------------------------------------------------------------
__global__ void f32_kv_update_kernel(const char *__restrict__ blob, const float *__restrict__ qkv,
                                     const float *__restrict__ rope, int max_rope_pos,
                                     float *__restrict__ qbuf, float *__restrict__ kc,
                                     float *__restrict__ vc, float *__restrict__ stage, int heads,
                                     int d, int slots) {
  const int t = blockIdx.x, hd = blockIdx.y, i = threadIdx.x, half = d / 2;
  if (i >= half) return;
  const BatchView bv = batch_view(blob);
  const ffmi_token_info tk = bv.tokens[t];
  const int Hl = heads * d;
  const float *row = qkv + (size_t)t * 3 * Hl + hd * d;
  const int p = min(max(tk.pos, 0), max_rope_pos - 1);
  const float c = rope[((size_t)p * half + i) * 2], sn = rope[((size_t)p * half + i) * 2 + 1];
  const float qa = row[i], qb = row[i + half];
  const float ka = row[Hl + i], kb = row[Hl + i + half];
  const float va = row[2 * Hl + i], vb = row[2 * Hl + i + half];
  const float q0 = __fsub_rn(__fmul_rn(qa, c), __fmul_rn(qb, sn));
  const float q1 = __fadd_rn(__fmul_rn(qa, sn), __fmul_rn(qb, c));
  const float k0 = __fsub_rn(__fmul_rn(ka, c), __fmul_rn(kb, sn));
  const float k1 = __fadd_rn(__fmul_rn(ka, sn), __fmul_rn(kb, c));
  float *qo = qbuf + (size_t)t * Hl + hd * d;
  qo[i] = q0;
  qo[i + half] = q1;
  if (tk.store_slot >= 0 && tk.store_slot < slots) {
    const size_t base = (((size_t)tk.req * heads + hd) * slots + tk.store_slot) * d;
    kc[base + i] = k0;
    kc[base + i + half] = k1;
    vc[base + i] = va;
    vc[base + i + half] = vb;
  }
  if (stage) {
    float *st = stage + (size_t)t * 2 * Hl + hd * d;
    st[i] = k0;
    st[i + half] = k1;
    st[Hl + i] = va;
    st[Hl + i + half] = vb;
  }
}

// commit_tokens_kernel (tree_inc...cu:335-396): accepted tokens of the
// previous verify batch move from their staging row to their depth slot
__global__ void f32_commit_kernel(const char *__restrict__ blob, const float *__restrict__ stage,
                                  float *__restrict__ kc, float *__restrict__ vc, int heads, int d,
                                  int slots) {
  const int ci = blockIdx.x, hd = blockIdx.y;
  const BatchView bv = batch_view(blob);
  const ffmi_commit_info cm = bv.commits[ci];
  if (cm.depth < 0 || cm.depth >= slots) return;
  const int Hl = heads * d;
  const float *st = stage + (size_t)cm.src_token * 2 * Hl + hd * d;
  const size_t base = (((size_t)cm.req * heads + hd) * slots + cm.depth) * d;
  for (int i = threadIdx.x; i < d; i += blockDim.x) {
    kc[base + i] = st[i];
    vc[base + i] = st[Hl + i];
  }
}

hipError_t launch_kv_update_f32(const char *blob, int T, int C, const float *qkv, const float *rope,
                                int max_rope_pos, float *qbuf, float *kc, float *vc,
                                float *stage, int heads, int d, int slots, hipStream_t s) {
  // commits first (the reference's commit-then-store order), from the rows
  // the previous step staged; this step's stores then overwrite the stage
  if (C > 0) {
    if (!stage) return hipErrorInvalidValue;
    hipLaunchKernelGGL(f32_commit_kernel, dim3(C, heads), dim3(64), 0, s, blob, stage, kc, vc,
                       heads, d, slots);
  }
  if (T > 0)
    hipLaunchKernelGGL(f32_kv_update_kernel, dim3(T, heads), dim3(d / 2), 0, s, blob, qkv, rope,
                       max_rope_pos, qbuf, kc, vc, stage, heads, d, slots);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Attention of one (token, head): keys [0, prefix_len) plus the tree slots
// whose bit the token's visibility word holds (attention.hip key_visible);
// scores in LDS.  256 threads: d-wide output groups of 256/d threads split
// the keys, summed in group order.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void f32_attention_kernel(
    const char *__restrict__ blob, const float *__restrict__ qbuf, const float *__restrict__ kc,
    const float *__restrict__ vc, float *__restrict__ out, int heads, int d, int slots,
    float scale) {
  extern __shared__ float smem[];  // q [d] | partial outputs [256] | scores [slots]
  __shared__ float shf[4];
  __shared__ double shd[4];
  const int t = blockIdx.x, hd = blockIdx.y, tid = threadIdx.x;
  const BatchView bv = batch_view(blob);
  const ffmi_token_info tk = bv.tokens[t];
  const int Hl = heads * d;
  float *sq = smem, *spart = smem + d, *sc = smem + d + 256;
  for (int i = tid; i < d; i += blockDim.x) sq[i] = qbuf[(size_t)t * Hl + hd * d + i];
  int kv_end = max(tk.prefix_len, tk.tree_len > 0 ? tk.tree_base + tk.tree_len : 0);
  kv_end = min(kv_end, slots);
  __syncthreads();
  const float *K = kc + ((size_t)tk.req * heads + hd) * slots * d;
  const float *V = vc + ((size_t)tk.req * heads + hd) * slots * d;
  const float NEG = -3.402823466e38f;
  float mx = NEG;
  for (int j = tid; j < kv_end; j += blockDim.x) {
    const unsigned jj = (unsigned)(j - tk.tree_base);
    const bool vis = j < tk.prefix_len ||
                     (jj < (unsigned)tk.tree_len && ((tk.tree_vis >> (jj & 63)) & 1ull));
    float sv = NEG;
    if (vis) {
      const float *kr = K + (size_t)j * d;
      float acc = 0.f;
      for (int i = 0; i < d; i += 4) {
        const f4 kv = *reinterpret_cast<const f4 *>(kr + i);
#pragma unroll
        for (int e = 0; e < 4; ++e) acc = __fadd_rn(acc, __fmul_rn(sq[i + e], kv[e]));
      }
      sv = __fmul_rn(scale, acc);
      mx = fmaxf(mx, sv);
    }
    sc[j] = vis ? sv : __builtin_nanf("");  // NaN marks an invisible key
  }
  mx = block_reduce256(mx, shf, [](float p, float q) { return fmaxf(p, q); });
  double sum = 0.0;
  for (int j = tid; j < kv_end; j += blockDim.x) {
    const float sv = sc[j];
    const float e = sv == sv ? expf(__fsub_rn(sv, mx)) : 0.f;
    sc[j] = e;
    sum += (double)e;
  }
  sum = block_reduce256(sum, shd, [](double p, double q) { return p + q; });
  const float inv = __fdiv_rn(1.0f, __fadd_rn((float)sum, 1e-6f));
  // P.V: thread = (group gi, dim i), group gi takes keys gi, gi + G, ...
  const int G = blockDim.x / d, gi = tid / d, i = tid % d;
  float acc = 0.f;
  if (gi < G)
    for (int j = gi; j < kv_end; j += G) {
      const float e = sc[j];
      if (e != 0.f) acc = __fadd_rn(acc, __fmul_rn(__fmul_rn(e, inv), V[(size_t)j * d + i]));
    }
  spart[tid] = acc;
  __syncthreads();
  if (tid < d) {
    float o = spart[tid];
    for (int q = 1; q < G; ++q) o = __fadd_rn(o, spart[q * d + tid]);
    out[(size_t)t * Hl + hd * d + tid] = o;
  }
}

hipError_t launch_attention_f32(const char *blob, int T, const float *qbuf, const float *kc,
                                const float *vc, float *out, int heads, int d, int slots,
                                float scale, hipStream_t s) {
  if (T <= 0) return hipSuccess;
  const size_t lds = (size_t)(d + 256 + slots) * sizeof(float);
  if (lds > 64 * 1024 || (d != 32 && d != 64 && d != 128)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(f32_attention_kernel, dim3(T, heads), dim3(256), lds, s, blob, qbuf, kc, vc,
                     out, heads, d, slots, scale);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// softmax + argmax / arg-top-k on fp32 probabilities: p_i = expf(z_i - max) /
// (float)sum (sum in fp64); k rounds of a block arg-max under the order
// (p desc, index asc), each round taking the first element after the
// previous pick in that order (arg_topk.cu:208-330 ties: lower index first).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void f32_softmax_topk_kernel(const float *__restrict__ logits,
                                                               int V, int k,
                                                               int32_t *__restrict__ ids,
                                                               float *__restrict__ probs) {
  __shared__ float shf[16];
  __shared__ double shd[16];
  __shared__ float sp[16];
  __shared__ int si[16];
  const int t = blockIdx.x, tid = threadIdx.x, nw = blockDim.x >> 6;
  const float *z = logits + (size_t)t * V;
  float mx = -3.402823466e38f;
  for (int i = tid; i < V; i += blockDim.x) mx = fmaxf(mx, z[i]);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off));
  if ((tid & 63) == 0) shf[tid >> 6] = mx;
  __syncthreads();
  mx = shf[0];
  for (int w = 1; w < nw; ++w) mx = fmaxf(mx, shf[w]);
  double sum = 0.0;
  for (int i = tid; i < V; i += blockDim.x) sum += (double)expf(__fsub_rn(z[i], mx));
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) sum += __shfl_xor(sum, off);
  if ((tid & 63) == 0) shd[tid >> 6] = sum;
  __syncthreads();
  sum = shd[0];
  for (int w = 1; w < nw; ++w) sum += shd[w];
  const float s = (float)sum;
  float pprev = 3.402823466e38f;
  int iprev = -1;
  for (int r = 0; r < k; ++r) {
    float bp = -1.f;
    int bi = V;
    for (int i = tid; i < V; i += blockDim.x) {
      const float p = __fdiv_rn(expf(__fsub_rn(z[i], mx)), s);
      const bool after = p < pprev || (p == pprev && i > iprev);
      if (after && (p > bp || (p == bp && i < bi))) bp = p, bi = i;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const float op = __shfl_xor(bp, off);
      const int oi = __shfl_xor(bi, off);
      if (op > bp || (op == bp && oi < bi)) bp = op, bi = oi;
    }
    __syncthreads();  // sp / si of the previous round are consumed
    if ((tid & 63) == 0) sp[tid >> 6] = bp, si[tid >> 6] = bi;
    __syncthreads();
    bp = sp[0], bi = si[0];
    for (int w = 1; w < nw; ++w)
      if (sp[w] > bp || (sp[w] == bp && si[w] < bi)) bp = sp[w], bi = si[w];
    if (tid == 0) {
      ids[(size_t)t * k + r] = bi;
      probs[(size_t)t * k + r] = bp;
    }
    pprev = bp, iprev = bi;
  }
}

hipError_t launch_softmax_topk_f32(const float *logits, int T, int V, int k, int32_t *ids,
                                   float *probs, hipStream_t s) {
  if (T <= 0) return hipSuccess;
  if (k < 1 || k > V) return hipErrorInvalidValue;
  hipLaunchKernelGGL(f32_softmax_topk_kernel, dim3(T), dim3(1024), 0, s, logits, V, k, ids, probs);
  return hipGetLastError();
}

}  // namespace ffmi

// public kernel-level entries (include/ffmi.h)
extern "C" ffmi_status ffmi_linear_f32(const float *X, const float *W, float *Y, int T,
                                       int out_dim, int in_dim, ffmi_stream stream) {
  FFMI_CHECK(T >= 0 && out_dim > 0 && in_dim > 0, FFMI_ERR_INVALID);
  FFMI_CHECK(in_dim % 32 == 0, FFMI_ERR_UNSUPPORTED);
  FFMI_CHECK(T == 0 || (X && W && Y), FFMI_ERR_INVALID);
  FFMI_HIP(ffmi::launch_gemm_f32(X, W, Y, T, out_dim, in_dim, (hipStream_t)stream));
  return FFMI_OK;
}

extern "C" ffmi_status ffmi_rmsnorm_f32(const float *x, const float *w, float *out, int T, int H,
                                        float eps, ffmi_stream stream) {
  FFMI_CHECK(x && w && out && T >= 0 && H > 0, FFMI_ERR_INVALID);
  FFMI_HIP(ffmi::launch_rmsnorm_f32(x, nullptr, w, nullptr, out, T, H, eps, (hipStream_t)stream));
  return FFMI_OK;
}

extern "C" ffmi_status ffmi_residual_rmsnorm_f32(const float *x1, const float *x2, const float *w,
                                                 float *residual_out, float *out, int T, int H,
                                                 float eps, ffmi_stream stream) {
  FFMI_CHECK(x1 && x2 && w && residual_out && out && T >= 0 && H > 0, FFMI_ERR_INVALID);
  FFMI_HIP(ffmi::launch_rmsnorm_f32(x1, x2, w, residual_out, out, T, H, eps, (hipStream_t)stream));
  return FFMI_OK;
}

extern "C" ffmi_status ffmi_silu_mul_f32(const float *a, const float *b, float *out, size_t n,
                                         ffmi_stream stream) {
  FFMI_CHECK(a && b && out && n <= (size_t)INT32_MAX, FFMI_ERR_INVALID);
  FFMI_HIP(ffmi::launch_silu_mul_f32(a, b, out, 1, (int)n, n, n, (hipStream_t)stream));
  return FFMI_OK;
}

extern "C" ffmi_status ffmi_arg_topk_f32(const float *logits, int T, int V, int k, int32_t *ids,
                                         float *probs, ffmi_stream stream) {
  FFMI_CHECK(logits && ids && probs && T >= 0 && V > 0 && k >= 1 && k <= 4 && k <= V,
             FFMI_ERR_INVALID);
  FFMI_HIP(ffmi::launch_softmax_topk_f32(logits, T, V, k, ids, probs, (hipStream_t)stream));
  return FFMI_OK;
}
