// oracle.cc -- CPU restatement of the SpecInfer hot path (TEST INFRASTRUCTURE).
//
// See oracle.h for the contract.  Nothing in the product path (libffmi.so)
// links or calls this file.  Reference citations are file:line into
// hugolatendresse/FlexFlow @ 2025-01-17.
#include "oracle.h"

#include <immintrin.h>
#include <math.h>
#include <omp.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <memory>
#include <utility>
#include <vector>

// ----------------------------------------------------------------------------
// fp16 <-> fp32, round to nearest even (bit exact, subnormals kept)
// ----------------------------------------------------------------------------
extern "C" uint16_t orc_f2h(float f) {
  uint32_t x;
  memcpy(&x, &f, 4);
  uint32_t sign = (x >> 16) & 0x8000u;
  uint32_t a = x & 0x7fffffffu;
  if (a >= 0x7f800000u) {  // inf / nan
    return (uint16_t)(sign | 0x7c00u | (a > 0x7f800000u ? 0x200u : 0u));
  }
  if (a >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u);  // >= 65520 -> inf
  if (a < 0x38800000u) {                                    // half subnormal
    float af;
    memcpy(&af, &a, 4);
    float r = rintf(af * 16777216.0f);  // exact scale by 2^24, RNE
    return (uint16_t)(sign | (uint32_t)r);
  }
  uint32_t mant = a & 0x7fffffu;
  uint32_t e = (a >> 23) - 112u;  // rebias 127 -> 15
  uint32_t h = (e << 10) | (mant >> 13);
  uint32_t rem = mant & 0x1fffu;
  if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h++;
  return (uint16_t)(sign | h);
}

extern "C" float orc_h2f(uint16_t h) {
  uint32_t sign = ((uint32_t)h & 0x8000u) << 16;
  uint32_t e = (h >> 10) & 0x1fu;
  uint32_t m = h & 0x3ffu;
  uint32_t x;
  if (e == 0) {
    float v = (float)m * (1.0f / 16777216.0f);
    return sign ? -v : v;
  } else if (e == 31) {
    x = sign | 0x7f800000u | (m << 13);
  } else {
    x = sign | ((e + 112u) << 23) | (m << 13);
  }
  float f;
  memcpy(&f, &x, 4);
  return f;
}

extern "C" float orc_round16(float f) { return orc_h2f(orc_f2h(f)); }

static inline float R(float v, int fp16) { return fp16 ? orc_round16(v) : v; }

// ----------------------------------------------------------------------------
// Synthetic weights: counter-based splitmix64 keyed by the tensor name.
// The GPU generator (flexflow_amd/csrc/kernels/weights.hip) implements the
// identical spec, so oracle and GPU hold bit-identical weights.
// ----------------------------------------------------------------------------
static uint64_t fnv1a64(const char *s) {
  uint64_t h = 1469598103934665603ull;
  for (; *s; ++s) {
    h ^= (uint8_t)*s;
    h *= 1099511628211ull;
  }
  return h;
}

static inline uint64_t splitmix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// kind 0 / 1 as in oracle.h; kind ORC_WKIND_DEPTH | L: a residual-branch
// output matrix (o_proj, down_proj) of an L-layer model in the depth-scaled
// init, amp = 0.02*sqrt(3) / sqrt(2L) (computed here and by the GPU
// generator's host code with the same float operations)
extern "C" float orc_weight_amp(int kind) {
  if (kind == 1) return 0.1f;
  if (kind & ORC_WKIND_DEPTH) return 0.034641016f / sqrtf((float)(2 * (kind & 0xffff)));
  return 0.034641016f;  // 0.02*sqrt(3)
}

extern "C" void orc_gen_weight(const char *name, uint64_t seed, int kind,
                               size_t n, float *out) {
  orc_gen_weight_rows(name, seed, kind, n, 0, 1, 0, 1.0f, out);
}

// value i of a [rows][cols] tensor taken from element (perm(r), c) of the
// stream, perm(r) = (r * pa + pb) mod rows (cols == 0: the identity), the
// amplitude times `scale` (a power of two in every use: exact)
extern "C" void orc_gen_weight_rows(const char *name, uint64_t seed, int kind, size_t n,
                                    int cols, uint64_t pa, uint64_t pb, float scale,
                                    float *out) {
  const uint64_t key = seed ^ fnv1a64(name);
  const float center = kind == 1 ? 1.0f : 0.0f;
  const float amp = orc_weight_amp(kind) * scale;
  const uint64_t rows = cols > 0 ? n / cols : 1;
#pragma omp parallel for schedule(static)
  for (long i = 0; i < (long)n; ++i) {
    uint64_t src = (uint64_t)i;
    if (cols > 0) src = ((i / cols) * pa + pb) % rows * cols + i % cols;
    uint64_t x = splitmix64(key + (src + 1) * 0x9E3779B97F4A7C15ull);
    float u = (float)(x >> 40) * (1.0f / 16777216.0f);
    volatile float t = 2.0f * u - 1.0f;  // exact
    volatile float p = t * amp;           // one rounding
    out[i] = center + p;                  // one rounding
  }
}

// ----------------------------------------------------------------------------
// Kernel-level restatements
// ----------------------------------------------------------------------------

// Fixed-order fp32 dot: 8 interleaved partial sums combined pairwise.
[[maybe_unused]] static inline float dot8(const float *a, const float *b, int K) {
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int k = 0;
  for (; k + 8 <= K; k += 8)
    for (int j = 0; j < 8; ++j) s[j] += a[k + j] * b[k + j];
  for (; k < K; ++k) s[k & 7] += a[k] * b[k];
  return ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
}

// Reference fp16 compute type (fp16 == ORC_REF16): cublasGemmEx with
// compute_type = output_type = half (linear_kernels.cu:493-528; the prompt
// attention GEMMs likewise, inc_multihead_self_attention.cu:108-200).  The
// accumulator is a half; modelled as tensor-core MMA steps of g_ref_block
// products (fp16 x fp16 products are exact in fp32) summed in fp32 and added
// to the half accumulator with one rounding per step.  cuBLAS's kernel choice
// (k per MMA, split-K) is not pinned by anything the reference holds, so the
// block is a parameter (orc_set_ref_block; default 16 = mma.m16n8k16).
static int g_ref_block = 16;
extern "C" void orc_set_ref_block(int k) { g_ref_block = k > 0 ? k : 16; }

static inline float dot_ref16(const float *a, const float *b, int K) {
  float acc = 0.f;
  for (int k0 = 0; k0 < K; k0 += g_ref_block) {
    const int k1 = std::min(K, k0 + g_ref_block);
    float s = 0.f;
    for (int k = k0; k < k1; ++k) s += a[k] * b[k];
    acc = orc_round16(acc + s);
  }
  return acc;
}

// Summation-order variants of the fp32 dot (orc_set_dot_variant), tests
// only: v uses V = 2^v vectors of 8 interleaved partial sums (0 = dot8, the
// oracle's order; 1 = dot16; 2 = dot32): products k + 8i of each 8V-wide step
// go to vector i, the V vectors are combined as a pairwise tree, the k < 8V
// remainder goes on through vector 0, and the 8 lanes combine pairwise.  All
// are exact fp32 restatements of the same sum in different orders; running
// the model in several of them measures the drift that ANY change of fp32
// summation order produces (the noise floor a GPU/CPU comparison sits on).
static int g_dot_variant = 0;
extern "C" void orc_set_dot_variant(int v) { g_dot_variant = v >= 0 && v <= 2 ? v : 0; }

// One register tile of the blocked linear: RT activation rows x RN weight
// rows, V accumulator vectors per output, over k in [k0, k1) (a multiple of
// 8V steps); accumulators live in acc[t][n][V][8] between k-chunks, so every
// output still gets exactly its own V x 8 partial sums in k order.
template <int V, int RT, int RN>
static inline void lin_tile(const float *X, const float *W, int K, int k0, int k1,
                            float *acc, int accN) {
  __m256 a[RT][RN][V];
  for (int r = 0; r < RT; ++r)
    for (int j = 0; j < RN; ++j)
      for (int v = 0; v < V; ++v)
        a[r][j][v] = _mm256_load_ps(acc + (((size_t)r * accN + j) * V + v) * 8);
  for (int k = k0; k < k1; k += 8 * V) {
    for (int v = 0; v < V; ++v) {
      __m256 x[RT];
      for (int r = 0; r < RT; ++r) x[r] = _mm256_loadu_ps(X + (size_t)r * K + k + 8 * v);
      for (int j = 0; j < RN; ++j) {
        const __m256 w = _mm256_loadu_ps(W + (size_t)j * K + k + 8 * v);
        for (int r = 0; r < RT; ++r)
          a[r][j][v] = _mm256_add_ps(a[r][j][v], _mm256_mul_ps(x[r], w));
      }
    }
  }
  for (int r = 0; r < RT; ++r)
    for (int j = 0; j < RN; ++j)
      for (int v = 0; v < V; ++v)
        _mm256_store_ps(acc + (((size_t)r * accN + j) * V + v) * 8, a[r][j][v]);
}

// The same tile with AVX-512 (the GPU boxes' EPYC hosts have it; chosen at
// run time).  Bit-identical: every lane sees the same products added in the
// same order.  V = 1: a zmm holds the 8-lane sums of TWO activation rows at
// one weight row (rows r, r+1 in its halves, the weight chunk broadcast);
// V >= 2: an output's V 8-lane vectors are V/2 zmm of 16 consecutive k.
template <int V, int RT, int RN>
__attribute__((target("avx512f,avx512dq"))) static inline void lin_tile512(
    const float *X, const float *W, int K, int k0, int k1, float *acc, int accN) {
  if constexpr (V == 1) {
    static_assert(RT % 2 == 0, "row pairs");
    constexpr int RP = RT / 2;
    __m512 a[RP][RN];
    for (int p = 0; p < RP; ++p)
      for (int j = 0; j < RN; ++j) {
        const __m256 lo = _mm256_load_ps(acc + ((size_t)(2 * p) * accN + j) * 8);
        const __m256 hi = _mm256_load_ps(acc + ((size_t)(2 * p + 1) * accN + j) * 8);
        a[p][j] = _mm512_insertf32x8(_mm512_castps256_ps512(lo), hi, 1);
      }
    for (int k = k0; k < k1; k += 8) {
      __m512 x[RP];
      for (int p = 0; p < RP; ++p)
        x[p] = _mm512_insertf32x8(
            _mm512_castps256_ps512(_mm256_loadu_ps(X + (size_t)(2 * p) * K + k)),
            _mm256_loadu_ps(X + (size_t)(2 * p + 1) * K + k), 1);
      for (int j = 0; j < RN; ++j) {
        const __m512 w = _mm512_broadcast_f32x8(_mm256_loadu_ps(W + (size_t)j * K + k));
        for (int p = 0; p < RP; ++p) a[p][j] = _mm512_add_ps(a[p][j], _mm512_mul_ps(x[p], w));
      }
    }
    for (int p = 0; p < RP; ++p)
      for (int j = 0; j < RN; ++j) {
        _mm256_store_ps(acc + ((size_t)(2 * p) * accN + j) * 8, _mm512_castps512_ps256(a[p][j]));
        _mm256_store_ps(acc + ((size_t)(2 * p + 1) * accN + j) * 8,
                        _mm512_extractf32x8_ps(a[p][j], 1));
      }
  } else {
    constexpr int Z = V / 2;  // zmm per output
    __m512 a[RT][RN][Z];
    for (int r = 0; r < RT; ++r)
      for (int j = 0; j < RN; ++j)
        for (int z = 0; z < Z; ++z)
          a[r][j][z] = _mm512_load_ps(acc + (((size_t)r * accN + j) * V + 2 * z) * 8);
    for (int k = k0; k < k1; k += 8 * V)
      for (int z = 0; z < Z; ++z) {
        __m512 x[RT];
        for (int r = 0; r < RT; ++r) x[r] = _mm512_loadu_ps(X + (size_t)r * K + k + 16 * z);
        for (int j = 0; j < RN; ++j) {
          const __m512 w = _mm512_loadu_ps(W + (size_t)j * K + k + 16 * z);
          for (int r = 0; r < RT; ++r) a[r][j][z] = _mm512_add_ps(a[r][j][z], _mm512_mul_ps(x[r], w));
        }
      }
    for (int r = 0; r < RT; ++r)
      for (int j = 0; j < RN; ++j)
        for (int z = 0; z < Z; ++z)
          _mm512_store_ps(acc + (((size_t)r * accN + j) * V + 2 * z) * 8, a[r][j][z]);
  }
}

static bool has_avx512() {
  static const int ok = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512dq") &&
                        !(getenv("ORC_NO_AVX512") && atoi(getenv("ORC_NO_AVX512")));
  return ok;
}

// Blocked Y = X . W^T with the dot order of variant log2(V): threads take
// blocks of NB weight rows; K is walked in chunks (L1/L2 reuse of both
// operands), the partial-sum vectors of the block's [T][NB] outputs kept in
// a per-thread buffer between chunks.
template <int V>
static void linear_blocked(const float *X, const float *W, float *Y, int T, int N, int K,
                           int fp16) {
  constexpr int NB = 16, KC = 512;
  constexpr int RT = 3, RN = V == 1 ? 4 : (V == 2 ? 2 : 1);
  const int Kv = K - K % (8 * V);  // main loop; the rest as in the scalar order
  const int nblk = (N + NB - 1) / NB;
  const bool avx = has_avx512();
#pragma omp parallel
  {
    float *acc = (float *)aligned_alloc(64, (size_t)std::max(T, 1) * NB * V * 8 * sizeof(float));
#pragma omp for schedule(dynamic, 4)
    for (int b = 0; b < nblk; ++b) {
      const int n0 = b * NB, nn = std::min(NB, N - n0);
      memset(acc, 0, (size_t)T * NB * V * 8 * sizeof(float));
      for (int kc = 0; kc < Kv; kc += KC) {
        const int k1 = std::min(Kv, kc + KC);
        int t = 0;
        if (avx) {  // register tiles of 8 rows (V = 1: 4 row pairs) x 5 / 4 / 2 weight rows
          constexpr int RT5 = 8, RN5 = V == 1 ? 5 : (V == 2 ? 3 : 1);
          for (; t + RT5 <= T; t += RT5) {
            int j = 0;
            for (; j + RN5 <= nn; j += RN5)
              lin_tile512<V, RT5, RN5>(X + (size_t)t * K, W + (size_t)(n0 + j) * K, K, kc, k1,
                                       acc + ((size_t)t * NB + j) * V * 8, NB);
            for (; j < nn; ++j)
              lin_tile512<V, RT5, 1>(X + (size_t)t * K, W + (size_t)(n0 + j) * K, K, kc, k1,
                                     acc + ((size_t)t * NB + j) * V * 8, NB);
          }
        }
        for (; t + RT <= T; t += RT) {
          int j = 0;
          for (; j + RN <= nn; j += RN)
            lin_tile<V, RT, RN>(X + (size_t)t * K, W + (size_t)(n0 + j) * K, K, kc, k1,
                                acc + ((size_t)t * NB + j) * V * 8, NB);
          for (; j < nn; ++j)
            lin_tile<V, RT, 1>(X + (size_t)t * K, W + (size_t)(n0 + j) * K, K, kc, k1,
                               acc + ((size_t)t * NB + j) * V * 8, NB);
        }
        for (; t < T; ++t)
          for (int j = 0; j < nn; ++j)
            lin_tile<V, 1, 1>(X + (size_t)t * K, W + (size_t)(n0 + j) * K, K, kc, k1,
                              acc + ((size_t)t * NB + j) * V * 8, NB);
      }
      for (int t = 0; t < T; ++t)
        for (int j = 0; j < nn; ++j) {
          const float *av = acc + ((size_t)t * NB + j) * V * 8;
          const float *x = X + (size_t)t * K, *w = W + (size_t)(n0 + j) * K;
          __m256 s8 = _mm256_load_ps(av);
          if (V == 2) s8 = _mm256_add_ps(s8, _mm256_load_ps(av + 8));
          if (V == 4)
            s8 = _mm256_add_ps(_mm256_add_ps(s8, _mm256_load_ps(av + 8)),
                               _mm256_add_ps(_mm256_load_ps(av + 16), _mm256_load_ps(av + 24)));
          int k = Kv;
          for (; k + 8 <= K; k += 8)
            s8 = _mm256_add_ps(s8, _mm256_mul_ps(_mm256_loadu_ps(x + k), _mm256_loadu_ps(w + k)));
          float s[8];
          _mm256_storeu_ps(s, s8);
          for (; k < K; ++k) s[k & 7] += x[k] * w[k];
          Y[(size_t)t * N + n0 + j] =
              R(((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7])), fp16);
        }
    }
    free(acc);
  }
}

// linear_kernels.cu:450-582 (cublasGemmEx OP_T/OP_N, out = in . W^T).
extern "C" void orc_linear(const float *X, const float *W, float *Y, int T,
                           int N, int K, int fp16) {
  if (fp16 == ORC_REF16) {
#pragma omp parallel for schedule(static)
    for (int n = 0; n < N; ++n)
      for (int t = 0; t < T; ++t)
        Y[(size_t)t * N + n] = dot_ref16(X + (size_t)t * K, W + (size_t)n * K, K);
    return;
  }
  if (T <= 0 || N <= 0) return;
  if (g_dot_variant == 1) linear_blocked<2>(X, W, Y, T, N, K, fp16);
  else if (g_dot_variant == 2) linear_blocked<4>(X, W, Y, T, N, K, fp16);
  else linear_blocked<1>(X, W, Y, T, N, K, fp16);
}

static void rms_core(const float *x, const float *w, float *out, int H,
                     float eps, int fp16) {
  double ss = 0.0;
  for (int j = 0; j < H; ++j) ss += (double)x[j] * (double)x[j];
  float sum = (float)ss;
  // rms stored as T (rms_norm_kernels.cu:114)
  float rms = R(1.0f / sqrtf(sum / (float)H + eps), fp16);
  for (int j = 0; j < H; ++j) {
    float y = R(x[j] * rms, fp16);  // Y = X * rms (half)
    out[j] = R(y * w[j], fp16);     // out = Y * w (half)
  }
}

// rms_norm_kernels.cu:97-124
extern "C" void orc_rmsnorm(const float *X, const float *w, float *out, int T,
                            int H, float eps, int fp16) {
  for (int t = 0; t < T; ++t)
    rms_core(X + (size_t)t * H, w, out + (size_t)t * H, H, eps, fp16);
}

// residual_rms_norm_kernels.cu:98-131: X_out = X1 + X2 (half), then norm
extern "C" void orc_residual_rmsnorm(const float *X1, const float *X2,
                                     const float *w, float *res_out, float *out,
                                     int T, int H, float eps, int fp16) {
  for (int t = 0; t < T; ++t) {
    const float *a = X1 + (size_t)t * H;
    const float *b = X2 + (size_t)t * H;
    float *r = res_out + (size_t)t * H;
    for (int j = 0; j < H; ++j) r[j] = R((float)((double)a[j] + (double)b[j]), fp16);
    rms_core(r, w, out + (size_t)t * H, H, eps, fp16);
  }
}

// sigmoid_silu_multi.cu:37-47: out = a * T(sigmoid(a)) * b, left to right
extern "C" void orc_silu_mul(const float *A, const float *B, float *out,
                             size_t n, int fp16) {
#pragma omp parallel for schedule(static)
  for (long i = 0; i < (long)n; ++i) {
    float a = A[i];
    float sg = 1.0f / (1.0f + expf(-a));
    float t = R(a * R(sg, fp16), fp16);
    out[i] = R(t * B[i], fp16);
  }
}

// RoPE table: freq = pos * (1.0 / pow(theta, 2i/d)) with the reference's
// float/double mix (inc_multihead_self_attention.cu:701-703), the llama3
// scaling branch in f32 (:704-722: its wavelength is 2*pi / freq of the
// already position-scaled freq), cos/sin in f32.
extern "C" void orc_rope_table_llama3(float *tab, int max_pos, int d, float theta, int llama3,
                                      float factor, float low_ff, float high_ff, int orig_max) {
  const int h = d / 2;
  std::vector<double> inv(h);
  for (int i = 0; i < h; ++i) {
    float ex = (float)2 * (float)i / (float)d;
    inv[i] = 1.0 / (double)powf(theta, ex);
  }
  const float pi = 3.141592654f;
  const float low_wl = llama3 ? (float)orig_max / low_ff : 0.f;
  const float high_wl = llama3 ? (float)orig_max / high_ff : 0.f;
  for (int p = 0; p < max_pos; ++p)
    for (int i = 0; i < h; ++i) {
      float freq = (float)((double)p * inv[i]);
      if (llama3) {
        float wavelen = 2 * pi / freq;
        if (wavelen < high_wl) {
        } else if (wavelen > low_wl) {
          freq = freq / factor;
        } else {
          float smooth = ((float)orig_max / wavelen - low_ff) / (high_ff - low_ff);
          freq = (1 - smooth) * freq / factor + smooth * freq;
        }
      }
      tab[((size_t)p * h + i) * 2 + 0] = cosf(freq);
      tab[((size_t)p * h + i) * 2 + 1] = sinf(freq);
    }
}

extern "C" void orc_rope_table(float *tab, int max_pos, int d, float theta) {
  orc_rope_table_llama3(tab, max_pos, d, theta, 0, 1.f, 1.f, 1.f, 1);
}

// apply_rotary_embedding_hf (inc_multihead_self_attention.cu:664-738):
// pair (i, i + d/2), complex multiply in f32, store as T.
static void rope_apply(float *x, int d, const float *cs) {
  const int h = d / 2;
  for (int i = 0; i < h; ++i) {
    float c = cs[2 * i], s = cs[2 * i + 1];
    float a = x[i], b = x[i + h];
    float ac = a * c, bs = b * s, as = a * s, bc = b * c;
    x[i] = ac - bs;
    x[i + h] = as + bc;
  }
}

extern "C" void orc_rope_head(float *x, int d, int pos, float theta, int fp16) {
  std::vector<float> tab((size_t)(pos + 1) * d);
  orc_rope_table(tab.data(), pos + 1, d, theta);
  rope_apply(x, d, tab.data() + (size_t)pos * d);
  for (int i = 0; i < d; ++i) x[i] = R(x[i], fp16);
}

// compute_attention_kernel_generation_kernel (inc_...cu:372-623) and the
// masked variants (tree_inc...cu:135-333, spec_inc...cu:130-300).
extern "C" void orc_attention_row(const float *q, const float *K,
                                  const float *V, const uint8_t *visible,
                                  int n_keys, int d, float scale, float *out,
                                  int fp16) {
  std::vector<float> p(n_keys > 0 ? n_keys : 1);
  float mx = -3.402823466e38f;
  for (int j = 0; j < n_keys; ++j) {
    if (!visible[j]) continue;
    const float *k = K + (size_t)j * d;
    float acc = 0.f;
    for (int i = 0; i < d; ++i) acc += q[i] * k[i];
    p[j] = scale * acc;
    mx = std::max(mx, p[j]);
  }
  double sum = 0.0;
  for (int j = 0; j < n_keys; ++j) {
    p[j] = visible[j] ? expf(p[j] - mx) : 0.f;
    sum += p[j];
  }
  float inv = 1.0f / ((float)sum + 1e-6f);
  for (int i = 0; i < d; ++i) out[i] = 0.f;
  for (int j = 0; j < n_keys; ++j) {
    if (!visible[j]) continue;
    float w = p[j] * inv;
    const float *v = V + (size_t)j * d;
    for (int i = 0; i < d; ++i) out[i] += w * v[i];
  }
  for (int i = 0; i < d; ++i) out[i] = R(out[i], fp16);
}

// Prompt-phase attention of IncMultiHeadSelfAttention / SpecInc
// (compute_attention_kernel_prompt, inc_multihead_self_attention.cu:98-366)
// for ONE head of one request: T_new queries at positions start..start+T_new-1
// against keys 0..start+T_new-1.
//   QK^T: cublasGemmStridedBatchedEx, half compute type, alpha = (DT)(1/sqrt d)
//         (:154-157) -> scores = half(alpha16 * acc16);
//   fill_entries_above_diagonal -> -inf (:222-236);
//   cudnnSoftmaxForward, half in/out (:238-262);
//   softmax . V: half compute type (:264-300), stored as half.
// q [T_new][d], K/V [nk][d] (half-representable), out [T_new][d].
extern "C" void orc_attention_prompt_ref16(const float *q, const float *K, const float *V,
                                           int T_new, int start, int d, float *out) {
  const int nk = start + T_new;
  const float alpha = orc_round16(1.0f / sqrtf((float)d));
  std::vector<float> sc(nk), pr(nk), vt((size_t)d * nk);
  for (int j = 0; j < nk; ++j)
    for (int i = 0; i < d; ++i) vt[(size_t)i * nk + j] = V[(size_t)j * d + i];
  for (int t = 0; t < T_new; ++t) {
    const int pos = start + t;
    float mx = -INFINITY;
    for (int j = 0; j <= pos; ++j) {
      sc[j] = orc_round16(alpha * dot_ref16(q + (size_t)t * d, K + (size_t)j * d, d));
      mx = std::max(mx, sc[j]);
    }
    double sum = 0.0;
    for (int j = 0; j < nk; ++j) {
      pr[j] = j <= pos ? expf(sc[j] - mx) : 0.f;
      sum += pr[j];
    }
    for (int j = 0; j < nk; ++j) pr[j] = orc_round16(pr[j] / (float)sum);
    for (int i = 0; i < d; ++i) out[(size_t)t * d + i] = dot_ref16(pr.data(), &vt[(size_t)i * nk], nk);
  }
}

// softmax over the vocab (softmax.cu:262-288; output stored as T), then the
// greedy pick (argmax.cu:62-100: first maximum).
static void softmax_row(const float *x, int V, int fp16, float *p) {
  float mx = -3.402823466e38f;
  for (int i = 0; i < V; ++i) mx = std::max(mx, x[i]);
  double sum = 0.0;
  for (int i = 0; i < V; ++i) {
    p[i] = expf(x[i] - mx);
    sum += p[i];
  }
  float s = (float)sum;
  for (int i = 0; i < V; ++i) p[i] = R(p[i] / s, fp16);
}

extern "C" void orc_softmax_argmax(const float *logits, int T, int V, int fp16,
                                   int *out_ids, float *out_prob) {
  std::vector<float> p(V);
  for (int t = 0; t < T; ++t) {
    softmax_row(logits + (size_t)t * V, V, fp16, p.data());
    int best = 0;
    for (int i = 1; i < V; ++i)
      if (p[i] > p[best]) best = i;
    out_ids[t] = best;
    if (out_prob) out_prob[t] = p[best];
  }
}

// arg_topk.cu:208-330: min-heap preferring higher index for eviction ->
// equal values keep the lower index; output sorted by value desc, index asc.
extern "C" void orc_softmax_topk(const float *logits, int T, int V, int k,
                                 int fp16, int *out_ids, float *out_probs) {
  std::vector<float> p(V);
  std::vector<int> idx(V);
  for (int t = 0; t < T; ++t) {
    softmax_row(logits + (size_t)t * V, V, fp16, p.data());
    for (int i = 0; i < V; ++i) idx[i] = i;
    std::partial_sort(idx.begin(), idx.begin() + k, idx.end(), [&](int a, int b) {
      return p[a] > p[b] || (p[a] == p[b] && a < b);
    });
    for (int j = 0; j < k; ++j) {
      out_ids[(size_t)t * k + j] = idx[j];
      if (out_probs) out_probs[(size_t)t * k + j] = p[idx[j]];
    }
  }
}

// ----------------------------------------------------------------------------
// Model-level restatement: LLaMA graph of inference/models/llama.cc:23-317
// (embedding -> [rms | residual_rms] -> qkv -> IncMHA -> o -> residual_rms
//  -> gate/up -> silu_mul -> down) x L -> residual_rms "norm" -> lm_head.
// ----------------------------------------------------------------------------
// std::vector whose resize() leaves floats uninitialised: the weights are
// generated in parallel right after, and a serial zero-fill of 27 GB (LLaMA-7B
// in fp32) took longer than generating them
template <class T>
struct DefaultInitAlloc : std::allocator<T> {
  template <class U>
  struct rebind {
    using other = DefaultInitAlloc<U>;
  };
  DefaultInitAlloc() = default;
  template <class U>
  DefaultInitAlloc(const DefaultInitAlloc<U> &) {}
  template <class U>
  void construct(U *p) noexcept {
    ::new ((void *)p) U;
  }
  template <class U, class... A>
  void construct(U *p, A &&...a) {
    ::new ((void *)p) U(std::forward<A>(a)...);
  }
};
using fvec = std::vector<float, DefaultInitAlloc<float>>;

struct orc_model {
  orc_config c;
  int fp16;
  int max_requests, max_seq;
  int d;
  fvec emb, lm, final_norm;
  struct Layer {
    fvec in_norm, post_norm, wq, wk, wv, wo, wg, wu, wd;
  };
  std::vector<Layer> layers;
  std::vector<float> kc, vc;  // [req][layer][pos][H]
  std::vector<float> rope;    // [max_seq][d/2][2]
  std::vector<std::vector<float>> hidden;  // debug: per-layer output of last call
  // per-op tensors of the last orc_model_forward_ex call, by FFMI_DBG_* kind
  // (include/ffmi.h: 2 attn_norm, 3 qkv (pre-RoPE [Q|K|V]), 4 attn_out,
  // 5 o_proj, 6 ffn_norm, 7 mlp_act, 8 down, 9 embed), [layer][T * width]
  std::vector<std::vector<float>> ops[10];
  int ops_T = 0;
};

static void keep_op(orc_model *m, int kind, int layer, const float *src, size_t n) {
  auto &v = m->ops[kind];
  if ((int)v.size() <= layer) v.resize(layer + 1);
  v[layer].assign(src, src + n);
}

static void gen(fvec &dst, const std::string &name, uint64_t seed,
                int kind, size_t n, int fp16, int cols = 0, uint64_t pa = 1, float scale = 1.0f) {
  dst.resize(n);
  orc_gen_weight_rows(name.c_str(), seed, kind, n, cols, pa, ORC_CHAIN_B, scale, dst.data());
  if (fp16) {
    float *p = dst.data();
#pragma omp parallel for schedule(static)
    for (long i = 0; i < (long)n; ++i) p[i] = orc_round16(p[i]);
  }
}

extern "C" orc_model *orc_model_create(const orc_config *cfg, uint64_t seed,
                                       int fp16, int max_requests, int max_seq) {
  return orc_model_create_ex(cfg, seed, fp16, max_requests, max_seq, 0);
}

extern "C" float orc_chain_embed_scale(int num_layers, int hidden, int intermediate) {
  const long long ref = 32LL * (4096 + 2 * 11008);  // LLaMA-7B
  const long long own = (long long)num_layers * (hidden + 2LL * intermediate);
  long long f2 = 1;  // (scale / 128)^2
  float s = 128.0f;
  while (f2 * ref < own) f2 *= 4, s *= 2.0f;
  return s;
}

extern "C" orc_model *orc_model_create_ex(const orc_config *cfg, uint64_t seed, int fp16,
                                          int max_requests, int max_seq, int weight_init) {
  if (cfg->num_kv_heads != cfg->num_heads) return nullptr;  // MHA only
  orc_model *m = new orc_model();
  m->c = *cfg;
  m->fp16 = fp16;
  m->max_requests = max_requests;
  m->max_seq = max_seq;
  m->d = cfg->hidden / cfg->num_heads;
  const size_t H = cfg->hidden, F = cfg->intermediate, Vv = cfg->vocab_size;
  if (weight_init == 2) {
    // token-chain init: embeddings x orc_chain_embed_scale, lm_head row v =
    // the unscaled embedding row of perm(v) (a tied, permuted head): the
    // residual stream keeps the input token's direction, so the logit of
    // perm^-1(token) leads by a margin far above fp16 rounding noise
    gen(m->emb, "model.embed_tokens.weight", seed, 0, Vv * H, fp16, 0, 1,
        orc_chain_embed_scale(cfg->num_layers, cfg->hidden, cfg->intermediate));
    gen(m->lm, "model.embed_tokens.weight", seed, 0, Vv * H, fp16, (int)H, ORC_CHAIN_A);
  } else {
    gen(m->emb, "model.embed_tokens.weight", seed, 0, Vv * H, fp16);
    gen(m->lm, "lm_head.weight", seed, 0, Vv * H, fp16);
  }
  gen(m->final_norm, "model.norm.weight", seed, 1, H, fp16);
  m->layers.resize(cfg->num_layers);
  for (int l = 0; l < cfg->num_layers; ++l) {
    std::string p = "model.layers." + std::to_string(l) + ".";
    auto &L = m->layers[l];
    gen(L.in_norm, p + "input_layernorm.weight", seed, 1, H, fp16);
    gen(L.post_norm, p + "post_attention_layernorm.weight", seed, 1, H, fp16);
    gen(L.wq, p + "self_attn.q_proj.weight", seed, 0, H * H, fp16);
    gen(L.wk, p + "self_attn.k_proj.weight", seed, 0, H * H, fp16);
    gen(L.wv, p + "self_attn.v_proj.weight", seed, 0, H * H, fp16);
    // depth-scaled init: the residual-branch outputs at 1/sqrt(2L)
    const int kres = weight_init == 1 ? (ORC_WKIND_DEPTH | cfg->num_layers) : 0;
    gen(L.wo, p + "self_attn.o_proj.weight", seed, kres, H * H, fp16);
    gen(L.wg, p + "mlp.gate_proj.weight", seed, 0, F * H, fp16);
    gen(L.wu, p + "mlp.up_proj.weight", seed, 0, F * H, fp16);
    gen(L.wd, p + "mlp.down_proj.weight", seed, kres, H * F, fp16);
  }
  m->kc.assign((size_t)max_requests * cfg->num_layers * max_seq * H, 0.f);
  m->vc.assign((size_t)max_requests * cfg->num_layers * max_seq * H, 0.f);
  m->rope.resize((size_t)max_seq * m->d);
  orc_rope_table(m->rope.data(), max_seq, m->d, cfg->rope_theta);
  m->hidden.resize(cfg->num_layers + 1);
  return m;
}

extern "C" void orc_model_destroy(orc_model *m) { delete m; }

extern "C" void orc_model_reset(orc_model *m, int req) {
  (void)m;
  (void)req;  // cache rows are overwritten position by position
}

extern "C" long orc_model_weight(orc_model *m, const char *name, float *out) {
  std::string n(name);
  const fvec *src = nullptr;
  if (n == "model.embed_tokens.weight") src = &m->emb;
  else if (n == "lm_head.weight") src = &m->lm;
  else if (n == "model.norm.weight") src = &m->final_norm;
  else if (n.rfind("model.layers.", 0) == 0) {
    int l = atoi(n.c_str() + 13);
    if (l < 0 || l >= m->c.num_layers) return -1;
    auto &L = m->layers[l];
    std::string rest = n.substr(n.find('.', 13) + 1);
    if (rest == "input_layernorm.weight") src = &L.in_norm;
    else if (rest == "post_attention_layernorm.weight") src = &L.post_norm;
    else if (rest == "self_attn.q_proj.weight") src = &L.wq;
    else if (rest == "self_attn.k_proj.weight") src = &L.wk;
    else if (rest == "self_attn.v_proj.weight") src = &L.wv;
    else if (rest == "self_attn.o_proj.weight") src = &L.wo;
    else if (rest == "mlp.gate_proj.weight") src = &L.wg;
    else if (rest == "mlp.up_proj.weight") src = &L.wu;
    else if (rest == "mlp.down_proj.weight") src = &L.wd;
  }
  if (!src) return -1;
  if (out) memcpy(out, src->data(), src->size() * sizeof(float));
  return (long)src->size();
}

extern "C" int orc_model_forward_ex(orc_model *m, int req, const int *tokens, int T,
                                    int start_pos, float *logits, int prompt_phase);
extern "C" int orc_model_forward(orc_model *m, int req, const int *tokens, int T,
                                 int start_pos, float *logits) {
  return orc_model_forward_ex(m, req, tokens, T, start_pos, logits, 0);
}

// prompt_phase != 0 with fp16 == ORC_REF16: the attention of these T tokens
// takes the reference's prompt path (orc_attention_prompt_ref16) instead of
// the generation kernel's fp32 softmax -- as IncMHA does for a request in its
// prompt phase (inc_multihead_self_attention.cu:944-985).
extern "C" int orc_model_forward_ex(orc_model *m, int req, const int *tokens, int T,
                                    int start_pos, float *logits, int prompt_phase) {
  const orc_config &c = m->c;
  const int H = c.hidden, F = c.intermediate, d = m->d, nh = c.num_heads;
  const int fp16 = m->fp16;
  if (req < 0 || req >= m->max_requests || start_pos + T > m->max_seq) return -1;
  std::vector<float> x((size_t)T * H), h((size_t)T * H), res((size_t)T * H);
  std::vector<float> q((size_t)T * H), k((size_t)T * H), v((size_t)T * H);
  std::vector<float> att((size_t)T * H), o((size_t)T * H), mlp((size_t)T * H);
  std::vector<float> g((size_t)T * F), u((size_t)T * F), a((size_t)T * F);
  for (int t = 0; t < T; ++t)
    memcpy(&x[(size_t)t * H], &m->emb[(size_t)tokens[t] * H], H * sizeof(float));
  m->ops_T = T;
  keep_op(m, 9, 0, x.data(), x.size());
  const float scale = 1.0f / sqrtf((float)d);
  for (int l = 0; l < c.num_layers; ++l) {
    auto &L = m->layers[l];
    if (l == 0) {
      res = x;
      orc_rmsnorm(res.data(), L.in_norm.data(), h.data(), T, H, c.rms_eps, fp16);
    } else {
      std::vector<float> r2((size_t)T * H);
      orc_residual_rmsnorm(res.data(), mlp.data(), L.in_norm.data(), r2.data(),
                           h.data(), T, H, c.rms_eps, fp16);
      res.swap(r2);
    }
    keep_op(m, 2, l, h.data(), h.size());
    orc_linear(h.data(), L.wq.data(), q.data(), T, H, H, fp16);
    orc_linear(h.data(), L.wk.data(), k.data(), T, H, H, fp16);
    orc_linear(h.data(), L.wv.data(), v.data(), T, H, H, fp16);
    {
      std::vector<float> qkv3((size_t)T * 3 * H);
      for (int t = 0; t < T; ++t) {
        memcpy(&qkv3[(size_t)t * 3 * H], &q[(size_t)t * H], H * sizeof(float));
        memcpy(&qkv3[(size_t)t * 3 * H + H], &k[(size_t)t * H], H * sizeof(float));
        memcpy(&qkv3[(size_t)t * 3 * H + 2 * H], &v[(size_t)t * H], H * sizeof(float));
      }
      keep_op(m, 3, l, qkv3.data(), qkv3.size());
    }
    float *kc = &m->kc[(((size_t)req * c.num_layers + l) * m->max_seq) * H];
    float *vc = &m->vc[(((size_t)req * c.num_layers + l) * m->max_seq) * H];
    for (int t = 0; t < T; ++t) {
      int pos = start_pos + t;
      for (int hd = 0; hd < nh; ++hd) {
        float *qh = &q[(size_t)t * H + hd * d];
        float *kh = &k[(size_t)t * H + hd * d];
        rope_apply(qh, d, &m->rope[(size_t)pos * d]);
        rope_apply(kh, d, &m->rope[(size_t)pos * d]);
        for (int i = 0; i < d; ++i) {
          qh[i] = R(qh[i], fp16);
          kh[i] = R(kh[i], fp16);
        }
      }
      memcpy(kc + (size_t)pos * H, &k[(size_t)t * H], H * sizeof(float));
      memcpy(vc + (size_t)pos * H, &v[(size_t)t * H], H * sizeof(float));
    }
    const int nk = start_pos + T;
#pragma omp parallel
    {
      std::vector<float> Kh((size_t)nk * d), Vh((size_t)nk * d);
      std::vector<uint8_t> vis(nk);
#pragma omp for schedule(static)
      for (int hd = 0; hd < nh; ++hd) {
        for (int j = 0; j < nk; ++j) {
          memcpy(&Kh[(size_t)j * d], kc + (size_t)j * H + hd * d, d * sizeof(float));
          memcpy(&Vh[(size_t)j * d], vc + (size_t)j * H + hd * d, d * sizeof(float));
        }
        if (prompt_phase && fp16 == ORC_REF16) {
          std::vector<float> qh((size_t)T * d), oh((size_t)T * d);
          for (int t = 0; t < T; ++t)
            memcpy(&qh[(size_t)t * d], &q[(size_t)t * H + hd * d], d * sizeof(float));
          orc_attention_prompt_ref16(qh.data(), Kh.data(), Vh.data(), T, start_pos, d, oh.data());
          for (int t = 0; t < T; ++t)
            memcpy(&att[(size_t)t * H + hd * d], &oh[(size_t)t * d], d * sizeof(float));
          continue;
        }
        for (int t = 0; t < T; ++t) {
          int pos = start_pos + t;
          for (int j = 0; j < nk; ++j) vis[j] = j <= pos;
          orc_attention_row(&q[(size_t)t * H + hd * d], Kh.data(), Vh.data(),
                            vis.data(), nk, d, scale, &att[(size_t)t * H + hd * d], fp16);
        }
      }
    }
    keep_op(m, 4, l, att.data(), att.size());
    orc_linear(att.data(), L.wo.data(), o.data(), T, H, H, fp16);
    keep_op(m, 5, l, o.data(), o.size());
    {
      std::vector<float> r2((size_t)T * H);
      orc_residual_rmsnorm(res.data(), o.data(), L.post_norm.data(), r2.data(),
                           h.data(), T, H, c.rms_eps, fp16);
      res.swap(r2);
    }
    keep_op(m, 6, l, h.data(), h.size());
    orc_linear(h.data(), L.wg.data(), g.data(), T, F, H, fp16);
    orc_linear(h.data(), L.wu.data(), u.data(), T, F, H, fp16);
    orc_silu_mul(g.data(), u.data(), a.data(), (size_t)T * F, fp16);
    keep_op(m, 7, l, a.data(), a.size());
    orc_linear(a.data(), L.wd.data(), mlp.data(), T, H, F, fp16);
    keep_op(m, 8, l, mlp.data(), mlp.size());
    // debug: residual stream entering the next layer (= res + mlp)
    auto &dbg = m->hidden[l];
    dbg.resize((size_t)T * H);
    for (size_t i = 0; i < dbg.size(); ++i) dbg[i] = R(res[i] + mlp[i], fp16);
  }
  std::vector<float> r2((size_t)T * H);
  orc_residual_rmsnorm(res.data(), mlp.data(), m->final_norm.data(), r2.data(),
                       h.data(), T, H, c.rms_eps, fp16);
  m->hidden[c.num_layers] = h;
  if (logits)
    orc_linear(h.data(), m->lm.data(), logits, T, c.vocab_size, H, fp16);
  return 0;
}

extern "C" int orc_model_decode_batch(orc_model *m, const int *reqs, const int *tokens,
                                      const int *pos, int T, float *logits) {
  const orc_config &c = m->c;
  const int H = c.hidden, F = c.intermediate, d = m->d, nh = c.num_heads;
  const int fp16 = m->fp16;
  for (int t = 0; t < T; ++t)
    if (reqs[t] < 0 || reqs[t] >= m->max_requests || pos[t] >= m->max_seq) return -1;
  std::vector<float> res((size_t)T * H), h((size_t)T * H), r2((size_t)T * H);
  std::vector<float> q((size_t)T * H), k((size_t)T * H), v((size_t)T * H);
  std::vector<float> att((size_t)T * H), o((size_t)T * H), mlp((size_t)T * H);
  std::vector<float> g((size_t)T * F), u((size_t)T * F), a((size_t)T * F);
  for (int t = 0; t < T; ++t)
    memcpy(&res[(size_t)t * H], &m->emb[(size_t)tokens[t] * H], H * sizeof(float));
  const float scale = 1.0f / sqrtf((float)d);
  for (int l = 0; l < c.num_layers; ++l) {
    auto &L = m->layers[l];
    if (l == 0) {
      orc_rmsnorm(res.data(), L.in_norm.data(), h.data(), T, H, c.rms_eps, fp16);
    } else {
      orc_residual_rmsnorm(res.data(), mlp.data(), L.in_norm.data(), r2.data(), h.data(), T,
                           H, c.rms_eps, fp16);
      res.swap(r2);
    }
    orc_linear(h.data(), L.wq.data(), q.data(), T, H, H, fp16);
    orc_linear(h.data(), L.wk.data(), k.data(), T, H, H, fp16);
    orc_linear(h.data(), L.wv.data(), v.data(), T, H, H, fp16);
#pragma omp parallel for schedule(static)
    for (int t = 0; t < T; ++t) {
      const int req = reqs[t], p = pos[t];
      float *kc = &m->kc[(((size_t)req * c.num_layers + l) * m->max_seq) * H];
      float *vc = &m->vc[(((size_t)req * c.num_layers + l) * m->max_seq) * H];
      for (int hd = 0; hd < nh; ++hd) {
        float *qh = &q[(size_t)t * H + hd * d];
        float *kh = &k[(size_t)t * H + hd * d];
        rope_apply(qh, d, &m->rope[(size_t)p * d]);
        rope_apply(kh, d, &m->rope[(size_t)p * d]);
        for (int i = 0; i < d; ++i) {
          qh[i] = R(qh[i], fp16);
          kh[i] = R(kh[i], fp16);
        }
      }
      memcpy(kc + (size_t)p * H, &k[(size_t)t * H], H * sizeof(float));
      memcpy(vc + (size_t)p * H, &v[(size_t)t * H], H * sizeof(float));
      std::vector<float> Kh((size_t)(p + 1) * d), Vh((size_t)(p + 1) * d);
      std::vector<uint8_t> vis(p + 1, 1);
      for (int hd = 0; hd < nh; ++hd) {
        for (int j = 0; j <= p; ++j) {
          memcpy(&Kh[(size_t)j * d], kc + (size_t)j * H + hd * d, d * sizeof(float));
          memcpy(&Vh[(size_t)j * d], vc + (size_t)j * H + hd * d, d * sizeof(float));
        }
        orc_attention_row(&q[(size_t)t * H + hd * d], Kh.data(), Vh.data(), vis.data(), p + 1,
                          d, scale, &att[(size_t)t * H + hd * d], fp16);
      }
    }
    orc_linear(att.data(), L.wo.data(), o.data(), T, H, H, fp16);
    orc_residual_rmsnorm(res.data(), o.data(), L.post_norm.data(), r2.data(), h.data(), T, H,
                         c.rms_eps, fp16);
    res.swap(r2);
    orc_linear(h.data(), L.wg.data(), g.data(), T, F, H, fp16);
    orc_linear(h.data(), L.wu.data(), u.data(), T, F, H, fp16);
    orc_silu_mul(g.data(), u.data(), a.data(), (size_t)T * F, fp16);
    orc_linear(a.data(), L.wd.data(), mlp.data(), T, H, F, fp16);
  }
  orc_residual_rmsnorm(res.data(), mlp.data(), m->final_norm.data(), r2.data(), h.data(), T, H,
                       c.rms_eps, fp16);
  if (logits) orc_linear(h.data(), m->lm.data(), logits, T, c.vocab_size, H, fp16);
  return 0;
}

// Several requests' token blocks in one step (the CPU port of a tree-verify
// or SSM beam step for the cpu_baseline timing): the dense layers run once
// over all tokens (every weight read once per step, as the GPU step does),
// attention per request over its cache with causal visibility inside the
// block -- for a 21-token verify tree or a 3-token beam layer the same work
// as the reference's bitmask (tree_inc...cu:35-333, spec_inc...cu:36-309).
extern "C" int orc_model_forward_multi(orc_model *m, int nreq, const int *reqs, const int *counts,
                                       const int *start, const int *tokens, float *logits) {
  const orc_config &c = m->c;
  const int H = c.hidden, F = c.intermediate, d = m->d, nh = c.num_heads;
  const int fp16 = m->fp16;
  std::vector<int> off(nreq + 1, 0);
  for (int r = 0; r < nreq; ++r) {
    if (reqs[r] < 0 || reqs[r] >= m->max_requests || counts[r] <= 0 ||
        start[r] + counts[r] > m->max_seq)
      return -1;
    off[r + 1] = off[r] + counts[r];
  }
  const int T = off[nreq];
  std::vector<float> res((size_t)T * H), h((size_t)T * H), r2((size_t)T * H);
  std::vector<float> q((size_t)T * H), k((size_t)T * H), v((size_t)T * H);
  std::vector<float> att((size_t)T * H), o((size_t)T * H), mlp((size_t)T * H);
  std::vector<float> g((size_t)T * F), u((size_t)T * F), a((size_t)T * F);
  for (int t = 0; t < T; ++t)
    memcpy(&res[(size_t)t * H], &m->emb[(size_t)tokens[t] * H], H * sizeof(float));
  const float scale = 1.0f / sqrtf((float)d);
  for (int l = 0; l < c.num_layers; ++l) {
    auto &L = m->layers[l];
    if (l == 0) {
      orc_rmsnorm(res.data(), L.in_norm.data(), h.data(), T, H, c.rms_eps, fp16);
    } else {
      orc_residual_rmsnorm(res.data(), mlp.data(), L.in_norm.data(), r2.data(), h.data(), T, H,
                           c.rms_eps, fp16);
      res.swap(r2);
    }
    orc_linear(h.data(), L.wq.data(), q.data(), T, H, H, fp16);
    orc_linear(h.data(), L.wk.data(), k.data(), T, H, H, fp16);
    orc_linear(h.data(), L.wv.data(), v.data(), T, H, H, fp16);
    for (int r = 0; r < nreq; ++r) {
      float *kc = &m->kc[(((size_t)reqs[r] * c.num_layers + l) * m->max_seq) * H];
      float *vc = &m->vc[(((size_t)reqs[r] * c.num_layers + l) * m->max_seq) * H];
      for (int i = 0; i < counts[r]; ++i) {
        const int t = off[r] + i, pos = start[r] + i;
        for (int hd = 0; hd < nh; ++hd) {
          float *qh = &q[(size_t)t * H + hd * d];
          float *kh = &k[(size_t)t * H + hd * d];
          rope_apply(qh, d, &m->rope[(size_t)pos * d]);
          rope_apply(kh, d, &m->rope[(size_t)pos * d]);
          for (int e = 0; e < d; ++e) {
            qh[e] = R(qh[e], fp16);
            kh[e] = R(kh[e], fp16);
          }
        }
        memcpy(kc + (size_t)pos * H, &k[(size_t)t * H], H * sizeof(float));
        memcpy(vc + (size_t)pos * H, &v[(size_t)t * H], H * sizeof(float));
      }
    }
#pragma omp parallel for collapse(2) schedule(dynamic)
    for (int r = 0; r < nreq; ++r)
      for (int hd = 0; hd < nh; ++hd) {
        const float *kc = &m->kc[(((size_t)reqs[r] * c.num_layers + l) * m->max_seq) * H];
        const float *vc = &m->vc[(((size_t)reqs[r] * c.num_layers + l) * m->max_seq) * H];
        const int nk = start[r] + counts[r];
        std::vector<float> Kh((size_t)nk * d), Vh((size_t)nk * d);
        std::vector<uint8_t> vis(nk);
        for (int j = 0; j < nk; ++j) {
          memcpy(&Kh[(size_t)j * d], kc + (size_t)j * H + hd * d, d * sizeof(float));
          memcpy(&Vh[(size_t)j * d], vc + (size_t)j * H + hd * d, d * sizeof(float));
        }
        for (int i = 0; i < counts[r]; ++i) {
          const int t = off[r] + i, pos = start[r] + i;
          for (int j = 0; j < nk; ++j) vis[j] = j <= pos;
          orc_attention_row(&q[(size_t)t * H + hd * d], Kh.data(), Vh.data(), vis.data(), nk, d,
                            scale, &att[(size_t)t * H + hd * d], fp16);
        }
      }
    orc_linear(att.data(), L.wo.data(), o.data(), T, H, H, fp16);
    orc_residual_rmsnorm(res.data(), o.data(), L.post_norm.data(), r2.data(), h.data(), T, H,
                         c.rms_eps, fp16);
    res.swap(r2);
    orc_linear(h.data(), L.wg.data(), g.data(), T, F, H, fp16);
    orc_linear(h.data(), L.wu.data(), u.data(), T, F, H, fp16);
    orc_silu_mul(g.data(), u.data(), a.data(), (size_t)T * F, fp16);
    orc_linear(a.data(), L.wd.data(), mlp.data(), T, H, F, fp16);
  }
  orc_residual_rmsnorm(res.data(), mlp.data(), m->final_norm.data(), r2.data(), h.data(), T, H,
                       c.rms_eps, fp16);
  if (logits) orc_linear(h.data(), m->lm.data(), logits, T, c.vocab_size, H, fp16);
  return 0;
}

extern "C" int orc_model_get_hidden(orc_model *m, int layer, float *out) {
  if (layer < 0 || layer > m->c.num_layers) return -1;
  auto &v = m->hidden[layer];
  memcpy(out, v.data(), v.size() * sizeof(float));
  return (int)(v.size() / m->c.hidden);
}

extern "C" int orc_model_get_op(orc_model *m, int kind, int layer, float *out) {
  if (kind < 2 || kind > 9 || layer < 0 || layer >= (int)m->ops[kind].size()) return -1;
  const auto &v = m->ops[kind][layer];
  if (out) memcpy(out, v.data(), v.size() * sizeof(float));
  return m->ops_T;
}

extern "C" int orc_model_greedy(orc_model *m, int req, const int *prompt,
                                int n_prompt, int n_new, int *out_tokens) {
  const int V = m->c.vocab_size;
  std::vector<float> logits((size_t)n_prompt * V);
  if (orc_model_forward(m, req, prompt, n_prompt, 0, logits.data())) return -1;
  int tok;
  orc_softmax_argmax(&logits[(size_t)(n_prompt - 1) * V], 1, V, m->fp16, &tok, nullptr);
  int pos = n_prompt;
  for (int i = 0; i < n_new; ++i) {
    out_tokens[i] = tok;
    if (i + 1 == n_new) break;
    if (orc_model_forward(m, req, &tok, 1, pos, logits.data())) return -1;
    ++pos;
    orc_softmax_argmax(logits.data(), 1, V, m->fp16, &tok, nullptr);
  }
  return 0;
}

extern "C" int orc_num_threads(void) { return omp_get_max_threads(); }
