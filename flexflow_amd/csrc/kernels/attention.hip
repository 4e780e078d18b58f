// attention.hip -- incremental / speculative / tree-verify attention on MFMA.
//
// One kernel family serves the reference's three attention ops, because on
// the device they differ only in WHICH cache slots a query may see:
//  * IncMultiHeadSelfAttention    (inc_multihead_self_attention.cu:372-623,
//    prompt path :98-366): keys [0, pos] (causal);
//  * TreeIncMultiHeadSelfAttention (tree_inc_multihead_self_attention.cu:
//    35-333): keys [0, non_tree_cache_size) plus tree slot j iff
//    causalMask.mask[j] has the query's bit (layer-order token tree);
//  * SpecIncMultiHeadSelfAttention (spec_inc_multihead_self_attention.cu:
//    36-309): same bitmask rule with the query's tree index as its bit.
// The host packs that rule per token (ffmi_token_info: prefix_len,
// tree_base/len/bit), so the kernel is mode-agnostic.  (The reference's
// `1 << qi` on a 32-bit int, tree_inc...cu:168-169, is done in 64 bits here.)
//
// KV-cache layout (handle-owned, MI355X-first): K[req][head][slot][d] and
// V^T[req][head][d][slot], slots = S + tree rounded up to 32.  With these two
// orientations both attention GEMMs read their MFMA operands straight from
// HBM as 16-B / 8-B vectors:
//   S^T[key][q] = K . Q^T        (A = K rows, B = Q rows)   16x16x32 f16
//   O^T[d][q]  += V^T . P^T      (A = V^T rows, B = P^T)    16x16x32 f16
// and the S^T accumulator of a lane (query q = lane&15, keys 4g..4g+3 of
// each 16-key half, g = lane>>4) IS the lane's P^T B-fragment under the key
// permutation k(g,j) = (j<4 ? 4g+j : 16+4g+j-4) -- no LDS transpose.  P is
// fed as an fp16 hi/lo pair (two MFMAs), which keeps ~22 bits of P, matching
// the reference's fp32 P.V accumulation (inc...cu:575-581) instead of
// rounding P to fp16.  Softmax follows the reference: __expf, running max,
// out = sum(e_j v_j) / (sum_j e_j + 1e-6)   (inc...cu:532-547).
//
// Work decomposition: one workgroup per (work item = <=16 queries of one
// request, head); its 4 waves stride over 32-key chunks with private online
// softmax state and merge through LDS.  Every key/value byte of a request is
// read once per 16-query tile (the reference's tree kernel re-reads the
// whole K/V once per query, tree_inc...cu:135).
#include "../ffmi_internal.h"

namespace ffmi {

__device__ __forceinline__ float h2f(uint16_t v) { return __half2float(__ushort_as_half(v)); }
__device__ __forceinline__ uint16_t f2h(float v) { return __half_as_ushort(__float2half_rn(v)); }

// commit_tokens_kernel (tree_inc...cu:335-396): accepted tokens of the
// previous verify batch move from the staging rows to their depth slot.
__global__ void commit_kernel(const char *__restrict__ blob, int C,
                              const uint16_t *__restrict__ stage, uint16_t *__restrict__ kc,
                              uint16_t *__restrict__ vc, int heads, int d, int slots) {
  const int item = blockIdx.x;  // commit * heads + head
  const int ci = item / heads, h = item % heads;
  if (ci >= C) return;
  BatchView bv = batch_view(blob);
  const ffmi_commit_info cm = bv.commits[ci];
  if (cm.depth < 0 || cm.depth >= slots) return;
  const int Hl = heads * d;
  const uint16_t *st = stage + (size_t)cm.src_token * 2 * Hl + h * d;
  for (int i = threadIdx.x; i < d; i += blockDim.x) {
    kc[(((size_t)cm.req * heads + h) * slots + cm.depth) * d + i] = st[i];
    vc[(((size_t)cm.req * heads + h) * d + i) * slots + cm.depth] = st[Hl + i];
  }
}

hipError_t launch_commit(const char *blob, int C, const uint16_t *stage, uint16_t *kc,
                         uint16_t *vc, int heads, int d, int slots, hipStream_t s) {
  if (C <= 0) return hipSuccess;
  hipLaunchKernelGGL(commit_kernel, dim3(C * heads), dim3(64), 0, s, blob, C, stage, kc, vc,
                     heads, d, slots);
  return hipGetLastError();
}

// Fused KV update of one step: RoPE (HF rotate-half, inc...cu:664-738) + KV
// store (store_kv_cache inc...cu:35-61 / update_tree_branch_kv_cache_fused
// tree_inc...cu:433-478 / spec_inc_store_kv_cache spec_inc...cu:311-358) +
// staging copy for the next step's commits
// for each (attention work item = <= 16 consecutive tokens of a request, head),
// plus the TREE commits of the previous verify batch in extra blocks.
//  * V goes through LDS so that V^T rows are written as runs of consecutive
//    slots (16 lanes x 2 B) instead of one 2-byte store per (token, d);
//  * commits read the OTHER half of the ping-pong staging (stage_rd) than the
//    one this step writes (stage_wr), so both run in one launch.  The host
//    launches commits separately first when a commit depth coincides with a
//    slot this step stores (the reference's commit-then-store order).
template <int D>
__global__ __launch_bounds__(16 * D / 2) void kv_update_kernel(
    const char *__restrict__ blob, int T, int W, int C, const uint16_t *__restrict__ qkv,
    const float *__restrict__ part, int pS, int pNP, uint16_t *__restrict__ qbuf,
    uint16_t *__restrict__ kc, uint16_t *__restrict__ vc, uint16_t *__restrict__ stage_wr,
    const uint16_t *__restrict__ stage_rd, const float *__restrict__ rope, int heads, int slots,
    int max_rope_pos) {
  constexpr int HD = D / 2;  // one thread per (token of a 16-token half, rotation pair)
  constexpr int NQ = FFMI_ATTN_QTILE;
  __shared__ uint16_t sV[D][NQ + 1];
  __shared__ int sSlot[NQ];
  const int Hl = heads * D;
  const BatchView bv = batch_view(blob);
  const int item = blockIdx.x / heads, h = blockIdx.x % heads;
  if (item >= W) {  // ---- commit block (tree_inc...cu:335-396)
    const int ci = item - W;
    if (ci >= C) return;
    const ffmi_commit_info cm = bv.commits[ci];
    if (cm.depth < 0 || cm.depth >= slots) return;
    const uint16_t *st = stage_rd + (size_t)cm.src_token * 2 * Hl + h * D;
    const int i = threadIdx.x;
    if (i < D) {
      kc[(((size_t)cm.req * heads + h) * slots + cm.depth) * D + i] = st[i];
      vc[(((size_t)cm.req * heads + h) * D + i) * slots + cm.depth] = st[Hl + i];
    }
    return;
  }
  const ffmi_attn_work w = bv.work[item];
  const int i = threadIdx.x % HD;
  for (int tl = threadIdx.x / HD; tl < NQ; tl += 16) {
    if (tl >= w.q_count) break;
    const int t = w.q_start + tl;
    const ffmi_token_info ti = bv.tokens[t];
    auto qkv_at = [&](int col) -> float {
      return part ? partials_value(part, pS, pNP, T, t, col)
                  : h2f(qkv[(size_t)t * 3 * Hl + col]);
    };
    const int qc = h * D, kc0 = Hl + h * D, vc0 = 2 * Hl + h * D;
    const float qa = qkv_at(qc + i), qb = qkv_at(qc + i + HD);
    const float ka = qkv_at(kc0 + i), kb = qkv_at(kc0 + i + HD);
    const float va = qkv_at(vc0 + i), vb = qkv_at(vc0 + i + HD);
    const int pos = min(max(ti.pos, 0), max_rope_pos - 1);
    const float c = rope[((size_t)pos * HD + i) * 2 + 0];
    const float s = rope[((size_t)pos * HD + i) * 2 + 1];
    const uint16_t q0 = f2h(__fsub_rn(__fmul_rn(qa, c), __fmul_rn(qb, s)));
    const uint16_t q1 = f2h(__fadd_rn(__fmul_rn(qa, s), __fmul_rn(qb, c)));
    const uint16_t k0 = f2h(__fsub_rn(__fmul_rn(ka, c), __fmul_rn(kb, s)));
    const uint16_t k1 = f2h(__fadd_rn(__fmul_rn(ka, s), __fmul_rn(kb, c)));
    const uint16_t v0 = f2h(va), v1 = f2h(vb);
    uint16_t *qo = qbuf + (size_t)t * Hl + h * D;
    qo[i] = q0;
    qo[i + HD] = q1;
    const bool store = ti.store_slot >= 0 && ti.store_slot < slots;
    if (store) {
      uint16_t *kr = kc + (((size_t)ti.req * heads + h) * slots + ti.store_slot) * D;
      kr[i] = k0;
      kr[i + HD] = k1;
    }
    if (i == 0) sSlot[tl] = store ? ti.store_slot : -1;
    sV[i][tl] = v0;
    sV[i + HD][tl] = v1;
    if (stage_wr) {
      uint16_t *st = stage_wr + (size_t)t * 2 * Hl + h * D;
      st[i] = k0;
      st[i + HD] = k1;
      st[Hl + i] = v0;
      st[Hl + i + HD] = v1;
    }
  }
  __syncthreads();
  // ---- V^T[req][h][d][slot]: lanes run over consecutive tokens of a d-row
  uint16_t *vt = vc + ((size_t)w.req * heads + h) * D * slots;
  for (int e = threadIdx.x; e < D * NQ; e += blockDim.x) {
    const int dd = e / NQ, tt = e % NQ;
    if (tt >= w.q_count) continue;
    const int sl = sSlot[tt];
    if (sl >= 0) vt[(size_t)dd * slots + sl] = sV[dd][tt];
  }
}

hipError_t launch_kv_update(const char *blob, int T, int W, int C, const uint16_t *qkv,
                            Partials qkvp, uint16_t *qbuf, uint16_t *kc, uint16_t *vc,
                            uint16_t *stage_wr, const uint16_t *stage_rd, const float *rope,
                            int heads, int d, int slots, int max_rope_pos, hipStream_t s) {
  if (W <= 0 && C <= 0) return hipSuccess;
  const dim3 grid((W + C) * heads);
  const float *pp = qkvp.S > 0 ? qkvp.p : nullptr;
  if (d == 128)
    hipLaunchKernelGGL(kv_update_kernel<128>, grid, dim3(1024), 0, s, blob, T, W, C, qkv, pp,
                       qkvp.S, qkvp.NP, qbuf, kc, vc, stage_wr, stage_rd, rope, heads, slots,
                       max_rope_pos);
  else if (d == 64)
    hipLaunchKernelGGL(kv_update_kernel<64>, grid, dim3(512), 0, s, blob, T, W, C, qkv, pp,
                       qkvp.S, qkvp.NP, qbuf, kc, vc, stage_wr, stage_rd, rope, heads, slots,
                       max_rope_pos);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

// visibility from registers only: prefix range + the query's 64-bit tree word
__device__ __forceinline__ bool key_visible(int slot, int prefix_len, int tree_base,
                                            int tree_len, uint64_t tree_vis) {
  if (slot < prefix_len) return true;
  const unsigned j = (unsigned)(slot - tree_base);
  return j < (unsigned)tree_len && ((tree_vis >> j) & 1ull);
}

// Arguments of the fused prologue (FUSED kernels only; see attention_kernel).
struct KvUpdateArgs {
  int T, C;
  const uint16_t *qkv;
  const float *part;
  int pS, pNP;
  uint16_t *stage_wr;
  const uint16_t *stage_rd;
  const float *rope;
  int max_rope_pos;
};

// One workgroup per (work item = <= 16*QT consecutive queries of a request,
// head); 4 waves stride over 32-key chunks with private online-softmax state
// and merge through LDS.  QT query tiles share every K / V^T fragment load.
//
// FUSED (host-checked: each request has exactly one work item this step, as
// in decode, SSM beam steps and tree verify): the workgroup first applies its
// own request's TREE commits and the KV update of its own tokens for its
// head (kv_update_kernel's work), makes them visible to the workgroup, then
// attends -- one launch per step instead of two.
template <int D, int QT, bool FUSED>
__global__ __launch_bounds__(256, 2) void attention_kernel(
    const char *__restrict__ blob, uint16_t *__restrict__ qbuf, uint16_t *__restrict__ kc,
    uint16_t *__restrict__ vc, uint16_t *__restrict__ out, int heads, int slots, float scale,
    int out_packed, KvUpdateArgs kv) {
  constexpr int KS = D / 32;  // k-steps of the QK^T product
  constexpr int DT = D / 16;  // d-tiles of the PV product
  constexpr int NQ = 16 * QT;
  __shared__ float sm_m[4][NQ];
  __shared__ float sm_l[4][NQ];
  __shared__ __attribute__((aligned(16))) float sm_o[4][QT][DT][4][64];

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int qi = lane & 15;
  const int g = lane >> 4;
  const int h = blockIdx.y;
  const BatchView bv = batch_view(blob);
  const ffmi_attn_work w = bv.work[blockIdx.x];
  const int Hl = heads * D;

  if (FUSED) {
    constexpr int HD = D / 2;
    __shared__ uint16_t sV[D][NQ + 1];
    __shared__ int sSlot[NQ];
    // (1) commits of this request (commit before store, as the reference)
    for (int e = threadIdx.x; e < kv.C * D; e += blockDim.x) {
      const ffmi_commit_info cm = bv.commits[e / D];
      const int i = e % D;
      if (cm.req != w.req || cm.depth < 0 || cm.depth >= slots) continue;
      const uint16_t *st = kv.stage_rd + (size_t)cm.src_token * 2 * Hl + h * D;
      kc[(((size_t)cm.req * heads + h) * slots + cm.depth) * D + i] = st[i];
      vc[(((size_t)cm.req * heads + h) * D + i) * slots + cm.depth] = st[Hl + i];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // (2) RoPE + KV store + staging of this item's tokens, this head
    for (int e = threadIdx.x; e < NQ * HD; e += blockDim.x) {
      const int tl = e / HD, i = e % HD;
      if (tl >= w.q_count) continue;
      const int t = w.q_start + tl;
      const ffmi_token_info ti = bv.tokens[t];
      auto qkv_at = [&](int col) -> float {
        return kv.part ? partials_value(kv.part, kv.pS, kv.pNP, kv.T, t, col)
                       : h2f(kv.qkv[(size_t)t * 3 * Hl + col]);
      };
      const int qc = h * D, kc0 = Hl + h * D, vc0 = 2 * Hl + h * D;
      const float qa = qkv_at(qc + i), qb = qkv_at(qc + i + HD);
      const float ka = qkv_at(kc0 + i), kb = qkv_at(kc0 + i + HD);
      const float va = qkv_at(vc0 + i), vb = qkv_at(vc0 + i + HD);
      const int pos = min(max(ti.pos, 0), kv.max_rope_pos - 1);
      const float c = kv.rope[((size_t)pos * HD + i) * 2 + 0];
      const float sn = kv.rope[((size_t)pos * HD + i) * 2 + 1];
      const uint16_t k0 = f2h(__fsub_rn(__fmul_rn(ka, c), __fmul_rn(kb, sn)));
      const uint16_t k1 = f2h(__fadd_rn(__fmul_rn(ka, sn), __fmul_rn(kb, c)));
      const uint16_t v0 = f2h(va), v1 = f2h(vb);
      uint16_t *qo = qbuf + (size_t)t * Hl + h * D;
      qo[i] = f2h(__fsub_rn(__fmul_rn(qa, c), __fmul_rn(qb, sn)));
      qo[i + HD] = f2h(__fadd_rn(__fmul_rn(qa, sn), __fmul_rn(qb, c)));
      const bool store = ti.store_slot >= 0 && ti.store_slot < slots;
      if (store) {
        uint16_t *kr = kc + (((size_t)ti.req * heads + h) * slots + ti.store_slot) * D;
        kr[i] = k0;
        kr[i + HD] = k1;
      }
      if (i == 0) sSlot[tl] = store ? ti.store_slot : -1;
      sV[i][tl] = v0;
      sV[i + HD][tl] = v1;
      if (kv.stage_wr) {
        uint16_t *st = kv.stage_wr + (size_t)t * 2 * Hl + h * D;
        st[i] = k0;
        st[i + HD] = k1;
        st[Hl + i] = v0;
        st[Hl + i + HD] = v1;
      }
    }
    __syncthreads();
    uint16_t *vt = vc + ((size_t)w.req * heads + h) * D * slots;
    for (int e = threadIdx.x; e < D * NQ; e += blockDim.x) {
      const int dd = e / NQ, tt = e % NQ;
      if (tt >= w.q_count) continue;
      const int sl = sSlot[tt];
      if (sl >= 0) vt[(size_t)dd * slots + sl] = sV[dd][tt];
    }
    // this workgroup's stores become visible to its own loads below (the
    // (req, head) K/V lines are touched by no other workgroup this step)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  bool qvalid[QT];
  int pre[QT], tb[QT], tlen[QT];
  uint64_t tv[QT];
  h8 qf[QT][KS];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    const int q = qt * 16 + qi;
    qvalid[qt] = q < w.q_count;
    const ffmi_token_info ti = bv.tokens[w.q_start + (qvalid[qt] ? q : 0)];
    pre[qt] = ti.prefix_len, tb[qt] = ti.tree_base, tlen[qt] = ti.tree_len, tv[qt] = ti.tree_vis;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      qf[qt][ks] = qvalid[qt] ? *reinterpret_cast<const h8 *>(
                                    qbuf + (size_t)(w.q_start + q) * Hl + h * D + 32 * ks + 8 * g)
                              : h8{0, 0, 0, 0, 0, 0, 0, 0};
  }
  const uint16_t *kbase = kc + ((size_t)w.req * heads + h) * slots * D;
  const uint16_t *vbase = vc + ((size_t)w.req * heads + h) * D * slots;

  const float NEG = -INFINITY;
  float m_run[QT], l_run[QT];
  f4 o[QT][DT];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    m_run[qt] = NEG, l_run[qt] = 0.f;
#pragma unroll
    for (int t = 0; t < DT; ++t) o[qt][t] = f4{0.f, 0.f, 0.f, 0.f};
  }

  const int nchunks = (w.kv_len + 31) >> 5;
  for (int c = wave; c < nchunks; c += 4) {
    const int base = c * 32;
    h8 kf[2][KS];
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      const uint16_t *krow = kbase + (size_t)(base + sub * 16 + (lane & 15)) * D + 8 * g;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) kf[sub][ks] = *reinterpret_cast<const h8 *>(krow + 32 * ks);
    }
    // V^T fragments for this chunk (issued early; consumed after softmax)
    h8 va[DT];
#pragma unroll
    for (int t = 0; t < DT; ++t) {
      const uint16_t *vrow = vbase + (size_t)(t * 16 + (lane & 15)) * slots + base + 4 * g;
      h4 v0 = *reinterpret_cast<const h4 *>(vrow);
      h4 v1 = *reinterpret_cast<const h4 *>(vrow + 16);
      va[t] = h8{v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
    }
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
      // S^T = K . Q^T: this lane holds query qt*16+qi, keys base + 16 sub + 4 g + r
      f4 s[2];
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        s[sub] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
          s[sub] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf[sub][ks], qf[qt][ks], s[sub], 0, 0, 0);
      }
      float sc[8];
      bool vis[8];
      float cmax = NEG;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int slot = base + (j >> 2) * 16 + 4 * g + (j & 3);
        vis[j] = qvalid[qt] && slot < w.kv_len &&
                 key_visible(slot, pre[qt], tb[qt], tlen[qt], tv[qt]);
        sc[j] = __fmul_rn(scale, s[j >> 2][j & 3]);
        cmax = vis[j] ? fmaxf(cmax, sc[j]) : cmax;
      }
      cmax = fmaxf(cmax, __shfl_xor(cmax, 16));
      cmax = fmaxf(cmax, __shfl_xor(cmax, 32));
      const float m_new = fmaxf(m_run[qt], cmax);
      const float m_use = (m_new == NEG) ? 0.f : m_new;
      const float alpha = (m_run[qt] == NEG) ? 0.f : __expf(m_run[qt] - m_use);
      h8 phi, plo;
      float psum = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float e = vis[j] ? __expf(sc[j] - m_use) : 0.f;
        psum += e;
        const _Float16 hi = (_Float16)e;
        phi[j] = hi;
        plo[j] = (_Float16)(e - (float)hi);
      }
      l_run[qt] = l_run[qt] * alpha + psum;
      m_run[qt] = m_new;
#pragma unroll
      for (int t = 0; t < DT; ++t) {
        o[qt][t] *= alpha;
        o[qt][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(va[t], phi, o[qt][t], 0, 0, 0);
        o[qt][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(va[t], plo, o[qt][t], 0, 0, 0);
      }
    }
  }

  // per-query partial sum over the 4 lane groups (same m_run in all four)
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    float l = l_run[qt];
    l += __shfl_xor(l, 16);
    l += __shfl_xor(l, 32);
    if (g == 0) {
      sm_m[wave][qt * 16 + qi] = m_run[qt];
      sm_l[wave][qt * 16 + qi] = l;
    }
#pragma unroll
    for (int t = 0; t < DT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) sm_o[wave][qt][t][r][lane] = o[qt][t][r];
  }
  __syncthreads();

  // merge: wave w finalizes d-tiles t = w, w+4, ... of every query tile
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    const int q = qt * 16 + qi;
    float M = NEG;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) M = fmaxf(M, sm_m[ww][q]);
    float f[4], L = 0.f;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) {
      const float mw = sm_m[ww][q];
      f[ww] = (mw == NEG) ? 0.f : __expf(mw - M);
      L += f[ww] * sm_l[ww][q];
    }
    const float inv = 1.0f / (L + 1e-6f);
    if (!qvalid[qt]) continue;
    const int orow_m = w.q_start + q;
    uint16_t *orow = out + (size_t)orow_m * Hl + h * D;
    for (int t = wave; t < DT; t += 4) {
      uint16_t r4[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float acc = 0.f;
#pragma unroll
        for (int ww = 0; ww < 4; ++ww) acc += f[ww] * sm_o[ww][qt][t][r][lane];
        r4[r] = f2h(acc * inv);
      }
      uint2 pk;
      pk.x = r4[0] | ((uint32_t)r4[1] << 16);
      pk.y = r4[2] | ((uint32_t)r4[3] << 16);
      uint16_t *dst = out_packed ? out + act_packed_off(orow_m, h * D + t * 16 + 4 * g, Hl)
                                 : orow + t * 16 + 4 * g;
      *reinterpret_cast<uint2 *>(dst) = pk;
    }
  }
}

template <int D>
static hipError_t launch_attention_d(const char *blob, int W, int max_q, uint16_t *qbuf,
                                     uint16_t *kc, uint16_t *vc, uint16_t *out, int heads,
                                     int slots, float scale, hipStream_t s, int op, bool fused,
                                     const KvUpdateArgs &kv) {
  const dim3 grid(W, heads);
#define FFMI_ATT(QT, FU)                                                                     \
  hipLaunchKernelGGL((attention_kernel<D, QT, FU>), grid, dim3(256), 0, s, blob, qbuf, kc, vc, \
                     out, heads, slots, scale, op, kv)
  if (max_q <= 16) {
    if (fused) FFMI_ATT(1, true);
    else FFMI_ATT(1, false);
  } else {
    if (fused) FFMI_ATT(2, true);
    else FFMI_ATT(2, false);
  }
#undef FFMI_ATT
  return hipGetLastError();
}

// fused == false: the KV of this step must already be in the cache
// (launch_kv_update); fused == true: one workgroup per request (checked by the
// caller) does commits + KV update + attention.
hipError_t launch_attention(const char *blob, int W, int max_q, uint16_t *qbuf, uint16_t *kc,
                            uint16_t *vc, uint16_t *out, int heads, int d, int slots, float scale,
                            hipStream_t s, bool out_packed, bool fused, int T, int C,
                            const uint16_t *qkv, Partials qkvp, uint16_t *stage_wr,
                            const uint16_t *stage_rd, const float *rope, int max_rope_pos) {
  if (W <= 0) return hipSuccess;
  if (out_packed && (heads * d) % 32) return hipErrorInvalidValue;
  if (max_q > FFMI_ATTN_QTILE) return hipErrorInvalidValue;
  const KvUpdateArgs kv{T, C, qkv, qkvp.S > 0 ? qkvp.p : nullptr, qkvp.S, qkvp.NP,
                        stage_wr, stage_rd, rope, max_rope_pos};
  const int op = out_packed ? 1 : 0;
  if (d == 128)
    return launch_attention_d<128>(blob, W, max_q, qbuf, kc, vc, out, heads, slots, scale, s, op,
                                   fused, kv);
  if (d == 64)
    return launch_attention_d<64>(blob, W, max_q, qbuf, kc, vc, out, heads, slots, scale, s, op,
                                  fused, kv);
  return hipErrorInvalidValue;
}

}  // namespace ffmi
