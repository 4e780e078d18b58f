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
// request, head); its 8 waves stride over 32-key chunks with private online
// softmax state and merge through LDS.  Every key/value byte of a request is
// read once per 16-query tile (the reference's tree kernel re-reads the
// whole K/V once per query, tree_inc...cu:135).
#include <stdlib.h>

#include <algorithm>

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
// staging copy for the next step's commits, for one (attention work item =
// <= NQ consecutive tokens of a request, head).  Shared by kv_update_kernel
// and the FUSED attention prologue.
//  * a thread unit is 4 consecutive rotation pairs (d = i0..i0+3 and
//    i0+D/2..) of one token: 8-B fp16 or 16-B fp32-slab loads, 8-B stores;
//  * every load of a thread (all its units, all slabs) is issued before its
//    first store -- the update is a chain of dependent HBM round trips
//    otherwise (units past q_count load token 0 and store nothing);
//  * V goes through LDS so that V^T rows are written as runs of consecutive
//    slots instead of one 2-byte store per (token, d).
__device__ __forceinline__ f4 round_h4(f4 a) {  // fp16 value of the combined sum
  return f4{h2f(f2h(a[0])), h2f(f2h(a[1])), h2f(f2h(a[2])), h2f(f2h(a[3]))};
}
__device__ __forceinline__ void st_h4(uint16_t *p, uint16_t a, uint16_t b, uint16_t c,
                                      uint16_t d) {
  *reinterpret_cast<uint2 *>(p) = make_uint2(a | ((uint32_t)b << 16), c | ((uint32_t)d << 16));
}

// after_loads() runs once this thread's update loads are in flight (the
// fused attention issues its first K/V chunk there: loads complete in issue
// order, so anything issued BEFORE these would delay them).
// Tail mode (sKt != nullptr, the fused attention): K rows and V^T columns of
// the stored tokens also go to the workgroup's LDS tail tile (slot - tail0),
// where its attention reads them -- no wait for the global stores; V^T then
// goes to HBM from sVt.  before_stores() runs (in every thread) once the
// loads are back, before the first store.
// PSRC: 1 = qkv from split-K slabs, 0 = fp16 qkv, -1 = decided at run time
// by `part` (a compile-time source keeps the two load paths from joining:
// the join's register copies waited for half of the slab loads).
template <int D, int NQ, int NT, int PSRC = -1, class AfterLoads, class BeforeStores>
__device__ __forceinline__ void kv_update_item(
    const BatchView &bv, const WorkDev *__restrict__ wdp, int h, int heads, int slots, int T,
    const uint16_t *__restrict__ qkv, const float *__restrict__ part, int pS, int pNP,
    const float *__restrict__ rope, int max_rope_pos, uint16_t *__restrict__ qbuf,
    uint16_t *__restrict__ kc, uint16_t *__restrict__ stage_wr, uint16_t (*sV)[NQ + 1],
    int *sSlot, uint16_t (*sQ)[D + 8], uint16_t (*sKt)[D + 8],
    uint16_t (*sVt)[kTailSlots + 8], int tail0, AfterLoads &&after_loads,
    BeforeStores &&before_stores) {
  constexpr int HD = D / 2, G = HD / 4, UNITS = NQ * G, U = (UNITS + NT - 1) / NT;
  const int Hl = heads * D;
  const ffmi_attn_work w = wdp->w;
  // channels: 0 q lo, 1 q hi, 2 k lo, 3 k hi, 4 v lo, 5 v hi
  f4 x[U][6], y[U][6], cs[U][2];  // y: second fp32 slab
  int tslot[U], treq[U];  // (scalar fields: a struct copy would go to scratch)
  int tl[U], i0[U];
  // One round trip for every prologue load.  The RoPE positions of the
  // item's tokens come through the scalar cache (16 dwords of the work item,
  // lgkmcnt; readfirstlane keeps them there -- the per-lane select over them
  // was folded into a vector load), so the RoPE-row loads do not wait on any
  // vector load; the qkv
  // slabs (addresses known up front), the RoPE rows and the token records
  // then go out back to back.  (Vector loads complete in issue order: with
  // the positions loaded per lane, the RoPE rows waited for that load and
  // for everything issued before it.)
  const uint32_t *rp32 = reinterpret_cast<const uint32_t *>(wdp->rope_pos);
  uint32_t rpw[FFMI_ATTN_QTILE / 2];
#pragma unroll
  for (int j = 0; j < FFMI_ATTN_QTILE / 2; ++j) rpw[j] = __builtin_amdgcn_readfirstlane(rp32[j]);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int e = min((int)threadIdx.x + u * NT, UNITS - 1);
    tl[u] = e / G, i0[u] = (e % G) * 4;
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int t = w.q_start + (tl[u] < w.q_count ? tl[u] : 0);
    const int col[6] = {h * D + i0[u], h * D + i0[u] + HD, Hl + h * D + i0[u],
                        Hl + h * D + i0[u] + HD, 2 * Hl + h * D + i0[u],
                        2 * Hl + h * D + i0[u] + HD};
    if (PSRC == 1 || (PSRC < 0 && part)) {  // slabs 0 and 1 (slab 0 again when pS == 1: no branch)
      const float *p1 = part + (pS > 1 ? (size_t)T * pNP : 0);
#pragma unroll
      for (int c = 0; c < 6; ++c)
        x[u][c] = *reinterpret_cast<const f4 *>(part + (size_t)t * pNP + col[c]);
#pragma unroll
      for (int c = 0; c < 6; ++c)
        y[u][c] = *reinterpret_cast<const f4 *>(p1 + (size_t)t * pNP + col[c]);
    } else {  // raw fp16 bits now, converted after every load is out
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        const uint2 r = *reinterpret_cast<const uint2 *>(qkv + (size_t)t * 3 * Hl + col[c]);
        y[u][c] = f4{__uint_as_float(r.x), __uint_as_float(r.y), 0.f, 0.f};
      }
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int q = tl[u] < w.q_count ? tl[u] : 0;
    uint32_t wd = rpw[0];
#pragma unroll
    for (int j = 1; j < FFMI_ATTN_QTILE / 2; ++j) wd = (q >> 1) == j ? rpw[j] : wd;
    const int p = min((int)((q & 1) ? (wd >> 16) : (wd & 0xffffu)), max_rope_pos - 1);
    const f4 *r = reinterpret_cast<const f4 *>(rope + ((size_t)p * HD + i0[u]) * 2);
    cs[u][0] = r[0];  // c0 s0 c1 s1
    cs[u][1] = r[1];  // c2 s2 c3 s3
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int t = w.q_start + (tl[u] < w.q_count ? tl[u] : 0);
    tslot[u] = bv.tokens[t].store_slot;
    treq[u] = bv.tokens[t].req;
  }
  after_loads();
  // every prologue load is in flight before any of them is consumed: left
  // alone the scheduler summed the slabs right after they were issued and
  // gave their registers to the RoPE rows, so each group of loads waited for
  // the one before it (four round trips instead of one)
  __builtin_amdgcn_sched_barrier(0);
  if (PSRC == 0 || (PSRC < 0 && !part))
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        const uint32_t a = __float_as_uint(y[u][c][0]), b = __float_as_uint(y[u][c][1]);
        x[u][c] = f4{h2f(a & 0xffff), h2f(a >> 16), h2f(b & 0xffff), h2f(b >> 16)};
      }
  if (PSRC == 1 || (PSRC < 0 && part)) {  // slabs in slice order, then fp16 (partials_value)
    if (pS > 1)
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int c = 0; c < 6; ++c) x[u][c] += y[u][c];
    const size_t slab = (size_t)T * pNP;
    for (int sl = 2; sl < pS; ++sl)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int t = w.q_start + (tl[u] < w.q_count ? tl[u] : 0);
        const int col[6] = {h * D + i0[u], h * D + i0[u] + HD, Hl + h * D + i0[u],
                            Hl + h * D + i0[u] + HD, 2 * Hl + h * D + i0[u],
                            2 * Hl + h * D + i0[u] + HD};
#pragma unroll
        for (int c = 0; c < 6; ++c)
          x[u][c] += *reinterpret_cast<const f4 *>(part + sl * slab + (size_t)t * pNP + col[c]);
      }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int c = 0; c < 6; ++c) x[u][c] = round_h4(x[u][c]);
  }

  before_stores();
  // ---- stores
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (tl[u] >= w.q_count || (int)threadIdx.x + u * NT >= UNITS) continue;
    const int t = w.q_start + tl[u];
    uint16_t qlo[4], qhi[4], klo[4], khi[4], vlo[4], vhi[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float c = cs[u][j >> 1][(j & 1) * 2], sn = cs[u][j >> 1][(j & 1) * 2 + 1];
      const float qa = x[u][0][j], qb = x[u][1][j], ka = x[u][2][j], kb = x[u][3][j];
      qlo[j] = f2h(__fsub_rn(__fmul_rn(qa, c), __fmul_rn(qb, sn)));
      qhi[j] = f2h(__fadd_rn(__fmul_rn(qa, sn), __fmul_rn(qb, c)));
      klo[j] = f2h(__fsub_rn(__fmul_rn(ka, c), __fmul_rn(kb, sn)));
      khi[j] = f2h(__fadd_rn(__fmul_rn(ka, sn), __fmul_rn(kb, c)));
      vlo[j] = f2h(x[u][4][j]);
      vhi[j] = f2h(x[u][5][j]);
    }
    // rotated q: to LDS for the same workgroup's attention (fused), else HBM
    uint16_t *qo = sQ ? &sQ[tl[u]][i0[u]] : qbuf + (size_t)t * Hl + h * D + i0[u];
    st_h4(qo, qlo[0], qlo[1], qlo[2], qlo[3]);
    st_h4(qo + HD, qhi[0], qhi[1], qhi[2], qhi[3]);
    const bool store = tslot[u] >= 0 && tslot[u] < slots;
    if (store) {
      uint16_t *kr = kc + (((size_t)treq[u] * heads + h) * slots + tslot[u]) * D + i0[u];
      st_h4(kr, klo[0], klo[1], klo[2], klo[3]);
      st_h4(kr + HD, khi[0], khi[1], khi[2], khi[3]);
    }
    if (i0[u] == 0) sSlot[tl[u]] = store ? tslot[u] : -1;
    if (sKt) {  // (host-checked: every stored slot lies in the tail)
      if (store) {
        const int ts = tslot[u] - tail0;
        st_h4(&sKt[ts][i0[u]], klo[0], klo[1], klo[2], klo[3]);
        st_h4(&sKt[ts][i0[u] + HD], khi[0], khi[1], khi[2], khi[3]);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          sVt[i0[u] + j][ts] = vlo[j];
          sVt[i0[u] + HD + j][ts] = vhi[j];
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        sV[i0[u] + j][tl[u]] = vlo[j];
        sV[i0[u] + HD + j][tl[u]] = vhi[j];
      }
    }
    if (stage_wr) {
      uint16_t *st = stage_wr + (size_t)t * 2 * Hl + h * D + i0[u];
      st_h4(st, klo[0], klo[1], klo[2], klo[3]);
      st_h4(st + HD, khi[0], khi[1], khi[2], khi[3]);
      st_h4(st + Hl, vlo[0], vlo[1], vlo[2], vlo[3]);
      st_h4(st + Hl + HD, vhi[0], vhi[1], vhi[2], vhi[3]);
    }
  }
}

// V^T[req][h][d][slot] rows from the LDS tile: lanes run over consecutive
// tokens of a d-row (call after a barrier that follows kv_update_item)
template <int D, int NQ>
__device__ __forceinline__ void kv_store_vt(const ffmi_attn_work &w, int h, int heads, int slots,
                                            uint16_t *__restrict__ vc,
                                            const uint16_t (*sV)[NQ + 1], const int *sSlot) {
  uint16_t *vt = vc + ((size_t)w.req * heads + h) * D * slots;
  for (int e = threadIdx.x; e < D * NQ; e += blockDim.x) {
    const int dd = e / NQ, tt = e % NQ;
    if (tt >= w.q_count) continue;
    const int sl = sSlot[tt];
    if (sl >= 0) vt[(size_t)dd * slots + sl] = sV[dd][tt];
  }
}

// Standalone KV update (items with more tokens than one attention launch
// should carry in its prologue): one workgroup per (item, head), one thread
// per unit, plus the TREE commits of the previous verify batch in extra
// blocks.  Commits read the OTHER half of the ping-pong staging (stage_rd)
// than the one this step writes (stage_wr), so both run in one launch; the
// host launches commits separately first when a commit depth coincides with
// a slot this step stores (the reference's commit-then-store order).
template <int D>
__global__ __launch_bounds__(FFMI_ATTN_QTILE * D / 8) void kv_update_kernel(
    const char *__restrict__ blob, int T, int W, int C, const uint16_t *__restrict__ qkv,
    const float *__restrict__ part, int pS, int pNP, uint16_t *__restrict__ qbuf,
    uint16_t *__restrict__ kc, uint16_t *__restrict__ vc, uint16_t *__restrict__ stage_wr,
    const uint16_t *__restrict__ stage_rd, const float *__restrict__ rope, int heads, int slots,
    int max_rope_pos) {
  constexpr int NQ = FFMI_ATTN_QTILE;
  constexpr int NT = NQ * D / 8;
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
  const ffmi_attn_work w = bv.work[item].w;
  kv_update_item<D, NQ, NT>(bv, &bv.work[item], h, heads, slots, T, qkv, part, pS, pNP, rope,
                            max_rope_pos, qbuf, kc, stage_wr, sV, sSlot, nullptr, nullptr, nullptr,
                            0, [] {}, [] {});
  __syncthreads();
  kv_store_vt<D, NQ>(w, h, heads, slots, vc, sV, sSlot);
}

hipError_t launch_kv_update(const char *blob, int T, int W, int C, const uint16_t *qkv,
                            Partials qkvp, uint16_t *qbuf, uint16_t *kc, uint16_t *vc,
                            uint16_t *stage_wr, const uint16_t *stage_rd, const float *rope,
                            int heads, int d, int slots, int max_rope_pos, hipStream_t s) {
  if (W <= 0 && C <= 0) return hipSuccess;
  const dim3 grid((W + C) * heads);
  const float *pp = qkvp.S > 0 ? qkvp.p : nullptr;
  if (d == 128)
    hipLaunchKernelGGL(kv_update_kernel<128>, grid, dim3(FFMI_ATTN_QTILE * 16), 0, s, blob, T, W, C, qkv, pp,
                       qkvp.S, qkvp.NP, qbuf, kc, vc, stage_wr, stage_rd, rope, heads, slots,
                       max_rope_pos);
  else if (d == 64)
    hipLaunchKernelGGL(kv_update_kernel<64>, grid, dim3(FFMI_ATTN_QTILE * 8), 0, s, blob, T, W, C, qkv, pp,
                       qkvp.S, qkvp.NP, qbuf, kc, vc, stage_wr, stage_rd, rope, heads, slots,
                       max_rope_pos);
  else if (d == 32)  // (incremental decoding only: ffmi_attn_create)
    hipLaunchKernelGGL(kv_update_kernel<32>, grid, dim3(FFMI_ATTN_QTILE * 4), 0, s, blob, T, W, C, qkv, pp,
                       qkvp.S, qkvp.NP, qbuf, kc, vc, stage_wr, stage_rd, rope, heads, slots,
                       max_rope_pos);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

// visibility from registers only: prefix range + the query's 64-bit tree word
__device__ __forceinline__ bool key_visible(int slot, int prefix_len, int tree_base,
                                            int tree_len, uint64_t tree_vis) {
  const unsigned j = (unsigned)(slot - tree_base);
  const bool in_tree = j < (unsigned)tree_len && ((tree_vis >> (j & 63)) & 1ull);
  return (slot < prefix_len) | in_tree;  // no branches: one select per key
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
  long long *stamps;  // ST kernels: per-wave timeline (diagnostics)
};

// One workgroup per (work item = <= 16*QT consecutive queries of a request,
// head); NW = 8 waves (two per SIMD: each hides the other's load latency)
// stride over 32-key chunks with private online-softmax state
// and merge through LDS.  QT query tiles share every K / V^T fragment load.
//
// FUSED (host-checked: each request has exactly one work item this step, as
// in decode, SSM beam steps and tree verify): the workgroup first applies its
// own request's TREE commits and the KV update of its own tokens for its
// head (kv_update_kernel's work), makes them visible to the workgroup, then
// attends -- one launch per step instead of two.
//
// OP (FUSED, QT == 1; OprojArgs in ffmi_internal.h): the workgroup also
// multiplies its rounded output rows by its head's K-slice of Wo (MFMA with
// the packed weight block as the A operand and the output rows, from LDS, as
// B -- the S^T = K.Q^T arrangement) and stores the fp32 product as slab
// `head`.  The slice is loaded after the key loop, so the merge hides its
// latency; wave w owns column tiles w, w + NW, ... (N <= 16 * 8 * NW).
//
// QS == 2 (FUSED, QT == 1; grids with CUs to spare: TP >= 2 verify steps,
// <= 128 (request, head) pairs): the item's queries are split over two
// workgroups (blockIdx.z = which 16), each running the whole item's commits
// and KV update -- the same values to the same addresses, and every K/V it
// reads from memory is below the tail, which neither writes -- and attending
// its own 16: the key loop and merge work per workgroup halve.  Per query the
// arithmetic is the QT == 2 kernel's (MFMA columns are independent), so the
// output is bit-identical.
template <int D, int QT, int NW, bool FUSED, bool ST = false, int PSRC = -1, bool OP = false,
          int QS = 1>
__global__ __launch_bounds__(64 * NW, 1) void attention_kernel(
    const char *__restrict__ blob, uint16_t *__restrict__ qbuf, uint16_t *__restrict__ kc,
    uint16_t *__restrict__ vc, uint16_t *__restrict__ out, int heads, int slots, float scale,
    int out_packed, KvUpdateArgs kv, OprojArgs opa) {
  static_assert(!OP || (FUSED && QT == 1 && QS == 1), "output projection: fused, one query tile");
  static_assert(QS == 1 || (FUSED && QT == 1 && QS == 2), "query split: fused, 2 x 16 queries");
  constexpr int KS = D / 32;  // k-steps of the QK^T product
  constexpr int DT = D / 16;  // d-tiles of the PV product
  constexpr int NQ = 16 * QT;   // queries this workgroup attends
  constexpr int NQK = NQ * QS;  // tokens of the item (commits, KV update)
  const int qbase = QS > 1 ? (int)blockIdx.z * NQ : 0;
  constexpr int TS = kTailSlots;
  __shared__ float sm_m[NW][NQ];
  __shared__ float sm_l[NW][NQ];
  // the merge buffer shares its LDS with the FUSED tail tile (K rows and V^T
  // columns of slots [tail0, tail0 + TS)); a barrier separates their uses
  constexpr int SMO_BYTES = NW * QT * DT * 4 * 64 * 4;
  constexpr int TAIL_BYTES = FUSED ? (TS * (D + 8) + D * (TS + 8)) * 2 : 0;
  __shared__ __attribute__((aligned(16)))
  char smem[SMO_BYTES > TAIL_BYTES ? SMO_BYTES : TAIL_BYTES];
  auto sm_o = reinterpret_cast<float(*)[QT][DT][4][64]>(smem);
  auto sKt = reinterpret_cast<uint16_t(*)[D + 8]>(smem);
  auto sVt = reinterpret_cast<uint16_t(*)[TS + 8]>(smem + TS * (D + 8) * 2);

  // ST: lane 0 of each wave stores its timeline straight to kv.stamps
  long long *stp = nullptr;
  if (ST && kv.stamps && (threadIdx.x & 63) == 0)
    stp = kv.stamps + ((size_t)(blockIdx.y * gridDim.x + blockIdx.x) * NW + (threadIdx.x >> 6)) * 12;
  auto stamp = [&](int i) {
    if (ST && stp) stp[i] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int qi = lane & 15;
  const int g = lane >> 4;
  const int h = blockIdx.y;
  const BatchView bv = batch_view(blob);
  // (fields, not a copy of the WorkDev: a private copy of its rope_pos array
  // would be indexed per lane and live in scratch)
  const ffmi_attn_work w = bv.work[blockIdx.x].w;
  const int Hl = heads * D;
  const uint16_t *kbase = kc + ((size_t)w.req * heads + h) * slots * D;
  const uint16_t *vbase = vc + ((size_t)w.req * heads + h) * D * slots;
  // K rows and V^T columns of one 32-key chunk (chunk indices are clamped by
  // the caller: the cache is allocated to a multiple of 32 slots)
  auto load_chunk = [&](int c, h8 (&kf)[2][KS], h8 (&va)[DT]) {
    const int base = c * 32;
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      const uint16_t *krow = kbase + (size_t)(base + sub * 16 + (lane & 15)) * D + 8 * g;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) kf[sub][ks] = *reinterpret_cast<const h8 *>(krow + 32 * ks);
    }
#pragma unroll
    for (int t = 0; t < DT; ++t) {
      const uint16_t *vrow = vbase + (size_t)(t * 16 + (lane & 15)) * slots + base + 4 * g;
      h4 v0 = *reinterpret_cast<const h4 *>(vrow);
      h4 v1 = *reinterpret_cast<const h4 *>(vrow + 16);
      va[t] = h8{v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
    }
  };
  // FUSED: every slot this step writes for the request (its stores and TREE
  // commits) lies in the LDS tail [tail0, kv_len) (host-checked, lds_tail);
  // the keys below tail0 are untouched this step, so their chunks load from
  // HBM at any time and a wave's first one goes out with the prologue's
  // loads.  The tail's chunks are read from LDS: the prologue writes the new
  // K/V there as well as to HBM, and the attention never waits for its own
  // global stores.
  const int nchunks = (w.kv_len + 31) >> 5;
  const int tail0 = FUSED ? bv.work[blockIdx.x].tail0 : w.kv_len;
  const int ctail = tail0 >> 5;  // first chunk read from the LDS tail
  h8 kf0[2][KS], va0[DT];
  const bool early = FUSED && wave < nchunks && wave < ctail;

  // OP: this head's K-slice of Wo (k-steps h*KS .. h*KS + KS - 1) for the
  // wave's column tiles, issued right behind the prologue's loads (and the
  // first K/V chunk), so the KV update, key loop and merge hide its latency
  constexpr int OT = OP ? 8 : 1;
  h8 wo_f[OT][KS];
  const int o_tiles = OP ? opa.N >> 4 : 0;
  auto load_wo = [&]() {
    if constexpr (OP) {
#pragma unroll
      for (int j = 0; j < OT; ++j) {
        const int t = (wave + j * NW) * (int)gridDim.z + (int)blockIdx.z;  // (column split)
        if (t < o_tiles) {
#pragma unroll
          for (int ks = 0; ks < KS; ++ks)
            wo_f[j][ks] = *reinterpret_cast<const h8 *>(opa.wo + (size_t)t * opa.wts +
                                                        (size_t)(h * KS + ks) * opa.wks + lane * 8);
        }
      }
    }
  };

  // FUSED: this item's rotated queries stay in LDS (rows padded by 16 B)
  __shared__ __attribute__((aligned(16))) uint16_t sQ[FUSED ? NQK : 1][D + 8];
  __shared__ int4 sMrec[FUSED ? NQK : 1];
  __shared__ int sSlotV[FUSED ? NQK : 1];
  __shared__ uint64_t sMvis[FUSED ? NQK : 1];
  if (FUSED) {
    int *sSlot = sSlotV;
    const WorkDev *wdp = &bv.work[blockIdx.x];
    // the queries' visibility records go out with the prologue's loads and
    // reach the key loop through LDS (a load there was one more round trip)
    int4 mrec;
    uint64_t mvis;
    constexpr int NT = 64 * NW;
    constexpr int D8 = D / 8;
    // cached contents of the tail's first `told` (< 32) slots, which this
    // step does not write, 16-B pieces: K rows, then V^T row segments (the
    // V^T pieces cover the whole first chunk; the written slots among them
    // are overwritten in LDS after the barrier below)
    constexpr int TK = (32 * D8 + NT - 1) / NT, TV = (D * 4 + NT - 1) / NT;
    const int told = bv.work[blockIdx.x].told;
    uint4 tk[TK], tv[TV];
    // the request's commits (16-B pieces of the staging K and V rows)
    constexpr int CP = (kItemCommits * 2 * D8 + NT - 1) / NT;
    const int ncm = kv.C > 0 ? wdp->ncommit : 0;
    // commit sources through the scalar cache, with the work item: the
    // staging loads then wait on no vector load (one round trip, not two)
    // (readfirstlane keeps them scalar: a select over the loaded words was
    // folded into a per-lane load that the staging loads then waited for)
    const uint32_t *cs32 = reinterpret_cast<const uint32_t *>(wdp->cm_src);
    uint32_t csw[kItemCommits / 2];
#pragma unroll
    for (int jj = 0; jj < kItemCommits / 2; ++jj) csw[jj] = __builtin_amdgcn_readfirstlane(cs32[jj]);
    int csrc[CP];  // this thread's commit pieces: source staging rows
#pragma unroll
    for (int i = 0; i < CP; ++i) {
      const int j = min(((int)threadIdx.x + i * NT) / (2 * D8), kItemCommits - 1);
      uint32_t wd = csw[0];
#pragma unroll
      for (int jj = 1; jj < kItemCommits / 2; ++jj) wd = (j >> 1) == jj ? csw[jj] : wd;
      csrc[i] = (int)(int16_t)((j & 1) ? (wd >> 16) : (wd & 0xffffu));
    }
    uint4 cmv[CP];
    kv_update_item<D, NQK, NT, PSRC>(
        bv, wdp, h, heads, slots, kv.T, kv.qkv, kv.part, kv.pS, kv.pNP, kv.rope, kv.max_rope_pos,
        qbuf, kc, kv.stage_wr, nullptr, sSlot, sQ, sKt, sVt, tail0,
        [&] {  // after the KV update's own loads: commits, tail, first chunk
#pragma unroll
          for (int i = 0; i < CP; ++i) {
            const int e = threadIdx.x + i * NT, j = e / (2 * D8), r = e % (2 * D8);
            if (j < ncm) {
              const int src = csrc[i];
              cmv[i] = *reinterpret_cast<const uint4 *>(
                  kv.stage_rd + (size_t)src * 2 * Hl + (r >= D8 ? Hl : 0) + h * D + (r % D8) * 8);
            }
          }
#pragma unroll
          for (int i = 0; i < TK; ++i) {
            const int e = threadIdx.x + i * NT, row = e / D8;
            if (row < told)
              tk[i] = *reinterpret_cast<const uint4 *>(kbase + (size_t)(tail0 + row) * D + (e % D8) * 8);
          }
#pragma unroll
          for (int i = 0; i < TV; ++i) {
            const int e = threadIdx.x + i * NT, dd = e / 4, s8 = (e % 4) * 8;
            if (dd < D && s8 < told)
              tv[i] = *reinterpret_cast<const uint4 *>(vbase + (size_t)dd * slots + tail0 + s8);
          }
          if ((int)threadIdx.x < NQK) {
            const ffmi_token_info *ti = &bv.tokens[w.q_start + min((int)threadIdx.x, max(w.q_count - 1, 0))];
            mrec = make_int4(ti->prefix_len, ti->tree_base, ti->tree_len, 0);
            mvis = ti->tree_vis;
          }
          // (issued last: the waits below for the loads above leave it in flight)
          if (early) load_chunk(wave, kf0, va0);
          load_wo();
        },
        [&] {  // loads are back: the old tail to LDS, then the commits
          stamp(10);
          if ((int)threadIdx.x < NQK) sMrec[threadIdx.x] = mrec, sMvis[threadIdx.x] = mvis;
#pragma unroll
          for (int i = 0; i < TK; ++i) {
            const int e = threadIdx.x + i * NT, row = e / D8;
            if (row < told) *reinterpret_cast<uint4 *>(&sKt[row][(e % D8) * 8]) = tk[i];
          }
#pragma unroll
          for (int i = 0; i < TV; ++i) {
            const int e = threadIdx.x + i * NT, dd = e / 4, s8 = (e % 4) * 8;
            if (dd < D && s8 < told) {
              uint2 *dst = reinterpret_cast<uint2 *>(&sVt[dd][s8]);  // rows are 8-B aligned
              dst[0] = make_uint2(tv[i].x, tv[i].y);
              dst[1] = make_uint2(tv[i].z, tv[i].w);
            }
          }
          stamp(11);
          // keys past kv_len in the last chunk are masked, but P.V still
          // multiplies their V by 0: zero them (as the cache's never-written
          // slots are); a stored slot among them is written after the barrier
          for (int e = threadIdx.x; e < D * 32; e += NT) {
            const int dd = e >> 5, sl = w.kv_len - tail0 + (e & 31);
            if (sl < (nchunks - ctail) * 32) sVt[dd][sl] = 0;
          }
          __syncthreads();
          // commits (tree_inc...cu:335-396): staging row -> depth slot, in
          // HBM and in the tail (their slots differ from this step's stores:
          // a coinciding commit was applied by its own launch, kv.C == 0)
#pragma unroll
          for (int i = 0; i < CP; ++i) {
            const int e = threadIdx.x + i * NT, j = e / (2 * D8), r = e % (2 * D8);
            if (j >= ncm) continue;
            const int dep = wdp->cm_depth[j], i8 = (r % D8) * 8;
            if (dep < 0 || dep >= slots) continue;
            const int ts = dep - tail0;
            if (r < D8) {
              *reinterpret_cast<uint4 *>(kc + (((size_t)w.req * heads + h) * slots + dep) * D + i8) =
                  cmv[i];
              *reinterpret_cast<uint4 *>(&sKt[ts][i8]) = cmv[i];
            } else {
              uint16_t *vt = vc + (((size_t)w.req * heads + h) * D + i8) * slots + dep;
              const uint32_t vw[4] = {cmv[i].x, cmv[i].y, cmv[i].z, cmv[i].w};
#pragma unroll
              for (int jj = 0; jj < 8; ++jj) {
                const uint16_t v = (uint16_t)(vw[jj >> 1] >> (16 * (jj & 1)));
                vt[(size_t)jj * slots] = v;
                sVt[i8 + jj][ts] = v;
              }
            }
          }
          stamp(6);
        });
    stamp(7);
    __syncthreads();
    stamp(8);
    stamp(9);
  }

  stamp(1);
  bool qvalid[QT];
  int pre[QT], tb[QT], tlen[QT];
  uint64_t tv[QT];
  h8 qf[QT][KS];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    const int q = qbase + qt * 16 + qi;
    qvalid[qt] = q < w.q_count;
    if (FUSED) {
      const int4 mr = sMrec[qvalid[qt] ? q : 0];
      pre[qt] = mr.x, tb[qt] = mr.y, tlen[qt] = mr.z, tv[qt] = sMvis[qvalid[qt] ? q : 0];
    } else {
      const ffmi_token_info ti = bv.tokens[w.q_start + (qvalid[qt] ? q : 0)];
      pre[qt] = ti.prefix_len, tb[qt] = ti.tree_base, tlen[qt] = ti.tree_len, tv[qt] = ti.tree_vis;
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      qf[qt][ks] = !qvalid[qt] ? h8{0, 0, 0, 0, 0, 0, 0, 0}
                   : FUSED ? *reinterpret_cast<const h8 *>(&sQ[q][32 * ks + 8 * g])
                           : *reinterpret_cast<const h8 *>(
                                 qbuf + (size_t)(w.q_start + q) * Hl + h * D + 32 * ks + 8 * g);
  }

  const float NEG = -INFINITY;
  float m_run[QT], l_run[QT];
  f4 o[QT][DT];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    m_run[qt] = NEG, l_run[qt] = 0.f;
#pragma unroll
    for (int t = 0; t < DT; ++t) o[qt][t] = f4{0.f, 0.f, 0.f, 0.f};
  }

  auto compute_chunk = [&](int base, const h8 (&kf)[2][KS], const h8 (&va)[DT]) {
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
  };
  // wave w takes chunks w, w+NW, ... (two waves per SIMD hide each other's
  // load latency; per-wave double buffering would not fit the registers)
  // FUSED: chunks from ctail on come from the LDS tail
  auto load_chunk_lds = [&](int lc, h8 (&kf)[2][KS], h8 (&va)[DT]) {
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      const uint16_t *krow = &sKt[lc * 32 + sub * 16 + (lane & 15)][8 * g];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) kf[sub][ks] = *reinterpret_cast<const h8 *>(krow + 32 * ks);
    }
#pragma unroll
    for (int t = 0; t < DT; ++t) {
      const uint16_t *vrow = &sVt[t * 16 + (lane & 15)][lc * 32 + 4 * g];
      h4 v0 = *reinterpret_cast<const h4 *>(vrow);
      h4 v1 = *reinterpret_cast<const h4 *>(vrow + 16);
      va[t] = h8{v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
    }
  };
  stamp(2);
  for (int c = wave; c < nchunks; c += NW) {
    if (early && c == wave) {
      compute_chunk(c * 32, kf0, va0);
      continue;
    }
    h8 kf[2][KS], va[DT];
    if (FUSED && c >= ctail) load_chunk_lds(c - ctail, kf, va);
    else load_chunk(c, kf, va);
    compute_chunk(c * 32, kf, va);
  }

  stamp(3);
  if (FUSED) {
    // V^T of this step's tokens to HBM from the tail, by each wave once its
    // key loop is done (not waited for)
    uint16_t *vt = vc + ((size_t)w.req * heads + h) * D * slots;
    for (int e = threadIdx.x; e < D * NQK; e += blockDim.x) {
      const int dd = e / NQK, tt = e % NQK;
      if (tt >= w.q_count) continue;
      const int sl = sSlotV[tt];
      if (sl >= 0) vt[(size_t)dd * slots + sl] = sVt[dd][sl - tail0];
    }
    __syncthreads();  // the merge buffer reuses the tail's LDS
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
  stamp(4);

  // merge: wave w finalizes d-tiles t = w, w+NW, ... of every query tile
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    const int ql = qt * 16 + qi, q = qbase + ql;  // in the workgroup / in the item
    float M = NEG;
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) M = fmaxf(M, sm_m[ww][ql]);
    float f[NW], L = 0.f;
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) {
      const float mw = sm_m[ww][ql];
      f[ww] = (mw == NEG) ? 0.f : __expf(mw - M);
      L += f[ww] * sm_l[ww][ql];
    }
    const float inv = 1.0f / (L + 1e-6f);
    if (!qvalid[qt]) continue;
    const int orow_m = w.q_start + q;
    uint16_t *orow = out + (size_t)orow_m * Hl + h * D;
    for (int t = wave; t < DT; t += NW) {
      uint16_t r4[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float acc = 0.f;
#pragma unroll
        for (int ww = 0; ww < NW; ++ww) acc += f[ww] * sm_o[ww][qt][t][r][lane];
        r4[r] = f2h(acc * inv);
      }
      uint2 pk;
      pk.x = r4[0] | ((uint32_t)r4[1] << 16);
      pk.y = r4[2] | ((uint32_t)r4[3] << 16);
      uint16_t *dst = out_packed ? out + act_packed_off(orow_m, h * D + t * 16 + 4 * g, Hl)
                                 : orow + t * 16 + 4 * g;
      *reinterpret_cast<uint2 *>(dst) = pk;
      // OP: the rounded row also to LDS (the queries' tile is free by now)
      if (OP) *reinterpret_cast<uint2 *>(&sQ[q][t * 16 + 4 * g]) = pk;
    }
  }
  if constexpr (OP) {
    // slab[head][token][n] = sum_d out[token][head*d + d] * Wo[n][head*d + d]:
    // lane (qi, g) ends with n = 16 t + 4 g + r of query qi.  Rows of queries
    // past q_count hold stale LDS; their columns are computed, never stored.
    __syncthreads();
    h8 xb[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) xb[ks] = *reinterpret_cast<const h8 *>(&sQ[qi][32 * ks + 8 * g]);
    const bool qv = qi < w.q_count;
    float *srow = opa.slab + ((size_t)h * kv.T + w.q_start + qi) * opa.N + 4 * g;
#pragma unroll
    for (int j = 0; j < OT; ++j) {
      const int t = (wave + j * NW) * (int)gridDim.z + (int)blockIdx.z;
      if (t < o_tiles) {
        f4 c = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(wo_f[j][ks], xb[ks], c, 0, 0, 0);
        if (qv) *reinterpret_cast<f4 *>(srow + t * 16) = c;
      }
    }
  }
  if (ST && stp) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stamp(5);
  }
}

// Query split (attention_kernel QS == 2) of a fused launch with more than 16
// queries per item: when the (item, head) grid leaves half the CUs idle
// (TP >= 2 verify steps).  FFMI_ATTN_QSPLIT: 0 off, 1 auto (default), 2
// always (tests; read at every launch, so a test can switch it).
// a doubled grid still fits one wave of the device's CUs
static bool attn_split_fits(int wgs) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
  }
  return 2 * wgs <= cus;
}

static bool attn_qsplit(int wgs) {
  const char *e = getenv("FFMI_ATTN_QSPLIT");
  const int mode = e ? atoi(e) : 1;
  return mode == 2 || (mode == 1 && attn_split_fits(wgs));
}

static bool attn_osplit(int wgs) {
  const char *e = getenv("FFMI_ATTN_OSPLIT");
  const int mode = e ? atoi(e) : 1;
  return mode == 2 || (mode == 1 && attn_split_fits(wgs));
}

template <int D>
static hipError_t launch_attention_d(const char *blob, int W, int max_q, uint16_t *qbuf,
                                     uint16_t *kc, uint16_t *vc, uint16_t *out, int heads,
                                     int slots, float scale, hipStream_t s, int op, bool fused,
                                     const KvUpdateArgs &kv) {
  const dim3 grid(W, heads);
#define FFMI_ATT(QT, FU)                                                                      \
  do {                                                                                          \
    if (!FU)                                                                                    \
      hipLaunchKernelGGL((attention_kernel<D, QT, 8, false>), grid, dim3(512), 0, s, blob, qbuf, \
                         kc, vc, out, heads, slots, scale, op, kv, OprojArgs());                             \
    else if (kv.part)                                                                           \
      hipLaunchKernelGGL((attention_kernel<D, QT, 8, true, false, 1>), grid, dim3(512), 0, s,    \
                         blob, qbuf, kc, vc, out, heads, slots, scale, op, kv, OprojArgs());                 \
    else                                                                                        \
      hipLaunchKernelGGL((attention_kernel<D, QT, 8, true, false, 0>), grid, dim3(512), 0, s,    \
                         blob, qbuf, kc, vc, out, heads, slots, scale, op, kv, OprojArgs());                 \
  } while (0)
  // diagnostics build: FFMI_ATTN_STAMP=1 stamps the d = 128 (LLM) launches,
  // FFMI_ATTN_STAMP=64 the d = 64 (68M SSM) ones
  static const int stamp_d = getenv("FFMI_ATTN_STAMP") && atoi(getenv("FFMI_ATTN_STAMP")) == 64 ? 64 : 128;
  if (kv.stamps && D == stamp_d) {
#define FFMI_ATT_ST(QT)                                                                         \
  do {                                                                                          \
    if (fused)                                                                                  \
      hipLaunchKernelGGL((attention_kernel<D, QT, 8, true, true>), grid, dim3(512), 0, s, blob,  \
                         qbuf, kc, vc, out, heads, slots, scale, op, kv, OprojArgs());                       \
    else                                                                                        \
      hipLaunchKernelGGL((attention_kernel<D, QT, 8, false, true>), grid, dim3(512), 0, s, blob, \
                         qbuf, kc, vc, out, heads, slots, scale, op, kv, OprojArgs());                       \
  } while (0)
    if (max_q > 16) FFMI_ATT_ST(2);
    else FFMI_ATT_ST(1);
#undef FFMI_ATT_ST
    return hipGetLastError();
  }
  if (max_q > 16 && fused && attn_qsplit(W * heads)) {
    const dim3 grid2(W, heads, 2);
    if (kv.part)
      hipLaunchKernelGGL((attention_kernel<D, 1, 8, true, false, 1, false, 2>), grid2, dim3(512), 0,
                         s, blob, qbuf, kc, vc, out, heads, slots, scale, op, kv, OprojArgs());
    else
      hipLaunchKernelGGL((attention_kernel<D, 1, 8, true, false, 0, false, 2>), grid2, dim3(512), 0,
                         s, blob, qbuf, kc, vc, out, heads, slots, scale, op, kv, OprojArgs());
    return hipGetLastError();
  }
  // FFMI_ATTN_NW4=1 (A/B): fused one-query-tile launches (decode, SSM beam
  // steps) with 4 waves per workgroup instead of 8
  static const bool nw4 = getenv("FFMI_ATTN_NW4") && atoi(getenv("FFMI_ATTN_NW4")) != 0;
  if (max_q <= 16 && fused && nw4 && D == 128) {
    if (kv.part)
      hipLaunchKernelGGL((attention_kernel<D, 1, 4, true, false, 1>), grid, dim3(256), 0, s, blob,
                         qbuf, kc, vc, out, heads, slots, scale, op, kv, OprojArgs());
    else
      hipLaunchKernelGGL((attention_kernel<D, 1, 4, true, false, 0>), grid, dim3(256), 0, s, blob,
                         qbuf, kc, vc, out, heads, slots, scale, op, kv, OprojArgs());
    return hipGetLastError();
  }
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

// FFMI_ATTN_STAMP=1: d = 128 launches record a per-wave timeline
// {start, after prologue, before k-loop, after k-loop, after merge barrier,
// end, [fused] after commits, after KV update, after its barrier, after the
// V^T stores, HW_ID, chunks} (100 MHz realtime) for ffmi_debug_attn_stamps.
static long long *g_attn_stamps = nullptr;
static long g_attn_stamp_waves = 0;
static bool g_attn_stamp_gate = true;
// the model closes the gate for every launch but the one its markers bracket
void attn_stamp_gate(bool open) { g_attn_stamp_gate = open; }
static long long *attn_stamp_buf(int wgs) {
  static const bool on = getenv("FFMI_ATTN_STAMP") != nullptr;
  if (!on) return nullptr;
  // (allocated on the first launch, gate open or not: a later first use may
  // sit inside a graph capture, where hipMalloc fails)
  if (!g_attn_stamps && hipMalloc(&g_attn_stamps, (size_t)8 << 20) != hipSuccess) return nullptr;
  if (!g_attn_stamp_gate) return nullptr;
  g_attn_stamp_waves = std::min<long>((long)wgs * 8, ((long)8 << 20) / 96);
  return g_attn_stamps;
}

// FFMI_MARKERS=1 diagnostics: a one-wave kernel that records the 100 MHz
// realtime clock (the attention stamps' clock) into slot i when it starts,
// enqueued between the kernels of the model's last layer: with the wave
// stamps it splits a launch's duration into boundary and in-kernel time.
__global__ void marker_kernel(long long *buf, int i) {
  if (threadIdx.x == 0) buf[i] = __builtin_amdgcn_s_memrealtime();
}
static long long *g_markers = nullptr;
hipError_t launch_marker(int i, hipStream_t s) {
  if (i < 0 || i >= 64) return hipErrorInvalidValue;
  if (!g_markers && hipMalloc(&g_markers, 64 * sizeof(long long)) != hipSuccess)
    return hipErrorOutOfMemory;
  hipLaunchKernelGGL(marker_kernel, dim3(1), dim3(64), 0, s, g_markers, i);
  return hipGetLastError();
}
long debug_markers(long long *dst, long n) {
  if (!g_markers || n <= 0) return 0;
  n = std::min<long>(n, 64);
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpy(dst, g_markers, (size_t)n * sizeof(long long), hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  return n;
}

long attn_debug_stamps(long long *dst, long max_waves) {
  if (!g_attn_stamps || max_waves <= 0) return 0;
  const long n = std::min(max_waves, g_attn_stamp_waves);
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpy(dst, g_attn_stamps, (size_t)n * 96, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return n;
}

// fused == false: the KV of this step must already be in the cache
// (launch_kv_update); fused == true: one workgroup per request (checked by the
// caller) does commits + KV update + attention.
hipError_t launch_attention(const char *blob, int W, int max_q, uint16_t *qbuf, uint16_t *kc,
                            uint16_t *vc, uint16_t *out, int heads, int d, int slots, float scale,
                            hipStream_t s, bool out_packed, bool fused, int T, int C,
                            const uint16_t *qkv, Partials qkvp, uint16_t *stage_wr,
                            const uint16_t *stage_rd, const float *rope, int max_rope_pos,
                            const OprojArgs *opa) {
  if (W <= 0) return hipSuccess;
  if (out_packed && (heads * d) % 32) return hipErrorInvalidValue;
  if (max_q > FFMI_ATTN_QTILE) return hipErrorInvalidValue;
  const KvUpdateArgs kv{T,        C,        qkv,  qkvp.S > 0 ? qkvp.p : nullptr,
                        qkvp.S,   qkvp.NP,  stage_wr, stage_rd,
                        rope,     max_rope_pos, attn_stamp_buf(W * heads)};
  const int op = out_packed ? 1 : 0;
  if (opa) {  // output projection folded in (the caller checked fused, d, max_q, N)
    if (!fused || d != 64 || max_q > 16 || opa->N % 16 || opa->N > 16 * 8 * 8 || T > opa->max_T)
      return hipErrorInvalidValue;
    // output-column split: when the (item, head) grid leaves half the CUs
    // idle (the 68M SSM: 8 x 12 = 96 workgroups), two workgroups per (item,
    // head) each project half of the column tiles; both attend and run the
    // KV update (the same values to the same addresses, as the query split).
    // The projection's weight slice (96 KiB) and MFMAs per workgroup halve:
    // SSM step 102.9 -> 100.4 us over 5 same-box pairs (profiles/r04_attn_osplit_ab.log).
    // FFMI_ATTN_OSPLIT: 0 off, 1 auto (default), 2 always (read per launch).
    const dim3 grid(W, heads, attn_osplit(W * heads) ? 2 : 1);
    if (kv.part)
      hipLaunchKernelGGL((attention_kernel<64, 1, 8, true, false, 1, true>), grid, dim3(512), 0, s,
                         blob, qbuf, kc, vc, out, heads, slots, scale, op, kv, *opa);
    else
      hipLaunchKernelGGL((attention_kernel<64, 1, 8, true, false, 0, true>), grid, dim3(512), 0, s,
                         blob, qbuf, kc, vc, out, heads, slots, scale, op, kv, *opa);
    return hipGetLastError();
  }
  if (d == 128)
    return launch_attention_d<128>(blob, W, max_q, qbuf, kc, vc, out, heads, slots, scale, s, op,
                                   fused, kv);
  if (d == 64)
    return launch_attention_d<64>(blob, W, max_q, qbuf, kc, vc, out, heads, slots, scale, s, op,
                                  fused, kv);
  if (d == 32)  // incremental decoding's third head size (inc...cu:911-926)
    return launch_attention_d<32>(blob, W, max_q, qbuf, kc, vc, out, heads, slots, scale, s, op,
                                  fused, kv);
  return hipErrorInvalidValue;
}

}  // namespace ffmi
