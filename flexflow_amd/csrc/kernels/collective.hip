// collective.hip -- direct xGMI all-reduce over peer exchange buffers.
//
// Replaces the reference's ncclAllReduce (allreduce_kernels.cu:53-75, run as
// a concurrent Legion task per shard, allreduce.cc:291-331) for the
// tensor-parallel LLaMA step.  Each rank owns one exchange buffer (uncached
// device memory, exported with hipIpcGetMemHandle and mapped by every peer of
// the node); a
// single kernel per all-reduce does
//   1. copy-in: this rank's partial -> its own exchange buffer (area `in`,
//      parity e & 1 of the all-reduce epoch e);
//   2. signal: the last workgroup to finish the copy pushes e into every
//      rank's inbox slot for this rank (a system-scope release store over
//      xGMI; its own slot too, for its own early workgroups), so every rank
//      polls its LOCAL memory;
//   3. one-shot (small messages): every rank reads all N partials and sums
//      them in rank order 0..N-1 in fp32 -> bit-identical result on every
//      rank;
//      two-shot (large messages): rank r reduces chunk r of the vector
//      (reading it from every peer), publishes it in its `out` area, signals
//      again, then gathers the other chunks from their owners;
//   4. the last workgroup to finish stores epoch e for the next launch.
// The epoch lives in device memory, so the kernel's arguments are the same
// on every launch and the whole step can be captured in a HIP graph.
//
// Reuse of the parity-p areas at epoch e + 2 is safe without extra flags:
// a rank signals epoch e + 1 only after its all-reduce e has finished every
// read of its peers' epoch-e areas (stream order), and it waits for every
// peer's e + 1 signal before it writes a parity-p area again.
//
// Every wait is bounded (FFMI_PEER_TIMEOUT_S, default 10 s of s_memrealtime at
// 100 MHz): a dead or missing peer sets the communicator's host-visible error
// word and the kernel exits, so a broken exchange is an error, never a hang.
//
// All flag and counter stores are ordinary vector stores/atomics to global
// memory.
#include "../ffmi_internal.h"
#include "../collective.h"

namespace ffmi {

namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ void report_timeout(int *err, int code) {
  // host-mapped word (pinned), read after the step's stream synchronisation
  __hip_atomic_store(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// All workgroups arrive; the last one (returns true) may act for the grid.
__device__ __forceinline__ bool arrive_last(unsigned *cnt, unsigned G) {
  __shared__ unsigned last;
  __syncthreads();  // every wave of this workgroup has issued its stores
  if (threadIdx.x == 0) {
    // release at system scope: this workgroup's stores (its XCD's L2) are
    // written back before the count moves; acquire: the last arriver sees
    // every other workgroup's stores
    const unsigned old =
        __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_SYSTEM);
    last = old == G - 1 ? 1u : 0u;
    if (last) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  return last != 0;
}

// Push epoch e into every rank's inbox slot for this rank -- this rank's own
// slot included: the workgroups that arrived early must not read this rank's
// area before its LAST workgroup has finished writing it.
__device__ __forceinline__ void push_flags(const PeerArgs &a, size_t inbox_off, unsigned e) {
  for (int p = 0; p < a.nranks; ++p) {
    unsigned *f = reinterpret_cast<unsigned *>(a.base[p] + inbox_off + (size_t)a.rank * kFlagStride);
    __hip_atomic_store(f, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// Wait until every slot (every rank, this one included) of this rank's inbox
// holds >= e.  Returns false on timeout (error word set).
__device__ __forceinline__ bool wait_flags(const PeerArgs &a, size_t inbox_off, unsigned e,
                                           int code) {
  __shared__ int ok;
  if (threadIdx.x == 0) ok = 1;
  __syncthreads();
  const int p = threadIdx.x;
  if (p < a.nranks) {
    const unsigned *f =
        reinterpret_cast<const unsigned *>(a.base[a.rank] + inbox_off + (size_t)p * kFlagStride);
    const uint64_t t0 = wall_clock64();
    // peers are at most one epoch ahead (see the header), so >= e
    while ((int)(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - e) < 0) {
      __builtin_amdgcn_s_sleep(2);
      if (wall_clock64() - t0 > a.timeout_ticks) {
        report_timeout(a.err, code);
        ok = 0;
        break;
      }
    }
  }
  __syncthreads();
  // acquire (system scope: L1 and L2 invalidated): later loads of peer
  // areas see what the peers released, not lines cached two epochs ago
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  return ok != 0;
}

template <int DT>  // 0: f16, 1: f32
__device__ __forceinline__ void acc_vec(float (&acc)[8], uint4 v) {
  if constexpr (DT == 0) {
    const h8 h = __builtin_bit_cast(h8, v);
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] += (float)h[i];
  } else {
    const f4 f = __builtin_bit_cast(f4, v);
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] += f[i];
  }
}

template <int DT>
__device__ __forceinline__ uint4 pack_vec(const float (&acc)[8]) {
  if constexpr (DT == 0) {
    h8 h;
#pragma unroll
    for (int i = 0; i < 8; ++i) h[i] = (_Float16)acc[i];
    return __builtin_bit_cast(uint4, h);
  } else {
    f4 f;
#pragma unroll
    for (int i = 0; i < 4; ++i) f[i] = acc[i];
    return __builtin_bit_cast(uint4, f);
  }
}

// Vector v (16 B) of the logical [rows][cols] input -> its place in the
// strided output (row stride ld elements, column offset col0).
__device__ __forceinline__ uint4 *out_vec(const PeerArgs &a, size_t v) {
  const size_t e = v * a.vec_elems;
  const size_t row = e / a.cols, col = e % a.cols;
  return reinterpret_cast<uint4 *>(reinterpret_cast<char *>(a.out) +
                                   ((row * a.ld + a.col0 + col) * a.esz));
}

// copy-in of a split-K partial: the 8 fp16 outputs of vector v, every slab
// load issued before the first add (MAXS >= S; indices past S re-read the
// last slab and are not added), summed in slab order and rounded once
template <int MAXS>
__device__ __forceinline__ uint4 slab_vec(const PeerArgs &a, size_t v) {
  const size_t e = v * 8, row = e / a.cols, col = e % a.cols;
  const float *q = a.slabs + row * a.NP + col;
  const size_t slab = a.rows * a.NP;
  f4 lo[MAXS], hi[MAXS];
#pragma unroll
  for (int s = 0; s < MAXS; ++s) {
    const float *qs = q + (size_t)min(s, a.S - 1) * slab;
    lo[s] = *reinterpret_cast<const f4 *>(qs);
    hi[s] = *reinterpret_cast<const f4 *>(qs + 4);
  }
  f4 l = lo[0], h = hi[0];
#pragma unroll
  for (int s = 1; s < MAXS; ++s)
    if (s < a.S) l += lo[s], h += hi[s];
  h8 o;
#pragma unroll
  for (int i = 0; i < 4; ++i) o[i] = (_Float16)l[i], o[i + 4] = (_Float16)h[i];
  return __builtin_bit_cast(uint4, o);
}

template <int DT, bool TWO_SHOT, int MAXS = 0, bool RS = false>
__global__ __launch_bounds__(kThreads) void peer_allreduce_kernel(PeerArgs a) {
  char *own = a.base[a.rank];
  unsigned *hdr = reinterpret_cast<unsigned *>(own + kHdrCounters);
  const unsigned e = hdr[kEpochWord] + 1u;  // written by the previous launch
  const size_t par = e & 1u;
  const size_t in_off = kDataOff + par * a.cap;
  const size_t out_off = kDataOff + (2 + par) * a.cap;
  const unsigned G = gridDim.x;
  const size_t stride = (size_t)G * kThreads;
  const size_t tid0 = (size_t)blockIdx.x * kThreads + threadIdx.x;

  // 1. copy-in (MAXS > 0: the sum of the GEMM's split-K slabs)
  {
    uint4 *dst = reinterpret_cast<uint4 *>(own + in_off);
    if constexpr (MAXS > 0) {
      for (size_t v = tid0; v < a.nvec; v += stride) dst[v] = slab_vec<MAXS>(a, v);
    } else {
      const uint4 *src = reinterpret_cast<const uint4 *>(a.in);
      for (size_t v = tid0; v < a.nvec; v += stride) dst[v] = src[v];
    }
  }
  // 2. signal
  if (arrive_last(&hdr[kCnt0], G) && threadIdx.x == 0) push_flags(a, kInbox0, e);
  if (!wait_flags(a, kInbox0, e, 1)) return;

  if constexpr (!TWO_SHOT) {
    // 3a. one-shot: every rank sums all N partials in rank order
    for (size_t v = tid0; v < a.nvec; v += stride) {
      float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int p = 0; p < a.nranks; ++p)
        acc_vec<DT>(acc, reinterpret_cast<const uint4 *>(a.base[p] + in_off)[v]);
      *out_vec(a, v) = pack_vec<DT>(acc);
    }
  } else if constexpr (RS) {
    // 3c. reduce-scatter by rows: this rank's rows of the sum, kept local
    for (size_t v = a.rs_v0 + tid0; v < a.rs_v1; v += stride) {
      float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int p = 0; p < a.nranks; ++p)
        acc_vec<DT>(acc, reinterpret_cast<const uint4 *>(a.base[p] + in_off)[v]);
      *out_vec(a, v) = pack_vec<DT>(acc);
    }
  } else {
    // 3b. two-shot: reduce my chunk, publish, gather the others
    const size_t c0 = a.nvec * a.rank / a.nranks, c1 = a.nvec * (a.rank + 1) / a.nranks;
    uint4 *pub = reinterpret_cast<uint4 *>(own + out_off);
    for (size_t v = c0 + tid0; v < c1; v += stride) {
      float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int p = 0; p < a.nranks; ++p)
        acc_vec<DT>(acc, reinterpret_cast<const uint4 *>(a.base[p] + in_off)[v]);
      const uint4 r = pack_vec<DT>(acc);
      pub[v] = r;
      *out_vec(a, v) = r;
    }
    if (arrive_last(&hdr[kCnt1], G) && threadIdx.x == 0) push_flags(a, kInbox1, e);
    if (!wait_flags(a, kInbox1, e, 2)) return;
    for (int q = 1; q < a.nranks; ++q) {
      const int p = (a.rank + q) % a.nranks;  // spread the first reads over the links
      const size_t p0 = a.nvec * p / a.nranks, p1 = a.nvec * (p + 1) / a.nranks;
      const uint4 *src = reinterpret_cast<const uint4 *>(a.base[p] + out_off);
      for (size_t v = p0 + tid0; v < p1; v += stride) *out_vec(a, v) = src[v];
    }
  }
  // 4. the epoch of the next launch
  if (arrive_last(&hdr[kCnt2], G) && threadIdx.x == 0)
    __hip_atomic_store(&hdr[kEpochWord], e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ float h2f_c(uint16_t v) { return __half2float(__ushort_as_half(v)); }
__device__ __forceinline__ uint16_t f2h_c(float v) { return __half_as_ushort(__float2half_rn(v)); }

// All-reduce + residual RMSNorm (collective.h, PeerNormArgs).  NT threads per
// row and MAXC 8-element chunks per thread as rmsnorm_kernel at this width
// (launch_rmsnorm), the same expressions in the same order: the per-thread
// fp64 sum of squares over its chunks, the wave xor tree, the waves in order.
template <int NT, int MAXC, bool TWO_SHOT, int MAXS>
__global__ __launch_bounds__(NT) void peer_allreduce_norm_kernel(PeerArgs a, PeerNormArgs n) {
  __shared__ double scratch[NT / 64];
  char *own = a.base[a.rank];
  unsigned *hdr = reinterpret_cast<unsigned *>(own + kHdrCounters);
  const unsigned e = hdr[kEpochWord] + 1u;
  const size_t par = e & 1u;
  const size_t in_off = kDataOff + par * a.cap;
  const size_t out_off = kDataOff + (2 + par) * a.cap;
  const unsigned G = gridDim.x;
  const size_t stride = (size_t)G * NT;
  const size_t tid0 = (size_t)blockIdx.x * NT + threadIdx.x;

  // 1. copy-in of this rank's partial (columns [col0, H) of every row)
  {
    uint4 *dst = reinterpret_cast<uint4 *>(own + in_off);
    if constexpr (MAXS > 0) {
      for (size_t v = tid0; v < a.nvec; v += stride) dst[v] = slab_vec<MAXS>(a, v);
    } else {
      const uint4 *src = reinterpret_cast<const uint4 *>(a.in);
      for (size_t v = tid0; v < a.nvec; v += stride) dst[v] = src[v];
    }
  }
  // 2. signal
  if (arrive_last(&hdr[kCnt0], G) && threadIdx.x == 0) push_flags(a, kInbox0, e);
  if (!wait_flags(a, kInbox0, e, 1)) return;

  // 3. the rows: sum in rank order (as the all-reduce), residual add, norm
  const int H = n.H, nchunk = H >> 3;
  const int c0 = (int)(a.col0 >> 3);  // first chunk of the all-reduced columns
  const size_t vpr = a.cols >> 3;     // 16-B vectors per row of the partial
  uint4 *pub = reinterpret_cast<uint4 *>(own + out_off);
  for (int row = n.row0 + (int)blockIdx.x; row < n.row1; row += (int)G) {
    uint4 v[MAXC], wv[MAXC], xb[MAXC];
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int ch = min((int)threadIdx.x + c * NT, nchunk - 1);
      if (ch >= c0) {
        float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        const size_t vi = (size_t)row * vpr + (ch - c0);
        for (int p = 0; p < a.nranks; ++p)
          acc_vec<0>(acc, reinterpret_cast<const uint4 *>(a.base[p] + in_off)[vi]);
        xb[c] = pack_vec<0>(acc);
      } else {
        xb[c] = *reinterpret_cast<const uint4 *>(n.prev + (size_t)row * H + ch * 8);
      }
      v[c] = *reinterpret_cast<const uint4 *>(n.res + (size_t)row * H + ch * 8);
      wv[c] = *reinterpret_cast<const uint4 *>(n.w + ch * 8);
    }
    double ss = 0.0;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int ch = threadIdx.x + c * NT;
      if (ch < nchunk) {
        uint4 xa = v[c];
        const uint4 xbb = xb[c];
        const __half2 *pa = reinterpret_cast<const __half2 *>(&xa);
        const __half2 *pb = reinterpret_cast<const __half2 *>(&xbb);
        __half2 r[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) r[q] = __hadd2(pa[q], pb[q]);
        xa = *reinterpret_cast<uint4 *>(r);
        *reinterpret_cast<uint4 *>(n.res + (size_t)row * H + ch * 8) = xa;
        v[c] = xa;
        const uint16_t *el = reinterpret_cast<const uint16_t *>(&xa);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const float f = h2f_c(el[q]);
          ss += (double)f * (double)f;
        }
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o);
    if ((threadIdx.x & 63) == 0) scratch[threadIdx.x >> 6] = ss;
    __syncthreads();
    double tot = scratch[0];
#pragma unroll
    for (int q = 1; q < NT / 64; ++q) tot += scratch[q];
    __syncthreads();  // scratch is rewritten by the next row
    const float sum = (float)tot;
    const float rms_f = __fdiv_rn(1.0f, sqrtf(__fadd_rn(__fdiv_rn(sum, (float)H), n.eps)));
    const float rms = h2f_c(f2h_c(rms_f));
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int ch = threadIdx.x + c * NT;
      if (ch < nchunk) {
        const uint16_t *el = reinterpret_cast<const uint16_t *>(&v[c]);
        const uint16_t *we = reinterpret_cast<const uint16_t *>(&wv[c]);
        uint16_t o8[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          float y = h2f_c(f2h_c(__fmul_rn(h2f_c(el[q]), rms)));
          o8[q] = f2h_c(__fmul_rn(y, h2f_c(we[q])));
        }
        const uint4 ov = *reinterpret_cast<uint4 *>(o8);
        uint16_t *dst = n.packed ? n.h + act_packed_off(row, ch * 8, H) : n.h + (size_t)row * H + ch * 8;
        *reinterpret_cast<uint4 *>(dst) = ov;
        if (TWO_SHOT) pub[(size_t)row * nchunk + ch] = ov;  // row-major [T][H]
      }
    }
  }
  if constexpr (TWO_SHOT) {
    // 4. signal the published rows; gather every other rank's
    if (arrive_last(&hdr[kCnt1], G) && threadIdx.x == 0) push_flags(a, kInbox1, e);
    if (!wait_flags(a, kInbox1, e, 2)) return;
    for (int q = 1; q < a.nranks; ++q) {
      const int p = (a.rank + q) % a.nranks;
      const size_t r0 = (size_t)n.T * p / a.nranks, r1 = (size_t)n.T * (p + 1) / a.nranks;
      const uint4 *src = reinterpret_cast<const uint4 *>(a.base[p] + out_off);
      for (size_t v = r0 * nchunk + tid0; v < r1 * nchunk; v += stride) {
        const int row = (int)(v / nchunk), ch = (int)(v % nchunk);
        uint16_t *dst = n.packed ? n.h + act_packed_off(row, ch * 8, H) : n.h + (size_t)row * H + ch * 8;
        *reinterpret_cast<uint4 *>(dst) = src[v];
      }
    }
  }
  // 5. the epoch of the next launch
  if (arrive_last(&hdr[kCnt2], G) && threadIdx.x == 0)
    __hip_atomic_store(&hdr[kEpochWord], e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace

hipError_t launch_peer_allreduce_norm(const PeerArgs &a, const PeerNormArgs &n, bool two_shot,
                                      hipStream_t s) {
  const int nchunk = n.H / 8;
  if (n.T <= 0) return hipSuccess;
  if (a.esz != 2 || n.H % 8 || nchunk > 4096 || a.col0 % 8 || a.col0 + a.cols != (size_t)n.H ||
      (a.col0 > 0 && !n.prev) || (n.packed && n.H % 32) || n.row0 < 0 || n.row1 > n.T ||
      n.row0 > n.row1 || a.nvec != (size_t)n.T * a.cols / 8 || (a.slabs && (a.S < 1 || a.S > 8)))
    return hipErrorInvalidValue;
  // the published rows ([T][H] f16) share the `out` area's capacity
  if ((size_t)n.T * n.H * 2 > a.cap) return hipErrorInvalidValue;
  if (two_shot) {
    const int r0 = (int)((long)n.T * a.rank / a.nranks), r1 = (int)((long)n.T * (a.rank + 1) / a.nranks);
    if (n.row0 != r0 || n.row1 != r1) return hipErrorInvalidValue;
  } else if (n.row0 != 0 || n.row1 != n.T) {
    return hipErrorInvalidValue;
  }
  // (rows, threads): the workgroups of one launch hold at most as many
  // threads as the plain all-reduce's grid, so that every rank's grid stays
  // co-resident beside the others' (the transport's waits need it)
  const int NT = nchunk <= 128 ? 128 : nchunk <= 256 ? 256 : nchunk <= 512 ? 512 : 1024;
  const int rows = std::max(1, n.row1 - n.row0);
  const unsigned G = (unsigned)std::max(1, std::min(rows, kMaxPeerBlocks * kThreads / NT));
  const int ms = !a.slabs ? 0 : a.S <= 2 ? 2 : a.S <= 4 ? 4 : 8;
#define FFMI_ARN3(NTV, MC, TS, MS) \
  hipLaunchKernelGGL((peer_allreduce_norm_kernel<NTV, MC, TS, MS>), dim3(G), dim3(NTV), 0, s, a, n)
#define FFMI_ARN2(NTV, MC, TS)              \
  do {                                      \
    if (ms == 0) FFMI_ARN3(NTV, MC, TS, 0); \
    else if (ms == 2) FFMI_ARN3(NTV, MC, TS, 2); \
    else if (ms == 4) FFMI_ARN3(NTV, MC, TS, 4); \
    else FFMI_ARN3(NTV, MC, TS, 8);         \
  } while (0)
#define FFMI_ARN(NTV, MC)                      \
  do {                                         \
    if (two_shot) FFMI_ARN2(NTV, MC, true);    \
    else FFMI_ARN2(NTV, MC, false);            \
  } while (0)
  if (nchunk <= 128) FFMI_ARN(128, 1);
  else if (nchunk <= 256) FFMI_ARN(256, 1);
  else if (nchunk <= 512) FFMI_ARN(512, 1);
  else if (nchunk <= 1024) FFMI_ARN(1024, 1);
  else if (nchunk <= 2048) FFMI_ARN(1024, 2);
  else FFMI_ARN(1024, 4);
#undef FFMI_ARN
#undef FFMI_ARN2
#undef FFMI_ARN3
  return hipGetLastError();
}

hipError_t launch_peer_allreduce(const PeerArgs &a0, bool two_shot, hipStream_t s, int rs_row0,
                                 int rs_row1) {
  if (a0.nvec == 0) return hipSuccess;
  PeerArgs a = a0;
  const bool rs = rs_row0 >= 0;
  if (rs) {  // whole rows of 16-B vectors
    const size_t vpr = a.cols * a.esz / 16;
    if (!two_shot || a.esz != 2 || rs_row1 < rs_row0 || (a.cols * a.esz) % 16 ||
        (size_t)rs_row1 * vpr > a.nvec || (a.slabs && (a.S < 1 || a.S > 8)))
      return hipErrorInvalidValue;
    a.rs_v0 = (size_t)rs_row0 * vpr, a.rs_v1 = (size_t)rs_row1 * vpr;
  }
  // enough workgroups to keep xGMI reads in flight, few enough to be
  // co-resident with the GEMMs of a concurrent stream (every workgroup may
  // wait on a peer, so the whole grid must be resident)
  size_t per = two_shot ? (a.nvec + a.nranks - 1) / a.nranks : a.nvec;
  unsigned G = (unsigned)std::min<size_t>(kMaxPeerBlocks, (per + kThreads - 1) / kThreads);
  if (G == 0) G = 1;
  if (rs) {
#define FFMI_PEER_RS(MS) \
  hipLaunchKernelGGL((peer_allreduce_kernel<0, true, MS, true>), dim3(G), dim3(kThreads), 0, s, a)
    if (!a.slabs) FFMI_PEER_RS(0);
    else if (a.S <= 2) FFMI_PEER_RS(2);
    else if (a.S <= 4) FFMI_PEER_RS(4);
    else FFMI_PEER_RS(8);
#undef FFMI_PEER_RS
    return hipGetLastError();
  }
  if (a.slabs) {
    if (a.esz != 2 || a.S < 1 || a.S > 8) return hipErrorInvalidValue;
    const int ms = a.S <= 2 ? 2 : a.S <= 4 ? 4 : 8;
#define FFMI_PEER_SL(TS, MS) \
  hipLaunchKernelGGL((peer_allreduce_kernel<0, TS, MS>), dim3(G), dim3(kThreads), 0, s, a)
    if (two_shot) {
      if (ms == 2) FFMI_PEER_SL(true, 2);
      else if (ms == 4) FFMI_PEER_SL(true, 4);
      else FFMI_PEER_SL(true, 8);
    } else {
      if (ms == 2) FFMI_PEER_SL(false, 2);
      else if (ms == 4) FFMI_PEER_SL(false, 4);
      else FFMI_PEER_SL(false, 8);
    }
#undef FFMI_PEER_SL
  } else if (a.esz == 2) {
    if (two_shot) hipLaunchKernelGGL((peer_allreduce_kernel<0, true>), dim3(G), dim3(kThreads), 0, s, a);
    else hipLaunchKernelGGL((peer_allreduce_kernel<0, false>), dim3(G), dim3(kThreads), 0, s, a);
  } else {
    if (two_shot) hipLaunchKernelGGL((peer_allreduce_kernel<1, true>), dim3(G), dim3(kThreads), 0, s, a);
    else hipLaunchKernelGGL((peer_allreduce_kernel<1, false>), dim3(G), dim3(kThreads), 0, s, a);
  }
  return hipGetLastError();
}

}  // namespace ffmi
