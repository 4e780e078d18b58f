// collective.h -- the direct xGMI all-reduce's exchange-buffer layout and
// kernel arguments (kernels/collective.hip, api.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace ffmi {

constexpr int kMaxPeers = 8;        // one node: the 8 GPUs of an MI355X platform
// All-reduce grid cap.  Every workgroup may wait on a peer, so the whole
// grid must be resident -- and it runs beside the GEMM of the other stream:
// 32 workgroups (one per 8 CUs) keep ~1 MB of xGMI reads in flight and leave
// the other CUs whole for the GEMM (a grid spread over every CU starves a
// GEMM whose workgroups need a full CU's registers until the all-reduce ends)
constexpr int kMaxPeerBlocks = 32;
constexpr size_t kFlagStride = 256;  // one inbox slot per peer, own 256-B line
// exchange buffer: [inbox0 8 slots][inbox1 8 slots][counters][data areas]
constexpr size_t kInbox0 = 0;
constexpr size_t kInbox1 = kMaxPeers * kFlagStride;
constexpr size_t kHdrCounters = 2 * kMaxPeers * kFlagStride;
constexpr int kCnt0 = 0, kCnt1 = 64, kCnt2 = 128, kEpochWord = 192;  // u32 words, 256-B apart
constexpr size_t kDataOff = kHdrCounters + 4096;
// data areas of `cap` bytes each: in[parity 0], in[parity 1], out[0], out[1]
inline size_t peer_buffer_bytes(size_t cap) { return kDataOff + 4 * cap; }

struct PeerArgs {
  char *base[kMaxPeers];  // every rank's exchange buffer as mapped in this process
  int nranks, rank;
  size_t cap;             // bytes per data area
  const void *in;         // [rows][cols] contiguous
  void *out;              // row stride ld elements, starting at column col0
  size_t nvec;            // 16-B vectors of the input
  size_t vec_elems;       // elements per vector (8 f16 / 4 f32)
  size_t cols, ld, col0;
  size_t esz;
  int *err;               // host-mapped error word (0 = ok)
  uint64_t timeout_ticks;  // s_memrealtime ticks (100 MHz)
  // split-K input (f16 only): `in` unused, this rank's partial is the sum of
  // S fp32 slabs [S][rows][NP] in slab order, rounded once to fp16 -- the
  // value the GEMM's reduce pass would have written, folded into the copy-in
  const float *slabs = nullptr;
  int S = 0;
  size_t NP = 0, rows = 0;
  // reduce-scatter by rows (launch_peer_allreduce rs_rows): vectors [v0, v1)
  size_t rs_v0 = 0, rs_v1 = 0;
};

// rs_rows: reduce-scatter by rows only -- rows [row0, row1) of the sum into
// `out`, nothing published or gathered (the first column chunk of a fused
// all-reduce + residual norm, launch_peer_allreduce_norm)
hipError_t launch_peer_allreduce(const PeerArgs &a, bool two_shot, hipStream_t s,
                                 int rs_row0 = -1, int rs_row1 = -1);

// All-reduce fused with the residual RMSNorm that follows it
// (residual_rms_norm_kernels.cu:98-131 after allreduce_kernels.cu:53-75;
// model.cc:3421-3445).  The all-reduced partial covers columns [col0, H) of
// the [T][H] sum (PeerArgs cols = H - col0, f16); columns [0, col0) come from
// `prev`, the sum of an earlier column chunk (launch_peer_allreduce with
// rs_rows, or a whole one-shot all-reduce).  For rows [row0, row1):
//   res = half(res + sum)   (in place)
//   h   = RMSNorm(res) * w  (packed MFMA activation layout when `packed`)
// with rmsnorm_kernel's arithmetic and reduction order, so h and res are
// bit-identical to the all-reduce followed by the norm.  Two-shot: the rows
// are this rank's share (T * r / N ..), h rows are published in the exchange
// buffer and every rank gathers the others' -- h complete on every rank, res
// valid on this rank's rows only.  One-shot: every rank computes every row.
struct PeerNormArgs {
  uint16_t *res = nullptr;        // [T][H]
  const uint16_t *w = nullptr;    // [H]
  uint16_t *h = nullptr;          // [T][H]
  const uint16_t *prev = nullptr;  // [T][H] (columns < col0)
  int T = 0, H = 0, packed = 0, row0 = 0, row1 = 0;
  float eps = 0.f;
};
hipError_t launch_peer_allreduce_norm(const PeerArgs &a, const PeerNormArgs &n, bool two_shot,
                                      hipStream_t s);

}  // namespace ffmi
