// client.hip — the client-side response aggregation of MochiDBClient on the
// device, batched across many in-flight transactions:
//
//   k_tally_responses   Read / Write2 aggregation (MochiDBClient.java:148-175,
//                       355-382): per request, every response must return as
//                       many op results as the transaction has ops, and per op
//                       the number of non-WRONG_SHARD results must reach
//                       M = 2*(R/3)+1; the chosen result is the last such one.
//   k_write1_classify   the Write1 round (MochiDBClient.java:236-332 with
//                       isUniformTimeStampInMultiGrants :195-219 and
//                       removeWrongShardGrantFromMultiGrant :221-235).
//
// Lane = request: each request holds a handful of responses (R) and ops (k),
// so the loops are short and per-op state is recomputed by re-scanning rather
// than kept in per-lane arrays.  Same contracts as the host functions
// mochi_tally_responses / mochi_write1_classify (capi.cpp), restated by
// oracle_tally_responses / oracle_write1_classify.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mochi_hip.h"

namespace mochi {
namespace {

__global__ __launch_bounds__(256) void k_tally_responses(uint32_t n_requests, const uint32_t* __restrict__ resp_off,
                                                         const uint32_t* __restrict__ n_ops,
                                                         const uint32_t* __restrict__ resp_n_ops,
                                                         const uint64_t* __restrict__ status_off,
                                                         const uint8_t* __restrict__ status,
                                                         const uint64_t* __restrict__ chosen_off, uint32_t majority,
                                                         int32_t* __restrict__ chosen, uint8_t* __restrict__ reason,
                                                         uint32_t* __restrict__ accept_bits) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t why = 1;  // out-of-range lanes vote "reject" in the ballot
  if (r < n_requests) {
    const uint32_t k = n_ops[r], q0 = resp_off[r], q1 = resp_off[r + 1];
    // :159-161 / :366-368: a response with another op count throws; responses
    // before it have already been counted (their chosen results stand)
    uint32_t q_end = q1;
    why = 0;
    for (uint32_t q = q0; q < q1; q++)
      if (resp_n_ops[q] != k) {
        q_end = q;
        why = 1;
        break;
      }
    for (uint32_t j = 0; j < k; j++) {
      uint32_t cnt = 0;
      int32_t last = -1;
      for (uint32_t q = q0; q < q_end; q++)
        if (status[status_off[q] + j] != 1) {  // != WRONG_SHARD  :164-167 / :371-374
          cnt++;
          last = (int32_t)(q - q0);
        }
      if (chosen) chosen[chosen_off[r] + j] = last;
      if (!why && cnt < majority) why = 2;  // consistentTRCount[index] < getServerMajority()  :171-175 / :378-381
    }
    if (reason) reason[r] = (uint8_t)why;
  }
  const uint64_t acc = __ballot(r < n_requests && why == 0);
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wbase = (r - lane) >> 5, nwords = (n_requests + 31) >> 5;
  if (lane == 0 && wbase < nwords) accept_bits[wbase] = (uint32_t)acc;
  if (lane == 0 && wbase + 1 < nwords) accept_bits[wbase + 1] = (uint32_t)(acc >> 32);
}

__global__ __launch_bounds__(256) void k_write1_classify(uint32_t n_requests, const uint32_t* __restrict__ resp_off,
                                                         const uint8_t* __restrict__ resp_kind,
                                                         const uint32_t* __restrict__ resp_server,
                                                         const uint32_t* __restrict__ resp_grant_off,
                                                         const uint8_t* __restrict__ grant_key,
                                                         const int64_t* __restrict__ grant_ts,
                                                         const uint8_t* __restrict__ grant_status,
                                                         uint8_t* __restrict__ decision) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_requests) return;
  const uint32_t q0 = resp_off[r], q1 = resp_off[r + 1];
  bool failed = false, wrong_shard = false, all_ok = true;
  for (uint32_t q = q0; q < q1; q++) {
    const uint8_t kind = resp_kind[q];
    all_ok &= kind == MOCHI_W1_OK;                          // :284-287
    failed |= kind == MOCHI_W1_REQUEST_FAILED;              // :281-283
    if (kind == MOCHI_W1_OK || kind == MOCHI_W1_REFUSED)    // :295-307 -> :221-228
      for (uint32_t g = resp_grant_off[q]; g < resp_grant_off[q + 1]; g++) wrong_shard |= grant_status[g] == 1;
  }
  uint8_t d;
  if (failed) d = MOCHI_W1_THROW_FAILED;
  else if (wrong_shard) d = MOCHI_W1_THROW_UNSUPPORTED;
  else {
    // isUniformTimeStampInMultiGrants over write1mutiGrants: one MultiGrant per
    // serverId, the LAST OK response with that id (HashMap.put, :299); per key,
    // every grant's ts equals every other's (the first-seen comparison of
    // :206-214 is order-free).  Each kept grant is compared with the first kept
    // grant of its key.
    bool uniform = true;
    for (uint32_t q = q0; q < q1 && uniform; q++) {
      if (resp_kind[q] != MOCHI_W1_OK) continue;
      bool superseded = false;
      for (uint32_t p = q + 1; p < q1; p++) superseded |= resp_kind[p] == MOCHI_W1_OK && resp_server[p] == resp_server[q];
      if (superseded) continue;
      for (uint32_t g = resp_grant_off[q]; g < resp_grant_off[q + 1] && uniform; g++) {
        const uint8_t key = grant_key[g];
        if (key == 0xFF) continue;  // no op names it: never looked up (:202-205)
        // the first kept grant with this key (responses in order)
        bool found = false;
        int64_t ts0 = 0;
        for (uint32_t a = q0; a <= q && !found; a++) {
          if (resp_kind[a] != MOCHI_W1_OK) continue;
          bool sup = false;
          for (uint32_t p = a + 1; p < q1; p++) sup |= resp_kind[p] == MOCHI_W1_OK && resp_server[p] == resp_server[a];
          if (sup) continue;
          const uint32_t g_hi = a == q ? g : resp_grant_off[a + 1];
          for (uint32_t h = resp_grant_off[a]; h < g_hi; h++)
            if (grant_key[h] == key) {
              found = true;
              ts0 = grant_ts[h];
              break;
            }
        }
        if (found && ts0 != grant_ts[g]) uniform = false;
      }
    }
    d = !uniform ? MOCHI_W1_RETRY : all_ok ? MOCHI_W1_PROCEED : MOCHI_W1_THROW_REFUSED;  // :310-328
  }
  decision[r] = d;
}

}  // namespace
}  // namespace mochi

extern "C" {

int mochi_tally_responses_device(uint32_t n_requests, const uint32_t* resp_off, const uint32_t* n_ops,
                                 const uint32_t* resp_n_ops, const uint64_t* status_off, const uint8_t* status,
                                 const uint64_t* chosen_off, uint32_t replication_factor, int32_t* chosen,
                                 uint8_t* reason, uint32_t* accept_bits, void* stream) {
  if (n_requests && (!resp_off || !n_ops || !resp_n_ops || !status_off || !status || !accept_bits ||
                     (chosen && !chosen_off)))
    return MOCHI_EINVAL;
  if (!n_requests) return MOCHI_OK;
  const uint32_t M = 2 * (replication_factor / 3) + 1;  // getServerMajority  ClusterConfiguration.java:264-267
  hipLaunchKernelGGL(mochi::k_tally_responses, dim3((n_requests + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     n_requests, resp_off, n_ops, resp_n_ops, status_off, status, chosen_off, M, chosen, reason,
                     accept_bits);
  return hipGetLastError() == hipSuccess ? MOCHI_OK : MOCHI_EHIP;
}

int mochi_write1_classify_device(uint32_t n_requests, const uint32_t* resp_off, const uint8_t* resp_kind,
                                 const uint32_t* resp_server, const uint32_t* resp_grant_off, const uint8_t* grant_key,
                                 const int64_t* grant_ts, const uint8_t* grant_status, uint8_t* decision,
                                 void* stream) {
  if (n_requests && (!resp_off || !resp_kind || !resp_server || !resp_grant_off || !decision)) return MOCHI_EINVAL;
  if (!n_requests) return MOCHI_OK;
  hipLaunchKernelGGL(mochi::k_write1_classify, dim3((n_requests + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     n_requests, resp_off, resp_kind, resp_server, resp_grant_off, grant_key, grant_ts, grant_status,
                     decision);
  return hipGetLastError() == hipSuccess ? MOCHI_OK : MOCHI_EHIP;
}

}  // extern "C"
