// MPIAsyncPool state (src/MPIAsyncPools.jl:24-34) and the asyncmap!/waitall! state
// machine (src/MPIAsyncPools.jl:68-224), transport-agnostic.
#pragma once
#include <cstdint>
#include <vector>

#include "comm.hpp"

namespace mpa {

struct Pool {
  int64_t n = 0;
  // Field vectors: the C ABI hands out pointers into these, so they are sized once and
  // never reallocated (the reference's `pool.repochs` is returned by alias, :187).
  std::vector<int64_t> ranks, sepochs, repochs, stimestamps;
  std::vector<uint8_t> active, rreq_live;
  // received[i]: a reply of worker i has been harvested at least once (not reference state:
  // the descent loops weight stale chunks by it; repochs[i] == epoch0 cannot tell, since an
  // explicit epoch may equal epoch0)
  std::vector<uint8_t> received;
  std::vector<double> latency;
  int64_t nwait = 0;
  int64_t epoch = 0;
  Comm* comm = nullptr;  // the comm the outstanding requests were posted on

  Pool(int64_t n_, const int64_t* ranks_, int64_t epoch0, int64_t nwait_);
};

struct AsyncmapArgs {
  const void* sendbuf; size_t send_bytes;
  void* recvbuf; size_t recv_bytes; size_t recv_length;
  void* isendbuf; size_t isend_bytes;
  void* irecvbuf; size_t irecv_bytes;
  Comm* comm;
  int nwait_kind; int64_t nwait; mpa_nwait_fn fn; void* fn_ctx; const char* nwait_typename;
  int64_t epoch; int64_t tag;
};

void asyncmap(Pool& p, const AsyncmapArgs& a);
void waitall(Pool& p, void* recvbuf, size_t recv_bytes, size_t recv_length, void* irecvbuf, size_t irecv_bytes);

}  // namespace mpa
