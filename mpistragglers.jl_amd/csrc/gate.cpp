// Gated replay: the completion order of a transport fixed to a schedule (comm.hpp).
//
// The reference's order of completions is a race between worker processes.  A schedule
// taken from the oracle's virtual clock (oracle/oracle.py gate_schedule) says, for every
// observation point of the state machine (pool.cpp), which tasks have completed by then;
// the transport shows exactly those to MPI.Test! / Waitany! / Waitall!
// (src/MPIAsyncPools.jl:99,161,212) and nothing else, so the product replays the oracle's
// trace whatever order the device finishes its tasks in.  Only the visibility is gated:
// the tasks themselves run, and their replies land, as they would without it.
#include <chrono>
#include <thread>

#include "comm.hpp"

namespace mpa {

static const char* gate_kind_name(int k) {
  return k == MPA_GATE_CALL ? "call (phase 1)" : k == MPA_GATE_WAIT ? "Waitany!" : k == MPA_GATE_WAITALL ? "Waitall!" : "?";
}

void Comm::set_gate(const int* kinds, const int64_t* offsets, const int64_t* ranks, int64_t nsteps) {
  if (!gate_supported()) fail(MPA_ARGUMENT_ERROR, "this transport has no gated replay (HIP and HOST rank 0 do)");
  if (nsteps < 0 || (nsteps > 0 && (!kinds || !offsets))) fail(MPA_ARGUMENT_ERROR, "bad gate schedule");
  if (nsteps == 0) {
    gate_on_ = false;
    return;
  }
  if (offsets[0] != 0) fail(MPA_ARGUMENT_ERROR, "gate schedule: offsets[0] must be 0");
  for (int64_t k = 0; k < nsteps; ++k) {
    if (kinds[k] != MPA_GATE_CALL && kinds[k] != MPA_GATE_WAIT && kinds[k] != MPA_GATE_WAITALL)
      fail(MPA_ARGUMENT_ERROR, "gate schedule: step %lld has kind %d", (long long)k, kinds[k]);
    if (offsets[k + 1] < offsets[k]) fail(MPA_ARGUMENT_ERROR, "gate schedule: offsets must not decrease");
  }
  const int64_t nr = offsets[nsteps];
  if (nr > 0 && !ranks) fail(MPA_ARGUMENT_ERROR, "gate schedule: ranks is NULL");
  for (int64_t j = 0; j < nr; ++j)
    if (ranks[j] < 1 || ranks[j] > nworkers_)
      fail(MPA_ARGUMENT_ERROR, "gate schedule: rank %lld is not a worker rank (1:%lld)", (long long)ranks[j],
           (long long)nworkers_);
  gate_kinds_.assign(kinds, kinds + nsteps);
  gate_off_.assign(offsets, offsets + nsteps + 1);
  gate_ranks_.assign(ranks, ranks + nr);
  // whatever was posted before the schedule starts is released
  gate_rel_.assign(size_t(nworkers_), 0);
  for (int64_t r = 1; r <= nworkers_; ++r) gate_rel_[size_t(r - 1)] = gate_posted(r);
  gate_step_ = 0;
  gate_on_ = true;
}

void Comm::gate(int kind) {
  if (!gate_on_) return;
  if (gate_step_ == gate_kinds_.size()) {  // past the schedule: ungated from here on
    gate_on_ = false;
    return;
  }
  if (gate_kinds_[gate_step_] != kind)
    fail(MPA_ERROR, "gated replay: step %zu of the schedule is a %s observation, the state machine is at a %s",
         gate_step_, gate_kind_name(gate_kinds_[gate_step_]), gate_kind_name(kind));
  const int64_t a = gate_off_[gate_step_], e = gate_off_[gate_step_ + 1];
  for (int64_t j = a; j < e; ++j) {
    const int64_t r = gate_ranks_[size_t(j)];
    uint64_t& rel = gate_rel_[size_t(r - 1)];
    rel += 1;
    if (rel > gate_posted(r))
      fail(MPA_ERROR, "gated replay: step %zu releases task %llu of worker %lld, which has been posted %llu tasks",
           gate_step_, (unsigned long long)rel, (long long)r, (unsigned long long)gate_posted(r));
    gate_launch(r);
  }
  const auto t0 = std::chrono::steady_clock::now();
  const uint64_t t0_ns = uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(t0.time_since_epoch()).count());
  for (int64_t j = a; j < e; ++j) {
    const int64_t r = gate_ranks_[size_t(j)];
    PoliteSpin poll;  // hot, then sleeping between polls (comm.hpp)
    for (uint64_t spins = 0; gate_finished(r) < gate_rel_[size_t(r - 1)]; ++spins) {
      if ((spins & 0xFFF) == 0xFFF)
        gate_poll(std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
      poll();
    }
    gate_seen(r, gate_rel_[size_t(r - 1)], t0_ns);
  }
  ++gate_step_;
}

}  // namespace mpa
