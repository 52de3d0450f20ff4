// Host shared-memory mailboxes between the coordinator process and worker processes
// (one process per GPU).
//
// One POSIX shared-memory segment per communicator, registered with the HIP runtime
// (hipHostRegister, mapped) in every process, so that device kernels on any GPU can store
// into it and every host thread can poll it.  It carries, per logical worker, what the
// reference's MPI messages carry (src/MPIAsyncPools.jl:137-138): the message from the
// coordinator (Isend of isendbufs[i]) and the reply (the worker's Isend, received by
// Irecv! into irecvbufs[i]), plus the words that replace MPI request completion:
//
//   doorbell  seq of the last message posted to the worker; stored by the coordinator's
//             exchange kernel (system-scope release) after the message bytes
//   done      seq of the last reply; stored by the worker's task kernel (system-scope
//             release) after the reply bytes           -> MPI.Test! / Waitany! / Waitall!
//   gen       pause generation / shutdown word (the reference's control tag,
//             examples/iterative_example.jl:49-52), stored by the coordinator host
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>

namespace mpa {

// Message / reply payload path of a worker (BoxHeader::mode), decided by the coordinator
// at its first post to the worker once both processes have reported their side:
//   kPathHost    payloads in this segment (host memory; the worker stages the message)
//   kPathDevice  payloads in device memory over xGMI: the coordinator's kernels store the
//                message straight into the worker's device message slot, the worker's
//                task stores its reply into the coordinator's device reply inbox (both
//                fine-grained allocations shared by HIP IPC handles); doorbell and done
//                stay here
enum : uint32_t { kPathPending = 0, kPathHost = 1, kPathDevice = 2 };
enum : uint32_t { kIpcPending = 0, kIpcOk = 1, kIpcFailed = 2 };

struct alignas(256) BoxHeader {
  unsigned long long doorbell;
  unsigned long long done;
  unsigned long long msg_bytes;    // sizeof(sendbuf) of the posted message (:80)
  unsigned long long reply_bytes;  // bytes of the recv chunk (:81)
  unsigned long long pad[28];
  // device-memory path set-up
  int32_t server_dev, coord_dev;  // HIP device of the serving process / of rank 0
  volatile uint32_t msg_ipc;      // server: kIpc* of exporting its device message slot
  volatile uint32_t reply_ipc;    // rank 0: kIpc* of exporting the device reply inbox
  volatile uint32_t reply_open;   // server: kIpc* of opening that inbox
  volatile uint32_t mode;         // rank 0: kPath*
  uint32_t pad32[2];
  char msg_handle[64];    // hipIpcMemHandle_t of the server's message slot
  char reply_handle[64];  // hipIpcMemHandle_t of rank 0's reply inbox for this worker
  uint8_t pad2[96];
};
static_assert(sizeof(BoxHeader) == 512, "box header is two 256-byte line groups");

struct alignas(256) ShmHeader {
  uint64_t magic;
  uint64_t version;
  int64_t nworkers;
  uint64_t max_msg;
  uint64_t box_bytes;
  volatile uint64_t gen;       // bumped by the coordinator: servers return from serve()
  volatile uint64_t shutdown;  // set by the coordinator: servers stop serving
  unsigned int err;            // first device-side error code of any worker process
  unsigned int pad32;
  uint64_t pad[24];
};
static_assert(sizeof(ShmHeader) == 256, "shm header is one 256-byte line group");

class ShmRegion {
 public:
  // create (coordinator) or attach (worker processes); registers the mapping with HIP
  // with_hip = false maps the segment without registering it (host-only tests)
  static ShmRegion* create(const std::string& name, int64_t nworkers, size_t max_msg, bool with_hip = true);
  static ShmRegion* attach(const std::string& name, bool with_hip = true);
  ~ShmRegion();

  ShmHeader* header() const { return reinterpret_cast<ShmHeader*>(base_); }
  int64_t nworkers() const { return header()->nworkers; }
  size_t max_msg() const { return size_t(header()->max_msg); }
  // worker rank 1..n
  BoxHeader* box(int64_t rank) const {
    return reinterpret_cast<BoxHeader*>(base_ + sizeof(ShmHeader) + size_t(rank - 1) * header()->box_bytes);
  }
  uint8_t* msg(int64_t rank) const { return reinterpret_cast<uint8_t*>(box(rank)) + sizeof(BoxHeader); }
  uint8_t* reply(int64_t rank) const { return msg(rank) + header()->max_msg; }
  // the same addresses as device pointers (hipHostGetDevicePointer of the registration)
  template <typename P>
  P* dev(P* host) const {
    return reinterpret_cast<P*>(reinterpret_cast<uint8_t*>(host) - base_ + dbase_);
  }
  void unlink_name();

 private:
  ShmRegion() = default;
  void map_and_register(int fd, size_t bytes, bool with_hip);
  std::string name_;
  bool registered_ = false;
  uint8_t* base_ = nullptr;
  uint8_t* dbase_ = nullptr;
  size_t bytes_ = 0;
  bool owner_ = false;
  bool linked_ = false;
};

}  // namespace mpa
