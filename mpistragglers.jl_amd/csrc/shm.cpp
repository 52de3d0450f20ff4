#include "shm.hpp"

#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cstring>

#include "common.hpp"

namespace mpa {

namespace {
constexpr uint64_t kMagic = 0x4D50415348424F58ull;  // "MPASHBOX"
constexpr uint64_t kVersion = 2;

size_t round_up(size_t v, size_t a) { return (v + a - 1) / a * a; }
}  // namespace

void ShmRegion::map_and_register(int fd, size_t bytes, bool with_hip) {
  void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) fail(MPA_ERROR, "mmap of shared memory '%s' failed: %s", name_.c_str(), strerror(errno));
  base_ = static_cast<uint8_t*>(p);
  dbase_ = base_;
  bytes_ = bytes;
  if (!with_hip) return;
  hipError_t e = hipHostRegister(base_, bytes_, hipHostRegisterMapped | hipHostRegisterPortable);
  if (e != hipSuccess) fail(MPA_DEVICE_ERROR, "hipHostRegister of shared memory failed: %s", hipGetErrorString(e));
  registered_ = true;
  void* d = nullptr;
  e = hipHostGetDevicePointer(&d, base_, 0);
  if (e != hipSuccess) fail(MPA_DEVICE_ERROR, "hipHostGetDevicePointer failed: %s", hipGetErrorString(e));
  dbase_ = static_cast<uint8_t*>(d);
}

ShmRegion* ShmRegion::create(const std::string& name, int64_t nworkers, size_t max_msg, bool with_hip) {
  ShmRegion* r = new ShmRegion();
  r->name_ = name;
  r->owner_ = true;
  max_msg = round_up(max_msg ? max_msg : 16, 256);
  const size_t box = sizeof(BoxHeader) + 2 * max_msg;
  const size_t bytes = round_up(sizeof(ShmHeader) + size_t(nworkers) * box, 4096);
  int fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
  if (fd < 0) {
    delete r;
    fail(MPA_ERROR, "shm_open('%s') failed: %s", name.c_str(), strerror(errno));
  }
  if (ftruncate(fd, off_t(bytes)) != 0) {
    close(fd);
    shm_unlink(name.c_str());
    delete r;
    fail(MPA_ERROR, "ftruncate of shared memory failed: %s", strerror(errno));
  }
  r->linked_ = true;
  try {
    r->map_and_register(fd, bytes, with_hip);
  } catch (...) {
    delete r;
    throw;
  }
  std::memset(r->base_, 0, bytes);
  ShmHeader* h = r->header();
  h->nworkers = nworkers;
  h->max_msg = max_msg;
  h->box_bytes = box;
  h->version = kVersion;
  __atomic_store_n(&h->magic, kMagic, __ATOMIC_RELEASE);
  return r;
}

ShmRegion* ShmRegion::attach(const std::string& name, bool with_hip) {
  ShmRegion* r = new ShmRegion();
  r->name_ = name;
  int fd = shm_open(name.c_str(), O_RDWR, 0600);
  if (fd < 0) {
    delete r;
    fail(MPA_ERROR, "shm_open('%s') to attach failed: %s", name.c_str(), strerror(errno));
  }
  struct stat st;
  if (fstat(fd, &st) != 0 || st.st_size < off_t(sizeof(ShmHeader))) {
    close(fd);
    delete r;
    fail(MPA_ERROR, "shared memory '%s' is not initialised", name.c_str());
  }
  try {
    r->map_and_register(fd, size_t(st.st_size), with_hip);
  } catch (...) {
    delete r;
    throw;
  }
  if (__atomic_load_n(&r->header()->magic, __ATOMIC_ACQUIRE) != kMagic || r->header()->version != kVersion) {
    delete r;
    fail(MPA_ERROR, "shared memory '%s' has the wrong layout", name.c_str());
  }
  return r;
}

void ShmRegion::unlink_name() {
  if (owner_ && linked_) {
    shm_unlink(name_.c_str());
    linked_ = false;
  }
}

ShmRegion::~ShmRegion() {
  if (base_) {
    if (registered_) (void)hipHostUnregister(base_);
    munmap(base_, bytes_);
  }
  unlink_name();
}

}  // namespace mpa
