// Node-local control-plane collectives over POSIX shared memory.
//
// The serving job is one process per GPU on ONE node (the 8 MI355X of a
// box).  Every scheduler tick all ranks exchange a ~1 KiB load vector and a
// few KiB of request descriptors.  Over gloo that is several TCP round trips
// per tick (1.5 ms p50 / 3 ms p99 at 8 ranks on a MI355X box,
// profiles/r2_control_plane.md); over RCCL it queues behind the forward's
// GEMMs for CUs.  Here each rank owns a slot in one shared segment:
//
//   publish(op k):  wait until every rank has published op k-1 (so all of
//                   them are done reading op k-2, which used the same buffer
//                   parity), memcpy the payload into my buffer k&1, store the
//                   size, then `pub = k` with release order;
//   collect(op k):  wait until every rank's `pub >= k` (acquire), read.
//
// Two buffers per rank (by op parity) make that safe without a second
// barrier per op.  Waits spin briefly, then yield, then sleep in 20 us steps,
// and give up after a deadline (a dead peer becomes a Python PeerLost, never
// a hang).  The reference has no inter-process transport at all (SURVEY.md
// §0); this replaces the per-tick gloo collectives of parallel/comm.py when
// every rank is on the same node.
#pragma once

#include <fcntl.h>
#include <immintrin.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace llmq {

class ShmCollTimeout : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

class ShmCollective {
 public:
  static constexpr uint64_t kMagic = 0x6c6c6d71636f6c6cULL;   // "llmqcoll"

  // create=true: rank 0 makes a fresh segment (an old one of the same name is
  // replaced); create=false: attach to the segment rank 0 made.
  ShmCollective(const std::string& name, int world, int rank, uint64_t buf_bytes, bool create)
      : name_(name), world_(world), rank_(rank) {
    if (world < 1 || rank < 0 || rank >= world) throw std::invalid_argument("ShmCollective: bad world/rank");
    buf_bytes = (buf_bytes + 4095) & ~uint64_t(4095);
    const uint64_t slots_off = 256;
    const uint64_t bufs_off = (slots_off + sizeof(Slot) * world + 4095) & ~uint64_t(4095);
    bytes_ = bufs_off + (uint64_t)world * 2 * buf_bytes;
    int fd;
    if (create) {
      shm_unlink(name.c_str());
      fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
      if (fd < 0) throw std::runtime_error("ShmCollective: shm_open(create) failed: " + std::string(strerror(errno)));
      if (ftruncate(fd, (off_t)bytes_) != 0) {
        close(fd);
        throw std::runtime_error("ShmCollective: ftruncate failed: " + std::string(strerror(errno)));
      }
    } else {
      fd = shm_open(name.c_str(), O_RDWR, 0600);
      if (fd < 0) throw std::runtime_error("ShmCollective: shm_open(attach) failed: " + std::string(strerror(errno)));
      struct stat st {};
      if (fstat(fd, &st) != 0 || (uint64_t)st.st_size < bytes_) {
        close(fd);
        throw std::runtime_error("ShmCollective: segment size mismatch");
      }
    }
    void* p = mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) throw std::runtime_error("ShmCollective: mmap failed: " + std::string(strerror(errno)));
    base_ = static_cast<uint8_t*>(p);
    hdr_ = reinterpret_cast<Header*>(base_);
    slots_ = reinterpret_cast<Slot*>(base_ + slots_off);
    bufs_ = base_ + bufs_off;
    if (create) {
      for (int r = 0; r < world; ++r) {
        new (&slots_[r]) Slot();
        slots_[r].pub.store(0, std::memory_order_relaxed);
      }
      hdr_->world = (uint32_t)world;
      hdr_->buf_bytes = buf_bytes;
      hdr_->attached.store(0, std::memory_order_relaxed);
      std::atomic_thread_fence(std::memory_order_release);
      hdr_->magic = kMagic;
    } else if (hdr_->magic != kMagic || hdr_->world != (uint32_t)world || hdr_->buf_bytes != buf_bytes) {
      munmap(base_, bytes_);
      base_ = nullptr;
      throw std::runtime_error("ShmCollective: segment header mismatch (stale or foreign segment)");
    }
    buf_bytes_ = buf_bytes;
    hdr_->attached.fetch_add(1, std::memory_order_acq_rel);
  }

  ~ShmCollective() {
    if (base_) munmap(base_, bytes_);
  }

  ShmCollective(const ShmCollective&) = delete;
  ShmCollective& operator=(const ShmCollective&) = delete;

  int attached() const { return (int)hdr_->attached.load(std::memory_order_acquire); }
  int world() const { return world_; }
  int rank() const { return rank_; }
  void unlink() { shm_unlink(name_.c_str()); }
  uint64_t ops() const { return seq_; }
  uint64_t buf_bytes() const { return buf_bytes_; }
  static constexpr uint64_t kOverflow = ~uint64_t(0);

  // Every rank contributes `n` bytes; afterwards payload(r) is rank r's.
  // An oversized payload is published as an overflow marker instead of
  // throwing before the publish: every rank then fails the SAME op at once
  // (std::length_error) instead of the others spinning to their timeout.
  void exchange(const void* data, uint64_t n, double timeout_s) {
    post(data, n, timeout_s);
    complete(timeout_s);
  }

  // Split phase (the gateway keeps ingesting while its peers catch up):
  // post() publishes this rank's payload of the next op and returns at once
  // (it only waits for every rank to have published the PREVIOUS op, which a
  // rank that completed that op already knows); ready() tells whether every
  // rank has published it; complete() waits for that and checks overflow.
  // payload() is valid after complete().  One op in flight per rank.
  void post(const void* data, uint64_t n, double timeout_s) {
    if (posted_) throw std::logic_error("ShmCollective: post() while an op is in flight");
    const bool over = n > buf_bytes_;
    const uint64_t k = seq_ + 1;
    wait_all(k - 1, deadline_after(timeout_s));
    const int par = (int)(k & 1);
    if (n && !over) std::memcpy(buf(rank_, par), data, n);
    slots_[rank_].nbytes[par] = over ? kOverflow : n;
    slots_[rank_].pub.store(k, std::memory_order_release);
    seq_ = k;
    posted_ = true;
  }

  bool ready() const {
    for (int r = 0; r < world_; ++r)
      if (slots_[r].pub.load(std::memory_order_acquire) < seq_) return false;
    return true;
  }

  void complete(double timeout_s) {
    if (!posted_) throw std::logic_error("ShmCollective: complete() without post()");
    posted_ = false;
    wait_all(seq_, deadline_after(timeout_s));
    const int par = (int)(seq_ & 1);
    for (int r = 0; r < world_; ++r)
      if (slots_[r].nbytes[par] == kOverflow)
        throw std::length_error("ShmCollective: rank " + std::to_string(r) +
                                "'s payload exceeds the per-rank buffer of " + std::to_string(buf_bytes_) + " bytes");
  }

  // Non-blocking: how many OTHER ranks have already published the next op
  // (are waiting in it).  world - 1 means joining now completes it at once.
  int arrived_next() const {
    const uint64_t k = seq_ + 1;
    int n = 0;
    for (int r = 0; r < world_; ++r)
      if (r != rank_ && slots_[r].pub.load(std::memory_order_acquire) >= k) ++n;
    return n;
  }

  // After exchange(): rank r's payload of the last op.
  const uint8_t* payload(int r, uint64_t* n) const {
    const int par = (int)(seq_ & 1);
    *n = slots_[r].nbytes[par];
    return buf(r, par);
  }

 private:
  using clock = std::chrono::steady_clock;

  struct alignas(128) Header {
    uint64_t magic;
    uint32_t world;
    uint32_t pad;
    uint64_t buf_bytes;
    std::atomic<uint32_t> attached;
  };
  struct alignas(128) Slot {
    std::atomic<uint64_t> pub{0};
    uint64_t nbytes[2] = {0, 0};
  };

  uint8_t* buf(int r, int par) const { return bufs_ + ((uint64_t)r * 2 + par) * buf_bytes_; }

  static clock::time_point deadline_after(double timeout_s) {
    return clock::now() + std::chrono::duration_cast<clock::duration>(std::chrono::duration<double>(timeout_s));
  }

  void wait_all(uint64_t k, clock::time_point deadline) const {
    if (k == 0) return;
    for (int r = 0; r < world_; ++r) {
      int spins = 0;
      while (slots_[r].pub.load(std::memory_order_acquire) < k) {
        if (++spins < 2000) {
          _mm_pause();
        } else if (spins < 2100) {
          std::this_thread::yield();
        } else {
          if (clock::now() > deadline)
            throw ShmCollTimeout("rank " + std::to_string(rank_) + ": rank " + std::to_string(r) +
                                 " did not reach control op " + std::to_string(k));
          std::this_thread::sleep_for(std::chrono::microseconds(20));
        }
      }
    }
  }

  std::string name_;
  int world_, rank_;
  uint64_t bytes_ = 0, buf_bytes_ = 0, seq_ = 0;
  bool posted_ = false;
  uint8_t* base_ = nullptr;
  Header* hdr_ = nullptr;
  Slot* slots_ = nullptr;
  uint8_t* bufs_ = nullptr;
};

}  // namespace llmq
