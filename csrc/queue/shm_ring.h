// Process-shared request ring (SURVEY.md §5 "distributed communication
// backend" (a) and defect D14): a named POSIX shared-memory segment holding a
// bounded multi-producer / multi-consumer ring of variable-length records.
//
// The reference's microservices (cmd/api-gateway, cmd/queue-manager) each
// built a private in-process queue, so requests accepted by the gateway were
// never seen by the queue manager (cmd/api-gateway/main.go:66,
// cmd/queue-manager/main.go:58).  Here every ingress process (HTTP workers)
// pushes preprocessed messages into the ring and the dispatcher process pops
// them in batches; a second ring carries status events back.
//
// Layout: [Header (3 cache lines)] [data: cap bytes, cap a power of two].
// Records are [u32 len][u32 tag][payload][pad to 8]; a record that would
// straddle the end of the data area is preceded by a wrap marker.
// Offsets are monotonic u64 (masked on access), so full/empty never alias.
// A robust process-shared mutex guards the offsets (critical sections are a
// memcpy); consumers sleep on a shared futex bumped by every push, so an
// idle dispatcher costs nothing and wakes within microseconds.
#pragma once

#include <errno.h>
#include <fcntl.h>
#include <linux/futex.h>
#include <pthread.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <time.h>
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

constexpr uint64_t kMagic = 0x4c4c4d5152494e47ull;   // "LLMQRING"
constexpr uint32_t kVersion = 3;   // 3: owner generation + creator pid in the header
constexpr int kMaxConsumers = 64;     // consumer ids of the balanced share (pop `who`)
constexpr uint32_t kWrap = 0xffffffffu;

struct alignas(64) Header {
  std::atomic<uint64_t> magic;
  uint32_t version;
  uint32_t _pad0;
  uint64_t cap;
  // owner generation: the job incarnation that created the ring (a nonce
  // rank 0 broadcasts before any ring is opened, cli serve); an attach that
  // expects a generation refuses a segment of another incarnation -- a job
  // restarted under the same torchrun run id must never drain the dead
  // incarnation's leftover records or its balanced-share ledger
  uint64_t gen;
  int64_t creator_pid;
  pthread_mutex_t mu;
  alignas(64) uint64_t head;      // producer offset (monotonic)
  uint64_t tail;                  // consumer offset (monotonic)
  uint64_t count;                 // records in the ring
  uint64_t pushed, popped, dropped, bytes_in;
  alignas(64) std::atomic<uint32_t> seq;      // futex word: bumped by every push
  std::atomic<uint32_t> waiters;
  uint32_t _pad1;
  // balanced share (pop with `who`): records taken and the last pop attempt
  // (steady-clock ns) per consumer id, and whether it is parked in the futex
  // wait -- guarded by `mu` like the offsets
  alignas(64) uint64_t taken[kMaxConsumers];
  int64_t polled_ns[kMaxConsumers];
  uint8_t parked[kMaxConsumers];
};
static_assert(sizeof(Header) % 64 == 0, "header must be cache-line sized");

inline uint64_t align8(uint64_t x) { return (x + 7) & ~uint64_t(7); }

inline long futex(std::atomic<uint32_t>* addr, int op, uint32_t val, const timespec* ts) {
  return syscall(SYS_futex, reinterpret_cast<uint32_t*>(addr), op, val, ts, nullptr, 0);
}

class ShmRing {
 public:
  // mode "create": new ring (replacing a stale segment of the same name);
  // "attach": an existing ring; "open": attach if it exists, else create
  // (the ring -- and any requests still in it -- outlives its processes).
  // gen != 0: "create" stamps it into the header, "attach" / "open" refuse a
  // segment stamped with another generation (std::runtime_error "stale").
  ShmRing(const std::string& name, uint64_t capacity, const std::string& mode, uint64_t gen = 0)
      : name_(name.empty() || name[0] != '/' ? "/" + name : name) {
    if (mode == "attach" || (mode.empty() && capacity == 0)) {
      attach(gen);
    } else if (mode == "create" || mode.empty()) {
      shm_unlink(name_.c_str());
      if (!create(capacity, gen)) throw std::runtime_error("ShmRing create " + name_ + ": " + strerror(errno));
    } else if (mode == "open") {
      if (!create(capacity, gen)) {
        if (errno != EEXIST) throw std::runtime_error("ShmRing open " + name_ + ": " + strerror(errno));
        attach(gen);
      }
    } else {
      throw std::invalid_argument("ShmRing mode must be create|attach|open");
    }
  }
  ~ShmRing() { close(); }

  bool push(const std::string& rec, uint32_t tag) {
    std::vector<std::string> v{rec};
    return push_impl(v, tag) == 1;
  }

  size_t push_many(const std::vector<std::string>& recs, uint32_t tag) { return push_impl(recs, tag); }

  // Pop up to max_n records; waits up to timeout_ms for the first one
  // (0 = poll, <0 = wait forever).  Returns (tag, payload) pairs.
  // share > 1, who < 0: take at most ceil(count / share) of the records
  // present (at least one) -- a per-pop split of one ring drained by `share`
  // consumers; what is left goes to the next pop, so nothing is stranded.
  // That alone does not even out the totals: whichever consumer polls most
  // often still takes most (47-74k vs 37-69k per rank at 33k req/s,
  // profiles/r4_http_frontdoor_8ranks_box16{,_fair}.jsonl).
  // share > 1, 0 <= who < share: BALANCED -- consumer `who` takes what
  // brings its running total up to the even share of everything taken or
  // queued, and nothing once it is there, leaving the rest to the consumers
  // behind.  A consumer behind that has not polled for kStallNs (kParkedNs
  // while it sleeps in pop's futex wait, which a push ends) is skipped: the
  // others then take the per-pop split, so a busy, slow or dead consumer
  // delays records by at most that long and never strands them.  A deficit
  // is forgiven beyond kCatchUp records, so a consumer coming back does not
  // take the whole ring.
  static constexpr int64_t kStallNs = 2'000'000, kParkedNs = 100'000'000;
  static constexpr int64_t kCatchUp = 256;
  std::vector<std::pair<uint32_t, std::string>> pop(size_t max_n, int64_t timeout_ms, uint32_t share = 1,
                                                    int who = -1) {
    std::vector<std::pair<uint32_t, std::string>> out;
    const bool bal = share > 1 && who >= 0 && who < (int)share && share <= (uint32_t)kMaxConsumers;
    bool deferred = false;   // records were left to consumers behind: re-check within kStallNs
    auto quota = [&]() -> size_t {
      deferred = false;
      if (share <= 1) return max_n;
      const size_t fair = std::max<size_t>(1, (size_t)((h_->count + share - 1) / share));
      if (!bal) return std::min(max_n, fair);
      const int64_t now = steady_ns();
      h_->polled_ns[who] = now;
      uint64_t total = 0;
      for (uint32_t j = 0; j < share; ++j) total += h_->taken[j];
      const int64_t target = (int64_t)((total + h_->count + share - 1) / share);
      if (target - (int64_t)h_->taken[who] > kCatchUp) h_->taken[who] = (uint64_t)(target - kCatchUp);
      const int64_t mine = target - (int64_t)h_->taken[who];
      if (mine > 0) return std::min(max_n, (size_t)mine);
      for (uint32_t j = 0; j < share; ++j) {
        if ((int)j == who || (int64_t)h_->taken[j] >= target) continue;
        if (now - h_->polled_ns[j] > (h_->parked[j] ? kParkedNs : kStallNs)) return std::min(max_n, fair);
      }
      deferred = h_->count > 0;
      return 0;
    };
    auto take = [&]() {
      const size_t before = out.size();
      pop_locked(quota(), out);
      if (bal) h_->taken[who] += out.size() - before;
    };
    auto park = [&](bool on) {
      if (!bal) return;
      Lock l(h_);
      h_->parked[who] = on ? 1 : 0;
      h_->polled_ns[who] = steady_ns();
    };
    auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms < 0 ? 0 : timeout_ms);
    for (;;) {
      uint32_t seen;
      {
        Lock l(h_);
        take();
        if (!out.empty()) return out;
        seen = h_->seq.load(std::memory_order_acquire);
      }
      if (timeout_ms == 0) return out;
      timespec ts{}, *tsp = nullptr;
      if (timeout_ms > 0 || deferred) {
        int64_t ns = deferred ? kStallNs : INT64_MAX;
        if (timeout_ms > 0) {
          auto left = deadline - std::chrono::steady_clock::now();
          if (left <= std::chrono::steady_clock::duration::zero()) return out;
          ns = std::min<int64_t>(ns, std::chrono::duration_cast<std::chrono::nanoseconds>(left).count());
        }
        ts.tv_sec = ns / 1000000000;
        ts.tv_nsec = ns % 1000000000;
        tsp = &ts;
      }
      park(true);
      h_->waiters.fetch_add(1);
      long r = futex(&h_->seq, FUTEX_WAIT, seen, tsp);   // wake, timeout, or seq already changed
      h_->waiters.fetch_sub(1);
      park(false);
      if (r == 0) {
        // woken: return what is there -- possibly nothing after a wake_all,
        // so the caller can test its own stop flag
        Lock l(h_);
        take();
        return out;
      }
    }
  }

  uint64_t size() {
    Lock l(h_);
    return h_->count;
  }

  uint64_t bytes_used() {
    Lock l(h_);
    return h_->head - h_->tail;
  }

  uint64_t capacity() const { return h_ ? h_->cap : 0; }
  uint64_t generation() const { return h_ ? h_->gen : 0; }
  int64_t creator_pid() const { return h_ ? h_->creator_pid : 0; }

  // balanced-share ledger of consumers 0 .. n-1: records taken, plus any
  // deficit forgiven past kCatchUp (so >= what each actually took)
  std::vector<uint64_t> taken(int n) {
    Lock l(h_);
    std::vector<uint64_t> v;
    for (int j = 0; j < n && j < kMaxConsumers; ++j) v.push_back(h_->taken[j]);
    return v;
  }

  struct Stats {
    uint64_t size, pushed, popped, dropped_full, bytes_in, bytes_used, capacity;
  };
  Stats stats() {
    Lock l(h_);
    return Stats{h_->count, h_->pushed, h_->popped, h_->dropped, h_->bytes_in, h_->head - h_->tail, h_->cap};
  }

  // Wake every consumer blocked in pop (each returns what it finds, possibly
  // nothing); used by a process to stop its own consumer threads.
  void wake_all() {
    if (!h_) return;
    h_->seq.fetch_add(1);
    futex(&h_->seq, FUTEX_WAKE, INT32_MAX, nullptr);
  }

  void close() {
    if (base_) {
      munmap(base_, map_bytes_);
      base_ = nullptr;
      h_ = nullptr;
    }
  }

  void unlink() { shm_unlink(name_.c_str()); }
  const std::string& name() const { return name_; }

 private:
  struct Lock {
    Header* h;
    explicit Lock(Header* hh) : h(hh) {
      if (!h) throw std::runtime_error("ShmRing is closed");
      int r = pthread_mutex_lock(&h->mu);
      if (r == EOWNERDEAD) {
        // a producer/consumer died inside the critical section; offsets are
        // only published after the copy, so the ring is still consistent
        pthread_mutex_consistent(&h->mu);
      } else if (r != 0) {
        throw std::runtime_error("ShmRing mutex lock failed");
      }
    }
    ~Lock() { pthread_mutex_unlock(&h->mu); }
  };

  uint8_t* data() const { return reinterpret_cast<uint8_t*>(base_) + sizeof(Header); }

  static int64_t steady_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
  }

  void map(int fd, uint64_t bytes) {
    void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    ::close(fd);
    if (p == MAP_FAILED) throw std::runtime_error("ShmRing mmap failed: " + std::string(strerror(errno)));
    base_ = p;
    map_bytes_ = bytes;
    h_ = reinterpret_cast<Header*>(p);
  }

  // false (errno set) if the segment already exists
  bool create(uint64_t capacity, uint64_t gen) {
    uint64_t cap = 4096;
    while (cap < capacity) cap <<= 1;
    int fd = shm_open(name_.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0) return false;
    uint64_t bytes = sizeof(Header) + cap;
    if (ftruncate(fd, (off_t)bytes) != 0) {
      ::close(fd);
      throw std::runtime_error("ShmRing ftruncate failed");
    }
    map(fd, bytes);
    std::memset(static_cast<void*>(h_), 0, sizeof(Header));
    h_->version = kVersion;
    h_->cap = cap;
    h_->gen = gen;
    h_->creator_pid = (int64_t)getpid();
    pthread_mutexattr_t a;
    pthread_mutexattr_init(&a);
    pthread_mutexattr_setpshared(&a, PTHREAD_PROCESS_SHARED);
    pthread_mutexattr_setrobust(&a, PTHREAD_MUTEX_ROBUST);
    pthread_mutex_init(&h_->mu, &a);
    pthread_mutexattr_destroy(&a);
    h_->magic.store(kMagic, std::memory_order_release);   // published last
    return true;
  }

  void attach(uint64_t gen) {
    int fd = -1;
    for (int i = 0; i < 200 && fd < 0; ++i) {             // creator may still be starting
      fd = shm_open(name_.c_str(), O_RDWR, 0600);
      if (fd < 0) std::this_thread::sleep_for(std::chrono::milliseconds(10));
    }
    if (fd < 0) throw std::runtime_error("ShmRing " + name_ + " does not exist");
    struct stat st{};
    for (int i = 0; i < 200; ++i) {
      fstat(fd, &st);
      if ((uint64_t)st.st_size > sizeof(Header)) break;
      std::this_thread::sleep_for(std::chrono::milliseconds(10));
    }
    map(fd, (uint64_t)st.st_size);
    for (int i = 0; i < 200 && h_->magic.load(std::memory_order_acquire) != kMagic; ++i)
      std::this_thread::sleep_for(std::chrono::milliseconds(10));
    if (h_->magic.load() != kMagic || h_->version != kVersion) {
      close();
      throw std::runtime_error("ShmRing " + name_ + " is not an initialised ring");
    }
    if (gen != 0 && h_->gen != gen) {
      const uint64_t found = h_->gen;
      close();
      throw std::runtime_error("ShmRing " + name_ + " is stale: generation " + std::to_string(found) +
                               ", expected " + std::to_string(gen));
    }
  }

  size_t push_impl(const std::vector<std::string>& recs, uint32_t tag) {
    size_t n = 0;
    {
      Lock l(h_);
      const uint64_t cap = h_->cap, mask = cap - 1;
      for (const auto& r : recs) {
        uint64_t need = align8(8 + r.size());
        if (need > cap / 2) {            // never fits: count as dropped
          h_->dropped++;
          continue;
        }
        uint64_t off = h_->head & mask;
        uint64_t skip = (cap - off < need) ? cap - off : 0;   // wrap to the start
        if (cap - (h_->head - h_->tail) < need + skip) {
          h_->dropped += recs.size() - n;
          break;
        }
        if (skip) {
          uint32_t w[2] = {kWrap, 0};
          std::memcpy(data() + off, w, 8);
          h_->head += skip;
          off = 0;
        }
        uint32_t hdr[2] = {(uint32_t)r.size(), tag};
        std::memcpy(data() + off, hdr, 8);
        std::memcpy(data() + off + 8, r.data(), r.size());
        h_->head += need;
        h_->count++;
        h_->pushed++;
        h_->bytes_in += r.size();
        ++n;
      }
      if (n) h_->seq.fetch_add(1, std::memory_order_release);
    }
    if (n && h_->waiters.load() > 0) futex(&h_->seq, FUTEX_WAKE, INT32_MAX, nullptr);
    return n;
  }

  void pop_locked(size_t max_n, std::vector<std::pair<uint32_t, std::string>>& out) {
    const uint64_t cap = h_->cap, mask = cap - 1;
    while (h_->count > 0 && out.size() < max_n) {
      uint64_t off = h_->tail & mask;
      uint32_t hdr[2];
      std::memcpy(hdr, data() + off, 8);
      if (hdr[0] == kWrap) {
        h_->tail += cap - off;
        continue;
      }
      out.emplace_back(hdr[1], std::string(reinterpret_cast<const char*>(data() + off + 8), hdr[0]));
      h_->tail += align8(8 + hdr[0]);
      h_->count--;
      h_->popped++;
    }
  }

  std::string name_;
  void* base_ = nullptr;
  uint64_t map_bytes_ = 0;
  Header* h_ = nullptr;
};

}  // namespace llmq
