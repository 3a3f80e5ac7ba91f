// Pure C++ core of the native queue (no Python): MultiLevelQueue (N6) and
// the DelayedQueue timer heap (N7).  Bound to Python by mlq.cpp; built on its
// own with TSan/ASan by csrc/tests/stress_native.cpp.
//
// Behavioural parity with the reference (`internal/priorityqueue/queue.go`):
//   * each NAMED queue orders items by (priority asc, enqueue time asc)
//     (`queue.go:22-27`).  Priorities are small integers, so instead of a
//     binary heap each named queue is a *bucket queue*: one FIFO ring per
//     distinct priority value, kept sorted.  push/pop are O(#distinct prios)
//     ~ O(1) and FIFO-within-priority is exact (a monotone sequence number
//     replaces Go's `Timestamp.Before`, which is ambiguous on equal stamps).
//   * capacity: push fails with QUEUE_FULL when max_size>0 && len>=max_size
//     (`queue.go:101-103`);
//   * stats: pending++ on push; pending--/processing++ on pop;
//     processing-- and completed++/failed++ on complete/fail
//     (`queue.go:113-116,132-136,197-211`).  Wait/process totals are really
//     accumulated here (never updated in the reference -- defect D23).
//
// Differences by design:
//   * one mutex PER named queue, not one global RWMutex (D21); the queue map
//     has its own shared_mutex;
//   * stats are returned by value (D22);
//   * `pop_tiers` = the dispatcher's strict-priority batch pop across an
//     ordered tier list with aging (anti-starvation; claimed in
//     docs/architecture.md:90 but absent in the reference) and per-tier
//     in-flight budgets (`queue.levels[*].max_concurrent`, dead config keys
//     in the reference).
//   * every blocking entry point releases the GIL.
//
// The queue carries integer handles only; Python owns the Message objects.

#pragma once

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <memory>
#include <mutex>
#include <queue>
#include <shared_mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <tuple>
#include <unordered_map>
#include <vector>

namespace llmq {

static inline int64_t mono_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

enum Status : int { OK = 0, QUEUE_NOT_FOUND = 1, QUEUE_FULL = 2, QUEUE_EMPTY = 3 };

struct Item {
  int64_t handle;
  int32_t prio;
  int64_t enq_ns;
  uint64_t seq;
};

struct Stats {
  int64_t pending = 0, processing = 0, completed = 0, failed = 0;
  int64_t total_wait_ns = 0, total_process_ns = 0, last_update_ns = 0;
  int64_t pushed = 0, popped = 0, rejected_full = 0;
};

class NamedQueue {
 public:
  explicit NamedQueue(int64_t max_size) : max_size_(max_size) {}

  // caller holds mu
  int push_locked(int64_t handle, int32_t prio, int64_t now, uint64_t seq) {
    if (max_size_ > 0 && size_ >= max_size_) {
      st_.rejected_full++;
      return QUEUE_FULL;
    }
    auto it = std::lower_bound(buckets_.begin(), buckets_.end(), prio,
                               [](const Bucket& b, int32_t p) { return b.prio < p; });
    if (it == buckets_.end() || it->prio != prio) it = buckets_.insert(it, Bucket{prio, {}});
    it->ring.push_back(Item{handle, prio, now, seq});
    size_++;
    st_.pending++;
    st_.pushed++;
    st_.last_update_ns = now;
    return OK;
  }

  const Item* head_locked() const {
    for (const auto& b : buckets_)
      if (!b.ring.empty()) return &b.ring.front();
    return nullptr;
  }

  bool pop_locked(Item* out, int64_t now) {
    for (auto& b : buckets_) {
      if (!b.ring.empty()) {
        *out = b.ring.front();
        b.ring.pop_front();
        size_--;
        st_.pending--;
        st_.processing++;
        st_.popped++;
        st_.total_wait_ns += now - out->enq_ns;
        st_.last_update_ns = now;
        return true;
      }
    }
    return false;
  }

  // newest item of the most urgent non-empty bucket (adaptive LIFO)
  bool pop_tail_locked(Item* out, int64_t now) {
    for (auto& b : buckets_) {
      if (!b.ring.empty()) {
        *out = b.ring.back();
        b.ring.pop_back();
        size_--;
        st_.pending--;
        st_.processing++;
        st_.popped++;
        st_.total_wait_ns += now - out->enq_ns;
        st_.last_update_ns = now;
        return true;
      }
    }
    return false;
  }

  // Skip-aware variants: `skip` is a sorted list of handles the caller must
  // not take (turns that belong to another GPU).  Position = (bucket, index).
  static bool skipped(const std::vector<int64_t>& skip, int64_t h) {
    return std::binary_search(skip.begin(), skip.end(), h);
  }
  // oldest (tail=false) or newest (tail=true) item of the most urgent
  // bucket holding one that is not skipped
  const Item* find_locked(const std::vector<int64_t>& skip, bool tail, size_t* bi, size_t* ii) const {
    for (size_t b = 0; b < buckets_.size(); ++b) {
      const auto& r = buckets_[b].ring;
      const size_t n = r.size();
      for (size_t k = 0; k < n; ++k) {
        const size_t i = tail ? n - 1 - k : k;
        if (!skipped(skip, r[i].handle)) {
          *bi = b;
          *ii = i;
          return &r[i];
        }
      }
    }
    return nullptr;
  }
  // Oldest non-skipped item from a scan cursor (bucket, index) that only
  // moves forward: everything before it is known to be skipped.  Within one
  // pop_tiers call skipped items stay skipped and the queue is locked, so
  // each skipped handle is looked at once per call instead of once per
  // popped item (the full rescan made a pop O(count x skipped)).
  // After take_locked() at the returned position the next item shifts into
  // it, so the cursor stays valid.
  struct Cursor {
    size_t b = 0, k = 0;
  };
  const Item* find_front_locked(const std::vector<int64_t>& skip, Cursor* c, size_t* bi, size_t* ii) const {
    for (; c->b < buckets_.size(); ++c->b, c->k = 0) {
      const auto& r = buckets_[c->b].ring;
      for (; c->k < r.size(); ++c->k) {
        if (!skipped(skip, r[c->k].handle)) {
          *bi = c->b;
          *ii = c->k;
          return &r[c->k];
        }
      }
    }
    return nullptr;
  }
  void take_locked(size_t bi, size_t ii, Item* out, int64_t now) {
    auto& r = buckets_[bi].ring;
    *out = r[ii];
    if (ii == 0)
      r.pop_front();
    else if (ii + 1 == r.size())
      r.pop_back();
    else
      r.erase(r.begin() + (std::ptrdiff_t)ii);
    size_--;
    st_.pending--;
    st_.processing++;
    st_.popped++;
    st_.total_wait_ns += now - out->enq_ns;
    st_.last_update_ns = now;
  }

  // remove a specific handle (admin DELETE /queues/:type/:id)
  bool remove_locked(int64_t handle, int64_t now) {
    for (auto& b : buckets_) {
      for (auto it = b.ring.begin(); it != b.ring.end(); ++it) {
        if (it->handle == handle) {
          b.ring.erase(it);
          size_--;
          st_.pending--;
          st_.last_update_ns = now;
          return true;
        }
      }
    }
    return false;
  }

  std::vector<int64_t> snapshot_locked() const {
    std::vector<int64_t> out;
    out.reserve(size_);
    for (const auto& b : buckets_)
      for (const auto& it : b.ring) out.push_back(it.handle);
    return out;
  }

  void clear_locked(int64_t now) {
    st_.pending -= size_;
    buckets_.clear();
    size_ = 0;
    st_.last_update_ns = now;
  }

  std::mutex mu;
  Stats st_;
  int64_t size_ = 0;
  int64_t max_size_;

 private:
  struct Bucket {
    int32_t prio;
    std::deque<Item> ring;
  };
  std::vector<Bucket> buckets_;
};

class MultiLevelQueue {
 public:
  explicit MultiLevelQueue(int64_t max_size) : max_size_(max_size) {}

  // max_size < 0 -> the MLQ default; 0 -> unbounded
  void add_queue(const std::string& name, int64_t max_size) {
    std::unique_lock<std::shared_mutex> lk(map_mu_);
    if (!queues_.count(name))
      queues_.emplace(name, std::make_shared<NamedQueue>(max_size < 0 ? max_size_ : max_size));
  }
  bool remove_queue(const std::string& name) {
    std::unique_lock<std::shared_mutex> lk(map_mu_);
    return queues_.erase(name) > 0;
  }
  bool has_queue(const std::string& name) {
    std::shared_lock<std::shared_mutex> lk(map_mu_);
    return queues_.count(name) > 0;
  }
  std::vector<std::string> names() {
    std::shared_lock<std::shared_mutex> lk(map_mu_);
    std::vector<std::string> out;
    for (auto& kv : queues_) out.push_back(kv.first);
    std::sort(out.begin(), out.end());
    return out;
  }

  std::shared_ptr<NamedQueue> get(const std::string& name) {
    std::shared_lock<std::shared_mutex> lk(map_mu_);
    auto it = queues_.find(name);
    return it == queues_.end() ? nullptr : it->second;
  }

  // returns (status, enqueue_ns)
  std::pair<int, int64_t> push(const std::string& name, int64_t handle, int32_t prio) {
    auto q = get(name);
    if (!q) return {QUEUE_NOT_FOUND, 0};
    int64_t now = mono_ns();
    std::lock_guard<std::mutex> lk(q->mu);
    return {q->push_locked(handle, prio, now, seq_.fetch_add(1, std::memory_order_relaxed)), now};
  }

  // batch push into per-item queues given by index into `names`.
  std::vector<int> push_batch(const std::vector<std::string>& names, const int32_t* qi, const int64_t* h,
                              const int32_t* p, int64_t n) {
    std::vector<std::shared_ptr<NamedQueue>> qs;
    for (auto& nm : names) qs.push_back(get(nm));
    std::vector<int> status(n);
    int64_t now = mono_ns();
    for (int64_t i = 0; i < n; ++i) {
      int k = qi[i];
      if (k < 0 || k >= (int)qs.size() || !qs[k]) {
        status[i] = QUEUE_NOT_FOUND;
        continue;
      }
      std::lock_guard<std::mutex> lk(qs[k]->mu);
      status[i] = qs[k]->push_locked(h[i], p[i], now, seq_.fetch_add(1, std::memory_order_relaxed));
    }
    return status;
  }

  // (status, handle, prio, enq_ns)
  std::tuple<int, int64_t, int32_t, int64_t> pop(const std::string& name) {
    auto q = get(name);
    if (!q) return {QUEUE_EMPTY, 0, 0, 0};  // reference: missing queue -> ErrQueueEmpty
    std::lock_guard<std::mutex> lk(q->mu);
    Item it;
    if (!q->pop_locked(&it, mono_ns())) return {QUEUE_EMPTY, 0, 0, 0};
    return {OK, it.handle, it.prio, it.enq_ns};
  }

  std::tuple<int, int64_t, int32_t, int64_t> peek(const std::string& name) {
    auto q = get(name);
    if (!q) return {QUEUE_EMPTY, 0, 0, 0};
    std::lock_guard<std::mutex> lk(q->mu);
    const Item* it = q->head_locked();
    if (!it) return {QUEUE_EMPTY, 0, 0, 0};
    return {OK, it->handle, it->prio, it->enq_ns};
  }

  std::vector<int64_t> pop_batch(const std::string& name, int64_t count) {
    std::vector<int64_t> out;
    auto q = get(name);
    if (!q || count <= 0) return out;
    std::lock_guard<std::mutex> lk(q->mu);
    int64_t now = mono_ns();
    Item it;
    while ((int64_t)out.size() < count && q->pop_locked(&it, now)) out.push_back(it.handle);
    return out;
  }

  // Dispatcher batch pop: strict priority over `tiers` (ordered most urgent
  // first) with aging and per-tier budgets (<0 = unlimited).  Appends to
  // (hs, ti, enq): handle, tier index, enqueue time.
  //
  // Adaptive LIFO (`lifo_ns`, optional, per tier, 0 = off): while a tier's
  // head has waited longer than lifo_ns[i] the tier is overloaded, and its
  // NEWEST request is served instead of the oldest -- served requests keep a
  // short queue wait and the stale head runs into its deadline and is shed
  // (the gateway's expiry), instead of every request waiting nearly the
  // whole deadline under FIFO.  FIFO resumes once the head is younger.
  //
  // `skip` (optional, sorted handles): requests the caller must leave queued
  // -- a rank admitting into its own GPU passes the turns whose KV lives on
  // another GPU; they keep their queue position for the tick's plan, and
  // "head" / "newest" below mean the first / last request not skipped.
  void pop_tiers(const std::vector<std::string>& tiers, int64_t count, const std::vector<int64_t>& aging_ns,
                 std::vector<int64_t> budget, std::vector<int64_t>& hs, std::vector<int32_t>& ti,
                 std::vector<int64_t>& enq, const std::vector<int64_t>& lifo_ns = {},
                 const std::vector<int64_t>& skip = {}) {
    const size_t T = tiers.size();
    if (aging_ns.size() != T || budget.size() != T || (!lifo_ns.empty() && lifo_ns.size() != T))
      throw std::invalid_argument("tier arg mismatch");
    std::vector<std::shared_ptr<NamedQueue>> qs(T);
    for (size_t i = 0; i < T; ++i) qs[i] = get(tiers[i]);
    {
      // fixed lock order (tier index) -> no deadlock with other pop_tiers callers
      std::vector<std::unique_lock<std::mutex>> locks;
      for (size_t i = 0; i < T; ++i)
        if (qs[i]) locks.emplace_back(qs[i]->mu);
      int64_t now = mono_ns();
      hs.reserve(count);
      if (!skip.empty()) {
        pop_tiers_skip_locked(qs, count, aging_ns, budget, hs, ti, enq, lifo_ns, skip, now);
        return;
      }
      while ((int64_t)hs.size() < count) {
        int pick = -1;
        // 1) an overdue head (waited past its tier's max_wait_time): serve the
        //    most urgent overdue tier first.
        for (size_t i = 0; i < T && pick < 0; ++i) {
          if (!qs[i] || budget[i] == 0 || aging_ns[i] <= 0) continue;
          const Item* h = qs[i]->head_locked();
          if (h && now - h->enq_ns > aging_ns[i]) pick = (int)i;
        }
        // 2) otherwise strict priority.
        for (size_t i = 0; i < T && pick < 0; ++i) {
          if (!qs[i] || budget[i] == 0) continue;
          if (qs[i]->head_locked()) pick = (int)i;
        }
        if (pick < 0) break;
        Item it;
        const Item* h = qs[pick]->head_locked();
        if (!lifo_ns.empty() && lifo_ns[pick] > 0 && now - h->enq_ns > lifo_ns[pick])
          qs[pick]->pop_tail_locked(&it, now);
        else
          qs[pick]->pop_locked(&it, now);
        hs.push_back(it.handle);
        enq.push_back(it.enq_ns);
        ti.push_back(pick);
        if (budget[pick] > 0) budget[pick]--;
      }
    }
  }

 private:
  // pop_tiers' loop over the first / last request of each tier that is not
  // in `skip` (every tier locked by the caller)
  static void pop_tiers_skip_locked(const std::vector<std::shared_ptr<NamedQueue>>& qs, int64_t count,
                                    const std::vector<int64_t>& aging_ns, std::vector<int64_t>& budget,
                                    std::vector<int64_t>& hs, std::vector<int32_t>& ti, std::vector<int64_t>& enq,
                                    const std::vector<int64_t>& lifo_ns, const std::vector<int64_t>& skip,
                                    int64_t now) {
    const size_t T = qs.size();
    std::vector<NamedQueue::Cursor> cur(T);          // per tier, for the whole call
    while ((int64_t)hs.size() < count) {
      int pick = -1;
      size_t bi = 0, ii = 0;
      const Item* h = nullptr;
      for (size_t i = 0; i < T && pick < 0; ++i) {
        if (!qs[i] || budget[i] == 0 || aging_ns[i] <= 0) continue;
        const Item* c = qs[i]->find_front_locked(skip, &cur[i], &bi, &ii);
        if (c && now - c->enq_ns > aging_ns[i]) pick = (int)i, h = c;
      }
      for (size_t i = 0; i < T && pick < 0; ++i) {
        if (!qs[i] || budget[i] == 0) continue;
        const Item* c = qs[i]->find_front_locked(skip, &cur[i], &bi, &ii);
        if (c) pick = (int)i, h = c;
      }
      if (pick < 0) break;
      if (!lifo_ns.empty() && lifo_ns[pick] > 0 && now - h->enq_ns > lifo_ns[pick])
        qs[pick]->find_locked(skip, true, &bi, &ii);
      Item it;
      qs[pick]->take_locked(bi, ii, &it, now);
      hs.push_back(it.handle);
      enq.push_back(it.enq_ns);
      ti.push_back(pick);
      if (budget[pick] > 0) budget[pick]--;
    }
  }

 public:

  int64_t size(const std::string& name) {
    auto q = get(name);
    if (!q) return -1;
    std::lock_guard<std::mutex> lk(q->mu);
    return q->size_;
  }

  int64_t total_size() {
    std::vector<std::shared_ptr<NamedQueue>> qs;
    {
      std::shared_lock<std::shared_mutex> lk(map_mu_);
      for (auto& kv : queues_) qs.push_back(kv.second);
    }
    int64_t s = 0;
    for (auto& q : qs) {
      std::lock_guard<std::mutex> lk(q->mu);
      s += q->size_;
    }
    return s;
  }

  // copy of the named queue's counters (false if it does not exist)
  bool stats(const std::string& name, Stats* out) {
    auto q = get(name);
    if (!q) return false;
    std::lock_guard<std::mutex> lk(q->mu);
    *out = q->st_;
    return true;
  }

  bool complete(const std::string& name, int64_t process_ns) {
    auto q = get(name);
    if (!q) return false;
    std::lock_guard<std::mutex> lk(q->mu);
    q->st_.processing--;
    q->st_.completed++;
    q->st_.total_process_ns += process_ns;
    q->st_.last_update_ns = mono_ns();
    return true;
  }

  bool fail(const std::string& name) {
    auto q = get(name);
    if (!q) return false;
    std::lock_guard<std::mutex> lk(q->mu);
    q->st_.processing--;
    q->st_.failed++;
    q->st_.last_update_ns = mono_ns();
    return true;
  }

  // a popped message went back (retry re-push / requeue) without completing
  bool unprocess(const std::string& name) {
    auto q = get(name);
    if (!q) return false;
    std::lock_guard<std::mutex> lk(q->mu);
    q->st_.processing--;
    return true;
  }

  bool remove(const std::string& name, int64_t handle) {
    auto q = get(name);
    if (!q) return false;
    std::lock_guard<std::mutex> lk(q->mu);
    return q->remove_locked(handle, mono_ns());
  }

  std::vector<int64_t> snapshot(const std::string& name) {
    auto q = get(name);
    if (!q) return {};
    std::lock_guard<std::mutex> lk(q->mu);
    return q->snapshot_locked();
  }

  void clear(const std::string& name) {
    auto q = get(name);
    if (!q) return;
    std::lock_guard<std::mutex> lk(q->mu);
    q->clear_locked(mono_ns());
  }

  int64_t max_size() const { return max_size_; }

 private:
  int64_t max_size_;
  std::shared_mutex map_mu_;
  std::unordered_map<std::string, std::shared_ptr<NamedQueue>> queues_;
  std::atomic<uint64_t> seq_{0};
};

// --------------------------------------------------------------------------
// DelayedQueue (N7): min-heap on ready_at (monotonic ns) + a waker thread.
// Reference `delayed_queue.go`: items are delivered no earlier than ReadyAt
// (1 ms early-fire tolerance, `:136,:176`), ordered by ReadyAt.  Due items
// move to a ready FIFO that Python drains with `wait_ready` (GIL released).
class DelayedQueue {
 public:
  DelayedQueue() : stop_(false) { th_ = std::thread([this] { run(); }); }
  ~DelayedQueue() { shutdown(); }

  void shutdown() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (stop_) return;
      stop_ = true;
    }
    cv_.notify_all();
    ready_cv_.notify_all();
    if (th_.joinable()) th_.join();
  }

  // (Re)schedules ``handle``: a handle already waiting is moved to the new
  // time (its old heap entry turns stale and is skipped when it surfaces).
  void schedule(int64_t handle, int64_t ready_at_ns) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      uint64_t s = seq_++;
      live_[handle] = s;
      heap_.push(Entry{ready_at_ns, s, handle});
    }
    cv_.notify_all();
  }

  // Takes ``handle`` out of the queue, whether still waiting (lazy delete:
  // its heap entry is dropped when it reaches the top) or already due and
  // not yet drained.  False if it is not here (never scheduled, delivered).
  bool remove(int64_t handle) {
    std::lock_guard<std::mutex> lk(mu_);
    if (live_.erase(handle)) return true;
    for (auto it = ready_.begin(); it != ready_.end(); ++it) {
      if (*it == handle) {
        ready_.erase(it);
        return true;
      }
    }
    return false;
  }

  // blocks up to timeout_s for ready items; returns up to max_n handles
  std::vector<int64_t> wait_ready(int64_t max_n, double timeout_s) {
    std::vector<int64_t> out;
    std::unique_lock<std::mutex> lk(mu_);
    if (ready_.empty() && !stop_) {
      ready_cv_.wait_for(lk, std::chrono::duration<double>(timeout_s),
                         [this] { return !ready_.empty() || stop_; });
    }
    while (!ready_.empty() && (int64_t)out.size() < max_n) {
      out.push_back(ready_.front());
      ready_.pop_front();
    }
    return out;
  }

  int64_t size() {
    std::lock_guard<std::mutex> lk(mu_);
    return (int64_t)live_.size();
  }
  int64_t ready_size() {
    std::lock_guard<std::mutex> lk(mu_);
    return (int64_t)ready_.size();
  }

  // (ok, handle, ready_at_ns)
  std::tuple<bool, int64_t, int64_t> peek() {
    std::lock_guard<std::mutex> lk(mu_);
    drop_stale();
    if (heap_.empty()) return {false, 0, 0};
    return {true, heap_.top().handle, heap_.top().ready_at};
  }

  std::vector<int64_t> clear() {
    std::lock_guard<std::mutex> lk(mu_);
    std::vector<int64_t> out;
    while (!heap_.empty()) {
      const Entry& e = heap_.top();
      auto it = live_.find(e.handle);
      if (it != live_.end() && it->second == e.seq) out.push_back(e.handle);
      heap_.pop();
    }
    live_.clear();
    return out;
  }

 private:
  struct Entry {
    int64_t ready_at;
    uint64_t seq;
    int64_t handle;
    bool operator>(const Entry& o) const {
      return ready_at != o.ready_at ? ready_at > o.ready_at : seq > o.seq;
    }
  };

  void run() {
    std::unique_lock<std::mutex> lk(mu_);
    while (!stop_) {
      if (heap_.empty()) {
        cv_.wait(lk, [this] { return stop_ || !heap_.empty(); });
        continue;
      }
      int64_t now = mono_ns();
      const int64_t tol = 1000000;  // 1 ms early-fire tolerance
      bool moved = false;
      drop_stale();
      while (!heap_.empty() && heap_.top().ready_at < now + tol) {
        const Entry e = heap_.top();
        heap_.pop();
        auto it = live_.find(e.handle);
        if (it != live_.end() && it->second == e.seq) {   // (else removed / rescheduled: stale)
          live_.erase(it);
          ready_.push_back(e.handle);
          moved = true;
        }
        drop_stale();
      }
      if (moved) ready_cv_.notify_all();
      if (heap_.empty()) continue;
      auto wait = std::chrono::nanoseconds(heap_.top().ready_at - now);
      cv_.wait_for(lk, wait);
    }
  }

  // pops heap tops that no longer name a waiting item (caller holds mu_)
  void drop_stale() {
    while (!heap_.empty()) {
      const Entry& e = heap_.top();
      auto it = live_.find(e.handle);
      if (it != live_.end() && it->second == e.seq) return;
      heap_.pop();
    }
  }

  std::mutex mu_;
  std::condition_variable cv_, ready_cv_;
  std::priority_queue<Entry, std::vector<Entry>, std::greater<Entry>> heap_;
  std::unordered_map<int64_t, uint64_t> live_;   // waiting handle -> its current heap entry's seq
  std::deque<int64_t> ready_;
  uint64_t seq_ = 0;
  bool stop_;
  std::thread th_;
};

}  // namespace llmq
