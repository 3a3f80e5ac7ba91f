// Multi-threaded stress of the native host runtime, built WITHOUT Python so it
// can run under ThreadSanitizer / AddressSanitizer+UBSan (SURVEY.md §5 "race
// detection": the reference relies on `go test -race`, .github/workflows/go.yml:27).
//
//   g++ -std=c++17 -O1 -g -fsanitize=thread -Icsrc csrc/tests/stress_native.cpp -o /tmp/stress -lrt -pthread
//   /tmp/stress            # exit 0 = every invariant held (sanitizer reports fail the run)
//
// Covers: MultiLevelQueue (concurrent push/push_batch/pop_tiers/pop_batch/
// stats/complete across 4 tiers, exactly-once delivery, FIFO per producer
// within a tier), DelayedQueue (concurrent schedule + wait_ready, no early
// delivery), ShmRing (2 handles on one segment, MPMC exactly-once), Guard
// (concurrent token buckets never admit more than burst + rate x elapsed;
// concurrent JWT verification), ShmCollective (4 ranks as threads: every
// rank sees every other rank's payload of the same op over thousands of
// variable-size exchanges, both buffer parities; a rank that stops makes the
// others time out instead of hanging).
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <memory>
#include <random>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "ingress/guard.h"
#include "queue/mlq_core.h"
#include "queue/shm_coll.h"
#include "queue/shm_ring.h"
#include "text/text_cpu.h"

#define CHECK(c)                                                              \
  do {                                                                        \
    if (!(c)) {                                                               \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                           \
    }                                                                         \
  } while (0)

static void stress_mlq() {
  using namespace llmq;
  MultiLevelQueue q(0);
  const std::vector<std::string> tiers = {"realtime", "high", "normal", "low"};
  for (auto& t : tiers) q.add_queue(t, -1);
  constexpr int P = 4, N = 20000;
  std::atomic<int> done_producers{0};
  std::vector<std::thread> th;
  for (int p = 0; p < P; ++p) {
    th.emplace_back([&, p] {
      // handles are pushed in increasing order: runs of 64 via push_batch,
      // then 32 single pushes
      std::vector<int32_t> qi, pr;
      std::vector<int64_t> hs;
      for (int i = 0; i < N;) {
        if ((i / 32) % 3 != 2) {
          for (int k = 0; k < 64 && i < N; ++k, ++i) {
            int64_t h = (int64_t)p * N + i;
            qi.push_back((int32_t)(h % 4));
            hs.push_back(h);
            pr.push_back((int32_t)(h % 4) + 1);
          }
          auto st = q.push_batch(tiers, qi.data(), hs.data(), pr.data(), (int64_t)qi.size());
          for (int s : st) CHECK(s == OK);
          qi.clear(); hs.clear(); pr.clear();
        } else {
          for (int k = 0; k < 32 && i < N; ++k, ++i) {
            int64_t h = (int64_t)p * N + i;
            CHECK(q.push(tiers[h % 4], h, (int32_t)(h % 4) + 1).first == OK);
          }
        }
      }
      done_producers++;
    });
  }
  std::vector<std::vector<int64_t>> got(3);
  for (int c = 0; c < 3; ++c) {
    th.emplace_back([&, c] {
      std::vector<int64_t> hs, enq;
      std::vector<int32_t> ti;
      while (true) {
        bool fin = done_producers.load() == P;
        hs.clear(); ti.clear(); enq.clear();
        if (c == 2) {
          for (auto& t : tiers) {
            auto v = q.pop_batch(t, 17);
            for (auto h : v) { hs.push_back(h); ti.push_back((int32_t)(h % 4)); }
          }
        } else {
          q.pop_tiers(tiers, 97, {1000000, 0, 0, 5000000}, {-1, 50, -1, 20}, hs, ti, enq);
        }
        for (size_t k = 0; k < hs.size(); ++k) {
          CHECK(hs[k] % 4 == ti[k]);
          got[c].push_back(hs[k]);
          CHECK(q.complete(tiers[ti[k]], 10));
        }
        Stats s;
        CHECK(q.stats(tiers[c], &s));
        CHECK(s.pending >= 0);
        if (fin && hs.empty() && q.total_size() == 0) break;
      }
    });
  }
  for (auto& t : th) t.join();
  std::vector<int64_t> all;
  for (auto& g : got) all.insert(all.end(), g.begin(), g.end());
  std::sort(all.begin(), all.end());
  CHECK((int)all.size() == P * N);
  for (int i = 0; i < P * N; ++i) CHECK(all[i] == i);
  // per consumer: handles of one producer within one tier arrive in push order
  for (auto& g : got) {
    std::map<std::pair<int64_t, int64_t>, int64_t> last;
    for (auto h : g) {
      auto key = std::make_pair(h / N, h % 4);
      auto it = last.find(key);
      CHECK(it == last.end() || it->second < h);
      last[key] = h;
    }
  }
  int64_t completed = 0;
  for (auto& t : tiers) {
    Stats s;
    CHECK(q.stats(t, &s));
    CHECK(s.pending == 0 && s.processing == 0);
    completed += s.completed;
  }
  CHECK(completed == (int64_t)P * N);
  std::printf("mlq: %d items, 4 producers / 3 consumers OK\n", P * N);
}

static void stress_delayed() {
  using namespace llmq;
  DelayedQueue d;
  constexpr int P = 4, N = 500;
  std::vector<std::thread> th;
  std::vector<int64_t> due((size_t)P * N);
  for (int p = 0; p < P; ++p) {
    th.emplace_back([&, p] {
      for (int i = 0; i < N; ++i) {
        int64_t h = (int64_t)p * N + i;
        int64_t at = mono_ns() + (h % 37) * 200000;   // 0..7.2 ms
        due[h] = at;
        d.schedule(h, at);
      }
    });
  }
  std::set<int64_t> seen;
  std::thread cons([&] {
    while ((int)seen.size() < P * N) {
      auto v = d.wait_ready(64, 0.05);
      int64_t now = mono_ns();
      for (auto h : v) {
        CHECK(seen.insert(h).second);
        CHECK(now >= due[h] - 1000000);          // 1 ms early-fire tolerance
      }
    }
  });
  for (auto& t : th) t.join();
  cons.join();
  CHECK(d.size() == 0);
  d.shutdown();
  std::printf("delayed: %d items OK\n", P * N);
}

static void stress_ring() {
  using llmq::ShmRing;
  std::string name = "/llmq-stress-" + std::to_string(getpid());
  ShmRing a(name, 1 << 14, "create");
  ShmRing b(name, 0, "attach");
  constexpr int P = 3, N = 20000;
  std::vector<std::thread> th;
  for (int p = 0; p < P; ++p) {
    th.emplace_back([&, p] {
      ShmRing& r = (p % 2) ? a : b;
      for (int i = 0; i < N;) {
        std::string rec = std::to_string(p * N + i) + std::string(i % 40, '.');
        if (r.push(rec, (uint32_t)p)) ++i;
        else std::this_thread::yield();
      }
    });
  }
  std::atomic<int> total{0};
  std::vector<std::vector<int>> got(2);
  for (int c = 0; c < 2; ++c) {
    th.emplace_back([&, c] {
      ShmRing& r = c ? a : b;
      while (total.load() < P * N) {
        auto v = r.pop(32, 5, 2, c);          // balanced share between the two consumers
        for (auto& kv : v) {
          int id = std::atoi(kv.second.c_str());
          CHECK((int)kv.first == id / N);
          got[c].push_back(id);
        }
        total += (int)v.size();
      }
      r.wake_all();
    });
  }
  for (auto& t : th) t.join();
  std::vector<int> all;
  for (auto& g : got) all.insert(all.end(), g.begin(), g.end());
  std::sort(all.begin(), all.end());
  CHECK((int)all.size() == P * N);
  for (int i = 0; i < P * N; ++i) CHECK(all[i] == i);
  CHECK(!got[0].empty() && !got[1].empty());
  auto tk = a.taken(2);
  // the balance ledger counts what each consumer took, plus deficits forgiven
  // past kCatchUp (a consumer far behind is not owed the whole ring)
  CHECK(tk[0] >= got[0].size() && tk[1] >= got[1].size());
  auto s = a.stats();
  CHECK(s.size == 0 && s.pushed == (uint64_t)P * N && s.popped == (uint64_t)P * N);
  a.unlink();
  std::printf("shm ring: %d records, 3 producers / 2 balanced consumers (%zu / %zu) OK\n", P * N, got[0].size(),
              got[1].size());
}

static void stress_shm_coll() {
  using llmq::ShmCollective;
  const std::string name = "/llmq-coll-stress-" + std::to_string(getpid());
  constexpr int W = 4, OPS = 3000;
  std::vector<std::unique_ptr<ShmCollective>> c(W);
  c[0] = std::make_unique<ShmCollective>(name, W, 0, 1 << 16, true);
  for (int r = 1; r < W; ++r) c[r] = std::make_unique<ShmCollective>(name, W, r, 1 << 16, false);
  CHECK(c[0]->attached() == W);
  std::vector<std::thread> th;
  for (int r = 0; r < W; ++r) {
    th.emplace_back([&, r] {
      std::vector<uint32_t> buf;
      for (int op = 0; op < OPS; ++op) {
        const int n = 1 + (r * 7 + op * 13) % 300;     // words this rank sends this op
        buf.assign(n, 0);
        for (int i = 0; i < n; ++i) buf[i] = (uint32_t)(r << 24) ^ (uint32_t)(op << 8) ^ (uint32_t)i;
        c[r]->exchange(buf.data(), 4ull * n, 30.0);
        for (int s = 0; s < W; ++s) {
          uint64_t nb = 0;
          const uint32_t* p = reinterpret_cast<const uint32_t*>(c[r]->payload(s, &nb));
          const int ns = 1 + (s * 7 + op * 13) % 300;
          CHECK(nb == 4ull * ns);
          for (int i = 0; i < ns; ++i) CHECK(p[i] == ((uint32_t)(s << 24) ^ (uint32_t)(op << 8) ^ (uint32_t)i));
        }
      }
    });
  }
  for (auto& t : th) t.join();
  for (int r = 0; r < W; ++r) CHECK(c[r]->ops() == (uint64_t)OPS);
  // rank W-1 stops: the others must give up within the timeout, not hang
  std::atomic<int> timeouts{0};
  th.clear();
  for (int r = 0; r < W - 1; ++r) {
    th.emplace_back([&, r] {
      uint32_t v = (uint32_t)r;
      try {
        c[r]->exchange(&v, 4, 0.3);
      } catch (const llmq::ShmCollTimeout&) {
        ++timeouts;
      }
    });
  }
  for (auto& t : th) t.join();
  CHECK(timeouts.load() == W - 1);
  c[0]->unlink();
  std::printf("shm collective: %d ranks x %d exchanges OK, dead-peer timeout OK\n", W, OPS);
}

static void fuzz_text_cpu() {
  // the CPU twin of the preprocess kernel reads untrusted request bodies:
  // random bytes (invalid UTF-8, truncated sequences, fold-special bytes,
  // Unicode spaces at the very end) of random lengths, with a pattern table
  // that includes bordered and case-insensitive patterns -- every message is
  // analysed in an exactly-sized heap buffer so ASan sees any overread
  using llmq::textcpu::Analyzer;
  using llmq::textcpu::PatternTable;
  PatternTable pt{};
  const char* pats[] = {"urgent", "aa", "\xc5\xbf", "now", "zz"};
  pt.npat = 5;
  for (int j = 0; j < pt.npat; ++j) {
    const std::string p = j == 2 ? std::string("\xe2\x80", 2) : std::string(pats[j]);
    std::memset(pt.text[j], 0, 16);
    std::memcpy(pt.text[j], p.data(), p.size());
    std::memset(pt.mask[j], 0, 16);
    std::memset(pt.mask[j], 0xFF, p.size());
    pt.len[j] = (int)p.size();
    pt.slot[j] = j % 8;
    pt.flags[j] = (j == 0 ? 1 : 0) | (j == 1 || j == 4 ? 2 : 0);
  }
  const Analyzer an(pt, 64);
  std::mt19937 rng(7);
  const uint8_t alphabet[] = {' ', 'a', 'A', 'z', 'u', '?', 0xC2, 0x85, 0xA0, 0xE2, 0x80, 0x81, 0x9F, 0xE3,
                              0xC5, 0xBF, 0xC4, 0xB0, 0x84, 0xAA, 0xF0, 0x9F, 0x98, 0x80, 0xFF, 0x00, '\t'};
  int32_t st[16];
  uint32_t h[64];
  long words = 0;
  for (int it = 0; it < 20000; ++it) {
    const int len = (int)(rng() % 300);
    std::unique_ptr<uint8_t[]> buf(new uint8_t[len > 0 ? len : 1]);
    for (int i = 0; i < len; ++i)
      buf[i] = (rng() & 3) ? alphabet[rng() % sizeof(alphabet)] : (uint8_t)rng();
    an.analyze(buf.get(), len, st, h);
    CHECK(st[5] >= 0 && st[5] <= 64 && st[5] <= st[0] && st[0] <= len);
    words += st[0];
  }
  std::printf("text cpu fuzz: 20000 random messages, %ld words, no fault\n", words);
}

static void stress_guard() {
  // 8 threads hammer one global bucket + per-user buckets with a fixed clock
  // window: admitted count must equal the token budget exactly.
  llmq::Guard g("jwt", "X-API-Key", {}, "k", "", 0, true, {{"user", {"message:*"}}}, "user", 1000.0, 50.0, 0, 0,
                1000.0, 100.0);
  std::vector<std::string> toks;
  for (int t = 0; t < 8; ++t) toks.push_back(g.sign_jwt("{\"sub\":\"t" + std::to_string(t) + "\"}"));
  std::atomic<int> ok_global{0}, ok_user{0}, bad{0};
  const int64_t t0 = 1'000'000'000;
  std::vector<std::thread> th;
  for (int t = 0; t < 8; ++t)
    th.emplace_back([&, t] {
      for (int i = 0; i < 200; ++i) {
        // 100 ms of simulated time spread over the calls: global gets 50 + 100 tokens
        const int64_t now = t0 + (int64_t)i * 500'000;
        auto r = g.check("POST", "/api/v1/messages", "10.0.0." + std::to_string(t), "", "Bearer " + toks[t], "", now, 0);
        if (r.code == 0) ok_global++;
        else if (r.code != 429) bad++;
        double ra = 0;
        if (g.allow_user("u" + std::to_string(t & 1), &ra)) ok_user++;
      }
    });
  for (auto& x : th) x.join();
  CHECK(bad.load() == 0);
  // every admitted request consumed one token: <= burst + rps * 0.1 s (+1 for the refill boundary)
  CHECK(ok_global.load() >= 50 && ok_global.load() <= 151);
  CHECK(ok_user.load() >= 2 * 100);   // two users, burst 100 each (real clock refills on top)
  std::printf("guard: %d admitted of 1600 (global budget 150), JWT verified concurrently OK\n", ok_global.load());
}

// The JWT / claim parser reads untrusted bytes: mutate valid tokens and feed
// random strings; every result must be a clean 401 or a valid verdict (ASan /
// UBSan builds of this harness catch any out-of-bounds read).
static void fuzz_guard_parser() {
  llmq::Guard g("jwt", "X-API-Key", {}, "secret", "iss", 0, false, {}, "user", 0, 0, 0, 0, 0, 0);
  const std::string good = g.sign_jwt("{\"sub\":\"a\",\"iss\":\"iss\",\"exp\":9999999999,\"x\":[1,{\"y\":\"\\u00e9\"}]}");
  std::mt19937_64 rng(7);
  const std::string alphabet = "ABCxyz019-_.=\"{}[]:,\\ u\x00\xff";
  int ok = 0, rejected = 0;
  for (int i = 0; i < 20000; ++i) {
    std::string t;
    if (i % 2 == 0) {
      t = good;
      const int edits = 1 + (int)(rng() % 4);
      for (int e = 0; e < edits && !t.empty(); ++e) {
        const size_t at = rng() % t.size();
        switch (rng() % 3) {
          case 0: t[at] = alphabet[rng() % alphabet.size()]; break;
          case 1: t.erase(at, 1 + rng() % 8); break;
          default: t.insert(at, 1, alphabet[rng() % alphabet.size()]);
        }
      }
    } else {
      const size_t n = rng() % 96;
      for (size_t k = 0; k < n; ++k) t.push_back(alphabet[rng() % alphabet.size()]);
    }
    auto r = g.check("GET", "/api/v1/messages", "", "", "Bearer " + t, "", 1, 1'700'000'000);
    CHECK(r.code == 0 || r.code == 401);
    (r.code == 0 ? ok : rejected)++;
    llmq::Claims c;
    llmq::parse_claims(t, &c);                 // raw parser on arbitrary bytes
  }
  CHECK(g.check("GET", "/api/v1/messages", "", "", "Bearer " + good, "", 1, 1'700'000'000).code == 0);
  std::printf("guard parser fuzz: 20000 inputs, %d accepted, %d rejected, no fault\n", ok, rejected);
}

int main() {
  stress_mlq();
  stress_delayed();
  stress_ring();
  stress_shm_coll();
  fuzz_text_cpu();
  stress_guard();
  fuzz_guard_parser();
  std::printf("ALL OK\n");
  return 0;
}
