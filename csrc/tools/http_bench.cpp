// Open-loop HTTP load generator for POST /api/v1/messages (the reference's
// k6 / Go load tests are doc-only, docs/performance.md:1039-1155).  Python
// clients saturate at a few thousand requests/s; this one keeps the client
// out of the measurement.
//
//   g++ -O2 -std=c++17 -pthread csrc/tools/http_bench.cpp -o /tmp/http_bench
//   /tmp/http_bench <host> <port> <rate_total> <seconds> <threads> <conns_per_thread> [bodies.jsonl]
//
// With a bodies file (one JSON body per line -- e.g. bench.py's synthetic
// 4-tier workload, written by bench/http_load.py) requests cycle through it
// in order; otherwise four fixed bodies are drawn with the 10/30/40/20 mix.
//
// Each thread owns `conns` keep-alive connections and issues requests on a
// Poisson schedule at rate/threads, round-robin over its connections,
// pipelining when a connection is still busy (latency is measured from the
// scheduled send time, so queueing in the client counts against the server:
// no coordinated omission).  Prints one JSON line.
#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <random>
#include <string>
#include <thread>
#include <vector>

static int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

static const char* kBodies[4] = {
    "{\"content\":\"EMERGENCY: the payment service is down right now\",\"user_id\":\"rt\"}",
    "{\"content\":\"urgent: please review the deploy before noon\",\"user_id\":\"hi\"}",
    "{\"content\":\"can you summarise the meeting notes for the team?\",\"user_id\":\"n\"}",
    "{\"content\":\"background batch job report\",\"user_id\":\"lo\",\"priority\":\"low\"}"};
static const double kMix[4] = {0.1, 0.3, 0.4, 0.2};

struct Conn {
  int fd = -1;
  std::deque<int64_t> sent;   // scheduled times of requests awaiting a response
  std::string in, out;
};

struct Result {
  std::vector<int64_t> lat;
  int64_t ok = 0, other = 0, errors = 0, sent = 0;
};

static int dial(const char* host, int port) {
  int fd = socket(AF_INET, SOCK_STREAM, 0);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons(port);
  inet_pton(AF_INET, host, &a.sin_addr);
  if (connect(fd, (sockaddr*)&a, sizeof a) < 0) {
    close(fd);
    return -1;
  }
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  fcntl(fd, F_SETFL, O_NONBLOCK);
  return fd;
}

static std::vector<std::string> g_file_bodies;

static void worker(const char* host, int port, double rate, double secs, int nconn, uint64_t seed, Result* res,
                   int tid, int nthreads) {
  std::vector<Conn> cs(nconn);
  for (auto& c : cs) c.fd = dial(host, port);
  std::mt19937_64 rng(seed);
  std::exponential_distribution<double> gap(rate);
  std::discrete_distribution<int> pick(kMix, kMix + 4);
  std::vector<std::string> reqs;
  auto add = [&](const std::string& b) {
    char hdr[256];
    snprintf(hdr, sizeof hdr, "POST /api/v1/messages HTTP/1.1\r\nHost: x\r\nContent-Type: application/json\r\n"
                              "Content-Length: %zu\r\n\r\n", b.size());
    reqs.push_back(std::string(hdr) + b);
  };
  if (!g_file_bodies.empty()) {
    for (size_t i = (size_t)tid; i < g_file_bodies.size(); i += (size_t)nthreads) add(g_file_bodies[i]);
  } else {
    for (auto* b : kBodies) add(b);
  }
  const bool from_file = !g_file_bodies.empty() && !reqs.empty();
  size_t next_body = 0;
  const int64_t t0 = now_ns(), t_end = t0 + (int64_t)(secs * 1e9);
  int64_t t_next = t0;
  size_t rr = 0;
  std::vector<pollfd> pf(nconn);
  char buf[65536];
  auto outstanding = [&] {
    size_t n = 0;
    for (auto& c : cs) n += c.sent.size();
    return n;
  };
  while (true) {
    const int64_t now = now_ns();
    if (now >= t_end && outstanding() == 0) break;
    if (now > t_end + (int64_t)10e9) break;                          // drain limit
    while (t_next <= now && t_next < t_end) {                        // due requests
      Conn& c = cs[rr++ % cs.size()];
      if (c.fd < 0) {
        res->errors++;
      } else {
        c.out += from_file ? reqs[next_body++ % reqs.size()] : reqs[pick(rng)];
        c.sent.push_back(t_next);
        res->sent++;
      }
      t_next += (int64_t)(gap(rng) * 1e9);
    }
    for (size_t i = 0; i < cs.size(); ++i) {
      pf[i].fd = cs[i].fd;
      pf[i].events = POLLIN | (cs[i].out.empty() ? 0 : POLLOUT);
      pf[i].revents = 0;
    }
    int64_t wait_ms = t_next < t_end ? std::max<int64_t>(0, (t_next - now_ns()) / 1000000) : 10;
    poll(pf.data(), pf.size(), (int)std::min<int64_t>(wait_ms, 10));
    for (size_t i = 0; i < cs.size(); ++i) {
      Conn& c = cs[i];
      if (c.fd < 0) continue;
      if ((pf[i].revents & POLLOUT) && !c.out.empty()) {
        ssize_t w = write(c.fd, c.out.data(), c.out.size());
        if (w > 0) c.out.erase(0, (size_t)w);
      }
      if (pf[i].revents & (POLLIN | POLLHUP | POLLERR)) {
        ssize_t r = read(c.fd, buf, sizeof buf);
        if (r <= 0) {
          res->errors += (int64_t)c.sent.size();
          c.sent.clear();
          close(c.fd);
          c.fd = dial(host, port);
          continue;
        }
        c.in.append(buf, (size_t)r);
        for (;;) {                                                   // complete responses
          size_t he = c.in.find("\r\n\r\n");
          if (he == std::string::npos) break;
          size_t cl = 0;
          const char* p = strcasestr(c.in.c_str(), "content-length:");
          if (p && (size_t)(p - c.in.c_str()) < he) cl = strtoul(p + 15, nullptr, 10);
          if (c.in.size() < he + 4 + cl) break;
          int code = atoi(c.in.c_str() + 9);
          if (!c.sent.empty()) {
            res->lat.push_back(now_ns() - c.sent.front());
            c.sent.pop_front();
          }
          if (code == 202) res->ok++;
          else res->other++;
          c.in.erase(0, he + 4 + cl);
        }
      }
    }
  }
  for (auto& c : cs)
    if (c.fd >= 0) close(c.fd);
}

int main(int argc, char** argv) {
  if (argc < 7) {
    fprintf(stderr, "usage: %s host port rate seconds threads conns_per_thread\n", argv[0]);
    return 2;
  }
  const char* host = argv[1];
  int port = atoi(argv[2]);
  double rate = atof(argv[3]), secs = atof(argv[4]);
  int threads = atoi(argv[5]), conns = atoi(argv[6]);
  if (argc > 7) {
    FILE* f = fopen(argv[7], "r");
    if (!f) {
      fprintf(stderr, "cannot open %s\n", argv[7]);
      return 2;
    }
    char* line = nullptr;
    size_t cap = 0;
    ssize_t n;
    while ((n = getline(&line, &cap, f)) > 0) {
      while (n > 0 && (line[n - 1] == '\n' || line[n - 1] == '\r')) --n;
      if (n > 0) g_file_bodies.emplace_back(line, (size_t)n);
    }
    free(line);
    fclose(f);
  }
  std::vector<Result> rs(threads);
  std::vector<std::thread> th;
  const int64_t t0 = now_ns();
  for (int i = 0; i < threads; ++i)
    th.emplace_back(worker, host, port, rate / threads, secs, conns, 1234567ull * (i + 1), &rs[i], i, threads);
  for (auto& t : th) t.join();
  const double wall = (now_ns() - t0) / 1e9;
  std::vector<int64_t> lat;
  int64_t ok = 0, other = 0, err = 0, sent = 0;
  for (auto& r : rs) {
    lat.insert(lat.end(), r.lat.begin(), r.lat.end());
    ok += r.ok;
    other += r.other;
    err += r.errors;
    sent += r.sent;
  }
  std::sort(lat.begin(), lat.end());
  auto pct = [&](double q) { return lat.empty() ? 0.0 : lat[std::min(lat.size() - 1, (size_t)(q * lat.size()))] / 1e6; };
  printf("{\"offered_rps\": %.0f, \"sent\": %lld, \"accepted\": %lld, \"accepted_rps\": %.1f, \"non_202\": %lld, "
         "\"errors\": %lld, \"p50_ms\": %.3f, \"p99_ms\": %.3f, \"p999_ms\": %.3f, \"wall_s\": %.2f}\n",
         rate, (long long)sent, (long long)ok, ok / secs, (long long)other, (long long)err, pct(0.5), pct(0.99),
         pct(0.999), wall);
  return 0;
}
