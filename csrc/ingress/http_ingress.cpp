// Native HTTP ingress for the hot path: POST /api/v1/messages.
//
// The reference serves every route from one Gin process (api/handlers.go:75-
// 118) and documents a > 10,000 messages/s target (docs/performance.md:9).
// A Python ASGI stack tops out at ~1-2k requests/s per process, so the
// submit route gets a native front end: N epoll threads (SO_REUSEPORT, one
// listener each), HTTP/1.1 keep-alive + pipelining, a single-pass scan of the
// JSON body (validation + top-level "id"/"priority"/"user_id" extraction; the
// body itself is forwarded verbatim), a UUIDv4 when the client gave no id,
// and a push into the process-shared request ring (shm_ring.h) as a RAW
// record.  The GPU dispatcher drains the ring in large batches, so
// preprocessing (text_analyze + MFMA classifier) sees big batches too.
// Other routes (status, conversations, admin) stay on the Python API server;
// with an upstream set (``set_upstream``, the multi-GPU `cli serve` front
// door) they are reverse-proxied to it, so one public port serves the whole
// REST surface.  Messages with a conversation_id can be routed to a separate
// ring (``set_conv_ring``) drained by the process that owns conversation
// state; the rest go to the shared ring every GPU rank drains.
//
// Response: 202 {"message_id", "priority", "queue_time", "estimated_wait"}
// where priority is the requested one (0 = to be decided by the
// preprocessor, which runs asynchronously after the ack); 400 on a malformed
// body, 503 when the ring is full (back-pressure).  With a Guard attached
// (guard.h) every request is authenticated (API key / JWT), authorised
// (RBAC) and rate-limited (global / per IP / per user) inline: 401 / 403 /
// 429 + Retry-After.  ``envelope`` wraps bodies in the documented
// {"code","message","data","timestamp"} format (docs/api.md:12-20).
#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <ctime>
#include <memory>
#include <random>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "ingress/guard.h"
#include "queue/shm_ring.h"

namespace py = pybind11;

namespace {

constexpr uint32_t TAG_RAW = 3;   // [u64 arrival_mono_ns][36 B uuid][u32 body_len][body]
constexpr size_t kMaxBody = 4u << 20;   // POST body cap (413 beyond; the read buffer caps at 8 MiB)
constexpr size_t kMaxHeader = 64u << 10; // request line + headers cap (431 beyond)

// ------------------------------------------------------------------ JSON scan
struct Scan {
  bool ok = false;
  bool has_conv = false;   // a non-empty conversation_id (routed to the conversation owner's ring)
  std::string id, user_id;
  int priority = 0;
  std::string error;   // why the body was refused (400 text)
};

struct JsonScanner {
  const char* p;
  const char* e;
  int depth = 0;
  void ws() {
    while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p;
  }
  static int hexv(char c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
  }
  bool hex4(unsigned* cp) {
    if (e - p < 4) return false;
    unsigned v = 0;
    for (int k = 0; k < 4; ++k) {
      const int h = hexv(p[k]);
      if (h < 0) return false;
      v = v * 16 + (unsigned)h;
    }
    p += 4;
    *cp = v;
    return true;
  }
  static void put_utf8(std::string* out, unsigned cp) {
    if (!out) return;
    if (cp < 0x80) {
      out->push_back((char)cp);
    } else if (cp < 0x800) {
      out->push_back((char)(0xC0 | (cp >> 6)));
      out->push_back((char)(0x80 | (cp & 0x3F)));
    } else if (cp < 0x10000) {
      out->push_back((char)(0xE0 | (cp >> 12)));
      out->push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
      out->push_back((char)(0x80 | (cp & 0x3F)));
    } else {
      out->push_back((char)(0xF0 | (cp >> 18)));
      out->push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
      out->push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
      out->push_back((char)(0x80 | (cp & 0x3F)));
    }
  }
  // one well-formed UTF-8 sequence (what Python's strict utf-8 decoder
  // accepts: no overlongs, no encoded surrogates, <= U+10FFFF)
  bool utf8(std::string* out) {
    const unsigned char c = (unsigned char)*p;
    int n;
    unsigned cp;
    if (c < 0x80) { n = 0; cp = c; }
    else if (c >= 0xC2 && c <= 0xDF) { n = 1; cp = c & 0x1F; }
    else if (c >= 0xE0 && c <= 0xEF) { n = 2; cp = c & 0x0F; }
    else if (c >= 0xF0 && c <= 0xF4) { n = 3; cp = c & 0x07; }
    else return false;
    if (e - p < n + 1) return false;
    for (int k = 1; k <= n; ++k) {
      const unsigned char d = (unsigned char)p[k];
      if ((d & 0xC0) != 0x80) return false;
      cp = (cp << 6) | (d & 0x3F);
    }
    if ((n == 2 && cp < 0x800) || (n == 3 && (cp < 0x10000 || cp > 0x10FFFF)) || (cp >= 0xD800 && cp <= 0xDFFF))
      return false;
    if (out) out->append(p, (size_t)n + 1);
    p += n + 1;
    return true;
  }
  // RFC 8259 string: valid escapes only (\uXXXX decoded, surrogate pairs
  // joined; a lone surrogate is kept as Python keeps it, but callers that
  // need a printable id reject it), well-formed UTF-8, no raw controls
  bool str(std::string* out) {
    if (p >= e || *p != '"') return false;
    ++p;
    while (p < e && *p != '"') {
      if (*p == '\\') {
        if (p + 1 >= e) return false;
        const char c = p[1];
        p += 2;
        switch (c) {
          case '"': if (out) out->push_back('"'); break;
          case '\\': if (out) out->push_back('\\'); break;
          case '/': if (out) out->push_back('/'); break;
          case 'b': if (out) out->push_back('\b'); break;
          case 'f': if (out) out->push_back('\f'); break;
          case 'n': if (out) out->push_back('\n'); break;
          case 'r': if (out) out->push_back('\r'); break;
          case 't': if (out) out->push_back('\t'); break;
          case 'u': {
            unsigned cp;
            if (!hex4(&cp)) return false;
            if (cp >= 0xD800 && cp <= 0xDBFF && e - p >= 6 && p[0] == '\\' && p[1] == 'u') {
              const char* save = p;
              p += 2;
              unsigned lo;
              if (!hex4(&lo)) return false;
              if (lo >= 0xDC00 && lo <= 0xDFFF) cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
              else p = save;
            }
            if (cp >= 0xD800 && cp <= 0xDFFF) lone_surrogate = true;
            put_utf8(out, cp);
            break;
          }
          default: return false;
        }
        continue;
      }
      if ((unsigned char)*p < 0x20) return false;
      if (!utf8(out)) return false;
    }
    if (p >= e) return false;
    ++p;
    return true;
  }
  // RFC 8259 number: -?(0|[1-9][0-9]*)(.[0-9]+)?([eE][+-]?[0-9]+)?
  bool num(double* out) {
    const char* s = p;
    if (p < e && *p == '-') ++p;
    if (p >= e) return false;
    if (*p == '0') {
      ++p;
    } else if (*p >= '1' && *p <= '9') {
      while (p < e && *p >= '0' && *p <= '9') ++p;
    } else {
      return false;
    }
    bool is_int = true;
    if (p < e && *p == '.') {
      ++p;
      is_int = false;
      if (p >= e || *p < '0' || *p > '9') return false;
      while (p < e && *p >= '0' && *p <= '9') ++p;
    }
    if (p < e && (*p == 'e' || *p == 'E')) {
      ++p;
      is_int = false;
      if (p < e && (*p == '+' || *p == '-')) ++p;
      if (p >= e || *p < '0' || *p > '9') return false;
      while (p < e && *p >= '0' && *p <= '9') ++p;
    }
    last_is_int = is_int;
    if (out) *out = strtod(std::string(s, p - s).c_str(), nullptr);
    return true;
  }
  bool last_is_int = true;
  bool lone_surrogate = false;
  bool lit(const char* w) {
    size_t n = strlen(w);
    if ((size_t)(e - p) < n || memcmp(p, w, n) != 0) return false;
    p += n;
    return true;
  }
  bool value() {  // skip any value
    ws();
    if (p >= e) return false;
    if (*p == '"') return str(nullptr);
    if (*p == '{' || *p == '[') {
      if (++depth > 64) return false;
      const char close = *p == '{' ? '}' : ']';
      const bool obj = *p == '{';
      ++p;
      ws();
      if (p < e && *p == close) {
        ++p;
        --depth;
        return true;
      }
      for (;;) {
        ws();
        if (obj) {
          if (!str(nullptr)) return false;
          ws();
          if (p >= e || *p != ':') return false;
          ++p;
        }
        if (!value()) return false;
        ws();
        if (p < e && *p == ',') {
          ++p;
          continue;
        }
        if (p < e && *p == close) {
          ++p;
          --depth;
          return true;
        }
        return false;
      }
    }
    if (*p == 't') return lit("true");
    if (*p == 'f') return lit("false");
    if (*p == 'n') return lit("null");
    return num(nullptr);
  }
};

// The same rule as models/message.py:parse_priority (the Python front door and
// the rank's decode): ASCII-trimmed, case-insensitive level name ("urgent" is
// realtime, "medium" normal) or a decimal integer 0..4; anything else -> -1.
int priority_from_string(const std::string& s) {
  size_t a = 0, b = s.size();
  auto ws = [](char c) { return c == ' ' || (c >= '\t' && c <= '\r'); };
  while (a < b && ws(s[a])) ++a;
  while (b > a && ws(s[b - 1])) --b;
  std::string l;
  for (size_t i = a; i < b; ++i) l.push_back((char)tolower((unsigned char)s[i]));
  if (l == "realtime" || l == "urgent") return 1;
  if (l == "high") return 2;
  if (l == "normal" || l == "medium") return 3;
  if (l == "low") return 4;
  const bool neg = !l.empty() && l[0] == '-';
  size_t i = (!l.empty() && (l[0] == '+' || neg)) ? 1 : 0;
  if (i == l.size()) return -1;
  int v = 0;
  for (; i < l.size(); ++i) {
    if (l[i] < '0' || l[i] > '9') return -1;
    v = v * 10 + (l[i] - '0');
    if (v > 4) return -1;
  }
  return (neg && v != 0) ? -1 : v;                   // "-0" is 0
}

// Go duration text as utils/duration.parse_duration_ns accepts it:
// [+-]? ( [0-9]*\.?[0-9]+ (ns|us|µs|μs|ms|s|m|h) )+  , or "" / "0"
bool go_duration(const std::string& raw) {
  size_t a = 0, b = raw.size();
  while (a < b && isspace((unsigned char)raw[a])) ++a;
  while (b > a && isspace((unsigned char)raw[b - 1])) --b;
  std::string s = raw.substr(a, b - a);
  if (s.empty() || s == "0") return true;
  size_t i = 0;
  if (s[i] == '+' || s[i] == '-') ++i;
  if (i >= s.size()) return false;
  while (i < s.size()) {
    const size_t d0 = i;
    while (i < s.size() && isdigit((unsigned char)s[i])) ++i;
    if (i < s.size() && s[i] == '.') {
      ++i;
      const size_t f0 = i;
      while (i < s.size() && isdigit((unsigned char)s[i])) ++i;
      if (i == f0) return false;
    } else if (i == d0) {
      return false;
    }
    static const char* units[] = {"ns", "us", "\xC2\xB5s", "\xCE\xBCs", "ms", "s", "m", "h"};
    bool hit = false;
    for (const char* u : units) {
      const size_t L = strlen(u);
      if (s.compare(i, L, u) == 0) {
        i += L;
        hit = true;
        break;
      }
    }
    if (!hit) return false;
  }
  return true;
}

// RFC 3339 timestamp as models.message.parse_time reads it back
// (YYYY-MM-DDTHH:MM:SS[.frac](Z|+HH:MM|-HH:MM), real calendar dates)
bool rfc3339(const std::string& s) {
  auto dig = [&](size_t i, size_t n) {
    if (i + n > s.size()) return false;
    for (size_t k = i; k < i + n; ++k)
      if (!isdigit((unsigned char)s[k])) return false;
    return true;
  };
  auto num = [&](size_t i, size_t n) { return atoi(s.substr(i, n).c_str()); };
  if (s.size() < 20 || !dig(0, 4) || s[4] != '-' || !dig(5, 2) || s[7] != '-' || !dig(8, 2) || s[10] != 'T' ||
      !dig(11, 2) || s[13] != ':' || !dig(14, 2) || s[16] != ':' || !dig(17, 2))
    return false;
  const int y = num(0, 4), mo = num(5, 2), d = num(8, 2);
  static const int mdays[12] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
  const bool leap = (y % 4 == 0 && y % 100 != 0) || y % 400 == 0;
  if (y < 1 || mo < 1 || mo > 12 || d < 1 || d > mdays[mo - 1] + (mo == 2 && leap ? 1 : 0)) return false;
  if (num(11, 2) > 23 || num(14, 2) > 59 || num(17, 2) > 59) return false;
  size_t i = 19;
  if (i < s.size() && s[i] == '.') {
    ++i;
    const size_t f0 = i;
    while (i < s.size() && isdigit((unsigned char)s[i])) ++i;
    if (i == f0) return false;
  }
  if (i < s.size() && s[i] == 'Z') return i + 1 == s.size();
  return i + 6 == s.size() && (s[i] == '+' || s[i] == '-') && dig(i + 1, 2) && s[i + 3] == ':' && dig(i + 4, 2) &&
         num(i + 1, 2) <= 23 && num(i + 4, 2) <= 59;
}

// id / user_id travel into the 202 JSON and the ring record unescaped:
// printable ASCII without quote or backslash only
bool plain_token(const std::string& s) {
  for (unsigned char c : s)
    if (c < 0x20 || c > 0x7E || c == '"' || c == '\\') return false;
  return true;
}

Scan scan_message(const char* b, size_t n) {
  Scan r;
  r.error = "Invalid message format";
  JsonScanner js{b, b + n};
  js.ws();
  if (js.p >= js.e || *js.p != '{') return r;
  ++js.p;
  js.ws();
  if (js.p < js.e && *js.p == '}') {
    ++js.p;
    js.ws();
    r.ok = js.p == js.e;                             // nothing may follow the object, as below
    if (r.ok) r.error.clear();
    return r;
  }
  for (;;) {
    js.ws();
    std::string key;
    if (!js.str(&key)) return r;
    js.ws();
    if (js.p >= js.e || *js.p != ':') return r;
    ++js.p;
    js.ws();
    const char c0 = js.p < js.e ? *js.p : 0;
    if (key == "id" || key == "user_id") {
      std::string v;
      if (c0 == '"') {
        js.lone_surrogate = false;                    // (set by an earlier field's escapes)
        if (!js.str(&v)) return r;
        if (js.lone_surrogate || !plain_token(v)) {
          r.error = key + " must be printable ASCII without quotes or backslashes";
          return r;
        }
        (key == "id" ? r.id : r.user_id) = v;
      } else if (c0 == 'n') {
        if (!js.lit("null")) return r;
      } else {
        r.error = key + " must be a string";
        return r;
      }
    } else if (key == "priority") {
      if (c0 == '"') {
        std::string v;
        if (!js.str(&v)) return r;
        r.priority = priority_from_string(v);
        if (r.priority < 0) {                          // unknown priority name -> 400
          r.error = "invalid priority";
          return r;
        }
      } else if (c0 == 'n') {
        if (!js.lit("null")) return r;
      } else {
        double d = 0;
        if (!js.num(&d) || !(d >= 0 && d <= 4) || d != (double)(int)d) {   // range first: no out-of-range cast
          r.error = "invalid priority";
          return r;
        }
        r.priority = (int)d;
      }
    } else if (key == "conversation_id") {             // Message.from_dict: str(v or "")
      const char* v0 = js.p;
      if (!js.value()) return r;
      const std::string raw(v0, js.p - v0);
      r.has_conv = !(raw == "null" || raw == "false" || raw == "\"\"" || raw == "0" || raw == "[]" ||
                     raw == "{}" || raw == "0.0" || raw == "-0");
    } else if (key == "metadata") {                    // Message.from_dict: object (or null)
      if (c0 != '{' && c0 != 'n') {
        r.error = "metadata must be an object";
        return r;
      }
      if (!js.value()) return r;
    } else if (key == "timeout" || key == "max_retries" || key == "retry_count") {
      // numbers (finite, int64 range) or null; timeout also a Go duration string
      if (c0 == 'n') {
        if (!js.lit("null")) return r;
      } else if (c0 == '"' && key == "timeout") {
        std::string v;
        if (!js.str(&v) || !go_duration(v)) {
          r.error = "invalid timeout";
          return r;
        }
      } else {
        double d = 0;
        if (!js.num(&d) || !(d > -9.2e18 && d < 9.2e18)) {
          r.error = "invalid " + key;
          return r;
        }
      }
    } else if (key == "created_at" || key == "updated_at" || key == "scheduled_at" || key == "completed_at") {
      if (c0 == 'n') {
        if (!js.lit("null")) return r;
      } else if (c0 == '"') {
        std::string v;
        if (!js.str(&v) || !(v.empty() || rfc3339(v))) {
          r.error = "invalid " + key;
          return r;
        }
      } else {
        double d = 0;
        if (!js.num(&d) || !(d > -9.2e18 && d < 9.2e18)) {
          r.error = "invalid " + key;
          return r;
        }
      }
    } else if (!js.value()) {
      return r;
    }
    js.ws();
    if (js.p < js.e && *js.p == ',') {
      ++js.p;
      continue;
    }
    if (js.p < js.e && *js.p == '}') {
      ++js.p;
      js.ws();
      r.ok = js.p == js.e;
      if (r.ok) r.error.clear();
      return r;
    }
    return r;
  }
}

// ------------------------------------------------------------------ HTTP
struct Conn {
  std::string in, out, ip;
  size_t out_off = 0;
  bool close_after = false;
  bool continued = false;   // "100 Continue" already sent for the pending request
  bool out_armed = false;   // EPOLLOUT registered (a write hit EAGAIN)
  bool proxying = false;    // a request is with the API server: later (pipelined) ones wait in `in`
  uint64_t gen = 0;         // accept generation (a proxy answer for a reused fd is dropped)
  int fd = -1;
  int64_t last_ns = 0;      // last byte received (idle / slow-client reaping)
};

// Per epoll thread: proxy answers handed back by the proxy workers.  All
// socket writes stay on the epoll thread; the workers only do the blocking
// upstream round trip.
struct ProxyDone {
  int fd;
  uint64_t gen;
  std::string resp;
  bool close;
};
struct LoopCtx {
  int efd = -1;                  // eventfd: "answers waiting"
  std::mutex mu;
  std::vector<ProxyDone> done;
  uint64_t next_gen = 0;
};
struct ProxyTask {
  LoopCtx* lp;
  int fd;
  uint64_t gen;
  std::string req;
  bool keep;
};

int64_t mono_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

std::string rfc3339_now() {
  auto now = std::chrono::system_clock::now();
  auto ns = std::chrono::duration_cast<std::chrono::nanoseconds>(now.time_since_epoch()).count();
  time_t s = (time_t)(ns / 1000000000);
  struct tm tmv;
  gmtime_r(&s, &tmv);
  char buf[64];
  size_t k = strftime(buf, sizeof buf, "%Y-%m-%dT%H:%M:%S", &tmv);
  snprintf(buf + k, sizeof buf - k, ".%09lldZ", (long long)(ns % 1000000000));
  return buf;
}

class HttpIngress {
 public:
  HttpIngress(int port, const std::string& ring, int threads, const std::string& host)
      : port_(port), host_(host), ring_(ring, 1 << 26, "open"), nthreads_(threads > 0 ? threads : 4) {}
  ~HttpIngress() { stop(); }

  int start() {
    if (running_.exchange(true)) return port_;
    {
      std::lock_guard<std::mutex> g(pq_mu_);
      pq_stop_ = false;
    }
    for (int i = 0; i < kProxyWorkers; ++i) pw_.emplace_back([this] { proxy_worker(); });
    for (int i = 0; i < nthreads_; ++i) {
      ctx_.push_back(std::make_unique<LoopCtx>());
      ctx_.back()->efd = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    }
    for (int i = 0; i < nthreads_; ++i) {
      int fd = listen_socket();
      if (fd < 0) {
        stop();
        throw std::runtime_error("ingress: cannot listen on port " + std::to_string(port_) + ": " + strerror(errno));
      }
      if (port_ == 0) {  // ephemeral: reuse the port the first listener got
        sockaddr_in a{};
        socklen_t al = sizeof a;
        getsockname(fd, (sockaddr*)&a, &al);
        port_ = ntohs(a.sin_port);
      }
      lfds_.push_back(fd);
      LoopCtx* lp = ctx_[i].get();
      th_.emplace_back([this, fd, i, lp] { loop(fd, i, lp); });
    }
    return port_;
  }

  void stop() {
    if (!running_.exchange(false)) return;
    for (auto& t : th_)
      if (t.joinable()) t.join();
    th_.clear();
    {
      std::lock_guard<std::mutex> g(pq_mu_);
      pq_stop_ = true;
      pq_.clear();
    }
    pq_cv_.notify_all();
    for (auto& t : pw_)
      if (t.joinable()) t.join();
    pw_.clear();
    for (auto& c : ctx_)
      if (c->efd >= 0) ::close(c->efd);
    ctx_.clear();
    for (int fd : lfds_) ::close(fd);
    lfds_.clear();
  }

  py::dict stats() const {
    py::dict d;
    d["accepted"] = accepted_.load();
    d["rejected_full"] = rejected_full_.load();
    d["bad_request"] = bad_.load();
    d["requests"] = requests_.load();
    d["connections"] = conns_.load();
    d["port"] = port_;
    d["unauthorized"] = unauth_.load();
    d["forbidden"] = forbidden_.load();
    d["rate_limited"] = limited_.load();
    d["refused_no_fd"] = refused_fd_.load();
    d["idle_closed"] = idle_closed_.load();
    d["proxied"] = proxied_.load();
    d["proxy_errors"] = proxy_errors_.load();
    return d;
  }

  void set_guard(std::shared_ptr<llmq::Guard> g) { guard_ = std::move(g); }
  // Messages that carry a conversation_id go to this ring instead (the
  // process that owns conversation state drains it); others to the shared one.
  void set_conv_ring(const std::string& name) {
    conv_ring_ = name.empty() ? nullptr : std::make_unique<llmq::ShmRing>(name, 1 << 26, "open");
  }
  // Every route but the hot submit path (and /health) is forwarded to the
  // API server at host:port -- one public port for the whole REST surface.
  void set_upstream(const std::string& host, int port) {
    upstream_host_ = host;
    upstream_port_ = port;
  }
  void set_envelope(bool on) { envelope_ = on; }
  // `cli api-gateway --native`: the submit reply also carries the reference
  // api-gateway's fields ({"message": "Message accepted", "id"},
  // cmd/api-gateway/main.go:113), so clients of either binary read it
  void set_gateway_compat(bool on) { gateway_compat_ = on; }

  // Health of the process behind the door (the serve loop's stall
  // watchdog): while unhealthy, GET /health answers 503 with the reason, so
  // probes replace a stalled rank instead of seeing it alive.
  void set_health(bool ok, const std::string& reason) {
    std::string r;
    for (char c : reason) {                // the reason travels inside a JSON string
      if (c == '"' || c == '\\') r += '\\';
      if ((unsigned char)c >= 0x20) r += c;
    }
    {
      std::lock_guard<std::mutex> g(health_mu_);
      health_reason_ = r;
    }
    healthy_.store(ok, std::memory_order_release);
  }
  void set_idle_timeout(double seconds) { idle_ns_.store(seconds > 0 ? (int64_t)(seconds * 1e9) : 0); }

 private:
  int listen_socket() {
    int fd = socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK, 0);
    if (fd < 0) return -1;
    int one = 1;
    setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    setsockopt(fd, SOL_SOCKET, SO_REUSEPORT, &one, sizeof one);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons(port_);
    inet_pton(AF_INET, host_.c_str(), &a.sin_addr);
    if (bind(fd, (sockaddr*)&a, sizeof a) < 0 || listen(fd, SOMAXCONN) < 0) {
      ::close(fd);
      return -1;
    }
    return fd;
  }

  void loop(int lfd, int tid, LoopCtx* lp) {
    int ep = epoll_create1(0);
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.fd = lfd;
    epoll_ctl(ep, EPOLL_CTL_ADD, lfd, &ev);
    epoll_event eev{};
    eev.events = EPOLLIN;
    eev.data.fd = lp->efd;
    epoll_ctl(ep, EPOLL_CTL_ADD, lp->efd, &eev);
    std::unordered_map<int, Conn> conns;
    std::mt19937_64 rng((uint64_t)mono_ns() ^ ((uint64_t)tid << 40) ^ (uint64_t)(uintptr_t)this);
    std::vector<epoll_event> evs(256);
    char buf[65536];
    // out of descriptors: accept + close with this spare so the pending
    // connection is refused instead of the level-triggered listener spinning
    int spare = ::open("/dev/null", O_RDONLY | O_CLOEXEC);
    int64_t next_sweep = mono_ns() + 1'000'000'000;
    while (running_.load()) {
      int n = epoll_wait(ep, evs.data(), (int)evs.size(), 100);
      const int64_t idle = idle_ns_.load(std::memory_order_relaxed);
      if (idle > 0 && mono_ns() >= next_sweep) {
        // reap connections silent for longer than the idle timeout: idle
        // keep-alives and slow / stalled senders (slowloris) alike
        const int64_t now = mono_ns();
        next_sweep = now + std::min<int64_t>(idle / 4 + 1, 1'000'000'000);
        for (auto it = conns.begin(); it != conns.end();) {
          if (now - it->second.last_ns > idle && it->second.out_off >= it->second.out.size() &&
              !it->second.proxying) {
            epoll_ctl(ep, EPOLL_CTL_DEL, it->first, nullptr);
            ::close(it->first);
            it = conns.erase(it);
            conns_--;
            idle_closed_++;
          } else {
            ++it;
          }
        }
      }
      for (int k = 0; k < n; ++k) {
        int fd = evs[k].data.fd;
        if (fd == lp->efd) {                         // proxy answers are back
          uint64_t cnt;
          while (::read(lp->efd, &cnt, sizeof cnt) > 0) {
          }
          std::vector<ProxyDone> done;
          {
            std::lock_guard<std::mutex> g(lp->mu);
            done.swap(lp->done);
          }
          for (auto& d : done) {
            auto it = conns.find(d.fd);
            if (it == conns.end() || it->second.gen != d.gen) continue;   // closed meanwhile
            Conn& cn = it->second;
            cn.proxying = false;
            cn.out.append(d.resp);
            if (d.close) cn.close_after = true;
            if (!cn.close_after) process(cn, rng, lp);  // requests pipelined behind it
            bool dead = !cn.out.empty() && !flush(d.fd, cn, ep);
            if (dead || (cn.close_after && cn.out.empty() && !cn.proxying)) {
              epoll_ctl(ep, EPOLL_CTL_DEL, d.fd, nullptr);
              ::close(d.fd);
              conns.erase(it);
              conns_--;
            }
          }
          continue;
        }
        if (fd == lfd) {
          for (;;) {
            sockaddr_in pa{};
            socklen_t pl = sizeof pa;
            int c = accept4(lfd, (sockaddr*)&pa, &pl, SOCK_NONBLOCK);
            if (c < 0) {
              if ((errno == EMFILE || errno == ENFILE) && spare >= 0) {
                ::close(spare);
                // (accept reports EMFILE before it looks at the backlog)
                int d = accept4(lfd, nullptr, nullptr, 0);
                if (d >= 0) ::close(d);
                spare = ::open("/dev/null", O_RDONLY | O_CLOEXEC);
                if (d < 0) break;                    // backlog drained
                refused_fd_++;
                continue;
              }
              break;
            }
            int one = 1;
            setsockopt(c, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
            epoll_event ce{};
            ce.events = EPOLLIN | EPOLLRDHUP;
            ce.data.fd = c;
            epoll_ctl(ep, EPOLL_CTL_ADD, c, &ce);
            char ipb[INET_ADDRSTRLEN] = {0};
            inet_ntop(AF_INET, &pa.sin_addr, ipb, sizeof ipb);
            conns[c] = Conn();
            conns[c].ip = ipb;
            conns[c].last_ns = mono_ns();
            conns[c].gen = ++lp->next_gen;
            conns[c].fd = c;
            conns_++;
          }
          continue;
        }
        auto it = conns.find(fd);
        if (it == conns.end()) continue;
        Conn& cn = it->second;
        bool dead = (evs[k].events & (EPOLLERR | EPOLLHUP)) != 0, eof = false;
        if (evs[k].events & EPOLLIN) {
          for (;;) {
            ssize_t r = ::read(fd, buf, sizeof buf);
            if (r > 0) {
              cn.last_ns = mono_ns();
              cn.in.append(buf, (size_t)r);
              if (cn.in.size() > (8u << 20)) dead = true;
              continue;
            }
            if (r == 0) eof = true;   // peer half-closed: answer what it sent, then close
            break;
          }
          if (!dead && !cn.proxying) process(cn, rng, lp);
          if (eof) cn.close_after = true;
        }
        if (!dead && !cn.out.empty()) dead = !flush(fd, cn, ep);
        if (!dead && cn.out.empty() && cn.out_armed) {
          // drained: back to read interest only (level-triggered EPOLLOUT on
          // an idle writable socket would wake this thread forever)
          epoll_event ce{};
          ce.events = EPOLLIN | EPOLLRDHUP;
          ce.data.fd = fd;
          epoll_ctl(ep, EPOLL_CTL_MOD, fd, &ce);
          cn.out_armed = false;
        }
        if (dead || (cn.close_after && cn.out.empty() && !cn.proxying)) {
          epoll_ctl(ep, EPOLL_CTL_DEL, fd, nullptr);
          ::close(fd);
          conns.erase(it);
          conns_--;
        }
      }
    }
    for (auto& kv : conns) ::close(kv.first);
    if (spare >= 0) ::close(spare);
    ::close(ep);
  }

  bool flush(int fd, Conn& cn, int ep) {
    while (cn.out_off < cn.out.size()) {
      ssize_t w = ::write(fd, cn.out.data() + cn.out_off, cn.out.size() - cn.out_off);
      if (w > 0) {
        cn.out_off += (size_t)w;
        continue;
      }
      if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
        if (!cn.out_armed) {
          epoll_event ce{};
          ce.events = EPOLLIN | EPOLLOUT | EPOLLRDHUP;
          ce.data.fd = fd;
          epoll_ctl(ep, EPOLL_CTL_MOD, fd, &ce);
          cn.out_armed = true;
        }
        return true;
      }
      return false;
    }
    cn.out.clear();
    cn.out_off = 0;
    return true;
  }

  void respond(Conn& cn, int code, const char* reason, const std::string& raw, bool keep,
               const std::string& extra_hdr = "") {
    std::string body;
    if (envelope_) {
      // error bodies are {"error": "..."}: lift the text into "message"
      const bool err = code >= 400;
      std::string msg = "success";
      if (err) {
        const size_t a = raw.find(":\"");
        const size_t b = raw.rfind('"');
        msg = (a != std::string::npos && b > a + 2) ? raw.substr(a + 2, b - a - 2) : reason;
      }
      body = "{\"code\":" + std::to_string(code) + ",\"message\":\"" + msg + "\"," +
             (err ? "\"error\":\"" + msg + "\"" : "\"data\":" + raw) + ",\"timestamp\":\"" + rfc3339_now() + "\"}";
    }
    const std::string& b = envelope_ ? body : raw;
    char hdr[256];
    int n = snprintf(hdr, sizeof hdr,
                     "HTTP/1.1 %d %s\r\nContent-Type: application/json\r\nContent-Length: %zu\r\n%s", code,
                     reason, b.size(), keep ? "" : "Connection: close\r\n");
    cn.out.append(hdr, (size_t)n);
    cn.out.append(extra_hdr);
    cn.out.append("\r\n");
    cn.out.append(b);
    if (!keep) cn.close_after = true;
  }

  // 401 / 403 / 429 for a guard verdict; returns true when the request may proceed
  bool admit(Conn& cn, const std::string& method, const std::string& path, const std::string& key,
             const std::string& auth, const std::string& user, bool keep) {
    if (!guard_) return true;
    llmq::GuardResult g = guard_->check(method, path, cn.ip, key, auth, user);
    if (g.code == llmq::G_OK) return true;
    std::string why;
    for (char c : g.reason) why.push_back(c == '"' || c == '\\' ? '\'' : c);
    if (g.code == llmq::G_UNAUTHORIZED) {
      unauth_++;
      respond(cn, 401, "Unauthorized", "{\"error\":\"" + why + "\"}", keep,
              "WWW-Authenticate: " + std::string(guard_->key_header() == "authorization" ? "Bearer" : "Bearer, ApiKey") + "\r\n");
    } else if (g.code == llmq::G_FORBIDDEN) {
      forbidden_++;
      respond(cn, 403, "Forbidden", "{\"error\":\"" + why + "\"}", keep);
    } else {
      limited_++;
      const int ra = std::max(1, (int)std::ceil(g.retry_after_s));
      respond(cn, 429, "Too Many Requests", "{\"error\":\"" + why + "\"}", keep,
              "Retry-After: " + std::to_string(ra) + "\r\n");
    }
    return false;
  }

  static std::string uuid4(std::mt19937_64& rng) {
    uint64_t a = rng(), b = rng();
    a = (a & 0xFFFFFFFFFFFF0FFFull) | 0x0000000000004000ull;
    b = (b & 0x3FFFFFFFFFFFFFFFull) | 0x8000000000000000ull;
    char s[40];
    snprintf(s, sizeof s, "%08x-%04x-%04x-%04x-%012llx", (unsigned)(a >> 32), (unsigned)((a >> 16) & 0xFFFF),
             (unsigned)(a & 0xFFFF), (unsigned)(b >> 48), (unsigned long long)(b & 0xFFFFFFFFFFFFull));
    return s;
  }

  void process(Conn& cn, std::mt19937_64& rng, LoopCtx* lp) {
    size_t pos = 0;
    while (!cn.close_after && !cn.proxying) {
      size_t he = cn.in.find("\r\n\r\n", pos);
      if (he == std::string::npos) {
        if (cn.in.size() - pos > kMaxHeader)
          respond(cn, 431, "Request Header Fields Too Large", "{\"error\":\"header too large\"}", false);
        break;
      }
      const char* h = cn.in.data() + pos;
      size_t hl = he - pos;
      // request line
      const char* sp1 = (const char*)memchr(h, ' ', hl);
      if (!sp1) {
        respond(cn, 400, "Bad Request", "{\"error\":\"bad request line\"}", false);
        break;
      }
      const char* sp2 = (const char*)memchr(sp1 + 1, ' ', hl - (sp1 + 1 - h));
      if (!sp2) {
        respond(cn, 400, "Bad Request", "{\"error\":\"bad request line\"}", false);
        break;
      }
      std::string method(h, sp1 - h), path(sp1 + 1, sp2 - sp1 - 1);
      bool http10 = std::string(sp2 + 1, std::min<size_t>(8, hl - (sp2 + 1 - h))) == "HTTP/1.0";
      size_t clen = 0;
      bool keep = !http10, bad_len = false, chunked = false, expect100 = false;
      std::string api_key, authz;
      // headers (case-insensitive names)
      const char* line = (const char*)memchr(h, '\n', hl);
      while (line && line < h + hl) {
        ++line;
        const char* eol = (const char*)memchr(line, '\n', h + hl - line);
        const char* le = eol ? eol : h + hl;
        const char* colon = (const char*)memchr(line, ':', le - line);
        if (colon) {
          std::string name(line, colon - line);
          for (auto& c : name) c = (char)tolower((unsigned char)c);
          const char* v = colon + 1;
          while (v < le && (*v == ' ' || *v == '\t')) ++v;
          std::string val(v, le - v);
          while (!val.empty() && (val.back() == '\r' || val.back() == ' ')) val.pop_back();
          if (name == "content-length") {
            // digits only, bounded before any arithmetic on it (an unchecked
            // 2^64-1 would wrap the body-complete test below)
            bad_len = val.empty() || val.size() > 12 ||
                      val.find_first_not_of("0123456789") != std::string::npos;
            clen = bad_len ? 0 : (size_t)strtoull(val.c_str(), nullptr, 10);
          } else if (name == "transfer-encoding") chunked = true;
          else if (name == "expect") {
            for (auto& c : val) c = (char)tolower((unsigned char)c);
            expect100 = val == "100-continue";
          }
          else if (name == "authorization") authz = val;
          else if (guard_ && name == guard_->key_header()) api_key = val;
          else if (name == "connection") {
            for (auto& c : val) c = (char)tolower((unsigned char)c);
            if (val == "close") keep = false;
            else if (val == "keep-alive") keep = true;
          }
        }
        line = eol;
      }
      if (bad_len || chunked || clen > kMaxBody) {
        bad_++;
        if (clen > kMaxBody)
          respond(cn, 413, "Payload Too Large", "{\"error\":\"body exceeds 4 MiB\"}", false);
        else if (chunked)
          respond(cn, 501, "Not Implemented", "{\"error\":\"chunked transfer encoding not supported\"}", false);
        else
          respond(cn, 400, "Bad Request", "{\"error\":\"bad Content-Length\"}", false);
        break;
      }
      if (cn.in.size() < he + 4 + clen) {  // body not complete yet
        // curl and friends hold a large body back until told to send it
        if (expect100 && !cn.continued) {
          cn.out.append("HTTP/1.1 100 Continue\r\n\r\n");
          cn.continued = true;
        }
        break;
      }
      cn.continued = false;
      const char* body = cn.in.data() + he + 4;
      requests_++;
      if (method == "POST" && (path == "/api/v1/messages" || path == "/api/v1/messages/")) {
        Scan s = scan_message(body, clen);
        if (!admit(cn, method, path, api_key, authz, s.ok ? s.user_id : std::string(), keep)) {
          // rejected by the guard (401 / 403 / 429)
        } else if (!s.ok) {
          bad_++;
          respond(cn, 400, "Bad Request", "{\"error\":\"" + s.error + "\"}", keep);
        } else {
          std::string id = s.id.empty() ? uuid4(rng) : s.id;
          std::string rec(8 + 36 + 4 + clen, '\0');
          const int64_t t = mono_ns();
          memcpy(&rec[0], &t, 8);
          memcpy(&rec[8], id.data(), std::min<size_t>(36, id.size()));
          const uint32_t bl = (uint32_t)clen;
          memcpy(&rec[44], &bl, 4);
          memcpy(&rec[48], body, clen);
          llmq::ShmRing& dst = (s.has_conv && conv_ring_) ? *conv_ring_ : ring_;
          if (id.size() > 36 || !dst.push(rec, TAG_RAW)) {
            if (id.size() > 36) {
              bad_++;
              respond(cn, 400, "Bad Request", "{\"error\":\"id longer than 36 bytes\"}", keep);
            } else {
              rejected_full_++;
              respond(cn, 503, "Service Unavailable", "{\"error\":\"Failed to queue message: queue full\"}", keep);
            }
          } else {
            accepted_++;
            std::string out = "{\"message_id\":\"" + id + "\",\"priority\":" + std::to_string(s.priority) +
                              ",\"queue_time\":\"" + rfc3339_now() + "\",\"estimated_wait\":0";
            if (gateway_compat_) out += ",\"message\":\"Message accepted\",\"id\":\"" + id + "\"";
            out += "}";
            respond(cn, 202, "Accepted", out, keep);
          }
        }
      } else if (method == "GET" && (path == "/health" || path == "/api/v1/health")) {
        if (healthy_.load(std::memory_order_acquire)) {
          respond(cn, 200, "OK", "{\"status\":\"ok\",\"version\":\"1.0.0\",\"time\":\"" + rfc3339_now() + "\"}", keep);
        } else {
          std::string why;
          {
            std::lock_guard<std::mutex> g(health_mu_);
            why = health_reason_;
          }
          respond(cn, 503, "Service Unavailable", "{\"status\":\"unhealthy\",\"reason\":\"" + why +
                  "\",\"version\":\"1.0.0\",\"time\":\"" + rfc3339_now() + "\"}", keep);
        }
      } else if (upstream_port_ > 0) {
        // handed to a proxy worker; the connection's later requests wait in
        // `in` until the answer is back (responses stay in request order)
        proxied_++;
        start_proxy(cn, lp, h, hl, body, clen, keep);
      } else {
        respond(cn, 404, "Not Found", "{\"error\":\"route served by the API server\"}", keep);
      }
      pos = he + 4 + clen;
    }
    if (pos) cn.in.erase(0, pos);
  }

  // Reverse proxy of one request to the API server (status, conversation
  // and admin routes).  The epoll thread only builds the upstream request and
  // queues it; one of kProxyWorkers threads does the blocking round trip
  // (Connection: close upstream) and hands the framed answer back through the
  // loop's eventfd -- a slow admin query never stalls the other connections of
  // that epoll thread, and every socket write stays on it.  The client's
  // keep-alive is kept when the answer is framed by Content-Length.
  void start_proxy(Conn& cn, LoopCtx* lp, const char* h, size_t hl, const char* body, size_t clen, bool keep) {
    std::string req;
    req.reserve(hl + clen + 128);
    const char* line_end = (const char*)memchr(h, '\n', hl);
    const char* cur = line_end ? line_end + 1 : h + hl;
    req.append(h, cur - h);                                      // request line (with its CRLF)
    while (cur < h + hl) {
      const char* eol = (const char*)memchr(cur, '\n', h + hl - cur);
      const char* le = eol ? eol + 1 : h + hl;
      const char* colon = (const char*)memchr(cur, ':', le - cur);
      std::string name = colon ? std::string(cur, colon - cur) : std::string();
      for (auto& c : name) c = (char)tolower((unsigned char)c);
      if (name != "connection" && name != "expect" && name != "keep-alive" && name != "x-forwarded-for") {
        req.append(cur, le - cur);
        if (req.back() != '\n') req.append("\r\n");
      }
      cur = le;
    }
    req.append("Connection: close\r\nX-Forwarded-For: " + cn.ip + "\r\n\r\n");
    req.append(body, clen);
    cn.proxying = true;
    {
      std::lock_guard<std::mutex> g(pq_mu_);
      pq_.push_back(ProxyTask{lp, cn.fd, cn.gen, std::move(req), keep});
    }
    pq_cv_.notify_one();
  }

  void proxy_worker() {
    for (;;) {
      ProxyTask t;
      {
        std::unique_lock<std::mutex> g(pq_mu_);
        pq_cv_.wait(g, [&] { return pq_stop_ || !pq_.empty(); });
        if (pq_stop_) return;
        t = std::move(pq_.front());
        pq_.pop_front();
      }
      bool close = false;
      std::string resp = proxy_fetch(t.req, t.keep, &close);
      {
        std::lock_guard<std::mutex> g(t.lp->mu);
        t.lp->done.push_back(ProxyDone{t.fd, t.gen, std::move(resp), close});
      }
      const uint64_t one = 1;
      if (::write(t.lp->efd, &one, sizeof one) < 0) {
      }
    }
  }

  // The upstream round trip; returns the bytes for the client (502 when the
  // API server is unreachable or answers garbage).
  std::string proxy_fetch(const std::string& req, bool keep, bool* close) {
    std::string resp;
    bool ok = false;
    int fd = socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
    if (fd >= 0) {
      timeval tv{30, 0};
      setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
      setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof tv);
      sockaddr_in a{};
      a.sin_family = AF_INET;
      a.sin_port = htons((uint16_t)upstream_port_);
      inet_pton(AF_INET, upstream_host_.c_str(), &a.sin_addr);
      if (connect(fd, (sockaddr*)&a, sizeof a) == 0) {
        size_t off = 0;
        while (off < req.size()) {
          ssize_t w = ::send(fd, req.data() + off, req.size() - off, MSG_NOSIGNAL);
          if (w <= 0) break;
          off += (size_t)w;
        }
        if (off == req.size()) {
          char b[65536];
          for (;;) {
            ssize_t r = ::recv(fd, b, sizeof b, 0);
            if (r <= 0) {
              ok = r == 0;
              break;
            }
            resp.append(b, (size_t)r);
            if (resp.size() > (64u << 20)) break;
          }
        }
      }
      ::close(fd);
    }
    const size_t he = resp.find("\r\n\r\n");
    if (!ok || he == std::string::npos || resp.compare(0, 5, "HTTP/") != 0) {
      proxy_errors_++;
      Conn tmp;
      respond(tmp, 502, "Bad Gateway", "{\"error\":\"API server unreachable\"}", keep);
      *close = tmp.close_after;
      return tmp.out;
    }
    // drop the upstream's Connection header; keep the client connection open
    // only when the body length is explicit
    std::string head;
    bool has_len = false, chunked = false;
    size_t p = 0;
    while (p < he) {
      size_t e = resp.find("\r\n", p);
      if (e == std::string::npos || e > he) e = he;
      std::string ln = resp.substr(p, e - p);
      std::string low = ln;
      for (auto& c : low) c = (char)tolower((unsigned char)c);
      if (low.compare(0, 15, "content-length:") == 0) has_len = true;
      if (low.compare(0, 18, "transfer-encoding:") == 0) chunked = true;
      if (p == 0 || low.compare(0, 11, "connection:") != 0) head += ln + "\r\n";
      p = e + 2;
    }
    const bool k = keep && has_len && !chunked;
    if (!k) head += "Connection: close\r\n";
    std::string out = head + "\r\n";
    out.append(resp, he + 4, std::string::npos);
    *close = !k;
    return out;
  }

  int port_;
  std::string host_;
  llmq::ShmRing ring_;
  std::unique_ptr<llmq::ShmRing> conv_ring_;
  std::string upstream_host_ = "127.0.0.1";
  int upstream_port_ = 0;
  std::atomic<int64_t> proxied_{0}, proxy_errors_{0};
  static constexpr int kProxyWorkers = 4;
  std::vector<std::unique_ptr<LoopCtx>> ctx_;
  std::vector<std::thread> pw_;
  std::mutex pq_mu_;
  std::condition_variable pq_cv_;
  std::deque<ProxyTask> pq_;
  bool pq_stop_ = false;
  int nthreads_;
  std::atomic<bool> running_{false};
  std::atomic<bool> healthy_{true};
  std::mutex health_mu_;
  std::string health_reason_;
  std::vector<std::thread> th_;
  std::vector<int> lfds_;
  std::atomic<int64_t> accepted_{0}, rejected_full_{0}, bad_{0}, requests_{0}, conns_{0};
  std::atomic<int64_t> unauth_{0}, forbidden_{0}, limited_{0}, refused_fd_{0}, idle_closed_{0};
  std::atomic<int64_t> idle_ns_{60'000'000'000};   // 60 s; 0 = never reap
  std::shared_ptr<llmq::Guard> guard_;
  bool envelope_ = false;
  bool gateway_compat_ = false;
};

}  // namespace

PYBIND11_MODULE(_ingress, m) {
  m.doc() = "native HTTP ingress for POST /api/v1/messages -> shared request ring";
  m.attr("TAG_RAW") = TAG_RAW;
  py::class_<HttpIngress>(m, "HttpIngress")
      .def(py::init<int, const std::string&, int, const std::string&>(), py::arg("port"), py::arg("ring"),
           py::arg("threads") = 4, py::arg("host") = "0.0.0.0")
      .def("start", &HttpIngress::start)
      .def("stop", &HttpIngress::stop, py::call_guard<py::gil_scoped_release>())
      .def("stats", &HttpIngress::stats)
      .def("set_guard", &HttpIngress::set_guard)
      .def("set_conv_ring", &HttpIngress::set_conv_ring, py::arg("name"))
      .def("set_upstream", &HttpIngress::set_upstream, py::arg("host"), py::arg("port"))
      .def("set_envelope", &HttpIngress::set_envelope)
      .def("set_gateway_compat", &HttpIngress::set_gateway_compat)
      .def("set_health", &HttpIngress::set_health, py::arg("ok"), py::arg("reason") = "")
      .def("set_idle_timeout", &HttpIngress::set_idle_timeout, py::arg("seconds"));
  py::class_<llmq::Guard, std::shared_ptr<llmq::Guard>>(m, "Guard")
      .def(py::init<std::string, std::string, std::vector<std::string>, std::string, std::string, int64_t, bool,
                    std::unordered_map<std::string, std::vector<std::string>>, std::string, double, double, double,
                    double, double, double, double>(),
           py::arg("method") = "none", py::arg("api_key_header") = "X-API-Key",
           py::arg("api_keys") = std::vector<std::string>{}, py::arg("jwt_secret") = "", py::arg("jwt_issuer") = "",
           py::arg("jwt_leeway_s") = 0, py::arg("rbac") = false,
           py::arg("roles") = std::unordered_map<std::string, std::vector<std::string>>{},
           py::arg("default_role") = "user", py::arg("global_rps") = 0.0, py::arg("global_burst") = 0.0,
           py::arg("ip_rps") = 0.0, py::arg("ip_burst") = 0.0, py::arg("user_rps") = 0.0, py::arg("user_burst") = 0.0,
           py::arg("idle_s") = 60.0)
      .def("check",
           [](llmq::Guard& g, const std::string& method, const std::string& path, const std::string& ip,
              const std::string& api_key, const std::string& authorization, const std::string& user,
              int64_t now_ns, int64_t wall_s) {
             llmq::GuardResult r;
             {
               py::gil_scoped_release nogil;
               r = g.check(method, path, ip, api_key, authorization, user, now_ns, wall_s);
             }
             return py::make_tuple(r.code, r.subject, r.role, r.reason, r.retry_after_s);
           },
           py::arg("method"), py::arg("path"), py::arg("ip") = "", py::arg("api_key") = "",
           py::arg("authorization") = "", py::arg("user") = "", py::arg("now_ns") = 0, py::arg("wall_s") = 0)
      .def("allow_user",
           [](llmq::Guard& g, const std::string& user) {
             double ra = 0;
             bool ok = g.allow_user(user, &ra);
             return py::make_tuple(ok, ra);
           })
      .def("sign_jwt", &llmq::Guard::sign_jwt)
      .def("role_allows", &llmq::Guard::role_allows)
      .def_property_readonly("key_header", &llmq::Guard::key_header)
      .def_property_readonly("auth_enabled", &llmq::Guard::auth_enabled)
      .def_property_readonly("active", &llmq::Guard::any)
      .def("tracked_keys", &llmq::Guard::tracked_keys)
      .def_static("permission_for", &llmq::Guard::permission_for);
  m.def("scan_message", [](py::bytes b) {
    std::string s = b;
    Scan r = scan_message(s.data(), s.size());
    return py::make_tuple(r.ok, r.id, r.priority, r.user_id, r.error, r.has_conv);
  });
}
