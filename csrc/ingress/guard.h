// Request guard: authentication (API key / JWT HS256), RBAC authorisation and
// token-bucket rate limiting (global, per client IP, per user).
//
// The reference documents these but never implements them:
//   * docs/configuration.md:732-775  security.authentication: jwt | api_key
//     (X-API-Key header, valid_keys; JWT secret / HS256 / issuer / expiry);
//   * docs/configuration.md:777-805  security.authorization: rbac roles ->
//     permissions ("*", "message:read", "message:write", "conversation:read"),
//     default_role;
//   * docs/configuration.md:503-537  loadbalancer.rate_limiting: global /
//     per_ip / per_user {requests_per_second, burst_size}.
// One native implementation serves both front ends: the C++ epoll ingress
// checks every POST /api/v1/messages inline (no GIL, sharded locks), and the
// Python API server calls the same object from its middleware.
//
// Pure C++17 + libcrypto (HMAC-SHA256, constant-time compare); no Python
// here, so the sanitizer stress (csrc/tests) links it directly.
#pragma once

#include <openssl/crypto.h>
#include <openssl/evp.h>
#include <openssl/hmac.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <ctime>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace llmq {

inline int64_t guard_mono_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// ------------------------------------------------------------------ rate limiting
// Token bucket: capacity `burst`, refilled at `rps` tokens/s.  Keyed buckets
// live in 64 mutex-sharded maps; a bucket that has been full for longer than
// `idle_ns` is dropped on the next sweep of its shard (bounded memory under
// many distinct client IPs).
class RateLimiter {
 public:
  RateLimiter(double rps = 0, double burst = 0, int64_t idle_ns = 60'000'000'000LL)
      : rps_(rps), burst_(burst > 0 ? burst : std::max(1.0, rps)), idle_ns_(idle_ns) {}

  bool enabled() const { return rps_ > 0; }

  // true = admitted.  `retry_after_s` (if given) = seconds until one token.
  bool allow(const std::string& key, int64_t now_ns, double* retry_after_s = nullptr) {
    if (!enabled()) return true;
    Shard& sh = shards_[std::hash<std::string>{}(key) & (kShards - 1)];
    std::lock_guard<std::mutex> g(sh.mu);
    if (++sh.ops % 4096 == 0) sweep(sh, now_ns);
    auto it = sh.b.find(key);
    if (it == sh.b.end()) it = sh.b.emplace(key, Bucket{burst_, now_ns}).first;
    Bucket& b = it->second;
    const double dt = (double)(now_ns - b.last_ns) * 1e-9;
    if (dt > 0) {
      b.tokens = std::min(burst_, b.tokens + dt * rps_);
      b.last_ns = now_ns;
    }
    if (b.tokens >= 1.0) {
      b.tokens -= 1.0;
      return true;
    }
    if (retry_after_s) *retry_after_s = (1.0 - b.tokens) / rps_;
    return false;
  }

  // Give back a token taken by allow() for a request a later check refused.
  void refund(const std::string& key) {
    if (!enabled()) return;
    Shard& sh = shards_[std::hash<std::string>{}(key) & (kShards - 1)];
    std::lock_guard<std::mutex> g(sh.mu);
    auto it = sh.b.find(key);
    if (it != sh.b.end()) it->second.tokens = std::min(burst_, it->second.tokens + 1.0);
  }

  size_t keys() {
    size_t n = 0;
    for (auto& sh : shards_) {
      std::lock_guard<std::mutex> g(sh.mu);
      n += sh.b.size();
    }
    return n;
  }

 private:
  struct Bucket {
    double tokens;
    int64_t last_ns;
  };
  struct Shard {
    std::mutex mu;
    std::unordered_map<std::string, Bucket> b;
    uint64_t ops = 0;
  };
  void sweep(Shard& sh, int64_t now) {
    for (auto it = sh.b.begin(); it != sh.b.end();) {
      const double full_at = (double)it->second.last_ns + (burst_ - it->second.tokens) / rps_ * 1e9;
      if ((double)now - full_at > (double)idle_ns_) it = sh.b.erase(it);
      else ++it;
    }
  }
  static constexpr size_t kShards = 64;
  double rps_, burst_;
  int64_t idle_ns_;
  Shard shards_[kShards];
};

// ------------------------------------------------------------------ base64url / JWT
inline bool b64url_decode(const char* s, size_t n, std::string* out) {
  static int8_t tab[256];
  static bool init = [] {
    memset(tab, -1, sizeof tab);
    const char* a = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_";
    for (int i = 0; i < 64; ++i) tab[(uint8_t)a[i]] = (int8_t)i;
    return true;
  }();
  (void)init;
  out->clear();
  uint32_t acc = 0;
  int bits = 0;
  for (size_t i = 0; i < n; ++i) {
    if (s[i] == '=') break;
    const int v = tab[(uint8_t)s[i]];
    if (v < 0) return false;
    acc = (acc << 6) | (uint32_t)v;
    bits += 6;
    if (bits >= 8) {
      bits -= 8;
      out->push_back((char)((acc >> bits) & 0xFF));
    }
  }
  return true;
}

inline std::string b64url_encode(const uint8_t* p, size_t n) {
  const char* a = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_";
  std::string o;
  uint32_t acc = 0;
  int bits = 0;
  for (size_t i = 0; i < n; ++i) {
    acc = (acc << 8) | p[i];
    bits += 8;
    while (bits >= 6) {
      bits -= 6;
      o.push_back(a[(acc >> bits) & 63]);
    }
  }
  if (bits > 0) o.push_back(a[(acc << (6 - bits)) & 63]);
  return o;
}

// Minimal claim reader for a flat JSON object: string / number values of the
// top-level keys we need ("sub", "iss", "role", "exp", "nbf", "alg", "typ").
// Nested values are skipped.  Returns false on malformed JSON.
struct Claims {
  std::unordered_map<std::string, std::string> str;
  std::unordered_map<std::string, double> num;
};

inline bool parse_claims(const std::string& js, Claims* c) {
  const char* p = js.data();
  const char* e = p + js.size();
  auto ws = [&] { while (p < e && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p; };
  auto str = [&](std::string* o) -> bool {
    if (p >= e || *p != '"') return false;
    ++p;
    while (p < e && *p != '"') {
      if (*p == '\\') {
        if (++p >= e) return false;
        const char ch = *p;
        if (ch == 'u') {  // keep the escape verbatim (claims we compare are ASCII)
          if (e - p < 5) return false;
          if (o) o->append(p - 1, 6);
          p += 5;
          continue;
        }
        if (o) o->push_back(ch == 'n' ? '\n' : ch == 't' ? '\t' : ch == 'r' ? '\r' : ch == 'b' ? '\b' : ch == 'f' ? '\f' : ch);
        ++p;
        continue;
      }
      if (o) o->push_back(*p);
      ++p;
    }
    if (p >= e) return false;
    ++p;
    return true;
  };
  // skip any JSON value (strings, numbers, literals, nested containers)
  auto skip = [&]() -> bool {
    ws();
    if (p >= e) return false;
    if (*p == '"') return str(nullptr);
    if (*p == '{' || *p == '[') {
      int d = 0;
      while (p < e) {
        if (*p == '"') {
          if (!str(nullptr)) return false;
          continue;
        }
        if (*p == '{' || *p == '[') ++d;
        else if (*p == '}' || *p == ']') {
          if (--d == 0) {
            ++p;
            return true;
          }
        }
        ++p;
      }
      return false;
    }
    const char* s = p;
    while (p < e && *p != ',' && *p != '}' && *p != ']' && *p != ' ' && *p != '\n') ++p;
    return p > s;
  };
  ws();
  if (p >= e || *p != '{') return false;
  ++p;
  ws();
  if (p < e && *p == '}') return true;
  for (;;) {
    ws();
    std::string k;
    if (!str(&k)) return false;
    ws();
    if (p >= e || *p != ':') return false;
    ++p;
    ws();
    if (p < e && *p == '"') {
      std::string v;
      if (!str(&v)) return false;
      c->str[k] = v;
    } else if (p < e && (*p == '-' || (*p >= '0' && *p <= '9'))) {
      char* q = nullptr;
      const std::string tmp(p, std::min<size_t>(64, e - p));
      const double d = strtod(tmp.c_str(), &q);
      if (q == tmp.c_str()) return false;
      p += (q - tmp.c_str());
      c->num[k] = d;
    } else if (!skip()) {
      return false;
    }
    ws();
    if (p < e && *p == ',') {
      ++p;
      continue;
    }
    if (p < e && *p == '}') return true;
    return false;
  }
}

inline std::string hmac_sha256(const std::string& key, const char* msg, size_t n) {
  uint8_t mac[EVP_MAX_MD_SIZE];
  unsigned int ml = 0;
  HMAC(EVP_sha256(), key.data(), (int)key.size(), (const uint8_t*)msg, n, mac, &ml);
  return std::string((const char*)mac, ml);
}

// ------------------------------------------------------------------ guard
enum GuardCode : int { G_OK = 0, G_UNAUTHORIZED = 401, G_FORBIDDEN = 403, G_RATE_LIMITED = 429 };

struct GuardResult {
  int code = G_OK;
  std::string subject;     // authenticated user (JWT "sub" / API key owner), may be empty
  std::string role;
  std::string reason;
  double retry_after_s = 0;
};

class Guard {
 public:
  // method: "none" | "api_key" | "jwt"
  Guard(std::string method, std::string api_key_header, std::vector<std::string> api_keys,
        std::string jwt_secret, std::string jwt_issuer, int64_t jwt_leeway_s, bool rbac,
        std::unordered_map<std::string, std::vector<std::string>> roles, std::string default_role,
        double global_rps, double global_burst, double ip_rps, double ip_burst, double user_rps,
        double user_burst, double idle_s = 60.0)
      : method_(std::move(method)),
        key_header_(lower(api_key_header.empty() ? std::string("X-API-Key") : api_key_header)),
        secret_(std::move(jwt_secret)),
        issuer_(std::move(jwt_issuer)),
        leeway_s_(jwt_leeway_s),
        rbac_(rbac),
        default_role_(std::move(default_role)),
        global_(global_rps, global_burst),
        per_ip_(ip_rps, ip_burst, (int64_t)(idle_s * 1e9)),
        per_user_(user_rps, user_burst, (int64_t)(idle_s * 1e9)) {
    for (auto& k : api_keys) {
      // "key" or "key:user" or "key:user:role"
      const size_t a = k.find(':');
      KeyInfo ki;
      std::string key = a == std::string::npos ? k : k.substr(0, a);
      if (a != std::string::npos) {
        const size_t b = k.find(':', a + 1);
        ki.user = k.substr(a + 1, b == std::string::npos ? std::string::npos : b - a - 1);
        if (b != std::string::npos) ki.role = k.substr(b + 1);
      }
      keys_.emplace_back(std::move(key), std::move(ki));
    }
    for (auto& kv : roles) roles_[kv.first] = std::unordered_set<std::string>(kv.second.begin(), kv.second.end());
    if (method_ != "none" && method_ != "api_key" && method_ != "jwt")
      throw std::invalid_argument("security.authentication.method must be none, api_key or jwt");
    if (method_ == "jwt" && secret_.empty()) throw std::invalid_argument("jwt authentication needs a secret");
  }

  const std::string& key_header() const { return key_header_; }
  bool auth_enabled() const { return method_ != "none"; }
  bool any() const { return auth_enabled() || rbac_ || global_.enabled() || per_ip_.enabled() || per_user_.enabled(); }

  // Permission a route needs ("" = public).
  static std::string permission_for(const std::string& method, const std::string& path) {
    if (path == "/health" || path == "/api/v1/health" || path == "/metrics") return "";
    const bool read = method == "GET" || method == "HEAD";
    auto starts = [&](const char* p) { return path.compare(0, strlen(p), p) == 0; };
    if (starts("/api/v1/admin") || starts("/api/v1/config")) return "admin:write";
    if (starts("/api/v1/messages")) return read ? "message:read" : "message:write";
    if (starts("/api/v1/conversations") || starts("/api/v1/users")) return read ? "conversation:read" : "conversation:write";
    if (starts("/api/v1/queues") || starts("/api/v1/metrics")) return "queue:read";
    if (starts("/api/v1/resources") || starts("/api/v1/endpoints")) return read ? "resource:read" : "resource:write";
    return read ? "api:read" : "api:write";
  }

  bool role_allows(const std::string& role, const std::string& perm) const {
    if (perm.empty() || !rbac_) return true;
    auto it = roles_.find(role);
    if (it == roles_.end()) return false;
    const auto& ps = it->second;
    if (ps.count("*") || ps.count(perm)) return true;
    const size_t c = perm.find(':');
    return c != std::string::npos && ps.count(perm.substr(0, c) + ":*");
  }

  // Authenticate + authorise + rate-limit one request.  `api_key` is the
  // value of key_header(), `authorization` the Authorization header,
  // `user_hint` the request's user id when the body names one (ignored for
  // rate limiting since r2: only an authenticated subject keys the per-user
  // limits fall back to it when the caller is anonymous).
  GuardResult check(const std::string& method, const std::string& path, const std::string& ip,
                    const std::string& api_key, const std::string& authorization, const std::string& user_hint,
                    int64_t now_ns = 0, int64_t wall_s = 0) {
    GuardResult r;
    if (now_ns == 0) now_ns = guard_mono_ns();
    if (wall_s == 0) wall_s = (int64_t)time(nullptr);
    const std::string perm = permission_for(method, path);
    r.role = default_role_;
    if (perm.empty()) return r;          // /health, /metrics: public and never throttled (probes, scrapes)
    {
      if (method_ == "api_key") {
        const KeyInfo* ki = match_key(api_key);
        if (!ki) return fail(r, G_UNAUTHORIZED, "missing or invalid API key");
        r.subject = ki->user;
        if (!ki->role.empty()) r.role = ki->role;
      } else if (method_ == "jwt") {
        std::string why;
        if (!verify_jwt(authorization, wall_s, &r, &why)) return fail(r, G_UNAUTHORIZED, why);
      }
      if (!role_allows(r.role, perm)) return fail(r, G_FORBIDDEN, "role '" + r.role + "' lacks " + perm);
    }
    // A refused request drains NO bucket: buckets are taken most specific
    // first, and a token already taken is refunded when a later bucket
    // refuses (a client held back by the per-user or global limit keeps its
    // per-IP budget; one abusive client cannot exhaust the global bucket
    // through requests its own limit refuses).  The per-user bucket is keyed
    // on the AUTHENTICATED subject only; an anonymous caller is limited by
    // its address (per-IP bucket) -- a body's user_id is a claim anyone can
    // make, so keying on it would let a client spend another user's quota.
    (void)user_hint;
    double ra = 0;
    const bool by_ip = !ip.empty(), by_user = !r.subject.empty();
    if (by_ip && !per_ip_.allow(ip, now_ns, &ra)) return limited(r, "per_ip", ra);
    if (by_user && !per_user_.allow(r.subject, now_ns, &ra)) {
      if (by_ip) per_ip_.refund(ip);
      return limited(r, "per_user", ra);
    }
    if (!global_.allow("*", now_ns, &ra)) {
      if (by_ip) per_ip_.refund(ip);
      if (by_user) per_user_.refund(r.subject);
      return limited(r, "global", ra);
    }
    return r;
  }

  // Per-user limit alone (front ends that learn the user id after the body
  // is parsed call this once they know it).
  bool allow_user(const std::string& user, double* retry_after_s = nullptr) {
    return user.empty() || per_user_.allow(user, guard_mono_ns(), retry_after_s);
  }

  bool verify_jwt(const std::string& authorization, int64_t wall_s, GuardResult* r, std::string* why) const {
    std::string tok = authorization;
    if (tok.size() > 7 && (tok.compare(0, 7, "Bearer ") == 0 || tok.compare(0, 7, "bearer ") == 0)) tok = tok.substr(7);
    else {
      *why = "missing bearer token";
      return false;
    }
    const size_t d1 = tok.find('.');
    const size_t d2 = d1 == std::string::npos ? d1 : tok.find('.', d1 + 1);
    if (d2 == std::string::npos || tok.find('.', d2 + 1) != std::string::npos) {
      *why = "malformed token";
      return false;
    }
    std::string hdr, pay, sig;
    if (!b64url_decode(tok.data(), d1, &hdr) || !b64url_decode(tok.data() + d1 + 1, d2 - d1 - 1, &pay) ||
        !b64url_decode(tok.data() + d2 + 1, tok.size() - d2 - 1, &sig)) {
      *why = "malformed token";
      return false;
    }
    Claims h, c;
    if (!parse_claims(hdr, &h) || !parse_claims(pay, &c)) {
      *why = "malformed token";
      return false;
    }
    if (h.str["alg"] != "HS256") {   // never "none", never an asymmetric alg with the HMAC secret
      *why = "unsupported alg";
      return false;
    }
    const std::string mac = hmac_sha256(secret_, tok.data(), d2);
    if (sig.size() != mac.size() || CRYPTO_memcmp(sig.data(), mac.data(), mac.size()) != 0) {
      *why = "bad signature";
      return false;
    }
    auto ex = c.num.find("exp");
    if (ex != c.num.end() && (double)wall_s > ex->second + (double)leeway_s_) {
      *why = "token expired";
      return false;
    }
    auto nb = c.num.find("nbf");
    if (nb != c.num.end() && (double)wall_s + (double)leeway_s_ < nb->second) {
      *why = "token not yet valid";
      return false;
    }
    if (!issuer_.empty() && c.str["iss"] != issuer_) {
      *why = "wrong issuer";
      return false;
    }
    r->subject = c.str["sub"];
    auto ro = c.str.find("role");
    if (ro != c.str.end() && !ro->second.empty()) r->role = ro->second;
    return true;
  }

  std::string sign_jwt(const std::string& payload_json) const {
    const std::string h = "{\"alg\":\"HS256\",\"typ\":\"JWT\"}";
    std::string t = b64url_encode((const uint8_t*)h.data(), h.size()) + "." +
                    b64url_encode((const uint8_t*)payload_json.data(), payload_json.size());
    const std::string mac = hmac_sha256(secret_, t.data(), t.size());
    return t + "." + b64url_encode((const uint8_t*)mac.data(), mac.size());
  }

  size_t tracked_keys() { return global_.keys() + per_ip_.keys() + per_user_.keys(); }

 private:
  struct KeyInfo {
    std::string user, role;
  };
  const KeyInfo* match_key(const std::string& k) const {
    const KeyInfo* hit = nullptr;
    for (auto& kv : keys_)   // constant-time per candidate, no early exit on a match
      if (kv.first.size() == k.size() && CRYPTO_memcmp(kv.first.data(), k.data(), k.size()) == 0) hit = &kv.second;
    return k.empty() ? nullptr : hit;
  }
  static GuardResult& fail(GuardResult& r, int code, std::string why) {
    r.code = code;
    r.reason = std::move(why);
    return r;
  }
  static GuardResult& limited(GuardResult& r, const char* which, double ra) {
    r.code = G_RATE_LIMITED;
    r.reason = std::string("rate limit exceeded (") + which + ")";
    r.retry_after_s = ra;
    return r;
  }
  static std::string lower(std::string s) {
    for (auto& c : s) c = (char)tolower((unsigned char)c);
    return s;
  }

  std::string method_, key_header_, secret_, issuer_;
  int64_t leeway_s_;
  bool rbac_;
  std::string default_role_;
  std::vector<std::pair<std::string, KeyInfo>> keys_;
  std::unordered_map<std::string, std::unordered_set<std::string>> roles_;
  RateLimiter global_, per_ip_, per_user_;
};

}  // namespace llmq
