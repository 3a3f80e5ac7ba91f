// Host (CPU) twin of text_analyze_kernel (csrc/kernels/text_kernels.h) for
// gateways without a GPU: the same tokenize/hash + keyword scoring +
// sentiment/question analysis with the exact Go semantics of the reference's
// preprocessor (`internal/preprocessor/preprocessor.go:56-114, 117-168,
// 204-248`; spelled out in preprocess/oracle.py), one message at a time.
//
// The GPU kernel evaluates every byte position of a 64-byte chunk in a lane
// and reduces with ballots; here one loop walks the positions in order and
// applies the same per-position predicates (rune start, Unicode space, word
// start, pattern hit, fold-special byte), so both produce identical stats
// rows and token hashes (tests/test_text_cpu.py checks this against the oracle,
// tests/test_gpu_kernels.py the kernel).  Output layout = the kernel's:
// stats [B][16] (words, pos, neg, question, flags, ntok, best slot, code,
// scores[8]) and hashes [B][L].
#pragma once

#include <cstdint>
#include <cstring>

namespace llmq {
namespace textcpu {

constexpr int MAX_PAT = 32;
constexpr int SLOTS = 8;
constexpr int STAT_COLS = 16;
constexpr int MAX_TOKEN_BYTES = 32;
enum : int32_t { FLAG_FOLD = 1 };

// byte layout of PatternTable in text_kernels.h (ops/text.py:pack_patterns)
struct PatternTable {
  uint32_t text[MAX_PAT][4];
  uint32_t mask[MAX_PAT][4];
  int32_t len[MAX_PAT];
  int32_t slot[MAX_PAT];
  int32_t flags[MAX_PAT];  // bit0 case-insensitive, bit1 self-overlapping
  int32_t npat;
};

inline bool is_cont(uint32_t c) { return (c & 0xC0u) == 0x80u; }

inline int utf8_width(uint32_t c, uint32_t b1, uint32_t b2, uint32_t b3) {
  if (c < 0x80u || c < 0xC2u) return 1;
  if (c < 0xE0u) return is_cont(b1) ? 2 : 1;
  if (c < 0xF0u) {
    const uint32_t lo = (c == 0xE0u) ? 0xA0u : 0x80u, hi = (c == 0xEDu) ? 0x9Fu : 0xBFu;
    return (b1 >= lo && b1 <= hi && is_cont(b2)) ? 3 : 1;
  }
  if (c < 0xF5u) {
    const uint32_t lo = (c == 0xF0u) ? 0x90u : 0x80u, hi = (c == 0xF4u) ? 0x8Fu : 0xBFu;
    return (b1 >= lo && b1 <= hi && is_cont(b2) && is_cont(b3)) ? 4 : 1;
  }
  return 1;
}

// width of the unicode.IsSpace rune starting at c (0: not a space)
inline int space_width(uint32_t c, uint32_t b1, uint32_t b2) {
  if (c == 0x20u || (c >= 0x09u && c <= 0x0Du)) return 1;
  if (c == 0xC2u) return (b1 == 0x85u || b1 == 0xA0u) ? 2 : 0;
  if (c == 0xE1u) return (b1 == 0x9Au && b2 == 0x80u) ? 3 : 0;
  if (c == 0xE2u) {
    if (b1 == 0x80u) return ((b2 >= 0x80u && b2 <= 0x8Au) || b2 == 0xA8u || b2 == 0xA9u || b2 == 0xAFu) ? 3 : 0;
    if (b1 == 0x81u) return b2 == 0x9Fu ? 3 : 0;
    return 0;
  }
  if (c == 0xE3u) return (b1 == 0x80u && b2 == 0x80u) ? 3 : 0;
  return 0;
}

inline uint32_t lower_ascii(uint32_t c) { return (c >= 0x41u && c <= 0x5Au) ? (c | 0x20u) : c; }

struct Analyzer {
  const PatternTable& pt;
  int L;
  uint32_t first[256];            // patterns whose first byte matches raw byte b (case-folded for (?i))
  uint8_t pat[MAX_PAT][16];

  Analyzer(const PatternTable& t, int l) : pt(t), L(l) {
    std::memset(first, 0, sizeof(first));
    for (int j = 0; j < pt.npat; ++j) {
      std::memcpy(pat[j], pt.text[j], 16);        // pattern bytes (already lowered if case-insensitive)
      for (int b = 0; b < 256; ++b)
        if (((pt.flags[j] & 1) ? lower_ascii((uint32_t)b) : (uint32_t)b) == pat[j][0]) first[b] |= 1u << j;
    }
  }

  void analyze(const uint8_t* s, int len, int32_t* st, uint32_t* hashes) const {
    static const char* kPos[5] = {"good", "great", "excellent", "happy", "satisfied"};
    static const int kPosLen[5] = {4, 5, 9, 5, 9};
    static const char* kNeg[5] = {"bad", "terrible", "awful", "angry", "frustrated"};
    static const int kNegLen[5] = {3, 8, 5, 5, 10};
    static const char* kQ[6] = {"what ", "how ", "why ", "when ", "where ", "who "};
    static const int kQLen[6] = {5, 4, 4, 5, 6, 4};
    int words = 0, pos = 0, neg = 0, ntok = 0;
    bool question = false, fold = false;
    int score[SLOTS] = {0, 0, 0, 0, 0, 0, 0, 0};
    int next_ok[MAX_PAT];
    for (int j = 0; j < MAX_PAT; ++j) next_ok[j] = 0;
    auto at = [&](int i) -> uint32_t { return (i >= 0 && i < len) ? s[i] : 0u; };
    // one pass: the width of the Unicode space starting at every byte (0: none)
    uint8_t sw_stack[1024];
    uint8_t* swb = len + 3 <= (int)sizeof(sw_stack) ? sw_stack : new uint8_t[len + 3];
    uint8_t* sw = swb + 3;                           // sw[-3..-1] = 0
    swb[0] = swb[1] = swb[2] = 0;
    for (int i = 0; i < len; ++i) {
      const uint32_t c = s[i];
      sw[i] = (uint8_t)(c < 0x80u ? (c == 0x20u || (c >= 0x09u && c <= 0x0Du)) : space_width(c, at(i + 1), at(i + 2)));
    }
    auto lowered_eq = [&](int p, const char* word, int n) -> bool {
      for (int i = 0; i < n; ++i)
        if (lower_ascii(s[p + i]) != (uint8_t)word[i]) return false;
      return true;
    };
    for (int p = 0; p < len; ++p) {
      const uint32_t c0 = s[p];
      bool rune_start = !is_cont(c0);
      if (!rune_start) {                             // covered by a valid sequence starting 1..3 bytes back?
        const uint32_t c1 = at(p + 1), c2 = at(p + 2), m1 = at(p - 1), m2 = at(p - 2), m3 = at(p - 3);
        if (!is_cont(m1)) rune_start = !(utf8_width(m1, c0, c1, c2) > 1);
        else if (!is_cont(m2)) rune_start = !(utf8_width(m2, m1, c0, c1) > 2);
        else if (!is_cont(m3)) rune_start = !(utf8_width(m3, m2, m1, c0) > 3);
        else rune_start = true;
      }
      const bool in_space = sw[p] > 0 || sw[p - 1] >= 2 || sw[p - 2] == 3;
      const bool prev_space = (p == 0) || sw[p - 1] > 0 || sw[p - 2] >= 2 || sw[p - 3] == 3;
      const bool wstart = rune_start && !in_space && prev_space;
      if (c0 >= 0xC4u) {
        const uint32_t c1 = at(p + 1);
        fold |= (c0 == 0xC5u && c1 == 0xBFu) || (c0 == 0xC4u && c1 == 0xB0u) ||
                (c0 == 0xE2u && c1 == 0x84u && at(p + 2) == 0xAAu);
      }
      const uint32_t l0 = lower_ascii(c0);
      if (!question) {
        question = (p == len - 1 && c0 == 0x3Fu);
        if (l0 == 'w' || l0 == 'h')                   // every question word starts with w or h
          for (int k = 0; k < 6 && !question; ++k)
            question = p + kQLen[k] <= len && lowered_eq(p, kQ[k], kQLen[k]);
      }
      if (wstart) {
        for (int k = 0; k < 5; ++k) {
          const int np = kPosLen[k], nn = kNegLen[k];
          if (p + np <= len && lowered_eq(p, kPos[k], np) && (p + np >= len || sw[p + np] > 0)) ++pos;
          if (p + nn <= len && lowered_eq(p, kNeg[k], nn) && (p + nn >= len || sw[p + nn] > 0)) ++neg;
        }
      }
      for (uint32_t cand = first[c0]; cand; cand &= cand - 1) {
        const int j = __builtin_ctz(cand);
        const int plen = pt.len[j];
        const bool ci = pt.flags[j] & 1;
        if (p + plen > len) continue;
        bool hit = true;
        for (int i = 1; i < plen && hit; ++i) hit = (ci ? lower_ascii(s[p + i]) : (uint32_t)s[p + i]) == pat[j][i];
        if (!hit) continue;
        if (pt.flags[j] & 2) {                       // bordered: greedy leftmost non-overlapping
          if (p < next_ok[j]) continue;
          next_ok[j] = p + plen;
        }
        ++score[pt.slot[j] & (SLOTS - 1)];
      }
      if (wstart) {
        if (ntok < L) {
          uint32_t h = 0x811C9DC5u;
          for (int n = 0, q = p; n < MAX_TOKEN_BYTES && q < len; ++n, ++q) {
            if (n > 0 && sw[q] > 0) break;
            h ^= lower_ascii(s[q]);
            h *= 0x01000193u;
          }
          hashes[ntok] = h;
          ++ntok;
        }
        ++words;
      }
    }
    if (swb != sw_stack) delete[] swb;
    st[0] = words;
    st[1] = pos;
    st[2] = neg;
    st[3] = question ? 1 : 0;
    st[4] = fold ? FLAG_FOLD : 0;
    st[5] = ntok;
    int best_slot = -1, best = 0;
    for (int k = 0; k < SLOTS; ++k) {
      st[8 + k] = score[k];
      if (score[k] > best) { best = score[k]; best_slot = k; }
    }
    st[6] = best_slot;
    st[7] = (pos > neg ? 1 : (neg > pos ? 2 : 0)) | (question ? 4 : 0) | (fold ? 8 : 0);
  }
};

}  // namespace textcpu
}  // namespace llmq
