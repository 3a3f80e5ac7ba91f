// text_analyze: fused tokenize/hash + keyword scoring + sentiment/question
// (N1+N2+N3) for a micro-batch of UTF-8 messages.  gfx950, wave64.
//
// Replaces the reference's per-request CPU work in
// `internal/preprocessor/preprocessor.go`:
//   * strings.Fields / unicode.IsSpace word split            (:204, :257)
//   * regexp FindAllString keyword counting per priority      (:141-149)
//   * bag-of-words sentiment + question detection             (:211-248)
// with the exact Go semantics spelled out in preprocess/oracle.py.
//
// Layout: ONE WAVE PER MESSAGE, 4 waves (256 threads) per workgroup.  The wave
// walks its message in 64-byte chunks; lane l owns byte p = base + l.  Each
// chunk (plus a 4-byte look-behind and a 28-byte look-ahead halo) is staged
// once into a per-wave LDS window with coalesced byte loads; every per-lane
// test then reads a 16-byte window at p with 5 aligned ds_read_b32 +
// v_alignbyte (no unaligned LDS access).  Counts are wave-uniform: every
// predicate is reduced with one __ballot + popcount, so there are no atomics
// and a single lane writes the message's results.
//
// Exactness: bytes whose Go lower-casing / (?i) folding crosses into ASCII
// (U+017F, U+212A, U+0130) set FLAG_FOLD and the host re-scores that message
// with the oracle; everything else (including invalid UTF-8) is exact here.

#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace llmq {

constexpr int TA_MAX_PAT = 32;
constexpr int TA_SLOTS = 8;
constexpr int TA_STAT_COLS = 16;
constexpr int TA_MAX_TOKEN_BYTES = 32;   // classifier tokenizer hashes <= 32 bytes/token
constexpr int TA_WAVES = 4;
// staged bytes per wave per chunk: 4 look-behind + 64 + 36 look-ahead, so a
// token starting at the chunk's last byte (<= 32 bytes + the 2-byte space
// test after it) is hashed from LDS too
constexpr int TA_WIN = 104;

enum : int32_t { FLAG_FOLD = 1 };
enum : int32_t { ST_WORDS = 0, ST_POS = 1, ST_NEG = 2, ST_QUESTION = 3, ST_FLAGS = 4,
                 ST_NTOK = 5, ST_BEST_SLOT = 6, ST_CODE = 7, ST_SCORES = 8 };

struct PatternTable {
  uint32_t text[TA_MAX_PAT][4];  // pattern bytes (lower-cased if case-insensitive)
  uint32_t mask[TA_MAX_PAT][4];  // 0xFF per valid byte
  int32_t len[TA_MAX_PAT];
  int32_t slot[TA_MAX_PAT];      // score slot 0..7
  int32_t flags[TA_MAX_PAT];     // bit0: case-insensitive, bit1: self-overlapping (bordered)
  int32_t npat;
};

__device__ __forceinline__ uint32_t swar_lower(uint32_t w) {
  // ASCII 'A'..'Z' -> 'a'..'z' on 4 bytes at once; non-ASCII bytes untouched.
  const uint32_t h = w & 0x7F7F7F7Fu;
  const uint32_t ge_a = h + 0x3F3F3F3Fu;   // bit7 set iff byte >= 0x41
  const uint32_t gt_z = h + 0x25252525u;   // bit7 set iff byte >= 0x5B
  const uint32_t up = ge_a & ~gt_z & ~w & 0x80808080u;
  return w | (up >> 2);
}

__device__ __forceinline__ uint32_t byte_of(const uint32_t (&w)[4], int i) {
  return (w[i >> 2] >> ((i & 3) * 8)) & 0xFFu;
}

__device__ __forceinline__ bool is_cont(uint32_t c) { return (c & 0xC0u) == 0x80u; }

// Go utf8 decode width of a sequence starting with lead byte c (1 for
// invalid/truncated sequences, which decode as RuneError of width 1).
__device__ __forceinline__ int utf8_width(uint32_t c, uint32_t b1, uint32_t b2, uint32_t b3) {
  if (c < 0x80u) return 1;
  if (c < 0xC2u) return 1;
  if (c < 0xE0u) return is_cont(b1) ? 2 : 1;
  if (c < 0xF0u) {
    const uint32_t lo = (c == 0xE0u) ? 0xA0u : 0x80u;
    const uint32_t hi = (c == 0xEDu) ? 0x9Fu : 0xBFu;
    return (b1 >= lo && b1 <= hi && is_cont(b2)) ? 3 : 1;
  }
  if (c < 0xF5u) {
    const uint32_t lo = (c == 0xF0u) ? 0x90u : 0x80u;
    const uint32_t hi = (c == 0xF4u) ? 0x8Fu : 0xBFu;
    return (b1 >= lo && b1 <= hi && is_cont(b2) && is_cont(b3)) ? 4 : 1;
  }
  return 1;
}

// Width of the unicode.IsSpace rune starting at a byte (0 if not a space).
__device__ __forceinline__ int space_width(uint32_t c, uint32_t b1, uint32_t b2) {
  if (c == 0x20u || (c >= 0x09u && c <= 0x0Du)) return 1;
  if (c == 0xC2u) return (b1 == 0x85u || b1 == 0xA0u) ? 2 : 0;
  if (c == 0xE1u) return (b1 == 0x9Au && b2 == 0x80u) ? 3 : 0;
  if (c == 0xE2u) {
    if (b1 == 0x80u)
      return ((b2 >= 0x80u && b2 <= 0x8Au) || b2 == 0xA8u || b2 == 0xA9u || b2 == 0xAFu) ? 3 : 0;
    if (b1 == 0x81u) return b2 == 0x9Fu ? 3 : 0;
    return 0;
  }
  if (c == 0xE3u) return (b1 == 0x80u && b2 == 0x80u) ? 3 : 0;
  return 0;
}

__device__ __forceinline__ uint64_t wave_ballot(bool p) { return __ballot(p); }

__device__ __forceinline__ int lanes_below(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Sentiment / question vocabulary (lower-case ASCII, <= 12 bytes), packed
// little-endian at compile time.
struct Word { uint32_t w0, w1, w2; int len; };
constexpr Word mkword(const char* s) {
  Word w{0u, 0u, 0u, 0};
  int n = 0;
  while (s[n]) {
    const uint32_t b = (uint32_t)(uint8_t)s[n];
    if (n < 4) w.w0 |= b << (8 * n);
    else if (n < 8) w.w1 |= b << (8 * (n - 4));
    else w.w2 |= b << (8 * (n - 8));
    ++n;
  }
  w.len = n;
  return w;
}
__device__ __constant__ Word kPosWords[5] = {mkword("good"), mkword("great"), mkword("excellent"),
                                             mkword("happy"), mkword("satisfied")};
__device__ __constant__ Word kNegWords[5] = {mkword("bad"), mkword("terrible"), mkword("awful"),
                                             mkword("angry"), mkword("frustrated")};
// question keywords followed by a space (substring test, preprocessor.go:239)
__device__ __constant__ Word kQWords[6] = {mkword("what "), mkword("how "), mkword("why "),
                                           mkword("when "), mkword("where "), mkword("who ")};

__device__ __forceinline__ bool word_prefix_eq(const uint32_t (&wl)[4], const Word& w) {
  const int L = w.len;
  const uint32_t m0 = L >= 4 ? 0xFFFFFFFFu : ((1u << (8 * L)) - 1u);
  const uint32_t m1 = L >= 8 ? 0xFFFFFFFFu : (L > 4 ? ((1u << (8 * (L - 4))) - 1u) : 0u);
  const uint32_t m2 = L >= 12 ? 0xFFFFFFFFu : (L > 8 ? ((1u << (8 * (L - 8))) - 1u) : 0u);
  return ((wl[0] & m0) == w.w0) && ((wl[1] & m1) == w.w1) && ((wl[2] & m2) == w.w2);
}

__global__ void __launch_bounds__(256)
text_analyze_kernel(const uint8_t* __restrict__ bytes, const int64_t* __restrict__ offsets,
                    int B, int L, PatternTable pt, int32_t* __restrict__ stats,
                    uint32_t* __restrict__ hashes, float* __restrict__ zero_rows, int zero_len) {
  __shared__ uint32_t win32[TA_WAVES][TA_WIN / 4];
  __shared__ int32_t next_ok[TA_WAVES][TA_MAX_PAT];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int msg = blockIdx.x * TA_WAVES + wv;
  if (msg >= B) return;  // whole wave exits together (msg is wave-uniform)
  if (zero_rows) {       // the classifier's pooled row of this message (embed_pool accumulates into it)
    float4* z = reinterpret_cast<float4*>(zero_rows + (int64_t)msg * zero_len);
    for (int i = lane; i < zero_len / 4; i += 64) z[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  uint8_t* win8 = reinterpret_cast<uint8_t*>(win32[wv]);

  const int64_t start = offsets[msg];
  const int len = (int)(offsets[msg + 1] - start);
  const uint8_t* src = bytes + start;

  if (lane < TA_MAX_PAT) next_ok[wv][lane] = 0;

  int words = 0, pos = 0, neg = 0, ntok = 0;
  bool question = false, fold = false;
  int score[TA_SLOTS];
#pragma unroll
  for (int s = 0; s < TA_SLOTS; ++s) score[s] = 0;

  // Software-pipelined byte staging: the bytes of chunk base + 64 are loaded
  // (clamped addresses, no predicate) while chunk base is processed, so a
  // message costs one load round trip instead of one per 64-byte chunk (the
  // flat ~27 us at serving batch sizes, profiles/r5_preprocess_kernels_pmc.md)
  auto ldb = [&](int i) -> uint32_t { return src[min(max(i, 0), len - 1)]; };
  uint32_t b0 = 0u, b1 = 0u;
  if (len > 0) {
    b0 = ldb(lane - 4);
    b1 = ldb(lane + 60);
  }
  for (int base = 0; base < len; base += 64) {
    // ---- stage bytes [base-4, base+100) into this wave's LDS window
    {
      const int i0 = base - 4 + lane;
      win8[lane] = (i0 >= 0 && i0 < len) ? (uint8_t)b0 : (uint8_t)0;
      if (lane < TA_WIN - 64) {
        const int i1 = base + 60 + lane;
        win8[64 + lane] = (i1 < len) ? (uint8_t)b1 : (uint8_t)0;
      }
    }
    if (base + 64 < len) {          // wave-uniform: the next chunk's bytes, in flight during this one
      b0 = ldb(base + 60 + lane);
      b1 = ldb(base + 124 + lane);
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): staged bytes visible to all lanes
    __builtin_amdgcn_wave_barrier();

    const int p = base + lane;
    const bool valid = p < len;
    // 16-byte window at p (LDS byte offset lane+4) via aligned dword reads
    uint32_t w[4], wl[4];
    {
      const int o = lane + 4;
      const int a = o >> 2, sh = o & 3;
      uint32_t d[5];
#pragma unroll
      for (int i = 0; i < 5; ++i) d[i] = win32[wv][a + i];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        w[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], (uint32_t)sh);
        wl[i] = swar_lower(w[i]);
      }
    }
    const uint32_t c0 = byte_of(w, 0), c1 = byte_of(w, 1), c2 = byte_of(w, 2), c3 = byte_of(w, 3);
    const uint32_t m1 = win8[lane + 3], m2 = win8[lane + 2], m3 = win8[lane + 1];

    // ---- UTF-8 rune starts and whitespace
    bool rune_start = !is_cont(c0);
    if (!rune_start) {
      // covered by a valid sequence starting 1..3 bytes back?
      if (!is_cont(m1)) rune_start = !(utf8_width(m1, c0, c1, c2) > 1);
      else if (!is_cont(m2)) rune_start = !(utf8_width(m2, m1, c0, c1) > 2);
      else if (!is_cont(m3)) rune_start = !(utf8_width(m3, m2, m1, c0) > 3);
      else rune_start = true;
    }
    const int sw0 = space_width(c0, c1, c2);
    const int swm1 = space_width(m1, c0, c1);
    const int swm2 = space_width(m2, m1, c0);
    const int swm3 = space_width(m3, m2, m1);
    const bool in_space = sw0 > 0 || swm1 >= 2 || swm2 == 3;
    const bool prev_space = (p == 0) || swm1 > 0 || swm2 >= 2 || swm3 == 3;
    const bool wstart = valid && rune_start && !in_space && prev_space;

    const uint64_t wmask = wave_ballot(wstart);
    const int tok_idx = ntok + lanes_below(wmask);
    words += __popcll(wmask);

    // ---- fold-special characters (oracle fallback)
    const bool special = valid && ((c0 == 0xC5u && c1 == 0xBFu) || (c0 == 0xC4u && c1 == 0xB0u) ||
                                   (c0 == 0xE2u && c1 == 0x84u && c2 == 0xAAu));
    fold |= wave_ballot(special) != 0ull;

    // ---- question: literal last byte '?', or "<kw> " anywhere in the lowered text
    bool q = valid && (p == len - 1) && c0 == 0x3Fu;
#pragma unroll
    for (int k = 0; k < 6; ++k) q |= valid && (p + kQWords[k].len <= len) && word_prefix_eq(wl, kQWords[k]);
    question |= wave_ballot(q) != 0ull;

    // ---- sentiment: whole token equal to a vocabulary word
    bool is_pos = false, is_neg = false;
    if (wstart) {
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        const int Lw = kPosWords[k].len;
        if (word_prefix_eq(wl, kPosWords[k])) {
          const int e = p + Lw;
          const bool ends = e >= len || space_width(byte_of(w, Lw), byte_of(w, Lw + 1), byte_of(w, Lw + 2)) > 0;
          is_pos |= ends;
        }
        const int Ln = kNegWords[k].len;
        if (word_prefix_eq(wl, kNegWords[k])) {
          const int e = p + Ln;
          const bool ends = e >= len || space_width(byte_of(w, Ln), byte_of(w, Ln + 1), byte_of(w, Ln + 2)) > 0;
          is_neg |= ends;
        }
      }
    }
    pos += __popcll(wave_ballot(is_pos));
    neg += __popcll(wave_ballot(is_neg));

    // ---- keyword patterns: non-overlapping leftmost counts
    for (int j = 0; j < pt.npat; ++j) {
      const int plen = pt.len[j];
      const int fl = pt.flags[j];
      const uint32_t* t = pt.text[j];
      const uint32_t* mk = pt.mask[j];
      const uint32_t* s = (fl & 1) ? wl : w;
      const bool hit = valid && (p + plen <= len) && ((s[0] & mk[0]) == t[0]) &&
                       ((s[1] & mk[1]) == t[1]) && ((s[2] & mk[2]) == t[2]) &&
                       ((s[3] & mk[3]) == t[3]);
      uint64_t hm = wave_ballot(hit);
      int cnt;
      if (!(fl & 2)) {
        cnt = __popcll(hm);  // cannot self-overlap: every occurrence counts
      } else {
        // bordered pattern: greedy leftmost non-overlapping scan (wave-uniform)
        int nxt = next_ok[wv][j];
        cnt = 0;
        while (hm) {
          const int b = __builtin_ctzll(hm);
          hm &= hm - 1;
          if (base + b >= nxt) {
            ++cnt;
            nxt = base + b + plen;
          }
        }
        if (lane == 0) next_ok[wv][j] = nxt;
      }
      const int sl = pt.slot[j];
#pragma unroll
      for (int s2 = 0; s2 < TA_SLOTS; ++s2) score[s2] += (sl == s2) ? cnt : 0;
    }

    // ---- token hashes: the word-start lane walks its token (<= 32 bytes).
    // Bytes p .. p+15 are already in registers (w): the first 14 steps read
    // them there (the space test looks 2 bytes ahead), longer tokens go on in
    // the LDS window (bytes past len are staged as 0, as the bounds below read)
    if (wstart && tok_idx < L) {
      uint32_t h = 0x811C9DC5u;
      int n = 0;
      bool done = false;
#pragma unroll
      for (int i = 0; i < 14; ++i) {
        if (!done) {
          if (p + i >= len) {
            done = true;
          } else {
            const uint32_t c = byte_of(w, i);
            if (i > 0) {
              const uint32_t d1 = (p + i + 1 < len) ? byte_of(w, i + 1) : 0u;
              const uint32_t d2 = (p + i + 2 < len) ? byte_of(w, i + 2) : 0u;
              done = space_width(c, d1, d2) > 0;
            }
            if (!done) {
              h ^= (c >= 0x41u && c <= 0x5Au) ? (c | 0x20u) : c;
              h *= 0x01000193u;
              ++n;
            }
          }
        }
      }
      const uint8_t* wb = win8 + 4 - base;              // wb[i] = byte i of the message
      for (int q2 = p + n; !done && n < TA_MAX_TOKEN_BYTES && q2 < len; ++n, ++q2) {
        const uint32_t c = wb[q2];
        const uint32_t d1 = (q2 + 1 < len) ? wb[q2 + 1] : 0u;
        const uint32_t d2 = (q2 + 2 < len) ? wb[q2 + 2] : 0u;
        if (space_width(c, d1, d2) > 0) break;
        h ^= (c >= 0x41u && c <= 0x5Au) ? (c | 0x20u) : c;
        h *= 0x01000193u;
      }
      hashes[(int64_t)msg * L + tok_idx] = h;
    }
    ntok = min(L, ntok + __popcll(wmask));
    __builtin_amdgcn_wave_barrier();  // window reuse (WAR) in the next chunk
  }

  if (lane == 0) {
    int32_t* st = stats + (int64_t)msg * TA_STAT_COLS;
    st[ST_WORDS] = words;
    st[ST_POS] = pos;
    st[ST_NEG] = neg;
    st[ST_QUESTION] = question ? 1 : 0;
    st[ST_FLAGS] = fold ? FLAG_FOLD : 0;
    st[ST_NTOK] = ntok;
    // the host's per-message decisions, precomputed: keyword slot with the
    // highest strictly positive score (first maximum = the more urgent level,
    // slots ascend in priority; unused slots score 0), and one code word
    // (sentiment 0 neutral / 1 positive / 2 negative | question << 2 | fold << 3)
    int best_slot = -1, best = 0;
#pragma unroll
    for (int s = 0; s < TA_SLOTS; ++s) {
      st[ST_SCORES + s] = score[s];
      if (score[s] > best) { best = score[s]; best_slot = s; }
    }
    st[ST_BEST_SLOT] = best_slot;
    st[ST_CODE] = (pos > neg ? 1 : (neg > pos ? 2 : 0)) | (question ? 4 : 0) | (fold ? 8 : 0);
  }
}

// One readback of a preprocess batch into host-mapped memory: stats rows,
// classifier predictions at o_pred, the first `cap` token hashes of every
// message at o_ph (int32 offsets into dst).  Replaces three copies and the
// strided-slice gather of the per-launch path.
__global__ void __launch_bounds__(256)
text_readback_kernel(const int32_t* __restrict__ stats, const int32_t* __restrict__ pred,
                     const uint32_t* __restrict__ hashes, int B, int L, int cap, int32_t* __restrict__ dst,
                     int64_t o_pred, int64_t o_ph) {
  const int64_t n_st = (int64_t)B * TA_STAT_COLS;
  const int64_t n_pr = pred ? B : 0;
  const int64_t n_ph = (int64_t)B * cap;
  const int64_t n = n_st + n_pr + n_ph;
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    if (i < n_st) {
      dst[i] = stats[i];
    } else if (i < n_st + n_pr) {
      dst[o_pred + (i - n_st)] = pred[i - n_st];
    } else {
      const int64_t k = i - n_st - n_pr;
      const int64_t b = k / cap, c = k - b * cap;
      dst[o_ph + k] = (int32_t)hashes[b * L + c];
    }
  }
  __threadfence_system();   // visible to the host once the stream's event completes
}

}  // namespace llmq
