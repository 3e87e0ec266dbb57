// Native tokenizers (replaces the reference's Rust HF `tokenizers` via DJL JNI and the
// Java jtokkit cl100k counter -- SURVEY §2.10 N2/N3, TXT/TiktokenLengthFunction.java:21-44,
// AbstractHuggingFaceEmbeddingService.java:155).
//
//  * ByteBPE  : byte-level BPE (GPT-2 / tiktoken cl100k / Llama-3 family).  Vocab is a
//               byte-string -> id table; merge priority comes from an explicit merges
//               list (HF tokenizer.json) or, tiktoken-style, from the rank of the merged
//               token.  Pre-tokenisation approximates the cl100k regex without ICU
//               (letters = ASCII letters + any non-ASCII UTF-8 sequence).  Per-word
//               results are cached.  Encode of a batch runs on a thread pool with the
//               GIL released.
//  * WordPiece: BERT basic tokenizer (clean, optional lower-case + accent strip for
//               Latin-1, punctuation / CJK splitting) + greedy longest-match "##" pieces.
//  * train_bpe: frequency-based BPE trainer (incremental pair counts + lazy max-heap),
//               used to build self-contained vocabularies when no tokenizer files exist
//               (this environment has no network / model hub).
#include <pybind11/pybind11.h>
#include <pybind11/numpy.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <mutex>
#include <queue>
#include <set>
#include <shared_mutex>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace py = pybind11;

namespace {

inline bool is_ascii_letter(unsigned char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z'); }
inline bool is_digit(unsigned char c) { return c >= '0' && c <= '9'; }
inline bool is_space(unsigned char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f'; }
inline bool is_nl(unsigned char c) { return c == '\n' || c == '\r'; }
inline int utf8_len(unsigned char c) {
  if (c < 0x80) return 1;
  if ((c >> 5) == 6) return 2;
  if ((c >> 4) == 14) return 3;
  if ((c >> 3) == 30) return 4;
  return 1;
}
// "letter" class for pre-tokenisation: ASCII letters and any multi-byte UTF-8 char
inline bool is_letter_at(const std::string& s, size_t i) {
  const unsigned char c = s[i];
  return is_ascii_letter(c) || c >= 0x80;
}

// Approximation of the cl100k_base split pattern:
//  '(?i:[sdmt]|ll|ve|re) | [^\r\n\p{L}\p{N}]?\p{L}+ | \p{N}{1,3} | ' '?[^\s\p{L}\p{N}]+[\r\n]* |
//  \s*[\r\n] | \s+(?!\S) | \s+
std::vector<std::pair<size_t, size_t>> pretokenize(const std::string& s) {
  std::vector<std::pair<size_t, size_t>> out;
  const size_t n = s.size();
  size_t i = 0;
  auto letter_run = [&](size_t j) {
    while (j < n && is_letter_at(s, j)) j += utf8_len((unsigned char)s[j]);
    return j;
  };
  while (i < n) {
    const unsigned char c = s[i];
    // contractions
    if (c == '\'' && i + 1 < n) {
      const char a = (char)std::tolower((unsigned char)s[i + 1]);
      if (a == 's' || a == 'd' || a == 'm' || a == 't') {
        if (!(i + 2 < n && is_letter_at(s, i + 2))) { out.push_back({i, 2}); i += 2; continue; }
      }
      if (i + 2 < n) {
        const char b = (char)std::tolower((unsigned char)s[i + 2]);
        if ((a == 'l' && b == 'l') || (a == 'v' && b == 'e') || (a == 'r' && b == 'e')) {
          out.push_back({i, 3});
          i += 3;
          continue;
        }
      }
    }
    // optional single non-letter/non-digit/non-newline prefix followed by letters
    if (is_letter_at(s, i)) {
      size_t j = letter_run(i);
      out.push_back({i, j - i});
      i = j;
      continue;
    }
    if (!is_nl(c) && !is_digit(c) && i + 1 < n && is_letter_at(s, i + 1) && !(c >= 0x80)) {
      size_t j = letter_run(i + 1);
      out.push_back({i, j - i});
      i = j;
      continue;
    }
    if (is_digit(c)) {
      size_t j = i;
      while (j < n && j - i < 3 && is_digit((unsigned char)s[j])) ++j;
      out.push_back({i, j - i});
      i = j;
      continue;
    }
    if (is_space(c)) {
      size_t j = i;
      while (j < n && is_space((unsigned char)s[j])) ++j;
      // \s*[\r\n] : whitespace run ending with a newline
      size_t last_nl = std::string::npos;
      for (size_t k = i; k < j; ++k)
        if (is_nl((unsigned char)s[k])) last_nl = k;
      if (last_nl != std::string::npos) {
        out.push_back({i, last_nl + 1 - i});
        i = last_nl + 1;
        continue;
      }
      // \s+(?!\S): leave the last space to prefix the next word
      if (j < n && j - i > 1) {
        out.push_back({i, j - i - 1});
        i = j - 1;
        continue;
      }
      if (j < n && j - i == 1) {
        // single space before a non-space: attaches to the following punctuation run
        const unsigned char d = s[j];
        if (!is_letter_at(s, j) && !is_digit(d)) {
          size_t k = j;
          while (k < n && !is_space((unsigned char)s[k]) && !is_letter_at(s, k) && !is_digit((unsigned char)s[k])) ++k;
          while (k < n && is_nl((unsigned char)s[k])) ++k;
          out.push_back({i, k - i});
          i = k;
          continue;
        }
        // space before letters handled by the letter rule with prefix
        size_t k = letter_run(j);
        if (k > j) {
          out.push_back({i, k - i});
          i = k;
          continue;
        }
      }
      out.push_back({i, j - i});
      i = j;
      continue;
    }
    // punctuation run (+ trailing newlines)
    size_t j = i;
    while (j < n && !is_space((unsigned char)s[j]) && !is_letter_at(s, j) && !is_digit((unsigned char)s[j])) ++j;
    while (j < n && is_nl((unsigned char)s[j])) ++j;
    if (j == i) j = i + 1;
    out.push_back({i, j - i});
    i = j;
  }
  return out;
}

struct PairHash {
  size_t operator()(const std::pair<int, int>& p) const noexcept {
    return std::hash<uint64_t>()(((uint64_t)(uint32_t)p.first << 32) | (uint32_t)p.second);
  }
};

class ByteBPE {
 public:
  // vocab: token bytes -> id.  merges: list of (left bytes, right bytes) in priority
  // order; empty -> tiktoken mode (priority = id/rank of the merged token).
  ByteBPE(const std::vector<std::pair<py::bytes, int>>& vocab, const std::vector<std::pair<py::bytes, py::bytes>>& merges,
          const std::vector<std::pair<std::string, int>>& specials) {
    for (auto& kv : vocab) {
      std::string b = kv.first;
      tok2id_[b] = kv.second;
      if ((int)id2tok_.size() <= kv.second) id2tok_.resize(kv.second + 1);
      id2tok_[kv.second] = b;
    }
    for (int c = 0; c < 256; ++c) {
      auto it = tok2id_.find(std::string(1, (char)c));
      byte_id_[c] = it == tok2id_.end() ? -1 : it->second;
    }
    if (!merges.empty()) {
      int rank = 0;
      for (auto& m : merges) {
        std::string a = m.first, b = m.second;
        auto ia = tok2id_.find(a), ib = tok2id_.find(b), ic = tok2id_.find(a + b);
        if (ia == tok2id_.end() || ib == tok2id_.end() || ic == tok2id_.end()) { ++rank; continue; }
        pair_rank_[{ia->second, ib->second}] = {rank++, ic->second};
      }
      tiktoken_ = false;
    } else {
      tiktoken_ = true;
    }
    std::set<size_t> lens;
    for (auto& s : specials) {
      specials_[s.first] = s.second;
      if ((int)id2tok_.size() <= s.second) id2tok_.resize(s.second + 1);
      id2tok_[s.second] = s.first;
      special_ids_.insert(s.second);
      if (!s.first.empty()) {
        special_first_[(unsigned char)s.first[0]] = true;
        lens.insert(s.first.size());
      }
    }
    special_lens_.assign(lens.rbegin(), lens.rend());  // longest match first
  }

  // Special tokens are matched in one left-to-right scan: only positions whose byte can
  // start a special are probed, with one hash lookup per distinct special length (Llama-3
  // vocabularies carry ~250 reserved specials; synthetic ones >100k).
  std::vector<int> encode(const std::string& text, bool allow_special) {
    std::vector<int> out;
    if (allow_special && !specials_.empty()) {
      size_t start = 0;
      for (size_t i = 0; i < text.size(); ++i) {
        if (!special_first_[(unsigned char)text[i]]) continue;
        for (size_t L : special_lens_) {
          if (i + L > text.size()) continue;
          auto it = specials_.find(text.substr(i, L));
          if (it == specials_.end()) continue;
          if (i > start) encode_ordinary(text.substr(start, i - start), out);
          out.push_back(it->second);
          start = i + L;
          i = start - 1;
          break;
        }
      }
      if (start < text.size()) encode_ordinary(text.substr(start), out);
    } else {
      encode_ordinary(text, out);
    }
    return out;
  }

  std::vector<std::vector<int>> encode_batch(const std::vector<std::string>& texts, bool allow_special, int threads) {
    std::vector<std::vector<int>> out(texts.size());
    py::gil_scoped_release nogil;
    const int nt = std::max(1, std::min<int>(threads, (int)texts.size()));
    std::atomic<size_t> next{0};
    auto work = [&]() {
      for (size_t i = next++; i < texts.size(); i = next++) out[i] = encode(texts[i], allow_special);
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < nt; ++t) pool.emplace_back(work);
    work();
    for (auto& t : pool) t.join();
    return out;
  }

  size_t count(const std::string& text) {
    std::vector<int> out;
    encode_ordinary(text, out);
    return out.size();
  }

  py::bytes decode_bytes(const std::vector<int>& ids, bool skip_special) {
    std::string s;
    for (int id : ids) {
      if (id < 0 || id >= (int)id2tok_.size()) continue;
      if (skip_special && special_ids_.count(id)) continue;
      s += id2tok_[id];
    }
    return py::bytes(s);
  }

  int vocab_size() const { return (int)id2tok_.size(); }
  int token_to_id(const std::string& t) const {
    auto it = specials_.find(t);
    if (it != specials_.end()) return it->second;
    auto jt = tok2id_.find(t);
    return jt == tok2id_.end() ? -1 : jt->second;
  }
  py::bytes id_to_token(int id) const {
    if (id < 0 || id >= (int)id2tok_.size()) return py::bytes("");
    return py::bytes(id2tok_[id]);
  }

 private:
  void encode_ordinary(const std::string& text, std::vector<int>& out) {
    for (auto& span : pretokenize(text)) {
      const std::string word = text.substr(span.first, span.second);
      {
        std::shared_lock<std::shared_mutex> g(cache_mu_);
        auto it = cache_.find(word);
        if (it != cache_.end()) {
          out.insert(out.end(), it->second.begin(), it->second.end());
          continue;
        }
      }
      std::vector<int> ids = bpe_word(word);
      out.insert(out.end(), ids.begin(), ids.end());
      std::unique_lock<std::shared_mutex> g(cache_mu_);
      if (cache_.size() > 200000) cache_.clear();
      cache_.emplace(word, std::move(ids));
    }
  }

  std::vector<int> bpe_word(const std::string& w) {
    auto whole = tok2id_.find(w);
    if (whole != tok2id_.end() && tiktoken_) return {whole->second};
    // symbols as (start, len) into w with current ids
    std::vector<int> ids;
    std::vector<std::string> syms;
    for (unsigned char c : w) {
      syms.emplace_back(1, (char)c);
      ids.push_back(byte_id_[c] >= 0 ? byte_id_[c] : 0);
    }
    while (syms.size() > 1) {
      int best = INT32_MAX, bi = -1, bid = -1;
      for (size_t i = 0; i + 1 < syms.size(); ++i) {
        int r, nid;
        if (tiktoken_) {
          auto it = tok2id_.find(syms[i] + syms[i + 1]);
          if (it == tok2id_.end()) continue;
          r = nid = it->second;
        } else {
          auto it = pair_rank_.find({ids[i], ids[i + 1]});
          if (it == pair_rank_.end()) continue;
          r = it->second.first;
          nid = it->second.second;
        }
        if (r < best) { best = r; bi = (int)i; bid = nid; }
      }
      if (bi < 0) break;
      syms[bi] += syms[bi + 1];
      ids[bi] = bid;
      syms.erase(syms.begin() + bi + 1);
      ids.erase(ids.begin() + bi + 1);
    }
    return ids;
  }

  std::unordered_map<std::string, int> tok2id_;
  std::vector<std::string> id2tok_;
  std::unordered_map<std::pair<int, int>, std::pair<int, int>, PairHash> pair_rank_;
  std::unordered_map<std::string, int> specials_;
  std::unordered_set<int> special_ids_;
  bool special_first_[256] = {};
  std::vector<size_t> special_lens_;
  int byte_id_[256];
  bool tiktoken_ = true;
  std::unordered_map<std::string, std::vector<int>> cache_;
  std::shared_mutex cache_mu_;
};

// ----------------------------------------------------------------- WordPiece
inline bool is_punct_cp(uint32_t cp) {
  if ((cp >= 33 && cp <= 47) || (cp >= 58 && cp <= 64) || (cp >= 91 && cp <= 96) || (cp >= 123 && cp <= 126))
    return true;
  return (cp >= 0x2000 && cp <= 0x206F) || (cp >= 0x3000 && cp <= 0x303F) || (cp >= 0xFF00 && cp <= 0xFF0F);
}
inline bool is_cjk(uint32_t cp) {
  return (cp >= 0x4E00 && cp <= 0x9FFF) || (cp >= 0x3400 && cp <= 0x4DBF) || (cp >= 0x20000 && cp <= 0x2A6DF) ||
         (cp >= 0xF900 && cp <= 0xFAFF) || (cp >= 0x2F800 && cp <= 0x2FA1F);
}

std::vector<uint32_t> utf8_decode(const std::string& s) {
  std::vector<uint32_t> cps;
  for (size_t i = 0; i < s.size();) {
    const unsigned char c = s[i];
    const int l = utf8_len(c);
    uint32_t cp = c;
    if (l == 2 && i + 1 < s.size()) cp = ((c & 0x1F) << 6) | (s[i + 1] & 0x3F);
    else if (l == 3 && i + 2 < s.size()) cp = ((c & 0x0F) << 12) | ((s[i + 1] & 0x3F) << 6) | (s[i + 2] & 0x3F);
    else if (l == 4 && i + 3 < s.size())
      cp = ((c & 0x07) << 18) | ((s[i + 1] & 0x3F) << 12) | ((s[i + 2] & 0x3F) << 6) | (s[i + 3] & 0x3F);
    cps.push_back(cp);
    i += l;
  }
  return cps;
}

void utf8_append(std::string& s, uint32_t cp) {
  if (cp < 0x80) s += (char)cp;
  else if (cp < 0x800) { s += (char)(0xC0 | (cp >> 6)); s += (char)(0x80 | (cp & 0x3F)); }
  else if (cp < 0x10000) {
    s += (char)(0xE0 | (cp >> 12)); s += (char)(0x80 | ((cp >> 6) & 0x3F)); s += (char)(0x80 | (cp & 0x3F));
  } else {
    s += (char)(0xF0 | (cp >> 18)); s += (char)(0x80 | ((cp >> 12) & 0x3F));
    s += (char)(0x80 | ((cp >> 6) & 0x3F)); s += (char)(0x80 | (cp & 0x3F));
  }
}

// Latin-1 lower + accent strip (NFD approximation for U+00C0..U+00FF)
uint32_t fold_latin(uint32_t cp, bool lower, bool strip) {
  static const char* base = "AAAAAAACEEEEIIIIDNOOOOOxOUUUUYTsaaaaaaaceeeeiiiidnooooo/ouuuuyty";
  if (strip && cp >= 0xC0 && cp <= 0xFF) {
    const char b = base[cp - 0xC0];
    if (b != 'x' && b != '/' && b != 'T' && b != 't' && b != 's') cp = (uint32_t)b;
  }
  if (lower) {
    if (cp >= 'A' && cp <= 'Z') cp += 32;
    else if (cp >= 0xC0 && cp <= 0xDE && cp != 0xD7) cp += 32;
  }
  return cp;
}

class WordPiece {
 public:
  WordPiece(const std::vector<std::string>& vocab, bool lower, bool strip_accents, const std::string& unk,
            int max_chars)
      : lower_(lower), strip_(strip_accents), max_chars_(max_chars) {
    for (size_t i = 0; i < vocab.size(); ++i) vocab_[vocab[i]] = (int)i;
    id2tok_ = vocab;
    auto it = vocab_.find(unk);
    unk_id_ = it == vocab_.end() ? 0 : it->second;
    // allocation-free lookup tables: word-initial pieces and "##" continuations, keyed
    // by string_views into id2tok_ (never resized after this point)
    for (size_t i = 0; i < id2tok_.size(); ++i) {
      const std::string& t = id2tok_[i];
      if (t.size() > 2 && t[0] == '#' && t[1] == '#') {
        std::string_view k(t.data() + 2, t.size() - 2);
        cont_.emplace(k, (int)i);
        max_cont_ = std::max(max_cont_, k.size());
      } else if (!t.empty()) {
        std::string_view k(t);
        head_.emplace(k, (int)i);
        max_head_ = std::max(max_head_, k.size());
      }
    }
  }

  std::vector<std::string> basic_tokens(const std::string& text) const {
    std::vector<std::string> words;
    std::string cur;
    auto flush = [&]() { if (!cur.empty()) { words.push_back(cur); cur.clear(); } };
    for (uint32_t cp : utf8_decode(text)) {
      if (cp == 0 || cp == 0xFFFD || (cp < 32 && cp != '\t' && cp != '\n' && cp != '\r')) continue;
      if (cp == ' ' || cp == '\t' || cp == '\n' || cp == '\r' || cp == 0xA0 || cp == 0x3000) { flush(); continue; }
      cp = fold_latin(cp, lower_, strip_);
      if (strip_ && cp >= 0x300 && cp <= 0x36F) continue;  // combining marks
      if (is_punct_cp(cp) || is_cjk(cp)) {
        flush();
        std::string t;
        utf8_append(t, cp);
        words.push_back(t);
        continue;
      }
      utf8_append(cur, cp);
    }
    flush();
    return words;
  }

  // Greedy longest-match-first WordPiece of one normalised word, appended to out.
  // Candidate pieces are string_views into the word (no allocation per attempt); the
  // search starts at the longest vocabulary piece instead of the whole remaining word.
  void wordpiece(const std::string& w, std::vector<uint32_t>& offs, std::vector<int>& out) const {
    offs.clear();
    for (size_t o = 0; o < w.size(); o += utf8_len((unsigned char)w[o])) offs.push_back((uint32_t)o);
    const size_t ncp = offs.size();
    offs.push_back((uint32_t)w.size());
    if ((int)ncp > max_chars_) { out.push_back(unk_id_); return; }
    const size_t mark = out.size();
    size_t start = 0;
    while (start < ncp) {
      const auto& map = start == 0 ? head_ : cont_;
      const size_t maxb = start == 0 ? max_head_ : max_cont_;
      size_t end = ncp;
      int found = -1;
      for (; end > start; --end) {
        const size_t nb = offs[end] - offs[start];
        if (nb > maxb) continue;
        auto it = map.find(std::string_view(w.data() + offs[start], nb));
        if (it != map.end()) { found = it->second; break; }
      }
      if (found < 0) {   // the whole word is unknown
        out.resize(mark);
        out.push_back(unk_id_);
        return;
      }
      out.push_back(found);
      start = end;
    }
  }

  std::vector<int> encode(const std::string& text) const {
    std::vector<int> out;
    out.reserve(text.size() / 3 + 4);
    std::string cur;
    std::vector<uint32_t> offs;
    auto flush = [&]() {
      if (!cur.empty()) { wordpiece(cur, offs, out); cur.clear(); }
    };
    const unsigned char* p = (const unsigned char*)text.data();
    const size_t n = text.size();
    for (size_t i = 0; i < n;) {
      // one code point, decoded exactly as utf8_decode does
      const unsigned char c = p[i];
      const int l = utf8_len(c);
      uint32_t cp = c;
      if (l == 2 && i + 1 < n) cp = ((c & 0x1F) << 6) | (p[i + 1] & 0x3F);
      else if (l == 3 && i + 2 < n) cp = ((c & 0x0F) << 12) | ((p[i + 1] & 0x3F) << 6) | (p[i + 2] & 0x3F);
      else if (l == 4 && i + 3 < n)
        cp = ((c & 0x07) << 18) | ((p[i + 1] & 0x3F) << 12) | ((p[i + 2] & 0x3F) << 6) | (p[i + 3] & 0x3F);
      i += l;
      if (cp == 0 || cp == 0xFFFD || (cp < 32 && cp != '\t' && cp != '\n' && cp != '\r')) continue;
      if (cp == ' ' || cp == '\t' || cp == '\n' || cp == '\r' || cp == 0xA0 || cp == 0x3000) { flush(); continue; }
      cp = fold_latin(cp, lower_, strip_);
      if (strip_ && cp >= 0x300 && cp <= 0x36F) continue;  // combining marks
      if (is_punct_cp(cp) || is_cjk(cp)) {
        flush();
        utf8_append(cur, cp);
        flush();
        continue;
      }
      utf8_append(cur, cp);
    }
    flush();
    return out;
  }

  std::vector<std::vector<int>> encode_batch(const std::vector<std::string>& texts, int threads) const {
    std::vector<std::vector<int>> out(texts.size());
    py::gil_scoped_release nogil;
    const int nt = std::max(1, std::min<int>(threads, (int)texts.size()));
    std::atomic<size_t> next{0};
    auto work = [&]() {
      for (size_t i = next++; i < texts.size(); i = next++) out[i] = encode(texts[i]);
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < nt; ++t) pool.emplace_back(work);
    work();
    for (auto& t : pool) t.join();
    return out;
  }

  // [CLS] + ids[:max_len-2] + [SEP] of every text, packed: (ids int32 [sum lens],
  // lens int32 [n]) -- no per-token Python objects on the way to the encoder.
  py::tuple encode_batch_packed(const std::vector<std::string>& texts, int max_len, int cls, int sep,
                                int threads) const {
    std::vector<std::vector<int>> toks = encode_batch(texts, threads);
    const size_t n = toks.size();
    const int keep = std::max(0, max_len - 2);
    py::array_t<int32_t> lens((py::ssize_t)n);
    auto L = lens.mutable_unchecked<1>();
    size_t total = 0;
    for (size_t i = 0; i < n; ++i) {
      const int l = (int)std::min<size_t>(toks[i].size(), (size_t)keep) + 2;
      L(i) = l;
      total += l;
    }
    py::array_t<int32_t> ids((py::ssize_t)total);
    int32_t* d = ids.mutable_data();
    for (size_t i = 0; i < n; ++i) {
      *d++ = cls;
      const size_t m = (size_t)L(i) - 2;
      std::copy(toks[i].begin(), toks[i].begin() + m, d);
      d += m;
      *d++ = sep;
    }
    return py::make_tuple(ids, lens);
  }

  std::string decode(const std::vector<int>& ids) const {
    std::string s;
    for (int id : ids) {
      if (id < 0 || id >= (int)id2tok_.size()) continue;
      const std::string& t = id2tok_[id];
      if (t.size() >= 2 && t[0] == '#' && t[1] == '#') s += t.substr(2);
      else { if (!s.empty()) s += ' '; s += t; }
    }
    return s;
  }

  int token_to_id(const std::string& t) const {
    auto it = vocab_.find(t);
    return it == vocab_.end() ? -1 : it->second;
  }
  int vocab_size() const { return (int)id2tok_.size(); }

 private:
  std::unordered_map<std::string, int> vocab_;
  std::vector<std::string> id2tok_;
  std::unordered_map<std::string_view, int> head_, cont_;
  size_t max_head_ = 0, max_cont_ = 0;
  bool lower_, strip_;
  int max_chars_;
  int unk_id_;
};

// ----------------------------------------------------------------- BPE trainer
// Returns merges as (left bytes, right bytes) in learned order.
std::vector<std::pair<py::bytes, py::bytes>> train_bpe(const std::vector<std::string>& texts, int num_merges,
                                                       int min_freq) {
  std::vector<std::pair<std::string, std::string>> merges;
  {
    py::gil_scoped_release nogil;
    std::unordered_map<std::string, int64_t> word_freq;
    for (auto& t : texts)
      for (auto& sp : pretokenize(t)) word_freq[t.substr(sp.first, sp.second)]++;
    std::vector<std::vector<std::string>> words;
    std::vector<int64_t> freq;
    for (auto& kv : word_freq) {
      std::vector<std::string> syms;
      for (unsigned char c : kv.first) syms.emplace_back(1, (char)c);
      words.push_back(std::move(syms));
      freq.push_back(kv.second);
    }
    struct SPH {
      size_t operator()(const std::pair<std::string, std::string>& p) const noexcept {
        return std::hash<std::string>()(p.first) * 1000003u ^ std::hash<std::string>()(p.second);
      }
    };
    std::unordered_map<std::pair<std::string, std::string>, int64_t, SPH> counts;
    std::unordered_map<std::pair<std::string, std::string>, std::unordered_set<int>, SPH> where;
    for (size_t w = 0; w < words.size(); ++w)
      for (size_t i = 0; i + 1 < words[w].size(); ++i) {
        auto p = std::make_pair(words[w][i], words[w][i + 1]);
        counts[p] += freq[w];
        where[p].insert((int)w);
      }
    using Item = std::pair<int64_t, std::pair<std::string, std::string>>;
    std::priority_queue<Item> heap;
    for (auto& kv : counts) heap.push({kv.second, kv.first});
    while ((int)merges.size() < num_merges && !heap.empty()) {
      Item top = heap.top();
      heap.pop();
      auto cit = counts.find(top.second);
      if (cit == counts.end() || cit->second != top.first) continue;  // stale
      if (top.first < min_freq) break;
      const auto pair = top.second;
      merges.push_back(pair);
      const std::string merged = pair.first + pair.second;
      std::unordered_set<int> affected = where[pair];
      for (int w : affected) {
        auto& syms = words[w];
        // remove old pair counts of this word
        for (size_t i = 0; i + 1 < syms.size(); ++i) {
          auto p = std::make_pair(syms[i], syms[i + 1]);
          counts[p] -= freq[w];
        }
        std::vector<std::string> ns;
        for (size_t i = 0; i < syms.size();) {
          if (i + 1 < syms.size() && syms[i] == pair.first && syms[i + 1] == pair.second) {
            ns.push_back(merged);
            i += 2;
          } else {
            ns.push_back(syms[i]);
            i += 1;
          }
        }
        syms.swap(ns);
        for (size_t i = 0; i + 1 < syms.size(); ++i) {
          auto p = std::make_pair(syms[i], syms[i + 1]);
          int64_t& c = counts[p];
          c += freq[w];
          where[p].insert(w);
          heap.push({c, p});
        }
      }
      counts.erase(pair);
      where.erase(pair);
    }
  }
  std::vector<std::pair<py::bytes, py::bytes>> r;
  for (auto& m : merges) r.emplace_back(py::bytes(m.first), py::bytes(m.second));
  return r;
}

std::vector<std::pair<size_t, size_t>> pretokenize_py(const std::string& s) { return pretokenize(s); }

}  // namespace

void bind_tokenizer(py::module_& m) {
  py::class_<ByteBPE>(m, "ByteBPE")
      .def(py::init<const std::vector<std::pair<py::bytes, int>>&, const std::vector<std::pair<py::bytes, py::bytes>>&,
                    const std::vector<std::pair<std::string, int>>&>())
      .def("encode", &ByteBPE::encode, py::arg("text"), py::arg("allow_special") = true,
           py::call_guard<py::gil_scoped_release>())
      .def("encode_batch", &ByteBPE::encode_batch, py::arg("texts"), py::arg("allow_special") = true,
           py::arg("threads") = 4)
      .def("count", &ByteBPE::count, py::call_guard<py::gil_scoped_release>())
      .def("decode_bytes", &ByteBPE::decode_bytes, py::arg("ids"), py::arg("skip_special") = false)
      .def("vocab_size", &ByteBPE::vocab_size)
      .def("token_to_id", &ByteBPE::token_to_id)
      .def("id_to_token", &ByteBPE::id_to_token);
  py::class_<WordPiece>(m, "WordPiece")
      .def(py::init<const std::vector<std::string>&, bool, bool, const std::string&, int>(), py::arg("vocab"),
           py::arg("lower") = true, py::arg("strip_accents") = true, py::arg("unk") = "[UNK]",
           py::arg("max_chars") = 100)
      .def("encode", &WordPiece::encode, py::call_guard<py::gil_scoped_release>())
      .def("encode_batch", &WordPiece::encode_batch, py::arg("texts"), py::arg("threads") = 8)
      .def("encode_batch_packed", &WordPiece::encode_batch_packed, py::arg("texts"), py::arg("max_len"),
           py::arg("cls"), py::arg("sep"), py::arg("threads") = 8)
      .def("basic_tokens", &WordPiece::basic_tokens)
      .def("decode", &WordPiece::decode)
      .def("token_to_id", &WordPiece::token_to_id)
      .def("vocab_size", &WordPiece::vocab_size);
  m.def("train_bpe", &train_bpe, py::arg("texts"), py::arg("num_merges"), py::arg("min_freq") = 2);
  m.def("pretokenize", &pretokenize_py);
}
