// Native byte-level BPE tokenizer: the Llama-3 `tokenizer.json` (the `llama3.1` model tag of
// the reference's co-pilot, `web/streamlit_app.py:28`) encoded and decoded exactly as the
// HF `tokenizers` library does it, so the engine C ABI serves a real tokenizer without
// entering Python.
//
// Covered (anything else in the file leaves the tokenizer "not native" and the request
// takes Python's HFTokenizer):
//   * model: BPE over the GPT-2 byte-to-unicode alphabet, merges as "a b" strings or
//     [a, b] pairs, `ignore_merges` (a whole pre-token found in the vocab is one token), no
//     dropout / subword prefix / suffix / byte fallback;
//   * added tokens (the Llama-3 specials) split out of the text first, leftmost-longest,
//     without lstrip / rstrip / single-word options;
//   * pre-tokenizer: Split(Llama-3 pattern, Isolated) + ByteLevel(use_regex=false), or
//     ByteLevel(use_regex=true) with the GPT-2 pattern; the patterns are hand-compiled
//     matchers (below), with \p{L} / \p{N} from unicode_tables.h and \s = White_Space;
//   * decoder: ByteLevel, special tokens skipped, lossy UTF-8 (U+FFFD per maximal
//     ill-formed subpart, as Rust's from_utf8_lossy).
// Parity: tests/test_native_bpe_tok.py trains a Llama-3-style tokenizer with `tokenizers`
// and compares ids and text on ASCII and non-ASCII chat text.
#pragma once
#include <stdint.h>

#include <algorithm>
#include <fstream>
#include <queue>
#include <sstream>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "engine/unicode_tables.h"
#include "net/json.h"

namespace p2p {

namespace uni {

template <size_t N>
inline bool in_table(const uint32_t (&t)[N][2], uint32_t c) {
  size_t lo = 0, hi = N;
  while (lo < hi) {
    const size_t mid = (lo + hi) / 2;
    if (c < t[mid][0]) hi = mid;
    else if (c > t[mid][1]) lo = mid + 1;
    else return true;
  }
  return false;
}

inline bool letter(uint32_t c) {
  if (c < 0x80) return (c | 32) - 'a' < 26u;
  return in_table(kLetter, c);
}

inline bool number(uint32_t c) {
  if (c < 0x80) return c - '0' < 10u;
  return in_table(kNumber, c);
}

// regex \s: the White_Space property
inline bool space(uint32_t c) {
  return (c >= 9 && c <= 13) || c == 32 || c == 0x85 || c == 0xA0 || c == 0x1680 ||
         (c >= 0x2000 && c <= 0x200A) || c == 0x2028 || c == 0x2029 || c == 0x202F ||
         c == 0x205F || c == 0x3000;
}

// Python str.isspace (what HFTokenizer.decode's .strip() removes)
inline bool py_space(uint32_t c) { return space(c) || (c >= 0x1C && c <= 0x1F); }

// strict UTF-8 -> code points (+ byte offset of each, and the end); false if ill-formed
inline bool utf8_decode(const std::string& s, std::vector<uint32_t>* cps, std::vector<size_t>* offs) {
  const size_t n = s.size();
  size_t i = 0;
  while (i < n) {
    const unsigned char b = (unsigned char)s[i];
    uint32_t c;
    int len;
    if (b < 0x80) c = b, len = 1;
    else if (b >= 0xC2 && b <= 0xDF) c = b & 0x1F, len = 2;
    else if (b >= 0xE0 && b <= 0xEF) c = b & 0x0F, len = 3;
    else if (b >= 0xF0 && b <= 0xF4) c = b & 0x07, len = 4;
    else return false;
    if (i + len > n) return false;
    for (int k = 1; k < len; ++k) {
      const unsigned char x = (unsigned char)s[i + k];
      if ((x & 0xC0) != 0x80) return false;
      c = (c << 6) | (x & 0x3F);
    }
    if ((len == 3 && (c < 0x800 || (c >= 0xD800 && c < 0xE000))) || (len == 4 && (c < 0x10000 || c > 0x10FFFF)))
      return false;
    cps->push_back(c);
    offs->push_back(i);
    i += len;
  }
  offs->push_back(n);
  return true;
}

inline void utf8_put(uint32_t c, std::string* out) {
  if (c < 0x80) {
    out->push_back((char)c);
  } else if (c < 0x800) {
    out->push_back((char)(0xC0 | (c >> 6)));
    out->push_back((char)(0x80 | (c & 0x3F)));
  } else if (c < 0x10000) {
    out->push_back((char)(0xE0 | (c >> 12)));
    out->push_back((char)(0x80 | ((c >> 6) & 0x3F)));
    out->push_back((char)(0x80 | (c & 0x3F)));
  } else {
    out->push_back((char)(0xF0 | (c >> 18)));
    out->push_back((char)(0x80 | ((c >> 12) & 0x3F)));
    out->push_back((char)(0x80 | ((c >> 6) & 0x3F)));
    out->push_back((char)(0x80 | (c & 0x3F)));
  }
}

// bytes -> valid UTF-8, one U+FFFD per maximal ill-formed subpart (Unicode "substitution of
// maximal subparts", which Rust's String::from_utf8_lossy and Python's errors="replace" follow)
inline std::string utf8_lossy(const std::string& s) {
  std::string out;
  const size_t n = s.size();
  size_t i = 0;
  auto cont = [&](size_t k, unsigned lo, unsigned hi) {
    return k < n && (unsigned char)s[k] >= lo && (unsigned char)s[k] <= hi;
  };
  while (i < n) {
    const unsigned char b = (unsigned char)s[i];
    int len = 0;
    if (b < 0x80) {
      out.push_back((char)b);
      ++i;
      continue;
    }
    // (lead range) -> allowed range of the 2nd byte (Unicode Table 3-7)
    unsigned lo2 = 0x80, hi2 = 0xBF;
    if (b >= 0xC2 && b <= 0xDF) len = 2;
    else if (b == 0xE0) len = 3, lo2 = 0xA0;
    else if ((b >= 0xE1 && b <= 0xEC) || b == 0xEE || b == 0xEF) len = 3;
    else if (b == 0xED) len = 3, hi2 = 0x9F;
    else if (b == 0xF0) len = 4, lo2 = 0x90;
    else if (b >= 0xF1 && b <= 0xF3) len = 4;
    else if (b == 0xF4) len = 4, hi2 = 0x8F;
    if (len == 0) {  // not a lead byte
      out += "\xEF\xBF\xBD";
      ++i;
      continue;
    }
    size_t k = i + 1;
    bool okseq = cont(k, lo2, hi2);
    if (okseq) {
      ++k;
      while ((int)(k - i) < len && cont(k, 0x80, 0xBF)) ++k;
      okseq = (int)(k - i) == len;
    }
    if (okseq) {
      out.append(s, i, len);
      i += len;
    } else {
      out += "\xEF\xBF\xBD";
      i = k;  // the maximal subpart (at least the lead byte)
    }
  }
  return out;
}

}  // namespace uni

class BpeTok {
 public:
  enum Pattern { kLlama3, kGpt2 };

  // tokenizer.json text -> ready, or throws std::runtime_error naming what is not covered
  void load_json(const std::string& text) {
    const Json t = Json::parse(text);
    const Json& m = t.get("model");
    if (m.get_string("type") != "BPE") throw std::runtime_error("model is not BPE");
    if (!m.get("dropout").is_null() || !m.get("continuing_subword_prefix").is_null() ||
        !m.get("end_of_word_suffix").is_null() || m.get_bool("byte_fallback", false))
      throw std::runtime_error("BPE options not covered");
    ignore_merges_ = m.get_bool("ignore_merges", false);
    if (!t.get("normalizer").is_null()) throw std::runtime_error("normalizer not covered");
    parse_pre(t.get("pre_tokenizer"));
    if (t.get("decoder").get_string("type") != "ByteLevel") throw std::runtime_error("decoder not covered");
    // byte-level alphabet (GPT-2 bytes_to_unicode)
    int extra = 0;
    for (int b = 0; b < 256; ++b) {
      const bool keep = (b >= 33 && b <= 126) || (b >= 161 && b <= 172) || (b >= 174 && b <= 255);
      const uint32_t c = keep ? (uint32_t)b : (uint32_t)(256 + extra++);
      byte_char_[b].clear();
      uni::utf8_put(c, &byte_char_[b]);
      char_byte_[c] = (uint8_t)b;
    }
    for (auto& kv : m.get("vocab").fields()) {
      const int id = (int)kv.second.integer();
      vocab_[kv.first] = id;
      if (id >= (int)id_str_.size()) id_str_.resize(id + 1);
      id_str_[id] = kv.first;
    }
    int rank = 0;
    for (auto& mg : m.get("merges").items()) {
      std::string a, b;
      if (mg.is_string()) {
        const std::string& s = mg.str();
        const size_t sp = s.find(' ', 1);
        if (sp == std::string::npos) throw std::runtime_error("bad merge");
        a = s.substr(0, sp);
        b = s.substr(sp + 1);
      } else {
        a = mg.at(0).str();
        b = mg.at(1).str();
      }
      auto ia = vocab_.find(a), ib = vocab_.find(b), ic = vocab_.find(a + b);
      if (ia == vocab_.end() || ib == vocab_.end() || ic == vocab_.end())
        throw std::runtime_error("merge of tokens outside the vocab");
      merges_.emplace(key(ia->second, ib->second), std::make_pair(rank++, ic->second));
    }
    for (auto& at : t.get("added_tokens").items()) {
      if (at.get_bool("lstrip", false) || at.get_bool("rstrip", false) || at.get_bool("single_word", false))
        throw std::runtime_error("added-token options not covered");
      const int id = (int)at.get("id").integer();
      const std::string& c = at.get("content").str();
      if (c.empty()) continue;
      added_.push_back({c, id, at.get_bool("special", false)});
      if (id >= (int)id_str_.size()) id_str_.resize(id + 1);
      added_id_[id] = added_.size() - 1;
    }
    std::sort(added_.begin(), added_.end(), [](const Added& x, const Added& y) { return x.text.size() > y.text.size(); });
    added_id_.clear();
    for (size_t i = 0; i < added_.size(); ++i) {
      added_id_[added_[i].id] = i;
      first_[(unsigned char)added_[i].text[0]] = true;
    }
    ok_ = true;
  }

  void load_file(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("cannot open " + path);
    std::stringstream ss;
    ss << f.rdbuf();
    load_json(ss.str());
  }

  bool ok() const { return ok_; }

  int token_id(const std::string& s) const {
    for (auto& a : added_)
      if (a.text == s) return a.id;
    auto it = vocab_.find(s);
    return it == vocab_.end() ? -1 : it->second;
  }

  // tok.encode(text, add_special_tokens=False).ids; false if the text is not UTF-8 or a byte
  // is missing from the vocab (then Python decides)
  bool encode(const std::string& text, std::vector<int>* out) const {
    size_t i = 0, seg = 0;
    const size_t n = text.size();
    while (i < n) {
      const Added* a = added_at(text, i);
      if (!a) {
        ++i;
        continue;
      }
      if (!encode_plain(text.substr(seg, i - seg), out)) return false;
      out->push_back(a->id);
      i += a->text.size();
      seg = i;
    }
    return encode_plain(text.substr(seg), out);
  }

  // tok.decode(ids, skip_special_tokens=True) (not yet stripped)
  std::string decode(const std::vector<int>& ids) const {
    std::string bytes;
    for (int id : ids) {
      auto ai = added_id_.find(id);
      const std::string* tok = nullptr;
      if (ai != added_id_.end()) {
        if (added_[ai->second].special) continue;
        tok = &added_[ai->second].text;
      } else if (id >= 0 && id < (int)id_str_.size() && !id_str_[id].empty()) {
        tok = &id_str_[id];
      } else {
        continue;  // unknown id: dropped, as tokenizers does
      }
      std::vector<uint32_t> cps;
      std::vector<size_t> offs;
      std::string mapped;
      bool all = uni::utf8_decode(*tok, &cps, &offs);
      for (size_t k = 0; all && k < cps.size(); ++k) {
        auto it = char_byte_.find(cps[k]);
        if (it == char_byte_.end()) all = false;
        else mapped.push_back((char)it->second);
      }
      bytes += all ? mapped : *tok;
    }
    return uni::utf8_lossy(bytes);
  }

 private:
  struct Added {
    std::string text;
    int id;
    bool special;
  };

  static uint64_t key(int a, int b) { return ((uint64_t)(uint32_t)a << 32) | (uint32_t)b; }

  void parse_pre(const Json& p) {
    static const char* kL3 =
        "(?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\\r\\n\\p{L}\\p{N}]?\\p{L}+|\\p{N}{1,3}| "
        "?[^\\s\\p{L}\\p{N}]+[\\r\\n]*|\\s*[\\r\\n]+|\\s+(?!\\S)|\\s+";
    if (p.get_string("type") == "Sequence") {
      const Json& v = p.get("pretokenizers");
      if (v.size() != 2) throw std::runtime_error("pre-tokenizer sequence not covered");
      const Json& sp = v.at(0);
      const Json& bl = v.at(1);
      if (sp.get_string("type") != "Split" || sp.get("pattern").get_string("Regex") != kL3 ||
          sp.get_string("behavior") != "Isolated" || sp.get_bool("invert", false))
        throw std::runtime_error("split pattern not covered");
      if (bl.get_string("type") != "ByteLevel" || bl.get_bool("add_prefix_space", false) ||
          bl.get_bool("use_regex", true))
        throw std::runtime_error("byte-level options not covered");
      pat_ = kLlama3;
      return;
    }
    if (p.get_string("type") == "ByteLevel" && p.get_bool("use_regex", true) &&
        !p.get_bool("add_prefix_space", false)) {
      pat_ = kGpt2;
      return;
    }
    throw std::runtime_error("pre-tokenizer not covered");
  }

  const Added* added_at(const std::string& s, size_t i) const {
    if (!first_[(unsigned char)s[i]]) return nullptr;
    for (auto& a : added_)  // longest first
      if (s.compare(i, a.text.size(), a.text) == 0) return &a;
    return nullptr;
  }

  // end (exclusive) of the pattern's match at code point i, 0 if none matches there
  size_t match(const std::vector<uint32_t>& c, size_t i) const {
    const size_t n = c.size();
    auto L = [&](size_t k) { return k < n && uni::letter(c[k]); };
    auto N = [&](size_t k) { return k < n && uni::number(c[k]); };
    auto S = [&](size_t k) { return k < n && uni::space(c[k]); };
    auto other = [&](size_t k) { return k < n && !uni::space(c[k]) && !uni::letter(c[k]) && !uni::number(c[k]); };
    auto nl = [&](size_t k) { return k < n && (c[k] == '\r' || c[k] == '\n'); };
    const bool ci = pat_ == kLlama3;  // (?i:...) contractions
    auto low = [&](size_t k) -> uint32_t {
      if (k >= n) return 0;
      uint32_t x = c[k];
      if (ci) {
        if (x >= 'A' && x <= 'Z') x += 32;
        if (x == 0x17F) x = 's';  // LATIN SMALL LETTER LONG S case-folds to s
      }
      return x;
    };
    // 's|'t|'re|'ve|'m|'ll|'d
    if (c[i] == '\'') {
      const uint32_t a = low(i + 1);
      if (a == 's' || a == 't' || a == 'm' || a == 'd') return i + 2;
      if ((a == 'r' || a == 'v') && low(i + 2) == 'e') return i + 3;
      if (a == 'l' && low(i + 2) == 'l') return i + 3;
    }
    if (pat_ == kLlama3) {
      // [^\r\n\p{L}\p{N}]?\p{L}+
      size_t k = i;
      if (!L(i) && !N(i) && !nl(i) && L(i + 1)) k = i + 1;
      if (L(k)) {
        while (L(k)) ++k;
        return k;
      }
      // \p{N}{1,3}
      if (N(i)) {
        k = i;
        while (k < i + 3 && N(k)) ++k;
        return k;
      }
      // ' ?[^\s\p{L}\p{N}]+[\r\n]*'
      k = i;
      if (c[i] == ' ' && other(i + 1)) k = i + 1;
      if (other(k)) {
        while (other(k)) ++k;
        while (nl(k)) ++k;
        return k;
      }
      // \s*[\r\n]+ : up to the last line break of the whitespace run
      if (S(i)) {
        size_t j = i;
        while (S(j)) ++j;
        size_t p = j;
        while (p > i && !nl(p - 1)) --p;
        if (p > i) return p;
      }
    } else {
      // ' ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+'
      const size_t k = (c[i] == ' ' && i + 1 < n) ? i + 1 : i;
      for (int cls = 0; cls < 3; ++cls) {
        auto in = [&](size_t x) { return cls == 0 ? L(x) : cls == 1 ? N(x) : other(x); };
        size_t e = in(k) ? k : (in(i) ? i : n + 1);
        if (e == n + 1) continue;
        while (in(e)) ++e;
        return e;
      }
    }
    // \s+(?!\S) | \s+
    if (S(i)) {
      size_t j = i;
      while (S(j)) ++j;
      if (j == n) return j;
      if (j - i >= 2) return j - 1;
      return j;
    }
    return 0;
  }

  bool encode_plain(const std::string& text, std::vector<int>* out) const {
    if (text.empty()) return true;
    std::vector<uint32_t> cps;
    std::vector<size_t> offs;
    if (!uni::utf8_decode(text, &cps, &offs)) return false;
    size_t i = 0, gap = 0;
    const size_t n = cps.size();
    while (i < n) {
      const size_t e = match(cps, i);
      if (e == 0) {  // no match here: part of a gap piece (Isolated keeps it)
        ++i;
        continue;
      }
      if (gap < i && !bpe_piece(text.substr(offs[gap], offs[i] - offs[gap]), out)) return false;
      if (!bpe_piece(text.substr(offs[i], offs[e] - offs[i]), out)) return false;
      i = gap = e;
    }
    if (gap < n && !bpe_piece(text.substr(offs[gap]), out)) return false;
    return true;
  }

  bool bpe_piece(const std::string& piece, std::vector<int>* out) const {
    std::string mapped;
    for (unsigned char b : piece) mapped += byte_char_[b];
    if (ignore_merges_) {
      auto it = vocab_.find(mapped);
      if (it != vocab_.end()) {
        out->push_back(it->second);
        return true;
      }
    }
    struct Sym {
      int id, prev, next;
    };
    std::vector<Sym> sy;
    for (size_t k = 0; k < piece.size(); ++k) {
      auto it = vocab_.find(byte_char_[(unsigned char)piece[k]]);
      if (it == vocab_.end()) return false;
      sy.push_back({it->second, (int)k - 1, k + 1 < piece.size() ? (int)k + 1 : -1});
    }
    // (rank, position) min-heap of candidate merges; stale entries are skipped on pop
    struct Cand {
      int rank, pos, left, right, merged;
      bool operator>(const Cand& o) const { return rank != o.rank ? rank > o.rank : pos > o.pos; }
    };
    std::priority_queue<Cand, std::vector<Cand>, std::greater<Cand>> heap;
    auto push = [&](int p) {
      if (p < 0 || sy[p].next < 0) return;
      auto it = merges_.find(key(sy[p].id, sy[sy[p].next].id));
      if (it != merges_.end()) heap.push({it->second.first, p, sy[p].id, sy[sy[p].next].id, it->second.second});
    };
    for (int p = 0; p < (int)sy.size(); ++p) push(p);
    while (!heap.empty()) {
      const Cand cd = heap.top();
      heap.pop();
      Sym& a = sy[cd.pos];
      if (a.id != cd.left || a.next < 0 || sy[a.next].id != cd.right) continue;  // stale
      const int b = a.next;
      a.id = cd.merged;
      a.next = sy[b].next;
      if (a.next >= 0) sy[a.next].prev = cd.pos;
      sy[b].id = -1;  // removed
      push(a.prev);
      push(cd.pos);
    }
    for (int p = 0; p >= 0; p = sy[p].next) out->push_back(sy[p].id);
    return true;
  }

  bool ok_ = false;
  bool ignore_merges_ = false;
  Pattern pat_ = kLlama3;
  std::string byte_char_[256];
  std::unordered_map<uint32_t, uint8_t> char_byte_;
  std::unordered_map<std::string, int> vocab_;
  std::vector<std::string> id_str_;
  std::unordered_map<uint64_t, std::pair<int, int>> merges_;
  std::vector<Added> added_;
  std::unordered_map<int, size_t> added_id_;
  bool first_[256] = {};  // first bytes of the added tokens
};

}  // namespace p2p
