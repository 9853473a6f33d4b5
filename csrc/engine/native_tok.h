// Native form of the engine's tokenizers (engine/tokenizer.py: SyntheticTokenizer, and
// HFTokenizer over a byte-level BPE tokenizer.json such as Llama-3's, bpe_tok.h) and of the
// Ollama prompt templates, so the engine C ABI turns a request into prompt ids and
// generated ids into text without the interpreter.
//
// Encoding splits text with the pattern  \s*\w+ | \s*[^\w\s] | \s+  and maps each piece to
// lo + crc32(piece) % (hi - lo), exactly as the Python class does; the native side handles
// printable ASCII (plus \t \n \r) and reports anything else as "not native", in which case
// the caller asks Python (Unicode \w / \s classes are not re-implemented here).  Decoding
// uses the built-in table exported by Python (`native_spec`) and recomputes the
// pseudo-words of other ids.  A "bpe" spec (HFTokenizer.native_spec) names the
// tokenizer.json; encoding and decoding then follow the HF library exactly (bpe_tok.h),
// for any UTF-8 text.
#pragma once
#include <stdint.h>

#include <map>
#include <memory>
#include <string>
#include <vector>

#include "engine/bpe_tok.h"
#include "net/json.h"

namespace p2p {

class NativeTok {
 public:
  bool ok = false;  // a spec this class implements was loaded
  bool llama3 = false;
  int lo = 3, hi = 0, bos = 1;
  std::vector<int> eos;
  std::map<std::string, int> special;
  std::map<int, std::string> pieces;
  std::shared_ptr<BpeTok> bpe;  // "bpe" specs

  // spec: SyntheticTokenizer / HFTokenizer .native_spec() as JSON; anything else (or a
  // tokenizer.json with parts bpe_tok.h does not cover: it throws) leaves ok = false
  void load(const std::string& spec_json) {
    Json s = Json::parse(spec_json);
    if (s.get_string("kind") == "bpe") {
      auto b = std::make_shared<BpeTok>();
      b->load_file(s.get_string("path"));
      llama3 = s.get_bool("llama3", false);
      bos = (int)s.get("bos").integer();
      for (auto& e : s.get("eos").items()) eos.push_back((int)e.integer());
      for (auto& kv : s.get("special").fields()) special[kv.first] = (int)kv.second.integer();
      bpe = b;
      ok = true;
      return;
    }
    if (s.get_string("kind") != "synthetic") return;
    llama3 = s.get_bool("llama3", false);
    lo = (int)s.get("lo").integer();
    hi = (int)s.get("hi").integer();
    bos = (int)s.get("bos").integer();
    for (auto& e : s.get("eos").items()) eos.push_back((int)e.integer());
    for (auto& kv : s.get("special").fields()) special[kv.first] = (int)kv.second.integer();
    for (auto& p : s.get("pieces").items()) pieces[(int)p.at(0).integer()] = p.at(1).str();
    ok = hi > lo;
  }

  static bool ascii_text(const std::string& t) {
    for (unsigned char c : t)
      if (!((c >= 0x20 && c < 0x7f) || c == '\t' || c == '\n' || c == '\r')) return false;
    return true;
  }

  static uint32_t crc32(const std::string& s) {
    static uint32_t table[256];
    static bool init = [] {
      for (uint32_t i = 0; i < 256; ++i) {
        uint32_t c = i;
        for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
        table[i] = c;
      }
      return true;
    }();
    (void)init;
    uint32_t c = 0xFFFFFFFFu;
    for (unsigned char b : s) c = table[(c ^ b) & 0xFF] ^ (c >> 8);
    return c ^ 0xFFFFFFFFu;
  }

  // false if the text needs Python (synthetic: non-ASCII; bpe: not UTF-8)
  bool encode(const std::string& t, std::vector<int>* out) const {
    if (bpe) return bpe->encode(t, out);
    if (!ascii_text(t)) return false;
    auto sp = [](unsigned char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; };
    auto wd = [](unsigned char c) { return isalnum(c) || c == '_'; };
    const size_t n = t.size();
    size_t i = 0;
    while (i < n) {
      size_t j = i;
      while (j < n && sp((unsigned char)t[j])) ++j;
      size_t e;
      if (j < n && wd((unsigned char)t[j])) {
        e = j;
        while (e < n && wd((unsigned char)t[e])) ++e;
      } else if (j < n) {
        e = j + 1;  // one punctuation mark after the whitespace
      } else {
        e = j;  // trailing whitespace
      }
      out->push_back(lo + (int)(crc32(t.substr(i, e - i)) % (uint32_t)(hi - lo)));
      i = e;
    }
    return true;
  }

  int sp_id(const char* name) const {
    auto it = special.find(name);
    return it == special.end() ? -1 : it->second;
  }

  // SyntheticTokenizer.chat_ids: one user turn, the assistant header open
  bool chat_ids(const std::string& user, std::vector<int>* ids) const {
    if (llama3) {
      ids->push_back(sp_id("<|begin_of_text|>"));
      ids->push_back(sp_id("<|start_header_id|>"));
      if (!encode("user", ids)) return false;
      ids->push_back(sp_id("<|end_header_id|>"));
      if (!encode("\n\n" + user, ids)) return false;
      ids->push_back(sp_id("<|eot_id|>"));
      ids->push_back(sp_id("<|start_header_id|>"));
      if (!encode("assistant", ids)) return false;
      ids->push_back(sp_id("<|end_header_id|>"));
      return encode("\n\n", ids);
    }
    ids->push_back(bos);
    return encode("[INST] " + user + " [/INST]", ids);
  }

  // tokenizer._render_messages (Ollama /api/chat); false if a message is not plain strings
  // (an explicit null role / content included: Python renders str(None) = "None"; only a
  // missing key takes the default)
  bool messages_ids(const Json& msgs, std::vector<int>* ids) const {
    if (!msgs.is_null() && !msgs.is_array()) return false;
    std::vector<std::pair<std::string, std::string>> ms;
    for (auto& m : msgs.items()) {
      if (!m.is_object()) continue;
      const bool hr = m.has("role"), hc = m.has("content");
      const Json& r = m.get("role");
      const Json& c = m.get("content");
      if ((hr && !r.is_string()) || (hc && !c.is_string())) return false;
      ms.emplace_back(hr ? r.str() : "user", hc ? c.str() : "");
    }
    ids->push_back(bos);
    if (llama3) {
      for (auto& m : ms) {
        ids->push_back(sp_id("<|start_header_id|>"));
        if (!encode(m.first, ids)) return false;
        ids->push_back(sp_id("<|end_header_id|>"));
        if (!encode("\n\n" + m.second, ids)) return false;
        ids->push_back(sp_id("<|eot_id|>"));
      }
      ids->push_back(sp_id("<|start_header_id|>"));
      if (!encode("assistant", ids)) return false;
      ids->push_back(sp_id("<|end_header_id|>"));
      return encode("\n\n", ids);
    }
    // "\n\n".join of every system content (empty ones included, as in Python)
    std::string system;
    bool first = true;
    for (auto& m : ms)
      if (m.first == "system") {
        system += (first ? "" : "\n\n") + m.second;
        first = false;
      }
    for (auto& m : ms) {
      if (m.first == "system") continue;
      if (m.first == "assistant") {
        if (!encode(" " + m.second, ids)) return false;
        if (!eos.empty()) ids->push_back(eos[0]);
        continue;
      }
      std::string content = m.second;
      if (!system.empty()) {
        content = system + "\n\n" + content;
        system.clear();
      }
      if (!encode("[INST] " + content + " [/INST]", ids)) return false;
    }
    return true;
  }

  static std::string pseudo(int64_t i) {
    static const char* cons = "bdfgklmnprstvz";
    static const char* vows = "aeiou";
    std::string out = " ";
    int64_t n = i;
    while (true) {
      out += cons[n % 14];
      out += vows[(n / 14) % 5];
      n /= 70;
      if (n == 0) break;
    }
    return out;
  }

  // HFTokenizer.decode: tokenizers' decode, then Python's str.strip()
  static std::string py_strip(const std::string& s) {
    std::vector<uint32_t> cps;
    std::vector<size_t> offs;
    if (!uni::utf8_decode(s, &cps, &offs)) return s;
    size_t a = 0, b = cps.size();
    while (a < b && uni::py_space(cps[a])) ++a;
    while (b > a && uni::py_space(cps[b - 1])) --b;
    return s.substr(offs[a], offs[b] - offs[a]);
  }

  std::string decode(const std::vector<int>& ids) const {
    if (bpe) return py_strip(bpe->decode(ids));
    std::string out;
    for (int i : ids) {
      bool skip = i == bos;
      for (int e : eos) skip = skip || i == e;
      if (llama3)
        for (auto& kv : special) skip = skip || i == kv.second;
      if (skip) continue;
      auto it = pieces.find(i);
      out += it != pieces.end() ? it->second : pseudo(i);
    }
    const char* ws = " \t\n\r\v\f";
    const size_t a = out.find_first_not_of(ws);
    if (a == std::string::npos) return "";
    return out.substr(a, out.find_last_not_of(ws) - a + 1);
  }
};

}  // namespace p2p
