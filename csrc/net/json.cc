#include "json.h"

#include <math.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <stdexcept>

namespace p2p {

static const Json kNull;

const std::string& Json::str() const {
  if (t_ != String) throw JsonError("json: not a string");
  return s_;
}
double Json::num() const {
  if (t_ != Number) throw JsonError("json: not a number");
  return n_;
}
long long Json::integer() const {
  if (t_ != Number) throw JsonError("json: not a number");
  return is_int_ ? i_ : (long long)n_;
}
bool Json::boolean() const {
  if (t_ != Bool) throw JsonError("json: not a bool");
  return b_;
}
void Json::push(Json v) {
  if (t_ == Null) t_ = Array;
  if (t_ != Array) throw JsonError("json: not an array");
  arr_.push_back(std::move(v));
}
size_t Json::size() const { return t_ == Array ? arr_.size() : (t_ == Object ? obj_.size() : 0); }
const Json& Json::at(size_t i) const {
  if (t_ != Array || i >= arr_.size()) throw JsonError("json: bad index");
  return arr_[i];
}
Json& Json::set(const std::string& k, Json v) {
  if (t_ == Null) t_ = Object;
  if (t_ != Object) throw JsonError("json: not an object");
  for (auto& kv : obj_)
    if (kv.first == k) {
      kv.second = std::move(v);
      return kv.second;
    }
  obj_.emplace_back(k, std::move(v));
  return obj_.back().second;
}
bool Json::has(const std::string& k) const {
  if (t_ != Object) return false;
  for (auto& kv : obj_)
    if (kv.first == k) return true;
  return false;
}
const Json& Json::get(const std::string& k) const {
  if (t_ != Object) return kNull;
  // last occurrence wins (like Go's decoder)
  for (auto it = obj_.rbegin(); it != obj_.rend(); ++it)
    if (it->first == k) return it->second;
  return kNull;
}
std::string Json::get_string(const std::string& k, const std::string& def) const {
  const Json& v = get(k);
  return v.is_string() ? v.s_ : def;
}
double Json::get_number(const std::string& k, double def) const {
  const Json& v = get(k);
  return v.is_number() ? v.n_ : def;
}
bool Json::get_bool(const std::string& k, bool def) const {
  const Json& v = get(k);
  return v.is_bool() ? v.b_ : def;
}

std::string json_escape(const std::string& s) {
  std::string out;
  out.reserve(s.size() + 2);
  out += '"';
  for (size_t i = 0; i < s.size(); ++i) {
    unsigned char c = (unsigned char)s[i];
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      case '<': out += "\\u003c"; break;
      case '>': out += "\\u003e"; break;
      case '&': out += "\\u0026"; break;
      default:
        if (c < 0x20) {
          char b[8];
          snprintf(b, sizeof(b), "\\u%04x", c);
          out += b;
        } else if (c == 0xE2 && i + 2 < s.size() && (unsigned char)s[i + 1] == 0x80 &&
                   ((unsigned char)s[i + 2] == 0xA8 || (unsigned char)s[i + 2] == 0xA9)) {
          out += ((unsigned char)s[i + 2] == 0xA8) ? "\\u2028" : "\\u2029";
          i += 2;
        } else {
          out += (char)c;
        }
    }
  }
  out += '"';
  return out;
}

void Json::dump_to(std::string& out, bool sorted) const {
  switch (t_) {
    case Null: out += "null"; break;
    case Bool: out += b_ ? "true" : "false"; break;
    case Number: {
      char b[64];
      if (is_int_) {
        snprintf(b, sizeof(b), "%lld", i_);
      } else if (std::isfinite(n_) && n_ == floor(n_) && fabs(n_) < 1e15) {
        snprintf(b, sizeof(b), "%.0f", n_);
      } else {
        snprintf(b, sizeof(b), "%.17g", n_);
      }
      out += b;
      break;
    }
    case String: out += json_escape(s_); break;
    case Array:
      out += '[';
      for (size_t i = 0; i < arr_.size(); ++i) {
        if (i) out += ',';
        arr_[i].dump_to(out, sorted);
      }
      out += ']';
      break;
    case Object: {
      out += '{';
      std::vector<const std::pair<std::string, Json>*> kv;
      for (auto& p : obj_) kv.push_back(&p);
      if (sorted)
        std::stable_sort(kv.begin(), kv.end(), [](auto a, auto b) { return a->first < b->first; });
      for (size_t i = 0; i < kv.size(); ++i) {
        if (i) out += ',';
        out += json_escape(kv[i]->first);
        out += ':';
        kv[i]->second.dump_to(out, sorted);
      }
      out += '}';
      break;
    }
  }
}

std::string Json::dump() const {
  std::string s;
  dump_to(s, false);
  return s;
}
std::string Json::dump_sorted() const {
  std::string s;
  dump_to(s, true);
  return s;
}

namespace {
struct Parser {
  const std::string& s;
  size_t i = 0;
  int depth = 0;
  explicit Parser(const std::string& t) : s(t) {}
  [[noreturn]] void fail(const char* m) {
    char b[160];
    snprintf(b, sizeof(b), "json: %s at offset %zu", m, i);
    throw JsonError(b);
  }
  // Go encoding/json wording for the common syntax errors (gin BindJSON bodies).
  [[noreturn]] void fail_char(const char* ctx) {
    if (i >= s.size()) throw JsonError("unexpected EOF");
    char b[160];
    char c = s[i];
    if (c == '\'') snprintf(b, sizeof(b), "invalid character '\\'' %s", ctx);
    else if ((unsigned char)c < 0x20) snprintf(b, sizeof(b), "invalid character '\\x%02x' %s", (unsigned char)c, ctx);
    else snprintf(b, sizeof(b), "invalid character '%c' %s", c, ctx);
    throw JsonError(b);
  }
  void ws() {
    while (i < s.size() && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) ++i;
  }
  static void put_utf8(std::string& o, unsigned cp) {
    if (cp < 0x80) {
      o += (char)cp;
    } else if (cp < 0x800) {
      o += (char)(0xC0 | (cp >> 6));
      o += (char)(0x80 | (cp & 0x3F));
    } else if (cp < 0x10000) {
      o += (char)(0xE0 | (cp >> 12));
      o += (char)(0x80 | ((cp >> 6) & 0x3F));
      o += (char)(0x80 | (cp & 0x3F));
    } else {
      o += (char)(0xF0 | (cp >> 18));
      o += (char)(0x80 | ((cp >> 12) & 0x3F));
      o += (char)(0x80 | ((cp >> 6) & 0x3F));
      o += (char)(0x80 | (cp & 0x3F));
    }
  }
  unsigned hex4() {
    if (i + 4 > s.size()) fail("bad \\u escape");
    unsigned v = 0;
    for (int k = 0; k < 4; ++k) {
      char c = s[i++];
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else fail("bad hex digit");
    }
    return v;
  }
  std::string str() {
    if (s[i] != '"') fail("expected string");
    ++i;
    std::string o;
    while (true) {
      if (i >= s.size()) fail("unterminated string");
      char c = s[i++];
      if (c == '"') break;
      if ((unsigned char)c < 0x20) fail("control character in string");
      if (c != '\\') {
        o += c;
        continue;
      }
      if (i >= s.size()) fail("bad escape");
      char e = s[i++];
      switch (e) {
        case '"': o += '"'; break;
        case '\\': o += '\\'; break;
        case '/': o += '/'; break;
        case 'b': o += '\b'; break;
        case 'f': o += '\f'; break;
        case 'n': o += '\n'; break;
        case 'r': o += '\r'; break;
        case 't': o += '\t'; break;
        case 'u': {
          unsigned cp = hex4();
          if (cp >= 0xD800 && cp < 0xDC00 && i + 6 <= s.size() && s[i] == '\\' && s[i + 1] == 'u') {
            i += 2;
            unsigned lo = hex4();
            if (lo >= 0xDC00 && lo < 0xE000) cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            else cp = 0xFFFD;
          } else if (cp >= 0xD800 && cp < 0xE000) {
            cp = 0xFFFD;
          }
          put_utf8(o, cp);
          break;
        }
        default: fail("bad escape");
      }
    }
    return o;
  }
  Json value() {
    ws();
    if (i >= s.size()) throw JsonError("unexpected end of JSON input");
    if (++depth > 512) fail("nesting too deep");
    Json out;
    char c = s[i];
    if (c == '{') {
      ++i;
      out = Json::object();
      ws();
      if (i < s.size() && s[i] == '}') {
        ++i;
      } else {
        while (true) {
          ws();
          if (i >= s.size()) fail("unexpected end");
          std::string k = str();
          ws();
          if (i >= s.size() || s[i] != ':') fail("expected ':'");
          ++i;
          Json v = value();
          out.set(k, std::move(v));
          ws();
          if (i < s.size() && s[i] == ',') { ++i; continue; }
          if (i < s.size() && s[i] == '}') { ++i; break; }
          fail("expected ',' or '}'");
        }
      }
    } else if (c == '[') {
      ++i;
      out = Json::array();
      ws();
      if (i < s.size() && s[i] == ']') {
        ++i;
      } else {
        while (true) {
          out.push(value());
          ws();
          if (i < s.size() && s[i] == ',') { ++i; continue; }
          if (i < s.size() && s[i] == ']') { ++i; break; }
          fail("expected ',' or ']'");
        }
      }
    } else if (c == '"') {
      out = Json(str());
    } else if (s.compare(i, 4, "true") == 0) {
      i += 4;
      out = Json(true);
    } else if (s.compare(i, 5, "false") == 0) {
      i += 5;
      out = Json(false);
    } else if (s.compare(i, 4, "null") == 0) {
      i += 4;
    } else if (c == '-' || (c >= '0' && c <= '9')) {
      size_t st = i;
      bool isint = true;
      if (s[i] == '-') ++i;
      while (i < s.size() && isdigit((unsigned char)s[i])) ++i;
      if (i < s.size() && s[i] == '.') {
        isint = false;
        ++i;
        while (i < s.size() && isdigit((unsigned char)s[i])) ++i;
      }
      if (i < s.size() && (s[i] == 'e' || s[i] == 'E')) {
        isint = false;
        ++i;
        if (i < s.size() && (s[i] == '+' || s[i] == '-')) ++i;
        while (i < s.size() && isdigit((unsigned char)s[i])) ++i;
      }
      std::string num = s.substr(st, i - st);
      if (num == "-" || num.empty()) fail("bad number");
      if (isint && num.size() < 18) out = Json((long long)strtoll(num.c_str(), nullptr, 10));
      else out = Json(strtod(num.c_str(), nullptr));
    } else {
      fail_char("looking for beginning of value");
    }
    --depth;
    return out;
  }
};
}  // namespace

Json Json::parse(const std::string& text) {
  Parser p(text);
  Json v = p.value();
  p.ws();
  if (p.i != text.size()) p.fail_char("after top-level value");
  return v;
}

}  // namespace p2p
