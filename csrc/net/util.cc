#include "util.h"

#include <openssl/rand.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <stdarg.h>

#include <algorithm>
#include <atomic>
#include <mutex>

namespace p2p {

void put_uvarint(Bytes& out, uint64_t v) {
  while (v >= 0x80) {
    out.push_back((uint8_t)(v | 0x80));
    v >>= 7;
  }
  out.push_back((uint8_t)v);
}

Bytes uvarint(uint64_t v) {
  Bytes b;
  put_uvarint(b, v);
  return b;
}

uint64_t get_uvarint(const uint8_t* data, size_t len, size_t* pos) {
  uint64_t v = 0;
  int shift = 0;
  for (int i = 0; i < 10; ++i) {
    if (*pos >= len) throw NetError("varint: truncated");
    uint8_t b = data[(*pos)++];
    v |= (uint64_t)(b & 0x7f) << shift;
    if (!(b & 0x80)) return v;
    shift += 7;
  }
  throw NetError("varint: overflow");
}

int peek_uvarint(const uint8_t* data, size_t len, uint64_t* v) {
  uint64_t x = 0;
  int shift = 0;
  for (size_t i = 0; i < len && i < 10; ++i) {
    x |= (uint64_t)(data[i] & 0x7f) << shift;
    if (!(data[i] & 0x80)) {
      *v = x;
      return (int)i + 1;
    }
    shift += 7;
  }
  if (len >= 10) throw NetError("varint: overflow");
  return -1;
}

static const char* kB58 = "123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz";

std::string base58_encode(const Bytes& in) {
  size_t zeros = 0;
  while (zeros < in.size() && in[zeros] == 0) ++zeros;
  std::vector<uint8_t> b58((in.size() - zeros) * 138 / 100 + 1, 0);
  size_t length = 0;
  for (size_t i = zeros; i < in.size(); ++i) {
    int carry = in[i];
    size_t j = 0;
    for (auto it = b58.rbegin(); (carry != 0 || j < length) && it != b58.rend(); ++it, ++j) {
      carry += 256 * (*it);
      *it = carry % 58;
      carry /= 58;
    }
    length = j;
  }
  auto it = b58.begin() + (b58.size() - length);
  while (it != b58.end() && *it == 0) ++it;
  std::string out(zeros, '1');
  for (; it != b58.end(); ++it) out += kB58[*it];
  return out;
}

Bytes base58_decode(const std::string& s) {
  int8_t map[256];
  memset(map, -1, sizeof(map));
  for (int i = 0; i < 58; ++i) map[(uint8_t)kB58[i]] = (int8_t)i;
  size_t zeros = 0;
  while (zeros < s.size() && s[zeros] == '1') ++zeros;
  std::vector<uint8_t> b256((s.size() - zeros) * 733 / 1000 + 1, 0);
  size_t length = 0;
  for (size_t i = zeros; i < s.size(); ++i) {
    int carry = map[(uint8_t)s[i]];
    if (carry < 0) throw NetError("base58: bad character");
    size_t j = 0;
    for (auto it = b256.rbegin(); (carry != 0 || j < length) && it != b256.rend(); ++it, ++j) {
      carry += 58 * (*it);
      *it = carry % 256;
      carry /= 256;
    }
    length = j;
  }
  auto it = b256.begin() + (b256.size() - length);
  while (it != b256.end() && *it == 0) ++it;
  Bytes out(zeros, 0);
  out.insert(out.end(), it, b256.end());
  return out;
}

std::string hex_encode(const Bytes& in) {
  static const char* h = "0123456789abcdef";
  std::string s;
  s.reserve(in.size() * 2);
  for (uint8_t b : in) {
    s += h[b >> 4];
    s += h[b & 15];
  }
  return s;
}

Bytes hex_decode(const std::string& s) {
  if (s.size() % 2) throw NetError("hex: odd length");
  auto nib = [](char c) -> int {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    throw NetError("hex: bad char");
  };
  Bytes out(s.size() / 2);
  for (size_t i = 0; i < out.size(); ++i) out[i] = (uint8_t)(nib(s[2 * i]) << 4 | nib(s[2 * i + 1]));
  return out;
}

std::vector<PbField> pb_parse(const uint8_t* data, size_t len) {
  std::vector<PbField> out;
  size_t pos = 0;
  while (pos < len) {
    uint64_t key = get_uvarint(data, len, &pos);
    PbField f;
    f.field = (uint32_t)(key >> 3);
    f.wire = (uint32_t)(key & 7);
    switch (f.wire) {
      case 0:
        f.varint = get_uvarint(data, len, &pos);
        break;
      case 1:
        if (pos + 8 > len) throw NetError("pb: truncated fixed64");
        memcpy(&f.varint, data + pos, 8);
        pos += 8;
        break;
      case 2: {
        uint64_t n = get_uvarint(data, len, &pos);
        if (n > len - pos) throw NetError("pb: truncated bytes");
        f.bytes.assign(data + pos, data + pos + n);
        pos += n;
        break;
      }
      case 5: {
        if (pos + 4 > len) throw NetError("pb: truncated fixed32");
        uint32_t v;
        memcpy(&v, data + pos, 4);
        f.varint = v;
        pos += 4;
        break;
      }
      default:
        throw NetError("pb: unsupported wire type");
    }
    out.push_back(std::move(f));
  }
  return out;
}

std::string rfc3339_now_local() {
  auto now = std::chrono::system_clock::now();
  auto us = std::chrono::duration_cast<std::chrono::microseconds>(now.time_since_epoch()).count();
  time_t secs = (time_t)(us / 1000000);
  long frac = (long)(us % 1000000);
  struct tm lt;
  localtime_r(&secs, &lt);
  char buf[64];
  strftime(buf, sizeof(buf), "%Y-%m-%dT%H:%M:%S", &lt);
  long off = lt.tm_gmtoff;
  char tz[16];
  if (off == 0) {
    snprintf(tz, sizeof(tz), "Z");
  } else {
    char sign = off < 0 ? '-' : '+';
    off = off < 0 ? -off : off;
    snprintf(tz, sizeof(tz), "%c%02ld:%02ld", sign, off / 3600, (off % 3600) / 60);
  }
  char out[96];
  snprintf(out, sizeof(out), "%s.%06ld%s", buf, frac, tz);
  return out;
}

double parse_rfc3339(const std::string& s) {
  int Y, M, D, h, m, sec;
  if (s.size() < 19 || sscanf(s.c_str(), "%4d-%2d-%2dT%2d:%2d:%2d", &Y, &M, &D, &h, &m, &sec) != 6)
    throw NetError("bad RFC3339 timestamp");
  size_t i = 19;
  double frac = 0;
  if (i < s.size() && s[i] == '.') {
    ++i;
    double scale = 0.1;
    while (i < s.size() && isdigit((unsigned char)s[i])) {
      frac += (s[i] - '0') * scale;
      scale /= 10;
      ++i;
    }
  }
  long off = 0;
  if (i < s.size()) {
    if (s[i] == 'Z' || s[i] == 'z') {
      off = 0;
    } else if (s[i] == '+' || s[i] == '-') {
      int oh = 0, om = 0;
      if (sscanf(s.c_str() + i + 1, "%2d:%2d", &oh, &om) != 2) throw NetError("bad tz offset");
      off = (oh * 3600 + om * 60) * (s[i] == '-' ? -1 : 1);
    } else {
      throw NetError("bad RFC3339 suffix");
    }
  }
  struct tm t = {};
  t.tm_year = Y - 1900;
  t.tm_mon = M - 1;
  t.tm_mday = D;
  t.tm_hour = h;
  t.tm_min = m;
  t.tm_sec = sec;
  time_t utc = timegm(&t);
  return (double)(utc - off) + frac;
}

int64_t unix_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(
             std::chrono::system_clock::now().time_since_epoch())
      .count();
}

std::string uuid4() {
  uint8_t b[16];
  if (RAND_bytes(b, 16) != 1) throw NetError("RAND_bytes failed");
  b[6] = (b[6] & 0x0f) | 0x40;
  b[8] = (b[8] & 0x3f) | 0x80;
  char out[40];
  snprintf(out, sizeof(out),
           "%02x%02x%02x%02x-%02x%02x-%02x%02x-%02x%02x-%02x%02x%02x%02x%02x%02x", b[0], b[1],
           b[2], b[3], b[4], b[5], b[6], b[7], b[8], b[9], b[10], b[11], b[12], b[13], b[14], b[15]);
  return out;
}

static std::atomic<bool> g_quiet{false};
static std::mutex g_log_mu;

void set_log_quiet(bool q) { g_quiet = q; }

void logf(const char* fmt, ...) {
  if (g_quiet) return;
  char msg[4096];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(msg, sizeof(msg), fmt, ap);
  va_end(ap);
  time_t now = time(nullptr);
  struct tm lt;
  localtime_r(&now, &lt);
  char ts[32];
  strftime(ts, sizeof(ts), "%Y/%m/%d %H:%M:%S", &lt);
  std::lock_guard<std::mutex> lk(g_log_mu);
  size_t n = strlen(msg);
  fprintf(stderr, "%s %s%s", ts, msg, (n && msg[n - 1] == '\n') ? "" : "\n");
  fflush(stderr);
}

std::string env_or(const char* key, const std::string& def) {
  const char* v = getenv(key);
  if (v && *v) return v;
  return def;
}

}  // namespace p2p
