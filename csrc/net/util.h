// Byte utilities for the native libp2p subset: unsigned varint (multiformats),
// base58btc, hex, minimal protobuf wire encoding, time formatting.
#pragma once
#include <stdint.h>

#include <chrono>
#include <stdexcept>
#include <string>
#include <vector>

namespace p2p {

using Bytes = std::vector<uint8_t>;

struct NetError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

inline Bytes to_bytes(const std::string& s) { return Bytes(s.begin(), s.end()); }
inline std::string to_string(const Bytes& b) { return std::string(b.begin(), b.end()); }
inline void append(Bytes& a, const Bytes& b) { a.insert(a.end(), b.begin(), b.end()); }
inline void append(Bytes& a, const std::string& b) { a.insert(a.end(), b.begin(), b.end()); }

// ---- unsigned varint (LEB128, max 9 bytes for multiformats) ----
void put_uvarint(Bytes& out, uint64_t v);
Bytes uvarint(uint64_t v);
// Decodes at data[*pos]; advances *pos.  Throws NetError on truncation/overflow.
uint64_t get_uvarint(const uint8_t* data, size_t len, size_t* pos);
inline uint64_t get_uvarint(const Bytes& b, size_t* pos) { return get_uvarint(b.data(), b.size(), pos); }
// Returns -1 if incomplete, else the number of bytes of the varint.
int peek_uvarint(const uint8_t* data, size_t len, uint64_t* v);

// ---- base58btc / hex / base64 ----
std::string base58_encode(const Bytes& in);
Bytes base58_decode(const std::string& s);  // throws NetError
std::string hex_encode(const Bytes& in);
Bytes hex_decode(const std::string& s);

// ---- protobuf wire helpers (proto2/proto3 subset used by libp2p) ----
struct PbWriter {
  Bytes buf;
  void varint_field(uint32_t field, uint64_t v) {
    put_uvarint(buf, (uint64_t)field << 3 | 0);
    put_uvarint(buf, v);
  }
  void bytes_field(uint32_t field, const Bytes& v) {
    put_uvarint(buf, (uint64_t)field << 3 | 2);
    put_uvarint(buf, v.size());
    append(buf, v);
  }
  void bytes_field(uint32_t field, const std::string& v) { bytes_field(field, to_bytes(v)); }
};

struct PbField {
  uint32_t field = 0;
  uint32_t wire = 0;
  uint64_t varint = 0;
  Bytes bytes;
};

// Parses all fields of a message (varint, 64-bit, length-delimited, 32-bit).
std::vector<PbField> pb_parse(const uint8_t* data, size_t len);
inline std::vector<PbField> pb_parse(const Bytes& b) { return pb_parse(b.data(), b.size()); }

// ---- time ----
// RFC3339 with microseconds and the local UTC offset, e.g. 2025-09-02T21:11:32.154084+02:00
// (Go's time.Time JSON is RFC3339Nano; microseconds keep Python 3.10 fromisoformat happy).
std::string rfc3339_now_local();
// Parses any RFC3339 timestamp (0-9 fractional digits, Z or +hh:mm); returns unix seconds.
double parse_rfc3339(const std::string& s);
int64_t unix_ms();

std::string uuid4();
// Go `log` package format: "2006/01/02 15:04:05 message" on stderr.
void logf(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
void set_log_quiet(bool quiet);
std::string env_or(const char* key, const std::string& def);

}  // namespace p2p
