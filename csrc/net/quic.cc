// QUIC v1 transport for libp2p -- see quic.h for the design.
#include "quic.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <openssl/err.h>
#include <openssl/evp.h>
#include <openssl/hmac.h>
#include <openssl/ssl.h>
#include <openssl/x509.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>

#include "tls.h"

namespace p2p {

namespace {

using Clock = std::chrono::steady_clock;

constexpr size_t kMaxDatagram = 1200;
constexpr size_t kMaxPayload = kMaxDatagram - 64;  // room for the long header + AEAD tag
constexpr uint64_t kStreamWindow = 4ull << 20;
constexpr uint64_t kConnWindow = 16ull << 20;
constexpr uint64_t kStreamLimit = 256;  // concurrent peer-opened bidi streams
constexpr size_t kMaxInFlight = 256;     // ack-eliciting 1-RTT packets outstanding
constexpr int kIdleMs = 30000, kKeepAliveMs = 10000;
constexpr uint64_t kMaxCryptoBuffer = 64 << 10;  // out-of-order CRYPTO bytes per space
// NewReno (RFC 9002 §7.2, B.2): windows in bytes of max_datagram_size
constexpr uint64_t kInitialWindow = 10 * kMaxDatagram;
constexpr uint64_t kMinWindow = 2 * kMaxDatagram;
constexpr uint64_t kPacketThreshold = 3;  // RFC 9002 §6.1.1
std::atomic<uint64_t> g_key_update_interval{1ull << 22};

// A peer's protocol violation with its RFC 9000 §20.1 transport error code.
struct QuicProtoError : std::runtime_error {
  uint64_t code;
  QuicProtoError(const std::string& m, uint64_t c) : std::runtime_error(m), code(c) {}
};
const uint8_t kInitialSalt[20] = {0x38, 0x76, 0x2c, 0xf7, 0xf5, 0x59, 0x34, 0xb3, 0x4d, 0x17,
                                  0x9a, 0xe6, 0xa4, 0xc8, 0x0c, 0xad, 0xcc, 0xbb, 0x7f, 0x0a};
const unsigned char kAlpnLibp2p[] = "\x06libp2p";

// ---------------------------------------------------------------- varints (RFC 9000 §16)
void put_varint(Bytes& b, uint64_t v) {
  if (v < 64) {
    b.push_back((uint8_t)v);
  } else if (v < 16384) {
    b.push_back((uint8_t)(0x40 | (v >> 8)));
    b.push_back((uint8_t)v);
  } else if (v < (1ull << 30)) {
    for (int i = 3; i >= 0; --i) b.push_back((uint8_t)((i == 3 ? 0x80 : 0) | (v >> (8 * i))));
  } else {
    for (int i = 7; i >= 0; --i) b.push_back((uint8_t)((i == 7 ? 0xc0 : 0) | (v >> (8 * i))));
  }
}

uint64_t get_varint(const uint8_t* p, size_t n, size_t* pos) {
  if (*pos >= n) throw NetError("quic: truncated varint");
  const int len = 1 << (p[*pos] >> 6);
  if (*pos + len > n) throw NetError("quic: truncated varint");
  uint64_t v = p[*pos] & 0x3f;
  for (int i = 1; i < len; ++i) v = (v << 8) | p[*pos + i];
  *pos += len;
  return v;
}

const uint8_t* take(const uint8_t* p, size_t n, size_t* pos, size_t len) {
  if (*pos + len > n) throw NetError("quic: truncated frame");
  const uint8_t* r = p + *pos;
  *pos += len;
  return r;
}

// ---------------------------------------------------------------- crypto (RFC 9001 §5)
Bytes hmac256(const Bytes& key, const Bytes& data) {
  unsigned int len = 32;
  Bytes out(32);
  HMAC(EVP_sha256(), key.data(), (int)key.size(), data.data(), data.size(), out.data(), &len);
  return out;
}

Bytes hkdf_expand_label(const Bytes& secret, const std::string& label, size_t len) {
  Bytes info;
  info.push_back((uint8_t)(len >> 8));
  info.push_back((uint8_t)len);
  const std::string full = "tls13 " + label;
  info.push_back((uint8_t)full.size());
  info.insert(info.end(), full.begin(), full.end());
  info.push_back(0);  // empty context
  Bytes out, t;
  for (uint8_t i = 1; out.size() < len; ++i) {
    Bytes in = t;
    in.insert(in.end(), info.begin(), info.end());
    in.push_back(i);
    t = hmac256(secret, in);
    out.insert(out.end(), t.begin(), t.end());
  }
  out.resize(len);
  return out;
}

// RFC 9001 §6.1: next-generation 1-RTT secret; its key/iv replace the old ones, the
// header protection key is never updated.
Bytes next_secret(const Bytes& secret) { return hkdf_expand_label(secret, "quic ku", secret.size()); }

void derive_keys(const Bytes& secret, QuicKeys* k);

void next_keys(const Bytes& secret, const QuicKeys& cur, QuicKeys* out) {
  derive_keys(secret, out);
  memcpy(out->hp, cur.hp, 16);
}

void derive_keys(const Bytes& secret, QuicKeys* k) {
  const Bytes key = hkdf_expand_label(secret, "quic key", 16);
  const Bytes iv = hkdf_expand_label(secret, "quic iv", 12);
  const Bytes hp = hkdf_expand_label(secret, "quic hp", 16);
  memcpy(k->key, key.data(), 16);
  memcpy(k->iv, iv.data(), 12);
  memcpy(k->hp, hp.data(), 16);
  k->ok = true;
}

// AES-128-GCM seal/open; nonce = iv XOR big-endian 64-bit counter
void make_nonce(const uint8_t iv[12], uint64_t n, uint8_t out[12]) {
  memcpy(out, iv, 12);
  for (int i = 0; i < 8; ++i) out[11 - i] ^= (uint8_t)(n >> (8 * i));
}

Bytes aead_seal(const uint8_t key[16], const uint8_t iv[12], uint64_t n, const uint8_t* aad,
                size_t aadn, const uint8_t* pt, size_t ptn) {
  uint8_t nonce[12];
  make_nonce(iv, n, nonce);
  EVP_CIPHER_CTX* c = EVP_CIPHER_CTX_new();
  Bytes out(ptn + 16);
  int l = 0;
  bool ok = EVP_EncryptInit_ex(c, EVP_aes_128_gcm(), nullptr, key, nonce) == 1 &&
            (aadn == 0 || EVP_EncryptUpdate(c, nullptr, &l, aad, (int)aadn) == 1) &&
            (ptn == 0 || EVP_EncryptUpdate(c, out.data(), &l, pt, (int)ptn) == 1) &&
            EVP_EncryptFinal_ex(c, out.data() + ptn, &l) == 1 &&
            EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_GCM_GET_TAG, 16, out.data() + ptn) == 1;
  EVP_CIPHER_CTX_free(c);
  if (!ok) throw NetError("quic: seal failed");
  return out;
}

bool aead_open(const uint8_t key[16], const uint8_t iv[12], uint64_t n, const uint8_t* aad,
               size_t aadn, const uint8_t* ct, size_t ctn, Bytes* pt) {
  if (ctn < 16) return false;
  uint8_t nonce[12];
  make_nonce(iv, n, nonce);
  EVP_CIPHER_CTX* c = EVP_CIPHER_CTX_new();
  pt->resize(ctn - 16);
  int l = 0;
  bool ok = EVP_DecryptInit_ex(c, EVP_aes_128_gcm(), nullptr, key, nonce) == 1 &&
            (aadn == 0 || EVP_DecryptUpdate(c, nullptr, &l, aad, (int)aadn) == 1) &&
            (ctn == 16 || EVP_DecryptUpdate(c, pt->data(), &l, ct, (int)(ctn - 16)) == 1) &&
            EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_GCM_SET_TAG, 16, (void*)(ct + ctn - 16)) == 1 &&
            EVP_DecryptFinal_ex(c, pt->data() + pt->size(), &l) == 1;
  EVP_CIPHER_CTX_free(c);
  return ok;
}

void hp_mask(const uint8_t hp[16], const uint8_t* sample, uint8_t mask[16]) {
  EVP_CIPHER_CTX* c = EVP_CIPHER_CTX_new();
  int l = 0;
  EVP_EncryptInit_ex(c, EVP_aes_128_ecb(), nullptr, hp, nullptr);
  EVP_CIPHER_CTX_set_padding(c, 0);
  EVP_EncryptUpdate(c, mask, &l, sample, 16);
  EVP_CIPHER_CTX_free(c);
}

// TLS 1.3 record keys ("key"/"iv") of a traffic secret
void record_keys(const Bytes& secret, uint8_t key[16], uint8_t iv[12]) {
  const Bytes k = hkdf_expand_label(secret, "key", 16);
  const Bytes v = hkdf_expand_label(secret, "iv", 12);
  memcpy(key, k.data(), 16);
  memcpy(iv, v.data(), 12);
}

Bytes from_hex(const std::string& h) {
  Bytes b;
  for (size_t i = 0; i + 1 < h.size(); i += 2) b.push_back((uint8_t)std::stoi(h.substr(i, 2), nullptr, 16));
  return b;
}

// RFC 9001 §5.8: AES-128-GCM with a fixed key and nonce, empty plaintext, the Retry
// pseudo-packet (ODCID length + ODCID + the Retry packet up to its tag) as AAD
Bytes retry_tag(const Bytes& odcid, const uint8_t* retry, size_t len) {
  static const uint8_t kKey[16] = {0xbe, 0x0c, 0x69, 0x0b, 0x9f, 0x66, 0x57, 0x5a,
                                   0x1d, 0x76, 0x6b, 0x54, 0xe3, 0x68, 0xc8, 0x4e};
  static const uint8_t kNonce[12] = {0x46, 0x15, 0x99, 0xd3, 0x5d, 0x63,
                                     0x2b, 0xf2, 0x23, 0x98, 0x25, 0xbb};
  Bytes pseudo;
  pseudo.push_back((uint8_t)odcid.size());
  pseudo.insert(pseudo.end(), odcid.begin(), odcid.end());
  pseudo.insert(pseudo.end(), retry, retry + len);
  return aead_seal(kKey, kNonce, 0, pseudo.data(), pseudo.size(), nullptr, 0);
}

Bytes rand_cid() {
  Bytes b(QuicConn::kCidLen);
  random_bytes(b.data(), b.size());
  return b;
}

double ms_since(Clock::time_point t, Clock::time_point now) {
  return std::chrono::duration<double, std::milli>(now - t).count();
}

// ---------------------------------------------------------------- OpenSSL callbacks
QuicConn* conn_of(const SSL* s) { return (QuicConn*)SSL_get_app_data(s); }

void keylog_cb(const SSL* s, const char* line) { conn_of(s)->tls_keylog(line); }

int tp_add_cb(SSL* s, unsigned int, unsigned int, const unsigned char** out, size_t* outlen, X509*,
           size_t, int*, void*) {
  const Bytes tp = conn_of(s)->tp_encode();
  unsigned char* b = (unsigned char*)OPENSSL_malloc(tp.size());
  memcpy(b, tp.data(), tp.size());
  *out = b;
  *outlen = tp.size();
  return 1;
}

void tp_free_cb(SSL*, unsigned int, unsigned int, const unsigned char* out, void*) {
  OPENSSL_free((void*)out);
}

int tp_parse_cb(SSL* s, unsigned int, unsigned int, const unsigned char* in, size_t inlen, X509*,
             size_t, int* al, void*) {
  try {
    conn_of(s)->tp_parse(in, inlen);
  } catch (...) {
    *al = SSL_AD_DECODE_ERROR;
    return 0;
  }
  return 1;
}

int accept_any(int, X509_STORE_CTX*) { return 1; }  // authenticated after the handshake

int alpn_libp2p(SSL*, const unsigned char** out, unsigned char* outlen, const unsigned char* in,
                unsigned int inlen, void*) {
  for (unsigned i = 0; i < inlen;) {
    const unsigned l = in[i];
    if (i + 1 + l > inlen) break;
    if (l == 6 && memcmp(in + i + 1, "libp2p", 6) == 0) {
      *out = in + i + 1;
      *outlen = 6;
      return SSL_TLSEXT_ERR_OK;
    }
    i += 1 + l;
  }
  return SSL_TLSEXT_ERR_ALERT_FATAL;
}

}  // namespace

void quic_initial_keys(const Bytes& dcid, QuicKeys* client, QuicKeys* server) {
  const Bytes init = hmac256(Bytes(kInitialSalt, kInitialSalt + 20), dcid);  // HKDF-Extract
  derive_keys(hkdf_expand_label(init, "client in", 32), client);
  derive_keys(hkdf_expand_label(init, "server in", 32), server);
}

// ================================================================ stream
QuicStream::QuicStream(std::shared_ptr<QuicConn> c, uint64_t id) : c_(std::move(c)), id_(id) {}

std::string QuicStream::remote_addr() const { return c_->remote_addr(); }

size_t QuicStream::read_some(uint8_t* buf, size_t n) {
  std::unique_lock<std::mutex> lk(c_->mu_);
  const auto deadline = Clock::now() + std::chrono::milliseconds(timeout_ms_);
  while (true) {
    if (rpos_ < rbuf_.size()) {
      const size_t k = std::min(n, rbuf_.size() - rpos_);
      memcpy(buf, rbuf_.data() + rpos_, k);
      rpos_ += k;
      if (rpos_ == rbuf_.size()) {
        rbuf_.clear();
        rpos_ = 0;
      }
      c_->credit_after_read(this, k);
      c_->maybe_remove(this);
      c_->flush();
      return k;
    }
    if (reset_) throw NetError("stream reset");
    if (recv_off_ == fin_off_) {
      c_->maybe_remove(this);
      return 0;
    }
    if (c_->closed_) throw NetError("connection closed");
    if (timeout_ms_ > 0) {
      if (c_->cv_.wait_until(lk, deadline) == std::cv_status::timeout && Clock::now() >= deadline &&
          rpos_ >= rbuf_.size() && !reset_ && recv_off_ != fin_off_)
        throw NetError("read timeout");
    } else {
      c_->cv_.wait(lk);
    }
  }
}

void QuicStream::write_all(const uint8_t* buf, size_t n) {
  std::unique_lock<std::mutex> lk(c_->mu_);
  while (n > 0) {
    if (c_->closed_) throw NetError("connection closed");
    if (reset_ || stop_sending_) throw NetError("stream reset");
    if (fin_pending_ || fin_sent_) throw NetError("write after close");
    // back-pressure: at most one stream window queued beyond what was packetised
    if (queued() >= kStreamWindow) {
      c_->cv_.wait_for(lk, std::chrono::milliseconds(50));
      continue;
    }
    const size_t k = std::min(n, (size_t)(kStreamWindow - queued()));
    sq_.insert(sq_.end(), buf, buf + k);
    buf += k;
    n -= k;
    c_->send_ready_.insert(id_);
    c_->flush();
  }
}

void QuicStream::close_write() {
  std::lock_guard<std::mutex> lk(c_->mu_);
  if (fin_pending_ || fin_sent_ || reset_) return;
  fin_pending_ = true;
  c_->send_ready_.insert(id_);
  c_->flush();
  c_->maybe_remove(this);
}

void QuicStream::close() {
  close_write();
  std::lock_guard<std::mutex> lk(c_->mu_);
  local_closed_ = true;
  rbuf_.clear();
  rpos_ = 0;
  c_->maybe_remove(this);
  c_->cv_.notify_all();
}

void QuicStream::reset() {
  std::lock_guard<std::mutex> lk(c_->mu_);
  if (reset_) return;
  reset_ = true;
  if (!c_->closed_) {
    Bytes f;
    f.push_back(0x04);  // RESET_STREAM id, error 0, final size
    put_varint(f, id_);
    put_varint(f, 0);
    put_varint(f, send_off_);
    c_->sp_[QuicConn::APP].queued.push_back(f);
    Bytes g;
    g.push_back(0x05);  // STOP_SENDING id, error 0
    put_varint(g, id_);
    put_varint(g, 0);
    c_->sp_[QuicConn::APP].queued.push_back(g);
    sq_.clear();
    sq_head_ = 0;
    c_->flush();
  }
  c_->maybe_remove(this);
  c_->cv_.notify_all();
}

// ================================================================ connection
QuicConn::QuicConn(std::shared_ptr<QuicTransport> t, bool client, const sockaddr_in& peer,
                   const PrivateKey& key)
    : tr_(t), fd_(t->fd_), client_(client), peer_(peer), key_(key) {
  last_recv_ = last_send_ = Clock::now();
  recv_max_data_ = kConnWindow;
  cwnd_ = kInitialWindow;
  max_remote_streams_ = kStreamLimit;
}

QuicConn::~QuicConn() {
  if (ssl_) SSL_free((SSL*)ssl_);
  if (ctx_) SSL_CTX_free((SSL_CTX*)ctx_);
}

std::string QuicConn::remote_addr() const {
  char ip[INET_ADDRSTRLEN] = {0};
  inet_ntop(AF_INET, &peer_.sin_addr, ip, sizeof(ip));
  return std::string(ip) + ":" + std::to_string(ntohs(peer_.sin_port));
}

Bytes QuicConn::transport_params() const {
  Bytes b;
  auto param = [&](uint64_t id, uint64_t v) {
    Bytes val;
    put_varint(val, v);
    put_varint(b, id);
    put_varint(b, val.size());
    b.insert(b.end(), val.begin(), val.end());
  };
  auto param_bytes = [&](uint64_t id, const Bytes& v) {
    put_varint(b, id);
    put_varint(b, v.size());
    b.insert(b.end(), v.begin(), v.end());
  };
  if (!client_) param_bytes(0x00, odcid_);  // original_destination_connection_id
  param(0x01, kIdleMs);                      // max_idle_timeout
  param(0x04, kConnWindow);                  // initial_max_data
  param(0x05, kStreamWindow);                // initial_max_stream_data_bidi_local
  param(0x06, kStreamWindow);                // initial_max_stream_data_bidi_remote
  param(0x07, 0);                            // initial_max_stream_data_uni
  param(0x08, kStreamLimit);                 // initial_max_streams_bidi
  param(0x09, 0);                            // initial_max_streams_uni
  param_bytes(0x0c, Bytes());                // disable_active_migration
  param_bytes(0x0f, scid_);                  // initial_source_connection_id
  if (!client_ && !retry_scid_.empty()) param_bytes(0x10, retry_scid_);  // retry_source_cid
  return b;
}

void QuicConn::parse_transport_params(const uint8_t* p, size_t n) {
  size_t pos = 0;
  while (pos < n) {
    const uint64_t id = get_varint(p, n, &pos);
    const uint64_t len = get_varint(p, n, &pos);
    const uint8_t* v = take(p, n, &pos, len);
    size_t q = 0;
    auto num = [&] { return get_varint(v, len, &q); };
    switch (id) {
      case 0x00: peer_odcid_.assign(v, v + len); break;
      case 0x10:
        peer_has_retry_scid_ = true;
        peer_retry_scid_.assign(v, v + len);
        break;
      case 0x01: peer_idle_ms_ = num(); break;
      case 0x04: peer_max_data_ = num(); break;
      case 0x05: peer_sd_local_ = num(); break;
      case 0x06: peer_sd_remote_ = num(); break;
      case 0x08: peer_max_bidi_ = num(); break;
      default: break;  // unknown / unused parameters are ignored (RFC 9000 §18.1)
    }
  }
  peer_tp_ = true;
}

void QuicConn::tls_keylog(const char* line) {
  const std::string l(line);
  const size_t a = l.find(' '), b = l.rfind(' ');
  if (a == std::string::npos || b == a) return;
  const std::string label = l.substr(0, a);
  const Bytes secret = from_hex(l.substr(b + 1));
  if (label == "CLIENT_HANDSHAKE_TRAFFIC_SECRET") sec_[0][0] = secret;
  else if (label == "SERVER_HANDSHAKE_TRAFFIC_SECRET") sec_[0][1] = secret;
  else if (label == "CLIENT_TRAFFIC_SECRET_0") sec_[1][0] = secret;
  else if (label == "SERVER_TRAFFIC_SECRET_0") sec_[1][1] = secret;
}

void QuicConn::begin(const Bytes& dcid, const Bytes& scid, const Bytes& odcid,
                     const Bytes& key_cid, const Bytes& retry_scid) {
  std::lock_guard<std::mutex> lk(mu_);
  dcid_ = dcid;
  scid_ = scid;
  odcid_ = odcid;
  retry_scid_ = retry_scid;
  QuicKeys c, s;
  quic_initial_keys(key_cid.empty() ? odcid : key_cid, &c, &s);
  sp_[INITIAL].tx = client_ ? c : s;
  sp_[INITIAL].rx = client_ ? s : c;
  ERR_clear_error();
  SSL_CTX* ctx = SSL_CTX_new(TLS_method());
  if (!ctx) throw NetError("quic: SSL_CTX_new failed");
  ctx_ = ctx;
  SSL_CTX_set_min_proto_version(ctx, TLS1_3_VERSION);
  SSL_CTX_set_max_proto_version(ctx, TLS1_3_VERSION);
  SSL_CTX_set_ciphersuites(ctx, "TLS_AES_128_GCM_SHA256");
  SSL_CTX_clear_options(ctx, SSL_OP_ENABLE_MIDDLEBOX_COMPAT);  // QUIC: no CCS, empty session id
  SSL_CTX_set_options(ctx, SSL_OP_NO_TICKET);
  SSL_CTX_set_num_tickets(ctx, 0);
  SSL_CTX_set_keylog_callback(ctx, keylog_cb);
  void* ck = nullptr;
  void* cert = nullptr;
  tls_make_cert(key_, &ck, &cert);
  const bool ok = SSL_CTX_use_certificate(ctx, (X509*)cert) == 1 &&
                  SSL_CTX_use_PrivateKey(ctx, (EVP_PKEY*)ck) == 1;
  X509_free((X509*)cert);
  EVP_PKEY_free((EVP_PKEY*)ck);
  if (!ok) throw NetError("quic: certificate setup failed");
  SSL_CTX_set_verify(ctx, SSL_VERIFY_PEER | SSL_VERIFY_FAIL_IF_NO_PEER_CERT, accept_any);
  const unsigned ctxs = SSL_EXT_CLIENT_HELLO | SSL_EXT_TLS1_3_ENCRYPTED_EXTENSIONS;
  if (SSL_CTX_add_custom_ext(ctx, 0x39, ctxs, tp_add_cb, tp_free_cb, nullptr, tp_parse_cb, nullptr) != 1)
    throw NetError("quic: transport parameter extension");
  if (!client_) SSL_CTX_set_alpn_select_cb(ctx, alpn_libp2p, nullptr);
  SSL* ssl = SSL_new(ctx);
  ssl_ = ssl;
  SSL_set_app_data(ssl, this);
  BIO* rb = BIO_new(BIO_s_mem());
  BIO* wb = BIO_new(BIO_s_mem());
  BIO_set_mem_eof_return(rb, -1);
  SSL_set_bio(ssl, rb, wb);
  rbio_ = rb;
  wbio_ = wb;
  if (client_) {
    SSL_set_alpn_protos(ssl, kAlpnLibp2p, sizeof(kAlpnLibp2p) - 1);
    SSL_set_connect_state(ssl);
    Events ev;
    tls_drive(ev);  // ClientHello -> Initial CRYPTO
    flush();
  } else {
    SSL_set_accept_state(ssl);
  }
}

// ---- TLS record <-> CRYPTO translation
void QuicConn::tls_collect_output() {
  BIO* wb = (BIO*)wbio_;
  uint8_t buf[16384];
  int r;
  while ((r = BIO_read(wb, buf, sizeof(buf))) > 0) tls_out_.insert(tls_out_.end(), buf, buf + r);
  size_t p = 0;
  while (tls_out_.size() - p >= 5) {
    const uint8_t type = tls_out_[p];
    const size_t len = ((size_t)tls_out_[p + 3] << 8) | tls_out_[p + 4];
    if (tls_out_.size() - p < 5 + len) break;
    const uint8_t* hdr = tls_out_.data() + p;
    const uint8_t* body = hdr + 5;
    if (type == 22) {  // plaintext handshake: ClientHello / ServerHello -> Initial
      Bytes& cp = sp_[INITIAL].crypto_pending;
      cp.insert(cp.end(), body, body + len);
    } else if (type == 23) {
      const int me = client_ ? 0 : 1;
      Bytes pt;
      bool opened = false;
      for (int attempt = 0; attempt < 2 && !opened; ++attempt) {
        const Bytes& sec = sec_[wr_epoch_][me];
        if (sec.empty()) break;
        uint8_t k[16], iv[12];
        record_keys(sec, k, iv);
        opened = aead_open(k, iv, wr_seq_, hdr, 5, body, len, &pt);
        if (!opened && wr_epoch_ == 0 && !sec_[1][me].empty()) {
          wr_epoch_ = 1;
          wr_seq_ = 0;
        } else {
          break;
        }
      }
      if (!opened) throw NetError("quic: cannot open own TLS record");
      ++wr_seq_;
      while (!pt.empty() && pt.back() == 0) pt.pop_back();
      if (pt.empty()) throw NetError("quic: empty TLS inner plaintext");
      const uint8_t inner = pt.back();
      pt.pop_back();
      if (inner == 22) {
        Bytes& cp = sp_[wr_epoch_ == 0 ? HANDSHAKE : APP].crypto_pending;
        cp.insert(cp.end(), pt.begin(), pt.end());
      } else if (inner == 21) {
        error_ = "tls alert " + std::to_string(pt.size() > 1 ? pt[1] : 0);
      }
    } else if (type == 21) {
      error_ = "tls alert " + std::to_string(len > 1 ? body[1] : 0);
    }  // 20 (change_cipher_spec) never appears: middlebox compatibility is off
    p += 5 + len;
  }
  tls_out_.erase(tls_out_.begin(), tls_out_.begin() + p);
}

void QuicConn::tls_feed(int level, const uint8_t* data, size_t len) {
  BIO* rb = (BIO*)rbio_;
  const int peer = client_ ? 1 : 0;
  for (size_t off = 0; off < len;) {
    const size_t k = std::min<size_t>(len - off, 16000);
    if (level == INITIAL) {
      uint8_t h[5] = {22, 3, 3, (uint8_t)(k >> 8), (uint8_t)k};
      BIO_write(rb, h, 5);
      BIO_write(rb, data + off, (int)k);
    } else {
      const int epoch = level == HANDSHAKE ? 0 : 1;
      const Bytes& sec = sec_[epoch][peer];
      if (sec.empty()) throw NetError("quic: CRYPTO data before its secret");
      uint8_t key[16], iv[12];
      record_keys(sec, key, iv);
      Bytes inner(data + off, data + off + k);
      inner.push_back(22);
      const size_t clen = inner.size() + 16;
      uint8_t h[5] = {23, 3, 3, (uint8_t)(clen >> 8), (uint8_t)clen};
      const Bytes ct = aead_seal(key, iv, rd_seq_[epoch]++, h, 5, inner.data(), inner.size());
      BIO_write(rb, h, 5);
      BIO_write(rb, ct.data(), (int)ct.size());
    }
    off += k;
  }
}

void QuicConn::install_keys() {
  const int me = client_ ? 0 : 1, peer = 1 - me;
  if (!sp_[HANDSHAKE].tx.ok && !sec_[0][me].empty()) derive_keys(sec_[0][me], &sp_[HANDSHAKE].tx);
  if (!sp_[HANDSHAKE].rx.ok && !sec_[0][peer].empty()) derive_keys(sec_[0][peer], &sp_[HANDSHAKE].rx);
  // 1-RTT keys: the server may send (0.5-RTT) once its Finished is out; both sides
  // accept 1-RTT packets as soon as the keys exist.
  if (!sp_[APP].tx.ok && !sec_[1][me].empty() && (tls_done_ || !client_)) {
    derive_keys(sec_[1][me], &sp_[APP].tx);
    app_sec_tx_ = sec_[1][me];
  }
  if (!sp_[APP].rx.ok && !sec_[1][peer].empty()) {
    derive_keys(sec_[1][peer], &sp_[APP].rx);
    app_sec_rx_ = sec_[1][peer];
    next_keys(next_secret(app_sec_rx_), sp_[APP].rx, &rx_next_);
  }
}

void quic_set_key_update_interval(uint64_t packets) { g_key_update_interval = packets ? packets : 1; }

void QuicConn::update_tx_keys() {
  app_sec_tx_ = next_secret(app_sec_tx_);
  QuicKeys k;
  next_keys(app_sec_tx_, sp_[APP].tx, &k);
  sp_[APP].tx = k;
  key_phase_ ^= 1;
  phase_first_pn_ = sp_[APP].next_pn;
  phase_sent_ = 0;
  phase_acked_ = false;
  ++key_updates_;
}

void QuicConn::update_rx_keys() {
  rx_prev_ = sp_[APP].rx;
  sp_[APP].rx = rx_next_;
  app_sec_rx_ = next_secret(app_sec_rx_);
  next_keys(next_secret(app_sec_rx_), sp_[APP].rx, &rx_next_);
}

bool QuicConn::force_key_update() {
  std::lock_guard<std::mutex> lk(mu_);
  if (!established_ || !sp_[APP].tx.ok || !sp_[APP].rx.ok || !phase_acked_) return false;
  update_tx_keys();
  update_rx_keys();
  return true;
}

void QuicConn::tls_drive(Events& ev) {
  if (tls_done_) {
    tls_collect_output();
    return;
  }
  SSL* ssl = (SSL*)ssl_;
  const int r = SSL_do_handshake(ssl);
  tls_collect_output();
  if (r == 1) {
    tls_done_ = true;
    install_keys();
    on_handshake_complete(ev);
    return;
  }
  const int e = SSL_get_error(ssl, r);
  if (e != SSL_ERROR_WANT_READ) {
    unsigned long code = ERR_get_error();
    char buf[256] = {0};
    ERR_error_string_n(code, buf, sizeof(buf));
    fail(std::string("tls handshake failed: ") + buf + (error_.empty() ? "" : " (" + error_ + ")"),
         0x100 + 40, ev);
    return;
  }
  install_keys();
}

void QuicConn::on_handshake_complete(Events& ev) {
  X509* pc = SSL_get1_peer_certificate((SSL*)ssl_);
  if (!pc) return fail("peer sent no certificate", 0x100 + 42, ev);
  try {
    tls_verify_peer_cert(pc, &remote_key_, &remote_);
  } catch (const std::exception& e) {
    X509_free(pc);
    return fail(e.what(), 0x100 + 42, ev);
  }
  X509_free(pc);
  if (!peer_tp_) return fail("peer sent no transport parameters", 0x08, ev);
  if (client_ && peer_odcid_ != odcid_) return fail("original_destination_connection_id mismatch", 0x08, ev);
  if (client_ && (retry_seen_ != peer_has_retry_scid_ ||
                  (retry_seen_ && peer_retry_scid_ != retry_scid_)))
    return fail("retry_source_connection_id mismatch", 0x08, ev);
  if (!client_) {
    sp_[APP].queued.push_back(Bytes{0x1e});  // HANDSHAKE_DONE
    confirmed_ = true;
    // handshake confirmed: Initial and Handshake retransmission state is done
    sp_[INITIAL].sent.clear();
    sp_[HANDSHAKE].sent.clear();
    sp_[INITIAL].queued.clear();
    sp_[HANDSHAKE].queued.clear();
    ev.accepted = true;
  }
  established_ = true;
  cv_.notify_all();
}

void QuicConn::send_raw_frame_for_test(const Bytes& frame) {
  std::lock_guard<std::mutex> lk(mu_);  // flush() runs under the connection lock
  sp_[APP].queued.push_back(frame);
  flush();
}

std::string QuicConn::error_text() {
  std::lock_guard<std::mutex> lk(mu_);
  return error_;
}

void QuicConn::fail(const std::string& why, uint64_t code, Events& ev) {
  if (error_.empty() || error_.rfind("tls alert", 0) == 0) error_ = "quic: " + why;
  close_locked(code, false, ev);
}

// ---- receive path
void QuicConn::on_datagram(const uint8_t* d, size_t n) {
  Events ev;
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (closed_) return;
    last_recv_ = Clock::now();
    size_t off = 0;
    while (off < n && !closed_) {
      const uint8_t b0 = d[off];
      if (b0 & 0x80) {  // long header
        size_t p = off + 1;
        if (n - off < 7) break;
        const uint32_t ver = ((uint32_t)d[p] << 24) | ((uint32_t)d[p + 1] << 16) |
                             ((uint32_t)d[p + 2] << 8) | d[p + 3];
        p += 4;
        const size_t dl = d[p++];
        if (p + dl + 1 > n) break;
        p += dl;
        const size_t sl = d[p++];
        if (p + sl > n) break;
        const Bytes scid(d + p, d + p + sl);
        p += sl;
        if (ver == 0) {
          // Version Negotiation (RFC 9000 §6.2): only before the handshake made progress;
          // one that lists the version we sent is discarded, otherwise the attempt fails
          if (client_ && !established_ && sp_[HANDSHAKE].recvd.empty()) {
            bool has_v1 = false;
            std::string list;
            for (size_t q = p; q + 4 <= n; q += 4) {
              const uint32_t v = ((uint32_t)d[q] << 24) | ((uint32_t)d[q + 1] << 16) |
                                 ((uint32_t)d[q + 2] << 8) | d[q + 3];
              has_v1 |= v == 1;
              char buf[16];
              snprintf(buf, sizeof(buf), "%s0x%08x", list.empty() ? "" : ",", v);
              list += buf;
            }
            if (!has_v1) {  // abandon silently (no CONNECTION_CLOSE: RFC 9000 §6.2)
              error_ = "quic: version negotiation: server supports only " + list;
              close_locked(0, false, ev, false);
            }
          }
          break;
        }
        if (ver != 1) break;
        const int type = (b0 >> 4) & 3;
        if (type == 3) {
          // Retry (RFC 9000 §17.2.5): at most one, only before any server Initial, with a
          // valid integrity tag (RFC 9001 §5.8) and a SCID that differs from the DCID we
          // sent; anything else is discarded.  A Retry fills its datagram.
          if (client_ && !retry_seen_ && !dcid_switched_ && sp_[INITIAL].recvd.empty() &&
              n - p >= 16 && scid != dcid_) {
            const Bytes tag = retry_tag(odcid_, d + off, n - 16 - off);
            if (CRYPTO_memcmp(tag.data(), d + n - 16, 16) == 0)
              on_retry(scid, Bytes(d + p, d + n - 16));
          }
          break;
        }
        if (type == 0) {
          const uint64_t tl = get_varint(d, n, &p);
          p += tl;
        } else if (type != 2) {
          break;  // 0-RTT / Retry are not used
        }
        const uint64_t len = get_varint(d, n, &p);
        if (p + len > n) break;
        const int space = type == 0 ? INITIAL : HANDSHAKE;
        if (client_ && !dcid_switched_) {  // adopt the server's chosen connection id
          dcid_ = scid;
          dcid_switched_ = true;
        }
        handle_packet(Bytes(d + off, d + p + len), p - off, space, true, ev);
        off = p + len;
      } else {
        if (n - off < 1 + kCidLen + 20) break;
        handle_packet(Bytes(d + off, d + n), 1 + kCidLen, APP, false, ev);
        off = n;
      }
    }
    flush();
  }
  run(ev);
}

// Client, mutex held: switch to the server's new connection id, re-derive the Initial
// keys from it, and resend the first flight (CRYPTO frames) in new Initials carrying the
// token; packet numbers continue, loss recovery restarts (RFC 9002 §6.3).
void QuicConn::on_retry(const Bytes& scid, const Bytes& token) {
  retry_seen_ = true;
  retry_scid_ = scid;
  retry_token_ = token;
  dcid_ = scid;
  QuicKeys c, s;
  quic_initial_keys(scid, &c, &s);
  Space& S = sp_[INITIAL];
  S.tx = c;
  S.rx = s;
  S.undecryptable.clear();
  std::deque<Bytes> again;
  for (auto& kv : S.sent) {
    for (auto& f : kv.second.frames) again.push_back(f);
    bytes_in_flight_ -= std::min<uint64_t>(bytes_in_flight_, kv.second.bytes);
  }
  S.sent.clear();
  for (auto it = again.rbegin(); it != again.rend(); ++it) S.queued.push_front(*it);
  pto_count_ = 0;
}

void QuicConn::handle_packet(Bytes pkt, size_t pn_off, int space, bool long_hdr, Events& ev) {
  Space& S = sp_[space];
  if (!S.rx.ok) {
    if (S.undecryptable.size() < 16) S.undecryptable.push_back(pkt);
    return;
  }
  if (pkt.size() < pn_off + 4 + 16) return;
  uint8_t mask[16];
  hp_mask(S.rx.hp, pkt.data() + pn_off + 4, mask);
  pkt[0] ^= mask[0] & (long_hdr ? 0x0f : 0x1f);
  const size_t pnl = (pkt[0] & 3) + 1;
  uint64_t trunc = 0;
  for (size_t i = 0; i < pnl; ++i) {
    pkt[pn_off + i] ^= mask[1 + i];
    trunc = (trunc << 8) | pkt[pn_off + i];
  }
  // RFC 9000 §A.3 packet number decoding
  const uint64_t largest = S.recvd.empty() ? 0 : *S.recvd.rbegin();
  const uint64_t expected = S.recvd.empty() ? 0 : largest + 1;
  const uint64_t win = 1ull << (pnl * 8), hwin = win / 2, msk = win - 1;
  uint64_t pn = (expected & ~msk) | trunc;
  if (pn + hwin <= expected && pn < (1ull << 62) - win) pn += win;
  else if (pn > expected + hwin && pn >= win) pn -= win;
  Bytes pt;
  const size_t hl = pn_off + pnl;
  const int kp = (pkt[0] >> 2) & 1;
  if (space != APP || kp == key_phase_) {
    if (!aead_open(S.rx.key, S.rx.iv, pn, pkt.data(), hl, pkt.data() + hl, pkt.size() - hl, &pt))
      return;  // undecryptable (corrupt / stale keys): drop
  } else if (rx_prev_.ok && aead_open(rx_prev_.key, rx_prev_.iv, pn, pkt.data(), hl,
                                      pkt.data() + hl, pkt.size() - hl, &pt)) {
    // a late packet of the previous key phase
  } else if (rx_next_.ok && aead_open(rx_next_.key, rx_next_.iv, pn, pkt.data(), hl,
                                      pkt.data() + hl, pkt.size() - hl, &pt)) {
    // the peer started a key update (RFC 9001 §6.2): follow it on both directions
    update_rx_keys();
    update_tx_keys();
  } else {
    return;
  }
  if (pn < S.recv_floor || S.recvd.count(pn)) return;  // duplicate
  S.recvd.insert(pn);
  while (S.recvd.size() > 512) {
    S.recv_floor = *S.recvd.begin() + 1;
    S.recvd.erase(S.recvd.begin());
  }
  bool elicit = false;
  try {
    process_frames(space, pt.data(), pt.size(), &elicit, ev);
  } catch (const QuicProtoError& e) {
    return fail(std::string("protocol error: ") + e.what(), e.code, ev);
  } catch (const std::exception& e) {
    return fail(std::string("frame error: ") + e.what(), 0x07, ev);
  }
  if (elicit) S.ack_pending = true;
  if (!client_ && space == HANDSHAKE && !sp_[INITIAL].sent.empty()) {
    sp_[INITIAL].sent.clear();  // server: Initial keys are done once Handshake arrives
    sp_[INITIAL].queued.clear();
  }
}

void QuicConn::process_frames(int space, const uint8_t* p, size_t n, bool* elicit, Events& ev) {
  size_t pos = 0;
  while (pos < n && !closed_) {
    const uint64_t type = get_varint(p, n, &pos);
    if (type != 0x00 && type != 0x02 && type != 0x03 && type != 0x1c && type != 0x1d) *elicit = true;
    if (type == 0x00 || type == 0x01) continue;  // PADDING, PING
    if (type == 0x02 || type == 0x03) {
      on_ack(space, p, n, &pos, type == 0x03);
    } else if (type == 0x04) {  // RESET_STREAM
      const uint64_t id = get_varint(p, n, &pos);
      get_varint(p, n, &pos);
      get_varint(p, n, &pos);
      auto it = streams_.find(id);
      if (it != streams_.end()) {
        it->second->reset_ = true;
        maybe_remove(it->second.get());
      }
    } else if (type == 0x05) {  // STOP_SENDING
      const uint64_t id = get_varint(p, n, &pos);
      get_varint(p, n, &pos);
      auto it = streams_.find(id);
      if (it != streams_.end()) {
        it->second->stop_sending_ = true;
        it->second->sq_.clear();
        it->second->sq_head_ = 0;
        maybe_remove(it->second.get());
      }
    } else if (type == 0x06) {  // CRYPTO
      const uint64_t off = get_varint(p, n, &pos);
      const uint64_t len = get_varint(p, n, &pos);
      const uint8_t* data = take(p, n, &pos, len);
      on_crypto(space, off, data, len, ev);
    } else if (type == 0x07) {  // NEW_TOKEN
      const uint64_t len = get_varint(p, n, &pos);
      take(p, n, &pos, len);
    } else if (type >= 0x08 && type <= 0x0f) {  // STREAM
      const uint64_t id = get_varint(p, n, &pos);
      const uint64_t off = (type & 0x04) ? get_varint(p, n, &pos) : 0;
      const uint64_t len = (type & 0x02) ? get_varint(p, n, &pos) : n - pos;
      const uint8_t* data = take(p, n, &pos, len);
      if (space != APP) throw NetError("STREAM outside 1-RTT");
      on_stream_frame(id, off, data, len, type & 0x01, ev);
    } else if (type == 0x10) {
      peer_max_data_ = std::max(peer_max_data_, get_varint(p, n, &pos));
    } else if (type == 0x11) {
      const uint64_t id = get_varint(p, n, &pos);
      const uint64_t v = get_varint(p, n, &pos);
      auto it = streams_.find(id);
      if (it != streams_.end()) it->second->max_send_ = std::max(it->second->max_send_, v);
    } else if (type == 0x12) {
      peer_max_bidi_ = std::max(peer_max_bidi_, get_varint(p, n, &pos));
    } else if (type == 0x13 || type == 0x14 || type == 0x16 || type == 0x17) {
      get_varint(p, n, &pos);
    } else if (type == 0x15) {
      get_varint(p, n, &pos);
      get_varint(p, n, &pos);
    } else if (type == 0x18) {  // NEW_CONNECTION_ID: we keep using the first id
      get_varint(p, n, &pos);
      get_varint(p, n, &pos);
      const size_t l = *take(p, n, &pos, 1);
      take(p, n, &pos, l + 16);
    } else if (type == 0x19) {
      get_varint(p, n, &pos);
    } else if (type == 0x1a) {  // PATH_CHALLENGE -> PATH_RESPONSE
      const uint8_t* data = take(p, n, &pos, 8);
      Bytes f{0x1b};
      f.insert(f.end(), data, data + 8);
      sp_[APP].queued.push_back(f);
    } else if (type == 0x1b) {
      take(p, n, &pos, 8);
    } else if (type == 0x1c || type == 0x1d) {  // CONNECTION_CLOSE
      const uint64_t code = get_varint(p, n, &pos);
      if (type == 0x1c) get_varint(p, n, &pos);
      const uint64_t rl = get_varint(p, n, &pos);
      const uint8_t* r = take(p, n, &pos, rl);
      if (error_.empty())
        error_ = "quic: closed by peer (code " + std::to_string(code) + ")" +
                 (rl ? ": " + std::string((const char*)r, rl) : "");
      close_locked(0, false, ev, false);
      return;
    } else if (type == 0x1e) {  // HANDSHAKE_DONE
      if (client_ && !confirmed_) {
        confirmed_ = true;
        for (int s : {INITIAL, HANDSHAKE}) {
          sp_[s].sent.clear();
          sp_[s].queued.clear();
        }
      }
    } else {
      throw NetError("unknown frame type " + std::to_string(type));
    }
  }
}

void QuicConn::on_ack(int space, const uint8_t* p, size_t n, size_t* pos, bool ecn) {
  Space& S = sp_[space];
  const uint64_t largest = get_varint(p, n, pos);
  get_varint(p, n, pos);  // ack delay
  const uint64_t count = get_varint(p, n, pos);
  uint64_t hi = largest, lo = largest - std::min(largest, get_varint(p, n, pos));
  std::vector<std::pair<uint64_t, uint64_t>> ranges{{lo, hi}};
  for (uint64_t i = 0; i < count; ++i) {
    const uint64_t gap = get_varint(p, n, pos), len = get_varint(p, n, pos);
    if (lo < gap + 2) break;
    hi = lo - gap - 2;
    lo = hi - std::min(hi, len);
    ranges.push_back({lo, hi});
  }
  if (ecn)
    for (int i = 0; i < 3; ++i) get_varint(p, n, pos);
  bool newly = false;
  const auto now = Clock::now();
  for (auto& r : ranges) {
    auto it = S.sent.lower_bound(r.first);
    while (it != S.sent.end() && it->first <= r.second) {
      on_packet_acked(it->second);
      if (space == APP && it->first >= phase_first_pn_) phase_acked_ = true;
      if (it->first == largest) {  // RTT sample (RFC 9002 §5.3, ack delay ignored)
        const double rtt = ms_since(it->second.t, now);
        latest_rtt_ms_ = rtt;
        if (srtt_ms_ == 0) {
          srtt_ms_ = rtt;
          rttvar_ms_ = rtt / 2;
        } else {
          rttvar_ms_ = 0.75 * rttvar_ms_ + 0.25 * std::abs(srtt_ms_ - rtt);
          srtt_ms_ = 0.875 * srtt_ms_ + 0.125 * rtt;
        }
      }
      it = S.sent.erase(it);
      newly = true;
    }
    if (space == APP)
      for (auto pi = pings_.lower_bound(r.first); pi != pings_.end() && pi->first <= r.second; ++pi)
        pi->second = true;
  }
  if (newly) {
    pto_count_ = 0;
    detect_lost(space, largest, now);
  }
  cv_.notify_all();
}

void QuicConn::on_crypto(int space, uint64_t off, const uint8_t* data, size_t len, Events& ev) {
  Space& S = sp_[space];
  if (off + len <= S.crypto_in_off) return;  // retransmitted
  // RFC 9000 §7.5: bound what an (unauthenticated) peer can make us buffer ahead
  if (off + len > S.crypto_in_off + kMaxCryptoBuffer || S.crypto_in_bytes + len > kMaxCryptoBuffer)
    throw QuicProtoError("CRYPTO data beyond the buffer", 0x0d);  // CRYPTO_BUFFER_EXCEEDED
  Bytes& slot = S.crypto_in[off];
  if (slot.size() >= len) return;
  S.crypto_in_bytes += len - slot.size();
  slot.assign(data, data + len);
  Bytes ready;
  while (!S.crypto_in.empty() && S.crypto_in.begin()->first <= S.crypto_in_off) {
    auto it = S.crypto_in.begin();
    const uint64_t o = it->first;
    const Bytes& b = it->second;
    if (o + b.size() > S.crypto_in_off) {
      ready.insert(ready.end(), b.begin() + (S.crypto_in_off - o), b.end());
      S.crypto_in_off = o + b.size();
    }
    S.crypto_in_bytes -= b.size();
    S.crypto_in.erase(it);
  }
  if (ready.empty()) return;
  if (space == APP && tls_done_) return;  // post-handshake messages (none are sent to us)
  tls_feed(space, ready.data(), ready.size());
  tls_drive(ev);
  // keys for the next level may now exist: replay packets that arrived early
  for (int s = HANDSHAKE; s <= APP; ++s) {
    if (!sp_[s].rx.ok || sp_[s].undecryptable.empty()) continue;
    std::vector<Bytes> pend;
    pend.swap(sp_[s].undecryptable);
    for (auto& pk : pend) {
      size_t pn_off;
      if (s == APP) {
        pn_off = 1 + kCidLen;
      } else {
        size_t p = 1 + 4;
        p += 1 + pk[p];
        p += 1 + pk[p];
        get_varint(pk.data(), pk.size(), &p);
        pn_off = p;
      }
      handle_packet(pk, pn_off, s, s != APP, ev);
    }
  }
}

std::shared_ptr<QuicStream> QuicConn::peer_stream(uint64_t id, Events& ev) {
  auto it = streams_.find(id);
  if (it != streams_.end()) return it->second;
  const bool peer_init = (id & 1) == (client_ ? 1u : 0u);
  if (!peer_init || (id & 2)) return nullptr;  // closed local stream / unidirectional
  const uint64_t idx = id >> 2;
  if (idx < next_remote_idx_) return nullptr;  // opened before and already finished
  if (idx >= max_remote_streams_) throw NetError("STREAM_LIMIT_ERROR");
  // RFC 9000 §3.2: opening stream N implicitly opens every lower-numbered stream
  // of that type (their first frames may simply have been lost or reordered)
  std::shared_ptr<QuicStream> s;
  for (uint64_t i = next_remote_idx_; i <= idx; ++i) {
    const uint64_t sid = (i << 2) | (client_ ? 1 : 0);
    s = std::make_shared<QuicStream>(shared_from_this(), sid);
    s->max_send_ = peer_sd_local_;
    s->recv_limit_ = kStreamWindow;
    streams_[sid] = s;
    if (started_ && on_stream_) ev.streams.push_back(s);
    else pending_inbound_.push_back(s);
  }
  next_remote_idx_ = idx + 1;
  return s;
}

void QuicConn::on_stream_frame(uint64_t id, uint64_t off, const uint8_t* data, size_t len,
                               bool fin, Events& ev) {
  auto s = peer_stream(id, ev);
  if (!s) return;
  // RFC 9000 §4: data past the advertised stream / connection limits is a
  // FLOW_CONTROL_ERROR (never buffered: rbuf_/ooo_ stay bounded by our windows)
  const uint64_t end = off + len;
  if (end > s->recv_limit_) throw QuicProtoError("stream data beyond MAX_STREAM_DATA", 0x03);
  if (end > s->recv_high_) {
    if (recv_total_ + (end - s->recv_high_) > recv_max_data_)
      throw QuicProtoError("data beyond MAX_DATA", 0x03);
    recv_total_ += end - s->recv_high_;
    s->recv_high_ = end;
  }
  if (fin) s->fin_off_ = off + len;
  if (s->local_closed_ || s->reset_) {
    // input discarded, but the credit is returned so the peer is never blocked
    if (off + len > s->recv_off_) {
      const uint64_t adv = off + len - s->recv_off_;
      s->recv_off_ = off + len;
      credit_after_read(s.get(), adv);
    }
    maybe_remove(s.get());
    return;
  }
  if (off + len > s->recv_off_) {
    if (off <= s->recv_off_) {
      s->rbuf_.insert(s->rbuf_.end(), data + (s->recv_off_ - off), data + len);
      s->recv_off_ = off + len;
      while (!s->ooo_.empty() && s->ooo_.begin()->first <= s->recv_off_) {
        auto it = s->ooo_.begin();
        const uint64_t o = it->first;
        const Bytes& b = it->second;
        if (o + b.size() > s->recv_off_) {
          s->rbuf_.insert(s->rbuf_.end(), b.begin() + (s->recv_off_ - o), b.end());
          s->recv_off_ = o + b.size();
        }
        s->ooo_.erase(it);
      }
    } else {
      Bytes& slot = s->ooo_[off];
      if (slot.size() < len) slot.assign(data, data + len);
    }
  }
  cv_.notify_all();
}

void QuicConn::credit_after_read(QuicStream* s, size_t n) {
  s->consumed_ += n;
  recv_consumed_ += n;
  if (s->recv_limit_ - s->consumed_ < kStreamWindow / 2 && s->fin_off_ == ~0ull) {
    s->recv_limit_ = s->consumed_ + kStreamWindow;
    Bytes f{0x11};
    put_varint(f, s->id_);
    put_varint(f, s->recv_limit_);
    sp_[APP].queued.push_back(f);
  }
  if (recv_max_data_ - recv_consumed_ < kConnWindow / 2) {
    recv_max_data_ = recv_consumed_ + kConnWindow;
    Bytes f{0x10};
    put_varint(f, recv_max_data_);
    sp_[APP].queued.push_back(f);
  }
}

void QuicConn::maybe_remove(QuicStream* s) {
  const bool send_done = s->fin_sent_ || s->reset_ || s->stop_sending_;
  const bool recv_done =
      s->reset_ || s->local_closed_ || (s->recv_off_ == s->fin_off_ && s->rpos_ >= s->rbuf_.size());
  if (!send_done || !recv_done) return;
  auto it = streams_.find(s->id_);
  if (it == streams_.end() || it->second.get() != s) return;
  const bool peer_init = (s->id_ & 1) == (client_ ? 1u : 0u);
  streams_.erase(it);
  send_ready_.erase(s->id_);
  if (peer_init && ++remote_closed_ % 32 == 0) {
    max_remote_streams_ = remote_closed_ + kStreamLimit;
    Bytes f{0x12};
    put_varint(f, max_remote_streams_);
    sp_[APP].queued.push_back(f);
  }
}

// ---- send path
Bytes QuicConn::ack_frame(int space) {
  Space& S = sp_[space];
  Bytes f{0x02};
  std::vector<std::pair<uint64_t, uint64_t>> ranges;  // (hi, lo), descending
  for (auto it = S.recvd.rbegin(); it != S.recvd.rend(); ++it) {
    if (!ranges.empty() && ranges.back().second == *it + 1) ranges.back().second = *it;
    else if (ranges.size() < 32) ranges.push_back({*it, *it});
    else break;
  }
  put_varint(f, ranges[0].first);
  put_varint(f, 0);
  put_varint(f, ranges.size() - 1);
  put_varint(f, ranges[0].first - ranges[0].second);
  for (size_t i = 1; i < ranges.size(); ++i) {
    put_varint(f, ranges[i - 1].second - ranges[i].first - 2);
    put_varint(f, ranges[i].first - ranges[i].second);
  }
  return f;
}

void QuicConn::send_packet(int space, const Bytes& payload_in, bool elicit,
                           std::vector<Bytes> frames) {
  Space& S = sp_[space];
  const uint64_t pn = S.next_pn++;
  Bytes hdr;
  size_t pn_off;
  Bytes payload = payload_in;
  if (space != APP) {
    hdr.push_back((uint8_t)(0xc0 | ((space == INITIAL ? 0 : 2) << 4) | 0x03));
    hdr.insert(hdr.end(), {0, 0, 0, 1});
    hdr.push_back((uint8_t)dcid_.size());
    hdr.insert(hdr.end(), dcid_.begin(), dcid_.end());
    hdr.push_back((uint8_t)scid_.size());
    hdr.insert(hdr.end(), scid_.begin(), scid_.end());
    if (space == INITIAL) {  // token (a client echoes the Retry's; empty otherwise)
      put_varint(hdr, retry_token_.size());
      hdr.insert(hdr.end(), retry_token_.begin(), retry_token_.end());
    }
    if (space == INITIAL && elicit) {        // RFC 9000 §14.1: 1200-byte datagrams
      const size_t total = hdr.size() + 2 + 4 + payload.size() + 16;
      if (total < kMaxDatagram) payload.resize(payload.size() + (kMaxDatagram - total), 0);
    }
    const size_t len = 4 + payload.size() + 16;
    hdr.push_back((uint8_t)(0x40 | (len >> 8)));
    hdr.push_back((uint8_t)len);
  } else {
    hdr.push_back((uint8_t)(0x40 | (key_phase_ << 2) | 0x03));
    hdr.insert(hdr.end(), dcid_.begin(), dcid_.end());
  }
  pn_off = hdr.size();
  for (int i = 3; i >= 0; --i) hdr.push_back((uint8_t)(pn >> (8 * i)));
  const Bytes ct = aead_seal(S.tx.key, S.tx.iv, pn, hdr.data(), hdr.size(), payload.data(), payload.size());
  Bytes pkt = hdr;
  pkt.insert(pkt.end(), ct.begin(), ct.end());
  uint8_t mask[16];
  hp_mask(S.tx.hp, pkt.data() + pn_off + 4, mask);
  pkt[0] ^= mask[0] & (space != APP ? 0x0f : 0x1f);
  for (int i = 0; i < 4; ++i) pkt[pn_off + i] ^= mask[1 + i];
  ::sendto(fd_, pkt.data(), pkt.size(), 0, (const sockaddr*)&peer_, sizeof(peer_));
  const auto now = Clock::now();
  if (elicit) {
    S.sent[pn] = SentPkt{now, std::move(frames), pkt.size()};
    bytes_in_flight_ += pkt.size();
    last_send_ = now;
  }
  if (space == APP && ++phase_sent_ >= g_key_update_interval && phase_acked_ && sp_[APP].rx.ok) {
    update_tx_keys();  // AEAD usage limit: next packets go out in the new phase
    update_rx_keys();
  }
}

// ---- NewReno (RFC 9002 §7, Appendix B)
void QuicConn::on_packet_acked(const SentPkt& p) {
  bytes_in_flight_ -= std::min<uint64_t>(bytes_in_flight_, p.bytes);
  if (p.t <= recovery_start_) return;  // no growth for packets sent before the recovery
  if (cwnd_ < ssthresh_) cwnd_ += p.bytes;                              // slow start
  else cwnd_ += std::max<uint64_t>(1, kMaxDatagram * p.bytes / cwnd_);  // congestion avoidance
}

void QuicConn::on_packets_lost(int, Clock::time_point newest_lost_sent) {
  if (newest_lost_sent <= recovery_start_) return;  // one reduction per round trip
  recovery_start_ = Clock::now();
  ssthresh_ = std::max(cwnd_ / 2, kMinWindow);
  cwnd_ = ssthresh_;
  ++congestion_events_;
}

// RFC 9002 §6.1: a packet is lost once kPacketThreshold later packets were acknowledged,
// or it was sent more than 9/8 of an RTT before an acknowledged one.
void QuicConn::detect_lost(int space, uint64_t largest_acked, Clock::time_point now) {
  Space& S = sp_[space];
  const double rtt = std::max(srtt_ms_, latest_rtt_ms_);
  const double thr_ms = std::max(9.0 / 8.0 * (rtt > 0 ? rtt : 50.0), 1.0);
  bool any = false;
  Clock::time_point newest{};
  for (auto it = S.sent.begin(); it != S.sent.end() && it->first < largest_acked;) {
    if (it->first + kPacketThreshold <= largest_acked || ms_since(it->second.t, now) > thr_ms) {
      for (auto f = it->second.frames.rbegin(); f != it->second.frames.rend(); ++f)
        S.queued.push_front(*f);
      retx_count_ += it->second.frames.size();
      bytes_in_flight_ -= std::min<uint64_t>(bytes_in_flight_, it->second.bytes);
      newest = std::max(newest, it->second.t);
      any = true;
      it = S.sent.erase(it);
    } else {
      ++it;
    }
  }
  if (any) on_packets_lost(space, newest);
}

void QuicConn::flush() {
  if (closed_) return;
  for (int space = INITIAL; space <= APP; ++space) {
    Space& S = sp_[space];
    if (!S.tx.ok) continue;
    while (true) {
      Bytes pl;
      std::vector<Bytes> frames;
      bool elicit = false;
      if (S.ack_pending && !S.recvd.empty()) {
        const Bytes a = ack_frame(space);
        pl.insert(pl.end(), a.begin(), a.end());
        S.ack_pending = false;
      }
      auto add = [&](Bytes f) {
        pl.insert(pl.end(), f.begin(), f.end());
        frames.push_back(std::move(f));
        elicit = true;
      };
      while (!S.queued.empty() && pl.size() + S.queued.front().size() <= kMaxPayload) {
        add(std::move(S.queued.front()));
        S.queued.pop_front();
      }
      while (!S.crypto_pending.empty() && pl.size() + 24 < kMaxPayload) {
        const size_t k = std::min(S.crypto_pending.size(), kMaxPayload - pl.size() - 20);
        Bytes f{0x06};
        put_varint(f, S.crypto_send_off);
        put_varint(f, k);
        f.insert(f.end(), S.crypto_pending.begin(), S.crypto_pending.begin() + k);
        S.crypto_pending.erase(S.crypto_pending.begin(), S.crypto_pending.begin() + k);
        S.crypto_send_off += k;
        add(std::move(f));
      }
      // stream data: NewReno congestion window (bytes in flight), plus a packet cap
      if (space == APP && established_ && S.sent.size() < kMaxInFlight &&
          bytes_in_flight_ + kMaxDatagram <= cwnd_) {
        for (auto it = send_ready_.begin(); it != send_ready_.end() && pl.size() + 32 < kMaxPayload;) {
          auto si = streams_.find(*it);
          if (si == streams_.end()) {
            it = send_ready_.erase(it);
            continue;
          }
          QuicStream* s = si->second.get();
          const uint64_t credit = std::min(peer_max_data_ - std::min(peer_max_data_, sent_data_),
                                           s->max_send_ - std::min(s->max_send_, s->send_off_));
          const size_t k = (size_t)std::min<uint64_t>({s->queued(), credit, kMaxPayload - pl.size() - 28});
          const bool fin = s->fin_pending_ && k == s->queued();
          if (k == 0 && !fin) {
            if (s->queued() == 0) it = send_ready_.erase(it);
            else ++it;  // blocked by flow control
            continue;
          }
          Bytes f{(uint8_t)(0x08 | 0x04 | 0x02 | (fin ? 1 : 0))};
          put_varint(f, s->id_);
          put_varint(f, s->send_off_);
          put_varint(f, k);
          f.insert(f.end(), s->sq_.begin() + s->sq_head_, s->sq_.begin() + s->sq_head_ + k);
          s->sq_head_ += k;
          if (s->sq_head_ == s->sq_.size()) {
            s->sq_.clear();
            s->sq_head_ = 0;
          } else if (s->sq_head_ >= (1u << 16)) {
            s->sq_.erase(s->sq_.begin(), s->sq_.begin() + s->sq_head_);
            s->sq_head_ = 0;
          }
          s->send_off_ += k;
          sent_data_ += k;
          if (fin) {
            s->fin_pending_ = false;
            s->fin_sent_ = true;
          }
          add(std::move(f));
          if (s->queued() == 0 && !s->fin_pending_) {
            it = send_ready_.erase(it);
            if (fin) maybe_remove(s);
          }
        }
        cv_.notify_all();  // writers waiting on queue space
      }
      if (pl.empty()) break;
      send_packet(space, pl, elicit, std::move(frames));
    }
  }
}

// ---- timers / lifecycle
void QuicConn::tick(Clock::time_point now) {
  Events ev;
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (closed_) return;
    if (ms_since(last_recv_, now) > (established_ ? kIdleMs : 10000)) {
      if (error_.empty()) error_ = established_ ? "quic: idle timeout" : "quic: handshake timeout";
      close_locked(0, false, ev, false);
    } else {
      const double srtt = srtt_ms_ > 0 ? srtt_ms_ : 50.0;
      const double pto = (srtt + std::max(4 * rttvar_ms_, 1.0) + 5.0) * (1 << std::min(pto_count_, 6));
      bool fired = false;
      for (int s = INITIAL; s <= APP; ++s) {
        Space& S = sp_[s];
        if (S.sent.empty() || ms_since(S.sent.begin()->second.t, now) < pto) continue;
        std::deque<Bytes> again;
        for (auto& kv : S.sent) {
          for (auto& f : kv.second.frames) again.push_back(f);
          bytes_in_flight_ -= std::min<uint64_t>(bytes_in_flight_, kv.second.bytes);
        }
        S.sent.clear();
        if (again.empty()) again.push_back(Bytes{0x01});  // PING probe
        for (auto it = again.rbegin(); it != again.rend(); ++it) S.queued.push_front(*it);
        retx_count_ += again.size();
        fired = true;
      }
      if (fired && ++pto_count_ >= 3 && cwnd_ > kMinWindow) {
        // RFC 9002 §7.6: repeated probe timeouts = persistent congestion
        cwnd_ = kMinWindow;
        recovery_start_ = now;
        ++congestion_events_;
      }
      if (established_ && ms_since(last_send_, now) > kKeepAliveMs) sp_[APP].queued.push_back(Bytes{0x01});
      flush();
    }
  }
  run(ev);
}

void QuicConn::close_locked(uint64_t code, bool app, Events& ev, bool send) {
  if (closed_) return;
  if (send) {
    for (int s = APP; s >= INITIAL; --s) {
      if (!sp_[s].tx.ok) continue;
      Bytes f{(uint8_t)(app && s == APP ? 0x1d : 0x1c)};
      put_varint(f, code);
      if (!(app && s == APP)) put_varint(f, 0);
      put_varint(f, 0);
      send_packet(s, f, false, {});
      break;
    }
  }
  closed_ = true;
  ev.closed = true;
  cv_.notify_all();
}

void QuicConn::run(Events& ev) {
  if (ev.accepted) {
    if (auto t = tr_.lock()) {
      std::function<void(QuicConnPtr)> cb;
      {
        std::lock_guard<std::mutex> lk(t->mu_);
        cb = t->accept_;
      }
      if (cb) {
        auto self = shared_from_this();
        t->busy_++;
        std::thread([t, cb, self] {
          cb(self);
          t->busy_--;
        }).detach();
      }
    }
  }
  for (auto& s : ev.streams) {
    auto cb = on_stream_;
    std::thread([cb, s] {
      try {
        cb(s);
      } catch (...) {
      }
    }).detach();
  }
  if (ev.closed) {
    if (auto t = tr_.lock()) t->forget(this);
    std::function<void()> cb;
    {
      std::lock_guard<std::mutex> lk(mu_);
      cb.swap(on_close_);
    }
    if (cb) cb();
  }
}

bool QuicConn::wait_established(int timeout_ms) {
  std::unique_lock<std::mutex> lk(mu_);
  cv_.wait_for(lk, std::chrono::milliseconds(timeout_ms), [&] { return established_ || closed_; });
  return established_ && !closed_;
}

void QuicConn::start(std::function<void(StreamPtr)> on_stream, std::function<void()> on_close) {
  Events ev;
  {
    std::lock_guard<std::mutex> lk(mu_);
    on_stream_ = std::move(on_stream);
    on_close_ = std::move(on_close);
    started_ = true;
    if (on_stream_) ev.streams.swap(pending_inbound_);
    if (closed_) ev.closed = true;
  }
  if (ev.closed) {
    std::function<void()> cb;
    {
      std::lock_guard<std::mutex> lk(mu_);
      cb.swap(on_close_);
    }
    if (cb) cb();
    ev.closed = false;
  }
  run(ev);
}

StreamPtr QuicConn::open_stream() {
  std::unique_lock<std::mutex> lk(mu_);
  cv_.wait_for(lk, std::chrono::seconds(10), [&] { return closed_ || next_local_idx_ < peer_max_bidi_; });
  if (closed_) throw NetError(error_.empty() ? "quic: connection closed" : error_);
  if (next_local_idx_ >= peer_max_bidi_) throw NetError("quic: stream limit reached");
  const uint64_t id = (next_local_idx_++ << 2) | (client_ ? 0 : 1);
  auto s = std::make_shared<QuicStream>(shared_from_this(), id);
  s->max_send_ = peer_sd_remote_;
  s->recv_limit_ = kStreamWindow;
  streams_[id] = s;
  return s;
}

void QuicConn::close() {
  Events ev;
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (closed_) return;
    flush();  // queued stream data / FINs go out before the close
    close_locked(0, established_.load(), ev);
  }
  run(ev);
}

long QuicConn::ping(int timeout_ms) {
  std::unique_lock<std::mutex> lk(mu_);
  if (closed_ || !sp_[APP].tx.ok) return -1;
  const auto t0 = Clock::now(), deadline = t0 + std::chrono::milliseconds(timeout_ms);
  std::vector<uint64_t> pns;  // a lost probe is re-sent in a fresh packet
  auto acked = [&] {
    for (uint64_t pn : pns)
      if (pings_[pn]) return true;
    return false;
  };
  while (!closed_ && !acked() && Clock::now() < deadline) {
    pns.push_back(sp_[APP].next_pn);
    pings_[pns.back()] = false;
    send_packet(APP, Bytes{0x01}, true, {Bytes{0x01}});
    cv_.wait_until(lk, std::min(deadline, Clock::now() + std::chrono::milliseconds(200)),
                   [&] { return closed_ || acked(); });
  }
  const bool ok = acked();
  for (uint64_t pn : pns) pings_.erase(pn);
  if (!ok) return -1;
  return (long)std::chrono::duration_cast<std::chrono::microseconds>(Clock::now() - t0).count();
}

size_t QuicConn::num_streams() {
  std::lock_guard<std::mutex> lk(mu_);
  return streams_.size();
}

// ================================================================ transport
std::shared_ptr<QuicTransport> QuicTransport::create(const std::string& host, int port,
                                                     const PrivateKey& key) {
  std::shared_ptr<QuicTransport> t(new QuicTransport(key));
  t->fd_ = ::socket(AF_INET, SOCK_DGRAM | SOCK_CLOEXEC, 0);
  if (t->fd_ < 0) throw NetError("quic: socket failed");
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port);
  if (inet_pton(AF_INET, host.c_str(), &a.sin_addr) != 1) throw NetError("quic: bad host " + host);
  if (::bind(t->fd_, (sockaddr*)&a, sizeof(a)) != 0) {
    ::close(t->fd_);
    throw NetError("quic: bind " + host + ":" + std::to_string(port) + " failed");
  }
  int buf = 4 << 20;
  setsockopt(t->fd_, SOL_SOCKET, SO_RCVBUF, &buf, sizeof(buf));
  setsockopt(t->fd_, SOL_SOCKET, SO_SNDBUF, &buf, sizeof(buf));
  socklen_t al = sizeof(a);
  getsockname(t->fd_, (sockaddr*)&a, &al);
  t->port_ = ntohs(a.sin_port);
  t->host_ = host;
  t->token_key_.resize(32);
  random_bytes(t->token_key_.data(), t->token_key_.size());
  const char* rr = getenv("P2P_QUIC_RETRY");
  t->require_retry_ = rr && rr[0] == '1';
  auto self = t;
  t->th_ = std::thread([self] { self->loop(); });
  return t;
}

QuicTransport::~QuicTransport() {
  close();
  if (fd_ >= 0) ::close(fd_);
}

void QuicTransport::set_accept(std::function<void(QuicConnPtr)> cb) {
  std::lock_guard<std::mutex> lk(mu_);
  accept_ = std::move(cb);
}

void QuicTransport::register_cid(const Bytes& cid, const QuicConnPtr& c) {
  std::lock_guard<std::mutex> lk(mu_);
  by_cid_[cid] = c;
}

void QuicTransport::forget(const QuicConn* c) {
  std::lock_guard<std::mutex> lk(mu_);
  for (auto it = by_cid_.begin(); it != by_cid_.end();) {
    if (it->second.get() == c) it = by_cid_.erase(it);
    else ++it;
  }
}

QuicConnPtr QuicTransport::dial(const std::string& host, int port, const PeerId& expected,
                                int timeout_ms) {
  if (closed_) throw NetError("quic: transport closed");
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port);
  if (inet_pton(AF_INET, host.c_str(), &a.sin_addr) != 1) throw NetError("quic: bad host " + host);
  auto c = std::make_shared<QuicConn>(shared_from_this(), true, a, key_);
  const Bytes scid = rand_cid(), dcid = rand_cid();
  register_cid(scid, c);
  try {
    c->begin(dcid, scid, dcid);
  } catch (...) {
    forget(c.get());
    throw;
  }
  if (!c->wait_established(timeout_ms)) {
    std::string err;
    {
      std::lock_guard<std::mutex> lk(c->mu_);
      err = c->error_;
    }
    c->close();
    throw NetError(err.empty() ? "quic: handshake timeout" : err);
  }
  if (!expected.empty() && c->remote_peer() != expected) {
    c->close();
    throw NetError("quic: peer id mismatch (expected " + expected.to_base58() + ", got " +
                   c->remote_peer().to_base58() + ")");
  }
  return c;
}

// RFC 9000 §6 / §17.2.1: a long-header packet of a version this endpoint does not speak,
// in a datagram large enough to be a client's first flight, is answered with a Version
// Negotiation packet (version 0) listing the supported versions, with the connection ids
// echoed back swapped.  (Never in response to a Version Negotiation packet.)
void QuicTransport::send_version_negotiation(const uint8_t* d, size_t n, const sockaddr_in& to) {
  if (n < 7) return;
  const size_t dl = d[5];
  if (6 + dl + 1 > n || dl > 20) return;
  const size_t sl = d[6 + dl];
  if (7 + dl + sl > n || sl > 20) return;
  Bytes vn;
  vn.push_back((uint8_t)(0x80 | (rand_cid()[0] & 0x7f)));
  for (int i = 0; i < 4; ++i) vn.push_back(0);                  // version 0 = VN
  vn.push_back((uint8_t)sl);
  vn.insert(vn.end(), d + 7 + dl, d + 7 + dl + sl);             // DCID = client's SCID
  vn.push_back((uint8_t)dl);
  vn.insert(vn.end(), d + 6, d + 6 + dl);                       // SCID = client's DCID
  const uint32_t versions[2] = {0x00000001u, 0x1a2a3a4au};      // v1 + a reserved (greasing) one
  for (uint32_t v : versions)
    for (int i = 3; i >= 0; --i) vn.push_back((uint8_t)(v >> (8 * i)));
  ::sendto(fd_, vn.data(), vn.size(), 0, (const sockaddr*)&to, sizeof(to));
  vn_sent_++;
}

// Retry tokens: expiry (ms since epoch, 8 bytes BE) | odcid len | odcid | 16-byte MAC
// (HMAC-SHA256 under the transport's random key over the client's address + the body).
// The token is bound to the address and to the Retry SCID (= the DCID the client must
// use next), and valid for 10 s.
Bytes QuicTransport::token_mac(const sockaddr_in& peer, const uint8_t* body, size_t n) const {
  Bytes m(body, body + n);
  const uint8_t* ip = reinterpret_cast<const uint8_t*>(&peer.sin_addr);
  m.insert(m.end(), ip, ip + 4);
  m.push_back((uint8_t)(ntohs(peer.sin_port) >> 8));
  m.push_back((uint8_t)ntohs(peer.sin_port));
  Bytes h = hmac256(token_key_, m);
  h.resize(16);
  return h;
}

static uint64_t wall_ms() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::milliseconds>(
             std::chrono::system_clock::now().time_since_epoch()).count();
}

void QuicTransport::send_retry(const Bytes& odcid, const Bytes& client_scid, const sockaddr_in& to) {
  const Bytes rscid = rand_cid();
  Bytes body;
  const uint64_t exp = wall_ms() + 10000;
  for (int i = 7; i >= 0; --i) body.push_back((uint8_t)(exp >> (8 * i)));
  body.push_back((uint8_t)odcid.size());
  body.insert(body.end(), odcid.begin(), odcid.end());
  Bytes bound = body;  // the MAC also covers the SCID the client will address
  bound.insert(bound.end(), rscid.begin(), rscid.end());
  const Bytes mac = token_mac(to, bound.data(), bound.size());
  Bytes pkt;
  pkt.push_back((uint8_t)(0xf0 | (rscid[0] & 0x0f)));  // long header, type 3 (Retry)
  pkt.insert(pkt.end(), {0, 0, 0, 1});
  pkt.push_back((uint8_t)client_scid.size());
  pkt.insert(pkt.end(), client_scid.begin(), client_scid.end());
  pkt.push_back((uint8_t)rscid.size());
  pkt.insert(pkt.end(), rscid.begin(), rscid.end());
  pkt.insert(pkt.end(), body.begin(), body.end());
  pkt.insert(pkt.end(), mac.begin(), mac.end());
  const Bytes tag = retry_tag(odcid, pkt.data(), pkt.size());
  pkt.insert(pkt.end(), tag.begin(), tag.end());
  ::sendto(fd_, pkt.data(), pkt.size(), 0, (const sockaddr*)&to, sizeof(to));
  retries_sent_++;
}

bool QuicTransport::check_token(const Bytes& token, const Bytes& dcid, const sockaddr_in& from,
                                Bytes* odcid) const {
  if (token.size() < 8 + 1 + 16) return false;
  const size_t ol = token[8];
  if (ol > 20 || token.size() != 8 + 1 + ol + 16) return false;
  Bytes bound(token.begin(), token.end() - 16);
  bound.insert(bound.end(), dcid.begin(), dcid.end());
  const Bytes mac = token_mac(from, bound.data(), bound.size());
  if (CRYPTO_memcmp(mac.data(), token.data() + token.size() - 16, 16) != 0) return false;
  uint64_t exp = 0;
  for (int i = 0; i < 8; ++i) exp = (exp << 8) | token[i];
  if (wall_ms() > exp) return false;
  odcid->assign(token.begin() + 9, token.begin() + 9 + ol);
  return true;
}

void QuicTransport::dispatch(const uint8_t* d, size_t n, const sockaddr_in& from) {
  if (n < 1 + QuicConn::kCidLen) return;
  Bytes dcid;
  bool initial = false;
  if (d[0] & 0x80) {
    if (n < 6) return;
    const uint32_t ver = ((uint32_t)d[1] << 24) | ((uint32_t)d[2] << 16) | ((uint32_t)d[3] << 8) | d[4];
    const size_t dl = d[5];
    if (6 + dl > n || dl > 20) return;
    dcid.assign(d + 6, d + 6 + dl);
    if (ver != 1 && ver != 0) {  // unknown version: no connection may have it
      bool listening;
      {
        std::lock_guard<std::mutex> lk(mu_);
        listening = (bool)accept_;
      }
      if (listening && n >= kMaxDatagram) send_version_negotiation(d, n, from);
      return;
    }
    initial = ver == 1 && ((d[0] >> 4) & 3) == 0;
  } else {
    dcid.assign(d + 1, d + 1 + QuicConn::kCidLen);
  }
  QuicConnPtr c;
  {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = by_cid_.find(dcid);
    if (it != by_cid_.end()) c = it->second;
  }
  if (!c) {
    bool listening;
    {
      std::lock_guard<std::mutex> lk(mu_);
      listening = (bool)accept_;
    }
    if (!initial || !listening || n < kMaxDatagram || dcid.size() < 8) return;
    // fresh client Initial: new server-side connection
    const size_t sl = d[6 + dcid.size()];
    if (7 + dcid.size() + sl > n || sl > 20) return;
    const Bytes peer_scid(d + 7 + dcid.size(), d + 7 + dcid.size() + sl);
    size_t tp = 7 + dcid.size() + sl;
    const uint64_t tl = get_varint(d, n, &tp);
    if (tp > n || tl > n - tp) return;
    const Bytes token(d + tp, d + tp + tl);
    Bytes odcid = dcid, retry_scid;
    if (require_retry_) {
      if (token.empty()) {
        send_retry(dcid, peer_scid, from);
        return;
      }
      if (!check_token(token, dcid, from, &odcid)) {  // forged, expired or another path's
        tokens_rejected_++;
        return;
      }
      retry_scid = dcid;  // the client now addresses the Retry's SCID
    }
    c = std::make_shared<QuicConn>(shared_from_this(), false, from, key_);
    const Bytes scid = rand_cid();
    register_cid(scid, c);
    register_cid(dcid, c);
    try {
      c->begin(peer_scid, scid, odcid, dcid, retry_scid);
    } catch (...) {
      forget(c.get());
      return;
    }
  }
  c->on_datagram(d, n);
}

void QuicTransport::loop() {
  std::vector<uint8_t> buf(65536);
  auto last_tick = Clock::now();
  uint64_t rng = 0x9e3779b97f4a7c15ull ^ (uint64_t)port_;
  while (!closed_) {
    pollfd p{fd_, POLLIN, 0};
    ::poll(&p, 1, 5);
    while (!closed_) {
      sockaddr_in from{};
      socklen_t fl = sizeof(from);
      const ssize_t r = ::recvfrom(fd_, buf.data(), buf.size(), MSG_DONTWAIT, (sockaddr*)&from, &fl);
      if (r <= 0) break;
      if (drop_rate_ > 0) {
        rng ^= rng << 13;
        rng ^= rng >> 7;
        rng ^= rng << 17;
        if ((double)(rng >> 11) / (double)(1ull << 53) < drop_rate_) continue;
      }
      try {
        dispatch(buf.data(), (size_t)r, from);
      } catch (...) {
      }
    }
    const auto now = Clock::now();
    if (ms_since(last_tick, now) >= 5) {
      last_tick = now;
      std::vector<QuicConnPtr> conns;
      {
        std::lock_guard<std::mutex> lk(mu_);
        for (auto& kv : by_cid_)
          if (conns.empty() || conns.back() != kv.second) conns.push_back(kv.second);
      }
      std::sort(conns.begin(), conns.end());
      conns.erase(std::unique(conns.begin(), conns.end()), conns.end());
      for (auto& c : conns) {
        try {
          c->tick(now);
        } catch (...) {
        }
      }
    }
  }
}

void QuicTransport::close() {
  if (closed_.exchange(true)) return;
  std::vector<QuicConnPtr> conns;
  {
    std::lock_guard<std::mutex> lk(mu_);
    for (auto& kv : by_cid_) conns.push_back(kv.second);
  }
  std::sort(conns.begin(), conns.end());
  conns.erase(std::unique(conns.begin(), conns.end()), conns.end());
  for (auto& c : conns) c->close();
  if (th_.joinable()) {
    if (th_.get_id() == std::this_thread::get_id()) th_.detach();
    else th_.join();
  }
  for (int i = 0; i < 500 && busy_.load() > 0; ++i)
    std::this_thread::sleep_for(std::chrono::milliseconds(10));
  std::lock_guard<std::mutex> lk(mu_);
  by_cid_.clear();
}

void quic_put_varint(Bytes& b, uint64_t v) { put_varint(b, v); }

Bytes quic_retry_tag(const Bytes& odcid, const uint8_t* retry, size_t len) {
  return retry_tag(odcid, retry, len);
}

}  // namespace p2p
