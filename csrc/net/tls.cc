// libp2p TLS 1.3 (`/tls/1.0.0`) -- see tls.h.
#include "tls.h"

#include <openssl/bio.h>
#include <openssl/bn.h>
#include <openssl/err.h>
#include <openssl/evp.h>
#include <openssl/objects.h>
#include <openssl/ssl.h>
#include <openssl/x509.h>
#include <openssl/x509v3.h>

#include <cstring>

namespace p2p {

const char* kTlsProto = "/tls/1.0.0";

namespace {

const char* kExtOid = "1.3.6.1.4.1.53594.1.1";
const char* kSigPrefix = "libp2p-tls-handshake:";
const char* kYamuxAlpn = "yamux/1.0.0";
// ALPN wire list, client preference: early muxer negotiation, then plain libp2p
const unsigned char kAlpn[] = "\x0byamux/1.0.0\x06libp2p";

std::string ssl_err(const char* what) {
  std::string s = std::string("tls: ") + what;
  unsigned long e;
  while ((e = ERR_get_error()) != 0) {
    char buf[256];
    ERR_error_string_n(e, buf, sizeof(buf));
    s += std::string(" [") + buf + "]";
  }
  return s;
}

void der_len(Bytes& out, size_t n) {
  if (n < 0x80) {
    out.push_back((uint8_t)n);
  } else if (n < 0x100) {
    out.push_back(0x81);
    out.push_back((uint8_t)n);
  } else if (n < 0x10000) {
    out.push_back(0x82);
    out.push_back((uint8_t)(n >> 8));
    out.push_back((uint8_t)n);
  } else {
    out.push_back(0x83);
    out.push_back((uint8_t)(n >> 16));
    out.push_back((uint8_t)(n >> 8));
    out.push_back((uint8_t)n);
  }
}

// reads one DER TLV at *pos with the given tag; returns its contents
bool der_read(const Bytes& d, size_t* pos, uint8_t tag, Bytes* val) {
  size_t p = *pos;
  if (p + 2 > d.size() || d[p] != tag) return false;
  ++p;
  size_t n = d[p++];
  if (n & 0x80) {
    const int k = n & 0x7f;
    if (k < 1 || k > 3 || p + k > d.size()) return false;
    n = 0;
    for (int i = 0; i < k; ++i) n = (n << 8) | d[p++];
  }
  if (p + n > d.size()) return false;
  if (val) val->assign(d.begin() + p, d.begin() + p + n);
  *pos = p + n;
  return true;
}

Bytes spki_der(EVP_PKEY* k) {
  unsigned char* p = nullptr;
  const int n = i2d_PUBKEY(k, &p);
  if (n <= 0) throw NetError(ssl_err("i2d_PUBKEY"));
  Bytes out(p, p + n);
  OPENSSL_free(p);
  return out;
}

// fresh P-256 certificate key + self-signed certificate carrying the SignedKey extension
void make_cert(const PrivateKey& id, EVP_PKEY** key_out, X509** cert_out) {
  EVP_PKEY* ck = EVP_PKEY_Q_keygen(nullptr, nullptr, "EC", "P-256");
  if (!ck) throw NetError(ssl_err("certificate keygen"));
  X509* x = X509_new();
  X509_set_version(x, 2);
  BIGNUM* bn = BN_new();
  BN_rand(bn, 63, BN_RAND_TOP_ANY, BN_RAND_BOTTOM_ANY);
  BN_to_ASN1_INTEGER(bn, X509_get_serialNumber(x));
  BN_free(bn);
  X509_gmtime_adj(X509_getm_notBefore(x), -3600L);
  X509_gmtime_adj(X509_getm_notAfter(x), 100L * 365 * 24 * 3600);
  X509_NAME* nm = X509_get_subject_name(x);
  X509_NAME_add_entry_by_txt(nm, "CN", MBSTRING_ASC, (const unsigned char*)"libp2p", -1, -1, 0);
  X509_set_issuer_name(x, nm);
  X509_set_pubkey(x, ck);
  Bytes msg(kSigPrefix, kSigPrefix + strlen(kSigPrefix));
  const Bytes spki = spki_der(ck);
  msg.insert(msg.end(), spki.begin(), spki.end());
  const Bytes der = tls_signed_key_der(id.public_key().marshal(), id.sign(msg));
  ASN1_OBJECT* obj = OBJ_txt2obj(kExtOid, 1);
  ASN1_OCTET_STRING* os = ASN1_OCTET_STRING_new();
  ASN1_OCTET_STRING_set(os, der.data(), (int)der.size());
  X509_EXTENSION* ext = X509_EXTENSION_create_by_OBJ(nullptr, obj, 0, os);
  const bool ok = ext && X509_add_ext(x, ext, -1) == 1 && X509_sign(x, ck, EVP_sha256()) > 0;
  X509_EXTENSION_free(ext);
  ASN1_OCTET_STRING_free(os);
  ASN1_OBJECT_free(obj);
  if (!ok) {
    X509_free(x);
    EVP_PKEY_free(ck);
    throw NetError(ssl_err("certificate"));
  }
  *key_out = ck;
  *cert_out = x;
}

// authenticates the peer certificate -> its libp2p identity
void verify_peer_cert(X509* pc, PublicKey* key, PeerId* id) {
  EVP_PKEY* pk = X509_get0_pubkey(pc);
  if (!pk || X509_verify(pc, pk) != 1) throw NetError("tls: peer certificate is not self-signed");
  if (X509_cmp_current_time(X509_get0_notBefore(pc)) >= 0 ||
      X509_cmp_current_time(X509_get0_notAfter(pc)) <= 0)
    throw NetError("tls: peer certificate outside its validity period");
  ASN1_OBJECT* obj = OBJ_txt2obj(kExtOid, 1);
  const int idx = X509_get_ext_by_OBJ(pc, obj, -1);
  ASN1_OBJECT_free(obj);
  if (idx < 0) throw NetError("tls: peer certificate lacks the libp2p extension");
  const ASN1_OCTET_STRING* d = X509_EXTENSION_get_data(X509_get_ext(pc, idx));
  const Bytes der(ASN1_STRING_get0_data(d), ASN1_STRING_get0_data(d) + ASN1_STRING_length(d));
  Bytes pb, sig;
  if (!tls_parse_signed_key(der, &pb, &sig)) throw NetError("tls: malformed SignedKey");
  const PublicKey k = PublicKey::unmarshal(pb);
  Bytes msg(kSigPrefix, kSigPrefix + strlen(kSigPrefix));
  const Bytes spki = spki_der(pk);
  msg.insert(msg.end(), spki.begin(), spki.end());
  if (!k.verify(msg, sig)) throw NetError("tls: bad SignedKey signature");
  *key = k;
  *id = PeerId::from_public_key(k);
}

int accept_any_cert(int, X509_STORE_CTX*) { return 1; }  // authenticated after the handshake

int alpn_select(SSL*, const unsigned char** out, unsigned char* outlen, const unsigned char* in,
                unsigned int inlen, void*) {
  // server preference: yamux (early muxer negotiation), else libp2p
  for (const char* want : {kYamuxAlpn, "libp2p"}) {
    const size_t wl = strlen(want);
    for (unsigned i = 0; i < inlen;) {
      const unsigned l = in[i];
      if (i + 1 + l > inlen) break;
      if (l == wl && memcmp(in + i + 1, want, wl) == 0) {
        *out = in + i + 1;
        *outlen = (unsigned char)l;
        return SSL_TLSEXT_ERR_OK;
      }
      i += 1 + l;
    }
  }
  return SSL_TLSEXT_ERR_ALERT_FATAL;
}

}  // namespace

Bytes tls_signed_key_der(const Bytes& pubkey_pb, const Bytes& sig) {
  Bytes body;
  body.push_back(0x04);
  der_len(body, pubkey_pb.size());
  body.insert(body.end(), pubkey_pb.begin(), pubkey_pb.end());
  body.push_back(0x04);
  der_len(body, sig.size());
  body.insert(body.end(), sig.begin(), sig.end());
  Bytes out;
  out.push_back(0x30);
  der_len(out, body.size());
  out.insert(out.end(), body.begin(), body.end());
  return out;
}

void tls_make_cert(const PrivateKey& id, void** key_out, void** cert_out) {
  EVP_PKEY* k = nullptr;
  X509* c = nullptr;
  make_cert(id, &k, &c);
  *key_out = k;
  *cert_out = c;
}

void tls_verify_peer_cert(void* x509, PublicKey* key, PeerId* id) {
  verify_peer_cert((X509*)x509, key, id);
}

bool tls_parse_signed_key(const Bytes& der, Bytes* pubkey_pb, Bytes* sig) {
  size_t p = 0;
  Bytes seq;
  if (!der_read(der, &p, 0x30, &seq) || p != der.size()) return false;
  size_t q = 0;
  return der_read(seq, &q, 0x04, pubkey_pb) && der_read(seq, &q, 0x04, sig) && q == seq.size();
}

std::shared_ptr<TlsConn> TlsConn::handshake(ConnPtr c, const PrivateKey& id_key, bool initiator,
                                            const PeerId& expected) {
  std::shared_ptr<TlsConn> t(new TlsConn());
  t->c_ = std::move(c);
  ERR_clear_error();
  SSL_CTX* ctx = SSL_CTX_new(TLS_method());
  if (!ctx) throw NetError(ssl_err("SSL_CTX_new"));
  t->ctx_ = ctx;
  SSL_CTX_set_min_proto_version(ctx, TLS1_3_VERSION);
  SSL_CTX_set_max_proto_version(ctx, TLS1_3_VERSION);
  SSL_CTX_set_num_tickets(ctx, 0);  // no post-handshake session tickets
  SSL_CTX_set_options(ctx, SSL_OP_NO_TICKET);
  EVP_PKEY* ck = nullptr;
  X509* cert = nullptr;
  make_cert(id_key, &ck, &cert);
  const bool ok = SSL_CTX_use_certificate(ctx, cert) == 1 && SSL_CTX_use_PrivateKey(ctx, ck) == 1;
  X509_free(cert);
  EVP_PKEY_free(ck);
  if (!ok) throw NetError(ssl_err("use certificate"));
  SSL_CTX_set_verify(ctx, SSL_VERIFY_PEER | SSL_VERIFY_FAIL_IF_NO_PEER_CERT, accept_any_cert);
  if (!initiator) SSL_CTX_set_alpn_select_cb(ctx, alpn_select, nullptr);
  SSL* ssl = SSL_new(ctx);
  if (!ssl) throw NetError(ssl_err("SSL_new"));
  t->ssl_ = ssl;
  BIO* rb = BIO_new(BIO_s_mem());
  BIO* wb = BIO_new(BIO_s_mem());
  BIO_set_mem_eof_return(rb, -1);  // empty = "retry", not EOF
  SSL_set_bio(ssl, rb, wb);        // the SSL owns both
  t->rbio_ = rb;
  t->wbio_ = wb;
  if (initiator) {
    SSL_set_alpn_protos(ssl, kAlpn, sizeof(kAlpn) - 1);
    SSL_set_connect_state(ssl);
  } else {
    SSL_set_accept_state(ssl);
  }
  while (true) {
    int r;
    {
      std::unique_lock<std::mutex> lk(t->ssl_mu_);
      r = SSL_do_handshake(ssl);
      t->flush_locked_out(lk);
    }
    if (r == 1) break;
    const int e = SSL_get_error(ssl, r);
    if (e == SSL_ERROR_WANT_READ) {
      if (!t->feed()) throw NetError("tls: connection closed during the handshake");
      continue;
    }
    throw NetError(ssl_err("handshake failed"));
  }
  X509* pc = SSL_get1_peer_certificate(ssl);
  if (!pc) throw NetError("tls: peer sent no certificate");
  try {
    verify_peer_cert(pc, &t->remote_key_, &t->remote_);
  } catch (...) {
    X509_free(pc);
    throw;
  }
  X509_free(pc);
  if (!expected.empty() && t->remote_ != expected)
    throw NetError("tls: peer id mismatch (expected " + expected.to_base58() + ", got " +
                   t->remote_.to_base58() + ")");
  const unsigned char* alpn = nullptr;
  unsigned alen = 0;
  SSL_get0_alpn_selected(ssl, &alpn, &alen);
  if (alen == strlen(kYamuxAlpn) && memcmp(alpn, kYamuxAlpn, alen) == 0) t->muxer_ = kYamuxAlpn;
  return t;
}

TlsConn::~TlsConn() {
  if (ssl_) SSL_free((SSL*)ssl_);  // frees both BIOs
  if (ctx_) SSL_CTX_free((SSL_CTX*)ctx_);
}

// Moves the encrypted bytes the SSL object produced to the socket.  Called with
// ssl_mu_ held; releases it around the socket write (wmu_ orders the writers).
void TlsConn::flush_locked_out(std::unique_lock<std::mutex>& ssl_lk) {
  BIO* wb = (BIO*)wbio_;
  if (BIO_ctrl_pending(wb) == 0) return;
  ssl_lk.unlock();
  {
    std::lock_guard<std::mutex> w(wmu_);
    Bytes out;
    {
      std::lock_guard<std::mutex> l(ssl_mu_);
      const size_t n = BIO_ctrl_pending(wb);
      out.resize(n);
      if (n) out.resize((size_t)std::max(0, BIO_read(wb, out.data(), (int)n)));
    }
    if (!out.empty()) c_->write_all(out.data(), out.size());
  }
  ssl_lk.lock();
}

bool TlsConn::feed() {
  uint8_t buf[16384];
  const size_t n = c_->read_some(buf, sizeof(buf));
  if (n == 0) return false;
  std::lock_guard<std::mutex> l(ssl_mu_);
  return BIO_write((BIO*)rbio_, buf, (int)n) == (int)n;
}

size_t TlsConn::read_some(uint8_t* buf, size_t n) {
  if (n == 0) return 0;
  while (true) {
    {
      std::unique_lock<std::mutex> lk(ssl_mu_);
      if (eof_) return 0;
      ERR_clear_error();
      const int r = SSL_read((SSL*)ssl_, buf, (int)std::min<size_t>(n, 1 << 30));
      const int e = r > 0 ? SSL_ERROR_NONE : SSL_get_error((SSL*)ssl_, r);
      flush_locked_out(lk);  // e.g. a KeyUpdate answer
      if (r > 0) return (size_t)r;
      if (e == SSL_ERROR_ZERO_RETURN) {  // close_notify: the peer closed its write side
        eof_ = true;
        return 0;
      }
      if (e != SSL_ERROR_WANT_READ) throw NetError(ssl_err("read"));
    }
    if (!feed()) return 0;
  }
}

void TlsConn::write_all(const uint8_t* buf, size_t n) {
  std::lock_guard<std::mutex> w(wmu_);
  Bytes out;
  {
    std::lock_guard<std::mutex> l(ssl_mu_);
    ERR_clear_error();
    size_t off = 0;
    while (off < n) {
      const int chunk = (int)std::min<size_t>(n - off, 1 << 20);
      const int r = SSL_write((SSL*)ssl_, buf + off, chunk);
      if (r <= 0) throw NetError(ssl_err("write"));
      off += (size_t)r;
    }
    BIO* wb = (BIO*)wbio_;
    out.resize(BIO_ctrl_pending(wb));
    if (!out.empty()) out.resize((size_t)std::max(0, BIO_read(wb, out.data(), (int)out.size())));
  }
  if (!out.empty()) c_->write_all(out.data(), out.size());
}

void TlsConn::close_write() {
  {
    std::lock_guard<std::mutex> w(wmu_);
    Bytes out;
    {
      std::lock_guard<std::mutex> l(ssl_mu_);
      SSL_shutdown((SSL*)ssl_);  // queues close_notify
      BIO* wb = (BIO*)wbio_;
      out.resize(BIO_ctrl_pending(wb));
      if (!out.empty()) out.resize((size_t)std::max(0, BIO_read(wb, out.data(), (int)out.size())));
    }
    try {
      if (!out.empty()) c_->write_all(out.data(), out.size());
    } catch (...) {
    }
  }
  c_->close_write();
}

}  // namespace p2p
