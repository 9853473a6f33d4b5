#include "crypto.h"

#include <openssl/evp.h>
#include <openssl/hmac.h>
#include <openssl/rand.h>
#include <openssl/x509.h>
#include <string.h>

namespace p2p {

namespace {
struct PkeyDel {
  void operator()(EVP_PKEY* p) const { EVP_PKEY_free(p); }
};
struct MdCtxDel {
  void operator()(EVP_MD_CTX* p) const { EVP_MD_CTX_free(p); }
};
struct PctxDel {
  void operator()(EVP_PKEY_CTX* p) const { EVP_PKEY_CTX_free(p); }
};
struct CipherDel {
  void operator()(EVP_CIPHER_CTX* p) const { EVP_CIPHER_CTX_free(p); }
};
using Pkey = std::unique_ptr<EVP_PKEY, PkeyDel>;

[[noreturn]] void fail(const char* what) { throw NetError(std::string("crypto: ") + what); }

Pkey ed25519_priv(const Bytes& seed) {
  Pkey k(EVP_PKEY_new_raw_private_key(EVP_PKEY_ED25519, nullptr, seed.data(), 32));
  if (!k) fail("ed25519 private key");
  return k;
}

Pkey rsa_priv_from_der(const Bytes& der) {
  const unsigned char* p = der.data();
  Pkey k(d2i_PrivateKey(EVP_PKEY_RSA, nullptr, &p, (long)der.size()));
  if (!k) fail("rsa private key DER");
  return k;
}

Bytes rsa_pub_der(EVP_PKEY* k) {
  int n = i2d_PUBKEY(k, nullptr);
  if (n <= 0) fail("i2d_PUBKEY");
  Bytes out(n);
  unsigned char* p = out.data();
  i2d_PUBKEY(k, &p);
  return out;
}

Bytes digest_sign(EVP_PKEY* k, const EVP_MD* md, const Bytes& msg) {
  std::unique_ptr<EVP_MD_CTX, MdCtxDel> ctx(EVP_MD_CTX_new());
  if (EVP_DigestSignInit(ctx.get(), nullptr, md, nullptr, k) != 1) fail("DigestSignInit");
  size_t n = 0;
  if (EVP_DigestSign(ctx.get(), nullptr, &n, msg.data(), msg.size()) != 1) fail("DigestSign len");
  Bytes sig(n);
  if (EVP_DigestSign(ctx.get(), sig.data(), &n, msg.data(), msg.size()) != 1) fail("DigestSign");
  sig.resize(n);
  return sig;
}

bool digest_verify(EVP_PKEY* k, const EVP_MD* md, const Bytes& msg, const Bytes& sig) {
  std::unique_ptr<EVP_MD_CTX, MdCtxDel> ctx(EVP_MD_CTX_new());
  if (EVP_DigestVerifyInit(ctx.get(), nullptr, md, nullptr, k) != 1) return false;
  return EVP_DigestVerify(ctx.get(), sig.data(), sig.size(), msg.data(), msg.size()) == 1;
}
}  // namespace

// ------------------------------------------------------------------ keys
Bytes PublicKey::marshal() const {
  PbWriter w;
  w.varint_field(1, (uint64_t)type_);
  w.bytes_field(2, data_);
  return w.buf;
}

PublicKey PublicKey::unmarshal(const Bytes& pb) {
  PublicKey k;
  bool have_type = false, have_data = false;
  for (auto& f : pb_parse(pb)) {
    if (f.field == 1 && f.wire == 0) {
      k.type_ = (KeyType)f.varint;
      have_type = true;
    } else if (f.field == 2 && f.wire == 2) {
      k.data_ = f.bytes;
      have_data = true;
    }
  }
  if (!have_type || !have_data) fail("bad PublicKey protobuf");
  if (k.type_ == KeyType::Ed25519 && k.data_.size() != 32) fail("bad ed25519 key size");
  if (k.type_ != KeyType::Ed25519 && k.type_ != KeyType::RSA) fail("unsupported key type");
  return k;
}

bool PublicKey::verify(const Bytes& msg, const Bytes& sig) const {
  if (type_ == KeyType::Ed25519) {
    Pkey k(EVP_PKEY_new_raw_public_key(EVP_PKEY_ED25519, nullptr, data_.data(), data_.size()));
    if (!k) return false;
    return digest_verify(k.get(), nullptr, msg, sig);
  }
  if (type_ == KeyType::RSA) {
    const unsigned char* p = data_.data();
    Pkey k(d2i_PUBKEY(nullptr, &p, (long)data_.size()));
    if (!k) return false;
    return digest_verify(k.get(), EVP_sha256(), msg, sig);
  }
  return false;
}

PrivateKey PrivateKey::generate(KeyType t, int bits) {
  PrivateKey out;
  out.type_ = t;
  if (t == KeyType::Ed25519) {
    Bytes seed(32);
    random_bytes(seed.data(), 32);
    Pkey k = ed25519_priv(seed);
    Bytes pub(32);
    size_t n = 32;
    if (EVP_PKEY_get_raw_public_key(k.get(), pub.data(), &n) != 1) fail("ed25519 pub");
    out.data_ = seed;
    append(out.data_, pub);
  } else if (t == KeyType::RSA) {
    Pkey k(EVP_RSA_gen((unsigned)bits));
    if (!k) fail("RSA keygen");
    int n = i2d_PrivateKey(k.get(), nullptr);
    if (n <= 0) fail("i2d_PrivateKey");
    out.data_.resize(n);
    unsigned char* p = out.data_.data();
    i2d_PrivateKey(k.get(), &p);
  } else {
    fail("unsupported key type");
  }
  return out;
}

PublicKey PrivateKey::public_key() const {
  PublicKey pk;
  pk.type_ = type_;
  if (type_ == KeyType::Ed25519) {
    pk.data_.assign(data_.begin() + 32, data_.end());
  } else {
    Pkey k = rsa_priv_from_der(data_);
    pk.data_ = rsa_pub_der(k.get());
  }
  return pk;
}

Bytes PrivateKey::sign(const Bytes& msg) const {
  if (type_ == KeyType::Ed25519) {
    Pkey k = ed25519_priv(Bytes(data_.begin(), data_.begin() + 32));
    return digest_sign(k.get(), nullptr, msg);
  }
  Pkey k = rsa_priv_from_der(data_);
  return digest_sign(k.get(), EVP_sha256(), msg);
}

Bytes PrivateKey::marshal() const {
  PbWriter w;
  w.varint_field(1, (uint64_t)type_);
  w.bytes_field(2, data_);
  return w.buf;
}

PrivateKey PrivateKey::unmarshal(const Bytes& pb) {
  PrivateKey k;
  bool have = false;
  for (auto& f : pb_parse(pb)) {
    if (f.field == 1 && f.wire == 0) k.type_ = (KeyType)f.varint;
    if (f.field == 2 && f.wire == 2) {
      k.data_ = f.bytes;
      have = true;
    }
  }
  if (!have) fail("bad PrivateKey protobuf");
  if (k.type_ == KeyType::Ed25519) {
    if (k.data_.size() == 32) {  // seed only: derive pub
      Pkey p = ed25519_priv(k.data_);
      Bytes pub(32);
      size_t n = 32;
      EVP_PKEY_get_raw_public_key(p.get(), pub.data(), &n);
      append(k.data_, pub);
    }
    if (k.data_.size() != 64) fail("bad ed25519 private key size");
  } else if (k.type_ == KeyType::RSA) {
    rsa_priv_from_der(k.data_);  // validate
  } else {
    fail("unsupported private key type");
  }
  return k;
}

// ------------------------------------------------------------------ peer ids
PeerId PeerId::from_public_key(const PublicKey& k) {
  Bytes pb = k.marshal();
  PeerId id;
  if (pb.size() <= 42) {
    id.mh_.push_back(0x00);
    put_uvarint(id.mh_, pb.size());
    append(id.mh_, pb);
  } else {
    id.mh_ = {0x12, 0x20};
    append(id.mh_, sha256(pb));
  }
  return id;
}

PeerId PeerId::from_bytes(const Bytes& mh) {
  size_t pos = 0;
  uint64_t code = get_uvarint(mh, &pos);
  uint64_t len = get_uvarint(mh, &pos);
  if (pos + len != mh.size()) fail("peer id: bad multihash length");
  if (code == 0x12 && len != 32) fail("peer id: bad sha2-256 length");
  if (code != 0x12 && code != 0x00) fail("peer id: unsupported multihash");
  PeerId id;
  id.mh_ = mh;
  return id;
}

static Bytes base32_decode_lower(const std::string& s) {
  Bytes out;
  uint32_t buf = 0;
  int bits = 0;
  for (char c : s) {
    int v;
    if (c >= 'a' && c <= 'z') v = c - 'a';
    else if (c >= '2' && c <= '7') v = c - '2' + 26;
    else fail("base32: bad character");
    buf = (buf << 5) | (uint32_t)v;
    bits += 5;
    if (bits >= 8) {
      bits -= 8;
      out.push_back((uint8_t)(buf >> bits));
    }
  }
  return out;
}

PeerId PeerId::decode(const std::string& s) {
  if (s.empty()) fail("empty peer id");
  if (s[0] == 'b') {  // CIDv1, multibase base32 (libp2p-key codec 0x72)
    Bytes c = base32_decode_lower(s.substr(1));
    size_t pos = 0;
    if (get_uvarint(c, &pos) != 1) fail("peer id CID: bad version");
    if (get_uvarint(c, &pos) != 0x72) fail("peer id CID: not libp2p-key");
    return from_bytes(Bytes(c.begin() + pos, c.end()));
  }
  return from_bytes(base58_decode(s));
}

bool PeerId::extract_public_key(PublicKey* out) const {
  size_t pos = 0;
  uint64_t code = get_uvarint(mh_, &pos);
  uint64_t len = get_uvarint(mh_, &pos);
  if (code != 0x00) return false;
  *out = PublicKey::unmarshal(Bytes(mh_.begin() + pos, mh_.begin() + pos + len));
  return true;
}

// ------------------------------------------------------------------ primitives
Bytes sha256(const Bytes& data) {
  Bytes out(32);
  unsigned n = 32;
  if (EVP_Digest(data.data(), data.size(), out.data(), &n, EVP_sha256(), nullptr) != 1)
    fail("sha256");
  return out;
}

Bytes hmac_sha256(const Bytes& key, const Bytes& data) {
  Bytes out(32);
  unsigned n = 32;
  if (!HMAC(EVP_sha256(), key.data(), (int)key.size(), data.data(), data.size(), out.data(), &n))
    fail("hmac");
  return out;
}

void random_bytes(uint8_t* out, size_t n) {
  if (RAND_bytes(out, (int)n) != 1) fail("RAND_bytes");
}

X25519Key X25519Key::generate() {
  X25519Key k;
  k.priv.resize(32);
  random_bytes(k.priv.data(), 32);
  Pkey p(EVP_PKEY_new_raw_private_key(EVP_PKEY_X25519, nullptr, k.priv.data(), 32));
  if (!p) fail("x25519 key");
  k.pub.resize(32);
  size_t n = 32;
  if (EVP_PKEY_get_raw_public_key(p.get(), k.pub.data(), &n) != 1) fail("x25519 pub");
  return k;
}

Bytes x25519(const Bytes& priv, const Bytes& peer_pub) {
  if (priv.size() != 32 || peer_pub.size() != 32) fail("x25519: bad key size");
  Pkey a(EVP_PKEY_new_raw_private_key(EVP_PKEY_X25519, nullptr, priv.data(), 32));
  Pkey b(EVP_PKEY_new_raw_public_key(EVP_PKEY_X25519, nullptr, peer_pub.data(), 32));
  if (!a || !b) fail("x25519 keys");
  std::unique_ptr<EVP_PKEY_CTX, PctxDel> ctx(EVP_PKEY_CTX_new(a.get(), nullptr));
  if (EVP_PKEY_derive_init(ctx.get()) != 1 || EVP_PKEY_derive_set_peer(ctx.get(), b.get()) != 1)
    fail("x25519 derive init");
  Bytes out(32);
  size_t n = 32;
  if (EVP_PKEY_derive(ctx.get(), out.data(), &n) != 1) fail("x25519 derive");
  return out;
}

static void make_nonce(uint64_t n, uint8_t iv[12]) {
  memset(iv, 0, 4);
  for (int i = 0; i < 8; ++i) iv[4 + i] = (uint8_t)(n >> (8 * i));
}

Bytes chachapoly_encrypt(const Bytes& key, uint64_t nonce, const Bytes& ad, const Bytes& pt) {
  std::unique_ptr<EVP_CIPHER_CTX, CipherDel> c(EVP_CIPHER_CTX_new());
  uint8_t iv[12];
  make_nonce(nonce, iv);
  int len = 0;
  if (EVP_EncryptInit_ex(c.get(), EVP_chacha20_poly1305(), nullptr, nullptr, nullptr) != 1 ||
      EVP_CIPHER_CTX_ctrl(c.get(), EVP_CTRL_AEAD_SET_IVLEN, 12, nullptr) != 1 ||
      EVP_EncryptInit_ex(c.get(), nullptr, nullptr, key.data(), iv) != 1)
    fail("chachapoly init");
  if (!ad.empty() && EVP_EncryptUpdate(c.get(), nullptr, &len, ad.data(), (int)ad.size()) != 1)
    fail("chachapoly ad");
  Bytes out(pt.size() + 16);
  int n = 0;
  if (!pt.empty() && EVP_EncryptUpdate(c.get(), out.data(), &n, pt.data(), (int)pt.size()) != 1)
    fail("chachapoly enc");
  int f = 0;
  if (EVP_EncryptFinal_ex(c.get(), out.data() + n, &f) != 1) fail("chachapoly final");
  if (EVP_CIPHER_CTX_ctrl(c.get(), EVP_CTRL_AEAD_GET_TAG, 16, out.data() + pt.size()) != 1)
    fail("chachapoly tag");
  return out;
}

Bytes chachapoly_decrypt(const Bytes& key, uint64_t nonce, const Bytes& ad, const Bytes& ct) {
  if (ct.size() < 16) fail("chachapoly: short ciphertext");
  std::unique_ptr<EVP_CIPHER_CTX, CipherDel> c(EVP_CIPHER_CTX_new());
  uint8_t iv[12];
  make_nonce(nonce, iv);
  int len = 0;
  if (EVP_DecryptInit_ex(c.get(), EVP_chacha20_poly1305(), nullptr, nullptr, nullptr) != 1 ||
      EVP_CIPHER_CTX_ctrl(c.get(), EVP_CTRL_AEAD_SET_IVLEN, 12, nullptr) != 1 ||
      EVP_DecryptInit_ex(c.get(), nullptr, nullptr, key.data(), iv) != 1)
    fail("chachapoly init");
  if (!ad.empty() && EVP_DecryptUpdate(c.get(), nullptr, &len, ad.data(), (int)ad.size()) != 1)
    fail("chachapoly ad");
  size_t n_pt = ct.size() - 16;
  Bytes out(n_pt);
  int n = 0;
  if (n_pt && EVP_DecryptUpdate(c.get(), out.data(), &n, ct.data(), (int)n_pt) != 1)
    fail("chachapoly dec");
  if (EVP_CIPHER_CTX_ctrl(c.get(), EVP_CTRL_AEAD_SET_TAG, 16, (void*)(ct.data() + n_pt)) != 1)
    fail("chachapoly set tag");
  int f = 0;
  if (EVP_DecryptFinal_ex(c.get(), out.data() + n, &f) != 1)
    throw NetError("chachapoly: authentication failed");
  return out;
}

}  // namespace p2p
