// libp2p identity crypto on OpenSSL 3: RSA-2048 (the reference's key type,
// `go/cmd/node/main.go:293-299`) and Ed25519 identities, the libp2p
// PublicKey/PrivateKey protobuf encodings, PeerID derivation, plus the
// primitives Noise XX needs (X25519, ChaCha20-Poly1305, SHA-256, HKDF).
#pragma once
#include <memory>
#include <string>

#include "util.h"

namespace p2p {

enum class KeyType : int { RSA = 0, Ed25519 = 1, Secp256k1 = 2, ECDSA = 3 };

class PublicKey {
 public:
  PublicKey() = default;
  KeyType type() const { return type_; }
  // libp2p protobuf: message PublicKey { KeyType Type = 1; bytes Data = 2; }
  Bytes marshal() const;
  static PublicKey unmarshal(const Bytes& pb);
  bool verify(const Bytes& msg, const Bytes& sig) const;
  const Bytes& raw() const { return data_; }  // RSA: PKIX DER; Ed25519: 32 bytes

 private:
  KeyType type_ = KeyType::Ed25519;
  Bytes data_;
  friend class PrivateKey;
};

class PrivateKey {
 public:
  static PrivateKey generate(KeyType t, int bits = 2048);
  PublicKey public_key() const;
  Bytes sign(const Bytes& msg) const;
  KeyType type() const { return type_; }
  // libp2p protobuf PrivateKey: RSA Data = PKCS#1 DER; Ed25519 Data = priv(32)||pub(32)
  Bytes marshal() const;
  static PrivateKey unmarshal(const Bytes& pb);

 private:
  KeyType type_ = KeyType::Ed25519;
  Bytes data_;
};

// PeerID = multihash(PublicKey protobuf): identity when <= 42 bytes, else sha2-256.
class PeerId {
 public:
  PeerId() = default;
  static PeerId from_public_key(const PublicKey& k);
  static PeerId from_bytes(const Bytes& mh);       // validates the multihash
  static PeerId decode(const std::string& s);      // base58btc (Qm.., 12D3KooW..) or CIDv1 base32
  const Bytes& bytes() const { return mh_; }
  std::string to_base58() const { return base58_encode(mh_); }
  bool empty() const { return mh_.empty(); }
  bool operator==(const PeerId& o) const { return mh_ == o.mh_; }
  bool operator!=(const PeerId& o) const { return mh_ != o.mh_; }
  bool operator<(const PeerId& o) const { return mh_ < o.mh_; }
  // For identity-multihash ids the public key is embedded.
  bool extract_public_key(PublicKey* out) const;
  bool matches(const PublicKey& k) const { return from_public_key(k) == *this; }

 private:
  Bytes mh_;
};

Bytes sha256(const Bytes& data);
Bytes hmac_sha256(const Bytes& key, const Bytes& data);
void random_bytes(uint8_t* out, size_t n);

// X25519
struct X25519Key {
  Bytes priv, pub;  // 32 bytes each
  static X25519Key generate();
};
Bytes x25519(const Bytes& priv, const Bytes& peer_pub);

// ChaCha20-Poly1305 (IETF, 96-bit nonce).  Returns ciphertext||tag.
Bytes chachapoly_encrypt(const Bytes& key, uint64_t nonce, const Bytes& ad, const Bytes& pt);
// Throws NetError on authentication failure.
Bytes chachapoly_decrypt(const Bytes& key, uint64_t nonce, const Bytes& ad, const Bytes& ct);

}  // namespace p2p
