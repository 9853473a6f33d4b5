"""Byte-exact wire fixtures of the libp2p subset, written from the specs (VERDICT r2
"next round" item 8).  Every expected byte string below is built in this file from the
spec text -- multistream-select 1.0, yamux (hashicorp spec), libp2p peer-ids / keys
protobuf, the Noise libp2p handshake payload, the circuit-relay-v2 reservation voucher
(RFC 0002 signed envelope) -- with an independent pure-Python Ed25519 (RFC 8032) and the
OpenSSL command line's RSA DER output, never with our C++ code.  The C++ output must
match byte for byte.  The reference's host is go-libp2p v0.43 (`go/cmd/node/go.mod:8`,
`go/cmd/node/main.go:137-148`); go-libp2p itself cannot run here (no Go, no network), so
"interop" means "identical bytes to the spec", and what the specs leave to the
implementation is listed at the end as parity unpinned."""
import base64
import hashlib

import pytest

from p2p_llm_chat_go_amd.native import available, load

pytestmark = pytest.mark.skipif(not available(), reason="native module not built")


@pytest.fixture(scope="module")
def N():
    m = load()
    m.set_log_quiet(True)
    return m


# ------------------------------------------------------------------ spec helpers
def uvarint(v):
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        out.append(b | (0x80 if v else 0))
        if not v:
            return bytes(out)


def pb_bytes(field, data):  # protobuf wire type 2
    return uvarint(field << 3 | 2) + uvarint(len(data)) + data


def pb_varint(field, v):  # protobuf wire type 0
    return uvarint(field << 3) + uvarint(v)


B58 = "123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz"


def b58(b):
    n = int.from_bytes(b, "big")
    s = ""
    while n:
        n, r = divmod(n, 58)
        s = B58[r] + s
    return "1" * (len(b) - len(b.lstrip(b"\0"))) + s


# RFC 8032 Ed25519, the reference algorithm in pure Python (TEST 1 checked below)
_P = 2 ** 255 - 19
_L = 2 ** 252 + 27742317777372353535851937790883648493


def _inv(x):
    return pow(x, _P - 2, _P)


_D = -121665 * _inv(121666) % _P
_I = pow(2, (_P - 1) // 4, _P)


def _xrec(y):
    xx = (y * y - 1) * _inv(_D * y * y + 1)
    x = pow(xx, (_P + 3) // 8, _P)
    if (x * x - xx) % _P:
        x = x * _I % _P
    return _P - x if x % 2 else x


_BY = 4 * _inv(5) % _P
_BX = _xrec(_BY)
_BASE = (_BX, _BY, 1, _BX * _BY % _P)


def _add(p, q):
    x1, y1, z1, t1 = p
    x2, y2, z2, t2 = q
    a = (y1 - x1) * (y2 - x2) % _P
    b = (y1 + x1) * (y2 + x2) % _P
    c = t1 * 2 * _D * t2 % _P
    d = z1 * 2 * z2 % _P
    e, f, g, h = b - a, d - c, d + c, b + a
    return (e * f % _P, g * h % _P, f * g % _P, e * h % _P)


def _mul(s, p):
    q = (0, 1, 1, 0)
    while s:
        if s & 1:
            q = _add(q, p)
        p = _add(p, p)
        s >>= 1
    return q


def _enc(p):
    x, y, z, _t = p
    zi = _inv(z)
    return ((y * zi % _P) | ((x * zi % _P) & 1) << 255).to_bytes(32, "little")


def _expand(seed):
    h = hashlib.sha512(seed).digest()
    a = int.from_bytes(h[:32], "little") & ((1 << 254) - 8) | (1 << 254)
    return a, h[32:]


def ed25519_pub(seed):
    return _enc(_mul(_expand(seed)[0], _BASE))


def ed25519_sign(seed, msg):
    a, prefix = _expand(seed)
    pk = _enc(_mul(a, _BASE))
    r = int.from_bytes(hashlib.sha512(prefix + msg).digest(), "little") % _L
    R = _enc(_mul(r, _BASE))
    k = int.from_bytes(hashlib.sha512(R + pk + msg).digest(), "little") % _L
    return R + ((r + k * a) % _L).to_bytes(32, "little")


SEED = bytes.fromhex("9d61b19deffd5a60ba844af492ec2cc44449c5697b326919703bac031cae7f60")
SEED2 = bytes.fromhex("4ccd089b28ff96da9db6c346ec114e0f5b8a319f35aba624da8cf6ed4fb8a6fb")
KT_RSA, KT_ED25519 = 0, 1  # libp2p crypto.proto KeyType


def ed_keys(seed):
    """(libp2p PrivateKey protobuf, PublicKey protobuf, PeerID) of an Ed25519 seed: the Go
    private key Data is seed || public key (64 bytes); the PeerID of a key whose public
    protobuf is <= 42 bytes is its identity multihash (0x00, length)."""
    pub = ed25519_pub(seed)
    priv_pb = pb_varint(1, KT_ED25519) + pb_bytes(2, seed + pub)
    pub_pb = pb_varint(1, KT_ED25519) + pb_bytes(2, pub)
    return priv_pb, pub_pb, b58(b"\x00" + uvarint(len(pub_pb)) + pub_pb)


def test_ed25519_reference_vectors():
    """The pure-Python Ed25519 above reproduces RFC 8032 section 7.1 TEST 1 and TEST 2."""
    assert ed25519_pub(SEED).hex() == \
        "d75a980182b10ab7d54bfed3c964073a0ee172f3daa62325af021a68f707511a"
    assert ed25519_sign(SEED, b"").hex() == (
        "e5564300c360ac729086e2cc806e828a84877f1eb8e5d974d873e06522490155"
        "5fb8821590a33bacc61e39701cf9b46bd25bf5f0595bbe24655141438e7a100b")
    assert ed25519_pub(SEED2).hex() == \
        "3d4017c3e843895a92b70aa74d1b7ebc9c982ccf2ec4968cc0cd55f12af4660c"


# ------------------------------------------------------------------ keys / PeerIDs
def test_ed25519_peer_id_and_signature_bytes(N):
    priv_pb, pub_pb, pid = ed_keys(SEED)
    assert pid.startswith("12D3KooW")
    assert N.peer_id_from_public_key(pub_pb) == pid
    assert N.peer_id_decode(pid) == b"\x00\x24" + pub_pb  # identity multihash, 36 bytes
    msg = b"noise-libp2p-static-key:" + bytes(range(32))
    sig = N.sign(priv_pb, msg)
    assert sig == ed25519_sign(SEED, msg)  # Ed25519 is deterministic: exact bytes
    assert N.verify(pub_pb, msg, sig)


# a fixed RSA-2048 key, generated once with `openssl genrsa 2048`; the DER forms are
# `openssl rsa -traditional -outform DER` (PKCS#1) and `openssl rsa -pubout -outform DER` (PKIX)
RSA_PKCS1_DER = bytes.fromhex(
    "308204a30201000282010100b5326637b70f28a00f4e4f0e7ba08a104bc918681a510d961bf085ba80896af0"
    "b74b1d39f212b07ab4b920447a8fdad7c26a3c1fe798c66acb09e8c0516d83e4f6dc7caa818f07091cd8f3c0"
    "16b345dff2b802114da332a1fa149d7fec9ad58c029a2771b671d831b7248270a6ef31cbf076c21f5bd38041"
    "c48fa3f523c4181f84d0b2206e1b9b2206a46e7f6bd04ede379623e5ef18f7e316f5c3dd0e777721ab1c076a"
    "401cde28fc3b52c05021d2ba818f5017f967774c88e6d7f78a95c12b087c7b006972d29ece8959e1855d6eb5"
    "c643c66f86bdd7a9e52827579c52c5184b5ea2fb32fd46f0d571cf60fbde80f70e1e1d1b1a0741b35907cd4e"
    "166f356f02030100010282010016a08c933890f409c8df868fd07063cd55296f9ad06e7ebbd8115921c91b5f"
    "f75f6c49e20a90bae917d8666726c70015217a12b8093bd2cb533f918932a1f26e8d454b6c1f71b4f7365b01"
    "5563804fa17fb5eacc2e5dcadcdf55e3b52ddec7fc0bf72425d71ab05cc4fa122fef28bf9730182475b609db"
    "625b2174e00fef54f3a4c3e07643d67d525b4af1c75a8715b3b89d6f024b2b8fdefe5144da207833e01d3272"
    "ccae68c033787236b6d2a591badf2fb8528dd6a55115febcc2d35559cb62224830e256d0311214d0f2f1fe9f"
    "17e6a97bbf409ccf9cae6960814db6814e9c5dbce4f191ea8fb99fb439af34d2655693b171e44783cede2fb1"
    "11354abb0102818100e5859f092eb3eb3e45e399ccbc23ce554f6eb4bc8bec628b1245aaa757eceada7e4c0e"
    "a25e82ca32e787d09d16c4bd693aa476139a00e0ee6cfe3399d19ecca222ee8a95c8ac1b4a0a6bf9f76016d3"
    "f18d3107366ec96472fc2bef7d3e9562f129138d6d9223aed07cfadb2165987c795b8cee3954562261455a1a"
    "40aa0ab61f02818100ca199ce891562239914a8e8ec43e231b1a2ab2fc868693831df450e878a870fdd1e4be"
    "0025ffb87d715d334737797966c4f5a0a3d5faa22332afc01826d1020665809a7bd0d526b1891f883620b8ee"
    "a5033a35d0db04b57b89f3fe76930c3db51865d227538f648650798618f128b0576134978f434543a8193a9c"
    "40864b76b102818100bb92aaf8ff20ec9474db5f9ad0fad62a24034e53746a97d21df9af50996bb6371fd61a"
    "7399977b9584601b1df6388caf0dcccfee8f023ed0bb64375972d53b591a012662e89fb6a198c8cb7cde1b69"
    "d453560915f40e4438305bdb99d8668f7894e034c9a20fe552df80c74a90d3c08e1142a88153aa1ce8af9bc6"
    "2ea8889e73028180673a8bf612fe5efeeea2998c7cda8c4df4a0a8c9e9e0e58a0c8bd5a3d8b598f95cf3acc5"
    "20a3acd58e491fbf19abd781d1caf0e19e93a5abbae1208a75913eaa8bc013a878b3d74ec98eaca1913744d6"
    "4e7eb62c5722e19c178be48726771331e4236623a63fd105f6270c82c2f398971954a6b18b97de860754f3a8"
    "d5afc8110281805b543621f9c7c8081f6665522ecbe9ca952628b612ad55d482b534eb1c91a0c0d326388714"
    "3794e5c04b814b6db7a5dad4e4aa3a4699877fc6d34ad5ab299e5360cb24b047426cfe269cc4dfb6d024a185"
    "e64863a1a3292d4bbb956b2dbe7c9e101ad4c3fdba0ebff69ba1056cb52355bdd2f6e5160559ad9bdee483d1"
    "684ef4")
RSA_PKIX_PUB_DER = bytes.fromhex(
    "30820122300d06092a864886f70d01010105000382010f003082010a0282010100b5326637b70f28a00f4e4f"
    "0e7ba08a104bc918681a510d961bf085ba80896af0b74b1d39f212b07ab4b920447a8fdad7c26a3c1fe798c6"
    "6acb09e8c0516d83e4f6dc7caa818f07091cd8f3c016b345dff2b802114da332a1fa149d7fec9ad58c029a27"
    "71b671d831b7248270a6ef31cbf076c21f5bd38041c48fa3f523c4181f84d0b2206e1b9b2206a46e7f6bd04e"
    "de379623e5ef18f7e316f5c3dd0e777721ab1c076a401cde28fc3b52c05021d2ba818f5017f967774c88e6d7"
    "f78a95c12b087c7b006972d29ece8959e1855d6eb5c643c66f86bdd7a9e52827579c52c5184b5ea2fb32fd46"
    "f0d571cf60fbde80f70e1e1d1b1a0741b35907cd4e166f356f0203010001")


def test_rsa_peer_id_bytes(N):
    """RSA (the reference's key type, `go/cmd/node/main.go:293-299`): the private key
    protobuf carries PKCS#1 DER, the public one PKIX (SubjectPublicKeyInfo) DER, and the
    PeerID is the sha2-256 multihash of the public protobuf, base58 'Qm...'."""
    priv_pb = pb_varint(1, KT_RSA) + pb_bytes(2, RSA_PKCS1_DER)
    pub_pb = pb_varint(1, KT_RSA) + pb_bytes(2, RSA_PKIX_PUB_DER)
    want = b58(b"\x12\x20" + hashlib.sha256(pub_pb).digest())
    assert want.startswith("Qm") and len(want) == 46
    assert N.peer_id_from_public_key(pub_pb) == want
    msg = b"libp2p wire fixture"
    sig = N.sign(priv_pb, msg)  # PKCS#1 v1.5 / SHA-256 is deterministic too
    assert N.verify(pub_pb, msg, sig) and len(sig) == 256


# ------------------------------------------------------------------ multistream-select
def ms(line):
    return uvarint(len(line) + 1) + line.encode() + b"\n"


def test_multistream_select_dialer_bytes(N):
    """Dialer: header and proposal in one write (go-multistream's lazy/pipelined select):
    <0x13>"/multistream/1.0.0\\n" <0x14>"/p2p-llm-chat/1.0.0\\n"."""
    got = N.wire_ms_select("/p2p-llm-chat/1.0.0")
    assert got == ms("/multistream/1.0.0") + ms("/p2p-llm-chat/1.0.0")
    assert got[:1] == b"\x13" and got[20:21] == b"\x14"
    assert N.wire_ms_select("/yamux/1.0.0") == ms("/multistream/1.0.0") + ms("/yamux/1.0.0")


def test_multistream_listener_na_then_accept(N):
    """Listener: header, then "na" for an unsupported proposal, then the echo of the
    supported one (the Noise-vs-TLS fall-through of a dialer)."""
    chosen, got = N.wire_ms_handle(["/tls/1.0.0", "/noise"], ["/noise"])
    assert chosen == "/noise"
    assert got == ms("/multistream/1.0.0") + ms("na") + ms("/noise")
    assert ms("na") == b"\x03na\n"


# ------------------------------------------------------------------ yamux
def yamux_hdr(typ, flags, sid, length):
    return bytes([0, typ]) + flags.to_bytes(2, "big") + sid.to_bytes(4, "big") + \
        length.to_bytes(4, "big")


def test_yamux_frames_of_one_chat_send(N):
    """One chat message on a fresh dialer session (spec: version 0; types Data 0,
    WindowUpdate 1; flags SYN 1, ACK 2, FIN 4, RST 8; dialer stream ids odd): a
    WindowUpdate+SYN with delta 0 opens stream 1, a Data frame carries the JSON, and a
    WindowUpdate+FIN half-closes it (what lets the receiver's read-to-EOF end,
    `go/cmd/node/main.go:160`)."""
    msg = b'{"id":"x","from_user":"a","to_user":"b","content":"hi","timestamp":"t"}'
    got = N.wire_yamux_client_stream(msg)
    want = yamux_hdr(1, 1, 1, 0) + yamux_hdr(0, 0, 1, len(msg)) + msg + yamux_hdr(1, 4, 1, 0)
    assert got == want


# ------------------------------------------------------------------ Noise payload
def test_noise_handshake_payload_bytes(N):
    """NoiseHandshakePayload {identity_key = 1: PublicKey protobuf, identity_sig = 2:
    sign("noise-libp2p-static-key:" || static X25519 public key), extensions = 4:
    NoiseExtensions {stream_muxers = 2: "/yamux/1.0.0"}} -- Ed25519 signatures are
    deterministic, so the whole payload is a fixed byte string."""
    priv_pb, pub_pb, _ = ed_keys(SEED)
    static_pub = bytes.fromhex("8520f0098930a754748b7ddcb43ef75a0dbf3a0d26381af4eba4a98eaa9b4e6a")
    sig = ed25519_sign(SEED, b"noise-libp2p-static-key:" + static_pub)
    want = pb_bytes(1, pub_pb) + pb_bytes(2, sig) + pb_bytes(4, pb_bytes(2, b"/yamux/1.0.0"))
    got = N.noise_handshake_payload(priv_pb, static_pub)
    assert got == want
    assert got[:2] == b"\x0a\x24" and got[38:40] == b"\x12\x40"


# ------------------------------------------------------------------ relay voucher
def test_relay_reservation_voucher_envelope_bytes(N):
    """Circuit relay v2 reservation voucher: ReservationVoucher {relay = 1, peer = 2
    (PeerID bytes), expiration = 3} in a signed envelope (RFC 0002) {public_key = 1,
    payload_type = 2, payload = 3, signature = 5}; payload_type is the two raw bytes
    0x03 0x02 (go-libp2p circuitv2 proto.RecordCodec; NOT the uvarint 0x82 0x06), and
    the signature covers uvarint-length-prefixed domain "libp2p-relay-rsvp", type and
    payload (the earlier uvarint type broke both directions with go-libp2p)."""
    rpriv, rpub, rpid = ed_keys(SEED)
    _, _, ppid = ed_keys(SEED2)
    expire = 1_760_000_000
    payload = (pb_bytes(1, N.peer_id_decode(rpid)) + pb_bytes(2, N.peer_id_decode(ppid))
               + pb_varint(3, expire))
    ptype = b"\x03\x02"
    dom = b"libp2p-relay-rsvp"
    signed = uvarint(len(dom)) + dom + uvarint(len(ptype)) + ptype + uvarint(len(payload)) + payload
    want = (pb_bytes(1, rpub) + pb_bytes(2, ptype) + pb_bytes(3, payload)
            + pb_bytes(5, ed25519_sign(SEED, signed)))
    got = N.relay_voucher(rpriv, rpid, ppid, expire)
    assert got == want
    assert N.relay_voucher_verify(want, rpid, ppid, expire)
    # the old (uvarint) payload type must not verify
    bad = (pb_bytes(1, rpub) + pb_bytes(2, b"\x82\x06") + pb_bytes(3, payload)
           + pb_bytes(5, ed25519_sign(SEED, signed)))
    assert not N.relay_voucher_verify(bad, rpid, ppid, expire)


# Parity unpinned (the specs leave these to the implementation, so only go-libp2p itself
# could pin them; none is observable in the reference's own files):
#   * the Noise payload's extensions: go-libp2p v0.43 sends stream_muxers only when early
#     muxer negotiation is on for that transport;
#   * the order / merging of yamux frames a Go session writes for the same send (a Go
#     writer may coalesce the SYN into the first Data frame);
#   * RSA signature bytes (PKCS#1 v1.5 / SHA-256 is deterministic, but no Go-produced
#     vector for a key of ours exists here).
