"""Loopback integration of the chat plane (BASELINE config 1 plumbing).

Directory + N node daemons on 127.0.0.1 with ephemeral libp2p ports, exactly
the reference's manual test topology (`start_all.sh:5-40`), checked against
the HTTP contracts of SURVEY §2A.1 (`go/cmd/node/main.go:213-283`,
`go/cmd/directory/main.go:57-97`), plus the relay-only path.
"""
import json
import os
import time

import pytest

from netutil import BIN, Procs, free_port, http, wait_http
from p2p_llm_chat_go_amd.native import load as native

pytestmark = pytest.mark.skipif(not os.path.exists(os.path.join(BIN, "p2p-node")),
                                reason="native daemons not built")


@pytest.fixture()
def procs():
    p = Procs()
    yield p
    p.close()


def start_directory(procs, ttl=0):
    port = free_port()
    procs.spawn("p2p-directory", {"ADDR": "127.0.0.1:%d" % port, "DIRECTORY_TTL": str(ttl)})
    url = "http://127.0.0.1:%d" % port
    wait_http(url + "/health")
    return url


def start_node(procs, name, dir_url, extra=None, key="ed25519"):
    port = free_port()
    env = {"MYNAMEIS": name, "HTTP_ADDR": "127.0.0.1:%d" % port, "DIRECTORY_URL": dir_url,
           "KEY_TYPE": key, "LISTEN_ADDRS": "/ip4/127.0.0.1/tcp/0"}
    env.update(extra or {})
    procs.spawn("p2p-node", env)
    url = "http://127.0.0.1:%d" % port
    wait_http(url + "/me")
    return url


# ------------------------------------------------------------------ directory
def test_directory_contract(procs):
    d = start_directory(procs)
    assert http("POST", d + "/register", {"username": "a", "peer_id": "P", "addrs": ["/x"]})[:2] == \
        (200, '{"ok":true}')
    assert http("POST", d + "/register", {"username": "", "peer_id": "P"})[:2] == (400, "missing fields")
    assert http("POST", d + "/register", {"username": "a"})[:2] == (400, "missing fields")
    st, body, _ = http("POST", d + "/register", "not json")
    assert st == 400 and body.startswith("invalid character")
    assert http("POST", d + "/register", "")[:2] == (400, "EOF")
    assert http("GET", d + "/lookup")[:2] == (400, "username required")
    assert http("GET", d + "/lookup?username=zz")[:2] == (404, "not found")
    st, body, hdr = http("GET", d + "/lookup?username=a")
    assert st == 200 and json.loads(body) == {"addrs": ["/x"], "peer_id": "P"}
    assert hdr["Content-Type"].startswith("application/json")
    # last writer wins
    http("POST", d + "/register", {"username": "a", "peer_id": "Q", "addrs": []})
    assert json.loads(http("GET", d + "/lookup?username=a")[1])["peer_id"] == "Q"
    # usernames with reserved characters round-trip through URL escaping
    http("POST", d + "/register", {"username": "a b&c", "peer_id": "R", "addrs": []})
    assert json.loads(http("GET", d + "/lookup?username=a%20b%26c")[1])["peer_id"] == "R"


def test_directory_ttl(procs):
    d = start_directory(procs, ttl=1)
    http("POST", d + "/register", {"username": "a", "peer_id": "P", "addrs": []})
    assert http("GET", d + "/lookup?username=a")[0] == 200
    time.sleep(1.3)
    assert http("GET", d + "/lookup?username=a")[0] == 404


# ------------------------------------------------------------------ nodes
@pytest.mark.parametrize("key", ["ed25519", "rsa"])
def test_two_nodes_send_inbox_me(procs, key):
    d = start_directory(procs)
    a = start_node(procs, "Najy", d, key=key)
    b = start_node(procs, "Cannan", d, key=key)
    st, body, _ = http("GET", a + "/me")
    me = json.loads(body)
    assert st == 200 and list(me) == ["addrs", "peer_id", "username"] and me["username"] == "Najy"
    assert me["peer_id"].startswith("12D3KooW" if key == "ed25519" else "Qm")
    assert all(x.endswith("/p2p/" + me["peer_id"]) for x in me["addrs"])
    # directory holds the same record
    rec = json.loads(http("GET", d + "/lookup?username=Najy")[1])
    assert rec["peer_id"] == me["peer_id"] and rec["addrs"] == me["addrs"]

    assert http("GET", b + "/inbox")[1] == "[]"
    ids = []
    for i in range(3):
        st, body, _ = http("POST", a + "/send", {"to_username": "Cannan", "content": "msg %d <&>" % i})
        r = json.loads(body)
        assert st == 200 and list(r) == ["id", "status"] and r["status"] == "sent"
        ids.append(r["id"])
    for _ in range(100):
        inbox = json.loads(http("GET", b + "/inbox?after=")[1])
        if len(inbox) == 3:
            break
        time.sleep(0.05)
    assert [m["id"] for m in inbox] == ids
    m0 = inbox[0]
    assert list(m0) == ["id", "from_user", "to_user", "content", "timestamp"]
    assert m0["from_user"] == "Najy" and m0["to_user"] == "Cannan" and m0["content"] == "msg 0 <&>"
    from datetime import datetime
    datetime.fromisoformat(m0["timestamp"].replace("Z", "+00:00"))  # reference UI parse_ts
    # Drain(after) semantics: strictly after, non-destructive, unknown id -> []
    assert [m["id"] for m in json.loads(http("GET", b + "/inbox?after=" + ids[0])[1])] == ids[1:]
    assert json.loads(http("GET", b + "/inbox?after=" + ids[2])[1]) == []
    assert json.loads(http("GET", b + "/inbox?after=nope")[1]) == []
    assert len(json.loads(http("GET", b + "/inbox")[1])) == 3
    # reply the other way
    st, _, _ = http("POST", b + "/send", {"to_username": "Najy", "content": "back"})
    assert st == 200
    for _ in range(100):
        got = json.loads(http("GET", a + "/inbox")[1])
        if got:
            break
        time.sleep(0.05)
    assert got[0]["content"] == "back" and got[0]["from_user"] == "Cannan"


def test_send_error_contract(procs):
    d = start_directory(procs)
    a = start_node(procs, "A", d)
    assert http("POST", a + "/send", {"to_username": "ghost", "content": "x"})[:2] == \
        (404, '{"error":"user not found"}')
    st, body, _ = http("POST", a + "/send", {"to_username": "A", "content": "x"})
    assert st == 500 and json.loads(body)["error"].startswith("open stream failed:")
    st, body, _ = http("POST", a + "/send", "{bad")
    assert st == 400 and "error" in json.loads(body)
    st, body, _ = http("POST", a + "/send", {"to_username": 5})
    assert st == 400 and "cannot unmarshal number" in json.loads(body)["error"]
    # a directory entry with an undecodable peer id -> 400 bad peer id
    http("POST", d + "/register", {"username": "bad", "peer_id": "not-a-peer-id", "addrs": []})
    assert http("POST", a + "/send", {"to_username": "bad", "content": "x"})[:2] == \
        (400, '{"error":"bad peer id"}')
    # a registered but unreachable peer -> 500 open stream failed
    from p2p_llm_chat_go_amd.native import load
    _, _, pid = load().keygen("ed25519")
    http("POST", d + "/register", {"username": "gone", "peer_id": pid,
                                   "addrs": ["/ip4/127.0.0.1/tcp/%d/p2p/%s" % (free_port(), pid)]})
    st, body, _ = http("POST", a + "/send", {"to_username": "gone", "content": "x"})
    assert st == 500 and json.loads(body)["error"].startswith("open stream failed:")


def test_directory_down_is_404(procs):
    d = start_directory(procs)
    a = start_node(procs, "A", d)
    procs.procs[0].terminate()
    procs.procs[0].wait()
    assert http("POST", a + "/send", {"to_username": "B", "content": "x"})[:2] == \
        (404, '{"error":"user not found"}')


def test_node_exits_when_directory_unreachable(procs):
    port = free_port()
    p = procs.spawn("p2p-node", {"MYNAMEIS": "x", "HTTP_ADDR": "127.0.0.1:%d" % port,
                                 "DIRECTORY_URL": "http://127.0.0.1:%d" % free_port()})
    assert p.wait(timeout=20) == 1  # log.Fatal("directory register failed")


def test_bootstrap_and_peers(procs):
    d = start_directory(procs)
    a = start_node(procs, "A", d)
    boot = json.loads(http("GET", a + "/me")[1])["addrs"][0]
    b = start_node(procs, "B", d, {"BOOTSTRAP_ADDRS": " %s , /bad/addr ," % boot})
    pid_a = json.loads(http("GET", a + "/me")[1])["peer_id"]
    for _ in range(100):
        peers = json.loads(http("GET", b + "/peers")[1])
        if peers and peers[0]["protocols"]:
            break
        time.sleep(0.05)
    assert peers[0]["peer_id"] == pid_a  # connected via bootstrap, identify ran
    assert "/p2p-llm-chat/1.0.0" in peers[0]["protocols"]


def test_relay_only_path(procs, tmp_path):
    """Node B has no listener; it is reachable only through a circuit-relay-v2 reservation."""
    d = start_directory(procs)
    out = tmp_path / "relay.out"
    with open(out, "w") as f:
        procs.spawn("p2p-relay", {"RELAY_LISTEN": "/ip4/127.0.0.1/tcp/0"}, stdout=f)
    for _ in range(200):
        lines = [x.strip() for x in open(out).read().splitlines() if "/p2p/" in x]
        if lines:
            break
        time.sleep(0.05)
    relay = lines[0]
    a = start_node(procs, "A", d)
    b = start_node(procs, "B", d, {"LISTEN_ADDRS": "none", "RELAY_ADDRS": relay})
    me_b = json.loads(http("GET", b + "/me")[1])
    assert me_b["addrs"] and all("/p2p-circuit/p2p/" in x for x in me_b["addrs"])
    st, body, _ = http("POST", a + "/send", {"to_username": "B", "content": "via relay"})
    assert st == 200, body
    for _ in range(100):
        inbox = json.loads(http("GET", b + "/inbox")[1])
        if inbox:
            break
        time.sleep(0.05)
    assert inbox[0]["content"] == "via relay"
    # and back: B dials A directly
    assert http("POST", b + "/send", {"to_username": "A", "content": "direct back"})[0] == 200


def test_identity_and_inbox_persistence(procs, tmp_path):
    d = start_directory(procs)
    idf, ibf = str(tmp_path / "id.key"), str(tmp_path / "inbox.jsonl")
    a = start_node(procs, "A", d)
    b = start_node(procs, "B", d, {"IDENTITY_FILE": idf, "INBOX_FILE": ibf})
    pid1 = json.loads(http("GET", b + "/me")[1])["peer_id"]
    assert http("POST", a + "/send", {"to_username": "B", "content": "persist me"})[0] == 200
    for _ in range(200):  # "sent" = bytes written; the receiver pushes asynchronously
        if json.loads(http("GET", b + "/inbox")[1]):
            break
        time.sleep(0.05)
    procs.procs[-1].terminate()
    procs.procs[-1].wait()
    b2 = start_node(procs, "B", d, {"IDENTITY_FILE": idf, "INBOX_FILE": ibf})
    assert json.loads(http("GET", b2 + "/me")[1])["peer_id"] == pid1
    assert json.loads(http("GET", b2 + "/inbox")[1])[0]["content"] == "persist me"


def test_suggest_without_engine_is_503(procs):
    d = start_directory(procs)
    a = start_node(procs, "A", d)
    st, body, _ = http("POST", a + "/suggest", {"message": "hi"})
    assert st == 503 and "LLM unavailable" in json.loads(body)["error"]
    assert http("GET", a + "/metrics")[0] == 200


def test_kad_dht_find_peer_through_bootstrap_chain(procs):
    """A <- B <- C bootstrap chain: C never talked to A, yet finds A's addresses by
    an iterative /ipfs/kad/1.0.0 FIND_NODE lookup through B."""
    d = start_directory(procs)
    a = start_node(procs, "A", d)
    me_a = json.loads(http("GET", a + "/me")[1])
    b = start_node(procs, "B", d, {"BOOTSTRAP_ADDRS": me_a["addrs"][0]})
    me_b = json.loads(http("GET", b + "/me")[1])
    c = start_node(procs, "C", d, {"BOOTSTRAP_ADDRS": me_b["addrs"][0]})
    # routing tables fill from identify (peers advertising the kad protocol)
    for _ in range(100):
        pa = [p["peer_id"] for p in json.loads(http("GET", a + "/dht/peers")[1])]
        pc = [p["peer_id"] for p in json.loads(http("GET", c + "/dht/peers")[1])]
        if me_b["peer_id"] in pa and me_b["peer_id"] in pc:
            break
        time.sleep(0.05)
    assert me_b["peer_id"] in pa and me_b["peer_id"] in pc
    assert me_a["peer_id"] not in pc
    st, body, _ = http("GET", c + "/dht/find?peer=" + me_a["peer_id"])
    assert st == 200, body
    found = json.loads(body)
    assert found["peer_id"] == me_a["peer_id"] and found["addrs"]
    assert any(x.split("/p2p/")[0] in found["addrs"] for x in me_a["addrs"])
    # the lookup taught C about A
    pc = [p["peer_id"] for p in json.loads(http("GET", c + "/dht/peers")[1])]
    assert me_a["peer_id"] in pc
    assert http("GET", c + "/dht/find?peer=notapeer")[0] == 400
    # a node started with DHT_MODE=off serves no kad protocol
    e = start_node(procs, "E", d, {"DHT_MODE": "off"})
    assert http("GET", e + "/dht/find?peer=" + me_a["peer_id"])[0] == 503


def test_python_node_cli_flags(procs):
    """`python -m p2p_llm_chat_go_amd.net.node` flags mirror the env vars (flag wins)."""
    import subprocess
    import sys

    d = start_directory(procs)
    port = free_port()
    env = dict(os.environ, MYNAMEIS="from-env", PYTHONPATH=os.path.dirname(BIN))
    p = subprocess.Popen([sys.executable, "-m", "p2p_llm_chat_go_amd.net.node", "--username",
                          "from-flag", "--http-addr", "127.0.0.1:%d" % port, "--directory-url", d,
                          "--engine", "0", "--key-type", "ed25519", "--listen",
                          "/ip4/127.0.0.1/tcp/0"], env=env, stdout=subprocess.DEVNULL,
                         stderr=subprocess.DEVNULL)
    procs.procs.append(p)
    url = "http://127.0.0.1:%d" % port
    wait_http(url + "/me", timeout=60)
    me = json.loads(http("GET", url + "/me")[1])
    assert me["username"] == "from-flag" and me["peer_id"].startswith("12D3KooW")
    assert json.loads(http("GET", d + "/lookup?username=from-flag")[1])["peer_id"] == me["peer_id"]


def test_nat_pmp_port_mapping(procs):
    """NAT_PMP=<gateway>: the node maps its TCP port on the gateway (RFC 6886) and
    advertises the external address (reference: libp2p.NATPortMap()); SIGTERM deletes
    the mapping.  The gateway is a fake NAT-PMP responder on loopback."""
    import socket
    import struct
    import threading

    srv = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    srv.bind(("127.0.0.1", 0))
    srv.settimeout(0.2)
    log = []
    stop = threading.Event()

    def serve():
        while not stop.is_set():
            try:
                data, addr = srv.recvfrom(64)
            except socket.timeout:
                continue
            if data[:2] == b"\x00\x00":
                srv.sendto(struct.pack(">BBHI4B", 0, 128, 0, 1, 203, 0, 113, 7), addr)
            elif data[1] == 2:
                _v, _op, _r, iport, eport, life = struct.unpack(">BBHHHI", data[:12])
                log.append((iport, eport, life))
                srv.sendto(struct.pack(">BBHIHHI", 0, 130, 0, 1, iport,
                                       (iport + 10000) % 65536 if life else 0, life), addr)
    t = threading.Thread(target=serve, daemon=True)
    t.start()
    try:
        d = start_directory(procs)
        a = start_node(procs, "A", d, {"NAT_PMP": "127.0.0.1:%d" % srv.getsockname()[1]})
        me = json.loads(http("GET", a + "/me")[1])
        iport = int(me["addrs"][0].split("/tcp/")[1].split("/")[0])
        ext = "/ip4/203.0.113.7/tcp/%d/p2p/%s" % ((iport + 10000) % 65536, me["peer_id"])
        assert ext in me["addrs"], me["addrs"]
        assert (iport, iport, 3600) in log
        assert ext in json.loads(http("GET", d + "/lookup?username=A")[1])["addrs"]
        node = procs.procs[-1]
        node.terminate()
        node.wait(timeout=10)
        assert any(x[0] == iport and x[2] == 0 for x in log), log  # unmapped on shutdown
    finally:
        stop.set()
        t.join(timeout=2)
        srv.close()


@pytest.mark.parametrize("sec_a,sec_b,ok", [("tls", "tls", True), ("tls,noise", "noise", True),
                                            ("noise,tls", "tls", True), ("tls", "noise", False)])
def test_security_transports(procs, sec_a, sec_b, ok):
    """SECURITY picks the secure channels (go-libp2p hosts offer /tls/1.0.0 and /noise):
    outbound proposals fall through multistream "na" to the next one; with no common
    channel the send fails with the reference's 500 "open stream failed"."""
    d = start_directory(procs)
    a = start_node(procs, "A", d, {"SECURITY": sec_a})
    b = start_node(procs, "B", d, {"SECURITY": sec_b})
    st, body, _ = http("POST", a + "/send", {"to_username": "B", "content": "over " + sec_a})
    if not ok:
        assert st == 500 and json.loads(body)["error"].startswith("open stream failed:")
        return
    assert st == 200, body
    for _ in range(100):
        got = json.loads(http("GET", b + "/inbox")[1])
        if got:
            break
        time.sleep(0.05)
    assert got[0]["content"] == "over " + sec_a and got[0]["from_user"] == "A"
    assert http("POST", b + "/send", {"to_username": "A", "content": "back"})[0] == 200


@pytest.mark.parametrize("sec", ["noise", "tls"])
def test_secure_channel_authenticates_peer(procs, sec):
    """A directory entry that pairs B's addresses with another identity: the secure
    handshake proves B's key, the PeerID check fails, nothing is delivered."""
    from p2p_llm_chat_go_amd.native import load

    d = start_directory(procs)
    a = start_node(procs, "A", d, {"SECURITY": sec})
    b = start_node(procs, "B", d, {"SECURITY": sec})
    me_b = json.loads(http("GET", b + "/me")[1])
    _, _, other = load().keygen("ed25519")
    addrs = [x.split("/p2p/")[0] + "/p2p/" + other for x in me_b["addrs"]]
    http("POST", d + "/register", {"username": "evil", "peer_id": other, "addrs": addrs})
    st, body, _ = http("POST", a + "/send", {"to_username": "evil", "content": "x"})
    assert st == 500 and json.loads(body)["error"].startswith("open stream failed:")
    time.sleep(0.2)
    assert json.loads(http("GET", b + "/inbox")[1]) == []


def test_upnp_igd_port_mapping(procs):
    """UPNP=<ssdp responder>: SSDP M-SEARCH -> device description -> WANIPConnection
    control URL -> GetExternalIPAddress + AddPortMapping; the external address is
    advertised and registered, SIGTERM sends DeletePortMapping (reference:
    libp2p.NATPortMap(), its UPnP half).  The gateway is a fake IGD on loopback."""
    import re
    import socket
    import threading
    from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

    calls = []
    desc = ("<?xml version=\"1.0\"?><root xmlns=\"urn:schemas-upnp-org:device-1-0\"><device>"
            "<deviceType>urn:schemas-upnp-org:device:InternetGatewayDevice:1</deviceType>"
            "<deviceList><device><deviceList><device><serviceList><service>"
            "<serviceType>urn:schemas-upnp-org:service:WANIPConnection:1</serviceType>"
            "<serviceId>urn:upnp-org:serviceId:WANIPConn1</serviceId>"
            "<controlURL>/ctl/IPConn</controlURL></service></serviceList></device></deviceList>"
            "</device></deviceList></device></root>")

    class H(BaseHTTPRequestHandler):
        def log_message(self, *a):
            pass

        def do_GET(self):
            b = desc.encode()
            self.send_response(200)
            self.send_header("Content-Length", str(len(b)))
            self.end_headers()
            self.wfile.write(b)

        def do_POST(self):
            body = self.rfile.read(int(self.headers["Content-Length"])).decode()
            action = self.headers["SOAPAction"].strip('"').split("#")[1]
            calls.append((action, body))
            out = ""
            if action == "GetExternalIPAddress":
                out = "<NewExternalIPAddress>198.51.100.9</NewExternalIPAddress>"
            b = ("<s:Envelope><s:Body><u:%sResponse>%s</u:%sResponse></s:Body></s:Envelope>"
                 % (action, out, action)).encode()
            self.send_response(200)
            self.send_header("Content-Length", str(len(b)))
            self.end_headers()
            self.wfile.write(b)

    web = ThreadingHTTPServer(("127.0.0.1", 0), H)
    threading.Thread(target=web.serve_forever, daemon=True).start()
    ssdp = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    ssdp.bind(("127.0.0.1", 0))
    ssdp.settimeout(0.2)
    stop = threading.Event()

    def answer():
        while not stop.is_set():
            try:
                data, addr = ssdp.recvfrom(2048)
            except socket.timeout:
                continue
            if data.startswith(b"M-SEARCH"):
                ssdp.sendto(("HTTP/1.1 200 OK\r\nST: urn:schemas-upnp-org:device:"
                             "InternetGatewayDevice:1\r\nLOCATION: http://127.0.0.1:%d/rootDesc.xml"
                             "\r\n\r\n" % web.server_address[1]).encode(), addr)
    t = threading.Thread(target=answer, daemon=True)
    t.start()
    try:
        d = start_directory(procs)
        a = start_node(procs, "A", d, {"UPNP": "127.0.0.1:%d" % ssdp.getsockname()[1]})
        me = json.loads(http("GET", a + "/me")[1])
        iport = int(me["addrs"][0].split("/tcp/")[1].split("/")[0])
        ext = "/ip4/198.51.100.9/tcp/%d/p2p/%s" % (iport, me["peer_id"])
        assert ext in me["addrs"], me["addrs"]
        assert ext in json.loads(http("GET", d + "/lookup?username=A")[1])["addrs"]
        add = [b for act, b in calls if act == "AddPortMapping"]
        assert add and "<NewInternalPort>%d</NewInternalPort>" % iport in add[0]
        assert re.search(r"<NewInternalClient>127\.0\.0\.1</NewInternalClient>", add[0])
        node = procs.procs[-1]
        node.terminate()
        node.wait(timeout=10)
        assert any(act == "DeletePortMapping" and "<NewExternalPort>%d<" % iport in b
                   for act, b in calls), [c[0] for c in calls]
    finally:
        stop.set()
        t.join(timeout=2)
        ssdp.close()
        web.shutdown()


_CLUSTER_DP2 = {"ENGINE_GPUS": "2", "ENGINE_VIRTUAL_RANKS": "1", "ENGINE_KV_PAGES": "256",
                "ENGINE_WARMUP": "0", "ENGINE_SD_SEED": "3"}
_CLUSTER_TP2 = dict(_CLUSTER_DP2, ENGINE_TP="2", ENGINE_MODEL="tiny-llama-gqa")


@pytest.mark.parametrize("dev,tokfile,cluster", [
    ("cpu", False, None), pytest.param("cuda:0", False, None, marks=pytest.mark.gpu),
    pytest.param("cuda:0", True, None, marks=pytest.mark.gpu),
    pytest.param("cuda:0", True, _CLUSTER_DP2, marks=pytest.mark.gpu),
    pytest.param("cuda:0", False, _CLUSTER_TP2, marks=pytest.mark.gpu)],
    ids=["cpu", "gpu", "gpu-bpe", "gpu-dp2-bpe", "gpu-tp2"])
def test_node_daemon_hosts_engine_in_process(procs, dev, tokfile, cluster, tmp_path):
    """ENGINE=inproc: the C++ node daemon loads the engine C ABI (libp2p_engine.so,
    csrc/engine/engine_capi.h) and serves /api/generate (plain and streaming NDJSON)
    and /suggest from the engine in its own process -- the node links the engine the
    way the BASELINE north star's Go node links it through cgo (CPU tiny-llama here).
    gpu-bpe: with TOKENIZER_PATH naming a Llama-3-style tokenizer.json the native BPE
    tokenizer (csrc/engine/bpe_tok.h) serves it, still with no interpreter entry.
    gpu-dp2-bpe / gpu-tp2: a multi-GPU node (ENGINE_GPUS=2 replicas, or one ENGINE_TP=2
    group; virtual ranks: every rank process on the box's one GPU) -- the C ABI routes each
    request to a replica leader's native loop over its socket (runtime/loop_remote.h), so
    these serve with no interpreter entry either."""
    lib = os.path.join(os.path.dirname(BIN), "p2p_llm_chat_go_amd", "_lib", "libp2p_engine.so")
    if not os.path.exists(lib):
        pytest.skip("engine C ABI not built")
    d = start_directory(procs)
    port = free_port()
    env = {"MYNAMEIS": "A", "HTTP_ADDR": "127.0.0.1:%d" % port, "DIRECTORY_URL": d,
           "KEY_TYPE": "ed25519", "LISTEN_ADDRS": "/ip4/127.0.0.1/tcp/0", "ENGINE": "inproc",
           "ENGINE_MODEL": "tiny-llama", "ENGINE_DEVICE": dev}
    if tokfile:  # ids < tiny-llama's 512-token vocab: 500 BPE tokens + the 6 specials
        from tokutil import train_bpe_tokenizer

        env["TOKENIZER_PATH"] = train_bpe_tokenizer(tmp_path, vocab=500)
    if cluster:
        env.update(cluster)
    err = open(os.path.join(str(tmp_path), "node.err"), "w")
    procs.spawn("p2p-node", env, stderr=err)

    def log():  # the node's (and its engine's) stderr, for the assertion messages
        err.flush()
        with open(err.name, errors="replace") as f:
            return f.read()[-4000:]

    a = "http://127.0.0.1:%d" % port
    wait_http(a + "/me", timeout=600 if cluster else 120)
    st, body, _ = http("POST", a + "/api/generate", {"model": "llama3.1", "prompt": "hello",
                                                      "stream": False,
                                                      "options": {"num_predict": 5}})
    assert st == 200, (st, body, log())
    out = json.loads(body)
    assert out["done"] and out["eval_count"] == 5 and out["prompt_eval_count"] > 0
    st, body, _ = http("POST", a + "/api/generate", {"model": "llama3.1", "prompt": "hello",
                                                      "options": {"num_predict": 3}})
    lines = [json.loads(x) for x in body.strip().splitlines()]
    assert st == 200 and lines[-1]["done"] and lines[-1]["eval_count"] == 3
    assert "".join(x.get("response", "") for x in lines) == out["response"][:len(
        "".join(x.get("response", "") for x in lines))]
    st, body, _ = http("POST", a + "/suggest", {"message": "Hey! How's it going?"})
    assert st == 200 and "suggestion" in json.loads(body)
    if dev.startswith("cuda"):
        # on a GPU the server runs the native loop and the C ABI serves requests without
        # the interpreter: JSON -> native tokenizer -> EngineLoop -> text -> JSON in C++
        # (the one GIL entry counted is this /metrics call's own)
        m = {}
        for line in http("GET", a + "/metrics")[1].splitlines():
            k, _, v = line.partition(" ")
            m[k] = float(v) if v else 0.0
        assert m.get("p2p_engine_capi_native_requests", 0) >= 3, m
        assert m.get("p2p_engine_capi_native_tokenizer") == 1, m
        assert m.get("p2p_engine_capi_python_tokenize") == 0, m
        assert m.get("p2p_engine_capi_python_decode") == 0, m
        assert m.get("p2p_engine_capi_gil_entries") == 1, m
        st, body, _ = http("POST", a + "/api/generate", {"model": "llama3.1", "stream": False,
                                                          "prompt": "Grüße — 日本語? 😀",
                                                          "options": {"num_predict": 4}})
        assert st == 200 and json.loads(body)["eval_count"] == 4, (st, body, log())
        m2 = {}
        for line in http("GET", a + "/metrics")[1].splitlines():
            k, _, v = line.partition(" ")
            m2[k] = float(v) if v else 0.0
        # non-ASCII text: native with a tokenizer.json, Python's with the synthetic tokenizer
        assert (m2.get("p2p_engine_capi_python_tokenize") == 0) == tokfile, m2
        assert m2.get("p2p_engine_capi_python_decode") == 0, m2
        if cluster:  # served by the replica leaders' loops over their sockets
            assert m2.get("p2p_engine_capi_remote_requests", 0) >= 4, m2


def test_connection_manager_trims_to_low_watermark(procs):
    """CONN_LOW / CONN_HIGH / CONN_GRACE (go-libp2p's connmgr, default 160/192/1 min):
    beyond `high` live connections the least recently used idle ones are closed down
    to `low`; a trimmed peer is re-dialed transparently on its next message."""
    d = start_directory(procs)
    a = start_node(procs, "A", d, {"CONN_LOW": "1", "CONN_HIGH": "2", "CONN_GRACE": "0"})
    me_a = json.loads(http("GET", a + "/me")[1])
    others = [start_node(procs, n, d, {"BOOTSTRAP_ADDRS": me_a["addrs"][0]}) for n in "BCDE"]
    def trimmed():  # Prometheus text exposition
        for line in http("GET", a + "/metrics")[1].splitlines():
            if line.startswith("p2p_connections_trimmed_total "):
                return int(line.split()[1])
        return -1

    for _ in range(100):
        if trimmed() >= 2:
            break
        time.sleep(0.05)
    assert trimmed() >= 2
    assert len(json.loads(http("GET", a + "/peers")[1])) <= 2
    # every peer still reaches A and A reaches every peer (re-dial after trimming)
    for n, u in zip("BCDE", others):
        assert http("POST", u + "/send", {"to_username": "A", "content": "hi " + n})[0] == 200
        assert http("POST", a + "/send", {"to_username": n, "content": "yo " + n})[0] == 200
    for _ in range(100):
        if len(json.loads(http("GET", a + "/inbox")[1])) == 4:
            break
        time.sleep(0.05)
    assert sorted(x["content"] for x in json.loads(http("GET", a + "/inbox")[1])) == \
        ["hi B", "hi C", "hi D", "hi E"]


def test_resource_manager_refuses_inbound_connections(procs):
    """RCMGR_* limits (go-libp2p's resource manager): with no inbound connection
    allowed, B cannot open a connection to A; A can still dial B, and B then reaches A
    over that connection.  The refusal shows in A's /metrics."""
    d = start_directory(procs)
    a = start_node(procs, "A", d, {"RCMGR_SYSTEM_CONNS_INBOUND": "0"})
    b = start_node(procs, "B", d)
    assert http("POST", b + "/send", {"to_username": "A", "content": "blocked"})[0] != 200

    def metric(name):
        for line in http("GET", a + "/metrics")[1].splitlines():
            if line.startswith("p2p_" + name + " "):
                return int(line.split()[1])
        return -1

    assert metric("rcmgr_refused_conns") >= 1
    assert http("POST", a + "/send", {"to_username": "B", "content": "hi B"})[0] == 200
    assert http("POST", b + "/send", {"to_username": "A", "content": "hi A"})[0] == 200
    assert [x["content"] for x in _wait_inbox(a, 1)] == ["hi A"]
    assert metric("rcmgr_conns_outbound") == 1 and metric("rcmgr_conns_inbound") == 0


@pytest.mark.parametrize("transport", ["tcp", "quic"])
def test_resource_manager_stream_limits(transport):
    """Per-peer and per-protocol inbound stream scopes: streams past the limit are
    reset, and the slots come back once the held streams close."""
    accepted, refused, reopened, stats = native().rcmgr_check(transport, 4, 2048, 7)
    assert (accepted, refused, reopened) == (4, 3, True), stats
    assert json.loads(stats)["refused_streams"] == 3
    accepted, refused, reopened, _ = native().rcmgr_check(transport, 100, 3, 6)
    assert (accepted, refused, reopened) == (3, 3, True)


# ------------------------------------------------------------------ QUIC transport
def _wait_inbox(url, n):
    for _ in range(200):
        inbox = json.loads(http("GET", url + "/inbox")[1])
        if len(inbox) >= n:
            return inbox
        time.sleep(0.05)
    return inbox


@pytest.mark.parametrize("key", ["ed25519", "rsa"])
def test_quic_only_nodes_exchange_messages(procs, key):
    """Both nodes listen on /udp/.../quic-v1 only (the reference's second listener,
    `go/cmd/node/main.go:140`): the chat stream runs over a native QUIC stream with
    TLS 1.3 (libp2p certificate) inside the QUIC handshake."""
    d = start_directory(procs)
    q = {"LISTEN_ADDRS": "/ip4/127.0.0.1/udp/0/quic-v1"}
    a = start_node(procs, "A", d, q, key=key)
    b = start_node(procs, "B", d, q, key=key)
    me = json.loads(http("GET", a + "/me")[1])
    assert me["addrs"] and all("/udp/" in x and "/quic-v1/p2p/" in x for x in me["addrs"])
    for i in range(3):
        assert http("POST", a + "/send", {"to_username": "B", "content": "q%d" % i})[0] == 200
    # one stream per message, each handled on its own thread (as the reference's
    # per-stream goroutines, `go/cmd/node/main.go:156-172`): arrival order is not ordered
    assert sorted(m["content"] for m in _wait_inbox(b, 3)) == ["q0", "q1", "q2"]
    assert http("POST", b + "/send", {"to_username": "A", "content": "back"})[0] == 200
    assert _wait_inbox(a, 1)[0]["content"] == "back"
    peers = json.loads(http("GET", a + "/peers")[1])
    assert peers and peers[0]["transport"] == "quic-v1"
    for _ in range(100):  # identify ran over a QUIC stream too
        peers = json.loads(http("GET", a + "/peers")[1])
        if peers[0]["protocols"]:
            break
        time.sleep(0.05)
    assert "/p2p-llm-chat/1.0.0" in peers[0]["protocols"]


@pytest.mark.parametrize("prefer,transport", [("quic", "quic-v1"), ("order", "tcp")])
def test_dial_ranking_tcp_and_quic(procs, prefer, transport):
    """With TCP and QUIC listeners (the reference's default pair), the dialer ranks
    QUIC first like go-libp2p; DIAL_PREFER=order keeps the advertised order (TCP)."""
    d = start_directory(procs)
    both = {"LISTEN_ADDRS": "/ip4/127.0.0.1/tcp/0,/ip4/127.0.0.1/udp/0/quic-v1",
            "DIAL_PREFER": prefer}
    a = start_node(procs, "A", d, both)
    b = start_node(procs, "B", d, both)
    addrs = json.loads(http("GET", b + "/me")[1])["addrs"]
    assert any("/tcp/" in x for x in addrs) and any("/quic-v1/" in x for x in addrs)
    assert http("POST", a + "/send", {"to_username": "B", "content": "hi"})[0] == 200
    assert _wait_inbox(b, 1)[0]["content"] == "hi"
    assert json.loads(http("GET", a + "/peers")[1])[0]["transport"] == transport


def test_inbox_cap_keeps_newest(procs):
    """INBOX_CAP bounds the inbox (the reference's slice grows without bound,
    `go/cmd/node/main.go:102-106`): the newest messages are kept, in order."""
    d = start_directory(procs)
    a = start_node(procs, "A", d)
    b = start_node(procs, "B", d, {"INBOX_CAP": "3"})
    for i in range(5):  # one at a time: each delivered before the next is sent
        st, body, _ = http("POST", a + "/send", {"to_username": "B", "content": "m%d" % i})
        assert st == 200, body
        for _ in range(200):
            inbox = json.loads(http("GET", b + "/inbox")[1])
            if inbox and inbox[-1]["content"] == "m%d" % i:
                break
            time.sleep(0.02)
    assert [m["content"] for m in inbox] == ["m2", "m3", "m4"]


def test_stream_reset_mid_message_leaves_inbox_untouched(procs):
    """SURVEY §5 fault injection "drop connection mid-stream": a sender that resets its
    chat stream before EOF makes the receiver's read fail (the reference's io.ReadAll
    error path, `go/cmd/node/main.go:160-164`): nothing is pushed.  A well-formed stream
    from the same injector (FIN after the JSON) is delivered."""
    d = start_directory(procs)
    b = start_node(procs, "B", d)
    addr = json.loads(http("GET", b + "/me")[1])["addrs"][0]
    msg = {"id": "m-1", "from_user": "X", "to_user": "B", "content": "whole message",
           "timestamp": "2025-09-02T21:11:32.154084+02:00"}
    raw = json.dumps(msg).encode()
    native().chat_inject(addr, raw[:len(raw) // 2], "reset")  # half a message, then RST
    native().chat_inject(addr, raw, "reset")  # a whole JSON body but no EOF: still an error
    time.sleep(0.5)
    assert json.loads(http("GET", b + "/inbox")[1]) == []
    native().chat_inject(addr, raw, "close")
    inbox = _wait_inbox(b, 1)
    assert [m["id"] for m in inbox] == ["m-1"] and inbox[0]["content"] == "whole message"


def test_directory_killed_after_startup_send_is_404(procs):
    """SURVEY §5 fault injection "kill directory": a node that registered and already
    delivered messages answers /send with 404 user not found once the Directory is gone
    (every send looks the recipient up again, `go/cmd/node/main.go:225-228`); its inbox
    and /me keep working."""
    d = start_directory(procs)
    a = start_node(procs, "A", d)
    b = start_node(procs, "B", d)
    assert http("POST", a + "/send", {"to_username": "B", "content": "before"})[0] == 200
    _wait_inbox(b, 1)
    procs.procs[0].terminate()
    procs.procs[0].wait()
    assert http("POST", a + "/send", {"to_username": "B", "content": "after"})[:2] == \
        (404, '{"error":"user not found"}')
    assert len(json.loads(http("GET", b + "/inbox")[1])) == 1
    assert http("GET", a + "/me")[0] == 200
