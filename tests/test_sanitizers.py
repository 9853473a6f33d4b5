"""Sanitizer runs of the native chat plane (SURVEY.md §5 "Race detection /
sanitizers"; the reference has none -- no `go test -race`).

The three daemons are built with ASan+UBSan and with TSan (`_build
--sanitize`), then driven through the full loopback scenario: directory
contract, direct send both ways with RSA and Ed25519 identities, concurrent
sends, the error contract, and the circuit-relay-v2-only path.  Any sanitizer
report on a daemon's stderr fails the test.
"""
import concurrent.futures as cf
import json
import os
import subprocess
import time

import pytest

from netutil import ROOT, free_port, http, wait_http

REPORT_MARKERS = ("ERROR: AddressSanitizer", "runtime error:", "WARNING: ThreadSanitizer",
                  "ERROR: LeakSanitizer", "SUMMARY: UndefinedBehaviorSanitizer")


@pytest.fixture(scope="module", params=["asan", "tsan"])
def sanbin(request):
    from p2p_llm_chat_go_amd import _build

    try:
        _build.build_sanitized(request.param, jobs=min(8, os.cpu_count() or 1))
    except RuntimeError as e:  # toolchain without the sanitizer runtime
        pytest.skip("sanitizer build unavailable: %s" % str(e)[:200])
    return request.param, os.path.join(ROOT, "bin", request.param)


class SanProcs:
    def __init__(self, bindir, logdir, kind):
        self.bindir, self.logdir, self.kind = bindir, logdir, kind
        self.procs = []

    def spawn(self, name, env, stdout=None):
        e = dict(os.environ)
        e.update(env)
        # leak reports would flag the daemons' process-lifetime singletons at SIGTERM
        e["ASAN_OPTIONS"] = "detect_leaks=0:abort_on_error=0"
        e["TSAN_OPTIONS"] = "second_deadlock_stack=1"
        log = os.path.join(self.logdir, "%s-%d.err" % (name, len(self.procs)))
        p = subprocess.Popen([os.path.join(self.bindir, name)], env=e,
                             stdout=stdout or subprocess.DEVNULL, stderr=open(log, "w"))
        self.procs.append((p, log))
        return p

    def close(self):
        for p, _ in self.procs:
            if p.poll() is None:
                p.terminate()
        for p, _ in self.procs:
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()

    def reports(self):
        bad = []
        for _, log in self.procs:
            txt = open(log, errors="replace").read()
            if any(m in txt for m in REPORT_MARKERS):
                bad.append((log, txt[-4000:]))
        return bad


def _node(sp, name, d, extra=None, key="ed25519"):
    port = free_port()
    env = {"MYNAMEIS": name, "HTTP_ADDR": "127.0.0.1:%d" % port, "DIRECTORY_URL": d,
           "KEY_TYPE": key, "LISTEN_ADDRS": "/ip4/127.0.0.1/tcp/0"}
    env.update(extra or {})
    sp.spawn("p2p-node", env)
    url = "http://127.0.0.1:%d" % port
    wait_http(url + "/me", timeout=60)
    return url


def _wait_inbox(url, n, timeout=20):
    t0 = time.time()
    while time.time() - t0 < timeout:
        box = json.loads(http("GET", url + "/inbox")[1])
        if len(box) >= n:
            return box
        time.sleep(0.05)
    return json.loads(http("GET", url + "/inbox")[1])


def test_daemons_clean_under_sanitizer(sanbin, tmp_path):
    kind, bindir = sanbin
    sp = SanProcs(bindir, str(tmp_path), kind)
    try:
        dport = free_port()
        sp.spawn("p2p-directory", {"ADDR": "127.0.0.1:%d" % dport})
        d = "http://127.0.0.1:%d" % dport
        wait_http(d + "/health", timeout=60)
        assert http("GET", d + "/lookup")[0] == 400
        a = _node(sp, "A", d, key="rsa")
        b = _node(sp, "B", d, {"SECURITY": "tls"})  # A proposes noise, falls to TLS
        assert http("POST", a + "/send", {"to_username": "B", "content": "hi"})[0] == 200
        assert http("POST", b + "/send", {"to_username": "A", "content": "yo"})[0] == 200
        # concurrent sends exercise the yamux session / inbox locking across threads
        with cf.ThreadPoolExecutor(8) as ex:
            sts = list(ex.map(lambda i: http("POST", a + "/send",
                                             {"to_username": "B", "content": "m%d" % i})[0],
                              range(16)))
        assert sts == [200] * 16
        assert len(_wait_inbox(b, 17)) == 17
        assert http("POST", a + "/send", {"to_username": "ghost", "content": "x"})[0] == 404
        assert http("POST", a + "/send", {"to_username": "A", "content": "self"})[0] == 500
        assert http("POST", a + "/send", "nope")[0] == 400
        # relay-only node
        out = tmp_path / "relay.out"
        with open(out, "w") as f:
            sp.spawn("p2p-relay", {"RELAY_LISTEN": "/ip4/127.0.0.1/tcp/0"}, stdout=f)
        lines = []
        for _ in range(400):
            lines = [x.strip() for x in open(out).read().splitlines() if "/p2p/" in x]
            if lines:
                break
            time.sleep(0.05)
        assert lines, "relay did not print its address"
        c = _node(sp, "C", d, {"LISTEN_ADDRS": "none", "RELAY_ADDRS": lines[0]})
        assert http("POST", a + "/send", {"to_username": "C", "content": "via relay"})[0] == 200
        assert _wait_inbox(c, 1)[0]["content"] == "via relay"
        # QUIC pair: transport thread, stream readers and senders share each connection
        q = {"LISTEN_ADDRS": "/ip4/127.0.0.1/udp/0/quic-v1"}
        e = _node(sp, "E", d, q)
        f = _node(sp, "F", d, q, key="rsa")
        with cf.ThreadPoolExecutor(8) as ex:
            sts = list(ex.map(lambda i: http("POST", e + "/send",
                                             {"to_username": "F", "content": "q%d" % i})[0],
                              range(16)))
        assert sts == [200] * 16
        assert http("POST", f + "/send", {"to_username": "E", "content": "back"})[0] == 200
        assert len(_wait_inbox(f, 16, timeout=60)) == 16  # TSan: 5-15x slower, PTO backoff
        assert _wait_inbox(e, 1)[0]["content"] == "back"
    finally:
        sp.close()
    bad = sp.reports()
    assert not bad, bad


def test_engine_loop_clean_under_sanitizer(sanbin, tmp_path):
    """The native engine step loop (csrc/runtime/engine_loop.cc) with the host-only HIP
    stand-in and a simulated model (csrc/apps/p2p-loop-selftest.cc): concurrent submitters,
    cancellations, streaming waits and a stall against the loop thread, every reply checked
    and every KV page returned -- under ASan+UBSan and under TSan."""
    kind, bindir = sanbin
    e = dict(os.environ)
    e["ASAN_OPTIONS"] = "detect_leaks=0:abort_on_error=0"
    e["TSAN_OPTIONS"] = "second_deadlock_stack=1"
    r = subprocess.run([os.path.join(bindir, "p2p-loop-selftest")], env=e, stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, text=True, timeout=600)
    assert r.returncode == 0 and "LOOP_SELFTEST_OK" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
    assert not any(m in r.stderr for m in REPORT_MARKERS), r.stderr[-4000:]
