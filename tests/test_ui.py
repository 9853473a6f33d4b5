"""Browser UI (SURVEY A15 chat UI, A17 suggest / send-AI-reply, A18 2 s refresh) driven
end to end under Node.js: the node serves web/index.html at GET / (UI_FILE), and
tests/ui_harness.js runs its script against a minimal DOM with fetch() bound to the
node's HTTP API, through the reference Streamlit page's flow
(web/streamlit_app.py:140-193): send from the form, a peer's message appears on the
periodic refresh, "Suggest a reply" calls the co-pilot (in-process CPU tiny-llama
engine, ENGINE=inproc), "Send AI reply" delivers it to the peer."""
import json
import os
import shutil
import subprocess

import pytest

from netutil import BIN, Procs, free_port, http, wait_http

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NODE_JS = shutil.which("node") or shutil.which("nodejs")
ENGINE_LIB = os.path.join(ROOT, "p2p_llm_chat_go_amd", "_lib", "libp2p_engine.so")

pytestmark = [
    pytest.mark.skipif(not os.path.exists(os.path.join(BIN, "p2p-node")), reason="native daemons not built"),
    pytest.mark.skipif(NODE_JS is None, reason="no Node.js to run the UI script"),
    pytest.mark.skipif(not os.path.exists(ENGINE_LIB), reason="engine C ABI not built"),
]


@pytest.fixture()
def procs():
    p = Procs()
    yield p
    p.close()


def _node(procs, name, dir_url, extra=None):
    port = free_port()
    env = {"MYNAMEIS": name, "HTTP_ADDR": "127.0.0.1:%d" % port, "DIRECTORY_URL": dir_url,
           "KEY_TYPE": "ed25519", "LISTEN_ADDRS": "/ip4/127.0.0.1/tcp/0",
           "UI_FILE": os.path.join(ROOT, "web", "index.html")}
    env.update(extra or {})
    procs.spawn("p2p-node", env)
    url = "http://127.0.0.1:%d" % port
    wait_http(url + "/me", timeout=120)
    return url


def test_ui_send_refresh_suggest_reply(procs):
    dport = free_port()
    procs.spawn("p2p-directory", {"ADDR": "127.0.0.1:%d" % dport})
    d = "http://127.0.0.1:%d" % dport
    wait_http(d + "/health")
    a = _node(procs, "userA", d, {"ENGINE": "inproc", "ENGINE_MODEL": "tiny-llama",
                                 "ENGINE_DEVICE": "cpu"})
    b = _node(procs, "userB", d)
    st, body, hdr = http("GET", a + "/")
    assert st == 200 and hdr["Content-Type"].startswith("text/html") and "setInterval" in body

    p = subprocess.run([NODE_JS, os.path.join(ROOT, "tests", "ui_harness.js"), a, b, "userB"],
                       capture_output=True, text=True, timeout=300)
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert lines, p.stdout + p.stderr
    out = json.loads(lines[-1])
    assert "error" not in out, out["error"]
    assert out["me"] == "userA"
    assert out["interval_ms"] == 2000  # the reference's 2 s refresh (streamlit_app.py:193)
    assert out["sent_bubble"]
    assert "userB → You" in out["recv_text"] and "how are you?" in out["recv_text"]
    assert out["recv_latency_ms"] < 4500  # picked up by the next poll, not a reload
    assert 1 <= out["inbox_polls"] <= 3  # ~one poll per 2 s over the 2.3 s window
    assert out["suggest_method"] == "POST"
    assert out["suggestion_text"].startswith("💡 AI Suggestion:")
    assert out["html_violations"] == 0  # message text never goes through innerHTML

    # B's inbox holds the form message and the AI reply, in order
    inbox = json.loads(http("GET", b + "/inbox")[1])
    contents = [m["content"] for m in inbox if m["from_user"] == "userA"]
    suggestion = out["suggestion_text"][len("💡 AI Suggestion:"):]
    assert contents[0] == "hello from the ui"
    assert len(contents) == 2 and suggestion.startswith(contents[1])
