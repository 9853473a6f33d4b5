// Drives the node's browser UI (web/index.html, served by the node at GET /) under
// Node.js with a minimal DOM and a fetch() bound to the node's HTTP API, through the
// reference Streamlit page's user flow (web/streamlit_app.py:140-193): send a message,
// see a received one appear on the 2 s refresh, ask the co-pilot for a suggestion, send
// the AI reply.  Prints one JSON line of observations for tests/test_ui.py to check.
//   node ui_harness.js <node A url> <node B url> <peer B username>
"use strict";
const http = require("http");
const vm = require("vm");

const [A, B, PEER] = process.argv.slice(2);

function request(method, url, body) {
  return new Promise((resolve, reject) => {
    const u = new URL(url);
    const data = body === undefined ? undefined : Buffer.from(body);
    const req = http.request({ host: u.hostname, port: u.port, path: u.pathname + u.search, method,
                               headers: data ? { "Content-Type": "application/json",
                                                 "Content-Length": data.length } : {} }, (res) => {
      const chunks = [];
      res.on("data", (c) => chunks.push(c));
      res.on("end", () => resolve({ status: res.statusCode, text: Buffer.concat(chunks).toString("utf8") }));
    });
    req.on("error", reject);
    req.setTimeout(120000, () => req.destroy(new Error("timeout")));
    if (data) req.write(data);
    req.end();
  });
}

const calls = [];
async function fetchShim(path, opts) {
  opts = opts || {};
  calls.push({ path, method: opts.method || "GET", t: Date.now() });
  const r = await request(opts.method || "GET", A + path, opts.body);
  return { ok: r.status >= 200 && r.status < 300, status: r.status,
           text: async () => r.text, json: async () => JSON.parse(r.text) };
}

const htmlViolations = [];
class El {
  constructor(tag) {
    this.tagName = tag; this.children = []; this.className = ""; this._text = "";
    this.value = ""; this.disabled = false; this.onclick = null;
  }
  set textContent(t) { this._text = String(t); this.children = []; }
  get textContent() { return this._text + this.children.map((c) => c.textContent).join(""); }
  set innerHTML(v) { htmlViolations.push(String(v)); }
  appendChild(c) { this.children.push(c); return c; }
  replaceChildren() { this.children = []; }
}
const ids = {};
for (const id of ["me", "to", "msg", "send", "status", "hist"]) ids[id] = new El(id === "send" ? "button" : "div");
const document = { getElementById: (id) => ids[id], createElement: (t) => new El(t) };
const store = {};
const sessionStorage = { getItem: (k) => (k in store ? store[k] : null), setItem: (k, v) => { store[k] = String(v); } };
const intervals = [];
const ctx = vm.createContext({
  document, sessionStorage, fetch: fetchShim, console, Date, JSON, Object, isNaN, Promise,
  setInterval: (fn, ms) => { intervals.push(ms); return setInterval(fn, ms); },
});

const sleep = (ms) => new Promise((r) => setTimeout(r, ms));
async function until(pred, ms, what) {
  const t0 = Date.now();
  while (Date.now() - t0 < ms) {
    const v = pred();
    if (v) return v;
    await sleep(50);
  }
  throw new Error("timed out waiting for " + what);
}
const kids = () => ids.hist.children;
function buttonAfter(pred, label) {
  const ch = kids();
  const i = ch.findIndex(pred);
  if (i < 0) return null;
  for (let j = i + 1; j < ch.length; ++j) {
    if (ch[j].className.startsWith("bubble")) break;
    if (ch[j].tagName === "button" && ch[j].textContent.startsWith(label)) return ch[j];
  }
  return null;
}

(async () => {
  const page = await request("GET", A + "/");
  const m = /<script>([\s\S]*)<\/script>/.exec(page.text);
  if (page.status !== 200 || !m) throw new Error("GET / did not serve the UI");
  vm.runInContext(m[1], ctx);
  const out = { interval_ms: intervals[0] };
  out.me = await until(() => ids.me.textContent !== "…" && ids.me.textContent, 5000, "/me");

  // 1. send from the form
  ids.to.value = PEER; ids.msg.value = "hello from the ui";
  ids.send.onclick();
  await until(() => ids.status.textContent === "Sent!", 10000, "send");
  out.sent_bubble = kids().some((c) => c.className === "bubble sent" &&
                                       c.textContent.includes("You → " + PEER) &&
                                       c.textContent.includes("hello from the ui"));

  // 2. a message from the peer shows up on the periodic refresh
  const polls0 = calls.filter((c) => c.path.startsWith("/inbox")).length;
  const t0 = Date.now();
  const r = await request("POST", B + "/send", JSON.stringify({ to_username: out.me, content: "how are you?" }));
  if (r.status !== 200) throw new Error("peer send failed: " + r.text);
  const isRecv = (c) => c.className === "bubble recv" && c.textContent.includes("how are you?");
  await until(() => kids().some(isRecv), 8000, "received message rendered");
  out.recv_latency_ms = Date.now() - t0;
  out.recv_text = kids().find(isRecv).textContent;
  await sleep(2300);
  out.inbox_polls = calls.filter((c) => c.path.startsWith("/inbox")).length - polls0;

  // 3. co-pilot suggestion for that message, then send it as the reply
  buttonAfter(isRecv, "🤖 Suggest a reply").onclick();
  const isSug = (c) => c.className === "bubble sug";
  await until(() => kids().some(isSug), 120000, "suggestion rendered");
  out.suggestion_text = kids().find(isSug).textContent;
  const suggest = calls.find((c) => c.path === "/suggest");
  out.suggest_method = suggest && suggest.method;
  ids.status.textContent = "";
  buttonAfter(isSug, "Send AI reply to").onclick();
  await until(() => ids.status.textContent === "Sent!", 10000, "AI reply sent");
  out.html_violations = htmlViolations.length;
  console.log(JSON.stringify(out));
  process.exit(0);
})().catch((e) => { console.log(JSON.stringify({ error: String(e && e.stack || e) })); process.exit(1); });
