"""Loopback fixtures: free ports, daemon processes, tiny HTTP client."""
import json
import os
import socket
import subprocess
import time
import urllib.error
import urllib.request

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "bin")


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def http(method, url, body=None, timeout=10):
    data = None
    headers = {}
    if body is not None:
        data = body if isinstance(body, (bytes, str)) else json.dumps(body)
        if isinstance(data, str):
            data = data.encode()
        headers["Content-Type"] = "application/json"
    req = urllib.request.Request(url, data=data, method=method, headers=headers)
    try:
        with urllib.request.urlopen(req, timeout=timeout) as r:
            return r.status, r.read().decode(), dict(r.headers)
    except urllib.error.HTTPError as e:
        return e.code, e.read().decode(), dict(e.headers)


def wait_http(url, timeout=20):
    t0 = time.time()
    while time.time() - t0 < timeout:
        try:
            http("GET", url, timeout=1)
            return True
        except Exception:
            time.sleep(0.05)
    raise TimeoutError(url)


class Procs:
    def __init__(self):
        self.procs = []

    def spawn(self, name, env=None, args=None, stdout=None, stderr=None):
        e = dict(os.environ)
        e.update(env or {})
        cmd = [os.path.join(BIN, name)] if args is None else args
        p = subprocess.Popen(cmd, env=e, stdout=stdout or subprocess.DEVNULL,
                             stderr=stderr or subprocess.DEVNULL)
        self.procs.append(p)
        return p

    def close(self):
        for p in self.procs:
            if p.poll() is None:
                p.terminate()
        for p in self.procs:
            try:
                p.wait(timeout=5)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
