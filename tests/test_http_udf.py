"""HTTP function UDF (AzureFunctionHandler.scala:14-65, AzureFunctionCaller.scala:21-103): one request per distinct
argument tuple, GET / POST parameter passing, retries, and a per-batch deadline."""
import json
import threading
import time
import urllib.parse
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import pytest

from dxa.engine.column import ConstColumn, column_from_pylist
from dxa.udf.http import HttpFunctionUDF


class _Handler(BaseHTTPRequestHandler):
    calls = []
    fail_first = 0

    def log_message(self, *a):
        pass

    def _reply(self, args):
        type(self).calls.append(args)
        if type(self).fail_first > 0:
            type(self).fail_first -= 1
            self.send_response(500)
            self.end_headers()
            return
        body = ("|".join(f"{k}={args[k]}" for k in sorted(args) if k != "code")).encode()
        self.send_response(200)
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        self.wfile.write(body)

    def do_GET(self):
        q = dict(urllib.parse.parse_qsl(urllib.parse.urlparse(self.path).query, keep_blank_values=True))
        self._reply(q)

    def do_POST(self):
        n = int(self.headers.get("Content-Length") or 0)
        self._reply(json.loads(self.rfile.read(n)))


@pytest.fixture
def server():
    _Handler.calls = []
    _Handler.fail_first = 0
    srv = ThreadingHTTPServer(("127.0.0.1", 0), _Handler)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    yield f"http://127.0.0.1:{srv.server_address[1]}"
    srv.shutdown()


@pytest.mark.parametrize("method", ["get", "post"])
def test_one_request_per_distinct_tuple(server, method):
    udf = HttpFunctionUDF(server, "lookup", "k3y", method, ["a", "b"])
    a = column_from_pylist(["x", "y", "x", None, "x", "y"] * 50, "string", "cpu")
    b = ConstColumn(7, "long", 300, "cpu")
    out = udf([a, b], None, 300, "cpu").to_pylist()
    assert out[:6] == ["a=x|b=7", "a=y|b=7", "a=x|b=7", "a=|b=7", "a=x|b=7", "a=y|b=7"]
    assert len(_Handler.calls) == 3                      # x, y, null
    assert all(c.get("code") == "k3y" for c in _Handler.calls) or method == "post"


def test_retries_then_succeeds(server):
    _Handler.fail_first = 2
    udf = HttpFunctionUDF(server, "f", None, "get", ["a"])
    out = udf([column_from_pylist(["q"], "string", "cpu")], None, 1, "cpu").to_pylist()
    assert out == ["a=q"] and len(_Handler.calls) == 3


def test_deadline_bounds_a_dead_endpoint():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    s.listen(8)                                          # accepts, never answers
    try:
        udf = HttpFunctionUDF(f"http://127.0.0.1:{s.getsockname()[1]}", "f", None, "get", ["a"], retries=5,
                              timeout=10.0, budget_s=0.6)
        t0 = time.monotonic()
        out = udf([column_from_pylist(["p", "q"], "string", "cpu")], None, 2, "cpu").to_pylist()
        assert out == [None, None]
        assert time.monotonic() - t0 < 3.0               # not 5 retries × 10 s
    finally:
        s.close()


def test_empty_batch(server):
    udf = HttpFunctionUDF(server, "f", None, "get", ["a"])
    assert udf([column_from_pylist([], "string", "cpu")], None, 0, "cpu").to_pylist() == []
