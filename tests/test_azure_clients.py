"""Azure REST clients (Blob SharedKey, Event Hubs SAS, Cosmos DB master key) against an in-process fake service.
The fake re-derives each signature from the request it actually received (its own canonicalisation, written
independently here), so a mismatch between what the client signs and what it sends fails the test."""
import base64
import gzip
import hashlib
import hmac
import json
import threading
import urllib.parse
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import pytest

from dxa.io import azure, fs

KEY = base64.b64encode(b"0123456789abcdef0123456789abcdef").decode()
EH_KEY = "ehsecretkey="


class _Fake:
    def __init__(self):
        self.blobs = {}
        self.events = []
        self.docs = {}
        self.errors = []


def _hmac_b64(key: bytes, text: str) -> str:
    return base64.b64encode(hmac.new(key, text.encode(), hashlib.sha256).digest()).decode()


def _make_handler(state: _Fake):
    class H(BaseHTTPRequestHandler):
        def log_message(self, *a):
            pass

        def _body(self):
            n = int(self.headers.get("Content-Length") or 0)
            return self.rfile.read(n) if n else b""

        def _reply(self, code, body=b"", ctype="application/xml"):
            self.send_response(code)
            self.send_header("Content-Type", ctype)
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        # -- blob SharedKey check ------------------------------------------------------------------------------
        def _blob_auth_ok(self):
            u = urllib.parse.urlsplit(self.path)
            hdr = {k.lower(): v for k, v in self.headers.items()}
            length = hdr.get("content-length", "")
            lines = [self.command, hdr.get("content-encoding", ""), hdr.get("content-language", ""),
                     "" if length == "0" else length, hdr.get("content-md5", ""), hdr.get("content-type", ""), "",
                     "", "", "", "", ""]
            xms = sorted((k, v) for k, v in hdr.items() if k.startswith("x-ms-"))
            canon = "".join(f"{k}:{v}\n" for k, v in xms)
            res = "/acct" + u.path
            q = urllib.parse.parse_qs(u.query)
            for k in sorted(q):
                res += f"\n{k}:{','.join(q[k])}"
            want = "SharedKey acct:" + _hmac_b64(base64.b64decode(KEY), "\n".join(lines) + "\n" + canon + res)
            return self.headers.get("Authorization") == want

        def _route(self):
            u = urllib.parse.urlsplit(self.path)
            parts = u.path.split("/")
            if parts[1] == "acct":                                  # /acct/<container>/<blob...>
                if not self._blob_auth_ok():
                    state.errors.append(("blob-auth", self.command, self.path))
                    return self._reply(403)
                container, blob = parts[2], urllib.parse.unquote("/".join(parts[3:]))
                if self.command == "PUT":
                    assert self.headers.get("x-ms-blob-type") == "BlockBlob"
                    state.blobs[(container, blob)] = (self._body(), self.headers.get("Content-Encoding"))
                    return self._reply(201)
                if self.command == "DELETE":
                    state.blobs.pop((container, blob), None)
                    return self._reply(202)
                q = urllib.parse.parse_qs(u.query)
                if q.get("comp") == ["list"]:
                    pre = q.get("prefix", [""])[0]
                    names = sorted(b for c, b in state.blobs if c == container and b.startswith(pre))
                    xml = "<EnumerationResults><Blobs>" + "".join(
                        f"<Blob><Name>{n}</Name></Blob>" for n in names) + "</Blobs><NextMarker/></EnumerationResults>"
                    return self._reply(200, xml.encode())
                if (container, blob) not in state.blobs:
                    return self._reply(404)
                return self._reply(200, state.blobs[(container, blob)][0], "application/octet-stream")
            if parts[1] == "dbs":                                   # /dbs/<db>/colls/<c>/docs[/<id>]
                by_id = len(parts) > 6
                link = urllib.parse.unquote("/".join(parts[1:7] if by_id else parts[1:5]))
                date = self.headers.get("x-ms-date")
                want = urllib.parse.quote("type=master&ver=1.0&sig=" + _hmac_b64(
                    base64.b64decode(KEY), f"{self.command.lower()}\ndocs\n{link}\n{date.lower()}\n\n"), safe="")
                if self.headers.get("Authorization") != want or (
                        self.command == "POST" and self.headers.get("x-ms-documentdb-is-upsert") != "True"):
                    state.errors.append(("cosmos-auth", self.path))
                    return self._reply(401)
                db, coll = parts[2], parts[4]
                if self.command == "POST":
                    doc = json.loads(self._body())
                    state.docs[(db, coll, doc["id"])] = doc
                    return self._reply(201, b"{}", "application/json")
                if by_id:
                    key = (db, coll, urllib.parse.unquote(parts[6]))
                    if key not in state.docs:
                        return self._reply(404, b"{}", "application/json")
                    if self.command == "DELETE":
                        del state.docs[key]
                        return self._reply(204)
                    return self._reply(200, json.dumps({**state.docs[key], "_rid": "x", "_etag": "e"}).encode(),
                                       "application/json")
                docs = [d for (d0, c0, _), d in sorted(state.docs.items()) if (d0, c0) == (db, coll)]
                return self._reply(200, json.dumps({"Documents": docs, "_count": len(docs)}).encode(),
                                   "application/json")
            if len(parts) == 3 and parts[2] == "messages":            # /<hub>/messages
                tok = self.headers.get("Authorization", "")
                fields = dict(kv.split("=", 1) for kv in tok[len("SharedAccessSignature "):].split("&"))
                uri = f"http://{self.headers['Host']}/{parts[1]}"
                sr = urllib.parse.quote_plus(uri)
                sig = _hmac_b64(EH_KEY.encode(), f"{sr}\n{fields['se']}")
                if fields.get("sr") != sr or urllib.parse.unquote_plus(fields.get("sig", "")) != sig or \
                        fields.get("skn") != "send":
                    state.errors.append(("eh-auth", tok))
                    return self._reply(401)
                state.events.append((parts[1], self.headers.get("Content-Type"), self._body(),
                                     self.headers.get("tag")))
                return self._reply(201)
            return self._reply(404)

        do_GET = do_PUT = do_DELETE = do_POST = _route
    return H


@pytest.fixture()
def fake():
    state = _Fake()
    srv = ThreadingHTTPServer(("127.0.0.1", 0), _make_handler(state))
    th = threading.Thread(target=srv.serve_forever, daemon=True)
    th.start()
    state.port = srv.server_address[1]
    yield state
    srv.shutdown()
    srv.server_close()


def test_blob_client_put_get_list_delete(fake):
    conn = f"DefaultEndpointsProtocol=http;AccountName=acct;AccountKey={KEY};BlobEndpoint=http://127.0.0.1:{fake.port}/acct"
    c = azure.BlobClient.from_connection_string(conn)
    c.put_blob("out", "a/b c/part-1.json", b'{"x":1}', "application/json")
    c.put_blob("out", "a/z.bin", b"\x00\x01")
    assert c.get_blob("out", "a/b c/part-1.json") == b'{"x":1}'
    assert c.list_blobs("out", "a/") == ["a/b c/part-1.json", "a/z.bin"]
    c.delete_blob("out", "a/z.bin")
    assert c.list_blobs("out") == ["a/b c/part-1.json"]
    assert not fake.errors


def test_wasbs_paths_go_to_blob_service(fake, monkeypatch):
    monkeypatch.setenv("DXA_STORAGE_KEY_ACCT", KEY)
    monkeypatch.setenv("DXA_BLOB_ENDPOINT_ACCT", f"http://127.0.0.1:{fake.port}/acct")
    base = "wasbs://state@acct.blob.core.windows.net/job1"
    fs.write_atomic(base + "/v1/data.json", '{"k":1}\n', gzip_it=True)
    body, enc = fake.blobs[("state", "job1/v1/data.json")]
    assert enc == "gzip" and gzip.decompress(body) == b'{"k":1}\n'
    assert fs.read_bytes(base + "/v1/data.json") == b'{"k":1}\n'       # gzip-aware read
    assert fs.exists(base + "/v1") and not fs.exists(base + "/v2")
    assert fs.list_files(base) == [] and fs.list_files(base, recursive=True) == [base + "/v1/data.json"]
    fs.delete(base)
    assert not fake.blobs and not fake.errors


def test_storage_key_from_keyvault_secret(fake, monkeypatch, tmp_path):
    monkeypatch.setenv("DXA_KEYVAULT", "myvault")
    monkeypatch.setenv("DXA_SECRETS_DIR", str(tmp_path))
    (tmp_path / "myvault").mkdir()
    (tmp_path / "myvault" / "datax-sa-acct").write_text(KEY)
    assert azure.storage_key_for("acct") == KEY
    assert azure.storage_key_for("other") is None
    assert azure.blob_client_for_url("wasbs://c@other.blob.core.windows.net/x") is None


def test_eventhub_sink_sends_gzip_chunks(fake):
    from dxa.config.settings import SettingDictionary
    from dxa.io.sinks import build_outputs
    conn = f"Endpoint=sb://127.0.0.1:{fake.port}/;SharedAccessKeyName=send;SharedAccessKey={EH_KEY};EntityPath=alerts"
    d = SettingDictionary({"datax.job.output.Alerts.eventhub.connectionstring": conn,
                           "datax.job.output.Alerts.eventhub.compressiontype": "gzip",
                           "datax.job.output.Alerts.eventhub.appendproperty.tag": "dxa"})
    op = build_outputs(d)[0]
    sink = op.sinks[0]
    lines = [json.dumps({"i": i}) for i in range(450)]
    assert sink.write(lines, None, None, None) == 450
    assert not fake.errors
    assert len(fake.events) == 3                                      # chunks of 200 rows, one event each
    got = [l for _, _, body, _ in fake.events for l in gzip.decompress(body).decode().split("\n")]
    assert got == lines
    assert fake.events[0][0] == "alerts" and fake.events[0][3] == '"dxa"'


def test_eventhub_batch_send(fake):
    conn = f"Endpoint=sb://127.0.0.1:{fake.port}/;SharedAccessKeyName=send;SharedAccessKey={EH_KEY}"
    s = azure.EventHubSender(conn, "hub2")
    s.send_batch([b'{"a":1}', b'{"a":2}'])
    hub, ctype, body, _ = fake.events[0]
    assert hub == "hub2" and ctype == "application/vnd.microsoft.servicebus.json"
    assert [json.loads(x["Body"]) for x in json.loads(body)] == [{"a": 1}, {"a": 2}]


def test_cosmos_sink_upserts(fake):
    from dxa.config.settings import SettingDictionary
    from dxa.io.sinks import build_outputs
    conn = f"AccountEndpoint=http://127.0.0.1:{fake.port}/;AccountKey={KEY};"
    d = SettingDictionary({"datax.job.output.Devices.cosmosdb.connectionstring": conn,
                           "datax.job.output.Devices.cosmosdb.database": "iot",
                           "datax.job.output.Devices.cosmosdb.collection": "devices"})
    sink = build_outputs(d)[0].sinks[0]
    assert sink.write([json.dumps({"id": "d1", "t": 1}), json.dumps({"id": "d1", "t": 2}),
                       json.dumps({"id": "d2"})], None, None, None) == 3
    assert not fake.errors
    assert fake.docs[("iot", "devices", "d1")] == {"id": "d1", "t": 2}   # upsert keeps the last write
    assert ("iot", "devices", "d2") in fake.docs


def test_cosmos_document_store_round_trip(fake):
    """The control plane's design-time store over Cosmos DB: flows saved by one control plane are visible to another."""
    from dxa.service.store import CosmosDocumentStore, open_store
    conn = f"AccountEndpoint=http://127.0.0.1:{fake.port}/;AccountKey={KEY};"
    a = open_store(f"cosmos:{conn}Database=dx")
    assert isinstance(a, CosmosDocumentStore) and a.db == "dx"
    a.upsert("flows", "iot", {"name": "iot", "gui": {"x": 1}})
    a.upsert("flows", "home", {"name": "home"})
    b = CosmosDocumentStore(conn, "dx")
    assert b.get("flows", "iot") == {"name": "iot", "gui": {"x": 1}}
    assert [d["name"] for d in b.get_all("flows")] == ["home", "iot"]
    assert b.get("flows", "nope") is None
    assert b.delete("flows", "home") and not b.delete("flows", "home")
    assert [d["name"] for d in a.get_all("flows")] == ["iot"]
    assert not fake.errors
