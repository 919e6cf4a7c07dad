"""Azure service wire clients used by the sinks, sources and filesystem layer. Each one is a plain REST call
built from the standard library (``urllib`` + ``hmac``), so there are no SDK dependencies.

* **Blob storage (SharedKey)**: PUT/GET/DELETE blob and list blobs. This is what the reference's HadoopClient does
  through the wasbs driver (DataProcessing/datax-host/src/main/scala/datax/fs/HadoopClient.scala:73-199 resolves the
  account key, :391-439 writes temp-then-rename).
  The account key comes from a storage connection string or from the secret ``<vault>/datax-sa-<account>``
  (HadoopClient.scala:127-153, with the vault read from ``DXA_KEYVAULT``).
* **Event Hubs (SAS)**: HTTPS batch send to ``/<hub>/messages``. The reference uses the AMQP SDK
  (sink/EventHubStreamPoster.scala:15-82, client/eventhub/EventHubSender.scala:13-69). Its Kafka endpoint is served
  by ``io/kafka.py``.
* **Cosmos DB (master key)**: document upsert, mirroring sink/CosmosDBSinker.scala (the reference uses the Spark
  connector's upsert mode).

All endpoints may be local emulators. A loopback host (``127.0.0.1``, ``localhost``) is spoken to over plain HTTP,
which is how the tests drive these clients against in-process fake servers that verify the signatures.
"""
from __future__ import annotations

import base64
import datetime as _dt
import hashlib
import hmac
import json
import os
import re
import time
import urllib.error
import urllib.parse
import urllib.request
import xml.etree.ElementTree as ET
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

BLOB_API_VERSION = "2020-10-02"
COSMOS_API_VERSION = "2018-12-31"
_LOOPBACK = ("127.0.0.1", "localhost", "::1")


class AzureError(RuntimeError):
    def __init__(self, msg: str, status: int = 0):
        super().__init__(msg)
        self.status = status


def _conn_parts(conn: str) -> Dict[str, str]:
    out = {}
    for part in conn.split(";"):
        if "=" in part:
            k, v = part.split("=", 1)
            out[k.strip().lower()] = v.strip()
    return out


def _rfc1123(now: Optional[float] = None) -> str:
    t = _dt.datetime.fromtimestamp(now if now is not None else time.time(), _dt.timezone.utc)
    return t.strftime("%a, %d %b %Y %H:%M:%S GMT")


def _request(method: str, url: str, body: Optional[bytes], headers: Dict[str, str], timeout: float):
    req = urllib.request.Request(url, data=body, method=method, headers=headers)
    try:
        with urllib.request.urlopen(req, timeout=timeout) as r:
            return r.status, dict(r.headers), r.read()
    except urllib.error.HTTPError as e:
        raise AzureError(f"{method} {url} → HTTP {e.code}: {e.read()[:300]!r}", e.code) from None


# ---------------------------------------------------------------------------------------------------------------
# Blob storage
# ---------------------------------------------------------------------------------------------------------------

@dataclass
class StorageAccount:
    name: str
    key: str                       # base64 account key
    endpoint: str                  # e.g. https://acct.blob.core.windows.net  (no trailing slash)


def parse_storage_connection_string(conn: str) -> StorageAccount:
    """``DefaultEndpointsProtocol=https;AccountName=a;AccountKey=k;EndpointSuffix=core.windows.net`` or an
    emulator-style string with ``BlobEndpoint=http://127.0.0.1:10000/a``."""
    p = _conn_parts(conn)
    name, key = p.get("accountname"), p.get("accountkey")
    if not name or not key:
        raise AzureError("storage connection string needs AccountName and AccountKey")
    ep = p.get("blobendpoint")
    if not ep:
        proto = p.get("defaultendpointsprotocol", "https")
        ep = f"{proto}://{name}.blob.{p.get('endpointsuffix', 'core.windows.net')}"
    return StorageAccount(name, key, ep.rstrip("/"))


def shared_key_string_to_sign(account: str, method: str, path: str, query: Dict[str, str],
                              headers: Dict[str, str]) -> str:
    """Blob service SharedKey string-to-sign (version 2009-09-19 and later)."""
    h = {k.lower(): v for k, v in headers.items()}
    length = h.get("content-length", "")
    if length == "0":
        length = ""
    std = [method.upper(), h.get("content-encoding", ""), h.get("content-language", ""), length,
           h.get("content-md5", ""), h.get("content-type", ""), "" if "x-ms-date" in h else h.get("date", ""),
           h.get("if-modified-since", ""), h.get("if-match", ""), h.get("if-none-match", ""),
           h.get("if-unmodified-since", ""), h.get("range", "")]
    canon_headers = "".join(f"{k}:{h[k].strip()}\n" for k in sorted(k for k in h if k.startswith("x-ms-")))
    resource = f"/{account}{path}"
    for k in sorted(query, key=str.lower):
        resource += f"\n{k.lower()}:{query[k]}"
    return "\n".join(std) + "\n" + canon_headers + resource


def sign_shared_key(key_b64: str, string_to_sign: str) -> str:
    mac = hmac.new(base64.b64decode(key_b64), string_to_sign.encode("utf-8"), hashlib.sha256)
    return base64.b64encode(mac.digest()).decode()


class BlobClient:
    def __init__(self, account: StorageAccount, timeout: float = 30.0):
        self.account = account
        self.timeout = timeout
        u = urllib.parse.urlsplit(account.endpoint)
        self._base_path = u.path.rstrip("/")        # emulator endpoints carry "/<account>"

    @classmethod
    def from_connection_string(cls, conn: str, **kw) -> "BlobClient":
        return cls(parse_storage_connection_string(conn), **kw)

    def _call(self, method: str, container: str, blob: str = "", query: Optional[Dict[str, str]] = None,
              body: Optional[bytes] = None, headers: Optional[Dict[str, str]] = None):
        query = dict(query or {})
        path = f"/{container}" + (f"/{urllib.parse.quote(blob)}" if blob else "")
        hdrs = {"x-ms-date": _rfc1123(), "x-ms-version": BLOB_API_VERSION}
        hdrs.update(headers or {})
        if body is not None:
            hdrs["Content-Length"] = str(len(body))
        # the canonical resource uses the URL path as sent (including an emulator's account prefix)
        sts = shared_key_string_to_sign(self.account.name, method, self._base_path + path, query, hdrs)
        hdrs["Authorization"] = f"SharedKey {self.account.name}:{sign_shared_key(self.account.key, sts)}"
        url = self.account.endpoint + path + ("?" + urllib.parse.urlencode(query) if query else "")
        return _request(method, url, body, hdrs, self.timeout)

    def put_blob(self, container: str, blob: str, data: bytes, content_type: str = "application/octet-stream",
                 content_encoding: Optional[str] = None):
        h = {"x-ms-blob-type": "BlockBlob", "Content-Type": content_type}
        if content_encoding:
            h["Content-Encoding"] = content_encoding
        self._call("PUT", container, blob, body=bytes(data), headers=h)

    def get_blob(self, container: str, blob: str) -> bytes:
        return self._call("GET", container, blob)[2]

    def delete_blob(self, container: str, blob: str):
        self._call("DELETE", container, blob)

    def list_blobs(self, container: str, prefix: str = "") -> List[str]:
        names, marker = [], None
        while True:
            q = {"restype": "container", "comp": "list"}
            if prefix:
                q["prefix"] = prefix
            if marker:
                q["marker"] = marker
            body = self._call("GET", container, query=q)[2]
            root = ET.fromstring(body)
            names += [b.findtext("Name") for b in root.iter("Blob")]
            marker = root.findtext("NextMarker")
            if not marker:
                return names


_WASB = re.compile(r"^wasbs?://([^@/]+)@([^./]+)\.blob\.([^/]+)/?(.*)$", re.I)


def parse_wasb_url(url: str) -> Optional[Tuple[str, str, str, str]]:
    """``wasbs://container@account.blob.core.windows.net/path`` → (container, account, suffix, path)."""
    m = _WASB.match(url)
    return m.groups() if m else None


def storage_key_for(account: str) -> Optional[str]:
    """Account key lookup: ``DXA_STORAGE_KEY_<ACCOUNT>``, then the secret ``<DXA_KEYVAULT>/datax-sa-<account>``
    (keyvault:// then secretscope://, as in HadoopClient.resolveStorageAccount)."""
    env = os.environ.get("DXA_STORAGE_KEY_" + re.sub(r"[^A-Za-z0-9]", "_", account).upper())
    if env:
        return env
    vault = os.environ.get("DXA_KEYVAULT")
    if not vault:
        return None
    from ..config import secrets
    for scheme in ("keyvault", "secretscope"):
        try:
            return secrets.resolve(f"{scheme}://{vault}/datax-sa-{account}")
        except secrets.SecretError:
            continue
    return None


def blob_client_for_url(url: str) -> Optional[Tuple[BlobClient, str, str]]:
    """A client plus (container, blob path) for a wasbs URL whose account key is known; None otherwise (the caller
    falls back to the local mapping under ``DXA_FS_ROOT``).  ``DXA_BLOB_ENDPOINT_<ACCOUNT>`` overrides the service
    endpoint (emulators)."""
    parts = parse_wasb_url(url)
    if parts is None:
        return None
    container, account, suffix, path = parts
    key = storage_key_for(account)
    if key is None:
        return None
    ep = os.environ.get("DXA_BLOB_ENDPOINT_" + re.sub(r"[^A-Za-z0-9]", "_", account).upper()) or \
        f"https://{account}.blob.{suffix}"
    return BlobClient(StorageAccount(account, key, ep.rstrip("/"))), container, path


# ---------------------------------------------------------------------------------------------------------------
# Event Hubs (REST send with a SAS token)
# ---------------------------------------------------------------------------------------------------------------

@dataclass
class EventHubConn:
    namespace_uri: str             # https://ns.servicebus.windows.net (or http://127.0.0.1:port)
    key_name: str
    key: str
    entity: Optional[str]


def parse_eventhub_connection_string(conn: str) -> EventHubConn:
    p = _conn_parts(conn)
    ep = p.get("endpoint")
    if not ep or "sharedaccesskey" not in p:
        raise AzureError("event hub connection string needs Endpoint and SharedAccessKey")
    u = urllib.parse.urlsplit(ep)
    host = u.hostname or ""
    scheme = "http" if host in _LOOPBACK else "https"
    return EventHubConn(f"{scheme}://{u.netloc}", p.get("sharedaccesskeyname", ""), p["sharedaccesskey"],
                        p.get("entitypath"))


def sas_token(resource_uri: str, key_name: str, key: str, ttl_s: int = 3600, now: Optional[float] = None) -> str:
    expiry = str(int((now if now is not None else time.time()) + ttl_s))
    encoded = urllib.parse.quote_plus(resource_uri)
    sig = base64.b64encode(hmac.new(key.encode("utf-8"), f"{encoded}\n{expiry}".encode("utf-8"),
                                    hashlib.sha256).digest()).decode()
    return (f"SharedAccessSignature sr={encoded}&sig={urllib.parse.quote_plus(sig)}&se={expiry}"
            f"&skn={urllib.parse.quote_plus(key_name)}")


class EventHubSender:
    """Batch sender; each item becomes one event (``application/vnd.microsoft.servicebus.json`` batch body)."""

    def __init__(self, conn: str, hub: Optional[str] = None, timeout: float = 30.0):
        self.c = parse_eventhub_connection_string(conn)
        self.hub = self.c.entity or hub
        if not self.hub:
            raise AzureError("event hub name missing (EntityPath)")
        self.timeout = timeout

    def send(self, body: bytes, properties: Optional[Dict[str, str]] = None):
        """One event with an arbitrary (e.g. gzip) body; user properties travel as HTTP headers."""
        uri = f"{self.c.namespace_uri}/{self.hub}"
        hdrs = {"Authorization": sas_token(uri, self.c.key_name, self.c.key),
                "Content-Type": "application/atom+xml;type=entry;charset=utf-8"}
        for k, v in (properties or {}).items():
            hdrs[k] = json.dumps(v) if not isinstance(v, str) else f'"{v}"'
        _request("POST", f"{uri}/messages?timeout=60&api-version=2014-01", bytes(body), hdrs, self.timeout)

    def send_batch(self, bodies: List[bytes], properties: Optional[Dict[str, str]] = None):
        if not bodies:
            return
        uri = f"{self.c.namespace_uri}/{self.hub}"
        items = []
        for b in bodies:
            it = {"Body": bytes(b).decode("utf-8", errors="replace")}
            if properties:
                it["UserProperties"] = properties
            items.append(it)
        body = json.dumps(items).encode()
        hdrs = {"Authorization": sas_token(uri, self.c.key_name, self.c.key),
                "Content-Type": "application/vnd.microsoft.servicebus.json"}
        _request("POST", f"{uri}/messages?timeout=60&api-version=2014-01", body, hdrs, self.timeout)


# ---------------------------------------------------------------------------------------------------------------
# Cosmos DB (document upsert with the master key)
# ---------------------------------------------------------------------------------------------------------------

def cosmos_auth(verb: str, resource_type: str, resource_link: str, date: str, key_b64: str) -> str:
    text = f"{verb.lower()}\n{resource_type.lower()}\n{resource_link}\n{date.lower()}\n\n"
    sig = base64.b64encode(hmac.new(base64.b64decode(key_b64), text.encode("utf-8"), hashlib.sha256).digest())
    return urllib.parse.quote(f"type=master&ver=1.0&sig={sig.decode()}", safe="")


class CosmosClient:
    def __init__(self, conn: str, timeout: float = 30.0):
        p = _conn_parts(conn)
        if "accountendpoint" not in p or "accountkey" not in p:
            raise AzureError("cosmos connection string needs AccountEndpoint and AccountKey")
        self.endpoint = p["accountendpoint"].rstrip("/")
        self.key = p["accountkey"]
        self.timeout = timeout

    def upsert(self, db: str, coll: str, doc: Dict, partition_key: Optional[str] = None):
        link = f"dbs/{db}/colls/{coll}"
        date = _rfc1123()
        hdrs = {"Authorization": cosmos_auth("POST", "docs", link, date, self.key), "x-ms-date": date,
                "x-ms-version": COSMOS_API_VERSION, "x-ms-documentdb-is-upsert": "True",
                "Content-Type": "application/json"}
        if partition_key is not None:
            hdrs["x-ms-documentdb-partitionkey"] = json.dumps([doc.get(partition_key)])
        _request("POST", f"{self.endpoint}/{link}/docs", json.dumps(doc).encode(), hdrs, self.timeout)


    # -- reads / deletes (design-time document store: dxa/service/store.py CosmosDocumentStore) -------------------
    def _hdrs(self, verb: str, rtype: str, link: str, partition: Optional[str] = None) -> Dict[str, str]:
        date = _rfc1123()
        h = {"Authorization": cosmos_auth(verb, rtype, link, date, self.key), "x-ms-date": date,
             "x-ms-version": COSMOS_API_VERSION}
        if partition is not None:
            h["x-ms-documentdb-partitionkey"] = json.dumps([partition])
        return h

    def get(self, db: str, coll: str, doc_id: str, partition: Optional[str] = None) -> Optional[Dict]:
        link = f"dbs/{db}/colls/{coll}/docs/{doc_id}"
        try:
            _, _, body = _request("GET", f"{self.endpoint}/{urllib.parse.quote(link)}", None,
                                  self._hdrs("GET", "docs", link, partition), self.timeout)
        except AzureError as e:
            if e.status == 404:
                return None
            raise
        return json.loads(body)

    def delete(self, db: str, coll: str, doc_id: str, partition: Optional[str] = None) -> bool:
        link = f"dbs/{db}/colls/{coll}/docs/{doc_id}"
        try:
            _request("DELETE", f"{self.endpoint}/{urllib.parse.quote(link)}", None,
                     self._hdrs("DELETE", "docs", link, partition), self.timeout)
        except AzureError as e:
            if e.status == 404:
                return False
            raise
        return True

    def list(self, db: str, coll: str) -> List[Dict]:
        """All documents of a collection (ReadFeed, following continuation tokens)."""
        link = f"dbs/{db}/colls/{coll}"
        out: List[Dict] = []
        cont = None
        while True:
            h = self._hdrs("GET", "docs", link)
            if cont:
                h["x-ms-continuation"] = cont
            _, rh, body = _request("GET", f"{self.endpoint}/{link}/docs", None, h, self.timeout)
            out.extend(json.loads(body).get("Documents", []))
            cont = {k.lower(): v for k, v in rh.items()}.get("x-ms-continuation")
            if not cont:
                return out


def is_cosmos_connection(conn: str) -> bool:
    p = _conn_parts(conn)
    return "accountendpoint" in p and "accountkey" in p


def is_eventhub_connection(conn: str) -> bool:
    p = _conn_parts(conn)
    return p.get("endpoint", "").lower().startswith("sb://") and "sharedaccesskey" in p
