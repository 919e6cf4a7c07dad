"""AMQP 1.0 receiver for Azure Event Hubs / IoT Hub's Event Hub-compatible endpoint — the direct stream the
reference reads with azure-eventhubs-spark (DataProcessing/datax-host/src/main/scala/datax/input/
EventHubStreamingFactory.scala:23-118; settings EventHubInputSetting.scala:24-31), written against the protocol with
the standard library (no AMQP package is available here).

* transport: TCP (+ TLS for ``amqps``, port 5671), the SASL layer (PLAIN with the shared-access key name / key —
  Event Hubs accepts it in place of a CBS token — or ANONYMOUS), then the AMQP layer: open, begin, attach;
* per partition one receiver link on ``<hub>/ConsumerGroups/<group>/Partitions/<id>`` with the Event Hubs selector
  filter (``amqp.annotation.x-opt-sequence-number > 'N'`` or ``x-opt-enqueued-time > 'ms'``), settled delivery, and
  link credit replenished as messages arrive;
* a message's ``data`` sections are the event body; its ``application-properties`` become the event's Properties
  and the ``x-opt-*`` message annotations (sequence number, offset, enqueued time, partition key) its
  SystemProperties — the columns DirectProcessor builds from EventData;
* the partition ids come from the ``$management`` node (``READ`` of ``com.microsoft:eventhub``).

``AmqpCodec`` covers the AMQP type system these frames use: null, booleans, (u)byte/short/int/long, float/double,
timestamp, uuid, binary, string, symbol, list, map, array and described types.
"""
from __future__ import annotations

import socket
import ssl
import struct
import threading
import time
import uuid
from typing import Any, Dict, List, Optional, Tuple


class AmqpError(Exception):
    pass


class Described:
    __slots__ = ("descriptor", "value")

    def __init__(self, descriptor, value):
        self.descriptor = descriptor
        self.value = value

    def __repr__(self):
        return f"Described({self.descriptor!r}, {self.value!r})"

    def __eq__(self, o):
        return isinstance(o, Described) and (self.descriptor, self.value) == (o.descriptor, o.value)


class Symbol(str):
    pass


class ULong(int):
    pass


class UInt(int):
    pass


class UByte(int):
    pass


class UShort(int):
    pass


class Timestamp(int):
    """Milliseconds since the epoch."""


# ---------------------------------------------------------------------------------------------------------------
# codec
# ---------------------------------------------------------------------------------------------------------------

def encode(v) -> bytes:
    if v is None:
        return b"\x40"
    if isinstance(v, Described):
        return b"\x00" + encode(v.descriptor) + encode(v.value)
    if isinstance(v, bool):
        return b"\x41" if v else b"\x42"
    if isinstance(v, ULong):
        if v == 0:
            return b"\x44"
        if v < 256:
            return b"\x53" + struct.pack(">B", v)
        return b"\x80" + struct.pack(">Q", v)
    if isinstance(v, UInt):
        if v == 0:
            return b"\x43"
        if v < 256:
            return b"\x52" + struct.pack(">B", v)
        return b"\x70" + struct.pack(">I", v)
    if isinstance(v, UShort):
        return b"\x60" + struct.pack(">H", v)
    if isinstance(v, UByte):
        return b"\x50" + struct.pack(">B", v)
    if isinstance(v, Timestamp):
        return b"\x83" + struct.pack(">q", v)
    if isinstance(v, int):
        if -128 <= v <= 127:
            return b"\x55" + struct.pack(">b", v)
        return b"\x81" + struct.pack(">q", v)
    if isinstance(v, float):
        return b"\x82" + struct.pack(">d", v)
    if isinstance(v, uuid.UUID):
        return b"\x98" + v.bytes
    if isinstance(v, Symbol):
        b = v.encode("ascii")
        return (b"\xa3" + struct.pack(">B", len(b)) if len(b) < 256 else b"\xb3" + struct.pack(">I", len(b))) + b
    if isinstance(v, str):
        b = v.encode("utf-8")
        return (b"\xa1" + struct.pack(">B", len(b)) if len(b) < 256 else b"\xb1" + struct.pack(">I", len(b))) + b
    if isinstance(v, (bytes, bytearray, memoryview)):
        b = bytes(v)
        return (b"\xa0" + struct.pack(">B", len(b)) if len(b) < 256 else b"\xb0" + struct.pack(">I", len(b))) + b
    if isinstance(v, (list, tuple)):
        if not v:
            return b"\x45"
        body = b"".join(encode(x) for x in v)
        return b"\xd0" + struct.pack(">II", len(body) + 4, len(v)) + body
    if isinstance(v, dict):
        body = b"".join(encode(k) + encode(x) for k, x in v.items())
        return b"\xd1" + struct.pack(">II", len(body) + 4, 2 * len(v)) + body
    raise AmqpError(f"cannot encode {type(v).__name__}")


_FIXED = {0x50: (">B", UByte), 0x51: (">b", int), 0x60: (">H", UShort), 0x61: (">h", int), 0x70: (">I", UInt),
          0x71: (">i", int), 0x80: (">Q", ULong), 0x81: (">q", int), 0x72: (">f", float), 0x82: (">d", float),
          0x83: (">q", Timestamp), 0x52: (">B", UInt), 0x53: (">B", ULong), 0x54: (">b", int), 0x55: (">b", int),
          0x56: (">B", bool), 0x73: (">I", int)}


def decode(b: bytes, i: int = 0) -> Tuple[Any, int]:
    c = b[i]
    i += 1
    if c == 0x00:
        d, i = decode(b, i)
        v, i = decode(b, i)
        return Described(d, v), i
    if c == 0x40:
        return None, i
    if c == 0x41:
        return True, i
    if c == 0x42:
        return False, i
    if c == 0x43:
        return UInt(0), i
    if c == 0x44:
        return ULong(0), i
    if c == 0x45:
        return [], i
    if c in _FIXED:
        fmt, cls = _FIXED[c]
        n = struct.calcsize(fmt)
        v = struct.unpack_from(fmt, b, i)[0]
        return (cls(v) if cls is not bool else bool(v)), i + n
    if c == 0x98:
        return uuid.UUID(bytes=bytes(b[i:i + 16])), i + 16
    if c in (0xa0, 0xa1, 0xa3, 0xb0, 0xb1, 0xb3):
        if c & 0x10:
            n = struct.unpack_from(">I", b, i)[0]
            i += 4
        else:
            n = b[i]
            i += 1
        raw = bytes(b[i:i + n])
        i += n
        if c in (0xa0, 0xb0):
            return raw, i
        if c in (0xa3, 0xb3):
            return Symbol(raw.decode("ascii")), i
        return raw.decode("utf-8"), i
    if c in (0xc0, 0xc1, 0xd0, 0xd1):
        if c & 0x10:
            size, count = struct.unpack_from(">II", b, i)
            i += 8
            end = i + size - 4
        else:
            size, count = b[i], b[i + 1]
            i += 2
            end = i + size - 1
        items = []
        for _ in range(count):
            x, i = decode(b, i)
            items.append(x)
        i = end
        if c in (0xc0, 0xd0):
            return items, i
        return {items[k]: items[k + 1] for k in range(0, len(items), 2)}, i
    if c in (0xe0, 0xf0):
        if c == 0xf0:
            size, count = struct.unpack_from(">II", b, i)
            i += 8
            end = i + size - 4
        else:
            size, count = b[i], b[i + 1]
            i += 2
            end = i + size - 1
        ctor = b[i]
        items = []
        for _ in range(count):
            x, j = decode(bytes([ctor]) + bytes(b[i + 1:end]), 0)
            items.append(x)
            i += j - 1
        return items, end
    raise AmqpError(f"unsupported AMQP type code 0x{c:02x}")


# performative / section descriptors
OPEN, BEGIN, ATTACH, FLOW, TRANSFER, DISPOSITION, DETACH, END, CLOSE = (ULong(x) for x in range(0x10, 0x19))
SASL_MECHANISMS, SASL_INIT, SASL_OUTCOME = ULong(0x40), ULong(0x41), ULong(0x44)
SOURCE, TARGET = ULong(0x28), ULong(0x29)
S_HEADER, S_DELIVERY_ANN, S_MESSAGE_ANN, S_PROPERTIES, S_APP_PROPS, S_DATA, S_SEQUENCE, S_VALUE, S_FOOTER = \
    (ULong(x) for x in range(0x70, 0x79))
SELECTOR_FILTER = Symbol("apache.org:selector-filter:string")

PROTO_AMQP = b"AMQP\x00\x01\x00\x00"
PROTO_SASL = b"AMQP\x03\x01\x00\x00"


def frame(performative: Described, channel: int = 0, payload: bytes = b"", ftype: int = 0) -> bytes:
    body = encode(performative) + payload
    return struct.pack(">IBBH", len(body) + 8, 2, ftype, channel) + body


def decode_message(payload: bytes) -> Dict[str, Any]:
    """Bare message sections → {"body": bytes, "annotations": {...}, "properties": {...}, "app": {...}}."""
    out = {"body": b"", "annotations": {}, "properties": None, "app": {}}
    i = 0
    body = []
    while i < len(payload):
        sec, i = decode(payload, i)
        if not isinstance(sec, Described):
            raise AmqpError("malformed message section")
        d = sec.descriptor
        if d == S_MESSAGE_ANN:
            out["annotations"] = dict(sec.value or {})
        elif d == S_APP_PROPS:
            out["app"] = dict(sec.value or {})
        elif d == S_PROPERTIES:
            out["properties"] = sec.value
        elif d == S_DATA:
            body.append(bytes(sec.value))
        elif d == S_VALUE:
            out["value"] = sec.value
            if isinstance(sec.value, (bytes, str)):
                body.append(sec.value if isinstance(sec.value, bytes) else sec.value.encode())
    out["body"] = b"".join(body)
    return out


def encode_message(body: bytes, annotations: Optional[dict] = None, app: Optional[dict] = None) -> bytes:
    out = b""
    if annotations:
        out += encode(Described(S_MESSAGE_ANN, {Symbol(k): v for k, v in annotations.items()}))
    if app:
        out += encode(Described(S_APP_PROPS, dict(app)))
    return out + encode(Described(S_DATA, bytes(body)))


# ---------------------------------------------------------------------------------------------------------------
# connection
# ---------------------------------------------------------------------------------------------------------------

class AmqpConnection:
    """One AMQP connection with one session; links are attached on it by handle."""

    def __init__(self, host: str, port: int = 5671, use_tls: bool = True, username: Optional[str] = None,
                 password: Optional[str] = None, timeout: float = 30.0, max_frame: int = 256 * 1024,
                 container_id: Optional[str] = None):
        raw = socket.create_connection((host, port), timeout=timeout)
        if use_tls:
            raw = ssl.create_default_context().wrap_socket(raw, server_hostname=host)
        self.sock = raw
        self._buf = bytearray()
        self._lock = threading.Lock()
        self.max_frame = max_frame
        self.links: Dict[int, "ReceiverLink"] = {}
        self._next_handle = 0
        self.closed = False
        self._sasl(username, password)
        self.sock.sendall(PROTO_AMQP)
        if self._read_exact(8) != PROTO_AMQP:
            raise AmqpError("server refused the AMQP protocol header")
        self.send(Described(OPEN, [container_id or f"dxa-{uuid.uuid4()}", host, UInt(max_frame), UShort(255)]))
        perf, _ = self.read_frame()
        if perf.descriptor != OPEN:
            raise AmqpError(f"expected open, got {perf!r}")
        self.send(Described(BEGIN, [None, UInt(0), UInt(100000), UInt(100000)]))
        perf, _ = self.read_frame()
        if perf.descriptor != BEGIN:
            raise AmqpError(f"expected begin, got {perf!r}")

    # -- transport
    def _read_exact(self, n: int) -> bytes:
        while len(self._buf) < n:
            chunk = self.sock.recv(1 << 16)
            if not chunk:
                raise AmqpError("connection closed")
            self._buf += chunk
        out = bytes(self._buf[:n])
        del self._buf[:n]
        return out

    def read_frame(self) -> Tuple[Optional[Described], bytes]:
        """→ (performative, trailing payload); heartbeat (empty) frames are skipped."""
        while True:
            size, doff, _ftype, _ch = struct.unpack(">IBBH", self._read_exact(8))
            rest = self._read_exact(size - 8)
            ext = doff * 4 - 8
            body = rest[ext:]
            if not body:
                continue
            perf, i = decode(body, 0)
            return perf, body[i:]

    def send(self, performative: Described, payload: bytes = b"", channel: int = 0, ftype: int = 0):
        with self._lock:
            self.sock.sendall(frame(performative, channel, payload, ftype))

    def _sasl(self, username, password):
        self.sock.sendall(PROTO_SASL)
        if self._read_exact(8) != PROTO_SASL:
            raise AmqpError("server refused the SASL protocol header")
        perf, _ = self.read_frame()
        mechs = perf.value[0] if perf.value else []
        mechs = mechs if isinstance(mechs, list) else [mechs]
        if username is not None and "PLAIN" in mechs:
            init = Described(SASL_INIT, [Symbol("PLAIN"), b"\x00" + username.encode() + b"\x00" +
                                         (password or "").encode()])
        elif "ANONYMOUS" in mechs:
            init = Described(SASL_INIT, [Symbol("ANONYMOUS"), b""])
        else:
            raise AmqpError(f"no usable SASL mechanism in {mechs}")
        self.sock.sendall(frame(init, ftype=1))
        perf, _ = self.read_frame()
        if perf.descriptor != SASL_OUTCOME or perf.value[0] != 0:
            raise AmqpError("SASL authentication failed")

    # -- links
    def attach_receiver(self, address: str, filter_expr: Optional[str] = None, credit: int = 1000
                        ) -> "ReceiverLink":
        handle = self._next_handle
        self._next_handle += 1
        filt = {SELECTOR_FILTER: Described(SELECTOR_FILTER, filter_expr)} if filter_expr else None
        # source: address, durable, expiry-policy, timeout, dynamic, dynamic-node-properties, distribution-mode,
        # filter
        source = Described(SOURCE, [address, UInt(0), Symbol("session-end"), UInt(0), False, None, None, filt])
        name = f"dxa-rx-{uuid.uuid4().hex[:8]}"
        # role receiver (True), snd-settle-mode settled (1), rcv-settle-mode first (0)
        self.send(Described(ATTACH, [name, UInt(handle), True, UByte(1), UByte(0), source,
                                     Described(TARGET, [None])]))
        link = ReceiverLink(self, handle, name, credit)
        self.links[handle] = link
        return link

    def pump(self, timeout: float, enough=None) -> None:
        """Read frames for up to ``timeout`` seconds (or until ``enough()``), routing transfers to their links."""
        deadline = time.monotonic() + timeout
        try:
            while time.monotonic() < deadline and not (enough is not None and enough()):
                self.sock.settimeout(max(0.01, deadline - time.monotonic()))
                perf, payload = self.read_frame()
                d = perf.descriptor
                if d == ATTACH:
                    link = next((l for l in self.links.values() if l.name == perf.value[0]), None)
                    if link is not None:
                        link.remote_attached = True
                        link.flow()
                    continue
                if d == TRANSFER:
                    link = self.links.get(int(perf.value[0]))
                    if link is not None:
                        link.on_transfer(perf, payload)
                    continue
                if d == DETACH:
                    link = self.links.get(int(perf.value[0]))
                    if link is not None:
                        link.detached = perf.value[2] if len(perf.value) > 2 else True
                    continue
                if d in (CLOSE, END):
                    self.closed = True
                    raise AmqpError(f"server closed the connection: {perf.value!r}")
                # flow / disposition: nothing to do for a settled receiver
        except socket.timeout:
            pass

    def close(self):
        try:
            self.send(Described(CLOSE, []))
        except OSError:
            pass
        try:
            self.sock.close()
        except OSError:
            pass
        self.closed = True


class ReceiverLink:
    def __init__(self, conn: AmqpConnection, handle: int, name: str, credit: int):
        self.conn = conn
        self.handle = handle
        self.name = name
        self.credit = credit
        self.delivered = 0
        self.queue: List[Dict[str, Any]] = []
        self._partial = b""
        self.remote_attached = False
        self.detached = None

    def flow(self):
        self.conn.send(Described(FLOW, [UInt(0), UInt(100000), UInt(0), UInt(100000), UInt(self.handle),
                                        UInt(self.delivered), UInt(self.credit)]))

    def on_transfer(self, perf: Described, payload: bytes):
        self._partial += payload
        more = perf.value[5] if len(perf.value) > 5 else False
        if more:
            return
        self.queue.append(decode_message(self._partial))
        self._partial = b""
        self.delivered += 1
        if self.delivered % max(1, self.credit // 2) == 0:
            self.flow()                                       # replenish credit (ProcessRef: link credit)

    def drain(self, max_n: Optional[int] = None) -> List[Dict[str, Any]]:
        n = len(self.queue) if max_n is None else min(max_n, len(self.queue))
        out, self.queue = self.queue[:n], self.queue[n:]
        return out


def management_partitions(conn: AmqpConnection, hub: str, key_name: Optional[str] = None,
                          timeout: float = 10.0) -> List[str]:
    """Partition ids of ``hub`` from the ``$management`` node (request/response over a sender + receiver link)."""
    reply_to = f"dxa-mgmt-{uuid.uuid4().hex[:8]}"
    rx = conn.attach_receiver("$management", credit=10)
    # sender link (role False) to $management
    handle = conn._next_handle
    conn._next_handle += 1
    conn.send(Described(ATTACH, [f"{reply_to}-tx", UInt(handle), False, UByte(1), UByte(0),
                                 Described(SOURCE, [reply_to]), Described(TARGET, ["$management"]), None, False,
                                 UInt(0)]))
    app = {"operation": "READ", "name": hub, "type": "com.microsoft:eventhub"}
    props = Described(S_PROPERTIES, [str(uuid.uuid4()), None, None, None, reply_to])
    msg = encode(props) + encode(Described(S_APP_PROPS, app)) + encode(Described(S_VALUE, None))
    conn.send(Described(TRANSFER, [UInt(handle), UInt(0), b"\x00", UInt(0), True, False]), msg)
    conn.pump(timeout, enough=lambda: bool(rx.queue))
    if not rx.queue:
        raise AmqpError("no reply from $management")
    reply = rx.drain(1)[0]
    raw = reply.get("value")
    if not isinstance(raw, dict) or "partition_ids" not in raw:
        raise AmqpError(f"unexpected $management reply {raw!r}")
    return [str(p) for p in raw["partition_ids"]]


def parse_eventhub_connection(conn: str) -> Dict[str, str]:
    parts = {}
    for p in conn.split(";"):
        if "=" in p:
            k, v = p.split("=", 1)
            parts[k.strip().lower()] = v.strip()
    ep = parts.get("endpoint", "")
    if not ep.lower().startswith(("sb://", "amqps://", "amqp://")):
        raise AmqpError("Event Hubs connection string has no sb:// endpoint")
    scheme, rest = ep.split("://", 1)
    hostport = rest.strip("/").split("/")[0]
    host, _, port = hostport.partition(":")
    tls = scheme.lower() != "amqp"
    return {"host": host, "port": port or ("5671" if tls else "5672"), "tls": "1" if tls else "0",
            "keyname": parts.get("sharedaccesskeyname", ""), "key": parts.get("sharedaccesskey", ""),
            "entity": parts.get("entitypath", "")}
