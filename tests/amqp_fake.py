"""In-process fake Event Hubs endpoint speaking enough AMQP 1.0 for the EventHub source tests: SASL PLAIN /
ANONYMOUS, open / begin, receiver links on ``<hub>/ConsumerGroups/<g>/Partitions/<p>`` honouring the selector
filter (sequence number >=, offset > -1 / @latest, enqueued time >) and link credit, and the ``$management`` READ of
``com.microsoft:eventhub`` (partition ids).  Events are appended with ``send(partition, body, props)``."""
import re
import socket
import struct
import threading
import time

from dxa.io import amqp as A


class FakeEventHub:
    def __init__(self, hub="iot", partitions=2, key_name="RootManageSharedAccessKey", key="secret"):
        self.hub, self.key_name, self.key = hub, key_name, key
        self.parts = {str(p): [] for p in range(partitions)}      # [(seq, enqueued_ms, body, props)]
        self.lock = threading.Lock()
        self.sock = socket.create_server(("127.0.0.1", 0))
        self.port = self.sock.getsockname()[1]
        self.stopped = False
        self.links = []                                           # live receiver links for push
        threading.Thread(target=self._accept, daemon=True).start()

    @property
    def connection_string(self):
        return (f"Endpoint=amqp://127.0.0.1:{self.port}/;SharedAccessKeyName={self.key_name};"
                f"SharedAccessKey={self.key};EntityPath={self.hub}")

    def send(self, partition, body: bytes, props=None, enqueued_ms=None):
        with self.lock:
            log = self.parts[str(partition)]
            log.append((len(log), enqueued_ms or int(time.time() * 1000), body, props or {}))

    def close(self):
        self.stopped = True
        self.sock.close()

    def _accept(self):
        while not self.stopped:
            try:
                c, _ = self.sock.accept()
            except OSError:
                return
            threading.Thread(target=self._serve, args=(c,), daemon=True).start()

    # -- protocol
    def _serve(self, c):
        conn = _Conn(c)
        try:
            assert conn.read_exact(8) == A.PROTO_SASL
            c.sendall(A.PROTO_SASL)
            c.sendall(A.frame(A.Described(A.SASL_MECHANISMS, [[A.Symbol("PLAIN"), A.Symbol("ANONYMOUS")]]), ftype=1))
            perf, _ = conn.read_frame()
            mech, resp = perf.value[0], perf.value[1]
            ok = mech == "ANONYMOUS" or resp == b"\x00" + self.key_name.encode() + b"\x00" + self.key.encode()
            c.sendall(A.frame(A.Described(A.SASL_OUTCOME, [A.UByte(0 if ok else 1)]), ftype=1))
            if not ok:
                return
            assert conn.read_exact(8) == A.PROTO_AMQP
            c.sendall(A.PROTO_AMQP)
            links = {}            # handle → state
            mgmt_reply_to = {}
            while not self.stopped:
                perf, payload = conn.read_frame(timeout=0.05)
                if perf is not None:
                    d = perf.descriptor
                    if d == A.OPEN:
                        c.sendall(A.frame(A.Described(A.OPEN, ["fake-eh", None, A.UInt(256 * 1024)])))
                    elif d == A.BEGIN:
                        c.sendall(A.frame(A.Described(A.BEGIN, [A.UShort(0), A.UInt(0), A.UInt(100000),
                                                                 A.UInt(100000)])))
                    elif d == A.ATTACH:
                        name, handle, role = perf.value[0], int(perf.value[1]), perf.value[2]
                        src = perf.value[5].value if perf.value[5] is not None else []
                        tgt = perf.value[6].value if len(perf.value) > 6 and perf.value[6] is not None else []
                        addr = src[0] if src else None
                        st = {"name": name, "role": role, "addr": addr, "credit": 0, "next": 0, "sent": 0}
                        if role:            # client receives from us
                            if addr == "$management":
                                st["mgmt"] = True
                            else:
                                m = re.match(r"(.+)/ConsumerGroups/(.+)/Partitions/(.+)", addr)
                                st["part"] = m.group(3)
                                filt = src[7] if len(src) > 7 and src[7] else {}
                                expr = next(iter(filt.values())).value if filt else None
                                st["next"] = self._start(st["part"], expr)
                        else:
                            st["target"] = tgt[0] if tgt else None
                            mgmt_reply_to[handle] = src[0] if src else None
                        links[handle] = st
                        c.sendall(A.frame(A.Described(A.ATTACH, [name, A.UInt(handle), not role, A.UByte(1),
                                                                  A.UByte(0), perf.value[5], perf.value[6]])))
                    elif d == A.FLOW:
                        h = perf.value[4]
                        if h is not None and int(h) in links:
                            st = links[int(h)]
                            st["credit"] = int(perf.value[6]) - (st["sent"] - int(perf.value[5] or 0))
                    elif d == A.TRANSFER:
                        h = int(perf.value[0])
                        st = links.get(h)
                        msg = A.decode_message(payload)
                        if st is not None and st.get("target") == "$management":
                            reply = (A.encode(A.Described(A.S_APP_PROPS, {"status-code": 200})) +
                                     A.encode(A.Described(A.S_VALUE, {"name": self.hub,
                                                                      "partition_ids": sorted(self.parts)})))
                            for rh, rst in links.items():
                                if rst.get("mgmt"):
                                    c.sendall(_transfer(rh, rst["sent"], reply))
                                    rst["sent"] += 1
                    elif d == A.CLOSE:
                        c.sendall(A.frame(A.Described(A.CLOSE, [])))
                        return
                # push events to receivers with credit
                for h, st in links.items():
                    if not st["role"] or st.get("mgmt") or "part" not in st:
                        continue
                    with self.lock:
                        log = self.parts[st["part"]]
                        ready = log[st["next"]:st["next"] + max(0, st["credit"])]
                    for seq, enq, body, props in ready:
                        ann = {"x-opt-sequence-number": seq, "x-opt-offset": str(seq * 100),
                               "x-opt-enqueued-time": A.Timestamp(enq)}
                        c.sendall(_transfer(h, st["sent"], A.encode_message(body, ann, props)))
                        st["sent"] += 1
                        st["credit"] -= 1
                        st["next"] = seq + 1
        except (OSError, AssertionError, A.AmqpError):
            pass
        finally:
            c.close()

    def _start(self, part, expr):
        log = self.parts[part]
        if not expr:
            return len(log)
        m = re.match(r"amqp\.annotation\.(x-opt-[a-z-]+) (>=|>) '(.+)'", expr)
        field, op, val = m.groups()
        if field == "x-opt-offset":
            return 0 if val == "-1" else len(log)
        if field == "x-opt-sequence-number":
            return int(val) + (1 if op == ">" else 0)
        if field == "x-opt-enqueued-time":
            return next((s for s, enq, _b, _p in log if enq > int(val)), len(log))
        return len(log)


def _transfer(handle, delivery_id, payload):
    return A.frame(A.Described(A.TRANSFER, [A.UInt(handle), A.UInt(delivery_id), struct.pack(">I", delivery_id),
                                            A.UInt(0), True, False]), payload=payload)


class _Conn:
    def __init__(self, s):
        self.s = s
        self.buf = bytearray()

    def read_exact(self, n, timeout=None):
        self.s.settimeout(timeout)
        while len(self.buf) < n:
            try:
                chunk = self.s.recv(1 << 16)
            except socket.timeout:
                return None
            if not chunk:
                raise OSError("closed")
            self.buf += chunk
        out = bytes(self.buf[:n])
        del self.buf[:n]
        return out

    def read_frame(self, timeout=None):
        if len(self.buf) < 8:
            hdr = self.read_exact(8, timeout)
            if hdr is None:
                return None, b""
        else:
            hdr = self.read_exact(8)
        size, doff, _t, _ch = struct.unpack(">IBBH", hdr)
        rest = self.read_exact(size - 8, None)
        body = rest[doff * 4 - 8:]
        if not body:
            return None, b""
        perf, i = A.decode(body, 0)
        return perf, body[i:]
