"""A tiny in-process Kafka broker for tests: Metadata v1, ListOffsets v1, Fetch v4, Produce v3, SaslHandshake v1 and
SaslAuthenticate v0 (PLAIN).  Record batches are stored verbatim with the broker-assigned base offset patched in —
what a real broker does for magic-2 batches."""
import socket
import struct
import threading


class FakeBroker:
    def __init__(self, topics, partitions=2, sasl_password=None):
        self.sock = socket.create_server(("127.0.0.1", 0))
        self.port = self.sock.getsockname()[1]
        self.logs = {(t, p): [] for t in topics for p in range(partitions)}   # [(base, last, bytes)]
        self.next = {k: 0 for k in self.logs}
        self.sasl_password = sasl_password
        self.lock = threading.Lock()
        self.stopped = False
        threading.Thread(target=self._accept, daemon=True).start()

    def close(self):
        self.stopped = True
        self.sock.close()

    # -- plumbing -----------------------------------------------------------------------------------------------
    def _accept(self):
        while not self.stopped:
            try:
                c, _ = self.sock.accept()
            except OSError:
                return
            threading.Thread(target=self._serve, args=(c,), daemon=True).start()

    def _serve(self, c):
        authed = self.sasl_password is None
        with c:
            while True:
                h = self._read(c, 4)
                if h is None:
                    return
                msg = self._read(c, struct.unpack(">i", h)[0])
                api, ver, corr = struct.unpack_from(">hhi", msg, 0)
                clen = struct.unpack_from(">h", msg, 8)[0]
                body = memoryview(msg)[10 + max(0, clen):]
                if not authed and api not in (17, 36):
                    return
                out, authed = self._handle(api, ver, body, authed)
                resp = struct.pack(">i", corr) + out
                c.sendall(struct.pack(">i", len(resp)) + resp)

    @staticmethod
    def _read(c, n):
        b = bytearray()
        while len(b) < n:
            x = c.recv(n - len(b))
            if not x:
                return None
            b += x
        return bytes(b)

    # -- handlers -----------------------------------------------------------------------------------------------
    def _handle(self, api, ver, b, authed):
        r = _R(b)
        if api == 17:
            r.str()
            return struct.pack(">h", 0) + struct.pack(">i", 1) + _s("PLAIN"), authed
        if api == 36:
            tok = r.bytes()
            _, user, pw = tok.split(b"\0")
            ok = pw.decode() == self.sasl_password
            return struct.pack(">h", 0 if ok else 58) + _s(None if ok else "bad credentials") + _b(b""), ok
        if api == 3:
            topics = sorted({t for t, _ in self.logs})
            out = struct.pack(">i", 1) + struct.pack(">i", 0) + _s("127.0.0.1") + struct.pack(">i", self.port) + \
                _s(None) + struct.pack(">i", 0) + struct.pack(">i", len(topics))
            for t in topics:
                parts = sorted(p for tt, p in self.logs if tt == t)
                out += struct.pack(">h", 0) + _s(t) + struct.pack(">b", 0) + struct.pack(">i", len(parts))
                for p in parts:
                    out += struct.pack(">hii", 0, p, 0) + struct.pack(">ii", 1, 0) + struct.pack(">ii", 1, 0)
            return out, authed
        if api == 2:
            r.i32()
            out = bytearray(struct.pack(">i", r.i32()))
            t = r.str()
            out += _s(t)
            n = r.i32()
            out += struct.pack(">i", n)
            for _ in range(n):
                p, ts = r.i32(), r.i64()
                if ts >= 0:                                   # by timestamp: first batch whose max timestamp >= ts
                    off = next((base for base, _last, raw in self.logs[(t, p)]
                                if struct.unpack_from(">q", raw, 35)[0] >= ts), -1)
                else:
                    off = 0 if ts == -2 else self.next[(t, p)]
                out += struct.pack(">ihqq", p, 0, -1, off)
            return bytes(out), authed
        if api == 1:
            r.i32(), r.i32(), r.i32(), r.i32(), r.i8()
            out = bytearray(struct.pack(">i", 0))
            nt = r.i32()
            out += struct.pack(">i", nt)
            for _ in range(nt):
                t = r.str()
                out += _s(t)
                np_ = r.i32()
                out += struct.pack(">i", np_)
                for _ in range(np_):
                    p, off, maxb = r.i32(), r.i64(), r.i32()
                    with self.lock:
                        data = bytearray()
                        for base, last, raw in self.logs[(t, p)]:
                            if last >= off and (not data or len(data) + len(raw) <= maxb):
                                data += raw
                        hw = self.next[(t, p)]
                    out += struct.pack(">ihqq", p, 0, hw, hw) + struct.pack(">i", 0) + _b(bytes(data))
            return bytes(out), authed
        if api == 0:
            r.str(), r.i16(), r.i32()
            out = bytearray()
            nt = r.i32()
            out += struct.pack(">i", nt)
            for _ in range(nt):
                t = r.str()
                out += _s(t)
                np_ = r.i32()
                out += struct.pack(">i", np_)
                for _ in range(np_):
                    p = r.i32()
                    batch = bytearray(r.bytes())
                    with self.lock:
                        base = self.next[(t, p)]
                        last_delta = struct.unpack_from(">i", batch, 23)[0]
                        batch[0:8] = struct.pack(">q", base)
                        self.logs[(t, p)].append((base, base + last_delta, bytes(batch)))
                        self.next[(t, p)] = base + last_delta + 1
                    out += struct.pack(">ihqq", p, 0, base, -1)
            out += struct.pack(">i", 0)
            return bytes(out), authed
        raise ValueError(f"unsupported api {api}")


def _s(v):
    if v is None:
        return struct.pack(">h", -1)
    e = v.encode()
    return struct.pack(">h", len(e)) + e


def _b(v):
    return struct.pack(">i", len(v)) + v


class _R:
    def __init__(self, b):
        self.b, self.p = b, 0

    def _t(self, f, n):
        v = struct.unpack_from(f, self.b, self.p)[0]
        self.p += n
        return v

    def i8(self):
        return self._t(">b", 1)

    def i16(self):
        return self._t(">h", 2)

    def i32(self):
        return self._t(">i", 4)

    def i64(self):
        return self._t(">q", 8)

    def str(self):
        n = self.i16()
        if n < 0:
            return None
        v = bytes(self.b[self.p:self.p + n]).decode()
        self.p += n
        return v

    def bytes(self):
        n = self.i32()
        v = bytes(self.b[self.p:self.p + n])
        self.p += n
        return v
