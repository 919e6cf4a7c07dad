"""In-process fake SQL Server speaking enough TDS 7.4 for the SQL sink tests: PRELOGIN (encryption off / login-only
TLS / full TLS), LOGIN7 (SQL auth, checked), SQL batches (CREATE TABLE / TRUNCATE guarded by OBJECT_ID, multi-row
INSERT … VALUES) and bulk load (INSERT BULK + COLMETADATA/ROW tokens).  Tables live in ``self.tables``."""
import re
import socket
import ssl
import struct
import threading

from dxa.io import tds as T


def _done(count=None, status_more=False):
    status = (0x10 if count is not None else 0) | (0x01 if status_more else 0)
    return b"\xfd" + struct.pack("<HHQ", status, 0xC1, count or 0)


def _error(number, msg):
    body = struct.pack("<iBB", number, 1, 16) + struct.pack("<H", len(msg)) + msg.encode("utf-16-le")
    body += b"\x00" + b"\x00" + struct.pack("<i", 1)
    return b"\xaa" + struct.pack("<H", len(body)) + body


def _loginack():
    prog = "FakeSQL"
    body = bytes([1]) + struct.pack(">I", T.TDS74) + bytes([len(prog)]) + prog.encode("utf-16-le") + bytes([15, 0, 0, 0])
    return b"\xad" + struct.pack("<H", len(body)) + body


def _parse_values(text):
    """``(1, N'a''b', NULL, 2.5), (…)`` → list of tuples."""
    rows, row, i = [], None, 0
    while i < len(text):
        ch = text[i]
        if ch == "(":
            row = []
            i += 1
        elif ch == ")":
            rows.append(tuple(row))
            i += 1
        elif ch in " ,\n\t":
            i += 1
        elif text.startswith("N'", i) or ch == "'":
            j = i + (2 if ch == "N" else 1)
            buf = []
            while True:
                if text[j] == "'" and text[j + 1:j + 2] == "'":
                    buf.append("'")
                    j += 2
                elif text[j] == "'":
                    break
                else:
                    buf.append(text[j])
                    j += 1
            row.append("".join(buf))
            i = j + 1
        elif text.startswith("NULL", i):
            row.append(None)
            i += 4
        else:
            m = re.match(r"-?[0-9.eE+\-]+", text[i:])
            tok = m.group(0)
            row.append(float(tok) if any(c in tok for c in ".eE") else int(tok))
            i += len(tok)
    return rows


class FakeSqlServer:
    def __init__(self, user="sa", password="p@ss", encryption="none", certfile=None, keyfile=None):
        self.user, self.password = user, password
        self.encryption = encryption          # none | login | full
        self.certfile, self.keyfile = certfile, keyfile
        self.tables = {}
        self.statements = []
        self.logins = []
        self.protocol_errors = []
        self.sock = socket.create_server(("127.0.0.1", 0))
        self.port = self.sock.getsockname()[1]
        self._stop = False
        threading.Thread(target=self._accept, daemon=True).start()

    def close(self):
        self._stop = True
        self.sock.close()

    def _accept(self):
        while not self._stop:
            try:
                c, _ = self.sock.accept()
            except OSError:
                return
            threading.Thread(target=self._serve, args=(c,), daemon=True).start()

    # ---- transport on the server side
    def _serve(self, c):
        ch = T._Channel(c)
        try:
            t, payload = ch.read_message()
            assert t == T.PT_PRELOGIN
            client_enc = T.parse_prelogin(payload)[0x01][0]
            enc = {"none": T.ENCRYPT_NOT_SUP, "login": T.ENCRYPT_OFF, "full": T.ENCRYPT_ON}[self.encryption]
            if enc == T.ENCRYPT_OFF and client_enc == T.ENCRYPT_ON:
                enc = T.ENCRYPT_ON
            c.sendall(T._packet(T.PT_REPLY, T._prelogin_payload(enc), 4096))
            if enc != T.ENCRYPT_NOT_SUP:
                self._tls_accept(ch)
            t, login = ch.read_message()
            assert t == T.PT_LOGIN7
            if enc == T.ENCRYPT_OFF:
                ch.stop_tls()
            user, pw, db = self._login_fields(login)
            self.logins.append((user, db, enc))
            if (user, pw) != (self.user, self.password):
                ch.send(T._packet(T.PT_REPLY, _error(18456, f"Login failed for user '{user}'.") + _done(), 4096))
                return
            ch.send(T._packet(T.PT_REPLY, _loginack() + _done(), 4096))
            bulk_target = None
            while True:
                t, msg = ch.read_message()
                if t != T.PT_BULK and bulk_target is not None:
                    # after INSERT BULK the server expects the BulkLoadBCP message and nothing else: a real SQL
                    # Server fails the request and drops the connection
                    self.protocol_errors.append(f"packet type {t} after INSERT BULK")
                    return
                if t == T.PT_SQLBATCH:
                    hdr = struct.unpack("<I", msg[:4])[0]
                    sql = msg[hdr:].decode("utf-16-le")
                    self.statements.append(sql)
                    reply, bulk_target = self._exec(sql, bulk_target)
                elif t == T.PT_BULK:
                    n = self._bulk(bulk_target, msg)
                    bulk_target = None
                    reply = _done(n)
                else:
                    reply = _error(50000, f"unexpected packet type {t}") + _done()
                ch.send(T._packet(T.PT_REPLY, reply, 4096))
        except (T.TdsError, OSError, AssertionError):
            pass
        finally:
            c.close()

    def _tls_accept(self, ch):
        ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
        ctx.load_cert_chain(self.certfile, self.keyfile)
        ctx.maximum_version = ssl.TLSVersion.TLSv1_2
        ch.inc, ch.out = ssl.MemoryBIO(), ssl.MemoryBIO()
        obj = ctx.wrap_bio(ch.inc, ch.out, server_side=True)
        while True:
            try:
                obj.do_handshake()
                break
            except ssl.SSLWantReadError:
                out = ch.out.read()
                if out:
                    ch.sock.sendall(T._packet(T.PT_PRELOGIN, out, 4096))
                _t, payload = ch.read_message()
                ch.inc.write(payload)
        out = ch.out.read()
        if out:
            ch.sock.sendall(T._packet(T.PT_PRELOGIN, out, 4096))
        ch.tls = obj

    @staticmethod
    def _login_fields(b):
        def field(k):
            off, ln = struct.unpack("<HH", b[36 + 4 * k:40 + 4 * k])
            return b[off:off + 2 * ln]
        return (field(1).decode("utf-16-le"), T.decode_password(field(2)), field(8).decode("utf-16-le"))

    # ---- a tiny SQL engine
    def _exec(self, sql, bulk_target):
        def nm(x):
            return x.replace("].[", ".").strip("[]")
        m = re.match(r"IF OBJECT_ID\(N'(.+?)', N'U'\) IS NULL CREATE TABLE (\S+) \((.*)\)$", sql, re.S)
        if m:
            self.tables.setdefault(nm(m.group(2)), {"cols": re.findall(r"\[([^\]]+)\] ([a-z0-9()]+)", m.group(3)),
                                                    "rows": []})
            return _done(), bulk_target
        m = re.match(r"IF OBJECT_ID\(N'(.+?)', N'U'\) IS NOT NULL TRUNCATE TABLE (\S+)$", sql)
        if m:
            if nm(m.group(2)) in self.tables:
                self.tables[nm(m.group(2))]["rows"].clear()
            return _done(), bulk_target
        m = re.match(r"INSERT INTO (\S+) \((.*?)\) VALUES (.*)$", sql, re.S)
        if m:
            name = nm(m.group(1))
            if name not in self.tables:
                return _error(208, f"Invalid object name '{name}'.") + _done(), bulk_target
            rows = _parse_values(m.group(3))
            self.tables[name]["rows"].extend(rows)
            return _done(len(rows)), bulk_target
        m = re.match(r"INSERT BULK (\S+) \((.*)\)", sql, re.S)
        if m:
            return _done(), nm(m.group(1))
        return _error(102, f"Incorrect syntax near '{sql[:20]}'.") + _done(), bulk_target

    def _bulk(self, table, b):
        assert b[0] == 0x81
        n = struct.unpack("<H", b[1:3])[0]
        i = 3
        types = []
        for _ in range(n):
            i += 6
            t = b[i]
            i += 1
            if t in (0x26, 0x6D, 0x68, 0x2A):
                i += 1
            elif t == 0xE7:
                i += 2 + 5
            nl = b[i]
            i += 1 + 2 * nl
            types.append(t)
        rows = []
        while b[i] == 0xD1:
            i += 1
            row = []
            for t in types:
                if t == 0xE7:
                    ln = struct.unpack("<H", b[i:i + 2])[0]
                    i += 2
                    if ln == 0xFFFF:
                        row.append(None)
                    else:
                        row.append(b[i:i + ln].decode("utf-16-le"))
                        i += ln
                else:
                    ln = b[i]
                    i += 1
                    raw = b[i:i + ln]
                    i += ln
                    if ln == 0:
                        row.append(None)
                    elif t == 0x26:
                        row.append(struct.unpack("<q", raw)[0])
                    elif t == 0x6D:
                        row.append(struct.unpack("<d", raw)[0])
                    elif t == 0x68:
                        row.append(bool(raw[0]))
                    else:                                   # datetime2(7): (ticks, days)
                        row.append((int.from_bytes(raw[:5], "little"), int.from_bytes(raw[5:8], "little")))
            rows.append(tuple(row))
        assert b[i] == 0xFD
        self.tables[table]["rows"].extend(rows)
        return len(rows)
