"""SQL Server / Azure SQL client over TDS 7.4 (the wire protocol behind the reference's JDBC / bulk-copy SQL sink,
DataProcessing/datax-host/src/main/scala/datax/sink/SqlSinker.scala:19-107, settings SqlOutputSetting.scala:12-61).

No driver package is available here, so this speaks the protocol directly with the standard library:

* PRELOGIN with encryption negotiation; TLS (``ssl.MemoryBIO``) runs inside PRELOGIN packets during the handshake,
  then either wraps the whole connection (``encrypt=true`` / server requires it) or only the LOGIN7 packet
  (login-only encryption, the TDS default when both sides say ENCRYPT_OFF);
* LOGIN7 with SQL authentication (password obfuscated per MS-TDS 2.2.6.4) and the initial database;
* SQL batches (ALL_HEADERS + UCS-2 text); the token stream is parsed for LOGINACK / ENVCHANGE (packet size) /
  INFO / ERROR / DONE* — an ERROR token raises ``TdsError`` with the server's message;
* bulk load (``INSERT BULK`` + a BulkLoadBCP message of COLMETADATA + ROW tokens) for ``usebulkinsert=true``
  (SqlSinker.writeUsingSqlBulkCopy), multi-row ``INSERT … VALUES`` statements (≤1000 rows each) otherwise.

Connection strings: JDBC (``jdbc:sqlserver://host:port;database=…;user=…;password=…;encrypt=true;…``) and ADO.NET
(``Server=tcp:host,1433;Initial Catalog=…;User ID=…;Password=…;Encrypt=True;…``).
"""
from __future__ import annotations

import datetime as _dt
import math
import os
import socket
import ssl
import struct
from typing import Any, Dict, List, Optional, Sequence, Tuple

PT_SQLBATCH, PT_LOGIN7, PT_BULK, PT_PRELOGIN, PT_REPLY = 0x01, 0x10, 0x07, 0x12, 0x04
ENCRYPT_OFF, ENCRYPT_ON, ENCRYPT_NOT_SUP, ENCRYPT_REQ = 0, 1, 2, 3
TDS74 = 0x74000004


class TdsError(Exception):
    def __init__(self, msg: str, number: int = 0):
        super().__init__(msg)
        self.number = number


# ---------------------------------------------------------------------------------------------------------------
# connection strings
# ---------------------------------------------------------------------------------------------------------------

def _truthy(v, default=False) -> bool:
    if v is None:
        return default
    return str(v).strip().lower() in ("true", "yes", "1", "on", "mandatory", "strict")


def parse_connection_string(conn: str) -> Dict[str, Any]:
    """JDBC or ADO.NET SQL Server connection string → {host, port, database, user, password, encrypt,
    trust_server_certificate, host_name_in_certificate, timeout}."""
    conn = conn.strip()
    out: Dict[str, Any] = {"port": 1433}
    if conn.lower().startswith("jdbc:sqlserver://"):
        rest = conn[len("jdbc:sqlserver://"):]
        server, _, props = rest.partition(";")
        hostport, _, _inst = server.partition("\\")
        host, _, port = hostport.partition(":")
        out["host"] = host
        if port:
            out["port"] = int(port)
        kv = {}
        for part in props.split(";"):
            if "=" in part:
                k, v = part.split("=", 1)
                kv[k.strip().lower()] = v.strip()
        out["database"] = kv.get("database") or kv.get("databasename")
        out["user"] = kv.get("user") or kv.get("username")
        out["password"] = kv.get("password")
        out["encrypt"] = kv.get("encrypt")
        out["trust_server_certificate"] = kv.get("trustservercertificate")
        out["host_name_in_certificate"] = kv.get("hostnameincertificate")
        out["timeout"] = kv.get("logintimeout")
        return out
    kv = {}
    for part in conn.split(";"):
        if "=" in part:
            k, v = part.split("=", 1)
            kv[k.strip().lower()] = v.strip()
    server = kv.get("server") or kv.get("data source") or kv.get("address") or kv.get("addr")
    if not server:
        raise ValueError("SQL Server connection string names no server")
    if server.lower().startswith("tcp:"):
        server = server[4:]
    host, _, port = server.partition(",")
    out["host"] = host.split("\\")[0]
    if port:
        out["port"] = int(port)
    out["database"] = kv.get("initial catalog") or kv.get("database")
    out["user"] = kv.get("user id") or kv.get("uid") or kv.get("user")
    out["password"] = kv.get("password") or kv.get("pwd")
    out["encrypt"] = kv.get("encrypt")
    out["trust_server_certificate"] = kv.get("trustservercertificate")
    out["host_name_in_certificate"] = kv.get("hostnameincertificate")
    out["timeout"] = kv.get("connection timeout") or kv.get("connect timeout")
    return out


def is_sqlserver_connection(conn: str) -> bool:
    c = conn.strip().lower()
    if c.startswith("jdbc:sqlserver://"):
        return True
    return any(c.startswith(p) or f";{p}" in c for p in ("server=", "data source="))


# ---------------------------------------------------------------------------------------------------------------
# transport
# ---------------------------------------------------------------------------------------------------------------

def _packet(ptype: int, payload: bytes, packet_size: int, pid_start: int = 1) -> bytes:
    out = bytearray()
    body = packet_size - 8
    chunks = [payload[i:i + body] for i in range(0, len(payload), body)] or [b""]
    for k, c in enumerate(chunks):
        status = 0x01 if k == len(chunks) - 1 else 0x00
        out += struct.pack(">BBHHBB", ptype, status, len(c) + 8, 0, (pid_start + k) & 0xFF, 0) + c
    return bytes(out)


class _Channel:
    """Raw socket, optionally with a TLS session layered on top through memory BIOs."""

    def __init__(self, sock: socket.socket):
        self.sock = sock
        self.tls: Optional[ssl.SSLObject] = None
        self.inc = self.out = None
        self._plain = bytearray()

    def _recv_raw(self, n: int) -> bytes:
        b = self.sock.recv(n)
        if not b:
            raise TdsError("connection closed by the server")
        return b

    # plain bytes, TLS-decrypted when a session is active
    def recv_exact(self, n: int) -> bytes:
        while len(self._plain) < n:
            if self.tls is None:
                self._plain += self._recv_raw(65536)
            else:
                try:
                    self._plain += self.tls.read(65536)
                except ssl.SSLWantReadError:
                    self.inc.write(self._recv_raw(65536))
        out = bytes(self._plain[:n])
        del self._plain[:n]
        return out

    def send(self, data: bytes):
        if self.tls is None:
            self.sock.sendall(data)
        else:
            self.tls.write(data)
            self.sock.sendall(self.out.read())

    def read_message(self) -> Tuple[int, bytes]:
        """One TDS message (packets up to EOM) → (type, payload)."""
        payload = bytearray()
        ptype = None
        while True:
            hdr = self.recv_exact(8)
            t, status, length = hdr[0], hdr[1], struct.unpack(">H", hdr[2:4])[0]
            ptype = t if ptype is None else ptype
            payload += self.recv_exact(length - 8)
            if status & 0x01:
                return ptype, bytes(payload)

    def start_tls(self, ctx: ssl.SSLContext, server_hostname: Optional[str], packet_size: int):
        """TLS handshake with the records carried in PRELOGIN packets (MS-TDS 2.2.6.5)."""
        self.inc, self.out = ssl.MemoryBIO(), ssl.MemoryBIO()
        obj = ctx.wrap_bio(self.inc, self.out, server_side=False, server_hostname=server_hostname)
        while True:
            try:
                obj.do_handshake()
                break
            except ssl.SSLWantReadError:
                pending = self.out.read()
                if pending:
                    self.sock.sendall(_packet(PT_PRELOGIN, pending, packet_size))
                _t, payload = self.read_message()
                self.inc.write(payload)
        pending = self.out.read()
        if pending:
            self.sock.sendall(_packet(PT_PRELOGIN, pending, packet_size))
        self.tls = obj

    def stop_tls(self):
        self.tls = None


# ---------------------------------------------------------------------------------------------------------------
# messages
# ---------------------------------------------------------------------------------------------------------------

def _prelogin_payload(encrypt: int) -> bytes:
    opts = [(0x00, struct.pack(">IH", 0x0F000000, 0)),      # VERSION
            (0x01, bytes([encrypt])),                       # ENCRYPTION
            (0x02, b"\x00"),                                # INSTOPT
            (0x03, struct.pack(">I", os.getpid() & 0xFFFFFFFF)),
            (0x04, b"\x00")]                                # MARS off
    head = len(opts) * 5 + 1
    out, data = bytearray(), bytearray()
    for tok, val in opts:
        out += struct.pack(">BHH", tok, head + len(data), len(val))
        data += val
    return bytes(out + b"\xff" + data)


def parse_prelogin(payload: bytes) -> Dict[int, bytes]:
    out, i = {}, 0
    while payload[i] != 0xFF:
        tok, off, ln = struct.unpack(">BHH", payload[i:i + 5])
        out[tok] = payload[off:off + ln]
        i += 5
    return out


def encode_password(pw: str) -> bytes:
    return bytes((((b << 4) & 0xF0) | (b >> 4)) ^ 0xA5 for b in pw.encode("utf-16-le"))


def decode_password(b: bytes) -> str:
    return bytes(((((x ^ 0xA5) << 4) & 0xF0) | ((x ^ 0xA5) >> 4)) for x in b).decode("utf-16-le")


def login7_payload(host: str, user: str, password: str, database: str, app: str = "dxa",
                   server: str = "", packet_size: int = 4096) -> bytes:
    fields = [("hostname", host), ("username", user), ("password", None), ("appname", app),
              ("servername", server), ("unused", ""), ("cltintname", "dxa-tds"), ("language", ""),
              ("database", database or "")]
    fixed = 94
    data = bytearray()
    offs = bytearray()
    for name, val in fields:
        if name == "password":
            enc = encode_password(password or "")
            offs += struct.pack("<HH", fixed + len(data), len(password or ""))
            data += enc
        else:
            enc = (val or "").encode("utf-16-le")
            offs += struct.pack("<HH", fixed + len(data), len(val or ""))
            data += enc
    head = struct.pack("<IIIIII", 0, TDS74, packet_size, 7, os.getpid() & 0xFFFFFFFF, 0)
    head += bytes([0xE0, 0x03, 0x00, 0x00]) + struct.pack("<iI", 0, 0x0409)
    tail = b"\x00" * 6 + struct.pack("<HH", fixed + len(data), 0) * 3 + struct.pack("<I", 0)
    body = head + offs + tail
    assert len(body) == fixed, len(body)
    total = body + bytes(data)
    return struct.pack("<I", len(total)) + total[4:]


def _all_headers() -> bytes:
    return struct.pack("<IIHQI", 22, 18, 2, 0, 1)


class Reply:
    def __init__(self):
        self.row_counts: List[int] = []
        self.infos: List[str] = []
        self.packet_size: Optional[int] = None
        self.logged_in = False
        self.rows: List[list] = []


def _us_varchar(b: bytes, i: int) -> Tuple[str, int]:
    n = struct.unpack("<H", b[i:i + 2])[0]
    return b[i + 2:i + 2 + 2 * n].decode("utf-16-le"), i + 2 + 2 * n


def _b_varchar(b: bytes, i: int) -> Tuple[str, int]:
    n = b[i]
    return b[i + 1:i + 1 + 2 * n].decode("utf-16-le"), i + 1 + 2 * n


def parse_reply(b: bytes) -> Reply:
    """Token stream of a server reply (the tokens a login / DML / DDL batch produces)."""
    r = Reply()
    i = 0
    cols: List[Tuple[int, int]] = []
    while i < len(b):
        tok = b[i]
        i += 1
        if tok in (0xFD, 0xFE, 0xFF):                          # DONE / DONEPROC / DONEINPROC
            status, _cmd, count = struct.unpack("<HHQ", b[i:i + 12])
            if status & 0x10:                                  # DONE_COUNT
                r.row_counts.append(count)
            i += 12
        elif tok in (0xAA, 0xAB):                              # ERROR / INFO
            ln = struct.unpack("<H", b[i:i + 2])[0]
            body = b[i + 2:i + 2 + ln]
            number, _state, klass = struct.unpack("<iBB", body[:6])
            msg, _ = _us_varchar(body, 6)
            i += 2 + ln
            if tok == 0xAA:
                raise TdsError(f"SQL Server error {number} (class {klass}): {msg}", number)
            r.infos.append(msg)
        elif tok == 0xAD:                                      # LOGINACK
            ln = struct.unpack("<H", b[i:i + 2])[0]
            i += 2 + ln
            r.logged_in = True
        elif tok == 0xE3:                                      # ENVCHANGE
            ln = struct.unpack("<H", b[i:i + 2])[0]
            body = b[i + 2:i + 2 + ln]
            if body and body[0] == 4:                          # packet size
                val, _ = _b_varchar(body, 1)
                r.packet_size = int(val)
            i += 2 + ln
        elif tok in (0xA9, 0xED, 0xA4, 0xA5):                  # ORDER, SSPI, TABNAME, COLINFO: skip
            ln = struct.unpack("<H", b[i:i + 2])[0]
            i += 2 + ln
        elif tok == 0x79:                                      # RETURNSTATUS
            i += 4
        elif tok == 0xAE:                                      # FEATUREEXTACK
            while b[i] != 0xFF:
                ln = struct.unpack("<I", b[i + 1:i + 5])[0]
                i += 5 + ln
            i += 1
        elif tok == 0x81:                                      # COLMETADATA (int / nvarchar results only)
            n = struct.unpack("<H", b[i:i + 2])[0]
            i += 2
            cols = []
            for _ in range(n if n != 0xFFFF else 0):
                i += 6                                         # usertype + flags
                t = b[i]
                i += 1
                if t in (0x26, 0x68, 0x6D, 0x6A, 0x6C):
                    ln = b[i]
                    i += 1
                    if t in (0x6A, 0x6C):
                        i += 2
                elif t in (0xE7, 0xA7, 0xEF, 0xAF):
                    ln = struct.unpack("<H", b[i:i + 2])[0]
                    i += 2 + 5
                elif t in (0x38, 0x7F, 0x3E, 0x30, 0x34, 0x32):
                    ln = {0x38: 4, 0x7F: 8, 0x3E: 8, 0x30: 1, 0x34: 2, 0x32: 1}[t]
                else:
                    raise TdsError(f"unsupported result column type 0x{t:02x}")
                _name, i = _b_varchar(b, i)
                cols.append((t, ln))
        elif tok == 0xD1:                                      # ROW
            row = []
            for t, ln in cols:
                if t in (0x38, 0x7F, 0x3E, 0x30, 0x34, 0x32):
                    raw = b[i:i + ln]
                    i += ln
                    row.append(_fixed_value(t, raw))
                elif t in (0xE7, 0xA7, 0xEF, 0xAF):
                    n = struct.unpack("<H", b[i:i + 2])[0]
                    i += 2
                    if n == 0xFFFF:
                        row.append(None)
                    else:
                        raw = b[i:i + n]
                        i += n
                        row.append(raw.decode("utf-16-le") if t in (0xE7, 0xEF) else raw.decode("latin-1"))
                else:
                    n = b[i]
                    i += 1
                    raw = b[i:i + n]
                    i += n
                    row.append(None if n == 0 else _fixed_value({0x26: {1: 0x30, 2: 0x34, 4: 0x38, 8: 0x7F},
                                                                0x6D: {4: 0x3B, 8: 0x3E}, 0x68: {1: 0x32}}
                                                               .get(t, {}).get(n, t), raw))
            r.rows.append(row)
        else:
            raise TdsError(f"unexpected TDS token 0x{tok:02x}")
    return r


def _fixed_value(t, raw):
    if t == 0x38:
        return struct.unpack("<i", raw)[0]
    if t == 0x7F:
        return struct.unpack("<q", raw)[0]
    if t == 0x3E:
        return struct.unpack("<d", raw)[0]
    if t == 0x3B:
        return struct.unpack("<f", raw)[0]
    if t == 0x30:
        return raw[0]
    if t == 0x34:
        return struct.unpack("<h", raw)[0]
    if t == 0x32:
        return bool(raw[0])
    return raw


# ---------------------------------------------------------------------------------------------------------------
# client
# ---------------------------------------------------------------------------------------------------------------

class TdsClient:
    def __init__(self, host: str, port: int = 1433, user: str = "", password: str = "", database: str = "",
                 encrypt: Optional[bool] = None, trust_server_certificate: bool = False,
                 host_name_in_certificate: Optional[str] = None, timeout: float = 30.0,
                 query_timeout: float = 30.0, cafile: Optional[str] = None):
        self.host, self.port = host, port
        self.packet_size = 4096
        self.query_timeout = query_timeout
        sock = socket.create_connection((host, port), timeout=timeout)
        sock.settimeout(query_timeout)
        self.ch = _Channel(sock)
        # PRELOGIN: ask for full encryption when the connection string says so; otherwise offer login-only
        want = ENCRYPT_ON if encrypt else ENCRYPT_OFF
        self.ch.send(_packet(PT_PRELOGIN, _prelogin_payload(want), self.packet_size))
        _t, payload = self.ch.read_message()
        server_enc = parse_prelogin(payload).get(0x01, b"\x02")[0]
        if encrypt and server_enc == ENCRYPT_NOT_SUP:
            raise TdsError("encrypt=true but the server does not support encryption")
        use_tls = server_enc != ENCRYPT_NOT_SUP
        full_tls = use_tls and (want == ENCRYPT_ON or server_enc in (ENCRYPT_ON, ENCRYPT_REQ))
        if use_tls:
            ctx = ssl.create_default_context(cafile=cafile)
            # TDS 7.x carries TLS 1.2 inside PRELOGIN packets (TLS 1.3 needs TDS 8 "strict" mode, whose TLS starts
            # before PRELOGIN); 1.3's post-handshake tickets would also arrive after the client stopped reading them
            ctx.maximum_version = ssl.TLSVersion.TLSv1_2
            if trust_server_certificate:
                ctx.check_hostname = False
                ctx.verify_mode = ssl.CERT_NONE
            # the certificate must name the server (a wildcard certificate matches the real host name); an explicit
            # non-wildcard hostNameInCertificate replaces the host in the check
            name = host_name_in_certificate if (host_name_in_certificate and
                                                not host_name_in_certificate.startswith("*")) else host
            self.ch.start_tls(ctx, name, self.packet_size)
        self.ch.send(_packet(PT_LOGIN7, login7_payload(socket.gethostname(), user, password, database,
                                                       server=host, packet_size=self.packet_size),
                             self.packet_size))
        if use_tls and not full_tls:
            self.ch.stop_tls()                   # login-only encryption
        _t, reply = self.ch.read_message()
        r = parse_reply(reply)
        if not r.logged_in:
            raise TdsError("login failed: no LOGINACK")
        if r.packet_size:
            self.packet_size = r.packet_size

    def execute(self, sql: str) -> Reply:
        self.ch.send(_packet(PT_SQLBATCH, _all_headers() + sql.encode("utf-16-le"), self.packet_size))
        _t, reply = self.ch.read_message()
        return parse_reply(reply)

    def bulk_insert(self, table: str, columns: Sequence[Tuple[str, str]], rows: Sequence[Sequence[Any]],
                    table_lock: bool = False) -> int:
        """``INSERT BULK`` + BulkLoadBCP rows.  ``columns``: (name, spark type) — long/int, double, boolean,
        string, timestamp."""
        specs = [_bulk_type(t) for _n, t in columns]
        hints = " WITH (TABLOCK)" if table_lock else ""
        # the rows are encoded BEFORE the INSERT BULK statement goes out: a value the bulk format cannot carry
        # (a string over 4000 characters) raises here, while the connection is still idle — once INSERT BULK is
        # acknowledged the server accepts nothing but the BulkLoadBCP message, so a fallback to INSERT must start
        # from an idle connection
        msg = bytearray(b"\x81") + struct.pack("<H", len(columns))
        for (name, _t), spec in zip(columns, specs):
            msg += struct.pack("<IH", 0, 0x0009) + spec[1]
            enc = name.encode("utf-16-le")
            msg += bytes([len(name)]) + enc
        for row in rows:
            msg += b"\xd1"
            for v, spec in zip(row, specs):
                msg += spec[2](v)
        msg += b"\xfd" + struct.pack("<HHQ", 0, 0, 0)
        self.execute(f"INSERT BULK {quote_ident(table)} (" +
                     ", ".join(f"{quote_ident(n)} {s[0]}" for (n, _t), s in zip(columns, specs)) + ")" + hints)
        self.ch.send(_packet(PT_BULK, bytes(msg), self.packet_size))
        _t, reply = self.ch.read_message()
        r = parse_reply(reply)
        return r.row_counts[-1] if r.row_counts else len(rows)

    def close(self):
        try:
            self.ch.sock.close()
        except OSError:
            pass


def quote_ident(name: str) -> str:
    parts = [p.strip("[]") for p in name.split(".")]
    return ".".join("[" + p.replace("]", "]]") + "]" for p in parts)


_COLLATION = bytes([0x09, 0x04, 0xD0, 0x00, 0x34])       # LCID 1033, CI_AS, sort id 52


def _enc_intn(v):
    return b"\x00" if v is None else b"\x08" + struct.pack("<q", int(v))


def _enc_fltn(v):
    return b"\x00" if v is None else b"\x08" + struct.pack("<d", float(v))


def _enc_bitn(v):
    return b"\x00" if v is None else b"\x01" + (b"\x01" if v else b"\x00")


def _enc_nvarchar(v):
    if v is None:
        return b"\xff\xff"
    b = str(v).encode("utf-16-le")
    if len(b) > 8000:
        raise TdsError("string longer than 4000 characters in bulk mode")
    return struct.pack("<H", len(b)) + b


_EPOCH_DAYS = (_dt.date(1970, 1, 1) - _dt.date(1, 1, 1)).days


def _enc_datetime2(v):
    if v is None:
        return b"\x00"
    if isinstance(v, str):
        v = _dt.datetime.fromisoformat(v.replace("Z", "+00:00"))
    if isinstance(v, _dt.datetime):
        if v.tzinfo is not None:
            v = v.astimezone(_dt.timezone.utc).replace(tzinfo=None)
        days = (v.date() - _dt.date(1, 1, 1)).days
        ticks = ((v.hour * 60 + v.minute) * 60 + v.second) * 10_000_000 + v.microsecond * 10
    else:                                                       # microseconds since the epoch
        us = int(v)
        d, rem = divmod(us, 86_400_000_000)
        days, ticks = _EPOCH_DAYS + d, rem * 10
    return b"\x08" + ticks.to_bytes(5, "little") + days.to_bytes(3, "little")


def _bulk_type(spark: str):
    t = (spark if isinstance(spark, str) else "string").lower()
    if t in ("long", "int", "integer", "short", "byte", "bigint"):
        return "bigint", b"\x26\x08", _enc_intn
    if t in ("double", "float", "decimal"):
        return "float", b"\x6d\x08", _enc_fltn
    if t == "boolean":
        return "bit", b"\x68\x01", _enc_bitn
    if t == "timestamp":
        return "datetime2(7)", b"\x2a\x07", _enc_datetime2
    return "nvarchar(4000)", b"\xe7" + struct.pack("<H", 8000) + _COLLATION, _enc_nvarchar


def sql_type(spark) -> str:
    t = (spark if isinstance(spark, str) else "string").lower()
    if t in ("long", "int", "integer", "short", "byte", "bigint"):
        return "bigint"
    if t in ("double", "float", "decimal"):
        return "float"
    if t == "boolean":
        return "bit"
    if t == "timestamp":
        return "datetime2(7)"
    if t == "date":
        return "date"
    return "nvarchar(max)"


def sql_literal(v) -> str:
    if v is None:
        return "NULL"
    if isinstance(v, bool):
        return "1" if v else "0"
    if isinstance(v, int):
        return str(v)
    if isinstance(v, float):
        if math.isnan(v) or math.isinf(v):
            return "NULL"
        return repr(v)
    if isinstance(v, _dt.datetime):
        return "'" + v.strftime("%Y-%m-%dT%H:%M:%S.%f") + "'"
    if isinstance(v, _dt.date):
        return "'" + v.isoformat() + "'"
    return "N'" + str(v).replace("'", "''") + "'"


class SqlServerWriter:
    """The SQL sink's writer: creates the table when missing (Spark JDBC ``append`` does), truncates it for
    ``writemode=overwrite``, then bulk-loads or INSERTs the rows."""

    def __init__(self, conn: str, table: str, write_mode: str = "append", url: Optional[str] = None,
                 database: Optional[str] = None, user: Optional[str] = None, password: Optional[str] = None,
                 encrypt=None, trust_server_certificate=None, host_name_in_certificate=None,
                 connect_timeout: float = 30, query_timeout: float = 30, bulk: bool = False,
                 bulk_batch: int = 2000, table_lock: bool = False):
        p = parse_connection_string(url or conn)
        self.kw = dict(host=p["host"], port=p["port"], user=user or p.get("user") or "",
                       password=password or p.get("password") or "", database=database or p.get("database") or "",
                       encrypt=_truthy(encrypt if encrypt is not None else p.get("encrypt")),
                       trust_server_certificate=_truthy(trust_server_certificate if trust_server_certificate
                                                        is not None else p.get("trust_server_certificate")),
                       host_name_in_certificate=host_name_in_certificate or p.get("host_name_in_certificate"),
                       timeout=float(p.get("timeout") or connect_timeout), query_timeout=float(query_timeout))
        self.table = table
        self.write_mode = (write_mode or "append").lower()
        self.bulk = bulk
        self.bulk_batch = max(1, int(bulk_batch))
        self._client: Optional[TdsClient] = None
        self._prepared = False

    def _conn(self) -> TdsClient:
        if self._client is None:
            self._client = TdsClient(**self.kw)
        return self._client

    def write(self, names: List[str], types: List[Any], rows: List[Sequence[Any]]) -> int:
        try:
            return self._write(names, types, rows)
        except (OSError, TdsError):
            if self._client is not None:
                self._client.close()
                self._client = None
            raise

    def _write(self, names, types, rows) -> int:
        c = self._conn()
        t = quote_ident(self.table)
        if not self._prepared:
            obj = self.table.replace("'", "''")
            if self.write_mode == "overwrite":
                c.execute(f"IF OBJECT_ID(N'{obj}', N'U') IS NOT NULL TRUNCATE TABLE {t}")
            elif self.write_mode == "errorifexists":
                c.execute(f"IF OBJECT_ID(N'{obj}', N'U') IS NOT NULL RAISERROR('table {obj} exists', 16, 1)")
            c.execute(f"IF OBJECT_ID(N'{obj}', N'U') IS NULL CREATE TABLE {t} (" +
                      ", ".join(f"{quote_ident(n)} {sql_type(ty)}" for n, ty in zip(names, types)) + ")")
            self._prepared = True
        if not rows:
            return 0
        n = 0
        if self.bulk:
            for i in range(0, len(rows), self.bulk_batch):
                try:
                    n += c.bulk_insert(self.table, list(zip(names, types)), rows[i:i + self.bulk_batch])
                except TdsError as e:
                    if "longer than 4000" not in str(e):
                        raise
                    n += self._insert(c, t, names, rows[i:i + self.bulk_batch])
            return n
        return self._insert(c, t, names, rows)

    def _insert(self, c, t, names, rows) -> int:
        cols = ", ".join(quote_ident(x) for x in names)
        n = 0
        for i in range(0, len(rows), 1000):                 # SQL Server's VALUES limit
            chunk = rows[i:i + 1000]
            sql = f"INSERT INTO {t} ({cols}) VALUES " + ", ".join(
                "(" + ", ".join(sql_literal(v) for v in r) + ")" for r in chunk)
            r = c.execute(sql)
            n += r.row_counts[-1] if r.row_counts else len(chunk)
        return n

    def close(self):
        if self._client is not None:
            self._client.close()
            self._client = None
