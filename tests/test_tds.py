"""SQL Server sink over TDS 7.4 against the in-process fake server (tests/tds_fake.py): connection strings, login
(plain, login-only TLS, full TLS), INSERT and bulk-load paths, table creation / overwrite, server errors — plus the
"fail loudly" rule for SQL and Cosmos connection strings that parse as neither (SqlSinker.scala:19-107)."""
import datetime as dt
import subprocess

import pytest

from dxa.io import tds as T
from tests.tds_fake import FakeSqlServer


@pytest.fixture(scope="module")
def cert(tmp_path_factory):
    d = tmp_path_factory.mktemp("cert")
    key, crt = d / "k.pem", d / "c.pem"
    r = subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", str(key), "-out",
                        str(crt), "-days", "2", "-subj", "/CN=localhost", "-addext", "subjectAltName=DNS:localhost"],
                       capture_output=True)
    if r.returncode != 0:
        pytest.skip("openssl unavailable")
    return str(crt), str(key)


def test_connection_strings():
    j = T.parse_connection_string("jdbc:sqlserver://srv.database.windows.net:1444;database=iot;user=u@srv;"
                                  "password=p;encrypt=true;trustServerCertificate=false;"
                                  "hostNameInCertificate=*.database.windows.net;loginTimeout=30;")
    assert (j["host"], j["port"], j["database"], j["user"], j["password"], j["encrypt"]) == \
        ("srv.database.windows.net", 1444, "iot", "u@srv", "p", "true")
    a = T.parse_connection_string("Server=tcp:srv.database.windows.net,1433;Initial Catalog=iot;User ID=u;"
                                  "Password=p;Encrypt=True;TrustServerCertificate=False;Connection Timeout=30;")
    assert (a["host"], a["port"], a["database"], a["user"], a["password"]) == ("srv.database.windows.net", 1433,
                                                                               "iot", "u", "p")
    assert T.is_sqlserver_connection("jdbc:sqlserver://x:1;") and T.is_sqlserver_connection("Server=x;Database=y")
    assert not T.is_sqlserver_connection("sqlite:///x.db")
    assert T.decode_password(T.encode_password("p@ss wörd")) == "p@ss wörd"
    assert T.sql_literal("it's") == "N'it''s'" and T.sql_literal(None) == "NULL" and T.sql_literal(True) == "1"


def _table():
    from dxa.engine.column import Table
    from dxa.engine.types import StructField, StructType
    schema = StructType((StructField("deviceId", "long"), StructField("name", "string"),
                         StructField("temp", "double"), StructField("ok", "boolean"),
                         StructField("ts", "timestamp")))
    rows = [{"deviceId": i, "name": None if i == 2 else f"dev '{i}'", "temp": i * 1.5, "ok": i % 2 == 0,
             "ts": dt.datetime(2024, 5, 6, 7, 8, 9, 123456)} for i in range(5)]
    return Table.from_pylist(rows, schema)


def _sink(conn, **extra):
    from dxa.config.settings import SettingDictionary
    from dxa.io.sinks import _sql_sink
    d = {"connectionstring": conn, "table": "dbo.Devices"}
    d.update(extra)
    return _sql_sink(SettingDictionary(d), "Devices")


@pytest.mark.parametrize("encryption", ["none", "login", "full"])
def test_insert_path(encryption, cert):
    srv = FakeSqlServer(encryption=encryption, certfile=cert[0], keyfile=cert[1])
    try:
        enc = "true" if encryption == "full" else "false"
        s = _sink(f"jdbc:sqlserver://127.0.0.1:{srv.port};database=iot;user=sa;password=p@ss;encrypt={enc};"
                  f"trustServerCertificate=true;")
        t = _table()
        assert s.write(None, t, None, None) == 5
        assert s.write(None, t, None, None) == 5
        tab = srv.tables["dbo.Devices"]
        assert srv.logins[0][:2] == ("sa", "iot")
        # CREATE TABLE once (guarded), then INSERT … VALUES; NULLs and quotes survive the literal rendering
        assert any("CREATE TABLE [dbo].[Devices]" in q for q in srv.statements)
        assert "[deviceId] bigint" in next(q for q in srv.statements if "CREATE TABLE" in q)
        data = tab["rows"]
        assert len(data) == 10 and data[2][1] is None and data[1][1] == "dev '1'" and data[3][2] == 4.5
    finally:
        srv.close()


def test_bulk_path_and_overwrite(cert):
    srv = FakeSqlServer(encryption="login", certfile=cert[0], keyfile=cert[1])
    try:
        s = _sink(f"Server=tcp:127.0.0.1,{srv.port};Initial Catalog=iot;User ID=sa;Password=p@ss;"
                  "TrustServerCertificate=True;", usebulkinsert="true", bulkcopybatchsize="2", writemode="overwrite")
        assert s.write(None, _table(), None, None) == 5
        tab = srv.tables["dbo.Devices"]
        assert any(q.startswith("INSERT BULK [dbo].[Devices]") for q in srv.statements)
        assert any("TRUNCATE TABLE" in q for q in srv.statements)
        got = tab["rows"]
        assert len(got) == 5 and got[2][1] is None and got[4][0] == 4 and got[0][3] is True
        ticks, days = got[0][4]
        assert days == (dt.date(2024, 5, 6) - dt.date(1, 1, 1)).days
        assert ticks == ((7 * 60 + 8) * 60 + 9) * 10_000_000 + 1234560
    finally:
        srv.close()


def test_login_failure_and_server_error_raise():
    srv = FakeSqlServer(encryption="none")
    try:
        s = _sink(f"jdbc:sqlserver://127.0.0.1:{srv.port};database=iot;user=sa;password=wrong;")
        with pytest.raises(T.TdsError, match="Login failed"):
            s.write(None, _table(), None, None)
        c = T.TdsClient("127.0.0.1", srv.port, "sa", "p@ss", "iot")
        with pytest.raises(T.TdsError, match="Invalid object name"):
            c.execute("INSERT INTO [nope] ([a]) VALUES (1)")
        c.close()
    finally:
        srv.close()


def test_unparseable_connection_strings_fail_at_start():
    from dxa.config.settings import SettingDictionary
    from dxa.io.sinks import _cosmos_sink
    with pytest.raises(ValueError, match="sql.connectionstring"):
        _sink("Driver={ODBC};Something")
    with pytest.raises(ValueError, match="cosmosdb.connectionstring"):
        _cosmos_sink(SettingDictionary({"connectionstring": "mongodb://x"}), "o")
    assert _sink("local:") is not None and _sink("sqlite:////tmp/x.db") is not None
    assert _cosmos_sink(SettingDictionary({"connectionstring": "local:"}), "o") is not None


def test_bulk_falls_back_to_insert_for_long_strings():
    """A chunk holding a string over 4000 characters cannot travel as a bulk-load nvarchar(4000): the writer finds
    it while encoding, before INSERT BULK is sent, and INSERTs that chunk on the idle connection (the fake, like a
    real server, drops a connection that sends anything but the BulkLoadBCP message after INSERT BULK)."""
    from dxa.engine.column import Table
    from dxa.engine.types import StructField, StructType
    srv = FakeSqlServer(encryption="none")
    try:
        s = _sink(f"jdbc:sqlserver://127.0.0.1:{srv.port};database=iot;user=sa;password=p@ss;",
                  usebulkinsert="true", bulkcopybatchsize="2")
        schema = StructType((StructField("deviceId", "long"), StructField("name", "string")))
        rows = [{"deviceId": i, "name": ("x" * 5000) if i == 2 else f"d{i}"} for i in range(5)]
        assert s.write(None, Table.from_pylist(rows, schema), None, None) == 5
        assert not srv.protocol_errors
        got = sorted(srv.tables["dbo.Devices"]["rows"])
        assert [r[0] for r in got] == [0, 1, 2, 3, 4] and len(got[2][1]) == 5000
        assert sum(q.startswith("INSERT BULK") for q in srv.statements) == 2           # chunks {0,1} and {4}
        assert sum(q.startswith("INSERT INTO") for q in srv.statements) == 1           # chunk {2,3}
    finally:
        srv.close()
