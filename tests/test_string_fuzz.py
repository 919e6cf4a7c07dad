"""Differential fuzzing of the device string kernels (strings.hip, json_serialize.hip) against the engine's CPU
reference: random UTF-8 strings over a small alphabet (so that patterns and needles actually hit) through LIKE,
substring / left / right / trim, instr / locate, replace, concat_ws, CAST(string AS BIGINT/INT/DOUBLE) and
CAST(double AS STRING) over random bit patterns.  The CPU side is checked against Python's own semantics first."""
import math
import random
import re
import struct

import pytest

from dxa.engine.column import Table, column_from_pylist, strings_from_pylist
from dxa.engine.expr import EvalContext
from dxa.engine.query import Catalog, run_sql

_ALPHA = ["a", "b", "X", " ", "\t", "é", "日", "%", "_", "\\"]
N = 400


def _rand_str(rnd, k=12):
    if rnd.random() < 0.05:
        return None
    return "".join(rnd.choice(_ALPHA) for _ in range(rnd.randint(0, k)))


def _rand_pattern(rnd):
    out = []
    for _ in range(rnd.randint(0, 6)):
        r = rnd.random()
        out.append("%" if r < 0.25 else "_" if r < 0.4 else "\\%" if r < 0.45 else "\\_" if r < 0.5 else
                   rnd.choice(["a", "b", "X", " ", "é", "日"]))
    return "".join(out)


def _like_regex(p):
    rx, i = [], 0
    while i < len(p):
        ch = p[i]
        if ch == "\\" and i + 1 < len(p):
            rx.append(re.escape(p[i + 1]))
            i += 2
            continue
        rx.append(".*" if ch == "%" else "." if ch == "_" else re.escape(ch))
        i += 1
    return re.compile("".join(rx), re.S)


def _run(sql, vals, device, dtype="string"):
    col = strings_from_pylist(vals, device) if dtype == "string" else column_from_pylist(vals, dtype, device)
    cat = Catalog()
    cat.register("F", Table(["s"], [col]))
    return [c.to_pylist() for c in run_sql(sql, cat, EvalContext(device=device)).columns]


def _q(s):
    return s.replace("\\", "\\\\").replace("'", "\\'")


def test_like_cpu_matches_regex():
    rnd = random.Random(7)
    vals = [_rand_str(rnd) for _ in range(N)]
    for _ in range(20):
        pat = _rand_pattern(rnd)
        got = _run(f"SELECT s LIKE '{_q(pat)}' AS m FROM F", vals, "cpu")[0]
        rx = _like_regex(pat)
        assert got == [None if v is None else bool(rx.fullmatch(v)) for v in vals], pat


@pytest.mark.gpu
def test_like_fuzz_gpu_match_cpu(gpu):
    rnd = random.Random(11)
    vals = [_rand_str(rnd, 16) for _ in range(N)]
    for _ in range(60):
        pat = _rand_pattern(rnd)
        sql = f"SELECT s LIKE '{_q(pat)}' AS m FROM F"
        assert _run(sql, vals, gpu) == _run(sql, vals, "cpu"), pat


@pytest.mark.gpu
def test_character_functions_fuzz_gpu_match_cpu(gpu):
    rnd = random.Random(13)
    vals = [_rand_str(rnd) for _ in range(N)]
    for _ in range(25):
        p, n = rnd.randint(-14, 14), rnd.randint(-2, 14)
        a, b = rnd.choice(["a", "X", "é", "日", "a ", "", "%_"]), rnd.choice(["", "-", "日本", "zz"])
        k = rnd.randint(-1, 14)
        sql = (f"SELECT substring(s, {p}, {n}) AS a, substr(s, {p}) AS b, left(s, {n}) AS c, right(s, {n}) AS d, "
               f"trim(s) AS e, ltrim(s) AS f, rtrim(s) AS g, length(s) AS h, instr(s, '{a}') AS i, "
               f"locate('{a}', s, {k}) AS j, replace(s, '{a}', '{b}') AS k, concat_ws('{b}', s, '{a}', s) AS l "
               f"FROM F")
        assert _run(sql, vals, gpu) == _run(sql, vals, "cpu"), sql


def _rand_num_str(rnd):
    parts = rnd.choice([["", " ", "\t"], [""]])
    s = rnd.choice(parts) + rnd.choice(["", "+", "-"])
    s += "".join(rnd.choice("0123456789") for _ in range(rnd.randint(0, 22)))
    if rnd.random() < 0.4:
        s += "." + "".join(rnd.choice("0123456789") for _ in range(rnd.randint(0, 6)))
    if rnd.random() < 0.2:
        s += rnd.choice("eE") + rnd.choice(["", "-", "+"]) + str(rnd.randint(0, 400))
    if rnd.random() < 0.1:
        s += rnd.choice(["x", " ", "d", "f", "L"])
    return s


@pytest.mark.gpu
def test_string_to_number_fuzz_gpu_match_cpu(gpu):
    rnd = random.Random(17)
    vals = [_rand_num_str(rnd) for _ in range(2 * N)] + ["Infinity", "-Infinity", "NaN", "inf", "nan"]
    sql = "SELECT CAST(s AS BIGINT) AS l, CAST(s AS INT) AS i, CAST(s AS DOUBLE) AS d FROM F"
    canon = [[("nan" if isinstance(x, float) and x != x else x) for x in c] for c in _run(sql, vals, "cpu")]
    got = [[("nan" if isinstance(x, float) and x != x else x) for x in c] for c in _run(sql, vals, gpu)]
    for a, b, s in zip(zip(*canon), zip(*got), vals):
        assert a == b, s


def test_double_to_string_cpu_round_trips():
    rnd = random.Random(19)
    vals = [struct.unpack("<d", struct.pack("<Q", rnd.getrandbits(64)))[0] for _ in range(N)]
    vals = [v for v in vals if math.isfinite(v)]
    out = _run("SELECT CAST(s AS STRING) AS t FROM F", vals, "cpu", "double")[0]
    for v, s in zip(vals, out):
        assert float(s) == v, (v, s)          # shortest round-trip digits in Java's layout


@pytest.mark.gpu
def test_double_to_string_fuzz_gpu_match_cpu(gpu):
    rnd = random.Random(23)
    vals = [struct.unpack("<d", struct.pack("<Q", rnd.getrandbits(64)))[0] for _ in range(4 * N)]
    vals += [rnd.uniform(-1e8, 1e8) for _ in range(N)] + [float(rnd.randint(-10**9, 10**9)) for _ in range(N)]
    vals += [10.0 ** e for e in range(-12, 22)] + [None]
    sql = "SELECT CAST(s AS STRING) AS t FROM F"
    assert _run(sql, vals, gpu, "double") == _run(sql, vals, "cpu", "double")


def _rand_regex(rnd, depth=0):
    out = []
    for _ in range(rnd.randint(1, 4)):
        r = rnd.random()
        if r < 0.12 and depth < 2:
            atom = "(" + "|".join(_rand_regex(rnd, depth + 1) for _ in range(rnd.randint(1, 3))) + ")"
        elif r < 0.22:
            atom = rnd.choice(["[ab]", "[^a]", "[a-cX]", "[\\d\\s]", "[日é]", "[^ X]"])
        elif r < 0.32:
            atom = rnd.choice([".", "\\w", "\\W", "\\s", "\\S", "\\d", "\\D", "\\\\", "\\%", "\\t"])
        else:
            atom = rnd.choice(["a", "b", "X", " ", "é", "日", "%", "_"])
        q = rnd.random()
        atom += "" if q < 0.6 else rnd.choice(["*", "+", "?", "{2}", "{1,3}", "{0,}", "*?", "+?"])
        out.append(atom)
    s = "".join(out)
    if depth == 0:
        s = ("^" if rnd.random() < 0.2 else "") + s + ("$" if rnd.random() < 0.2 else "")
    return s


def test_rlike_dfa_matches_host_regex():
    from dxa.ops.regex_dfa import compile_rlike, java_to_python, run_dfa
    rnd = random.Random(29)
    vals = [v for v in (_rand_str(rnd, 10) for _ in range(300)) if v is not None] + ["a\n", "\r", "x "]
    for _ in range(150):
        pat = _rand_regex(rnd)
        dfa = compile_rlike(pat)
        rx = re.compile(java_to_python(pat), re.ASCII)
        for v in vals:
            assert run_dfa(dfa, v.encode()) == (rx.search(v) is not None), (pat, v)


@pytest.mark.gpu
def test_rlike_fuzz_gpu_match_cpu(gpu):
    rnd = random.Random(31)
    vals = [_rand_str(rnd, 16) for _ in range(N)]
    for _ in range(60):
        pat = _rand_regex(rnd)
        sql = f"SELECT s RLIKE '{_q(pat)}' AS m, s NOT RLIKE '{_q(pat)}' AS n FROM F"
        assert _run(sql, vals, gpu) == _run(sql, vals, "cpu"), pat


def test_digest_functions_cpu_reference():
    import base64
    import hashlib
    import zlib
    vals = ["", "abc", "日本語", None]
    out = _run("SELECT md5(s) AS a, sha1(s) AS b, sha2(s, 256) AS c, sha2(s, 224) AS d, crc32(s) AS e, hex(s) AS f, "
               "base64(s) AS g FROM F", vals, "cpu")
    for i, v in enumerate(vals):
        if v is None:
            assert all(c[i] is None for c in out)
            continue
        b = v.encode()
        assert [c[i] for c in out] == [hashlib.md5(b).hexdigest(), hashlib.sha1(b).hexdigest(),
                                       hashlib.sha256(b).hexdigest(), hashlib.sha224(b).hexdigest(),
                                       zlib.crc32(b), b.hex().upper(), base64.b64encode(b).decode()]


@pytest.mark.gpu
def test_digest_functions_gpu_match_cpu(gpu):
    rnd = random.Random(37)
    vals = [_rand_str(rnd, 40) for _ in range(N)]
    vals += ["x" * k for k in (0, 1, 54, 55, 56, 57, 63, 64, 65, 119, 120, 1000)] + ["é" * 28, "日" * 40]
    sql = ("SELECT md5(s) AS a, sha1(s) AS b, sha2(s, 256) AS c, sha2(s, 224) AS d, sha2(s, 0) AS e, crc32(s) AS f, "
           "hex(s) AS g, base64(s) AS h, sha2(s, 512) AS i FROM F")
    assert _run(sql, vals, gpu) == _run(sql, vals, "cpu")


def test_regexp_host_java_semantics():
    vals = ["key=abc;x=1", "no", "a\r", "baaac", None]
    out = _run("SELECT regexp_extract(s, 'key=(\\\\w*)', 1) AS a, regexp_replace(s, 'a*', '-') AS b, "
               "regexp_extract(s, 'a.', 0) AS c, regexp_replace(s, '(a)(a)?', '[$2$1]') AS d FROM F", vals, "cpu")
    assert out[0] == ["abc", "", "", "", None]
    assert out[1][3] == "-b--c-"                       # Java's empty-match stepping
    assert out[2][2] == ""                             # '.' does not take \r (Java)
    assert out[3][3] == "b[aa][a]c"


@pytest.mark.gpu
def test_regexp_fuzz_gpu_match_cpu(gpu):
    from dxa.ops import regex_vm, strings as S
    from dxa.engine.column import strings_from_pylist
    rnd = random.Random(41)
    vals = [_rand_str(rnd, 16) for _ in range(N)]
    col = strings_from_pylist(vals, gpu)
    for _ in range(60):
        pat = _rand_regex(rnd)
        prog = regex_vm.compile_vm(pat)
        g = rnd.randint(0, min(prog.ngroups, 9))
        rep = rnd.choice(["", "#", "<$0>", "[$1]" if prog.ngroups >= 1 else "x", "\\$"])
        sql = (f"SELECT regexp_extract(s, '{_q(pat)}', {g}) AS a, regexp_replace(s, '{_q(pat)}', '{_q(rep)}') AS b "
               f"FROM F")
        assert _run(sql, vals, gpu) == _run(sql, vals, "cpu"), (pat, g, rep)
        _, bad = S.regex_extract(col, prog, g)
        assert not bool(bad.any()), pat                  # the device path itself produced the answer


# Java's $ without MULTILINE (Pattern.Dollar): end of input, or before a final \r\n, \n (not right after \r), \r,
# U+0085, U+2028, U+2029.  Expected values are Java's.
DOLLAR_CASES = [
    ("a$", "a", True), ("a$", "a\n", True), ("a$", "a\r", True), ("a$", "a\r\n", True), ("a$", "a ", True),
    ("a$", "a ", True), ("a$", "a\u0085", True), ("a$", "a\n\n", False), ("a$", "a\r\r", False),
    ("a$", "ab", False), ("a\r$", "a\r\n", False), ("a\r$", "a\r", True), ("^x.*$", "xyz\r\n", True),
    ("b$", "ab c", False),
]


@pytest.mark.parametrize("pattern,value,want", DOLLAR_CASES)
def test_java_dollar_terminators_host_and_dfa(pattern, value, want):
    import re
    from dxa.ops.regex_dfa import compile_rlike, java_to_python, run_dfa
    assert bool(re.search(java_to_python(pattern), value, re.ASCII)) == want
    assert run_dfa(compile_rlike(pattern), value.encode("utf-8")) == want


@pytest.mark.gpu
def test_java_dollar_terminators_gpu(gpu):
    """The same $ cases through the device RLIKE (DFA kernel) and regexp_extract (VM, its EOL opcode)."""
    for pattern, value, want in DOLLAR_CASES:
        sql = f"SELECT s RLIKE '{_q(pattern)}' AS m, regexp_extract(s, '({_q(pattern)})', 1) AS x FROM F"
        got = _run(sql, [value], gpu)
        assert got == _run(sql, [value], "cpu"), (pattern, value)
        assert bool(got[0][0]) == want, (pattern, value, got)


@pytest.mark.parametrize("pattern,value,want", [
    ("(?m)^b$", "a\nb\nc", True), ("^b$", "a\nb\nc", False),           # MULTILINE: every line end / start
    ("(?m)a$", "a\r\nb", True), ("(?m)a\r$", "a\r\nb", False),          # never between \r and \n
    ("(?m)^c", "a c", True), ("(?m)^$", "a\n", False),             # ^ not after a final terminator
    ("(?s)a.b", "a\nb", True), ("a.b", "a\nb", False),                   # DOTALL
    ("(?d)a.b", "a\rb", True), ("a.b", "a\rb", False),                   # UNIX_LINES: \n only
    ("(?d)a$", "a\r", False), ("a$", "a\r", True),
    ("(?m:^b)|zz", "a\nb", True), ("(?m:x)|^b", "a\nb", False),          # scoped flags end with their group
    ("(?i)ABC", "xabc", True)])
def test_java_inline_flags_host(pattern, value, want):
    """Java's MULTILINE / DOTALL / UNIX_LINES inline flags on the host regex path (java.util.regex.Pattern's Caret,
    Dollar and Dot), which Python's ``re`` reads differently."""
    import re
    from dxa.ops.regex_dfa import java_to_python
    assert bool(re.search(java_to_python(pattern), value, re.ASCII)) == want
