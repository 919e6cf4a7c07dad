"""Java-regex (the subset that is a regular language) → byte-level DFA for RLIKE on the device.

RLIKE is a *find*: true when any substring matches.  The automaton runs over UTF-8 bytes plus two virtual
symbols, BOS (fed first) and EOS (fed last), so ``^`` and ``$`` are ordinary transitions.  The search prefix is a
loop on every symbol before the pattern and the accept state loops on every symbol after it, so once a row reaches
an accepting state it stays there (the kernel stops early), and the empty state set is a dead end (also early exit).

Supported: literals and escapes, ``.`` (one code point, not a line terminator — Java's default), classes with
ranges / negation / ``\\d\\w\\s`` (ASCII, as Java's defaults), ``\\D\\W\\S`` and negated classes (which also take every
multi-byte code point), groups ``( )`` / ``(?: )``, alternation, ``* + ? {n} {n,} {n,m}`` (greedy or lazy — the
same language), ``^``, ``$`` (end, or before a final line feed).  Anything else (backreferences, look-around,
``\\b``, inline flags, possessive quantifiers, non-ASCII ranges, …) raises :class:`Unsupported` and the caller runs
the host regex.  The DFA is built over byte equivalence classes and kept ≤ 16 K table entries so it fits in LDS.
"""
from __future__ import annotations

import re
from dataclasses import dataclass
from typing import Dict, FrozenSet, List, Optional, Tuple

BOS, EOS, NSYM = 256, 257, 258
MAX_ENTRIES = 16384
MAX_NFA = 4000


class Unsupported(ValueError):
    pass


_ALL = frozenset(range(NSYM))
_DIGIT = frozenset(range(48, 58))
_WORD = frozenset(list(range(48, 58)) + list(range(65, 91)) + list(range(97, 123)) + [95])
_SPACE = frozenset([9, 10, 11, 12, 13, 32])
_ASCII = frozenset(range(128))
_CONT = frozenset(range(0x80, 0xC0))


# ---- AST ------------------------------------------------------------------------------------------------------
# ("seq", [nodes]) ("alt", [nodes]) ("rep", node, lo, hi|None, lazy) ("set", frozenset bytes) ("bytes", b"...")
# ("group", index, node) a capturing group (the DFA reads it as its node)
# ("any",) one code point except line terminators; ("notset", frozenset ascii) any code point outside an ASCII
# set (incl. every multi-byte one); ("bos",) ("eos",)


def _ends_with_cr(node) -> bool:
    return (node[0] == "set" and node[1] == frozenset([13])) or (node[0] == "bytes" and node[1].endswith(b"\r"))


class _Parser:
    def __init__(self, p: str):
        self.p, self.i = p, 0
        self.groups = 0

    def peek(self):
        return self.p[self.i] if self.i < len(self.p) else None

    def take(self):
        c = self.p[self.i]
        self.i += 1
        return c

    def parse(self):
        node = self.alt()
        if self.i != len(self.p):
            raise Unsupported(f"unbalanced ')' at {self.i}")
        return node

    def alt(self):
        branches = [self.seq()]
        while self.peek() == "|":
            self.take()
            branches.append(self.seq())
        return branches[0] if len(branches) == 1 else ("alt", branches)

    def seq(self):
        items = []
        while self.peek() is not None and self.peek() not in "|)":
            q = self.quantified()
            if q == ("eos",) and items and _ends_with_cr(items[-1]):
                q = ("eos", True)          # a literal \r before $: a final \n there is half of \r\n
            items.append(q)
        return ("seq", items)

    def quantified(self):
        atom = self.atom()
        while True:
            c = self.peek()
            if c == "*":
                self.take()
                atom = ("rep", atom, 0, None, False)
            elif c == "+":
                self.take()
                atom = ("rep", atom, 1, None, False)
            elif c == "?":
                self.take()
                atom = ("rep", atom, 0, 1, False)
            elif c == "{" and self._is_counted():
                lo, hi = self._counted()
                atom = ("rep", atom, lo, hi, False)
            else:
                return atom
            if atom[0] == "rep" and atom[1][0] in ("bos", "eos"):
                raise Unsupported("quantified anchor")
            nxt = self.peek()
            if nxt == "?":                  # lazy: the same language (the DFA), another match choice (the VM)
                self.take()
                atom = atom[:4] + (True,)
            elif nxt == "+":
                raise Unsupported("possessive quantifier")

    def _is_counted(self):
        j = self.p.find("}", self.i)
        body = self.p[self.i + 1:j] if j > 0 else ""
        return j > 0 and body != "" and all(ch.isdigit() or ch == "," for ch in body) and body[0] != ","

    def _counted(self):
        j = self.p.index("}", self.i)
        body = self.p[self.i + 1:j]
        self.i = j + 1
        if "," in body:
            a, b = body.split(",", 1)
            lo, hi = int(a), (int(b) if b else None)
        else:
            lo = hi = int(body)
        if (hi if hi is not None else lo) > 200 or (hi is not None and hi < lo):
            raise Unsupported("repeat count")
        return lo, hi

    def atom(self):
        c = self.take()
        if c == "(":
            capture = True
            if self.peek() == "?":
                self.take()
                if self.peek() != ":":
                    raise Unsupported("group construct (?" + (self.peek() or ""))
                self.take()
                capture = False
            if capture:
                self.groups += 1
                idx = self.groups
            node = self.alt()
            if self.peek() != ")":
                raise Unsupported("unclosed group")
            self.take()
            return ("group", idx, node) if capture else node
        if c == ".":
            return ("any",)
        if c == "^":
            return ("bos",)
        if c == "$":
            return ("eos",)
        if c == "[":
            return self.char_class()
        if c == "\\":
            return self.escape(in_class=False)
        if c in "*+?":
            raise Unsupported("dangling quantifier")
        return ("bytes", c.encode("utf-8"))

    def escape(self, in_class: bool):
        if self.peek() is None:
            raise Unsupported("trailing backslash")
        c = self.take()
        simple = {"t": 9, "n": 10, "r": 13, "f": 12, "a": 7, "e": 27}
        if c in simple:
            return ("set", frozenset([simple[c]]))
        if c == "d":
            return ("set", _DIGIT)
        if c == "w":
            return ("set", _WORD)
        if c == "s":
            return ("set", _SPACE)
        if c in "DWS":
            return ("notset", {"D": _DIGIT, "W": _WORD, "S": _SPACE}[c])
        if c == "x":
            h = self.p[self.i:self.i + 2]
            if len(h) != 2 or any(ch not in "0123456789abcdefABCDEF" for ch in h):
                raise Unsupported("\\x escape")
            self.i += 2
            v = int(h, 16)
            return ("bytes", chr(v).encode("utf-8"))
        if c.isalnum():
            raise Unsupported(f"escape \\{c}")       # \b \B \A \z \Q \p{..} \1 …
        return ("bytes", c.encode("utf-8"))

    def char_class(self):
        neg = False
        if self.peek() == "^":
            self.take()
            neg = True
        members: set = set()
        multi: List[bytes] = []
        negsets: List[FrozenSet[int]] = []
        first = True
        while True:
            c = self.peek()
            if c is None:
                raise Unsupported("unclosed class")
            if c == "]" and not first:
                self.take()
                break
            first = False
            if c == "[" or (c == "&" and self.p[self.i:self.i + 2] == "&&"):
                raise Unsupported("class union / intersection")
            self.take()
            if c == "\\":
                node = self.escape(in_class=True)
                if node[0] == "notset":
                    negsets.append(node[1])
                    continue
                lo_node = node
            else:
                lo_node = ("bytes", c.encode("utf-8"))
            if self.peek() == "-" and self.p[self.i + 1:self.i + 2] not in ("]", ""):
                self.take()
                d = self.take()
                hi_node = self.escape(in_class=True) if d == "\\" else ("bytes", d.encode("utf-8"))
                lo, hi = _single_cp(lo_node), _single_cp(hi_node)
                if lo > hi:
                    raise Unsupported("bad range")
                if hi >= 128:
                    raise Unsupported("non-ASCII range")
                members.update(range(lo, hi + 1))
                continue
            if lo_node[0] == "set":
                members.update(lo_node[1])
            else:
                b = lo_node[1]
                if len(b) == 1:
                    members.add(b[0])
                else:
                    multi.append(b)
        if neg:
            if multi or negsets:
                raise Unsupported("negated class with non-ASCII members")
            return ("notset", frozenset(members))
        if negsets:
            if len(negsets) > 1 or members or multi:
                raise Unsupported("mixed negated escapes in a class")
            return ("notset", negsets[0])
        alts = [("set", frozenset(members))] if members else []
        alts += [("bytes", b) for b in multi]
        if not alts:
            raise Unsupported("empty class")
        return alts[0] if len(alts) == 1 else ("alt", alts)


def _single_cp(node) -> int:
    if node[0] == "set" and len(node[1]) == 1:
        return next(iter(node[1]))
    if node[0] == "bytes":
        s = node[1].decode("utf-8")
        if len(s) == 1:
            return ord(s)
    raise Unsupported("class range endpoint")


# ---- Thompson NFA over symbol sets ---------------------------------------------------------------------------
class _NFA:
    def __init__(self):
        self.eps: List[List[int]] = []
        self.edges: List[List[Tuple[FrozenSet[int], int]]] = []

    def state(self) -> int:
        if len(self.eps) >= MAX_NFA:
            raise Unsupported("pattern too large")
        self.eps.append([])
        self.edges.append([])
        return len(self.eps) - 1

    def chain(self, sets: List[FrozenSet[int]]) -> Tuple[int, int]:
        s = self.state()
        cur = s
        for st in sets:
            nx = self.state()
            self.edges[cur].append((st, nx))
            cur = nx
        return s, cur

    def build(self, node) -> Tuple[int, int]:
        k = node[0]
        if k == "seq":
            s = e = self.state()
            for item in node[1]:
                a, b = self.build(item)
                self.eps[e].append(a)
                e = b
            return s, e
        if k == "alt":
            s, e = self.state(), self.state()
            for br in node[1]:
                a, b = self.build(br)
                self.eps[s].append(a)
                self.eps[b].append(e)
            return s, e
        if k == "set":
            return self.chain([node[1]])
        if k == "bytes":
            return self.chain([frozenset([b]) for b in node[1]])
        if k == "bos":
            return self.chain([frozenset([BOS])])
        if k == "eos":
            # Java's $ without MULTILINE (Pattern.Dollar): end of input, or before a final line terminator —
            # \r\n, \n, \r, U+0085 (C2 85), U+2028 / U+2029 (E2 80 A8/A9).  A final \n right after a \r is the
            # second half of \r\n, where $ does not match: when the pattern puts a literal \r just before the $,
            # the lone-\n alternative is left out (the lookbehind an NFA cannot express in general)
            s, e = self.state(), self.state()
            terms = [[], [frozenset([13]), frozenset([10])], [frozenset([13])], [frozenset([0xC2]), frozenset([0x85])],
                     [frozenset([0xE2]), frozenset([0x80]), frozenset([0xA8])],
                     [frozenset([0xE2]), frozenset([0x80]), frozenset([0xA9])]]
            if not node[1:] or not node[1]:
                terms.append([frozenset([10])])
            for t in terms:
                a, b = self.chain(t + [frozenset([EOS])])
                self.eps[s].append(a)
                self.eps[b].append(e)
            return s, e
        if k in ("any", "notset"):
            s, e = self.state(), self.state()
            if k == "any":
                ascii_ok = _ASCII - {10, 13}
                seqs = [[frozenset([0xC2]), _CONT - {0x85}],                       # U+0085 excluded
                        [frozenset(range(0xC0, 0xC2)) | frozenset(range(0xC3, 0xE0)), _CONT],
                        [frozenset([0xE2]), frozenset([0x80]), _CONT - {0xA8, 0xA9}],  # U+2028 / U+2029 excluded
                        [frozenset([0xE2]), _CONT - {0x80}, _CONT],
                        [frozenset(range(0xE0, 0xF0)) - {0xE2}, _CONT, _CONT],
                        [frozenset(range(0xF0, 0xF8)), _CONT, _CONT, _CONT]]
            else:
                ascii_ok = _ASCII - node[1]
                seqs = [[frozenset(range(0xC0, 0xE0)), _CONT], [frozenset(range(0xE0, 0xF0)), _CONT, _CONT],
                        [frozenset(range(0xF0, 0xF8)), _CONT, _CONT, _CONT]]
            for sq in [[frozenset(ascii_ok)]] + seqs:
                a, b = self.chain(sq)
                self.eps[s].append(a)
                self.eps[b].append(e)
            return s, e
        if k == "group":
            return self.build(node[2])
        if k == "rep":
            _, sub, lo, hi, _lazy = node
            s = e = self.state()
            for _ in range(lo):
                a, b = self.build(sub)
                self.eps[e].append(a)
                e = b
            if hi is None:
                a, b = self.build(sub)
                loop = self.state()
                self.eps[e].append(loop)
                self.eps[loop].append(a)
                self.eps[b].append(loop)
                e = loop
            else:
                end = self.state()
                for _ in range(hi - lo):
                    self.eps[e].append(end)
                    a, b = self.build(sub)
                    self.eps[e].append(a)
                    e = b
                self.eps[e].append(end)
                e = end
            return s, e
        raise Unsupported(k)


@dataclass
class DFA:
    table: List[int]          # [n_states × n_classes] next state; bit 15 set when the target is terminal
    classes: List[int]        # symbol (0..257) → class
    accept: List[int]         # per state 1/0
    n_states: int
    n_classes: int
    start: int


_CACHE: Dict[str, DFA] = {}


def compile_rlike(pattern: str) -> DFA:
    """Pattern → DFA (cached); raises Unsupported for constructs outside the regular subset."""
    hit = _CACHE.get(pattern)
    if hit is not None:
        return hit
    ast = _Parser(pattern).parse()
    nfa = _NFA()
    s0 = nfa.state()
    nfa.edges[s0].append((_ALL, s0))             # search prefix
    a, b = nfa.build(ast)
    nfa.eps[s0].append(a)
    acc = nfa.state()
    nfa.eps[b].append(acc)
    nfa.edges[acc].append((_ALL, acc))           # once matched, always matched
    dfa = _subset(nfa, s0, acc)
    if len(_CACHE) > 256:
        _CACHE.clear()
    _CACHE[pattern] = dfa
    return dfa


def _subset(nfa: _NFA, s0: int, acc: int) -> DFA:
    # symbol equivalence classes: symbols that every edge set treats alike
    sets = {st for edges in nfa.edges for st, _ in edges}
    sig: Dict[Tuple, int] = {}
    classes = []
    for sym in range(NSYM):
        key = tuple(sym in st for st in sets)
        classes.append(sig.setdefault(key, len(sig)))
    ncls = len(sig)
    rep = [0] * ncls
    for sym in range(NSYM - 1, -1, -1):
        rep[classes[sym]] = sym

    def closure(states) -> FrozenSet[int]:
        out, stack = set(states), list(states)
        while stack:
            x = stack.pop()
            for y in nfa.eps[x]:
                if y not in out:
                    out.add(y)
                    stack.append(y)
        return frozenset(out)

    dead = frozenset()
    index: Dict[FrozenSet[int], int] = {dead: 0}
    order = [dead]
    start = closure([s0])
    index[start] = 1
    order.append(start)
    rows: List[List[int]] = []
    i = 0
    while i < len(order):
        cur = order[i]
        row = []
        for c in range(ncls):
            sym = rep[c]
            nxt = closure([t for x in cur for st, t in nfa.edges[x] if sym in st]) if cur else dead
            j = index.get(nxt)
            if j is None:
                j = len(order)
                index[nxt] = j
                order.append(nxt)
                if len(order) * ncls > MAX_ENTRIES:
                    raise Unsupported("DFA too large")
            row.append(j)
        rows.append(row)
        i += 1
    accept = [1 if acc in st else 0 for st in order]
    table = [(j | 0x8000) if (j == 0 or accept[j]) else j for row in rows for j in row]
    return DFA(table, classes, accept, len(order), ncls, 1)


def run_dfa(dfa: DFA, data: bytes) -> bool:
    """Host execution of the same automaton (tests and the CPU path)."""
    st = dfa.start
    for sym in (BOS, *data, EOS):
        st = dfa.table[st * dfa.n_classes + dfa.classes[sym]] & 0x7FFF
        if st == 0 or dfa.accept[st]:
            break
    return bool(dfa.accept[st])


_INLINE_FLAGS = re.compile(r"\(\?([idmsuxU]*)(?:-([idmsuxU]*))?([:)])")
_LT_ALL = "\\n\\r\\u0085\\u2028\\u2029"


def java_to_python(pattern: str) -> str:
    """Host-regex form of a Java pattern for the cases ``re`` reads differently (use with ``re.ASCII`` so that
    ``\\d\\w\\s`` are ASCII as in Java):

    * ``.`` takes no line terminator (\\n \\r U+0085 U+2028 U+2029) — any character under ``(?s)`` (DOTALL);
    * ``$`` is end of input or before a FINAL line terminator; under ``(?m)`` (MULTILINE) before ANY line terminator
      (never between \\r and \\n) or at the end (java.util.regex.Pattern.Dollar);
    * ``^`` under ``(?m)`` is the start, or after any line terminator except at the end of input (Pattern.Caret);
    * ``(?d)`` (UNIX_LINES) makes \\n the only line terminator for all three.

    Inline flags apply from where they appear to the end of the enclosing group, or inside ``(?flags:…)``; the
    ``m``/``s``/``d`` semantics are compiled into the output here, so those letters (and ``u``/``U``) are removed
    from the flag groups Python sees."""
    out, i, in_cls = [], 0, False
    flags = set()
    stack = []
    while i < len(pattern):
        c = pattern[i]
        if c == "\\" and i + 1 < len(pattern):
            out.append(pattern[i:i + 2])
            i += 2
            continue
        if not in_cls and c == "(":
            m = _INLINE_FLAGS.match(pattern, i)
            if m:
                on, off, end = set(m.group(1)), set(m.group(2) or ""), m.group(3)
                new = (flags | on) - off
                keep_on = "".join(f for f in m.group(1) if f in "ix")
                keep_off = "".join(f for f in (m.group(2) or "") if f in "ix")
                grp = keep_on + ("-" + keep_off if keep_off else "")
                if end == ":":
                    stack.append(flags)
                    flags = new
                    out.append(f"(?{grp}:" if grp else "(?:")
                else:
                    flags = new
                    if grp:
                        out.append(f"(?{grp})")
                i = m.end()
                continue
            stack.append(set(flags))
            out.append(c)
            i += 1
            continue
        if not in_cls and c == ")":
            if stack:
                flags = stack.pop()
            out.append(c)
            i += 1
            continue
        lt = "\\n" if "d" in flags else _LT_ALL
        if in_cls:
            if c == "]":
                in_cls = False
        elif c == "[":
            in_cls = True
            if pattern[i + 1:i + 2] == "^":
                out.append("[^")
                i += 2
                if pattern[i:i + 1] == "]":
                    out.append("]")
                    i += 1
                continue
            if pattern[i + 1:i + 2] == "]":
                out.append("[]")
                i += 2
                continue
        elif c == ".":
            out.append(r"[\s\S]" if "s" in flags else f"[^{lt}]")
            i += 1
            continue
        elif c == "$":
            if "d" in flags:
                out.append(r"(?=\n)" if "m" in flags else r"(?:(?=\n\Z)|\Z)")
            elif "m" in flags:
                # MULTILINE: before any line terminator (before the \r of \r\n, never between them), or the end
                out.append(r"(?:(?=[\r\u0085\u2028\u2029])|(?<!\r)(?=\n)|\Z)")
            else:
                # end of input, or before a final line terminator — \r\n, \n (not right after a \r), \r, U+0085,
                # U+2028, U+2029 (Pattern.Dollar); Python's $ knows only a final \n
                out.append(r"(?:(?=\r\n\Z)|(?<!\r)(?=\n\Z)|(?=[\r\u0085\u2028\u2029]\Z)|\Z)")
            i += 1
            continue
        elif c == "^" and "m" in flags:
            if "d" in flags:
                out.append(r"(?:\A|(?<=\n)(?!\Z))")
            else:
                out.append(r"(?:\A|(?<=[\n\u0085\u2028\u2029])(?!\Z)|(?<=\r)(?!\n)(?!\Z))")
            i += 1
            continue
        out.append(c)
        i += 1
    return "".join(out)
