"""Java regex → a backtracking program for regexp_extract / regexp_replace on the device (strings.hip,
``str_regex_kernel``).

Extraction needs the match the Java engine picks — leftmost, then by alternation order and greedy / lazy
preference — and the capture groups, which a DFA cannot give.  So the pattern (the parser of regex_dfa.py, the same
supported subset) is compiled to a small backtracking program (SPLIT x,y tries x first, as java.util.regex does) that
one lane runs per row, start position by start position, with a bounded backtrack stack and step budget.  A row that
runs out of either is flagged and recomputed by the host regex, so the result never depends on the budget.

Instructions (int32 × 4: op, a, b, c):
  CHAR b · SET k (ASCII byte in bitmap k) · ANY (one code point, not a line terminator) · NOTSET k (one code point,
  not an ASCII member of bitmap k) · SPLIT x y · JMP x · SAVE k · BOL · EOL (end, or before a final \\n) · MATCH ·
  LOOP k top out
An unbounded loop whose body can match empty records its start position each iteration (SAVE into a slot after the
captures); LOOP leaves instead of iterating again when the body consumed nothing, as Java's Loop node does, so
``(a*)*`` terminates.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List

from .regex_dfa import BOS, EOS, Unsupported, _Parser  # noqa: F401  (BOS/EOS: shared symbol numbering)

CHAR, SET, ANY, NOTSET, SPLIT, JMP, SAVE, BOL, EOL, MATCH, LOOP = range(11)
MAX_PROG = 4096
MAX_GROUPS = 9
LOOP_SLOTS = (20, 32)      # position registers of unbounded loops whose body can match empty (after the captures)


@dataclass
class Program:
    code: List[int] = field(default_factory=list)       # 4 ints per instruction
    sets: List[int] = field(default_factory=list)       # 8 uint32 words per bitmap
    ngroups: int = 0
    loops: int = 0
    pattern: str = ""

    def emit(self, op, a=0, b=0, c=0) -> int:
        if len(self.code) // 4 >= MAX_PROG:
            raise Unsupported("regex program too large")
        self.code += [op, a, b, c]
        return len(self.code) // 4 - 1

    def patch(self, at, a=None, b=None):
        if a is not None:
            self.code[4 * at + 1] = a
        if b is not None:
            self.code[4 * at + 2] = b

    def pc(self) -> int:
        return len(self.code) // 4

    def bitmap(self, members) -> int:
        words = [0] * 8
        for m in members:
            words[m >> 5] |= 1 << (m & 31)
        words = [w - (1 << 32) if w >= 1 << 31 else w for w in words]      # int32 storage
        self.sets += words
        return len(self.sets) // 8 - 1


def _nullable(node) -> bool:
    k = node[0]
    if k == "seq":
        return all(_nullable(x) for x in node[1])
    if k == "alt":
        return any(_nullable(x) for x in node[1])
    if k == "group":
        return _nullable(node[2])
    if k == "rep":
        return node[2] == 0 or _nullable(node[1])
    if k == "bytes":
        return len(node[1]) == 0
    return k in ("bos", "eos")


def _gen(prog: Program, node) -> None:
    k = node[0]
    if k == "seq":
        for item in node[1]:
            _gen(prog, item)
    elif k == "alt":
        jumps = []
        branches = node[1]
        for i, br in enumerate(branches):
            if i < len(branches) - 1:
                sp = prog.emit(SPLIT)
                prog.patch(sp, a=prog.pc())
                _gen(prog, br)
                jumps.append(prog.emit(JMP))
                prog.patch(sp, b=prog.pc())
            else:
                _gen(prog, br)
        for j in jumps:
            prog.patch(j, a=prog.pc())
    elif k == "group":
        idx = node[1]
        if idx <= MAX_GROUPS:
            prog.emit(SAVE, 2 * idx)
            _gen(prog, node[2])
            prog.emit(SAVE, 2 * idx + 1)
        else:
            _gen(prog, node[2])
    elif k == "bytes":
        for b in node[1]:
            prog.emit(CHAR, b)
    elif k == "set":
        prog.emit(SET, prog.bitmap(node[1]))
    elif k == "notset":
        prog.emit(NOTSET, prog.bitmap(node[1]))
    elif k == "any":
        prog.emit(ANY)
    elif k == "bos":
        prog.emit(BOL)
    elif k == "eos":
        prog.emit(EOL)
    elif k == "rep":
        _, sub, lo, hi, lazy = node
        for _ in range(lo):
            _gen(prog, sub)
        if hi is None:
            top = prog.emit(SPLIT)
            body = prog.pc()
            if _nullable(sub):
                slot = LOOP_SLOTS[0] + prog.loops
                if slot >= LOOP_SLOTS[1]:
                    raise Unsupported("too many empty-matching loops")
                prog.loops += 1
                prog.emit(SAVE, slot)
                _gen(prog, sub)
                lp = prog.emit(LOOP, slot, top)
                out = prog.pc()
                prog.patch(lp, b=top)
                prog.code[4 * lp + 3] = out
            else:
                _gen(prog, sub)
                prog.emit(JMP, top)
                out = prog.pc()
            prog.patch(top, *((out, body) if lazy else (body, out)))
        else:
            splits = []
            for _ in range(hi - lo):
                sp = prog.emit(SPLIT)
                splits.append((sp, prog.pc()))
                _gen(prog, sub)
            out = prog.pc()
            for sp, body in splits:
                prog.patch(sp, *((out, body) if lazy else (body, out)))
    else:
        raise Unsupported(k)


_CACHE: Dict[str, Program] = {}


def compile_vm(pattern: str) -> Program:
    hit = _CACHE.get(pattern)
    if hit is not None:
        return hit
    parser = _Parser(pattern)
    ast = parser.parse()
    prog = Program(ngroups=parser.groups, pattern=pattern)
    prog.emit(SAVE, 0)
    _gen(prog, ast)
    prog.emit(SAVE, 1)
    prog.emit(MATCH)
    if not prog.sets:
        prog.bitmap([])
    if len(_CACHE) > 256:
        _CACHE.clear()
    _CACHE[pattern] = prog
    return prog


def replacement_tokens(rep: str, ngroups: int) -> List[int]:
    """Java Matcher.appendReplacement template → tokens: a byte (0..255) or -1-k for group k ($k; \\x is x)."""
    out: List[int] = []
    i = 0
    while i < len(rep):
        c = rep[i]
        if c == "\\":
            if i + 1 >= len(rep):
                raise Unsupported("trailing backslash in replacement")
            out += list(rep[i + 1].encode("utf-8"))
            i += 2
        elif c == "$":
            j = i + 1
            if j >= len(rep) or not rep[j].isdigit():
                raise Unsupported("bad group reference in replacement")
            g = int(rep[j])
            j += 1
            # Java takes more digits while the number stays a valid group
            while j < len(rep) and rep[j].isdigit() and g * 10 + int(rep[j]) <= ngroups:
                g = g * 10 + int(rep[j])
                j += 1
            if g > ngroups or g > MAX_GROUPS:
                raise Unsupported("group reference out of range")
            out.append(-1 - g)
            i = j
        else:
            out += list(c.encode("utf-8"))
            i += 1
    return out
