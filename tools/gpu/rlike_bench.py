"""Device RLIKE / LIKE throughput on 2 M generated strings (≈40 B): DFA kernel vs the host regex it replaces."""
import random
import re
import time

import torch

from dxa.engine.column import strings_from_pylist
from dxa.ops import regex_dfa, strings as S

rnd = random.Random(3)
words = ["device", "temp", "home", "garage", "door", "open", "closed", "alert", "12", "7", "日本", "é"]
vals = [" ".join(rnd.choice(words) for _ in range(rnd.randint(3, 8))) for _ in range(2_000_000)]
col = strings_from_pylist(vals, "cuda")
torch.cuda.synchronize()
for pat in ["door (open|closed)", "^home.*alert$", "\\d{2} temp", "[^a-z ]", "(device|home) \\w+ (12|7)"]:
    dfa = regex_dfa.compile_rlike(pat)
    S.rlike(col, dfa)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(10):
        m = S.rlike(col, dfa)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / 10
    rx = re.compile(regex_dfa.java_to_python(pat), re.ASCII)
    t = time.perf_counter()
    ref = [rx.search(v) is not None for v in vals[:200000]]
    hdt = (time.perf_counter() - t) * 10
    assert m[:200000].cpu().tolist() == ref, pat
    print(f"{pat!r:34} states={dfa.n_states:4} classes={dfa.n_classes:3}  device {dt * 1e3:7.3f} ms "
          f"({len(vals) / dt / 1e9:6.2f} G rows/s)  host re {hdt * 1e3:8.1f} ms  hits={int(m.sum())}")

# regexp_extract / regexp_replace through the backtracking program (regex_vm.py)
from dxa.ops import regex_vm  # noqa: E402

for pat, g, rep in [("(door|home) (\\w+)", 2, "<$1>"), ("(\\d+) temp", 1, "#"), ("a.*?e", 0, "")]:
    prog = regex_vm.compile_vm(pat)
    for what in ("extract", "replace"):
        fn = (lambda: S.regex_extract(col, prog, g)) if what == "extract" else \
            (lambda: S.regex_replace(col, prog, regex_vm.replacement_tokens(rep, prog.ngroups)))
        out, bad = fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(5):
            out, bad = fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / 5
        print(f"regexp_{what} {pat!r:26} device {dt * 1e3:7.2f} ms ({len(vals) / dt / 1e9:5.2f} G rows/s) "
              f"fallback rows {int(bad.sum())}")

# md5 / sha1 / sha256 / sha224 / crc32 (one lane per row), checked against hashlib / zlib on a sample
import hashlib  # noqa: E402
import zlib  # noqa: E402


for kind, name in [(0, "md5"), (1, "sha1"), (2, "sha256"), (3, "sha224"), (4, "crc32")]:
    fn = (lambda: S.crc32(col)) if kind == 4 else (lambda: S.digest(col, kind))
    out = fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(10):
        out = fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / 10
    sample = vals[:2000]
    if kind == 4:
        assert out[:2000].cpu().tolist() == [zlib.crc32(v.encode()) for v in sample], name
    else:
        h = getattr(hashlib, name)
        got = out.to_pylist()[:2000]
        assert got == [h(v.encode()).hexdigest() for v in sample], name
    print(f"{name:8} device {dt * 1e3:7.3f} ms ({len(vals) / dt / 1e9:5.2f} G rows/s, "
          f"{int(col.lens.sum()) / dt / 1e9:6.1f} GB/s of input)")
