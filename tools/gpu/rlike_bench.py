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
