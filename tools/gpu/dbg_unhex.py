import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from dxa.engine.column import strings_from_pylist
from dxa.ops import strfuncs as SF
from dxa.ops import native as N
dev = torch.device("cuda")
vals = ["caaDAaaCAEA", "414243", "c", "0c", "caa"]
col = strings_from_pylist(vals, dev)
from dxa.engine.sqlfuncs import _dev_str
col = _dev_str(col)
n = col.length
lens = torch.empty(n, dtype=torch.int64, device=dev)
ok = torch.empty(n, dtype=torch.uint8, device=dev)
bad = torch.zeros(1, dtype=torch.int32, device=dev)
args = (N.ptr(col.arena), N.ptr(col.starts), N.ptr(col.lens), N.ptr(N.u8(col.valid)), n, 0)
N.call("dxa_str_decode", *args, None, None, N.ptr(lens), N.ptr(ok), N.ptr(bad), SF._st(col))
print("lens", lens.tolist(), "ok", ok.tolist())
from dxa.ops.strings import _offsets, _alloc_arena
off, total = _offsets(lens)
dst = _alloc_arena(total, dev)
N.call("dxa_str_decode", *args, N.ptr(off), N.ptr(dst), N.ptr(lens), N.ptr(ok), N.ptr(bad), SF._st(col))
torch.cuda.synchronize()
print("raw", dst[:total].cpu().tolist(), "off", off.tolist())
out = SF.decode(col, 0)
print("clean", [out.arena[s:s + l].cpu().tolist() for s, l in zip(out.starts.tolist(), out.lens.tolist())])
print(out.to_pylist())
# the test's data: the SQL path on 20 000 rows, GPU vs CPU, and the kernel path directly
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
from test_strfuncs import _rand_rows, _q, S
from dxa.engine.column import Table
rows = _rand_rows(1_000_000)[:20000]
g = _q("SELECT unhex(t) AS r FROM T", rows, dev)
c = _q("SELECT unhex(t) AS r FROM T", rows)
bad = [i for i in range(len(rows)) if g[i] != c[i]]
print("mismatches", len(bad), bad[:10])
for i in bad[:3]:
    print(i, repr(rows[i]["t"]), repr(g[i]), repr(c[i]))
t = Table.from_pylist(rows, S, dev)
col = _dev_str(t.columns[1])
d = SF.decode(col, 0).to_pylist()
print("direct mismatches", sum(1 for i in range(len(rows)) if d[i] != c[i]["r"]))
