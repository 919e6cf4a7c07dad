import os, sys
R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "tests"))
import torch
from dxa.ops import strfuncs as SF
from dxa.ops import native as N
from dxa.ops.strings import _offsets, _alloc_arena
from dxa.engine.column import Table
from dxa.engine.sqlfuncs import _dev_str
from test_strfuncs import _rand_rows, S
dev = torch.device("cuda")
rows = _rand_rows(1_000_000)[:20000]
t = Table.from_pylist(rows, S, dev)
col = _dev_str(t.columns[1])
print("starts", col.starts.dtype, col.lens.dtype, col.arena.dtype, col.arena.numel(), col.valid)
n = col.length
lens = torch.empty(n, dtype=torch.int64, device=dev)
ok = torch.empty(n, dtype=torch.uint8, device=dev)
bad = torch.zeros(1, dtype=torch.int32, device=dev)
args = (N.ptr(col.arena), N.ptr(col.starts), N.ptr(col.lens), N.ptr(N.u8(col.valid)), n, 0)
N.call("dxa_str_decode", *args, None, None, N.ptr(lens), N.ptr(ok), N.ptr(bad), SF._st(col))
off, total = _offsets(lens)
dst = _alloc_arena(total, dev)
N.call("dxa_str_decode", *args, N.ptr(off), N.ptr(dst), N.ptr(lens), N.ptr(ok), N.ptr(bad), SF._st(col))
torch.cuda.synchronize()
L, O, K, D = lens.tolist(), off.tolist(), ok.tolist(), dst.cpu().tolist()
nb = 0
for i in (41, 52, 103, 124):
    s = rows[i]["t"]
    h = ("0" + s) if len(s) % 2 else s
    try:
        want = list(bytes.fromhex(h))
    except ValueError:
        want = None
    print(i, repr(s), "len", L[i], "ok", K[i], "got", D[O[i]:O[i] + L[i]], "want", want)
for i in range(n):
    s = rows[i]["t"]
    h = ("0" + s) if len(s) % 2 else s
    try:
        want = list(bytes.fromhex(h))
    except ValueError:
        continue
    if D[O[i]:O[i] + L[i]] != want:
        nb += 1
print("raw mismatches", nb)
a = col.arena.cpu().tolist(); st = col.starts.tolist(); ln = col.lens.tolist()
print("arena bytes of row 52", a[st[52]:st[52] + ln[52]], "neighbour", a[st[52] - 4:st[52] + 4])
