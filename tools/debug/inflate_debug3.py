"""Repeat one-launch device inflate of 77 K gzip members several times: which members fail, with what status, and
is it the same member each time (deterministic) or not (a race)."""
import sys, os, collections, zlib
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
from dxa.io import kafka as K
from dxa.io import kafka_device as KD
from dxa.models import iot
from dxa.simulate.datagen import generate
from dxa.ops import native as N

dev = torch.device("cuda", 0)
E = int(sys.argv[1]) if len(sys.argv) > 1 else 2000000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
buf, offs = generate(iot.program(), E, dev, seed=1, row0=0, base_ms=1_700_000_000_000)
hb, ho = buf.cpu().numpy(), offs.cpu().numpy()
rs = K.encode_stream(hb, ho, 26, compression="gzip", threads=16)
plan = KD.plan_fetch(rs, 0)
nb = plan.nblk
d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
ddata = torch.cat([torch.from_numpy(rs).to(dev), torch.zeros(64, dtype=torch.uint8, device=dev)])
co, cl, sd, oo, cap = d(plan.k_comp_off), d(plan.k_comp_len), d(plan.k_stored), d(plan.k_out_off), d(plan.k_cap)
capn = plan.k_cap[:nb]
fails = []
for r in range(reps):
    out = torch.zeros(plan.out_bytes + 64, dtype=torch.uint8, device=dev)
    prod = torch.zeros(nb, dtype=torch.int64, device=dev)
    st = torch.full((nb,), -1, dtype=torch.int32, device=dev)
    N.call("dxa_inflate_into", N.ptr(ddata), N.ptr(co), N.ptr(cl), N.ptr(sd), N.ptr(oo), N.ptr(cap), nb, N.ptr(out),
           N.ptr(prod), N.ptr(st), N.stream_handle(dev))
    torch.cuda.synchronize()
    stl = st.cpu().numpy()
    bad = np.nonzero(stl != 0)[0]
    # content check of a sample of OK members
    o = out.cpu().numpy()
    wrong = []
    for b in list(range(0, nb, 500)) + bad[:3].tolist():
        lo, n = int(plan.k_comp_off[b]), int(plan.k_comp_len[b])
        ref = zlib.decompressobj(-15).decompress(rs[lo:lo + n].tobytes())
        base = int(plan.k_out_off[b])
        got = o[base:base + len(ref)].tobytes()
        if got != ref:
            fd = next(i for i in range(len(ref)) if ref[i] != got[i])
            wrong.append((b, int(stl[b]), int(prod[b]), len(ref), fd))
    print("rep", r, "failed", len(bad), collections.Counter(stl[bad].tolist()), "first", bad[:8].tolist(), "wrong content", wrong[:5])
    fails.append(set(bad.tolist()))
print("members failing in more than one rep", len(set.intersection(*fails)) if fails else 0)
