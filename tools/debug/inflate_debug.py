"""Device inflate of bench-shaped gzip Kafka batches vs zlib: per-block status histogram and the first failures."""
import sys, os, collections
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
from dxa.io import kafka as K
from dxa.io import kafka_device as KD
from dxa.models import iot
from dxa.simulate.datagen import generate

dev = torch.device("cuda", 0)
E = int(sys.argv[1]) if len(sys.argv) > 1 else 200000
chunks = int(sys.argv[2]) if len(sys.argv) > 2 else 4
buf, offs = generate(iot.program(), E, dev, seed=1, row0=0, base_ms=1_700_000_000_000)
hb, ho = buf.cpu().numpy(), offs.cpu().numpy()
rs = K.encode_stream(hb, ho, 26, compression="gzip", threads=16)
plan = KD.plan_fetch(rs, 0)
staging = torch.zeros(rs.size + 64, dtype=torch.uint8).pin_memory()
staging[:rs.size] = torch.from_numpy(rs)
dec = KD.DeviceRecordDecoder(dev, chunks=chunks, track=False)
dec.min_blocks_per_chunk = 1
raw, ev = dec.decode(staging, plan)
torch.cuda.synchronize()
# re-run the block decode alone to read per-block statuses
from dxa.ops import native as N
nb = plan.nblk
d = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
ddata = torch.from_numpy(rs).to(dev)
ddata = torch.cat([ddata, torch.zeros(64, dtype=torch.uint8, device=dev)])
out = torch.zeros(plan.out_bytes + 64, dtype=torch.uint8, device=dev)
prod = torch.zeros(nb, dtype=torch.int64, device=dev)
st = torch.full((nb,), -1, dtype=torch.int32, device=dev)
co, cl, sd, oo, cap = (d(plan.k_comp_off, 0), d(plan.k_comp_len, 0), d(plan.k_stored, 0), d(plan.k_out_off, 0),
                       d(plan.k_cap, 0))
N.call("dxa_inflate_into", N.ptr(ddata), N.ptr(co), N.ptr(cl), N.ptr(sd), N.ptr(oo), N.ptr(cap), nb, N.ptr(out),
       N.ptr(prod), N.ptr(st), N.stream_handle(dev))
torch.cuda.synchronize()
stl = st.cpu().numpy()
print("blocks", nb, "status histogram", collections.Counter(stl.tolist()))
import zlib
bad = np.nonzero(stl != 0)[0][:5]
o = out.cpu().numpy()
for b in bad:
    lo, n = int(plan.k_comp_off[b]), int(plan.k_comp_len[b])
    ref = zlib.decompressobj(-15).decompress(rs[lo:lo + n].tobytes())
    p = int(prod[b]); base = int(plan.k_out_off[b])
    got = o[base:base + p].tobytes()
    first_diff = next((i for i in range(min(len(ref), len(got))) if ref[i] != got[i]), None)
    # block types in the stream
    print("block", b, "status", stl[b], "cap", int(plan.k_cap[b]), "produced", p, "ref", len(ref), "first diff", first_diff,
          "comp_len", n, "off%4", lo % 4, "hdr0", rs[lo] & 7)
