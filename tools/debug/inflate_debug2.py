"""The bench's Kafka path with gzip batches (16 partitions through plan_many, 4 decode launches): which batches fail
and what their blocks' statuses are."""
import sys, os, collections
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
from dxa.io import kafka as K
from dxa.io import kafka_device as KD
from dxa.models import iot
from dxa.simulate.datagen import generate

dev = torch.device("cuda", 0)
E = int(sys.argv[1]) if len(sys.argv) > 1 else 2000000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
buf, offs = generate(iot.program(), E, dev, seed=1, row0=0, base_ms=1_700_000_000_000)
hb, ho = buf.cpu().numpy(), offs.cpu().numpy()
parts = 16
cuts = np.linspace(0, E, parts + 1).astype(np.int64)
sets = [K.encode_stream(hb, ho[cuts[q]:cuts[q + 1] + 1], 26, compression="gzip", threads=16) for q in range(parts)]
total = sum(x.size for x in sets)
staging = torch.empty(total + 64, dtype=torch.uint8).pin_memory()
sn = staging.numpy()
bounds, pos = [], 0
for x in sets:
    sn[pos:pos + x.size] = x
    bounds.append((pos, pos + x.size))
    pos += x.size
for chunks in (1, 4):
    for r in range(reps):
        plan = KD.plan_many(sn, bounds, [0] * parts, threads=16)
        dec = KD.DeviceRecordDecoder(dev, chunks=chunks)
        raw, ev = dec.decode(staging, plan)
        torch.cuda.synchronize()
        st = dec.checks[-1]
        try:
            dec.check()
            ok = True
        except KD.DecodeError as e:
            ok = str(e)
        # compare values with host
        s, e_ = raw.offs[:-1].cpu().numpy(), raw.ends.cpu().numpy()
        b = raw.buf.cpu().numpy()
        nbad = 0
        for i in range(0, raw.n, 997):
            if b[s[i]:e_[i]].tobytes() != hb[ho[i]:ho[i + 1]].tobytes():
                nbad += 1
        print("chunks", chunks, "rep", r, "check", ok, "sampled value mismatches", nbad, "of", len(range(0, raw.n, 997)))
