"""Stage-1 structural index prototype (csrc/json_index.hip) against a byte-at-a-time host scan: escaped quotes,
runs of backslashes across 64-byte chunk and 4-KiB step boundaries, structural characters inside strings."""
import json
import random

import pytest
import torch

pytestmark = pytest.mark.gpu


def _records(n, seed):
    rnd = random.Random(seed)
    out = []
    for i in range(n):
        s = "".join(rnd.choice(['a', '"', '\\', '{', '}', ',', ':', '[', ']', ' ', 'é']) for _ in range(rnd.randint(0, 90)))
        rec = {"id": i, "s": s, "arr": [1, {"k": s[:5]}, "x,y"], "bs": "\\" * rnd.randint(0, 130)}
        out.append((json.dumps(rec, ensure_ascii=rnd.random() < 0.5) + "\n").encode())
    return out


@pytest.mark.parametrize("per_seg", [1, 7, 64])
def test_structural_counts_match_host(gpu, per_seg):
    from dxa.ops.json_index import host_counts, structural_index
    recs = _records(3000, per_seg)
    data = b"".join(recs)
    offs = [0]
    for r in recs:
        offs.append(offs[-1] + len(r))
    buf = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(gpu)
    o = torch.tensor(offs, dtype=torch.int64, device=gpu)
    counts, words = structural_index(buf, o, per_seg, bits=True)
    assert counts.cpu().tolist() == host_counts(data, offs, per_seg)
    assert int(sum(bin(w & (2**64 - 1)).count("1") for w in words.cpu().tolist())) == sum(counts.cpu().tolist())
