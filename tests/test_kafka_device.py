"""GPU Kafka record-batch ingest (dxa.io.kafka_device): host plan of batch / LZ4-frame headers, device LZ4 decode
into capacity slots, device record framing.  CPU tests check the plan against the host decoder through a CPU
reference of the device steps; the GPU test runs the kernels."""
import json
import random

import numpy as np
import pytest
import torch

from dxa.io import kafka as K
from dxa.io import kafka_device as KD


def _values(n, seed=0):
    rnd = random.Random(seed)
    return [json.dumps({"id": i, "t": round(rnd.uniform(-40, 40), rnd.randint(0, 12)),
                        "s": rnd.choice(["DoorLock", "Heating", "x" * rnd.randint(0, 300)])}).encode()
            for i in range(n)]


def _record_set(vals, per_batch, compression="lz4", level=9, block=16384, base=0):
    """Concatenated v2 batches as a broker returns them (base offsets assigned like a log)."""
    out = bytearray()
    off = base
    for i in range(0, len(vals), per_batch):
        chunk = vals[i:i + per_batch]
        b = bytearray(K.encode_batch(chunk, 1_700_000_000_000, compression, level=level, block_size=block))
        b[0:8] = off.to_bytes(8, "big")               # broker-assigned base offset
        out += b
        off += len(chunk)
    return bytes(out)


@pytest.mark.parametrize("compression,level,block", [("lz4", 9, 16384), ("lz4", 1, 65536), ("lz4", 9, 4096),
                                                     ("none", 0, 0), ("gzip", 6, 0)])
def test_plan_matches_host_decoder(compression, level, block):
    vals = _values(500, seed=1)
    rs = _record_set(vals, 37, compression, level, block or 65536)
    for min_off in (0, 5, 37, 100):
        want_v, want_o, want_rec, want_next = K.decode_records(rs, min_off, pad=0)
        plan = KD.plan_fetch(rs, min_off)
        assert plan.nrec == len(want_rec) and plan.next_offset == want_next
        buf, starts, ends = KD.decode_on_host_like(np.frombuffer(rs, np.uint8), plan)
        got = [buf[s:e].tobytes() for s, e in zip(starts, ends)]
        assert got == vals[min_off:]


def test_merge_and_trim():
    vals = _values(300, seed=2)
    a = _record_set(vals[:150], 40, base=0)
    b = _record_set(vals[150:], 40, base=150)
    staging = np.frombuffer(a + b, np.uint8)
    pa, pb = KD.plan_fetch(a, 10), KD.plan_fetch(b, 150)
    plan = KD.merge([(pa, 0), (pb, len(a))])
    assert plan.nrec == 290
    buf, s, e = KD.decode_on_host_like(staging, plan)
    assert [buf[x:y].tobytes() for x, y in zip(s, e)] == vals[10:]
    t = KD.trim(plan, 100)
    assert t.nrec == 100 and t.next_offset == 110
    buf, s, e = KD.decode_on_host_like(staging, t)
    assert [buf[x:y].tobytes() for x, y in zip(s, e)] == vals[10:110]


def test_unsupported_codec_falls_back():
    """snappy / zstd batches (codecs 2 / 4) are decoded on the host: the planner refuses them."""
    rs = bytearray(_record_set(_values(20), 20, "none"))
    attrs = 12 + 9                                    # baseOffset, batchLength, leaderEpoch, magic, crc
    rs[attrs + 1] = (rs[attrs + 1] & ~7) | 4          # compression codec = zstd
    rs[12 + 5:12 + 9] = K.crc32c(bytes(rs[attrs:])).to_bytes(4, "big")
    with pytest.raises(KD.Unsupported):
        KD.plan_fetch(bytes(rs), 0)


def test_gzip_plan_strips_header_and_reads_isize():
    """gzip batches become one kind-2 block: the deflate data between the member header and the trailer, with the
    trailer's ISIZE as the exact output size (inflated on the device by inflate.hip)."""
    import zlib
    vals = _values(300, seed=21)
    rs = _record_set(vals, 70, "gzip") + _record_set(vals[:5], 5, "lz4", base=300)
    plan = KD.plan_fetch(rs, 0)
    kinds = plan.k_stored[:plan.nblk].tolist()
    assert kinds.count(2) == 5 and 0 in kinds
    for b in range(plan.nblk):
        if kinds[b] == 2:
            lo, n = int(plan.k_comp_off[b]), int(plan.k_comp_len[b])
            raw = zlib.decompressobj(-15).decompress(rs[lo:lo + n])
            assert len(raw) == int(plan.k_cap[b])
    buf, s, e = KD.decode_on_host_like(np.frombuffer(rs, np.uint8), plan)
    assert [buf[x:y].tobytes() for x, y in zip(s, e)] == vals + vals[:5]


@pytest.mark.gpu
def test_device_decode_matches_host(gpu):
    vals = _values(3000, seed=3)
    rs = _record_set(vals, 53, "lz4", 9, 16384) + _record_set(vals[:10], 10, "none", base=3000)
    plan = KD.trim(KD.plan_fetch(rs, 7), 2990)
    staging = torch.zeros(len(rs) + 64, dtype=torch.uint8).pin_memory()
    staging[:len(rs)] = torch.frombuffer(bytearray(rs), dtype=torch.uint8)
    dec = KD.DeviceRecordDecoder(gpu, chunks=3)
    raw, ev = dec.decode(staging, plan)
    torch.cuda.current_stream(gpu).wait_event(ev)
    dec.check()
    buf = raw.buf.cpu().numpy()
    s, e = raw.offs[:-1].cpu().tolist(), raw.ends.cpu().tolist()
    want = (vals + vals[:10])[7:7 + 2990]
    assert raw.n == 2990 and [buf[x:y].tobytes() for x, y in zip(s, e)] == want
    # the parser reads the values in place
    from dxa.engine.types import StructField, StructType
    from dxa.ops.jsonparse import ParsePlan, parse
    pl = ParsePlan(StructType((StructField("id", "long"), StructField("s", "string"))))
    col, ok = parse(raw.buf, raw.offs, pl, raw.ends)
    assert bool(ok.all()) and col.children[0].data.cpu().tolist() == [json.loads(v)["id"] for v in want]


@pytest.mark.gpu
def test_device_decode_launch_sizing(gpu):
    """Java-producer-sized batches (90 records, one 64 KiB-frame LZ4 block each): the decode is split into at most
    nblocks / min_blocks_per_chunk launches; one launch and four launches give the host decoder's records."""
    vals = _values(6000, seed=13)
    rs = _record_set(vals, 90, "lz4", 9, 65536)
    plan = KD.plan_fetch(rs, 0)
    staging = torch.zeros(len(rs) + 64, dtype=torch.uint8).pin_memory()
    staging[:len(rs)] = torch.frombuffer(bytearray(rs), dtype=torch.uint8)
    dec = KD.DeviceRecordDecoder(gpu, chunks=4)
    assert dec.min_blocks_per_chunk >= 64
    for mb in (1, 10 ** 9):                       # 4 launches / 1 launch
        dec.min_blocks_per_chunk = mb
        raw, ev = dec.decode(staging, KD.plan_fetch(rs, 0))
        torch.cuda.current_stream(gpu).wait_event(ev)
        dec.check()
        buf = raw.buf.cpu().numpy()
        s, e = raw.offs[:-1].cpu().tolist(), raw.ends.cpu().tolist()
        assert raw.n == plan.nrec == 6000 and [buf[x:y].tobytes() for x, y in zip(s, e)] == vals


@pytest.mark.gpu
@pytest.mark.parametrize("level", [1, 6, 9])
def test_device_inflate_matches_host(gpu, level):
    """gzip record batches inflated on the GPU (inflate.hip) next to LZ4 and uncompressed batches in one fetch: fixed
    and dynamic Huffman blocks, stored blocks (incompressible values), long matches and RLE runs."""
    import zlib
    rnd = random.Random(level)
    vals = _values(2500, seed=30 + level)
    vals += [bytes(rnd.getrandbits(8) for _ in range(rnd.choice([1, 100, 3000]))) for _ in range(40)]   # stored
    vals += [b"a" * rnd.choice([3, 258, 1000, 40000]) for _ in range(20)]                                # RLE
    vals += [b'{"x":1}'] * 50                                                                           # fixed codes
    enc = lambda vs, per, codec, base: _record_set(vs, per, codec, level, 16384, base)               # noqa: E731
    rs = (enc(vals[:1500], 60, "gzip", 0) + enc(vals[1500:2000], 40, "lz4", 1500) +
          enc(vals[2000:2100], 25, "none", 2000) + enc(vals[2100:], 1, "gzip", 2100))
    plan = KD.plan_fetch(rs, 0)
    assert (plan.k_stored[:plan.nblk] == 2).sum() > 30
    staging = torch.zeros(len(rs) + 64, dtype=torch.uint8).pin_memory()
    staging[:len(rs)] = torch.frombuffer(bytearray(rs), dtype=torch.uint8)
    dec = KD.DeviceRecordDecoder(gpu, chunks=2)
    raw, ev = dec.decode(staging, plan)
    torch.cuda.current_stream(gpu).wait_event(ev)
    dec.check()
    buf = raw.buf.cpu().numpy()
    s, e = raw.offs[:-1].cpu().tolist(), raw.ends.cpu().tolist()
    assert raw.n == len(vals) and [buf[x:y].tobytes() for x, y in zip(s, e)] == vals
    # a corrupted deflate stream is reported (nonzero status), never read or written out of range
    bad = bytearray(rs)
    b0 = int(np.nonzero(plan.k_stored[:plan.nblk] == 2)[0][0])
    lo = int(plan.k_comp_off[b0])
    for k in range(lo + 5, lo + 40):
        bad[k] ^= 0x5a
    plan2 = KD.plan_fetch(bytes(bad), 0, verify_crc=False)
    staging[:len(bad)] = torch.frombuffer(bad, dtype=torch.uint8)
    raw2, ev2 = dec.decode(staging, plan2)
    torch.cuda.current_stream(gpu).wait_event(ev2)
    with pytest.raises(KD.DecodeError):
        dec.check()


def test_plan_many_matches_merged_plans():
    vals = _values(400, seed=5)
    sets = [_record_set(vals[:130], 17), _record_set(vals[130:260], 29, "none"), _record_set(vals[260:], 41)]
    data, bounds = b"", []
    for x in sets:
        bounds.append((len(data), len(data) + len(x)))
        data += x
    a = np.frombuffer(data, np.uint8)
    many = KD.plan_many(a, bounds, [3, 0, 0], threads=3)
    merged = KD.merge([(KD.plan_fetch(a[lo:hi], m), lo) for (lo, hi), m in zip(bounds, [3, 0, 0])])
    for name, _dt, _k in KD._ARRAYS:
        assert np.array_equal(getattr(many, name), getattr(merged, name)), name
    buf, s, e = KD.decode_on_host_like(a, many)
    assert [buf[x:y].tobytes() for x, y in zip(s, e)] == vals[3:130] + vals[130:]


def test_plan_carries_crc_ranges_and_segmented_crc_matches():
    """The plan records each batch's CRC-covered range and stored CRC; the device's segmented combine
    (mirrored on the CPU) reproduces the serial CRC-32C for every length, and a flipped byte fails the check."""
    import random as R
    for n in list(range(4, 24)) + [127, 511, 512, 513, 1030, 4095, 16391]:
        b = bytes(R.Random(n).getrandbits(8) for _ in range(n))
        for al in (0, 3, 7):
            assert KD.crc32c_segmented(b, al) == K.crc32c(b), (n, al)
    vals = _values(200, seed=9)
    rs = _record_set(vals, 37, "lz4") + _record_set(vals[:20], 20, "none", base=200)
    plan = KD.plan_fetch(rs, 0)
    a = np.frombuffer(rs, np.uint8)
    for i in range(plan.nbat):
        lo, ln = int(plan.b_crc_off[i]), int(plan.b_crc_len[i])
        assert K.crc32c(rs[lo:lo + ln]) == int(plan.b_crc[i]) & 0xFFFFFFFF
    buf, s, e = KD.decode_on_host_like(a, plan, verify_crc=True)
    assert [buf[x:y].tobytes() for x, y in zip(s, e)] == vals + vals[:20]
    bad = bytearray(rs)
    bad[int(plan.b_crc_off[-1]) + 200] ^= 0x01            # inside the stored (codec none) batch's records
    with pytest.raises(KD.DecodeError):
        KD.decode_on_host_like(np.frombuffer(bytes(bad), np.uint8), KD.plan_fetch(bytes(bad), 0, verify_crc=False),
                               verify_crc=True)
    with pytest.raises(KD.Unsupported):
        KD.plan_fetch(bytes(bad), 0, verify_crc=True)     # the host check catches it too
    # offsets survive plan_many's set shifting
    many = KD.plan_many(np.frombuffer(rs + rs, np.uint8), [(0, len(rs)), (len(rs), 2 * len(rs))], [0, 0], threads=2)
    assert np.array_equal(many.b_crc_off[plan.nbat:], plan.b_crc_off + len(rs))


@pytest.mark.gpu
def test_device_crc_flags_corrupt_batch(gpu):
    vals = _values(400, seed=11)
    rs = bytearray(_record_set(vals, 50, "lz4") + _record_set(vals[:30], 30, "none", base=400))
    plan = KD.plan_fetch(bytes(rs), 0, verify_crc=False)
    staging = torch.zeros(len(rs) + 64, dtype=torch.uint8).pin_memory()
    staging[:len(rs)] = torch.frombuffer(bytearray(rs), dtype=torch.uint8)
    dec = KD.DeviceRecordDecoder(gpu, verify_crc=True)
    raw, ev = dec.decode(staging, plan)
    torch.cuda.current_stream(gpu).wait_event(ev)
    assert raw.status.failed() == 0
    dec.check()
    rs[int(plan.b_crc_off[-1]) + 100] ^= 0x20                # corrupt a value byte of the stored batch
    staging[:len(rs)] = torch.frombuffer(bytearray(rs), dtype=torch.uint8)
    raw, ev = dec.decode(staging, KD.plan_fetch(bytes(rs), 0, verify_crc=False))
    torch.cuda.current_stream(gpu).wait_event(ev)
    assert raw.status.failed() == 1                          # framing is intact: only the CRC catches it
    with pytest.raises(KD.DecodeError):
        dec.check()
