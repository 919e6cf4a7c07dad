"""Kafka snappy (codec 2) and zstd (codec 4) record batches: host codecs (host_snappy.cpp, host_zstd.cpp — written
from the snappy format description and RFC 8878) and the GPU decoders (snappy.hip, zstd.hip).

The reference's Kafka source uses kafka-clients 2.4.1 (DataProcessing/datax-host/pom.xml:164-167), which decodes
both codecs (KafkaStreamingFactory.scala:70-74).  Oracles: the system libzstd compresses the frames a zstd-jni
producer would write (no content size, no checksum) and our decoders must return the input; frames and blocks
hand-assembled here from the format descriptions check the decoders independently of any encoder; pyarrow's
bundled snappy / zstd / lz4 codecs (independent implementations) are a second oracle on the host and the GPU; the GPU
decode is compared with the host decode of the same fetch."""
import json
import random

import numpy as np
import pytest
import torch

from dxa.io import kafka as K
from dxa.io import kafka_device as KD


def _values(n, seed=0):
    rnd = random.Random(seed)
    return [json.dumps({"deviceId": rnd.randrange(1000), "t": round(rnd.uniform(-40, 40), rnd.randint(0, 12)),
                        "s": rnd.choice(["DoorLock", "Heating", "x" * rnd.randint(0, 300)]),
                        "ts": "2024-05-06T07:08:%02d.%03dZ" % (rnd.randrange(60), rnd.randrange(1000))}).encode()
            for i in range(n)]


def _record_set(vals, per_batch, compression, level=3, base=0):
    out = bytearray()
    off = base
    for i in range(0, len(vals), per_batch):
        chunk = vals[i:i + per_batch]
        b = bytearray(K.encode_batch(chunk, 1_700_000_000_000, compression, level=level))
        b[0:8] = off.to_bytes(8, "big")
        out += b
        off += len(chunk)
    return bytes(out)


def _samples():
    rnd = random.Random(7)
    text = b"\n".join(_values(400, seed=3))
    return [b"", b"a", b"abc" * 7, text[:16000], text, bytes(rnd.getrandbits(8) for _ in range(70000)),
            bytes(rnd.choice(b"ab") for _ in range(300000)), b"z" * 200000, text * 3]


# ---- host codecs ----------------------------------------------------------------------------------------------

@pytest.mark.parametrize("level", [1, 3, 9, 19, -3])
def test_zstd_host_decoder_matches_libzstd_frames(level):
    try:
        K.zstd_compress(b"x")
    except K.KafkaError:
        pytest.skip("libzstd not installed")
    for data in _samples():
        for cs, ck in ((False, False), (True, True)):
            frame = K.zstd_compress(data, level, content_size=cs, checksum=ck)
            assert K.zstd_decompress(frame) == data, (level, len(data), cs, ck)
    # concatenated frames with a skippable frame between them
    a, b = _samples()[3], _samples()[4]
    skip = (0x184D2A53).to_bytes(4, "little") + (5).to_bytes(4, "little") + b"12345"
    assert K.zstd_decompress(K.zstd_compress(a, level) + skip + K.zstd_compress(b, level)) == a + b


def test_snappy_host_round_trip_raw_and_xerial():
    for data in _samples():
        for xerial in (False, True):
            z = K.snappy_compress(data, xerial)
            assert K.snappy_decompress(z) == data
    assert K.snappy_compress(b"hello", True)[:8] == b"\x82SNAPPY\x00"


def _fse_table(norm, log):
    """RFC 8878 4.1.1 decoding table of a normalized distribution: [(symbol, nbits, baseline)] per state."""
    size = 1 << log
    sym = [0] * size
    high = size - 1
    for s, c in enumerate(norm):
        if c == -1:
            sym[high] = s
            high -= 1
    step, pos = (size >> 1) + (size >> 3) + 3, 0
    for s, c in enumerate(norm):
        for _ in range(max(c, 0)):
            sym[pos] = s
            pos = (pos + step) & (size - 1)
            while pos > high:
                pos = (pos + step) & (size - 1)
    nxt = [1 if c == -1 else c for c in norm]
    cells = []
    for c in range(size):
        s = sym[c]
        x = nxt[s]
        nxt[s] += 1
        nb = log - (x.bit_length() - 1)
        cells.append((s, nb, (x << nb) - size))
    return cells


LL_DEF = [4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2, 2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1,
          -1]
OF_DEF = [1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1]
ML_DEF = [1, 4, 3, 2, 2, 2, 2, 2, 2] + [1] * 37 + [-1] * 7


class _BackWriter:
    """Bits written low to high; the decoder reads them high to low (a zstd backward bitstream)."""

    def __init__(self):
        self.v, self.n = 0, 0

    def put(self, value, nbits):
        self.v |= (value & ((1 << nbits) - 1)) << self.n
        self.n += nbits

    def finish(self):
        self.put(1, 1)                                    # the end marker
        nbytes = (self.n + 7) // 8
        return self.v.to_bytes(nbytes, "little")


def _hand_frame():
    """A frame assembled from RFC 8878: a raw block, an RLE block, and a compressed block with raw literals and two
    sequences coded with the predefined tables (the second a repeat offset), plus trailing literals."""
    lits = b"wxyzQ!"
    lit_hdr = bytes([len(lits) << 3])                     # raw literals, 1-byte header (5-bit size)
    ll_t, of_t, ml_t = _fse_table(LL_DEF, 6), _fse_table(OF_DEF, 5), _fse_table(ML_DEF, 6)

    def state_of(table, symbol, then=None):
        """A state decoding ``symbol`` whose update can reach state ``then`` (for each symbol the cells' ranges
        [baseline, baseline + 2^nbits) tile the whole table, so exactly one such cell exists)."""
        return next(i for i, c in enumerate(table) if c[0] == symbol and
                    (then is None or c[2] <= then < c[2] + (1 << c[1])))
    # sequence 1: 4 literals, offset 4 (offset value 7: code 2, extra 3), match 8 (ML code 5)
    # sequence 2: 0 literals, offset value 1 — with ll == 0 that is Rep2, which after sequence 1's offset is 1
    #   (history [4, 1, 4]) → offset 1, match 3 (ML code 0): the last byte three more times
    seqs = [(4, 2, 3, 5), (0, 0, 0, 0)]                  # (ll code == ll, of code, of extra, ml code)
    st = [None] * len(seqs)
    for i in range(len(seqs) - 1, -1, -1):             # states chosen backward so every update reaches the next
        ll, oc, _, mc = seqs[i]
        nxt = st[i + 1] if i + 1 < len(seqs) else (None, None, None)
        st[i] = (state_of(ll_t, ll, nxt[0]), state_of(of_t, oc, nxt[1]), state_of(ml_t, mc, nxt[2]))
    w = _BackWriter()
    # written in reverse reading order: last sequence first
    for i in range(len(seqs) - 1, -1, -1):
        ll, oc, oe, mc = seqs[i]
        if i + 1 < len(seqs):                             # state updates after sequence i (read as LL, ML, OF)
            nl, no, nm = st[i + 1]
            cl, co, cm = ll_t[st[i][0]], of_t[st[i][1]], ml_t[st[i][2]]
            w.put(no - co[2], co[1])
            w.put(nm - cm[2], cm[1])
            w.put(nl - cl[2], cl[1])
        w.put(oe, oc)                                     # extra bits read as offset, match, literal length
    w.put(st[0][2], 6)                                    # initial states read LL, OF, ML
    w.put(st[0][1], 5)
    w.put(st[0][0], 6)
    bits = w.finish()
    seq_sec = bytes([len(seqs), 0]) + bits               # two sequences, all predefined modes
    block = lit_hdr + lits + seq_sec
    hdr = lambda last, typ, size: (last | (typ << 1) | (size << 3)).to_bytes(3, "little")   # noqa: E731
    content = b"abcd" + b"zzzzzz" + b"wxyz" + b"wxyzwxyz" + b"zzz" + b"Q!"
    frame = (0xFD2FB528).to_bytes(4, "little") + bytes([0x20, len(content)])          # single segment, 1-byte FCS
    frame += hdr(0, 0, 4) + b"abcd" + hdr(0, 1, 6) + b"z" + hdr(1, 2, len(block)) + block
    return frame, content


def test_zstd_hand_assembled_frame():
    frame, content = _hand_frame()
    assert K.zstd_decompress(frame) == content
    bad = bytearray(frame)
    bad[-1] ^= 0xFF                                        # the sequence bitstream's marker byte
    with pytest.raises(K.KafkaError):
        K.zstd_decompress(bytes(bad))


def test_snappy_hand_assembled_block():
    # preamble 27 | literal "abcd" | copy-1 len 4 off 4 | copy-2 len 8 off 8 | copy-4 len 5 off 2 | literal "!!" ...
    blk = bytes([27, 3 << 2]) + b"abcd"
    blk += bytes([1 | (0 << 2) | (0 << 5), 4])           # copy-1: len 4, offset 4
    blk += bytes([2 | (7 << 2), 8, 0])                   # copy-2: len 8, offset 8
    blk += bytes([3 | (4 << 2), 2, 0, 0, 0])             # copy-4: len 5, offset 2
    blk += bytes([5 << 2]) + b"xyzxyz"                   # literal of 6
    want = b"abcd" + b"abcd" + b"abcdabcd" + b"cdcdc" + b"xyzxyz"
    assert len(want) == 27
    assert K.snappy_decompress(blk) == want


@pytest.mark.parametrize("codec", ["snappy", "zstd"])
def test_kafka_codec_host_and_plan(codec):
    vals = _values(700, seed=11)
    rs = _record_set(vals, 53, codec) + _record_set(vals[:9], 9, "lz4", base=700)
    for min_off in (0, 7, 53, 200):
        got_v, got_o, recs, nxt = K.decode_records(rs, min_off, pad=0)
        got = [got_v[got_o[i]:got_o[i + 1]].tobytes() for i in range(len(got_o) - 1)]
        assert got == (vals + vals[:9])[min_off:] and nxt == 709
        plan = KD.plan_fetch(rs, min_off)
        kinds = set(plan.k_stored[:plan.nblk].tolist())
        assert kinds == {3 if codec == "snappy" else 4, 0}
        buf, s, e = KD.decode_on_host_like(np.frombuffer(rs, np.uint8), plan)
        assert [buf[x:y].tobytes() for x, y in zip(s, e)] == (vals + vals[:9])[min_off:]


def test_big_batches_make_multi_block_frames_and_chunks():
    vals = _values(3000, seed=12)
    rs = _record_set(vals, 1500, "zstd", level=3) + _record_set(vals, 1500, "snappy", base=3000)
    plan = KD.plan_fetch(rs, 0)
    kinds = plan.k_stored[:plan.nblk].tolist()
    assert kinds.count(4) == 2 and kinds.count(3) > 2          # xerial 32 KiB chunks
    buf, s, e = KD.decode_on_host_like(np.frombuffer(rs, np.uint8), plan)
    assert [buf[x:y].tobytes() for x, y in zip(s, e)] == vals + vals


# ---- independent oracle: pyarrow's bundled codecs -------------------------------------------------------------

pa = pytest.importorskip("pyarrow")


def _pa_compress(codec, data, level=None):
    c = pa.Codec(codec, compression_level=level) if level is not None else pa.Codec(codec)
    return c.compress(data).to_pybytes()


@pytest.mark.parametrize("level", [1, 3, 6, 9, 12, 19])
def test_zstd_host_decoder_matches_pyarrow(level):
    """pyarrow's zstd frames (content size in the header, single segment) decode with host_zstd.cpp; frames from
    our producer path decode with pyarrow."""
    for data in _samples():
        assert K.zstd_decompress(_pa_compress("zstd", data, level)) == data, (level, len(data))
    try:
        ours = K.zstd_compress(_samples()[4], level)
    except K.KafkaError:
        return
    assert pa.Codec("zstd").decompress(ours, decompressed_size=len(_samples()[4])).to_pybytes() == _samples()[4]


def test_snappy_host_decoder_matches_pyarrow():
    """Raw snappy blocks from pyarrow decode with host_snappy.cpp, and ours decode with pyarrow."""
    for data in _samples():
        assert K.snappy_decompress(_pa_compress("snappy", data)) == data, len(data)
        ours = K.snappy_compress(data, False)
        assert pa.Codec("snappy").decompress(ours, decompressed_size=len(data)).to_pybytes() == data


def test_lz4_frames_match_pyarrow():
    """LZ4 frames (the Kafka codec-3 payload) from pyarrow decode with host_lz4.cpp; ours decode with pyarrow."""
    from dxa.ops import lz4
    for data in _samples()[1:]:
        assert lz4.decompress_frame(_pa_compress("lz4", data)) == data, len(data)
        ours = lz4.compress_frame(np.frombuffer(data, np.uint8), 65536).tobytes()
        assert pa.Codec("lz4").decompress(ours, decompressed_size=len(data)).to_pybytes() == data


def _raw_batch(payload, count, codec, ts=1_700_000_000_000):
    """A v2 record batch around an already-compressed records payload, with a valid CRC-32C."""
    import struct
    tail = struct.pack(">hiqqqhii", codec, count - 1, ts, ts, -1, -1, -1, count) + payload
    crc = K.crc32c(tail)
    body = struct.pack(">ibI", 0, 2, crc) + tail
    return struct.pack(">qi", 0, len(body)) + body


def test_corrupt_declared_sizes_are_errors_not_allocations():
    """A zstd frame header claiming more content than its blocks can hold, and a snappy varint claiming more than its
    elements can expand to, are reported as malformed (never sized into an allocation), in the codec entry points and
    in a CRC-valid Kafka batch walked by the planner / host decoder."""
    frame = bytearray(_pa_compress("zstd", b"hello world " * 40, 3))
    assert frame[4] & 0xC0 == 0x40                         # 2-byte FCS (+256)
    frame[4] = (frame[4] & 0x3F) | 0xC0                   # 8-byte FCS, claims ~2^62 bytes
    huge = bytes(frame[:5]) + (1 << 62).to_bytes(8, "little") + bytes(frame[7:])
    with pytest.raises(K.KafkaError):
        K.zstd_decompress(huge)
    blk = bytes([0xFF, 0xFF, 0xFF, 0xFF, 0x07]) + bytes([3 << 2]) + b"abcd"   # varint 2^31-1 for 4 literal bytes
    with pytest.raises(K.KafkaError):
        K.snappy_decompress(blk)
    for codec, payload in (("zstd", huge), ("snappy", blk)):
        rs = _raw_batch(payload, 1, K.CODECS[codec])
        with pytest.raises(K.KafkaError):
            K.decode_records(rs, 0, pad=0)
        with pytest.raises(KD.Unsupported, match="malformed"):   # the device planner refuses it too
            KD.plan_fetch(rs, 0)


# ---- GPU decoders ---------------------------------------------------------------------------------------------

def _device_decode(gpu, rs, plan, chunks=2):
    staging = torch.zeros(len(rs) + 64, dtype=torch.uint8).pin_memory()
    staging[:len(rs)] = torch.frombuffer(bytearray(rs), dtype=torch.uint8)
    dec = KD.DeviceRecordDecoder(gpu, chunks=chunks)
    raw, ev = dec.decode(staging, plan)
    torch.cuda.current_stream(gpu).wait_event(ev)
    dec.check()
    buf = raw.buf.cpu().numpy()
    s, e = raw.offs[:-1].cpu().tolist(), raw.ends.cpu().tolist()
    return [buf[x:y].tobytes() for x, y in zip(s, e)], dec, staging


@pytest.mark.gpu
@pytest.mark.parametrize("level", [1, 3, 12, -5])
def test_device_zstd_matches_host(gpu, level):
    """zstd batches of 1 to 400 records (one- and multi-block frames, Huffman 1- and 4-stream literals, FSE /
    predefined / RLE / repeat sequence tables across blocks) next to LZ4, snappy and uncompressed batches."""
    rnd = random.Random(level)
    vals = _values(4000, seed=40 + level)
    vals += [bytes(rnd.getrandbits(8) for _ in range(rnd.choice([1, 100, 3000]))) for _ in range(30)]   # raw blocks
    vals += [b"a" * rnd.choice([3, 1000, 140000]) for _ in range(6)]                                    # RLE
    parts, base = [], 0
    for lo, hi, per, codec in ((0, 2500, 26, "zstd"), (2500, 3300, 400, "zstd"), (3300, 3600, 1, "zstd"),
                               (3600, 3800, 40, "snappy"), (3800, 3900, 30, "lz4"), (3900, len(vals), 7, "zstd")):
        parts.append(_record_set(vals[lo:hi], per, codec, level=level if codec == "zstd" else 3, base=base))
        base += hi - lo
    rs = b"".join(parts)
    plan = KD.plan_fetch(rs, 0)
    assert (plan.k_stored[:plan.nblk] == 4).sum() > 100
    got, dec, staging = _device_decode(gpu, rs, plan)
    assert got == vals
    # a corrupted frame is reported (nonzero status), never read or written out of range
    b0 = int(np.nonzero(plan.k_stored[:plan.nblk] == 4)[0][3])
    lo = int(plan.k_comp_off[b0])
    bad = bytearray(rs)
    # the frame's last byte ends its last block's sequence bitstream (no checksum): zero, it has no end marker.  The
    # header walk (planner) still succeeds; the device decode must report it.  (Damage inside raw literals — level
    # -5 stores them uncompressed — decodes to other bytes: only a content checksum could tell.)
    bad[lo + int(plan.k_comp_len[b0]) - 1] = 0
    plan2 = KD.plan_fetch(bytes(bad), 0, verify_crc=False)
    staging[:len(bad)] = torch.frombuffer(bad, dtype=torch.uint8)
    raw2, ev2 = dec.decode(staging, plan2)
    torch.cuda.current_stream(gpu).wait_event(ev2)
    with pytest.raises(KD.DecodeError):
        dec.check()


@pytest.mark.gpu
def test_device_snappy_matches_host(gpu):
    rnd = random.Random(5)
    vals = _values(3000, seed=50)
    vals += [bytes(rnd.getrandbits(8) for _ in range(rnd.choice([1, 70, 5000]))) for _ in range(20)]
    vals += [b"b" * rnd.choice([4, 65, 70000]) for _ in range(6)]
    rs = _record_set(vals[:2000], 26, "snappy") + _record_set(vals[2000:], 300, "snappy", base=2000)
    plan = KD.plan_fetch(rs, 0)
    got, dec, staging = _device_decode(gpu, rs, plan, chunks=3)
    assert got == vals


@pytest.mark.gpu
def test_device_decodes_hand_assembled_frames(gpu):
    """The hand-assembled zstd frame and snappy block run through the device kernels directly (one table entry
    each, kinds 4 and 3)."""
    from dxa.ops import native as N
    frame, content = _hand_frame()
    blk = bytes([27, 3 << 2]) + b"abcd" + bytes([1, 4]) + bytes([2 | (7 << 2), 8, 0]) + \
        bytes([3 | (4 << 2), 2, 0, 0, 0]) + bytes([5 << 2]) + b"xyzxyz"
    want_snappy = b"abcdabcdabcdabcdcdcdcxyzxyz"
    src = torch.zeros(len(frame) + len(blk) + 64, dtype=torch.uint8)
    src[:len(frame)] = torch.frombuffer(bytearray(frame), dtype=torch.uint8)
    src[len(frame):len(frame) + len(blk)] = torch.frombuffer(bytearray(blk), dtype=torch.uint8)
    src = src.to(gpu)
    dev = lambda xs, dt: torch.tensor(xs, dtype=dt, device=gpu)                  # noqa: E731
    co, cl = dev([0, len(frame)], torch.int64), dev([len(frame), len(blk)], torch.int32)
    kind = dev([4, 3], torch.uint8)
    oo, cap = dev([0, 64], torch.int64), dev([len(content), len(want_snappy)], torch.int64)
    out = torch.zeros(256, dtype=torch.uint8, device=gpu)
    produced = torch.zeros(2, dtype=torch.int64, device=gpu)
    status = torch.full((2,), -1, dtype=torch.int32, device=gpu)
    st = N.stream_handle(gpu)
    for entry in ("dxa_zstd_decode_into", "dxa_snappy_decode_into"):
        N.call(entry, N.ptr(src), N.ptr(co), N.ptr(cl), N.ptr(kind), N.ptr(oo), N.ptr(cap), 2, N.ptr(out),
               N.ptr(produced), N.ptr(status), st)
    torch.cuda.synchronize(gpu)
    assert status.tolist() == [0, 0] and produced.tolist() == [len(content), len(want_snappy)]
    o = out.cpu().numpy().tobytes()
    assert o[:len(content)] == content and o[64:64 + len(want_snappy)] == want_snappy


@pytest.mark.gpu
@pytest.mark.parametrize("level", [1, 3, 9, 19])
def test_device_decodes_pyarrow_frames(gpu, level):
    """zstd frames and snappy raw blocks written by pyarrow's codecs (independent of this package's encoders) through
    the device kernels, one table entry per frame / block."""
    from dxa.ops import native as N
    datas = _samples()[1:] + [b"\n".join(_values(26, seed=s)) for s in range(20)]
    for codec, kind, entry in (("zstd", 4, "dxa_zstd_decode_into"), ("snappy", 3, "dxa_snappy_decode_into")):
        comp = [_pa_compress(codec, d, level if codec == "zstd" else None) for d in datas]
        co, pos = [], 0
        for c in comp:
            co.append(pos)
            pos += len(c)
        src = torch.zeros(pos + 64, dtype=torch.uint8)
        src[:pos] = torch.frombuffer(bytearray(b"".join(comp)), dtype=torch.uint8)
        oo, opos = [], 0
        for d in datas:
            oo.append(opos)
            opos += (len(d) + 63) // 64 * 64
        dev = lambda xs, dt: torch.tensor(xs, dtype=dt, device=gpu)                  # noqa: E731
        n = len(datas)
        out = torch.zeros(opos + 64, dtype=torch.uint8, device=gpu)
        produced = torch.zeros(n, dtype=torch.int64, device=gpu)
        status = torch.full((n,), -1, dtype=torch.int32, device=gpu)
        # every operand held in a name until the launch has run (a temporary's block could be reused by the next
        # allocation before the kernel reads it)
        ops = [src.to(gpu), dev(co, torch.int64), dev([len(c) for c in comp], torch.int32), dev([kind] * n, torch.uint8),
               dev(oo, torch.int64), dev([len(d) for d in datas], torch.int64)]
        N.call(entry, *[N.ptr(x) for x in ops], n, N.ptr(out), N.ptr(produced), N.ptr(status), N.stream_handle(gpu))
        torch.cuda.synchronize(gpu)
        del ops
        assert status.tolist() == [0] * n, (codec, status.tolist())
        assert produced.tolist() == [len(d) for d in datas]
        o = out.cpu().numpy().tobytes()
        for d, off in zip(datas, oo):
            assert o[off:off + len(d)] == d, (codec, len(d))
