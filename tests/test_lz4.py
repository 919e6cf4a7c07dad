"""LZ4 block/frame codec (host), Kafka compressed record batches, and the device decoder + newline framing.

The host encoder is checked against an independent pure-Python block decoder written from the format
description (token / literal run / little-endian offset / match length extension), and xxHash32 against its
published test values."""
import random

import numpy as np
import pytest
import torch

from dxa.io import kafka as K
from dxa.ops import lz4


def _py_block_decode(src: bytes) -> bytes:
    out = bytearray()
    i = 0
    while i < len(src):
        tok = src[i]
        i += 1
        lit = tok >> 4
        if lit == 15:
            while True:
                b = src[i]
                i += 1
                lit += b
                if b != 255:
                    break
        out += src[i:i + lit]
        i += lit
        if i >= len(src):
            break
        off = src[i] | (src[i + 1] << 8)
        i += 2
        ml = tok & 15
        if ml == 15:
            while True:
                b = src[i]
                i += 1
                ml += b
                if b != 255:
                    break
        ml += 4
        assert 0 < off <= len(out)
        for _ in range(ml):
            out.append(out[-off])
    return bytes(out)


def _py_frame_decode(f: bytes) -> bytes:
    assert f[:4] == b"\x04\x22\x4d\x18"
    flg = f[4]
    p = 6 + (8 if flg & 0x08 else 0) + 1
    out = b""
    while True:
        w = int.from_bytes(f[p:p + 4], "little")
        p += 4
        if w == 0:
            return out
        n = w & 0x7FFFFFFF
        blk = f[p:p + n]
        out += blk if w >> 31 else _py_block_decode(blk)
        p += n


def _samples(seed=0):
    rnd = random.Random(seed)
    yield b""
    yield b"a"
    yield b"x" * 100000                                    # long runs: offset-1 overlapping matches
    yield bytes(rnd.getrandbits(8) for _ in range(5000))  # incompressible → stored blocks
    yield b"".join(b'{"deviceId":%d,"temp":%0.4f,"kind":"%s"}\n' % (rnd.randint(0, 99), rnd.uniform(-50, 50),
                   rnd.choice([b"door", b"heat", b"light"])) for _ in range(3000))


def test_xxh32_vectors():
    assert lz4.xxh32(b"") == 0x02CC5D05
    assert lz4.xxh32(b"abc") == 0x32D153FF


@pytest.mark.parametrize("block", [1024, 16384, 65536])
def test_frame_roundtrip_and_independent_decoder(block):
    for data in _samples():
        f = lz4.compress_frame(data, block)
        assert lz4.decompress_frame(f) == data
        assert _py_frame_decode(f.tobytes()) == data
        t = lz4.frame_table(f)
        assert t.content_size == len(data) and t.nblocks == (len(data) + block - 1) // block
        # header checksum byte = second byte of xxh32(descriptor)
        assert f[14] == (lz4.xxh32(f[4:14]) >> 8) & 0xFF


@pytest.mark.parametrize("level", [3, 6, 9])
def test_high_compression_levels_roundtrip(level):
    """The hash-chain (HC) compressor emits standard LZ4: the independent Python decoder reads it back, and on
    JSON it needs fewer sequences and bytes than the greedy compressor."""
    for data in _samples():
        f = lz4.compress_frame(data, 4096, level=level)
        assert lz4.decompress_frame(f) == data
        assert _py_frame_decode(f.tobytes()) == data
    js = b"".join(_samples(4))
    assert lz4.compress_frame(js, 16384, level=level).size <= lz4.compress_frame(js, 16384).size


def test_block_codec_and_malformed_input():
    data = b"abcdefgh" * 1000 + b"tail-bytes"
    blk = lz4.compress_block(data)
    assert len(blk) < len(data) // 10
    assert lz4.decompress_block(blk, len(data)) == data == _py_block_decode(blk)
    with pytest.raises(lz4.Lz4Error):
        lz4.decompress_block(blk, len(data) - 1)          # output overflow is detected
    for bad in (bytes([0x04, 0x01, 0x00]),                # match offset reaching before the output start
                bytes([0xF0]),                            # literal length extension missing
                bytes([0x30, 0x61, 0x62])):               # 3 literals announced, 2 present
        with pytest.raises(lz4.Lz4Error):
            lz4.decompress_block(bad, 100)


@pytest.mark.parametrize("codec", ["gzip", "lz4"])
def test_kafka_compressed_batches(codec):
    vals = [b'{"a":%d,"s":"%s"}' % (i, b"x" * (i % 50)) for i in range(500)]
    batch = K.encode_batch(vals, timestamp_ms=5, compression=codec)
    plain = K.encode_batch(vals, timestamp_ms=5)
    assert len(batch) < len(plain) // 2
    buf, offs, recoffs, nxt = K.decode_records(batch, 0)
    assert [bytes(buf[offs[i]:offs[i + 1]]) for i in range(len(vals))] == vals
    assert recoffs.tolist() == list(range(500)) and nxt == 500


@pytest.mark.gpu
def test_gpu_lz4_decode_matches_host():
    assert torch.cuda.is_available()
    dev = torch.device("cuda", 0)
    rnd = random.Random(5)
    data = b"".join(_samples(1)) + bytes(rnd.getrandbits(8) % 7 for _ in range(200000))
    for block in (1024, 16384, 65536):
        f = lz4.compress_frame(data, block)
        for known in (block, None):                       # known block sizes / device size pass
            fr = lz4.DeviceFrame.from_frame(f, known).to(dev)
            out = lz4.decompress_device(fr, check=True)
            torch.cuda.synchronize()
            got = out.cpu().numpy()
            assert got.size == len(data) + 16 and got[:len(data)].tobytes() == data and not got[len(data):].any()


@pytest.mark.gpu
def test_gpu_newline_framing():
    from dxa.ops.jsonparse import frame_lines_gpu
    assert torch.cuda.is_available()
    dev = torch.device("cuda", 0)
    rnd = random.Random(9)
    lines = [bytes(rnd.choice(b"abc{}:,\"0123") for _ in range(rnd.choice([0, 1, 5, 15, 16, 17, 200, 3000])))
             for _ in range(4000)]
    blob = b"\n".join(lines) + b"\n"
    buf = torch.zeros(len(blob) + 16, dtype=torch.uint8)
    buf[:len(blob)] = torch.frombuffer(bytearray(blob), dtype=torch.uint8)
    d = buf.to(dev)
    offs = frame_lines_gpu(d, len(blob), expected=len(lines)).cpu().tolist()
    want = [0]
    for ln in lines:
        want.append(want[-1] + len(ln) + 1)
    assert offs == want
    # a producer count that disagrees with the text: missing records are empty (never uninitialised offsets), extra
    # newlines are not framed, and both are reported through the deferred check
    from dxa.ops.jsonparse import check_framing
    checks = []
    short = frame_lines_gpu(d, len(blob), expected=len(lines) + 5, mismatches=checks).cpu().tolist()
    assert short == want + [len(blob)] * 5
    with pytest.raises(ValueError):
        check_framing(checks)
    long = frame_lines_gpu(d, len(blob), expected=len(lines) - 3, mismatches=checks).cpu().tolist()
    assert long == want[:len(lines) - 2]
    with pytest.raises(ValueError):
        check_framing(checks)
    frame_lines_gpu(d, len(blob), expected=len(lines), mismatches=checks)
    check_framing(checks)
    # counting mode drops empty lines
    offs2 = frame_lines_gpu(d, len(blob)).cpu().tolist()
    recs = [blob[offs2[i]:offs2[i + 1]].strip() for i in range(len(offs2) - 1)]
    assert recs == [ln for ln in lines if ln]


@pytest.mark.gpu
def test_gpu_lz4_wave_decoder_edge_cases():
    """The wave-per-block LDS decoder against the host codec: incompressible literal runs longer than the 512-B
    register window, RLE runs (offset 1), short periods (offset < 64), long matches, odd block sizes (unaligned
    16-B flush), and > 64 KiB blocks (per-lane fallback)."""
    assert torch.cuda.is_available()
    dev = torch.device("cuda", 0)
    rnd = random.Random(11)
    parts = []
    for i in range(300):
        k = i % 6
        if k == 0:
            parts.append(bytes(rnd.getrandbits(8) for _ in range(rnd.choice([1, 63, 64, 65, 300, 700, 2000]))))
        elif k == 1:
            parts.append(bytes([rnd.getrandbits(8)]) * rnd.choice([4, 5, 19, 64, 65, 1000, 5000]))
        elif k == 2:
            per = bytes(rnd.getrandbits(8) for _ in range(rnd.choice([2, 3, 7, 31, 63, 64, 65])))
            parts.append(per * rnd.choice([3, 10, 40]))
        elif k == 3:
            parts.append(b'{"deviceId":%d,"temperature":%d.5,"status":"ok"}\n' % (i, i * 7))
        else:
            parts.append(parts[rnd.randrange(len(parts))])
    data = b"".join(parts)
    for block, level in ((1000, 0), (4096, 0), (16384, 0), (16384, 9), (40000, 9), (65536, 0), (131072, 0)):
        f = lz4.compress_frame(data, block, level=level)
        for known in (block, None):
            fr = lz4.DeviceFrame.from_frame(f, known).to(dev)
            out = lz4.decompress_device(fr, check=True)
            torch.cuda.synchronize()
            got = out.cpu().numpy()
            assert got[:len(data)].tobytes() == data, (block, known)
            assert not got[len(data):].any()


@pytest.mark.gpu
def test_gpu_lz4_chunked_ingest():
    """Pinned host frame → chunked H2D copy / decode pipeline equals the host codec's output."""
    assert torch.cuda.is_available()
    dev = torch.device("cuda", 0)
    data = b"".join(_samples(3)) * 4
    f = lz4.compress_frame(data, 4096)
    fr = lz4.DeviceFrame.from_frame(f, 4096, pin=True)
    for chunks in (1, 3, 8):
        ing = lz4.ChunkedIngest(dev, chunks=chunks)
        out, ev = ing.stage(fr)
        torch.cuda.current_stream(dev).wait_event(ev)
        got = out.cpu().numpy()
        assert got[:len(data)].tobytes() == data and not got[len(data):].any()
