"""Wire-format checks against vectors taken from the protocols' published definitions rather than this repository's
own encoders: the CRC-32C check value (RFC 3720 appendix B.4), protobuf-style varint / zig-zag examples (the
encoding Kafka's record format adopts), a Kafka v2 RecordBatch assembled byte by byte from the field table of the
Kafka protocol guide, and AMQP 1.0 primitive type codes from the AMQP 1.0 types section (§1.6)."""
import struct

import pytest

from dxa.io import amqp
from dxa.io import kafka


def test_crc32c_check_value():
    assert kafka.crc32c(b"123456789") == 0xE3069283
    from dxa.io.kafka_device import crc32c_segmented
    assert crc32c_segmented(b"123456789") == 0xE3069283


def _uvarint(v):
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        out.append(b | (0x80 if v else 0))
        if not v:
            return bytes(out)


def _zigzag(v):
    return _uvarint((v << 1) ^ (v >> 63))


def test_varint_examples():
    # protobuf encoding guide: 150 -> 96 01, 300 -> AC 02; zig-zag: 0->0, -1->1, 1->2, -2->3, 2147483647->4294967294
    assert _uvarint(150) == b"\x96\x01" and _uvarint(300) == b"\xac\x02"
    assert [_zigzag(v) for v in (0, -1, 1, -2)] == [b"\x00", b"\x01", b"\x02", b"\x03"]
    assert _zigzag(2147483647) == _uvarint(4294967294)


def _spec_batch(base_offset, ts, values):
    """RecordBatch (magic 2) per the Kafka protocol guide: baseOffset int64, batchLength int32, partitionLeaderEpoch
    int32, magic int8, crc uint32 (CRC-32C of everything after it), attributes int16, lastOffsetDelta int32,
    baseTimestamp int64, maxTimestamp int64, producerId int64, producerEpoch int16, baseSequence int32, records
    [length varint, attributes int8, timestampDelta varlong, offsetDelta varint, keyLength varint (-1 = null),
    valueLength varint, value, headers count varint]."""
    recs = bytearray()
    for i, v in enumerate(values):
        body = b"\x00" + _zigzag(0) + _zigzag(i) + _zigzag(-1) + _zigzag(len(v)) + v + _zigzag(0)
        recs += _zigzag(len(body)) + body
    after_crc = struct.pack(">hiqqqhii", 0, len(values) - 1, ts, ts, -1, -1, -1, len(values)) + bytes(recs)
    crc = kafka.crc32c(after_crc)
    after_len = struct.pack(">ibI", 0, 2, crc) + after_crc
    return struct.pack(">qi", base_offset, len(after_len)) + after_len


def test_kafka_batch_from_the_spec_decodes():
    vals = [b"hello", b"", b'{"a":1}']
    batch = _spec_batch(42, 1_700_000_000_000, vals)
    arena, offs, rec_offsets, next_offset = kafka.decode_records(batch, 0)
    o = [int(x) for x in offs]
    assert [bytes(arena[o[i]:o[i + 1]]) for i in range(len(vals))] == vals
    assert [int(x) for x in rec_offsets] == [42, 43, 44] and next_offset == 45
    # records below the fetch's start offset are dropped (a fetch can start inside a batch)
    arena, offs, rec_offsets, next_offset = kafka.decode_records(batch, 43)
    assert [int(x) for x in rec_offsets] == [43, 44]
    # a flipped byte after the CRC field is reported
    bad = bytearray(batch)
    bad[-2] ^= 0x01
    with pytest.raises(Exception):
        kafka.decode_records(bytes(bad), 0)
    # this repository's encoder writes exactly the spec layout
    assert kafka.encode_batch(vals, timestamp_ms=1_700_000_000_000) == _spec_batch(0, 1_700_000_000_000, vals)


def test_amqp_primitive_codes():
    # AMQP 1.0 part 1 §1.6: null 0x40, true 0x41, false 0x42, uint0 0x43, ulong0 0x44, list0 0x45, smalluint 0x52,
    # smallulong 0x53, str8-utf8 0xa1, sym8 0xa3, described-type constructor 0x00
    assert amqp.encode(None) == b"\x40"
    assert amqp.encode(True) == b"\x41" and amqp.encode(False) == b"\x42"
    assert amqp.encode(amqp.UInt(0)) == b"\x43" and amqp.encode(amqp.ULong(0)) == b"\x44"
    assert amqp.encode([]) == b"\x45"
    assert amqp.encode(amqp.UInt(7)) == b"\x52\x07" and amqp.encode(amqp.ULong(16)) == b"\x53\x10"
    assert amqp.encode("ab") == b"\xa1\x02ab" and amqp.encode(amqp.Symbol("ab")) == b"\xa3\x02ab"
    d = amqp.encode(amqp.Described(amqp.ULong(0x10), []))          # an empty open performative
    assert d == b"\x00\x53\x10\x45"
    for raw, val in ((b"\x40", None), (b"\x41", True), (b"\x52\x07", 7), (b"\xa1\x02ab", "ab")):
        assert amqp.decode(raw)[0] == val
