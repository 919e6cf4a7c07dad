"""Device gzip (deflate.hip) — every output must inflate back to the input with Python's gzip / zlib."""
import gzip
import json
import random
import zlib

import pytest
import torch

pytestmark = pytest.mark.gpu


def _json_lines(n, seed=1):
    rnd = random.Random(seed)
    return "\n".join(json.dumps({"deviceDetails": {"deviceId": rnd.randint(1, 10000), "homeId": rnd.randint(1, 100),
                                                   "deviceType": rnd.choice(["DoorLock", "Heating", "WindowLock"])},
                                 "telemetry": {"temperature": round(rnd.uniform(-10, 40), 3), "ok": rnd.random() < .5},
                                 "Rules": [{"ruleId": "r1", "severity": "Critical"}] if rnd.random() < .3 else []})
                     for _ in range(n)).encode()


@pytest.mark.parametrize("dynamic", [False, True])
@pytest.mark.parametrize("chunk", [64, 4096, 32768])
def test_gzip_device_round_trip(gpu, chunk, dynamic):
    from dxa.ops.deflate import gzip_device
    rnd = random.Random(chunk)
    cases = [b"", b"a", b"abc", b"abcd" * 3, b"a" * 70000, bytes(rnd.getrandbits(8) for _ in range(50000)),
             _json_lines(3000), b"x" * (chunk - 1), b"yz" * chunk, bytes(range(256)) * 300]
    for data in cases:
        t = torch.frombuffer(bytearray(data + b"\0" * 16), dtype=torch.uint8).to(gpu)
        out = bytes(gzip_device(t, len(data), chunk, dynamic).cpu().numpy()) if data else b""
        if not data:
            continue
        assert gzip.decompress(out) == data, (chunk, len(data))


def test_gzip_device_ratio_on_json(gpu):
    from dxa.ops.deflate import gzip_device
    data = _json_lines(20000)
    t = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(gpu)
    sizes = []
    for dynamic in (False, True):
        out = bytes(gzip_device(t, len(data), dynamic=dynamic).cpu().numpy())
        assert gzip.decompress(out) == data
        sizes.append(len(out))
    assert sizes[0] < len(data) / 3 and sizes[1] < sizes[0], sizes
