"""Host-side native code under AddressSanitizer + UndefinedBehaviorSanitizer (GPU sanitizers are not available on
this platform): the Kafka codec, the LZ4 codec and the row serializer are compiled together with a self-check driver and
run as a standalone executable.  The snappy and zstd decoders also take truncated and garbage inputs there."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "dxa", "ops", "csrc")


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_host_codecs_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "host_codecs_check")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=undefined", "-I", CSRC, os.path.join(ROOT, "tests", "native", "host_codecs_check.cpp"),
           os.path.join(CSRC, "host_kafka.cpp"), os.path.join(CSRC, "host_lz4.cpp"), os.path.join(CSRC, "host_serialize.cpp"),
           os.path.join(CSRC, "host_snappy.cpp"), os.path.join(CSRC, "host_zstd.cpp"), "-lz", "-ldl", "-pthread", "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "0 failures" in r.stdout
