"""bench.py's gpu-sim source: batch j's events carry event times in the interval before its batch time, so the
windowed flows' 5-minute windows hold 300 one-second panes (profiles/round5/evtime/README.md)."""
import calendar
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402
from dxa.models import iot  # noqa: E402
from dxa.simulate.datagen import generate  # noqa: E402


def _event_secs(buf, offs):
    o = offs.tolist()
    b = bytes(buf.numpy())
    out = []
    for k in range(len(o) - 1):
        t = json.loads(b[o[k]:o[k + 1]])["deviceDetails"]["eventTime"]
        out.append(calendar.timegm(time.strptime(t, "%Y-%m-%dT%H:%M:%SZ")))
    return out


def test_gpu_sim_events_fall_in_the_interval_before_their_batch_time():
    E, interval_us = 400, 1_000_000
    clock0_us = 1_700_000_000 * 1_000_000
    prog = iot.program()
    for j in (0, 1, 7, 300):
        buf, offs = generate(prog, E, torch.device("cpu"), **bench.sim_gen_args(j, 0, E, clock0_us, interval_us))
        bt_s = (clock0_us + j * interval_us) // 1_000_000
        secs = _event_secs(buf, offs)
        assert min(secs) >= bt_s - 1 and max(secs) < bt_s, (j, min(secs), max(secs), bt_s)


def test_gpu_sim_batches_differ_per_rank_and_batch():
    a = bench.sim_gen_args(3, 0, 100, 0, 1_000_000)
    b = bench.sim_gen_args(3, 1, 100, 0, 1_000_000)
    c = bench.sim_gen_args(4, 0, 100, 0, 1_000_000)
    assert a["seed"] != b["seed"] and a["seed"] != c["seed"] and a["row0"] != c["row0"]
    assert a["base_ms"] == c["base_ms"]          # the base does not advance with the batch
