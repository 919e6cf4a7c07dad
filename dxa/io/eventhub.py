"""Event Hubs / IoT Hub direct stream over AMQP 1.0 (``dxa.io.amqp``) — the reference's EventHubStreamingFactory
(DataProcessing/datax-host/src/main/scala/datax/input/EventHubStreamingFactory.scala:23-118) and its checkpointer
(checkpoint/EventhubCheckpointer.scala:13-74).

* partitions come from the hub's ``$management`` node and are spread over ranks (sorted id position mod world);
* the starting position per partition is, in order: the sequence number in ``offsets.txt`` (unless
  ``flushexistingcheckpoints``), else ``startenqueuetime`` (0: start of stream, < 0: now-relative seconds,
  > 0: epoch seconds), else the end of the stream (EventHubStreamingFactory.scala:47-64);
* a batch takes up to ``maxrate`` events per partition (``maxRatePerPartition``); its ranges are
  ``(fromSeq, untilSeq)`` per partition, committed after the batch's outputs (at-least-once) in the reference's
  ``batchTimeMs,hub,partition,fromSeq,untilSeq`` lines;
* every event's application properties become its ``Properties`` map and its ``x-opt-*`` annotations its
  ``SystemProperties`` map (x-opt-sequence-number, x-opt-offset, x-opt-enqueued-time, x-opt-partition-key — plus
  iothub-* annotations for IoT Hub), as DirectProcessor builds them from EventData.
"""
from __future__ import annotations

import datetime as _dt
import time
from typing import Dict, List, Optional

import torch

from .amqp import AmqpConnection, AmqpError, management_partitions, parse_eventhub_connection
from .sources import Checkpointer, OffsetTrackedSource, RawBatch, _to_device_batch

EARLIEST, LATEST = -2, -1


def selector(seq: Optional[int], start: int) -> str:
    """Event Hubs selector filter for a partition's starting position."""
    if seq is not None:
        return f"amqp.annotation.x-opt-sequence-number >= '{seq}'"
    if start == EARLIEST:
        return "amqp.annotation.x-opt-offset > '-1'"
    if start == LATEST:
        return "amqp.annotation.x-opt-offset > '@latest'"
    return f"amqp.annotation.x-opt-enqueued-time > '{int(start)}'"


def _prop_value(v) -> str:
    if isinstance(v, bytes):
        return v.decode("utf-8", "replace")
    if isinstance(v, int) and type(v).__name__ == "Timestamp":
        return _dt.datetime.utcfromtimestamp(int(v) / 1000).strftime("%Y-%m-%d %H:%M:%S.%f")[:-3]
    return str(v)


class EventHubSource(OffsetTrackedSource):
    name = "eventhub"

    def __init__(self, connection_string: str, device, consumer_group: str = "$Default",
                 checkpoint_dir: Optional[str] = None, max_rate: Optional[int] = None, start: int = LATEST,
                 flush_existing: bool = False, rank: Optional[int] = None, world: Optional[int] = None,
                 hub: Optional[str] = None, partitions: Optional[List[str]] = None, wait_s: float = 0.5):
        from .. import parallel as P
        rank = P.rank() if rank is None else rank
        world = P.world() if world is None else world
        cs = parse_eventhub_connection(connection_string)
        self.hub = hub or cs["entity"]
        if not self.hub:
            raise AmqpError("no Event Hub name (EntityPath in the connection string, or eventhub.name)")
        self.device = torch.device(device)
        self.max_rate = max_rate
        self.wait_s = wait_s
        self.conn = AmqpConnection(cs["host"], int(cs["port"]), cs["tls"] == "1", username=cs["keyname"] or None,
                                   password=cs["key"] or None)
        parts = partitions or management_partitions(self.conn, self.hub)
        ordered = sorted(parts, key=lambda p: (len(p), p))
        self.parts = [p for i, p in enumerate(ordered) if i % world == rank]
        ckpt = Checkpointer(checkpoint_dir, rank, world) if checkpoint_dir else None
        restored = {} if (ckpt is None or flush_existing) else ckpt.restore()
        pos: Dict[str, Optional[int]] = {}
        self.links = {}
        for p in self.parts:
            seq = restored.get((self.hub, p))
            pos[p] = seq
            addr = f"{self.hub}/ConsumerGroups/{consumer_group}/Partitions/{p}"
            self.links[p] = self.conn.attach_receiver(addr, selector(seq, start),
                                                      credit=max(100, min(max_rate or 5000, 5000)))
        self._init_offsets(pos, ckpt, hub_of=lambda p: (self.hub, p))

    def next_batch(self, batch_time_us: int) -> Optional[RawBatch]:
        cap = self.max_rate

        def enough():
            return cap is not None and all(len(l.queue) >= cap for l in self.links.values())
        self.conn.pump(self.wait_s, enough)
        recs, props, sysprops = [], [], []
        ranges = {}
        for p, link in self.links.items():
            msgs = link.drain(cap)
            start = self.fetch_pos.get(p)
            last = None
            for m in msgs:
                ann = m["annotations"]
                seq = ann.get("x-opt-sequence-number")
                last = int(seq) if seq is not None else last
                recs.append(m["body"])
                props.append({str(k): _prop_value(v) for k, v in (m["app"] or {}).items()})
                sp = {str(k): _prop_value(v) for k, v in ann.items()}
                sp["x-opt-partition-id"] = p
                sysprops.append(sp)
            if msgs:
                first = int(msgs[0]["annotations"].get("x-opt-sequence-number", start or 0))
                ranges[p] = (start if start is not None else first, (last if last is not None else first) + 1)
            elif start is not None:
                ranges[p] = (start, start)
            # no position yet (reading from the end, nothing arrived): nothing to checkpoint for this partition
        self._record_batch(batch_time_us, ranges)
        raw = _to_device_batch(recs, self.device)
        if recs:
            from ..engine.column import column_from_pylist
            from ..engine.types import MapType
            mt = MapType("string", "string")
            raw.properties = column_from_pylist(props, mt, self.device)
            raw.system_properties = column_from_pylist(sysprops, mt, self.device)
        return raw

    def close(self):
        self.conn.close()


def build_eventhub_source(inp, device, rank: int = 0, world: int = 1) -> EventHubSource:
    """From ``datax.job.input.default.eventhub.*`` (EventHubInputSetting.scala:24-31)."""
    from ..config.secrets import resolve
    from .kafka import start_position
    conn = resolve(inp.get_string("eventhub.connectionstring"))
    st = inp.get("eventhub.startenqueuetime")
    start = start_position(st, None) if st not in (None, "") else LATEST
    rate = inp.get("eventhub.maxrate")
    return EventHubSource(conn, device, consumer_group=inp.get("eventhub.consumergroup") or "$Default",
                          checkpoint_dir=inp.get("eventhub.checkpointdir"), max_rate=int(rate) if rate else None,
                          start=start,
                          flush_existing=(inp.get("eventhub.flushexistingcheckpoints") or "false").lower() == "true",
                          rank=rank, world=world, hub=inp.get("eventhub.name") or None)
