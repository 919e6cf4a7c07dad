"""Simulated-data Kafka producer (reference: DataProcessing/datax-host/src/main/scala/datax/app/KafkaProducer.scala:
19-95 — random JSON from a schema, 10 messages/s per topic).  Events are rendered by the schema-driven generator
(GPU when available, else the bit-identical CPU path) and sent as v2 record batches, one batch per topic per tick.

    python -m dxa.simulate.kafka_producer --bootstrap 127.0.0.1:9092 --topics iot1,iot2 --schema schema.json \\
        --rate 10 --seconds 60
    python -m dxa.simulate.kafka_producer --eventhub "Endpoint=sb://ns.servicebus.windows.net/;...;EntityPath=hub"
"""
from __future__ import annotations

import argparse
import json
import time
from typing import List, Optional

import torch

from ..engine.types import schema_from_json
from ..io.kafka import KafkaClient, eventhub_kafka_settings
from .datagen import compile_simulated, compile_spark, generate


def render_events(prog, n: int, device, seed: int, row0: int) -> List[bytes]:
    buf, offs = generate(prog, n, device, seed=seed, row0=row0)
    b = bytes(buf.cpu().numpy())
    o = offs.cpu().tolist()
    return [b[o[i]:o[i + 1]] for i in range(n)]


def program_from_schema_text(text: str):
    obj = json.loads(text)
    if isinstance(obj, dict) and "dataSchema" in obj:
        return compile_simulated(obj["dataSchema"][0]["fields"])
    return compile_spark(schema_from_json(text))


def run(client: KafkaClient, topics: List[str], prog, rate: int, seconds: Optional[float], device="cpu",
        seed: int = 1, compression: str = "none") -> int:
    meta = client.metadata(topics)
    sent, row, t_end = 0, 0, None if seconds is None else time.time() + seconds
    tick = 0
    while t_end is None or time.time() < t_end:
        t0 = time.time()
        for t in topics:
            parts = meta.get(t) or [0]
            events = render_events(prog, rate, device, seed, row)
            row += rate
            client.produce(t, parts[tick % len(parts)], events, compression=compression)
            sent += len(events)
        tick += 1
        time.sleep(max(0.0, 1.0 - (time.time() - t0)))
    return sent


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--bootstrap")
    ap.add_argument("--eventhub", help="Event Hubs connection string (uses its Kafka endpoint)")
    ap.add_argument("--topics", default="")
    ap.add_argument("--schema", required=True, help="Spark schema JSON (DataGenerator metadata) or SimulatedData")
    ap.add_argument("--rate", type=int, default=10, help="events per second per topic")
    ap.add_argument("--seconds", type=float, default=None)
    ap.add_argument("--compression", choices=["none", "gzip", "lz4"], default="none",
                    help="record batch compression (Kafka compression.type)")
    args = ap.parse_args(argv)
    with open(args.schema) as f:
        prog = program_from_schema_text(f.read())
    if args.eventhub:
        es = eventhub_kafka_settings(args.eventhub)
        client = KafkaClient(es["bootstrap"], use_ssl=True, sasl=es["sasl"])
        topics = [es["topic"]]
    else:
        client = KafkaClient(args.bootstrap)
        topics = [t for t in args.topics.split(",") if t]
    device = "cuda" if torch.cuda.is_available() else "cpu"
    n = run(client, topics, prog, args.rate, args.seconds, device, compression=args.compression)
    print(json.dumps({"sent": n}))


if __name__ == "__main__":
    main()
