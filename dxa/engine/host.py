"""Job hosts: the streaming micro-batch driver loop and the blob batch host.

Reference: DataProcessing/datax-host/src/main/scala/datax/host/StreamingHost.scala:22-97 (StreamingContext with a
batch interval, per-batch ``processor.process``, checkpoint restore) and BlobBatchingHost.scala:25-105 (path templates
``{yyyy-MM-dd…}`` expanded over ``[processStartTime, processEndTime]`` by ``partitionIncrement``).

The streaming loop aligns batch times to the interval (like DStream batch times), fetches the source's batch, runs
the processor, commits the source offsets only after a successful batch (at-least-once, as the reference), and
applies the reference's failure policy: record telemetry, sleep 1 s and stop (the job supervisor restarts from the
last checkpoint).  ``pipeline=True`` prefetches batch t+1 from the source while batch t is processed.
"""
from __future__ import annotations

import datetime as _dt
import logging
import re
import signal
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from typing import Callable, Dict, List, Optional, Tuple

from ..io import fs
from .processor import Processor, RawBatch

log = logging.getLogger("dxa.host")


class StreamingHost:
    def __init__(self, processor: Processor, source, interval_s: float, max_batches: Optional[int] = None,
                 realtime: bool = True, pipeline: bool = True,
                 on_batch: Optional[Callable[[int, Dict[str, float]], None]] = None):
        self.processor = processor
        self.source = source
        self.interval_us = int(interval_s * 1e6)
        self.max_batches = max_batches
        self.realtime = realtime
        self.pipeline = pipeline
        self.on_batch = on_batch
        self._stop = threading.Event()
        self.batches = 0
        self.history: List[Dict[str, float]] = []
        declare = getattr(processor, "declare_source_metrics", None)
        if declare is not None:
            declare(getattr(source, "metric_names", ()))

    def stop(self):
        self._stop.set()

    def _batch_time(self, t_us: int) -> int:
        return (t_us // self.interval_us) * self.interval_us

    def run(self):
        from ..utils import settle_gc
        settle_gc()
        pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix="dxa-prefetch") if self.pipeline else None
        next_time = self._batch_time(int(time.time() * 1e6)) + (self.interval_us if self.realtime else 0)
        prefetched = None
        prev_cb = self.processor.on_batch_complete
        self.processor.on_batch_complete = self._completed
        from ..telemetry.appinsights import track_event, track_exception
        kind = "localstreaming" if getattr(self.source, "name", "") == "local" else "streaming"
        try:
            while not self._stop.is_set():
                if self.max_batches is not None and self.batches >= self.max_batches:
                    break
                if self.realtime:
                    wait = next_time / 1e6 - time.time()
                    if wait > 0 and self._stop.wait(wait):
                        break
                bt = next_time
                if prefetched is not None:
                    raw = prefetched.result()
                else:
                    raw = self.source.next_batch(bt)
                if pool is not None:
                    nbt = bt + self.interval_us
                    prefetched = pool.submit(self.source.next_batch, nbt)
                if raw is None:
                    break
                bt_str = _fmt_batch_time(bt)
                track_event(f"{kind}/batch/begin", {"batchTime": bt_str})
                try:
                    self.processor.process_batch(raw, bt, self.interval_us, _dt.datetime.utcfromtimestamp(bt / 1e6))
                except Exception as e:
                    # EventHubStreamingFactory.scala:100-106: the exception with the batch's per-partition start
                    # sequence numbers as measurements, then fail the job
                    track_exception("StreamingHost", bt_str, e, {"batchTime": bt_str}, self._offset_measures(bt))
                    log.exception("batch failed; stopping the job (restart resumes from the last checkpoint)")
                    time.sleep(1.0)
                    raise
                track_event(f"{kind}/batch/end", {"batchTime": bt_str})
                self.batches += 1
                next_time = bt + self.interval_us
                if prefetched is not None and prefetched.done() and prefetched.exception() is None:
                    nxt = prefetched.result()
                    prep = getattr(self.processor, "prepare", None)
                    if nxt is not None and prep is not None:
                        prep(nxt)                            # its parse queues behind this batch's kernels
            self.processor.drain()
        finally:
            self.processor.on_batch_complete = prev_cb
            if pool is not None:
                pool.shutdown(wait=False, cancel_futures=True)
            self.source.close()
        return self.history

    def _offset_measures(self, bt: int) -> Dict[str, float]:
        ranges = getattr(self.source, "_inflight", {}).get(bt, {}) if hasattr(self.source, "_inflight") else {}
        hub_of = getattr(self.source, "_hub_of", lambda k: (str(k), ""))
        out = {}
        for k, (s, _e) in ranges.items():
            name, part = hub_of(k)
            out[f"{name}-{part}-fromSeqNo"] = float(s)
        return out

    def _completed(self, bt: int, metrics: Dict[str, float]):
        """A batch's outputs are written: only now are its source offsets committed (at-least-once) — after the
        source confirms the batch decoded cleanly (device-side decoders report errors asynchronously)."""
        verify = getattr(self.source, "verify", None)
        if verify is not None:
            verify(bt)
        self.source.commit(bt)
        self.history.append(metrics)
        if self.on_batch:
            self.on_batch(bt, metrics)


def _fmt_batch_time(bt_us: int) -> str:
    """Spark ``Time.toString``: ``<ms> ms``."""
    return f"{bt_us // 1000} ms"


_TOKEN = re.compile(r"\{([^}]+)\}")


def _java_fmt_to_strftime(fmt: str) -> str:
    out = fmt
    for j, p in (("yyyy", "%Y"), ("MM", "%m"), ("dd", "%d"), ("HH", "%H"), ("mm", "%M"), ("ss", "%S")):
        out = out.replace(j, p)
    return out


def expand_path_template(template: str, start: _dt.datetime, end: _dt.datetime,
                         increment: _dt.timedelta) -> List[str]:
    """``wasbs://c@a/{yyyy-MM-dd}/{HH}/*.json`` → one path per time partition in [start, end]."""
    return [p for p, _t in expand_path_prefixes(template, start, end, increment)]


def expand_path_prefixes(template: str, start: _dt.datetime, end: _dt.datetime,
                         increment: _dt.timedelta) -> List[Tuple[str, _dt.datetime]]:
    """(path, partition time) per distinct time partition of ``template`` in [start, end], stepping by
    ``increment`` (BlobBatchingHost.getInputBlobPathPrefixes, BlobBatchingHost.scala:28-53).  A template without a
    ``{…}`` date pattern is one path stamped now, as the reference."""
    if not _TOKEN.search(template):
        return [(template, _dt.datetime.utcnow())]
    out = []
    t = start
    seen = set()
    while t <= end:
        p = _TOKEN.sub(lambda m: t.strftime(_java_fmt_to_strftime(m.group(1))), template)
        if p not in seen:
            seen.add(p)
            out.append((p, t))
        t += increment
    return out


class BlobBatchingHost:
    """Batch mode (BatchApp → BlobBatchingHost.runBatchApp, BlobBatchingHost.scala:68-105): expand every input
    blob's path template over its time range, list the files under every partition prefix (``fs.list_matching`` —
    local folders, globs and ``wasbs://`` containers alike), and process ALL of them as ONE batch stamped with the
    earliest partition time and a 1-hour interval.

    With W ranks each file is read by exactly one rank (``fs.owned_by_rank``), as Spark spreads ``makeRDD(files)``
    over executors; the batch's metrics are all-reduced by the processor, so ``InputBlobs`` counts every file once.
    ``blobs``: (path template, start, end, partition increment) per configured input blob."""

    def __init__(self, processor: Processor, device, path_templates: List[str], start: _dt.datetime = None,
                 end: _dt.datetime = None, increment: _dt.timedelta = None,
                 blobs: Optional[List[Tuple[str, _dt.datetime, _dt.datetime, _dt.timedelta]]] = None):
        self.processor = processor
        self.device = device
        specs = list(blobs or []) + [(tpl, start, end, increment) for tpl in path_templates]
        self.prefixes = [pt for tpl, s, e, inc in specs for pt in expand_path_prefixes(tpl, s, e, inc)]
        self.paths = [p for p, _t in self.prefixes]

    def list_files(self) -> List[str]:
        seen, out = set(), []
        for p, _t in self.prefixes:
            for f in fs.list_matching(p):
                if f not in seen:
                    seen.add(f)
                    out.append(f)
        return out

    def run(self) -> List[Dict[str, float]]:
        from .. import parallel as P
        from ..io.sources import frame_bytes
        from ..telemetry.appinsights import track_event
        track_event("batch/app/begin")
        t0 = time.perf_counter()
        files = self.list_files()
        mine = fs.owned_by_rank(files, P.rank(), P.world())
        data = bytearray()
        for f in mine:
            b = fs.read_bytes(f)
            if b:
                data += b if b.endswith(b"\n") else b + b"\n"
        raw = frame_bytes(bytes(data), self.device, file_info={"inputPath": ";".join(mine)} if mine else None)
        t_min = min((t for _p, t in self.prefixes), default=_dt.datetime.utcnow())
        bt = int(t_min.replace(tzinfo=_dt.timezone.utc).timestamp() * 1e6)
        m = self.processor.process_batch(raw, bt, 3600 * 1_000_000)
        m = self.processor.drain() or m
        m["InputBlobs"] = float(len(files))
        m["BatchProcessedET"] = time.perf_counter() - t0      # CommonProcessorFactory.scala:509-513
        track_event("batch/end", properties=None, measurements=m)
        return [m]
