"""Engine entry point — one process per MI355X (the reference's DirectStreamingApp / DirectLocalStreamingApp /
DirectKafkaStreamingApp / BlobStreamingApp / BatchApp ``main``s, DataProcessing/datax-host/src/main/scala/datax/app/*).

    python -m dxa.app conf=/path/job.conf [app=local|file|socket|queue|batch] [maxBatches=N] [realtime=false]
            [driverLogLevel=WARN] [checkpointEnabled=true]
    # multi-GPU: python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 -m dxa.app conf=…

Arguments follow the reference's ``k=v`` convention; ``DATAX_*`` environment variables are merged
(ConfigManager.scala:61-81).  Batch mode takes ``processStartTime=… processEndTime=… partitionIncrement=<minutes>``
and ``datax.job.input.default.blob.<name>.path`` templates.
"""
from __future__ import annotations

import datetime as _dt
import json
import logging
import os
import sys


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    import torch
    from .config import settings as S
    d = S.settings_from_arguments(argv)
    d = S.load_config(d)
    args = S.named_args(argv)
    logging.basicConfig(level=getattr(logging, (args.get("driverLogLevel") or "WARN").upper(), logging.WARN),
                        format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if torch.cuda.device_count() > local:
        from .parallel.affinity import bind_to_device
        bind_to_device(local)                  # before the HIP runtime starts threads: they inherit the mask
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
        from .ops import native
        native.lib()
    else:
        device = torch.device("cpu")
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl" if device.type == "cuda" else "gloo")
        from . import parallel
        parallel.init(dist.group.WORLD, device)
    from .engine.host import BlobBatchingHost, StreamingHost
    from .engine.processor import Processor
    from .io.sources import build_source
    from .telemetry.metrics import MetricStore
    from .telemetry import appinsights
    appinsights.configure(d)
    proc = Processor(d, device, metric_store=MetricStore.default())
    app = (args.get("app") or "").lower() or None
    if app == "batch":
        from .config.secrets import resolve
        from .service.scheduler import _parse_time
        blobs = list(d.group_by_sub_namespace(S.INPUT_PREFIX + "blob.").values())
        # per input blob: its own path template, time range and partition increment (BatchBlobInputSetting.scala:
        # 18-48); ``processStartTime=`` / ``processEndTime=`` / ``partitionIncrement=`` arguments override all
        specs = []
        for sub in blobs:
            s0 = _parse_time(args.get("processStartTime") or sub.get("processstarttime"))
            s1 = _parse_time(args.get("processEndTime") or sub.get("processendtime"))
            step = _dt.timedelta(minutes=float(args.get("partitionIncrement") or sub.get("partitionincrement") or 60))
            specs.append((resolve(sub.get_string("path")), s0, s1, step))
        res = BlobBatchingHost(proc, device, [], blobs=specs).run()
        print(json.dumps({"batches": len(res)}), flush=True)
        return 0
    src = build_source(d, device, app)
    interval = float(d.get(S.INPUT_PREFIX + "streaming.intervalinseconds") or 60)
    host = StreamingHost(proc, src, interval, int(args["maxBatches"]) if "maxBatches" in args else None,
                         realtime=(args.get("realtime", "true").lower() == "true"))
    import signal
    signal.signal(signal.SIGTERM, lambda *_: host.stop())
    hist = host.run()
    if int(os.environ.get("RANK", "0")) == 0:
        print(json.dumps({"batches": len(hist), "last": hist[-1] if hist else None}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
