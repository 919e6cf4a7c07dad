"""H2D bandwidth of the ingest copy on one MI355X: hipMemcpyAsync from pinned memory (what the Kafka / LZ4 ingest
uses; runs as the __amd_rocclr_copyBuffer blit kernel) vs the ROCr async copy on an SDMA engine (dxa_copy_sdma), and
the same copy while a compute kernel occupies the CUs.  Prints one JSON line per case."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from dxa.ops import native as N  # noqa: E402

dev = torch.device("cuda:0")
L = N.lib()
MB = 1 << 20
for total_mb, chunks in ((441, 4), (441, 1), (64, 1)):
    n = total_mb * MB
    host = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    host.random_(0, 255)
    dst = torch.empty(n, dtype=torch.uint8, device=dev)
    s = torch.cuda.Stream(dev)
    step = n // chunks
    res = {"bytes_mb": total_mb, "chunks": chunks}
    for rep in range(2):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for k in range(chunks):
            N.call("dxa_memcpy_h2d_async", dst.data_ptr() + k * step, host.data_ptr() + k * step, step, s.cuda_stream)
        s.synchronize()
        res["hip_memcpy_gbs"] = round(n / (time.perf_counter() - t) / 1e9, 1)
        t = time.perf_counter()
        for k in range(chunks):
            rc = L.dxa_copy_sdma(dst.data_ptr() + k * step, host.data_ptr() + k * step, step)
            assert rc == 0, rc
        res["sdma_gbs"] = round(n / (time.perf_counter() - t) / 1e9, 1)
    assert torch.equal(dst[:4096].cpu(), host[:4096])
    # concurrency: the copy while a long compute kernel runs on the default stream
    a = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(20):
        a @ a
    torch.cuda.synchronize()
    res["gemm_alone_ms"] = round((time.perf_counter() - t) * 1e3, 2)
    t = time.perf_counter()
    for _ in range(20):
        a @ a
    for k in range(chunks):
        N.call("dxa_memcpy_h2d_async", dst.data_ptr() + k * step, host.data_ptr() + k * step, step, s.cuda_stream)
    torch.cuda.synchronize()
    res["gemm_plus_blit_copy_ms"] = round((time.perf_counter() - t) * 1e3, 2)
    t = time.perf_counter()
    for _ in range(20):
        a @ a
    for k in range(chunks):
        L.dxa_copy_sdma(dst.data_ptr() + k * step, host.data_ptr() + k * step, step)
    torch.cuda.synchronize()
    res["gemm_plus_sdma_copy_ms"] = round((time.perf_counter() - t) * 1e3, 2)
    print(json.dumps(res), flush=True)
