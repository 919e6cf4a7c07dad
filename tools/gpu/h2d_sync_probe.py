"""Does a small pageable host→device copy block the host until the stream drains?  A ~20 ms spin kernel is queued,
then one 64-byte upload is timed (pageable .to(), pinned non_blocking .to(), torch.tensor(list, device=cuda))."""
import time

import torch

dev = torch.device("cuda", 0)
x = torch.zeros(1, device=dev)
torch.cuda.synchronize()
b = bytearray(64)


def spin():
    torch.cuda._sleep(int(2.4e9 * 0.02))      # ~20 ms of GPU cycles


for name, fn in [("pageable frombuffer.to", lambda: torch.frombuffer(b, dtype=torch.uint8).to(dev)),
                 ("pageable non_blocking", lambda: torch.frombuffer(b, dtype=torch.uint8).to(dev, non_blocking=True)),
                 ("torch.tensor(list, device)", lambda: torch.tensor(list(range(8)), device=dev)),
                 ("pinned non_blocking", lambda: torch.frombuffer(b, dtype=torch.uint8).pin_memory().to(
                     dev, non_blocking=True)),
                 ("tensor.item() (reference sync)", lambda: x.item())]:
    for rep in range(3):
        spin()
        t0 = time.perf_counter()
        fn()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
    print(f"{name:34s} host call {1e3 * (t1 - t0):7.3f} ms   rest of spin {1e3 * (t2 - t1):7.3f} ms", flush=True)
