"""Host-side NUMA placement for one-process-per-GPU jobs.

On a multi-socket MI355X node each GPU hangs off one socket's PCIe root.  Pinned host buffers (ingest frames, output
staging) are allocated by first touch, so a rank whose threads run on the far socket stages every H2D/D2H byte
across the inter-socket fabric — with eight ranks streaming ~50 GB/s each that link, not PCIe, becomes the limit.
``bind_to_device`` restricts the calling process to the CPUs local to its GPU (sysfs ``local_cpulist`` of the GPU's
PCI function) before any pinned buffer exists.  Everything here is best effort: missing sysfs entries, containers
without the right to change affinity, or CPU-only runs leave the process untouched.
"""
from __future__ import annotations

import os
from typing import Optional, Set


def parse_cpulist(text: str) -> Set[int]:
    """``"0-3,8,10-11"`` → {0, 1, 2, 3, 8, 10, 11}."""
    cpus: Set[int] = set()
    for part in text.strip().split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            lo, hi = part.split("-", 1)
            cpus.update(range(int(lo), int(hi) + 1))
        else:
            cpus.add(int(part))
    return cpus


def _visible_indices() -> Optional[list]:
    """Physical GPU ordinals exposed to this process (``ROCR_VISIBLE_DEVICES`` applies first, then
    ``HIP_VISIBLE_DEVICES`` / ``CUDA_VISIBLE_DEVICES`` index into what is left); None = all."""
    vis = None
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is None or not v.strip():
            continue
        try:
            ids = [int(x) for x in v.split(",") if x.strip()]
        except ValueError:               # UUID forms: give up on the sysfs mapping
            return None
        vis = ids if vis is None else [vis[i] for i in ids if i < len(vis)]
    return vis


def kfd_pci_path(index: int, topology: str = "/sys/class/kfd/kfd/topology/nodes",
                 pci_root: str = "/sys/bus/pci/devices") -> Optional[str]:
    """PCI sysfs folder of HIP device ``index`` from the KFD topology alone (no HIP call, so it can run before the
    runtime starts any thread): GPU nodes are those with SIMDs, in node order; ``location_id`` packs
    bus/device/function as ``bus << 8 | dev << 3 | fn``."""
    try:
        nodes = sorted((int(n) for n in os.listdir(topology) if n.isdigit()))
    except OSError:
        return None
    gpus = []
    for n in nodes:
        props = {}
        try:
            with open(os.path.join(topology, str(n), "properties")) as f:
                for line in f:
                    k, _, v = line.partition(" ")
                    props[k] = v.strip()
        except OSError:
            continue
        if int(props.get("simd_count", "0") or 0) > 0:
            gpus.append(props)
    vis = _visible_indices()
    if vis is not None:
        gpus = [gpus[i] for i in vis if i < len(gpus)]
    if index >= len(gpus):
        return None
    g = gpus[index]
    try:
        loc, dom = int(g.get("location_id", "")), int(g.get("domain", "0") or 0)
    except ValueError:
        return None
    bdf = f"{dom:04x}:{loc >> 8:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 7}"
    path = os.path.join(pci_root, bdf)
    return path if os.path.isdir(path) else None


def device_pci_path(index: int) -> Optional[str]:
    path = kfd_pci_path(index)
    if path is not None:
        return path
    import torch
    try:
        p = torch.cuda.get_device_properties(index)
        bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
    except Exception:
        return None
    path = f"/sys/bus/pci/devices/{bdf}"
    return path if os.path.isdir(path) else None


def local_cpus(index: int) -> Optional[Set[int]]:
    path = device_pci_path(index)
    if path is None:
        return None
    try:
        with open(os.path.join(path, "local_cpulist")) as f:
            cpus = parse_cpulist(f.read())
    except (OSError, ValueError):
        return None
    return cpus or None


def bind_to_device(index: int) -> Optional[Set[int]]:
    """Pin this process to the CPUs local to GPU ``index`` (intersected with the CPUs it may use now).

    Call it before ``torch.cuda.set_device`` / ``init_process_group``: Linux affinity is per thread and new threads
    inherit their creator's mask, so binding first places the HIP runtime's and RCCL's helper threads (and the
    pinned buffers they first-touch) on the GPU's socket.  Threads that already exist are re-bound too (every task
    of ``/proc/self/task``).  Returns the CPU set the process runs on (also when it already matched), or None when
    the local CPUs are unknown or binding is disabled (``DXA_NUMA_BIND=0``)."""
    if os.environ.get("DXA_NUMA_BIND", "1") == "0" or not hasattr(os, "sched_setaffinity"):
        return None
    cpus = local_cpus(index)
    if not cpus:
        return None
    allowed = os.sched_getaffinity(0)
    want = cpus & allowed
    if not want:
        return None
    if want == allowed:
        return want
    try:
        os.sched_setaffinity(0, want)
    except OSError:
        return None
    try:
        tids = [int(t) for t in os.listdir("/proc/self/task")]
    except OSError:
        tids = []
    for tid in tids:
        try:
            os.sched_setaffinity(tid, want)
        except OSError:
            pass
    return want


def host_threads(index: int, local_world: int = 1, cap: int = 16, floor: int = 2) -> int:
    """Worker threads one rank should start for host-side batch work (Kafka batch planning, CRC checks).

    Ranks whose GPUs share a socket are bound to the same CPU set (``bind_to_device``), so each takes its share:
    ``len(cpus) // ranks on that set``, clamped to [floor, cap].  With 8 ranks on a 2-socket node, 4 ranks per socket
    each start cpus/4 planner threads instead of all of them starting ``cap`` and oversubscribing the socket."""
    try:
        cpus = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        cpus = os.cpu_count() or floor
    mine = local_cpus(index)
    share = 1
    if mine and local_world > 1:
        share = sum(1 for j in range(local_world) if local_cpus(j) == mine) or 1
    elif local_world > 1:
        share = local_world
    return max(floor, min(cap, cpus // share))


# Host CRC-32C capacity, measured on an MI355X box (profiles/round6/host8/README.md): ~9 GB/s per planner thread
# when 16 threads check concurrently (11.5 GB/s for one), and the PCIe-bound ingest one rank checks (57 GB/s).
CRC_GBS_PER_THREAD = 9.0
INGEST_GBS_PER_RANK = 57.0
# Host memory traffic a node's ranks may spend on ingest: every host-checked byte is read twice (the CRC, then the
# DMA to the GPU).  1000 GB/s is ~85 % of a 2-socket DDR5-6400 node's peak; the 1-GPU box gives no way to measure the
# whole node (its 16-CPU share checked 144 GB/s without saturating), so it is a setting, not a measurement.
HOST_INGEST_BUDGET_GBS = 1000.0


def crc_placement(local_rank: int, local_world: int, threads: int, budget_gbs: float = HOST_INGEST_BUDGET_GBS,
                  need_gbs: float = INGEST_GBS_PER_RANK, per_thread_gbs: float = CRC_GBS_PER_THREAD) -> str:
    """``check.crcs=auto``: where the node's ranks check their Kafka batches' CRC-32C.

    The ranks of a job step in lockstep (every batch ends in collectives), so the slowest rank sets everyone's pace
    and all ranks of a node take the same decision:

    * ``"host"`` when a rank's planner threads check at its ingest rate (threads x per-thread rate ≥ the need) and
      the node's host memory budget covers every local rank's two reads of its ingest (CRC + DMA);
    * ``"device"`` otherwise — the GPU kernel costs ~20 % of a PCIe-bound step (profiles/crc/README.md), less than
      a starved host planner would."""
    if threads * per_thread_gbs < need_gbs:
        return "device"
    return "host" if local_world * 2.0 * need_gbs <= budget_gbs else "device"
