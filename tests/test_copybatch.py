"""Batched device copies (dxa/ops/csrc/copy_batch.hip) and the one-launch table concatenation built on them,
against torch.cat of the same tensors."""
import pytest
import torch

from dxa.engine.column import PrimColumn, Table, concat_tables, strings_from_pylist


@pytest.mark.gpu
def test_copy_batch_segments_and_fills():
    from dxa.ops.copybatch import copy_batch
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(3)
    srcs = [torch.randint(0, 255, (n,), generator=g, dtype=torch.uint8).to(dev) for n in (1, 7, 16, 33, 70_000,
                                                                                          200_003)]
    total = sum(s.numel() for s in srcs) + 5 + 64
    dst = torch.zeros(total, dtype=torch.uint8, device=dev)
    segs, pos, want = [], 0, []
    for s in srcs:
        segs.append((s, 0, dst, pos, s.numel(), 0))
        want.append(s.cpu())
        pos += s.numel()
    segs.append((None, 0, dst, pos, 5, 0xAB))            # a fill
    want.append(torch.full((5,), 0xAB, dtype=torch.uint8))
    pos += 5
    segs.append((srcs[4], 3, dst, pos, 64, 0))            # an unaligned slice
    want.append(srcs[4][3:67].cpu())
    copy_batch(segs, dev)
    assert torch.equal(dst.cpu(), torch.cat(want))


@pytest.mark.gpu
def test_concat_tables_one_launch_matches_cat():
    from launch_count import count_launches
    dev = torch.device("cuda")
    tabs = []
    for k, n in enumerate((3, 0, 1000, 17, 4096)):
        a = PrimColumn("long", torch.arange(n, device=dev) * (k + 1))
        b = PrimColumn("double", torch.rand(n, dtype=torch.float64, device=dev),
                       None if k % 2 else torch.rand(n, device=dev) > 0.3)
        c = PrimColumn("boolean", torch.rand(n, device=dev) > 0.5)
        w = PrimColumn("decimal(38,2)", torch.randint(-99, 99, (n, 2), device=dev))
        tabs.append(Table(["a", "b", "c", "w"], [a, b, c, w], n, dev))
    with count_launches() as log:
        out = concat_tables(tabs)
    assert log.count("dxa_copy_batch") == 1 and not any(x.startswith("cat") for x in log), log
    for j, nm in enumerate(["a", "b", "c", "w"]):
        want = torch.cat([t.columns[j].data for t in tabs])
        assert torch.equal(out.columns[j].data, want), nm
    vb = torch.cat([t.columns[1].valid_mask() for t in tabs])
    assert torch.equal(out.columns[1].valid, vb)
    assert out.columns[0].valid is None and out.length == sum(t.length for t in tabs)


def test_concat_tables_cpu_strings_and_prims():
    t1 = Table(["s", "x"], [strings_from_pylist(["a", None], "cpu"), PrimColumn("long", torch.tensor([1, 2]))], 2, "cpu")
    t2 = Table(["s", "x"], [strings_from_pylist(["bb"], "cpu"), PrimColumn("long", torch.tensor([3]),
                                                                     torch.tensor([False]))], 1)
    out = concat_tables([t1, t2])
    assert out.columns[0].to_pylist() == ["a", None, "bb"] and out.columns[1].to_pylist() == [1, 2, None]


@pytest.mark.gpu
def test_concat_tables_with_strings_matches_cpu():
    dev = torch.device("cuda")
    rows = [[("a", 1), (None, 2), ("héllo", 3)], [], [("x" * 40, 4)], [("", None), ("zz", 6)]]
    tabs_g, tabs_c = [], []
    for r in rows:
        s = [x[0] for x in r]
        v = [x[1] for x in r]
        from dxa.engine.column import column_from_pylist
        for dev_, out in ((dev, tabs_g), ("cpu", tabs_c)):
            out.append(Table(["s", "v"], [strings_from_pylist(s, dev_), column_from_pylist(v, "long", dev_)],
                             len(r), dev_))
    g, c = concat_tables(tabs_g), concat_tables(tabs_c)
    assert g.columns[0].to_pylist() == c.columns[0].to_pylist() == ["a", None, "héllo", "x" * 40, "", "zz"]
    assert g.columns[1].to_pylist() == c.columns[1].to_pylist()


def test_chunk_rows_split_segments_cpu():
    """Chunking of copy / fill segments into per-workgroup rows (host side of copy_batch): every byte of every
    segment covered exactly once, fills keep a null source, no row over the chunk size."""
    import numpy as np
    from dxa.ops.copybatch import chunk_rows
    src = np.array([1000, 0, 5000, 9000], dtype=np.int64)
    dst = np.array([100000, 200000, 300000, 400000], dtype=np.int64)
    nb = np.array([10, 25, 7, 16], dtype=np.int64)
    fill = np.array([0, 1, 0, 0], dtype=np.int64)
    rows = chunk_rows(src, dst, nb, fill, 8)
    assert (rows[:, 2] <= 8).all() and (rows[:, 2] > 0).all()
    for k in range(4):
        mine = rows[(rows[:, 1] >= dst[k]) & (rows[:, 1] < dst[k] + nb[k])]
        assert mine[:, 2].sum() == nb[k]
        assert sorted(mine[:, 1] - dst[k]) == list(range(0, nb[k], 8))
        if src[k] == 0:
            assert (mine[:, 0] == 0).all() and (mine[:, 3] == 1).all()
        else:
            assert (mine[:, 0] - src[k] == mine[:, 1] - dst[k]).all()
    one = chunk_rows(src, dst, nb, fill, 64)
    assert one.shape == (4, 4) and (one[:, 2] == nb).all()


def test_segments_accumulate_scalars_lists_and_arrays_cpu():
    """Segments.add takes scalars (repeated per segment), lists and numpy arrays; launch converts once."""
    import numpy as np
    from dxa.ops.copybatch import Segments
    sg = Segments()
    sg.add(0, 100, 8, 1)                                     # one fill segment
    sg.add([10, 20], np.array([200, 300]), np.array([4, 0]))  # two copies, one empty
    sg.add(np.array([5]), 400, [16], np.array([0]))
    assert sg.src == [0, 10, 20, 5] and sg.dst == [100, 200, 300, 400]
    assert sg.nb == [8, 4, 0, 16] and sg.fill == [1, 0, 0, 0]
    assert all(isinstance(v, int) for v in sg.src + sg.dst + sg.nb + sg.fill)
