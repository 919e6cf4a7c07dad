"""Device sort (radix_sort.hip via dxa.ops.sort): multi-word stable argsort, SQL order keys and string ranks —
the CPU path (plain torch) is checked against Python's sort here; the GPU tests compare the kernels with the CPU
path on the same inputs."""
import math
import random
import struct

import pytest
import torch

from dxa.engine.column import strings_from_pylist
from dxa.ops import sort as SO


def _u64(x):
    return x - (1 << 64) if x >= (1 << 63) else x


def _py_argsort_words(words):
    n = len(words[0])
    keys = [tuple((w[i] & ((1 << 64) - 1)) for w in reversed(words)) for i in range(n)]
    return sorted(range(n), key=lambda i: keys[i])


def _random_words(n, nwords, seed, small=False):
    rnd = random.Random(seed)
    out = []
    for _ in range(nwords):
        if small:
            vals = [rnd.randint(0, 5) for _ in range(n)]
        else:
            vals = [_u64(rnd.getrandbits(64)) if rnd.random() < 0.7 else rnd.choice([0, -1, 1 << 40, -(1 << 63)])
                    for _ in range(n)]
        out.append(vals)
    return out


@pytest.mark.parametrize("n,nwords,small", [(1, 1, False), (37, 2, True), (5000, 1, False), (9000, 3, True)])
def test_argsort_words_cpu_matches_python(n, nwords, small):
    words = _random_words(n, nwords, n + nwords, small)
    perm = SO.argsort_words([torch.tensor(w, dtype=torch.int64) for w in words]).tolist()
    assert perm == _py_argsort_words(words)          # stable: ties keep input order


def test_order_keys_cpu():
    ints = [5, -3, 0, 2**62, -(2**63), 2**63 - 1, -1]
    k = SO.order_key(torch.tensor(ints), "int")
    assert SO.argsort_words([k]).tolist() == sorted(range(len(ints)), key=lambda i: ints[i])
    kd = SO.order_key(torch.tensor(ints), "int", descending=True)
    assert SO.argsort_words([kd]).tolist() == sorted(range(len(ints)), key=lambda i: -ints[i])
    fl = [1.5, -0.0, 0.0, float("nan"), float("inf"), -float("inf"), -2.25, 1e-300, -1e300]
    k = SO.order_key(torch.tensor(fl, dtype=torch.float64), "float")
    order = SO.argsort_words([k]).tolist()
    # Spark: NaN is the largest value; -0.0 == 0.0 (stable: input order kept)
    spark_key = [(1, 0.0) if math.isnan(v) else (0, v + 0.0) for v in fl]
    assert order == sorted(range(len(fl)), key=lambda i: spark_key[i])


def _strings(seed, n):
    rnd = random.Random(seed)
    base = ["", "a", "ab", "ab\x00", "abcdefgh", "abcdefghi", "abcdefgh\x00", "abcdefghijklmnopqrstu",
            "abcdefghijklmnopqrstv", "zz", "Zebra", "é", "éa", "ÿ", "ÿ" * 20]
    out = []
    for _ in range(n):
        r = rnd.random()
        if r < 0.5:
            out.append(rnd.choice(base))
        elif r < 0.6:
            out.append(None)
        else:
            out.append("".join(rnd.choice("ab\x00é") for _ in range(rnd.randint(0, 30))))
    return out


@pytest.mark.parametrize("seed,n", [(1, 1), (2, 50), (3, 3000)])
def test_string_ranks_cpu_match_python(seed, n):
    vals = _strings(seed, n)
    col = strings_from_pylist(vals, "cpu")
    ranks = SO.string_ranks(col).tolist()
    nn = [i for i, v in enumerate(vals) if v is not None]
    distinct = sorted({vals[i].encode() for i in nn})
    want = {b: r for r, b in enumerate(distinct)}
    assert [ranks[i] for i in nn] == [want[vals[i].encode()] for i in nn]


@pytest.mark.gpu
@pytest.mark.parametrize("n,nwords,small", [(1, 1, False), (4095, 1, False), (4097, 2, True), (300000, 2, False),
                                            (1_000_003, 1, True)])
def test_gpu_radix_argsort_matches_cpu(n, nwords, small):
    assert torch.cuda.is_available()
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(n)
    words = []
    for j in range(nwords):
        if small:
            w = torch.randint(0, 7, (n,), generator=g, dtype=torch.int64)
        else:
            w = torch.randint(-(2**63), 2**63 - 1, (n,), generator=g, dtype=torch.int64)
            w[::5] = w[min(3, n - 1)]                       # duplicates: stability matters
        words.append(w)
    want = SO.argsort_words(words)
    got = SO.argsort_words([w.to(dev) for w in words]).cpu()
    assert torch.equal(got, want)


@pytest.mark.gpu
def test_gpu_order_keys_and_string_ranks_match_cpu():
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(3)
    f = torch.randn(100_000, generator=g, dtype=torch.float64) * 1e6
    f[::7] = float("nan")
    f[::11] = -0.0
    i = torch.randint(-(2**63), 2**63 - 1, (100_000,), generator=g, dtype=torch.int64)
    for data, kind in ((f, "float"), (i, "int")):
        for desc in (False, True):
            assert torch.equal(SO.order_key(data.to(dev), kind, desc).cpu(), SO.order_key(data, kind, desc))
    vals = _strings(7, 20000)
    cpu = SO.string_ranks(strings_from_pylist(vals, "cpu"))
    gpu = SO.string_ranks(strings_from_pylist(vals, dev)).cpu()
    nn = torch.tensor([v is not None for v in vals])
    assert torch.equal(gpu[nn], cpu[nn])
