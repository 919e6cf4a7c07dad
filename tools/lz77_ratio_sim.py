"""What ratio would a device gzip design reach?  A model of the one-wave-per-chunk deflate parse (deflate.hip) run
on SimulatedData JSON on the CPU: per-chunk members or chunks primed with the preceding bytes (one gzip member per
file), hash heads updated per 64-position group, 1..16-way buckets, greedy or lazy (one-step) matching.  The coded
size is the Shannon length of each chunk's literal/length and distance symbols plus extra bits and a dynamic-table
header — close to deflate's dynamic Huffman cost.  profiles/round6/gzip/README.md lists its output.

    python tools/lz77_ratio_sim.py"""
import sys, math, zlib, collections, torch
sys.path.insert(0, ".")
from dxa.models import iot
from dxa.simulate.datagen import generate
buf, offs = generate(iot.program(newline=True), 4000, torch.device("cpu"), seed=1, row0=0, base_ms=1_700_000_000_000)
data = bytes(buf[:int(offs[-1])].numpy())

def len_code(l):
    x = l - 3
    if l == 258: return 285, 0
    if x < 8: return 257 + x, 0
    hb = x.bit_length() - 1; eb = hb - 2
    return 257 + 4 * (hb - 1) + ((x >> eb) & 3), eb
def dist_code(d):
    y = d - 1
    if y < 4: return y, 0
    hb = y.bit_length() - 1; eb = hb - 1
    return 2 * hb + ((y >> eb) & 1), eb

def h4(b, p): return ((int.from_bytes(b[p:p+4], "little") * 2654435761) & 0xffffffff)
def mlen(b, a, p, end):
    n = 0; lim = min(258, end - p)
    while n < lim and b[a + n] == b[p + n]: n += 1
    return n

def parse(chunk_bytes, start, end, hbits, ways, lazy):
    """positions [start, end) of chunk_bytes are coded; [0, start) is history."""
    b = chunk_bytes
    H = 1 << hbits
    heads = [[-1] * ways for _ in range(H)]
    def ins(p):
        h = h4(b, p) >> (32 - hbits)
        hs = heads[h]; hs.insert(0, p); hs.pop()
    # history: insert all history positions
    for p in range(0, start - 3):
        ins(p)
    toks = []
    p = start
    g0 = start
    pending = []
    # group semantics: heads updated at group end (lookup sees earlier groups only)
    cand_cache = {}
    def cands(p):
        h = h4(b, p) >> (32 - hbits)
        return [c for c in heads[h] if c >= 0 and p - c <= 32768]
    group_start = start
    group_cands = {}
    def load_group(gs):
        group_cands.clear()
        for q in range(gs, min(gs + 64, end)):
            if q + 4 <= end:
                group_cands[q] = cands(q)
        for q in range(gs, min(gs + 64, end)):
            if q + 4 <= end: ins(q)
    load_group(group_start)
    def best(q):
        while q >= group_start + 64:
            pass
        cs = group_cands.get(q, [])
        bl, bc = 0, -1
        for c in cs:
            if b[c:c+4] == b[q:q+4]:
                l = mlen(b, c, q, end)
                if l > bl: bl, bc = l, c
        return bl, bc
    while p < end:
        while p >= group_start + 64:
            group_start += 64
            load_group(group_start)
        l, c = best(p)
        if l >= 4 and lazy and p + 1 < end:
            if p + 1 >= group_start + 64:
                l2 = 0
            else:
                l2, c2 = best(p + 1)
            if l2 > l:
                toks.append(("L", b[p])); p += 1; continue
        if l >= 4:
            toks.append(("M", l, p - c)); p += l
        else:
            toks.append(("L", b[p])); p += 1
    return toks

def cost(toks):
    ll = collections.Counter(); dd = collections.Counter(); extra = 0
    for t in toks:
        if t[0] == "L": ll[t[1]] += 1
        else:
            s, e = len_code(t[1]); ll[s] += 1; extra += e
            dc, de = dist_code(t[2]); dd[dc] += 1; extra += de
    ll[256] += 1
    def shannon(c):
        tot = sum(c.values()); return sum(f * max(1, math.ceil(math.log2(tot / f))) for f in c.values())
    return (shannon(ll) + shannon(dd) + extra + 17 + 57 + 4 * 300) / 8

def run(member, prime, hbits, ways, lazy):
    tot = 0
    for s in range(0, len(data), member):
        h0 = max(0, s - prime)
        seg = data[h0:s + member]
        toks = parse(seg, s - h0, len(seg), hbits, ways, lazy)
        tot += cost(toks) + (18 if prime == 0 else 5)
    return len(data) / tot

print("bytes", len(data))
for member, prime, hb, ways, lazy in [(8192, 0, 11, 1, False), (16384, 0, 11, 1, False), (32768, 0, 11, 1, False),
                                       (16384, 16384, 11, 1, False), (16384, 16384, 12, 1, False),
                                       (16384, 16384, 12, 1, True), (16384, 16384, 12, 2, False),
                                       (16384, 16384, 12, 2, True), (16384, 16384, 12, 4, True),
                                       (32768, 32768, 12, 2, True)]:
    print(member, prime, hb, ways, lazy, round(run(member, prime, hb, ways, lazy), 3), flush=True)
for member, prime, hb, ways, lazy in [(16384, 16384, 12, 8, True), (16384, 32768, 12, 4, True), (16384, 32768, 13, 8, True),
                                       (16384, 16384, 11, 4, True), (16384, 16384, 11, 8, True), (16384, 16384, 11, 16, True)]:
    print(member, prime, hb, ways, lazy, round(run(member, prime, hb, ways, lazy), 3), flush=True)
