"""Round 6: linear-probe chain lengths of the resident index (murr_index.hip's
key_hash restated in Python; rows inserted in order, where the GPU inserts
concurrently: the same occupied slots, chains of the same distribution) over
a bench's key sets:
mean / p99 / max probes per key and the mean / max of each 64-key group's
slowest key (a fused-gather workgroup waits for it).  Usage:
    python tools/r06/probe_chains.py 1000000 C     # config C, ~5 % misses
    python tools/r06/probe_chains.py 10000000 ref  # read_plain's keys (slow)
"""
import numpy as np
M64 = (1 << 64) - 1
def khash(b):
    n = len(b)
    w = np.zeros(8, np.uint32)
    p = b + b"\0" * (32 - n)
    w[:] = np.frombuffer(p[:32], np.uint32)
    h = 0xcbf29ce484222325 ^ n
    for j in range(8):
        h = ((h ^ int(w[j])) * 0x100000001b3) & M64
    h ^= h >> 33; h = (h * 0xff51afd7ed558ccd) & M64
    h ^= h >> 33; h = (h * 0xc4ceb9fe1a85ec53) & M64
    h ^= h >> 33
    return h
def run(n, kf, qf):
    cap = 1
    while cap < 2 * n: cap <<= 1
    mask = cap - 1
    occ = np.full(cap, -1, np.int64)
    home = {}
    for i in range(n):
        k = kf(i).encode(); s = khash(k) & mask
        while occ[s] != -1: s = (s + 1) & mask
        occ[s] = i
    res = []
    for rep in range(3):
        qs = qf(rep)
        it = []
        for k in qs:
            kb = k.encode(); s = khash(kb) & mask; c = 1
            while occ[s] != -1 and kf(int(occ[s])) != k:
                s = (s + 1) & mask; c += 1
            it.append(c)
        it = np.array(it)
        g = [it[i:i+64].max() for i in range(0, len(it), 64)]
        res.append((it.mean(), np.percentile(it, 99), it.max(), np.mean(g), max(g)))
    return cap, n / cap, res
import sys
n = int(sys.argv[1]); kind = sys.argv[2]
if kind == "C":
    kf = lambda i: f"key{i}"
    qf = lambda k: [f"key{int(i)}" for i in np.random.default_rng(44 + k).integers(0, int(n * 1.05), size=1000)]
else:
    kf = lambda i: str(i)
    qf = lambda k: [str(int(i)) for i in np.random.default_rng(1000 * 2_000_000 + k).integers(0, n, size=1000)]
print(kind, run(n, kf, qf))
