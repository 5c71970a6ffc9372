"""RocksDB data-block decode on the device (murr_sst_decode through the C ABI)
against the CPU restatement (oracle/murr_sst.c, itself checked against
pyarrow's Snappy / LZ4 codecs and the BlockBuilder restatement in
tests/sstgen.py): bit-exact keys, values, sequence numbers and types, the
first corrupt block named, and a table rehydrated from its SST blocks reading
exactly as the table it came from."""
import numpy as np
import pyarrow as pa
import pytest

import oracle as O
import sstgen as G
from murr_amd import SegmentError, sst
from murr_amd.resident import ResidentTable
from murr_amd.row import default_context

from test_gpu_resident import assert_same, batch_c, expected, schema_c

pytestmark = pytest.mark.gpu


def oracle_entries(stored):
    keys, vals, seqs, types = [], [], [], []
    for data, comp in stored:
        k, v, s, t = O.block_decode(O.block_contents(data, comp))
        keys += k
        vals += v
        seqs += s.tolist()
        types += t.tolist()
    return keys, vals, seqs, types


def check(stored):
    ctx = default_context()
    e = sst.decode_host(ctx, stored)
    keys, vals, seqs, types = e.to_host()
    wk, wv, ws, wt = oracle_entries(stored)
    assert e.n == len(wk)
    assert keys == wk
    assert vals == wv
    assert seqs.tolist() == ws
    assert types.tolist() == wt
    assert e.key_bytes == sum(map(len, wk)) and e.value_bytes == sum(map(len, wv))
    return e


@pytest.mark.parametrize("comp", [G.NONE, G.SNAPPY, G.LZ4])
@pytest.mark.parametrize("restart,hash_index", [(1, False), (8, True), (16, False)])
def test_blocks_bit_exact(comp, restart, hash_index):
    rng = np.random.default_rng(comp * 100 + restart + hash_index)
    entries = G.random_entries(rng, 3000, max_val=300, dup_p=0.2, del_p=0.1)
    blocks = G.blocks_of(entries, restart_interval=restart, hash_index=hash_index)
    check([(G.compress(b, comp), comp) for b in blocks])


def snappy_wrap(raw: bytes) -> bytes:
    """A Snappy stream of `raw` with a literal of length field 0xFFFFFFFF
    spliced in after the header (tag 0xFC: four length bytes).  The Snappy
    library computes len + 1 in 32 bits and reads an empty literal
    (tests/test_sst.py pins that against pyarrow's codec), so the block
    decodes as `raw` on the device too."""
    good = G.snappy(raw)
    hdr = G.varint32(len(raw))
    assert good.startswith(hdr)
    return hdr + b"\xfc\xff\xff\xff\xff" + good[len(hdr):]


def test_snappy_wrapped_literal_length_as_the_library():
    rng = np.random.default_rng(5)
    blocks = G.blocks_of(G.random_entries(rng, 300), restart_interval=8)
    check([(snappy_wrap(b) if i % 2 else G.snappy(b), G.SNAPPY) for i, b in enumerate(blocks)])


def test_mixed_compression_and_block_sizes():
    rng = np.random.default_rng(11)
    entries = G.random_entries(rng, 4000, max_key=60, max_val=2000, dup_p=0.1)
    stored = []
    for i, b in enumerate(G.blocks_of(entries, block_size=int(rng.integers(64, 16384)))):
        comp = (G.NONE, G.SNAPPY, G.LZ4, 5)[i % 4]  # 5 = LZ4HC, the same stored format
        stored.append((G.compress(b, comp if comp != 5 else G.LZ4), comp))
    check(stored)


def test_edge_blocks():
    empty = G.build_block([])
    one = G.build_block([(b"", 7, G.TYPE_VALUE, b"")])  # empty user key and value
    versions = G.build_block([(b"k", 100 - i, G.TYPE_VALUE, bytes([i]) * i) for i in range(30)])
    big = G.build_block([(b"big", 1, G.TYPE_VALUE, bytes(range(256)) * 400)])
    check([(empty, 0), (one, 0), (G.snappy(versions), 1), (G.lz4(big), 4), (G.snappy(empty), 1)])
    e = sst.decode_host(default_context(), [])
    assert e.n == 0


def test_long_keys_and_block_size_boundaries():
    # internal keys past the LDS key buffer (256 B), blocks at and around the
    # LDS slot tiers (1 KiB, 4 KiB uncompressed) and the thread-serial tier
    rng = np.random.default_rng(21)
    stored = []
    for klen in (240, 248, 249, 300, 1000):
        entries = sorted((bytes(rng.integers(97, 100, size=klen, dtype=np.uint8)) + b"%03d" % i, 9, 1, b"v" * i)
                         for i in range(12))
        stored.append((G.snappy(G.build_block(entries, restart_interval=4)), G.SNAPPY))
    for target in (1000, 1023, 1024, 1025, 2048, 4095, 4096, 4097, 5000):
        for comp in (G.NONE, G.SNAPPY, G.LZ4):
            e1 = [(b"a", 5, 1, b"")]
            base = len(G.build_block(e1 + [(b"b", 4, 1, b"")], hash_index=False))
            e2 = e1 + [(b"b", 4, 1, bytes(rng.integers(0, 256, size=target - base - 1, dtype=np.uint8)))]
            raw = G.build_block(e2, hash_index=False)
            assert abs(len(raw) - target) <= 2
            stored.append((G.compress(raw, comp), comp))
    check(stored)


def test_many_blocks_scan_carry():
    # > 1024 x 1024 blocks: the block scans run their multi-pass carry
    blk = G.snappy(G.build_block([(b"user-key-%d" % 7, 5, G.TYPE_VALUE, b"v" * 11)]))
    nb = 1024 * 1024 + 4321
    ctx = default_context()
    host = np.tile(np.frombuffer(blk, np.uint8), nb)
    buf = ctx.upload(np.concatenate([host, np.zeros(16, np.uint8)]))
    e = sst.decode(ctx, buf, [(i * len(blk), len(blk), 1) for i in range(nb)])
    assert e.n == nb and e.key_bytes == nb * 10 and e.value_bytes == nb * 11
    ko = e.key_offsets.download(4 * (nb + 1)).view(np.int32)
    vo = e.value_offsets.download(8 * (nb + 1)).view(np.uint64)
    assert np.array_equal(ko, np.arange(nb + 1, dtype=np.int32) * 10)
    assert np.array_equal(vo, np.arange(nb + 1, dtype=np.uint64) * 11)
    assert e.keys.download(e.key_bytes).tobytes() == b"user-key-7" * nb
    assert np.all(e.seqs.download(8 * nb).view(np.uint64) == 5)


@pytest.mark.parametrize("bad", ["truncated_snappy", "huge_len", "lz4_cut", "unknown_type", "footer", "varint",
                                 "shared"])
def test_first_corrupt_block_is_named(bad):
    rng = np.random.default_rng(3)
    blocks = G.blocks_of(G.random_entries(rng, 600), restart_interval=8)
    stored = [(G.snappy(b), G.SNAPPY) for b in blocks]
    assert len(stored) > 20
    raw = blocks[9]
    if bad == "truncated_snappy":
        broken = (G.snappy(raw)[:-3], G.SNAPPY)
    elif bad == "huge_len":
        # a length prefix of ~4 GiB no stream of this size can inflate to:
        # malformed before anything is allocated from it
        good = G.snappy(raw)
        broken = (G.varint32(0xFFFFFFF0) + good[len(G.varint32(len(raw))):], G.SNAPPY)
    elif bad == "lz4_cut":
        broken = (G.lz4(raw)[:-1], G.LZ4)
    elif bad == "unknown_type":
        broken = (raw, 7)  # ZSTD: not inflated on the device
    elif bad == "footer":
        broken = (raw[:-4] + (0x7FFFFFFF).to_bytes(4, "little"), G.NONE)
    elif bad == "varint":
        broken = (b"\xff\xff\xff\xff\xff\xff" + raw[6:], G.NONE)
    else:
        b = bytearray(raw)
        b[0] = 3  # a restart entry claiming shared bytes
        broken = (bytes(b), G.NONE)
    stored[9] = broken
    stored[15] = broken
    stored[4] = (raw, 7) if bad != "unknown_type" else (G.snappy(raw)[:-3], G.SNAPPY)  # another pass's error
    with pytest.raises(SegmentError, match=r"malformed.*row 4,"):
        sst.decode_host(default_context(), stored)
    stored[4] = (G.snappy(blocks[4]), G.SNAPPY)
    with pytest.raises(SegmentError, match=r"row 9,"):
        sst.decode_host(default_context(), stored)


def test_rehydrate_resident_table_from_sst():
    src = ResidentTable(schema_c())
    b0 = batch_c(6000, seed=42)
    src.write(b0)
    arena = src.arena.download(src.used).tobytes()
    offs = src.row_off.download(8 * (src.n + 1)).view(np.uint64)
    keys = b0.column(0).to_pylist()
    order = sorted(range(len(keys)), key=lambda i: keys[i].encode())
    entries = [(keys[i].encode(), 1000 + i, G.TYPE_VALUE, arena[offs[i]:offs[i + 1]]) for i in order]
    stored = [(G.snappy(b), G.SNAPPY) for b in G.blocks_of(entries)]
    t = ResidentTable(schema_c())
    t.load_sst(sst.decode_host(t.ctx, stored))
    rng = np.random.default_rng(8)
    q = [f"key{i}" for i in rng.integers(0, 6500, size=2000)]
    cols = [f"c{i}" for i in range(16)]
    assert_same(t.read(q, cols), expected([b0], q, cols))
    # appends after a rehydration grow the adopted arena
    b1 = batch_c(500, start=5900, seed=7)
    t.write(b1)
    assert_same(t.read(q, cols), expected([b0, b1], q, cols))


def test_rehydrate_rejects_tombstones():
    blk = G.build_block([(b"a", 2, G.TYPE_VALUE, b""), (b"b", 1, G.TYPE_DELETION, b"")])
    t = ResidentTable(schema_c())
    with pytest.raises(SegmentError, match="entry 1"):
        t.load_sst(sst.decode_host(t.ctx, [(blk, 0)]))


def _versions(batch, seq0):
    """(user key, seq, type, row blob) of every row of `batch`, as a table's
    write would store them."""
    src = ResidentTable(schema_c())
    src.write(batch)
    arena = src.arena.download(src.used).tobytes()
    offs = src.row_off.download(8 * (src.n + 1)).view(np.uint64)
    keys = batch.column(0).to_pylist()
    return [(keys[i].encode(), seq0 + i, G.TYPE_VALUE, arena[offs[i]:offs[i + 1]]) for i in range(len(keys))]


@pytest.mark.parametrize("layout", ["one_file", "newer_file_first", "newer_file_last"])
def test_rehydrate_duplicate_keys_take_the_highest_seq(layout):
    # keys 2500..2999 exist in two versions: the newer (higher seq) must win,
    # wherever it sits -- first of its key in one file (RocksDB's order: user
    # key ascending, seq descending), or in a second file listed before or
    # after the first
    old, new = batch_c(3000, seed=1), batch_c(1000, start=2500, seed=2)
    v_old, v_new = _versions(old, 100), _versions(new, 10_000)
    order = lambda es: sorted(es, key=lambda e: (e[0], -e[1]))  # noqa: E731
    if layout == "one_file":
        files = [order(v_old + v_new)]
    elif layout == "newer_file_first":
        files = [order(v_new), order(v_old)]
    else:
        files = [order(v_old), order(v_new)]
    stored = [(G.snappy(b), G.SNAPPY) for f in files for b in G.blocks_of(f)]
    t = ResidentTable(schema_c())
    t.load_sst(sst.decode_host(t.ctx, stored))
    rng = np.random.default_rng(9)
    q = [f"key{i}" for i in rng.integers(2400, 3600, size=1500)] + ["key2500", "key2999", "key0"]
    cols = [f"c{i}" for i in range(16)]
    assert_same(t.read(q, cols), expected([old, new], q, cols))


@pytest.mark.parametrize("comp", [G.SNAPPY, G.LZ4])
def test_short_offset_matches_and_slot_edge(comp):
    # values repeating with periods 1..17 (matches closer than 16 bytes: the
    # thread-per-block inflate stores their 16-byte pattern and overruns the
    # match end into the slot's pad), blocks grown up to the 1 KiB tier-0 edge
    rng = np.random.default_rng(70 + comp)
    stored = []
    for period in range(1, 18):
        for target in (200, 700, 1000, 1024, 1100):
            pat = bytes(rng.integers(0, 256, size=period, dtype=np.uint8))
            entries, size = [], 0
            i = 0
            while size < target - 80:
                v = (pat * (1 + 90 // period))[: 20 + int(rng.integers(0, 70))]
                entries.append((b"k%06d" % i, 1000 + i, G.TYPE_VALUE, v))
                size += len(v) + 20
                i += 1
            stored.append((G.compress(G.build_block(entries), comp), comp))
    check(stored)


def test_device_block_table_in_place():
    # the descriptors uploaded once (sst.device_table) decode exactly as the
    # host table; a device table's block without data is malformed (named),
    # the host table's an argument error
    rng = np.random.default_rng(81)
    blocks = G.blocks_of(G.random_entries(rng, 900, max_val=120), restart_interval=8)
    stored = [(G.compress(b, c), c) for b, c in zip(blocks, [G.SNAPPY, G.NONE, G.LZ4] * len(blocks))]
    ctx = default_context()
    buf, handles = sst.upload_blocks(ctx, stored)
    want = sst.decode(ctx, buf, handles).to_host()
    tab = sst.device_table(ctx, buf, handles)
    for _ in range(2):
        got = sst.decode(ctx, buf, tab).to_host()
        assert got[0] == want[0] and got[1] == want[1]
        assert got[2].tolist() == want[2].tolist() and got[3].tolist() == want[3].tolist()
    desc = sst.block_table(buf, handles)
    desc["data"][5] = 0
    with pytest.raises(Exception):
        sst.decode(ctx, buf, desc)
    bad = sst.SstTable(ctx.upload(desc.view(np.uint8)), len(desc))
    with pytest.raises(SegmentError, match=r"row 5,"):
        sst.decode(ctx, buf, bad)


def test_outputs_reused_after_free_never_while_live():
    # the entry buffers come from the context's reuse cache: a call made while
    # an earlier result is alive gets other buffers, one made after it is
    # freed may get its buffers back; every result reads as the oracle's
    rng = np.random.default_rng(91)
    stored = [(G.snappy(b), G.SNAPPY) for b in G.blocks_of(G.random_entries(rng, 700, max_val=90))]
    want = oracle_entries(stored)
    ctx = default_context()
    buf, handles = sst.upload_blocks(ctx, stored)

    def ptrs(e):
        return {e.keys.ptr, e.key_offsets.ptr, e.values.ptr, e.value_offsets.ptr, e.seqs.ptr, e.types.ptr}

    def same(e):
        k, v, s, t = e.to_host()
        assert k == want[0] and v == want[1] and s.tolist() == want[2] and t.tolist() == want[3]

    e1 = sst.decode(ctx, buf, handles)
    e2 = sst.decode(ctx, buf, handles)
    assert not (ptrs(e1) & ptrs(e2))
    same(e1)
    same(e2)
    old = ptrs(e1)
    del e1
    e3 = sst.decode(ctx, buf, handles)
    assert not (ptrs(e3) & ptrs(e2))
    same(e3)
    same(e2)
    assert ptrs(e3) & old  # (at least one buffer came back from the cache)


def test_output_freed_while_another_stream_reads_it():
    # ADVICE / VERDICT r5: a result freed while a kernel on another context
    # still reads it must not be handed to the next murr_sst_decode (and
    # overwritten) before that kernel is done.  The reader: a long decode on
    # a second context of 2000 copies of the entries' values (row blobs of
    # the config B schema); then the result is freed and a second SST of the
    # same sizes but other values is decoded on the first context.  Both
    # outputs must read as the oracle's.
    from murr_amd import synth
    from murr_amd.device import Context, DecodeOutputs, DecodePlan, download_array, encode_batch
    from murr_amd.schema import SegmentSchema

    n = 20000
    ctx = default_context()
    ctx2 = Context(ctx.device)

    def stored_for(scale):
        cols = synth.config_b(n)
        cols[0]["values"] = (cols[0]["values"] * scale).astype(np.float32)
        seg = SegmentSchema([(f"c{i}", c["dtype"]) for i, c in enumerate(cols)])
        blob, off, blen = encode_batch(ctx, seg, synth.upload_columns(ctx, cols), n)
        hb, ho = blob.download(blen).tobytes(), off.download(8 * (n + 1)).view(np.uint64)
        entries = [(b"%08d" % i, 10 + i, G.TYPE_VALUE, hb[ho[i]:ho[i + 1]]) for i in range(n)]
        return seg, [(G.snappy(b), G.SNAPPY) for b in G.blocks_of(entries)]

    seg, s1 = stored_for(1.0)
    _, s2 = stored_for(3.0)
    w1, w2 = oracle_entries(s1), oracle_entries(s2)
    assert [len(v) for v in w1[1]] == [len(v) for v in w2[1]] and w1[1] != w2[1]
    b1, h1 = sst.upload_blocks(ctx, s1)
    b2, h2 = sst.upload_blocks(ctx, s2)
    e1 = sst.decode(ctx, b1, h1)
    vblob = np.frombuffer(b"".join(w1[1]), np.uint8)
    voff = np.concatenate([[0], np.cumsum([len(v) for v in w1[1]])]).astype(np.uint64)
    want = O.decode_block(O.Segment([int(c.dtype) for c in seg.columns]), [0, 1], vblob, voff)
    blocks = [e1.block()] * 5000
    outs = DecodeOutputs(ctx2, seg, [0, 1], blocks)
    plan = DecodePlan(ctx2, seg, [0, 1], blocks, outs)
    plan.run_async()  # ctx2's stream reads e1's values ...
    for buf in (e1.keys, e1.key_offsets, e1.values, e1.value_offsets, e1.seqs, e1.types):
        buf.free()  # ... while they go back to ctx's reuse cache (murr_dev_free)
    e2 = sst.decode(ctx, b2, h2)  # of the same sizes: may get e1's buffers back
    plan.wait()
    k, v, s, t = e2.to_host()
    assert k == w2[0] and v == w2[1] and s.tolist() == w2[2] and t.tolist() == w2[3]
    for b in (0, 2500, 4999):
        for p in range(2):
            g = download_array(ctx2, outs.array(b, p), int(seg.columns[p].dtype), n)
            e = want[p]
            if e["dtype"] == 0:
                assert np.array_equal(g["offsets"], e["offsets"]), (b, p)
            assert bytes(g["values"][: len(e["values"])]) == e["values"], (b, p)
    plan.close()
