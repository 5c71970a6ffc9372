"""RocksDB data-block restatement (oracle/murr_sst.c) on the CPU: Snappy
against pyarrow's codec, block decode against the test-side BlockBuilder
restatement (tests/sstgen.py)."""
import numpy as np
import pyarrow as pa
import pytest

import oracle as O
import sstgen as G


@pytest.mark.parametrize("data", [b"", b"a", b"abcd" * 3, b"hello hello hello hello", bytes(range(256)) * 40,
                                  b"x" * 100000, b"ab" * 7000])
def test_snappy_matches_pyarrow(data):
    z = pa.Codec("snappy").compress(data, asbytes=True)
    assert O.snappy_decompress(z) == data


def test_snappy_random_matches_pyarrow():
    rng = np.random.default_rng(3)
    for k in range(200):
        n = int(rng.integers(0, 5000))
        # mix of runs (copies) and noise (literals)
        parts = []
        while sum(map(len, parts)) < n:
            if rng.random() < 0.5:
                parts.append(rng.integers(0, 256, size=int(rng.integers(1, 80)), dtype=np.uint8).tobytes())
            else:
                parts.append(bytes([int(rng.integers(0, 4))]) * int(rng.integers(1, 200)))
        data = b"".join(parts)[:n]
        assert O.snappy_decompress(pa.Codec("snappy").compress(data, asbytes=True)) == data


def test_snappy_corrupt_is_an_error():
    z = bytearray(pa.Codec("snappy").compress(b"hello hello hello hello", asbytes=True))
    z[-1] = 200  # a copy offset past the output
    with pytest.raises(O.OracleError):
        O.snappy_decompress(bytes(z))
    with pytest.raises(O.OracleError):
        O.snappy_decompress(b"\xff\xff\xff\xff\xff\xff")


def test_snappy_literal_of_2_pow_32_reads_as_snappy_does():
    # a 4-byte literal length of 0xFFFFFFFF spliced after the header: the
    # Snappy library (pyarrow's, the codec RocksDB links) computes len + 1 in
    # 32 bits and reads an empty literal, so the stream still decodes; the
    # restatement (and the device inflaters, tests/test_gpu_sst.py) do the same
    data = b"hello hello hello hello"
    good = pa.Codec("snappy").compress(data, asbytes=True)
    bad = good[:1] + b"\xfc\xff\xff\xff\xff" + good[1:]
    assert pa.Codec("snappy").decompress(bad, decompressed_size=len(data), asbytes=True) == data
    assert O.snappy_decompress(bad) == data


@pytest.mark.parametrize("data", [b"", b"a", b"abcd" * 3, b"hello hello hello hello", bytes(range(256)) * 40,
                                  b"x" * 100000, b"ab" * 7000])
def test_lz4_matches_pyarrow(data):
    assert O.lz4_decompress(G.lz4(data)) == data


def test_lz4_random_matches_pyarrow():
    rng = np.random.default_rng(5)
    for k in range(200):
        n = int(rng.integers(0, 5000))
        parts = []
        while sum(map(len, parts)) < n:
            if rng.random() < 0.5:
                parts.append(rng.integers(0, 256, size=int(rng.integers(1, 300)), dtype=np.uint8).tobytes())
            else:
                parts.append(bytes([int(rng.integers(0, 4))]) * int(rng.integers(1, 600)))
        data = b"".join(parts)[:n]
        assert O.lz4_decompress(G.lz4(data)) == data


def test_lz4_corrupt_is_an_error():
    z = bytearray(G.lz4(b"hello hello hello hello hello"))
    with pytest.raises(O.OracleError):
        O.lz4_decompress(bytes(z[:-1]))  # the last sequence cut short
    z[0] += 1  # the length prefix disagrees with the contents
    with pytest.raises(O.OracleError):
        O.lz4_decompress(bytes(z))


@pytest.mark.parametrize("restart,hash_index", [(1, False), (8, True), (8, False), (16, True)])
def test_block_roundtrip(restart, hash_index):
    rng = np.random.default_rng(restart * 7 + hash_index)
    entries = G.random_entries(rng, 300, dup_p=0.2, del_p=0.1)
    blk = G.build_block(entries, restart_interval=restart, hash_index=hash_index)
    keys, vals, seqs, types = O.block_decode(blk)
    assert keys == [e[0] for e in entries]
    assert vals == [e[3] for e in entries]
    assert seqs.tolist() == [e[1] for e in entries]
    assert types.tolist() == [e[2] for e in entries]


def test_block_versions_share_trailer_bytes():
    # versions of one key differ only in the trailer: shared > user key length
    entries = [(b"same", 1000 - i, G.TYPE_VALUE, bytes([i])) for i in range(20)]
    keys, vals, seqs, _ = O.block_decode(G.build_block(entries))
    assert keys == [b"same"] * 20 and seqs.tolist() == [1000 - i for i in range(20)]


def test_blocks_of_a_table_and_compression():
    rng = np.random.default_rng(9)
    entries = G.random_entries(rng, 2000)
    blocks = G.blocks_of(entries)
    assert len(blocks) > 50
    got = []
    for i, b in enumerate(blocks):
        comp = (G.NONE, G.SNAPPY, G.LZ4)[i % 3]
        k, v, _, _ = O.block_decode(O.block_contents(G.compress(b, comp), comp))
        got += list(zip(k, v))
    assert got == [(e[0], e[3]) for e in entries]


def test_corrupt_blocks_are_errors():
    blk = bytearray(G.build_block([(b"a", 1, 1, b"x"), (b"b", 2, 1, b"y")]))
    with pytest.raises(O.OracleError):
        O.block_decode(bytes(blk[:3]))
    bad = bytearray(blk)
    bad[0] = 5  # shared bytes at a restart point
    with pytest.raises(O.OracleError):
        O.block_decode(bytes(bad))


def test_bulk_decode_totals_match_per_block():
    rng = np.random.default_rng(13)
    blocks = G.blocks_of(G.random_entries(rng, 3000, dup_p=0.1))
    stored = [(G.compress(b, (G.NONE, G.SNAPPY, G.LZ4)[i % 3]), (G.NONE, G.SNAPPY, G.LZ4)[i % 3])
              for i, b in enumerate(blocks)]
    data = np.frombuffer(b"".join(d for d, _ in stored), np.uint8)
    sizes = np.array([len(d) for d, _ in stored], np.int64)
    h = np.stack([np.cumsum(sizes) - sizes, sizes, np.array([c for _, c in stored], np.int64)], axis=1)
    ne = kb = vb = 0
    for d, c in stored:
        k, v, _, _ = O.block_decode(O.block_contents(d, c))
        ne, kb, vb = ne + len(k), kb + sum(map(len, k)), vb + sum(map(len, v))
    assert O.sst_decode_all(data, h) == (ne, kb, vb)
